// Host-side launchers of the gfx950 kernels (raw pointers + stream; no torch
// headers here so the .hip files compile quickly).  Bound to torch in bindings.cpp.
#pragma once

#include <string>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <memory>

namespace mlop {

void launch_rmsnorm(void* out, const void* x, const void* w, float eps, int M, int H,
                    hipStream_t st);
void launch_add_rmsnorm(void* out, void* residual, const void* x, const void* w, float eps, int M,
                        int H, hipStream_t st);
void launch_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv, const int* pos,
                       const float* cos_sin, const int* slots, int T, int Hq, int Hkv, int D,
                       int qkv_stride, int BS, hipStream_t st);
void launch_silu_mul(void* out, const void* x, int M, int I, int interleaved, hipStream_t st);
void launch_device_delay(long long ticks, hipStream_t st);
void launch_embedding(void* out, const void* table, const long* ids, int T, int H, long vocab_start,
                      long vocab_end, hipStream_t st);
void launch_paged_attention(void* out, float* part_o, float* part_ml, const void* q,
                            const void* kc, const void* vc, const int* bt, int bt_stride,
                            const int* tile_seq, const int* tile_q0, const int* q_start,
                            const int* q_len, const int* ctx_len, int num_tiles, int Hq, int Hkv,
                            float scale_log2, int part_tokens, int nparts, int num_blocks,
                            int* sem, hipStream_t st);
int flash_persist(int set);  // 0: one workgroup per flash item; n: persistent grid, n per CU
int flash_stream(int set);   // 1: the persistent grid streams K / V pairs and Q across tiles
int gemm_grouped_balance(int set);  // 1: equal row ranges per expert m-tile; 2: + the 16-row MFMA skip
int gemm_grouped_order(int set);    // grouped tile order: 0 slot fastest, 1 expert-major, 2 auto
int moe_mid_tok(int set);            // tokens per workgroup of the mid MoE dispatch: 0 = by T, 2, 4, 8
void launch_flash_prefill(void* out, const void* q, const void* kc, const void* vc, const int* bt,
                          int bt_stride, const int* ptile_seq, const int* ptile_q0,
                          const int* q_start, const int* q_len, const int* ctx_len, int num_ptiles,
                          int Hq, int Hkv, float scale_log2, int num_blocks, hipStream_t st);
// QKV projection epilogue (EPI_ROPE): the GEMM's C tile is [q heads | k heads | v heads]
// of head_dim 128; q/k are rotated (HF rotate-half, cos/sin table [max_pos, 128]) and
// q goes to q_out [T, Hq, 128], k / v into the paged cache (k [NB, Hkv, BS, 128],
// v [NB, Hkv, 128, BS]; slot < 0 = padding row, no cache write) - rope_cache.hip's
// layout, done from the GEMM's LDS-staged tile instead of a [T, N] round trip.
struct RopeEpi {
  uint16_t* q_out;
  uint16_t* k_cache;
  uint16_t* v_cache;
  const int* pos;
  const float* cos_sin;
  const int* slots;
  int Hq, Hkv, BS;
  // four-wave norm chain (run_w4 only; the large-M TP=1 decoder with unit norm weights, see
  // launch_w4_chain).  Producer (C += A.B^T): ss_out = [M, N / 128] partial sums of squares of
  // the updated residual rows (one per row and wave column block), then ss_tot [M] = their row
  // sums, added in a fixed order by the last tile of each 256-row band (ss_cnt: one ticket per
  // band).  Consumer: ss_in = a producer's ss_tot; the accumulators of row r are scaled by
  // rsqrt(ss_in[r] * ss_inv_k + ss_eps) = RMSNorm applied after the GEMM.
  const float* ss_in = nullptr;
  float* ss_out = nullptr;
  float* ss_tot = nullptr;
  int* ss_cnt = nullptr;
  float ss_inv_k = 0.f, ss_eps = 0.f;
  // grouped GEMM: A row of permuted row r is a_rows[r] (moe_dispatch_mid: the experts read the
  // token rows in place, no gathered copy); nullptr = row r
  const int* a_rows = nullptr;
  // gemm_kernel: the weight (B) pieces of the LDS-DMA ring load non-temporal (read once by one
  // workgroup: MI355X_MICROARCH.md "nt-weights"); set by run_cfg (gemm_small_nt)
  int b_nt = 0;
  // gemm_kernel: split-K slabs stored non-temporal (not left dirty in L2 for the kernel boundary's
  // write-back; MI355X_MICROARCH.md "boundary"); set by run_cfg (gemm_slab_nt)
  int ws_nt = 0;
  // mid norm chain (gemm.hip mid_chain_finish): 1 = the finishing split reads the partials with
  // plain loads behind one agent acquire, 0 = with sc1 loads only (gemm_mid_chain op 2 / 1)
  int mid_acq = 0;
};
// RoPE + paged-cache stores from the QKV projection's fp32 split-K slabs ws[splits][T][N] (the
// split-K reduce fused in: small-M launch_gemm_rope)
void launch_rope_cache_slabs(const RopeEpi& re, const float* ws, int splits, int T, int N, hipStream_t st);
long gemm_workspace_floats(int M, int N, int K, int epi);
// large-M kernel variant of the GEMM planner (gemm.hip plan(): 0 256x128, 1/2 256x256
// 8-wave, 3 ping-pong, 5 four-wave asm K-loop); set >= 0 overrides (in-process A/B), returns the current value
int gemm_big_variant(int set);
int gemm_half_tile(int set);
int gemm_grouped_narrow(int set);
void gemm_grouped_plan(int bm, int bn, int stages, int splits);
void gemm_dense_plan(int variant, int bm, int bn, int splits, int stages = 0);
// variant 5: the four-wave hand-scheduled 256x256 kernel (gemm_w4.hip), variant 6 its 128x256
// half-height tile; epi 0 / 1 / 3
bool gemm_w4_ok(int M, int N, int K, int lda, int ldb, int ldc = 0);
// the four-wave kernel cuts its r = T % CUs tail tiles into K-halves (2r <= CUs, nk even)
bool gemm_w4_split_ok(int T, int nk);
bool gemm_sk_scratch(float** ws, int** cnt, int* cus);
bool gemm_sk_available(int* cus);
bool run_w4(int epi, const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M, int N,
            int K, hipStream_t st, const RopeEpi& re, int bm = 256);
// norm chain on the four-wave kernel (epi flags: 4 = C += A.B^T with ss partials, 8 = rows scaled
// by re.ss_in; 4, 0|8, 1|8, 3|8 are built): true when every such GEMM of this shape runs there
bool w4_chain_ok(int M, int N, int K);
bool launch_w4_chain(int epi, const void* A, int lda, const void* B, void* C, int ldc, int M, int N, int K,
                     const RopeEpi& re, hipStream_t st);
int gemm_small_stages(int set);  // LDS-DMA ring depth of the M <= 128 tiles (3, or 5/6)
int gemm_small_tile(int set);    // M <= 64 tiles: 0 = 64 x 64, 32 / 64 = row-fitted BM x BN
// non-temporal weight loads of the one-m-tile gemm_kernel launches: bit 0 dense, bit 1 grouped,
// bit 2 the grouped ping-pong kernel
int gemm_small_nt(int set);
// non-temporal K / V page loads of the decode attention kernel
int attn_kv_nt(int set);
int gemm_slab_nt(int set);
int gemm_rope_split(int set);
int gemm_split_target(int set);  // K ranges of the small-M QKV + RoPE launch (A/B)
// stream-K tail of the ping-pong GEMM: mode (1 on, 0 off; set >= 0 changes it) and the
// per-device partial / counter buffers (allocate once, outside graph capture)
int gemm_sk_mode(int set);
bool gemm_sk_reserve();
int gemm_sk_workgroups(int M, int N, int K);
// K2 skinny GEMV (gemv.hip): decode projections at M <= 8 (epi 0 none, 1 silu-mul, 3 rope)
bool gemv_takes(int M, int N, int K, int epi);
void launch_gemv(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                 int epi, hipStream_t st);
void launch_gemv_rope(const void* A, int lda, const void* B, int M, int N, int K, const RopeEpi& re,
                      hipStream_t st);
// the decode norm chain's row-scale prologue parameters (gemv.hip PRO_RS)
struct NormPro {
  float eps = 0.f;
};
// decode norm chain (gemv.hip PRO_RS / EPI_RES, M <= 4): C = epi(rowscale(A) . B^T) with
// rowscale = rsqrt(mean(A_row^2) + eps) (norm weights folded into B); residual += A . B^T
bool gemv_chain_takes(int M, int N, int K, int epi);
// weight-streaming MFMA GEMM (gemm_ws.hip) at gemv_chain_max_m() < M <= gemm_ws_max_m() (64):
// epi 0 plain, 1 SiLU-mul, 3 RoPE + paged K/V (re), 5 residual += (C in place); rs: A is the raw
// residual, rows scaled by rsqrt(mean(a^2) + eps) (norm weights folded into B)
bool ws_takes(int M, int N, int K, int epi);
int gemm_ws_max_m(int set);
void gemm_ws_plan(int rb, int u, int nt);
int gemm_ws_small_m(int set);
int gemm_ws_rope_m(int set);  // rows up to which QKV + RoPE takes the weight-streaming kernel
// the plain (non-chain) decode projections this kernel takes instead of the planner
bool ws_prefer(int M, int N, int K, int epi);
// mid-M norm chain on the planner's small tiles (gemm.hip): epi 0 = O / down (split-K, the
// last split adds into the residual and leaves the row sums of squares), 1 = gate_up (SiLU-mul,
// row-scaled), 3 = QKV + RoPE (row-scaled slab reduce, or the ws kernel at 5-8 rows)
int gemm_mid_chain(int set);
bool mid_chain_ok(int M, int N, int K, int epi);
bool launch_mid_res_ss(const void* A, int lda, const void* B, void* residual, int ldr, int M, int N, int K,
                       float* ss_tot, hipStream_t st);
bool launch_mid_rs(const void* A, int lda, const void* B, void* out, int ldo, int M, int N, int K,
                   const float* ss_tot, float eps, hipStream_t st);
// the decode norm chain's forms: the GEMV up to gemv_chain_max_m() rows, then the weight-
// streaming MFMA kernel up to gemm_ws_max_m()
int decode_chain_max_m();
bool decode_chain_takes(int M, int N, int K, int epi);
void launch_ws(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K, int epi,
               bool rs, const RopeEpi& re, float eps, hipStream_t st);
int gemv_chain_max_m();
void launch_gemv_rs(const void* A, int lda, const void* B, void* C, int ldc, int M, int N, int K, int epi,
                    const RopeEpi& re, float eps, hipStream_t st);
void launch_gemv_res(const void* A, int lda, const void* B, void* residual, int M, int N, int K, hipStream_t st);
bool gemv_grouped_takes(int M, int N, int K, int epi);
void launch_gemv_grouped(const void* A, const void* B, void* C, const int* offsets, int n_groups, int M, int N,
                         int K, int epi, hipStream_t st);
bool gemm_rope_supported(int M, int N, int K);
bool launch_gemm_rope(const void* A, int lda, const void* B, int M, int N, int K, const RopeEpi& re,
                      hipStream_t st);
void launch_gemm(const void* A, int lda, const void* B, int ldb, void* C, int ldc, float* ws,
                 long ws_floats, int M, int N, int K, int epi, hipStream_t st);
bool launch_gemm_add_rmsnorm(const void* A, int lda, const void* B, void* out, void* residual,
                             const void* w, float eps, float* ws, long ws_floats, int M, int N,
                             int K, hipStream_t st);
void launch_grouped_gemm(const void* A, const void* B, void* C, const int* offsets, int n_groups,
                         int M, int N, int K, int max_rows, int epi, hipStream_t st, const int* a_rows = nullptr,
                         float** defer_ws = nullptr, int* defer_splits = nullptr);
bool launch_moe_down_combine_add_rmsnorm(void* out, void* residual, void* y, const void* a, const void* w2,
                                         const int* offsets, int n_groups, int R, int H, int I, int max_rows,
                                         const int* inv, const float* topw, const void* norm_w, float eps, int T,
                                         int k, hipStream_t st);
// mid-size MoE dispatch (16 < T <= 16384 tokens): router GEMV + route per token workgroup, the last
// workgroup (agent-scope ticket) sorts the T*k slots by local expert -> offsets, inv and arow (the
// token row of each permuted row: the grouped GEMM reads x through it, no gather)
bool moe_dispatch_mid_takes(int T, int E, int k, int H);
int moe_mid_max_tokens(int set);
void launch_moe_dispatch_mid(float* topw, int* topi, int* offsets, int* arow, int* inv, const void* x, const void* wr,
                             int T, int E, int k, int H, int e0, int n_local, const void* pro_y, void* pro_res,
                             const void* pro_w, float pro_eps, void* pro_xn, hipStream_t st);
void launch_moe_route(float* topw, int* topi, const void* logits, int T, int E, int k,
                      hipStream_t st);
void launch_moe_permute(void* xp, int* offsets, int* src, int* inv, const void* x, const int* topi,
                        int T, int k, int H, int e0, int n_local, hipStream_t st);
void launch_moe_combine(void* out, const void* y, const int* inv, const float* topw, int T, int k,
                        int H, hipStream_t st);
// decode-size MoE dispatch in one launch: router GEMV + route + sort + gather (moe.hip)
bool moe_dispatch_small_takes(int T, int E, int k, int H);
// pro_y != nullptr: prologue residual += pro_y, x = rmsnorm(residual) * pro_w (written to pro_xn)
void launch_moe_dispatch_small(float* topw, int* topi, void* xp, int* offsets, int* src, int* inv, const void* x,
                               const void* wr, int T, int E, int k, int H, int e0, int n_local, const void* pro_y,
                               void* pro_res, const void* pro_w, float pro_eps, void* pro_xn, hipStream_t st);
// combine + residual add + RMSNorm in one launch; false = hidden size not instantiated
bool launch_moe_combine_add_rmsnorm(void* out, void* residual, const void* y, const int* inv, const float* topw,
                                    const void* w, float eps, int T, int k, int H, hipStream_t st);
void launch_argmax(long* out, const float* logits, int n, int V, long ld, hipStream_t st);
// bf16 greedy argmax; ws (>= argmax_splits(n, V) * n int64, or null) splits small batches' rows
int argmax_splits(int n, int V);
void launch_argmax_bf16(long* out, const void* logits, int n, int V, long ld, void* ws, hipStream_t st);
// temperature / top-k / top-p draw; small batches pre-select per-slice top-K candidates into ws
// (sample_workspace_bytes(n, V) bytes, 0 = not needed)
long sample_workspace_bytes(int n, int V);
void launch_sample(long* out, const float* logits, int n, int V, long ld, const float* temps,
                   const int* top_ks, const float* top_ps, const float* uniform, void* ws, bool full,
                   hipStream_t st);

// lazily backed KV arenas (vmm.hip): reserve VA, back chunks synchronously or on a native
// worker thread; the returned owner must outlive every use of the range
bool vmm_supported(int device);
long vmm_granularity(int device);
std::shared_ptr<void> vmm_reserve(long bytes, int device, void** base_out, long* reserved_out);
void vmm_forget(void* base);
bool vmm_map_chunks(void* base, long region_stride, int n_regions, long chunk_bytes, long first, long count,
                    bool async);
long vmm_chunks_ready(void* base);
int vmm_error(void* base);

// K15 custom one-shot all-reduce (allreduce.hip); handles are opaque state pointers
long car_create(int rank, int world, long max_bytes, int device, int split);
void car_ipc_handle(long h, void* out128);
void car_open(long h, const void* handles);
long car_max_bytes(long h);
// add_out: out = bf16(out + bf16(sum)) (the residual stream; one-shot only, out != in)
void car_all_reduce(long h, void* out, const void* in, long numel, hipStream_t st, bool two_shot = false,
                    bool add_out = false);
void car_broadcast(long h, void* out, const void* in, long nbytes, int root, hipStream_t st);
void car_all_gather(long h, void* out, long out_bytes, const void* in, long nbytes, hipStream_t st);
int car_error(long h);
int car_mem_mode(long h);
void car_destroy(long h);

// host-to-host step-header channel over POSIX shared memory (shm_channel.cc, host code)
long chan_create(const std::string& name, int nslots, int nconsumers);
long chan_open(const std::string& name);
bool chan_send(long h, const int64_t* w, int n, long timeout_us);
bool chan_recv(long h, int consumer, int64_t* w, int n, long timeout_us);
void chan_unlink(const std::string& name);
void chan_close(long h, bool unlink);
long xg_create(const std::string& name, int world, int nslots, long max_words);
long xg_open(const std::string& name, int rank);
long xg_max_words(long h);
bool xg_exchange(long h, const int64_t* in, long n, int64_t* out, int64_t* counts, long timeout_us);
void xg_close(long h);

// expert-parallel dispatch / combine over IPC peer memory (ep_exchange.hip)
long ep_create(int rank, int world, int E, int k, int H, int tcap, int device);
void ep_ipc_handle(long h, void* out64);
void ep_open(long h, const void* handles);
int ep_mem_mode(long h);
int ep_world(long h);
int ep_local_experts(long h);
int ep_hidden(long h);
int ep_topk(long h);
int ep_tcap(long h);
void ep_dispatch(long h, void* xp, long xp_rows, int* offsets, const void* x, const int* topi, int T, hipStream_t st);
void ep_combine(long h, void* out, const void* y, long y_rows, const float* topw, const int* topi, int T,
                hipStream_t st);
int ep_error(long h);
void ep_destroy(long h);

}  // namespace mlop
