// torch.ops.mlop.* registrations for the gfx950 kernels.
//
// Every op validates dtype / contiguity / shape on the host before launching
// (a faulting kernel can reset every GPU of the node), runs on the current
// HIP stream (so it is hipGraph-capturable) and mutates pre-allocated outputs
// (cdna_hip_programming.md Guideline 9; the one scratch tensor, gemm_rope_cache's V staging,
// comes from PyTorch's caching allocator, which serves captures from the graph's pool).
#include <cstdlib>
#include <string>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <cmath>

#include "launch.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_i32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kInt, name, " must be int32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void rmsnorm(Tensor out, Tensor x, Tensor w, double eps) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w");
  const int64_t H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && H <= 65536, "hidden size must be a multiple of 8");
  TORCH_CHECK(w.numel() == H && out.numel() == x.numel(), "rmsnorm shape mismatch");
  c10::DeviceGuard g(x.device());
  mlop::launch_rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), (float)eps,
                       (int)(x.numel() / H), (int)H, cur_stream());
}

void add_rmsnorm(Tensor out, Tensor residual, Tensor x, Tensor w, double eps) {
  check_bf16(out, "out"); check_bf16(residual, "residual"); check_bf16(x, "x"); check_bf16(w, "w");
  const int64_t H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && H <= 65536, "hidden size must be a multiple of 8");
  TORCH_CHECK(w.numel() == H && out.numel() == x.numel() && residual.numel() == x.numel(),
              "add_rmsnorm shape mismatch");
  c10::DeviceGuard g(x.device());
  mlop::launch_add_rmsnorm(out.data_ptr(), residual.data_ptr(), x.data_ptr(), w.data_ptr(),
                           (float)eps, (int)(x.numel() / H), (int)H, cur_stream());
}

void rope_cache(Tensor q_out, Tensor k_cache, Tensor v_cache, Tensor qkv, Tensor pos,
                Tensor cos_sin, Tensor slots) {
  check_bf16(q_out, "q_out"); check_bf16(k_cache, "k_cache"); check_bf16(v_cache, "v_cache");
  check_i32(pos, "pos"); check_i32(slots, "slots");
  TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.stride(-1) == 1,
              "qkv must be bf16 with unit inner stride");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous(), "cos_sin f32");
  TORCH_CHECK(q_out.dim() == 3 && k_cache.dim() == 4 && v_cache.dim() == 4, "rope_cache ranks");
  const int T = (int)q_out.size(0), Hq = (int)q_out.size(1), D = (int)q_out.size(2);
  const int Hkv = (int)k_cache.size(1), BS = (int)k_cache.size(2);
  TORCH_CHECK(k_cache.size(3) == D && v_cache.sizes() == k_cache.sizes(),
              "cache layouts: k and v [NB,Hkv,BS,D] (token-major)");
  TORCH_CHECK(D % 16 == 0, "head dim must be a multiple of 16");
  TORCH_CHECK(qkv.size(0) == T && qkv.size(-1) >= (Hq + 2 * Hkv) * D, "qkv shape");
  TORCH_CHECK(pos.numel() == T && slots.numel() == T, "pos/slots length");
  TORCH_CHECK(cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  c10::DeviceGuard g(qkv.device());
  mlop::launch_rope_cache(q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), qkv.data_ptr(),
                          pos.data_ptr<int>(), cos_sin.data_ptr<float>(), slots.data_ptr<int>(), T,
                          Hq, Hkv, D, (int)qkv.stride(0), BS, cur_stream());
}

void silu_mul(Tensor out, Tensor x, int64_t interleaved) {
  check_bf16(out, "out"); check_bf16(x, "x");
  const int64_t I2 = x.size(-1);
  TORCH_CHECK(I2 % (interleaved ? 32 : 16) == 0, "gate_up width must be a multiple of 16/32");
  const int64_t M = x.numel() / I2;
  TORCH_CHECK(out.numel() == M * (I2 / 2), "silu_mul shape mismatch");
  c10::DeviceGuard g(x.device());
  mlop::launch_silu_mul(out.data_ptr(), x.data_ptr(), (int)M, (int)(I2 / 2), (int)interleaved,
                        cur_stream());
}

// fault injection: a device-side delay of `us` microseconds on the current stream
void device_delay(int64_t us) {
  int dev = 0, khz = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "device_delay: hipGetDevice");
  TORCH_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0,
              "device_delay: wall clock rate");
  TORCH_CHECK(us >= 0 && us <= 10000000, "device_delay: 0..10 s");
  mlop::launch_device_delay((long long)us * khz / 1000, cur_stream());
}

void embedding(Tensor out, Tensor table, Tensor ids, int64_t vocab_start) {
  check_bf16(out, "out"); check_bf16(table, "table");
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids int64");
  const int64_t H = table.size(1);
  TORCH_CHECK(H % 8 == 0 && out.size(-1) == H && out.numel() == ids.numel() * H, "embedding shape");
  c10::DeviceGuard g(table.device());
  mlop::launch_embedding(out.data_ptr(), table.data_ptr(), ids.data_ptr<int64_t>(),
                         (int)ids.numel(), (int)H, vocab_start, vocab_start + table.size(0),
                         cur_stream());
}

void flash_prefill(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables,
                   Tensor ptile_seq, Tensor ptile_q0, Tensor q_start, Tensor q_len, Tensor ctx_len,
                   double scale) {
  check_bf16(out, "out"); check_bf16(q, "q"); check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(block_tables, "block_tables"); check_i32(ptile_seq, "ptile_seq");
  check_i32(ptile_q0, "ptile_q0"); check_i32(q_start, "q_start"); check_i32(q_len, "q_len");
  check_i32(ctx_len, "ctx_len");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 16 && k_cache.size(3) == 128,
              "k_cache must be [NB, Hkv, 16, 128]");
  TORCH_CHECK(v_cache.sizes() == at::IntArrayRef({k_cache.size(0), k_cache.size(1), 16, 128}),
              "v_cache must be [NB, Hkv, 16, 128] (token-major, as k_cache)");
  const int Hq = (int)q.size(1), Hkv = (int)k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  const int G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8, "flash prefill: GQA group must be 1, 2, 4 or 8");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(ptile_seq.numel() == ptile_q0.numel(), "tile arrays");
  // the stream kernel's O stores range-check at 2 GB (masked rows are stored past it)
  TORCH_CHECK(!mlop::flash_stream(-1) || out.numel() * 2 < (int64_t)0x7fffff00, "flash_stream: output >= 2 GB");
  TORCH_CHECK(q_start.numel() == q_len.numel() && q_len.numel() == ctx_len.numel() &&
                  block_tables.size(0) >= q_len.numel(),
              "per-sequence arrays");
  c10::DeviceGuard g(q.device());
  mlop::launch_flash_prefill(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                             block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                             ptile_seq.data_ptr<int>(), ptile_q0.data_ptr<int>(),
                             q_start.data_ptr<int>(), q_len.data_ptr<int>(), ctx_len.data_ptr<int>(),
                             (int)ptile_seq.numel(), Hq, Hkv, (float)(scale * 1.4426950408889634),
                             (int)k_cache.size(0), cur_stream());
}

// Largest (tile, kv head) pair count that takes the in-launch split-KV combine: no cap (a cap of
// 32 pairs measured the same at 16 x 32k contexts, BASELINE.md long context); settable in-process
// for the tests (attn_fused_max_pairs(); -1 reads it back).
static int g_attn_fused_pairs = 1 << 30;
static int attn_fused_pairs_cap() { return g_attn_fused_pairs; }
int64_t attn_fused_max_pairs(int64_t n) {
  const int prev = attn_fused_pairs_cap();
  if (n >= 0) g_attn_fused_pairs = (int)n;
  return prev;
}

void paged_attention(Tensor out, Tensor part_o, Tensor part_ml, Tensor part_sem, Tensor q, Tensor k_cache,
                     Tensor v_cache, Tensor block_tables, Tensor tile_seq, Tensor tile_q0,
                     Tensor q_start, Tensor q_len, Tensor ctx_len, double scale,
                     int64_t part_tokens, int64_t nparts) {
  check_bf16(out, "out"); check_bf16(q, "q"); check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(block_tables, "block_tables"); check_i32(tile_seq, "tile_seq");
  check_i32(tile_q0, "tile_q0"); check_i32(q_start, "q_start"); check_i32(q_len, "q_len");
  check_i32(ctx_len, "ctx_len");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 16 && k_cache.size(3) == 128,
              "k_cache must be [NB, Hkv, 16, 128]");
  TORCH_CHECK(v_cache.sizes() == at::IntArrayRef({k_cache.size(0), k_cache.size(1), 16, 128}),
              "v_cache must be [NB, Hkv, 16, 128] (token-major, as k_cache)");
  const int Hq = (int)q.size(1), Hkv = (int)k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  const int G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "GQA group must divide 16");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(tile_seq.numel() == tile_q0.numel(), "tile arrays");
  TORCH_CHECK(q_start.numel() == q_len.numel() && q_len.numel() == ctx_len.numel() &&
                  block_tables.size(0) >= q_len.numel(),
              "per-sequence arrays");
  TORCH_CHECK(part_tokens % 32 == 0 && part_tokens > 0 && nparts >= 1, "partition size");
  const int num_tiles = (int)tile_seq.numel();
  if (nparts > 1) {
    TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_ml.scalar_type() == at::kFloat,
                "partials f32");
    TORCH_CHECK(part_o.numel() >= (int64_t)num_tiles * Hkv * nparts * 16 * 128 &&
                    part_ml.numel() >= (int64_t)num_tiles * Hkv * nparts * 16 * 2,
                "partial workspace too small");
  }
  // part_sem: zero-initialised int32 tickets, one per (tile, kv head), re-armed by the
  // kernel; empty -> the split-KV combine runs as a second launch
  // Round 3 capped it at 32 pairs: every partition's agent release fence outweighed the
  // saved launch above that (batch 8: 1800 -> 1783 tok/s, scripts/run52.sh).  With the
  // partials stored sc1 and no producer fence it wins at every batch measured (batch 8 / 16
  // / 64: +0.7 / +0.7 / +0.2 %, scripts/history/r4_fusedc.sh), so the cap is off by default.
  const int max_pairs = attn_fused_pairs_cap();
  int* sem = nullptr;
  if (nparts > 1 && part_sem.numel() > 0 && num_tiles * Hkv <= max_pairs) {
    check_i32(part_sem, "part_sem");
    TORCH_CHECK(part_sem.numel() >= (int64_t)num_tiles * Hkv, "part_sem too small");
    sem = part_sem.data_ptr<int>();
  }
  c10::DeviceGuard g(q.device());
  const float scale_log2 = (float)(scale * 1.4426950408889634);
  mlop::launch_paged_attention(
      out.data_ptr(), nparts > 1 ? part_o.data_ptr<float>() : nullptr,
      nparts > 1 ? part_ml.data_ptr<float>() : nullptr, q.data_ptr(), k_cache.data_ptr(),
      v_cache.data_ptr(), block_tables.data_ptr<int>(), (int)block_tables.stride(0),
      tile_seq.data_ptr<int>(), tile_q0.data_ptr<int>(), q_start.data_ptr<int>(),
      q_len.data_ptr<int>(), ctx_len.data_ptr<int>(), num_tiles, Hq, Hkv, scale_log2,
      (int)part_tokens, (int)nparts, (int)k_cache.size(0), sem, cur_stream());
}

// ---- lazily backed KV arenas (vmm.hip)
bool vmm_supported(int64_t device) { return mlop::vmm_supported((int)device); }
int64_t vmm_granularity(int64_t device) { return mlop::vmm_granularity((int)device); }

// flat uint8 tensor over a reserved (unbacked) device range; its storage owns the arena
Tensor vmm_arena(int64_t bytes, int64_t device) {
  void* base = nullptr;
  long reserved = 0;
  std::shared_ptr<void> owner = mlop::vmm_reserve((long)bytes, (int)device, &base, &reserved);
  TORCH_CHECK(owner != nullptr, "hipMemAddressReserve failed");
  const at::Device dev(at::kCUDA, (int)device);
  // target_device: the range is not backed yet, so the pointer's device cannot be queried
  return at::for_blob(base, {(int64_t)reserved})
      .deleter([owner, base](void*) mutable {
        mlop::vmm_forget(base);
        owner.reset();
      })
      .options(at::TensorOptions().dtype(at::kByte).device(dev))
      .target_device(dev)
      .make_tensor();
}

bool vmm_map_chunks(Tensor flat, int64_t region_stride, int64_t n_regions, int64_t chunk_bytes, int64_t first,
                    int64_t count, bool async) {
  return mlop::vmm_map_chunks(flat.data_ptr(), (long)region_stride, (int)n_regions, (long)chunk_bytes,
                              (long)first, (long)count, async);
}
int64_t vmm_chunks_ready(Tensor flat) { return mlop::vmm_chunks_ready(flat.data_ptr()); }
int64_t vmm_error(Tensor flat) { return mlop::vmm_error(flat.data_ptr()); }

int64_t gemm_big_variant(int64_t set) { return mlop::gemm_big_variant((int)set); }
int64_t gemm_half_tile(int64_t set) { return mlop::gemm_half_tile((int)set); }
int64_t gemm_small_nt(int64_t set) { return mlop::gemm_small_nt((int)set); }
int64_t attn_kv_nt(int64_t set) { return mlop::attn_kv_nt((int)set); }
int64_t gemm_slab_nt(int64_t set) { return mlop::gemm_slab_nt((int)set); }
int64_t gemm_rope_split(int64_t set) { return mlop::gemm_rope_split((int)set); }
int64_t gemm_split_target(int64_t set) { return mlop::gemm_split_target((int)set); }
int64_t gemm_grouped_narrow(int64_t set) { return mlop::gemm_grouped_narrow((int)set); }
int64_t moe_mid_max_tokens(int64_t set) { return mlop::moe_mid_max_tokens((int)set); }
void gemm_dense_plan(int64_t variant, int64_t bm, int64_t bn, int64_t splits, int64_t stages) {
  mlop::gemm_dense_plan((int)variant, (int)bm, (int)bn, (int)splits, (int)stages);
}
void gemm_grouped_plan(int64_t bm, int64_t bn, int64_t stages, int64_t splits) {
  mlop::gemm_grouped_plan((int)bm, (int)bn, (int)stages, (int)splits);
}
int64_t gemm_small_stages(int64_t set) { return mlop::gemm_small_stages((int)set); }
int64_t gemm_small_tile(int64_t set) { return mlop::gemm_small_tile((int)set); }
int64_t gemm_sk_mode(int64_t set) { return mlop::gemm_sk_mode((int)set); }
bool gemm_sk_reserve() { return mlop::gemm_sk_reserve(); }
int64_t gemm_sk_workgroups(int64_t M, int64_t N, int64_t K) { return mlop::gemm_sk_workgroups((int)M, (int)N, (int)K); }

int64_t gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t epi) {
  if (epi == 2) return mlop::gemm_workspace_floats((int)M, (int)N, (int)K, 0);  // GEMM + add + RMSNorm: split-K slabs
  return mlop::gemm_workspace_floats((int)M, (int)N, (int)K, (int)epi);
}

// out[M, N or N/2] = epi(a[M, K] . w[N, K]^T)
void gemm(Tensor out, Tensor a, Tensor w, Tensor ws, int64_t epi) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1,
              "a must be bf16 [M, K] with unit inner stride");
  check_bf16(w, "w");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.dim() == 2 &&
                  out.stride(1) == 1, "out must be bf16 [M, N]");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "w must be [N, K]");
  TORCH_CHECK(K % 64 == 0, "K must be a multiple of 64");
  TORCH_CHECK(N % 8 == 0 && a.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "16-B aligned rows");
  TORCH_CHECK(epi == 0 || epi == 1, "epi");
  TORCH_CHECK(epi == 0 || N % 32 == 0, "silu_mul epilogue needs N % 32 == 0");
  TORCH_CHECK(out.size(0) == M && out.size(1) == (epi == 0 ? N : N / 2), "out shape");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "16-B aligned data");
  float* wsp = nullptr;
  int64_t wsn = 0;
  if (ws.defined() && ws.numel() > 0) {
    TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat, "ws f32");
    wsp = ws.data_ptr<float>();
    wsn = ws.numel();
  }
  c10::DeviceGuard g(a.device());
  mlop::launch_gemm(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, out.data_ptr(),
                    (int)out.stride(0), wsp, wsn, (int)M, (int)N, (int)K, (int)epi, cur_stream());
}

// QKV projection with RoPE + paged-cache stores in the GEMM epilogue; false = this M
// does not take the fused tiling (caller runs gemm + rope_cache)
bool gemm_rope_cache(Tensor q_out, Tensor k_cache, Tensor v_cache, Tensor a, Tensor w, Tensor pos,
                     Tensor cos_sin, Tensor slots) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(q_out, "q_out"); check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache"); check_i32(pos, "pos"); check_i32(slots, "slots");
  TORCH_CHECK(cos_sin.is_cuda() && cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous(),
              "cos_sin f32");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && K % 64 == 0, "w [N, K], K % 64");
  TORCH_CHECK(q_out.dim() == 3 && k_cache.dim() == 4 && v_cache.dim() == 4, "ranks");
  const int64_t Hq = q_out.size(1), D = q_out.size(2), Hkv = k_cache.size(1), BS = k_cache.size(2);
  TORCH_CHECK(D == 128 && k_cache.size(3) == D && v_cache.sizes() == k_cache.sizes(),
              "head_dim 128; k and v [NB,Hkv,BS,D]");
  TORCH_CHECK(N == (Hq + 2 * Hkv) * D && q_out.size(0) == M, "qkv width / q_out rows");
  TORCH_CHECK(pos.numel() == M && slots.numel() == M, "pos/slots length");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin [max_pos, D]");
  c10::DeviceGuard g(a.device());
  mlop::RopeEpi re{(uint16_t*)q_out.data_ptr(), (uint16_t*)k_cache.data_ptr(),
                   (uint16_t*)v_cache.data_ptr(), pos.data_ptr<int>(), cos_sin.data_ptr<float>(),
                   slots.data_ptr<int>(), (int)Hq, (int)Hkv, (int)BS};
  return mlop::launch_gemm_rope(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)M, (int)N, (int)K,
                                re, cur_stream());
}

bool gemm_rope_supported(int64_t M, int64_t N, int64_t K) {
  return mlop::gemm_rope_supported((int)M, (int)N, (int)K);
}

// ---- norm chain on the four-wave GEMM (large-M TP=1 decoder, unit norm weights) ----
// residual [M, N] += a . w^T in place; ss (f32, M * (N / 128 + 1)) = [M, N / 128] per-row,
// per-128-column partial sums of squares of the new residual, then the [M] row totals; false =
// the shape does not run on the four-wave kernel
bool w4_chain_ok_op(int64_t M, int64_t N, int64_t K) { return mlop::w4_chain_ok((int)M, (int)N, (int)K); }

static void check_ss(const Tensor& ss, int64_t M, int64_t H, const char* name) {
  TORCH_CHECK(ss.is_cuda() && ss.scalar_type() == at::kFloat && ss.is_contiguous() &&
                  ss.numel() == M * (H / 128 + 1), name, " must be f32 [M * (H / 128 + 1)] contiguous");
}

bool gemm_res_ss(Tensor residual, Tensor a, Tensor w, Tensor ss_out) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(residual, "residual");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "w [N, K]");
  TORCH_CHECK(residual.dim() == 2 && residual.size(0) == M && residual.size(1) == N && residual.stride(1) == 1 &&
                  residual.stride(0) % 8 == 0, "residual [M, N]");
  TORCH_CHECK(N % 128 == 0, "N % 128");
  check_ss(ss_out, M, N, "ss");
  if (M <= mlop::decode_chain_max_m()) {  // decode sizes: the GEMV (M <= 4) / weight-streaming MFMA chain
                 // (EPI_RES); its consumers take their row factors from the residual itself, so ss_out is not written
    if (residual.stride(0) != N || !mlop::decode_chain_takes((int)M, (int)N, (int)K, 0)) return false;
    c10::DeviceGuard g(a.device());
    if (M <= mlop::gemv_chain_max_m())
      mlop::launch_gemv_res(a.data_ptr(), (int)a.stride(0), w.data_ptr(), residual.data_ptr(), (int)M, (int)N,
                            (int)K, cur_stream());
    else
      mlop::launch_ws(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, residual.data_ptr(), (int)N, (int)M,
                      (int)N, (int)K, 5, false, mlop::RopeEpi{}, 0.f, cur_stream());
    return true;
  }
  mlop::RopeEpi re{};
  re.ss_out = ss_out.data_ptr<float>();
  re.ss_tot = re.ss_out + M * (N / 128);
  c10::DeviceGuard g(a.device());
  if (mlop::mid_chain_ok((int)M, (int)N, (int)K, 0))  // 5-64 rows: the planner's split-K tiles finish themselves
    return mlop::launch_mid_res_ss(a.data_ptr(), (int)a.stride(0), w.data_ptr(), residual.data_ptr(),
                                   (int)residual.stride(0), (int)M, (int)N, (int)K, re.ss_tot, cur_stream());
  return mlop::launch_w4_chain(4, a.data_ptr(), (int)a.stride(0), w.data_ptr(), residual.data_ptr(),
                               (int)residual.stride(0), (int)M, (int)N, (int)K, re, cur_stream());
}

// out = epi(diag(rsqrt(ss / K + eps)) . a . w^T): a is the un-normalised residual, ss_in its
// partial sums of squares (gemm_res_ss), w the consumer weight with the norm weight folded in
bool gemm_rs(Tensor out, Tensor a, Tensor w, Tensor ss_in, double eps, int64_t epi) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(out, "out");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "w [N, K]");
  TORCH_CHECK(epi == 0 || epi == 1, "epi");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == (epi == 0 ? N : N / 2) && out.stride(1) == 1 &&
                  out.stride(0) % 8 == 0, "out [M, N or N/2]");
  TORCH_CHECK(K % 128 == 0, "K % 128");
  check_ss(ss_in, M, K, "ss");
  if (M <= mlop::decode_chain_max_m()) {  // decode sizes: PRO_RS, row factors from the streamed chunks (ss_in unused)
    if (!mlop::decode_chain_takes((int)M, (int)N, (int)K, (int)epi)) return false;
    c10::DeviceGuard g(a.device());
    if (M <= mlop::gemv_chain_max_m())
      mlop::launch_gemv_rs(a.data_ptr(), (int)a.stride(0), w.data_ptr(), out.data_ptr(), (int)out.stride(0), (int)M,
                           (int)N, (int)K, (int)epi, mlop::RopeEpi{}, (float)eps, cur_stream());
    else
      mlop::launch_ws(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, out.data_ptr(), (int)out.stride(0),
                      (int)M, (int)N, (int)K, (int)epi, true, mlop::RopeEpi{}, (float)eps, cur_stream());
    return true;
  }
  mlop::RopeEpi re{};
  re.ss_in = ss_in.data_ptr<float>() + M * (K / 128);
  re.ss_inv_k = 1.f / (float)K;
  re.ss_eps = (float)eps;
  c10::DeviceGuard g(a.device());
  if (mlop::mid_chain_ok((int)M, (int)N, (int)K, (int)epi))  // 5-64 rows: the planner's SiLU tile, row-scaled
    return mlop::launch_mid_rs(a.data_ptr(), (int)a.stride(0), w.data_ptr(), out.data_ptr(), (int)out.stride(0),
                               (int)M, (int)N, (int)K, re.ss_in, (float)eps, cur_stream());
  return mlop::launch_w4_chain((int)epi | 8, a.data_ptr(), (int)a.stride(0), w.data_ptr(), out.data_ptr(),
                               (int)out.stride(0), (int)M, (int)N, (int)K, re, cur_stream());
}

// QKV projection of the norm chain: rows scaled as gemm_rs, then RoPE + paged K / staged V
bool gemm_rs_rope(Tensor q_out, Tensor k_cache, Tensor v_cache, Tensor a, Tensor w, Tensor pos, Tensor cos_sin,
                  Tensor slots, Tensor ss_in, double eps) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(q_out, "q_out"); check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache"); check_i32(pos, "pos"); check_i32(slots, "slots");
  TORCH_CHECK(cos_sin.is_cuda() && cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous(), "cos_sin f32");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && K % 64 == 0, "w [N, K], K % 64");
  TORCH_CHECK(q_out.dim() == 3 && k_cache.dim() == 4 && v_cache.dim() == 4, "ranks");
  const int64_t Hq = q_out.size(1), D = q_out.size(2), Hkv = k_cache.size(1), BS = k_cache.size(2);
  TORCH_CHECK(D == 128 && k_cache.size(3) == D && v_cache.sizes() == k_cache.sizes(),
              "head_dim 128; k and v [NB,Hkv,BS,D]");
  TORCH_CHECK(N == (Hq + 2 * Hkv) * D && q_out.size(0) == M, "qkv width / q_out rows");
  TORCH_CHECK(pos.numel() == M && slots.numel() == M, "pos/slots length");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin [max_pos, D]");
  TORCH_CHECK(K % 128 == 0, "K % 128");
  check_ss(ss_in, M, K, "ss");
  mlop::RopeEpi re{(uint16_t*)q_out.data_ptr(), (uint16_t*)k_cache.data_ptr(),
                   (uint16_t*)v_cache.data_ptr(), pos.data_ptr<int>(), cos_sin.data_ptr<float>(),
                   slots.data_ptr<int>(), (int)Hq, (int)Hkv, (int)BS};
  if (M <= mlop::decode_chain_max_m()) {  // decode sizes: PRO_RS + the RoPE / paged K/V epilogue (ss_in unused)
    if (!mlop::decode_chain_takes((int)M, (int)N, (int)K, 3)) return false;
    c10::DeviceGuard g(a.device());
    if (M <= mlop::gemv_chain_max_m())
      mlop::launch_gemv_rs(a.data_ptr(), (int)a.stride(0), w.data_ptr(), nullptr, 0, (int)M, (int)N, (int)K, 3, re,
                           (float)eps, cur_stream());
    else
      mlop::launch_ws(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, nullptr, 0, (int)M, (int)N, (int)K, 3,
                      true, re, (float)eps, cur_stream());
    return true;
  }
  re.ss_in = ss_in.data_ptr<float>() + M * (K / 128);
  re.ss_inv_k = 1.f / (float)K;
  re.ss_eps = (float)eps;
  if (mlop::mid_chain_ok((int)M, (int)N, (int)K, 3)) {  // 5-64 rows
    c10::DeviceGuard g(a.device());
    if (mlop::ws_prefer((int)M, (int)N, (int)K, 3)) {  // row scale computed from the streamed rows
      mlop::launch_ws(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, nullptr, 0, (int)M, (int)N, (int)K, 3,
                      true, re, (float)eps, cur_stream());
      return true;
    }
    return mlop::launch_gemm_rope(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)M, (int)N, (int)K, re,
                                  cur_stream());  // the slab path: row scale in the RoPE + cache reduce
  }
  if (!mlop::w4_chain_ok((int)M, (int)N, (int)K)) return false;
  c10::DeviceGuard g(a.device());
  return mlop::launch_w4_chain(3 | 8, a.data_ptr(), (int)a.stride(0), w.data_ptr(), nullptr, 0, (int)M, (int)N,
                               (int)K, re, cur_stream());
}

// out = rmsnorm(residual += a . w^T) * norm_w through the split-K path; false = not taken
bool gemm_add_rmsnorm(Tensor out, Tensor residual, Tensor a, Tensor w, Tensor norm_w, Tensor ws,
                      double eps) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(out, "out"); check_bf16(residual, "residual");
  check_bf16(norm_w, "norm_w");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 8 == 0, "w [N, K], K % 64");
  TORCH_CHECK(out.numel() == M * N && residual.numel() == M * N && norm_w.numel() == N, "shapes");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat, "ws f32");
  c10::DeviceGuard g(a.device());
  return mlop::launch_gemm_add_rmsnorm(a.data_ptr(), (int)a.stride(0), w.data_ptr(), out.data_ptr(),
                                       residual.data_ptr(), norm_w.data_ptr(), (float)eps,
                                       ws.data_ptr<float>(), ws.numel(), (int)M, (int)N, (int)K,
                                       cur_stream());
}

// Decode projection with the residual add + RMSNorm feeding it fused in as a prologue
// (gemv.hip NORM, M <= 4): res_out = bf16(res_in + y); out = epi(rmsnorm(res_out) * norm_w @ w^T).
// weight-streaming MFMA GEMM (gemm_ws.hip), plain / SiLU-mul / residual-add forms, optionally
// with the row-scale prologue; false = shape not taken
bool gemm_ws(Tensor out, Tensor a, Tensor w, int64_t epi, bool rs, double eps) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 2 && a.stride(1) == 1 &&
                  a.stride(0) % 8 == 0, "a must be bf16 [M, K], 16-B aligned rows");
  check_bf16(w, "w"); check_bf16(out, "out");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && w.stride(0) == K, "w [N, K] contiguous");
  TORCH_CHECK(epi == 0 || epi == 1 || epi == 5, "epi 0 / 1 / 5");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == (epi == 1 ? N / 2 : N) && out.stride(1) == 1,
              "out [M, N or N/2]");
  TORCH_CHECK(!(rs && epi == 5), "residual form has no row scale");
  if (!mlop::ws_takes((int)M, (int)N, (int)K, (int)epi)) return false;
  c10::DeviceGuard g(a.device());
  mlop::launch_ws(a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)K, out.data_ptr(), (int)out.stride(0), (int)M,
                  (int)N, (int)K, (int)epi, rs, mlop::RopeEpi{}, (float)eps, cur_stream());
  return true;
}

int64_t gemm_ws_max_m(int64_t set) { return mlop::gemm_ws_max_m((int)set); }
void gemm_ws_plan(int64_t rb, int64_t u, int64_t nt) { mlop::gemm_ws_plan((int)rb, (int)u, (int)nt); }
int64_t gemm_ws_small_m(int64_t set) { return mlop::gemm_ws_small_m((int)set); }
int64_t gemm_ws_rope_m(int64_t set) { return mlop::gemm_ws_rope_m((int)set); }
int64_t flash_persist(int64_t set) { return mlop::flash_persist((int)set); }
int64_t flash_stream(int64_t set) { return mlop::flash_stream((int)set); }
int64_t gemm_grouped_balance(int64_t set) { return mlop::gemm_grouped_balance((int)set); }
int64_t gemm_grouped_order(int64_t set) { return mlop::gemm_grouped_order((int)set); }
int64_t moe_mid_tok(int64_t set) { return mlop::moe_mid_tok((int)set); }
int64_t gemm_mid_chain(int64_t set) { return mlop::gemm_mid_chain((int)set); }
bool mid_chain_ok(int64_t M, int64_t N, int64_t K, int64_t epi) {
  return mlop::mid_chain_ok((int)M, (int)N, (int)K, (int)epi);
}

bool gemv_chain_supported(int64_t M, int64_t N, int64_t K, int64_t epi) {
  return mlop::decode_chain_takes((int)M, (int)N, (int)K, (int)epi);
}

int64_t decode_chain_max_m() { return mlop::decode_chain_max_m(); }

// grouped (MoE): rows of a sorted by group, offsets [G+1]; w [G, N, K]
void grouped_gemm(Tensor out, Tensor a, Tensor w, Tensor offsets, int64_t max_rows, int64_t epi,
                  std::optional<Tensor> a_rows) {
  check_bf16(out, "out"); check_bf16(a, "a"); check_bf16(w, "w"); check_i32(offsets, "offsets");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 3 && w.size(2) == a.size(1), "a [M, K], w [G, N, K]");
  // with a_rows the permuted rows are out's (M = out rows) and a holds the token rows they name
  const int64_t M = a_rows ? out.size(0) : a.size(0), K = a.size(1), N = w.size(1), G = w.size(0);
  TORCH_CHECK(offsets.numel() == G + 1, "offsets must be [G + 1]");
  TORCH_CHECK(K % 64 == 0 && N % 32 == 0, "K % 64, N % 32");
  TORCH_CHECK(out.size(0) == M && out.size(1) == (epi == 0 ? N : N / 2), "out shape");
  if (a_rows) {
    check_i32(*a_rows, "a_rows");
    TORCH_CHECK(a_rows->numel() >= M, "a_rows [M]: every permuted row's token row");
  }
  c10::DeviceGuard g(a.device());
  mlop::launch_grouped_gemm(a.data_ptr(), w.data_ptr(), out.data_ptr(), offsets.data_ptr<int>(),
                            (int)G, (int)M, (int)N, (int)K, (int)max_rows, (int)epi, cur_stream(),
                            a_rows ? a_rows->data_ptr<int>() : nullptr);
}

void moe_route(Tensor topw, Tensor topi, Tensor logits) {
  check_bf16(logits, "router logits");
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) <= 64, "router logits [T, E<=64]");
  const int64_t T = logits.size(0), E = logits.size(1), k = topi.size(1);
  TORCH_CHECK(k >= 1 && k <= E && k <= 8, "1 <= top_k <= min(E, 8)");
  check_i32(topi, "topi");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous() && topw.numel() == T * k &&
                  topi.numel() == T * k, "topw/topi [T, k]");
  c10::DeviceGuard g(logits.device());
  mlop::launch_moe_route(topw.data_ptr<float>(), topi.data_ptr<int>(), logits.data_ptr(), (int)T,
                         (int)E, (int)k, cur_stream());
}

void moe_permute(Tensor xp, Tensor offsets, Tensor src, Tensor inv, Tensor x, Tensor topi,
                 int64_t e0, int64_t n_local) {
  check_bf16(xp, "xp"); check_bf16(x, "x"); check_i32(offsets, "offsets"); check_i32(src, "src");
  check_i32(inv, "inv"); check_i32(topi, "topi");
  const int64_t T = topi.size(0), k = topi.size(1), H = x.size(1);
  TORCH_CHECK(x.dim() == 2 && x.size(0) == T && H % 8 == 0, "x [T, H]");
  TORCH_CHECK(xp.size(0) == T * k && xp.size(1) == H, "xp [T*k, H]");
  TORCH_CHECK(n_local >= 1 && n_local <= 256 && offsets.numel() == n_local + 1, "offsets");
  TORCH_CHECK(src.numel() == T * k && inv.numel() == T * k, "src/inv [T*k]");
  c10::DeviceGuard g(x.device());
  mlop::launch_moe_permute(xp.data_ptr(), offsets.data_ptr<int>(), src.data_ptr<int>(),
                           inv.data_ptr<int>(), x.data_ptr(), topi.data_ptr<int>(), (int)T, (int)k,
                           (int)H, (int)e0, (int)n_local, cur_stream());
}

// decode-size dispatch (T <= 16): router GEMV + route + sort + gather in one launch; false = not taken
bool moe_dispatch_small(Tensor topw, Tensor topi, Tensor xp, Tensor offsets, Tensor src, Tensor inv, Tensor x,
                        Tensor router_w, int64_t e0, int64_t n_local, std::optional<Tensor> pro_y,
                        std::optional<Tensor> pro_res, std::optional<Tensor> pro_w, double pro_eps) {
  check_bf16(xp, "xp"); check_bf16(x, "x"); check_bf16(router_w, "router_w"); check_i32(topi, "topi");
  check_i32(offsets, "offsets"); check_i32(src, "src"); check_i32(inv, "inv");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous(), "topw f32");
  const int64_t T = x.size(0), H = x.size(1), E = router_w.size(0), k = topi.size(1);
  if (!mlop::moe_dispatch_small_takes((int)T, (int)E, (int)k, (int)H)) return false;
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && router_w.size(1) == H, "x [T, H], router_w [E, H]");
  TORCH_CHECK(topi.size(0) == T && topw.numel() == T * k && xp.size(0) == T * k && xp.size(1) == H,
              "topi/topw [T, k], xp [T*k, H]");
  TORCH_CHECK(n_local >= 1 && n_local <= 64 && offsets.numel() == n_local + 1 && src.numel() == T * k &&
                  inv.numel() == T * k, "offsets / src / inv");
  const bool pro = pro_y.has_value();
  if (pro) {  // x is the OUTPUT of the prologue here
    check_bf16(*pro_y, "pro_y"); check_bf16(*pro_res, "pro_res"); check_bf16(*pro_w, "pro_w");
    TORCH_CHECK(pro_y->numel() == T * H && pro_res->numel() == T * H && pro_w->numel() == H && H <= 8192,
                "prologue y / residual [T, H], w [H]");
  }
  c10::DeviceGuard g(x.device());
  mlop::launch_moe_dispatch_small(topw.data_ptr<float>(), topi.data_ptr<int>(), xp.data_ptr(),
                                  offsets.data_ptr<int>(), src.data_ptr<int>(), inv.data_ptr<int>(), x.data_ptr(),
                                  router_w.data_ptr(), (int)T, (int)E, (int)k, (int)H, (int)e0, (int)n_local,
                                  pro ? pro_y->data_ptr() : nullptr, pro ? pro_res->data_ptr() : nullptr,
                                  pro ? pro_w->data_ptr() : nullptr, (float)pro_eps, pro ? x.data_ptr() : nullptr,
                                  cur_stream());
  return true;
}

// mid-size dispatch (16 < T <= moe_mid_max_tokens): router GEMV + route per workgroup, the last sorts; no
// gather (arow: token row of each permuted row); false = not taken
bool moe_dispatch_mid(Tensor topw, Tensor topi, Tensor offsets, Tensor arow, Tensor inv, Tensor x, Tensor router_w,
                      int64_t e0, int64_t n_local, std::optional<Tensor> pro_y, std::optional<Tensor> pro_res,
                      std::optional<Tensor> pro_w, double pro_eps) {
  check_bf16(x, "x"); check_bf16(router_w, "router_w"); check_i32(topi, "topi");
  check_i32(offsets, "offsets"); check_i32(arow, "arow"); check_i32(inv, "inv");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous(), "topw f32");
  const int64_t T = x.size(0), H = x.size(1), E = router_w.size(0), k = topi.size(1);
  if (!mlop::moe_dispatch_mid_takes((int)T, (int)E, (int)k, (int)H)) return false;
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && router_w.size(1) == H && router_w.is_contiguous(),
              "x [T, H], router_w [E, H]");
  TORCH_CHECK(topi.size(0) == T && topi.is_contiguous() && topw.numel() == T * k, "topi/topw [T, k]");
  TORCH_CHECK(n_local >= 1 && n_local <= 64 && offsets.numel() == n_local + 1 && arow.numel() == T * k &&
                  inv.numel() == T * k, "offsets / arow / inv");
  const bool pro = pro_y.has_value();
  if (pro) {  // x is the OUTPUT of the prologue here
    check_bf16(*pro_y, "pro_y"); check_bf16(*pro_res, "pro_res"); check_bf16(*pro_w, "pro_w");
    TORCH_CHECK(pro_y->numel() == T * H && pro_res->numel() == T * H && pro_w->numel() == H && H <= 8192,
                "prologue y / residual [T, H], w [H]");
  }
  c10::DeviceGuard g(x.device());
  mlop::launch_moe_dispatch_mid(topw.data_ptr<float>(), topi.data_ptr<int>(), offsets.data_ptr<int>(),
                                arow.data_ptr<int>(), inv.data_ptr<int>(), x.data_ptr(), router_w.data_ptr(), (int)T,
                                (int)E, (int)k, (int)H, (int)e0, (int)n_local, pro ? pro_y->data_ptr() : nullptr,
                                pro ? pro_res->data_ptr() : nullptr, pro ? pro_w->data_ptr() : nullptr, (float)pro_eps,
                                pro ? x.data_ptr() : nullptr, cur_stream());
  return true;
}

bool moe_combine_add_rmsnorm(Tensor out, Tensor residual, Tensor y, Tensor inv, Tensor topw, Tensor norm_w,
                             double eps) {
  check_bf16(out, "out"); check_bf16(residual, "residual"); check_bf16(y, "y"); check_bf16(norm_w, "norm_w");
  check_i32(inv, "inv");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous() && topw.dim() == 2, "topw");
  const int64_t T = topw.size(0), k = topw.size(1), H = y.size(1);
  TORCH_CHECK(out.numel() == T * H && residual.numel() == T * H && inv.numel() == T * k && norm_w.numel() == H,
              "combine + norm shapes");
  c10::DeviceGuard g(y.device());
  return mlop::launch_moe_combine_add_rmsnorm(out.data_ptr(), residual.data_ptr(), y.data_ptr(),
                                              inv.data_ptr<int>(), topw.data_ptr<float>(), norm_w.data_ptr(),
                                              (float)eps, (int)T, (int)k, (int)H, cur_stream());
}

// grouped down GEMM + combine + residual add + RMSNorm: the combine sums the GEMM's split-K slabs
// itself (y is written only when the GEMM does not split); false = shape not supported
bool moe_down_combine_add_rmsnorm(Tensor out, Tensor residual, Tensor y, Tensor a, Tensor w2, Tensor offsets,
                                  int64_t max_rows, Tensor inv, Tensor topw, Tensor norm_w, double eps) {
  check_bf16(out, "out"); check_bf16(residual, "residual"); check_bf16(y, "y"); check_bf16(a, "a");
  check_bf16(w2, "w2"); check_bf16(norm_w, "norm_w"); check_i32(offsets, "offsets"); check_i32(inv, "inv");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous() && topw.dim() == 2, "topw");
  TORCH_CHECK(a.dim() == 2 && w2.dim() == 3 && w2.size(2) == a.size(1), "a [R, I], w2 [G, H, I]");
  const int64_t R = a.size(0), I = a.size(1), H = w2.size(1), G = w2.size(0);
  const int64_t T = topw.size(0), k = topw.size(1);
  TORCH_CHECK(offsets.numel() == G + 1 && I % 64 == 0 && H % 32 == 0, "offsets [G + 1], I % 64, H % 32");
  TORCH_CHECK(y.size(0) == R && y.size(1) == H && out.numel() == T * H && residual.numel() == T * H &&
                  inv.numel() == T * k && norm_w.numel() == H, "y [R, H], out / residual [T, H]");
  c10::DeviceGuard g(a.device());
  return mlop::launch_moe_down_combine_add_rmsnorm(
      out.data_ptr(), residual.data_ptr(), y.data_ptr(), a.data_ptr(), w2.data_ptr(), offsets.data_ptr<int>(), (int)G,
      (int)R, (int)H, (int)I, (int)max_rows, inv.data_ptr<int>(), topw.data_ptr<float>(), norm_w.data_ptr(),
      (float)eps, (int)T, (int)k, cur_stream());
}

void moe_combine(Tensor out, Tensor y, Tensor inv, Tensor topw) {
  check_bf16(out, "out"); check_bf16(y, "y"); check_i32(inv, "inv");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_contiguous() && topw.dim() == 2, "topw");
  const int64_t T = topw.size(0), k = topw.size(1), H = y.size(1);
  TORCH_CHECK(out.size(0) == T && out.size(1) == H && inv.numel() == T * k && H % 8 == 0,
              "combine shapes");
  c10::DeviceGuard g(y.device());
  mlop::launch_moe_combine(out.data_ptr(), y.data_ptr(), inv.data_ptr<int>(),
                           topw.data_ptr<float>(), (int)T, (int)k, (int)H, cur_stream());
}

void check_logits(const Tensor& logits) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.dim() == 2 &&
                  logits.stride(1) == 1 && logits.stride(0) % 4 == 0,
              "logits must be f32 [n, V] with unit inner stride and 16-B aligned rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0, "logits 16-B aligned");
}

void argmax(Tensor out, Tensor logits) {
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == logits.size(0), "out int64 [n]");
  if (logits.scalar_type() == at::kBFloat16) {
    TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0,
                "bf16 logits must be [n, V] with unit inner stride and 16-B aligned rows");
    c10::DeviceGuard g(logits.device());
    const int n = (int)logits.size(0), V = (int)logits.size(1);
    const int S = mlop::argmax_splits(n, V);
    at::Tensor ws;  // per-(row, split) keys from the caching allocator (graph-capture safe)
    if (S > 1) ws = at::empty({(int64_t)n * S}, logits.options().dtype(at::kLong));
    mlop::launch_argmax_bf16(out.data_ptr<int64_t>(), logits.data_ptr(), n, V, logits.stride(0),
                             S > 1 ? ws.data_ptr() : nullptr, cur_stream());
    return;
  }
  check_logits(logits);
  c10::DeviceGuard g(logits.device());
  mlop::launch_argmax(out.data_ptr<int64_t>(), logits.data_ptr<float>(), (int)logits.size(0),
                      (int)logits.size(1), logits.stride(0), cur_stream());
}

void sample(Tensor out, Tensor logits, Tensor temps, Tensor top_ks, Tensor top_ps, Tensor uniform, bool full) {
  check_logits(logits);
  const int64_t n = logits.size(0);
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == n, "out int64 [n]");
  TORCH_CHECK(temps.scalar_type() == at::kFloat && temps.numel() == n && temps.is_cuda(), "temps");
  TORCH_CHECK(top_ps.scalar_type() == at::kFloat && top_ps.numel() == n && top_ps.is_cuda(), "top_ps");
  TORCH_CHECK(uniform.scalar_type() == at::kFloat && uniform.numel() == n && uniform.is_cuda(), "u");
  check_i32(top_ks, "top_ks");
  TORCH_CHECK(top_ks.numel() == n, "top_ks");
  c10::DeviceGuard g(logits.device());
  const long wsb = mlop::sample_workspace_bytes((int)n, (int)logits.size(1));
  at::Tensor ws;  // candidate buffers from the caching allocator (graph-capture safe)
  if (wsb > 0) ws = at::empty({wsb}, logits.options().dtype(at::kByte));
  mlop::launch_sample(out.data_ptr<int64_t>(), logits.data_ptr<float>(), (int)n,
                      (int)logits.size(1), logits.stride(0), temps.data_ptr<float>(),
                      top_ks.data_ptr<int>(), top_ps.data_ptr<float>(), uniform.data_ptr<float>(),
                      wsb > 0 ? ws.data_ptr() : nullptr, full, cur_stream());
}


// ---- K15 custom all-reduce: host-side state, int handles -------------------
int64_t car_create(int64_t rank, int64_t world, int64_t max_bytes, int64_t device, bool split) {
  return mlop::car_create((int)rank, (int)world, (long)max_bytes, (int)device, split ? 1 : 0);
}
Tensor car_ipc_handle(int64_t h) {
  Tensor t = at::empty({128}, at::TensorOptions().dtype(at::kByte));
  mlop::car_ipc_handle((long)h, t.data_ptr());
  return t;
}
void car_open(int64_t h, Tensor handles) {
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.is_contiguous() &&
              handles.dim() == 2 && handles.size(1) == 128, "handles: CPU uint8 [world, 128]");
  mlop::car_open((long)h, handles.data_ptr());
}
void car_all_reduce(int64_t h, Tensor out, Tensor inp, bool two_shot) {
  check_bf16(out, "out"); check_bf16(inp, "inp");
  TORCH_CHECK(out.numel() == inp.numel(), "all_reduce: out/inp size mismatch");
  TORCH_CHECK(inp.numel() % 8 == 0, "all_reduce: numel must be a multiple of 8");
  TORCH_CHECK(inp.numel() * 2 * (two_shot ? 2 : 1) <= mlop::car_max_bytes((long)h),
              "all_reduce: message exceeds the registered buffer");
  c10::DeviceGuard g(inp.device());
  mlop::car_all_reduce((long)h, out.data_ptr(), inp.data_ptr(), (long)inp.numel(), cur_stream(), two_shot);
}
// residual = bf16(residual + bf16(sum over ranks of inp)): one-shot all-reduce + the residual add
void car_all_reduce_add(int64_t h, Tensor residual, Tensor inp) {
  check_bf16(residual, "residual"); check_bf16(inp, "inp");
  TORCH_CHECK(residual.numel() == inp.numel() && residual.is_contiguous() && inp.is_contiguous(),
              "all_reduce_add: contiguous residual / inp of one size");
  TORCH_CHECK(residual.data_ptr() != inp.data_ptr(), "all_reduce_add: residual must not alias inp");
  TORCH_CHECK(inp.numel() % 8 == 0, "all_reduce_add: numel must be a multiple of 8");
  TORCH_CHECK(inp.numel() * 2 <= mlop::car_max_bytes((long)h), "all_reduce_add: message exceeds the registered buffer");
  c10::DeviceGuard g(inp.device());
  mlop::car_all_reduce((long)h, residual.data_ptr(), inp.data_ptr(), (long)inp.numel(), cur_stream(), false, true);
}
// in-place broadcast of any contiguous device tensor (bytes % 16 == 0) from `root`
void car_broadcast(int64_t h, Tensor buf, int64_t root) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "broadcast: contiguous device tensor");
  const long nbytes = (long)(buf.numel() * buf.element_size());
  c10::DeviceGuard g(buf.device());
  mlop::car_broadcast((long)h, buf.data_ptr(), buf.data_ptr(), nbytes, (int)root, cur_stream());
}
// out [world * piece] <- every rank's contiguous piece (bytes % 4 == 0), rank order
void car_all_gather(int64_t h, Tensor out, Tensor piece) {
  TORCH_CHECK(piece.is_cuda() && piece.is_contiguous() && out.is_cuda() && out.is_contiguous() &&
                  out.scalar_type() == piece.scalar_type(), "all-gather: contiguous device tensors of one dtype");
  const long nbytes = (long)(piece.numel() * piece.element_size());
  c10::DeviceGuard g(piece.device());
  mlop::car_all_gather((long)h, out.data_ptr(), (long)(out.numel() * out.element_size()), piece.data_ptr(), nbytes,
                       cur_stream());
}
int64_t car_error(int64_t h) { return mlop::car_error((long)h); }
int64_t car_mem_mode(int64_t h) { return mlop::car_mem_mode((long)h); }
void car_destroy(int64_t h) { mlop::car_destroy((long)h); }

// ---- TP step-header channel over POSIX shared memory (shm_channel.cc) -------------
int64_t chan_create(std::string name, int64_t slots, int64_t consumers) {
  return mlop::chan_create(name, (int)slots, (int)consumers);
}
int64_t chan_open(std::string name) { return mlop::chan_open(name); }
bool chan_send(int64_t h, Tensor vals, int64_t timeout_us) {
  TORCH_CHECK(!vals.is_cuda() && vals.scalar_type() == at::kLong && vals.is_contiguous(), "vals: CPU int64");
  return mlop::chan_send((long)h, vals.data_ptr<int64_t>(), (int)vals.numel(), (long)timeout_us);
}
bool chan_recv(int64_t h, int64_t consumer, Tensor out, int64_t timeout_us) {
  TORCH_CHECK(!out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous(), "out: CPU int64");
  return mlop::chan_recv((long)h, (int)consumer, out.data_ptr<int64_t>(), (int)out.numel(), (long)timeout_us);
}
void chan_unlink(std::string name) { mlop::chan_unlink(name); }
void chan_close(int64_t h, bool unlink) { mlop::chan_close((long)h, unlink); }
int64_t xg_create(std::string name, int64_t world, int64_t slots, int64_t max_words) {
  return mlop::xg_create(name, (int)world, (int)slots, (long)max_words);
}
int64_t xg_open(std::string name, int64_t rank) { return mlop::xg_open(name, (int)rank); }
bool xg_exchange(int64_t h, Tensor vals, Tensor out, Tensor counts, int64_t timeout_us) {
  const long mw = mlop::xg_max_words((long)h);
  TORCH_CHECK(!vals.is_cuda() && vals.scalar_type() == at::kLong && vals.is_contiguous() && vals.dim() == 1,
              "xg_exchange: vals must be a contiguous CPU int64 vector");
  TORCH_CHECK(!out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && out.dim() == 2 &&
              out.size(1) == mw, "xg_exchange: out must be CPU int64 [world, max_words]");
  TORCH_CHECK(!counts.is_cuda() && counts.scalar_type() == at::kLong && counts.is_contiguous() &&
              counts.numel() == out.size(0), "xg_exchange: counts must be CPU int64 [world]");
  return mlop::xg_exchange((long)h, vals.data_ptr<int64_t>(), (long)vals.numel(), out.data_ptr<int64_t>(),
                           counts.data_ptr<int64_t>(), (long)timeout_us);
}
void xg_close(int64_t h) { mlop::xg_close((long)h); }

// ---- expert-parallel exchange over IPC peer memory (ep_exchange.hip) -------------
int64_t ep_create(int64_t rank, int64_t world, int64_t E, int64_t k, int64_t H, int64_t tcap, int64_t device) {
  return mlop::ep_create((int)rank, (int)world, (int)E, (int)k, (int)H, (int)tcap, (int)device);
}
Tensor ep_ipc_handle(int64_t h) {
  Tensor t = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  mlop::ep_ipc_handle((long)h, t.data_ptr());
  return t;
}
void ep_open(int64_t h, Tensor handles) {
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.is_contiguous() &&
              handles.dim() == 2 && handles.size(1) == 64, "handles: CPU uint8 [world, 64]");
  mlop::ep_open((long)h, handles.data_ptr());
}
// xp [rows, H] bf16 <- this rank's received rows grouped by local expert; offsets int32 [n_local + 1]
void ep_dispatch(int64_t h, Tensor xp, Tensor offsets, Tensor x, Tensor topi) {
  const long H = mlop::ep_hidden((long)h), k = mlop::ep_topk((long)h);
  check_bf16(xp, "xp"); check_bf16(x, "x"); check_i32(topi, "topi"); check_i32(offsets, "offsets");
  TORCH_CHECK(x.dim() == 2 && x.size(1) == H && xp.dim() == 2 && xp.size(1) == H, "ep_dispatch: [*, H] rows");
  TORCH_CHECK(topi.dim() == 2 && topi.size(0) == x.size(0) && topi.size(1) == k, "ep_dispatch: topi [T, k]");
  TORCH_CHECK(offsets.numel() == mlop::ep_local_experts((long)h) + 1, "ep_dispatch: offsets [n_local + 1]");
  TORCH_CHECK(x.size(0) <= mlop::ep_tcap((long)h), "ep_dispatch: T exceeds the exchange's token capacity");
  c10::DeviceGuard g(x.device());
  mlop::ep_dispatch((long)h, xp.data_ptr(), (long)xp.size(0), offsets.data_ptr<int>(), x.data_ptr(),
                    topi.data_ptr<int>(), (int)x.size(0), cur_stream());
}
// out [T, H] bf16 <- sum_j topw[t, j] * expert_j(x[t]) from the owners of the experts
void ep_combine(int64_t h, Tensor out, Tensor y, Tensor topw, Tensor topi) {
  const long H = mlop::ep_hidden((long)h), k = mlop::ep_topk((long)h);
  check_bf16(out, "out"); check_bf16(y, "y"); check_i32(topi, "topi");
  TORCH_CHECK(topw.scalar_type() == at::kFloat && topw.is_cuda() && topw.is_contiguous(), "topw fp32");
  TORCH_CHECK(out.dim() == 2 && out.size(1) == H && y.dim() == 2 && y.size(1) == H, "ep_combine: [*, H] rows");
  TORCH_CHECK(topw.numel() == out.size(0) * k && topi.numel() == out.size(0) * k, "ep_combine: [T, k] routing");
  c10::DeviceGuard g(out.device());
  mlop::ep_combine((long)h, out.data_ptr(), y.data_ptr(), (long)y.size(0), topw.data_ptr<float>(),
                   topi.data_ptr<int>(), (int)out.size(0), cur_stream());
}
int64_t ep_error(int64_t h) { return mlop::ep_error((long)h); }
int64_t ep_mem_mode(int64_t h) { return mlop::ep_mem_mode((long)h); }
void ep_destroy(int64_t h) { mlop::ep_destroy((long)h); }

}  // namespace

// sha256 of the sources this library was built from (ops/build.py writes srchash.cpp)
extern "C" const char* mlop_src_hash();
std::string src_hash() { return std::string(mlop_src_hash()); }

TORCH_LIBRARY(mlop, m) {
  m.def("src_hash() -> str", &src_hash);
  m.def("device_delay(int us) -> ()", &device_delay);
  m.def("car_create(int rank, int world, int max_bytes, int device, bool split=False) -> int", &car_create);
  m.def("car_ipc_handle(int h) -> Tensor", &car_ipc_handle);
  m.def("car_open(int h, Tensor handles) -> ()", &car_open);
  m.def("car_all_reduce(int h, Tensor(a!) out, Tensor inp, bool two_shot=False) -> ()");
  m.def("car_all_reduce_add(int h, Tensor(a!) residual, Tensor inp) -> ()");
  m.def("car_broadcast(int h, Tensor(a!) buf, int root) -> ()");
  m.def("car_all_gather(int h, Tensor(a!) out, Tensor piece) -> ()");
  m.def("car_error(int h) -> int", &car_error);
  m.def("attn_fused_max_pairs(int n) -> int", &attn_fused_max_pairs);
  m.def("car_mem_mode(int h) -> int", &car_mem_mode);
  m.def("car_destroy(int h) -> ()", &car_destroy);
  m.def("chan_create(str name, int slots, int consumers) -> int", &chan_create);
  m.def("chan_open(str name) -> int", &chan_open);
  m.def("chan_send(int h, Tensor vals, int timeout_us) -> bool", &chan_send);
  m.def("chan_recv(int h, int consumer, Tensor(a!) out, int timeout_us) -> bool", &chan_recv);
  m.def("chan_unlink(str name) -> ()", &chan_unlink);
  m.def("chan_close(int h, bool unlink) -> ()", &chan_close);
  m.def("xg_create(str name, int world, int slots, int max_words) -> int", &xg_create);
  m.def("xg_open(str name, int rank) -> int", &xg_open);
  m.def("xg_exchange(int h, Tensor vals, Tensor(a!) out, Tensor(b!) counts, int timeout_us) -> bool", &xg_exchange);
  m.def("xg_close(int h) -> ()", &xg_close);
  m.def("ep_create(int rank, int world, int E, int k, int H, int tcap, int device) -> int", &ep_create);
  m.def("ep_ipc_handle(int h) -> Tensor", &ep_ipc_handle);
  m.def("ep_open(int h, Tensor handles) -> ()", &ep_open);
  m.def("ep_dispatch(int h, Tensor(a!) xp, Tensor(b!) offsets, Tensor x, Tensor topi) -> ()");
  m.def("ep_combine(int h, Tensor(a!) out, Tensor y, Tensor topw, Tensor topi) -> ()");
  m.def("ep_error(int h) -> int", &ep_error);
  m.def("ep_mem_mode(int h) -> int", &ep_mem_mode);
  m.def("ep_destroy(int h) -> ()", &ep_destroy);
  m.def("gemm_workspace(int M, int N, int K, int epi) -> int", &gemm_workspace);
  m.def("gemm_big_variant(int set=-1) -> int", &gemm_big_variant);
  m.def("gemm_half_tile(int set=-1) -> int", &gemm_half_tile);
  m.def("gemm_small_nt(int set=-1) -> int", &gemm_small_nt);
  m.def("attn_kv_nt(int set=-1) -> int", &attn_kv_nt);
  m.def("gemm_slab_nt(int set=-1) -> int", &gemm_slab_nt);
  m.def("gemm_rope_split(int set=-1) -> int", &gemm_rope_split);
  m.def("gemm_split_target(int set=-1) -> int", &gemm_split_target);
  m.def("gemm_grouped_narrow(int set=-1) -> int", &gemm_grouped_narrow);
  m.def("gemm_ws_max_m(int set=-1) -> int", &gemm_ws_max_m);
  m.def("decode_chain_max_m() -> int", &decode_chain_max_m);
  m.def("gemm_ws_plan(int rb, int u, int nt) -> ()", &gemm_ws_plan);
  m.def("gemm_ws_small_m(int set=-1) -> int", &gemm_ws_small_m);
  m.def("gemm_ws_rope_m(int set=-1) -> int", &gemm_ws_rope_m);
  m.def("flash_persist(int set=-1) -> int", &flash_persist);
  m.def("flash_stream(int set=-1) -> int", &flash_stream);
  m.def("gemm_grouped_balance(int set=-1) -> int", &gemm_grouped_balance);
  m.def("gemm_grouped_order(int set=-1) -> int", &gemm_grouped_order);
  m.def("moe_mid_tok(int set=-1) -> int", &moe_mid_tok);
  m.def("gemm_mid_chain(int set=-1) -> int", &gemm_mid_chain);
  m.def("mid_chain_ok(int M, int N, int K, int epi) -> bool", &mid_chain_ok);
  m.def("moe_mid_max_tokens(int set=-1) -> int", &moe_mid_max_tokens);
  m.def("gemm_grouped_plan(int bm, int bn, int stages, int splits) -> ()", &gemm_grouped_plan);
  m.def("gemm_dense_plan(int variant, int bm, int bn, int splits, int stages=0) -> ()", &gemm_dense_plan);
  m.def("gemm_small_stages(int set=-1) -> int", &gemm_small_stages);
  m.def("gemm_small_tile(int set=-1) -> int", &gemm_small_tile);
  m.def("gemm_sk_mode(int set=-1) -> int", &gemm_sk_mode);
  m.def("gemm_sk_reserve() -> bool", &gemm_sk_reserve);
  m.def("gemm_sk_workgroups(int M, int N, int K) -> int", &gemm_sk_workgroups);
  m.def("vmm_supported(int device) -> bool", &vmm_supported);
  m.def("vmm_granularity(int device) -> int", &vmm_granularity);
  m.def("vmm_arena(int bytes, int device) -> Tensor", &vmm_arena);
  m.def("vmm_map_chunks(Tensor flat, int region_stride, int n_regions, int chunk_bytes, int first, "
        "int count, bool async_) -> bool", &vmm_map_chunks);
  m.def("vmm_chunks_ready(Tensor flat) -> int", &vmm_chunks_ready);
  m.def("vmm_error(Tensor flat) -> int", &vmm_error);
  m.def("gemm_rope_supported(int M, int N, int K) -> bool", &gemm_rope_supported);
  m.def("w4_chain_ok(int M, int N, int K) -> bool", &w4_chain_ok_op);
  m.def("gemm_res_ss(Tensor(a!) residual, Tensor a, Tensor w, Tensor(b!) ss_out) -> bool");
  m.def("gemm_rs(Tensor(a!) out, Tensor a, Tensor w, Tensor ss_in, float eps, int epi) -> bool");
  m.def("gemm_rs_rope(Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor a, Tensor w, "
        "Tensor pos, Tensor cos_sin, Tensor slots, Tensor ss_in, float eps) -> bool");
  m.def("gemm_rope_cache(Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor a, Tensor w, "
        "Tensor pos, Tensor cos_sin, Tensor slots) -> bool");
  m.def("gemm(Tensor(a!) out, Tensor a, Tensor w, Tensor(b!) ws, int epi) -> ()");
  m.def("grouped_gemm(Tensor(a!) out, Tensor a, Tensor w, Tensor offsets, int max_rows, "
        "int epi, Tensor? a_rows=None) -> ()");
  m.def("gemm_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor a, Tensor w, Tensor norm_w, "
        "Tensor(c!) ws, float eps) -> bool");
  m.def("gemv_chain_supported(int M, int N, int K, int epi) -> bool", &gemv_chain_supported);
  m.def("moe_route(Tensor(a!) topw, Tensor(b!) topi, Tensor logits) -> ()");
  m.def("moe_permute(Tensor(a!) xp, Tensor(b!) offsets, Tensor(c!) src, Tensor(d!) inv, Tensor x, "
        "Tensor topi, int e0, int n_local) -> ()");
  m.def("moe_combine(Tensor(a!) out, Tensor y, Tensor inv, Tensor topw) -> ()");
  m.def("moe_dispatch_small(Tensor(a!) topw, Tensor(b!) topi, Tensor(c!) xp, Tensor(d!) offsets, Tensor(e!) src, "
        "Tensor(f!) inv, Tensor(g!) x, Tensor router_w, int e0, int n_local, Tensor? pro_y=None, "
        "Tensor(h!)? pro_res=None, Tensor? pro_w=None, float pro_eps=0.0) -> bool");
  m.def("moe_dispatch_mid(Tensor(a!) topw, Tensor(b!) topi, Tensor(c!) offsets, Tensor(d!) arow, Tensor(e!) inv, "
        "Tensor(f!) x, Tensor router_w, int e0, int n_local, Tensor? pro_y=None, Tensor(g!)? pro_res=None, "
        "Tensor? pro_w=None, float pro_eps=0.0) -> bool");
  m.def("moe_down_combine_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor(c!) y, Tensor a, Tensor w2, "
        "Tensor offsets, int max_rows, Tensor inv, Tensor topw, Tensor norm_w, float eps) -> bool");
  m.def("moe_combine_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor y, Tensor inv, Tensor topw, "
        "Tensor norm_w, float eps) -> bool");
  m.def("argmax(Tensor(a!) out, Tensor logits) -> ()");
  m.def("sample(Tensor(a!) out, Tensor logits, Tensor temps, Tensor top_ks, Tensor top_ps, "
        "Tensor uniform, bool full) -> ()");
  m.def("rmsnorm(Tensor(a!) out, Tensor x, Tensor w, float eps) -> ()");
  m.def("add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor x, Tensor w, float eps) -> ()");
  m.def("rope_cache(Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor qkv, "
        "Tensor pos, Tensor cos_sin, Tensor slots) -> ()");
  m.def("silu_mul(Tensor(a!) out, Tensor x, int interleaved=0) -> ()");
  m.def("embedding(Tensor(a!) out, Tensor table, Tensor ids, int vocab_start) -> ()");
  m.def("gemm_ws(Tensor(a!) out, Tensor a, Tensor w, int epi, bool rs, float eps) -> bool");
  m.def("flash_prefill(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor ptile_seq, Tensor ptile_q0, Tensor q_start, Tensor q_len, Tensor ctx_len, float scale) -> ()");
  m.def("paged_attention(Tensor(a!) out, Tensor(b!) part_o, Tensor(c!) part_ml, Tensor(d!) part_sem, Tensor q, "
        "Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor tile_seq, Tensor tile_q0, "
        "Tensor q_start, Tensor q_len, Tensor ctx_len, float scale, int part_tokens, "
        "int nparts) -> ()");
}

TORCH_LIBRARY_IMPL(mlop, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("add_rmsnorm", &add_rmsnorm);
  m.impl("rope_cache", &rope_cache);
  m.impl("silu_mul", &silu_mul);
  m.impl("embedding", &embedding);
  m.impl("paged_attention", &paged_attention);
  m.impl("flash_prefill", &flash_prefill);
  m.impl("gemm", &gemm);
  m.impl("gemm_ws", &gemm_ws);
  m.impl("grouped_gemm", &grouped_gemm);
  m.impl("gemm_add_rmsnorm", &gemm_add_rmsnorm);
  m.impl("gemm_res_ss", &gemm_res_ss);
  m.impl("gemm_rs", &gemm_rs);
  m.impl("gemm_rs_rope", &gemm_rs_rope);
  m.impl("gemm_rope_cache", &gemm_rope_cache);
  m.impl("moe_route", &moe_route);
  m.impl("moe_dispatch_small", &moe_dispatch_small);
  m.impl("moe_dispatch_mid", &moe_dispatch_mid);
  m.impl("moe_down_combine_add_rmsnorm", &moe_down_combine_add_rmsnorm);
  m.impl("moe_combine_add_rmsnorm", &moe_combine_add_rmsnorm);
  m.impl("moe_permute", &moe_permute);
  m.impl("moe_combine", &moe_combine);
  m.impl("argmax", &argmax);
  m.impl("sample", &sample);
  m.impl("car_all_reduce", &car_all_reduce);
  m.impl("car_all_reduce_add", &car_all_reduce_add);
  m.impl("car_broadcast", &car_broadcast);
  m.impl("car_all_gather", &car_all_gather);
  m.impl("ep_dispatch", &ep_dispatch);
  m.impl("ep_combine", &ep_combine);
}
