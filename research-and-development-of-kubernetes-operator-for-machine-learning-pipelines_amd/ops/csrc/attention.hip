// Paged attention over the block-table KV cache (K6 decode, and the ragged /
// chunked-prefill path of K7) with MFMA 16x16x32 bf16 on gfx950.
//
// Layouts (written by rope_cache.hip and the fused QKV GEMM epilogues):
//   k_cache[page, Hkv, 16, 128]  token-major  -> A operand of  S^T = K . Q^T
//   v_cache[page, Hkv, 16, 128]  token-major  -> staged in LDS, read back transposed
//                                                (ds_read_b64_tr_b16) as the A operand of
//                                                O^T = V^T . P^T
// A token's V row is one contiguous 256-B store for its writer (a decode token used to scatter
// 128 2-B stores over a dim-major page; scripts/bench_vt.py measured the two layouts).
// Both products keep the q-row on the lane (col = lane&15), so the online
// softmax (max, exp2, rescale of O) is entirely lane-local except the two
// cross-lane max steps (xor 16, xor 32), and P^T feeds the second MFMA straight
// from the first one's accumulator registers (cdna_hip_programming.md §3
// "An accumulator tile as the next MFMA's operand", with a permuted k order).
// Decode kernel token order of a page pair (A, B; pair token t = 16*page + offset):
// lane group g = lane>>4 owns the 8 CONSECUTIVE pair tokens 8g..8g+7 - the first S
// MFMA produces 8g..8g+3 of every group, the second 8g+4..8g+7 (its K rows are
// loaded in that permuted row order) - so each lane's V^T fragment is two transposed
// 4-row reads of the pair's LDS image and P^T = {S1 rows, S2 rows} as before.
//
// MFMA rows: 16 q-rows per tile = (16/G query tokens) x (G heads of one kv head).
// A workgroup = 4 waves = one (tile, kv head, kv partition); the waves split
// the partition's page pairs round-robin and merge (m, l, O) through LDS.
// Partitions > 1 (long context, small batch: fill 256 CUs) write fp32 partials
// that attn_reduce_kernel combines.
//
// Memory-bound: each K byte is loaded once per tile straight into VGPRs ("GEMV / M <= 16" row
// of the glds table, cdna_hip_programming.md §5); each V byte once into the wave's LDS image
// by LDS-DMA (the transpose needs it in LDS).
//
// REQUIREMENT: the cache is zero-initialised at allocation (masked lanes multiply
// p = 0 with whatever the unused slots hold; NaN garbage would poison O).
#include <type_traits>
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mlop {

// exp2 as the bare v_exp_f32: exp2f() wraps it in a denormal-range rescale (v_cmp +
// v_cndmask + v_ldexp per call, a fifth of the flash loop's VALU).  Softmax arguments are
// <= 0, so results below 2^-126 flushing to 0 changes nothing that survives bf16 P / f32 l.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

constexpr int kD = 128;
constexpr int kBS = 16;
constexpr float kNegBig = -1.0e30f;

// token-major V image in LDS: [rows][256 B], 16-B chunk c of row t at slot c ^ vswz(t)
// (cdna_hip_programming.md T10 image (b)); filled by LDS-DMA through the source address and
// read back transposed with ds_read_b64_tr_b16: a half-wave's two 4-row blocks 8 rows apart in
// the same columns are conflict-free
__device__ __forceinline__ int vswz(int t) { return ((t & 3) << 2) | ((t >> 2) & 3); }
typedef short v4s16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s16 lds_v4s16;

// V^T fragment (A operand of O^T = V^T . P^T, 16x16x32) for dims 16d .. 16d+15 and image rows
// 8 g4 .. 8 g4 + 7 of lane group g4 = lane >> 4 (two ds_read_b64_tr_b16: rows +0..3, +4..7).
// Lane 4q + p of a group addresses row t = 8 g4 + 4h + q, dims 16d + 4p .. +3, i.e. byte
//   256 t + 16 ((2d + (p >> 1)) ^ vswz(t)) + 8 (p & 1) = vt_base(lane) ^ 32 d          (h = 0)
// because 2d only moves bits 5-7, which the rest leaves 0 (the image is 256-B aligned); rows
// t + 4 flip bit 0 of vswz and nothing else the offset uses, so h = 1 is (that ^ 16) + 1024: ONE
// base VGPR, two v_xor and an immediate offset per fragment.
__device__ __forceinline__ uint32_t vt_base(int lane) {
  const int g4 = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int row = 8 * g4 + q, sw = vswz(row & 15);
  return 256u * row + 16u * ((p >> 1) ^ (sw & 1)) + 8u * (p & 1) + 32u * (sw >> 1);
}
__device__ __forceinline__ bf16x8 vt_frag(uint32_t b, int d) {
  const uint32_t a0 = b ^ (32u * d), a1 = (a0 ^ 16u) + 1024u;
  const v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(uintptr_t)a0);
  const v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(uintptr_t)a1);
  bf16x8 f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[e] = lo[e];
    f[4 + e] = hi[e];
  }
  return f;
}

__device__ __forceinline__ int wid_of(unsigned t) { return __builtin_amdgcn_readfirstlane((int)(t >> 6)); }

template <int G, int NT>  // NT bit 0: K / V loads non-temporal, bit 1: the output stores
__global__ void __launch_bounds__(256) paged_attn_kernel(
    uint16_t* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml,
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0,
    const int* __restrict__ q_start, const int* __restrict__ q_len,
    const int* __restrict__ ctx_len, int Hq, int Hkv, float scale_log2, int part_tokens,
    int nparts, int num_blocks, int* __restrict__ sem) {
  constexpr int QT = 16 / G;
  // (3 waves per SIMD at 134 VGPRs; forcing 4 (127 VGPRs, amdgpu_waves_per_eu) measured the
  // same on every decode shape and the headline, scripts/history/r4_occ.sh)
  // wave w stages its page pair's V image (2 x 16 token rows x 256 B = 8 KB) inside sm_o[w]
  // (8448 B, 256-B aligned: vt_frag), which it alone writes after its loop.  (A second image per
  // wave, prefetching the next pair, measured 1-4 % SLOWER on every decode shape: r04 profile.)
  __shared__ __attribute__((aligned(256))) float sm_o[4][16][kD + 4];
  __shared__ float sm_m[4][16];
  __shared__ float sm_l[4][16];
  __shared__ int sm_last;

  const int tile = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int s = tile_seq[tile], q0 = tile_q0[tile];
  const int p_begin = part * part_tokens;
  // The wave's first page pair, read as soon as the sequence id is known (clamped into the
  // row, used only if the pair exists): in the same round trip as ctx_len / q_len instead of
  // behind them, so the chain to the first K load is tile_seq -> block table -> K.
  const int* bt = block_tables + (size_t)s * bt_stride;
  const int bt0 = 2 * ((p_begin >> 5) + wid_of(threadIdx.x));
  const int rawA = bt[min(bt0, bt_stride - 1)], rawB = bt[min(bt0 + 1, bt_stride - 1)];
  const int ql = q_len[s], ctx = ctx_len[s], qs = q_start[s];
  const int last_q = min(q0 + QT, ql) - 1;           // last valid query of the tile
  const int kv_end = last_q >= 0 ? ctx - ql + last_q + 1 : 0;
  const int p_end = min(kv_end, p_begin + part_tokens);
  if (p_begin >= p_end && nparts > 1) {              // reducer skips empty partitions
    // kv_end == 0 (graph-bucket padding rows, ctx 0): no partition draws the last ticket of
    // the in-launch combine, so partition 0 writes the zero row attn_reduce_kernel would
    if (sem != nullptr && part == 0 && kv_end <= 0) {
      const int rr = threadIdx.x >> 4, c = (threadIdx.x & 15) * 8;
      const int qi2 = q0 + rr / G;
      if (qi2 < ql)
        *reinterpret_cast<u32x4*>(out + ((size_t)(qs + qi2) * Hq + kvh * G + (rr % G)) * kD + c) =
            u32x4{0u, 0u, 0u, 0u};
    }
    return;
  }

  // this lane's q-row (B operand column) and its causal limit
  const int r = lane & 15, g4 = lane >> 4;
  const int qi = q0 + r / G;
  const bool row_ok = qi < ql;
  const int head = kvh * G + (r % G);
  const int pos_r = row_ok ? ctx - ql + qi : -1;

  bf16x8 qf[4];
  {
    const uint16_t* qrow = q + ((size_t)(qs + (row_ok ? qi : 0)) * Hq + head) * kD;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + kk * 32 + g4 * 8);
      qf[kk] = row_ok ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 o[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, l = 0.f;

  const int pp_begin = p_begin >> 5;
  const int pp_end = (p_end + 31) >> 5;
  const int n_pages = (p_end + kBS - 1) / kBS;
  const size_t page_stride = (size_t)Hkv * kBS * kD;

  // (a generic pointer's low 32 bits are the LDS offset)
  const uint32_t vimg = (uint32_t)(uintptr_t)&sm_o[0][0][0] + wid * 8448u;
  // clamp: a corrupt block table must not become an out-of-bounds fault
  auto page_a = [&](int pp) { return min(max(bt[2 * pp], 0), num_blocks - 1); };
  auto page_b = [&](int pp, int pa) { return (2 * pp + 1 < n_pages) ? min(max(bt[2 * pp + 1], 0), num_blocks - 1) : pa; };
  // the pair's 32 token rows of this kv head by LDS-DMA into this wave's V image
  auto issue_v = [&](int pa, int pb) {
    const uint16_t* vA = vc + pa * page_stride + (size_t)kvh * kBS * kD;
    const uint16_t* vB = vc + pb * page_stride + (size_t)kvh * kBS * kD;
    const uint32_t dst = vimg;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int trow = (4 * i + g4) & 15;
      const uint16_t* src = (i < 4 ? vA : vB) + trow * kD + ((r ^ vswz(trow)) << 3);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(uintptr_t)(dst + 1024u * i), 16, 0,
                                       (NT & 1) ? 2 /* nt */ : 0);
    }
  };
  // page ids one pair ahead: the block-table loads of pair pp + 4 run under pair pp
  int pgA = 0, pgB = 0;
  if (pp_begin + wid < pp_end) {
    pgA = min(max(rawA, 0), num_blocks - 1);
    pgB = (bt0 + 1 < n_pages) ? min(max(rawB, 0), num_blocks - 1) : pgA;
  }
  for (int pp = pp_begin + wid; pp < pp_end; pp += 4) {
    const uint16_t* kA = kc + pgA * page_stride + (size_t)kvh * kBS * kD;
    const uint16_t* kB = kc + pgB * page_stride + (size_t)kvh * kBS * kD;

    // K rows of MFMA row r: pair tokens 8*(r>>2) + (r&3) (first S MFMA) and +4 (second)
    const uint16_t* kR = (r >> 3 ? kB : kA) + (8 * ((r >> 2) & 1) + (r & 3)) * kD;
    bf16x8 ka[4], kb[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if constexpr ((NT & 1) != 0) {
        ka[kk] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kR + kk * 32 + g4 * 8));
        kb[kk] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kR + 4 * kD + kk * 32 + g4 * 8));
      } else {
        ka[kk] = *reinterpret_cast<const bf16x8*>(kR + kk * 32 + g4 * 8);
        kb[kk] = *reinterpret_cast<const bf16x8*>(kR + 4 * kD + kk * 32 + g4 * 8);
      }
    }
    // this pair's V image, issued behind the K loads (the S MFMAs wait for those only; the
    // previous pair's transposed reads are complete: their MFMAs consumed them)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue_v(pgA, pgB);
    if (pp + 4 < pp_end) {
      pgA = page_a(pp + 4);
      pgB = page_b(pp + 4, pgA);
    }
    bf16x8 vf8[8];
    // S^T[token][row]: lane holds row r, tokens 4*g4 + i of each page
    f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      sa = mfma16(ka[kk], qf[kk], sa);
      sb = mfma16(kb[kk], qf[kk], sb);
    }
    const int tokA = pp * 32 + g4 * 8, tokB = tokA + 4;
    float pa[4], pb[4];
    float mx = kNegBig;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ta = tokA + i, tb = tokB + i;
      pa[i] = (ta < p_end && ta <= pos_r) ? sa[i] * scale_log2 : -INFINITY;
      pb[i] = (tb < p_end && tb <= pos_r) ? sb[i] * scale_log2 : -INFINITY;
      mx = fmaxf(mx, fmaxf(pa[i], pb[i]));
    }
    mx = max_x16_x32(mx);
    const float m_new = fmaxf(m, mx);
    const float alpha = fast_exp2(m - m_new);
    m = m_new;
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pa[i] = fast_exp2(pa[i] - m_new);
      pb[i] = fast_exp2(pb[i] - m_new);
      rs += pa[i] + pb[i];
    }
    l = l * alpha + rs;
    bf16x8 pf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pf[i] = (short)f2bf(pa[i]);
      pf[4 + i] = (short)f2bf(pb[i]);
    }
    {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's V image has landed
      uint32_t b0 = vimg + vt_base(lane);
      asm volatile("" : "+v"(b0));  // no hoisting of the 16 read addresses out of the loop
#pragma unroll
      for (int d = 0; d < 8; ++d) vf8[d] = vt_frag(b0, d);
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      o[d] *= alpha;
      o[d] = mfma16(vf8[d], pf, o[d]);
    }
  }

  l = sum_x16_x32(l);
  // O^T[d][row]: lane holds row r, dims 16*dblk + 4*g4 + i
#pragma unroll
  for (int d = 0; d < 8; ++d)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm_o[wid][r][d * 16 + g4 * 4 + i] = o[d][i];
  if (g4 == 0) {
    sm_m[wid][r] = m;
    sm_l[wid][r] = l;
  }
  __syncthreads();

  const int rr = threadIdx.x >> 4, c = (threadIdx.x & 15) * 8;
  float M = kNegBig;
#pragma unroll
  for (int w = 0; w < 4; ++w) M = fmaxf(M, sm_m[w][rr]);
  float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float f = exp2f(sm_m[w][rr] - M);
    L += f * sm_l[w][rr];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f * sm_o[w][rr][c + j];
  }
  const int qi2 = q0 + rr / G;
  const bool row_valid = qi2 < ql;
  const int head2 = kvh * G + (rr % G);
  if (nparts == 1) {
    if (!row_valid) return;
    const float inv = L > 0.f ? 1.f / L : 0.f;
    u32x4 ov;
#pragma unroll
    for (int j = 0; j < 4; ++j) ov[j] = pack2(acc[2 * j] * inv, acc[2 * j + 1] * inv);
    u32x4* dst = reinterpret_cast<u32x4*>(out + ((size_t)(qs + qi2) * Hq + head2) * kD + c);
    if constexpr ((NT & 2) != 0) __builtin_nontemporal_store(ov, dst);
    else *dst = ov;
    return;
  }
  if (row_valid) {
    // The slab is stored sc1 (write-through to L2) so that the hand-off below needs no
    // agent release (MI355X_MICROARCH.md, hand-off producer rule (2)).  Buffer offsets
    // are relative to this (tile, kvh, part) slab: 16 rows x kD floats, 16 x 2 floats.
    const size_t slab = (((size_t)tile * Hkv + kvh) * nparts + part) * 16;
    const auto rs_o = __builtin_amdgcn_make_buffer_rsrc(part_o + slab * kD, 0, 16 * kD * 4, 0x00020000);
    const uint32_t oo = (uint32_t)(rr * kD + c) * 4u;
    u32x4 w0, w1;
    w0[0] = __float_as_uint(acc[0]); w0[1] = __float_as_uint(acc[1]);
    w0[2] = __float_as_uint(acc[2]); w0[3] = __float_as_uint(acc[3]);
    w1[0] = __float_as_uint(acc[4]); w1[1] = __float_as_uint(acc[5]);
    w1[2] = __float_as_uint(acc[6]); w1[3] = __float_as_uint(acc[7]);
    __builtin_amdgcn_raw_buffer_store_b128(w0, rs_o, oo, 0, 16 /* sc1 */);
    __builtin_amdgcn_raw_buffer_store_b128(w1, rs_o, oo + 16u, 0, 16 /* sc1 */);
    if ((threadIdx.x & 15) == 0) {
      const auto rs_ml = __builtin_amdgcn_make_buffer_rsrc(part_ml + slab * 2, 0, 16 * 2 * 4, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), rs_ml, (uint32_t)rr * 8u, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), rs_ml, (uint32_t)rr * 8u + 4u, 0, 16);
    }
  }
  if (sem == nullptr) return;  // attn_reduce_kernel combines in a second launch
  // In-launch combine (cdna_hip_programming.md §5 split-K item 2, counter form of the
  // §6 Guideline 16 hand-off).  Producer: sc1 stores, every wave waits vmcnt(0), a
  // workgroup barrier, then one lane draws a relaxed agent-scope ticket -- no release
  // fence (it cost every partition an L2 writeback).  Consumer: the partition that draws
  // nvalid-1 keeps the agent acquire (this kernel runs two workgroups per CU, outside the
  // guide's fence-free table row) and reduces every slab, then re-arms the counter for
  // the next launch (the buffer is zero-initialised once).
  const int nvalid = min(nparts, (kv_end + part_tokens - 1) / part_tokens);
  int* cnt = sem + (size_t)tile * Hkv + kvh;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm_last = (t == nvalid - 1);
  }
  __syncthreads();
  if (!sm_last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!row_valid) return;
  const size_t base = ((size_t)tile * Hkv + kvh) * nparts;
  float MM = kNegBig;
  for (int p = 0; p < nvalid; ++p) MM = fmaxf(MM, part_ml[((base + p) * 16 + rr) * 2]);
  float LL = 0.f, a2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < nvalid; ++p) {
    const size_t pb = (base + p) * 16 + rr;
    const float f = exp2f(part_ml[pb * 2] - MM);
    LL += f * part_ml[pb * 2 + 1];
    const float4* po = reinterpret_cast<const float4*>(part_o + pb * kD + c);
    const float4 x0 = po[0], x1 = po[1];
    a2[0] += f * x0.x; a2[1] += f * x0.y; a2[2] += f * x0.z; a2[3] += f * x0.w;
    a2[4] += f * x1.x; a2[5] += f * x1.y; a2[6] += f * x1.z; a2[7] += f * x1.w;
  }
  const float inv = LL > 0.f ? 1.f / LL : 0.f;
  u32x4 ov;
#pragma unroll
  for (int j = 0; j < 4; ++j) ov[j] = pack2(a2[2 * j] * inv, a2[2 * j + 1] * inv);
  *reinterpret_cast<u32x4*>(out + ((size_t)(qs + qi2) * Hq + head2) * kD + c) = ov;
}

template <int G>
__global__ void __launch_bounds__(256) attn_reduce_kernel(
    uint16_t* __restrict__ out, const float* __restrict__ part_o,
    const float* __restrict__ part_ml, const int* __restrict__ tile_seq,
    const int* __restrict__ tile_q0, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len, int Hq, int Hkv,
    int part_tokens, int nparts) {
  constexpr int QT = 16 / G;
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int s = tile_seq[tile], q0 = tile_q0[tile];
  const int ql = q_len[s], ctx = ctx_len[s], qs = q_start[s];
  const int last_q = min(q0 + QT, ql) - 1;
  const int kv_end = last_q >= 0 ? ctx - ql + last_q + 1 : 0;
  const int nvalid = min(nparts, (kv_end + part_tokens - 1) / part_tokens);
  const int rr = threadIdx.x >> 4, c = (threadIdx.x & 15) * 8;
  const int qi = q0 + rr / G;
  if (qi >= ql) return;
  const size_t base = ((size_t)tile * Hkv + kvh) * nparts;
  float M = kNegBig;
  for (int p = 0; p < nvalid; ++p) M = fmaxf(M, part_ml[((base + p) * 16 + rr) * 2]);
  float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < nvalid; ++p) {
    const size_t pb = (base + p) * 16 + rr;
    const float f = exp2f(part_ml[pb * 2] - M);
    L += f * part_ml[pb * 2 + 1];
    const float4* po = reinterpret_cast<const float4*>(part_o + pb * kD + c);
    float4 a = po[0], b = po[1];
    acc[0] += f * a.x; acc[1] += f * a.y; acc[2] += f * a.z; acc[3] += f * a.w;
    acc[4] += f * b.x; acc[5] += f * b.y; acc[6] += f * b.z; acc[7] += f * b.w;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  u32x4 ov;
#pragma unroll
  for (int j = 0; j < 4; ++j) ov[j] = pack2(acc[2 * j] * inv, acc[2 * j + 1] * inv);
  const int head = kvh * G + (rr % G);
  *reinterpret_cast<u32x4*>(out + ((size_t)(qs + qi) * Hq + head) * kD + c) = ov;
}

// K / V pages of the decode kernel non-temporal (read once per step by one workgroup; the
// headline step reads ~100 GB of them): headline +2.2 / +3.2 % interleaved (attn_kv_nt op, bit
// 0); bit 1 the output stores too (with gemm_slab_nt bit 3: +0.5 %)
static int g_attn_kv_nt = 3;
int attn_kv_nt(int set) {
  if (set >= 0) g_attn_kv_nt = set;
  return g_attn_kv_nt;
}

template <int G>
static void launch_g(void* out, float* part_o, float* part_ml, const void* q, const void* kc,
                     const void* vc, const int* bt, int bt_stride, const int* tile_seq,
                     const int* tile_q0, const int* q_start, const int* q_len, const int* ctx_len,
                     int num_tiles, int Hq, int Hkv, float scale_log2, int part_tokens, int nparts,
                     int num_blocks, int* sem, hipStream_t st) {
  dim3 grid(num_tiles, Hkv, nparts);
  // K / V pages non-temporal (attn_kv_nt op): each is read once per step by one workgroup
  // (below 8 query tiles the default policy: batch 4 lost 0.7 % with it, batch 16 gained 1.8 %)
  const int nt = num_tiles >= 8 ? g_attn_kv_nt : 0;
  auto kern = nt == 3 ? paged_attn_kernel<G, 3> : nt ? paged_attn_kernel<G, 1> : paged_attn_kernel<G, 0>;
  kern<<<grid, 256, 0, st>>>((uint16_t*)out, part_o, part_ml, (const uint16_t*)q, (const uint16_t*)kc,
                             (const uint16_t*)vc, bt, bt_stride, tile_seq, tile_q0, q_start, q_len, ctx_len,
                             Hq, Hkv, scale_log2, part_tokens, nparts, num_blocks, sem);
  if (nparts > 1 && sem == nullptr) {
    attn_reduce_kernel<G><<<dim3(num_tiles, Hkv), 256, 0, st>>>(
        (uint16_t*)out, part_o, part_ml, tile_seq, tile_q0, q_start, q_len, ctx_len, Hq, Hkv,
        part_tokens, nparts);
  }
}

void launch_paged_attention(void* out, float* part_o, float* part_ml, const void* q,
                            const void* kc, const void* vc, const int* bt, int bt_stride,
                            const int* tile_seq, const int* tile_q0, const int* q_start,
                            const int* q_len, const int* ctx_len, int num_tiles, int Hq, int Hkv,
                            float scale_log2, int part_tokens, int nparts, int num_blocks,
                            int* sem, hipStream_t st) {
  if (num_tiles == 0) return;
  const int G = Hq / Hkv;
#define MLOP_ATTN_CASE(GG)                                                                        \
  case GG:                                                                                        \
    launch_g<GG>(out, part_o, part_ml, q, kc, vc, bt, bt_stride, tile_seq, tile_q0, q_start,     \
                 q_len, ctx_len, num_tiles, Hq, Hkv, scale_log2, part_tokens, nparts, num_blocks, sem, st);   \
    break;
  switch (G) {
    MLOP_ATTN_CASE(1)
    MLOP_ATTN_CASE(2)
    MLOP_ATTN_CASE(4)
    MLOP_ATTN_CASE(8)
    MLOP_ATTN_CASE(16)
    default: break;
  }
#undef MLOP_ATTN_CASE
}

// ---------------------------------------------------------------------------
// K7 flash prefill on the 32x32x16 MFMA (cdna_hip_programming.md "Fused attention prefill":
// swapped QK^T, an accumulator tile as the next MFMA's operand).  One workgroup = 128 MFMA
// q-rows (128/G query tokens x the G heads of one kv head) against EVERY key of its causal
// range, so every K/V byte fetched from L2 feeds all 128 q-rows.  K/V page pairs (32 keys, 16 KB)
// stream through a 3-deep LDS ring by LDS-DMA (global_load_lds, counted vmcnt, one raw barrier
// per pair), swizzled through the SOURCE address:
//   K page [16 keys][16 x 16 B]: chunk c of key k at slot c ^ k       (ds_read_b128)
//   V page [16 keys][16 x 16 B]: chunk c of key k at slot c ^ vswz(k) (ds_read_b64_tr_b16)
// both conflict-free for the fragment reads below (SQ_LDS_BANK_CONFLICT = 0).  Per wave 32
// q-rows, ONE per lane column:
//   S^T [32 keys x 32 q] = K . Q^T: 8 MFMAs (A = K rows by ds_read_b128, B = Q^T in registers);
//     lane l holds the 16 keys (r & 3) + 8 (r >> 2) + 4 h (h = l >> 5) of q column l & 31, so
//     the row max is 15 lane-local max + ONE permlane32 swap, the row sum lane-local (the two
//     halves' partial sums meet once, in the epilogue);
//   O^T [128 d x 32 q] += V^T . P^T: 8 MFMAs, P^T straight from the S registers (registers
//     8s .. 8s+7 -> bf16 = the k-step s fragment, k order permuted), V^T by two
//     ds_read_b64_tr_b16 per fragment from the token-major image (keys 16s + 4h + 0..3 and
//     + 8, dims 32 dblk + (l & 31)).
// Half the MFMA issue slots of a 16x16x32 form for the same FLOPs (an MFMA holds the SIMD's
// vector issue for 8 cycles either way, MI355X_MICROARCH.md constants) and a quarter of its
// cross-lane max steps: +4 % at 1 x 8192, +19 % at 4 x 2048 and 16 x 512 over the round-4
// 16x16x32 kernel (profiles/r05_flash32.md).  Two workgroups per CU (up to 256 VGPRs) beat
// three (168) by 1-5 %.
using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr float kRescaleLog2 = 8.f;  // flash32 deferred-rescale threshold (exp2 units)
// two floats -> one dword of two bf16 in ONE v_cvt_pk_bf16_f32 (pack2's two scalar casts
// become two cvt + shift + or)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// byte offset (page 0, dim block 0, rows 4h + q) of lane l's first transposed V read: lane
// 4q + p of 16-lane group g addresses row t = 4h + q, chunk 2 (g & 1) + (p >> 1), half p & 1.
// Dim block dblk flips address bits 6-7 (^ 64 dblk: the chunk's high bits only meet q there),
// rows + 8 flip bit 5 and add 2048, page B adds 4096.
__device__ __forceinline__ uint32_t vt32_base(int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
  const int t = 4 * h + q, c = 2 * (g & 1) + (p >> 1);
  return 256u * t + 16u * (c ^ vswz(t)) + 8u * (p & 1);
}

// one flash tile (128 q-rows of ONE kv head against its whole causal key range)
template <int G>
__device__ __forceinline__ void flash32_item(
    uint16_t* smem, int tile, int kvh, uint16_t* __restrict__ out, const uint16_t* __restrict__ q,
    const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc, const int* __restrict__ block_tables,
    int bt_stride, const int* __restrict__ ptile_seq, const int* __restrict__ ptile_q0,
    const int* __restrict__ q_start, const int* __restrict__ q_len, const int* __restrict__ ctx_len, int Hq,
    int Hkv, float scale_log2, int num_blocks) {
  constexpr int QB = 128 / G;            // query tokens per workgroup
  constexpr int STAGES = 3;
  constexpr int STAGE = 4 * kBS * kD;    // bf16 per stage: K page A | K page B | V page A | V page B
  constexpr int PAGE = kBS * kD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int s = ptile_seq[tile], q0 = ptile_q0[tile];
  const int ql = q_len[s], ctx = ctx_len[s], qs = q_start[s];
  const int last_q = min(q0 + QB, ql) - 1;
  const int kv_end = ctx - ql + last_q + 1;
  const int n_pairs = (kv_end + 31) >> 5;
  const int n_pages = (kv_end + kBS - 1) / kBS;
  const int wg_min_pos = ctx - ql + q0;
  const int col = lane & 31, h = lane >> 5;

  // this lane's q row (MFMA column): R = 32 wid + col
  const int R = 32 * wid + col;
  const int qi = q0 + R / G;
  const bool q_ok = qi < ql;
  const int pos_r = q_ok ? ctx - ql + qi : -1;
  bf16x8 qf[8];
  {
    const uint16_t* qrow = q + ((size_t)(qs + (q_ok ? qi : 0)) * Hq + kvh * G + R % G) * kD + 8 * h;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + 16 * t);
      qf[t] = q_ok ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
  float m = kNegBig, l = 0.f;

  const int* bt = block_tables + (size_t)s * bt_stride;
  const size_t page_stride = (size_t)Hkv * PAGE;
  const int kkey = wid * 4 + (lane >> 4);
  // K image: chunk c of key k at slot c ^ k on BOTH pages (the 32x32 A-operand reads take keys
  // {0-3, 12-15} of one page and {4-11} of the other per 16-lane group: 16 distinct slots)
  const int k_off = kvh * PAGE + kkey * kD + (((lane & 15) ^ (kkey & 15)) << 3);
  const int v_off = kvh * PAGE + kkey * kD + (((lane & 15) ^ vswz(kkey)) << 3);
  auto page_of = [&](int idx) { return idx < n_pages ? min(max(bt[idx], 0), num_blocks - 1) : -1; };
  auto issue_pages = [&](int buf, int pgA, int pgB) {
    if (pgB < 0) pgB = pgA;
    uint16_t* base = smem + buf * STAGE + wid * 512;
    __builtin_amdgcn_global_load_lds((const void*)(kc + pgA * page_stride + k_off), (lds_void_t*)(base), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(kc + pgB * page_stride + k_off), (lds_void_t*)(base + PAGE), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vc + pgA * page_stride + v_off), (lds_void_t*)(base + 2 * PAGE), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vc + pgB * page_stride + v_off), (lds_void_t*)(base + 3 * PAGE), 16, 0, 0);
  };
  // K fragment t of this lane: key col of the pair (page col >> 4, row col & 15), chunk 2t + h at
  // slot (2t + h) ^ (col & 15): byte k_b0 ^ 32 t
  const int k15 = col & 15;
  const uint32_t k_b0 = (uint32_t)(uintptr_t)smem + (uint32_t)((col >> 4) * PAGE * 2 + k15 * 256 + ((h ^ k15) << 4));
  const uint32_t v_b0 = (uint32_t)(uintptr_t)smem + 2 * PAGE * 2 + vt32_base(lane);

  // S^T of the pair in ring slot ST: K fragment t at k_b0 ^ 32 t, four reads in flight (inline
  // asm with counted waits: as plain loads the compiler reused one register set and waited
  // lgkmcnt(0) in front of every MFMA, one LDS latency per fragment)
  auto qk = [&](auto st_tag) {
    constexpr uint32_t so = (uint32_t)(decltype(st_tag)::value * STAGE * 2);
    uint32_t kb = k_b0;
    asm volatile("" : "+v"(kb));
    auto kread = [&](int t, bf16x8& f) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(kb ^ (32u * t)), "n"(so));
    };
    f32x16 sc;
#pragma unroll
    for (int e = 0; e < 16; ++e) sc[e] = 0.f;
    bf16x8 kf[4];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // nothing else (SMEM) in the counts below
#pragma unroll
    for (int t = 0; t < 4; ++t) kread(t, kf[t]);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      bf16x8& f = kf[t & 3];
      if (t <= 4) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(f));
      else if (t == 5) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f));
      else if (t == 6) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(f));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f));
      sc = mfma32(f, qf[t], sc);
      if (t + 4 < 8) kread(t + 4, kf[t & 3]);
    }
    return sc;
  };
  // online softmax on the lane's 16 keys of its q column (raw score units; the scale folds into
  // the exponent's FMA) -> P^T fragments of the two k-steps; O and l rescaled when the max moved
  auto softmax = [&](f32x16 sc, int pp, bf16x8 (&pf)[2]) {
    if (pp * 32 + 31 > wg_min_pos) {  // a pair crossing the workgroup's causal diagonal
      // (a side effect keeps this a branch: if-converted, the 47 compare / select / add of the
      // mask ran on every pair, a third of the loop's VALU)
      asm volatile("");
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tok = pp * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        sc[r] = tok <= pos_r ? sc[r] : -INFINITY;
      }
    }
    float mx = fmaxf(fmaxf(sc[0], sc[1]), sc[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, sc[r]), sc[r + 1]);
    mx = fmaxf(mx, sc[15]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    // deferred rescale (cdna_hip_programming.md T13): the running max moves only when some row's
    // new max exceeds it by more than 2^kRescaleLog2 in exp2 units (always on a row's first
    // keys: m starts at -1e30); otherwise P stays scaled against the old max, <= 2^8, which
    // bf16 P and f32 O / l carry exactly as well.  The decision covers this pair's P and is
    // taken before it is exponentiated, with the previous pair's P.V complete, so O, l and P
    // all see the same factor.
    float alpha = 1.f;
    if (__ballot((mx - m) * scale_log2 > kRescaleLog2)) {
      const float m_new = fmaxf(m, mx);
      alpha = fast_exp2((m - m_new) * scale_log2);
      m = m_new;
#pragma unroll
      for (int d = 0; d < 4; ++d) o[d] *= alpha;
      l *= alpha;
    }
    const float mc = -m * scale_log2;
    float rs = 0.f;
    u32x4 w[2];
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const float p0 = fast_exp2(fmaf(sc[r], scale_log2, mc)), p1 = fast_exp2(fmaf(sc[r + 1], scale_log2, mc));
      rs += p0 + p1;
      w[r >> 3][(r & 7) >> 1] = cvt_pk_bf16(p0, p1);
    }
    pf[0] = __builtin_bit_cast(bf16x8, w[0]);
    pf[1] = __builtin_bit_cast(bf16x8, w[1]);
    l += rs;
  };
  // O^T += V^T . P^T from ring slot ST; the V^T fragment of (dblk, page) = two transposed reads.
  // The reads are inline asm: as builtins the compiler put s_waitcnt vmcnt(0) in front of them
  // (it cannot tell them from the in-flight LDS-DMA of the next pairs), which exposed the
  // latency of the DMA just issued on every pair.  The ring protocol (vmcnt + barrier at the
  // top of the step) already covers this pair; the asm waits below count only these reads.
  auto pv = [&](auto st_tag, const bf16x8 (&pf)[2]) {
    constexpr uint32_t so = (uint32_t)(decltype(st_tag)::value * STAGE * 2);
    uint32_t vb = v_b0;
    asm volatile("" : "+v"(vb));
    // both pages' fragments of dim block dblk: 4 reads, results in (lo, hi) of f0 (page A), f1
    auto issue = [&](int dblk, v4s16 (&r)[4]) {
      const uint32_t a0 = vb ^ (64u * dblk), a1 = a0 ^ 32u;
      asm volatile(
          "ds_read_b64_tr_b16 %0, %4 offset:%6\n"
          "ds_read_b64_tr_b16 %1, %5 offset:%7\n"
          "ds_read_b64_tr_b16 %2, %4 offset:%8\n"
          "ds_read_b64_tr_b16 %3, %5 offset:%9\n"
          : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
          : "v"(a0), "v"(a1), "n"(so), "n"(so + 2048u), "n"(so + 4096u), "n"(so + 6144u));
    };
    auto frag = [&](const v4s16& lo, const v4s16& hi) {
      bf16x8 f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = lo[e];
        f[4 + e] = hi[e];
      }
      return f;
    };
    v4s16 ra[4], rb[4];
    issue(0, ra);
#pragma unroll
    for (int dblk = 0; dblk < 4; ++dblk) {
      v4s16 (&cur)[4] = (dblk & 1) ? rb : ra;
      v4s16 (&nxt)[4] = (dblk & 1) ? ra : rb;
      if (dblk < 3) {
        issue(dblk + 1, nxt);
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
      }
      o[dblk] = mfma32(frag(cur[0], cur[1]), pf[0], o[dblk]);
      o[dblk] = mfma32(frag(cur[2], cur[3]), pf[1], o[dblk]);
    }
  };

  issue_pages(0, page_of(0), page_of(1));
  if (n_pairs > 1) issue_pages(1, page_of(2), page_of(3));
  int nxtA = page_of(4), nxtB = page_of(5);
  auto pair_step = [&](auto st_tag, int pp) {
    constexpr int ST = decltype(st_tag)::value;
    if (pp + 1 < n_pairs) wait_vmcnt<4>(); else wait_vmcnt<0>();
    raw_barrier();  // pair pp visible to every wave; ring slot (pp - 1) % 3 free
    if (pp + 2 < n_pairs) {
      issue_pages((ST + 2) % STAGES, nxtA, nxtB);
      nxtA = page_of(2 * pp + 6);
      nxtB = page_of(2 * pp + 7);
    }
    bf16x8 pf[2];
    softmax(qk(st_tag), pp, pf);
    pv(st_tag, pf);
  };
  for (int pp = 0; pp < n_pairs; pp += STAGES) {
    pair_step(std::integral_constant<int, 0>{}, pp);
    if (pp + 1 < n_pairs) pair_step(std::integral_constant<int, 1>{}, pp + 1);
    if (pp + 2 < n_pairs) pair_step(std::integral_constant<int, 2>{}, pp + 2);
  }

  // the two lane halves' partial row sums; O^T element r of dim block d is dim
  // 32 d + 8 (r >> 2) + 4 h + (r & 3) of q row R
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
    l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  if (!q_ok) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  uint16_t* orow = out + ((size_t)(qs + qi) * Hq + kvh * G + R % G) * kD + 4 * h;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      u32x2 v;
      v[0] = pack2(o[d][4 * b] * inv, o[d][4 * b + 1] * inv);
      v[1] = pack2(o[d][4 * b + 2] * inv, o[d][4 * b + 3] * inv);
      *reinterpret_cast<u32x2*>(orow + 32 * d + 8 * b) = v;
    }
}

// STREAM (flash_stream op): the persistent grid's tiles as ONE stream of K / V page pairs per
// workgroup, so a tile's fixed cost hides under the previous tile's pairs (the 29 us fixed term
// of profiles/r06_flash_persist.md):
//   * the 3-deep LDS ring runs across tiles: while the last pairs of tile i are consumed, the
//     first two pairs of tile i+1 (or i+2: one-pair tiles) are already being fetched;
//   * tile i+1's Q rows arrive by LDS-DMA into a wave-private 8 KB while tile i runs, and are
//     read into registers at tile i+1's start (80 KB of LDS: 2 workgroups per CU);
//   * the loop is unrolled by the ring depth, so every step's stage is a constant (LDS read
//     offsets in the instruction) and tile boundaries are a branch inside a step.
// Every vector memory operation of a wave is counted (4 LDS-DMAs per pair, 8 Q DMAs per tile,
// 16 O stores per tile: buffer stores, rows past the prompt dropped by the range check, so the
// count never depends on the data), and a pair's wait is vmcnt(operations issued after its DMAs):
// vmcnt(4) in the steady state.
// Tiles per workgroup, boustrophedon order and the kv head per XCD as the PERSIST grid.
//
// s_waitcnt vmcnt(n) for a run-time n (a multiple of 4; rounded down, and capped at 60: waiting
// for MORE retired operations than needed is always safe); n = 4 on the first compare
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  if (__builtin_expect(n == 4, 1)) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    return;
  }
  switch (n < 0 ? 0 : n > 60 ? 15 : n >> 2) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
  }
}

// item k of a persistent slot (boustrophedon rounds of S tiles), its causal extent in pairs and
// pages; tile -1 past the end of the list
struct FlashTile {
  int tile, q0, ql, ctx, qs, n_pairs, n_pages, wg_min_pos, seq;
};
// metadata reads through the constant address space: scalar loads (the tables are not written
// during the launch; as global pointers the loads after the first O store became vector loads,
// each followed by a vmcnt(0) that drained the in-flight K / V ring)
using cint_p = const __attribute__((address_space(4))) int*;
__device__ __forceinline__ int ld_const(const int* p, int i) {
  return ((cint_p)p)[__builtin_amdgcn_readfirstlane(i)];
}
template <int QB>
__device__ __forceinline__ FlashTile flash_tile(int k, int slot, int S, int num_ptiles, const int* __restrict__ ptile_seq,
                                                const int* __restrict__ ptile_q0, const int* __restrict__ q_start,
                                                const int* __restrict__ q_len, const int* __restrict__ ctx_len) {
  FlashTile it;
  const int t = k * S + ((k & 1) ? S - 1 - slot : slot);
  const bool ok = t < num_ptiles;
  const int tt = ok ? t : num_ptiles - 1;  // loads stay in bounds; the fields are ignored past the end
  it.tile = ok ? t : -1;
  it.seq = ld_const(ptile_seq, tt);
  it.q0 = ld_const(ptile_q0, tt);
  it.ql = ld_const(q_len, it.seq);
  it.ctx = ld_const(ctx_len, it.seq);
  it.qs = ld_const(q_start, it.seq);
  const int kv_end = it.ctx - it.ql + min(it.q0 + QB, it.ql);
  it.n_pairs = (kv_end + 31) >> 5;
  it.n_pages = (kv_end + kBS - 1) / kBS;
  it.wg_min_pos = it.ctx - it.ql + it.q0;
  return it;
}

template <int G>
__global__ void __launch_bounds__(256, 2) flash32_stream_kernel(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ptile_seq, const int* __restrict__ ptile_q0,
    const int* __restrict__ q_start, const int* __restrict__ q_len,
    const int* __restrict__ ctx_len, int Hq, int Hkv, float scale_log2, int num_blocks, int num_ptiles) {
  constexpr int QB = 128 / G;
  constexpr int STAGE = 4 * kBS * kD;  // bf16 per stage: K page A | K page B | V page A | V page B
  constexpr int PAGE = kBS * kD;
  constexpr int QW = 32 * kD;  // bf16 of one wave's 32 Q rows
  __shared__ __attribute__((aligned(256))) uint16_t smem[3 * STAGE + 4 * QW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5, R = 32 * wid + col;
  const int kvh = blockIdx.x % Hkv, slot = blockIdx.x / Hkv, S = gridDim.x / Hkv;
  const size_t page_stride = (size_t)Hkv * PAGE;
  const int kkey = wid * 4 + (lane >> 4);
  const int k_off = kvh * PAGE + kkey * kD + (((lane & 15) ^ (kkey & 15)) << 3);
  const int v_off = kvh * PAGE + kkey * kD + (((lane & 15) ^ vswz(kkey)) << 3);
#define MLOP_FT(k) flash_tile<QB>((k), slot, S, num_ptiles, ptile_seq, ptile_q0, q_start, q_len, ctx_len)

  FlashTile cur = MLOP_FT(0);
  if (cur.tile < 0) return;  // the whole workgroup, before any barrier

  // the issue pointer of the pair stream: item iss_k, its next pair iss_p, whose pages pA / pB
  // were looked up one issue ahead.  vm = vector memory operations this wave has issued; markS
  // = vm right after the DMAs of the pair in ring stage S.  Pair n goes to stage n % 3 and is
  // consumed by the loop's step n % 3.
  FlashTile iss = cur;
  int iss_k = 0, iss_p = 0, vm = 0, mark0 = 0, mark1 = 0, mark2 = 0;
  const int* iss_bt = block_tables + (size_t)iss.seq * bt_stride;
  int pA = min(max(ld_const(iss_bt, 0), 0), num_blocks - 1);
  int pB = iss.n_pages > 1 ? min(max(ld_const(iss_bt, 1), 0), num_blocks - 1) : pA;
  auto issue_next = [&](auto st_tag) __attribute__((always_inline)) {
    constexpr int ST = decltype(st_tag)::value;
    if (iss.tile < 0) return;
    uint16_t* base = smem + ST * STAGE + wid * 512;
    __builtin_amdgcn_global_load_lds((const void*)(kc + pA * page_stride + k_off), (lds_void_t*)(base), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(kc + pB * page_stride + k_off), (lds_void_t*)(base + PAGE), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vc + pA * page_stride + v_off), (lds_void_t*)(base + 2 * PAGE), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vc + pB * page_stride + v_off), (lds_void_t*)(base + 3 * PAGE), 16, 0, 0);
    vm += 4;
    if constexpr (ST == 0) mark0 = vm;
    else if constexpr (ST == 1) mark1 = vm;
    else mark2 = vm;
    if (++iss_p >= iss.n_pairs) {  // every item has >= 1 pair
      iss = MLOP_FT(++iss_k);
      iss_p = 0;
      iss_bt = block_tables + (size_t)iss.seq * bt_stride;
    }
    if (iss.tile >= 0) {
      const int a = 2 * iss_p, b = a + 1 < iss.n_pages ? a + 1 : a;
      pA = min(max(ld_const(iss_bt, a), 0), num_blocks - 1);
      pB = min(max(ld_const(iss_bt, b), 0), num_blocks - 1);
    }
  };
  // the next tile's Q rows by LDS-DMA into this wave's private 8 KB (the compiler neither
  // tracks nor copies them: as register loads its own wait for them became a vmcnt(0) that
  // drained the ring at every tile start).  DMA t writes 1 KB, lane L's 16 B at 16 L: row
  // 32 wid + (L & 31), dims 16 t + 8 (L >> 5) -- fragment t of lane L, read back linearly.
  uint16_t* const q_lds = smem + 3 * STAGE + wid * QW;
  int markQ = 0;
  auto q_issue = [&](const FlashTile& it) __attribute__((always_inline)) {
    const int qi = it.q0 + R / G;
    const uint16_t* qrow = q + ((size_t)(it.qs + (qi < it.ql ? qi : 0)) * Hq + kvh * G + R % G) * kD + 8 * h;
#pragma unroll
    for (int t = 0; t < 8; ++t)
      __builtin_amdgcn_global_load_lds((const void*)(qrow + 16 * t), (lds_void_t*)(q_lds + t * 512), 16, 0, 0);
    vm += 8;
    markQ = vm;
  };
  const uint32_t q_b0 = (uint32_t)(uintptr_t)q_lds + 16u * lane;
  const int k15 = col & 15;
  const uint32_t k_b0 = (uint32_t)(uintptr_t)smem + (uint32_t)((col >> 4) * PAGE * 2 + k15 * 256 + ((h ^ k15) << 4));
  const uint32_t v_b0 = (uint32_t)(uintptr_t)smem + 2 * PAGE * 2 + vt32_base(lane);
  // the O stores' range: every valid row below 2 GB (checked on the host), masked rows at 2 GB
  const auto rsO = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);

  // per-tile state: this lane's q row, its Q fragments, the accumulators
  int qi = 0, pos_r = -1, pp = 0, k = 0;
  bool q_ok = false;
  bf16x8 qf[8];
  f32x16 o[4];
  float m = kNegBig, l = 0.f;
  auto tile_start = [&]() __attribute__((always_inline)) {
    qi = cur.q0 + R / G;
    q_ok = qi < cur.ql;
    pos_r = q_ok ? cur.ctx - cur.ql + qi : -1;
    wait_vmcnt_rt(vm - markQ);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile(
        "ds_read_b128 %0, %8\n"
        "ds_read_b128 %1, %8 offset:1024\n"
        "ds_read_b128 %2, %8 offset:2048\n"
        "ds_read_b128 %3, %8 offset:3072\n"
        "ds_read_b128 %4, %8 offset:4096\n"
        "ds_read_b128 %5, %8 offset:5120\n"
        "ds_read_b128 %6, %8 offset:6144\n"
        "ds_read_b128 %7, %8 offset:7168\n"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(qf[0]), "=&v"(qf[1]), "=&v"(qf[2]), "=&v"(qf[3]), "=&v"(qf[4]), "=&v"(qf[5]), "=&v"(qf[6]),
          "=&v"(qf[7])
        : "v"(q_b0));
    if (!q_ok) {
#pragma unroll
      for (int t = 0; t < 8; ++t) qf[t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
    m = kNegBig;
    l = 0.f;
    pp = 0;
  };
  // epilogue: 16 buffer stores per lane, always issued (masked rows go past the range)
  auto tile_end = [&]() __attribute__((always_inline)) {
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
      l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const uint32_t obase =
        q_ok ? (uint32_t)((((size_t)(cur.qs + qi) * Hq + kvh * G + R % G) * kD + 4 * h) * 2) : 0x80000000u;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        u32x2 v;
        v[0] = pack2(o[d][4 * b] * inv, o[d][4 * b + 1] * inv);
        v[1] = pack2(o[d][4 * b + 2] * inv, o[d][4 * b + 3] * inv);
        __builtin_amdgcn_raw_buffer_store_b64(v, rsO, obase + (uint32_t)(32 * d + 8 * b) * 2u, 0, 0);
      }
    vm += 16;
    asm volatile("" ::: "memory");
  };

  // one stream step: consume the pair in ring stage ST (true: the stream has ended)
  FlashTile nxt;
  auto step = [&](auto st_tag) __attribute__((always_inline)) -> bool {
    constexpr int ST = decltype(st_tag)::value;
    constexpr uint32_t so = (uint32_t)(ST * STAGE * 2);
    wait_vmcnt_rt(vm - (ST == 0 ? mark0 : ST == 1 ? mark1 : mark2));
    raw_barrier();  // pair visible to every wave; the stage consumed one step ago is free
    issue_next(std::integral_constant<int, (ST + 2) % 3>{});
    if (pp == 0 && nxt.tile >= 0) q_issue(nxt);  // the next tile's Q under this tile's pairs
    // S^T = K . Q^T of this pair (flash32_item's qk)
    f32x16 sc;
    {
      uint32_t kb = k_b0;
      asm volatile("" : "+v"(kb));
#pragma unroll
      for (int e = 0; e < 16; ++e) sc[e] = 0.f;
      bf16x8 kf[4];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int t = 0; t < 4; ++t)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[t]) : "v"(kb ^ (32u * t)), "n"(so));
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        bf16x8& f = kf[t & 3];
        if (t <= 4) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(f));
        else if (t == 5) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f));
        else if (t == 6) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(f));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f));
        sc = mfma32(f, qf[t], sc);
        if (t + 4 < 8)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[t & 3]) : "v"(kb ^ (32u * (t + 4))), "n"(so));
      }
    }
    // online softmax (flash32_item's, deferred rescale)
    bf16x8 pf[2];
    {
      if (pp * 32 + 31 > cur.wg_min_pos) {
        asm volatile("");
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tok = pp * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          sc[r] = tok <= pos_r ? sc[r] : -INFINITY;
        }
      }
      float mx = fmaxf(fmaxf(sc[0], sc[1]), sc[2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, sc[r]), sc[r + 1]);
      mx = fmaxf(mx, sc[15]);
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      if (__ballot((mx - m) * scale_log2 > kRescaleLog2)) {
        const float m_new = fmaxf(m, mx);
        const float alpha = fast_exp2((m - m_new) * scale_log2);
        m = m_new;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] *= alpha;
        l *= alpha;
      }
      const float mc = -m * scale_log2;
      float rs = 0.f;
      u32x4 w[2];
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float p0 = fast_exp2(fmaf(sc[r], scale_log2, mc)), p1 = fast_exp2(fmaf(sc[r + 1], scale_log2, mc));
        rs += p0 + p1;
        w[r >> 3][(r & 7) >> 1] = cvt_pk_bf16(p0, p1);
      }
      pf[0] = __builtin_bit_cast(bf16x8, w[0]);
      pf[1] = __builtin_bit_cast(bf16x8, w[1]);
      l += rs;
    }
    // O^T += V^T . P^T (flash32_item's pv)
    {
      uint32_t vb = v_b0;
      asm volatile("" : "+v"(vb));
      v4s16 ra[4], rb[4];
#define MLOP_VT_ISSUE(dblk, r)                                                              \
  {                                                                                         \
    const uint32_t a0 = vb ^ (64u * (dblk)), a1 = a0 ^ 32u;                                 \
    asm volatile(                                                                           \
        "ds_read_b64_tr_b16 %0, %4 offset:%6\n"                                             \
        "ds_read_b64_tr_b16 %1, %5 offset:%7\n"                                             \
        "ds_read_b64_tr_b16 %2, %4 offset:%8\n"                                             \
        "ds_read_b64_tr_b16 %3, %5 offset:%9\n"                                             \
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])                                \
        : "v"(a0), "v"(a1), "n"(so), "n"(so + 2048u), "n"(so + 4096u), "n"(so + 6144u));  \
  }
      MLOP_VT_ISSUE(0, ra)
#pragma unroll
      for (int dblk = 0; dblk < 4; ++dblk) {
        v4s16 (&cv)[4] = (dblk & 1) ? rb : ra;
        v4s16 (&nv)[4] = (dblk & 1) ? ra : rb;
        if (dblk < 3) {
          MLOP_VT_ISSUE(dblk + 1, nv)
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(cv[0]), "+v"(cv[1]), "+v"(cv[2]), "+v"(cv[3]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cv[0]), "+v"(cv[1]), "+v"(cv[2]), "+v"(cv[3]));
        }
        bf16x8 f0, f1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f0[e] = cv[0][e];
          f0[4 + e] = cv[1][e];
          f1[e] = cv[2][e];
          f1[4 + e] = cv[3][e];
        }
        o[dblk] = mfma32(f0, pf[0], o[dblk]);
        o[dblk] = mfma32(f1, pf[1], o[dblk]);
      }
#undef MLOP_VT_ISSUE
    }
    if (++pp < cur.n_pairs) return false;
    tile_end();
    if (nxt.tile < 0) return true;
    cur = nxt;
    nxt = MLOP_FT(++k + 1);
    tile_start();
    return false;
  };

  q_issue(cur);
  issue_next(std::integral_constant<int, 0>{});
  issue_next(std::integral_constant<int, 1>{});
  nxt = MLOP_FT(1);
  tile_start();
  for (;;) {
    if (step(std::integral_constant<int, 0>{})) break;
    if (step(std::integral_constant<int, 1>{})) break;
    if (step(std::integral_constant<int, 2>{})) break;
  }
#undef MLOP_FT
}

// PERSIST: a persistent grid of S x Hkv workgroups (S slots per kv head; blockIdx % Hkv = kv
// head, so each head stays on one XCD as in the one-item grid) walks the tile list in rounds of
// S tiles, boustrophedon: slot j takes tile r S + j in even rounds and r S + S - 1 - j in odd
// ones.  The host's per-sequence latest-first tile order then pairs a heavy tile with its light
// mirror on every slot (16 x 512: positions p, 15 - p, p, 15 - p), and the launch holds whole
// rounds instead of ~2 k one-item workgroups.
template <int G, int WPC, bool PERSIST>
__global__ void __launch_bounds__(256, WPC) flash32_prefill_kernel(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ptile_seq, const int* __restrict__ ptile_q0,
    const int* __restrict__ q_start, const int* __restrict__ q_len,
    const int* __restrict__ ctx_len, int Hq, int Hkv, float scale_log2, int num_blocks, int num_ptiles) {
  constexpr int STAGES = 3;
  constexpr int STAGE = 4 * kBS * kD;    // bf16 per stage: K page A | K page B | V page A | V page B
  __shared__ __attribute__((aligned(256))) uint16_t smem[STAGES * STAGE];
  if constexpr (!PERSIST) {
    flash32_item<G>(smem, blockIdx.x / Hkv, blockIdx.x % Hkv, out, q, kc, vc, block_tables, bt_stride, ptile_seq,
                    ptile_q0, q_start, q_len, ctx_len, Hq, Hkv, scale_log2, num_blocks);
  } else {
    const int kvh = blockIdx.x % Hkv, j = blockIdx.x / Hkv, S = gridDim.x / Hkv;
    for (int r = 0; r * S < num_ptiles; ++r) {
      const int t = r * S + ((r & 1) ? S - 1 - j : j);
      if (t >= num_ptiles) continue;  // a partial last round: every slot still leaves the loop
      if (r > 0) __syncthreads();      // the previous tile's last ring reads before this tile's DMAs
      flash32_item<G>(smem, t, kvh, out, q, kc, vc, block_tables, bt_stride, ptile_seq, ptile_q0, q_start, q_len,
                      ctx_len, Hq, Hkv, scale_log2, num_blocks);
    }
  }
}

// flash_persist op: 0 = one workgroup per (tile, kv head) item; n = the persistent grid of n
// workgroups per CU (flash32_prefill_kernel PERSIST); n >= 64: exactly n / 64 slots per kv head
// (tests: several rounds on a few tiles).  Off by default: +3-5 % at 16 x 512 in the host's
// per-sequence order, nothing or -1-2 % at 1024+ tokens in the LPT order the engine uses there
// (profiles/r06_flash_persist.md).
static int g_flash_persist = 0;
int flash_persist(int set) {
  if (set >= 0) g_flash_persist = set;
  return g_flash_persist;
}

// flash_stream op: 1 = the persistent grid runs flash32_stream_kernel (cross-tile K / V ring and
// Q prefetch, 2 workgroups per CU) instead of flash32_item per tile; 0 = off
static int g_flash_stream = 0;
int flash_stream(int set) {
  if (set >= 0) g_flash_stream = set;
  return g_flash_stream;
}

static int device_cus() {
  static int cus[16] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) return 256;
  if (cus[dev] == 0) (void)hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev);
  return cus[dev] > 0 ? cus[dev] : 256;
}

void launch_flash_prefill(void* out, const void* q, const void* kc, const void* vc, const int* bt,
                          int bt_stride, const int* ptile_seq, const int* ptile_q0,
                          const int* q_start, const int* q_len, const int* ctx_len, int num_ptiles,
                          int Hq, int Hkv, float scale_log2, int num_blocks, hipStream_t st) {
  if (num_ptiles == 0) return;
  const int slots = g_flash_persist >= 64 ? g_flash_persist / 64
                    : g_flash_persist > 0 ? std::max(1, g_flash_persist * device_cus() / Hkv) : 0;
  const bool persist = slots > 0 && num_ptiles > slots;
  dim3 grid((persist ? slots : num_ptiles) * Hkv);
  const bool stream = persist && g_flash_stream;
#define MLOP_FLASH_CASE(GG)                                                                              \
  case GG:                                                                                               \
    if (stream)                                                                                          \
      flash32_stream_kernel<GG><<<grid, 256, 0, st>>>(                                                   \
          (uint16_t*)out, (const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, bt, bt_stride,   \
          ptile_seq, ptile_q0, q_start, q_len, ctx_len, Hq, Hkv, scale_log2, num_blocks, num_ptiles);    \
    else if (persist)                                                                                    \
      flash32_prefill_kernel<GG, 2, true><<<grid, 256, 0, st>>>(                                         \
          (uint16_t*)out, (const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, bt, bt_stride,   \
          ptile_seq, ptile_q0, q_start, q_len, ctx_len, Hq, Hkv, scale_log2, num_blocks, num_ptiles);    \
    else                                                                                                 \
      flash32_prefill_kernel<GG, 2, false><<<grid, 256, 0, st>>>(                                        \
          (uint16_t*)out, (const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, bt, bt_stride,   \
          ptile_seq, ptile_q0, q_start, q_len, ctx_len, Hq, Hkv, scale_log2, num_blocks, num_ptiles);    \
    break;
  switch (Hq / Hkv) {
    MLOP_FLASH_CASE(1)
    MLOP_FLASH_CASE(2)
    MLOP_FLASH_CASE(4)
    MLOP_FLASH_CASE(8)
    default: break;
  }
#undef MLOP_FLASH_CASE
}

}  // namespace mlop
