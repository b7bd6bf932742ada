// RoPE + paged K/V cache stores from a GEMM's LDS-staged C tile (EPI_ROPE of gemm.hip's
// kernels).  K and V pages are both token-major [NB, Hkv, 16, 128]: a token's head is one
// contiguous 256-B row (attention.hip reads V transposed out of LDS).
#pragma once
#include "common.h"
#include "launch.h"

namespace mlop {

// RoPE / paged-cache stores of `nheads` consecutive 128-wide heads of a staged 256-row
// C tile (EPI_ROPE).  `at(r, c)` returns the bf16-rounded projection output of tile row r,
// column c (column 0 = first column of head `head0`), so the math is rope_cache_kernel's
// on the same bf16 inputs.  Latency-shaped: every per-row index (position, slot) and the
// cos/sin values a thread needs are loaded up front in one batch (the accumulators are
// dead by now, so the registers are free), then the heads are rotated and stored; rows
// >= `rows` are skipped.
template <int NT, typename At>
__device__ __forceinline__ void rope_tile_store(const At& at, int head0, int nheads, int m0, int rows,
                                                const RopeEpi& re, int tid) {
  constexpr int D = 128, HALF = 64;
  constexpr int QK = 256 * (HALF / 8) / NT;  // (row, 8-column) items per thread and head
  const int cq = (tid & 7) * 8, rq = tid >> 3;       // item k: row rq + k * NT/8
  const int n_rope = re.Hq + re.Hkv, n_all = re.Hq + 2 * re.Hkv;
  const bool any_rope = head0 < n_rope, any_kv = head0 + nheads > re.Hq;
  int slot_q[QK];
  float4 cs[QK][4];
  if (any_kv) {  // K and V rows go to the same token-major page slot
#pragma unroll
    for (int k = 0; k < QK; ++k) {
      const int r = rq + k * (NT / 8);
      slot_q[k] = r < rows ? re.slots[m0 + r] : -1;
    }
  }
  if (any_rope) {
    int p[QK];
#pragma unroll
    for (int k = 0; k < QK; ++k) {
      const int r = rq + k * (NT / 8);
      p[k] = r < rows ? re.pos[m0 + r] : 0;
    }
#pragma unroll
    for (int k = 0; k < QK; ++k) {
      const float4* row = reinterpret_cast<const float4*>(re.cos_sin + (size_t)p[k] * D);
      cs[k][0] = row[cq / 4];
      cs[k][1] = row[cq / 4 + 1];
      cs[k][2] = row[(HALF + cq) / 4];
      cs[k][3] = row[(HALF + cq) / 4 + 1];
    }
  }
  for (int hh = 0; hh < nheads; ++hh) {
    const int head = head0 + hh;
    if (head >= n_all) break;
    if (head < n_rope) {
#pragma unroll
      for (int k = 0; k < QK; ++k) {
        const int r = rq + k * (NT / 8);
        if (r >= rows) continue;
        uint16_t* dst;
        if (head < re.Hq) {
          dst = re.q_out + ((size_t)(m0 + r) * re.Hq + head) * D;
        } else {
          const int slot = slot_q[k];
          if (slot < 0) continue;
          dst = re.k_cache + (((size_t)(slot / re.BS) * re.Hkv + (head - re.Hq)) * re.BS + slot % re.BS) * D;
        }
        const float cc[8] = {cs[k][0].x, cs[k][0].y, cs[k][0].z, cs[k][0].w,
                             cs[k][1].x, cs[k][1].y, cs[k][1].z, cs[k][1].w};
        const float ss[8] = {cs[k][2].x, cs[k][2].y, cs[k][2].z, cs[k][2].w,
                             cs[k][3].x, cs[k][3].y, cs[k][3].z, cs[k][3].w};
        u32x4 oa, ob;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x0 = at(r, hh * D + cq + 2 * j), x1 = at(r, hh * D + cq + 2 * j + 1);
          const float y0 = at(r, hh * D + HALF + cq + 2 * j), y1 = at(r, hh * D + HALF + cq + 2 * j + 1);
          oa[j] = pack2(x0 * cc[2 * j] - y0 * ss[2 * j], x1 * cc[2 * j + 1] - y1 * ss[2 * j + 1]);
          ob[j] = pack2(y0 * cc[2 * j] + x0 * ss[2 * j], y1 * cc[2 * j + 1] + x1 * ss[2 * j + 1]);
        }
        *reinterpret_cast<u32x4*>(dst + cq) = oa;
        *reinterpret_cast<u32x4*>(dst + HALF + cq) = ob;
      }
    } else {
      // V head: the token's row of its token-major page [NB, Hkv, BS, 128], 16-B stores
      const int kh = head - n_rope;
#pragma unroll
      for (int k = 0; k < QK; ++k) {
        const int r = rq + k * (NT / 8);
        const int slot = slot_q[k];
        if (r >= rows || slot < 0) continue;
        uint16_t* dst = re.v_cache + (((size_t)(slot / re.BS) * re.Hkv + kh) * re.BS + slot % re.BS) * D;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          u32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = hh * D + half * HALF + cq + 2 * j;
            o[j] = pack2(at(r, c), at(r, c + 1));
          }
          *reinterpret_cast<u32x4*>(dst + half * HALF + cq) = o;
        }
      }
    }
  }
}

}  // namespace mlop
