// Vector helpers shared by the TBE forward and backward translation units.
#pragma once
#include "common.hpp"

namespace {

using dlrm::kWave;

template <int VW>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
};
template <>
struct VecT<1> {
  using T = float;
};

__device__ __forceinline__ void vzero(float4& a) { a = make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void vzero(float& a) { a = 0.f; }
__device__ __forceinline__ void vadd(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}
__device__ __forceinline__ void vadd(float& a, const float& b) { a += b; }
// Compensated (Kahan) accumulation a += b, c carrying the lost low-order part: long runs
// of one row (hot rows: thousands of lookups) keep fp32 sums close to the exact sum.
__device__ __forceinline__ void vkahan(float& a, float& c, float b) {
  const float y = b - c;
  const float t = a + y;
  c = (t - a) - y;
  a = t;
}
__device__ __forceinline__ void vsub(float& a, const float& b) { a -= b; }
__device__ __forceinline__ void vsub(float4& a, const float4& b) {
  a.x -= b.x, a.y -= b.y, a.z -= b.z, a.w -= b.w;
}
__device__ __forceinline__ void vkahan(float4& a, float4& c, const float4& b) {
  vkahan(a.x, c.x, b.x);
  vkahan(a.y, c.y, b.y);
  vkahan(a.z, c.z, b.z);
  vkahan(a.w, c.w, b.w);
}
__device__ __forceinline__ void vfma(float4& a, float w, const float4& b) {
  a.x = fmaf(w, b.x, a.x);
  a.y = fmaf(w, b.y, a.y);
  a.z = fmaf(w, b.z, a.z);
  a.w = fmaf(w, b.w, a.w);
}
__device__ __forceinline__ void vfma(float& a, float w, const float& b) { a = fmaf(w, b, a); }
__device__ __forceinline__ void vscale(float4& a, float w) {
  a.x *= w;
  a.y *= w;
  a.z *= w;
  a.w *= w;
}
__device__ __forceinline__ void vscale(float& a, float w) { a *= w; }
// explicit fmas: the contraction of a.x*a.x + ... would otherwise be the compiler's choice
// per translation unit (the update passes run from two of them and must agree bitwise)
__device__ __forceinline__ float vdot(const float4& a) {
  return fmaf(a.w, a.w, fmaf(a.z, a.z, fmaf(a.y, a.y, a.x * a.x)));
}
__device__ __forceinline__ float vdot(const float& a) { return a * a; }

// ------------------------------------------------------ forward gather --
// Gather-reduce body over this workgroup's bags: `blk` / `nblk` = this workgroup's index and
// the number of gather workgroups (a launch may also hold other roles, tbe_bwd.hip).
template <int LPB, int VW, int MAXV, typename IdxT, typename OffT>
__device__ __forceinline__ void tbe_fwd_body(
    const float* __restrict__ W, int64_t D, const int64_t* __restrict__ row_base, int T, int B,
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const float* __restrict__ psw,
    float* __restrict__ out, int64_t out_bs, int32_t* __restrict__ err, int64_t blk,
    int64_t nblk) {
  using V = typename VecT<VW>::T;
  constexpr int GPW = kWave / LPB;  // bags per wave
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPB;
  const int gl = lane - g * LPB;
  const int nchunks = (int)(D / VW);
  const int64_t nbags = (int64_t)T * B;
  const int64_t wave_id = blk * (blockDim.x / kWave) + threadIdx.x / kWave;
  const int64_t nwaves = nblk * (blockDim.x / kWave);

  for (int64_t bag0 = wave_id * GPW; bag0 < nbags; bag0 += nwaves * GPW) {
    const int64_t bag = bag0 + g;
    const bool active = bag < nbags;
    int t = 0, b = 0;
    int64_t start = 0, end = 0, base = 0, nrows = 0;
    if (active) {
      t = (int)(bag / B);
      b = (int)(bag - (int64_t)t * B);
      start = (int64_t)off[bag];
      end = (int64_t)off[bag + 1];
      base = row_base[t];
      nrows = row_base[t + 1] - base;
    }
    V acc[MAXV];
#pragma unroll
    for (int c = 0; c < MAXV; ++c) vzero(acc[c]);

    for (int64_t l0 = start; l0 < end; l0 += LPB) {
      const int n = (int)((end - l0) < LPB ? (end - l0) : LPB);
      int64_t my_row = -1;
      float my_w = 1.f;
      if (gl < n) {
        int64_t r = (int64_t)idx[l0 + gl];
        if (r < 0 || r >= nrows) {
          if (err) atomicOr(err, DLRM_TBE_ERR_INDEX);
          r = -1;
        }
        my_row = r;
        if (psw) my_w = psw[l0 + gl];
      }
      for (int j = 0; j < n; j += 4) {
        int64_t r[4];
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = g * LPB + ((j + u) < LPB ? (j + u) : 0);
          r[u] = __shfl(my_row, src, kWave);
          w[u] = __shfl(my_w, src, kWave);
          if (j + u >= n) r[u] = -1;
        }
        V v[4][MAXV];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int c = 0; c < MAXV; ++c) {
            const int chunk = gl + c * LPB;
            if (r[u] >= 0 && chunk < nchunks) {
              v[u][c] = reinterpret_cast<const V*>(W + (base + r[u]) * D)[chunk];
            } else {
              vzero(v[u][c]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (r[u] >= 0) {
#pragma unroll
            for (int c = 0; c < MAXV; ++c) {
              if (psw)
                vfma(acc[c], w[u], v[u][c]);
              else
                vadd(acc[c], v[u][c]);
            }
          }
        }
      }
    }
    if (active) {
      V* o = reinterpret_cast<V*>(out + (int64_t)b * out_bs + (int64_t)t * D);
#pragma unroll
      for (int c = 0; c < MAXV; ++c) {
        const int chunk = gl + c * LPB;
        if (chunk < nchunks) o[chunk] = acc[c];
      }
    }
  }
}



// Bijective workgroup remap so each of the 8 XCDs (private 4 MiB L2 each; workgroups are
// dealt to XCDs round-robin) runs a CONTIGUOUS range of workgroup ids: over a sorted lookup
// array an XCD then works on one stretch of rows (C1: about one table), so the gradient
// rows and weight rows it touches stay in its own L2.
__device__ __forceinline__ int xcd_contiguous(int bid, int nwg) {
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace
