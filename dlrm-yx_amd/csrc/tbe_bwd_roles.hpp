// Embedding backward update phases (sorted-run block pass + cross-block combine) as
// device bodies: run by their own kernels (tbe_bwd.hip) or as extra workgroups of a
// grouped GEMM launch (gemm.hip, LaunchRole).  See tbe_bwd.hip for the pipeline.
#pragma once
#include <type_traits>

#include "head_roles.hpp"
#include "tbe_common.hpp"
#include "tbe_sort.hpp"

namespace {

constexpr int CH = 16;  // sorted lookups per block (all gradient rows of a block in flight)
// Large batches of lookups (>= kLongChN) use longer blocks (kLongCH): fewer runs cross a
// block edge, so fewer partial rows and less combine work; still 16 gradient rows in
// flight per lane group.  The partial buffer is sized for CH.
constexpr int kLongCH = 64;
constexpr int64_t kLongChN = 1 << 18;

// MODE_SGD_F16: exact SGD on fp16 weights (the fbgemm TBE's FP16 tables): the row is read
// as fp16, updated in fp32 and stored back rounded to nearest even.
enum { MODE_SGD = 0, MODE_ADAGRAD = 1, MODE_DENSE = 2, MODE_SGD_F16 = 3 };

// Weight-row element access by mode: fp32 rows, or fp16 rows (W then points at halves).
template <int MODE, int VW>
__device__ __forceinline__ typename VecT<VW>::T wload(const float* __restrict__ W, int64_t row,
                                                      int64_t D, int chunk) {
  if constexpr (MODE == MODE_SGD_F16) {
    const _Float16* h = reinterpret_cast<const _Float16*>(W) + row * D + (int64_t)chunk * VW;
    if constexpr (VW == 4) {
      const uint2 u = *reinterpret_cast<const uint2*>(h);
      return make_float4((float)__builtin_bit_cast(_Float16, (unsigned short)(u.x & 0xffff)),
                         (float)__builtin_bit_cast(_Float16, (unsigned short)(u.x >> 16)),
                         (float)__builtin_bit_cast(_Float16, (unsigned short)(u.y & 0xffff)),
                         (float)__builtin_bit_cast(_Float16, (unsigned short)(u.y >> 16)));
    } else {
      return (float)h[0];
    }
  } else {
    return reinterpret_cast<const typename VecT<VW>::T*>(W + row * D)[chunk];
  }
}

template <int MODE, int VW>
__device__ __forceinline__ void wstore(float* __restrict__ W, int64_t row, int64_t D, int chunk,
                                       const typename VecT<VW>::T& v) {
  if constexpr (MODE == MODE_SGD_F16) {
    _Float16* h = reinterpret_cast<_Float16*>(W) + row * D + (int64_t)chunk * VW;
    if constexpr (VW == 4) {
      auto bits = [](float f) { return (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)f); };
      uint2 u;
      u.x = bits(v.x) | (bits(v.y) << 16);
      u.y = bits(v.z) | (bits(v.w) << 16);
      *reinterpret_cast<uint2*>(h) = u;
    } else {
      h[0] = (_Float16)v;
    }
  } else {
    reinterpret_cast<typename VecT<VW>::T*>(W + row * D)[chunk] = v;
  }
}

// Apply the coalesced gradient g of one row (group-uniform control flow).
template <int LPB, int VW, int MAXV, int MODE>
__device__ __forceinline__ void finalize_row(float* __restrict__ W, float* __restrict__ mom,
                                             int64_t D, int64_t row,
                                             typename VecT<VW>::T (&g)[MAXV], int gl,
                                             int nchunks, float lr, float eps) {
  using V = typename VecT<VW>::T;
  V* wrow = reinterpret_cast<V*>(W + row * D);
  if (MODE == MODE_SGD || MODE == MODE_SGD_F16) {
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V w = wload<MODE, VW>(W, row, D, chunk);
        vfma(w, -lr, g[c]);
        wstore<MODE, VW>(W, row, D, chunk, w);
      }
    }
  } else if (MODE == MODE_DENSE) {
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V w = wrow[chunk];
        vadd(w, g[c]);
        wrow[chunk] = w;
      }
    }
  } else {  // RWSAdagrad: momentum += mean(g^2); w -= lr * g / (sqrt(momentum) + eps)
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < MAXV; ++c)
      if (gl + c * LPB < nchunks) sq += vdot(g[c]);
#pragma unroll
    for (int m = LPB / 2; m >= 1; m >>= 1) sq += __shfl_xor(sq, m, kWave);
    const float mnew = mom[row] + sq / (float)D;
    if (gl == 0) mom[row] = mnew;
    const float denom = sqrtf(mnew) + eps;
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V w = wrow[chunk];
        V u = g[c];
        if constexpr (VW == 4) {
          u.x /= denom;
          u.y /= denom;
          u.z /= denom;
          u.w /= denom;
        } else {
          u /= denom;
        }
        vfma(w, -lr, u);
        wrow[chunk] = w;
      }
    }
  }
}

// finalize_row with the row's weights (and momentum) already in registers: the load was
// issued with the gradient rows, so the read-modify-write costs no extra HBM round trip.
template <int LPB, int VW, int MAXV, int MODE>
__device__ __forceinline__ void finalize_row_pf(float* __restrict__ W, float* __restrict__ mom,
                                                int64_t D, int64_t row,
                                                typename VecT<VW>::T (&g)[MAXV],
                                                typename VecT<VW>::T (&w)[MAXV], float m0,
                                                int gl, int nchunks, float lr, float eps) {
  using V = typename VecT<VW>::T;
  V* wrow = reinterpret_cast<V*>(W + row * D);
  if (MODE == MODE_SGD || MODE == MODE_SGD_F16) {
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V x = w[c];
        vfma(x, -lr, g[c]);
        wstore<MODE, VW>(W, row, D, chunk, x);
      }
    }
  } else if (MODE == MODE_DENSE) {
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V x = w[c];
        vadd(x, g[c]);
        wrow[chunk] = x;
      }
    }
  } else {
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < MAXV; ++c)
      if (gl + c * LPB < nchunks) sq += vdot(g[c]);
#pragma unroll
    for (int m = LPB / 2; m >= 1; m >>= 1) sq += __shfl_xor(sq, m, kWave);
    const float mnew = m0 + sq / (float)D;
    if (gl == 0) mom[row] = mnew;
    const float denom = sqrtf(mnew) + eps;
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int chunk = gl + c * LPB;
      if (chunk < nchunks) {
        V x = w[c];
        V u = g[c];
        if constexpr (VW == 4) {
          u.x /= denom;
          u.y /= denom;
          u.z /= denom;
          u.w /= denom;
        } else {
          u /= denom;
        }
        vfma(x, -lr, u);
        wrow[chunk] = x;
      }
    }
  }
}

// SB: bag_of is indexed by sorted position (per-table sort) instead of by lookup position.
// FL: gradient rows in flight per lane group (16; 4 as a GEMM-launch role, whose
// register budget is 128 VGPRs - FL 8 spills there - and twice the waves are resident).
// FL only changes how many loads are issued ahead of the adds, never the order of the
// adds: same result.
// LEAN: no per-sample weights and a grad_out extent < 2^31 floats (32-bit row offsets):
// fewer registers for the role.
template <int LPB, int VW, int MAXV, typename KeyT, int MODE, bool SB, int FL = CH,
          bool LEAN = false>
__device__ __forceinline__ void tbe_bwd_block_body(
    float* __restrict__ W, float* __restrict__ mom, int64_t D, int B,
    const KeyT* __restrict__ keys, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ bag_of, const float* __restrict__ psw,
    const float* __restrict__ gout, int64_t gbs, int64_t N, float lr, float eps,
    KeyT sentinel, float* __restrict__ partial, int ch, int blk, int nblk) {
  using V = typename VecT<VW>::T;
  constexpr int GPW = kWave / LPB;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPB;
  const int gl = lane - g * LPB;
  const int nchunks = (int)(D / VW);
  const int64_t nblocks = (N + ch - 1) / ch;
  const int64_t wave_id = (int64_t)xcd_contiguous(blk, nblk) * (blockDim.x / kWave) +
                          threadIdx.x / kWave;
  const int64_t nwaves = (int64_t)nblk * (blockDim.x / kWave);

  for (int64_t k0 = wave_id * GPW; k0 < nblocks; k0 += nwaves * GPW) {
    const int64_t k = k0 + g;
    if (k >= nblocks) continue;
    const int64_t i0 = k * ch;
    const int64_t i1 = (i0 + ch < N) ? i0 + ch : N;
    const bool has_prev = i0 > 0;
    const bool has_next = i1 < N;
    const KeyT prev_key = has_prev ? keys[i0 - 1] : sentinel;
    const KeyT next_key = has_next ? keys[i1] : sentinel;

    V acc[MAXV], comp[MAXV];  // run sum, Kahan-compensated (hot rows: long runs)
#pragma unroll
    for (int c = 0; c < MAXV; ++c) vzero(acc[c]), vzero(comp[c]);
    KeyT cur = sentinel;
    int64_t seg_a = i0;
    bool have = false;

    // PF: the weight row (and momentum) of every run start in a chunk is loaded together
    // with the chunk's gradient rows (MAXV == 1 keeps that within the register budget)
    constexpr bool PF = MAXV == 1;
    V wcur[MAXV];
    float mcur = 0.f;
#pragma unroll
    for (int c = 0; c < MAXV; ++c) vzero(wcur[c]);

    auto flush = [&](int64_t b_end) {
      if (cur == sentinel) return;
#pragma unroll
      for (int c = 0; c < MAXV; ++c) vsub(acc[c], comp[c]);  // fold the compensation in
      const bool starts = (seg_a > i0) || !has_prev || (prev_key != cur);
      const bool ends = (b_end < i1) || !has_next || (next_key != cur);
      if (starts && ends) {
        if constexpr (PF)
          finalize_row_pf<LPB, VW, MAXV, MODE>(W, mom, D, (int64_t)cur, acc, wcur, mcur, gl,
                                               nchunks, lr, eps);
        else
          finalize_row<LPB, VW, MAXV, MODE>(W, mom, D, (int64_t)cur, acc, gl, nchunks, lr, eps);
      } else {
        V* dst = reinterpret_cast<V*>(partial + (2 * k + (seg_a == i0 ? 0 : 1)) * D);
#pragma unroll
        for (int c = 0; c < MAXV; ++c)
          if (gl + c * LPB < nchunks) dst[gl + c * LPB] = acc[c];
      }
    };

    // a sub-batch is SUB lookups (>= FL: narrow rows keep FL gradient rows in flight), each
    // lane of the group holding R = SUB / LPB of them
    static_assert(FL <= CH && CH % FL == 0, "FL divides the block length");
    constexpr int SUB = LPB >= FL ? LPB : FL;
    constexpr int R = SUB / LPB;
    for (int64_t base = i0; base < i1; base += SUB) {
      const int n = (int)((i1 - base) < SUB ? (i1 - base) : SUB);
      using GOff = std::conditional_t<LEAN, int32_t, int64_t>;
      KeyT my_key[R];
      GOff my_off[R];
      float my_w[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        my_key[r] = sentinel;
        my_off[r] = -1;
        my_w[r] = 1.f;
        const int li = r * LPB + gl;
        if (li < n) {
          my_key[r] = keys[base + li];
          int32_t bag;
          if constexpr (SB) {
            bag = bag_of[base + li];
            if (!LEAN && psw) my_w[r] = psw[pos[base + li]];
          } else {
            const int32_t p = pos[base + li];
            bag = p >= 0 ? bag_of[p] : -1;
            if (!LEAN && psw && p >= 0) my_w[r] = psw[p];
          }
          if (bag >= 0) {
            const int t = bag / B;
            const int b = bag - t * B;
            my_off[r] = (GOff)((int64_t)b * gbs + (int64_t)t * D);
          }
        }
      }
      constexpr int U = SUB < FL ? SUB : FL;  // gradient rows in flight per group (ch >= CH)
      for (int j = 0; j < n; j += U) {
        KeyT ku[U];
        GOff ou[U];
        float wu[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // lookup li of the sub-batch: lane li % LPB of the group, its register li / LPB
          // (R > 1 only for LPB < 16, where U == SUB and j == 0: li is a constant)
          static_assert(R == 1 || U == SUB, "narrow rows: one pass per sub-batch");
          const int li = R == 1 ? ((j + u) < LPB ? (j + u) : 0) : u;
          const int src = g * LPB + (R == 1 ? li : li % LPB);
          const int rr = R == 1 ? 0 : li / LPB;
          if constexpr (sizeof(KeyT) == 8)
            ku[u] = (KeyT)__shfl((long long)my_key[rr], src, kWave);
          else
            ku[u] = (KeyT)__shfl((int)my_key[rr], src, kWave);
          ou[u] = __shfl(my_off[rr], src, kWave);
          wu[u] = __shfl(my_w[rr], src, kWave);
          if (j + u >= n) ou[u] = -1;
        }
        V gv[U][MAXV];
        V wv[PF ? U : 1][MAXV];
        float mv[PF ? U : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int c = 0; c < MAXV; ++c) {
            const int chunk = gl + c * LPB;
            if (ou[u] >= 0 && chunk < nchunks) {
              gv[u][c] = reinterpret_cast<const V*>(gout + ou[u])[chunk];
              if (!LEAN && psw) vscale(gv[u][c], wu[u]);
            } else {
              vzero(gv[u][c]);
            }
          }
          if constexpr (PF) {
            // rows starting a run inside the chunk (repeats of one row load it once)
            const bool lead = (j + u < n) && ku[u] != sentinel && (u == 0 || ku[u] != ku[u - 1]);
#pragma unroll
            for (int c = 0; c < MAXV; ++c) {
              const int chunk = gl + c * LPB;
              if (lead && chunk < nchunks)
                wv[u][c] = wload<MODE, VW>(W, (int64_t)ku[u], D, chunk);
              else
                vzero(wv[u][c]);
            }
            mv[u] = (MODE == MODE_ADAGRAD && lead) ? mom[ku[u]] : 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (j + u < n) {
            if (!have || ku[u] != cur) {
              if (have) flush(base + j + u);
              have = true;
              cur = ku[u];
              seg_a = base + j + u;
#pragma unroll
              for (int c = 0; c < MAXV; ++c) vzero(acc[c]), vzero(comp[c]);
              if constexpr (PF) {
#pragma unroll
                for (int c = 0; c < MAXV; ++c) wcur[c] = wv[u][c];
                mcur = mv[u];
              }
            }
#pragma unroll
            for (int c = 0; c < MAXV; ++c) vkahan(acc[c], comp[c], gv[u][c]);
          }
        }
      }
    }
    if (have) flush(i1);
  }
}

// NF0: partial rows in flight (role: 8, see FL above; the add order is fixed either way)
template <int LPB, int VW, int MAXV, typename KeyT, int MODE, int NF0 = 16>
__device__ __forceinline__ void tbe_bwd_combine_body(
    float* __restrict__ W, float* __restrict__ mom, int64_t D, const KeyT* __restrict__ keys,
    int64_t N, float lr, float eps, KeyT sentinel, const float* __restrict__ partial, int ch,
    int blk, int nblk) {
  using V = typename VecT<VW>::T;
  constexpr int GPW = kWave / LPB;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPB;
  const int gl = lane - g * LPB;
  const int nchunks = (int)(D / VW);
  const int64_t nblocks = (N + ch - 1) / ch;
  const int64_t wave_id = (int64_t)xcd_contiguous(blk, nblk) * (blockDim.x / kWave) +
                          threadIdx.x / kWave;
  const int64_t nwaves = (int64_t)nblk * (blockDim.x / kWave);

  for (int64_t k0 = wave_id * GPW; k0 < nblocks; k0 += nwaves * GPW) {
    const int64_t k = k0 + g;
    if (k >= nblocks) continue;
    const int64_t i0 = k * ch;
    const int64_t i1 = (i0 + ch < N) ? i0 + ch : N;
    if (i1 >= N) continue;
    const KeyT last = keys[i1 - 1];
    if (last == sentinel || keys[i1] != last) continue;  // run ends inside this block
    // start of the last segment: first index of the block holding `last` (keys sorted)
    int64_t a = i1;
    for (int64_t i = i0 + gl; i < i1; i += LPB)
      if (keys[i] == last && i < a) a = i;
#pragma unroll
    for (int m = LPB / 2; m >= 1; m >>= 1) {
      const int64_t o = __shfl_xor(a, m, kWave);
      a = o < a ? o : a;
    }
    const bool starts = (a > i0) || (i0 == 0) || (keys[i0 - 1] != last);
    if (!starts) continue;  // the block where the run starts combines it
    // Last block of the run: the run is contiguous, so "block kk continues it" (its first
    // key equals `last`) holds for kk = k+1 .. kend and fails after.  The group's lanes
    // probe LPB blocks per round in parallel instead of walking them one by one.
    int64_t kend = k + 1;  // blocks k+1 .. kend-1 ... resolved below (kend = last one)
    {
      int64_t base = k + 1;
      while (true) {
        const int64_t kk = base + gl;
        const bool cont = kk < nblocks && keys[kk * ch] == last;
        // groups are LPB-aligned lane ranges: find the first lane (in order) that fails
        uint64_t fail = __ballot(!cont);
        if constexpr (LPB < 64) fail = (fail >> ((lane / LPB) * LPB)) & ((1ull << LPB) - 1);
        if (fail) {
          kend = base + __builtin_ctzll(fail) - 1;
          break;
        }
        base += LPB;
      }
    }
    V acc[MAXV];
    const V* src = reinterpret_cast<const V*>(partial + (2 * k + (a == i0 ? 0 : 1)) * D);
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      if (gl + c * LPB < nchunks)
        acc[c] = src[gl + c * LPB];
      else
        vzero(acc[c]);
    }
    // partials of blocks k+1 .. kend in block order, NF loads in flight, Kahan-compensated
    // (a hot row's run crosses hundreds of blocks)
    V comp[MAXV];
#pragma unroll
    for (int c = 0; c < MAXV; ++c) vzero(comp[c]);
    constexpr int NF = MAXV <= 2 ? NF0 : 8;
    for (int64_t kk0 = k + 1; kk0 <= kend; kk0 += NF) {
      V pv[NF][MAXV];
#pragma unroll
      for (int u = 0; u < NF; ++u) {
        const int64_t kk = kk0 + u;
        const V* s2 = reinterpret_cast<const V*>(partial + (2 * kk) * D);
#pragma unroll
        for (int c = 0; c < MAXV; ++c) {
          if (kk <= kend && gl + c * LPB < nchunks)
            pv[u][c] = s2[gl + c * LPB];
          else
            vzero(pv[u][c]);
        }
      }
#pragma unroll
      for (int u = 0; u < NF; ++u)
        if (kk0 + u <= kend) {
#pragma unroll
          for (int c = 0; c < MAXV; ++c) vkahan(acc[c], comp[c], pv[u][c]);
        }
    }
#pragma unroll
    for (int c = 0; c < MAXV; ++c) vsub(acc[c], comp[c]);  // fold the compensation back in
    finalize_row<LPB, VW, MAXV, MODE>(W, mom, D, (int64_t)last, acc, gl, nchunks, lr, eps);
  }
}


// The block pass and combine pass as kernels of their own.
template <int LPB, int VW, int MAXV, typename KeyT, int MODE, bool SB>
__global__ __launch_bounds__(256) void tbe_bwd_block_kernel(
    float* __restrict__ W, float* __restrict__ mom, int64_t D, int B,
    const KeyT* __restrict__ keys, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ bag_of, const float* __restrict__ psw,
    const float* __restrict__ gout, int64_t gbs, int64_t N, float lr, float eps,
    KeyT sentinel, float* __restrict__ partial, int ch) {
  tbe_bwd_block_body<LPB, VW, MAXV, KeyT, MODE, SB>(W, mom, D, B, keys, pos, bag_of, psw, gout,
                                                    gbs, N, lr, eps, sentinel, partial, ch,
                                                    blockIdx.x, gridDim.x);
}

template <int LPB, int VW, int MAXV, typename KeyT, int MODE>
__global__ __launch_bounds__(256) void tbe_bwd_combine_kernel(
    float* __restrict__ W, float* __restrict__ mom, int64_t D, const KeyT* __restrict__ keys,
    int64_t N, float lr, float eps, KeyT sentinel, const float* __restrict__ partial, int ch) {
  tbe_bwd_combine_body<LPB, VW, MAXV, KeyT, MODE>(W, mom, D, keys, N, lr, eps, sentinel, partial,
                                                  ch, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------ deferred update --
// An embedding-backward update whose two passes run as extra workgroups of two later
// launches (dlrm_tbe_backward_defer + dlrm_gemm_f32_group_role): the block pass (phase 1)
// and the combine pass (phase 2) are HBM-bound, the bottom-MLP backward GEMMs they share a
// launch with are MFMA-bound, and one launch holding both overlaps them with no
// cross-queue dependency.  Same bodies, same blocks, same result as the standalone kernels.
// Fused instantiations: float4 rows with one chunk per lane (D = 4 * LPB, LPB 4..32), SGD
// or row-wise Adagrad, 32-bit keys, bags by sorted position, no per-sample weights.
constexpr uint32_t kRoleMagic = 0x7b3e0001u;
struct LaunchRole {
  float* W;
  float* mom;
  const uint32_t* keys;
  const int32_t* pos;
  const int32_t* bag_of;
  const float* psw;
  const float* gout;
  float* partial;
  int64_t D, gbs, N;
  float lr, eps;
  uint32_t sentinel, magic;
  int32_t B, ch, mode, lpb;
  int32_t blocks;  // workgroups of either pass; 0 = nothing deferred
  int32_t kind;  // kRoleUpdate (phases 1, 2), kRoleHead (4)
  // phase 4, the head's finalize pass (dlrm_head_step_defer)
  struct {
    int64_t M, K, nblk;
    const float* part;
    float* w;
    float* dw;
    const float* row_loss;
    float* loss_out;
    float lr;
    int32_t accumulate;
  } head;
};
// (phase 3, the per-table sort as a role, is gone: measured slower than the sort in the
// lookup launch at C3, C2 and B = 256, profiles/r04_sort_role_ab.txt; ABI v7)
enum { kRoleNone = 0, kRoleUpdate = 1, kRoleHead = 3 };
inline int role_kind_of_phase(int phase) {
  return phase == 1 || phase == 2 ? kRoleUpdate : phase == 4 ? kRoleHead : kRoleNone;
}

inline bool tbe_role_fusable(int mode, int lpb, const float* psw, int64_t grad_extent) {
  return (mode == MODE_SGD || mode == MODE_ADAGRAD) && lpb >= 4 && lpb <= 32 && !psw &&
         grad_extent < (int64_t)INT32_MAX;
}

template <int PHASE, int LPB, int MODE>
__device__ __forceinline__ void tbe_role_pass(const LaunchRole& r, int blk) {
  if constexpr (PHASE == 1)
    tbe_bwd_block_body<LPB, 4, 1, uint32_t, MODE, true, 4, true>(r.W, r.mom, r.D, r.B, r.keys, r.pos,
                                                        r.bag_of, r.psw, r.gout, r.gbs, r.N,
                                                        r.lr, r.eps, r.sentinel, r.partial, r.ch,
                                                        blk, r.blocks);
  else
    tbe_bwd_combine_body<LPB, 4, 1, uint32_t, MODE, 8>(r.W, r.mom, r.D, r.keys, r.N, r.lr, r.eps,
                                                    r.sentinel, r.partial, r.ch, blk, r.blocks);
}

template <int PHASE, int LPB>
__device__ __forceinline__ void tbe_role_lpb(const LaunchRole& r, int blk) {
  if (r.mode == MODE_SGD)
    tbe_role_pass<PHASE, LPB, MODE_SGD>(r, blk);
  else
    tbe_role_pass<PHASE, LPB, MODE_ADAGRAD>(r, blk);
}

template <int PHASE>
__device__ __forceinline__ void tbe_role_run(const LaunchRole& r, int blk, void* lds) {
  if constexpr (PHASE == 4) {
    head_finalize_body(r.head.M, r.head.K, r.head.nblk, r.head.part, r.head.w, r.head.lr,
                       r.head.dw, r.head.accumulate, r.head.row_loss, r.head.loss_out, blk,
                       r.blocks, static_cast<float*>(lds));
    return;
  }
  switch (r.lpb) {
    case 4: tbe_role_lpb<PHASE, 4>(r, blk); break;
    case 8: tbe_role_lpb<PHASE, 8>(r, blk); break;
    case 16: tbe_role_lpb<PHASE, 16>(r, blk); break;
    default: tbe_role_lpb<PHASE, 32>(r, blk); break;
  }
}

// The update passes as launches of their own (the backward's default wherever the lean
// variant applies; same bodies as the GEMM-launch roles).
template <int PHASE>
__global__ __launch_bounds__(256, 4) void tbe_update_pass_kernel(const LaunchRole r) {
  tbe_role_run<PHASE>(r, blockIdx.x, nullptr);
}

}  // namespace
