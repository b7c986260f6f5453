// DLRM feature interaction (DLRM_Net.interact_features, dlrm_s_pytorch.py:627-665).
//
// dot:  T = [x, ly_1 .. ly_{F-1}] (F x D per sample), Z = T T^T, R = [x, Z[tril(F,F,-1|0)]]
// cat:  R = [x, ly_1, ..., ly_{F-1}]
//
// The dot interaction is a genuine batched (F x D)(D x F) product, so it runs on the
// fp32 matrix core: one wave per sample, the sample's F rows staged in LDS with an odd
// row pitch (D+1 floats: the 32 rows a half-wave reads are on 32 distinct banks), and
// Z accumulated in one 32x32 v_mfma_f32_32x32x2_f32 tile.  Because both operands are
// the same matrix, each lane feeds the same LDS value as A and B (lane (f, h) supplies
// T[f][k] for the k-slice of its half-wave); the k order only permutes the fmaf chain.
// The tril gather and the [x, Zflat] concat are fused into the tile epilogue.
// Backward: dT = (G + G^T) T with G the lower-triangular scatter of dR, built in LDS
// (no atomics: every (i,j) cell has exactly one writer), then 32x32 MFMA tiles over D.
// Features are addressed through per-feature (pointer, batch stride) pairs, so the
// same kernel reads [B][T][D] TBE output, the rank-major all-to-all receive buffer of
// distributed_forward, or the reference's list of per-table [B, D] tensors.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int kMaxF = 64;

struct FeatArgs {
  const float* ptr[kMaxF];
  int64_t bs[kMaxF];
};
struct GradArgs {
  float* ptr[kMaxF];
  int64_t bs[kMaxF];
};
// The one-hot lookup fused into the interaction (dlrm_interact_dot_forward_gather): feature
// f >= 1 of sample b is row row_base[f-1] + idx[(f-1) * B + b] of W (L = 1, table-major
// CSR indices: the lookup of apply_emb with one index per bag); feature 0 stays fa.ptr[0].
struct GatherArgs {
  const float* W;
  const int64_t* row_base;  // [F] device: table starts, row_base[F-1] = total rows
  const int32_t* idx;       // [(F-1) * B]
  int32_t* err;             // DLRM_TBE_ERR_INDEX on an index outside its table (may be null)
};

// p-th pair of the row-major lower triangle (i > j, or i >= j with self interaction).
__device__ __forceinline__ void pair_of(int p, bool self, int& i, int& j) {
  if (self) {
    int ii = (int)((sqrtf(1.f + 8.f * (float)p) - 1.f) * 0.5f);
    while (ii * (ii + 1) / 2 > p) --ii;
    while ((ii + 1) * (ii + 2) / 2 <= p) ++ii;
    i = ii;
    j = p - ii * (ii + 1) / 2;
  } else {
    int ii = (int)((1.f + sqrtf(1.f + 8.f * (float)p)) * 0.5f);
    while (ii * (ii - 1) / 2 > p) --ii;
    while ((ii + 1) * ii / 2 <= p) ++ii;
    i = ii;
    j = p - ii * (ii - 1) / 2;
  }
}

__device__ __forceinline__ int pair_index(int i, int j, bool self) {
  return self ? i * (i + 1) / 2 + j : i * (i - 1) / 2 + j;
}

// --------------------------------------------------------- MFMA forward --
// LDS-resident samples per workgroup (1..4 waves) so that the request stays <= 64 KiB.
int waves_for(size_t per_wave_bytes) {
  for (int w = 4; w >= 1; w >>= 1)
    if (per_wave_bytes * w <= 64 * 1024) return w;
  return 0;
}

__global__ __launch_bounds__(256) void interact_dot_fwd_mfma(int B, int F, int D, FeatArgs fa,
                                                             int self, float* __restrict__ out,
                                                             int64_t ld_out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const int DP = D + 1;
  float* Tl = lds + wave * F * DP;
  const int KH = (D + 1) / 2;  // k-slice per half-wave

  const int wpb = blockDim.x >> 6;
  for (int64_t bb = (int64_t)blockIdx.x * wpb; bb < B; bb += (int64_t)gridDim.x * wpb) {
    const int64_t b = bb + wave;
    const bool active = b < B;
    if (active) {
      for (int f = 0; f < F; ++f) {
        const float* src = fa.ptr[f] + b * fa.bs[f];
        for (int d = lane; d < D; d += 64) Tl[f * DP + d] = src[d];
      }
    }
    __syncthreads();
    if (active) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const bool rowok = l32 < F;
      const float* trow = Tl + l32 * DP + h * KH;
      for (int s = 0; s < KH; ++s) {
        const int k = h * KH + s;
        const float a = (rowok && k < D) ? trow[s] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, acc, 0, 0, 0);
      }
      float* orow = out + b * ld_out;
      for (int d = lane; d < D; d += 64) orow[d] = Tl[d];
      const int j = l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i < F && (self ? i >= j : i > j)) orow[D + pair_index(i, j, self)] = acc[r];
      }
    }
    __syncthreads();
  }
}

// -------------------------------------------------------- MFMA backward --
__global__ __launch_bounds__(256) void interact_dot_bwd_mfma(int B, int F, int D, FeatArgs fa,
                                                             int self,
                                                             const float* __restrict__ gout,
                                                             int64_t ld_g, GradArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const int DP = D + 1;
  constexpr int SP = 33;
  float* Tl = lds + wave * (F * DP + 32 * SP);
  float* Sl = Tl + F * DP;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int FK = (F + 1) & ~1;  // K extent rounded to the MFMA k-step

  const int wpb = blockDim.x >> 6;
  for (int64_t bb = (int64_t)blockIdx.x * wpb; bb < B; bb += (int64_t)gridDim.x * wpb) {
    const int64_t b = bb + wave;
    const bool active = b < B;
    if (active) {
      for (int f = 0; f < F; ++f) {
        const float* src = fa.ptr[f] + b * fa.bs[f];
        for (int d = lane; d < D; d += 64) Tl[f * DP + d] = src[d];
      }
      for (int c = lane; c < 32 * SP; c += 64) Sl[c] = 0.f;
    }
    __syncthreads();
    if (active) {
      const float* grow = gout + b * ld_g;
      for (int p = lane; p < npairs; p += 64) {
        int i, j;
        pair_of(p, self, i, j);
        const float v = grow[D + p];
        if (i == j) {
          Sl[i * SP + i] = 2.f * v;
        } else {
          Sl[i * SP + j] = v;
          Sl[j * SP + i] = v;
        }
      }
    }
    __syncthreads();
    if (active) {
      const float* grow = gout + b * ld_g;
      for (int n0 = 0; n0 < D; n0 += 32) {
        const int n = n0 + l32;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        for (int k0 = 0; k0 < FK; k0 += 2) {
          const int k = k0 + h;
          const float a = Sl[l32 * SP + k];
          const float bv = (k < F && n < D) ? Tl[k * DP + n] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc, 0, 0, 0);
        }
        if (n < D) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (i < F) {
              float v = acc[r];
              if (i == 0) v += grow[n];
              ga.ptr[i][b * ga.bs[i] + n] = v;
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------ LDS-staged kernels (compile-time D) --
// One wave per sample, four waves per workgroup stepping through the batch together.
// Loads and stores move whole feature rows as float4 with C4 = D/4 lanes per row, so a
// wave-instruction touches 64/C4 rows; the row pointers of an instruction are picked
// from the (uniform) kernel arguments with v_cndmask, never lane-indexed (a lane-indexed
// kernarg read compiles to a waterfall loop).
template <int D>
__device__ __forceinline__ const float* row_ptr(const FeatArgs& fa, int F, int64_t b, int i0,
                                                int sub) {
  constexpr int RPI = 64 / (D / 4);
  const float* p = fa.ptr[0];
  int64_t bs = 0;
#pragma unroll
  for (int j = 0; j < RPI; ++j) {
    const int f = i0 + j;
    const float* pj = f < F ? fa.ptr[f] : fa.ptr[0];
    const int64_t bj = f < F ? fa.bs[f] : 0;
    if (sub == j) p = pj, bs = bj;
  }
  return p + b * bs;
}

// Gather mode: lane f (1 <= f < F) looks up its feature's row for sample b (one index
// load per lane per sample; the table bounds were loaded once).  -1: index out of range
// (the row reads as zeros, like the TBE, which drops it from the bag, and is flagged).
__device__ __forceinline__ int64_t gather_row(const GatherArgs& gt, int F, int B, int64_t b,
                                              int lane, int64_t rb_lo, int64_t nrows,
                                              bool active) {
  if (lane < 1 || lane >= F) return 0;
  const int64_t r = gt.idx[(int64_t)(lane - 1) * B + b];
  if (r >= 0 && r < nrows) return rb_lo + r;
  if (active && gt.err) atomicOr(gt.err, DLRM_TBE_ERR_INDEX);
  return -1;
}

template <int D>
__device__ __forceinline__ float* grad_row_ptr(const GradArgs& ga, int F, int64_t b, int i0,
                                               int sub) {
  constexpr int RPI = 64 / (D / 4);
  float* p = ga.ptr[0];
  int64_t bs = 0;
#pragma unroll
  for (int j = 0; j < RPI; ++j) {
    const int f = i0 + j;
    float* pj = f < F ? ga.ptr[f] : ga.ptr[0];
    const int64_t bj = f < F ? ga.bs[f] : 0;
    if (sub == j) p = pj, bs = bj;
  }
  return p + b * bs;
}

// Forward: T (F x D) -> LDS with coalesced float4 loads; lane (f, h) then feeds T[f][k] for
// its k-half as both MFMA operands (Z = T T^T, two accumulator chains); the strict lower
// triangle and x are staged in LDS in output order and written as whole float4 rows.
template <int D, bool GATHER>
__global__ __launch_bounds__(256) void interact_dot_fwd_v4(int B, int F, FeatArgs fa, int self,
                                                           float* __restrict__ out,
                                                           int64_t ld_out, int width,
                                                           int vec_out, GatherArgs gt) {
  constexpr int DP = D + 4, C4 = D / 4, RPI = 64 / C4, KH = D / 2;
  constexpr int OUTP = D + 32 * 33 / 2 + 4;  // x + <= 528 pairs, rounded
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = lane >> 5, l32 = lane & 31;
  float* Tl = lds + wave * (32 * DP + OUTP);
  float* Ol = Tl + 32 * DP;
  const int sub = lane / C4, c = lane - sub * C4;
  const bool rowok = l32 < F;
  constexpr int NI = 32 / RPI;  // row-load instructions covering F <= 32 rows
  int64_t rb_lo = 0, nrows = 0;  // gather: lane f's table bounds (once per kernel)
  if (GATHER && lane >= 1 && lane < F) {
    rb_lo = gt.row_base[lane - 1];
    nrows = gt.row_base[lane] - rb_lo;
  }
  for (int64_t b0 = (int64_t)blockIdx.x * 4; b0 < B; b0 += (int64_t)gridDim.x * 4) {
    const int64_t b = b0 + wave;
    const bool active = b < B;
    {
      // every row load of the sample is issued before the first LDS write (one memory
      // latency per sample, not one per row group); rows >= F / inactive waves read a
      // valid row (feature 0 of sample 0) and store nothing
      const int64_t bl = active ? b : 0;
      const int64_t grow = GATHER ? gather_row(gt, F, B, bl, lane, rb_lo, nrows, active) : 0;
      float4 v[NI];
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if constexpr (GATHER) {
          const int f = q * RPI + sub;
          const int64_t g = __shfl(grow, f < 64 ? f : 0, 64);
          const float* src = (f >= 1 && g >= 0) ? gt.W + g * D : fa.ptr[0] + bl * fa.bs[0];
          v[q] = *reinterpret_cast<const float4*>(src + 4 * c);
          if (f >= 1 && g < 0) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          const float* src = row_ptr<D>(fa, F, bl, q * RPI, sub);
          v[q] = *reinterpret_cast<const float4*>(src + 4 * c);
        }
      }
      // unconditional stores (rows >= F are masked by rowok below; inactive waves' rows are
      // never read), so no load sinks into a branch and waits alone
#pragma unroll
      for (int q = 0; q < NI; ++q)
        *reinterpret_cast<float4*>(Tl + (q * RPI + sub) * DP + 4 * c) = v[q];
    }
    __syncthreads();
    if (active) {
      const float* trow = Tl + l32 * DP + h * KH;
      f32x16 acc0, acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
#pragma unroll
      for (int q = 0; q < KH / 4; ++q) {
        float4 v = *reinterpret_cast<const float4*>(trow + 4 * q);
        if (!rowok) v = make_float4(0.f, 0.f, 0.f, 0.f);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, v.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, v.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, v.w, acc1, 0, 0, 0);
      }
      for (int d = lane; d < D; d += 64) Ol[d] = Tl[d];  // x
      const int j = l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i < F && (self ? i >= j : i > j)) Ol[D + pair_index(i, j, self)] = acc0[r] + acc1[r];
      }
    }
    __syncthreads();
    if (active) {
      float* orow = out + b * ld_out;
      if (vec_out) {
        const int w4 = width / 4;
        for (int q = lane; q < w4; q += 64)
          *reinterpret_cast<float4*>(orow + 4 * q) = *reinterpret_cast<const float4*>(Ol + 4 * q);
        for (int q = 4 * w4 + lane; q < width; q += 64) orow[q] = Ol[q];
      } else {
        for (int q = lane; q < width; q += 64) orow[q] = Ol[q];
      }
    }
    __syncthreads();
  }
}

// Backward: T and the sample's dR row -> LDS (coalesced); S = G + G^T row by row from
// the staged dR; dT = S T per 32-column block on MFMA, each block written back over the
// T columns it consumed, then every feature's gradient row leaves as whole float4 rows.
// Feature 0 (the bottom-MLP output x) gets dR[0:D] added and, with relu_x, the ReLU' mask
// of x applied (the backward of the bottom MLP's last ReLU, fused).
template <int D, bool GATHER>
__global__ __launch_bounds__(256) void interact_dot_bwd_v3(int B, int F, FeatArgs fa, int self,
                                                           const float* __restrict__ gout,
                                                           int64_t ld_g, GradArgs ga,
                                                           int relu_x, int vec_g, GatherArgs gt) {
  constexpr int DP = D + 4, C4 = D / 4, RPI = 64 / C4;
  constexpr int GP = D + 32 * 33 / 2 + 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = lane >> 5, l32 = lane & 31;
  float* Tl = lds + wave * (32 * DP + GP);
  float* Gl = Tl + 32 * DP;
  const int sub = lane / C4, c = lane - sub * C4;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int width = D + npairs;
  constexpr int NI = 32 / RPI;          // row-load instructions covering 32 rows
  constexpr int NG = (GP / 4 + 63) / 64;  // float4 of the dR row per lane (vec_g)
  int64_t rb_lo = 0, nrows = 0;  // gather: lane f's table bounds (once per kernel)
  if (GATHER && lane >= 1 && lane < F) {
    rb_lo = gt.row_base[lane - 1];
    nrows = gt.row_base[lane] - rb_lo;
  }
  for (int64_t b0 = (int64_t)blockIdx.x * 4; b0 < B; b0 += (int64_t)gridDim.x * 4) {
    const int64_t b = b0 + wave;
    const bool active = b < B;
    {
      // all loads of the sample in flight at once (rows >= F are zero: they meet S's zeros)
      const int64_t bl = active ? b : 0;
      // (gather: the forward flagged bad indices; the backward reads them as zeros again)
      const int64_t grow = GATHER ? gather_row(gt, F, B, bl, lane, rb_lo, nrows, false) : 0;
      float4 v[NI];
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if constexpr (GATHER) {
          const int f = q * RPI + sub;
          const int64_t g = __shfl(grow, f < 64 ? f : 0, 64);
          const float* src = (f >= 1 && g >= 0) ? gt.W + g * D : fa.ptr[0] + bl * fa.bs[0];
          v[q] = *reinterpret_cast<const float4*>(src + 4 * c);
          if (f >= 1 && g < 0) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          const float* src = row_ptr<D>(fa, F, bl, q * RPI, sub);
          v[q] = *reinterpret_cast<const float4*>(src + 4 * c);
        }
      }
      const float* gsrc = gout + bl * ld_g;
      const int w4 = vec_g ? width / 4 : 0;
      float4 gv[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int q = lane + 64 * u;
        gv[u] = q < w4 ? *reinterpret_cast<const float4*>(gsrc + 4 * q)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      // unconditional stores into this wave's own LDS region (no load sinks into a branch)
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int f = q * RPI + sub;
        *reinterpret_cast<float4*>(Tl + f * DP + 4 * c) =
            f < F ? v[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int q = lane + 64 * u;
        if (4 * (lane + 64 * u) < GP) *reinterpret_cast<float4*>(Gl + 4 * q) = gv[u];
      }
      if (active)
        for (int q = 4 * w4 + lane; q < width; q += 64) Gl[q] = gsrc[q];
    }
    __syncthreads();
    if (active) {
      // S row l32, columns k = 16h + s: symmetric scatter of dR's pair gradients
      float sv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = 16 * h + s, i = l32;
        float v = 0.f;
        if (i < F && k < F) {
          if (i == k)
            v = self ? 2.f * Gl[D + pair_index(i, i, true)] : 0.f;
          else
            v = Gl[D + (i > k ? pair_index(i, k, self) : pair_index(k, i, self))];
        }
        sv[s] = v;
      }
#pragma unroll
      for (int n0 = 0; n0 < D; n0 += 32) {
        const int n = n0 + l32;
        float bv[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) bv[s] = n < D ? Tl[(16 * h + s) * DP + n] : 0.f;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sv[s], bv[s], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (n < D) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (i < F) {
              float v = acc[r];
              if (i == 0) {
                v += Gl[n];
                if (relu_x && !(Tl[n] > 0.f)) v = 0.f;
              }
              Tl[i * DP + n] = v;
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
    if (active) {
      for (int i0 = 0; i0 < F; i0 += RPI) {
        const int f = i0 + sub;
        float* dst = grad_row_ptr<D>(ga, F, b, i0, sub);
        if (f < F)
          *reinterpret_cast<float4*>(dst + 4 * c) = *reinterpret_cast<const float4*>(Tl + f * DP + 4 * c);
      }
    }
    __syncthreads();
  }
}

// Backward v4: one wave per (sample, 32-column block of D) - D / 32 waves per sample (one
// for D <= 32).  The wave stages its block of T (F rows x 32 columns, rows >= F zero) and
// the sample's dR row in its own LDS, builds S = G + G^T from the pairs as v3 does,
// computes dT_blk = S T_blk on MFMA (16 k-steps) and writes each gradient row's 32 block
// columns straight from the accumulators (a half-wave per row: 128 contiguous bytes).  At
// D = 128 the batch runs four times v3's waves with a quarter of its LDS each, so a
// sample's column blocks no longer run one after another in one wave.  Same products,
// same k order per element as v3: bitwise the same gradients.  Measured (r04_ibwd): Kaggle
// (D 16) 8.5 -> 6.8 us, but C3 (D 128) 20.6 -> 29.8 us - each of a sample's four waves
// rebuilds S and re-reads dR - so it is the default only for D <= 32 (one wave per sample);
// tuning INTERACT_BWD = 3 / 4 forces v3 / v4.
// Backward kernel for the compile-time D (tuning INTERACT_BWD: 3 / 4 / 5 forces v3 / v4 /
// v5; default v4 for D <= 32, above v5 for short batches, v3 for long ones); forward
// (INTERACT_FWD: 4 / 5; default v5 for D >= 64 and short batches).
// v5 pays where the batch is short against the chip (<= kV5MaxBatch samples: B = 256 C3
// step 181.4 -> 172.8 us, forward 9.7 -> 5.9 us, backward 15.2 -> 10.0 us); at B = 2048 its
// four times as many waves lose (forward 14.3 -> 16.2 us, backward 21.0 -> 26.3 us), so v4 /
// v3 keep the long batches (profiles/r05_interact_v5_ab.txt).
constexpr int64_t kV5MaxBatch = 1024;
inline int bwd_version(int D, int64_t B) {
  const int t = (int)dlrm::tuning(DLRM_TUNE_INTERACT_BWD);
  if (t == 3 || t == 4) return t;
  if (t == 5) return D >= 64 ? 5 : 4;
  if (D <= 32) return 4;
  return B <= kV5MaxBatch ? 5 : 3;
}
inline int fwd_version(int D, int64_t B) {
  const int t = (int)dlrm::tuning(DLRM_TUNE_INTERACT_FWD);
  if (t == 4) return 4;
  if (t == 5) return D >= 64 ? 5 : 4;
  return D >= 64 && B <= kV5MaxBatch ? 5 : 4;
}
inline int v5_grid(int64_t B) { return (int)std::min<int64_t>(B, 16384); }

template <int RPI>
__device__ __forceinline__ const float* row_ptr_n(const FeatArgs& fa, int F, int64_t b, int i0,
                                                  int sub) {
  const float* p = fa.ptr[0];
  int64_t bs = 0;
#pragma unroll
  for (int j = 0; j < RPI; ++j) {
    const int f = i0 + j;
    const float* pj = f < F ? fa.ptr[f] : fa.ptr[0];
    const int64_t bj = f < F ? fa.bs[f] : 0;
    if (sub == j) p = pj, bs = bj;
  }
  return p + b * bs;
}

template <int D, bool GATHER>
__global__ __launch_bounds__(256) void interact_dot_bwd_v4(int B, int F, FeatArgs fa, int self,
                                                           const float* __restrict__ gout,
                                                           int64_t ld_g, GradArgs ga,
                                                           int relu_x, int vec_g, GatherArgs gt) {
  constexpr int CB = D < 32 ? D : 32;       // columns per wave
  constexpr int NBLK = D / CB;              // waves per sample
  constexpr int TP = CB + 4;                // T-block row pitch
  constexpr int GP = D + 32 * 33 / 2 + 4;   // dR row: x part + <= 528 pairs
  constexpr int C4 = CB / 4, RPI = 64 / C4, NI = 32 / RPI;
  constexpr int NG = (GP / 4 + 63) / 64;    // float4 of the dR row per lane (vec_g)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = lane >> 5, l32 = lane & 31;
  float* Tl = lds + wave * (32 * TP + GP);
  float* Gl = Tl + 32 * TP;
  const int sub = lane / C4, c = lane - sub * C4;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int width = D + npairs;
  int64_t rb_lo = 0, nrows = 0;  // gather: lane f's table bounds (once per kernel)
  if (GATHER && lane >= 1 && lane < F) {
    rb_lo = gt.row_base[lane - 1];
    nrows = gt.row_base[lane] - rb_lo;
  }
  const int64_t nunits = (int64_t)B * NBLK;
  for (int64_t u0 = (int64_t)blockIdx.x * 4; u0 < nunits; u0 += (int64_t)gridDim.x * 4) {
    const int64_t u = u0 + wave;
    const bool active = u < nunits;
    const int64_t b = active ? u / NBLK : 0;
    const int c0 = active ? (int)(u - (u / NBLK) * NBLK) * CB : 0;
    {
      // the block's rows and the dR row, all loads in flight before the first LDS write
      const int64_t grow = GATHER ? gather_row(gt, F, B, b, lane, rb_lo, nrows, false) : 0;
      float4 v[NI];
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if constexpr (GATHER) {
          const int f = q * RPI + sub;
          const int64_t g = __shfl(grow, f < 64 ? f : 0, 64);
          const float* src = (f >= 1 && g >= 0) ? gt.W + g * D : fa.ptr[0] + b * fa.bs[0];
          v[q] = *reinterpret_cast<const float4*>(src + c0 + 4 * c);
          if (f >= 1 && g < 0) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          const float* src = row_ptr_n<RPI>(fa, F, b, q * RPI, sub);
          v[q] = *reinterpret_cast<const float4*>(src + c0 + 4 * c);
        }
      }
      const float* gsrc = gout + b * ld_g;
      const int w4 = vec_g ? width / 4 : 0;
      float4 gv[NG];
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int q = lane + 64 * k;
        gv[k] = q < w4 ? *reinterpret_cast<const float4*>(gsrc + 4 * q)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int f = q * RPI + sub;
        *reinterpret_cast<float4*>(Tl + f * TP + 4 * c) =
            f < F ? v[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int q = lane + 64 * k;
        if (4 * q < GP) *reinterpret_cast<float4*>(Gl + 4 * q) = gv[k];
      }
      if (active)
        for (int q = 4 * w4 + lane; q < width; q += 64) Gl[q] = gsrc[q];
    }
    __syncthreads();
    if (active) {
      // S row l32, columns k = 16h + s: symmetric scatter of dR's pair gradients
      float sv[16], bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = 16 * h + s, i = l32;
        float x = 0.f;
        if (i < F && k < F) {
          if (i == k)
            x = self ? 2.f * Gl[D + pair_index(i, i, true)] : 0.f;
          else
            x = Gl[D + (i > k ? pair_index(i, k, self) : pair_index(k, i, self))];
        }
        sv[s] = x;
        bv[s] = l32 < CB ? Tl[(16 * h + s) * TP + l32] : 0.f;
      }
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sv[s], bv[s], acc, 0, 0, 0);
      if (l32 < CB) {
        const int n = c0 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          // rows i0 (h = 0) and i0 + 4 (h = 1): row pointers picked from uniform arguments
          const int i0 = (r & 3) + 8 * (r >> 2), i = i0 + 4 * h;
          if (i < F) {
            float x = acc[r];
            if (i == 0) {
              x += Gl[n];
              if (relu_x && !(Tl[l32] > 0.f)) x = 0.f;
            }
            float* p0 = ga.ptr[i0 < kMaxF ? i0 : 0];
            float* p1 = ga.ptr[i0 + 4 < kMaxF ? i0 + 4 : 0];
            const int64_t s0 = ga.bs[i0 < kMaxF ? i0 : 0], s1 = ga.bs[i0 + 4 < kMaxF ? i0 + 4 : 0];
            float* dst = h ? p1 + b * s1 : p0 + b * s0;
            dst[n] = x;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------ v5: a workgroup per sample --
// D = 64 / 128: one sample per workgroup of D / 32 waves, each wave owning a 32-column
// block of T (F <= 32 rows staged once in LDS by the whole workgroup).  v4 ran one wave per
// sample, so a C3 batch of 2048 samples put 8 waves on a CU and every wave walked the
// whole sample (gather latency, 64 dependent MFMAs, the output row) alone; here the batch
// is D / 32 times as many waves with a quarter of the chain each.
//   forward: wave w multiplies its column block (Z_w = T_w T_w^T, 16 MFMAs); the partial
//            Grams meet in LDS and are added in block order for the lower triangle;
//   backward: wave w computes dT_w = S T_w (S = G + G^T from the staged dR, v3's products
//            in v3's k order: bitwise v3), writes it over its columns of T, and the
//            workgroup stores every gradient row as whole float4 rows.
template <int D>
__device__ __forceinline__ const float* row_ptr_w(const FeatArgs& fa, int F, int64_t b, int i0,
                                                  int sub) {
  constexpr int RPW = 64 / (D / 4);  // rows per wave-instruction
  const float* p = fa.ptr[0];
  int64_t bs = 0;
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int f = i0 + j;
    const float* pj = f < F ? fa.ptr[f] : fa.ptr[0];
    const int64_t bj = f < F ? fa.bs[f] : 0;
    if (sub == j) p = pj, bs = bj;
  }
  return p + b * bs;
}

template <int D>
__device__ __forceinline__ float* grad_ptr_w(const GradArgs& ga, int F, int64_t b, int i0,
                                             int sub) {
  constexpr int RPW = 64 / (D / 4);
  float* p = ga.ptr[0];
  int64_t bs = 0;
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int f = i0 + j;
    float* pj = f < F ? ga.ptr[f] : ga.ptr[0];
    const int64_t bj = f < F ? ga.bs[f] : 0;
    if (sub == j) p = pj, bs = bj;
  }
  return p + b * bs;
}

// T (F <= 32 rows, rows >= F zero) of sample b -> Tl (pitch DP), the whole workgroup.
template <int D, bool GATHER>
__device__ __forceinline__ void v5_load_t(int B, int F, const FeatArgs& fa, const GatherArgs& gt,
                                          int64_t b, float* Tl, bool flag) {
  constexpr int NT = 2 * D, C4 = D / 4, RPW = 64 / C4, RPB = NT / C4, NI = 32 / RPB;
  constexpr int DP = D + 4;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sw = lane / C4, c = lane - sw * C4;
  float4 v[NI];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int i0 = q * RPB + wave * RPW, f = i0 + sw;
    if constexpr (GATHER) {
      const float* src = fa.ptr[0] + b * fa.bs[0];
      bool zero = false;
      if (f >= 1 && f < F) {
        const int64_t lo = gt.row_base[f - 1], n = gt.row_base[f] - lo;
        const int64_t r = gt.idx[(int64_t)(f - 1) * B + b];
        if (r >= 0 && r < n) {
          src = gt.W + (lo + r) * D;
        } else {
          zero = true;
          if (flag && c == 0 && gt.err) atomicOr(gt.err, DLRM_TBE_ERR_INDEX);
        }
      }
      v[q] = *reinterpret_cast<const float4*>(src + 4 * c);
      if (zero) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      v[q] = *reinterpret_cast<const float4*>(row_ptr_w<D>(fa, F, b, i0, sw) + 4 * c);
    }
  }
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int f = q * RPB + wave * RPW + sw;
    *reinterpret_cast<float4*>(Tl + f * DP + 4 * c) =
        f < F ? v[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int D, bool GATHER>
__global__ __launch_bounds__(2 * D) void interact_dot_fwd_v5(int B, int F, FeatArgs fa, int self,
                                                             float* __restrict__ out,
                                                             int64_t ld_out, int width,
                                                             GatherArgs gt) {
  constexpr int NW = D / 32, DP = D + 4, PP = 33;
  __shared__ __attribute__((aligned(16))) float Tl[32 * DP];
  __shared__ float Pl[NW * 32 * PP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    v5_load_t<D, GATHER>(B, F, fa, gt, b, Tl, true);
    __syncthreads();
    {
      const float* trow = Tl + l32 * DP + 32 * wave + 16 * h;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(trow + 4 * q);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, v.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, v.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, v.w, acc, 0, 0, 0);
      }
      float* P = Pl + wave * 32 * PP;
#pragma unroll
      for (int r = 0; r < 16; ++r) P[((r & 3) + 8 * (r >> 2) + 4 * h) * PP + l32] = acc[r];
    }
    __syncthreads();
    float* orow = out + b * ld_out;
    for (int e = tid; e < width; e += 2 * D) {
      float v;
      if (e < D) {
        v = Tl[e];
      } else {
        int i, j;
        pair_of(e - D, self, i, j);
        v = Pl[i * PP + j];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += Pl[w * 32 * PP + i * PP + j];
      }
      orow[e] = v;
    }
    __syncthreads();
  }
}

template <int D, bool GATHER>
__global__ __launch_bounds__(2 * D) void interact_dot_bwd_v5(int B, int F, FeatArgs fa, int self,
                                                             const float* __restrict__ gout,
                                                             int64_t ld_g, GradArgs ga,
                                                             int relu_x, int vec_g,
                                                             GatherArgs gt) {
  constexpr int NT = 2 * D, DP = D + 4, C4 = D / 4, RPW = 64 / C4, RPB = NT / C4;
  constexpr int GP = D + 32 * 33 / 2 + 4;
  __shared__ __attribute__((aligned(16))) float Tl[32 * DP];
  __shared__ __attribute__((aligned(16))) float Gl[GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int width = D + npairs;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    {
      const float* gsrc = gout + b * ld_g;
      const int w4 = vec_g ? width / 4 : 0;
      for (int q = tid; q < w4; q += NT)
        *reinterpret_cast<float4*>(Gl + 4 * q) = *reinterpret_cast<const float4*>(gsrc + 4 * q);
      for (int q = 4 * w4 + tid; q < width; q += NT) Gl[q] = gsrc[q];
    }
    v5_load_t<D, GATHER>(B, F, fa, gt, b, Tl, false);
    __syncthreads();
    {
      // v3's S row l32 (columns k = 16h + s) and T block column n: same products, same order
      const int n = 32 * wave + l32;
      float sv[16], bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = 16 * h + s, i = l32;
        float v = 0.f;
        if (i < F && k < F) {
          if (i == k)
            v = self ? 2.f * Gl[D + pair_index(i, i, true)] : 0.f;
          else
            v = Gl[D + (i > k ? pair_index(i, k, self) : pair_index(k, i, self))];
        }
        sv[s] = v;
        bv[s] = Tl[(16 * h + s) * DP + n];
      }
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sv[s], bv[s], acc, 0, 0, 0);
      const bool xpos = Tl[n] > 0.f;  // row 0 of this column, read before it is overwritten
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i < F) {
          float v = acc[r];
          if (i == 0) {
            v += Gl[n];
            if (relu_x && !xpos) v = 0.f;
          }
          Tl[i * DP + n] = v;
        }
      }
    }
    __syncthreads();
    {
      const int sw = lane / C4, c = lane - sw * C4;
      for (int q = 0; q * RPB < F; ++q) {
        const int i0 = q * RPB + wave * RPW, f = i0 + sw;
        float* dst = grad_ptr_w<D>(ga, F, b, i0, sw);
        if (f < F)
          *reinterpret_cast<float4*>(dst + 4 * c) = *reinterpret_cast<const float4*>(Tl + f * DP + 4 * c);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------- generic VALU path (F > 32) --
__global__ __launch_bounds__(256) void interact_dot_fwd_generic(int B, int F, int D, FeatArgs fa,
                                                                int self, float* __restrict__ out,
                                                                int64_t ld_out) {
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int64_t W = D + npairs;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * W) return;
  const int64_t b = idx / W;
  const int c = (int)(idx - b * W);
  float* orow = out + b * ld_out;
  if (c < D) {
    orow[c] = fa.ptr[0][b * fa.bs[0] + c];
    return;
  }
  int i, j;
  pair_of(c - D, self, i, j);
  const float* ti = fa.ptr[i] + b * fa.bs[i];
  const float* tj = fa.ptr[j] + b * fa.bs[j];
  float s = 0.f;
  for (int d = 0; d < D; ++d) s = fmaf(ti[d], tj[d], s);
  orow[c] = s;
}

__global__ __launch_bounds__(256) void interact_dot_bwd_generic(int B, int F, int D, FeatArgs fa,
                                                                int self,
                                                                const float* __restrict__ gout,
                                                                int64_t ld_g, GradArgs ga) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * F * D) return;
  const int64_t b = idx / ((int64_t)F * D);
  const int rem = (int)(idx - b * F * D);
  const int i = rem / D;
  const int n = rem - i * D;
  const float* grow = gout + b * ld_g;
  float s = (i == 0) ? grow[n] : 0.f;
  for (int k = 0; k < F; ++k) {
    float g;
    if (k == i)
      g = self ? 2.f * grow[D + pair_index(i, i, true)] : 0.f;
    else if (k < i)
      g = grow[D + pair_index(i, k, self)];
    else
      g = grow[D + pair_index(k, i, self)];
    if (g != 0.f) s = fmaf(g, fa.ptr[k][b * fa.bs[k] + n], s);
  }
  ga.ptr[i][b * ga.bs[i] + n] = s;
}

// ------------------------------------------------------------------ cat --
__global__ __launch_bounds__(256) void interact_cat_fwd(int B, int F, int D, FeatArgs fa,
                                                        float* __restrict__ out, int64_t ld_out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * F * D) return;
  const int64_t b = idx / ((int64_t)F * D);
  const int rem = (int)(idx - b * F * D);
  const int f = rem / D;
  const int d = rem - f * D;
  out[b * ld_out + rem] = fa.ptr[f][b * fa.bs[f] + d];
}

__global__ __launch_bounds__(256) void interact_cat_bwd(int B, int F, int D,
                                                        const float* __restrict__ gout,
                                                        int64_t ld_g, GradArgs ga) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * F * D) return;
  const int64_t b = idx / ((int64_t)F * D);
  const int rem = (int)(idx - b * F * D);
  const int f = rem / D;
  const int d = rem - f * D;
  ga.ptr[f][b * ga.bs[f] + d] = gout[b * ld_g + rem];
}

// ReLU' of x applied to its gradient (fallback paths of relu_x): g0 *= (x > 0).
__global__ __launch_bounds__(256) void relu_mask_kernel(int B, int D, const float* __restrict__ x,
                                                        int64_t xbs, float* __restrict__ g,
                                                        int64_t gbs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * D) return;
  const int64_t b = i / D, d = i - b * D;
  if (!(x[b * xbs + d] > 0.f)) g[b * gbs + d] = 0.f;
}

int fill_feat(FeatArgs& fa, int F, const float* const* ptrs, const int64_t* bs, const char* name) {
  DLRM_ARG(ptrs && bs, "%s: null feature arrays", name);
  for (int f = 0; f < F; ++f) {
    DLRM_ARG(ptrs[f], "%s: null feature pointer %d", name, f);
    fa.ptr[f] = ptrs[f];
    fa.bs[f] = bs[f];
  }
  return DLRM_OK;
}

int fill_grad(GradArgs& ga, int F, float* const* ptrs, const int64_t* bs, const char* name) {
  DLRM_ARG(ptrs && bs, "%s: null gradient arrays", name);
  for (int f = 0; f < F; ++f) {
    DLRM_ARG(ptrs[f], "%s: null gradient pointer %d", name, f);
    ga.ptr[f] = ptrs[f];
    ga.bs[f] = bs[f];
  }
  return DLRM_OK;
}

// The v2 kernels move features as float4: every feature pointer and batch stride must
// keep 16-byte alignment.
bool aligned_feats(const FeatArgs& fa, int F) {
  for (int f = 0; f < F; ++f)
    if ((reinterpret_cast<uintptr_t>(fa.ptr[f]) & 15) || (fa.bs[f] & 3)) return false;
  return true;
}

int grid_for(int64_t B, int wpb) {
  int64_t g = dlrm::ceil_div(B, wpb);
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" int dlrm_interact_dot_forward(int32_t B, int32_t F, int32_t D,
                                         const float* const* feat_ptrs,
                                         const int64_t* feat_bstrides, int32_t self_interaction,
                                         float* out, int64_t ld_out, dlrm_stream_t stream) {
  const char* name = "dlrm_interact_dot_forward";
  DLRM_ARG(B >= 0 && F >= 1 && F <= kMaxF && D > 0, "%s: need F in [1,64], D > 0", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(out, "%s: null out", name);
  const int npairs = self_interaction ? F * (F + 1) / 2 : F * (F - 1) / 2;
  DLRM_ARG(ld_out >= D + npairs, "%s: ld_out < D + pairs", name);
  FeatArgs fa{};
  int rc = fill_feat(fa, F, feat_ptrs, feat_bstrides, name);
  if (rc) return rc;
  hipStream_t st = dlrm::as_stream(stream);
  // v4 (LDS-staged, coalesced rows) for the compile-time D; the runtime-D MFMA kernel or
  // the elementwise one otherwise
  const bool fast = F <= 32 && (D == 16 || D == 32 || D == 64 || D == 128) &&
                    aligned_feats(fa, F);
  if (fast && fwd_version(D, B) == 5) {
    const int width = D + npairs;
    if (D == 64)
      hipLaunchKernelGGL((interact_dot_fwd_v5<64, false>), dim3(v5_grid(B)), dim3(128), 0, st, B, F,
                         fa, self_interaction ? 1 : 0, out, ld_out, width, GatherArgs{});
    else
      hipLaunchKernelGGL((interact_dot_fwd_v5<128, false>), dim3(v5_grid(B)), dim3(256), 0, st, B,
                         F, fa, self_interaction ? 1 : 0, out, ld_out, width, GatherArgs{});
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  if (fast) {
    const int width = D + npairs;
    const int vec_out = ((reinterpret_cast<uintptr_t>(out) & 15) == 0 && ld_out % 4 == 0) ? 1 : 0;
    const size_t lds = 4 * (32 * (size_t)(D + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
    const int grid = (int)std::min<int64_t>(dlrm::ceil_div(B, 4), 8192);
#define L4(DD)                                                                                \
  hipLaunchKernelGGL((interact_dot_fwd_v4<DD, false>), dim3(grid), dim3(256), lds, st, B, F, fa, \
                     self_interaction ? 1 : 0, out, ld_out, width, vec_out, GatherArgs{})
    if (D == 16) L4(16); else if (D == 32) L4(32); else if (D == 64) L4(64); else L4(128);
#undef L4
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  const size_t per_wave = (size_t)F * (D + 1) * sizeof(float);
  const int wpb = waves_for(per_wave);
  if (F <= 32 && wpb > 0) {
    hipLaunchKernelGGL(interact_dot_fwd_mfma, dim3(grid_for(B, wpb)), dim3(64 * wpb),
                       per_wave * wpb, st, B, F, D, fa,
                       self_interaction ? 1 : 0, out, ld_out);
  } else {
    const int64_t n = (int64_t)B * (D + npairs);
    hipLaunchKernelGGL(interact_dot_fwd_generic, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0, st,
                       B, F, D, fa, self_interaction ? 1 : 0, out, ld_out);
  }
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

extern "C" int dlrm_interact_dot_backward(int32_t B, int32_t F, int32_t D,
                                          const float* const* feat_ptrs,
                                          const int64_t* feat_bstrides, int32_t self_interaction,
                                          const float* grad_out, int64_t ld_gout,
                                          float* const* grad_ptrs, const int64_t* grad_bstrides,
                                          int32_t relu_x, dlrm_stream_t stream) {
  const char* name = "dlrm_interact_dot_backward";
  DLRM_ARG(B >= 0 && F >= 1 && F <= kMaxF && D > 0, "%s: need F in [1,64], D > 0", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(grad_out, "%s: null grad_out", name);
  const int npairs = self_interaction ? F * (F + 1) / 2 : F * (F - 1) / 2;
  DLRM_ARG(ld_gout >= D + npairs, "%s: ld_gout < D + pairs", name);
  FeatArgs fa{};
  GradArgs ga{};
  int rc = fill_feat(fa, F, feat_ptrs, feat_bstrides, name);
  if (rc) return rc;
  rc = fill_grad(ga, F, grad_ptrs, grad_bstrides, name);
  if (rc) return rc;
  hipStream_t st = dlrm::as_stream(stream);
  // v3 (LDS-staged T and dR, coalesced rows, ReLU' fused) for the compile-time D; the
  // runtime-D MFMA kernel or the elementwise one otherwise (ReLU' then as a separate pass)
  const bool fast = F <= 32 && (D == 16 || D == 32 || D == 64 || D == 128) &&
                    aligned_feats(fa, F);
  bool grads_aligned = true;
  for (int f = 0; f < F; ++f)
    if ((reinterpret_cast<uintptr_t>(ga.ptr[f]) & 15) || (ga.bs[f] & 3)) grads_aligned = false;
  if (fast && grads_aligned) {
    const int vec_g = ((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0 && ld_gout % 4 == 0) ? 1 : 0;
    const int ver = bwd_version(D, B);
    if (ver == 5) {
      if (D == 64)
        hipLaunchKernelGGL((interact_dot_bwd_v5<64, false>), dim3(v5_grid(B)), dim3(128), 0, st, B,
                           F, fa, self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0,
                           vec_g, GatherArgs{});
      else
        hipLaunchKernelGGL((interact_dot_bwd_v5<128, false>), dim3(v5_grid(B)), dim3(256), 0, st, B,
                           F, fa, self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0,
                           vec_g, GatherArgs{});
      DLRM_LAUNCH_CHECK(name);
      return DLRM_OK;
    }
    if (ver == 4) {
      const int nblk = D > 32 ? D / 32 : 1, cb = D < 32 ? D : 32;
      const size_t lds = 4 * (32 * (size_t)(cb + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
      const int grid = (int)std::min<int64_t>(dlrm::ceil_div((int64_t)B * nblk, 4), 8192);
#define L4B(DD)                                                                               \
  hipLaunchKernelGGL((interact_dot_bwd_v4<DD, false>), dim3(grid), dim3(256), lds, st, B, F, fa, \
                     self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g,      \
                     GatherArgs{})
      if (D == 16) L4B(16); else if (D == 32) L4B(32); else if (D == 64) L4B(64); else L4B(128);
#undef L4B
      DLRM_LAUNCH_CHECK(name);
      return DLRM_OK;
    }
    const size_t lds = 4 * (32 * (size_t)(D + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
    const int grid = (int)std::min<int64_t>(dlrm::ceil_div(B, 4), 8192);
#define L3B(DD)                                                                               \
  hipLaunchKernelGGL((interact_dot_bwd_v3<DD, false>), dim3(grid), dim3(256), lds, st, B, F, fa, \
                     self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g,      \
                     GatherArgs{})
    if (D == 16) L3B(16); else if (D == 32) L3B(32); else if (D == 64) L3B(64); else L3B(128);
#undef L3B
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  const size_t per_wave = (size_t)(F * (D + 1) + 32 * 33) * sizeof(float);
  const int wpb = waves_for(per_wave);
  if (F <= 32 && wpb > 0) {
    hipLaunchKernelGGL(interact_dot_bwd_mfma, dim3(grid_for(B, wpb)), dim3(64 * wpb),
                       per_wave * wpb, st, B, F, D, fa,
                       self_interaction ? 1 : 0, grad_out, ld_gout, ga);
  } else {
    const int64_t n = (int64_t)B * F * D;
    hipLaunchKernelGGL(interact_dot_bwd_generic, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0, st,
                       B, F, D, fa, self_interaction ? 1 : 0, grad_out, ld_gout, ga);
  }
  DLRM_LAUNCH_CHECK(name);
  if (relu_x) {
    hipLaunchKernelGGL(relu_mask_kernel, dim3(dlrm::ceil_div((int64_t)B * D, 256)), dim3(256), 0,
                       st, B, D, fa.ptr[0], fa.bs[0], ga.ptr[0], ga.bs[0]);
    DLRM_LAUNCH_CHECK(name);
  }
  return DLRM_OK;
}

extern "C" int dlrm_interact_cat_forward(int32_t B, int32_t F, int32_t D,
                                         const float* const* feat_ptrs,
                                         const int64_t* feat_bstrides, float* out,
                                         int64_t ld_out, dlrm_stream_t stream) {
  const char* name = "dlrm_interact_cat_forward";
  DLRM_ARG(B >= 0 && F >= 1 && F <= kMaxF && D > 0, "%s: need F in [1,64], D > 0", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(out && ld_out >= (int64_t)F * D, "%s: bad out", name);
  FeatArgs fa{};
  int rc = fill_feat(fa, F, feat_ptrs, feat_bstrides, name);
  if (rc) return rc;
  const int64_t n = (int64_t)B * F * D;
  hipLaunchKernelGGL(interact_cat_fwd, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), B, F, D, fa, out, ld_out);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

extern "C" int dlrm_interact_cat_backward(int32_t B, int32_t F, int32_t D,
                                          const float* grad_out, int64_t ld_gout,
                                          float* const* grad_ptrs, const int64_t* grad_bstrides,
                                          dlrm_stream_t stream) {
  const char* name = "dlrm_interact_cat_backward";
  DLRM_ARG(B >= 0 && F >= 1 && F <= kMaxF && D > 0, "%s: need F in [1,64], D > 0", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(grad_out && ld_gout >= (int64_t)F * D, "%s: bad grad_out", name);
  GradArgs ga{};
  int rc = fill_grad(ga, F, grad_ptrs, grad_bstrides, name);
  if (rc) return rc;
  const int64_t n = (int64_t)B * F * D;
  hipLaunchKernelGGL(interact_cat_bwd, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), B, F, D, grad_out, ld_gout, ga);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

// One-hot lookup fused into the interaction (one GPU, L = 1): features 1..F-1 are gathered
// straight from the table buffer (no [B, T, D] pooled-embedding round trip through HBM).
// Same math and output as dlrm_interact_dot_forward on the looked-up rows.
extern "C" int dlrm_interact_dot_forward_gather(int32_t B, int32_t F, int32_t D, const float* x,
                                                int64_t x_bstride, const float* weights,
                                                const int64_t* row_base, const int32_t* indices,
                                                int32_t self_interaction, float* out,
                                                int64_t ld_out, int32_t* error_flag,
                                                dlrm_stream_t stream) {
  const char* name = "dlrm_interact_dot_forward_gather";
  DLRM_ARG(B >= 0 && F >= 2 && F <= 32, "%s: need F in [2,32]", name);
  DLRM_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128, DLRM_ERR_UNSUPPORTED,
               "%s: D must be 16, 32, 64 or 128", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(x && weights && row_base && indices && out, "%s: null pointer", name);
  DLRM_ARG(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weights)) & 15) == 0 &&
               x_bstride % 4 == 0,
           "%s: x / weights must be 16-B aligned, x_bstride %% 4 == 0", name);
  const int npairs = self_interaction ? F * (F + 1) / 2 : F * (F - 1) / 2;
  DLRM_ARG(ld_out >= D + npairs, "%s: ld_out < D + pairs", name);
  FeatArgs fa{};
  for (int f = 0; f < F; ++f) fa.ptr[f] = x, fa.bs[f] = x_bstride;
  const GatherArgs gt{weights, row_base, indices, error_flag};
  const int width = D + npairs;
  hipStream_t st = dlrm::as_stream(stream);
  if (fwd_version(D, B) == 5) {
    if (D == 64)
      hipLaunchKernelGGL((interact_dot_fwd_v5<64, true>), dim3(v5_grid(B)), dim3(128), 0, st, B, F,
                         fa, self_interaction ? 1 : 0, out, ld_out, width, gt);
    else
      hipLaunchKernelGGL((interact_dot_fwd_v5<128, true>), dim3(v5_grid(B)), dim3(256), 0, st, B,
                         F, fa, self_interaction ? 1 : 0, out, ld_out, width, gt);
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  const int vec_out = ((reinterpret_cast<uintptr_t>(out) & 15) == 0 && ld_out % 4 == 0) ? 1 : 0;
  const size_t lds = 4 * (32 * (size_t)(D + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
  const int grid = (int)std::min<int64_t>(dlrm::ceil_div(B, 4), 8192);
#define L4G(DD)                                                                              \
  hipLaunchKernelGGL((interact_dot_fwd_v4<DD, true>), dim3(grid), dim3(256), lds, st, B, F, fa, \
                     self_interaction ? 1 : 0, out, ld_out, width, vec_out, gt)
  if (D == 16) L4G(16); else if (D == 32) L4G(32); else if (D == 64) L4G(64); else L4G(128);
#undef L4G
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

// Its backward: T re-gathered from the same (not yet updated) rows; gradients as
// dlrm_interact_dot_backward (grad_ptrs[f] / grad_bstrides[f], e.g. the [B, T, D] buffer
// the TBE backward reads), ReLU' of x optional.
extern "C" int dlrm_interact_dot_backward_gather(
    int32_t B, int32_t F, int32_t D, const float* x, int64_t x_bstride, const float* weights,
    const int64_t* row_base, const int32_t* indices, int32_t self_interaction,
    const float* grad_out, int64_t ld_gout, float* const* grad_ptrs,
    const int64_t* grad_bstrides, int32_t relu_x, dlrm_stream_t stream) {
  const char* name = "dlrm_interact_dot_backward_gather";
  DLRM_ARG(B >= 0 && F >= 2 && F <= 32, "%s: need F in [2,32]", name);
  DLRM_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128, DLRM_ERR_UNSUPPORTED,
               "%s: D must be 16, 32, 64 or 128", name);
  if (B == 0) return DLRM_OK;
  DLRM_ARG(x && weights && row_base && indices && grad_out, "%s: null pointer", name);
  DLRM_ARG(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weights)) & 15) == 0 &&
               x_bstride % 4 == 0,
           "%s: x / weights must be 16-B aligned, x_bstride %% 4 == 0", name);
  const int npairs = self_interaction ? F * (F + 1) / 2 : F * (F - 1) / 2;
  DLRM_ARG(ld_gout >= D + npairs, "%s: ld_gout < D + pairs", name);
  GradArgs ga{};
  int rc = fill_grad(ga, F, grad_ptrs, grad_bstrides, name);
  if (rc) return rc;
  for (int f = 0; f < F; ++f)
    DLRM_ARG(((reinterpret_cast<uintptr_t>(ga.ptr[f]) & 15) == 0) && (ga.bs[f] & 3) == 0,
             "%s: gradient rows must be 16-B aligned", name);
  FeatArgs fa{};
  for (int f = 0; f < F; ++f) fa.ptr[f] = x, fa.bs[f] = x_bstride;
  const GatherArgs gt{weights, row_base, indices, nullptr};
  const int vec_g = ((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0 && ld_gout % 4 == 0) ? 1 : 0;
  hipStream_t st = dlrm::as_stream(stream);
  const int ver = bwd_version(D, B);
  if (ver == 5) {
    if (D == 64)
      hipLaunchKernelGGL((interact_dot_bwd_v5<64, true>), dim3(v5_grid(B)), dim3(128), 0, st, B, F,
                         fa, self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g,
                         gt);
    else
      hipLaunchKernelGGL((interact_dot_bwd_v5<128, true>), dim3(v5_grid(B)), dim3(256), 0, st, B, F,
                         fa, self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g,
                         gt);
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  if (ver == 4) {
    const int nblk = D > 32 ? D / 32 : 1, cb = D < 32 ? D : 32;
    const size_t lds4 = 4 * (32 * (size_t)(cb + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
    const int grid4 = (int)std::min<int64_t>(dlrm::ceil_div((int64_t)B * nblk, 4), 8192);
#define L4G(DD)                                                                               \
  hipLaunchKernelGGL((interact_dot_bwd_v4<DD, true>), dim3(grid4), dim3(256), lds4, st, B, F, fa, \
                     self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g, gt)
    if (D == 16) L4G(16); else if (D == 32) L4G(32); else if (D == 64) L4G(64); else L4G(128);
#undef L4G
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
  const size_t lds = 4 * (32 * (size_t)(D + 4) + D + 32 * 33 / 2 + 4) * sizeof(float);
  const int grid = (int)std::min<int64_t>(dlrm::ceil_div(B, 4), 8192);
#define L3G(DD)                                                                               \
  hipLaunchKernelGGL((interact_dot_bwd_v3<DD, true>), dim3(grid), dim3(256), lds, st, B, F, fa,  \
                     self_interaction ? 1 : 0, grad_out, ld_gout, ga, relu_x ? 1 : 0, vec_g, gt)
  if (D == 16) L3G(16); else if (D == 32) L3G(32); else if (D == 64) L3G(64); else L3G(128);
#undef L3G
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}
