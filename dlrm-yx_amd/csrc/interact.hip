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
                                          dlrm_stream_t stream) {
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
