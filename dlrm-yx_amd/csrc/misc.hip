// Small fused kernels of the DLRM step: bias-gradient column sums, the last layer +
// sigmoid + loss head, ReLU-masked outer product, dense optimizers, device RNG fills.
//
//  * dlrm_colsum_f32: Linear bias gradient (sum of dY over the batch), deterministic
//    two-pass (fixed 64-row chunks, then chunk partials in order), optional fused SGD.
//  * dlrm_head_forward_backward: top-MLP last layer (K -> 1) + nn.Sigmoid + loss_fn
//    (MSELoss / BCELoss mean, dlrm_s_pytorch.py:504-516, 170-178) and d loss / d logit
//    in one wave-per-row pass; the batch mean is a fixed-order block reduction.
//  * dlrm_sgd_update / dlrm_adagrad_update: torch.optim.SGD dense step and the dense
//    branch of RWSAdagrad (optim/rwsadagrad.py:117-120) on a flat parameter bucket.
#include "common.hpp"
#include "head_roles.hpp"
#include "tbe_bwd_roles.hpp"

namespace {

constexpr int kRowsPerChunk = 64;

__global__ __launch_bounds__(256) void colsum_partial_kernel(int64_t M, int64_t N,
                                                             const float* __restrict__ Y,
                                                             int64_t ldy,
                                                             const float* __restrict__ scale,
                                                             float* __restrict__ part) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t ms = blockIdx.y;
  if (n >= N) return;
  const int64_t m0 = ms * kRowsPerChunk;
  const int64_t m1 = (m0 + kRowsPerChunk < M) ? m0 + kRowsPerChunk : M;
  float s = 0.f;
  if (scale) {
    for (int64_t m = m0; m < m1; ++m) s = fmaf(scale[m], Y[m * ldy + n], s);
  } else {
    for (int64_t m = m0; m < m1; ++m) s += Y[m * ldy + n];
  }
  part[ms * N + n] = s;
}

__global__ __launch_bounds__(256) void colsum_final_kernel(int64_t N, int64_t MS,
                                                           const float* __restrict__ part,
                                                           float alpha, float* __restrict__ out,
                                                           int accumulate,
                                                           float* __restrict__ sgd_param,
                                                           float lr) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t ms = 0; ms < MS; ++ms) s += part[ms * N + n];
  if (out) out[n] = accumulate ? out[n] + alpha * s : alpha * s;
  if (sgd_param) sgd_param[n] = fmaf(-lr, s, sgd_param[n]);
}

__global__ __launch_bounds__(256) void head_rows_kernel(int64_t M, int64_t K,
                                                        const float* __restrict__ X, int64_t ldx,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bptr,
                                                        const float* __restrict__ target,
                                                        int loss_kind, float lo, float gscale,
                                                        float* __restrict__ prob,
                                                        float* __restrict__ dz,
                                                        float* __restrict__ row_loss) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const float bias = bptr ? bptr[0] : 0.f;
  const float invM = 1.f / (float)M;
  for (int64_t m = wave; m < M; m += nw) {
    const float* xr = X + m * ldx;
    float s = 0.f;
    for (int64_t k = lane; k < K; k += 64) s = fmaf(xr[k], w[k], s);
    s = wave_sum(s);
    if (lane == 0) {
      const float z = s + bias;
      const float p = 1.f / (1.f + expf(-z));
      float pc = p;
      bool pass = true;
      if (lo > 0.f && lo < 0.5f) {
        const float hi = 1.f - lo;
        pass = (p >= lo) && (p <= hi);
        pc = fminf(fmaxf(p, lo), hi);
      }
      const float t = target ? target[m] : 0.f;
      float l, dp;
      if (loss_kind == DLRM_LOSS_BCE) {
        const float lp = fmaxf(logf(pc), -100.f);
        const float l1p = fmaxf(logf(1.f - pc), -100.f);
        l = -(t * lp + (1.f - t) * l1p);
        dp = (pc - t) / fmaxf((1.f - pc) * pc, 1e-12f) * invM;
      } else {
        const float d = pc - t;
        l = d * d;
        dp = 2.f * d * invM;
      }
      dp *= gscale;
      if (!pass) dp = 0.f;
      if (prob) prob[m] = pc;
      if (dz) dz[m] = dp * (1.f - p) * p;
      row_loss[m] = l;
    }
  }
}

// ---------------------------------------------------------------- fused head --
// Per-row loss math shared by the head kernels: returns (prob, dz, row loss).
__device__ __forceinline__ void head_row_math(float z, float t, int loss_kind, float lo,
                                              float gscale, float invM, float& pc, float& dzv,
                                              float& l) {
  const float p = 1.f / (1.f + expf(-z));
  pc = p;
  bool pass = true;
  if (lo > 0.f && lo < 0.5f) {
    const float hi = 1.f - lo;
    pass = (p >= lo) && (p <= hi);
    pc = fminf(fmaxf(p, lo), hi);
  }
  float dp;
  if (loss_kind == DLRM_LOSS_BCE) {
    const float lp = fmaxf(logf(pc), -100.f);
    const float l1p = fmaxf(logf(1.f - pc), -100.f);
    l = -(t * lp + (1.f - t) * l1p);
    dp = (pc - t) / fmaxf((1.f - pc) * pc, 1e-12f) * invM;
  } else {
    const float d = pc - t;
    l = d * d;
    dp = 2.f * d * invM;
  }
  dp *= gscale;
  if (!pass) dp = 0.f;
  dzv = dp * (1.f - p) * p;
}

constexpr int kHeadRows = 4;  // rows per workgroup (one per wave)
constexpr int kHeadMaxK = 2048;

// One pass over the rows of the last layer's input X [M, K] (K includes the folded bias
// column): z = X w, sigmoid, loss term, dz, the ReLU-masked input gradient
// dX = dz w^T (.) (X > 0), and this workgroup's column partial sum of dz X (the weight
// gradient) in fixed row order.
template <int NC>
__global__ __launch_bounds__(256) void head_fused_rows_kernel(
    int64_t M, int64_t K, const float* __restrict__ X, int64_t ldx, const float* __restrict__ w,
    const float* __restrict__ target, int loss_kind, float lo, float gscale,
    float* __restrict__ prob, float* __restrict__ dz, float* __restrict__ row_loss,
    float* __restrict__ dX, int64_t lddx, int mask, float* __restrict__ part) {
  __shared__ float red[4][NC * 64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const float invM = 1.f / (float)M;
  float wr[NC], cp[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int64_t k = lane + 64 * c;
    wr[c] = k < K ? w[k] : 0.f;
    cp[c] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * kHeadRows + wave * (kHeadRows / 4);
  for (int q = 0; q < kHeadRows / 4; ++q) {
    const int64_t m = r0 + q;
    if (m >= M) break;
    const float* xr = X + m * ldx;
    float xv[NC];
    float sacc = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int64_t k = lane + 64 * c;
      xv[c] = k < K ? xr[k] : 0.f;
      sacc = fmaf(xv[c], wr[c], sacc);
    }
    sacc = wave_sum(sacc);
    float pc = 0.f, dzv = 0.f, l = 0.f;
    if (lane == 0) {
      head_row_math(sacc, target ? target[m] : 0.f, loss_kind, lo, gscale, invM, pc, dzv, l);
      if (prob) prob[m] = pc;
      if (dz) dz[m] = dzv;
      row_loss[m] = l;
    }
    dzv = __shfl(dzv, 0, 64);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int64_t k = lane + 64 * c;
      if (k < K) {
        float g = dzv * wr[c];
        if (mask && !(xv[c] > 0.f)) g = 0.f;
        if (dX) dX[m * lddx + k] = g;
      }
      cp[c] = fmaf(dzv, xv[c], cp[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[wave][lane + 64 * c] = cp[c];
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256)
    part[(int64_t)blockIdx.x * K + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
}

// Column sums of the row-block partials -> weight gradient (stored, accumulated, or
// applied as SGD to w) and the mean loss: head_roles.hpp.
__global__ __launch_bounds__(256) void head_finalize_kernel(int64_t M, int64_t K, int64_t nblk,
                                                            const float* __restrict__ part,
                                                            float* __restrict__ w, float lr,
                                                            float* __restrict__ dw, int accumulate,
                                                            const float* __restrict__ row_loss,
                                                            float* __restrict__ loss_out) {
  __shared__ float red[4];
  head_finalize_body(M, K, nblk, part, w, lr, dw, accumulate, row_loss, loss_out, blockIdx.x,
                     gridDim.x, red);
}

__global__ __launch_bounds__(256) void mean_kernel(int64_t M, const float* __restrict__ v,
                                                   float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < M; i += 256) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] / (float)M;
}

__global__ __launch_bounds__(256) void outer_drelu_kernel(int64_t M, int64_t K,
                                                          const float* __restrict__ dz,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ X,
                                                          int64_t ldx, int mask,
                                                          float* __restrict__ dX, int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * K) return;
  const int64_t m = i / K, k = i - m * K;
  float v = dz[m] * w[k];
  if (mask && !(X[m * ldx + k] > 0.f)) v = 0.f;
  dX[m * lddx + k] = v;
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p,
                                                  const float* __restrict__ g, int64_t n,
                                                  float lr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < n; j += stride) p[j] = fmaf(-lr, g[j], p[j]);
}

__global__ __launch_bounds__(256) void adagrad_kernel(float* __restrict__ p,
                                                      const float* __restrict__ g,
                                                      float* __restrict__ ss, int64_t n,
                                                      float clr, float eps, float gs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < n; j += stride) {
    const float gj = g[j] * gs;  // (gs = 1: exact; else the rounding dlrm_scale_f32 gives)
    const float s = fmaf(gj, gj, ss[j]);
    ss[j] = s;
    p[j] = fmaf(-clr, gj / (sqrtf(s) + eps), p[j]);
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, int64_t n, float a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < n; j += stride) x[j] *= a;
}

__global__ __launch_bounds__(256) void sigmoid_fwd_kernel(int64_t n, const float* __restrict__ x,
                                                          float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < n; j += stride) y[j] = 1.f / (1.f + expf(-x[j]));
}

__global__ __launch_bounds__(256) void sigmoid_bwd_kernel(int64_t n, const float* __restrict__ dy,
                                                          const float* __restrict__ y,
                                                          float* __restrict__ dx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < n; j += stride) dx[j] = dy[j] * (1.f - y[j]) * y[j];
}

__global__ __launch_bounds__(256) void relu_bwd_kernel(int64_t M, int64_t K,
                                                       const float* __restrict__ dy, int64_t lddy,
                                                       const float* __restrict__ y, int64_t ldy,
                                                       float* __restrict__ dx, int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = i; j < M * K; j += stride) {
    const int64_t m = j / K, k = j - m * K;
    dx[m * lddx + k] = y[m * ldy + k] > 0.f ? dy[m * lddy + k] : 0.f;
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void uniform_fill_kernel(float* __restrict__ out, int64_t n,
                                                           float lo, float hi, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint64_t key = splitmix64(seed);
  for (int64_t j = i; j < n; j += stride) {
    const uint64_t x = splitmix64(key ^ (uint64_t)j);
    const float u = (float)(x >> 40) * (1.f / 16777216.f);
    out[j] = lo + (hi - lo) * u;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void uniform_int_kernel(T* __restrict__ out, int64_t n,
                                                          uint64_t hi, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint64_t key = splitmix64(seed);
  for (int64_t j = i; j < n; j += stride) {
    const uint64_t x = splitmix64(key ^ (uint64_t)j);
    out[j] = (T)__umul64hi(x, hi);
  }
}

int grid_stride_blocks(int64_t n) {
  int64_t b = dlrm::ceil_div(n, 256);
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" size_t dlrm_colsum_workspace_size(int64_t M, int64_t N) {
  const int64_t ms = dlrm::ceil_div(M > 0 ? M : 1, kRowsPerChunk);
  return (size_t)(ms * (N > 0 ? N : 1)) * sizeof(float) + 256;
}

extern "C" int dlrm_colsum_f32(int64_t M, int64_t N, const float* Y, int64_t ldy,
                               const float* scale, float alpha, float* out, int32_t accumulate,
                               float* sgd_param, float lr, void* workspace,
                               size_t workspace_bytes, dlrm_stream_t stream) {
  const char* name = "dlrm_colsum_f32";
  DLRM_ARG(M >= 0 && N >= 0, "%s: negative size", name);
  if (N == 0) return DLRM_OK;
  DLRM_ARG(M == 0 || (Y && ldy >= N), "%s: bad Y", name);
  DLRM_ARG(workspace, "%s: null workspace", name);
  DLRM_REQUIRE(workspace_bytes >= dlrm_colsum_workspace_size(M, N), DLRM_ERR_WORKSPACE,
               "%s: workspace too small", name);
  hipStream_t st = dlrm::as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const int64_t ms = M > 0 ? dlrm::ceil_div(M, kRowsPerChunk) : 0;
  if (ms > 0) {
    DLRM_REQUIRE(ms < 65536, DLRM_ERR_UNSUPPORTED, "%s: M too large", name);
    hipLaunchKernelGGL(colsum_partial_kernel, dim3(dlrm::ceil_div(N, 256), ms), dim3(256), 0, st,
                       M, N, Y, ldy, scale, part);
    DLRM_LAUNCH_CHECK(name);
  }
  hipLaunchKernelGGL(colsum_final_kernel, dim3(dlrm::ceil_div(N, 256)), dim3(256), 0, st, N, ms,
                     part, alpha, out, accumulate, sgd_param, lr);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

extern "C" size_t dlrm_head_workspace_size(int64_t M) {
  return (size_t)(M > 0 ? M : 1) * sizeof(float) + 256;
}

extern "C" int dlrm_head_forward_backward(int64_t M, int64_t K, const float* X, int64_t ldx,
                                          const float* w, const float* b, const float* target,
                                          int32_t loss_kind, float clamp_lo, float grad_scale,
                                          float* prob_out, float* dz_out, float* loss_out,
                                          void* workspace, size_t workspace_bytes,
                                          dlrm_stream_t stream) {
  const char* name = "dlrm_head_forward_backward";
  DLRM_ARG(M > 0 && K > 0, "%s: bad sizes", name);
  DLRM_ARG(X && w && ldx >= K, "%s: bad X/w", name);
  DLRM_ARG(loss_kind == DLRM_LOSS_MSE || loss_kind == DLRM_LOSS_BCE, "%s: bad loss", name);
  DLRM_ARG(workspace, "%s: null workspace", name);
  DLRM_REQUIRE(workspace_bytes >= dlrm_head_workspace_size(M), DLRM_ERR_WORKSPACE,
               "%s: workspace too small", name);
  DLRM_ARG(target || (!dz_out && !loss_out), "%s: loss/grad need target", name);
  hipStream_t st = dlrm::as_stream(stream);
  float* row_loss = static_cast<float*>(workspace);
  int64_t blocks = dlrm::ceil_div(M, 4);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(head_rows_kernel, dim3(blocks), dim3(256), 0, st, M, K, X, ldx, w, b,
                     target, loss_kind, clamp_lo, grad_scale, prob_out, dz_out, row_loss);
  DLRM_LAUNCH_CHECK(name);
  if (loss_out) {
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, st, M, row_loss, loss_out);
    DLRM_LAUNCH_CHECK(name);
  }
  return DLRM_OK;
}

extern "C" int dlrm_outer_drelu(int64_t M, int64_t K, const float* dz, const float* w,
                                const float* X, int64_t ldx, int32_t relu_mask, float* dX,
                                int64_t lddx, dlrm_stream_t stream) {
  const char* name = "dlrm_outer_drelu";
  DLRM_ARG(M >= 0 && K >= 0, "%s: bad sizes", name);
  if (M == 0 || K == 0) return DLRM_OK;
  DLRM_ARG(dz && w && dX && lddx >= K, "%s: null pointer", name);
  DLRM_ARG(!relu_mask || (X && ldx >= K), "%s: mask needs X", name);
  hipLaunchKernelGGL(outer_drelu_kernel, dim3(dlrm::ceil_div(M * K, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), M, K, dz, w, X, ldx, relu_mask, dX, lddx);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

extern "C" int dlrm_sgd_update(float* param, const float* grad, int64_t n, float lr,
                               dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_sgd_update: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(param && grad, "dlrm_sgd_update: null pointer");
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), param, grad, n, lr);
  DLRM_LAUNCH_CHECK("dlrm_sgd_update");
  return DLRM_OK;
}

extern "C" int dlrm_adagrad_update(float* param, const float* grad, float* state_sum, int64_t n,
                                   float clr, float eps, dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_adagrad_update: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(param && grad && state_sum, "dlrm_adagrad_update: null pointer");
  hipLaunchKernelGGL(adagrad_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), param, grad, state_sum, n, clr, eps, 1.0f);
  DLRM_LAUNCH_CHECK("dlrm_adagrad_update");
  return DLRM_OK;
}

extern "C" int dlrm_adagrad_update_scaled(float* param, const float* grad, float* state_sum,
                                          int64_t n, float grad_scale, float clr, float eps,
                                          dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_adagrad_update_scaled: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(param && grad && state_sum, "dlrm_adagrad_update_scaled: null pointer");
  hipLaunchKernelGGL(adagrad_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), param, grad, state_sum, n, clr, eps, grad_scale);
  DLRM_LAUNCH_CHECK("dlrm_adagrad_update_scaled");
  return DLRM_OK;
}

extern "C" int dlrm_scale_f32(float* x, int64_t n, float alpha, dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_scale_f32: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(x, "dlrm_scale_f32: null pointer");
  hipLaunchKernelGGL(scale_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), x, n, alpha);
  DLRM_LAUNCH_CHECK("dlrm_scale_f32");
  return DLRM_OK;
}

extern "C" int dlrm_uniform_fill(float* out, int64_t n, float lo, float hi, uint64_t seed,
                                 dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_uniform_fill: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(out, "dlrm_uniform_fill: null pointer");
  hipLaunchKernelGGL(uniform_fill_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), out, n, lo, hi, seed);
  DLRM_LAUNCH_CHECK("dlrm_uniform_fill");
  return DLRM_OK;
}

extern "C" int dlrm_uniform_int_fill(void* out, int32_t out_bits, int64_t n, int64_t hi,
                                     uint64_t seed, dlrm_stream_t stream) {
  DLRM_ARG(n >= 0 && hi > 0, "dlrm_uniform_int_fill: bad n/hi");
  DLRM_ARG(out_bits == 32 || out_bits == 64, "dlrm_uniform_int_fill: bad out_bits");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(out, "dlrm_uniform_int_fill: null pointer");
  hipStream_t st = dlrm::as_stream(stream);
  if (out_bits == 32)
    hipLaunchKernelGGL(uniform_int_kernel<int32_t>, dim3(grid_stride_blocks(n)), dim3(256), 0, st,
                       static_cast<int32_t*>(out), n, (uint64_t)hi, seed);
  else
    hipLaunchKernelGGL(uniform_int_kernel<int64_t>, dim3(grid_stride_blocks(n)), dim3(256), 0, st,
                       static_cast<int64_t*>(out), n, (uint64_t)hi, seed);
  DLRM_LAUNCH_CHECK("dlrm_uniform_int_fill");
  return DLRM_OK;
}

extern "C" int dlrm_sigmoid_forward(int64_t n, const float* x, float* y, dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_sigmoid_forward: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(x && y, "dlrm_sigmoid_forward: null pointer");
  hipLaunchKernelGGL(sigmoid_fwd_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), n, x, y);
  DLRM_LAUNCH_CHECK("dlrm_sigmoid_forward");
  return DLRM_OK;
}

extern "C" int dlrm_sigmoid_backward(int64_t n, const float* dy, const float* y, float* dx,
                                     dlrm_stream_t stream) {
  DLRM_ARG(n >= 0, "dlrm_sigmoid_backward: bad n");
  if (n == 0) return DLRM_OK;
  DLRM_ARG(dy && y && dx, "dlrm_sigmoid_backward: null pointer");
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(grid_stride_blocks(n)), dim3(256), 0,
                     dlrm::as_stream(stream), n, dy, y, dx);
  DLRM_LAUNCH_CHECK("dlrm_sigmoid_backward");
  return DLRM_OK;
}

extern "C" int dlrm_relu_backward(int64_t M, int64_t K, const float* dy, int64_t lddy,
                                  const float* y, int64_t ldy, float* dx, int64_t lddx,
                                  dlrm_stream_t stream) {
  DLRM_ARG(M >= 0 && K >= 0, "dlrm_relu_backward: bad sizes");
  if (M == 0 || K == 0) return DLRM_OK;
  DLRM_ARG(dy && y && dx, "dlrm_relu_backward: null pointer");
  DLRM_ARG(lddy >= K && ldy >= K && lddx >= K, "dlrm_relu_backward: bad leading dims");
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_stride_blocks(M * K)), dim3(256), 0,
                     dlrm::as_stream(stream), M, K, dy, lddy, y, ldy, dx, lddx);
  DLRM_LAUNCH_CHECK("dlrm_relu_backward");
  return DLRM_OK;
}

extern "C" size_t dlrm_head_step_workspace_size(int64_t M, int64_t K) {
  const int64_t nblk = dlrm::ceil_div(M > 0 ? M : 1, kHeadRows);
  return (size_t)(M > 0 ? M : 1) * sizeof(float) + 256 +
         (size_t)nblk * (K > 0 ? K : 1) * sizeof(float) + 256;
}

namespace {

int head_step(int64_t M, int64_t K, const float* X, int64_t ldx, float* w, const float* target,
              int32_t loss_kind, float clamp_lo, float grad_scale, float* prob_out,
              float* dz_out, float* loss_out, float* dX, int64_t lddx, int32_t relu_mask,
              float* dw_out, int32_t accumulate, float lr, void* workspace,
              size_t workspace_bytes, LaunchRole* defer, dlrm_stream_t stream, const char* name) {
  DLRM_ARG(M > 0 && K > 0, "%s: bad sizes", name);
  DLRM_ARG(X && w && ldx >= K && target, "%s: null X/w/target", name);
  DLRM_ARG(loss_kind == DLRM_LOSS_MSE || loss_kind == DLRM_LOSS_BCE, "%s: bad loss", name);
  DLRM_ARG(!dX || lddx >= K, "%s: bad lddx", name);
  DLRM_REQUIRE(K <= kHeadMaxK, DLRM_ERR_UNSUPPORTED, "%s: K > %d", name, kHeadMaxK);
  DLRM_ARG(workspace, "%s: null workspace", name);
  DLRM_REQUIRE(workspace_bytes >= dlrm_head_step_workspace_size(M, K), DLRM_ERR_WORKSPACE,
               "%s: workspace too small", name);
  WsCarver wc(workspace);
  float* row_loss = wc.take<float>(M);
  const int64_t nblk = dlrm::ceil_div(M, kHeadRows);
  float* part = wc.take<float>(nblk * K);
  hipStream_t st = dlrm::as_stream(stream);
  const int nc = (int)dlrm::ceil_div(K, 64);
#define HR(NC_)                                                                               \
  hipLaunchKernelGGL(head_fused_rows_kernel<NC_>, dim3(nblk), dim3(256), 0, st, M, K, X, ldx, w, \
                     target, loss_kind, clamp_lo, grad_scale, prob_out, dz_out, row_loss, dX,  \
                     lddx, relu_mask, part)
  if (nc <= 2) HR(2); else if (nc <= 4) HR(4); else if (nc <= 5) HR(5); else if (nc <= 8) HR(8);
  else if (nc <= 12) HR(12); else if (nc <= 17) HR(17); else if (nc <= 24) HR(24); else HR(32);
#undef HR
  DLRM_LAUNCH_CHECK(name);
  if (defer) {  // the finalize pass rides on a later launch (dlrm_gemm_f32_group_role)
    defer->head.M = M, defer->head.K = K, defer->head.nblk = nblk, defer->head.part = part;
    defer->head.w = w, defer->head.dw = dw_out, defer->head.row_loss = row_loss;
    defer->head.loss_out = loss_out, defer->head.lr = lr, defer->head.accumulate = accumulate;
    defer->blocks = (int32_t)(dlrm::ceil_div(dlrm::ceil_div(K, (int64_t)4), (int64_t)8) * 8);
    defer->kind = kRoleHead;
    return DLRM_OK;
  }
  hipLaunchKernelGGL(head_finalize_kernel, dim3(dlrm::ceil_div(K, 4)), dim3(256), 0, st, M, K,
                     nblk, part, w, lr, dw_out, accumulate, row_loss, loss_out);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

}  // namespace

extern "C" int dlrm_head_step(int64_t M, int64_t K, const float* X, int64_t ldx, float* w,
                              const float* target, int32_t loss_kind, float clamp_lo,
                              float grad_scale, float* prob_out, float* dz_out, float* loss_out,
                              float* dX, int64_t lddx, int32_t relu_mask, float* dw_out,
                              int32_t accumulate, float lr, void* workspace,
                              size_t workspace_bytes, dlrm_stream_t stream) {
  return head_step(M, K, X, ldx, w, target, loss_kind, clamp_lo, grad_scale, prob_out, dz_out,
                   loss_out, dX, lddx, relu_mask, dw_out, accumulate, lr, workspace,
                   workspace_bytes, nullptr, stream, "dlrm_head_step");
}

extern "C" int dlrm_head_step_defer(int64_t M, int64_t K, const float* X, int64_t ldx, float* w,
                                    const float* target, int32_t loss_kind, float clamp_lo,
                                    float grad_scale, float* prob_out, float* dz_out,
                                    float* loss_out, float* dX, int64_t lddx, int32_t relu_mask,
                                    float* dw_out, int32_t accumulate, float lr, void* workspace,
                                    size_t workspace_bytes, dlrm_launch_role* role,
                                    dlrm_stream_t stream) {
  const char* name = "dlrm_head_step_defer";
  DLRM_ARG(role, "%s: null role", name);
  auto* r = reinterpret_cast<LaunchRole*>(role);
  *r = LaunchRole{};
  r->magic = kRoleMagic;
  return head_step(M, K, X, ldx, w, target, loss_kind, clamp_lo, grad_scale, prob_out, dz_out,
                   loss_out, dX, lddx, relu_mask, dw_out, accumulate, lr, workspace,
                   workspace_bytes, r, stream, name);
}

// ---------------------------------------------------------------------------------------
// Criteo binary record decode (the CriteoBinDataset.__getitem__ + _transform_features
// path, data_loader_terabyte.py:83-114, 237-252).  A record is int32
// [label | n_dense | n_sparse]; one thread per int32 field in FLAT order, so the raw
// block is read fully coalesced and each field is written where the step reads it:
//   label            -> label[b] = (float)v
//   dense field j    -> dense[b * ld_dense + j] = log((float)v + 1)
//   sparse field t   -> indices[t * n + b] = v mod max_ind_range (floor mod, torch `%`),
//                       table-major as lS_i = x_cat.t() / cat(lS_i) (:93-98)
// and, for the table-batched form, offsets[i] = i for i <= n_sparse * n (L = 1, :99-100).
// Integer work is bit-exact; the log is fp32.
namespace {

template <typename IT>
__global__ __launch_bounds__(256) void criteo_decode_kernel(
    const int32_t* __restrict__ rec, int64_t n, int32_t n_dense, int32_t n_sparse,
    int64_t max_ind_range, float* __restrict__ dense, int64_t ld_dense,
    float* __restrict__ label, IT* __restrict__ indices) {
  const int32_t nf = 1 + n_dense + n_sparse;
  const int64_t total = n * nf;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / nf;
    const int32_t f = (int32_t)(i - b * nf);
    const int32_t v = __builtin_nontemporal_load(rec + i);
    if (f == 0) {
      if (label) label[b] = (float)v;
    } else if (f <= n_dense) {
      if (dense) dense[b * ld_dense + (f - 1)] = logf((float)v + 1.f);
    } else {
      int64_t x = v;
      if (max_ind_range > 0) {
        x %= max_ind_range;
        if (x < 0) x += max_ind_range;
      }
      indices[(int64_t)(f - 1 - n_dense) * n + b] = (IT)x;
    }
  }
}

template <typename OT>
__global__ __launch_bounds__(256) void iota_kernel(OT* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (OT)i;
}

}  // namespace

extern "C" int dlrm_criteo_decode(const int32_t* records, int64_t n, int32_t n_dense,
                                  int32_t n_sparse, int64_t max_ind_range, float* dense,
                                  int64_t ld_dense, float* label, void* indices,
                                  int32_t index_bits, void* offsets, int32_t offset_bits,
                                  dlrm_stream_t stream) {
  const char* name = "dlrm_criteo_decode";
  DLRM_ARG(n >= 0 && n_dense >= 0 && n_sparse >= 0, "%s: bad sizes", name);
  DLRM_ARG(ld_dense >= n_dense, "%s: ld_dense < n_dense", name);
  DLRM_ARG(index_bits == 32 || index_bits == 64, "%s: bad index_bits", name);
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "%s: bad offset_bits", name);
  DLRM_ARG(n == 0 || (records && (indices || n_sparse == 0)), "%s: null pointer", name);
  DLRM_REQUIRE(index_bits == 64 || max_ind_range <= (int64_t)INT32_MAX + 1, DLRM_ERR_UNSUPPORTED,
               "%s: int32 indices with max_ind_range > 2^31", name);
  hipStream_t st = dlrm::as_stream(stream);
  const int64_t total = n * (1 + n_dense + n_sparse);
  if (total == 0) {
    // nothing to decode; the CSR below still gets its single offsets[0] = 0
  } else if (index_bits == 32)
    hipLaunchKernelGGL(criteo_decode_kernel<int32_t>, dim3(grid_stride_blocks(total)), dim3(256),
                       0, st, records, n, n_dense, n_sparse, max_ind_range, dense, ld_dense, label,
                       static_cast<int32_t*>(indices));
  else
    hipLaunchKernelGGL(criteo_decode_kernel<int64_t>, dim3(grid_stride_blocks(total)), dim3(256),
                       0, st, records, n, n_dense, n_sparse, max_ind_range, dense, ld_dense, label,
                       static_cast<int64_t*>(indices));
  if (offsets) {
    const int64_t no = (int64_t)n_sparse * n + 1;
    DLRM_REQUIRE(offset_bits == 64 || no <= (int64_t)INT32_MAX, DLRM_ERR_UNSUPPORTED,
                 "%s: int32 offsets overflow", name);
    if (offset_bits == 32)
      hipLaunchKernelGGL(iota_kernel<int32_t>, dim3(grid_stride_blocks(no)), dim3(256), 0, st,
                         static_cast<int32_t*>(offsets), no);
    else
      hipLaunchKernelGGL(iota_kernel<int64_t>, dim3(grid_stride_blocks(no)), dim3(256), 0, st,
                         static_cast<int64_t*>(offsets), no);
  }
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}
