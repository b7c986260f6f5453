// The DLRM head's finalize pass (column sums of the row-block partials -> the weight
// gradient / fused SGD, and the mean loss) as a device body: run by head_finalize_kernel
// (misc.hip) or as extra workgroups of the next grouped GEMM launch (gemm.hip, LaunchRole
// phase 4 via dlrm_head_step_defer) - the top-MLP backward's first launch reads dX, not
// the head weight the pass updates.
#pragma once
#include "common.hpp"

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// One wave per column k = blk * 4 + wave: lane l sums blocks l, l+64, ... in order, then a
// fixed xor-tree across lanes (deterministic).  Workgroup nwg - 1 also reduces the per-row
// loss terms the same way (red: 4 floats of LDS).
__device__ __forceinline__ void head_finalize_body(int64_t M, int64_t K, int64_t nblk,
                                                   const float* __restrict__ part,
                                                   float* __restrict__ w, float lr,
                                                   float* __restrict__ dw, int accumulate,
                                                   const float* __restrict__ row_loss,
                                                   float* __restrict__ loss_out, int blk, int nwg,
                                                   float* red) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blk * 4 + (threadIdx.x >> 6);
  if (k < K) {
    float s = 0.f;
    for (int64_t b = lane; b < nblk; b += 64) s += part[b * K + k];
    s = wave_sum(s);
    if (lane == 0) {
      if (dw) dw[k] = accumulate ? dw[k] + s : s;
      else if (lr != 0.f) w[k] = fmaf(-lr, s, w[k]);
    }
  }
  if (blk == nwg - 1 && loss_out) {
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < M; i += 256) s += row_loss[i];
    s = wave_sum(s);
    if (lane == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) loss_out[0] = ((red[0] + red[1]) + red[2] + red[3]) / (float)M;
  }
}

}  // namespace
