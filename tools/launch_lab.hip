// Launch-overhead lab (experiment, not product code): what a launch boundary and a
// grid-wide barrier cost on MI355X, to size a persistent small-batch step.
//   lab_empty   : G workgroups that do nothing
//   lab_touch   : G workgroups, one float4 load + store per thread
//   lab_barrier : G workgroups crossing `nbar` grid barriers (monotonic agent-scope
//                 counter; every spin bounded, a timeout raises err[0])
// Built by tools/launch_lab.py --build into tools/_lab/liblaunch_lab.so.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void k_empty(int* sink) {
  if (sink && threadIdx.x == 1024) sink[0] = 1;  // never taken
}

__global__ __launch_bounds__(256) void k_touch(const float4* __restrict__ a, float4* __restrict__ b) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  float4 v = a[i];
  v.x += 1.f;
  b[i] = v;
}

__device__ __forceinline__ bool grid_sync(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  return true;
}

__global__ __launch_bounds__(256) void k_barrier(unsigned* ctr, unsigned base, int nbar, int* err,
                                                 float* out) {
  const unsigned G = gridDim.x;
  float acc = 0.f;
  for (int i = 0; i < nbar; ++i) {
    grid_sync(ctr, base + (unsigned)(i + 1) * G, err);
    acc += 1.f;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

extern "C" {
int lab_empty(int grid, void* stream) {
  hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int*)nullptr);
  return (int)hipGetLastError();
}
int lab_touch(int grid, const void* a, void* b, void* stream) {
  hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)a,
                     (float4*)b);
  return (int)hipGetLastError();
}
// ctr must be zero before the first call; `base` = grid * (total barriers crossed before).
int lab_barrier(int grid, void* ctr, unsigned base, int nbar, void* err, void* out, void* stream) {
  hipLaunchKernelGGL(k_barrier, dim3(grid), dim3(256), 0, (hipStream_t)stream, (unsigned*)ctr, base,
                     nbar, (int*)err, (float*)out);
  return (int)hipGetLastError();
}
}
