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
__device__ __forceinline__ float vdot(const float4& a) {
  return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
}
__device__ __forceinline__ float vdot(const float& a) { return a * a; }


}  // namespace
