// Shared by the 2D conv units (k_conv2d.hip: MFMA kernels; k_planes.hip: the VALU plane-input kernels): 4-channel
// NHWC load / store and the epilogue tail (residual before ReLU, ReLU, residual after ReLU, store).
#pragma once

#include "damvs_device.h"

namespace damvs {
namespace {

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float* r);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float* r) {
  float4 v = *reinterpret_cast<const float4*>(p);
  r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
}
template <>
__device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float* r) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  r[0] = __uint_as_float(v.x << 16); r[1] = __uint_as_float(v.x & 0xffff0000u);
  r[2] = __uint_as_float(v.y << 16); r[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float* r);
template <>
__device__ __forceinline__ void st4<float>(float* p, const float* r) {
  *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
}
template <>
__device__ __forceinline__ void st4<bf16_t>(bf16_t* p, const float* r) {
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f2bf(r[0]) | ((uint32_t)f2bf(r[1]) << 16),
                                            (uint32_t)f2bf(r[2]) | ((uint32_t)f2bf(r[3]) << 16));
}

// Residual before ReLU, ReLU, (upsampled) residual after ReLU, store of 4 channels (32-bit indices:
// the launcher keeps every operand below 2^31 elements).
template <typename T>
__device__ __forceinline__ void tail4(const Conv2dArgs& a, int b, int oy, int ox, int co, float* r) {
  const uint32_t ob = (uint32_t)(((b * a.Ho + oy) * a.Wo + ox) * a.cout + co);
  if (a.res_pre) {
    float q[4];
    ld4<T>(reinterpret_cast<const T*>(a.res_pre) + ob, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] += q[i];
  }
  if (a.relu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
  }
  if (a.res_post) {
    const int up = a.post_up;  // 1, or 2 for a nearest-x2 upsampled source of half resolution
    const uint32_t pb = (uint32_t)(((b * (a.Ho / up) + oy / up) * (a.Wo / up) + ox / up) * a.cout + co);
    float q[4];
    ld4<T>(reinterpret_cast<const T*>(a.res_post) + pb, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] += q[i];
  }
  st4<T>(reinterpret_cast<T*>(a.out) + ob, r);
}

}  // namespace
}  // namespace damvs
