// 2D front-end convolutions (FeatureNet, models/module.py:355-462; GeoFeatureFusion,
// models/geometry.py:14-277) as NHWC implicit GEMM on MFMA, with the glue the reference runs as
// separate ops fused in:
//   * channel concat of two feature tensors (torch.cat([r2p, s2]) etc.): K runs over in0 then in1;
//   * up to 4 fp32 planar "geometry" inputs (the 1-channel depth planes BasicBlockGeo concatenates,
//     or the RGB/depth planes of the 2-4 channel init convs) added by VALU in the epilogue;
//   * bias (BN folded host side), residual before ReLU (BasicBlockGeo identity/downsample),
//     ReLU, residual after ReLU (decoder skips, FPN's nearest-x2 upsampled top-down path).
// Conv and ConvTranspose share one kernel: a transposed conv of stride s is s^2 output-parity
// phases, each a dense sub-convolution over the input grid (no structural zeros on MFMA).
#include "damvs_device.h"

namespace damvs {

namespace {

template <typename T> struct Frag2;
template <> struct Frag2<float> {
  typedef float4 raw;
  __device__ __forceinline__ static void mma(const raw& w, const raw& x, f32x4_t& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x.w, acc, 0, 0, 0);
  }
  __device__ __forceinline__ static raw zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <> struct Frag2<bf16_t> {
  typedef uint4 raw;
  __device__ __forceinline__ static void mma(const raw& w, const raw& x, f32x4_t& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, w), __builtin_bit_cast(bf16x8_t, x),
                                                  acc, 0, 0, 0);
  }
  __device__ __forceinline__ static raw zero() { return make_uint4(0u, 0u, 0u, 0u); }
};

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

constexpr int kG2 = 4;  // 16-pixel groups per wave

// Epilogue shared by the MFMA and the VALU-only kernels: geometry planes, bias, residuals, ReLU.
template <typename T>
__device__ __forceinline__ void epilogue4(const Conv2dArgs& a, const Conv2dPhase& ph, int b, int qy, int qx, int co,
                                          float* r) {
  const int oy = qy * a.out_stride + ph.py, ox = qx * a.out_stride + ph.px;
  if (a.ngeo > 0) {
    const float* wg = a.wgeo + (size_t)ph.g_off * a.cout_pad;  // [tap][g][cout_pad]
    for (int t = 0; t < ph.ntaps; ++t) {
      const int iy = qy * a.in_stride + ph.tap[t][0], ix = qx * a.in_stride + ph.tap[t][1];
      if ((unsigned)iy >= (unsigned)a.Hi || (unsigned)ix >= (unsigned)a.Wi) continue;
      for (int g = 0; g < a.ngeo; ++g) {
        const float v = a.geo[g][(size_t)b * a.geo_bstride[g] + (size_t)iy * a.Wi + ix];
        const float4 w = *reinterpret_cast<const float4*>(wg + ((size_t)t * a.ngeo + g) * a.cout_pad + co);
        r[0] += w.x * v; r[1] += w.y * v; r[2] += w.z * v; r[3] += w.w * v;
      }
    }
  }
  const size_t ob = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.cout + co;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] += a.bias[co + i];
  if (a.res_pre) {
    float q[4];
    ld4<T>(reinterpret_cast<const T*>(a.res_pre) + ob, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] += q[i];
  }
  if (a.relu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = fmaxf(r[i], 0.f);
  }
  if (a.res_post) {
    const int up = a.post_up;  // 1, or 2 for a nearest-x2 upsampled source of half resolution
    const size_t pb = (((size_t)b * (a.Ho / up) + oy / up) * (a.Wo / up) + ox / up) * a.cout + co;
    float q[4];
    ld4<T>(reinterpret_cast<const T*>(a.res_post) + pb, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] += q[i];
  }
  st4<T>(reinterpret_cast<T*>(a.out) + ob, r);
}

template <typename T, int MT>
__global__ __launch_bounds__(256) void conv2d_mfma_kernel(const Conv2dArgs a, int nqblk) {
  typedef typename Frag2<T>::raw raw;
  constexpr int E = Stor<T>::E;
  constexpr int KC = 4 * E;
  // logical block = (q-block, phase), phase fastest, XCD-contiguous (see conv3d_mfma_kernel)
  const int nblk = nqblk * a.nphase;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int qblk = L / a.nphase;
  const Conv2dPhase& ph = a.ph[L - qblk * a.nphase];
  const int mt0 = blockIdx.y * MT;  // first 16-channel output tile of this block

  __shared__ int s_tap[32];
  if (threadIdx.x < 25) s_tap[threadIdx.x] = ((int)(ph.tap[threadIdx.x][0] + 8)) | ((int)(ph.tap[threadIdx.x][1] + 8) << 8);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const long long Qtot = (long long)a.B * a.Hq * a.Wq;
  const long long base = ((long long)qblk * 4 + wave) * (kG2 * 16);
  if (base >= Qtot) return;
  int vb[kG2], vy[kG2], vx[kG2];
  bool valid[kG2];
#pragma unroll
  for (int j = 0; j < kG2; ++j) {
    long long q = base + j * 16 + n;
    valid[j] = q < Qtot;
    if (!valid[j]) q = 0;
    vx[j] = (int)(q % a.Wq); q /= a.Wq;
    vy[j] = (int)(q % a.Hq);
    vb[j] = (int)(q / a.Hq);
  }
  f32x4_t acc[kG2][MT];
#pragma unroll
  for (int j = 0; j < kG2; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int ctot = a.c0 + a.c1;
  if (ctot > 0) {
    const T* __restrict__ in0 = reinterpret_cast<const T*>(a.in0);
    const T* __restrict__ in1 = reinterpret_cast<const T*>(a.in1);
    const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 64 + lane;
    for (int s = 0; s < ph.kchunks; ++s) {
      const int k0 = s * KC + g * E;
      const int t = k0 / ctot;
      int ci = k0 - t * ctot;
      const bool tv = t < ph.ntaps;
      const int code = s_tap[tv ? t : 0];
      const int dy = (code & 0xff) - 8, dx = ((code >> 8) & 0xff) - 8;
      const bool second = ci >= a.c0;
      const T* src = second ? in1 : in0;
      const int cs = second ? a.c1 : a.c0;
      ci = second ? ci - a.c0 : ci;
      raw wf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)(s * a.MTtot + m) * 64];
      raw xf[kG2];
#pragma unroll
      for (int j = 0; j < kG2; ++j) {
        const int iy = vy[j] * a.in_stride + dy, ix = vx[j] * a.in_stride + dx;
        const bool ok = valid[j] && tv && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
        const size_t off = ok ? (((size_t)vb[j] * a.Hi + iy) * a.Wi + ix) * cs + ci : 0;
        const raw v = *reinterpret_cast<const raw*>((ok ? src : in0) + off);
        xf[j] = ok ? v : Frag2<T>::zero();
      }
#pragma unroll
      for (int j = 0; j < kG2; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) Frag2<T>::mma(wf[m], xf[j], acc[j][m]);
    }
  }

#pragma unroll
  for (int j = 0; j < kG2; ++j) {
    if (!valid[j]) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int co = (mt0 + m) * 16 + g * 4;
      if (co >= a.cout) continue;
      float r[4] = {acc[j][m][0], acc[j][m][1], acc[j][m][2], acc[j][m][3]};
      epilogue4<T>(a, ph, vb[j], vy[j], vx[j], co, r);
    }
  }
}

template <typename T, int MT>
hipError_t launch_mt(hipStream_t s, const Conv2dArgs& a) {
  const long long Qtot = (long long)a.B * a.Hq * a.Wq;
  const int nq = (int)((Qtot + 4LL * kG2 * 16 - 1) / (4LL * kG2 * 16));
  dim3 grid((unsigned)(nq * a.nphase), (unsigned)((a.MTtot + MT - 1) / MT));
  hipLaunchKernelGGL((conv2d_mfma_kernel<T, MT>), grid, dim3(256), 0, s, a, nq);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_t(hipStream_t s, const Conv2dArgs& a) {
  if (a.MTtot >= 4 && a.MTtot % 4 == 0) return launch_mt<T, 4>(s, a);
  if (a.MTtot >= 2 && a.MTtot % 2 == 0) return launch_mt<T, 2>(s, a);
  return launch_mt<T, 1>(s, a);
}

}  // namespace

hipError_t launch_conv2d(hipStream_t s, int store, const Conv2dArgs& a) {
  return store == ST_BF16 ? launch_t<bf16_t>(s, a) : launch_t<float>(s, a);
}

}  // namespace damvs
