// Fused homography warp + cross-view cost aggregation (one pass, one write of the volume).
//
// Replaces, per stage, the reference's per-source-view chain (models/cas_mvsnet.py:30-87):
//   ref_volume repeat (:30) -> homo_warping grid build + F.grid_sample (models/module.py:297-332)
//   -> (ref - warped)^2 (:66) -> AggWeightNetVolume (module.py:544-563) -> acc += (w+1) x (:73-76)
//   -> / (N-1) (:87)                                   [adaptive, the default agg_mode]
//   or  sum, sum^2 -> sq/N - (sum/N)^2 (:35-36,62-63,85) [variance]
// None of the (B,3,D,h*w) grids, (B,C,D,h,w) warped volumes or the repeated reference volume
// are materialised: one thread owns one voxel (b, d, y, x), keeps the reference C-vector and
// the running aggregate in registers, and writes the C-vector of the aggregated volume once
// (NDHWC, 16-byte stores, consecutive threads -> consecutive voxels).
//
// Warp arithmetic follows models/module.py:318-329 exactly: q = (R [x y 1]^T) d + t,
// u = q_x / q_z, g = u / ((W-1)/2) - 1 (align-corners style normalisation), then grid_sample's
// align_corners=False unnormalisation ix = ((g + 1) W - 1) / 2, bilinear, zero padding.
#include "damvs_device.h"

namespace damvs {

namespace {

template <typename T, int C>
__device__ __forceinline__ void sample_bilinear(const T* __restrict__ src, int h, int w, float ix, float iy, float* s) {
#pragma unroll
  for (int c = 0; c < C; ++c) s[c] = 0.f;
  // Non-finite or far-away coordinates sample nothing (all four taps out of bounds).
  if (!(ix > -2.f && ix < (float)w + 1.f && iy > -2.f && iy < (float)h + 1.f)) return;
  const float x0f = floorf(ix), y0f = floorf(iy);
  const int x0 = (int)x0f, y0 = (int)y0f;
  const float wx1 = ix - x0f, wx0 = (x0f + 1.f) - ix;
  const float wy1 = iy - y0f, wy0 = (y0f + 1.f) - iy;
  const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};  // nw, ne, sw, se
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
    if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;
    float v[C];
    load_vec<T, C>(src + ((size_t)yy * w + xx) * C, v);
#pragma unroll
    for (int c = 0; c < C; ++c) s[c] += v[c] * wt[k];
  }
}

template <typename T, int C, int MODE>
__global__ __launch_bounds__(256) void warp_aggregate_kernel(const WarpArgs a) {
  const int hw = a.h * a.w;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int d = blockIdx.y, b = blockIdx.z;
  if (p >= hw) return;
  const int y = p / a.w, x = p - y * a.w;
  const size_t vox = ((size_t)b * a.D + d) * hw + p;
  const float hyp = a.hyps[vox];
  const float fx = (float)x, fy = (float)y;
  const float nx = (float)(a.w - 1) * 0.5f, ny = (float)(a.h - 1) * 0.5f;

  float ref[C], acc[C], sq[C];
  if (MODE != AGG_WARP_ONLY) {
    load_vec<T, C>(reinterpret_cast<const T*>(a.feats[0]) + ((size_t)b * hw + p) * C, ref);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    acc[c] = (MODE == AGG_VARIANCE) ? ref[c] : 0.f;
    sq[c] = (MODE == AGG_VARIANCE) ? ref[c] * ref[c] : 0.f;
  }

  for (int v = 1; v < a.N; ++v) {
    const float* m = a.rt + ((size_t)b * (a.N - 1) + (v - 1)) * 12;
    const float rx = m[0] * fx + m[1] * fy + m[2];
    const float ry = m[3] * fx + m[4] * fy + m[5];
    const float rz = m[6] * fx + m[7] * fy + m[8];
    const float qx = rx * hyp + m[9], qy = ry * hyp + m[10], qz = rz * hyp + m[11];
    const float gx = (qx / qz) / nx - 1.f, gy = (qy / qz) / ny - 1.f;
    const float ix = ((gx + 1.f) * (float)a.w - 1.f) * 0.5f;
    const float iy = ((gy + 1.f) * (float)a.h - 1.f) * 0.5f;
    float s[C];
    sample_bilinear<T, C>(reinterpret_cast<const T*>(a.feats[v]) + (size_t)b * hw * C, a.h, a.w, ix, iy, s);
    if (MODE == AGG_WARP_ONLY) {
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = s[c];
    } else if (MODE == AGG_VARIANCE) {
#pragma unroll
      for (int c = 0; c < C; ++c) { acc[c] += s[c]; sq[c] += s[c] * s[c]; }
    } else {
      float dot = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float df = ref[c] - s[c];
        s[c] = df * df;
        dot += a.k1[c] * s[c];
      }
      const float a1 = fmaxf(dot * a.s1 + a.t1, 0.f);
      const float wt = fmaxf(a1 * a.s2 + a.t2, 0.f) + 1.f;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += wt * s[c];
    }
  }

  float o[C];
  if (MODE == AGG_VARIANCE) {
    const float n = (float)a.N;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float mean = acc[c] / n;
      o[c] = sq[c] / n - mean * mean;
    }
  } else if (MODE == AGG_ADAPTIVE) {
    const float n1 = (float)(a.N - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = acc[c] / n1;
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = acc[c];
  }
  store_vec<T, C>(reinterpret_cast<T*>(a.out) + vox * C, o);
}

template <typename T, int MODE>
hipError_t launch_c(hipStream_t s, const WarpArgs& a) {
  dim3 grid((a.h * a.w + 255) / 256, a.D, a.B);
  switch (a.C) {
    case 8: hipLaunchKernelGGL((warp_aggregate_kernel<T, 8, MODE>), grid, dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL((warp_aggregate_kernel<T, 16, MODE>), grid, dim3(256), 0, s, a); break;
    case 32: hipLaunchKernelGGL((warp_aggregate_kernel<T, 32, MODE>), grid, dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_t(hipStream_t s, int mode, const WarpArgs& a) {
  switch (mode) {
    case AGG_ADAPTIVE: return launch_c<T, AGG_ADAPTIVE>(s, a);
    case AGG_VARIANCE: return launch_c<T, AGG_VARIANCE>(s, a);
    case AGG_WARP_ONLY: return launch_c<T, AGG_WARP_ONLY>(s, a);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_warp_aggregate(hipStream_t s, int store, int mode, const WarpArgs& a) {
  return store == ST_BF16 ? launch_t<bf16_t>(s, mode, a) : launch_t<float>(s, mode, a);
}

}  // namespace damvs
