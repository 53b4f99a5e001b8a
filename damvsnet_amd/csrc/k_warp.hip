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
// Warp arithmetic follows models/module.py:318-329: q = (R [x y 1]^T) d + t, u = q_x / q_z,
// g = u / ((W-1)/2) - 1 (align-corners style normalisation), then grid_sample's
// align_corners=False unnormalisation ix = ((g + 1) W - 1) / 2, bilinear, zero padding; the
// normalise/unnormalise pair is folded algebraically (ix = u W/(W-1) - 1/2).
#include <cstdlib>

#include "damvs_device.h"

namespace damvs {

namespace {

// Bilinear sample of C channels at (ix, iy), zero padding. Branch-free: invalid taps load from a
// clamped in-bounds address with weight 0 (all four loads issue back to back). BLK selects the
// channel-blocked layout [C/E][h][w][E] (one contiguous 16-byte plane per chunk: a wave's gather
// touches half the cache lines of plain NHWC for C > E).
template <typename T, int C, bool BLK>
__device__ __forceinline__ void sample_bilinear(const T* __restrict__ src, int h, int w, float ix, float iy, float* s) {
  constexpr int E = Stor<T>::E;
  const bool inside = ix > -2.f && ix < (float)w + 1.f && iy > -2.f && iy < (float)h + 1.f;  // false for NaN
  const float cx = inside ? ix : -4.f, cy = inside ? iy : -4.f;
  const float x0f = floorf(cx), y0f = floorf(cy);
  const int x0 = (int)x0f, y0 = (int)y0f;
  const float wx1 = cx - x0f, wx0 = (x0f + 1.f) - cx;
  const float wy1 = cy - y0f, wy0 = (y0f + 1.f) - cy;
  float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};  // nw, ne, sw, se
  int idx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
    const bool ok = xx >= 0 && xx < w && yy >= 0 && yy < h;
    idx[k] = ok ? yy * w + xx : 0;
    wt[k] = ok ? wt[k] : 0.f;
  }
  const size_t plane = (size_t)h * w * E;
#pragma unroll
  for (int q = 0; q < C / E; ++q) {
    float v[4][E];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      Stor<T>::load16(BLK ? src + q * plane + (size_t)idx[k] * E : src + (size_t)idx[k] * C + q * E, v[k]);
#pragma unroll
    for (int e = 0; e < E; ++e)
      s[q * E + e] = ((v[0][e] * wt[0] + v[1][e] * wt[1]) + v[2][e] * wt[2]) + v[3][e] * wt[3];
  }
}

// Work decomposition (locality): a block owns 256 consecutive pixels of one image row band and a
// chunk of `dchunk` consecutive depth planes, and each thread walks its pixel through those planes.
// Consecutive hypotheses of one pixel sample along one epipolar segment, so a block's gathers stay
// inside a narrow band of each source image; blocks are dealt so that each XCD gets a contiguous
// range of (pixel-chunk, depth-chunk) work and its L2 holds that band (the naive (pixels, D) grid
// spreads every depth slice over all 8 XCDs and serves the gathers from the Infinity Cache).
template <typename T, int C, int MODE, bool BLK, int NVC>
__global__ __launch_bounds__(256) void warp_aggregate_kernel(const WarpArgs a, int npix_blocks, int dchunk,
                                                             int ndchunks) {
  const int hw = a.h * a.w, ohw = a.rows * a.w;  // feature-map plane, computed rows (y0 .. y0 + rows - 1)
  const int nblk = npix_blocks * ndchunks * a.B;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;  // bijective XCD remap
  const int dc = L % ndchunks; L /= ndchunks;
  const int pb = L % npix_blocks;
  const int b = L / npix_blocks;
  // this batch element's [N-1][12] source cameras in LDS: the per-plane reads below are broadcast
  // ds_reads instead of 12 vector-memory loads per view per plane through the (gather-bound) TA
  __shared__ __attribute__((aligned(16))) float s_rtf[(kMaxViews - 1) * 12];
  if (threadIdx.x < (a.N - 1) * 12) s_rtf[threadIdx.x] = a.rt[(size_t)b * (a.N - 1) * 12 + threadIdx.x];
  __syncthreads();
  const float4* s_rt = reinterpret_cast<const float4*>(s_rtf);
  const int p = pb * 256 + threadIdx.x;
  if (p >= ohw) return;
  const int yl = p / a.w, x = p - yl * a.w;
  const int y = a.y0 + yl, pg = y * a.w + x;  // reference-image row and pixel
  const float fx = (float)x, fy = (float)y;
  const float kx = (float)a.w / (float)(a.w - 1), ky = (float)a.h / (float)(a.h - 1);

  float ref[C];
  if (MODE != AGG_WARP_ONLY) {
    const T* f0 = reinterpret_cast<const T*>(a.feats[0]) + (size_t)b * hw * C;
    constexpr int E = Stor<T>::E;
#pragma unroll
    for (int q = 0; q < C / E; ++q)
      Stor<T>::load16(BLK ? f0 + ((size_t)q * hw + pg) * E : f0 + (size_t)pg * C + q * E, ref + q * E);
  }

  const float inv_n = 1.f / (float)a.N, inv_n1 = 1.f / (float)(a.N - 1);  // exact for N = 5 (the default)
  const int d0 = dc * dchunk, d1 = min(a.D, d0 + dchunk);
  for (int d = d0; d < d1; ++d) {
    const size_t vox = (((size_t)b * a.D + d) * a.out_rows + a.out_y) * a.w + p;
    const float hyp = a.hyps[vox];
    float acc[C], sq[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      acc[c] = (MODE == AGG_VARIANCE) ? ref[c] : 0.f;
      sq[c] = (MODE == AGG_VARIANCE) ? ref[c] * ref[c] : 0.f;
    }
    // NVC > 0: the source-view count is a compile-time constant and the view loop unrolls, so the
    // gathers of several views are in flight together
    const int nviews = NVC > 0 ? NVC + 1 : a.N;
    constexpr int kUnrollV = NVC > 0 ? NVC : 1;
#pragma unroll kUnrollV
    for (int v = 1; v < nviews; ++v) {
      const float4 m0 = s_rt[(v - 1) * 3], m1 = s_rt[(v - 1) * 3 + 1], m2 = s_rt[(v - 1) * 3 + 2];
      const float m[12] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w, m2.x, m2.y, m2.z, m2.w};
      const float rx = m[0] * fx + m[1] * fy + m[2];
      const float ry = m[3] * fx + m[4] * fy + m[5];
      const float rz = m[6] * fx + m[7] * fy + m[8];
      const float qx = rx * hyp + m[9], qy = ry * hyp + m[10], qz = rz * hyp + m[11];
      // g = (q/qz) / ((W-1)/2) - 1 and ix = ((g + 1) W - 1) / 2 fold to ix = (q/qz) W/(W-1) - 1/2:
      // one reciprocal instead of four IEEE divisions (coordinates agree to ~1 ulp)
      const float iz = __builtin_amdgcn_rcpf(qz);
      const float ix = qx * iz * kx - 0.5f;
      const float iy = qy * iz * ky - 0.5f;
      float s[C];
      sample_bilinear<T, C, BLK>(reinterpret_cast<const T*>(a.feats[v]) + (size_t)b * hw * C, a.h, a.w, ix, iy, s);
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
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float mean = acc[c] * inv_n;
        o[c] = sq[c] * inv_n - mean * mean;
      }
    } else if (MODE == AGG_ADAPTIVE) {
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = acc[c] * inv_n1;
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = acc[c];
    }
    store_vec<T, C>(reinterpret_cast<T*>(a.out) + vox * C, o);
  }
}

template <typename T, int C, int MODE, bool BLK>
void launch_k(hipStream_t s, const WarpArgs& a, dim3 grid, int npb, int dchunk, int ndc) {
  if (a.N == 5 && C <= 16)  // C = 32: the unrolled views cost more registers than they hide
    hipLaunchKernelGGL((warp_aggregate_kernel<T, C, MODE, BLK, 4>), grid, dim3(256), 0, s, a, npb, dchunk, ndc);
  else
    hipLaunchKernelGGL((warp_aggregate_kernel<T, C, MODE, BLK, 0>), grid, dim3(256), 0, s, a, npb, dchunk, ndc);
}

template <typename T, int MODE, bool BLK>
hipError_t launch_c(hipStream_t s, const WarpArgs& a) {
  const int npb = (a.rows * a.w + 255) / 256;
  // depth chunk: as long as possible (locality) while keeping >= ~4 blocks per CU in flight
  int dchunk = a.D;
  static const long long minblk = [] {
    const char* e = getenv("DAMVS_WARP_MINBLK");
    return e ? atoll(e) : 2048LL;
  }();
  while (dchunk > 2 && (long long)npb * a.B * ((a.D + dchunk - 1) / dchunk) < minblk) dchunk = (dchunk + 1) / 2;
  const int ndc = (a.D + dchunk - 1) / dchunk;
  dim3 grid((unsigned)(npb * ndc * a.B));
  switch (a.C) {
    case 8: launch_k<T, 8, MODE, BLK>(s, a, grid, npb, dchunk, ndc); break;
    case 16: launch_k<T, 16, MODE, BLK>(s, a, grid, npb, dchunk, ndc); break;
    case 32: launch_k<T, 32, MODE, BLK>(s, a, grid, npb, dchunk, ndc); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T, bool BLK>
hipError_t launch_t(hipStream_t s, int mode, const WarpArgs& a) {
  switch (mode) {
    case AGG_ADAPTIVE: return launch_c<T, AGG_ADAPTIVE, BLK>(s, a);
    case AGG_VARIANCE: return launch_c<T, AGG_VARIANCE, BLK>(s, a);
    case AGG_WARP_ONLY: return launch_c<T, AGG_WARP_ONLY, BLK>(s, a);
  }
  return hipErrorInvalidValue;
}

// [N views][B][h][w][C] -> [B][C/E][h][w][E] per view; one thread per (view, b, pixel, chunk).
template <typename T>
__global__ __launch_bounds__(256) void block_channels_kernel(const FeatPtrs src, FeatPtrs dst, int B, int hw, int C,
                                                             int N) {
  constexpr int E = Stor<T>::E;
  const int CH = C / E;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per_view = (long long)B * hw * CH;
  if (i >= per_view * N) return;
  const int v = (int)(i / per_view);
  long long r = i - v * per_view;
  const int p = (int)(r % hw);
  r /= hw;
  const int q = (int)(r % CH);
  const int b = (int)(r / CH);
  const T* sp = reinterpret_cast<const T*>(src.p[v]) + ((size_t)b * hw + p) * C + q * E;
  T* dp = const_cast<T*>(reinterpret_cast<const T*>(dst.p[v])) + (((size_t)b * CH + q) * hw + p) * E;
  *reinterpret_cast<uint4*>(dp) = *reinterpret_cast<const uint4*>(sp);
}

}  // namespace

hipError_t launch_warp_aggregate(hipStream_t s, int store, int mode, const WarpArgs& a, bool blocked) {
  if (blocked) return store == ST_BF16 ? launch_t<bf16_t, true>(s, mode, a) : launch_t<float, true>(s, mode, a);
  return store == ST_BF16 ? launch_t<bf16_t, false>(s, mode, a) : launch_t<float, false>(s, mode, a);
}

hipError_t launch_block_channels(hipStream_t s, int store, const FeatPtrs& src, const FeatPtrs& dst, int N, int B,
                                 int hw, int C) {
  const long long n = (long long)N * B * hw * (C / (store == ST_BF16 ? 8 : 4));
  dim3 grid((unsigned)((n + 255) / 256));
  if (store == ST_BF16)
    hipLaunchKernelGGL(block_channels_kernel<bf16_t>, grid, dim3(256), 0, s, src, dst, B, hw, C, N);
  else
    hipLaunchKernelGGL(block_channels_kernel<float>, grid, dim3(256), 0, s, src, dst, B, hw, C, N);
  return hipGetLastError();
}

}  // namespace damvs
