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
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "damvs_device.h"

namespace damvs {

namespace {

constexpr int kWarpBlock = 256;  // threads per warp block

// One 16-byte storage record -> E floats.
template <typename T> struct Rec16;
template <> struct Rec16<float> {
  __device__ __forceinline__ static void unpack(const uint4& q, float* v) {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
  }
};
template <> struct Rec16<bf16_t> {
  __device__ __forceinline__ static void unpack(const uint4& q, float* v) {
    const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
};

// Bilinear footprint of one sample at (ix, iy): byte offsets of the nw, ne, sw, se pixel records inside one
// batch element's map (rec bytes per record) and their weights. A corner outside the map gets the offset
// kOOB, so its buffer load returns 0: grid_sample's zero padding without a weight select. Samples far
// outside (or NaN) are moved to (-4, -4), where all four corners are outside.
struct Taps {
  uint32_t off[4];
  float wt[4];
};
__device__ __forceinline__ Taps bilinear_taps(int h, int w, uint32_t rec, float ix, float iy) {
  const bool inside = ix > -2.f && ix < (float)w + 1.f && iy > -2.f && iy < (float)h + 1.f;  // false for NaN
  const float cx = inside ? ix : -4.f, cy = inside ? iy : -4.f;
  const float x0f = floorf(cx), y0f = floorf(cy);
  const int x0 = (int)x0f, y0 = (int)y0f;
  const float wx1 = cx - x0f, wx0 = (x0f + 1.f) - cx;
  const float wy1 = cy - y0f, wy0 = (y0f + 1.f) - cy;
  Taps t;
  t.wt[0] = wx0 * wy0;
  t.wt[1] = wx1 * wy0;
  t.wt[2] = wx0 * wy1;
  t.wt[3] = wx1 * wy1;
  const bool vx0 = (unsigned)x0 < (unsigned)w, vx1 = (unsigned)(x0 + 1) < (unsigned)w;
  const bool vy0 = (unsigned)y0 < (unsigned)h, vy1 = (unsigned)(y0 + 1) < (unsigned)h;
  const uint32_t o = (uint32_t)(y0 * w + x0) * rec, ow = (uint32_t)w * rec;  // wraps for x0 / y0 = -1: fine
  t.off[0] = vx0 && vy0 ? o : kOOB;
  t.off[1] = vx1 && vy0 ? o + rec : kOOB;
  t.off[2] = vx0 && vy1 ? o + ow : kOOB;
  t.off[3] = vx1 && vy1 ? o + ow + rec : kOOB;
  return t;
}

// Reference pixel (index into the computed rows) of thread slot i (0 .. ppb - 1) of pixel block pb, -1 outside them.
__device__ __forceinline__ int warp_pixel(const WarpArgs& a, int pb, int i, int ppb) {
  if (a.tile_r == 0) {
    const int p = pb * ppb + i;
    return p < a.rows * a.w ? p : -1;
  }
  const int tc = ppb / a.tile_r;
  const int tiles_y = (a.rows + a.tile_r - 1) / a.tile_r;
  const int per_strip = a.tile_sw * tiles_y;
  const int strip = pb / per_strip, r = pb - strip * per_strip;
  const int sw = min(a.tile_sw, a.tiles_x - strip * a.tile_sw);
  const int ty = r / sw, tx = strip * a.tile_sw + (r - ty * sw);
  const int tr = i / tc;
  const int x = tx * tc + (i - tr * tc), yl = ty * a.tile_r + tr;
  return (x < a.w && yl < a.rows) ? yl * a.w + x : -1;
}

// Work decomposition (locality): a block owns its block size of consecutive pixels of one image row band and a
// chunk of `dchunk` consecutive depth planes, and each thread walks its pixel through those planes.
// Consecutive hypotheses of one pixel sample along one epipolar segment, so a block's gathers stay
// inside a narrow band of each source image; blocks are dealt so that each XCD gets a contiguous
// range of (pixel-chunk, depth-chunk) work and its L2 holds that band (the naive (pixels, D) grid
// spreads every depth slice over all 8 XCDs and serves the gathers from the Infinity Cache).
//
// Per thread the depth-independent part of each view's homography (the ray R [x y 1]^T) is computed
// once; the cameras' translations are block-uniform (SGPRs). Gathers are buffer loads with 32-bit offsets (the
// batch element and channel chunk in the scalar offset), so a tap costs one select instead of 64-bit
// address arithmetic and a weight select. With NVC > 0 (the source-view count a compile-time constant)
// the (depth, view) sequence is software-pipelined one view deep: the 4 x C/E records of the next view
// (across the depth boundary too, from a hypothesis loaded a plane ahead) are in flight while the
// current view is reduced, and the loads are unconditional (the last plane re-reads its own last
// view) so the vmcnt waits count exactly.
template <typename T, int C, int MODE, bool BLK, int NVC>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kWarpBlock))) DAMVS_WAVES((sizeof(T) == 2 && C == 32 && NVC == 0 && MODE == AGG_ADAPTIVE ? 3 : 1)) void warp_aggregate_kernel(const WarpArgs a, const float* __restrict__ cams,
                                                             int npix_blocks, int dchunk, int ndchunks) {
  constexpr int BLOCK = kWarpBlock;
  constexpr int E = Stor<T>::E, NQ = C / E;
  static_assert(NVC % 2 == 0 || NVC < 0, "the view pipeline alternates two register sets");
  const int hw = a.h * a.w;  // feature-map plane (computed rows: y0 .. y0 + rows - 1)
  const int nblk = npix_blocks * ndchunks * a.B;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;  // bijective XCD remap
  const int dc = L % ndchunks; L /= ndchunks;
  const int pb = L % npix_blocks;
  const int b = L / npix_blocks;
  // this batch element's [N-1][12] source cameras: block-uniform reads through a read-only, non-aliased
  // kernel argument, i.e. scalar loads into SGPRs. (Staged in LDS and read back by the compiler's wide broadcast
  // ds_read_b128 / ds_read2_b64, lanes 48-63 of some waves got wrong cameras beside U-Net kernels on another
  // stream, while ds_read_b32 reads of the same copy were always right: DESIGN.md section 4, "Concurrent streams".)
  const float* __restrict__ cam = cams + (size_t)b * (a.N - 1) * 12;
  const int p0 = warp_pixel(a, pb, threadIdx.x, BLOCK);
  // fp32: lanes past the image walk pixel 0 with their stores dropped, so every lane reaches the wave's magnitude
  // reduction at the end (the volume's prescale slot, damvs_device.h prescale_of); bf16 records no magnitude
  const bool pv = p0 >= 0;
  if (sizeof(T) == 2 && !pv) return;
  const int p = pv ? p0 : 0;
  unsigned am = 0u;
  const int yl = p / a.w, x = p - yl * a.w;
  const int y = a.y0 + yl, pg = y * a.w + x;  // reference-image row and pixel
  const float fx = (float)x, fy = (float)y;
  const float kx = (float)a.w / (float)(a.w - 1), ky = (float)a.h / (float)(a.h - 1);

  // byte geometry of a feature map: record = one pixel (NHWC) or one pixel's chunk (blocked)
  const uint32_t bbytes = (uint32_t)hw * C * sizeof(T);
  const uint32_t rec = BLK ? 16u : (uint32_t)(C * sizeof(T));
  const uint32_t qstep = BLK ? (uint32_t)hw * 16u : 16u;  // bytes between a record's channel chunks
  const uint32_t sb = (uint32_t)b * bbytes;
  const long long fbytes = (long long)a.B * bbytes;

  float ref[C];
  if (MODE != AGG_WARP_ONLY) {
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.feats[0], fbytes);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      Rec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r0, (uint32_t)pg * rec, sb + q * qstep, 0)),
                       ref + q * E);
  }
  const float inv_n = 1.f / (float)a.N, inv_n1 = 1.f / (float)(a.N - 1);  // exact for N = 5 (the default)
  const int d0 = dc * dchunk, d1 = min(a.D, d0 + dchunk);
  auto vox_of = [&](int d) { return (((size_t)b * a.D + d) * a.out_rows + a.out_y) * a.w + p; };

  // per-channel reduction of one view's sample into the running aggregate
  auto reduce = [&](const uint4* rv, const float* wt, float* acc, float* sq) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float v[4][E];
#pragma unroll
      for (int k = 0; k < 4; ++k) Rec16<T>::unpack(rv[q * 4 + k], v[k]);
      float s[E];
#pragma unroll
      for (int e = 0; e < E; ++e) s[e] = ((v[0][e] * wt[0] + v[1][e] * wt[1]) + v[2][e] * wt[2]) + v[3][e] * wt[3];
      if (MODE == AGG_WARP_ONLY) {
#pragma unroll
        for (int e = 0; e < E; ++e) acc[q * E + e] = s[e];
      } else if (MODE == AGG_VARIANCE) {
#pragma unroll
        for (int e = 0; e < E; ++e) { acc[q * E + e] += s[e]; sq[q * E + e] += s[e] * s[e]; }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float df = ref[q * E + e] - s[e];
          sq[q * E + e] = df * df;  // adaptive: the squared difference, weighted below
        }
      }
    }
    if (MODE == AGG_ADAPTIVE) {
      float dot = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) dot += a.k1[c] * sq[c];
      const float a1 = fmaxf(dot * a.s1 + a.t1, 0.f);
      const float wv = fmaxf(a1 * a.s2 + a.t2, 0.f) + 1.f;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += wv * sq[c];
    }
  };
  auto finish = [&](int d, float* acc, float* sq) {
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
    if constexpr (sizeof(T) == 4) {
      unsigned m = am;
#pragma unroll
      for (int c = 0; c < C; ++c) m = amax_fold(m, o[c]);
      am = pv ? m : am;
      if (pv) store_vec<T, C>(reinterpret_cast<T*>(a.out) + vox_of(d) * C, o);
    } else {
      store_vec<T, C>(reinterpret_cast<T*>(a.out) + vox_of(d) * C, o);
    }
  };
  auto init = [&](float* acc, float* sq) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      acc[c] = (MODE == AGG_VARIANCE) ? ref[c] : 0.f;
      sq[c] = (MODE == AGG_VARIANCE) ? ref[c] * ref[c] : 0.f;
    }
  };

  if constexpr (NVC != 0) {
    // source view j = 1 + v: ray (per lane), translation (block-uniform) and descriptor. NVC > 0: the view count
    // is a compile-time constant and the rays are hoisted out of the depth loop; NVC < 0: any even number of
    // source views (a.N - 1, checked by the launcher), the view loop not unrolled and each view's ray recomputed
    // from the SGPR camera (the same expression, so the same coordinates), so registers do not grow with N.
    constexpr int NH = NVC > 0 ? NVC : 1;
    const int nv = NVC > 0 ? NVC : a.N - 1;
    float rx[NH], ry[NH], rz[NH], tx[NH], ty[NH], tz[NH];
    __amdgpu_buffer_rsrc_t rs[NH];
    if constexpr (NVC > 0) {
#pragma unroll
      for (int v = 0; v < NVC; ++v) {
        const float* m = cam + v * 12;
        rx[v] = m[0] * fx + m[1] * fy + m[2];
        ry[v] = m[3] * fx + m[4] * fy + m[5];
        rz[v] = m[6] * fx + m[7] * fy + m[8];
        tx[v] = m[9];
        ty[v] = m[10];
        tz[v] = m[11];
        rs[v] = make_rsrc(a.feats[v + 1], fbytes);
      }
    }
    auto taps = [&](int v, float hyp) {
      float qx, qy, qz;
      if constexpr (NVC > 0) {
        qx = rx[v] * hyp + tx[v], qy = ry[v] * hyp + ty[v], qz = rz[v] * hyp + tz[v];
      } else {
        const float* m = cam + v * 12;
        const float vx = m[0] * fx + m[1] * fy + m[2];
        const float vy = m[3] * fx + m[4] * fy + m[5];
        const float vz = m[6] * fx + m[7] * fy + m[8];
        qx = vx * hyp + m[9], qy = vy * hyp + m[10], qz = vz * hyp + m[11];
      }
      // g = (q/qz) / ((W-1)/2) - 1 and ix = ((g + 1) W - 1) / 2 fold to ix = (q/qz) W/(W-1) - 1/2:
      // one reciprocal instead of four IEEE divisions (coordinates agree to ~1 ulp)
      const float iz = __builtin_amdgcn_rcpf(qz);
      return bilinear_taps(a.h, a.w, rec, qx * iz * kx - 0.5f, qy * iz * ky - 0.5f);
    };
    auto issue = [&](int v, const Taps& t, uint4* rv, float* wt) {
      __amdgpu_buffer_rsrc_t r;
      if constexpr (NVC > 0) r = rs[v];
      else r = make_rsrc(a.feats[v + 1], fbytes);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          rv[q * 4 + k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, t.off[k], sb + q * qstep, 0));
#pragma unroll
      for (int k = 0; k < 4; ++k) wt[k] = t.wt[k];
    };
    uint4 ra[4 * NQ], rb[4 * NQ];
    float wa[4], wb[4];
    float hyp = a.hyps[vox_of(d0)];
    float hyp_n = a.hyps[vox_of(min(d0 + 1, d1 - 1))];
    issue(0, taps(0, hyp), ra, wa);
    for (int d = d0; d < d1; ++d) {
      const float hyp_nn = a.hyps[vox_of(min(d + 2, d1 - 1))];  // two planes ahead, first in the plane's loads
      float acc[C], sq[C];
      init(acc, sq);
      // view v's records are in (cur, wcur); the next (view, plane)'s go to (nxt, wnxt) before v is reduced
      auto step = [&](int v, const uint4* cur, const float* wcur, uint4* nxt, float* wnxt) {
        if (v + 1 < nv) issue(v + 1, taps(v + 1, hyp), nxt, wnxt);
        else issue(0, taps(0, hyp_n), nxt, wnxt);  // next plane's first view (the last plane: a re-read)
        reduce(cur, wcur, acc, sq);
      };
      if constexpr (NVC > 0) {
#pragma unroll
        for (int v = 0; v < NVC; v += 2) {
          step(v, ra, wa, rb, wb);
          step(v + 1, rb, wb, ra, wa);
        }
      } else {
#pragma unroll 1
        for (int v = 0; v < nv; v += 2) {
          step(v, ra, wa, rb, wb);
          step(v + 1, rb, wb, ra, wa);
        }
      }
      hyp = hyp_n;
      hyp_n = hyp_nn;
      finish(d, acc, sq);
    }
  } else {
    const int nviews = a.N;
    for (int d = d0; d < d1; ++d) {
      const float hyp = a.hyps[vox_of(d)];
      float acc[C], sq[C];
      init(acc, sq);
      for (int j = 1; j < nviews; ++j) {
        const float* m = cam + (j - 1) * 12;
        const float rx = m[0] * fx + m[1] * fy + m[2];
        const float ry = m[3] * fx + m[4] * fy + m[5];
        const float rz = m[6] * fx + m[7] * fy + m[8];
        const float qx = rx * hyp + m[9], qy = ry * hyp + m[10], qz = rz * hyp + m[11];
        const float iz = __builtin_amdgcn_rcpf(qz);
        const Taps t = bilinear_taps(a.h, a.w, rec, qx * iz * kx - 0.5f, qy * iz * ky - 0.5f);
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.feats[j], fbytes);
        uint4 rv[4 * NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            rv[q * 4 + k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, t.off[k], sb + q * qstep, 0));
        reduce(rv, t.wt, acc, sq);
      }
      finish(d, acc, sq);
    }
  }
  if constexpr (sizeof(T) == 4) amax_flush(am, a.out_amax ? a.out_amax + (size_t)b * kAmaxSlotWords : nullptr, blockIdx.x * (BLOCK / 64) + (int)(threadIdx.x >> 6));
}

// Channel-split form (NHWC maps whose pixel is S = C * sizeof(T) / 16 chunks of 16 bytes, S = 2, 4 or 8 -- 8: the
// fp32 path's 32-channel stage-1 maps, 128-byte pixels): S
// consecutive lanes share one voxel, lane q owning channel chunk q. Per (voxel, view) sample each lane issues 4
// loads (its chunk of the 4 bilinear corners) instead of 4 S, and the S lanes of a voxel read one contiguous
// 16 S-byte pixel record per corner in the SAME instruction: one L1 tag lookup per corner per voxel where the
// one-lane-per-voxel form needs S (the TA, not HBM, bounds the gather: DESIGN.md section 6). The sample
// coordinates are computed redundantly by the S lanes; the adaptive weight net's channel dot product is summed
// across them with DPP quad permutes (VALU only). The per-(plane, view) sequence is pipelined one view deep as in
// warp_aggregate_kernel (NVC > 0: view count a compile-time constant, rays hoisted; NVC < 0: runtime view loop).
__device__ __forceinline__ float dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ float swz_xor4(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x101F));  // and 0x1F, xor 4 (no LDS memory)
}

template <typename T, int C, int MODE, int NVC>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kWarpBlock))) void warp_split_kernel(const WarpArgs a, const float* __restrict__ cams,
                                                                int npix_blocks, int dchunk, int ndchunks) {
  constexpr int E = Stor<T>::E;  // channels per 16-byte chunk
  constexpr int S = C / E;       // lanes per voxel
  constexpr int PPB = kWarpBlock / S;  // pixels per block
  static_assert(S == 2 || S == 4 || S == 8, "channel-split form: 2, 4 or 8 chunks per pixel");
  static_assert(NVC % 2 == 0 || NVC < 0, "the view pipeline alternates two register sets");
  const int hw = a.h * a.w;
  const int bid = blockIdx.x;
  auto xcd_remap = [](int i, int n) {
    const int q8 = n / 8, r8 = n % 8, x = i % 8;
    return (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + i / 8;
  };
  int L = xcd_remap(bid, npix_blocks * ndchunks * a.B);
  const int dc = L % ndchunks; L /= ndchunks;
  const int pb = L % npix_blocks;
  const int b = L / npix_blocks;
  const float* __restrict__ cam = cams + (size_t)b * (a.N - 1) * 12;
  const int q = threadIdx.x & (S - 1);                // this lane's channel chunk
  const int p0 = warp_pixel(a, pb, (int)(threadIdx.x / S), PPB);  // the S lanes of a pixel are consecutive: they exit together
  // fp32: lanes past the image walk pixel 0 with their stores dropped (the magnitude reduction at the end needs every
  // lane of the wave); bf16 records no magnitude and returns
  const bool pv = p0 >= 0;
  if (sizeof(T) == 2 && !pv) return;
  const int p = pv ? p0 : 0;
  unsigned am = 0u;
  const int yl = p / a.w, x = p - yl * a.w;
  const int y = a.y0 + yl, pg = y * a.w + x;
  const float fx = (float)x, fy = (float)y;
  const float kx = (float)a.w / (float)(a.w - 1), ky = (float)a.h / (float)(a.h - 1);
  constexpr uint32_t rec = C * sizeof(T);
  const uint32_t bbytes = (uint32_t)hw * rec;
  const uint32_t sb = (uint32_t)b * bbytes;
  const uint32_t qoff = (uint32_t)q * 16u;
  const long long fbytes = (long long)a.B * bbytes;

  float ref[E];
  if (MODE != AGG_WARP_ONLY) {
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.feats[0], fbytes);
    Rec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r0, (uint32_t)pg * rec + qoff, sb, 0)),
                     ref);
  }
  float kq[E];  // this lane's chunk of the weight net's first 1x1 conv (selects, no dynamic kernarg indexing)
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float k = a.k1[e];
#pragma unroll
    for (int j = 1; j < S; ++j) k = q == j ? a.k1[j * E + e] : k;
    kq[e] = k;
  }
  const float inv_n = 1.f / (float)a.N, inv_n1 = 1.f / (float)(a.N - 1);
  const int d0 = dc * dchunk, d1 = min(a.D, d0 + dchunk);
  auto vox_of = [&](int d) { return (((size_t)b * a.D + d) * a.out_rows + a.out_y) * a.w + p; };

  auto reduce = [&](const uint4* rv, const float* wt, float* acc, float* sq) {
    float v[4][E];
#pragma unroll
    for (int k = 0; k < 4; ++k) Rec16<T>::unpack(rv[k], v[k]);
    float s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) s[e] = ((v[0][e] * wt[0] + v[1][e] * wt[1]) + v[2][e] * wt[2]) + v[3][e] * wt[3];
    if (MODE == AGG_WARP_ONLY) {
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = s[e];
    } else if (MODE == AGG_VARIANCE) {
#pragma unroll
      for (int e = 0; e < E; ++e) { acc[e] += s[e]; sq[e] += s[e] * s[e]; }
    } else {
      float dot = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float df = ref[e] - s[e];
        sq[e] = df * df;
        dot += kq[e] * sq[e];
      }
      dot += dpp_xor1(dot);
      if (S >= 4) dot += dpp_xor2(dot);
      if (S == 8) dot += swz_xor4(dot);
      const float a1 = fmaxf(dot * a.s1 + a.t1, 0.f);
      const float wv = fmaxf(a1 * a.s2 + a.t2, 0.f) + 1.f;
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += wv * sq[e];
    }
  };
  auto finish = [&](int d, float* acc, float* sq) {
    float o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (MODE == AGG_VARIANCE) {
        const float mean = acc[e] * inv_n;
        o[e] = sq[e] * inv_n - mean * mean;
      } else if (MODE == AGG_ADAPTIVE) {
        o[e] = acc[e] * inv_n1;
      } else {
        o[e] = acc[e];
      }
    }
    if constexpr (sizeof(T) == 4) {
      unsigned m = am;
#pragma unroll
      for (int e = 0; e < E; ++e) m = amax_fold(m, o[e]);
      am = pv ? m : am;
      if (pv) store_vec<T, E>(reinterpret_cast<T*>(a.out) + vox_of(d) * C + q * E, o);
    } else {
      store_vec<T, E>(reinterpret_cast<T*>(a.out) + vox_of(d) * C + q * E, o);
    }
  };
  auto init = [&](float* acc, float* sq) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      acc[e] = (MODE == AGG_VARIANCE) ? ref[e] : 0.f;
      sq[e] = (MODE == AGG_VARIANCE) ? ref[e] * ref[e] : 0.f;
    }
  };

  constexpr int NH = NVC > 0 ? NVC : 1;
  const int nv = NVC > 0 ? NVC : a.N - 1;
  float rx[NH], ry[NH], rz[NH], tx[NH], ty[NH], tz[NH];
  __amdgpu_buffer_rsrc_t rs[NH];
  if constexpr (NVC > 0) {
#pragma unroll
    for (int v = 0; v < NVC; ++v) {
      const float* m = cam + v * 12;
      rx[v] = m[0] * fx + m[1] * fy + m[2];
      ry[v] = m[3] * fx + m[4] * fy + m[5];
      rz[v] = m[6] * fx + m[7] * fy + m[8];
      tx[v] = m[9];
      ty[v] = m[10];
      tz[v] = m[11];
      rs[v] = make_rsrc(a.feats[v + 1], fbytes);
    }
  }
  auto taps = [&](int v, float hyp) {
    float qx, qy, qz;
    if constexpr (NVC > 0) {
      qx = rx[v] * hyp + tx[v], qy = ry[v] * hyp + ty[v], qz = rz[v] * hyp + tz[v];
    } else {
      const float* m = cam + v * 12;
      const float vx = m[0] * fx + m[1] * fy + m[2];
      const float vy = m[3] * fx + m[4] * fy + m[5];
      const float vz = m[6] * fx + m[7] * fy + m[8];
      qx = vx * hyp + m[9], qy = vy * hyp + m[10], qz = vz * hyp + m[11];
    }
    const float iz = __builtin_amdgcn_rcpf(qz);
    return bilinear_taps(a.h, a.w, rec, qx * iz * kx - 0.5f, qy * iz * ky - 0.5f);
  };
  auto issue = [&](int v, const Taps& t, uint4* rv, float* wt) {
    __amdgpu_buffer_rsrc_t r;
    if constexpr (NVC > 0) r = rs[v];
    else r = make_rsrc(a.feats[v + 1], fbytes);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      rv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, t.off[k] + qoff, sb, 0));
#pragma unroll
    for (int k = 0; k < 4; ++k) wt[k] = t.wt[k];
  };
  uint4 ra[4], rb[4];
  float wa[4], wb[4];
  float hyp = a.hyps[vox_of(d0)];
  float hyp_n = a.hyps[vox_of(min(d0 + 1, d1 - 1))];
  issue(0, taps(0, hyp), ra, wa);
  for (int d = d0; d < d1; ++d) {
    const float hyp_nn = a.hyps[vox_of(min(d + 2, d1 - 1))];
    float acc[E], sq[E];
    init(acc, sq);
    auto step = [&](int v, const uint4* cur, const float* wcur, uint4* nxt, float* wnxt) {
      if (v + 1 < nv) issue(v + 1, taps(v + 1, hyp), nxt, wnxt);
      else issue(0, taps(0, hyp_n), nxt, wnxt);
      reduce(cur, wcur, acc, sq);
    };
    if constexpr (NVC > 0) {
#pragma unroll
      for (int v = 0; v < NVC; v += 2) {
        step(v, ra, wa, rb, wb);
        step(v + 1, rb, wb, ra, wa);
      }
    } else {
#pragma unroll 1
      for (int v = 0; v < nv; v += 2) {
        step(v, ra, wa, rb, wb);
        step(v + 1, rb, wb, ra, wa);
      }
    }
    hyp = hyp_n;
    hyp_n = hyp_nn;
    finish(d, acc, sq);
  }
  if constexpr (sizeof(T) == 4) amax_flush(am, a.out_amax ? a.out_amax + (size_t)b * kAmaxSlotWords : nullptr, blockIdx.x * (kWarpBlock / 64) + (int)(threadIdx.x >> 6));
}

// Lanes per voxel the launcher uses for C-channel maps: the channel-split kernel for NHWC maps of 2, 4 or 8 16-byte
// chunks per pixel when the view pipeline takes the view count (odd N >= 3), else 1 (the one-lane kernel).
// DAMVS_WARP_SPLIT=0 (one lane per voxel everywhere) and DAMVS_WARP_NO_PIPE=1 (no view pipeline) both give 1, so the
// launcher's block geometry and launch_k's kernel choice follow one predicate.
bool warp_no_pipe() {
  static const bool v = [] {
    const char* e = getenv("DAMVS_WARP_NO_PIPE");
    return e && e[0] == '1';
  }();
  return v;
}
bool warp_split_enabled() {
  static const bool off = [] {
    const char* v = getenv("DAMVS_WARP_SPLIT");
    return v && v[0] == '0';
  }();
  return !off && !warp_no_pipe();
}

template <typename T, int C, bool BLK>
int split_lanes(const WarpArgs& a) {
  constexpr int S = C * (int)sizeof(T) / 16;
  return !BLK && warp_split_for(C * (int)sizeof(T), a.N) ? S : 1;
}

template <typename T, int C, int MODE, bool BLK>
void launch_k(hipStream_t s, const WarpArgs& a, dim3 grid, int npb, int dchunk, int ndc) {
  const bool no_pipe = warp_no_pipe();
  static const bool runtime_views = [] {  // DAMVS_WARP_RUNTIME_VIEWS=1: the runtime view loop for N = 5 too
    const char* v = getenv("DAMVS_WARP_RUNTIME_VIEWS");
    return v && v[0] == '1';
  }();
  if constexpr (!BLK && (C * sizeof(T) == 32 || C * sizeof(T) == 64 || C * sizeof(T) == 128)) {
    if (split_lanes<T, C, BLK>(a) > 1) {
      // N = 5: the unrolled view loop at both storage types. Its fp32 form computed wrong voxels in lanes 48-63 beside
      // another stream's U-Net kernels while the warp unit was built with packed-FP32 VALU ops; built without them
      // (build.py FILE_FLAGS) it passes every stream case and runs 2 % faster than the runtime loop (stages 1-3: 0.520 /
      // 0.749 / 0.535 against 0.532 / 0.766 / 0.548 ms, profiles/r05/diag_streams/r05y; DESIGN.md section 4
      // "Concurrent streams")
      if (a.N == 5 && !runtime_views)
        hipLaunchKernelGGL((warp_split_kernel<T, C, MODE, 4>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
      // N = 7 (cfgD) unrolled too, except the fp32 8-channel maps: cfgD B=4 stages 1 / 2 bf16 2.392 / 2.462 -> 2.293 /
      // 2.393 ms, fp32 3.525 / 4.240 -> 3.438 / 4.041 ms; fp32 stage 3 3.174 -> 3.233 ms stays on the runtime loop
      // (profiles/r05/ab_warp_n7)
      else if (a.N == 7 && !runtime_views && !(sizeof(T) == 4 && C == 8))
        hipLaunchKernelGGL((warp_split_kernel<T, C, MODE, (sizeof(T) == 4 && C == 8) ? 4 : 6>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
      else
        hipLaunchKernelGGL((warp_split_kernel<T, C, MODE, -1>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
      return;
    }
  }
  // view pipeline: unrolled for N = 5 (the DTU default) at 16 channels (stage 2; A/B: 2.29 against 2.37 ms, while
  // stage 3 runs 1.47 against 1.50 ms on the runtime loop), a runtime view loop for any other odd
  // N (7, 11: the cfgD / cfgE benchmark configs; 3) and for 32 channels (the unrolled form needs 360 registers)
  const bool pipe = !no_pipe && a.N >= 3 && (a.N - 1) % 2 == 0;
  if constexpr (C == 16) {
    if (pipe && a.N == 5 && !runtime_views) {
      hipLaunchKernelGGL((warp_aggregate_kernel<T, C, MODE, BLK, 4>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
      return;
    }
  }
  if (pipe)
    hipLaunchKernelGGL((warp_aggregate_kernel<T, C, MODE, BLK, -1>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
  else
    hipLaunchKernelGGL((warp_aggregate_kernel<T, C, MODE, BLK, 0>), grid, dim3(kWarpBlock), 0, s, a, a.rt, npb, dchunk, ndc);
}

template <typename T, int MODE, bool BLK>
hipError_t launch_c(hipStream_t s, const WarpArgs& a0) {
  WarpArgs a = a0;
  // 32-bit buffer offsets: each view's feature tensor must stay below 2 GiB
  if ((long long)a.B * a.h * a.w * a.C * (long long)sizeof(T) >= (1LL << 31)) return hipErrorInvalidValue;
  // lanes per voxel and block size of the kernel launch_k will pick (pixels per block = block / lanes)
  int lanes = 1, block = 256;
  auto pick = [&](auto cc) {
    constexpr int CC = decltype(cc)::value;
    lanes = split_lanes<T, CC, BLK>(a);
    block = kWarpBlock;
  };
  switch (a.C) {
    case 8: pick(IntC<8>()); break;
    case 16: pick(IntC<16>()); break;
    case 32: pick(IntC<32>()); break;
  }
  const int ppb = block / lanes;
  // Pixel blocks as R-row tiles (R divides ppb) dealt across the full width, or in strips SW pixels wide:
  // DAMVS_WARP_TILE="R,SW", default R = 8; "0": ppb consecutive pixels of the row-major computed rows. The
  // 8-row tiles keep vertically adjacent pixels, whose bilinear footprints share source rows, on one CU: stage-2
  // L1 -> L2 requests -19 % and L2 hit 0.62 -> 0.71 already at 4 rows (profiles/r03/pmc_l2_tile.json); in the
  // pipeline (B=4) stage 3 1.48 -> 1.24 ms, stage 2 2.00 -> 1.82 ms, stage 1 1.40 -> 1.31 ms; 16 / 32 / 64 rows
  // slower again (profiles/r03/ab_warp_tile.jsonl).
  static const int tile_env[2] = {[] {
                                    const char* e = getenv("DAMVS_WARP_TILE");
                                    return e ? atoi(e) : 8;
                                  }(),
                                  [] {
                                    const char* e = getenv("DAMVS_WARP_TILE");
                                    const char* c = e ? strchr(e, ',') : nullptr;
                                    return c ? atoi(c + 1) : 0;
                                  }()};
  a.tile_r = 0;
  int npb = (a.rows * a.w + ppb - 1) / ppb;
  if (tile_env[0] > 0 && ppb % tile_env[0] == 0) {
    const int tc = ppb / tile_env[0];
    a.tile_r = tile_env[0];
    a.tiles_x = (a.w + tc - 1) / tc;
    a.tile_sw = tile_env[1] >= tc ? std::min(a.tiles_x, tile_env[1] / tc) : a.tiles_x;
    npb = a.tiles_x * ((a.rows + a.tile_r - 1) / a.tile_r);
  }
  // depth chunk: as long as possible (locality) while keeping >= ~4 blocks per CU in flight
  int dchunk = a.D;
  // (in 256-thread blocks: 512 - 32768 measured flat within 3 %, 16384+ slower in the pipeline)
  const long long minblk = 2048LL * 256 / block;
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

// [N views][B][h][w][C] -> [B][C/E][h][w][E] per view. One thread per pixel: it reads the pixel's NQ
// consecutive 16-byte chunks (one contiguous C-vector) and writes chunk q to plane q, so both the reads and
// each plane's writes are contiguous across the wave; blockIdx.y = view * B + batch element (no division).
template <int NQ>
__global__ __launch_bounds__(256) void block_channels_kernel(const FeatPtrs src, FeatPtrs dst, int B, int hw) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= hw) return;
  const int v = blockIdx.y / B, b = blockIdx.y - v * B;
  // the view's pointers by a select chain (indexing the by-value pointer arrays with v would copy them to scratch)
  const void* sv = src.p[0];
  const void* dv = dst.p[0];
#pragma unroll
  for (int i = 1; i < kMaxViews; ++i) {
    sv = v == i ? src.p[i] : sv;
    dv = v == i ? dst.p[i] : dv;
  }
  const uint4* sp = reinterpret_cast<const uint4*>(sv) + ((size_t)b * hw + p) * NQ;
  uint4* dp = const_cast<uint4*>(reinterpret_cast<const uint4*>(dv)) + (size_t)b * NQ * hw + p;
  // groups of at most 4 chunks: a register array of 6-8 uint4 was kept in scratch by hipcc
#pragma unroll
  for (int q0 = 0; q0 < NQ; q0 += 4) {
    constexpr int G = NQ < 4 ? NQ : 4;
    uint4 r[G];
#pragma unroll
    for (int q = 0; q < G; ++q)
      if (q0 + q < NQ) r[q] = sp[q0 + q];
#pragma unroll
    for (int q = 0; q < G; ++q)
      if (q0 + q < NQ) dp[(size_t)(q0 + q) * hw] = r[q];
  }
}

}  // namespace

// Whether launch_warp_aggregate runs the channel-split kernel for NHWC maps of `bytes`-byte pixels at N views (the
// predicate split_lanes applies per launch; capi's feature-layout choice asks it before the maps are laid out).
bool warp_split_for(int bytes, int N) {
  return warp_split_enabled() && (bytes == 32 || bytes == 64 || bytes == 128) && N >= 3 && (N - 1) % 2 == 0;
}

hipError_t launch_warp_aggregate(hipStream_t s, int store, int mode, const WarpArgs& a, bool blocked) {
  if (blocked) return store == ST_BF16 ? launch_t<bf16_t, true>(s, mode, a) : launch_t<float, true>(s, mode, a);
  return store == ST_BF16 ? launch_t<bf16_t, false>(s, mode, a) : launch_t<float, false>(s, mode, a);
}

hipError_t launch_block_channels(hipStream_t s, int store, const FeatPtrs& src, const FeatPtrs& dst, int N, int B,
                                 int hw, int C) {
  const int nq = C / (store == ST_BF16 ? 8 : 4);
  dim3 grid((unsigned)((hw + 255) / 256), (unsigned)(N * B));
  switch (nq) {
    case 1: hipLaunchKernelGGL(block_channels_kernel<1>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 2: hipLaunchKernelGGL(block_channels_kernel<2>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 3: hipLaunchKernelGGL(block_channels_kernel<3>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 4: hipLaunchKernelGGL(block_channels_kernel<4>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 5: hipLaunchKernelGGL(block_channels_kernel<5>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 6: hipLaunchKernelGGL(block_channels_kernel<6>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 7: hipLaunchKernelGGL(block_channels_kernel<7>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    case 8: hipLaunchKernelGGL(block_channels_kernel<8>, grid, dim3(256), 0, s, src, dst, B, hw); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace damvs
