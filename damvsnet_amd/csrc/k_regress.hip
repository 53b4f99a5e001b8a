// Final probability conv + depth regression.
//
//  prob_conv : CostRegNet.prob, Conv3d(base, 1, k3, p1, bias=False) (models/module.py:530,540).
//              One thread per pixel column (b, y, x) slides over the D planes: each input plane's
//              3x3 x Cb neighbourhood is loaded once and contributes to logits d-1, d, d+1
//              (3x fewer loads than a per-output gather). Optional prob_volume_init is added
//              (models/cas_mvsnet.py:107-108).
//  regress   : softmax over D (:110), depth = sum p*d (module.py:609-615), photometric
//              confidence = sum of p over [i*-1, i*+2] at i* = clamp(long(sum p*i), 0, D-1)
//              (:113-118, the 4*avg_pool3d of the padded volume), exp-variance
//              3*sqrt(sum (d - depth)^2 p) (:121-124); optional prob volume write.
#include <cstdlib>
#include <type_traits>

#include "damvs_device.h"

namespace damvs {

namespace {

template <typename T, int CB>
__global__ __launch_bounds__(256) void prob_conv_kernel(int B, int D, int h, int w, const T* __restrict__ feat,
                                                        const float* __restrict__ wprob,
                                                        const float* __restrict__ prob_init,
                                                        float* __restrict__ logits) {
  const float* sw = wprob;  // [kd][kh][kw][c], wave-uniform -> scalar loads
  const int hw = h * w;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= hw) return;
  const int y = p / w, x = p - y * w;
  float am1 = 0.f, a0 = 0.f;  // partial logits for d = plane-1 (after this plane) and d = plane+1
  for (int pl = 0; pl < D; ++pl) {
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;  // kd = 0 -> d = pl+1, kd = 1 -> d = pl, kd = 2 -> d = pl-1
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = y + ky - 1;
      if (yy < 0 || yy >= h) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = x + kx - 1;
        if (xx < 0 || xx >= w) continue;
        float v[CB];
        load_vec<T, CB>(feat + ((((size_t)b * D + pl) * h + yy) * w + xx) * CB, v);
        // wave-uniform weights through the scalar cache (SGPR operands of v_fmac)
        const float* w0 = wprob + ((0 * 3 + ky) * 3 + kx) * CB;
        const float* w1 = wprob + ((1 * 3 + ky) * 3 + kx) * CB;
        const float* w2 = wprob + ((2 * 3 + ky) * 3 + kx) * CB;
#pragma unroll
        for (int c = 0; c < CB; ++c) {
          c0 += w0[c] * v[c];
          c1 += w1[c] * v[c];
          c2 += w2[c] * v[c];
        }
      }
    }
    float* lo = logits + ((size_t)b * D) * hw + p;
    if (pl >= 1) {
      float l = am1 + c2;
      if (prob_init) l += prob_init[((size_t)b * D + pl - 1) * hw + p];
      lo[(size_t)(pl - 1) * hw] = l;
    }
    am1 = a0 + c1;
    a0 = c0;
  }
  float l = am1;
  if (prob_init) l += prob_init[((size_t)b * D + D - 1) * hw + p];
  logits[((size_t)b * D + D - 1) * hw + p] = l;
}

__global__ __launch_bounds__(256) void regress_kernel(int B, int D, int hw, const float* __restrict__ logits,
                                                      const float* __restrict__ hyps, float* __restrict__ depth,
                                                      float* __restrict__ conf, float* __restrict__ var,
                                                      float* __restrict__ prob) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= hw) return;
  const float* lg = logits + (size_t)b * D * hw + p;
  const float* hy = hyps + (size_t)b * D * hw + p;
  float mx = -INFINITY;
  for (int d = 0; d < D; ++d) mx = fmaxf(mx, lg[(size_t)d * hw]);
  float sum = 0.f;
  for (int d = 0; d < D; ++d) sum += expf(lg[(size_t)d * hw] - mx);
  float dep = 0.f, idx = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = expf(lg[(size_t)d * hw] - mx) / sum;
    dep += pr * hy[(size_t)d * hw];
    idx += pr * (float)d;
    if (prob) prob[((size_t)b * D + d) * hw + p] = pr;
  }
  int ii = (int)idx;  // .long() truncation; idx >= 0
  ii = ii < 0 ? 0 : (ii > D - 1 ? D - 1 : ii);
  float c = 0.f, vs = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = expf(lg[(size_t)d * hw] - mx) / sum;
    const float df = hy[(size_t)d * hw] - dep;
    vs += df * df * pr;
    if (d >= ii - 1 && d <= ii + 2) c += pr;
  }
  depth[(size_t)b * hw + p] = dep;
  conf[(size_t)b * hw + p] = c;
  var[(size_t)b * hw + p] = 3.f * sqrtf(vs);
}

// Fused prob conv + regression. One 256-thread block owns an 8 x 32 pixel tile for all D planes:
// each input plane's (8+2) x (32+2) x Cb halo tile is staged once in LDS as fp32 (double-buffered, one
// barrier per plane, next plane's global loads issued before this plane's FMAs; bf16 is widened once
// per voxel at staging, not once per tap), every thread slides its 3x3x3 window over the planes keeping
// the two open logits in registers, completed logits go to an LDS column [D][256] and the regression
// runs from there. Logits never reach HBM. The channel sums run as packed fp32 FMAs (even / odd channel
// partial sums, added at the end of the plane) with the 72 weights of one kernel row as scalar operands
// (the ky loop is not unrolled: all 216 weights at once would spill to VGPR lanes).
constexpr int kTY = 8, kTX = 32, kHY = kTY + 2, kHX = kTX + 2;
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// TWO: first pass of the two-pass form — the same LDS-tiled prob conv, logits (+prob_init) written
// to HBM ([B][D][h][w], argument `prob`) for regress_kernel; LDS then holds only the plane tiles, so
// 3x more blocks share a CU than with the D-deep logit column.
template <typename T, int CB, bool TWO>
__global__ __launch_bounds__(256) void prob_regress_kernel(int B, int D, int h, int w, const T* __restrict__ feat,
                                                           const float* __restrict__ wprob,
                                                           const float* __restrict__ prob_init,
                                                           const float* __restrict__ hyps, float* __restrict__ depth,
                                                           float* __restrict__ conf, float* __restrict__ var,
                                                           float* __restrict__ prob) {
  constexpr int E = Stor<T>::E;
  constexpr int CH = CB / E;                 // 16-byte storage chunks per voxel
  constexpr int NVOX = kHY * kHX;
  constexpr int TILE_CHUNKS = NVOX * CH;
  constexpr int PER_T = (TILE_CHUNKS + 255) / 256;
  constexpr int FQ = CB / 4;                 // fp32 quads per voxel in LDS, quad-major ([FQ][NVOX]):
                                             // 16 consecutive pixels read 16 consecutive quads
  typedef typename std::conditional<sizeof(T) == 4, float4, uint4>::type raw;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float4* tile = reinterpret_cast<float4*>(smem);               // 2 x FQ x NVOX (double buffer)
  // [D - 1][256] logits, column per thread; the last plane's logit stays in a register: at D = 32 that 1 KB
  // is what lets a third block onto the CU (2 x 21.3 KB tiles + 31 KB column = 52.3 KB)
  float* lg = reinterpret_cast<float*>(tile + 2 * FQ * NVOX);

  const int tid = threadIdx.x;
  const int ty = tid / kTX, tx = tid % kTX;
  const int y0 = blockIdx.y * kTY, x0 = blockIdx.x * kTX;
  const int b = blockIdx.z;
  const T* fb = feat + (size_t)b * D * h * w * CB;
  raw regs[PER_T];
  auto gload = [&](int pl) {
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      const int c = tid + k * 256;
      raw v;
      if constexpr (sizeof(T) == 4) v = make_float4(0.f, 0.f, 0.f, 0.f); else v = make_uint4(0u, 0u, 0u, 0u);
      if (c < TILE_CHUNKS) {
        const int vox = c / CH, part = c % CH;
        const int yy = y0 - 1 + vox / kHX, xx = x0 - 1 + vox % kHX;
        if (yy >= 0 && yy < h && xx >= 0 && xx < w)
          v = *reinterpret_cast<const raw*>(fb + (((size_t)pl * h + yy) * w + xx) * CB + part * E);
      }
      regs[k] = v;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      const int c = tid + k * 256;
      if (c < TILE_CHUNKS) {
        const int vox = c / CH, part = c % CH;
        float4* dst = tile + buf * FQ * NVOX + part * (E / 4) * NVOX + vox;
        if constexpr (sizeof(T) == 4) {
          dst[0] = regs[k];
        } else {
          const uint4 r = regs[k];
          dst[0] = make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                               __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u));
          dst[NVOX] = make_float4(__uint_as_float(r.z << 16), __uint_as_float(r.z & 0xffff0000u),
                                  __uint_as_float(r.w << 16), __uint_as_float(r.w & 0xffff0000u));
        }
      }
    }
  };

  gload(0);
  lstore(0);
  __syncthreads();
  float am1 = 0.f, a0 = 0.f;
  for (int pl = 0; pl < D; ++pl) {
    if (pl + 1 < D) gload(pl + 1);
    const float4* tb = tile + (pl & 1) * FQ * NVOX + ty * kHX + tx;
    f32x2_t c0 = {0.f, 0.f}, c1 = {0.f, 0.f}, c2 = {0.f, 0.f};
#pragma unroll 1
    for (int ky = 0; ky < 3; ++ky) {
      // wave-uniform weights through the scalar cache (SGPR operands), one kernel row per iteration
      const float* wr = wprob + ky * 3 * CB;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float v[CB];
#pragma unroll
        for (int q = 0; q < FQ; ++q) {
          const float4 f = tb[q * NVOX + ky * kHX + kx];
          v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
        }
        const float* w0 = wr + kx * CB;           // dz = 0: w[((dz * 3 + ky) * 3 + kx) * CB + c]
        const float* w1 = wr + 9 * CB + kx * CB;  // dz = 1
        const float* w2 = wr + 18 * CB + kx * CB; // dz = 2
#pragma unroll
        for (int c = 0; c < CB; c += 2) {
          const f32x2_t x = {v[c], v[c + 1]};
          c0 += (f32x2_t){w0[c], w0[c + 1]} * x;
          c1 += (f32x2_t){w1[c], w1[c + 1]} * x;
          c2 += (f32x2_t){w2[c], w2[c + 1]} * x;
        }
      }
    }
    const float s0 = c0.x + c0.y, s1 = c1.x + c1.y, s2 = c2.x + c2.y;
    if (TWO) {
      const int y = y0 + ty, x = x0 + tx;
      if (pl >= 1 && y < h && x < w) {
        const size_t o = (((size_t)b * D + pl - 1) * h + y) * w + x;
        prob[o] = am1 + s2 + (prob_init ? prob_init[o] : 0.f);
      }
    } else if (pl >= 1) {
      lg[(pl - 1) * 256 + tid] = am1 + s2;
    }
    am1 = a0 + s1;
    a0 = s0;
    if (pl + 1 < D) lstore((pl + 1) & 1);
    __syncthreads();
  }
  if (TWO) {
    const int y = y0 + ty, x = x0 + tx;
    if (y < h && x < w) {
      const size_t o = (((size_t)b * D + D - 1) * h + y) * w + x;
      prob[o] = am1 + (prob_init ? prob_init[o] : 0.f);
    }
    return;
  }
  float last = am1;  // plane D - 1

  const int y = y0 + ty, x = x0 + tx;
  if (y >= h || x >= w) return;
  const size_t hw = (size_t)h * w, pix = (size_t)y * w + x;
  const float* hy = hyps + (size_t)b * D * hw + pix;
  const float* pin = prob_init ? prob_init + (size_t)b * D * hw + pix : nullptr;
  float* lcol = lg + tid;
  auto col = [&](int d) -> float& { return d == D - 1 ? last : lcol[d * 256]; };
  if (pin)
    for (int d = 0; d < D; ++d) col(d) += pin[(size_t)d * hw];
  float mx = -INFINITY;
  for (int d = 0; d < D; ++d) mx = fmaxf(mx, col(d));
  float sum = 0.f;
  for (int d = 0; d < D; ++d) {
    const float e = expf(col(d) - mx);
    col(d) = e;
    sum += e;
  }
  float dep = 0.f, idx = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = col(d) / sum;
    col(d) = pr;
    dep += pr * hy[(size_t)d * hw];
    idx += pr * (float)d;
  }
  int ii = (int)idx;
  ii = ii < 0 ? 0 : (ii > D - 1 ? D - 1 : ii);
  float c = 0.f, vs = 0.f;
  float* po = prob ? prob + (size_t)b * D * hw + pix : nullptr;
  for (int d = 0; d < D; ++d) {
    const float pr = col(d);
    const float df = hy[(size_t)d * hw] - dep;
    vs += df * df * pr;
    if (d >= ii - 1 && d <= ii + 2) c += pr;
    if (po) po[(size_t)d * hw] = pr;
  }
  depth[(size_t)b * hw + pix] = dep;
  conf[(size_t)b * hw + pix] = c;
  var[(size_t)b * hw + pix] = 3.f * sqrtf(vs);
}

// Prob conv on MFMA (bf16 storage, 8 channels). Cout = 1 would leave 15 of 16 MFMA rows empty, so
// the rows are 16 consecutive OUTPUT PLANES instead: with K = (input plane r = 0..17 relative to
// d0 - 1, ky, kx, channel), the 16 x K operand is the banded weight matrix W[r - m] (capi.cpp,
// pack_prob_banded; fp32 weights as bf16 hi + lo, two MFMAs per chunk). Lane group g of a B
// fragment is one tap = one 16-byte voxel (8 channels), so every B load is a coalesced 16-pixel row
// segment. Wave w owns planes [16w, 16w+16) of a 64-pixel row segment (4 N-tiles reuse each A
// fragment); the D logits of the block's 64 pixels meet in LDS and 64 threads run the regression.
constexpr int kPR = 4;  // 16-pixel N-tiles per wave

__global__ __launch_bounds__(256) void prob_mfma_kernel(int B, int D, int h, int w, int tiles_x,
                                                        const bf16_t* __restrict__ feat, const uint4* __restrict__ apack,
                                                        const float* __restrict__ prob_init,
                                                        const float* __restrict__ hyps, float* __restrict__ depth,
                                                        float* __restrict__ conf, float* __restrict__ var,
                                                        float* __restrict__ prob) {
  __shared__ float lg[64 * 64];  // [plane][pixel of the block]
  const int tx = blockIdx.x % tiles_x, yb = blockIdx.x / tiles_x;
  const int y = yb % h, b = yb / h;
  const int x0 = tx * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int d0 = wave * 16;
  const __amdgpu_buffer_rsrc_t rf = make_rsrc(feat, (long long)B * D * h * w * 8 * 2);
  const uint4* ap = apack + lane;
  f32x4_t acc[kPR];
#pragma unroll
  for (int r = 0; r < kPR; ++r) acc[r] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  auto fetch = [&](int s, uint4& ah, uint4& al, uint4* xb) {
    ah = ap[(size_t)(2 * s) * 64];
    al = ap[(size_t)(2 * s + 1) * 64];
    const int tp = s * 4 + g;  // this lane group's tap
    const int rr = tp / 9, t9 = tp - rr * 9;
    const int iz = d0 - 1 + rr, yy = y + t9 / 3 - 1, dx = t9 % 3 - 1;
    const bool okz = tp < 18 * 9 && (unsigned)iz < (unsigned)D && (unsigned)yy < (unsigned)h;
    const int rowbase = ((b * D + iz) * h + yy) * w;
#pragma unroll
    for (int r = 0; r < kPR; ++r) {
      const int xx = x0 + r * 16 + n + dx;
      const bool ok = okz && (unsigned)xx < (unsigned)w;
      xb[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rf, ok ? (uint32_t)(rowbase + xx) * 16u : kOOB, 0, 0));
    }
  };
  // only input planes d0 - 1 .. min(d0 + 16, D - 1) exist: skip the chunks past them (D = 8: 21 of 41)
  const int nplanes = min(18, D - d0 + 1);
  const int nch = min(kProbChunks, (nplanes * 9 + 3) / 4);
  uint4 ah, al, xb[kPR];
  fetch(0, ah, al, xb);
  for (int s = 0; s < nch; ++s) {
    uint4 nh, nl, nb[kPR];
    if (s + 1 < nch) fetch(s + 1, nh, nl, nb);
#pragma unroll
    for (int r = 0; r < kPR; ++r) {
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ah), __builtin_bit_cast(bf16x8_t, xb[r]),
                                                       acc[r], 0, 0, 0);
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, al), __builtin_bit_cast(bf16x8_t, xb[r]),
                                                       acc[r], 0, 0, 0);
    }
    if (s + 1 < nch) {
      ah = nh;
      al = nl;
#pragma unroll
      for (int r = 0; r < kPR; ++r) xb[r] = nb[r];
    }
  }
  // lane (n, g) holds planes d0 + 4g .. +3 of pixel r * 16 + n
  const size_t hw = (size_t)h * w;
#pragma unroll
  for (int r = 0; r < kPR; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = d0 + 4 * g + i, px = r * 16 + n, x = x0 + px;
      if (d < D) {
        float l = acc[r][i];
        if (prob_init && x < w) l += prob_init[((size_t)b * D + d) * hw + (size_t)y * w + x];
        lg[d * 64 + px] = l;
      }
    }
  __syncthreads();
  const int t = threadIdx.x, x = x0 + t;
  if (t >= 64 || x >= w) return;
  const size_t pix = (size_t)y * w + x;
  const float* hy = hyps + (size_t)b * D * hw + pix;
  float* lcol = lg + t;
  float mx = -INFINITY;
  for (int d = 0; d < D; ++d) mx = fmaxf(mx, lcol[d * 64]);
  float sum = 0.f;
  for (int d = 0; d < D; ++d) {
    const float e = expf(lcol[d * 64] - mx);
    lcol[d * 64] = e;
    sum += e;
  }
  float dep = 0.f, idx = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = lcol[d * 64] / sum;
    lcol[d * 64] = pr;
    dep += pr * hy[(size_t)d * hw];
    idx += pr * (float)d;
  }
  int ii = (int)idx;
  ii = ii < 0 ? 0 : (ii > D - 1 ? D - 1 : ii);
  float c = 0.f, vs = 0.f;
  float* po = prob ? prob + (size_t)b * D * hw + pix : nullptr;
  for (int d = 0; d < D; ++d) {
    const float pr = lcol[d * 64];
    const float df = hy[(size_t)d * hw] - dep;
    vs += df * df * pr;
    if (d >= ii - 1 && d <= ii + 2) c += pr;
    if (po) po[(size_t)d * hw] = pr;
  }
  depth[(size_t)b * hw + pix] = dep;
  conf[(size_t)b * hw + pix] = c;
  var[(size_t)b * hw + pix] = 3.f * sqrtf(vs);
}

template <typename T, int CB>
size_t prob_regress_smem(int D) {
  return 2 * (size_t)kHY * kHX * CB * 4 + (size_t)(D > 0 ? D - 1 : 0) * 256 * 4;  // fp32 plane tiles + logit column
}

template <typename T, int CB>
hipError_t launch_pr_t(hipStream_t s, int B, int D, int h, int w, const void* feat, const float* wprob,
                       const float* prob_init, const float* hyps, float* depth, float* conf, float* var, float* prob) {
  const size_t smem = prob_regress_smem<T, CB>(D);
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  auto k = prob_regress_kernel<T, CB, false>;
  if (smem > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
  }
  dim3 grid((w + kTX - 1) / kTX, (h + kTY - 1) / kTY, B);
  hipLaunchKernelGGL(k, grid, dim3(256), smem, s, B, D, h, w, reinterpret_cast<const T*>(feat), wprob, prob_init, hyps,
                     depth, conf, var, prob);
  return hipGetLastError();
}

template <typename T, int CB>
hipError_t launch_pc_lds(hipStream_t s, int B, int D, int h, int w, const void* feat, const float* wprob,
                         const float* prob_init, float* logits) {
  const size_t smem = prob_regress_smem<T, CB>(0);
  dim3 grid((w + kTX - 1) / kTX, (h + kTY - 1) / kTY, B);
  hipLaunchKernelGGL((prob_regress_kernel<T, CB, true>), grid, dim3(256), smem, s, B, D, h, w,
                     reinterpret_cast<const T*>(feat), wprob, prob_init, nullptr, nullptr, nullptr, nullptr, logits);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pc(hipStream_t s, int B, int Cb, int D, int h, int w, const void* feat, const float* wprob,
                     const float* prob_init, float* logits) {
  if (Cb == 8) return launch_pc_lds<T, 8>(s, B, D, h, w, feat, wprob, prob_init, logits);
  if (Cb == 16) return launch_pc_lds<T, 16>(s, B, D, h, w, feat, wprob, prob_init, logits);
  dim3 grid((h * w + 255) / 256, B);
  const T* f = reinterpret_cast<const T*>(feat);
  switch (Cb) {
    case 8: hipLaunchKernelGGL((prob_conv_kernel<T, 8>), grid, dim3(256), 0, s, B, D, h, w, f, wprob, prob_init, logits); break;
    case 16: hipLaunchKernelGGL((prob_conv_kernel<T, 16>), grid, dim3(256), 0, s, B, D, h, w, f, wprob, prob_init, logits); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_prob_conv(hipStream_t s, int store, int B, int Cb, int D, int h, int w, const void* feat,
                            const float* wprob, const float* prob_init, float* logits) {
  return store == ST_BF16 ? launch_pc<bf16_t>(s, B, Cb, D, h, w, feat, wprob, prob_init, logits)
                          : launch_pc<float>(s, B, Cb, D, h, w, feat, wprob, prob_init, logits);
}

hipError_t launch_prob_regress(hipStream_t s, int store, int B, int Cb, int D, int h, int w, const void* feat,
                               const float* wprob, const float* prob_init, const float* hyps, float* depth,
                               float* conf, float* var, float* prob) {
  if (Cb == 8)
    return store == ST_BF16 ? launch_pr_t<bf16_t, 8>(s, B, D, h, w, feat, wprob, prob_init, hyps, depth, conf, var, prob)
                            : launch_pr_t<float, 8>(s, B, D, h, w, feat, wprob, prob_init, hyps, depth, conf, var, prob);
  if (Cb == 16)
    return store == ST_BF16 ? launch_pr_t<bf16_t, 16>(s, B, D, h, w, feat, wprob, prob_init, hyps, depth, conf, var, prob)
                            : launch_pr_t<float, 16>(s, B, D, h, w, feat, wprob, prob_init, hyps, depth, conf, var, prob);
  return hipErrorInvalidValue;
}

size_t prob_regress_smem_bytes(int store, int Cb, int D) {
  static const bool two_pass = [] {  // measured slower at cfgC (A/B knob)
    const char* v = getenv("DAMVS_PROBREG_TWOPASS");
    return v && v[0] == '1';
  }();
  if (two_pass) return (size_t)-1;  // the caller takes the two-pass form
  if (Cb == 8) return store == ST_BF16 ? prob_regress_smem<bf16_t, 8>(D) : prob_regress_smem<float, 8>(D);
  return store == ST_BF16 ? prob_regress_smem<bf16_t, 16>(D) : prob_regress_smem<float, 16>(D);
}

hipError_t launch_regress(hipStream_t s, int B, int D, int h, int w, const float* logits, const float* hyps,
                          float* depth, float* conf, float* var, float* prob) {
  int hw = h * w;
  hipLaunchKernelGGL(regress_kernel, dim3((hw + 255) / 256, B), dim3(256), 0, s, B, D, hw, logits, hyps, depth, conf,
                     var, prob);
  return hipGetLastError();
}

}  // namespace damvs

namespace damvs {

hipError_t launch_prob_mfma(hipStream_t s, int B, int D, int h, int w, const void* feat, const void* apack,
                            const float* prob_init, const float* hyps, float* depth, float* conf, float* var,
                            float* prob) {
  if (D < 1 || D > 64) return hipErrorInvalidValue;
  if ((long long)B * D * h * w * 16 >= (1LL << 32)) return hipErrorInvalidValue;  // 32-bit buffer offsets
  const int tiles_x = (w + 63) / 64, ngroups = (D + 15) / 16;
  const long long nblk = (long long)tiles_x * h * B;
  hipLaunchKernelGGL(prob_mfma_kernel, dim3((unsigned)nblk), dim3(64 * ngroups), 0, s, B, D, h, w, tiles_x,
                     reinterpret_cast<const bf16_t*>(feat), reinterpret_cast<const uint4*>(apack), prob_init, hyps,
                     depth, conf, var, prob);
  return hipGetLastError();
}

// The banded-MFMA prob conv runs only with DAMVS_PROB_MFMA=1 (read per call: tests flip it): since the
// VALU prob_regress widens its tiles once per voxel and runs packed FMAs it is as fast at D = 32-48
// (stage-1/2 forwards 2.93 / 4.92 ms against 2.99 / 5.01 at B=4) and keeps the exact fp32 weights.
bool prob_mfma_disabled() {
  const char* v = getenv("DAMVS_PROB_MFMA");
  return !(v && v[0] == '1');
}

}  // namespace damvs
