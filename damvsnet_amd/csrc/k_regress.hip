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

#include <algorithm>

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
// runs from there. Logits never reach HBM. The channel sums run as fp32 FMAs (even / odd channel partial sums, added
// at the end of the plane; packed FMAs until round 6, the same operations) with the 72 weights of one kernel row as
// scalar operands
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
  // this thread's staged chunks: byte offset inside a plane (kOOB: outside the image or past the tile), the same for every
  // plane; buffer loads over the sample's volume return zeros for kOOB (no branch, no 64-bit address math per plane)
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(feat + (size_t)b * D * h * w * CB, (long long)D * h * w * CB * sizeof(T));
  const uint32_t pstride = (uint32_t)(h * w * CB * sizeof(T));
  uint32_t voff[PER_T];
#pragma unroll
  for (int k = 0; k < PER_T; ++k) {
    const int c = tid + k * 256;
    const int vox = c / CH, part = c % CH;
    const int yy = y0 - 1 + vox / kHX, xx = x0 - 1 + vox % kHX;
    const bool ok = c < TILE_CHUNKS && yy >= 0 && yy < h && xx >= 0 && xx < w;
    voff[k] = ok ? (uint32_t)(((yy * w + xx) * CB + part * E) * sizeof(T)) : kOOB;
  }
  raw regs[PER_T];
  auto gload = [&](int pl, raw (&regs)[PER_T]) {
#pragma unroll
    for (int k = 0; k < PER_T; ++k)
      regs[k] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(
                                            rv, voff[k] == kOOB ? kOOB : voff[k] + (uint32_t)pl * pstride, 0, 0));
  };
  auto lstore = [&](int buf, const raw (&regs)[PER_T]) {
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

  float am1 = 0.f, a0 = 0.f;
  // plane pl's conv from LDS buffer pl & 1, plane pl + 1 loaded meanwhile (two planes ahead measured flat at fp32:
  // profiles/r06/ab_prob_r06q)
  gload(0, regs);
  lstore(0, regs);
  __syncthreads();
  for (int pl = 0; pl < D; ++pl) {
    if (pl + 1 < D) gload(pl + 1, regs);
    const float4* tb = tile + (pl & 1) * FQ * NVOX + ty * kHX + tx;
    // even / odd channel partial sums per kernel depth (scalar FMAs: k_regress.hip is built without packed-FP32 ops)
    float c0e = 0.f, c0o = 0.f, c1e = 0.f, c1o = 0.f, c2e = 0.f, c2o = 0.f;
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
          c0e += w0[c] * v[c];
          c0o += w0[c + 1] * v[c + 1];
          c1e += w1[c] * v[c];
          c1o += w1[c + 1] * v[c + 1];
          c2e += w2[c] * v[c];
          c2o += w2[c + 1] * v[c + 1];
        }
      }
    }
    const float s0 = c0e + c0o, s1 = c1e + c1o, s2 = c2e + c2o;
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
    if (pl + 1 < D) lstore((pl + 1) & 1, regs);
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

// Prob conv on MFMA + regression (bf16 storage, 8 channels). A block owns an 8 x 32 pixel tile for all D planes,
// as prob_regress_kernel, but each input plane's (8+2) x (32+2) halo is staged in LDS as the raw 16-byte bf16
// voxels (no widening) and the conv runs on the matrix cores. Wave w computes rows 4(w>>1) .. +3 x columns
// 16(w&1) .. +15 of the tile as one 16 x 16 output tile per plane:
//   columns n   = 16 pixels of a row,
//   rows m      = 4 j + dz: pixel row j (0..3) of the wave, kernel depth dz (0..2; m & 3 == 3 stays zero),
//   K           = 18 voxel slots (input row r = 0..5 relative to the wave's first row - 1, kx) x 8 channels,
//                 5 chunks of 32 (slots 18, 19 are zero weights),
//   A[m][r,kx,c] = W[c][dz][ky = r - j][kx] when 0 <= ky <= 2 (pack_prob_rows, capi.cpp).
// Lane group g of a B fragment is one slot = one 16-byte voxel read from LDS (16 lanes: 256 contiguous bytes).
// The fp32 weights enter as two bf16 terms (hi + lo: ~16 mantissa bits, a relative weight error below 2^-17, far
// under the 2^-9 rounding of the bf16 activations they multiply; bf16 x bf16 products are exact). Three terms
// (DAMVS_PROB_TERMS=3: 24 bits, the fp32 conv up to summation order) cost the kernel its fourth wave per SIMD:
// stage 3 0.50 against 0.42 ms at B=4 (tools/gpu_r03_probab.sh). Lane (n, g) then holds rows 4g .. 4g+3 = pixel row g,
// column n, partial logits of kernel depth 0, 1, 2: exactly the three sums prob_regress_kernel slides over the
// planes; the same lane keeps its pixel's two open logits and later runs that pixel's regression from the LDS
// logit column. Per plane and wave: 2 staging loads, 5 ds_read_b128 and 10 MFMAs (the VALU kernel: 118
// packed FMAs per voxel).
constexpr int kPRChunks = kProbRowChunks, kPRTerms = kProbRowTerms;
constexpr int kPRVox = kHY * kHX;  // 340 staged voxels per plane
#ifndef DAMVS_PROB_AHEAD
#define DAMVS_PROB_AHEAD 4  // (A/B builds only)
#endif
constexpr int kPRAhead = DAMVS_PROB_AHEAD;  // input planes in flight per block

// T = float (the fp32 path): the same plan on split-f16 MFMAs (damvs_device.h mma_split32): each staged fp32 voxel
// (32 bytes, two loads) is split into its f16 hi / lo halves at the LDS write (two planes of 340 slots), the weights
// are the rows above split on the host (2^k scaled, pscale = 2^-k; damvs_stage prob_split), three MFMAs per chunk.
template <typename T>
__global__ __launch_bounds__(256) void prob_mfma_kernel(int B, int D, int h, int w, const T* __restrict__ feat,
                                                        const uint4* __restrict__ apack, float pscale,
                                                        const float* __restrict__ prob_init,
                                                        const float* __restrict__ hyps, float* __restrict__ depth,
                                                        float* __restrict__ conf, float* __restrict__ var,
                                                        float* __restrict__ prob, int vec_ok) {
  constexpr int PL = sizeof(T) == 4 ? 2 : 1;  // 16-byte pieces per voxel (and LDS planes per tile)
  constexpr int NA = PL == 1 ? kPRChunks * kPRTerms : kPRChunks * 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* tile = reinterpret_cast<uint4*>(smem);                 // 2 x PL x 340 voxels (double buffer)
  float* lg = reinterpret_cast<float*>(tile + 2 * PL * kPRVox); // [D][256] logits, column per pixel
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int y0 = blockIdx.y * kTY, x0 = blockIdx.x * kTX;
  const int b = blockIdx.z;
  const int R0 = 4 * (wave >> 1), C0 = 16 * (wave & 1);
  const int pix = (R0 + g) * kTX + C0 + n;  // this lane's pixel in the tile: its logit column
  const __amdgpu_buffer_rsrc_t rf = make_rsrc(feat, (long long)B * D * h * w * 16 * PL);

  uint4 af[NA];  // bf16: [chunk][term]; fp32: [chunk][hi, lo]
#pragma unroll
  for (int k = 0; k < kPRChunks; ++k) {
    if constexpr (PL == 1) {
#pragma unroll
      for (int t = 0; t < kPRTerms; ++t) af[k * kPRTerms + t] = apack[(k * kPRTerms + t) * 64 + lane];
    } else {
      af[2 * k] = apack[k * 128 + lane];
      af[2 * k + 1] = apack[k * 128 + 64 + lane];
    }
  }
  int boff[kPRChunks];  // LDS voxel of this lane's slot in every chunk
#pragma unroll
  for (int k = 0; k < kPRChunks; ++k) {
    const int sl = 4 * k + g, slc = sl < 18 ? sl : 17;
    boff[k] = (R0 + slc / 3) * kHX + C0 + n + slc % 3;
  }
  const bool bpad = g >= 2;  // chunk 4: slots 18, 19

  // staging: voxel v = tid, tid + 256 (< 340) of the halo tile
  uint32_t goff[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = tid + 256 * k, row = v / kHX, col = v - row * kHX;
    const int yy = y0 - 1 + row, xx = x0 - 1 + col;
    const bool ok = v < kPRVox && (unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w;
    goff[k] = ok ? (uint32_t)(((size_t)b * D * h + yy) * w + xx) * (16u * PL) : kOOB;
  }
  // Input planes are fetched kPRAhead planes ahead into a register ring (the per-plane work is ~20 instructions:
  // one fetch in flight per block left every plane waiting out a full memory latency); fetches past the last plane
  // are out-of-range buffer loads (no traffic, but counted like the others, so the wait counts stay static).
  const uint32_t pstride = (uint32_t)h * w * 16u * PL;
  uint4 ring[kPRAhead][2][PL];
  auto gload = [&](int pl, uint4 (&st)[2][PL]) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int hh = 0; hh < PL; ++hh)
        st[k][hh] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rf, goff[k] == kOOB || pl >= D ? kOOB : goff[k] + (uint32_t)pl * pstride + 16u * hh, 0, 0));
  };
  auto lstore = [&](int bi, const uint4 (&st)[2][PL]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int v = tid + 256 * k;
      if (k == 1 && v >= kPRVox) break;
      if constexpr (PL == 1) {
        tile[bi * kPRVox + v] = st[k][0];
      } else {
        const F16Pair p = split8(__builtin_bit_cast(float4, st[k][0]), __builtin_bit_cast(float4, st[k][1]));
        tile[(bi * 2) * kPRVox + v] = p.h;
        tile[(bi * 2 + 1) * kPRVox + v] = p.l;
      }
    }
  };

#pragma unroll
  for (int u = 0; u < kPRAhead; ++u) gload(u, ring[u]);
  lstore(0, ring[0]);
  gload(kPRAhead, ring[0]);
  __syncthreads();
  float am1 = 0.f, a0 = 0.f;
  for (int pl0 = 0; pl0 < D; pl0 += kPRAhead) {
#pragma unroll
    for (int u = 0; u < kPRAhead; ++u) {
      const int pl = pl0 + u;
      if (pl >= D) break;
      f32x4_t sum;
      if constexpr (PL == 1) {
        const uint4* tb = tile + (pl & 1) * kPRVox;
        f32x4_t acc[kPRTerms];
#pragma unroll
        for (int t = 0; t < kPRTerms; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kPRChunks; ++k) {
          uint4 bv = tb[boff[k]];
          if (k == kPRChunks - 1 && bpad) bv = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
          for (int t = 0; t < kPRTerms; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[k * kPRTerms + t]),
                                                             __builtin_bit_cast(bf16x8_t, bv), acc[t], 0, 0, 0);
        }
        sum = acc[kPRTerms - 1];  // hi + lo (+ mid)
#pragma unroll
        for (int t = kPRTerms - 2; t >= 0; --t) sum = acc[t] + sum;
      } else {
        const uint4* th = tile + ((pl & 1) * 2) * kPRVox;
        const uint4* tl = th + kPRVox;
        f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kPRChunks; ++k) {
          F16Pair bv{th[boff[k]], tl[boff[k]]};
          if (k == kPRChunks - 1 && bpad) bv = F16Pair{make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
          mma_split32(F16Pair{af[2 * k], af[2 * k + 1]}, bv, acc);
        }
        sum = acc * pscale;  // 2^-k: exact
      }
      if (pl >= 1) lg[(pl - 1) * 256 + pix] = am1 + sum[2];
      am1 = a0 + sum[1];
      a0 = sum[0];
      const int un = (u + 1) % kPRAhead;  // ring slot of plane pl + 1 (pl0 is a multiple of kPRAhead)
      lstore((pl + 1) & 1, ring[un]);  // past the last plane: zeros into the idle buffer
      gload(pl + 1 + kPRAhead, ring[un]);
      __syncthreads();
    }
  }
  float last = am1;  // plane D - 1

  const int y = y0 + R0 + g, x = x0 + C0 + n;
  const size_t hw = (size_t)h * w, p = (size_t)y * w + x;
  // w % 4 == 0: the probabilities go out as 16-byte runs of 4 pixels of a tile row from the LDS column (below)
  // instead of one 4-byte store per pixel and plane
  const bool vec = prob && vec_ok;
  if (y < h && x < w) {
  const float* hy = hyps + (size_t)b * D * hw + p;
  const float* pin = prob_init ? prob_init + (size_t)b * D * hw + p : nullptr;
  float* lcol = lg + pix;
  auto col = [&](int d) -> float& { return d == D - 1 ? last : lcol[d * 256]; };
  if (pin)
    for (int d = 0; d < D; ++d) col(d) += pin[(size_t)d * hw];
  float mx = -INFINITY;
  for (int d = 0; d < D; ++d) mx = fmaxf(mx, col(d));
  float sm = 0.f;
  for (int d = 0; d < D; ++d) {
    const float e = expf(col(d) - mx);
    col(d) = e;
    sm += e;
  }
  // hypothesis loads in groups of 8 ahead of their use (one memory latency per group, not per plane)
  float dep = 0.f, idx = 0.f;
  for (int d0 = 0; d0 < D; d0 += 8) {
    float hv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) hv[i] = d0 + i < D ? hy[(size_t)(d0 + i) * hw] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int d = d0 + i;
      if (d < D) {
        const float pr = col(d) / sm;
        col(d) = pr;
        dep += pr * hv[i];
        idx += pr * (float)d;
      }
    }
  }
  int ii = (int)idx;
  ii = ii < 0 ? 0 : (ii > D - 1 ? D - 1 : ii);
  float c = 0.f, vs = 0.f;
  float* po = prob && !vec ? prob + (size_t)b * D * hw + p : nullptr;
  for (int d0 = 0; d0 < D; d0 += 8) {
    float hv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) hv[i] = d0 + i < D ? hy[(size_t)(d0 + i) * hw] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int d = d0 + i;
      if (d < D) {
        const float pr = col(d);
        const float df = hv[i] - dep;
        vs += df * df * pr;
        if (d >= ii - 1 && d <= ii + 2) c += pr;
        if (po) po[(size_t)d * hw] = pr;
      }
    }
  }
  if (vec) lg[(D - 1) * 256 + pix] = last;  // the column's last plane
  depth[(size_t)b * hw + p] = dep;
  conf[(size_t)b * hw + p] = c;
  var[(size_t)b * hw + p] = 3.f * sqrtf(vs);
  }
  if (vec) {
    __syncthreads();  // every pixel's normalised column is in LDS
    for (int i = tid; i < D * 64; i += 256) {
      const int d = i >> 6, r = (i >> 3) & 7, c4 = i & 7;
      const int yy = y0 + r, xx = x0 + 4 * c4;
      if (yy < h && xx < w)
        *reinterpret_cast<float4*>(prob + ((size_t)(b * D + d) * h + yy) * w + xx) =
            *reinterpret_cast<const float4*>(lg + d * 256 + r * kTX + 4 * c4);
    }
  }
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
  if ((long long)D * h * w * CB * (long long)sizeof(T) >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit offsets
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
  if ((long long)D * h * w * CB * (long long)sizeof(T) >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit offsets
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
  if (Cb == 8) return store == ST_BF16 ? prob_regress_smem<bf16_t, 8>(D) : prob_regress_smem<float, 8>(D);
  return store == ST_BF16 ? prob_regress_smem<bf16_t, 16>(D) : prob_regress_smem<float, 16>(D);
}

// The range check at the end of damvs_stage_forward: depth, confidence and variance maps read once (a grid-stride loop
// over ~2 blocks per CU, coalesced 4-byte loads: any alignment); any non-finite value sets status[0] = 1 by a vector
// store. The status word is sticky: nothing in a forward clears it; only damvs_stage_status reads and clears it, and the
// caller zeroes it when it allocates the workspace (include/damvs.h). 12 bytes per pixel: ~15 us at stage 3 of cfgC.
__global__ __launch_bounds__(256) void finite_check_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ c, long long n, int* __restrict__ status) {
  bool bad = false;
  for (long long i = blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    bad |= (a[i] * 0.f + b[i] * 0.f + c[i] * 0.f) != 0.f;  // x * 0 is 0 unless x is inf or NaN
  if (bad) __builtin_amdgcn_raw_buffer_store_b32(1u, make_rsrc(status, 4), 0, 0, 0);
}

// max |x| of n floats folded into a magnitude slot (damvs_device.h prescale_of): for tensors no product kernel recorded
// (a volume handed to damvs_costreg_logits, damvs_tensor_amax). Grid-stride, one atomic per wave.
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long long n, unsigned* __restrict__ slot) {
  unsigned m = 0u;
  for (long long i = blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) m = amax_fold(m, x[i]);
  amax_flush(m, slot, blockIdx.x * 4 + (int)(threadIdx.x >> 6));
}

hipError_t launch_amax(hipStream_t s, const float* x, long long n, unsigned* slot) {
  const long long blocks = std::min<long long>((n + 255) / 256, 2048);
  if (blocks < 1) return hipSuccess;
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, slot);
  return hipGetLastError();
}

hipError_t launch_regress(hipStream_t s, int B, int D, int h, int w, const float* logits, const float* hyps,
                          float* depth, float* conf, float* var, float* prob) {
  int hw = h * w;
  hipLaunchKernelGGL(regress_kernel, dim3((hw + 255) / 256, B), dim3(256), 0, s, B, D, hw, logits, hyps, depth, conf,
                     var, prob);
  return hipGetLastError();
}

hipError_t launch_finite_check(hipStream_t s, const float* a, const float* b, const float* c, long long n, int* status) {
  const long long nb = (n + 255) / 256;
  hipLaunchKernelGGL(finite_check_kernel, dim3((unsigned)(nb < 512 ? (nb > 0 ? nb : 1) : 512)), dim3(256), 0, s, a, b, c,
                     n, status);
  return hipGetLastError();
}

}  // namespace damvs

namespace damvs {

size_t prob_mfma_smem(int store, int D) {
  return 2 * (size_t)kPRVox * 16 * (store == ST_BF16 ? 1 : 2) + (size_t)(D > 0 ? D : 0) * 256 * 4;
}

hipError_t launch_prob_mfma(hipStream_t s, int store, int B, int D, int h, int w, const void* feat, const void* apack,
                            float pscale, const float* prob_init, const float* hyps, float* depth, float* conf,
                            float* var, float* prob) {
  const size_t smem = prob_mfma_smem(store, D);
  const int PL = store == ST_BF16 ? 1 : 2;
  if (D < 1 || smem > 160 * 1024) return hipErrorInvalidValue;
  if ((long long)B * D * h * w * 16 * PL >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit buffer offsets
  const void* k = store == ST_BF16 ? reinterpret_cast<const void*>(prob_mfma_kernel<bf16_t>)
                                   : reinterpret_cast<const void*>(prob_mfma_kernel<float>);
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
  }
  const dim3 grid((w + kTX - 1) / kTX, (h + kTY - 1) / kTY, B);
  // 16-byte probability stores need w % 4 == 0 (DAMVS_PROB_VEC=0, read per call: one 4-byte store per pixel and plane)
  const char* pv = getenv("DAMVS_PROB_VEC");
  const int vec_ok = (w & 3) == 0 && !(pv && pv[0] == '0');
  if (store == ST_BF16)
    hipLaunchKernelGGL(prob_mfma_kernel<bf16_t>, grid, dim3(256), smem, s, B, D, h, w,
                       reinterpret_cast<const bf16_t*>(feat), reinterpret_cast<const uint4*>(apack), 1.f, prob_init,
                       hyps, depth, conf, var, prob, vec_ok);
  else
    hipLaunchKernelGGL(prob_mfma_kernel<float>, grid, dim3(256), smem, s, B, D, h, w,
                       reinterpret_cast<const float*>(feat), reinterpret_cast<const uint4*>(apack), pscale, prob_init,
                       hyps, depth, conf, var, prob, vec_ok);
  return hipGetLastError();
}

// DAMVS_PROB_MFMA=0 (read per call: tests flip it) sends bf16 stages to the VALU prob_regress_kernel.
bool prob_mfma_disabled() {
  const char* v = getenv("DAMVS_PROB_MFMA");
  return v && v[0] == '0';
}

// The stage regression's prob conv on MFMA for this storage type: bf16 by default; fp32 (the split-f16 form) only
// with DAMVS_PROB_MFMA=1 -- three MFMAs per product measured slower than the VALU kernel (cfgC B=4 fp32: 1.66
// against 1.56 ms per step, profiles/r04/prof_steps_f32_r04j.txt).
bool prob_mfma_enabled(int store) {
  const char* v = getenv("DAMVS_PROB_MFMA");
  if (v && v[0] == '0') return false;
  return store == ST_BF16 || (v && v[0] == '1');
}

}  // namespace damvs
