// Fused cost-regularization head: conv11 + conv0 skip + prob conv + softmax regression in one kernel.
//
//   x = conv0 + self.conv11(x); prob = self.prob(x)        (models/module.py:537-541)
//   softmax over D, depth, photometric confidence, exp-variance (models/cas_mvsnet.py:105-124)
//
// Unfused, conv11 writes the full-resolution 8-channel U-Net output (16 B / 32 B per voxel) and the prob conv reads
// it back with a one-voxel halo. Here a block owns an 8 x 30 pixel column of the output for all D planes and walks
// the conv9 output (conv11's input, half resolution, 16 channels) one q-plane at a time; each q-plane yields output
// planes 2p and 2p+1. Per q-plane:
//   1. conv11 on the matrix cores for the (8+2) x (30+2) halo tile of both output planes, the x-pair form of
//      deconv_xpair_zslide_kernel (same A fragments, K order and epilogue: bias, ReLU, + skip), from a 3-slot LDS
//      ring of 6 x 17 q-voxel input planes; the results (zero outside the image: the prob conv's padding) go to an
//      LDS feature tile, never to HBM;
//   2. the prob conv of prob_mfma_kernel (k_regress.hip) on both planes: per wave a 16 x 16 output tile of rows
//      4 j + dz (pixel row j, kernel depth dz) x 16 pixels, the two open partial logits slid along the planes, the
//      closed logit into an LDS column per pixel;
// then the regression of prob_mfma_kernel runs on the column. The tile is 30 columns wide (x0 odd) and starts at an
// odd row so that the halo tile is exactly 16 q-columns x 5 q-rows of the deconv's x / y pairs: one MFMA column
// group per q-row and no partial pairs.
// bf16 (T = bf16_t): the deconv products, the bf16 rounding of the feature and the prob conv are those of the
// unfused kernels, so the outputs are bitwise equal to deconv_xpair_zslide + prob_mfma (tests/test_gpu_parity.py).
// fp32 (T = float): the split-f16 form of both convs (damvs_device.h mma_split32): the feature tile keeps each fp32
// voxel as its f16 hi / lo halves, the prob weights are split on the host (2^k scaled, pscale = 2^-k).
#include <cstdlib>
#include <type_traits>

#include "damvs_device.h"

namespace damvs {

namespace {

constexpr int kHTY = 8, kHTX = 30;         // output pixels per block tile
constexpr int kHFY = kHTY + 2, kHFX = 34;  // feature tile: rows y0-1 .. y0+8, columns x0-1 .. x0+32 (32, 33 zero)
constexpr int kHFV = kHFY * kHFX;          // 340 voxels
constexpr int kHQY = 6, kHQX = 17;         // conv9-output tile per q-plane: q-rows qy0 .. qy0+5, q-cols qx0 .. qx0+16
constexpr int kHPix = 256;                 // logit column stride (8 rows x 32 columns; columns 30, 31 unused)
template <int V> using IC = std::integral_constant<int, V>;

template <typename T> struct HeadForm;
#ifndef DAMVS_HEAD_NFB
#define DAMVS_HEAD_NFB 2  // (A/B builds: 1 = one feature tile and two barriers per q-plane for bf16 too)
#endif
template <> struct HeadForm<bf16_t> {
  static constexpr int NFB = DAMVS_HEAD_NFB;  // feature tile buffers (double: one barrier per q-plane)
  static constexpr bool ALDS = false;  // conv11 A fragments in registers
  static constexpr int PCH = kProbRowChunks * kProbRowTerms;  // prob A fragments (uint4) per lane
};
template <> struct HeadForm<float> {
  static constexpr int NFB = 1;
  static constexpr bool ALDS = true;
  static constexpr int PCH = kProbRowChunks * 2;
};

size_t head_smem_t(int store, int D) {
  const bool bf = store == ST_BF16;
  const int PL = bf ? 1 : 2, NFB = bf ? DAMVS_HEAD_NFB : 1;
  size_t b = 3 * (size_t)kHQY * kHQX * 2 * PL * 16;  // input ring
  b += (size_t)NFB * 2 * kHFV * PL * 16;              // feature tiles (2 planes each)
  if (!bf) b += 9 * 128 * 16;                         // conv11 A fragments (fp32)
  b += (size_t)D * kHPix * 4;                          // logit column
  return b;
}

template <typename T>
__global__ __launch_bounds__(256) DAMVS_WAVES(2) void head_kernel(const HeadArgs a, int tiles_x, int tiles_y,
                                                                   int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  typedef HeadForm<T> H;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int CH = 2, S = CH * PL, PW = kHQX, PH = kHQY;
  constexpr int RPLANE = PH * PW * S;             // 16-byte slots per ring plane
  constexpr int NRC = PH * PW * CH;               // 8-channel chunks per ring plane (204: one per thread)
  constexpr int FPLANE = kHFV * PL;               // 16-byte slots per feature plane (fp32: hi plane, then lo plane)
  constexpr int NFB = H::NFB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);
  uint4* ftile = ring + 3 * RPLANE;               // [NFB][2 planes][FPLANE]
  uint4* alds = ftile + NFB * 2 * FPLANE;         // fp32: 9 x 128 conv11 A slots
  float* lg = reinterpret_cast<float*>(alds + (H::ALDS ? 9 * 128 : 0));  // [D][256]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x;
  tt /= tiles_x;
  const int ty = tt % tiles_y;
  const int b = tt / tiles_y;
  const int y0 = kHTY * ty - 1, x0 = kHTX * tx - 1;  // first output pixel of the tile
  const int qy0 = 4 * ty - 1, qx0 = 15 * tx - 1;     // q-voxel of the halo row / column (y0 - 1 = 2 qy0)
  const int D = a.D, h = a.h, w = a.w, Di = a.Di, Hi = a.Hi, Wi = a.Wi;

  // ---- conv11 input ring (x-pair layout of deconv_xpair_zslide_kernel)
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.x, (long long)a.B * Di * Hi * Wi * 16 * ES);
  auto load_plane = [&](int iz, uint4 (&v)[PL]) {
    const int c = tid, row = c / (PW * CH), col = c - row * (PW * CH);
    const int iy = qy0 + row, ix = qx0 + col / CH;
    const bool ok = c < NRC && iz < Di && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
    const uint32_t off = ok ? (uint32_t)((((b * Di + iz) * Hi + iy) * Wi + ix) * CH + (col % CH)) * (16u * PL) : 0u;
#pragma unroll
    for (int hh = 0; hh < PL; ++hh) v[hh] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * hh : kOOB);
  };
  auto store_plane = [&](int iz, const uint4 (&v)[PL]) {
    const int c = tid;
    if (c >= NRC) return;
    uint4* dst = ring + (iz % 3) * RPLANE;
    if constexpr (PL == 1) {
      dst[c] = v[0];
    } else {
      const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
      const F16Pair p = split8(__builtin_bit_cast(float4, v[0]), __builtin_bit_cast(float4, v[1]));
      dst[vox * S + (q ^ sw)] = p.h;
      dst[vox * S + ((CH + q) ^ sw)] = p.l;
    }
  };

  // ---- A fragments
  frag wreg[H::ALDS ? 1 : 9];
  if constexpr (!H::ALDS) {
#pragma unroll
    for (int s = 0; s < 9; ++s) wreg[s] = Z::wload(reinterpret_cast<const uint4*>(a.wdec), s, lane);
  } else {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(a.wdec);
    for (int i = tid; i < 9 * 128; i += 256) alds[i] = wsrc[i];
  }
  auto wfrag = [&](int s) -> frag {
    if constexpr (!H::ALDS) return wreg[s];
    else return Z::wload(alds, s, lane);
  };
  uint4 pw[H::PCH];  // prob A: bf16 [chunk][term], fp32 [chunk][hi, lo]
  {
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.wprob);
#pragma unroll
    for (int k = 0; k < kProbRowChunks; ++k) {
      if constexpr (PL == 1) {
#pragma unroll
        for (int t = 0; t < kProbRowTerms; ++t) pw[k * kProbRowTerms + t] = src[(k * kProbRowTerms + t) * 64 + lane];
      } else {
        pw[2 * k] = src[k * 128 + lane];
        pw[2 * k + 1] = src[k * 128 + 64 + lane];
      }
    }
  }

  // ---- conv11 lane geometry: wave w computes q-row w (all four (pd, py) phases) and phase w of q-row 4
  const bool lead = (g & 1) == 0;
  const int lcol = n + (g >> 1), lsw = Z::template zsw<S>(lcol);
  const int lch = PL == 1 ? 0 : (g & 1);
  const int lofs = lcol * S + (PL == 1 ? (g & 1) : 0);
  float b8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b8[i] = a.bdec[i];
  const long long nskip = (long long)a.B * D * h * w * 8 * ES;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.skip, nskip);
  // the five outputs of this lane (unit u: q-row, phase), their feature-tile slot (or -1) and skip offset
  auto out_geom = [&](int p, int r, int ph, uint32_t& off) -> int {
    const int pd = ph >> 1, py = ph & 1;
    const int oz = 2 * p + pd, oy = 2 * (qy0 + r) + py, ox = 2 * (qx0 + n) + (g >> 1);
    const bool in = lead && oz < D && (unsigned)oy < (unsigned)h && (unsigned)ox < (unsigned)w;
    off = in ? (uint32_t)((((b * D + oz) * h + oy) * w + ox) * 8) * (uint32_t)ES : kOOB;
    return lead ? pd * FPLANE + (2 * r + py) * kHFX + 2 * n + (g >> 1) : -1;
  };
  // skip records of q-plane p's five outputs into rq (past the last plane: out-of-range loads, no traffic)
  auto load_skip = [&](int p, uint4 (&rq)[5][PL]) {
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      uint32_t off;
      (void)out_geom(p, u < 4 ? wave : 4, u < 4 ? u : wave, off);
      if (p >= Di) off = kOOB;
#pragma unroll
      for (int hh = 0; hh < PL; ++hh) rq[u][hh] = BufIO<bf16_t>::frag(rs, off == kOOB ? kOOB : off + 16u * hh);
    }
  };

  // ---- prob conv lane geometry (prob_mfma_kernel)
  const int R0 = 4 * (wave >> 1), C0 = 16 * (wave & 1);
  const int pix = (R0 + g) * 32 + C0 + n;
  int boff[kProbRowChunks];
#pragma unroll
  for (int k = 0; k < kProbRowChunks; ++k) {
    const int sl = 4 * k + g, slc = sl < 18 ? sl : 17;
    boff[k] = (R0 + slc / 3) * kHFX + C0 + n + slc % 3;
  }
  const bool bpad = g >= 2;

  // ---- prologue: q-planes 0, 1 into the ring, 2 and 3 into the two register sets, the skip records of q-planes 0
  // and 1, all requested together; zero the feature tiles (columns 32, 33 stay zero). From here on every global
  // load has two q-plane steps of cover: step p consumes the skip records and stores the ring plane requested at
  // step p - 2 (the per-step work is short: one exposed memory latency per step bound the first form).
  uint4 pa[PL], pb[PL];
  uint4 rqa[5][PL], rqb[5][PL];
  load_plane(0, pa);
  load_plane(1, pb);
  load_skip(0, rqa);
  load_skip(1, rqb);
  for (int i = tid; i < NFB * 2 * FPLANE; i += 256) ftile[i] = make_uint4(0u, 0u, 0u, 0u);
  store_plane(0, pa);
  store_plane(1, pb);
  load_plane(2, pa);
  load_plane(3, pb);
  __syncthreads();

  float am1 = 0.f, a0 = 0.f;
  auto prob_plane = [&](const uint4* ft, int pl) {
    f32x4_t sum;
    if constexpr (PL == 1) {
      f32x4_t acc[kProbRowTerms];
#pragma unroll
      for (int t = 0; t < kProbRowTerms; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < kProbRowChunks; ++k) {
        uint4 bv = ft[boff[k]];
        if (k == kProbRowChunks - 1 && bpad) bv = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int t = 0; t < kProbRowTerms; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, pw[k * kProbRowTerms + t]),
                                                           __builtin_bit_cast(bf16x8_t, bv), acc[t], 0, 0, 0);
      }
      sum = acc[kProbRowTerms - 1];
#pragma unroll
      for (int t = kProbRowTerms - 2; t >= 0; --t) sum = acc[t] + sum;
    } else {
      f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < kProbRowChunks; ++k) {
        F16Pair bv{ft[boff[k]], ft[kHFV + boff[k]]};
        if (k == kProbRowChunks - 1 && bpad) bv = F16Pair{make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
        mma_split32(F16Pair{pw[2 * k], pw[2 * k + 1]}, bv, acc);
      }
      sum = acc * a.pscale;  // 2^-k: exact
    }
    if (pl >= 1) lg[(pl - 1) * kHPix + pix] = am1 + sum[2];
    am1 = a0 + sum[1];
    a0 = sum[0];
  };

  auto step = [&](int p, uint4 (&rq)[5][PL], uint4 (&pl)[PL]) {
    uint4* ft = ftile + (p % NFB) * 2 * FPLANE;
    const uint4* r0 = ring + (p % 3) * RPLANE + lofs;        // q-plane p (z offset 0)
    const uint4* r1 = ring + ((p + 1) % 3) * RPLANE + lofs;  // q-plane p + 1 (z offset +1)
    // conv11: 5 units of one (q-row, phase) each, the epilogue straight into the feature tile
    // unit u (compile-time: the skip record slot) = q-row r, phase PH (compile-time: the A fragment indices)
    auto unit = [&](auto phc, auto uc, int r) {
      constexpr int ph = decltype(phc)::value, u = decltype(uc)::value;
      constexpr int pd = ph >> 1, py = ph & 1;
      constexpr int na = pd ? 2 : 1, nb = py ? 2 : 1;
      constexpr int w0 = ph == 0 ? 0 : ph == 1 ? 1 : ph == 2 ? 3 : 5;
      f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ca = 0; ca < na; ++ca)
#pragma unroll
        for (int cb = 0; cb < nb; ++cb) {
          const int zo = pd ? (ca == 0 ? 1 : 0) : 0, yo = py ? (cb == 0 ? 1 : 0) : 0;
          const uint4* src = (zo ? r1 : r0) + (r + yo) * PW * S;
          Z::mma(wfrag(w0 + ca * nb + cb), Z::bread(src, lch, CH, lsw), acc);
        }
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[i];
        v[4 + i] = __shfl_down(acc[i], 16);
      }
      uint32_t off;
      const int slot = out_geom(p, r, ph, off);
      if constexpr (PL == 1) {
        const uint32_t q4[4] = {rq[u][0].x, rq[u][0].y, rq[u][0].z, rq[u][0].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] += b8[i];
          v[i] = relu(v[i]);
          v[i] += __uint_as_float((i & 1) ? (q4[i >> 1] & 0xffff0000u) : (q4[i >> 1] << 16));
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float4 f = __builtin_bit_cast(float4, rq[u][i >> 2]);
          v[i] = v[i] * a.wscale + b8[i];
          v[i] = relu(v[i]);
          v[i] += (i & 3) == 0 ? f.x : (i & 3) == 1 ? f.y : (i & 3) == 2 ? f.z : f.w;
        }
      }
      if (a.diag && slot >= 0 && off != kOOB) {
        const int tr = 2 * r + py, tc = 2 * n + (g >> 1);
        if (tr >= 1 && tr <= kHTY && tc >= 1 && tc <= kHTX) {
          float* dd = a.diag + (size_t)off / ES;
#pragma unroll
          for (int i = 0; i < 8; ++i) dd[i] = v[i];
        }
      }
      if (slot >= 0) {
        if (off == kOOB) {  // outside the image: the prob conv's zero padding
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = 0.f;
        }
        if constexpr (PL == 1) {
          uint32_t q[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) q[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
          ft[slot] = make_uint4(q[0], q[1], q[2], q[3]);
        } else {
          const F16Pair s2 = split8(v);
          ft[slot] = s2.h;
          ft[kHFV + slot] = s2.l;
        }
      }
    };
    unit(IC<0>{}, IC<0>{}, wave);
    unit(IC<1>{}, IC<1>{}, wave);
    unit(IC<2>{}, IC<2>{}, wave);
    unit(IC<3>{}, IC<3>{}, wave);
    switch (wave) {  // q-row 4: phase = wave (a wave-uniform branch, each case with a constant phase)
      case 0: unit(IC<0>{}, IC<4>{}, 4); break;
      case 1: unit(IC<1>{}, IC<4>{}, 4); break;
      case 2: unit(IC<2>{}, IC<4>{}, 4); break;
      default: unit(IC<3>{}, IC<4>{}, 4); break;
    }
    load_skip(p + 2, rq);
    // ring: q-plane p + 2 (requested at step p - 2) into the slot of p - 1 (last read before the previous barrier),
    // then request p + 4 into the same registers
    store_plane(p + 2, pl);
    load_plane(p + 4, pl);
    __syncthreads();
    prob_plane(ft, 2 * p);
    prob_plane(ft + FPLANE, 2 * p + 1);
    if constexpr (NFB == 1) __syncthreads();
  };
  for (int p = 0; p < Di; p += 2) {  // unrolled by two: the register sets alternate statically
    step(p, rqa, pa);
    if (p + 1 < Di) step(p + 1, rqb, pb);
  }
  float last = am1;  // plane D - 1

  // ---- regression (prob_mfma_kernel)
  const int y = y0 + R0 + g, x = x0 + C0 + n;
  const size_t hw = (size_t)h * w, pp = (size_t)y * w + x;
  if (C0 + n < kHTX && (unsigned)y < (unsigned)h && (unsigned)x < (unsigned)w) {
    const float* hy = a.hyps + (size_t)b * D * hw + pp;
    const float* pin = a.prob_init ? a.prob_init + (size_t)b * D * hw + pp : nullptr;
    float* lcol = lg + pix;
    auto col = [&](int d) -> float& { return d == D - 1 ? last : lcol[d * kHPix]; };
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
        }
      }
    }
    lg[(D - 1) * kHPix + pix] = last;
    a.depth[(size_t)b * hw + pp] = dep;
    a.conf[(size_t)b * hw + pp] = c;
    a.var[(size_t)b * hw + pp] = 3.f * sqrtf(vs);
  }
  if (a.prob) {
    __syncthreads();  // every pixel's normalised column is in LDS: rows of 30 consecutive pixels per plane
    for (int i = tid; i < D * kHPix; i += 256) {
      const int d = i >> 8, r = (i >> 5) & 7, cc = i & 31;
      const int yy = y0 + r, xx = x0 + cc;
      if (cc < kHTX && (unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
        a.prob[((size_t)(b * D + d) * h + yy) * w + xx] = lg[i];
    }
  }
}

}  // namespace

size_t head_smem(int store, int D) { return head_smem_t(store, D); }

hipError_t launch_head(hipStream_t s, int store, const HeadArgs& a) {
  if (a.D != 2 * a.Di || a.h != 2 * a.Hi || a.w != 2 * a.Wi || a.D < 2) return hipErrorInvalidValue;
  const size_t smem = head_smem_t(store, a.D);
  const int ES = store == ST_BF16 ? 2 : 4;
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  if ((long long)a.B * a.D * a.h * a.w * 8 * ES >= (1LL << 31) ||
      (long long)a.B * a.Di * a.Hi * a.Wi * 16 * ES >= (1LL << 31))
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  const int tiles_x = (a.w + 1 + kHTX - 1) / kHTX, tiles_y = (a.h + 1 + kHTY - 1) / kHTY;
  const long long nt = (long long)tiles_x * tiles_y * a.B;
  const void* k = store == ST_BF16 ? reinterpret_cast<const void*>(head_kernel<bf16_t>)
                                   : reinterpret_cast<const void*>(head_kernel<float>);
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
  }
  if (store == ST_BF16)
    hipLaunchKernelGGL(head_kernel<bf16_t>, dim3((unsigned)nt), dim3(256), smem, s, a, tiles_x, tiles_y, (int)nt);
  else
    hipLaunchKernelGGL(head_kernel<float>, dim3((unsigned)nt), dim3(256), smem, s, a, tiles_x, tiles_y, (int)nt);
  return hipGetLastError();
}

}  // namespace damvs
