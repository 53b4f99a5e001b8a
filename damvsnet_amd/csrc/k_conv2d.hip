// 2D front-end convolutions (FeatureNet, models/module.py:355-462; GeoFeatureFusion,
// models/geometry.py:14-277) as NHWC implicit GEMM on MFMA, with the glue the reference runs as
// separate ops fused in:
//   * channel concat of two feature tensors (torch.cat([r2p, s2]) etc.): K runs over in0 then in1;
//   * up to 4 fp32 planar "geometry" inputs (the 1-channel depth planes BasicBlockGeo concatenates)
//     as extra K rows (tap x plane) after the tensor-input chunks; layers whose only inputs are
//     planes (the RGB/depth init convs) run on a direct VALU kernel instead;
//   * bias (BN folded host side), residual before ReLU (BasicBlockGeo identity/downsample),
//     ReLU, residual after ReLU (decoder skips, FPN's nearest-x2 upsampled top-down path).
// Conv and ConvTranspose share one kernel: a transposed conv of stride s is s^2 output-parity
// phases, each a dense sub-convolution over the input grid (no structural zeros on MFMA).
#include <cstdlib>

#include <type_traits>

#include "conv2d_common.h"

namespace damvs {

namespace {

template <typename T> using Frag2 = MmaFrag<T>;

template <typename T> struct T_is_bf16 { static constexpr bool value = false; };
template <> struct T_is_bf16<bf16_t> { static constexpr bool value = true; };

constexpr int kG2 = 4;  // 16-pixel groups per wave

template <typename T> __device__ __forceinline__ typename Frag2<T>::raw pack_vals(const float* v);
template <> __device__ __forceinline__ float4 pack_vals<float>(const float* v) { return make_float4(v[0], v[1], v[2], v[3]); }
template <> __device__ __forceinline__ uint4 pack_vals<bf16_t>(const float* v) {
  return make_uint4((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16), (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16),
                    (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16), (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16));
}

// Implicit-GEMM conv on MFMA. A wave owns 64 output pixels (kG2 groups of 16) x MT 16-channel
// tiles. K runs over (tap, concatenated channel) in chunks of KC = 4E, then over (tap, plane) for
// the fp32 planes. Index arithmetic is 32-bit and incremental (no divisions in the K loop): the
// kernel is otherwise VALU-bound on address math for the thin full-resolution layers.
// XP (a.xpair layers: ConvTranspose stride 2, cout 8): MFMA row r = (x parity r >> 3, channel r & 7),
// so lane group g holds channels (g & 1) * 4 of output x = 2 qx + (g >> 1); group g + 1 hands its 4
// channels to group g (g even), which loads / stores the pixel's whole 8-channel record.
// K32 (T = float, the fp32 path; a.wide32: the layer's 32-K split packing, channels in multiples of 8): K chunks of 32
// (tap, channel) entries, 8 consecutive channels of one tap per lane (two 16-byte loads, split once into f16 hi / lo)
// and mma_split32 (16x16x32, full f16 rate) instead of the 16-K form's three 16x16x16 per 4 channels: half the MFMA
// issue for the same products (conv3d_mfma_kernel's K32 form, round 4).
template <typename T, int MT, bool TWO, bool XP = false, bool K32 = false>
__global__ __launch_bounds__(256) DAMVS_WAVES((sizeof(T) == 2 && MT == 4 && !TWO ? 3 : K32 && MT == 4 ? 2 : 1)) void conv2d_mfma_kernel(const Conv2dArgs a, int nqblk) {
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  typedef typename std::conditional<K32, F16Pair, raw>::type frag;
  static_assert(!K32 || (sizeof(T) == 4 && !XP), "32-K form: fp32 storage, no x-pair phases");
  constexpr int E = K32 ? 8 : Stor<T>::E;  // K entries per lane and chunk
  constexpr int KC = 4 * E;
  constexpr uint32_t ES = sizeof(T);
  // logical block = (q-block, phase), phase fastest, XCD-contiguous (see conv3d_mfma_kernel)
  const int nblk = nqblk * a.nphase;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int qblk = L / a.nphase;
  const Conv2dPhase& ph = a.ph[L - qblk * a.nphase];
  const int mt0 = blockIdx.y * MT;  // first 16-channel output tile of this block

  __shared__ int s_tap[32];  // packed (dy + 8) | (dx + 8) << 8
  if (threadIdx.x < 25) s_tap[threadIdx.x] = ((int)(ph.tap[threadIdx.x][0] + 8)) | ((int)(ph.tap[threadIdx.x][1] + 8) << 8);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int Qtot = a.B * a.Hq * a.Wq;
  const int base = (qblk * 4 + wave) * (kG2 * 16);
  if (base >= Qtot) return;
  // per pixel group: input origin (y, x, flat pixel index), output flat pixel index
  int ys[kG2], xs[kG2], pin[kG2], pout[kG2], ppost[kG2];
  bool valid[kG2];
#pragma unroll
  for (int j = 0; j < kG2; ++j) {
    int q = base + j * 16 + n;
    valid[j] = q < Qtot;
    q = valid[j] ? q : 0;
    const int r = fdiv(a.div_wq, q), qx = q - r * a.Wq;
    const int b = fdiv(a.div_hq, r), qy = r - b * a.Hq;
    ys[j] = qy * a.in_stride;
    xs[j] = qx * a.in_stride;
    pin[j] = (b * a.Hi + ys[j]) * a.Wi + xs[j];
    const int oy = qy * a.out_stride + ph.py, ox = qx * a.out_stride + (XP ? (g >> 1) : ph.px);
    pout[j] = (b * a.Ho + oy) * a.Wo + ox;
    const int us = a.post_up >> 1;  // post_up is 1 or 2
    ppost[j] = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
  }
  f32x4_t acc[kG2][MT];
#pragma unroll
  for (int j = 0; j < kG2; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 64 + lane;
  // K32: [chunk][tile][hi: 64 lanes][lo: 64 lanes] (split_weights_blocked)
  const uint4* __restrict__ wp32 =
      reinterpret_cast<const uint4*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 128 + lane;
  auto wload = [&](int chunk, int m) -> frag {
    if constexpr (K32) {
      const uint4* q = wp32 + ((size_t)chunk * a.MTtot + m) * 128;
      return F16Pair{q[0], q[64]};
    } else {
      return wp[(size_t)(chunk * a.MTtot + m) * 64];
    }
  };
  auto mma = [&](const frag& w, const frag& x, f32x4_t& acc) {
    if constexpr (K32) mma_split32(w, x, acc);
    else Frag2<T>::mma(w, x, acc);
  };
  const int npix = a.B * a.Hi * a.Wi;
  const int ctot = a.c0 + a.c1;
  const int nk = ph.kchunks;
  if (nk > 0) {
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.in0, (long long)npix * a.c0 * ES);
    const __amdgpu_buffer_rsrc_t r1 = make_rsrc(TWO ? a.in1 : a.in0, TWO ? (long long)npix * a.c1 * ES : 0);
    int t = (g * E) / ctot, ci = g * E - t * ctot;  // this lane's (tap, channel) at k = s*KC + g*E
    const int qt = KC / ctot, rc = KC - qt * ctot;
    // fragments of chunk s (then advances the lane's (tap, channel) to chunk s+1)
    auto fetch = [&](int s, frag* wf, frag* xf) {
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wload(s, m);
      const bool tv = t < ph.ntaps;
      const int code = s_tap[tv ? t : 0];
      const int dy = (code & 0xff) - 8, dx = ((code >> 8) & 0xff) - 8;
      const int tapoff = dy * a.Wi + dx;
      const bool second = TWO && ci >= a.c0;
      const int cs = second ? a.c1 : a.c0, cl = second ? ci - a.c0 : ci;
#pragma unroll
      for (int j = 0; j < kG2; ++j) {
        const int iy = ys[j] + dy, ix = xs[j] + dx;
        const bool ok = valid[j] && tv && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
        const uint32_t off = (uint32_t)((pin[j] + tapoff) * cs + cl) * ES;
        if constexpr (K32) {  // 8 channels of one tap (channel counts are multiples of 8): two loads, split once
          const __amdgpu_buffer_rsrc_t r = (TWO && second) ? r1 : r0;
          const uint32_t o = ok ? off : kOOB, o2 = ok ? off + 16u : kOOB;
          xf[j] = split8(IO::frag(r, o), IO::frag(r, o2));
        } else if (TWO) {
          xf[j] = IO::merge(IO::frag(r0, ok && !second ? off : kOOB), IO::frag(r1, ok && second ? off : kOOB));
        } else {
          xf[j] = IO::frag(r0, ok ? off : kOOB);
        }
      }
      ci += rc;
      t += qt;
      if (ci >= ctot) { ci -= ctot; ++t; }
    };
    // software-pipelined one chunk ahead: chunk s+1's loads are in flight during chunk s's MFMAs
    // (the deep low-resolution layers run at 1-2 waves per SIMD, too few to hide load latency)
    frag wf[MT], xf[kG2];
    if constexpr (MT <= 2) {  // thin layers: occupancy hides the latency, the registers buy nothing
#pragma unroll 1
      for (int s = 0; s < nk; ++s) {
        fetch(s, wf, xf);
#pragma unroll
        for (int j = 0; j < kG2; ++j)
#pragma unroll
          for (int m = 0; m < MT; ++m) mma(wf[m], xf[j], acc[j][m]);
      }
    } else {
      fetch(0, wf, xf);
      for (int s = 0; s < nk; ++s) {
        frag wn[MT], xn[kG2];
        const bool more = s + 1 < nk;
        if (more) fetch(s + 1, wn, xn);
#pragma unroll
        for (int j = 0; j < kG2; ++j)
#pragma unroll
          for (int m = 0; m < MT; ++m) mma(wf[m], xf[j], acc[j][m]);
        if (more) {
#pragma unroll
          for (int m = 0; m < MT; ++m) wf[m] = wn[m];
#pragma unroll
          for (int j = 0; j < kG2; ++j) xf[j] = xn[j];
        }
      }
    }
  }

  // the fp32 plane (BasicBlockGeo's concatenated depth plane; host allows at most one next to
  // tensor inputs) as extra K rows, one per tap, rounded to the compute type like the reference's
  // torch.cat(...).to(dtype)
  if (ph.gchunks > 0) {
    const int plane = a.Hi * a.Wi;
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.geo[0], ((long long)(a.B - 1) * a.geo_bstride[0] + plane) * 4);
    int pg[kG2];  // plane offset of the pixel's tap-(0,0) input
#pragma unroll
    for (int j = 0; j < kG2; ++j) {  // batch of the pixel group: recover from its flat input index
      const int b = fdiv(a.div_hq, fdiv(a.div_wq, valid[j] ? base + j * 16 + n : 0));
      pg[j] = b * (int)a.geo_bstride[0] + (pin[j] - b * plane);
    }
    for (int s = 0; s < ph.gchunks; ++s) {
      frag wf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wload(nk + s, m);
      float v[kG2][E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int t = s * KC + g * E + e;
        const bool tv = t < ph.ntaps;
        const int code = s_tap[tv ? t : 0];
        const int dy = (code & 0xff) - 8, dx = ((code >> 8) & 0xff) - 8;
        const int tapoff = dy * a.Wi + dx;
#pragma unroll
        for (int j = 0; j < kG2; ++j) {
          const int iy = ys[j] + dy, ix = xs[j] + dx;
          const bool ok = valid[j] && tv && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
          v[j][e] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rg, ok ? (uint32_t)(pg[j] + tapoff) * 4u : kOOB, 0, 0));
        }
      }
      frag xf[kG2];
#pragma unroll
      for (int j = 0; j < kG2; ++j) {
        if constexpr (K32) xf[j] = split8(v[j]);
        else xf[j] = pack_vals<T>(v[j]);
      }
#pragma unroll
      for (int j = 0; j < kG2; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) mma(wf[m], xf[j], acc[j][m]);
    }
  }

  // epilogue: residual loads first, then bias / residual / ReLU / store
  typedef typename IO::quad quad;
  const int up = a.post_up;
  const long long nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  if constexpr (XP && sizeof(T) == 4) {
    // fp32: every lane owns the 4 channels (16 bytes) of output x = 2 qx + (g >> 1) in channel half g & 1 -- no shuffle,
    // every lane loads its residuals and stores (bf16, below: 8-byte halves, so the even lane group takes the record)
    const int ch = (g & 1) * 4;
    float b4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[i] = a.bias[ch + i];
#pragma unroll
    for (int j = 0; j < kG2; ++j) {
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][0][i], a.wscale, b4[i]);
      const bool ok = valid[j];
      const uint32_t o = ok ? (uint32_t)(pout[j] * 8 + ch) * ES : kOOB;
      if (a.res_pre) IO::addq(IO::ldq(rpre, o), r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) IO::addq(IO::ldq(rpost, ok ? (uint32_t)(ppost[j] * 8 + ch) * ES : kOOB), r);
      IO::stq(ro, o, r);
    }
    return;
  }
  if constexpr (XP) {
    const bool lead = (g & 1) == 0;
    float b8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) b8[i] = a.bias[i];
#pragma unroll
    for (int j = 0; j < kG2; ++j) {
      float r[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        r[i] = fmaf(acc[j][0][i], a.wscale, b8[i]);
        r[4 + i] = fmaf(__shfl_down(acc[j][0][i], 16), a.wscale, b8[4 + i]);
      }
      if (!lead) continue;
      const bool ok = valid[j];
      if (a.res_pre) Vox8<T>::add(rpre, ok ? (uint32_t)(pout[j] * 8) * ES : kOOB, r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) Vox8<T>::add(rpost, ok ? (uint32_t)(ppost[j] * 8) * ES : kOOB, r);
      Vox8<T>::store(ro, ok ? (uint32_t)(pout[j] * 8) * ES : kOOB, r);
    }
    return;
  }
  float bias[MT][4];
  bool cok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = (mt0 + m) * 16 + g * 4;
    cok[m] = co < a.cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = a.bias[co + i];  // padded to cout_pad
  }
#pragma unroll
  for (int j = 0; j < kG2; ++j) {  // residual loads of one pixel group first, then the math
    quad qpre[MT], qpost[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const bool ok = valid[j] && cok[m];
      const int co = (mt0 + m) * 16 + g * 4;
      if (a.res_pre) qpre[m] = IO::ldq(rpre, ok ? (uint32_t)(pout[j] * a.cout + co) * ES : kOOB);
      if (a.res_post) qpost[m] = IO::ldq(rpost, ok ? (uint32_t)(ppost[j] * a.cout + co) * ES : kOOB);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][m][i], a.wscale, bias[m][i]);
      if (a.res_pre) IO::addq(qpre[m], r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) IO::addq(qpost[m], r);
      const uint32_t off = (uint32_t)(pout[j] * a.cout + (mt0 + m) * 16 + g * 4) * ES;
      IO::stq(ro, valid[j] && cok[m] ? off : kOOB, r);
    }
  }
}

// LDS-staged variant for the thin stride-1 3x3 layers (one tensor input of CIN <= 32 channels, at most
// one fp32 plane): the full-resolution FeatureNet / GeoFeatureFusion convs that the global-gather
// kernel runs TA-bound (each input pixel is fetched by 9 taps through L1). A block owns an
// 8-row x 64-column output tile; its (8+2) x (64+2) x CIN halo is read once with 16-byte loads
// (zero padding by range-checked buffer loads) and every B fragment is a ds_read_b128. Wave w owns
// columns [16w, 16w+16), group j output row j. For CIN < KC a K chunk spans KC/CIN taps; the
// per-lane tap offsets are compile-time constants once the K loop unrolls (see conv3d_lds_kernel).
// Round 6: the GeoBlock convs' depth plane (cat(g, y) / cat(x, g): 16+g -> 16 / 32 at half resolution, which ran on
// the gather kernel at 0.2-0.3 of their HBM roofline) as the gather kernel's trailing K chunk (one value per tap,
// rounded to the compute type), its (8+2) x (64+2) fp32 halo staged beside the tensor halo: the same MFMA sequence
// per accumulator as the gather kernel (chunks in packed order, then the plane chunk), so bitwise its results. bf16
// only: GeoFF stage 3 5.18 -> 4.99 ms, bench 205.9 -> 208.5 maps/s in one call (profiles/r06/ab_lds_plane).
constexpr int L2H = 8, L2W = 64, L2HH = L2H + 2, L2HW = L2W + 2;

template <int CH>
__device__ constexpr int halo2_toff(int t) {
  return t >= 9 ? halo2_toff<CH>(8) : ((t / 3) * L2HW + t % 3) * CH;
}

template <typename T, int CIN, int MT>
__global__ __launch_bounds__(256) DAMVS_WAVES((sizeof(T) != 2 ? 1 : CIN == 32 ? (MT == 2 ? 3 : 1) : MT == 1 ? 6 : 1)) void conv2d_lds_kernel(const Conv2dArgs a, int tiles_x, int tiles_y, int ntiles) {
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  constexpr int E = Stor<T>::E;
  constexpr int KC = 4 * E;
  constexpr int CH = CIN / E;  // 16-byte chunks per pixel
  constexpr int KCHUNKS = (9 * CIN + KC - 1) / KC;
  constexpr int ROW = L2HW * CH;
  constexpr int TILE_CHUNKS = L2HH * ROW;
  constexpr uint32_t ES = sizeof(T);
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  __shared__ raw tile[TILE_CHUNKS];
  __shared__ float ptile[L2HH * L2HW];  // the plane's halo (a.ngeo == 1)

  // XCD-aware bijective remap (consecutive tiles along x share an XCD and its L2)
  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y;
  const int b = tt / tiles_y;
  const int y0 = ty * L2H, x0 = tx * L2W;

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in0, (long long)a.B * a.Hi * a.Wi * CIN * ES);
  const int pin0 = b * a.Hi * a.Wi;
  stage_chunks<TILE_CHUNKS, 8>(tile, [&](int c) {
    const int row = c / ROW, col = c - row * ROW;
    const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
    const bool ok = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    const uint32_t off = (uint32_t)(((pin0 + iy * a.Wi + x0 - 1) * CH + col) * 16);
    return IO::frag(rin, ok ? off : kOOB);
  }, [](const raw& r) { return Frag2<T>::stage(r); });
  if (a.ngeo) {
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.geo[0], ((long long)(a.B - 1) * a.geo_bstride[0] + (long long)a.Hi * a.Wi) * 4);
    const int pg0 = b * (int)a.geo_bstride[0];
    for (int p = threadIdx.x; p < L2HH * L2HW; p += 256) {
      const int row = p / L2HW, col = p - row * L2HW;
      const int iy = y0 - 1 + row, ix = x0 - 1 + col;
      const bool ok = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      ptile[p] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, ok ? (uint32_t)(pg0 + iy * a.Wi + ix) * 4u : kOOB, 0, 0));
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  f32x4_t acc[L2H][MT];
#pragma unroll
  for (int j = 0; j < L2H; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const raw* tl = tile + (wave * 16 + n) * CH;
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + lane;
  const int gi = (g * E) / CIN;      // tap sub-index of this lane group (KC > CIN)
  const int gc = (g * E) % CIN / E;  // 16-byte channel chunk within the pixel
  auto fetch = [&](int s, raw* xf, raw* wf) {
#pragma unroll
    for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)(s * a.MTtot + m) * 64];
    const int kt = (s * KC) / CIN, kc = ((s * KC) % CIN) / E;
    int off = halo2_toff<CH>(kt);
    if (KC > CIN) {
      off = gi == 1 ? halo2_toff<CH>(kt + 1) : off;
      off = gi == 2 ? halo2_toff<CH>(kt + 2) : off;
      off = gi == 3 ? halo2_toff<CH>(kt + 3) : off;
    }
    // taps past the 9th (K padding) read a valid pixel against zero weights
    const raw* src = tl + off + kc + gc;
#pragma unroll
    for (int j = 0; j < L2H; ++j) xf[j] = src[j * ROW];
  };
  raw xa[L2H], wa[MT];
  fetch(0, xa, wa);
#pragma unroll
  for (int s = 0; s < KCHUNKS; ++s) {
    raw xb[L2H], wb[MT];
    if (s + 1 < KCHUNKS) fetch(s + 1, xb, wb);
#pragma unroll
    for (int j = 0; j < L2H; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) Frag2<T>::mma_staged(wa[m], xa[j], acc[j][m]);
    if (s + 1 < KCHUNKS) {
#pragma unroll
      for (int j = 0; j < L2H; ++j) xa[j] = xb[j];
#pragma unroll
      for (int m = 0; m < MT; ++m) wa[m] = wb[m];
    }
  }
  if (a.ngeo) {  // the plane chunk (packed after the tensor chunks): lane group g holds taps g E .. g E + E - 1
    static_assert(9 <= KC, "one plane chunk");
    raw wg[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wg[m] = wp[(size_t)(KCHUNKS * a.MTtot + m) * 64];
    const float* pt = ptile + wave * 16 + n;
#pragma unroll
    for (int j = 0; j < L2H; ++j) {
      float v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int t = g * E + e;
        v[e] = t < 9 ? pt[(j + t / 3) * L2HW + t % 3] : 0.f;
      }
      const raw x = pack_vals<T>(v);
#pragma unroll
      for (int m = 0; m < MT; ++m) Frag2<T>::mma(wg[m], x, acc[j][m]);
    }
  }

  // epilogue (as conv2d_mfma_kernel): bias, residual before ReLU, ReLU, residual after ReLU, store
  typedef typename IO::quad quad;
  const int up = a.post_up, us = a.post_up >> 1;
  const long long nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  float bias[MT][4];
  bool cok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = m * 16 + g * 4;
    cok[m] = co < a.cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = a.bias[co + i];  // padded to cout_pad
  }
  const int ox = x0 + wave * 16 + n;
#pragma unroll
  for (int j = 0; j < L2H; ++j) {
    const int oy = y0 + j;
    const bool vok = oy < a.Ho && ox < a.Wo;
    const int pout = (b * a.Ho + oy) * a.Wo + ox;
    const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
    quad qpre[MT], qpost[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const bool ok = vok && cok[m];
      const int co = m * 16 + g * 4;
      if (a.res_pre) qpre[m] = IO::ldq(rpre, ok ? (uint32_t)(pout * a.cout + co) * ES : kOOB);
      if (a.res_post) qpost[m] = IO::ldq(rpost, ok ? (uint32_t)(ppost * a.cout + co) * ES : kOOB);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][m][i], a.wscale, bias[m][i]);
      if (a.res_pre) IO::addq(qpre[m], r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) IO::addq(qpost[m], r);
      const uint32_t off = (uint32_t)(pout * a.cout + m * 16 + g * 4) * ES;
      IO::stq(ro, vok && cok[m] ? off : kOOB, r);
    }
  }
}

// LDS-staged x-pair transposed conv (round 6; bf16, and fp32 on the 16-K split form): the 16 -> 8 channel stride-2 ConvTranspose layers whose two
// x-pair phases (build_phases_xpair: py = 0, 1; MFMA row r = (x parity r >> 3, channel r & 7)) read input offsets
// -1 .. 1 -- GeoFeatureFusion's full-resolution k5 s2 decoders, which the x-pair gather kernel ran at ~0.2 of their
// HBM roofline (each input pixel fetched through L1 by every tap of both phases). A block owns 8 x 64 input-grid
// positions for BOTH phases: its (8+2) x (64+2) x 16-channel halo is read once (as conv2d_lds_kernel's), each phase's
// taps are looked up per lane and chunk from the phase's tap list (K entry s KC + g E = tap t, channel half), and the
// epilogue is the x-pair gather kernel's (lane group g + 1 hands its 4 channels to g; residuals, ReLU, 16-byte
// records). Per phase and accumulator the same MFMA sequence as the gather kernel (chunks in packed order, padding taps
// as zeros), so bitwise its results.
template <typename T>
__global__ __launch_bounds__(256) void conv2d_xpair_lds_kernel(const Conv2dArgs a, int tiles_x, int tiles_y, int ntiles) {
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  constexpr int E = Stor<T>::E, KC = 4 * E, CH = 16 / E;  // 16 channels: CH 16-byte chunks per pixel
  constexpr int ROW = L2HW * CH;
  constexpr int TILE_CHUNKS = L2HH * ROW;
  constexpr uint32_t ES = sizeof(T);
  __shared__ raw tile[TILE_CHUNKS];
  __shared__ int s_toff[2][16];  // per phase: tap t's halo offset in 16-byte chunks (-1: padding tap)

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y;
  const int b = tt / tiles_y;
  const int y0 = ty * L2H, x0 = tx * L2W;
  if (threadIdx.x < 32) {
    const int p = threadIdx.x >> 4, t = threadIdx.x & 15;
    s_toff[p][t] = t < a.ph[p].ntaps ? ((a.ph[p].tap[t][0] + 1) * L2HW + a.ph[p].tap[t][1] + 1) * CH : -1;
  }
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in0, (long long)a.B * a.Hi * a.Wi * 16 * ES);
  const int pin0 = b * a.Hi * a.Wi;
  stage_chunks<TILE_CHUNKS, 8>(tile, [&](int c) {
    const int row = c / ROW, col = c - row * ROW;
    const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
    const bool ok = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    const uint32_t off = (uint32_t)(((pin0 + iy * a.Wi + x0 - 1) * CH + col) * 16);
    return IO::frag(rin, ok ? off : kOOB);
  }, [](const raw& r) { return r; });
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const raw* tl = tile + (wave * 16 + n) * CH + (g * E) % 16 / E;  // the lane's column and channel chunk
  const long long nout = (long long)a.B * a.Ho * a.Wo * 8;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const int up = a.post_up, us = a.post_up >> 1;
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  float b8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b8[i] = a.bias[i];
  const int qx = x0 + wave * 16 + n;
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    const Conv2dPhase& ph = a.ph[p];
    const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + (size_t)ph.w_off * 64 + lane;  // MTtot 1
    f32x4_t acc[L2H];
#pragma unroll
    for (int j = 0; j < L2H; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < ph.kchunks; ++s) {
      const raw w = wp[(size_t)s * 64];
      const int off = s_toff[p][(s * KC + g * E) >> 4];  // 16 channels a tap (bf16: lane group g holds tap 2 s + (g >> 1))
      raw x[L2H];
#pragma unroll
      for (int j = 0; j < L2H; ++j) x[j] = off >= 0 ? tl[off + j * ROW] : Frag2<T>::zero();
#pragma unroll
      for (int j = 0; j < L2H; ++j) Frag2<T>::mma(w, x[j], acc[j]);
    }
    // epilogue (the x-pair gather kernel's): output x = 2 qx + (g >> 1), y = 2 qy + py
    const int ox = 2 * qx + (g >> 1);
    if constexpr (sizeof(T) == 4) {  // fp32: every lane its 4 channels (16 bytes) of channel half g & 1
      const int ch = (g & 1) * 4;
#pragma unroll
      for (int j = 0; j < L2H; ++j) {
        float r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][i], a.wscale, b8[ch + i]);
        const int qy = y0 + j, oy = 2 * qy + ph.py;
        const bool ok = qy < a.Hi && qx < a.Wi && oy < a.Ho && ox < a.Wo;
        const int pout = (b * a.Ho + oy) * a.Wo + ox;
        const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
        const uint32_t o = ok ? (uint32_t)(pout * 8 + ch) * ES : kOOB;
        if (a.res_pre) IO::addq(IO::ldq(rpre, o), r);
        if (a.relu) {
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
        }
        if (a.res_post) IO::addq(IO::ldq(rpost, ok ? (uint32_t)(ppost * 8 + ch) * ES : kOOB), r);
        IO::stq(ro, o, r);
      }
    } else {
      const bool lead = (g & 1) == 0;
#pragma unroll
      for (int j = 0; j < L2H; ++j) {
        float r[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          r[i] = fmaf(acc[j][i], a.wscale, b8[i]);
          r[4 + i] = fmaf(__shfl_down(acc[j][i], 16), a.wscale, b8[4 + i]);
        }
        if (!lead) continue;
        const int qy = y0 + j, oy = 2 * qy + ph.py;
        const bool ok = qy < a.Hi && qx < a.Wi && oy < a.Ho && ox < a.Wo;
        const int pout = (b * a.Ho + oy) * a.Wo + ox;
        const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
        if (a.res_pre) Vox8<T>::add(rpre, ok ? (uint32_t)(pout * 8) * ES : kOOB, r);
        if (a.relu) {
#pragma unroll
          for (int i = 0; i < 8; ++i) r[i] = relu(r[i]);
        }
        if (a.res_post) Vox8<T>::add(rpost, ok ? (uint32_t)(ppost * 8) * ES : kOOB, r);
        Vox8<T>::store(ro, ok ? (uint32_t)(pout * 8) * ES : kOOB, r);
      }
    }
  }
}

// LDS-staged variant for the thin stride-2 5x5 convs (one tensor input of CIN 8 or 16 channels, padding 2, no plane):
// FeatureNet's downsampling convs conv1.0 (8 -> 16 at 1184 x 1600) and conv2.0 (16 -> 32 at 592 x 800), which the
// gather kernel runs at 0.3 of their HBM roofline (each input pixel fetched by ~6 output pixels' taps through L1;
// models/module.py FeatureNet). A block owns a TR-row x 64-column output tile; its (2 TR + 3) x 131-pixel input halo is
// read once with 16-byte loads (zero padding by range-checked buffer loads) and every B fragment is a ds_read_b128.
// Each halo row is stored as its even then its odd columns (66 pixels each), so the 16 lanes of an N-group (16
// consecutive output columns, input columns 2 apart) read 16 consecutive LDS pixels at every tap. Wave w owns columns
// [16w, 16w + 16), group j output row j; a K chunk spans KC / CIN taps (per-lane tap offsets are compile-time constants
// once the K loop unrolls, as in conv2d_lds_kernel).
constexpr int S2W = 64, S2NC = 2 * (S2W - 1) + 5, S2HCP = (S2NC + 1) / 2, S2PITCH = 2 * S2HCP;

template <int CH>
__device__ constexpr int s2_toff(int t) {  // tap t = (ty, tx) of the 5 x 5 block, in 16-byte chunks
  return t >= 25 ? s2_toff<CH>(24) : ((t / 5) * S2PITCH + (t % 5 & 1) * S2HCP + (t % 5 >> 1)) * CH;
}

template <typename T, int CIN, int MT, int TR>
__global__ __launch_bounds__(256) void conv2d_lds_s2_kernel(const Conv2dArgs a, int tiles_x, int tiles_y, int ntiles) {
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  constexpr int E = Stor<T>::E;
  constexpr int KC = 4 * E;
  constexpr int CH = CIN / E;  // 16-byte chunks per pixel
  constexpr int KCHUNKS = (25 * CIN + KC - 1) / KC;
  constexpr int HR = 2 * (TR - 1) + 5;
  constexpr int ROW = S2PITCH * CH;
  constexpr int TILE_CHUNKS = HR * ROW;
  constexpr uint32_t ES = sizeof(T);
  static_assert(KC % CIN == 0, "a K chunk spans whole taps");
  __shared__ raw tile[TILE_CHUNKS];

  // XCD-aware bijective remap (consecutive tiles along x share an XCD and its L2)
  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x;
  tt /= tiles_x;
  const int ty = tt % tiles_y;
  const int b = tt / tiles_y;
  const int y0 = ty * TR, x0 = tx * S2W;
  const int iy0 = 2 * y0 - 2, ix0 = 2 * x0 - 2;

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in0, (long long)a.B * a.Hi * a.Wi * CIN * ES);
  const int pin0 = b * a.Hi * a.Wi;
  stage_chunks<TILE_CHUNKS, 8>(tile, [&](int c) {
    const int row = c / ROW, rem = c - row * ROW;
    const int p = rem / CH, ch = rem - p * CH;
    const int par = p >= S2HCP;
    const int col = 2 * (p - par * S2HCP) + par;
    const int iy = iy0 + row, ix = ix0 + col;
    const bool ok = col < S2NC && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    const uint32_t off = (uint32_t)(((pin0 + iy * a.Wi + ix) * CH + ch) * 16);
    return IO::frag(rin, ok ? off : kOOB);
  }, [](const raw& r) { return Frag2<T>::stage(r); });
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  f32x4_t acc[TR][MT];
#pragma unroll
  for (int j = 0; j < TR; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const raw* tl = tile + (wave * 16 + n) * CH;
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + lane;
  const int gi = (g * E) / CIN;      // tap sub-index of this lane group
  const int gc = (g * E) % CIN / E;  // 16-byte channel chunk within the pixel
  auto fetch = [&](int s, raw* xf, raw* wf) {
#pragma unroll
    for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)(s * a.MTtot + m) * 64];
    const int kt = (s * KC) / CIN;
    int off = s2_toff<CH>(kt);
    if constexpr (KC / CIN > 1) off = gi == 1 ? s2_toff<CH>(kt + 1) : off;
    if constexpr (KC / CIN > 2) {
      off = gi == 2 ? s2_toff<CH>(kt + 2) : off;
      off = gi == 3 ? s2_toff<CH>(kt + 3) : off;
    }
    // taps past the 25th (K padding) read a valid pixel against zero weights
    const raw* src = tl + off + gc;
#pragma unroll
    for (int j = 0; j < TR; ++j) xf[j] = src[2 * j * ROW];
  };
  raw xa[TR], wa[MT];
  fetch(0, xa, wa);
#pragma unroll
  for (int s = 0; s < KCHUNKS; ++s) {
    raw xb[TR], wb[MT];
    if (s + 1 < KCHUNKS) fetch(s + 1, xb, wb);
#pragma unroll
    for (int j = 0; j < TR; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) Frag2<T>::mma_staged(wa[m], xa[j], acc[j][m]);
    if (s + 1 < KCHUNKS) {
#pragma unroll
      for (int j = 0; j < TR; ++j) xa[j] = xb[j];
#pragma unroll
      for (int m = 0; m < MT; ++m) wa[m] = wb[m];
    }
  }

  // epilogue (as conv2d_lds_kernel)
  typedef typename IO::quad quad;
  const int up = a.post_up, us = a.post_up >> 1;
  const long long nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  float bias[MT][4];
  bool cok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = m * 16 + g * 4;
    cok[m] = co < a.cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = a.bias[co + i];  // padded to cout_pad
  }
  const int ox = x0 + wave * 16 + n;
#pragma unroll
  for (int j = 0; j < TR; ++j) {
    const int oy = y0 + j;
    const bool vok = oy < a.Ho && ox < a.Wo;
    const int pout = (b * a.Ho + oy) * a.Wo + ox;
    const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
    quad qpre[MT], qpost[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const bool ok = vok && cok[m];
      const int co = m * 16 + g * 4;
      if (a.res_pre) qpre[m] = IO::ldq(rpre, ok ? (uint32_t)(pout * a.cout + co) * ES : kOOB);
      if (a.res_post) qpost[m] = IO::ldq(rpost, ok ? (uint32_t)(ppost * a.cout + co) * ES : kOOB);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][m][i], a.wscale, bias[m][i]);
      if (a.res_pre) IO::addq(qpre[m], r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) IO::addq(qpost[m], r);
      const uint32_t off = (uint32_t)(pout * a.cout + m * 16 + g * 4) * ES;
      IO::stq(ro, vok && cok[m] ? off : kOOB, r);
    }
  }
}

// Halo-tiled implicit GEMM for the wide layers (Cin a multiple of KC, in_stride 1: GeoFeatureFusion's
// stride-1 GeoBlock convs, k3/k5 decoders and the k5 s2 transposed decoders' phases). A block owns a
// 4-row x 64-column tile of the q-grid for one phase and MT 16-channel output tiles; wave w owns
// columns [16w, 16w+16) and group j row j (wave tile MT x 4 MFMA tiles, as conv2d_mfma_kernel). K
// runs over Cin slices of KC channels: each slice's input halo ((4 + span) x (64 + span) pixels x KC
// channels, one 16-byte chunk per lane group) is staged in LDS once and feeds every tap of the phase
// (the gather kernel re-fetches each input pixel once per tap through L1), double-buffered so slice
// c+1 streams in during slice c's MFMAs. A fragments come from global (L2-resident packed weights,
// one coalesced 1 KB load per MFMA tile), prefetched one tap ahead. The fp32 plane, if any, runs as
// the trailing K chunk(s) with global loads.
constexpr int HGR = 4, HGC = 64;  // q-tile rows (one per group) x columns (16 per wave)

// WM: waves stacked along the output channels (1: 4 waves side by side over the 4 column groups,
// each with MT cout tiles x 4 rows; 2: a 2 x 2 wave grid, each wave MT cout tiles x 2 column groups x
// 4 rows — half the A (weight) stream per MFMA for the wide layers).
// W32 (T = float, the fp32 path's 32-K form: a.wide32, the layer's 32-K split packing): K chunks of 32 channels as
// split-f16 MFMAs (mma_split32, 16x16x32 at full rate) instead of the 16-K form's three 16x16x16 per 16 channels; a
// halo pixel keeps each 8-channel chunk as its f16 hi / lo halves in 8 slots, slot s at s ^ ((pixel >> 1) & 7) (the
// 16 lanes of an N-group read 16 consecutive pixels); one halo buffer, rewritten between two barriers after a slice's
// last tap (twice the bytes of the bf16 tile).
// RS (W32 only): the rolling tap loop -- tap offsets by v_readlane, each N-group's B pair for the next tap read as soon
// as that group's MFMAs are issued (pinned by sched_group_barrier), the next tap's A pairs loaded before the MFMAs; the
// same MFMA sequence per accumulator as the plain W32 loop, so bitwise equal (DAMVS_HALO_RS=0 selects that loop).
template <typename T, int MT, int WM, bool TWO, bool W32 = false, bool RS = false>
__global__ __launch_bounds__(256) void conv2d_halo_kernel(const Conv2dArgs a, int tiles_x, int tiles_y, int nsl,
                                                          int dmin, int span) {
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  typedef typename std::conditional<W32, F16Pair, raw>::type frag;
  static_assert(!W32 || sizeof(T) == 4, "32-K split form: fp32 storage");
  constexpr int E = Stor<T>::E;
  constexpr int KC = W32 ? 32 : 4 * E;
  constexpr int SL = W32 ? 8 : 4;   // 16-byte LDS slots per halo pixel and slice
  constexpr int CE = KC / 4;        // channels per lane group and chunk
  constexpr uint32_t ES = sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  raw* buf = reinterpret_cast<raw*>(smem);
  uint4* ubuf = reinterpret_cast<uint4*>(smem);
  const int HR = HGR + span - 1, HC = HGC + span - 1;  // halo rows / columns
  const int HP = HR * HC;                               // halo pixels (4 chunks each)
  auto wslot = [](int p, int q) { return q ^ ((p >> 1) & 7); };

  // logical block = (tile, phase), phase fastest, XCD-contiguous
  const int ntile = tiles_x * tiles_y * a.B;
  const int nblk = ntile * a.nphase;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tl = L / a.nphase;
  const Conv2dPhase& ph = a.ph[L - tl * a.nphase];
  const int tx = tl % tiles_x, ty = (tl / tiles_x) % tiles_y, b = tl / (tiles_x * tiles_y);
  const int qy0 = ty * HGR, qx0 = tx * HGC;
  constexpr int WN = 4 / WM, CG = 4 / WN, GW = HGR * CG;  // waves along N, column groups and groups per wave
  const int wm = (threadIdx.x >> 6) / WN, wn = (threadIdx.x >> 6) % WN;
  const int mt0 = blockIdx.y * (MT * WM) + wm * MT;

  __shared__ int s_toff[32];  // tap offset inside the halo, in pixels
  if (threadIdx.x < 25)
    s_toff[threadIdx.x] = threadIdx.x < ph.ntaps ? (ph.tap[threadIdx.x][0] - dmin) * HC + (ph.tap[threadIdx.x][1] - dmin) : 0;

  // halo fill of slice c into buffer bi: pixel p = (row, col), 4 chunks of CE channels
  const int npix = a.B * a.Hi * a.Wi;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.in0, (long long)npix * a.c0 * ES);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(TWO ? a.in1 : a.in0, TWO ? (long long)npix * a.c1 * ES : 0);
  const int iy0 = qy0 + dmin, ix0 = qx0 + dmin, pb = b * a.Hi * a.Wi;
  constexpr int PER = 8;             // chunks per thread per fill (covers 2048 chunks = 512 halo pixels)
  constexpr int NR = W32 ? 2 : 1;    // 16-byte loads per chunk
  raw regs[PER][NR];
  auto gfill = [&](int c) {
    const bool second = TWO && c * KC >= a.c0;
    const int cs = second ? a.c1 : a.c0, cb = (second ? c * KC - a.c0 : c * KC);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * 256;
      const int p = i >> 2, part = i & 3;
      const int row = p / HC, col = p - row * HC;
      const int iy = iy0 + row, ix = ix0 + col;
      const bool ok = p < HP && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((pb + iy * a.Wi + ix) * cs + cb + part * CE) * ES;
#pragma unroll
      for (int h = 0; h < NR; ++h) {
        const uint32_t o = ok ? off + 16u * h : kOOB;
        regs[k][h] = (TWO && second) ? IO::frag(r1, o) : IO::frag(r0, o);
      }
    }
  };
  auto lstore = [&](int bi) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * 256;
      const int p = i >> 2, part = i & 3;
      if (p >= HP) continue;
      if constexpr (W32) {
        const F16Pair v = split8(regs[k][0], regs[k][1]);
        uint4* px = ubuf + (bi * HP + p) * 8;
        px[wslot(p, part)] = v.h;
        px[wslot(p, part + 4)] = v.l;
      } else {
        buf[bi * HP * 4 + i] = Frag2<T>::stage(regs[k][0]);
      }
    }
  };

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  f32x4_t acc[GW][MT];
#pragma unroll
  for (int j = 0; j < GW; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // A: 16-K form [chunk][tile][lane] raw fragments; W32 [chunk][tile][hi: 64 lanes][lo: 64 lanes]
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 64 + lane;
  const uint4* __restrict__ wp32 =
      reinterpret_cast<const uint4*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 128 + lane;
  auto wload = [&](int chunk, int m) -> frag {
    if constexpr (W32) {
      const uint4* q = wp32 + ((size_t)chunk * a.MTtot + m) * 128;
      return F16Pair{q[0], q[64]};
    } else {
      return wp[((size_t)chunk * a.MTtot + m) * 64];
    }
  };
  const int nt = ph.ntaps;
  const int pcol = wn * CG * 16 + n;             // this lane's halo pixel column offset (row 0, first column + n)
  const int lbase = pcol * 4 + g;                // 16-K form: its chunk
  constexpr int NHB = W32 ? 1 : 2;
  (void)wave;

  gfill(0);
  lstore(0);
  __syncthreads();
  if constexpr (RS) {
    static_assert(W32, "rolling tap loop: the 32-K form");
    const int ltoff = lane < nt ? (ph.tap[lane][0] - dmin) * HC + (ph.tap[lane][1] - dmin) : 0;  // lane t: tap t
    auto bread = [&](int t, frag (&xf)[GW]) DAMVS_INLINE {  // B pairs of tap t (one halo buffer)
      const int to = __builtin_amdgcn_readlane(ltoff, t) + pcol;
#pragma unroll
      for (int j = 0; j < GW; ++j) {
        const int pl = to + (j % HGR) * HC + (j / HGR) * 16;
        const uint4* px = ubuf + pl * 8;
        xf[j] = F16Pair{px[wslot(pl, g)], px[wslot(pl, g + 4)]};
      }
    };
    for (int c = 0; c < nsl; ++c) {
      if (c + 1 < nsl) gfill(c + 1);
      frag wf[MT], xf[GW];
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wload(c, m);  // chunk (tap 0, slice c)
      bread(0, xf);
      for (int t = 0; t < nt; ++t) {
        const int t1 = t + 1 < nt ? t + 1 : t;  // past the last tap: a harmless re-read
        frag wn2[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) wn2[m] = wload(t1 * nsl + c, m);
        const int to = __builtin_amdgcn_readlane(ltoff, t1) + pcol;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < GW; ++j) {
#pragma unroll
          for (int m = 0; m < MT; ++m) mma_split32(wf[m], xf[j], acc[j][m]);
          const int pl = to + (j % HGR) * HC + (j / HGR) * 16;
          const uint4* px = ubuf + pl * 8;
          xf[j] = F16Pair{px[wslot(pl, g)], px[wslot(pl, g + 4)]};
        }
#pragma unroll
        for (int j = 0; j < GW; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * MT, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < MT; ++m) wf[m] = wn2[m];
      }
      if (c + 1 < nsl) {
        __syncthreads();  // every wave is done with slice c's halo
        lstore(0);
        __syncthreads();
      }
    }
  } else
  for (int c = 0; c < nsl; ++c) {
    if (c + 1 < nsl) gfill(c + 1);
    const int bi = NHB == 2 ? (c & 1) : 0;
    frag wf[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wf[m] = wload(c, m);  // chunk (tap 0, slice c)
    for (int t = 0; t < nt; ++t) {
      frag wn2[MT];
      if (t + 1 < nt) {
#pragma unroll
        for (int m = 0; m < MT; ++m) wn2[m] = wload((t + 1) * nsl + c, m);
      }
      frag xf[GW];  // group j: row j % HGR, column group j / HGR of this wave
      if constexpr (W32) {
#pragma unroll
        for (int j = 0; j < GW; ++j) {
          const int pl = s_toff[t] + (j % HGR) * HC + (j / HGR) * 16 + pcol;
          const uint4* px = ubuf + (bi * HP + pl) * 8;
          xf[j] = F16Pair{px[wslot(pl, g)], px[wslot(pl, g + 4)]};
        }
      } else {
        const raw* hb = buf + bi * HP * 4 + lbase;
        const int to = s_toff[t] * 4;
#pragma unroll
        for (int j = 0; j < GW; ++j) xf[j] = hb[to + ((j % HGR) * HC + (j / HGR) * 16) * 4];
      }
#pragma unroll
      for (int j = 0; j < GW; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if constexpr (W32) mma_split32(wf[m], xf[j], acc[j][m]);
          else Frag2<T>::mma_staged(wf[m], xf[j], acc[j][m]);
        }
      if (t + 1 < nt) {
#pragma unroll
        for (int m = 0; m < MT; ++m) wf[m] = wn2[m];
      }
    }
    if (c + 1 < nsl) {
      if (NHB == 1) __syncthreads();  // every wave is done with slice c's halo
      lstore(NHB == 2 ? (c + 1) & 1 : 0);  // (NHB 2: buffer (c + 1) & 1 was last read before the previous barrier)
      __syncthreads();
    }
  }

  // the fp32 plane as trailing K chunks (tap x plane), as in conv2d_mfma_kernel
  if (ph.gchunks > 0) {
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.geo[0], ((long long)(a.B - 1) * a.geo_bstride[0] + a.Hi * a.Wi) * 4);
    const int pg0 = b * (int)a.geo_bstride[0];
    for (int s = 0; s < ph.gchunks; ++s) {
      frag wf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wload(ph.kchunks + s, m);
      float v[GW][CE];
#pragma unroll
      for (int e = 0; e < CE; ++e) {
        const int t = s * KC + g * CE + e;
        const bool tv = t < nt;
        const int dy = tv ? ph.tap[t][0] : 0, dx = tv ? ph.tap[t][1] : 0;
#pragma unroll
        for (int j = 0; j < GW; ++j) {
          const int iy = qy0 + j % HGR + dy, ix = qx0 + (wn * CG + j / HGR) * 16 + n + dx;
          const bool ok = tv && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
          v[j][e] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rg, ok ? (uint32_t)(pg0 + iy * a.Wi + ix) * 4u : kOOB, 0, 0));
        }
      }
#pragma unroll
      for (int j = 0; j < GW; ++j) {
        if constexpr (W32) {
          const F16Pair xf = split8(v[j]);
#pragma unroll
          for (int m = 0; m < MT; ++m) mma_split32(wf[m], xf, acc[j][m]);
        } else {
          const raw xf = pack_vals<T>(v[j]);
#pragma unroll
          for (int m = 0; m < MT; ++m) Frag2<T>::mma(wf[m], xf, acc[j][m]);
        }
      }
    }
  }
  // epilogue (as conv2d_mfma_kernel)
  typedef typename IO::quad quad;
  const int up = a.post_up, us = a.post_up >> 1;
  const long long nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  float bias[MT][4];
  bool cok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = (mt0 + m) * 16 + g * 4;
    cok[m] = co < a.cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = a.bias[co + i];
  }
#pragma unroll
  for (int j = 0; j < GW; ++j) {
    const int qy = qy0 + j % HGR, qx = qx0 + (wn * CG + j / HGR) * 16 + n;
    const int oy = qy * a.out_stride + ph.py, ox = qx * a.out_stride + ph.px;
    const bool vok = qy < a.Hq && qx < a.Wq;
    const int pout = (b * a.Ho + oy) * a.Wo + ox;
    const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
    quad qpre[MT], qpost[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const bool ok = vok && cok[m];
      const int co = (mt0 + m) * 16 + g * 4;
      if (a.res_pre) qpre[m] = IO::ldq(rpre, ok ? (uint32_t)(pout * a.cout + co) * ES : kOOB);
      if (a.res_post) qpost[m] = IO::ldq(rpost, ok ? (uint32_t)(ppost * a.cout + co) * ES : kOOB);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaf(acc[j][m][i], a.wscale, bias[m][i]);
      if (a.res_pre) IO::addq(qpre[m], r);
      if (a.relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = relu(r[i]);
      }
      if (a.res_post) IO::addq(qpost[m], r);
      const uint32_t off = (uint32_t)(pout * a.cout + (mt0 + m) * 16 + g * 4) * ES;
      IO::stq(ro, vok && cok[m] ? off : kOOB, r);
    }
  }
}

template <typename T, int MT, int WM, bool W32 = false, bool RS = false>
hipError_t launch_halo_t(hipStream_t s, const Conv2dArgs& a, int dmin, int span) {
  constexpr int KC = W32 ? 32 : 4 * Stor<T>::E;
  const int tx = (a.Wq + HGC - 1) / HGC, ty = (a.Hq + HGR - 1) / HGR;
  const int nsl = (a.c0 + a.c1) / KC;
  const size_t hp = (size_t)(HGR + span - 1) * (HGC + span - 1);
  const size_t smem = W32 ? hp * 8 * 16 : (nsl > 1 ? 2 : 1) * hp * 4 * 16;  // one slice (or W32): one buffer
  const long long nblk = (long long)tx * ty * a.B * a.nphase;
  const dim3 grid((unsigned)nblk, (unsigned)(a.MTtot / (MT * WM)));
  auto k = a.c1 > 0 ? conv2d_halo_kernel<T, MT, WM, true, W32, RS> : conv2d_halo_kernel<T, MT, WM, false, W32, RS>;
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)smem);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), smem, s, a, tx, ty, nsl, dmin, span);
  return hipGetLastError();
}

// Returns hipErrorNotSupported when the halo kernel does not take the layer. W32: the fp32 layer's 32-K split form.
template <typename T, bool W32 = false>
hipError_t launch_halo(hipStream_t s, const Conv2dArgs& a, bool dry = false) {
  constexpr int KC = W32 ? 32 : 4 * Stor<T>::E;
  // largest cout tile count (MTtot) the halo kernel takes: its B reuse pays off for narrow outputs,
  // while wide outputs are bound by the A (weight) stream the gather kernel already amortises
  constexpr int max_mt = 2;  // (8: the wide layers too, measured 192-194 against 203-204 maps/s in round 3)
  // one-slice inputs (Cin = KC) and single cout tiles as well: the half-resolution GeoBlock convs with a depth
  // plane (32+g -> 32: 173 -> 146 us, 32+g -> 16: 101 -> 79 us at B=4); DAMVS_CONV2D_HALO_THIN=0 restores the
  // gather kernel for them
  static const bool thin = [] {
    const char* v = getenv("DAMVS_CONV2D_HALO_THIN");
    return !(v && v[0] == '0');
  }();
  if (a.MTtot > max_mt || (a.MTtot > 2 && a.MTtot < 8) || a.in_stride != 1 || a.c0 % KC || a.c1 % KC ||
      a.c0 + a.c1 < (thin ? KC : 2 * KC) || a.MTtot < (thin ? 1 : 2) || a.ngeo > 1)
    return hipErrorNotSupported;
  int dmin = 0, dmax = 0;
  for (int p = 0; p < a.nphase; ++p)
    for (int t = 0; t < a.ph[p].ntaps; ++t)
      for (int d = 0; d < 2; ++d) {
        dmin = a.ph[p].tap[t][d] < dmin ? a.ph[p].tap[t][d] : dmin;
        dmax = a.ph[p].tap[t][d] > dmax ? a.ph[p].tap[t][d] : dmax;
      }
  const int span = dmax - dmin + 1;
  if ((HGR + span - 1) * (HGC + span - 1) > 512) return hipErrorNotSupported;  // PER = 8 fill pieces a thread
  // cout tile as wide as keeps about one wave per SIMD busy (the tile count is small for these layers)
  const long long tiles = (long long)((a.Wq + HGC - 1) / HGC) * ((a.Hq + HGR - 1) / HGR) * a.B * a.nphase;
  if (dry) return (a.MTtot >= 8 ? a.MTtot % 8 == 0 : (W32 ? a.MTtot <= 2 : true)) ? hipSuccess : hipErrorNotSupported;
  if constexpr (W32) {  // fp32 32-K form: the narrow layers (cout <= 32); the rolling tap loop unless DAMVS_HALO_RS=0
    const char* rv = getenv("DAMVS_HALO_RS");  // (read per call: the bitwise test flips it)
    const bool rs = !(rv && rv[0] == '0');
    if (a.MTtot == 2) return rs ? launch_halo_t<T, 2, 1, true, true>(s, a, dmin, span) : launch_halo_t<T, 2, 1, true>(s, a, dmin, span);
    if (a.MTtot == 1) return rs ? launch_halo_t<T, 1, 1, true, true>(s, a, dmin, span) : launch_halo_t<T, 1, 1, true>(s, a, dmin, span);
    return hipErrorNotSupported;
  }
  if (a.MTtot >= 8) {  // wide: 2 x 2 wave grid, 4 cout tiles x 128 pixels a wave
    if (a.MTtot % 8 == 0) return launch_halo_t<T, 4, 2>(s, a, dmin, span);
    return hipErrorNotSupported;
  }
  if (T_is_bf16<T>::value && a.MTtot % 8 == 0 && tiles * (a.MTtot / 8) >= 240) return launch_halo_t<T, 8, 1>(s, a, dmin, span);
  if (a.MTtot % 4 == 0 && tiles * (a.MTtot / 4) >= 240) return launch_halo_t<T, 4, 1>(s, a, dmin, span);
  if (a.MTtot % 2 == 0) return launch_halo_t<T, 2, 1>(s, a, dmin, span);
  if (a.MTtot == 1) return launch_halo_t<T, 1, 1>(s, a, dmin, span);
  return hipErrorNotSupported;
}

// Wide-layer implicit GEMM (bf16; 128-channel cout blocks; Cin slices of 32; in_stride 1): the stride-1
// GeoBlock convs at 128-256 channels and the k5 s2 transposed decoders' phases of GeoFeatureFusion
// (models/geometry.py:381-433,475-480). A block owns 128 output channels x a 2-row x 64-column tile of
// one phase's q-grid; its 4 waves form a 2 x 2 grid (wave (wm, wn): 4 cout tiles x q-row wn = 64 pixels,
// 4 MFMA N-groups). Both MFMA operands come from LDS:
//  * A: the block's 8 cout tiles of one K chunk (tap, 32-channel slice) = 8 KB of packed fragments, copied
//    once per block (buffer loads at a wave-uniform SGPR offset, two chunks ahead, into alternating
//    register pairs; written one chunk ahead) and read by the two waves of each cout half (the gather
//    kernel streams 8 KB per wave per chunk through L1);
//  * B: the slice's input halo ((2 + span - 1) x (64 + span - 1) pixels x 64 B), staged once per slice and
//    read at every tap's offset; a pixel's 16-byte chunk sits at position chunk ^ ((pixel >> 2) & 3) so the
//    16 lanes of a quarter-wave (16 consecutive pixels, one chunk) hit distinct banks.
// One barrier per K chunk. The depth plane's halo is staged once per block; the plane chunk's weights come
// straight from global memory after the K loop. Epilogue through LDS: each wave stages its 64 x 64 fp32 tile
// and every lane finishes one pixel's 32-channel half (bias, residuals, ReLU) with 16-byte residual loads and
// stores (the accumulator layout holds 4 channels of a pixel per lane: 8-byte accesses 16 pixels apart; GeoFF
// stage 3 5.93 -> 5.73 ms); the launcher therefore takes only cout % 32 == 0. (Reading chunk k + 1's fragments
// during chunk k's MFMAs measured no faster: 271 against 268 us on case N. An LDS-DMA variant measured slower: hipcc drains every outstanding DMA before each LDS read it cannot
// prove disjoint. Two q-rows per wave, 32 MFMAs a chunk, needed 182 VGPRs + 128 AGPRs: one wave per SIMD,
// 318 against 270 us on case N.)
#ifndef DAMVS_WIDE_DIAG
#define DAMVS_WIDE_DIAG 0  // diagnostic builds only (tools/build_diag_wide.sh): skip parts of the K loop
#endif
constexpr int WC = 64, WR = 2;  // q-tile columns x rows
// A wave whose q-columns past the grid leave it at most one valid 16-column N-group (the last tile column of the 200-
// and 400-column grids of GeoFF stage 3: 8 / 16 valid columns of 64) runs its K loop on that N-group alone: no MFMAs
// and B reads for the other three (2 or 3 valid groups run all 4). The fp32 rolling loop and the stride-2 AG loops; not
// the stride-1 AG loops, whose second loop copy spilled (60-75 VGPRs). Build with -DDAMVS_WIDE_NG_SKIP=0 for the A/B.
#ifndef DAMVS_WIDE_NG_SKIP
#define DAMVS_WIDE_NG_SKIP 1
#endif
constexpr bool WIDE_NG_SKIP = DAMVS_WIDE_NG_SKIP;

// Input halo geometry of a WR x WC q-tile for taps spanning `span` input pixels (IS = input stride). Stride 1: rows of
// WC + span - 1 pixels. Stride 2: 2 (WR - 1) + span rows of 2 (WC - 1) + span columns, each row stored as its even
// columns then its odd columns (hcp pixels each), so the 16 lanes of an N-group (16 consecutive q-columns) read 16
// consecutive LDS pixels at every tap, as at stride 1.
template <int IS, int WRT = WR>
struct WideHalo {
  int pitch, hcp, rows, ncols, hp;
  __host__ __device__ WideHalo(int span) {
    if (IS == 1) {
      ncols = WC + span - 1, hcp = ncols, pitch = ncols, rows = WRT + span - 1;
    } else {
      ncols = 2 * (WC - 1) + span, hcp = (ncols + 1) / 2, pitch = 2 * hcp, rows = 2 * (WRT - 1) + span;
    }
    hp = rows * pitch;
  }
  // LDS pixel of halo (row, column c)
  __host__ __device__ int pix(int row, int c) const { return IS == 1 ? row * pitch + c : row * pitch + (c & 1) * hcp + (c >> 1); }
  // halo (row, column) of LDS pixel p; column -1 for the odd half's padding slot
  __device__ void rc(int p, int& row, int& c) const {
    row = p / pitch;
    const int r = p - row * pitch;
    if (IS == 1) {
      c = r;
    } else {
      const int par = r >= hcp;
      c = 2 * (r - par * hcp) + par;
      c = c < ncols ? c : -1;
    }
  }
};

// Storage forms of the wide kernel. bf16: a K fragment is 8 bf16 channels (one 16-byte slot), 4 slots per halo pixel
// and slice, chunk slot s at s ^ ((p >> 2) & 3). fp32 (T = float): every product on split-f16 MFMAs (damvs_device.h,
// mma_split32): a fragment is the hi and lo halves of 8 channels (two slots), 8 slots per halo pixel and slice (hi of
// chunk s in slot s, lo in slot 4 + s), slot position q at q ^ ((p >> 1) & 7): the 16 lanes of an N-group (16
// consecutive pixels, 128 bytes apart) then read 16 distinct 16-byte bank groups. The A chunk of a cout tile is
// [hi: 64 lanes x 16 B][lo: 64 lanes x 16 B] (pack_2d at 32 K per chunk, split_weights_blocked).
template <typename T> struct WideForm;
template <> struct WideForm<bf16_t> {
  static constexpr int PL = 1, SLOTS = 4;  // 16-byte pieces per 8-channel fragment; LDS slots per pixel
  __device__ __forceinline__ static int slot(int p, int q) { return q ^ ((p >> 2) & 3); }
};
template <> struct WideForm<float> {
  static constexpr int PL = 2, SLOTS = 8;
  __device__ __forceinline__ static int slot(int p, int q) { return q ^ ((p >> 1) & 7); }
};

// WM = 2: a block owns 128 output channels x a 2 x 64 q-tile, its 4 waves a 2 x 2 grid (cout half, q-row); WM = 1:
// 64 output channels (cout 64 layers) x a 4 x 64 q-tile, the 4 waves one q-row each; WM = 1 at input stride 2 (the
// 4-row halo would not fit): a 2 x 64 q-tile, the 4 waves a 2 x 2 grid (q-row, 32-column half).
// T = float: the fp32 parity path's form (one halo buffer, rewritten between two barriers after a slice's last tap).
// RS (fp32, input stride 1, 128-channel block, taps spanning <= 3 pixels, >= 4 taps per phase): the rolling K loop
// below (A one chunk ahead, B of the next chunk read as each N-group's MFMAs finish, the next slice's halo in two
// 8-channel pieces per tap for the first taps of a slice, one barrier per slice).
// R1 (fp32, input stride 2, 128-channel block): a 1 x 64 q-tile, the 4 waves a 2 x 2 grid (cout half, 32-column half):
// a 390-pixel halo (50 KB) instead of the 2-row tile's 650 (83 KB), so two blocks share a CU.
template <typename T, bool TWO, int IS, int WM, bool RS = false, bool R1 = false>
__global__ __launch_bounds__(256) DAMVS_WAVES(sizeof(T) == 4 ? (IS == 1 || R1 ? 2 : 1) : IS == 1 ? 3 : 2) void conv2d_wide_kernel(
    const Conv2dArgs a, int tiles_x, int tiles_y, int nsl, int dmin, int span) {
  typedef uint4 raw;
  typedef WideForm<T> Fm;
  constexpr bool SP = sizeof(T) == 4;
  static_assert(!RS || (SP && IS == 1 && WM == 2), "rolling K loop: fp32, input stride 1, 128-channel block");
  constexpr int PL = Fm::PL, SLOTS = Fm::SLOTS;
  constexpr uint32_t ES = sizeof(T);
  static_assert(!R1 || (SP && IS == 2 && WM == 2), "one-row tile: fp32, input stride 2, 128-channel block");
  // 8-channel halo pieces per thread: up to 320 / 448 / 448 / 704 pixels
  constexpr int WPER = RS ? 5 : IS == 1 || R1 ? 7 : 11;
  constexpr bool HALFW = (WM == 1 && IS == 2) || R1;  // waves of 32 q-columns
  constexpr int NGW = HALFW ? 2 : 4;             // 16-column N-groups per wave
  constexpr int WRT = R1 ? 1 : HALFW ? 2 : 4 / WM;  // q-tile rows
  constexpr int AR = WM * 256 * PL;        // 16-byte slots of one K chunk's A fragments (WM x 4 cout tiles)
  constexpr int NA = WM * PL;              // A loads per thread and chunk
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  raw* abuf = reinterpret_cast<raw*>(smem);  // 2 x AR slots
  const WideHalo<IS, WRT> hg(span);
  const int HP = hg.hp;
  // AG (below): A fragments from L1 / L2 per wave, no A buffer in LDS -- fp32, and bf16 except the 32-column waves of
  // the stride-2 64-channel block (A/B, bf16 GeoFF layers at B=4, profiles/r05/ab_wide_ag_bf16: cout-64 stride-1
  // layers 0.207 -> 0.170 and 0.123 -> 0.103 ms, stride-2 128-channel 0.299 -> 0.282 ms, the stride-2 64-channel block
  // 0.120 -> 0.130 ms)
  constexpr bool AG = SP || !HALFW;
  // stride 1: the next slice's halo goes to the other of two buffers; stride 2 (2.5x the pixels) and the fp32 64-channel
  // block: one buffer, rewritten between two barriers after the slice's last tap
  constexpr int NHB = IS == 1 && !(SP && WM == 1) ? 2 : 1;  // fp32 64-channel block: its 4-row halo twice = 1 block / CU
  raw* hbuf = abuf + (AG ? 0 : 2 * AR);      // NHB x HP * SLOTS slots

  // logical block = (tile, phase), phase fastest, XCD-contiguous
  const int ntile = tiles_x * tiles_y * a.B;
  const int nblk = ntile * a.nphase;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tl = L / a.nphase;
  const Conv2dPhase& ph = a.ph[L - tl * a.nphase];
  const int tx = tl % tiles_x, ty = (tl / tiles_x) % tiles_y, b = tl / (tiles_x * tiles_y);
  const int qy0 = ty * WRT, qx0 = tx * WC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = WM == 2 ? wave >> 1 : 0, wn = R1 ? 0 : WM == 2 ? wave & 1 : HALFW ? wave >> 1 : wave;
  const int wc = HALFW ? (wave & 1) * 32 : 0;  // the wave's first q-column in the tile
  const int n = lane & 15, g = lane >> 4;
  const int mt0 = blockIdx.y * 4 * WM;

  __shared__ int s_toff[32];  // tap offset inside the halo, in pixels
  if (tid < 25) s_toff[tid] = tid < ph.ntaps ? hg.pix(ph.tap[tid][0] - dmin, ph.tap[tid][1] - dmin) : 0;

  const int nt = ph.ntaps;  // loop order (slice, tap); packed order chunk = tap * nsl + slice
  const raw* __restrict__ wsrc = reinterpret_cast<const raw*>(a.wpack) + ((size_t)ph.w_off * a.MTtot + mt0) * 64 * PL;
  const size_t cstride = (size_t)a.MTtot * 64 * PL;  // slots between consecutive packed chunks
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wpack, 0x7fffffffLL);
  const uint32_t wbase = (uint32_t)(((size_t)ph.w_off * a.MTtot + mt0) * 64 * 16 * PL);
  const uint32_t cbytes = (uint32_t)a.MTtot * 64 * 16 * PL;  // bytes between consecutive packed chunks
  const int npix = a.B * a.Hi * a.Wi;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.in0, (long long)npix * a.c0 * ES);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(TWO ? a.in1 : a.in0, TWO ? (long long)npix * a.c1 * ES : 0);
  const int iy0 = IS * qy0 + dmin, ix0 = IS * qx0 + dmin, pb = b * a.Hi * a.Wi;
  // this thread's halo pieces (8 channels each): input pixel index (-1: outside the image or past the halo), the
  // channel offset it fetches and the LDS slot(s) it fills, the same for every slice
  int hpix[WPER], hch[WPER], hsl[WPER];
#pragma unroll
  for (int k = 0; k < WPER; ++k) {
    const int i = tid + k * 256;
    const int p = i >> 2, q = i & 3;
    int row, col;
    hg.rc(p, row, col);
    const int iy = iy0 + row, ix = ix0 + col;
    const bool ok = p < HP && col >= 0 && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    hpix[k] = ok ? pb + iy * a.Wi + ix : -1;
    if (SP) {
      hch[k] = q * 8;                                   // chunk q: hi to slot q, lo to slot 4 + q
      hsl[k] = p < HP ? p * SLOTS : -1;
    } else {
      hch[k] = (q ^ ((p >> 2) & 3)) * 8;                // chunk q ^ sw to slot q (the thread's own)
      hsl[k] = p < HP ? i : -1;
    }
  }
  raw hreg[WPER][PL];
  auto hload = [&](int c) DAMVS_INLINE {
    const bool second = TWO && c * 32 >= a.c0;
    const int cs = second ? a.c1 : a.c0, cb = second ? c * 32 - a.c0 : c * 32;
#pragma unroll
    for (int k = 0; k < WPER; ++k) {
      const uint32_t off = hpix[k] >= 0 ? (uint32_t)(hpix[k] * cs + cb + hch[k]) * ES : kOOB;
#pragma unroll
      for (int h = 0; h < PL; ++h) {
        const uint32_t o = off == kOOB ? kOOB : off + 16u * h;
        hreg[k][h] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128((TWO && second) ? r1 : r0, o, 0, 0));
      }
    }
  };
  auto hstore = [&](int bi) DAMVS_INLINE {
#pragma unroll
    for (int k = 0; k < WPER; ++k) {
      if (hsl[k] < 0) continue;
      if constexpr (SP) {
        const int p = hsl[k] / SLOTS, q = hch[k] >> 3;
        const F16Pair v = split8(__builtin_bit_cast(float4, hreg[k][0]), __builtin_bit_cast(float4, hreg[k][1]));
        raw* hb = hbuf + bi * HP * SLOTS + hsl[k];
        hb[Fm::slot(p, q)] = v.h;
        hb[Fm::slot(p, q + 4)] = v.l;
      } else {
        hbuf[bi * HP * SLOTS + hsl[k]] = hreg[k][0];
      }
    }
  };

  f32x4_t acc[4][NGW];  // [cout tile][N-group: 16 columns of the wave's q-row]
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < NGW; ++j) acc[m][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // the fp32 depth plane's halo (zero outside the image) for the trailing plane chunk, staged once
  // (bf16 AG: at least the epilogue's 4 x 32 x 68-float staging tiles below it)
  const int gofs = SP || !AG ? NHB * HP * SLOTS : max(NHB * HP * SLOTS, 4 * 32 * 68 / 4);
  float* gbuf = reinterpret_cast<float*>(hbuf + gofs);  // HP floats
  if (ph.gchunks > 0) {
    const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.geo[0], ((long long)(a.B - 1) * a.geo_bstride[0] + a.Hi * a.Wi) * 4);
    const int pg0 = b * (int)a.geo_bstride[0];
    for (int p = tid; p < HP; p += 256) {
      int row, col;
      hg.rc(p, row, col);
      const int iy = iy0 + row, ix = ix0 + col;
      const bool ok = col >= 0 && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      gbuf[p] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, ok ? (uint32_t)(pg0 + iy * a.Wi + ix) * 4u : kOOB, 0, 0));
    }
  }

  // One K chunk per barrier, slices outer and taps inner. A: chunk k + 2 is loaded (scalar offset: no
  // per-chunk VGPR address math) into one register set while the other set (chunk k + 1) goes to LDS
  // after chunk k's MFMAs; loads past the last chunk re-read it (unconditional: exact vmcnt counting).
  // Halo of slice c + 1: loaded after tap 0's A store of slice c (hipcc counts the vmcnt in front of that
  // store as if no halo load were pending, so issuing them later keeps them out of it), stored after the
  // slice's last tap.
  raw pa[NA], qa[NA];
  int lc = 0, lt = 0;  // (slice, tap) of the next chunk to load, two ahead of the chunk computed
  auto next = [&](int& cc, int& tt) {
    if (++tt == nt) {
      tt = 0;
      cc = cc + 1 < nsl ? cc + 1 : cc;  // past the end: stays on the last slice (clamped re-read)
    }
  };
  auto wld = [&](raw (&x)[NA]) DAMVS_INLINE {
    const uint32_t so = wbase + (uint32_t)(lt * nsl + lc) * cbytes;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      x[i] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(tid + 256 * i) * 16u, so, 0));
    if (!(lc == nsl - 1 && lt == nt - 1)) next(lc, lt);
  };
  // fp32 (AG): no block-wide A copy. Each wave reads its own 4 cout tiles' A pairs of a chunk from
  // L1 / L2 (the two waves of a cout half share them through L1), one chunk ahead in alternating register sets, so
  // the K loop needs no barrier inside a slice: the next slice's halo goes to the other halo buffer after the slice's
  // last tap and one barrier per 32-channel slice switches buffers (instead of one barrier per chunk). The split form's
  // 48 MFMAs per chunk and wave cover the loads.
  if constexpr (!AG) {
    wld(pa);
    wld(qa);
  }
  hload(0);
  if constexpr (!AG) {
#pragma unroll
    for (int i = 0; i < NA; ++i) abuf[tid + 256 * i] = pa[i];
  }
  hstore(0);
  __syncthreads();
  const int lanepix = wn * IS * hg.pitch + wc + n;
  int k = 0;
  auto step = [&](int c, int t, raw (&ld)[NA], const raw (&st)[NA]) DAMVS_INLINE {
    if (!(DAMVS_WIDE_DIAG & 8)) wld(ld);
    const int p0x = s_toff[t] + lanepix;
    const raw* hb = hbuf + (NHB == 2 ? (c & 1) * HP * SLOTS : 0) + p0x * SLOTS;
    if constexpr (SP) {
      // A: tile m of the wave's cout half at m * 128 (hi) and m * 128 + 64 (lo); B: pixel + 16 j keeps the swizzle
      const raw* ab = abuf + (k & 1) * AR + wm * 512 + lane;
      F16Pair af[4], bf[NGW];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = F16Pair{ab[m * 128], ab[m * 128 + 64]};
      const int sh = Fm::slot(p0x, g), sl = Fm::slot(p0x, g + 4);
#pragma unroll
      for (int j = 0; j < NGW; ++j) bf[j] = F16Pair{hb[j * 16 * SLOTS + sh], hb[j * 16 * SLOTS + sl]};
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < NGW; ++j) mma_split32(af[m], bf[j], acc[m][j]);
    } else {
      const raw* ab = abuf + (k & 1) * AR + wm * 256 + lane;
      raw af[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = ab[m * 64];
      // 16 pixels apart keeps (p >> 2) & 3: one swizzled address, the 4 N-groups at immediate offsets
      const raw* hbs = hb + Fm::slot(p0x, g);
      raw bf[NGW];
#pragma unroll
      for (int j = 0; j < NGW; ++j) bf[j] = hbs[j * 64];
      if (!(DAMVS_WIDE_DIAG & 1)) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int j = 0; j < NGW; ++j) Frag2<bf16_t>::mma(af[m], bf[j], acc[m][j]);
      } else {
        acc[0][0][0] += __uint_as_float(af[0].x ^ bf[0].y);
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) abuf[((k + 1) & 1) * AR + tid + 256 * i] = st[i];  // past the last chunk: a harmless copy
    if (!(DAMVS_WIDE_DIAG & 4)) {
      if (t == 0 && c + 1 < nsl) hload(c + 1);
      if (t == nt - 1 && c + 1 < nsl) {
        if (NHB == 1) __syncthreads();  // every wave is done with slice c's halo
        hstore(NHB == 2 ? (c + 1) & 1 : 0);
      }
    }
    if (!(DAMVS_WIDE_DIAG & 2)) __syncthreads();
    ++k;
  };
  int c = 0, t = 0;
  const int nk = nt * nsl;
  if constexpr (RS) {
    // Rolling K loop. Per chunk (slice c, tap t) and wave: wait for the previous chunk's loads, store the halo pieces
    // they brought (next slice, other buffer), at a slice's last tap one barrier (every piece of the next slice is in
    // LDS, and every wave's reads of this slice were issued), then issue the next chunk's A pairs (buffer loads at an
    // SGPR chunk offset) and this tap's piece loads, and run the 48 MFMAs N-group by N-group, each group's B pair
    // re-read for the next chunk (its own slice and tap) as soon as its 12 MFMAs are issued. Pieces of slice c + 1:
    // 0, 1 loaded at tap 0, 2, 3 at tap 1, 4 at tap 2, each stored one tap later (5 pieces = 1280 8-channel chunks >=
    // the 4 x 264 of a span-3 halo). The last slice re-reads itself into the idle buffer (harmless, branch-free).
    // Per accumulator the MFMA sequence is the AG loop's (chunks in (slice, tap) order, mma_split32), so the results
    // are bitwise equal.
    const int ltoff = lane < nt ? hg.pix(ph.tap[lane][0] - dmin, ph.tap[lane][1] - dmin) : 0;  // lane t: tap t's offset
    const uint32_t av0 = (uint32_t)(wm * 512 + lane) * 16u, av1 = av0 + 4096u;  // tile m: hi at m * 2048, lo + 1024
    auto aload = [&](F16Pair (&x)[4], int cc, int tt) DAMVS_INLINE {
      const uint32_t so = wbase + (uint32_t)(tt * nsl + cc) * cbytes;
      auto ld = [&](uint32_t v) DAMVS_INLINE { return __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(rw, v, so, 0)); };
      x[0] = F16Pair{ld(av0), ld(av0 + 1024u)};
      x[1] = F16Pair{ld(av0 + 2048u), ld(av0 + 3072u)};
      x[2] = F16Pair{ld(av1), ld(av1 + 1024u)};
      x[3] = F16Pair{ld(av1 + 2048u), ld(av1 + 3072u)};
    };
    raw pr[2][2];  // two halo pieces in flight (fp32: two 16-byte loads each)
    auto pload = [&](int k, int slot, int cc) DAMVS_INLINE {
      const bool second = TWO && cc * 32 >= a.c0;
      const int cs = second ? a.c1 : a.c0, cb = second ? cc * 32 - a.c0 : cc * 32;
      const uint32_t off = hpix[k] >= 0 ? (uint32_t)(hpix[k] * cs + cb + hch[k]) * ES : kOOB;
      const __amdgpu_buffer_rsrc_t r = (TWO && second) ? r1 : r0;
      pr[slot][0] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      pr[slot][1] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(r, off == kOOB ? kOOB : off + 16u, 0, 0));
    };
    // a piece past the halo goes to 8 spare slots behind the plane halo (launch_wide_t reserves them): no branch, so
    // the stores stay in the step's straight-line code
    const int spare = NHB * HP * SLOTS + (HP * 4 + 15) / 16;
    auto pstore = [&](int k, int slot, int bi) DAMVS_INLINE {
      const bool ok = hsl[k] >= 0;
      const int p = ok ? hsl[k] / SLOTS : 0, q = hch[k] >> 3;
      const F16Pair v = split8(__builtin_bit_cast(float4, pr[slot][0]), __builtin_bit_cast(float4, pr[slot][1]));
      raw* hb = hbuf + (ok ? bi * HP * SLOTS + hsl[k] : spare);
      hb[Fm::slot(p, q)] = v.h;
      hb[Fm::slot(p, q + 4)] = v.l;
    };
    // B pair of N-group j of chunk (cc, tt): halo buffer cc & 1, pixel tap offset + the lane's column (+ 16 j keeps
    // the swizzle)
    int bh = 0, bl = 0;
    auto baddr = [&](int cc, int tt) DAMVS_INLINE {
      const int p0x = __builtin_amdgcn_readlane(ltoff, tt) + lanepix;
      const int base = ((cc & 1) * HP + p0x) * SLOTS;
      bh = base + Fm::slot(p0x, g);
      bl = base + Fm::slot(p0x, g + 4);
    };
    // NG: the wave's N-groups that hold q-columns inside the grid (uniform per block: its tile column), the only ones
    // whose MFMAs and B reads run -- the last tile column of a 200-column grid has 8 valid columns of 64
    auto rs_loop = [&](auto NGc) DAMVS_INLINE {
    constexpr int NG = decltype(NGc)::value;
    F16Pair b[NGW];
    baddr(0, 0);
#pragma unroll
    for (int j = 0; j < NG; ++j) b[j] = F16Pair{hbuf[bh + j * 16 * SLOTS], hbuf[bl + j * 16 * SLOTS]};
    // PS: the tap's piece phase (0..2 load, 1..3 store; 4 none)
    auto rstep = [&](auto PS, const F16Pair (&cur)[4], F16Pair (&nxt)[4]) DAMVS_INLINE {
      constexpr int ps = decltype(PS)::value;
      const int nb = (c + 1) & 1;               // the buffer the next slice's pieces go to
      const int cn = c + 1 < nsl ? c + 1 : c;   // the slice they come from (the last slice: itself, unused)
      if constexpr (ps == 1) { pstore(0, 0, nb); pstore(1, 1, nb); }
      if constexpr (ps == 2) { pstore(2, 0, nb); pstore(3, 1, nb); }
      if constexpr (ps == 3) pstore(4, 0, nb);
      if (t == nt - 1) __syncthreads();
      int c1 = c, t1 = t + 1;
      if (t1 == nt) {
        t1 = 0;
        c1 = c + 1 < nsl ? c + 1 : c;
      }
      aload(nxt, c1, t1);
      if constexpr (ps == 0) { pload(0, 0, cn); pload(1, 1, cn); }
      if constexpr (ps == 1) { pload(2, 0, cn); pload(3, 1, cn); }
      if constexpr (ps == 2) pload(4, 0, cn);
      baddr(c1, t1);
      // the loads above stay above the MFMAs (the scheduler would otherwise sink them next to their uses, a chunk later)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
#pragma unroll
        for (int m = 0; m < 4; ++m) mma_split32(cur[m], b[j], acc[m][j]);
        b[j] = F16Pair{hbuf[bh + j * 16 * SLOTS], hbuf[bl + j * 16 * SLOTS]};
      }
      // per N-group: its 12 MFMAs, then its two B reads for the next chunk
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (++t == nt) { t = 0; ++c; }
    };
    F16Pair a0[4], a1[4];
    aload(a0, 0, 0);
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    for (int cc = 0; cc < nsl; ++cc) {
      // taps 0..3 carry the piece phases (nt >= 4); then the remaining taps two at a time (register sets alternate)
      rstep(I0{}, a0, a1);
      rstep(I1{}, a1, a0);
      rstep(I2{}, a0, a1);
      rstep(I3{}, a1, a0);
      int tt = 4;
      for (; tt + 1 < nt; tt += 2) {
        rstep(I4{}, a0, a1);
        rstep(I4{}, a1, a0);
      }
      if (tt < nt) {  // odd tap count: one more step, then the sets are swapped for the next slice
        rstep(I4{}, a0, a1);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const F16Pair x = a0[m];
          a0[m] = a1[m];
          a1[m] = x;
        }
      }
    }
    };
    if (WIDE_NG_SKIP && a.Wq - qx0 - wc <= 16) rs_loop(std::integral_constant<int, 1>{});
    else rs_loop(std::integral_constant<int, NGW>{});
    __syncthreads();  // the epilogue's staging tiles overwrite the halo region other waves may still read
  } else if constexpr (AG && !SP) {
    // bf16 AG: the fp32 AG loop below with one 16-byte A fragment per cout tile (tile m of the wave's cout half at
    // m * 64 slots of the chunk) and one MFMA per product
    const raw* wa = wsrc + wm * 256 + lane;
    auto aload = [&](raw (&x)[4], int cc, int tt) DAMVS_INLINE {
      const raw* q = wa + (size_t)(tt * nsl + cc) * cstride;
#pragma unroll
      for (int m = 0; m < 4; ++m) x[m] = q[m * 64];
    };
    auto gstep = [&](auto NGc, const raw (&cur)[4], raw (&nxt)[4]) DAMVS_INLINE {
      constexpr int NG = decltype(NGc)::value;  // N-groups inside the q-grid
      int c1 = c, t1 = t + 1;
      if (t1 == nt) {
        c1 = c + 1 < nsl ? c + 1 : c;
        t1 = c + 1 < nsl ? 0 : nt - 1;
      }
      aload(nxt, c1, t1);
      const int p0x = s_toff[t] + lanepix;
      const raw* hbs = hbuf + (NHB == 2 ? (c & 1) * HP * SLOTS : 0) + p0x * SLOTS + Fm::slot(p0x, g);
      raw bf[NGW];
#pragma unroll
      for (int j = 0; j < NG; ++j) bf[j] = hbs[j * 64];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < NG; ++j) Frag2<bf16_t>::mma(cur[m], bf[j], acc[m][j]);
      if (t == 0 && c + 1 < nsl) hload(c + 1);
      if (t == nt - 1 && c + 1 < nsl) {
        if (NHB == 1) __syncthreads();
        hstore(NHB == 2 ? (c + 1) & 1 : 0);
        __syncthreads();
      }
      if (++t == nt) { t = 0; ++c; }
    };
    raw a0[4], a1[4];
    aload(a0, 0, 0);
    auto ag_loop = [&](auto NGc) DAMVS_INLINE {
      for (int kk = 0; kk < nk; kk += 2) {
        gstep(NGc, a0, a1);
        if (kk + 1 < nk) gstep(NGc, a1, a0);
      }
    };
    if (IS == 2 && WIDE_NG_SKIP && a.Wq - qx0 - wc <= 16) ag_loop(std::integral_constant<int, IS == 2 ? 1 : NGW>{});
    else ag_loop(std::integral_constant<int, NGW>{});
    __syncthreads();
  } else if constexpr (AG) {
    const raw* wa = wsrc + wm * 512 + lane;  // the wave's cout half: tile m's hi at m * 128, lo at m * 128 + 64
    auto aload = [&](F16Pair (&x)[4], int cc, int tt) DAMVS_INLINE {
      const raw* q = wa + (size_t)(tt * nsl + cc) * cstride;
#pragma unroll
      for (int m = 0; m < 4; ++m) x[m] = F16Pair{q[m * 128], q[m * 128 + 64]};
    };
    // chunk (c, t) with A in `cur`; chunk (c, t) + 1 (clamped to the last) loaded into `nxt` first
    auto gstep = [&](auto NGc, const F16Pair (&cur)[4], F16Pair (&nxt)[4]) DAMVS_INLINE {
      constexpr int NG = decltype(NGc)::value;  // N-groups inside the q-grid
      int c1 = c, t1 = t + 1;
      if (t1 == nt) {
        t1 = 0;
        c1 = c + 1 < nsl ? c + 1 : c;
        t1 = c + 1 < nsl ? 0 : nt - 1;
      }
      aload(nxt, c1, t1);
      const int p0x = s_toff[t] + lanepix;
      const raw* hb = hbuf + (NHB == 2 ? (c & 1) * HP * SLOTS : 0) + p0x * SLOTS;
      const int sh = Fm::slot(p0x, g), sl = Fm::slot(p0x, g + 4);
      F16Pair bf[NGW];
#pragma unroll
      for (int j = 0; j < NG; ++j) bf[j] = F16Pair{hb[j * 16 * SLOTS + sh], hb[j * 16 * SLOTS + sl]};
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < NG; ++j) mma_split32(cur[m], bf[j], acc[m][j]);
      if (t == 0 && c + 1 < nsl) hload(c + 1);
      if (t == nt - 1 && c + 1 < nsl) {
        // two buffers: the one slice c - 1 used, which every wave left at the previous slice switch
        if (NHB == 1) __syncthreads();  // one buffer: every wave is done with slice c's halo
        hstore(NHB == 2 ? (c + 1) & 1 : 0);
        __syncthreads();
      }
      if (++t == nt) { t = 0; ++c; }
    };
    F16Pair a0[4], a1[4];
    aload(a0, 0, 0);
    auto ag_loop = [&](auto NGc) DAMVS_INLINE {
      for (int kk = 0; kk < nk; kk += 2) {  // unrolled by two: the register sets alternate statically
        gstep(NGc, a0, a1);
        if (kk + 1 < nk) gstep(NGc, a1, a0);
      }
    };
    if (IS == 2 && WIDE_NG_SKIP && a.Wq - qx0 - wc <= 16) ag_loop(std::integral_constant<int, IS == 2 ? 1 : NGW>{});
    else ag_loop(std::integral_constant<int, NGW>{});
    __syncthreads();  // the epilogue's staging tiles overwrite the halo region other waves may still read
  } else {
    for (int kk = 0; kk < nk; kk += 2) {  // unrolled by two: the register sets alternate statically
      step(c, t, pa, qa);
      if (++t == nt) { t = 0; ++c; }
      if (kk + 1 < nk) {
        step(c, t, qa, pa);
        if (++t == nt) { t = 0; ++c; }
      }
    }
  }

  // tail: the plane chunk (A fragments straight from global memory), then the epilogue
  const int qyw = qy0 + wn;  // the wave's q-row
  const int up = a.post_up, us = a.post_up >> 1;
  const long long nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout * ES);
  const __amdgpu_buffer_rsrc_t rpre = make_rsrc(a.res_pre ? a.res_pre : a.out, a.res_pre ? nout * ES : 0);
  const __amdgpu_buffer_rsrc_t rpost = make_rsrc(a.res_post ? a.res_post : a.out, a.res_post ? nout / (up * up) * ES : 0);
  // the fp32 plane as a trailing K chunk (tap x plane), B from the staged plane halo
  if (ph.gchunks > 0) {
    float v[NGW][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int tt = g * 8 + e;
      const bool tv = tt < nt;
      const int po = s_toff[tv ? tt : 0] + lanepix;
#pragma unroll
      for (int j = 0; j < NGW; ++j) v[j][e] = tv ? gbuf[po + j * 16] : 0.f;
    }
    if constexpr (SP) {
      const raw* wg = wsrc + (size_t)ph.kchunks * cstride + wm * 512 + lane;
      F16Pair ag[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) ag[m] = F16Pair{wg[m * 128], wg[m * 128 + 64]};
#pragma unroll
      for (int j = 0; j < NGW; ++j) {
        const F16Pair xf = split8(v[j]);
#pragma unroll
        for (int m = 0; m < 4; ++m) mma_split32(ag[m], xf, acc[m][j]);
      }
    } else {
      const raw* wg = wsrc + (size_t)ph.kchunks * cstride + wm * 256 + lane;
      raw ag[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) ag[m] = wg[m * 64];
#pragma unroll
      for (int j = 0; j < NGW; ++j) {
        const raw xf = pack_vals<bf16_t>(v[j]);
#pragma unroll
        for (int m = 0; m < 4; ++m) Frag2<bf16_t>::mma(ag[m], xf, acc[m][j]);
      }
    }
  }

  // epilogue (as conv2d_mfma_kernel): residual before ReLU, ReLU, (upsampled) residual after, store
  {
    // through LDS: the wave's 64 channels x 64 pixels go to a wave-private fp32 staging tile in two halves of 32
    // pixels (the K loop's A and halo buffers are free after its last barrier; 4 x 8.5 KB stay below the plane
    // halo, which other waves may still read), and each lane then finishes one pixel's
    // 32-channel half: contiguous residual loads and stores (16-byte accesses; the accumulator layout
    // stores 8 bytes per lane, 16 pixels apart). Row pitch 68 floats: the b128 writes of 16 lanes (16 pixels,
    // one column) and reads (16 pixels) hit distinct banks.
    constexpr int PITCH = 68;
    float* st = reinterpret_cast<float*>(abuf) + wave * (32 * PITCH);
    const int cb = (mt0 + wm * 4) * 16;       // the wave's first output channel
    const int lp = lane & 31, hc = lane >> 5;  // this lane's pixel within the half, its 32-channel half
    const int co0 = cb + hc * 32;
    const bool cvalid = co0 < a.cout;
    const float* bias = a.bias + (cvalid ? co0 : 0);  // a padded channel tile past cout reads channel 0's bias
    auto add8 = [](const raw* q, float* v) {  // 8 channels of a residual record (bf16: one slot, fp32: two)
      if constexpr (SP) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 f = __builtin_bit_cast(float4, q[h]);
          v[4 * h] += f.x; v[4 * h + 1] += f.y; v[4 * h + 2] += f.z; v[4 * h + 3] += f.w;
        }
      } else {
        const uint32_t w[4] = {q[0].x, q[0].y, q[0].z, q[0].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[2 * i] += __uint_as_float(w[i] << 16);
          v[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
        }
      }
    };
#pragma unroll
    for (int h = 0; h < NGW / 2; ++h) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const f32x4_t v = acc[m][2 * h + jj];
          *reinterpret_cast<float4*>(st + (jj * 16 + n) * PITCH + m * 16 + g * 4) = make_float4(v[0], v[1], v[2], v[3]);
        }
      asm volatile("" ::: "memory");  // one wave's LDS accesses complete in order: only the compiler must keep it
      const int j = 2 * h + (lp >> 4);
      const int qx = qx0 + wc + j * 16 + (lp & 15);
      const int oy = qyw * a.out_stride + ph.py, ox = qx * a.out_stride + ph.px;
      const int pout = (b * a.Ho + oy) * a.Wo + ox;
      const int ppost = (b * (a.Ho >> us) + (oy >> us)) * (a.Wo >> us) + (ox >> us);
      const bool ok = qyw < a.Hq && qx < a.Wq && cvalid;
      const uint32_t ooff = ok ? (uint32_t)(pout * a.cout + co0) * ES : kOOB;
      const uint32_t poff = ok ? (uint32_t)(ppost * a.cout + co0) * ES : kOOB;
      raw pre[4][PL], post[4][PL];  // all residual records requested before the first store
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
        for (int h2 = 0; h2 < PL; ++h2) {
          const uint32_t d = 16u * (k2 * PL + h2);
          if (a.res_pre) pre[k2][h2] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(rpre, ooff + d, 0, 0));
          if (a.res_post) post[k2][h2] = __builtin_bit_cast(raw, __builtin_amdgcn_raw_buffer_load_b128(rpost, poff + d, 0, 0));
        }
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {  // 8 channels at a time
        float r[8];
        const float4 v0 = *reinterpret_cast<const float4*>(st + lp * PITCH + hc * 32 + 8 * k2);
        const float4 v1 = *reinterpret_cast<const float4*>(st + lp * PITCH + hc * 32 + 8 * k2 + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(bias + 8 * k2);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + 8 * k2 + 4);
        r[0] = fmaf(v0.x, a.wscale, b0.x); r[1] = fmaf(v0.y, a.wscale, b0.y);
        r[2] = fmaf(v0.z, a.wscale, b0.z); r[3] = fmaf(v0.w, a.wscale, b0.w);
        r[4] = fmaf(v1.x, a.wscale, b1.x); r[5] = fmaf(v1.y, a.wscale, b1.y);
        r[6] = fmaf(v1.z, a.wscale, b1.z); r[7] = fmaf(v1.w, a.wscale, b1.w);
        if (a.res_pre) add8(pre[k2], r);
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = relu(r[e]);
        }
        if (a.res_post) add8(post[k2], r);
        if constexpr (SP) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(v4u32_t, make_float4(r[4 * h2], r[4 * h2 + 1], r[4 * h2 + 2], r[4 * h2 + 3])), ro,
                ooff + 32u * k2 + 16u * h2, 0, 0);
        } else {
          uint32_t w[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(r[2 * i]) | ((uint32_t)f2bf(r[2 * i + 1]) << 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, make_uint4(w[0], w[1], w[2], w[3])), ro,
                                                 ooff + 16u * k2, 0, 0);
        }
      }
      asm volatile("" ::: "memory");  // the next half overwrites the staging tile
    }
  }
}

template <typename T, int IS, int WM, bool RS = false, bool R1 = false>
hipError_t launch_wide_t(hipStream_t s, const Conv2dArgs& a, int dmin, int span) {
  constexpr bool SP = sizeof(T) == 4;
  constexpr int WRT = R1 ? 1 : WM == 1 && IS == 2 ? 2 : 4 / WM, AR = WM * 256 * WideForm<T>::PL, SLOTS = WideForm<T>::SLOTS;
  const WideHalo<IS, WRT> hg(span);
  constexpr int NHB = IS == 1 && !(SP && WM == 1) ? 2 : 1, WPER = RS ? 5 : IS == 1 || R1 ? 7 : 11;
  constexpr bool AG = SP || !(WM == 1 && IS == 2);  // A fragments from L1 / L2, no A buffers in LDS (the kernel's AG)
  if (hg.hp * 4 > WPER * 256) return hipErrorNotSupported;
  size_t below_plane = (AG ? 0 : 2 * (size_t)AR * 16) + NHB * (size_t)hg.hp * SLOTS * 16;
  if (!SP && AG && below_plane < 4 * 32 * 68 * 4) below_plane = 4 * 32 * 68 * 4;  // as gofs in the kernel
  if (below_plane < 4 * 32 * 68 * 4) return hipErrorNotSupported;  // the epilogue's staging tiles stay below the plane halo
  const int tx = (a.Wq + WC - 1) / WC, ty = (a.Hq + WRT - 1) / WRT;
  const int nsl = (a.c0 + a.c1) / 32;
  const size_t smem = below_plane + (size_t)hg.hp * 4 + (RS ? 16 + SLOTS * 16 : 0);  // A chunks, halo slices, plane
                                                                                    // halo (RS: spare piece slots)
  if (smem > 160 * 1024) return hipErrorNotSupported;
  const long long nblk = (long long)tx * ty * a.B * a.nphase;
  const dim3 grid((unsigned)nblk, (unsigned)(a.MTtot / (4 * WM)));
  auto k = a.c1 > 0 ? conv2d_wide_kernel<T, true, IS, WM, RS, R1> : conv2d_wide_kernel<T, false, IS, WM, RS, R1>;
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)smem);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), smem, s, a, tx, ty, nsl, dmin, span);
  return hipGetLastError();
}

// Shape checks of the wide kernel (K chunks of 32: bf16 packing, or the fp32 layer's 32-K split packing); returns
// the tap offset range in dmin / span.
bool wide_shape_ok(const Conv2dArgs& a, int& dmin, int& span) {
  static const bool s2 = [] {
    const char* v = getenv("DAMVS_CONV2D_WIDE_S2");
    return !(v && v[0] == '0');
  }();
  static const bool w64 = [] {
    const char* v = getenv("DAMVS_CONV2D_WIDE64");
    return !(v && v[0] == '0');
  }();
  const bool stride_ok = a.in_stride == 1 || (a.in_stride == 2 && s2 && a.nphase == 1 && a.out_stride == 1);
  const bool half = w64 && a.MTtot == 4;  // 64 output channels
  if (!stride_ok || a.xpair || a.ngeo > 1 || (a.MTtot % 8 && !half) || a.c0 % 32 || a.c1 % 32 || a.c0 + a.c1 < 64 ||
      a.cout % 32)  // the epilogue finishes whole 32-channel halves per lane
    return false;
  int lo = 0, hi = 0;
  for (int p = 0; p < a.nphase; ++p)
    for (int t = 0; t < a.ph[p].ntaps; ++t)
      for (int d = 0; d < 2; ++d) {
        lo = a.ph[p].tap[t][d] < lo ? a.ph[p].tap[t][d] : lo;
        hi = a.ph[p].tap[t][d] > hi ? a.ph[p].tap[t][d] : hi;
      }
  for (int p = 0; p < a.nphase; ++p)  // geo taps beyond one K chunk; fewer than 4 taps (halo schedule)
    if (a.ph[p].gchunks > 1 || a.ph[p].ntaps < 4) return false;
  dmin = lo;
  span = hi - lo + 1;
  return true;
}

// Returns hipErrorNotSupported when the wide kernel does not take the layer. Input stride 2 (the stride-2 GeoBlock
// convs, one phase) unless DAMVS_CONV2D_WIDE_S2=0; cout 64 at input stride 1 on the 64-channel block (WM = 1) unless
// DAMVS_CONV2D_WIDE64=0. T = float: `a` carries the layer's 32-K split packing (a.wide32, damvs_conv2d_forward).
template <typename T>
hipError_t launch_wide(hipStream_t s, const Conv2dArgs& a) {
  static const bool off = [] {
    const char* v = getenv("DAMVS_CONV2D_WIDE");
    return v && v[0] == '0';
  }();
  // fp32 rolling K loop (conv2d_wide_kernel RS) for the stride-1 128-channel block when its halo fits 5 pieces a thread
  // (taps spanning <= 3 pixels); DAMVS_WIDE_RS=0 keeps the AG loop (read per call: the bitwise test flips it)
  const char* rsv = getenv("DAMVS_WIDE_RS");
  const bool rs_off = rsv && rsv[0] == '0';
  int dmin = 0, span = 0;
  if (off || !wide_shape_ok(a, dmin, span)) return hipErrorNotSupported;
  if (a.MTtot % 8) {
    // fp32 64-channel block at input stride 2 (32-column waves, one block per CU): the 32-K gather kernel is faster
    // (kbench2d H 91.6 -> 63.5 us, profiles/r06/ab_wide_s2r1_r06x/)
    if (sizeof(T) == 4 && a.in_stride == 2) return hipErrorNotSupported;
    return a.in_stride == 1 ? launch_wide_t<T, 1, 1>(s, a, dmin, span) : launch_wide_t<T, 2, 1>(s, a, dmin, span);
  }
  if constexpr (sizeof(T) == 4) {
    if (a.in_stride == 1 && span <= 3 && !rs_off) return launch_wide_t<T, 1, 2, true>(s, a, dmin, span);
  }
  if constexpr (sizeof(T) == 4) {
    // the fp32 stride-2 128-channel block on one-row tiles (two blocks per CU): kbench2d E 120 -> 103 us, parity path
    // 103.0 -> 103.2-103.6 maps/s (profiles/r06/ab_wide_s2r1_r06x/); DAMVS_WIDE_S2R1=0 (read per call) keeps 2-row tiles
    const char* r1 = getenv("DAMVS_WIDE_S2R1");
    if (a.in_stride == 2 && !(r1 && r1[0] == '0')) return launch_wide_t<T, 2, 2, false, true>(s, a, dmin, span);
  }
  return a.in_stride == 1 ? launch_wide_t<T, 1, 2>(s, a, dmin, span) : launch_wide_t<T, 2, 2>(s, a, dmin, span);
}

// conv2d_xpair_lds_kernel's layers: x-pair phases of a 16-channel single-input transposed stride-2 conv whose taps
// all lie in -1 .. 1 (DAMVS_CONV2D_XPAIR_LDS=0, read per call: the XP gather kernel)
bool xpair_lds_ok(const Conv2dArgs& a, int KC) {
  const char* v = getenv("DAMVS_CONV2D_XPAIR_LDS");
  if ((v && v[0] == '0') || a.c0 != 16 || a.c1 != 0 || a.in_stride != 1 || a.out_stride != 2 || a.Hq != a.Hi ||
      a.Wq != a.Wi)
    return false;
  for (int p = 0; p < 2; ++p) {
    if (a.ph[p].ntaps > 16 || a.ph[p].kchunks != (a.ph[p].ntaps * 16 + KC - 1) / KC || a.ph[p].gchunks != 0 ||
        a.ph[p].py != p)
      return false;
    for (int t = 0; t < a.ph[p].ntaps; ++t)
      if (a.ph[p].tap[t][0] < -1 || a.ph[p].tap[t][0] > 1 || a.ph[p].tap[t][1] < -1 || a.ph[p].tap[t][1] > 1) return false;
  }
  return true;
}

// True when the layer is a plain 3x3 stride-1 padding-1 conv with dense row-major taps.
bool lds3_ok(const Conv2dArgs& a) {
  // at most one plane, next to at most 16 channels (the layers the gather kernel ran; 32+g goes to the halo kernel);
  // DAMVS_CONV2D_LDS_PLANE=0 (read per call): planes stay on the gather kernel
  const char* pv = getenv("DAMVS_CONV2D_LDS_PLANE");
  const int maxg = (pv && pv[0] == '0') || a.c0 > 16 ? 0 : 1;
  if (a.nphase != 1 || a.out_stride != 1 || a.in_stride != 1 || a.ph[0].ntaps != 9 || a.ngeo > maxg || a.c1 != 0 ||
      a.Ho != a.Hi || a.Wo != a.Wi || (a.ngeo && a.ph[0].gchunks != 1))
    return false;
  for (int t = 0; t < 9; ++t)
    if (a.ph[0].tap[t][0] != t / 3 - 1 || a.ph[0].tap[t][1] != t % 3 - 1) return false;
  return true;
}

template <typename T, int CIN, int MT>
hipError_t launch_lds2_t(hipStream_t s, const Conv2dArgs& a) {
  const int tx = (a.Wo + L2W - 1) / L2W, ty = (a.Ho + L2H - 1) / L2H;
  const long long nt = (long long)tx * ty * a.B;
  hipLaunchKernelGGL((conv2d_lds_kernel<T, CIN, MT>), dim3((unsigned)nt), dim3(256), 0, s, a, tx, ty, (int)nt);
  return hipGetLastError();
}

// Returns hipErrorNotSupported when the LDS variant does not take the layer.
template <typename T>
hipError_t launch_lds2(hipStream_t s, const Conv2dArgs& a, bool dry = false) {
  static const bool off = [] {
    const char* v = getenv("DAMVS_CONV2D_NO_LDS");
    return v && v[0] == '1';
  }();
  // fp32 layers with a plane stay on the 32-K gather kernel (kbench J 27.8 against 31.2 us on the 16-K LDS form; bench
  // flat, profiles/r06/ab_lds_plane)
  if (off || !lds3_ok(a) || a.MTtot > 2 || (sizeof(T) == 4 && (a.c0 > 16 || a.ngeo))) return hipErrorNotSupported;  // LDS <= 42 KB
  if (dry) return a.c0 == 8 || a.c0 == 16 || (sizeof(T) == 2 && a.c0 == 32) ? hipSuccess : hipErrorNotSupported;
  const int MT = a.MTtot;
  switch (a.c0) {
    case 8: return MT == 1 ? launch_lds2_t<T, 8, 1>(s, a) : launch_lds2_t<T, 8, 2>(s, a);
    case 16: return MT == 1 ? launch_lds2_t<T, 16, 1>(s, a) : launch_lds2_t<T, 16, 2>(s, a);
    case 32:
      if constexpr (sizeof(T) == 2) return MT == 1 ? launch_lds2_t<T, 32, 1>(s, a) : launch_lds2_t<T, 32, 2>(s, a);
      return hipErrorNotSupported;
    default: return hipErrorNotSupported;
  }
}


// True when the layer is a 5x5 stride-2 padding-2 conv with dense row-major taps (one phase, one tensor input).
bool lds_s2_ok(const Conv2dArgs& a) {
  if (a.nphase != 1 || a.out_stride != 1 || a.in_stride != 2 || a.ph[0].ntaps != 25 || a.ngeo != 0 || a.c1 != 0 ||
      a.xpair)
    return false;
  for (int t = 0; t < 25; ++t)
    if (a.ph[0].tap[t][0] != t / 5 - 2 || a.ph[0].tap[t][1] != t % 5 - 2) return false;
  return true;
}

template <typename T, int CIN, int MT, int TR>
hipError_t launch_lds_s2_t(hipStream_t s, const Conv2dArgs& a) {
  const int tx = (a.Wo + S2W - 1) / S2W, ty = (a.Ho + TR - 1) / TR;
  const long long nt = (long long)tx * ty * a.B;
  hipLaunchKernelGGL((conv2d_lds_s2_kernel<T, CIN, MT, TR>), dim3((unsigned)nt), dim3(256), 0, s, a, tx, ty, (int)nt);
  return hipGetLastError();
}

// Returns hipErrorNotSupported when the stride-2 LDS variant does not take the layer (CIN 8 / 16, cout <= 32);
// DAMVS_CONV2D_LDS_S2=0 (read per call) leaves those layers to the gather kernel. Tile rows: 4 (LDS <= 47 KB), 2 for
// fp32 CIN 16 (59 KB).
template <typename T>
hipError_t launch_lds_s2(hipStream_t s, const Conv2dArgs& a, bool dry = false) {
  const char* v = getenv("DAMVS_CONV2D_LDS_S2");
  if ((v && v[0] == '0') || !lds_s2_ok(a) || a.MTtot > 2 || (a.c0 != 8 && a.c0 != 16)) return hipErrorNotSupported;
  if (dry) return hipSuccess;
  const bool m2 = a.MTtot == 2;
  constexpr bool SP = sizeof(T) == 4;
  if (a.c0 == 8) return m2 ? launch_lds_s2_t<T, 8, 2, 4>(s, a) : launch_lds_s2_t<T, 8, 1, 4>(s, a);
  return m2 ? launch_lds_s2_t<T, 16, 2, SP ? 2 : 4>(s, a) : launch_lds_s2_t<T, 16, 1, SP ? 2 : 4>(s, a);
}


template <typename T, int MT, bool K32 = false>
hipError_t launch_mt(hipStream_t s, const Conv2dArgs& a) {
  const long long Qtot = (long long)a.B * a.Hq * a.Wq;
  const int nq = (int)((Qtot + 4LL * kG2 * 16 - 1) / (4LL * kG2 * 16));
  dim3 grid((unsigned)(nq * a.nphase), (unsigned)((a.MTtot + MT - 1) / MT));
  if (a.c1 > 0)
    hipLaunchKernelGGL((conv2d_mfma_kernel<T, MT, true, false, K32>), grid, dim3(256), 0, s, a, nq);
  else
    hipLaunchKernelGGL((conv2d_mfma_kernel<T, MT, false, false, K32>), grid, dim3(256), 0, s, a, nq);
  return hipGetLastError();
}

// The gather kernel's cout tile: the widest that still puts about one wave on every SIMD (the low-resolution
// GeoFeatureFusion layers have few pixels and many channels); 0 when the tile count rules out every width.
int gather_mt(const Conv2dArgs& a, bool bf16) {
  const long long tiles = ((long long)a.B * a.Hq * a.Wq + 63) / 64 * a.nphase;
  constexpr long long want = 900;  // (600 / 1400 and a widest tile of 4 measured within the run-to-run spread)
  if (bf16 && a.MTtot % 8 == 0 && tiles * (a.MTtot / 8) >= want) return 8;
  if (a.MTtot % 4 == 0 && tiles * (a.MTtot / 4) >= want) return 4;
  if (a.MTtot % 2 == 0 && tiles * (a.MTtot / 2) >= want) return 2;
  return 1;
}

// fp32 32-K gather form (conv2d_mfma_kernel K32) for the layers with a 32-K packing that neither the wide nor the halo
// kernel takes; DAMVS_CONV2D_G32=0 (read per call: the parity test flips it) returns them to the 16-K form.
template <typename T>
hipError_t launch_gather32(hipStream_t s, const Conv2dArgs& a) {
  const char* v = getenv("DAMVS_CONV2D_G32");
  if ((v && v[0] == '0') || a.xpair || a.c0 % 8 || a.c1 % 8 || a.ngeo > 1) return hipErrorNotSupported;
  switch (gather_mt(a, false)) {
    case 4: return launch_mt<T, 4, true>(s, a);
    case 2: return launch_mt<T, 2, true>(s, a);
    default: return launch_mt<T, 1, true>(s, a);
  }
}


template <typename T>
hipError_t launch_t(hipStream_t s, const Conv2dArgs& a) {
  // 32-bit indices / buffer offsets: every operand must stay below 2 GiB
  const long long lim = 1LL << 31, es = sizeof(T);
  const long long npix = (long long)a.B * a.Hi * a.Wi, nout = (long long)a.B * a.Ho * a.Wo * a.cout;
  if (npix * (a.c0 > a.c1 ? a.c0 : a.c1) * es >= lim || nout * es >= lim || (long long)a.B * a.Hq * a.Wq >= lim)
    return hipErrorInvalidValue;
  for (int g = 0; g < a.ngeo; ++g)
    if (((long long)(a.B - 1) * a.geo_bstride[g] + npix / a.B) * 4 >= lim) return hipErrorInvalidValue;
  if (a.c0 + a.c1 == 0) return launch_conv2d_planes(s, sizeof(T) == 2 ? ST_BF16 : ST_F32, a);  // k_planes.hip
  if (a.ngeo > 1) return hipErrorInvalidValue;  // the MFMA path takes at most one plane
  if (a.wide32) {  // fp32 layer with its 32-K split packing: the wide kernel, else the narrow halo kernel, else (unless
                   // the thin-layer LDS kernel takes it on the 16-K packing) the 32-K gather kernel, else
                   // hipErrorNotSupported (damvs_conv2d_forward then runs the 16-K packing)
    if constexpr (sizeof(T) == 4) {
      hipError_t e = launch_wide<T>(s, a);
      if (e != hipErrorNotSupported) return e;
      if (a.c0 % 32 == 0 && a.c1 % 32 == 0) {
        e = launch_halo<T, true>(s, a);
        if (e != hipErrorNotSupported) return e;
      }
      // the layers the 16-K route gives to the LDS-tiled kernels stay there (thin 3x3 layers, 16-channel slices)
      if (launch_lds2<T>(s, a, true) == hipSuccess || launch_lds_s2<T>(s, a, true) == hipSuccess ||
          launch_halo<T>(s, a, true) == hipSuccess)
        return hipErrorNotSupported;
      return launch_gather32<T>(s, a);
    }
    return hipErrorInvalidValue;
  }
  if (a.xpair) {  // x-pair phases (built at layer creation): the LDS x-pair kernel where it fits, else the XP gather kernel
    if (a.cout != 8 || a.MTtot != 1 || a.ngeo != 0 || a.nphase != 2) return hipErrorInvalidValue;
    if (xpair_lds_ok(a, 4 * Stor<T>::E)) {
      const int tx = (a.Wq + L2W - 1) / L2W, ty = (a.Hq + L2H - 1) / L2H;
      const long long nt = (long long)tx * ty * a.B;
      hipLaunchKernelGGL(conv2d_xpair_lds_kernel<T>, dim3((unsigned)nt), dim3(256), 0, s, a, tx, ty, (int)nt);
      return hipGetLastError();
    }
    const long long Qtot = (long long)a.B * a.Hq * a.Wq;
    const int nq = (int)((Qtot + 4LL * kG2 * 16 - 1) / (4LL * kG2 * 16));
    const dim3 grid((unsigned)(nq * a.nphase), 1);
    if (a.c1 > 0)
      hipLaunchKernelGGL((conv2d_mfma_kernel<T, 1, true, true>), grid, dim3(256), 0, s, a, nq);
    else
      hipLaunchKernelGGL((conv2d_mfma_kernel<T, 1, false, true>), grid, dim3(256), 0, s, a, nq);
    return hipGetLastError();
  }
  {
    hipError_t e = launch_lds2<T>(s, a);
    if (e != hipErrorNotSupported) return e;
    e = launch_lds_s2<T>(s, a);
    if (e != hipErrorNotSupported) return e;
    e = launch_halo<T>(s, a);
    if (e != hipErrorNotSupported) return e;
    if constexpr (T_is_bf16<T>::value) {
      e = launch_wide<T>(s, a);
      if (e != hipErrorNotSupported) return e;
    }
  }
  // Widest cout tile (each loaded input fragment feeds MT MFMAs) that still puts about one wave on
  // every SIMD: the low-resolution GeoFeatureFusion layers have few pixels and many channels.
  const int gmt = gather_mt(a, T_is_bf16<T>::value);
  if (gmt == 8) return launch_mt<T, 8>(s, a);
  if (gmt == 4) return launch_mt<T, 4>(s, a);
  if (gmt == 2) return launch_mt<T, 2>(s, a);
  return launch_mt<T, 1>(s, a);
}

// Border correction of a 3x3 padding-1 conv whose bias was the full 9-tap sum: at each border pixel
// subtract the taps that fall outside the image (used by the re-associated FPN top level, where the
// bias of a 1x1 conv travels through a zero-padded 3x3 conv).
template <typename T>
__global__ __launch_bounds__(256) void border_bias_kernel(BorderArgs a, int B, int H, int W, int cstored, int cout, T* out) {
  const int per = 2 * W + 2 * (H - 2);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * per) return;
  const int b = i / per;
  int r = i - b * per, y, x;
  if (r < W) { y = 0; x = r; }
  else if (r < 2 * W) { y = H - 1; x = r - W; }
  else { r -= 2 * W; y = 1 + r / 2; x = (r & 1) ? W - 1 : 0; }
  T* o = out + (((size_t)b * H + y) * W + x) * cstored;
  for (int c = 0; c < cout; ++c) {
    float v = Stor<T>::to_f(o[c]);
    for (int t = 0; t < 9; ++t) {
      const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) v -= a.corr[t * 16 + c];
    }
    o[c] = Stor<T>::from_f(v);
  }
}

// FeatureNet's FPN top level in one launch (bf16): out = conv3x3_p1(c0; Wc) + ConvTranspose2d_k4s2p1(f; Wt) + bias,
// the two layers fpn_top_layers (frontend_hip.py) re-associates out3(up2(f) + inner2(c0)) into
// (models/module.py:455-459), fused so the transposed conv's full-resolution 8-channel output never makes an
// HBM round trip (at cfgC 606 MB written and read back). Both terms share the x-pair MFMA layout of the
// transposed conv: the 16 A rows are (output x parity px, channel co), the 16 B columns q-positions (output
// x = 2q + px). The 3x3 conv joins through x-pair taps too: output pair (2q, 2q+1) reads c0 at 2q-1..2q+2,
// one tap per lane group (8 channels), so each kernel row is one K chunk with A[(px, co)][(g, ci)] =
// Wc[co][ci][dy][g - px] (0 outside 0..2). A block owns 8 output rows x 64 q-columns (128 output columns):
// c0's (8+2) x 130-pixel halo sits in LDS split by x parity (16 consecutive q read 16 consecutive records)
// and f's 6 x 66-pixel x 32-channel halo with its 16-byte chunks XOR-swizzled by (pixel >> 2) & 3; both are
// filled by stage_chunks (8 loads in flight per lane). Per output row 3 + 6 MFMAs, the 15 A chunks in
// registers for the whole block. Row parity py of output row y0 + j is j & 1 (y0 is a multiple of 8).
constexpr int FT_Q = 64;
// T = float (the fp32 parity path): the same plan on split-f16 MFMAs (damvs_device.h mma_split32). c0's halo keeps each
// 8-channel record as its f16 hi / lo halves in two planes; f's 128-byte pixels keep chunk q's halves in slots q and
// 4 + q, slot position s at s ^ ((pixel >> 1) & 7) (WideForm<float>); A chunks [hi: 64 lanes][lo: 64 lanes] of
// A * 2^k, the epilogue scales by wscale = 2^-k. 4 output rows per block (59 KB of LDS: two blocks per CU).
template <typename T> struct FpnTopForm;
template <> struct FpnTopForm<bf16_t> {
  static constexpr int R = 8, PL = 1, FS = 4;  // output rows per block; 16-byte pieces per chunk; slots per f pixel
  __device__ __forceinline__ static int fslot(int fc, int q) { return q ^ ((fc >> 2) & 3); }
};
template <> struct FpnTopForm<float> {
  static constexpr int R = 4, PL = 2, FS = 8;
  __device__ __forceinline__ static int fslot(int fc, int q) { return q ^ ((fc >> 1) & 7); }
};

template <typename T>
__global__ __launch_bounds__(256) void fpn_top_kernel(const T* __restrict__ c0, const T* __restrict__ f,
                                                      const uint4* __restrict__ apack, float wscale,
                                                      const float* __restrict__ bias, T* __restrict__ out, int B, int H,
                                                      int W, int tiles_x, int tiles_y, int ntiles) {
  typedef FpnTopForm<T> Fm;
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int FT_R = Fm::R, PL = Fm::PL, FS = Fm::FS;
  constexpr uint32_t ES = sizeof(T);
  constexpr int CW = FT_Q + 2;                       // c0 records per (row, parity): q0-1 .. q0+64
  constexpr int C0_CHUNKS = (FT_R + 2) * 2 * CW;
  constexpr int FR = FT_R / 2 + 2, FC = FT_Q + 2;    // f halo rows x columns
  constexpr int F_CHUNKS = FR * FC * 4;              // 8-channel chunks of the f halo
  __shared__ uint4 sc0[C0_CHUNKS * PL];              // fp32: hi plane, then lo plane
  __shared__ uint4 sf[FR * FC * FS];

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y;
  const int b = tt / tiles_y;
  const int y0 = ty * FT_R, q0 = tx * FT_Q;
  const int Hh = H >> 1, Wh = W >> 1;
  const __amdgpu_buffer_rsrc_t rc0 = make_rsrc(c0, (long long)B * H * W * 8 * ES);
  const __amdgpu_buffer_rsrc_t rf = make_rsrc(f, (long long)B * Hh * Wh * 32 * ES);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;

  frag af[15];
#pragma unroll
  for (int c = 0; c < 15; ++c) af[c] = Z::wload(apack, c, lane);

  auto c0_off = [&](int c) -> uint32_t {  // byte offset of c0 halo record c (row, x parity, q)
    const int hr = c / (2 * CW), rem = c - hr * (2 * CW), par = rem / CW, jj = rem - par * CW;
    const int y = y0 - 1 + hr, x = 2 * (q0 - 1 + jj) + par;
    const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    return ok ? (uint32_t)((b * H + y) * W + x) * 8u * ES : kOOB;
  };
  auto f_off = [&](int p, int chunk) -> uint32_t {  // byte offset of chunk `chunk` of f halo pixel p
    const int fr = p / FC, fc = p - fr * FC;
    const int y = (y0 >> 1) - 1 + fr, x = q0 - 1 + fc;
    const bool ok = (unsigned)y < (unsigned)Hh && (unsigned)x < (unsigned)Wh;
    return ok ? (uint32_t)(((b * Hh + y) * Wh + x) * 4 + chunk) * 8u * ES : kOOB;
  };
  if constexpr (PL == 1) {
    stage_chunks<C0_CHUNKS, 8>(sc0, [&](int c) { return BufIO<bf16_t>::frag(rc0, c0_off(c)); });
    stage_chunks<F_CHUNKS, 8>(sf, [&](int c) {
      const int p = c >> 2, fc = p % FC;
      return BufIO<bf16_t>::frag(rf, f_off(p, (c & 3) ^ ((fc >> 2) & 3)));
    });
  } else {
    // 8-channel chunks as two 16-byte loads each, split at the LDS write; 4 chunks (8 loads) in flight per lane
    constexpr int NC = (C0_CHUNKS + 255) / 256, NF = (F_CHUNKS + 255) / 256;
#pragma unroll
    for (int i0 = 0; i0 < NC + NF; i0 += 4) {
      uint4 r[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = i0 + i, c = threadIdx.x + (k < NC ? k : k - NC) * 256;
        const bool isc = k < NC, ok = isc ? c < C0_CHUNKS : (k < NC + NF && c < F_CHUNKS);
        const uint32_t o = !ok ? kOOB : isc ? c0_off(c) : f_off(c >> 2, c & 3);
        const __amdgpu_buffer_rsrc_t rr = isc ? rc0 : rf;
        r[i][0] = BufIO<bf16_t>::frag(rr, o);
        r[i][1] = BufIO<bf16_t>::frag(rr, o == kOOB ? kOOB : o + 16u);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = i0 + i, c = threadIdx.x + (k < NC ? k : k - NC) * 256;
        const F16Pair v = split8(__builtin_bit_cast(float4, r[i][0]), __builtin_bit_cast(float4, r[i][1]));
        if (k < NC) {
          if (c < C0_CHUNKS) {
            sc0[c] = v.h;
            sc0[C0_CHUNKS + c] = v.l;
          }
        } else if (k < NC + NF && c < F_CHUNKS) {
          const int p = c >> 2, q = c & 3, fc = p % FC;
          sf[p * FS + Fm::fslot(fc, q)] = v.h;
          sf[p * FS + Fm::fslot(fc, q + 4)] = v.l;
        }
      }
    }
  }
  __syncthreads();

  f32x4_t acc[FT_R];
#pragma unroll
  for (int j = 0; j < FT_R; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int qn = wave * 16 + n;
  // c0 record of lane group g (x = 2q - 1 + g): parity plane (g + 1) & 1, index q - q0 + 1 + ((g - 1) >> 1)
  const uint4* c0b = sc0 + ((g + 1) & 1) * CW + qn + 1 + ((g - 1) >> 1);
  auto c0frag = [&](int i) -> frag {
    if constexpr (PL == 1) return c0b[i];
    else return F16Pair{c0b[i], c0b[C0_CHUNKS + i]};
  };
  auto ffrag = [&](int fr, int fc) -> frag {
    const uint4* px = sf + (fr * FC + fc) * FS;
    if constexpr (PL == 1) return px[Fm::fslot(fc, g)];
    else return F16Pair{px[Fm::fslot(fc, g)], px[Fm::fslot(fc, g + 4)]};
  };
#pragma unroll
  for (int j = 0; j < FT_R; ++j) {
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) Z::mma(af[dy], c0frag((j + dy) * 2 * CW), acc[j]);
    const int py = j & 1;
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
      for (int xx = 0; xx < 3; ++xx) Z::mma(af[3 + py * 6 + r2 * 3 + xx], ffrag(j / 2 + r2 + py, qn + xx), acc[j]);
  }

  const __amdgpu_buffer_rsrc_t ro = make_rsrc(out, (long long)B * H * W * 8 * ES);
  const int px = g >> 1, cb = (g & 1) * 4;
  float bs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bs[i] = bias[cb + i];
  const int x = 2 * (q0 + qn) + px;
#pragma unroll
  for (int j = 0; j < FT_R; ++j) {
    const int y = y0 + j;
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (PL == 1 ? acc[j][i] : acc[j][i] * wscale) + bs[i];  // 2^-k: exact
    const bool ok = y < H && x < W;
    BufIO<T>::stq(ro, ok ? (uint32_t)(((b * H + y) * W + x) * 8 + cb) * ES : kOOB, r);
  }
}

}  // namespace

hipError_t launch_fpn_top(hipStream_t s, int store, int B, int H, int W, const void* c0, const void* f,
                          const void* apack, float wscale, const float* bias, void* out) {
  const int R = store == ST_BF16 ? FpnTopForm<bf16_t>::R : FpnTopForm<float>::R;
  const int tx = (W / 2 + FT_Q - 1) / FT_Q, ty = (H + R - 1) / R;
  const long long nt = (long long)tx * ty * B;
  if (store == ST_BF16)
    hipLaunchKernelGGL(fpn_top_kernel<bf16_t>, dim3((unsigned)nt), dim3(256), 0, s, static_cast<const bf16_t*>(c0),
                       static_cast<const bf16_t*>(f), static_cast<const uint4*>(apack), 1.f, bias,
                       static_cast<bf16_t*>(out), B, H, W, tx, ty, (int)nt);
  else
    hipLaunchKernelGGL(fpn_top_kernel<float>, dim3((unsigned)nt), dim3(256), 0, s, static_cast<const float*>(c0),
                       static_cast<const float*>(f), static_cast<const uint4*>(apack), wscale, bias,
                       static_cast<float*>(out), B, H, W, tx, ty, (int)nt);
  return hipGetLastError();
}

hipError_t launch_border_bias(hipStream_t s, int store, const BorderArgs& a, int B, int H, int W, int cstored, int cout,
                              void* out) {
  const long long n = (long long)B * (2 * W + 2 * (H - 2));
  const dim3 grid((unsigned)((n + 255) / 256));
  if (store == ST_BF16)
    hipLaunchKernelGGL(border_bias_kernel<bf16_t>, grid, dim3(256), 0, s, a, B, H, W, cstored, cout, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(border_bias_kernel<float>, grid, dim3(256), 0, s, a, B, H, W, cstored, cout, static_cast<float*>(out));
  return hipGetLastError();
}

bool conv2d_wide_shape_ok(const Conv2dArgs& a) {
  int dmin = 0, span = 0;
  return wide_shape_ok(a, dmin, span);
}

hipError_t launch_conv2d(hipStream_t s, int store, const Conv2dArgs& a) {
  return store == ST_BF16 ? launch_t<bf16_t>(s, a) : launch_t<float>(s, a);
}

}  // namespace damvs
