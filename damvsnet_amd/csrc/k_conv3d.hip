// MFMA implicit-GEMM 3D convolution for the cost-regularisation U-Net (CostRegNet,
// models/module.py:510-541; wrappers Conv3d :117-159 and Deconv3d :161-202).
//
// Every layer is conv(bias=False) + BatchNorm3d (eval) + ReLU, optionally followed by a skip add
// (:537-539). BN is folded into the packed weights (scale) and a per-channel bias (shift); the
// ReLU and skip add run in the epilogue, so each layer is one read of its input and one write of
// its output (the skip tensor is read and overwritten in place).
//
// GEMM mapping (per 64-lane wave, 16x16 MFMA tiles):
//   A (M x K)  = folded weights, M = output channels (16 per tile, padded), K = taps x Cin
//   B (K x N)  = input patches,  N = 16 consecutive output voxels (one per lane column)
//   C (M x N)  = lane holds 4 consecutive output channels of one voxel -> one 8/16-byte store.
// With the NDHWC layout the B fragment of a lane is ONE 16-byte load: 8 bf16 (16x16x32 MFMA) or
// 4 f32 (16x16x4 f32 MFMA, exact fp32 — no xf32 on gfx950) consecutive input channels of one
// neighbouring voxel. Weights are pre-packed host side in exactly the A-fragment lane order.
//
// ConvTranspose3d(k3, s2, p1, op1) runs as 8 output-parity phases, each a dense sub-convolution
// with 1..8 taps (sub-pixel decomposition): no MFMA work on the structural zeros a
// zero-inserted transposed conv would carry.
#include <cstdlib>
#include <cstring>

#include "damvs_device.h"

namespace damvs {

namespace {

template <typename T> using Frag = MmaFrag<T>;

template <typename T>
__device__ __forceinline__ void store4(T* p, const float* r);
template <>
__device__ __forceinline__ void store4<float>(float* p, const float* r) {
  *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
}
template <>
__device__ __forceinline__ void store4<bf16_t>(bf16_t* p, const float* r) {
  uint32_t lo = (uint32_t)f2bf(r[0]) | ((uint32_t)f2bf(r[1]) << 16);
  uint32_t hi = (uint32_t)f2bf(r[2]) | ((uint32_t)f2bf(r[3]) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* r);
template <>
__device__ __forceinline__ void load4<float>(const float* p, float* r) {
  float4 v = *reinterpret_cast<const float4*>(p);
  r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
}
template <>
__device__ __forceinline__ void load4<bf16_t>(const bf16_t* p, float* r) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  r[0] = __uint_as_float(v.x << 16); r[1] = __uint_as_float(v.x & 0xffff0000u);
  r[2] = __uint_as_float(v.y << 16); r[3] = __uint_as_float(v.y & 0xffff0000u);
}

constexpr int kGroups = 4;  // 16-voxel column groups per wave (64 output voxels per wave)

// DAMVS_DIAG_SKIP_EPI selects the bf16 in-place skip epilogue of conv3d_mfma_kernel in DIAGNOSTIC builds only
// (tools/diag_skip_epilogue.py; the product is always 0): 0 = 16-byte records (lane group g+1 hands its 4
// channels to g); 1 = the former 8-byte-per-lane form (skip loaded through the `rr` descriptor, stored through
// `ro`); 2 = form 1 with one descriptor for both; 3 = form 1 with device-scope (sc1) skip loads, which miss the
// CU's L1; 4 = form 1 with every skip load of the wave issued before its first store. Forms 1-4 also run the
// x-pair deconv (XP) through the 8-byte path, as round 1 did before the 16-byte records.
#ifndef DAMVS_DIAG_SKIP_EPI
#define DAMVS_DIAG_SKIP_EPI 0
#endif

// The fp32 prescale of a conv kernel's input for batch element b (damvs_device.h prescale_of; one magnitude slot per
// batch element, so a sample's scales -- and bits -- do not depend on the other samples of its batch); bf16 kernels are
// unscaled (no load).
template <typename T>
__device__ __forceinline__ Prescale ps_in(const ConvArgs& a, int b) {
  if constexpr (sizeof(T) == 4) return prescale_of(a.in_amax ? a.in_amax + (size_t)b * kAmaxSlotWords : nullptr);
  else return Prescale{1.f, 1.f};
}
// the epilogue's accumulator scale: the weights' 2^-k (fp32) times the input's 2^-k
template <typename T>
__device__ __forceinline__ float ps_wscale(const ConvArgs& a, const Prescale& ps) {
  if constexpr (sizeof(T) == 4) return a.wscale * ps.inv;
  else return a.wscale;
}
// fold the stored values v[0..n) of an fp32 layer into the running output maximum (ok: the store is not dropped)
template <typename T, int NV>
__device__ __forceinline__ void am_fold(unsigned& am, bool ok, const float* v) {
  if constexpr (sizeof(T) == 4) {
    unsigned m = am;
#pragma unroll
    for (int i = 0; i < NV; ++i) m = amax_fold(m, v[i]);
    am = ok ? m : am;
  }
}
template <typename T>
__device__ __forceinline__ void am_flush(const ConvArgs& a, unsigned am, int b, int r) {
  if constexpr (sizeof(T) == 4) amax_flush(am, a.out_amax ? a.out_amax + (size_t)b * kAmaxSlotWords : nullptr, r);
}
// a loaded 16-byte fragment times the prescale (fp32; bf16 as is)
__device__ __forceinline__ float4 ps_scale(const float4& x, float s) { return scale4(x, s); }
__device__ __forceinline__ uint4 ps_scale(const uint4& x, float) { return x; }

// Epilogue for 4 channels: bias, ReLU, skip add (after the ReLU, models/module.py:537-539), store.
template <typename T>
__device__ __forceinline__ void finish4(const ConvArgs& a, __amdgpu_buffer_rsrc_t ro, __amdgpu_buffer_rsrc_t rr,
                                        const typename BufIO<T>::quad& q, bool has_res, uint32_t off, bool ok,
                                        const float* bias, const f32x4_t& acc, float wsc, unsigned& am) {
  float r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = fmaf(acc[i], wsc, bias[i]);
    if (a.relu) r[i] = relu(r[i]);
  }
  if (has_res) BufIO<T>::addq(q, r);
  am_fold<T, 4>(am, ok, r);
  BufIO<T>::stq(ro, ok ? off : kOOB, r);
  (void)rr;
}

// Global-gather implicit GEMM (strided convs, deconv phases, and any layer the LDS variant does not
// take). 32-bit incremental indexing: no divisions in the K loop, magic-number division for the
// voxel decomposition, range-checked buffer loads for the zero padding.
// XP: x-parity-pair deconv phases (build_phases_xpair): MFMA row r = (x parity r >> 3, channel r & 7),
// so lane group g stores channels (g & 1) * 4 .. +3 of output x = 2 qx + (g >> 1).
// K32 (fp32 only): 32 K per chunk as split-f16 16x16x32 MFMAs (8 channels per lane, split when loaded; A pairs from
// ConvArgs::wgat32, phases re-chunked at 32 K by the launcher): half the MFMA issue of the 16-K form.
template <typename T, int MT, bool XP, bool K32 = false>
__global__ __launch_bounds__(256) DAMVS_WAVES((sizeof(T) == 2 && MT == 4 ? 3 : 1)) void conv3d_mfma_kernel(const ConvArgs a, int nqblk) {
  constexpr int KG = kGroups;  // 16-voxel column groups per wave
  typedef BufIO<T> IO;
  typedef typename IO::raw raw;
  static_assert(!K32 || sizeof(T) == 4, "the 32-K split form is fp32 only");
  constexpr int E = K32 ? 8 : Stor<T>::E;  // input channels per lane per K-chunk
  constexpr int KC = 4 * E;      // K per chunk (4 lane groups)
  constexpr uint32_t ES = sizeof(T);
  // Logical block = (q-block, phase) with the phase fastest, dealt XCD-contiguously: the 8 output
  // parities of one deconv q-range run together on one XCD, so their interleaved half-line writes
  // (and the skip tensor's reads) merge in that L2.
  const int nblk = nqblk * a.nphase;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int qblk = L / a.nphase;
  const ConvPhase& ph = a.ph[L - qblk * a.nphase];
  __shared__ int s_tap[32];
  if (threadIdx.x < 27) {
    const signed char* t = ph.tap[threadIdx.x];
    s_tap[threadIdx.x] = ((int)(t[0] + 8)) | ((int)(t[1] + 8) << 8) | ((int)(t[2] + 8) << 16);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int Qtot = a.B * a.Dq * a.Hq * a.Wq;
  const int base = (qblk * 4 + wave) * (KG * 16);
  if (base >= Qtot) return;  // (whole waves: the rest keep all lanes to the end, as amax_flush needs)
  // fp32 magnitude slots are per batch element: a wave's 64 voxels span at most two elements (the launcher takes B > 1
  // only with Dq * Hq * Wq >= 64), b_lo and b_hi; each voxel's inputs are scaled by its own element's prescale, its
  // accumulators scaled back by it, and its outputs folded into that element's slot
  const int qpb = a.Dq * a.Hq * a.Wq;
  const int b_lo = base / qpb, b_hi = (min(base + KG * 16, Qtot) - 1) / qpb;
  const Prescale ps0 = ps_in<T>(a, b_lo), ps1 = b_hi != b_lo ? ps_in<T>(a, b_hi) : ps0;
  unsigned am0 = 0u, am1 = 0u;  // max |stored value| of b_lo's and b_hi's voxels (fp32: their magnitude slots)

  const int IS = a.in_stride, OS = a.out_stride;
  int zs[KG], ys[KG], xs[KG], pin[KG], pout[KG];
  bool valid[KG], hij[KG];  // hij: the voxel belongs to b_hi
  float sj[KG], wscj[KG];   // its input prescale, its accumulator scale
#pragma unroll
  for (int j = 0; j < KG; ++j) {
    int q = base + j * 16 + n;
    valid[j] = q < Qtot;
    q = valid[j] ? q : 0;
    const int r1 = fdiv(a.div_wq, q), qx = q - r1 * a.Wq;
    const int r2 = fdiv(a.div_hq, r1), qy = r1 - r2 * a.Hq;
    const int b = fdiv(a.div_dq, r2), qz = r2 - b * a.Dq;
    hij[j] = b != b_lo;
    sj[j] = hij[j] ? ps1.s : ps0.s;
    wscj[j] = ps_wscale<T>(a, hij[j] ? ps1 : ps0);
    zs[j] = qz * IS; ys[j] = qy * IS; xs[j] = qx * IS;
    pin[j] = ((b * a.Di + zs[j]) * a.Hi + ys[j]) * a.Wi + xs[j];
    pout[j] = ((b * a.Do + qz * OS + ph.pd) * a.Ho + qy * OS + ph.ph) * a.Wo + qx * OS + (XP ? (g >> 1) : ph.pw);
  }

  f32x4_t acc[KG][MT];
#pragma unroll
  for (int j = 0; j < KG; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.resid ? a.resid : a.out, a.resid ? nout : 0);
  constexpr bool kSkip16 = sizeof(T) == 2 && DAMVS_DIAG_SKIP_EPI == 0;
  const bool skip16 = kSkip16 && a.resid && (a.Cout & 7) == 0;

  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * a.Cin * ES);
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + (size_t)ph.w_off * 64 + lane;
  const int HW = a.Hi * a.Wi;
  int t = (g * E) / a.Cin, ci = g * E - t * a.Cin;  // this lane's (tap, channel) at k = s*KC + g*E
  const int qt = KC / a.Cin, rc = KC - qt * a.Cin;
  // loads of chunk s (the (t, ci) cursor is at chunk s and moves on to s + 1)
  auto load = [&](int s, raw (&wf)[MT], raw (&xf)[KG]) {
#pragma unroll
    for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)(s * MT + m) * 64];
    const bool tv = t < ph.ntaps;
    const int code = s_tap[tv ? t : 0];
    const int dz = (code & 0xff) - 8, dy = ((code >> 8) & 0xff) - 8, dx = ((code >> 16) & 0xff) - 8;
    const int tapoff = dz * HW + dy * a.Wi + dx;
#pragma unroll
    for (int j = 0; j < KG; ++j) {
      const int iz = zs[j] + dz, iy = ys[j] + dy, ix = xs[j] + dx;
      const bool ok = valid[j] && tv && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      xf[j] = IO::frag(r0, ok ? (uint32_t)((pin[j] + tapoff) * a.Cin + ci) * ES : kOOB);
      if constexpr (sizeof(T) == 4) xf[j] = scale4(xf[j], sj[j]);
    }
    ci += rc;
    t += qt;
    if (ci >= a.Cin) { ci -= a.Cin; ++t; }
  };
  auto mma = [&](const raw (&wf)[MT], const raw (&xf)[KG]) {
#pragma unroll
    for (int j = 0; j < KG; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) Frag<T>::mma(wf[m], xf[j], acc[j][m]);
  };
  if constexpr (K32) {
    const uint4* __restrict__ wq = reinterpret_cast<const uint4*>(a.wgat32) + (size_t)ph.w_off * 128 + lane;
    for (int s = 0; s < ph.kchunks; ++s) {
      F16Pair wf[MT], xf[KG];
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = F16Pair{wq[(size_t)(s * MT + m) * 128], wq[(size_t)(s * MT + m) * 128 + 64]};
      const bool tv = t < ph.ntaps;
      const int code = s_tap[tv ? t : 0];
      const int dz = (code & 0xff) - 8, dy = ((code >> 8) & 0xff) - 8, dx = ((code >> 16) & 0xff) - 8;
      const int tapoff = dz * HW + dy * a.Wi + dx;
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        const int iz = zs[j] + dz, iy = ys[j] + dy, ix = xs[j] + dx;
        const bool ok = valid[j] && tv && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                        (unsigned)ix < (unsigned)a.Wi;
        const uint32_t off = (uint32_t)((pin[j] + tapoff) * a.Cin + ci) * ES;
        const float4 lo4 = IO::frag(r0, ok ? off : kOOB), hi4 = IO::frag(r0, ok ? off + 16u : kOOB);
        xf[j] = split8s(lo4, hi4, sj[j]);
      }
      ci += rc;
      t += qt;
      if (ci >= a.Cin) { ci -= a.Cin; ++t; }
#pragma unroll
      for (int j = 0; j < KG; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) mma_split32(wf[m], xf[j], acc[j][m]);
    }
  } else {
    for (int s = 0; s < ph.kchunks; ++s) {
      raw wf[MT], xf[KG];
      load(s, wf, xf);
      mma(wf, xf);
    }
  }

  if constexpr (XP && DAMVS_DIAG_SKIP_EPI == 0) {
    // Cout = 8: lane group g + 1 hands its 4 channels to group g (g even), which then owns the whole
    // 8-channel record of output x = 2 qx + (g >> 1): one 16-byte (bf16) skip load and store per voxel.
    const bool lead = (g & 1) == 0;
    float b8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) b8[i] = a.bias[i];
#pragma unroll
    for (int j = 0; j < KG; ++j) {
      float r[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        r[i] = acc[j][0][i];
        r[4 + i] = __shfl_down(acc[j][0][i], 16);
      }
      if (!lead) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        r[i] = fmaf(r[i], wscj[j], b8[i]);
        if (a.relu) r[i] = relu(r[i]);
      }
      const uint32_t off = valid[j] ? (uint32_t)(pout[j] * 8) * ES : kOOB;
      if (a.resid) Vox8<T>::add(rr, off, r);
      unsigned amj = 0u;
      am_fold<T, 8>(amj, valid[j], r);
      am0 = hij[j] ? am0 : max(am0, amj);
      am1 = hij[j] ? max(am1, amj) : am1;
      Vox8<T>::store(ro, off, r);
    }
    am_flush<T>(a, am0, b_lo, blockIdx.x * 4 + wave);
    if (b_hi != b_lo) am_flush<T>(a, am1, b_hi, blockIdx.x * 4 + wave);
    return;
  }
  if constexpr (kSkip16) {
    if (skip16) {
      // bf16 in-place skip: lane group g + 1 hands its 4 channels to group g (g even), which loads / stores the
      // 8 channels as one 16-byte access. (The 8-byte-per-lane form of this in-place skip epilogue
      // lost the skip term of lane group 3's even channels in a few hundred voxels per launch on
      // gfx950, nondeterministically: tools/diag_unet_repro.py)
      const bool lead = (g & 1) == 0;
#pragma unroll
      for (int j = 0; j < KG; ++j) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          float r[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            r[i] = acc[j][m][i];
            r[4 + i] = __shfl_down(acc[j][m][i], 16);
          }
          const int co = m * 16 + g * 4;
          if (!lead || co >= a.Cout) continue;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            r[i] += a.bias[co + i];
            if (a.relu) r[i] = relu(r[i]);
          }
          const uint32_t off = valid[j] ? (uint32_t)(pout[j] * a.Cout + co) * ES : kOOB;
          if (a.resid) Vox8<T>::add(rr, off, r);
          Vox8<T>::store(ro, off, r);
        }
      }
      return;
    }
  }
  float bias[MT][4];
  bool cok[MT];
  const int cg = XP ? (g & 1) * 4 : g * 4;  // first channel of this lane group's 4
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = m * 16 + cg;
    cok[m] = co < a.Cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = cok[m] ? a.bias[co + i] : 0.f;
  }
  const __amdgpu_buffer_rsrc_t rq = DAMVS_DIAG_SKIP_EPI == 2 ? ro : rr;
  typename IO::quad q[KG][MT];
  auto load_skip = [&](int j) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint32_t off = valid[j] && cok[m] ? (uint32_t)(pout[j] * a.Cout + m * 16 + cg) * ES : kOOB;
      if (a.resid) q[j][m] = DAMVS_DIAG_SKIP_EPI == 3 ? IO::ldq_dev(rq, off) : IO::ldq(rq, off);
    }
  };
  if (DAMVS_DIAG_SKIP_EPI == 4) {
#pragma unroll
    for (int j = 0; j < KG; ++j) load_skip(j);
  }
#pragma unroll
  for (int j = 0; j < KG; ++j) {
    if (DAMVS_DIAG_SKIP_EPI != 4) load_skip(j);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint32_t off = (uint32_t)(pout[j] * a.Cout + m * 16 + cg) * ES;
      unsigned amj = 0u;
      finish4<T>(a, ro, rr, q[j][m], a.resid != nullptr, off, valid[j] && cok[m], bias[m], acc[j][m], wscj[j], amj);
      am0 = hij[j] ? am0 : max(am0, amj);
      am1 = hij[j] ? max(am1, amj) : am1;
    }
  }
  am_flush<T>(a, am0, b_lo, blockIdx.x * 4 + wave);
  if (b_hi != b_lo) am_flush<T>(a, am1, b_hi, blockIdx.x * 4 + wave);
}

// ---------------------------------------------------------------------------------------------
// LDS-staged variant for stride-1 k3 convs (conv0/2/4/6): a block owns a 4 x 8 x 16 output tile
// (512 voxels, 8 sixteen-voxel groups per wave). Its (4+2) x (8+2) x (16+2) x Cin halo is read from
// HBM/L2 once (16-byte loads, zero padding) into LDS; every K-chunk's B fragment is then a
// conflict-light ds_read_b128 instead of an L1 gather, cutting the L1/TA traffic that bounds the
// global-gather kernel by ~27x (each input voxel feeds 27 taps). Blocks are dealt so that
// consecutive tiles along x land on one XCD (bijective remap): neighbours' halos hit that L2.
constexpr int LTD = 4, LTH = 8, LTW = 16;
constexpr int LHD = LTD + 2, LHH = LTH + 2, LHW = LTW + 2;
constexpr int kLdsGroups = 8;  // per wave: 4 waves x 8 groups x 16 voxels = 512 = LTD*LTH*LTW

// chunk offset of tap t (= (kz, ky, kx) row-major) inside the halo tile, in 16-byte chunks
template <int CH>
__device__ constexpr int halo_toff(int t) {
  return t >= 27 ? halo_toff<CH>(26) : (((t / 9) * LHH + (t / 3) % 3) * LHW + t % 3) * CH;
}

template <typename T, int CIN>
constexpr size_t lds_tile_bytes() { return (size_t)LHD * LHH * LHW * CIN * sizeof(T); }

template <typename T, int CIN, int MT>
__global__ __launch_bounds__(256) void conv3d_lds_kernel(const ConvArgs a, int tiles_x, int tiles_y, int tiles_z,
                                                         int ntiles) {
  typedef typename Frag<T>::raw raw;
  constexpr int E = Stor<T>::E;
  constexpr int KC = 4 * E;
  constexpr int CH = CIN / E;                              // 16-byte chunks per voxel
  constexpr int KCHUNKS = (27 * CIN + KC - 1) / KC;
  constexpr int ROW = LHW * CH;                            // 16-byte chunks per halo row
  constexpr int TILE_CHUNKS = LHD * LHH * ROW;
  static_assert(kLdsGroups == LTH, "a wave owns one z-slice of the tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  raw* tile = reinterpret_cast<raw*>(smem);

  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous tile range.
  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  int tt = t;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % tiles_z;
  const int b = tt / tiles_z;
  const int z0 = tz * LTD, y0 = ty * LTH, x0 = tx * LTW;

  // halo fill: chunk c = (row, col) with row = (hz, hy); one row is LHW contiguous voxels in HBM
  const Prescale ps = ps_in<T>(a, b);
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * CIN * sizeof(T));
  const int vin0 = b * a.Di * a.Hi * a.Wi;
  stage_chunks<TILE_CHUNKS, 8>(tile, [&](int c) {
    const int row = c / ROW, col = c - row * ROW;
    const int hz = row / LHH, hy = row - hz * LHH;
    const int iz = z0 - 1 + hz, iy = y0 - 1 + hy, ix = x0 - 1 + col / CH;
    const bool ok = (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    const uint32_t off = (uint32_t)(((vin0 + (iz * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * 16);
    return BufIO<T>::frag(rin, ok ? off : kOOB);
  }, [&](const raw& r) { return Frag<T>::stage(ps_scale(r, ps.s)); });
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  f32x4_t acc[kLdsGroups][MT];
#pragma unroll
  for (int j = 0; j < kLdsGroups; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // wave = output z-slice, group j = output row y, lane column n = output x; group j's chunk is the
  // lane base + a compile-time offset j * ROW (folds into the ds_read immediate)
  const raw* tl = tile + (wave * LHH * LHW + n) * CH;
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack) + lane;
  // K index s*KC + g*E = tap*CIN + ci with tap = s*KC/CIN + (g*E)/CIN (KC is a multiple of CIN or
  // CIN a multiple of KC): with the loop fully unrolled, a lane's tap offset is one of <= 4
  // compile-time constants per chunk, picked by its lane group - no LDS table, no divisions.
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  const int gi = (g * E) / CIN;          // tap sub-index of this lane group (KC > CIN)
  const int gc = (g * E) % CIN / E;      // 16-byte channel chunk within the voxel
  auto frag_src = [&](int s) -> const raw* {
    const int kt = (s * KC) / CIN;       // first tap of chunk s (compile time after unrolling)
    const int kc = ((s * KC) % CIN) / E; // channel chunk offset of chunk s
    int off = halo_toff<CH>(kt);
    if (KC > CIN) {
      off = gi == 1 ? halo_toff<CH>(kt + 1) : off;
      off = gi == 2 ? halo_toff<CH>(kt + 2) : off;
      off = gi == 3 ? halo_toff<CH>(kt + 3) : off;
    }
    return tl + off + kc + gc;
  };
  raw xa[kLdsGroups], wa[MT];
  auto fetch = [&](int s, raw* xf, raw* wf) {
#pragma unroll
    for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)(s * MT + m) * 64];
    const raw* src = frag_src(s);
#pragma unroll
    for (int j = 0; j < kLdsGroups; ++j) xf[j] = src[j * ROW];
  };
  // K = 9 tap rows (kz, ky) x 3 taps (kx) x CIN. Long K loops (>= 54 chunks) iterate over the tap
  // rows at run time with the row body unrolled: a fully unrolled 108-chunk f32 loop takes the
  // compiler tens of minutes and buys nothing over a 12-chunk unrolled body.
  constexpr int CPT = CIN >= KC ? CIN / KC : 1;  // chunks per tap
  constexpr int RCH = 3 * CPT;                   // chunks per tap row
  if constexpr (CIN >= KC && KCHUNKS >= 54) {
    auto fetch_row = [&](int r, int s, raw* xf, raw* wf) {
      const int kz = r / 3, ky = r - kz * 3;
#pragma unroll
      for (int m = 0; m < MT; ++m) wf[m] = wp[(size_t)((r * RCH + s) * MT + m) * 64];
      const raw* src = tl + ((kz * LHH + ky) * LHW + s / CPT) * CH + (s % CPT) * (KC / E) + gc;
#pragma unroll
      for (int j = 0; j < kLdsGroups; ++j) xf[j] = src[j * ROW];
    };
    fetch_row(0, 0, xa, wa);
#pragma unroll 1
    for (int r = 0; r < 9; ++r) {
#pragma unroll
      for (int s = 0; s < RCH; ++s) {
        raw xb[kLdsGroups], wb[MT];
        const bool more = s + 1 < RCH || r + 1 < 9;
        if (s + 1 < RCH) fetch_row(r, s + 1, xb, wb);
        else if (r + 1 < 9) fetch_row(r + 1, 0, xb, wb);
#pragma unroll
        for (int j = 0; j < kLdsGroups; ++j)
#pragma unroll
          for (int m = 0; m < MT; ++m) Frag<T>::mma_staged(wa[m], xa[j], acc[j][m]);
        if (more) {
#pragma unroll
          for (int j = 0; j < kLdsGroups; ++j) xa[j] = xb[j];
#pragma unroll
          for (int m = 0; m < MT; ++m) wa[m] = wb[m];
        }
      }
    }
  } else if constexpr (CIN >= 32 && MT == 1) {
    // 27 chunks at 2 blocks per CU: the pipelined schedule's extra registers cost more than it hides
#pragma unroll
    for (int s = 0; s < KCHUNKS; ++s) {
      fetch(s, xa, wa);
#pragma unroll
      for (int j = 0; j < kLdsGroups; ++j) Frag<T>::mma_staged(wa[0], xa[j], acc[j][0]);
    }
  } else {
    // software-pipelined one chunk ahead: chunk s+1's fragments are read while chunk s's MFMAs run
    fetch(0, xa, wa);
#pragma unroll
    for (int s = 0; s < KCHUNKS; ++s) {
      raw xb[kLdsGroups], wb[MT];
      if (s + 1 < KCHUNKS) fetch(s + 1, xb, wb);
#pragma unroll
      for (int j = 0; j < kLdsGroups; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) Frag<T>::mma_staged(wa[m], xa[j], acc[j][m]);
      if (s + 1 < KCHUNKS) {
        __builtin_amdgcn_sched_group_barrier(0x100, kLdsGroups, 0);       // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, kLdsGroups * MT, 0);  // MFMA
#pragma unroll
        for (int j = 0; j < kLdsGroups; ++j) xa[j] = xb[j];
#pragma unroll
        for (int m = 0; m < MT; ++m) wa[m] = wb[m];
      }
    }
  }

  constexpr uint32_t ES = sizeof(T);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.resid ? a.resid : a.out, a.resid ? nout : 0);
  float bias[MT][4];
  bool cok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = m * 16 + g * 4;
    cok[m] = co < a.Cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[m][i] = cok[m] ? a.bias[co + i] : 0.f;
  }
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
#pragma unroll
  for (int j = 0; j < kLdsGroups; ++j) {
    const int oz = z0 + wave, oy = y0 + j, ox = x0 + n;
    const bool vok = oz < a.Do && oy < a.Ho && ox < a.Wo;
    const int pout = ((b * a.Do + oz) * a.Ho + oy) * a.Wo + ox;
    typename BufIO<T>::quad q[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint32_t off = (uint32_t)(pout * a.Cout + m * 16 + g * 4) * ES;
      if (a.resid) q[m] = BufIO<T>::ldq(rr, vok && cok[m] ? off : kOOB);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint32_t off = (uint32_t)(pout * a.Cout + m * 16 + g * 4) * ES;
      finish4<T>(a, ro, rr, q[m], a.resid != nullptr, off, vok && cok[m], bias[m], acc[j][m], wsc, am);
    }
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

// Row-pair variant for Cout <= 8 (conv0 of every stage): a 16-row MFMA tile holds 8 channels of
// output rows y and y+1 (pack_layer_pair), so no A row is padding and each B fragment (input row
// y-1+dy', dy' = 0..3) feeds both rows: per output row 18*CIN K instead of 27*CIN, i.e. 1.5x fewer
// MFMAs and LDS reads than conv3d_lds_kernel with half its M rows empty. Same tile and halo; a
// wave's 4 groups are the 4 row pairs of its z-slice, and every lane stores 4 useful channels.
template <int CH>
__device__ constexpr int halo_pair_toff(int t) {
  return t >= 36 ? halo_pair_toff<CH>(35) : (((t / 12) * LHH + (t / 3) % 4) * LHW + t % 3) * CH;
}

template <typename T, int CIN>
__global__ __launch_bounds__(256) void conv3d_lds_pair_kernel(const ConvArgs a, int tiles_x, int tiles_y, int tiles_z,
                                                              int ntiles) {
  typedef typename Frag<T>::raw raw;
  constexpr int E = Stor<T>::E;
  constexpr int KC = 4 * E;
  constexpr int CH = CIN / E;
  constexpr int KCHUNKS = (36 * CIN + KC - 1) / KC;
  constexpr int ROW = LHW * CH;
  constexpr int TILE_CHUNKS = LHD * LHH * ROW;
  constexpr int NP = LTH / 2;  // row pairs per z-slice
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  raw* tile = reinterpret_cast<raw*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  int tt = t;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % tiles_z;
  const int b = tt / tiles_z;
  const int z0 = tz * LTD, y0 = ty * LTH, x0 = tx * LTW;

  const Prescale ps = ps_in<T>(a, b);
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * CIN * sizeof(T));
  const int vin0 = b * a.Di * a.Hi * a.Wi;
  stage_chunks<TILE_CHUNKS, 8>(tile, [&](int c) {
    const int row = c / ROW, col = c - row * ROW;
    const int hz = row / LHH, hy = row - hz * LHH;
    const int iz = z0 - 1 + hz, iy = y0 - 1 + hy, ix = x0 - 1 + col / CH;
    const bool ok = (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
    const uint32_t off = (uint32_t)(((vin0 + (iz * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * 16);
    return BufIO<T>::frag(rin, ok ? off : kOOB);
  }, [&](const raw& r) { return Frag<T>::stage(ps_scale(r, ps.s)); });
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  f32x4_t acc[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const raw* tl = tile + (wave * LHH * LHW + n) * CH;
  const raw* __restrict__ wp = reinterpret_cast<const raw*>(a.wpack_pair) + lane;
  const int gi = (g * E) / CIN;
  const int gc = (g * E) % CIN / E;
  auto fetch = [&](int s, raw* xf, raw& wf) {
    wf = wp[(size_t)s * 64];
    const int kt = (s * KC) / CIN, kc = ((s * KC) % CIN) / E;
    int off = halo_pair_toff<CH>(kt);
    if (KC > CIN) {
      off = gi == 1 ? halo_pair_toff<CH>(kt + 1) : off;
      off = gi == 2 ? halo_pair_toff<CH>(kt + 2) : off;
      off = gi == 3 ? halo_pair_toff<CH>(kt + 3) : off;
    }
    const raw* src = tl + off + kc + gc;
#pragma unroll
    for (int j = 0; j < NP; ++j) xf[j] = src[2 * j * ROW];
  };
  raw xa[NP], wa;
  fetch(0, xa, wa);
#pragma unroll
  for (int s = 0; s < KCHUNKS; ++s) {
    raw xb[NP], wb;
    if (s + 1 < KCHUNKS) fetch(s + 1, xb, wb);
#pragma unroll
    for (int j = 0; j < NP; ++j) Frag<T>::mma_staged(wa, xa[j], acc[j]);
    if (s + 1 < KCHUNKS) {
#pragma unroll
      for (int j = 0; j < NP; ++j) xa[j] = xb[j];
      wa = wb;
    }
  }

  // lane group g holds rows 4g..4g+3 = channels (g & 1)*4 .. +3 of output row y + (g >> 1)
  constexpr uint32_t ES = sizeof(T);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.resid ? a.resid : a.out, a.resid ? nout : 0);
  const int co = (g & 1) * 4, r = g >> 1;
  const bool cok = co < a.Cout;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = cok ? a.bias[co + i] : 0.f;
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int oz = z0 + wave, oy = y0 + 2 * j + r, ox = x0 + n;
    const bool vok = oz < a.Do && oy < a.Ho && ox < a.Wo && cok;
    const int pout = ((b * a.Do + oz) * a.Ho + oy) * a.Wo + ox;
    const uint32_t off = (uint32_t)(pout * a.Cout + co) * ES;
    typename BufIO<T>::quad q;
    if (a.resid) q = BufIO<T>::ldq(rr, vok ? off : kOOB);
    finish4<T>(a, ro, rr, q, a.resid != nullptr, off, vok, bias, acc[j], wsc, am);
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

// z-sliding row-pair variant (conv0): a block owns an 8-row x TX-column output window over ZC
// consecutive z-planes and streams the input through a 4-plane ring of (8+2) x (TX+2) x CIN halo
// planes in LDS. Each output plane needs one new input plane, fetched into registers while the
// current plane's MFMAs run and written to the ring slot freed by the plane before (one barrier
// per plane): HBM/L2 re-reads drop from 2.1x (6x10x18 halo per 4x8x16 tile) to ~1.66x and the
// fill latency is hidden behind compute instead of preceding it. bf16: same K order, weights
// (pack_layer_pair) and accumulation chain as conv3d_lds_pair_kernel, identical results. fp32 (T = float, CIN 8 / 16):
// the split-f16 form (ZForm<float>), the row-pair packing at 32 K per chunk (ConvArgs::wpack32).
// Wave w owns row pair (y0 + 2w, y0 + 2w + 1); lane column n the output x = x0 + 16 xg + n.
template <typename T, int CIN, int TXG>
__global__ __launch_bounds__(256) DAMVS_WAVES(sizeof(T) == 4 && CIN <= 8 ? 2 : 1) void conv3d_zslide_pair_kernel(const ConvArgs a, int tiles_x, int tiles_y,
                                                                 int nzc, int zc, int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int E = 8, KC = 32, CH = CIN / E, S = CH * PL;
  constexpr int TX = 16 * TXG, PW = TX + 2, PH = LTH + 2;
  constexpr int PLANE = PH * PW * S;        // 16-byte slots per halo plane
  constexpr int NLD = (PH * PW * CH + 255) / 256;  // 8-channel chunks per thread per plane
  constexpr int KCHUNKS = 36 * CIN / KC;
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int x0 = tx * TX, y0 = ty * LTH, zb = tz * zc;
  const int zend = min(zb + zc, a.Do);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * CIN * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + ((iz + 4) & 3) * PLANE;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= PH * PW * CH) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
        const F16Pair p = split8s(v[i][0], v[i][1], ps.s);
        dst[vox * S + (q ^ sw)] = p.h;
        dst[vox * S + ((CH + q) ^ sw)] = p.l;
      }
    }
  };
  // the layer's A fragments stay in registers for all ZC planes (bf16: 18 / 36 VGPR quads for CIN 16 / 32)
  frag wreg[KCHUNKS];
  {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(PL == 1 ? a.wpack_pair : a.wpack32) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < KCHUNKS; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  }
  uint4 pa[NLD][PL], pb[NLD][PL];
#pragma unroll
  for (int p = -1; p <= 1; ++p) {
    load_plane(zb + p, pa);
    store_plane(zb + p, pa);
  }
  if (zb + 1 < zend) load_plane(zb + 2, pa);  // two planes ahead from here on
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int gi = (g * E) / CIN, gc = (g * E) % CIN / E;
  // bf16: this lane's chunk at tap (dy' = 0, dx = 0); fp32: its voxel (the chunk and its column swizzle per tap)
  const int lbase = PL == 1 ? (2 * wave * PW + n) * CH + gc : (2 * wave * PW + n) * S;
  const int sw0 = Z::template zsw<S>(n), sw1 = Z::template zsw<S>(n + 1), sw2 = Z::template zsw<S>(n + 2);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const int co = (g & 1) * 4, r = g >> 1;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = co < a.Cout ? a.bias[co + i] : 0.f;  // (Cout 4 leaves group 1 idle)
  const int oy = y0 + 2 * wave + r;

  // one output plane: plane z + 2 (in `cur`, loaded one plane earlier) goes to the ring after the
  // MFMAs; plane z + 3 is fetched into `nxt` before them, so each load has two planes of cover
  auto step = [&](int z, uint4 (*cur)[PL], uint4 (*nxt)[PL]) {
    if (z + 2 < zend) load_plane(z + 3, nxt);
    const uint4* pl[3] = {ring + ((z + 3) & 3) * PLANE + lbase, ring + ((z + 4) & 3) * PLANE + lbase,
                          ring + ((z + 5) & 3) * PLANE + lbase};
    f32x4_t acc[TXG];
#pragma unroll
    for (int xg = 0; xg < TXG; ++xg) acc[xg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    auto coord = [&](int s, int& off, int& kc, int& dx) DAMVS_INLINE {  // K chunk s: slot offset, chunk, column
      const int kt = (s * KC) / CIN;
      kc = ((s * KC) % CIN) / E;
      const int dz = kt / 12;  // uniform over the chunk's taps (12 taps per dz, 1/2/4 taps per chunk)
      auto toff = [](int t) { return (((t / 3) % 4) * PW + t % 3) * (PL == 1 ? CH : S); };
      off = toff(kt), dx = kt % 3;
      if (KC > CIN) {
        off = gi == 1 ? toff(kt + 1) : off;
        off = gi == 2 ? toff(kt + 2) : off;
        off = gi == 3 ? toff(kt + 3) : off;
        if (PL == 2) dx = (kt + gi) % 3;
      }
      off += (int)(pl[dz] - ring);
    };
    if constexpr (PL == 1) {
#pragma unroll
      for (int s = 0; s < KCHUNKS; ++s) {
        const frag wf = wreg[s];
        const int kt = (s * KC) / CIN, kc = ((s * KC) % CIN) / E;
        const int dz = kt / 12;  // uniform over the chunk's taps (12 taps per dz, 1/2/4 taps per chunk)
        auto toff = [](int t) { return (((t / 3) % 4) * PW + t % 3) * CH; };
        int off = toff(kt);
        if (KC > CIN) {
          off = gi == 1 ? toff(kt + 1) : off;
          off = gi == 2 ? toff(kt + 2) : off;
          off = gi == 3 ? toff(kt + 3) : off;
        }
        const uint4* src = pl[dz] + off + kc;
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) Z::mma(wf, src[16 * xg * CH], acc[xg]);
      }
    } else if constexpr (CIN != 8) {  // (fp32 CIN 16 / 32: the input-plane walk runs these layers; no prefetch, which
                                      // spills at CIN 16)
#pragma unroll
      for (int s = 0; s < KCHUNKS; ++s) {
        int off, kc, dx;
        coord(s, off, kc, dx);
        const int sw = dx == 0 ? sw0 : dx == 1 ? sw1 : sw2;
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) Z::mma(wreg[s], Z::bread(ring + off + 16 * xg * S, kc + gc, CH, sw), acc[xg]);
      }
    } else {
      // fp32 CIN 8 (stage-3 conv0): chunk s + 1's B pieces read while chunk s's MFMAs run (the sched_group_barriers
      // hold that order; the compiler's own schedule read each piece pair just before its MFMAs and waited on it):
      // stage 3 1.27 -> 1.24 ms at B = 4 (tools/unet_layers.py, profiles/r05/ab_conv0_r05j.txt)
      frag b0[TXG], b1[TXG];
#pragma unroll
      for (int s = -1; s < KCHUNKS; ++s) {
        if (s + 1 < KCHUNKS) {
          int off, kc, dx;
          coord(s + 1, off, kc, dx);
          const int sw = dx == 0 ? sw0 : dx == 1 ? sw1 : sw2;  // +16 columns keep the swizzle
#pragma unroll
          for (int xg = 0; xg < TXG; ++xg) {
            const frag f = Z::bread(ring + off + 16 * xg * S, kc + gc, CH, sw);
            if ((s + 1) & 1) b1[xg] = f;
            else b0[xg] = f;
          }
        }
        if (s < 0) continue;
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) Z::mma(wreg[s], (s & 1) ? b1[xg] : b0[xg], acc[xg]);
        if (s + 1 < KCHUNKS) __builtin_amdgcn_sched_group_barrier(0x100, 2 * TXG, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * TXG, 0);
      }
    }
#pragma unroll
    for (int xg = 0; xg < TXG; ++xg) {
      const int ox = x0 + 16 * xg + n;
      const bool vok = oy < a.Ho && ox < a.Wo && co < a.Cout;
      const uint32_t off = (uint32_t)((((b * a.Do + z) * a.Ho + oy) * a.Wo + ox) * a.Cout + co) * (uint32_t)ES;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (PL == 1 ? acc[xg][i] : acc[xg][i] * wsc) + bias[i];  // 2^-k: exact
        if (a.relu) v[i] = relu(v[i]);
      }
      am_fold<T, 4>(am, vok, v);
      BufIO<T>::stq(ro, vok ? off : kOOB, v);
    }
    if (z + 1 < zend) store_plane(z + 2, cur);  // slot of plane z - 2, last read before the previous barrier
    __syncthreads();
  };
  for (int z = zb; z < zend; z += 2) {
    step(z, pa, pb);
    if (z + 1 < zend) step(z + 1, pb, pa);
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

// conv0 with each input plane's B fragments read from LDS once (round 3): input plane p feeds output planes p + 1,
// p and p - 1 (kernel depths 0, 1, 2), so a block walks the INPUT planes and runs, per plane, the three depth
// slices' MFMAs on the same B fragments into three rotating accumulator sets (outputs p + 1, p, p - 1); output p - 1
// is complete after plane p and is written then. conv3d_zslide_pair_kernel reads every plane's fragments three times
// (once per output plane it feeds): one ds_read_b128 per MFMA, which bound it by LDS bandwidth at CIN 32 (stage 1).
// Per output plane and column group the MFMA chain is the same sequence (depth 0's chunks from plane z - 1, then
// depth 1's from plane z, then depth 2's from plane z + 1, chunks ascending; zero planes outside the volume
// included): bitwise the same results. Same weights; a 2-slot ring (loads two planes ahead) and, at CIN 32, 8 x 32
// output windows (TXG 2: twice the MFMAs per plane step).
template <typename T, int CIN, int TXG>
__global__ __launch_bounds__(256) DAMVS_WAVES(sizeof(T) == 4 ? (CIN == 32 ? 1 : 2) : CIN == 32 ? 2 : CIN == 16 ? 3 : 1) void conv3d_zreuse_pair_kernel(
    const ConvArgs a, int tiles_x, int tiles_y, int nzc, int zc, int ntiles) {
  // T = float: the split-f16 form of conv3d_zslide_pair_kernel<float> (ZForm<float>: hi / lo slots, column swizzle; the
  // 32-K row-pair packing wpack32) on the same input-plane walk: each plane's B fragments (hi and lo) are read from LDS
  // once for the three output planes they feed, a third of the zslide kernel's LDS reads
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int E = 8, KC = 32, CH = CIN / E, S = CH * PL;
  constexpr int TX = 16 * TXG, PW = TX + 2, PH = LTH + 2;
  constexpr int PLANE = PH * PW * S;            // 16-byte slots per halo plane
  constexpr int NLD = (PH * PW * CH + 255) / 256;  // 8-channel chunks per thread per plane
  constexpr int KCHUNKS = 36 * CIN / KC;
  constexpr int NJ = KCHUNKS / 3;  // K chunks per kernel depth
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int x0 = tx * TX, y0 = ty * LTH, zb = tz * zc;
  const int zend = min(zb + zc, a.Do);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * CIN * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + ((iz + 2) & 1) * PLANE;  // two slots: plane p + 1 goes where plane p - 1 was
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= PH * PW * CH) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
        const F16Pair p = split8s(v[i][0], v[i][1], ps.s);
        dst[vox * S + (q ^ sw)] = p.h;
        dst[vox * S + ((CH + q) ^ sw)] = p.l;
      }
    }
  };
  frag wreg[KCHUNKS];
  {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(PL == 1 ? a.wpack_pair : a.wpack32) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < KCHUNKS; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  }
  uint4 pa[NLD][PL], pb[NLD][PL];
  load_plane(zb - 1, pa);
  store_plane(zb - 1, pa);
  load_plane(zb, pa);  // stored at the end of step zb - 1; from there on planes are fetched two steps ahead
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int gi = (g * E) / CIN, gc = (g * E) % CIN / E;
  // bf16: this lane's chunk at tap (dy' = 0, dx = 0); fp32: its voxel (the chunk and its column swizzle per tap)
  const int lbase = PL == 1 ? (2 * wave * PW + n) * CH + gc : (2 * wave * PW + n) * S;
  const int sw0 = Z::template zsw<S>(n), sw1 = Z::template zsw<S>(n + 1), sw2 = Z::template zsw<S>(n + 2);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const int co = (g & 1) * 4, r = g >> 1;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = co < a.Cout ? a.bias[co + i] : 0.f;
  const int oy = y0 + 2 * wave + r;

  f32x4_t an[TXG], ac[TXG], ap[TXG];  // outputs p + 1, p, p - 1 of step p
#pragma unroll
  for (int xg = 0; xg < TXG; ++xg) an[xg] = ac[xg] = ap[xg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto epilogue = [&](int z, const f32x4_t* acc) {
#pragma unroll
    for (int xg = 0; xg < TXG; ++xg) {
      const int ox = x0 + 16 * xg + n;
      const bool vok = oy < a.Ho && ox < a.Wo && co < a.Cout;
      const uint32_t off = (uint32_t)((((b * a.Do + z) * a.Ho + oy) * a.Wo + ox) * a.Cout + co) * (uint32_t)ES;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (PL == 1 ? acc[xg][i] : acc[xg][i] * wsc) + bias[i];  // 2^-k: exact
        if (a.relu) v[i] = relu(v[i]);
      }
      am_fold<T, 4>(am, vok, v);
      BufIO<T>::stq(ro, vok ? off : kOOB, v);
    }
  };
  // step p: plane p + 1 (in `cur`) goes to the ring after the MFMAs, plane p + 2 is fetched into `nxt` before them
  auto step = [&](int p, uint4 (*cur)[PL], uint4 (*nxt)[PL]) {
    if (p + 2 <= zend) load_plane(p + 2, nxt);
    const uint4* src = ring + ((p + 2) & 1) * PLANE + lbase;
    const bool d0 = p + 1 < zend, d1 = p >= zb && p < zend, d2 = p - 1 >= zb;  // outputs p + 1, p, p - 1 here
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kt = (j * KC) / CIN, kc = ((j * KC) % CIN) / E;
      auto toff = [](int t) { return (((t / 3) % 4) * PW + t % 3) * (PL == 1 ? CH : S); };
      int off = toff(kt), dx = kt % 3;
      if (KC > CIN) {
        off = gi == 1 ? toff(kt + 1) : off;
        off = gi == 2 ? toff(kt + 2) : off;
        off = gi == 3 ? toff(kt + 3) : off;
        if (PL == 2) dx = (kt + gi) % 3;
      }
#pragma unroll
      for (int xg = 0; xg < TXG; ++xg) {
        frag bv;
        if constexpr (PL == 1) {
          bv = src[off + kc + 16 * xg * CH];
        } else {
          const int sw = dx == 0 ? sw0 : dx == 1 ? sw1 : sw2;  // +16 columns keep the swizzle
          bv = Z::bread(src + off + 16 * xg * S, kc + gc, CH, sw);
        }
        if (d0) Z::mma(wreg[j], bv, an[xg]);           // kernel depth 0
        if (d1) Z::mma(wreg[NJ + j], bv, ac[xg]);      // kernel depth 1
        if (d2) Z::mma(wreg[2 * NJ + j], bv, ap[xg]);  // kernel depth 2
      }
    }
    if (d2) epilogue(p - 1, ap);  // output p - 1 is complete
#pragma unroll
    for (int xg = 0; xg < TXG; ++xg) {
      ap[xg] = ac[xg];
      ac[xg] = an[xg];
      an[xg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    }
    if (p + 1 <= zend) store_plane(p + 1, cur);  // slot of plane p - 1, last read before the previous barrier
    __syncthreads();
  };
  for (int p = zb - 1; p <= zend; p += 2) {
    step(p, pa, pb);
    if (p + 1 <= zend) step(p + 1, pb, pa);
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

// fp32 conv0 with the kernel depths on different waves (round 6). The input-plane walk above keeps all 36 / 18 A pairs
// (CIN 32 / 16) of a layer in every wave: 288 / 144 registers, one / two waves per SIMD, MFMA busy 0.30 (stage 1 conv0
// 1.76 ms against a 0.57 ms MFMA floor). Here a block of 3 RP waves walks the input planes of an (2 RP) x (16 TXG)
// output window: wave (rp, dz) holds only kernel depth dz's NJ = KCHUNKS / 3 A pairs (96 / 48 / 24 registers) and, at
// input plane p, runs depth dz's MFMAs for output plane o = p + 1 - dz of row pair rp. The three partial sums of an
// output plane are chained through LDS in the walk order: depth 0's wave starts the accumulator at step o - 1 and
// leaves it in chain01, depth 1's wave continues it at step o (MFMAs into the loaded accumulator) and leaves it in
// chain12, depth 2's wave finishes it at step o + 1 and runs the epilogue. Per output plane and column group that is
// the input-plane walk's MFMA chain (depth 0's chunks, then depth 1's, then depth 2's, chunks ascending, fp32
// accumulator stored and reloaded exactly): bitwise the same results (test_conv0_dz_fp32_bitwise). The three depth
// waves read the same B fragments (3 ds_read_b128 pairs per plane where the walk read one), which the LDS carries at
// 2 / 3 of its rate beside the MFMAs at full rate. Ring: 2 slots as in the walk; chain buffers double-buffered by the
// output plane's parity.
template <int CIN, int RP, int TXG>
__global__ __launch_bounds__(192 * RP) DAMVS_WAVES(CIN == 8 ? 4 : 3) void conv0_dz_kernel(
    const ConvArgs a, int tiles_x, int tiles_y, int nzc, int zc, int ntiles) {
  typedef ZForm<float> Z;
  typedef Z::frag frag;
  constexpr int PL = 2, ES = 4, NT = 192 * RP;
  constexpr int E = 8, KC = 32, CH = CIN / E, S = CH * PL;
  constexpr int LR = 2 * RP;  // output rows per block
  constexpr int TX = 16 * TXG, PW = TX + 2, PH = LR + 2;
  constexpr int PLANE = PH * PW * S;             // 16-byte slots per halo plane
  constexpr int NLD = (PH * PW * CH + NT - 1) / NT;  // 8-channel chunks per thread per plane
  constexpr int KCHUNKS = 36 * CIN / KC;
  constexpr int NJ = KCHUNKS / 3;  // K chunks per kernel depth
  constexpr int CHAIN = RP * TXG * 64;  // float4 per chain buffer (one per lane, row pair and column group)
  static_assert(KC % CIN == 0 || CIN % KC == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);
  f32x4_t* chain = reinterpret_cast<f32x4_t*>(smem + 2 * PLANE * 16);  // [2 chains][2 parities][CHAIN]

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int x0 = tx * TX, y0 = ty * LR, zb = tz * zc;
  const int zend = min(zb + zc, a.Do);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * CIN * ES);
  const Prescale ps = ps_in<float>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<float>(a, ps);
  unsigned am = 0u;  // max |stored value| (the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) DAMVS_INLINE {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * NT;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) DAMVS_INLINE {
    uint4* dst = ring + ((iz + 2) & 1) * PLANE;  // two slots: plane p + 1 goes where plane p - 1 was
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * NT;
      if (c >= PH * PW * CH) continue;
      const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
      const F16Pair pr = split8s(v[i][0], v[i][1], ps.s);
      dst[vox * S + (q ^ sw)] = pr.h;
      dst[vox * S + ((CH + q) ^ sw)] = pr.l;
    }
  };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rp = wave % RP, dz = wave / RP;  // wave-uniform
  frag wreg[NJ];
  {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(a.wpack32) + lane;
#pragma unroll
    for (int j = 0; j < NJ; ++j) wreg[j] = Z::wload(wsrc, dz * NJ + j, 0);
  }
  uint4 pa[NLD][PL], pb[NLD][PL];
  load_plane(zb - 1, pa);
  store_plane(zb - 1, pa);
  load_plane(zb, pa);  // stored at the end of step zb - 1; from there on planes are fetched two steps ahead
  __syncthreads();

  const int n = lane & 15, g = lane >> 4;
  const int gi = (g * E) / CIN, gc = (g * E) % CIN / E;
  const int lbase = (2 * rp * PW + n) * S;
  const int sw0 = Z::template zsw<S>(n), sw1 = Z::template zsw<S>(n + 1), sw2 = Z::template zsw<S>(n + 2);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * a.Cout * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const int co = (g & 1) * 4, r = g >> 1;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = co < a.Cout ? a.bias[co + i] : 0.f;
  const int oy = y0 + 2 * rp + r;
  f32x4_t* const ch_in = chain + (dz == 2 ? 2 * CHAIN : 0);   // dz 1 reads chain01, dz 2 chain12
  f32x4_t* const ch_out = chain + (dz == 0 ? 0 : 2 * CHAIN);  // dz 0 writes chain01, dz 1 chain12
  const int cslot = rp * TXG * 64 + lane;

  // step p: input plane p (ring slot p & 1); plane p + 1 (in `cur`) goes to the ring after the MFMAs, plane p + 2 is
  // fetched into `nxt` before them
  auto step = [&](int p, uint4 (*cur)[PL], uint4 (*nxt)[PL]) DAMVS_INLINE {
    if (p + 2 <= zend) load_plane(p + 2, nxt);
    const int o = p + 1 - dz;  // this wave's output plane at this step
    if (o >= zb && o < zend) {
      f32x4_t acc[TXG];
      const int par = (o & 1) * CHAIN + cslot;
#pragma unroll
      for (int xg = 0; xg < TXG; ++xg)
        acc[xg] = dz == 0 ? (f32x4_t){0.f, 0.f, 0.f, 0.f} : ch_in[par + xg * 64];
      const uint4* src = ring + (p & 1) * PLANE + lbase;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int kt = (j * KC) / CIN, kc = ((j * KC) % CIN) / E;
        auto toff = [](int t) { return (((t / 3) % 4) * PW + t % 3) * S; };
        int off = toff(kt), dx = kt % 3;
        if (KC > CIN) {
          off = gi == 1 ? toff(kt + 1) : off;
          off = gi == 2 ? toff(kt + 2) : off;
          off = gi == 3 ? toff(kt + 3) : off;
          dx = (kt + gi) % 3;
        }
        const int sw = dx == 0 ? sw0 : dx == 1 ? sw1 : sw2;  // +16 columns keep the swizzle
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) Z::mma(wreg[j], Z::bread(src + off + 16 * xg * S, kc + gc, CH, sw), acc[xg]);
      }
      if (dz < 2) {
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) ch_out[par + xg * 64] = acc[xg];
      } else {
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg) {
          const int ox = x0 + 16 * xg + n;
          const bool vok = oy < a.Ho && ox < a.Wo && co < a.Cout;
          const uint32_t off = (uint32_t)((((b * a.Do + o) * a.Ho + oy) * a.Wo + ox) * a.Cout + co) * (uint32_t)ES;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[xg][i] * wsc + bias[i];  // 2^-k: exact
            if (a.relu) v[i] = relu(v[i]);
          }
          am_fold<float, 4>(am, vok, v);
          BufIO<float>::stq(ro, vok ? off : kOOB, v);
        }
      }
    }
    if (p + 1 <= zend) store_plane(p + 1, cur);  // slot of plane p - 1, last read before the previous barrier
    __syncthreads();
  };
  for (int p = zb - 1; p <= zend; p += 2) {
    step(p, pa, pb);
    if (p + 1 <= zend) step(p + 1, pb, pa);
  }
  am_flush<float>(a, am, b, blockIdx.x * 3 * RP + wave);
}

template <int CIN, int RP, int TXG>
hipError_t launch_dz_t(hipStream_t s, const ConvArgs& a) {
  constexpr int PLANE = (2 * RP + 2) * (16 * TXG + 2) * (CIN / 8) * 2;
  const size_t smem = 2 * PLANE * 16 + 4 * (size_t)RP * TXG * 64 * 16;
  constexpr int zc = 16;
  const int tx = (a.Wo + 16 * TXG - 1) / (16 * TXG), ty = (a.Ho + 2 * RP - 1) / (2 * RP), nzc = (a.Do + zc - 1) / zc;
  const long long nt = (long long)tx * ty * nzc * a.B;
  auto k = conv0_dz_kernel<CIN, RP, TXG>;
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)smem);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(192 * RP), smem, s, a, tx, ty, nzc, zc, (int)nt);
  return hipGetLastError();
}

// DAMVS_CONV0_DZ (read per call): "0" = off (the input-plane walk / output-plane walk as DAMVS_CONV0_REUSE says), "1"
// or "RP,TXG" = on at every CIN (RP,TXG: the block shape); unset: on at CIN 32 only. Measured at cfgC B = 4
// (tools/unet_layers.py, profiles/r06/layers_conv0_dz_r06e.txt): stage 1 (CIN 32) 1.787 -> 1.665 ms; stage 2 (CIN 16)
// 2.074 -> 2.614 ms and stage 3 (CIN 8) 1.304 -> 1.577 ms slower -- with one accumulator chain per wave (TXG 1) each
// B fragment's three split MFMAs depend on each other, where the walk interleaves three depths' accumulators; at CIN 32
// the three waves per SIMD (against one) cover that latency.
bool conv0_dz_shape(int CIN, int& rp, int& txg) {
  const char* v = getenv("DAMVS_CONV0_DZ");
  rp = 4;
  txg = CIN == 8 ? 2 : 1;
  if (!v || !v[0]) return CIN == 32;  // unset or empty: the default
  if (v[0] == '1' && !v[1]) return true;
  if (v[0] == '0') return false;
  const char* c = strchr(v, ',');
  rp = atoi(v);
  txg = c ? atoi(c + 1) : txg;
  return true;
}

template <int CIN>
hipError_t launch_dz(hipStream_t s, const ConvArgs& a, int rp, int txg) {
  // the shapes that build without spills (tests/test_codeobj.py): CIN 32 (4, 1); CIN 16 (4, 1), (2, 1); CIN 8 all four
  if (rp == 4 && txg == 1) return launch_dz_t<CIN, 4, 1>(s, a);
  if constexpr (CIN <= 16) {
    if (rp == 2 && txg == 1) return launch_dz_t<CIN, 2, 1>(s, a);
  }
  if constexpr (CIN == 8) {
    if (rp == 4 && txg == 2) return launch_dz_t<CIN, 4, 2>(s, a);
    if (rp == 2 && txg == 2) return launch_dz_t<CIN, 2, 2>(s, a);
  }
  return hipErrorInvalidValue;
}

bool zslide_disabled() {  // read per call: tests flip it between launches
  const char* v = getenv("DAMVS_CONV_NO_ZSLIDE");
  return v && v[0] == '1';
}

template <typename T, int CIN, int TXG>
hipError_t launch_zslide_pair_t(hipStream_t s, const ConvArgs& a) {
  constexpr int PLANE = (LTH + 2) * (16 * TXG + 2) * (CIN / 8) * ZForm<T>::PL;
  const size_t smem = 4 * PLANE * 16;
  constexpr int zc = 16;  // z-planes per block; measured: 16 beats 8 and 32 over stages 1-2 at B=4
  const int tx = (a.Wo + 16 * TXG - 1) / (16 * TXG), ty = (a.Ho + LTH - 1) / LTH, nzc = (a.Do + zc - 1) / zc;
  const long long nt = (long long)tx * ty * nzc * a.B;
  auto k = conv3d_zslide_pair_kernel<T, CIN, TXG>;
  if (smem > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)smem);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, nzc, zc, (int)nt);
  return hipGetLastError();
}

// conv0 on the input-plane walk (conv3d_zreuse_pair_kernel, 2-slot ring)
template <typename T, int CIN, int TXG>
hipError_t launch_zreuse_pair_t(hipStream_t s, const ConvArgs& a) {
  constexpr int PLANE = (LTH + 2) * (16 * TXG + 2) * (CIN / 8) * ZForm<T>::PL;
  const size_t smem = 2 * PLANE * 16;
  constexpr int zc = 16;
  const int tx = (a.Wo + 16 * TXG - 1) / (16 * TXG), ty = (a.Ho + LTH - 1) / LTH, nzc = (a.Do + zc - 1) / zc;
  const long long nt = (long long)tx * ty * nzc * a.B;
  hipLaunchKernelGGL((conv3d_zreuse_pair_kernel<T, CIN, TXG>), dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, nzc, zc,
                     (int)nt);
  return hipGetLastError();
}

template <typename T, int CIN>
hipError_t launch_lds_pair_t(hipStream_t s, const ConvArgs& a) {
  if constexpr (sizeof(T) == 2) {
    if (!a.resid && !zslide_disabled()) {
      // DAMVS_CONV0_REUSE (read per call): 1 = the input-plane walk at every CIN, 0 = never; default: CIN 32 only
      // (at CIN 8 / 16 its registers cost a wave per SIMD: stage 2 / 3 U-Net 2.09 / 1.89 -> 2.22 / 2.01 ms)
      const char* rv = getenv("DAMVS_CONV0_REUSE");
      const bool reuse = rv ? rv[0] == '1' : CIN == 32;
      if (reuse) return launch_zreuse_pair_t<T, CIN, 2>(s, a);
      if constexpr (CIN == 32) return launch_zslide_pair_t<T, CIN, 1>(s, a);
      else return launch_zslide_pair_t<T, CIN, 2>(s, a);
    }
  } else {
    // fp32: the split-f16 z-streamed kernel on the 32-K row-pair packing, A fragments in registers (CIN 32: 36 pairs,
    // 288 VGPRs, with the 92 KB ring one block and one wave per SIMD)
    if (!a.resid && a.wpack32 && !zslide_disabled()) {
      int rp, txg;
      if (conv0_dz_shape(CIN, rp, txg)) return launch_dz<CIN>(s, a, rp, txg);
      // DAMVS_CONV0_REUSE (read per call): 1 = the input-plane walk, 0 = the output-plane walk; default: the walk at CIN
      // 16 / 32 (bitwise equal, test_conv0_reuse_fp32_bitwise)
      const char* rv = getenv("DAMVS_CONV0_REUSE");
      const bool reuse = rv ? rv[0] == '1' : CIN >= 16;
      if (reuse) return launch_zreuse_pair_t<T, CIN, CIN >= 16 ? 1 : 2>(s, a);
      if constexpr (CIN >= 16) return launch_zslide_pair_t<T, CIN, 1>(s, a);  // 8 x 16 windows, no spill
      else return launch_zslide_pair_t<T, CIN, 2>(s, a);
    }
  }
  const size_t smem = lds_tile_bytes<T, CIN>();
  auto k = conv3d_lds_pair_kernel<T, CIN>;
  if (smem > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
  }
  const int tx = (a.Wo + LTW - 1) / LTW, ty = (a.Ho + LTH - 1) / LTH, tz = (a.Do + LTD - 1) / LTD;
  const long long nt = (long long)tx * ty * tz * a.B;
  hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, tz, (int)nt);
  return hipGetLastError();
}

template <typename T, int CIN, int MT>
hipError_t launch_lds_t(hipStream_t s, const ConvArgs& a) {
  const size_t smem = lds_tile_bytes<T, CIN>();
  auto k = conv3d_lds_kernel<T, CIN, MT>;
  if (smem > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
  }
  const int tx = (a.Wo + LTW - 1) / LTW, ty = (a.Ho + LTH - 1) / LTH, tz = (a.Do + LTD - 1) / LTD;
  const long long nt = (long long)tx * ty * tz * a.B;
  hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, tz, (int)nt);
  return hipGetLastError();
}

// conv2 (Conv3d k3 s1 p1, 16 -> 16 channels) streamed along z on conv0's plan (4-slot ring of
// (8+2) x (TX+2) x 16-channel planes, two planes ahead), with 16 output channels as the MFMA rows
// instead of conv0's row pairs: K = 27 taps x 16 channels in 14 chunks of 2 taps (lane group g:
// tap 2s + (g >> 1), channel half g & 1; a chunk's two taps may sit in different planes), the 14 A
// fragments in registers. bf16 (TXG 2): same K order and weights as conv3d_lds_kernel. fp32 (T = float, TXG 1:
// 8 x 16 windows, so the 14 split A pairs fit beside two waves per SIMD): the split-f16 form on the layer's 32-K
// packing (ConvArgs::wpack32).
template <typename T, int TXG>
__global__ __launch_bounds__(256) DAMVS_WAVES(sizeof(T) == 4 ? 2 : 1) void conv_s1_c16_zslide_kernel(const ConvArgs a, int tiles_x, int tiles_y, int nzc,
                                                                 int zc, int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int CH = 2, S = CH * PL, TX = 16 * TXG, PW = TX + 2, PH = LTH + 2;
  constexpr int PLANE = PH * PW * S;
  constexpr int NLD = (PH * PW * CH + 255) / 256;
  constexpr int KCH = 14;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int x0 = tx * TX, y0 = ty * LTH, zb = tz * zc;
  const int zend = min(zb + zc, a.Do);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * 16 * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = y0 - 1 + row, ix = x0 - 1 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + x0 - 1) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + ((iz + 4) & 3) * PLANE;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= PH * PW * CH) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
        const F16Pair p = split8s(v[i][0], v[i][1], ps.s);
        dst[vox * S + (q ^ sw)] = p.h;
        dst[vox * S + ((CH + q) ^ sw)] = p.l;
      }
    }
  };
  frag wreg[KCH];
  {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(PL == 1 ? a.wpack : a.wpack32) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < KCH; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  }
  uint4 pa[NLD][PL], pb[NLD][PL];
#pragma unroll
  for (int p = -1; p <= 1; ++p) {
    load_plane(zb + p, pa);
    store_plane(zb + p, pa);
  }
  if (zb + 1 < zend) load_plane(zb + 2, pa);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int gi = g >> 1, gc = g & 1;
  // output row 2w (halo row 2w at dy = 0), column n: bf16 the lane's chunk, fp32 its voxel
  const int lbase = PL == 1 ? (2 * wave * PW + n) * CH + gc : (2 * wave * PW + n) * S;
  const int sw0 = Z::template zsw<S>(n), sw1 = Z::template zsw<S>(n + 1), sw2 = Z::template zsw<S>(n + 2);
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * 16 * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = a.bias[g * 4 + i];

  auto step = [&](int z, uint4 (*cur)[PL], uint4 (*nxt)[PL]) {
    if (z + 2 < zend) load_plane(z + 3, nxt);
    const uint4* pl[3] = {ring + ((z + 3) & 3) * PLANE + lbase, ring + ((z + 4) & 3) * PLANE + lbase,
                          ring + ((z + 5) & 3) * PLANE + lbase};
    f32x4_t acc[2][TXG];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int xg = 0; xg < TXG; ++xg) acc[r][xg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KCH; ++s) {
      auto tap = [&](int t) {  // (plane, in-plane offset, dx); tap 27 (K padding) reads tap 26 against zero weights
        const int tc = t < 27 ? t : 26;
        return (tc / 9) * 65536 + (((tc / 3) % 3) * PW + tc % 3) * (PL == 1 ? CH : S) * 4 + tc % 3;
      };
      const int code = gi ? tap(2 * s + 1) : tap(2 * s);
      const int dz = code >> 16, o = (code & 0xffff) >> 2, dx = code & 3;
      const uint4* src = (dz == 0 ? pl[0] : dz == 1 ? pl[1] : pl[2]) + o;
      const int sw = dx == 0 ? sw0 : dx == 1 ? sw1 : sw2;  // fp32: the tap's column swizzle (+16 columns keep it)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int xg = 0; xg < TXG; ++xg)
          Z::mma(wreg[s],
                 Z::bread(src + r * PW * (PL == 1 ? CH : S) + 16 * xg * (PL == 1 ? CH : S), PL == 1 ? 0 : gc, CH, sw),
                 acc[r][xg]);  // bf16: lbase already holds the lane's chunk
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int xg = 0; xg < TXG; ++xg) {
        const int oy = y0 + 2 * wave + r, ox = x0 + 16 * xg + n;
        const bool ok = oy < a.Ho && ox < a.Wo;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = (PL == 1 ? acc[r][xg][i] : acc[r][xg][i] * wsc) + bias[i];  // 2^-k: exact
          if (a.relu) v[i] = relu(v[i]);
        }
        am_fold<T, 4>(am, ok, v);
        BufIO<T>::stq(ro, ok ? (uint32_t)((((b * a.Do + z) * a.Ho + oy) * a.Wo + ox) * 16 + g * 4) * (uint32_t)ES : kOOB, v);
      }
    if (z + 1 < zend) store_plane(z + 2, cur);
    __syncthreads();
  };
  for (int z = zb; z < zend; z += 2) {
    step(z, pa, pb);
    if (z + 1 < zend) step(z + 1, pb, pa);
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

// Returns hipErrorNotSupported when no LDS variant fits this layer (caller falls back).
template <typename T>
hipError_t launch_lds(hipStream_t s, const ConvArgs& a) {
  if (a.nphase != 1 || a.in_stride != 1 || a.out_stride != 1 || a.ph[0].ntaps != 27) return hipErrorNotSupported;
  const int MT = a.MT;
  if (a.wpack_pair && a.Cout <= 8) {
    if (a.Cin == 8) return launch_lds_pair_t<T, 8>(s, a);
    if (a.Cin == 16) return launch_lds_pair_t<T, 16>(s, a);
    if (a.Cin == 32) return launch_lds_pair_t<T, 32>(s, a);  // fp32: the 138 KB tile (one block per CU)
  }
  if ((sizeof(T) == 2 || a.wpack32) && a.Cin == 16 && a.Cout == 16 && MT == 1 && !a.resid && !zslide_disabled()) {
    constexpr int zc = 16, TXG = sizeof(T) == 2 ? 2 : 1;
    const int tx = (a.Wo + 16 * TXG - 1) / (16 * TXG), ty = (a.Ho + LTH - 1) / LTH, nzc = (a.Do + zc - 1) / zc;
    const long long nt = (long long)tx * ty * nzc * a.B;
    const size_t smem = 4 * (LTH + 2) * (16 * TXG + 2) * 2 * 16 * ZForm<T>::PL;
    hipLaunchKernelGGL((conv_s1_c16_zslide_kernel<T, TXG>), dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, nzc, zc,
                       (int)nt);
    return hipGetLastError();
  }
  // The 4 x 8 x 16 tile stages a 6-plane halo: with fewer than 4 output planes (the deep levels at D = 8) most of
  // it is padding, and at 64 channels (conv6) it takes 138 KB of LDS (one block per CU). Measured (B=4, bf16)
  // the gather kernel wins both: conv6 98 -> 64 us (stage 2), 165 -> 53 us (stage 3); conv4 at stage 3 (2
  // planes) 137 -> 117 us, while conv4 at stage 2 (8 planes) keeps the tile (93 against 137 us).
  if (a.Do < LTD || a.Cin >= 64) return hipErrorNotSupported;
  if (a.Cin == 8 && MT == 1) return launch_lds_t<T, 8, 1>(s, a);
  if (a.Cin == 16 && MT == 1) return launch_lds_t<T, 16, 1>(s, a);
  if (a.Cin == 32 && MT == 1) return launch_lds_t<T, 32, 1>(s, a);
  if (a.Cin == 32 && MT == 2) return launch_lds_t<T, 32, 2>(s, a);
  return hipErrorNotSupported;
}

// conv11 (ConvTranspose3d k3 s2 p1 op1, 16 -> 8 channels, in-place skip) streamed along z:
// a block owns 8 x 16 input-grid columns (q) over DZ consecutive q-planes; input planes pass
// through a 4-slot LDS ring ((8+1) x (16+1) x 16 channels: the deconv only reaches offsets 0 and
// +1), loaded two planes ahead. Per q-plane each wave produces, for its 2 q-rows, the 4 (pz, py)
// x-pair phases of build_phases_xpair (K chunk (a, b) = z offset a, y offset b, lane group g >> 1 =
// x offset, g & 1 = channel half) with the 9 A fragments in registers, so the whole layer is the
// skip read + output write + one pass over the input, with no per-lane tap decoding or bounds tests
// in the K loop. bf16: same K order and weights as the x-pair gather kernel, identical results. fp32 (T = float):
// the split-f16 form (ZForm<float>: fp32 loads split once into the ring, 3 MFMAs per product, fp32 skip and output).
template <typename T>
__global__ __launch_bounds__(256) DAMVS_WAVES(sizeof(T) == 2 ? 3 : 2) void deconv_xpair_zslide_kernel(const ConvArgs a, int tiles_x, int tiles_y,
                                                                  int nzc, int zc, int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int CH = 2, S = CH * PL, QX = 16, QY = 8, PW = QX + 1, PH = QY + 1;
  constexpr int PLANE = PH * PW * S;           // 16-byte slots per ring plane
  constexpr int NLD = (PH * PW * CH + 255) / 256;  // 8-channel chunks per thread per plane
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int qx0 = tx * QX, qy0 = ty * QY, zb = tz * zc;
  const int zend = min(zb + zc, a.Di);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * 16 * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = qy0 + row, ix = qx0 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + qx0) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + (iz & 3) * PLANE;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= PH * PW * CH) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
        const F16Pair p = split8s(v[i][0], v[i][1], ps.s);
        dst[vox * S + (q ^ sw)] = p.h;
        dst[vox * S + ((CH + q) ^ sw)] = p.l;
      }
    }
  };
  // A fragments: bf16 in registers (9 x 4 VGPRs); fp32 (split, twice the registers) in LDS after the ring, read per
  // use, so the kernel keeps two waves per SIMD
  constexpr int NWR = PL == 1 ? 9 : 1;
  frag wreg[NWR];
  uint4* alds = ring + 4 * PLANE;  // fp32: 9 chunks x 128 slots
  if constexpr (PL == 1) {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(a.wpack) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < 9; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  } else {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(a.wpack);
    for (int i = threadIdx.x; i < 9 * 128; i += 256) alds[i] = wsrc[i];
  }
  auto wfrag = [&](int s) -> frag {
    if constexpr (PL == 1) return wreg[s];
    else return Z::wload(alds, s, threadIdx.x & 63);
  };
  uint4 pa[NLD][PL], pb[NLD][PL];
  load_plane(zb, pa);
  store_plane(zb, pa);
  load_plane(zb + 1, pa);
  store_plane(zb + 1, pa);
  if (zb + 1 < zend) load_plane(zb + 2, pa);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const bool lead = (g & 1) == 0;
  const int lcol = n + (g >> 1), lsw = Z::template zsw<S>(lcol);
  const int lbase = (2 * wave * PW + lcol) * S + (PL == 1 ? (g & 1) : 0);  // q-row 2w, column n, x offset g>>1
  const int lch = PL == 1 ? 0 : (g & 1);  // chunk (channel half) of this lane group, split form
  float b8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b8[i] = a.bias[i];
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * 8 * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.resid ? a.resid : a.out, a.resid ? nout : 0);
  const int qx = qx0 + n;

  auto step = [&](int qz, uint4 (*cur)[PL], uint4 (*nxt)[PL]) {
    if (qz + 2 < zend) load_plane(qz + 3, nxt);
    // output offsets and the skip records of this plane's 8 outputs, loaded before the MFMAs. bf16: lane group g (even)
    // owns the whole 16-byte record of output x = 2 qx + (g >> 1) (its partner's 4 channels by a shuffle); fp32: every
    // lane owns its 4 channels' 16 bytes (channel half g & 1), so all lanes load and store and no shuffle is needed
    uint32_t off[8];
    uint4 rq[8][1];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int pd = k >> 2, py = (k >> 1) & 1, r = k & 1;
      const int qy = qy0 + 2 * wave + r;
      const bool ok = (PL == 2 || lead) && qy < a.Hi && qx < a.Wi;
      const int oz = 2 * qz + pd, oy = 2 * qy + py, ox = 2 * qx + (g >> 1);
      off[k] = ok ? (uint32_t)((((b * a.Do + oz) * a.Ho + oy) * a.Wo + ox) * 8) * (uint32_t)ES + (PL == 2 ? 16u * (g & 1) : 0u)
                  : kOOB;
      rq[k][0] = BufIO<bf16_t>::frag(rr, off[k]);  // zero when there is no skip tensor (empty range)
    }
    const uint4* p0 = ring + (qz & 3) * PLANE + lbase;        // q-plane qz (z offset 0)
    const uint4* p1 = ring + ((qz + 1) & 3) * PLANE + lbase;  // q-plane qz + 1 (z offset +1)
    f32x4_t acc[8];  // [pd][py][r]
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pd = 0; pd < 2; ++pd)
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        const int na = pd ? 2 : 1, nb = py ? 2 : 1;
        const int w0 = (pd * 2 + py) == 0 ? 0 : (pd * 2 + py) == 1 ? 1 : (pd * 2 + py) == 2 ? 3 : 5;
#pragma unroll
        for (int ca = 0; ca < na; ++ca)
#pragma unroll
          for (int cb = 0; cb < nb; ++cb) {
            const int zo = pd ? (ca == 0 ? 1 : 0) : 0, yo = py ? (cb == 0 ? 1 : 0) : 0;
            const frag w = wfrag(w0 + ca * nb + cb);
            const uint4* src = (zo ? p1 : p0) + yo * PW * S;
#pragma unroll
            for (int r = 0; r < 2; ++r)
              Z::mma(w, Z::bread(src + r * PW * S, lch, CH, lsw), acc[(pd * 2 + py) * 2 + r]);
          }
      }
    // epilogue per output: (bf16: partner channels,) bias, ReLU, skip (after the ReLU), 16-byte store
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (PL == 2) {
        const float4 f = __builtin_bit_cast(float4, rq[k][0]);
        const float sk[4] = {f.x, f.y, f.z, f.w};
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[k][i] * wsc + b8[(g & 1) * 4 + i];  // 2^-k: exact
          if (a.relu) v[i] = relu(v[i]);
          v[i] += sk[i];
        }
        BufIO<T>::stq(ro, off[k], v);
        continue;
      }
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[k][i];
        v[4 + i] = __shfl_down(acc[k][i], 16);
      }
      if constexpr (PL == 1) {
        const uint32_t q4[4] = {rq[k][0].x, rq[k][0].y, rq[k][0].z, rq[k][0].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] += b8[i];
          if (a.relu) v[i] = relu(v[i]);
          v[i] += __uint_as_float((i & 1) ? (q4[i >> 1] & 0xffff0000u) : (q4[i >> 1] << 16));
        }
      }
      if (lead) Vox8<T>::store(ro, off[k], v);
    }
    if (qz + 1 < zend) store_plane(qz + 2, cur);  // slot of plane qz - 2, released by the last barrier
    __syncthreads();
  };
  for (int qz = zb; qz < zend; qz += 2) {
    step(qz, pa, pb);
    if (qz + 1 < zend) step(qz + 1, pb, pa);
  }
}

// conv9 (ConvTranspose3d k3 s2 p1 op1, 32 -> 16 channels, in-place skip) streamed along z like
// deconv_xpair_zslide_kernel: 4-slot LDS ring of (8+1) x (16+1) x 32-channel input q-planes loaded
// two ahead, the 27 A fragments (8 single-parity phases of build_phases, 1 tap per K chunk, lane
// group g = channel block g); per q-plane and half (pd) each wave issues its 8 skip records, then the
// 4 (py, px) phases x 2 q-rows, then the 16-byte epilogue (lane group g + 1 hands its 4 channels to group g).
// bf16 (ALDS): the A fragments in LDS after the ring (27 KB) instead of 108 VGPRs, two waves per SIMD; same K order
// and weights as the gather kernel. fp32 (T = float, split-f16 form, the 32-K packing ConvArgs::wpack32): the 78 KB
// ring leaves one block per CU, so the 27 A pairs sit in registers (one wave per SIMD, no LDS reads for A).
template <typename T, bool ALDS>
__global__ __launch_bounds__(256) DAMVS_WAVES(ALDS ? 2 : 1) void deconv_c16_zslide_kernel(const ConvArgs a, int tiles_x, int tiles_y, int nzc,
                                                                int zc, int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int CH = 4, S = CH * PL, QX = 16, QY = 8, PW = QX + 1, PH = QY + 1;
  constexpr int PLANE = PH * PW * S;
  constexpr int NLD = (PH * PW * CH + 255) / 256;
  static_assert(!ALDS || PL == 1, "A fragments in LDS: bf16 form");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int qx0 = tx * QX, qy0 = ty * QY, zb = tz * zc;
  const int zend = min(zb + zc, a.Di);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * 32 * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / (PW * CH), col = c - row * (PW * CH);
      const int iy = qy0 + row, ix = qx0 + col / CH;
      const bool ok = c < PH * PW * CH && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)((((b * a.Di + iz) * a.Hi + iy) * a.Wi + qx0) * CH + col) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + (iz & 3) * PLANE;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= PH * PW * CH) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int vox = c / CH, q = c - vox * CH, sw = Z::template zsw<S>(vox % PW);
        const F16Pair p = split8s(v[i][0], v[i][1], ps.s);
        dst[vox * S + (q ^ sw)] = p.h;
        dst[vox * S + ((CH + q) ^ sw)] = p.l;
      }
    }
  };
  frag wreg[ALDS ? 1 : 27];
  uint4* aw = ring + 4 * PLANE;
  if constexpr (ALDS) {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(a.wpack);
    for (int i = threadIdx.x; i < 27 * 64; i += 256) aw[i] = wsrc[i];
  } else {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(PL == 1 ? a.wpack : a.wpack32) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < 27; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  }
  uint4 pa[NLD][PL], pb[NLD][PL];
  load_plane(zb, pa);
  store_plane(zb, pa);
  load_plane(zb + 1, pa);
  store_plane(zb + 1, pa);
  if (zb + 1 < zend) load_plane(zb + 2, pa);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const bool lead = (g & 1) == 0;
  const int co = g * 4;                             // lead lanes own channels co .. co + 7
  // q-row 2w, column n: bf16 the lane's channel block g, fp32 its voxel (chunk g at the column's swizzle)
  const int lbase = PL == 1 ? (2 * wave * PW + n) * CH + g : (2 * wave * PW + n) * S;
  const int sw0 = Z::template zsw<S>(n), sw1 = Z::template zsw<S>(n + 1);
  float b8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b8[i] = a.bias[(co & 8) + i];
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * 16 * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.resid ? a.resid : a.out, a.resid ? nout : 0);
  const int qx = qx0 + n;
  constexpr int WOFF[8] = {0, 1, 3, 5, 9, 11, 15, 19};  // build_phases chunk offsets (Cin 32)

  auto step = [&](int qz, uint4 (*cur)[PL], uint4 (*nxt)[PL]) {
    if (qz + 2 < zend) load_plane(qz + 3, nxt);
    const uint4* p0 = ring + (qz & 3) * PLANE + lbase;
    const uint4* p1 = ring + ((qz + 1) & 3) * PLANE + lbase;
#pragma unroll
    for (int pd = 0; pd < 2; ++pd) {
      // this half's 8 skip records (k = (py, px, r)): bf16 requested before its MFMAs; fp32 (twice the registers, beside
      // 27 A pairs) after them
      // bf16: lead lanes own 8 channels (a 16-byte record, partner's 4 by a shuffle); fp32: every lane its own 4 channels
      // co .. co + 3 (16 bytes), no shuffle
      uint32_t off[8];
      uint4 rq[8];
      auto skip_load = [&]() {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int py = k >> 2, px = (k >> 1) & 1, r = k & 1;
          const int qy = qy0 + 2 * wave + r;
          const bool ok = (PL == 2 || lead) && qy < a.Hi && qx < a.Wi;
          const int oz = 2 * qz + pd, oy = 2 * qy + py, ox = 2 * qx + px;
          off[k] = ok ? (uint32_t)((((b * a.Do + oz) * a.Ho + oy) * a.Wo + ox) * 16 + (PL == 2 ? co : (co & 8))) * (uint32_t)ES
                      : kOOB;
          rq[k] = BufIO<bf16_t>::frag(rr, off[k]);
        }
      };
      if constexpr (PL == 1) skip_load();
      f32x4_t acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int py = 0; py < 2; ++py)
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const int ph = pd * 4 + py * 2 + px;
          const int na = pd ? 2 : 1, nb = py ? 2 : 1, nc = px ? 2 : 1;
#pragma unroll
          for (int ia = 0; ia < na; ++ia)
#pragma unroll
            for (int ib = 0; ib < nb; ++ib)
#pragma unroll
              for (int ic = 0; ic < nc; ++ic) {
                const int zo = pd ? (ia == 0 ? 1 : 0) : 0, yo = py ? (ib == 0 ? 1 : 0) : 0;
                const int xo = px ? (ic == 0 ? 1 : 0) : 0;
                const int s = WOFF[ph] + (ia * nb + ib) * nc + ic;
                frag w;
                if constexpr (ALDS) w = aw[s * 64 + (threadIdx.x & 63)];
                else w = wreg[s];
                const uint4* src = (zo ? p1 : p0) + (yo * PW + xo) * (PL == 1 ? CH : S);
#pragma unroll
                for (int r = 0; r < 2; ++r)
                  Z::mma(w, Z::bread(src + r * PW * (PL == 1 ? CH : S), PL == 1 ? 0 : g, CH, xo ? sw1 : sw0),
                         acc[(py * 2 + px) * 2 + r]);
              }
        }
      if constexpr (PL == 2) skip_load();
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (PL == 2) {
          const float4 f = __builtin_bit_cast(float4, rq[k]);
          const float sk[4] = {f.x, f.y, f.z, f.w};
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[k][i] * wsc + b8[(co & 4) + i];  // 2^-k: exact
            if (a.relu) v[i] = relu(v[i]);
            v[i] += sk[i];
          }
          am_fold<T, 4>(am, off[k] != kOOB, v);
          BufIO<T>::stq(ro, off[k], v);
          continue;
        }
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[k][i];
          v[4 + i] = __shfl_down(acc[k][i], 16);
        }
        if constexpr (PL == 1) {
          const uint32_t q4[4] = {rq[k].x, rq[k].y, rq[k].z, rq[k].w};
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            v[i] += b8[i];
            if (a.relu) v[i] = relu(v[i]);
            v[i] += __uint_as_float((i & 1) ? (q4[i >> 1] & 0xffff0000u) : (q4[i >> 1] << 16));
          }
        }
        if (lead) {
          am_fold<T, 8>(am, off[k] != kOOB, v);
          Vox8<T>::store(ro, off[k], v);
        }
      }
    }
    if (qz + 1 < zend) store_plane(qz + 2, cur);
    __syncthreads();
  };
  for (int qz = zb; qz < zend; qz += 2) {
    step(qz, pa, pb);
    if (qz + 1 < zend) step(qz + 1, pb, pa);
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + (threadIdx.x >> 6));
}

// conv1 (Conv3d k3 s2 p1, 8 -> 16 channels) streamed along z: output plane z reads input planes
// 2z-1 .. 2z+1, so a block keeps a 5-slot LDS ring of (2*8+1) x (2*16+1) x 8-channel input planes
// and fetches the next two planes while it computes the current output plane. K = 27 taps x 8
// channels in 7 chunks of 4 taps (lane group g = tap 4s + g; past tap 26 the weights are zero), the
// 7 A fragments in registers. bf16: same K order and weights as the gather kernel. fp32 (T = float): the split-f16
// form on the 32-K packing (ConvArgs::wpack32), each ring row stored as its even then its odd columns (a lane's
// stride-2 taps then read consecutive pixels: conflict-free with the hi / lo slot swizzle).
template <typename T>
__global__ __launch_bounds__(256) void conv_s2_c8_zslide_kernel(const ConvArgs a, int tiles_x, int tiles_y, int nzc,
                                                                int zc, int ntiles) {
  typedef ZForm<T> Z;
  typedef typename Z::frag frag;
  constexpr int PL = Z::PL, ES = sizeof(T);
  constexpr int QX = 16, QY = 8, PW = 2 * QX + 1, PH = 2 * QY + 1;
  constexpr int HCE = (PW + 1) / 2, PWE = PL == 1 ? PW : 2 * HCE;  // fp32: even / odd column halves of a row
  constexpr int NPIX = PH * PW;         // 8-channel pixels per halo plane
  constexpr int PLANE = PH * PWE * PL;  // 16-byte slots per ring plane
  constexpr int NLD = (NPIX + 255) / 256;
  // ring slots: bf16 5 (planes 2z - 1 .. 2z + 3: the next two planes stored after the MFMAs, one barrier per plane);
  // fp32 4 (74 KB instead of 92: two blocks per CU instead of one), plane 2z + 3 then goes into the slot of 2z - 1
  // behind a second barrier
  constexpr int NS = PL == 1 ? 5 : 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);

  const int bid = blockIdx.x, q8 = ntiles / 8, r8 = ntiles % 8, xcd = bid % 8;
  int tt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = tt % tiles_x; tt /= tiles_x;
  const int ty = tt % tiles_y; tt /= tiles_y;
  const int tz = tt % nzc;
  const int b = tt / nzc;
  const int ox0 = tx * QX, oy0 = ty * QY, zb = tz * zc;
  const int zend = min(zb + zc, a.Do);
  const int ix0 = 2 * ox0 - 1, iy0 = 2 * oy0 - 1;

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in, (long long)a.B * a.Di * a.Hi * a.Wi * 8 * ES);
  const Prescale ps = ps_in<T>(a, b);  // fp32: the input tensor's magnitude (damvs_device.h)
  const float wsc = ps_wscale<T>(a, ps);
  unsigned am = 0u;  // max |stored value| (fp32: the output's magnitude slot)
  auto load_plane = [&](int iz, uint4 (*v)[PL]) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      const int row = c / PW, col = c - row * PW;
      const int iy = iy0 + row, ix = ix0 + col;
      const bool ok = c < NPIX && (unsigned)iz < (unsigned)a.Di && (unsigned)iy < (unsigned)a.Hi &&
                      (unsigned)ix < (unsigned)a.Wi;
      const uint32_t off = (uint32_t)(((b * a.Di + iz) * a.Hi + iy) * a.Wi + ix) * (16u * PL);
#pragma unroll
      for (int h = 0; h < PL; ++h) v[i][h] = BufIO<bf16_t>::frag(rin, ok ? off + 16u * h : kOOB);
    }
  };
  auto store_plane = [&](int iz, const uint4 (*v)[PL]) {
    uint4* dst = ring + ((iz + NS) % NS) * PLANE;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c >= NPIX) continue;
      if constexpr (PL == 1) {
        dst[c] = v[i][0];
      } else {
        const int row = c / PW, col = c - row * PW, hp = col >> 1;
        const int p = row * PWE + (col & 1) * HCE + hp, sw = Z::template zsw<2>(hp);
        const F16Pair q = split8s(v[i][0], v[i][1], ps.s);
        dst[p * 2 + sw] = q.h;
        dst[p * 2 + (1 ^ sw)] = q.l;
      }
    }
  };
  frag wreg[7];
  {
    const uint4* __restrict__ wsrc = reinterpret_cast<const uint4*>(PL == 1 ? a.wpack : a.wpack32) + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < 7; ++s) wreg[s] = Z::wload(wsrc, s, 0);
  }
  {
    uint4 v[NLD][PL];
#pragma unroll
    for (int p = -1; p <= 1; ++p) {
      load_plane(2 * zb + p, v);
      store_plane(2 * zb + p, v);
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  // output row 2w (halo row 2*2w), column n: bf16 the pixel slot of tap (0, 0); fp32 the row's pixel base
  const int lbase = PL == 1 ? (2 * (2 * wave) * PW + 2 * n) : 2 * (2 * wave) * PWE;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = a.bias[g * 4 + i];
  const long long nout = (long long)a.B * a.Do * a.Ho * a.Wo * 16 * ES;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out, nout);
  const int ox = ox0 + n;

  for (int z = zb; z < zend; ++z) {
    const bool more = z + 1 < zend;
    uint4 na[NLD][PL], nb[NLD][PL];
    if (more) {
      load_plane(2 * z + 2, na);
      load_plane(2 * z + 3, nb);
    }
    const uint4* pl[3] = {ring + ((2 * z - 1 + NS) % NS) * PLANE, ring + ((2 * z) % NS) * PLANE,
                          ring + ((2 * z + 1) % NS) * PLANE};
    f32x4_t acc[2] = {(f32x4_t){0.f, 0.f, 0.f, 0.f}, (f32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int t0 = 4 * s;
      // (plane, in-plane pixel offset, dx) of tap t (past 26: a valid pixel, zero weight)
      auto tap = [&](int t) {
        const int tc = t < 27 ? t : 26;
        return (tc / 9) * 65536 + (((tc / 3) % 3) * (PL == 1 ? PW : PWE) + (PL == 1 ? tc % 3 : 0)) * 4 + tc % 3;
      };
      int code = tap(t0);
      code = g == 1 ? tap(t0 + 1) : code;
      code = g == 2 ? tap(t0 + 2) : code;
      code = g == 3 ? tap(t0 + 3) : code;
      const int dz = code >> 16, o = (code & 0xffff) >> 2, dx = code & 3;
      const uint4* pz = dz == 0 ? pl[0] : dz == 1 ? pl[1] : pl[2];
      if constexpr (PL == 1) {
        const uint4* src = pz + lbase + o;
#pragma unroll
        for (int r = 0; r < 2; ++r) Z::mma(wreg[s], src[r * 2 * PW], acc[r]);
      } else {
        // column 2n + dx: half (dx & 1), index n + (dx >> 1)
        const int hp = n + (dx >> 1), p = lbase + o + (dx & 1) * HCE + hp, sw = Z::template zsw<2>(hp);
#pragma unroll
        for (int r = 0; r < 2; ++r) Z::mma(wreg[s], Z::bread(pz + (p + r * 2 * PWE) * 2, 0, 1, sw), acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int oy = oy0 + 2 * wave + r;
      const bool ok = oy < a.Ho && ox < a.Wo;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (PL == 1 ? acc[r][i] : acc[r][i] * wsc) + bias[i];  // 2^-k: exact
        if (a.relu) v[i] = relu(v[i]);
      }
      am_fold<T, 4>(am, ok, v);
      BufIO<T>::stq(ro, ok ? (uint32_t)((((b * a.Do + z) * a.Ho + oy) * a.Wo + ox) * 16 + g * 4) * (uint32_t)ES : kOOB, v);
    }
    if (more) {  // NS 5: slots of planes 2z - 3 and 2z - 2, last read before the previous barrier
      store_plane(2 * z + 2, na);
      if (NS == 4) __syncthreads();  // plane 2z + 3 goes where 2z - 1 was, read by this step's MFMAs
      store_plane(2 * z + 3, nb);
    }
    __syncthreads();
  }
  am_flush<T>(a, am, b, blockIdx.x * 4 + wave);
}

bool deconv_zslide_disabled() {  // read per call: tests flip it between launches
  const char* v = getenv("DAMVS_DECONV_NO_ZSLIDE");
  return v && v[0] == '1';
}

template <typename T>
hipError_t launch_t(hipStream_t s, const ConvArgs& a) {
  long long Qtot = (long long)a.B * a.Dq * a.Hq * a.Wq;
  long long per_block = 4LL * kGroups * 16;
  const int nq = (int)((Qtot + per_block - 1) / per_block);
  dim3 grid((unsigned)(nq * a.nphase));
  if ((sizeof(T) == 2 || a.wpack32) && a.xpair && a.Cin == 16 && a.Cout == 8 && a.nphase == 4 &&
      !deconv_zslide_disabled()) {
    constexpr int zc = 8;
    const int tx = (a.Wi + 15) / 16, ty = (a.Hi + 7) / 8, nzc = (a.Di + zc - 1) / zc;
    const long long nt = (long long)tx * ty * nzc * a.B;
    const size_t smem = 4 * 9 * 17 * 2 * 16 * ZForm<T>::PL + (sizeof(T) == 4 ? 9 * 128 * 16 : 0);
    ConvArgs az = a;
    if (sizeof(T) == 4) az.wpack = a.wpack32;  // fp32: the blocked 32-K split packing of the x-pair phases
    hipLaunchKernelGGL(deconv_xpair_zslide_kernel<T>, dim3((unsigned)nt), dim3(256), smem, s, az, tx, ty, nzc, zc, (int)nt);
    return hipGetLastError();
  }
  if ((sizeof(T) == 2 || a.wpack32) && a.nphase == 1 && a.in_stride == 2 && a.Cin == 8 && a.Cout == 16 && a.MT == 1 &&
      !a.resid && a.ph[0].ntaps == 27 && !deconv_zslide_disabled()) {
    constexpr int zc = 8;
    const int tx = (a.Wo + 15) / 16, ty = (a.Ho + 7) / 8, nzc = (a.Do + zc - 1) / zc;
    const long long nt = (long long)tx * ty * nzc * a.B;
    const size_t smem = sizeof(T) == 2 ? 5 * 17 * 33 * 16 : 4 * 17 * 34 * 32;  // ring slots (NS) x plane
    auto k = conv_s2_c8_zslide_kernel<T>;
    if (smem > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(256), smem, s, a, tx, ty, nzc, zc, (int)nt);
    return hipGetLastError();
  }
  if ((sizeof(T) == 2 || a.wpack32) && !a.xpair && a.nphase == 8 && a.Cin == 32 && a.Cout == 16 && a.MT == 1 &&
      !deconv_zslide_disabled()) {
    constexpr int zc = 8;
    const int tx = (a.Wi + 15) / 16, ty = (a.Hi + 7) / 8, nzc = (a.Di + zc - 1) / zc;
    const long long nt = (long long)tx * ty * nzc * a.B;
    const size_t ring = 4 * 9 * 17 * 4 * 16 * ZForm<T>::PL;
    if constexpr (sizeof(T) == 2) {
      // the A fragments in LDS (27 KB) instead of 108 VGPRs: two waves per SIMD instead of one, U-Net 1.136-1.149 /
      // 2.071-2.102 / 1.879-1.884 -> 1.128-1.129 / 2.020-2.024 / 1.826-1.837 ms (profiles/r03/ab_conv9.jsonl)
      hipLaunchKernelGGL((deconv_c16_zslide_kernel<T, true>), dim3((unsigned)nt), dim3(256), ring + 27 * 64 * 16, s, a,
                         tx, ty, nzc, zc, (int)nt);
    } else {
      auto k = deconv_c16_zslide_kernel<T, false>;
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)ring);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k, dim3((unsigned)nt), dim3(256), ring, s, a, tx, ty, nzc, zc, (int)nt);
    }
    return hipGetLastError();
  }
  if (sizeof(T) == 4 && a.B > 1 && (a.in_amax || a.out_amax) && a.Dq * a.Hq * a.Wq < kGroups * 16) {
    // the gather kernel's waves straddle at most two batch elements (per-voxel prescales); a q-grid of fewer voxels
    // than a wave runs one batch element per launch
    const long long in_b = (long long)a.Di * a.Hi * a.Wi * a.Cin * 4, out_b = (long long)a.Do * a.Ho * a.Wo * a.Cout * 4;
    for (int b = 0; b < a.B; ++b) {
      ConvArgs a1 = a;
      a1.B = 1;
      a1.in = static_cast<const char*>(a.in) + b * in_b;
      a1.out = static_cast<char*>(a.out) + b * out_b;
      a1.resid = a.resid ? static_cast<const char*>(a.resid) + b * out_b : nullptr;
      a1.in_amax = a.in_amax ? a.in_amax + (size_t)b * kAmaxSlotWords : nullptr;
      a1.out_amax = a.out_amax ? a.out_amax + (size_t)b * kAmaxSlotWords : nullptr;
      const hipError_t e = launch_t<T>(s, a1);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (a.xpair) {
    if (a.MT != 1 || a.Cout != 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv3d_mfma_kernel<T, 1, true>), grid, dim3(256), 0, s, a, nq);
    return hipGetLastError();
  }
  if constexpr (sizeof(T) == 4) {
    // fp32: the 32-K split form where the layer has its packing (DAMVS_CONV3D_K16=1, read per call: the 16-K form)
    const char* kv = getenv("DAMVS_CONV3D_K16");
    if (a.wgat32 && !(kv && kv[0] == '1')) {
      ConvArgs a2 = a;
      for (int p = 0; p < a.nphase; ++p) {  // the phases of the 32-K packing (LayerPlan, build_phases(., 32))
        a2.ph[p].kchunks = a.k32_chunks[p];
        a2.ph[p].w_off = a.k32_off[p];
      }
      switch (a.MT) {
        case 1: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 1, false, true>), grid, dim3(256), 0, s, a2, nq); break;
        case 2: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 2, false, true>), grid, dim3(256), 0, s, a2, nq); break;
        case 4: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 4, false, true>), grid, dim3(256), 0, s, a2, nq); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  switch (a.MT) {
    case 1: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 1, false>), grid, dim3(256), 0, s, a, nq); break;
    case 2: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 2, false>), grid, dim3(256), 0, s, a, nq); break;
    case 4: hipLaunchKernelGGL((conv3d_mfma_kernel<T, 4, false>), grid, dim3(256), 0, s, a, nq); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_conv3d(hipStream_t s, int store, const ConvArgs& a0) {
  ConvArgs a = a0;
  a.div_wq = make_fastdiv(a.Wq);
  a.div_hq = make_fastdiv(a.Hq);
  a.div_dq = make_fastdiv(a.Dq);
  // 32-bit device offsets: operands of 2 GiB or more run one batch element per launch
  const long long es = store == ST_BF16 ? 2 : 4;
  const long long in_b = (long long)a.Di * a.Hi * a.Wi * a.Cin * es, out_b = (long long)a.Do * a.Ho * a.Wo * a.Cout * es;
  if (a.B > 1 && (in_b * a.B >= (1LL << 31) || out_b * a.B >= (1LL << 31))) {
    for (int b = 0; b < a.B; ++b) {
      ConvArgs a1 = a0;
      a1.B = 1;
      a1.in = static_cast<const char*>(a0.in) + b * in_b;
      a1.out = static_cast<char*>(a0.out) + b * out_b;
      a1.resid = a0.resid ? static_cast<const char*>(a0.resid) + b * out_b : nullptr;
      a1.in_amax = a0.in_amax ? a0.in_amax + (size_t)b * kAmaxSlotWords : nullptr;  // per-sample magnitude slots
      a1.out_amax = a0.out_amax ? a0.out_amax + (size_t)b * kAmaxSlotWords : nullptr;
      const hipError_t e = launch_conv3d(s, store, a1);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (in_b >= (1LL << 31) || out_b >= (1LL << 31)) return hipErrorInvalidValue;
  if (!conv_lds_disabled()) {
    hipError_t e = store == ST_BF16 ? launch_lds<bf16_t>(s, a) : launch_lds<float>(s, a);
    if (e != hipErrorNotSupported) return e;
  }
  return store == ST_BF16 ? launch_t<bf16_t>(s, a) : launch_t<float>(s, a);
}

// The x-pair conv11 runs by default; DAMVS_CONV_XPAIR=0 selects the 8-phase form (A/B and diagnosis).
bool conv_xpair_disabled() {
  static const bool off = [] {
    const char* v = getenv("DAMVS_CONV_XPAIR");
    return v && v[0] == '0';
  }();
  return off;
}

bool conv_lds_disabled() {
  static const bool off = [] {
    const char* v = getenv("DAMVS_CONV_NO_LDS");
    return v && v[0] == '1';
  }();
  return off;
}

}  // namespace damvs
