// Device-side helpers: storage conversion and 16-byte vector access for NHWC / NDHWC data.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "damvs_internal.h"

namespace damvs {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__device__ __forceinline__ float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// ---------------------------------------------------------------- fp32 convolutions as split-f16 MFMAs
// The fp32 path stores fp32 and computes every conv product on f16 matrix cores: x = xh + xl with xh = f16(x) and
// xl = f16(x - xh) (round to nearest even, subnormals kept; x - xh is exact), and
//   w * x ~ wl*xh + wh*xl + wh*xh          (three v_mfma_f32_16x16x16_f16, fp32 accumulation)
// leaving out only wl*xl (~2^-22 relative) and the pieces' own rounding (~2^-22): per product ~2^-21, inside the
// fp32 FMA chain's accumulation error over the K of these layers. Measured against float64 (tools/mfma_f16,
// profiles/r04/mfma_f16.json): max error / sum|w x| 2.7e-7 / 3.8e-7 / 5.7e-7 at K = 64 / 288 / 864 against the exact
// fp32 MFMA's 2.4e-7 / 4.8e-7 / 7.7e-7; subnormal pieces pass through the MFMA exactly. The cascade-level model
// (tools/split_precision_model.py: every conv of the oracle forward emulated this way) keeps the end-to-end
// fp32-vs-fp64 statistics at 0.86-1.36x the reference's own. Rate: three 16-cycle MFMAs per 16 K instead of four
// 32-cycle exact-fp32 ones (v_mfma_f32_16x16x16_f16 runs at half the FLOP rate of 16x16x32 but keeps the fp32
// kernels' 4-channel K fragments). Weights are split on the host, scaled by 2^k per layer so the largest |w| lies in
// (2^13, 2^14] (normal-range lo pieces); the epilogues multiply by wscale = 2^-k. A 16-byte fragment holds
// [hi0..hi3 | lo0..lo3]. |x| must stay below 65504 (f16 range): larger activations turn into inf / NaN outputs.
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 split_f16(const float4& x) {
  const f16x4_t h = {(_Float16)x.x, (_Float16)x.y, (_Float16)x.z, (_Float16)x.w};
  const f16x4_t l = {(_Float16)(x.x - (float)h[0]), (_Float16)(x.y - (float)h[1]), (_Float16)(x.z - (float)h[2]),
                     (_Float16)(x.w - (float)h[3])};
  const f32x2v_t hv = __builtin_bit_cast(f32x2v_t, h), lv = __builtin_bit_cast(f32x2v_t, l);
  return make_float4(hv[0], hv[1], lv[0], lv[1]);
}
// acc += A (pre-split weights w) * B (pre-split activations xs), one 16 x 16 x 16 K step
__device__ __forceinline__ void mma_split16(const float4& w, const float4& xs, f32x4_t& acc) {
  const f16x4_t wh = __builtin_bit_cast(f16x4_t, (f32x2v_t){w.x, w.y}), wl = __builtin_bit_cast(f16x4_t, (f32x2v_t){w.z, w.w});
  const f16x4_t xh = __builtin_bit_cast(f16x4_t, (f32x2v_t){xs.x, xs.y}), xl = __builtin_bit_cast(f16x4_t, (f32x2v_t){xs.z, xs.w});
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(wl, xh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(wh, xl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(wh, xh, acc, 0, 0, 0);
}

// The same split on the full-rate v_mfma_f32_16x16x32_f16 (8 channels per lane and K fragment, the bf16 kernels'
// fragment shape): hi and lo halves of 8 values, 16 bytes each. Kernels that keep their fragments in LDS or
// registers for many MFMAs (conv2d_wide_kernel<float>) use this form; the weights are packed as [hi8 | lo8].
struct F16Pair {
  uint4 h, l;
};
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ F16Pair split8(const float* v) {
  f16x8_t h, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = (_Float16)v[i];
    l[i] = (_Float16)(v[i] - (float)h[i]);
  }
  return F16Pair{__builtin_bit_cast(uint4, h), __builtin_bit_cast(uint4, l)};
}
__device__ __forceinline__ F16Pair split8(const float4& a, const float4& b) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return split8(v);
}
__device__ __forceinline__ void mma_split32(const F16Pair& w, const F16Pair& x, f32x4_t& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, w.l), __builtin_bit_cast(f16x8_t, x.h), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, w.h), __builtin_bit_cast(f16x8_t, x.l), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, w.h), __builtin_bit_cast(f16x8_t, x.h), acc, 0, 0, 0);
}

// ---------------------------------------------------------------- activation prescale (fp32 path, round 6)
// The split pieces are f16: unscaled, |x| >= 65520 overflows the hi piece and |x| < 2^-3 leaves the lo piece subnormal
// (absolute floor 2^-25). Every activation tensor of the stage (cost volume, U-Net levels) therefore carries its
// magnitude: each producer records max |y| of what it stores (per wave, one vector atomic max of the float's bit pattern
// -- non-negative floats order as unsigned integers, NaN above inf -- into one of kAmaxReps replicas of the tensor's
// slot), and each consumer reads the slot at its start and splits x * 2^k instead of x, with k chosen so that the
// tensor's maximum lands in [2^13, 2^14): both pieces are then normal f16 for every value down to max * 2^-17. Its
// epilogue multiplies the accumulator by wscale * 2^-k. Power-of-two scaling is exact, and f16 / fp32 rounding of
// normal numbers is scale-invariant, so wherever the unscaled pieces were both normal the result is bitwise the same;
// elsewhere it is the exact fp32 product the unscaled split could not represent. Slots are zeroed per stage forward.

struct Prescale {
  float s, inv;  // x * s is split; the accumulator is scaled back by inv (= 1 / s)
};
__device__ __forceinline__ Prescale prescale_from_max(unsigned m);
// max of a slot's replicas (every lane of the wave must be active: each of the first kAmaxReps lanes loads one)
__device__ __forceinline__ Prescale prescale_of(const unsigned* __restrict__ amax) {
  if (!amax) return Prescale{1.f, 1.f};
  const int lane = threadIdx.x & 63;
  unsigned m = lane < kAmaxReps ? __hip_atomic_load(amax + lane * kAmaxStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
  for (int o = 32; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  return prescale_from_max(__builtin_amdgcn_readfirstlane(m));
}
// the scale of a tensor whose max |x| has the bit pattern m (uniform)
__device__ __forceinline__ Prescale prescale_from_max(unsigned m) {
  if (m == 0u) return Prescale{1.f, 1.f};  // an all-zero tensor
  int e = (int)((m >> 23) & 0xff) - 127;  // floor(log2(max)); subnormal maxima count as 2^-127, NaN / inf as 2^128
  int k = 13 - (e < -127 ? -127 : e);
  k = k < -100 ? -100 : k > 100 ? 100 : k;  // s and 1 / s stay normal fp32, with the weights' 2^-k too
  return Prescale{__uint_as_float((unsigned)(127 + k) << 23), __uint_as_float((unsigned)(127 - k) << 23)};
}
// |v| folded into a running maximum (bit patterns; NaN propagates)
__device__ __forceinline__ unsigned amax_fold(unsigned m, float v) { return max(m, __float_as_uint(v) & 0x7fffffffu); }
// one wave's maximum into replica r of the slot (every lane of the wave must be active)
__device__ __forceinline__ void amax_flush(unsigned m, unsigned* __restrict__ amax, int r) {
  if (!amax) return;
#pragma unroll
  for (int o = 32; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0 && m != 0u) atomicMax(amax + (r & (kAmaxReps - 1)) * kAmaxStride, m);
}

__device__ __forceinline__ float4 scale4(const float4& x, float s) { return make_float4(x.x * s, x.y * s, x.z * s, x.w * s); }
// split8 of (a, b) * s
__device__ __forceinline__ F16Pair split8s(const float4& a, const float4& b, float s) {
  return split8(scale4(a, s), scale4(b, s));
}
__device__ __forceinline__ F16Pair split8s(const uint4& a, const uint4& b, float s) {
  return split8s(__builtin_bit_cast(float4, a), __builtin_bit_cast(float4, b), s);
}

// MFMA K-fragment traits shared by the conv kernels. raw: one lane's 16-byte K fragment (A or B).
//   mma(w, x, acc):     x as loaded from the activation tensor (fp32: split here, per use)
//   stage(x):           the form an LDS tile keeps (fp32: split once when the tile is filled)
//   mma_staged(w, s, acc): x from such a tile
template <typename T> struct MmaFrag;
template <> struct MmaFrag<float> {
  typedef float4 raw;
  __device__ __forceinline__ static raw stage(const raw& x) { return split_f16(x); }
  __device__ __forceinline__ static void mma_staged(const raw& w, const raw& xs, f32x4_t& acc) { mma_split16(w, xs, acc); }
  __device__ __forceinline__ static void mma(const raw& w, const raw& x, f32x4_t& acc) { mma_split16(w, split_f16(x), acc); }
  __device__ __forceinline__ static raw zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <> struct MmaFrag<bf16_t> {
  typedef uint4 raw;
  __device__ __forceinline__ static raw stage(const raw& x) { return x; }
  __device__ __forceinline__ static void mma(const raw& w, const raw& x, f32x4_t& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, w), __builtin_bit_cast(bf16x8_t, x),
                                                  acc, 0, 0, 0);
  }
  __device__ __forceinline__ static void mma_staged(const raw& w, const raw& x, f32x4_t& acc) { mma(w, x, acc); }
  __device__ __forceinline__ static raw zero() { return make_uint4(0u, 0u, 0u, 0u); }
};

// Storage forms of the z-streamed kernels' LDS rings. bf16: a voxel of CH 8-channel chunks is CH 16-byte slots, chunk c
// in slot c. fp32 (the split-f16 form, damvs_device.h mma_split32): 2 CH slots, the hi / lo halves of chunk c in slots
// c and CH + c, XOR-swizzled by the voxel's column (zsw) so that 16 lanes reading one chunk of 16 consecutive voxels
// (one MFMA B fragment) hit distinct bank groups; rows and planes shift by whole voxels and keep the swizzle.
template <typename T> struct ZForm;
template <> struct ZForm<bf16_t> {
  typedef uint4 frag;
  static constexpr int PL = 1;  // 16-byte slots (and HBM loads) per 8-channel chunk
  template <int S> __device__ __forceinline__ static int zsw(int) { return 0; }
  __device__ __forceinline__ static void mma(const frag& w, const frag& x, f32x4_t& acc) { MmaFrag<bf16_t>::mma(w, x, acc); }
  // A fragment s of a [chunk][lane] packing
  __device__ __forceinline__ static frag wload(const uint4* __restrict__ w, int s, int lane) { return w[(size_t)s * 64 + lane]; }
  // B fragment of chunk c of the voxel at ring slot base vs (column swizzle sw)
  __device__ __forceinline__ static frag bread(const uint4* p, int c, int CH, int sw) { (void)CH; (void)sw; return p[c]; }
};
template <> struct ZForm<float> {
  typedef F16Pair frag;
  static constexpr int PL = 2;
  template <int S> __device__ __forceinline__ static int zsw(int col) { return (col / (16 / S)) % S; }
  __device__ __forceinline__ static void mma(const frag& w, const frag& x, f32x4_t& acc) { mma_split32(w, x, acc); }
  // [chunk][hi: 64 lanes][lo: 64 lanes] (split_weights_blocked)
  __device__ __forceinline__ static frag wload(const uint4* __restrict__ w, int s, int lane) {
    return F16Pair{w[(size_t)s * 128 + lane], w[(size_t)s * 128 + 64 + lane]};
  }
  __device__ __forceinline__ static frag bread(const uint4* p, int c, int CH, int sw) {
    return F16Pair{p[c ^ sw], p[(CH + c) ^ sw]};
  }
};

// Storage traits: E = elements per 16-byte chunk.
template <typename T> struct Stor;
template <> struct Stor<float> {
  static constexpr int E = 4;
  __device__ __forceinline__ static void load16(const float* p, float* v) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void store16(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Stor<bf16_t> {
  static constexpr int E = 8;
  __device__ __forceinline__ static float to_f(bf16_t v) { return __uint_as_float((uint32_t)v << 16); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
  __device__ __forceinline__ static void load16(const bf16_t* p, float* v) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store16(bf16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf2f(*p); }
};

// Load / store C contiguous channels (C a multiple of Stor<T>::E).
template <typename T, int C>
__device__ __forceinline__ void load_vec(const T* p, float* v) {
#pragma unroll
  for (int i = 0; i < C; i += Stor<T>::E) Stor<T>::load16(p + i, v + i);
}
template <typename T, int C>
__device__ __forceinline__ void store_vec(T* p, const float* v) {
#pragma unroll
  for (int i = 0; i < C; i += Stor<T>::E) Stor<T>::store16(p + i, v + i);
}

// Occupancy cap: amdgpu_waves_per_eu(n) bounds the register allocation (VGPRs + AGPRs) so n waves fit per SIMD.
// Used where a kernel's natural allocation sits just above a wave boundary (e.g. 132 + 64 AGPRs -> 160 VGPRs, no
// spill: 2 -> 3 waves). n = 1 leaves the allocation free. -DDAMVS_NO_OCC builds drop every cap (A/B).
#ifdef DAMVS_NO_OCC
#define DAMVS_WAVES(n)
#else
#define DAMVS_WAVES(n) __attribute__((amdgpu_waves_per_eu(n)))
#endif

// ReLU with torch.relu's NaN semantics (NaN stays NaN; fmaxf(NaN, 0) would give 0 under IEEE maxNum). A NaN from an
// out-of-range split-f16 product (|x| >= 65520, the fp32 path) thus reaches the stage outputs, where the range check
// of damvs_stage_forward reports it (damvs_stage_status) instead of a finite wrong depth.
__device__ __forceinline__ float relu(float x) { return x < 0.f ? 0.f : x; }

// For kernel-local lambdas with large bodies used at two or more call sites: hipcc may otherwise emit them as
// functions, the by-reference closure then lives in scratch and LDS pointers reaching them turn generic (flat
// stores). conv2d_wide_kernel<float> at input stride 2 had exactly that (512 B of scratch, flat halo stores:
// 5-7x the bf16 kernel's time instead of ~3x).
#define DAMVS_INLINE __attribute__((always_inline))

// compile-time bool for generic-lambda specialisation (step(BoolC<true>(), ...): decltype(arg)::value)
template <bool B> struct BoolC {
  static constexpr bool value = B;
};
template <int I> struct IntC {
  static constexpr int value = I;
};

typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32_t __attribute__((ext_vector_type(2)));

// Buffer loads/stores: 32-bit byte offsets against a descriptor whose range check returns 0 for an
// offset past the end (and drops such a store), so padding taps and tail pixels need no branch.
constexpr uint32_t kOOB = 0x80000000u;  // every operand is < 2 GiB (checked by the launcher)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <typename T> struct BufIO;
template <> struct BufIO<float> {
  typedef float4 raw;   // one MFMA K fragment (4 channels x 4 K-steps)
  typedef float4 quad;  // 4 output channels
  __device__ __forceinline__ static raw frag(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  }
  __device__ __forceinline__ static raw merge(const raw& x, const raw& y) {
    return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
  __device__ __forceinline__ static quad ldq(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  }
  __device__ __forceinline__ static quad ldq_dev(__amdgpu_buffer_rsrc_t r, uint32_t off) {  // device scope (sc1)
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
  }
  __device__ __forceinline__ static void addq(const quad& q, float* v) { v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w; }
  __device__ __forceinline__ static void stq(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, make_float4(v[0], v[1], v[2], v[3])), r, off, 0, 0);
  }
};
template <> struct BufIO<bf16_t> {
  typedef uint4 raw;
  typedef uint2 quad;
  __device__ __forceinline__ static raw frag(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  }
  __device__ __forceinline__ static raw merge(const raw& x, const raw& y) {
    return make_uint4(x.x | y.x, x.y | y.y, x.z | y.z, x.w | y.w);
  }
  __device__ __forceinline__ static quad ldq(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  }
  __device__ __forceinline__ static quad ldq_dev(__amdgpu_buffer_rsrc_t r, uint32_t off) {  // device scope (sc1)
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16));
  }
  __device__ __forceinline__ static void addq(const quad& q, float* v) {
    v[0] += __uint_as_float(q.x << 16); v[1] += __uint_as_float(q.x & 0xffff0000u);
    v[2] += __uint_as_float(q.y << 16); v[3] += __uint_as_float(q.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void stq(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* v) {
    const uint2 w = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                               (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, w), r, off, 0, 0);
  }
};

// One whole 8-channel voxel / pixel record (16 B bf16 / 32 B f32): load into floats / store from floats.
template <typename T> struct Vox8;
template <> struct Vox8<bf16_t> {
  __device__ __forceinline__ static void add(__amdgpu_buffer_rsrc_t r, uint32_t off, float* v) {
    const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] += __uint_as_float(w[i] << 16);
      v[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, make_uint4(w[0], w[1], w[2], w[3])), r, off, 0, 0);
  }
};
template <> struct Vox8<float> {
  __device__ __forceinline__ static void add(__amdgpu_buffer_rsrc_t r, uint32_t off, float* v) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 q = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * h, 0, 0));
      v[4 * h] += q.x; v[4 * h + 1] += q.y; v[4 * h + 2] += q.z; v[4 * h + 3] += q.w;
    }
  }
  __device__ __forceinline__ static void store(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* v) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(v4u32_t, make_float4(v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3])), r, off + 16 * h, 0, 0);
  }
};

// Stage N 16-byte chunks into LDS with a 256-thread block: chunk c = threadIdx.x + 256 i comes from
// load(c). Loads are issued BATCH at a time before their ds_writes, so each lane keeps BATCH HBM
// reads in flight (a plain strided `lds[c] = load(c)` loop waits for every load before its write:
// one read in flight per lane). Past-the-end chunks re-load chunk N - 1 and are not written.
// `post` maps a loaded chunk to the form the tile keeps (MmaFrag<T>::stage), applied at the ds_write so that the
// batch's loads are all in flight first.
struct StageIdentity {
  template <typename Raw> __device__ __forceinline__ Raw operator()(const Raw& r) const { return r; }
};
template <int N, int BATCH, typename Raw, typename F, typename P = StageIdentity>
__device__ __forceinline__ void stage_chunks(Raw* lds, F&& load, P post = P()) {
  constexpr int PER = (N + 255) / 256;
#pragma unroll
  for (int i0 = 0; i0 < PER; i0 += BATCH) {
    Raw r[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int c = threadIdx.x + (i0 + i) * 256;
      if (i0 + i < PER) r[i] = load(c < N ? c : N - 1);
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int c = threadIdx.x + (i0 + i) * 256;
      if (i0 + i < PER && c < N) lds[c] = post(r[i]);
    }
  }
}


// Diagnostic builds only (-DDAMVS_DIAG, tools/build_variant.sh; never the product library): a per-translation-unit
// record buffer that kernels append to (vector atomics on global memory) and damvs_diag_take_<unit>() reads and
// clears from the host. A record is 8 words: kind, block, index, observed bits, expected bits, HW_ID, LDS_ALLOC,
// XCC_ID (the last three from s_getreg: the CU / SIMD / wave slot, the LDS allocation the hardware gave the workgroup
// and the XCD it runs on).
#ifdef DAMVS_DIAG
constexpr int kDiagRecords = 64;
static __device__ unsigned g_diag[8 + 8 * kDiagRecords];
__device__ __forceinline__ void diag_record(unsigned kind, unsigned idx, unsigned seen, unsigned want) {
  const unsigned slot = atomicAdd(&g_diag[0], 1u);
  if (slot >= (unsigned)kDiagRecords) return;
  unsigned* r = g_diag + 8 + 8 * slot;
  r[0] = kind;
  r[1] = blockIdx.x;
  r[2] = idx;
  r[3] = seen;
  r[4] = want;
  r[5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
  r[6] = __builtin_amdgcn_s_getreg((31 << 11) | 6);   // LDS_ALLOC
  r[7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
}
#define DAMVS_DIAG_EXPORT(unit)                                                              \
  extern "C" int damvs_diag_take_##unit(unsigned* host, int nwords) {                        \
    const size_t n = (size_t)(nwords < (int)(sizeof(damvs::g_diag) / 4) ? nwords : sizeof(damvs::g_diag) / 4); \
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(damvs::g_diag), n * 4, 0, hipMemcpyDeviceToHost) != hipSuccess) \
      return -4;                                                                             \
    static const unsigned zero[8 + 8 * damvs::kDiagRecords] = {0};                                   \
    return hipMemcpyToSymbol(HIP_SYMBOL(damvs::g_diag), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess \
               ? 0 : -4;                                                                     \
  }
#endif

}  // namespace damvs
