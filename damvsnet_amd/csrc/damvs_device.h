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
template <int N, int BATCH, typename Raw, typename F>
__device__ __forceinline__ void stage_chunks(Raw* lds, F&& load) {
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
      if (i0 + i < PER && c < N) lds[c] = r[i];
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
