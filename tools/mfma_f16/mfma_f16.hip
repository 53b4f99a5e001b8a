// Split-fp16 MFMA probe (gfx950): issue rate of the f16 / bf16 / f32 16x16 MFMA forms, and the numerics of
// x*w = xh*wh + xh*wl + xl*wh with f16 pieces (subnormal lo pieces included) against a float64 reference.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_f16 mfma_f16.hip && ./mfma_f16
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int kIters = 4096;

// 4 independent accumulators, kIters x 4 MFMAs per wave; out keeps the compiler honest
template <int KIND>
__global__ __launch_bounds__(256) void rate_kernel(float* out, float seed) {
  f4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = (f4){seed, 0.f, 0.f, 0.f};
  const float s = seed * (threadIdx.x + 1);
  h4 a4 = (h4){(_Float16)s, (_Float16)1.f, (_Float16)2.f, (_Float16)3.f};
  h8 a8 = (h8){(_Float16)s, (_Float16)1.f, (_Float16)2.f, (_Float16)3.f, (_Float16)s, (_Float16)1.f, (_Float16)2.f,
               (_Float16)3.f};
  b8 bb = (b8){(__bf16)s, (__bf16)1.f, (__bf16)2.f, (__bf16)3.f, (__bf16)s, (__bf16)1.f, (__bf16)2.f, (__bf16)3.f};
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, acc[i], 0, 0, 0);
      if constexpr (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, acc[i], 0, 0, 0);
      if constexpr (KIND == 2) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb, bb, acc[i], 0, 0, 0);
      if constexpr (KIND == 3) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(s, s, acc[i], 0, 0, 0);
    }
  }
  float r = 0.f;
  for (int i = 0; i < 4; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__device__ __forceinline__ void split(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// One 16x16 output tile, C[m][n] = sum_k A[m][k] B[k][n], K a multiple of 16, with 16x16x16 f16 MFMAs on split
// pieces: lane l holds A[l&15][4(l>>4)+j], B[4(l>>4)+j][l&15].
__global__ void gemm_split(const float* A, const float* B, float* C, int K, int terms) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16) {
    h4 ah, al, bh, bl;
    for (int j = 0; j < 4; ++j) {
      _Float16 h, lo;
      split(A[r * K + k0 + 4 * g + j], h, lo);
      ah[j] = h; al[j] = lo;
      split(B[(k0 + 4 * g + j) * 16 + r], h, lo);
      bh[j] = h; bl[j] = lo;
    }
    if (terms >= 3) acc = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, acc, 0, 0, 0);
    if (terms >= 2) acc = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];
}

// the same product with 16x16x32 f16 MFMAs (lane l holds A[l&15][8(l>>4)+j])
__global__ void gemm_split32(const float* A, const float* B, float* C, int K) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32) {
    h8 ah, al, bh, bl;
    for (int j = 0; j < 8; ++j) {
      _Float16 h, lo;
      split(A[r * K + k0 + 8 * g + j], h, lo);
      ah[j] = h; al[j] = lo;
      split(B[(k0 + 8 * g + j) * 16 + r], h, lo);
      bh[j] = h; bl[j] = lo;
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];
}

// exact f32 MFMA, the reference kernels' fp32 path
__global__ void gemm_f32(const float* A, const float* B, float* C, int K) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[r * K + k0 + g], B[(k0 + g) * 16 + r], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];
}

// a subnormal f16 operand through the MFMA: 2^-20 * 1 (and 2^-24, the smallest)
__global__ void denorm_probe(float* out) {
  const int l = threadIdx.x;
  h4 a = (h4){(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
  h4 b = a;
  if ((l >> 4) == 0) {
    a[0] = (_Float16)ldexpf(1.f, -20);
    a[1] = (_Float16)ldexpf(1.f, -24);
    b[0] = (_Float16)1.f;
    b[1] = (_Float16)1.f;
  }
  f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, acc, 0, 0, 0);
  if (l == 0) {
    out[0] = acc[0];
    out[1] = ldexpf(1.f, -20) + ldexpf(1.f, -24);
  }
  _Float16 h, lo;
  split(1.f + ldexpf(1.f, -20), h, lo);  // lo = 2^-20 is subnormal in f16
  if (l == 0) {
    out[2] = (float)lo;
    out[3] = ldexpf(1.f, -20);
  }
}

int main() {
  float* dout;
  const int blocks = 256 * 8;
  CHECK(hipMalloc(&dout, blocks * 256 * sizeof(float)));
  const char* names[4] = {"v_mfma_f32_16x16x16_f16", "v_mfma_f32_16x16x32_f16", "v_mfma_f32_16x16x32_bf16",
                          "v_mfma_f32_16x16x4_f32"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int kind = 0; kind < 4; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      CHECK(hipEventRecord(e0));
      if (kind == 0) rate_kernel<0><<<blocks, 256>>>(dout, 1e-3f);
      if (kind == 1) rate_kernel<1><<<blocks, 256>>>(dout, 1e-3f);
      if (kind == 2) rate_kernel<2><<<blocks, 256>>>(dout, 1e-3f);
      if (kind == 3) rate_kernel<3><<<blocks, 256>>>(dout, 1e-3f);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double n = (double)blocks * 4 * kIters * 4;  // wave-MFMAs
      const int kk[4] = {16, 32, 32, 4};
      const double flop = n * 2.0 * 16 * 16 * kk[kind];
      // cycles per MFMA per SIMD at an assumed 2.4 GHz: (time * 2.4e9 * 1024 SIMDs) / wave-MFMAs
      if (rep) printf("{\"instr\": \"%s\", \"ms\": %.3f, \"TFLOP/s\": %.1f, \"cyc_per_mfma_at_2.4GHz\": %.2f}\n", names[kind], ms,
                      flop / ms / 1e9, ms * 1e-3 * 2.4e9 * 1024 / n);
    }
  }

  // numerics
  for (int K : {64, 288, 864}) {
    std::vector<float> A(16 * K), B(K * 16), C(256), C2(256), C3(256), Cf(256);
    srand(K);
    for (auto& v : A) v = (rand() / (float)RAND_MAX - 0.3f) * 0.2f;   // BN-folded-weight-like
    for (auto& v : B) v = (rand() / (float)RAND_MAX) * ((rand() & 7) ? 1.f : 0.01f);  // post-ReLU-like, some small
    float *dA, *dB, *dC;
    CHECK(hipMalloc(&dA, A.size() * 4));
    CHECK(hipMalloc(&dB, B.size() * 4));
    CHECK(hipMalloc(&dC, 256 * 4));
    CHECK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    gemm_split<<<1, 64>>>(dA, dB, dC, K, 3);
    CHECK(hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost));
    gemm_split32<<<1, 64>>>(dA, dB, dC, K);
    CHECK(hipMemcpy(C3.data(), dC, 1024, hipMemcpyDeviceToHost));
    gemm_split<<<1, 64>>>(dA, dB, dC, K, 1);
    CHECK(hipMemcpy(C2.data(), dC, 1024, hipMemcpyDeviceToHost));
    gemm_f32<<<1, 64>>>(dA, dB, dC, K);
    CHECK(hipMemcpy(Cf.data(), dC, 1024, hipMemcpyDeviceToHost));
    double e3 = 0, e3b = 0, e1 = 0, ef = 0;
    for (int m = 0; m < 16; ++m)
      for (int n = 0; n < 16; ++n) {
        double ref = 0, mag = 0;
        for (int k = 0; k < K; ++k) {
          ref += (double)A[m * K + k] * B[k * 16 + n];
          mag += fabs((double)A[m * K + k] * B[k * 16 + n]);
        }
        e3 = fmax(e3, fabs(C[m * 16 + n] - ref) / mag);
        e3b = fmax(e3b, fabs(C3[m * 16 + n] - ref) / mag);
        e1 = fmax(e1, fabs(C2[m * 16 + n] - ref) / mag);
        ef = fmax(ef, fabs(Cf[m * 16 + n] - ref) / mag);
      }
    printf("{\"K\": %d, \"err_over_sum_abs\": {\"split3_16x16x16\": %.3e, \"split3_16x16x32\": %.3e, \"f16_1term\": %.3e, "
           "\"f32_mfma\": %.3e}}\n", K, e3, e3b, e1, ef);
    CHECK(hipFree(dA));
    CHECK(hipFree(dB));
    CHECK(hipFree(dC));
  }
  denorm_probe<<<1, 64>>>(dout);
  float d[4];
  CHECK(hipMemcpy(d, dout, 16, hipMemcpyDeviceToHost));
  printf("{\"denorm_mfma\": %.9e, \"expected\": %.9e, \"split_lo\": %.9e, \"expected_lo\": %.9e}\n", d[0], d[1], d[2], d[3]);
  return 0;
}
