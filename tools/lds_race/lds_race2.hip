// LDS read forms beside a kernel with heavy 16-byte LDS traffic on another stream (round-3 diagnosis: with its
// cameras staged in LDS, the stage-2 warp computed wrong rays for exactly lanes 48-63 of some waves when a U-Net
// kernel ran concurrently, while a per-thread ds_read_b32 check of the same LDS words was always clean).
//
//   hog:    every block streams ds_write_b128 / ds_read_b128 over 48 KiB of dynamic LDS (the z-streamed conv
//           kernels' pattern), checking what it reads back.
//   reader<FORM>: 256-thread blocks stage 48 words in LDS (threads 0-47 write, barrier), then repeatedly read them
//           with FORM and compare per lane; mismatches are counted per 16-lane group of the wave:
//     0 bcast32   every lane reads word i (ds_read_b32, same address in all lanes)
//     1 bcast64   every lane reads words i, i+1 (ds_read_b64)
//     2 bcast128  every lane reads words i..i+3 (ds_read_b128)
//     3 lane128   lane l reads words 4 (l % 12) .. +3 (ds_read_b128, per-lane addresses)
//     4 bcast128_once  as 2 but read once right after the barrier into registers and checked at the end of a
//                      long VALU loop (the warp's hoisted-ray pattern)
// Output: one JSON line per (form, with/without hog) with mismatches per lane group.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void hog(int iters, unsigned* err) {
  extern __shared__ f4 sh[];
  constexpr int N = 48 * 1024 / 16;
  unsigned bad = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < N; i += 256) sh[i] = (f4){(float)(i + it), (float)blockIdx.x, 1.f, 2.f};
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += 256) {
      const f4 v = sh[(i * 7 + it) % N];
      bad += v.x != (float)((i * 7 + it) % N + it) || v.y != (float)blockIdx.x;
    }
    __syncthreads();
  }
  if (bad) atomicAdd(err, bad);
}

__device__ __forceinline__ float val(unsigned blk, int i) { return (float)(blk * 64u + (unsigned)i) * 0.25f + 1.f; }

template <int FORM>
__global__ __launch_bounds__(256) void reader(int iters, unsigned* grp_err) {
  __shared__ __attribute__((aligned(16))) float s[64];
  if (threadIdx.x < 48) s[threadIdx.x] = val(blockIdx.x, threadIdx.x);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned bad = 0;
  if constexpr (FORM == 4) {
    f4 r[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) r[k] = *reinterpret_cast<const f4*>(s + 4 * k);
    float acc = 0.f;
    for (int it = 0; it < iters * 8; ++it) acc = fmaf(acc, 0.999f, (float)it);  // a long VALU stretch
#pragma unroll
    for (int k = 0; k < 12; ++k)
      bad += (r[k].x != val(blockIdx.x, 4 * k)) + (r[k].y != val(blockIdx.x, 4 * k + 1)) +
             (r[k].z != val(blockIdx.x, 4 * k + 2)) + (r[k].w != val(blockIdx.x, 4 * k + 3));
    bad += acc == -1.f;
  } else {
    for (int it = 0; it < iters; ++it) {
      asm volatile("" ::: "memory");  // re-read LDS every iteration (the compiler may not cache it in registers)
      const int i = (it * 4) % 48;
      if constexpr (FORM == 0) {
        bad += s[i] != val(blockIdx.x, i);
      } else if constexpr (FORM == 1) {
        const f2 v = *reinterpret_cast<const f2*>(s + i);
        bad += (v.x != val(blockIdx.x, i)) + (v.y != val(blockIdx.x, i + 1));
      } else if constexpr (FORM == 2) {
        const f4 v = *reinterpret_cast<const f4*>(s + i);
        bad += (v.x != val(blockIdx.x, i)) + (v.y != val(blockIdx.x, i + 1)) + (v.z != val(blockIdx.x, i + 2)) +
               (v.w != val(blockIdx.x, i + 3));
      } else {
        const int j = 4 * ((lane + it) % 12);
        const f4 v = *reinterpret_cast<const f4*>(s + j);
        bad += (v.x != val(blockIdx.x, j)) + (v.y != val(blockIdx.x, j + 1)) + (v.z != val(blockIdx.x, j + 2)) +
               (v.w != val(blockIdx.x, j + 3));
      }
    }
  }
  if (bad) atomicAdd(grp_err + lane / 16, bad);
}

int main() {
  unsigned* d;
  CK(hipMalloc(&d, 64));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const char* names[5] = {"bcast32", "bcast64", "bcast128", "lane128", "bcast128_once"};
  printf("{\"experiment\": \"lds_race2\", \"results\": [\n");
  bool first = true;
  for (int withhog = 0; withhog < 2; ++withhog)
    for (int f = 0; f < 5; ++f) {
      CK(hipMemset(d, 0, 64));
      for (int r = 0; r < 12; ++r) {
        if (withhog) hipLaunchKernelGGL(hog, dim3(2048), dim3(256), 48 * 1024, s1, 200, d + 8);
        switch (f) {
          case 0: hipLaunchKernelGGL(reader<0>, dim3(16384), dim3(256), 0, s2, 400, d); break;
          case 1: hipLaunchKernelGGL(reader<1>, dim3(16384), dim3(256), 0, s2, 400, d); break;
          case 2: hipLaunchKernelGGL(reader<2>, dim3(16384), dim3(256), 0, s2, 400, d); break;
          case 3: hipLaunchKernelGGL(reader<3>, dim3(16384), dim3(256), 0, s2, 400, d); break;
          default: hipLaunchKernelGGL(reader<4>, dim3(16384), dim3(256), 0, s2, 400, d); break;
        }
        CK(hipGetLastError());
      }
      CK(hipDeviceSynchronize());
      unsigned h[16];
      CK(hipMemcpy(h, d, 64, hipMemcpyDeviceToHost));
      printf("%s  {\"form\": \"%s\", \"beside_hog\": %d, \"mismatch_per_lane_group\": [%u, %u, %u, %u], \"hog_mismatch\": %u}",
             first ? "" : ",\n", names[f], withhog, h[0], h[1], h[2], h[3], h[8]);
      first = false;
      fflush(stdout);
    }
  printf("\n]}\n");
  return 0;
}
