// Standalone LDS co-residency experiment (diagnosis of the round-2 concurrent-stream corruption,
// DESIGN.md section 4 "Concurrent streams"): does a workgroup of one kernel see its LDS altered while
// a kernel with a large dynamic LDS allocation runs on another stream?
//
//   big<S>:  every block fills S bytes of dynamic LDS with a block/iteration-tagged pattern, barrier,
//            checks it, barrier, repeat (mismatches = someone else wrote into this block's LDS);
//   small:   720 bytes of static LDS (the warp's former camera copy), written once, then re-checked
//            for a while (mismatches = its LDS changed under it).
// Block 0 of every launch records s_getreg(LDS_ALLOC) (the allocation the hardware gave the
// workgroup), HW_ID and XCC_ID; every mismatching small block records its own LDS_ALLOC / HW_ID.
// Build: hipcc -O2 --offload-arch=gfx950 lds_race.hip -o lds_race   (tools/lds_race/run.sh)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

struct Rec {
  unsigned lds_alloc, hw_id, xcc_id, block;
};

__device__ __forceinline__ Rec me() {
  Rec r;
  r.lds_alloc = __builtin_amdgcn_s_getreg((31 << 11) | 6);
  r.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  r.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  r.block = blockIdx.x;
  return r;
}

__device__ __forceinline__ unsigned pat(unsigned tag, unsigned i, unsigned it) { return (tag ^ (i * 2654435761u)) + it; }

__global__ __launch_bounds__(256) void big_kernel(int words, int iters, unsigned* err, Rec* rec0) {
  extern __shared__ unsigned s[];
  if (blockIdx.x == 0 && threadIdx.x == 0) *rec0 = me();
  const unsigned tag = blockIdx.x * 131u + 7u;
  unsigned bad = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < words; i += 256) s[i] = pat(tag, i, it);
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += 256) bad += s[i] != pat(tag, i, it);
    __syncthreads();
  }
  if (bad) atomicAdd(err, bad);
}

constexpr int kSmallWords = 180;  // 720 bytes

__global__ __launch_bounds__(256) void small_kernel(int iters, unsigned* err, Rec* rec0, Rec* bad_recs, int max_bad) {
  __shared__ unsigned s[kSmallWords];
  if (blockIdx.x == 0 && threadIdx.x == 0) *rec0 = me();
  const unsigned tag = blockIdx.x * 977u + 3u;
  if (threadIdx.x < kSmallWords) s[threadIdx.x] = pat(tag, threadIdx.x, 0);
  __syncthreads();
  unsigned bad = 0;
  for (int it = 0; it < iters; ++it) {
    if (threadIdx.x < kSmallWords) bad += s[threadIdx.x] != pat(tag, threadIdx.x, 0);
    __builtin_amdgcn_s_sleep(4);
  }
  if (bad) {
    atomicAdd(err, bad);
    if (threadIdx.x % 64 == 0) {
      const unsigned slot = atomicAdd(err + 1, 1u);  // record counter
      if (slot < (unsigned)max_bad) bad_recs[slot] = me();
    }
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 8;
  const int sizes[] = {16384, 49152, 65536, 66560, 69120, 69888, 98304, 138240, 163840};
  unsigned *d_err;
  Rec* d_rec;
  CK(hipMalloc(&d_err, 4 * sizeof(unsigned)));
  CK(hipMalloc(&d_rec, 64 * sizeof(Rec)));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(big_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  printf("{\"experiment\": \"lds_race\", \"rounds\": %d, \"results\": [\n", rounds);
  bool first = true;
  for (int mode = 0; mode < 3; ++mode) {  // 0: big alone, 1: small alone, 2: both on two streams
    for (int S : sizes) {
      if (mode == 1 && S != sizes[0]) continue;
      CK(hipMemset(d_err, 0, 4 * sizeof(unsigned)));
      CK(hipMemset(d_rec, 0, 64 * sizeof(Rec)));
      for (int r = 0; r < rounds; ++r) {
        if (mode != 1) hipLaunchKernelGGL(big_kernel, dim3(1024), dim3(256), (size_t)S, s1, S / 4, 400, d_err + 0, d_rec + 0);
        if (mode != 0) hipLaunchKernelGGL(small_kernel, dim3(8192), dim3(256), 0, s2, 3000, d_err + 1, d_rec + 1, d_rec + 2, 62);
        CK(hipGetLastError());
      }
      CK(hipDeviceSynchronize());
      unsigned err[4];
      Rec rec[64];
      CK(hipMemcpy(err, d_err, sizeof(err), hipMemcpyDeviceToHost));
      CK(hipMemcpy(rec, d_rec, sizeof(rec), hipMemcpyDeviceToHost));
      printf("%s  {\"mode\": \"%s\", \"big_lds_bytes\": %d, \"big_mismatch\": %u, \"small_mismatch\": %u, "
             "\"big_lds_alloc\": \"0x%08x\", \"big_hw_id\": \"0x%08x\", \"small_lds_alloc\": \"0x%08x\", \"small_bad\": [",
             first ? "" : ",\n", mode == 0 ? "big" : mode == 1 ? "small" : "both", mode == 1 ? 0 : S, err[0], err[1],
             rec[0].lds_alloc, rec[0].hw_id, rec[1].lds_alloc);
      first = false;
      const int nb = err[2] < 62 ? (int)err[2] : 62;
      for (int i = 0, k = 0; i < nb && k < 8; ++i) {
        if (!rec[2 + i].hw_id && !rec[2 + i].lds_alloc) continue;
        printf("%s{\"lds_alloc\": \"0x%08x\", \"hw_id\": \"0x%08x\", \"xcc\": %u, \"block\": %u}", k ? ", " : "",
               rec[2 + i].lds_alloc, rec[2 + i].hw_id, rec[2 + i].xcc_id, rec[2 + i].block);
        ++k;
      }
      printf("]}");
      fflush(stdout);
    }
  }
  printf("\n]}\n");
  return 0;
}
