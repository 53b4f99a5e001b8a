// Does s_waitcnt vmcnt(N) count vector-memory operations strictly in issue order on gfx950? (round-3 diagnosis
// of the concurrent-stream corruption)
//
// Each lane, in ONE inline-asm block (so the compiler inserts no waits of its own):
//   A := sentinel;  A = buffer_load_dword (a cold line of a 1 GiB table: an HBM miss, ~1-2 us);
//   issue op B;  s_waitcnt vmcnt(1)  (= "all but the youngest done", i.e. A must be done);  snap := A;
//   s_waitcnt vmcnt(0)
// and counts lanes whose snapshot is still the sentinel: vmcnt(1) released before A's data arrived, i.e. op B
// was counted complete ahead of the older load A. Ops B:
//   inrange   buffer_load_dword of a hot line (control: must be 0)
//   oob       buffer_load_dword at an offset past the descriptor's range (returns 0 without a memory access)
//   store     buffer_store_dword (default policy) to a scratch line
//   store_nt  buffer_store_dword nt to a scratch line
//   gstore / gstore_nt  global_store_dword (default policy / nt) to a scratch line (the warp's volume stores)
// Build + run: tools/vmcnt_probe/run.sh
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

constexpr unsigned kSentinel = 0xdeadbeefu;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(const unsigned* __restrict__ table, unsigned table_words, unsigned* scratch,
                                             unsigned iters, unsigned* early, unsigned* wrong) {
  const __amdgpu_buffer_rsrc_t rt = rsrc(table, table_words * 4u);
  const __amdgpu_buffer_rsrc_t rs = rsrc(scratch, 1u << 20);
  const unsigned gid = blockIdx.x * 256 + threadIdx.x;
  unsigned n_early = 0, n_wrong = 0;
  for (unsigned it = 0; it < iters; ++it) {
    // a cold line: a random 128-byte line of the 1 GiB table for every (lane, iteration)
    const unsigned line = ((gid * 2654435761u) ^ (it * 40503u + 0x9e3779b9u)) % (table_words / 32u);
    const unsigned offA = line * 128u;
    const unsigned offB = MODE == 0 ? (gid % 32u) * 4u                    // hot: first line of the table
                          : MODE == 1 ? 0x80000000u                       // out of range
                                      : ((gid * 64u) & ((1u << 20) - 64u));  // scratch line
    unsigned a, b = 0, snap;
    if constexpr (MODE == 0 || MODE == 1) {
      asm volatile(
          "v_mov_b32 %0, %5\n\t"
          "buffer_load_dword %0, %3, %6, 0 offen\n\t"
          "buffer_load_dword %1, %4, %6, 0 offen\n\t"
          "s_waitcnt vmcnt(1)\n\t"
          "v_mov_b32 %2, %0\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(a), "=&v"(b), "=&v"(snap)
          : "v"(offA), "v"(offB), "v"(kSentinel), "s"(rt)
          : "memory");
    } else if constexpr (MODE == 2) {
      asm volatile(
          "v_mov_b32 %0, %4\n\t"
          "buffer_load_dword %0, %2, %5, 0 offen\n\t"
          "buffer_store_dword %4, %3, %6, 0 offen\n\t"
          "s_waitcnt vmcnt(1)\n\t"
          "v_mov_b32 %1, %0\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(a), "=&v"(snap)
          : "v"(offA), "v"(offB), "v"(kSentinel), "s"(rt), "s"(rs)
          : "memory");
    } else if constexpr (MODE == 4 || MODE == 5) {
      unsigned* dst = scratch + offB / 4u;
      if constexpr (MODE == 4)
        asm volatile(
            "v_mov_b32 %0, %4\n\t"
            "buffer_load_dword %0, %2, %5, 0 offen\n\t"
            "global_store_dword %3, %4, off\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "v_mov_b32 %1, %0\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(a), "=&v"(snap)
            : "v"(offA), "v"(dst), "v"(kSentinel), "s"(rt)
            : "memory");
      else
        asm volatile(
            "v_mov_b32 %0, %4\n\t"
            "buffer_load_dword %0, %2, %5, 0 offen\n\t"
            "global_store_dword %3, %4, off nt\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "v_mov_b32 %1, %0\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(a), "=&v"(snap)
            : "v"(offA), "v"(dst), "v"(kSentinel), "s"(rt)
            : "memory");
    } else {
      asm volatile(
          "v_mov_b32 %0, %4\n\t"
          "buffer_load_dword %0, %2, %5, 0 offen\n\t"
          "buffer_store_dword %4, %3, %6, 0 offen nt\n\t"
          "s_waitcnt vmcnt(1)\n\t"
          "v_mov_b32 %1, %0\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(a), "=&v"(snap)
          : "v"(offA), "v"(offB), "v"(kSentinel), "s"(rt), "s"(rs)
          : "memory");
    }
    (void)b;
    n_early += snap == kSentinel;
    n_wrong += a != line * 32u;  // table[w] = w: the first word of line L is 32 L
  }
  if (n_early) atomicAdd(early, n_early);
  if (n_wrong) atomicAdd(wrong, n_wrong);
}

__global__ void fill(unsigned* t, unsigned n) {
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) t[i] = i;
}

int main() {
  const unsigned words = 1u << 28;  // 1 GiB
  unsigned *table, *scratch, *cnt;
  CK(hipMalloc(&table, (size_t)words * 4));
  CK(hipMalloc(&scratch, 1 << 20));
  CK(hipMalloc(&cnt, 64));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, table, words);
  CK(hipDeviceSynchronize());
  const char* names[6] = {"inrange", "oob", "store", "store_nt", "gstore", "gstore_nt"};
  const unsigned iters = 64, blocks = 4096;
  printf("{\"probe\": \"vmcnt_in_order\", \"lanes_x_iters\": %llu, \"results\": [\n",
         (unsigned long long)blocks * 256 * iters);
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 6; ++m) {
      CK(hipMemset(cnt, 0, 64));
      switch (m) {
        case 0: hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
        case 1: hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
        case 2: hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
        case 3: hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
        case 4: hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
        default: hipLaunchKernelGGL(probe<5>, dim3(blocks), dim3(256), 0, 0, table, words, scratch, iters, cnt, cnt + 1); break;
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned h[2];
      CK(hipMemcpy(h, cnt, 8, hipMemcpyDeviceToHost));
      printf("%s  {\"op_b\": \"%s\", \"rep\": %d, \"released_before_older_load\": %u, \"final_value_wrong\": %u}",
             rep || m ? ",\n" : "", names[m], rep, h[0], h[1]);
      fflush(stdout);
    }
  printf("\n]}\n");
  return 0;
}
