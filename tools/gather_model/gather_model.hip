// What does a 16-byte-per-lane gather instruction cost on gfx950 as a function of how many distinct cache lines
// its 64 lanes touch? (round-3 warp study: the warp's gathers are the issue-bound part of the step.)
// Lanes form groups of G consecutive lanes reading 16 G contiguous bytes; group k starts at k * GAP bytes (+ a
// per-iteration shift inside a small region, so every access hits L1 or L2). Each wave issues ITERS x 8 such
// buffer_load_dwordx4. Prints one JSON line per pattern: ns per wave-instruction per CU and the lines touched.
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

__global__ __launch_bounds__(256) void gather(const unsigned char* base, unsigned region, int G, int GAP, int SHIFT,
                                              int iters, unsigned* sink) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(base), (short)0,
                                                                    (int)(region * 2u), 0x00020000);
  const int lane = threadIdx.x & 63;
  const unsigned lo = (unsigned)((lane / G) * GAP + (lane % G) * 16);
  const unsigned boff = (blockIdx.x % 64) * (region / 64u) & ~127u;  // blocks spread over the region
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned off = (boff + lo + (unsigned)((it * 8 + k) * SHIFT)) % region;
      const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      acc ^= v.x + v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const unsigned region = argc > 1 ? (unsigned)atoi(argv[1]) : (1u << 20);  // bytes touched by the whole grid
  unsigned char* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, region * 2u));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, region * 2u));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  struct P { int G, GAP, SHIFT; const char* what; };
  const P pats[] = {
      {64, 0, 1024, "1 KB contiguous (8 lines)"},
      {2, 32, 1024, "32 pairs x 32 B contiguous (8 lines)"},
      {4, 64, 1024, "16 quads x 64 B contiguous (8 lines)"},
      {2, 36, 1024, "32 pairs x 32 B, 36-B pitch (~10 lines, unaligned)"},
      {2, 40, 1024, "32 pairs x 32 B, 40-B pitch (~11 lines)"},
      {2, 48, 1024, "32 pairs x 32 B, 48-B pitch (~12 lines)"},
      {2, 64, 2048, "32 pairs, 64-B pitch (16 lines)"},
      {4, 128, 2048, "16 quads x 64 B, 128-B pitch (16 lines)"},
      {2, 128, 4096, "32 pairs, 128-B pitch (32 lines)"},
      {1, 128, 8192, "64 x 16 B, 128-B pitch (64 lines)"},
      {8, 1024, 8192, "8 groups x 128 B, 1 KB pitch (8 lines, spread)"},
      {4, 272, 4096, "16 quads x 64 B, 272-B pitch (16-32 lines)"},
      {2, 800 * 32 / 24, 4096, "32 pairs along a steep line (32 lines)"},
  };
  const int iters = 64, blocks = cus * 16;
  printf("{\"experiment\": \"gather_model\", \"cus\": %d, \"region_bytes\": %u, \"results\": [\n", cus, region);
  for (size_t i = 0; i < sizeof(pats) / sizeof(pats[0]); ++i) {
    const P& p = pats[i];
    for (int rep = 0; rep < 2; ++rep)
      hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, buf, region, p.G, p.GAP, p.SHIFT, iters, sink);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    const int reps = 5;
    for (int rep = 0; rep < reps; ++rep)
      hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, buf, region, p.G, p.GAP, p.SHIFT, iters, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double instr = (double)reps * blocks * 4 * iters * 8;  // wave-instructions
    const double ns_per_instr_cu = ms * 1e6 / (instr / cus);
    printf("%s  {\"G\": %d, \"gap\": %d, \"pattern\": \"%s\", \"ns_per_wave_instr_per_cu\": %.3f, \"cycles_at_2.4GHz\": %.1f,"
           " \"lane_TBps\": %.2f}",
           i ? ",\n" : "", p.G, p.GAP, p.what, ns_per_instr_cu, ns_per_instr_cu * 2.4, instr * 1024 / (ms * 1e-3) / 1e12);
    fflush(stdout);
  }
  printf("\n]}\n");
  return 0;
}
