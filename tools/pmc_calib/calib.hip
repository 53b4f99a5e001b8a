// FETCH_SIZE calibration for gather reads. Each kernel reads a 1 GiB table (4x the 256 MiB
// Infinity Cache, so every line comes from HBM) with a known byte count, so rocprofv3's FETCH_SIZE per dispatch
// can be compared with the bytes the pattern must move:
//   stream16   16 B per lane, consecutive lanes consecutive records (the guide's calibrated case: FETCH = 1/2 bytes)
//   line16     16 B per lane, 8 lanes per 128-B line, the lines of a wave instruction in random order (whole lines)
//   rec16      16 B per lane, every 16-B record once, records in random order (no two lanes share a line)
//   rec32      32 B per lane (two adjacent 16-B loads), every 32-B record once, random order
//   rec64      64 B per lane-quad... as 4 lanes x 16 B of one 64-B record, records in random order
// Every record is read exactly once per dispatch, so the algorithmic bytes are the table size for every kernel; the
// difference between the kernels is the request granularity the L2 sends to the fabric.
// Build + run: tools/pmc_calib/run.sh (rocprofv3 --pmc FETCH_SIZE per pass).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {  // bijection on [0, 2^k) when masked with an odd multiplier
  return x * 2654435761u;
}

// rec index -> permuted rec index over n = 2^k records: affine bijection mod 2^k (odd multiplier) then xor
__device__ __forceinline__ uint32_t perm(uint32_t i, uint32_t mask) { return ((mix(i) + 0x9e3779b9u) ^ 0x5bd1e995u) & mask; }

__global__ __launch_bounds__(256) void stream16(const u4* __restrict__ t, uint32_t n16, u4* out) {
  u4 acc = {0, 0, 0, 0};
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) acc ^= t[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

// wave instruction j covers 8 lines: lane l reads 16 B chunk (l & 7) of line perm(8 j + (l >> 3))
__global__ __launch_bounds__(256) void line16(const u4* __restrict__ t, uint32_t nlines, u4* out) {
  u4 acc = {0, 0, 0, 0};
  const uint32_t mask = nlines - 1, lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, nwaves = gridDim.x * 4;
  for (uint32_t j = wave; j * 8 < nlines; j += nwaves) {
    const uint32_t line = perm(j * 8 + (lane >> 3), mask);
    acc ^= t[(size_t)line * 8 + (lane & 7)];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

template <int REC16>  // record = REC16 consecutive 16-B chunks, read by one lane
__global__ __launch_bounds__(256) void recN(const u4* __restrict__ t, uint32_t nrec, u4* out) {
  u4 acc = {0, 0, 0, 0};
  const uint32_t mask = nrec - 1;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nrec; i += gridDim.x * 256) {
    const uint32_t r = perm(i, mask);
#pragma unroll
    for (int k = 0; k < REC16; ++k) acc ^= t[(size_t)r * REC16 + k];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

// 64-B record read by a lane quad (4 lanes x 16 B, the way a coalesced 4-lane group reads one record)
__global__ __launch_bounds__(256) void rec64q(const u4* __restrict__ t, uint32_t nrec, u4* out) {
  u4 acc = {0, 0, 0, 0};
  const uint32_t mask = nrec - 1;
  const uint32_t q = (blockIdx.x * 256 + threadIdx.x) >> 2, nq = gridDim.x * 64;
  for (uint32_t i = q; i < nrec; i += nq) acc ^= t[(size_t)perm(i, mask) * 4 + (threadIdx.x & 3)];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = 1ull << 30;
  u4 *t, *out;
  CK(hipMalloc(&t, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(t, 0x5a, bytes));
  const uint32_t n16 = (uint32_t)(bytes / 16);
  const dim3 grid(2048), blk(256);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char* name, auto launch) {
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"kernel\": \"%s\", \"rep\": %d, \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", name, r, bytes, ms,
             bytes / ms / 1e6);
    }
  };
  timed("stream16", [&] { hipLaunchKernelGGL(stream16, grid, blk, 0, 0, t, n16, out); });
  timed("line16", [&] { hipLaunchKernelGGL(line16, grid, blk, 0, 0, t, (uint32_t)(bytes / 128), out); });
  timed("rec16", [&] { hipLaunchKernelGGL(recN<1>, grid, blk, 0, 0, t, n16, out); });
  timed("rec32", [&] { hipLaunchKernelGGL(recN<2>, grid, blk, 0, 0, t, n16 / 2, out); });
  timed("rec64q", [&] { hipLaunchKernelGGL(rec64q, grid, blk, 0, 0, t, n16 / 4, out); });
  CK(hipDeviceSynchronize());
  return 0;
}
