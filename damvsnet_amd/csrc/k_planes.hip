// The 2D front end's plane-input layers on the VALU (FeatureNet's RGB conv, GeoFeatureFusion's RGB+depth and
// depth+depth init convs; models/module.py:355-462, models/geometry.py:87-277): moved out of k_conv2d.hip in round 6 and
// built without the SLP vectorizer (damvsnet_amd/build.py FILE_FLAGS), with one scalar FMA per channel instead of the
// former explicit channel-pair v_pk_fma_f32 -- the same fused multiply-adds, so bitwise the same outputs. Rule behind
// it: no kernel without MFMA instructions carries packed-FP32 VALU ops (tests/test_isa_pins.py), because the warp's
// packed FMAs computed wrong values in lanes 48-63 while MFMA kernels of another stream shared the CU (DESIGN.md
// section 4, "Concurrent streams"); these kernels run beside the other sub-batch's MFMA kernels in every two-stream
// forward.
#include <cstdint>
#include <cstdlib>

#include "conv2d_common.h"

namespace damvs {

namespace {

// Direct conv for layers whose only inputs are fp32 planes (c0 = c1 = 0: FeatureNet's RGB conv
// 3x3 3->8, GeoFeatureFusion's RGB+depth 5x5 4->8 and depth+depth 5x5 2->8 init convs). The MFMA
// kernel would run these in its epilogue with half the lanes idle and one dependent load chain per
// tap. Here (stride 1, padding K/2) one thread computes 2 vertically adjacent output pixels x all
// COUT channels: the K+1 input rows they need are loaded row by row (K*NG branch-free coalesced
// loads in flight per row, each row feeding both pixels); weights sit in LDS as wave-uniform
// broadcast reads.
template <typename T, int COUT, int K, int NG>
__global__ __launch_bounds__(256) void conv2d_planes_kernel(const Conv2dArgs a, const float* __restrict__ wg) {
  constexpr int P = K / 2;
  const int Hp = (a.Ho + 1) / 2;
  const int Qtot = a.B * Hp * a.Wo;  // host checks it fits in int
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Qtot) return;
  const int ox = q % a.Wo;
  const int oy0 = (q / a.Wo) % Hp * 2;
  const int b = q / (a.Wo * Hp);
  // Weights are wave-uniform: scalar loads (restrict const argument) feed one fused multiply-add per channel
  // (scalar FMAs, no packed-FP32 ops: see k_planes.hip's header). Input row r feeds pixel 0 with kernel row r (r < K)
  // and pixel 1 with kernel row r-1 (r > 0).
  float acc0[COUT], acc1[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc0[c] = acc1[c] = a.bias[c];
  const float* gp[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) gp[g] = a.geo[g] + (size_t)b * a.geo_bstride[g];
  const int cp = a.cout_pad;
#pragma unroll 1  // (fully unrolled: all rows' loads hoisted, 1.2-2.4x slower)
  for (int r = 0; r <= K; ++r) {
    const int iy = oy0 - P + r;
    const bool oky = (unsigned)iy < (unsigned)a.Hi;
    const int rowoff = (oky ? iy : 0) * a.Wi;
    float v[K][NG];
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int ix = ox - P + kx;
      const bool ok = oky && (unsigned)ix < (unsigned)a.Wi;
      const int off = rowoff + (ok ? ix : 0);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float x = gp[g][off];  // clamped address, unconditional load
        v[kx][g] = ok ? x : 0.f;
      }
    }
    auto row = [&](const float* w, float* acc) {
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const float x = v[kx][g];
          const float* wt = w + (kx * NG + g) * cp;
#pragma unroll
          for (int c = 0; c < COUT; ++c) acc[c] = fmaf(wt[c], x, acc[c]);
        }
    };
    if (r < K) row(wg + (size_t)r * K * NG * cp, acc0);
    if (r > 0) row(wg + (size_t)(r - 1) * K * NG * cp, acc1);
  }
  float* o0 = acc0;
  float* o1 = acc1;
  const bool two = oy0 + 1 < a.Ho;
#pragma unroll
  for (int c0 = 0; c0 < COUT; c0 += 4) {
    if (c0 >= a.cout) break;
    tail4<T>(a, b, oy0, ox, c0, o0 + c0);
    if (two) tail4<T>(a, b, oy0 + 1, ox, c0, o1 + c0);
  }
}

// Plane-only layers (as conv2d_planes_kernel) with 4 consecutive output columns x 2 rows per thread: each input row
// arrives as three aligned 16-byte loads per plane (columns x0 - 4 .. x0 + 7) instead of K scalar loads per pixel
// column, a quarter of the load instructions for the same fused multiply-adds (same order per output: bitwise the
// one-column kernel). Needs Wi % 4 == 0 and 16-byte aligned planes (launch_planes checks); COUT 8.
template <typename T, int COUT, int K, int NG>
__global__ __launch_bounds__(256) void conv2d_planes4_kernel(const Conv2dArgs a, const float* __restrict__ wg) {
  constexpr int P = K / 2;
  const int Hp = (a.Ho + 1) / 2, Wg = a.Wo / 4;
  const int Qtot = a.B * Hp * Wg;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Qtot) return;
  const int ox0 = (q % Wg) * 4;
  const int oy0 = (q / Wg) % Hp * 2;
  const int b = q / (Wg * Hp);
  float acc[2][4][COUT];  // [output row][column][channel]
#pragma unroll
  for (int c = 0; c < COUT; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[0][j][c] = acc[1][j][c] = a.bias[c];
  __amdgpu_buffer_rsrc_t rg[NG];
  uint32_t gb[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    rg[g] = make_rsrc(a.geo[g], ((long long)(a.B - 1) * a.geo_bstride[g] + (long long)a.Hi * a.Wi) * 4);
    gb[g] = (uint32_t)((long long)b * a.geo_bstride[g]) * 4u;
  }
  const int cp = a.cout_pad;
#pragma unroll 1
  for (int r = 0; r <= K; ++r) {
    const int iy = oy0 - P + r;
    const bool oky = (unsigned)iy < (unsigned)a.Hi;
    float v[NG][12];  // columns ox0 - 4 .. ox0 + 7
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int ix = ox0 - 4 + 4 * h;
        const bool ok = oky && ix >= 0 && ix < a.Wi;  // whole 16-byte groups: Wi % 4 == 0
        const float4 f = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                        rg[g], ok ? (uint32_t)(iy * a.Wi + ix) * 4u : kOOB, gb[g], 0));
        v[g][4 * h] = f.x; v[g][4 * h + 1] = f.y; v[g][4 * h + 2] = f.z; v[g][4 * h + 3] = f.w;
      }
    auto row = [&](const float* w, float (*acc_r)[COUT]) {
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const float* wt = w + (kx * NG + g) * cp;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xv = v[g][4 - P + j + kx];
#pragma unroll
            for (int c = 0; c < COUT; ++c) acc_r[j][c] = fmaf(wt[c], xv, acc_r[j][c]);
          }
        }
    };
    if (r < K) row(wg + (size_t)r * K * NG * cp, acc[0]);
    if (r > 0) row(wg + (size_t)(r - 1) * K * NG * cp, acc[1]);
  }
  const bool two = oy0 + 1 < a.Ho;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float* o0 = acc[0][j];
    float* o1 = acc[1][j];
#pragma unroll
    for (int c0 = 0; c0 < COUT; c0 += 4) {
      if (c0 >= a.cout) break;
      tail4<T>(a, b, oy0, ox0 + j, c0, o0 + c0);
      if (two) tail4<T>(a, b, oy0 + 1, ox0 + j, c0, o1 + c0);
    }
  }
}

// Any other plane-only layer (stride 2, transposed; no production layer): one thread per output
// pixel of a phase, all (<= 16) output channels.
template <typename T>
__global__ __launch_bounds__(256) void conv2d_planes_generic_kernel(const Conv2dArgs a) {
  const int Qtot = a.B * a.Hq * a.Wq;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const Conv2dPhase& ph = a.ph[blockIdx.y];
  if (q >= Qtot) return;
  const int qx = q % a.Wq, qy = (q / a.Wq) % a.Hq, b = q / (a.Wq * a.Hq);
  float acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = a.bias[c];
  const float* wg = a.wgeo + (size_t)ph.g_off * a.cout_pad;
  for (int t = 0; t < ph.ntaps; ++t) {
    const int iy = qy * a.in_stride + ph.tap[t][0], ix = qx * a.in_stride + ph.tap[t][1];
    if ((unsigned)iy >= (unsigned)a.Hi || (unsigned)ix >= (unsigned)a.Wi) continue;
    for (int g = 0; g < a.ngeo; ++g) {
      const float v = a.geo[g][b * a.geo_bstride[g] + iy * a.Wi + ix];
      const float* w = wg + (t * a.ngeo + g) * a.cout_pad;
#pragma unroll
      for (int c = 0; c < 16; ++c) acc[c] += w[c] * v;
    }
  }
  const int oy = qy * a.out_stride + ph.py, ox = qx * a.out_stride + ph.px;
  for (int c0 = 0; c0 < a.cout; c0 += 4) tail4<T>(a, b, oy, ox, c0, acc + c0);
}

// True when the layer is a plain (non-transposed) KxK conv with padding K/2 and dense row-major taps.
bool planes_fast_ok(const Conv2dArgs& a, int K) {
  if (a.nphase != 1 || a.out_stride != 1 || a.in_stride != 1 || (long long)a.B * a.Ho * a.Wo >= (1LL << 31) || a.ph[0].ntaps != K * K || a.ph[0].g_off != 0) return false;
  for (int t = 0; t < K * K; ++t)
    if (a.ph[0].tap[t][0] != t / K - K / 2 || a.ph[0].tap[t][1] != t % K - K / 2) return false;
  return true;
}

template <typename T, int K>
hipError_t launch_planes4_k(hipStream_t st, const Conv2dArgs& a) {
  const long long Qtot = (long long)a.B * ((a.Ho + 1) / 2) * (a.Wo / 4);
  dim3 grid((unsigned)((Qtot + 255) / 256));
  switch (a.ngeo) {
    case 1: hipLaunchKernelGGL((conv2d_planes4_kernel<T, 8, K, 1>), grid, dim3(256), 0, st, a, a.wgeo); break;
    case 2: hipLaunchKernelGGL((conv2d_planes4_kernel<T, 8, K, 2>), grid, dim3(256), 0, st, a, a.wgeo); break;
    case 3: hipLaunchKernelGGL((conv2d_planes4_kernel<T, 8, K, 3>), grid, dim3(256), 0, st, a, a.wgeo); break;
    default: hipLaunchKernelGGL((conv2d_planes4_kernel<T, 8, K, 4>), grid, dim3(256), 0, st, a, a.wgeo); break;
  }
  return hipGetLastError();
}

// conv2d_planes4_kernel's conditions: 4-column groups of whole 16-byte plane pieces (DAMVS_PLANES4=0, read per call:
// the one-column kernel)
bool planes4_ok(const Conv2dArgs& a) {
  const char* v = getenv("DAMVS_PLANES4");
  if ((v && v[0] == '0') || a.cout > 8 || a.Wi % 4 || a.Wo != a.Wi) return false;
  for (int g = 0; g < a.ngeo; ++g)
    if (reinterpret_cast<uintptr_t>(a.geo[g]) % 16 || a.geo_bstride[g] % 4) return false;
  return true;
}

template <typename T, int COUT, int K>
hipError_t launch_planes_k(hipStream_t st, const Conv2dArgs& a) {
  const long long Qtot = (long long)a.B * ((a.Ho + 1) / 2) * a.Wo;
  dim3 grid((unsigned)((Qtot + 255) / 256));
  switch (a.ngeo) {
    case 1: hipLaunchKernelGGL((conv2d_planes_kernel<T, COUT, K, 1>), grid, dim3(256), 0, st, a, a.wgeo); break;
    case 2: hipLaunchKernelGGL((conv2d_planes_kernel<T, COUT, K, 2>), grid, dim3(256), 0, st, a, a.wgeo); break;
    case 3: hipLaunchKernelGGL((conv2d_planes_kernel<T, COUT, K, 3>), grid, dim3(256), 0, st, a, a.wgeo); break;
    default: hipLaunchKernelGGL((conv2d_planes_kernel<T, COUT, K, 4>), grid, dim3(256), 0, st, a, a.wgeo); break;
  }
  return hipGetLastError();
}

// Returns hipErrorNotSupported when the layer is not of the fast form (caller uses the MFMA kernel).
template <typename T>
hipError_t launch_planes(hipStream_t st, const Conv2dArgs& a) {
  const int K = a.ph[0].ntaps == 9 ? 3 : a.ph[0].ntaps == 25 ? 5 : 0;
  if (K == 0 || a.ngeo < 1 || a.ngeo > 4 || a.cout > 16 || a.cout_pad < 16 || !planes_fast_ok(a, K))
    return hipErrorNotSupported;
  // 5x5 only: GeoFF stage-3 init convs 5.21-5.28 against 5.30-5.43 ms; at 3x3 (FeatureNet's RGB conv, half of each
  // 12-column window unused, a quarter of the threads) features 2.86-2.89 against 2.77 ms (profiles/r03/ab_planes4.jsonl)
  if (K == 5 && planes4_ok(a)) return launch_planes4_k<T, 5>(st, a);
  if (a.cout <= 8) return K == 3 ? launch_planes_k<T, 8, 3>(st, a) : launch_planes_k<T, 8, 5>(st, a);
  return K == 3 ? launch_planes_k<T, 16, 3>(st, a) : launch_planes_k<T, 16, 5>(st, a);
}

// The fast kernels where they take the layer (launch_planes), else the generic one (stride 2, transposed).
template <typename T>
hipError_t launch_planes_any(hipStream_t s, const Conv2dArgs& a) {
  const hipError_t e = launch_planes<T>(s, a);
  if (e != hipErrorNotSupported) return e;
  if (a.cout > 16 || a.cout_pad < 16) return hipErrorInvalidValue;
  dim3 grid((unsigned)((a.B * a.Hq * a.Wq + 255) / 256), a.nphase);
  hipLaunchKernelGGL(conv2d_planes_generic_kernel<T>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_conv2d_planes(hipStream_t st, int store, const Conv2dArgs& a) {
  return store == ST_BF16 ? launch_planes_any<bf16_t>(st, a) : launch_planes_any<float>(st, a);
}

}  // namespace damvs
