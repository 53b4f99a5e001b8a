// The 2D front end's plane-input layers on the VALU (FeatureNet's RGB conv, GeoFeatureFusion's RGB+depth and
// depth+depth init convs; models/module.py:355-462, models/geometry.py:87-277): moved out of k_conv2d.hip in round 6 and
// built without the SLP vectorizer (damvsnet_amd/build.py FILE_FLAGS), with one scalar FMA per channel instead of the
// former explicit channel-pair v_pk_fma_f32 -- the same fused multiply-adds, so bitwise the same outputs. Rule behind
// it: no kernel without MFMA instructions carries packed-FP32 VALU ops (tests/test_isa_pins.py), because the warp's
// packed FMAs computed wrong values in lanes 48-63 while MFMA kernels of another stream shared the CU (DESIGN.md
// section 4, "Concurrent streams"); these kernels run beside the other sub-batch's MFMA kernels in every two-stream
// forward. Since late round 6 the production layers (cout 4 / 8, W % 4 == 0) run on conv2d_planes_mfma_kernel below
// (split-f16 MFMAs); the VALU kernels serve the other shapes and DAMVS_PLANES_MFMA=0.
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

// Plane-only layers as an implicit GEMM on split-f16 MFMAs (round 6; mma_split32, damvs_device.h). The VALU kernels
// above spend ~K*K*NG fused multiply-adds per output channel and pixel and run at 0.27-0.38 of the VALU peak (2.9x the
// HBM floor at FeatureNet's RGB conv, 6x at GeoFF's RGB+depth init). Here a block owns a 16 x 64 output tile; its
// (16 + K - 1) x 72 x NG halo (columns x0 - 4 .. x0 + 67, aligned 16-byte loads) goes to LDS once, each element as
// one dword [f16 hi | f16 lo] of x * 2^ka (ka from the block's max |x|, as the activation prescale: both pieces
// normal for every value down to max * 2^-17). The MFMA rows are a row pair (rows 0-7: output row y, channels 0-7;
// rows 8-15: row y + 1), so one B column -- the (K + 1) x K x NG window of an output column, ordered (input row,
// tap column, plane) -- feeds both rows: K' = (K + 1) K NG, in 32-K chunks (K 5, 4 planes: 4 chunks for 32 outputs
// against 8 for one-row tiles). A fragments are built per wave from the fp32 weights (wgeo) scaled by 2^kw (its max
// |w|, same rule) and split once; a lane's 8 B values per chunk are 8 ds_read_b32 at per-lane offsets computed once
// and a v_perm per pair into the hi / lo fragments. Accumulators are scaled back by 2^-(ka + kw) (exact) before the
// bias. Per product the split form's ~2^-21 (fp32 VALU: ~2^-24); K-padding columns read the window's last element
// against zero weights. DAMVS_PLANES_MFMA=0 (read per call): the VALU kernels.
template <typename T, int K, int NG>
__global__ __launch_bounds__(256) void conv2d_planes_mfma_kernel(const Conv2dArgs a, int tiles_x, int tiles_y, int nt) {
  constexpr int P = K / 2;
  constexpr int TR = 16, TC = 64;        // output tile
  constexpr int HR = TR + K - 1;         // halo rows
  constexpr int PITCH = TC + 8, C4 = PITCH / 4;
  constexpr int PLANE = HR * PITCH;
  constexpr int NGP = NG == 3 ? 4 : NG;  // planes per tap in the K order (3 padded to 4: a divisor of 8)
  constexpr int KP = (K + 1) * K * NGP;  // row-pair K
  constexpr int NCH = (KP + 31) / 32;    // 32-K chunks
  constexpr int TPF = 8 / NGP;           // taps per 8-element K fragment
  constexpr int NLD = (HR * C4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint32_t halo[NG * PLANE];
  __shared__ unsigned s_max[4];

  // logical block = (column of tiles, group of nt tile rows, image), XCD-contiguous; the group's tiles run in turn
  const int tgroups = (tiles_y + nt - 1) / nt;
  const int nblk = tiles_x * tgroups * a.B;
  const int bid = blockIdx.x, q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tx = L % tiles_x, tg = (L / tiles_x) % tgroups, b = L / (tiles_x * tgroups);
  const int x0 = tx * TC, ty0 = tg * nt, ty1 = min(ty0 + nt, tiles_y);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;

  // halo of the tile at output row y0: NG planes x HR rows x C4 aligned 16-byte pieces (Wi % 4 == 0: a piece is
  // inside or outside the image as a whole), into registers; the next tile's is in flight during a tile's MFMAs
  __amdgpu_buffer_rsrc_t rg[NG];
  uint32_t gb[NG];
#pragma unroll
  for (int pl = 0; pl < NG; ++pl) {
    rg[pl] = make_rsrc(a.geo[pl], ((long long)(a.B - 1) * a.geo_bstride[pl] + (long long)a.Hi * a.Wi) * 4);
    gb[pl] = (uint32_t)((long long)b * a.geo_bstride[pl]) * 4u;
  }
  float4 hv[NG][NLD];
  auto hload = [&](int y0) {
#pragma unroll
    for (int pl = 0; pl < NG; ++pl)
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        const int i = tid + k * 256, row = i / C4, c4 = i - row * C4;
        const int iy = y0 - P + row, ix = x0 - 4 + 4 * c4;
        const bool ok = i < HR * C4 && (unsigned)iy < (unsigned)a.Hi && ix >= 0 && ix < a.Wi;
        hv[pl][k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rg[pl], ok ? (uint32_t)(iy * a.Wi + ix) * 4u : kOOB, gb[pl], 0));
      }
  };
  hload(ty0 * TR);

  // A fragments of this wave: lane (row m, K group g); row m = output row m >> 3 of the pair, channel m & 7
  const int co_a = n & 7, dr = n >> 3;
  float wv[NCH][8];
  unsigned wm = 0u;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = 32 * c + 8 * g + e;
      const int r = kk / (K * NGP), kx = (kk / NGP) % K, ch = kk % NGP, rr = r - dr;
      const bool ok = kk < KP && ch < NG && co_a < a.cout && rr >= 0 && rr < K;
      const float w = a.wgeo[ok ? ((rr * K + kx) * NG + ch) * a.cout_pad + co_a : 0];  // unconditional, in range
      wv[c][e] = ok ? w : 0.f;
      wm = amax_fold(wm, wv[c][e]);
    }
#pragma unroll
  for (int o = 32; o; o >>= 1) wm = max(wm, (unsigned)__shfl_xor((int)wm, o));
  const Prescale pw = prescale_from_max(__builtin_amdgcn_readfirstlane(wm));
  F16Pair A[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = wv[c][e] * pw.s;
    A[c] = split8(t);
  }
  // B offsets of this lane (output column n of the unit, K group g): element e of chunk c is plane e % NGP (an
  // immediate offset; plane 3 of 3 reads plane 0 against zero weights) of tap (32 c + 8 g) / NGP + e / NGP, whose
  // offset (wave's first row pair included) is one register per tap; K padding reads the window's last tap
  int boff[NCH][TPF];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < TPF; ++j) {
      const int t = min((32 * c + 8 * g) / NGP + j, (K + 1) * K - 1);
      boff[c][j] = (2 * wave + t / K) * PITCH + t % K + 4 - P + n;
    }
  const int co = (g & 1) * 4, orow = g >> 1;
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = co + i < a.cout ? a.bias[co + i] : 0.f;

  for (int ty = ty0; ty < ty1; ++ty) {
    const int y0 = ty * TR;
    unsigned mx = 0u;
#pragma unroll
    for (int pl = 0; pl < NG; ++pl)
#pragma unroll
      for (int k = 0; k < NLD; ++k)
        mx = amax_fold(amax_fold(amax_fold(amax_fold(mx, hv[pl][k].x), hv[pl][k].y), hv[pl][k].z), hv[pl][k].w);
#pragma unroll
    for (int o = 32; o; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
    if (lane == 0) s_max[wave] = mx;
    __syncthreads();  // s_max complete; every wave is done with the previous tile's halo
    const Prescale ps = prescale_from_max(max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3])));
#pragma unroll
    for (int pl = 0; pl < NG; ++pl)
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        const int i = tid + k * 256;
        if (i >= HR * C4) continue;
        const float v[4] = {hv[pl][k].x * ps.s, hv[pl][k].y * ps.s, hv[pl][k].z * ps.s, hv[pl][k].w * ps.s};
        uint32_t d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const _Float16 h = (_Float16)v[j], l = (_Float16)(v[j] - (float)h);
          d[j] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
        }
        const int row = i / C4, c4 = i - row * C4;
        *reinterpret_cast<uint4*>(halo + pl * PLANE + row * PITCH + 4 * c4) = make_uint4(d[0], d[1], d[2], d[3]);
      }
    if (ty + 1 < ty1) hload(y0 + TR);
    __syncthreads();  // the halo is in LDS

    // wave w: row pairs w and w + 4 of the tile, 4 column groups of 16 each
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int cg = 0; cg < 4; ++cg) {
        const uint32_t* hb = halo + 8 * u * PITCH + 16 * cg;
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          uint32_t d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = hb[boff[c][e / NGP] + (e % NGP % NG) * PLANE];
          F16Pair bf;
          uint32_t h[4], l[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            h[j] = __builtin_amdgcn_perm(d[2 * j + 1], d[2 * j], 0x05040100u);  // low halves: hi pieces
            l[j] = __builtin_amdgcn_perm(d[2 * j + 1], d[2 * j], 0x07060302u);  // high halves: lo pieces
          }
          bf.h = make_uint4(h[0], h[1], h[2], h[3]);
          bf.l = make_uint4(l[0], l[1], l[2], l[3]);
          mma_split32(A[c], bf, acc);
        }
        const int oy = y0 + 2 * (wave + 4 * u) + orow, ox = x0 + 16 * cg + n;
        if (oy < a.Ho && ox < a.Wo && co < a.cout) {
          float r[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = acc[i] * ps.inv * pw.inv + bias[i];  // two exact scalings (no underflow)
          tail4<T>(a, b, oy, ox, co, r);
        }
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

// conv2d_planes_mfma_kernel's conditions (on top of planes_fast_ok): cout 4 or 8, whole 16-byte plane pieces, 32-bit
// byte offsets
bool planes_mfma_ok(const Conv2dArgs& a) {
  const char* v = getenv("DAMVS_PLANES_MFMA");
  if ((v && v[0] == '0') || (a.cout != 4 && a.cout != 8) || a.Wi % 4 || a.Wo != a.Wi || a.Ho != a.Hi) return false;
  for (int g = 0; g < a.ngeo; ++g)
    if (reinterpret_cast<uintptr_t>(a.geo[g]) % 16 || a.geo_bstride[g] % 4 ||
        ((long long)(a.B - 1) * a.geo_bstride[g] + (long long)a.Hi * a.Wi) * 4 >= (1LL << 31))
      return false;
  return (long long)a.B * a.Ho * a.Wo * a.cout < (1LL << 31);
}

template <typename T, int K>
hipError_t launch_planes_mfma_k(hipStream_t st, const Conv2dArgs& a) {
  const int tx = (a.Wo + 63) / 64, ty = (a.Ho + 15) / 16;
  // tiles per block (DAMVS_PLANES_NT, read per call, 1-16; default 4: FeatureNet's RGB conv x20 / GeoFF RGB+depth /
  // depth init at B=4, bf16, 405 / 117 / 73 us at 1 tile, 354 / 99 / 62 at 2, 326 / 93 / 59 at 4, 324 / 92 / 59 at 8,
  // profiles/r06/ab_planes_mfma)
  const char* v = getenv("DAMVS_PLANES_NT");
  int nt = v && v[0] ? atoi(v) : 4;
  nt = nt < 1 ? 1 : nt > 16 ? 16 : nt;
  const dim3 grid((unsigned)(tx * ((ty + nt - 1) / nt) * a.B));
  switch (a.ngeo) {
    case 1: hipLaunchKernelGGL((conv2d_planes_mfma_kernel<T, K, 1>), grid, dim3(256), 0, st, a, tx, ty, nt); break;
    case 2: hipLaunchKernelGGL((conv2d_planes_mfma_kernel<T, K, 2>), grid, dim3(256), 0, st, a, tx, ty, nt); break;
    case 3: hipLaunchKernelGGL((conv2d_planes_mfma_kernel<T, K, 3>), grid, dim3(256), 0, st, a, tx, ty, nt); break;
    default: hipLaunchKernelGGL((conv2d_planes_mfma_kernel<T, K, 4>), grid, dim3(256), 0, st, a, tx, ty, nt); break;
  }
  return hipGetLastError();
}

// Returns hipErrorNotSupported when the layer is not of the fast form (caller uses the MFMA kernel).
template <typename T>
hipError_t launch_planes(hipStream_t st, const Conv2dArgs& a) {
  const int K = a.ph[0].ntaps == 9 ? 3 : a.ph[0].ntaps == 25 ? 5 : 0;
  if (K == 0 || a.ngeo < 1 || a.ngeo > 4 || a.cout > 16 || a.cout_pad < 16 || !planes_fast_ok(a, K))
    return hipErrorNotSupported;
  if (planes_mfma_ok(a)) return K == 3 ? launch_planes_mfma_k<T, 3>(st, a) : launch_planes_mfma_k<T, 5>(st, a);
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
