// Dynamic-consistency depth fusion for one reference view (SURVEY.md section 8(f) row f4;
// filter/dypcd.py:98-297): for every pixel, every source view's depth is reprojected through the
// reference depth (ref pixel -> 3D -> source pixel -> bilinear source depth -> 3D -> ref pixel),
// masks count the views that agree within i * dist_base pixels and i * rel_diff_base relative depth
// (i = 2..10), the agreeing reprojected depths are averaged with the reference depth, and pixels
// passing the photometric (three confidences) and dynamic geometric tests are lifted to world points.
//
// One thread per reference pixel walks the source views; no intermediate per-view map reaches HBM
// (the reference materialises ~12 full-resolution float64 arrays per source view). Arithmetic
// follows the reference's numpy dtypes: projections in float64 with the camera products formed in
// float32 on the host (as numpy does for float32 matrices), float32 where the reference casts
// (source coordinates, reprojected depth and coordinates, relative depth test), the source-depth
// lookup as cv2.remap INTER_LINEAR (1/32-pixel fixed-point coordinates, float weight table,
// zero border), with explicit round-to-nearest float ops (no FMA contraction) on that path.
#include "damvs_device.h"

namespace damvs {

namespace {

__device__ __forceinline__ float remap_linear(const float* __restrict__ src, int H, int W, float mx, float my) {
  // cv2: X = cvRound(mx * 32), sx = X >> 5, fx = (X & 31) / 32 (INTER_BITS = 5)
  const float X = rintf(__fmul_rn(mx, 32.f)), Y = rintf(__fmul_rn(my, 32.f));
  if (!(X > -2147483648.f && X < 2147483520.f && Y > -2147483648.f && Y < 2147483520.f)) return 0.f;
  const int xi = (int)X, yi = (int)Y;
  const int sx = min(max(xi >> 5, -32768), 32767), sy = min(max(yi >> 5, -32768), 32767);
  if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) return 0.f;
  const float fx = __fmul_rn((float)(xi & 31), 0.03125f), fy = __fmul_rn((float)(yi & 31), 0.03125f);
  const float cx0 = __fsub_rn(1.f, fx), cy0 = __fsub_rn(1.f, fy);
  const float w[4] = {__fmul_rn(cy0, cx0), __fmul_rn(cy0, fx), __fmul_rn(fy, cx0), __fmul_rn(fy, fx)};
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = sx + (k & 1), yy = sy + (k >> 1);
    v[k] = (xx >= 0 && xx < W && yy >= 0 && yy < H) ? src[(size_t)yy * W + xx] : 0.f;
  }
  return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(v[0], w[0]), __fmul_rn(v[1], w[1])), __fmul_rn(v[2], w[2])),
                   __fmul_rn(v[3], w[3]));
}

// 3x3 (row-major, float32 -> double) times a double 3-vector
__device__ __forceinline__ void mv3(const float* m, const double* v, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
    o[i] = (double)m[3 * i] * v[0] + (double)m[3 * i + 1] * v[1] + (double)m[3 * i + 2] * v[2];
}
// rows 0-2 of a 4x4 (float32 -> double) times (v, 1)
__device__ __forceinline__ void mv34(const float* m, const double* v, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
    o[i] = (double)m[4 * i] * v[0] + (double)m[4 * i + 1] * v[1] + (double)m[4 * i + 2] * v[2] + (double)m[4 * i + 3];
}

__global__ __launch_bounds__(256) void fusion_view_kernel(const FusionArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.H * a.W) return;
  const int y = p / a.W, x = p - y * a.W;
  const float dref = a.depth_ref[p];
  const double v0[3] = {(double)x * (double)dref, (double)y * (double)dref, (double)dref};
  double xyz_ref[3];
  mv3(a.kinv_ref, v0, xyz_ref);
  float sum_rep = 0.f;
  int geo_sum = 0;
  int geo_sums[9];  // views passing the mask at i = 2..10
#pragma unroll
  for (int i = 0; i < 9; ++i) geo_sums[i] = 0;
  for (int v = 0; v < a.nsrc; ++v) {
    const FusionCam& c = a.src[v];
    double xs[3], kxs[3];
    mv34(c.t_sr, xyz_ref, xs);
    mv3(c.k_src, xs, kxs);
    const double xsd = kxs[0] / kxs[2], ysd = kxs[1] / kxs[2];
    const float sampled = remap_linear(a.depth_src[v], a.H, a.W, (float)xsd, (float)ysd);
    const double v1[3] = {xsd * (double)sampled, ysd * (double)sampled, (double)sampled};
    double xs2[3], xr[3], kxr[3];
    mv3(c.kinv_src, v1, xs2);
    mv34(c.t_rs, xs2, xr);
    const float depth_rep = (float)xr[2];
    mv3(a.k_ref, xr, kxr);
    if (kxr[2] == 0.0) kxr[2] += 0.00001;
    const float xrep = (float)(kxr[0] / kxr[2]), yrep = (float)(kxr[1] / kxr[2]);
    const double dx = (double)xrep - (double)x, dy = (double)yrep - (double)y;
    const double dist = sqrt(dx * dx + dy * dy);
    const float rel = __fdiv_rn(fabsf(__fsub_rn(depth_rep, dref)), dref);
    // masks i = 2..10; the i = 10 one gates the average (filter/dypcd.py:152-157, 219-225)
#pragma unroll
    for (int i = 2; i <= 10; ++i) {
      const bool m = dist < a.dist_thr[i - 2] && rel < a.rel_thr[i - 2];
      if (i - 2 < a.nsrc - 1) geo_sums[i - 2] += m;
      if (i == 10 && m) {
        ++geo_sum;
        sum_rep = __fadd_rn(sum_rep, depth_rep);
      }
    }
  }
  // (sum of reprojected depths + ref) / (count + 1): float32 sum, float64 division (int32 promotes)
  const double davg = (double)__fadd_rn(sum_rep, dref) / (double)(geo_sum + 1);
  bool geo = geo_sum >= a.nsrc + 1;
#pragma unroll
  for (int i = 2; i <= 10; ++i) geo = geo || (i <= a.nsrc && geo_sums[i - 2] >= i);
  bool photo = true;
  if (a.conf[0]) photo = a.conf[0][p] > a.conf_thr[2] && a.conf[1][p] > a.conf_thr[1] && a.conf[2][p] > a.conf_thr[0];
  const bool fin = photo && geo;
  a.depth_avg[p] = (float)davg;
  a.mask[p] = (unsigned char)((photo ? 1 : 0) | (geo ? 2 : 0) | (fin ? 4 : 0));
  if (a.xyz) {
    float o[3] = {0.f, 0.f, 0.f};
    if (fin) {
      const double v2[3] = {(double)x * davg, (double)y * davg, davg};
      double cam[3], w[3];
      mv3(a.kinv_ref, v2, cam);
      mv34(a.einv_ref, cam, w);
      o[0] = (float)w[0]; o[1] = (float)w[1]; o[2] = (float)w[2];
    }
    a.xyz[3 * (size_t)p] = o[0];
    a.xyz[3 * (size_t)p + 1] = o[1];
    a.xyz[3 * (size_t)p + 2] = o[2];
  }
}

}  // namespace

hipError_t launch_fusion_view(hipStream_t s, const FusionArgs& a) {
  const long long n = (long long)a.H * a.W;
  hipLaunchKernelGGL(fusion_view_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace damvs
