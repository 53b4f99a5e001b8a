// Final probability conv + depth regression.
//
//  prob_conv : CostRegNet.prob, Conv3d(base, 1, k3, p1, bias=False) (models/module.py:530,540).
//              One thread per pixel column (b, y, x) slides over the D planes: each input plane's
//              3x3 x Cb neighbourhood is loaded once and contributes to logits d-1, d, d+1
//              (3x fewer loads than a per-output gather). Optional prob_volume_init is added
//              (models/cas_mvsnet.py:107-108).
//  regress   : softmax over D (:110), depth = sum p*d (module.py:609-615), photometric
//              confidence = sum of p over [i*-1, i*+2] at i* = clamp(long(sum p*i), 0, D-1)
//              (:113-118, the 4*avg_pool3d of the padded volume), exp-variance
//              3*sqrt(sum (d - depth)^2 p) (:121-124); optional prob volume write.
#include "damvs_device.h"

namespace damvs {

namespace {

template <typename T, int CB>
__global__ __launch_bounds__(256) void prob_conv_kernel(int B, int D, int h, int w, const T* __restrict__ feat,
                                                        const float* __restrict__ wprob,
                                                        const float* __restrict__ prob_init,
                                                        float* __restrict__ logits) {
  __shared__ float sw[27 * CB];  // [kd][kh][kw][c]
  for (int i = threadIdx.x; i < 27 * CB; i += blockDim.x) sw[i] = wprob[i];
  __syncthreads();
  const int hw = h * w;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= hw) return;
  const int y = p / w, x = p - y * w;
  float am1 = 0.f, a0 = 0.f;  // partial logits for d = plane-1 (after this plane) and d = plane+1
  for (int pl = 0; pl < D; ++pl) {
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;  // kd = 0 -> d = pl+1, kd = 1 -> d = pl, kd = 2 -> d = pl-1
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = y + ky - 1;
      if (yy < 0 || yy >= h) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = x + kx - 1;
        if (xx < 0 || xx >= w) continue;
        float v[CB];
        load_vec<T, CB>(feat + ((((size_t)b * D + pl) * h + yy) * w + xx) * CB, v);
        const float* w0 = sw + ((0 * 3 + ky) * 3 + kx) * CB;
        const float* w1 = sw + ((1 * 3 + ky) * 3 + kx) * CB;
        const float* w2 = sw + ((2 * 3 + ky) * 3 + kx) * CB;
#pragma unroll
        for (int c = 0; c < CB; ++c) {
          c0 += w0[c] * v[c];
          c1 += w1[c] * v[c];
          c2 += w2[c] * v[c];
        }
      }
    }
    float* lo = logits + ((size_t)b * D) * hw + p;
    if (pl >= 1) {
      float l = am1 + c2;
      if (prob_init) l += prob_init[((size_t)b * D + pl - 1) * hw + p];
      lo[(size_t)(pl - 1) * hw] = l;
    }
    am1 = a0 + c1;
    a0 = c0;
  }
  float l = am1;
  if (prob_init) l += prob_init[((size_t)b * D + D - 1) * hw + p];
  logits[((size_t)b * D + D - 1) * hw + p] = l;
}

__global__ __launch_bounds__(256) void regress_kernel(int B, int D, int hw, const float* __restrict__ logits,
                                                      const float* __restrict__ hyps, float* __restrict__ depth,
                                                      float* __restrict__ conf, float* __restrict__ var,
                                                      float* __restrict__ prob) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= hw) return;
  const float* lg = logits + (size_t)b * D * hw + p;
  const float* hy = hyps + (size_t)b * D * hw + p;
  float mx = -INFINITY;
  for (int d = 0; d < D; ++d) mx = fmaxf(mx, lg[(size_t)d * hw]);
  float sum = 0.f;
  for (int d = 0; d < D; ++d) sum += expf(lg[(size_t)d * hw] - mx);
  float dep = 0.f, idx = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = expf(lg[(size_t)d * hw] - mx) / sum;
    dep += pr * hy[(size_t)d * hw];
    idx += pr * (float)d;
    if (prob) prob[((size_t)b * D + d) * hw + p] = pr;
  }
  int ii = (int)idx;  // .long() truncation; idx >= 0
  ii = ii < 0 ? 0 : (ii > D - 1 ? D - 1 : ii);
  float c = 0.f, vs = 0.f;
  for (int d = 0; d < D; ++d) {
    const float pr = expf(lg[(size_t)d * hw] - mx) / sum;
    const float df = hy[(size_t)d * hw] - dep;
    vs += df * df * pr;
    if (d >= ii - 1 && d <= ii + 2) c += pr;
  }
  depth[(size_t)b * hw + p] = dep;
  conf[(size_t)b * hw + p] = c;
  var[(size_t)b * hw + p] = 3.f * sqrtf(vs);
}

template <typename T>
hipError_t launch_pc(hipStream_t s, int B, int Cb, int D, int h, int w, const void* feat, const float* wprob,
                     const float* prob_init, float* logits) {
  dim3 grid((h * w + 255) / 256, B);
  const T* f = reinterpret_cast<const T*>(feat);
  switch (Cb) {
    case 8: hipLaunchKernelGGL((prob_conv_kernel<T, 8>), grid, dim3(256), 0, s, B, D, h, w, f, wprob, prob_init, logits); break;
    case 16: hipLaunchKernelGGL((prob_conv_kernel<T, 16>), grid, dim3(256), 0, s, B, D, h, w, f, wprob, prob_init, logits); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_prob_conv(hipStream_t s, int store, int B, int Cb, int D, int h, int w, const void* feat,
                            const float* wprob, const float* prob_init, float* logits) {
  return store == ST_BF16 ? launch_pc<bf16_t>(s, B, Cb, D, h, w, feat, wprob, prob_init, logits)
                          : launch_pc<float>(s, B, Cb, D, h, w, feat, wprob, prob_init, logits);
}

hipError_t launch_regress(hipStream_t s, int B, int D, int h, int w, const float* logits, const float* hyps,
                          float* depth, float* conf, float* var, float* prob) {
  int hw = h * w;
  hipLaunchKernelGGL(regress_kernel, dim3((hw + 255) / 256, B), dim3(256), 0, s, B, D, hw, logits, hyps, depth, conf,
                     var, prob);
  return hipGetLastError();
}

}  // namespace damvs
