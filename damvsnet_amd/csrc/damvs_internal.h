// Internal declarations shared by the HIP kernels and the C-ABI layer (not installed).
//
// Layouts (all device, row-major, innermost last):
//   features  [B][h][w][C]            (NHWC, T = float | bf16)
//   volume    [B][D][h][w][C]         (NDHWC, T)
//   hyps      [B][D][h][w]            float
//   rt        [B][N-1][12]            float: R row-major (9) then t (3) of P_src * inv(P_ref)
//   logits    [B][D][h][w]            float
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace damvs {

typedef uint16_t bf16_t;  // bf16 storage (upper half of an IEEE f32)

enum StoreType { ST_F32 = 0, ST_BF16 = 1 };
enum AggMode { AGG_ADAPTIVE = 0, AGG_VARIANCE = 1, AGG_WARP_ONLY = 2 };

constexpr int kMaxViews = 16;
// magnitude slots of the fp32 prescale (damvs_device.h prescale_of; include/damvs.h DAMVS_AMAX_SLOT_BYTES)
constexpr int kAmaxReps = 32;    // replicas per slot (one 128-byte line each): atomics spread over 32 addresses
constexpr int kAmaxStride = 32;  // words between replicas
constexpr int kAmaxSlotWords = kAmaxReps * kAmaxStride;
constexpr int kMaxPhases = 8;

// ---------------------------------------------------------------- warp + aggregation
struct WarpArgs {
  const void* feats[kMaxViews];  // N views, view 0 = reference
  const float* rt;               // [B][N-1][12]
  const float* hyps;             // [B][D][out_rows][w]
  void* out;                     // [B][D][out_rows][w][C]
  int B, N, C, D, h, w;          // h x w: the feature maps (and the full reference image grid)
  int y0, rows;                  // computed: reference rows [y0, y0 + rows) (0, h: the whole image) ...
  int out_rows, out_y;           // ... at rows [out_y, out_y + rows) of the hyps / out planes
  // adaptive weight net, BN folded: a = relu(sum_c k1[c] x_c * s1 + t1); wt = relu(a * s2 + t2)
  float k1[32];
  float s1, t1, s2, t2;
  // pixel-block shape (set by the warp launcher): tile_r = 0 -> a block is ppb consecutive pixels of the row-major
  // computed rows; else a tile of tile_r rows x ppb / tile_r columns, tiles dealt strip by strip (tile_sw tiles wide,
  // top to bottom), so the blocks in flight on one XCD cover a compact 2D region of the reference image
  int tile_r, tile_sw, tiles_x;
  unsigned* out_amax;  // fp32: magnitude slots of the written volume, one per batch element (prescale_of), or nullptr
};

// n / d for 0 <= n < 2^31 without a hardware divide: q = (umulhi(n, mul) + n) >> shift.
struct FastDiv {
  uint32_t mul, shift;
  int d;
};
inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  f.d = d;
  uint32_t sh = 0;
  while (sh < 31 && (1u << sh) < (uint32_t)d) ++sh;
  f.shift = sh;
  f.mul = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << sh) - (uint64_t)d)) / (uint64_t)d + 1);
  return f;
}
#ifdef __HIPCC__
__device__ __forceinline__ int fdiv(const FastDiv& f, int n) {
  return (int)((__umulhi((uint32_t)n, f.mul) + (uint32_t)n) >> f.shift);
}
#endif

// ---------------------------------------------------------------- MFMA implicit-GEMM conv3d
// A "phase" is one regular sub-convolution: for an iteration-grid point q,
//   input  coord = q * in_stride + tap_offset        (zero outside the input)
//   output coord = q * out_stride + (pd, ph, pw)
// Conv3d k3 s1/s2 has one phase with 27 taps; ConvTranspose3d k3 s2 p1 op1 is 8 phases of
// 1..8 taps each (sub-pixel decomposition), so no MFMA work is spent on structural zeros.
struct ConvPhase {
  int ntaps, kchunks, w_off, pd, ph, pw;
  signed char tap[27][4];  // dz, dy, dx, (pad)
};

struct ConvArgs {
  const void* in;
  void* out;
  const void* resid;   // added after ReLU (may alias out); nullptr if none
  const void* wpack;   // packed A fragments, see pack_conv_weights()
  const void* wpack_pair;  // row-pair packing (stride-1, Cout <= 8), nullptr if none
  const void* wpack32;     // fp32: the z-streamed kernel's packing of this layer, 32 K per chunk, split-f16
  const void* wgat32;      // fp32: the gather kernel's packing at 32 K per chunk (split-f16; phases of build_phases(., 32))
                           // [chunk][hi: 64 lanes][lo: 64 lanes] (x-pair for conv11, row pairs for conv0), or nullptr
  const float* bias;   // [Cout] (folded BN shift)
  int B, Cin, Cout, MT;
  int Di, Hi, Wi;
  int Dq, Hq, Wq;
  int Do, Ho, Wo;
  int in_stride, out_stride;
  int relu;
  int nphase;
  int xpair;  // deconv phases are (pz, py) with both x parities in the MFMA rows (Cout <= 8)
  float wscale;  // accumulator scale of the epilogue: 2^-k of the split-f16 fp32 weights (damvs_device.h), 1 for bf16
  FastDiv div_wq, div_hq, div_dq;  // set by launch_conv3d
  ConvPhase ph[kMaxPhases];
  // fp32: the phases of wgat32 (build_phases(., 32) at layer creation): K chunks and weight offsets at 32 K per chunk
  // (the taps are those of ph)
  int k32_chunks[kMaxPhases], k32_off[kMaxPhases];
  // fp32 activation prescale (damvs_device.h prescale_of): the input tensor's magnitude slots (nullptr: unscaled) and
  // the slots this layer's stored outputs are recorded into (nullptr: not recorded), one slot (kAmaxSlotWords words)
  // per batch element: a sample's scales do not depend on the rest of its batch; bf16 ignores both
  const unsigned* in_amax;
  unsigned* out_amax;
};

// ---------------------------------------------------------------- 2D front-end convolutions
// One phase of a 2D conv / transposed conv: input = q * in_stride + tap offset, output =
// q * out_stride + (py, px). Weights for the tensor inputs are packed like the 3D kernel's
// (A-fragment order, K = taps x (c0 + c1)); geometry-plane weights are fp32 [tap][g][cout_pad].
struct Conv2dPhase {
  int ntaps, kchunks, gchunks, w_off, g_off, py, px;  // kchunks: tensor-input K chunks; gchunks: plane K chunks
  signed char tap[25][2];  // dy, dx (up to 5 x 5)
  signed char wtap[25];    // weight tap index ky*k + kx
  signed char pad_[3];
};

struct Conv2dArgs {
  const void* in0;
  const void* in1;
  int c0, c1;
  const float* geo[4];      // planar fp32 [B][Hi][Wi] planes at the input resolution
  long long geo_bstride[4]; // elements between batches of each geo plane
  int ngeo;
  const void* wpack;
  const float* wgeo;
  const float* bias;        // [cout_pad]
  const void* res_pre;      // added before ReLU, [B][Ho][Wo][cout]
  const void* res_post;     // added after ReLU, [B][Ho/up][Wo/up][cout]
  int post_up;
  void* out;                // [B][Ho][Wo][cout]
  int cout, cout_pad, MTtot;
  int B, Hi, Wi, Hq, Wq, Ho, Wo, in_stride, out_stride, relu, nphase;
  FastDiv div_wq, div_hq;   // output-grid decomposition q -> (b, qy, qx)
  int xpair;                // transposed stride 2, cout 8: both x parities in one phase's 16 MFMA rows
  float wscale;             // accumulator scale of the epilogue (see ConvArgs)
  int wide32;               // fp32: ph / wpack are the 32-K split packing of conv2d_wide_kernel<float>
  Conv2dPhase ph[4];
};

// ---------------------------------------------------------------- launchers (return hipError_t)
hipError_t launch_proj_prepare(hipStream_t s, int B, int N, const float* proj, float* rt);
// status[0] = 1 when any of the n floats of a, b or c is non-finite (sticky: damvs_stage_status clears it)
hipError_t launch_finite_check(hipStream_t s, const float* a, const float* b, const float* c, long long n, int* status);
// fold max |x| of n floats into a magnitude slot (damvs_device.h prescale_of)
hipError_t launch_amax(hipStream_t s, const float* x, long long n, unsigned* slot);
hipError_t launch_hyp_linear(hipStream_t s, int B, int D, int h, int w, const float* dv, int Dv, float* out);
hipError_t launch_hyp_refine(hipStream_t s, int B, int D, int H, int W, int scale, const float* pd,
                             const float* pv, int hp, int wp, float* out);
hipError_t launch_sparse_pyramid(hipStream_t s, int B, int h, int w, const float* depth, const float* dv, int Dv,
                                 const float* mask, float* d0, float* d1, float* d2, float* d3, float* m1, float* m2);
struct FeatPtrs {
  const void* p[kMaxViews];
};
// blocked = features in channel-blocked layout [B][C/E][h][w][E] (E = 16 bytes of channels)
hipError_t launch_warp_aggregate(hipStream_t s, int store, int mode, const WarpArgs& a, bool blocked);
bool warp_split_for(int bytes, int N);  // the channel-split warp serves NHWC maps of these pixels at N views
hipError_t launch_block_channels(hipStream_t s, int store, const FeatPtrs& src, const FeatPtrs& dst, int N, int B,
                                 int hw, int C);
hipError_t launch_conv3d(hipStream_t s, int store, const ConvArgs& a);
hipError_t launch_conv2d(hipStream_t s, int store, const Conv2dArgs& a);
bool conv2d_wide_shape_ok(const Conv2dArgs& a);
// layers whose only inputs are fp32 planes (c0 = c1 = 0), on the VALU (k_planes.hip)
hipError_t launch_conv2d_planes(hipStream_t s, int store, const Conv2dArgs& a);  // the wide kernel takes the layer (given 32-K phase data)
struct BorderArgs {
  float corr[9 * 16];  // [tap][channel] of a 3x3 conv, channels < 16
};
hipError_t launch_fpn_top(hipStream_t s, int store, int B, int H, int W, const void* c0, const void* f,
                          const void* apack, float wscale, const float* bias, void* out);
hipError_t launch_border_bias(hipStream_t s, int store, const BorderArgs& a, int B, int H, int W, int cstored, int cout,
                              void* out);
// ---------------------------------------------------------------- depth fusion (filter/dypcd.py)
constexpr int kFusionMaxSrc = 10;  // the reference's masks run to i = 10 (dypcd.py:152)
struct FusionCam {
  float t_sr[16], k_src[9], kinv_src[9], t_rs[16];  // E_src inv(E_ref), K_src, inv(K_src), E_ref inv(E_src)
};
struct FusionArgs {
  int H, W, nsrc;
  const float* depth_ref;
  const float* depth_src[kFusionMaxSrc];
  const float* conf[3];  // final, stage-2, stage-1 confidences (nullptr: photometric test off)
  float conf_thr[3];     // args.conf: stage-1, stage-2, stage-3 thresholds
  float kinv_ref[9], k_ref[9], einv_ref[16];
  FusionCam src[kFusionMaxSrc];
  double dist_thr[9];    // i * dist_base, i = 2..10
  float rel_thr[9];      // float32(i * rel_diff_base)
  float* depth_avg;
  unsigned char* mask;   // bit 0 photo, bit 1 geo, bit 2 final
  float* xyz;            // world points of final pixels (0 elsewhere), or nullptr
};
hipError_t launch_fusion_view(hipStream_t s, const FusionArgs& a);

bool conv_lds_disabled();  // DAMVS_CONV_NO_LDS=1 selects the global-gather conv kernel (A/B testing)
bool conv_xpair_disabled();  // x-pair deconv phases only with DAMVS_CONV_XPAIR=1
hipError_t launch_prob_conv(hipStream_t s, int store, int B, int Cb, int D, int h, int w, const void* feat,
                            const float* wprob, const float* prob_init, float* logits);
hipError_t launch_prob_regress(hipStream_t s, int store, int B, int Cb, int D, int h, int w, const void* feat,
                               const float* wprob, const float* prob_init, const float* hyps, float* depth,
                               float* conf, float* var, float* prob);
size_t prob_regress_smem_bytes(int store, int Cb, int D);
// MFMA prob conv + regression (bf16 storage, base 8; LDS bounds D): apack from pack_prob_rows (capi.cpp)
#ifndef DAMVS_PROB_TERMS
#define DAMVS_PROB_TERMS 2  // bf16 terms per fp32 prob-conv weight (3: exact fp32 weights; A/B builds)
#endif
constexpr int kProbRowChunks = 5, kProbRowTerms = DAMVS_PROB_TERMS;  // prob_mfma_kernel: 18 voxel slots x 8 channels
// store ST_F32: the split-f16 form (apack = damvs_stage prob_split, pscale its 2^-k)
hipError_t launch_prob_mfma(hipStream_t s, int store, int B, int D, int h, int w, const void* feat, const void* apack,
                            float pscale, const float* prob_init, const float* hyps, float* depth, float* conf,
                            float* var, float* prob);
size_t prob_mfma_smem(int store, int D);
bool prob_mfma_disabled();  // DAMVS_PROB_MFMA=0 (A/B testing)
bool prob_mfma_enabled(int store);  // bf16 unless DAMVS_PROB_MFMA=0; fp32 only with DAMVS_PROB_MFMA=1
hipError_t launch_regress(hipStream_t s, int B, int D, int h, int w, const float* logits, const float* hyps,
                          float* depth, float* conf, float* var, float* prob);


}  // namespace damvs
