/* damvs.h — C ABI of the MI355X cascade-MVS cost-volume engine (libdamvs.so).
 *
 * Drop-in boundary for the per-stage hot path of wsmtht520/DAMVSNet. The reference has no
 * native/FFI layer; its boundary is the Python module API, which the
 * package damvsnet_amd mirrors on top of this ABI. Each entry point names the reference
 * interface it replaces (paths relative to the reference repo).
 *
 * Conventions
 *   - Plain C types only. Tensor arguments are DEVICE pointers owned by the caller; parameter
 *     structs passed to damvs_stage_create are HOST pointers (copied, BN-folded, packed).
 *   - No allocation, no host synchronisation inside the *_forward / kernel entry points: work is
 *     enqueued on `stream` (a hipStream_t, NULL = default stream) and is graph-capturable.
 *   - Return 0 (DAMVS_OK) or a negative DAMVS_E_* code; damvs_last_error_string() gives the
 *     message of the last failure on the calling thread.
 *   - A damvs_stage is immutable after create and may be used concurrently from several threads
 *     on different streams (workspaces must differ).
 *   - Layouts: features NHWC [B][h][w][C]; cost volume NDHWC [B][D][h][w][C]; hypotheses,
 *     logits and probabilities [B][D][h][w] float; projections [B][N][2][4][4] float with
 *     [..,0,:,:] the world->camera extrinsic and [..,1,:3,:3] the stage intrinsics
 *     (datasets/general_eval.py:158-175).
 */
#ifndef DAMVS_H
#define DAMVS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAMVS_ABI_VERSION 1

enum {
  DAMVS_OK = 0,
  DAMVS_E_ARG = -1,       /* null pointer / bad enum */
  DAMVS_E_SHAPE = -2,     /* unsupported or inconsistent shape */
  DAMVS_E_DTYPE = -3,     /* unsupported storage type */
  DAMVS_E_HIP = -4,       /* HIP runtime error */
  DAMVS_E_NOMEM = -5,     /* device allocation failed (create only) */
  DAMVS_E_WORKSPACE = -6, /* workspace too small */
  DAMVS_E_RANGE = -7      /* non-finite depth / confidence / variance (damvs_stage_status) */
};

enum { DAMVS_F32 = 0, DAMVS_BF16 = 1 };                       /* storage of features / volumes */
enum { DAMVS_AGG_ADAPTIVE = 0, DAMVS_AGG_VARIANCE = 1 };      /* models/cas_mvsnet.py:11-16 */

/* BatchNorm in eval form: y = (x - running_mean) / sqrt(running_var + eps) * weight + bias. */
typedef struct {
  const float* weight;
  const float* bias;
  const float* running_mean;
  const float* running_var;
  float eps;
} damvs_bn;

/* CostRegNet (models/module.py:510-541). conv_weight[i] for i = 0..9 is
 * conv0..conv6 (Conv3d, [Cout][Cin][3][3][3]) then conv7, conv9, conv11
 * (ConvTranspose3d, [Cin][Cout][3][3][3]); bn[i] the matching BatchNorm3d;
 * prob_weight is prob.weight [1][base][3][3][3] (no bias, no BN). */
typedef struct {
  int in_channels;
  int base_channels;
  const float* conv_weight[10];
  damvs_bn bn[10];
  const float* prob_weight;
} damvs_costreg_params;

/* AggWeightNetVolume (models/module.py:544-563): w_net.0 = Conv3d(C,1,1)+BN+ReLU (w1 is [C]),
 * w_net.1 = Conv3d(1,1,1)+BN+ReLU (w2 is [1]). conv0 is unused by the reference forward. */
typedef struct {
  int in_channels;
  const float* w1;
  damvs_bn bn1;
  const float* w2;
  damvs_bn bn2;
} damvs_aggweight_params;

typedef struct damvs_stage damvs_stage;

int damvs_abi_version(void);
const char* damvs_last_error_string(void);
/* Provenance: sha256 (hex, first 16 digits) of the sources, headers and compiler flags this library was built
 * from (damvsnet_amd/build.py), "unstamped" for builds outside build.py. The Python binding compares it with the
 * sources next to it and refuses a stale library. */
const char* damvs_build_id(void);

/* One cascade stage's weights (replaces DepthNet.weight_net[s] + cost_regularization[s],
 * models/cas_mvsnet.py:16,180-182). `aggw` may be NULL for DAMVS_AGG_VARIANCE. Uses the
 * current HIP device. */
int damvs_stage_create(const damvs_costreg_params* costreg, const damvs_aggweight_params* aggw, int agg_mode,
                       int dtype, damvs_stage** out);
int damvs_stage_destroy(damvs_stage* st);

/* Bytes of device workspace damvs_stage_forward needs for this problem size. */
int damvs_stage_workspace_size(const damvs_stage* st, int B, int N, int D, int h, int w, size_t* bytes);

/* DepthNet.forward (models/cas_mvsnet.py:18-134) for one stage: warp + aggregation,
 * CostRegNet, softmax regression, confidence, exp-variance.
 *   feats[N]  : N device pointers (host array), view 0 = reference, each [B][h][w][C] of dtype
 *   proj      : [B][N][2][4][4]      hyps: [B][D][h][w]      prob_init: NULL or [B][D][h][w]
 *   depth, conf, var : [B][h][w]     prob: NULL or [B][D][h][w] (prob_volume output)
 * D, h, w must be multiples of 8 (three stride-2 levels, models/module.py:515-528). */
int damvs_stage_forward(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                        const void* const* feats, const float* proj, const float* hyps, const float* prob_init,
                        void* workspace, size_t workspace_bytes, float* depth, float* conf, float* var,
                        float* prob);

/* Range status of the damvs_stage_forward calls that used `workspace` since the previous damvs_stage_status on it
 * (synchronises `stream`, the stream they ran on, then clears the status): DAMVS_OK, or DAMVS_E_RANGE when any depth,
 * confidence or variance value one of them wrote is non-finite. The status is the workspace's first 4 bytes: zero them
 * when the workspace is allocated (hipMemset), or call damvs_stage_status once before the first forward and ignore the
 * result. Why it exists: the fp32 path computes every conv product on split-f16 MFMAs (x = f16 hi + f16 lo), so an
 * activation of magnitude >= 65520 (beyond the f16 range) turns into NaN there; ReLU keeps NaN as torch.relu does, and
 * the stage's outputs carry it. The forward itself never synchronises (its last kernel checks the three output maps
 * and sets the status); damvsnet_amd asks once per CascadeMVSNet.forward. The reference's fp32 convolutions have no
 * such limit (the volume of models/cas_mvsnet.py:64-76 is the first tensor that can reach it). */
int damvs_stage_status(const damvs_stage* st, void* stream, const void* workspace, size_t workspace_bytes);

/* damvs_stage_forward with in-pipeline timing probes: events (NULL, or 4 hipEvent_t, any may be NULL) are
 * recorded on `stream` before the warp + aggregation launch, after it, after the U-Net and after the
 * regression -- the per-kernel-group durations of the stage as the product runs it (bench.py roofline). */
int damvs_stage_forward_probed(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                               const void* const* feats, const float* proj, const float* hyps, const float* prob_init,
                               void* workspace, size_t workspace_bytes, float* depth, float* conf, float* var,
                               float* prob, void* const* events);

/* ---- split entry points (used by the parity tests and by sharded execution) ---- */

/* Per (b, src view): 3x4 [R|t] of P_src * inv(P_ref) with P = [K E[:3,:4]; E[3]]
 * (models/cas_mvsnet.py:44-47, models/module.py:308-310). rt: [B][N-1][12]. */
int damvs_proj_prepare(void* stream, int B, int N, const float* proj, float* rt);

/* homo_warping(src_fea, src_proj, ref_proj, depth_values) (models/module.py:297-332) for one source
 * view: src [B][h][w][C], rt [B][12] (from damvs_proj_prepare with N = 2), hyps [B][D][h][w],
 * out [B][D][h][w][C]. C in {8, 16, 32}. */
int damvs_homo_warp(void* stream, int dtype, int B, int C, int D, int h, int w, const void* src, const float* rt,
                    const float* hyps, void* out);

/* Feature layouts accepted by damvs_warp_aggregate. */
enum { DAMVS_LAYOUT_NHWC = 0, DAMVS_LAYOUT_CBLOCK = 1 /* [B][C/E][h][w][E], E = 16 bytes of channels */ };

/* Aggregated cost volume (models/cas_mvsnet.py:26-87): volume [B][D][h][w][C]. `layout` gives the
 * feature layout (damvs_stage_forward repacks NHWC to DAMVS_LAYOUT_CBLOCK internally when C spans
 * several 16-byte chunks: each gather instruction then touches half the cache lines). */
int damvs_warp_aggregate(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                         const void* const* feats, int layout, const float* rt, const float* hyps, void* volume);

/* NHWC [B][h][w][C] -> DAMVS_LAYOUT_CBLOCK for N maps (src[v] -> dst[v], device buffers). */
/* 1 if the stage forward gathers C-channel maps of this dtype at N views from channel-blocked copies
 * (damvs_block_channels: pixels wider than 32 bytes that the channel-split warp does not take -- it takes 32 / 64 /
 * 128-byte pixels at odd N >= 3), 0 if it gathers the NHWC maps in place, negative on a bad argument. The split entry
 * point damvs_warp_aggregate takes either layout; callers that mirror damvs_stage_forward ask here.
 * damvs_warp_feat_blocked(dtype, C) is the N = 5 answer (the round-4 entry point, kept for existing callers). */
int damvs_warp_feat_blocked_n(int dtype, int C, int N);
int damvs_warp_feat_blocked(int dtype, int C);
int damvs_block_channels(void* stream, int dtype, int N, int B, int h, int w, int C, const void* const* src,
                         void* const* dst);

/* CostRegNet forward incl. the final prob conv (models/module.py:532-541): logits [B][D][h][w]. */
int damvs_costreg_logits(const damvs_stage* st, void* stream, int B, int D, int h, int w, const void* volume,
                         void* workspace, size_t workspace_bytes, float* logits);

/* ---- pieces of one stage for sharded execution (damvsnet_amd/sharded.py: one depth map over P GPUs) ---- */

/* The aggregated volume of reference rows [y0, y0 + rows) only (models/cas_mvsnet.py:26-87 restricted to
 * those rows; the feature maps stay whole: [B][h][w][C] or channel-blocked per `layout`), read from / written
 * to rows [out_y, out_y + rows) of planes of out_rows rows: hyps [B][D][out_rows][w], volume
 * [B][D][out_rows][w][C] (a haloed H-slab; other rows untouched). Voxels are bitwise those of
 * damvs_warp_aggregate. */
int damvs_warp_aggregate_rows(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w, int y0, int rows,
                              int out_rows, int out_y, const void* const* feats, int layout, const float* rt,
                              const float* hyps, void* volume);

/* One CostRegNet layer (models/module.py:532-540; Conv3d / Deconv3d wrappers :117-202): layer 0..9 =
 * conv0..conv6, conv7, conv9, conv11. D, h, w are the level-0 volume dims (multiples of 8); level l has
 * D>>l, h>>l, w>>l. in: the layer input at its level ([B][Dl][hl][wl][cin]); out: its output. For
 * conv7 / conv9 / conv11, `out` holds the skip tensor (conv4 / conv2 / conv0 output) on entry and
 * relu(deconv(in)) + skip on exit (models/module.py:537-539). Zero padding at every tensor edge. */
int damvs_costreg_layer(const damvs_stage* st, void* stream, int layer, int B, int D, int h, int w, const void* in,
                        void* out);

/* Magnitude slots (fp32 stages). The fp32 path splits each activation x into f16 pieces x * 2^k = hi + lo with k
 * chosen per tensor and batch element from its largest magnitude, so large activations do not overflow the f16 range
 * and small ones keep their lo piece normal (the reference's fp32 convolutions have no range limit:
 * models/cas_mvsnet.py:64-76, models/module.py:510-541), and a sample's result does not depend on the rest of its
 * batch. damvs_stage_forward keeps the slots of its tensors in its workspace. A caller running the U-Net layer by layer
 * (sharded execution) owns them: per tensor B slots of DAMVS_AMAX_SLOT_BYTES of device memory (slot b for batch
 * element b, consecutive), zeroed before use; producers fold max |value| into them (atomically; bit patterns of
 * non-negative floats compare as unsigned integers), consumers read them. Any replica word of a slot may hold the
 * maximum: to set a slot by hand, zero it and write the float's bits (as uint32) into its first word. */
#define DAMVS_AMAX_SLOT_BYTES 4096

/* damvs_costreg_layer with magnitude slots (fp32; bf16 stages ignore them): in_slot = the input tensor's B slots
 * (NULL: unscaled split, exact only while the activations stay inside [2^-3, 65504)), out_slot = the B slots this
 * layer's stored outputs are folded into (NULL: not recorded). damvs_costreg_layer = both NULL. */
int damvs_costreg_layer_scaled(const damvs_stage* st, void* stream, int layer, int B, int D, int h, int w,
                               const void* in, void* out, const void* in_slot, void* out_slot);

/* Fold max |x[i]| of n floats (device) into one magnitude slot (stream-ordered; the slot is not cleared): call it
 * per batch element with that element's slot. */
int damvs_tensor_amax(void* stream, const float* x, long long n, void* slot);

/* The tail of damvs_stage_forward: prob conv (models/module.py:541) + softmax regression, confidence and
 * exp-variance (models/cas_mvsnet.py:105-124) on the U-Net output c0 [B][D][h][w][base].
 * scratch: [B][D][h][w] float (used only when the fused kernels cannot hold a pixel's logits). */
int damvs_stage_regress(const damvs_stage* st, void* stream, int B, int D, int h, int w, const void* c0,
                        const float* hyps, const float* prob_init, float* scratch, float* depth, float* conf, float* var,
                        float* prob);

/* Softmax regression on logits (models/cas_mvsnet.py:105-124). prob_init / prob may be NULL. */
int damvs_regress(void* stream, int B, int D, int h, int w, const float* logits, const float* hyps,
                  const float* prob_init, float* depth, float* conf, float* var, float* prob);

/* Stage hypotheses at stage resolution h = H/scale, w = W/scale (models/cas_mvsnet.py:238-296 with
 * uncertainty_aware_samples, models/module.py:999-1038):
 *   prev_depth == NULL : stage 1, linspace(depth_values[b,0], depth_values[b,Dv-1], D)
 *   otherwise          : uncertainty-aware samples around prev_depth / prev_var ([B][hp][wp]),
 *                        bilinearly upsampled to H x W, then trilinearly resampled to h x w.
 * hyps: [B][D][h][w]. scale must be 1, 2 (refinement) or any value for stage 1. */
int damvs_hypotheses(void* stream, int B, int D, int H, int W, int scale, const float* depth_values, int Dv,
                     const float* prev_depth, const float* prev_var, int hp, int wp, float* hyps);

/* GeoFeatureFusion's sparse depth pyramid (models/geometry.py:90-96, 117-121; SparseDownSampleClose,
 * models/geometry.py:443-455): d0 = (depth - depth_values[b][0]) / (depth_values[b][Dv-1] - depth_values[b][0]),
 * valid mask = mask ? mask : (d0 > 0) ('basic'), then three 2x2 stride-2 closest-valid poolings.
 * depth / mask: [B][h][w] fp32, h, w >= 8; d_l: [B][h >> l][w >> l] (floor sizes, as max_pool2d); scratch: at least
 * B*(h/2)*(w/2) + B*(h/4)*(w/4) floats (the level-1/2 masks). Bitwise equal to the reference's torch ops. */
int damvs_sparse_depth_pyramid(void* stream, int B, int h, int w, const float* depth, const float* depth_values, int Dv,
                               const float* mask, float* d0, float* d1, float* d2, float* d3, float* scratch);

/* ---- 2D front-end convolutions (FeatureNet models/module.py:355-462,
 * GeoFeatureFusion models/geometry.py:14-277). One layer = Conv2d or ConvTranspose2d with BN already
 * folded into weight/bias by the caller, optional ReLU, fused concat of up to two NHWC tensors and up
 * to four fp32 planar inputs (the reference's torch.cat of feature maps and depth planes), and fused
 * residual adds before / after the ReLU. */
typedef struct {
  int transposed;        /* 0: Conv2d weight [cout][cin][k][k]; 1: ConvTranspose2d weight [cin][cout][k][k] */
  int kernel, stride, padding, output_padding;
  int cin, cout;         /* channels of the weight */
  int c0, c0_at;         /* NHWC tensor input 0: channel count, first weight input channel it feeds */
  int c1, c1_at;         /* NHWC tensor input 1 (c1 = 0: none) */
  int ngeo;              /* fp32 planar inputs, each one weight input channel: <= 4 when c0 = c1 = 0
                            (then cout <= 16), else <= 1 (BasicBlockGeo's depth plane) */
  int geo_at[4];
  int relu;
} damvs_conv2d_desc;

typedef struct damvs_conv2d damvs_conv2d;

/* weight / bias: host fp32 (bias may be NULL). c0, c1 must be multiples of 8 (bf16) / 4 (f32);
 * the output is stored with cout rounded up to a multiple of 4 (extra channels are 0 + ReLU).
 * Every operand of a forward call must be smaller than 2 GiB (32-bit device offsets). */
int damvs_conv2d_create(const damvs_conv2d_desc* desc, const float* weight, const float* bias, int dtype,
                        damvs_conv2d** out);
int damvs_conv2d_destroy(damvs_conv2d* layer);
/* Output spatial size for an Hi x Wi input. */
int damvs_conv2d_out_size(const damvs_conv2d* layer, int Hi, int Wi, int* Ho, int* Wo, int* cout_stored);
/* in0/in1: [B][Hi][Wi][c0/c1]; geo[g]: fp32 [Hi][Wi] planes, batch b at geo[g] + b*geo_batch_stride[g];
 * res_pre / res_post: [B][Ho][Wo][cout_stored] (res_post at (Ho/post_up, Wo/post_up), nearest);
 * out: [B][Ho][Wo][cout_stored]. */
int damvs_conv2d_forward(const damvs_conv2d* layer, void* stream, int B, int Hi, int Wi, const void* in0,
                         const void* in1, const float* const* geo, const long long* geo_batch_stride, const void* res_pre,
                         const void* res_post, int post_up, void* out);

/* Border fix-up for a 3x3 padding-1 conv whose bias held the full 9-tap sum of a per-tap constant
 * (a bias that reached the 3x3 conv through a 1x1 conv, FeatureNet's inner2 -> out3,
 * models/module.py:455-459): at every border pixel of out [B][H][W][cout_stored] subtract
 * corr[t * cout + c] (host fp32, t = ky*3 + kx, cout <= 16) for the taps t outside the image. */
int damvs_conv2d_border_bias(void* stream, int dtype, int B, int H, int W, int cout_stored, int cout, const float* corr,
                             void* out);

/* FeatureNet's FPN top level (models/module.py:455-459, out3(up2(f) + inner2(c0))) in one launch, bf16:
 * out = conv3x3_p1(c0) + ConvTranspose2d_k4s2p1(f) + bias — the two layers of the re-association in
 * damvsnet_amd/frontend_hip.py:fpn_top_layers, fused. c0 [B][H][W][8], f [B][H/2][W/2][32], out [B][H][W][8]
 * (bf16); apack: 15 MFMA A chunks x 64 lanes x 8 bf16 (frontend_hip.pack_fpn_top: chunks 0-2 the 3x3 conv's
 * kernel rows as x-pair taps, 3-14 the transposed conv's (row parity, input row, x offset) taps); bias: device
 * fp32 [8]. H, W even. The border fix-up (damvs_conv2d_border_bias) follows as a separate call. */
int damvs_fpn_top_forward(void* stream, int B, int H, int W, const void* c0, const void* f, const void* apack,
                          const float* bias, void* out);

/* The same in fp32 storage (the fp32 parity path): c0, f, out fp32; the products as split-f16 MFMAs. apack: the
 * 15 A chunks scaled by 2^k (max |A| in (2^13, 2^14]) as f16 halves, [chunk][hi: 64 lanes x 8][lo: 64 lanes x 8]
 * (frontend_hip.pack_fpn_top_split); wscale = 2^-k. */
int damvs_fpn_top_forward_f32(void* stream, int B, int H, int W, const void* c0, const void* f, const void* apack,
                              float wscale, const float* bias, void* out);

/* ------------------------------------------------------------------ depth fusion (f4)
 * One reference view of the reference's dynamic-consistency fusion (filter/dypcd.py:98-297,
 * filter_depth per ref view): all maps [H][W] fp32 device buffers of one resolution. Camera
 * products are float32, formed on the host exactly as numpy forms them for float32 matrices. */
#define DAMVS_FUSION_MAX_SRC 10
typedef struct {
  float kinv_ref[9], k_ref[9], einv_ref[16];            /* inv(K_ref), K_ref, inv(E_ref) */
  float t_sr[DAMVS_FUSION_MAX_SRC][16];                  /* E_src . inv(E_ref) */
  float k_src[DAMVS_FUSION_MAX_SRC][9];
  float kinv_src[DAMVS_FUSION_MAX_SRC][9];
  float t_rs[DAMVS_FUSION_MAX_SRC][16];                  /* E_ref . inv(E_src) */
} damvs_fusion_cams;

/* conf: 3 maps (final-stage, stage-2, stage-1 confidence at the final resolution) or NULL (photo
 * test off); conf_thr: args.conf[0..2] (stage-1, stage-2, stage-3). Outputs: depth_avg (averaged
 * depth), mask (bit 0 photo, bit 1 geometric, bit 2 final), xyz [H][W][3] world points of final
 * pixels (0 elsewhere; NULL: not written). 1 <= nsrc <= DAMVS_FUSION_MAX_SRC. */
int damvs_fusion_view(void* stream, int H, int W, int nsrc, const float* depth_ref, const float* const* depth_src,
                      const float* const* conf, const float* conf_thr, const damvs_fusion_cams* cams, double dist_base,
                      double rel_diff_base, float* depth_avg, unsigned char* mask, float* xyz);

#ifdef __cplusplus
}
#endif

#endif /* DAMVS_H */
