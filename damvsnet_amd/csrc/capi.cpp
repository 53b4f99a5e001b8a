// C ABI of libdamvs.so (include/damvs.h): parameter folding/packing at create time and
// stream-ordered orchestration of the per-stage kernels.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "damvs.h"
#include "damvs_internal.h"

using namespace damvs;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return DAMVS_OK;
  return fail(DAMVS_E_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define DAMVS_TRY(expr)            \
  do {                             \
    int _rc = (expr);              \
    if (_rc != DAMVS_OK) return _rc; \
  } while (0)

uint16_t to_bf16(float f) {  // round to nearest even; NaN stays NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

enum LayerKind { CONV_S1 = 0, CONV_S2 = 1, DECONV_S2 = 2 };

struct LayerPlan {
  int kind = 0, cin = 0, cout = 0, mt = 0, nphase = 0;
  ConvPhase ph[kMaxPhases];
  void* wpack = nullptr;
  void* wpack_pair = nullptr;  // Cout <= 8: row-pair packing (stride 1, conv3d_lds_pair_kernel) or
                               // x-parity-pair phases (deconv, conv3d_mfma_kernel<.., XP>)
  int nphase_pair = 0;
  ConvPhase ph_pair[4];
  float* bias = nullptr;
  float wscale = 1.f;  // fp32: 2^-k of the split-f16 weights (split_weights)
  void* wpack32 = nullptr;  // fp32: the z-streamed kernel's 32-K split packing (ConvArgs::wpack32)
  void* wgat32 = nullptr;   // fp32: the gather kernel's 32-K split packing (ConvArgs::wgat32; may alias wpack32)
  int k32_chunks[kMaxPhases] = {0}, k32_off[kMaxPhases] = {0};  // its phases' K chunks / weight offsets (build_phases 32)
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

struct damvs_stage {
  int C = 0, base = 0, mode = 0, dtype = 0, device = 0;
  LayerPlan L[10];
  float* prob_w = nullptr;  // device [kd][kh][kw][c]
  void* prob_pack = nullptr;  // bf16, base 8: banded MFMA form of the prob conv (pack_prob_banded)
  void* prob_split = nullptr;  // fp32, base 8: the same rows as split-f16 pairs (the fused head, k_head.hip)
  float prob_scale = 1.f;      // 2^-k of prob_split
  float k1[32] = {0};
  float s1 = 0, t1 = 0, s2 = 0, t2 = 0;
};

namespace {

// Weight tap lists. Conv: t = kd*9 + kh*3 + kw at input offset k-1 (input = q*stride + k - 1).
// ConvTranspose k3 s2 p1 op1, output parity p per dim: p = 0 -> {k=1 at input q},
// p = 1 -> {k=0 at input q+1, k=2 at input q}   (from o = 2i - 1 + k).
void build_phases(LayerPlan& P, int kchunk_k) {
  auto kch = [&](int ntaps) { return (ntaps * P.cin + kchunk_k - 1) / kchunk_k; };
  std::memset(P.ph, 0, sizeof(P.ph));
  if (P.kind != DECONV_S2) {
    P.nphase = 1;
    ConvPhase& ph = P.ph[0];
    ph.ntaps = 27;
    for (int t = 0; t < 27; ++t) {
      ph.tap[t][0] = (signed char)(t / 9 - 1);
      ph.tap[t][1] = (signed char)((t / 3) % 3 - 1);
      ph.tap[t][2] = (signed char)(t % 3 - 1);
      ph.tap[t][3] = (signed char)t;  // weight tap index
    }
    ph.kchunks = kch(27);
    return;
  }
  P.nphase = 8;
  const int ks[2][2] = {{1, -1}, {0, 2}};
  const int off[2][2] = {{0, 0}, {1, 0}};
  const int cnt[2] = {1, 2};
  for (int p = 0; p < 8; ++p) {
    ConvPhase& ph = P.ph[p];
    ph.pd = (p >> 2) & 1;
    ph.ph = (p >> 1) & 1;
    ph.pw = p & 1;
    int t = 0;
    for (int a = 0; a < cnt[ph.pd]; ++a)
      for (int b = 0; b < cnt[ph.ph]; ++b)
        for (int c = 0; c < cnt[ph.pw]; ++c) {
          ph.tap[t][0] = (signed char)off[ph.pd][a];
          ph.tap[t][1] = (signed char)off[ph.ph][b];
          ph.tap[t][2] = (signed char)off[ph.pw][c];
          ph.tap[t][3] = (signed char)(ks[ph.pd][a] * 9 + ks[ph.ph][b] * 3 + ks[ph.pw][c]);
          ++t;
        }
    ph.ntaps = t;
    ph.kchunks = kch(t);
  }
}

// Pack BN-folded weights wf[co][ci][27] into A-fragment order:
//   element ((w_off + s*MT + m) * 64 + lane) * E + e  =  W[co = m*16 + (lane & 15)][k = s*KC + (lane >> 4)*E + e]
// with k -> (tap t = k / cin, ci = k % cin), zero beyond ntaps / cout.
template <typename S>
void pack_layer(LayerPlan& P, const std::vector<float>& wf, int E, std::vector<S>& out, S (*cvt)(float)) {
  const int KC = 4 * E;
  int w_off = 0;
  for (int p = 0; p < P.nphase; ++p) {
    ConvPhase& ph = P.ph[p];
    ph.w_off = w_off;
    for (int s = 0; s < ph.kchunks; ++s)
      for (int m = 0; m < P.mt; ++m)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < E; ++e) {
            const int co = m * 16 + (lane & 15);
            const int k = s * KC + (lane >> 4) * E + e;
            const int t = k / P.cin, ci = k % P.cin;
            float v = 0.f;
            if (co < P.cout && t < ph.ntaps) v = wf[((size_t)co * P.cin + ci) * 27 + (unsigned char)ph.tap[t][3]];
            out.push_back(cvt(v));
          }
    w_off += ph.kchunks * P.mt;
  }
}

// Row-pair packing for a stride-1 layer with cout <= 8: the 16 MFMA rows are (r, co) = output rows
// y + r (r = 0, 1) x 8 channels; K runs over 36 taps (dz, dy' = 0..3, dx) x cin, where dy' is the
// input row relative to y - 1, so row r sees kernel row ky = dy' - r (zero outside 0..2):
//   element (s * 64 + lane) * E + e  =  A[row = lane & 15][k = s*KC + (lane >> 4)*E + e].
template <typename S>
void pack_layer_pair(const LayerPlan& P, const std::vector<float>& wf, int E, std::vector<S>& out, S (*cvt)(float)) {
  const int KC = 4 * E;
  const int nch = (36 * P.cin + KC - 1) / KC;
  for (int s = 0; s < nch; ++s)
    for (int lane = 0; lane < 64; ++lane)
      for (int e = 0; e < E; ++e) {
        const int row = lane & 15, r = row >> 3, co = row & 7;
        const int k = s * KC + (lane >> 4) * E + e;
        const int t2 = k / P.cin, ci = k % P.cin;
        const int dz = t2 / 12, dy = (t2 / 3) % 4, dx = t2 % 3, ky = dy - r;
        float v = 0.f;
        if (t2 < 36 && co < P.cout && ky >= 0 && ky <= 2) v = wf[((size_t)co * P.cin + ci) * 27 + (dz * 3 + ky) * 3 + dx];
        out.push_back(cvt(v));
      }
}

// ConvTranspose k3 s2 (Cout <= 8) as 4 phases (pz, py) whose 16 MFMA rows are the two x parities
// x 8 channels: x-parity 0 takes kx = 1 at input offset 0, parity 1 takes kx = 2 at offset 0 and
// kx = 0 at offset +1, so both share the input x-offsets {0, +1} (tap[t][2] = dx, tap[t][3] = the
// (kz, ky) part of the weight tap). K per phase = nz * ny * 2 * cin; over the 4 phases 18 * cin
// instead of 27 * cin for the 8 single-parity phases, and no M row is padding.
void build_phases_xpair(LayerPlan& P, int kchunk_k) {
  const int ks[2][2] = {{1, -1}, {0, 2}};
  const int off[2][2] = {{0, 0}, {1, 0}};
  const int cnt[2] = {1, 2};
  std::memset(P.ph_pair, 0, sizeof(P.ph_pair));
  P.nphase_pair = 4;
  for (int p = 0; p < 4; ++p) {
    ConvPhase& ph = P.ph_pair[p];
    ph.pd = (p >> 1) & 1;
    ph.ph = p & 1;
    ph.pw = 0;
    int t = 0;
    for (int a = 0; a < cnt[ph.pd]; ++a)
      for (int b = 0; b < cnt[ph.ph]; ++b)
        for (int dx = 0; dx < 2; ++dx) {
          ph.tap[t][0] = (signed char)off[ph.pd][a];
          ph.tap[t][1] = (signed char)off[ph.ph][b];
          ph.tap[t][2] = (signed char)dx;
          ph.tap[t][3] = (signed char)(ks[ph.pd][a] * 9 + ks[ph.ph][b] * 3);  // + kx by (row parity, dx)
          ++t;
        }
    ph.ntaps = t;
    ph.kchunks = (t * P.cin + kchunk_k - 1) / kchunk_k;
  }
}

template <typename S>
void pack_layer_xpair(LayerPlan& P, const std::vector<float>& wf, int E, std::vector<S>& out, S (*cvt)(float)) {
  const int KC = 4 * E;
  const int kx_of[2][2] = {{1, -1}, {2, 0}};  // [x parity][dx]
  int w_off = 0;
  for (int p = 0; p < P.nphase_pair; ++p) {
    ConvPhase& ph = P.ph_pair[p];
    ph.w_off = w_off;
    for (int s = 0; s < ph.kchunks; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < E; ++e) {
          const int row = lane & 15, px = row >> 3, co = row & 7;
          const int k = s * KC + (lane >> 4) * E + e;
          const int t = k / P.cin, ci = k % P.cin;
          float v = 0.f;
          if (co < P.cout && t < ph.ntaps) {
            const int kx = kx_of[px][(int)ph.tap[t][2]];
            if (kx >= 0) v = wf[((size_t)co * P.cin + ci) * 27 + (unsigned char)ph.tap[t][3] + kx];
          }
          out.push_back(cvt(v));
        }
    w_off += ph.kchunks;
  }
}

int upload(const void* host, size_t bytes, void** dev);
float cvt_f32(float v) { return v; }
uint16_t cvt_bf16(float v) { return to_bf16(v); }

// fp32 layers compute on split-f16 MFMAs (damvs_device.h, mma_split16): the per-layer exponent k that puts the largest
// |w| * 2^k in (2^13, 2^14], so every lo piece that matters is a normal f16 (0 for an all-zero layer).
int split_exponent(const std::vector<float>& w) {
  float mx = 0.f;
  for (float v : w) mx = std::max(mx, std::fabs(v));
  if (!(mx > 0.f) || !std::isfinite(mx)) return 0;
  int e;
  std::frexp(mx, &e);  // mx = f * 2^e, f in [0.5, 1)
  return 14 - e;
}
// A fragments packed as fp32 (4 values per lane and chunk) -> [hi0..hi3 | lo0..lo3] f16 of w * 2^k
std::vector<uint16_t> split_weights(const std::vector<float>& pk, int k) {
  std::vector<uint16_t> out(pk.size() * 2);
  for (size_t q = 0; q < pk.size() / 4; ++q)
    for (int e = 0; e < 4; ++e) {
      const float v = std::ldexp(pk[q * 4 + e], k);
      const _Float16 hi = (_Float16)v;
      const _Float16 lo = (_Float16)(v - (float)hi);
      std::memcpy(&out[q * 8 + e], &hi, 2);
      std::memcpy(&out[q * 8 + 4 + e], &lo, 2);
    }
  return out;
}
// 32-K packing (8 values per lane and chunk, pack_2d at kchunk_k 32) -> per (chunk, cout tile): [hi: 64 lanes x 8 f16]
// [lo: 64 lanes x 8 f16] of w * 2^k (conv2d_wide_kernel<float>, WideForm<float>)
std::vector<uint16_t> split_weights_blocked(const std::vector<float>& pk, int k) {
  std::vector<uint16_t> out(pk.size() * 2);
  for (size_t blk = 0; blk < pk.size() / 512; ++blk)
    for (int lane = 0; lane < 64; ++lane)
      for (int e = 0; e < 8; ++e) {
        const float v = std::ldexp(pk[blk * 512 + lane * 8 + e], k);
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        std::memcpy(&out[blk * 1024 + lane * 8 + e], &hi, 2);
        std::memcpy(&out[blk * 1024 + 512 + lane * 8 + e], &lo, 2);
      }
  return out;
}
int upload_split(const std::vector<float>& pk, int k, void** dev) {
  const std::vector<uint16_t> h = split_weights(pk, k);
  return upload(h.data(), h.size() * 2, dev);
}

int fold_bn(const damvs_bn& bn, int c, std::vector<float>& scale, std::vector<float>& shift) {
  if (!bn.weight || !bn.bias || !bn.running_mean || !bn.running_var) return fail(DAMVS_E_ARG, "null BatchNorm tensor");
  scale.resize(c);
  shift.resize(c);
  for (int i = 0; i < c; ++i) {
    const double inv = 1.0 / std::sqrt((double)bn.running_var[i] + (double)bn.eps);
    scale[i] = (float)(inv * bn.weight[i]);
    shift[i] = (float)(bn.bias[i] - bn.running_mean[i] * inv * bn.weight[i]);
  }
  return DAMVS_OK;
}

int upload(const void* host, size_t bytes, void** dev) {
  if (hipMalloc(dev, bytes) != hipSuccess) return fail(DAMVS_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  return hip_check(hipMemcpy(*dev, host, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
}

struct Shapes {
  int D[4], H[4], W[4];  // level 0 (full), 1 (/2), 2 (/4), 3 (/8)
};

Shapes level_shapes(int D, int h, int w) {
  Shapes s;
  for (int l = 0; l < 4; ++l) {
    s.D[l] = D >> l;
    s.H[l] = h >> l;
    s.W[l] = w >> l;
  }
  return s;
}

struct Workspace {
  size_t status, amax, rt, feat, vol, c[7], logits, total;
};

// Magnitude slots of the fp32 stage's activation tensors (damvs_device.h prescale_of): the volume, conv0..conv6
// outputs, conv7 / conv9 outputs after their in-place skip adds (c4', c2'). conv11's output feeds the exact-fp32 VALU
// prob conv and needs none. Per tensor B slots of kAmaxSlotBytes (one per batch element), zeroed at the start of every
// stage forward.
enum { AM_VOL = 0, AM_C0 = 1, AM_C4S = 8, AM_C2S = 9, AM_SLOTS = 10 };
constexpr size_t kAmaxSlotBytes = (size_t)kAmaxSlotWords * 4;
static_assert(kAmaxSlotBytes == DAMVS_AMAX_SLOT_BYTES, "damvs.h slot size");

// c[i] holds conv_i's output for i = 0..6 (conv7/9/11 accumulate in place into c4/c2/c0).
// Channel-blocked copies of the feature maps ([B][C/E][h][w][E], one 16-byte chunk per plane) for the one-lane warp
// kernel's gathers when a pixel is wider than 32 bytes. 32-, 64- and 128-byte pixels (bf16 C 16 / 32, fp32 C 8 / 16 /
// 32) go to the channel-split warp when the view pipeline takes the view count (odd N >= 3): S = 2 / 4 / 8 lanes read a
// corner's whole pixel record in one instruction from the NHWC maps in place, no repack launch. Where the one-lane
// kernel gathers them instead (even N, DAMVS_WARP_SPLIT=0) pixels wider than 32 bytes are blocked as well: stage 1 at
// N = 6, cfgC B = 4, unblocked against blocked, fp32 (128-byte pixels) 8.44 against 3.62 ms, bf16 (64-byte) 2.04
// against 1.58 ms; at N = 5 the split kernel on NHWC maps wins, fp32 2.05 against 2.38 ms (bf16 1.40 against 1.34 ms
// before the 0.17 ms repack launch it saves; profiles/r05/ab_warp_layout_r05p.txt). damvs_warp_feat_blocked_n exports
// the decision (engine.warp_blocked asks it, so Python and the stage forward always agree).
bool feat_blocked(int dtype, int C, int N) {
  const int bytes = C * (dtype == DAMVS_BF16 ? 2 : 4);
  return bytes > 32 && !warp_split_for(bytes, N);
}
bool feat_needs_blocking(const damvs_stage* st, int N) { return feat_blocked(st->dtype, st->C, N); }

Workspace plan_ws(const damvs_stage* st, int B, int N, int D, int h, int w) {
  const size_t es = st->dtype == DAMVS_BF16 ? 2 : 4;
  const size_t V = (size_t)B * D * h * w;
  const int b = st->base;
  const size_t sz[7] = {V * b, V / 8 * 2 * b, V / 8 * 2 * b, V / 64 * 4 * b, V / 64 * 4 * b, V / 512 * 8 * b,
                        V / 512 * 8 * b};
  Workspace ws;
  size_t o = 0;
  ws.status = o;  // the range status word at offset 0 (damvs_stage_status needs no shape)
  o += align_up(4);
  ws.amax = o;  // fp32: the magnitude slots of the stage's activation tensors
  if (st->dtype == DAMVS_F32) o += align_up(AM_SLOTS * (size_t)B * kAmaxSlotBytes);
  ws.rt = o;
  o += align_up((size_t)B * (N > 1 ? N - 1 : 1) * 12 * 4);
  ws.feat = o;  // channel-blocked copies of the N feature maps (only when C spans several 16-B chunks)
  if (feat_needs_blocking(st, N)) o += (size_t)N * align_up((size_t)B * h * w * st->C * es);
  ws.vol = o;
  o += align_up(V * st->C * es);
  for (int i = 0; i < 7; ++i) {
    ws.c[i] = o;
    o += align_up(sz[i] * es);
  }
  ws.logits = o;
  o += align_up(V * 4);
  ws.total = o;
  return ws;
}

int check_stage_shape(const damvs_stage* st, int B, int N, int D, int h, int w) {
  if (B < 1 || N < 2 || N > kMaxViews) return fail(DAMVS_E_SHAPE, "need B >= 1 and 2 <= N <= %d (got B=%d N=%d)", kMaxViews, B, N);
  if (D < 8 || h < 8 || w < 8 || D % 8 || h % 8 || w % 8)
    return fail(DAMVS_E_SHAPE, "D, h, w must be positive multiples of 8 (got D=%d h=%d w=%d)", D, h, w);
  (void)st;
  return DAMVS_OK;
}

ConvArgs conv_args(const damvs_stage* st, int li, int B, const Shapes& S, int lin, int lout, const void* in, void* out,
                   const void* resid) {
  const LayerPlan& P = st->L[li];
  ConvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.in = in;
  a.out = out;
  a.resid = resid;
  a.wpack = P.wpack;
  a.wpack_pair = P.wpack_pair;
  a.wpack32 = P.wpack32;
  a.wgat32 = P.wgat32;
  std::memcpy(a.k32_chunks, P.k32_chunks, sizeof(a.k32_chunks));
  std::memcpy(a.k32_off, P.k32_off, sizeof(a.k32_off));
  a.bias = P.bias;
  a.B = B;
  a.Cin = P.cin;
  a.Cout = P.cout;
  a.MT = P.mt;
  a.Di = S.D[lin]; a.Hi = S.H[lin]; a.Wi = S.W[lin];
  a.Do = S.D[lout]; a.Ho = S.H[lout]; a.Wo = S.W[lout];
  if (P.kind == DECONV_S2) {  // iterate over the input grid, one phase per output parity
    a.Dq = a.Di; a.Hq = a.Hi; a.Wq = a.Wi;
    a.in_stride = 1;
    a.out_stride = 2;
  } else {
    a.Dq = a.Do; a.Hq = a.Ho; a.Wq = a.Wo;
    a.in_stride = P.kind == CONV_S2 ? 2 : 1;
    a.out_stride = 1;
  }
  a.relu = 1;
  a.wscale = P.wscale;
  a.nphase = P.nphase;
  std::memcpy(a.ph, P.ph, sizeof(a.ph));
  if (P.kind == DECONV_S2 && P.wpack_pair && P.cout == 8 && !conv_xpair_disabled()) {
    a.xpair = 1;
    a.wpack = P.wpack_pair;
    a.nphase = P.nphase_pair;
    std::memset(a.ph, 0, sizeof(a.ph));
    std::memcpy(a.ph, P.ph_pair, sizeof(P.ph_pair));
  }
  return a;
}

// layer i's input / output magnitude slots (-1: none): conv0 reads the volume's, convN writes c_N's, conv7 / conv9 write
// the skip sums c4' / c2' that conv9 / conv11 read
constexpr int kLayerSlots[10][2] = {{AM_VOL, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6}, {6, 7}, {7, AM_C4S},
                                    {AM_C4S, AM_C2S}, {AM_C2S, -1}};
void set_slots(ConvArgs& a, const damvs_stage* st, char* amax, int layer, int B) {
  if (st->dtype != DAMVS_F32 || !amax) return;
  const size_t per = (size_t)B * kAmaxSlotBytes;  // a tensor's B slots
  a.in_amax = reinterpret_cast<const unsigned*>(amax + kLayerSlots[layer][0] * per);
  a.out_amax = kLayerSlots[layer][1] < 0 ? nullptr : reinterpret_cast<unsigned*>(amax + kLayerSlots[layer][1] * per);
}

// U-Net through conv11 (+conv0 skip): the prob conv input ends in c[0]. fp32: the slots at ws + W.amax must hold the
// volume's magnitude (and zeros for the rest) on entry.
int run_unet(const damvs_stage* st, hipStream_t s, int B, int D, int h, int w, const void* vol, char* ws,
             const Workspace& W, int nlayers = 10) {
  const Shapes S = level_shapes(D, h, w);
  void* c[7];
  for (int i = 0; i < 7; ++i) c[i] = ws + W.c[i];
  // (layer, in level, out level, input, output, skip)
  struct Step { int li, lin, lout; const void* in; void* out; const void* res; };
  const Step steps[10] = {
      {0, 0, 0, vol, c[0], nullptr},  {1, 0, 1, c[0], c[1], nullptr}, {2, 1, 1, c[1], c[2], nullptr},
      {3, 1, 2, c[2], c[3], nullptr}, {4, 2, 2, c[3], c[4], nullptr}, {5, 2, 3, c[4], c[5], nullptr},
      {6, 3, 3, c[5], c[6], nullptr}, {7, 3, 2, c[6], c[4], c[4]},    {8, 2, 1, c[4], c[2], c[2]},
      {9, 1, 0, c[2], c[0], c[0]}};
  for (int i = 0; i < nlayers; ++i) {
    const Step& k = steps[i];
    ConvArgs a = conv_args(st, k.li, B, S, k.lin, k.lout, k.in, k.out, k.res);
    set_slots(a, st, ws + W.amax, k.li, B);
    DAMVS_TRY(hip_check(launch_conv3d(s, st->dtype, a), "conv3d launch"));
  }
  return DAMVS_OK;
}

WarpArgs warp_args(const damvs_stage* st, int B, int N, int C, int D, int h, int w, const void* const* feats,
                   const float* rt, const float* hyps, void* out) {
  WarpArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int v = 0; v < N; ++v) a.feats[v] = feats[v];
  a.rt = rt;
  a.hyps = hyps;
  a.out = out;
  a.B = B; a.N = N; a.C = C; a.D = D; a.h = h; a.w = w;
  a.y0 = 0;
  a.rows = h;
  a.out_rows = h;
  a.out_y = 0;
  if (st) {
    std::memcpy(a.k1, st->k1, sizeof(a.k1));
    a.s1 = st->s1; a.t1 = st->t1; a.s2 = st->s2; a.t2 = st->t2;
  }
  return a;
}

// Prob conv (models/module.py:541) + softmax regression, confidence and exp-variance
// (models/cas_mvsnet.py:105-124) on the U-Net output c0 [B][D][h][w][base].
int regress_tail(const damvs_stage* st, hipStream_t s, int B, int D, int h, int w, const void* feat, const float* hyps,
                 const float* prob_init, float* logits, float* depth, float* conf, float* var, float* prob) {
  // base 8: the prob conv on MFMA (logits in an LDS column, as the VALU kernel below); fp32 as split-f16 MFMAs
  const void* pk = st->dtype == DAMVS_BF16 ? st->prob_pack : st->prob_split;
  if (pk && prob_mfma_smem(st->dtype, D) <= 160 * 1024 && prob_mfma_enabled(st->dtype))
    return hip_check(launch_prob_mfma(s, st->dtype, B, D, h, w, feat, pk, st->dtype == DAMVS_BF16 ? 1.f : st->prob_scale,
                                      prob_init, hyps, depth, conf, var, prob),
                     "prob_mfma launch");
  if (prob_regress_smem_bytes(st->dtype, st->base, D) <= 160 * 1024)  // fused: logits stay in LDS
    return hip_check(launch_prob_regress(s, st->dtype, B, st->base, D, h, w, feat, st->prob_w, prob_init, hyps, depth,
                                         conf, var, prob),
                     "prob_regress launch");
  if (!logits) return fail(DAMVS_E_WORKSPACE, "this D needs the logits scratch buffer");
  DAMVS_TRY(hip_check(launch_prob_conv(s, st->dtype, B, st->base, D, h, w, feat, st->prob_w, prob_init, logits),
                      "prob conv launch"));
  return hip_check(launch_regress(s, B, D, h, w, logits, hyps, depth, conf, var, prob), "regress launch");
}

// U-Net layer i (conv0..conv6, conv7, conv9, conv11): (input level, output level)
constexpr int kLayerLevels[10][2] = {{0, 0}, {0, 1}, {1, 1}, {1, 2}, {2, 2}, {2, 3}, {3, 3}, {3, 2}, {2, 1}, {1, 0}};

}  // namespace

extern "C" {

int damvs_abi_version(void) { return DAMVS_ABI_VERSION; }

#ifndef DAMVS_BUILD_ID
#define DAMVS_BUILD_ID "unstamped"
#endif
const char* damvs_build_id(void) { return DAMVS_BUILD_ID; }

const char* damvs_last_error_string(void) { return g_err.c_str(); }

int damvs_stage_create(const damvs_costreg_params* cr, const damvs_aggweight_params* aw, int agg_mode, int dtype,
                       damvs_stage** out) {
  if (!cr || !out) return fail(DAMVS_E_ARG, "null argument");
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  if (agg_mode != DAMVS_AGG_ADAPTIVE && agg_mode != DAMVS_AGG_VARIANCE) return fail(DAMVS_E_ARG, "agg_mode %d", agg_mode);
  if (agg_mode == DAMVS_AGG_ADAPTIVE && !aw) return fail(DAMVS_E_ARG, "adaptive aggregation needs weight-net params");
  const int C = cr->in_channels, b = cr->base_channels;
  if (C != 8 && C != 16 && C != 32) return fail(DAMVS_E_SHAPE, "in_channels %d not in {8,16,32}", C);
  if (b != 8 && b != 16) return fail(DAMVS_E_SHAPE, "base_channels %d not in {8,16}", b);
  if (aw && aw->in_channels != C) return fail(DAMVS_E_SHAPE, "weight-net channels %d != %d", aw->in_channels, C);
  for (int i = 0; i < 10; ++i)
    if (!cr->conv_weight[i]) return fail(DAMVS_E_ARG, "null conv weight %d", i);
  if (!cr->prob_weight) return fail(DAMVS_E_ARG, "null prob weight");

  damvs_stage* st = new damvs_stage();
  st->C = C;
  st->base = b;
  st->mode = agg_mode;
  st->dtype = dtype;
  (void)hipGetDevice(&st->device);
  const int E = dtype == DAMVS_BF16 ? 8 : 4;
  // (cin, cout, kind) of conv0..conv6, conv7, conv9, conv11
  const int spec[10][3] = {{C, b, CONV_S1},         {b, 2 * b, CONV_S2},     {2 * b, 2 * b, CONV_S1},
                           {2 * b, 4 * b, CONV_S2}, {4 * b, 4 * b, CONV_S1}, {4 * b, 8 * b, CONV_S2},
                           {8 * b, 8 * b, CONV_S1}, {8 * b, 4 * b, DECONV_S2}, {4 * b, 2 * b, DECONV_S2},
                           {2 * b, b, DECONV_S2}};
  int rc = DAMVS_OK;
  for (int li = 0; li < 10 && rc == DAMVS_OK; ++li) {
    LayerPlan& P = st->L[li];
    P.cin = spec[li][0];
    P.cout = spec[li][1];
    P.kind = spec[li][2];
    P.mt = (P.cout + 15) / 16;
    if (P.mt == 3) P.mt = 4;
    build_phases(P, 4 * E);
    std::vector<float> scale, shift;
    rc = fold_bn(cr->bn[li], P.cout, scale, shift);
    if (rc != DAMVS_OK) break;
    // normalise to wf[co][ci][27] with BN scale folded in
    std::vector<float> wf((size_t)P.cout * P.cin * 27);
    const float* W = cr->conv_weight[li];
    for (int co = 0; co < P.cout; ++co)
      for (int ci = 0; ci < P.cin; ++ci)
        for (int t = 0; t < 27; ++t) {
          const float v = P.kind == DECONV_S2 ? W[((size_t)ci * P.cout + co) * 27 + t] : W[((size_t)co * P.cin + ci) * 27 + t];
          wf[((size_t)co * P.cin + ci) * 27 + t] = v * scale[co];
        }
    const int kexp = dtype == DAMVS_BF16 ? 0 : split_exponent(wf);
    P.wscale = std::ldexp(1.f, -kexp);
    if (dtype == DAMVS_BF16) {
      std::vector<uint16_t> pk;
      pack_layer<uint16_t>(P, wf, E, pk, cvt_bf16);
      rc = upload(pk.data(), pk.size() * 2, &P.wpack);
    } else {
      std::vector<float> pk;
      pack_layer<float>(P, wf, E, pk, cvt_f32);
      rc = upload_split(pk, kexp, &P.wpack);
    }
    if (rc == DAMVS_OK && dtype != DAMVS_BF16 &&
        ((P.kind == CONV_S1 && P.cin == 16 && P.cout == 16) || (P.kind == DECONV_S2 && P.cin == 32 && P.cout == 16) ||
         (P.kind == CONV_S2 && P.cin == 8 && P.cout == 16))) {
      // the z-streamed kernels of conv2, conv9 and conv1 (fp32 split-f16 forms): the plain packing at 32 K per chunk
      LayerPlan P32 = P;
      build_phases(P32, 32);
      std::vector<float> p32;
      pack_layer<float>(P32, wf, 8, p32, cvt_f32);
      const std::vector<uint16_t> h = split_weights_blocked(p32, kexp);
      rc = upload(h.data(), h.size() * 2, &P.wpack32);
      P.wgat32 = P.wpack32;  // the same plain 32-K packing serves the gather kernel
      for (int p = 0; p < P32.nphase; ++p) P.k32_chunks[p] = P32.ph[p].kchunks, P.k32_off[p] = P32.ph[p].w_off;
    } else if (rc == DAMVS_OK && dtype != DAMVS_BF16 && P.cout > 8) {
      // the gather kernel's 32-K form (conv3d_mfma_kernel<float, MT, false, true>: 16x16x32 f16 split products, twice the
      // 16-K form's MFMA rate) for the layers that run on it (conv3, conv5, conv6, conv7 and the tile kernels' fallbacks)
      LayerPlan P32 = P;
      build_phases(P32, 32);
      std::vector<float> p32;
      pack_layer<float>(P32, wf, 8, p32, cvt_f32);
      const std::vector<uint16_t> h = split_weights_blocked(p32, kexp);
      rc = upload(h.data(), h.size() * 2, &P.wgat32);
      for (int p = 0; p < P32.nphase; ++p) P.k32_chunks[p] = P32.ph[p].kchunks, P.k32_off[p] = P32.ph[p].w_off;
    }
    if (rc == DAMVS_OK && P.kind == DECONV_S2 && P.cout <= 8) {
      build_phases_xpair(P, 4 * E);
      if (dtype == DAMVS_BF16) {
        std::vector<uint16_t> pk;
        pack_layer_xpair<uint16_t>(P, wf, E, pk, cvt_bf16);
        rc = upload(pk.data(), pk.size() * 2, &P.wpack_pair);
      } else {
        std::vector<float> pk;
        pack_layer_xpair<float>(P, wf, E, pk, cvt_f32);
        rc = upload_split(pk, kexp, &P.wpack_pair);
        if (rc == DAMVS_OK && P.cin == 16 && P.cout == 8) {  // conv11's z-streamed kernel (deconv_xpair_zslide<float>)
          LayerPlan P32 = P;
          build_phases_xpair(P32, 32);
          std::vector<float> p32;
          pack_layer_xpair<float>(P32, wf, 8, p32, cvt_f32);
          const std::vector<uint16_t> h = split_weights_blocked(p32, kexp);
          rc = upload(h.data(), h.size() * 2, &P.wpack32);
        }
      }
    }
    if (rc == DAMVS_OK && P.kind == CONV_S1 && P.cout <= 8) {
      if (dtype == DAMVS_BF16) {
        std::vector<uint16_t> pk;
        pack_layer_pair<uint16_t>(P, wf, E, pk, cvt_bf16);
        rc = upload(pk.data(), pk.size() * 2, &P.wpack_pair);
      } else {
        std::vector<float> pk;
        pack_layer_pair<float>(P, wf, E, pk, cvt_f32);
        rc = upload_split(pk, kexp, &P.wpack_pair);
        if (rc == DAMVS_OK) {  // conv0's z-streamed kernel (conv3d_zslide_pair<float>, CIN 8 / 16 / 32)
          std::vector<float> p32;
          pack_layer_pair<float>(P, wf, 8, p32, cvt_f32);
          const std::vector<uint16_t> h = split_weights_blocked(p32, kexp);
          rc = upload(h.data(), h.size() * 2, &P.wpack32);
        }
      }
    }
    if (rc == DAMVS_OK) rc = upload(shift.data(), shift.size() * 4, reinterpret_cast<void**>(&P.bias));
  }
  if (rc == DAMVS_OK) {
    std::vector<float> pw((size_t)27 * b);  // [kd][kh][kw][c] from [1][c][kd][kh][kw]
    for (int c = 0; c < b; ++c)
      for (int t = 0; t < 27; ++t) pw[(size_t)t * b + c] = cr->prob_weight[(size_t)c * 27 + t];
    rc = upload(pw.data(), pw.size() * 4, reinterpret_cast<void**>(&st->prob_w));
  }
  if (rc == DAMVS_OK && dtype == DAMVS_BF16 && b == 8) {
    // pack_prob_rows: the prob conv (Conv3d(8, 1, k3), models/module.py:530) as prob_mfma_kernel's A operand
    // (k_regress.hip): rows m = 4 j + dz (output pixel row j of four, kernel depth dz), K = (voxel slot
    // sl = 3 r + kx of input row r = 0..5, channel), entry W[c][dz][ky = r - j][kx] when dz < 3, sl < 18 and
    // 0 <= ky <= 2, else 0; [chunk][term][lane][8], the fp32 weight as kProbRowTerms bf16 terms (hi + lo).
    std::vector<uint16_t> pk((size_t)kProbRowChunks * kProbRowTerms * 64 * 8, 0);
    for (int k = 0; k < kProbRowChunks; ++k)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < 8; ++e) {
          const int m = lane & 15, j = m >> 2, dz = m & 3, sl = 4 * k + (lane >> 4), r = sl / 3, kx = sl % 3;
          const int ky = r - j;
          float v = 0.f;
          if (dz < 3 && sl < 18 && ky >= 0 && ky <= 2) v = cr->prob_weight[(size_t)e * 27 + dz * 9 + ky * 3 + kx];
          for (int t = 0; t < kProbRowTerms; ++t) {
            const uint16_t q = to_bf16(v);
            pk[(((size_t)k * kProbRowTerms + t) * 64 + lane) * 8 + e] = q;
            float qf;
            const uint32_t qb = (uint32_t)q << 16;
            std::memcpy(&qf, &qb, 4);
            v -= qf;  // exact: the remainder of a round-to-nearest bf16 term
          }
        }
    rc = upload(pk.data(), pk.size() * 2, &st->prob_pack);
  }
  if (rc == DAMVS_OK && dtype == DAMVS_F32 && b == 8) {
    // the rows of pack_prob_rows (above) with fp32 weights, split-f16 at 32 K per chunk: prob_mfma_kernel<float>
    std::vector<float> pf((size_t)kProbRowChunks * 64 * 8, 0.f), all(cr->prob_weight, cr->prob_weight + 27 * 8);
    for (int k = 0; k < kProbRowChunks; ++k)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < 8; ++e) {
          const int m = lane & 15, j = m >> 2, dz = m & 3, sl = 4 * k + (lane >> 4), r = sl / 3, kx = sl % 3;
          const int ky = r - j;
          if (dz < 3 && sl < 18 && ky >= 0 && ky <= 2)
            pf[((size_t)k * 64 + lane) * 8 + e] = cr->prob_weight[(size_t)e * 27 + dz * 9 + ky * 3 + kx];
        }
    const int kp = split_exponent(all);
    st->prob_scale = std::ldexp(1.f, -kp);
    const std::vector<uint16_t> hsp = split_weights_blocked(pf, kp);
    rc = upload(hsp.data(), hsp.size() * 2, &st->prob_split);
  }
  if (rc == DAMVS_OK && agg_mode == DAMVS_AGG_ADAPTIVE) {
    std::vector<float> sc1, sh1, sc2, sh2;
    rc = fold_bn(aw->bn1, 1, sc1, sh1);
    if (rc == DAMVS_OK) rc = fold_bn(aw->bn2, 1, sc2, sh2);
    if (rc == DAMVS_OK) {
      if (!aw->w1 || !aw->w2) {
        rc = fail(DAMVS_E_ARG, "null weight-net conv");
      } else {
        for (int c = 0; c < C; ++c) st->k1[c] = aw->w1[c];
        st->s1 = sc1[0];
        st->t1 = sh1[0];
        st->s2 = aw->w2[0] * sc2[0];
        st->t2 = sh2[0];
      }
    }
  }
  if (rc != DAMVS_OK) {
    damvs_stage_destroy(st);
    return rc;
  }
  *out = st;
  return DAMVS_OK;
}

int damvs_stage_destroy(damvs_stage* st) {
  if (!st) return DAMVS_OK;
  for (auto& P : st->L) {
    if (P.wpack) (void)hipFree(P.wpack);
    if (P.wpack_pair) (void)hipFree(P.wpack_pair);
    if (P.wgat32 && P.wgat32 != P.wpack32) (void)hipFree(P.wgat32);
    if (P.wpack32) (void)hipFree(P.wpack32);
    if (P.bias) (void)hipFree(P.bias);
  }
  if (st->prob_w) (void)hipFree(st->prob_w);
  if (st->prob_pack) (void)hipFree(st->prob_pack);
  if (st->prob_split) (void)hipFree(st->prob_split);
  delete st;
  return DAMVS_OK;
}

int damvs_stage_workspace_size(const damvs_stage* st, int B, int N, int D, int h, int w, size_t* bytes) {
  if (!st || !bytes) return fail(DAMVS_E_ARG, "null argument");
  DAMVS_TRY(check_stage_shape(st, B, N, D, h, w));
  *bytes = plan_ws(st, B, N, D, h, w).total;
  return DAMVS_OK;
}

int damvs_stage_forward(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                        const void* const* feats, const float* proj, const float* hyps, const float* prob_init,
                        void* workspace, size_t workspace_bytes, float* depth, float* conf, float* var,
                        float* prob) {
  return damvs_stage_forward_probed(st, stream, B, N, D, h, w, feats, proj, hyps, prob_init, workspace, workspace_bytes,
                                    depth, conf, var, prob, nullptr);
}

int damvs_stage_forward_probed(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                               const void* const* feats, const float* proj, const float* hyps, const float* prob_init,
                               void* workspace, size_t workspace_bytes, float* depth, float* conf, float* var,
                               float* prob, void* const* events) {
  if (!st || !feats || !proj || !hyps || !workspace || !depth || !conf || !var) return fail(DAMVS_E_ARG, "null argument");
  DAMVS_TRY(check_stage_shape(st, B, N, D, h, w));
  for (int v = 0; v < N; ++v)
    if (!feats[v]) return fail(DAMVS_E_ARG, "null feature pointer for view %d", v);
  const Workspace W = plan_ws(st, B, N, D, h, w);
  if (workspace_bytes < W.total) return fail(DAMVS_E_WORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, W.total);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  float* rt = reinterpret_cast<float*>(ws + W.rt);
  int* status = reinterpret_cast<int*>(ws + W.status);
  DAMVS_TRY(hip_check(launch_proj_prepare(s, B, N, proj, rt), "proj_prepare launch"));
  const bool blk = feat_needs_blocking(st, N);
  const void* fv[kMaxViews];
  for (int v = 0; v < N; ++v) fv[v] = feats[v];
  if (blk) {  // repack to [B][C/E][h][w][E]: halves the cache lines each gather instruction touches
    FeatPtrs src, dst;
    const size_t per = align_up((size_t)B * h * w * st->C * (st->dtype == DAMVS_BF16 ? 2 : 4));
    for (int v = 0; v < N; ++v) {
      src.p[v] = feats[v];
      dst.p[v] = ws + W.feat + v * per;
      fv[v] = dst.p[v];
    }
    DAMVS_TRY(hip_check(launch_block_channels(s, st->dtype, src, dst, N, B, h * w, st->C), "block_channels launch"));
  }
  auto mark = [&](int i) {
    return events && events[i] ? hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(events[i]), s), "hipEventRecord")
                               : DAMVS_OK;
  };
  WarpArgs wa = warp_args(st, B, N, st->C, D, h, w, fv, rt, hyps, ws + W.vol);
  if (st->dtype == DAMVS_F32) {  // fresh magnitude slots; the warp records the volume's
    DAMVS_TRY(hip_check(hipMemsetAsync(ws + W.amax, 0, AM_SLOTS * (size_t)B * kAmaxSlotBytes, s), "slot clear"));
    wa.out_amax = reinterpret_cast<unsigned*>(ws + W.amax + AM_VOL * (size_t)B * kAmaxSlotBytes);
  }
  DAMVS_TRY(mark(0));
  DAMVS_TRY(hip_check(launch_warp_aggregate(s, st->dtype, st->mode, wa, blk), "warp_aggregate launch"));
  DAMVS_TRY(mark(1));
  DAMVS_TRY(run_unet(st, s, B, D, h, w, ws + W.vol, ws, W));
  DAMVS_TRY(mark(2));
  DAMVS_TRY(regress_tail(st, s, B, D, h, w, ws + W.c[0], hyps, prob_init, reinterpret_cast<float*>(ws + W.logits), depth,
                         conf, var, prob));
  DAMVS_TRY(mark(3));
  // range check of the outputs (sticky status word, damvs_stage_status), after the last probe: not in the regression's time
  return hip_check(launch_finite_check(s, depth, conf, var, (long long)B * h * w, status), "finite check launch");
}

int damvs_stage_status(const damvs_stage* st, void* stream, const void* workspace, size_t workspace_bytes) {
  if (!st || !workspace) return fail(DAMVS_E_ARG, "null argument");
  if (workspace_bytes < 4) return fail(DAMVS_E_WORKSPACE, "workspace %zu bytes", workspace_bytes);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int v = 0;
  DAMVS_TRY(hip_check(hipMemcpyAsync(&v, workspace, 4, hipMemcpyDeviceToHost, s), "status copy"));
  DAMVS_TRY(hip_check(hipMemsetAsync(const_cast<void*>(workspace), 0, 4, s), "status clear"));
  DAMVS_TRY(hip_check(hipStreamSynchronize(s), "hipStreamSynchronize"));
  if (v != 0)
    return fail(DAMVS_E_RANGE,
                "non-finite depth / confidence / variance in the stage output: an activation beyond the f16 range of "
                "the fp32 path's split-f16 products (|x| >= 65520) or non-finite inputs");
  return DAMVS_OK;
}

int damvs_proj_prepare(void* stream, int B, int N, const float* proj, float* rt) {
  if (!proj || !rt) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || N < 2) return fail(DAMVS_E_SHAPE, "need B >= 1, N >= 2");
  return hip_check(launch_proj_prepare(reinterpret_cast<hipStream_t>(stream), B, N, proj, rt), "proj_prepare launch");
}

int damvs_homo_warp(void* stream, int dtype, int B, int C, int D, int h, int w, const void* src, const float* rt,
                    const float* hyps, void* out) {
  if (!src || !rt || !hyps || !out) return fail(DAMVS_E_ARG, "null argument");
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  if (C != 8 && C != 16 && C != 32) return fail(DAMVS_E_SHAPE, "C %d not in {8,16,32}", C);
  if (B < 1 || D < 1 || h < 2 || w < 2) return fail(DAMVS_E_SHAPE, "bad shape");
  const void* feats[2] = {src, src};
  WarpArgs a = warp_args(nullptr, B, 2, C, D, h, w, feats, rt, hyps, out);
  return hip_check(launch_warp_aggregate(reinterpret_cast<hipStream_t>(stream), dtype, AGG_WARP_ONLY, a, false),
                   "homo_warp launch");
}

int damvs_warp_aggregate(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w,
                         const void* const* feats, int layout, const float* rt, const float* hyps, void* volume) {
  if (!st || !feats || !rt || !hyps || !volume) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || N < 2 || N > kMaxViews || D < 1 || h < 2 || w < 2) return fail(DAMVS_E_SHAPE, "bad shape");
  if (layout != DAMVS_LAYOUT_NHWC && layout != DAMVS_LAYOUT_CBLOCK) return fail(DAMVS_E_ARG, "layout %d", layout);
  WarpArgs a = warp_args(st, B, N, st->C, D, h, w, feats, rt, hyps, volume);
  return hip_check(launch_warp_aggregate(reinterpret_cast<hipStream_t>(stream), st->dtype, st->mode, a,
                                         layout == DAMVS_LAYOUT_CBLOCK),
                   "warp_aggregate launch");
}

int damvs_warp_feat_blocked_n(int dtype, int C, int N) {
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  if (C < 1) return fail(DAMVS_E_SHAPE, "C %d", C);
  if (N < 2 || N > kMaxViews) return fail(DAMVS_E_SHAPE, "N %d", N);
  return feat_blocked(dtype, C, N) ? 1 : 0;
}

int damvs_warp_feat_blocked(int dtype, int C) { return damvs_warp_feat_blocked_n(dtype, C, 5); }

int damvs_block_channels(void* stream, int dtype, int N, int B, int h, int w, int C, const void* const* src,
                         void* const* dst) {
  if (!src || !dst) return fail(DAMVS_E_ARG, "null argument");
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  const int E = dtype == DAMVS_BF16 ? 8 : 4;
  if (N < 1 || N > kMaxViews || B < 1 || h < 1 || w < 1 || C < E || C % E)
    return fail(DAMVS_E_SHAPE, "bad shape (C must be a multiple of %d)", E);
  FeatPtrs s, d;
  for (int v = 0; v < N; ++v) {
    if (!src[v] || !dst[v]) return fail(DAMVS_E_ARG, "null feature pointer for map %d", v);
    s.p[v] = src[v];
    d.p[v] = dst[v];
  }
  return hip_check(launch_block_channels(reinterpret_cast<hipStream_t>(stream), dtype, s, d, N, B, h * w, C),
                   "block_channels launch");
}

int damvs_costreg_logits(const damvs_stage* st, void* stream, int B, int D, int h, int w, const void* volume,
                         void* workspace, size_t workspace_bytes, float* logits) {
  if (!st || !volume || !workspace || !logits) return fail(DAMVS_E_ARG, "null argument");
  DAMVS_TRY(check_stage_shape(st, B, 2, D, h, w));
  const Workspace W = plan_ws(st, B, 2, D, h, w);
  if (workspace_bytes < W.total) return fail(DAMVS_E_WORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, W.total);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  if (st->dtype == DAMVS_F32) {  // the handed-in volume's magnitude per batch element, measured once
    DAMVS_TRY(hip_check(hipMemsetAsync(ws + W.amax, 0, AM_SLOTS * (size_t)B * kAmaxSlotBytes, s), "slot clear"));
    const long long n = (long long)D * h * w * st->C;
    for (int b = 0; b < B; ++b)
      DAMVS_TRY(hip_check(launch_amax(s, static_cast<const float*>(volume) + b * n, n,
                                      reinterpret_cast<unsigned*>(ws + W.amax + (AM_VOL * (size_t)B + b) * kAmaxSlotBytes)),
                          "amax launch"));
  }
  DAMVS_TRY(run_unet(st, s, B, D, h, w, volume, ws, W));
  return hip_check(launch_prob_conv(s, st->dtype, B, st->base, D, h, w, ws + W.c[0], st->prob_w, nullptr, logits),
                   "prob conv launch");
}

int damvs_costreg_layer(const damvs_stage* st, void* stream, int layer, int B, int D, int h, int w, const void* in,
                        void* out) {
  return damvs_costreg_layer_scaled(st, stream, layer, B, D, h, w, in, out, nullptr, nullptr);
}

int damvs_costreg_layer_scaled(const damvs_stage* st, void* stream, int layer, int B, int D, int h, int w,
                               const void* in, void* out, const void* in_slot, void* out_slot) {
  if (!st || !in || !out) return fail(DAMVS_E_ARG, "null argument");
  if (layer < 0 || layer > 9) return fail(DAMVS_E_ARG, "layer %d not in 0..9", layer);
  DAMVS_TRY(check_stage_shape(st, B, 2, D, h, w));
  const Shapes S = level_shapes(D, h, w);
  const bool deconv = layer >= 7;  // conv7 / conv9 / conv11: relu(deconv) + skip, in place on `out`
  ConvArgs a = conv_args(st, layer, B, S, kLayerLevels[layer][0], kLayerLevels[layer][1], in, out, deconv ? out : nullptr);
  if (st->dtype == DAMVS_F32) {
    a.in_amax = static_cast<const unsigned*>(in_slot);
    a.out_amax = static_cast<unsigned*>(out_slot);
  }
  return hip_check(launch_conv3d(reinterpret_cast<hipStream_t>(stream), st->dtype, a), "conv3d launch");
}

int damvs_tensor_amax(void* stream, const float* x, long long n, void* slot) {
  if (!x || !slot) return fail(DAMVS_E_ARG, "null argument");
  if (n < 0) return fail(DAMVS_E_SHAPE, "n %lld", n);
  return hip_check(launch_amax(reinterpret_cast<hipStream_t>(stream), x, n, static_cast<unsigned*>(slot)), "amax launch");
}

int damvs_stage_regress(const damvs_stage* st, void* stream, int B, int D, int h, int w, const void* c0,
                        const float* hyps, const float* prob_init, float* scratch, float* depth, float* conf, float* var,
                        float* prob) {
  if (!st || !c0 || !hyps || !depth || !conf || !var) return fail(DAMVS_E_ARG, "null argument");
  DAMVS_TRY(check_stage_shape(st, B, 2, D, h, w));
  return regress_tail(st, reinterpret_cast<hipStream_t>(stream), B, D, h, w, c0, hyps, prob_init, scratch, depth, conf,
                      var, prob);
}

int damvs_warp_aggregate_rows(const damvs_stage* st, void* stream, int B, int N, int D, int h, int w, int y0, int rows,
                              int out_rows, int out_y, const void* const* feats, int layout, const float* rt,
                              const float* hyps, void* volume) {
  if (!st || !feats || !rt || !hyps || !volume) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || N < 2 || N > kMaxViews || D < 1 || h < 2 || w < 2) return fail(DAMVS_E_SHAPE, "bad shape");
  if (y0 < 0 || rows < 1 || y0 + rows > h) return fail(DAMVS_E_SHAPE, "rows [%d, %d) outside 0..%d", y0, y0 + rows, h);
  if (out_y < 0 || out_y + rows > out_rows)
    return fail(DAMVS_E_SHAPE, "rows [%d, %d) outside the %d-row output planes", out_y, out_y + rows, out_rows);
  if (layout != DAMVS_LAYOUT_NHWC && layout != DAMVS_LAYOUT_CBLOCK) return fail(DAMVS_E_ARG, "layout %d", layout);
  WarpArgs a = warp_args(st, B, N, st->C, D, h, w, feats, rt, hyps, volume);
  a.y0 = y0;
  a.rows = rows;
  a.out_rows = out_rows;
  a.out_y = out_y;
  return hip_check(launch_warp_aggregate(reinterpret_cast<hipStream_t>(stream), st->dtype, st->mode, a,
                                         layout == DAMVS_LAYOUT_CBLOCK),
                   "warp_aggregate launch");
}

int damvs_regress(void* stream, int B, int D, int h, int w, const float* logits, const float* hyps,
                  const float* prob_init, float* depth, float* conf, float* var, float* prob) {
  if (!logits || !hyps || !depth || !conf || !var) return fail(DAMVS_E_ARG, "null argument");
  if (prob_init) return fail(DAMVS_E_ARG, "prob_init is applied by damvs_stage_forward; add it to the logits");
  if (B < 1 || D < 1 || h < 1 || w < 1) return fail(DAMVS_E_SHAPE, "bad shape");
  return hip_check(launch_regress(reinterpret_cast<hipStream_t>(stream), B, D, h, w, logits, hyps, depth, conf, var,
                                  prob),
                   "regress launch");
}

int damvs_hypotheses(void* stream, int B, int D, int H, int W, int scale, const float* depth_values, int Dv,
                     const float* prev_depth, const float* prev_var, int hp, int wp, float* hyps) {
  if (!hyps) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || D < 2 || H < 1 || W < 1 || scale < 1 || H % scale || W % scale) return fail(DAMVS_E_SHAPE, "bad shape");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!prev_depth) {
    if (!depth_values || Dv < 2) return fail(DAMVS_E_ARG, "stage 1 needs depth_values with Dv >= 2");
    return hip_check(launch_hyp_linear(s, B, D, H / scale, W / scale, depth_values, Dv, hyps), "hyp_linear launch");
  }
  if (!prev_var) return fail(DAMVS_E_ARG, "refinement needs prev_var");
  if (scale != 1 && scale != 2) return fail(DAMVS_E_SHAPE, "refinement scale must be 1 or 2 (got %d)", scale);
  if (hp < 1 || wp < 1) return fail(DAMVS_E_SHAPE, "bad previous-stage shape");
  return hip_check(launch_hyp_refine(s, B, D, H, W, scale, prev_depth, prev_var, hp, wp, hyps), "hyp_refine launch");
}

int damvs_sparse_depth_pyramid(void* stream, int B, int h, int w, const float* depth, const float* depth_values, int Dv,
                               const float* mask, float* d0, float* d1, float* d2, float* d3, float* scratch) {
  if (!depth || !depth_values || !d0 || !d1 || !d2 || !d3 || !scratch) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || h < 8 || w < 8 || Dv < 1) return fail(DAMVS_E_SHAPE, "bad shape (h, w >= 8)");
  if ((long long)B * h * w >= (1ll << 31)) return fail(DAMVS_E_SHAPE, "depth map too large");
  float* m1 = scratch;
  float* m2 = scratch + (size_t)B * (h / 2) * (w / 2);
  return hip_check(launch_sparse_pyramid(reinterpret_cast<hipStream_t>(stream), B, h, w, depth, depth_values, Dv, mask,
                                         d0, d1, d2, d3, m1, m2),
                   "sparse_pool launch");
}

}  // extern "C"

// ============================================================================ 2D convolutions
struct damvs_conv2d {
  damvs_conv2d_desc d;
  int dtype = 0, cout_pad = 0, cout_store = 0, MTtot = 0, nphase = 0, kchunk_k = 0;
  int xpair = 0;  // x-parity-pair phases (build_phases_2d_xpair / pack_2d_xpair)
  float wscale = 1.f;  // fp32: 2^-k of the split-f16 weights (split_weights)
  Conv2dPhase ph[4];
  void* wpack = nullptr;
  Conv2dPhase ph32[4];      // fp32 layers the wide kernel may take: phases and [hi8 | lo8] weights at 32 K per chunk
  void* wpack32 = nullptr;
  float* wgeo = nullptr;
  float* bias = nullptr;
};

namespace {

// Tap lists. Conv: input = q*s + (k - p), one phase. Transposed conv of stride s: output parity r
// per dim takes the kernel taps k with (r + p - k) % s == 0 at input offset (r + p - k) / s.
int build_phases_2d(damvs_conv2d* L) {
  const damvs_conv2d_desc& d = L->d;
  const int K = d.kernel, s = d.stride, p = d.padding;
  const int ctot = d.c0 + d.c1;
  std::memset(L->ph, 0, sizeof(L->ph));
  std::vector<int> offs[2], ks[2];  // per parity r
  if (!d.transposed) {
    L->nphase = 1;
    for (int k = 0; k < K; ++k) { offs[0].push_back(k - p); ks[0].push_back(k); }
  } else {
    if (s != 1 && s != 2) return fail(DAMVS_E_SHAPE, "transposed stride %d unsupported", s);
    L->nphase = s * s;
    // taps in ascending input offset: a stride-1 transposed conv then has exactly the tap list of a plain conv
    // (offsets -p .. K-1-p, row-major), so the LDS-tiled 3x3 kernel (lds3_ok) takes the full-resolution decoder
    // layers instead of the gather kernel
    for (int r = 0; r < s; ++r)
      for (int k = K - 1; k >= 0; --k)
        if (((r + p - k) % s + s) % s == 0) { offs[r].push_back((r + p - k) / s); ks[r].push_back(k); }
  }
  int w_off = 0, g_off = 0;
  for (int ph = 0; ph < L->nphase; ++ph) {
    Conv2dPhase& P = L->ph[ph];
    const int ry = d.transposed ? ph / s : 0, rx = d.transposed ? ph % s : 0;
    P.py = ry;
    P.px = rx;
    int t = 0;
    for (size_t a = 0; a < offs[ry].size(); ++a)
      for (size_t b = 0; b < offs[rx].size(); ++b) {
        if (t >= 25) return fail(DAMVS_E_SHAPE, "more than 25 taps per phase");
        P.tap[t][0] = (signed char)offs[ry][a];
        P.tap[t][1] = (signed char)offs[rx][b];
        P.wtap[t] = (signed char)(ks[ry][a] * K + ks[rx][b]);
        ++t;
      }
    P.ntaps = t;
    P.kchunks = ctot > 0 ? (t * ctot + L->kchunk_k - 1) / L->kchunk_k : 0;
    P.gchunks = d.ngeo > 0 ? (t * d.ngeo + L->kchunk_k - 1) / L->kchunk_k : 0;
    P.w_off = w_off;
    P.g_off = g_off;
    w_off += P.kchunks + P.gchunks;
    g_off += t * d.ngeo;
  }
  return DAMVS_OK;
}

// ConvTranspose2d stride 2 with cout = 8 as 2 phases (output row parity ry): the 16 MFMA rows are
// (output x parity px, channel), and the taps are (input row offsets of ry) x (the union of the input
// x offsets of both parities). A row whose parity does not use an x offset gets zero weights. Per
// output pixel pair this is |offs[ry]| * |union| taps instead of |offs[ry]| * (|offs[0]| + |offs[1]|)
// over two phases with half the MFMA rows empty, and the 16 channels of an x pair are one 32-byte
// store. wtap keeps the ky * K part; pack_2d_xpair resolves kx per row parity.
int build_phases_2d_xpair(damvs_conv2d* L) {
  const damvs_conv2d_desc& d = L->d;
  const int K = d.kernel, p = d.padding;
  std::memset(L->ph, 0, sizeof(L->ph));
  std::vector<int> offs[2], ks[2];
  for (int r = 0; r < 2; ++r)
    for (int k = 0; k < K; ++k)
      if (((r + p - k) % 2 + 2) % 2 == 0) { offs[r].push_back((r + p - k) / 2); ks[r].push_back(k); }
  std::vector<int> xo;  // union of x offsets over both parities, ascending
  for (int r = 0; r < 2; ++r)
    for (int o : offs[r])
      if (std::find(xo.begin(), xo.end(), o) == xo.end()) xo.push_back(o);
  std::sort(xo.begin(), xo.end());
  L->nphase = 2;
  int w_off = 0;
  for (int ry = 0; ry < 2; ++ry) {
    Conv2dPhase& P = L->ph[ry];
    P.py = ry;
    P.px = 0;
    int t = 0;
    for (size_t a = 0; a < offs[ry].size(); ++a)
      for (int dx : xo) {
        if (t >= 25) return fail(DAMVS_E_SHAPE, "more than 25 taps per phase");
        P.tap[t][0] = (signed char)offs[ry][a];
        P.tap[t][1] = (signed char)dx;
        P.wtap[t] = (signed char)(ks[ry][a] * K);
        ++t;
      }
    P.ntaps = t;
    P.kchunks = (t * (d.c0 + d.c1) + L->kchunk_k - 1) / L->kchunk_k;
    P.gchunks = 0;
    P.w_off = w_off;
    w_off += P.kchunks;
  }
  return DAMVS_OK;
}

float wget(const damvs_conv2d_desc& d, const float* W, int co, int wc, int wt) {
  const int KK = d.kernel * d.kernel;
  return d.transposed ? W[((size_t)wc * d.cout + co) * KK + wt] : W[((size_t)co * d.cin + wc) * KK + wt];
}

template <typename S>
void pack_2d(const damvs_conv2d* L, const float* W, std::vector<S>& out, S (*cvt)(float)) {
  const damvs_conv2d_desc& d = L->d;
  const int E = L->kchunk_k / 4, ctot = d.c0 + d.c1;
  for (int ph = 0; ph < L->nphase; ++ph) {
    const Conv2dPhase& P = L->ph[ph];
    // tensor-input chunks (K = tap x concatenated channel), then plane chunks (K = tap x plane)
    for (int s = 0; s < P.kchunks + P.gchunks; ++s)
      for (int m = 0; m < L->MTtot; ++m)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < E; ++e) {
            const int co = m * 16 + (lane & 15);
            const bool plane = s >= P.kchunks;
            const int k = (plane ? s - P.kchunks : s) * L->kchunk_k + (lane >> 4) * E + e;
            const int per = plane ? d.ngeo : ctot;
            const int t = k / per, ci = k % per;
            float v = 0.f;
            if (co < d.cout && t < P.ntaps) {
              const int wc = plane ? d.geo_at[ci] : ci < d.c0 ? d.c0_at + ci : d.c1_at + (ci - d.c0);
              v = wget(d, W, co, wc, (unsigned char)P.wtap[t]);
            }
            out.push_back(cvt(v));
          }
  }
}

// A rows = (x parity px = row >> 3, channel co = row & 7); kx from the parity's tap list.
template <typename S>
void pack_2d_xpair(const damvs_conv2d* L, const float* W, std::vector<S>& out, S (*cvt)(float)) {
  const damvs_conv2d_desc& d = L->d;
  const int E = L->kchunk_k / 4, ctot = d.c0 + d.c1, K = d.kernel, p = d.padding;
  auto kx_of = [&](int px, int dx) {
    for (int k = 0; k < K; ++k)
      if (((px + p - k) % 2 + 2) % 2 == 0 && (px + p - k) / 2 == dx) return k;
    return -1;
  };
  for (int ph = 0; ph < L->nphase; ++ph) {
    const Conv2dPhase& P = L->ph[ph];
    for (int s = 0; s < P.kchunks; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < E; ++e) {
          const int row = lane & 15, px = row >> 3, co = row & 7;
          const int k = s * L->kchunk_k + (lane >> 4) * E + e;
          const int t = k / ctot, ci = k % ctot;
          float v = 0.f;
          if (co < d.cout && t < P.ntaps) {
            const int kx = kx_of(px, P.tap[t][1]);
            const int wc = ci < d.c0 ? d.c0_at + ci : d.c1_at + (ci - d.c0);
            if (kx >= 0) v = wget(d, W, co, wc, (unsigned char)P.wtap[t] + kx);
          }
          out.push_back(cvt(v));
        }
  }
}

bool conv2d_wide32_disabled() {  // DAMVS_CONV2D_WIDE32=0: fp32 wide layers on the 16-K generic kernels (A/B)
  const char* v = getenv("DAMVS_CONV2D_WIDE32");
  return v && v[0] == '0';
}

bool conv2d_xpair_disabled() {
  const char* v = getenv("DAMVS_CONV2D_XPAIR");
  return v && v[0] == '0';
}

void conv2d_out(const damvs_conv2d* L, int Hi, int Wi, int* Ho, int* Wo) {
  const damvs_conv2d_desc& d = L->d;
  if (d.transposed) {
    *Ho = (Hi - 1) * d.stride - 2 * d.padding + d.kernel + d.output_padding;
    *Wo = (Wi - 1) * d.stride - 2 * d.padding + d.kernel + d.output_padding;
  } else {
    *Ho = (Hi + 2 * d.padding - d.kernel) / d.stride + 1;
    *Wo = (Wi + 2 * d.padding - d.kernel) / d.stride + 1;
  }
}

}  // namespace

extern "C" {

int damvs_conv2d_create(const damvs_conv2d_desc* desc, const float* weight, const float* bias, int dtype,
                        damvs_conv2d** out) {
  if (!desc || !weight || !out) return fail(DAMVS_E_ARG, "null argument");
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  const damvs_conv2d_desc& d = *desc;
  const int E = dtype == DAMVS_BF16 ? 8 : 4;
  if (d.kernel < 1 || d.kernel > 5 || d.stride < 1 || d.stride > 2 || d.cout < 1 || d.cin < 1)
    return fail(DAMVS_E_SHAPE, "kernel %d stride %d cout %d cin %d unsupported", d.kernel, d.stride, d.cout, d.cin);
  if (d.c0 % E || d.c1 % E || d.c0 < 0 || d.c1 < 0 || (d.c0 == 0 && d.c1 > 0))
    return fail(DAMVS_E_SHAPE, "tensor input channels must be multiples of %d", E);
  if (d.ngeo < 0 || d.ngeo > 4 || d.c0 + d.c1 + d.ngeo != d.cin)
    return fail(DAMVS_E_SHAPE, "c0 + c1 + ngeo (%d) != cin (%d)", d.c0 + d.c1 + d.ngeo, d.cin);
  if (d.c0 + d.c1 > 0 && d.ngeo > 1)
    return fail(DAMVS_E_SHAPE, "at most one fp32 plane next to tensor inputs (got %d)", d.ngeo);
  if (d.c0 + d.c1 == 0 && d.cout > 16)
    return fail(DAMVS_E_SHAPE, "plane-only layers support cout <= 16 (got %d)", d.cout);
  damvs_conv2d* L = new damvs_conv2d();
  L->d = d;
  L->dtype = dtype;
  L->kchunk_k = 4 * E;
  L->MTtot = (d.cout + 15) / 16;
  L->cout_pad = L->MTtot * 16;
  L->cout_store = (d.cout + 3) / 4 * 4;
  L->xpair = d.transposed && d.stride == 2 && d.cout == 8 && d.ngeo == 0 && d.c0 + d.c1 > 0 && !conv2d_xpair_disabled();
  int rc = L->xpair ? build_phases_2d_xpair(L) : build_phases_2d(L);
  if (rc == DAMVS_OK && d.c0 + d.c1 + d.ngeo > 0) {
    if (dtype == DAMVS_BF16) {
      std::vector<uint16_t> pk;
      if (L->xpair) pack_2d_xpair<uint16_t>(L, weight, pk, cvt_bf16);
      else pack_2d<uint16_t>(L, weight, pk, cvt_bf16);
      rc = upload(pk.data(), pk.size() * 2, &L->wpack);
    } else {
      std::vector<float> pk;
      if (L->xpair) pack_2d_xpair<float>(L, weight, pk, cvt_f32);
      else pack_2d<float>(L, weight, pk, cvt_f32);
      const int kexp = split_exponent(pk);
      L->wscale = std::ldexp(1.f, -kexp);
      rc = upload_split(pk, kexp, &L->wpack);
      // the 32-K split form of the wide kernel (conv2d_wide_kernel<float>), of the narrow halo kernel
      // (conv2d_halo_kernel<float, ..., W32>) and of the gather kernel (conv2d_mfma_kernel<float, ..., K32>: channel
      // counts in multiples of 8): phases and weights at 32 K per chunk
      const int ctot = d.c0 + d.c1;
      if (rc == DAMVS_OK && !L->xpair && d.c0 % 8 == 0 && d.c1 % 8 == 0 && ctot >= 8 && d.ngeo <= 1) {
        damvs_conv2d T32 = *L;
        T32.wpack = nullptr;
        T32.kchunk_k = 32;
        rc = build_phases_2d(&T32);
        if (rc == DAMVS_OK) {
          std::vector<float> p32;
          pack_2d<float>(&T32, weight, p32, cvt_f32);
          const std::vector<uint16_t> h = split_weights_blocked(p32, kexp);
          rc = upload(h.data(), h.size() * 2, &L->wpack32);
          std::memcpy(L->ph32, T32.ph, sizeof(L->ph32));
        }
      }
    }
  }
  if (rc == DAMVS_OK && d.ngeo > 0) {
    std::vector<float> wg;
    for (int ph = 0; ph < L->nphase; ++ph)
      for (int t = 0; t < L->ph[ph].ntaps; ++t)
        for (int g = 0; g < d.ngeo; ++g)
          for (int co = 0; co < L->cout_pad; ++co)
            wg.push_back(co < d.cout ? wget(d, weight, co, d.geo_at[g], (unsigned char)L->ph[ph].wtap[t]) : 0.f);
    rc = upload(wg.data(), wg.size() * 4, reinterpret_cast<void**>(&L->wgeo));
  }
  if (rc == DAMVS_OK) {
    std::vector<float> b(L->cout_pad, 0.f);
    if (bias)
      for (int i = 0; i < d.cout; ++i) b[i] = bias[i];
    rc = upload(b.data(), b.size() * 4, reinterpret_cast<void**>(&L->bias));
  }
  if (rc != DAMVS_OK) {
    damvs_conv2d_destroy(L);
    return rc;
  }
  *out = L;
  return DAMVS_OK;
}

int damvs_fpn_top_forward(void* stream, int B, int H, int W, const void* c0, const void* f, const void* apack,
                          const float* bias, void* out) {
  if (!c0 || !f || !apack || !bias || !out) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || H < 2 || W < 2 || H % 2 || W % 2) return fail(DAMVS_E_SHAPE, "B %d H %d W %d (H, W even)", B, H, W);
  if ((long long)B * H * W * 16 >= (1ll << 31)) return fail(DAMVS_E_SHAPE, "operands must be smaller than 2 GiB");
  return hip_check(launch_fpn_top(static_cast<hipStream_t>(stream), ST_BF16, B, H, W, c0, f, apack, 1.f, bias, out),
                   "fpn_top launch");
}

int damvs_fpn_top_forward_f32(void* stream, int B, int H, int W, const void* c0, const void* f, const void* apack,
                              float wscale, const float* bias, void* out) {
  if (!c0 || !f || !apack || !bias || !out) return fail(DAMVS_E_ARG, "null argument");
  if (B < 1 || H < 2 || W < 2 || H % 2 || W % 2) return fail(DAMVS_E_SHAPE, "B %d H %d W %d (H, W even)", B, H, W);
  if ((long long)B * H * W * 32 >= (1ll << 31)) return fail(DAMVS_E_SHAPE, "operands must be smaller than 2 GiB");
  if (!(wscale > 0.f)) return fail(DAMVS_E_ARG, "wscale %g", (double)wscale);
  return hip_check(launch_fpn_top(static_cast<hipStream_t>(stream), ST_F32, B, H, W, c0, f, apack, wscale, bias, out),
                   "fpn_top launch");
}

int damvs_conv2d_border_bias(void* stream, int dtype, int B, int H, int W, int cout_stored, int cout, const float* corr,
                             void* out) {
  if (!corr || !out) return fail(DAMVS_E_ARG, "null argument");
  if (dtype != DAMVS_F32 && dtype != DAMVS_BF16) return fail(DAMVS_E_DTYPE, "dtype %d unsupported", dtype);
  if (B < 1 || H < 2 || W < 2 || cout < 1 || cout > 16 || cout_stored < cout)
    return fail(DAMVS_E_SHAPE, "B %d H %d W %d cout %d stored %d unsupported", B, H, W, cout, cout_stored);
  BorderArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int t = 0; t < 9; ++t)
    for (int c = 0; c < cout; ++c) a.corr[t * 16 + c] = corr[t * cout + c];
  return hip_check(launch_border_bias(static_cast<hipStream_t>(stream), dtype == DAMVS_BF16 ? ST_BF16 : ST_F32, a, B, H,
                                      W, cout_stored, cout, out),
                   "border_bias launch");
}

int damvs_fusion_view(void* stream, int H, int W, int nsrc, const float* depth_ref, const float* const* depth_src,
                      const float* const* conf, const float* conf_thr, const damvs_fusion_cams* cams, double dist_base,
                      double rel_diff_base, float* depth_avg, unsigned char* mask, float* xyz) {
  if (!depth_ref || !depth_src || !cams || !depth_avg || !mask) return fail(DAMVS_E_ARG, "null argument");
  if (H < 1 || W < 1 || (long long)H * W >= (1LL << 31)) return fail(DAMVS_E_SHAPE, "bad shape %d x %d", H, W);
  if (nsrc < 1 || nsrc > kFusionMaxSrc) return fail(DAMVS_E_SHAPE, "nsrc %d not in [1, %d]", nsrc, kFusionMaxSrc);
  if (conf && (!conf[0] || !conf[1] || !conf[2] || !conf_thr)) return fail(DAMVS_E_ARG, "incomplete confidence maps");
  FusionArgs a;
  std::memset(&a, 0, sizeof(a));
  a.H = H;
  a.W = W;
  a.nsrc = nsrc;
  a.depth_ref = depth_ref;
  for (int v = 0; v < nsrc; ++v) {
    if (!depth_src[v]) return fail(DAMVS_E_ARG, "null source depth %d", v);
    a.depth_src[v] = depth_src[v];
    std::memcpy(a.src[v].t_sr, cams->t_sr[v], sizeof(a.src[v].t_sr));
    std::memcpy(a.src[v].k_src, cams->k_src[v], sizeof(a.src[v].k_src));
    std::memcpy(a.src[v].kinv_src, cams->kinv_src[v], sizeof(a.src[v].kinv_src));
    std::memcpy(a.src[v].t_rs, cams->t_rs[v], sizeof(a.src[v].t_rs));
  }
  if (conf)
    for (int i = 0; i < 3; ++i) {
      a.conf[i] = conf[i];
      a.conf_thr[i] = conf_thr[i];
    }
  std::memcpy(a.kinv_ref, cams->kinv_ref, sizeof(a.kinv_ref));
  std::memcpy(a.k_ref, cams->k_ref, sizeof(a.k_ref));
  std::memcpy(a.einv_ref, cams->einv_ref, sizeof(a.einv_ref));
  for (int i = 2; i <= 10; ++i) {
    a.dist_thr[i - 2] = i * dist_base;
    a.rel_thr[i - 2] = (float)(i * rel_diff_base);
  }
  a.depth_avg = depth_avg;
  a.mask = mask;
  a.xyz = xyz;
  return hip_check(launch_fusion_view(static_cast<hipStream_t>(stream), a), "fusion_view launch");
}

int damvs_conv2d_destroy(damvs_conv2d* L) {
  if (!L) return DAMVS_OK;
  if (L->wpack) (void)hipFree(L->wpack);
  if (L->wpack32) (void)hipFree(L->wpack32);
  if (L->wgeo) (void)hipFree(L->wgeo);
  if (L->bias) (void)hipFree(L->bias);
  delete L;
  return DAMVS_OK;
}

int damvs_conv2d_out_size(const damvs_conv2d* L, int Hi, int Wi, int* Ho, int* Wo, int* cout_stored) {
  if (!L || !Ho || !Wo) return fail(DAMVS_E_ARG, "null argument");
  conv2d_out(L, Hi, Wi, Ho, Wo);
  if (cout_stored) *cout_stored = L->cout_store;
  return DAMVS_OK;
}

int damvs_conv2d_forward(const damvs_conv2d* L, void* stream, int B, int Hi, int Wi, const void* in0,
                         const void* in1, const float* const* geo, const long long* geo_batch_stride, const void* res_pre,
                         const void* res_post, int post_up, void* out) {
  if (!L || !out) return fail(DAMVS_E_ARG, "null argument");
  const damvs_conv2d_desc& d = L->d;
  if ((d.c0 > 0 && !in0) || (d.c1 > 0 && !in1)) return fail(DAMVS_E_ARG, "missing tensor input");
  if (d.ngeo > 0 && (!geo || !geo_batch_stride)) return fail(DAMVS_E_ARG, "missing geometry planes");
  if (B < 1 || Hi < 1 || Wi < 1) return fail(DAMVS_E_SHAPE, "bad shape");
  if (res_post && post_up != 1 && post_up != 2) return fail(DAMVS_E_ARG, "post_up must be 1 or 2");
  Conv2dArgs a;
  std::memset(&a, 0, sizeof(a));
  a.in0 = in0;
  a.in1 = in1;
  a.c0 = d.c0;
  a.c1 = d.c1;
  a.ngeo = d.ngeo;
  for (int g = 0; g < d.ngeo; ++g) {
    if (!geo[g]) return fail(DAMVS_E_ARG, "null geometry plane %d", g);
    a.geo[g] = geo[g];
    a.geo_bstride[g] = geo_batch_stride[g];
  }
  a.wpack = L->wpack;
  a.wgeo = L->wgeo;
  a.bias = L->bias;
  a.res_pre = res_pre;
  a.res_post = res_post;
  a.post_up = res_post ? post_up : 1;
  a.out = out;
  a.cout = L->cout_store;
  a.cout_pad = L->cout_pad;
  a.MTtot = L->MTtot;
  a.B = B;
  a.Hi = Hi;
  a.Wi = Wi;
  conv2d_out(L, Hi, Wi, &a.Ho, &a.Wo);
  if (a.Ho < 1 || a.Wo < 1) return fail(DAMVS_E_SHAPE, "empty output");
  if (d.transposed) {
    if (a.Ho != d.stride * Hi || a.Wo != d.stride * Wi)
      return fail(DAMVS_E_SHAPE, "transposed conv must produce stride x input size");
    a.Hq = Hi;
    a.Wq = Wi;
    a.in_stride = 1;
    a.out_stride = d.stride;
  } else {
    a.Hq = a.Ho;
    a.Wq = a.Wo;
    a.in_stride = d.stride;
    a.out_stride = 1;
  }
  if (res_post && (a.Ho % a.post_up || a.Wo % a.post_up)) return fail(DAMVS_E_SHAPE, "bad upsample shape");
  a.relu = d.relu;
  a.wscale = L->wscale;
  a.nphase = L->nphase;
  a.xpair = L->xpair;
  a.div_wq = make_fastdiv(a.Wq);
  a.div_hq = make_fastdiv(a.Hq);
  std::memcpy(a.ph, L->ph, sizeof(a.ph));
  if (L->wpack32 && !conv2d_wide32_disabled()) {  // fp32: the 32-K split packing when the wide or halo kernel takes it
    Conv2dArgs a32 = a;
    std::memcpy(a32.ph, L->ph32, sizeof(a32.ph));
    a32.wpack = L->wpack32;
    a32.wide32 = 1;
    const hipError_t e = launch_conv2d(reinterpret_cast<hipStream_t>(stream), L->dtype, a32);
    if (e != hipErrorNotSupported) return hip_check(e, "conv2d launch");
  }
  return hip_check(launch_conv2d(reinterpret_cast<hipStream_t>(stream), L->dtype, a), "conv2d launch");
}

}  // extern "C"
