// Native runtime of the keypoint-detection hot path: weight registry keyed by
// the reference's state-dict names, BN folding + NHWC/MFMA repacking, a
// shape-keyed device workspace, and the kernel schedule of the eval forward.
// Exposes the C ABI declared in include/kpd.h.
//
// Reference call stack reproduced by kpd_forward:
//   backbone (torchvision mobilenet_v3_small features.0..12 + LightweightFPN)
//     dll/models/backbone.py:29-39, 258-264
//   select_top_k_channels          dll/models/keypoint_model.py:90, 653-661
//   per-box ROI / heatmap / decode dll/models/keypoint_model.py:143-199
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kpd.h"
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return fail(KPD_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));               \
  } while (0)

inline int pad16(int c) { return (c + 15) / 16 * 16; }

}  // namespace

int kpd_fail_einval(const char* msg) { return fail(KPD_EINVAL, msg); }
int kpd_fail_hip(hipError_t e, const char* where) {
  return fail(KPD_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

namespace {

struct HostT {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

// (in, kernel, expanded, out, use_se, act(1 relu / 3 hswish), stride) -- torchvision table
struct BneckCfg { int cin, k, exp, cout; bool se; int act, s; };
const BneckCfg kBneck[11] = {
    {16, 3, 16, 16, true, ACT_RELU, 2},    {16, 3, 72, 24, false, ACT_RELU, 2},
    {24, 3, 88, 24, false, ACT_RELU, 1},   {24, 5, 96, 40, true, ACT_HSWISH, 2},
    {40, 5, 240, 40, true, ACT_HSWISH, 1}, {40, 5, 240, 40, true, ACT_HSWISH, 1},
    {40, 5, 120, 48, true, ACT_HSWISH, 1}, {48, 5, 144, 48, true, ACT_HSWISH, 1},
    {48, 5, 288, 96, true, ACT_HSWISH, 2}, {96, 5, 576, 96, true, ACT_HSWISH, 1},
    {96, 5, 576, 96, true, ACT_HSWISH, 1}};
const int kFpnIn[4] = {16, 24, 48, 576};

int se_squeeze(int c) {
  const int v = c / 4;
  int n = std::max(8, (int)(v + 4) / 8 * 8);
  if (n < 0.9 * v) n += 8;
  return n;
}

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct DevConv {
  int cin = 0, cout = 0, cin_p = 0, cout_p = 0, k = 1;
  bool bf16 = false;
  void* w = nullptr;
  float* b = nullptr;
  // split (fp32-accurate) copy for the heatmap-head convs: f16 [cout][9][cin/32][hi32 | lo32]
  // of w * 2^w_exp, and the output bound |y| <= bc + bs * max|x| (bc = max|b|, bs = max_co sum|w|)
  void* ws = nullptr;
  int w_exp = 0;
  float bc = 0.f, bs = 0.f;
  int ws_kc = 0;   // 1x1 split copy (kh_att2_kernel): f16 [cout_p][ws_kc][hi32 | lo32], K zero-padded to 32
};
struct DevDW { int C = 0, Cp = 0, k = 3, s = 1, act = 0; float* w = nullptr; float* b = nullptr; };
struct DevSE { int C = 0, Cp = 0, sq = 0; float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr, *b2 = nullptr; };
struct DevBneck {
  BneckCfg cfg;
  bool has_exp = false;
  DevConv expand, project;
  DevDW dw;
  DevSE se;
};

// KEYPOINT_HEAD conv as a split hmconv (MODE 2): several convs' columns side
// by side, f16 [cout][ntap][cin] [hi32 | lo32] weights scaled 2^w_exp, per
// column bias / second affine (ps, pt) / downsample bias (bd)
struct KhSplit {
  void* ws = nullptr;
  int w_exp = 0;
  float *b = nullptr, *ps = nullptr, *pt = nullptr, *bd = nullptr;
  int cin = 0, cout = 0, ntap = 9, ns = 0, nf = 0;
};

struct Work {  // device workspace carve for one (B,H,W,nbox,P) shape
  float* stem = nullptr;
  float* e[11] = {};
  float* d[11] = {};
  float* sesc[11] = {};
  float* o[11] = {};
  float* last = nullptr;
  float* lat[4] = {};
  float* feat = nullptr;
  float* stats = nullptr;
  int32_t* topk = nullptr;
  float* scores = nullptr;
  int32_t* slot = nullptr;
  float* roi = nullptr;
  float* roi_stats = nullptr;
  float* cw = nullptr;
  float* hsc = nullptr;   // split heatmap convs: per-ROI bounds [R][4] (max|xs|, max|h1|)
  float* smap = nullptr;
  void* xs = nullptr;
  void* h1 = nullptr;
  void* h2 = nullptr;
  float* h3 = nullptr;
  float* heat = nullptr;  // internal heat buffer when the caller passes NULL
  float* splitk = nullptr;  // split-K partial sums for small-M 1x1 convs (kSplitKFloats)
  float* pool = nullptr;    // [B][1024] SE channel means from the fused expand+depthwise kernel
  float* separt = nullptr;  // [B][kSePartFloats] SE fc1 partials (exdw_kernel -> seproj_kernel)
  float* sc = nullptr;    // split FPN scale inputs: per-image max|tap0| [B], max|lateral1| [B] (amax_publish_img)
  bool sc_dirty = true;   // sc may hold a previous forward's maxima (topk_kernel re-zeroes it)
  // person-detector glue
  float* pd_pool = nullptr;     // [B][56*56][128]
  float* pd_head = nullptr;     // [B][56*56][48]
  float* pd_boxes = nullptr;    // [B][28224][4]
  float* pd_scores = nullptr;   // [B][28224]
  int32_t* pd_keep = nullptr;   // [B][P]
  int32_t* pd_nkeep = nullptr;  // [B]
  uint8_t* pd_alive = nullptr;  // [B][28224]
  // KEYPOINT_HEAD
  float *kx = nullptr, *ksa = nullptr, *kds1 = nullptr, *krb1 = nullptr, *kds2 = nullptr, *krb2 = nullptr;
  float *kr3 = nullptr, *kv1 = nullptr, *kpr = nullptr, *kpv = nullptr, *klr = nullptr, *klv = nullptr;
  // KEYPOINT_HEAD on the split hmconv path: zero-bordered [R][57 x 57][C] f16
  // [hi32 | lo32] operands (x * att, ResidualBlock 1 / 2 outputs) and the
  // per-image FPN level-0 maximum (their scale bound, written by topk_kernel)
  void *kxs = nullptr, *kr1s = nullptr, *kr2s = nullptr;
  float* imax = nullptr;
};

struct Dims {
  int B = 0, H = 0, W = 0, NB = 0, P = 0, flags = 0;
  int h[12] = {}, w[12] = {};  // spatial dims after stem (0) and after bneck i (i+1)
  int Hf = 0, Wf = 0, tiles = 0;
  bool fused_stats = false;
  // a workspace carved for `o` serves this pass: same geometry, no larger
  // batch (kernels index by the pass's own B / NB / P; the zero borders of the
  // padded heatmap maps are written once at carve time and never overwritten)
  bool fits(const Dims& o) const {
    return H == o.H && W == o.W && flags == o.flags && tiles == o.tiles && B <= o.B && NB <= o.NB && P <= o.P &&
           (size_t)NB * P <= (size_t)o.NB * o.P;
  }
};

}  // namespace

struct kpd_plan {
  int device = 0;
  int in_ch = 3;
  int precision = KPD_PRECISION_FP32;
  bool finalized = false;
  std::map<std::string, HostT> t;
  std::vector<void*> allocs;
  // packed device weights
  float *stem_w = nullptr, *stem_b = nullptr;
  DevBneck bn[11];
  DevConv last;
  DevConv lat[4];
  float lat_S[4] = {0.f, 0.f, 0.f, 0.f};   // max over output channels of sum |lateral weight| (lateral_chain bound)
  DevConv fpn0;
  DevConv fpn_lv[3];   // fpn_convs.1-3 (MobileNetV3Wrapper.forward only; the model's forward skips them)
  bool has_body = false, has_fpn = false, has_ca = false, has_hm = false;   // components registered
  float *ca_w0 = nullptr, *ca_b0 = nullptr, *ca_w2 = nullptr, *ca_b2 = nullptr;
  float *hca_w0 = nullptr, *hca_b0 = nullptr, *hca_w2 = nullptr, *hca_b2 = nullptr;
  float *sa_w = nullptr, *sa_b = nullptr;
  DevConv hm1, hm2, hm3;
  struct {
    _Float16* w0 = nullptr;     // composite conv3x3.L0 weights [128][5][64]
    _Float16* weff = nullptr;   // per position class [128][groups][4][64]
    int w0_bytes = 0, weff_bytes = 0, w_exp0 = 0, w_expE = 0;
    int cls_woff[16] = {}, cls_ng[16] = {}, cls_g[16][kFpn0xMaxGroups] = {};
  } fpn0x;  // FPN level 0 by linearity (conv_glds.hip, fpn0x_kernel)
  float *fin_w = nullptr, *fin_b = nullptr;
  float* zero_bias = nullptr;  // 128 zeros for bias-free laterals
  // person-detector glue: box_heads[0] ++ cls_heads[0] as one 1x1 conv (45 -> 48 ch)
  DevConv pd;
  float* anchors = nullptr;    // [28224][4] reference buffer
  float det_conf = 0.3f, det_iou = 0.3f;
  // KEYPOINT_HEAD (present when keypoint_head.* tensors were registered)
  bool has_kh = false;
  int kh_o = 14;               // regression pool size (height // 4)
  DevConv kh_sa1, kh_ds1, kh_rb1, kh_ds2, kh_rb2, kh_c3, kh_v1, kh_lr, kh_lv;
  float *kh_sa2_w = nullptr, *kh_sa2_b = nullptr;
  float *kh_bn1a_s = nullptr, *kh_bn1a_t = nullptr, *kh_bn1b_s = nullptr, *kh_bn1b_t = nullptr;
  float *kh_lnr_g = nullptr, *kh_lnr_b = nullptr, *kh_fr_w = nullptr, *kh_fr_b = nullptr;
  float *kh_lnv_g = nullptr, *kh_lnv_b = nullptr, *kh_fv_w = nullptr, *kh_fv_b = nullptr;
  // split (fp32-accurate) KEYPOINT_HEAD convs on hmconv_kernel: [ResidualBlock 1
  // (+ downsample tap) | visibility conv], [ResidualBlock 2 (+ downsample)],
  // [regression 3x3]; kh_split = all three packed (split / mixed precision)
  KhSplit kh_s[3];
  bool kh_split = false;
  // workspace, one per concurrent sub-batch (kpd_plan_set_streams)
  static constexpr int kMaxSub = 4;
  static constexpr int kOpWs = kMaxSub;   // workspace of the stand-alone operator entry points
  void* ws[kMaxSub + 1] = {};
  size_t ws_bytes[kMaxSub + 1] = {};
  Dims dims[kMaxSub + 1];
  Work work[kMaxSub + 1];
  bool have_work[kMaxSub + 1] = {};
  int streams = 1;                        // requested sub-batch streams (kpd_plan_set_streams)
  hipStream_t sub_st[kMaxSub] = {};       // [0] unused: sub-batch 0 runs on the caller's stream
  hipEvent_t fork_ev = nullptr, join_ev[kMaxSub] = {};
  // pipelined sub-batches (KPD_PIPE): sub-batch k+1 starts when sub-batch k
  // passes a stage mark, so its latency-bound body overlaps k's heavy stages
  hipEvent_t pipe_ev[kMaxSub] = {};
  bool keep_laterals = false;   // kpd_backbone: every lateral level is an output (no fused chain)
  // kpd_backbone_body: the forward stops after the MobileNet body; its four
  // taps (NHWC, channels padded to 16) are left in the workspace here
  bool body_only = false;
  const float* body_taps[4] = {};
  // hipGraph replay of whole forwards (KPD_GRAPH=1): one executable graph per
  // call signature (shapes, flags, every buffer address, stream), valid while
  // the workspace carve and the weights are the ones it was captured on
  // never: instantiation failed for this signature -> always eager
  // done: recorded after each launch of exec on its caller's stream; retiring
  // an entry waits on it (not on the whole device) before destroying exec
  struct GraphEntry {
    hipGraphExec_t exec = nullptr; hipEvent_t done = nullptr; long epoch = -1; int seen = 0; bool never = false;
  };
  std::map<std::vector<uintptr_t>, GraphEntry> graphs;
  long ws_epoch = 0;             // bumped whenever a workspace is re-carved or the weights re-packed
  bool use_graphs = getenv("KPD_GRAPH") != nullptr && atoi(getenv("KPD_GRAPH")) != 0;   // kpd_plan_set_graphs (KPD_GRAPH=1: on)
  hipStream_t graph_st = nullptr;   // capture stream (the caller's may be the legacy default stream)
  bool graph_abandon_next = false;  // kpd_plan_set_graphs(p, 2): abandon the next capture (tests the retry)
  hipStream_t sub_st_pri[kMaxSub] = {};   // high-priority sub-batch streams (KPD_PIPE_PRI)
  std::map<std::string, std::pair<const void*, size_t>> debug;
  unsigned long long* stamps = nullptr;   // KPD_STAMPS diagnostic buffer (kStampWords)
  // per-stage HIP-event timing (kpd_plan_timing)
  struct Timer { std::vector<std::pair<hipEvent_t, hipEvent_t>> ev; size_t used = 0; };
  bool timing = false;
  std::string timing_only;   // non-empty: record only this stage (kpd_plan_timing_stage)
  std::map<std::string, Timer> timers;
};

namespace {

// ------------------------------------------------------------------ weight helpers
const HostT* get(kpd_plan* p, const std::string& name, std::string& missing) {
  auto it = p->t.find(name);
  if (it == p->t.end()) {
    missing += name + " ";
    return nullptr;
  }
  return &it->second;
}

template <typename T>
int upload(kpd_plan* p, const std::vector<T>& h, T** out) {
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
  p->allocs.push_back(d);
  if (!h.empty()) HIP_TRY(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = reinterpret_cast<T*>(d);
  return KPD_OK;
}

// BN fold: scale = gamma / sqrt(var + eps), shift = beta - mean * scale (+ conv bias * scale)
void bn_fold(const HostT* g, const HostT* b, const HostT* m, const HostT* v, double eps, int n,
             const HostT* conv_bias, std::vector<double>& scale, std::vector<double>& shift) {
  scale.assign(n, 1.0);
  shift.assign(n, 0.0);
  for (int i = 0; i < n; ++i) {
    const double cb = conv_bias ? conv_bias->data[i] : 0.0;
    if (g) {
      const double s = (double)g->data[i] / std::sqrt((double)v->data[i] + eps);
      scale[i] = s;
      shift[i] = (double)b->data[i] - (double)m->data[i] * s + cb * s;
    } else {
      shift[i] = cb;
    }
  }
}

// Dense conv weights [cout][cin][k][k] -> packed [cout_p][k*k][cin_p] with BN scale.
int pack_conv(kpd_plan* p, const std::string& wname, const std::string& bias_name, const std::string& bn,
              double eps, int k, bool bf16, DevConv& dc, std::string& missing) {
  const HostT* w = get(p, wname, missing);
  const HostT* cb = bias_name.empty() ? nullptr : get(p, bias_name, missing);
  const HostT *g = nullptr, *b = nullptr, *m = nullptr, *v = nullptr;
  if (!bn.empty()) {
    g = get(p, bn + ".weight", missing); b = get(p, bn + ".bias", missing);
    m = get(p, bn + ".running_mean", missing); v = get(p, bn + ".running_var", missing);
  }
  if (!w || (!bias_name.empty() && !cb) || (!bn.empty() && (!g || !b || !m || !v))) return KPD_ESTATE;
  const bool linear = w->shape.size() == 2 && k == 1;   // nn.Linear [out][in] as a 1x1 conv
  if (!linear && (w->shape.size() != 4 || w->shape[2] != k || w->shape[3] != k))
    return fail(KPD_EINVAL, "bad shape for " + wname);
  dc.ws = nullptr;   // split copies belong to the previous finalize's (freed) allocations
  dc.w_exp = 0;
  dc.ws_kc = 0;
  dc.cout = (int)w->shape[0];
  dc.cin = (int)w->shape[1];
  dc.k = k;
  dc.bf16 = bf16;
  dc.cin_p = bf16 ? (dc.cin + 63) / 64 * 64 : pad16(dc.cin);
  dc.cout_p = pad16(dc.cout);
  std::vector<double> scale, shift;
  bn_fold(g, b, m, v, eps, dc.cout, cb, scale, shift);
  const int kk = k * k;
  std::vector<float> pw((size_t)dc.cout_p * kk * dc.cin_p, 0.f);
  for (int co = 0; co < dc.cout; ++co)
    for (int ci = 0; ci < dc.cin; ++ci)
      for (int t = 0; t < kk; ++t)
        pw[((size_t)co * kk + t) * dc.cin_p + ci] =
            (float)((double)w->data[((size_t)co * dc.cin + ci) * kk + t] * scale[co]);
  std::vector<float> pb(dc.cout_p, 0.f);
  for (int co = 0; co < dc.cout; ++co) pb[co] = (float)shift[co];
  if (bf16) {
    std::vector<uint16_t> hb(pw.size());
    for (size_t i = 0; i < pw.size(); ++i) hb[i] = f2bf(pw[i]);
    uint16_t* d = nullptr;
    if (int rc = upload(p, hb, &d)) return rc;
    dc.w = d;
  } else {
    float* d = nullptr;
    if (int rc = upload(p, pw, &d)) return rc;
    dc.w = d;
  }
  return upload(p, pb, &dc.b);
}

int pack_dw(kpd_plan* p, const std::string& pre, int k, int s, int act, DevDW& dw, std::string& missing) {
  const HostT* w = get(p, pre + ".0.weight", missing);
  const HostT *g = get(p, pre + ".1.weight", missing), *b = get(p, pre + ".1.bias", missing);
  const HostT *m = get(p, pre + ".1.running_mean", missing), *v = get(p, pre + ".1.running_var", missing);
  if (!w || !g || !b || !m || !v) return KPD_ESTATE;
  dw.C = (int)w->shape[0];
  dw.Cp = pad16(dw.C);
  dw.k = k; dw.s = s; dw.act = act;
  std::vector<double> scale, shift;
  bn_fold(g, b, m, v, 1e-3, dw.C, nullptr, scale, shift);
  std::vector<float> pw((size_t)k * k * dw.Cp, 0.f), pb(dw.Cp, 0.f);
  for (int c = 0; c < dw.C; ++c) {
    for (int t = 0; t < k * k; ++t) pw[(size_t)t * dw.Cp + c] = (float)(w->data[(size_t)c * k * k + t] * scale[c]);
    pb[c] = (float)shift[c];
  }
  if (int rc = upload(p, pw, &dw.w)) return rc;
  return upload(p, pb, &dw.b);
}

// [rows][cols] (a 1x1 conv / linear weight) -> uploaded as [cols][rows]
int pack_transposed(kpd_plan* p, const std::string& name, int rows, int cols, float** out, std::string& missing) {
  const HostT* w = get(p, name, missing);
  if (!w) return KPD_ESTATE;
  if (w->data.size() != (size_t)rows * cols) return fail(KPD_EINVAL, "bad size for " + name);
  std::vector<float> t((size_t)rows * cols);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) t[(size_t)c * rows + r] = w->data[(size_t)r * cols + c];
  return upload(p, t, out);
}

// BatchNorm as a per-channel affine (scale, shift), padded to cout_p -- for a
// BN that sits behind a non-linearity and cannot be folded into a conv.
int pack_bn_affine(kpd_plan* p, const std::string& bn, int cout_p, float** s_out, float** t_out,
                   std::string& missing) {
  const HostT *g = get(p, bn + ".weight", missing), *b = get(p, bn + ".bias", missing);
  const HostT *m = get(p, bn + ".running_mean", missing), *v = get(p, bn + ".running_var", missing);
  if (!g || !b || !m || !v) return KPD_ESTATE;
  const int n = (int)g->data.size();
  std::vector<double> sc, sh;
  bn_fold(g, b, m, v, 1e-5, n, nullptr, sc, sh);
  std::vector<float> s(cout_p, 0.f), t(cout_p, 0.f);
  for (int i = 0; i < n; ++i) { s[i] = (float)sc[i]; t[i] = (float)sh[i]; }
  if (int rc = upload(p, s, s_out)) return rc;
  return upload(p, t, t_out);
}

int pack_plain(kpd_plan* p, const std::string& name, float** out, std::string& missing, size_t expect = 0) {
  const HostT* w = get(p, name, missing);
  if (!w) return KPD_ESTATE;
  if (expect && w->data.size() != expect) return fail(KPD_EINVAL, "bad size for " + name);
  return upload(p, w->data, out);
}

// Split (fp32-accurate) weights of a heatmap-head 3x3 conv (hmconv_kernel
// SPLIT): the packed fp32 weights [cout_p][9][cin_p] scaled by 2^w_exp so
// max|w| < 2^15, each value as f16 hi + lo, stored per 32 input channels as
// [hi32 | lo32] (one 128-byte K-step row).  Also the output bound constants:
// |y_co| <= |b_co| + sum|w_co| * max|x| <= bc + bs * max|x| (rounded up).
int pack_split_hm(kpd_plan* p, DevConv& dc) {
  const int cin = dc.cin_p, kk = dc.k * dc.k;
  if (cin % 32 != 0) return fail(KPD_EINVAL, "split heatmap conv needs cin % 32 == 0");
  const size_t n = (size_t)dc.cout_p * kk * cin;
  std::vector<float> w(n), b(dc.cout_p);
  HIP_TRY(hipMemcpy(w.data(), dc.w, n * sizeof(float), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(b.data(), dc.b, b.size() * sizeof(float), hipMemcpyDeviceToHost));
  float mx = 0.f;
  double bs = 0.0, bc = 0.0;
  for (int co = 0; co < dc.cout_p; ++co) {
    double sa = 0.0;
    for (size_t i = 0; i < (size_t)kk * cin; ++i) {
      const float v = w[(size_t)co * kk * cin + i];
      mx = std::max(mx, std::fabs(v));
      sa += std::fabs((double)v);
    }
    bs = std::max(bs, sa);
    bc = std::max(bc, std::fabs((double)b[co]));
  }
  int e = 0;
  if (mx > 0.f) std::frexp(mx, &e);
  const int w_exp = std::min(std::max(14 - e, -100), 100);
  std::vector<_Float16> hl(2 * n);
  for (size_t row = 0; row < (size_t)dc.cout_p * kk; ++row)
    for (int ci = 0; ci < cin; ++ci) {
      const float x = std::ldexp(w[row * cin + ci], w_exp);
      const _Float16 hi = (_Float16)x, lo = (_Float16)(x - (float)hi);
      const size_t o = row * 2 * cin + (size_t)(ci / 32) * 64 + ci % 32;
      hl[o] = hi;
      hl[o + 32] = lo;
    }
  _Float16* d = nullptr;
  if (int rc = upload(p, hl, &d)) return rc;
  dc.ws = d;
  dc.w_exp = w_exp;
  dc.bc = std::nextafter((float)(bc * (1.0 + 1e-6)), INFINITY);
  dc.bs = std::nextafter((float)(bs * (1.0 + 1e-6)), INFINITY);
  return KPD_OK;
}

// Split (fp32-accurate) copy of a 1x1 conv (kh_att2_kernel: KEYPOINT_HEAD's
// spatial-attention 1x1 128 -> 64): the packed fp32
// weights [cout_p][cin_p] scaled by 2^w_exp (max|w| < 2^15), each value as f16
// hi + lo, stored per 32 input channels as [hi32 | lo32] (K zero-padded to 32).
int pack_split_1x1(kpd_plan* p, DevConv& dc) {
  if (dc.k != 1 || dc.bf16) return fail(KPD_EINVAL, "split 1x1 copy of a non-1x1 conv");
  const int cin = dc.cin_p, kc = (cin + 31) / 32;
  const size_t n = (size_t)dc.cout_p * cin;
  std::vector<float> w(n);
  HIP_TRY(hipMemcpy(w.data(), dc.w, n * sizeof(float), hipMemcpyDeviceToHost));
  float mx = 0.f;
  for (float v : w) mx = std::max(mx, std::fabs(v));
  int e = 0;
  if (mx > 0.f) std::frexp(mx, &e);
  const int w_exp = std::min(std::max(14 - e, -100), 100);
  std::vector<_Float16> hl((size_t)dc.cout_p * kc * 64, (_Float16)0.f);
  for (int co = 0; co < dc.cout_p; ++co)
    for (int ci = 0; ci < cin; ++ci) {
      const float x = std::ldexp(w[(size_t)co * cin + ci], w_exp);
      const _Float16 hi = (_Float16)x, lo = (_Float16)(x - (float)hi);
      const size_t o = ((size_t)co * kc + ci / 32) * 64 + ci % 32;
      hl[o] = hi;
      hl[o + 32] = lo;
    }
  _Float16* d = nullptr;
  if (int rc = upload(p, hl, &d)) return rc;
  dc.ws = d;
  dc.w_exp = w_exp;
  dc.ws_kc = kc;
  return KPD_OK;
}

// KEYPOINT_HEAD convs for hmconv_kernel MODE 2 (keypoint_head.py:22-48,
// 64-90): the parts' output columns side by side from column `col`, taps 0-8
// their 3x3 weights (BN folded), tap 9 (ntap 10) the ResidualBlock's 1x1
// downsample (BN folded) for its own columns, zero elsewhere; columns beyond
// the parts are zero padding.  Per column: bias, the ResidualBlock.bn1 affine
// (ps, pt; 1 and 0 for plain conv + BN + ReLU6 columns) and the downsample
// bias.  Split into f16 hi + lo after one power-of-two scale (as pack_split_hm).
struct KhPart { const DevConv* conv; const DevConv* ds; const float* ps; const float* pt; int col; };
int pack_split_kh(kpd_plan* p, KhSplit& ks, int cin, int cout, int ntap, std::initializer_list<KhPart> parts) {
  std::vector<float> W((size_t)cout * ntap * cin, 0.f), b(cout, 0.f), ps(cout, 1.f), pt(cout, 0.f), bd(cout, 0.f);
  for (const KhPart& q : parts) {
    const DevConv& c = *q.conv;
    if (c.k != 3 || c.bf16 || c.cin_p != cin || q.col + c.cout > cout) return fail(KPD_EINVAL, "KH split pack: shape");
    std::vector<float> w((size_t)c.cout_p * 9 * cin), cb(c.cout_p);
    HIP_TRY(hipMemcpy(w.data(), c.w, w.size() * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(cb.data(), c.b, cb.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int co = 0; co < c.cout; ++co) {
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          W[((size_t)(q.col + co) * ntap + t) * cin + ci] = w[((size_t)co * 9 + t) * cin + ci];
      b[q.col + co] = cb[co];
    }
    if (q.ps) {
      std::vector<float> s(c.cout), t(c.cout);
      HIP_TRY(hipMemcpy(s.data(), q.ps, s.size() * sizeof(float), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(t.data(), q.pt, t.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (int co = 0; co < c.cout; ++co) { ps[q.col + co] = s[co]; pt[q.col + co] = t[co]; }
    }
    if (q.ds) {
      const DevConv& d = *q.ds;
      if (ntap != 10 || d.k != 1 || d.bf16 || d.cin_p != cin || d.cout != c.cout) return fail(KPD_EINVAL, "KH split pack: ds");
      std::vector<float> dw((size_t)d.cout_p * cin), db(d.cout_p);
      HIP_TRY(hipMemcpy(dw.data(), d.w, dw.size() * sizeof(float), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(db.data(), d.b, db.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (int co = 0; co < d.cout; ++co) {
        for (int ci = 0; ci < cin; ++ci) W[((size_t)(q.col + co) * ntap + 9) * cin + ci] = dw[(size_t)co * cin + ci];
        bd[q.col + co] = db[co];
      }
    }
  }
  float mx = 0.f;
  for (float v : W) mx = std::max(mx, std::fabs(v));
  int e = 0;
  if (mx > 0.f) std::frexp(mx, &e);
  const int w_exp = std::min(std::max(14 - e, -100), 100);
  std::vector<_Float16> hl(2 * W.size());
  for (size_t row = 0; row < (size_t)cout * ntap; ++row)
    for (int ci = 0; ci < cin; ++ci) {
      const float x = std::ldexp(W[row * cin + ci], w_exp);
      const _Float16 hi = (_Float16)x, lo = (_Float16)(x - (float)hi);
      const size_t o = row * 2 * cin + (size_t)(ci / 32) * 64 + ci % 32;
      hl[o] = hi;
      hl[o + 32] = lo;
    }
  _Float16* d = nullptr;
  if (int rc = upload(p, hl, &d)) return rc;
  ks.ws = d;
  ks.w_exp = w_exp;
  ks.cin = cin; ks.cout = cout; ks.ntap = ntap;
  if (int rc = upload(p, b, &ks.b)) return rc;
  if (int rc = upload(p, ps, &ks.ps)) return rc;
  if (int rc = upload(p, pt, &ks.pt)) return rc;
  return upload(p, bd, &ks.bd);
}

// FPN level 0 by linearity (fpn0x_kernel): W0 = W3 . L0 (the 3x3 conv on the
// 16-channel stem tap through the bias-free lateral 0) and, per output position
// class (y % 4, x % 4), the 3x3 taps summed by the lateral-1 pixel they read
// after the exact 4x nearest upsample.  Products in double; split into f16
// hi + lo after a power-of-two scale (one per weight set).
int pack_fpn0x(kpd_plan* p, const DevConv& dc, const DevConv& lat0) {
  if (dc.cin_p != 128 || dc.cout_p != 128 || lat0.cin_p != 16 || lat0.cout_p != 128) return KPD_OK;   // path unused
  const size_t n3 = (size_t)128 * 9 * 128;
  std::vector<float> w3(n3), l0((size_t)128 * 16);
  HIP_TRY(hipMemcpy(w3.data(), dc.w, n3 * sizeof(float), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(l0.data(), lat0.w, l0.size() * sizeof(float), hipMemcpyDeviceToHost));
  auto W3 = [&](int co, int t, int k) { return (double)w3[((size_t)co * 9 + t) * 128 + k]; };
  // composite tap0 weights [co][t][c]
  std::vector<double> w0((size_t)128 * 9 * 16, 0.0);
  double m0 = 0.0;
  for (int co = 0; co < 128; ++co)
    for (int t = 0; t < 9; ++t)
      for (int c = 0; c < 16; ++c) {
        double acc = 0.0;
        for (int k = 0; k < 128; ++k) acc += W3(co, t, k) * (double)l0[(size_t)k * 16 + c];
        w0[((size_t)co * 9 + t) * 16 + c] = acc;
        m0 = std::max(m0, std::fabs(acc));
      }
  // per class: tap groups by lateral-1 pixel offset
  auto off = [](int a, int d) { return a + d < 0 ? -1 : (a + d > 3 ? 1 : 0); };
  std::vector<double> weff;
  double mE = 0.0;
  int woff = 0;
  for (int cls = 0; cls < 16; ++cls) {
    const int a = cls >> 2, b = cls & 3;
    int gid[9], ng = 0;
    for (int t = 0; t < 9; ++t) {
      const int gg = (off(a, t / 3 - 1) + 1) * 3 + (off(b, t % 3 - 1) + 1);
      int g = 0;
      while (g < ng && p->fpn0x.cls_g[cls][g] != gg) ++g;
      if (g == ng) {
        if (ng == kFpn0xMaxGroups) return fail(KPD_ESTATE, "fpn0x: more than 4 tap groups");
        p->fpn0x.cls_g[cls][ng++] = gg;
      }
      gid[t] = g;
    }
    p->fpn0x.cls_ng[cls] = ng;
    p->fpn0x.cls_woff[cls] = woff;
    std::vector<double> blk((size_t)128 * ng * 128, 0.0);   // [co][g][k]
    for (int co = 0; co < 128; ++co)
      for (int t = 0; t < 9; ++t)
        for (int k = 0; k < 128; ++k) blk[((size_t)co * ng + gid[t]) * 128 + k] += W3(co, t, k);
    for (double v : blk) mE = std::max(mE, std::fabs(v));
    weff.insert(weff.end(), blk.begin(), blk.end());
    woff += 128 * ng * 128 * 2;   // f16 elements (hi + lo)
  }
  auto wexp = [](double m) {
    int e = 0;
    if (m > 0.0) std::frexp(m, &e);
    return std::min(std::max(14 - e, -100), 100);
  };
  const int e0 = wexp(m0), eE = wexp(mE);
  auto split = [](double x, _Float16* hi, _Float16* lo) {
    *hi = (_Float16)x;
    *lo = (_Float16)(x - (double)*hi);
  };
  // W0 rows [co][kt][hi16(2kt) hi16(2kt+1) lo16(2kt) lo16(2kt+1)], tap 9 = zero
  std::vector<_Float16> h0((size_t)128 * 5 * 64, (_Float16)0.f);
  for (int co = 0; co < 128; ++co)
    for (int t = 0; t < 9; ++t)
      for (int c = 0; c < 16; ++c) {
        _Float16 hi, lo;
        split(std::ldexp(w0[((size_t)co * 9 + t) * 16 + c], e0), &hi, &lo);
        const size_t row = ((size_t)co * 5 + t / 2) * 64, sub = (t & 1) * 16 + c;
        h0[row + sub] = hi;
        h0[row + 32 + sub] = lo;
      }
  // W_eff rows [co][g][kc][hi32 | lo32]
  std::vector<_Float16> hE((size_t)woff, (_Float16)0.f);
  size_t src = 0;
  for (int cls = 0; cls < 16; ++cls) {
    const int ng = p->fpn0x.cls_ng[cls];
    _Float16* dst = hE.data() + p->fpn0x.cls_woff[cls];
    for (int co = 0; co < 128; ++co)
      for (int g = 0; g < ng; ++g)
        for (int k = 0; k < 128; ++k) {
          _Float16 hi, lo;
          split(std::ldexp(weff[src + ((size_t)co * ng + g) * 128 + k], eE), &hi, &lo);
          const size_t row = (((size_t)co * ng + g) * 4 + k / 32) * 64;
          dst[row + k % 32] = hi;
          dst[row + 32 + k % 32] = lo;
        }
    src += (size_t)128 * ng * 128;
  }
  if (int rc = upload(p, h0, &p->fpn0x.w0)) return rc;
  if (int rc = upload(p, hE, &p->fpn0x.weff)) return rc;
  p->fpn0x.w0_bytes = (int)(h0.size() * 2);
  p->fpn0x.weff_bytes = (int)(hE.size() * 2);
  p->fpn0x.w_exp0 = e0;
  p->fpn0x.w_expE = eE;
  return KPD_OK;
}

// ------------------------------------------------------------------ workspace
constexpr long kSplitKFloats = 1L << 22;   // 16 MiB of split-K partials per workspace
constexpr int kFuseMaxPix = 32 * 24;        // input maps up to this size take the fused expand+depthwise
constexpr int kSePartFloats = 8192;         // per image: (Ep / CS) slices x sq fc1 partials

struct Carver {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t n) {
    off = (off + 255) / 256 * 256;
    T* r = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return r;
  }
};

// mixed precision runs the HeatmapHead convs on zero-bordered ROI maps
// (hmconv_kernel); KPD_NO_HMCONV=1 keeps the unpadded generic conv (A/B)
bool hm_padded(const kpd_plan* p) {
  static const bool off = kpd_diag_env("KPD_NO_HMCONV") != nullptr;
  return (p->precision == KPD_PRECISION_MIXED || p->precision == KPD_PRECISION_SPLIT) && !off;
}

size_t carve(kpd_plan* p, const Dims& d, char* base, Work& w) {
  Carver c{base};
  const int B = d.B;
  const size_t R = (size_t)d.NB * d.P;
  w.stem = c.take<float>((size_t)B * d.h[0] * d.w[0] * 16);
  for (int i = 0; i < 11; ++i) {
    const DevBneck& bn = p->bn[i];
    const int ep = pad16(bn.cfg.exp), op = pad16(bn.cfg.cout);
    if (bn.has_exp) w.e[i] = c.take<float>((size_t)B * d.h[i] * d.w[i] * ep);
    w.d[i] = c.take<float>((size_t)B * d.h[i + 1] * d.w[i + 1] * ep);
    if (bn.cfg.se) w.sesc[i] = c.take<float>((size_t)B * ep);
    w.o[i] = c.take<float>((size_t)B * d.h[i + 1] * d.w[i + 1] * op);
  }
  w.last = c.take<float>((size_t)B * d.h[11] * d.w[11] * 576);
  const int lh[4] = {d.h[0], d.h[3], d.h[8], d.h[11]}, lw[4] = {d.w[0], d.w[3], d.w[8], d.w[11]};
  for (int i = 0; i < 4; ++i) w.lat[i] = c.take<float>((size_t)B * lh[i] * lw[i] * 128);
  w.feat = c.take<float>((size_t)B * d.Hf * d.Wf * 128);
  w.stats = c.take<float>((size_t)B * d.tiles * 2 * 128);
  w.sc = c.take<float>((size_t)2 * B * kAmaxStride);
  w.splitk = c.take<float>(kSplitKFloats);
  w.pool = c.take<float>((size_t)B * 1024);
  w.separt = c.take<float>((size_t)B * kSePartFloats);
  w.topk = c.take<int32_t>((size_t)B * 64);
  w.scores = c.take<float>((size_t)B * 128);
  w.imax = c.take<float>((size_t)B);
  if (R > 0) {
    const size_t px = R * 3136;
    const size_t es = p->precision == KPD_PRECISION_MIXED ? 2 : 4;   // bf16, or f16 hi + lo / fp32
    w.slot = c.take<int32_t>(R);
    w.roi = c.take<float>(px * 64);
    w.roi_stats = c.take<float>(R * 56 * 2 * 64);
    w.cw = c.take<float>(R * 64);
    w.hsc = c.take<float>(R * 4);
    w.smap = c.take<float>(px * 2);
    // mixed: zero-bordered ROI maps (hmconv layout, kpd_kernels.h) for the padded heatmap convs (hmconv_kernel)
    const size_t pxp = hm_padded(p) ? R * kHmRoiPos : px;
    w.xs = c.take<char>(pxp * 64 * es);
    w.h1 = c.take<char>(pxp * 256 * es);
    w.h2 = c.take<char>(pxp * 256 * es);
    w.h3 = c.take<float>(px * 64);
    w.heat = c.take<float>(R * 17 * 3136);
    if (d.flags & KPD_FLAG_DUAL_HEAD) {
      const int o = p->kh_o;
      w.kx = c.take<float>(px * 128);
      w.ksa = c.take<float>(px * 64);
      w.kds1 = c.take<float>(px * 64);
      w.krb1 = c.take<float>(px * 64);
      w.kds2 = c.take<float>(px * 32);
      w.krb2 = c.take<float>(px * 32);
      w.kr3 = c.take<float>(px * 16);
      w.kv1 = c.take<float>(px * 32);
      w.kpr = c.take<float>(R * (size_t)pad16(16 * o * o));
      w.kpv = c.take<float>(R * 512);
      w.klr = c.take<float>(R * 256);
      w.klv = c.take<float>(R * 128);
      if (p->kh_split) {
        const size_t pp = R * kHmRoiPos;
        w.kxs = c.take<char>(pp * 128 * 4);
        w.kr1s = c.take<char>(pp * (size_t)p->kh_s[0].ns * 4);
        w.kr2s = c.take<char>(pp * (size_t)p->kh_s[1].ns * 4);
      }
    }
  }
  if (d.flags & KPD_FLAG_DETECT) {
    const size_t na = (size_t)B * 3136 * 9;
    w.pd_pool = c.take<float>((size_t)B * 3136 * 128);
    w.pd_head = c.take<float>((size_t)B * 3136 * 48);
    w.pd_boxes = c.take<float>(na * 4);
    w.pd_scores = c.take<float>(na);
    w.pd_keep = c.take<int32_t>((size_t)B * std::max(d.P, 1));
    w.pd_nkeep = c.take<int32_t>(B);
    w.pd_alive = c.take<uint8_t>(na);
  }
  return c.off + 256;
}

// split-K scratch of the workspace the current forward_one uses (set on entry)
thread_local float* g_splitk = nullptr;

// conv with the second affine + residual + final activation epilogue
int conv_post(const DevConv& L, const void* in, int N, int H, int W, int in_cstride, void* out, int act,
              const float* ps, const float* pt, int act2, const float* res, int act3, hipStream_t st) {
  ConvArgs a{};
  a.in = in; a.wt = L.w; a.bias = L.b; a.out = out; a.res = res;
  a.N = N; a.H = H; a.W = W; a.cin_p = L.cin_p; a.cout_p = L.cout_p;
  a.in_cstride = in_cstride; a.out_cstride = L.cout_p;
  a.rh = H; a.rw = W; a.act = act; a.M = N * H * W;
  a.post_scale = ps; a.post_shift = pt; a.act2 = act2; a.act3 = act3;
  a.splitk_ws = g_splitk; a.splitk_cap = kSplitKFloats;
  HIP_TRY(launch_conv(a, CONV_F32, L.k, st));
  return KPD_OK;
}

// RAII stage marker: records a start/end event pair on the launch stream
// when timing is enabled (events are pooled per stage and reused).
struct Stage {
  kpd_plan* p;
  hipStream_t st;
  hipEvent_t end = nullptr;
  Stage(kpd_plan* plan, const char* name, hipStream_t stream) : p(plan), st(stream) {
    if (!p->timing || (!p->timing_only.empty() && p->timing_only != name)) return;
    auto& t = p->timers[name];
    if (t.used == t.ev.size()) {
      // timing-only events: no system-scope fence when they are recorded (the
      // default event's release writes back / invalidates the L2s, ~6 us a
      // record on this device, inside the measured interval and in the way of
      // the next kernel); KPD_EVENT_FENCE=1 (diagnostic build): default events, A/B
      static const unsigned flags = kpd_diag_env("KPD_EVENT_FENCE") ? hipEventDefault : hipEventDisableSystemFence;
      hipEvent_t a, b;
      if (hipEventCreateWithFlags(&a, flags) != hipSuccess || hipEventCreateWithFlags(&b, flags) != hipSuccess) return;
      t.ev.emplace_back(a, b);
    }
    auto& pr = t.ev[t.used++];
    (void)hipEventRecord(pr.first, st);
    end = pr.second;
  }
  ~Stage() {
    if (end) (void)hipEventRecord(end, st);
  }
};

int conv(const DevConv& L, const void* in, int N, int H, int W, int in_cstride, void* out, int act,
         const float* res, int rh, int rw, const float* a_scale, float* stats, int tiles, int out_kind,
         hipStream_t st, float* amax = nullptr) {
  ConvArgs a{};
  a.amax = amax;
  a.in = in; a.wt = L.w; a.bias = L.b; a.out = out; a.res = res; a.a_scale = a_scale; a.stats = stats;
  a.N = N; a.H = H; a.W = W; a.cin_p = L.cin_p; a.cout_p = L.cout_p;
  a.in_cstride = in_cstride; a.out_cstride = L.cout_p;
  a.rh = rh; a.rw = rw; a.act = act; a.M = N * H * W; a.tiles_per_img = tiles;
  a.splitk_ws = g_splitk; a.splitk_cap = kSplitKFloats;
  const ConvDType dt = !L.bf16 ? CONV_F32 : (out_kind == 1 ? CONV_BF16_OUT_BF16 : CONV_BF16_OUT_F32);
  if (L.k == 1 && !L.bf16 && out_kind == 0 && pw_small_ok(a)) {   // small-K 1x1: direct-to-fragment MFMA
    HIP_TRY(launch_pw_small(a, st));
    return KPD_OK;
  }
  HIP_TRY(launch_conv(a, dt, L.k, st));
  return KPD_OK;
}

// HeatmapHead 3x3 conv + bias + BN + ReLU on the 56x56 ROI maps: bf16 weights
// go to the LDS-DMA kernel (conv_glds.hip), fp32 to the generic one.
// out_kind: 1 = bf16 output, 2 = fp32 output (bf16 weights); fp32 otherwise.
// fin (bf16 path, out_kind 2 only): fuse the final 1x1 + sigmoid into the
// epilogue and write the heatmap instead of `out` (conv_glds.hip).
struct HmFinal { const float *w, *b; const int32_t* slot; int P; float* heat; };
// split mode: per-ROI operand bounds (HmConvArgs) -- input u_in = in_c + in_s *
// hsc[r][in_idx], output u_out = out_c + out_s * hsc[r][out_idx], max|out|
// published into hsc[r][amax_idx]
struct HmSplit { float* hsc; float in_c, in_s; int in_idx; float out_c, out_s; int out_idx, amax_idx; };
int hm_conv(const kpd_plan* p, const DevConv& L, const void* in, int R, int in_cstride, void* out, int out_kind,
            hipStream_t st, const HmFinal* fin = nullptr, unsigned long long* stamps = nullptr,
            const HmSplit* sp = nullptr) {
  if (L.ws) {   // fp32-accurate split products on the padded ROI maps
    if (!sp || !hm_padded(p)) return fail(KPD_EINVAL, "split heatmap conv needs the padded layout and bounds");
    HmConvArgs h{};
    h.in = in; h.wt = L.ws; h.bias = L.b; h.out = out; h.R = R; h.cin = L.cin_p; h.cout = L.cout_p;
    h.stamps = stamps;
    h.split = 1; h.hsc = sp->hsc; h.w_exp = L.w_exp;
    h.in_c = sp->in_c; h.in_s = sp->in_s; h.in_idx = sp->in_idx;
    h.out_c = sp->out_c; h.out_s = sp->out_s; h.out_idx = sp->out_idx; h.amax_idx = sp->amax_idx;
    if (fin) {
      if (L.cout_p != 64) return fail(KPD_EINVAL, "fused final layer needs the 64-channel conv");
      h.fin_w = fin->w; h.fin_b = fin->b; h.slot = fin->slot; h.P = fin->P; h.heat = fin->heat;
      h.out_idx = -1;
    }
    HIP_TRY(launch_hmconv(h, st));
    return KPD_OK;
  }
  if (!L.bf16) return conv(L, in, R, 56, 56, in_cstride, out, ACT_RELU, nullptr, 0, 0, nullptr, nullptr, 0, 0, st);
  if (hm_padded(p)) {
    if (in_cstride != L.cin_p) return fail(KPD_EINVAL, "hmconv: input channel stride must equal cin");
    HmConvArgs h{};
    h.in = in; h.wt = L.w; h.bias = L.b; h.out = out; h.R = R; h.cin = L.cin_p; h.cout = L.cout_p;
    h.stamps = stamps;
    if (fin) {
      if (out_kind != 2 || L.cout_p != 64) return fail(KPD_EINVAL, "fused final layer needs the 64-channel conv");
      h.fin_w = fin->w; h.fin_b = fin->b; h.slot = fin->slot; h.P = fin->P; h.heat = fin->heat;
    } else if (out_kind != 1) {
      return fail(KPD_EINVAL, "hmconv: bf16 output or the fused final layer only");
    }
    HIP_TRY(launch_hmconv(h, st));
    return KPD_OK;
  }
  Conv16Args a{};
  if (fin) {
    if (out_kind != 2 || L.cout_p != 64) return fail(KPD_EINVAL, "fused final layer needs the 64-channel conv");
    a.fin_w = fin->w; a.fin_b = fin->b; a.slot = fin->slot; a.P = fin->P; a.heat = fin->heat;
  }
  a.in = in; a.wt = L.w; a.bias = L.b; a.out = out;
  a.N = R; a.H = 56; a.W = 56; a.cin_e = L.cin_p; a.cout_p = L.cout_p; a.in_cstride = in_cstride;
  a.out_cstride = L.cout_p; a.act = ACT_RELU; a.M = R * 56 * 56;
  HIP_TRY(launch_conv16(a, 0, out_kind == 1, st));
  return KPD_OK;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* kpd_last_error(void) { return g_err.c_str(); }
const char* kpd_version(void) { return "kpd 0.1 gfx950"; }
int kpd_build_flags(void) { return KPD_DIAG ? KPD_BUILD_DIAG : 0; }

int kpd_plan_create(int device, int in_channels, kpd_plan** out) {
  if (!out) return fail(KPD_EINVAL, "out is NULL");
  if (in_channels != 1 && in_channels != 3) return fail(KPD_EINVAL, "in_channels must be 1 or 3");
  auto* p = new kpd_plan();
  p->device = device;
  p->in_ch = in_channels;
  *out = p;
  return KPD_OK;
}

int kpd_plan_set_tensor(kpd_plan* p, const char* name, const float* host, const int64_t* shape, int ndim) {
  if (!p || !name || (!host && ndim > 0)) return fail(KPD_EINVAL, "null argument");
  HostT t;
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    if (shape[i] < 0) return fail(KPD_EINVAL, "negative dim");
    t.shape.push_back(shape[i]);
    n *= (size_t)shape[i];
  }
  t.data.assign(host, host + n);
  p->t[name] = std::move(t);
  p->finalized = false;
  return KPD_OK;
}

// wait for a captured forward's last launch (its own event, not the device),
// then destroy it
static hipError_t retire_graph(kpd_plan::GraphEntry& g) {
  hipError_t e = hipSuccess;
  if (g.done) {
    e = hipEventSynchronize(g.done);
    (void)hipEventDestroy(g.done);
    g.done = nullptr;
  }
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  g.exec = nullptr;
  return e;
}

void kpd_plan_destroy(kpd_plan* p) {
  if (!p) return;
  int cur = 0;
  if (hipGetDevice(&cur) == hipSuccess) (void)hipSetDevice(p->device);
  for (void* a : p->allocs) (void)hipFree(a);
  for (int k = 0; k <= kpd_plan::kMaxSub; ++k)
    if (p->ws[k]) (void)hipFree(p->ws[k]);
  for (int k = 0; k < kpd_plan::kMaxSub; ++k) {
    if (p->sub_st[k]) (void)hipStreamDestroy(p->sub_st[k]);
    if (p->join_ev[k]) (void)hipEventDestroy(p->join_ev[k]);
    if (p->sub_st_pri[k]) (void)hipStreamDestroy(p->sub_st_pri[k]);
    if (p->pipe_ev[k]) (void)hipEventDestroy(p->pipe_ev[k]);
  }
  if (p->fork_ev) (void)hipEventDestroy(p->fork_ev);
  for (auto& kv : p->graphs) (void)retire_graph(kv.second);
  if (p->graph_st) (void)hipStreamDestroy(p->graph_st);
  for (auto& kv : p->timers)
    for (auto& e : kv.second.ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  (void)hipSetDevice(cur);
  delete p;
}

int kpd_plan_finalize(kpd_plan* p, int precision) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  if (precision != KPD_PRECISION_FP32 && precision != KPD_PRECISION_MIXED && precision != KPD_PRECISION_SPLIT)
    return fail(KPD_EINVAL, "unknown precision");
  HIP_TRY(hipSetDevice(p->device));
  for (void* a : p->allocs) (void)hipFree(a);
  p->allocs.clear();
  p->fpn0x.w0 = p->fpn0x.weff = nullptr;
  p->stamps = nullptr;
  p->pd = DevConv();
  p->anchors = nullptr;
  p->hm1 = DevConv();
  p->hm2 = DevConv();
  p->hm3 = DevConv();
  for (auto& c : p->fpn_lv) c = DevConv();
  p->kh_ds1 = DevConv();
  p->kh_ds2 = DevConv();
  for (auto& k : p->kh_s) k = KhSplit();
  p->kh_split = false;
  p->has_kh = false;
  for (int k = 0; k <= kpd_plan::kMaxSub; ++k) {
    if (p->ws[k]) { (void)hipFree(p->ws[k]); p->ws[k] = nullptr; p->ws_bytes[k] = 0; }
    p->have_work[k] = false;
  }
  p->precision = precision;
  std::string missing;
  int rc = KPD_OK;
  auto chk = [&](int r) { if (r != KPD_OK && rc == KPD_OK) rc = r; };
  // Components present in the registered state dict (a submodule's own plan
  // -- HeatmapHead, KEYPOINT_HEAD, the backbone -- registers only its part);
  // a present component must be complete.
  auto has = [&](const char* prefix) {
    auto it = p->t.lower_bound(prefix);
    return it != p->t.end() && it->first.compare(0, strlen(prefix), prefix) == 0;
  };
  p->has_body = has("backbone.body.");
  p->has_fpn = has("backbone.fpn.");
  p->has_ca = has("channel_attention.");
  p->has_hm = has("heatmap_head.");
  const bool has_pd = has("person_detector.");
  const std::string F = "backbone.body.features.";
  // stem: [16][Cin][3][3] + BN, packed [16][Cin*9]
  if (p->has_body) {
    const HostT* w = get(p, F + "0.0.weight", missing);
    const HostT *g = get(p, F + "0.1.weight", missing), *b = get(p, F + "0.1.bias", missing);
    const HostT *m = get(p, F + "0.1.running_mean", missing), *v = get(p, F + "0.1.running_var", missing);
    if (w && g && b && m && v) {
      if (w->shape.size() != 4 || w->shape[0] != 16 || w->shape[1] != p->in_ch)
        return fail(KPD_EINVAL, "stem weight shape does not match in_channels");
      std::vector<double> sc, sh;
      bn_fold(g, b, m, v, 1e-3, 16, nullptr, sc, sh);
      std::vector<float> pw(w->data.size()), pb(16);
      const size_t per = w->data.size() / 16;
      for (int co = 0; co < 16; ++co) {
        for (size_t k = 0; k < per; ++k) pw[co * per + k] = (float)(w->data[co * per + k] * sc[co]);
        pb[co] = (float)sh[co];
      }
      chk(upload(p, pw, &p->stem_w));
      chk(upload(p, pb, &p->stem_b));
    } else {
      chk(KPD_ESTATE);
    }
  for (int i = 0; i < 11; ++i) {
    DevBneck& bn = p->bn[i];
    bn.cfg = kBneck[i];
    bn.has_exp = bn.cfg.exp != bn.cfg.cin;
    const std::string pre = F + std::to_string(i + 1) + ".block.";
    int j = 0;
    if (bn.has_exp) {
      chk(pack_conv(p, pre + "0.0.weight", "", pre + "0.1", 1e-3, 1, false, bn.expand, missing));
      ++j;
    }
    chk(pack_dw(p, pre + std::to_string(j), bn.cfg.k, bn.cfg.s, bn.cfg.act, bn.dw, missing));
    ++j;
    if (bn.cfg.se) {
      const std::string s = pre + std::to_string(j);
      bn.se.C = bn.cfg.exp; bn.se.Cp = pad16(bn.cfg.exp); bn.se.sq = se_squeeze(bn.cfg.exp);
      chk(pack_plain(p, s + ".fc1.weight", &bn.se.w1, missing, (size_t)bn.se.sq * bn.se.C));
      chk(pack_plain(p, s + ".fc1.bias", &bn.se.b1, missing, bn.se.sq));
      chk(pack_transposed(p, s + ".fc2.weight", bn.se.C, bn.se.sq, &bn.se.w2, missing));
      chk(pack_plain(p, s + ".fc2.bias", &bn.se.b2, missing, bn.se.C));
      ++j;
    }
    const std::string pj = pre + std::to_string(j);
    chk(pack_conv(p, pj + ".0.weight", "", pj + ".1", 1e-3, 1, false, bn.project, missing));
  }
  chk(pack_conv(p, F + "12.0.weight", "", F + "12.1", 1e-3, 1, false, p->last, missing));
  }
  if (p->has_fpn) {
  for (int i = 0; i < 4; ++i) {
    const std::string wn = "backbone.fpn.lateral_convs." + std::to_string(i) + ".weight";
    chk(pack_conv(p, wn, "", "", 0, 1, false, p->lat[i], missing));
    if (const HostT* lw = get(p, wn, missing)) {
      const size_t cout = (size_t)lw->shape[0], cin = lw->data.size() / std::max<size_t>(cout, 1);
      double smax = 0.0;
      for (size_t o = 0; o < cout; ++o) {
        double sum = 0.0;
        for (size_t k = 0; k < cin; ++k) sum += std::fabs((double)lw->data[o * cin + k]);
        smax = std::max(smax, sum);
      }
      float sf = (float)smax;
      if ((double)sf < smax) sf = std::nextafter(sf, INFINITY);
      p->lat_S[i] = sf;
    }
  }
  chk(pack_conv(p, "backbone.fpn.fpn_convs.0.0.weight", "", "backbone.fpn.fpn_convs.0.1", 1e-5, 3, false,
                p->fpn0, missing));
  if (precision != KPD_PRECISION_FP32 && rc == KPD_OK && missing.empty()) chk(pack_fpn0x(p, p->fpn0, p->lat[0]));
  // levels 1-3 (dead in the model's forward; MobileNetV3Wrapper.forward returns them)
  for (int i = 1; i < 4; ++i) {
    const std::string c = "backbone.fpn.fpn_convs." + std::to_string(i);
    if (p->t.count(c + ".0.weight"))
      chk(pack_conv(p, c + ".0.weight", "", c + ".1", 1e-5, 3, false, p->fpn_lv[i - 1], missing));
  }
  }
  if (p->has_ca) {
  chk(pack_plain(p, "channel_attention.fc.0.weight", &p->ca_w0, missing, 8 * 128));
  chk(pack_plain(p, "channel_attention.fc.0.bias", &p->ca_b0, missing, 8));
  chk(pack_plain(p, "channel_attention.fc.2.weight", &p->ca_w2, missing, 128 * 8));
  chk(pack_plain(p, "channel_attention.fc.2.bias", &p->ca_b2, missing, 128));
  }
  const std::string Hh = "heatmap_head.";
  if (p->has_hm) {
  chk(pack_plain(p, Hh + "channel_attention.fc.0.weight", &p->hca_w0, missing, 4 * 64));
  chk(pack_plain(p, Hh + "channel_attention.fc.0.bias", &p->hca_b0, missing, 4));
  chk(pack_plain(p, Hh + "channel_attention.fc.2.weight", &p->hca_w2, missing, 64 * 4));
  chk(pack_plain(p, Hh + "channel_attention.fc.2.bias", &p->hca_b2, missing, 64));
  chk(pack_plain(p, Hh + "spatial_attention.conv.weight", &p->sa_w, missing, 98));
  chk(pack_plain(p, Hh + "spatial_attention.conv.bias", &p->sa_b, missing, 1));
  const bool bf = precision == KPD_PRECISION_MIXED;
  chk(pack_conv(p, Hh + "deconv_layers.0.weight", Hh + "deconv_layers.0.bias", Hh + "deconv_layers.1", 1e-5, 3,
                bf, p->hm1, missing));
  chk(pack_conv(p, Hh + "deconv_layers.4.weight", Hh + "deconv_layers.4.bias", Hh + "deconv_layers.5", 1e-5, 3,
                bf, p->hm2, missing));
  chk(pack_conv(p, Hh + "final_layer.0.weight", Hh + "final_layer.0.bias", Hh + "final_layer.1", 1e-5, 3, bf,
                p->hm3, missing));
  if (precision == KPD_PRECISION_SPLIT && rc == KPD_OK && missing.empty()) {
    chk(pack_split_hm(p, p->hm1));
    chk(pack_split_hm(p, p->hm2));
    chk(pack_split_hm(p, p->hm3));
  }
  chk(pack_plain(p, Hh + "final_layer.3.weight", &p->fin_w, missing, 17 * 64));
  chk(pack_plain(p, Hh + "final_layer.3.bias", &p->fin_b, missing, 17));
  }
  {
    std::vector<float> z(128, 0.f);
    chk(upload(p, z, &p->zero_bias));
  }
  // person-detector glue: box_heads[0] ++ cls_heads[0] -> one 1x1 conv (45 outputs)
  if (has_pd) {
    const HostT* bw = get(p, "person_detector.box_heads.0.weight", missing);
    const HostT* bb = get(p, "person_detector.box_heads.0.bias", missing);
    const HostT* cw = get(p, "person_detector.cls_heads.0.weight", missing);
    const HostT* cb = get(p, "person_detector.cls_heads.0.bias", missing);
    const HostT* an = get(p, "person_detector.anchors", missing);
    if (bw && bb && cw && cb && an) {
      if (bw->shape[0] != 36 || cw->shape[0] != 9 || an->data.size() != (size_t)56 * 56 * 9 * 4)
        return fail(KPD_EINVAL, "person head expects 9 anchors on the 56x56 grid (1 class)");
      HostT w, b;
      w.shape = {45, bw->shape[1], 1, 1};
      w.data = bw->data;
      w.data.insert(w.data.end(), cw->data.begin(), cw->data.end());
      b.shape = {45};
      b.data = bb->data;
      b.data.insert(b.data.end(), cb->data.begin(), cb->data.end());
      p->t["__pd.weight"] = std::move(w);
      p->t["__pd.bias"] = std::move(b);
      chk(pack_conv(p, "__pd.weight", "__pd.bias", "", 0, 1, false, p->pd, missing));
      chk(upload(p, an->data, &p->anchors));
    }
  }
  // KEYPOINT_HEAD (optional)
  p->has_kh = p->t.count("keypoint_head.spatial_attention.0.weight") > 0;
  if (p->has_kh) {
    const std::string K = "keypoint_head.", R = K + "regression_branch.", V = K + "visibility_branch.";
    chk(pack_conv(p, K + "spatial_attention.0.weight", K + "spatial_attention.0.bias", "", 0, 1, false, p->kh_sa1,
                  missing));
    chk(pack_plain(p, K + "spatial_attention.2.weight", &p->kh_sa2_w, missing, 64));
    chk(pack_plain(p, K + "spatial_attention.2.bias", &p->kh_sa2_b, missing, 1));
    DevConv* ds[2] = {&p->kh_ds1, &p->kh_ds2};
    DevConv* rb[2] = {&p->kh_rb1, &p->kh_rb2};
    float** bs[2] = {&p->kh_bn1a_s, &p->kh_bn1b_s};
    float** bt[2] = {&p->kh_bn1a_t, &p->kh_bn1b_t};
    for (int i = 0; i < 2; ++i) {
      const std::string B = R + std::to_string(i) + ".";
      chk(pack_conv(p, B + "conv1.0.weight", B + "conv1.0.bias", B + "conv1.1", 1e-5, 3, false, *rb[i], missing));
      if (p->t.count(B + "downsample.0.weight"))
        chk(pack_conv(p, B + "downsample.0.weight", B + "downsample.0.bias", B + "downsample.1", 1e-5, 1, false,
                      *ds[i], missing));
      chk(pack_bn_affine(p, B + "bn1", rb[i]->cout_p ? rb[i]->cout_p : 64, bs[i], bt[i], missing));
    }
    chk(pack_conv(p, R + "2.weight", R + "2.bias", R + "3", 1e-5, 3, false, p->kh_c3, missing));
    chk(pack_conv(p, R + "7.weight", R + "7.bias", "", 0, 1, false, p->kh_lr, missing));
    chk(pack_plain(p, R + "8.weight", &p->kh_lnr_g, missing, 256));
    chk(pack_plain(p, R + "8.bias", &p->kh_lnr_b, missing, 256));
    chk(pack_plain(p, R + "11.weight", &p->kh_fr_w, missing, 34 * 256));
    chk(pack_plain(p, R + "11.bias", &p->kh_fr_b, missing, 34));
    chk(pack_conv(p, V + "0.weight", V + "0.bias", V + "1", 1e-5, 3, false, p->kh_v1, missing));
    chk(pack_conv(p, V + "5.weight", V + "5.bias", "", 0, 1, false, p->kh_lv, missing));
    chk(pack_plain(p, V + "6.weight", &p->kh_lnv_g, missing, 128));
    chk(pack_plain(p, V + "6.bias", &p->kh_lnv_b, missing, 128));
    chk(pack_plain(p, V + "9.weight", &p->kh_fv_w, missing, 51 * 128));
    chk(pack_plain(p, V + "9.bias", &p->kh_fv_b, missing, 51));
    if (rc == KPD_OK && missing.empty()) {
      const int in = p->kh_lr.cin;
      int o = 1;
      while (16 * (o + 1) * (o + 1) <= in) ++o;
      if (16 * o * o != in || p->kh_c3.cout != 16 || p->kh_v1.cout != 32 || p->kh_lv.cin != 512 ||
          p->kh_sa1.cin != 128 || p->kh_sa1.cout != 64)
        return fail(KPD_EINVAL, "KEYPOINT_HEAD shape not supported (needs in 128, regression 32, square pool)");
      p->kh_o = o;
    }
    // split KEYPOINT_HEAD convs (the default channel plan: ResidualBlocks
    // 128 -> 64 -> 32 with downsamples, 3x3 32 -> 16, visibility 128 -> 32)
    const bool std_kh = p->kh_rb1.cin == 128 && p->kh_rb1.cout == 64 && p->kh_ds1.w && p->kh_rb2.cin == 64 &&
                        p->kh_rb2.cout == 32 && p->kh_ds2.w && p->kh_c3.cin == 32 && p->kh_v1.cin == 128;
    static const bool no_kh_split = kpd_diag_env("KPD_NO_KH_SPLIT") != nullptr;   // A/B switch
    if (precision != KPD_PRECISION_FP32 && rc == KPD_OK && missing.empty() && std_kh && !no_kh_split) {
      chk(pack_split_kh(p, p->kh_s[0], 128, 128, 10, {{&p->kh_rb1, &p->kh_ds1, p->kh_bn1a_s, p->kh_bn1a_t, 0},
                                                      {&p->kh_v1, nullptr, nullptr, nullptr, 64}}));
      p->kh_s[0].ns = 64; p->kh_s[0].nf = 32;
      chk(pack_split_kh(p, p->kh_s[1], 64, 64, 10, {{&p->kh_rb2, &p->kh_ds2, p->kh_bn1b_s, p->kh_bn1b_t, 0}}));
      p->kh_s[1].ns = 32; p->kh_s[1].nf = 0;
      chk(pack_split_kh(p, p->kh_s[2], 32, 64, 9, {{&p->kh_c3, nullptr, nullptr, nullptr, 0}}));
      p->kh_s[2].ns = 0; p->kh_s[2].nf = 16;
      if (p->kh_sa1.cin_p == 128 && p->kh_sa1.cout_p == 64) chk(pack_split_1x1(p, p->kh_sa1));   // kh_att2_kernel
      p->kh_split = rc == KPD_OK;
    }
  }
  if (!missing.empty()) return fail(KPD_ESTATE, "missing tensors: " + missing);
  if (rc != KPD_OK) return rc;
  // shape checks the kernels rely on
  if (p->has_fpn && (p->fpn0.cin != 128 || p->fpn0.cout != 128)) return fail(KPD_EINVAL, "fpn_convs.0 must be 128->128");
  if (p->has_hm && (p->hm1.cin != 64 || p->hm3.cout != 64 || p->hm1.cout != p->hm2.cin || p->hm2.cout != p->hm3.cin))
    return fail(KPD_EINVAL, "heatmap head channel chain mismatch");
  if (p->has_body && p->bn[0].cfg.cin != 16) return fail(KPD_EINVAL, "bad body");
  p->finalized = true;
  ++p->ws_epoch;
  return KPD_OK;
}

// Images per forward pass: fpn0x_kernel's 32-bit store offsets (output and
// tap0 / lateral-1 split rows) and its per-image unscale table bound the
// batch one launch may cover; kpd_forward runs larger batches as several
// passes (images are independent, so results do not depend on the split).
static int max_pass_images(int H, int W) {
  const long hf = (H - 1) / 2 + 1, wf = (W - 1) / 2 + 1;
  const long by_extent = 0x7fffffffL / (hf * wf * 512);
  return (int)std::max(1L, std::min<long>(kFpn0xMaxImg, by_extent));
}

// FPN level 0 by linearity applies (mixed precision, packed composite weights,
// lateral 1 an exact 4x nearest upsample of the level-0 grid)
static bool fpn0x_ok(const kpd_plan* p, const Dims& d) {
  static const bool no_lin = kpd_diag_env("KPD_NO_FPN0X") != nullptr;   // A/B switch
  return p->precision != KPD_PRECISION_FP32 && !no_lin && p->fpn0x.w0 != nullptr && d.Hf == 4 * d.h[3] &&
         d.Wf == 4 * d.w[3] && (long)((d.h[3] * d.w[3] + 255) / 256) * 256 < 65536;
}

static int ensure_work(kpd_plan* p, const Dims& d, int k, hipStream_t st) {
  if (p->have_work[k] && d.fits(p->dims[k])) return KPD_OK;
  // re-carving (a larger shape) rewrites and re-zeroes the buffers: let every
  // earlier use of this workspace, on whichever stream, finish first (rare)
  if (p->have_work[k]) HIP_TRY(hipDeviceSynchronize());
  Work w;
  const size_t need = carve(p, d, nullptr, w);
  if (need > p->ws_bytes[k]) {
    if (p->ws[k]) HIP_TRY(hipFree(p->ws[k]));
    p->ws[k] = nullptr;
    HIP_TRY(hipMalloc(&p->ws[k], need));
    p->ws_bytes[k] = need;
  }
  carve(p, d, reinterpret_cast<char*>(p->ws[k]), p->work[k]);
  p->work[k].sc_dirty = true;
  ++p->ws_epoch;   // captured graphs hold the old carve's addresses
  // zero once: the padded heatmap-conv maps keep their zero border (the
  // kernels write interiors only)
  if (hm_padded(p)) HIP_TRY(hipMemsetAsync(p->ws[k], 0, need, st));
  p->dims[k] = d;
  p->have_work[k] = true;
  return KPD_OK;
}

// HeatmapHead (heatmap_head.py:81-151) on the [R][56][56][64] NHWC ROI
// features in w.roi with their per-row statistics in w.roi_stats: channel
// attention, spatial attention, the three 3x3 convs and the final 1x1 +
// sigmoid, heatmaps written at the ROIs' slots (w.slot, P).  parts selects
// the stages (KPD_HEAD_*; a disabled attention uses weights 1); sw_out
// (nullable) receives the spatial weights [R][56][56].
static int run_heatmap_head(kpd_plan* p, Work& w, int R, int P, float* heat_out, hipStream_t st, int parts,
                            float* sw_out, unsigned long long* stamps2, unsigned long long* stamps3,
                            unsigned long long* stamps1 = nullptr, int abs_in = 0) {
  std::unique_ptr<Stage> att_stage(new Stage(p, "hm_attention", st));
  // split: per-ROI operand bounds, hsc[r] = {max|xs| (written here), max|h1| (conv 1)}
  const bool hsplit = p->precision == KPD_PRECISION_SPLIT;
  HIP_TRY(launch_hm_chattn(w.roi_stats, R, p->hca_w0, p->hca_b0, p->hca_w2, p->hca_b2, w.cw,
                           hsplit ? w.hsc : nullptr, st, abs_in));
  if (!(parts & KPD_HEAD_CHANNEL_ATT)) HIP_TRY(launch_fill(w.cw, (long)R * 64, 1.f, st));
  const bool bf = p->precision == KPD_PRECISION_MIXED;
  const int xs_mode = hsplit ? 3 : bf ? (hm_padded(p) ? 2 : 1) : 0;
  static const bool att_2k = kpd_diag_env("KPD_HM_ATT_2K") != nullptr;   // A/B: pool and apply as two launches
  if (att_2k) {
    HIP_TRY(launch_hm_spool(w.roi, w.cw, R, w.smap, st));
    HIP_TRY(launch_hm_sapply(w.roi, w.cw, w.smap, p->sa_w, p->sa_b, R, w.xs, xs_mode, st, w.hsc,
                             (parts & KPD_HEAD_SPATIAL_ATT) != 0, sw_out));
  } else {
    HIP_TRY(launch_hm_attn(w.roi, w.cw, p->sa_w, p->sa_b, R, w.xs, xs_mode, st, w.hsc,
                           (parts & KPD_HEAD_SPATIAL_ATT) != 0, sw_out));
  }
  att_stage.reset();
  if (!(parts & KPD_HEAD_CONVS)) return KPD_OK;
  // bounds: |xs| <= U0; |h1| <= bc1 + bs1 U0; |h2| <= bc2 + bs2 max|h1| (the
  // exponent each producer scales by and its consumer unscales by)
  const HmSplit sp1{w.hsc, 0.f, 1.f, 0, p->hm1.bc, p->hm1.bs, 0, 1};
  const HmSplit sp2{w.hsc, p->hm1.bc, p->hm1.bs, 0, p->hm2.bc, p->hm2.bs, 1, -1};
  const HmSplit sp3{w.hsc, p->hm2.bc, p->hm2.bs, 1, 0.f, 0.f, -1, -1};
  std::unique_ptr<Stage> c1(new Stage(p, "hm_conv1", st));
  if (int rc = hm_conv(p, p->hm1, w.xs, R, 64, w.h1, 1, st, nullptr, stamps1, &sp1)) return rc;
  c1.reset();
  std::unique_ptr<Stage> c2(new Stage(p, "hm_conv2", st));
  if (int rc = hm_conv(p, p->hm2, w.h1, R, p->hm1.cout_p, w.h2, 1, st, nullptr, stamps2, &sp2))
    return rc;
  c2.reset();
  std::unique_ptr<Stage> c3(new Stage(p, "hm_conv3", st));
  // mixed / split: the final 1x1 + sigmoid runs in conv 3's epilogue (no h3 round trip)
  static const bool no_fin_fuse = kpd_diag_env("KPD_NO_FINAL_FUSE") != nullptr;   // A/B switch
  const bool fin_fused = (p->hm3.bf16 || p->hm3.ws) && p->hm3.cout_p == 64 && (!no_fin_fuse || p->hm3.ws);
  const HmFinal fin{p->fin_w, p->fin_b, w.slot, P, heat_out};
  if (int rc = hm_conv(p, p->hm3, w.h2, R, p->hm2.cout_p, w.h3, 2, st, fin_fused ? &fin : nullptr, stamps3, &sp3))
    return rc;
  c3.reset();
  if (!fin_fused) HIP_TRY(launch_hm_final(w.h3, R, p->fin_w, p->fin_b, w.slot, P, heat_out, st));
  return KPD_OK;
}

// KEYPOINT_HEAD (keypoint_head.py:50-62, ResidualBlock :64-90) on the
// [R][56][56][128] NHWC ROI features in w.kx; outputs at the ROIs' slots.
// bound (split path): the bound of |x| for ROI r is bound[(r / bdiv) * bstride]
// x_ready: the first conv's split operand (x * attention) is already in
// w.kxs (roi_kh_kernel wrote it with the HeatmapHead's ROI align).
static int run_keypoint_head(kpd_plan* p, Work& w, int R, int P, float* kh_kpts, float* kh_vis, hipStream_t st,
                             const float* bound, int bdiv, int bstride, bool x_ready = false,
                             unsigned long long* const* stamps = nullptr) {
  const size_t px = (size_t)R * 3136;
  if (p->kh_split && w.kxs) {
    // fp32-accurate split products on zero-bordered maps (hmconv_kernel MODE 2):
    // [ResidualBlock 1 (+ downsample as a tenth tap) | visibility conv] ->
    // ResidualBlock 2 (+ downsample) -> regression 3x3; ReLU6 bounds every
    // intermediate by 6, the input by the FPN level-0 maximum.  The spatial
    // attention (1x1 convs + sigmoid + apply) is one kernel writing the first
    // conv's operand (KPD_KH_ATT1=1: the fp32 1x1 conv + apply kernel, A/B).
    static const bool att1 = kpd_diag_env("KPD_KH_ATT1") != nullptr;
    if (x_ready) {
      // (roi_kh_kernel)
    } else if (att1 || !p->kh_sa1.ws) {
      if (int rc = conv(p->kh_sa1, w.kx, R, 56, 56, 128, w.ksa, ACT_RELU6, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
        return rc;
      HIP_TRY(launch_kh_att_split(w.kx, w.ksa, p->kh_sa2_w, p->kh_sa2_b, R, bound, bdiv, bstride, w.hsc, w.kxs, st));
    } else {
      HIP_TRY(launch_kh_att2(w.kx, p->kh_sa1.ws, p->kh_sa1.w_exp, p->kh_sa1.b, p->kh_sa2_w, p->kh_sa2_b, R, bound,
                             bdiv, bstride, w.hsc, w.kxs, st));
    }
    const void* ins[3] = {w.kxs, w.kr1s, w.kr2s};
    void* outs[3] = {w.kr1s, w.kr2s, nullptr};
    float* outf[3] = {w.kv1, nullptr, w.kr3};
    for (int i = 0; i < 3; ++i) {
      const KhSplit& k = p->kh_s[i];
      HmConvArgs h{};
      h.in = ins[i]; h.wt = k.ws; h.bias = k.b; h.out = outs[i]; h.outf = outf[i];
      h.R = R; h.cin = k.cin; h.cout = k.cout; h.ntap = k.ntap; h.ns = k.ns; h.nf = k.nf;
      h.kh_ps = k.ps; h.kh_pt = k.pt; h.kh_bd = k.ntap == 10 ? k.bd : nullptr;
      h.split = 1; h.hsc = w.hsc; h.w_exp = k.w_exp;
      h.in_c = i == 0 ? 0.f : 6.f; h.in_s = i == 0 ? 1.f : 0.f; h.in_idx = 2;
      h.out_c = 6.f; h.out_s = 0.f; h.out_idx = k.ns > 0 ? 2 : -1; h.amax_idx = -1;
      h.stamps = stamps ? stamps[i] : nullptr;   // (KPD_STAMPS, diagnostic build)
      HIP_TRY(launch_hmconv(h, st));
    }
    const int o = p->kh_o, kr = pad16(16 * o * o);
    if (kr != 16 * o * o) HIP_TRY(hipMemsetAsync(w.kpr, 0, sizeof(float) * R * kr, st));
    HIP_TRY(launch_kh_pool(w.kr3, R, 16, o, w.kpr, kr, st));
    HIP_TRY(launch_kh_pool(w.kv1, R, 32, 4, w.kpv, 512, st));
    if (int rc = conv(p->kh_lr, w.kpr, R, 1, 1, kr, w.klr, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
      return rc;
    if (int rc = conv(p->kh_lv, w.kpv, R, 1, 1, 512, w.klv, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
      return rc;
    HIP_TRY(launch_kh_final(w.klr, p->kh_lr.cout_p, w.klv, p->kh_lv.cout_p, p->kh_lnr_g, p->kh_lnr_b, p->kh_fr_w,
                            p->kh_fr_b, p->kh_lnv_g, p->kh_lnv_b, p->kh_fv_w, p->kh_fv_b, w.slot, R, P, kh_kpts,
                            kh_vis, st));
    return KPD_OK;
  }
  if (int rc = conv(p->kh_sa1, w.kx, R, 56, 56, 128, w.ksa, ACT_RELU6, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
    return rc;
  HIP_TRY(launch_kh_att(w.kx, w.ksa, p->kh_sa2_w, p->kh_sa2_b, px, st));
  // ResidualBlock(128 -> 64): relu6(relu6(bn1(relu6(conv_bn(x)))) + downsample(x))
  const float* id1 = w.kx;
  if (p->kh_ds1.w) {
    if (int rc = conv(p->kh_ds1, w.kx, R, 56, 56, 128, w.kds1, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
      return rc;
    id1 = w.kds1;
  }
  if (int rc = conv_post(p->kh_rb1, w.kx, R, 56, 56, 128, w.krb1, ACT_RELU6, p->kh_bn1a_s, p->kh_bn1a_t,
                         ACT_RELU6, id1, ACT_RELU6, st))
    return rc;
  const float* id2 = w.krb1;
  if (p->kh_ds2.w) {
    if (int rc = conv(p->kh_ds2, w.krb1, R, 56, 56, p->kh_rb1.cout_p, w.kds2, ACT_NONE, nullptr, 0, 0, nullptr,
                      nullptr, 0, 0, st))
      return rc;
    id2 = w.kds2;
  }
  if (int rc = conv_post(p->kh_rb2, w.krb1, R, 56, 56, p->kh_rb1.cout_p, w.krb2, ACT_RELU6, p->kh_bn1b_s,
                         p->kh_bn1b_t, ACT_RELU6, id2, ACT_RELU6, st))
    return rc;
  if (int rc = conv(p->kh_c3, w.krb2, R, 56, 56, p->kh_rb2.cout_p, w.kr3, ACT_RELU6, nullptr, 0, 0, nullptr,
                    nullptr, 0, 0, st))
    return rc;
  if (int rc = conv(p->kh_v1, w.kx, R, 56, 56, 128, w.kv1, ACT_RELU6, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
    return rc;
  const int o = p->kh_o, kr = pad16(16 * o * o);
  if (kr != 16 * o * o) HIP_TRY(hipMemsetAsync(w.kpr, 0, sizeof(float) * R * kr, st));
  HIP_TRY(launch_kh_pool(w.kr3, R, 16, o, w.kpr, kr, st));
  HIP_TRY(launch_kh_pool(w.kv1, R, 32, 4, w.kpv, 512, st));
  // the two Linear layers as 1x1 MFMA GEMMs over all ROIs (M = R)
  if (int rc = conv(p->kh_lr, w.kpr, R, 1, 1, kr, w.klr, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
    return rc;
  if (int rc = conv(p->kh_lv, w.kpv, R, 1, 1, 512, w.klv, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
    return rc;
  HIP_TRY(launch_kh_final(w.klr, p->kh_lr.cout_p, w.klv, p->kh_lv.cout_p, p->kh_lnr_g, p->kh_lnr_b, p->kh_fr_w,
                          p->kh_fr_b, p->kh_lnv_g, p->kh_lnv_b, p->kh_fv_w, p->kh_fv_b, w.slot, R, P, kh_kpts,
                          kh_vis, st));
  return KPD_OK;
}

// One sub-batch of the forward pass on one stream, with workspace k.
// Arguments are validated by kpd_forward; pointers are already offset to the
// sub-batch's first image.  Debug buffers are recorded only when debug != 0.
static int forward_one(kpd_plan* p, int k, bool debug, const float* image, int B, int C, int H, int W, float* boxes,
                       int NB, int P, int flags, float* kpts, float* vis, float* heat, float* kh_kpts, float* kh_vis,
                       float* box_scores, int32_t* topk_out, hipStream_t st, hipEvent_t mark_ev = nullptr,
                       int mark_at = 0) {
  const bool detect = flags & KPD_FLAG_DETECT, dual = flags & KPD_FLAG_DUAL_HEAD;
  // pipelined sub-batches: mark_ev is recorded once this sub-batch has passed
  // stage mark_at (1 body, 2 FPN laterals, 3 FPN level 0, 4 top-k, 5 ROI align)
  auto mark = [&](int at) -> int {
    if (mark_ev && mark_at == at) HIP_TRY(hipEventRecord(mark_ev, st));
    return KPD_OK;
  };
  Dims d;
  d.B = B; d.H = H; d.W = W; d.NB = NB; d.P = P; d.flags = flags & ~KPD_FLAG_FULL_LEVEL0;   // (no workspace effect)
  d.h[0] = (H - 1) / 2 + 1; d.w[0] = (W - 1) / 2 + 1;
  for (int i = 0; i < 11; ++i) {
    const int k = kBneck[i].k, s = kBneck[i].s, pd = (k - 1) / 2;
    d.h[i + 1] = (d.h[i] + 2 * pd - k) / s + 1;
    d.w[i + 1] = (d.w[i] + 2 * pd - k) / s + 1;
  }
  d.Hf = d.h[0]; d.Wf = d.w[0];
  const int HWf = d.Hf * d.Wf;
  // split (fp32-accurate f16 hi + lo) FPN level 0 by linearity: when lateral 1
  // is an exact 4x nearest upsample of the level-0 grid (kpd_forward caps the
  // pass at max_pass_images, which keeps the 31-bit buffer extents); other
  // geometries run the fp32 level-0 conv
  const bool lin = fpn0x_ok(p, d) && B <= max_pass_images(H, W);
  const int TM = conv_tile_m();
  const int tpc = (d.h[3] * d.w[3] + 255) / 256;   // fpn0x tiles per (position class, image)
  d.fused_stats = lin || (HWf % TM) == 0;
  d.tiles = lin ? 16 * tpc : (d.fused_stats ? HWf / TM : std::min(64, HWf));
  if (int rc = ensure_work(p, d, k, st)) return rc;
  Work& w = p->work[k];
  g_splitk = w.splitk;
  std::map<std::string, std::pair<const void*, size_t>> dbg;

  // KPD_STAMPS: per-workgroup phase stamps of the SE-block kernels (debug
  // buffers "stamps_exdw_<i>" / "stamps_seproj_<i>", single-stream forwards)
  static const bool want_stamps = kpd_diag_env("KPD_STAMPS") != nullptr;
  constexpr size_t kStampWords = 1 << 20;
  if (want_stamps && !p->stamps) {
    HIP_TRY(hipMalloc(&p->stamps, kStampWords * 8));
    p->allocs.push_back(p->stamps);
  }
  size_t stamp_off = 0;
  auto take_stamps = [&](const std::string& name, size_t wgs) -> unsigned long long* {
    if (!want_stamps || !debug || stamp_off + wgs * 8 > kStampWords) return nullptr;
    unsigned long long* r = p->stamps + stamp_off;
    stamp_off += wgs * 8;
    dbg[name] = {r, wgs * 64};
    p->debug[name] = {r, wgs * 64};   // (p->debug is replaced by dbg mid-forward; heads register late)
    return r;
  };

  // ---------------- MobileNetV3-Small body ----------------
  std::unique_ptr<Stage> body_stage(new Stage(p, "body", st));
  if (lin && w.sc_dirty) HIP_TRY(hipMemsetAsync(w.sc, 0, (size_t)2 * B * kAmaxStride * sizeof(float), st));
  if (lin) w.sc_dirty = true;   // until this forward's topk_kernel zeroes the slots it used
  HIP_TRY(launch_stem(image, B, C, H, W, p->stem_w, p->stem_b, w.stem, d.h[0], d.w[0], lin ? w.sc : nullptr, st));
  const float* x = w.stem;
  const float* taps[4] = {w.stem, nullptr, nullptr, nullptr};
  for (int i = 0; i < 11; ++i) {
    const DevBneck& bn = p->bn[i];
    const int hi = d.h[i], wi = d.w[i], ho = d.h[i + 1], wo = d.w[i + 1];
    const int inp = pad16(bn.cfg.cin);
    // coarse maps: expand + depthwise (+ SE means) fused when the image fits LDS
    ExDwArgs xa{};
    xa.x = x; xa.Hi = hi; xa.Wi = wi; xa.cin_p = inp;
    xa.we = bn.has_exp ? static_cast<const float*>(bn.expand.w) : nullptr;
    xa.be = bn.has_exp ? bn.expand.b : nullptr;
    xa.act_e = bn.cfg.act; xa.wd = bn.dw.w; xa.bd = bn.dw.b; xa.act_d = bn.dw.act; xa.Ep = bn.dw.Cp;
    xa.out = w.d[i]; xa.Ho = ho; xa.Wo = wo; xa.pooled = bn.cfg.se ? w.pool : nullptr;
    bool fused = false;
    static const bool no_fuse = kpd_diag_env("KPD_NO_FUSE") != nullptr;   // A/B switch for measurements
    // no SE: the whole block (expand, depthwise, project, residual) in one kernel on row tiles
    // fused by default only at stride 2 (features.2: -31 us per step); the stride-1
    // block (features.3) measured 6 us slower fused than as three kernels.
    // KPD_FIR_MASK (bit i = block i) overrides for A/B runs.
    static const int fir_mask = kpd_diag_env("KPD_FIR_MASK") ? atoi(kpd_diag_env("KPD_FIR_MASK")) : -1;
    const bool fir_on = fir_mask < 0 ? bn.cfg.s == 2 : ((fir_mask >> i) & 1) != 0;
    // features.1: 16 channels, no expand, SE -> depthwise + tile sums, excitation + project
    static const bool no_f1 = kpd_diag_env("KPD_NO_F1") != nullptr;   // A/B switch
    if (!no_f1 && !bn.has_exp && bn.cfg.se && bn.dw.Cp == 16 && bn.cfg.cout == 16 && bn.project.cout_p == 16 &&
        bn.project.cin_p == 16 && bn.project.k == 1 && !bn.project.bf16 && bn.se.sq <= 16 && bn.dw.k == 3 &&
        !(bn.cfg.s == 1 && bn.cfg.cin == bn.cfg.cout) && 4 * ((wo + 3) / 4) * 4 <= 256) {
      int nt = 0;
      HIP_TRY(launch_dwsum(x, B, hi, wi, bn.dw.w, bn.dw.b, bn.dw.act, w.d[i], ho, wo, bn.dw.k, bn.dw.s, w.separt, &nt,
                           st));
      HIP_TRY(launch_se16_proj(w.d[i], B, ho * wo, nt, w.separt, bn.se.w1, bn.se.b1, bn.se.w2, bn.se.b2, bn.se.sq,
                               static_cast<const float*>(bn.project.w), bn.project.b, w.o[i], st));
      x = w.o[i];
      continue;
    }
    // features.2 + features.3 (3x3 stride 2, then 3x3 stride 1 with the
    // residual; no SE) in one launch: fir23.hip
    static const bool no_fir23 = kpd_diag_env("KPD_NO_FIR23") != nullptr;   // A/B switch
    if (!no_fuse && !no_fir23 && i + 1 < 11) {
      const DevBneck& b3 = p->bn[i + 1];
      auto plain = [](const DevConv& c) { return c.k == 1 && !c.bf16; };
      const bool f23 = bn.has_exp && !bn.cfg.se && bn.dw.k == 3 && bn.dw.s == 2 && inp == 16 && plain(bn.expand) &&
                       plain(bn.project) && bn.expand.cin_p == 16 && bn.expand.cout_p == bn.dw.Cp &&
                       bn.project.cin_p == bn.dw.Cp && bn.project.cout_p == 32 && b3.has_exp && !b3.cfg.se &&
                       b3.dw.k == 3 && b3.dw.s == 1 && plain(b3.expand) && plain(b3.project) &&
                       b3.expand.cin_p == 32 && b3.expand.cout_p == b3.dw.Cp && b3.project.cin_p == b3.dw.Cp &&
                       b3.project.cout_p == 32 && b3.cfg.cin == b3.cfg.cout && bn.cfg.cout == b3.cfg.cin;
      Fir23Args fa{};
      fa.x = x; fa.H1 = hi; fa.W1 = wi;
      fa.we2 = static_cast<const float*>(bn.expand.w); fa.be2 = bn.expand.b; fa.wd2 = bn.dw.w; fa.bd2 = bn.dw.b;
      fa.wp2 = static_cast<const float*>(bn.project.w); fa.bp2 = bn.project.b;
      fa.we3 = static_cast<const float*>(b3.expand.w); fa.be3 = b3.expand.b; fa.wd3 = b3.dw.w; fa.bd3 = b3.dw.b;
      fa.wp3 = static_cast<const float*>(b3.project.w); fa.bp3 = b3.project.b;
      fa.E2 = bn.dw.Cp; fa.E3 = b3.dw.Cp;
      fa.act2e = bn.cfg.act; fa.act2d = bn.dw.act; fa.act3e = b3.cfg.act; fa.act3d = b3.dw.act;
      fa.out = w.o[i + 1]; fa.H2 = ho; fa.W2 = wo;
      if (f23 && d.h[i + 2] == ho && d.w[i + 2] == wo && fir23_pick_rows(fa)) {
        fa.stamps = take_stamps("stamps_fir23_0", (size_t)((ho + fa.T - 1) / fa.T) * B);
        HIP_TRY(launch_fir23(fa, B, st));
        ++i;   // features.3 done too
        x = w.o[i];
        if (i + 1 == 3) taps[1] = x;
        continue;
      }
    }
    if (!no_fuse && fir_on && !bn.cfg.se && bn.has_exp && bn.expand.cout_p == bn.dw.Cp &&
        bn.project.cin_p == bn.dw.Cp) {
      FirArgs fa{};
      fa.x = x; fa.Hi = hi; fa.Wi = wi; fa.cin_p = inp;
      fa.we = static_cast<const float*>(bn.expand.w); fa.be = bn.expand.b;
      fa.wd = bn.dw.w; fa.bd = bn.dw.b;
      fa.wp = static_cast<const float*>(bn.project.w); fa.bp = bn.project.b;
      fa.act_e = bn.cfg.act; fa.act_d = bn.dw.act; fa.Ep = bn.dw.Cp; fa.cout_p = bn.project.cout_p;
      fa.out = w.o[i]; fa.Ho = ho; fa.Wo = wo;
      fa.res = bn.cfg.s == 1 && bn.cfg.cin == bn.cfg.cout;
      if (fir_pick_rows(fa, bn.dw.k, bn.dw.s)) {
        fa.stamps = take_stamps("stamps_fir_" + std::to_string(i), (size_t)((ho + fa.TH - 1) / fa.TH) * B);
        HIP_TRY(launch_fir(fa, B, bn.dw.k, bn.dw.s, st));
        x = w.o[i];
        if (i + 1 == 3) taps[1] = x;
        if (i + 1 == 8) taps[2] = x;
        continue;
      }
    }
    if (!no_fuse && hi * wi <= kFuseMaxPix && bn.has_exp && bn.expand.cout_p == bn.dw.Cp && inp % 16 == 0 &&
        inp <= 96) {
      // slice width fixed per layer (never per batch: the fc1 partial sums
      // must not depend on what an image is batched with)
      static const int cs_env = kpd_diag_env("KPD_EXDW_CS") ? atoi(kpd_diag_env("KPD_EXDW_CS")) : 0;   // A/B sweeps
      // 32 channels from 288 expanded channels up, else 16 (48 for the
      // 576-wide blocks measured slower: 188 VGPRs, 30 vs 23 us)
      xa.CS = cs_env > 0 ? cs_env : (bn.dw.Cp >= 288 ? 32 : 16);
      // no SE and under two workgroups per CU: split the output rows in two
      // bands (features.3 at 64 images: 384 -> 768 workgroups)
      static const int nband_env = kpd_diag_env("KPD_EXDW_NBAND") ? atoi(kpd_diag_env("KPD_EXDW_NBAND")) : 0;   // A/B
      xa.nband = !bn.cfg.se && (long)(bn.dw.Cp / xa.CS) * B < 512 ? 2 : 1;
      if (nband_env > 0 && !bn.cfg.se) xa.nband = std::min(nband_env, ho);
      fused = bn.dw.Cp % xa.CS == 0 && exdw_lds_bytes(xa, bn.dw.k) <= 160 * 1024;
    }
    // SE blocks on the coarse maps: fc1 partials in exdw_kernel, then the
    // excitation + project (+ residual) in one seproj_kernel launch
    static const bool no_seproj = kpd_diag_env("KPD_NO_SEPROJ") != nullptr;   // A/B switch
    const bool seproj = fused && bn.cfg.se && !no_seproj && bn.project.k == 1 && !bn.project.bf16 &&
                        bn.project.cin_p == bn.dw.Cp && bn.se.sq <= 144 && bn.se.C % 4 == 0 &&
                        (ho * wo == 48 || ho * wo == 192) && (size_t)(bn.dw.Cp / xa.CS) * bn.se.sq <= kSePartFloats;
    if (fused) {
      if (seproj) {
        xa.part = w.separt; xa.w1 = bn.se.w1; xa.sq = bn.se.sq; xa.C = bn.se.C;
      }
      xa.stamps = take_stamps("stamps_exdw_" + std::to_string(i), (size_t)(bn.dw.Cp / xa.CS) * B * std::max(1, xa.nband));
      HIP_TRY(launch_exdw(xa, B, bn.dw.k, bn.dw.s, st));
    }
    if (seproj) {
      SeProjArgs sa{};
      sa.d = w.d[i]; sa.Po = ho * wo; sa.Ep = bn.dw.Cp;
      sa.part = w.separt; sa.nsl = bn.dw.Cp / xa.CS; sa.sq = bn.se.sq; sa.C = bn.se.C;
      sa.b1 = bn.se.b1; sa.w2t = bn.se.w2; sa.b2 = bn.se.b2;
      sa.wp = static_cast<const float*>(bn.project.w); sa.bp = bn.project.b; sa.cout_p = bn.project.cout_p;
      static const int nt_env = kpd_diag_env("KPD_SEPROJ_NT") ? atoi(kpd_diag_env("KPD_SEPROJ_NT")) : 0;
      // 192-pixel maps: all 48 output channels per workgroup and the rows in
      // four (launch_seproj), so an image's excitation is recomputed by 4
      // workgroups instead of 6 (its fc2 weight columns are most of a
      // workgroup's L2 reads): body -8..-12 us at C2 (same-box A/B)
      sa.NT = nt_env > 0 ? nt_env : (sa.Po == 48 ? 32 : 48);
      if (sa.cout_p % sa.NT) sa.NT = 16;
      const bool res = bn.cfg.s == 1 && bn.cfg.cin == bn.cfg.cout;
      sa.res = res ? x : nullptr;
      sa.out = w.o[i];
      // wide blocks (C >= 288): the excitation as its own launch (one fc2
      // pass per image instead of one per project workgroup)
      static const int se_split_env = kpd_diag_env("KPD_SE_SPLIT") ? atoi(kpd_diag_env("KPD_SE_SPLIT")) : -1;   // A/B
      if (se_split_env == 1 || (se_split_env < 0 && bn.se.C >= 288)) {
        HIP_TRY(launch_se_excite(sa, B, w.sesc[i], st));
        sa.sesc = w.sesc[i];
      }
      sa.stamps = take_stamps("stamps_seproj_" + std::to_string(i), (size_t)(sa.cout_p / sa.NT) * B * 2);   // (x msplit)
      HIP_TRY(launch_seproj(sa, B, st));
      x = w.o[i];
      if (i + 1 == 3) taps[1] = x;
      if (i + 1 == 8) taps[2] = x;
      continue;
    }
    if (!fused) {
      const float* e = x;
      if (bn.has_exp) {
        if (int rc = conv(bn.expand, x, B, hi, wi, inp, w.e[i], bn.cfg.act, nullptr, 0, 0, nullptr, nullptr, 0, 0, st))
          return rc;
        e = w.e[i];
      }
      HIP_TRY(launch_dwconv(e, bn.dw.w, bn.dw.b, w.d[i], B, hi, wi, bn.dw.Cp, ho, wo, bn.dw.k, bn.dw.s, bn.dw.act, st));
    }
    if (bn.cfg.se)
      HIP_TRY(launch_se(w.d[i], B, ho * wo, bn.se.C, bn.se.Cp, bn.se.w1, bn.se.b1, bn.se.w2, bn.se.b2, bn.se.sq,
                        w.sesc[i], st, fused ? w.pool : nullptr));
    const bool res = bn.cfg.s == 1 && bn.cfg.cin == bn.cfg.cout;
    if (int rc = conv(bn.project, w.d[i], B, ho, wo, bn.dw.Cp, w.o[i], ACT_NONE, res ? x : nullptr, ho, wo,
                      bn.cfg.se ? w.sesc[i] : nullptr, nullptr, 0, 0, st))
      return rc;
    x = w.o[i];
    if (i + 1 == 3) taps[1] = x;
    if (i + 1 == 8) taps[2] = x;
  }
  if (int rc = conv(p->last, x, B, d.h[11], d.w[11], pad16(96), w.last, ACT_HSWISH, nullptr, 0, 0, nullptr,
                    nullptr, 0, 0, st))
    return rc;
  taps[3] = w.last;
  body_stage.reset();
  if (p->body_only) {   // kpd_backbone_body
    for (int i = 0; i < 4; ++i) p->body_taps[i] = taps[i];
    return KPD_OK;
  }
  if (int rc = mark(1)) return rc;

  // ---------------- FPN laterals (top-down) + level-0 3x3 ----------------
  const int lh[4] = {d.h[0], d.h[3], d.h[8], d.h[11]}, lw[4] = {d.w[0], d.w[3], d.w[8], d.w[11]};
  std::unique_ptr<Stage> lat_stage(new Stage(p, "fpn_lateral", st));
  // laterals 3 -> 1 in one launch (lateral_chain.hip) when only lateral 1 is
  // consumed (kpd_backbone returns every level: the per-level convs then)
  static const bool no_chain = kpd_diag_env("KPD_NO_LAT_CHAIN") != nullptr;   // A/B switch
  LatChainArgs lc{};
  lc.t1 = taps[1]; lc.t2 = taps[2]; lc.t3 = taps[3];
  lc.L1 = static_cast<const float*>(p->lat[1].w); lc.L2 = static_cast<const float*>(p->lat[2].w);
  lc.L3 = static_cast<const float*>(p->lat[3].w);
  lc.c1 = pad16(kFpnIn[1]); lc.c2 = pad16(kFpnIn[2]); lc.c3 = pad16(kFpnIn[3]);
  lc.c1r = kFpnIn[1]; lc.c2r = kFpnIn[2]; lc.c3r = kFpnIn[3];
  lc.S1 = p->lat_S[1]; lc.S2 = p->lat_S[2]; lc.S3 = p->lat_S[3];
  lc.w_exp0 = p->fpn0x.w_exp0; lc.w_expE = p->fpn0x.w_expE;
  lc.h1 = lh[1]; lc.w1 = lw[1]; lc.h2 = lh[2]; lc.w2 = lw[2]; lc.h3 = lh[3]; lc.w3 = lw[3];
  lc.lat1 = w.lat[1];
  // split: lateral 1 goes straight to the hi|lo rows fpn0x_kernel reads (after the tap0 rows)
  lc.lat1_split = lin ? reinterpret_cast<_Float16*>(reinterpret_cast<char*>(w.lat[0]) + (size_t)B * lh[0] * lw[0] * 64)
                      : nullptr;
  lc.amax = lin ? w.sc : nullptr;
  static const bool no_chain_t0 = kpd_diag_env("KPD_NO_CHAIN_TAP0") != nullptr;   // A/B: tap0 split as its own launch
  if (lin && !no_chain_t0) {
    lc.t0 = taps[0];
    lc.t0_split = reinterpret_cast<_Float16*>(w.lat[0]);
    lc.P0 = lh[0] * lw[0];
  }
  lc.stamps = take_stamps("stamps_latchain_0", (size_t)8 * ((B + 7) / 8 * 8));
  const bool chain = !no_chain && !p->keep_laterals && !p->lat[1].bf16 && !p->lat[2].bf16 && !p->lat[3].bf16 &&
                     p->lat[1].cin_p == lc.c1 && p->lat[2].cin_p == lc.c2 && p->lat[3].cin_p == lc.c3 &&
                     p->lat[1].cout_p == 128 && p->lat[2].cout_p == 128 && p->lat[3].cout_p == 128 &&
                     lateral_chain_ok(lc);
  if (chain) HIP_TRY(launch_lateral_chain(lc, B, st));
  for (int i = 3; i >= 0; --i) {
    if (chain && i > 0) continue;
    const DevConv& L = p->lat[i];
    const float* res = i < 3 ? w.lat[i + 1] : nullptr;
    if (i == 0 && lin) {   // no lateral 0: tap0 and lateral 1 go to the split layouts fpn0x_kernel reads
      char* base = reinterpret_cast<char*>(w.lat[0]);
      if (!chain || !lc.t0)
        HIP_TRY(launch_split_rows(taps[0], B, (long)lh[0] * lw[0], 16, w.sc, 0, p->fpn0x.w_exp0, p->fpn0x.w_expE,
                                  base, st));
      if (!chain)
        HIP_TRY(launch_split_rows(w.lat[1], B, (long)lh[1] * lw[1], 128, w.sc, 1, p->fpn0x.w_exp0,
                                  p->fpn0x.w_expE, base + (size_t)B * lh[0] * lw[0] * 64, st));
      continue;
    }
    if (i == 0 && L.cin_p <= 32) {   // the 16-channel stem tap: a 403 MB/step stream, not a GEMM
      HIP_TRY(launch_lateral_stream(taps[0], L.cin_p, (const float*)L.w, L.b, res, B, lh[0], lw[0], lh[1], lw[1],
                                    w.lat[0], st));
      continue;
    }
    if (int rc = conv(L, taps[i], B, lh[i], lw[i], pad16(kFpnIn[i]), w.lat[i], ACT_NONE, res,
                      i < 3 ? lh[i + 1] : 0, i < 3 ? lw[i + 1] : 0, nullptr, nullptr, 0, 0, st,
                      (i == 1 && lin) ? w.sc + (size_t)B * kAmaxStride : nullptr))
      return rc;
  }
  lat_stage.reset();
  if (int rc = mark(2)) return rc;
  std::unique_ptr<Stage> fpn_stage(new Stage(p, "fpn0", st));
  // caller boxes: level 0 is stored only where the ROI aligns read it (the
  // 400 MB fp32 map per 64 images otherwise; KPD_FLAG_FULL_LEVEL0 stores all)
  const bool footprint = lin && !detect && boxes && NB * P > 0 && !(flags & KPD_FLAG_FULL_LEVEL0) && p->has_ca;
  if (lin) {
    Fpn0xArgs a{};
    char* base = reinterpret_cast<char*>(w.lat[0]);
    a.f_split = base;
    a.l_split = base + (size_t)B * lh[0] * lw[0] * 64;
    a.w0 = p->fpn0x.w0; a.weff = p->fpn0x.weff;
    for (int c = 0; c < 16; ++c) {
      a.cls_woff[c] = p->fpn0x.cls_woff[c];
      a.cls_ng[c] = p->fpn0x.cls_ng[c];
      for (int g = 0; g < kFpn0xMaxGroups; ++g) a.cls_g[c][g] = p->fpn0x.cls_g[c][g];
    }
    a.bias = p->fpn0.b; a.out = w.feat; a.stats = w.stats; a.sc = w.sc; a.sc_n = B;
    a.N = B; a.Hf = d.Hf; a.Wf = d.Wf; a.rh = lh[1]; a.rw = lw[1]; a.tpc = tpc;
    a.w_exp0 = p->fpn0x.w_exp0; a.w_expE = p->fpn0x.w_expE;
    a.f_bytes = (int)std::min<size_t>((size_t)B * lh[0] * lw[0] * 64, 0x7fffffff);
    a.l_bytes = (int)std::min<size_t>((size_t)B * lh[1] * lw[1] * 512, 0x7fffffff);
    a.w0_bytes = p->fpn0x.w0_bytes; a.weff_bytes = p->fpn0x.weff_bytes;
    a.stamps = take_stamps("stamps_fpn0x", (size_t)16 * B * tpc);
    if (footprint) {
      a.fp_boxes = boxes; a.fp_NB = NB; a.fp_P = P;
    }
    HIP_TRY(launch_fpn0x(a, st));
  } else if (int rc = conv(p->fpn0, w.lat[0], B, d.Hf, d.Wf, 128, w.feat, ACT_RELU, nullptr, 0, 0, nullptr,
                           d.fused_stats ? w.stats : nullptr, d.tiles, 0, st)) {
    return rc;
  }
  fpn_stage.reset();
  if (int rc = mark(3)) return rc;
  std::unique_ptr<Stage> topk_stage(new Stage(p, "topk", st));
  if (!p->has_ca) return KPD_OK;   // backbone-only plan (kpd_backbone)
  if (!d.fused_stats) HIP_TRY(launch_channel_stats(w.feat, B, HWf, 128, d.tiles, w.stats, st));
  // given boxes for every image: the slot map rides along with the top-k launch
  const bool slot_in_topk = !detect && NB == B && NB * P > 0 && boxes != nullptr;
  HIP_TRY(launch_topk(w.stats, B, d.tiles, HWf, p->ca_w0, p->ca_b0, p->ca_w2, p->ca_b2, w.topk, w.scores, st,
                      slot_in_topk ? boxes : nullptr, P, slot_in_topk ? w.slot : nullptr, w.imax,
                      lin ? w.sc : nullptr, B));
  if (lin) w.sc_dirty = false;
  topk_stage.reset();
  if (int rc = mark(4)) return rc;
  if (topk_out) HIP_TRY(hipMemcpyAsync(topk_out, w.topk, sizeof(int32_t) * B * 64, hipMemcpyDeviceToDevice, st));
  if (!footprint) dbg["feat0"] = {w.feat, sizeof(float) * (size_t)B * HWf * 128};
  dbg["scores"] = {w.scores, sizeof(float) * (size_t)B * 128};
  dbg["tap0"] = {taps[0], sizeof(float) * (size_t)B * lh[0] * lw[0] * 16};
  dbg["tap1"] = {taps[1], sizeof(float) * (size_t)B * lh[1] * lw[1] * pad16(24)};
  dbg["tap2"] = {taps[2], sizeof(float) * (size_t)B * lh[2] * lw[2] * pad16(48)};
  dbg["tap3"] = {taps[3], sizeof(float) * (size_t)B * lh[3] * lw[3] * 576};
  if (debug) p->debug = dbg;

  // ---------------- person-detector glue (boxes become an output) ----------------
  if (detect) {
    Stage sg(p, "person_detect", st);
    // pool + heads + decode in one launch (person_detect_kernel); KPD_PD_UNFUSED=1:
    // the three launches with the pooled / head maps through HBM (A/B)
    static const bool pd_unfused = kpd_diag_env("KPD_PD_UNFUSED") != nullptr;
    if (!pd_unfused && p->pd.cin == 128 && p->pd.cin_p == 128 && p->pd.cout_p == 48 && !p->pd.bf16 &&
        person_detect_fits(d.Wf)) {
      HIP_TRY(launch_person_detect(w.feat, B, d.Hf, d.Wf, static_cast<const float*>(p->pd.w), p->pd.b, p->anchors, H,
                                   W, p->det_conf, w.pd_boxes, w.pd_scores, st));
    } else {
      HIP_TRY(launch_adaptive_pool56(w.feat, B, d.Hf, d.Wf, 128, w.pd_pool, st));
      if (int rc = conv(p->pd, w.pd_pool, B, 56, 56, 128, w.pd_head, ACT_NONE, nullptr, 0, 0, nullptr, nullptr, 0, 0,
                        st))
        return rc;
      HIP_TRY(launch_person_decode(w.pd_head, B, p->pd.cout_p, p->anchors, H, W, p->det_conf, w.pd_boxes,
                                   w.pd_scores, st));
    }
    HIP_TRY(launch_nms_sets(w.pd_boxes, w.pd_scores, B, 56 * 56 * 9, p->det_iou, P, P, w.pd_keep, w.pd_nkeep,
                            w.pd_alive, st, 1, boxes, box_scores));
  }

  const int R = NB * P;
  if (R == 0) return KPD_OK;

  // ---------------- per-ROI heads ----------------
  float* heat_out = heat ? heat : w.heat;
  // no output memsets: the padding slots are written (zeros / dummy person) by
  // hm_final_kernel, decode_kernel and kh_final_kernel through the slot map
  // dual head, split: one ROI-align pass for both heads with KEYPOINT_HEAD's
  // spatial attention fused (roi_kh_kernel); KPD_NO_ROI_KH=1: the separate
  // launches (A/B)
  static const bool no_roi_kh = kpd_diag_env("KPD_NO_ROI_KH") != nullptr;
  const bool roi_kh = dual && p->kh_split && w.kxs && p->kh_sa1.ws && !no_roi_kh &&
                      kpd_diag_env("KPD_KH_ATT1") == nullptr;
  {
    Stage sg(p, "roi_align", st);
    if (!slot_in_topk) HIP_TRY(launch_slotmap(boxes, NB, P, w.slot, st));
    if (roi_kh)
      HIP_TRY(launch_roi_kh(w.feat, d.Hf, d.Wf, w.topk, boxes, R, P, w.roi, w.roi_stats, p->kh_sa1.ws,
                            p->kh_sa1.w_exp, p->kh_sa1.b, p->kh_sa2_w, p->kh_sa2_b, w.imax, P, 1, w.hsc, w.kxs, st,
                            take_stamps("stamps_roikh_0", (size_t)56 * R)));
    else
      HIP_TRY(launch_roi_align(w.feat, d.Hf, d.Wf, 128, w.topk, boxes, R, P, w.roi, w.roi_stats, st,
                               take_stamps("stamps_roi_0", (size_t)56 * R)));
  }
  if (int rc = mark(5)) return rc;
  if (debug) p->debug["roi"] = {w.roi, sizeof(float) * (size_t)R * 3136 * 64};
  if (int rc = run_heatmap_head(p, w, R, P, heat_out, st, KPD_HEAD_ALL, nullptr,
                                 take_stamps("stamps_hm2", (size_t)(((long)R * kHmRoiPos - kHmPitch + 255) / 224) * 2),
                                 take_stamps("stamps_hm3", (size_t)(((long)R * kHmRoiPos - kHmPitch + 255) / 256) * 2),
                                 take_stamps("stamps_hm1", (size_t)(((long)R * kHmRoiPos - kHmPitch + 255) / 224) * 2)))
    return rc;
  {
    Stage sg(p, "hm_final_decode", st);
    HIP_TRY(launch_decode(heat_out, boxes, w.slot, R, P, kpts, vis, st));
  }
  if (dual) {
    // KEYPOINT_HEAD on ROI-align of the 128-channel FPN level 0 (keypoint_head.py:51-62)
    Stage sg(p, "keypoint_head", st);
    if (!roi_kh) HIP_TRY(launch_roi_align(w.feat, d.Hf, d.Wf, 128, nullptr, boxes, R, P, w.kx, nullptr, st));
    const long khrows = (long)R * kHmRoiPos - kHmPitch;
    // sized for 256-row tiles, the smallest launch_hmconv_kh picks (KPD_KH_BM256 /
    // KPD_KH_TPS1 take them for every conv; by default convs 2 / 3 use 384 / 512)
    unsigned long long* khst[3] = {take_stamps("stamps_kh1", (size_t)((khrows + 255) / 256)),
                                   take_stamps("stamps_kh2", (size_t)((khrows + 255) / 256)),
                                   take_stamps("stamps_kh3", (size_t)((khrows + 255) / 256))};
    if (int rc = run_keypoint_head(p, w, R, P, kh_kpts, kh_vis, st, w.imax, P, 1, roi_kh, khst)) return rc;
  }
  return KPD_OK;
}

static int forward_impl(kpd_plan* p, const float* image, int B, int C, int H, int W, float* boxes, int NB, int P,
                        int flags, float* kpts, float* vis, float* heat, float* kh_kpts, float* kh_vis,
                        float* box_scores, int32_t* topk_out, void* stream);

// launch a captured forward on the caller's stream and mark its completion
static int launch_graph(kpd_plan::GraphEntry& g, hipStream_t st) {
  HIP_TRY(hipGraphLaunch(g.exec, st));
  if (!g.done) HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(g.done, st));
  return KPD_OK;
}

// KPD_GRAPH=1: a forward is a launch-bound chain of ~60 kernels (at one image
// the launches, not the kernels, set the latency), so a repeated call with the
// same signature replays one captured hipGraph.  The first call of a
// signature runs eagerly (it may allocate the workspace); the second is
// captured on the plan's own stream (the caller's may be the legacy default
// stream, which cannot capture) and launched on the caller's; later calls
// only launch.  Stage timing and debug buffers need eager forwards: graphs
// are off while timing is on.
int kpd_forward(kpd_plan* p, const float* image, int B, int C, int H, int W, float* boxes, int NB, int P,
                int flags, float* kpts, float* vis, float* heat, float* kh_kpts, float* kh_vis, float* box_scores,
                int32_t* topk_out, void* stream) {
  if (!p || !p->use_graphs || !p->finalized || p->timing)
    return forward_impl(p, image, B, C, H, W, boxes, NB, P, flags, kpts, vis, heat, kh_kpts, kh_vis, box_scores,
                        topk_out, stream);
  const std::vector<uintptr_t> key = {
      (uintptr_t)image, (uintptr_t)B, (uintptr_t)C, (uintptr_t)H, (uintptr_t)W, (uintptr_t)boxes, (uintptr_t)NB,
      (uintptr_t)P, (uintptr_t)flags, (uintptr_t)kpts, (uintptr_t)vis, (uintptr_t)heat, (uintptr_t)kh_kpts,
      (uintptr_t)kh_vis, (uintptr_t)box_scores, (uintptr_t)topk_out, (uintptr_t)stream, (uintptr_t)p->streams};
  auto eager = [&](void* s_) {
    return forward_impl(p, image, B, C, H, W, boxes, NB, P, flags, kpts, vis, heat, kh_kpts, kh_vis, box_scores,
                        topk_out, s_);
  };
  if (p->graphs.size() >= 64 && !p->graphs.count(key)) {   // signatures that never repeat: bounded
    // the executable graphs may still be running on their callers' streams:
    // each waits for its own last launch only
    HIP_TRY(hipSetDevice(p->device));
    for (auto& kv : p->graphs) HIP_TRY(retire_graph(kv.second));
    p->graphs.clear();
  }
  kpd_plan::GraphEntry& g = p->graphs[key];
  if (g.never) return eager(stream);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (g.exec && g.epoch == p->ws_epoch) {
    HIP_TRY(hipSetDevice(p->device));
    // the graph assumes zeroed split-scale slots (each forward's top-k kernel
    // re-zeroes the ones it used); a forward without top-k in between
    // (kpd_backbone) leaves them set: zero them here, as an eager forward would
    for (int k = 0; k <= kpd_plan::kMaxSub; ++k)
      if (p->have_work[k] && p->work[k].sc_dirty) {
        HIP_TRY(hipMemsetAsync(p->work[k].sc, 0, (size_t)2 * p->dims[k].B * kAmaxStride * sizeof(float), st));
        p->work[k].sc_dirty = false;
      }
    return launch_graph(g, st);
  }
  if (g.exec) {   // stale (re-carve, re-finalize, detector change): its last launch may still be running
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(retire_graph(g));
    g.seen = 0;
  }
  if (g.seen++ == 0)   // eager: allocations and first-use setup happen outside any capture
    return eager(stream);
  HIP_TRY(hipSetDevice(p->device));
  if (!p->graph_st) HIP_TRY(hipStreamCreateWithFlags(&p->graph_st, hipStreamNonBlocking));
  // The captured forward_impl updates host-side workspace state (sc_dirty,
  // and on a re-carve have_work / dims) as if its work had run.  If the
  // capture is abandoned, none of it ran: restore that state, so the eager
  // retry zeroes what it must (a dirty split-scale slot, a re-carved
  // workspace's zero borders).
  bool dirty0[kpd_plan::kMaxSub + 1], have0[kpd_plan::kMaxSub + 1];
  for (int k = 0; k <= kpd_plan::kMaxSub; ++k) {
    dirty0[k] = p->work[k].sc_dirty;
    have0[k] = p->have_work[k];
  }
  auto abandon = [&]() {
    for (int k = 0; k <= kpd_plan::kMaxSub; ++k) {
      p->work[k].sc_dirty = dirty0[k] || p->have_work[k] != have0[k];
      // a slot (re-)carved inside the capture: its memset never ran -> carve again eagerly
      if (p->have_work[k] && !have0[k]) p->have_work[k] = false;
    }
  };
  const long epoch0 = p->ws_epoch;
  HIP_TRY(hipStreamBeginCapture(p->graph_st, hipStreamCaptureModeRelaxed));
  const int rc = forward_impl(p, image, B, C, H, W, boxes, NB, P, flags, kpts, vis, heat, kh_kpts, kh_vis,
                              box_scores, topk_out, p->graph_st);
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(p->graph_st, &graph);
  const bool forced = p->graph_abandon_next;
  p->graph_abandon_next = false;
  if (rc != KPD_OK || ec != hipSuccess || p->ws_epoch != epoch0 || forced) {
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipGetLastError();
    // not capturable here (an allocation or sync inside it, the carve changed
    // under it): this call runs eagerly and reports its own errors
    abandon();
    if (p->ws_epoch != epoch0)   // a re-carve inside the capture: every slot re-carves (and re-zeroes) eagerly
      for (int k = 0; k <= kpd_plan::kMaxSub; ++k) p->have_work[k] = false;
    g.seen = 0;
    return eager(stream);
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) {   // never capturable for this signature: eager from now on
    (void)hipGetLastError();
    abandon();
    g.never = true;
    g.seen = 0;
    return eager(stream);
  }
  g.exec = exec;
  g.epoch = p->ws_epoch;
  return launch_graph(g, st);
}

static int forward_impl(kpd_plan* p, const float* image, int B, int C, int H, int W, float* boxes, int NB, int P,
                        int flags, float* kpts, float* vis, float* heat, float* kh_kpts, float* kh_vis,
                        float* box_scores, int32_t* topk_out, void* stream) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  if (!p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_body || !p->has_fpn || !p->has_ca || !p->has_hm)
    return fail(KPD_ESTATE, "plan lacks backbone / fpn / channel_attention / heatmap_head weights");
  if (!image || B <= 0 || H < 32 || W < 32) return fail(KPD_EINVAL, "bad image shape");
  if (C != p->in_ch) return fail(KPD_EINVAL, "image channels do not match backbone in_channels");
  if (flags & ~(KPD_FLAG_DETECT | KPD_FLAG_DUAL_HEAD | KPD_FLAG_FULL_LEVEL0)) return fail(KPD_EINVAL, "unknown flags");
  const bool detect = flags & KPD_FLAG_DETECT, dual = flags & KPD_FLAG_DUAL_HEAD;
  if (detect && (NB != B || P <= 0 || !boxes)) return fail(KPD_EINVAL, "detect mode: boxes must be [B][P>0][4]");
  if (detect && !p->anchors) return fail(KPD_ESTATE, "person detector weights missing");
  if (dual && !p->has_kh) return fail(KPD_ESTATE, "dual head requested but no keypoint_head.* weights");
  if (dual && NB * P > 0 && (!kh_kpts || !kh_vis)) return fail(KPD_EINVAL, "null dual-head output pointer");
  if (NB < 0 || NB > B || P < 0) return fail(KPD_EINVAL, "bad box batch");
  if (NB * P > 0 && (!boxes || !kpts || !vis)) return fail(KPD_EINVAL, "null box/output pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  p->debug.clear();

  // Images are independent (eval BN, per-image ROI loops -- SURVEY §8(e)), so
  // a large batch runs as S contiguous sub-batches on S streams: the many
  // small latency-bound launches of one sub-batch (MobileNet body, heads)
  // overlap the other's.  Sub-batch 0 uses the caller's stream; the others
  // fork from it and join back before return.  A sub-batch larger than
  // max_pass_images runs as consecutive passes on its stream, reusing its
  // workspace.  Debug buffers need one pass.
  constexpr int kMinSub = 16;
  const int S = std::max(1, std::min({p->streams, kpd_plan::kMaxSub, B / kMinSub}));
  const int cap = max_pass_images(H, W);
  const size_t img_sz = (size_t)C * H * W, per_kp = (size_t)P * 17;
  auto run = [&](int k, bool debug, int b0, int b1, hipStream_t sk, hipEvent_t mev = nullptr, int mat = 0) -> int {
    const int nb = b1 - b0;
    const int npass = (nb + cap - 1) / cap;
    for (int q = 0; q < npass; ++q) {
      const int c0 = b0 + (int)((long)nb * q / npass), c1 = b0 + (int)((long)nb * (q + 1) / npass);
      const int cbox = std::max(0, std::min(NB, c1) - c0);
      auto off = [&](float* ptr, size_t per) { return ptr ? ptr + (size_t)c0 * per : ptr; };
      if (int rc = forward_one(p, k, debug && npass == 1, image + (size_t)c0 * img_sz, c1 - c0, C, H, W,
                               cbox > 0 || detect ? off(boxes, (size_t)P * 4) : nullptr, cbox, P, flags,
                               off(kpts, per_kp * 2), off(vis, per_kp * 3), off(heat, per_kp * 3136),
                               off(kh_kpts, per_kp * 2), off(kh_vis, per_kp * 3), off(box_scores, (size_t)P),
                               topk_out ? topk_out + (size_t)c0 * 64 : nullptr, sk, q + 1 == npass ? mev : nullptr,
                               mat))
        return rc;
    }
    return KPD_OK;
  };
  if (S == 1) return run(0, true, 0, B, st);
  // A/B (KPD_PIPE=<stage>): sub-batch k+1 waits until sub-batch k has passed
  // that stage (1 body .. 5 ROI align) instead of starting at once;
  // KPD_PIPE_PRI=1 runs sub-batches 1.. on high-priority streams, so their
  // workgroups are dispatched ahead of the running sub-batch's at every free CU
  static const int pipe_at = kpd_diag_env("KPD_PIPE") ? atoi(kpd_diag_env("KPD_PIPE")) : 0;
  static const bool pipe_pri = kpd_diag_env("KPD_PIPE_PRI") != nullptr;
  if (!p->fork_ev) HIP_TRY(hipEventCreateWithFlags(&p->fork_ev, hipEventDisableTiming));
  for (int k = 1; k < S; ++k) {
    if (!p->sub_st[k]) HIP_TRY(hipStreamCreateWithFlags(&p->sub_st[k], hipStreamNonBlocking));
    if (!p->join_ev[k]) HIP_TRY(hipEventCreateWithFlags(&p->join_ev[k], hipEventDisableTiming));
    if (pipe_pri && !p->sub_st_pri[k]) {
      int lo = 0, hi = 0;
      HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_TRY(hipStreamCreateWithPriority(&p->sub_st_pri[k], hipStreamNonBlocking, hi));
    }
  }
  for (int k = 0; k < S && pipe_at > 0; ++k)
    if (!p->pipe_ev[k]) HIP_TRY(hipEventCreateWithFlags(&p->pipe_ev[k], hipEventDisableTiming));
  HIP_TRY(hipEventRecord(p->fork_ev, st));
  int rc = KPD_OK;
  for (int k = 0; k < S && rc == KPD_OK; ++k) {
    const int b0 = (int)((long)B * k / S), b1 = (int)((long)B * (k + 1) / S);
    hipStream_t sk = k ? (pipe_pri ? p->sub_st_pri[k] : p->sub_st[k]) : st;
    if (k) HIP_TRY(hipStreamWaitEvent(sk, p->fork_ev, 0));
    if (k && pipe_at > 0) HIP_TRY(hipStreamWaitEvent(sk, p->pipe_ev[k - 1], 0));
    rc = run(k, false, b0, b1, sk, pipe_at > 0 && k + 1 < S ? p->pipe_ev[k] : nullptr, pipe_at);
  }
  for (int k = 1; k < S; ++k) {
    HIP_TRY(hipEventRecord(p->join_ev[k], pipe_pri ? p->sub_st_pri[k] : p->sub_st[k]));
    HIP_TRY(hipStreamWaitEvent(st, p->join_ev[k], 0));
  }
  return rc;
}

int kpd_plan_set_streams(kpd_plan* p, int n) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  if (n < 1 || n > kpd_plan::kMaxSub) return fail(KPD_EINVAL, "streams must be in [1, 4]");
  p->streams = n;
  return KPD_OK;
}

int kpd_plan_set_graphs(kpd_plan* p, int enable) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  if (enable < 0 || enable > 2) return fail(KPD_EINVAL, "enable must be 0, 1 or 2");
  p->use_graphs = enable != 0;
  p->graph_abandon_next = enable == 2;
  return KPD_OK;
}

int kpd_plan_set_detector(kpd_plan* p, float conf_threshold, float nms_iou_threshold) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  if (!(conf_threshold >= 0.f && conf_threshold <= 1.f) || !(nms_iou_threshold >= 0.f && nms_iou_threshold <= 1.f))
    return fail(KPD_EINVAL, "thresholds must be in [0, 1]");
  p->det_conf = conf_threshold;
  p->det_iou = nms_iou_threshold;
  ++p->ws_epoch;   // captured forwards hold the old thresholds
  return KPD_OK;
}

int kpd_plan_timing(kpd_plan* p, int enable) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  p->timing = enable != 0;
  if (p->timing)
    for (auto& kv : p->timers) kv.second.used = 0;
  return KPD_OK;
}

int kpd_plan_timing_stage(kpd_plan* p, const char* stage) {
  if (!p) return fail(KPD_EINVAL, "null plan");
  p->timing_only = stage ? stage : "";
  return KPD_OK;
}

int kpd_plan_timing_query(kpd_plan* p, const char* stage, double* total_ms, int* count) {
  if (!p || !stage || !total_ms || !count) return fail(KPD_EINVAL, "null argument");
  *total_ms = 0.0;
  *count = 0;
  auto it = p->timers.find(stage);
  if (it == p->timers.end()) return KPD_OK;
  for (size_t i = 0; i < it->second.used; ++i) {
    auto& e = it->second.ev[i];
    HIP_TRY(hipEventSynchronize(e.second));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, e.first, e.second));
    *total_ms += ms;
  }
  *count = (int)it->second.used;
  return KPD_OK;
}

int kpd_debug_copy(kpd_plan* p, const char* name, void* dst, size_t bytes, size_t* size_out, void* stream) {
  if (!p || !name) return fail(KPD_EINVAL, "null argument");
  auto it = p->debug.find(name);
  if (it == p->debug.end()) return fail(KPD_EINVAL, std::string("no debug buffer ") + name);
  if (size_out) *size_out = it->second.second;
  if (!dst) return KPD_OK;
  if (bytes < it->second.second) return fail(KPD_EINVAL, "destination too small");
  HIP_TRY(hipMemcpyAsync(dst, it->second.first, it->second.second, hipMemcpyDeviceToDevice,
                         reinterpret_cast<hipStream_t>(stream)));
  return KPD_OK;
}

// ---------------------------------------------------------------- stand-alone operators
// The reference's submodule forwards, called outside the model's forward
// (each on a plan holding that submodule's weights).

static int op_work(kpd_plan* p, int R, int flags, hipStream_t st, Work** w) {
  Dims d;
  // one carve serves both stand-alone heads: the union of their flags, so
  // alternating HeatmapHead / KEYPOINT_HEAD calls never re-carve
  d.B = 0; d.NB = R; d.P = 1; d.flags = flags | (p->has_kh ? KPD_FLAG_DUAL_HEAD : 0);
  if (int rc = ensure_work(p, d, kpd_plan::kOpWs, st)) return rc;
  *w = &p->work[kpd_plan::kOpWs];
  // the split-K scratch of THIS workspace: the thread's last forward may have
  // run on another plan, whose workspace can be gone by now
  g_splitk = (*w)->splitk;
  return KPD_OK;
}

int kpd_heatmap_head(kpd_plan* p, const float* x, int R, int H, int W, int parts, float* heat, float* ch_w,
                     float* sp_w, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_hm) return fail(KPD_ESTATE, "plan has no heatmap_head weights");
  if (R < 0 || H != 56 || W != 56) return fail(KPD_EINVAL, "HeatmapHead input must be [R][64][56][56]");
  if (parts & ~KPD_HEAD_ALL) return fail(KPD_EINVAL, "unknown HeatmapHead parts");
  if (R == 0) return KPD_OK;
  if (!x || ((parts & KPD_HEAD_CONVS) && !heat)) return fail(KPD_EINVAL, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  Work* w = nullptr;
  if (int rc = op_work(p, R, 0, st, &w)) return rc;
  // any input sign: the split convs' bound is max |x| (hsc[r][2]), not the max
  const bool hsplit = p->precision == KPD_PRECISION_SPLIT;
  if (hsplit) HIP_TRY(hipMemsetAsync(w->hsc, 0, sizeof(float) * 4 * R, st));
  HIP_TRY(launch_nchw_rows_to_nhwc(x, R, 64, 56, 56, w->roi, w->roi_stats, st, hsplit ? w->hsc + 2 : nullptr, 4));
  HIP_TRY(hipMemsetAsync(w->slot, 0, sizeof(int32_t) * R, st));   // ROI r -> heat[r] (P = 1)
  if (int rc = run_heatmap_head(p, *w, R, 1, heat, st, parts, sp_w, nullptr, nullptr, nullptr, 1)) return rc;
  if (ch_w) HIP_TRY(hipMemcpyAsync(ch_w, w->cw, sizeof(float) * R * 64, hipMemcpyDeviceToDevice, st));
  return KPD_OK;
}

int kpd_keypoint_head(kpd_plan* p, const float* x, int R, int H, int W, float* kpts, float* vis, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_kh) return fail(KPD_ESTATE, "plan has no keypoint_head weights");
  if (R < 0 || H != 56 || W != 56) return fail(KPD_EINVAL, "KEYPOINT_HEAD input must be [R][128][56][56]");
  if (R == 0) return KPD_OK;
  if (!x || !kpts || !vis) return fail(KPD_EINVAL, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  Work* w = nullptr;
  if (int rc = op_work(p, R, KPD_FLAG_DUAL_HEAD, st, &w)) return rc;
  // any input sign: the split path's bound is max |x| per ROI (hsc[r][2])
  if (p->kh_split) HIP_TRY(hipMemsetAsync(w->hsc, 0, sizeof(float) * 4 * R, st));
  HIP_TRY(launch_nchw_rows_to_nhwc(x, R, 128, 56, 56, w->kx, nullptr, st, p->kh_split ? w->hsc + 2 : nullptr, 4));
  HIP_TRY(hipMemsetAsync(w->slot, 0, sizeof(int32_t) * R, st));
  return run_keypoint_head(p, *w, R, 1, kpts, vis, st, w->hsc + 2, 1, 4);
}

int kpd_backbone(kpd_plan* p, const float* image, int B, int C, int H, int W, float* out0, float* out1, float* out2,
                 float* out3, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_body || !p->has_fpn) return fail(KPD_ESTATE, "plan lacks backbone.body / backbone.fpn weights");
  for (int i = 0; i < 3; ++i)
    if (!p->fpn_lv[i].w) return fail(KPD_ESTATE, "plan lacks backbone.fpn.fpn_convs.1-3 weights");
  if (!image || B <= 0 || H < 32 || W < 32) return fail(KPD_EINVAL, "bad image shape");
  if (C != p->in_ch) return fail(KPD_EINVAL, "image channels do not match backbone in_channels");
  float* outs[4] = {out0, out1, out2, out3};
  for (float* o : outs)
    if (!o) return fail(KPD_EINVAL, "null output pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  // level sizes: stem (features.0), features.3, .8, .12 -- as forward_one's Dims
  int h[12], wd[12];
  h[0] = (H - 1) / 2 + 1; wd[0] = (W - 1) / 2 + 1;
  for (int i = 0; i < 11; ++i) {
    const int k = kBneck[i].k, s = kBneck[i].s, pd = (k - 1) / 2;
    h[i + 1] = (h[i] + 2 * pd - k) / s + 1;
    wd[i + 1] = (wd[i] + 2 * pd - k) / s + 1;
  }
  const int lh[4] = {h[0], h[3], h[8], h[11]}, lw[4] = {wd[0], wd[3], wd[8], wd[11]};
  const int cap = max_pass_images(H, W), npass = (B + cap - 1) / cap;
  for (int q = 0; q < npass; ++q) {
    const int b0 = (int)((long)B * q / npass), b1 = (int)((long)B * (q + 1) / npass), nb = b1 - b0;
    p->keep_laterals = true;
    const int rc1 = forward_one(p, 0, false, image + (size_t)b0 * C * H * W, nb, C, H, W, nullptr, 0, 0, 0, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st);
    p->keep_laterals = false;
    if (rc1) return rc1;
    Work& w = p->work[0];
    HIP_TRY(launch_nhwc_to_nchw(w.feat, nb, lh[0] * lw[0], 128, outs[0] + (size_t)b0 * 128 * lh[0] * lw[0], st));
    for (int i = 1; i < 4; ++i) {   // fpn_convs[i] on lateral i (backbone.py:39), into the free level-0 buffer
      if (int rc = conv(p->fpn_lv[i - 1], w.lat[i], nb, lh[i], lw[i], 128, w.feat, ACT_RELU, nullptr, 0, 0, nullptr,
                        nullptr, 0, 0, st))
        return rc;
      HIP_TRY(launch_nhwc_to_nchw(w.feat, nb, lh[i] * lw[i], 128, outs[i] + (size_t)b0 * 128 * lh[i] * lw[i], st));
    }
  }
  return KPD_OK;
}

int kpd_backbone_body(kpd_plan* p, const float* image, int B, int C, int H, int W, float* feat0, float* feat1,
                      float* feat2, float* feat3, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_body) return fail(KPD_ESTATE, "plan lacks backbone.body weights");
  if (!image || B <= 0 || H < 32 || W < 32) return fail(KPD_EINVAL, "bad image shape");
  if (C != p->in_ch) return fail(KPD_EINVAL, "image channels do not match backbone in_channels");
  float* outs[4] = {feat0, feat1, feat2, feat3};
  for (float* o : outs)
    if (!o) return fail(KPD_EINVAL, "null output pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  int h[12], wd[12];
  h[0] = (H - 1) / 2 + 1; wd[0] = (W - 1) / 2 + 1;
  for (int i = 0; i < 11; ++i) {
    const int k = kBneck[i].k, s = kBneck[i].s, pd = (k - 1) / 2;
    h[i + 1] = (h[i] + 2 * pd - k) / s + 1;
    wd[i + 1] = (wd[i] + 2 * pd - k) / s + 1;
  }
  const int lv[4] = {0, 3, 8, 11};
  const int cap = max_pass_images(H, W), npass = (B + cap - 1) / cap;
  for (int q = 0; q < npass; ++q) {
    const int b0 = (int)((long)B * q / npass), b1 = (int)((long)B * (q + 1) / npass), nb = b1 - b0;
    p->body_only = true;
    const int rc1 = forward_one(p, 0, false, image + (size_t)b0 * C * H * W, nb, C, H, W, nullptr, 0, 0, 0, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st);
    p->body_only = false;
    if (rc1) return rc1;
    for (int i = 0; i < 4; ++i) {
      const int c = kFpnIn[i], hw = h[lv[i]] * wd[lv[i]];
      HIP_TRY(launch_nhwc_pad_to_nchw(p->body_taps[i], nb, hw, c, pad16(c), outs[i] + (size_t)b0 * c * hw, st));
    }
  }
  return KPD_OK;
}

int kpd_backbone_fpn(kpd_plan* p, const float* feat0, const float* feat1, const float* feat2, const float* feat3, int B,
                     const int* sizes, float* out0, float* out1, float* out2, float* out3, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_fpn) return fail(KPD_ESTATE, "plan lacks backbone.fpn weights");
  for (int i = 0; i < 3; ++i)
    if (!p->fpn_lv[i].w) return fail(KPD_ESTATE, "plan lacks backbone.fpn.fpn_convs.1-3 weights");
  if (B < 0 || !sizes) return fail(KPD_EINVAL, "bad FPN arguments");
  if (B == 0) return KPD_OK;
  const float* feats[4] = {feat0, feat1, feat2, feat3};
  float* outs[4] = {out0, out1, out2, out3};
  int hh[4], ww[4];
  size_t in_f = 0, lat_f = 0, out_f = 0;
  for (int i = 0; i < 4; ++i) {
    hh[i] = sizes[2 * i]; ww[i] = sizes[2 * i + 1];
    if (!feats[i] || !outs[i]) return fail(KPD_EINVAL, "null FPN tensor");
    if (hh[i] <= 0 || ww[i] <= 0) return fail(KPD_EINVAL, "bad FPN level size");
    if (p->lat[i].cin != kFpnIn[i]) return fail(KPD_EINVAL, "lateral conv channels do not match the taps");
    const size_t hw = (size_t)B * hh[i] * ww[i];
    if (hw * 576 >= (1UL << 31)) return fail(KPD_EINVAL, "FPN tensors must stay below 2^31 elements");
    in_f += hw * p->lat[i].cin_p;
    lat_f += hw * 128;
    out_f = std::max(out_f, hw * 128);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  float* scratch = nullptr;
  const size_t total = in_f + lat_f + out_f + kSplitKFloats;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&scratch), total * sizeof(float), st));
  float *tin[4], *lat[4];
  float* cur = scratch;
  for (int i = 0; i < 4; ++i) { tin[i] = cur; cur += (size_t)B * hh[i] * ww[i] * p->lat[i].cin_p; }
  for (int i = 0; i < 4; ++i) { lat[i] = cur; cur += (size_t)B * hh[i] * ww[i] * 128; }
  float* lvl = cur;
  cur += out_f;
  g_splitk = cur;
  // LightweightFPN.forward (backbone.py:29-39): laterals top-down, each
  // nearest-upsampled to the next finer size and added, then fpn_convs[i]
  int rc = KPD_OK;
  hipError_t e = hipSuccess;
  for (int i = 0; i < 4 && e == hipSuccess; ++i)
    e = launch_nchw_to_nhwc_pad(feats[i], B, hh[i] * ww[i], kFpnIn[i], p->lat[i].cin_p, tin[i], st);
  for (int i = 3; i >= 0 && e == hipSuccess && rc == KPD_OK; --i) {
    const float* res = i < 3 ? lat[i + 1] : nullptr;
    const int rh = i < 3 ? hh[i + 1] : 0, rw = i < 3 ? ww[i + 1] : 0;
    if (i == 0 && p->lat[i].cin_p <= 32)   // the 16-channel stem tap (as forward_one)
      e = launch_lateral_stream(tin[i], p->lat[i].cin_p, (const float*)p->lat[i].w, p->lat[i].b, res, B, hh[i], ww[i],
                                rh, rw, lat[i], st);
    else
      rc = conv(p->lat[i], tin[i], B, hh[i], ww[i], p->lat[i].cin_p, lat[i], ACT_NONE, res, rh, rw, nullptr, nullptr, 0,
                0, st);
  }
  for (int i = 0; i < 4 && e == hipSuccess && rc == KPD_OK; ++i) {
    const DevConv& L = i == 0 ? p->fpn0 : p->fpn_lv[i - 1];
    rc = conv(L, lat[i], B, hh[i], ww[i], 128, lvl, ACT_RELU, nullptr, 0, 0, nullptr, nullptr, 0, 0, st);
    if (rc == KPD_OK) e = launch_nhwc_to_nchw(lvl, B, hh[i] * ww[i], 128, outs[i], st);
  }
  (void)hipFreeAsync(scratch, st);
  HIP_TRY(e);
  return rc;
}

int kpd_channel_attention(kpd_plan* p, const float* x, int B, int C, int H, int W, float* scores, int32_t* topk,
                          int k, float* selected, void* stream) {
  if (!p || !p->finalized) return fail(KPD_ESTATE, "plan not finalized");
  if (!p->has_ca) return fail(KPD_ESTATE, "plan has no channel_attention weights");
  if (C != 128 || k != 64 || B < 0 || H <= 0 || W <= 0)
    return fail(KPD_EINVAL, "ChannelAttention path is built for 128 channels and top-64");
  if (B == 0) return KPD_OK;
  if (!x) return fail(KPD_EINVAL, "null input");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(p->device));
  char* scratch = nullptr;
  const size_t sb = (size_t)B * 2 * 128 * 4, tb = (size_t)B * 64 * 4, cb = (size_t)B * 128 * 4;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&scratch), sb + tb + cb, st));
  float* stats = reinterpret_cast<float*>(scratch);
  int32_t* tk = reinterpret_cast<int32_t*>(scratch + sb);
  float* sc = reinterpret_cast<float*>(scratch + sb + tb);
  hipError_t e = launch_nchw_channel_stats(x, B, 128, H * W, stats, st);
  if (e == hipSuccess)
    e = launch_topk(stats, B, 1, H * W, p->ca_w0, p->ca_b0, p->ca_w2, p->ca_b2, tk, sc, st, nullptr, 0, nullptr);
  if (e == hipSuccess && scores) e = hipMemcpyAsync(scores, sc, cb, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && topk) e = hipMemcpyAsync(topk, tk, tb, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && selected) e = launch_gather_planes(x, B, 128, H * W, tk, 64, selected, st);
  (void)hipFreeAsync(scratch, st);
  HIP_TRY(e);
  return KPD_OK;
}

int kpd_decode_heatmaps(const float* heat, int planes, int H, int W, int mode, float param, float* kpts,
                        float* scores, float* vis, void* stream) {
  if (planes < 0 || H < 2 || W < 2 || (planes > 0 && (!heat || !kpts)) || (mode == KPD_DECODE_MODEL && planes > 0 && !vis))
    return fail(KPD_EINVAL, "bad decode arguments");
  HIP_TRY(launch_decode_planes(heat, planes, H, W, mode, param, kpts, scores, vis,
                               reinterpret_cast<hipStream_t>(stream)));
  return KPD_OK;
}

int kpd_roi_align(const float* feat, int B, int C, int H, int W, const float* rois, int R, int out_h, int out_w,
                  float spatial_scale, int sampling_ratio, int aligned, float* out, void* stream) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || R < 0 || out_h <= 0 || out_w <= 0 || (R > 0 && (!feat || !rois || !out)))
    return fail(KPD_EINVAL, "bad roi_align arguments");
  HIP_TRY(launch_roi_align_nchw(feat, C, H, W, rois, R, out_h, out_w, spatial_scale, sampling_ratio, aligned, out,
                                reinterpret_cast<hipStream_t>(stream)));
  return KPD_OK;
}

int kpd_conv1x1(const float* x, int B, int Cin, int HW, const float* w, const float* b, int Cout, float* out,
                void* stream) {
  if (B < 0 || Cin <= 0 || HW < 0 || Cout <= 0 || (B > 0 && HW > 0 && (!x || !w || !out)))
    return fail(KPD_EINVAL, "bad conv1x1 arguments");
  HIP_TRY(launch_conv1x1_nchw(x, B, Cin, HW, w, b, Cout, out, reinterpret_cast<hipStream_t>(stream)));
  return KPD_OK;
}

int kpd_conv3x3_forward(const float* x, const float* w, const float* b, int N, int C, int H, int W, int O, float* y,
                        void* stream) {
  if (N < 0 || C <= 0 || H <= 0 || W <= 0 || O <= 0 || (N > 0 && (!x || !w || !y)))
    return fail(KPD_EINVAL, "bad conv3x3 arguments");
  if ((long)N * C * H * W >= (1L << 31) || (long)N * O * H * W >= (1L << 31) || (long)O * C * 9 >= (1L << 31))
    return fail(KPD_EINVAL, "conv3x3: tensors must stay below 2^31 elements");
  HIP_TRY(launch_conv3_forward(x, w, b, N, C, H, W, O, y, reinterpret_cast<hipStream_t>(stream)));
  return KPD_OK;
}

int kpd_conv3x3_backward(const float* x, const float* w, const float* gy, int N, int C, int H, int W, int O,
                         float* gx, float* gw, float* gb, void* stream) {
  if (N < 0 || C <= 0 || H <= 0 || W <= 0 || O <= 0 || (N > 0 && !gy) || (gx && !w) || (gw && !x))
    return fail(KPD_EINVAL, "bad conv3x3 backward arguments");
  if ((long)N * C * H * W >= (1L << 31) || (long)N * O * H * W >= (1L << 31) || (long)O * C * 9 >= (1L << 31))
    return fail(KPD_EINVAL, "conv3x3: tensors must stay below 2^31 elements");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N == 0) {   // empty batch: zero parameter gradients
    if (gw) HIP_TRY(hipMemsetAsync(gw, 0, sizeof(float) * O * C * 9, st));
    if (gb) HIP_TRY(hipMemsetAsync(gb, 0, sizeof(float) * O, st));
    return KPD_OK;
  }
  float* part = nullptr;
  if (gw && conv3_wgrad_slices(N, H, W)) HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&part),
                                 sizeof(float) * conv3_wgrad_slices(N, H, W) * O * C * 9, st));
  const hipError_t e = launch_conv3_backward(x, w, gy, N, C, H, W, O, gx, gw, gb, part, st);
  if (part) HIP_TRY(hipFreeAsync(part, st));
  HIP_TRY(e);
  return KPD_OK;
}

int kpd_nms(const float* boxes, const float* scores, int n, float thr, int max_out, int32_t* keep, int32_t* n_keep,
            void* stream) {
  if (n < 0 || (n > 0 && (!boxes || !scores || !keep)) || !n_keep) return fail(KPD_EINVAL, "bad nms args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  void* scratch = nullptr;
  if (n > 0) HIP_TRY(hipMallocAsync(&scratch, (size_t)n, st));
  const hipError_t e =
      launch_nms_sets(boxes, scores, 1, n, thr, max_out, std::max(n, 1), keep, n_keep, scratch, st, 0, nullptr, nullptr);
  if (scratch) HIP_TRY(hipFreeAsync(scratch, st));
  HIP_TRY(e);
  return KPD_OK;
}

}  // extern "C"
