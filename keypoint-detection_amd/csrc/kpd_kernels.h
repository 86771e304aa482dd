// Internal launcher declarations (host side of each .hip translation unit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct ConvArgs {
  const void* in;        // NHWC [N][H][W][in_cstride] (TA)
  const void* wt;        // [cout_p][KS*KS][cin_p] (TA), BN folded
  const float* bias;     // [cout_p]
  void* out;             // NHWC [N][H][W][out_cstride] (TO)
  const float* res;      // optional residual NHWC [N][rh][rw][cout_p] (f32), added after act
  const float* a_scale;  // optional [N][cin_p] per-image input-channel scale (SE), f32 path only
  float* stats;          // optional [N][tiles_per_img][2][cout_p] channel sum / max partials
  int N, H, W;
  int cin_p, cout_p;
  int in_cstride, out_cstride;
  int rh, rw;
  int act;
  int M;                 // N*H*W
  int tiles_per_img;
  float* amax;           // optional: per-image max|out|, slot n = amax[n * kAmaxStride] (amax_publish_img; caller zeroes)
  const float* post_scale;  // optional second affine after act (see conv_epilogue.h)
  const float* post_shift;
  int act2, act3;
  int in_bytes, wt_bytes;   // buffer-descriptor extents; filled by launch_conv (each < 2^31)
  // optional split-K scratch for small-M 1x1 fp32 GEMMs (launch_conv decides):
  // partial sums [k_split][M][cout_p] + a reduce/epilogue kernel, fixed order
  float* splitk_ws;
  long splitk_cap;          // floats available at splitk_ws
  int k_split;              // set by launch_conv
};

// 16-bit-operand 3x3 conv with LDS-DMA staging (conv_glds.hip): bf16 operands,
// or "split" f16 hi|lo operands (fp32-accurate, FPN level 0).
struct Conv16Args {
  const void* in;        // NHWC [N][H][W][in_cstride] 16-bit; split: per 32 channels [hi32|lo32]
  const void* wt;        // [cout_p][9][cin_e] 16-bit (BN folded; split: same interleave, scaled 2^w_exp)
  const float* bias;     // [cout_p]
  void* out;             // NHWC [N][H][W][out_cstride] (f32 or bf16)
  float* stats;          // optional [N][tiles_per_img][2][cout_p] (H*W % 256 == 0)
  int N, H, W;
  int cin_e;             // 16-bit elements per tap row (cin, or 2*cin in split mode), % 64 == 0
  int cout_p, in_cstride, out_cstride, act, M, tiles_per_img;
  // split mode (kpd_bench_conv16 diagnostics only): products unscaled by split_scale
  float split_scale;
  int in_bytes, wt_bytes;   // filled by the launcher
  // optional fused HeatmapHead final_layer (1x1 64->17 + sigmoid) for the
  // BN = 64 fp32-out conv: heatmap [B][P][17][H][W] at the ROI's slot
  const float* fin_w;    // [17][64]
  const float* fin_b;    // [17]
  const int32_t* slot;   // [R] (launch_slotmap)
  int P;
  float* heat;
  int r0;                // first ROI of this launch (set by the launcher per chunk)
};
hipError_t launch_conv16(const Conv16Args& a, int split, int out_bf16, hipStream_t st);

// HeatmapHead 3x3 conv on zero-bordered ROI maps [R][57 x 57][C] bf16
// (conv_glds.hip, hmconv_kernel).  fin_w == null: bf16 output in the same
// padded layout (interior only); else cout == 64 and the final 1x1 + sigmoid
// is fused, writing heat [B][P][17][56][56] at the ROI's slot.
struct HmConvArgs {
  const void* in;        // [R][57 x 57][cin] bf16, or (split) f16 [hi32 | lo32] per 32 channels
  const void* wt;        // [cout][9][cin] bf16 (BN folded), or (split) f16 [hi32 | lo32] scaled 2^w_exp
  const float* bias;     // [cout]
  void* out;             // [R][57 x 57][cout] bf16, or (split) f16 [hi32 | lo32]
  int R, cin, cout;
  // split (fp32-accurate) mode: per-ROI bounds hsc[r][4]; the operand scale of
  // ROI r is 2^a with a = split_exp_of(c + s * hsc[r][idx]) (kpd_common.h)
  int split;
  float* hsc;
  float in_c, in_s;      // input bound
  int in_idx;
  float out_c, out_s;    // output bound (out_idx < 0: fp32 epilogue, conv 3)
  int out_idx;
  int amax_idx;          // >= 0: atomicMax of max|out| per ROI into hsc[r][amax_idx]
  int w_exp;
  const float *fin_w, *fin_b;   // [17][64], [17]
  const int32_t* slot;
  int P;
  float* heat;
  int r0;                // first ROI of the launch chunk (launcher)
  int m_off;             // launcher: first GEMM row of tile 0 (tail launch of conv 3)
  int mix_F, mix_H, mix_lead;   // launcher: hmconv_mixed_kernel's full / tail tile counts, lead pairs per XCD
  int in_bytes, wt_bytes;   // launcher
  int stagger;              // launcher: split K loop, waves 4-7 issue their DMA one pass later
  unsigned long long* stamps;   // diagnostic phase stamps [grid][8] (KPD_STAMPS), normally null
  // KEYPOINT_HEAD mode (kh_ps != null; split only): wt is [cout][ntap][cin] with
  // ntap = 10 when the ResidualBlock's 1x1 downsample rides along as a tenth
  // tap; per column co: v = relu6(acc + bias), v = relu6(v * kh_ps + kh_pt),
  // (ntap 10) v = relu6(v + downsample + kh_bd); columns [0, ns) -> out (split,
  // [R][57 x 57][ns]), [ns, ns + nf) -> outf fp32 [R][56][56][nf]
  const float *kh_ps, *kh_pt, *kh_bd;
  float* outf;
  int ns, nf, ntap;
};
hipError_t launch_hmconv(const HmConvArgs& a, hipStream_t st);
// The hmconv layout of the per-ROI activation maps (HeatmapHead and
// KEYPOINT_HEAD convs): per ROI 57 rows of 57 positions, interior pixel
// (y, x) at position r * kHmRoiPos + (y + 1) * kHmPitch + x.  Row 0 and
// column 56 are zero: column 56 is the right border of its row and the left
// border of the next row, row 0 the top border of its ROI and the bottom
// border of the previous one; ROI 0's top-left neighbour (position -1) and
// the last ROI's bottom border lie outside the tensor and read as zero (the
// conv kernels' window loads are range-checked).  3249 positions per ROI
// instead of a 58 x 58 frame's 3364: 3.4 % fewer GEMM rows in every conv.
constexpr int kHmPitch = 57, kHmRoiPos = kHmPitch * kHmPitch;
__host__ __device__ inline size_t hm_pos(size_t r, int y, int x) {
  return r * kHmRoiPos + (size_t)(y + 1) * kHmPitch + x;
}

// FPN level 0 by linearity (split mode): conv3x3(L0(tap0) + up4(lat1)) =
// conv3x3'(tap0) [composite weights W3.L0, 16 input channels]
// + per-position-class combinations of lat1 [taps summed by the lat1 pixel they
// read after the exact 4x nearest upsample].  Output pixels are processed by
// class (y % 4, x % 4), so every MFMA row of a tile uses the same weights.
constexpr int kFpn0xMaxGroups = 4;
constexpr int kFpn0xMaxImg = 512;   // images per fpn0x launch (per-image unscale table in LDS)
struct Fpn0xArgs {
  const void* f_split;     // tap0 as f16 [N][Hf][Wf][hi16 | lo16] (scale 2^a_f)
  const void* l_split;     // lateral 1 as f16 [N][rh][rw][4 x (hi32 | lo32)] (scale 2^a_l)
  const void* w0;          // [128][5 K-tiles][hi16(t) hi16(t+1) lo16(t) lo16(t+1)] (scale 2^w_exp0)
  const void* weff;        // per class: [128][groups][4 chunks][hi32 | lo32] (scale 2^w_expE)
  int cls_woff[16];        // f16-element offset of each class block in weff
  int cls_ng[16];          // lat1 pixel groups of the class (1, 2 or 4)
  int cls_g[16][kFpn0xMaxGroups];   // group g = (oy + 1) * 3 + (ox + 1)
  const float* bias;       // [128] (fpn conv + BN, folded)
  float* out;              // NHWC [N][Hf][Wf][128] fp32 (ReLU)
  float* stats;            // [N][16 * tpc][2][128] channel sum / max per tile
  const float* sc;         // per-image max|tap0| [sc_n] then max|lat1| [sc_n], stride kAmaxStride
  int sc_n;                // images between the two slot arrays (>= N)
  int N, Hf, Wf, rh, rw, tpc, w_exp0, w_expE;
  int f_bytes, l_bytes, w0_bytes, weff_bytes;
  int stagger;             // launcher: waves 4-7 issue their K-loop DMA one pass later
  int out_nt;              // launcher: non-temporal output stores
  int order;               // launcher: 1 = class-half tile order (grid % 8 == 0), 0 = class-fastest rounds
  unsigned long long* stamps;   // diagnostic phase stamps [grid][8] (KPD_STAMPS), normally null
  // footprint stores (boxes != null): image n's output pixels are stored only
  // inside the rectangle its ROI aligns read -- the union over its fp_P
  // cxcywh boxes [fp_NB][fp_P][4] of the sampled rows / columns, one pixel of
  // margin; images >= fp_NB store nothing
  const float* fp_boxes;
  int fp_NB, fp_P;
};
hipError_t launch_fpn0x(const Fpn0xArgs& a, hipStream_t st);
// fp32 NHWC -> f16 hi|lo split rows (groups of 32 channels, or 16 for cin 16),
// each image scaled by its own power of two (per-image slots sc, see fpn0x_exps)
hipError_t launch_split_rows(const float* in, int N, long hw, int cin, const float* sc, int which, int w_exp0,
                             int w_expE, void* out, hipStream_t st);
int conv16_tile_m();

enum ConvDType : int { CONV_F32 = 0, CONV_BF16_OUT_BF16 = 1, CONV_BF16_OUT_F32 = 2 };

int conv_tile_m();
hipError_t launch_conv(const ConvArgs& a, ConvDType dt, int ks, hipStream_t st);

// ---- MobileNetV3 body (body_kernels.hip) ----
hipError_t launch_stem(const float* img, int N, int Cin, int H, int W, const float* w, const float* b,
                       float* out, int Ho, int Wo, float* amax, hipStream_t st);
hipError_t launch_dwconv(const float* in, const float* w, const float* b, float* out, int N, int H, int W,
                         int Cp, int Ho, int Wo, int k, int s, int act, hipStream_t st);
hipError_t launch_se(const float* x, int N, int HW, int C, int Cp, const float* w1, const float* b1,
                     const float* w2, const float* b2, int sq, float* scale, hipStream_t st,
                     const float* pooled = nullptr);
// fused inverted residual WITHOUT squeeze-excitation on row tiles
// (body_kernels.hip, fir_kernel): expand 1x1 + act -> depthwise KxK stride S
// + act -> project 1x1 (+ residual), the expanded tensor never leaves LDS
struct FirArgs {
  const float* x;        // NHWC [N][Hi][Wi][cin_p]
  int Hi, Wi, cin_p;
  const float *we, *be;  // expand [Ep][cin_p], [Ep] (BN folded)
  const float *wd, *bd;  // depthwise [K*K][Ep], [Ep]
  const float *wp, *bp;  // project [cout_p][Ep], [cout_p]
  int act_e, act_d, Ep, cout_p;
  float* out;            // NHWC [N][Ho][Wo][cout_p]
  int Ho, Wo, res;       // res: add x (stride 1, cin_p == cout_p)
  int TH;                // output rows per workgroup (host-chosen)
  unsigned long long* stamps;   // diagnostic phase stamps [grid][8] (KPD_STAMPS), normally null
};
size_t fir_lds_bytes(const FirArgs& a, int K, int S);
int fir_pick_rows(FirArgs& a, int K, int S);   // sets a.TH; 0 when the layer does not fit
hipError_t launch_fir(const FirArgs& a, int N, int K, int S, hipStream_t st);
// features.2 + features.3 (the two SE-less inverted residuals, 3x3 stride 2
// then 3x3 stride 1 with the residual) in one launch on row tiles (fir23.hip)
struct Fir23Args {
  const float* x;                      // features.1 output NHWC [N][H1][W1][16]
  int H1, W1;
  const float *we2, *be2, *wd2, *bd2;  // features.2 expand [E2][16], [E2]; depthwise [9][E2], [E2]
  const float *wp2, *bp2;              // features.2 project [32][E2], [32]
  const float *we3, *be3, *wd3, *bd3;  // features.3 expand [E3][32], [E3]; depthwise [9][E3], [E3]
  const float *wp3, *bp3;              // features.3 project [32][E3], [32]
  int E2, E3;                          // padded expanded widths (multiples of 16)
  int act2e, act2d, act3e, act3d;
  float* out;                          // features.3 output NHWC [N][H2][W2][32]
  int H2, W2;
  int T;                               // features.3 rows per workgroup (fir23_pick_rows)
  unsigned long long* stamps;          // diagnostic phase stamps [grid][8] (KPD_STAMPS), normally null
};
int fir23_pick_rows(Fir23Args& a);   // sets a.T; 0 when the shapes do not fit
hipError_t launch_fir23(const Fir23Args& a, int N, hipStream_t st);
// fused expand 1x1 + depthwise + channel means (body_kernels.hip, exdw_kernel)
struct ExDwArgs {
  const float* x;        // NHWC [N][Hi][Wi][cin_p]
  int Hi, Wi, cin_p;
  const float* we;       // expand [Ep][cin_p] (BN folded), cin_p a multiple of 16, <= 96
  const float* be;
  int act_e;
  const float* wd;       // depthwise [K*K][Ep] (BN folded), bias bd [Ep]
  const float* bd;
  int act_d, Ep;
  float* out;            // [N][Ho][Wo][Ep]
  int Ho, Wo;
  float* pooled;         // optional [N][Ep] channel means of out (SE squeeze)
  int CS;                // expanded channels per workgroup (16 or 32, divides Ep)
  const float* w1;       // SE fc1 [sq][C] (row-major) for the partials
  float* part;           // optional [N][Ep/CS][sq] fc1 partial products (needs pooled)
  int sq, C;
  unsigned long long* stamps;   // diagnostic phase stamps, [grid][8] (KPD_STAMPS), normally null
  int nband;             // > 1 (no SE only): output rows split over nband workgroups per (image, slice)
};
size_t exdw_lds_bytes(const ExDwArgs& a, int K);
hipError_t launch_exdw(const ExDwArgs& a, int N, int K, int S, hipStream_t st);
// SE excitation (from exdw_kernel's fc1 partials) + project 1x1 + residual
// (body_kernels.hip, seproj_kernel)
struct SeProjArgs {
  const float* d;        // depthwise output [N][Po][Ep]
  int Po, Ep;
  const float* part;     // [N][nsl][sq] fc1 partials
  int nsl, sq, C;
  const float *b1, *w2t, *b2;   // fc1 bias [sq]; fc2 transposed [sq][C]; fc2 bias [C]
  const float *wp, *bp;  // project [cout_p][Ep], [cout_p] (BN folded)
  int cout_p, NT;        // output channels per workgroup (multiple of 16)
  const float* res;      // optional residual [N][Po][cout_p]
  float* out;            // [N][Po][cout_p]
  unsigned long long* stamps;   // diagnostic phase stamps, [grid][8] (KPD_STAMPS), normally null
  const float* sesc;     // optional precomputed excitation [N][Ep] (se_excite_kernel); null: computed here
};
size_t seproj_lds_bytes(const SeProjArgs& a);
hipError_t launch_seproj(const SeProjArgs& a, int N, hipStream_t st);
// features.1 (16 channels, no expand): depthwise + per-tile channel sums, then
// excitation + project (body_kernels.hip, dwsum_kernel / se16_proj_kernel)
hipError_t launch_dwsum(const float* in, int N, int Hi, int Wi, const float* w, const float* b, int act, float* out,
                         int Ho, int Wo, int k, int s, float* part, int* ntiles, hipStream_t st);
hipError_t launch_se16_proj(const float* d, int N, int npx, int ntiles, const float* part, const float* w1,
                            const float* b1, const float* w2t, const float* b2, int sq, const float* wp,
                            const float* bp, float* out, hipStream_t st);
// small-K fp32 1x1 conv with direct-to-fragment loads (body_kernels.hip,
// pw_small_kernel): cin_p <= 96, cout_p % 64 == 0, act + optional residual/amax
bool pw_small_ok(const ConvArgs& a);
hipError_t launch_pw_small(const ConvArgs& a, hipStream_t st);
// the excitation alone, for the wide blocks: sesc [N][Ep]
hipError_t launch_se_excite(const SeProjArgs& a, int N, float* sesc, hipStream_t st);
hipError_t launch_channel_stats(const float* x, int N, int HW, int Cp, int tiles, float* stats,
                                hipStream_t st);
// LightweightFPN laterals 3 -> 2 -> 1 with the top-down adds in one launch
// (lateral_chain.hip): taps t_i NHWC [N][h_i * w_i][c_i] (c_i = padded input
// channels: 32, 48, 576; c_ir real ones; lateral 3 at most 128 pixels),
// weights L_i [128][c_i] (no bias).  Writes lat1 fp32 [N][h1*w1][128], or with
// lat1_split the f16 hi|lo rows of fpn0x_kernel, scaled per image by
// fpn0x_exps(amax[n], bound) and the bound S1 m1 + S2 m2 + S3 m3 published at
// amax[(N + n) * kAmaxStride] (S_i = max_co sum_k |L_i[co][k]|).
struct LatChainArgs {
  const float *t1, *t2, *t3, *L1, *L2, *L3;
  int c1, c2, c3, c1r, c2r, c3r, h1, w1, h2, w2, h3, w3;
  int n;   // images (set by launch_lateral_chain)
  float* lat1;
  _Float16* lat1_split;
  float* amax;          // split: per-image slots, [0, N) max|tap0| (read), [N, 2N) the bound (published)
  float S1, S2, S3;
  int w_exp0, w_expE;
  const float* t0;      // split: optional stem tap [N][P0][16] -> t0_split hi|lo rows (2^a_f), else null
  _Float16* t0_split;
  int P0;
  unsigned long long* stamps;   // diagnostic phase stamps [grid][8] (KPD_STAMPS), normally null
};
size_t lateral_chain_lds_bytes(const LatChainArgs& a);
bool lateral_chain_ok(const LatChainArgs& a);   // shapes launch_lateral_chain takes
hipError_t launch_lateral_chain(const LatChainArgs& a, int N, hipStream_t st);
hipError_t launch_lateral_stream(const float* in, int cin_p, const float* w, const float* bias, const float* res,
                                 int N, int H, int W, int rh, int rw, void* out, hipStream_t st);

// ---- channel attention / ROI / heatmap head / decode (head_kernels.hip) ----
// slot != nullptr: also writes the slot map of boxes [N][P][4] (launch_slotmap's work)
hipError_t launch_topk(const float* stats, int N, int tiles, int HW, const float* w0, const float* b0,
                       const float* w2, const float* b2, int32_t* topk, float* scores, hipStream_t st,
                       const float* boxes = nullptr, int P = 0, int32_t* slot = nullptr, float* imax = nullptr,
                       float* sc_zero = nullptr, int sc_n = 0);
hipError_t launch_slotmap(const float* boxes, int B, int P, int32_t* slot,
                          hipStream_t st);
// Dual head, split precision: one 128-channel ROI align pass writing the top-k
// HeatmapHead input (roi, roi_stats) and KEYPOINT_HEAD's attention-applied
// split operand (out: [R][57 x 57][128] hi|lo f16 interior; hsc[r][2] = bound)
hipError_t launch_roi_kh(const float* feat, int Hf, int Wf, const int32_t* topk, const float* boxes, int R, int P,
                        float* roi, float* roi_stats, const void* w1s, int w1_exp, const float* b1, const float* w2,
                        const float* b2, const float* bound, int bdiv, int bstride, float* hsc, void* out,
                        hipStream_t st, unsigned long long* stamps = nullptr);
hipError_t launch_roi_align(const float* feat, int Hf, int Wf, int Cf, const int32_t* topk,
                            const float* boxes, int R, int P, float* roi, float* roi_stats,
                            hipStream_t st, unsigned long long* stamps = nullptr);   // stamps: KPD_STAMPS [grid][8]
// hsc != null (split heatmap convs): writes hsc[r][0] = max of ROI r's
// features (the bound of |xs|: the model's ROI features follow a ReLU) and
// zeroes hsc[r][1]; abs_in = 1: the features may be negative, hsc[r][2]
// holds their max |x| (launch_nchw_rows_to_nhwc) and joins the bound
hipError_t launch_hm_chattn(const float* roi_stats, int R, const float* w0, const float* b0,
                            const float* w2, const float* b2, float* cw, float* hsc, hipStream_t st,
                            int abs_in = 0);
hipError_t launch_hm_spool(const float* roi, const float* cw, int R, float* smap, hipStream_t st);
// use_sp = 0: no spatial attention (weights 1); sw_out != null: the spatial
// weights [R][56][56] (HeatmapHead.forward's attention_weights[1])
// hm_spool + hm_sapply in one launch (bands of 8 rows; no pooled map in HBM)
hipError_t launch_hm_attn(const float* roi, const float* cw, const float* saw, const float* sab, int R, void* xs,
                          int out_bf16, hipStream_t st, const float* hsc, int use_sp, float* sw_out);
hipError_t launch_hm_sapply(const float* roi, const float* cw, const float* smap, const float* saw,
                            const float* sab, int R, void* xs, int out_bf16, hipStream_t st,
                            const float* hsc = nullptr, int use_sp = 1, float* sw_out = nullptr);
hipError_t launch_hm_final(const float* h3, int R, const float* w, const float* b, const int32_t* slot,
                           int P, float* heat_out, hipStream_t st);
hipError_t launch_decode(const float* heat_out, const float* boxes, const int32_t* slot, int R, int P,
                         float* kpts_out, float* vis_out, hipStream_t st);

// ---- person head / NMS (nms.hip) ----
hipError_t launch_nms(const float* boxes, const float* scores, int n, float thr, int max_out,
                      int32_t* keep, int32_t* n_keep, void* scratch, size_t scratch_bytes, hipStream_t st);
// one workgroup per set; filter=1 starts candidates with score -inf dead; optional
// zero-padded gather of the kept boxes/scores into out_boxes [sets][max_keep][4]
hipError_t launch_nms_sets(const float* boxes, const float* scores, int sets, int n, float thr, int max_out,
                           int max_keep, int32_t* keep, int32_t* n_keep, void* scratch, hipStream_t st, int filter,
                           float* out_boxes, float* out_scores);
size_t nms_scratch_bytes(int n);

// ---- person-detector glue + KEYPOINT_HEAD (aux_heads.hip) ----
hipError_t launch_adaptive_pool56(const float* in, int B, int Hf, int Wf, int C, float* out, hipStream_t st);
// adaptive pool + 1x1 heads (w [48][128] fp32, bias [48]) + decode in one launch (the default detector path;
// level-0 widths with person_detect_fits(Wf): the column sums fit the LDS)
bool person_detect_fits(int Wf);
hipError_t launch_person_detect(const float* feat, int B, int Hf, int Wf, const float* w, const float* bias,
                                const float* anchors, int img_h, int img_w, float conf, float* cand_boxes,
                                float* cand_scores, hipStream_t st);
hipError_t launch_person_decode(const float* head, int B, int hc, const float* anchors, int img_h, int img_w,
                                float conf, float* cand_boxes, float* cand_scores, hipStream_t st);
hipError_t launch_kh_att(float* x, const float* sa1, const float* w, const float* b, size_t npix, hipStream_t st);
// the attention-weighted KEYPOINT_HEAD input as the split operand of the first
// hmconv (KH mode): [R][57 x 57][128] f16 [hi32 | lo32], ROI r scaled by
// 2^split_exp_of(bound[(r / bdiv) * bstride]), which is also stored to hsc[r][2]
// the same with the spatial attention's 1x1 128 -> 64 fused (split f16 MFMA;
// w1s = pack_split_1x1 layout [64][4][hi32 | lo32] scaled 2^w1_exp)
hipError_t launch_kh_att2(const float* x, const void* w1s, int w1_exp, const float* b1, const float* w2,
                          const float* b2, int R, const float* bound, int bdiv, int bstride, float* hsc, void* out,
                          hipStream_t st);
hipError_t launch_kh_att_split(const float* x, const float* sa1, const float* w, const float* b, int R,
                               const float* bound, int bdiv, int bstride, float* hsc, void* out, hipStream_t st);
hipError_t launch_kh_pool(const float* in, int R, int C, int o, float* out, int out_stride, hipStream_t st);
hipError_t launch_kh_final(const float* lin_r, int r_stride, const float* lin_v, int v_stride, const float* ln_rg,
                           const float* ln_rb, const float* w_r, const float* b_r, const float* ln_vg,
                           const float* ln_vb, const float* w_v, const float* b_v, const int32_t* slot, int R, int P,
                           float* kh_kpts, float* kh_vis, hipStream_t st);

// error reporting shared with the C ABI entry points outside kpd_plan.hip
int kpd_fail_einval(const char* msg);
int kpd_fail_hip(hipError_t e, const char* where);

// ---- stand-alone operators (ops_kernels.hip) ----
// mode: KPD_DECODE_* (include/kpd.h)
hipError_t launch_decode_planes(const float* heat, int planes, int H, int W, int mode, float param, float* kpts,
                                float* scores, float* vis, hipStream_t st);
hipError_t launch_roi_align_nchw(const float* feat, int C, int H, int W, const float* rois, int R, int oh, int ow,
                                 float scale, int sr, int aligned, float* out, hipStream_t st);
hipError_t launch_nchw_rows_to_nhwc(const float* in, int N, int C, int H, int W, float* out, float* stats,
                                    hipStream_t st, float* amax = nullptr, int amax_stride = 0);
hipError_t launch_nhwc_to_nchw(const float* in, int N, int HW, int C, float* out, hipStream_t st);
// padded-channel NHWC <-> NCHW (any C <= Cp; the padding channels written as zero)
hipError_t launch_nhwc_pad_to_nchw(const float* in, int N, int HW, int C, int Cp, float* out, hipStream_t st);
hipError_t launch_nchw_to_nhwc_pad(const float* in, int N, int HW, int C, int Cp, float* out, hipStream_t st);
hipError_t launch_nchw_channel_stats(const float* x, int N, int C, int HW, float* stats, hipStream_t st);
hipError_t launch_gather_planes(const float* x, int N, int C, int HW, const int32_t* idx, int K, float* out,
                                hipStream_t st);
hipError_t launch_conv1x1_nchw(const float* x, int N, int Cin, int HW, const float* w, const float* b, int Cout,
                               float* out, hipStream_t st);
hipError_t launch_fill(float* p, long n, float v, hipStream_t st);

// ---- the heatmap head's 3x3 conv forward / backward on NCHW (conv3_grad.hip) ----
hipError_t launch_conv3_forward(const float* x, const float* w, const float* b, int N, int C, int H, int W, int O,
                                float* y, hipStream_t st);
size_t conv3_wgrad_slices(int N, int H, int W);   // wgrad_part: slices * O * 9C floats
hipError_t launch_conv3_backward(const float* x, const float* w, const float* gy, int N, int C, int H, int W, int O,
                                 float* gx, float* gw, float* gb, float* wgrad_part, hipStream_t st);
