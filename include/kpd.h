/* kpd.h -- C ABI of the MI355X-native keypoint-detection hot path (libkpd.so).
 *
 * Drop-in boundary for the reference's `MultiPersonKeypointModel.forward`
 * (eval, caller-given person boxes).  Plain pointers and sizes only; device
 * pointers are HIP device memory on the plan's device, streams are
 * hipStream_t passed as void*.  The library owns the plan (packed weights,
 * workspace); the caller owns every input/output buffer.
 *
 * Reference interfaces replaced (paths under the reference repo):
 *   kpd_plan_create/set_tensor/finalize
 *       <- MultiPersonKeypointModel.__init__ + load_state_dict
 *          dll/models/keypoint_model.py:49-71, scripts/predict.py:30-62
 *          (tensor names are the reference's state-dict keys; BN folding and
 *           NHWC/MFMA repacking happen inside finalize)
 *   kpd_forward
 *       <- MultiPersonKeypointModel.forward(batch) with batch['bboxes']
 *          dll/models/keypoint_model.py:73-210 (eval / no_grad branch):
 *          backbone.py:258-264, keypoint_model.py:653-661, :212-228,
 *          heatmap_head.py:81-113, keypoint_model.py:250-313, :230-248
 *   kpd_nms
 *       <- PERSON_HEAD.non_max_suppression  dll/models/person_head.py:96-139
 *
 * Every function returns 0 on success or a negative KPD_E* code; the message
 * of the last failure on the calling thread is available from kpd_last_error().
 */
#ifndef KPD_H_
#define KPD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KPD_OK 0
#define KPD_EINVAL (-1)     /* bad argument / shape (reference raises ValueError) */
#define KPD_EHIP (-2)       /* HIP runtime error */
#define KPD_ESTATE (-3)     /* plan not finalized / missing weights */

#define KPD_PRECISION_FP32 0   /* every conv on fp32-input MFMA (exact fp32 products) */
#define KPD_PRECISION_MIXED 1  /* heatmap-head convs on bf16 MFMA, fp32 accumulate; backbone fp32 */
#define KPD_PRECISION_SPLIT 2  /* fp32-accurate: FPN level 0 and the heatmap-head convs as three
                                  f16 MFMA products of hi/lo operand splits, fp32 accumulate */

typedef struct kpd_plan kpd_plan;

const char* kpd_last_error(void);
const char* kpd_version(void);

/* Create an empty plan bound to HIP device `device`.  in_channels: 1 or 3
 * (BackboneConfig.in_channels, reference backbone.py:251-252). */
int kpd_plan_create(int device, int in_channels, kpd_plan** out);

/* Register one reference state-dict tensor (fp32, host memory, contiguous,
 * shape as in the reference).  Unknown names are ignored (the reference's
 * predict.py filters unknown keys the same way, predict.py:47-57). */
int kpd_plan_set_tensor(kpd_plan* plan, const char* name, const float* host_data,
                        const int64_t* shape, int ndim);

/* Fold BN, repack weights (NHWC / MFMA layouts) and upload them.
 * Fails with KPD_ESTATE listing any missing tensor. */
int kpd_plan_finalize(kpd_plan* plan, int precision);

void kpd_plan_destroy(kpd_plan* plan);

/* HeatmapHead stages (kpd_heatmap_head) */
#define KPD_HEAD_CHANNEL_ATT 1
#define KPD_HEAD_SPATIAL_ATT 2
#define KPD_HEAD_CONVS 4
#define KPD_HEAD_ALL 7

#define KPD_FLAG_DETECT 1     /* no caller boxes: person detector + NMS WRITE boxes [B][P][4] */
#define KPD_FLAG_DUAL_HEAD 2  /* also run KEYPOINT_HEAD on 128-ch ROI features */
/* Write every pixel of FPN level 0.  By default, with caller boxes, the
 * level-0 conv stores only the pixels the ROI aligns of the image's boxes
 * read (the channel statistics of the top-k still see every pixel), and
 * kpd_debug_copy has no "feat0"; this flag stores the whole map (inspection,
 * tests).  Outputs are identical either way. */
#define KPD_FLAG_FULL_LEVEL0 4

/* Full eval forward.
 *   image:  [B][C][H][W] fp32 (NCHW, as the reference receives it), device
 *   boxes:  [nbox_images][P][4] fp32 cxcywh normalised to [0,1], device;
 *           nbox_images <= B (the reference iterates over the box list).
 *           With KPD_FLAG_DETECT it is an OUTPUT (nbox_images == B, P = max
 *           persons kept per image, zero padded) -- build-defined glue for
 *           the reference's person-detector branch.
 *   keypoints:    [nbox_images][P][1][17][2]  fp32 out
 *   visibilities: [nbox_images][P][1][17][3]  fp32 out (one-hot 3-class)
 *   heatmap:      [nbox_images][P][17][56][56] fp32 out, may be NULL
 *   kh_keypoints / kh_visibilities: [nbox_images][P][1][17][2|3] sigmoid
 *                 outputs of KEYPOINT_HEAD (KPD_FLAG_DUAL_HEAD), else NULL
 *   box_scores:   [B][P] detector scores (KPD_FLAG_DETECT), may be NULL
 *   topk_out:     [B][64] int32 channel indices, may be NULL (debug)
 * All-zero boxes are skipped and the remaining persons compacted, images
 * without a valid box get the reference's dummy person, P is kept as the
 * padded person count -- exactly keypoint_model.py:138-206. */
int kpd_forward(kpd_plan* plan, const float* image, int B, int C, int H, int W,
                float* boxes, int nbox_images, int P, int flags,
                float* keypoints, float* visibilities, float* heatmap,
                float* kh_keypoints, float* kh_visibilities, float* box_scores,
                int32_t* topk_out, void* stream);

/* Detector thresholds (PersonDetectionConfig.conf_threshold /
 * nms_iou_threshold, model_config.py:27-28); defaults 0.3 / 0.3. */
int kpd_plan_set_detector(kpd_plan* plan, float conf_threshold, float nms_iou_threshold);

/* Copy an internal buffer recorded by the last kpd_forward into `dst`
 * (device memory, `bytes` long).  Names: "feat0" ([B][Hf][Wf][128] NHWC f32),
 * "scores" ([B][128] f32), "roi" ([R][56][56][64] f32), "tap0".."tap3".
 * Writes the buffer size to *size_out when dst == NULL. */
int kpd_debug_copy(kpd_plan* plan, const char* name, void* dst, size_t bytes, size_t* size_out,
                   void* stream);

/* Per-stage device timing with HIP events recorded on the launch stream.
 * kpd_plan_timing(plan, 1) clears previous records and enables recording for
 * subsequent kpd_forward calls; kpd_plan_timing_query returns the summed
 * milliseconds and the number of recorded launches of one stage
 * ("body", "fpn_lateral", "fpn0", "topk", "roi_align", "hm_attention",
 * "hm_conv1", "hm_conv2", "hm_conv3", "hm_final_decode"). */
int kpd_plan_timing(kpd_plan* plan, int enable);
/* Restrict the recording to one stage (NULL or "" = every stage): a single
 * kernel timed inside a throughput run without the other stages' event
 * bubbles. */
int kpd_plan_timing_stage(kpd_plan* plan, const char* stage);
int kpd_plan_timing_query(kpd_plan* plan, const char* stage, double* total_ms, int* count);

/* Greedy NMS on one set of n cxcywh boxes (device), reference semantics
 * (IoU > thr suppressed, score-descending order, ties -> lower index).
 * keep: [n] int32 out (first *n_keep valid), n_keep: [1] int32 out (device).
 * max_output <= 0 means unlimited. */
int kpd_nms(const float* boxes, const float* scores, int n, float iou_threshold, int max_output,
            int32_t* keep, int32_t* n_keep, void* stream);

/* Preprocessing: the reference's ITransform
 * (dll/data/transforms.py:9-113) on the device.  src: uint8 HWC image
 * (C = 1 or 3, row pitch in bytes, device memory); dst: fp32 [C'][out_h][out_w]
 * (device), C' = 1 with KPD_PRE_GRAY.  Stages in order: RGB->gray (cv2
 * fixed point), CLAHE per plane (clip_limit, tiles_x x tiles_y), the gray
 * pipeline's edge blend (to_grayscale_clahe :55-73: blur, median, Canny,
 * morphology, addWeighted; single plane only), Gaussian 3x3 sigma 0.5 (RGB
 * pipeline, :105), PIL-exact bilinear resize, ToTensor + Normalize(mean, std)
 * (host arrays of C' floats).  Stream-ordered scratch (hipMallocAsync).
 * Replaces ITransform.__call__ (transforms.py:110-113). */
#define KPD_PRE_GRAY 1
#define KPD_PRE_CLAHE 2
#define KPD_PRE_BLUR 4
#define KPD_PRE_EDGES 8
int kpd_preprocess(const uint8_t* src, int height, int width, int channels, int pitch, int flags, float clip_limit,
                   int tiles_x, int tiles_y, int out_h, int out_w, const float* mean, const float* std, float* dst,
                   void* stream);

/* Training / evaluation targets: generate_target_heatmap
 * (dll/models/heatmap_head.py:163-224).  kpts: [planes][2] normalised (x, y)
 * (device), out: [planes][H][W] fp32 (device); the (6*int(sigma)+1)^2
 * normalised Gaussian is centred at (floor(x*W), floor(y*H)) and cropped;
 * keypoints outside [0,1) leave their plane zero.  Synchronises the stream
 * (the kernel table is staged from host memory). */
int kpd_target_heatmaps(const float* kpts, int planes, int H, int W, float sigma, float* out, void* stream);

/* Validation metrics: Trainer._calculate_validation_metrics
 * (dll/training/trainer.py:384-429).  pred, gt: [n][2], vis: [n] (device);
 * thresholds: host array (<= 16).  out (device) = [ADE, PCK_t...]: ADE = mean
 * ||pred-gt|| over vis > 0, PCK_t = #(dist <= t and vis > 0) / n; all zero
 * when nothing is visible. */
int kpd_keypoint_metrics(const float* pred, const float* gt, const float* vis, long n, const float* thresholds,
                         int n_thresholds, float* out, void* stream);

/* Training loss: AdaptiveHeatmapLoss.forward
 * (dll/losses/keypoint_loss.py:202-280).  pred, gt: [B][K][H][W] fp32,
 * target_weight: [B][K] or NULL (all device).  Threshold = clamp(torch.quantile(
 * gt, 0.9), 0.05, 0.3) when adaptive_threshold (radix select on the device,
 * torch's fp32 rank / lerp), else 0.1.  loss_out (device, 1 float) = mean of
 * the weighted focal MSE; grad_pred (device [B][K][H][W] or NULL) = d loss /
 * d pred; threshold_out (device, 1 float, or NULL) = the threshold used.
 * Deterministic (fixed-order double reductions). */
int kpd_adaptive_heatmap_loss(const float* pred, const float* gt, const float* target_weight, int B, int K, int H,
                              int W, float keypoint_weight, float background_weight, int adaptive_threshold,
                              float focal_alpha, float* loss_out, float* grad_pred, float* threshold_out,
                              void* stream);

/* Concurrency: a forward pass over B >= 32 images runs as min(n, B/16)
 * contiguous sub-batches on as many streams (forked from / joined back into
 * the caller's stream), so the latency-bound small launches of one sub-batch
 * overlap the other's.  n in [1, 4]; default 1 (n = 2 measured +4% images/s at
 * C2, but every kernel then shares the GPU with the other sub-batch, so
 * per-kernel timings no longer describe the kernel).  Results do not depend
 * on n: every split-precision scale is per image / per ROI. */
int kpd_plan_set_streams(kpd_plan* plan, int n);

/* Not part of the reference interface: replay whole forwards as hipGraphs.
 * With enable != 0, a kpd_forward call whose signature (shapes, flags, every
 * buffer address, the stream) repeats runs eagerly once, is captured the
 * second time and from then on is one hipGraphLaunch on the caller's stream
 * (the ~60 launches of a forward, not its kernels, set the latency of a
 * small batch).  A workspace re-carve or re-finalize invalidates the graphs;
 * stage timing forces eager forwards.  Results are identical either way.
 * Default: off (KPD_GRAPH=1 in the environment: on).  Measured at 64 and 1
 * images back to back, replay is no faster than the eager launches (the GPU
 * is the bound there); one synchronous 1-image forward (C1) took 0.62 ms
 * replayed against 0.67 ms eager.
 * The signature includes every buffer address: replay needs caller-owned
 * buffers reused from call to call (a caller that allocates new outputs per
 * call gets a new signature, i.e. an eager run, whenever an address changes).
 * enable = 2: on, and the next capture is abandoned as if it had failed (the
 * call then runs eagerly with the plan's workspace state restored) -- a test
 * hook for that recovery path. */
int kpd_plan_set_graphs(kpd_plan* plan, int enable);

/* Diagnostics (not part of the reference interface): times the LDS-DMA 3x3
 * conv (conv_glds.hip) on synthetic operands, N x H x W pixels, cin -> cout;
 * split != 0 selects the fp32-accurate FPN level-0 form (cin = cout = 128).
 * dbg: 0 full kernel, 1 without the K-loop loads, 2 without the MFMAs,
 * 4 with an L2-resident A working set.  *ms = mean time per launch.  The
 * ablations (dbg != 0) exist only in a diagnostic build (kpd_build_flags). */
int kpd_bench_conv16(int split, int N, int H, int W, int cin, int cout, int dbg, int iters, float* ms);

/* Build flags of this library: bit 0 (KPD_BUILD_DIAG) = diagnostic build
 * (make DIAG=1), which reads the KPD_* A/B and ablation switches and the
 * KPD_STAMPS phase stamps from the environment.  The default build reads
 * none of them (only KPD_GRAPH, the kpd_plan_set_graphs default). */
#define KPD_BUILD_DIAG 1
int kpd_build_flags(void);

/* ---- Stand-alone operators: the reference's submodule forwards and helper
 * functions, for callers that use them outside MultiPersonKeypointModel.forward.
 * Tensors are NCHW fp32 device memory, exactly as the reference modules take
 * and return them.  Plan-based entries need a plan holding that submodule's
 * weights under the model's state-dict names (a partial plan is fine: a
 * finalize packs the components it finds -- backbone.body, backbone.fpn,
 * channel_attention, heatmap_head, person_detector, keypoint_head). */

/* HeatmapHead.forward (heatmap_head.py:81-113): x [R][64][56][56] ->
 * heat [R][17][56][56] (sigmoid maps); attention weights ch_w [R][64] and
 * sp_w [R][56][56] (nullable).  parts = KPD_HEAD_* selects the stages: a
 * disabled attention uses weights 1 (use_attention=False), parts without
 * KPD_HEAD_CONVS computes only the attention weights (the attention modules'
 * own forwards, :129-151). */
int kpd_heatmap_head(kpd_plan* plan, const float* x, int R, int H, int W, int parts, float* heat, float* ch_w,
                     float* sp_w, void* stream);

/* KEYPOINT_HEAD.forward (keypoint_head.py:50-62): x [R][128][56][56] ->
 * keypoints [R][17][2], visibility [R][17][3] (sigmoid outputs). */
int kpd_keypoint_head(kpd_plan* plan, const float* x, int R, int H, int W, float* keypoints, float* visibility,
                      void* stream);

/* MobileNetV3Wrapper.forward (backbone.py:258-264 + LightweightFPN :29-39):
 * image [B][C][H][W] -> the four FPN levels out_i [B][128][h_i][w_i] at the
 * strides of features.0 / .3 / .8 / .12 (2, 8, 16, 32). */
int kpd_backbone(kpd_plan* plan, const float* image, int B, int C, int H, int W, float* out0, float* out1,
                 float* out2, float* out3, void* stream);

/* MobileNetV3Wrapper.body(x) (backbone.py:250-254: create_feature_extractor
 * over mobilenet_v3_small, return_nodes features.0 / .3 / .8 / .12):
 * image [B][C][H][W] -> feat0 [B][16][h0][w0], feat1 [B][24][h3][w3],
 * feat2 [B][48][h8][w8], feat3 [B][576][h11][w11] (strides 2, 8, 16, 32). */
int kpd_backbone_body(kpd_plan* plan, const float* image, int B, int C, int H, int W, float* feat0, float* feat1,
                      float* feat2, float* feat3, void* stream);

/* LightweightFPN.forward (backbone.py:29-39) on caller taps feat_i
 * [B][c_i][h_i][w_i], c = 16, 24, 48, 576; sizes = {h0, w0, h1, w1, h2, w2,
 * h3, w3} (host array).  Lateral i+1 is nearest-resized to (h_i, w_i) and added to lateral
 * i (F.interpolate 'nearest' indexing); out_i [B][128][h_i][w_i] = fpn_convs[i]
 * (3x3 + BN + ReLU) of lateral i, exact fp32 products. */
int kpd_backbone_fpn(kpd_plan* plan, const float* feat0, const float* feat1, const float* feat2, const float* feat3,
                     int B, const int* sizes, float* out0, float* out1, float* out2, float* out3, void* stream);

/* ChannelAttention.forward (keypoint_model.py:33-44) on x [B][128][H][W] ->
 * scores [B][128] (sigmoid); select_top_k_channels (:653-661): topk [B][k]
 * int32 (descending score, ties to the lower index) and selected
 * [B][k][H][W] = x[b, topk[b]] (both nullable).  k = 64. */
int kpd_channel_attention(kpd_plan* plan, const float* x, int B, int C, int H, int W, float* scores, int32_t* topk,
                          int k, float* selected, void* stream);

/* Heatmap decoders over `planes` maps of H x W (device):
 *   KPD_DECODE_ARGMAX     decode_heatmaps (heatmap_head.py:265-296)
 *   KPD_DECODE_SUBPIXEL   decode_heatmaps_subpixel (:298-370), param = window size
 *   KPD_DECODE_SOFTARGMAX decode_heatmaps_soft_argmax (:372-413), param = temperature
 *   KPD_DECODE_MODEL      MultiPersonKeypointModel.decode_heatmap (keypoint_model.py:250-313):
 *                         soft-argmax + 3-class visibility vis [planes][3]
 * keypoints [planes][2] normalised, scores [planes] (the maximum; nullable). */
#define KPD_DECODE_ARGMAX 0
#define KPD_DECODE_SUBPIXEL 1
#define KPD_DECODE_SOFTARGMAX 2
#define KPD_DECODE_MODEL 3
int kpd_decode_heatmaps(const float* heat, int planes, int H, int W, int mode, float param, float* keypoints,
                        float* scores, float* vis, void* stream);

/* torchvision.ops.roi_align as extract_roi_features calls it
 * (keypoint_model.py:212-228): features [B][C][H][W], rois [R][5] =
 * (batch index, x1, y1, x2, y2) -> out [R][C][out_h][out_w]. */
int kpd_roi_align(const float* features, int B, int C, int H, int W, const float* rois, int R, int out_h, int out_w,
                  float spatial_scale, int sampling_ratio, int aligned, float* out, void* stream);

/* 1x1 convolution with bias on NCHW (PERSON_HEAD.forward's box head,
 * person_head.py:141-166): out [B][Cout][HW] = w [Cout][Cin] . x [B][Cin][HW] + b. */
int kpd_conv1x1(const float* x, int B, int Cin, int HW, const float* w, const float* b, int Cout, float* out,
                void* stream);

/* Training side (the backward of the heatmap head's 3x3
 * convolutions: nn.Conv2d(C, O, 3, padding=1), heatmap_head.py:31-45,55-66,
 * whose gradients the reference takes from autograd in Trainer.train,
 * trainer.py:263,272).  NCHW fp32 device tensors; fp32-accurate arithmetic
 * (the heatmap convs' split f16 hi / lo products with fp32 accumulation at
 * 56 x 56 with 64 | 256 channels, and for every wgrad; exact fp32 products
 * otherwise), deterministic fixed-order sums.  Scratch comes from the
 * stream-ordered allocator; no host synchronisation.
 *   kpd_conv3x3_forward:  y [N][O][H][W] = conv(x [N][C][H][W], w [O][C][3][3]) + b (b nullable)
 *   kpd_conv3x3_backward: for gy = dL/dy [N][O][H][W]: gx = dL/dx, gw = dL/dw
 *                         [O][C][3][3], gb = dL/db [O] (each nullable). */
int kpd_conv3x3_forward(const float* x, const float* w, const float* b, int N, int C, int H, int W, int O, float* y,
                        void* stream);
int kpd_conv3x3_backward(const float* x, const float* w, const float* gy, int N, int C, int H, int W, int O,
                         float* gx, float* gw, float* gb, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KPD_H_ */
