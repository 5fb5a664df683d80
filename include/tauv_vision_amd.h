/*
 * tauv-vision_amd — C ABI of the MI355X (gfx950) CenterNet detection hot path.
 *
 * Drop-in boundary for TAUV-Vision's per-frame CenterNet path (reference
 * Tartan-AUV/TAUV-Vision @ 2024_10_08). The reference is pure Python on PyTorch; each
 * entry point below replaces the reference interface cited next to it. Plain pointers
 * and sizes only (device pointers are HIP device addresses, e.g. a torch tensor's
 * data_ptr()); `stream` is a hipStream_t (NULL = default stream). No exceptions cross
 * this ABI: every call returns TV_OK or a TV_E* code and sets a thread-local message
 * readable with tv_last_error().
 *
 * Layouts
 *   image input   fp32 NCHW [B,3,in_h,in_w], ImageNet-normalised (Centernet.forward,
 *                 centernet.py:65) — or raw u8 frames NHWC [B,in_h,in_w,3] with the
 *                 node's ToTensor+Normalize fused (centernet_node.py:90-92).
 *   head output   fp32 NHWC [B,out_h,out_w,out_cpad]; channel order = the reference
 *                 get_head_channels() order (centernet.py:114-142), out_cpad = round
 *                 up of the channel total to 4. Prediction fields are channel slices.
 *   records       fp32 [B][K][10] = label, score, y, x, h, w, depth (NaN if absent),
 *                 flat peak index (label*H*W + y*W + x), aux0, aux1 (optional pair
 *                 gathered at (label, y, x), e.g. the keypoint affinity of
 *                 decode.py:121-122; NaN if absent); counts int32 [B] = number of
 *                 records with score >= threshold (the host loop's break, decode.py:207).
 */
#ifndef TAUV_VISION_AMD_H
#define TAUV_VISION_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TV_OK 0
#define TV_EINVAL 1    /* bad argument (maps to ValueError / AssertionError) */
#define TV_ESHAPE 2    /* shape the reference would also reject */
#define TV_EHIP 3      /* HIP runtime error */
#define TV_ENOTFOUND 4 /* missing state_dict key */
#define TV_ENOMEM 5

/* TV_F32X3: fp32 activations and weights, each conv product on the pipelined implicit GEMM as three
 * fp16 MFMAs (hi = fp16(x), lo = fp16(x - hi): a_hi*b_hi + a_hi*b_lo + a_lo*b_hi, fp32 accumulation,
 * ~22-bit operands): within the fp32 path's 1e-4 golden tolerance, ~2x its throughput; TV_F32 is the
 * exact-f32 MFMA path. */
typedef enum tv_dtype { TV_F32 = 0, TV_F16 = 1, TV_BF16 = 2, TV_F32X3 = 3 } tv_dtype;

/* Model description: the fields of ModelConfig (config.py:6-35) plus the head list of
 * get_head_channels() (centernet.py:114-142). `arch` selects the network family:
 * TV_ARCH_CENTERNET = Centernet(DLABackbone(heights, channels, downsamples)) (centernet.py:32-92,
 * dla.py:393-416); TV_ARCH_DLA34 = CenterpointDLA34 (centerpoint_dla.py:544-578: DLA-34 base,
 * DLAUp/IDAUp with DCNv2, down ratio 4, head_conv 256; n_levels/heights/channels/downsamples
 * are ignored); TV_ARCH_PROTONET = the YOLACT protonet Masknet (masknet.py:8-55): channels[0] =
 * feature_depth, head_channels[0] = n_prototype_masks, (in_h, in_w) = the fpn[0] feature size;
 * tv_engine_forward takes fpn[0] as fp32 NCHW [B, feature_depth, in_h, in_w] and writes the
 * prototypes as fp32 NHWC [B, 4 in_h, 4 in_w, out_cpad]; TV_ARCH_CENTERNET_BACKBONE = the
 * DLABackbone alone (dla.py:393-416, DLABackbone.forward): the parameters are the "backbone.*"
 * keys of TV_ARCH_CENTERNET, n_heads / head_channels are ignored, and the output is the
 * IDAUpReverse feature map as fp32 NHWC [B, in_h / 2^downsamples, in_w / 2^downsamples,
 * channels[0]]. */
#define TV_ARCH_CENTERNET 0
#define TV_ARCH_DLA34 1
#define TV_ARCH_PROTONET 2
#define TV_ARCH_CENTERNET_BACKBONE 3
typedef struct tv_model_desc {
  int32_t n_levels;          /* len(backbone_heights) */
  int32_t heights[8];        /* backbone_heights */
  int32_t channels[9];       /* backbone_channels, n_levels + 1 entries */
  int32_t downsamples;       /* ModelConfig.downsamples */
  int32_t n_heads;
  int32_t head_channels[16]; /* get_head_channels(object_config) */
  int32_t in_h, in_w;        /* ModelConfig.in_h / in_w */
  int32_t compute_dtype;     /* tv_dtype: TV_F32 = exact-f32 parity mode, TV_F32X3 its three-fp16-MFMA form */
  int32_t arch;              /* TV_ARCH_* */
} tv_model_desc;

typedef struct tv_engine tv_engine;

typedef struct tv_weight_view {
  const char* name;  /* reference state_dict key, e.g. "backbone.dla_down.projection_layer.0.weight" */
  const float* data; /* host fp32, contiguous, PyTorch layout */
  int64_t numel;
} tv_weight_view;

/* Reference state_dict layout of Centernet(DLABackbone(...)) in registration order
 * (what nn.Module.state_dict() yields; replaces model.state_dict() key/shape discovery,
 * centernet.py:32-61, dla.py:8-416). num_batches_tracked entries have ndim 0. */
int tv_model_param_count(const tv_model_desc* desc, int32_t* count);
int tv_model_param_info(const tv_model_desc* desc, int32_t index, char* name, int32_t name_cap,
                        int64_t shape[4], int32_t* ndim);
/* Algorithmic FLOPs per frame (2*MAC over every conv / conv-transpose) and output geometry. */
int tv_model_geometry(const tv_model_desc* desc, double* flops_per_frame, int32_t* out_h, int32_t* out_w,
                      int32_t* out_channels, int32_t* out_cpad);

/* Build an engine from reference-layout weights (replaces Centernet(...).to(device) +
 * load_state_dict(torch.load(...)) + eval(), centernet_node.py:46-48). BatchNorm is
 * folded (eval semantics, eps 1e-5); the engine owns its device copy and is immutable
 * after create, so concurrent forwards on different streams are safe. */
int tv_engine_create(const tv_model_desc* desc, const tv_weight_view* weights, int32_t n_weights,
                     int32_t device, tv_engine** out);
/* Diagnostics only (kernel A/B experiments, tools/): tv_engine_create with kernel-choice
 * overrides given explicitly as "NAME=VALUE;NAME=VALUE" (TV_C3_TW, TV_LAT, TV_SLICES, ... — the
 * list in engine.cpp); an unknown name is TV_EINVAL. The product entry point above takes none
 * and reads no environment variable. */
int tv_engine_create_diag(const tv_model_desc* desc, const tv_weight_view* weights, int32_t n_weights,
                          int32_t device, const char* knobs, tv_engine** out);
int tv_engine_destroy(tv_engine* engine);
/* Workspaces: the first forward of a batch size on a stream allocates that (stream, batch)
 * pair's activation arena (hipMalloc: not inside a graph capture) and keeps it for later calls;
 * a caller that cycles through many batch sizes or streams bounds the device memory with
 * tv_engine_trim. */
/* Allocate the per-(stream, batch) workspace up front (required before graph capture). */
int tv_engine_prepare(tv_engine* engine, int32_t batch, void* stream);
/* Free every cached workspace (synchronises the device; no forward on this engine may be in
 * flight or concurrent, and graphs captured over the freed arenas must not be replayed). */
int tv_engine_trim(tv_engine* engine);
/* Centernet.forward(img) -> Prediction heads (centernet.py:65-92). Async on `stream`. */
int tv_engine_forward(tv_engine* engine, const float* img_nchw, int32_t batch, float* out_nhwc, void* stream);
/* Same from raw u8 RGB frames with ToTensor + Normalize fused (centernet_node.py:90-92). */
int tv_engine_forward_u8(tv_engine* engine, const uint8_t* frames_nhwc, int32_t batch, float* out_nhwc,
                         void* stream);
/* Per-launch timing of one forward (HIP events on `stream`, synchronous): ms[i], flops[i]
 * per launch i < *n_ops (cap entries max); label(i) describes launch i. */
int tv_engine_profile(tv_engine* engine, const float* img_nchw, int32_t batch, float* out_nhwc, void* stream,
                      float* ms, double* flops, int32_t cap, int32_t* n_ops);
/* The same over raw u8 frames (the tv_engine_forward_u8 path). */
int tv_engine_profile_u8(tv_engine* engine, const uint8_t* frames_nhwc, int32_t batch, float* out_nhwc,
                         void* stream, float* ms, double* flops, int32_t cap, int32_t* n_ops);
/* Diagnostic: one forward_u8 exactly as it runs (concurrent slices, grouped launches) with a HIP
 * event before each launch on its slice's stream (synchronous): ms[k * cap + i] = in-situ duration
 * of op i's launch in slice k (a grouped launch's on its first op, 0 for the others), *n_slices
 * slices (tv_engine_slices). The durations include waiting for CUs the other slices hold, which is
 * what rocprofv3's kernel trace of the same run reports. */
int tv_engine_forward_insitu_u8(tv_engine* engine, const uint8_t* frames_nhwc, int32_t batch, float* out_nhwc,
                                void* stream, float* ms, int32_t cap, int32_t* n_slices);
/* Diagnostic: while on, every forward records the group events tv_engine_forward_insitu uses, also
 * into a graph captured meanwhile (event record nodes); tv_engine_insitu_read returns the times the
 * B-frame forward on `stream` (its workspaces' key: the capture stream) last recorded, e.g. after
 * a replay, in the ms[k * cap + i] layout above. */
int tv_engine_set_insitu(tv_engine* engine, int32_t on);
int tv_engine_insitu_read(tv_engine* engine, int32_t batch, void* stream, float* ms, int32_t cap, int32_t* n_slices);
/* The same over the normalised fp32 NCHW input (the tv_engine_forward path). */
int tv_engine_forward_insitu(tv_engine* engine, const float* img_nchw, int32_t batch, float* out_nhwc, void* stream,
                             float* ms, int32_t cap, int32_t* n_slices);
const char* tv_engine_op_label(tv_engine* engine, int32_t index);
/* Kernel family launch `index` uses at this batch size ("conv_pipe", "conv_igemm", "conv_halo",
 * "prep"); "" before the batch's workspace exists. Diagnostic (roofline attribution). */
const char* tv_engine_op_kernel(tv_engine* engine, int32_t batch, int32_t index);
/* How a forward of `batch` frames is launched: as *n_slices (1..TV_MAX_SLICES) concurrent slices
 * of slice_batch[0..n_slices) frames, the rest of slice_batch zeroed (diagnostic: per-launch
 * roofline attribution). */
#define TV_MAX_SLICES 8
int tv_engine_slices(tv_engine* engine, int32_t batch, int32_t* n_slices, int32_t slice_batch[TV_MAX_SLICES]);

/* The node's preprocessing of camera frames (centernet_node.py:90-92): T.ToTensor (u8 / 255) ->
 * T.Resize((dst_h, dst_w)) (torchvision 0.15.2 tensor path: bilinear, align_corners=False, no
 * antialias, evaluated as torch's CPU upsample_bilinear2d does) -> T.Normalize(ImageNet). u8 RGB
 * frames NHWC [B, src_h, src_w, 3] -> normalised fp32 NCHW [B, 3, dst_h, dst_w], the input of
 * tv_engine_forward. (Frames already at the model size take tv_engine_forward_u8 instead: the
 * resize is then the identity and ToTensor + Normalize are fused into the stem.) */
int tv_preprocess_u8(const uint8_t* frames, int32_t B, int32_t src_h, int32_t src_w, int32_t dst_h, int32_t dst_w,
                     float* img_nchw, void* stream);

/* heatmap_nms(sigmoid?(heat), k) (decode.py:239-252) over any strided [B,C,H,W] fp32
 * view; `out` is dense [B,C,H,W]. k must be odd and >= 1 (else TV_EINVAL, like the
 * reference's assert). */
int tv_heatmap_nms(const float* heat, const int64_t strides[4], int32_t B, int32_t C, int32_t H, int32_t W,
                   int32_t kernel_size, int32_t apply_sigmoid, float* out, void* stream);
/* heatmap_detect (decode.py:255-279) on a dense [B, n] map: exact top-K per row,
 * descending, ties to the smaller flat index. */
int tv_heatmap_topk(const float* peaks, int32_t B, int64_t n, int32_t K, float* score, int32_t* index,
                    void* stream);
/* heatmap_detect()'s index [B,K,2] (y, x) and label [B,K] (int64) from flat indices
 * (decode.py:271-277; integer division, identical to the reference's float32 division
 * while C*H*W < 2^24). */
int tv_index_split(const int32_t* flat, int32_t B, int32_t K, int32_t H, int32_t W, int64_t* index, int64_t* label,
                   void* stream);
/* decode() (decode.py:179-236) / the object and keypoint parts of decode_keypoints()
 * (decode.py:56-135).
 * mode 0: y = (R*iy + offset_y)/in_h, depth = 1/sigmoid(d) - 1; mode 1: y = iy/out_h,
 * depth = 1/sigmoid(d), offset unused. Strides are element strides of the [B,C,H,W]
 * heatmap view and of the [B,H,W,ch] size/offset/depth views (depth may be NULL).
 * aux (may be NULL): pair gathered per record at element (b, label, j, y, x) with
 * aux_strides[5] (the [B,K,2,H,W] keypoint_affinity view).
 * workspace: tv_decode_workspace_size() bytes of device memory, ZERO-FILLED before its first use
 * (it carries the per-image peak keys and the arrival counters of the call's single launch, which
 * leaves the counters at zero again for the next call) — one call at a time per workspace. The
 * counters sit at fixed offsets (a 512 KiB head: one pair per image index up to 65535), so one
 * zero-filled workspace serves every later call whose tv_decode_workspace_size() it covers, at
 * any B or heatmap geometry. */
int tv_decode_workspace_size(int32_t B, int32_t C, int32_t H, int32_t W, int32_t K, int64_t* bytes);
int tv_decode(const float* heat, const int64_t heat_strides[4], const float* size, const int64_t size_strides[4],
              const float* offset, const int64_t offset_strides[4], const float* depth,
              const int64_t depth_strides[4], int32_t B, int32_t C, int32_t H, int32_t W, int32_t K,
              int32_t mode, int32_t ratio, int32_t in_h, int32_t in_w, float score_threshold,
              const float* aux, const int64_t aux_strides[5], float* records, int32_t* counts, void* workspace,
              int64_t workspace_bytes, void* stream);

/* YOLACT post-processing (reference src/tauv_vision/yolact/model/), fp32,
 * device pointers, async on `stream`.
 * box_decode (boxes.py:55-61): enc [B,A,4] (y, x, h, w encodings), anchor [anchor_batch,A,4]
 *   (anchor_batch 1 broadcasts like the reference's [1,A,4] anchors), out [B,A,4]. */
int tv_yolact_box_decode(const float* box_encoding, const float* anchor, int32_t B, int32_t A, int32_t anchor_batch,
                         float variance0, float variance1, float* box, void* stream);
/* box_encode (boxes.py:45-53): box [B,A,4] (y, x, h, w), anchor [anchor_batch,A,4] -> encodings [B,A,4]. */
int tv_yolact_box_encode(const float* box, const float* anchor, int32_t B, int32_t A, int32_t anchor_batch,
                         float variance0, float variance1, float* box_encoding, void* stream);
/* nms (nms.py:7-29): class-agnostic fast NMS of batch 0 — classification [A, C+1] logits and
 * box [A, 4] of batch 0; writes the kept anchor indices (descending confidence) to det[<= top_k]
 * (int64) and their number to *n_det (device int32). Any anchor count; the sort workspace is
 * allocated stream-ordered (hipMallocAsync) — use the batched entry point under graph capture. */
int tv_yolact_fast_nms(const float* classification, int32_t A, int32_t n_classes_with_bg, const float* box,
                       int32_t top_k, float iou_threshold, float confidence_threshold, int64_t* det, int32_t* n_det,
                       void* stream);
/* The same for B images at once (the reference's nms applied to every image of a batch):
 * classification [B,A,C+1], box [B,A,4] -> det [B][min(top_k, A)] int64 (row b: n_det[b] kept
 * indices), n_det [B] int32; workspace of tv_yolact_nms_workspace_size() bytes. */
int tv_yolact_nms_workspace_size(int32_t B, int32_t A, int32_t top_k, int64_t* bytes);
int tv_yolact_fast_nms_batched(const float* classification, int32_t B, int32_t A, int32_t n_classes_with_bg,
                               const float* box, int32_t top_k, float iou_threshold, float confidence_threshold,
                               int64_t* det, int32_t* n_det, void* workspace, int64_t workspace_bytes, void* stream);
/* assemble_mask (masks.py:8-21): prototypes [K,H,W] at element strides proto_strides (k, y, x) —
 * contiguous NCHW or the protonet's NHWC output view —, coefficients [n,K], box [n,4] (y, x, h, w
 * normalised) or NULL -> mask [n,H,W] = sigmoid(coeff . proto) x inclusive box mask. K <= 37. */
int tv_yolact_assemble_mask(const float* mask_prototype, const int64_t proto_strides[3], int32_t K, int32_t H,
                            int32_t W, const float* mask_coeff, const float* box, int32_t n, float* mask,
                            void* stream);
/* The same for B images: prototypes at strides (b, k, y, x), coefficients [B][n_max][K], boxes
 * [B][n_max][4] or NULL, counts [B] (device int32, detections per image; NULL = n_max) ->
 * masks [B][n_max][H][W] (rows d >= counts[b] untouched). */
int tv_yolact_assemble_masks(const float* mask_prototype, const int64_t proto_strides[4], int32_t B, int32_t K,
                             int32_t H, int32_t W, const float* mask_coeff, const float* box, const int32_t* counts,
                             int32_t n_max, float* mask, void* stream);
/* The node's mask step straight from the batched NMS output (yolact_node.py:134:
 * assemble_mask(proto[b], mask_coeff[b, det], box[b, det])): coefficients [B][A][K] and boxes
 * [B][A][4] (or NULL) of every anchor, det [B][n_max] int64 kept anchors and counts [B] as written
 * by tv_yolact_fast_nms_batched (n_max = its min(top_k, A)) -> masks [B][n_max][H][W]. */
int tv_yolact_assemble_masks_indexed(const float* mask_prototype, const int64_t proto_strides[4], int32_t B,
                                     int32_t K, int32_t H, int32_t W, const float* mask_coeff, const float* box,
                                     int32_t A, const int64_t* det, const int32_t* counts, int32_t n_max, float* mask,
                                     void* stream);

/* Training targets of the CenterNet loss (loss.py:31-135), fp32, device pointers, async on `stream`.
 * generate_heatmap (loss.py:31-72): valid [B,n_objects] u8 (bool), label [B,n_objects] int64,
 *   center [B,n_objects,2] fp32 (y, x normalised) -> heatmap [B,n_labels,in_h/ratio,in_w/ratio]:
 *   per valid object exp(-((x-cx)^2 + (y-cy)^2) / (2 sigma^2)) maxed into its label's plane, with
 *   (cy, cx) = floor(center * in / ratio) and sigma = max(sigma, 0.1) (the reference passes
 *   TrainConfig.keypoint_heatmap_sigma); nan_to_num. A label outside [0, n_labels) is skipped
 *   (the Python wrapper raises IndexError first, like the reference's indexing). */
int tv_train_heatmap(const uint8_t* valid, const int64_t* label, const float* center, int32_t B, int32_t n_objects,
                     int32_t n_labels, int32_t in_h, int32_t in_w, int32_t downsample_ratio, double sigma,
                     float* heatmap, void* stream);
/* generate_keypoint_heatmap (loss.py:75-135): keypoint instances [B,n_instances] (valid u8, label
 * int64, center fp32 x2, owning object index int64 into center [B,n_objects,2]) -> heatmap and
 * affinity_weight [B,n_keypoints,H,W] (Gaussians of heatmap_sigma / affinity_sigma, max), affinity
 * [B,n_keypoints,2,H,W] (unit displacement from the owning object's center to each cell, of the
 * instance nearest to that cell; the earliest instance wins ties); nan_to_num of all three. */
int tv_train_keypoint_targets(const uint8_t* keypoint_valid, const int64_t* keypoint_label,
                              const float* keypoint_center, const int64_t* keypoint_object_index, const float* center,
                              int32_t B, int32_t n_instances, int32_t n_objects, int32_t n_keypoints, int32_t in_h,
                              int32_t in_w, int32_t downsample_ratio, double heatmap_sigma, double affinity_sigma,
                              float* heatmap, float* affinity_weight, float* affinity, void* stream);

/* Diagnostics (GPU tests): one DeformConv2d(x, offset, sigmoid(mask)) (DeformConv.forward,
 * centerpoint_dla.py:389-391: 3x3, stride 1, pad 1) + bias + activation (0 none, 1 ReLU, 2 leaky)
 * through the kernel the engine uses for DLA-34's DeformConv layers. x: compute-dtype NHWC
 * [B,H,W,C]; om: compute-dtype NHWC [B,H,W,om_ldc] = (dy, dx) per tap (18) + 9 mask logits (the
 * engine's fused offset/mask conv output); weight: host fp32 [N][C][3][3], bias host fp32 [N];
 * out: compute-dtype NHWC [B,H,W,N]. variant: 0 = fused dcn_gemm (32-channel k-steps),
 * 1 = fused dcn_gemm64 (tile by size), 2 = dcn_gemm64 with 64-pixel tiles, 3 = unfused sampling +
 * implicit GEMM (the fp32 path; the only variant for TV_F32), 4 = dcn_win (the LDS-window kernel the
 * engine uses for C == N == 64; TV_EINVAL otherwise), 5 = dcn_gemm64d (gathers two k-steps ahead),
 * 6 / 7 / 8 = dcn_gemm64 on 64-pixel tiles with split-K over 3 / 4 / 9 tap ranges (the engine's
 * small-batch form). Synchronous; allocates. */
int tv_diag_dcn_conv(const void* x, const void* om, int32_t B, int32_t H, int32_t W, int32_t C, int32_t om_ldc,
                     const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, int32_t variant,
                     void* out, void* stream);

/* Diagnostics (GPU tests): a Root-style 1x1 conv (dla.py:58-76: Conv2d(sum C, N, 1) over
 * torch.cat(children, 1) + bias + activation) through conv1x1_stream, the kernel the engine runs for
 * stride-1 1x1 layers. src[k]: compute-dtype [M][ldc[k]] pixel rows of segment k (C[k] channels,
 * a multiple of 64); weight: host fp32 [N][sum C] in segment order; bias: host fp32 [N]; out:
 * compute-dtype [M][out_ldc], N channels (N a multiple of 8, <= 512). TV_F16 / TV_BF16 only.
 * Synchronous; allocates. Returns TV_EINVAL for shapes the kernel does not take. */
int tv_diag_conv1x1(const void* const* src, const int32_t* C, const int32_t* ldc, int32_t nseg, int32_t M,
                    const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, void* out,
                    int32_t out_ldc, void* stream);

/* Diagnostics (GPU tests): one conv over nseg concatenated-K segments through conv_burst, the
 * engine's one-shot kernel for the small pyramid levels (Tree convs with the fused 1x1
 * conv_residual dla.py:8-52, Roots dla.py:58-76, IDAUp convs dla.py:212-284). Segment k:
 * src[k] compute-dtype NHWC [B, H, W, ldc] with geom[6k..6k+5] = H, W, C, ldc, kernel (1 or 3,
 * padding kernel / 2), stride; a 3x3 segment must be stride 1 over the output grid. weight: host
 * fp32 [N][K] (K segment-major, tap-major, channel-minor), bias: host fp32 [N]; out: compute-dtype
 * [B, Ho, Wo, out_ldc]. TV_F16 / TV_BF16; TV_EINVAL for layers the kernel does not take.
 * Synchronous; allocates. */
int tv_diag_conv_burst(const void* const* src, const int32_t* geom, int32_t nseg, int32_t B, int32_t Ho, int32_t Wo,
                       const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, void* out,
                       int32_t out_ldc, void* stream);

/* Diagnostics (host only, no GPU needed): conv_burst's launch plan for a layer geometry (geom as
 * tv_diag_conv_burst, N output channels). out[0] = 1 when the kernel takes the layer, out[1] its
 * dynamic LDS bytes, out[2] the end of the highest LDS byte any of its accesses touches over every
 * tile position (the kernel's own index arithmetic; <= out[1], else the plan refuses the layer),
 * out[3] the LDS the layer's staging would need. */
int tv_diag_burst_plan(const int32_t* geom, int32_t nseg, int32_t B, int32_t Ho, int32_t Wo, int32_t N, int32_t* out);

/* Diagnostics (GPU tests): one narrow-channel Conv2d(C, N, 3, stride, padding 1) + bias + activation
 * (DLA-34's full-resolution base levels, centerpoint_dla.py:242-246 `_make_conv_level`) through
 * conv_small, the engine's kernel for them: C -> N in {16 -> 16, 16 -> 32, 32 -> 32 (stride 1),
 * 32 -> 64 (stride 2)}. src: compute-dtype NHWC [B, H, W, ldc]; weight: host fp32 [N][C][3][3];
 * bias: host fp32 [N]; out: compute-dtype NHWC [B, Ho, Wo, out_ldc]. variant: 0 = per-lane register
 * gathers, 1 = LDS-halo tiles (a tile per workgroup), 2 = LDS-halo tiles on a persistent grid. TV_F16 / TV_BF16; TV_EINVAL for shapes the kernel does not take.
 * Synchronous; allocates. */
int tv_diag_conv_small(const void* src, int32_t B, int32_t H, int32_t W, int32_t C, int32_t ldc, const float* weight,
                       const float* bias, int32_t N, int32_t stride, int32_t act, int32_t dtype, int32_t variant,
                       void* out, int32_t out_ldc, void* stream);

/* Diagnostics (GPU tests): one ConvTranspose2d(C, N, 3, stride 2, padding 1, output_padding 1) +
 * bias + activation (YOLACT protonet up-sampling, masknet.py:21,33) through convt3, the engine's
 * kernel for it. src: compute-dtype NHWC [B, H, W, ldc], C channels (a multiple of 32); weight: host
 * fp32 [C][N][3][3] (nn.ConvTranspose2d layout), N a multiple of 64; bias: host fp32 [N]; out:
 * compute-dtype NHWC [B, 2H, 2W, out_ldc]. tile_w x tile_h: the input tile (<= 256 pixels, halo
 * (tile_w + 1)(tile_h + 1) <= 307), 0 = the kernel's choice. TV_F16 / TV_BF16; TV_EINVAL for shapes
 * the kernel does not take. Synchronous; allocates. */
int tv_diag_convt3(const void* src, int32_t B, int32_t H, int32_t W, int32_t C, int32_t ldc, const float* weight,
                   const float* bias, int32_t N, int32_t act, int32_t dtype, int32_t tile_w, int32_t tile_h, void* out,
                   int32_t out_ldc, void* stream);

const char* tv_last_error(void);
const char* tv_version(void);

#ifdef __cplusplus
}
#endif
#endif
