// extern "C" boundary (include/tauv_vision_amd.h). No exceptions cross it.
#include <cstring>
#include <new>
#include <string>

#include "engine.h"

namespace tv {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace tv

using namespace tv;

#define TV_GUARD(...)                                      \
  try {                                                    \
    __VA_ARGS__                                            \
  } catch (const std::bad_alloc&) {                        \
    set_error("host allocation failed");                   \
    return TV_ENOMEM;                                      \
  } catch (const std::exception& e) {                      \
    set_error(e.what());                                   \
    return TV_EINVAL;                                      \
  } catch (...) {                                          \
    set_error("unknown C++ exception");                    \
    return TV_EINVAL;                                      \
  }

struct tv_engine {
  Engine e;
};

extern "C" {

const char* tv_last_error(void) { return g_err.c_str(); }
const char* tv_version(void) { return "tauv-vision_amd 0.1 (gfx950)"; }

int tv_model_param_count(const tv_model_desc* d, int32_t* count) {
  TV_GUARD({
    if (!d || !count) { set_error("null argument"); return TV_EINVAL; }
    Plan p;
    int rc = build_plan(*d, &p);
    if (rc) return rc;
    *count = (int32_t)p.params.size();
    return TV_OK;
  })
}

int tv_model_param_info(const tv_model_desc* d, int32_t i, char* name, int32_t cap, int64_t shape[4], int32_t* ndim) {
  TV_GUARD({
    if (!d || !name || !shape || !ndim) { set_error("null argument"); return TV_EINVAL; }
    Plan p;
    int rc = build_plan(*d, &p);
    if (rc) return rc;
    if (i < 0 || i >= (int)p.params.size()) { set_error("param index out of range"); return TV_EINVAL; }
    const ParamInfo& pi = p.params[i];
    if ((int)pi.name.size() + 1 > cap) { set_error("name buffer too small"); return TV_EINVAL; }
    std::memcpy(name, pi.name.c_str(), pi.name.size() + 1);
    *ndim = (int32_t)pi.shape.size();
    for (size_t k = 0; k < 4; ++k) shape[k] = k < pi.shape.size() ? pi.shape[k] : 0;
    return TV_OK;
  })
}

int tv_model_geometry(const tv_model_desc* d, double* flops, int32_t* oh, int32_t* ow, int32_t* oc, int32_t* ocp) {
  TV_GUARD({
    if (!d) { set_error("null argument"); return TV_EINVAL; }
    Plan p;
    int rc = build_plan(*d, &p);
    if (rc) return rc;
    if (flops) *flops = p.flops_per_frame;
    if (oh) *oh = p.out_h;
    if (ow) *ow = p.out_w;
    if (oc) *oc = p.out_c;
    if (ocp) *ocp = p.out_cpad;
    return TV_OK;
  })
}

int tv_engine_create(const tv_model_desc* d, const tv_weight_view* w, int32_t n, int32_t device, tv_engine** out) {
  TV_GUARD({
    if (!d || !out || (n && !w)) { set_error("null argument"); return TV_EINVAL; }
    tv_engine* e = new tv_engine();
    int rc = e->e.create(*d, w, n, device);
    if (rc) {
      delete e;
      return rc;
    }
    *out = e;
    return TV_OK;
  })
}

int tv_engine_create_diag(const tv_model_desc* d, const tv_weight_view* w, int32_t n, int32_t device,
                          const char* knobs, tv_engine** out) {
  TV_GUARD({
    if (!d || !out || (n && !w)) { set_error("null argument"); return TV_EINVAL; }
    std::vector<std::pair<std::string, std::string>> kv;
    for (const char* c = knobs ? knobs : ""; *c;) {
      const char* e = c;
      while (*e && *e != ';') ++e;
      std::string item(c, e);
      c = *e ? e + 1 : e;
      if (item.empty()) continue;
      const size_t eq = item.find('=');
      if (eq == std::string::npos) { set_error("engine knob without '=': " + item); return TV_EINVAL; }
      kv.emplace_back(item.substr(0, eq), item.substr(eq + 1));
    }
    tv_engine* e = new tv_engine();
    int rc = e->e.create(*d, w, n, device, kv);
    if (rc) {
      delete e;
      return rc;
    }
    *out = e;
    return TV_OK;
  })
}

int tv_engine_destroy(tv_engine* e) {
  TV_GUARD({
    delete e;
    return TV_OK;
  })
}

int tv_engine_prepare(tv_engine* e, int32_t B, void* stream) {
  TV_GUARD({
    if (!e || B < 1) { set_error("bad argument"); return TV_EINVAL; }
    return e->e.prepare(B, (hipStream_t)stream);
  })
}

int tv_engine_trim(tv_engine* e) {
  TV_GUARD({
    if (!e) { set_error("null engine"); return TV_EINVAL; }
    return e->e.trim();
  })
}

int tv_engine_forward(tv_engine* e, const float* img, int32_t B, float* out, void* stream) {
  TV_GUARD({
    if (!e) { set_error("null engine"); return TV_EINVAL; }
    return e->e.forward(img, 0, B, out, (hipStream_t)stream);
  })
}

int tv_engine_forward_u8(tv_engine* e, const uint8_t* frames, int32_t B, float* out, void* stream) {
  TV_GUARD({
    if (!e) { set_error("null engine"); return TV_EINVAL; }
    return e->e.forward(frames, 1, B, out, (hipStream_t)stream);
  })
}

int tv_engine_profile(tv_engine* e, const float* img, int32_t B, float* out, void* stream, float* ms, double* flops,
                      int32_t cap, int32_t* n_ops) {
  TV_GUARD({
    if (!e || !ms || !flops || !n_ops) { set_error("null argument"); return TV_EINVAL; }
    int n = 0;
    int rc = e->e.profile(img, 0, B, out, (hipStream_t)stream, ms, flops, cap, &n);
    *n_ops = n;
    return rc;
  })
}

int tv_engine_profile_u8(tv_engine* e, const uint8_t* frames, int32_t B, float* out, void* stream, float* ms,
                         double* flops, int32_t cap, int32_t* n_ops) {
  TV_GUARD({
    if (!e || !ms || !flops || !n_ops) { set_error("null argument"); return TV_EINVAL; }
    int n = 0;
    int rc = e->e.profile(frames, 1, B, out, (hipStream_t)stream, ms, flops, cap, &n);
    *n_ops = n;
    return rc;
  })
}

int tv_engine_set_insitu(tv_engine* e, int32_t on) {
  TV_GUARD({
    if (!e) { set_error("null engine"); return TV_EINVAL; }
    e->e.insitu = on ? 1 : 0;
    return TV_OK;
  })
}

int tv_engine_insitu_read(tv_engine* e, int32_t B, void* stream, float* ms, int32_t cap, int32_t* n_slices) {
  TV_GUARD({
    if (!e || !ms || !n_slices || cap < 1 || B < 1) { set_error("bad argument"); return TV_EINVAL; }
    int n = 0;
    int rc = e->e.insitu_read(B, (hipStream_t)stream, ms, cap, &n);
    *n_slices = n;
    return rc;
  })
}

int tv_engine_forward_insitu(tv_engine* e, const float* img, int32_t B, float* out, void* stream, float* ms,
                             int32_t cap, int32_t* n_slices) {
  TV_GUARD({
    if (!e || !img || !out || !ms || !n_slices || cap < 1) { set_error("null argument"); return TV_EINVAL; }
    int n = 0;
    int rc = e->e.forward_insitu(img, 0, B, out, (hipStream_t)stream, ms, cap, &n);
    *n_slices = n;
    return rc;
  })
}

int tv_engine_forward_insitu_u8(tv_engine* e, const uint8_t* frames, int32_t B, float* out, void* stream, float* ms,
                                int32_t cap, int32_t* n_slices) {
  TV_GUARD({
    if (!e || !frames || !out || !ms || !n_slices || cap < 1) { set_error("null argument"); return TV_EINVAL; }
    int n = 0;
    int rc = e->e.forward_insitu(frames, 1, B, out, (hipStream_t)stream, ms, cap, &n);
    *n_slices = n;
    return rc;
  })
}

const char* tv_engine_op_label(tv_engine* e, int32_t i) {
  if (!e || i < 0 || i >= (int)e->e.plan.ops.size()) return "";
  return e->e.plan.ops[i].label.c_str();
}

int tv_engine_slices(tv_engine* e, int32_t B, int32_t* n, int32_t sb[TV_MAX_SLICES]) {
  TV_GUARD({
    if (!e || !n || !sb || B < 1) { set_error("bad argument"); return TV_EINVAL; }
    const std::vector<int> sz = e->e.slice_sizes(B);
    *n = (int32_t)sz.size();
    for (int k = 0; k < TV_MAX_SLICES; ++k) sb[k] = k < (int)sz.size() ? sz[k] : 0;
    return TV_OK;
  })
}

const char* tv_engine_op_kernel(tv_engine* e, int32_t B, int32_t i) {
  if (!e || i < 0 || i >= (int)e->e.plan.ops.size()) return "";
  return e->e.op_kernel(B, i);
}

int tv_preprocess_u8(const uint8_t* frames, int32_t B, int32_t src_h, int32_t src_w, int32_t dst_h, int32_t dst_w,
                     float* img_nchw, void* stream) {
  TV_GUARD({
    if (!frames || !img_nchw) { set_error("null argument"); return TV_EINVAL; }
    return launch_preprocess_u8(frames, B, src_h, src_w, dst_h, dst_w, img_nchw, (hipStream_t)stream);
  })
}

int tv_heatmap_nms(const float* heat, const int64_t st[4], int32_t B, int32_t C, int32_t H, int32_t W, int32_t k,
                   int32_t apply_sigmoid, float* out, void* stream) {
  TV_GUARD({
    if (k < 1 || k % 2 == 0) { set_error("kernel_size must be odd and >= 1"); return TV_EINVAL; }
    if (!heat || !st || !out || B < 0 || C < 0 || H < 0 || W < 0) { set_error("bad argument"); return TV_EINVAL; }
    return launch_peaks(heat, st, B, C, H, W, k, apply_sigmoid, out, (hipStream_t)stream);
  })
}

int tv_heatmap_topk(const float* peaks, int32_t B, int64_t n, int32_t K, float* score, int32_t* index, void* stream) {
  TV_GUARD({
    if (!peaks || !score || !index || B < 1) { set_error("bad argument"); return TV_EINVAL; }
    return launch_topk(peaks, B, n, K, score, index, (hipStream_t)stream);
  })
}

int tv_index_split(const int32_t* flat, int32_t B, int32_t K, int32_t H, int32_t W, int64_t* index, int64_t* label,
                   void* stream) {
  TV_GUARD({
    if (!flat || !index || !label || B < 0 || K < 0 || H < 1 || W < 1) { set_error("bad argument"); return TV_EINVAL; }
    return launch_index_split(flat, B, K, H, W, index, label, (hipStream_t)stream);
  })
}

int tv_yolact_box_decode(const float* enc, const float* anchor, int32_t B, int32_t A, int32_t anchor_batch, float v0,
                         float v1, float* box, void* stream) {
  TV_GUARD({
    if (!enc || !anchor || !box) { set_error("bad argument"); return TV_EINVAL; }
    return launch_yolact_box_decode(enc, anchor, B, A, anchor_batch, v0, v1, box, (hipStream_t)stream);
  })
}

int tv_yolact_box_encode(const float* box, const float* anchor, int32_t B, int32_t A, int32_t anchor_batch, float v0,
                         float v1, float* enc, void* stream) {
  TV_GUARD({
    if (!enc || !anchor || !box) { set_error("bad argument"); return TV_EINVAL; }
    return launch_yolact_box_encode(box, anchor, B, A, anchor_batch, v0, v1, enc, (hipStream_t)stream);
  })
}

int tv_yolact_nms_workspace_size(int32_t B, int32_t A, int32_t top_k, int64_t* bytes) {
  TV_GUARD({
    if (!bytes || B < 1 || A < 1 || top_k < 1) { set_error("bad argument"); return TV_EINVAL; }
    const size_t n = yolact_nms_workspace_bytes(B, A, top_k);
    if (!n) return TV_EHIP;
    *bytes = (int64_t)n;
    return TV_OK;
  })
}

int tv_yolact_fast_nms_batched(const float* cls, int32_t B, int32_t A, int32_t C1, const float* box, int32_t top_k,
                               float iou_thr, float conf_thr, int64_t* det, int32_t* n_det, void* ws, int64_t ws_bytes,
                               void* stream) {
  TV_GUARD({
    if (!cls || !box || !det || !n_det || !ws || ws_bytes < 0) { set_error("bad argument"); return TV_EINVAL; }
    const int K = top_k < A ? top_k : A;
    return launch_yolact_fast_nms(cls, (long long)A * C1, A, C1, box, (long long)A * 4, B, top_k, iou_thr, conf_thr,
                                  ws, (size_t)ws_bytes, (long long*)det, K, n_det, (hipStream_t)stream);
  })
}

int tv_yolact_fast_nms(const float* cls, int32_t A, int32_t C1, const float* box, int32_t top_k, float iou_thr,
                       float conf_thr, int64_t* det, int32_t* n_det, void* stream) {
  TV_GUARD({
    if (!cls || !box || !det || !n_det || A < 1 || top_k < 1) { set_error("bad argument"); return TV_EINVAL; }
    hipStream_t s = (hipStream_t)stream;
    const size_t need = yolact_nms_workspace_bytes(1, A, top_k);
    if (!need) return TV_EHIP;
    void* ws = nullptr;
    TV_HIP(hipMallocAsync(&ws, need, s));
    const int K = top_k < A ? top_k : A;
    int rc = launch_yolact_fast_nms(cls, (long long)A * C1, A, C1, box, (long long)A * 4, 1, top_k, iou_thr, conf_thr,
                                    ws, need, (long long*)det, K, n_det, s);
    TV_HIP(hipFreeAsync(ws, s));
    return rc;
  })
}

int tv_yolact_assemble_mask(const float* proto, const int64_t pst[3], int32_t K, int32_t H, int32_t W,
                            const float* coeff, const float* box, int32_t n, float* mask, void* stream) {
  TV_GUARD({
    if (n == 0) return TV_OK;
    if (!proto || !pst || !coeff || !mask || n < 0) { set_error("bad argument"); return TV_EINVAL; }
    const long long st[4] = {0, pst[0], pst[1], pst[2]};
    return launch_yolact_assemble_mask(proto, st, 1, K, H, W, coeff, box, nullptr, nullptr, 0, n, mask,
                                       (hipStream_t)stream);
  })
}

int tv_yolact_assemble_masks(const float* proto, const int64_t pst[4], int32_t B, int32_t K, int32_t H, int32_t W,
                             const float* coeff, const float* box, const int32_t* counts, int32_t n_max, float* mask,
                             void* stream) {
  TV_GUARD({
    if (n_max == 0) return TV_OK;
    if (!proto || !pst || !coeff || !mask || n_max < 0) { set_error("bad argument"); return TV_EINVAL; }
    const long long st[4] = {pst[0], pst[1], pst[2], pst[3]};
    return launch_yolact_assemble_mask(proto, st, B, K, H, W, coeff, box, counts, nullptr, 0, n_max, mask,
                                       (hipStream_t)stream);
  })
}

int tv_yolact_assemble_masks_indexed(const float* proto, const int64_t pst[4], int32_t B, int32_t K, int32_t H,
                                     int32_t W, const float* coeff, const float* box, int32_t A, const int64_t* det,
                                     const int32_t* counts, int32_t n_max, float* mask, void* stream) {
  TV_GUARD({
    if (n_max == 0) return TV_OK;
    if (!proto || !pst || !coeff || !det || !counts || !mask || n_max < 0 || A < 1) {
      set_error("bad argument");
      return TV_EINVAL;
    }
    const long long st[4] = {pst[0], pst[1], pst[2], pst[3]};
    return launch_yolact_assemble_mask(proto, st, B, K, H, W, coeff, box, counts, (const long long*)det, A, n_max,
                                       mask, (hipStream_t)stream);
  })
}

int tv_decode_workspace_size(int32_t B, int32_t C, int32_t H, int32_t W, int32_t K, int64_t* bytes) {
  if (!bytes || B < 1 || C < 1 || H < 1 || W < 1 || K < 1) { set_error("bad argument"); return TV_EINVAL; }
  *bytes = (int64_t)decode_workspace_bytes(B, C, H, W, K);
  return TV_OK;
}

int tv_decode(const float* heat, const int64_t hs[4], const float* size, const int64_t ss[4], const float* offset,
              const int64_t os[4], const float* depth, const int64_t ds[4], int32_t B, int32_t C, int32_t H, int32_t W,
              int32_t K, int32_t mode, int32_t ratio, int32_t in_h, int32_t in_w, float thr, const float* aux,
              const int64_t aux_st[5], float* records, int32_t* counts, void* ws, int64_t ws_bytes, void* stream) {
  TV_GUARD({
    int64_t need = 0;
    int rc = tv_decode_workspace_size(B, C, H, W, K, &need);
    if (rc) return rc;
    if (!heat || !hs || !size || !ss || !records || !counts || !ws || ws_bytes < need) {
      set_error("bad argument or workspace too small");
      return TV_EINVAL;
    }
    if (mode == 0 && (!offset || !os)) { set_error("decode needs the offset head"); return TV_EINVAL; }
    if (depth && !ds) { set_error("depth strides missing"); return TV_EINVAL; }
    hipStream_t s = (hipStream_t)stream;
    DecodeParams p{};
    p.B = B; p.K = K; p.C = C; p.H = H; p.W = W;
    p.size = size;
    p.offset = offset;
    p.depth = depth;
    for (int i = 0; i < 4; ++i) {
      p.size_st[i] = ss[i];
      p.offset_st[i] = offset ? os[i] : 0;
      p.depth_st[i] = depth ? ds[i] : 0;
    }
    p.depth_mode = mode == 0 ? 0 : 1;
    p.pos_mode = mode == 0 ? 0 : 1;
    p.ratio = ratio; p.in_h = in_h; p.in_w = in_w;
    p.out_h = ratio > 0 ? in_h / ratio : H;
    p.out_w = ratio > 0 ? in_w / ratio : W;
    p.score_thr = thr;
    p.aux = aux;
    if (aux) {
      if (!aux_st) { set_error("aux strides missing"); return TV_EINVAL; }
      for (int i = 0; i < 5; ++i) p.aux_st[i] = aux_st[i];
    }
    p.records = records;
    p.counts = counts;
    return launch_decode(heat, hs, B, C, H, W, K, ws, (size_t)ws_bytes, p, s);
  })
}

int tv_diag_dcn_conv(const void* x, const void* om, int32_t B, int32_t H, int32_t W, int32_t C, int32_t om_ldc,
                     const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, int32_t variant,
                     void* out, void* stream) {
  TV_GUARD({ return tv::diag_dcn_conv(x, om, B, H, W, C, om_ldc, weight, bias, N, act, dtype, variant, out,
                                      (hipStream_t)stream); })
}

int tv_diag_conv1x1(const void* const* src, const int32_t* C, const int32_t* ldc, int32_t nseg, int32_t M,
                    const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, void* out,
                    int32_t out_ldc, void* stream) {
  TV_GUARD({ return tv::diag_conv1x1(src, C, ldc, nseg, M, weight, bias, N, act, dtype, out, out_ldc,
                                     (hipStream_t)stream); })
}

int tv_diag_conv_burst(const void* const* src, const int32_t* geom, int32_t nseg, int32_t B, int32_t Ho, int32_t Wo,
                       const float* weight, const float* bias, int32_t N, int32_t act, int32_t dtype, void* out,
                       int32_t out_ldc, void* stream) {
  TV_GUARD({ return tv::diag_conv_burst(src, geom, nseg, B, Ho, Wo, weight, bias, N, act, dtype, out, out_ldc,
                                        (hipStream_t)stream); })
}

int tv_diag_burst_plan(const int32_t* geom, int32_t nseg, int32_t B, int32_t Ho, int32_t Wo, int32_t N, int32_t* out) {
  TV_GUARD({ return tv::diag_burst_plan(geom, nseg, B, Ho, Wo, N, out); })
}

int tv_diag_conv_small(const void* src, int32_t B, int32_t H, int32_t W, int32_t C, int32_t ldc, const float* weight,
                       const float* bias, int32_t N, int32_t stride, int32_t act, int32_t dtype, int32_t variant,
                       void* out, int32_t out_ldc, void* stream) {
  TV_GUARD({ return tv::diag_conv_small(src, B, H, W, C, ldc, weight, bias, N, stride, act, dtype, variant, out,
                                        out_ldc, (hipStream_t)stream); })
}

int tv_diag_convt3(const void* src, int32_t B, int32_t H, int32_t W, int32_t C, int32_t ldc, const float* weight,
                   const float* bias, int32_t N, int32_t act, int32_t dtype, int32_t tile_w, int32_t tile_h, void* out,
                   int32_t out_ldc, void* stream) {
  TV_GUARD({ return tv::diag_convt3(src, B, H, W, C, ldc, weight, bias, N, act, dtype, tile_w, tile_h, out, out_ldc,
                                    (hipStream_t)stream); })
}

int tv_train_heatmap(const uint8_t* valid, const int64_t* label, const float* center, int32_t B, int32_t n_objects,
                     int32_t n_labels, int32_t in_h, int32_t in_w, int32_t downsample_ratio, double sigma,
                     float* heatmap, void* stream) {
  TV_GUARD({
    return tv::launch_train_heatmap(valid, reinterpret_cast<const long long*>(label), center, B, n_objects, n_labels,
                                    in_h, in_w, downsample_ratio, sigma, heatmap, (hipStream_t)stream);
  })
}

int tv_train_keypoint_targets(const uint8_t* keypoint_valid, const int64_t* keypoint_label,
                              const float* keypoint_center, const int64_t* keypoint_object_index, const float* center,
                              int32_t B, int32_t n_instances, int32_t n_objects, int32_t n_keypoints, int32_t in_h,
                              int32_t in_w, int32_t downsample_ratio, double heatmap_sigma, double affinity_sigma,
                              float* heatmap, float* affinity_weight, float* affinity, void* stream) {
  TV_GUARD({
    return tv::launch_train_keypoints(keypoint_valid, reinterpret_cast<const long long*>(keypoint_label),
                                      keypoint_center, reinterpret_cast<const long long*>(keypoint_object_index),
                                      center, B, n_instances, n_objects, n_keypoints, in_h, in_w, downsample_ratio,
                                      heatmap_sigma, affinity_sigma, heatmap, affinity_weight, affinity,
                                      (hipStream_t)stream);
  })
}

}  // extern "C"
