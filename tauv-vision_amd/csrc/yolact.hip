// YOLACT post-processing on gfx950 (reference src/tauv_vision/yolact/model/):
//   box_decode     boxes.py:55-61   c = a_c + e_c * v0 * a_hw, hw = a_hw * exp(e_hw * v1)
//   fast_nms       nms.py:7-29      softmax -> max non-background confidence -> descending sort ->
//                                   top_k -> upper-triangular IoU (boxes.py:64-85) -> column max ->
//                                   keep (iou_max <= thr) & (conf >= cthr); batch 0 only (:14, 25)
//   assemble_mask  masks.py:8-21    sigmoid(sum_k c_k P_k) x inclusive box mask (boxes.py:88-103)
// All fp32 (the reference runs them in fp32), expression order as in the reference.
// fast_nms is one workgroup: the whole problem (<= 16384 anchors, top_k <= 1024) lives in LDS —
// a bitonic sort of (confidence, anchor) keys, then one thread per kept column j scans i < j.
#include "common.h"

// the reference rounds every product before the sum (separate torch ops): no FMA contraction
#pragma clang fp contract(off)

namespace tv {
namespace yolact {

__global__ __launch_bounds__(256) void box_decode(const float* __restrict__ enc, const float* __restrict__ anchor,
                                                  int B, int A, int anchor_batch, float v0, float v1,
                                                  float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)B * A) return;
  const unsigned b = i / (unsigned)A, a = i % (unsigned)A;
  const float4 e = reinterpret_cast<const float4*>(enc)[i];
  const float4 an = reinterpret_cast<const float4*>(anchor)[(anchor_batch == 1 ? 0 : b) * (unsigned)A + a];
  float4 o;
  // torch: anchor[..., :2] + enc[..., :2] * v0 * anchor[..., 2:]  (left to right)
  o.x = an.x + e.x * v0 * an.z;
  o.y = an.y + e.y * v0 * an.w;
  o.z = an.z * expf(e.z * v1);
  o.w = an.w * expf(e.w * v1);
  reinterpret_cast<float4*>(out)[i] = o;
}

constexpr int kNmsThreads = 1024;
constexpr int kNmsMaxAnchors = 16384;

// keys: confidence bits (non-negative floats order like their bit patterns) in the high word,
// ~anchor in the low word, so the descending sort breaks exact ties toward the smaller anchor
__global__ __launch_bounds__(kNmsThreads) void fast_nms(const float* __restrict__ cls, int A, int C1,
                                                        const float* __restrict__ box, int top_k, float iou_thr,
                                                        float conf_thr, long long* __restrict__ det,
                                                        int* __restrict__ n_det) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];  // [P] (P = pow2 >= A)
  const int tid = threadIdx.x;
  int P = 1;
  while (P < A) P <<= 1;
  for (int a = tid; a < P; a += kNmsThreads) {
    unsigned long long key = 0;  // padding sorts last
    if (a < A) {
      const float* c = cls + (size_t)a * C1;
      float m = c[0];
      for (int j = 1; j < C1; ++j) m = fmaxf(m, c[j]);
      float s = 0.f;
      for (int j = 0; j < C1; ++j) s += expf(c[j] - m);
      float best = 0.f;
      for (int j = 1; j < C1; ++j) best = fmaxf(best, expf(c[j] - m) / s);
      key = ((unsigned long long)__float_as_uint(best) << 32) | (unsigned)(~(unsigned)a);
    }
    keys[a] = key;
  }
  __syncthreads();
  // bitonic sort, descending
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += kNmsThreads) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = keys[i], b = keys[l];
          const bool desc = (i & k) == 0;
          if (desc ? a < b : a > b) {
            keys[i] = b;
            keys[l] = a;
          }
        }
      }
      __syncthreads();
    }
  const int K = min(top_k, A);
  // column j survives if no higher-confidence box i < j overlaps it by more than iou_thr
  for (int j = tid; j < K; j += kNmsThreads) {
    const unsigned aj = ~(unsigned)(keys[j] & 0xffffffffu);
    const float conf = __uint_as_float((unsigned)(keys[j] >> 32));
    const float4 bj = reinterpret_cast<const float4*>(box)[aj];
    // corners (boxes.py:14-26) and area (:79-80) exactly as the reference forms them
    const float jy0 = bj.x - bj.z / 2, jx0 = bj.y - bj.w / 2, jy1 = bj.x + bj.z / 2, jx1 = bj.y + bj.w / 2;
    const float area_j = bj.z * bj.w;
    float iou_max = 0.f;  // torch.triu zeroes i >= j; the max includes those zeros
    for (int i = 0; i < j; ++i) {
      const unsigned ai = ~(unsigned)(keys[i] & 0xffffffffu);
      const float4 bi = reinterpret_cast<const float4*>(box)[ai];
      const float iy0 = bi.x - bi.z / 2, ix0 = bi.y - bi.w / 2, iy1 = bi.x + bi.z / 2, ix1 = bi.y + bi.w / 2;
      const float ih = fmaxf(fminf(iy1, jy1) - fmaxf(iy0, jy0), 0.f);
      const float iw = fmaxf(fminf(ix1, jx1) - fmaxf(ix0, jx0), 0.f);
      const float inter = ih * iw;
      const float uni = (bi.z * bi.w + area_j) - inter;
      iou_max = fmaxf(iou_max, inter / uni);
    }
    const bool keep = iou_max <= iou_thr && conf >= conf_thr;
    // order-preserving compaction: write a flag, compact after the barrier
    reinterpret_cast<int*>(keys + P)[j] = keep ? 1 : 0;
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    const int* flag = reinterpret_cast<const int*>(keys + P);
    for (int j = 0; j < K; ++j)
      if (flag[j]) det[n++] = (long long)(~(unsigned)(keys[j] & 0xffffffffu));
    *n_det = n;
  }
}

// out[n][y][x] = sigmoid(sum_k coeff[n][k] * proto[k][y][x]) * box_mask(n, y, x)
__global__ __launch_bounds__(256) void assemble_mask(const float* __restrict__ proto, int K, int H, int W,
                                                     const float* __restrict__ coeff, const float* __restrict__ box,
                                                     int n, float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned hw = (unsigned)H * W;
  if (i >= (unsigned)n * hw) return;
  const unsigned d = i / hw, pix = i % hw;
  const unsigned y = pix / (unsigned)W, x = pix % (unsigned)W;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += coeff[(size_t)d * K + k] * proto[(size_t)k * hw + pix];
  float m = 1.f / (1.f + expf(-s));
  if (box) {
    const float* b = box + (size_t)d * 4;
    const float by = b[0] * (float)H, bx = b[1] * (float)W, bh = b[2] * (float)H, bw = b[3] * (float)W;
    const float left = bx - bw / 2, right = bx + bw / 2, top = by - bh / 2, bottom = by + bh / 2;
    const float fx = (float)x, fy = (float)y;
    m *= (fx >= left && fx <= right && fy >= top && fy <= bottom) ? 1.f : 0.f;
  }
  out[i] = m;
}

}  // namespace yolact

int launch_yolact_box_decode(const float* enc, const float* anchor, int B, int A, int anchor_batch, float v0, float v1,
                             float* out, hipStream_t s) {
  if (B < 1 || A < 1 || (anchor_batch != 1 && anchor_batch != B) || (long)B * A >= (1L << 31)) {
    set_error("box_decode: bad shapes (anchor batch must be 1 or B)");
    return 2;  // TV_ESHAPE
  }
  const unsigned n = (unsigned)B * A;
  hipLaunchKernelGGL(yolact::box_decode, dim3((n + 255) / 256), dim3(256), 0, s, enc, anchor, B, A, anchor_batch, v0,
                     v1, out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_yolact_fast_nms(const float* cls, int A, int C1, const float* box, int top_k, float iou_thr, float conf_thr,
                           long long* det, int* n_det, hipStream_t s) {
  if (A < 1 || A > yolact::kNmsMaxAnchors / 2 || C1 < 2 || top_k < 1) {
    set_error("fast_nms: need 1 <= anchors <= 8192, >= 2 classes (incl. background), top_k >= 1");
    return 2;  // TV_ESHAPE
  }
  int P = 1;
  while (P < A) P <<= 1;
  const size_t lds = (size_t)P * 8 + (size_t)std::min(top_k, A) * 4 + 16;
  static bool attr = false;
  if (!attr) {
    TV_HIP(hipFuncSetAttribute((const void*)yolact::fast_nms, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(yolact::fast_nms, dim3(1), dim3(yolact::kNmsThreads), lds, s, cls, A, C1, box, top_k, iou_thr,
                     conf_thr, det, n_det);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_yolact_assemble_mask(const float* proto, int K, int H, int W, const float* coeff, const float* box, int n,
                                float* out, hipStream_t s) {
  if (K < 1 || H < 1 || W < 1 || n < 0 || (long)n * H * W >= (1L << 31)) {
    set_error("assemble_mask: bad shapes");
    return 2;  // TV_ESHAPE
  }
  if (n == 0) return 0;
  const unsigned t = (unsigned)n * H * W;
  hipLaunchKernelGGL(yolact::assemble_mask, dim3((t + 255) / 256), dim3(256), 0, s, proto, K, H, W, coeff, box, n,
                     out);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
