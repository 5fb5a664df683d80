// YOLACT post-processing on gfx950 (reference src/tauv_vision/yolact/model/):
//   box_decode     boxes.py:55-61   c = a_c + e_c * v0 * a_hw, hw = a_hw * exp(e_hw * v1)
//   box_encode     boxes.py:45-53   e_c = (b_c - a_c) / (v0 * a_hw), e_hw = log(b_hw / a_hw) / v1
//   fast_nms       nms.py:7-29      softmax -> max non-background confidence -> descending sort ->
//                                   top_k -> upper-triangular IoU (boxes.py:64-85) -> column max ->
//                                   keep (iou_max <= thr) & (conf >= cthr)
//   assemble_mask  masks.py:8-21    sigmoid(sum_k c_k P_k) x inclusive box mask (boxes.py:88-103)
// All fp32 (the reference runs them in fp32), expression order as in the reference.
//
// fast_nms, any anchor count, B images per launch (the reference runs image 0 only: :14,25):
//   nms_keys    one thread per anchor: the confidence as an order-preserving 32-bit key;
//   nms_topk    one 1024-thread workgroup per image (top_k <= 1024, anchors <= 32768): the
//               anchors' 64-bit keys (confidence key << 32 | ~anchor: unique, descending order
//               = the reference's stable descending sort, equal confidences in ascending anchor
//               order) in registers, the K-th largest found by 8 radix passes of 8-bit digits
//               over LDS histograms, the K keys >= it compacted into LDS and bitonic-sorted;
//   nms_sort    larger top_k / anchor counts (up to the full sort): one workgroup per image
//               streams the keys from L2 instead of holding them, and sorts the top K in rank
//               ranges of <= 16384 keys (each range's lower bound = one more radix select,
//               its keys compacted into LDS and bitonic-sorted): the same order, no library;
//   nms_iou     one thread per kept column j < min(top_k, A); rows i < j staged through LDS in
//               256-box chunks; the column max propagates NaN like torch.max (0/0 IoUs of two
//               zero-area boxes drop the column: NaN <= thr is false);
//   nms_compact one workgroup per image: order-preserving compaction of the kept columns.
// assemble_mask: one workgroup per 1024 pixels of one image; the block's prototypes (any
// strides: NCHW or the protonet's NHWC output) are staged in LDS as [k][pixel] and the
// detections' coefficient rows and box bounds in chunks of 64 (gathered through the NMS output
// when given), each thread forms 4 adjacent pixels of every detection and stores them as one
// 16-byte vector (the kernel is HBM-write-bound: n x H x W x 4 bytes per image).
#include "common.h"

#include <cstring>
#include <mutex>

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

__global__ __launch_bounds__(256) void box_encode(const float* __restrict__ box, const float* __restrict__ anchor,
                                                  int B, int A, int anchor_batch, float v0, float v1,
                                                  float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)B * A) return;
  const unsigned b = i / (unsigned)A, a = i % (unsigned)A;
  const float4 g = reinterpret_cast<const float4*>(box)[i];
  const float4 an = reinterpret_cast<const float4*>(anchor)[(anchor_batch == 1 ? 0 : b) * (unsigned)A + a];
  float4 o;
  // g_cxcy = box[:2] - anchor[:2]; g_cxcy /= (v0 * anchor[2:]); g_wh = log(box[2:] / anchor[2:]) / v1
  o.x = (g.x - an.x) / (v0 * an.z);
  o.y = (g.y - an.y) / (v0 * an.w);
  o.z = logf(g.z / an.z) / v1;
  o.w = logf(g.w / an.w) / v1;
  reinterpret_cast<float4*>(out)[i] = o;
}

__device__ __forceinline__ uint32_t order_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unorder_bits(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// max over classes 1.. of softmax(cls row) (nms.py:10-11)
__global__ __launch_bounds__(256) void nms_keys(const float* __restrict__ cls, long long cls_bstride, int A, int C1,
                                                int B, uint32_t* __restrict__ keys) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)B * A) return;
  const unsigned b = i / (unsigned)A, a = i % (unsigned)A;
  const float* c = cls + (size_t)b * cls_bstride + (size_t)a * C1;
  float m = c[0];
  for (int j = 1; j < C1; ++j) m = fmaxf(m, c[j]);
  float s = 0.f;
  for (int j = 0; j < C1; ++j) s += expf(c[j] - m);
  float best = 0.f;
  for (int j = 1; j < C1; ++j) {
    const float v = expf(c[j] - m) / s;
    best = (v > best || v != v) ? v : best;  // torch.max propagates a NaN softmax (NaN logits)
  }
  // a NaN confidence sorts first (torch.sort, descending) and fails conf >= thr, like the reference
  keys[i] = order_bits(best);
}

constexpr int kIouThreads = 256;

// keep[b][j] for the K highest-confidence anchors of image b (sorted order)
__global__ __launch_bounds__(kIouThreads) void nms_iou(const float* __restrict__ box, long long box_bstride, int A,
                                                       int K, const uint32_t* __restrict__ skeys,
                                                       const int* __restrict__ sidx, float iou_thr, float conf_thr,
                                                       uint8_t* __restrict__ keep) {
  __shared__ float4 corner[kIouThreads];  // y0, x0, y1, x1 of the staged rows
  __shared__ float area[kIouThreads];
  const int b = blockIdx.y;
  const int j = blockIdx.x * kIouThreads + threadIdx.x;
  const size_t seg = (size_t)b * A;
  const float4* bx = reinterpret_cast<const float4*>(box + (size_t)b * box_bstride);
  float jy0 = 0, jx0 = 0, jy1 = 0, jx1 = 0, area_j = 0, conf = 0;
  if (j < K) {
    const float4 bj = bx[sidx[seg + j] - (int)seg];
    // corners (boxes.py:14-26) and area (:79-80) exactly as the reference forms them
    jy0 = bj.x - bj.z / 2; jx0 = bj.y - bj.w / 2; jy1 = bj.x + bj.z / 2; jx1 = bj.y + bj.w / 2;
    area_j = bj.z * bj.w;
    conf = unorder_bits(skeys[seg + j]);
  }
  float iou_max = 0.f;  // torch.triu zeroes i >= j; the max includes those zeros
  const int jmax = min(K, (int)(blockIdx.x + 1) * kIouThreads);  // rows needed by this block: i < jmax - 1
  for (int i0 = 0; i0 < jmax - 1; i0 += kIouThreads) {
    __syncthreads();
    const int ii = i0 + threadIdx.x;
    if (ii < K) {
      const float4 bi = bx[sidx[seg + ii] - (int)seg];
      corner[threadIdx.x] = make_float4(bi.x - bi.z / 2, bi.y - bi.w / 2, bi.x + bi.z / 2, bi.y + bi.w / 2);
      area[threadIdx.x] = bi.z * bi.w;
    }
    __syncthreads();
    const int n = min(kIouThreads, j - i0);  // rows i0 .. j-1 of this chunk
    for (int t = 0; t < n; ++t) {
      const float4 ci = corner[t];
      const float ih = fmaxf(fminf(ci.z, jy1) - fmaxf(ci.x, jy0), 0.f);
      const float iw = fmaxf(fminf(ci.w, jx1) - fmaxf(ci.y, jx0), 0.f);
      const float inter = ih * iw;
      const float v = inter / ((area[t] + area_j) - inter);
      iou_max = (v > iou_max || v != v) ? v : iou_max;  // NaN sticks (torch.max propagates it)
    }
  }
  if (j < K) keep[(size_t)b * K + j] = (iou_max <= iou_thr && conf >= conf_thr) ? 1 : 0;
}

constexpr int kCompactThreads = 1024;

__global__ __launch_bounds__(kCompactThreads) void nms_compact(const uint8_t* __restrict__ keep, int A, int K,
                                                               const int* __restrict__ sidx, long long* __restrict__ det,
                                                               int det_stride, int* __restrict__ n_det) {
  __shared__ int wsum[kCompactThreads / 64];
  __shared__ int base;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) base = 0;
  for (int j0 = 0; j0 < K; j0 += kCompactThreads) {
    const int j = j0 + tid;
    const int f = j < K ? keep[(size_t)b * K + j] : 0;
    const unsigned long long m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();  // `base` of the previous chunk is final
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    if (f) det[(size_t)b * det_stride + off + before] = (long long)(sidx[(size_t)b * A + j] - b * A);
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < kCompactThreads / 64; ++w) t += wsum[w];
      base += t;
    }
  }
  __syncthreads();
  if (tid == 0) n_det[b] = base;
}

// ---- exact per-image top-K of the NMS keys (nms_topk) ---------------------------------------
constexpr int kTopkThreads = 1024;
constexpr int kTopkMaxK = 1024;
template <int PER>  // keys per thread: A <= PER * 1024
__global__ __launch_bounds__(kTopkThreads) void nms_topk(const uint32_t* __restrict__ keys, int A, int K,
                                                         uint32_t* __restrict__ skeys, int* __restrict__ sidx) {
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sel[kTopkMaxK];
  __shared__ unsigned s_digit, s_above, s_n;
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t seg = (size_t)b * A;
  unsigned long long k[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int a = tid + j * kTopkThreads;
    // key 0 never occurs for a real anchor: its low word ~a is nonzero for a < 2^32 - 1
    k[j] = a < A ? ((unsigned long long)keys[seg + a] << 32) | (0xFFFFFFFFu - (unsigned)a) : 0ull;
  }
  // radix select of the K-th largest key, most significant digit first
  unsigned long long prefix = 0, pmask = 0;
  unsigned need = (unsigned)K;
  for (int shift = 56; shift >= 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (k[j] != 0 && (k[j] & pmask) == prefix) atomicAdd(&hist[(unsigned)(k[j] >> shift) & 255u], 1u);
    __syncthreads();
    if (tid < 64) {  // one wave: the digit whose suffix count first reaches `need`
      const unsigned h0 = hist[255 - 4 * tid], h1 = hist[254 - 4 * tid], h2 = hist[253 - 4 * tid], h3 = hist[252 - 4 * tid];
      const unsigned own = h0 + h1 + h2 + h3;
      unsigned incl = own;  // inclusive prefix over lanes (digits descending)
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d, 64);
        if (tid >= d) incl += o;
      }
      const unsigned excl = incl - own;
      if (excl < need && incl >= need) {
        unsigned above = excl;
        const unsigned hs[4] = {h0, h1, h2, h3};
        int q = 0;
        while (above + hs[q] < need) above += hs[q++];
        s_digit = 255u - 4u * (unsigned)tid - (unsigned)q;
        s_above = above;
      }
    }
    __syncthreads();
    prefix |= (unsigned long long)s_digit << shift;
    pmask |= 255ull << shift;
    need -= s_above;
    __syncthreads();
  }
  // prefix = the K-th largest key: exactly K keys are >= it (keys are unique)
  if (tid == 0) s_n = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (k[j] != 0 && k[j] >= prefix) sel[atomicAdd(&s_n, 1u)] = k[j];
  __syncthreads();
  int n2 = 1;
  while (n2 < K) n2 <<= 1;
  for (int i = K + tid; i < n2; i += kTopkThreads) sel[i] = 0;
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += kTopkThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long x = sel[i], y = sel[j];
          if (desc ? x < y : x > y) {
            sel[i] = y;
            sel[j] = x;
          }
        }
      }
      __syncthreads();
    }
  for (int r = tid; r < K; r += kTopkThreads) {
    const unsigned long long key = sel[r];
    skeys[seg + r] = (uint32_t)(key >> 32);
    sidx[seg + r] = (int)(seg + (0xFFFFFFFFu - (uint32_t)key));
  }
}

// ---- any top_k / anchor count (nms_sort) -----------------------------------------------------
constexpr int kSortThreads = 1024;
constexpr int kSortCap = 16384;  // keys per rank range (128 KiB of LDS)

// 64-bit key of anchor a (the nms_topk order); never 0
__device__ __forceinline__ unsigned long long nms_key(const uint32_t* __restrict__ keys, size_t seg, int a) {
  return ((unsigned long long)keys[seg + a] << 32) | (0xFFFFFFFFu - (unsigned)a);
}

__global__ __launch_bounds__(kSortThreads) void nms_sort(const uint32_t* __restrict__ keys, int A, int K,
                                                         uint32_t* __restrict__ skeys, int* __restrict__ sidx) {
  extern __shared__ unsigned long long sel[];  // [kSortCap]
  __shared__ unsigned hist[256];
  __shared__ unsigned s_digit, s_above, s_n;
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t seg = (size_t)b * A;
  // the rank-th largest key (1 <= rank <= A): exactly `rank` keys are >= it (keys are unique)
  auto select = [&](unsigned rank) {
    unsigned long long prefix = 0, pmask = 0;
    unsigned need = rank;
    for (int shift = 56; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
      for (int a = tid; a < A; a += kSortThreads) {
        const unsigned long long k = nms_key(keys, seg, a);
        if ((k & pmask) == prefix) atomicAdd(&hist[(unsigned)(k >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid < 64) {  // one wave: the digit whose suffix count first reaches `need` (nms_topk)
        const unsigned h0 = hist[255 - 4 * tid], h1 = hist[254 - 4 * tid], h2 = hist[253 - 4 * tid],
                       h3 = hist[252 - 4 * tid];
        const unsigned own = h0 + h1 + h2 + h3;
        unsigned incl = own;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const unsigned o = __shfl_up(incl, d, 64);
          if (tid >= d) incl += o;
        }
        const unsigned excl = incl - own;
        if (excl < need && incl >= need) {
          unsigned above = excl;
          const unsigned hs[4] = {h0, h1, h2, h3};
          int q = 0;
          while (above + hs[q] < need) above += hs[q++];
          s_digit = 255u - 4u * (unsigned)tid - (unsigned)q;
          s_above = above;
        }
      }
      __syncthreads();
      prefix |= (unsigned long long)s_digit << shift;
      pmask |= 255ull << shift;
      need -= s_above;
      __syncthreads();
    }
    return prefix;
  };
  unsigned long long hi = 0;  // the previous range's lower bound (exclusive upper bound of this one)
  for (int r0 = 0; r0 < K; r0 += kSortCap) {
    const int r1 = min(K, r0 + kSortCap), n = r1 - r0;
    const unsigned long long lo = select((unsigned)r1);
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int a = tid; a < A; a += kSortThreads) {
      const unsigned long long k = nms_key(keys, seg, a);
      if (k >= lo && (r0 == 0 || k < hi)) sel[atomicAdd(&s_n, 1u)] = k;  // exactly n keys
    }
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = n + tid; i < n2; i += kSortThreads) sel[i] = 0;  // (0: below every key)
    __syncthreads();
    for (int size = 2; size <= n2; size <<= 1)  // bitonic sort, descending
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < n2; i += kSortThreads) {
          const int j = i ^ stride;
          if (j > i) {
            const bool desc = (i & size) == 0;
            const unsigned long long x = sel[i], y = sel[j];
            if (desc ? x < y : x > y) {
              sel[i] = y;
              sel[j] = x;
            }
          }
        }
        __syncthreads();
      }
    for (int r = tid; r < n; r += kSortThreads) {
      const unsigned long long key = sel[r];
      skeys[seg + r0 + r] = (uint32_t)(key >> 32);
      sidx[seg + r0 + r] = (int)(seg + (0xFFFFFFFFu - (uint32_t)key));
    }
    hi = lo;
    __syncthreads();  // sel consumed before the next range's compaction
  }
}

// masks[b][d][y][x] = sigmoid(sum_k coeff[b][d][k] * proto[b][k][y][x]) * box_mask(b, d, y, x)
constexpr int kMaskThreads = 256;
constexpr int kMaskPix = 4 * kMaskThreads;  // pixels per workgroup (4 adjacent per thread)

struct MaskParams {
  const float* proto;
  long long ps_b, ps_k, ps_y, ps_x;  // element strides
  int K, H, W;
  const float* coeff;                // [B][n_max][K]
  const float* box;                  // [B][n_max][4] or null
  const int* counts;                 // [B] or null (= n_max)
  const long long* det;              // [B][n_max] coefficient / box row per detection, or null (= d)
  int rows;                          // coefficient / box rows per image (A when det, else n_max)
  int n_max;
  float* out;                        // [B][n_max][H][W]
};

constexpr int kMaskDets = 64;  // detections whose coefficients / box bounds are staged in LDS at once

__global__ __launch_bounds__(kMaskThreads) void assemble_mask(const MaskParams p) {
  extern __shared__ __attribute__((aligned(16))) float pr[];  // [K][kMaskPix], then the detection chunk
  float* dc = pr + p.K * kMaskPix;                             // [kMaskDets][K] coefficients
  float4* db4 = reinterpret_cast<float4*>(dc + kMaskDets * p.K);  // [kMaskDets] left, right, top, bottom
  const int b = blockIdx.y;
  const int n = p.counts ? min(p.counts[b], p.n_max) : p.n_max;
  if (n <= 0) return;
  const int hw = p.H * p.W;
  const int pix0 = blockIdx.x * kMaskPix;
  const float* pb = p.proto + (size_t)b * p.ps_b;
  // stage the block's prototypes: element (k, q) at pr[k * kMaskPix + q]; consecutive threads
  // walk the stride-1 axis (channels for NHWC views, pixels for NCHW)
  const bool chan_fast = p.ps_k < p.ps_x;
  for (int e = threadIdx.x; e < p.K * kMaskPix; e += kMaskThreads) {
    int k, q;
    if (chan_fast) { k = e % p.K; q = e / p.K; } else { q = e % kMaskPix; k = e / kMaskPix; }
    const int pix = pix0 + q;
    float v = 0.f;
    if (pix < hw) {
      const int y = pix / p.W, x = pix - y * p.W;
      v = pb[(size_t)k * p.ps_k + (size_t)y * p.ps_y + (size_t)x * p.ps_x];
    }
    pr[k * kMaskPix + q] = v;
  }
  const int q0 = 4 * threadIdx.x;
  const int pix = pix0 + q0;
  int yy[4], xx[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    yy[e] = (pix + e) / p.W;
    xx[e] = (pix + e) - yy[e] * p.W;
  }
  const bool vec = (hw & 3) == 0;  // 16-byte stores: every row of a detection starts 16-byte aligned
  const float* cb = p.coeff + (size_t)b * p.rows * p.K;
  const float* bb = p.box ? p.box + (size_t)b * p.rows * 4 : nullptr;
  const long long* db = p.det ? p.det + (size_t)b * p.n_max : nullptr;
  float* ob = p.out + (size_t)b * p.n_max * hw;
  for (int d0 = 0; d0 < n; d0 += kMaskDets) {
    const int nd = min(kMaskDets, n - d0);
    __syncthreads();  // prototypes staged / the previous chunk consumed
    // the chunk's coefficient rows (the NMS-kept anchors when det is given) and box bounds
    for (int e = threadIdx.x; e < nd * p.K; e += kMaskThreads) {
      const int d = e / p.K, k = e - d * p.K;
      const size_t row = db ? (size_t)db[d0 + d] : (size_t)(d0 + d);
      dc[e] = cb[row * p.K + k];
    }
    if (bb)
      for (int d = threadIdx.x; d < nd; d += kMaskThreads) {
        const size_t row = db ? (size_t)db[d0 + d] : (size_t)(d0 + d);
        const float* q = bb + row * 4;
        // box_to_mask (boxes.py:88-103): box scaled by (H, W, H, W), bounds as the reference forms them
        const float by = q[0] * (float)p.H, bx = q[1] * (float)p.W, bh = q[2] * (float)p.H, bw = q[3] * (float)p.W;
        db4[d] = make_float4(bx - bw / 2, bx + bw / 2, by - bh / 2, by + bh / 2);
      }
    __syncthreads();
    if (pix >= hw) continue;
    for (int d = 0; d < nd; ++d) {
      const float* c = dc + d * p.K;
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < p.K; ++k) {
        const float ck = c[k];
        const float4 v = *reinterpret_cast<const float4*>(pr + k * kMaskPix + q0);
        s[0] += ck * v.x;
        s[1] += ck * v.y;
        s[2] += ck * v.z;
        s[3] += ck * v.w;
      }
      // sigmoid on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each) instead of the
      // IEEE expf + division sequences that made this write-bound kernel VALU-bound (2.3 TB/s);
      // |error| < 1e-7 against torch.sigmoid's fp32 result
      float m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        m[e] = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-s[e] * 1.4426950408889634f));
      if (bb) {
        const float4 bd = db4[d];  // left, right, top, bottom
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float fx = (float)xx[e], fy = (float)yy[e];
          m[e] *= (fx >= bd.x && fx <= bd.y && fy >= bd.z && fy <= bd.w) ? 1.f : 0.f;
        }
      }
      float* o = ob + (size_t)(d0 + d) * hw + pix;
      if (vec) {
        *reinterpret_cast<float4*>(o) = make_float4(m[0], m[1], m[2], m[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (pix + e < hw) o[e] = m[e];
      }
    }
  }
}

// assemble_mask for K <= KT prototypes: the same arithmetic with each thread's 4 pixels x K
// prototype values held in registers (loaded once) instead of re-read from LDS for every
// detection — the LDS variant above read 8 x 16 B of prototypes per 16 B written and ran at
// ~3 TB/s; here a detection costs two broadcast LDS reads per thread (its coefficients and
// bounds), and the kernel runs at the write stream
template <int KT>
__global__ __launch_bounds__(kMaskThreads) void assemble_mask_reg(const MaskParams p) {
  __shared__ float dc[kMaskDets * KT];  // [kMaskDets][KT] coefficients (zero past K)
  __shared__ float4 db4[kMaskDets];     // left, right, top, bottom
  const int b = blockIdx.y;
  const int n = p.counts ? min(p.counts[b], p.n_max) : p.n_max;
  if (n <= 0) return;
  const int hw = p.H * p.W;
  const int pix = blockIdx.x * kMaskPix + 4 * threadIdx.x;
  const float* pb = p.proto + (size_t)b * p.ps_b;
  int yy[4], xx[4];
  float pv[KT][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int q = min(pix + e, hw - 1);
    yy[e] = q / p.W;
    xx[e] = q - yy[e] * p.W;
  }
#pragma unroll
  for (int k = 0; k < KT; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      pv[k][e] = k < p.K ? pb[(size_t)k * p.ps_k + (size_t)yy[e] * p.ps_y + (size_t)xx[e] * p.ps_x] : 0.f;
  const bool vec = (hw & 3) == 0;
  const float* cb = p.coeff + (size_t)b * p.rows * p.K;
  const float* bb = p.box ? p.box + (size_t)b * p.rows * 4 : nullptr;
  const long long* db = p.det ? p.det + (size_t)b * p.n_max : nullptr;
  float* ob = p.out + (size_t)b * p.n_max * hw;
  for (int d0 = 0; d0 < n; d0 += kMaskDets) {
    const int nd = min(kMaskDets, n - d0);
    __syncthreads();  // the previous chunk consumed
    for (int e = threadIdx.x; e < nd * KT; e += kMaskThreads) {
      const int d = e / KT, k = e - d * KT;
      const size_t row = db ? (size_t)db[d0 + d] : (size_t)(d0 + d);
      dc[e] = k < p.K ? cb[row * p.K + k] : 0.f;
    }
    if (bb)
      for (int d = threadIdx.x; d < nd; d += kMaskThreads) {
        const size_t row = db ? (size_t)db[d0 + d] : (size_t)(d0 + d);
        const float* q = bb + row * 4;
        const float by = q[0] * (float)p.H, bx = q[1] * (float)p.W, bh = q[2] * (float)p.H, bw = q[3] * (float)p.W;
        db4[d] = make_float4(bx - bw / 2, bx + bw / 2, by - bh / 2, by + bh / 2);
      }
    __syncthreads();
    if (pix >= hw) continue;
    for (int d = 0; d < nd; ++d) {
      const float* c = dc + d * KT;
      float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KT; ++k) {  // (k >= K: zero products; s is never -0, so adding them is exact)
        const float ck = c[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += ck * pv[k][e];
      }
      float m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        m[e] = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-s[e] * 1.4426950408889634f));
      if (bb) {
        const float4 bd = db4[d];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float fx = (float)xx[e], fy = (float)yy[e];
          m[e] *= (fx >= bd.x && fx <= bd.y && fy >= bd.z && fy <= bd.w) ? 1.f : 0.f;
        }
      }
      float* o = ob + (size_t)(d0 + d) * hw + pix;
      if (vec) {
        *reinterpret_cast<float4*>(o) = make_float4(m[0], m[1], m[2], m[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (pix + e < hw) o[e] = m[e];
      }
    }
  }
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

int launch_yolact_box_encode(const float* box, const float* anchor, int B, int A, int anchor_batch, float v0, float v1,
                             float* out, hipStream_t s) {
  if (B < 1 || A < 1 || (anchor_batch != 1 && anchor_batch != B) || (long)B * A >= (1L << 31)) {
    set_error("box_encode: bad shapes (anchor batch must be 1 or B)");
    return 2;
  }
  const unsigned n = (unsigned)B * A;
  hipLaunchKernelGGL(yolact::box_encode, dim3((n + 255) / 256), dim3(256), 0, s, box, anchor, B, A, anchor_batch, v0,
                     v1, out);
  TV_HIP(hipGetLastError());
  return 0;
}

namespace {

struct NmsLayout {
  size_t keys, skeys, sidx, keep, total;
};

size_t al(size_t x) { return (x + 255) / 256 * 256; }

int nms_layout(int B, int A, int K, NmsLayout* L) {
  const size_t n = (size_t)B * A;
  size_t o = 0;
  L->keys = o;  o += al(n * 4);
  L->skeys = o; o += al(n * 4);
  L->sidx = o;  o += al(n * 4);
  L->keep = o;  o += al((size_t)B * K);
  L->total = o;
  return 0;
}

}  // namespace

size_t yolact_nms_workspace_bytes(int B, int A, int top_k) {
  NmsLayout L{};
  if (B < 1 || A < 1 || top_k < 1 || nms_layout(B, A, std::min(top_k, A), &L)) return 0;
  return L.total;
}

int launch_yolact_fast_nms(const float* cls, long long cls_bstride, int A, int C1, const float* box,
                           long long box_bstride, int B, int top_k, float iou_thr, float conf_thr, void* ws,
                           size_t ws_bytes, long long* det, int det_stride, int* n_det, hipStream_t s) {
  if (A < 1 || B < 1 || C1 < 2 || top_k < 1 || (long long)B * A >= (1LL << 31)) {
    set_error("fast_nms: need anchors >= 1, >= 2 classes (incl. background), top_k >= 1");
    return 2;  // TV_ESHAPE
  }
  const int K = std::min(top_k, A);
  if (det_stride < K) { set_error("fast_nms: det row stride < min(top_k, anchors)"); return 1; }
  NmsLayout L{};
  int rc = nms_layout(B, A, K, &L);
  if (rc) return rc;
  if (!ws || ws_bytes < L.total) { set_error("fast_nms: workspace too small"); return 1; }
  char* w = (char*)ws;
  uint32_t* keys = (uint32_t*)(w + L.keys);
  uint32_t* skeys = (uint32_t*)(w + L.skeys);
  int* sidx = (int*)(w + L.sidx);
  uint8_t* keep = (uint8_t*)(w + L.keep);
  const unsigned n = (unsigned)B * A;
  hipLaunchKernelGGL(yolact::nms_keys, dim3((n + 255) / 256), dim3(256), 0, s, cls, cls_bstride, A, C1, B, keys);
  TV_HIP(hipGetLastError());
  if (K <= yolact::kTopkMaxK && A <= 32 * yolact::kTopkThreads) {
    // (first K entries of each segment: all nms_iou / nms_compact read)
    if (A <= 8 * yolact::kTopkThreads)
      hipLaunchKernelGGL(yolact::nms_topk<8>, dim3(B), dim3(yolact::kTopkThreads), 0, s, keys, A, K, skeys, sidx);
    else if (A <= 16 * yolact::kTopkThreads)
      hipLaunchKernelGGL(yolact::nms_topk<16>, dim3(B), dim3(yolact::kTopkThreads), 0, s, keys, A, K, skeys, sidx);
    else
      hipLaunchKernelGGL(yolact::nms_topk<32>, dim3(B), dim3(yolact::kTopkThreads), 0, s, keys, A, K, skeys, sidx);
    TV_HIP(hipGetLastError());
  } else {
    constexpr int lds = yolact::kSortCap * 8;
    static std::once_flag once;
    hipError_t attr = hipSuccess;
    std::call_once(once, [&] {
      attr = hipFuncSetAttribute((const void*)yolact::nms_sort, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    });
    TV_HIP(attr);
    hipLaunchKernelGGL(yolact::nms_sort, dim3(B), dim3(yolact::kSortThreads), lds, s, keys, A, K, skeys, sidx);
    TV_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(yolact::nms_iou, dim3((K + yolact::kIouThreads - 1) / yolact::kIouThreads, B),
                     dim3(yolact::kIouThreads), 0, s, box, box_bstride, A, K, skeys, sidx, iou_thr, conf_thr, keep);
  TV_HIP(hipGetLastError());
  hipLaunchKernelGGL(yolact::nms_compact, dim3(B), dim3(yolact::kCompactThreads), 0, s, keep, A, K, sidx, det,
                     det_stride, n_det);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_yolact_assemble_mask(const float* proto, const long long pst[4], int B, int K, int H, int W,
                                const float* coeff, const float* box, const int* counts, const long long* det,
                                int rows, int n_max, float* out, hipStream_t s) {
  if (B < 1 || K < 1 || H < 1 || W < 1 || n_max < 0 || (long)H * W >= (1L << 30) || B > 65535) {
    set_error("assemble_mask: bad shapes");
    return 2;  // TV_ESHAPE
  }
  if (n_max == 0) return 0;
  yolact::MaskParams p{proto, pst[0], pst[1], pst[2], pst[3], K, H, W, coeff, box, counts, det, det ? rows : n_max,
                       n_max, out};
  const int hw = H * W;
  const dim3 grid((hw + yolact::kMaskPix - 1) / yolact::kMaskPix, B);
  if (K <= 16) {  // prototypes in registers (the protonet's k = 8; any K up to 16)
    if (K <= 8) hipLaunchKernelGGL(yolact::assemble_mask_reg<8>, grid, dim3(yolact::kMaskThreads), 0, s, p);
    else hipLaunchKernelGGL(yolact::assemble_mask_reg<16>, grid, dim3(yolact::kMaskThreads), 0, s, p);
    TV_HIP(hipGetLastError());
    return 0;
  }
  const size_t lds = ((size_t)K * yolact::kMaskPix + (size_t)yolact::kMaskDets * (K + 4)) * sizeof(float);
  if (lds > 160 * 1024) { set_error("assemble_mask: more than 37 prototypes"); return 2; }
  static std::once_flag attr_once;
  hipError_t attr_err = hipSuccess;
  std::call_once(attr_once, [&] {
    attr_err = hipFuncSetAttribute((const void*)yolact::assemble_mask, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
  });
  TV_HIP(attr_err);
  hipLaunchKernelGGL(yolact::assemble_mask, grid, dim3(yolact::kMaskThreads), lds, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
