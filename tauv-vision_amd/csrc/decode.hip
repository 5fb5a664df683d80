// Heatmap peak decode on gfx950: sigmoid + k x k peak NMS, exact per-image top-K, and the
// per-detection gather of size/offset/depth (decode.py:179-279, 51-98).
//
//  peaks   : one thread per heatmap element, any input strides (NCHW views or the
//            engine's NHWC head tensor); output is the dense heatmap_nms() map.
//  topk    : one 1024-thread workgroup per image. Exact radix select on the 64-bit key
//            (orderable score bits << 32 | ~flat_index), so the result is the true top-K
//            with ties broken toward the smaller flat index (torch.topk leaves tie order
//            unspecified, decode.py:269). 11-bit digit histograms in LDS; once the
//            threshold bucket holds <= 4096 keys they are sorted in LDS (bitonic).
//  records : one workgroup per image; [label, score, y, x, h, w, depth, flat index, aux0,
//            aux1] per detection (aux = the keypoint affinity pair of decode.py:121-122)
//            plus the count of scores >= threshold (the host loop's break, decode.py:207).
#include "common.h"

namespace tv {

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void peaks_kernel(const float* __restrict__ heat, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                             int B, int C, int H, int W, int r, int apply_sigmoid, float* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)B * C * H * W;
  if (i >= total) return;
  int x = i % W;
  int y = (i / W) % H;
  size_t bc = i / ((size_t)H * W);
  int c = bc % C;
  int b = bc / C;
  const float* base = heat + b * s0 + c * s1;
  float v = base[y * s2 + x * s3];
  if (apply_sigmoid) v = sigmoidf_ref(v);
  float m = v;
  for (int dy = -r; dy <= r; ++dy) {
    int yy = y + dy;
    if (yy < 0 || yy >= H) continue;
    for (int dx = -r; dx <= r; ++dx) {
      int xx = x + dx;
      if (xx < 0 || xx >= W) continue;
      float u = base[yy * s2 + xx * s3];
      if (apply_sigmoid) u = sigmoidf_ref(u);
      m = fmaxf(m, u);
    }
  }
  out[i] = (float)(m == v) * v;
}

int launch_peaks(const float* heat, const int64_t st[4], int B, int C, int H, int W, int k, int apply_sigmoid,
                 float* peaks, hipStream_t s) {
  size_t total = (size_t)B * C * H * W;
  if (total == 0) return 0;
  hipLaunchKernelGGL(peaks_kernel, dim3((total + 255) / 256), dim3(256), 0, s, heat, st[0], st[1], st[2], st[3],
                     B, C, H, W, (k - 1) / 2, apply_sigmoid, peaks);
  TV_HIP(hipGetLastError());
  return 0;
}

// ---- exact top-K --------------------------------------------------------------------
constexpr int kSelThreads = 1024;
constexpr int kBins = 2048;
constexpr int kCap = 4096;
constexpr int kMaxK = 1024;

__device__ __forceinline__ uint32_t order_bits(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unorder_bits(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ uint64_t make_key(float f, uint32_t idx) {
  return ((uint64_t)order_bits(f) << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}

// block-wide inclusive scan of one int per thread (1024 threads = 16 waves)
__device__ int block_scan_incl(int v, int* wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  if (lane == 63) wsum[wave] = v;
  __syncthreads();
  if (wave == 0) {
    int w = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      int t = __shfl_up(w, o);
      if (lane >= o) w += t;
    }
    if (lane < 16) wsum[lane] = w;
  }
  __syncthreads();
  int r = v + (wave > 0 ? wsum[wave - 1] : 0);
  __syncthreads();
  return r;
}

__device__ void bitonic_desc(uint64_t* a, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kSelThreads) {
        int ixj = i ^ j;
        if (ixj > i) {
          uint64_t x = a[i], y = a[ixj];
          bool up = (i & k) == 0;  // this run ends descending
          if (up ? (x < y) : (x > y)) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(kSelThreads) void topk_kernel(const float* __restrict__ peaks, int64_t n, int K,
                                                           float* __restrict__ out_score,
                                                           int32_t* __restrict__ out_index) {
  __shared__ int hist[kBins];
  __shared__ uint64_t eq[kCap];
  __shared__ uint64_t top[kMaxK];
  __shared__ int wsum[16];
  __shared__ int sel_digit, sel_before, sel_count, n_top, n_eq;
  const float* v = peaks + (size_t)blockIdx.x * n;
  const int tid = threadIdx.x;

  uint64_t prefix = 0, pmask = 0;
  int need = K, shift = 64;
  for (;;) {
    const int nshift = shift > 11 ? shift - 11 : 0;
    const int width = shift - nshift;
    const int nb = 1 << width;
    for (int i = tid; i < kBins; i += kSelThreads) hist[i] = 0;
    __syncthreads();
    const uint64_t dmask = (uint64_t)(nb - 1);
    for (int64_t i = tid; i < n; i += kSelThreads) {
      uint64_t key = make_key(v[i], (uint32_t)i);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> nshift) & dmask], 1);
    }
    __syncthreads();
    // bins ordered from the top: thread t owns top-order positions 2t, 2t+1
    int d0 = nb - 1 - 2 * tid, d1 = d0 - 1;
    int h0 = d0 >= 0 ? hist[d0] : 0;
    int h1 = d1 >= 0 ? hist[d1] : 0;
    int incl = block_scan_incl(h0 + h1, wsum);
    int before = incl - h0 - h1;
    if (d0 >= 0 && before < need && need <= before + h0) {
      sel_digit = d0; sel_before = before; sel_count = h0;
    }
    if (d1 >= 0 && before + h0 < need && need <= before + h0 + h1) {
      sel_digit = d1; sel_before = before + h0; sel_count = h1;
    }
    __syncthreads();
    prefix |= (uint64_t)sel_digit << nshift;
    pmask |= dmask << nshift;
    need -= sel_before;
    const int cnt = sel_count;
    shift = nshift;
    __syncthreads();
    if (cnt <= kCap || shift == 0) break;
  }

  // collect: keys strictly above the prefix are in; keys equal to it compete for `need`
  if (tid == 0) { n_top = 0; n_eq = 0; }
  __syncthreads();
  for (int64_t i = tid; i < n; i += kSelThreads) {
    uint64_t key = make_key(v[i], (uint32_t)i);
    uint64_t hi = key & pmask;
    if (hi > prefix) top[atomicAdd(&n_top, 1)] = key;
    else if (hi == prefix) eq[atomicAdd(&n_eq, 1)] = key;
  }
  __syncthreads();
  const int ne = n_eq;
  int P = 1;
  while (P < ne) P <<= 1;
  for (int i = ne + tid; i < P; i += kSelThreads) eq[i] = 0;
  __syncthreads();
  bitonic_desc(eq, P);
  const int nt = n_top;  // == K - need
  for (int i = tid; i < need; i += kSelThreads) top[nt + i] = eq[i];
  __syncthreads();
  int PK = 1;
  while (PK < K) PK <<= 1;
  for (int i = K + tid; i < PK; i += kSelThreads) top[i] = 0;
  __syncthreads();
  bitonic_desc(top, PK);
  for (int i = tid; i < K; i += kSelThreads) {
    uint64_t key = top[i];
    out_score[(size_t)blockIdx.x * K + i] = unorder_bits((uint32_t)(key >> 32));
    out_index[(size_t)blockIdx.x * K + i] = (int32_t)(0xFFFFFFFFu - (uint32_t)key);
  }
}

int launch_topk(const float* peaks, int B, int64_t n, int K, float* score, int32_t* index, hipStream_t s) {
  if (K < 1 || K > kMaxK || K > n) { set_error("topk: need 1 <= K <= min(1024, C*H*W)"); return 1; }
  if (n >= (int64_t)0xFFFFFFFF) { set_error("topk: image too large"); return 1; }
  hipLaunchKernelGGL(topk_kernel, dim3(B), dim3(kSelThreads), 0, s, peaks, n, K, score, index);
  TV_HIP(hipGetLastError());
  return 0;
}

// ---- detection records ------------------------------------------------------------------
__global__ void records_kernel(const DecodeParams p, int64_t ss0, int64_t ss1, int64_t ss2, int64_t ss3,
                               int64_t os0, int64_t os1, int64_t os2, int64_t os3, int64_t ds0, int64_t ds1,
                               int64_t ds2, int64_t ds3) {
  __shared__ int cnt;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const int hw = p.H * p.W;
  int local = 0;
  for (int k = threadIdx.x; k < p.K; k += blockDim.x) {
    const float score = p.score[(size_t)b * p.K + k];
    const int idx = p.index[(size_t)b * p.K + k];
    const int label = idx / hw;
    const int rem = idx - label * hw;
    const int iy = rem / p.W;
    const int ix = rem - iy * p.W;
    float* r = p.records + ((size_t)b * p.K + k) * 10;
    const float* sz = p.size + b * ss0 + iy * ss1 + ix * ss2;
    float y, x;
    if (p.pos_mode == 0) {
      const float* of = p.offset + b * os0 + iy * os1 + ix * os2;
      y = (float)(((double)p.ratio * (double)iy + (double)of[0]) / (double)p.in_h);
      x = (float)(((double)p.ratio * (double)ix + (double)of[os3]) / (double)p.in_w);
    } else {
      y = (float)iy / (float)p.out_h;
      x = (float)ix / (float)p.out_w;
    }
    float depth = __builtin_nanf("");
    if (p.depth) {
      float d = p.depth[b * ds0 + iy * ds1 + ix * ds2];
      float sg = 1.0f / (1.0f + expf(-d));
      depth = p.depth_mode == 0 ? (1.0f / sg) - 1.0f : 1.0f / sg;
    }
    r[0] = (float)label;
    r[1] = score;
    r[2] = y;
    r[3] = x;
    r[4] = sz[0];
    r[5] = sz[ss3];
    r[6] = depth;
    r[7] = (float)idx;
    if (p.aux) {
      const float* a = p.aux + b * p.aux_st[0] + label * p.aux_st[1] + iy * p.aux_st[3] + ix * p.aux_st[4];
      r[8] = a[0];
      r[9] = a[p.aux_st[2]];
    } else {
      r[8] = r[9] = __builtin_nanf("");
    }
    local += score >= p.score_thr ? 1 : 0;
  }
  atomicAdd(&cnt, local);
  __syncthreads();
  if (threadIdx.x == 0) p.counts[b] = cnt;
}

int launch_decode_records(const DecodeParams& p, hipStream_t s) {
  const int64_t z[4] = {0, 0, 0, 0};
  const int64_t* os = p.offset_st ? p.offset_st : z;
  const int64_t* ds = p.depth_st ? p.depth_st : z;
  hipLaunchKernelGGL(records_kernel, dim3(p.B), dim3(256), 0, s, p, p.size_st[0], p.size_st[1], p.size_st[2],
                     p.size_st[3], os[0], os[1], os[2], os[3], ds[0], ds[1], ds[2], ds[3]);
  TV_HIP(hipGetLastError());
  return 0;
}

__global__ void index_split_kernel(const int32_t* __restrict__ flat, int n, int hw, int W,
                                   int64_t* __restrict__ index, int64_t* __restrict__ label) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int f = flat[i];
  int l = f / hw;
  int rem = f - l * hw;
  label[i] = l;
  index[2 * i] = rem / W;
  index[2 * i + 1] = rem % W;
}

int launch_index_split(const int32_t* flat, int B, int K, int H, int W, int64_t* index, int64_t* label,
                       hipStream_t s) {
  int n = B * K;
  if (n == 0) return 0;
  hipLaunchKernelGGL(index_split_kernel, dim3((n + 255) / 256), dim3(256), 0, s, flat, n, H * W, W, index, label);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
