// Heatmap peak decode on gfx950: sigmoid + 3x3 peak NMS, exact per-image top-K and the
// per-detection gather of size/offset/depth (decode.py:179-279, 51-98), as two launches that
// read the head tensor once:
//
//  tile_select : grid B x tiles. A tile is (channel group, row band, column band) of one
//                image. Its elements plus a one-pixel halo are loaded ONCE into LDS (sigmoid
//                applied once per element, out-of-image = -inf like max_pool2d's implicit
//                padding), each thread forms the 3x3 NMS keys of its 16 elements in
//                registers, and an exact block radix select (8-bit digits over the 64-bit key
//                = orderable score bits << 32 | ~flat index) keeps the tile's top K, written
//                unordered to a fixed K-slot list (zero-key padded when the tile has < K).
//  merge       : grid B (x groups). Up to kMergeCap candidate keys per workgroup in registers,
//                the same radix select -> top K; the final level sorts them (bitonic, LDS)
//                and writes score / flat index and, for tv_decode, the detection records
//                ([label, score, y, x, h, w, depth, flat index, aux0, aux1] + the count of
//                scores >= threshold, the host loop's break at decode.py:207).
// Keys are unique (the flat index is in the low word), so the selection is exact and ties
// in score resolve toward the smaller flat index (torch.topk: unspecified, decode.py:269).
//
//  peaks       : heatmap_nms() as a dense map (tv_heatmap_nms, parity API only).
#include "common.h"

#include <algorithm>
#include <vector>

namespace tv {

// diagnostic builds only (EXTRA=-DTV_DEC_STAMPS=1): thread 0's shader-clock stamps at the decode
// kernel's phase boundaries, written by the selecting workgroup into its image's last two records
#if defined(TV_DEC_STAMPS)
#define DSTAMP(arr, i)                                                                   \
  do {                                                                                   \
    if (threadIdx.x == 0) {                                                              \
      unsigned long long t_;                                                             \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
      (arr)[i] = t_;                                                                     \
    }                                                                                    \
  } while (0)
#else
#define DSTAMP(arr, i) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---- heatmap_nms as a dense map (tv_heatmap_nms) ----------------------------------------
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

// ---- keys and the block radix select ----------------------------------------------------
constexpr int kTileThreads = 512;
constexpr int kTilePer = 16;                             // keys per thread in tile_select
constexpr int kTileElems = kTileThreads * kTilePer;      // 8192 elements per tile
constexpr int kMergeThreads = 1024;
constexpr int kMergePer = 16;
constexpr int kMergeCap = kMergeThreads * kMergePer;     // 16384 candidates per merge workgroup
constexpr int kMaxK = 1024;
constexpr int kSmallMergeThreads = 256, kSmallMergePer = 4;
constexpr int kSmallMergeCap = kSmallMergeThreads * kSmallMergePer;

__device__ __forceinline__ uint32_t order_bits(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unorder_bits(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
// > 0 for every real element (flat index < 2^32 - 1), so 0 marks padding
__device__ __forceinline__ uint64_t make_key(float f, uint32_t idx) {
  return ((uint64_t)order_bits(f) << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}

struct SelectShared {
  int hist[256];
  unsigned long long red_lo[16], red_hi[16];
  int red_n[16];
  int sel_digit, sel_above, sel_count, nreal, nout;
};

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// block-wide (min, max) of 64-bit values and sum of ints
template <int NT>
__device__ void block_minmax_sum(uint64_t& lo, uint64_t& hi, int& n, SelectShared& sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t l = shfl_xor_u64(lo, m), h = shfl_xor_u64(hi, m);
    lo = l < lo ? l : lo;
    hi = h > hi ? h : hi;
    n += __shfl_xor(n, m);
  }
  if (lane == 0) { sh.red_lo[wave] = lo; sh.red_hi[wave] = hi; sh.red_n[wave] = n; }
  __syncthreads();
  lo = ~0ull; hi = 0; n = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    lo = sh.red_lo[w] < lo ? sh.red_lo[w] : lo;
    hi = sh.red_hi[w] > hi ? sh.red_hi[w] : hi;
    n += sh.red_n[w];
  }
  __syncthreads();
}

// Threshold T with |{real keys >= T}| == need (1 <= need <= number of real keys; real keys are
// non-zero). Keys are unique. Every pass first narrows the key range to the keys still in play
// (block min / max), then histograms the 8-bit digit just below their common high bits — so
// passes never spend themselves on bits all candidates share, and LDS atomics spread over the
// candidates' actual value range (a flat heatmap puts every score in one fixed-digit bucket).
// Keys of positive scores and the rest (NMS-suppressed zeros, negatives) are split first: when
// fewer than `need` keys have a positive score, all of them are in and the rest is selected
// among the others (ties at score 0 go to the smaller flat index).
template <int NT, int PER>
__device__ uint64_t block_select(const uint64_t (&k)[PER], int need, SelectShared& sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr uint64_t kZ = (0x80000000ull << 32) | 0xFFFFFFFFull;  // largest key of score +0.0
  int upper = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) upper += k[j] > kZ;
  {
    uint64_t a = ~0ull, b = 0;
    block_minmax_sum<NT>(a, b, upper, sh);
  }
  const bool lower_mode = upper < need;
  if (lower_mode) need -= upper;
  uint64_t prefix = 0, pmask = 0;
  for (;;) {
    // keys still in play: eligible class, matching the fixed high bits
    uint64_t lo = ~0ull, hi = 0;
    int dummy = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t key = k[j];
      const bool el = key != 0 && (key > kZ) != lower_mode && (key & pmask) == prefix;
      if (el) { lo = key < lo ? key : lo; hi = key > hi ? key : hi; }
    }
    block_minmax_sum<NT>(lo, hi, dummy, sh);
    const uint64_t diff = lo ^ hi;
    if (diff == 0) return hi;  // one key left in play: it is the need-th (need == 1)
    const int msb = 63 - __builtin_clzll(diff);
    const int shift = msb > 7 ? msb - 7 : 0;
    // bits above the window are shared by every key in play; bits fixed by earlier passes may
    // reach into the window (a narrow final range) and stay fixed
    pmask |= shift + 8 >= 64 ? 0 : ~((1ull << (shift + 8)) - 1);
    prefix = hi & pmask;
    for (int i = tid; i < 256; i += NT) sh.hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t key = k[j];
      if (key != 0 && (key > kZ) != lower_mode && (key & pmask) == prefix)
        atomicAdd(&sh.hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (wave == 0) {
      // lane l owns digits 255-4l .. 252-4l (top-down order); exclusive scan from the top
      int c[4], sum = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) { c[i] = sh.hist[255 - 4 * lane - i]; sum += c[i]; }
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      int before = incl - sum;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (before < need && need <= before + c[i]) {
          sh.sel_digit = 255 - 4 * lane - i;
          sh.sel_above = before;
          sh.sel_count = c[i];
        }
        before += c[i];
      }
    }
    __syncthreads();
    const int digit = sh.sel_digit, above = sh.sel_above, cnt = sh.sel_count;
    __syncthreads();
    prefix |= (uint64_t)digit << shift;
    pmask |= (uint64_t)255 << shift;
    need -= above;
    if (shift == 0) return prefix;  // full key: a single (unique) key
    if (cnt == need) {
      // the whole bucket is in: the threshold is its smallest key (a real key, so `key >= T`
      // never reaches below the eligible class)
      uint64_t m = ~0ull, h = 0;
      int d = 0;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint64_t key = k[j];
        if (key != 0 && (key > kZ) != lower_mode && (key & pmask) == prefix) m = key < m ? key : m;
      }
      block_minmax_sum<NT>(m, h, d, sh);
      return m;
    }
  }
}

template <int NT>
__device__ int block_count_real(int local, SelectShared& sh) {
  if (threadIdx.x == 0) sh.nreal = 0;
  __syncthreads();
  if (local) atomicAdd(&sh.nreal, local);
  __syncthreads();
  return sh.nreal;
}

// ---- stage 1: per-tile NMS + top-K candidates -------------------------------------------
struct TileGeom {
  int cg, th, tw;          // tile extent: channels, rows, columns
  int ncg, nth, ntw;       // tiles per image along each
  int r;                   // NMS radius (0 = no NMS), halo width
  int apply_sigmoid;
  int chan_fast;           // LDS fill order: 1 = channel fastest (NHWC views), 0 = column fastest
};

__global__ __launch_bounds__(kTileThreads) void tile_select(const float* __restrict__ heat, int64_t s0, int64_t s1,
                                                            int64_t s2, int64_t s3, int C, int H, int W,
                                                            const TileGeom g, int K, uint64_t* __restrict__ cand) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  __shared__ SelectShared sh;
  const int b = blockIdx.y;
  int t = blockIdx.x;
  const int tx = t % g.ntw; t /= g.ntw;
  const int ty = t % g.nth;
  const int tc = t / g.nth;
  const int c0 = tc * g.cg, y0 = ty * g.th, x0 = tx * g.tw;
  const int nc = min(g.cg, C - c0), nh = min(g.th, H - y0), nw = min(g.tw, W - x0);
  const int r = g.r;
  const int LH = nh + 2 * r, LW = nw + 2 * r;
  const float* base = heat + b * s0;

  // tile + halo -> LDS [cc][yy][xx], sigmoid applied once per element; outside the image -inf.
  // Loads are issued in batches of kFillBatch per thread before any is consumed, so a block pays
  // one memory latency per batch instead of one per element.
  const int nl = nc * LH * LW;
  constexpr int kFillBatch = 8;
  for (int e0 = 0; e0 < nl; e0 += kTileThreads * kFillBatch) {
    float v[kFillBatch];
    int dst[kFillBatch];
    bool inb[kFillBatch];
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j) {
      const int e = e0 + j * kTileThreads + threadIdx.x;
      int cc, yy, xx;
      if (g.chan_fast) {
        cc = e % nc;
        const int p = e / nc;
        xx = p % LW;
        yy = p / LW;
      } else {
        xx = e % LW;
        const int p = e / LW;
        yy = p % LH;
        cc = p / LH;
      }
      const int y = y0 + yy - r, x = x0 + xx - r;
      const bool in = e < nl && y >= 0 && y < H && x >= 0 && x < W;
      inb[j] = in;
      v[j] = in ? base[(int64_t)(c0 + cc) * s1 + (int64_t)y * s2 + (int64_t)x * s3] : 0.f;
      dst[j] = e < nl ? (cc * LH + yy) * LW + xx : -1;
    }
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j) {
      if (dst[j] < 0) continue;
      tile[dst[j]] = !inb[j] ? -INFINITY : g.apply_sigmoid ? sigmoidf_ref(v[j]) : v[j];
    }
  }
  __syncthreads();

  // NMS keys of this thread's elements (element e = tid + j * NT, column fastest)
  const int ne = nc * nh * nw;
  uint64_t k[kTilePer];
#pragma unroll
  for (int j = 0; j < kTilePer; ++j) {
    const int e = threadIdx.x + j * kTileThreads;
    k[j] = 0;
    if (e < ne) {
      const int xx = e % nw;
      const int p = e / nw;
      const int yy = p % nh;
      const int cc = p / nh;
      const float* row = tile + (cc * LH + yy + r) * LW + xx + r;
      const float v = row[0];
      float m = v;
      if (r) {
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) m = fmaxf(m, row[dy * LW + dx]);
      }
      const float pv = (float)(m == v) * v;  // (hmax == h).float() * h (decode.py:252)
      const uint32_t flat = (uint32_t)(((c0 + cc) * H + y0 + yy) * W + x0 + xx);
      k[j] = make_key(pv, flat);
    }
  }
  const int kt = min(K, ne);
  const uint64_t T = block_select<kTileThreads, kTilePer>(k, kt, sh);
  if (threadIdx.x == 0) sh.nout = 0;
  __syncthreads();
  uint64_t* out = cand + ((size_t)b * gridDim.x + blockIdx.x) * K;
#pragma unroll
  for (int j = 0; j < kTilePer; ++j)
    if (k[j] != 0 && k[j] >= T) out[atomicAdd(&sh.nout, 1)] = k[j];
  __syncthreads();
  for (int i = sh.nout + threadIdx.x; i < K; i += kTileThreads) out[i] = 0;
}

// ---- stage 2: merge candidate lists (K slots each) -> top K -----------------------------

template <int NT>
__device__ void bitonic_desc(uint64_t* a, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;  // this run ends descending
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

struct MergeOut {
  float* score;        // [B][K] (final level)
  int32_t* index;      // [B][K]
  int records;         // 1: also write detection records (DecodeParams)
};

// A detection record's inputs, gathered from its key (decode.py:204-234 / 71-98 field meaning):
// issued before the key's rank is known, so the loads overlap the ranking
struct RecIn {
  float sz0, sz1, of0, of1, d, a0, a1;
};
__device__ __forceinline__ RecIn gather_record(uint64_t key, int b, const DecodeParams& p) {
  RecIn r;
  const int idx = (int)(0xFFFFFFFFu - (uint32_t)key);
  const int hw = p.H * p.W;
  const int label = idx / hw;
  const int rem = idx - label * hw;
  const int iy = rem / p.W;
  const int ix = rem - iy * p.W;
  const float* sz = p.size + b * p.size_st[0] + iy * p.size_st[1] + ix * p.size_st[2];
  r.sz0 = sz[0];
  r.sz1 = sz[p.size_st[3]];
  r.of0 = r.of1 = 0.f;
  if (p.pos_mode == 0) {
    const float* of = p.offset + b * p.offset_st[0] + iy * p.offset_st[1] + ix * p.offset_st[2];
    r.of0 = of[0];
    r.of1 = of[p.offset_st[3]];
  }
  r.d = p.depth ? p.depth[b * p.depth_st[0] + iy * p.depth_st[1] + ix * p.depth_st[2]] : 0.f;
  r.a0 = r.a1 = __builtin_nanf("");
  if (p.aux) {
    const float* a = p.aux + b * p.aux_st[0] + label * p.aux_st[1] + iy * p.aux_st[3] + ix * p.aux_st[4];
    r.a0 = a[0];
    r.a1 = a[p.aux_st[2]];
  }
  return r;
}

// output slot i (rank i, descending) of image b from its key (and, for records, its gathered
// inputs): score / flat index and / or the detection record; returns score >= threshold
__device__ __forceinline__ int store_record(uint64_t key, const RecIn& in, int i, int K, int b, const MergeOut& mo,
                                            const DecodeParams& p) {
  const float score = unorder_bits((uint32_t)(key >> 32));
  const int idx = (int)(0xFFFFFFFFu - (uint32_t)key);
  if (mo.score) {
    mo.score[(size_t)b * K + i] = score;
    mo.index[(size_t)b * K + i] = idx;
  }
  if (!mo.records) return 0;
  const int hw = p.H * p.W;
  const int label = idx / hw;
  const int rem = idx - label * hw;
  const int iy = rem / p.W;
  const int ix = rem - iy * p.W;
  float* rr = p.records + ((size_t)b * K + i) * 10;
  float y, x;
  if (p.pos_mode == 0) {
    y = (float)(((double)p.ratio * (double)iy + (double)in.of0) / (double)p.in_h);
    x = (float)(((double)p.ratio * (double)ix + (double)in.of1) / (double)p.in_w);
  } else {
    y = (float)iy / (float)p.out_h;
    x = (float)ix / (float)p.out_w;
  }
  float depth = __builtin_nanf("");
  if (p.depth) {
    const float sg = 1.0f / (1.0f + expf(-in.d));
    depth = p.depth_mode == 0 ? (1.0f / sg) - 1.0f : 1.0f / sg;
  }
  rr[0] = (float)label;
  rr[1] = score;
  rr[2] = y;
  rr[3] = x;
  rr[4] = in.sz0;
  rr[5] = in.sz1;
  rr[6] = depth;
  rr[7] = (float)idx;
  rr[8] = in.a0;
  rr[9] = in.a1;
  return score >= p.score_thr ? 1 : 0;
}

__device__ __forceinline__ int write_record(uint64_t key, int i, int K, int b, const MergeOut& mo,
                                            const DecodeParams& p) {
  return store_record(key, mo.records ? gather_record(key, b, p) : RecIn{}, i, K, b, mo, p);
}

// top[0..K) (descending keys) -> score / flat index and, for tv_decode, the detection records
// + the count of scores >= threshold
template <int NT>
__device__ void write_outputs(const uint64_t* top, int K, int b, const MergeOut& mo, const DecodeParams& p,
                              int& cnt_thr) {
  int local_thr = 0;
  for (int i = threadIdx.x; i < K; i += NT) local_thr += write_record(top[i], i, K, b, mo, p);
  if (mo.records) {
    if (local_thr) atomicAdd(&cnt_thr, local_thr);
    __syncthreads();
    if (threadIdx.x == 0) p.counts[b] = cnt_thr;
  }
}


// NT x PER candidate slots per workgroup: the full-size variant (1024 x 16) for the intermediate
// levels, a 256 x 4 one when a single workgroup's candidates fit (B x 10 lists of K = 100 at
// 120x160): a quarter of the waves in every block-wide step
template <int NT, int PER>
__global__ __launch_bounds__(NT) void merge_select(const uint64_t* __restrict__ in, int lists, int group, int K,
                                                   uint64_t* __restrict__ next, int final_level, const MergeOut mo,
                                                   const DecodeParams p) {
  __shared__ SelectShared sh;
  __shared__ uint64_t top[kMaxK];
  __shared__ int cnt_thr;
  const int b = blockIdx.y, grp = blockIdx.x;
  const int l0 = grp * group, nl = min(group, lists - l0);
  const uint64_t* src = in + ((size_t)b * lists + l0) * K;
  const int n = nl * K;
  uint64_t k[PER];
  int local = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + j * NT;
    k[j] = e < n ? src[e] : 0;
    local += k[j] != 0;
  }
  const int real = block_count_real<NT>(local, sh);
  const int kt = min(K, real);
  const uint64_t T = block_select<NT, PER>(k, kt, sh);
  if (threadIdx.x == 0) { sh.nout = 0; cnt_thr = 0; }
  __syncthreads();
  if (!final_level) {
    uint64_t* out = next + ((size_t)b * gridDim.x + grp) * K;
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (k[j] != 0 && k[j] >= T) out[atomicAdd(&sh.nout, 1)] = k[j];
    __syncthreads();
    for (int i = sh.nout + threadIdx.x; i < K; i += NT) out[i] = 0;
    return;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (k[j] != 0 && k[j] >= T) top[atomicAdd(&sh.nout, 1)] = k[j];
  int P = 1;
  while (P < K) P <<= 1;
  __syncthreads();
  for (int i = sh.nout + threadIdx.x; i < P; i += NT) top[i] = 0;
  __syncthreads();
  bitonic_desc<NT>(top, P);
  write_outputs<NT>(top, K, b, mo, p, cnt_thr);
}


// ---- decode fast path: one launch (tv_decode: sigmoid, 3x3 NMS, exact top-K, records) ---------
// The per-tile block selects above cost ~20 barriers per tile and per merge level; the decode
// path instead makes one pass over the heatmap that keeps only what the exact top-K can need, and
// the image's last tile to finish selects:
//  peak_scan : grid B x tiles. Tile + halo -> LDS (sigmoid once), NMS keys in registers; the keys
//              of the "positive" class (score > +0, the only class the top K draws from while an
//              image has >= K of them) that can still be in the tile's top K (an 8-bit digit
//              pre-filter) are appended to the image's key array (one atomic per workgroup for the
//              base) with write-through stores; then one agent-scope ticket per workgroup. The
//              workgroup drawing the image's last ticket selects (fused_select): 8-bit radix
//              passes over the image's keys (LDS histogram, one bin per thread) until at most
//              kRankCap keys can still be in the top K; those are ranked exactly (keys are unique)
//              into descending order and the records written. An image with fewer than K
//              positive keys (degenerate: scores saturated to 0, NaN maps) takes an exact
//              streaming block select over all of its keys instead. The last workgroup leaves the
//              image's key count and ticket at zero for the next call (the workspace starts
//              zero-filled), so a captured graph replays without a reset launch.
constexpr int kScanThreads = 256, kScanPer = 16;
constexpr int kScanElems = kScanThreads * kScanPer;   // 4096 elements per tile (and key slots per tile)
constexpr int kRankCap = 256;                         // candidates ranked directly (or K when larger)
constexpr int kMaxScanTiles = 4096;                   // tiles per image
constexpr uint64_t kZeroKey = (0x80000000ull << 32) | 0xFFFFFFFFull;  // largest key of score +0.0

struct ScanWs {
  uint32_t* img_cnt;  // image b's keys appended so far at [2b] (zero between calls)
  uint32_t* ticket;   // image b's tiles finished at [2b] (zero between calls)
  uint64_t* keys;     // [B][tiles * kScanElems] the image's appended keys
  int tiles;          // per image
  uint32_t N;         // C * H * W
};

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ void raw_buffer_store_v2(u32x2 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v2i32");
__device__ u32x2 raw_buffer_load_v2(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
constexpr int kSC1 = 16;  // aux cache bits: sc1 (write-through store / L1- and L2-coherent load)
typedef __attribute__((address_space(1))) uint32_t gu32;

// the image's key array as a buffer resource (keys at 8-byte offsets)
__device__ __forceinline__ i32x4 keys_rsrc(const ScanWs& w, int b) {
  const unsigned long long a = (unsigned long long)(w.keys + (size_t)b * w.tiles * kScanElems);
  i32x4 r;
  r.x = (int)(unsigned)a;
  r.y = (int)(unsigned)(a >> 32);
  r.z = (int)((unsigned)w.tiles * kScanElems * 8u);
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ uint64_t load_key(const i32x4& rs, int i) {
  const u32x2 v = raw_buffer_load_v2(rs, i * 8, 0, kSC1);
  return ((uint64_t)v.y << 32) | v.x;
}

// Wave-aggregated append: the lanes with `pred` get consecutive slots of *counter (one LDS
// atomic per wave). Call from wave-uniform control flow.
__device__ __forceinline__ int wave_append_slot(int* counter, bool pred) {
  const int lane = threadIdx.x & 63;
  const uint64_t bal = __ballot(pred);
  int base = 0;
  if (lane == 0 && bal) base = atomicAdd(counter, (int)__popcll(bal));
  base = __shfl(base, 0);
  return base + (int)__popcll(bal & ((1ull << lane) - 1));
}

// LDS histogram increment that stays cheap whether the wave's bins crowd or spread: the lanes
// sharing the first active lane's bin add once (one atomic), the others add individually.
// Call from wave-uniform control flow.
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t bin, bool valid) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(valid);
  if (!act) return;
  const int leader = __ffsll((unsigned long long)act) - 1;
  const uint32_t lb = (uint32_t)__shfl((int)bin, leader);
  const uint64_t same = __ballot(valid && bin == lb);
  if (lane == leader) atomicAdd(&h[lb], (uint32_t)__popcll(same));
  if (valid && bin != lb) atomicAdd(&h[bin], 1u);
}

// q = n / d for 0 <= n < 2^24 (float reciprocal + one correction each way)
__device__ __forceinline__ int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  q += (q + 1) * d <= n ? 1 : 0;
  q -= q * d > n ? 1 : 0;
  return q;
}

// key of flat element e of image b, recomputed from the heatmap exactly as peak_scan / tile_select
// form it (fallback path)
__device__ uint64_t nms_key_global(const float* base, int64_t s1, int64_t s2, int64_t s3, int H, int W, uint32_t e) {
  const int hw = H * W;
  const int c = (int)(e / (uint32_t)hw);
  const int rem = (int)e - c * hw;
  const int y = rem / W, x = rem - (rem / W) * W;
  const float* pc = base + (int64_t)c * s1;
  const float v = sigmoidf_ref(pc[(int64_t)y * s2 + (int64_t)x * s3]);
  float m = v;
  for (int dy = -1; dy <= 1; ++dy)
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = y + dy, xx = x + dx;
      const float u = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? sigmoidf_ref(pc[(int64_t)yy * s2 + (int64_t)xx * s3])
                                                               : -INFINITY;
      m = fmaxf(m, u);
    }
  return make_key((float)(m == v) * v, e);
}

// The image's last-arriving scan workgroup: exact top K of its n appended positive keys (rank
// order = descending key) -> records (write_outputs). NT threads; NT == 256: one histogram bin
// per thread.
template <int NT>
__device__ void fused_select(const i32x4 krs, int n, int b, const float* __restrict__ heat,
                             int64_t s0, int64_t s1, int64_t s2, int64_t s3, int H, int W, int K, uint32_t N,
                             SelectShared& sh, char* lds, int* ncand, int* cnt_thr, const MergeOut& mo,
                             const DecodeParams& p, unsigned long long* stamps) {
  (void)stamps;
  static_assert(NT == 256, "one digit bin per thread");
  int P = 1;
  while (P < K) P <<= 1;
  uint64_t* top = reinterpret_cast<uint64_t*>(lds);  // P keys (fallback path)
  uint64_t* cand = top + (P < 2 ? 2 : P);             // <= max(K, kRankCap) candidates (+ a pad), 16-B aligned
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int KPT = 16;  // keys per thread when the image's keys fit in registers
  if (tid == 0) { *ncand = 0; *cnt_thr = 0; }
  if (n >= K) {
    const bool cached = n <= KPT * NT;
    uint64_t rk[KPT];
    if (cached) {
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const int i = tid + j * NT;
        rk[j] = i < n ? load_key(krs, i) : 0ull;
      }
    }
    // every key (wave-uniform calls): registers, or the array in global memory
    auto for_each_key = [&](auto&& f) __attribute__((always_inline)) {
      if (cached) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) f(rk[j], tid + j * NT < n);
      } else {
        for (int i0 = 0; i0 < n; i0 += NT) {
          const int i = i0 + tid;
          f(i < n ? load_key(krs, i) : 0ull, i < n);
        }
      }
    };
    const int cap = K > kRankCap ? K : kRankCap;
    uint64_t prefix = 0, pmask = 0;
    int need = K, above = 0;
    for (;;) {
      // the keys still in play share (key & pmask) == prefix: their range, then the 8-bit digit
      // just below the bits they all share
      uint64_t lo = ~0ull, hi = 0;
      int dummy = 0;
      for_each_key([&](uint64_t key, bool valid) {
        if (valid && (key & pmask) == prefix) {
          lo = key < lo ? key : lo;
          hi = key > hi ? key : hi;
        }
      });
      block_minmax_sum<NT>(lo, hi, dummy, sh);
      DSTAMP(stamps, 6);
      if (lo == hi) {  // one key in play (need == 1): it is the threshold
        prefix = hi;
        pmask = ~0ull;
        break;
      }
      const int msb = 63 - __builtin_clzll(lo ^ hi);
      const int shift = msb > 7 ? msb - 7 : 0;
      pmask |= shift + 8 >= 64 ? 0 : ~((1ull << (shift + 8)) - 1);
      prefix = hi & pmask;
      sh.hist[tid] = 0;
      __syncthreads();
      for_each_key([&](uint64_t key, bool valid) {
        const bool in = valid && (key & pmask) == prefix;
        hist_add(reinterpret_cast<uint32_t*>(sh.hist), in ? (uint32_t)(key >> shift) & 255u : 0u, in);
      });
      __syncthreads();
      // thread t owns digit 255 - t; running count from the top
      const int c = sh.hist[255 - tid];
      int incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
      }
      if (lane == 63) sh.red_n[wave] = incl;
      __syncthreads();
      int before = incl - c;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) before += i < wave ? sh.red_n[i] : 0;
      if (before < need && need <= before + c) {
        sh.sel_digit = 255 - tid;
        sh.sel_above = before;
        sh.sel_count = c;
      }
      __syncthreads();
      const int d = sh.sel_digit, a = sh.sel_above, bc = sh.sel_count;
      __syncthreads();
      prefix |= (uint64_t)d << shift;
      pmask |= 255ull << shift;
      need -= a;
      above += a;
      if (above + bc <= cap || shift == 0) break;
    }
    DSTAMP(stamps, 7);
    // candidates: every key at or above the threshold bucket (above + its count, <= cap)
    if (cached) {
      // wave counts -> wave offsets (one barrier), then ballot positions (ballots recomputed:
      // no 16 x 64-bit masks held across the barrier)
      int wc = 0;
#pragma unroll
      for (int j = 0; j < KPT; ++j) wc += (int)__popcll(__ballot(tid + j * NT < n && (rk[j] & pmask) >= prefix));
      if (lane == 0) sh.red_n[wave] = wc;
      __syncthreads();
      int pos = 0;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) pos += i < wave ? sh.red_n[i] : 0;
      if (tid == NT - 1) *ncand = pos + wc;
      const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const bool in = tid + j * NT < n && (rk[j] & pmask) >= prefix;
        const uint64_t bal = __ballot(in);
        if (in) cand[pos + (int)__popcll(bal & lt)] = rk[j];
        pos += (int)__popcll(bal);
      }
    } else {
      __syncthreads();  // (ncand zeroed)
      for_each_key([&](uint64_t key, bool valid) {
        const bool in = valid && (key & pmask) >= prefix;
        const int slot = wave_append_slot(ncand, in);
        if (in) cand[slot] = key;
      });
    }
    __syncthreads();
    DSTAMP(stamps, 8);
    const int m = *ncand;
    // each candidate's rank = the candidates above it (keys are unique); ranks below K write
    // their output slot directly
    int local_thr = 0;
    if (m <= NT) {
      // one owner thread per candidate: its record inputs gathered first (the loads run under
      // the ranking), its rank from 16-byte LDS reads (two keys each; an odd count padded with a
      // zero key, below every real one)
      if (tid == 0 && (m & 1)) cand[m] = 0;
      const uint64_t mykey = tid < m ? cand[tid] : 0;
      const RecIn in = tid < m && mo.records ? gather_record(mykey, b, p) : RecIn{};
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (the pad key)
      int r = 0;
      const int m2 = (m + 1) >> 1;
      const ulonglong2* c2 = reinterpret_cast<const ulonglong2*>(cand);
#pragma unroll 8
      for (int j = 0; j < m2; ++j) {
        const ulonglong2 v = c2[j];
        r += (v.x > mykey ? 1 : 0) + (v.y > mykey ? 1 : 0);
      }
      if (tid < m && r < K) local_thr += store_record(mykey, in, r, K, b, mo, p);
    } else {
      for (int ci = tid; ci < m; ci += NT) {
        const uint64_t mykey = cand[ci];
        int r = 0;
#pragma unroll 8
        for (int j = 0; j < m; ++j) r += cand[j] > mykey ? 1 : 0;
        if (r < K) local_thr += write_record(mykey, r, K, b, mo, p);
      }
    }
    DSTAMP(stamps, 9);
    if (mo.records) {
      if (local_thr) atomicAdd(cnt_thr, local_thr);
      // (a raw barrier: __syncthreads()'s fence would wait for every record store)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) p.counts[b] = *cnt_thr;
    }
  } else {
    // fewer positive keys than K: exact streaming select over every key of the image (the top
    // so far rides along in CARRY slots per thread: kMaxK keys over NT threads)
    constexpr int CARRY = (kMaxK + NT - 1) / NT, PER = 12 + CARRY, CH = 12 * NT;
    const float* base = heat + b * s0;
    int have = 0;
    for (uint32_t e0 = 0; e0 < N; e0 += CH) {
      uint64_t k[PER];
      int loc = 0;
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const uint32_t e = e0 + tid + j * NT;
        k[j] = e < N ? nms_key_global(base, s1, s2, s3, H, W, e) : 0;
        loc += k[j] != 0;
      }
#pragma unroll
      for (int j = 0; j < CARRY; ++j) {
        const int i = tid + j * NT;
        k[12 + j] = i < have ? top[i] : 0;
        loc += k[12 + j] != 0;
      }
      const int real = block_count_real<NT>(loc, sh);
      const int kt = min(K, real);
      const uint64_t T2 = block_select<NT, PER>(k, kt, sh);
      if (tid == 0) sh.nout = 0;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if (k[j] != 0 && k[j] >= T2) top[atomicAdd(&sh.nout, 1)] = k[j];
      __syncthreads();
      have = kt;
    }
    for (int i = have + tid; i < P; i += NT) top[i] = 0;
    __syncthreads();
    bitonic_desc<NT>(top, P);
    write_outputs<NT>(top, K, b, mo, p, *cnt_thr);
  }
  DSTAMP(stamps, 10);
#if defined(TV_DEC_STAMPS)
  if (threadIdx.x == 0)
    for (int i = 1; i <= 10; ++i)
      p.records[((size_t)b * K + K - 2) * 10 + (i - 1)] = (float)(long long)(stamps[i] - stamps[0]);
#endif
}

// Tile element (cc, yy, xx) at image (c0 + cc, y0 + yy, x0 + xx); per-image offsets fit 32 bits
// (launch_decode checks). CHAN_FAST: LDS fill order channel-fastest (1: NHWC views, whose
// channels of a pixel are adjacent; 2: the same with 4 unit-stride 16-byte-aligned channels,
// one float4 per pixel) or column-fastest (0: NCHW).
template <int CHAN_FAST>
// (5 workgroups per CU: <= 96 VGPRs, and the LDS of the R18 head tile fits 5 x 32 KiB)
__global__ __launch_bounds__(kScanThreads) __attribute__((amdgpu_waves_per_eu(5, 8))) void peak_scan(const float* __restrict__ heat, int64_t s0, int s1, int s2,
                                                           int s3, int C, int H, int W, int K, const TileGeom g,
                                                           const ScanWs w, const MergeOut mo, const DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  __shared__ uint32_t wsum[kScanThreads / 64 + 1];
  __shared__ int red_n[kScanThreads / 64];
  __shared__ int keep_digit;
  __shared__ uint32_t keep_cnt, seg_base, last_flag;
  __shared__ SelectShared ssh;
  __shared__ int ncand, cnt_thr;
  uint32_t* fhist = reinterpret_cast<uint32_t*>(ssh.hist);  // (the select's histogram, later)
#if defined(TV_DEC_STAMPS)
  __shared__ unsigned long long stamps[12];
#else
  unsigned long long* stamps = nullptr;
#endif
  DSTAMP(stamps, 0);
  const int b = blockIdx.y;
  int t = blockIdx.x;
  const int tx = t % g.ntw; t /= g.ntw;
  const int ty = t % g.nth;
  const int tc = t / g.nth;
  const int c0 = tc * g.cg, y0 = ty * g.th, x0 = tx * g.tw;
  const int nc = min(g.cg, C - c0), nh = min(g.th, H - y0), nw = min(g.tw, W - x0);
  const int LH = nh + 2, LW = nw + 2;
  const int LP = ((LW + 3) & ~3) + 4;  // LDS row pitch (floats): 16-byte rows, room for the last strip's window
  fhist[threadIdx.x] = 0;
  static_assert(kScanThreads == 256, "one filter-histogram bin per thread");
  const float* base = heat + b * s0 + c0 * s1;

  // tile + halo -> LDS [cc][yy][xx], sigmoid once per element, outside the image -inf
  const int nl = nc * LH * LW;
  const float inv_nc = 1.0f / (float)nc, inv_lw = 1.0f / (float)LW, inv_lh = 1.0f / (float)LH;
  constexpr int kFillBatch = 8;
  if (CHAN_FAST == 2) {
    // NHWC view, 4 channels per tile, unit channel stride, 16-byte aligned pixels: one float4
    // load per pixel
    const int np = LH * LW;
    for (int p0 = 0; p0 < np; p0 += kScanThreads * kFillBatch) {
      float4 v[kFillBatch];
      int pix[kFillBatch];
      bool inb[kFillBatch];
#pragma unroll
      for (int j = 0; j < kFillBatch; ++j) {
        const int pp = p0 + j * kScanThreads + threadIdx.x;
        const int yy = fdiv(pp, LW, inv_lw);
        const int xx = pp - yy * LW;
        const int y = y0 + yy - 1, x = x0 + xx - 1;
        const bool in = pp < np && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        inb[j] = in;
        v[j] = in ? *reinterpret_cast<const float4*>(base + y * s2 + x * s3) : make_float4(0.f, 0.f, 0.f, 0.f);
        pix[j] = pp < np ? yy * LP + xx : -1;
      }
#pragma unroll
      for (int j = 0; j < kFillBatch; ++j) {
        if (pix[j] < 0) continue;
        const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) tile[cc * LH * LP + pix[j]] = inb[j] ? sigmoidf_ref(e[cc]) : -INFINITY;
      }
    }
  } else
  for (int e0 = 0; e0 < nl; e0 += kScanThreads * kFillBatch) {
    float v[kFillBatch];
    int dst[kFillBatch];
    bool inb[kFillBatch];
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j) {
      const int e = e0 + j * kScanThreads + threadIdx.x;
      int cc, yy, xx;
      if constexpr (CHAN_FAST != 0) {
        const int p = fdiv(e, nc, inv_nc);
        cc = e - p * nc;
        yy = fdiv(p, LW, inv_lw);
        xx = p - yy * LW;
      } else {
        const int p = fdiv(e, LW, inv_lw);
        xx = e - p * LW;
        cc = fdiv(p, LH, inv_lh);
        yy = p - cc * LH;
      }
      const int y = y0 + yy - 1, x = x0 + xx - 1;
      const bool in = e < nl && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      inb[j] = in;
      v[j] = in ? base[cc * s1 + y * s2 + x * s3] : 0.f;
      dst[j] = e < nl ? (cc * LH + yy) * LP + xx : -1;
    }
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j)
      if (dst[j] >= 0) tile[dst[j]] = inb[j] ? sigmoidf_ref(v[j]) : -INFINITY;
  }
  __syncthreads();
  DSTAMP(stamps, 1);

  // NMS keys over strips of 4 columns (strip q = tid + j * NT: column-strip fastest, then row,
  // then channel): the 3 x 6 window is read once per strip; per element the same fmaxf order
  // as tile_select / nms_key_global (centre first, then rows top-down, columns left-right)
  const int nsx = (nw + 3) >> 2;
  const int nq = nc * nh * nsx;
  const float inv_nsx = 1.0f / (float)nsx, inv_nh = 1.0f / (float)nh;
  uint64_t k[kScanPer];
  uint32_t mine = 0;
#pragma unroll
  for (int j = 0; j < kScanPer / 4; ++j) {
    const int q = threadIdx.x + j * kScanThreads;
    const bool qv = q < nq;
    const int p = fdiv(qv ? q : 0, nsx, inv_nsx);
    const int xs = (qv ? q : 0) - p * nsx;
    const int cc = fdiv(p, nh, inv_nh);
    const int yy = p - cc * nh;
    const int xb = 4 * xs;
    // window rows yy .. yy + 2, columns xb .. xb + 5 (16 + 8 bytes per row; columns past LW only
    // reach the masked elements of a partial strip)
    const float* r0 = tile + (cc * LH + yy) * LP + xb;
    float win[3][6];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const float4 a4 = *reinterpret_cast<const float4*>(r0 + r * LP);
      const float2 a2 = *reinterpret_cast<const float2*>(r0 + r * LP + 4);
      win[r][0] = a4.x; win[r][1] = a4.y; win[r][2] = a4.z; win[r][3] = a4.w;
      win[r][4] = a2.x; win[r][5] = a2.y;
    }
    const uint32_t flat0 = (uint32_t)(((c0 + cc) * H + y0 + yy) * W + x0 + xb);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = win[1][i + 1];
      float m = v;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) m = fmaxf(m, win[r][i + c]);
      const float pv = (float)(m == v) * v;  // (hmax == h).float() * h (decode.py:252)
      const uint64_t key = make_key(pv, flat0 + i);
      const bool keep = qv && xb + i < nw && key > kZeroKey;
      k[4 * j + i] = keep ? key : 0;
      mine += keep ? 1u : 0u;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // compact the tile's positive keys into LDS (over the tile's sigmoid values: the NMS is done)
  uint64_t* list = reinterpret_cast<uint64_t*>(tile);
  uint32_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();  // every wave is past its window reads: the tile LDS may be overwritten
  uint32_t off = 0, nk = 0;
#pragma unroll
  for (int i = 0; i < kScanThreads / 64; ++i) {
    off += i < wave ? wsum[i] : 0u;
    nk += wsum[i];
  }
  {
    uint64_t* d = list + off + (incl - mine);
#pragma unroll
    for (int j = 0; j < kScanPer; ++j)
      if (k[j]) *d++ = k[j];
  }
  __syncthreads();
  DSTAMP(stamps, 2);
  // per-tile pre-filter: every key of the image's top K is among its tile's top K, so when the
  // tile has more than K keep only those whose 8-bit score digit (just below the score bits all
  // the tile's keys share) reaches the digit of the tile's K-th largest — K plus at most one
  // digit's worth instead of every peak. Ties in score share a digit, so they stay together.
  uint32_t kd = 0;
  int sh = 0;
  if ((int)nk > K) {  // uniform
    uint32_t lo = ~0u, hi = 0;
    for (uint32_t i = threadIdx.x; i < nk; i += kScanThreads) {
      const uint32_t sc = (uint32_t)(list[i] >> 32);
      lo = sc < lo ? sc : lo;
      hi = sc > hi ? sc : hi;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t l = (uint32_t)__shfl_xor((int)lo, o), h = (uint32_t)__shfl_xor((int)hi, o);
      lo = l < lo ? l : lo;
      hi = h > hi ? h : hi;
    }
    if (lane == 0) { red_n[wave] = (int)lo; wsum[wave] = hi; }
    __syncthreads();
    lo = ~0u; hi = 0;
#pragma unroll
    for (int i = 0; i < kScanThreads / 64; ++i) {
      lo = (uint32_t)red_n[i] < lo ? (uint32_t)red_n[i] : lo;
      hi = wsum[i] > hi ? wsum[i] : hi;
    }
    const uint32_t diff = lo ^ hi;
    if (diff) {
      const int msb = 31 - __builtin_clz(diff);
      sh = msb > 7 ? msb - 7 : 0;
      for (uint32_t i0 = 0; i0 < nk; i0 += kScanThreads) {
        const uint32_t i = i0 + threadIdx.x;
        hist_add(fhist, i < nk ? (uint32_t)(list[i] >> (32 + sh)) & 255u : 0u, i < nk);
      }
      __syncthreads();
      // thread t owns digit 255 - t; running count from the top
      const int c = (int)fhist[255 - threadIdx.x];
      int inc2 = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(inc2, o);
        if (lane >= o) inc2 += u;
      }
      __syncthreads();  // the min / max slots are read: reuse red_n for the wave totals
      if (lane == 63) red_n[wave] = inc2;
      __syncthreads();
      int before = inc2 - c;
#pragma unroll
      for (int i = 0; i < kScanThreads / 64; ++i) before += i < wave ? red_n[i] : 0;
      if (before < K && K <= before + c) {
        keep_digit = 255 - (int)threadIdx.x;
        keep_cnt = (uint32_t)(before + c);  // the keys whose digit reaches it
      }
      __syncthreads();
      kd = (uint32_t)keep_digit;
    }
  }
  DSTAMP(stamps, 3);
  // the kept keys -> the image's key array at a base drawn with one atomic (ballot positions),
  // write-through stores (read by whichever workgroup of the image finishes last)
  if (threadIdx.x == 0) {
    const uint32_t kept = kd ? keep_cnt : nk;
    seg_base = kept ? __hip_atomic_fetch_add((gu32*)(w.img_cnt + 2 * b), kept, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : 0u;
  }
  __syncthreads();
  const i32x4 krs = keys_rsrc(w, b);
  uint32_t pos = seg_base;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t i0 = 0; i0 < nk; i0 += kScanThreads) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t key = i < nk ? list[i] : 0;
    const bool keep = i < nk && ((uint32_t)(key >> (32 + sh)) & 255u) >= kd;
    const uint64_t bal = __ballot(keep);
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t wo = 0, tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < kScanThreads / 64; ++w2) {
      wo += w2 < wave ? wsum[w2] : 0u;
      tot += wsum[w2];
    }
    if (keep)
      raw_buffer_store_v2(u32x2{(uint32_t)key, (uint32_t)(key >> 32)}, krs,
                          (int)((pos + wo + (uint32_t)__popcll(bal & lt)) * 8u), 0, kSC1);
    pos += tot;
    // (raw barriers: the stores drain once, at the hand-off below)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // hand-off (cdna_hip_programming.md §6 Guideline 16, write-through form): every storing wave
  // drains its stores, the barrier orders them before ONE relaxed agent-scope ticket; the
  // workgroup drawing the image's last ticket selects from sc1 loads and resets the count and
  // the ticket for the next call
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DSTAMP(stamps, 4);
  if (threadIdx.x == 0)
    last_flag = __hip_atomic_fetch_add((gu32*)(w.ticket + 2 * b), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (last_flag != (uint32_t)(w.tiles - 1)) return;  // workgroup-uniform
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: every key load below is sc1
  if (threadIdx.x == 0) seg_base = __hip_atomic_load((gu32*)(w.img_cnt + 2 * b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int n = (int)seg_base;
  if (threadIdx.x == 0) {
    __hip_atomic_store((gu32*)(w.img_cnt + 2 * b), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32*)(w.ticket + 2 * b), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  DSTAMP(stamps, 5);
  fused_select<kScanThreads>(krs, n, b, heat, s0, s1, s2, s3, H, W, K, w.N, ssh, reinterpret_cast<char*>(tile), &ncand,
                             &cnt_thr, mo, p, stamps);
}

// ---- host side --------------------------------------------------------------------------
namespace {

TileGeom tile_geom(int C, int H, int W, int r, int apply_sigmoid, int chan_fast) {
  TileGeom g{};
  g.tw = std::min(W, 512);
  g.cg = std::min(C, std::max(1, kTileElems / (g.tw * 4)));
  g.th = std::min(H, std::max(1, kTileElems / (g.tw * g.cg)));
  g.ncg = (C + g.cg - 1) / g.cg;
  g.nth = (H + g.th - 1) / g.th;
  g.ntw = (W + g.tw - 1) / g.tw;
  g.r = r;
  g.apply_sigmoid = apply_sigmoid;
  g.chan_fast = chan_fast;
  return g;
}

size_t tile_lds(const TileGeom& g) { return (size_t)g.cg * (g.th + 2 * g.r) * (g.tw + 2 * g.r) * sizeof(float); }

// merge levels: lists per image at each level (level 0 = tiles)
std::vector<int> merge_levels(int tiles, int K) {
  const int group = std::max(1, kMergeCap / K);
  std::vector<int> lv{tiles};
  while (lv.back() > group) lv.push_back((lv.back() + group - 1) / group);
  return lv;
}

}  // namespace

size_t select_workspace_bytes(int B, int C, int H, int W, int K) {
  const TileGeom g = tile_geom(C, H, W, 1, 1, 1);
  const int tiles = g.ncg * g.nth * g.ntw;
  const std::vector<int> lv = merge_levels(tiles, K);
  // level i reads buffer i & 1 and writes buffer (i + 1) & 1; list counts only shrink, so
  // buffer 0 is sized by level 0 and buffer 1 by level 1
  const size_t b0 = (size_t)B * lv[0] * K * 8, b1 = lv.size() > 1 ? (size_t)B * lv[1] * K * 8 : 0;
  return (b0 + 255) / 256 * 256 + (b1 + 255) / 256 * 256;
}

int launch_select(const float* heat, const int64_t st[4], int B, int C, int H, int W, int nms, int apply_sigmoid,
                  int K, void* ws, size_t ws_bytes, float* score, int32_t* index, const DecodeParams* rec,
                  hipStream_t s) {
  const int64_t n = (int64_t)C * H * W;
  if (K < 1 || K > kMaxK || K > n) { set_error("topk: need 1 <= K <= min(1024, C*H*W)"); return 1; }
  if (n >= (int64_t)0xFFFFFFFF) { set_error("topk: image too large"); return 1; }
  if (B == 0) return 0;
  const TileGeom g = tile_geom(C, H, W, nms ? 1 : 0, apply_sigmoid, st[1] < st[3] ? 1 : 0);
  const int tiles = g.ncg * g.nth * g.ntw;
  const std::vector<int> lv = merge_levels(tiles, K);
  if (ws_bytes < select_workspace_bytes(B, C, H, W, K)) { set_error("decode workspace too small"); return 1; }
  if (tiles > 65535 || B > 65535) { set_error("decode: grid too large"); return 1; }
  const size_t lds = tile_lds(g);
  uint64_t* buf[2] = {(uint64_t*)ws, (uint64_t*)((char*)ws + ((size_t)B * lv[0] * K * 8 + 255) / 256 * 256)};
  hipLaunchKernelGGL(tile_select, dim3(tiles, B), dim3(kTileThreads), lds, s, heat, st[0], st[1], st[2], st[3], C, H,
                     W, g, K, buf[0]);
  TV_HIP(hipGetLastError());
  const int group = std::max(1, kMergeCap / K);
  MergeOut mo{score, index, rec ? 1 : 0};
  DecodeParams p = rec ? *rec : DecodeParams{};
  for (size_t i = 0; i < lv.size(); ++i) {
    const int lists = lv[i];
    const int groups = (lists + group - 1) / group;
    const int fin = groups == 1;
    uint64_t* in = buf[i & 1];
    uint64_t* nxt = buf[(i + 1) & 1];
    if (fin && lists * K <= kSmallMergeCap)
      hipLaunchKernelGGL((merge_select<kSmallMergeThreads, kSmallMergePer>), dim3(groups, B), dim3(kSmallMergeThreads), 0,
                         s, in, lists, group, K, nxt, fin, mo, p);
    else
      hipLaunchKernelGGL((merge_select<kMergeThreads, kMergePer>), dim3(groups, B), dim3(kMergeThreads), 0, s, in, lists,
                         group, K, nxt, fin, mo, p);
    TV_HIP(hipGetLastError());
    if (fin) break;
  }
  return 0;
}

namespace {
TileGeom scan_geom(int C, int H, int W, int chan_fast) {
  TileGeom g{};
  g.tw = std::min(W, 512);
  g.cg = std::min(C, std::max(1, kScanElems / (g.tw * 4)));
  // at most 4 strips of 4 columns per thread (peak_scan's kScanPer keys)
  g.th = std::min(H, std::max(1, (kScanElems / 4) / (g.cg * ((g.tw + 3) / 4))));
  g.ncg = (C + g.cg - 1) / g.cg;
  g.nth = (H + g.th - 1) / g.th;
  g.ntw = (W + g.tw - 1) / g.tw;
  g.r = 1;
  g.apply_sigmoid = 1;
  g.chan_fast = chan_fast;
  return g;
}
}  // namespace

// Head: per image b a key count (word 2b) and a ticket (word 2b + 1) at a FIXED offset for every
// image a launch can take (B <= 65535), so the counters never move with B or the heatmap geometry
// and no call's keys land on them: a workspace zero-filled once stays valid for any later call
// that fits it (each call leaves every counter it used at zero). Then [B][tiles][kScanElems] keys.
constexpr int kMaxDecodeB = 65535;
size_t decode_head_bytes(int B) {
  (void)B;
  return (size_t)(kMaxDecodeB + 1) * 8;
}
size_t decode_workspace_bytes(int B, int C, int H, int W, int K) {
  (void)K;
  const TileGeom g = scan_geom(C, H, W, 1);
  const size_t T = (size_t)g.ncg * g.nth * g.ntw;
  return decode_head_bytes(B) + (size_t)B * T * kScanElems * 8;
}

int launch_decode(const float* heat, const int64_t st[4], int B, int C, int H, int W, int K, void* ws,
                  size_t ws_bytes, const DecodeParams& rec, hipStream_t s) {
  const int64_t n = (int64_t)C * H * W;
  if (K < 1 || K > kMaxK || K > n) { set_error("decode: need 1 <= K <= min(1024, C*H*W)"); return 1; }
  if (n >= (int64_t)0xFFFFFFFF) { set_error("decode: image too large"); return 1; }
  if (B == 0) return 0;
  if (ws_bytes < decode_workspace_bytes(B, C, H, W, K)) { set_error("decode workspace too small"); return 1; }
  const TileGeom g = scan_geom(C, H, W, st[1] < st[3] ? 1 : 0);
  const int tiles = g.ncg * g.nth * g.ntw;
  if (tiles > kMaxScanTiles || B > kMaxDecodeB) { set_error("decode: heatmap too large (tiles per image)"); return 1; }
  // the tile (+ halo) in fp32, later reused for the tile's compacted keys (at most one per tile
  // element) and the select's lists (top: K rounded up to a power of two; candidates)
  int P = 1;
  while (P < K) P <<= 1;
  const size_t lds = std::max({(size_t)g.cg * (g.th + 2) * ((((g.tw + 2) + 3) & ~3) + 4) * sizeof(float),
                               (size_t)g.cg * g.th * g.tw * sizeof(uint64_t),
                               (size_t)(std::max(P, 2) + std::max(K, kRankCap) + 2) * sizeof(uint64_t)});
  ScanWs w;
  w.img_cnt = (uint32_t*)ws;  // image b: img_cnt[2b], ticket[2b] (stride 2: decode_head_bytes)
  w.ticket = w.img_cnt + 1;
  w.keys = (uint64_t*)((char*)ws + decode_head_bytes(B));
  w.tiles = tiles;
  w.N = (uint32_t)n;
  // per-image element offsets in 32 bits
  const int64_t span = (int64_t)(C - 1) * st[1] + (int64_t)(H - 1) * st[2] + (int64_t)(W - 1) * st[3];
  if (st[1] < 0 || st[2] < 0 || st[3] < 0 || span >= (int64_t)0x7FFFFFFF) {
    set_error("decode: heatmap view strides out of range");
    return 1;
  }
  const bool vec4 = g.chan_fast && st[1] == 1 && C == 4 && g.cg == 4 && st[3] % 4 == 0 && st[2] % 4 == 0 &&
                    st[0] % 4 == 0 && ((uintptr_t)heat & 15) == 0;
  const MergeOut mo{nullptr, nullptr, 1};
  if (vec4)
    hipLaunchKernelGGL(peak_scan<2>, dim3(tiles, B), dim3(kScanThreads), lds, s, heat, st[0], (int)st[1], (int)st[2],
                       (int)st[3], C, H, W, K, g, w, mo, rec);
  else if (g.chan_fast)
    hipLaunchKernelGGL(peak_scan<1>, dim3(tiles, B), dim3(kScanThreads), lds, s, heat, st[0], (int)st[1], (int)st[2],
                       (int)st[3], C, H, W, K, g, w, mo, rec);
  else
    hipLaunchKernelGGL(peak_scan<0>, dim3(tiles, B), dim3(kScanThreads), lds, s, heat, st[0], (int)st[1], (int)st[2],
                       (int)st[3], C, H, W, K, g, w, mo, rec);
  TV_HIP(hipGetLastError());
  return 0;
}

// heatmap_detect on a dense [B, n] map: C = 1, H = 1, W = n, no NMS, no sigmoid
int launch_topk(const float* peaks, int B, int64_t n, int K, float* score, int32_t* index, hipStream_t s) {
  if (n < 1 || n >= (int64_t)0x7FFFFFFF) { set_error("topk: bad row length"); return 1; }
  const size_t need = select_workspace_bytes(B, 1, 1, (int)n, K);
  void* ws = nullptr;
  TV_HIP(hipMallocAsync(&ws, std::max<size_t>(need, 256), s));
  const int64_t st[4] = {n, 0, 0, 1};
  int rc = launch_select(peaks, st, B, 1, 1, (int)n, 0, 0, K, ws, need, score, index, nullptr, s);
  TV_HIP(hipFreeAsync(ws, s));
  return rc;
}

// ---- heatmap_detect()'s (index, label) as int64 ---------------------------------------------
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
