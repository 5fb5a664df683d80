// Narrow-channel 3x3 convolution (gfx950, fp16 / bf16): the full-resolution DLA-34 base levels
// (centerpoint_dla.py:242-246 `_make_conv_level`: level0 3x3 16 -> 16 at 480x640, level1 3x3 s2
// 16 -> 32, level2's first BasicBlock conv 32 -> 64 s2), conv + BN (folded) + ReLU.
//
// Why a kernel of its own: with 16-32 channels these layers move 32-64 B per pixel and do
// ~5-20 kFLOP per pixel — HBM-bound (the input row is re-read 9x, but from L1/L2). The implicit
// GEMMs tile them as 256 pixels x 128 channels, so 7/8 of every MFMA tile is padding and the
// K = 144 loop is mostly pipeline fill (level0 ran 1.3 ms per 32 frames, 34 TFLOP/s).
//
// Design: v_mfma_f32_16x16x32_{f16,bf16} with A = weights (16 output channels x 32 of K), B = 16
// output pixels of one row (32 of K x 16), C = 16 channels x 16 pixels: lane l holds channels
// 4(l>>4) .. +3 of pixel l&15, i.e. 8 contiguous output bytes, and the 4 lane groups of a pixel
// cover its 16 channels (32 B). K = tap * CIN + channel, in slabs of 32: a lane's 8 K values are
// 8 consecutive channels of one tap of one input pixel — one 16-byte global load straight from
// the NHWC input (zero for the padding taps), no LDS. All weights live in registers for the
// whole kernel (NS x COUT/16 fragments); each wave streams 16-pixel row segments, the loads of the
// next segment issued before the current segment's MFMAs and stores.
//
// That register-gather kernel is variant 0 (knob TV_CSM_HALO=0); since round 5 the engine runs the
// LDS-halo variant below (same MFMA sequence, bit-identical results) on a persistent grid.
#include "conv_common.h"

namespace tv {
namespace csm {

template <typename T> struct M16;
template <> struct M16<_Float16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0,
                                                 0, 0);
  }
};
template <> struct M16<__bf16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
  }
};

constexpr int NT = 256;  // 4 waves

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

template <typename T, int CIN, int COUT, int STRIDE, int ACT>
__global__ __launch_bounds__(NT) void conv_small(const ConvParams* __restrict__ pp) {
  constexpr int NS = (9 * CIN + 31) / 32;  // K slabs of 32
  constexpr int NB = COUT / 16;            // 16-channel output blocks
  const ConvParams& p = *pp;
  const ConvSegment& sg = p.seg[0];
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, px = lane & 15;
  const int H = sg.H, W = sg.W, ldc = sg.ldc;
  const int Ho = p.Ho, Wo = p.Wo;
  const int segs = (Wo + 15) / 16;                 // 16-pixel segments per output row
  const int total = p.M / Wo * segs;               // (frame, output row) x segments
  const int wave_g = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * (NT / 64);

  // weights: A[row = 16 ob + px][k = 32 s + 8 g .. + 7] (zero past K = 9 CIN); bias of this
  // lane's 4 output channels per block
  uint4 wa[NB][NS];
  f32x4 bias[NB];
#pragma unroll
  for (int ob = 0; ob < NB; ++ob) {
    const T* wr = reinterpret_cast<const T*>(p.weight) + (size_t)(16 * ob + px) * p.Kpad;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k0 = 32 * s + 8 * g;
      wa[ob][s] = k0 < 9 * CIN ? gload16(wr + k0) : make_uint4(0, 0, 0, 0);
    }
    const int c0 = 16 * ob + 4 * g;
    bias[ob] = f32x4{p.bias[c0], p.bias[c0 + 1], p.bias[c0 + 2], p.bias[c0 + 3]};
  }

  // this lane's K slice of slab s: tap and first channel
  auto load_b = [&](int item, uint4 (&b)[NS]) __attribute__((always_inline)) {
    const int seg = item % segs;
    const int row = item / segs;        // b * Ho + oy
    const int fr = row / Ho, oy = row - fr * Ho;
    const int ox = seg * 16 + px;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k0 = 32 * s + 8 * g;
      const int tap = k0 / CIN, c0 = k0 - tap * CIN;
      const int iy = oy * STRIDE + tap / 3 - 1, ix = ox * STRIDE + tap % 3 - 1;
      const bool ok = item < total && tap < 9 && ox < Wo && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const T* src = reinterpret_cast<const T*>(sg.src) + ((size_t)(fr * H + iy) * W + ix) * ldc + c0;
      b[s] = ok ? gload16(src) : make_uint4(0, 0, 0, 0);
    }
  };

  uint4 b0[NS], b1[NS];
  int item = wave_g;
  if (item >= total) return;
  load_b(item, b0);
  auto step = [&](int it, const uint4 (&b)[NS]) __attribute__((always_inline)) {
    f32x4 acc[NB];
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) {
      acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) M16<T>::run(wa[ob][s], b[s], acc[ob]);
    }
    const int seg = it % segs;
    const int row = it / segs;
    const int ox = seg * 16 + px;
    if (ox >= Wo) return;
    T* dst = reinterpret_cast<T*>(p.out) + ((size_t)row * Wo + ox) * p.out_ldc + p.out_coff;
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = acc[ob][r] + bias[ob][r];
        if constexpr (ACT == 1) t = fmaxf(t, 0.0f);
        else if constexpr (ACT == 2) t = fmaxf(t, 0.01f * t);
        v[r] = t;
      }
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(dst + 16 * ob + 4 * g) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
    }
  };
  // two register sets: the next item's operands are in flight under this item's MFMAs and stores
  for (;;) {
    const int n1 = item + nwaves;
    if (n1 < total) load_b(n1, b1);
    step(item, b0);
    if (n1 >= total) break;
    const int n2 = n1 + nwaves;
    if (n2 < total) load_b(n2, b0);
    step(n1, b1);
    if (n2 >= total) break;
    item = n2;
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-halo variant (round 5): the register-gather kernel above reads every input chunk 9 times
// (once per tap) through the vector L1 with only two 16-pixel segments in flight per wave, and
// ran level0 (16 -> 16 at 480x640) at ~2.6 TB/s of HBM bytes. Here one workgroup owns a tile of
// TR output rows x TW output columns of one frame: its input halo ((TR-1)S+3 rows x (TW-1)S+3
// columns, all CIN channels) comes in once by LDS-DMA (1 KiB per wave instruction, zeros outside
// the frame from the buffer's range check), then the B operands are ds_read_b128 from LDS. The
// tile is small (24-40 KiB), so several workgroups per CU overlap one's staging with another's
// MFMAs; no double buffering. On a persistent grid (variant 2) each workgroup keeps its weight
// fragments in registers across the tiles of its XCD-contiguous range (variant 1: a tile per
// workgroup, every one reloading the weights).
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ void raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size, int voffset,
                                    int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ __forceinline__ i32x4 rsrc_of(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = (int)(unsigned)a;
  r.y = (int)(unsigned)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}
typedef const __attribute__((address_space(3))) u32x4 lds_u32x4;
constexpr int OOB = (int)0x80000000u;

template <int CIN, int STRIDE, int TW, int TR> struct HaloGeo {
  static constexpr int CPP = CIN / 8;                 // 16-byte chunks per input pixel
  static constexpr int HCOLS = (TW - 1) * STRIDE + 3;
  static constexpr int HROWS = (TR - 1) * STRIDE + 3;
  static constexpr int CHUNKS = HROWS * HCOLS * CPP;
  static constexpr int PPW = ((CHUNKS + 63) / 64 + 3) / 4;  // 1 KiB pieces per wave
  static constexpr int LDS = PPW * 4 * 1024;
  static constexpr int SEGS = TW / 16;
  static constexpr int ITEMS = TR * SEGS;               // 16-pixel row segments per tile
  static_assert(TW % 16 == 0 && ITEMS % 4 == 0, "tile shape");
  static_assert(LDS <= 64 * 1024, "halo tile");
};

template <typename T, int CIN, int COUT, int STRIDE, int TW, int TR, int ACT>
__global__ __launch_bounds__(NT) void conv_small_halo(const ConvParams* __restrict__ pp) {
  using G = HaloGeo<CIN, STRIDE, TW, TR>;
  constexpr int NS = (9 * CIN + 31) / 32;
  constexpr int NB = COUT / 16;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* lds = (lds_char*)smem;
  const ConvParams& p = *pp;
  const ConvSegment& sg = p.seg[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, px = lane & 15;
  const int H = sg.H, W = sg.W, ldc = sg.ldc;
  const int Ho = p.Ho, Wo = p.Wo;
  const int tiles_x = (Wo + TW - 1) / TW, tiles_y = (Ho + TR - 1) / TR;
  const int ntiles = p.M / (Ho * Wo) * tiles_y * tiles_x;
  // XCD-aware: workgroup b runs on XCD b % 8, so each XCD walks a contiguous tile range (shared
  // halo rows in its L2); one tile per workgroup when the grid is the tile count, else persistent
  const int nb = gridDim.x, bid = blockIdx.x;
  int first, end, step;
  if ((nb & 7) == 0) {
    first = (int)((long long)ntiles * (bid & 7) / 8) + (bid >> 3);
    end = (int)((long long)ntiles * ((bid & 7) + 1) / 8);
    step = nb >> 3;
  } else {
    first = bid;
    end = ntiles;
    step = nb;
  }
  const unsigned frame_bytes = (unsigned)H * W * ldc * (unsigned)sizeof(T);
  // stage tile t's halo: chunk q*64 + lane of the tile, pixel-major, CPP chunks per pixel
  auto stage = [&](int t) __attribute__((always_inline)) {
    const int tx = t % tiles_x, fy = t / tiles_x;
    const int ty = fy % tiles_y, fr = fy / tiles_y;
    const int iy0 = ty * TR * STRIDE - 1, ix0 = tx * TW * STRIDE - 1;
    const i32x4 rs = rsrc_of(reinterpret_cast<const char*>(sg.src) + (size_t)fr * frame_bytes, frame_bytes);
#pragma unroll
    for (int k = 0; k < G::PPW; ++k) {
      const int q = wave * G::PPW + k;
      const int ch = q * 64 + lane;
      const int h = ch / G::CPP, c = ch - h * G::CPP;
      const int hy = h / G::HCOLS, hx = h - hy * G::HCOLS;
      const int y = iy0 + hy, x = ix0 + hx;
      const bool ok = ch < G::CHUNKS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      raw_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + q * 1024), 16,
                          ok ? (int)((((unsigned)y * W + x) * ldc + c * 8) * sizeof(T)) : OOB, 0, 0, 0);
    }
  };
  if (first >= end) return;
  stage(first);
  // weights (A fragments) and biases into registers under the first staging, once per workgroup
  uint4 wa[NB][NS];
  f32x4 bias[NB];
#pragma unroll
  for (int ob = 0; ob < NB; ++ob) {
    const T* wr = reinterpret_cast<const T*>(p.weight) + (size_t)(16 * ob + px) * p.Kpad;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k0 = 32 * s + 8 * g;
      wa[ob][s] = k0 < 9 * CIN ? gload16(wr + k0) : make_uint4(0, 0, 0, 0);
    }
    const int c0 = 16 * ob + 4 * g;
    bias[ob] = f32x4{p.bias[c0], p.bias[c0 + 1], p.bias[c0 + 2], p.bias[c0 + 3]};
  }
  // this lane's LDS offset of slab s relative to the segment's first halo pixel (tap (dy, dx),
  // chunk c); -1 past K = 9 CIN (zero operand)
  int toff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k0 = 32 * s + 8 * g;
    const int tap = k0 / CIN, c = (k0 - tap * CIN) / 8;
    toff[s] = tap < 9 ? (((tap / 3) * G::HCOLS + tap % 3) * G::CPP + c) * 16 : -1;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  for (int t = first;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int tx = t % tiles_x, fy = t / tiles_x;
    const int ty = fy % tiles_y, fr = fy / tiles_y;
    const int oy0 = ty * TR, ox0 = tx * TW;
#pragma unroll
    for (int j = 0; j < G::ITEMS / 4; ++j) {
      const int it = wave + 4 * j;
      const int r = it / G::SEGS, seg = it - r * G::SEGS;
      const int lx = seg * 16 + px;
      const unsigned base = lds0 + (unsigned)((r * STRIDE * G::HCOLS + lx * STRIDE) * G::CPP * 16);
      uint4 b[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (toff[s] >= 0) {
          const u32x4 v = *reinterpret_cast<lds_u32x4*>(base + toff[s]);
          b[s] = make_uint4(v.x, v.y, v.z, v.w);
        } else {
          b[s] = make_uint4(0, 0, 0, 0);
        }
      }
      f32x4 acc[NB];
#pragma unroll
      for (int ob = 0; ob < NB; ++ob) {
        acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NS; ++s) M16<T>::run(wa[ob][s], b[s], acc[ob]);
      }
      const int oy = oy0 + r, ox = ox0 + lx;
      if (oy >= Ho || ox >= Wo) continue;
      T* dst = reinterpret_cast<T*>(p.out) + ((size_t)(fr * Ho + oy) * Wo + ox) * p.out_ldc + p.out_coff;
#pragma unroll
      for (int ob = 0; ob < NB; ++ob) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float y = acc[ob][e] + bias[ob][e];
          if constexpr (ACT == 1) y = fmaxf(y, 0.0f);
          else if constexpr (ACT == 2) y = fmaxf(y, 0.01f * y);
          v[e] = y;
        }
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2*>(dst + 16 * ob + 4 * g) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
      }
    }
    const int tn = t + step;
    // persistent grids: every wave's LDS reads of this tile done before the next tile's staging
    // overwrites it (the other resident workgroups cover this one's staging latency)
    if (tn < end) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
      stage(tn);
    }
    if (tn >= end) break;
    t = tn;
  }
}

// halo tile (output columns x rows) per shape: 24-40 KiB of LDS
template <int CIN, int STRIDE> struct HaloTile {
  static constexpr int TW = STRIDE == 1 ? 64 : 32;
  static constexpr int TR = CIN == 16 ? 8 : 4;
};

template <typename T, int CIN, int COUT, int STRIDE, int ACT>
static int launch_t(const ConvParams& p, const ConvParams* dp, int cu_count, int halo, hipStream_t s) {
  if (halo) {
    constexpr int TW = HaloTile<CIN, STRIDE>::TW, TR = HaloTile<CIN, STRIDE>::TR;
    const long frames = p.M / ((long)p.Ho * p.Wo);
    const long blocks = frames * ((p.Ho + TR - 1) / TR) * ((p.Wo + TW - 1) / TW);
    if ((long)p.seg[0].H * p.seg[0].W * p.seg[0].ldc * 2 >= (1L << 31) || blocks >= (1L << 31)) {
      set_error("conv_small: frame too large for the halo kernel");
      return 1;
    }
    auto kern = conv_small_halo<T, CIN, COUT, STRIDE, TW, TR, ACT>;
    long grid = blocks;
    if (halo == 2) {  // persistent: the resident workgroups of one wave of the grid, a multiple of 8
      static int per_cu = 0;  // (occupancy query enqueues nothing: safe under stream capture)
      if (!per_cu && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NT, 0) != hipSuccess) per_cu = 1;
      grid = std::min<long>(blocks, (long)std::max(1, per_cu) * cu_count);
      if (grid < blocks && grid >= 8) grid &= ~7L;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, s, dp);
    TV_HIP(hipGetLastError());
    return 0;
  }
  const long items = (long)(p.M / p.Wo) * ((p.Wo + 15) / 16);
  const long waves = std::min<long>(items, (long)cu_count * 16);  // ~4 resident 4-wave blocks per CU
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL((conv_small<T, CIN, COUT, STRIDE, ACT>), dim3(blocks), dim3(NT), 0, s, dp);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T>
static int dispatch(const ConvParams& p, const ConvParams* dp, int cin, int cout, int stride, int cu, int halo,
                    hipStream_t s) {
  const int act = p.act;
#define TV_CSM(CI, CO, ST)                                                              \
  if (cin == CI && cout == CO && stride == ST) {                                        \
    if (act == 0) return launch_t<T, CI, CO, ST, 0>(p, dp, cu, halo, s);                \
    if (act == 1) return launch_t<T, CI, CO, ST, 1>(p, dp, cu, halo, s);                \
    return launch_t<T, CI, CO, ST, 2>(p, dp, cu, halo, s);                              \
  }
  TV_CSM(16, 16, 1)
  TV_CSM(16, 32, 2)
  TV_CSM(32, 32, 1)
  TV_CSM(32, 64, 2)
  TV_CSM(16, 16, 2)
  TV_CSM(16, 32, 1)
#undef TV_CSM
  set_error("conv_small: unsupported channel / stride combination");
  return 1;
}

}  // namespace csm

bool conv_small_supported(int cin, int cout, int stride, int cin_ldc, int out_ldc) {
  const bool shape = (cin == 16 && cout == 16) || (cin == 16 && cout == 32) || (cin == 32 && cout == 32 && stride == 1) ||
                     (cin == 32 && cout == 64 && stride == 2);
  return shape && (stride == 1 || stride == 2) && cin_ldc % 8 == 0 && out_ldc % 4 == 0;
}

int launch_conv_small(const ConvParams& p, const ConvParams* dp, int dtype, int cu_count, int halo, hipStream_t s) {
  const ConvSegment& sg = p.seg[0];
  if (p.nseg != 1 || sg.kh != 3 || sg.kw != 3 || sg.pad != 1 || sg.pad_w != 1 || p.act < 0 || p.act > 2) {
    set_error("conv_small: 3x3 pad-1 single-segment convs only");
    return 1;
  }
  if (dtype == F16) return csm::dispatch<_Float16>(p, dp, sg.C, p.N, sg.stride, cu_count, halo, s);
  if (dtype == BF16) return csm::dispatch<__bf16>(p, dp, sg.C, p.N, sg.stride, cu_count, halo, s);
  set_error("conv_small: fp16/bf16 only");
  return 1;
}

}  // namespace tv
