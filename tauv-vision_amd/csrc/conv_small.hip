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

template <typename T, int CIN, int COUT, int STRIDE, int ACT>
static int launch_t(const ConvParams& p, const ConvParams* dp, int cu_count, hipStream_t s) {
  const long items = (long)(p.M / p.Wo) * ((p.Wo + 15) / 16);
  const long waves = std::min<long>(items, (long)cu_count * 16);  // ~4 resident 4-wave blocks per CU
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL((conv_small<T, CIN, COUT, STRIDE, ACT>), dim3(blocks), dim3(NT), 0, s, dp);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T>
static int dispatch(const ConvParams& p, const ConvParams* dp, int cin, int cout, int stride, int cu, hipStream_t s) {
  const int act = p.act;
#define TV_CSM(CI, CO, ST)                                                              \
  if (cin == CI && cout == CO && stride == ST) {                                        \
    if (act == 0) return launch_t<T, CI, CO, ST, 0>(p, dp, cu, s);                      \
    if (act == 1) return launch_t<T, CI, CO, ST, 1>(p, dp, cu, s);                      \
    return launch_t<T, CI, CO, ST, 2>(p, dp, cu, s);                                    \
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

int launch_conv_small(const ConvParams& p, const ConvParams* dp, int dtype, int cu_count, hipStream_t s) {
  const ConvSegment& sg = p.seg[0];
  if (p.nseg != 1 || sg.kh != 3 || sg.kw != 3 || sg.pad != 1 || sg.pad_w != 1 || p.act < 0 || p.act > 2) {
    set_error("conv_small: 3x3 pad-1 single-segment convs only");
    return 1;
  }
  if (dtype == F16) return csm::dispatch<_Float16>(p, dp, sg.C, p.N, sg.stride, cu_count, s);
  if (dtype == BF16) return csm::dispatch<__bf16>(p, dp, sg.C, p.N, sg.stride, cu_count, s);
  set_error("conv_small: fp16/bf16 only");
  return 1;
}

}  // namespace tv
