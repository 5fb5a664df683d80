// Streaming 1x1 convolution over concatenated inputs (gfx950, fp16 / bf16): the DLA Root
// (dla.py:58-76: Conv2d(sum of children's channels, C, 1) over torch.cat(children) + BN + ReLU;
// centerpoint_dla.py's Roots alike) and any other stride-1 1x1 conv whose K fits in LDS.
//
// A 1x1 conv reads K and writes N values per pixel for 2 K N FLOPs: K N / (K + N) FLOP per byte
// (85 at K = 256, N = 128) against the ~310 of the MFMA peak over HBM, so it is bound by the
// stream of its input and output. The pipelined implicit GEMM (conv_pipe.hip)
// stages each 256-pixel tile's operands through an LDS-DMA ring with one barrier per 64-deep
// k-step, 4-6 k-steps per tile: fill and drain dominate (0.2-0.26 PFLOP/s, ~2x the stream time).
// Here, as in convt.hip:
//  * the layer's weights ([N][K], bias) move to LDS once per workgroup (conflict-free row pitch);
//  * each wave streams its own run of 32-pixel tiles with no barrier: the MFMA B operand (16
//    bytes of the pixel's channels per lane) comes straight from global memory in chunks of 64
//    channels, the next chunk (of this tile or the next) in flight under the current one's 4 x
//    NI MFMAs; the A operand (weights) is read from LDS two k-steps ahead;
//  * the epilogue works on the accumulators in place (bias, activation, one rounding,
//    v_permlane32_swap into 16-byte stores), in conv_pipe's epilogue order.
// Numerics: the same fp32 products as conv_pipe, summed in segment / channel order.
#include "conv_common.h"

#include <algorithm>
#include <mutex>
#include <type_traits>

namespace tv {
namespace c1x1 {

constexpr int NT = 512, NW = NT / 64;
constexpr int KC = 64;                 // channels per chunk (4 MFMA k-steps of 16)
constexpr int MAXK = 576;              // K bound: 128 rows x (576 x 2 + 16) B = 149 KiB of weights
constexpr int LDS_MAX = 160 * 1024;

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

struct Chunk {
  uint4 x[4];  // B operand: 4 k-steps of 16 channels, lane half lh holding channels 8 lh .. + 8
};

// NI = output channels / 32 (4: 128, 2: 64)
// (N > 128: workgroup g runs the 128-channel slice g % ntiles of the output over its share of the
// pixel tiles; the input is read once per slice)
template <typename T, int NI>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void conv1x1_stream(
    const ConvParams* __restrict__ pp, int wpitch, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ConvParams& p = *pp;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int nrows = NI * 32;
  const int K = p.Kpad;  // packed row length: segment s's channels at [seg.kbase * 64, + C)
  const int nt = blockIdx.x % ntiles, wgi = blockIdx.x / ntiles, nwg = gridDim.x / ntiles;
  const int n0 = nt * 128, nloc = min(p.N - n0, nrows);

  // ---- weights [nrows][K] and bias into LDS (all loads issued before the stores)
  {
    const int cpr = K * (int)sizeof(T) / 16;  // 16-byte chunks per row
    const int total = nrows * cpr;
    const char* wsrc = reinterpret_cast<const char*>(p.weight) + (size_t)n0 * K * sizeof(T);
    for (int base = 0; base < total; base += 8 * NT) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = base + u * NT + tid;
        const int r = c / cpr, q = c - r * cpr;
        v[u] = c < total ? gload16(wsrc + ((size_t)r * K * sizeof(T)) + q * 16) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = base + u * NT + tid;
        const int r = c / cpr, q = c - r * cpr;
        if (c < total) *reinterpret_cast<uint4*>(smem + r * wpitch + q * 16) = v[u];
      }
    }
    float* lb = reinterpret_cast<float*>(smem + nrows * wpitch);
    if (tid < nrows) lb[tid] = tid < nloc ? p.bias[n0 + tid] : 0.0f;
  }
  __syncthreads();

  const int M = p.M;
  const int mt = (M + 31) / 32;
  const long long gw = (long long)wgi * NW + wave, nw = (long long)nwg * NW;
  const int t_begin = (int)(mt * gw / nw);
  const int t_end = (int)(mt * (gw + 1) / nw);
  if (t_begin >= t_end) return;

  // chunk q of a tile: segment sq, channels [cq, cq + 64): the chunk list walks the segments
  int nch = 0;
  for (int s = 0; s < p.nseg; ++s) nch += p.seg[s].C / KC;
  auto load_chunk = [&](int t, int q, Chunk& c) __attribute__((always_inline)) {
    int s = 0;
    while (q >= p.seg[s].C / KC) q -= p.seg[s].C / KC, ++s;  // (uniform)
    const ConvSegment& sg = p.seg[s];
    const int m = t * 32 + l32;
    const T* src = reinterpret_cast<const T*>(sg.src) + (size_t)(m < M ? m : 0) * sg.ldc + q * KC + 8 * lh;
#pragma unroll
    for (int j = 0; j < 4; ++j) c.x[j] = gload16(src + 16 * j);
  };
  auto chunk_k0 = [&](int q) __attribute__((always_inline)) {  // weight column of the chunk's first channel
    int s = 0;
    while (q >= p.seg[s].C / KC) q -= p.seg[s].C / KC, ++s;
    return p.seg[s].kbase * (128 / (int)sizeof(T)) + q * KC;
  };

  const char* wl = smem + l32 * wpitch + lh * 16;
  const float* lb = reinterpret_cast<const float*>(smem + nrows * wpitch);
  f32x16 acc[NI];
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int m = t * 32 + l32;
    const bool ok = m < M;
    T* out = reinterpret_cast<T*>(p.out) + (size_t)(ok ? m : 0) * p.out_ldc + p.out_coff + n0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        float v[2][4];
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int G2 = 2 * mm + gg;
          const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float y = acc[i][4 * G2 + e] + bb[e];
            if (p.act == 1) y = fmaxf(y, 0.0f);
            else if (p.act == 2) y = y >= 0.0f ? y : 0.01f * y;
            v[gg][e] = y;
          }
        }
        const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
        const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
        const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const int ch = 32 * i + 16 * mm + 8 * lh;
        if (ok && ch < nloc) gstore16(out + ch, make_uint4(r0[0], r1[0], r0[1], r1[1]));
      }
    }
  };

  auto compute = [&](const Chunk& c, int qq, bool first) __attribute__((always_inline)) {
    const int k0 = chunk_k0(qq);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint4 w[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        w[i] = *reinterpret_cast<const uint4*>(wl + (size_t)(32 * i) * wpitch + (k0 + 16 * j) * (int)sizeof(T));
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (first && j == 0) acc[i] = f32x16{};
        Mfma<T>::run(w[i], c.x[j], acc[i]);
      }
    }
  };
  // the chunk stream: (tile t, chunk q) in order through a 3-slot register ring, the chunks two
  // positions ahead in flight under the current one's MFMAs (one ahead measured ~2x the stream time)
  auto next = [&](int& tt, int& qq) __attribute__((always_inline)) {
    if (++qq == nch) qq = 0, ++tt;
  };
  Chunk cb[3];
  int tc = t_begin, qc = 0;  // chunk being computed
  int tl = t_begin, ql = 0;  // next chunk to load
  load_chunk(tl, ql, cb[0]);
  next(tl, ql);
  if (tl < t_end) load_chunk(tl, ql, cb[1]);
  next(tl, ql);
  auto stage = [&](auto r) __attribute__((always_inline)) {
    constexpr int R = decltype(r)::value;
    if (tl < t_end) load_chunk(tl, ql, cb[(R + 2) % 3]);
    next(tl, ql);
    compute(cb[R], qc, qc == 0);
    if (qc == nch - 1) epilogue(tc);
    next(tc, qc);
    return tc < t_end;
  };
  while (stage(std::integral_constant<int, 0>{}) && stage(std::integral_constant<int, 1>{}) &&
         stage(std::integral_constant<int, 2>{})) {
  }
}

}  // namespace c1x1

bool conv1x1_stream_supported(const ConvParams& p, int esz) {
  if (esz != 2 || p.nseg < 1 || p.nseg > kMaxSeg || p.N < 8 || p.N > 4 * 128 || p.N % 8 || p.out_ldc % 8 ||
      p.out_coff % 8 || p.Kpad > c1x1::MAXK || p.Kpad % 64 || p.up_s)
    return false;
  for (int s = 0; s < p.nseg; ++s) {
    const ConvSegment& g = p.seg[s];
    if (g.kh != 1 || g.kw != 1 || g.stride != 1 || g.pad != 0 || g.C % c1x1::KC || g.ldc % 8 ||
        g.H != p.Ho || g.W != p.Wo || g.kbase * 64 + g.C > p.Kpad)
      return false;
  }
  return true;
}

int launch_conv1x1_stream(const ConvParams& p, const ConvParams* dp, int dtype, int cu_count, hipStream_t s) {
  using namespace c1x1;
  if (!conv1x1_stream_supported(p, 2) || !p.out) {
    set_error("conv1x1_stream: unsupported layer");
    return 1;
  }
  const int ntiles = (p.N + 127) / 128;
  const int ni = p.N > 64 ? 4 : 2;
  const int wpitch = p.Kpad * 2 + 16;
  const int lds = ni * 32 * wpitch + ni * 32 * 4;
  if (lds > LDS_MAX) {
    set_error("conv1x1_stream: weights exceed LDS");
    return 1;
  }
  const long mt = ((long)p.M + 31) / 32;
  const int per = (int)std::max(1L, std::min<long>(std::max(1, cu_count / ntiles), (mt + NW - 1) / NW));
  const int grid = per * ntiles;
  using L = void (*)(const ConvParams*, int, int);
  L k = nullptr;
  if (dtype == F16) k = ni == 4 ? conv1x1_stream<_Float16, 4> : conv1x1_stream<_Float16, 2>;
  else if (dtype == BF16) k = ni == 4 ? conv1x1_stream<__bf16, 4> : conv1x1_stream<__bf16, 2>;
  else {
    set_error("conv1x1_stream: fp16/bf16 only");
    return 1;
  }
  static std::once_flag once[4];
  const int which = (dtype == F16 ? 0 : 2) + (ni == 4 ? 0 : 1);
  hipError_t attr = hipSuccess;
  std::call_once(once[which], [&] {
    attr = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  });
  TV_HIP(attr);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, s, dp, wpitch, ntiles);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
