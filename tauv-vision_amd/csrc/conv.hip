// Implicit-GEMM convolution on CDNA4 MFMA (gfx950).
//
// GEMM view: rows = output pixels (NHWC, M = B*Ho*Wo), columns = output channels,
// K = sum over segments of kh*kw*C (tap-major, channel-minor). One workgroup = 256 threads
// (4 waves) computes a 128-pixel x 128-channel tile; each wave a 64x64 sub-tile as 2x2
// MFMA 32x32 tiles. K advances 128 bytes per step (64 fp16/bf16 or 32 fp32 elements):
// 16-byte chunks are register-staged from global memory (im2col on the fly, zero padding
// by predicate) into a double-buffered, XOR-swizzled LDS image, so a 16-lane group of
// ds_read_b128 touches 16 distinct bank slots.
//   f16/bf16: v_mfma_f32_32x32x16_{f16,bf16}   (perf mode)
//   f32     : v_mfma_f32_32x32x2_f32           (exact-f32 parity mode; no xf32 on gfx950)
// Weights are the MFMA A operand (rows = channels) and pixels the B operand, so each
// lane's accumulator holds 4 consecutive channels of one pixel: the epilogue (+bias with
// BN folded, ReLU/LeakyReLU) stages the tile through LDS and writes whole 16-byte chunks.
// Mode 1 turns the same GEMM into a non-overlapping ConvTranspose2d (k == s): columns are
// (phase, channel) and the epilogue scatters each phase to its target pixel and adds the
// skip tensor (IDAUp: f + pad_to_match(up(project(x))), dla.py:277-278, 352-353).
#include "conv_common.h"

namespace tv {



// Stage k-step `ks`: 4 activation chunks (im2col on the fly) and 4 weight chunks per thread.
// Out-of-image taps load a clamped in-bounds address and are zeroed by a select, so the
// loads stay branch-free.
template <typename T>
__device__ __forceinline__ void load_tile(const ConvParams& p, int ks, int lc, const int (&pb)[4],
                                          const int (&poy)[4], const int (&pox)[4], const bool (&pvalid)[4],
                                          const T* const (&wrow)[4], uint4 (&ra)[4], uint4 (&rw)[4]) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = kRowBytes / sizeof(T);
  int s = 0;
#pragma unroll
  for (int t = 1; t < kMaxSeg; ++t)
    if (t < p.nseg && ks >= p.seg[t].kbase) s = t;
  const ConvSegment& sg = p.seg[s];
  const int ke = (ks - sg.kbase) * BK + lc * VEC;
  const int tap = ke / sg.C;
  const int ci = ke - tap * sg.C;
  const int ky = tap / sg.kw;
  const int kx = tap - ky * sg.kw;
  const bool tap_ok = tap < sg.kh * sg.kw;
  const T* src = reinterpret_cast<const T*>(sg.src);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int iy = poy[i] * sg.stride + ky - sg.pad;
    int ix = pox[i] * sg.stride + kx - sg.pad_w;
    bool ok = pvalid[i] && tap_ok && iy >= 0 && iy < sg.H && ix >= 0 && ix < sg.W;
    iy = min(max(iy, 0), sg.H - 1);
    ix = min(max(ix, 0), sg.W - 1);
    uint4 v = gload16(src + ((size_t)(pb[i] * sg.H + iy) * sg.W + ix) * sg.ldc + (tap_ok ? ci : 0));
    ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
    rw[i] = gload16(wrow[i] + (size_t)ks * BK);
  }
}

__device__ __forceinline__ void stash_tile(char* smem, int stage, int lr, int lc, const uint4 (&ra)[4],
                                           const uint4 (&rw)[4]) {
  char* xs = smem + stage * kStageBytes;
  char* ws = xs + kTileM * kRowBytes;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    *reinterpret_cast<uint4*>(xs + swz(lr + 32 * i, lc)) = ra[i];
    *reinterpret_cast<uint4*>(ws + swz(lr + 32 * i, lc)) = rw[i];
  }
}

template <typename T, typename OutT, int MODE>
__global__ __launch_bounds__(kThreads, 2) void conv_igemm(const ConvParams* __restrict__ pp, void* out_ptr) {
  // Launch parameters live in device memory so the per-k-step segment lookup is a
  // wave-uniform scalar load (a by-value struct indexed at run time spills to scratch).
  const ConvParams& p = *pp;
  constexpr int VEC = 16 / sizeof(T);      // elements per 16-byte chunk
  // (k-step width BK = kRowBytes / sizeof(T) elements)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  // XCD-aware bijective remap: consecutive tiles (which share input halo rows and the
  // weight panel) run on the same XCD's L2.
  const int nb = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ntile = lin % p.ntiles;
  const int mtile = lin / p.ntiles;
  const int m0 = mtile * kTileM;
  const int n0 = ntile * kTileN;

  // ---- loader geometry: rows (tid>>3) + 32*i, 16-byte chunk tid&7
  const int lc = tid & 7;
  const int lr = tid >> 3;
  int pb[4], poy[4], pox[4];
  bool pvalid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + lr + 32 * i;
    pvalid[i] = m < p.M;
    int mm = pvalid[i] ? m : 0;
    int hw = p.Ho * p.Wo;
    pb[i] = mm / hw;
    int rem = mm - pb[i] * hw;
    poy[i] = rem / p.Wo;
    pox[i] = rem - poy[i] * p.Wo;
  }

  const int total_ks = p.seg[p.nseg - 1].kbase + p.seg[p.nseg - 1].ksteps;
  const T* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    wrow[i] = reinterpret_cast<const T*>(p.weight) + (size_t)(n0 + lr + 32 * i) * p.Kpad + lc * VEC;

  uint4 ra[4], rw[4];

  // ---- compute geometry: wave (wc, wp) owns channels [wc*64,+64) x pixels [wp*64,+64)
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave & 1;
  const int wp = wave >> 1;
  const int lrow = lane & 31;
  const int lh = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  load_tile<T>(p, 0, lc, pb, poy, pox, pvalid, wrow, ra, rw);
  stash_tile(smem, 0, lr, lc, ra, rw);
  __syncthreads();

  for (int ks = 0; ks < total_ks; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < total_ks;
    if (more) load_tile<T>(p, ks + 1, lc, pb, poy, pox, pvalid, wrow, ra, rw);
    const char* xs = smem + cur * kStageBytes;
    const char* ws = xs + kTileM * kRowBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 2 * j + lh;
      uint4 fw[2], fx[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fw[t] = *reinterpret_cast<const uint4*>(ws + swz(wc * 64 + t * 32 + lrow, c));
        fx[t] = *reinterpret_cast<const uint4*>(xs + swz(wp * 64 + t * 32 + lrow, c));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) Mfma<T>::run(fw[a], fx[b], acc[a][b]);
    }
    if (more) stash_tile(smem, cur ^ 1, lr, lc, ra, rw);
    __syncthreads();
  }

  // ---- epilogue: bias + activation, fp32 staging tile [pixel][channel]
  float* stg = reinterpret_cast<float*>(smem);
  constexpr int SR = kStageRow / 4;  // floats per staged row
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int pix = wp * 64 + b * 32 + lrow;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = wc * 64 + a * 32 + 8 * g + 4 * lh;
        const uint4 braw = gload16(p.bias + n0 + ch);
        const f32x4 bias4 = f32x4{__uint_as_float(braw.x), __uint_as_float(braw.y), __uint_as_float(braw.z),
                                  __uint_as_float(braw.w)};
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[a][b][4 * g + e] + bias4[e];
          if (p.act == 1) x = fmaxf(x, 0.0f);
          else if (p.act == 2) x = x >= 0.0f ? x : 0.01f * x;
          v[e] = x;
        }
        *reinterpret_cast<f32x4*>(stg + pix * SR + ch) = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
  }
  __syncthreads();

  constexpr int OVEC = 16 / sizeof(OutT);
  constexpr int CPR = kTileN / OVEC;  // chunks per row
  for (int qd = tid; qd < kTileM * CPR; qd += kThreads) {
    const int row = qd / CPR;
    const int cc = qd - row * CPR;
    const int m = m0 + row;
    const int n = n0 + cc * OVEC;
    if (m >= p.M || n >= p.N) continue;
    const float* sv = stg + row * SR + cc * OVEC;
    if (MODE == 0) {
      OutT* dst = reinterpret_cast<OutT*>(out_ptr) + (size_t)m * p.out_ldc + p.out_coff + n;
      store_chunk<OutT>(dst, sv);
    } else {
      const int hw = p.Ho * p.Wo;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int oy = rem / p.Wo;
      const int ox = rem - oy * p.Wo;
      const int phase = n / p.up_cout;
      const int co = n - phase * p.up_cout;
      const int Y = oy * p.up_s + phase / p.up_s + p.sy;
      const int X = ox * p.up_s + phase % p.up_s + p.sx;
      if (Y >= p.tH || X >= p.tW) continue;
      const size_t tpix = (size_t)(b * p.tH + Y) * p.tW + X;
      const T* ad = reinterpret_cast<const T*>(p.add) + tpix * p.add_ldc + co;
      float v[OVEC];
      const uint4 raw = p.add ? gload16(ad) : make_uint4(0, 0, 0, 0);  // no skip tensor: plain scatter
      const uint32_t rw4[4] = {raw.x, raw.y, raw.z, raw.w};
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int e = 0; e < OVEC; ++e) v[e] = __uint_as_float(rw4[e]) + sv[e];
      } else {
#pragma unroll
        for (int e = 0; e < OVEC; ++e) {
          const uint16_t bits = (uint16_t)(rw4[e >> 1] >> (16 * (e & 1)));
          v[e] = to_f(__builtin_bit_cast(T, bits)) + sv[e];
        }
      }
      OutT* dst = reinterpret_cast<OutT*>(out_ptr) + tpix * p.out_ldc + co;
      store_chunk<OutT>(dst, v);
    }
  }
}

template <typename T, typename OutT, int MODE>
static int launch_t(const ConvParams& p, const ConvParams* dp, void* out, hipStream_t s) {
  auto k = conv_igemm<T, OutT, MODE>;
  if (int r = ensure_lds<conv_igemm<T, OutT, MODE>>(kLdsBytes)) return r;
  dim3 grid(p.mtiles * p.ntiles);
  hipLaunchKernelGGL(k, grid, dim3(kThreads), kLdsBytes, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_conv(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int out_f32, int mode,
                hipStream_t s) {
  if (dtype == F32) {
    return mode == 0 ? launch_t<float, float, 0>(p, dp, out, s) : launch_t<float, float, 1>(p, dp, out, s);
  } else if (dtype == F16) {
    if (mode == 1) return launch_t<_Float16, _Float16, 1>(p, dp, out, s);
    return out_f32 ? launch_t<_Float16, float, 0>(p, dp, out, s) : launch_t<_Float16, _Float16, 0>(p, dp, out, s);
  } else {
    if (mode == 1) return launch_t<__bf16, __bf16, 1>(p, dp, out, s);
    return out_f32 ? launch_t<__bf16, float, 0>(p, dp, out, s) : launch_t<__bf16, __bf16, 0>(p, dp, out, s);
  }
}

}  // namespace tv
