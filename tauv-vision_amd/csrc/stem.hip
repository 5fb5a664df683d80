// Fused input staging + 7x7 stem convolution (gfx950, fp16 / bf16): the reference's
// ToTensor + Normalize (centernet_node.py:90-92) followed by DLADown.projection_layer
// = Conv2d(3, C0, 7, padding=3) + BatchNorm + ReLU at full input resolution
// (dla.py:150-154, 182-183).
//
// Why a kernel of its own: at 480x640 the stem writes 128 channels x 2 B per input pixel
// (5 GB per 64-frame batch) while its contraction is only K = 147, so it is bound by HBM
// WRITES, not by the matrix cores. The generic implicit GEMM spent 3.1 ms on it (plus 0.5 ms
// for a separate staging kernel writing a 0.94 GB row-expanded input): per 256-pixel tile a
// 3-k-step pipeline prologue, an LDS-staged epilogue and no overlap of one tile's stores with
// the next tile's work. Here:
//  * one persistent 512-thread workgroup per CU loops over 16x32-pixel tiles x all C0 <= 128
//    output channels; the weights (fragment order, 44 KiB) and the bias stay in LDS;
//  * the tile's input window (22 x 38 pixels x 3 channels) is read straight from the caller's
//    frames — raw u8 HWC (normalised through a 768-entry LUT built with prep_u8's exact fp32
//    expression) or normalised fp32 NCHW — with zeros outside the image (the conv's padding),
//    then expanded in LDS to the row-expanded operand E[row][x][24] (7 horizontal taps x 3
//    channels + 3 zeros), so K = 7 rows x 24 = 168 -> 11 MFMA k-steps of 16 (147 real);
//  * the next tile's input loads are issued before the current tile's MFMAs, and the epilogue
//    stores straight from the accumulators (bias + ReLU, v_permlane32_swap into 16-byte stores),
//    so a tile's 128 KiB of stores drain while the next tile computes.
#include "conv_common.h"

namespace tv {
namespace stem {

constexpr int NT = 512;
constexpr int TW = 32, TH = 16;             // output tile (one 32-pixel MFMA fragment per row)
constexpr int RR = TH + 6, RX = TW + 6;      // input window rows / pixels
constexpr int NVAL = RR * RX * 3;            // input values per tile = 2508
constexpr int NPITCH = 256;                  // bytes per normalised input row in LDS (114 x 2 B used)
constexpr int EPIX = 48;                     // bytes per expanded pixel (24 values)
constexpr int EBUF = RR * TW * EPIX;         // 33,792
constexpr int KS = 11;                       // MFMA k-steps (K = 176 >= 168)
constexpr int WF_BYTES = KS * 4 * 64 * 16;   // weights in B-fragment order = 45,056
// LDS layout per NI. NI = 4: two E buffers (the next tile expanded while this one's MFMAs run),
// one 512-thread workgroup per CU. NI = 1 (16-32 output channels: little MFMA work per tile, the
// window staging and expansion dominate): one E buffer and only the 11 KiB of block-0 weight
// fragments, 53 KiB in all, so several workgroups per CU overlap one's staging with another's
// MFMAs (round 5: the workgroup's own double buffering left the staging serial).
template <int NI> struct Lay {
  static constexpr int NE = NI == 1 ? 1 : 2;
  static constexpr int OFF_E = 0;
  static constexpr int OFF_W = OFF_E + NE * EBUF;
  static constexpr int WBYTES = KS * NI * 64 * 16;   // fragments (k-step j, block i) at (j NI + i) KiB
  static constexpr int OFF_N = OFF_W + WBYTES;
  static constexpr int OFF_LUT = OFF_N + RR * NPITCH;
  static constexpr int OFF_B = OFF_LUT + 768 * 2;
  static constexpr int LDS = OFF_B + 128 * 4;
  static constexpr int WGS = NI == 1 ? 2 : 1;        // workgroups per CU the grid is sized for (3 spills)
  static_assert(LDS * WGS <= 160 * 1024, "LDS budget");
};

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

// Workgroup barrier for LDS hand-offs only. __syncthreads() also waits for every outstanding
// global store (vmcnt(0)), which would drain a tile's 128 KiB of stores before the next tile's
// work instead of letting them stream under it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// input staging modes: 0 normalised fp32 NCHW, 1 u8 HWC (any width), 2 u8 HWC with in_w % 4 == 0
// (whole rows are dword aligned: the window is read as 30 dwords per row)
template <int MODE> struct Window;
template <> struct Window<0> { static constexpr int NS = (NVAL + NT - 1) / NT; };  // 5 values per thread
template <> struct Window<1> { static constexpr int NS = (NVAL + NT - 1) / NT; };
template <> struct Window<2> { static constexpr int NS = (RR * 30 + NT - 1) / NT; };  // 2 dwords per thread

// NI: 32-channel output blocks computed (4 for C0 = 128; 1 for DLA-34's 16-channel base layer,
// whose tiles would otherwise spend 3/4 of their MFMAs and epilogue on padding channels)
template <typename T, int MODE, int NI>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2 * Lay<NI>::WGS, 2 * Lay<NI>::WGS)))
void stem_conv(StemParams p) {
  using L = Lay<NI>;
  constexpr int OFF_E = L::OFF_E, OFF_W = L::OFF_W, OFF_N = L::OFF_N, OFF_LUT = L::OFF_LUT, OFF_B = L::OFF_B;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool U8 = MODE != 0;
  constexpr int NS = Window<MODE>::NS;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int H = p.H, W = p.W;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int tiles_f = tiles_x * tiles_y;
  const int ntot = p.B * tiles_f;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntot) return;

  // ---- resident operands: weights (host-packed in B-fragment order), bias, u8 LUT
  {
    const uint4* ws = reinterpret_cast<const uint4*>(p.weight);
    uint4* wd = reinterpret_cast<uint4*>(smem + OFF_W);
    // all loads issued before the LDS writes (one memory latency, not one per chunk)
    // LDS chunk d = fragment (j, i) = (d / 64 / NI, d / 64 % NI), 16-byte lane chunk d % 64, of the
    // host's 4-block fragment order
    constexpr int NCH = (L::WBYTES / 16 + NT - 1) / NT;
    auto src_chunk = [](int d) { return ((d >> 6) / NI * 4 + (d >> 6) % NI) * 64 + (d & 63); };
    uint4 wv[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      wv[k] = tid + k * NT < L::WBYTES / 16 ? ws[src_chunk(tid + k * NT)] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (tid + k * NT < L::WBYTES / 16) wd[tid + k * NT] = wv[k];
    float* lb = reinterpret_cast<float*>(smem + OFF_B);
    if (tid < 128) lb[tid] = tid < p.N ? p.bias[tid] : 0.0f;
    if constexpr (U8) {
      T* lut = reinterpret_cast<T*>(smem + OFF_LUT);
      for (int i = tid; i < 768; i += NT) {
        const int v = i / 3, c = i - v * 3;
        lut[i] = (T)(((float)v / 255.0f - kMean[c]) / kStd[c]);  // prep_u8's expression, bit for bit
      }
    }
  }

  // ---- input window of a tile: rows y0-3 .. y0+18, pixels x0-3 .. x0+34, 3 channels.
  // Two register sets: tile j's window is loaded at the start of tile j-2 (set j % 2). Vector
  // memory completes in issue order, so a load issued right behind a tile's 128 KiB of stores
  // could not be consumed before those stores drain; two tiles ahead, the wait is for stores
  // issued two tiles earlier (long done) while the last tile's stores keep streaming.
  auto tile_origin = [&](int t, int& fr, int& y0, int& x0) __attribute__((always_inline)) {
    fr = t / tiles_f;
    const int r = t - fr * tiles_f;
    const int ty = r / tiles_x;
    y0 = ty * TH - 3;
    x0 = (r - ty * tiles_x) * TW - 3;
  };
  unsigned raw0[NS], raw1[NS];
  auto load_window = [&](int t, unsigned (&raw)[NS]) __attribute__((always_inline)) {
    int fr, y0, x0;
    tile_origin(t, fr, y0, x0);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int idx = tid + k * NT;
      if constexpr (MODE == 2) {
        const int r = idx / 30, dw = idx - r * 30;
        const int y = y0 + r;
        const int bx = x0 * 3 - 3 + 4 * dw;  // byte within the row; x0*3 - 3 is dword aligned
        const bool ok = idx < RR * 30 && (unsigned)y < (unsigned)H && bx >= 0 && bx < 3 * W;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(p.input) + (size_t)(fr * H + (ok ? y : 0)) * W * 3;
        raw[k] = ok ? *reinterpret_cast<const unsigned*>(src + bx) : 0u;
      } else {
        const int r = idx / (RX * 3), q = idx - r * (RX * 3);
        const int xx = q / 3, c = q - xx * 3;
        const int y = y0 + r, x = x0 + xx;
        const bool ok = idx < NVAL && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        if constexpr (MODE == 1) {
          const uint8_t* src = reinterpret_cast<const uint8_t*>(p.input);
          raw[k] = ok ? (unsigned)src[((size_t)(fr * H + y) * W + x) * 3 + c] : ~0u;
        } else {
          const float* src = reinterpret_cast<const float*>(p.input);
          raw[k] = ok ? __float_as_uint(src[((size_t)(fr * 3 + c) * H + y) * W + x]) : 0u;
        }
      }
    }
  };
  // normalised window -> LDS N[row][x*3 + c] (zeros outside the image = the conv's padding)
  auto store_window = [&](int t, const unsigned (&raw)[NS]) __attribute__((always_inline)) {
    T* nimg = reinterpret_cast<T*>(smem + OFF_N);
    const T* lut = reinterpret_cast<const T*>(smem + OFF_LUT);
    int fr, y0, x0;
    tile_origin(t, fr, y0, x0);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int idx = tid + k * NT;
      if constexpr (MODE == 2) {
        if (idx >= RR * 30) continue;
        const int r = idx / 30, dw = idx - r * 30;
        const bool rok = (unsigned)(y0 + r) < (unsigned)H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = 4 * dw + j - 3;  // value index in the window row
          if (q < 0 || q >= RX * 3) continue;
          const int xx = q / 3, c = q - xx * 3;
          const bool ok = rok && (unsigned)(x0 + xx) < (unsigned)W;
          nimg[r * (NPITCH / 2) + q] = ok ? lut[((raw[k] >> (8 * j)) & 0xffu) * 3 + c] : (T)0.0f;
        }
      } else {
        if (idx >= NVAL) continue;
        const int r = idx / (RX * 3), q = idx - r * (RX * 3);
        T v;
        if constexpr (MODE == 1) v = raw[k] != ~0u ? lut[raw[k] * 3 + (q % 3)] : (T)0.0f;
        else v = (T)__uint_as_float(raw[k]);
        nimg[r * (NPITCH / 2) + q] = v;
      }
    }
  };
  // N -> E[row][x][24]: chunk p of pixel x = values N[row][3x + 8p + 0..7] (zeros past 21)
  auto expand = [&](int ebuf) __attribute__((always_inline)) {
    const char* nimg = smem + OFF_N;
    char* e = smem + OFF_E + ebuf * EBUF;
    for (int idx = tid; idx < RR * TW * 3; idx += NT) {
      const int pp = idx % 3, px = idx / 3;
      const int row = px / TW, x = px - row * TW;
      const int boff = row * NPITCH + 6 * x + 16 * pp;
      const unsigned* d = reinterpret_cast<const unsigned*>(nimg + (boff & ~3));
      const unsigned sh = (unsigned)(boff & 3);  // 0 or 2
      unsigned v[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) v[j] = d[j];
      uint4 o;
      o.x = __builtin_amdgcn_alignbyte(v[1], v[0], sh);
      o.y = __builtin_amdgcn_alignbyte(v[2], v[1], sh);
      o.z = __builtin_amdgcn_alignbyte(v[3], v[2], sh);
      o.w = __builtin_amdgcn_alignbyte(v[4], v[3], sh);
      if (pp == 2) {  // values 16..23: 16..20 real, 21..23 zero
        o.z &= 0xffffu;
        o.w = 0u;
      }
      *reinterpret_cast<uint4*>(e + px * EPIX + 16 * pp) = o;
    }
  };

  // ---- fragment addresses: wave owns tile rows 2*wave + f (f = 0, 1), lane pixel l32.
  // k-step j reads chunk c8 = 2j + lh of the 21 (ky, part) chunks (the pad chunk re-reads chunk
  // 20; its weights are zero): offset(c8) = (c8 / 3) * TW * EPIX + (c8 % 3) * 16 — a compile-time
  // offset from one of three per-lane bases (lane half 1 adds 16 B, or a row step minus 32 B).
  const char* ab0 = smem + OFF_E + ((2 * wave) * TW + l32) * EPIX;
  const char* ab16 = ab0 + lh * 16;
  const char* abrow = ab0 + lh * (TW * EPIX - 32);
  const char* wfl = smem + OFF_W + lane * 16;

  // one output row f of the wave's two: its 16 KiB of stores (epilogue) then drain under the
  // other row's MFMAs instead of all 128 KiB of a tile leaving at once
  f32x16 acc[2][4];
  auto mfma_row = [&](int ebuf, auto fc) __attribute__((always_inline)) {
    constexpr int f = decltype(fc)::value;
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[f][i] = f32x16{};
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      const int c0 = 2 * j;  // lane half 0's chunk
      const int off0 = (c0 / 3) * TW * EPIX + (c0 % 3) * 16 + ebuf * EBUF;
      const char* base = j == KS - 1 ? ab0 : (c0 % 3 == 2 ? abrow : ab16);
      uint4 b[NI];
      const uint4 a = *reinterpret_cast<const uint4*>(base + off0 + f * TW * EPIX);
#pragma unroll
      for (int i = 0; i < NI; ++i) b[i] = *reinterpret_cast<const uint4*>(wfl + (j * NI + i) * 1024);
#pragma unroll
      for (int i = 0; i < NI; ++i) Mfma<T>::run(b[i], a, acc[f][i]);
    }
  };

  auto epilogue = [&](int t, auto fc) __attribute__((always_inline)) {
    constexpr int f = decltype(fc)::value;
    const int fr = t / tiles_f;
    const int r = t - fr * tiles_f;
    const int ty = r / tiles_x;
    const int y0 = ty * TH, x0 = (r - ty * tiles_x) * TW;
    const float* lb = reinterpret_cast<const float*>(smem + OFF_B);
    {
      const int y = y0 + 2 * wave + f, x = x0 + l32;
      const bool ok = y < H && x < W;
      T* dst = reinterpret_cast<T*>(p.out) + ((size_t)(fr * H + (ok ? y : 0)) * W + (ok ? x : 0)) * p.out_ldc;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float v[2][4];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int G2 = 2 * m + gg;
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[gg][e] = fmaxf(acc[f][i][4 * G2 + e] + bb[e], 0.0f);
          }
          const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
          const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
          const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
          const int ch = 32 * i + 16 * m + 8 * lh;
          if (ok && ch < p.N) gstore16(dst + ch, make_uint4(r0[0], r1[0], r0[1], r1[1]));
        }
      }
    }
  };

  // ---- prologue: windows of the first two tiles, the first expanded into E[0]
  const int t0 = blockIdx.x;
  load_window(t0, raw0);
  if (t0 + G < ntot) load_window(t0 + G, raw1);
  lds_barrier();  // LUT ready
  store_window(t0, raw0);
  lds_barrier();
  expand(0);
  lds_barrier();
  // tile k of this block: t = t0 + k*G, E buffer k % 2, window of tile k+1 in set (k+1) % 2
  auto tile = [&](int t, int eb, unsigned (&raw_next)[NS], unsigned (&raw_k2)[NS]) __attribute__((always_inline)) {
    const int tn = t + G, tn2 = t + 2 * G;
    if constexpr (L::NE == 1) eb = 0;
    if (tn2 < ntot) load_window(tn2, raw_k2);  // tile k's set: already consumed
    mfma_row(eb, std::integral_constant<int, 0>{});
    epilogue(t, std::integral_constant<int, 0>{});
    mfma_row(eb, std::integral_constant<int, 1>{});
    epilogue(t, std::integral_constant<int, 1>{});
    if (tn < ntot) {
      store_window(tn, raw_next);  // N is free: its last reader (expand) finished before the last barrier
      lds_barrier();               // (one E buffer: also every wave's MFMA reads of E done)
      expand(L::NE == 1 ? 0 : eb ^ 1);  // E[eb ^ 1] was last read by the previous tile's MFMAs
      lds_barrier();
    }
  };
  for (int t = t0; t < ntot; t += 2 * G) {
    tile(t, 0, raw1, raw0);
    if (t + G < ntot) tile(t + G, 1, raw0, raw1);
  }
}

template <typename T, int MODE, int NI>
static int launch_t(const StemParams& p, int grid, hipStream_t s) {
  auto k = stem_conv<T, MODE, NI>;
  if (int r = ensure_lds<stem_conv<T, MODE, NI>>(Lay<NI>::LDS)) return r;
  const long ntot = (long)p.B * ((p.H + TH - 1) / TH) * ((p.W + TW - 1) / TW);
  grid = (int)std::min<long>(ntot, (long)grid * Lay<NI>::WGS);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), Lay<NI>::LDS, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace stem

size_t stem_weight_bytes() { return stem::WF_BYTES; }  // the host's 4-block fragment order

// [Npad][Kpad] packed stem weights (K = ky * 24 + kx * 3 + c) -> B-fragment order:
// fragment (k-step j, channel block i), lane l: 8 values n = 32i + l%32, k = 16j + 8(l/32) + e
void stem_fragment_order(const uint16_t* w, int Npad, int Kpad, uint16_t* out) {
  for (int j = 0; j < stem::KS; ++j)
    for (int i = 0; i < 4; ++i)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) {
          const int n = 32 * i + (l & 31), k = 16 * j + 8 * (l >> 5) + e;
          out[((j * 4 + i) * 64 + l) * 8 + e] = (n < Npad && k < Kpad) ? w[(size_t)n * Kpad + k] : 0;
        }
}

int launch_stem(const StemParams& p, int dtype, int grid, hipStream_t s) {
  if (p.N < 1 || p.N > 128 || p.N % 8 || p.out_ldc % 8 || p.B < 1 || p.H < 1 || p.W < 1) {
    set_error("stem: unsupported geometry");
    return 1;
  }
  const long ntot = (long)p.B * ((p.H + stem::TH - 1) / stem::TH) * ((p.W + stem::TW - 1) / stem::TW);
  if (grid > ntot) grid = (int)ntot;
  const int mode = p.u8 ? (p.W % 4 == 0 ? 2 : 1) : 0;
  using L = int (*)(const StemParams&, int, hipStream_t);
  static const L f16[2][3] = {
      {stem::launch_t<_Float16, 0, 4>, stem::launch_t<_Float16, 1, 4>, stem::launch_t<_Float16, 2, 4>},
      {stem::launch_t<_Float16, 0, 1>, stem::launch_t<_Float16, 1, 1>, stem::launch_t<_Float16, 2, 1>}};
  static const L b16[2][3] = {
      {stem::launch_t<__bf16, 0, 4>, stem::launch_t<__bf16, 1, 4>, stem::launch_t<__bf16, 2, 4>},
      {stem::launch_t<__bf16, 0, 1>, stem::launch_t<__bf16, 1, 1>, stem::launch_t<__bf16, 2, 1>}};
  const int narrow = p.N <= 32 ? 1 : 0;
  if (dtype == F16) return f16[narrow][mode](p, grid, s);
  if (dtype == BF16) return b16[narrow][mode](p, grid, s);
  set_error("stem: fp16/bf16 only");
  return 1;
}

}  // namespace tv
