// ConvTranspose2d(3, stride 2, padding 1, output_padding 1) on a shared input halo (gfx950, fp16 /
// bf16): the YOLACT protonet's up-sampling layers (masknet.py:21,33, `_upsample_layer_{1,2}` +
// LeakyReLU) as ONE launch per layer.
//
// Output parity (pi, pj) of pixel (2m + pi, 2n + pj) is a (1 + pi) x (1 + pj) conv with no padding
// over the low-resolution input: tap (dy, dx) reads input (m + dy, n + dx) with kernel element
// ky = 1 (pi = 0) or 2 - 2 dy (pi = 1), kx likewise. The four phases together use 9 (phase, tap)
// products per input pixel and channel, over only 4 distinct input shifts (0 / 1 per axis) — a
// 3x3 conv's reuse, but the round-4 engine ran them as 4 separate implicit GEMMs (conv_pipe: the
// input read once per phase, 1-4 taps of K per launch: ~430 TFLOP/s).
//
// Here a workgroup (8 waves, one per CU, persistent over a static, XCD-contiguous unit list) owns a
// tile of tw x tr <= 256 input pixels (shape chosen per layer: convt3_tile) x 64 output channels x
// all 4 phases: wave w owns tile pixels 32 w .. 32 w + 31 in raster order (two 16-pixel fragments,
// which may span tile rows) x 64 channels x 4 phases = 32 accumulators of v_mfma_f32_16x16x32
// (128 VGPRs). K order: channel blocks of 32; per block the (tw + 1) x (tr + 1) input halo moves
// into LDS once (LDS-DMA, 80-byte pixel pitch, out-of-image pixels and the pad slot buffer-OOB
// zeros) together with the block's 9 (phase, tap) weight fragments x 64 channels (36 KiB, pre-packed
// in MFMA A-operand lane order: one contiguous 1 KiB LDS-DMA piece per fragment) and, with a unit's
// last block, its biases; the next block (or the next unit's first) streams into the other buffer
// set under the current block's 72 MFMAs per wave, whose weight fragments come through a ring of
// registers CT3_WD fragments ahead. One raw barrier per block (counted vmcnt: a unit's epilogue
// stores stay in flight across it). The input fragments use conv3x3.hip's conflict-free lane
// permutation (pixel pi(n), 16-byte chunk sigma(c)); the weights carry the matching channel order.
// Epilogue from the accumulators: bias, activation, one rounding, v_permlane16_swap into 16-byte
// stores of each phase's output pixels (2m + pi, 2n + pj).
#include "conv_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace tv {
namespace ct3 {

constexpr int NT = 512, NW = 8;
constexpr int HPIECES = 24;                   // LDS-DMA pieces of 1 KiB per halo (3 per wave)
constexpr int PITCH = 80;                     // 32 channels (64 B) + 16 B pad per halo pixel
constexpr int HPIX_MAX = HPIECES * 64 / 5;    // 307 halo pixels: (tw + 1) (tr + 1) <= 307
constexpr int HBUF = HPIECES * 1024;
constexpr int NCO = 64;                       // output channels per unit
constexpr int NQ = 9;                         // (phase, tap) products
constexpr int WPIECES = NQ * (NCO / 16);      // 36 fragments of 1 KiB per channel block
constexpr int WBUF = WPIECES * 1024;
constexpr int OFF_W = 2 * HBUF;
constexpr int OFF_B = OFF_W + 2 * WBUF;
constexpr int LDS = OFF_B + 2 * NCO * 4;  // (a bias slot per buffer set)
static_assert(LDS <= 160 * 1024, "LDS budget");
constexpr int OOB = (int)0x80000000u;
#ifndef CT3_WD
#define CT3_WD 8   // weight fragments in flight per wave (ring depth)
#endif
#ifndef CT3_SCHED
#define CT3_SCHED 1
#endif

// (phase, tap) q: the phase p = 2 pi + pj and the tap t = 2 dy + dx it multiplies; the order the
// packed weights use (taps grouped: tap 0 serves all 4 phases, taps 1 / 2 two, tap 3 one)
constexpr int Q_PH[NQ] = {0, 1, 2, 3, 1, 3, 2, 3, 3};
constexpr int Q_TAP[NQ] = {0, 0, 0, 0, 1, 1, 2, 2, 3};

typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
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
__device__ __forceinline__ u32x4 lds16(unsigned addr) { return *reinterpret_cast<lds_u32x4*>(addr); }

// conv3x3.hip's 16x16x32 lane permutation: fragment column n reads pixel pi(n), K group c reads
// 16-byte chunk sigma(c) (ds_read_b128 lane groups on distinct 4-bank sets at the 80-byte pitch)
__host__ __device__ constexpr int sigma16(int c) { return ((c & 1) << 1) | (c >> 1); }
__device__ __forceinline__ int pi16(int n) { return n < 4 ? 2 * n : n < 12 ? 2 * n - 7 : 2 * n - 16; }

template <typename T> struct Mf;
template <> struct Mf<_Float16> {
  __device__ static void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0, 0, 0);
  }
};
template <> struct Mf<__bf16> {
  __device__ static void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

template <int V>
using IC = std::integral_constant<int, V>;

template <typename T, int ACT>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void convt3(ConvT3Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* lds = (lds_char*)smem;
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n16 = lane & 15, c16 = lane >> 4;
  const int pin = pi16(n16), sig = sigma16(c16);

  const int H = p.H, W = p.W;
  const int tw = p.tw, tr = p.tr, HS = tw + 1;  // input tile (columns, rows); halo row stride
  const int tiles_x = (W + tw - 1) / tw, tiles_y = (H + tr - 1) / tr;
  const int nco = p.N / NCO;
  const int ncb = p.C / 32;
  const int nunits = p.B * tiles_y * tiles_x * nco;
  // XCD-aware contiguous unit ranges (the channel tiles of an input tile adjacent: the same halo)
  const int G = gridDim.x, bid = blockIdx.x;
  int first, stride, end;
  if ((G & 7) == 0) {
    first = (int)((long long)nunits * (bid & 7) / 8) + (bid >> 3);
    end = (int)((long long)nunits * ((bid & 7) + 1) / 8);
    stride = G >> 3;
  } else {
    first = bid;
    end = nunits;
    stride = G;
  }
  if (first >= end) return;
  auto unit_of = [&](int u, int& fr, int& y0, int& x0, int& co) __attribute__((always_inline)) {
    co = u % nco;
    int t = u / nco;
    const int tx = t % tiles_x;
    t /= tiles_x;
    const int ty = t % tiles_y;
    fr = t / tiles_y;
    y0 = ty * tr;
    x0 = tx * tw;
  };

  const unsigned frame_bytes = (unsigned)H * W * p.ldc * (unsigned)sizeof(T);
  // this lane's 16-byte chunk of each of the wave's 3 halo pieces: halo pixel (hy, hx), channel
  // slot s5 (slot 4 = the pad: never loaded); hy = -1 marks a chunk outside the halo
  int hy_k[3], hx_k[3], s5_k[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int g = (wave + k * NW) * 64 + lane;
    const int h = g / 5;
    s5_k[k] = g - h * 5;
    hy_k[k] = h / HS;
    hx_k[k] = h - hy_k[k] * HS;
    if (s5_k[k] == 4 || hy_k[k] > tr) hy_k[k] = -1;
  }
  const i32x4 wrs = rsrc_of(p.w, (unsigned)(nco * ncb * WBUF));
  const i32x4 brs = rsrc_of(p.bias, (unsigned)(p.N * 4));
  // a unit's staging geometry, computed once per unit: the frame's buffer resource, this lane's
  // byte offsets of its 3 halo chunks at channel block 0 (OOB outside the frame / halo), the
  // weight and bias bases of its channel tile
  struct Geo {
    i32x4 rs;
    int hoff[3];
    int wblk0, boff;
  };
  auto geo = [&](int u) __attribute__((always_inline)) {
    int fr, y0, x0, co;
    unit_of(u, fr, y0, x0, co);
    Geo g;
    g.rs = rsrc_of(reinterpret_cast<const char*>(p.src) + (size_t)fr * frame_bytes, frame_bytes);
#pragma unroll
    for (int k = 0; k < HPIECES / NW; ++k) {
      const int y = y0 + hy_k[k], x = x0 + hx_k[k];
      const bool ok = hy_k[k] >= 0 && y < H && x < W;
      g.hoff[k] = ok ? (int)((((unsigned)y * W + x) * p.ldc + s5_k[k] * 8) * sizeof(T)) : OOB;
    }
    g.wblk0 = co * ncb * WBUF;
    g.boff = (co * NCO + lane) * 4;
    return g;
  };
  // stage (unit geometry g, channel block cb) into buffer set bs: the halo pieces, the weight
  // pieces, with a unit's last block its biases
  auto stage = [&](const Geo& g, int cb, int bs, bool first_stage = false) __attribute__((always_inline)) {
    (void)first_stage;
#pragma unroll
    for (int k = 0; k < HPIECES / NW; ++k) {
      const int q = wave + k * NW;
#if defined(TV_CT3_EXP) && (TV_CT3_EXP == 2 || TV_CT3_EXP == 3)
      if (!first_stage) continue;  // timing experiment: stale halo
#endif
      raw_buffer_load_lds(g.rs, (__attribute__((address_space(3))) void*)(lds + bs * HBUF + q * 1024), 16,
                          g.hoff[k] + cb * 32 * (int)sizeof(T), 0, 0, 0);
    }
    const int wblk = g.wblk0 + cb * WBUF;
#pragma unroll
    for (int k = 0; k < (WPIECES + NW - 1) / NW; ++k) {
      const int q = wave + k * NW;
      if (q >= WPIECES) break;
#if defined(TV_CT3_EXP) && (TV_CT3_EXP == 1 || TV_CT3_EXP == 3)
      if (!first_stage) continue;  // timing experiment: stale weights
#endif
      raw_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(lds + OFF_W + bs * WBUF + q * 1024), 16,
                          wblk + q * 1024 + lane * 16, 0, 0, 0);
    }
    // (the slot's next fill is two stages later, past a barrier)
    if (cb == ncb - 1 && wave == 0)
      raw_buffer_load_lds(brs, (__attribute__((address_space(3))) void*)(lds + OFF_B + bs * NCO * 4), 4, g.boff, 0, 0,
                          0);
  };

  f32x4 acc[4][4][2];  // [phase][16-channel fragment][pixel fragment]
  // this lane's pixel of fragment f: tile pixel 32 wave + 16 f + pi(n) in raster order over the tw x tr
  // tile (past its end: the last pixel again, computed and not stored), chunk sigma(c)
  int pr[2], pc[2];
  bool pv[2];
  unsigned xrel[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int px = 32 * wave + 16 * f + pin;
    pv[f] = px < tw * tr;
    if (!pv[f]) px = tw * tr - 1;
    pr[f] = px / tw;
    pc[f] = px - pr[f] * tw;
    xrel[f] = (unsigned)((pr[f] * HS + pc[f]) * PITCH + sig * 16);
  }
  const unsigned tapoff[4] = {0u, (unsigned)PITCH, (unsigned)(HS * PITCH), (unsigned)((HS + 1) * PITCH)};

  // one channel block from buffer set bs: the 4 taps' input fragments up front, then the 36
  // weight fragments in packing order (q-major: tap 0's four phases first) through a ring of
  // WD registers, each read WD fragments (2 WD MFMAs) ahead of its use; the schedule barriers keep
  // the compiler from sinking the reads next to their MFMAs (LDS latency exposed per pair)
  auto block = [&](int bs) __attribute__((always_inline)) {
    const unsigned hb = lds0 + (unsigned)(bs * HBUF);
    const unsigned wb = lds0 + (unsigned)(OFF_W + bs * WBUF) + (unsigned)lane * 16u;
    constexpr int WD = CT3_WD;
    u32x4 X[4][2], Wr[WD];
#pragma unroll
    for (int i = 0; i < WD; ++i) Wr[i] = lds16(wb + (unsigned)(i * 1024));
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int f = 0; f < 2; ++f) X[t][f] = lds16(hb + xrel[f] + tapoff[t]);
#pragma unroll
    for (int i = 0; i < WPIECES; ++i) {
      const int q = i >> 2, c = i & 3;
      const u32x4 wf = Wr[i % WD];
      if (i + WD < WPIECES) Wr[i % WD] = lds16(wb + (unsigned)((i + WD) * 1024));
#pragma unroll
      for (int f = 0; f < 2; ++f) {
#if defined(TV_CT3_EXP) && TV_CT3_EXP == 4
        acc[Q_PH[q]][c][f][0] += __builtin_bit_cast(float, wf[0] ^ X[Q_TAP[q]][f][1]);  // timing experiment: no MFMA
#else
        Mf<T>::run(acc[Q_PH[q]][c][f], wf, X[Q_TAP[q]][f]);
#endif
      }
    }
#if CT3_SCHED
    // order: the WD + 8 prologue reads, then per fragment (one read, two MFMAs), then the last MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, WD + 8, 0);
#pragma unroll
    for (int i = 0; i < WPIECES - WD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * WD, 0);
#endif
  };

  // bias + activation + 16-byte stores of the unit's 4 phases (conv3x3.hip epilogue16 layout:
  // lane (c, n) holds channels 16 i + 4 c + e of pixel pi(n); one v_permlane16_swap per dword of a
  // channel-fragment pair gives every lane 8 consecutive channels at 16 (c & 1) + 8 (c >> 1))
  const int cofs16 = 16 * (c16 & 1) + 8 * (c16 >> 1);
  const int tH = 2 * H, tW = 2 * W;
  const unsigned out_frame = (unsigned)tH * tW * p.out_ldc * (unsigned)sizeof(T);
  auto epilogue = [&](int u, int bs) __attribute__((always_inline)) {
    int fr, y0, x0, co;
    unit_of(u, fr, y0, x0, co);
    const float* lb = reinterpret_cast<const float*>(smem + OFF_B + bs * NCO * 4);
    const i32x4 ors = rsrc_of(reinterpret_cast<const char*>(p.out) + (size_t)fr * out_frame, out_frame);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int y = y0 + pr[f], x = x0 + pc[f];
      const bool ok = pv[f] && y < H && x < W;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int ty = 2 * y + (ph >> 1), tx = 2 * x + (ph & 1);
        const int obase = ok ? (int)((((unsigned)ty * tW + tx) * p.out_ldc + co * NCO + cofs16) * sizeof(T)) : OOB;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v[2][4];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + 32 * j + 16 * hh + 4 * c16);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = acc[ph][2 * j + hh][f][e] + bb[e];
              if constexpr (ACT == 1) t = fmaxf(t, 0.0f);
              else if constexpr (ACT == 2) t = fmaxf(t, 0.01f * t);
              v[hh][e] = t;
            }
          }
          const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
          const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
          const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
          raw_buffer_store_v4(u32x4{r0[0], r1[0], r0[1], r1[1]}, ors,
                              ok ? obase + (int)(32 * j * sizeof(T)) : OOB, 0, 0);
        }
      }
    }
  };

  // ---- the unit list: stage (first, 0); per block stage the next (block or unit) under compute
  Geo gcur = geo(first);
  stage(gcur, 0, 0, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int bs = 0;
  for (int u = first; u < end; u += stride) {
    const bool more = u + stride < end;
    const Geo gnext = geo(more ? u + stride : u);
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[ph][c][f] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int cb = 0; cb < ncb; ++cb) {
      if (cb + 1 < ncb) stage(gcur, cb + 1, bs ^ 1);
      else if (more) stage(gnext, 0, bs ^ 1);
      block(bs);
      // (raw barriers: __syncthreads()'s fence would wait for every outstanding store)
      if (cb + 1 == ncb) {
        epilogue(u, bs);
        // the next stage's LDS-DMA (issued before the epilogue's 16 stores) has landed once at most
        // the 16 stores are outstanding (vector memory ops retire in issue order): the stores
        // drain under the next unit's first block instead of stalling this barrier
        asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      bs ^= 1;
    }
    gcur = gnext;
  }
}

template <typename T, int ACT>
static int launch_a(const ConvT3Params& p, int grid, hipStream_t s) {
  if (int r = ensure_lds<convt3<T, ACT>>(LDS)) return r;
  hipLaunchKernelGGL((convt3<T, ACT>), dim3(grid), dim3(NT), LDS, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}
template <typename T>
static int launch_t(const ConvT3Params& p, int grid, hipStream_t s) {
  return p.act == 1 ? launch_a<T, 1>(p, grid, s) : p.act == 2 ? launch_a<T, 2>(p, grid, s) : launch_a<T, 0>(p, grid, s);
}

}  // namespace ct3

bool convt3_supported(int C, int N, int ldc, int out_ldc, int H, int W, int esz) {
  return esz == 2 && C % 32 == 0 && C >= 32 && N % ct3::NCO == 0 && ldc % 8 == 0 && out_ldc % 8 == 0 &&
         (size_t)H * W * ldc * 2 < (1ull << 31) && (size_t)4 * H * W * out_ldc * 2 < (1ull << 31);
}

size_t convt3_weight_bytes(int C, int N) { return (size_t)(N / ct3::NCO) * (C / 32) * ct3::WBUF; }

// host: pack a ConvTranspose2d(3, s2, p1) weight [C][N][3][3] (fp32) into the kernel's fragments,
// element (co tile, channel block cb, q, fragment c, lane l = 16 kc + m, e) =
// W[ci = 32 cb + 8 sigma(kc) + e][co = 64 tile + 16 c + m][ky][kx] of q's (phase, tap)
void convt3_pack(const float* w, int C, int N, int dtype, void* out) {
  using namespace ct3;
  const int ncb = C / 32, nco = N / NCO;
  auto put = [&](size_t i, float v) {
    if (dtype == F16) {
      reinterpret_cast<_Float16*>(out)[i] = (_Float16)v;
    } else {
      uint32_t u;
      std::memcpy(&u, &v, 4);
      if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) u = (u >> 16) | 0x40;
      else u = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
      reinterpret_cast<uint16_t*>(out)[i] = (uint16_t)u;
    }
  };
  for (int t = 0; t < nco; ++t)
    for (int cb = 0; cb < ncb; ++cb)
      for (int q = 0; q < NQ; ++q) {
        const int ph = Q_PH[q], tp = Q_TAP[q];
        const int pi = ph >> 1, pj = ph & 1, dy = tp >> 1, dx = tp & 1;
        const int ky = pi == 0 ? 1 : 2 - 2 * dy, kx = pj == 0 ? 1 : 2 - 2 * dx;
        for (int c = 0; c < 4; ++c)
          for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) {
              const int m = l & 15, kc = l >> 4;
              const int ci = 32 * cb + 8 * sigma16(kc) + e, co = NCO * t + 16 * c + m;
              const size_t i = ((((size_t)(t * ncb + cb) * NQ + q) * 4 + c) * 64 + l) * 8 + e;
              put(i, w[(((size_t)ci * N + co) * 3 + ky) * 3 + kx]);
            }
      }
}

// the input tile: tw x tr <= 256 pixels (16 MFMA fragments), halo (tw + 1) (tr + 1) <= 307 pixels,
// fewest tiles over the H x W grid, ties to the larger tile, then the squarer one
void convt3_tile(int H, int W, int* tw, int* tr) {
  long best = -1;
  int bw = 16, br = 16;
  for (int w = 4; w <= 64; ++w) {
    int r = 256 / w;
    while (r > 1 && (w + 1) * (r + 1) > ct3::HPIX_MAX) --r;
    if ((w + 1) * (r + 1) > ct3::HPIX_MAX) continue;
    const long tiles = (long)((H + r - 1) / r) * ((W + w - 1) / w);
    const long key = tiles * 1000000L - (long)w * r * 1000 + std::abs(w - r);
    if (best < 0 || key < best) best = key, bw = w, br = r;
  }
  *tw = bw;
  *tr = br;
}

int launch_convt3(const ConvT3Params& p_in, int dtype, int cu_count, hipStream_t s) {
  using namespace ct3;
  ConvT3Params p = p_in;
  if (p.tw <= 0 || p.tr <= 0) convt3_tile(p.H, p.W, &p.tw, &p.tr);
  if (p.tw * p.tr > 256 || (p.tw + 1) * (p.tr + 1) > HPIX_MAX) {
    set_error("convt3: tile too large");
    return 1;
  }
  if (!convt3_supported(p.C, p.N, p.ldc, p.out_ldc, p.H, p.W, dtype_size(dtype)) || !p.src || !p.w || !p.out ||
      !p.bias || p.B < 1 || p.H < 1 || p.W < 1 || p.act < 0 || p.act > 2) {
    set_error("convt3: unsupported layer");
    return 1;
  }
  const long units = (long)p.B * ((p.H + p.tr - 1) / p.tr) * ((p.W + p.tw - 1) / p.tw) * (p.N / NCO);
  int grid = (int)std::min<long>(units, cu_count);
  if (grid >= 8 && units > 2L * grid) grid -= grid % 8;
  if (dtype == F16) return launch_t<_Float16>(p, grid, s);
  if (dtype == BF16) return launch_t<__bf16>(p, grid, s);
  set_error("convt3: fp16/bf16 only");
  return 1;
}

}  // namespace tv
