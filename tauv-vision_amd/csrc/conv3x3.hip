// Persistent halo-tile 3x3 / stride 1 / pad 1 convolution (gfx950, fp16 / bf16) — the
// dominant shape of the DLA backbone at 120x160 (IDA projection/output convs, tree conv1s,
// the stacked heads), reference dla.py ResidualBlock/IDAUp convs and centernet.py heads.
//
// Why not the implicit GEMM (conv_pipe.hip) for these: per 256-pixel tile the implicit GEMM
// moves each input pixel 9 times (once per tap) and the 295 KB weight panel once, ~880 KB of
// L2 -> LDS traffic per 75 MFLOP; measured, its main loop ran at ~21 B/clk/CU of LDS-DMA and
// its per-tile prologue (first ring stages from L2/HBM) and LDS-staged epilogue were exposed
// (tools/stamps.py: 13.5k + 41k + 9k cycles per tile against 18k of MFMA work).
//
// Design:
//  * one 256-thread workgroup per CU (4 waves, one per SIMD, 512 registers each), persistent
//    over a static list of (spatial tile, 128-channel tile) pairs, XCD-aware: each XCD owns a
//    contiguous tile range so neighbouring tiles (shared halo rows) meet in its L2;
//  * a tile = TH x TW = 512 output pixels of one frame x 128 output channels; each wave owns
//    128 pixels x 128 channels (4 x 4 tiles of v_mfma_f32_32x32x16, 256 accumulators);
//  * K order: channel blocks of 32 (64 B), 9 taps each. The (TH+2) x (TW+2) input halo of one
//    channel block moves into LDS ONCE (buffer_load ... lds: out-of-image and pad slots are
//    buffer-OOB, so they read as zero with no per-lane branches) and the 9 taps read shifted
//    windows of it at compile-time immediate ds_read offsets: 1.2x input traffic instead of 9x;
//  * two halo buffers (the next channel block — or the next tile's first — streams in during
//    taps 0..3 of the current one), a 4-slot weight ring (8 KiB per k-step, LDS-DMA), one raw
//    s_barrier per k-step with an exact counted vmcnt;
//  * fragments of k-step s+1 are read (16 ds_read_b128) while the 32 MFMAs of k-step s run;
//  * the epilogue stores straight from the accumulators (bias from LDS, activation, fp16/bf16
//    pack, v_permlane32_swap pairs into 16-byte stores), so the next tile's prefetched halo and
//    weights are already in flight while it runs: no per-tile prologue, no LDS staging.
// LDS: halo 2 x 48 KiB (pixel pitch 80 B = 64 B of channels + 16 B pad: conflict-free
// ds_read_b128 for 32-pixel rows), weight ring 4 x 8 KiB (XOR-swizzled 64 B rows), bias.
#include "conv_common.h"

#include <type_traits>

namespace tv {
namespace c3 {

constexpr int NT = 256, NW = 4, BN = 128, P = 512;
constexpr int CBK = 32;                       // channels per k-step
constexpr int PITCH = 80;                     // halo pixel pitch (bytes)
constexpr int HPIX = 612;                     // (16+2)x(32+2) = (32+2)x(16+2) halo pixels
constexpr int HPIECES = 48;                   // ceil(612 * 5 / 64) LDS-DMA pieces of 1 KiB
constexpr int HBUF = HPIECES * 1024;          // one halo buffer
constexpr int HPW = HPIECES / NW;             // halo pieces per wave per channel block = 12
constexpr int HCH = 3;                        // halo pieces per wave per k-step (taps 0..3)
constexpr int WSLOT = BN * 64;                // weights of one k-step: 128 rows x 64 B
constexpr int D = 4;                          // weight ring slots = weight prefetch distance
constexpr int WPW = WSLOT / 1024 / NW;        // weight pieces per wave per k-step = 2
constexpr int OFF_W = 2 * HBUF;
constexpr int OFF_B = OFF_W + D * WSLOT;
constexpr int LDS = OFF_B + kConv3MaxN * 4;
static_assert(HPW == 4 * HCH, "halo chunks");
static_assert(HPIECES * 64 >= HPIX * 5, "halo pieces");

typedef __attribute__((address_space(3))) char lds_char;
typedef const __attribute__((address_space(1))) void gvoid;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ void raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size, int voffset,
                                    int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ void dma16(const void* src, lds_char* dst) {
  __builtin_amdgcn_global_load_lds((gvoid*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
template <int OFF>
__device__ __forceinline__ u32x4 ds_read16(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt takes an immediate: dispatch the (wave-uniform, exact) count
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    default: wait_vm<13>(); break;
  }
}

template <int V>
using IC = std::integral_constant<int, V>;

struct Frags {
  u32x4 x[2][4];  // [sub-step j][pixel fragment f]
  u32x4 w[2][4];  // [sub-step j][channel fragment i]
};

// 16-byte store of 8 channels from two MFMA register groups (k, k+1) of one 32x32 tile:
// lanes 0-31 hold channels 8k+0..3 (group k) / 8k+8..11 (group k+1) of pixel l, lanes 32-63
// the +4 halves; one v_permlane32_swap per dword pair gives every lane 8 consecutive channels
// (lanes 0-31: group k, lanes 32-63: group k+1 of pixel l-32), stored at +8*lh channels.
template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}
template <typename T>
__device__ __forceinline__ void store_out(T* dst, const float (&v)[2][4], int lh) {
  const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
  const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
  const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
  gstore16(dst + 8 * lh, make_uint4(r0[0], r1[0], r0[1], r1[1]));
}

template <typename T, typename OutT, int TW, int ACT>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(1, 1))) void conv3x3(
    const ConvParams* __restrict__ pp, void* out_ptr) {
  constexpr int TH = P / TW;
  constexpr int RS = TW + 2;                               // halo row stride (pixels)
  constexpr int FOFF = (TW == 32 ? 1 : 2) * RS * PITCH;    // next 32-pixel fragment
  static_assert((TH + 2) * RS == HPIX, "halo shape");
  const ConvParams& p = *pp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;

  const ConvSegment& sg = p.seg[0];
  const int H = sg.H, W = sg.W, C = sg.C, ldc = sg.ldc;
  const int tiles_x = (W + TW - 1) / TW;
  const int tiles_f = ((H + TH - 1) / TH) * tiles_x;
  const int ntiles = p.ntiles;
  const int ntot = p.mtiles * ntiles;
  constexpr int NCB = 128 / CBK;  // channel blocks per tile (C == 128, host check)
  const int spt = 9 * NCB;        // k-steps per tile

  // ---- this block's tiles: XCD-aware contiguous ranges
  const int G = gridDim.x, bid = blockIdx.x;
  int first, stride, end;
  if ((G & 7) == 0) {
    const int per = G >> 3, xcd = bid & 7;
    first = (int)((long long)ntot * xcd / 8) + (bid >> 3);
    end = (int)((long long)ntot * (xcd + 1) / 8);
    stride = per;
  } else {
    first = bid;
    end = ntot;
    stride = G;
  }
  const int ntl = first < end ? (end - first + stride - 1) / stride : 0;
  if (ntl == 0) return;
  const int S_tot = ntl * spt;

  // bias of every output channel into LDS (read in the epilogues)
  float* lbias = reinterpret_cast<float*>(smem + OFF_B);
  for (int c = tid; c < ntiles * BN; c += NT) lbias[c] = c < p.N ? p.bias[c] : 0.0f;

  // ---- sources
  const T* src = reinterpret_cast<const T*>(sg.src);
  i32x4 rsrc;
  {
    const unsigned long long a = (unsigned long long)src;
    rsrc.x = (int)(unsigned)a;
    rsrc.y = (int)(unsigned)(a >> 32);
    rsrc.z = (int)(unsigned)((unsigned long long)p.M * ldc * sizeof(T));  // bytes (host checks < 2^31)
    rsrc.w = 0x00020000;
  }
  const T* wts = reinterpret_cast<const T*>(p.weight);
  const int Kpad = p.Kpad;

  // ---- tile decode
  auto tile_of = [&](int idx, int& fr, int& y0, int& x0, int& n0) __attribute__((always_inline)) {
    const int t = first + idx * stride;
    const int nt = t % ntiles, mt = t / ntiles;
    fr = mt / tiles_f;
    const int r = mt - fr * tiles_f;
    const int ty = r / tiles_x;
    y0 = ty * TH;
    x0 = (r - ty * tiles_x) * TW;
    n0 = nt * BN;
  };

  // ---- halo DMA: chunk g = piece*64 + lane -> halo pixel g/5, slot g%5 (slot 4 = pad).
  // Tile-independent geometry packed once per lane and piece: hy<<16 | hx<<8 | slot, or ~0.
  unsigned hgeo[HPW], hoff[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int g = (wave * HPW + i) * 64 + lane;
    const int h = g / 5, s5 = g - (g / 5) * 5;
    const int hy = h / RS, hx = h - (h / RS) * RS;
    hgeo[i] = (s5 < 4 && h < HPIX) ? (unsigned)((hy << 16) | (hx << 8) | s5) : ~0u;
  }
  const unsigned pix_bytes = (unsigned)ldc * (unsigned)sizeof(T);
  auto halo_offsets = [&](int fr, int y0, int x0) __attribute__((always_inline)) {
    const int ybase = fr * H;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const unsigned gq = hgeo[i];
      const int y = y0 - 1 + (int)(gq >> 16);
      const int x = x0 - 1 + (int)((gq >> 8) & 0xff);
      const bool ok = gq != ~0u && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      hoff[i] = ok ? ((unsigned)(ybase + y) * (unsigned)W + (unsigned)x) * pix_bytes + (gq & 0xff) * 16u
                   : 0x80000000u;
    }
  };
  auto issue_halo = [&](auto chunk, int cb, int bsel) __attribute__((always_inline)) {
    lds_char* base = lds + bsel * HBUF + wave * HPW * 1024;
#pragma unroll
    for (int k = 0; k < HCH; ++k) {
      const int i = decltype(chunk)::value * HCH + k;
      raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(base + i * 1024), 16, (int)hoff[i],
                          cb * CBK * (int)sizeof(T), 0, 0);
    }
  };

  // ---- weight DMA: piece = 16 rows x 64 B; lane -> row piece*16 + lane/4, slot lane%4 holds
  // chunk slot ^ ((row>>2)&3) (conflict-free ds_read_b128 of 32-row fragments)
  unsigned woff[WPW];
#pragma unroll
  for (int k = 0; k < WPW; ++k) {
    const int row = (wave * WPW + k) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    woff[k] = (unsigned)(row * Kpad + chunk * 8) * sizeof(T);
  }
  // weight issue cursor: (tile index, channel block, tap) of the next k-step to stream
  int wc_idx = 0, wc_cb = 0, wc_tap = 0, wc_n0 = 0, wc_q = 0;
  {
    int a, b_, c_;
    tile_of(0, a, b_, c_, wc_n0);
  }
  auto issue_w = [&]() __attribute__((always_inline)) {
    const char* base =
        reinterpret_cast<const char*>(wts + (size_t)wc_n0 * Kpad + wc_tap * C + wc_cb * CBK);
    lds_char* dst = lds + OFF_W + (wc_q % D) * WSLOT + wave * WPW * 1024;
#pragma unroll
    for (int k = 0; k < WPW; ++k) dma16(base + woff[k], dst + k * 1024);
    ++wc_q;
    if (++wc_tap == 9) {
      wc_tap = 0;
      if (++wc_cb == NCB) {
        wc_cb = 0;
        if (++wc_idx < ntl) {
          int a, b_, c_;
          tile_of(wc_idx, a, b_, c_, wc_n0);
        }
      }
    }
  };

  // ---- fragment addresses
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  unsigned xa;  // pixel 128*wave + l32 of the tile, tap (0,0), lane-half chunk
  {
    const int q = 128 * wave + l32;
    const int r = q / TW, c = q - (q / TW) * TW;
    xa = lds0 + (unsigned)((r * RS + c) * PITCH + lh * 16);
  }
  unsigned wa[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    wa[j] = lds0 + OFF_W + (unsigned)(l32 * 64 + (((2 * j + lh) ^ ((l32 >> 2) & 3)) << 4));

  auto read_frags = [&](auto tap, int bsel, int slot, Frags& F) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tap)::value;
    constexpr int TOFF = ((TAP / 3) * RS + (TAP % 3)) * PITCH;
    const unsigned xb = xa + bsel * HBUF;
    const unsigned wb0 = wa[0] + slot * WSLOT, wb1 = wa[1] + slot * WSLOT;
    F.x[0][0] = ds_read16<TOFF + 0 * FOFF>(xb);
    F.x[0][1] = ds_read16<TOFF + 1 * FOFF>(xb);
    F.x[0][2] = ds_read16<TOFF + 2 * FOFF>(xb);
    F.x[0][3] = ds_read16<TOFF + 3 * FOFF>(xb);
    F.w[0][0] = ds_read16<0 * 2048>(wb0);
    F.w[0][1] = ds_read16<1 * 2048>(wb0);
    F.w[0][2] = ds_read16<2 * 2048>(wb0);
    F.w[0][3] = ds_read16<3 * 2048>(wb0);
    F.x[1][0] = ds_read16<TOFF + 32 + 0 * FOFF>(xb);
    F.x[1][1] = ds_read16<TOFF + 32 + 1 * FOFF>(xb);
    F.x[1][2] = ds_read16<TOFF + 32 + 2 * FOFF>(xb);
    F.x[1][3] = ds_read16<TOFF + 32 + 3 * FOFF>(xb);
    F.w[1][0] = ds_read16<0 * 2048>(wb1);
    F.w[1][1] = ds_read16<1 * 2048>(wb1);
    F.w[1][2] = ds_read16<2 * 2048>(wb1);
    F.w[1][3] = ds_read16<3 * 2048>(wb1);
  };

  f32x16 acc[4][4];  // [pixel fragment f][channel fragment i]
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[f][i] = f32x16{};

  auto mfmas = [&](const Frags& F) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int f = 0; f < 4; ++f) Mfma<T>::run(to_u4(F.w[j][i]), to_u4(F.x[j][f]), acc[f][i]);
  };

  // ---- epilogue of the tile (fr, y0, x0, n0): straight from the accumulators
  auto epilogue = [&](int fr, int y0, int x0, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int q = 128 * wave + 32 * f + l32;
      const int y = y0 + q / TW, x = x0 + q % TW;
      const bool ok = y < H && x < W;
      OutT* dst = reinterpret_cast<OutT*>(out_ptr) +
                  ((size_t)(fr * H + (ok ? y : 0)) * W + (ok ? x : 0)) * p.out_ldc + p.out_coff + n0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float v[2][4];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int G2 = 2 * m + gg;
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lbias + n0 + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = acc[f][i][4 * G2 + e] + bb[e];
              if constexpr (ACT == 1) t = fmaxf(t, 0.0f);
              else if constexpr (ACT == 2) t = fmaxf(t, 0.01f * t);  // == (t >= 0 ? t : 0.01t)
              v[gg][e] = t;
            }
          }
          const int ch = n0 + 32 * i + 16 * m;
          if (ok && ch < p.N) store_out<OutT>(dst + 32 * i + 16 * m, v, lh);
          __builtin_amdgcn_sched_barrier(0);  // bound the live set: one 8-channel group at a time
        }
      }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[f][i] = f32x16{};
  };

  // ---- prologue: halo of (tile 0, block 0), weights of k-steps 0..D-1
  int cur_fr, cur_y0, cur_x0, cur_n0;
  tile_of(0, cur_fr, cur_y0, cur_x0, cur_n0);
  halo_offsets(cur_fr, cur_y0, cur_x0);
  issue_halo(IC<0>{}, 0, 0);
  issue_halo(IC<1>{}, 0, 0);
  issue_halo(IC<2>{}, 0, 0);
  issue_halo(IC<3>{}, 0, 0);
  for (int q = 0; q < D; ++q)
    if (q < S_tot) issue_w();
  {
    const int younger = 2 * (S_tot - 1 < D - 1 ? S_tot - 1 : D - 1);  // weights 1..D-1
    wait_vm_n(younger);
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  Frags F0, F1;
  read_frags(IC<0>{}, 0, 0, F0);

  int s = 0;   // global k-step
  int tl = 0;  // tile index within this block's list
  int cb = 0;  // channel block within the tile (compile-time inside cblock)
  // the channel block after the current one: same tile cb+1, or the next tile's block 0
  bool nxt_exists = true, nxt_newtile = false;

  // one k-step with compile-time tap; Fc holds its fragments, Fn receives the next k-step's.
  // Halo buffer of channel block cb is cb & 1 (NCB is even, so parity is per-tile fixed).
  auto step = [&](auto tap, Frags& Fc, Frags& Fn) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tap)::value;
    // LDS-DMA instructions issued after weights(s+1): weights of s+2, s+3 (steps s-2, s-1),
    // halo chunks at steps s-3..s-1 that had tap <= 3 (same channel block)
    constexpr int hsteps = (TAP >= 1 && TAP <= 3) ? TAP : (TAP >= 4 && TAP <= 6 ? 7 - TAP : 0);
    const int wyoung = 2 * ((s + 2 < S_tot) + (s + 3 < S_tot));
    const int younger = wyoung + (nxt_exists ? HCH * hsteps : 0);
    wait_vm_n(s + 1 < S_tot ? younger : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + D < S_tot) issue_w();
    if constexpr (TAP <= 3) {
      if (nxt_exists) {
        if constexpr (TAP == 0) {
          if (nxt_newtile) {
            int fr, y0, x0, n0;
            tile_of(tl + 1, fr, y0, x0, n0);
            halo_offsets(fr, y0, x0);
          }
        }
        issue_halo(IC<TAP>{}, nxt_newtile ? 0 : cb + 1, (cb + 1) & 1);
      }
    }
    if (s + 1 < S_tot) {
      if constexpr (TAP == 8) read_frags(IC<0>{}, (cb + 1) & 1, (s + 1) % D, Fn);
      else read_frags(IC<TAP + 1>{}, cb & 1, (s + 1) % D, Fn);
    }
    mfmas(Fc);
    ++s;
  };

  auto cblock = [&](auto cbc, Frags& Fa, Frags& Fb) __attribute__((always_inline)) {
    constexpr int CB = decltype(cbc)::value;
    cb = CB;
    nxt_newtile = CB + 1 == NCB;
    nxt_exists = !nxt_newtile || tl + 1 < ntl;
    step(IC<0>{}, Fa, Fb);
    step(IC<1>{}, Fb, Fa);
    step(IC<2>{}, Fa, Fb);
    step(IC<3>{}, Fb, Fa);
    step(IC<4>{}, Fa, Fb);
    step(IC<5>{}, Fb, Fa);
    step(IC<6>{}, Fa, Fb);
    step(IC<7>{}, Fb, Fa);
    step(IC<8>{}, Fa, Fb);
  };

  // NCB = 4 channel blocks per tile, fully unrolled (36 k-steps of straight-line code): the
  // accumulators keep one register assignment through the whole tile
  static_assert(NCB == 4, "tile body is unrolled for 4 channel blocks");
  for (; tl < ntl;) {
    cblock(IC<0>{}, F0, F1);
    cblock(IC<1>{}, F1, F0);
    cblock(IC<2>{}, F0, F1);
    cblock(IC<3>{}, F1, F0);
    epilogue(cur_fr, cur_y0, cur_x0, cur_n0);
    ++tl;
    if (tl < ntl) tile_of(tl, cur_fr, cur_y0, cur_x0, cur_n0);
  }
}

template <typename T, int TW, int ACT>
static int launch_t(const ConvParams& p, const ConvParams* dp, void* out, int grid, hipStream_t s) {
  auto k = conv3x3<T, T, TW, ACT>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) {
      set_error(std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
      return 3;
    }
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), LDS, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace c3

int conv3x3_tiles(int B, int H, int W, int tw) {
  const int th = c3::P / tw;
  return B * ((H + th - 1) / th) * ((W + tw - 1) / tw);
}

int launch_conv3x3(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid,
                   hipStream_t s) {
  using namespace c3;
  if (p.act < 0 || p.act > 2) {
    set_error("conv3x3: bad activation");
    return 1;
  }
  using L = int (*)(const ConvParams&, const ConvParams*, void*, int, hipStream_t);
  static const L f16[2][3] = {{launch_t<_Float16, 16, 0>, launch_t<_Float16, 16, 1>, launch_t<_Float16, 16, 2>},
                              {launch_t<_Float16, 32, 0>, launch_t<_Float16, 32, 1>, launch_t<_Float16, 32, 2>}};
  static const L b16[2][3] = {{launch_t<__bf16, 16, 0>, launch_t<__bf16, 16, 1>, launch_t<__bf16, 16, 2>},
                              {launch_t<__bf16, 32, 0>, launch_t<__bf16, 32, 1>, launch_t<__bf16, 32, 2>}};
  if (dtype == F16) return f16[tw == 32][p.act](p, dp, out, grid, s);
  if (dtype == BF16) return b16[tw == 32][p.act](p, dp, out, grid, s);
  set_error("conv3x3: fp16/bf16 only");
  return 1;
}

}  // namespace tv
