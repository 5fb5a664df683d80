// Persistent halo-tile 3x3 / stride 2 / pad 1 convolution (gfx950, fp16 / bf16): the
// downsampling ResidualBlock conv1 of the reference DLA (dla.py:13-19 with stride 2; DLADown's
// block_layers and each Tree's first block, dla.py:100-135, 170-180) at 128 channels.
//
// Why not the implicit GEMM (conv_pipe.hip): it moves every input pixel from L2 to LDS once per
// tap (9x), which left it LDS-DMA-bound at ~620 TFLOP/s on the 480x640 -> 240x320 block. This
// kernel keeps conv3x3.hip's structure (persistent 512-thread workgroups, 512-pixel x 128-channel
// tiles, 8 waves of 64 pixels x 128 channels on v_mfma_f32_32x32x16, register-staged weight
// ring, one s_barrier per k-step) and reads each input pixel into LDS once per tile:
//  * virtual space-to-depth: a stride-2 3x3 conv is the sum over the four input phases
//    (row, column parity) (p, q) of stride-1 convs with 1 or 2 taps per axis. Tap (ky, kx) of
//    output pixel (oy, ox) reads input row 2oy - 1 + ky, of row phase p = (ky + 1) & 1. The halo
//    of phase block (p, q) holds plane pixels (oy0 - p + hy, ox0 - q + hx), i.e. input pixels
//    (2(oy0 - p + hy) + p, 2(ox0 - q + hx) + q), and the tap is the halo offset
//    (ty, tx) = ((ky + p - 1) / 2, (kx + q - 1) / 2) in {0, 1}^2 — the same immediate-offset
//    fragment reads as the stride-1 kernel;
//  * per 32-channel block the four phase blocks are (1,1) [4 taps], (1,0) [2], (0,1) [2],
//    (0,0) [1] = 9 k-steps; each block's halo (<= 17 x 33 pixels, 80 B pitch) moves into LDS by
//    buffer_load ... lds with per-lane source addresses (out-of-image pixels read as zero);
//  * three halo buffers: block n+2 is issued at the start of block n (into block n-1's buffer)
//    and has blocks n and n+1 (>= 3 k-steps) to land; counted vmcnt waits at block boundaries.
// LDS: 3 x 44 KiB halo + 3 x 8 KiB weight ring + 512 B bias = 156.5 KiB.
#include "conv_common.h"

#include <type_traits>

namespace tv {
namespace c3s2 {

constexpr int NT = 512, BN = 128, TW = 32, TH = 16;
constexpr int CBK = 32;           // channels per k-step
constexpr int NCB = 128 / CBK;    // channel blocks per tile
constexpr int SPT = 9 * NCB;      // k-steps per tile
constexpr int PITCH = 80;         // halo pixel pitch (bytes)
constexpr int RS = TW + 1;        // halo row stride of a phase block (pixels)
constexpr int HROWS = TH + 1;
constexpr int HPIX = HROWS * RS;  // 561
constexpr int HPIECES = 44;       // ceil(561 * 5 / 64) LDS-DMA pieces of 1 KiB
constexpr int HBUF = HPIECES * 1024;
constexpr int NBUF = 3;
constexpr int WSLOT = BN * 64;    // weights of one k-step: 128 rows x 64 B
constexpr int RING = 3;
constexpr int OFF_W = NBUF * HBUF;
constexpr int OFF_B = OFF_W + RING * WSLOT;
constexpr int OFF_D = OFF_B + BN * 4;  // 1 KiB sink of the 6th halo piece of waves 4-7 (OOB: zeros)
constexpr int LDS = OFF_D + 1024;
static_assert(LDS <= 160 * 1024, "LDS budget");
static_assert(HPIECES * 64 >= HPIX * 5, "halo pieces");
constexpr int HPW = 6;            // halo pieces per wave: waves 0-3 issue 6, waves 4-7 issue 5 (44)

// k-step j of a channel block -> tap offset (ty, tx) inside its phase block: j 0..3 block
// (p, q) = (1,1), j 4, 5 block (1,0), j 6, 7 block (0,1), j 8 block (0,0)
constexpr int J_TY[9] = {0, 0, 1, 1, 0, 1, 0, 0, 0};
constexpr int J_TX[9] = {0, 1, 0, 1, 0, 0, 0, 1, 0};
// original tap ky*3+kx of k-step j: ky = 2ty + 1 - p, kx = 2tx + 1 - q
constexpr int J_TAP[9] = {0, 2, 6, 8, 1, 7, 3, 5, 4};

// Block order of a tile: channel blocks in pairs (c0, c1) = (2P, 2P+1), and within a pair the
// two channel blocks' copies of one phase block back to back — a pixel's 32-channel halves of
// one 128-byte line are then fetched a block apart (the second from L2) instead of a whole
// channel block (9 k-steps) apart, when the first half has left the L2. The 1-k-step (0,0)
// blocks sit between the longer ones so every block n+2, issued at the start of block n, has
// >= 3 k-steps to land.
constexpr int NBLK = 8;                               // blocks per channel-block pair
constexpr int BLK_PB[NBLK] = {0, 0, 3, 1, 1, 3, 2, 2};  // phase block: 0 (1,1), 1 (1,0), 2 (0,1), 3 (0,0)
constexpr int BLK_CB[NBLK] = {0, 1, 0, 0, 1, 1, 0, 1};  // channel block within the pair
constexpr int PB_LEN[4] = {4, 2, 2, 1};
constexpr int PB_J0[4] = {0, 4, 6, 8};                // first k-step j of the phase block
#ifndef TV_S2_SPREAD
#define TV_S2_SPREAD 1  // 0: all at the first step; 1 (default since round 4): a block's 6 halo pieces spread over its first two k-steps where the cover allows
#endif
// Halo pieces of block b + 2 issued at step t of block b (position b8 in the pair), HPW in all.
// Default: all at the block's first step. TV_S2_SPREAD: 3 + 3 over the first two steps of a
// 4-step block, and of a 2-step block followed by one of >= 2 steps (the second half still has
// >= 2 steps of cover before block b + 2 starts); the 1-step blocks and a 2-step block before a
// 1-step one keep all 6 at their first step.
constexpr int piece_cnt(int b8, int t) {
  const int L = PB_LEN[BLK_PB[b8]], Ln = PB_LEN[BLK_PB[(b8 + 1) % NBLK]];
  if (TV_S2_SPREAD && (L >= 4 || (L == 2 && Ln >= 2))) return t == 0 ? 3 : t == 1 ? HPW - 3 : 0;
  return t == 0 ? HPW : 0;
}
constexpr int piece_p0(int b8, int t) {
  int p = 0;
  for (int u = 0; u < t; ++u) p += piece_cnt(b8, u);
  return p;
}
constexpr int piece_tlast(int b8) {
  int tl = 0;
  for (int u = 0; u < PB_LEN[BLK_PB[b8]]; ++u)
    if (piece_cnt(b8, u) > 0) tl = u;
  return tl;
}
// VMEM operations issued after the last piece of block B + 1's halo when block B's last k-step
// starts (exact; block B + 1 was issued during block B - 1): that step's weight load, the weight
// loads of block B - 1's later steps, then every earlier step of block B: its pieces and its load
constexpr int younger_of(int b8) {
  const int bp = (b8 + NBLK - 1) % NBLK;
  int y = 1 + (PB_LEN[BLK_PB[bp]] - 1 - piece_tlast(bp));
  for (int t = 0; t + 1 < PB_LEN[BLK_PB[b8]]; ++t) y += piece_cnt(b8, t) + 1;
  return y;
}
struct Sched {
  int cb[SPT], j[SPT], blk[SPT], t[SPT];
};
constexpr Sched make_sched() {
  Sched sc{};
  int q = 0;
  for (int P = 0; P < NCB / 2; ++P)
    for (int b = 0; b < NBLK; ++b)
      for (int t = 0; t < PB_LEN[BLK_PB[b]]; ++t) {
        sc.cb[q] = 2 * P + BLK_CB[b];
        sc.j[q] = PB_J0[BLK_PB[b]] + t;
        sc.blk[q] = P * NBLK + b;
        sc.t[q] = t;
        ++q;
      }
  return sc;
}
constexpr Sched SCH = make_sched();
static_assert(SCH.blk[SPT - 1] == 2 * NBLK - 1 && SCH.j[SPT - 1] == PB_J0[BLK_PB[NBLK - 1]] + 1, "schedule covers the tile");

typedef __attribute__((address_space(3))) char lds_char;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size, int voffset,
                                    int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

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

template <int Q, int N, typename F>
__device__ __forceinline__ void unroll(F& f) {
  if constexpr (Q < N) {
    f(IC<Q>{});
    unroll<Q + 1, N>(f);
  }
}

struct Half {  // fragments of one 16-deep sub-step
  u32x4 x[2];  // pixel fragments f
  u32x4 w[4];  // channel fragments i
};

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

template <typename T, int ACT>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void conv3x3s2(
    const ConvParams* __restrict__ pp, void* out_ptr) {
  const ConvParams& p = *pp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int npw = wave < 4 ? 6 : 5;  // halo pieces this wave issues per block
  const int pbase = wave < 4 ? wave * 6 : 24 + (wave - 4) * 5;

  const ConvSegment& sg = p.seg[0];
  const int H = sg.H, W = sg.W, ldc = sg.ldc;  // input
  const int Ho = p.Ho, Wo = p.Wo;              // output
  const int tiles_x = (Wo + TW - 1) / TW;
  const int tiles_f = ((Ho + TH - 1) / TH) * tiles_x;
  const int ntot = p.mtiles;                   // one 128-channel tile (N == 128)

  // ---- this block's tiles: XCD-aware contiguous ranges
  const int G = gridDim.x, bid = blockIdx.x;
  int first, stride, end;
  if ((G & 7) == 0) {
    first = (int)((long long)ntot * (bid & 7) / 8) + (bid >> 3);
    end = (int)((long long)ntot * ((bid & 7) + 1) / 8);
    stride = G >> 3;
  } else {
    first = bid;
    end = ntot;
    stride = G;
  }
  const int ntl = first < end ? (end - first + stride - 1) / stride : 0;
  if (ntl == 0) return;
  const int S_tot = ntl * SPT;

  float* lbias = reinterpret_cast<float*>(smem + OFF_B);
  for (int c = tid; c < BN; c += NT) lbias[c] = c < p.N ? p.bias[c] : 0.0f;

  // ---- sources: one buffer resource per frame (offsets within a frame stay below 2^31)
  const unsigned pix_bytes = (unsigned)ldc * (unsigned)sizeof(T);
  const unsigned long long frame_bytes = (unsigned long long)H * W * pix_bytes;
  auto rsrc_of = [&](int fr) __attribute__((always_inline)) {
    i32x4 r;
    const unsigned long long a = (unsigned long long)sg.src + (unsigned long long)fr * frame_bytes;
    r.x = (int)(unsigned)a;
    r.y = (int)(unsigned)(a >> 32);
    r.z = (int)(unsigned)frame_bytes;
    r.w = 0x00020000;
    return r;
  };

  auto tile_of = [&](int idx, int& fr, int& y0, int& x0) __attribute__((always_inline)) {
    const int t = first + idx * stride;
    fr = t / tiles_f;
    const int r = t - fr * tiles_f;
    const int ty = r / tiles_x;
    y0 = ty * TH;
    x0 = (r - ty * tiles_x) * TW;
  };

  // ---- halo DMA geometry: chunk g = piece*64 + lane -> halo pixel g/5 (row stride RS), slot g%5
  unsigned hgeo[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int g = (pbase + i) * 64 + lane;
    const int h = g / 5, s5 = g - (g / 5) * 5;
    const int hy = h / RS, hx = h - (h / RS) * RS;
    hgeo[i] = (i < npw && s5 < 4 && h < HPIX) ? (unsigned)((hy << 16) | (hx << 8) | s5) : ~0u;
  }
  // issue the halo of phase block pb, channel block cb of tile (fr, y0, x0) into buffer buf
  auto issue_block = [&](int fr, int y0, int x0, int cb, int pb, int buf, auto loc, auto hic) __attribute__((always_inline)) {
    constexpr int LO = decltype(loc)::value, HI = decltype(hic)::value;
    const int pr = pb < 2 ? 1 : 0, pc = (pb & 1) == 0 ? 1 : 0;  // PB_P, PB_Q
    const i32x4 rs = rsrc_of(fr);
    lds_char* base = lds + buf * HBUF + pbase * 1024;
    // every wave issues HPW pieces: unconditional VMEM keeps the compiler's vmcnt for the weight
    // ds_write exact (a conditional load makes it vmcnt(0)); waves 4-7 send their 6th, all-OOB
    // piece to the LDS sink
#pragma unroll
    for (int i = LO; i < HI; ++i) {
      const unsigned gq = hgeo[i];
      const int hy = (int)(gq >> 16), hx = (int)((gq >> 8) & 0xff);
      const int y = 2 * y0 - pr + 2 * hy, x = 2 * x0 - pc + 2 * hx;
      const bool ok = gq != ~0u && hy < TH + pr && hx < TW + pc && (unsigned)y < (unsigned)H &&
                      (unsigned)x < (unsigned)W;
      const unsigned off = ok ? ((unsigned)y * (unsigned)W + (unsigned)x) * pix_bytes + (gq & 0xff) * 16u : 0x80000000u;
      lds_char* dst = i < npw ? base + i * 1024 : lds + OFF_D;
      raw_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, (int)off, cb * CBK * (int)sizeof(T), 0, 0);
    }
  };

  // ---- register-staged weights (as conv3x3.hip): k-step q loaded at step q-3, written at q-2
  // through a buffer resource: one lane-offset VGPR, the k-step offset in an SGPR
  int wc_in = 0;
  u32x4 wreg[4];  // k-step q is loaded at step q-5 into set q % 4, written to LDS at step q-2
  i32x4 wrsrc;
  {
    const unsigned long long a = (unsigned long long)p.weight;
    wrsrc.x = (int)(unsigned)a;
    wrsrc.y = (int)(unsigned)(a >> 32);
    wrsrc.z = SPT * WSLOT;
    wrsrc.w = 0x00020000;
  }
  const int wvoff = wave * 1024 + lane * 16;
  auto w_load = [&](u32x4& dst) __attribute__((always_inline)) {
    dst = raw_buffer_load_v4(wrsrc, wvoff, wc_in * WSLOT, 0);
    if (++wc_in == SPT) wc_in = 0;
  };

  // ---- fragment addresses
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  const unsigned xa = lds0 + (unsigned)(((2 * wave) * RS + l32) * PITCH + lh * 16);  // row 2w, col l32
  constexpr int FOFF = RS * PITCH;  // fragment f = 1: the next tile row
  unsigned wa[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    wa[j] = lds0 + OFF_W + (unsigned)(l32 * 64 + (((2 * j + lh) ^ ((l32 >> 2) & 3)) << 4));

  // read R (0..5) of sub-step J of k-step j: x[f] for R < 2, else w[i]
  auto read_one = [&](auto r, auto sj, auto kj, unsigned xb, unsigned wb, Half& F) __attribute__((always_inline)) {
    constexpr int R = decltype(r)::value, SJ = decltype(sj)::value, KJ = decltype(kj)::value;
    constexpr int TOFF = (J_TY[KJ] * RS + J_TX[KJ]) * PITCH;
    if constexpr (R < 2) F.x[R] = ds_read16<TOFF + 32 * SJ + R * FOFF>(xb);
    else F.w[R - 2] = ds_read16<(R - 2) * 2048>(wb);
  };

  f32x16 acc[2][4];
  auto mfma_pair = [&](auto i, auto first, const Half& F) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
    if constexpr (decltype(first)::value) {
      acc[0][I] = f32x16{};
      acc[1][I] = f32x16{};
    }
    Mfma<T>::run(to_u4(F.w[I]), to_u4(F.x[0]), acc[0][I]);
    Mfma<T>::run(to_u4(F.w[I]), to_u4(F.x[1]), acc[1][I]);
  };

  auto epilogue = [&](int fr, int y0, int x0) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int y = y0 + 2 * wave + f, x = x0 + l32;
      const bool ok = y < Ho && x < Wo;
      T* dst = reinterpret_cast<T*>(out_ptr) + ((size_t)(fr * Ho + (ok ? y : 0)) * Wo + (ok ? x : 0)) * p.out_ldc +
               p.out_coff;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float v[2][4];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int G2 = 2 * m + gg;
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lbias + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = acc[f][i][4 * G2 + e] + bb[e];
              if constexpr (ACT == 1) t = fmaxf(t, 0.0f);
              else if constexpr (ACT == 2) t = fmaxf(t, 0.01f * t);
              v[gg][e] = t;
            }
          }
          const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
          const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
          const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
          const int ch = 32 * i + 16 * m;
          if (ok && ch < p.N) gstore16(dst + ch + 8 * lh, make_uint4(r0[0], r1[0], r0[1], r1[1]));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };

  // ---- prologue: halos of blocks 0, 1 of tile 0 (buffers 0, 1), weights of k-steps 0..2
  int cur_fr, cur_y0, cur_x0;
  tile_of(0, cur_fr, cur_y0, cur_x0);
  issue_block(cur_fr, cur_y0, cur_x0, SCH.cb[0], BLK_PB[0], 0, IC<0>{}, IC<HPW>{});
  issue_block(cur_fr, cur_y0, cur_x0, BLK_CB[1], BLK_PB[1], 1, IC<0>{}, IC<HPW>{});
  __builtin_amdgcn_sched_barrier(0);  // the counted wait below needs the halos issued first
  w_load(wreg[0]);
  w_load(wreg[1]);
  *reinterpret_cast<u32x4*>(smem + OFF_W + wave * 1024 + lane * 16) = wreg[0];
  *reinterpret_cast<u32x4*>(smem + OFF_W + WSLOT + wave * 1024 + lane * 16) = wreg[1];
  w_load(wreg[2]);
  w_load(wreg[3]);
  w_load(wreg[0]);
  wait_vm<3>();  // both halos landed (issued before the weights); k-steps 2..4 may stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  Half H0, H1;
  read_one(IC<0>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
  read_one(IC<1>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
  read_one(IC<2>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
  read_one(IC<3>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
  read_one(IC<4>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
  read_one(IC<5>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);

  int s = 0;    // global k-step
  int tl = 0;   // tile index within this block's list
  int buf = 0;  // halo buffer of the current phase block (blocks rotate over NBUF buffers)
  int nx_fr = 0, nx_y0 = 0, nx_x0 = 0;  // the next tile (target of the next channel block's halos at cb 3)
  bool nx_exists = false;

  // One k-step: compile-time position Q in the tile's schedule (SCH): k-step
  // J of it, block BLK (0..15) and step TB within the block.
  auto step = [&](auto qc) __attribute__((always_inline)) {
    constexpr int Q = decltype(qc)::value;
    constexpr int J = SCH.j[Q], BLK = SCH.blk[Q], TB = SCH.t[Q];
    constexpr int B8 = BLK % NBLK;
    constexpr int L = PB_LEN[BLK_PB[B8]], LPREV = PB_LEN[BLK_PB[(B8 + NBLK - 1) % NBLK]];
    constexpr bool BOUNDARY = TB == L - 1;  // the next k-step starts a new block
    // VMEM operations issued after the last piece of the next block's halo (exact): it was
    // issued at the start of the previous block, before that step's weight load; since then one
    // weight load per k-step and, if this block is longer than one k-step, this block's own issue
    // (at its first step, before that step's weight load)
    constexpr int YOUNGER = younger_of(B8);
    static_assert(TV_S2_SPREAD || YOUNGER == LPREV + L - 1 + (L >= 2 ? HPW : 0), "the all-at-first-step count");
    static_assert(YOUNGER <= 13, "wait_vm_n range");
    if constexpr (BOUNDARY) wait_vm_n(s + 1 < S_tot ? YOUNGER : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    constexpr int NJ = SCH.j[(Q + 1) % SPT];  // next k-step's j
    const bool do_r = s + 1 < S_tot;
    const int nbuf = BOUNDARY ? (buf == NBUF - 1 ? 0 : buf + 1) : buf;
    const unsigned xc = xa + (unsigned)(buf * HBUF);
    const unsigned xn = xa + (unsigned)(nbuf * HBUF);
    const unsigned wc1 = wa[1] + (unsigned)((s % RING) * WSLOT);
    const unsigned wn0 = wa[0] + (unsigned)(((s + 1) % RING) * WSLOT);
    constexpr bool FIRST = Q == 0;
    constexpr int PAR = Q & 3;  // SPT % 4 == 0: the weight register set is static
    // at a block's first k-step: block BLK + 2 (this tile or the next one) into the buffer block
    // BLK - 1 used (free since this step's barrier), two pieces after each of the first half's
    // MFMA pairs (an LDS-DMA instruction holds its wave at issue)
    constexpr int NB = BLK + 2, NB8 = NB % NBLK;
    constexpr bool NEXT_TILE = NB >= 2 * NBLK;
    constexpr int ICB = 2 * ((NB % (2 * NBLK)) / NBLK) + BLK_CB[NB8], IPB = BLK_PB[NB8];
    // this step's pieces [P0, P1) of block BLK + 2, split over the three issue points
    constexpr int P0 = piece_p0(B8, TB), P1 = P0 + piece_cnt(B8, TB);
    auto issue_part = [&](auto lo, auto hi) __attribute__((always_inline)) {
      constexpr int LO = decltype(lo)::value > P0 ? decltype(lo)::value : P0;
      constexpr int HI = decltype(hi)::value < P1 ? decltype(hi)::value : P1;
      if constexpr (LO < HI) {
        const int tbuf = buf == 0 ? 2 : buf - 1;  // (buf + 2) % 3
        if constexpr (NEXT_TILE) issue_block(nx_fr, nx_y0, nx_x0, ICB, IPB, tbuf, IC<LO>{}, IC<HI>{});  // (last tile: itself, into a free buffer)
        else issue_block(cur_fr, cur_y0, cur_x0, ICB, IPB, tbuf, IC<LO>{}, IC<HI>{});
      }
    };
    mfma_pair(IC<0>{}, IC<FIRST>{}, H0);
    read_one(IC<0>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    read_one(IC<1>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    issue_part(IC<0>{}, IC<2>{});
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<1>{}, IC<FIRST>{}, H0);
    read_one(IC<2>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    read_one(IC<3>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    *reinterpret_cast<u32x4*>(smem + OFF_W + ((s + 2) % RING) * WSLOT + wave * 1024 + lane * 16) = wreg[(PAR + 2) & 3];
    issue_part(IC<2>{}, IC<4>{});
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<2>{}, IC<FIRST>{}, H0);
    read_one(IC<4>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    read_one(IC<5>{}, IC<1>{}, IC<J>{}, xc, wc1, H1);
    issue_part(IC<4>{}, IC<HPW>{});
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<3>{}, IC<FIRST>{}, H0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // H1 landed
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<0>{}, IC<false>{}, H1);
    w_load(wreg[(PAR + 1) & 3]);  // k-step s+5 (past the end: re-reads the panel; away from the barrier)
    if (do_r) {
      read_one(IC<0>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
      read_one(IC<1>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<1>{}, IC<false>{}, H1);
    if (do_r) {
      read_one(IC<2>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
      read_one(IC<3>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<2>{}, IC<false>{}, H1);
    if (do_r) {
      read_one(IC<4>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
      read_one(IC<5>{}, IC<0>{}, IC<NJ>{}, xn, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<3>{}, IC<false>{}, H1);
    __builtin_amdgcn_sched_barrier(0);
    buf = nbuf;
    ++s;
  };

  static_assert(NCB == 4 && SPT % 4 == 0, "tile body is unrolled for 4 channel blocks; 4 weight register sets");
  for (; tl < ntl;) {
    nx_exists = tl + 1 < ntl;
    if (nx_exists) tile_of(tl + 1, nx_fr, nx_y0, nx_x0);
    else nx_fr = cur_fr, nx_y0 = cur_y0, nx_x0 = cur_x0;
    unroll<0, SPT>(step);  // the whole tile, straight-line
    epilogue(cur_fr, cur_y0, cur_x0);
    ++tl;
    cur_fr = nx_fr;
    cur_y0 = nx_y0;
    cur_x0 = nx_x0;
  }
}

// [Npad][Kpad] (K = tap * 128 + channel) -> [k-step q][128 rows][4 x 16 B] in this kernel's
// schedule (channel block SCH.cb[q], tap J_TAP[SCH.j[q]]), slot s of row r holding chunk
// s ^ ((r >> 2) & 3)
__global__ void repack_weights_s2(const uint4* __restrict__ w, int kpad16, uint4* __restrict__ out) {
  const int n = SPT * BN * 4;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const int slot = o & 3, row = (o >> 2) & (BN - 1), q = o >> 9;
    const int chunk = slot ^ ((row >> 2) & 3);
    const int cb = SCH.cb[q], j = SCH.j[q];
    const int k16 = (J_TAP[j] * 128 + cb * CBK) / 8 + chunk;
    out[o] = w[(size_t)row * kpad16 + k16];
  }
}

template <typename T, int ACT>
static int launch_t(const ConvParams& p, const ConvParams* dp, void* out, int grid, hipStream_t s) {
  auto k = conv3x3s2<T, ACT>;
  if (int r = ensure_lds<conv3x3s2<T, ACT>>(LDS)) return r;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), LDS, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace c3s2

int conv3x3s2_tiles(int B, int Ho, int Wo) {
  return B * ((Ho + c3s2::TH - 1) / c3s2::TH) * ((Wo + c3s2::TW - 1) / c3s2::TW);
}

size_t conv3x3s2_weight_bytes() { return (size_t)c3s2::SPT * c3s2::WSLOT; }

int conv3x3s2_repack(const void* w, int Kpad, int esz, void* out, hipStream_t s) {
  if ((Kpad * esz) % 16 || Kpad < 9 * 128) {
    set_error("conv3x3s2_repack: bad Kpad");
    return 1;
  }
  hipLaunchKernelGGL(c3s2::repack_weights_s2, dim3(64), dim3(256), 0, s, (const uint4*)w, Kpad * esz / 16, (uint4*)out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_conv3x3s2(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int grid, hipStream_t s) {
  using namespace c3s2;
  if (p.act < 0 || p.act > 2 || p.ntiles != 1 || p.N > BN) {
    set_error("conv3x3s2: one 128-channel tile, activation none/relu/leaky");
    return 1;
  }
  using L = int (*)(const ConvParams&, const ConvParams*, void*, int, hipStream_t);
  static const L f16[3] = {launch_t<_Float16, 0>, launch_t<_Float16, 1>, launch_t<_Float16, 2>};
  static const L b16[3] = {launch_t<__bf16, 0>, launch_t<__bf16, 1>, launch_t<__bf16, 2>};
  if (dtype == F16) return f16[p.act](p, dp, out, grid, s);
  if (dtype == BF16) return b16[p.act](p, dp, out, grid, s);
  set_error("conv3x3s2: fp16/bf16 only");
  return 1;
}

}  // namespace tv
