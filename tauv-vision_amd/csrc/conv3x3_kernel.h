// conv3x3_kernel.h — the kernel template, included by conv3x3.hip (repack, dispatch) and by
// conv3x3_n{2,4,8}.hip (the instances for 64 / 128 / 256 input channels, compiled in parallel).
//
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
//  * one 512-thread workgroup per CU (8 waves, two per SIMD), persistent over a static list of
//    (spatial tile, 128-channel tile) pairs, XCD-aware: each XCD owns a contiguous tile range so
//    neighbouring tiles (shared halo rows) meet in its L2. Two waves per SIMD because an
//    LDS-DMA instruction stalls its wave for ~60-180 cycles at issue: with one wave per SIMD
//    that stall idles the matrix core (measured: 1550 instead of 1024 cycles per k-step);
//  * a tile = TH x TW = 512 output pixels of one frame x 128 output channels; each wave owns
//    64 pixels x 128 channels (2 x 4 tiles of v_mfma_f32_32x32x16, 128 accumulators);
//  * K order: channel blocks of 32 (64 B), 9 taps each. The (TH+2) x (TW+2) input halo of one
//    channel block moves into LDS ONCE (buffer_load ... lds: out-of-image and pad slots are
//    buffer-OOB, so they read as zero with no per-lane branches) and the 9 taps read shifted
//    windows of it at compile-time immediate ds_read offsets: 1.2x input traffic instead of 9x;
//  * two halo buffers (the next channel block — or the next tile's first — streams in during
//    taps 0..5 of the current one), a 3-slot weight ring (8 KiB per k-step from a k-step-major,
//    pre-swizzled copy of the weights: each wave's 1 KiB piece is contiguous; loaded into
//    registers five k-steps ahead (4 register sets) and written with ds_write_b128 two steps
//    before use — deep enough for the few-tile layers that stream weights from HBM), one raw
//    s_barrier per k-step with an exact counted vmcnt;
//  * fragment reads run one 16-deep sub-step ahead of the MFMAs (6 ds_read_b128 per half
//    k-step, two register sets) and the k-step's LDS-DMA pieces are issued between MFMA pairs;
//  * the epilogue stores straight from the accumulators (bias from LDS, activation, fp16/bf16
//    pack, v_permlane32_swap pairs into 16-byte stores), so the next tile's prefetched halo and
//    weights are already in flight while it runs: no per-tile prologue, no LDS staging.
// LDS: halo 2 x 48 KiB (pixel pitch 80 B = 64 B of channels + 16 B pad: conflict-free
// ds_read_b128 for 32-pixel rows), weight ring 3 x 8 KiB (XOR-swizzled 64 B rows), bias.
#pragma once
#include "conv_common.h"

#ifndef TV_C3_EXP
#define TV_C3_EXP 0  // diagnostic builds (tools/gpu_libab.sh): 2 = no epilogue stores, 3 = 16x16x32 MFMAs
                     // (timing only, wrong results); 9 = per-wave cycle stamps into ConvParams.dbg
#endif
#if TV_C3_EXP == 9
// s_memtime + lgkmcnt(0) as one statement (cdna_hip_programming.md §7, in-kernel stamps); the
// cycles since the previous stamp go to bucket B
#define C3_STAMP(B)                                                                    \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    unsigned long long t_;                                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    st_b[B] += t_ - st_last;                                                           \
    st_last = t_;                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#else
#define C3_STAMP(B) \
  do {              \
  } while (0)
#endif

#ifndef TV_C3_MF
#define TV_C3_MF 16  // MFMA shape of the plain NI 4 tile body (K16): 16 = v_mfma_f32_16x16x32, 32 = 32x32x16
#endif

#include <type_traits>

namespace tv {
namespace c3 {

// 16x16x32 body (M16): a k-step (one tap x 32 channels) is ONE K=32 MFMA step; a wave's 64 pixels are
// 4 fragments of 16 and its 128 channels 8 fragments of 16 (32 MFMAs per k-step, as 16 of 32x32x16).
// Lane l = 16c + n supplies fragment row/column n and K group c, which reads the 16-byte chunk
// sigma(c) = (0, 2, 1, 3)[c] of the 64-byte channel block, and fragment column n is pixel pi(n) of
// the fragment: pi maps {0..3, 12..15} to the even and {4..11} to the odd pixels, so that the
// ds_read_b128 lane groups hit 16 distinct 4-bank sets on the 80-byte-pitch halo; weight rows are
// swizzled chunk ^ ((row >> 3) & 1) (wswz) (MI355X_MICROARCH.md LDS table; checked by tools/bank_check.py).
constexpr bool M16 = TV_C3_MF == 16;
__device__ __forceinline__ int m16_sigma(int c) { return ((c & 1) << 1) | (c >> 1); }
__device__ __forceinline__ int m16_pi(int n) { return n < 4 ? 2 * n : n < 12 ? 2 * n - 7 : 2 * n - 16; }
// host + device: the weight-row chunk swizzle of the LDS ring (and of the repacked weights)
__host__ __device__ constexpr int wswz(int row, bool k16) { return k16 ? (row >> 3) & 1 : (row >> 2) & 3; }

template <typename T> struct Mfma16;
template <> struct Mfma16<_Float16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0, 0, 0);
  }
};
template <> struct Mfma16<__bf16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};

// The main-loop 16x16x32 MFMAs as asm statements with the accumulator tied to C: through the
// builtin, hipcc gave a third of them a fresh destination (an accumulator rotation across k-steps
// that doubled the accumulator registers and spilled ~100 VGPRs). Hazards, placed by hand: every
// accumulator's only in-loop reader is the next MFMA taking it whole as C (0 wait states); the
// epilogue's first reader sits behind mfma16_drain() (8-pass XDL D -> VALU: 12 states); the A/B
// operands come from ds_read_b128 behind counted lgkmcnt waits (no VALU producer).
template <typename T, bool FIRST>
__device__ __forceinline__ void mfma16_asm(f32x4& acc, const u32x4& a, const u32x4& b) {
  if constexpr (FIRST) {
    if constexpr (std::is_same<T, __bf16>::value)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  } else {
    if constexpr (std::is_same<T, __bf16>::value)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  }
}
__device__ __forceinline__ void mfma16_drain() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

constexpr int NT = 512, NW = 8, BN = 128, P = 512;
constexpr int WP = P / NW;                    // pixels per wave = 64 (two 32-pixel fragments)
constexpr int CBK = 32;                       // channels per k-step
// NCB: channel blocks per tile = C / 32 (4 for the 128-channel DLA levels, 8 for 256-channel inputs:
// the YOLACT protonet's 3x3 convs, DLA-34's 256-channel level)
template <int RES, int NCB = 4>
constexpr int spt() { return (9 + RES) * NCB; }
constexpr int PITCH = 80;                     // halo pixel pitch (bytes)
constexpr int HPIX = 612;                     // (16+2)x(32+2) = (32+2)x(16+2) halo pixels
constexpr int HPIECES = 48;                   // ceil(612 * 5 / 64) LDS-DMA pieces of 1 KiB
constexpr int HBUF = HPIECES * 1024;          // one halo buffer
constexpr int HPW = HPIECES / NW;             // halo pieces per wave per channel block = 6
constexpr int HTAPS = HPW;                    // one halo piece per k-step, taps 0..5
constexpr int WSLOT = BN * 64;                // weights of one k-step: 128 rows x 64 B
constexpr int RING = 3;                       // weight ring slots (register-staged: k-step q is
                                              // loaded at step q-3, written to LDS at step q-2)
constexpr int OFF_W = 2 * HBUF;
constexpr int OFF_B = OFF_W + RING * WSLOT;
constexpr int OFF_R = OFF_B + kConv3MaxN * 4;  // RES: one channel block of the residual input
constexpr int RBUF = 512 * 64;                  // 512 pixels x 32 channels (XOR-swizzled 16 B chunks)
constexpr int RPW = RBUF / 1024 / NW;           // residual pieces per wave per channel block = 4
// EPI 1 (fused 1x1 heads, never RES): the heads' A-fragments of a channel tile (8 k-steps x 64
// lanes x 16 B) staged by LDS-DMA into one of two buffers in the RES region, one 1 KiB piece per wave
constexpr int OFF_HW = OFF_R;
constexpr int HWB = 8 * 1024;
// EPI 1: per wave a 32-pixel x 16-row fp32 scratch for the transposed head atomics
constexpr int OFF_HS = OFF_HW + 2 * HWB;
constexpr int HSW = 32 * 16 * 4;
template <int RES, int EPI = 0>
constexpr int lds_bytes() { return OFF_R + (RES ? RBUF : EPI ? 2 * HWB + NW * HSW : 0); }
static_assert(lds_bytes<1>() <= 160 * 1024 && lds_bytes<0, 1>() <= 160 * 1024, "LDS budget");
static_assert(WSLOT / 1024 == NW, "one weight piece per wave per k-step");
static_assert(HPIECES * 64 >= HPIX * 5, "halo pieces");

// Tile geometry per workgroup size: NWV = 8 waves (one 512-thread workgroup per CU, the constants
// above) or 4 (two independent 256-thread workgroups per CU, 256-pixel tiles: while one
// workgroup waits at its per-k-step barrier or streams its epilogue stores, the other's waves keep
// the same SIMDs' matrix cores busy; plain epilogue only, <= 256 output channels, 80 KiB of LDS).
template <int NWV, int TW>
struct Geo {
  static constexpr int NW = NWV, NT = 64 * NWV, P = 64 * NWV, TH = P / TW, RS = TW + 2;
  static constexpr int HPIX = (TH + 2) * RS;
  static constexpr int HPIECES = (HPIX * 5 + 63) / 64;         // LDS-DMA pieces of 1 KiB per halo
  static constexpr int HPW = (HPIECES + NW - 1) / NW;          // halo pieces per wave per channel block
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr bool SINK = HPW * NW > HPIECES;             // surplus pieces (all lanes OOB) land here
  static constexpr int OFF_D = 2 * HBUF;
  static constexpr int OFF_W = 2 * HBUF + (SINK ? 1024 : 0);
  static constexpr int OFF_B = OFF_W + RING * WSLOT;
  static constexpr int MAXN = NWV == 8 ? kConv3MaxN : 256;     // bias entries in LDS
  static constexpr int OFF_R = OFF_B + MAXN * 4;
  static constexpr int RPW = RBUF / 1024 / NW;
  static constexpr int OFF_HW = OFF_R, OFF_HS = OFF_HW + 2 * HWB;
  template <int RES, int EPI>
  static constexpr int lds() { return OFF_R + (RES ? RBUF : EPI ? 2 * HWB + NW * HSW : 0); }
};
static_assert(Geo<8, 32>::OFF_W == OFF_W && Geo<8, 16>::HPIX == HPIX && Geo<8, 32>::HPW == HPW, "8-wave geometry");
static_assert(Geo<4, 32>::lds<0, 0>() <= 80 * 1024 && Geo<4, 16>::lds<0, 0>() <= 80 * 1024, "two 4-wave workgroups per CU");


typedef __attribute__((address_space(3))) char lds_char;
typedef const __attribute__((address_space(1))) void gvoid;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ u32x2 raw_buffer_load_v2(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
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
    default: wait_vm<8>(); break;
  }
}

template <int V>
using IC = std::integral_constant<int, V>;

template <int NI>
struct Half {  // fragments of one 16-deep sub-step
  u32x4 x[2];    // pixel fragments f
  u32x4 w[NI];   // channel fragments i
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

// NI: 32-channel fragments per wave — 4 (a 128-channel tile) or 2 (a 64-channel half tile, twice
// the work units for layers whose 128-channel tiles leave the last round of CUs mostly idle)
template <typename T, typename OutT, int TW, int ACT, int EPI, int RES, int NI, int NCB, int NWV = 8>
__global__ __attribute__((amdgpu_flat_work_group_size(64 * NWV, 64 * NWV), amdgpu_waves_per_eu(2, 2))) void conv3x3(
    const ConvParams* __restrict__ pp, void* out_ptr) {
  constexpr int RG = RING, WD = 2;  // weight ring slots; k-steps between a slot's ds_write and its first use
  using Gm = Geo<NWV, TW>;
  constexpr int NW = Gm::NW, NT = Gm::NT, P = Gm::P, HPIX = Gm::HPIX, HPW = Gm::HPW, HTAPS = Gm::HPW, HBUF = Gm::HBUF;
  constexpr int HPIECES = Gm::HPIECES, OFF_W = Gm::OFF_W, OFF_B = Gm::OFF_B, OFF_R = Gm::OFF_R, RPW = Gm::RPW;
  constexpr int OFF_HW = Gm::OFF_HW, OFF_HS = Gm::OFF_HS;
  static_assert(NWV == 8 || (NWV == 4 && !RES && EPI == 0), "4-wave workgroups: plain epilogue only");
  // The 16x16x32 body for the plain 128-channel-tile instances only. Measured (profiles/r3b): the
  // dominant 120x160 layer 1.476 -> 1.423 ms per slice; the fused-heads epilogue on 16x16 tiles
  // (16-pixel fragments, twice the head MFMAs' issue slots per pixel) 0.883 -> 0.950 ms; the
  // half-tile (NI 2) instances +1-3%; the residual instances need ~12 VGPRs more than the 256 of
  // two waves per SIMD.
  constexpr bool K16 = M16 && !RES && EPI == 0 && NI == 4 && NWV == 8;
  static_assert(NI == 4 || (NI == 2 && EPI == 0), "half tiles: plain epilogue only");
  static_assert(!(EPI == 1 && RES), "fused heads use the residual LDS region for their 1x1 weights");
  constexpr int SPTK = spt<RES, NCB>();  // k-steps per tile
  constexpr int BNK = 32 * NI;      // output channels per tile
  constexpr int WSL = BNK * 64;     // weight bytes per k-step (an LDS ring slot holds up to WSLOT)
  constexpr int WPL = WSL / NT;     // weight bytes per lane per k-step (8, 16 or 32)
  constexpr int WLN = WPL == 32 ? 2 : 1;  // weight load instructions per lane per k-step
  struct W32 {
    u32x4 a, b;
  };
  using WReg = typename std::conditional<WPL == 32, W32, typename std::conditional<WPL == 16, u32x4, u32x2>::type>::type;
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
  const int H = sg.H, W = sg.W, ldc = sg.ldc;
  const int tiles_x = (W + TW - 1) / TW;
  const int tiles_f = ((H + TH - 1) / TH) * tiles_x;
  // channel tiles of BNK (p.ntiles counts 128-channel tiles); N <= 64 with half tiles: one tile
  // (the second half would be all padding, e.g. DLA-34's 27-channel DCN offset / mask convs)
  const int ntiles = (NI == 2 && p.N <= 64) ? 1 : p.ntiles * (4 / NI);
  const int ntot = p.mtiles * ntiles;
  const int nframes = p.M / (H * W);       // stride 1: M = B * H * W
  [[maybe_unused]] const unsigned long long out_frame_bytes = (unsigned long long)H * W * p.out_ldc * sizeof(OutT);  // < 2^31 (host)

  // ---- this block's tiles: XCD-aware contiguous ranges. With 2 channel blocks (18 k-steps per
  // tile) the tile body is two tiles long (36 k-steps: the weight register sets rotate by a
  // compile-time position), so the list is scheduled in pairs of consecutive units; the second
  // unit of the last pair may be past the end (a phantom: its loads are buffer-OOB zeros and its
  // epilogue stores are dropped).
  constexpr int UP = NCB == 2 ? 2 : 1;  // units per scheduled item
  const int nitems = (ntot + UP - 1) / UP;
  const int G = gridDim.x, bid = blockIdx.x;
  int first, stride, end;
  if ((G & 7) == 0) {
    first = (int)((long long)nitems * (bid & 7) / 8) + (bid >> 3);
    end = (int)((long long)nitems * ((bid & 7) + 1) / 8);
    stride = G >> 3;
  } else {
    first = bid;
    end = nitems;
    stride = G;
  }
  const int ntl = first < end ? UP * ((end - first + stride - 1) / stride) : 0;
  if (ntl == 0) return;
#if TV_C3_EXP == 9
  // buckets: 0 barrier (+ tap-8 vmcnt) wait, 1 first half-step (+ H1 drain), 2 second half-step
  // (+ next H0 drain), 3 epilogue, 4 prologue, 5 k-steps
  // 6 tap-8 vmcnt wait (next block's halo), 7 the barrier after it
  unsigned long long st_b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  const int S_tot = ntl * SPTK;

  // bias of every output channel into LDS (read in the epilogues)
  float* lbias = reinterpret_cast<float*>(smem + OFF_B);
  for (int c = tid; c < ntiles * BN; c += NT) lbias[c] = c < p.N ? p.bias[c] : 0.0f;

  // ---- sources
  i32x4 rsrc;
  {
    const unsigned long long a = (unsigned long long)sg.src;
    rsrc.x = (int)(unsigned)a;
    rsrc.y = (int)(unsigned)(a >> 32);
    rsrc.z = (int)(unsigned)((unsigned long long)p.M * ldc * sizeof(T));  // bytes (host checks < 2^31)
    rsrc.w = 0x00020000;
  }
  // k-step-major weights: [ntile][k-step][BNK rows][64 B], chunks pre-swizzled; one WSL/8 piece
  // per wave per k-step at (ntile * SPT + q) * WSL + wave * WSL / 8
  // (read through a buffer resource: one lane-offset VGPR, the k-step offset in an SGPR)
  i32x4 wrsrc;
  {
    const unsigned long long a = (unsigned long long)p.weight;
    wrsrc.x = (int)(unsigned)a;
    wrsrc.y = (int)(unsigned)(a >> 32);
    wrsrc.z = ntiles * SPTK * WSL;
    wrsrc.w = 0x00020000;
  }
  const int wvoff = wave * (WSL / NW) + lane * WPL;

  // ---- tile decode
  auto tile_of = [&](int idx, int& fr, int& y0, int& x0, int& nt) __attribute__((always_inline)) {
    const int t = UP * (first + (idx / UP) * stride) + idx % UP;
    nt = t % ntiles;
    const int mt = t / ntiles;
    fr = t < ntot ? mt / tiles_f : nframes;  // a phantom unit reads past the last frame
    const int r = mt - fr * tiles_f;
    const int ty = r / tiles_x;
    y0 = ty * TH;
    x0 = (r - ty * tiles_x) * TW;
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
  // one halo piece (index I of this wave's HPW) of channel block cb into buffer bsel
  auto halo_piece = [&](auto pc, int cb, int bsel) __attribute__((always_inline)) {
    constexpr int I = decltype(pc)::value;
    // (a surplus piece past the halo's last — 4-wave workgroups — reads OOB zeros into the sink)
    lds_char* base = !Gm::SINK || wave * HPW + I < HPIECES ? lds + bsel * HBUF + (wave * HPW + I) * 1024 : lds + Gm::OFF_D;
    raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)base, 16, (int)hoff[I],
                        cb * CBK * (int)sizeof(T), 0, 0);
  };

  // EPI 1: this wave's 1 KiB piece (k-step `wave` of the 1x1 heads) of channel tile nt's A-fragments
  [[maybe_unused]] auto head_piece = [&](int nt, int hsel) __attribute__((always_inline)) {
    dma16(reinterpret_cast<const char*>(p.head_w) + ((size_t)(nt * 8 + wave) * 64 + lane) * 16,
          lds + OFF_HW + hsel * HWB + wave * 1024);
  };

  // ---- RES: the ResidualBlock's 1x1 conv_residual (dla.py:32-37), or DLA-34 BasicBlock's identity
  // residual (centerpoint_dla.py:30-59, an identity 1x1), as a 10th k-step per channel block. Its input x (second segment, stride rstr) for the tile's 512 output pixels
  // moves into one 32 KiB LDS buffer per channel block: chunk L = piece*64 + lane holds pixel
  // q = L/4, source chunk (L % 4) ^ ((q >> 2) & 3) (conflict-free fragment reads). One buffer
  // resource per frame keeps offsets below 2^31.
  [[maybe_unused]] unsigned rgeo[RPW];
  [[maybe_unused]] const ConvSegment& sr = p.seg[RES ? 1 : 0];
  [[maybe_unused]] const unsigned rpix_bytes = (unsigned)sr.ldc * (unsigned)sizeof(T);
  if constexpr (RES) {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int L = (wave * RPW + i) * 64 + lane;
      const int q = L >> 2;
      rgeo[i] = (unsigned)((q << 2) | ((L & 3) ^ ((q >> 2) & 3)));
    }
  }
  auto res_piece = [&](int i, int fr, int y0, int x0, int cb) __attribute__((always_inline)) {
    const unsigned long long fb = (unsigned long long)sr.H * sr.W * rpix_bytes;
    const unsigned long long a = (unsigned long long)sr.src + (unsigned long long)fr * fb;
    i32x4 rs;
    rs.x = (int)(unsigned)a;
    rs.y = (int)(unsigned)(a >> 32);
    rs.z = (int)(unsigned)fb;
    rs.w = 0x00020000;
    const int q = (int)(rgeo[i] >> 2), c = (int)(rgeo[i] & 3);
    const int y = y0 + q / TW, x = x0 + q % TW;
    // a phantom unit's frame is past the tensor, and a residual input narrower than the 3x3 input
    // (DLA-34 Tree's 1x1 `project` of the pooled bottom: C / 2 channels) has no block cb: OOB zeros
    const bool ok = y < H && x < W && fr < nframes && cb * CBK < sr.C;
    const unsigned off = ok ? ((unsigned)(y * sr.stride) * (unsigned)sr.W + (unsigned)(x * sr.stride)) * rpix_bytes +
                                  (unsigned)c * 16u
                            : 0x80000000u;
    raw_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + OFF_R + (wave * RPW + i) * 1024), 16,
                        (int)off, cb * CBK * (int)sizeof(T), 0, 0);
  };

  // ---- weight issue cursor: k-step counter and the global k-step index of the next piece
  int wc_idx = 0, wc_in = 0, wc_nt = 0;
  {
    int a, b_, c_;
    tile_of(0, a, b_, c_, wc_nt);
  }
  // register-staged weights: one 16-byte global load per lane per k-step, written to the
  // ring slot with ds_write_b128 one step later (instead of an LDS-DMA piece per k-step)
  WReg wreg[4];  // k-step q's weights are loaded at step q-5 into set q % 4
  auto w_load = [&](WReg& dst) __attribute__((always_inline)) {
    if constexpr (WPL == 32) {
      dst.a = raw_buffer_load_v4(wrsrc, wvoff, (wc_nt * SPTK + wc_in) * WSL, 0);
      dst.b = raw_buffer_load_v4(wrsrc, wvoff + 16, (wc_nt * SPTK + wc_in) * WSL, 0);
    } else if constexpr (WPL == 16) {
      dst = raw_buffer_load_v4(wrsrc, wvoff, (wc_nt * SPTK + wc_in) * WSL, 0);
    } else {
      dst = raw_buffer_load_v2(wrsrc, wvoff, (wc_nt * SPTK + wc_in) * WSL, 0);
    }
    if (++wc_in == SPTK) {
      wc_in = 0;
      if (++wc_idx < ntl) {
        int a, b_, c_;
        tile_of(wc_idx, a, b_, c_, wc_nt);
      }
    }
  };

  // ---- fragment addresses
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  unsigned xa;  // pixel WP*wave + l32 of the tile, tap (0,0), lane-half chunk
  {
    const int q = WP * wave + l32;
    const int r = q / TW, c = q - (q / TW) * TW;
    xa = lds0 + (unsigned)((r * RS + c) * PITCH + lh * 16);
  }
  unsigned wa[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    wa[j] = lds0 + OFF_W + (unsigned)(l32 * 64 + (((2 * j + lh) ^ ((l32 >> 2) & 3)) << 4));

  // RES: fragment base of pixel q0 = WP*wave + l32 in the residual buffer, per sub-step J
  // (fragment f = 1 is q0 + 32: +2 KiB, same swizzle)
  [[maybe_unused]] unsigned rxa[2];
  if constexpr (RES && !K16) {
    const int q0 = WP * wave + l32;
#pragma unroll
    for (int j = 0; j < 2; ++j) rxa[j] = lds0 + OFF_R + (unsigned)(q0 * 64 + (((2 * j + lh) ^ ((q0 >> 2) & 3)) << 4));
  }

  // ---- K16 fragment addresses: lane (c16, n16) reads chunk m16_sigma(c16) of pixel
  // WP*wave + 16f + m16_pi(n16) (fragment f: a compile-time offset) / of weight row 16i + n16
  const int n16 = lane & 15, c16 = lane >> 4;
  [[maybe_unused]] const int pin = m16_pi(n16), sig = m16_sigma(c16);
  [[maybe_unused]] unsigned xa16 = 0, wa16 = 0, rxa16 = 0;
  if constexpr (K16) {
    const int q = WP * wave + pin;
    const int r = q / TW, c = q - (q / TW) * TW;
    xa16 = lds0 + (unsigned)((r * RS + c) * PITCH + sig * 16);
    wa16 = lds0 + OFF_W + (unsigned)(n16 * 64 + ((sig ^ wswz(n16, true)) << 4));
    if constexpr (RES) rxa16 = lds0 + OFF_R + (unsigned)(q * 64 + ((sig ^ ((q >> 2) & 3)) << 4));
  }
  // pixel fragment f's offset from fragment 0 in the halo (TW 32: two 16-pixel halves of a row
  // pair; TW 16: one row each)
  constexpr int FO16[4] = {0, TW == 32 ? 16 * PITCH : RS * PITCH, TW == 32 ? RS * PITCH : 2 * RS * PITCH,
                           TW == 32 ? (RS + 16) * PITCH : 3 * RS * PITCH};

  // read R (0..5) of sub-step J of a k-step: x[f] for R < 2, else w[i]; TAP 9 = residual k-step
  auto read_one = [&](auto r, auto j, auto tap, unsigned xb, unsigned wb, Half<NI>& F) __attribute__((always_inline)) {
    constexpr int R = decltype(r)::value, J = decltype(j)::value, TAP = decltype(tap)::value;
    if constexpr (TAP == 9) {
      if constexpr (R < 2) F.x[R] = ds_read16<R * 2048>(rxa[J]);
      else F.w[R - 2] = ds_read16<(R - 2) * 2048>(wb);
    } else {
      constexpr int TOFF = ((TAP / 3) * RS + (TAP % 3)) * PITCH;
      if constexpr (R < 2) F.x[R] = ds_read16<TOFF + 32 * J + R * FOFF>(xb);
      else F.w[R - 2] = ds_read16<(R - 2) * 2048>(wb);
    }
  };

  f32x16 acc[2][NI];  // [pixel fragment f][channel fragment i]; first written by a tile's first k-step
  [[maybe_unused]] f32x4 a16[4][2 * NI];  // K16: [16-pixel fragment f][16-channel fragment i]
  [[maybe_unused]] u32x4 X16[1][4];        // K16: the 4 pixel fragments of a k-step
  [[maybe_unused]] u32x4 W16[2][NI];       // K16: channel fragments 0..NI-1 / NI..2NI-1 of a k-step

  // K16: fragment reads (tap 9 = the residual k-step) and the 4 MFMAs of channel fragment I
  [[maybe_unused]] auto rd_x16 = [&](auto f, auto tap, unsigned xb) __attribute__((always_inline)) {
    constexpr int F = decltype(f)::value, TAP = decltype(tap)::value;
    if constexpr (TAP == 9) return ds_read16<F * 1024>(rxa16);
    else return ds_read16<((TAP / 3) * RS + (TAP % 3)) * PITCH + FO16[F]>(xb);
  };
  [[maybe_unused]] auto quad16 = [&](auto i, auto first, const u32x4& w, const u32x4 (&x)[4]) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
#pragma unroll
    for (int f = 0; f < 4; ++f) mfma16_asm<T, decltype(first)::value>(a16[f][I], w, x[f]);
  };
#if TV_C3_EXP == 3
  f32x4 acc4[2][NI][2];  // timing-only 16x16x32 accumulators (copied into acc before the epilogue)
#endif

  // the 2 MFMAs of channel fragment I of one sub-step; FIRST: the tile's first products
  // (accumulate onto zero instead of clearing the accumulators in the epilogue)
  auto mfma_pair = [&](auto i, auto first, const Half<NI>& F) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
    if constexpr (decltype(first)::value) {
      acc[0][I] = f32x16{};
      acc[1][I] = f32x16{};
    }
#if TV_C3_EXP == 3  // timing only: the same MACs as two 16x16x32 MFMAs each (wrong results)
    if constexpr (decltype(first)::value) {
      acc4[0][I][0] = acc4[0][I][1] = acc4[1][I][0] = acc4[1][I][1] = f32x4{};
    }
    acc4[0][I][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, to_u4(F.w[I])), __builtin_bit_cast(half8, to_u4(F.x[0])), acc4[0][I][0], 0, 0, 0);
    acc4[1][I][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, to_u4(F.w[I])), __builtin_bit_cast(half8, to_u4(F.x[1])), acc4[1][I][0], 0, 0, 0);
    acc4[0][I][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, to_u4(F.x[0])), __builtin_bit_cast(half8, to_u4(F.w[I])), acc4[0][I][1], 0, 0, 0);
    acc4[1][I][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, to_u4(F.x[1])), __builtin_bit_cast(half8, to_u4(F.w[I])), acc4[1][I][1], 0, 0, 0);
#else
    Mfma<T>::run(to_u4(F.w[I]), to_u4(F.x[0]), acc[0][I]);
    Mfma<T>::run(to_u4(F.w[I]), to_u4(F.x[1]), acc[1][I]);
#endif
  };

  // ---- epilogue of the tile (fr, y0, x0, nt): straight from the accumulators
  auto epilogue = [&](int fr, int y0, int x0, int nt, int hsel) __attribute__((always_inline)) {
    const int n0 = nt * BNK;
#if TV_C3_EXP == 3
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[f][i][e] = acc4[f][i][0][e];
          acc[f][i][4 + e] = acc4[f][i][1][e];
        }
#endif
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int q = WP * wave + 32 * f + l32;
      const int y = y0 + q / TW, x = x0 + q % TW;
      const bool ok = y < H && x < W && fr < nframes;
      [[maybe_unused]] OutT* dst = reinterpret_cast<OutT*>(out_ptr) +
                  ((size_t)(fr * H + (ok ? y : 0)) * W + (ok ? x : 0)) * p.out_ldc + p.out_coff + n0;
      // EPI 0: stores through a per-frame buffer resource, every lane always issuing (invalid
      // pixels / channels -> OOB offset, dropped): a fixed count of VMEM operations per tile
      [[maybe_unused]] i32x4 orsrc;
      [[maybe_unused]] unsigned obase = 0;
      if constexpr (EPI == 0) {
        const unsigned long long a = (unsigned long long)out_ptr + (unsigned long long)fr * out_frame_bytes;
        orsrc.x = (int)(unsigned)a;
        orsrc.y = (int)(unsigned)(a >> 32);
        orsrc.z = (int)out_frame_bytes;
        orsrc.w = 0x00020000;
        obase = ok ? ((unsigned)(y * W + x) * (unsigned)p.out_ldc + (unsigned)(p.out_coff + n0 + 8 * lh)) * (unsigned)sizeof(OutT)
                   : 0x80000000u;
      }
      [[maybe_unused]] f32x16 hacc = f32x16{};  // EPI 1: the 1x1 heads' partial sums of this pixel
#pragma unroll
      for (int i = 0; i < NI; ++i) {
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
          if constexpr (EPI == 0) {
            const int ch = n0 + 32 * i + 16 * m;
            const unsigned a0 = pack2<OutT>(v[0][0], v[0][1]), a1 = pack2<OutT>(v[0][2], v[0][3]);
            const unsigned b0 = pack2<OutT>(v[1][0], v[1][1]), b1 = pack2<OutT>(v[1][2], v[1][3]);
            const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
#if TV_C3_EXP == 2  // timing only: the tile's stores dropped (zero-size resource)
            orsrc.z = 0;
#endif
            raw_buffer_store_v4(u32x4{r0[0], r1[0], r0[1], r1[1]}, orsrc,
                                ch < p.N ? (int)(obase + (unsigned)((32 * i + 16 * m) * sizeof(OutT))) : (int)0x80000000u, 0, 0);
          } else {
            // the 8 hidden channels 32i+16m+8lh.. of this pixel are the MFMA B operand of k-step
            // 2i+m of the 1x1, as a hi + lo pair of T values (hi = T(v), lo = T(v - hi)): the
            // 1x1 sees the fp32 hidden activation to ~2x T's precision, not its T rounding
            // (the reference's hidden tensor is fp32; +16 MFMAs per 576-MFMA tile)
            float lo[2][4];
#pragma unroll
            for (int gg = 0; gg < 2; ++gg)
#pragma unroll
              for (int e = 0; e < 4; ++e) lo[gg][e] = v[gg][e] - (float)(T)v[gg][e];
            const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
            const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
            const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
            const uint4 hv = make_uint4(r0[0], r1[0], r0[1], r1[1]);
            const unsigned c0 = pack2<T>(lo[0][0], lo[0][1]), c1 = pack2<T>(lo[0][2], lo[0][3]);
            const unsigned d0 = pack2<T>(lo[1][0], lo[1][1]), d1 = pack2<T>(lo[1][2], lo[1][3]);
            const auto s0 = __builtin_amdgcn_permlane32_swap(c0, d0, false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(c1, d1, false, false);
            const uint4 hl = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            // (staged in LDS by the tile's block 0: head_piece; landed and visible since that
            // block's tap-8 wait and the barriers after it)
            const uint4 hwf = *reinterpret_cast<const uint4*>(smem + OFF_HW + hsel * HWB + (2 * i + m) * 1024 + lane * 16);
            Mfma<T>::run(hwf, hv, hacc);
            Mfma<T>::run(hwf, hl, hacc);
          }
          __builtin_amdgcn_sched_barrier(0);  // bound the live set: one 8-channel group at a time
        }
      }
      if constexpr (EPI == 1) {
        // rows r = 8G + 4lh + e of the 1x1 result (lane: pixel l32): output column head_row0[nt] + r
        // of the pixel. The partial sums are added with float atomics (the two 128-channel halves
        // of a 256-channel head meet in the output), which run at the memory side in 64-byte
        // requests: a lane-per-pixel add touches 32 pixels' lines per instruction. So each half
        // of 16 rows is transposed through this wave's LDS scratch first, and lane idx of the adds
        // takes (pixel idx / n, row idx % n): one instruction covers 64 / n pixels' contiguous rows.
        const int nr = p.head_nrows[nt];
        const float* hb = p.head_b + nt * 32;
        float* hs = reinterpret_cast<float*>(smem + OFF_HS + wave * HSW);
        float* hout = reinterpret_cast<float*>(out_ptr) + p.head_row0[nt];
        const int qf = WP * wave + 32 * f;  // the fragment's first pixel in the tile
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int n = min(16, nr - 16 * hh);  // wave-uniform
          if (n <= 0) break;
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            const int G = 2 * hh + g;
            *reinterpret_cast<f32x4*>(hs + l32 * 16 + 8 * g + 4 * lh) =
                f32x4{hacc[4 * G + 0], hacc[4 * G + 1], hacc[4 * G + 2], hacc[4 * G + 3]};
          }
          // lanes read rows other lanes wrote: order the wave's LDS writes before its reads
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const bool plain = p.head_store;  // (uniform) each output column from exactly one tile
          for (int idx = lane; idx < 32 * n; idx += 64) {
            const int px = idx / n, r = idx - px * n;
            const int qq = qf + px;
            const int yy = y0 + qq / TW, xx = x0 + qq % TW;
            if (yy < H && xx < W && fr < nframes) {
              float* dst = hout + ((size_t)(fr * H + yy) * W + xx) * p.head_ldc + 16 * hh + r;
              const float val = hs[px * 16 + r] + hb[16 * hh + r];
              if (plain) *dst = 0.0f + val;  // (the atomic path's sum onto a zeroed output: 0 + v)
              else unsafeAtomicAdd(dst, val);
            }
          }
          // ... and those reads before the next half's / fragment's writes of the scratch
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
  };

  // ---- K16 epilogue: lane (c16, n16) holds channels 16i + 4c16 + e of pixel pin of fragment f.
  // Per channel-fragment pair (2j, 2j+1) one v_permlane16_swap per dword gives every lane 8
  // consecutive channels — rows c16 = 0..3 of the pair: 32j + {0, 16, 8, 24} — one 16-byte store
  // (a pixel's 64 contiguous bytes per instruction).
  [[maybe_unused]] const int cofs16 = 16 * (c16 & 1) + 8 * (c16 >> 1);
  [[maybe_unused]] auto epilogue16 = [&](int fr, int y0, int x0, int nt) __attribute__((always_inline)) {
    mfma16_drain();
    const int n0 = nt * BNK;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int q = WP * wave + 16 * f + pin;
      const int y = y0 + q / TW, x = x0 + q % TW;
      const bool ok = y < H && x < W && fr < nframes;
      i32x4 orsrc;
      const unsigned long long a = (unsigned long long)out_ptr + (unsigned long long)fr * out_frame_bytes;
      orsrc.x = (int)(unsigned)a;
      orsrc.y = (int)(unsigned)(a >> 32);
      orsrc.z = (int)out_frame_bytes;
      orsrc.w = 0x00020000;
      const unsigned obase = ok ? ((unsigned)(y * W + x) * (unsigned)p.out_ldc + (unsigned)(p.out_coff + n0 + cofs16)) * (unsigned)sizeof(OutT)
                                : 0x80000000u;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        float v[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 bb = *reinterpret_cast<const f32x4*>(lbias + n0 + 32 * j + 16 * h + 4 * c16);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float t = a16[f][2 * j + h][e] + bb[e];
            if constexpr (ACT == 1) t = fmaxf(t, 0.0f);
            else if constexpr (ACT == 2) t = fmaxf(t, 0.01f * t);
            v[h][e] = t;
          }
        }
        const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
        const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
        const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
        const u32x4 hv = u32x4{r0[0], r1[0], r0[1], r1[1]};
        const int ch = n0 + 32 * j + cofs16;
        raw_buffer_store_v4(hv, orsrc, ch < p.N ? (int)(obase + (unsigned)(32 * j * sizeof(OutT))) : (int)0x80000000u, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // bound the live set: one channel-fragment pair at a time
      }
    }
  };

  // ---- prologue: halo of (tile 0, block 0), weights of k-steps 0..2
  int cur_fr, cur_y0, cur_x0, cur_nt;
  tile_of(0, cur_fr, cur_y0, cur_x0, cur_nt);
  halo_offsets(cur_fr, cur_y0, cur_x0);
  auto halo_all = [&](auto self, auto i) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
    if constexpr (I < HPW) {
      halo_piece(IC<I>{}, 0, 0);
      self(self, IC<I + 1>{});
    }
  };
  halo_all(halo_all, IC<0>{});
  __builtin_amdgcn_sched_barrier(0);  // the counted wait below needs the halo issued first
  // weights: k-steps 0, 1 into ring slots 0, 1; k-steps 2, 3, 4 in flight in sets 2, 3, 0
  // (S_tot >= SPTK > 5). Every VMEM operation of the main loop is issued unconditionally —
  // past the end of the list the weight loads re-read the last tile's k-steps and the halo
  // pieces reload the current tile into the idle buffer — so that the compiler's own vmcnt
  // for each weight ds_write is exact: a conditional load makes it fall back to vmcnt(0),
  // which drains the halo pieces and weight loads issued since (measured: ~20% of the layer).
  w_load(wreg[0]);
  w_load(wreg[1]);
  *reinterpret_cast<WReg*>(smem + OFF_W + wvoff) = wreg[0];
  *reinterpret_cast<WReg*>(smem + OFF_W + WSLOT + wvoff) = wreg[1];
  w_load(wreg[2]);
  w_load(wreg[3]);
  w_load(wreg[0]);
  if constexpr (EPI == 0) {
    // as many (dropped: zero-size resource) stores as a tile epilogue issues, so that both paths
    // into the tile loop carry the same VMEM sequence and the compiler's vmcnt for the first
    // weight ds_writes of a tile leaves the previous tile's stores in flight
    __builtin_amdgcn_sched_barrier(0);
    i32x4 nul;
    nul.x = (int)(unsigned)(unsigned long long)out_ptr;
    nul.y = (int)(unsigned)((unsigned long long)out_ptr >> 32);
    nul.z = 0;
    nul.w = 0x00020000;
#pragma unroll
    for (int k = 0; k < 4 * NI; ++k) raw_buffer_store_v4(u32x4{0u, 0u, 0u, 0u}, nul, k * 16, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the halo (issued first) landed; the weights of k-steps 2..4 (and the dropped stores) may stay in flight
  wait_vm<3 * WLN + (EPI == 0 ? 4 * NI : 0)>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  Half<NI> H0, H1;  // sub-step 0 / 1 fragments
  if constexpr (K16) {
    X16[0][0] = rd_x16(IC<0>{}, IC<0>{}, xa16);
    X16[0][1] = rd_x16(IC<1>{}, IC<0>{}, xa16);
    X16[0][2] = rd_x16(IC<2>{}, IC<0>{}, xa16);
    X16[0][3] = rd_x16(IC<3>{}, IC<0>{}, xa16);
#pragma unroll
    for (int i = 0; i < NI; ++i) W16[0][i] = ds_read16<0>(wa16 + i * 1024);
  } else {
    read_one(IC<0>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
    read_one(IC<1>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
    read_one(IC<2>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
    read_one(IC<3>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
    if constexpr (NI == 4) {
      read_one(IC<4>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
      read_one(IC<5>{}, IC<0>{}, IC<0>{}, xa, wa[0], H0);
    }
  }

  C3_STAMP(4);
  // static priority for the second-dispatched half (waves 4-7, the SIMD partners of waves 0-3):
  // the arbitration loser on every segment otherwise (MI355X_MICROARCH.md, two waves per SIMD,
  // item 4). Measured: 60x80 layers -3%, the others -0.4..-1%
  if (NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  int s = 0;   // global k-step
  int tl = 0;  // tile index within this block's list
  int cb = 0;  // channel block within the tile (compile-time inside cblock)
  // the channel block after the current one: same tile cb+1, or the next tile's block 0
  bool nxt_exists = true, nxt_newtile = false;

  // One k-step with compile-time tap. On entry H0 holds its sub-step-0 fragments; the first
  // half (8 MFMAs on H0) overlaps the reads of its sub-step-1 fragments into H1, the second
  // half (8 MFMAs on H1) the reads of the NEXT k-step's sub-step-0 fragments into H0. The
  // k-step's LDS-DMA pieces (1 weight, <= 1 halo) are issued between MFMA pairs.
  // Halo buffer of channel block cb is cb & 1 (NCB is even, so parity is per-tile fixed).
  auto step = [&](auto tap, auto first, auto par) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tap)::value;
    // Weights of k-step s+1 were written to LDS at step s-1 (lgkmcnt + barrier below); halo and
    // residual data arrive by LDS-DMA and are waited for with an exact vmcnt: the count of
    // vector-memory operations issued after the last piece the next k-step reads. A weight load
    // is issued at every step q >= 0; within a step the order is halo piece (taps 0..5, next
    // channel block), residual piece (RES, taps 1..4, this channel block), weight load.
    //  * tap 8 without RES / residual step (tap 9): the next k-step reads the NEXT channel
    //    block's halo (last piece at tap 5): younger = the weight loads of taps 5, 6, 7 (and 8);
    //  * tap 8 with RES: the residual step reads this block's residual input (last piece at
    //    tap 4): younger = weight loads of taps 4, 5, 6, 7 + the tap-5 halo piece.
    static_assert(HTAPS == 6 || (HTAPS == 7 && !RES), "the tap-8 count: the last halo piece at tap 5 or 6");
    C3_STAMP(2);
#if TV_C3_EXP == 9
    st_b[5] += 1;
#endif
    auto wl = [&](int q) { return q >= 0 ? WLN : 0; };
    // (the last halo piece goes out at tap HTAPS - 1: taps 5 or 6; the weight loads of the taps
    // from there to 7 are younger)
    if constexpr (TAP == 8 && !RES) wait_vm_n(s + 1 < S_tot ? (HTAPS <= 6 ? wl(s - 3) : 0) + wl(s - 2) + wl(s - 1) : 0);
    if constexpr (TAP == 8 && RES) wait_vm_n(s + 1 < S_tot ? wl(s - 4) + wl(s - 3) + wl(s - 2) + wl(s - 1) + 1 : 0);
    if constexpr (TAP == 9) wait_vm_n(s + 1 < S_tot ? wl(s - 4) + wl(s - 3) + wl(s - 2) + wl(s - 1) : 0);
    if constexpr (TAP >= 8) C3_STAMP(6);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if TV_C3_EXP == 4  // timing only: barrier only at tap 8 (wrong results)
    if constexpr (TAP >= 8) __builtin_amdgcn_s_barrier();
#else
    __builtin_amdgcn_s_barrier();
#endif
    __builtin_amdgcn_sched_barrier(0);
    C3_STAMP(TAP >= 8 ? 7 : 0);

    constexpr int NTAP = TAP == 8 ? (RES ? 9 : 0) : TAP == 9 ? 0 : TAP + 1;
    const bool do_r = s + 1 < S_tot;
    const int hbuf = (cb + 1) & 1;
    const unsigned xc = xa + (cb & 1) * HBUF;                                  // this k-step's halo
    const unsigned xn = xa + (NTAP == 0 ? hbuf : (cb & 1)) * HBUF;             // next k-step's halo
    const unsigned wc1 = wa[1] + (unsigned)((s % RG) * WSLOT);
    const unsigned wn0 = wa[0] + (unsigned)(((s + 1) % RG) * WSLOT);
    // first half: sub-step 0 MFMAs; sub-step 1 reads of this k-step go out first (H1 is free)
    constexpr bool FIRST = TAP == 0 && decltype(first)::value;
    constexpr int PAR = decltype(par)::value;  // s % 4 (36 or 40 k-steps per tile: static)
    if constexpr (K16) {
      // first half: channel fragments 0..NI-1 (W16[0], read during the previous k-step) x the 4
      // pixel fragments, channel-major; this k-step's fragments NI..2NI-1 go out first (W16[1] is
      // free). Second half: W16[1] x the pixel fragments, pixel-major, so that each pixel fragment
      // retires after its NI MFMAs and the next k-step's fragment is read into the same registers
      // (one operand set live: 4 + 2 NI fragments, as the 32x32 body's two sub-step sets); the
      // next k-step's channel fragments 0..NI-1 go into W16[0], free since the first half.
      const unsigned x16n = xa16 + (NTAP == 0 ? hbuf : (cb & 1)) * HBUF;
      const unsigned w16c = wa16 + (unsigned)((s % RG) * WSLOT);
      const unsigned w16n = wa16 + (unsigned)(((s + 1) % RG) * WSLOT);
      u32x4(&X)[4] = X16[0];
      u32x4(&WA)[NI] = W16[0];
      u32x4(&WB)[NI] = W16[1];
      quad16(IC<0>{}, IC<FIRST>{}, WA[0], X);
      WB[0] = ds_read16<NI * 1024>(w16c);
      WB[1] = ds_read16<(NI + 1) * 1024>(w16c);
      __builtin_amdgcn_sched_barrier(0);
      quad16(IC<1>{}, IC<FIRST>{}, WA[1], X);
      if constexpr (NI == 4) {
        WB[2] = ds_read16<6 * 1024>(w16c);
        WB[3] = ds_read16<7 * 1024>(w16c);
      }
#if TV_C3_EXP != 6
      *reinterpret_cast<WReg*>(smem + OFF_W + ((s + WD) % RG) * WSLOT + wvoff) = wreg[(PAR + WD) & 3];
#endif
      if constexpr (TAP == 0) {
        if (nxt_exists && nxt_newtile) {
          int fr, y0, x0, nt;
          tile_of(tl + 1, fr, y0, x0, nt);
          halo_offsets(fr, y0, x0);
        }
      }
      if constexpr (NI == 4) {
        __builtin_amdgcn_sched_barrier(0);
        quad16(IC<2>{}, IC<FIRST>{}, WA[2], X);
      }
      if constexpr (TAP < HTAPS) halo_piece(IC<TAP>{}, nxt_newtile ? 0 : cb + 1, hbuf);
      if constexpr (RES && TAP >= 1 && TAP <= RPW) res_piece(TAP - 1, cur_fr, cur_y0, cur_x0, cb);
      if constexpr (NI == 4) {
        __builtin_amdgcn_sched_barrier(0);
        quad16(IC<3>{}, IC<FIRST>{}, WA[3], X);
      }
      __builtin_amdgcn_sched_barrier(0);
      C3_STAMP(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // W16[1] landed
      __builtin_amdgcn_sched_barrier(0);
      auto group = [&](auto f) __attribute__((always_inline)) {  // pixel fragment F x W16[1]
        constexpr int F = decltype(f)::value;
#pragma unroll
        for (int i = 0; i < NI; ++i) mfma16_asm<T, FIRST>(a16[F][NI + i], WB[i], X[F]);
      };
      group(IC<0>{});
      w_load(wreg[(PAR + 1) & 3]);
      WA[0] = ds_read16<0>(w16n);
      WA[1] = ds_read16<1024>(w16n);
      X[0] = rd_x16(IC<0>{}, IC<NTAP>{}, x16n);
      __builtin_amdgcn_sched_barrier(0);
      group(IC<1>{});
      if constexpr (NI == 4) {
        WA[2] = ds_read16<2048>(w16n);
        WA[3] = ds_read16<3072>(w16n);
      }
      X[1] = rd_x16(IC<1>{}, IC<NTAP>{}, x16n);
      __builtin_amdgcn_sched_barrier(0);
      group(IC<2>{});
      X[2] = rd_x16(IC<2>{}, IC<NTAP>{}, x16n);
      __builtin_amdgcn_sched_barrier(0);
      group(IC<3>{});
      X[3] = rd_x16(IC<3>{}, IC<NTAP>{}, x16n);
      __builtin_amdgcn_sched_barrier(0);
      ++s;
      return;
    }
    mfma_pair(IC<0>{}, IC<FIRST>{}, H0);
    read_one(IC<0>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
    read_one(IC<1>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<1>{}, IC<FIRST>{}, H0);
    read_one(IC<2>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
    read_one(IC<3>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
    // k-step s+2 (loaded at step s-3) into its ring slot: it last held k-step s-1, read
    // completely before this step's barrier (past the end: an unread slot)
#if TV_C3_EXP != 6  // 6: timing only, no weight ds_write (wrong results)
    *reinterpret_cast<WReg*>(smem + OFF_W + ((s + WD) % RG) * WSLOT + wvoff) = wreg[(PAR + WD) & 3];
#endif
    if constexpr (TAP == 0) {
      if (nxt_exists && nxt_newtile) {
        int fr, y0, x0, nt;
        tile_of(tl + 1, fr, y0, x0, nt);
        halo_offsets(fr, y0, x0);
      }
    }
    if constexpr (NI == 4) {
      __builtin_amdgcn_sched_barrier(0);
      mfma_pair(IC<2>{}, IC<FIRST>{}, H0);
      read_one(IC<4>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
      read_one(IC<5>{}, IC<1>{}, IC<TAP>{}, xc, wc1, H1);
    }
    if constexpr (TAP < HTAPS)
#if TV_C3_EXP != 5  // 5: timing only, no halo DMA in the main loop (wrong results)
      halo_piece(IC<TAP>{}, nxt_newtile ? 0 : cb + 1, hbuf);  // (no next block: the idle buffer)
#endif
    if constexpr (RES && TAP >= 1 && TAP <= RPW) res_piece(TAP - 1, cur_fr, cur_y0, cur_x0, cb);
    if constexpr (NI == 4) {
      __builtin_amdgcn_sched_barrier(0);
      mfma_pair(IC<3>{}, IC<FIRST>{}, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    C3_STAMP(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // H1 landed
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<0>{}, IC<false>{}, H1);
    // k-step s+5 into the set whose k-step s+1 went to LDS at step s-1. Issued here, after the
    // halo/residual pieces and away from the barrier where all 8 waves issue at once (-4%)
    w_load(wreg[(PAR + 1) & 3]);
    if (do_r) {
      read_one(IC<0>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
      read_one(IC<1>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_pair(IC<1>{}, IC<false>{}, H1);
    if (do_r) {
      read_one(IC<2>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
      read_one(IC<3>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
    }
    if constexpr (NI == 4) {
      __builtin_amdgcn_sched_barrier(0);
      mfma_pair(IC<2>{}, IC<false>{}, H1);
      if (do_r) {
        read_one(IC<4>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
        read_one(IC<5>{}, IC<0>{}, IC<NTAP>{}, xn, wn0, H0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_pair(IC<3>{}, IC<false>{}, H1);
    }
    __builtin_amdgcn_sched_barrier(0);
    ++s;
  };

  auto cblock = [&](auto cbc, auto tpos) __attribute__((always_inline)) {
    constexpr int CB = decltype(cbc)::value;
    cb = CB;
    nxt_newtile = CB + 1 == NCB;
    nxt_exists = !nxt_newtile || tl + 1 < ntl;
    // k-step index of the block's tap 0 within the tile body (a pair of tiles when NCB == 2)
    constexpr int P0 = decltype(tpos)::value * SPTK + CB * (9 + RES);
    step(IC<0>{}, IC<CB == 0>{}, IC<(P0 + 0) & 3>{});
    // EPI 1: the tile's 1x1 head weights into LDS buffer tl & 1 (the other buffer may still be read
    // by the previous tile's epilogue). Issued before this block's tap-5 halo piece, so the tap-8
    // counted wait drains it; unconditional, like every main-loop VMEM operation.
    if constexpr (EPI == 1 && CB == 0) head_piece(cur_nt, tl & 1);
    step(IC<1>{}, IC<false>{}, IC<(P0 + 1) & 3>{});
    step(IC<2>{}, IC<false>{}, IC<(P0 + 2) & 3>{});
    step(IC<3>{}, IC<false>{}, IC<(P0 + 3) & 3>{});
    step(IC<4>{}, IC<false>{}, IC<(P0 + 4) & 3>{});
    step(IC<5>{}, IC<false>{}, IC<(P0 + 5) & 3>{});
    step(IC<6>{}, IC<false>{}, IC<(P0 + 6) & 3>{});
    step(IC<7>{}, IC<false>{}, IC<(P0 + 7) & 3>{});
    step(IC<8>{}, IC<false>{}, IC<(P0 + 8) & 3>{});
    if constexpr (RES) step(IC<9>{}, IC<false>{}, IC<(P0 + 9) & 3>{});
  };

  // NCB channel blocks per tile, fully unrolled (36 / 72 k-steps of straight-line code): the
  // accumulators keep one register assignment through the whole tile
  static_assert(NCB % 2 == 0 && (UP * SPTK) % 4 == 0, "tile body: an even number of channel blocks (halo buffer parity), k-steps per body a multiple of the 4 weight register sets");
  auto blocks = [&](auto self, auto i, auto tpos) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
    if constexpr (I < NCB) {
      cblock(IC<I>{}, tpos);
      self(self, IC<I + 1>{}, tpos);
    }
  };
  for (; tl < ntl;) {
    blocks(blocks, IC<0>{}, IC<0>{});
    C3_STAMP(2);
    if constexpr (K16) epilogue16(cur_fr, cur_y0, cur_x0, cur_nt);
    else epilogue(cur_fr, cur_y0, cur_x0, cur_nt, tl & 1);
    C3_STAMP(3);
    ++tl;
    if (tl < ntl) tile_of(tl, cur_fr, cur_y0, cur_x0, cur_nt);
    if constexpr (UP == 2) {  // the pair's second unit (ntl is even)
      blocks(blocks, IC<0>{}, IC<1>{});
      C3_STAMP(2);
      if constexpr (K16) epilogue16(cur_fr, cur_y0, cur_x0, cur_nt);
      else epilogue(cur_fr, cur_y0, cur_x0, cur_nt, tl & 1);
      C3_STAMP(3);
      ++tl;
      if (tl < ntl) tile_of(tl, cur_fr, cur_y0, cur_x0, cur_nt);
    }
  }
#if TV_C3_EXP == 9
  if (p.dbg && lane == 0) {
    unsigned long long* d = p.dbg + ((size_t)blockIdx.x * NW + wave) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = st_b[k];
  }
#endif
}

template <typename T, int TW, int ACT, int EPI = 0, int RES = 0, int NI = 4, int NCB = 4, int NWV = 8>
inline int launch_t(const ConvParams& p, const ConvParams* dp, void* out, int grid, hipStream_t s) {
  auto k = conv3x3<T, T, TW, ACT, EPI, RES, NI, NCB, NWV>;
  using Gm = Geo<NWV, TW>;
  constexpr int lds = Gm::template lds<RES, EPI>();
  if (NWV == 4 && p.ntiles * BN > Gm::MAXN) {
    set_error("conv3x3: 4-wave workgroups take <= 256 output channels");
    return 1;
  }
  if (int r = ensure_lds<conv3x3<T, T, TW, ACT, EPI, RES, NI, NCB, NWV>>(lds)) return r;
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NWV), lds, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}


using Launch = int (*)(const ConvParams&, const ConvParams*, void*, int, hipStream_t);
// the plain-epilogue instances of a channel-block count and workgroup size: [bf16][ni == 4][tw == 32][act]
template <int NCB, int NWV>
int launch_plain(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s, int ni) {
  static const Launch t[2][2][2][3] = {
      {{{launch_t<_Float16, 16, 0, 0, 0, 2, NCB, NWV>, launch_t<_Float16, 16, 1, 0, 0, 2, NCB, NWV>, launch_t<_Float16, 16, 2, 0, 0, 2, NCB, NWV>},
        {launch_t<_Float16, 32, 0, 0, 0, 2, NCB, NWV>, launch_t<_Float16, 32, 1, 0, 0, 2, NCB, NWV>, launch_t<_Float16, 32, 2, 0, 0, 2, NCB, NWV>}},
       {{launch_t<_Float16, 16, 0, 0, 0, 4, NCB, NWV>, launch_t<_Float16, 16, 1, 0, 0, 4, NCB, NWV>, launch_t<_Float16, 16, 2, 0, 0, 4, NCB, NWV>},
        {launch_t<_Float16, 32, 0, 0, 0, 4, NCB, NWV>, launch_t<_Float16, 32, 1, 0, 0, 4, NCB, NWV>, launch_t<_Float16, 32, 2, 0, 0, 4, NCB, NWV>}}},
      {{{launch_t<__bf16, 16, 0, 0, 0, 2, NCB, NWV>, launch_t<__bf16, 16, 1, 0, 0, 2, NCB, NWV>, launch_t<__bf16, 16, 2, 0, 0, 2, NCB, NWV>},
        {launch_t<__bf16, 32, 0, 0, 0, 2, NCB, NWV>, launch_t<__bf16, 32, 1, 0, 0, 2, NCB, NWV>, launch_t<__bf16, 32, 2, 0, 0, 2, NCB, NWV>}},
       {{launch_t<__bf16, 16, 0, 0, 0, 4, NCB, NWV>, launch_t<__bf16, 16, 1, 0, 0, 4, NCB, NWV>, launch_t<__bf16, 16, 2, 0, 0, 4, NCB, NWV>},
        {launch_t<__bf16, 32, 0, 0, 0, 4, NCB, NWV>, launch_t<__bf16, 32, 1, 0, 0, 4, NCB, NWV>, launch_t<__bf16, 32, 2, 0, 0, 4, NCB, NWV>}}}};
  if (dtype != F16 && dtype != BF16) {
    set_error("conv3x3: fp16/bf16 only");
    return 1;
  }
  return t[dtype == BF16][ni == 4][tw == 32][p.act](p, dp, out, grid, s);
}
// per input-channel-count instance tables (conv3x3_n2/n4/n8.hip)
int launch_ncb2(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s,
                int epi, int res, int ni, int nw);
int launch_ncb4(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s,
                int epi, int res, int ni, int nw);
int launch_ncb8(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s,
                int epi, int res, int ni, int nw);
// the residual (RES) instances of a channel-block count: ReLU, plain stores, [bf16][tw == 32][ni == 4]
template <int NCB>
int launch_res(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s,
               int epi, int ni) {
  if (p.act != 1 || epi != 0 || p.nseg != 2) {
    set_error("conv3x3: residual k-steps need ReLU, plain stores and two segments");
    return 1;
  }
  static const Launch r[2][2][2] = {
      {{launch_t<_Float16, 16, 1, 0, 1, 2, NCB>, launch_t<_Float16, 16, 1, 0, 1, 4, NCB>},
       {launch_t<_Float16, 32, 1, 0, 1, 2, NCB>, launch_t<_Float16, 32, 1, 0, 1, 4, NCB>}},
      {{launch_t<__bf16, 16, 1, 0, 1, 2, NCB>, launch_t<__bf16, 16, 1, 0, 1, 4, NCB>},
       {launch_t<__bf16, 32, 1, 0, 1, 2, NCB>, launch_t<__bf16, 32, 1, 0, 1, 4, NCB>}}};
  if (dtype != F16 && dtype != BF16) {
    set_error("conv3x3: fp16/bf16 only");
    return 1;
  }
  return r[dtype == BF16][tw == 32][ni == 4](p, dp, out, grid, s);
}

}  // namespace c3
}  // namespace tv
