// Fused input staging + 7x7 stem + ResidualBlock conv1 (3x3 / stride 2) (gfx950, fp16 / bf16):
// the reference's ToTensor + Normalize (centernet_node.py:90-92), DLADown.projection_layer
// (Conv2d(3, 128, 7, padding=3) + BatchNorm + ReLU at full resolution, dla.py:150-154, 182-183) and
// block_layers[0].conv1 (Conv2d(128, 128, 3, stride 2, padding 1) + BN + ReLU, dla.py:13-19, 185-186)
// in one launch, plus the stride-2 samples of the stem output that the block's 1x1 conv_residual
// reads (dla.py:32-37).
//
// Why: unfused, the stem writes 128 channels x 2 B per input pixel (5.0 GB per 64-frame batch)
// and conv1 + the residual read them back (~10 GB of fetches with halo re-reads): the largest
// avoidable HBM round trip of the R18 step. Here the stem output never reaches HBM:
//  * a persistent 512-thread workgroup per CU (8 waves, two per SIMD) owns 16 x 32 conv1 output
//    tiles; wave w computes rows 2w, 2w + 1 x all 128 channels (8 32x32 MFMA accumulators, 8
//    MFMAs per 16-deep sub-step on 6 fragment reads). Measured alternatives (profiles/r4): 8 x 32
//    tiles (64 x 64 per wave) 1.41-1.47 ms per 32-frame slice, the per-k-step overhead on half
//    the MFMAs; one 512-register wave per SIMD (4 waves, 128 x 128 each) 1.94 ms; this form
//    1.19-1.22 ms against 1.30 for stem.hip + conv3x3s2.hip;
//  * conv1's K loop is 36 k-steps (9 taps x 4 channel blocks of 32), as in conv3x3s2.hip —
//    virtual space-to-depth: for each (input row parity p, column parity q) phase block the taps
//    read a (16 + p) x (32 + q) halo of stem pixels (2(oy0 - p + hy) + p, 2(ox0 - q + hx) + q) at
//    80-byte pitch with compile-time immediate ds_read offsets; weights register-staged five
//    k-steps ahead into a 3-slot LDS ring, one barrier per k-step;
//  * the halo of one (phase block, channel block) is not loaded: it is COMPUTED into LDS right
//    before its 1-4 k-steps (stem phase: the 7x7 conv of the block's pixels for its 32 channels,
//    32x32x16 MFMAs in pairs of independent fragments, K = 7 rows x 24 = 168 of the row-expanded
//    input E, bias + ReLU, zeros outside the image = conv1's padding; one fragment per wave at a
//    time: the SIMD's two waves interleave their dependent accumulation chains);
//  * the block order (q = 1 then q = 0; per channel block p = 0 then p = 1) lets E hold one
//    column parity at a time (39 rows x 33 pixels x 48 B) and lets the next channel block's stem
//    weights (44 VGPRs, A operands) load under the longer p = 1 block's k-steps;
//  * the next tile's input window (39 x 71 pixels of u8 HWC, 5 dwords per thread) is fetched into
//    registers in the middle of the current tile and normalised through the 768-entry LUT; the
//    other inputs (normalised fp32 NCHW, u8 of a width not a multiple of 4: 17 values per
//    thread) load at the tile's start, which keeps the kernel inside 256 VGPRs;
//  * the (0, 0) phase block of each channel block IS the stem at the even pixels: it is copied
//    from LDS to `res` (the residual input, [B, Ho, Wo, 128]), which conv2's fused 1x1 residual
//    then reads at stride 1 instead of the 128 x 480 x 640 stem tensor at stride 2.
// Every vector-memory operation of the tile body is issued unconditionally (out-of-range lanes
// use out-of-range buffer offsets), so the compiler's counted waits for the weight ring are exact.
// LDS: halo 44,880 + E 61,776 + window 17,472 + conv1 weight ring 24,576 + biases + LUT = 151,264 B.
// Numerics: the stem values are rounded to the compute dtype exactly as stem.hip stores them;
// conv1 accumulates the same products in fp32 in another k-step order than conv3x3s2.hip.
#include "conv_common.h"

#include <type_traits>

#ifndef TV_C3_EXP
#define TV_C3_EXP 0  // 9: the stamp build (conv3x3_kernel.h) — per-wave cycle buckets into StemS2Params.dbg
#endif
#if TV_C3_EXP == 9
#define SS2_STAMP(B)                                                                   \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    unsigned long long t_;                                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    if (lane == 0) st_b[B] += (unsigned)t_ - st_last; /* LDS: no SGPRs held */         \
    st_last = (unsigned)t_;                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#else
#define SS2_STAMP(B) \
  do {               \
  } while (0)
#endif

#ifndef SS2_RD_AHEAD
#define SS2_RD_AHEAD 2  // stem-phase operands (E reads) in flight per wave
#endif

#ifndef TV_SS2_EXP
#define TV_SS2_EXP 0  // timing-only diagnostic builds (wrong results): 1 = no stem MFMAs, 3 = k-step barriers only
                      // at a block's first k-step, 4 = no conv1 weight staging (ring loads / writes)
#endif

namespace tv {
namespace ss2 {

constexpr int NT = 512, NWV = 8, BN = 128, TH = 16, TW = 32;
constexpr int RPW = TH / NWV;                     // output rows (32-pixel fragments) per wave
constexpr int RS = TW + 1;                        // halo row stride (pixels)
constexpr int PITCH = 80;                         // halo pixel pitch (bytes): 32 channels + pad
constexpr int HBYTES = (TH + 1) * RS * PITCH;     // one (phase block, channel block) halo
constexpr int WR = 2 * TH + 7, WCOL = 2 * TW + 7; // input window rows / pixels (39 x 71)
constexpr int NVROW = WCOL * 3;                   // values per window row (213)
constexpr int NPITCH = 448;                       // bytes per normalised window row in LDS
constexpr int EPIX = 48, ECOLS = RS;              // row-expanded operand: 24 values per (row, pixel)
constexpr int EBYTES = WR * ECOLS * EPIX;
constexpr int KS = 11;                            // stem MFMA k-steps (K = 176 >= 168)
constexpr int WSLOT = BN * 64;                    // conv1 weights of one k-step
constexpr int WPL = WSLOT / NT;                   // weight bytes per lane per k-step (16)
constexpr int RING = 3;
constexpr int OFF_H = 0;
constexpr int OFF_E = OFF_H + HBYTES;
constexpr int OFF_N = OFF_E + EBYTES;
constexpr int OFF_W = OFF_N + WR * NPITCH;
constexpr int OFF_B1 = OFF_W + RING * WSLOT;
constexpr int OFF_BS = OFF_B1 + BN * 4;
constexpr int OFF_LUT = OFF_BS + BN * 4;
constexpr int LDS = OFF_LUT + 768 * 2;
static_assert(LDS <= 160 * 1024, "LDS budget");
static_assert(OFF_E % 16 == 0 && OFF_N % 16 == 0 && OFF_W % 16 == 0 && OFF_B1 % 16 == 0 && OFF_LUT % 16 == 0,
              "16-byte aligned carve");
static_assert(NPITCH >= NVROW * 2 + 20, "expand reads 5 dwords past a chunk start");
static_assert(WPL == 16, "one 16-byte weight chunk per lane per k-step");

// ---- block / k-step schedule of a tile: block b = (column parity q, channel block cb, row
// parity p): q = 1 for b < 8; cb = (b & 7) / 2; p = b & 1
constexpr int NBLK = 16, SPT = 36;
constexpr int blk_q(int b) { return b < 8 ? 1 : 0; }
constexpr int blk_cb(int b) { return (b & 7) >> 1; }
constexpr int blk_p(int b) { return b & 1; }
constexpr int pb_len(int p, int q) { return (p ? 2 : 1) * (q ? 2 : 1); }
// conv3x3s2.hip's k-step index j of phase block (p, q): (1,1) 0..3, (1,0) 4..5, (0,1) 6..7, (0,0) 8
constexpr int pb_j0(int p, int q) { return p ? (q ? 0 : 4) : (q ? 6 : 8); }
constexpr int J_TY[9] = {0, 0, 1, 1, 0, 1, 0, 0, 0};
constexpr int J_TX[9] = {0, 1, 0, 1, 0, 0, 0, 1, 0};
constexpr int J_TAP[9] = {0, 2, 6, 8, 1, 7, 3, 5, 4};  // ky * 3 + kx of k-step j
struct Sched {
  int blk[SPT], j[SPT], t[SPT], len[SPT], first[NBLK];
};
constexpr Sched make_sched() {
  Sched sc{};
  int s = 0;
  for (int b = 0; b < NBLK; ++b) {
    const int p = blk_p(b), q = blk_q(b), L = pb_len(p, q);
    sc.first[b] = s;
    for (int t = 0; t < L; ++t, ++s) {
      sc.blk[s] = b;
      sc.j[s] = pb_j0(p, q) + t;
      sc.t[s] = t;
      sc.len[s] = L;
    }
  }
  return sc;
}
constexpr Sched SCH = make_sched();
static_assert(SCH.first[NBLK - 1] + pb_len(1, 0) == SPT, "36 k-steps per tile");

template <int MODE> struct Win;  // input window staging: registers per thread
template <> struct Win<0> { static constexpr int NS = (WR * NVROW + NT - 1) / NT; };  // fp32 NCHW values
template <> struct Win<1> { static constexpr int NS = (WR * NVROW + NT - 1) / NT; };  // u8 bytes
template <> struct Win<2> { static constexpr int DW = 54, NS = (WR * 54 + NT - 1) / NT; };  // u8 dwords (W % 4 == 0)

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ unsigned raw_buffer_load_u32(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ unsigned char raw_buffer_load_u8(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i8");
__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");

constexpr int OOB = (int)0x80000000u;  // a buffer offset past every resource: loads 0, stores dropped

__device__ __forceinline__ i32x4 rsrc_of(const void* base, unsigned long long bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = (int)(unsigned)a;
  r.y = (int)(unsigned)(a >> 32);
  r.z = (int)(unsigned)bytes;
  r.w = 0x00020000;
  return r;
}

template <int OFF>
__device__ __forceinline__ u32x4 ds_read16(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

template <int V>
using IC = std::integral_constant<int, V>;
template <int Q, int N, typename F>
__device__ __forceinline__ void unroll(F& f) {
  if constexpr (Q < N) {
    f(IC<Q>{});
    unroll<Q + 1, N>(f);
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

struct Half {     // conv1 fragments of one 16-deep sub-step
  u32x4 x[RPW];   // pixel fragments: tile rows 4w + f
  u32x4 w[4];     // channel fragments: channels 32 i
};
struct WReg {
  u32x4 a;
};

// a lane value the compiler must recompute where it is used: keeps the per-block stem / copy /
// staging addresses (functions of the lane alone) from being hoisted out of the tile loop, where
// 16 blocks' worth of them would stay live across the whole tile
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <typename T, int MODE>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void stem_s2(StemS2Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NS = Win<MODE>::NS;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int H = p.H, W = p.W, Ho = p.Ho, Wo = p.Wo;
  const int tiles_x = (Wo + TW - 1) / TW;
  const int tiles_f = ((Ho + TH - 1) / TH) * tiles_x;
  const int ntot = p.B * tiles_f;

  // ---- this block's tiles: XCD-aware contiguous ranges (conv3x3s2.hip)
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
#if TV_C3_EXP == 9
  // buckets: 0 block barrier wait, 1 stem phase, 2 k-step barrier wait (+ a block's first reads),
  // 3 k-step MFMA halves, 4 staging under the k-steps, 5 epilogue, 6 prologue / tile end, 7 k-steps
  unsigned* st_b = reinterpret_cast<unsigned*>(smem + LDS) + wave * 8;  // the stamp build's extra LDS
  if (lane < 8) st_b[lane] = 0;
  unsigned st_last;
  {
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    st_last = (unsigned)t0;
  }
#endif
  auto tile_of = [&](int idx, int& fr, int& oy0, int& ox0) __attribute__((always_inline)) {
    const int t = first + min(idx, ntl - 1) * stride;  // past the list: the last tile again
    fr = t / tiles_f;
    const int r = t - fr * tiles_f;
    const int ty = r / tiles_x;
    oy0 = ty * TH;
    ox0 = (r - ty * tiles_x) * TW;
  };

  // ---- resident: biases, LUT
  {
    float* lb1 = reinterpret_cast<float*>(smem + OFF_B1);
    float* lbs = reinterpret_cast<float*>(smem + OFF_BS);
    if (tid < BN) lb1[tid] = p.bias1[tid];
    else if (tid < 2 * BN) lbs[tid - BN] = p.stem_bias[tid - BN];
    if constexpr (MODE != 0) {
      T* lut = reinterpret_cast<T*>(smem + OFF_LUT);
      for (int i = tid; i < 768; i += NT) {
        const int v = i / 3, c = i - v * 3;
        lut[i] = (T)(((float)v / 255.0f - kMean[c]) / kStd[c]);  // prep_u8's expression, bit for bit
      }
    }
  }

  // ---- input window of a tile: rows 2 oy0 - 4 .. + 38, pixels 2 ox0 - 4 .. + 70
  const unsigned long long in_frame = MODE == 0 ? (unsigned long long)3 * H * W * 4 : (unsigned long long)H * W * 3;
  unsigned raw[NS];
  auto load_window = [&](int fr, int oy0, int ox0) __attribute__((always_inline)) {
    const int wy0 = 2 * oy0 - 4, wx0 = 2 * ox0 - 4;
    const i32x4 rs = rsrc_of((const char*)p.input + (size_t)fr * in_frame, in_frame);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int idx = opaque(tid) + k * NT;
      if constexpr (MODE == 2) {
        const int r = idx / Win<2>::DW, dw = idx - r * Win<2>::DW;
        const int y = wy0 + r, bx = 3 * wx0 + 4 * dw;  // 3 wx0 = 6 ox0 - 12 is dword aligned
        const bool ok = idx < WR * Win<2>::DW && (unsigned)y < (unsigned)H && bx >= 0 && bx < 3 * W;
        raw[k] = raw_buffer_load_u32(rs, ok ? y * 3 * W + bx : OOB, 0, 0);
      } else {
        const int r = idx / NVROW, q = idx - r * NVROW;
        const int xx = q / 3, c = q - xx * 3;
        const int y = wy0 + r, x = wx0 + xx;
        const bool ok = idx < WR * NVROW && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        if constexpr (MODE == 1) raw[k] = raw_buffer_load_u8(rs, ok ? (y * W + x) * 3 + c : OOB, 0, 0);
        else raw[k] = raw_buffer_load_u32(rs, ok ? ((c * H + y) * W + x) * 4 : OOB, 0, 0);
      }
    }
  };
  // normalised window -> LDS N[row][x * 3 + c] (zeros outside the image = the stem's padding)
  auto store_window = [&](int oy0, int ox0) __attribute__((always_inline)) {
    const int wy0 = 2 * oy0 - 4, wx0 = 2 * ox0 - 4;
    T* nimg = reinterpret_cast<T*>(smem + OFF_N);
    const T* lut = reinterpret_cast<const T*>(smem + OFF_LUT);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int idx = opaque(tid) + k * NT;
      if constexpr (MODE == 2) {
        if (idx >= WR * Win<2>::DW) continue;
        const int r = idx / Win<2>::DW, dw = idx - r * Win<2>::DW;
        const bool rok = (unsigned)(wy0 + r) < (unsigned)H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = 4 * dw + j;
          if (q >= NVROW) continue;
          const int xx = q / 3, c = q - xx * 3;
          const bool ok = rok && (unsigned)(wx0 + xx) < (unsigned)W;
          nimg[r * (NPITCH / 2) + q] = ok ? lut[((raw[k] >> (8 * j)) & 0xffu) * 3 + c] : (T)0.0f;
        }
      } else {
        if (idx >= WR * NVROW) continue;
        const int r = idx / NVROW, q = idx - r * NVROW;
        if constexpr (MODE == 1) {
          const int xx = q / 3, c = q - xx * 3;
          const bool ok = (unsigned)(wy0 + r) < (unsigned)H && (unsigned)(wx0 + xx) < (unsigned)W;
          nimg[r * (NPITCH / 2) + q] = ok ? lut[(raw[k] & 0xffu) * 3 + c] : (T)0.0f;
        } else {
          nimg[r * (NPITCH / 2) + q] = (T)__uint_as_float(raw[k]);  // out-of-image loads read 0.0f
        }
      }
    }
  };
  // N -> E for column parity Q: E[r][hx] = the 24 values from window pixel 2 hx - Q + 1 on
  // (7 horizontal taps x 3 channels of stem column 2 ox0 + 2 hx - Q; values 21..23 zero)
  // (part `part` of `nparts`: the entries idx = tid + NT (part + nparts n))
  // Thread t < 5 x 3 NC owns one (pixel hx, part pp) column of E and rows r0 + 5 i (r0 = t / 3 NC):
  // one division per call, and compile-time LDS offsets from two base addresses per row step.
  auto expand = [&](auto qc, int part, int nparts) __attribute__((always_inline)) {
    constexpr int Q = decltype(qc)::value, NC = TW + Q, NU = 3 * NC, RSTEP = NT / NU;
    constexpr int NI = (WR + RSTEP - 1) / RSTEP;
    static_assert(RSTEP == 5 && NI == 8, "5 rows per pass, 8 passes");
    const int t = opaque(tid);
    const int r0 = t / NU, u = t - r0 * NU;
    const int hx = u / 3, pp = u - hx * 3;
    const int boff = r0 * NPITCH + 6 * (2 * hx - Q + 1) + 16 * pp;
    const char* src = smem + OFF_N + (boff & ~3);
    char* dst = smem + OFF_E + (r0 * ECOLS + hx) * EPIX + 16 * pp;
    const unsigned sh = (unsigned)(boff & 3);  // 0 or 2
    const unsigned mz = pp == 2 ? 0xffffu : 0xffffffffu, mw = pp == 2 ? 0u : 0xffffffffu;
    if (r0 < RSTEP) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (i < part * NI / nparts || i >= (part + 1) * NI / nparts) continue;
        if (r0 + RSTEP * i >= WR) continue;
        const unsigned* d = reinterpret_cast<const unsigned*>(src + i * RSTEP * NPITCH);
        unsigned v[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) v[j] = d[j];
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(v[1], v[0], sh);
        o.y = __builtin_amdgcn_alignbyte(v[2], v[1], sh);
        o.z = __builtin_amdgcn_alignbyte(v[3], v[2], sh) & mz;
        o.w = __builtin_amdgcn_alignbyte(v[4], v[3], sh) & mw;
        *reinterpret_cast<uint4*>(dst + i * RSTEP * ECOLS * EPIX) = o;
      }
    }
  };

  // ---- stem weights of one channel block: A-fragments (32 channels x 16 K per k-step), one
  // 16-byte load per k-step per lane (stem_fragment_order; L2-resident), through a buffer resource
  uint4 wst[KS];
  const i32x4 srsrc = rsrc_of(p.stem_w, (unsigned long long)KS * 4 * 1024);
  auto load_stem_w = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KS; ++j) wst[j] = to_u4(raw_buffer_load_v4(srsrc, lane * 16, (j * 4 + cb) * 1024, 0));
  };

  // ---- stem phase: the halo of phase block (P, Q), channel block CB of tile (oy0, ox0) into LDS.
  // Fragment k = 32 consecutive pixels of the (16 + P) x (32 + Q) block (row-major); wave w
  // computes fragments w, w + 8, ... (a single accumulation chain issues back to back,
  // MI355X_MICROARCH.md); lane (l32, lh): pixel l32, K half lh.
  auto stem_phase = [&](auto bc, int oy0, int ox0) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value;
    constexpr int P = blk_p(B), Q = blk_q(B), CB = blk_cb(B);
    constexpr int NC = TW + Q, NPX = (TH + P) * NC, NFR = (NPX + 31) / 32;
    const float* lbs = reinterpret_cast<const float*>(smem + OFF_BS) + CB * 32;
    for (int k = wave; k < NFR; k += NWV) {  // (wave-uniform trip count; the SIMD's two waves interleave)
      int ff = 32 * k + opaque(l32);
      const bool valid = ff < NPX;
      ff = valid ? ff : NPX - 1;
      const int hy = ff / NC, hx = ff - hy * NC;
      const char* e0 = smem + OFF_E + ((2 * hy - P + 1) * ECOLS + hx) * EPIX;
      const char* e16 = e0 + lh * 16;
      const char* erow = e0 + lh * (ECOLS * EPIX - 32);
      auto rd = [&](int j) __attribute__((always_inline)) {
        const int c0 = 2 * j;  // lane half 0's chunk (ky = c0 / 3, part = c0 % 3); half 1 reads c0 + 1
        const int off = (c0 / 3) * ECOLS * EPIX + (c0 % 3) * 16;
        const char* base = j == KS - 1 ? e0 : (c0 % 3 == 2 ? erow : e16);  // (k-step 10's half 1: zero weights)
        return *reinterpret_cast<const uint4*>(base + off);
      };
      // operands RA k-steps ahead through a register ring: left to itself the compiler re-used
      // one register set, one LDS round trip exposed before every MFMA (1.33 -> 1.25-1.27 ms per
      // slice with 2 or 4 ahead; the next fragment's first operands issued before this one's
      // epilogue as well: no further change, profiles/r4l, r4m)
      constexpr int RA = SS2_RD_AHEAD;
      uint4 bq[RA];
#pragma unroll
      for (int j = 0; j < RA; ++j) bq[j] = rd(j);
      f32x16 acc = f32x16{};
#pragma unroll
      for (int j = 0; j < KS; ++j) {
#if TV_SS2_EXP == 1
        acc[j] += __uint_as_float(bq[j % RA].x ^ wst[j].y);
#else
        Mfma<T>::run(wst[j], bq[j % RA], acc);
#endif
        if (j + RA < KS) bq[j % RA] = rd(j + RA);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int sy = 2 * oy0 + 2 * hy - P, sx = 2 * ox0 + 2 * hx - Q;
      const bool in = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
      const unsigned keep = in ? 0xffffffffu : 0u;  // outside the image: conv1's zero padding
      char* hdst = smem + OFF_H + (hy * RS + hx) * PITCH;
      // bias on packed fp32 adds, ReLU, one v_cvt_pk per pair, the image mask on the packed pair
      // (the select before the conversion split every v_cvt_pk into two converts and a pack)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float v[2][4];
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int G2 = 2 * m + gg;
          const f32x4 bb = *reinterpret_cast<const f32x4*>(lbs + 8 * G2 + 4 * lh);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 t = f32x2{acc[4 * G2 + e], acc[4 * G2 + e + 1]} + f32x2{bb[e], bb[e + 1]};
            v[gg][e] = fmaxf(t[0], 0.0f);
            v[gg][e + 1] = fmaxf(t[1], 0.0f);
          }
        }
        const unsigned a0 = pack2<T>(v[0][0], v[0][1]) & keep, a1 = pack2<T>(v[0][2], v[0][3]) & keep;
        const unsigned b0 = pack2<T>(v[1][0], v[1][1]) & keep, b1 = pack2<T>(v[1][2], v[1][3]) & keep;
        const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        if (valid) *reinterpret_cast<uint4*>(hdst + (16 * m + 8 * lh) * sizeof(T)) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
      }
    }
  };

  // ---- conv1: register-staged weight ring (conv3x3s2.hip): k-step q loaded at step q - 5 into
  // set q % 4, written to ring slot q % 3 at step q - 2; [k-step][128 rows][4 x 16 B] (stem_s2_repack)
  int wc_in = 0;
  WReg wreg[4];
  const i32x4 wrsrc = rsrc_of(p.w1, (unsigned long long)SPT * WSLOT);
  const int wvoff = tid * WPL;
  auto w_load = [&](WReg& dst) __attribute__((always_inline)) {
    dst.a = raw_buffer_load_v4(wrsrc, wvoff, wc_in * WSLOT, 0);
    if (++wc_in == SPT) wc_in = 0;
  };
  auto w_store = [&](int slot, const WReg& v) __attribute__((always_inline)) {
    *reinterpret_cast<u32x4*>(smem + OFF_W + slot * WSLOT + wvoff) = v.a;
  };
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  // wave w: tile rows RPW w + f (f = 0..3) x all 128 output channels (fragments i = 0..3)
  const unsigned xa = lds0 + OFF_H + (unsigned)((RPW * wave * RS + l32) * PITCH + lh * 16);
  constexpr int FOFF = RS * PITCH;
  unsigned wa[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) wa[j] = lds0 + OFF_W + (unsigned)(l32 * 64 + (((2 * j + lh) ^ ((l32 >> 2) & 3)) << 4));
  // fragment R of sub-step SJ of k-step j: x[R] for R < RPW, else w[R - RPW]
  auto read_one = [&](auto r, auto sj, auto kj, unsigned xb, unsigned wb, Half& F) __attribute__((always_inline)) {
    constexpr int R = decltype(r)::value, SJ = decltype(sj)::value, KJ = decltype(kj)::value;
    constexpr int TOFF = (J_TY[KJ] * RS + J_TX[KJ]) * PITCH;
    if constexpr (R < RPW) F.x[R] = ds_read16<TOFF + 32 * SJ + R * FOFF>(xb);
    else F.w[R - RPW] = ds_read16<(R - RPW) * 2048>(wb);
  };
  f32x16 acc[RPW][4];
  // the RPW MFMAs of channel fragment I (all pixel fragments)
  auto mfma_col = [&](auto i, auto firstc, const Half& F) __attribute__((always_inline)) {
    constexpr int I = decltype(i)::value;
#pragma unroll
    for (int f = 0; f < RPW; ++f) {
      if constexpr (decltype(firstc)::value) acc[f][I] = f32x16{};
      Mfma<T>::run(to_u4(F.w[I]), to_u4(F.x[f]), acc[f][I]);
    }
  };

  // residual input: the (0, 0) phase block of channel block CB = stem(2 (oy0 + hy), 2 (ox0 + hx))
  // for the tile's 16 x 32 output pixels, LDS -> res (8 chunks of 16 B per thread)
  const unsigned long long res_frame = (unsigned long long)Ho * Wo * p.res_ldc * sizeof(T);
  auto copy_res = [&](auto cbc, int fr, int oy0, int ox0) __attribute__((always_inline)) {
    constexpr int CB = decltype(cbc)::value;
    const i32x4 rs = rsrc_of((const char*)p.res + (size_t)fr * res_frame, res_frame);
#pragma unroll
    for (int k = 0; k < TH * TW * 4 / NT; ++k) {
      const int g = opaque(tid) + k * NT;
      const int px = g >> 2, c4 = g & 3;
      const int hy = px >> 5, hx = px & 31;
      const uint4 v = *reinterpret_cast<const uint4*>(smem + OFF_H + (hy * RS + hx) * PITCH + c4 * 16);
      const int y = oy0 + hy, x = ox0 + hx;
      const bool ok = y < Ho && x < Wo;
      raw_buffer_store_v4(u32x4{v.x, v.y, v.z, v.w}, rs,
                          ok ? (int)(((unsigned)(y * Wo + x) * (unsigned)p.res_ldc + CB * 32 + c4 * 8) * sizeof(T)) : OOB,
                          0, 0);
    }
  };

  Half H0, H1;
  int cur_fr = 0, cur_y0 = 0, cur_x0 = 0, nx_fr = 0, nx_y0 = 0, nx_x0 = 0;
  // one conv1 k-step at schedule position QS of the tile (block SCH.blk, tap j)
  auto step = [&](auto qc) __attribute__((always_inline)) {
    constexpr int QS = decltype(qc)::value;
    constexpr int J = SCH.j[QS], TB = SCH.t[QS], L = SCH.len[QS], BLK = SCH.blk[QS];
    constexpr bool FIRSTK = TB == 0, LASTK = TB == L - 1;
    constexpr int PAR = QS & 3, SLOT = QS % RING;
    constexpr bool FIRST = QS == 0;  // the tile's first products
    static_assert(SPT % 4 == 0 && SPT % RING == 0, "static register set / ring slot per position");
    SS2_STAMP(3);  // (the previous k-step's tail, or the stem phase's when FIRSTK: charged below)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if TV_SS2_EXP == 3
    if constexpr (FIRSTK) __builtin_amdgcn_s_barrier();
#else
    __builtin_amdgcn_s_barrier();  // the block's halo (stem phase) / k-step QS + 1's weights visible
#endif
    __builtin_amdgcn_sched_barrier(0);
    const unsigned wc0 = wa[0] + (unsigned)(SLOT * WSLOT);
    const unsigned wc1 = wa[1] + (unsigned)(SLOT * WSLOT);
    const unsigned wn0 = wa[0] + (unsigned)(((QS + 1) % RING) * WSLOT);
    if constexpr (FIRSTK) {  // the block's first k-step: its sub-step-0 fragments were not read ahead
      auto rd = [&](auto r) __attribute__((always_inline)) { read_one(r, IC<0>{}, IC<J>{}, xa, wc0, H0); };
      unroll<0, RPW + 4>(rd);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    SS2_STAMP(2);
#if TV_C3_EXP == 9
    if (lane == 0) st_b[7] += 1;
#endif
    // first half: sub-step 0 (H0) MFMAs, channel fragment by channel fragment, with sub-step 1's
    // reads (H1) and the ring write issued between them
    mfma_col(IC<0>{}, IC<FIRST>{}, H0);
    read_one(IC<0>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    read_one(IC<1>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<1>{}, IC<FIRST>{}, H0);
    read_one(IC<2>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    read_one(IC<3>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    // k-step QS + 2 (loaded at step QS - 3) into the slot k-step QS - 1 used (read before this barrier)
#if TV_SS2_EXP != 4
    w_store((QS + 2) % RING, wreg[(PAR + 2) & 3]);
#endif
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<2>{}, IC<FIRST>{}, H0);
    read_one(IC<4>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    read_one(IC<5>{}, IC<1>{}, IC<J>{}, xa, wc1, H1);
    if constexpr (blk_p(BLK) == 0 && blk_q(BLK) == 0) copy_res(IC<blk_cb(BLK)>{}, cur_fr, cur_y0, cur_x0);
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<3>{}, IC<FIRST>{}, H0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // H1 landed
    __builtin_amdgcn_sched_barrier(0);
    // second half: sub-step 1 (H1), the next k-step's sub-step-0 reads (within the block) between
    mfma_col(IC<0>{}, IC<false>{}, H1);
#if TV_SS2_EXP != 4
    w_load(wreg[(PAR + 1) & 3]);  // k-step QS + 5 (past the tile's end: the next tile's, same weights)
#endif
    if constexpr (!LASTK) {
      read_one(IC<0>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
      read_one(IC<1>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<1>{}, IC<false>{}, H1);
    if constexpr (!LASTK) {
      read_one(IC<2>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
      read_one(IC<3>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<2>{}, IC<false>{}, H1);
    if constexpr (!LASTK) {
      read_one(IC<4>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
      read_one(IC<5>{}, IC<0>{}, IC<J + 1>{}, xa, wn0, H0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_col(IC<3>{}, IC<false>{}, H1);
    __builtin_amdgcn_sched_barrier(0);
    SS2_STAMP(3);
    // u8 frames (the product path): the tile's serial staging moved under the k-steps, where the
    // SIMD's other wave keeps issuing MFMAs — E for q = 0 under block 7 (E's q = 1 copy was last
    // read by block 7's stem phase, before these k-steps' barriers), the next tile's window into
    // registers at block 8, into N at block 12 (N was last read by the expansion under block 7),
    // the next tile's E for q = 1 under block 15 (E's q = 0 copy was last read by block 15's stem)
    if constexpr (MODE == 2) {
      if constexpr (BLK == 7) expand(IC<0>{}, TB, L);
      if constexpr (BLK == 8 && TB == 0) load_window(nx_fr, nx_y0, nx_x0);
      if constexpr (BLK == 12 && TB == 0) store_window(nx_y0, nx_x0);
      if constexpr (BLK == 15) expand(IC<1>{}, TB, L);
      __builtin_amdgcn_sched_barrier(0);
    }
    SS2_STAMP(4);
  };

  // conv1 epilogue: bias + activation + 16-byte stores (out-of-range pixels: dropped)
  const unsigned long long out_frame = (unsigned long long)Ho * Wo * p.out_ldc * sizeof(T);
  auto epilogue = [&](int fr, int oy0, int ox0) __attribute__((always_inline)) {
    const float* lb1 = reinterpret_cast<const float*>(smem + OFF_B1);
    const i32x4 ors = rsrc_of((const char*)p.out + (size_t)fr * out_frame, out_frame);
#pragma unroll
    for (int f = 0; f < RPW; ++f) {
      const int y = oy0 + RPW * wave + f, x = ox0 + l32;
      const bool ok = y < Ho && x < Wo;
      const int obase = ok ? (int)(((unsigned)(y * Wo + x) * (unsigned)p.out_ldc + 8 * lh) * sizeof(T)) : OOB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float v[2][4];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int G2 = 2 * m + gg;
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lb1 + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[gg][e] = fmaxf(acc[f][i][4 * G2 + e] + bb[e], 0.0f);
          }
          const unsigned a0 = pack2<T>(v[0][0], v[0][1]), a1 = pack2<T>(v[0][2], v[0][3]);
          const unsigned b0 = pack2<T>(v[1][0], v[1][1]), b1 = pack2<T>(v[1][2], v[1][3]);
          const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
          raw_buffer_store_v4(u32x4{r0[0], r1[0], r0[1], r1[1]}, ors,
                              ok ? obase + (int)((32 * i + 16 * m) * sizeof(T)) : OOB, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };

  // ---- prologue: tile 0's window, channel block 0's stem weights, conv1 weights of k-steps 0..4
  tile_of(0, cur_fr, cur_y0, cur_x0);
  if constexpr (MODE == 2) load_window(cur_fr, cur_y0, cur_x0);  // (stored after the barrier below)
  load_stem_w(0);
  w_load(wreg[0]);
  w_load(wreg[1]);
  w_store(0, wreg[0]);
  w_store(1, wreg[1]);
  w_load(wreg[2]);
  w_load(wreg[3]);
  w_load(wreg[0]);
  __syncthreads();  // LUT, biases, ring slots 0 and 1

  // one block: [barrier] stem phase [stem weights of the next channel block] k-steps
  auto block = [&](auto bc) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value;
    SS2_STAMP(6);
    lds_barrier();  // the previous block's k-steps have read the halo
    SS2_STAMP(0);
    stem_phase(IC<B>{}, cur_y0, cur_x0);
    if constexpr (blk_p(B) == 1) load_stem_w(blk_cb((B + 1) % NBLK));  // lands under this block's k-steps
    SS2_STAMP(1);
    auto ks = [&](auto t) __attribute__((always_inline)) {
      constexpr int T_ = decltype(t)::value;
      step(IC<SCH.first[B] + T_>{});
    };
    unroll<0, pb_len(blk_p(B), blk_q(B))>(ks);
  };
  if constexpr (MODE == 2) {  // the first tile's N and E (later tiles': under the previous tile)
    store_window(cur_y0, cur_x0);
    lds_barrier();
    expand(IC<1>{}, 0, 1);
  }
  for (int tl = 0; tl < ntl; ++tl) {
    tile_of(tl + 1, nx_fr, nx_y0, nx_x0);  // (past the list: this tile again)
    if constexpr (MODE != 2) {
      load_window(cur_fr, cur_y0, cur_x0);
      store_window(cur_y0, cur_x0);  // N was last read by expand<0> in the previous tile
      lds_barrier();
      expand(IC<1>{}, 0, 1);         // E was last read by block 15's stem phase
    }
    unroll<0, 8>(block);
    if constexpr (MODE != 2) expand(IC<0>{}, 0, 1);  // E's q = 1 copy was last read by block 7's stem phase
    auto blk2 = [&](auto bc) __attribute__((always_inline)) { block(IC<8 + decltype(bc)::value>{}); };
    unroll<0, 8>(blk2);
    SS2_STAMP(6);
    epilogue(cur_fr, cur_y0, cur_x0);
    SS2_STAMP(5);
    cur_fr = nx_fr;
    cur_y0 = nx_y0;
    cur_x0 = nx_x0;
    lds_barrier();  // block 15's k-steps are done with the halo / E before the next tile's writes
  }
#if TV_C3_EXP == 9
  SS2_STAMP(6);
  if (p.dbg && lane == 0) {
    unsigned long long* d = p.dbg + ((size_t)blockIdx.x * NWV + wave) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = st_b[k];  // (< 2^32 cycles per wave and bucket)
  }
#endif
}

// [Npad][Kpad] conv1 weights (K = tap * 128 + channel) -> [k-step s][128 rows][4 x 16 B] in this
// kernel's schedule, slot c of row r holding chunk c ^ ((r >> 2) & 3)
__global__ void repack_weights(const uint4* __restrict__ w, int kpad16, uint4* __restrict__ out) {
  const int n = SPT * BN * 4;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const int slot = o & 3, row = (o >> 2) & (BN - 1), s = o >> 9;
    const int chunk = slot ^ ((row >> 2) & 3);
    const int cb = blk_cb(SCH.blk[s]), j = SCH.j[s];
    out[o] = w[(size_t)row * kpad16 + (J_TAP[j] * 128 + cb * 32) / 8 + chunk];
  }
}

template <typename T, int MODE>
static int launch_t(const StemS2Params& p, int grid, hipStream_t s) {
  auto k = stem_s2<T, MODE>;
  constexpr int lds = LDS + (TV_C3_EXP == 9 ? NWV * 8 * 4 : 0);  // (the stamp build's buckets)
  if (int r = ensure_lds<stem_s2<T, MODE>>(lds)) return r;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace ss2

int stem_s2_tiles(int B, int Ho, int Wo) {
  return B * ((Ho + ss2::TH - 1) / ss2::TH) * ((Wo + ss2::TW - 1) / ss2::TW);
}

size_t stem_s2_weight_bytes() { return (size_t)ss2::SPT * ss2::WSLOT; }

int stem_s2_repack(const void* w, int Kpad, int esz, void* out, hipStream_t s) {
  if ((Kpad * esz) % 16 || Kpad < 9 * 128) {
    set_error("stem_s2_repack: bad Kpad");
    return 1;
  }
  hipLaunchKernelGGL(ss2::repack_weights, dim3(64), dim3(256), 0, s, (const uint4*)w, Kpad * esz / 16, (uint4*)out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_stem_s2(const StemS2Params& p, int dtype, int cu_count, hipStream_t s) {
  using namespace ss2;
  const long tiles = (long)stem_s2_tiles(p.B, p.Ho, p.Wo);
  const unsigned long long in_frame = p.u8 ? (unsigned long long)p.H * p.W * 3 : (unsigned long long)12 * p.H * p.W;
  if (p.B < 1 || p.H < 1 || p.W < 1 || p.Ho != (p.H + 1) / 2 || p.Wo != (p.W + 1) / 2 || p.out_ldc % 8 ||
      p.res_ldc % 8 || p.out_ldc < BN || p.res_ldc < BN || in_frame >= (1ull << 31) ||
      (unsigned long long)p.Ho * p.Wo * p.out_ldc * 2 >= (1ull << 31) ||
      (unsigned long long)p.Ho * p.Wo * p.res_ldc * 2 >= (1ull << 31) || !p.input || !p.out || !p.res) {
    set_error("stem_s2: unsupported geometry");
    return 1;
  }
  int grid = (int)std::min<long>(tiles, cu_count);
  if (grid >= 8 && tiles > 2L * grid) grid -= grid % 8;
  const int mode = p.u8 ? (p.W % 4 == 0 ? 2 : 1) : 0;
  using L = int (*)(const StemS2Params&, int, hipStream_t);
  static const L f16[3] = {launch_t<_Float16, 0>, launch_t<_Float16, 1>, launch_t<_Float16, 2>};
  static const L b16[3] = {launch_t<__bf16, 0>, launch_t<__bf16, 1>, launch_t<__bf16, 2>};
  if (dtype == F16) return f16[mode](p, grid, s);
  if (dtype == BF16) return b16[mode](p, grid, s);
  set_error("stem_s2: fp16/bf16 only");
  return 1;
}

}  // namespace tv
