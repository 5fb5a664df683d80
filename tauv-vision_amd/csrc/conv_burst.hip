// One-shot small-level convolution (gfx950, fp16 / bf16): the deep DLA levels (dla.py:79-135
// Trees, their Roots dla.py:58-76, the IDAUp projections / outputs dla.py:212-284 at those levels)
// and, at B = 1, everything from 60x80 down.
//
// These layers are latency-bound: a 15x20 level of a 32-frame slice or a 60x80 level of one frame
// is a few MFLOP per CU. conv_lat.hip walks each tile's K loop as a chain of LDS-DMA stages (2 in
// flight per K group, ~1.3 us per 64-deep k-step) and, split over workgroups, hands fp32 partial
// tiles through a ticket: measured 15-18 us per launch whatever the layer's size.
//
// Here a workgroup's whole operand set is requested at once and waited for once:
//  * a workgroup owns 64 consecutive output pixels of one frame (raster order: any width) x 32
//    output channels; its 4 waves split K in four (<= 20 k-steps of 16 each, K <= 1280);
//  * each wave's weight fragments for its whole K quarter go straight from L2 into registers (one
//    16-byte load per lane per k-step from a pre-packed [32-channel tile][k-step][lane] copy:
//    1 KiB coalesced per wave-instruction, no LDS, no barrier);
//  * the input the tile reads moves into LDS once by LDS-DMA: for a 3x3 / stride 1 segment the
//    output rows' window (rows y-1 .. y+1 at full width + the zero padding columns), for a 1x1
//    segment (Root children, the ResidualBlock's conv_residual at stride 1 or 2) the tile's 64
//    pixels; 272-byte pixel pitch per 128-channel plane (raster fragments: conflict-free
//    ds_read_b128 except at a row wrap), out-of-image taps and the pad slot are buffer-OOB zeros;
//  * one vmcnt(0) + barrier, then per k-step two ds_read_b128 (the lane's pixel, shifted by the
//    tap) and two v_mfma_f32_32x32x16; the four K quarters' fp32 partial tiles are summed through
//    LDS in wave order (deterministic), + bias, activation, 16-byte stores.
// Several independent layers of one dependency level run in one launch (the engine's schedule).
#include "conv_common.h"

#include <algorithm>
#include <type_traits>

namespace tv {
namespace burst {

constexpr int NT = 256, NW = 4, PX = 64, NCH = 32;
constexpr int PP = 272;                 // LDS bytes per staged pixel per 128-channel plane
constexpr int SLOTS = PP / 16;          // 16 data chunks + 1 pad slot (OOB zeros)
constexpr int SR = 36;                  // partial-tile row pitch (floats)
constexpr int PART = PX * SR * 4;       // one wave's partial tile
constexpr int ZERO_BYTES = 256;         // LDS zeros: A operand of the padding k-steps
constexpr int LDS_MAX = 160 * 1024;
constexpr int OOB = (int)0x80000000u;

typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
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
// an LDS read the compiler tracks (it places the lgkmcnt waits before the MFMAs that consume it)
typedef const __attribute__((address_space(3))) u32x4 lds_u32x4;
__device__ __forceinline__ u32x4 ds_read16(unsigned addr) { return *reinterpret_cast<lds_u32x4*>(addr); }
__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}

// one workgroup's tile of layer p (bid: its index within the layer)
template <typename T, int KPW>
__device__ __forceinline__ void burst_tile(const BurstParams& p, const int bid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;

  // XCD-aware order: contiguous runs of (pixel tile, channel tile) per XCD, the channel tiles of a
  // pixel tile adjacent (they stage the same input window: L2 hits)
  const int nbk = p.ptiles * p.ntiles;
  const int q8 = nbk >> 3, r8 = nbk & 7, xcd = bid & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int nt = lin % p.ntiles, pt = lin / p.ntiles;
  const int fr = pt / p.tiles_pf;
  const int hw = p.Ho * p.Wo;
  const int r0 = (pt - fr * p.tiles_pf) * PX;        // first output pixel (raster, within the frame)
  const int npx = min(PX, hw - r0);                  // valid pixels of the tile
  const int y_first = r0 / p.Wo;
  const int wy0 = y_first - 1;                       // first window row of a 3x3 segment
  const int n0 = nt * NCH;

  // ---- bias (this thread's 8 output channels) and the weights of this wave's K quarter
  const int c8 = (tid & 3) * 8;
  const bool nok = n0 + c8 < p.N;
  // (every global access of the kernel is a bounds-checked buffer operation: an out-of-range lane
  // reads zeros / drops its store instead of faulting)
  const i32x4 brs = rsrc_of(p.bias, (unsigned)p.N * 4u);
  const int boff = nok ? (n0 + c8) * 4 : OOB;
  const f32x4 b0 = __builtin_bit_cast(f32x4, raw_buffer_load_v4(brs, boff, 0, 0));
  const f32x4 b1 = __builtin_bit_cast(f32x4, raw_buffer_load_v4(brs, boff + 16, 0, 0));
  const int nk = p.nk16;
  const int kq0 = wave * ((nk + NW - 1) / NW);
  const int nkw = max(0, min(KPW, nk - kq0));       // this wave's k-steps (wave-uniform)
  u32x4 wreg[KPW];
  {
    const i32x4 wr = rsrc_of(p.w, (unsigned)(p.ntiles * nk * 64 * 16));
    const int wbase = ((nt * nk + kq0) * 64 + lane) * 16;
#pragma unroll
    for (int i = 0; i < KPW; ++i) wreg[i] = raw_buffer_load_v4(wr, i < nkw ? wbase + i * 1024 : OOB, 0, 0);
  }

  // ---- stage every segment's input into LDS (LDS-DMA pieces of 1 KiB, round-robin over waves)
  for (int s = 0; s < p.nseg; ++s) {
    const BurstSeg& sg = p.seg[s];
    const unsigned fbytes = (unsigned)sg.H * sg.W * sg.ldc * (unsigned)sizeof(T);
    const i32x4 rs = rsrc_of(reinterpret_cast<const char*>(sg.src) + (size_t)fr * fbytes, fbytes);
    const int npix = sg.npix;                          // staged pixels per plane
    const int per_plane = npix * SLOTS;
    const int chunks = sg.planes * per_plane;
    const float inv_row = sg.kind == 0 ? 1.0f / (float)sg.wrow : 0.f;
    for (int q = wave; q * 64 < chunks; q += NW) {
      const int g = q * 64 + lane;
      const int plane = g / per_plane;
      const int rem = g - plane * per_plane;
      const int pix = rem / SLOTS, slot = rem - pix * SLOTS;
      int y, x;
      if (sg.kind == 0) {                              // window pixel (row, column) -> (y, x)
        const int ry = (int)(((float)pix + 0.5f) * inv_row);
        y = wy0 + ry;
        x = pix - ry * sg.wrow - 1;
      } else {                                         // the tile's pixel pix at the segment's stride
        const int r = r0 + pix;
        const int yo = r / p.Wo;
        y = (r < hw && pix < PX) ? yo * sg.stride : -1;
        x = (r - yo * p.Wo) * sg.stride;
      }
      const bool ok = g < chunks && slot < 16 && (unsigned)y < (unsigned)sg.H && (unsigned)x < (unsigned)sg.W;
      const int off = ok ? (int)((((unsigned)y * sg.W + x) * sg.ldc + plane * 128 + slot * 8) * sizeof(T)) : OOB;
      raw_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(smem + sg.lds_off + q * 1024), 16, off, 0, 0, 0);
    }
  }
  if (tid < ZERO_BYTES / 16) *reinterpret_cast<uint4*>(smem + p.zero_off + tid * 16) = make_uint4(0u, 0u, 0u, 0u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- the lane's pixel in each segment's staging (fragment f: tile pixel 32 f + l32; pixels past
  // the tile's end read pixel 0: their results are never stored)
  unsigned abase[kBurstMaxSeg][2];
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
#pragma unroll
  for (int s = 0; s < kBurstMaxSeg; ++s) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int pp = 32 * f + l32;
      const int pq = pp < npx ? pp : 0;
      unsigned pos = (unsigned)pq;
      if (s < p.nseg && p.seg[s].kind == 0) {
        const int r = r0 + pq;
        const int y = r / p.Wo, x = r - y * p.Wo;
        pos = (unsigned)((y - y_first) * p.seg[s].wrow + x);  // tap (0, 0): input (y - 1, x - 1) = window (y - 1 - wy0, x)
      }
      abase[s][f] = lds0 + (s < p.nseg ? (unsigned)p.seg[s].lds_off : 0u) + pos * PP + (unsigned)lh * 16;
    }
  }
  const unsigned zaddr = lds0 + (unsigned)p.zero_off + (unsigned)lh * 16;

  // ---- this wave's k-steps: (segment, tap, 16-channel block) -> LDS offset from the lane base
  f32x16 acc0 = f32x16{}, acc1 = f32x16{};
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int j = kq0 + i;
    const bool live = i < nkw;
    int s = 0;
#pragma unroll
    for (int t = 1; t < kBurstMaxSeg; ++t)
      if (t < p.nseg && j >= p.seg[t].kbase16) s = t;
    const BurstSeg& sg = p.seg[s];
    const int kk = j - sg.kbase16;
    const int cpt = sg.C >> 4;                        // 16-channel blocks per tap
    const int tap = kk / cpt, c16 = kk - tap * cpt;
    int off = (c16 >> 3) * sg.npix * PP + (c16 & 7) * 32;
    if (sg.kind == 0) off += ((tap / 3) * sg.wrow + tap % 3) * PP;
    unsigned a0 = 0, a1 = 0;
    // (the segment index is wave-uniform: select its two lane bases)
#pragma unroll
    for (int t = 0; t < kBurstMaxSeg; ++t)
      if (t == s) a0 = abase[t][0], a1 = abase[t][1];
    const u32x4 x0 = ds_read16(live ? a0 + off : zaddr);
    const u32x4 x1 = ds_read16(live ? a1 + off : zaddr);
    Mfma<T>::run(to_u4(wreg[i]), to_u4(x0), acc0);
    Mfma<T>::run(to_u4(wreg[i]), to_u4(x1), acc1);
  }

  // ---- the four K quarters' partial tiles, summed in wave order (LDS aliases the staging: barrier)
  __syncthreads();
  float* part = reinterpret_cast<float*>(smem) + wave * (PART / 4);
  // acc element 4g + e: channel 8g + 4lh + e of pixel l32 (+ 32 for acc1)
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    *reinterpret_cast<f32x4*>(part + l32 * SR + 8 * g + 4 * lh) =
        f32x4{acc0[4 * g], acc0[4 * g + 1], acc0[4 * g + 2], acc0[4 * g + 3]};
    *reinterpret_cast<f32x4*>(part + (32 + l32) * SR + 8 * g + 4 * lh) =
        f32x4{acc1[4 * g], acc1[4 * g + 1], acc1[4 * g + 2], acc1[4 * g + 3]};
  }
  __syncthreads();
  const int px = tid >> 2;
  if (px >= npx || !nok) return;
  const float* rd = reinterpret_cast<const float*>(smem) + px * SR + c8;
  f32x4 s0 = *reinterpret_cast<const f32x4*>(rd), s1 = *reinterpret_cast<const f32x4*>(rd + 4);
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    s0 += *reinterpret_cast<const f32x4*>(rd + w * (PART / 4));
    s1 += *reinterpret_cast<const f32x4*>(rd + w * (PART / 4) + 4);
  }
  float v[8] = {s0[0] + b0[0], s0[1] + b0[1], s0[2] + b0[2], s0[3] + b0[3],
                s1[0] + b1[0], s1[1] + b1[1], s1[2] + b1[2], s1[3] + b1[3]};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (p.act == 1) v[e] = fmaxf(v[e], 0.0f);
    else if (p.act == 2) v[e] = v[e] >= 0.0f ? v[e] : 0.01f * v[e];
  }
  const unsigned fbytes = (unsigned)hw * p.out_ldc * (unsigned)sizeof(T);
  const i32x4 ors = rsrc_of(reinterpret_cast<const char*>(p.out) + (size_t)fr * fbytes, fbytes);
  u32x4 o;
  o.x = pack2<T>(v[0], v[1]);
  o.y = pack2<T>(v[2], v[3]);
  o.z = pack2<T>(v[4], v[5]);
  o.w = pack2<T>(v[6], v[7]);
  raw_buffer_store_v4(o, ors, (int)(((unsigned)(r0 + px) * p.out_ldc + p.out_coff + n0 + c8) * sizeof(T)), 0, 0);
}

template <typename T, int KPW>
__global__ __launch_bounds__(NT) void conv_burst(const BurstGroup g) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < g.n && b >= g.end[k]) ++k;  // (workgroup-uniform)
  burst_tile<T, KPW>(g.p[k], b - (k ? g.end[k - 1] : 0));
}

template <typename T, int KPW>
static int launch_t(const BurstGroup& g, int lds, hipStream_t s) {
  if (int r = ensure_lds<conv_burst<T, KPW>>(LDS_MAX)) return r;
  hipLaunchKernelGGL((conv_burst<T, KPW>), dim3(g.end[g.n - 1]), dim3(NT), lds, s, g);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T>
static int launch_k(const BurstGroup& g, int kpw, int lds, hipStream_t s) {
  switch (kpw) {
    case 4: return launch_t<T, 4>(g, lds, s);
    case 6: return launch_t<T, 6>(g, lds, s);
    case 8: return launch_t<T, 8>(g, lds, s);
    case 12: return launch_t<T, 12>(g, lds, s);
    case 18: return launch_t<T, 18>(g, lds, s);
    default: return launch_t<T, 20>(g, lds, s);
  }
}

}  // namespace burst

// the register-resident weight k-steps per wave of a layer (a compiled instance size)
static int burst_kpw(int nk16) {
  const int q = (nk16 + burst::NW - 1) / burst::NW;
  for (int v : {4, 6, 8, 12, 18, 20})
    if (q <= v) return v;
  return 0;
}

// The exclusive end of every LDS byte burst_tile() touches for layer p, over every tile position of a
// frame (the kernel's own index arithmetic, restated next to it so the two cannot drift apart), or -1
// when a tap would read a window pixel the staging did not write (the read stays inside the LDS but
// returns another segment's / plane's bytes). Round 5: B = 2, 15x20, one 128-channel 3x3 segment
// faulted ("an illegal memory access", then NaN outputs once the fault was masked) while the kernel
// was being written; an LDS address past the launch's dynamic allocation faults on gfx950.
// conv_burst_plan() refuses a layer whose extent exceeds p.lds, and every launch re-checks it.
int conv_burst_lds_extent(const BurstParams& p) {
  using namespace burst;
  const int hw = p.Ho * p.Wo;
  int end = p.zero_off + ZERO_BYTES;                  // the zero block (written by 16 threads)
  end = std::max(end, NW * PART);                     // the partial tiles (alias the staging)
  for (int s = 0; s < p.nseg; ++s) {
    const BurstSeg& sg = p.seg[s];
    const int per_plane = sg.npix * SLOTS;
    const int chunks = sg.planes * per_plane;
    const int pieces = (chunks + 63) / 64;            // staging: piece q covers [q KiB, q KiB + 1 KiB)
    if (s + 1 < p.nseg && sg.lds_off + pieces * 1024 > p.seg[s + 1].lds_off) return -1;
    if (s + 1 == p.nseg && sg.lds_off + pieces * 1024 > p.zero_off) return -1;
    end = std::max(end, sg.lds_off + pieces * 1024);
    if (sg.kind == 0) {                               // window row of a staged pixel: the kernel's float form
      const float inv_row = 1.0f / (float)sg.wrow;
      for (int pix = 0; pix < sg.npix; ++pix)
        if ((int)(((float)pix + 0.5f) * inv_row) != pix / sg.wrow) return -1;
    }
    const int nk = (sg.kind == 0 ? 9 : 1) * sg.C / 16;
    const int cpt = sg.C >> 4;
    for (int t = 0; t < p.tiles_pf; ++t) {
      const int r0 = t * PX, npx = std::min(PX, hw - r0), y_first = r0 / p.Wo;
      for (int pp = 0; pp < PX; ++pp) {
        const int pq = pp < npx ? pp : 0;
        int pos = pq;
        if (sg.kind == 0) {
          const int r = r0 + pq, y = r / p.Wo, x = r - y * p.Wo;
          pos = (y - y_first) * sg.wrow + x;
        }
        for (int kk = 0; kk < nk; ++kk) {
          const int tap = kk / cpt, c16 = kk - tap * cpt;
          const int tpos = sg.kind == 0 ? pos + (tap / 3) * sg.wrow + tap % 3 : pos;
          if (tpos >= sg.npix || (c16 >> 3) >= sg.planes) return -1;
          const int off = (c16 >> 3) * sg.npix * PP + (c16 & 7) * 32;
          end = std::max(end, sg.lds_off + tpos * PP + off + 16 + 16);  // ds_read_b128 of lane half lh = 1
        }
      }
    }
  }
  return end;
}

bool conv_burst_plan(const ConvParams& cp, int B, BurstParams* out) {
  using namespace burst;
  BurstParams p{};
  if (cp.nseg < 1 || cp.nseg > kBurstMaxSeg || cp.up_s || cp.N < 8 || cp.N % 8 || cp.out_ldc % 8 || cp.out_coff % 8 ||
      !cp.out || cp.Ho < 1 || cp.Wo < 1)
    return false;
  p.nseg = cp.nseg;
  p.B = B;
  p.Ho = cp.Ho;
  p.Wo = cp.Wo;
  const int hw = cp.Ho * cp.Wo;
  p.tiles_pf = (hw + PX - 1) / PX;
  p.ptiles = p.tiles_pf * B;
  p.ntiles = (cp.N + NCH - 1) / NCH;
  // rows a 64-pixel raster run can touch: ceil(64 / Wo) + 1
  const int out_rows = std::min(cp.Ho, (PX + cp.Wo - 1) / cp.Wo + 1);
  int k16 = 0, off = 0;
  for (int s = 0; s < cp.nseg; ++s) {
    const ConvSegment& g = cp.seg[s];
    BurstSeg& b = p.seg[s];
    if (g.C % 128 || g.ldc % 8 || (size_t)g.H * g.W * g.ldc * 2 >= (1ull << 31)) return false;
    b.src = g.src;
    b.H = g.H;
    b.W = g.W;
    b.C = g.C;
    b.ldc = g.ldc;
    b.planes = g.C / 128;
    b.kbase16 = k16;
    if (g.kh == 3 && g.kw == 3 && g.stride == 1 && g.pad == 1 && g.pad_w == 1 && g.H == cp.Ho && g.W == cp.Wo) {
      b.kind = 0;
      b.stride = 1;
      b.wrow = cp.Wo + 2;
      b.npix = (out_rows + 2) * b.wrow;
      k16 += 9 * g.C / 16;
    } else if (g.kh == 1 && g.kw == 1 && g.pad == 0 && (g.pad_w == 0 || g.pad_w < 0) && g.stride >= 1 &&
               g.H >= (cp.Ho - 1) * g.stride + 1 && g.W >= (cp.Wo - 1) * g.stride + 1) {
      b.kind = 1;
      b.stride = g.stride;
      b.wrow = 0;
      b.npix = PX;
      k16 += g.C / 16;
    } else {
      return false;
    }
    // the segment's k-steps must be where the engine's [Npad][Kpad] packing put them
    if (g.kbase * 64 != b.kbase16 * 16) return false;
    b.lds_off = off;
    const int chunks = b.planes * b.npix * SLOTS;
    off += (chunks + 63) / 64 * 1024;
  }
  p.nk16 = k16;
  if (!burst_kpw(k16) || k16 * 16 != cp.Kpad) return false;
  p.zero_off = off;
  off += ZERO_BYTES;
  p.lds = std::max(off, NW * PART);
  if (p.lds > LDS_MAX) return false;
  p.lds_end = conv_burst_lds_extent(p);
  if (p.lds_end < 0 || p.lds_end > p.lds) return false;
  p.bias = cp.bias;
  p.act = cp.act;
  p.out = cp.out;
  p.out_ldc = cp.out_ldc;
  p.out_coff = cp.out_coff;
  p.N = cp.N;
  *out = p;
  return true;
}

size_t conv_burst_weight_bytes(const BurstParams& p) { return (size_t)p.ntiles * p.nk16 * 64 * 16; }

// [Npad][Kpad] (K = the engine's segment / tap / channel order) -> [32-channel tile][k-step of 16][lane][8]:
// lane (l32, lh) of k-step j holds W[32 nt + l32][16 j + 8 lh .. + 8] (the MFMA A fragment)
__global__ void burst_repack(const uint4* __restrict__ w, long n_in, int kpad16, int ntiles, int nk16,
                             uint4* __restrict__ out) {
  const long n = (long)ntiles * nk16 * 64;
  for (long o = (long)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (long)gridDim.x * blockDim.x) {
    const int lane = (int)(o & 63);
    const long t = o >> 6;
    const int j = (int)(t % nk16), nt = (int)(t / nk16);
    const int row = nt * 32 + (lane & 31);
    const long src = (long)row * kpad16 + 2 * j + (lane >> 5);
    out[o] = src < n_in ? w[src] : make_uint4(0u, 0u, 0u, 0u);
  }
}

int conv_burst_repack(const void* w, int Kpad, int esz, const BurstParams& p, void* out, hipStream_t s) {
  if ((Kpad * esz) % 16 || p.nk16 * 16 != Kpad || esz != 2) {
    set_error("conv_burst_repack: bad Kpad");
    return 1;
  }
  // (the [Npad][Kpad] source holds Npad = 128-row multiples >= 32 * ntiles rows)
  const long n_in = (long)((p.ntiles * 32 + 127) / 128 * 128) * (Kpad * esz / 16);
  hipLaunchKernelGGL(burst_repack, dim3(64), dim3(256), 0, s, (const uint4*)w, n_in, Kpad * esz / 16, p.ntiles,
                     p.nk16, (uint4*)out);
  TV_HIP(hipGetLastError());
  return 0;
}

int conv_burst_workgroups(const BurstParams& p) { return p.ptiles * p.ntiles; }

int launch_conv_burst(const BurstParams* const* ps, int n, int dtype, hipStream_t s) {
  using namespace burst;
  if (n < 1 || n > kBurstGroupMax) {
    set_error("conv_burst: 1..kBurstGroupMax layers");
    return 1;
  }
  BurstGroup g{};
  g.n = n;
  int wg = 0, lds = 0, kpw = 0;
  for (int k = 0; k < n; ++k) {
    const BurstParams& p = *ps[k];
    if (!p.w || !p.out || p.nseg < 1 || p.lds > LDS_MAX || !burst_kpw(p.nk16) || p.lds_end <= 0 || p.lds_end > p.lds) {
      set_error("conv_burst: inconsistent layer");
      return 1;
    }
    g.p[k] = p;
    wg += conv_burst_workgroups(p);
    g.end[k] = wg;
    lds = std::max(lds, p.lds);
    kpw = std::max(kpw, burst_kpw(p.nk16));
  }
  if (dtype == F16) return burst::launch_k<_Float16>(g, kpw, lds, s);
  if (dtype == BF16) return burst::launch_k<__bf16>(g, kpw, lds, s);
  set_error("conv_burst: fp16/bf16 only");
  return 1;
}

}  // namespace tv
