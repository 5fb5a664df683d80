// Split-K implicit GEMM for the small pyramid levels (gfx950, fp16 / bf16 / fp32).
//
// The deep DLA levels (dla.py:79-135 Trees at 30x40 .. 4x5 for a 640x480 frame, their Roots,
// the IDAUp projections at those levels; centerpoint_dla.py's 256/512-channel levels 4-5) hold a
// few thousand output pixels per 32-frame slice. The halo kernels tile 512 pixels x 128 channels
// per workgroup and walk the whole K = 9 C loop (18-72 k-steps) in that one workgroup, so such a
// layer is a handful of tiles on 256 CUs and costs ~20 us whatever its size: one tile's K-loop
// latency.
//
// Here a workgroup owns a 64-pixel x 128-channel tile and its 8 waves form two K groups of 4
// waves: group g walks the k-step descriptors [g * ceil(nks/2), ...) of the layer (the same KStep
// table conv_pipe.hip uses — any mix of 3x3 / 1x1 / strided segments, Root's concatenated
// children, ResidualBlock's fused 1x1 residual, BasicBlock's identity residual), each wave a
// 32 x 64 sub-tile. Per group a 3-slot LDS ring of 24 KiB stages (64 pixel rows + 128 weight rows
// x 128 B, filled by LDS-DMA with the XOR swizzle on the source address, padding taps from a
// zero page), one s_barrier per k-step with counted vmcnt, fragments read one k-step ahead — the
// conv_pipe discipline with half the K loop per workgroup. The two groups' partial tiles are summed
// through LDS in a fixed order (deterministic), then bias + activation + 16-byte NHWC stores.
#include "conv_common.h"

namespace tv {
namespace lat {

constexpr int NT = 512, PX = 64, CH = 128, S = 3;
constexpr int ROWB = 128;                    // bytes of K per k-step per row
constexpr int A_BYTES = PX * ROWB;           // 8 KiB
constexpr int B_BYTES = CH * ROWB;           // 16 KiB
constexpr int STAGE = A_BYTES + B_BYTES;     // 24 KiB
constexpr int GRP_RING = S * STAGE;          // 72 KiB per K group
constexpr int LDS = 2 * GRP_RING;            // 144 KiB
constexpr int GA = PX / 8 / 4;               // A pieces (1 KiB) per wave per k-step = 2
constexpr int GB = CH / 8 / 4;               // B pieces per wave per k-step = 4
constexpr int G = GA + GB;                   // LDS-DMA instructions per wave per k-step
constexpr int SR = CH + 4;                   // staged fp32 row (floats)
static_assert(PX * SR * 4 <= LDS - 16, "reduction tile fits the ring (below the split-K ticket word)");

typedef __attribute__((address_space(3))) char lds_char;
typedef const __attribute__((address_space(1))) void gvoid;
typedef const __attribute__((address_space(4))) u32x4 c_u32x4;

__device__ __forceinline__ void dma16(const void* src, lds_char* dst_wave_base) {
  __builtin_amdgcn_global_load_lds((gvoid*)src, (__attribute__((address_space(3))) void*)dst_wave_base, 16, 0, 0);
}
__device__ __forceinline__ u32x4 ds_read16(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;  // global (never flat) agent-scope ticket words
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");

// one workgroup's tile (or split-K slice of a tile) of the layer *pp; bid = its index in the layer
template <typename T, bool X3 = false>  // X3: fp32 operands, products as three fp16 MFMAs (conv_pipe.hip X3)
__device__ __forceinline__ void conv_lat_tile(const ConvParams* __restrict__ pp, const int bid) {
  const ConvParams& p = *pp;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = ROWB / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;   // K group
  const int wq = wave & 3;     // wave within the group: (wp, wc) = 32-pixel half x 64-channel half
  const int wp = wq & 1, wc = wq >> 1;

  // XCD-aware order: contiguous runs of the linear tile index per XCD, the channel tiles of a
  // pixel tile adjacent (they read the same input pixels)
  // (split-K: the ksplit slices of a tile adjacent too, so they tend to share an XCD — speed only)
  const int ksplit = p.ksplit > 1 ? p.ksplit : 1;
  const int nbk = p.mtiles * p.ntiles * ksplit;
  const int q8 = nbk >> 3, r8 = nbk & 7, xcd = bid & 7;
  const int lin_s = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int lin = lin_s / ksplit;      // tile
  const int slice = lin_s - lin * ksplit;
  const int ntile = lin % p.ntiles;
  const int mtile = lin / p.ntiles;
  const int m0 = mtile * PX;
  const int n0 = ntile * CH;

  // K range of this slice, then of this group
  const int ks0 = (int)((long)p.nks * slice / ksplit), ks1 = (int)((long)p.nks * (slice + 1) / ksplit);
  const int half = (ks1 - ks0 + 1) >> 1;
  const int kbeg = ks0 + grp * half;
  const int nk = grp ? (ks1 - ks0) - half : half;  // wave-uniform; group 1 may have one step fewer

  // ---- DMA geometry: A piece i of this wave covers tile rows (wq*GA + i)*8 + lane/8; the lane's
  // LDS chunk is lane%8 and it fetches source chunk (lane%8) ^ ((row>>1)&7) of that row
  int pb[GA], poy[GA], pox[GA], pc[GA];
  bool pv[GA];
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = (wq * GA + i) * 8 + (lane >> 3);
    const int m = m0 + row;
    pv[i] = m < p.M;
    const int mm = pv[i] ? m : 0;
    pb[i] = mm / hw;
    const int rem = mm - pb[i] * hw;
    poy[i] = rem / p.Wo;
    pox[i] = rem - poy[i] * p.Wo;
    pc[i] = (lane & 7) ^ ((row >> 1) & 7);
  }
  const T* wbase = reinterpret_cast<const T*>(p.weight) + (size_t)n0 * p.Kpad;
  uint32_t woff[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int row = (wq * GB + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    woff[i] = (uint32_t)(row * p.Kpad + c * VEC);
  }
  const void* const zero = p.zero;
  const __attribute__((address_space(4))) KStep* kdesc = (const __attribute__((address_space(4))) KStep*)p.ks;
  const T* lbase[GA];
  uint32_t lmask[GA];
  int cur_seg = -1;
  lds_char* const ring = lds + grp * GRP_RING;

  // k-step descriptors (scalar loads) are fetched one k-step before their DMA is issued: a cold
  // descriptor is an L2 / MALL round trip, which on the issue path delayed every k-step's DMA
  // (the latency chain these tiny layers are bound by). Past the layer's end: its last step.
  auto load_desc = [&](int j) __attribute__((always_inline)) -> KStep {
    const int ks = min(kbeg + j, p.nks - 1);
    c_u32x4* kq = (c_u32x4*)(kdesc + ks);
    struct { u32x4 q[5]; } raw = {{kq[0], kq[1], kq[2], kq[3], kq[4]}};
    return __builtin_bit_cast(KStep, raw);
  };
  // k-step kbeg + j (descriptor d) of this group into ring slot `slot`
  auto issue = [&](int j, int slot, const KStep& d) __attribute__((always_inline)) {
    const int ks = kbeg + j;
    if (d.seg != cur_seg) {
      cur_seg = d.seg;
      const T* src = reinterpret_cast<const T*>(d.src);
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int iy0 = poy[i] * d.stride - d.pad_h;
        const int ix0 = pox[i] * d.stride - d.pad_w;
        lbase[i] = src + ((long long)(pb[i] * d.H + iy0) * d.W + ix0) * d.ldc + pc[i] * VEC;
        uint32_t mk = 0;
        for (int ky = 0; ky < d.kh; ++ky) {
          const bool rok = (unsigned)(iy0 + ky) < (unsigned)d.H;
          for (int kx = 0; kx < d.kw; ++kx)
            mk |= (uint32_t)(rok && (unsigned)(ix0 + kx) < (unsigned)d.W) << (ky * d.kw + kx);
        }
        lmask[i] = pv[i] ? mk : 0u;
      }
    }
    lds_char* abase = ring + slot * STAGE + wq * GA * 1024;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const bool ok = (lmask[i] >> d.tap) & 1u;
      dma16(ok ? (const void*)(lbase[i] + d.off) : zero, abase + i * 1024);
    }
    lds_char* bbase = ring + slot * STAGE + A_BYTES + wq * GB * 1024;
    const T* wk = wbase + (size_t)ks * BK;
#pragma unroll
    for (int i = 0; i < GB; ++i) dma16(wk + woff[i], bbase + i * 1024);
  };

  // ---- MFMA geometry: wave (wp, wc) owns pixels [wp*32, +32) x channels [wc*64, +64)
  const int lrow = lane & 31;
  const int lh = lane >> 5;
  const int xr = wp * 32 + lrow;
  const int wr = wc * 64 + lrow;   // weight row of fragment nb = 0 (nb = 1 at +32 rows)
  unsigned xaddr[4], waddr[4];
  const unsigned lds0 = (unsigned)(uintptr_t)ring;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = X3 ? 4 * (j >> 1) + 2 * lh + (j & 1) : 2 * j + lh;  // X3: lane half lh of sub-step pair s = K group 2s + lh
    xaddr[j] = lds0 + xr * ROWB + ((c ^ ((xr >> 1) & 7)) << 4);
    waddr[j] = lds0 + A_BYTES + wr * ROWB + ((c ^ ((wr >> 1) & 7)) << 4);
  }
  f32x16 acc[2] = {f32x16{}, f32x16{}};
  u32x4 fa[4][3], fb[4][3];  // per 16-deep sub-step j: weights nb = 0, 1, then pixels
  auto read_frags = [&](int j0, u32x4(&f)[4][3]) __attribute__((always_inline)) {
    const unsigned so = (unsigned)((j0 % S) * STAGE);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j][0] = ds_read16(waddr[j] + so);
      f[j][1] = ds_read16(waddr[j] + so + 32 * ROWB);
      f[j][2] = ds_read16(xaddr[j] + so);
    }
  };
  auto mfmas = [&](const u32x4(&f)[4][3]) __attribute__((always_inline)) {
    if constexpr (X3) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const u32x4 c0 = f[2 * st][2], c1 = f[2 * st + 1][2];
        const float v[8] = {__uint_as_float(c0.x), __uint_as_float(c0.y), __uint_as_float(c0.z), __uint_as_float(c0.w),
                            __uint_as_float(c1.x), __uint_as_float(c1.y), __uint_as_float(c1.z), __uint_as_float(c1.w)};
        half8 xh, xl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[e] = (_Float16)v[e];
          xl[e] = (_Float16)(v[e] - (float)xh[e]);
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const half8 wh = __builtin_bit_cast(half8, f[2 * st][nb]), wl = __builtin_bit_cast(half8, f[2 * st + 1][nb]);
          acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc[nb], 0, 0, 0);
          acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc[nb], 0, 0, 0);
          acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc[nb], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) Mfma<T>::run(to_u4(f[j][nb]), to_u4(f[j][2]), acc[nb]);
    }
  };
  // iteration j (both groups run `half` iterations so every wave meets every barrier; group 1
  // idles through its last one when nks is odd): stage j's fragments are in `cur`
  KStep dn;  // descriptor of the next k-step to issue
  auto step = [&](int j, u32x4(&cur)[4][3], u32x4(&nxt)[4][3]) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (j + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");  // stage j+1 landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage j+1 visible to the group, slot j%S released
    __builtin_amdgcn_sched_barrier(0);
    if (j + S < nk) issue(j + S, j % S, dn);
    if (j + S + 1 < nk) dn = load_desc(j + S + 1);  // waited at the next step's lgkmcnt(0)
    if (j + 1 < nk) read_frags(j + 1, nxt);
    __builtin_amdgcn_sched_barrier(0);
    if (j < nk) mfmas(cur);
    __builtin_amdgcn_sched_barrier(0);
  };

  // this thread's epilogue bias chunks, loaded up front: issued after the loop they were one more
  // memory round trip at the end of a latency-bound kernel
  constexpr int RPT = PX * (CH / 8) / NT;  // 8-channel output chunks per thread (2)
  uint4 bpre[RPT][2];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int n = n0 + ((tid + r * NT) & 15) * 8;
    const bool ok = n < p.N;
    bpre[r][0] = ok ? gload16(p.bias + n) : make_uint4(0, 0, 0, 0);
    bpre[r][1] = ok ? gload16(p.bias + n + 4) : make_uint4(0, 0, 0, 0);
  }
  const int npro = nk < S ? nk : S;
  static_assert(S == 3, "prologue descriptors");
  const KStep d0 = load_desc(0), d1 = load_desc(1), d2 = load_desc(2);  // all in flight at once
  if (npro > 0) issue(0, 0, d0);
  if (npro > 1) issue(1, 1, d1);
  if (npro > 2) issue(2, 2, d2);
  dn = load_desc(S);
  if (npro >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
  else if (npro == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (nk > 0) read_frags(0, fa);
  for (int j = 0; j < half; j += 2) {
    step(j, fa, fb);
    if (j + 1 < half) step(j + 1, fb, fa);
  }

  // ---- reduction: group 1's partial tile through LDS into group 0's accumulators (fixed order)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  float* stg = reinterpret_cast<float*>(smem);
  // acc[nb] element 4g + e: channel wc*64 + nb*32 + 8g + 4lh + e of pixel xr
  if (grp == 1) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(stg + xr * SR + wc * 64 + nb * 32 + 8 * g + 4 * lh) =
            f32x4{acc[nb][4 * g], acc[nb][4 * g + 1], acc[nb][4 * g + 2], acc[nb][4 * g + 3]};
  }
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4* q = reinterpret_cast<f32x4*>(stg + xr * SR + wc * 64 + nb * 32 + 8 * g + 4 * lh);
        const f32x4 o = *q;
        *q = f32x4{acc[nb][4 * g] + o[0], acc[nb][4 * g + 1] + o[1], acc[nb][4 * g + 2] + o[2],
                   acc[nb][4 * g + 3] + o[3]};
      }
  }
  __syncthreads();
  f32x4 xs[RPT][2];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int it = tid + r * NT;
    const float* sv = stg + (it >> 4) * SR + (it & 15) * 8;
    xs[r][0] = *reinterpret_cast<const f32x4*>(sv);
    xs[r][1] = *reinterpret_cast<const f32x4*>(sv + 4);
  }
  if (ksplit > 1) {
    // Split-K hand-off (cdna_hip_programming.md §6 Guideline 16, write-through form): this slice's
    // partial tile goes to slab[tile][slice] with sc1 stores (no release fence), every storing
    // wave drains them (vmcnt(0)), the workgroup barrier orders that before ONE relaxed agent-scope
    // ticket; the workgroup drawing ksplit - 1 sums every slice in slice order 0, 1, ... (its own
    // from registers, the others by sc1 loads: bit-identical whichever workgroup arrives last) and
    // resets the ticket. The engine also zeroes the tickets before each forward.
    i32x4 rs;
    {
      const unsigned long long a = (unsigned long long)(p.slab + (size_t)lin * ksplit * (PX * CH));
      rs.x = (int)(unsigned)a;
      rs.y = (int)(unsigned)(a >> 32);
      rs.z = ksplit * PX * CH * 4;
      rs.w = 0x00020000;
    }
    constexpr int SC1 = 16;  // aux cache bits: sc1 (write-through store / L1-bypassing load)
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int it = tid + r * NT;
      if (m0 + (it >> 4) >= p.M) continue;  // only live rows travel
      const int off = (slice * (PX * CH) + it * 8) * 4;
      raw_buffer_store_v4(__builtin_bit_cast(u32x4, xs[r][0]), rs, off, 0, SC1);
      raw_buffer_store_v4(__builtin_bit_cast(u32x4, xs[r][1]), rs, off + 16, 0, SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its slab bytes landed
    __syncthreads();
    unsigned* last_flag = reinterpret_cast<unsigned*>(smem + LDS - 16);
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add((gu32*)(p.cnt + lin), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_flag = t;
    }
    __syncthreads();
    if (*last_flag != (unsigned)(ksplit - 1)) return;  // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: every slab load below is sc1
    f32x4 sum[RPT][2];
#pragma unroll
    for (int r = 0; r < RPT; ++r) sum[r][0] = sum[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < ksplit; ++q) {
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int it = tid + r * NT;
        f32x4 a0 = xs[r][0], a1 = xs[r][1];
        if (q != slice) {
          const int off = (q * (PX * CH) + it * 8) * 4;
          const bool live = m0 + (it >> 4) < p.M;
          a0 = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, live ? off : (int)0x80000000u, 0, SC1));
          a1 = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, live ? off + 16 : (int)0x80000000u, 0, SC1));
        }
        if (q == 0) {
          sum[r][0] = a0;
          sum[r][1] = a1;
        } else {
          sum[r][0] += a0;
          sum[r][1] += a1;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      xs[r][0] = sum[r][0];
      xs[r][1] = sum[r][1];
    }
    if (tid == 0) __hip_atomic_store((gu32*)(p.cnt + lin), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // bias + activation + 16-byte stores: 64 pixels x 16 chunks of 8 channels, 2 per thread
  T* const out = reinterpret_cast<T*>(p.out);
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int it = tid + r * NT;
    const int px = it >> 4, c8 = (it & 15) * 8;
    const int m = m0 + px;
    const int n = n0 + c8;
    if (m >= p.M || n >= p.N) continue;
    const f32x4 x0 = xs[r][0];
    const f32x4 x1 = xs[r][1];
    const uint4 b0 = bpre[r][0], b1 = bpre[r][1];
    float v[8] = {x0[0] + __uint_as_float(b0.x), x0[1] + __uint_as_float(b0.y), x0[2] + __uint_as_float(b0.z),
                  x0[3] + __uint_as_float(b0.w), x1[0] + __uint_as_float(b1.x), x1[1] + __uint_as_float(b1.y),
                  x1[2] + __uint_as_float(b1.z), x1[3] + __uint_as_float(b1.w)};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (p.act == 1) v[e] = fmaxf(v[e], 0.0f);
      else if (p.act == 2) v[e] = v[e] >= 0.0f ? v[e] : 0.01f * v[e];
    }
    if constexpr (sizeof(T) == 4) {  // fp32: 8 channels are two 16-byte chunks
      store_chunk<T>(out + (size_t)m * p.out_ldc + p.out_coff + n, v);
      store_chunk<T>(out + (size_t)m * p.out_ldc + p.out_coff + n + 4, v + 4);
    } else {
      store_chunk<T>(out + (size_t)m * p.out_ldc + p.out_coff + n, v);
    }
  }
}

template <typename T, bool X3 = false>
__global__ __launch_bounds__(NT, 1) void conv_lat(const ConvParams* __restrict__ pp) {
  conv_lat_tile<T, X3>(pp, blockIdx.x);
}

// several independent layers in one launch (the engine's schedule: layers of one dependency
// level): workgroups [end[k-1], end[k]) run layer k, each with its own split-K slab / tickets
struct LatGroup {
  const ConvParams* p[kLatGroupMax];
  int end[kLatGroupMax];
  int n;
};
template <typename T, bool X3 = false>
__global__ __launch_bounds__(NT, 1) void conv_lat_group(const LatGroup g) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < g.n && b >= g.end[k]) ++k;  // (workgroup-uniform)
  conv_lat_tile<T, X3>(g.p[k], b - (k ? g.end[k - 1] : 0));
}

template <typename T, bool X3 = false>
static int launch_group_t(const LatGroup& g, hipStream_t s) {
  if (int r = ensure_lds<conv_lat_group<T, X3>>(LDS)) return r;
  hipLaunchKernelGGL((conv_lat_group<T, X3>), dim3(g.end[g.n - 1]), dim3(NT), LDS, s, g);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T, bool X3 = false>
static int launch_t(const ConvParams& p, const ConvParams* dp, hipStream_t s) {
  if (int r = ensure_lds<conv_lat<T, X3>>(LDS)) return r;
  hipLaunchKernelGGL((conv_lat<T, X3>), dim3(p.mtiles * p.ntiles * (p.ksplit > 1 ? p.ksplit : 1)), dim3(NT), LDS, s, dp);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace lat

int conv_lat_tiles(int M, int N, int* mtiles, int* ntiles) {
  *mtiles = (M + lat::PX - 1) / lat::PX;
  *ntiles = (N + lat::CH - 1) / lat::CH;
  return *mtiles * *ntiles;
}

static bool lat_geometry_ok(const ConvParams& p) {
  return p.ks && p.nks > 0 && p.mtiles == (p.M + lat::PX - 1) / lat::PX && p.ntiles * lat::CH >= p.N && p.N % 8 == 0 &&
         p.out_ldc % 8 == 0 && p.out_coff % 8 == 0 && p.out && !(p.ksplit > 1 && (!p.slab || !p.cnt || p.ksplit > p.nks));
}

int launch_conv_lat(const ConvParams& p, const ConvParams* dp, int dtype, hipStream_t s, int x3) {
  if (!lat_geometry_ok(p)) {
    set_error("conv_lat: inconsistent launch geometry");
    return 1;
  }
  if (dtype == F16) return lat::launch_t<_Float16>(p, dp, s);
  if (dtype == BF16) return lat::launch_t<__bf16>(p, dp, s);
  return x3 ? lat::launch_t<float, true>(p, dp, s) : lat::launch_t<float>(p, dp, s);
  return 1;
}

int launch_conv_lat_group(const ConvParams* const* hp, const ConvParams* const* dp, int n, int dtype, hipStream_t s,
                          int x3) {
  if (n < 1 || n > kLatGroupMax) {
    set_error("conv_lat group: 1..kLatGroupMax layers");
    return 1;
  }
  lat::LatGroup g{};
  g.n = n;
  int wg = 0;
  for (int k = 0; k < n; ++k) {
    const ConvParams& p = *hp[k];
    if (!lat_geometry_ok(p)) {
      set_error("conv_lat group: inconsistent launch geometry");
      return 1;
    }
    wg += p.mtiles * p.ntiles * (p.ksplit > 1 ? p.ksplit : 1);
    g.p[k] = dp[k];
    g.end[k] = wg;
  }
  if (dtype == F16) return lat::launch_group_t<_Float16>(g, s);
  if (dtype == BF16) return lat::launch_group_t<__bf16>(g, s);
  return x3 ? lat::launch_group_t<float, true>(g, s) : lat::launch_group_t<float>(g, s);
}

}  // namespace tv
