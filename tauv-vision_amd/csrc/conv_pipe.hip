// Pipelined implicit-GEMM convolution for large layers (gfx950).
//
// Same GEMM view and epilogues as conv.hip (rows = NHWC output pixels, columns = output
// channels, K = taps x channels), restructured for MI355X's memory system:
//   * 256-pixel x 128-channel tile per 512-thread workgroup (8 waves = 2 per SIMD, each
//     wave a 64x64 sub-tile of 2x2 v_mfma_f32_32x32x16 / 32x32x2f32 tiles);
//   * operands move global -> LDS by LDS-DMA (global_load_lds_dwordx4), no staging VGPRs:
//     one wave-instruction fills 1 KiB = 8 rows x 128 B; the XOR bank swizzle is applied to
//     the per-lane SOURCE address (the LDS image is lane-linear); padding taps read a
//     zero page instead of being masked;
//   * a 3-slot LDS ring (48 KiB per k-step) with one raw s_barrier per k-step and a counted
//     `s_waitcnt vmcnt`, so two k-steps of DMA stay in flight under the MFMAs;
//   * fragment reads are inline-asm ds_read_b128 (double-buffered per 16-deep sub-step) so
//     the compiler does not insert a vmcnt(0) drain in front of LDS reads while DMA to
//     other ring slots is in flight.
#include "conv_common.h"

namespace tv {
namespace pipe {

constexpr int BM = 256, BN = 128, NT = 512, NW = NT / 64, S = 3;
constexpr int ROWB = 128;                    // bytes of K per k-step per row
constexpr int A_BYTES = BM * ROWB;           // 32 KiB
constexpr int B_BYTES = BN * ROWB;           // 16 KiB
constexpr int STAGE = A_BYTES + B_BYTES;     // 48 KiB
constexpr int RING = S * STAGE;              // 144 KiB
constexpr int EROW = BN * 4 + 16;            // fp32 epilogue row (bytes)
constexpr int LDS = RING > BM * EROW ? RING : BM * EROW;
constexpr int GA = BM / 8 / NW;              // A pieces (1 KiB) per wave per k-step = 4
constexpr int GB = BN / 8 / NW;              // B pieces per wave per k-step = 2
constexpr int G = GA + GB;                   // LDS-DMA instructions per wave per k-step

typedef __attribute__((address_space(3))) char lds_char;
typedef const __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(1))) unsigned gu32;  // global (never flat) agent-scope ticket words
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");

__device__ __forceinline__ void dma16(const void* src, lds_char* dst_wave_base) {
  __builtin_amdgcn_global_load_lds((gvoid*)src, (__attribute__((address_space(3))) void*)dst_wave_base, 16, 0, 0);
}

__device__ __forceinline__ u32x4 ds_read16(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int OFF>
__device__ __forceinline__ u32x4 ds_read16_off(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

// X3 (T = float only): fp32 operands, products as three fp16 MFMAs — a = a_hi + a_lo, b = b_hi + b_lo
// with hi = fp16(x), lo = fp16(x - hi) (22 significant bits), a*b = a_hi*b_hi + a_hi*b_lo + a_lo*b_hi
// (+ a_lo*b_lo ~ 2^-22 relative, dropped) accumulated in fp32: v_mfma_f32_32x32x16_f16 at 16x the
// MACs per instruction of v_mfma_f32_32x32x2_f32, three of them per product. The weights come
// pre-split (conv_pipe_x3_repack: per group of 8 K values 16 B of hi halves then 16 B of lo halves,
// the same bytes per row as fp32); the activation fragments are split in registers per sub-step.
// Lane half lh of sub-step s reads chunks 4s + 2lh (+1): K group 2s + lh of the 32-deep k-step in
// both operands (hi / lo halves of the weights, two 4-float chunks of the activations).
template <typename T, typename OutT, int MODE, bool X3 = false>
__global__ __launch_bounds__(NT, 2) void conv_pipe(const ConvParams* __restrict__ pp, void* out_ptr) {
  static_assert(!X3 || sizeof(T) == 4, "X3: fp32 operands");
  const ConvParams& p = *pp;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = ROWB / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): LDS-DMA base in M0

  // split-K (ksplit > 1; either epilogue): ksplit workgroups per tile, adjacent in the XCD-contiguous order
  // so a tile's slices tend to share an L2; slice s walks k-steps [ks0, ks1)
  const int ksplit = p.ksplit > 1 ? p.ksplit : 1;
  const int nb = p.mtiles * p.ntiles * ksplit;
  const int bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  const int lin_s = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int lin = lin_s / ksplit;
  const int slice = lin_s - lin * ksplit;
  const int ks0 = (int)((long)p.nks * slice / ksplit);
  const int ntile = lin % p.ntiles;
  const int mtile = lin / p.ntiles;
  const int m0 = mtile * BM;
  const int n0 = ntile * BN;

  // ---- DMA geometry. A piece i of this wave covers tile rows (wave*GA + i)*8 + lane/8; the
  // lane's LDS slot is lane%8 and it fetches chunk (lane%8) ^ ((row>>1)&7) of that row.
  int pb[GA], poy[GA], pox[GA], pc[GA];
  bool pv[GA];
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = (wave * GA + i) * 8 + (lane >> 3);
    const int m = m0 + row;
    pv[i] = m < p.M;
    const int mm = pv[i] ? m : 0;
    pb[i] = mm / hw;
    const int rem = mm - pb[i] * hw;
    poy[i] = rem / p.Wo;
    pox[i] = rem - poy[i] * p.Wo;
    pc[i] = (lane & 7) ^ ((row >> 1) & 7);
  }
  const T* wsrc[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int row = (wave * GB + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    wsrc[i] = reinterpret_cast<const T*>(p.weight) + (size_t)(n0 + row) * p.Kpad + c * VEC;
  }
  const int total_ks = (int)((long)p.nks * (slice + 1) / ksplit) - ks0;
  const void* const zero = p.zero;  // hoisted: the DMA intrinsic is treated as a memory clobber
  // constant address space: the per-k-step descriptor read is a scalar load, not a
  // (vmcnt-counted) vector load that would drain the DMA pipeline
  const __attribute__((address_space(4))) KStep* kdesc = (const __attribute__((address_space(4))) KStep*)p.ks + ks0;

  // Per-segment lane state for uniform-tap k-steps: the lane's base pointer (pixel
  // (b, oy*stride - pad_h, ox*stride - pad_w), its chunk) and a bit mask of the taps that land
  // inside the image. A k-step then costs one bit test and one 64-bit add per piece.
  const T* lbase[GA];
  uint32_t lmask[GA];
  int cur_seg = -1;
  // weights: uniform base advanced per k-step, per-lane 32-bit offsets
  const T* wbase = reinterpret_cast<const T*>(p.weight) + (size_t)n0 * p.Kpad;
  uint32_t woff[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) woff[i] = (uint32_t)(wsrc[i] - wbase);
  wbase += (size_t)ks0 * BK;  // this slice's first k-step

  // wave-uniform descriptor: 80 bytes by scalar loads (constant address space), fetched one
  // k-step before its DMA is issued (the prologue's three at once): a cold descriptor is an L2 /
  // MALL round trip that otherwise sits on every k-step's issue path. Past the end: the last one.
  auto load_desc = [&](int ks) __attribute__((always_inline)) -> KStep {
    const __attribute__((address_space(4))) u32x4* kq =
        (const __attribute__((address_space(4))) u32x4*)(kdesc + min(ks, total_ks - 1));
    struct { u32x4 q[5]; } raw = {{kq[0], kq[1], kq[2], kq[3], kq[4]}};
    return __builtin_bit_cast(KStep, raw);
  };
  auto issue = [&](int ks, int slot, const KStep& d) __attribute__((always_inline)) {
    const T* src = reinterpret_cast<const T*>(d.src);
    lds_char* abase = lds + slot * STAGE + wave * GA * 1024;
    if (d.mode == 0) {
      if (d.seg != cur_seg) {
        cur_seg = d.seg;
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
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const bool ok = (lmask[i] >> d.tap) & 1u;
        dma16(ok ? (const void*)(lbase[i] + d.off) : zero, abase + i * 1024);
      }
    } else {
      // C below BK: every 16-byte chunk resolves its own tap (cpt chunks per tap)
      cur_seg = -1;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int q = d.q0 + pc[i];
        const int tap = (int)(((float)q + 0.5f) * d.cpt_inv);
        const int ci = (q - tap * d.cpt) * VEC;
        const int ky = (int)(((float)tap + 0.5f) * d.kw_inv);
        const int kx = tap - ky * d.kw;
        const int iy = poy[i] * d.stride + ky - d.pad_h;
        const int ix = pox[i] * d.stride + kx - d.pad_w;
        const bool ok = pv[i] && tap < d.kh * d.kw && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const void* a = ok ? (const void*)(src + ((size_t)(pb[i] * d.H + iy) * d.W + ix) * d.ldc + ci) : zero;
        dma16(a, abase + i * 1024);
      }
    }
    lds_char* bbase = lds + slot * STAGE + A_BYTES + wave * GB * 1024;
    const T* wk = wbase + (size_t)ks * BK;
#pragma unroll
    for (int i = 0; i < GB; ++i) dma16(wk + woff[i], bbase + i * 1024);
  };

  // ---- MFMA geometry: wave (wm, wn) owns pixels [wm*64,+64) x channels [wn*64,+64)
  const int wm = wave & 3;
  const int wn = wave >> 2;
  const int lrow = lane & 31;
  const int lh = lane >> 5;
  const int xr = wm * 64 + lrow;   // pixel row of fragment t=0 (t=1 at +32 rows = +4096 B)
  const int wr = wn * 64 + lrow;   // weight row
  unsigned xaddr[4], waddr[4];
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = X3 ? 4 * (j >> 1) + 2 * lh + (j & 1) : 2 * j + lh;
    xaddr[j] = lds0 + xr * ROWB + ((c ^ ((xr >> 1) & 7)) << 4);
    waddr[j] = lds0 + A_BYTES + wr * ROWB + ((c ^ ((wr >> 1) & 7)) << 4);
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  // Fragments of one k-step (per sub-step j: W rows t=0,1 then X rows t=0,1). Two register
  // sets: the next k-step's fragments are read while this k-step's MFMAs run, so LDS latency
  // never sits between an MFMA and its operands.
  u32x4 fa[4][4], fb[4][4];
  auto read_frags = [&](int ks, u32x4(&f)[4][4]) __attribute__((always_inline)) {
    const unsigned so = (unsigned)((ks % S) * STAGE);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j][0] = ds_read16(waddr[j] + so);
      f[j][1] = ds_read16_off<32 * ROWB>(waddr[j] + so);
      f[j][2] = ds_read16(xaddr[j] + so);
      f[j][3] = ds_read16_off<32 * ROWB>(xaddr[j] + so);
    }
  };
  auto mfmas = [&](const u32x4(&f)[4][4]) __attribute__((always_inline)) {
    if constexpr (X3) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // one split activation fragment live at a time
          const u32x4 c0 = f[2 * st][2 + b], c1 = f[2 * st + 1][2 + b];
          const float v[8] = {__uint_as_float(c0.x), __uint_as_float(c0.y), __uint_as_float(c0.z), __uint_as_float(c0.w),
                              __uint_as_float(c1.x), __uint_as_float(c1.y), __uint_as_float(c1.z), __uint_as_float(c1.w)};
          half8 xh, xl;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            xh[e] = (_Float16)v[e];
            xl[e] = (_Float16)(v[e] - (float)xh[e]);
          }
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const half8 wh = __builtin_bit_cast(half8, f[2 * st][a]), wl = __builtin_bit_cast(half8, f[2 * st + 1][a]);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc[a][b], 0, 0, 0);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) Mfma<T>::run(to_u4(f[j][a]), to_u4(f[j][2 + b]), acc[a][b]);
    }
  };
  KStep dn;  // descriptor of the next k-step to issue
  // one k-step: stage ks's fragments are in `cur`; DMA keeps stages ks+2, ks+3 in flight
  auto step = [&](int ks, u32x4(&cur)[4][4], u32x4(&nxt)[4][4]) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of stage ks landed
    if (ks + 2 < total_ks) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");  // stage ks+1 landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave: stage ks+1 visible, slot ks%S released
    __builtin_amdgcn_sched_barrier(0);
    if (ks + S < total_ks) issue(ks + S, ks % S, dn);
    if (ks + S + 1 < total_ks) dn = load_desc(ks + S + 1);  // waited at the next step's lgkmcnt(0)
    if (ks + 1 < total_ks) read_frags(ks + 1, nxt);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(cur);
    __builtin_amdgcn_sched_barrier(0);
  };

  const int npro = total_ks < S ? total_ks : S;
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
  read_frags(0, fa);
  for (int ks = 0; ks < total_ks; ks += 2) {
    step(ks, fa, fb);
    if (ks + 1 < total_ks) step(ks + 1, fb, fa);
  }

  // ---- epilogue: bias + activation into an fp32 staging tile, then 16-byte stores (split-K: the
  // raw partial tile; bias and activation after the slices are summed)
  __syncthreads();
  float* stg = reinterpret_cast<float*>(smem);
  constexpr int SR = EROW / 4;
  const bool split = ksplit > 1;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int pix = wm * 64 + b * 32 + lrow;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = wn * 64 + a * 32 + 8 * g + 4 * lh;
        const uint4 braw = gload16(p.bias + n0 + ch);
        const float bias4[4] = {__uint_as_float(braw.x), __uint_as_float(braw.y), __uint_as_float(braw.z),
                                __uint_as_float(braw.w)};
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[a][b][4 * g + e];
          if (split) {
            v[e] = x;
            continue;
          }
          x += bias4[e];
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
  constexpr int CPR = BN / OVEC;       // 16-byte chunks per staged row
  constexpr int RSTEP = NT / CPR;      // rows covered per pass; each thread keeps one chunk column
  constexpr int NP = BM / RSTEP;       // passes
  const int cc = tid % CPR;
  const int r0 = tid / CPR;
  const int n = n0 + cc * OVEC;
  if (split) {
    // Split-K hand-off (the conv_lat.hip scheme): the partial tile goes to slab[tile][slice] with
    // write-through sc1 stores, each wave drains them, the workgroup barrier orders that before one
    // relaxed agent-scope ticket; the workgroup drawing ksplit - 1 sums the slices in slice order
    // (its own from LDS, the others by L1-bypassing sc1 loads: bit-identical whichever arrives
    // last), applies bias + activation, stores, and resets the ticket.
    constexpr int TILE_F = BM * BN;
    constexpr int SC1 = 16;
    i32x4 rs;
    {
      const unsigned long long a = (unsigned long long)(p.slab + (size_t)lin * ksplit * TILE_F);
      rs.x = (int)(unsigned)a;
      rs.y = (int)(unsigned)(a >> 32);
      rs.z = ksplit * TILE_F * 4;
      rs.w = 0x00020000;
    }
    constexpr int FCPR = BN / 4, FRSTEP = NT / FCPR, FNP = BM / FRSTEP;
    const int fcc = tid % FCPR, fr0 = tid / FCPR;
#pragma unroll
    for (int k = 0; k < FNP; ++k) {
      const int row = fr0 + k * FRSTEP;
      if (m0 + row >= p.M) break;
      const f32x4 v = *reinterpret_cast<const f32x4*>(stg + row * SR + fcc * 4);
      raw_buffer_store_v4(__builtin_bit_cast(u32x4, v), rs, ((slice * BM + row) * BN + fcc * 4) * 4, 0, SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* last_flag = reinterpret_cast<unsigned*>(smem + LDS - 16);
    if (tid == 0) *last_flag = __hip_atomic_fetch_add((gu32*)(p.cnt + lin), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*last_flag != (unsigned)(ksplit - 1)) return;  // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: every slab load below is sc1
    const int nf = n0 + fcc * 4;
    const uint4 braw = gload16(p.bias + nf);
    const float bias4[4] = {__uint_as_float(braw.x), __uint_as_float(braw.y), __uint_as_float(braw.z),
                            __uint_as_float(braw.w)};
    // every slice from the slab, this one included (its own sc1 stores have landed): no per-element
    // register-or-load select, which would make hipcc branch and wait per load; rows past M read
    // slab bytes that are never stored
    int roff[FNP];
#pragma unroll
    for (int k = 0; k < FNP; ++k) roff[k] = ((fr0 + k * FRSTEP) * BN + fcc * 4) * 4;
    f32x4 sum[FNP];
#pragma unroll
    for (int k = 0; k < FNP; ++k) sum[k] = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, roff[k], 0, SC1));
#pragma unroll 1
    for (int q = 1; q < ksplit; ++q) {
      f32x4 a[FNP];
#pragma unroll
      for (int k = 0; k < FNP; ++k) a[k] = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, roff[k] + q * (TILE_F * 4), 0, SC1));
#pragma unroll
      for (int k = 0; k < FNP; ++k) sum[k] += a[k];
    }
    // back through the staging tile so the stores keep the OutT chunking of the plain path
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FNP; ++k) {
      const int row = fr0 + k * FRSTEP;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = sum[k][e] + bias4[e];
        if (p.act == 1) x = fmaxf(x, 0.0f);
        else if (p.act == 2) x = x >= 0.0f ? x : 0.01f * x;
        v[e] = x;
      }
      *reinterpret_cast<f32x4*>(stg + row * SR + fcc * 4) = f32x4{v[0], v[1], v[2], v[3]};
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store((gu32*)(p.cnt + lin), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (MODE == 0) {
    if (n < p.N) {
#pragma unroll 4
      for (int k = 0; k < NP; ++k) {
        const int row = r0 + k * RSTEP;
        const int m = m0 + row;
        if (m >= p.M) break;
        OutT* dst = reinterpret_cast<OutT*>(out_ptr) + (size_t)m * p.out_ldc + p.out_coff + n;
        store_chunk<OutT>(dst, stg + row * SR + cc * OVEC);
      }
    }
  } else {
    // ConvTranspose phase scatter + skip add: this thread's channel chunk fixes (phase, co);
    // all skip-tensor loads of the thread are issued before any is consumed.
    const int phase = n / p.up_cout;
    const int co = n - phase * p.up_cout;
    const int pi = phase / p.up_s, pj = phase - pi * p.up_s;
    size_t toff[NP];
    uint4 av[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int m = m0 + r0 + k * RSTEP;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int oy = rem / p.Wo;
      const int ox = rem - oy * p.Wo;
      const int Y = oy * p.up_s + pi + p.sy;
      const int X = ox * p.up_s + pj + p.sx;
      const bool ok = n < p.N && m < p.M && Y < p.tH && X < p.tW;
      toff[k] = ok ? (size_t)(b * p.tH + Y) * p.tW + X : ~(size_t)0;
      av[k] = ok && p.add ? gload16(reinterpret_cast<const T*>(p.add) + toff[k] * p.add_ldc + co)
                          : make_uint4(0, 0, 0, 0);  // no skip tensor (protonet ConvT phases): plain scatter
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      if (toff[k] == ~(size_t)0) continue;
      const float* sv = stg + (r0 + k * RSTEP) * SR + cc * OVEC;
      const uint32_t rw4[4] = {av[k].x, av[k].y, av[k].z, av[k].w};
      float v[OVEC];
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
      store_chunk<OutT>(reinterpret_cast<OutT*>(out_ptr) + toff[k] * p.out_ldc + co, v);
    }
  }
}

template <typename T, typename OutT, int MODE, bool X3 = false>
static int launch_pipe_t(const ConvParams& p, const ConvParams* dp, void* out, hipStream_t s) {
  auto k = conv_pipe<T, OutT, MODE, X3>;
  if (int r = ensure_lds<conv_pipe<T, OutT, MODE, X3>>(LDS)) return r;
  const int ksplit = p.ksplit > 1 ? p.ksplit : 1;
  if (ksplit > 1 && (!p.slab || !p.cnt || ksplit > p.nks)) return 1;  // TV_EINVAL
  hipLaunchKernelGGL(k, dim3(p.mtiles * p.ntiles * ksplit), dim3(NT), LDS, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}

// [Npad][Kpad] fp32 -> the X3 weight copy: per row, per group of 8 K values, 8 hi then 8 lo halves
__global__ void x3_repack(const float* __restrict__ w, long groups, uint4* __restrict__ out) {
  for (long g = (long)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (long)gridDim.x * blockDim.x) {
    half8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = w[g * 8 + e];
      h[e] = (_Float16)v;
      l[e] = (_Float16)(v - (float)h[e]);
    }
    out[2 * g] = __builtin_bit_cast(uint4, h);
    out[2 * g + 1] = __builtin_bit_cast(uint4, l);
  }
}

}  // namespace pipe

int conv_pipe_x3_repack(const void* w, int Npad, int Kpad, void* out, hipStream_t s) {
  if (Kpad % 8 || !w || !out) {
    set_error("conv_pipe_x3_repack: Kpad must be a multiple of 8");
    return 1;
  }
  hipLaunchKernelGGL(pipe::x3_repack, dim3(256), dim3(256), 0, s, (const float*)w, (long)Npad * Kpad / 8, (uint4*)out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_conv_pipe(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int out_f32, int mode,
                     hipStream_t s, int x3) {
  using namespace pipe;
  if (dtype == F32) {
    if (x3)
      return mode == 0 ? launch_pipe_t<float, float, 0, true>(p, dp, out, s)
                       : launch_pipe_t<float, float, 1, true>(p, dp, out, s);
    return mode == 0 ? launch_pipe_t<float, float, 0>(p, dp, out, s) : launch_pipe_t<float, float, 1>(p, dp, out, s);
  } else if (dtype == F16) {
    if (mode == 1) return launch_pipe_t<_Float16, _Float16, 1>(p, dp, out, s);
    return out_f32 ? launch_pipe_t<_Float16, float, 0>(p, dp, out, s)
                   : launch_pipe_t<_Float16, _Float16, 0>(p, dp, out, s);
  } else {
    if (mode == 1) return launch_pipe_t<__bf16, __bf16, 1>(p, dp, out, s);
    return out_f32 ? launch_pipe_t<__bf16, float, 0>(p, dp, out, s) : launch_pipe_t<__bf16, __bf16, 0>(p, dp, out, s);
  }
}

}  // namespace tv
