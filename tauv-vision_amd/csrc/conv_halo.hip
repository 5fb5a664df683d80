// Halo-tile direct convolution for 3x3 / stride 1 / pad 1 layers (gfx950) — the dominant
// shape of the DLA backbone (IDA projection/output convs, tree conv1s, stacked heads).
//
// One 512-thread workgroup (8 waves, 2 per SIMD) computes a TH x TW = 256-pixel spatial block
// of one frame for 128 output channels. Instead of re-gathering the input once per tap
// (9x per channel block, conv_pipe.hip), the (TH+2) x (TW+2) input halo of one channel block
// (BK channels = 128 bytes) is moved into LDS once by LDS-DMA, and the nine taps read shifted
// windows of it at compile-time-immediate ds_read offsets. Per k-step only the 16 KiB weight
// panel streams (3-slot ring, counted vmcnt, one raw barrier), and the next channel block's
// halo is prefetched into the second halo buffer a whole channel block (9 k-steps) ahead.
//
// LDS: halo buffers 2 x 48 KiB (pixel pitch 144 B: 128 B of channels + 16 B pad, which makes
// 16 consecutive pixels hit 16 distinct bank slots), weight ring 3 x 16 KiB at 96 KiB.
// MFMA mapping, epilogue and fragment layouts are those of conv_pipe.hip.
#include "conv_common.h"

namespace tv {
namespace halo {

constexpr int NT = 512, NW = 8, BN = 128, S = 3;
constexpr int ROWB = 128;                  // bytes of K per k-step per row
constexpr int PITCH = 144;                 // halo pixel pitch (bytes)
constexpr int HBUF = 48 * 1024;            // one halo buffer (48 pieces of 1 KiB)
constexpr int HPIECES = HBUF / 1024 / NW;  // halo DMA instructions per wave = 6
constexpr int RING0 = 2 * HBUF;            // weight ring base
constexpr int WSLOT = BN * ROWB;           // 16 KiB
constexpr int GW = WSLOT / 1024 / NW;      // weight DMA instructions per wave per k-step = 2
constexpr int EROW = BN * 4 + 16;
constexpr int LDS = (RING0 + S * WSLOT) > 256 * EROW ? (RING0 + S * WSLOT) : 256 * EROW;

typedef __attribute__((address_space(3))) char lds_char;
typedef const __attribute__((address_space(1))) void gvoid;

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt needs an immediate: dispatch the (wave-uniform) count over the values that occur
__device__ __forceinline__ void wait_vm_dyn(int n) {
  if (n >= 14) wait_vm<14>();
  else if (n >= 12) wait_vm<12>();
  else if (n >= 8) wait_vm<8>();
  else if (n >= 6) wait_vm<6>();
  else if (n >= 2) wait_vm<2>();
  else wait_vm<0>();
}

// X fragments of one 16-deep sub-step j for tap (ky, kx) in halo buffer `buf`
template <int TW, int BUF, int KY, int KX, int J>
__device__ __forceinline__ void read_x(unsigned xb0, unsigned xb1, u32x4& f0, u32x4& f1) {
  constexpr int OFF = BUF * HBUF + (KY * (TW + 2) + KX) * PITCH + 32 * J;
  f0 = ds_read16_off<OFF>(xb0);
  f1 = ds_read16_off<OFF>(xb1);
}

template <typename T, int TW, int BUF, int KY, int KX>
__device__ __forceinline__ void tap_mfma(unsigned xb0, unsigned xb1, const unsigned (&wa)[4], unsigned so,
                                         f32x16 (&acc)[2][2]) {
  u32x4 fw[2][2], fx[2][2];
  fw[0][0] = ds_read16(wa[0] + so);
  fw[0][1] = ds_read16_off<32 * ROWB>(wa[0] + so);
  read_x<TW, BUF, KY, KX, 0>(xb0, xb1, fx[0][0], fx[0][1]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cb = j & 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (j < 3) {
      fw[cb ^ 1][0] = ds_read16(wa[j + 1] + so);
      fw[cb ^ 1][1] = ds_read16_off<32 * ROWB>(wa[j + 1] + so);
      if (j == 0) read_x<TW, BUF, KY, KX, 1>(xb0, xb1, fx[1][0], fx[1][1]);
      if (j == 1) read_x<TW, BUF, KY, KX, 2>(xb0, xb1, fx[0][0], fx[0][1]);
      if (j == 2) read_x<TW, BUF, KY, KX, 3>(xb0, xb1, fx[1][0], fx[1][1]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) Mfma<T>::run(to_u4(fw[cb][a]), to_u4(fx[cb][b]), acc[a][b]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <typename T, int TW, int BUF>
__device__ __forceinline__ void tap_dispatch(int tap, unsigned xb0, unsigned xb1, const unsigned (&wa)[4],
                                             unsigned so, f32x16 (&acc)[2][2]) {
  switch (tap) {
    case 0: tap_mfma<T, TW, BUF, 0, 0>(xb0, xb1, wa, so, acc); break;
    case 1: tap_mfma<T, TW, BUF, 0, 1>(xb0, xb1, wa, so, acc); break;
    case 2: tap_mfma<T, TW, BUF, 0, 2>(xb0, xb1, wa, so, acc); break;
    case 3: tap_mfma<T, TW, BUF, 1, 0>(xb0, xb1, wa, so, acc); break;
    case 4: tap_mfma<T, TW, BUF, 1, 1>(xb0, xb1, wa, so, acc); break;
    case 5: tap_mfma<T, TW, BUF, 1, 2>(xb0, xb1, wa, so, acc); break;
    case 6: tap_mfma<T, TW, BUF, 2, 0>(xb0, xb1, wa, so, acc); break;
    case 7: tap_mfma<T, TW, BUF, 2, 1>(xb0, xb1, wa, so, acc); break;
    default: tap_mfma<T, TW, BUF, 2, 2>(xb0, xb1, wa, so, acc); break;
  }
}

template <typename T, typename OutT, int TW>
__global__ __launch_bounds__(NT, 2) void conv_halo(const ConvParams* __restrict__ pp, void* out_ptr) {
  constexpr int TH = 256 / TW;
  constexpr int HW_ = TW + 2;                 // halo width
  constexpr int NPIX = (TH + 2) * HW_;        // halo pixels
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = ROWB / sizeof(T);
  static_assert(NPIX * PITCH <= HBUF, "halo does not fit");
  const ConvParams& p = *pp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const ConvSegment& sg = p.seg[0];
  const int H = sg.H, W = sg.W, ldc = sg.ldc;
  const int tiles_y = (H + TH - 1) / TH, tiles_x = (W + TW - 1) / TW;
  const int nb = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ntile = lin % p.ntiles;
  const int mtile = lin / p.ntiles;
  const int n0 = ntile * BN;
  const int b = mtile / (tiles_y * tiles_x);
  const int trem = mtile - b * tiles_y * tiles_x;
  const int y0 = (trem / tiles_x) * TH;
  const int x0 = (trem % tiles_x) * TW;

  const T* src = reinterpret_cast<const T*>(sg.src);
  const void* const zero = p.zero;
  const int ncb = sg.C / BK;            // channel blocks
  const int nks = 9 * ncb;

  // ---- halo DMA geometry: chunk g = piece*64 + lane -> halo pixel g/9, part g%9 (8 = pad)
  const T* hsrc[HPIECES];
  bool hok[HPIECES];
#pragma unroll
  for (int i = 0; i < HPIECES; ++i) {
    const int g = (wave * HPIECES + i) * 64 + lane;
    const int hp = g / 9;
    const int part = g - hp * 9;
    const int hy = hp / HW_, hx = hp - (hp / HW_) * HW_;
    const int y = y0 - 1 + hy, x = x0 - 1 + hx;
    hok[i] = part < 8 && hp < NPIX && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    hsrc[i] = src + ((long long)(b * H + (hok[i] ? y : 0)) * W + (hok[i] ? x : 0)) * ldc + part * VEC;
  }
  auto issue_halo = [&](int cb) __attribute__((always_inline)) {
    lds_char* base = lds + (cb & 1) * HBUF + wave * HPIECES * 1024;
#pragma unroll
    for (int i = 0; i < HPIECES; ++i) dma16(hok[i] ? (const void*)(hsrc[i] + cb * BK) : zero, base + i * 1024);
  };

  // ---- weight DMA: rows n0 + (wave*GW + i)*8 + lane/8, swizzled chunk; k-step (cb, tap)
  // reads packed columns [tap*C + cb*BK, +BK)
  const T* wbase = reinterpret_cast<const T*>(p.weight) + (size_t)n0 * p.Kpad;
  uint32_t woff[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int row = (wave * GW + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    woff[i] = (uint32_t)(row * p.Kpad + c * VEC);
  }
  auto issue_w = [&](int ks) __attribute__((always_inline)) {
    const int cb = ks / 9, tap = ks - cb * 9;
    const T* wk = wbase + (size_t)(tap * sg.C + cb * BK);
    lds_char* base = lds + RING0 + (ks % S) * WSLOT + wave * GW * 1024;
#pragma unroll
    for (int i = 0; i < GW; ++i) dma16(wk + woff[i], base + i * 1024);
  };

  // ---- MFMA geometry
  const int wm = wave & 3;
  const int wn = wave >> 2;
  const int lrow = lane & 31;
  const int lh = lane >> 5;
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  unsigned xb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int q = wm * 64 + t * 32 + lrow;  // tile pixel
    const int r = q / TW, c = q - (q / TW) * TW;
    xb[t] = lds0 + (r * HW_ + c) * PITCH + lh * 16;
  }
  unsigned wa[4];
  const int wr = wn * 64 + lrow;
#pragma unroll
  for (int j = 0; j < 4; ++j) wa[j] = lds0 + RING0 + wr * ROWB + (((2 * j + lh) ^ ((wr >> 1) & 7)) << 4);

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = f32x16{};

  // prologue: halos of channel blocks 0 and 1, weights of k-steps 0 and 1
  issue_halo(0);
  if (ncb > 1) issue_halo(1);
  issue_w(0);
  if (nks > 1) issue_w(1);
  // DMA instructions per wave issued in iteration i (after its weight stage): weights GW,
  // plus the halo of channel block cb+1 at the first k-step of cb >= 1
  for (int ks = 0; ks < nks; ++ks) {
    // younger than w(ks): what iteration ks-2 issued after it, plus all of iteration ks-1
    const int cbm2 = (ks - 2) / 9, cbm1 = (ks - 1) / 9;
    const bool h2 = ks >= 2 && (ks - 2) % 9 == 0 && cbm2 >= 1 && cbm2 + 1 < ncb;
    const bool h1 = ks >= 1 && (ks - 1) % 9 == 0 && cbm1 >= 1 && cbm1 + 1 < ncb;
    const int younger = (h2 ? HPIECES : 0) + (ks + 1 < nks ? GW : 0) + (h1 ? HPIECES : 0);
    wait_vm_dyn(younger);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (ks + 2 < nks) issue_w(ks + 2);
    const int cb = ks / 9, tap = ks - cb * 9;
    if (tap == 0 && cb >= 1 && cb + 1 < ncb) issue_halo(cb + 1);
    const unsigned so = (unsigned)((ks % S) * WSLOT);
    if (cb & 1) tap_dispatch<T, TW, 1>(tap, xb[0], xb[1], wa, so, acc);
    else tap_dispatch<T, TW, 0>(tap, xb[0], xb[1], wa, so, acc);
  }

  // ---- epilogue: bias + activation into an fp32 staging tile, then 16-byte stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* stg = reinterpret_cast<float*>(smem);
  constexpr int SR = EROW / 4;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int pix = wm * 64 + bb * 32 + lrow;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = wn * 64 + a * 32 + 8 * g + 4 * lh;
        const uint4 braw = gload16(p.bias + n0 + ch);
        const float bias4[4] = {__uint_as_float(braw.x), __uint_as_float(braw.y), __uint_as_float(braw.z),
                                __uint_as_float(braw.w)};
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[a][bb][4 * g + e] + bias4[e];
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
  constexpr int CPR = BN / OVEC;
  constexpr int RSTEP = NT / CPR;
  const int cc = tid % CPR;
  const int n = n0 + cc * OVEC;
  if (n < p.N) {
    for (int q = tid / CPR; q < 256; q += RSTEP) {
      const int y = y0 + q / TW, x = x0 + q % TW;
      if (y >= H || x >= W) continue;
      const size_t m = ((size_t)b * H + y) * W + x;
      OutT* dst = reinterpret_cast<OutT*>(out_ptr) + m * p.out_ldc + p.out_coff + n;
      store_chunk<OutT>(dst, stg + q * SR + cc * OVEC);
    }
  }
}

template <typename T, typename OutT, int TW>
static int launch_halo_t(const ConvParams& p, const ConvParams* dp, void* out, hipStream_t s) {
  auto k = conv_halo<T, OutT, TW>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) {
      set_error(std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
      return 3;
    }
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(p.mtiles * p.ntiles), dim3(NT), LDS, s, dp, out);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T, typename OutT>
static int launch_halo_tw(const ConvParams& p, const ConvParams* dp, void* out, int tw, hipStream_t s) {
  return tw == 32 ? launch_halo_t<T, OutT, 32>(p, dp, out, s) : launch_halo_t<T, OutT, 16>(p, dp, out, s);
}

}  // namespace halo

int halo_tiles(int B, int H, int W, int tw) {
  const int th = 256 / tw;
  return B * ((H + th - 1) / th) * ((W + tw - 1) / tw);
}

int launch_conv_halo(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int out_f32, int tw,
                     hipStream_t s) {
  using namespace halo;
  if (dtype == F32) return launch_halo_tw<float, float>(p, dp, out, tw, s);
  if (dtype == F16)
    return out_f32 ? launch_halo_tw<_Float16, float>(p, dp, out, tw, s)
                   : launch_halo_tw<_Float16, _Float16>(p, dp, out, tw, s);
  return out_f32 ? launch_halo_tw<__bf16, float>(p, dp, out, tw, s) : launch_halo_tw<__bf16, __bf16>(p, dp, out, tw, s);
}

}  // namespace tv
