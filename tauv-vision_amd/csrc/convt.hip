// ConvTranspose2d(k = s, stride = s) + pad_to_match + skip add (gfx950, fp16 / bf16) — the
// IDAUp / IDAUpReverse up-path of the reference: `f_i + pad_to_match(up(project(x)), f_i)`
// (dla.py:265-284, 340-357, pad_to_match :195-209, including its H/W-swapped F.pad quirk,
// folded into the target shift (sy, sx) by the planner).
//
// A k = s transposed conv is a per-pixel linear map: input pixel (iy, ix) produces the s x s
// block of target pixels (iy*s + py + sy, ix*s + px + sx), one 128-channel GEMM row per phase
// (py, px). Per phase it is a GEMM [input pixels] x [128 x 128], K = 128, and the pass is bound
// by HBM: per input pixel and phase it reads 256 B of skip tensor and writes 256 B (the 256 B of
// input pixel come from L2 after the first phase). The generic implicit GEMM staged that
// through a 3-slot LDS ring and an fp32 LDS epilogue per 256-pixel tile (2.7 TB/s). Here:
//  * a 256-thread workgroup owns one phase and a run of 32-pixel tiles; the phase's weights
//    (128 x 128, 34 KiB with a conflict-free 272 B row pitch) move to LDS once;
//  * each wave streams its own tiles with no barrier: the MFMA B operand (8 x 16 B of the
//    pixel's channels per lane) and the skip chunks the epilogue adds are loaded straight
//    into registers one tile ahead — issued before the previous tile's stores, so waiting for
//    them never waits for those stores (vector memory completes in issue order);
//  * the epilogue works on the accumulators in place (bias, + skip in fp32, one rounding,
//    v_permlane32_swap into 16-byte stores), in the same arithmetic order as conv_pipe's
//    mode-1 epilogue: (acc + bias) + skip.
#include "conv_common.h"

namespace tv {
namespace convt {

constexpr int NT = 512;        // 8 waves
constexpr int NW = NT / 64;
constexpr int C = 128;         // output channels per phase (4 MFMA row tiles)
constexpr int KJ = 8;          // K = 128 input channels = 8 MFMA k-steps of 16
constexpr int WPITCH = 272;    // LDS weight row pitch (bytes): odd multiple of 16 -> no bank conflicts
constexpr int PW = C * WPITCH; // one phase's weights
constexpr int NPG = 4;         // phases per workgroup on large inputs: the input tile is loaded once for all
template <int NP>
constexpr int lds_bytes() { return NP * (PW + C * 4); }

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}
template <typename T>
__device__ __forceinline__ float lo_f(unsigned u) {
  return (float)__builtin_bit_cast(T, (uint16_t)(u & 0xffffu));
}
template <typename T>
__device__ __forceinline__ float hi_f(unsigned u) {
  return (float)__builtin_bit_cast(T, (uint16_t)(u >> 16));
}

struct XSet {
  uint4 x[KJ];   // B operand: input pixel channels 16j + 8*lh .. +8
};
struct ASet {
  uint4 a[8];    // skip / residual chunks (i, m): channels 32i + 16m + 8*lh .. +8 at the target pixel
};

// A workgroup owns NP consecutive phases of the s*s and a run of 32-pixel input tiles; per tile
// a wave loads the input operand once and runs the NP phases, the skip chunks of the next phase
// step in flight under the current one (NP = 4 on large inputs; NP = 1 spreads small inputs over
// s*s times more workgroups).
template <typename T, int NP>
__device__ __forceinline__ void convt_tile(const ConvTParams& p, const int bx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(NP == 1 || NP % 2 == 0, "phase group");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int group = bx / p.nchunks;
  const int chunk = bx - group * p.nchunks;
  const int phase0 = group * NP;

  // ---- the group's weights and bias into LDS (rows n = phase*C + co of the packed [N][Kpad])
  // (every load of the copy is issued before the first LDS write: one memory latency for the whole
  // prologue instead of one per 16-byte chunk, which serialised ~16 L2/HBM round trips per wave)
  {
    const char* wsrc = reinterpret_cast<const char*>(p.weight) + (size_t)phase0 * C * p.Kpad * sizeof(T);
    constexpr int NCH = NP * C * 16 / NT;  // 16-byte chunks per thread (NP * 4)
    static_assert((NP * C * 16) % NT == 0 && NP * C <= NT, "prologue split");
    uint4 wv[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int i = tid + k * NT;
      const int r = i >> 4, c = i & 15;  // r = phase-in-group * C + co
      wv[k] = *reinterpret_cast<const uint4*>(wsrc + (size_t)r * p.Kpad * sizeof(T) + c * 16);
    }
    float* lb = reinterpret_cast<float*>(smem + NP * PW);
    const float bv = tid < NP * C ? p.bias[phase0 * C + tid] : 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int i = tid + k * NT;
      *reinterpret_cast<uint4*>(smem + (i >> 4) * WPITCH + (i & 15) * 16) = wv[k];
    }
    if (tid < NP * C) lb[tid] = bv;
  }
  __syncthreads();

  // GEMM rows are input pixels (b, iy, ix)
  const int hw = p.h * p.w;
  const int M = p.B * hw;
  const int mt = (M + 31) / 32;
  // this wave's contiguous run of the group's tiles: an even split over all the group's waves
  // (every CU busy: the pass is bound by each CU's own ~10 B/clk of HBM loads)
  const long long gw = (long long)chunk * NW + wave, nw = (long long)p.nchunks * NW;
  const int t_begin = (int)(mt * gw / nw);
  const int t_end = (int)(mt * (gw + 1) / nw);
  if (t_begin >= t_end) return;

  // target element offset (channel 0) of this lane's pixel in tile t for phase ph, or -1
  auto target = [&](int t, int ph) __attribute__((always_inline)) -> long long {
    const int m = t * 32 + l32;
    if (m >= M) return -1;
    const int phase = phase0 + ph;
    const int py = phase / p.s, px = phase - py * p.s;
    const int b = m / hw;
    const int rem = m - b * hw;
    const int iy = rem / p.w, ix = rem - iy * p.w;
    const int Y = iy * p.s + py + p.sy, X = ix * p.s + px + p.sx;
    if (Y >= p.tH || X >= p.tW) return -1;
    return ((long long)(b * p.tH + Y) * p.tW + X);
  };
  auto load_x = [&](int t, XSet& S) __attribute__((always_inline)) {
    const int m = t * 32 + l32;
    const size_t sp = (size_t)(m < M ? m : 0);
    const T* src = reinterpret_cast<const T*>(p.src) + sp * p.src_ldc + 8 * lh;
#pragma unroll
    for (int j = 0; j < KJ; ++j) S.x[j] = gload16(src + 16 * j);
  };
  auto load_a = [&](int t, int ph, ASet& S) __attribute__((always_inline)) {
    const long long tg = target(t, ph);
    const T* add = reinterpret_cast<const T*>(p.add) + (tg < 0 ? 0 : tg) * p.add_ldc + 8 * lh;
#pragma unroll
    for (int q = 0; q < 8; ++q) S.a[q] = gload16(add + 16 * q);  // q = 2i + m -> channel 16q + 8lh
  };

  auto compute_store = [&](int t, int ph, const XSet& X, const ASet& A) __attribute__((always_inline)) {
    const char* wl = smem + ph * PW + l32 * WPITCH + lh * 16;
    const float* lb = reinterpret_cast<const float*>(smem + NP * PW) + ph * C;
    const long long tg = target(t, ph);
    T* out = reinterpret_cast<T*>(p.out) + (tg < 0 ? 0 : tg) * p.out_ldc;
    // two halves of 64 output channels: half the accumulators live at a time (the x operand is
    // reused, the weights are re-read from LDS) — keeps the kernel inside 256 VGPRs without spills
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      f32x16 acc[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i] = f32x16{};
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        uint4 wv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) wv[i] = *reinterpret_cast<const uint4*>(wl + (2 * hf + i) * 32 * WPITCH + j * 32);
#pragma unroll
        for (int i = 0; i < 2; ++i) Mfma<T>::run(wv[i], X.x[j], acc[i]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * hf + ii;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float v[2][4];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int G2 = 2 * m + gg;
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[gg][e] = acc[ii][4 * G2 + e] + bb[e];
          }
          // registers -> 16-byte chunk: lanes 0-31 channels 32i+16m+0..7, lanes 32-63 +8..15
          float f[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0][e]), __float_as_uint(v[1][e]), false,
                                                            false);
            f[e] = __uint_as_float(r[0]);
            f[4 + e] = __uint_as_float(r[1]);
          }
          unsigned o[4];
          const uint4 sk = A.a[2 * i + m];
          const unsigned sw[4] = {sk.x, sk.y, sk.z, sk.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack2<T>(lo_f<T>(sw[e]) + f[2 * e], hi_f<T>(sw[e]) + f[2 * e + 1]);
          if (tg >= 0) gstore16(out + 32 * i + 16 * m + 8 * lh, make_uint4(o[0], o[1], o[2], o[3]));
        }
      }
    }
  };

  // Steps (tile, phase) in order; the operands of the next step are loaded before the current
  // step's stores are issued (vector memory completes in issue order). Register sets
  // alternate: x by tile parity, skip by step parity (NP is 1 or even) -> unrolled by 2 tiles.
  XSet x0, x1;
  ASet a0, a1;
  load_x(t_begin, x0);
  load_a(t_begin, 0, a0);
  if constexpr (NP == 1) {
    // single phase: both sets alternate per tile
    for (int t = t_begin; t < t_end; t += 2) {
      if (t + 1 < t_end) {
        load_x(t + 1, x1);
        load_a(t + 1, 0, a1);
      }
      compute_store(t, 0, x0, a0);
      if (t + 1 >= t_end) break;
      if (t + 2 < t_end) {
        load_x(t + 2, x0);
        load_a(t + 2, 0, a0);
      }
      compute_store(t + 1, 0, x1, a1);
    }
  } else {
    // NP (even) phases per tile: skip sets alternate per phase (even phases a0), x per tile
    auto tile = [&](int t, XSet& xc, XSet& xn) __attribute__((always_inline)) {
#pragma unroll
      for (int ph = 0; ph < NP; ph += 2) {
        load_a(t, ph + 1, a1);
        compute_store(t, ph, xc, a0);
        __builtin_amdgcn_sched_barrier(0);
        if (ph + 2 < NP) {
          load_a(t, ph + 2, a0);
        } else if (t + 1 < t_end) {
          load_x(t + 1, xn);
          load_a(t + 1, 0, a0);
        }
        compute_store(t, ph + 1, xc, a1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    for (int t = t_begin; t < t_end; t += 2) {
      tile(t, x0, x1);
      if (t + 1 >= t_end) break;
      tile(t + 1, x1, x0);
    }
  }
}

template <typename T, int NP>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void convt_add(ConvTParams p) {
  convt_tile<T, NP>(p, blockIdx.x);
}

// several independent up-steps in one launch (the engine's schedule: ops of one dependency level
// on the latency path): workgroups [end[k-1], end[k]) run up-step k
struct ConvTGroup {
  ConvTParams p[kConvTGroupMax];
  int end[kConvTGroupMax];
  int n;
};
template <typename T, int NP>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void convt_add_group(
    const ConvTGroup g) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < g.n && b >= g.end[k]) ++k;  // (workgroup-uniform)
  convt_tile<T, NP>(g.p[k], b - (k ? g.end[k - 1] : 0));
}

template <typename T, int NP>
static int launch_group_t(const ConvTGroup& g, hipStream_t s) {
  constexpr int lds = lds_bytes<NP>();
  if (int r = ensure_lds<convt_add_group<T, NP>>(lds)) return r;
  auto k = convt_add_group<T, NP>;
  hipLaunchKernelGGL(k, dim3(g.end[g.n - 1]), dim3(NT), lds, s, g);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename T, int NP>
static int launch_t(const ConvTParams& p, hipStream_t s) {
  auto k = convt_add<T, NP>;
  constexpr int lds = lds_bytes<NP>();
  if (int r = ensure_lds<convt_add<T, NP>>(lds)) return r;
  const int groups = p.s * p.s / NP;
  hipLaunchKernelGGL(k, dim3(groups * p.nchunks), dim3(NT), lds, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace convt

bool convt_supported(int cin, int cout, int src_ldc, int add_ldc, int out_ldc) {
  return cin == convt::KJ * 16 && cout == convt::C && src_ldc % 8 == 0 && add_ldc % 8 == 0 && out_ldc % 8 == 0;
}

// one resident 8-wave workgroup per CU over the whole launch, the tiles split evenly over the
// waves of each phase group (round-2 schedule: whole tiles-per-wave counts, which left 56 of 256
// CUs idle on the 120x160 up-steps)
void convt_schedule(ConvTParams& p, int cu_count) {
  const long M = (long)p.B * p.h * p.w;
  const long mt = (M + 31) / 32;
  const long waves_target = (long)convt::NW * cu_count;
  // phase groups of 4 once every wave of the launch gets >= 2 tiles that way
  p.np = (p.s * p.s % convt::NPG == 0 &&
          mt * (p.s * p.s / convt::NPG) >= 2 * waves_target) ? convt::NPG : 1;
  const long groups = (long)p.s * p.s / p.np;
  long chunks = cu_count / groups;                       // workgroups per phase group
  const long need = (mt + convt::NW - 1) / convt::NW;    // no more than one tile per wave's worth
  if (chunks > need) chunks = need;
  if (chunks < 1) chunks = 1;
  p.nchunks = (int)chunks;
  p.tpw = (int)((mt + chunks * convt::NW - 1) / (chunks * convt::NW));  // most tiles any wave runs
}

int convt_workgroups(const ConvTParams& p) { return p.s * p.s / std::max(1, p.np) * p.nchunks; }

int launch_convt_group(const ConvTParams* const* ps, int n, int dtype, hipStream_t s) {
  using namespace convt;
  if (n < 1 || n > kConvTGroupMax) {
    set_error("convt group: 1..kConvTGroupMax up-steps");
    return 1;
  }
  ConvTGroup g{};
  g.n = n;
  int wg = 0;
  for (int k = 0; k < n; ++k) {
    const ConvTParams& p = *ps[k];
    if (p.tpw < 1 || p.nchunks < 1 || p.s < 1 || p.np != ps[0]->np || (p.np != 1 && p.np != NPG)) {
      set_error("convt group: unscheduled or mixed phase groups");
      return 1;
    }
    wg += convt_workgroups(p);
    g.p[k] = p;
    g.end[k] = wg;
  }
  const bool np4 = ps[0]->np == NPG;
  if (dtype == F16) return np4 ? launch_group_t<_Float16, NPG>(g, s) : launch_group_t<_Float16, 1>(g, s);
  if (dtype == BF16) return np4 ? launch_group_t<__bf16, NPG>(g, s) : launch_group_t<__bf16, 1>(g, s);
  set_error("convt: fp16/bf16 only");
  return 1;
}

int launch_convt(const ConvTParams& p, int dtype, hipStream_t s) {
  if (p.tpw < 1 || p.nchunks < 1 || p.s < 1) {
    set_error("convt: not scheduled");
    return 1;
  }
  using namespace convt;
  if (p.np != 1 && p.np != NPG) {
    set_error("convt: bad phase group");
    return 1;
  }
  if (dtype == F16) return p.np == NPG ? launch_t<_Float16, NPG>(p, s) : launch_t<_Float16, 1>(p, s);
  if (dtype == BF16) return p.np == NPG ? launch_t<__bf16, NPG>(p, s) : launch_t<__bf16, 1>(p, s);
  set_error("convt: fp16/bf16 only");
  return 1;
}

}  // namespace tv
