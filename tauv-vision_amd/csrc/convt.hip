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
//
// MODE 1 reuses the same machinery for a 1x1 convolution with stride: output pixel (b, oy, ox)
// reads input pixel (b, oy*stride, ox*stride); optional ReLU. MODE 2 is MODE 1 plus a tensor
// added at the output pixel before the ReLU: ResidualBlock's tail relu(bn2(conv2(y)) +
// bn_residual(conv_residual(x))) (dla.py:39-52) when the planner splits the 1x1 residual out of
// conv2's GEMM (conv2 then runs on the 3x3 halo kernel and stores bn2(conv2(y)) unactivated).
#include "conv_common.h"

namespace tv {
namespace convt {

constexpr int NT = 256;        // 4 waves
constexpr int C = 128;         // output channels per phase (4 MFMA row tiles)
constexpr int KJ = 8;          // K = 128 input channels = 8 MFMA k-steps of 16
constexpr int WPITCH = 272;    // LDS weight row pitch (bytes): odd multiple of 16 -> no bank conflicts
constexpr int OFF_B = C * WPITCH;
constexpr int LDS = OFF_B + C * 4;

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

struct Set {
  uint4 x[KJ];   // B operand: input pixel channels 16j + 8*lh .. +8
  uint4 a[8];    // skip chunks (i, m): channels 32i + 16m + 8*lh .. +8 at the target pixel
};

template <typename T, int MODE>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(2, 2))) void convt_add(ConvTParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int phase = blockIdx.x / p.nchunks;
  const int chunk = blockIdx.x - phase * p.nchunks;
  const int py = phase / p.s, px = phase - py * p.s;

  // ---- the phase's weights and bias into LDS (rows n = phase*C + co of the packed [N][Kpad])
  {
    const char* wsrc = reinterpret_cast<const char*>(p.weight) + (size_t)phase * C * p.Kpad * sizeof(T);
    for (int i = tid; i < C * 16; i += NT) {
      const int r = i >> 4, c = i & 15;
      *reinterpret_cast<uint4*>(smem + r * WPITCH + c * 16) =
          *reinterpret_cast<const uint4*>(wsrc + (size_t)r * p.Kpad * sizeof(T) + c * 16);
    }
    float* lb = reinterpret_cast<float*>(smem + OFF_B);
    if (tid < C) lb[tid] = p.bias[phase * C + tid];
  }
  __syncthreads();

  // MODE 0: GEMM rows are input pixels (b, iy, ix); MODE 1: output pixels (b, oy, ox)
  const int hw = MODE == 0 ? p.h * p.w : p.tH * p.tW;
  const int M = p.B * hw;
  const int mt = (M + 31) / 32;
  const int t_begin = (chunk * 4 + wave) * p.tpw;
  const int t_end = min(t_begin + p.tpw, mt);
  if (t_begin >= t_end) return;

  // target element offset (channel 0) of this lane's pixel in tile t, or -1
  auto target = [&](int t) __attribute__((always_inline)) -> long long {
    const int m = t * 32 + l32;
    if (m >= M) return -1;
    if constexpr (MODE != 0) return m;
    const int b = m / hw;
    const int rem = m - b * hw;
    const int iy = rem / p.w, ix = rem - iy * p.w;
    const int Y = iy * p.s + py + p.sy, X = ix * p.s + px + p.sx;
    if (Y >= p.tH || X >= p.tW) return -1;
    return ((long long)(b * p.tH + Y) * p.tW + X);
  };
  auto load = [&](int t, Set& S) __attribute__((always_inline)) {
    const int m = t * 32 + l32;
    size_t sp = (size_t)(m < M ? m : 0);
    if constexpr (MODE != 0) {  // strided 1x1: input pixel (b, oy*stride, ox*stride)
      const int b = (int)sp / hw;
      const int rem = (int)sp - b * hw;
      const int oy = rem / p.tW, ox = rem - oy * p.tW;
      sp = ((size_t)(b * p.h + oy * p.stride)) * p.w + (size_t)ox * p.stride;
    }
    const T* src = reinterpret_cast<const T*>(p.src) + sp * p.src_ldc + 8 * lh;
#pragma unroll
    for (int j = 0; j < KJ; ++j) S.x[j] = gload16(src + 16 * j);
    if constexpr (MODE == 1) return;
    const long long tg = target(t);  // MODE 2: the output pixel itself
    const T* add = reinterpret_cast<const T*>(p.add) + (tg < 0 ? 0 : tg) * p.add_ldc + 8 * lh;
#pragma unroll
    for (int q = 0; q < 8; ++q) S.a[q] = gload16(add + 16 * q);  // q = 2i + m -> channel 16q + 8lh
  };

  const char* wl = smem + l32 * WPITCH + lh * 16;
  const float* lb = reinterpret_cast<const float*>(smem + OFF_B);
  auto compute_store = [&](int t, const Set& S) __attribute__((always_inline)) {
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x16{};
    // weight fragments one k-step at a time (bounded live set: the two register sets, the
    // accumulators and 16 fragment registers)
#pragma unroll
    for (int j = 0; j < KJ; ++j) {
      uint4 wv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = *reinterpret_cast<const uint4*>(wl + i * 32 * WPITCH + j * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i) Mfma<T>::run(wv[i], S.x[j], acc[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    const long long tg = target(t);
    T* out = reinterpret_cast<T*>(p.out) + (tg < 0 ? 0 : tg) * p.out_ldc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float v[2][4];
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int G2 = 2 * m + gg;
          const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + 32 * i + 8 * G2 + 4 * lh);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[gg][e] = acc[i][4 * G2 + e] + bb[e];
        }
        // registers -> 16-byte chunk: lanes 0-31 channels 32i+16m+0..7, lanes 32-63 +8..15
        const unsigned a0 = __float_as_uint(v[0][0]), a1 = __float_as_uint(v[0][1]);
        const unsigned a2 = __float_as_uint(v[0][2]), a3 = __float_as_uint(v[0][3]);
        const unsigned b0 = __float_as_uint(v[1][0]), b1 = __float_as_uint(v[1][1]);
        const unsigned b2 = __float_as_uint(v[1][2]), b3 = __float_as_uint(v[1][3]);
        const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const auto r2 = __builtin_amdgcn_permlane32_swap(a2, b2, false, false);
        const auto r3 = __builtin_amdgcn_permlane32_swap(a3, b3, false, false);
        // lane now holds 8 consecutive channels: (r0[0], r1[0], r2[0], r3[0], r0[1], ..., r3[1])
        const float f[8] = {__uint_as_float(r0[0]), __uint_as_float(r1[0]), __uint_as_float(r2[0]),
                            __uint_as_float(r3[0]), __uint_as_float(r0[1]), __uint_as_float(r1[1]),
                            __uint_as_float(r2[1]), __uint_as_float(r3[1])};
        unsigned o[4];
        if constexpr (MODE != 1) {
          const uint4 sk = S.a[2 * i + m];
          const unsigned sw[4] = {sk.x, sk.y, sk.z, sk.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float u0 = lo_f<T>(sw[e]) + f[2 * e], u1 = hi_f<T>(sw[e]) + f[2 * e + 1];
            if (MODE == 2 && p.act == 1) u0 = fmaxf(u0, 0.0f), u1 = fmaxf(u1, 0.0f);
            o[e] = pack2<T>(u0, u1);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float u0 = f[2 * e], u1 = f[2 * e + 1];
            if (p.act == 1) u0 = fmaxf(u0, 0.0f), u1 = fmaxf(u1, 0.0f);
            o[e] = pack2<T>(u0, u1);
          }
        }
        if (tg >= 0) gstore16(out + 32 * i + 16 * m + 8 * lh, make_uint4(o[0], o[1], o[2], o[3]));
      }
  };

  // one tile ahead, two register sets (loop unrolled by two so the sets stay in registers)
  Set s0, s1;
  load(t_begin, s0);
  for (int t = t_begin; t < t_end; t += 2) {
    if (t + 1 < t_end) load(t + 1, s1);
    compute_store(t, s0);
    if (t + 1 >= t_end) break;
    if (t + 2 < t_end) load(t + 2, s0);
    compute_store(t + 1, s1);
  }
}

template <typename T, int MODE>
static int launch_t(const ConvTParams& p, hipStream_t s) {
  auto k = convt_add<T, MODE>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) {
      set_error(std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
      return 3;
    }
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3((MODE == 0 ? p.s * p.s : 1) * p.nchunks), dim3(NT), LDS, s, p);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace convt

bool convt_supported(int cin, int cout, int src_ldc, int add_ldc, int out_ldc) {
  return cin == convt::KJ * 16 && cout == convt::C && src_ldc % 8 == 0 && add_ldc % 8 == 0 && out_ldc % 8 == 0;
}

// tiles per wave: about 2 resident workgroups (8 waves) per CU over the whole launch, at least 4 tiles per wave
void convt_schedule(ConvTParams& p, int cu_count) {
  if (p.mode != 0) p.s = 1;  // one "phase"
  const long M = (long)p.B * (p.mode != 0 ? (long)p.tH * p.tW : (long)p.h * p.w);
  const long mt = (M + 31) / 32;
  const long waves_target = 2L * 4 * cu_count;  // 2 workgroups x 4 waves per CU
  long per_phase = (waves_target + p.s * p.s - 1) / (p.s * p.s);
  long tpw = (mt + per_phase - 1) / per_phase;
  if (tpw < 4) tpw = 4;
  p.tpw = (int)tpw;
  p.nchunks = (int)((mt + 4 * tpw - 1) / (4 * tpw));
}

int launch_convt(const ConvTParams& p, int dtype, hipStream_t s) {
  if (p.tpw < 1 || p.nchunks < 1 || p.s < 1) {
    set_error("convt: not scheduled");
    return 1;
  }
  using L = int (*)(const ConvTParams&, hipStream_t);
  static const L f16[3] = {convt::launch_t<_Float16, 0>, convt::launch_t<_Float16, 1>, convt::launch_t<_Float16, 2>};
  static const L b16[3] = {convt::launch_t<__bf16, 0>, convt::launch_t<__bf16, 1>, convt::launch_t<__bf16, 2>};
  if (p.mode < 0 || p.mode > 2) {
    set_error("convt: bad mode");
    return 1;
  }
  if (dtype == F16) return f16[p.mode](p, s);
  if (dtype == BF16) return b16[p.mode](p, s);
  set_error("convt: fp16/bf16 only");
  return 1;
}

}  // namespace tv
