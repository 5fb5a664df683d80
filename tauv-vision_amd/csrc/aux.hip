// Memory-bound helper kernels around the conv stack (gfx950).
//  * input staging: NCHW fp32 (Centernet.forward's contract, centernet.py:65) or raw u8 HWC
//    frames with the node's ToTensor + Normalize(ImageNet) fused (centernet_node.py:90-92),
//    written row-expanded for the 7x7 stem (7 horizontal taps x 3 channels per pixel);
//  * the pad_to_match margin: target pixels that the shifted upsample does not cover get the
//    skip tensor alone (dla.py:205-207 zero padding).
#include "common.h"

#include <algorithm>

// expression order as the reference's torch ops (explicit __fmaf_rn where torch's CPU kernel fuses)
#pragma clang fp contract(off)

namespace tv {

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

// Row-expanded staging for the 7x7 stem (see planner.cpp): output pixel (y, x) holds
// [kx*3 + c] = input(y, x + kx - 3, c) for kx < 7 (zero outside the image), then zeros up to
// `cpad` (a whole number of 16-byte chunks). One thread per output pixel.
template <typename T>
__device__ __forceinline__ void write_expanded(T* dst, const float (&v)[7][3], int cpad) {
  T t[24];
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) t[k * 3 + c] = (T)v[k][c];
#pragma unroll
  for (int j = 21; j < 24; ++j) t[j] = (T)0.0f;
  const uint4* src = reinterpret_cast<const uint4*>(t);
  uint4* out = reinterpret_cast<uint4*>(dst);
  const int chunks = cpad * (int)sizeof(T) / 16;
#pragma unroll
  for (int q = 0; q < 24 * (int)sizeof(T) / 16; ++q)
    if (q < chunks) out[q] = src[q];
}

template <typename T>
__global__ void prep_nchw(const float* __restrict__ img, int B, int H, int W, int cpad, T* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)H * W;
  if (i >= (size_t)B * HW) return;
  const size_t b = i / HW, px = i - b * HW;
  const int x = px % W;
  const float* base = img + b * 3 * HW + (px - x);
  float v[7][3];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int xx = x + k - 3;
    const bool ok = xx >= 0 && xx < W;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[k][c] = ok ? base[c * HW + xx] : 0.0f;
  }
  write_expanded<T>(out + i * cpad, v, cpad);
}

template <typename T>
__global__ void prep_u8(const uint8_t* __restrict__ fr, int B, int H, int W, int cpad, T* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)H * W;
  if (i >= (size_t)B * HW) return;
  const int x = (i % HW) % W;
  const uint8_t* row = fr + (i - x) * 3;
  float v[7][3];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int xx = x + k - 3;
    const bool ok = xx >= 0 && xx < W;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[k][c] = ok ? ((float)row[xx * 3 + c] / 255.0f - kMean[c]) / kStd[c] : 0.0f;
  }
  write_expanded<T>(out + i * cpad, v, cpad);
}

// The node's preprocessing at camera resolution (centernet_node.py:90-92): ToTensor (u8 / 255),
// torchvision 0.15.2 tensor Resize = F.interpolate(bilinear, align_corners=False, antialias=False)
// as torch's CPU kernel evaluates it (upsample_bilinear2d: scale = in / out in fp32, source index
// fma(scale, dst + 0.5, -0.5) clamped at 0, weights l1 = src - floor, l0 = 1 - l1, the row blend
// fma(top, wh0, bottom * wh1) of the column blends fma(left, ww0, right * ww1)), then Normalize
// ((v - mean) / std). One thread per output pixel; fp32 NCHW out (the Centernet.forward input).
__device__ __forceinline__ void lin_index(int d, int in, float scale, int& i0, int& i1, float& l0, float& l1) {
  float src = __fmaf_rn(scale, (float)d + 0.5f, -0.5f);
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
}

__global__ void preprocess_u8(const uint8_t* __restrict__ fr, int B, int Hs, int Ws, int Ho, int Wo, float sh, float sw,
                              float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t hw = (size_t)Ho * Wo;
  if (i >= (size_t)B * hw) return;
  const int b = (int)(i / hw);
  const int p = (int)(i - (size_t)b * hw);
  const int y = p / Wo, x = p - (p / Wo) * Wo;
  int h0, h1, w0, w1;
  float a0, a1, b0, b1;
  lin_index(y, Hs, sh, h0, h1, a0, a1);
  lin_index(x, Ws, sw, w0, w1, b0, b1);
  const uint8_t* f = fr + (size_t)b * Hs * Ws * 3;
  const uint8_t* r0 = f + (size_t)h0 * Ws * 3;
  const uint8_t* r1 = f + (size_t)h1 * Ws * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float A = (float)r0[w0 * 3 + c] / 255.0f, Bv = (float)r0[w1 * 3 + c] / 255.0f;
    const float C = (float)r1[w0 * 3 + c] / 255.0f, D = (float)r1[w1 * 3 + c] / 255.0f;
    const float t0 = __fmaf_rn(A, b0, Bv * b1);
    const float t1 = __fmaf_rn(C, b0, D * b1);
    const float v = __fmaf_rn(t0, a0, t1 * a1);
    out[((size_t)b * 3 + c) * hw + p] = (v - kMean[c]) / kStd[c];
  }
}

int launch_preprocess_u8(const uint8_t* frames, int B, int Hs, int Ws, int Ho, int Wo, float* out, hipStream_t s) {
  if (B < 1 || Hs < 1 || Ws < 1 || Ho < 1 || Wo < 1 || (long)B * Ho * Wo >= (1L << 31)) {
    set_error("preprocess: bad shapes");
    return 1;
  }
  const size_t n = (size_t)B * Ho * Wo;
  hipLaunchKernelGGL(preprocess_u8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, frames, B, Hs, Ws, Ho, Wo,
                     (float)Hs / (float)Ho, (float)Ws / (float)Wo, out);
  TV_HIP(hipGetLastError());
  return 0;
}

template <typename F>
static int dispatch_dtype(int dtype, F&& f) {
  if (dtype == F32) return f((float*)nullptr);
  if (dtype == F16) return f((_Float16*)nullptr);
  return f((__bf16*)nullptr);
}

int launch_prep_nchw(const float* img, int B, int H, int W, void* out, int cpad, int dtype, hipStream_t s) {
  if (cpad != 24) { set_error("prep: row-expanded stem input must have 24 channels"); return 1; }
  size_t n = (size_t)B * H * W;
  return dispatch_dtype(dtype, [&](auto tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(prep_nchw<T>, dim3((n + 255) / 256), dim3(256), 0, s, img, B, H, W, cpad, (T*)out);
    TV_HIP(hipGetLastError());
    return 0;
  });
}

int launch_prep_u8(const uint8_t* frames, int B, int H, int W, void* out, int cpad, int dtype, hipStream_t s) {
  if (cpad != 24) { set_error("prep: row-expanded stem input must have 24 channels"); return 1; }
  size_t n = (size_t)B * H * W;
  return dispatch_dtype(dtype, [&](auto tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(prep_u8<T>, dim3((n + 255) / 256), dim3(256), 0, s, frames, B, H, W, cpad, (T*)out);
    TV_HIP(hipGetLastError());
    return 0;
  });
}

// fp32 NCHW [B, C, H, W] -> NHWC compute dtype (pixel stride ldc): 64 x 64 (channel, pixel)
// tiles transposed through LDS. Reads: 16 B per lane (4 pixels of one channel row, 16 lanes per
// 64-pixel row); writes: 8 channels of one pixel per lane (one 16-byte store for fp16 / bf16, two
// for fp32), 8 lanes per pixel's 64-channel run. (The per-element version — 4-byte reads, 2-byte
// writes — moved the YOLACT fpn[0] input at ~1.4 TB/s.)
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc(const float* __restrict__ img, int C, int HW, int ldc,
                                                    T* __restrict__ out) {
  __shared__ float t[64][65];
  const int b = blockIdx.z, c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
  const float* src = img + (size_t)b * C * HW;
  const bool rows16 = (HW & 3) == 0 && ((uintptr_t)img & 15) == 0;  // every channel row 16-byte aligned
  for (int i = threadIdx.x; i < 64 * 16; i += 256) {
    const int c = i >> 4, q = (i & 15) * 4;
    const float* row = src + (size_t)(c0 + c) * HW + p0 + q;
    float v[4];
    if (c0 + c < C && rows16 && p0 + q + 3 < HW) {
      const float4 f = *reinterpret_cast<const float4*>(row);
      v[0] = f.x, v[1] = f.y, v[2] = f.z, v[3] = f.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (c0 + c < C && p0 + q + j < HW) ? row[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) t[c][q + j] = v[j];
  }
  __syncthreads();
  T* dst = out + (size_t)b * HW * ldc;
  const bool vec = (ldc & 7) == 0 && ((uintptr_t)out & 15) == 0;
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int q = i >> 3, g = (i & 7) * 8;
    if (p0 + q >= HW) continue;
    T o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (T)t[g + j][q];
    T* d = dst + (size_t)(p0 + q) * ldc + c0 + g;
    if (vec && c0 + g + 8 <= C) {
      if constexpr (sizeof(T) == 2) {
        typedef T t2 __attribute__((ext_vector_type(2)));
        uint4 u;
        u.x = __builtin_bit_cast(unsigned, t2{o[0], o[1]});
        u.y = __builtin_bit_cast(unsigned, t2{o[2], o[3]});
        u.z = __builtin_bit_cast(unsigned, t2{o[4], o[5]});
        u.w = __builtin_bit_cast(unsigned, t2{o[6], o[7]});
        *reinterpret_cast<uint4*>(d) = u;
      } else {
        reinterpret_cast<float4*>(d)[0] = make_float4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<float4*>(d)[1] = make_float4(o[4], o[5], o[6], o[7]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + g + j < C) d[j] = o[j];
    }
  }
}

int launch_nchw_to_nhwc(const float* img, int B, int C, int H, int W, void* out, int ldc, int dtype, hipStream_t s) {
  if (B < 1 || C < 1 || (long)H * W >= (1L << 31) || ldc < C || B > 65535) {
    set_error("nchw_to_nhwc: bad shapes");
    return 1;
  }
  const int HW = H * W;
  dim3 grid((HW + 63) / 64, (C + 63) / 64, B);
  return dispatch_dtype(dtype, [&](auto tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(nchw_to_nhwc<T>, grid, dim3(256), 0, s, img, C, HW, ldc, (T*)out);
    TV_HIP(hipGetLastError());
    return 0;
  });
}

// x = leaky_relu(x) in place over n fp32 values (the activation after a fused 1x1 whose channel
// tiles were summed with atomics)
__global__ void leaky_inplace(float4* __restrict__ x, size_t n4) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 v = x[i];
  v.x = fmaxf(v.x, 0.01f * v.x);
  v.y = fmaxf(v.y, 0.01f * v.y);
  v.z = fmaxf(v.z, 0.01f * v.z);
  v.w = fmaxf(v.w, 0.01f * v.w);
  x[i] = v;
}

int launch_leaky_inplace(float* x, size_t n, hipStream_t s) {
  if (n % 4) { set_error("leaky_inplace: n must be a multiple of 4"); return 1; }
  const size_t n4 = n / 4;
  if (!n4) return 0;
  hipLaunchKernelGGL(leaky_inplace, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, (float4*)x, n4);
  TV_HIP(hipGetLastError());
  return 0;
}

// zero n16 16-byte chunks. The engine's zeroing inside a forward (the fused heads' atomic target):
// a kernel, not hipMemsetAsync — a memset node in a captured graph broke every replay after the
// first on this ROCm (HIP's graph packet capture; tools/replay_diag3.py, tests/test_gpu_replay_b1.py)
__global__ void fill_zero16(uint4* __restrict__ p, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

int launch_fill_zero(void* p, size_t bytes, hipStream_t s) {
  if (bytes % 16 || ((uintptr_t)p & 15)) { set_error("fill_zero: 16-byte aligned whole chunks only"); return 1; }
  const size_t n16 = bytes / 16;
  if (!n16) return 0;
  const size_t blocks = std::min<size_t>((n16 + 255) / 256, 4096);
  hipLaunchKernelGGL(fill_zero16, dim3((unsigned)blocks), dim3(256), 0, s, (uint4*)p, n16);
  TV_HIP(hipGetLastError());
  return 0;
}

// the target pixels outside the ConvT's covered rectangle [y0,y1) x [x0,x1) take the skip tensor
// as is (pad_to_match's zero margin + add). One thread per (uncovered pixel, 16-byte chunk): per
// image the band above the rectangle (y0 rows), the band below it (tH - y1 rows) and the columns
// left / right of it in its rows, enumerated in that order — the grid covers only those pixels
// (the covered interior, nearly all of the target, launches nothing)
__global__ void uncovered_copy(const uint4* __restrict__ add, int add_ldc16, uint4* __restrict__ out,
                               int out_ldc16, int chunks, int B, int tH, int tW, int y0, int y1, int x0, int x1,
                               int per_img) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * per_img * chunks) return;
  const int c = (int)(i % chunks);
  const long long q = i / chunks;
  const int b = (int)(q / per_img);
  int r = (int)(q - (long long)b * per_img);
  const int ntop = y0 * tW, nbot = (tH - y1) * tW, side = x0 + (tW - x1);
  int y, x;
  if (r < ntop) {
    y = r / tW;
    x = r - y * tW;
  } else if ((r -= ntop) < nbot) {
    y = y1 + r / tW;
    x = r - (y - y1) * tW;
  } else {
    r -= nbot;
    const int k = r / side, m = r - k * side;
    y = y0 + k;
    x = m < x0 ? m : x1 + (m - x0);
  }
  const size_t pix = ((size_t)b * tH + y) * tW + x;
  out[pix * out_ldc16 + c] = add[pix * add_ldc16 + c];
}

int launch_uncovered_copy(const void* add, int add_ldc, void* out, int out_ldc, int C, int B, int tH, int tW,
                          int y0, int y1, int x0, int x1, int dtype, hipStream_t s) {
  int es = dtype_size(dtype);
  if ((C * es) % 16 || (add_ldc * es) % 16 || (out_ldc * es) % 16) {
    set_error("uncovered_copy: rows must be whole 16-byte chunks");
    return 1;
  }
  y0 = std::max(0, std::min(y0, tH));
  y1 = std::max(y0, std::min(y1, tH));
  x0 = std::max(0, std::min(x0, tW));
  x1 = std::max(x0, std::min(x1, tW));
  const int chunks = C * es / 16;
  const int per_img = tH * tW - (y1 - y0) * (x1 - x0);
  const long long total = (long long)B * per_img * chunks;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(uncovered_copy, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const uint4*)add,
                     add_ldc * es / 16, (uint4*)out, out_ldc * es / 16, chunks, B, tH, tW, y0, y1, x0, x1, per_img);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
