// Memory-bound helper kernels around the conv stack (gfx950).
//  * input staging: NCHW fp32 (Centernet.forward's contract, centernet.py:65) or raw u8 HWC
//    frames with the node's ToTensor + Normalize(ImageNet) fused (centernet_node.py:90-92),
//    written as NHWC with channels zero-padded to one 16-byte chunk per pixel;
//  * the pad_to_match margin: target pixels that the shifted upsample does not cover get the
//    skip tensor alone (dla.py:205-207 zero padding).
#include "common.h"

namespace tv {

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

template <typename T>
__device__ __forceinline__ void write_pixel(T* dst, float r, float g, float b) {
  constexpr int V = 16 / sizeof(T);
  T t[V];
#pragma unroll
  for (int e = 0; e < V; ++e) t[e] = (T)0.0f;
  t[0] = (T)r;
  t[1] = (T)g;
  t[2] = (T)b;
  *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(t);
}

template <typename T>
__global__ void prep_nchw(const float* __restrict__ img, int B, int HW, T* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)B * HW) return;
  size_t b = i / HW, px = i - b * HW;
  const float* base = img + b * 3 * HW + px;
  constexpr int V = 16 / sizeof(T);
  write_pixel<T>(out + i * V, base[0], base[HW], base[2 * HW]);
}

template <typename T>
__global__ void prep_u8(const uint8_t* __restrict__ fr, size_t npix, T* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t* p = fr + i * 3;
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = ((float)p[c] / 255.0f - kMean[c]) / kStd[c];
  constexpr int V = 16 / sizeof(T);
  write_pixel<T>(out + i * V, v[0], v[1], v[2]);
}

template <typename F>
static int dispatch_dtype(int dtype, F&& f) {
  if (dtype == F32) return f((float*)nullptr);
  if (dtype == F16) return f((_Float16*)nullptr);
  return f((__bf16*)nullptr);
}

int launch_prep_nchw(const float* img, int B, int H, int W, void* out, int cpad, int dtype, hipStream_t s) {
  if (cpad * dtype_size(dtype) != 16) { set_error("prep: pixel must be one 16-byte chunk"); return 1; }
  size_t n = (size_t)B * H * W;
  return dispatch_dtype(dtype, [&](auto tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(prep_nchw<T>, dim3((n + 255) / 256), dim3(256), 0, s, img, B, H * W, (T*)out);
    TV_HIP(hipGetLastError());
    return 0;
  });
}

int launch_prep_u8(const uint8_t* frames, int B, int H, int W, void* out, int cpad, int dtype, hipStream_t s) {
  if (cpad * dtype_size(dtype) != 16) { set_error("prep: pixel must be one 16-byte chunk"); return 1; }
  size_t n = (size_t)B * H * W;
  return dispatch_dtype(dtype, [&](auto tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(prep_u8<T>, dim3((n + 255) / 256), dim3(256), 0, s, frames, n, (T*)out);
    TV_HIP(hipGetLastError());
    return 0;
  });
}

// one thread per (target pixel, 16-byte chunk); covered rectangle [y0,y1) x [x0,x1) skipped
__global__ void uncovered_copy(const uint4* __restrict__ add, int add_ldc16, uint4* __restrict__ out,
                               int out_ldc16, int chunks, int B, int tH, int tW, int y0, int y1, int x0, int x1) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)B * tH * tW * chunks;
  if (i >= total) return;
  int c = i % chunks;
  size_t pix = i / chunks;
  int x = pix % tW;
  int y = (pix / tW) % tH;
  if (y >= y0 && y < y1 && x >= x0 && x < x1) return;
  out[pix * out_ldc16 + c] = add[pix * add_ldc16 + c];
}

int launch_uncovered_copy(const void* add, int add_ldc, void* out, int out_ldc, int C, int B, int tH, int tW,
                          int y0, int y1, int x0, int x1, int dtype, hipStream_t s) {
  int es = dtype_size(dtype);
  if ((C * es) % 16 || (add_ldc * es) % 16 || (out_ldc * es) % 16) {
    set_error("uncovered_copy: rows must be whole 16-byte chunks");
    return 1;
  }
  int chunks = C * es / 16;
  size_t total = (size_t)B * tH * tW * chunks;
  hipLaunchKernelGGL(uncovered_copy, dim3((total + 255) / 256), dim3(256), 0, s, (const uint4*)add,
                     add_ldc * es / 16, (uint4*)out, out_ldc * es / 16, chunks, B, tH, tW, y0, y1, x0, x1);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
