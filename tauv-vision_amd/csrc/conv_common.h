// Helpers shared by the implicit-GEMM conv kernels (gfx950).
#pragma once
#include "common.h"

namespace tv {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kTileM = 128;
constexpr int kTileN = 128;
constexpr int kRowBytes = 128;                       // bytes of K per step, per row
constexpr int kStageBytes = (kTileM + kTileN) * kRowBytes;  // 32 KiB
constexpr int kStageRow = kTileN * 4 + 16;           // fp32 epilogue row stride (bytes)
constexpr int kLdsBytes = (2 * kStageBytes > kTileM * kStageRow) ? 2 * kStageBytes : kTileM * kStageRow;

// byte offset of 16-byte chunk `c` of row `r` in a [rows][128 B] swizzled image
__device__ __forceinline__ int swz(int r, int c) { return r * kRowBytes + ((c ^ ((r >> 1) & 7)) << 4); }

template <typename T> struct Mfma;
template <> struct Mfma<_Float16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x16& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b),
                                                 acc, 0, 0, 0);
  }
};
template <> struct Mfma<__bf16> {
  __device__ static void run(const uint4& a, const uint4& b, f32x16& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                  acc, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  // lane half h holds k = 4*(2j+h) + e for e = 0..3: four K=2 steps per 16-byte chunk
  __device__ static void run(const uint4& a, const uint4& b, f32x16& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

// Global (not flat) 16-byte accesses: pointers read from the parameter block are generic.
__device__ __forceinline__ uint4 gload16(const void* ptr) {
  u32x4 v = *(g_cu32x4*)(ptr);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore16(void* ptr, uint4 v) { *(g_u32x4*)(ptr) = u32x4{v.x, v.y, v.z, v.w}; }

template <typename OutT>
__device__ __forceinline__ void store_chunk(OutT* dst, const float* v);
template <>
__device__ __forceinline__ void store_chunk<float>(float* dst, const float* v) {
  gstore16(dst, make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])));
}
template <typename OutT>
__device__ __forceinline__ void store_chunk(OutT* dst, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    OutT lo = (OutT)v[2 * e], hi = (OutT)v[2 * e + 1];
    w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
  }
  gstore16(dst, make_uint4(w[0], w[1], w[2], w[3]));
}

}  // namespace tv
