// CenterpointDLA34 bandwidth kernels (gfx950): the non-GEMM ops of the DLA-34 network
// (src/tauv_vision/centernet/model/backbones/centerpoint_dla.py). All NHWC, one thread per
// 16-byte channel chunk of an output pixel, so a wave's loads and stores are whole 64-lane
// runs of contiguous 16-byte vectors; arithmetic in fp32, one rounding to the compute dtype.
//   maxpool2_ceil  MaxPool2d(2, 2, ceil_mode=True)               (Tree.downsample, :199-200)
//   dcn_sample     DCNv2 columns: bilinear sample x sigmoid(mask) (DeformConv.forward, :386-392;
//                  torchvision deform_conv2d semantics, see oracle/ref_dla34.py)
//   dwconvt_add    depthwise ConvTranspose2d(2f, stride f, pad f/2, groups = C, no bias)
//                  + pad_to_match + add                           (IDAUp.forward, :453-460)
// The GEMM that contracts the DCN columns with the DeformConv2d weight (K = 9 * C) runs on the
// implicit-GEMM MFMA kernels (conv.hip / conv_pipe.hip) as a 1x1 conv over the column tensor.
#include "common.h"

namespace tv {
namespace dla {

template <typename T>
struct Vec {
  static constexpr int N = 16 / sizeof(T);
  float v[N];
};

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, Vec<T>& o) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) o.v[i] = (float)e[i];
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const Vec<T>& o) {
  uint4 u;
  T* e = reinterpret_cast<T*>(&u);
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) e[i] = (T)o.v[i];
  *reinterpret_cast<uint4*>(p) = u;
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool2_ceil(const T* __restrict__ src, int B, int H, int W, int C,
                                                     T* __restrict__ out, int Ho, int Wo) {
  constexpr int V = Vec<T>::N;
  const int nq = C / V;
  const unsigned total = (unsigned)B * Ho * Wo * nq;  // < 2^31 (checked by the launcher)
  {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    // 32-bit index math: 64-bit division is a long software sequence on CDNA
    const unsigned q = i % (unsigned)nq;
    const unsigned pix = i / (unsigned)nq;
    const unsigned ox = pix % (unsigned)Wo;
    const unsigned r = pix / (unsigned)Wo;
    const unsigned oy = r % (unsigned)Ho;
    const unsigned b = r / (unsigned)Ho;
    Vec<T> m;
#pragma unroll
    for (int e = 0; e < V; ++e) m.v[e] = -__builtin_inff();
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int y = 2 * oy + dy, x = 2 * ox + dx;
        if (y < H && x < W) {  // ceil mode: the last window may hang over the edge
          Vec<T> t;
          load_vec(src + (((size_t)b * H + y) * W + x) * C + q * V, t);
#pragma unroll
          for (int e = 0; e < V; ++e) m.v[e] = fmaxf(m.v[e], t.v[e]);
        }
      }
    store_vec(out + (size_t)pix * C + q * V, m);
  }
}

// One thread per (pixel, tap, channel chunk); chunks of one (pixel, tap) are adjacent lanes, so
// the four corner reads of a wave are contiguous C-channel runs.
template <typename T>
__global__ __launch_bounds__(256) void dcn_sample(const T* __restrict__ x, int B, int H, int W, int C,
                                                  const T* __restrict__ om, int om_ldc, T* __restrict__ cols) {
  constexpr int V = Vec<T>::N;
  const int nq = C / V;
  const unsigned total = (unsigned)B * H * W * 9 * nq;
  {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const unsigned q = i % (unsigned)nq;
    const unsigned r = i / (unsigned)nq;
    const int k = (int)(r % 9u);
    const unsigned pix = r / 9u;
    const int ox = (int)(pix % (unsigned)W);
    const unsigned r2 = pix / (unsigned)W;
    const int oy = (int)(r2 % (unsigned)H);
    const unsigned b = r2 / (unsigned)H;
    const T* o = om + (size_t)pix * om_ldc;
    const float dy = (float)o[2 * k], dx = (float)o[2 * k + 1];
    const float mask = 1.0f / (1.0f + expf(-(float)o[18 + k]));
    // torchvision: y = (oy * stride - pad) + i * dilation + offset_y (stride 1, pad 1)
    const float py = (float)(oy - 1 + k / 3) + dy;
    const float px = (float)(ox - 1 + k % 3) + dx;
    Vec<T> acc;
#pragma unroll
    for (int e = 0; e < V; ++e) acc.v[e] = 0.f;
    if (py > -1.f && py < (float)H && px > -1.f && px < (float)W) {
      const float fy = floorf(py), fx = floorf(px);
      const int y0 = (int)fy, x0 = (int)fx;
      const float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
      const float wt[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
      const T* base = x + (size_t)b * H * W * C + q * V;
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const int yy = y0 + (c4 >> 1), xx = x0 + (c4 & 1);
        if (yy >= 0 && yy <= H - 1 && xx >= 0 && xx <= W - 1) {
          Vec<T> t;
          load_vec(base + ((size_t)yy * W + xx) * C, t);
#pragma unroll
          for (int e = 0; e < V; ++e) acc.v[e] += wt[c4] * t.v[e];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) acc.v[e] *= mask;
    store_vec(cols + (size_t)pix * (9 * C) + k * C + q * V, acc);
  }
}

// weight: fp32 [2f][2f][C] (tap-major, channel-minor). Target pixel (y, x) of the padded and
// cropped map reads the transposed-conv output at (y - sy, x - sx); each output of a k = 2f,
// s = f transposed conv receives exactly the taps ky = (u + p) mod f (+ f), likewise kx.
template <typename T>
__global__ __launch_bounds__(256) void dwconvt_add(const T* __restrict__ src, int B, int h, int w, int C,
                                                   const float* __restrict__ weight, int f, const T* __restrict__ add,
                                                   int add_ldc, T* __restrict__ out, int tH, int tW, int sy, int sx) {
  constexpr int V = Vec<T>::N;
  const int nq = C / V;
  const int p = f / 2, k = 2 * f;
  const int hu = (h - 1) * f - 2 * p + k, wu = (w - 1) * f - 2 * p + k;
  const unsigned total = (unsigned)B * tH * tW * nq;
  {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const unsigned q = i % (unsigned)nq;
    const unsigned pix = i / (unsigned)nq;
    const int x = (int)(pix % (unsigned)tW);
    const unsigned r = pix / (unsigned)tW;
    const int y = (int)(r % (unsigned)tH);
    const unsigned b = r / (unsigned)tH;
    Vec<T> acc;
#pragma unroll
    for (int e = 0; e < V; ++e) acc.v[e] = 0.f;
    const int u = y - sy, v = x - sx;
    if (u >= 0 && u < hu && v >= 0 && v < wu) {
      const int ky0 = (u + p) % f, kx0 = (v + p) % f;
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int ky = ky0 + a * f, ny = u + p - ky;
        if (ny < 0) continue;
        const int iy = ny / f;
        if (iy >= h) continue;
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
          const int kx = kx0 + c2 * f, nx = v + p - kx;
          if (nx < 0) continue;
          const int ix = nx / f;
          if (ix >= w) continue;
          Vec<T> t;
          load_vec(src + (((size_t)b * h + iy) * w + ix) * C + q * V, t);
          const float* wp = weight + (ky * k + kx) * C + q * V;
#pragma unroll
          for (int e = 0; e < V; ++e) acc.v[e] += t.v[e] * wp[e];
        }
      }
    }
    Vec<T> s;
    load_vec(add + (size_t)pix * add_ldc + q * V, s);
#pragma unroll
    for (int e = 0; e < V; ++e) acc.v[e] = acc.v[e] + s.v[e];
    store_vec(out + (size_t)pix * C + q * V, acc);
  }
}

// The same for the power-of-two upsampling factors of DLA-34 (f = 2, 4, 8) and a power-of-two
// chunk count per pixel: shifts and masks instead of the signed divisions by f and the division by
// the chunk count; the skip chunk is loaded before the taps. Same taps in the same order: identical
// results.
template <typename T, int LF>
__global__ __launch_bounds__(256) void dwconvt_add_p2(const T* __restrict__ src, int B, int h, int w, int C,
                                                      const float* __restrict__ weight, const T* __restrict__ add,
                                                      int add_ldc, T* __restrict__ out, int tH, int tW, int sy, int sx,
                                                      int lnq) {
  constexpr int V = Vec<T>::N;
  constexpr int f = 1 << LF, p = f / 2, k = 2 * f;
  const unsigned total = ((unsigned)B * tH * tW) << lnq;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const unsigned q = i & ((1u << lnq) - 1u);
  const unsigned pix = i >> lnq;
  const int x = (int)(pix % (unsigned)tW);
  const unsigned r = pix / (unsigned)tW;
  const int y = (int)(r % (unsigned)tH);
  const unsigned b = r / (unsigned)tH;
  Vec<T> s;
  load_vec(add + (size_t)pix * add_ldc + q * V, s);
  Vec<T> acc;
#pragma unroll
  for (int e = 0; e < V; ++e) acc.v[e] = 0.f;
  const int hu = (h - 1) * f - 2 * p + k, wu = (w - 1) * f - 2 * p + k;
  const int u = y - sy, v = x - sx;
  if (u >= 0 && u < hu && v >= 0 && v < wu) {
    const int ky0 = (u + p) & (f - 1), kx0 = (v + p) & (f - 1);
    const int iy0 = (u + p) >> LF, ix0 = (v + p) >> LF;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int iy = iy0 - a;
      if (iy < 0 || iy >= h) continue;
      const int ky = ky0 + a * f;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int ix = ix0 - c2;
        if (ix < 0 || ix >= w) continue;
        const int kx = kx0 + c2 * f;
        Vec<T> t;
        load_vec(src + (((size_t)b * h + iy) * w + ix) * C + q * V, t);
        const float* wp = weight + (ky * k + kx) * C + q * V;
#pragma unroll
        for (int e = 0; e < V; ++e) acc.v[e] += t.v[e] * wp[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) acc.v[e] = acc.v[e] + s.v[e];
  store_vec(out + (size_t)pix * C + q * V, acc);
}

inline int grid_for(long threads) { return (int)std::max<long>((threads + 255) / 256, 1); }

}  // namespace dla

#define TV_DLA_DISPATCH(dtype, FN, ...)                                          \
  do {                                                                           \
    if ((dtype) == F32) return FN<float>(__VA_ARGS__);                           \
    if ((dtype) == F16) return FN<_Float16>(__VA_ARGS__);                        \
    if ((dtype) == BF16) return FN<__bf16>(__VA_ARGS__);                         \
    set_error("dla34 kernels: bad dtype");                                       \
    return 1;                                                                    \
  } while (0)

namespace {
template <typename T>
int maxpool_t(const void* src, int B, int H, int W, int C, void* out, int Ho, int Wo, hipStream_t s) {
  const long n = (long)B * Ho * Wo * (C / dla::Vec<T>::N);
  hipLaunchKernelGGL(dla::maxpool2_ceil<T>, dim3(dla::grid_for(n)), dim3(256), 0, s, (const T*)src, B, H, W, C,
                     (T*)out, Ho, Wo);
  TV_HIP(hipGetLastError());
  return 0;
}
template <typename T>
int dcn_t(const void* x, int B, int H, int W, int C, const void* om, int om_ldc, void* cols, hipStream_t s) {
  const long n = (long)B * H * W * 9 * (C / dla::Vec<T>::N);
  hipLaunchKernelGGL(dla::dcn_sample<T>, dim3(dla::grid_for(n)), dim3(256), 0, s, (const T*)x, B, H, W, C,
                     (const T*)om, om_ldc, (T*)cols);
  TV_HIP(hipGetLastError());
  return 0;
}
template <typename T>
int dwconvt_t(const void* src, int B, int h, int w, int C, const float* weight, int f, const void* add, int add_ldc,
              void* out, int tH, int tW, int sy, int sx, hipStream_t s) {
  const int nq = C / dla::Vec<T>::N;
  const long n = (long)B * tH * tW * nq;
  const int lnq = __builtin_ctz((unsigned)nq);
  const int lf = (f == 2 || f == 4 || f == 8) && (nq & (nq - 1)) == 0 ? __builtin_ctz((unsigned)f) : 0;
  auto kp = lf == 1 ? dla::dwconvt_add_p2<T, 1> : lf == 2 ? dla::dwconvt_add_p2<T, 2> : dla::dwconvt_add_p2<T, 3>;
  if (lf)
    hipLaunchKernelGGL(kp, dim3(dla::grid_for(n)), dim3(256), 0, s, (const T*)src, B, h, w, C, weight,
                       (const T*)add, add_ldc, (T*)out, tH, tW, sy, sx, lnq);
  else
    hipLaunchKernelGGL(dla::dwconvt_add<T>, dim3(dla::grid_for(n)), dim3(256), 0, s, (const T*)src, B, h, w, C, weight,
                       f, (const T*)add, add_ldc, (T*)out, tH, tW, sy, sx);
  TV_HIP(hipGetLastError());
  return 0;
}
bool chunked(int C, int dtype) { return C > 0 && C % (16 / dtype_size(dtype)) == 0; }
// one thread per 16-byte chunk, 32-bit thread indices
bool fits(long B, long pix, long chunks) { return B * pix * chunks < (1L << 31); }
}  // namespace

int launch_maxpool2(const void* src, int B, int H, int W, int C, void* out, int Ho, int Wo, int dtype, hipStream_t s) {
  if (!chunked(C, dtype) || Ho != (H + 1) / 2 || Wo != (W + 1) / 2 || !fits(B, (long)Ho * Wo, C)) {
    set_error("maxpool2: channels must be whole 16-byte chunks and the output ceil(H/2) x ceil(W/2)");
    return 2;
  }
  TV_DLA_DISPATCH(dtype, maxpool_t, src, B, H, W, C, out, Ho, Wo, s);
}

int launch_dcn_sample(const void* x, int B, int H, int W, int C, const void* om, int om_ldc, void* cols, int dtype,
                      hipStream_t s) {
  if (!chunked(C, dtype) || om_ldc < 27 || !fits(B, (long)H * W, 9L * C)) {
    set_error("dcn_sample: channels must be whole 16-byte chunks, offset/mask tensor >= 27 channels");
    return 2;
  }
  TV_DLA_DISPATCH(dtype, dcn_t, x, B, H, W, C, om, om_ldc, cols, s);
}

int launch_dwconvt_add(const void* src, int B, int h, int w, int C, const float* weight, int f, const void* add,
                       int add_ldc, void* out, int tH, int tW, int sy, int sx, int dtype, hipStream_t s) {
  if (!chunked(C, dtype) || f < 1 || add_ldc < C || sy < 0 || sx < 0 || !fits(B, (long)tH * tW, C)) {
    set_error("dwconvt_add: bad geometry");
    return 2;
  }
  TV_DLA_DISPATCH(dtype, dwconvt_t, src, B, h, w, C, weight, f, add, add_ldc, out, tH, tW, sy, sx, s);
}

}  // namespace tv
