// Training targets of the CenterNet loss (reference loss.py:31-135), gfx950.
//
// The reference loops over samples and objects in Python and, per object, evaluates a Gaussian
// over the whole output map (out_h x out_w exp per object) and takes an elementwise max into
// the object's plane. Here one thread owns one cell of one (sample, plane) and walks that
// sample's objects in the reference's order, so every cell's value is the same sequence of
// fp32 operations the reference applies to it:
//   center cell   floor(fl32(fl32(c * in) / ratio))                       (loss.py:52-53, 103-104)
//   Gaussian      exp(fl32(-d2) / fl32(2 sigma^2)), d2 exact integer      (:64-67, 106-114)
//   max           torch.maximum (NaN propagates), nan_to_num at the end   (:70, 131-133)
//   affinity      unit displacement from the owning object's center to the cell, taken where
//                 its length is strictly below the running minimum: the earliest instance
//                 wins ties (:116-129)
// Output planes are written once, coalesced (consecutive threads = consecutive cells). The
// reference's exp is torch's CPU expf; this is the device expf (both ~1 ulp). The affinity's
// sqrt and quotient are correctly rounded here; torch's CPU sqrt (MKL VML vsSqrt) returns one
// ulp below the correctly rounded root for ~0.6% of fp32 inputs (tests/test_targets.py).
#include "common.h"

#include <cfloat>
#include <cmath>

namespace tv {
namespace targets {

__device__ __forceinline__ float maximum_nan(float a, float b) {  // torch.maximum
  return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b);
}
__device__ __forceinline__ float nan_to_num(float v, float nan) {  // torch.nan_to_num(v, nan)
  return v != v ? nan : v == INFINITY ? FLT_MAX : v == -INFINITY ? -FLT_MAX : v;
}
__device__ __forceinline__ int cell(float c, int in_size, int ratio) {
  return (int)floorf(__fdiv_rn(__fmul_rn(c, (float)in_size), (float)ratio));
}
__device__ __forceinline__ float gauss(int x, int y, int cx, int cy, float den) {
  const long long dx = (long long)x - cx, dy = (long long)y - cy;
  const float d2 = (float)(dx * dx + dy * dy);
  return expf(__fdiv_rn(-d2, den));
}

// heatmap [B][L][H][W]: grid (cells / 256, L, B)
__global__ __launch_bounds__(256) void heatmap(const uint8_t* __restrict__ valid, const long long* __restrict__ label,
                                                const float* __restrict__ center, int n_obj, int L, int in_h,
                                                int in_w, int ratio, int H, int W, float den, float* __restrict__ out) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int l = blockIdx.y, b = blockIdx.z;
  if (q >= H * W) return;
  const int y = q / W, x = q - y * W;
  float v = 0.f;
  for (int o = 0; o < n_obj; ++o) {
    const size_t bo = (size_t)b * n_obj + o;
    if (!valid[bo] || label[bo] != l) continue;
    const int cy = cell(center[2 * bo], in_h, ratio), cx = cell(center[2 * bo + 1], in_w, ratio);
    v = maximum_nan(v, gauss(x, y, cx, cy, den));
  }
  out[((size_t)b * L + l) * H * W + q] = nan_to_num(v, 0.f);
}

// keypoint heatmap / affinity weight [B][K][H][W], affinity [B][K][2][H][W]: grid (cells / 256, K, B)
__global__ __launch_bounds__(256) void keypoints(const uint8_t* __restrict__ kvalid, const long long* __restrict__ klabel,
                                                  const float* __restrict__ kcenter, const long long* __restrict__ kobj,
                                                  const float* __restrict__ center, int n_inst, int n_obj, int K,
                                                  int in_h, int in_w, int ratio, int H, int W, float den_h, float den_a,
                                                  float* __restrict__ heat, float* __restrict__ aw,
                                                  float* __restrict__ aff) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y, b = blockIdx.z;
  if (q >= H * W) return;
  const int y = q / W, x = q - y * W;
  // the cell's normalised position, as torch.stack((y / out_h, x / out_w)) forms it
  const float py = __fdiv_rn((float)y, (float)H), px = __fdiv_rn((float)x, (float)W);
  float vh = 0.f, va = 0.f, a0 = 0.f, a1 = 0.f, dist = INFINITY;
  for (int i = 0; i < n_inst; ++i) {
    const size_t bi = (size_t)b * n_inst + i;
    if (!kvalid[bi] || klabel[bi] != k) continue;
    const int cy = cell(kcenter[2 * bi], in_h, ratio), cx = cell(kcenter[2 * bi + 1], in_w, ratio);
    vh = maximum_nan(vh, gauss(x, y, cx, cy, den_h));
    va = maximum_nan(va, gauss(x, y, cx, cy, den_a));
    const size_t bo = (size_t)b * n_obj + (size_t)kobj[bi];
    const float d0 = nan_to_num(__fsub_rn(py, center[2 * bo]), 0.f);
    const float d1 = nan_to_num(__fsub_rn(px, center[2 * bo + 1]), 0.f);
    const float dd = nan_to_num(__fsqrt_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1))), 1.f);
    if (dd < dist) {
      a0 = __fdiv_rn(d0, dd);
      a1 = __fdiv_rn(d1, dd);
    }
    dist = fminf(dist, dd);  // dd is never NaN here
  }
  const size_t plane = (size_t)b * K + k;
  heat[plane * H * W + q] = nan_to_num(vh, 0.f);
  aw[plane * H * W + q] = nan_to_num(va, 0.f);
  aff[(2 * plane) * H * W + q] = nan_to_num(a0, 0.f);
  aff[(2 * plane + 1) * H * W + q] = nan_to_num(a1, 0.f);
}

// fl32(2 sigma^2) with sigma^2 in double, as the Python expression `2 * sigma ** 2` hands it to torch
float den_of(double sigma) { return (float)(2.0 * (sigma * sigma)); }

}  // namespace targets

int launch_train_heatmap(const uint8_t* valid, const long long* label, const float* center, int B, int n_obj, int L,
                         int in_h, int in_w, int ratio, double sigma, float* out, hipStream_t s) {
  if (B < 1 || n_obj < 0 || L < 1 || in_h < 1 || in_w < 1 || ratio < 1 || !out || (n_obj && (!valid || !label || !center))) {
    set_error("generate_heatmap: bad arguments");
    return 1;
  }
  const int H = in_h / ratio, W = in_w / ratio;
  if (H < 1 || W < 1) {
    set_error("generate_heatmap: empty output map");
    return 2;
  }
  if (sigma < 0.1) sigma = 0.1;  // loss.py:59-63
  hipLaunchKernelGGL(targets::heatmap, dim3((H * W + 255) / 256, L, B), dim3(256), 0, s, valid, label, center, n_obj, L,
                     in_h, in_w, ratio, H, W, targets::den_of(sigma), out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_train_keypoints(const uint8_t* kvalid, const long long* klabel, const float* kcenter, const long long* kobj,
                           const float* center, int B, int n_inst, int n_obj, int K, int in_h, int in_w, int ratio,
                           double heat_sigma, double aff_sigma, float* heat, float* aw, float* aff, hipStream_t s) {
  if (B < 1 || n_inst < 0 || n_obj < 0 || K < 1 || in_h < 1 || in_w < 1 || ratio < 1 || !heat || !aw || !aff ||
      (n_inst && (!kvalid || !klabel || !kcenter || !kobj || !center))) {
    set_error("generate_keypoint_heatmap: bad arguments");
    return 1;
  }
  const int H = in_h / ratio, W = in_w / ratio;
  if (H < 1 || W < 1) {
    set_error("generate_keypoint_heatmap: empty output map");
    return 2;
  }
  hipLaunchKernelGGL(targets::keypoints, dim3((H * W + 255) / 256, K, B), dim3(256), 0, s, kvalid, klabel, kcenter, kobj,
                     center, n_inst, n_obj, K, in_h, in_w, ratio, H, W, targets::den_of(heat_sigma),
                     targets::den_of(aff_sigma), heat, aw, aff);
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
