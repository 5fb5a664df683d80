// Diagnostic C-ABI entry points (include/tauv_vision_amd.h, "Diagnostics"): single kernels driven
// directly, for the GPU tests that pin them to identities the reference implies. Not on the
// product path (synchronous, allocate per call).
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "common.h"
#include "../../include/tauv_vision_amd.h"

namespace {

uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

void put(std::vector<uint8_t>& buf, size_t i, float v, int dtype) {
  if (dtype == tv::F32) {
    std::memcpy(buf.data() + 4 * i, &v, 4);
  } else if (dtype == tv::F16) {
    const _Float16 h = (_Float16)v;
    std::memcpy(buf.data() + 2 * i, &h, 2);
  } else {
    const uint16_t b = to_bf16(v);
    std::memcpy(buf.data() + 2 * i, &b, 2);
  }
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

namespace tv {

// DeformConv2d(x, offset, sigmoid(mask)) (torchvision semantics as used by DeformConv.forward,
// centerpoint_dla.py:389-391; 3x3, stride 1, pad 1) + bias + activation, as the engine runs it:
// variant 0 = fused dcn_gemm (32-channel k-steps), 1 = fused dcn_gemm64 (tile by size),
// 2 = dcn_gemm64 with 64-pixel tiles, 3 = unfused (dcn_sample column tensor + implicit GEMM: the
// fp32 path), 4 = dcn_win (C == N == 64), 5 = dcn_gemm64d (gathers two k-steps ahead). weight: host fp32 [N][C][3][3] (PyTorch layout), K packed tap-major as the engine does.
int diag_dcn_conv(const void* x, const void* om, int B, int H, int W, int C, int om_ldc, const float* weight,
                  const float* bias, int N, int act, int dtype, int variant, void* out, hipStream_t s) {
  if (!x || !om || !weight || !bias || !out || B < 1 || H < 1 || W < 1 || C < 1 || N < 1 || om_ldc < 27 ||
      variant < 0 || variant > 8 || dtype < F32 || dtype > BF16 || act < 0 || act > 2) {
    set_error("diag_dcn_conv: bad argument");
    return TV_EINVAL;
  }
  if (dtype == F32 && variant != 3) {
    set_error("diag_dcn_conv: the fused kernels are fp16/bf16 (fp32 runs variant 3)");
    return TV_EINVAL;
  }
  const int esz = dtype_size(dtype);
  const int BK = 128 / esz;  // one 128-byte k-step
  const int K = 9 * C;
  const int ksteps = (K + BK - 1) / BK;
  const int Kpad = ksteps * BK;
  const int Npad = (N + 127) / 128 * 128;
  std::vector<uint8_t> hw((size_t)Npad * Kpad * esz, 0);
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < C; ++c)
      for (int t = 0; t < 9; ++t) put(hw, (size_t)n * Kpad + (size_t)t * C + c, weight[((size_t)n * C + c) * 9 + t], dtype);
  std::vector<float> hb(Npad, 0.f);
  std::memcpy(hb.data(), bias, N * sizeof(float));
  DevBuf dw, db, dcols, dpar, dzero, dslab, dcnt;
  TV_HIP(hipMalloc(&dw.p, hw.size()));
  TV_HIP(hipMemcpy(dw.p, hw.data(), hw.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc(&db.p, hb.size() * 4));
  TV_HIP(hipMemcpy(db.p, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  int rc = 0;
  if (variant != 3) {
    DcnParams q{};
    q.x = x;
    q.B = B;
    q.H = H;
    q.W = W;
    q.C = C;
    q.ldx = C;
    q.om = om;
    q.om_ldc = om_ldc;
    q.w = dw.p;
    q.Kpad = Kpad;
    q.bias = (const float*)db.p;
    q.act = act;
    q.out = out;
    q.out_ldc = N;
    q.N = N;
    if (variant >= 1 && C % 64) {
      set_error("diag_dcn_conv: dcn_gemm64 needs C % 64 == 0");
      return TV_EINVAL;
    }
    if (variant == 4 && !dcn_win_supported(q)) {
      set_error("diag_dcn_conv: dcn_win needs C == N == 64");
      return TV_EINVAL;
    }
    int dev = 0, cus = 0;
    TV_HIP(hipGetDevice(&dev));
    TV_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int mode = variant == 4 ? 3 : variant;
    if (variant >= 6) {  // dcn_gemm64 on 64-pixel tiles, split-K over 3 / 4 / 9 tap ranges
      mode = 2;
      q.ksplit = variant == 6 ? 3 : variant == 7 ? 4 : 9;
      const long units = ((long)B * H * W + 63) / 64 * (N / (N % 128 == 0 ? 128 : 64));
      TV_HIP(hipMalloc(&dslab.p, (size_t)dcn_split_floats(q, mode, q.ksplit) * sizeof(float)));
      TV_HIP(hipMalloc(&dcnt.p, (size_t)units * sizeof(unsigned)));
      TV_HIP(hipMemset(dcnt.p, 0, (size_t)units * sizeof(unsigned)));
      q.slab = (float*)dslab.p;
      q.cnt = (unsigned*)dcnt.p;
    }
    rc = launch_dcn_gemm(q, dtype, mode, cus, s);
  } else {
    const size_t cols_bytes = (size_t)B * H * W * K * esz;
    TV_HIP(hipMalloc(&dcols.p, cols_bytes));
    TV_HIP(hipMalloc(&dzero.p, 256));
    TV_HIP(hipMemset(dzero.p, 0, 256));
    rc = launch_dcn_sample(x, B, H, W, C, om, om_ldc, dcols.p, dtype, s);
    if (!rc) {
      ConvParams p{};
      p.seg[0] = ConvSegment{dcols.p, H, W, K, K, 1, 1, 1, 0, 0, ksteps, 0};
      p.nseg = 1;
      p.Ho = H;
      p.Wo = W;
      p.M = B * H * W;
      p.N = N;
      p.Kpad = Kpad;
      p.weight = dw.p;
      p.bias = (const float*)db.p;
      p.act = act;
      p.out = out;
      p.out_ldc = N;
      p.mtiles = (p.M + 127) / 128;
      p.ntiles = Npad / 128;
      p.zero = dzero.p;
      TV_HIP(hipMalloc(&dpar.p, sizeof(ConvParams)));
      TV_HIP(hipMemcpy(dpar.p, &p, sizeof(ConvParams), hipMemcpyHostToDevice));
      rc = launch_conv(p, (const ConvParams*)dpar.p, out, dtype, 0, 0, s);
    }
  }
  if (rc) return rc == TV_EHIP ? rc : TV_EINVAL;
  TV_HIP(hipStreamSynchronize(s));  // the staging buffers are freed on return
  return TV_OK;
}

// Root-style 1x1 conv (dla.py:58-76: Conv2d over torch.cat(children) + bias + activation) on the
// streaming kernel the engine uses for stride-1 1x1 layers (conv1x1.hip): nseg inputs of M pixels,
// segment k compute-dtype [M][ldc[k]] with C[k] channels; weight host fp32 [N][sum C] (the
// concatenated input channels in segment order), bias host fp32 [N]; out compute-dtype [M][out_ldc].
// Packed as the engine packs a Root: segment k's channels at k-step kbase[k] (128-byte k-steps).
int diag_conv1x1(const void* const* src, const int* C, const int* ldc, int nseg, int M, const float* weight,
                 const float* bias, int N, int act, int dtype, void* out, int out_ldc, hipStream_t s) {
  if (!src || !C || !ldc || !weight || !bias || !out || nseg < 1 || nseg > kMaxSeg || M < 1 || N < 1 || act < 0 ||
      act > 2 || (dtype != F16 && dtype != BF16)) {
    set_error("diag_conv1x1: bad argument");
    return TV_EINVAL;
  }
  const int esz = dtype_size(dtype);
  const int BK = 128 / esz;
  ConvParams p{};
  int kbase = 0, ctot = 0;
  for (int k = 0; k < nseg; ++k) {
    if (!src[k] || C[k] < 1 || ldc[k] < C[k]) {
      set_error("diag_conv1x1: bad segment");
      return TV_EINVAL;
    }
    const int ks = (C[k] + BK - 1) / BK;
    p.seg[k] = ConvSegment{src[k], 1, M, C[k], ldc[k], 1, 1, 1, 0, 0, ks, kbase};
    kbase += ks;
    ctot += C[k];
  }
  const int Kpad = kbase * BK;
  const int Npad = (N + 127) / 128 * 128;
  std::vector<uint8_t> hw((size_t)Npad * Kpad * esz, 0);
  for (int n = 0; n < N; ++n) {
    int c0 = 0;
    for (int k = 0; k < nseg; ++k) {
      for (int c = 0; c < C[k]; ++c)
        put(hw, (size_t)n * Kpad + (size_t)p.seg[k].kbase * BK + c, weight[(size_t)n * ctot + c0 + c], dtype);
      c0 += C[k];
    }
  }
  std::vector<float> hb(Npad, 0.f);
  std::memcpy(hb.data(), bias, N * sizeof(float));
  p.nseg = nseg;
  p.Ho = 1;
  p.Wo = M;
  p.M = M;
  p.N = N;
  p.Kpad = Kpad;
  p.act = act;
  p.out = out;
  p.out_ldc = out_ldc;
  if (!conv1x1_stream_supported(p, esz)) {
    set_error("diag_conv1x1: shape not supported by conv1x1_stream");
    return TV_EINVAL;
  }
  DevBuf dw, db, dpar;
  TV_HIP(hipMalloc(&dw.p, hw.size()));
  TV_HIP(hipMemcpy(dw.p, hw.data(), hw.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc(&db.p, hb.size() * 4));
  TV_HIP(hipMemcpy(db.p, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  p.weight = dw.p;
  p.bias = (const float*)db.p;
  TV_HIP(hipMalloc(&dpar.p, sizeof(ConvParams)));
  TV_HIP(hipMemcpy(dpar.p, &p, sizeof(ConvParams), hipMemcpyHostToDevice));
  int dev = 0, ncu = 256;
  TV_HIP(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  const int rc = launch_conv1x1_stream(p, (const ConvParams*)dpar.p, dtype, ncu, s);
  if (rc) return rc == TV_EHIP ? rc : TV_EINVAL;
  TV_HIP(hipStreamSynchronize(s));  // the staging buffers are freed on return
  return TV_OK;
}

// One conv through the one-shot small-level kernel (conv_burst.hip), packed as the engine packs a
// multi-segment conv: segment k = a kxk (k = 1 or 3, pad k / 2) conv at `stride` over
// src[k] (compute dtype NHWC [B, H, W, ldc], C channels); geom[6 k ..] = H, W, C, ldc, k, stride;
// weight host fp32 [N][K], K = segment-major, tap-major, channel-minor; bias host fp32 [N];
// out compute dtype [B, Ho, Wo, out_ldc].
int diag_conv_burst(const void* const* src, const int* geom, int nseg, int B, int Ho, int Wo, const float* weight,
                    const float* bias, int N, int act, int dtype, void* out, int out_ldc, hipStream_t s) {
  if (!src || !geom || !weight || !bias || !out || nseg < 1 || nseg > kBurstMaxSeg || B < 1 || Ho < 1 || Wo < 1 ||
      N < 1 || act < 0 || act > 2 || (dtype != F16 && dtype != BF16)) {
    set_error("diag_conv_burst: bad argument");
    return TV_EINVAL;
  }
  const int BK = 64;
  ConvParams p{};
  int kbase = 0;
  std::vector<int> koff(nseg);
  int ktot = 0;
  for (int k = 0; k < nseg; ++k) {
    const int* g = geom + 6 * k;
    const int H = g[0], W = g[1], C = g[2], ldc = g[3], kk = g[4], st = g[5];
    if (!src[k] || H < 1 || W < 1 || C < 1 || ldc < C || (kk != 1 && kk != 3) || st < 1) {
      set_error("diag_conv_burst: bad segment");
      return TV_EINVAL;
    }
    const int ks = (kk * kk * C + BK - 1) / BK;
    p.seg[k] = ConvSegment{src[k], H, W, C, ldc, kk, kk, st, kk / 2, kk / 2, ks, kbase};
    koff[k] = ktot;
    ktot += kk * kk * C;
    kbase += ks;
  }
  const int Kpad = kbase * BK;
  const int Npad = (N + 127) / 128 * 128;
  std::vector<uint8_t> hw((size_t)Npad * Kpad * 2, 0);
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < nseg; ++k) {
      const int kk = geom[6 * k + 4], C = geom[6 * k + 2];
      for (int t = 0; t < kk * kk * C; ++t)
        put(hw, (size_t)n * Kpad + (size_t)p.seg[k].kbase * BK + t, weight[(size_t)n * ktot + koff[k] + t], dtype);
    }
  std::vector<float> hb(Npad, 0.f);
  std::memcpy(hb.data(), bias, N * sizeof(float));
  p.nseg = nseg;
  p.Ho = Ho;
  p.Wo = Wo;
  p.M = B * Ho * Wo;
  p.N = N;
  p.Kpad = Kpad;
  p.act = act;
  p.out = out;
  p.out_ldc = out_ldc;
  DevBuf dw, db, dwb;
  TV_HIP(hipMalloc(&dw.p, hw.size()));
  TV_HIP(hipMemcpy(dw.p, hw.data(), hw.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc(&db.p, hb.size() * 4));
  TV_HIP(hipMemcpy(db.p, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  p.weight = dw.p;
  p.bias = (const float*)db.p;
  BurstParams bp{};
  if (!conv_burst_plan(p, B, &bp)) {
    set_error("diag_conv_burst: layer not representable by conv_burst");
    return TV_EINVAL;
  }
  TV_HIP(hipMalloc(&dwb.p, conv_burst_weight_bytes(bp)));
  int rc = conv_burst_repack(dw.p, Kpad, 2, bp, dwb.p, s);
  if (!rc) {
    bp.w = dwb.p;
    const BurstParams* pp = &bp;
    rc = launch_conv_burst(&pp, 1, dtype, s);
  }
  if (rc) return rc == TV_EHIP ? rc : TV_EINVAL;
  TV_HIP(hipStreamSynchronize(s));
  return TV_OK;
}

// conv_burst_plan() for a layer geometry, host only (no device memory, no launch): geom as
// diag_conv_burst; out[0..3] = representable (1 / 0), the launch's dynamic LDS bytes, the extent of
// the kernel's LDS accesses (conv_burst_lds_extent: <= the former whenever representable) and the
// LDS bytes the layer's staging would need (set even when the plan refuses it).
int diag_burst_plan(const int* geom, int nseg, int B, int Ho, int Wo, int N, int* out) {
  if (!geom || !out || nseg < 1 || nseg > kBurstMaxSeg || B < 1 || Ho < 1 || Wo < 1 || N < 1) {
    set_error("diag_burst_plan: bad argument");
    return TV_EINVAL;
  }
  const int BK = 64;
  static const char dummy[16] = {};
  ConvParams p{};
  int kbase = 0;
  for (int k = 0; k < nseg; ++k) {
    const int* g = geom + 6 * k;
    const int H = g[0], W = g[1], C = g[2], ldc = g[3], kk = g[4], st = g[5];
    if (H < 1 || W < 1 || C < 1 || ldc < C || (kk != 1 && kk != 3) || st < 1) {
      set_error("diag_burst_plan: bad segment");
      return TV_EINVAL;
    }
    const int ks = (kk * kk * C + BK - 1) / BK;
    p.seg[k] = ConvSegment{dummy, H, W, C, ldc, kk, kk, st, kk / 2, kk / 2, ks, kbase};
    kbase += ks;
  }
  p.nseg = nseg;
  p.Ho = Ho;
  p.Wo = Wo;
  p.M = B * Ho * Wo;
  p.N = N;
  p.Kpad = kbase * BK;
  p.act = 1;
  p.out = (void*)dummy;
  p.out_ldc = (N + 7) / 8 * 8;
  BurstParams bp{};
  const bool ok = conv_burst_plan(p, B, &bp);
  out[0] = ok ? 1 : 0;
  out[1] = ok ? bp.lds : 0;
  out[2] = ok ? bp.lds_end : 0;
  // the staging the layer would need (what the plan compares with the 160 KiB LDS)
  int need = 0;
  const int out_rows = std::min(Ho, (64 + Wo - 1) / Wo + 1);
  for (int k = 0; k < nseg; ++k) {
    const int* g = geom + 6 * k;
    const int npix = g[4] == 3 ? (out_rows + 2) * (Wo + 2) : 64;
    need += ((g[2] + 127) / 128 * npix * 17 + 63) / 64 * 1024;
  }
  out[3] = need + 256;
  return TV_OK;
}

// One ConvTranspose2d(3, stride 2, padding 1, output_padding 1) + bias + activation through convt3.hip
// (the engine's kernel for the protonet up-sampling, masknet.py:21,33): src compute dtype NHWC
// [B, H, W, ldc] (C channels); weight host fp32 [C][N][3][3] (nn.ConvTranspose2d layout); bias host
// fp32 [N]; out compute dtype NHWC [B, 2H, 2W, out_ldc]; (tw, tr) the input tile (0: the launch's choice).
int diag_convt3(const void* src, int B, int H, int W, int C, int ldc, const float* weight, const float* bias, int N,
                int act, int dtype, int tw, int tr, void* out, int out_ldc, hipStream_t s) {
  if (!src || !weight || !bias || !out || B < 1 || H < 1 || W < 1 || act < 0 || act > 2 ||
      (dtype != F16 && dtype != BF16) || !convt3_supported(C, N, ldc, out_ldc, H, W, 2)) {
    set_error("diag_convt3: bad argument or shape not supported by convt3");
    return TV_EINVAL;
  }
  std::vector<uint8_t> hw(convt3_weight_bytes(C, N));
  convt3_pack(weight, C, N, dtype, hw.data());
  DevBuf dw, db;
  TV_HIP(hipMalloc(&dw.p, hw.size()));
  TV_HIP(hipMemcpy(dw.p, hw.data(), hw.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc(&db.p, (size_t)N * 4));
  TV_HIP(hipMemcpy(db.p, bias, (size_t)N * 4, hipMemcpyHostToDevice));
  ConvT3Params p{};
  p.src = src;
  p.B = B;
  p.H = H;
  p.W = W;
  p.C = C;
  p.ldc = ldc;
  p.w = dw.p;
  p.bias = (const float*)db.p;
  p.act = act;
  p.out = out;
  p.out_ldc = out_ldc;
  p.N = N;
  p.tw = tw;
  p.tr = tr;
  int dev = 0, ncu = 256;
  TV_HIP(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  const int rc = launch_convt3(p, dtype, ncu, s);
  if (rc) return rc == TV_EHIP ? rc : TV_EINVAL;
  TV_HIP(hipStreamSynchronize(s));  // the staging buffers are freed on return
  return TV_OK;
}

// One narrow-channel 3x3 pad-1 conv + bias + activation through conv_small.hip (the engine's kernel
// for DLA-34's full-resolution base levels, centerpoint_dla.py:242-246): weight host fp32
// [N][C][3][3] packed as the engine packs it ([N][Kpad], K tap-major, channel-minor); halo selects
// the LDS-halo variant.
int diag_conv_small(const void* src, int B, int H, int W, int C, int ldc, const float* weight, const float* bias,
                    int N, int stride, int act, int dtype, int halo, void* out, int out_ldc, hipStream_t s) {
  if (!src || !weight || !bias || !out || B < 1 || H < 1 || W < 1 || act < 0 || act > 2 || (stride != 1 && stride != 2) ||
      (dtype != F16 && dtype != BF16) || !conv_small_supported(C, N, stride, ldc, out_ldc) || out_ldc < N) {
    set_error("diag_conv_small: bad argument or shape not supported by conv_small");
    return TV_EINVAL;
  }
  const int Kpad = (9 * C + 63) / 64 * 64;
  std::vector<uint8_t> hw((size_t)N * Kpad * 2, 0);
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < C; ++c)
      for (int t = 0; t < 9; ++t) put(hw, (size_t)n * Kpad + t * C + c, weight[((size_t)n * C + c) * 9 + t], dtype);
  ConvParams p{};
  p.seg[0] = ConvSegment{src, H, W, C, ldc, 3, 3, stride, 1, 1, Kpad / 64, 0};
  p.nseg = 1;
  p.Ho = (H - 1) / stride + 1;
  p.Wo = (W - 1) / stride + 1;
  p.M = B * p.Ho * p.Wo;
  p.N = N;
  p.Kpad = Kpad;
  p.act = act;
  p.out = out;
  p.out_ldc = out_ldc;
  DevBuf dw, db, dp;
  TV_HIP(hipMalloc(&dw.p, hw.size()));
  TV_HIP(hipMemcpy(dw.p, hw.data(), hw.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc(&db.p, (size_t)N * 4));
  TV_HIP(hipMemcpy(db.p, bias, (size_t)N * 4, hipMemcpyHostToDevice));
  p.weight = dw.p;
  p.bias = (const float*)db.p;
  TV_HIP(hipMalloc(&dp.p, sizeof(ConvParams)));
  TV_HIP(hipMemcpy(dp.p, &p, sizeof(ConvParams), hipMemcpyHostToDevice));
  int dev = 0, ncu = 256;
  TV_HIP(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  const int rc = launch_conv_small(p, (const ConvParams*)dp.p, dtype, ncu, halo, s);
  if (rc) return rc == TV_EHIP ? rc : TV_EINVAL;
  TV_HIP(hipStreamSynchronize(s));
  return TV_OK;
}

}  // namespace tv
