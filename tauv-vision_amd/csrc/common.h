// Shared definitions for the tauv-vision_amd HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
// gfx950 only. The cross-workgroup hand-offs (decode.hip's single-launch select, conv_lat's split-K
// tickets) rely on gfx950's SC1 cache-bit semantics: write-through sc1 stores and L1-bypassing sc1
// loads stand in for a release / acquire pair (MI355X_MICROARCH.md, inter-workgroup visibility).
// On another target they would compile cleanly and could read stale bytes through the L2.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "tauv_vision_amd kernels are written for gfx950 (MI355X) only"
#endif
#include <cstdint>
#include <string>

namespace tv {

enum DType : int { F32 = 0, F16 = 1, BF16 = 2 };

inline int dtype_size(int dt) { return dt == F32 ? 4 : 2; }

// Thread-local error string behind tv_last_error().
void set_error(const std::string& msg);

// Raise kernel K's dynamic-LDS limit to `bytes` once per process. The function-local static is
// initialised under the C++ static-init guard, so concurrent first launches from several threads
// (engines on side streams, callers' threads) set it exactly once; a failure is sticky.
template <auto K>
inline int ensure_lds(int bytes) {
  static const hipError_t e = hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) {
    set_error(std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
    return 3;
  }
  return 0;
}

#define TV_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::tv::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));              \
      return 3; /* TV_EHIP */                                                           \
    }                                                                                   \
  } while (0)

// ---- implicit-GEMM convolution ----------------------------------------------------
// One K-segment of a fused GEMM: a kh x kw convolution (stride, pad) over an NHWC source
// tensor. Several segments sum into one output (channel concat of Root, the 1x1 residual
// branch of ResidualBlock fused into conv2's K).
struct ConvSegment {
  const void* src;  // element (b,y,x,c) at ((b*H + y)*W + x)*ldc + c
  int H, W, C, ldc;
  int kh, kw, stride, pad, pad_w;
  int ksteps;  // ceil(kh*kw*C / BK); BK = 128 bytes of elements
  int kbase;   // first k-step of this segment in the packed weight rows
};

constexpr int kMaxSeg = 8;

// Host-precomputed descriptor of one 128-byte k-step of the pipelined kernel: which source
// tensor and which tap/channel window it reads (one scalar load per k-step in the kernel).
struct KStep {
  const void* src;
  long long off;             // mode 0: element offset of (tap, c0) from the lane's segment base pixel
  int seg, tap, mode;        // mode 0: the k-step lies in one tap; 1: per-lane taps (C < BK)
  int H, W, ldc, stride, pad_h, pad_w, kh, kw;
  int q0, cpt;               // mode 1: first 16-byte chunk (within the segment's K), chunks per tap
  float cpt_inv, kw_inv;     // mode 1: reciprocals for exact small-integer division
};
static_assert(sizeof(KStep) == 80, "KStep layout");

struct ConvParams {
  ConvSegment seg[kMaxSeg];
  int nseg;
  int Ho, Wo, M;        // output grid of the GEMM (M = B*Ho*Wo pixels)
  int N;                // GEMM columns actually stored (multiple of the 16-byte vector)
  int Kpad;             // packed weight row length, elements
  const void* weight;   // [Npad][Kpad] compute dtype
  const float* bias;    // [Npad] fp32 (BN folded)
  int act;              // 0 none, 1 relu, 2 leaky_relu(0.01)
  void* out;            // mode 0: out pixel m at m*out_ldc + out_coff; mode 1: target grid
  int out_ldc, out_coff;
  int mtiles, ntiles;
  // mode 1: non-overlapping ConvTranspose2d (k == s) phase scatter + add, with the
  // pad_to_match shift (dla.py:195-209) folded into the target coordinates.
  int up_s, up_cout;    // scale; output channels per phase (n = phase*up_cout + co)
  int tH, tW, sy, sx;   // target grid and (row, col) shift
  const void* add;      // tensor added at the target pixel (compute dtype)
  int add_ldc;
  const void* zero;     // >= 16 zero bytes: source of padding taps for LDS-DMA loads
  const KStep* ks;      // pipelined kernel: one descriptor per k-step (nks of them)
  int nks;
  // conv3x3 EPI = 1 (stacked heads with the block-diagonal 1x1 heads fused, centernet.py:46-61):
  // N-tile nt's 128 hidden channels feed output columns [head_row0[nt], + head_nrows[nt]) of the
  // caller's fp32 output (pixel stride head_ldc), accumulated with fp32 atomic adds
  const void* head_w;   // [ntiles][8 k-steps][64 lanes][16 B] MFMA A-fragments of the 1x1 weights
  const float* head_b;  // [ntiles][32] 1x1 bias on the first tile of each head, zeros elsewhere
  int head_ldc;
  int head_row0[16], head_nrows[16];
  int head_store;       // 1: every output column written by exactly one tile -> plain stores (no zeroing)
  unsigned long long* dbg;  // diagnostic stamp builds only (conv3x3 TV_C3_EXP == 9): per-wave cycle buckets
  // conv_lat split-K over workgroups: ksplit workgroups per tile each walk a slice of the k-steps,
  // write their fp32 partial tile to slab[tile][slice] (write-through), and the last to arrive
  // (cnt[tile], agent-scope counter, zero before the launch) sums the slices in slice order
  int ksplit;
  float* slab;
  unsigned* cnt;
};

// Pipelined variant (conv_pipe.hip): 256-pixel tiles, LDS-DMA ring; needs ConvParams.ks.
int launch_conv_pipe(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int out_f32, int mode,
                     hipStream_t s, int x3 = 0);
// fp32 weights [Npad][Kpad] -> conv_pipe's X3 copy (x3 launches: fp32 products as three fp16 MFMAs)
int conv_pipe_x3_repack(const void* w, int Npad, int Kpad, void* out, hipStream_t s);
constexpr int kPipeTileM = 256;
// Split-K variant for the small levels (conv_lat.hip): 64-pixel x 128-channel tiles, the k-step
// descriptors split over two 4-wave K groups; ConvParams.mtiles / ntiles from conv_lat_tiles();
// mode-0 k-steps only (every segment's channel count a multiple of 64 / 128 bytes)
int conv_lat_tiles(int M, int N, int* mtiles, int* ntiles);
int launch_conv_lat(const ConvParams& p, const ConvParams* dp, int dtype, hipStream_t s, int x3 = 0);
// One-shot small-level conv (conv_burst.hip): 64 output pixels (raster, one frame) x 32 channels
// per 256-thread workgroup, K split over its 4 waves (<= 20 k-steps of 16 each, weights in
// registers), every input the tile reads staged in LDS at once. Segments: 3x3 / stride 1 / pad 1
// over the output grid, or 1x1 at any stride; 128-channel multiples.
constexpr int kBurstMaxSeg = 3;
constexpr int kBurstGroupMax = 4;  // layers per grouped launch
struct BurstSeg {
  const void* src;
  int H, W, C, ldc;
  int planes;     // C / 128
  int kind;       // 0: 3x3 / s1 / p1 window, 1: 1x1 at `stride`
  int stride;
  int wrow;       // kind 0: window row pitch (pixels) = Wo + 2
  int npix;       // staged pixels per 128-channel plane
  int kbase16;    // first k-step (of 16) of the segment
  int lds_off;    // staging region (bytes)
};
struct BurstParams {
  BurstSeg seg[kBurstMaxSeg];
  int nseg;
  int B, Ho, Wo, tiles_pf, ptiles, ntiles, nk16;
  const void* w;        // conv_burst_repack() copy
  const float* bias;
  int act;
  void* out;
  int out_ldc, out_coff, N;
  int lds, zero_off;    // dynamic LDS bytes; the zero block's offset
  int lds_end;          // conv_burst_lds_extent(): end of the highest LDS byte any access touches (<= lds)
};
struct BurstGroup {
  BurstParams p[kBurstGroupMax];
  int end[kBurstGroupMax];
  int n;
};
// the launch geometry of a conv (p: the engine's ConvParams for a B-frame workspace); false when
// the layer is not representable (strided 3x3, channel counts, LDS)
bool conv_burst_plan(const ConvParams& p, int B, BurstParams* out);
int conv_burst_lds_extent(const BurstParams& p);
size_t conv_burst_weight_bytes(const BurstParams& p);
int conv_burst_repack(const void* w, int Kpad, int esz, const BurstParams& p, void* out, hipStream_t s);
int conv_burst_workgroups(const BurstParams& p);
int launch_conv_burst(const BurstParams* const* ps, int n, int dtype, hipStream_t s);
// streaming stride-1 1x1 conv over concatenated inputs, weights resident in LDS (conv1x1.hip)
bool conv1x1_stream_supported(const ConvParams& p, int esz);
int launch_conv1x1_stream(const ConvParams& p, const ConvParams* dp, int dtype, int cu_count, hipStream_t s);
constexpr int kLatGroupMax = 4;  // layers per grouped conv_lat launch
// independent layers in one launch (hp: host copies for validation, dp: their device copies)
int launch_conv_lat_group(const ConvParams* const* hp, const ConvParams* const* dp, int n, int dtype, hipStream_t s,
                          int x3 = 0);
// fp32 slab floats one conv_lat split-K tile slice needs (64 x 128)
constexpr int kLatSlabFloats = 64 * 128;

// Persistent halo-tile 3x3 / stride 1 / pad 1 kernel (conv3x3.hip), fp16/bf16, 128- or 256-channel
// input (seg[0].C): 512-pixel
// tiles of tw (16 or 32) columns; ConvParams.mtiles = conv3x3_tiles(B, H, W, tw); `grid`
// persistent workgroups (one per CU, a multiple of 8 when >= 8).
constexpr int kConv3MaxN = 2048;
// epi = 0: store the activations; epi = 1: fused 1x1 heads into the fp32 output `out` (head_*)
// res = 1: two segments — seg 0 the 3x3 input, seg 1 a 1x1 conv (stride seg[1].stride) over a
// 128-channel tensor summed into the same accumulators (ResidualBlock conv2 + conv_residual)
// ni = 4: 128-channel tiles; ni = 2: 64-channel half tiles (epi 0 only; p.ntiles still counts
// 128-channel tiles, the grid covers mtiles * ntiles * 2 work units)
// nw = 8: one 512-thread workgroup per CU, 512-pixel tiles; nw = 4: two 256-thread workgroups per
// CU, 256-pixel tiles (epi 0, res 0, 128-channel inputs, <= 256 output channels)
int launch_conv3x3(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid,
                   hipStream_t s, int epi = 0, int res = 0, int ni = 4, int nw = 8);
int conv3x3_tiles(int B, int H, int W, int tw, int nw = 8);
// Persistent halo-tile 3x3 / stride 2 / pad 1 kernel (conv3x3s2.hip), fp16/bf16, 128 -> 128
// channels: 16x32-pixel output tiles; ConvParams.mtiles = conv3x3s2_tiles(B, Ho, Wo), ntiles = 1
int conv3x3s2_tiles(int B, int Ho, int Wo);
size_t conv3x3s2_weight_bytes();
int conv3x3s2_repack(const void* w, int Kpad, int esz, void* out, hipStream_t s);
int launch_conv3x3s2(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int grid, hipStream_t s);
// k-step-major, pre-swizzled weight copy the kernel streams (from the [Npad][Kpad] packing)
// (ncb = input channel blocks of 32: 4 for 128-channel inputs, 8 for 256)
size_t conv3x3_weight_bytes(int ntiles, int res, int ncb);
int conv3x3_repack(const void* w, int Kpad, int esz, int ntiles, int res, int ni, int ncb, int k16, void* out, hipStream_t s);
// whether the conv3x3 instance (epi, res, ni) runs the 16x16x32 body (its weights use that body's swizzle)
int conv3x3_k16(int epi, int res, int ni, int nw);

// p: host copy (grid geometry); dp: the same struct in device memory; out: output base.
int launch_conv(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int out_f32, int mode,
                hipStream_t s);

// Fused DCNv2 (dcn.hip), fp16/bf16: bilinear samples x sigmoid(mask) gathered into the MFMA operand
// tile (no column tensor) x the DeformConv2d weight packed as [Npad][Kpad], K = tap * C + c; bias
// (BN folded) + activation; NHWC
struct DcnParams {
  const void* x;      // input [B, H, W, ldx], C channels used
  int B, H, W, C, ldx;
  const void* om;     // offset / mask conv output [B, H, W, om_ldc]: dy, dx per tap (18), mask logits (9)
  int om_ldc;
  const void* w;      // [Npad][Kpad]
  int Kpad;
  const float* bias;  // [Npad]
  int act;
  void* out;          // [B, H, W, out_ldc], N channels
  int out_ldc, N;
  // split-K (dcn_gemm64 only; ksplit <= 1: off): ksplit workgroups per (pixel tile, channel tile),
  // each over a tap range; fp32 partials meet in slab (dcn_split_floats each), tickets in cnt
  // (one per tile, zero-filled once: the last slice resets its own)
  int ksplit;
  float* slab;
  unsigned* cnt;
};
// dcn_gemm64's tile for a layer as launch_dcn_gemm picks it (BN output channels x PX pixels) and
// the slab floats one split layer needs
void dcn64_tile(const DcnParams& p, int dcn64_mode, int* bn, int* px);
long dcn_split_floats(const DcnParams& p, int dcn64_mode, int ksplit);
bool dcn_gemm_supported(long M, int C, int N, int ldx, int om_ldc, int out_ldc, int Kpad);
// dcn64_mode: 0 dcn_gemm; 1 64-channel k-steps when C % 64 == 0 (dcn_gemm64); 2 the same on 64-pixel
// tiles; 3 the LDS-window kernel (dcn_win) where dcn_win_supported, else as 1; 5 dcn_gemm64d (gathers two
// k-steps ahead, 64-pixel tiles) when C % 64 == 0 and om_ldc is even
int launch_dcn_gemm(const DcnParams& p, int dtype, int dcn64_mode, int cu_count, hipStream_t s);
bool dcn_win_supported(const DcnParams& p);
// targets.hip: training targets of the loss (loss.py:31-135)
int launch_train_heatmap(const uint8_t* valid, const long long* label, const float* center, int B, int n_obj, int L,
                         int in_h, int in_w, int ratio, double sigma, float* out, hipStream_t s);
int launch_train_keypoints(const uint8_t* kvalid, const long long* klabel, const float* kcenter, const long long* kobj,
                           const float* center, int B, int n_inst, int n_obj, int K, int in_h, int in_w, int ratio,
                           double heat_sigma, double aff_sigma, float* heat, float* aw, float* aff, hipStream_t s);
// diag.cpp: one DeformConv2d + bias + activation through a chosen DCN kernel (GPU tests)
int diag_dcn_conv(const void* x, const void* om, int B, int H, int W, int C, int om_ldc, const float* weight,
                  const float* bias, int N, int act, int dtype, int variant, void* out, hipStream_t s);
// diag.cpp: a Root-style 1x1 conv over nseg concatenated inputs through conv1x1_stream (GPU tests)
int diag_conv1x1(const void* const* src, const int* C, const int* ldc, int nseg, int M, const float* weight,
                 const float* bias, int N, int act, int dtype, void* out, int out_ldc, hipStream_t s);
// diag.cpp: one multi-segment conv (3x3 / 1x1 segments) through conv_burst (GPU tests)
int diag_burst_plan(const int* geom, int nseg, int B, int Ho, int Wo, int N, int* out);
int diag_conv_burst(const void* const* src, const int* geom, int nseg, int B, int Ho, int Wo, const float* weight,
                    const float* bias, int N, int act, int dtype, void* out, int out_ldc, hipStream_t s);

// diag.cpp: one narrow-channel 3x3 conv through conv_small (GPU tests)
int diag_conv_small(const void* src, int B, int H, int W, int C, int ldc, const float* weight, const float* bias,
                    int N, int stride, int act, int dtype, int halo, void* out, int out_ldc, hipStream_t s);
// diag.cpp: one ConvTranspose2d(3, s2, p1, op1) + bias + activation through convt3 (GPU tests)
int diag_convt3(const void* src, int B, int H, int W, int C, int ldc, const float* weight, const float* bias, int N,
                int act, int dtype, int tw, int tr, void* out, int out_ldc, hipStream_t s);

// Narrow-channel 3x3 / pad 1 conv (conv_small.hip), fp16/bf16: 16 -> 16/32 and 32 -> 32/64 input ->
// output channels at stride 1 or 2 (DLA-34 base levels), bias + activation, NHWC
bool conv_small_supported(int cin, int cout, int stride, int cin_ldc, int out_ldc);
// halo: 0 = per-lane register gathers, 1 = LDS-halo tiles (input tile staged once by LDS-DMA), one
// tile per workgroup, 2 = LDS-halo tiles on a persistent grid
int launch_conv_small(const ConvParams& p, const ConvParams* dp, int dtype, int cu_count, int halo, hipStream_t s);

// Fused input staging + 7x7 stem conv (stem.hip), fp16/bf16, C0 <= 128 output channels.
struct StemParams {
  const void* input;  // u8 NHWC [B,H,W,3] frames (u8 = 1) or normalised fp32 NCHW [B,3,H,W]
  int u8;
  int B, H, W;
  void* out;          // NHWC compute dtype, pixel stride out_ldc
  int out_ldc, N;
  const void* weight; // stem_weight_bytes() in B-fragment order (stem_fragment_order)
  const float* bias;  // [>= N] fp32, BN folded
};
size_t stem_weight_bytes();
void stem_fragment_order(const uint16_t* w, int Npad, int Kpad, uint16_t* out);
int launch_stem(const StemParams& p, int dtype, int grid, hipStream_t s);

// Fused staging + 7x7 stem + ResidualBlock conv1 (3x3 / stride 2) (stem_s2.hip), fp16/bf16, 128
// channels: writes conv1's activations and the stem at the even pixels (the block's residual input)
struct StemS2Params {
  const void* input;      // u8 NHWC [B,H,W,3] frames (u8 = 1) or normalised fp32 NCHW [B,3,H,W]
  int u8;
  int B, H, W, Ho, Wo;    // Ho = ceil(H / 2), Wo = ceil(W / 2)
  const void* stem_w;     // stem_weight_bytes() in B-fragment order (stem_fragment_order), 128 channels
  const float* stem_bias; // [128] fp32, BN folded
  const void* w1;         // stem_s2_weight_bytes(): conv1 weights in the kernel's k-step order (stem_s2_repack)
  const float* bias1;     // [128] fp32, BN folded
  void* out;              // conv1 + BN + ReLU, NHWC [B,Ho,Wo,out_ldc]
  int out_ldc;
  void* res;              // stem(2y, 2x), NHWC [B,Ho,Wo,res_ldc]
  int res_ldc;
  unsigned long long* dbg;  // stamp builds (TV_C3_EXP=9) only: 8 cycle buckets per wave, else null
};
int stem_s2_tiles(int B, int Ho, int Wo);
size_t stem_s2_weight_bytes();
int stem_s2_repack(const void* w, int Kpad, int esz, void* out, hipStream_t s);
int launch_stem_s2(const StemS2Params& p, int dtype, int cu_count, hipStream_t s);

// ConvTranspose2d(k = s) + pad_to_match + skip add (convt.hip), fp16/bf16, 128 -> 128 channels.
struct ConvTParams {
  const void* src;    // low-res input NHWC [B,h,w,*]
  int h, w, src_ldc;
  const void* weight; // packed [s*s*128][Kpad] (row = phase*128 + co)
  int Kpad;
  const float* bias;  // [s*s*128]
  const void* add;    // skip tensor [B,tH,tW,*]
  int add_ldc;
  void* out;          // [B,tH,tW,*]
  int out_ldc;
  int B, s, tH, tW, sy, sx;
  int tpw, nchunks, np;  // schedule (convt_schedule): tiles per wave, workgroups per phase group, phases per group
};
bool convt_supported(int cin, int cout, int src_ldc, int add_ldc, int out_ldc);
void convt_schedule(ConvTParams& p, int cu_count);
int launch_convt(const ConvTParams& p, int dtype, hipStream_t s);
constexpr int kConvTGroupMax = 4;  // up-steps per grouped convt launch
int convt_workgroups(const ConvTParams& p);
int launch_convt_group(const ConvTParams* const* ps, int n, int dtype, hipStream_t s);

// ConvTranspose2d(3, stride 2, padding 1, output_padding 1) + bias + activation, all four output
// phases over one shared input halo (convt3.hip), fp16/bf16: the YOLACT protonet up-sampling.
struct ConvT3Params {
  const void* src;    // NHWC [B, H, W, ldc], C channels used
  int B, H, W, C, ldc;
  const void* w;      // convt3_pack() fragments
  const float* bias;  // [N]
  int act;
  void* out;          // NHWC [B, 2H, 2W, out_ldc], N channels
  int out_ldc, N;
  int tw, tr;         // input tile (columns, rows); 0: convt3_tile()'s choice
};
void convt3_tile(int H, int W, int* tw, int* tr);
bool convt3_supported(int C, int N, int ldc, int out_ldc, int H, int W, int esz);
size_t convt3_weight_bytes(int C, int N);
// host: weight [C][N][3][3] fp32 (nn.ConvTranspose2d layout) -> fragments in dtype (F16 / BF16)
void convt3_pack(const float* w, int C, int N, int dtype, void* out);
int launch_convt3(const ConvT3Params& p, int dtype, int cu_count, hipStream_t s);

// ---- small kernels -----------------------------------------------------------------
int launch_prep_nchw(const float* img, int B, int H, int W, void* out, int cpad, int dtype,
                     hipStream_t s);
int launch_prep_u8(const uint8_t* frames, int B, int H, int W, void* out, int cpad, int dtype,
                   hipStream_t s);
// ToTensor + bilinear Resize (torchvision 0.15.2 tensor semantics) + Normalize of u8 HWC frames at
// camera resolution -> normalised fp32 NCHW [B, 3, Ho, Wo] (centernet_node.py:90-92)
int launch_preprocess_u8(const uint8_t* frames, int B, int Hs, int Ws, int Ho, int Wo, float* out, hipStream_t s);
// zero `bytes` (a multiple of 16, 16-byte aligned) with a kernel (graph-capture safe; see aux.hip)
int launch_fill_zero(void* p, size_t bytes, hipStream_t s);
// leaky_relu(0.01) in place over n fp32 values (n % 4 == 0)
int launch_leaky_inplace(float* x, size_t n, hipStream_t s);
// fp32 NCHW [B, C, H, W] -> NHWC compute dtype with pixel stride ldc (protonet input)
int launch_nchw_to_nhwc(const float* img, int B, int C, int H, int W, void* out, int ldc, int dtype, hipStream_t s);
// out[target] = add[target] for target pixels not covered by the shifted upsample.
// CenterpointDLA34 bandwidth kernels (dla34.hip): NHWC, channels in whole 16-byte chunks.
// MaxPool2d(2, 2, ceil_mode=True): out [B, ceil(H/2), ceil(W/2), C]
int launch_maxpool2(const void* src, int B, int H, int W, int C, void* out, int Ho, int Wo, int dtype, hipStream_t s);
// DCNv2 columns cols[pixel][tap][C] = sigmoid(om[18 + tap]) * bilinear(x, y + offset[2 tap], x + offset[2 tap + 1])
int launch_dcn_sample(const void* x, int B, int H, int W, int C, const void* om, int om_ldc, void* cols, int dtype,
                      hipStream_t s);
// out = add + pad_to_match(depthwise ConvTranspose2d(src; weight fp32 [2f][2f][C], stride f, pad f/2)),
// (sy, sx) = pad_to_match's (pad_above, pad_left)
int launch_dwconvt_add(const void* src, int B, int h, int w, int C, const float* weight, int f, const void* add,
                       int add_ldc, void* out, int tH, int tW, int sy, int sx, int dtype, hipStream_t s);
// YOLACT post-processing (yolact.hip), fp32: box_decode (boxes.py:55-61), box_encode (:45-53),
// fast NMS of B images (nms.py:7-29; det[b] = kept anchor indices in descending-confidence order,
// n_det[b] their number), assemble_mask over B images (masks.py:8-21; prototypes at element strides
// pst = (batch, k, y, x), coefficients [B][n_max][K], boxes [B][n_max][4] or null, counts [B] or null)
int launch_yolact_box_decode(const float* enc, const float* anchor, int B, int A, int anchor_batch, float v0, float v1,
                             float* out, hipStream_t s);
int launch_yolact_box_encode(const float* box, const float* anchor, int B, int A, int anchor_batch, float v0, float v1,
                             float* out, hipStream_t s);
size_t yolact_nms_workspace_bytes(int B, int A, int top_k);
int launch_yolact_fast_nms(const float* cls, long long cls_bstride, int A, int C1, const float* box,
                           long long box_bstride, int B, int top_k, float iou_thr, float conf_thr, void* ws,
                           size_t ws_bytes, long long* det, int det_stride, int* n_det, hipStream_t s);
// (det: [B][n_max] row of coefficients / boxes per detection among `rows` per image, or null)
int launch_yolact_assemble_mask(const float* proto, const long long pst[4], int B, int K, int H, int W,
                                const float* coeff, const float* box, const int* counts, const long long* det,
                                int rows, int n_max, float* out, hipStream_t s);
int launch_uncovered_copy(const void* add, int add_ldc, void* out, int out_ldc, int C, int B,
                          int tH, int tW, int y0, int y1, int x0, int x1, int dtype,
                          hipStream_t s);

// ---- decode ------------------------------------------------------------------------
int launch_peaks(const float* heat, const int64_t st[4], int B, int C, int H, int W, int k,
                 int apply_sigmoid, float* peaks, hipStream_t s);
int launch_topk(const float* peaks, int B, int64_t n, int K, float* score, int32_t* index,
                hipStream_t s);
// Detection-record gather of the final decode stage (passed by value to the kernel).
struct DecodeParams {
  int B, K, C, H, W;
  const float* size;    int64_t size_st[4];    // element (b,y,x,ch) strides
  const float* offset;  int64_t offset_st[4];  // may be null (keypoint object path)
  const float* depth;   int64_t depth_st[4];   // may be null
  int depth_mode;       // 0: 1/sigmoid(d) - 1 (decode), 1: 1/sigmoid(d) (decode_keypoints)
  int ratio, in_h, in_w, out_h, out_w;
  int pos_mode;         // 0: (R*i + offset)/in (decode), 1: i/out (decode_keypoints)
  const float* aux;     // optional pair gather (keypoint affinity): element (b, label, j, y, x)
  int64_t aux_st[5];
  float score_thr;
  float* records;       // [B][K][10]: label, score, y, x, h, w, depth, flat index, aux0, aux1
  int32_t* counts;      // [B]
};
// Exact per-image top-K of the (sigmoid ->) 3x3-NMS keys of a strided [B,C,H,W] fp32 view (nms 0:
// plain top-K), ties to the smaller flat index: tile_select + merge_select (decode.hip). Writes
// score / flat index [B][K] (either may be null) and, when rec != null, the detection records.
size_t select_workspace_bytes(int B, int C, int H, int W, int K);
int launch_select(const float* heat, const int64_t st[4], int B, int C, int H, int W, int nms, int apply_sigmoid,
                  int K, void* ws, size_t ws_bytes, float* score, int32_t* index, const DecodeParams* rec,
                  hipStream_t s);
// tv_decode's path (sigmoid + 3x3 NMS + exact top-K + records): peak_scan, one launch (decode.hip).
// Workspace: decode_workspace_bytes(), zero-filled once before its first use; its per-image
// counters sit at fixed offsets (independent of B and of the heatmap geometry) and every call
// leaves them at zero, so the zero-filled workspace serves any later call that fits it.
size_t decode_workspace_bytes(int B, int C, int H, int W, int K);
int launch_decode(const float* heat, const int64_t st[4], int B, int C, int H, int W, int K, void* ws,
                  size_t ws_bytes, const DecodeParams& rec, hipStream_t s);
// heatmap_detect()'s (index[B,K,2], label[B,K]) as int64 from flat top-K indices.
int launch_index_split(const int32_t* flat, int B, int K, int H, int W, int64_t* index, int64_t* label,
                       hipStream_t s);

}  // namespace tv
