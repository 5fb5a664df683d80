// Fused DCNv2 (gfx950, fp16 / bf16): DeformConv.forward (centerpoint_dla.py:386-392) =
// relu(bn(deform_conv2d(x, offset, sigmoid(mask), W) + b)) as ONE kernel — the bilinear samples
// are gathered straight into the LDS operand tile of the MFMA GEMM instead of a 9 x C column
// tensor in HBM (dcn_sample + an implicit GEMM over the columns moved 2 x 9C x 2 B per pixel: 1.4 GB
// per 64-channel layer at 32 frames of 120x160).
//
// GEMM view: rows = BN output channels (A = the DeformConv2d weight, BN folded, K = tap * C + c as
// the column GEMM packs it), columns = 128 output pixels (B = the sampled values), K in steps of 32
// (one tap, 32 channels). Workgroup = 4 waves; wave w owns pixels 32w .. 32w + 31 x the BN
// channels (BN / 32 v_mfma_f32_32x32x16 accumulators).
// Producer: thread (pixel p = tid / 2, half h = tid % 2) samples 16 channels of its pixel per
// k-step: per tap it forms the 4 corner offsets and bilinear weights from the offset / mask conv
// output (the om values of the next tap are loaded one tap ahead), per k-step it loads its 4 x 32 B
// of corner data one step ahead (buffer loads: invalid corners read as zero), blends in fp32 as
// sum of (w_c * mask) * v_c with one rounding to T (dcn_sample multiplies by the mask after the
// corner sum: the same value up to fp32 rounding) and writes 32 B to the double-buffered LDS
// tile; the BN x 32 weight slice of the step is BN / 64 16-byte loads per thread (BN = 128 output
// channels when N allows, so one sampled tile feeds 8 MFMAs per wave, else 64). One barrier per k-step: the MFMAs of step s
// read buffer s & 1 while the producers fill buffer (s + 1) & 1.
#include "conv_common.h"

#include <type_traits>

namespace tv {
namespace dcn {

constexpr int NT = 256, BMP = 128, KS = 32;
constexpr int PITCH = 80;                 // LDS row pitch (bytes): 64 B of K + 16 B pad, conflict-free
constexpr int ABUF = BMP * PITCH;         // sampled pixels x 32 K
template <int BN> constexpr int wbuf() { return BN * PITCH; }  // weight rows x 32 K
template <int BN> constexpr int lds_bytes() { return 2 * (ABUF + wbuf<BN>()); }
constexpr int kOOB = 0x7ff00000;          // buffer offset past any num_records (host checks the sizes)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;  // global (never flat) agent-scope ticket words
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void raw_buffer_store_v4(u32x4 data, i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
__device__ void raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size, int voffset,
                                    int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ __forceinline__ uint4 to_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, t2{(T)a, (T)b});
}
// w * f16 (low / high half of v) [+ acc] in fp32
__device__ __forceinline__ float mix_lo(float w, unsigned v) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[0,1,0]" : "=v"(r) : "v"(w), "v"(v));
  return r;
}
__device__ __forceinline__ float mix_hi(float w, unsigned v) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(r) : "v"(w), "v"(v));
  return r;
}
__device__ __forceinline__ float mix_lo_acc(float w, unsigned v, float acc) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(r) : "v"(w), "v"(v), "v"(acc));
  return r;
}
__device__ __forceinline__ float mix_hi_acc(float w, unsigned v, float acc) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(r) : "v"(w), "v"(v), "v"(acc));
  return r;
}
template <typename T>
__device__ __forceinline__ float elem(const uint4& u, int i) {
  const T* e = reinterpret_cast<const T*>(&u);
  return (float)e[i];
}

template <typename T, int BN>
__global__ __launch_bounds__(NT) void dcn_gemm(const DcnParams p) {
  constexpr int NA = BN / 32;  // 32-channel accumulator blocks per wave
  constexpr int WBUF = wbuf<BN>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int HW = p.H * p.W;
  const int M = p.B * HW;
  // XCD-aware order: workgroup b runs on XCD b % 8; give each XCD a contiguous range of pixel tiles
  // (its L2 then holds the rows those tiles' corners read) and keep the output-channel blocks of a
  // tile adjacent in time
  const int G = gridDim.x, ny = p.N / BN;
  const int q = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int m0 = (q / ny) * BMP, n0 = (q % ny) * BN;
  const int ncb = p.C / KS;
  const int S = 9 * ncb;

  // ---- producer geometry: pixel p, 16-channel half h
  const int pp = tid >> 1, h = tid & 1;
  const int m = m0 + pp;
  const bool mval = m < M;
  const int b = mval ? m / HW : 0;
  const int rem = mval ? m - b * HW : 0;
  const int oy = rem / p.W, ox = rem - (rem / p.W) * p.W;
  const T* om = reinterpret_cast<const T*>(p.om) + (size_t)(mval ? m : 0) * p.om_ldc;

  // x and the weights through buffer resources: per tap, one byte offset per corner (an invalid
  // corner's offset lies past num_records, so its load returns zeros and the blend needs no
  // select), the channel block / k-step in the scalar offset
  i32x4 xr, wrs;
  {
    const unsigned long long a = (unsigned long long)p.x, aw = (unsigned long long)p.w;
    xr = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)((unsigned)M * p.ldx * (unsigned)sizeof(T)), 0x00020000};
    wrs = i32x4{(int)(unsigned)aw, (int)(unsigned)(aw >> 32), (int)((unsigned)p.N * p.Kpad * (unsigned)sizeof(T)),
                0x00020000};
  }
  const int xlane = (b * HW * p.ldx + 16 * h) * (int)sizeof(T);

  // per-tap sampling state (dcn_sample's expressions; the mask is folded into the corner weights)
  int voff[4];
  float wt[4];
  auto tap_params = [&](int k, float dy, float dx, float logit) __attribute__((always_inline)) {
    const float mask = 1.0f / (1.0f + expf(-logit));
    const float py = (float)(oy - 1 + k / 3) + dy;
    const float px = (float)(ox - 1 + k % 3) + dx;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      voff[c] = kOOB;
      wt[c] = 0.f;
    }
    if (mval && py > -1.f && py < (float)p.H && px > -1.f && px < (float)p.W) {
      const float fy = floorf(py), fx = floorf(px);
      const int y0 = (int)fy, x0 = (int)fx;
      const float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
      const float w4[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int yy = y0 + (c >> 1), xx = x0 + (c & 1);
        if (yy >= 0 && yy <= p.H - 1 && xx >= 0 && xx <= p.W - 1) {
          voff[c] = xlane + (yy * p.W + xx) * p.ldx * (int)sizeof(T);
          wt[c] = w4[c] * mask;
        }
      }
    }
  };
  // om values of tap k (loaded one tap ahead)
  float nom[3];
  auto load_om = [&](int k) __attribute__((always_inline)) {
    nom[0] = (float)om[2 * k];
    nom[1] = (float)om[2 * k + 1];
    nom[2] = (float)om[18 + k];
  };
  // corner data of step s = (tap, cb): 4 corners x 2 x 16 B
  uint4 cv[4][2];
  auto load_corners = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      cv[c][0] = to_u4(raw_buffer_load_v4(xr, voff[c], cb * KS * (int)sizeof(T), 0));
      cv[c][1] = to_u4(raw_buffer_load_v4(xr, voff[c], cb * KS * (int)sizeof(T) + 16, 0));
    }
  };
  // weight slice of step s: row r = tid / 4, 16-byte chunk tid % 4 (K = tap * C + cb * 32 = 32 s)
  const int wr = tid >> 2, wc = tid & 3;
  const int wvoff = ((n0 + wr) * p.Kpad + 8 * wc) * (int)sizeof(T);
  uint4 wv[BN / 64];  // rows wr, wr + 64
  auto load_w = [&](int s) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < BN / 64; ++j)
      wv[j] = to_u4(raw_buffer_load_v4(wrs, wvoff + j * 64 * p.Kpad * (int)sizeof(T), s * KS * (int)sizeof(T), 0));
  };

  auto produce = [&](int s) __attribute__((always_inline)) {
    char* A = smem + (s & 1) * (ABUF + WBUF);
    char* Wl = A + ABUF;
    unsigned o[8];
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      float a0, a1;
      if constexpr (std::is_same<T, _Float16>::value) {
        // v_fma_mix reads the f16 halves in place (op_sel picks the high one): one VALU op per
        // element and corner
        const unsigned* d0 = reinterpret_cast<const unsigned*>(&cv[0][e >> 3]);
        a0 = mix_lo(wt[0], d0[(e & 7) >> 1]);
        a1 = mix_hi(wt[0], d0[(e & 7) >> 1]);
#pragma unroll
        for (int c = 1; c < 4; ++c) {
          const unsigned dw = reinterpret_cast<const unsigned*>(&cv[c][e >> 3])[(e & 7) >> 1];
          a0 = mix_lo_acc(wt[c], dw, a0);
          a1 = mix_hi_acc(wt[c], dw, a1);
        }
      } else {
        a0 = 0.f;
        a1 = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a0 += wt[c] * elem<T>(cv[c][e >> 3], e & 7);
          a1 += wt[c] * elem<T>(cv[c][e >> 3], (e & 7) + 1);
        }
      }
      o[e >> 1] = pack2<T>(a0, a1);
    }
    *reinterpret_cast<uint4*>(A + pp * PITCH + 32 * h) = make_uint4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<uint4*>(A + pp * PITCH + 32 * h + 16) = make_uint4(o[4], o[5], o[6], o[7]);
#pragma unroll
    for (int j = 0; j < BN / 64; ++j) *reinterpret_cast<uint4*>(Wl + (wr + 64 * j) * PITCH + 16 * wc) = wv[j];
  };

  f32x16 acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = f32x16{};
  auto consume = [&](int s) __attribute__((always_inline)) {
    const char* A = smem + (s & 1) * (ABUF + WBUF);
    const char* Wl = A + ABUF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // two 16-deep sub-steps
      const uint4 xf = *reinterpret_cast<const uint4*>(A + (32 * wave + l32) * PITCH + 32 * j + 16 * lh);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const uint4 wf = *reinterpret_cast<const uint4*>(Wl + (32 * i + l32) * PITCH + 32 * j + 16 * lh);
        Mfma<T>::run(wf, xf, acc[i]);
      }
    }
  };

  // ---- pipeline: params of tap 0, om of tap 1, operands of step 0
  load_om(0);
  tap_params(0, nom[0], nom[1], nom[2]);
  if (S > ncb) load_om(1);
  load_corners(0);
  load_w(0);
  for (int s = 0; s < S; ++s) {
    produce(s);  // blends step s's corners (loaded one step ahead) into LDS buffer s & 1
    const int s1 = s + 1;
    if (s1 < S) {
      const int k1 = s1 / ncb, cb1 = s1 - k1 * ncb;
      if (cb1 == 0) {  // a new tap: its sampling state from the om values loaded a tap ahead
        tap_params(k1, nom[0], nom[1], nom[2]);
        if (k1 + 1 < 9) load_om(k1 + 1);
      }
      load_corners(cb1);
      load_w(s1);
    }
    __syncthreads();  // buffer s & 1 complete; every wave's reads of buffer (s - 1) & 1 are done
    consume(s);
  }

  // ---- epilogue: channel rows (r & 3) + 8 (r >> 2) + 4 lh of block i, pixel column l32
  const int mo = m0 + 32 * wave + l32;
  if (mo >= M) return;
  T* dst = reinterpret_cast<T*>(p.out) + (size_t)mo * p.out_ldc + n0;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 32 * i + 8 * g + 4 * lh;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][4 * g + e] + p.bias[n0 + ch + e];
        if (p.act == 1) t = fmaxf(t, 0.0f);
        else if (p.act == 2) t = fmaxf(t, 0.01f * t);
        v[e] = t;
      }
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(dst + ch) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
    }
}


// ---- 64-channel k-steps (C % 64 == 0, every DLA-34 DeformConv): full-line gathers.
// The kernel above gives a thread 16 channels of ONE pixel, so each corner-load instruction
// touches 32 pixels' rows for 32 B each: measured, its gathers run at ~12 TB/s of useful bytes,
// a quarter of the L1 lines they touch. Here a k-step is one tap x 64 channels and a thread owns
// one 16-byte channel chunk c = tid % 8 of 4 pixels g + 32 j (g = tid / 8): the 8 lanes of a
// pixel read its 128-byte corner row together, so an instruction fetches 8 whole lines. The
// per-(pixel, tap) sampling state (4 corner offsets, 4 mask-folded weights) is computed once by
// thread p < 128 two taps ahead into an LDS ring of 3 taps and read by the pixel's 8 lanes
// (broadcast). Same blend arithmetic and the same K order as dcn_gemm: the results are identical.
// LDS rows of 128 B (64 K values), 16-byte chunk c of row r stored at chunk c ^ ((r >> 1) & 7)
// (conflict-free fragment reads without padding: two workgroups per CU fit)
constexpr int ROW2 = 128;
__device__ __forceinline__ int sw2(int r, int c) { return r * ROW2 + ((c ^ ((r >> 1) & 7)) << 4); }
// PX pixels per workgroup (128, or 64: half the registers and LDS, twice the resident workgroups
// to hide the corner gathers' latency on layers whose MFMA work per k-step is small)
template <int PX> constexpr int abuf2() { return PX * ROW2; }
template <int BN> constexpr int wbuf2() { return BN * ROW2; }
template <int PX> constexpr int pslot() { return PX * 32; }  // one tap's sampling state: (4 int + 4 float) per pixel
template <int BN, int PX> constexpr int lds_bytes2() { return 2 * (abuf2<PX>() + wbuf2<BN>()) + 3 * pslot<PX>(); }

// resident workgroups per CU the register budget is sized for: as many as the LDS admits (<= 4)
template <int BN, int PX> constexpr int min_blocks2() {
  return 160 * 1024 / lds_bytes2<BN, PX>() < 4 ? 160 * 1024 / lds_bytes2<BN, PX>() : 4;
}
static_assert(min_blocks2<64, 64>() == 4 && min_blocks2<128, 64>() == 2 && min_blocks2<128, 128>() == 2,
              "dcn_gemm64 occupancy hints follow the LDS budget");

template <typename T, int BN, int PX>
__global__ __launch_bounds__(NT, (min_blocks2<BN, PX>())) void dcn_gemm64(const DcnParams p) {
  constexpr int PJ = PX / 32;            // pixels per thread per k-step
  constexpr int WPX = PX / 32;           // waves along pixels (32 each); the rest split the channels
  constexpr int NA = BN / 32 / (4 / WPX);  // 32-channel accumulator blocks per wave
  constexpr int WBUF = wbuf2<BN>();
  constexpr int ABUF2 = abuf2<PX>();
  constexpr int PSLOT = pslot<PX>();
  constexpr int WCH = BN * 8 / NT;       // 16-byte weight chunks per thread per k-step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const Pring = smem + 2 * (ABUF2 + WBUF);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int HW = p.H * p.W;
  const int M = p.B * HW;
  const int G = gridDim.x, ny = p.N / BN;
  const int q = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  // split-K (ksplit > 1): the ksplit workgroups of a tile are adjacent in the XCD-contiguous order;
  // slice sl runs taps [9 sl / ksplit, 9 (sl + 1) / ksplit) (whole taps: the sampling-state ring
  // starts at a tap)
  const int ksplit = p.ksplit > 1 ? p.ksplit : 1;
  const int unit = q / ksplit, slice = q - unit * ksplit;
  const int m0 = (unit / ny) * PX, n0 = (unit % ny) * BN;
  const int ncb = p.C / 64;
  const int k_lo = 9 * slice / ksplit, k_hi = 9 * (slice + 1) / ksplit;
  const int S0 = k_lo * ncb, S = k_hi * ncb;

  i32x4 xr, wrs;
  {
    const unsigned long long a = (unsigned long long)p.x, aw = (unsigned long long)p.w;
    xr = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)((unsigned)M * p.ldx * (unsigned)sizeof(T)), 0x00020000};
    wrs = i32x4{(int)(unsigned)aw, (int)(unsigned)(aw >> 32), (int)((unsigned)p.N * p.Kpad * (unsigned)sizeof(T)),
                0x00020000};
  }

  // ---- sampling-state producer: thread tid < PX owns pixel tid (dcn_sample's expressions)
  const int pm = m0 + (tid & (PX - 1));
  const bool pval = tid < PX && pm < M;
  const int pb = pval ? pm / HW : 0;
  const int prem = pval ? pm - pb * HW : 0;
  const int poy = prem / p.W, pox = prem - (prem / p.W) * p.W;
  const T* om = reinterpret_cast<const T*>(p.om) + (size_t)(pval ? pm : 0) * p.om_ldc;
  float nom[3] = {0.f, 0.f, 0.f};  // om values of the next tap_state call's tap (loaded one call ahead)
  auto load_om = [&](int k) __attribute__((always_inline)) {
    if (pval) {
      nom[0] = (float)om[2 * k];
      nom[1] = (float)om[2 * k + 1];
      nom[2] = (float)om[18 + k];
    }
  };
  auto tap_state = [&](int k) __attribute__((always_inline)) {
    // om values of tap k -> 4 corner byte offsets of the pixel (kOOB: outside) + weights x mask
    int vo[4] = {kOOB, kOOB, kOOB, kOOB};
    float wt[4] = {0.f, 0.f, 0.f, 0.f};
    const float dy = nom[0], dx = nom[1], logit = nom[2];
    if (k + 1 < 9) load_om(k + 1);
    if (pval) {
      const float mask = 1.0f / (1.0f + expf(-logit));
      const float py = (float)(poy - 1 + k / 3) + dy;
      const float px = (float)(pox - 1 + k % 3) + dx;
      if (py > -1.f && py < (float)p.H && px > -1.f && px < (float)p.W) {
        const float fy = floorf(py), fx = floorf(px);
        const int y0 = (int)fy, x0 = (int)fx;
        const float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
        const float w4[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int yy = y0 + (c >> 1), xx = x0 + (c & 1);
          if (yy >= 0 && yy <= p.H - 1 && xx >= 0 && xx <= p.W - 1) {
            vo[c] = ((pb * HW + yy * p.W + xx) * p.ldx) * (int)sizeof(T);
            wt[c] = w4[c] * mask;
          }
        }
      }
    }
    if (tid < PX) {
      int* d = reinterpret_cast<int*>(Pring + (k % 3) * PSLOT + tid * 32);
      *reinterpret_cast<int4*>(d) = make_int4(vo[0], vo[1], vo[2], vo[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(wt[0], wt[1], wt[2], wt[3]);
    }
  };

  // ---- gather geometry: chunk c of pixels g + 32 j
  const int gc = tid & 7, gg = tid >> 3;
  int voff[PJ][4];
  float wts[PJ][4];
  auto read_state = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int* d = reinterpret_cast<const int*>(Pring + (k % 3) * PSLOT + (gg + 32 * j) * 32);
      const int4 o = *reinterpret_cast<const int4*>(d);
      const float4 w = *reinterpret_cast<const float4*>(d + 4);
      voff[j][0] = o.x + 16 * gc; voff[j][1] = o.y + 16 * gc; voff[j][2] = o.z + 16 * gc; voff[j][3] = o.w + 16 * gc;
      wts[j][0] = w.x; wts[j][1] = w.y; wts[j][2] = w.z; wts[j][3] = w.w;
    }
  };
  uint4 cv[PJ][4];  // [pixel j][corner]
  auto load_corners = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PJ; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) cv[j][c] = to_u4(raw_buffer_load_v4(xr, voff[j][c], cb * 64 * (int)sizeof(T), 0));
  };
  // weights of k-step s: chunk i of this thread = row (tid + NT i) / 8, 16-byte column (tid % 8)
  uint4 wv[WCH];
  auto load_w = [&](int s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int r = (tid + NT * i) >> 3;
      wv[i] = to_u4(raw_buffer_load_v4(wrs, ((n0 + r) * p.Kpad + 8 * gc) * (int)sizeof(T), s * 64 * (int)sizeof(T), 0));
    }
  };
  auto produce = [&](int s) __attribute__((always_inline)) {
    char* A = smem + (s & 1) * (ABUF2 + WBUF);
    char* Wl = A + ABUF2;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        float a0, a1;
        if constexpr (std::is_same<T, _Float16>::value) {
          const unsigned d0 = reinterpret_cast<const unsigned*>(&cv[j][0])[e >> 1];
          a0 = mix_lo(wts[j][0], d0);
          a1 = mix_hi(wts[j][0], d0);
#pragma unroll
          for (int c = 1; c < 4; ++c) {
            const unsigned dw = reinterpret_cast<const unsigned*>(&cv[j][c])[e >> 1];
            a0 = mix_lo_acc(wts[j][c], dw, a0);
            a1 = mix_hi_acc(wts[j][c], dw, a1);
          }
        } else {
          a0 = 0.f;
          a1 = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            a0 += wts[j][c] * elem<T>(cv[j][c], e);
            a1 += wts[j][c] * elem<T>(cv[j][c], e + 1);
          }
        }
        o[e >> 1] = pack2<T>(a0, a1);
      }
      *reinterpret_cast<uint4*>(A + sw2(gg + 32 * j, gc)) = make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) *reinterpret_cast<uint4*>(Wl + sw2((tid + NT * i) >> 3, gc)) = wv[i];
  };

  f32x16 acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = f32x16{};
  // wave (wp, wc): pixels 32 wp .. + 31 x accumulator blocks wc * NA .. + NA - 1
  const int wp = wave % WPX, wc = wave / WPX;
  auto consume = [&](int s) __attribute__((always_inline)) {
    const char* A = smem + (s & 1) * (ABUF2 + WBUF);
    const char* Wl = A + ABUF2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // four 16-deep sub-steps
      const uint4 xf = *reinterpret_cast<const uint4*>(A + sw2(32 * wp + l32, 2 * j + lh));
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const uint4 wf = *reinterpret_cast<const uint4*>(Wl + sw2(32 * (wc * NA + i) + l32, 2 * j + lh));
        Mfma<T>::run(wf, xf, acc[i]);
      }
    }
  };

  // ---- pipeline: sampling state of taps 0 and 1, then step 0's operands. Tap k's state is
  // written at the first step of tap k - 2 (slot k % 3, last read when tap k - 3's state was
  // consumed, a barrier or more earlier) and read when step 0 of tap k is issued (the last step
  // of tap k - 1: at least one barrier after it was written).
  load_om(k_lo);
  tap_state(k_lo);
  if (k_lo + 1 < 9) tap_state(k_lo + 1);
  load_w(S0);
  __syncthreads();
  read_state(k_lo);
  load_corners(0);
  for (int s = S0; s < S; ++s) {
    const int k = s / ncb, cb = s - k * ncb;
    produce(s);  // blends step s's corners into LDS buffer s & 1
    if (cb == 0 && k + 2 < 9) tap_state(k + 2);
    const int s1 = s + 1;
    if (s1 < S) {
      const int k1 = s1 / ncb, cb1 = s1 - k1 * ncb;
      if (cb1 == 0) read_state(k1);
      load_corners(cb1);
      load_w(s1);
    }
    __syncthreads();  // buffer s & 1 complete; every wave's reads of buffer (s - 1) & 1 are done
    consume(s);
  }

  if (ksplit > 1) {
    // Split-K hand-off (conv_pipe.hip's scheme): each thread's raw partial accumulators go to
    // slab[unit][slice][thread] with write-through sc1 stores; every wave drains them and the
    // workgroup barrier orders that before one relaxed agent-scope ticket; the workgroup drawing
    // ksplit - 1 sums every slice from the slab in slice order (sc1 loads, its own included:
    // bit-identical whichever arrives last), resets the ticket and runs the epilogue below
    constexpr int SC1 = 16, PER = NA * 16;  // floats per thread
    i32x4 rs;
    {
      const unsigned long long a = (unsigned long long)(p.slab + (size_t)unit * ksplit * NT * PER);
      rs = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32), ksplit * NT * PER * 4, 0x00020000};
    }
    const int toff = tid * PER * 4;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        raw_buffer_store_v4(u32x4{__float_as_uint(acc[i][4 * g]), __float_as_uint(acc[i][4 * g + 1]),
                                  __float_as_uint(acc[i][4 * g + 2]), __float_as_uint(acc[i][4 * g + 3])},
                            rs, toff + (i * 4 + g) * 16, slice * NT * PER * 4, SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* last_flag = reinterpret_cast<unsigned*>(smem);  // (operand buffers: every read done)
    if (tid == 0) *last_flag = __hip_atomic_fetch_add((gu32*)(p.cnt + unit), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*last_flag != (unsigned)(ksplit - 1)) return;  // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: every slab load below is sc1
    if (tid == 0) __hip_atomic_store((gu32*)(p.cnt + unit), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, toff + (i * 4 + g) * 16, 0, SC1));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][4 * g + e] = v[e];
      }
#pragma unroll 1
    for (int sl = 1; sl < ksplit; ++sl) {
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = __builtin_bit_cast(f32x4, raw_buffer_load_v4(rs, toff + (i * 4 + g) * 16, sl * NT * PER * 4, SC1));
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][4 * g + e] += v[e];
        }
    }
  }

  // ---- epilogue (as dcn_gemm)
  const int mo = m0 + 32 * wp + l32;
  if (mo >= M) return;
  T* dst = reinterpret_cast<T*>(p.out) + (size_t)mo * p.out_ldc + n0;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 32 * (wc * NA + i) + 8 * g + 4 * lh;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][4 * g + e] + p.bias[n0 + ch + e];
        if (p.act == 1) t = fmaxf(t, 0.0f);
        else if (p.act == 2) t = fmaxf(t, 0.01f * t);
        v[e] = t;
      }
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(dst + ch) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
    }
}

// ---- dcn_gemm64 with the corner gathers two k-steps ahead (knob TV_DCN64=5, round 6). PMC on the
// B=32 DLA-34 forward (SQ_WAIT_ANY / SQ_WAVE_CYCLES): dcn_gemm64<64, 64>'s waves are parked on
// s_waitcnt / the k-step barrier 57% of their cycles, VALU 14%, MFMA 9% busy: each wave waits every
// k-step for the corner rows it requested one k-step earlier, and one k-step of blend + MFMA work
// (x 4 waves per SIMD) is shorter than an L2 / MALL gather round trip. Here every thread owns two
// operand sets (corners, blend weights, weight chunks) and step s + 2's gathers are issued right
// after step s's blend freed its set, so a gather has two k-steps of the SIMD's work to land in.
// Every global load of the main loop is unconditional (clamped step, OOB offsets) so the compiler's
// counted waits stay exact; the per-(pixel, tap) sampling state is computed three taps ahead into a
// 4-slot LDS ring from offset / mask values loaded one k-step before they are needed. Same
// expressions, blend arithmetic, K order and MFMA sequence as dcn_gemm64: identical results.
template <int BN, int PX> constexpr int lds_bytes2d() { return 2 * (abuf2<PX>() + wbuf2<BN>()) + 4 * pslot<PX>(); }
template <int BN, int PX> constexpr int min_blocks2d() {
  return 160 * 1024 / lds_bytes2d<BN, PX>() < 3 ? 160 * 1024 / lds_bytes2d<BN, PX>() : 3;
}
__device__ unsigned raw_buffer_load_u32(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
template <typename T>
__device__ __forceinline__ float half_of(unsigned v, int hi) {
  const uint16_t b = (uint16_t)(hi ? v >> 16 : v & 0xffffu);
  return (float)__builtin_bit_cast(T, b);
}

template <typename T, int BN, int PX>
__global__ __launch_bounds__(NT, (min_blocks2d<BN, PX>())) void dcn_gemm64d(const DcnParams p) {
  constexpr int PJ = PX / 32;
  constexpr int WPX = PX / 32;
  constexpr int NA = BN / 32 / (4 / WPX);
  constexpr int WBUF = wbuf2<BN>();
  constexpr int ABUF2 = abuf2<PX>();
  constexpr int PSLOT = pslot<PX>();
  constexpr int WCH = BN * 8 / NT;
  constexpr int RSL = 4;  // sampling-state ring slots
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const Pring = smem + 2 * (ABUF2 + WBUF);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int HW = p.H * p.W;
  const int M = p.B * HW;
  const int G = gridDim.x, ny = p.N / BN;
  const int q = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int m0 = (q / ny) * PX, n0 = (q % ny) * BN;
  const int ncb = p.C / 64;
  const int S = 9 * ncb;

  i32x4 xr, wrs, omr;
  {
    const unsigned long long a = (unsigned long long)p.x, aw = (unsigned long long)p.w, ao = (unsigned long long)p.om;
    xr = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)((unsigned)M * p.ldx * (unsigned)sizeof(T)), 0x00020000};
    wrs = i32x4{(int)(unsigned)aw, (int)(unsigned)(aw >> 32), (int)((unsigned)p.N * p.Kpad * (unsigned)sizeof(T)),
                0x00020000};
    omr = i32x4{(int)(unsigned)ao, (int)(unsigned)(ao >> 32), (int)((unsigned)M * p.om_ldc * (unsigned)sizeof(T)),
                0x00020000};
  }

  // ---- sampling-state producer: thread tid < PX owns pixel tid (dcn_sample's expressions)
  const int pm = m0 + (tid & (PX - 1));
  const bool pval = tid < PX && pm < M;
  const int pb = pval ? pm / HW : 0;
  const int prem = pval ? pm - pb * HW : 0;
  const int poy = prem / p.W, pox = prem - (prem / p.W) * p.W;
  const int ombase = pval ? pm * p.om_ldc * (int)sizeof(T) : kOOB;  // (om_ldc even: 4-byte aligned pairs)
  // om values of tap k: the (dy, dx) pair and the dword holding the mask logit (half k & 1)
  auto om_load = [&](int k, unsigned& dydx, unsigned& lg) __attribute__((always_inline)) {
    dydx = raw_buffer_load_u32(omr, ombase + 4 * k, 0, 0);
    lg = raw_buffer_load_u32(omr, ombase + 36 + 4 * (k >> 1), 0, 0);
  };
  auto tap_state = [&](int k, unsigned dydx, unsigned lg, bool write) __attribute__((always_inline)) {
    int vo[4] = {kOOB, kOOB, kOOB, kOOB};
    float wt[4] = {0.f, 0.f, 0.f, 0.f};
    const float dy = half_of<T>(dydx, 0), dx = half_of<T>(dydx, 1), logit = half_of<T>(lg, k & 1);
    if (pval) {
      const float mask = 1.0f / (1.0f + expf(-logit));
      const float py = (float)(poy - 1 + k / 3) + dy;
      const float px = (float)(pox - 1 + k % 3) + dx;
      if (py > -1.f && py < (float)p.H && px > -1.f && px < (float)p.W) {
        const float fy = floorf(py), fx = floorf(px);
        const int y0 = (int)fy, x0 = (int)fx;
        const float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
        const float w4[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int yy = y0 + (c >> 1), xx = x0 + (c & 1);
          if (yy >= 0 && yy <= p.H - 1 && xx >= 0 && xx <= p.W - 1) {
            vo[c] = ((pb * HW + yy * p.W + xx) * p.ldx) * (int)sizeof(T);
            wt[c] = w4[c] * mask;
          }
        }
      }
    }
    if (write && tid < PX) {
      int* d = reinterpret_cast<int*>(Pring + (k % RSL) * PSLOT + tid * 32);
      *reinterpret_cast<int4*>(d) = make_int4(vo[0], vo[1], vo[2], vo[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(wt[0], wt[1], wt[2], wt[3]);
    }
  };

  // ---- operand sets: corners, blend weights and weight chunks of one k-step
  const int gc = tid & 7, gg = tid >> 3;
  struct Set {
    uint4 cv[PJ][4];
    float wts[PJ][4];
    uint4 wv[WCH];
  };
  Set A, B;
  // step s's operands into set X: its tap's state from the ring (offsets -> gathers, weights kept)
  auto prepare = [&](int s, Set& X) __attribute__((always_inline)) {
    const int k = s / ncb, cb = s - k * ncb;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int* d = reinterpret_cast<const int*>(Pring + (k % RSL) * PSLOT + (gg + 32 * j) * 32);
      const int4 o = *reinterpret_cast<const int4*>(d);
      const float4 w = *reinterpret_cast<const float4*>(d + 4);
      const int vo[4] = {o.x, o.y, o.z, o.w};
      X.wts[j][0] = w.x; X.wts[j][1] = w.y; X.wts[j][2] = w.z; X.wts[j][3] = w.w;
#pragma unroll
      for (int c = 0; c < 4; ++c) X.cv[j][c] = to_u4(raw_buffer_load_v4(xr, vo[c] + 16 * gc, cb * 64 * (int)sizeof(T), 0));
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int r = (tid + NT * i) >> 3;
      X.wv[i] = to_u4(raw_buffer_load_v4(wrs, ((n0 + r) * p.Kpad + 8 * gc) * (int)sizeof(T), s * 64 * (int)sizeof(T), 0));
    }
  };
  auto produce = [&](int s, const Set& X) __attribute__((always_inline)) {
    char* Ab = smem + (s & 1) * (ABUF2 + WBUF);
    char* Wl = Ab + ABUF2;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        float a0, a1;
        if constexpr (std::is_same<T, _Float16>::value) {
          const unsigned d0 = reinterpret_cast<const unsigned*>(&X.cv[j][0])[e >> 1];
          a0 = mix_lo(X.wts[j][0], d0);
          a1 = mix_hi(X.wts[j][0], d0);
#pragma unroll
          for (int c = 1; c < 4; ++c) {
            const unsigned dw = reinterpret_cast<const unsigned*>(&X.cv[j][c])[e >> 1];
            a0 = mix_lo_acc(X.wts[j][c], dw, a0);
            a1 = mix_hi_acc(X.wts[j][c], dw, a1);
          }
        } else {
          a0 = 0.f;
          a1 = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            a0 += X.wts[j][c] * elem<T>(X.cv[j][c], e);
            a1 += X.wts[j][c] * elem<T>(X.cv[j][c], e + 1);
          }
        }
        o[e >> 1] = pack2<T>(a0, a1);
      }
      *reinterpret_cast<uint4*>(Ab + sw2(gg + 32 * j, gc)) = make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) *reinterpret_cast<uint4*>(Wl + sw2((tid + NT * i) >> 3, gc)) = X.wv[i];
  };

  f32x16 acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = f32x16{};
  const int wp = wave % WPX, wc = wave / WPX;
  auto consume = [&](int s) __attribute__((always_inline)) {
    const char* Ab = smem + (s & 1) * (ABUF2 + WBUF);
    const char* Wl = Ab + ABUF2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 xf = *reinterpret_cast<const uint4*>(Ab + sw2(32 * wp + l32, 2 * j + lh));
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const uint4 wf = *reinterpret_cast<const uint4*>(Wl + sw2(32 * (wc * NA + i) + l32, 2 * j + lh));
        Mfma<T>::run(wf, xf, acc[i]);
      }
    }
  };

  // ---- prologue: the states of taps 0..2, the om values for the loop's first state (tap 3), the
  // operands of steps 0 and 1
  {
    unsigned d0, l0, d1, l1, d2, l2;
    om_load(0, d0, l0);
    om_load(1, d1, l1);
    om_load(2, d2, l2);
    tap_state(0, d0, l0, true);
    tap_state(1, d1, l1, true);
    tap_state(2, d2, l2, true);
  }
  unsigned om_dydx, om_lg;  // om values for the state computed in the next iteration
  om_load(3, om_dydx, om_lg);
  __syncthreads();
  prepare(0, A);
  prepare(min(1, S - 1), B);
  // iteration s: blend step s (its set then free), the tap-(k+3) state when s starts tap k, the
  // om values of the next iteration's state, step s + 2's operands into the freed set (past the
  // end: the last step again, unused), barrier, step s's MFMAs
  auto iter = [&](int s, Set& X) __attribute__((always_inline)) {
    const int k = s / ncb, cb = s - k * ncb;
    produce(s, X);
    const int tk = min(k + 3, 8);
    tap_state(tk, om_dydx, om_lg, cb == 0 && k + 3 < 9);
    const int s1 = s + 1;
    const int k1n = min(min(s1, S - 1) / ncb + 3, 8);
    om_load(k1n, om_dydx, om_lg);
    prepare(min(s + 2, S - 1), X);
    __syncthreads();
    consume(s);
  };
  for (int s = 0;;) {
    iter(s, A);
    if (++s == S) break;
    iter(s, B);
    if (++s == S) break;
  }

  // ---- epilogue (as dcn_gemm64)
  const int mo = m0 + 32 * wp + l32;
  if (mo >= M) return;
  T* dst = reinterpret_cast<T*>(p.out) + (size_t)mo * p.out_ldc + n0;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 32 * (wc * NA + i) + 8 * g + 4 * lh;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][4 * g + e] + p.bias[n0 + ch + e];
        if (p.act == 1) t = fmaxf(t, 0.0f);
        else if (p.act == 2) t = fmaxf(t, 0.01f * t);
        v[e] = t;
      }
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(dst + ch) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
    }
}

// ---- window variant (C == N == 64: DLA-34's 120x160 DeformConvs, node_k of ida_2 / ida_up, two
// thirds of its DCN time). dcn_gemm64 gathers every corner from L1/L2: 9 taps x 4 corners x 128 B
// per pixel, ~15 TB/s of useful bytes, the TA/TD rate of 16-byte gathers (MI355X_MICROARCH.md,
// indexed rows). The corners of a tile's samples lie within a few pixels of the tile (the offsets
// are a smooth learned field: |offset| <= 1.6 on every DLA-34 layer at the bench weights), so here:
//  * a persistent 512-thread workgroup per CU walks 16 x 16-pixel tiles; the tile's input window
//    (rows / columns -1 - MG .. 16 + MG around it, 64 channels, 128-B pixel rows, 16-byte chunks
//    XOR-swizzled by the window pixel) moves into LDS ONCE per tile by LDS-DMA (out-of-image pixels
//    read as buffer-OOB zeros), and every corner inside it is read from LDS (ds_read_b128: 4x the
//    per-CU rate of the L1 gathers); a corner outside the window but inside the image (offsets past
//    MG) is gathered from global memory in a branch taken only by waves that have one;
//  * the DeformConv2d weights of all 9 taps (64 x 576, 72 KiB) stay resident in LDS;
//  * wave w owns tile pixels 32 w .. 32 w + 31 x all 64 output channels: lane (l32, lh) computes its
//    pixel's sampling state per tap and blends the 16-byte chunk 2 j + lh of each 16-deep sub-step
//    j straight into the MFMA B operand register (no LDS round trip, no per-k-step barrier);
//  * one barrier per tile (the window), and the next tile's window DMA is issued as soon as the last
//    tap's corners are read, under that tap's MFMAs and the epilogue.
// Same sampling expressions, blend arithmetic, K order and MFMA sequence as dcn_gemm64: the
// results are bit-identical to it (tests/test_gpu_dcn.py).
#if defined(TV_DCN_STAMPS)  // stamp build (EXTRA=-DTV_DCN_STAMPS=1, tools/dcn_stamps.py): per-wave cycle buckets
#define WSTAMP(B)                                                                      \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    unsigned long long t_;                                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    st_b[B] += t_ - st_last;                                                           \
    st_last = t_;                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#else
#define WSTAMP(B) \
  do {            \
  } while (0)
#endif
namespace win {
constexpr int WNT = 512, TH = 16, TW = 16, MG = 2;
constexpr int WR = TH + 2 + 2 * MG, WC = TW + 2 + 2 * MG;  // window rows / columns (22 x 22)
constexpr int WPIX = WR * WC;                               // 484 window pixels
constexpr int WCHUNKS = WPIX * 8;                           // 16-byte chunks of the window
constexpr int WPIECES = (WCHUNKS + WNT - 1) / WNT;            // LDS-DMA rounds (8 x 512 chunks)
constexpr int OFF_W = 0;                                    // weights [9 taps][64 co][128 B]
constexpr int OFF_X = OFF_W + 9 * 64 * 128;                 // window [WPIECES * 512 chunks][16 B]
constexpr int OFF_Z = OFF_X + WPIECES * WNT * 16;            // 128 zero bytes: invalid corners
constexpr int OFF_B = OFF_Z + 128;                          // the 64 biases (fp32)
constexpr int LDS = OFF_B + 64 * 4;
static_assert(LDS <= 160 * 1024, "LDS budget");
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
}  // namespace win

template <typename T>
__global__ __attribute__((amdgpu_flat_work_group_size(win::WNT, win::WNT), amdgpu_waves_per_eu(2, 2))) void dcn_win(
    const DcnParams p) {
  using namespace win;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int H = p.H, W = p.W;
  const int tiles_x = (W + TW - 1) / TW, tiles_f = ((H + TH - 1) / TH) * tiles_x;
  const int ntot = p.B * tiles_f;
  // XCD-aware contiguous tile ranges (neighbouring tiles share window rows in the XCD's L2)
  const int G = gridDim.x, bid = blockIdx.x;
  int first, stride, end;
  if ((G & 7) == 0) {
    first = (int)((long long)ntot * (bid & 7) / 8) + (bid >> 3);
    end = (int)((long long)ntot * ((bid & 7) + 1) / 8);
    stride = G >> 3;
  } else {
    first = bid;
    end = ntot;
    stride = G;
  }
  if (first >= end) return;

  i32x4 xr;
  {
    const unsigned long long a = (unsigned long long)p.x;
    xr = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32),
               (int)((unsigned)p.B * H * W * p.ldx * (unsigned)sizeof(T)), 0x00020000};
  }
  auto dma = [&](int off, int lds_off) __attribute__((always_inline)) {
    raw_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(smem + lds_off), 16, off, 0, 0, 0);
  };
  // the window of tile t into LDS: chunk g = window pixel g / 8, slot g % 8 holds source chunk
  // slot ^ swz(pixel) (the reads un-swizzle); chunks past the window land in its slack
  auto stage = [&](int t) __attribute__((always_inline)) {
    const int fr = t / tiles_f, r = t - fr * tiles_f, ty = r / tiles_x;
    const int wy0 = ty * TH - 1 - MG, wx0 = (r - ty * tiles_x) * TW - 1 - MG;
#pragma unroll
    for (int q = 0; q < WPIECES; ++q) {
      const int g = q * WNT + tid;
      const int wp = g >> 3, c = (g & 7) ^ swz(g >> 3);
      const int wy = wp / WC, wx = wp - (wp / WC) * WC;
      const int y = wy0 + wy, x = wx0 + wx;
      const bool ok = g < WCHUNKS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      dma(ok ? ((fr * H + y) * W + x) * p.ldx * (int)sizeof(T) + c * 16 : kOOB, OFF_X + (q * WNT + wave * 64) * 16);
    }
  };

  // ---- resident: the weights of the 9 taps (row k * 64 + co, chunk c at c ^ swz(row)) and the zeros
  {
    const T* w = reinterpret_cast<const T*>(p.w);
    constexpr int NCH = 9 * 64 * 8 / WNT;
    uint4 wv[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int g = i * WNT + tid, row = g >> 3, c = g & 7, k = row >> 6, co = row & 63;
      wv[i] = *reinterpret_cast<const uint4*>(w + (size_t)co * p.Kpad + k * 64 + 8 * c);
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int g = i * WNT + tid, row = g >> 3, c = g & 7;
      *reinterpret_cast<uint4*>(smem + OFF_W + row * 128 + ((c ^ swz(row)) << 4)) = wv[i];
    }
    if (tid < 8) *reinterpret_cast<uint4*>(smem + OFF_Z + tid * 16) = make_uint4(0u, 0u, 0u, 0u);
    if (tid < 64) reinterpret_cast<float*>(smem + OFF_B)[tid] = p.bias[tid];
  }
  // the 27 offset / mask values of this lane's pixel of tile t (32 fp16 = 4 x 16 B: om_ldc >= 32,
  // 16-byte rows), loaded a tile ahead with the window
  const int q = 32 * wave + l32;  // this lane's tile pixel
  i32x4 omr;
  {
    const unsigned long long a = (unsigned long long)p.om;
    omr = i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32),
                (int)((unsigned)p.B * H * W * p.om_ldc * (unsigned)sizeof(T)), 0x00020000};
  }
  uint4 omv[4];
  auto load_om = [&](int t) __attribute__((always_inline)) {
    const int fr = t / tiles_f, r = t - fr * tiles_f, ty = r / tiles_x;
    const int oy = ty * TH + (q >> 4), ox = (r - ty * tiles_x) * TW + (q & 15);
    const int off = oy < H && ox < W ? ((fr * H + oy) * W + ox) * p.om_ldc * (int)sizeof(T) : kOOB;
#pragma unroll
    for (int i = 0; i < 4; ++i) omv[i] = to_u4(raw_buffer_load_v4(omr, off, 16 * i, 0));
  };
  auto om_at = [&](int e) __attribute__((always_inline)) -> float {
    const unsigned d = reinterpret_cast<const unsigned*>(omv)[e >> 1];
    return (float)__builtin_bit_cast(T, (unsigned short)((e & 1) ? d >> 16 : d & 0xffffu));
  };
  stage(first);
  load_om(first);
#if defined(TV_DCN_STAMPS)
  // buckets: 0 tile-top wait, 1 sampling state, 2 corner reads + blend, 3 MFMAs, 4 tap-8 barrier +
  // next window issue, 5 epilogue, 6 tiles
  unsigned long long st_b[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif

  for (int t = first; t < end; t += stride) {
    const int fr = t / tiles_f, r = t - fr * tiles_f, ty = r / tiles_x;
    const int y0 = ty * TH, x0 = (r - ty * tiles_x) * TW;
    const int wy0 = y0 - 1 - MG, wx0 = x0 - 1 - MG;
    const int oy = y0 + (q >> 4), ox = x0 + (q & 15);
    const bool pval = oy < H && ox < W;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's window pieces and om values landed
    __syncthreads();                                   // ... and every other thread's window pieces
    WSTAMP(0);
#if defined(TV_DCN_STAMPS)
    st_b[6] += 1;
#endif
    float omf[27];
#pragma unroll
    for (int e = 0; e < 27; ++e) omf[e] = om_at(e);

    // sampling state of (pixel, tap k), branch-free (dcn_gemm64's expressions and values): corner c
    // reads LDS at A[c] ^ (chunk << 4) (its window pixel's 128-B row | swizzle << 4, or the zero row
    // for a corner outside the image) or, outside the window, global memory at go[c]
    struct St {
      int A[4], go[4];
      float wt[4];
      bool fb;
    };
    auto state = [&](int k, St& S) __attribute__((always_inline)) {
      const float dy = omf[2 * k], dx = omf[2 * k + 1], logit = omf[18 + k];
      const float mask = 1.0f / (1.0f + expf(-logit));
      const float py = (float)(oy - 1 + k / 3) + dy;
      const float px = (float)(ox - 1 + k % 3) + dx;
      const bool vs = pval && py > -1.f && py < (float)H && px > -1.f && px < (float)W;
      const float fy = floorf(vs ? py : 0.f), fx = floorf(vs ? px : 0.f);
      const int yc = (int)fy, xc = (int)fx;
      const float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
      const float w4[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
      S.fb = false;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int yy = yc + (c >> 1), xx = xc + (c & 1);
        const bool in = vs && yy >= 0 && yy <= H - 1 && xx >= 0 && xx <= W - 1;
        const int wy = yy - wy0, wx = xx - wx0;
        const bool inw = (unsigned)wy < (unsigned)WR && (unsigned)wx < (unsigned)WC;
        const int wp = wy * WC + wx;
        S.wt[c] = in ? w4[c] * mask : 0.f;
        S.A[c] = in && inw ? (OFF_X + wp * 128) | (swz(wp) << 4) : OFF_Z;
        S.go[c] = in && !inw ? ((fr * H + yy) * W + xx) * p.ldx * (int)sizeof(T) : kOOB;
        S.fb = S.fb || (in && !inw);
      }
    };
    // the tap's 4 sub-steps x 4 corners: chunk 2 j + lh of each corner (LDS, then the rare global
    // gathers of corners outside the window: per-lane offsets, no waterfall)
    auto reads = [&](const St& S, uint4 (&cv)[4][4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          cv[j][c] = *reinterpret_cast<const uint4*>(smem + (S.A[c] ^ ((2 * j + lh) << 4)));
      if (__builtin_amdgcn_ballot_w64(S.fb) != 0) {  // (wave-uniform)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint4 g = to_u4(raw_buffer_load_v4(xr, S.go[c] + (2 * j + lh) * 16, 0, 0));
            if (S.go[c] != kOOB) cv[j][c] = g;
          }
      }
    };
    auto blend = [&](const St& S, const uint4 (&cv)[4][4], uint4 (&xf)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unsigned o[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          float a0, a1;
          if constexpr (std::is_same<T, _Float16>::value) {
            const unsigned d0 = reinterpret_cast<const unsigned*>(&cv[j][0])[e >> 1];
            a0 = mix_lo(S.wt[0], d0);
            a1 = mix_hi(S.wt[0], d0);
#pragma unroll
            for (int c = 1; c < 4; ++c) {
              const unsigned dw = reinterpret_cast<const unsigned*>(&cv[j][c])[e >> 1];
              a0 = mix_lo_acc(S.wt[c], dw, a0);
              a1 = mix_hi_acc(S.wt[c], dw, a1);
            }
          } else {
            a0 = 0.f;
            a1 = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              a0 += S.wt[c] * elem<T>(cv[j][c], e);
              a1 += S.wt[c] * elem<T>(cv[j][c], e + 1);
            }
          }
          o[e >> 1] = pack2<T>(a0, a1);
        }
        xf[j] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    };

    f32x16 acc[2] = {f32x16{}, f32x16{}};
    St S[2];
    uint4 cv[2][4][4];
    state(0, S[0]);
    reads(S[0], cv[0]);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      WSTAMP(1);
      uint4 xf[4];
      blend(S[k & 1], cv[k & 1], xf);
      WSTAMP(2);
      if (k == 8) {
        // every wave's corner reads of this tile are done (lgkmcnt): once all waves are here the
        // window is free, and the next tile's DMA runs under the last MFMAs and the epilogue
        __syncthreads();
        if (t + stride < end) {
          stage(t + stride);
          load_om(t + stride);
        }
        WSTAMP(4);
      } else {
        // the next tap's state and corner reads in flight under this tap's MFMAs
        state(k + 1, S[(k + 1) & 1]);
        reads(S[(k + 1) & 1], cv[(k + 1) & 1]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = k * 64 + 32 * i + l32;
          const uint4 wf = *reinterpret_cast<const uint4*>(smem + OFF_W + row * 128 + (((2 * j + lh) ^ swz(row)) << 4));
          Mfma<T>::run(wf, xf[j], acc[i]);
        }
      WSTAMP(3);
    }

    // ---- epilogue (as dcn_gemm64): channel rows (r & 3) + 8 (r >> 2) + 4 lh of block i, pixel l32
    if (pval) {
      T* dst = reinterpret_cast<T*>(p.out) + (size_t)((fr * H + oy) * W + ox) * p.out_ldc;
      const float* lb = reinterpret_cast<const float*>(smem + OFF_B);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ch = 32 * i + 8 * g + 4 * lh;
          const f32x4 bb = *reinterpret_cast<const f32x4*>(lb + ch);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float tt = acc[i][4 * g + e] + bb[e];
            if (p.act == 1) tt = fmaxf(tt, 0.0f);
            else if (p.act == 2) tt = fmaxf(tt, 0.01f * tt);
            v[e] = tt;
          }
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2*>(dst + ch) = u32x2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        }
    }
    WSTAMP(5);
  }
#if defined(TV_DCN_STAMPS)
  __syncthreads();
  if (lane == 0) {  // (the stamp build overwrites the output's first bytes)
    unsigned long long* d = reinterpret_cast<unsigned long long*>(p.out) + ((size_t)bid * 8 + wave) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = st_b[k];
  }
#endif
}

template <typename T>
static void launch_win(const DcnParams& p, int cu_count, hipStream_t s) {
  (void)ensure_lds<dcn_win<T>>(win::LDS);
  const long tiles = (long)p.B * ((p.H + win::TH - 1) / win::TH) * ((p.W + win::TW - 1) / win::TW);
  int grid = (int)std::min<long>(tiles, cu_count);
  if (grid >= 8 && tiles > 2L * grid) grid -= grid % 8;
  hipLaunchKernelGGL((dcn_win<T>), dim3(grid), dim3(win::WNT), win::LDS, s, p);
}

template <typename T, int BN, int PX>
static void launch64d(const DcnParams& p, hipStream_t s) {
  constexpr int lds = lds_bytes2d<BN, PX>();
  (void)ensure_lds<dcn_gemm64d<T, BN, PX>>(lds);
  const long M = (long)p.B * p.H * p.W;
  const dim3 grid((unsigned)((M + PX - 1) / PX * (p.N / BN)));
  hipLaunchKernelGGL((dcn_gemm64d<T, BN, PX>), grid, dim3(NT), lds, s, p);
}

template <typename T, int BN, int PX>
static void launch64(const DcnParams& p, hipStream_t s) {
  constexpr int lds = lds_bytes2<BN, PX>();
  (void)ensure_lds<dcn_gemm64<T, BN, PX>>(lds);
  const long M = (long)p.B * p.H * p.W;
  const dim3 grid((unsigned)((M + PX - 1) / PX * (p.N / BN) * (p.ksplit > 1 ? p.ksplit : 1)));
  hipLaunchKernelGGL((dcn_gemm64<T, BN, PX>), grid, dim3(NT), lds, s, p);
}

}  // namespace dcn

void dcn64_tile(const DcnParams& p, int dcn64_mode, int* bn, int* px) {
  // launch_dcn_gemm's choice for dcn_gemm64 (modes 1 / 2 and the fallback of 3 / 4)
  const long M = (long)p.B * p.H * p.W;
  const bool wide = p.N % 128 == 0;
  const long tiles128 = (M + 127) / 128 * (p.N / 128);
  *bn = wide ? 128 : 64;
  *px = !wide || dcn64_mode == 2 || tiles128 < 1024 ? 64 : 128;
}

long dcn_split_floats(const DcnParams& p, int dcn64_mode, int ksplit) {
  int bn, px;
  dcn64_tile(p, dcn64_mode, &bn, &px);
  const long M = (long)p.B * p.H * p.W;
  const int na = bn / 32 / (4 / (px / 32));
  return (M + px - 1) / px * (p.N / bn) * ksplit * dcn::NT * na * 16;
}

bool dcn_gemm_supported(long M, int C, int N, int ldx, int om_ldc, int out_ldc, int Kpad) {
  // buffer offsets are 32-bit: the input and weight tensors stay below the out-of-range marker
  if (M * ldx * 2 >= dcn::kOOB || (long)N * Kpad * 2 >= dcn::kOOB) return false;
  return C % dcn::KS == 0 && N % 64 == 0 && ldx % 8 == 0 && om_ldc >= 27 && out_ldc % 4 == 0;
}

bool dcn_win_supported(const DcnParams& p) {
  return p.C == 64 && p.N == 64 && p.ldx % 8 == 0 && p.out_ldc % 4 == 0 && p.Kpad >= 9 * 64 &&
         p.om_ldc >= 32 && p.om_ldc % 8 == 0 &&
         (long)p.B * p.H * p.W * p.ldx * 2 < dcn::kOOB;
}

int launch_dcn_gemm(const DcnParams& p, int dtype, int dcn64_mode, int cu_count, hipStream_t s) {
  if (!dcn_gemm_supported((long)p.B * p.H * p.W, p.C, p.N, p.ldx, p.om_ldc, p.out_ldc, p.Kpad) || p.Kpad < 9 * p.C) {
    set_error("dcn_gemm: channels must be multiples of 32 (input) / 64 (output), tensors below 2 GB");
    return 1;
  }
  const long M = (long)p.B * p.H * p.W;
  // 128 output channels per workgroup when N allows: each sampled tile feeds twice the MFMAs
  const bool wide = p.N % 128 == 0;
  dim3 grid((unsigned)((M + dcn::BMP - 1) / dcn::BMP * (p.N / (wide ? 128 : 64))));
  if (dtype != F16 && dtype != BF16) {
    set_error("dcn_gemm: fp16/bf16 only");
    return 1;
  }
  if (p.ksplit > 1 && (!p.slab || !p.cnt || p.ksplit > 9 || p.C % 64 || !dcn64_mode || dcn64_mode >= 3)) {
    set_error("dcn_gemm: split-K needs dcn_gemm64 (modes 1 / 2), a slab, tickets and <= 9 slices");
    return 1;
  }
  if ((dcn64_mode == 3 || dcn64_mode == 4) && dcn_win_supported(p)) {  // LDS window (C == N == 64; mode 4: diagnostics only)
    if (dtype == F16) dcn::launch_win<_Float16>(p, cu_count, s);
    else dcn::launch_win<__bf16>(p, cu_count, s);
  } else if (p.C % 64 == 0 && dcn64_mode) {  // full-line gathers (every DLA-34 DeformConv); mode 2: 64-pixel tiles
    // 64-pixel tiles (measured: 4 resident workgroups per CU hide the corner gathers better than
    // 2 of 128 pixels; the 64-channel layers 5561 -> 5775 frames/s at B=64); 128-channel outputs
    // too when 128-pixel tiles would leave few workgroups per CU (B=1: 1.65 -> 1.52 ms; B=64 neutral)
    const long tiles128 = (M + 127) / 128 * (p.N / 128);
    const bool px64w = dcn64_mode == 2 || tiles128 < 1024;
    if (dcn64_mode == 5 && p.om_ldc % 2 == 0) {  // gathers two k-steps ahead (64-pixel tiles)
      if (dtype == F16) {
        if (wide) dcn::launch64d<_Float16, 128, 64>(p, s);
        else dcn::launch64d<_Float16, 64, 64>(p, s);
      } else {
        if (wide) dcn::launch64d<__bf16, 128, 64>(p, s);
        else dcn::launch64d<__bf16, 64, 64>(p, s);
      }
    } else if (dtype == F16) {
      if (wide) px64w ? dcn::launch64<_Float16, 128, 64>(p, s) : dcn::launch64<_Float16, 128, 128>(p, s);
      else dcn::launch64<_Float16, 64, 64>(p, s);
    } else {
      if (wide) px64w ? dcn::launch64<__bf16, 128, 64>(p, s) : dcn::launch64<__bf16, 128, 128>(p, s);
      else dcn::launch64<__bf16, 64, 64>(p, s);
    }
  } else if (dtype == F16) {
    if (wide) hipLaunchKernelGGL((dcn::dcn_gemm<_Float16, 128>), grid, dim3(dcn::NT), dcn::lds_bytes<128>(), s, p);
    else hipLaunchKernelGGL((dcn::dcn_gemm<_Float16, 64>), grid, dim3(dcn::NT), dcn::lds_bytes<64>(), s, p);
  } else {
    if (wide) hipLaunchKernelGGL((dcn::dcn_gemm<__bf16, 128>), grid, dim3(dcn::NT), dcn::lds_bytes<128>(), s, p);
    else hipLaunchKernelGGL((dcn::dcn_gemm<__bf16, 64>), grid, dim3(dcn::NT), dcn::lds_bytes<64>(), s, p);
  }
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
