// Fused DCNv2 (gfx950, fp16 / bf16): DeformConv.forward (centerpoint_dla.py:386-392) =
// relu(bn(deform_conv2d(x, offset, sigmoid(mask), W) + b)) as ONE kernel — the bilinear samples
// are gathered straight into the LDS operand tile of the MFMA GEMM instead of a 9 x C column
// tensor in HBM (dcn_sample + an implicit GEMM over the columns moved 2 x 9C x 2 B per pixel: 1.4 GB
// per 64-channel layer at 32 frames of 120x160).
//
// GEMM view: rows = 64 output channels (A = the DeformConv2d weight, BN folded, K = tap * C + c as
// the column GEMM packs it), columns = 128 output pixels (B = the sampled values), K in steps of 32
// (one tap, 32 channels). Workgroup = 4 waves; wave w owns pixels 32w .. 32w + 31 x the 64
// channels (two v_mfma_f32_32x32x16 accumulators).
// Producer: thread (pixel p = tid / 2, half h = tid % 2) samples 16 channels of its pixel per
// k-step: per tap it forms the 4 corner offsets and bilinear weights from the offset / mask conv
// output (the om values of the next tap are loaded one tap ahead), per k-step it loads its 4 x 32 B
// of corner data one step ahead (buffer loads: invalid corners read as zero), blends in fp32 as
// sum of (w_c * mask) * v_c with one rounding to T (dcn_sample multiplies by the mask after the
// corner sum: the same value up to fp32 rounding) and writes 32 B to the double-buffered LDS tile; the 64 x 32 weight
// slice of the step is one 16-byte load per thread. One barrier per k-step: the MFMAs of step s
// read buffer s & 1 while the producers fill buffer (s + 1) & 1.
#include "conv_common.h"

#include <type_traits>

namespace tv {
namespace dcn {

constexpr int NT = 256, BMP = 128, BNC = 64, KS = 32;
constexpr int PITCH = 80;                 // LDS row pitch (bytes): 64 B of K + 16 B pad, conflict-free
constexpr int ABUF = BMP * PITCH;         // sampled pixels x 32 K
constexpr int WBUF = BNC * PITCH;         // weight rows x 32 K
constexpr int LDS = 2 * (ABUF + WBUF);
constexpr int kOOB = 0x7ff00000;          // buffer offset past any num_records (host checks the sizes)

typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
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

template <typename T>
__global__ __launch_bounds__(NT) void dcn_gemm(const DcnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, lh = lane >> 5;
  const int HW = p.H * p.W;
  const int M = p.B * HW;
  const int m0 = blockIdx.x * BMP, n0 = blockIdx.y * BNC;
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
  float wt[4];  // the tap being issued
  struct Set {
    uint4 cv[4][2];
    uint4 wv;
    float wt[4];
  };
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
  const int wr = tid >> 2, wc = tid & 3;
  const int wvoff = ((n0 + wr) * p.Kpad + 8 * wc) * (int)sizeof(T);
  // step s = (tap, cb) into a register set: 4 corners x 2 x 16 B + the weight chunk
  auto issue = [&](int s, Set& st) __attribute__((always_inline)) {
    const int k = s / ncb, cb = s - k * ncb;
    if (cb == 0) {
      tap_params(k, nom[0], nom[1], nom[2]);
      if (k + 1 < 9) load_om(k + 1);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      st.wt[c] = wt[c];
      st.cv[c][0] = to_u4(raw_buffer_load_v4(xr, voff[c], cb * KS * (int)sizeof(T), 0));
      st.cv[c][1] = to_u4(raw_buffer_load_v4(xr, voff[c], cb * KS * (int)sizeof(T) + 16, 0));
    }
    st.wv = to_u4(raw_buffer_load_v4(wrs, wvoff, s * KS * (int)sizeof(T), 0));
  };

  auto produce = [&](int s, const Set& st) __attribute__((always_inline)) {
    char* A = smem + (s & 1) * (ABUF + WBUF);
    char* Wl = A + ABUF;
    unsigned o[8];
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      float a0, a1;
      if constexpr (std::is_same<T, _Float16>::value) {
        // v_fma_mix reads the f16 halves in place (op_sel picks the high one): one VALU op per
        // element and corner
        const unsigned* d0 = reinterpret_cast<const unsigned*>(&st.cv[0][e >> 3]);
        a0 = mix_lo(st.wt[0], d0[(e & 7) >> 1]);
        a1 = mix_hi(st.wt[0], d0[(e & 7) >> 1]);
#pragma unroll
        for (int c = 1; c < 4; ++c) {
          const unsigned dw = reinterpret_cast<const unsigned*>(&st.cv[c][e >> 3])[(e & 7) >> 1];
          a0 = mix_lo_acc(st.wt[c], dw, a0);
          a1 = mix_hi_acc(st.wt[c], dw, a1);
        }
      } else {
        a0 = 0.f;
        a1 = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a0 += st.wt[c] * elem<T>(st.cv[c][e >> 3], e & 7);
          a1 += st.wt[c] * elem<T>(st.cv[c][e >> 3], (e & 7) + 1);
        }
      }
      o[e >> 1] = pack2<T>(a0, a1);
    }
    *reinterpret_cast<uint4*>(A + pp * PITCH + 32 * h) = make_uint4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<uint4*>(A + pp * PITCH + 32 * h + 16) = make_uint4(o[4], o[5], o[6], o[7]);
    *reinterpret_cast<uint4*>(Wl + wr * PITCH + 16 * wc) = st.wv;
  };

  f32x16 acc[2] = {f32x16{}, f32x16{}};
  auto consume = [&](int s) __attribute__((always_inline)) {
    const char* A = smem + (s & 1) * (ABUF + WBUF);
    const char* Wl = A + ABUF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // two 16-deep sub-steps
      const uint4 xf = *reinterpret_cast<const uint4*>(A + (32 * wave + l32) * PITCH + 32 * j + 16 * lh);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint4 wf = *reinterpret_cast<const uint4*>(Wl + (32 * i + l32) * PITCH + 32 * j + 16 * lh);
        Mfma<T>::run(wf, xf, acc[i]);
      }
    }
  };

  // ---- pipeline (S = 9 * ncb is even): step s's operands in set s & 1, issued two steps ahead
  Set st0, st1;
  load_om(0);
  issue(0, st0);
  issue(1, st1);
  for (int s = 0; s < S; s += 2) {
    produce(s, st0);
    if (s + 2 < S) issue(s + 2, st0);
    __syncthreads();
    consume(s);
    produce(s + 1, st1);
    if (s + 3 < S) issue(s + 3, st1);
    __syncthreads();
    consume(s + 1);
  }

  // ---- epilogue: channel rows (r & 3) + 8 (r >> 2) + 4 lh of block i, pixel column l32
  const int mo = m0 + 32 * wave + l32;
  if (mo >= M) return;
  T* dst = reinterpret_cast<T*>(p.out) + (size_t)mo * p.out_ldc + n0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
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

}  // namespace dcn

bool dcn_gemm_supported(long M, int C, int N, int ldx, int om_ldc, int out_ldc, int Kpad) {
  // buffer offsets are 32-bit: the input and weight tensors stay below the out-of-range marker
  if (M * ldx * 2 >= dcn::kOOB || (long)N * Kpad * 2 >= dcn::kOOB) return false;
  return C % (2 * dcn::KS) == 0 && N % dcn::BNC == 0 && ldx % 8 == 0 && om_ldc >= 27 && out_ldc % 4 == 0;
}

int launch_dcn_gemm(const DcnParams& p, int dtype, hipStream_t s) {
  if (!dcn_gemm_supported((long)p.B * p.H * p.W, p.C, p.N, p.ldx, p.om_ldc, p.out_ldc, p.Kpad) || p.Kpad < 9 * p.C) {
    set_error("dcn_gemm: channels must be multiples of 32 (input) / 64 (output), tensors below 2 GB");
    return 1;
  }
  const long M = (long)p.B * p.H * p.W;
  dim3 grid((unsigned)((M + dcn::BMP - 1) / dcn::BMP), (unsigned)(p.N / dcn::BNC));
  if (dtype == F16) {
    hipLaunchKernelGGL(dcn::dcn_gemm<_Float16>, grid, dim3(dcn::NT), dcn::LDS, s, p);
  } else if (dtype == BF16) {
    hipLaunchKernelGGL(dcn::dcn_gemm<__bf16>, grid, dim3(dcn::NT), dcn::LDS, s, p);
  } else {
    set_error("dcn_gemm: fp16/bf16 only");
    return 1;
  }
  TV_HIP(hipGetLastError());
  return 0;
}

}  // namespace tv
