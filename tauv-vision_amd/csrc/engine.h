#pragma once
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common.h"
#include "planner.h"

namespace tv {

struct Packed {
  void* w = nullptr;       // [Npad][Kpad] compute dtype
  void* w_c3 = nullptr;    // conv3x3.hip / conv3x3s2.hip k-step-major copy (made on first use)
  void* w_c3h = nullptr;   // conv3x3.hip copy for 64-channel half tiles (ni = 2)
  void* w_c3e = nullptr;   // conv3x3.hip copy for the fused-heads body when its swizzle differs (conv3x3_k16)
  void* w_ss2 = nullptr;   // stem_s2.hip k-step-ordered copy of block0.conv1's weights (made on first use)
  void* w_burst = nullptr; // conv_burst.hip [32-channel tile][k-step][lane] copy (made on first use)
  void* w_x3 = nullptr;    // conv_pipe.hip X3 copy of the fp32 weights: hi / lo fp16 halves (made on first use)
  void* w_ct3 = nullptr;   // convt3.hip fragments of a whole ConvTranspose2d(3, s2) (its phase-(0,0) op)
  float* bias = nullptr;   // [Npad]
  int Npad = 0, Kpad = 0;
  std::vector<int> seg_ksteps;
  // block-diagonal 1x1 heads only: MFMA A-fragments per 128-channel tile of the stacked 3x3
  // heads' output, for the fused epilogue (conv3x3 EPI 1); head_ok = 0 when not representable
  int head_ok = 0;
  void* head_w = nullptr;
  float* head_b = nullptr;
  int head_row0[16] = {}, head_nrows[16] = {};
};

struct Workspace {
  int B = 0;
  void* arena = nullptr;
  size_t bytes = 0;
  std::vector<size_t> off;          // per tensor
  std::vector<ConvParams> params;   // per op (host copy)
  ConvParams* dparams = nullptr;    // per op (device copy)
  std::vector<int> use_pipe;        // per op: 1 = conv_pipe (256-pixel tiles), 0 = conv_igemm
  std::vector<int> c3_tw, c3_grid;  // per op: > 0 = persistent conv3x3 (tile width, workgroups); overrides all
  std::vector<int> c3_res;          // per op: 1 = conv3x3 with the 1x1 residual segment (RES)
  std::vector<int> c3_ni;           // per op: channel fragments per wave (4: 128-channel tiles, 2: 64)
  std::vector<int> c3_nw;           // per op: waves per workgroup (8: one per CU, 4: two per CU)
  std::vector<int> s2_grid;         // per op: > 0 = persistent stride-2 conv3x3s2 (workgroups)
  std::vector<int> head_fused;      // per op: 1 = stacked 3x3 heads with the 1x1 heads fused in
  std::vector<int> head_skip;       // per op: 1 = block-diagonal 1x1 heads done by the op before
  std::vector<int> small;           // per op: 1 = narrow-channel 3x3 conv on conv_small.hip
  std::vector<int> lat;             // per op: 1 = split-K small-level GEMM on conv_lat.hip
  std::vector<int> burst;           // per op: 1 = one-shot small-level conv on conv_burst.hip
  std::vector<BurstParams> bparams; // per op: its conv_burst launch geometry
  std::vector<int> c1x1;            // per op: 1 = streaming 1x1 conv (Roots) on conv1x1.hip
  std::vector<int> dcn_skip;        // per op: 1 = DCN sampling done inside the next op's fused kernel
  std::vector<DcnParams> dcn;       // per op: fused DCNv2 launch (dcn.hip) when dcn[i].x != null
  std::vector<int> convt;           // per op: 1 = OP_CONVT_ADD on convt.hip
  std::vector<ConvTParams> tparams; // per op: convt.hip launch parameters
  std::vector<int> ct3;             // per op: 1 = ConvTranspose2d(3, s2) phase (0,0) launching all four on convt3.hip,
                                    // 2 = a phase that launch covers
  std::vector<ConvT3Params> ct3p;   // per op: convt3.hip launch parameters (ct3 == 1)
  KStep* dks = nullptr;             // k-step descriptors of all pipelined ops
  float* slab = nullptr;            // conv_lat split-K partial tiles (one region per slot of a grouped launch)
  unsigned* cnt = nullptr;          // conv_lat split-K tickets, one per tile and slot, zeroed per forward
  float* pslab = nullptr;           // conv_pipe split-K partial tiles (one layer at a time)
  unsigned* pcnt = nullptr;         // conv_pipe split-K tickets, one per tile (reset by the last slice)
  float* dslab = nullptr;           // dcn_gemm64 split-K partial accumulators (one layer at a time)
  unsigned* dcnt = nullptr;         // dcn_gemm64 split-K tickets, one per tile (reset by the last slice)
  std::vector<int> level;           // per op: dependency level (the arena's time; plan order when not grouping)
  std::vector<int> order;           // the ops in execution order: by level, then plan order
  std::vector<std::vector<int>> groups;  // the schedule: conv_lat layers of one level in one launch, others alone
  size_t cnt_bytes = 0;
  std::vector<std::string> kname;   // per op: kernel instance name (diagnostics), filled lazily
  std::vector<hipEvent_t> gev;      // forward_insitu(): one event before each schedule group + one after the last
};

struct Engine {
  tv_model_desc desc{};
  Plan plan;
  int device = 0;
  int dtype = F32;
  std::vector<Packed> packed;  // per op
  size_t weight_bytes = 0;
  void* zero_page = nullptr;   // 256 zero bytes: padding source for LDS-DMA
  int pipe_mode = 1;           // -1 auto (>= 256 tiles), 0 never, 1 whenever representable (env TV_CONV_PIPE)
  int c3_tw_force = 0;         // conv3x3 tile width override (env TV_C3_TW = 16 / 32)
  int s2_min_tiles = 1;        // stride-2 halo kernel from this many tiles (env TV_S2_MINTILES; -1 = cu_count; measured:
                               // at B=1 the halo kernel beats the implicit GEMM on the small levels too)
  int c3_ni_force = 0;         // conv3x3 channel tile: 0 = by grid rounds, 2 / 4 forced (env TV_C3_NI)
  int c3_nw_mode = 0;          // conv3x3 workgroup size: 0 = 4-wave where eligible, 8 = always 8 (TV_C3_NW)
  int c3_half_cost = 70;       // cost of a 64-channel half tile in % of a full one (env TV_C3_HALF_COST, 0 = never;
                               // swept r5: 70-85 best at B=64, 100 loses B=1, profiles/r5/half_cost_sweep.txt)
  int csm_halo = 2;            // conv_small.hip variant (knob TV_CSM_HALO): 0 = register gathers, 1 = LDS-halo
                               // tiles, one per workgroup, 2 = LDS-halo tiles on a persistent grid (measured r5:
                               // fastest for all three DLA-34 layers, profiles/r5/csm_halo.txt)
  int csm_variant(int stride) const { return stride > 0 ? csm_halo : 0; }
  int conv3_min_pix = 1;       // halo kernels only for frames of >= this many pixels (env TV_CONV3_MINPIX)
  int s2_mode = 1;             // stride-2 halo kernel for eligible fp16/bf16 layers (env TV_CONV3S2=0 off)
  int conv3_mode = 1;          // persistent halo 3x3 kernel for eligible fp16/bf16 layers (env TV_CONV3=0 off)
  int cu_count = 256;          // compute units (persistent grids)
  int headfuse_mode = 1;       // fuse the 1x1 heads into the 3x3 heads epilogue (env TV_HEADFUSE=0 off)
  int convt_mode = 1;          // convt.hip for eligible fp16/bf16 up-paths (knob TV_CONVT=0 off)
  int stem_mode = 1;           // fused staging + stem kernel for fp16/bf16 (env TV_STEM=0 off)
  int lat_mode = 1;            // conv_lat.hip for layers whose chosen kernel fills < lat_units work units
                               // (env TV_LAT=0 off)
  int dcn64_mode = 1;          // fused DCN with 64-channel k-steps (full-line gathers) when C % 64 == 0 (knob TV_DCN64:
                               // 0 dcn_gemm, 2 dcn_gemm64 on 64-pixel tiles, 3 the LDS-window dcn_win for C == N == 64:
                               // bit-equal, measured 194 vs 187 us per 120x160 layer, so not the default; 5 dcn_gemm64d:
                               // the corner gathers two k-steps ahead)
  int lat_units = -1;          // threshold in work units (env TV_LAT_UNITS; -1 = cu_count)
  int dcn_split_max = 4;       // dcn_gemm64 split-K over tap ranges for layers whose tiles fill <= half the CUs
                               // (the latency path: DLA-34 at B=1), at most this many slices (knob TV_DCN_SPLIT, <2 off;
                               // B=1 DLA-34 1.263 -> 1.149 ms; 6 / 9 slices equal, counting 2 / 4 resident
                               // workgroups per CU as slots slower: 1.186 / 1.225 ms)
  int c1x1_mode = 1;           // stride-1 1x1 convs on the streaming kernel (knob TV_C1X1; 2 = N <= 128 only)
  int lat_group = 1;           // independent conv_lat layers of one dependency level in one launch (knob TV_LATGROUP)
  int lat_group_max_b = 8;     // ... on workspaces of at most this many frames (knob TV_LATGROUP_B)
  int ct3_mode = 1;            // ConvTranspose2d(3, s2, p1) phases in one convt3.hip launch (knob TV_CT3=0 off)
  int burst_mode = 1;          // conv_burst.hip for the small conv_lat layers it represents (knob TV_BURST=0 off,
                               // 2 = every layer it represents: diagnostics / tests)
  int lat_split_max = 4;       // conv_lat workgroups per tile (split-K) on under-filled layers (knob TV_LAT_SPLIT, 1 = off)
  int f32x3 = 0;               // fp32 engines: conv_pipe products as three fp16 MFMAs (hi/lo split, ~22-bit
                               // operands, fp32 accumulation) instead of v_mfma_f32_32x32x2_f32 (knob TV_F32X3)
  int pipe_split_mode = 1;     // conv_pipe split-K on under-filled layers: 0 off, 1 fp32 only, 2 every dtype (TV_PIPE_SPLIT)
  int pipe_split_max = 16;     // ... at most this many slices per tile (knob TV_PIPE_SPLIT_MAX)
  int pipe_split_red = 5;      // ... hand-off cost per slice in tenths of a k-step (knob TV_PIPE_SPLIT_RED)
  int lat_f32 = 1;             // conv_lat.hip on the fp32 path too (knob TV_LAT_F32=0 off)
  int lat_split_max_f32 = 8;   // ... its split-K cap there (knob TV_LAT_SPLIT_F32)
  int lat_split_min_nks = 32;  // ... for layers of at least this many k-steps (knob TV_LAT_SPLIT_MIN)
  int stamp_op = -1;           // diagnostics: op whose conv3x3 launch gets a stamp buffer (knob TV_C3_STAMPS=op:ptr)
  unsigned long long* stamp_buf = nullptr;
  int profiled_u8 = 0;         // input kind of the last profile() (kernel instance names)
  int stem_op = -1;            // op index of the 7x7 stem conv when it runs on stem.hip, else -1
  int stemfuse_mode = 1;       // stem + block0.conv1 (+ the residual's stride-2 stem samples) in one launch
                               // (stem_s2.hip) when the plan has that shape (knob TV_STEMFUSE=0 off)
  int ss2_op = -1;             // op index of block0.conv1 when it runs fused with the stem, else -1
  // concurrent slices: a batch of >= slices * slice_min frames runs as `slices` near-equal parts,
  // the first on the caller's stream and the others on side streams (fork / join events), so one
  // slice's latency-bound small layers and grid tails overlap another's large layers
  // (knob TV_SLICES: count, 1 = off; TV_SLICE_SIZES=a,b,...: explicit sizes for experiments)
  static constexpr int kMaxSlices = 8;  // == TV_MAX_SLICES (include/tauv_vision_amd.h)
  int slices = 2;
  int slice_min = 8;
  int insitu = 0;     // forward_insitu() in progress: run_all records the group events
  int slice_lag = 0;  // diagnostics (knob TV_SLICE_LAG): slice 1 starts after slice 0's op `slice_lag`
  std::vector<int> slice_sizes_env;
  std::vector<int> slice_sizes(int B) const;
  struct SideStreams {
    std::vector<hipStream_t> s;
    hipEvent_t fork = nullptr;
    std::vector<hipEvent_t> join;
  };
  std::map<void*, SideStreams> side;  // per caller stream
  std::mutex mu;
  std::map<std::pair<void*, int>, Workspace*> workspaces;
  std::unordered_map<std::string, std::pair<const float*, int64_t>> host_w;  // during create only

  ~Engine();
  int create(const tv_model_desc& d, const tv_weight_view* w, int n, int dev,
             const std::vector<std::pair<std::string, std::string>>& knobs = {});
  int get_workspace(int B, hipStream_t s, Workspace** out);
  int prepare(int B, hipStream_t s);  // workspaces (and side stream) for forward(B) on s
  int trim();                         // free every cached workspace (no forward may be in flight)
  int forward(const void* input, int input_u8, int B, float* out, hipStream_t s);
  int profile(const void* input, int input_u8, int B, float* out, hipStream_t s, float* ms, double* flops, int cap, int* n_ops);
  // the forward as it runs (concurrent slices, schedule groups) with an event before each launch on
  // its slice's stream: ms[k * cap + i] = launch time of op i in slice k (a grouped launch's time on
  // its first op), *n_slices slices, synchronous (diagnostic: in-situ per-launch durations)
  int forward_insitu(const void* input, int input_u8, int B, float* out, hipStream_t s, float* ms, int cap,
                     int* n_slices);
  // the times the group events of the B-frame forward on s last recorded (an eager forward_insitu,
  // or the replay of a graph captured while `insitu` was set)
  int insitu_read(int B, hipStream_t s, float* ms, int cap, int* n_slices);
  const char* op_kernel(int B, size_t i);

 private:
  const float* weight(const std::string& name, int64_t numel);
  int fold(const std::string& conv, const std::string& bn, int cout, std::vector<double>& scale,
           std::vector<double>& shift);
  int pack_op(size_t i);
  int make_workspace(int B, Workspace* ws);
  int run_op(size_t i, Workspace* ws, const void* input, int input_u8, float* out, hipStream_t s);
  int run_all(const void* input, int input_u8, int B, float* out, hipStream_t s, size_t op0 = 0,
              size_t op1 = (size_t)-1);
  int get_side(hipStream_t s, int n, SideStreams** out);
};

}  // namespace tv
