"""Throughput benchmark of the native CenterNet-R18 hot path on MI355X.

One step = one batch of synthetic 640x480 u8 RGB frames (resident in HBM) through
preprocess (fused) -> Centernet forward -> decode (sigmoid + 3x3 peak NMS + exact top-K
+ record gather, K=100, threshold 0.3) -> async copy of the records to pinned host memory
(+ RCCL all-gather of the records across ranks when N > 1).

"R18" = reference Centernet(DLABackbone([2]*5, [128]*6, downsamples=2)) with 4 plain classes
(heads [4, 2, 2]): SURVEY.md §0 maps BASELINE's "CenterNet-R18" to this model.
Weights: seeded synthetic (xavier convs, randomised BN; no checkpoints travel).

Launch:  python bench.py [--gpus 1] [--steps 20] [--warmup 5]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import tauv_vision_amd as tv  # noqa: E402
from tauv_vision_amd.decode import DeviceDecoder  # noqa: E402
from tauv_vision_amd.sharding import RecordGather  # noqa: E402
from tauv_vision_amd.weights import seeded_state_dict  # noqa: E402

HEIGHTS, CHANNELS, DOWNSAMPLES, N_LABELS = [2] * 5, [128] * 6, 2, 4
PEAK_TFLOPS = {"fp16": 2500.0, "bf16": 2500.0, "fp32": 157.3}  # dense MFMA, MI355X_MICROARCH.md
METRIC = "frames/sec CenterNet-R18 640x480 batch=1 & 64; 1/2/4/8 MI355X + %roofline"


def build_model(precision, device, arch="r18"):
    A = tv.AngleConfig
    if arch == "dla34":  # DLA34 with the keypoint heads [4, 4, 8, 2, 2]
        oc = tv.ObjectConfigSet([tv.ObjectConfig(f"class{i}", A(False, None), A(False, None), A(False, None), False,
                                                 True, [(0.0, 0.0, 0.0)]) for i in range(N_LABELS)])
        model = tv.CenterpointDLA34(oc, precision=precision)
    else:
        oc = tv.ObjectConfigSet([tv.ObjectConfig(f"class{i}", A(False, None), A(False, None), A(False, None), False,
                                                 False, None) for i in range(N_LABELS)])
        model = tv.Centernet(tv.DLABackbone(HEIGHTS, CHANNELS, DOWNSAMPLES), oc, precision=precision)
    sd = seeded_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()])
    model.load_state_dict(sd)
    return model.to(device).eval(), oc, sd


class Pipeline:
    """Static buffers for one (batch) configuration: forward_u8 + device decode + async D2H."""

    def __init__(self, model, oc, mc, B, K, thr, device):
        self.eng = model.engine(device, mc.in_h, mc.in_w)
        self.eng.prepare(B)
        self.out = self.eng.alloc_out(B)
        self.pred = tv.centernet.prediction_from_nhwc(self.out, oc)
        C, H, W = self.pred.heatmap.shape[1:]
        self.dec = DeviceDecoder(B, C, H, W, K, device)
        self.mc, self.thr, self.B = mc, thr, B
        self.host = torch.empty((B, K, 10), dtype=torch.float32, pin_memory=True)
        self.host_counts = torch.empty((B,), dtype=torch.int32, pin_memory=True)

    def step(self, frames, gather=None):
        self.eng.forward_u8(frames, self.out)
        p = self.pred
        rec, cnt = self.dec(p.heatmap, p.size, p.offset, p.depth, 0, self.mc.downsample_ratio, self.mc.in_h,
                            self.mc.in_w, self.thr)
        if gather is not None:
            gather(rec, cnt)
        self.host.copy_(rec, non_blocking=True)
        self.host_counts.copy_(cnt, non_blocking=True)


def load_traffic(kernel, batch, precision):
    """HBM bytes per launch of `kernel` from the committed PMC profile (tools/traffic.py over
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per MI355X_MICROARCH.md),
    or None when no profile of this exact workload is committed."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    if t.get("batch") != batch or t.get("precision") != precision:
        return None
    k = t.get("kernels", {}).get(kernel)
    return None if k is None else k["bytes_per_launch"]


def conv_roofline(pipe, frames, precision, reps=3):
    """Per-launch HIP-event timing of one forward (tv_engine_profile: events recorded on the
    launch stream around every launch; a separate pass after the timed region). The timed path
    launches a B-frame forward as concurrent slices (engine.slices), so the pass times one
    slice's launches — the same kernel instances, grids and per-launch work rocprofv3 reports.
    The dominant kernel is the conv instance with the largest summed time; achieved = its
    algorithmic FLOPs (2*MAC per launch) / its summed launch durations (= FLOPs per
    launch / average launch duration)."""
    bs = pipe.eng.slices(pipe.B)[0]
    fr = frames[:bs].contiguous()
    out = pipe.eng.alloc_out(bs)
    best = None
    for _ in range(reps):
        ops = pipe.eng.profile(fr, out)
        if best is None:
            best = [list(o) for o in ops]
        else:
            for b, o in zip(best, ops):
                b[1] = min(b[1], o[1])
    if os.environ.get("TV_PROFILE_OUT"):
        with open(os.environ["TV_PROFILE_OUT"], "w") as f:
            json.dump([{"op": o[0], "ms": o[1], "gflop": o[2] / 1e9, "kernel": o[3]} for o in best], f, indent=0)
    conv = [o for o in best if o[2] > 0]
    kern = {}
    for o in conv:
        k = kern.setdefault(o[3], [0, 0.0, 0.0])
        k[0] += 1
        k[1] += o[1]
        k[2] += o[2]
    name, (n, ms, flops) = max(kern.items(), key=lambda kv: kv[1][1])
    achieved = flops / (ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[precision]
    all_ms = sum(o[1] for o in conv)
    all_fl = sum(o[2] for o in conv)
    top = sorted(best, key=lambda o: -o[1])[:6]
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": load_traffic(name, bs, precision),
            "launch_batch": bs,
            "kernel": f"{name}: {n} launches/forward, avg {ms / n:.4f} ms, avg {flops / n / 1e9:.2f} GFLOP/launch",
            "all_conv": {"launches": len(conv), "ms": round(all_ms, 3), "tflops": round(all_fl / all_ms / 1e9, 1)},
            "per_kernel": {k: {"launches": v[0], "ms": round(v[1], 3), "tflops": round(v[2] / v[1] / 1e9, 1)}
                           for k, v in kern.items()},
            "top_launches": [{"op": o[0], "ms": round(o[1], 4),
                              "tflops": round(o[2] / max(o[1], 1e-9) / 1e9, 1)} for o in top]}


def cpu_baseline(sd, seconds, K, thr, arch="r18"):
    """The repo's PyTorch-CPU restatement of the reference path (oracle/), fp32, timed on a
    bounded sample of single 640x480 frames (forward + decode) on this host's cores."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import oracle
    from recipe import normalize
    # the host's share of cores: torch's default (OMP_NUM_THREADS; 16 on the GPU box). Setting
    # os.cpu_count() there oversubscribes the box's CPU share by ~16x.
    g = torch.Generator().manual_seed(1234)
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            u8 = torch.randint(0, 256, (1, 480, 640, 3), generator=g, dtype=torch.uint8)
            img = normalize(u8.permute(0, 3, 1, 2).float() / 255.0)
            if arch == "dla34":
                from oracle.ref_dla34 import centerpoint_dla34_forward
                pred = centerpoint_dla34_forward({k[len("model."):]: v for k, v in sd.items()}, img,
                                                 {"keypoints": True}, 5)
            else:
                pred = oracle.centernet_forward(sd, img, HEIGHTS, DOWNSAMPLES, {})
            oracle.decode(pred, 480, 640, DOWNSAMPLES, K, thr)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": round(n / el, 4), "unit": "frames/sec", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} single frames 640x480 (B=1), fp32 forward + decode(K={K}) in {el:.1f}s; "
                      f"oracle/ PyTorch-CPU restatement, bit-identical to the reference on CPU"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="frames per GPU per step")
    ap.add_argument("--precision", default="fp16", choices=["fp16", "bf16", "fp32"])
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--thr", type=float, default=0.3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-b1", action="store_true")
    ap.add_argument("--b1-steps", type=int, default=200)
    ap.add_argument("--model", default="r18", choices=["r18", "dla34"],
                    help="r18: the BASELINE CenterNet-R18 (headline); dla34: CenterpointDLA34, heads [4,4,8,2,2]")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    H, W, B, K = 480, 640, args.batch, args.k
    model, oc, sd = build_model(args.precision, device, args.model)
    mc = tv.ModelConfig(HEIGHTS, CHANNELS, H, W, DOWNSAMPLES, 1.0)
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    frames = torch.randint(0, 256, (B, H, W, 3), generator=gen, device=device, dtype=torch.uint8)
    pipe = Pipeline(model, oc, mc, B, K, args.thr, device)

    # detections of every rank on every rank: one RCCL all-gather of the packed records
    gather = RecordGather(B, K, device) if world > 1 else None

    for _ in range(args.warmup):
        pipe.step(frames, gather)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step(frames, gather)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # roofline of the dominant kernel (separate pass with per-launch events)
    roof = conv_roofline(pipe, frames, args.precision)
    flops_frame = pipe.eng.geom["flops_per_frame"]

    b1 = None
    if not args.no_b1:
        p1 = Pipeline(model, oc, mc, 1, K, args.thr, device)
        f1 = frames[:1].contiguous()
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _ in range(3):
                p1.step(f1)
        torch.cuda.current_stream(device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            p1.step(f1)
        for _ in range(10):
            graph.replay()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.b1_steps):
            graph.replay()
        torch.cuda.synchronize()
        lat = (time.perf_counter() - t1) / args.b1_steps
        b1 = {"batch": 1, "ms_per_frame": round(lat * 1e3, 4), "frames_per_sec": round(1.0 / lat, 2),
              "path": "hipGraph replay of forward_u8 + decode + D2H", "n_gpus_used": 1}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline({k: v.detach().cpu() for k, v in sd.items()}, args.cpu_seconds, K, args.thr, args.model)

    if rank == 0:
        workload = (f"CenterNet-R18 (Centernet+DLABackbone [2]*5/[128]*6, ds 2, heads [4,2,2]) " if args.model == "r18"
                    else "CenterpointDLA34 (DLA-34 + DLAUp/IDAUp with DCNv2, heads [4,4,8,2,2]) ")
        line = {
            "metric": METRIC if args.model == "r18" else METRIC.replace("CenterNet-R18", "CenterpointDLA34"), "value": round(value, 2), "unit": "frames/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": workload + f"640x480 u8 frames, batch={B}/GPU, forward + decode(K={K}, thr={args.thr})",
                       "global_batch": B * world, "parallelism": f"dp{world} (frame-sharded, RCCL all-gather of "
                                                                  f"detections)" if world > 1 else "dp1"},
            "e2e_tflops": round(value * flops_frame / 1e12, 2),
            "e2e_frac_of_peak": round(value * flops_frame / 1e12 / PEAK_TFLOPS[args.precision], 4),
            "roofline": roof, "latency_b1": b1, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
