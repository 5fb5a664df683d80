"""Throughput benchmark of the native CenterNet-R18 hot path on MI355X.

One step = one batch of synthetic 640x480 u8 RGB frames (resident in HBM) through
preprocess (fused) -> Centernet forward -> decode (sigmoid + 3x3 peak NMS + exact top-K
+ record gather, K=100, threshold 0.3) -> async copy of the records to pinned host memory
(+ RCCL all-gather of the records across ranks when N > 1).

"R18" = reference Centernet(DLABackbone([2]*5, [128]*6, downsamples=2)) with 4 plain classes
(heads [4, 2, 2]): SURVEY.md §0 maps BASELINE's "CenterNet-R18" to this model.
Weights: seeded synthetic (xavier convs, randomised BN; no checkpoints travel) — the same
recipe as the committed golden fixture tests/golden/model_r18_c128_b1_480x640.npz, so the
parity leg compares the benchmarked kernels against the reference's own outputs.

Extra keys next to the contract's (all measured in this run, on rank 0):
  roofline         dominant conv kernel: per-launch HIP events on the launch stream
  decode_roofline  the decode kernels' achieved HBM GB/s (algorithmic bytes / event time)
  parity           the timed precision's detections on the golden frame (inside a B-frame
                   batch) vs the reference's decode(K=100) records (tests/golden/detcmp.py)
  fp32_value       frames/s of the same step in fp32 (the reference's arithmetic)
  fp32x3           the same in precision "fp32x3" (fp32 operands, each pipelined conv product as three
                   fp16 MFMAs) and its heads' max relative difference from the fp32 engine's
  latency_b1       B=1 hipGraph replay (forward + decode + D2H), in fp16 and in bf16
  host_feed        frames/s when the u8 frames start in pinned host memory (H2D on a
                   side stream, double-buffered, overlapped with the previous step)
  cpu_baseline     the oracle's PyTorch-CPU forward + decode on this host
  api              the drop-in API (Centernet.forward_frames, graph-cached, + decode_records) at
                   the bench batch, beside the hand-built graph's value
  node_b1          the ROS node's per-frame call (centernet_node.py:90-116): CenterpointDLA34
                   model(img) -> decode_keypoints at B=1, fp32 and fp16, graph cache on / off

Launch:  python bench.py [--gpus 1] [--steps 20] [--warmup 5]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints one JSON line. Any TV_* environment knob (kernel-choice overrides, an
alternative library) makes the bench refuse to run unless --allow-env-knobs is given, and
is then stamped into the line as "env_knobs".
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import tauv_vision_amd as tv  # noqa: E402
from tauv_vision_amd.decode import DeviceDecoder  # noqa: E402
from tauv_vision_amd.sharding import RecordGather  # noqa: E402
from tauv_vision_amd.weights import seeded_state_dict  # noqa: E402

HEIGHTS, CHANNELS, DOWNSAMPLES, N_LABELS = [2] * 5, [128] * 6, 2, 4
PEAK_TFLOPS = {"fp16": 2500.0, "bf16": 2500.0, "fp32": 157.3}  # dense MFMA, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
METRIC = "frames/sec CenterNet-R18 640x480 batch=1 & 64; 1/2/4/8 MI355X + %roofline"
GOLDEN = {"r18": ("model_r18_c128_b1_480x640", 105), "dla34": ("dla34_b1_480x640_kp", 202)}


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
        # pinned mirror of the decoder's packed records + counts (one D2H copy per step)
        self.host_packed = torch.empty(self.dec.packed.numel(), dtype=torch.uint8, pin_memory=True)
        nrec = B * K * 10 * 4
        self.host = self.host_packed[:nrec].view(torch.float32).view(B, K, 10)
        self.host_counts = self.host_packed[nrec:].view(torch.int32)
        self.host_gathered = None  # pinned [N * bytes] mirror of the gathered block (N > 1 ranks)

    def decode(self):
        p = self.pred
        return self.dec(p.heatmap, p.size, p.offset, p.depth, 0, self.mc.downsample_ratio, self.mc.in_h,
                        self.mc.in_w, self.thr)

    def compute(self, frames):
        self.eng.forward_u8(frames, self.out)
        return self.decode()

    def finish(self, rec, cnt, gather=None):
        """D2H of this step's records + counts (one copy of the decoder's packed buffer); with N
        ranks, ONE RCCL all-gather of every rank's packed buffer first and one D2H of the gathered
        [N, bytes] block (RecordGather.unpack gives the [N*B, K, 10] records / counts)."""
        if gather is not None:
            buf = gather(self.dec.packed)
            if self.host_gathered is None:
                self.host_gathered = torch.empty(buf.numel(), dtype=torch.uint8, pin_memory=True)
            self.host_gathered.copy_(buf.view(-1), non_blocking=True)
        else:
            self.host_packed.copy_(self.dec.packed, non_blocking=True)

    def step(self, frames, gather=None):
        rec, cnt = self.compute(frames)
        self.finish(rec, cnt, gather)


class GraphStep:
    """The step as one hipGraph (torch.cuda.CUDAGraph): forward_u8 (two concurrent slices, their
    fork / join events captured) + decode + D2H of the records; with N ranks the RCCL all-gather
    and the D2H run eagerly after the replay. The pipeline's workspaces are keyed to the capture
    stream (prepared by an eager warm-up on it); tests/test_gpu_capture.py checks replay == eager
    bit for bit."""

    def __init__(self, pipe, frames, gather, device):
        self.pipe, self.frames, self.gather = pipe, frames, gather
        self.stream = torch.cuda.Stream(device)
        self.stream.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(self.stream):
            for _ in range(2):
                pipe.step(frames, gather)
        torch.cuda.current_stream(device).wait_stream(self.stream)
        torch.cuda.synchronize(device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.rec, self.cnt = pipe.compute(frames)
            if gather is None:
                pipe.finish(self.rec, self.cnt)

    def __call__(self):
        self.graph.replay()
        if self.gather is not None:
            self.pipe.finish(self.rec, self.cnt, self.gather)


def timed(fn, steps, warmup, world=1, device=None):
    """W untimed calls, then K timed ones bracketed by barrier + synchronize; max over ranks."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def load_traffic(kernel, batch, precision, model="r18"):
    """HBM bytes per launch of `kernel` from the committed PMC profile (tools/traffic.py over
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per MI355X_MICROARCH.md;
    profiles/hbm_traffic.json for R18, hbm_traffic_<model>.json for the others), or None when no
    profile of this exact workload is committed."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json" if model == "r18" else f"hbm_traffic_{model}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    if t.get("batch") != batch or t.get("precision") != precision:
        return None
    k = t.get("kernels", {}).get(kernel)
    return None if k is None else k["bytes_per_launch"]


def insitu_launch_ms(eng, inp, out, idx, n_ops, reps):
    """Mean in-situ duration (ms) of launches `idx` over all concurrent slices of one forward of
    `inp`, timed as the timed region runs it: the forward captured as a hipGraph (its slices'
    fork / join and an event record node before every launch on its slice's stream:
    engine.set_insitu) and replayed `reps` times: the mean over all those launches (the two slices
    overlap differently from replay to replay, as in the timed region). Returns (ms, how);
    if the runtime cannot time graph-recorded events, the eager forward with the same events
    (engine.profile_insitu) stands in."""
    dev = inp.device
    fwd = eng.forward_u8 if inp.dtype == torch.uint8 else eng.forward
    B = inp.shape[0]
    try:
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        eng.set_insitu(True)
        try:
            with torch.cuda.stream(st):
                for _ in range(2):
                    fwd(inp, out)
            torch.cuda.current_stream(dev).wait_stream(st)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                fwd(inp, out)
        finally:
            eng.set_insitu(False)
        g.replay()
        torch.cuda.synchronize(dev)
        d = []
        for _ in range(reps):
            g.replay()
            torch.cuda.synchronize(dev)
            d += [t[i] for t in eng.insitu_read(B, st, cap=n_ops) for i in idx]
        return float(np.mean(d)), "graph"
    except RuntimeError as e:
        print(f"bench.py: in-situ graph timing unavailable ({e}); eager in-situ pass instead", file=sys.stderr)
    eng.profile_insitu(inp, out, cap=n_ops)
    per_rep = []
    for _ in range(reps):
        d = [t[i] for t in eng.profile_insitu(inp, out, cap=n_ops) for i in idx]
        per_rep.append(sum(d) / len(d))
    return float(np.median(per_rep)), "eager"


def conv_roofline(pipe, frames, precision, reps=5, model="r18"):
    """Per-launch HIP-event timing. The timed path launches a B-frame forward as concurrent
    slices (engine.slices). The dominant kernel is the conv instance with the largest summed time
    in one slice's serialised pass (tv_engine_profile: events around every launch on the launch
    stream, `reps` passes: the per-op times of BENCH_PROFILE_OUT). `achieved` = its algorithmic
    FLOPs per launch (2*MAC) / its median serialised launch duration (the kernel with
    the chip to itself); `*_insitu` = the same over its launches in the B-frame forward replayed as
    the timed region runs it, with an event record node before every launch (insitu_launch_ms):
    durations stretched by the CUs the concurrent slice holds, and by the event nodes themselves
    (rocprofv3's timed-region durations sit between the two: DESIGN.md §5)."""
    bs = pipe.eng.slices(pipe.B)[0]
    fr = frames[:bs].contiguous()
    out = pipe.eng.alloc_out(bs)
    runs = [pipe.eng.profile(fr, out) for _ in range(reps)]
    # per launch: the median over the passes (what `frac` uses) and the minimum (`frac_best`)
    best = [[o[0], float(np.median([r[i][1] for r in runs])), o[2], o[3]] for i, o in enumerate(runs[0])]
    mins = [min(r[i][1] for r in runs) for i in range(len(runs[0]))]
    if os.environ.get("BENCH_PROFILE_OUT"):
        with open(os.environ["BENCH_PROFILE_OUT"], "w") as f:
            json.dump([{"op": o[0], "ms": o[1], "ms_min": m, "gflop": o[2] / 1e9, "kernel": o[3]}
                       for o, m in zip(best, mins)], f, indent=0)
    conv = [o for o in best if o[2] > 0]
    kern = {}
    for o in conv:
        k = kern.setdefault(o[3], [0, 0.0, 0.0])
        k[0] += 1
        k[1] += o[1]
        k[2] += o[2]
    name, (n, ms, flops) = max(kern.items(), key=lambda kv: kv[1][1])
    ms_min = sum(m for o, m in zip(best, mins) if o[2] > 0 and o[3] == name)
    achieved_iso = flops / (ms * 1e-3) / 1e12
    achieved_best = flops / (ms_min * 1e-3) / 1e12
    peak = PEAK_TFLOPS[precision]
    # in situ: the whole pipe.B-frame forward as the timed region runs it (concurrent slices, grouped
    # launches), an event before each launch on its slice's stream; the dominant kernel's launches
    # then include waiting for CUs the other slice holds — the durations rocprofv3's kernel trace of
    # this bench reports. `achieved` / `frac` = its FLOPs per launch / the mean in-situ launch
    # duration (median over `reps` forwards); the isolated passes above stay as *_isolated.
    idx = [i for i, o in enumerate(best) if o[2] > 0 and o[3] == name]
    ms_situ, how = insitu_launch_ms(pipe.eng, frames[:pipe.B].contiguous(), pipe.eng.alloc_out(pipe.B), idx,
                                    len(best), 4 * reps)
    achieved_situ = flops / n / (ms_situ * 1e-3) / 1e12
    achieved = achieved_iso
    all_ms = sum(o[1] for o in conv)
    all_fl = sum(o[2] for o in conv)
    top = sorted(best, key=lambda o: -o[1])[:6]
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "timing": (f"one slice's launches serialised, median of {reps} passes (best: their minimum); "
                       f"*_insitu ({how}): the {pipe.B}-frame forward captured with an event record node before "
                       f"every launch and replayed as the timed region runs (concurrent slices), mean over "
                       f"{4 * reps} replays ({ms_situ:.4f} ms per launch)"),
            "launch_ms": round(ms / n, 4), "launch_ms_insitu": round(ms_situ, 4),
            "achieved_insitu": round(achieved_situ, 2), "frac_insitu": round(achieved_situ / peak, 4),
            "achieved_best": round(achieved_best, 2), "frac_best": round(achieved_best / peak, 4),
            # the PMC profile is of one pipe.B-frame forward (its launches are the same per-slice
            # launches timed here), so it is looked up by the forward batch
            "traffic": load_traffic(name, pipe.B, precision, model),
            "launch_batch": bs,
            "kernel": (f"{name}: {n} launches per slice forward, avg {ms / n:.4f} ms serialised ({ms_situ:.4f} ms "
                       f"in situ), avg {flops / n / 1e9:.2f} GFLOP/launch"),
            "all_conv": {"launches": len(conv), "ms": round(all_ms, 3), "tflops": round(all_fl / all_ms / 1e9, 1)},
            "per_kernel": {k: {"launches": v[0], "ms": round(v[1], 3), "tflops": round(v[2] / v[1] / 1e9, 1)}
                           for k, v in kern.items()},
            "top_launches": [{"op": o[0], "ms": round(o[1], 4),
                              "tflops": round(o[2] / max(o[1], 1e-9) / 1e9, 1)} for o in top]}


def decode_roofline(pipe, reps=20):
    """HIP-event time of the device decode (on the stream it launches on) over the bench
    batch's head tensor. Algorithmic bytes: the heatmap read once
    (B*C*Ho*Wo*4 B) + per record the size/offset gathers (4 x 4 B) + the record written
    (10 x 4 B) + counts."""
    B, C, H, W, K = pipe.dec.shape
    s = torch.cuda.current_stream()
    pipe.decode()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = None
    for _ in range(reps):
        ev[0].record(s)
        pipe.decode()
        ev[1].record(s)
        ev[1].synchronize()
        t = ev[0].elapsed_time(ev[1])
        best = t if best is None else min(best, t)
    nbytes = B * C * H * W * 4 + B * K * (16 + 40) + B * 4
    gbs = nbytes / (best * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "ms": round(best, 4), "bytes": nbytes,
            "batch": B, "K": K}


def parity_leg(model, oc, mc, arch, B, K, device):
    """The timed precision's engine + decode on the golden frame (placed at frames 0 and B//2+8,
    one per concurrent slice, among random frames) vs the reference's decode(K=100) records
    and Prediction.heatmap stored in tests/golden (data, not oracle code)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from detcmp import peak_parity
    name, seed = GOLDEN[arch]
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    gen = torch.Generator().manual_seed(seed)
    frame = torch.randint(0, 256, (1, mc.in_h, mc.in_w, 3), generator=gen, dtype=torch.uint8)
    frames = torch.randint(0, 256, (B, mc.in_h, mc.in_w, 3), generator=torch.Generator().manual_seed(7),
                           dtype=torch.uint8)
    slots = sorted({0, min(B - 1, B // 2 + 8)})
    for sl in slots:
        frames[sl] = frame[0]
    pipe = Pipeline(model, oc, mc, B, K, 0.0, device)
    pipe.step(frames.to(device))
    torch.cuda.synchronize()
    rec = pipe.host.numpy()
    res = {"agreement": 1.0, "determined": 0, "determined_found": 0, "extra_ok": True, "max_score_err": 0.0,
           "max_box_err": 0.0, "heatmap_drift": 0.0}
    for sl in slots:
        hm = pipe.pred.heatmap[sl].cpu().numpy()
        drift = float(np.abs(hm - g["heatmap"][0]).max())
        pp = peak_parity(rec[sl:sl + 1], g["heatmap"][:1], g["decode_k100_index"][:1], g["decode_k100"][:1],
                         max(drift, 1e-6))
        res["agreement"] = min(res["agreement"], pp["agreement"])
        res["determined"] += pp["determined"]
        res["determined_found"] += pp["determined_found"]
        res["extra_ok"] &= pp["extra_ok"]
        for k in ("max_score_err", "max_box_err"):
            res[k] = max(res[k], pp[k])
        res["heatmap_drift"] = max(res["heatmap_drift"], drift)
    res = {k: (round(v, 7) if isinstance(v, float) else v) for k, v in res.items()}
    # which bar the timed precision meets: the north star's "detections within 1e-4 of reference"
    # is an fp32 statement; the fp32 path meets it (fp32_value; tests/test_gpu_forward.py), the
    # fp16 / bf16 paths are held to detection-level parity (tests/test_gpu_parity_lowp.py)
    # (determined peaks: those whose heatmap score clears the measured drift from the next one)
    res["within_1e-4"] = bool(res["determined_found"] == res["determined"] and res["extra_ok"] and
                              res["max_box_err"] <= 1e-4 and res["max_score_err"] <= 1e-4)
    res.update({"K": K, "frames_checked": len(slots), "batch": B,
                "reference": f"tests/golden/{name}.npz (reference decode K=100 records)"})
    return res


def latency_b1(model, oc, mc, K, thr, device, frames, steps):
    p1 = Pipeline(model, oc, mc, 1, K, thr, device)
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
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    lat = (time.perf_counter() - t1) / steps
    return {"batch": 1, "ms_per_frame": round(lat * 1e3, 4), "frames_per_sec": round(1.0 / lat, 2),
            "path": "hipGraph replay of forward_u8 + decode + D2H", "n_gpus_used": 1}


def host_feed(pipe, frames, steps, warmup, device):
    """Frames start in pinned host memory: step i's H2D copy (side stream, double buffer)
    overlaps step i-1's compute; the compute stream waits for its copy's event."""
    B = pipe.B
    host = [frames.cpu().pin_memory(), frames.cpu().pin_memory()]
    dev = [torch.empty_like(frames), torch.empty_like(frames)]
    copy_s = torch.cuda.Stream(device)
    comp = torch.cuda.current_stream(device)
    done = [torch.cuda.Event(), torch.cuda.Event()]
    used = [torch.cuda.Event(), torch.cuda.Event()]
    for e in used:
        e.record(comp)
    state = {"i": 0}

    def issue(i):
        j = i & 1
        with torch.cuda.stream(copy_s):
            copy_s.wait_event(used[j])
            dev[j].copy_(host[j], non_blocking=True)
            done[j].record(copy_s)

    def step():
        i = state["i"]
        if i == 0:
            issue(0)
        issue(i + 1)  # next step's frames in flight during this step
        comp.wait_event(done[i & 1])
        pipe.step(dev[i & 1])
        used[i & 1].record(comp)
        state["i"] = i + 1

    el = timed(step, steps, warmup)
    nbytes = B * frames[0].numel()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(copy_s)
    with torch.cuda.stream(copy_s):
        dev[0].copy_(host[0], non_blocking=True)
    ev[1].record(copy_s)
    ev[1].synchronize()
    h2d = nbytes / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
    return {"value": round(B * steps / el, 2), "unit": "frames/sec", "batch": B,
            "h2d_GBps": round(h2d, 1), "bytes_per_step": nbytes,
            "path": "pinned host u8 frames -> H2D on a side stream (double-buffered) -> forward_u8 + decode + D2H"}


def api_leg(model, oc, mc, frames, K, thr, steps, value):
    """The drop-in API at the bench batch: `model.forward_frames(frames)` (the reference-shaped
    call; graph-cached: replayed from the 2nd call on) + `decode_records` (device decode, one D2H
    and one host sync per step), against the hand-built GraphStep `value`."""
    from tauv_vision_amd.decode import decode_records
    B = frames.shape[0]

    def step():
        decode_records(model.forward_frames(frames), mc, K, thr)

    el = timed(step, steps, 3)
    v = B * steps / el
    return {"value": round(v, 2), "vs_replay_value": round(v / value, 4), "batch": B,
            "path": "Centernet.forward_frames (hipGraph cache) + decode_records, one host sync per step"}


def node_leg(device, steps):
    """centernet_node.py:90-116 at B=1 with the node's model (CenterpointDLA34, :46): the
    normalised [1, 3, 480, 640] fp32 image on the device -> `model(img)` -> `decode_keypoints(
    prediction, model_config, object_config, M_projection, n_detections=10, keypoint_n_detections=50,
    score_threshold=0.6, keypoint_score_threshold=0.3, keypoint_angle_threshold=0.3)` (a host list of
    detections) per frame; the drop-in default precision fp32, fp32x3 and fp16, with the forward's
    graph cache (default) and eager."""
    from tauv_vision_amd.decode import decode_keypoints
    mc = tv.ModelConfig(HEIGHTS, CHANNELS, 480, 640, DOWNSAMPLES, 1.0)
    M = np.array([[307.0, 0.0, 160.0], [0.0, 307.0, 120.0], [0.0, 0.0, 0.0]])
    img = torch.randn((1, 3, 480, 640), generator=torch.Generator().manual_seed(5)).to(device)
    out = {"model": "CenterpointDLA34 (centernet_node.py:46), keypoint heads", "batch": 1,
           "call": "model(img) -> decode_keypoints(K=10/50, thr 0.6/0.3), host detections"}
    for prec in ("fp32", "fp32x3", "fp16"):
        model, oc, _ = build_model(prec, device, "dla34")
        r = {}
        for mode, replay in (("replay_ms", True), ("eager_ms", False)):
            model.graph_replay = replay

            def step():
                decode_keypoints(model(img), mc, oc, M, 10, 50, 0.6, 0.3, 0.3)

            el = timed(step, steps, 5)
            r[mode] = round(el / steps * 1e3, 4)
        out[prec] = r
        del model
    return out


def fp32_throughput(arch, mc, B, K, thr, device, frames, steps, precision="fp32"):
    """the same step in fp32 on a freshly built model: >= 10 timed steps after 3 warm-ups (round 3
    timed 3 after 1, and the number was bimodal across boxes)"""
    model, oc, _ = build_model(precision, device, arch)
    pipe = Pipeline(model, oc, mc, B, K, thr, device)
    el = timed(lambda: pipe.step(frames), max(10, steps), 3)
    return round(B * max(10, steps) / el, 2)


def fp32x3_leg(arch, mc, B, K, thr, device, frames, steps):
    """precision="fp32x3" (each pipelined conv product as three fp16 MFMAs on fp32 operands): the
    step's frames/s, and its heads against the exact-fp32 engine's on the first 4 bench frames
    (max |difference| / max |fp32 value| per head tensor)"""
    value = fp32_throughput(arch, mc, B, K, thr, device, frames, steps, "fp32x3")
    outs = {}
    for prec in ("fp32", "fp32x3"):
        model, oc, _ = build_model(prec, device, arch)
        eng = model.engine(device, mc.in_h, mc.in_w)
        outs[prec] = eng.forward_u8(frames[:4].contiguous()).float()
        del model, eng
    ref, got = outs["fp32"], outs["fp32x3"]
    rel = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    return {"value": value, "max_rel_diff_vs_fp32": rel, "frames_compared": 4}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


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
            "cpu_model": cpu_model(),
            "sample": f"{n} single frames 640x480 (B=1), fp32 forward + decode(K={K}) in {el:.1f}s; "
                      f"oracle/ PyTorch-CPU restatement, bit-identical to the reference on CPU"}


YOLACT_METRIC = "frames/sec YOLACT protonet + box decode + fast NMS + mask assembly 550x550 batch=32 + %roofline"


def yolact_setup(B, precision, device, rank=0):
    """The YOLACT step's resident inputs and its step function (run_yolact; tools/prof_forward.py
    --model yolact for the PMC passes). Synthetic fpn[0] / head outputs of the reference shapes."""
    from tauv_vision_amd.yolact import (Masknet, YolactConfig, BatchedNMS, box_decode, get_anchor,
                                        assemble_masks_indexed)
    F, k, C1 = 256, 8, 8
    cfg = YolactConfig(550, 550, (24, 48, 96, 192, 384), (1,), (0.1, 0.2), feature_depth=F, n_prototype_masks=k)
    fpn = [(69, 69), (35, 35), (18, 18), (9, 9), (5, 5)]
    anchor = torch.cat([get_anchor(i, s, cfg) for i, s in enumerate(fpn)], 1).to(device)
    A = anchor.shape[1]
    top_k = 100
    net = Masknet(cfg, precision=precision)
    g = torch.Generator(device=device).manual_seed(2000 + rank)
    x = torch.randn((B, F, 69, 69), generator=g, device=device)
    cls = torch.randn((B, A, C1), generator=g, device=device) * 2.0
    enc = torch.randn((B, A, 4), generator=g, device=device) * 0.5
    coeff = torch.randn((B, A, k), generator=g, device=device)
    eng = net.engine(device, 69, 69)
    eng.prepare(B)
    proto = eng.alloc_out(B)                       # [B, 276, 276, 8] fp32 NHWC
    pview = proto[..., :k].permute(0, 3, 1, 2)     # the reference's [B, k, 276, 276]
    bnms = BatchedNMS(B, A, top_k, device)
    masks = torch.empty((B, bnms.K, 276, 276), dtype=torch.float32, device=device)
    host_counts = torch.empty((B,), dtype=torch.int32, pin_memory=True)
    box_out = {}

    def step():
        eng.forward(x, proto)
        box_out["box"] = box = box_decode(enc, anchor, cfg)
        det, cnt = bnms(cls, box, 0.5, 0.05)
        assemble_masks_indexed(pview, coeff, box, det, cnt, out=masks)
        host_counts.copy_(cnt, non_blocking=True)

    return dict(cfg=cfg, anchor=anchor, A=A, top_k=top_k, net=net, x=x, cls=cls, enc=enc, coeff=coeff, eng=eng,
                proto=proto, pview=pview, bnms=bnms, masks=masks, box_out=box_out, step=step, k=k, F=F)


PROTO_TOL = {"fp32": 1e-4, "fp16": 8e-4, "bf16": 6e-3}  # tests/test_yolact.py: ~3x the MI355X drift


def yolact_parity(B, precision, device, name="protonet_f256_k8_b1_69x69"):
    """The timed protonet's kernel instances (F = 256 at fpn[0] 69x69, batch B: the engine's
    concurrent slices) on the reference's golden input, placed at the first frame of every slice
    among random frames, against the golden output samples and per-channel sums stored in
    tests/golden (made by gen_golden_yolact.py from the reference Masknet, masknet.py:45-55)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from recipe import protonet_case, protonet_inputs, protonet_sample_index
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    c = protonet_case(name)
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    sd, x1 = protonet_inputs(c)
    net = Masknet(YolactConfig(550, 550, (24, 48, 96, 192, 384), (1,), (0.1, 0.2), feature_depth=c["F"],
                               n_prototype_masks=c["k"]), precision=precision)
    net.load_state_dict(sd)
    eng = net.engine(device, c["H"], c["W"])
    sizes = eng.slices(B)
    slots = [int(v) for v in np.cumsum([0] + list(sizes[:-1]))]
    x = torch.randn((B, c["F"], c["H"], c["W"]), generator=torch.Generator().manual_seed(77))
    for sl in slots:
        x[sl] = x1[0]
    y = net(x.to(device))
    torch.cuda.synchronize()
    idx = protonet_sample_index(c)
    assert torch.equal(idx, torch.from_numpy(g["sample_index"]).long()), "sample recipe drifted"
    scale = float(np.abs(g["sample"]).max())
    res = {"max_abs_err": 0.0, "max_chan_sum_err": 0.0}
    tol = PROTO_TOL[precision]
    ok = True
    for sl in slots:
        ys = y[sl:sl + 1].cpu()
        got = ys.contiguous().reshape(-1)[idx].numpy()
        err = float(np.abs(got - g["sample"]).max())
        cs = ys.double().sum(dim=(0, 2, 3)).numpy()
        npix = ys.shape[2] * ys.shape[3]
        cerr = np.abs(cs - g["chan_sum"])
        bound = tol * np.abs(g["chan_sum"]) + 4 * tol * max(1.0, scale) * npix ** 0.5
        res["max_abs_err"] = max(res["max_abs_err"], err)
        res["max_chan_sum_err"] = max(res["max_chan_sum_err"], float(cerr.max()))
        ok = ok and err <= tol * max(1.0, scale) and bool((cerr <= bound).all())
    res = {k: round(v, 7) for k, v in res.items()}
    res.update({"ref_absmax": round(scale, 5), "tol": tol, "within_tol": ok, "batch": B, "slices": sizes,
                "frames_checked": len(slots), "samples_per_frame": int(idx.numel()),
                "reference": f"tests/golden/{name}.npz (reference Masknet output samples + channel sums)"})
    return res


def run_yolact(args, world, rank, device):
    """BASELINE config 5 (YOLACT 550x550, batch 32): one step = fpn[0] [B, 256, 69, 69] resident
    in HBM -> Masknet protonet (masknet.py:8-55; F = 256, k = 8 prototypes, train.py:28-33) ->
    box_decode of every anchor (boxes.py:55-61; 6416 anchors at 550x550) -> fast NMS per image
    (nms.py:7-29; top_k 100 as evaluate_batch.py:51, IoU 0.5, confidence 0.05) -> assemble_mask
    of the kept detections (masks.py:8-21, at prototype resolution 276x276) -> counts to host.
    The ResNet backbone / FPN / prediction head are not on the north-star path (they need
    torchvision, absent here): their outputs are synthetic tensors of the reference's shapes."""
    from tauv_vision_amd.yolact import box_decode, assemble_masks_indexed
    B = args.batch if args.batch != 64 else 32
    w = yolact_setup(B, args.precision, device, rank)
    cfg, anchor, A, top_k, net, k, F = w["cfg"], w["anchor"], w["A"], w["top_k"], w["net"], w["k"], w["F"]
    x, cls, enc, coeff, proto, pview = w["x"], w["cls"], w["enc"], w["coeff"], w["proto"], w["pview"]
    eng, bnms, masks, box_out, step = w["eng"], w["bnms"], w["masks"], w["box_out"], w["step"]

    elapsed = timed(step, args.steps, args.warmup, world, device)
    value = world * B * args.steps / elapsed
    flops_frame = eng.geom["flops_per_frame"]
    ranks = dist.get_world_size() if world > 1 else 1
    if world > 1:
        dist.destroy_process_group()  # the legs below are rank 0's alone (no collective)
        if rank != 0:
            return

    # dominant protonet kernel (per-launch HIP events) and the mask kernel's HBM rate
    prof = eng.profile(x, proto)
    kern = {}
    for lab, ms, fl, kname in prof:
        if fl > 0:
            kk = kern.setdefault(kname, [0, 0.0, 0.0])
            kk[0] += 1
            kk[1] += ms
            kk[2] += fl
    name, (n, ms, fl) = max(kern.items(), key=lambda kv: kv[1][1])
    peak = PEAK_TFLOPS[args.precision]
    # in situ (as conv_roofline): the dominant kernel's launches timed inside the forward as the
    # timed region runs it (concurrent slices); the serialised whole-batch profile above is *_isolated
    # the slices' own launches (their workspaces' kernel choice may differ from the whole batch's)
    bs = eng.slices(B)[0]
    prof_s = eng.profile(x[:bs].contiguous(), proto[:bs])
    ks = {}
    for i, (lab, ms_i, fl_i, kname) in enumerate(prof_s):
        if fl_i > 0:
            ks.setdefault(kname, []).append((i, ms_i, fl_i))
    sname, sl = max(ks.items(), key=lambda kv: sum(t[1] for t in kv[1]))
    idx = [t[0] for t in sl]
    ms_situ, how = insitu_launch_ms(eng, x, proto, idx, len(prof_s), 20)
    ach = sum(t[2] for t in sl) / len(sl) / (ms_situ * 1e-3) / 1e12
    roof = {"bound": "mfma", "achieved": round(fl / (ms * 1e-3) / 1e12, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4),
            "timing": (f"the whole batch's launches serialised; *_insitu ({how}): {sname}'s mean launch duration "
                       f"over the forward's concurrent slices (event record nodes, graph replays), 20 replays"),
            "launch_ms_insitu": round(ms_situ, 4),
            "achieved_insitu": round(ach, 2), "frac_insitu": round(ach / peak, 4),
            "traffic": load_traffic(name, B, args.precision, "yolact"), "launch_batch": B,
            "kernel": f"{name}: {n} launches/forward, avg {ms / n:.4f} ms, avg {fl / n / 1e9:.2f} GFLOP/launch",
            "per_kernel": {kn: {"launches": v[0], "ms": round(v[1], 3), "tflops": round(v[2] / v[1] / 1e9, 1)}
                           for kn, v in kern.items()},
            "protonet_ms": round(sum(o[1] for o in prof), 4)}
    s = torch.cuda.current_stream(device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    box = box_out["box"]
    det, cnt = bnms(cls, box, 0.5, 0.05)
    best = None
    for _ in range(10):
        ev[0].record(s)
        assemble_masks_indexed(pview, coeff, box, det, cnt, out=masks)
        ev[1].record(s)
        ev[1].synchronize()
        t = ev[0].elapsed_time(ev[1])
        best = t if best is None else min(best, t)
    kept = int(cnt.sum())
    nbytes = kept * 276 * 276 * 4 + B * 276 * 276 * k * 4 + kept * (k + 4) * 4
    mask_roof = {"bound": "hbm", "achieved": round(nbytes / (best * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                 "unit": "GB/s", "frac": round(nbytes / (best * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                 "ms": round(best, 4), "bytes": nbytes, "masks": kept}
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best_nms = None
    for _ in range(10):
        ev0[0].record(s)
        bx = box_decode(enc, anchor, cfg)
        bnms(cls, bx, 0.5, 0.05)
        ev0[1].record(s)
        ev0[1].synchronize()
        t = ev0[0].elapsed_time(ev0[1])
        best_nms = t if best_nms is None else min(best_nms, t)

    parity = yolact_parity(B, args.precision, device) if not args.no_extras else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import ref_yolact as ry
        sd = {kk: v.detach().cpu() for kk, v in net.state_dict().items()}
        xc, clc, bxc, cfc = x[:1].cpu(), cls[:1].cpu(), box[:1].cpu(), coeff[:1].cpu()
        nfr, t0 = 0, time.perf_counter()
        with torch.no_grad():
            while True:
                pr = ry.masknet(sd, xc)
                bb = ry.box_decode(enc[:1].cpu(), anchor.cpu(), cfg.box_variances)
                d = ry.nms(clc, bb, top_k, 0.5, 0.05)
                ry.assemble_mask(pr[0], cfc[0, d], bb[0, d])
                nfr += 1
                el = time.perf_counter() - t0
                if el >= args.cpu_seconds:
                    break
        cpu = {"value": round(nfr / el, 4), "unit": "frames/sec", "cores": torch.get_num_threads(), "kind": "port",
               "cpu_model": cpu_model(),
               "sample": f"{nfr} single frames (B=1): fp32 protonet + box_decode + nms + assemble_mask in {el:.1f}s; "
                         f"oracle/ PyTorch-CPU restatement, bit-identical to the reference on CPU"}
    if rank == 0:
        line = {
            "metric": YOLACT_METRIC, "value": round(value, 2), "unit": "frames/sec", "n_gpus": world, "ranks": ranks,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic",
            "config": {"workload": f"YOLACT 550x550: Masknet protonet (F={F}, k={k}) on fpn[0] 69x69 -> protos "
                                   f"276x276, box_decode of {A} anchors, fast NMS (top_k {top_k}, IoU 0.5, conf 0.05) "
                                   f"per frame, assemble_mask of the kept detections; batch={B}/GPU",
                       "global_batch": B * world, "parallelism": f"dp{world}"},
            "e2e_tflops": round(value * flops_frame / 1e12, 2),
            "e2e_frac_of_peak": round(value * flops_frame / 1e12 / peak, 4),
            "roofline": roof, "mask_roofline": mask_roof, "nms_ms": round(best_nms, 4),
            "detections_per_frame": round(kept / B, 2), "parity": parity, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


def launch_ranks(n):
    """`--gpus N` (N > 1) run outside torch.distributed.run: start the N ranks as ONE child
    `python -m torch.distributed.run` (rendezvous on 127.0.0.1) before this process touches
    the GPU, and return its exit code (the parent never initialises HIP, so nothing is
    exec'd over a GPU context)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.call(cmd, env=env)


def dryrun_records(frame, K):
    """Deterministic stand-in for one frame's packed decode records (the --cpu-dryrun step)."""
    r = torch.zeros((K, 10), dtype=torch.float32)
    r[:, 0] = torch.arange(K) % N_LABELS
    r[:, 1] = 1.0 - 0.001 * torch.arange(K) - 1e-6 * frame
    r[:, 2:6] = frame + 0.25 * torch.arange(4)[None, :]
    r[:, 7] = torch.arange(K) + 1000 * frame
    return r, frame % (K + 1)


def run_dryrun(args, world, rank):
    """Launcher / sharding / gather plumbing check on CPU (gloo): every rank fills its
    `batch` frames' records (global frames rank*B .. rank*B+B-1) and all-gathers them exactly
    as the GPU step does (RecordGather); rank 0 checks the gathered block against the records
    one process makes for all world*B frames. No kernels run: the line is not a measurement."""
    B, K = args.batch, min(args.k, 8)
    if world > 1:
        dist.init_process_group("gloo")
    rec = torch.zeros((B, K, 10))
    cnt = torch.zeros((B,), dtype=torch.int32)
    for i in range(B):
        rec[i], cnt[i] = dryrun_records(rank * B + i, K)
    gather = RecordGather(B, K, "cpu") if world > 1 else None
    out = {}

    packed = RecordGather.pack(rec, cnt)

    def step():
        if gather is not None:
            gather(packed)  # one collective: records + counts in one buffer
            out["rec"], out["cnt"] = gather.unpack()
        else:
            out["rec"], out["cnt"] = rec, cnt

    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    if rank == 0:
        want = [dryrun_records(f, K) for f in range(world * B)]
        ok = all(torch.equal(out["rec"][f], want[f][0]) and int(out["cnt"][f]) == want[f][1]
                 for f in range(world * B)) and out["rec"].shape[0] == world * B
        print(json.dumps({"metric": "cpu-dryrun (launcher + frame sharding + record all-gather; no kernels)",
                          "value": None, "unit": "frames/sec", "n_gpus": args.gpus,
                          "ranks": dist.get_world_size() if world > 1 else 1,
                          "backend": "gloo" if world > 1 else None, "batch_per_rank": B, "steps": args.steps,
                          "gathered_frames": int(out["rec"].shape[0]), "gather_ok": bool(ok),
                          "wall_s": round(el, 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def env_knobs():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("TV_")}


# TV_* variables that select a library build rather than an engine knob: TV_LIB (this script and
# tools/), TV_TEST_LIB (tests/conftest.py). Everything else is forwarded to the engine, which
# refuses names it does not know.
PACKAGE_KNOBS = ("TV_LIB", "TV_TEST_LIB")


def forward_env_knobs(knobs):
    """Diagnostics (A/B runs, tools/): hand TV_* knobs to the package explicitly — the library
    and the package read no environment. TV_LIB = another build of the library."""
    if not knobs:
        return
    from tauv_vision_amd import _lib
    from tauv_vision_amd.engine import set_diagnostic_knobs
    if "TV_LIB" in knobs:
        _lib.set_library_path(knobs["TV_LIB"])
    set_diagnostic_knobs({k: v for k, v in knobs.items() if k not in PACKAGE_KNOBS})


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
    ap.add_argument("--no-extras", action="store_true", help="skip parity / fp32 / host-feed / decode legs")
    ap.add_argument("--b1-steps", type=int, default=200)
    ap.add_argument("--fp32-steps", type=int, default=10)
    ap.add_argument("--node-steps", type=int, default=100, help="frames per node_b1 timing")
    ap.add_argument("--allow-env-knobs", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="launch the timed step eagerly instead of replaying it as one hipGraph")
    ap.add_argument("--cpu-dryrun", action="store_true",
                    help="CPU/gloo check of the --gpus N launcher, frame sharding and record all-gather (no kernels)")
    ap.add_argument("--model", default="r18", choices=["r18", "dla34", "yolact"],
                    help="r18: the BASELINE CenterNet-R18 (headline); dla34: CenterpointDLA34, heads [4,4,8,2,2]; "
                         "yolact: protonet + post-processing at 550x550, batch 32 (BASELINE config 5)")
    args = ap.parse_args()
    knobs = env_knobs()
    if knobs and not args.allow_env_knobs:
        sys.exit(f"bench.py: TV_* environment knobs set ({knobs}); unset them or pass --allow-env-knobs")
    forward_env_knobs(knobs)

    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # before any GPU call: the ranks are children
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_dryrun:
        return run_dryrun(args, world, rank)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    if args.model == "yolact":
        return run_yolact(args, world, rank, device)

    H, W, B, K = 480, 640, args.batch, args.k
    model, oc, sd = build_model(args.precision, device, args.model)
    mc = tv.ModelConfig(HEIGHTS, CHANNELS, H, W, DOWNSAMPLES, 1.0)
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    frames = torch.randint(0, 256, (B, H, W, 3), generator=gen, device=device, dtype=torch.uint8)
    # detections of every rank on every rank: one RCCL all-gather of the packed records
    gather = RecordGather(B, K, device) if world > 1 else None
    launch = "eager"
    eager_value = None
    if args.eager:
        pipe = Pipeline(model, oc, mc, B, K, args.thr, device)
        step = lambda: pipe.step(frames, gather)  # noqa: E731
    else:
        side = torch.cuda.Stream(device)
        with torch.cuda.stream(side):  # workspaces keyed to the capture stream
            pipe = Pipeline(model, oc, mc, B, K, args.thr, device)
        step = GraphStep(pipe, frames, gather, device)
        launch = "hipGraph replay"
    elapsed = timed(step, args.steps, args.warmup, world, device)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed
    if not args.eager:  # the same step launched eagerly, for comparison (same buffers)
        el_e = timed(lambda: pipe.step(frames, gather), args.steps, 2, world, device)
        eager_value = round(world * B * args.steps / el_e, 2)
    gathered = gather.world * gather.b_local if gather is not None else B
    ranks = dist.get_world_size() if world > 1 else 1
    if world > 1:
        dist.destroy_process_group()  # the legs below are rank 0's alone (no collective)
        if rank != 0:
            return

    # roofline of the dominant kernel (separate pass with per-launch events)
    roof = conv_roofline(pipe, frames, args.precision, model=args.model)
    flops_frame = pipe.eng.geom["flops_per_frame"]
    extras = {}
    if rank == 0 and not args.no_extras:
        extras["decode_roofline"] = decode_roofline(pipe)
        if args.precision != "fp32":
            extras["parity"] = parity_leg(model, oc, mc, args.model, B, K, device)
        extras["host_feed"] = host_feed(pipe, frames, max(5, args.steps // 2), 2, device)

    b1 = None
    if not args.no_b1:
        b1 = {args.precision: latency_b1(model, oc, mc, K, args.thr, device, frames, args.b1_steps)}
        if args.precision == "fp16":  # BASELINE config 2 names bf16 for the latency path
            m16, oc16, _ = build_model("bf16", device, args.model)
            b1["bf16"] = latency_b1(m16, oc16, mc, K, args.thr, device, frames, args.b1_steps)
            del m16
    if rank == 0 and not args.no_extras:
        extras["api"] = api_leg(model, oc, mc, frames, K, args.thr, max(10, args.steps // 2), value)
        if not args.no_b1:
            extras["node_b1"] = node_leg(device, args.node_steps)
    if rank == 0 and not args.no_extras and args.precision != "fp32":
        del pipe
        torch.cuda.synchronize()
        extras["fp32_value"] = fp32_throughput(args.model, mc, B, K, args.thr, device, frames, args.fp32_steps)
        torch.cuda.synchronize()
        extras["fp32x3"] = fp32x3_leg(args.model, mc, B, K, args.thr, device, frames, args.fp32_steps)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline({k: v.detach().cpu() for k, v in sd.items()}, args.cpu_seconds, K, args.thr, args.model)

    if rank == 0:
        workload = (f"CenterNet-R18 (Centernet+DLABackbone [2]*5/[128]*6, ds 2, heads [4,2,2]) " if args.model == "r18"
                    else "CenterpointDLA34 (DLA-34 + DLAUp/IDAUp with DCNv2, heads [4,4,8,2,2]) ")
        line = {
            "metric": METRIC if args.model == "r18" else METRIC.replace("CenterNet-R18", "CenterpointDLA34"),
            "value": round(value, 2), "unit": "frames/sec", "n_gpus": world, "ranks": ranks,
            "gathered_frames_per_step": gathered, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": workload + f"640x480 u8 frames, batch={B}/GPU, forward + decode(K={K}, thr={args.thr})",
                       "global_batch": B * world, "parallelism": f"dp{world} (frame-sharded, RCCL all-gather of "
                                                                  f"detections)" if world > 1 else "dp1"},
            "e2e_tflops": round(value * flops_frame / 1e12, 2),
            "e2e_frac_of_peak": round(value * flops_frame / 1e12 / PEAK_TFLOPS[args.precision], 4),
            "launch": launch, "eager_value": eager_value,
            "roofline": roof, "latency_b1": b1, "cpu_baseline": cpu,
        }
        line.update(extras)
        if knobs:
            line["env_knobs"] = knobs
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
