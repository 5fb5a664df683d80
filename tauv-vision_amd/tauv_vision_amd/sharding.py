"""Frame-sharded data parallelism for the detection path (one process per GPU).

Frames are independent through Centernet.forward and decode (no cross-frame state anywhere
on the path), so a batch of frames splits into contiguous per-rank shards and
the only collective is ONE all-gather of the fixed-size packed detection records
([B_local, K, 10] fp32 + [B_local] int32 counts, ~4 KB per frame at K=100) — over RCCL/xGMI
on GPUs (`all_gather_into_tensor`), over gloo in the CPU tests.
"""
from typing import List, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .decode import REC, Detection


def shard_bounds(n_frames: int, rank: int, world: int) -> Tuple[int, int]:
    """Frames [start, stop) of `rank`: contiguous blocks of ceil(n/world) (the last ones may
    be short or empty), so concatenating the ranks' padded blocks in rank order and trimming
    to n restores the frame order."""
    if world < 1 or not 0 <= rank < world or n_frames < 0:
        raise ValueError(f"bad shard request n={n_frames} rank={rank} world={world}")
    per = -(-n_frames // world)
    return min(n_frames, rank * per), min(n_frames, (rank + 1) * per)


class RecordGather:
    """All-gather of every rank's detection records (static buffers, so the step can be
    graph-captured). Each rank contributes exactly `b_local` frames (pad short shards with
    counts = 0 frames)."""

    def __init__(self, b_local: int, k: int, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.rec = torch.empty((self.world, b_local, k, REC), dtype=torch.float32, device=self.device)
        self.cnt = torch.empty((self.world, b_local), dtype=torch.int32, device=self.device)
        self._into_tensor = dist.get_backend(group) == "nccl"

    def __call__(self, rec: torch.Tensor, cnt: torch.Tensor):
        if self._into_tensor:
            dist.all_gather_into_tensor(self.rec, rec, group=self.group)
            dist.all_gather_into_tensor(self.cnt, cnt, group=self.group)
        else:
            dist.all_gather(list(self.rec.unbind(0)), rec, group=self.group)
            dist.all_gather(list(self.cnt.unbind(0)), cnt, group=self.group)
        return self.rec.flatten(0, 1), self.cnt.flatten(0, 1)


def records_to_detections(records: np.ndarray, counts: np.ndarray, has_depth: bool) -> List[List[Detection]]:
    """Host conversion of packed records [B, K, 10] / counts [B] into decode()'s
    List[List[Detection]] (decode.py:206-236 field meaning)."""
    out = []
    for b in range(records.shape[0]):
        dets = []
        for r in records[b, :int(counts[b])]:
            d = Detection(label=torch.tensor(int(r[0])), score=torch.tensor(r[1]), y=float(r[2]), x=float(r[3]),
                          h=float(r[4]), w=float(r[5]))
            if has_depth:
                d.depth = float(r[6])
            dets.append(d)
        out.append(dets)
    return out
