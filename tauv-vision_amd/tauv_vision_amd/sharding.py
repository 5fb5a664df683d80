"""Frame-sharded data parallelism for the detection path (one process per GPU).

Frames are independent through Centernet.forward and decode (no cross-frame state anywhere
on the path), so a batch of frames splits into contiguous per-rank shards and
the only collective is ONE all-gather of the fixed-size packed detection records
([B_local, K, 10] fp32 + [B_local] int32 counts in one byte buffer, ~4 KB per frame at K=100) —
over RCCL/xGMI on GPUs (`all_gather_into_tensor`), over gloo in the CPU tests.
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
    """All-gather of every rank's detection records as ONE collective: each rank contributes its
    decoder's packed buffer (DeviceDecoder.packed: [b_local, K, 10] fp32 records then [b_local]
    int32 counts, one allocation), gathered into a static [world, bytes] buffer (so the step can be
    graph-captured). Each rank contributes exactly `b_local` frames (pad short shards with
    counts = 0 frames)."""

    def __init__(self, b_local: int, k: int, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.b_local, self.k = b_local, k
        self.nrec = b_local * k * REC
        self.bytes = (self.nrec + b_local) * 4
        self.buf = torch.empty((self.world, self.bytes), dtype=torch.uint8, device=self.device)
        self._into_tensor = dist.get_backend(group) == "nccl"

    @staticmethod
    def pack(rec: torch.Tensor, cnt: torch.Tensor) -> torch.Tensor:
        """records [b, K, 10] fp32 + counts [b] int32 -> the packed byte layout (a copy; the device
        decoder writes this layout in place)."""
        return torch.cat((rec.contiguous().view(-1).view(torch.uint8), cnt.contiguous().view(-1).view(torch.uint8)))

    def __call__(self, packed: torch.Tensor) -> torch.Tensor:
        """packed: this rank's uint8 [bytes] buffer; returns the gathered [world, bytes] buffer."""
        if packed.numel() != self.bytes or packed.dtype != torch.uint8:
            raise ValueError(f"packed records: expected {self.bytes} uint8, got {packed.numel()} {packed.dtype}")
        if self._into_tensor:
            dist.all_gather_into_tensor(self.buf.view(-1), packed, group=self.group)
        else:
            dist.all_gather(list(self.buf.unbind(0)), packed, group=self.group)
        return self.buf

    def unpack(self, buf: torch.Tensor = None):
        """The gathered buffer (device, or its host copy) -> records [world*b, K, 10] fp32 and counts
        [world*b] int32, frames in rank order."""
        buf = self.buf if buf is None else buf.view(self.world, self.bytes)
        rec = buf[:, :self.nrec * 4].contiguous().view(torch.float32).view(self.world * self.b_local, self.k, REC)
        cnt = buf[:, self.nrec * 4:].contiguous().view(torch.int32).view(self.world * self.b_local)
        return rec, cnt


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
