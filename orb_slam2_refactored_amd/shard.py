"""Batched many-frame mode across GPUs (BASELINE.json configs[4]).

Frames are independent, so the work is sharded by frame over one process per GPU with no
data-path collective.  The one exchange is the loop-closure descriptor all-gather: after a rank
has extracted its shard, every rank receives every frame's padded keypoint / descriptor slots
(the input of KeyFrameDatabase::DetectLoopCandidates-style candidate search, which in the
reference walks all keyframes' descriptors, src/KeyFrameDatabase.cc:68-171).

The exchange is asynchronous and double-buffered: the collectives for step k are issued on the
process group's own stream (RCCL over xGMI with backend "nccl"), and step k+1's kernels are
enqueued on the compute stream right behind them.  A set of slot buffers is written again
only after its gather has been waited on (`SlotExchange.acquire`), which orders the compute
stream after the collective without a host sync.  The same class runs on `gloo` with CPU
tensors, which is how tests/test_shard_gloo.py covers the N>1 path here.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [start, start+count) of n_total frames for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world) or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def cross_shard_predecessor(rank: int, world: int, frames_per_rank: int) -> int:
    """Index, in the gathered slot buffer (rank-major: rank r's local frame f at r*frames_per_rank + f),
    of the predecessor of this rank's first frame: global frame g0 - 1, i.e. rank r-1's last frame
    (wrapping to the job's last frame for rank 0).  §8d C5: "frame i matched to i-1"."""
    if world <= 0 or not (0 <= rank < world) or frames_per_rank <= 0:
        raise ValueError("bad shard arguments")
    return (rank * frames_per_rank - 1) % (world * frames_per_rank)


@dataclass
class Slots:
    """One rank's extraction output for a batch of frames (device or CPU tensors)."""
    kps: torch.Tensor      # (B, cap, 7) int32, orbx_keypoint layout
    desc: torch.Tensor     # (B, cap, 32) uint8
    counts: torch.Tensor   # (B,) int32

    @staticmethod
    def empty(frames: int, cap: int, device) -> "Slots":
        return Slots(torch.empty((frames, cap, 7), dtype=torch.int32, device=device),
                     torch.empty((frames, cap, 32), dtype=torch.uint8, device=device),
                     torch.zeros((frames,), dtype=torch.int32, device=device))


class SlotExchange:
    """Double-buffered all-gather of every rank's `Slots` (equal shard sizes on every rank).

    Usage per step k::

        local = ex.acquire()            # slot set (k % depth), its previous gather completed
        ... enqueue extraction into local.kps / local.desc / local.counts ...
        ex.publish()                    # async all-gather of `local` into ex.gathered(k % depth)
    and `ex.drain()` before reading the last gathered set.
    """

    def __init__(self, frames: int, cap: int, device, group=None, depth: int = 2):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.frames, self.cap, self.depth = frames, cap, depth
        self.local = [Slots.empty(frames, cap, device) for _ in range(depth)]
        self.glob = [Slots.empty(self.world * frames, cap, device) for _ in range(depth)]
        self._work: list[list] = [[] for _ in range(depth)]
        self._cur = -1

    def acquire(self) -> Slots:
        """Next local slot set, ready to be overwritten (its earlier gather is complete)."""
        self._cur = (self._cur + 1) % self.depth
        self._wait(self._cur)
        return self.local[self._cur]

    def publish(self) -> int:
        """Start the all-gather of the slot set returned by the last acquire(); returns its index."""
        i = self._cur
        if i < 0:
            raise RuntimeError("publish() before acquire()")
        src, dst = self.local[i], self.glob[i]
        if self.world == 1:
            dst.kps.copy_(src.kps)
            dst.desc.copy_(src.desc)
            dst.counts.copy_(src.counts)
            return i
        self._work[i] = [
            dist.all_gather_into_tensor(dst.counts, src.counts, group=self.group, async_op=True),
            dist.all_gather_into_tensor(dst.kps, src.kps, group=self.group, async_op=True),
            dist.all_gather_into_tensor(dst.desc, src.desc, group=self.group, async_op=True),
        ]
        return i

    def _wait(self, i: int) -> None:
        for w in self._work[i]:
            w.wait()
        self._work[i] = []

    def wait(self, i: int) -> None:
        """Order the current stream after the gather of set i (no host sync with NCCL; gloo blocks)."""
        self._wait(i)

    def drain(self) -> None:
        for i in range(self.depth):
            self._wait(i)

    def gathered(self, i: int) -> Slots:
        """Gathered slots of set i: frame r*frames + f is rank r's local frame f."""
        return self.glob[i]


def unpack(slots: Slots):
    """Per-frame (keypoints[n], descriptors[n]) views, dropping the padding of every slot."""
    counts = slots.counts.cpu().tolist()
    return [(slots.kps[f, :n], slots.desc[f, :n]) for f, n in enumerate(counts)]
