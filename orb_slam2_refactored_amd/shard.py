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

`CompactExchange` is the descriptor-sized form bench.py runs: the per-frame counts are gathered
first, then each rank sends one contiguous block of its Σn descriptors (32 B each; padded at the tail
to the largest block of the step, since RCCL's all-gather moves equal-sized blocks) instead of
2024-slot padded keypoint + descriptor slots -- about 0.37x the bytes at C2.  The payload of step k
is packed and gathered on a side stream one step later (the host needs step k's counts to size it),
overlapping step k+1's extraction.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from ._lib import check, lib, stream_ptr, tptr


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [start, start+count) of n_total frames for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world) or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def cross_shard_predecessor(rank: int, world: int, frames_per_rank: int) -> int:
    """Index, in the gathered slot buffer (rank-major: rank r's local frame f at r*frames_per_rank + f),
    of the predecessor of this rank's first frame: global frame g0 - 1, i.e. rank r-1's last frame.
    Rank 0's first frame is global frame 0, which has no predecessor: -1 (the caller skips it).
    §8d C5: "frame i matched to i-1"."""
    if world <= 0 or not (0 <= rank < world) or frames_per_rank <= 0:
        raise ValueError("bad shard arguments")
    return rank * frames_per_rank - 1 if rank > 0 else -1


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


class CompactExchange:
    """Double-buffered ragged all-gather of every rank's descriptors (equal frame counts per rank).

    Usage per step k (after enqueueing step k's extraction into `local(k)` on the current stream)::

        ex.publish(k)        # counts all-gather of step k; then, for step k-1 (counts now on the
                             # host): pack + payload all-gather on the side stream
        ex.wait(k - 1)       # current stream waits for step k-1's payload (no host sync)

    and `ex.drain()` at the end (finishes the last published step).  After wait(i), `block(i, r)` is
    rank r's descriptors of step i as one [tot_r, 32] uint8 tensor (frame order), `frame(i, r, f)` one
    frame's rows.  Works on CUDA (RCCL, side stream, events) and on CPU (gloo, synchronous).
    """

    def __init__(self, frames: int, cap: int, device, group=None, depth: int = 2):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.frames, self.cap, self.depth = frames, cap, depth
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.slots = [Slots.empty(frames, cap, device) for _ in range(depth)]
        self.counts_all = [torch.zeros(self.world * frames, dtype=torch.int32, device=device) for _ in range(depth)]
        pin = self.cuda
        self.counts_host = [torch.zeros(self.world * frames, dtype=torch.int32, pin_memory=pin) for _ in range(depth)]
        self.send = [torch.zeros((0, 32), dtype=torch.uint8, device=device) for _ in range(depth)]
        self.recv = [torch.zeros((0, 32), dtype=torch.uint8, device=device) for _ in range(depth)]
        self.maxtot = [0] * depth
        self.tot = [[0] * self.world for _ in range(depth)]
        self.pending = None   # step whose payload is not yet packed / gathered
        self.side = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.ev_extract = [torch.cuda.Event() for _ in range(depth)] if self.cuda else None
        self.ev_counts = [torch.cuda.Event() for _ in range(depth)] if self.cuda else None
        self.ev_payload = [torch.cuda.Event() for _ in range(depth)] if self.cuda else None
        self._timing = []            # (start, end) events around each payload all-gather, not yet read
        self.gather_ms = []          # payload all-gather time per step (CUDA events)
        self.payload_bytes = []      # gathered payload bytes per step (world x maxtot x 32)

    def local(self, k: int) -> Slots:
        return self.slots[k % self.depth]

    def _side(self):
        return torch.cuda.stream(self.side) if self.cuda else _NullCtx()

    def publish(self, k: int) -> None:
        i = k % self.depth
        src = self.slots[i]
        if self.cuda:
            self.ev_extract[i].record()
        with self._side():
            if self.cuda:
                self.side.wait_event(self.ev_extract[i])
            if self.world > 1:
                dist.all_gather_into_tensor(self.counts_all[i], src.counts, group=self.group)
            else:
                self.counts_all[i].copy_(src.counts)
            self.counts_host[i].copy_(self.counts_all[i], non_blocking=self.cuda)
            if self.cuda:
                self.ev_counts[i].record(self.side)
        if self.pending is not None:
            self._payload(self.pending)
        self.pending = k

    def _payload(self, k: int) -> None:
        i = k % self.depth
        if self.cuda:
            self.ev_counts[i].synchronize()
        c = self.counts_host[i].view(self.world, self.frames).to(torch.int64)
        tot = c.sum(1).tolist()
        self.tot[i] = tot
        maxtot = max(tot) if tot else 0
        self.maxtot[i] = maxtot
        mine = c[self.rank]
        src = self.slots[i]
        with self._side():
            if self.send[i].shape[0] < maxtot:   # grown with headroom: a block rarely outgrows it again
                self.send[i] = torch.zeros((maxtot + maxtot // 4, 32), dtype=torch.uint8, device=self.device)
            if self.recv[i].shape[0] < self.world * maxtot:
                self.recv[i] = torch.zeros((self.world * (maxtot + maxtot // 4), 32), dtype=torch.uint8,
                                           device=self.device)
            n = tot[self.rank]
            if n and self.cuda:
                # one HIP launch (orbx_pack_descriptors) from the device-side counts of this rank; the
                # torch gather below costs ~4.7 ms per 8192-frame step on the byte-wise index_select
                cnt = self.counts_all[i].view(self.world, self.frames)[self.rank]
                incl = torch.cumsum(cnt, 0, dtype=torch.int32)
                check(lib().orbx_pack_descriptors(tptr(src.desc), self.cap, tptr(cnt), tptr(incl), self.frames,
                                                  tptr(self.send[i]), int(self.send[i].shape[0]), stream_ptr(self.side)),
                      "orbx_pack_descriptors")
            elif n:
                # (CPU / gloo) row r of the block: frame fr = the frame whose prefix range holds r, slot r - start[fr]
                cnt = mine.to(self.device)
                start = torch.cumsum(cnt, 0) - cnt
                fr = torch.repeat_interleave(torch.arange(self.frames, device=self.device), cnt, output_size=n)
                row = torch.arange(n, device=self.device) - start[fr]
                torch.index_select(src.desc.view(-1, 32), 0, fr * self.cap + row, out=self.send[i][:n])
            if self.cuda:
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(self.side)
            if self.world > 1:
                dist.all_gather_into_tensor(self.recv[i][:self.world * maxtot], self.send[i][:maxtot], group=self.group)
            else:
                self.recv[i][:maxtot].copy_(self.send[i][:maxtot])
            if self.cuda:
                t1.record(self.side)
                self._timing.append((t0, t1))
                self.ev_payload[i].record(self.side)
        self.payload_bytes.append(self.world * maxtot * 32)

    def wait(self, k: int) -> None:
        """Current stream waits for step k's payload (published one step earlier)."""
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_event(self.ev_payload[k % self.depth])

    def drain(self) -> None:
        if self.pending is not None:
            self._payload(self.pending)
            self.wait(self.pending)
            self.pending = None

    def collect_gather_times(self) -> None:
        """Adds the payload all-gather times of the steps gathered so far (CUDA; call after a sync)."""
        for t0, t1 in self._timing:
            self.gather_ms.append(t0.elapsed_time(t1))
        self._timing = []

    def counts(self, k: int) -> torch.Tensor:
        return self.counts_host[k % self.depth].view(self.world, self.frames)

    def block(self, k: int, r: int) -> torch.Tensor:
        i = k % self.depth
        return self.recv[i][r * self.maxtot[i]: r * self.maxtot[i] + self.tot[i][r]]

    def frame(self, k: int, r: int, f: int) -> torch.Tensor:
        c = self.counts(k)[r].to(torch.int64)
        s0 = int(c[:f].sum())
        return self.block(k, r)[s0: s0 + int(c[f])]


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
