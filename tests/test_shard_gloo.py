"""N>1 path on CPU: frame sharding and the double-buffered slot all-gather over `gloo`, world_size 2
(the same SlotExchange that bench.py runs over RCCL).  The gathered buffer must equal the
concatenation of every rank's slots byte for byte."""
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from orb_slam2_refactored_amd.shard import CompactExchange, SlotExchange, Slots, cross_shard_predecessor, shard_range, unpack  # noqa: E402

FRAMES, CAP, STEPS = 3, 40, 5


def fake_slots(global_frame0: int, step: int) -> Slots:
    """Deterministic stand-in for one rank's extraction output (ragged counts, incl. 0 and CAP)."""
    s = Slots.empty(FRAMES, CAP, "cpu")
    for f in range(FRAMES):
        g = global_frame0 + f
        gen = torch.Generator().manual_seed(1000 * step + g)
        s.kps[f] = torch.randint(-2**31, 2**31 - 1, (CAP, 7), generator=gen, dtype=torch.int64).to(torch.int32)
        s.desc[f] = torch.randint(0, 256, (CAP, 32), generator=gen, dtype=torch.int64).to(torch.uint8)
        s.counts[f] = [0, CAP, (7 * g + step) % CAP][(g + step) % 3]
    return s


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        start, count = shard_range(world * FRAMES, world, rank)
        assert count == FRAMES
        ex = SlotExchange(FRAMES, CAP, "cpu")
        for step in range(STEPS):
            local = ex.acquire()
            src = fake_slots(start, step)
            local.kps.copy_(src.kps)
            local.desc.copy_(src.desc)
            local.counts.copy_(src.counts)
            i = ex.publish()
        ex.drain()
        # the last published set holds step STEPS-1 from every rank, in rank order
        g = ex.gathered(i)
        for r in range(world):
            r0, _ = shard_range(world * FRAMES, world, r)
            want = fake_slots(r0, STEPS - 1)
            sl = slice(r * FRAMES, (r + 1) * FRAMES)
            assert torch.equal(g.kps[sl], want.kps)
            assert torch.equal(g.desc[sl], want.desc)
            assert torch.equal(g.counts[sl], want.counts)
        # and the other set holds step STEPS-2
        g2 = ex.gathered(1 - i)
        for r in range(world):
            r0, _ = shard_range(world * FRAMES, world, r)
            assert torch.equal(g2.desc[r * FRAMES:(r + 1) * FRAMES], fake_slots(r0, STEPS - 2).desc)
        per_frame = unpack(g)
        assert len(per_frame) == world * FRAMES
        assert [int(k.shape[0]) for k, _ in per_frame] == g.counts.tolist()
        # C5 cross-shard pairing: this rank's first frame (global g0) is matched against the gathered
        # slot of global frame g0 - 1, rank r-1's last local frame; rank 0's first frame is global frame
        # 0 and has no predecessor (-1)
        pred = cross_shard_predecessor(rank, world, FRAMES)
        if rank == 0:
            assert pred == -1
        else:
            pr, pf = divmod(pred, FRAMES)
            assert pr == rank - 1 and pf == FRAMES - 1
            assert shard_range(world * FRAMES, world, pr)[0] + pf == start - 1
            want_prev = fake_slots(shard_range(world * FRAMES, world, pr)[0], STEPS - 1)
            assert torch.equal(g.desc[pred], want_prev.desc[FRAMES - 1])
            assert int(g.counts[pred]) == int(want_prev.counts[FRAMES - 1])
            # the cross-shard match on the gathered data equals the match against the predecessor's slots
            import oracle_api as O
            mine = fake_slots(start, STEPS - 1)
            na, nb = int(mine.counts[0]), int(g.counts[pred])
            a = mine.desc[0, :na].numpy()
            got = O.bf_match(a, g.desc[pred, :nb].numpy())
            exp = O.bf_match(a, want_prev.desc[FRAMES - 1, :nb].numpy())
            for x, y in zip(got, exp):
                assert (x == y).all()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # pragma: no cover - reported by the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_slot_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_shard_range_partitions():
    for n in range(0, 40):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard_range(n, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_cross_shard_predecessor():
    assert cross_shard_predecessor(0, 1, 5) == -1
    assert [cross_shard_predecessor(r, 4, 3) for r in range(4)] == [-1, 2, 5, 8]
    with pytest.raises(ValueError):
        cross_shard_predecessor(2, 2, 3)


def test_single_process_exchange_is_copy():
    ex = SlotExchange(FRAMES, CAP, "cpu")
    local = ex.acquire()
    src = fake_slots(0, 0)
    local.kps.copy_(src.kps)
    local.desc.copy_(src.desc)
    local.counts.copy_(src.counts)
    i = ex.publish()
    ex.drain()
    assert torch.equal(ex.gathered(i).desc, src.desc)
    assert torch.equal(ex.gathered(i).counts, src.counts)


def _packed(s: Slots) -> torch.Tensor:
    """A rank's descriptor block: every frame's first counts[f] rows, frame order."""
    return torch.cat([s.desc[f, :int(s.counts[f])] for f in range(s.desc.shape[0])])


def _compact_worker(rank, world, port, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        start, _ = shard_range(world * FRAMES, world, rank)
        ex = CompactExchange(FRAMES, CAP, "cpu")

        def check(k):   # step k has been gathered: every rank's block and the predecessor frame
            for r in range(world):
                r0, _ = shard_range(world * FRAMES, world, r)
                want = fake_slots(r0, k)
                assert torch.equal(ex.counts(k)[r], want.counts)
                assert torch.equal(ex.block(k, r), _packed(want))
                for f in range(FRAMES):
                    assert torch.equal(ex.frame(k, r, f), want.desc[f, :int(want.counts[f])])
            assert ex.payload_bytes[-1] == world * max(int(fake_slots(shard_range(world * FRAMES, world, r)[0], k)
                                                           .counts.sum()) for r in range(world)) * 32
            pred = cross_shard_predecessor(rank, world, FRAMES)
            if rank > 0:
                pr, pf = divmod(pred, FRAMES)
                prev = fake_slots(shard_range(world * FRAMES, world, pr)[0], k)
                assert torch.equal(ex.frame(k, pr, pf), prev.desc[pf, :int(prev.counts[pf])])

        for k in range(STEPS):
            loc = ex.local(k)
            src = fake_slots(start, k)
            loc.kps.copy_(src.kps)
            loc.desc.copy_(src.desc)
            loc.counts.copy_(src.counts)
            ex.publish(k)
            if k >= 1:
                ex.wait(k - 1)
                check(k - 1)
        ex.drain()
        check(STEPS - 1)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # pragma: no cover - reported by the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_compact_exchange_gloo(world):
    """The ragged descriptor all-gather bench.py runs over RCCL: per step, every rank's Σn x 32 B block
    (ragged counts incl. 0 and CAP) arrives intact, one step after publish, and the cross-shard
    predecessor frame is read from it."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_compact_worker, args=(r, world, port, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_compact_exchange_single_process():
    ex = CompactExchange(FRAMES, CAP, "cpu")
    for k in range(3):
        src = fake_slots(0, k)
        loc = ex.local(k)
        loc.desc.copy_(src.desc)
        loc.counts.copy_(src.counts)
        ex.publish(k)
    ex.drain()
    assert torch.equal(ex.block(2, 0), _packed(fake_slots(0, 2)))


def _pack_rows_reference(desc, cap, counts, incl, out_rows):
    """The index math of orbx_pack_descriptors (csrc/orbx.hip pack_rows_kernel) on the CPU: frame f's first
    min(max(counts[f], 0), cap) rows go to out rows from incl[f] - counts[f], clipped to [0, out_rows)."""
    out = torch.zeros((out_rows, 32), dtype=torch.uint8)
    for f in range(desc.shape[0]):
        c = int(counts[f])
        n = min(max(c, 0), cap)
        start = int(incl[f]) - c
        for r in range(max(start, 0), min(start + n, out_rows)):
            out[r] = desc[f, r - start]
    return out


def test_cuda_pack_index_math_matches_gloo_pack():
    """the device pack (inclusive-prefix offsets, bench.py's CUDA path) and the gloo path's
    repeat_interleave / index_select pack produce the same block for ragged counts incl. 0 and cap."""
    g = torch.Generator().manual_seed(11)
    for frames, cap in ((1, 5), (6, 7), (33, 40)):
        desc = torch.randint(0, 256, (frames, cap, 32), generator=g, dtype=torch.int64).to(torch.uint8)
        counts = torch.randint(0, cap + 1, (frames,), generator=g, dtype=torch.int64).to(torch.int32)
        counts[0] = 0
        counts[-1] = cap
        incl = torch.cumsum(counts, 0, dtype=torch.int32)
        n = int(counts.sum())
        # the gloo branch of CompactExchange._payload
        start = torch.cumsum(counts, 0) - counts
        fr = torch.repeat_interleave(torch.arange(frames), counts.to(torch.int64), output_size=n)
        row = torch.arange(n) - start[fr]
        gloo = torch.index_select(desc.view(-1, 32), 0, fr * cap + row)
        assert torch.equal(_pack_rows_reference(desc, cap, counts, incl, n), gloo)
