"""The multi-GPU descriptor exchange on the device: CompactExchange on CUDA packs each step's ragged
descriptor block with the HIP kernel behind orbx_pack_descriptors (single process, world 1: the
payload "all-gather" is the local copy), and the block must equal the concatenation of every frame's
valid rows byte for byte (ragged counts including 0 and the full slot capacity)."""
import pytest
import torch

from orb_slam2_refactored_amd import _lib
from orb_slam2_refactored_amd.shard import CompactExchange

pytestmark = pytest.mark.gpu


def _slots(ex, k, seed, frames, cap):
    g = torch.Generator().manual_seed(seed)
    loc = ex.local(k)
    counts = torch.randint(0, cap + 1, (frames,), generator=g, dtype=torch.int32)
    counts[0], counts[-1] = 0, cap
    desc = torch.randint(0, 256, (frames, cap, 32), generator=g, dtype=torch.uint8)
    loc.desc.copy_(desc.cuda())
    loc.counts.copy_(counts.cuda())
    return desc, counts


@pytest.mark.parametrize("frames,cap", [(7, 33), (64, 2024)])
def test_compact_exchange_cuda_pack(frames, cap):
    ex = CompactExchange(frames, cap, "cuda")
    want = {}
    for k in range(4):
        desc, counts = _slots(ex, k, 100 + k, frames, cap)
        last = (desc, counts)
        want[k] = torch.cat([desc[f, :int(counts[f])] for f in range(frames)])
        ex.publish(k)
        if k >= 1:
            ex.wait(k - 1)
            torch.cuda.synchronize()
            assert torch.equal(ex.block(k - 1, 0).cpu(), want[k - 1])
    ex.drain()
    torch.cuda.synchronize()
    assert torch.equal(ex.block(3, 0).cpu(), want[3])
    desc, counts = last
    for f in (0, frames // 2, frames - 1):
        assert torch.equal(ex.frame(3, 0, f).cpu(), desc[f, :int(counts[f])])


def test_pack_descriptors_rejects_misaligned():
    d = torch.zeros(2 * 4 * 32 + 1, dtype=torch.uint8, device="cuda")
    c = torch.ones(2, dtype=torch.int32, device="cuda")
    with pytest.raises(_lib.OrbError):
        _lib.check(_lib.lib().orbx_pack_descriptors(_lib.tptr(d[1:]), 4, _lib.tptr(c), _lib.tptr(c), 2,
                                                    _lib.tptr(d), 2, _lib.stream_ptr()), "orbx_pack_descriptors")


def test_pack_descriptors_clamps_counts_and_output():
    """counts past the slot capacity copy only `cap` rows, and rows past out_rows are never
    written (a guard row after the output stays intact)."""
    frames, cap = 3, 4
    g = torch.Generator().manual_seed(7)
    desc = torch.randint(0, 256, (frames, cap, 32), generator=g, dtype=torch.uint8)
    counts = torch.tensor([2, 9, 3], dtype=torch.int32)   # frame 1 claims more rows than its slots
    incl = torch.cumsum(counts, 0, dtype=torch.int32)      # the caller's layout: rows 0-1, 2-10, 11-13
    out_rows = 12
    buf = torch.full((out_rows + 1, 32), 0xA5, dtype=torch.uint8, device="cuda")
    # device copies held by name: a temporary's memory could be reused before the kernel reads it
    d_desc, d_counts, d_incl = desc.cuda(), counts.cuda(), incl.cuda()
    _lib.check(_lib.lib().orbx_pack_descriptors(_lib.tptr(d_desc), cap, _lib.tptr(d_counts), _lib.tptr(d_incl),
                                                frames, _lib.tptr(buf), out_rows, _lib.stream_ptr()),
               "orbx_pack_descriptors")
    torch.cuda.synchronize()
    got = buf.cpu()
    assert torch.equal(got[0:2], desc[0, :2])
    assert torch.equal(got[2:6], desc[1, :4])               # clamped to cap rows
    assert (got[6:11] == 0xA5).all()                        # the rows frame 1 claimed beyond cap: untouched
    assert torch.equal(got[11:12], desc[2, :1])             # frame 2 clipped at out_rows
    assert (got[12] == 0xA5).all()                          # the guard row after out_rows: untouched


@pytest.mark.parametrize("frames,cap,seed", [(1, 1, 0), (5, 3, 1), (33, 64, 2), (128, 2024, 3)])
def test_pack_descriptors_kernel_matches_gloo_pack(frames, cap, seed):
    """the device kernel behind orbx_pack_descriptors against the gloo (CPU) path's own pack
    (shard.CompactExchange's repeat_interleave / index_select block) on ragged layouts, counts of 0 and of
    the full slot capacity included."""
    from orb_slam2_refactored_amd.shard import CompactExchange
    g = torch.Generator().manual_seed(seed)
    counts = torch.randint(0, cap + 1, (frames,), generator=g, dtype=torch.int32)
    counts[0] = 0
    counts[-1] = cap
    if frames > 2:
        counts[1] = cap
        counts[2] = 0
    desc = torch.randint(0, 256, (frames, cap, 32), generator=g, dtype=torch.uint8)
    cpu = CompactExchange(frames, cap, "cpu")   # world 1, no process group: the gloo path's pack, run locally
    loc = cpu.local(0)
    loc.desc.copy_(desc)
    loc.counts.copy_(counts)
    cpu.publish(0)
    cpu.drain()
    want = cpu.block(0, 0)
    assert torch.equal(want, torch.cat([desc[f, :int(counts[f])] for f in range(frames)]))
    total = int(counts.sum())
    incl = torch.cumsum(counts, 0, dtype=torch.int32)
    out = torch.full((total + 1, 32), 0x5A, dtype=torch.uint8, device="cuda")
    d_desc, d_counts, d_incl = desc.cuda(), counts.cuda(), incl.cuda()
    _lib.check(_lib.lib().orbx_pack_descriptors(_lib.tptr(d_desc), cap, _lib.tptr(d_counts), _lib.tptr(d_incl),
                                                frames, _lib.tptr(out), total, _lib.stream_ptr()),
               "orbx_pack_descriptors")
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.equal(got[:total], want)
    assert (got[total] == 0x5A).all()
