"""BASELINE configs[4] (C5) at its full size on the one MI355X of the test box: 8 ranks x 2^30
uniform u32 keys (2^33 in total; the bench's stream -- one splitmix64 sequence, seed 0x5EED,
block-distributed by rank), range-partitioned with one exchange, through the C ABI
(rsort_u32_multi_transport) with the in-process loopback transport: one thread per rank, all on
cuda:0 (~150 GB of the 288-GB HBM). The reference has no multi-GPU path (Parallel7.cu:10, :697
hard-code device 0); SURVEY §8e defines parity at 2^33 (Baseline1's `int n` cannot take it):
  - every rank's output is sorted and last_r <= first_{r+1}; the counts sum to 2^33 and the offsets
    are their exclusive scan; the multiset fingerprints of the outputs sum to the inputs';
  - every rank's output equals the slice [offset_r, offset_r + count_r) of the globally sorted keys,
    built on the device as (copies of its lowest key) + rocPRIM's sort of the input keys strictly
    inside its key range + (copies of its highest key), with the copy counts from global counts;
  - one rank (rank 3) bit-exact against the oracle (Baseline1.cu:15-64 restated) on the same slice.
The phase times of the run are printed (DESIGN §5 records them)."""
import json
import os
import threading

import numpy as np
import pytest

from _rs import rs
from _util import oracle_sort

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

WORLD = 8
N = 1 << 30
SEED = 0x5EED


def _u64(t):
    return t.to(torch.int64) & 0xFFFFFFFF


def _count(inputs, pred):
    """sum over the ranks' inputs of pred(keys as int64), in 2^27-key pieces"""
    tot = 0
    for x in inputs:
        for i in range(0, x.numel(), 1 << 27):
            tot += int(pred(_u64(x[i:i + (1 << 27)])).sum().item())
    return tot


def _gather_between(inputs, lo, hi):
    """the input keys with lo < key < hi (as u32), concatenated on the device"""
    parts = []
    for x in inputs:
        for i in range(0, x.numel(), 1 << 27):
            v = _u64(x[i:i + (1 << 27)])
            parts.append(x[i:i + (1 << 27)][(v > lo) & (v < hi)])
    return torch.cat(parts)


def test_c5_full_size_loopback_world8():
    if torch.cuda.get_device_properties(0).total_memory < 200 * (1 << 30):
        pytest.skip("C5 at full size needs ~150 GB of device memory")
    torch.cuda.set_device(0)
    cap = rs.default_capacity(N)
    inputs, outs, vouts = [], [], []
    for r in range(WORLD):
        x = rs.empty_u32(N)
        rs.gen_uniform(x, SEED + r * N)
        inputs.append(x)
        outs.append(rs.empty_u32(cap))
    wsb = int(rs._lib().rsort_multi_workspace_size(N, cap, 8, 0, WORLD))
    wss = [rs.workspace(wsb) for _ in range(WORLD)]
    fp_in = sum(rs.fingerprint(x)[0] for x in inputs) & 0xFFFFFFFFFFFFFFFF
    torch.cuda.synchronize()

    grp = rs.LoopbackGroup(WORLD)
    res = [None] * WORLD
    stats = [None] * WORLD
    rs.multi_set_profiling(True)

    def run(r):
        torch.cuda.set_device(0)
        st = torch.cuda.Stream()
        try:
            with torch.cuda.stream(st):
                res[r] = rs.multi_sort_device(grp.transport(r), inputs[r], 8, capacity=cap, stream=st, ws=wss[r],
                                              out=(outs[r], None))
                st.synchronize()
                stats[r] = rs.multi_last_stats()
        except rs.RSortError as e:
            res[r] = e.status

    th = [threading.Thread(target=run, args=(r,)) for r in range(WORLD)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    rs.multi_set_profiling(False)
    alive = any(t.is_alive() for t in th)
    if not alive:
        grp.close()
    assert not alive, "loopback ranks did not finish"
    assert all(isinstance(x, tuple) for x in res), res
    del wss
    torch.cuda.empty_cache()

    ph = ("ms_plan", "ms_partition", "ms_exchange", "ms_local_sort", "ms_total")
    if os.environ.get("RSORT_C5_RECORD"):  # (the lab run that records DESIGN §5's C5 row)
        with open(os.environ["RSORT_C5_RECORD"], "w") as fh:
            json.dump({"world": WORLD, "keys_per_rank": N, "transport": "loopback, 8 threads on one GPU",
                       "stats": stats}, fh)
    print("\nC5 loopback world 8 x 2^30 (8 ranks sharing one GPU; phases contend): per rank " +
          "; ".join(f"r{r} " + " ".join(f"{k[3:]} {stats[r][k]:.1f}" for k in ph) + f" out {stats[r]['n_out']}"
                    for r in range(WORLD)))

    counts = [x[0].numel() for x in res]
    offs = [x[2] for x in res]
    assert sum(counts) == WORLD * N
    assert offs == list(np.cumsum([0] + counts[:-1]))
    assert max(counts) - min(counts) <= 0.05 * N, counts  # balanced within 5 %
    fp_out, firsts, lasts = 0, [], []
    for ok, _, _ in res:
        h, desc = rs.fingerprint(ok)
        assert desc == 0  # sorted
        fp_out = (fp_out + h) & 0xFFFFFFFFFFFFFFFF
        firsts.append(int(ok[0].item()) & 0xFFFFFFFF)
        lasts.append(int(ok[-1].item()) & 0xFFFFFFFF)
    assert fp_out == fp_in
    assert all(lasts[r] <= firsts[r + 1] for r in range(WORLD - 1)), (firsts, lasts)

    # every rank against the globally sorted slice: its lowest key's copies, rocPRIM's sort of the
    # keys strictly inside its range, its highest key's copies
    for r in range(WORLD):
        ok = res[r][0]
        lo, hi = firsts[r], lasts[r]
        below_lo = _count(inputs, lambda v: v < lo)
        eq_lo = _count(inputs, lambda v: v == lo)
        mid = _gather_between(inputs, lo, hi)
        if lo == hi:
            want_lo, want_hi = counts[r], 0
        else:
            want_lo = below_lo + eq_lo - offs[r]  # this rank's share of lo's copies (it holds the first)
            want_hi = counts[r] - want_lo - mid.numel()
        assert 0 < want_lo <= eq_lo and want_hi >= 0, (r, want_lo, eq_lo, want_hi)
        srt = rs.empty_u32(mid.numel())
        if mid.numel():
            rs.vendor_sort_device(mid, srt)
        assert bool((_u64(ok[:want_lo]) == lo).all()), r
        assert torch.equal(ok[want_lo:want_lo + mid.numel()], srt), r
        if want_hi:
            assert bool((_u64(ok[want_lo + mid.numel():]) == hi).all()), r
        if r == 3:
            # bit-exact against the oracle: Baseline1 on the input keys that make up this slice (the
            # strictly-inside keys in their input order, the boundary keys' copies in front)
            host = np.concatenate([np.full(want_lo, lo, np.uint32), np.full(want_hi, hi, np.uint32),
                                   rs.to_numpy_u32(mid)])
            assert np.array_equal(rs.to_numpy_u32(ok), oracle_sort(host, 8))
        del mid, srt
