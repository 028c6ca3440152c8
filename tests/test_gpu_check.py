"""GPU: the per-tile rank check of the lane-ordered kernels (the reference checks every
sort, checkCorrectness at Parallel7.cu:679-687). The default ranking rests on gfx950 serving the lanes of one
returning LDS add that hit the same address in lane order (rs_lane_order_probe checks it once per process);
every lane-ordered scatter kernel now re-checks it on the first slot of every full tile and records a
failure in the sort's check word (rsort_plan_check bit 1; the host entries return RSORT_ERR_CHECK).

The test hook rsort_inject_rank_fault swaps the ranks of the first two lanes of each digit in that slot --
what a device serving those lanes out of order would do. Every kernel family that ranks this way must catch
it (keys k = 8 plain and clustered, pairs k = 8, k = 4 next-digit lines, k = 6 pairs lines, the generic
kernel at k = 11 and 13), and with the hook cleared the same sorts are bit-exact against the oracle with a
clean check word. Runs on the MI355X box (-m gpu)."""
import numpy as np
import pytest

from _rs import rs
from _util import oracle_sort, oracle_sort_pairs, uniform_keys, zipf_keys

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = [
    # (k, n, pairs, distribution, the kernel family the plan runs)
    (8, 1 << 23, False, "uniform", "rs_scatter_lines"),           # digit groups, plain kernel
    (8, 1 << 23, False, "zipf", "rs_scatter_lines"),              # cut plans, clustered kernel
    (8, (1 << 22) + 77, True, "zipf", "rs_scatter_pairs"),
    (4, (1 << 21) + 5, False, "uniform", "rs_scatter_lines"),     # next-digit counts, raw tables
    (6, (1 << 23) + 9, True, "uniform", "rs_scatter_lines"),      # 64-B pairs lines
    (11, (1 << 20) + 3, False, "uniform", "rs_scatter"),
    (13, (1 << 20) + 11, True, "uniform", "rs_scatter"),
]


def _inputs(n, pairs, dist, k):
    x = (zipf_keys if dist == "zipf" else uniform_keys)(n, seed=1000 + k)
    v = np.arange(n, dtype=np.uint32) if pairs else None
    return x, v


def _sort(x, v, k, p, ws):
    d_in = rs.from_numpy_u32(x)
    d_out = rs.empty_u32(x.size)
    dv_in = rs.from_numpy_u32(v) if v is not None else None
    dv_out = rs.empty_u32(x.size) if v is not None else None
    rs.sort_device(d_in, d_out, k, vals_in=dv_in, vals_out=dv_out, ws=ws, plan_=p)
    return rs.to_numpy_u32(d_out), (rs.to_numpy_u32(dv_out) if v is not None else None)


@pytest.mark.parametrize("k,n,pairs,dist,family", CASES)
def test_rank_check_catches_a_broken_lane_order(k, n, pairs, dist, family):
    x, v = _inputs(n, pairs, dist, k)
    p = rs.plan(n, k, pairs)
    ws = rs.workspace(p.workspace_bytes)
    rs.scatter_kernels_used(reset=True)
    ko, vo = _sort(x, v, k, p, ws)
    used = rs.scatter_kernels_used(reset=True)
    assert any(u.startswith(family + "<") for u in used), used
    assert rs.plan_check(p, ws) == 0
    if pairs:
        wk, wv = oracle_sort_pairs(x, v, k)
        assert np.array_equal(ko, wk) and np.array_equal(vo, wv)
    else:
        assert np.array_equal(ko, oracle_sort(x, k))
    with rs.rank_fault():
        ko2, vo2 = _sort(x, v, k, p, ws)
        assert rs.plan_check(p, ws) & rs.CHECK_RANK_ORDER
    # the fault makes an unstable sort: pairs come out in a wrong order (keys-only outputs are wrong only
    # where the swapped lanes' keys differ in a later digit: the last pass's swaps always do)
    if pairs:
        assert not np.array_equal(vo2, wv)
    else:
        assert not np.array_equal(ko2, ko)
    # the hook cleared, the next sort in the same workspace is clean again
    ko3, _ = _sort(x, v, k, p, ws)
    assert rs.plan_check(p, ws) == 0 and np.array_equal(ko3, ko)


@pytest.mark.parametrize("k", [8, 4])
def test_host_entry_returns_check_error_on_a_broken_lane_order(k):
    """The host entries wait for the device anyway: they read the check word and return RSORT_ERR_CHECK
    (11) for a sort whose rank check failed."""
    n = (1 << 22) + 3
    x = uniform_keys(n, seed=k)
    with rs.rank_fault():
        with pytest.raises(rs.RSortError) as e:
            rs.sortByDevice(x, n, np.empty_like(x), k)
        assert e.value.status == 11
    y = np.empty_like(x)
    rs.sortByDevice(x, n, y, k)
    assert np.array_equal(y, np.sort(x))


def test_rank_check_clean_on_clustered_extremes():
    """Inputs that drive the ranking's aggregation paths (every key equal, one hot key on a quarter of the
    positions, few distinct keys): no false alarm from the check."""
    n = 1 << 23
    base = uniform_keys(n, seed=77)
    cases = [np.full(n, 0x1234567, dtype=np.uint32),
             np.where(base % 4 == 0, np.uint32(0xC0FFEE), base).astype(np.uint32),
             (base % 3).astype(np.uint32)]
    for x in cases:
        for k in (8, 4):
            p = rs.plan(n, k)
            ws = rs.workspace(p.workspace_bytes)
            ko, _ = _sort(x, None, k, p, ws)
            assert rs.plan_check(p, ws) == 0
            assert np.array_equal(ko, np.sort(x))


def test_partition_check_and_multi_gpu_sort_report_a_broken_lane_order():
    """The multi-GPU partition (rsort_partition_device: the line kernel with splitter digits) runs the same
    rank check; rsort_partition_check reads it, and rsort_u32_multi* turns a failure on any rank into
    RSORT_ERR_CHECK on every rank before any key moves (loopback transport, 3 ranks on this card)."""
    import sys
    import threading
    n = (1 << 22) + 17
    x = uniform_keys(n, seed=5)
    d = rs.from_numpy_u32(x)
    out = rs.empty_u32(n)
    spl = [1 << 30, 1 << 31, 3 << 30]
    starts = torch.empty(len(spl) + 2, dtype=torch.int32, device="cuda")
    ws = rs.workspace(int(rs._lib().rsort_partition_workspace_size(n, len(spl) + 1, 0)))
    rs.partition_device(d, out, spl, starts, ws=ws)
    assert rs.partition_check(n, len(spl) + 1, False, ws) == 0
    with rs.rank_fault():
        rs.partition_device(d, out, spl, starts, ws=ws)
        assert rs.partition_check(n, len(spl) + 1, False, ws) & rs.CHECK_RANK_ORDER
    world = 3
    grp = rs.LoopbackGroup(world)
    inputs = [rs.from_numpy_u32(uniform_keys(n, seed=50 + r)) for r in range(world)]
    res = [None] * world

    def run(r):
        torch.cuda.set_device(0)
        st = torch.cuda.Stream()
        try:
            with torch.cuda.stream(st):
                rs.multi_sort_device(grp.transport(r), inputs[r], 8, capacity=world * n, stream=st)
                st.synchronize()
                res[r] = 0
        except rs.RSortError as e:
            res[r] = e.status

    with rs.rank_fault():
        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
    assert not any(t.is_alive() for t in th)
    grp.close()
    assert res == [11] * world, res
