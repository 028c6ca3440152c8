"""The multi-GPU sort's host-side planning (include/rsort.h "multi-GPU planning",
cuda.radixsort_amd/csrc/rsort_exchange.cpp) on the CPU, at world sizes 1..16: the functions both
rsort_u32_multi* and multi.py take every decision from.

* test_planning_fuzz_sanitized: tests/c/exchange_fuzz.cpp + rsort_exchange.cpp built with
  g++ -fsanitize=address,undefined (SURVEY §5's sanitizer build of the host code) -- 20 000 random
  worlds, ragged / empty / hot-bucket counts, tight capacities; invariants: sends cover each
  partition in order, every rank's plan agrees with every other's, offsets are the exclusive scan,
  the capacity verdict is the same on every rank, equal-key cuts land on the balanced target.
* test_plan_matches_restatement: against an independent numpy restatement of the protocol
  (global (bucket, source, position) order, boundaries at r * total / world clamped into the
  boundary's bucket).
* test_loaded_library_matches: the same functions through librsort.so (what the product calls).
"""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from _rs import rs

ROOT = Path(__file__).resolve().parent.parent


def test_planning_fuzz_sanitized(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "exchange_fuzz"
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "c" / "exchange_fuzz.cpp"),
                    str(ROOT / "cuda.radixsort_amd" / "csrc" / "rsort_exchange.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok 20000")


def _restated_plan(world, counts, splitters, cut_bucket, cut_inside):
    """Independent restatement: every key's global position in (bucket, source rank, position in
    the source's bucket) order; boundary r at clamp(r * total // world) inside its equal-keys
    bucket, or at the start of its bucket; rank r owns [G_r, G_{r+1})."""
    counts = np.asarray(counts, np.int64)
    buckets = counts.shape[1]
    gb = np.concatenate([[0], np.cumsum(counts.sum(axis=0))])
    total = int(gb[-1])
    G = [0]
    for r in range(1, world):
        b = cut_bucket[r]
        g = min(max(r * total // world, gb[b]), gb[b + 1]) if cut_inside[r] else gb[b]
        G.append(max(int(g), G[-1]))
    G.append(total)
    # send[s][r] = keys of source s whose global position is in [G_r, G_{r+1})
    send = np.zeros((world, world), np.int64)
    for s in range(world):
        for b in range(buckets):
            c = counts[s, b]
            if c == 0:
                continue
            start = gb[b] + counts[:s, b].sum()  # global position of s's first key of bucket b
            for r in range(world):
                lo, hi = max(start, G[r]), min(start + c, G[r + 1])
                send[s, r] += max(0, hi - lo)
    return send, G


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8, 9, 12, 16])
def test_plan_matches_restatement(world):
    rng = np.random.default_rng(world)
    for case in range(60):
        q = np.sort(rng.integers(0, 64 if case % 2 else 1 << 32, size=max(0, world - 1), dtype=np.uint64))
        # every key hot (rsort_multi_splitters_make), random hot flags, none hot (make_hot)
        hot = None if case % 3 == 0 else (rng.random(max(0, world - 1)) < 0.5).tolist() if case % 3 == 1 \
            else [0] * max(0, world - 1)
        spl = rs.multi_splitters(world, q.tolist(), hot)
        nb = spl.nsplit + 1
        counts = rng.integers(0, 500, size=(world, nb)) * (rng.random((world, nb)) < 0.7)
        if case % 5 == 0:
            counts[:, 1::2] *= 50  # hot equal-key buckets
        counts = counts.astype(np.int64)
        send, G = _restated_plan(world, counts, spl.splitters, list(spl.cut_bucket), list(spl.cut_inside))
        cap = np.full(world, int(counts.sum()), np.int64)
        for me in range(world):
            xp = rs.multi_exchange_plan(world, me, counts, spl, cap)
            assert list(xp.send_cnt)[:world] == send[me].tolist()
            assert list(xp.recv_cnt)[:world] == send[:, me].tolist()
            assert xp.offset == G[me] and xp.n_recv == G[me + 1] - G[me]


def test_splitters_equal_key_buckets():
    spl = rs.multi_splitters(4, [10, 10, 20])
    assert spl.splitters == [10, 11, 20, 21]
    assert list(spl.cut_bucket)[1:4] == [1, 1, 3] and list(spl.cut_inside)[1:4] == [1, 1, 1]
    spl = rs.multi_splitters(3, [5, 0xFFFFFFFF])  # no bucket above the largest key
    assert spl.splitters == [5, 6, 0xFFFFFFFF]
    assert list(spl.cut_bucket)[1:3] == [1, 3]
    spl = rs.multi_splitters(16, list(range(100, 1600, 100)))  # every world: 2 x 15 = 30 splitters (<= 31)
    assert spl.splitters == sum(([v, v + 1] for v in range(100, 1600, 100)), [])
    assert list(spl.cut_bucket)[1:16] == list(range(1, 30, 2)) and all(list(spl.cut_inside)[1:16])
    assert rs.multi_splitters(1, []).nsplit == 0
    with pytest.raises(rs.RSortError):
        rs.multi_splitters(3, [5, 4])  # not sorted


def test_splitters_hot_flags():
    """Only hot quantile keys get an equal-keys bucket; the others are plain splitters (boundary at the
    start of their bucket); a run of equal quantile keys is hot whatever its flags."""
    spl = rs.multi_splitters(4, [10, 20, 30], hot=[0, 0, 0])
    assert spl.splitters == [10, 20, 30]
    assert list(spl.cut_bucket)[1:4] == [1, 2, 3] and list(spl.cut_inside)[1:4] == [0, 0, 0]
    spl = rs.multi_splitters(4, [10, 20, 30], hot=[0, 1, 0])
    assert spl.splitters == [10, 20, 21, 30]
    assert list(spl.cut_bucket)[1:4] == [1, 2, 4] and list(spl.cut_inside)[1:4] == [0, 1, 0]
    spl = rs.multi_splitters(5, [7, 7, 9, 0xFFFFFFFF], hot=[0, 0, 0, 1])
    assert spl.splitters == [7, 8, 9, 0xFFFFFFFF]
    assert list(spl.cut_bucket)[1:5] == [1, 1, 3, 4] and list(spl.cut_inside)[1:5] == [1, 1, 0, 1]
    # all hot == the flag-less call
    a = rs.multi_splitters(6, [1, 5, 5, 9, 12], hot=[1] * 5)
    b = rs.multi_splitters(6, [1, 5, 5, 9, 12])
    assert a.splitters == b.splitters and list(a.cut_bucket) == list(b.cut_bucket)
    assert list(a.cut_inside) == list(b.cut_inside)


def test_hot_flags_from_sample():
    """rs.hot_flags (multi.py; rsort_u32_multi* computes the same on the device's sorted sample): a quantile
    key is hot when the sample holds it hot_reach positions away on either side."""
    world = 4
    s = np.sort(np.concatenate([np.arange(0, 3000, 3, dtype=np.uint32), np.full(200, 1500, np.uint32)]))
    L = rs.hot_reach(world, s.size)
    assert L == max(1, s.size // (world * 128))
    pos = [int(np.searchsorted(s, 1500)) + 50, 10, s.size - 5]
    assert rs.hot_flags(s, pos, world) == [1, 0, 0]


def test_capacity_verdict_is_shared():
    spl = rs.multi_splitters(3, [100, 200])
    counts = np.array([[10, 5, 10, 5, 10], [0, 0, 0, 0, 0], [30, 0, 0, 0, 0]], np.int64)
    for me in range(3):
        with pytest.raises(rs.RSortError) as e:
            rs.multi_exchange_plan(3, me, counts, spl, [1000, 1000, 1])  # rank 2's output holds 1 key
        assert e.value.status == 9


def test_sample_plan():
    sp = rs.multi_sample_plan([1 << 30] * 8, (1 << 20) // 8)
    assert sp.stride == 1 << 13 and list(sp.count)[:8] == [1 << 17] * 8 and sp.row_len == 1 << 17
    sp = rs.multi_sample_plan([10, 0, 3], 100)
    assert sp.stride == 1 and list(sp.count)[:3] == [10, 0, 3] and sp.row_len == 10 and sp.total == 13
    assert [rs.multi_quantile_index(sp, i) for i in (1, 2)] == [4, 8]
    sp = rs.multi_sample_plan([0, 0], 5)
    assert sp.total == 0 and sp.row_len == 1
