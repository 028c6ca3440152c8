"""Multi-GPU path (cuda.radixsort_amd/multi.py) on CPU: the distributed logic —
global top-bits histogram, splitter choice, stable partition, count + key all-to-all, local
sort, global offsets — run with the gloo backend over world_size 2 and 4 processes. The three
per-device steps are replaced by a numpy restatement of what the HIP kernels compute
(rsort_top_histogram, rsort_partition_device, the LSD sort checked by the oracle), so this
checks the exchange protocol; the kernels themselves are covered by test_gpu_parity.py.

Parity: concatenating the ranks' outputs in rank order must equal Baseline1 (the oracle) on the
union of all ranks' inputs; with payloads the order must be the stable one."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import oracle_sort, oracle_sort_pairs, uniform_keys, zipf_keys

PKG = Path(__file__).resolve().parent.parent / "cuda.radixsort_amd"
if str(PKG) not in sys.path:
    sys.path.insert(0, str(PKG))
import multi  # noqa: E402


def _u32(t):
    return t.numpy().view(np.uint32)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32).copy())


class NumpyOps:
    """CPU stand-in for multi.GpuOps with the kernels' exact semantics (test-only)."""

    def sample(self, keys, stride, count, row_len):
        # rsort_sample_device: key[min(n - 1, j * stride + stride / 2)] for j < count, then padding
        k = _u32(keys)
        out = np.full(row_len, 0xFFFFFFFF, np.uint32)
        if count and k.size:
            j = np.arange(count, dtype=np.int64)
            out[:count] = k[np.minimum(k.size - 1, j * stride + stride // 2)]
        return _t(out)

    def sort_keys(self, keys):
        return _t(np.sort(_u32(keys)))

    def partition(self, keys, vals, splitters):
        k = _u32(keys)
        # bucket = number of splitters <= key (the kernels' kDigitSplit digit)
        b = np.searchsorted(np.asarray(splitters, np.uint32), k, side="right")
        order = np.argsort(b, kind="stable")
        starts = np.searchsorted(b[order], np.arange(len(splitters) + 2), side="left").astype(np.int32)
        vo = _t(_u32(vals)[order]) if vals is not None else None
        return _t(k[order]), vo, torch.from_numpy(starts)

    def sort(self, keys, vals, k_bits):
        if vals is None:
            return _t(oracle_sort(_u32(keys), k_bits)), None
        rk, rv = oracle_sort_pairs(_u32(keys), _u32(vals), k_bits)
        return _t(rk), _t(rv)


def _inputs(rank, n, dist_name, pairs):
    gen = zipf_keys if dist_name == "zipf" else uniform_keys
    keys = gen(n + 37 * rank, seed=0x5EED + rank)  # ragged: ranks hold different counts
    if dist_name == "skewed":
        keys = keys & np.uint32(0x0000FFFF)  # every key in the lowest 1/65536 of the key range
    elif dist_name == "hot":
        keys = keys.copy()
        keys[: keys.size * 3 // 4] = 0xC0FFEE  # one key holds 3/4 of every rank's keys
    elif dist_name == "equal":
        keys = np.full(keys.size, 7, np.uint32)
    elif dist_name == "maxkey":
        keys = keys.copy()
        keys[::2] = 0xFFFFFFFF  # half the keys are the largest key (no bucket above it)
    elif dist_name == "empty1" and rank == 1:
        keys = keys[:0]
    vals = (np.arange(keys.size, dtype=np.uint32) + np.uint32(rank << 24)) if pairs else None
    return keys, vals


def _worker(rank, world, port, n, dist_name, pairs, out_dir, max_message=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if max_message:
        multi.MAX_PIECE = max_message  # exchange in several rounds of pieces
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, vals = _inputs(rank, n, dist_name, pairs)
        ok, ov, off = multi.dist_sort(_t(keys), k_bits=8, vals=_t(vals) if pairs else None, ops=NumpyOps())
        np.save(f"{out_dir}/k{rank}.npy", _u32(ok))
        if pairs:
            np.save(f"{out_dir}/v{rank}.npy", _u32(ov))
        np.save(f"{out_dir}/o{rank}.npy", np.array([off], np.int64))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,dist_name,pairs,max_message", [(2, "uniform", False, None), (2, "zipf", True, None),
                                                               (4, "uniform", True, None), (4, "skewed", False, None),
                                                               (3, "zipf", False, None), (3, "uniform", True, 1000),
                                                               (2, "skewed", False, 777), (8, "uniform", True, 3000),
                                                               (8, "zipf", False, None), (4, "hot", True, None),
                                                               (8, "equal", True, 5000), (3, "maxkey", False, None),
                                                               (4, "empty1", True, None)])
def test_dist_sort_gloo(tmp_path, world, dist_name, pairs, max_message):
    """max_message: keys per exchange message (multi.MAX_PIECE, 2^28 by default: RCCL drops the
    second half of >= 2 GiB messages): small values force several rounds."""
    n = 50_000
    mp.spawn(_worker, args=(world, _free_port(), n, dist_name, pairs, str(tmp_path), max_message), nprocs=world,
             join=True)
    all_k, all_v = zip(*[_inputs(r, n, dist_name, pairs) for r in range(world)])
    keys = np.concatenate(all_k)
    got = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    offs = [int(np.load(tmp_path / f"o{r}.npy")[0]) for r in range(world)]
    assert offs == list(np.cumsum([0] + [g.size for g in got[:-1]]))
    if pairs:
        vals = np.concatenate(all_v)
        rk, rv = oracle_sort_pairs(keys, vals, 8)
        assert np.array_equal(np.concatenate(got), rk)
        assert np.array_equal(np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)]), rv)
    else:
        assert np.array_equal(np.concatenate(got), oracle_sort(keys, 8))
    sizes = np.array([g.size for g in got])
    if dist_name in ("uniform", "zipf", "hot", "equal", "maxkey"):
        # exact-key splitters from the regular sample, hot keys split across ranks: every rank
        # within 5 % of the mean (duplicate-heavy input no longer piles up)
        assert np.abs(sizes - keys.size / world).max() < 0.05 * keys.size / world, sizes


def _cap_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, _ = _inputs(rank, 20_000, "uniform", False)
        cap = 1000 if rank == 1 else None  # one rank's output is far too small
        try:
            multi.dist_sort(_t(keys), 8, ops=NumpyOps(), capacity=cap)
            res = "ok"
        except multi.rs.RSortError as e:
            res = str(e.status)
        (Path(out_dir) / f"r{rank}").write_text(res)
    finally:
        dist.destroy_process_group()


def test_dist_sort_capacity_error_on_every_rank(tmp_path):
    """a capacity overflow on one rank is reported by EVERY rank, before the
    exchange, so no rank is left waiting in a collective (the test would hang otherwise)."""
    world = 3
    mp.spawn(_cap_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert [(tmp_path / f"r{r}").read_text() for r in range(world)] == ["9"] * world


def test_exchange_rounds_never_exceed_the_limit():
    """pieces are a multiple of 64 keys, never above the limit, even when the limit is not
    a multiple of 64 (limit 65, max_message 130: pieces of 64, 3 rounds -- rounding up gave 128); they
    round up only where that stays within the limit, so a message under the limit is one round."""
    import multi
    assert multi.exchange_rounds(130, 65) == (3, 64)
    assert multi.exchange_rounds(0, 1 << 28) == (0, 0)
    # a message that fits the limit is one round (C5's largest, ~2^27 keys: pieces rounded UP to 64)
    assert multi.exchange_rounds(134107614, 1 << 28) == (1, 134107648)
    assert multi.exchange_rounds(1 << 28, 1 << 28) == (1, 1 << 28)
    rng = np.random.default_rng(7)
    for _ in range(2000):
        m = int(rng.integers(1, 1 << 40))
        limit = int(rng.integers(64, 1 << 30))
        rounds, piece = multi.exchange_rounds(m, limit)
        assert 64 <= piece <= limit and piece % 64 == 0
        assert rounds * piece >= m > (rounds - 1) * piece
