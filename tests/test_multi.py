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

    def top_histogram(self, keys, top_bits, stride=1):
        k = _u32(keys)
        if stride > 1:  # rsort_top_histogram_sampled: every stride-th block of 256 keys
            k = k[(np.arange(k.size) // 256) % stride == 0]
        return torch.from_numpy(np.bincount(k >> np.uint32(32 - top_bits), minlength=1 << top_bits).astype(np.int32))

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
        keys = keys & np.uint32(0x0000FFFF)  # all keys in the lowest top-bits bin
    vals = (np.arange(keys.size, dtype=np.uint32) + np.uint32(rank << 24)) if pairs else None
    return keys, vals


def _worker(rank, world, port, n, dist_name, pairs, out_dir, max_message=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if max_message:
        multi.MAX_MESSAGE = max_message  # exchange in several rounds of pieces
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
                                                               (8, "zipf", False, None)])
def test_dist_sort_gloo(tmp_path, world, dist_name, pairs, max_message):
    """max_message: pieces per message in the exchange (multi.MAX_MESSAGE, 2^27 keys by default,
    works around RCCL dropping the second half of >= 2 GiB messages): small values force rounds."""
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
    if dist_name == "uniform":  # splitters (from a 1/16 block sample) balance within a few percent
        sizes = np.array([g.size for g in got])
        assert np.abs(sizes - keys.size / world).max() < 0.05 * keys.size


def test_choose_splitters():
    h = np.zeros(16, np.int64)
    h[[1, 5, 9, 13]] = 10
    s = multi.choose_splitters(h, 4, 4)
    assert s == [2 << 28, 6 << 28, 10 << 28]
    # everything in one bin: later splitters saturate and stay monotone
    h = np.zeros(16, np.int64)
    h[15] = 100
    s = multi.choose_splitters(h, 4, 4)
    assert s == sorted(s) and s[-1] == 0xFFFFFFFF
    assert multi.choose_splitters(np.ones(4096, np.int64), 1, 12) == []
