"""The multi-GPU sort (cuda.radixsort_amd/multi.py) with the real kernels on the MI355X box:
two ranks sharing cuda:0 over gloo (host-side exchange), and one rank over RCCL ("nccl") --
the driver's 8-GPU run uses the same code with one rank per GPU. Parity: the ranks' outputs,
concatenated in rank order, equal Baseline1 (the oracle) on the union of the inputs."""
import os
import socket
import sys
import tempfile
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from _util import oracle_sort, oracle_sort_pairs, uniform_keys, zipf_keys  # noqa: E402

pytestmark = pytest.mark.gpu
PKG = Path(__file__).resolve().parent.parent / "cuda.radixsort_amd"


def _inputs(rank, n, dist_name, pairs):
    gen = zipf_keys if dist_name == "zipf" else uniform_keys
    keys = gen(n + 1031 * rank, seed=0x5EED + rank)
    vals = (np.arange(keys.size, dtype=np.uint32) + np.uint32(rank << 24)) if pairs else None
    return keys, vals


def _worker(rank, world, port, n, dist_name, pairs, k, out_dir):
    sys.path.insert(0, str(PKG))
    import multi
    import radixsort as rs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, vals = _inputs(rank, n, dist_name, pairs)
        dk = rs.from_numpy_u32(keys)
        dv = rs.from_numpy_u32(vals) if pairs else None
        ok, ov, off = multi.dist_sort(dk, k_bits=k, vals=dv)
        torch.cuda.synchronize()
        np.save(f"{out_dir}/k{rank}.npy", rs.to_numpy_u32(ok))
        if pairs:
            np.save(f"{out_dir}/v{rank}.npy", rs.to_numpy_u32(ov))
        np.save(f"{out_dir}/o{rank}.npy", np.array([off], np.int64))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,dist_name,pairs,k", [(2, "uniform", False, 8), (2, "zipf", True, 8),
                                                     (3, "uniform", True, 4)])
def test_dist_sort_ranks_sharing_one_gpu(tmp_path, world, dist_name, pairs, k):
    n = 1 << 20
    mp.spawn(_worker, args=(world, _free_port(), n, dist_name, pairs, k, str(tmp_path)), nprocs=world, join=True)
    all_k, all_v = zip(*[_inputs(r, n, dist_name, pairs) for r in range(world)])
    keys = np.concatenate(all_k)
    got = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    offs = [int(np.load(tmp_path / f"o{r}.npy")[0]) for r in range(world)]
    assert offs == list(np.cumsum([0] + [g.size for g in got[:-1]]))
    if pairs:
        rk, rv = oracle_sort_pairs(keys, np.concatenate(all_v), k)
        assert np.array_equal(np.concatenate(got), rk)
        assert np.array_equal(np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)]), rv)
    else:
        assert np.array_equal(np.concatenate(got), oracle_sort(keys, k))


def test_dist_sort_rccl_single_rank():
    """The RCCL path end to end (all_reduce, all_to_all_single on device tensors) at world 1."""
    sys.path.insert(0, str(PKG))
    import multi
    import radixsort as rs
    torch.cuda.set_device(0)
    with tempfile.TemporaryDirectory() as td:
        store = dist.FileStore(os.path.join(td, "store"), 1)
        dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            x = zipf_keys(700001, seed=9)
            vals = np.arange(x.size, dtype=np.uint32)
            ok, ov, off = multi.dist_sort(rs.from_numpy_u32(x), 8, vals=rs.from_numpy_u32(vals))
            torch.cuda.synchronize()
            rk, rv = oracle_sort_pairs(x, vals, 8)
            assert off == 0
            assert np.array_equal(rs.to_numpy_u32(ok), rk) and np.array_equal(rs.to_numpy_u32(ov), rv)
        finally:
            dist.destroy_process_group()


# ------------------------------------------------------------------ C ABI: rsort_u32_multi over RCCL
def test_c_multi_single_rank():
    """rsort_u32_multi with a one-rank RCCL communicator: every step (top histogram, all-reduce,
    partition, all-gather, grouped send/recv, in-place local sort) runs; result = Baseline1."""
    sys.path.insert(0, str(PKG))
    import radixsort as rs
    torch.cuda.set_device(0)
    comm = rs.RcclComm(1, 0, rs.rccl_unique_id())
    try:
        for n, pairs in ((1000003, False), (600001, True), (0, False)):
            x = zipf_keys(n, seed=n) if n else np.zeros(0, np.uint32)
            vals = np.arange(n, dtype=np.uint32) if pairs else None
            ok, ov, off = rs.multi_sort_device(comm, rs.from_numpy_u32(x), 8,
                                               vals=rs.from_numpy_u32(vals) if pairs else None)
            torch.cuda.synchronize()
            assert off == 0 and ok.numel() == n
            if pairs:
                rk, rv = oracle_sort_pairs(x, vals, 8)
                assert np.array_equal(rs.to_numpy_u32(ok), rk) and np.array_equal(rs.to_numpy_u32(ov), rv)
            else:
                assert np.array_equal(rs.to_numpy_u32(ok), oracle_sort(x, 8))
        # capacity too small is reported, not overrun
        x = uniform_keys(5000)
        with pytest.raises(rs.RSortError) as e:
            rs.multi_sort_device(comm, rs.from_numpy_u32(x), 8, capacity=100)
        assert e.value.status == 9
    finally:
        comm.close()


def _c_multi_worker(rank, world, uid_path, out_dir, n, pairs):
    sys.path.insert(0, str(PKG))
    import radixsort as rs
    torch.cuda.set_device(0)
    uid = Path(uid_path).read_bytes()
    comm = rs.RcclComm(world, rank, uid)
    try:
        keys, vals = _inputs(rank, n, "zipf", pairs)
        ok, ov, off = rs.multi_sort_device(comm, rs.from_numpy_u32(keys), 8,
                                           vals=rs.from_numpy_u32(vals) if pairs else None)
        torch.cuda.synchronize()
        np.save(f"{out_dir}/k{rank}.npy", rs.to_numpy_u32(ok))
        if pairs:
            np.save(f"{out_dir}/v{rank}.npy", rs.to_numpy_u32(ov))
        np.save(f"{out_dir}/o{rank}.npy", np.array([off], np.int64))
    finally:
        comm.close()


def test_c_multi_two_ranks_one_gpu(tmp_path):
    """Two RCCL ranks on one GPU (the pool's boxes have one): the exchange logic of the 8-GPU
    path with real kernels. Skipped if RCCL refuses two ranks on one device."""
    sys.path.insert(0, str(PKG))
    import radixsort as rs
    uid_path = tmp_path / "uid"
    uid_path.write_bytes(rs.rccl_unique_id())
    n, world, pairs = 1 << 19, 2, True
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_c_multi_worker, args=(r, world, str(uid_path), str(tmp_path), n, pairs))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    if any(p.exitcode != 0 for p in procs):
        for p in procs:
            if p.is_alive():
                p.kill()
        pytest.skip(f"RCCL with {world} ranks on one GPU unavailable (exit codes {[p.exitcode for p in procs]})")
    all_k, all_v = zip(*[_inputs(r, n, "zipf", pairs) for r in range(world)])
    got = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    offs = [int(np.load(tmp_path / f"o{r}.npy")[0]) for r in range(world)]
    assert offs == list(np.cumsum([0] + [g.size for g in got[:-1]]))
    rk, rv = oracle_sort_pairs(np.concatenate(all_k), np.concatenate(all_v), 8)
    assert np.array_equal(np.concatenate(got), rk)
    assert np.array_equal(np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)]), rv)


# ------------------------------------------------------------------ >= 2 GiB exchange messages
def _sorted_ref(d_keys):
    return torch.sort(d_keys.to(torch.int64) & 0xFFFFFFFF)[0]


def test_dist_sort_rccl_2gib_message():
    """One rank sending itself 2^29 + 3 keys (a 2 GiB message): this RCCL leaves the second half
    of such a message unwritten, so multi.py exchanges it in rounds of <= 512 MiB pieces."""
    sys.path.insert(0, str(PKG))
    import multi
    import radixsort as rs
    torch.cuda.set_device(0)
    n = (1 << 29) + 3
    with tempfile.TemporaryDirectory() as td:
        store = dist.FileStore(os.path.join(td, "store"), 1)
        dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            keys = rs.empty_u32(n)
            rs.gen_uniform(keys, 77)
            ok, _, off = multi.dist_sort(keys, 8)
            torch.cuda.synchronize()
            assert off == 0 and ok.numel() == n
            assert torch.equal(ok.to(torch.int64) & 0xFFFFFFFF, _sorted_ref(keys))
        finally:
            dist.destroy_process_group()


def test_c_multi_2gib_message():
    """rsort_u32_multi at one rank with a 2 GiB self message: grouped send/recv in pieces."""
    sys.path.insert(0, str(PKG))
    import radixsort as rs
    torch.cuda.set_device(0)
    n = (1 << 29) + 5
    comm = rs.RcclComm(1, 0, rs.rccl_unique_id())
    try:
        keys = rs.empty_u32(n)
        rs.gen_uniform(keys, 78)
        ok, _, off = rs.multi_sort_device(comm, keys, 8)
        torch.cuda.synchronize()
        assert off == 0 and ok.numel() == n
        assert torch.equal(ok.to(torch.int64) & 0xFFFFFFFF, _sorted_ref(keys))
    finally:
        comm.close()
