"""Shared test helpers: oracle loaders, synthetic workloads, digests.

The oracle (``oracle/liboracle.so``) and the reference build (``oracle/_ref/libref.so``) are
TEST INFRASTRUCTURE: only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg load them. The product path is ``cuda.radixsort_amd`` (HIP) and never imports this file.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
GOLDEN_DIR = ROOT / "tests" / "golden"

_u32p = ctypes.POINTER(ctypes.c_uint32)


def _ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u32p)


_ORACLE = None


def oracle() -> ctypes.CDLL:
    """liboracle.so (CPU restatement of Baseline1/Baseline4); built on first use."""
    global _ORACLE
    if _ORACLE is None:
        so = ORACLE_DIR / "liboracle.so"
        src = ORACLE_DIR / "rsort_oracle.c"
        if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "liboracle.so"], check=True)
        lib = ctypes.CDLL(str(so))
        i64, c_int = ctypes.c_int64, ctypes.c_int
        lib.oracle_sort_by_host.argtypes = [_u32p, i64, _u32p, c_int]
        lib.oracle_sort_pairs_by_host.argtypes = [_u32p, _u32p, i64, _u32p, _u32p, c_int]
        lib.oracle_block_pass.argtypes = [_u32p, i64, c_int, c_int, i64, i64, _u32p, _u32p, _u32p, _u32p]
        lib.oracle_block_sort.argtypes = [_u32p, i64, _u32p, c_int, i64]
        lib.oracle_fnv1a64.argtypes = [_u32p, i64]
        lib.oracle_fnv1a64.restype = ctypes.c_uint64
        lib.oracle_fill_rand.argtypes = [_u32p, i64, c_int]
        _ORACLE = lib
    return _ORACLE


def ref_lib():
    """oracle/_ref/libref.so: the reference's own sortByHost / Baseline4 sort, or None."""
    so = ORACLE_DIR / "_ref" / "libref.so"
    if not so.exists():
        if Path("/root/reference/SourceCode").is_dir():
            subprocess.run(["bash", str(ORACLE_DIR / "build_ref.sh")], check=True,
                           stdout=subprocess.DEVNULL)
        if not so.exists():
            return None
    lib = ctypes.CDLL(str(so))
    lib.ref_sort_by_host.argtypes = [_u32p, ctypes.c_int, _u32p, ctypes.c_int]
    lib.ref_block_sort.argtypes = [_u32p, ctypes.c_int, _u32p, ctypes.c_int, ctypes.c_int]
    return lib


# ----------------------------------------------------------------------------- oracle calls
def oracle_sort(keys: np.ndarray, nbits: int) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    out = np.empty_like(keys)
    assert oracle().oracle_sort_by_host(_ptr(keys), keys.size, _ptr(out), nbits) == 0
    return out


def oracle_sort_pairs(keys: np.ndarray, vals: np.ndarray, nbits: int):
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    vals = np.ascontiguousarray(vals, dtype=np.uint32)
    ko, vo = np.empty_like(keys), np.empty_like(vals)
    assert oracle().oracle_sort_pairs_by_host(_ptr(keys), _ptr(vals), keys.size, _ptr(ko), _ptr(vo), nbits) == 0
    return ko, vo


def oracle_block_pass(keys: np.ndarray, nbits: int, bit: int, tile: int, chunk: int):
    """Per-pass intermediates of Baseline4: (hist_cm, scan_cm, local, out)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    n = keys.size
    nchunks = (n - 1) // chunk + 1
    h = np.empty((1 << nbits) * nchunks, np.uint32)
    s = np.empty_like(h)
    loc = np.empty_like(keys)
    out = np.empty_like(keys)
    rc = oracle().oracle_block_pass(_ptr(keys), n, nbits, bit, tile, chunk, _ptr(h), _ptr(s), _ptr(loc), _ptr(out))
    assert rc == 0
    return h, s, loc, out


def fnv1a64(a: np.ndarray) -> str:
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return "%016x" % oracle().oracle_fnv1a64(_ptr(a), a.size)


def glibc_rand(n: int, debug: bool = False) -> np.ndarray:
    """The reference's own input stream: glibc rand(), default seed (Parallel7.cu:717-723)."""
    a = np.empty(n, np.uint32)
    oracle().oracle_fill_rand(_ptr(a), n, 1 if debug else 0)
    return a


# ----------------------------------------------------------------------------- workloads
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_keys(n: int, seed: int = 0x5EED) -> np.ndarray:
    """key[i] = high 32 bits of splitmix64(seed + i)  (SURVEY §8d); == rsort_gen_uniform."""
    i = np.arange(n, dtype=np.uint64) + np.uint64(seed)
    return (splitmix64(i) >> np.uint64(32)).astype(np.uint32)


def fmix32(h: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = h.astype(np.uint32)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
        return h


def zipf_cdf_u32(ranks: int = 1 << 20, s: float = 1.0) -> np.ndarray:
    """Inclusive CDF of Zipf(s) over `ranks`, scaled to u32 thresholds (last = 2^32-1)."""
    w = 1.0 / np.arange(1, ranks + 1, dtype=np.float64) ** s
    c = np.cumsum(w)
    c /= c[-1]
    t = np.floor(c * 4294967296.0)
    t = np.minimum(t, 4294967295.0)
    t[-1] = 4294967295.0
    return t.astype(np.uint32)


def zipf_keys(n: int, seed: int = 0x5EED, ranks: int = 1 << 20, s: float = 1.0) -> np.ndarray:
    """key = fmix32(rank), rank ~ Zipf(s) by inverse CDF of u = uniform_keys (== rsort_gen_zipf)."""
    u = uniform_keys(n, seed)
    cdf = zipf_cdf_u32(ranks, s)
    rank = np.searchsorted(cdf, u, side="left")  # first r with u <= cdf[r]
    rank = np.minimum(rank, ranks - 1).astype(np.uint32)
    return fmix32(rank)


def env_flag(name: str) -> bool:
    return os.environ.get(name, "") not in ("", "0", "false", "False")
