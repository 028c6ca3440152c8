"""Pin the CPU oracle (oracle/rsort_oracle.c) before trusting it as the parity checker.

1. Against the golden vectors in tests/golden/reference_vectors.json, which hold the
   REFERENCE's own outputs (oracle/_ref, built from Baseline1.cu:15-64 / Baseline4.cu:67-273).
2. Against the reference build itself, live, where /root/reference exists (build container).
3. Internal consistency of the Baseline4 block-pass intermediates (Baseline4.cu:102-242).
"""
import numpy as np
import pytest

from _util import (fnv1a64, glibc_rand, oracle_block_pass, oracle_sort, oracle_sort_pairs,
                   ref_lib, uniform_keys, zipf_keys, _ptr)


def _inputs(case):
    src = case["source"]
    if src == "glibc_rand_debug":
        return glibc_rand(case["n"], debug=True)
    if src == "glibc_rand":
        return glibc_rand(case["n"])
    if src == "uniform":
        return uniform_keys(case["n"], case["seed"])
    if src == "zipf":
        return zipf_keys(case["n"], case["seed"])
    raise AssertionError(src)


def test_golden_inputs_regenerate(golden):
    """The generators used by tests and bench reproduce the fixtures' inputs."""
    for case in golden["sort_cases"]:
        x = _inputs(case)
        assert fnv1a64(x) == case["fnv_in"], case["name"]
        if "input" in case:
            assert x.tolist() == case["input"]


def test_oracle_matches_reference_golden(golden):
    for case in golden["sort_cases"]:
        x = _inputs(case)
        y = oracle_sort(x, case["k"])
        assert fnv1a64(y) == case["fnv_out"], case["name"]
        for i, v in case.get("samples", {}).items():
            assert int(y[int(i)]) == v
        if "output" in case:
            assert y.tolist() == case["output"]


def test_oracle_block_sort_matches_reference_golden(golden):
    lib = __import__("_util").oracle()
    for case in golden["block_cases"]:
        x = glibc_rand(case["n"])
        out = np.empty_like(x)
        assert lib.oracle_block_sort(_ptr(x), x.size, _ptr(out), case["k"], case["block"]) == 0
        assert fnv1a64(out) == case["fnv_out"], case["name"]


def test_known_answers_from_survey(golden):
    """SURVEY §8c known answers of the reference's own runs (out[0], out[n/2], out[n-1])."""
    dbg = next(c for c in golden["sort_cases"] if c["name"] == "ref_debug_513_k4")
    assert (dbg["output"][0], dbg["output"][256], dbg["output"][512]) == (0, 128, 255)
    big = next(c for c in golden["sort_cases"] if c["name"].startswith("ref_default") and c["k"] == 8)
    n = big["n"]
    s = big["samples"]
    assert (s["0"], s[str(n // 2)], s[str(n - 1)]) == (37, 1073726730, 2147483611)


@pytest.mark.parametrize("k", [1, 3, 4, 7, 8, 11, 12, 16])
def test_oracle_vs_numpy(k):
    x = uniform_keys(20011, seed=k)
    assert np.array_equal(oracle_sort(x, k), np.sort(x))


def test_oracle_in_place_and_empty():
    x = uniform_keys(1001)
    y = x.copy()
    lib = __import__("_util").oracle()
    assert lib.oracle_sort_by_host(_ptr(y), y.size, _ptr(y), 8) == 0
    assert np.array_equal(y, np.sort(x))
    e = np.empty(0, np.uint32)
    assert lib.oracle_sort_by_host(_ptr(e), 0, _ptr(e), 8) == 0


def test_oracle_pairs_is_stable():
    k = zipf_keys(50001)
    v = np.arange(k.size, dtype=np.uint32)
    ko, vo = oracle_sort_pairs(k, v, 8)
    order = np.argsort(k, kind="stable")
    assert np.array_equal(ko, k[order])
    assert np.array_equal(vo, v[order])


@pytest.mark.parametrize("n,k,tile,chunk", [(513, 4, 64, 64), (5000, 8, 256, 1024), (70001, 8, 4096, 4096 * 3),
                                            (4097, 5, 512, 512)])
def test_block_pass_intermediates(n, k, tile, chunk):
    x = uniform_keys(n, seed=n)
    bit = 0 if k != 5 else 30  # 30: short last digit (32 - 30 = 2 bits)
    h, s, loc, out = oracle_block_pass(x, k, bit, tile, chunk)
    R = 1 << k
    nchunks = (n - 1) // chunk + 1
    d = (x >> np.uint32(bit)) & np.uint32(R - 1)
    # histogram table, column-major [digit][chunk]
    ref_h = np.zeros((R, nchunks), np.uint32)
    np.add.at(ref_h, (d, np.arange(n) // chunk), 1)
    assert np.array_equal(h, ref_h.ravel())
    assert np.array_equal(s, np.concatenate([[0], np.cumsum(ref_h.ravel())[:-1]]).astype(np.uint32))
    # each tile stably sorted by digit
    for t0 in range(0, n, tile):
        seg = x[t0:t0 + tile]
        sd = (seg >> np.uint32(bit)) & np.uint32(R - 1)
        assert np.array_equal(loc[t0:t0 + tile], seg[np.argsort(sd, kind="stable")])
    # pass output == stable counting sort by that digit
    assert np.array_equal(out, x[np.argsort(d, kind="stable")])


ref = ref_lib()


@pytest.mark.skipif(ref is None, reason="reference build needs /root/reference (build container only)")
@pytest.mark.parametrize("n,k", [(513, 4), (65537, 8), (100003, 3), (99991, 16), (1 << 18, 7)])
def test_oracle_vs_live_reference(n, k):
    x = uniform_keys(n, seed=n + k)
    y_ref = np.empty_like(x)
    ref.ref_sort_by_host(_ptr(x), n, _ptr(y_ref), k)
    assert np.array_equal(oracle_sort(x, k), y_ref)


@pytest.mark.skipif(ref is None, reason="reference build needs /root/reference (build container only)")
@pytest.mark.parametrize("n,k,bs", [(513, 4, 64), (100003, 8, 1000), (4097, 2, 512), (70001, 16, 4096)])
def test_block_oracle_vs_live_reference(n, k, bs):
    x = zipf_keys(n, seed=bs)
    y_ref = np.empty_like(x)
    ref.ref_block_sort(_ptr(x), n, _ptr(y_ref), k, bs)
    lib = __import__("_util").oracle()
    y = np.empty_like(x)
    assert lib.oracle_block_sort(_ptr(x), n, _ptr(y), k, bs) == 0
    assert np.array_equal(y, y_ref)


@pytest.mark.skipif(ref is None, reason="reference build needs /root/reference (build container only)")
@pytest.mark.parametrize("k", [3, 5, 7])
def test_reference_block_algorithm_breaks_when_k_does_not_divide_32(k):
    """Documented reference defect: Baseline4.cu:162/:172/:182 shift by (bit + innerBit) >= 32
    on the last digit when k does not divide 32 (UB; x86 masks the count), so its local sort
    is by the wrong bits and its output is not even a permutation. Baseline1 (the parity
    target, Baseline1.cu:30-49) has no such shift and is correct; our oracle_block_pass clamps
    the last digit to 32 - bit bits and agrees with Baseline1."""
    n, bs = 4097, 512
    x = zipf_keys(n, seed=bs)
    # The defect is undefined behaviour that also writes out of bounds, so the reference runs in
    # a child process: either it dies (heap corruption) or its output is not a permutation.
    import subprocess
    import sys
    import tempfile
    from pathlib import Path
    with tempfile.TemporaryDirectory() as td:
        xin, yout = Path(td) / "x.npy", Path(td) / "y.npy"
        np.save(xin, x)
        code = (
            "import ctypes, numpy as np, sys; sys.path.insert(0, %r); from _util import ref_lib\n"
            "x = np.load(%r); y = np.empty_like(x); lib = ref_lib()\n"
            "lib.ref_block_sort(x.ctypes.data, x.size, y.ctypes.data, %d, %d); np.save(%r, y)\n"
        ) % (str(Path(__file__).parent), str(xin), k, bs, str(yout))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120)
        if r.returncode == 0:
            y_ref = np.load(yout)
            assert not np.array_equal(np.sort(y_ref), np.sort(x))
    lib = __import__("_util").oracle()
    y = np.empty_like(x)
    assert lib.oracle_block_sort(_ptr(x), n, _ptr(y), k, bs) == 0
    y1 = np.empty_like(x)
    ref.ref_sort_by_host(_ptr(x), n, _ptr(y1), k)
    assert np.array_equal(y, y1)
