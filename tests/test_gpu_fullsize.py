"""Full BASELINE sizes (2^26 and 2^30 keys, 2^30 pairs) on the GPU: bit-exact against the
oracle (the Baseline1.cu:15-64 restatement, pinned to the reference build) at C2, C3 and C4, and
through size-independent properties: sortedness, equality with the vendor sort (rocPRIM; a sort's
output is unique), an order-independent multiset fingerprint, and for pairs the exact gather
identity keys_out[i] == keys_in[vals_out[i]] plus stability (vals increasing within runs of equal
keys, vals being the input index). Beyond the configs: one sort of 2^31 + 12345 keys (rsort.h
promises n < 2^32; every position is carried in u32)."""
import numpy as np
import pytest

from _rs import rs
from _util import oracle_sort, oracle_sort_pairs, zipf_cdf_u32

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

M32 = 0xFFFFFFFF


def as_u64(t):
    return t.to(torch.int64) & M32


def fingerprint(t):
    """Order-independent: (sum x, sum mix(x)) mod 2^64 over the u32 keys."""
    x = as_u64(t)
    h = x * 0x9E3779B1
    h = h ^ ((h >> 15) & 0x1FFFF)
    h = h * 0x85EBCA77
    return int(x.sum()), int(h.sum())


def is_sorted(t):
    x = as_u64(t)
    return bool((x[1:] >= x[:-1]).all())


@pytest.mark.parametrize("n,k", [(1 << 26, 4), (1 << 30, 8), ((1 << 28) + 77, 4), ((1 << 27) - 3, 3)])
def test_fullsize_uniform(n, k):
    keys = rs.empty_u32(n)
    rs.gen_uniform(keys, 0x5EED)
    out = rs.empty_u32(n)
    rs.sort_device(keys, out, k)
    ref = rs.empty_u32(n)
    rs.vendor_sort_device(keys, ref)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert is_sorted(out)
    assert fingerprint(out) == fingerprint(keys)
    del ref


@pytest.mark.parametrize("n,k", [(1 << 26, 4), (1 << 30, 8)])
def test_fullsize_vs_baseline1(n, k):
    """C2 (2^26, k=4) and C3 (2^30, k=8) uniform keys, bit-exact against the oracle -- the
    reference's own self-check (Parallel7.cu:747-767: sortByHost vs sortByDevice) at the config
    sizes. The oracle runs on the host (~9 s at 2^30)."""
    keys = rs.empty_u32(n)
    rs.gen_uniform(keys, 0x5EED)
    out = rs.empty_u32(n)
    rs.sort_device(keys, out, k)
    torch.cuda.synchronize()
    expect = oracle_sort(rs.to_numpy_u32(keys), k)
    assert np.array_equal(rs.to_numpy_u32(out), expect)


def test_fullsize_pairs_zipf_vs_oracle():
    """C4 (2^30 Zipf keys + index payloads, k=8), bit-exact against the oracle's stable pairs sort
    (the Baseline1 loop carrying the payload)."""
    n = 1 << 30
    keys = rs.empty_u32(n)
    rs.gen_zipf(keys, rs.from_numpy_u32(zipf_cdf_u32()), 0x5EED)
    vals = rs.empty_u32(n)
    rs.gen_iota(vals, 0)
    ko, vo = rs.empty_u32(n), rs.empty_u32(n)
    rs.sort_device(keys, ko, 8, vals_in=vals, vals_out=vo)
    torch.cuda.synchronize()
    rk, rv = oracle_sort_pairs(rs.to_numpy_u32(keys), rs.to_numpy_u32(vals), 8)
    assert np.array_equal(rs.to_numpy_u32(ko), rk)
    assert np.array_equal(rs.to_numpy_u32(vo), rv)


def test_beyond_2_31_keys():
    """n = 2^31 + 12345 (8.6 GB per buffer), k = 8: every chunk, group and table position above
    2^31 in u32. Checked on the device: sorted, the input's multiset fingerprint, equal to rocPRIM."""
    n = (1 << 31) + 12345
    keys = rs.empty_u32(n)
    rs.gen_uniform(keys, 0xB16)
    out = rs.empty_u32(n)
    rs.sort_device(keys, out, 8)
    fp_in = rs.fingerprint(keys)[0]
    assert rs.fingerprint(out) == (fp_in, 0)
    ref = rs.empty_u32(n)
    rs.vendor_sort_device(keys, ref)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_near_2_32_keys_unaligned_output():
    """n = 2^32 - 20 keys into an output 31 keys past a 128-B boundary. The whole-line
    kernels count positions from the output's 128-B-aligned base, so n + 31 would not fit their 32-bit
    positions: the passes into that output must take rs_scatter (and the sort fixed chunks) -- sorted, the input's
    multiset, and the words around the output untouched. (~52 GB of device memory.)"""
    n = (1 << 32) - 20
    keys = rs.empty_u32(n)
    rs.gen_uniform(keys, 0x2_32)
    big = torch.full((n + 32 + 64,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    off = 32 + 31  # 128-B-aligned base + 31 keys (torch allocations are 256-B aligned)
    out = big[off:off + n]
    assert (out.data_ptr() & 127) == 124
    rs.scatter_kernels_used(reset=True)
    rs.sort_device(keys, out, 8)
    used = rs.scatter_kernels_used(reset=True)
    # the passes into `out` take rs_scatter; those into the (256-B-aligned) workspace keep the lines
    assert any(k.startswith("rs_scatter<") for k in used), used
    fp_in = rs.fingerprint(keys)[0]
    del keys
    assert rs.fingerprint(out) == (fp_in, 0)
    torch.cuda.synchronize()
    assert int((big[:off] != 0x5A5A5A5A).sum()) == 0 and int((big[off + n:] != 0x5A5A5A5A).sum()) == 0


def test_fullsize_pairs_zipf():
    n = 1 << 30
    cdf = rs.from_numpy_u32(zipf_cdf_u32())
    keys = rs.empty_u32(n)
    rs.gen_zipf(keys, cdf, 0x5EED)
    vals = rs.empty_u32(n)
    rs.gen_iota(vals, 0)
    ko, vo = rs.empty_u32(n), rs.empty_u32(n)
    rs.sort_device(keys, ko, 8, vals_in=vals, vals_out=vo)
    torch.cuda.synchronize()
    assert is_sorted(ko)
    idx = as_u64(vo)
    assert torch.equal(keys[idx], ko)                       # a permutation carrying its key
    assert int(torch.bincount(idx[:: 1 << 10] >> 20, minlength=1024).min()) >= 0
    same = ko[1:] == ko[:-1]
    assert bool((idx[1:][same] > idx[:-1][same]).all())     # stable
    assert fingerprint(ko) == fingerprint(keys)


@pytest.mark.parametrize("dist_name", ["uniform", "zipf"])
def test_fullsize_ballot_ranking_agrees(dist_name):
    """C3 size through RSORT_RANK_BALLOT (wave64 ballot peer match, no lane-order premise) and
    through the default lane-ordered LDS-add ranking: two independent rankings, one unique sorted
    output -- bit-identical, sorted, same multiset."""
    n = 1 << 30
    keys = rs.empty_u32(n)
    if dist_name == "uniform":
        rs.gen_uniform(keys, 0xB411)
    else:
        rs.gen_zipf(keys, rs.from_numpy_u32(zipf_cdf_u32()), 0xB411)
    out = rs.empty_u32(n)
    rs.sort_device(keys, out, 8)
    fp_default = rs.fingerprint(out)
    with rs.rank_algo(rs.RANK_BALLOT):
        out_b = rs.empty_u32(n)
        rs.sort_device(keys, out_b, 8)
    torch.cuda.synchronize()
    assert torch.equal(out, out_b)
    assert fp_default == (rs.fingerprint(keys)[0], 0)
