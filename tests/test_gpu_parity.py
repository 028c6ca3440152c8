"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference's own
golden vectors. Bit-exact everywhere (integer work). Runs on the MI355X box (-m gpu)."""
import numpy as np
import pytest

from _rs import rs
from _util import (fnv1a64, glibc_rand, oracle_block_pass, oracle_sort, oracle_sort_pairs, uniform_keys,
                   zipf_cdf_u32, zipf_keys)

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RANKS = [rs.RANK_MATCH, rs.RANK_SPLIT, rs.RANK_BALLOT]


def dev(a):
    return rs.from_numpy_u32(a)


def host(t):
    return rs.to_numpy_u32(t)


def gpu_sort(x, k, algo=rs.RANK_MATCH, tiles_per_chunk=0):
    with rs.rank_algo(algo):
        p = rs.plan(x.size, k, False, tiles_per_chunk)
        d_in = dev(x)
        d_out = rs.empty_u32(x.size)
        rs.sort_device(d_in, d_out, k, plan_=p)
        torch.cuda.synchronize()
        assert np.array_equal(host(d_in), x), "input buffer was modified"
        return host(d_out)


# ------------------------------------------------------------------ reference golden vectors
def test_reference_debug_vector(golden):
    case = next(c for c in golden["sort_cases"] if c["name"] == "ref_debug_513_k4")
    x = np.array(case["input"], np.uint32)
    for algo in RANKS:
        y = gpu_sort(x, 4, algo)
        assert y.tolist() == case["output"]


@pytest.mark.parametrize("k", [8, 4])
def test_reference_default_vector(golden, k):
    """The reference's own default run: n=(1<<24)+1 glibc rand() keys (Parallel7.cu:708,:721)."""
    case = next(c for c in golden["sort_cases"] if c["name"] == f"ref_default_{(1 << 24) + 1}_k{k}")
    x = glibc_rand(case["n"])
    assert fnv1a64(x) == case["fnv_in"]
    for algo in RANKS:
        y = gpu_sort(x, k, algo)
        assert fnv1a64(y) == case["fnv_out"]
        for i, v in case["samples"].items():
            assert int(y[int(i)]) == v


def test_all_golden_cases(golden):
    for case in golden["sort_cases"]:
        if case["source"] not in ("uniform", "zipf"):
            continue
        x = uniform_keys(case["n"], case["seed"]) if case["source"] == "uniform" else zipf_keys(case["n"], case["seed"])
        y = gpu_sort(x, case["k"])
        assert fnv1a64(y) == case["fnv_out"], case["name"]


# ------------------------------------------------------------------ oracle sweeps
SIZES = [1, 2, 3, 63, 64, 65, 255, 4095, 4096, 4097, 8191, 65536 + 17, 100003, (1 << 20) + 5]


@pytest.mark.parametrize("k", list(range(1, 14)))  # 13: the reference's largest digit (P7:740-745)
@pytest.mark.parametrize("algo", RANKS)
def test_sizes_and_bits_vs_oracle(k, algo):
    for n in SIZES:
        if k == 1 and n > 100003:
            continue
        x = uniform_keys(n, seed=1000 * k + n)
        assert np.array_equal(gpu_sort(x, k, algo), oracle_sort(x, k)), (n, k, algo)


@pytest.mark.parametrize("dist", ["zipf", "allsame", "sorted", "reversed", "fewbits", "topbit"])
def test_distributions(dist):
    n = 300007
    if dist == "zipf":
        x = zipf_keys(n, seed=7)
    elif dist == "allsame":
        x = np.full(n, 0xDEADBEEF, np.uint32)
    elif dist == "sorted":
        x = np.sort(uniform_keys(n))
    elif dist == "reversed":
        x = np.sort(uniform_keys(n))[::-1].copy()
    elif dist == "fewbits":
        x = uniform_keys(n) & np.uint32(0x00F000F0)
    else:
        x = uniform_keys(n) | np.uint32(0x80000000)
    for k in (4, 8, 11):
        for algo in RANKS:
            assert np.array_equal(gpu_sort(x, k, algo), oracle_sort(x, k)), (dist, k, algo)


@pytest.mark.parametrize("k", [8, 6, 5, 4, 3, 2])
def test_large_tile_geometries(k):
    """n >= 2 * CUs * tile selects the 16384-key line tiles (k = 5..8), 4096-key line tiles
    (k = 3, 4) or 8192-key tiles (k <= 2); ragged tails and zipf keys, keys and pairs, against
    the oracle."""
    n = (1 << 23) + 12345
    keys = zipf_keys(n, seed=k) if k % 2 else uniform_keys(n, seed=k)
    p = rs.plan(n, k, False)
    assert p.tile_keys == {8: 16384, 6: 16384, 5: 16384, 4: 4096, 3: 4096, 2: 8192}[k], p.as_dict()
    assert np.array_equal(gpu_sort(keys, k), oracle_sort(keys, k))
    if k >= 5:
        vals = np.arange(n, dtype=np.uint32)
        ko, vo = rs.empty_u32(n), rs.empty_u32(n)
        rs.sort_device(dev(keys), ko, k, vals_in=dev(vals), vals_out=vo)
        torch.cuda.synchronize()
        rk, rv = oracle_sort_pairs(keys, vals, k)
        assert np.array_equal(host(ko), rk) and np.array_equal(host(vo), rv)


def test_lane_order_probe():
    """The default ranking's hardware premise holds on the MI355X (dev/lds_order_lab.hip)."""
    assert rs.lane_order_probe() == 1


@pytest.mark.parametrize("dist", ["uniform", "zipf", "allsame", "fewdigits"])
@pytest.mark.parametrize("tpc", [0, 1, 3, 7])
def test_whole_line_scatter(dist, tpc):
    """k = 5..8 keys at n >= 2 * CUs * 16384 run rs_scatter_lines (whole 128-B lines, per-digit
    carries across tiles, masked first/last lines per chunk): chunk geometries, skew, ragged n."""
    n = (1 << 23) + 4099
    if dist == "uniform":
        x = uniform_keys(n, seed=tpc)
    elif dist == "zipf":
        x = zipf_keys(n, seed=tpc)
    elif dist == "allsame":
        x = np.full(n, 0x12345678, np.uint32)
    else:
        x = uniform_keys(n, seed=tpc) & np.uint32(0x03030303)
    for k in (8, 5, 7):
        p = rs.plan(n, k, False, tpc)
        assert p.tile_keys == 16384 and p.threads == 1024
        assert np.array_equal(gpu_sort(x, k, tiles_per_chunk=tpc), oracle_sort(x, k)), (dist, tpc, k)


def test_whole_line_scatter_unaligned_output():
    """An output pointer that is 4-B but not 16-B aligned keeps the whole-line kernels: positions
    count from its 128-B-aligned base (ScatterArgs::pos_shift) and the slots before it are masked,
    so k = 8 (1024 x 16 line tiles), k = 4 (next-digit counts) and k = 3 all write whole cache
    lines into any 4-B-aligned buffer; bit-exact."""
    n = (1 << 23) + 77
    x = zipf_keys(n, seed=5)
    big = rs.empty_u32(n + 64)
    for k in (8, 4, 3):
        ref = oracle_sort(x, k)
        for off in (1, 2, 3, 17, 31):
            out = big[off:off + n]
            rs.scatter_kernels_used(reset=True)
            rs.sort_device(dev(x), out, k)
            torch.cuda.synchronize()
            assert np.array_equal(host(out), ref), (k, off)
            assert all(u.startswith("rs_scatter_lines") for u in rs.scatter_kernels_used(reset=True)), (k, off)


def test_unaligned_output_leaves_neighbours_untouched():
    """The masked slots before an unaligned output and after its end stay as they were."""
    n = (1 << 22) + 5
    x = uniform_keys(n, seed=55)
    for off in (1, 13, 30):
        big = torch.full((n + 96,), -7, dtype=torch.int32, device="cuda")
        out = big[off:off + n]
        rs.sort_device(dev(x), out, 8)
        torch.cuda.synchronize()
        h = host(big)
        assert np.array_equal(h[off:off + n], oracle_sort(x, 8))
        assert (h[:off] == np.uint32(0xFFFFFFF9)).all() and (h[off + n:] == np.uint32(0xFFFFFFF9)).all(), off


def test_pairs_values_misaligned_against_keys_falls_back():
    """Pairs need (vout - kout) % 16 == 0 for the whole-line kernels (keys and values share the
    line positions); otherwise the same tiles go through rs_scatter. Same result either way."""
    n = (1 << 23) + 19
    x = zipf_keys(n, seed=6)
    vals = np.arange(n, dtype=np.uint32)
    rk, rv = oracle_sort_pairs(x, vals, 8)
    bigk, bigv = rs.empty_u32(n + 8), rs.empty_u32(n + 8)
    for ko, vo, lines in ((0, 1, False), (3, 3, True), (2, 6, True), (5, 2, False)):
        out, vout = bigk[ko:ko + n], bigv[vo:vo + n]
        rs.scatter_kernels_used(reset=True)
        rs.sort_device(dev(x), out, 8, vals_in=dev(vals), vals_out=vout)
        torch.cuda.synchronize()
        assert np.array_equal(host(out), rk) and np.array_equal(host(vout), rv), (ko, vo)
        # (the passes into the workspace's ping-pong buffers take the line kernels either way; the
        # passes into the caller's buffers take rs_scatter when their offsets disagree)
        used = rs.scatter_kernels_used(reset=True)
        assert any(u.startswith("rs_scatter<") for u in used) == (not lines), used


def test_whole_line_scatter_16b_aligned_output():
    """A 16-B but not 128-B aligned output keeps the line kernel (positions shifted to the
    128-B-aligned base, so its lines are still whole L2 lines); keys and pairs."""
    n = (1 << 23) + 333
    x = zipf_keys(n, seed=9)
    vals = np.arange(n, dtype=np.uint32)
    rk, rv = oracle_sort_pairs(x, vals, 8)
    big = rs.empty_u32(n + 32)
    bigv = rs.empty_u32(n + 32)
    for off in (4, 8, 28):
        out = big[off:off + n]
        rs.sort_device(dev(x), out, 8)
        torch.cuda.synchronize()
        assert np.array_equal(host(out), rk), off
        vout = bigv[off:off + n]
        rs.sort_device(dev(x), out, 8, vals_in=dev(vals), vals_out=vout)
        torch.cuda.synchronize()
        assert np.array_equal(host(out), rk) and np.array_equal(host(vout), rv), off


@pytest.mark.parametrize("tpc", [1, 2, 3, 17])
def test_chunk_geometry_does_not_change_the_result(tpc):
    x = zipf_keys(200003, seed=tpc)
    for algo in RANKS:
        assert np.array_equal(gpu_sort(x, 8, algo, tiles_per_chunk=tpc), oracle_sort(x, 8))


# ------------------------------------------------------------------ pairs (stability)
@pytest.mark.parametrize("k", [4, 8, 5, 12])
@pytest.mark.parametrize("algo", RANKS)
def test_pairs_stable_vs_oracle(k, algo):
    for n in (1, 4097, 250001):
        keys = zipf_keys(n, seed=n + k)
        vals = np.arange(n, dtype=np.uint32) ^ np.uint32(0x5A5A5A5A)
        ko_ref, vo_ref = oracle_sort_pairs(keys, vals, k)
        with rs.rank_algo(algo):
            dk, dv = dev(keys), dev(vals)
            ok, ov = rs.empty_u32(n), rs.empty_u32(n)
            rs.sort_device(dk, ok, k, vals_in=dv, vals_out=ov)
            torch.cuda.synchronize()
        assert np.array_equal(host(ok), ko_ref)
        assert np.array_equal(host(ov), vo_ref)


@pytest.mark.parametrize("k", [5, 6, 7, 8])
@pytest.mark.parametrize("dist_name", ["uniform", "zipf"])
def test_pairs_line_tiles_vs_oracle(k, dist_name):
    """Pairs large enough for the 1024 x 8 pair tiles (kGeomLinesPairs): k = 7, 8 through
    rs_scatter_pairs (128-B lines in both arrays, register carries), k = 5, 6 through the 64-B-line
    rs_scatter_lines instances; ragged n, bit-exact against the oracle's stable pairs sort."""
    n = (1 << 23) + 4321
    keys = zipf_keys(n, seed=k) if dist_name == "zipf" else uniform_keys(n, seed=k)
    vals = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)
    ko_ref, vo_ref = oracle_sort_pairs(keys, vals, k)
    p = rs.plan(n, k, True)
    assert (p.threads, p.tile_keys) == (1024, 8192)
    ok, ov = rs.empty_u32(n), rs.empty_u32(n)
    rs.scatter_kernels_used(reset=True)
    rs.sort_device(dev(keys), ok, k, vals_in=dev(vals), vals_out=ov)
    torch.cuda.synchronize()
    used = rs.scatter_kernels_used(reset=True)
    assert np.array_equal(host(ok), ko_ref) and np.array_equal(host(ov), vo_ref)
    assert any(u.startswith("rs_scatter_pairs" if k >= 7 else "rs_scatter_lines") for u in used), used


def test_pairs_host_entry():
    n = 70001
    keys = zipf_keys(n, seed=3)
    vals = np.arange(n, dtype=np.uint32)
    ko, vo = np.empty_like(keys), np.empty_like(vals)
    rs.sortPairsByDevice(keys, vals, n, ko, vo, 8)
    rk, rv = oracle_sort_pairs(keys, vals, 8)
    assert np.array_equal(ko, rk) and np.array_equal(vo, rv)


# ------------------------------------------------------------------ per-pass intermediates (a4-a8)
@pytest.mark.parametrize("n,k,bit,tpc", [(513, 4, 0, 1), (100003, 8, 8, 3), (70001, 5, 30, 2),
                                          (1 << 18, 8, 24, 1), (50001, 12, 12, 2), (4096 * 5, 3, 3, 5)])
@pytest.mark.parametrize("algo", RANKS)
def test_pass_intermediates_vs_block_oracle(n, k, bit, tpc, algo):
    """histogram table / column-major scan / locally sorted tiles / pass output, each against
    the Baseline4 restatement run with the same tile (4096) and chunk geometry."""
    x = zipf_keys(n, seed=n) if k != 12 else uniform_keys(n, seed=n)
    p = rs.plan(n, k, False, tpc)
    h_ref, s_ref, loc_ref, out_ref = oracle_block_pass(x, k, bit, p.tile_keys, p.chunk_keys)
    with rs.rank_algo(algo):
        d = dev(x)
        table = rs.empty_u32(p.table_entries)
        bsums = rs.empty_u32(max(1, p.scan_blocks))
        rs.pass_histogram(p, d, bit, table)
        torch.cuda.synchronize()
        assert np.array_equal(host(table), h_ref)
        rs.pass_scan(p, table, bsums)
        torch.cuda.synchronize()
        assert np.array_equal(host(table), s_ref)
        loc = rs.empty_u32(n)
        rs.pass_local_sort(p, d, loc, bit)
        out = rs.empty_u32(n)
        rs.pass_scatter(p, d, out, bit, table)
        torch.cuda.synchronize()
        assert np.array_equal(host(loc), loc_ref)
        assert np.array_equal(host(out), out_ref)


# ------------------------------------------------------------------ API semantics
@pytest.mark.parametrize("k", [8, 5, 4, 3])
def test_in_place(k):
    """in == out is allowed (odd pass counts stage through the workspace first)."""
    x = uniform_keys(123457, seed=k)
    d = dev(x)
    rs.sort_device(d, d, k)
    torch.cuda.synchronize()
    assert np.array_equal(host(d), np.sort(x))


def test_empty_and_tiny():
    lib = rs._lib()
    assert lib.rsort_u32_device(None, None, 0, 8, None, 0, None) == 0
    y = np.zeros(1, np.uint32)
    rs.sortByDevice(np.array([7], np.uint32), 1, y, 8)
    assert y[0] == 7


def test_workspace_too_small_is_reported():
    x = dev(uniform_keys(10000))
    out = rs.empty_u32(10000)
    ws = rs.workspace(1024)
    st = rs._lib().rsort_u32_device(x.data_ptr(), out.data_ptr(), 10000, 8, ws.data_ptr(), 1024,
                                    torch.cuda.current_stream().cuda_stream)
    assert st == 7


def test_host_entry_and_reference_dispatcher(golden, capsys):
    case = next(c for c in golden["sort_cases"] if c["name"] == "ref_debug_513_k4")
    x = np.array(case["input"], np.uint32)
    y = np.zeros_like(x)
    times = {}
    rs.sortByDevice(x, x.size, y, 4, 512, times=times)
    assert y.tolist() == case["output"]
    # k = 4: 8 scatter passes; one key-reading histogram (the next-digit counts carry the rest)
    assert times["scatter"]["launches"] == 8 and times["histogram"]["launches"] == 1
    z = np.zeros_like(x)
    rs.sort(x, x.size, z, rs.SORT_BY_DEVICE, 4, 512)
    out = capsys.readouterr().out
    assert "Radix Sort by device:" in out and "Time:" in out
    assert np.array_equal(z, y)


def test_vendor_comparator():
    x = uniform_keys(1 << 20, seed=5)
    y = np.zeros_like(x)
    rs.sortByThrust(x, x.size, y)
    assert np.array_equal(y, np.sort(x))


def test_generators_match_host_generators():
    n = (1 << 20) + 3
    d = rs.empty_u32(n)
    rs.gen_uniform(d, 0x5EED)
    torch.cuda.synchronize()
    assert np.array_equal(host(d), uniform_keys(n))
    cdf = dev(zipf_cdf_u32())
    rs.gen_zipf(d, cdf, 0x5EED)
    torch.cuda.synchronize()
    assert np.array_equal(host(d), zipf_keys(n))
    rs.gen_iota(d, 5)
    torch.cuda.synchronize()
    assert np.array_equal(host(d), (np.arange(n, dtype=np.uint64) + 5).astype(np.uint32))


def test_profile_counts_launches():
    x = dev(uniform_keys(1 << 20))
    out = rs.empty_u32(1 << 20)
    with rs.Profile() as prof:
        rs.sort_device(x, out, 8)
    t = prof.times
    assert t["scatter"]["launches"] == 4 and t["histogram"]["launches"] == 4 and t["scan"]["launches"] == 4
    assert t["scatter"]["ms"] > 0 and t["scatter"]["keys"] == 4 * (1 << 20)


# ------------------------------------------------------------------ multi-GPU building blocks
def test_top_histogram():
    x = zipf_keys(300001, seed=9)
    h = rs.empty_u32(1 << 12)
    rs.top_histogram(dev(x), 12, h)
    torch.cuda.synchronize()
    assert np.array_equal(host(h), np.bincount(x >> np.uint32(20), minlength=4096).astype(np.uint32))


@pytest.mark.parametrize("n,stride,bits", [(300001, 1, 12), (300001, 16, 12), (1 << 22, 16, 12),
                                            (1000, 7, 5), (0, 16, 12), (5 << 20, 3, 8)])
def test_top_histogram_sampled(n, stride, bits):
    """rsort_top_histogram_sampled = numpy's bincount over every stride-th 256-key block."""
    x = zipf_keys(n, seed=n + stride) if n else np.zeros(0, np.uint32)
    h = rs.empty_u32(1 << bits)
    rs.top_histogram_sampled(dev(x) if n else rs.empty_u32(0), bits, stride, h)
    torch.cuda.synchronize()
    sample = x[(np.arange(n) // 256) % stride == 0]
    assert np.array_equal(host(h), np.bincount(sample >> np.uint32(32 - bits), minlength=1 << bits).astype(np.uint32))


@pytest.mark.parametrize("nb", [1, 2, 3, 8, 16, 17, 32])
def test_partition_stable(nb):
    n = 200003
    x = zipf_keys(n, seed=nb)
    v = np.arange(n, dtype=np.uint32)
    split = np.sort(uniform_keys(nb - 1, seed=nb)) if nb > 1 else np.array([], np.uint32)
    bucket = np.searchsorted(split, x, side="right")
    order = np.argsort(bucket, kind="stable")
    ko, vo = rs.empty_u32(n), rs.empty_u32(n)
    starts = rs.empty_u32(nb + 1)
    rs.partition_device(dev(x), ko, split.tolist(), starts, vals_in=dev(v), vals_out=vo)
    torch.cuda.synchronize()
    assert np.array_equal(host(ko), x[order])
    assert np.array_equal(host(vo), v[order])
    exp = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nb))]).astype(np.uint32)
    assert np.array_equal(host(starts), exp)


def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize("nb,repeat", [(1, False), (2, False), (3, False), (4, True), (8, True), (15, True), (16, False),
                                       (31, True), (32, False)])
def test_partition_stable_large(nb, repeat):
    """keys-only partitions of n >= 2 x CUs x 8192 keys run the 512 x 16 line tiles with
    splitter digits (rsort_capi.cpp choose_geom). n = 2 x CUs x 8192 + odd, Zipf keys; with
    `repeat`, splitters in the equal-key-bucket shape of the multi-GPU sort (v, v + 1 pairs, v + 1
    equal to the next v, so some buckets are empty). Against numpy's stable argsort and the bucket
    starts."""
    n = 2 * _cus() * 8192 + 4099
    x = zipf_keys(n, seed=nb + 100)
    q = np.unique(x[:: max(1, n // 512)])
    rng = np.random.default_rng(nb)
    if repeat:
        vs = [int(v) for v in np.sort(rng.choice(q, size=nb // 2, replace=False))]
        vs[1] = vs[0] + 1  # splitters v0, v0 + 1, v0 + 1, v0 + 2: a repeated splitter, an empty bucket
        split = np.array(sorted(sum(([v, v + 1] for v in vs), []))[: nb - 1], np.uint64)
    else:
        split = np.sort(rng.choice(q, size=nb - 1, replace=False)).astype(np.uint64)
    split = np.minimum(split, 0xFFFFFFFF).astype(np.uint32)
    assert split.size == nb - 1 and np.all(split[1:] >= split[:-1])
    bucket = np.searchsorted(split, x, side="right")
    order = np.argsort(bucket, kind="stable")
    ko = rs.empty_u32(n)
    starts = rs.empty_u32(nb + 1)
    rs.partition_device(dev(x), ko, split.tolist(), starts)
    torch.cuda.synchronize()
    assert np.array_equal(host(ko), x[order])
    exp = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nb))]).astype(np.uint32)
    assert np.array_equal(host(starts), exp)


def _prefix_table_case(case, rng):
    """Splitters that stress the partition kernels' split digits (Digit: an 11-bit prefix table, then
    compares against the splitters inside the key's prefix range): every splitter inside one prefix,
    the extreme values, repeated splitters."""
    if case in ("one_prefix", "one_prefix31"):  # 15 (31) splitters, 16 (32) buckets, in one 2^21-key prefix
        base = 0x2A5 << 21
        m = 31 if case == "one_prefix31" else 15
        return np.sort(base + rng.choice(1 << 21, size=m, replace=False)).astype(np.uint32)
    if case == "many31":  # 32 buckets: 31 random splitters, 4 of them in one prefix
        v = rng.integers(0, 1 << 32, size=27, dtype=np.uint64).tolist() + [(0x123 << 21) + i for i in (0, 5, 9, 77)]
        return np.sort(np.array(v, np.uint64)).astype(np.uint32)
    if case == "edges":  # 0, 1, prefix boundaries and ~0u
        v = [0, 1, (1 << 21) - 1, 1 << 21, 0x7FFFFFFF, 0x80000000, 0xFFE00000, 0xFFFFFFFE, 0xFFFFFFFF]
        v += [int(x) for x in rng.integers(0, 1 << 32, size=6, dtype=np.uint64)]
        return np.sort(np.array(v, np.uint64)).astype(np.uint32)
    # repeated splitters, 8 buckets (empty ones between the repeats)
    s = int(rng.integers(1 << 20, 1 << 31))
    return np.array([s, s, s, s + 1, s + 1, s + (1 << 21), 0xFFFFFFFF], np.uint32)


@pytest.mark.parametrize("case", ["one_prefix", "one_prefix31", "many31", "edges", "dups"])
@pytest.mark.parametrize("size", ["small", "large", "pairs"])
def test_partition_prefix_table(case, size):
    """Partitions whose keys sit on and next to every splitter and every prefix boundary near one, in
    all three split-digit kernels (histogram, 4096-key and 8192-key line tiles; pairs), against numpy's
    stable argsort of searchsorted(side='right') buckets and the bucket starts."""
    rng = np.random.default_rng(len(case) * 7 + len(size))
    split = _prefix_table_case(case, rng)
    nb = split.size + 1
    n = 2 * _cus() * 8192 + 4099 if size == "large" else 150001
    near = []
    for s in split.astype(np.int64):
        p = (s >> 21) << 21
        near += [s - 1, s, s + 1, p - 1, p, p + (1 << 21) - 1, p + (1 << 21)]
    near = np.array([x for x in near if 0 <= x <= 0xFFFFFFFF], np.uint64).astype(np.uint32)
    x = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    pos = rng.choice(n, size=n // 2, replace=False)
    x[pos] = near[rng.integers(0, near.size, size=pos.size)]
    bucket = np.searchsorted(split, x, side="right")
    order = np.argsort(bucket, kind="stable")
    ko = rs.empty_u32(n)
    starts = rs.empty_u32(nb + 1)
    if size == "pairs":
        v = np.arange(n, dtype=np.uint32)
        vo = rs.empty_u32(n)
        rs.partition_device(dev(x), ko, split.tolist(), starts, vals_in=dev(v), vals_out=vo)
        torch.cuda.synchronize()
        assert np.array_equal(host(vo), v[order])
    else:
        rs.partition_device(dev(x), ko, split.tolist(), starts)
        torch.cuda.synchronize()
    assert np.array_equal(host(ko), x[order])
    exp = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nb))]).astype(np.uint32)
    assert np.array_equal(host(starts), exp)


def test_partition_fuzz():
    """60 random partitions (seeded): 1..32 buckets, splitters drawn uniformly, from a few prefixes or
    from the keys themselves (so some repeat), keys and pairs, small and 512 x 16-tile sizes -- every split
    digit path (compares, register counts, the prefix table with spans of 0..7+, the few-bucket ranking)
    against numpy's stable argsort of searchsorted(side='right') buckets."""
    rng = np.random.default_rng(20261018)
    big = 2 * _cus() * 8192 + 333
    for trial in range(60):
        nb = int(rng.integers(1, 33))
        n = int(rng.choice([1, 97, 4096 * 3 + 5, 65537, big]))
        mode = trial % 3
        x = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        if mode == 0:
            split = rng.integers(0, 1 << 32, size=nb - 1)
        elif mode == 1:  # splitters crowded into two 2^21-key prefixes, half the keys next to them
            p = rng.integers(0, 1 << 11, size=2) << 21
            split = p[rng.integers(0, 2, size=nb - 1)] + rng.integers(0, 1 << 21, size=nb - 1)
            if nb > 1:
                near = split[rng.integers(0, nb - 1, size=n // 2)] + rng.integers(-2, 3, size=n // 2)
                x[: n // 2] = np.clip(near, 0, 0xFFFFFFFF).astype(np.uint32)
        else:  # splitters are keys (repeats likely with a small key set)
            x = rng.choice((np.arange(40, dtype=np.int64) * 0x06000001) & 0xFFFFFFFF, size=n).astype(np.uint32)
            split = rng.choice(x, size=nb - 1).astype(np.int64)
        split = np.sort(np.clip(split, 0, 0xFFFFFFFF)).astype(np.uint32)
        bucket = np.searchsorted(split, x, side="right")
        order = np.argsort(bucket, kind="stable")
        pairs = trial % 4 == 1
        ko = rs.empty_u32(n)
        starts = rs.empty_u32(nb + 1)
        if pairs:
            v = np.arange(n, dtype=np.uint32)
            vo = rs.empty_u32(n)
            rs.partition_device(dev(x), ko, split.tolist(), starts, vals_in=dev(v), vals_out=vo)
        else:
            rs.partition_device(dev(x), ko, split.tolist(), starts)
        torch.cuda.synchronize()
        assert np.array_equal(host(ko), x[order]), (trial, nb, n, mode)
        if pairs:
            assert np.array_equal(host(vo), v[order]), (trial, nb, n, mode)
        exp = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nb))]).astype(np.uint32)
        assert np.array_equal(host(starts), exp), (trial, nb, n, mode)


def test_plan_check_and_kernels_used():
    """rsort_plan_check reports the tail scans' self-check (0 = every next-pass table summed to n)
    after k = 3, 4 sorts; rsort_scatter_kernels_used names what the dispatch launched."""
    rs.scatter_kernels_used(reset=True)
    for n, k in [((1 << 22) + 77, 4), ((1 << 21) - 3, 3)]:
        x = uniform_keys(n, seed=n)
        p = rs.plan(n, k)
        ws = rs.workspace(p.workspace_bytes)
        out = rs.empty_u32(n)
        rs.sort_device(dev(x), out, k, ws=ws, plan_=p)
        assert rs.plan_check(p, ws) == 0
        assert np.array_equal(host(out), oracle_sort(x, k))
    used = rs.scatter_kernels_used(reset=True)
    assert used and all(u.startswith("rs_scatter") for u in used), used
    assert any(u.startswith("rs_scatter_lines<4,") for u in used), used
    n = 1 << 24
    x = uniform_keys(n, seed=5)
    out = rs.empty_u32(n)
    rs.sort_device(dev(x), out, 8)
    torch.cuda.synchronize()
    used = rs.scatter_kernels_used()
    assert any(u.startswith("rs_scatter_lines<8, 1024, 16, 32, false") for u in used), used


# ------------------------------------------------------------------ reference harness (CLI)
@pytest.mark.parametrize("args", [["--debug"], [], ["512", "4"], ["256", "5", "--n", "1000003"]])
def test_reference_harness_cli(args):
    """tools/rsort_cli reproduces the reference main's flow and prints (Parallel7.cu:696-775):
    host, Thrust(rocPRIM) and device sorts of glibc rand() keys, each CORRECT."""
    import subprocess
    from pathlib import Path
    cli = Path(__file__).resolve().parent.parent / "tools" / "rsort_cli"
    r = subprocess.run([str(cli), *args, "--strict"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout
    assert out.count("CORRECT :)") == 2 and "INCORRECT" not in out
    for line in ("Radix Sort by host", "Radix Sort by Thrust library", "Radix Sort by device:", "Time: "):
        assert line in out
