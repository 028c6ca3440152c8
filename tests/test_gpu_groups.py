"""GPU parity of digit-group chunks (k = 8 plans with 256 chunks; rs_histogram_joint and
rsort_capi.cpp sort_planned): passes 1 and 3 take the previous pass's digit groups as chunks and
copy their histogram from the joint (digit, next digit) counts the pass before counted.
Where the groups are unbalanced, passes 1 and 3 take equal chunks cutting them (cut plans).
Bit-exact against the oracle (Baseline1.cu:15-64 restated) with the path on and off, and the
flags say how each odd pass took its chunks. Runs on the MI355X box (-m gpu)."""
import numpy as np
import pytest

from _rs import rs
from _util import oracle_sort, oracle_sort_pairs, uniform_keys, zipf_keys

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LINE_TILE = 16384      # kGeomLines tile (keys)
PAIRS_TILE = 8192      # kGeomLinesPairs tile


def group_plan(n, pairs=False):
    """Plan with exactly 256 chunks (tiles_per_chunk forced), the shape group chunks need (line
    tiles need n >= 512 tiles, so ragged sizes sit just under 768 or 1024 tiles)."""
    tile = PAIRS_TILE if pairs else LINE_TILE
    tiles = (n + tile - 1) // tile
    assert tiles % 256 == 0
    p = rs.plan(n, 8, pairs, tiles // 256)
    assert p.num_chunks == 256 and p.tile_keys == tile, p.as_dict()
    return p


_LAST_STATS = [None]  # run(): the last sort's rsort_cut_plan_stats


def run(x, p, vals=None, groups=True):
    with rs.group_chunks(groups):
        d_in = rs.from_numpy_u32(x)
        d_out = rs.empty_u32(x.size)
        ws = rs.workspace(p.workspace_bytes)
        if vals is None:
            rs.sort_device(d_in, d_out, 8, ws=ws, plan_=p)
            flags = rs.group_flags(p, ws)
            _LAST_STATS[0] = rs.cut_plan_stats(p, ws)
            assert np.array_equal(rs.to_numpy_u32(d_in), x), "input buffer was modified"
            return rs.to_numpy_u32(d_out), flags
        v_in = rs.from_numpy_u32(vals)
        v_out = rs.empty_u32(x.size)
        rs.sort_device(d_in, d_out, 8, vals_in=v_in, vals_out=v_out, ws=ws, plan_=p)
        flags = rs.group_flags(p, ws)
        _LAST_STATS[0] = rs.cut_plan_stats(p, ws)
        return (rs.to_numpy_u32(d_out), rs.to_numpy_u32(v_out)), flags


@pytest.mark.parametrize("n", [512 * LINE_TILE, 768 * LINE_TILE - 5, 767 * LINE_TILE + 1, 1024 * LINE_TILE - 77])
def test_uniform_keys_on_groups(n):
    x = uniform_keys(n, seed=n)
    want = oracle_sort(x, 8)
    y, flags = run(x, group_plan(n))
    assert flags == [1, 1]
    assert np.array_equal(y, want)
    y0, flags0 = run(x, group_plan(n), groups=False)
    assert flags0 == [0, 0]
    assert np.array_equal(y0, want)


def test_zipf_keys_cut_plan():
    """Zipf digit groups are far from balanced: pass 1 takes equal chunks that cut the big groups
    (kGroupsCut) and counts only the cut groups' pieces; pass 2 counts the (digit 2, digit 3) joint
    counts on its clustered input (runs of equal pairs added once), so pass 3 takes a cut plan of
    its own and counts only its pieces too."""
    n = 768 * LINE_TILE - 3
    x = zipf_keys(n, seed=7)
    y, flags = run(x, group_plan(n))
    assert flags == [2, 2]
    assert np.array_equal(y, oracle_sort(x, 8))
    y0, flags0 = run(x, group_plan(n), groups=False)
    assert flags0 == [0, 0]
    assert np.array_equal(y0, y)


def _cut_input(kind, n, seed):
    rng = np.random.default_rng(seed)
    x = uniform_keys(n, seed=seed)
    if kind == "one_group":
        # every key has digits 0 and 2 = 0x5A: passes 1 and 3 see one group of n keys (255 pieces)
        return ((x & np.uint32(0xFF00FF00)) | np.uint32(0x005A005A)).astype(np.uint32)
    if kind == "half_hot":
        # half the keys have digit 0 = 7 (a group of ~128 chunks), the rest spread: small groups
        # of half a chunk, boundaries cutting them
        m = rng.random(n) < 0.5
        x[m] = (x[m] & np.uint32(0xFFFFFF00)) | np.uint32(7)
        return x
    if kind == "two_chunk_groups":
        # digit 0 in 0..127 only, equally often: groups of ~2 chunks, every second boundary inside
        # one (two equal segments: the tie picks the derived one by slot)
        d0 = (np.arange(n, dtype=np.uint64) * 128 // n).astype(np.uint32)
        rng.shuffle(d0)
        return ((x & np.uint32(0xFFFFFF00)) | d0).astype(np.uint32)
    assert kind == "steps"
    # group sizes 1, 2, 4, ... keys up to whole chunks and past them, plus empty groups
    sizes = np.zeros(256, np.int64)
    sizes[::3] = np.minimum(2 ** (np.arange(0, 256, 3) % 24), n)
    sizes = (sizes * (n / sizes.sum())).astype(np.int64)
    sizes[0] += n - sizes.sum()
    d0 = np.repeat(np.arange(256, dtype=np.uint32), sizes)
    rng.shuffle(d0)
    return ((x & np.uint32(0xFFFFFF00)) | d0).astype(np.uint32)


@pytest.mark.parametrize("kind", ["one_group", "half_hot", "two_chunk_groups", "steps"])
@pytest.mark.parametrize("n", [512 * LINE_TILE, 768 * LINE_TILE - 13])
def test_cut_plan_shapes(kind, n):
    """Cut plans (rs_joint_bounds kGroupsCut, pieces counted by rs_histogram, table assembled by
    rs_scan_reduce's cut_entry) on group shapes that hit every case: chunks inside one group,
    chunks spanning many small groups, boundaries snapped onto group boundaries, equal segments,
    empty groups. Bit-exact against the oracle."""
    x = _cut_input(kind, n, seed=n % 1000 + len(kind))
    y, flags = run(x, group_plan(n))
    assert flags[0] == 2
    assert np.array_equal(y, oracle_sort(x, 8))


@pytest.mark.parametrize("seed", range(6))
def test_cut_plan_random_shapes(seed):
    """Random group shapes for pass 1 (digit 0) and pass 3 (digit 2): Dirichlet group sizes with
    a few heavy groups, empty groups, ragged n. Bit-exact against the oracle."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.choice([768, 1024])) * LINE_TILE - int(rng.integers(0, 4096))
    x = uniform_keys(n, seed=200 + seed)
    for shift in (0, 16):
        w = rng.dirichlet(np.full(256, rng.choice([0.05, 0.3, 1.0])))
        w[rng.integers(0, 256, int(rng.integers(0, 4)))] += rng.uniform(0.01, 0.3)
        d = rng.choice(256, size=n, p=w / w.sum()).astype(np.uint32)
        x = ((x & ~np.uint32(0xFF << shift)) | (d << np.uint32(shift))).astype(np.uint32)
    y, flags = run(x, group_plan(n))
    assert flags[0] in (1, 2)
    assert np.array_equal(y, oracle_sort(x, 8))


@pytest.mark.parametrize("kind", ["half_hot", "one_group"])
def test_cut_plan_pairs(kind):
    n = 768 * PAIRS_TILE - 5
    x = _cut_input(kind, n, seed=41)
    v = np.arange(n, dtype=np.uint32)
    (ko, vo), flags = run(x, group_plan(n, pairs=True), vals=v)
    assert flags[0] == 2
    wk, wv = oracle_sort_pairs(x, v, 8)
    assert np.array_equal(ko, wk) and np.array_equal(vo, wv)


def test_joint_counter_spill():
    """Chunk c holds only digit pair (c, 0) (32768 or 65536 equal pairs per workgroup): the 16-bit
    joint counters pass 2^15 and spill, and the groups are exactly the chunks (balanced)."""
    for tiles in (512, 1024):
        n = tiles * LINE_TILE
        rng = np.random.default_rng(tiles)
        chunk = n // 256
        c = (np.arange(n, dtype=np.uint64) // chunk).astype(np.uint32)
        hi = rng.integers(0, 1 << 16, n, dtype=np.uint32)
        x = (c | (hi << 16)).astype(np.uint32)
        y, flags = run(x, group_plan(n))
        assert flags[0] == 1
        assert np.array_equal(y, oracle_sort(x, 8))


def test_cut_plan_rows_with_spills():
    """A cut plan whose pieces come from the per-chunk joint-count rows (HistArgs::rows) while the
    chunks. 16-bit joint counters spill: 60 % of the keys share digits 0 and 1 (>= 2^15 equal pairs per
    workgroup: the rows take the spilled 2^15s on top), the rest uniform. Bit-exact against the oracle,
    keys and pairs."""
    for tiles, pairs in ((1024, False), (2048, True)):
        n = tiles * (PAIRS_TILE if pairs else LINE_TILE) - 7
        rng = np.random.default_rng(tiles)
        x = uniform_keys(n, seed=tiles)
        hot = rng.random(n) < 0.6
        x[hot] = (x[hot] & np.uint32(0xFFFF0000)) | np.uint32(0x1234)
        if pairs:
            v = np.arange(n, dtype=np.uint32)
            (ko, vo), flags = run(x, group_plan(n, pairs=True), vals=v)
            wk, wv = oracle_sort_pairs(x, v, 8)
            assert np.array_equal(ko, wk) and np.array_equal(vo, wv)
        else:
            y, flags = run(x, group_plan(n))
            assert np.array_equal(y, oracle_sort(x, 8))
        assert flags[0] == 2
        # the pieces really came from the rows (a fallback to counting them from the keys would
        # pass the checks above too): pass 1's cut plan summed rows
        st = _LAST_STATS[0]
        assert st[0]["row_tasks"] > 0, st


@pytest.mark.parametrize("pairs", [False, True])
def test_cut_plan_rows_hot_key_runs(pairs):
    """40 % of the keys one value, the rest uniform: both odd passes cut (the hot key's digit 0 and
    digit 2 groups). Pass 3's pieces end inside previous chunks that hold nothing but the hot key's
    copies (one next digit: direct adds, no key read) and pass 1's inside mixed ones (key ranges, or
    their complements counted negatively). Bit-exact against the oracle."""
    n = 768 * (PAIRS_TILE if pairs else LINE_TILE) - 3
    rng = np.random.default_rng(77)
    x = uniform_keys(n, seed=77)
    x[rng.random(n) < 0.4] = np.uint32(0x9E3779B9)
    if pairs:
        v = np.arange(n, dtype=np.uint32)
        (ko, vo), flags = run(x, group_plan(n, pairs=True), vals=v)
        wk, wv = oracle_sort_pairs(x, v, 8)
        assert np.array_equal(ko, wk) and np.array_equal(vo, wv)
    else:
        y, flags = run(x, group_plan(n))
        assert np.array_equal(y, oracle_sort(x, 8))
    assert list(flags) == [2, 2]
    # every piece kind was emitted -- row tasks, direct adds (pass 3: chunks of nothing but the
    # hot key's copies) and ranges counted negatively -- not a silent fallback to counting from the keys
    st = _LAST_STATS[0]
    print("cut plan stats", st)
    assert st[0]["row_tasks"] > 0 and st[1]["row_tasks"] > 0, st
    assert st[1]["direct_adds"] > 0, st
    assert st[0]["negative_ranges"] + st[1]["negative_ranges"] > 0, st


def test_empty_groups():
    """64 of the 256 digit-0 values never occur; the other groups still fit one tile over a chunk."""
    n = 512 * LINE_TILE
    rng = np.random.default_rng(5)
    x = uniform_keys(n, seed=5)
    d0 = rng.integers(0, 192, n, dtype=np.uint32)
    d0 = d0 + d0 // 3  # skip every 4th value
    x = ((x & np.uint32(0xFFFFFF00)) | d0).astype(np.uint32)
    y, flags = run(x, group_plan(n))
    assert flags[0] == 1
    assert np.array_equal(y, oracle_sort(x, 8))


def test_pass1_balanced_pass3_not():
    """Uniform low 16 bits, constant digit 2: pass 1 runs on groups, pass 3 cuts the one group."""
    n = 768 * LINE_TILE - 1
    x = (uniform_keys(n, seed=9) & np.uint32(0xFF00FFFF)) | np.uint32(0x00AB0000)
    y, flags = run(x, group_plan(n))
    assert flags == [1, 2]
    assert np.array_equal(y, oracle_sort(x, 8))


@pytest.mark.parametrize("kind", ["equal", "runs"])
def test_joint_count_clustered(kind):
    """Pass 0's joint count on clustered input (rs_histogram JOINT, run path: a run of lanes holding
    one pair adds once): all-equal keys (every batch takes the run path; the 16-bit counters spill in
    steps of up to 64) and runs of 1..300 equal keys (batches of both kinds in one workgroup)."""
    n = 768 * LINE_TILE - 7
    rng = np.random.default_rng(23)
    if kind == "equal":
        x = np.full(n, 0x89ABCDEF, dtype=np.uint32)
    else:
        lens = rng.integers(1, 301, n // 100 + 2)
        vals = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
        x = np.repeat(vals, lens)[:n].copy()
    y, _ = run(x, group_plan(n))
    assert np.array_equal(y, oracle_sort(x, 8))


@pytest.mark.parametrize("kind", ["equal", "hot_runs", "zipf"])
def test_joint_count_after_cut_pass(kind):
    """Pass 2's joint count after a cut pass 1 (rs_histogram JOINT on clustered input) at 2^25 - 12345
    keys, 256 chunks of ~131K keys: a pair's count in one chunk runs to 2^17 (all-equal keys: the
    16-bit counters spill four times), runs of one pair mix with plain batches (hot runs), and the C4
    key distribution."""
    n = 2048 * LINE_TILE - 12345
    rng = np.random.default_rng(41)
    if kind == "equal":
        x = np.full(n, 0x0BADF00D, dtype=np.uint32)
        x[rng.integers(0, n, 1000)] = rng.integers(0, 1 << 32, 1000, dtype=np.uint64).astype(np.uint32)
    elif kind == "hot_runs":
        x = uniform_keys(n, seed=41)
        x[rng.random(n) < 0.3] = np.uint32(0xC0FFEE11)  # one group of ~30 % of the keys: a cut plan
        lens = rng.integers(1, 2000, n // 1000 + 2)
        vals = rng.integers(0, 1 << 16, lens.size, dtype=np.uint64).astype(np.uint32) << np.uint32(16)
        hi = np.repeat(vals, lens)[:n]
        m = rng.random(n) < 0.5
        x[m] = (x[m] & np.uint32(0xFFFF)) | hi[m]  # long runs of one (digit 2, digit 3) pair
    else:
        x = zipf_keys(n, seed=41)
    y, flags = run(x, group_plan(n))
    assert flags[0] == 2
    assert np.array_equal(y, oracle_sort(x, 8))


@pytest.mark.parametrize("pairs", [False, True])
def test_clustered_kernels(pairs):
    """Unbalanced groups select the clustered-input kernels (rank_add_hot) for passes 1..3. Input
    built to exercise both aggregation candidates: blocks where one hot key holds 40-95 % of the
    positions (the first lane of a slot often holds another key, the wave's last aggregated digit
    is then the candidate), hot keys that change between blocks, and background keys."""
    tile = PAIRS_TILE if pairs else LINE_TILE
    n = 768 * tile - 11
    rng = np.random.default_rng(17)
    x = uniform_keys(n, seed=17)
    hot = rng.integers(0, 1 << 32, 64, dtype=np.uint64).astype(np.uint32)
    blk = 3000
    for b in range(0, n, blk):
        h = hot[rng.integers(0, 64)]
        dens = rng.uniform(0.4, 0.95)
        m = rng.random(min(blk, n - b)) < dens
        x[b:b + m.size][m] = h
    # one heavy key overall: the digit groups are unbalanced, so the clustered kernels run
    x[rng.random(n) < 0.1] = hot[0]
    v = np.arange(n, dtype=np.uint32) if pairs else None
    out, flags = run(x, group_plan(n, pairs=pairs), vals=v)
    assert flags[0] == 2 and flags[1] in (1, 2)
    if pairs:
        wk, wv = oracle_sort_pairs(x, v, 8)
        assert np.array_equal(out[0], wk) and np.array_equal(out[1], wv)
    else:
        assert np.array_equal(out, oracle_sort(x, 8))


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_pairs_on_groups(dist):
    n = 768 * PAIRS_TILE - 9
    x = uniform_keys(n, seed=3) if dist == "uniform" else zipf_keys(n, seed=3)
    v = np.arange(n, dtype=np.uint32)
    (ko, vo), flags = run(x, group_plan(n, pairs=True), vals=v)
    assert flags == ([1, 1] if dist == "uniform" else [2, 2])
    wk, wv = oracle_sort_pairs(x, v, 8)
    assert np.array_equal(ko, wk) and np.array_equal(vo, wv)


def test_default_plan_2p27():
    """The default plan at 2^27 keys (256 chunks on a 256-CU MI355X) takes the group path."""
    n = 1 << 27
    p = rs.plan(n, 8)
    if p.num_chunks != 256:
        pytest.skip(f"{p.num_chunks} chunks on this device")
    d_in = rs.empty_u32(n)
    rs.gen_uniform(d_in, 0x5EED)
    d_out = rs.empty_u32(n)
    ws = rs.workspace(p.workspace_bytes)
    rs.sort_device(d_in, d_out, 8, ws=ws, plan_=p)
    assert rs.group_flags(p, ws) == [1, 1]
    ref, _ = torch.sort(d_in.to(torch.int64) & 0xFFFFFFFF)
    got = d_out.to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(got, ref)


def test_in_place_on_groups():
    """in == out (P = 4: pass 0 reads the caller's buffer, the ping-pong ends in it)."""
    n = 768 * LINE_TILE - 11
    x = uniform_keys(n, seed=11)
    p = group_plan(n)
    d = rs.from_numpy_u32(x)
    ws = rs.workspace(p.workspace_bytes)
    rs.sort_device(d, d, 8, ws=ws, plan_=p)
    assert rs.group_flags(p, ws) == [1, 1]
    assert np.array_equal(rs.to_numpy_u32(d), oracle_sort(x, 8))


def test_unaligned_output_keeps_groups():
    """An output buffer that is 4-B but not 16-B aligned still takes the whole-line kernels (positions
    from its 128-B-aligned base): digit groups on both odd passes."""
    n = 512 * LINE_TILE
    x = uniform_keys(n, seed=12)
    p = group_plan(n)
    d_in = rs.from_numpy_u32(x)
    big = rs.empty_u32(n + 1)
    d_out = big[1:]
    ws = rs.workspace(p.workspace_bytes)
    rs.sort_device(d_in, d_out, 8, ws=ws, plan_=p)
    assert rs.group_flags(p, ws) == [1, 1]
    assert np.array_equal(rs.to_numpy_u32(d_out), oracle_sort(x, 8))


def test_pairs_mismatched_alignment_falls_back():
    """Pairs whose values sit at other than a multiple of 16 B from the keys cannot take the
    whole-line kernels: fixed chunks, the same result."""
    n = 512 * LINE_TILE
    x = zipf_keys(n, seed=13)
    v = np.arange(n, dtype=np.uint32)
    p = rs.plan(n, 8, True)
    ws = rs.workspace(p.workspace_bytes)
    bigv = rs.empty_u32(n + 1)
    ko, vo = rs.empty_u32(n), bigv[1:]
    rs.sort_device(rs.from_numpy_u32(x), ko, 8, vals_in=rs.from_numpy_u32(v), vals_out=vo, ws=ws, plan_=p)
    assert rs.group_flags(p, ws) == [0, 0]
    rk, rv = oracle_sort_pairs(x, v, 8)
    assert np.array_equal(rs.to_numpy_u32(ko), rk) and np.array_equal(rs.to_numpy_u32(vo), rv)


# ------------------------------------------------------------------ next-digit counts (k = 3, 4)
def _keys(dist, n, seed):
    if dist == "uniform":
        return uniform_keys(n, seed=seed)
    if dist == "zipf":
        return zipf_keys(n, seed=seed)
    if dist == "allsame":
        return np.full(n, 0x9E3779B9, np.uint32)
    if dist == "sorted":
        return np.sort(uniform_keys(n, seed=seed))
    if dist == "reversed":
        return np.sort(uniform_keys(n, seed=seed))[::-1].copy()
    return uniform_keys(n, seed=seed) & np.uint32(0x0F0F00FF)  # "sparse": many empty digits


@pytest.mark.parametrize("k", [3, 4])
@pytest.mark.parametrize("dist", ["uniform", "zipf", "allsame", "sorted", "reversed", "sparse"])
@pytest.mark.parametrize("n", [4096 * 40 + 3, (1 << 21) + 517])
def test_next_digit_counts(k, dist, n):
    """k = 3, 4 keys-only plans: every pass adds the next pass's chunk table from where it writes
    each key (rs_scatter_lines, a.next_table), so passes 1.. read no keys for their histogram --
    bit-exact against the oracle with the path on and off, on balanced and extreme inputs (one
    digit holding a whole chunk spans two of the next pass's chunks)."""
    x = _keys(dist, n, n + k)
    want = oracle_sort(x, k)
    for on in (True, False):
        with rs.group_chunks(on):
            d_in = rs.from_numpy_u32(x)
            d_out = rs.empty_u32(n)
            rs.sort_device(d_in, d_out, k)
            assert np.array_equal(rs.to_numpy_u32(d_out), want), (k, dist, n, on)


@pytest.mark.parametrize("tpc", [1, 3, 17])
def test_next_digit_counts_chunk_geometries(tpc):
    """Small chunks (one tile per chunk and up): digit ranges cross the next pass's chunk
    boundaries in every tile."""
    n = 4096 * 97 + 11
    x = zipf_keys(n, seed=tpc)
    p = rs.plan(n, 4, False, tpc)
    d_out = rs.empty_u32(n)
    rs.sort_device(rs.from_numpy_u32(x), d_out, 4, plan_=p)
    assert np.array_equal(rs.to_numpy_u32(d_out), oracle_sort(x, 4))


# ------------------------------------------------------------------ raw tables vs tail scans
@pytest.mark.parametrize("n,tpc,want_raw", [((1 << 22) + 9, 1, True), ((1 << 23) + 9, 1, False), ((1 << 24) + 5, 2, False),
                                            ((1 << 26), 0, True)])
def test_raw_tables_only_for_small_chunk_counts(n, tpc, want_raw):
    """Raw next-digit tables make every workgroup read the whole R x C table (O(R C^2) per pass), so a
    plan takes them only up to 1280 chunks; a small tiles_per_chunk (2^23 keys in 4096-key chunks:
    2049 chunks) keeps the tail scan. rsort_plan_features says which ran; the output is the oracle's
    either way, and the sort's self-check is clean."""
    p = rs.plan(n, 4, False, tpc)
    f = rs.plan_features(p)
    assert f & rs.FEAT_NEXT_DIGIT, f
    assert bool(f & rs.FEAT_RAW_TABLES) == want_raw and bool(f & rs.FEAT_TAIL_SCAN) == (not want_raw), (p.num_chunks, f)
    assert (p.num_chunks <= 1280) == want_raw
    x = uniform_keys(n, seed=n ^ tpc)
    ws = rs.workspace(p.workspace_bytes)
    d_out = rs.empty_u32(n)
    rs.sort_device(rs.from_numpy_u32(x), d_out, 4, ws=ws, plan_=p)
    assert rs.plan_check(p, ws) == 0
    got = rs.to_numpy_u32(d_out)
    if n <= (1 << 24) + 5:
        assert np.array_equal(got, oracle_sort(x, 4))
    else:
        assert np.array_equal(got, np.sort(x))


def test_plan_features_of_the_default_plans():
    assert rs.plan_features(rs.plan(1 << 30, 8)) == rs.FEAT_GROUPS
    assert rs.plan_features(rs.plan(1 << 26, 4)) == rs.FEAT_NEXT_DIGIT | rs.FEAT_RAW_TABLES
    assert rs.plan_features(rs.plan(1 << 20, 11)) == 0
    with rs.group_chunks(False):
        assert rs.plan_features(rs.plan(1 << 26, 4)) == 0


@pytest.mark.parametrize("k", [3, 4])
def test_corrupted_raw_table_is_reported(k):
    """the raw-table failure path. With the test hook one word of the table pass 1 reads
    is corrupted: that pass's workgroups see a total that is not n, write nothing and record it, so
    rsort_plan_check reports bit 0 (device entry) and the host entry returns RSORT_ERR_CHECK (11).
    The hook cleared, the same sorts are correct again."""
    n = (1 << 20) + 33
    x = uniform_keys(n, seed=k)
    p = rs.plan(n, k)
    assert rs.plan_features(p) & rs.FEAT_RAW_TABLES
    ws = rs.workspace(p.workspace_bytes)
    d_out = rs.empty_u32(n)
    with rs.table_fault():
        rs.sort_device(rs.from_numpy_u32(x), d_out, k, ws=ws, plan_=p)
        assert rs.plan_check(p, ws) == 1
        with pytest.raises(rs.RSortError) as e:
            rs.sortByDevice(x, n, np.empty_like(x), k)
        assert e.value.status == 11
    rs.sort_device(rs.from_numpy_u32(x), d_out, k, ws=ws, plan_=p)
    assert rs.plan_check(p, ws) == 0
    want = oracle_sort(x, k)
    assert np.array_equal(rs.to_numpy_u32(d_out), want)
    y = np.empty_like(x)
    rs.sortByDevice(x, n, y, k)
    assert np.array_equal(y, want)


_LAB_SNIPPET = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import radixsort as rs
from _util import oracle_sort, uniform_keys, zipf_keys
out = []
for k, gen, n in ((3, uniform_keys, (1 << 21) + 3), (4, zipf_keys, (1 << 21) + 7), (8, zipf_keys, 1 << 24)):
    x = gen(n, seed=k)
    p = rs.plan(n, k)
    ws = rs.workspace(p.workspace_bytes)
    d = rs.empty_u32(n)
    rs.sort_device(rs.from_numpy_u32(x), d, k, ws=ws, plan_=p)
    ok = np.array_equal(rs.to_numpy_u32(d), oracle_sort(x, k)) and rs.plan_check(p, ws) == 0
    flags = ",".join(map(str, rs.group_flags(p, ws))) if k == 8 else ""
    out.append(f"k{k}:{int(ok)}:{rs.plan_features(p)}:{flags}")
print("LAB " + " ".join(out))
'''


@pytest.mark.parametrize("env,feat4", [({"RSORT_LAB": "1", "RSORT_NX_TAIL": "1", "RSORT_CUT_WEIGHTS": "0"}, 2 | 8),
                                       ({"RSORT_NX_TAIL": "1", "RSORT_CUT_WEIGHTS": "0"}, 2 | 4),
                                       ({"RSORT_LAB": "1", "RSORT_PIECE_ROWS": "0"}, 2 | 4)])
def test_lab_switches_in_a_subprocess(env, feat4):
    """The A/B switches are read once per process, and only under RSORT_LAB=1: with
    it, k = 3, 4 sorts take the tail scans (features) and the Zipf k = 8 sort equal-count cut plans
    (or, RSORT_PIECE_ROWS=0, cut plans whose pieces are all counted from the keys); without it the
    same variables change nothing. All sort correctly."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    e = dict(os.environ)
    e.pop("RSORT_LAB", None)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _LAB_SNIPPET, str(root / "cuda.radixsort_amd"), str(root / "tests")],
                       capture_output=True, text=True, timeout=240, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("LAB ")]
    assert line, r.stdout[-2000:]
    parts = line[-1].split()[1:]
    assert [x.split(":")[1] for x in parts] == ["1", "1", "1"], r.stdout
    assert parts[0].split(":")[2] == str(feat4) and parts[1].split(":")[2] == str(feat4), r.stdout
    assert parts[2].split(":")[3] == "2,2", r.stdout  # Zipf keys: cut plans on passes 1 and 3
