"""Per-workgroup durations of a sort's scatter passes (dev/var_wgt.so: the library built with
-DRSORT_WG_TIMES, copied over cuda.radixsort_amd/librsort.so on the box first) and, for the pass
given, what the slowest and fastest chunks hold. Backs DESIGN §8 round 4 item 4 (Zipf pass 1).

    python dev/wgtimes_lab.py [--dist zipf] [--log2n 29] [--pass 1] [--pairs]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import radixsort as rs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dist", default="zipf")
ap.add_argument("--log2n", type=int, default=29)
ap.add_argument("--pass", dest="pss", type=int, default=1)
ap.add_argument("--pairs", action="store_true")
ap.add_argument("--k", type=int, default=8, help="digit bits (k = 4: C2's eight passes; no chunk contents)")
ap.add_argument("--dump", default="", help="write every chunk of the pass as CSV (us, keys, top digit share, H)")
ap.add_argument("--hist", action="store_true",
                help="also the joint-count histograms (passes 0 and 2) and what the slowest pass-2 chunks hold")
ap.add_argument("--reps", type=int, default=0,
                help="rate correlation over this many more sorts: by XCC, by physical CU, by chunk (VERDICT r4 #3)")
ap.add_argument("--hxcc", type=int, default=0,
                help="the joint-count histograms' workgroup durations by XCC over this many sorts (then exit)")
a = ap.parse_args()
n = 1 << a.log2n
lib = rs._lib()
fn = lib.rsort_lab_wg_times
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
keys = rs.empty_u32(n)
if a.dist == "zipf":
    from _util import zipf_cdf_u32
    rs.gen_zipf(keys, rs.from_numpy_u32(zipf_cdf_u32()), 0x5EED)
else:
    rs.gen_uniform(keys, 0x5EED)
vals = None
if a.pairs:
    vals = rs.empty_u32(n)
    rs.gen_iota(vals, 0)
out = rs.empty_u32(n)
vout = rs.empty_u32(n) if a.pairs else None
p = rs.plan(n, a.k, a.pairs)
ws = rs.workspace(p.workspace_bytes)
for _ in range(3):
    rs.sort_device(keys, out, a.k, vals_in=vals, vals_out=vout, ws=ws, plan_=p)
torch.cuda.synchronize()
nch = min(p.num_chunks, 2048)


def records():
    """(scatter records [pass, chunk, {t0, t1, beg, end}], histogram records, where [pass, chunk, {xcc,
    se, sh, cu}]) of the last sort; the lab build packs HW_ID / XCC_ID over the range words."""
    both = np.zeros(8 * 2048 * 4 + 4 * 256 * 4, dtype=np.uint64)
    assert fn(both.ctypes.data) == 0
    b = both[: 8 * 2048 * 4].reshape(8, 2048, 4)[:, :nch].copy()
    hb = both[8 * 2048 * 4:].reshape(4, 256, 4).copy()
    hw = (b[:, :, 2] >> np.uint64(32)).astype(np.int64)
    where = np.stack([(b[:, :, 3] >> np.uint64(32)).astype(np.int64) & 15, (hw >> 13) & 7, (hw >> 12) & 1,
                      (hw >> 8) & 15], axis=-1)
    for x in (b, hb):
        x[:, :, 2] &= np.uint64(0xFFFFFFFF)
        x[:, :, 3] &= np.uint64(0xFFFFFFFF)
    return b, hb, where


def rate_correlation(reps):
    """is a workgroup's rate (us per Mkey) a property of where it runs (XCC, CU) or of
    its chunk (address / index)? `reps` more sorts; per pass the rate's spread by XCC, and across sorts the
    correlation of the rate per physical CU and per chunk index."""
    rows = []  # (sort, pass, chunk, xcc, cu_uid, rate, dur, end offset)
    for r in range(reps):
        rs.sort_device(keys, out, a.k, vals_in=vals, vals_out=vout, ws=ws, plan_=p)
        torch.cuda.synchronize()
        b, _, where = records()
        for ps in range(p.passes):
            t0, t1, cb, ce = (b[ps, :, i].astype(np.int64) for i in range(4))
            dur = (t1 - t0) * 10 / 1e3
            rate = dur / np.maximum(1, ce - cb) * 1e6
            uid = ((where[ps, :, 0] * 8 + where[ps, :, 1]) * 2 + where[ps, :, 2]) * 16 + where[ps, :, 3]
            for c in range(nch):
                rows.append((r, ps, c, where[ps, c, 0], uid[c], rate[c], dur[c], (t1[c] - t1.min()) * 10 / 1e3))
    R = np.array(rows, dtype=np.float64)
    print(f"\nrate correlation: {reps} sorts x {p.passes} passes x {nch} chunks")
    for ps in range(p.passes):
        m = R[:, 1] == ps
        xr = [R[m & (R[:, 3] == x), 5] for x in range(8)]
        print(f"  pass {ps}: us/Mkey by XCC (mean over sorts):", " ".join(f"{x.mean():6.1f}" if x.size else "  -  "
                                                                         for x in xr),
              f" | overall sd {R[m, 5].std():.1f}, between-XCC sd {np.std([x.mean() for x in xr if x.size]):.1f}")
    # the same physical CU across sorts (pass means): does a slow CU stay slow?
    by_uid = {}
    for r in range(reps):
        m = R[:, 0] == r
        for u in np.unique(R[m, 4]):
            mm = m & (R[:, 4] == u)
            by_uid.setdefault(int(u), [np.nan] * reps)[r] = R[mm, 5].mean()
    M = np.array([v for v in by_uid.values() if not np.isnan(v).any()])
    if M.shape[0] > 2 and reps >= 2:
        cc = [np.corrcoef(M[:, i], M[:, j])[0, 1] for i in range(reps) for j in range(i + 1, reps)]
        print(f"  per physical CU ({M.shape[0]} CUs seen in every sort): rate correlation across sorts "
              f"min/mean/max {min(cc):.2f} {np.mean(cc):.2f} {max(cc):.2f}; CU mean rate sd {M.mean(axis=1).std():.1f} "
              f"us/Mkey, within-CU sd across sorts {M.std(axis=1).mean():.1f}")
    # the same chunk index across sorts, per pass
    for ps in range(p.passes):
        C = np.array([R[(R[:, 0] == r) & (R[:, 1] == ps), 5] for r in range(reps)])
        if reps >= 2:
            cc = [np.corrcoef(C[i], C[j])[0, 1] for i in range(reps) for j in range(i + 1, reps)]
            same_cu = np.mean([np.mean(R[(R[:, 0] == i) & (R[:, 1] == ps), 4] == R[(R[:, 0] == j) & (R[:, 1] == ps), 4])
                               for i in range(reps) for j in range(i + 1, reps)])
            print(f"  pass {ps}: per chunk index, rate correlation across sorts mean {np.mean(cc):.2f} "
                  f"(chunk on the same CU in {same_cu:.0%} of sort pairs); rate vs chunk index r "
                  f"{np.corrcoef(np.arange(nch), C.mean(axis=0))[0, 1]:.2f}")
    # several workgroups per CU (C2: 4): the k-th workgroup of a CU in blockIdx order (its dispatch
    # slot) -- an older wave wins the CU's arbitration, so equal chunks may end in slot order
    for ps in range(min(p.passes, 3)):
        m = (R[:, 1] == ps)
        slot = np.zeros(m.sum(), np.int64)
        sub = R[m]
        for r in range(reps):
            mr = sub[:, 0] == r
            idx = np.flatnonzero(mr)
            for u in np.unique(sub[mr, 4]):
                iu = idx[sub[idx, 4] == u]
                iu = iu[np.argsort(sub[iu, 2])]
                slot[iu] = np.arange(iu.size)
        per = [sub[slot == k] for k in range(slot.max() + 1)]
        print(f"  pass {ps}: by slot on its CU (k-th workgroup of the CU by blockIdx): " +
              "  ".join(f"slot {k}: {x[:, 5].mean():7.1f} us/Mkey, dur {x[:, 6].mean():6.1f} us, "
                        f"ends {x[:, 7].mean():5.1f} us before the last" if False else
                        f"slot {k}: {x[:, 5].mean():7.1f} us/Mkey dur {x[:, 6].mean():6.1f} us"
                        for k, x in enumerate(per) if x.size))
        blk = [sub[(sub[:, 2] // max(1, nch // 4)) == q, 5].mean() for q in range(4)]
        print(f"           by blockIdx quarter: " + " ".join(f"{b:7.1f}" for b in blk))
    m = R[:, 1] >= 0
    print(f"  every pass: rate vs XCC (eta^2) {eta2(R[m, 5], R[m, 3]):.3f}, vs physical CU {eta2(R[m, 5], R[m, 4]):.3f}, "
          f"vs chunk index {eta2(R[m, 5], R[m, 2]):.3f}")


def eta2(y, g):
    """share of y's variance explained by the group labels g"""
    tot = ((y - y.mean()) ** 2).sum()
    if tot == 0:
        return 0.0
    b = sum(((y[g == u].mean() - y.mean()) ** 2) * (g == u).sum() for u in np.unique(g))
    return float(b / tot)


def hist_xcc(reps):
    """The joint-count histograms (passes 0, 2; one chunk per workgroup, a pure read of the keys): their
    workgroups' durations by XCC (the lab build packs XCC_ID over the range's end word, as for the
    scatter), and the wall against the mean -- does the pass wait for one half of the XCCs?"""
    for r in range(reps):
        rs.sort_device(keys, out, a.k, vals_in=vals, vals_out=vout, ws=ws, plan_=p)
        torch.cuda.synchronize()
        both = np.zeros(8 * 2048 * 4 + 4 * 256 * 4, dtype=np.uint64)
        assert fn(both.ctypes.data) == 0
        hb = both[8 * 2048 * 4:].reshape(4, 256, 4)
        for ps in (0, 2):
            t0, t1 = hb[ps, :, 0].astype(np.int64), hb[ps, :, 1].astype(np.int64)
            xcc = (hb[ps, :, 3] >> np.uint64(32)).astype(np.int64) & 15
            dur = (t1 - t0) * 10 / 1e3
            wall = (t1.max() - t0.min()) * 10 / 1e3
            by = [dur[xcc == x].mean() if (xcc == x).any() else float("nan") for x in range(8)]
            print(f"sort {r} joint histogram pass {ps}: wall {wall:7.1f} us, dur min/med/max {dur.min():6.1f} "
                  f"{np.median(dur):6.1f} {dur.max():6.1f}, start spread {(t0.max() - t0.min()) * 10 / 1e3:5.1f}, "
                  f"by XCC " + " ".join(f"{v:6.1f}" for v in by))


if a.hxcc:
    hist_xcc(a.hxcc)
    sys.exit(0)
buf, hbuf, where = records()
print("modes", rs.group_flags(p, ws), "chunks", p.num_chunks)
for ps in range(p.passes):
    t0, t1, cb, ce = (buf[ps, :, i].astype(np.int64) for i in range(4))
    dur = (t1 - t0) * 10 / 1e3  # 100 MHz ticks -> us
    start = (t0 - t0.min()) * 10 / 1e3
    size = ce - cb
    print(f"pass {ps}: wall {((t1.max() - t0.min()) * 10 / 1e3):8.1f} us  per-wg dur min/med/max "
          f"{dur.min():7.1f} {np.median(dur):7.1f} {dur.max():7.1f}  start spread {start.max():5.1f} us  "
          f"keys/chunk min/max {size.min()} {size.max()}  us per Mkey min/med/max "
          f"{(dur / size * 1e6).min():.1f} {np.median(dur / size * 1e6):.1f} {(dur / size * 1e6).max():.1f}  "
          f"end spread {((t1.max() - t1.min()) * 10 / 1e3):5.1f} us")
if a.reps:
    rate_correlation(a.reps)
if a.k != 8 or a.reps:
    sys.exit(0)
# the chunks of the pass asked for: what they hold (its input = the previous pass's output: the keys
# stably sorted by the lower digits, computed here)
ps = a.pss
h = rs.to_numpy_u32(keys)
inp = h[np.argsort(h & ((1 << (8 * ps)) - 1), kind="stable")] if ps > 0 else h
t0, t1, cb, ce = (buf[ps, :, i].astype(np.int64) for i in range(4))
dur = (t1 - t0) * 10 / 1e3
order = np.argsort(dur)
print(f"\npass {ps} chunks, slowest and fastest: us, keys, top key share, distinct digits, top digit share, "
      f"distinct keys, distinct lower-digit groups")
for c in list(order[-12:][::-1]) + list(order[:6]):
    x = inp[cb[c]:ce[c]]
    d = (x >> (8 * ps)) & 255
    u, cnt = np.unique(x, return_counts=True)
    du, dcnt = np.unique(d, return_counts=True)
    g = np.unique(x & ((1 << (8 * ps)) - 1)).size if ps > 0 else 0
    print(f"  chunk {c:3d} {dur[c]:8.1f} us {x.size:9d}  top key {cnt.max() / x.size:.3f}  digits {du.size:3d}  "
          f"top digit {dcnt.max() / x.size:.3f}  keys {u.size:8d}  groups {g}")

if a.dump:
    with open(a.dump, "w") as fh:
        fh.write("chunk,us,keys,top_digit,herfindahl,digits,groups\n")
        for c in range(256):
            x = inp[cb[c]:ce[c]]
            if x.size == 0:
                continue
            d = (x >> (8 * ps)) & 255
            dc = np.bincount(d, minlength=256) / x.size
            g = np.unique(x & ((1 << (8 * ps)) - 1)).size if ps > 0 else 0
            fh.write(f"{c},{dur[c]:.1f},{x.size},{dc.max():.4f},{(dc * dc).sum():.5f},{(dc > 0).sum()},{g}\n")
    print("wrote", a.dump)

if a.hist:
    print()
    for ps in (0, 2):
        t0, t1, cb, ce = (hbuf[ps, :, i].astype(np.int64) for i in range(4))
        dur = (t1 - t0) * 10 / 1e3
        print(f"joint histogram pass {ps}: wall {((t1.max() - t0.min()) * 10 / 1e3):8.1f} us  per-wg dur min/med/max "
              f"{dur.min():7.1f} {np.median(dur):7.1f} {dur.max():7.1f}  keys/chunk {(ce - cb).max()}")
    # pass 2's histogram input: the keys sorted by their low 16 bits; it counts (digit 2, digit 3)
    t0, t1, cb, ce = (hbuf[2, :, i].astype(np.int64) for i in range(4))
    dur = (t1 - t0) * 10 / 1e3
    inp = h[np.argsort(h & 0xFFFF, kind="stable")]
    print("pass 2 joint-count chunks, slowest and fastest: us, top pair share, distinct pairs, mean pair run, "
          "keys in runs >= 4, quads with one pair")
    for c in list(np.argsort(dur)[-10:][::-1]) + list(np.argsort(dur)[:6]):
        x = inp[cb[c]:ce[c]] >> 16
        u, cnt = np.unique(x, return_counts=True)
        brk = np.flatnonzero(np.diff(x) != 0)
        runs = np.diff(np.concatenate(([0], brk + 1, [x.size])))
        q = x[: x.size // 4 * 4].reshape(-1, 4)
        one = (q == q[:, :1]).all(axis=1).mean()
        print(f"  chunk {c:3d} {dur[c]:8.1f} us  top pair {cnt.max() / x.size:.3f}  pairs {u.size:8d}  run "
              f"{x.size / runs.size:7.2f}  in runs>=4 {runs[runs >= 4].sum() / x.size:.3f}  one-pair quads {one:.3f}")
