"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

It loads oracle/_ref/libref.so -- the reference's own sortByHost (Baseline1.cu:15-64) and
sortByHostUsingParallelAlgorithm (Baseline4.cu:67-273), compiled from the unmodified sources
by oracle/build_ref.sh -- runs them on
  * the reference's own inputs: glibc rand() with its default seed (Parallel7.cu:717-723),
    DEBUG n=513 (keys rand()&0xFF, k=4; :705-706, :719, :737-738) and the default
    n=(1<<24)+1 (k=8 and k=4; :708, :740),
  * full-32-bit synthetic inputs (splitmix64 uniform and Zipf) at small sizes,
and stores inputs (when small), outputs (when small), FNV-1a-64 digests and sampled values.
The fixtures are DATA only (the reference's outputs); no reference source text is stored.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from _util import (GOLDEN_DIR, _ptr, fnv1a64, glibc_rand, ref_lib,  # noqa: E402
                   uniform_keys, zipf_keys)


def ref_sort(lib, keys, nbits):
    out = np.empty_like(keys)
    lib.ref_sort_by_host(_ptr(keys), keys.size, _ptr(out), nbits)
    return out


def ref_block_sort(lib, keys, nbits, block):
    out = np.empty_like(keys)
    lib.ref_block_sort(_ptr(keys), keys.size, _ptr(out), nbits, block)
    return out


def sample_idx(n):
    return sorted({0, 1, n // 3, n // 2, (2 * n) // 3, n - 2, n - 1} - {-1}) if n > 1 else [0]


def main():
    lib = ref_lib()
    if lib is None:
        raise SystemExit("oracle/_ref/libref.so unavailable (needs /root/reference)")
    cases = []

    # (1) the reference's DEBUG configuration: n=513, rand()&0xFF, k=4
    x = glibc_rand(513, debug=True)
    y = ref_sort(lib, x, 4)
    cases.append(dict(name="ref_debug_513_k4", source="glibc_rand_debug", n=513, k=4,
                      input=x.tolist(), output=y.tolist(),
                      fnv_in=fnv1a64(x), fnv_out=fnv1a64(y)))

    # (2) the reference's default configuration: n=(1<<24)+1, rand(), k=8 and k=4
    n = (1 << 24) + 1
    x = glibc_rand(n)
    for k in (8, 4):
        y = ref_sort(lib, x, k)
        idx = sample_idx(n)
        cases.append(dict(name=f"ref_default_{n}_k{k}", source="glibc_rand", n=n, k=k,
                          fnv_in=fnv1a64(x), fnv_out=fnv1a64(y),
                          samples={str(i): int(y[i]) for i in idx}))

    # (3) full 32-bit synthetic keys (bit 31 set half the time) at ragged sizes and all k
    for dist, n, k in [("uniform", 1000, 8), ("uniform", 4097, 4), ("uniform", 65537, 8),
                       ("uniform", 100003, 5), ("uniform", 100003, 11), ("uniform", 12345, 1),
                       ("uniform", 70000, 12), ("uniform", 1 << 20, 8),
                       ("zipf", 100003, 8), ("zipf", 1 << 20, 4)]:
        x = uniform_keys(n) if dist == "uniform" else zipf_keys(n)
        y = ref_sort(lib, x, k)
        idx = sample_idx(n)
        cases.append(dict(name=f"{dist}_{n}_k{k}", source=dist, seed=0x5EED, n=n, k=k,
                          fnv_in=fnv1a64(x), fnv_out=fnv1a64(y),
                          samples={str(i): int(y[i]) for i in idx}))

    # (4) the reference's block algorithm (Baseline4) on SURVEY §4's (n, k, bs) grid
    block_cases = []
    for n, k, bs in [(513, 4, 512), (513, 4, 64), (1048577, 8, 512), (1048577, 4, 256),
                     (100003, 8, 1000)]:
        x = glibc_rand(n)
        y = ref_block_sort(lib, x, k, bs)
        block_cases.append(dict(name=f"ref_block_{n}_k{k}_bs{bs}", source="glibc_rand", n=n, k=k,
                                block=bs, fnv_in=fnv1a64(x), fnv_out=fnv1a64(y)))

    out = dict(
        generator="tests/golden/make_golden.py",
        produced_by="oracle/_ref/libref.so (reference Baseline1.cu:15-64 / Baseline4.cu:67-273)",
        digest="FNV-1a-64 over little-endian u32 bytes",
        sort_cases=cases,
        block_cases=block_cases,
    )
    path = GOLDEN_DIR / "reference_vectors.json"
    path.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {path} ({len(cases)} sort cases, {len(block_cases)} block cases)")


if __name__ == "__main__":
    main()
