"""CPU-side checks of the C ABI: the library builds, loads, and exports every symbol that
include/rsort.h declares; planning and argument validation (no kernel launches here)."""
import ctypes
import re
from pathlib import Path

import pytest

from _rs import PKG, rs

ROOT = Path(__file__).resolve().parent.parent


def _declared_symbols():
    text = (ROOT / "include" / "rsort.h").read_text()
    return sorted(set(re.findall(r"RSORT_API\s+[\w\s\*]+?\b(rsort_\w+)\s*\(", text)))


def test_library_present_and_loads():
    assert rs.lib_path().exists(), "run __graft_entry__.build() first"
    lib = rs._lib()
    assert isinstance(lib, ctypes.CDLL)
    assert rs.version() == "0.1.0"


def test_every_declared_symbol_is_exported_and_bound():
    declared = _declared_symbols()
    assert len(declared) >= 25
    lib = rs._lib()
    for name in declared:
        assert hasattr(lib, name), name
        assert name in rs.SIGNATURES, f"{name} has no ctypes signature in radixsort.py"
    assert set(rs.SIGNATURES) == set(declared)


def test_status_strings():
    lib = rs._lib()
    for st in range(12):
        assert lib.rsort_status_string(st) != b"unknown status", st
        assert rs.STATUS_NAMES[st].startswith("RSORT_")
    assert lib.rsort_status_string(12) == b"unknown status"
    assert lib.rsort_status_string(2) == b"k_bits outside [1, 13]"


@pytest.mark.parametrize("n,k", [(0, 8), (1, 8), (513, 4), ((1 << 24) + 1, 8), (1 << 26, 4), (1 << 30, 8),
                                 ((1 << 32) - 1, 8), (100003, 12), (5, 1)])
def test_plan_geometry(n, k):
    p = rs.plan(n, k, False, tiles_per_chunk=0)
    assert p.passes == -(-32 // k)
    assert p.bins == 1 << k
    assert (p.threads, p.tile_keys) in {(256, 4096), (512, 16384), (512, 8192), (1024, 16384)}
    if n >= 2 * 256 * 16384 and 5 <= k <= 8:
        assert (p.threads, p.tile_keys) == (1024, 16384)  # whole-line (rs_scatter_lines) tiles
        assert (rs.plan(n, k, True).threads, rs.plan(n, k, True).tile_keys) == (1024, 8192)  # pairs lines
    assert p.chunk_keys == p.tiles_per_chunk * p.tile_keys
    assert p.num_chunks * p.chunk_keys >= n
    assert (p.num_chunks - 1) * p.chunk_keys < max(n, 1)
    assert p.table_entries == p.bins * p.num_chunks
    assert p.workspace_bytes >= 4 * n + 4 * p.table_entries
    assert rs.workspace_size(n, k) == p.workspace_bytes
    pp = rs.plan(n, k, True)
    assert pp.workspace_bytes >= 8 * n + 4 * pp.table_entries


def test_plan_explicit_tiles_per_chunk():
    p = rs.plan(1 << 20, 8, tiles_per_chunk=1)
    assert p.num_chunks == 256 and p.chunk_keys == 4096
    p = rs.plan(1 << 20, 8, tiles_per_chunk=7)
    assert p.num_chunks == -(-256 // 7)


@pytest.mark.parametrize("n,k,status", [(10, 0, 2), (10, 14, 2), (-1, 8, 3), (1 << 32, 8, 3)])
def test_plan_rejects(n, k, status):
    with pytest.raises(rs.RSortError) as e:
        rs.plan(n, k)
    assert e.value.status == status


def test_device_entry_validates_before_touching_the_gpu():
    lib = rs._lib()
    # bad k, bad n: rejected before any HIP call
    assert lib.rsort_u32_device(None, None, 10, 0, None, 0, None) == 2
    assert lib.rsort_u32_device(None, None, -5, 8, None, 0, None) == 3
    # n == 0 is a no-op that needs no buffers
    assert lib.rsort_u32_device(None, None, 0, 8, None, 0, None) == 0
    # NULL buffers with n > 0
    assert lib.rsort_u32_device(None, None, 10, 8, None, 0, None) == 1
    # misaligned pointers
    assert lib.rsort_u32_device(ctypes.c_void_p(2), ctypes.c_void_p(8), 10, 8, ctypes.c_void_p(256), 1 << 20, None) == 4
    # workspace too small
    assert lib.rsort_u32_device(ctypes.c_void_p(256), ctypes.c_void_p(512), 10, 8, ctypes.c_void_p(1024), 16, None) == 7
    assert lib.rsort_set_rank_algo(7) == 1
    assert lib.rsort_set_rank_algo(3) == 1
    assert lib.rsort_partition_device(None, None, None, None, 10, None, 0, None, None, 0, None) == 1
    assert lib.rsort_partition_device(None, None, None, None, 10, None, 17, None, None, 0, None) == 1


def test_python_mirror_error_behaviour():
    import numpy as np
    with pytest.raises(ValueError):
        rs.sort(np.zeros(4, np.uint32), 4, np.zeros(4, np.uint32), rs.SORT_BY_HOST)
    with pytest.raises(TypeError):
        rs.sortByDevice(np.zeros(4, np.int64), 4, np.zeros(4, np.uint32), 8)
    with pytest.raises(rs.RSortError) as e:
        rs.sortByDevice(np.zeros(4, np.uint32), 4, np.zeros(4, np.uint32), 14)
    assert e.value.status == 2


def test_no_cpu_fallback_without_device():
    """On a machine without a GPU the host entry must FAIL (RSORT_ERR_NODEV), not sort on CPU."""
    from _rs import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    import numpy as np
    x = np.arange(100, dtype=np.uint32)[::-1].copy()
    y = np.zeros_like(x)
    with pytest.raises(rs.RSortError) as e:
        rs.sortByDevice(x, x.size, y, 8)
    assert e.value.status == 8
    assert not y.any()


def test_package_sources_do_not_reference_the_oracle():
    for f in list(PKG.rglob("*.py")) + list(PKG.rglob("*.cpp")) + list(PKG.rglob("*.hip")) + \
            list((ROOT / "include").glob("*")):
        text = f.read_text()
        assert "liboracle" not in text and "oracle_sort" not in text and "_ref/libref" not in text, f


def test_reference_harness_cli_builds_and_links():
    """tools/rsort_cli: the reference main (Parallel7.cu:696-775) on include/radixsort.hpp."""
    import subprocess
    cli = ROOT / "tools" / "rsort_cli"
    assert cli.exists(), "built by __graft_entry__.build()"
    out = subprocess.run(["ldd", str(cli)], capture_output=True, text=True).stdout
    assert "librsort.so" in out and "not found" not in out.split("librsort.so")[1].split("\n")[0]


def test_compat_header_compiles_with_reference_style_main(tmp_path):
    """A Parallel*.cu-style caller (own sortByHost + main, the reference's sort() signature and
    default arguments) compiles and links unchanged against radixsort.hpp + librsort.so."""
    import subprocess
    src = tmp_path / "caller.cpp"
    src.write_text(r'''
#include "radixsort.hpp"
#include <string.h>
void sortByHost(const uint32_t *in, int n, uint32_t *out, int nBits) { memcpy(out, in, n * 4); (void)nBits; }
int main() {
    uint32_t in[4] = {3, 1, 2, 0}, out[4];
    sort(in, 4, out);                       // default SORT_BY_HOST, numBits = 4, blockSize = 1
    sort(in, 4, out, SORT_BY_DEVICE, 8, 512);
    sort(in, 4, out, SORT_BY_THRUST);
    return 0;
}
''')
    exe = tmp_path / "caller"
    cmd = ["g++", "-std=c++17", f"-I{ROOT / 'include'}", str(src), "-o", str(exe),
           f"-L{PKG}", "-lrsort", f"-Wl,-rpath,{PKG}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("n,world", [(1 << 27, 8), (1 << 22, 2), (3 << 24, 4)])
def test_multi_workspace_holds_any_local_sort(n, world):
    """rsort_multi_workspace_size covers the local sort of any received count up to the capacity --
    including counts whose plan is a digit-group plan with its joint-count rows (64 MiB) where the
    capacity's own plan is not one: the partition buffer (4 n B) plus the largest sort workspace."""
    lib = rs._lib()
    cap = rs.default_capacity(n)
    mw = int(lib.rsort_multi_workspace_size(n, cap, 8, 0, world))
    sizes = {cap, cap // 2 + 1, n, 1 << 25, (1 << 24) + 5, 1 << 23, 3 << 22, 1 << 20, 1}
    need = max(rs.workspace_size(m, 8) for m in sizes if m <= cap)
    assert mw >= 4 * n + need, (mw, need)
