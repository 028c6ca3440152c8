"""Python host mirror of the reference's sort interface, over the C ABI (include/rsort.h).

Names and argument meaning follow truongchauhien/CUDA.RadixSort (Parallel7.cu):
  Implementation                 enum {SORT_BY_HOST, SORT_BY_THRUST, SORT_BY_DEVICE}  (P7:22)
  sort(in, n, out, implementation, numBits, blockSize)                              (P7:641-662)
  sortByDevice(h_input, n, h_output, numBits, blockSize)                            (P7:530-639)
  sortByThrust(input, n, output)                                                   (P7:69-73)
plus device-resident entry points over torch tensors (torch is plumbing: device memory and
streams only) and the per-pass building blocks used by the parity tests.

Error behaviour: the reference prints and exit(EXIT_FAILURE)s on any CUDA error
(common.h:6-16); here every non-zero rsort_status raises RSortError carrying the status.

There is NO CPU fallback: the library must be built (python cuda.radixsort_amd/build.py) and
a HIP device visible, otherwise these functions raise. SORT_BY_HOST, the reference's
sequential CPU sort, is not part of this library (it is the test oracle, oracle/; the C++
compat header include/radixsort.hpp offers it to C++ callers of the reference API).
"""
from __future__ import annotations

import ctypes
import enum
import os
import time
from contextlib import contextmanager
from pathlib import Path

import numpy as np

try:  # load torch first so librsort binds to the same HIP runtime instance
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host->host API
    torch = None

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "librsort.so"

RSORT_OK = 0
STATUS_NAMES = {0: "RSORT_OK", 1: "RSORT_ERR_ARG", 2: "RSORT_ERR_BITS", 3: "RSORT_ERR_SIZE",
                4: "RSORT_ERR_ALIGN", 5: "RSORT_ERR_ALLOC", 6: "RSORT_ERR_HIP",
                7: "RSORT_ERR_WORKSPACE", 8: "RSORT_ERR_NODEV", 9: "RSORT_ERR_CAPACITY",
                10: "RSORT_ERR_COMM", 11: "RSORT_ERR_CHECK"}
RANK_MATCH, RANK_SPLIT, RANK_BALLOT = 0, 1, 2
PHASES = ("histogram", "scan", "scatter", "copy", "partition")


class Implementation(enum.IntEnum):
    SORT_BY_HOST = 0
    SORT_BY_THRUST = 1
    SORT_BY_DEVICE = 2


SORT_BY_HOST = Implementation.SORT_BY_HOST
SORT_BY_THRUST = Implementation.SORT_BY_THRUST
SORT_BY_DEVICE = Implementation.SORT_BY_DEVICE


class RSortError(RuntimeError):
    def __init__(self, status: int, where: str):
        self.status = status
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)} ({_lib().rsort_status_string(status).decode()})")


class Plan(ctypes.Structure):
    """rsort_plan (include/rsort.h)."""
    _fields_ = [("n", ctypes.c_int64), ("k_bits", ctypes.c_int32), ("passes", ctypes.c_int32),
                ("bins", ctypes.c_int32), ("threads", ctypes.c_int32), ("tile_keys", ctypes.c_int32),
                ("pairs", ctypes.c_int32), ("tiles_per_chunk", ctypes.c_int64),
                ("chunk_keys", ctypes.c_int64), ("num_chunks", ctypes.c_int64),
                ("table_entries", ctypes.c_int64), ("scan_blocks", ctypes.c_int64),
                ("workspace_bytes", ctypes.c_size_t)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class PhaseTimes(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double * len(PHASES)), ("launches", ctypes.c_int64 * len(PHASES)),
                ("keys", ctypes.c_int64 * len(PHASES))]

    def as_dict(self):
        return {p: {"ms": self.ms[i], "launches": self.launches[i], "keys": self.keys[i]}
                for i, p in enumerate(PHASES)}


MAX_RANKS = 16  # RSORT_MAX_RANKS


class SamplePlan(ctypes.Structure):
    """rsort_sample_plan (include/rsort.h, multi-GPU planning)."""
    _fields_ = [("world", ctypes.c_int32), ("stride", ctypes.c_int64), ("count", ctypes.c_int64 * MAX_RANKS),
                ("row_len", ctypes.c_int64), ("total", ctypes.c_int64)]


class MultiSplitters(ctypes.Structure):
    """rsort_multi_splitters."""
    _fields_ = [("world", ctypes.c_int32), ("nsplit", ctypes.c_int32),
                ("split", ctypes.c_uint32 * (2 * (MAX_RANKS - 1))), ("cut_bucket", ctypes.c_int32 * MAX_RANKS),
                ("cut_inside", ctypes.c_int32 * MAX_RANKS)]

    @property
    def splitters(self) -> list[int]:
        return [int(self.split[i]) for i in range(self.nsplit)]


class ExchangePlan(ctypes.Structure):
    """rsort_exchange_plan."""
    _fields_ = [("world", ctypes.c_int32), ("me", ctypes.c_int32),
                ("send_off", ctypes.c_int64 * MAX_RANKS), ("send_cnt", ctypes.c_int64 * MAX_RANKS),
                ("recv_off", ctypes.c_int64 * MAX_RANKS), ("recv_cnt", ctypes.c_int64 * MAX_RANKS),
                ("n_recv", ctypes.c_int64), ("offset", ctypes.c_int64), ("total", ctypes.c_int64),
                ("max_message", ctypes.c_int64), ("over_capacity", ctypes.c_int32)]


_AG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                          ctypes.c_void_p)
_EX_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                          ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_void_p),
                          ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p)


class Transport(ctypes.Structure):
    """rsort_transport: the multi-GPU sort's communication plug-in."""
    _fields_ = [("ctx", ctypes.c_void_p), ("world", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("allgather", _AG_FN), ("exchange", _EX_FN)]


_HAG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_HEX_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                           ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_void_p),
                           ctypes.POINTER(ctypes.c_size_t))


class HostTransportFns(ctypes.Structure):
    """rsort_host_transport: a transport over host memory (wrapped by rsort_host_transport_wrap)."""
    _fields_ = [("ctx", ctypes.c_void_p), ("world", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("allgather", _HAG_FN), ("exchange", _HEX_FN)]


class MultiStats(ctypes.Structure):
    """rsort_multi_stats: the phases and traffic of one multi-GPU sort (rsort_multi_last_stats)."""
    _fields_ = [("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("halves", ctypes.c_int32),
                ("direct", ctypes.c_int32), ("rounds", ctypes.c_int64), ("bytes_per_key", ctypes.c_int64),
                ("send_keys", ctypes.c_int64 * MAX_RANKS), ("recv_keys", ctypes.c_int64 * MAX_RANKS),
                ("n_in", ctypes.c_int64), ("n_out", ctypes.c_int64),
                ("ms_plan", ctypes.c_double), ("ms_partition", ctypes.c_double), ("ms_exchange", ctypes.c_double),
                ("ms_local_sort", ctypes.c_double), ("ms_total", ctypes.c_double)]

    def as_dict(self):
        w = self.world
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("send_keys", "recv_keys")}
        d["send_keys"] = [int(self.send_keys[i]) for i in range(w)]
        d["recv_keys"] = [int(self.recv_keys[i]) for i in range(w)]
        return d


# Every symbol include/rsort.h declares, with its ctypes signature.
_u32p, _vp, _i64, _int, _sz = (ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_int, ctypes.c_size_t)
_i = _int
_PP = ctypes.POINTER(Plan)
SIGNATURES = {
    "rsort_status_string": ([_int], ctypes.c_char_p),
    "rsort_version": ([], _int),
    "rsort_plan_make": ([_i64, _int, _int, _i64, _PP], _int),
    "rsort_workspace_size": ([_i64, _int, _int], _sz),
    "rsort_u32_device": ([_vp, _vp, _i64, _int, _vp, _sz, _vp], _int),
    "rsort_u32_pairs_device": ([_vp, _vp, _vp, _vp, _i64, _int, _vp, _sz, _vp], _int),
    "rsort_sort_planned": ([_PP, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _int),
    "rsort_u32": ([_vp, _vp, _i64, _int], _int),
    "rsort_u32_ex": ([_vp, _vp, _i64, _int, _int, ctypes.POINTER(PhaseTimes)], _int),
    "rsort_u32_pairs": ([_vp, _vp, _vp, _vp, _i64, _int], _int),
    "rsort_pass_histogram": ([_PP, _vp, _int, _vp, _vp], _int),
    "rsort_pass_scan": ([_PP, _vp, _vp, _vp], _int),
    "rsort_pass_scatter": ([_PP, _vp, _vp, _vp, _vp, _int, _vp, _vp], _int),
    "rsort_pass_local_sort": ([_PP, _vp, _vp, _vp, _vp, _int, _vp], _int),
    "rsort_set_rank_algo": ([_int], _int),
    "rsort_get_rank_algo": ([], _int),
    "rsort_set_group_chunks": ([_int], _int),
    "rsort_get_group_chunks": ([], _int),
    "rsort_group_flags": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], _int),
    "rsort_lane_order_probe": ([], _int),
    "rsort_plan_check": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], _int),
    "rsort_cut_plan_stats": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], _int),
    "rsort_plan_features": ([_PP], _int),
    "rsort_inject_table_fault": ([_int], _int),
    "rsort_inject_rank_fault": ([_int], _int),
    "rsort_scatter_kernels_used": ([ctypes.c_char_p, _sz, _int], _sz),
    "rsort_profile_begin": ([], _int),
    "rsort_profile_end": ([ctypes.POINTER(PhaseTimes)], _int),
    "rsort_partition_workspace_size": ([_i64, _int, _int], _sz),
    "rsort_partition_device": ([_vp, _vp, _vp, _vp, _i64, _u32p, _int, _vp, _vp, _sz, _vp], _int),
    "rsort_partition_check": ([_i64, _int, _int, _vp, ctypes.c_void_p, _vp], _int),
    "rsort_top_histogram": ([_vp, _i64, _int, _vp, _vp, _sz, _vp], _int),
    "rsort_top_histogram_sampled": ([_vp, _i64, _int, _int, _vp, _vp], _int),
    "rsort_multi_workspace_size": ([_i64, _i64, _int, _int, _int], _sz),
    "rsort_u32_multi": ([_vp, _vp, _i64, _vp, _vp, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64), _int, _vp,
                         _vp, _sz, _vp], _int),
    "rsort_multi_sample_plan": ([_i, ctypes.POINTER(_i64), _i64, ctypes.POINTER(SamplePlan)], _int),
    "rsort_sample_device": ([_vp, _i64, _i64, _i64, _i64, _vp, _vp], _int),
    "rsort_multi_quantile_index": ([ctypes.POINTER(SamplePlan), _int], _i64),
    "rsort_multi_splitters_make": ([_int, _u32p, ctypes.POINTER(MultiSplitters)], _int),
    "rsort_multi_splitters_make_hot": ([_int, _u32p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(MultiSplitters)],
                                       _int),
    "rsort_multi_exchange_plan": ([_int, _int, _int, ctypes.POINTER(_i64), ctypes.POINTER(MultiSplitters),
                                   ctypes.POINTER(_i64), ctypes.POINTER(ExchangePlan)], _int),
    "rsort_u32_multi_transport": ([_vp, _vp, _i64, _vp, _vp, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64), _int,
                                   ctypes.POINTER(Transport), _vp, _sz, _vp], _int),
    "rsort_set_exchange_piece": ([_i64], _i64),
    "rsort_set_multi_options": ([_int], _int),
    "rsort_multi_exchange_rounds": ([_i64, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64)], _int),
    "rsort_multi_set_profiling": ([_int], _int),
    "rsort_rccl_unique_id": ([_vp], _int),
    "rsort_rccl_comm_init": ([ctypes.POINTER(ctypes.c_void_p), _int, _int, _vp, _int], _int),
    "rsort_rccl_comm_destroy": ([_vp], _int),
    "rsort_set_comm_timeout": ([_int], _int),
    "rsort_multi_inject_failure": ([_int, _int, _int], _int),
    "rsort_multi_last_stats": ([ctypes.POINTER(MultiStats)], _int),
    "rsort_host_transport_wrap": ([ctypes.POINTER(HostTransportFns), ctypes.POINTER(Transport)], _int),
    "rsort_host_transport_free": ([ctypes.POINTER(Transport)], None),
    "rsort_loopback_create": ([_int, ctypes.POINTER(ctypes.c_void_p)], _int),
    "rsort_loopback_transport": ([ctypes.c_void_p, _int, ctypes.POINTER(Transport)], _int),
    "rsort_loopback_destroy": ([ctypes.c_void_p], None),
    "rsort_vendor_workspace_size": ([_i64], _sz),
    "rsort_u32_vendor_device": ([_vp, _vp, _i64, _vp, _sz, _vp], _int),
    "rsort_u32_vendor": ([_vp, _vp, _i64], _int),
    "rsort_fingerprint_device": ([_vp, _vp, _i64, _vp, _vp], _int),
    "rsort_gen_uniform": ([_vp, _i64, ctypes.c_uint64, _vp], _int),
    "rsort_gen_zipf": ([_vp, _i64, ctypes.c_uint64, _vp, _i64, _vp], _int),
    "rsort_gen_iota": ([_vp, _i64, ctypes.c_uint32, _vp], _int),
}

_LIB = None


def _lib() -> ctypes.CDLL:
    """Load librsort.so; raise loudly when it is missing (no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is not built: run `python cuda.radixsort_amd/build.py` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(str(LIB_PATH))
        # (RSORT_LAB=1 RSORT_LAB_OLD_LIB=1: an older library for a same-box A/B, dev/lab.sh ab -- symbols
        # added since are left unbound; anywhere else a missing symbol is an error)
        old = os.environ.get("RSORT_LAB") == "1" and os.environ.get("RSORT_LAB_OLD_LIB") == "1"
        for name, (args, res) in SIGNATURES.items():
            if old and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = lib
    return _LIB


def lib_path() -> Path:
    return LIB_PATH


def _check(status: int, where: str):
    if status != RSORT_OK:
        raise RSortError(status, where)


def version() -> str:
    v = _lib().rsort_version()
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}"


# ------------------------------------------------------------------------------ host API
def _host_u32(a, n=None, name="array"):
    a = np.asarray(a)
    if a.dtype != np.uint32 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError(f"{name} must be a C-contiguous uint32 numpy array")
    if n is not None and a.size < n:
        raise ValueError(f"{name} holds {a.size} < n={n} elements")
    return a


def sortByDevice(h_input, n, h_output, numBits, blockSize=512, times: dict | None = None):
    """Drop-in for the reference's sortByDevice (Parallel7.cu:530-639): host arrays in/out,
    synchronous. `times`, if a dict, receives the per-phase kernel times of this call."""
    h_input = _host_u32(h_input, n, "h_input")
    h_output = _host_u32(h_output, n, "h_output")
    pt = PhaseTimes()
    st = _lib().rsort_u32_ex(h_input.ctypes.data, h_output.ctypes.data, int(n), int(numBits), int(blockSize),
                             ctypes.byref(pt) if times is not None else None)
    _check(st, "sortByDevice")
    if times is not None:
        times.update(pt.as_dict())


def sortByThrust(input, n, output):
    """The reference's vendor comparator (Parallel7.cu:69-73): rocPRIM radix sort on ROCm."""
    input = _host_u32(input, n, "input")
    output = _host_u32(output, n, "output")
    _check(_lib().rsort_u32_vendor(input.ctypes.data, output.ctypes.data, int(n)), "sortByThrust")


def sortPairsByDevice(keys_in, vals_in, n, keys_out, vals_out, numBits):
    """Stable key + u32 payload sort (BASELINE config 4; no reference counterpart)."""
    args = [_host_u32(a, n, nm) for a, nm in ((keys_in, "keys_in"), (vals_in, "vals_in"),
                                               (keys_out, "keys_out"), (vals_out, "vals_out"))]
    _check(_lib().rsort_u32_pairs(args[0].ctypes.data, args[1].ctypes.data, args[2].ctypes.data,
                                  args[3].ctypes.data, int(n), int(numBits)), "sortPairsByDevice")


def sort(input, n, output, implementation=SORT_BY_HOST, numBits=4, blockSize=1, verbose=True):
    """Mirror of the reference dispatcher (Parallel7.cu:641-662), same defaults and prints.
    Returns the elapsed wall time in ms (the reference prints it, :660-661)."""
    impl = Implementation(implementation)
    if impl == SORT_BY_HOST:
        raise ValueError("SORT_BY_HOST is the reference's sequential CPU sort (Baseline1.cu:15-64); "
                         "it is the test oracle (oracle/), not part of the device library")
    t0 = time.perf_counter()
    if impl == SORT_BY_THRUST:
        if verbose:
            print("\nRadix Sort by Thrust library")
        sortByThrust(input, n, output)
    else:
        if verbose:
            print("\nRadix Sort by device:")
        sortByDevice(input, n, output, numBits, blockSize)
    ms = (time.perf_counter() - t0) * 1e3
    if verbose:
        print("Time: %.3f ms" % ms)
    return ms


# ------------------------------------------------------------------------------ device API
def _need_torch():
    if torch is None:
        raise RuntimeError("the device API needs torch (device memory / streams)")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(stream=None):
    _need_torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def plan(n: int, k_bits: int, pairs: bool = False, tiles_per_chunk: int = 0) -> Plan:
    p = Plan()
    _check(_lib().rsort_plan_make(int(n), int(k_bits), 1 if pairs else 0, int(tiles_per_chunk), ctypes.byref(p)),
           "rsort_plan_make")
    return p


def workspace_size(n: int, k_bits: int, pairs: bool = False) -> int:
    return int(_lib().rsort_workspace_size(int(n), int(k_bits), 1 if pairs else 0))


def empty_u32(n, device="cuda"):
    """Device buffer for u32 keys (torch int32 storage; the bits are the u32 keys)."""
    _need_torch()
    return torch.empty(int(n), dtype=torch.int32, device=device)


def workspace(nbytes: int, device="cuda"):
    _need_torch()
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def sort_device(keys_in, keys_out, k_bits=8, vals_in=None, vals_out=None, ws=None, stream=None,
                plan_: Plan | None = None):
    """Stream-ordered device sort of torch int32/uint32 tensors (bits = u32 keys)."""
    n = keys_in.numel()
    pairs = vals_in is not None
    p = plan_ if plan_ is not None else plan(n, k_bits, pairs)
    if ws is None:
        ws = workspace(p.workspace_bytes, keys_in.device)
    _check(_lib().rsort_sort_planned(ctypes.byref(p), _ptr(keys_in), _ptr(vals_in), _ptr(keys_out),
                                     _ptr(vals_out), _ptr(ws), ws.numel(), _stream(stream)),
           "rsort_sort_planned")
    return keys_out


def group_flags(p: Plan, ws, stream=None) -> list[int]:
    """How the odd passes (1, 3) of the last sort with plan `p` and workspace `ws` took their chunks
    (rsort_group_flags; synchronises the stream): 1 digit groups, 2 equal chunks cutting unbalanced
    groups, 0 fixed chunks with counted histograms."""
    flags = (ctypes.c_int * 2)()
    _check(_lib().rsort_group_flags(ctypes.byref(p), _ptr(ws), flags, _stream(stream)), "rsort_group_flags")
    return [int(flags[0]), int(flags[1])]


def cut_plan_stats(p: Plan, ws, stream=None) -> list[dict]:
    """How the last sort's cut plans (passes 1 and 3) took their pieces' counts (rsort_cut_plan_stats;
    synchronises the stream): per pass {key_ranges, row_tasks, direct_adds, negative_ranges}."""
    st = (ctypes.c_int * 8)()
    _check(_lib().rsort_cut_plan_stats(ctypes.byref(p), _ptr(ws), st, _stream(stream)), "rsort_cut_plan_stats")
    keys = ("key_ranges", "row_tasks", "direct_adds", "negative_ranges")
    return [{k: int(st[4 * i + j]) for j, k in enumerate(keys)} for i in range(2)]


FEAT_GROUPS, FEAT_NEXT_DIGIT, FEAT_RAW_TABLES, FEAT_TAIL_SCAN = 1, 2, 4, 8


def plan_features(p: Plan) -> int:
    """rsort_plan_features: the carried-histogram scheme a sort with plan `p` takes (FEAT_* bits)."""
    f = int(_lib().rsort_plan_features(ctypes.byref(p)))
    if f < 0:
        raise RSortError(-f, "rsort_plan_features")
    return f


@contextmanager
def table_fault():
    """TEST HOOK (rsort_inject_table_fault): raw-table sorts corrupt the table pass 1 reads."""
    old = _lib().rsort_inject_table_fault(1)
    try:
        yield
    finally:
        _lib().rsort_inject_table_fault(old)


@contextmanager
def rank_fault():
    """TEST HOOK (rsort_inject_rank_fault): the lane-ordered scatter kernels swap two ranks per digit in
    the slot their per-tile rank check reads (a broken lane order); the check must report it."""
    old = _lib().rsort_inject_rank_fault(1)
    try:
        yield
    finally:
        _lib().rsort_inject_rank_fault(old)


CHECK_TABLE, CHECK_RANK_ORDER = 1, 2


def plan_check(p: Plan, ws, stream=None) -> int:
    """The on-device self-checks of the last sort with plan `p` and workspace `ws`
    (rsort_plan_check; synchronises the stream): 0 = all passed, else CHECK_TABLE / CHECK_RANK_ORDER bits."""
    f = ctypes.c_int()
    _check(_lib().rsort_plan_check(ctypes.byref(p), _ptr(ws), ctypes.byref(f), _stream(stream)), "rsort_plan_check")
    return int(f.value)


def scatter_kernels_used(reset: bool = False) -> list[str]:
    """The scatter kernel instantiations launched since the last reset (rsort_scatter_kernels_used):
    what actually ran, from the library's own dispatch."""
    n = int(_lib().rsort_scatter_kernels_used(None, 0, 0))
    buf = ctypes.create_string_buffer(n + 1)
    _lib().rsort_scatter_kernels_used(buf, n + 1, 1 if reset else 0)
    s = buf.value.decode()
    return s.split(";") if s else []


def pass_histogram(p: Plan, keys, shift, table, stream=None):
    _check(_lib().rsort_pass_histogram(ctypes.byref(p), _ptr(keys), int(shift), _ptr(table), _stream(stream)),
           "rsort_pass_histogram")


def pass_scan(p: Plan, table, block_sums, stream=None):
    _check(_lib().rsort_pass_scan(ctypes.byref(p), _ptr(table), _ptr(block_sums), _stream(stream)),
           "rsort_pass_scan")


def pass_scatter(p: Plan, kin, kout, shift, table, vin=None, vout=None, stream=None):
    _check(_lib().rsort_pass_scatter(ctypes.byref(p), _ptr(kin), _ptr(vin), _ptr(kout), _ptr(vout), int(shift),
                                     _ptr(table), _stream(stream)), "rsort_pass_scatter")


def pass_local_sort(p: Plan, kin, kout, shift, vin=None, vout=None, stream=None):
    _check(_lib().rsort_pass_local_sort(ctypes.byref(p), _ptr(kin), _ptr(vin), _ptr(kout), _ptr(vout), int(shift),
                                        _stream(stream)), "rsort_pass_local_sort")


def set_rank_algo(algo: int):
    _check(_lib().rsort_set_rank_algo(int(algo)), "rsort_set_rank_algo")


def get_rank_algo() -> int:
    return int(_lib().rsort_get_rank_algo())


def set_group_chunks(enable: bool):
    """Digit-group chunks on every second k = 8 pass (rsort_set_group_chunks; default on)."""
    _check(_lib().rsort_set_group_chunks(1 if enable else 0), "rsort_set_group_chunks")


def get_group_chunks() -> bool:
    return bool(_lib().rsort_get_group_chunks())


def scatter_kernel_name(p: Plan, out_aligned16: bool = True) -> str:
    """Which scatter kernel family a sort with plan `p` runs (a mirror of the dispatch in
    rsort_kernels.hip; scatter_kernels_used() reports what actually ran)."""
    lines = ((p.threads, p.tile_keys) == (1024, 16384) and not p.pairs) or \
        ((p.threads, p.tile_keys) == (1024, 8192) and p.pairs and 5 <= p.k_bits <= 8) or \
        ((p.threads, p.tile_keys) == (256, 4096) and not p.pairs and 3 <= p.k_bits <= 4)
    if lines and out_aligned16 and get_rank_algo() == RANK_MATCH and lane_order_probe() == 1:
        # RSORT_PAIRS64=1 under RSORT_LAB=1 (A/B runs) makes the library's dispatch take the 64-B-line
        # pairs kernel
        pairs64 = os.environ.get("RSORT_LAB", "") == "1" and os.environ.get("RSORT_PAIRS64", "") not in ("", "0")
        return "rs_scatter_pairs" if p.pairs and p.k_bits >= 7 and not pairs64 else "rs_scatter_lines"
    return "rs_scatter"


# ---------------------------------------------------------------- multi-GPU over RCCL (C ABI)
NCCL_UNIQUE_ID_BYTES = 128


def rccl_unique_id() -> bytes:
    """rsort_rccl_unique_id: made on one rank, sent to the others out of band."""
    buf = ctypes.create_string_buffer(NCCL_UNIQUE_ID_BYTES)
    _check(_lib().rsort_rccl_unique_id(buf), "rsort_rccl_unique_id")
    return buf.raw  # (raw: the id holds NUL bytes)


def set_comm_timeout(ms: int) -> int:
    """rsort_set_comm_timeout: how long one RCCL step of the multi-GPU sort may take before the
    communicator is aborted (RSORT_ERR_COMM instead of a hang); returns the old value."""
    return int(_lib().rsort_set_comm_timeout(int(ms)))


class RcclComm:
    """An RCCL communicator for rsort_u32_multi (one rank per GPU; the current device), set up
    non-blocking by rsort_rccl_comm_init: a peer that never joins ends in RSortError (status 10,
    RSORT_ERR_COMM) after `timeout_ms` (default: the library's communicator timeout) instead of a
    hang. After any RSORT_ERR_COMM from a sort the communicator may have been aborted; close() knows."""

    def __init__(self, world: int, rank: int, uid: bytes, timeout_ms: int = 0):
        if len(uid) != NCCL_UNIQUE_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        buf = ctypes.create_string_buffer(bytes(uid), NCCL_UNIQUE_ID_BYTES)
        self.handle = ctypes.c_void_p()
        _check(_lib().rsort_rccl_comm_init(ctypes.byref(self.handle), int(world), int(rank), buf, int(timeout_ms)),
               "rsort_rccl_comm_init")
        self.world, self.rank = world, rank

    def close(self):
        if self.handle:
            _lib().rsort_rccl_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()


def default_capacity(n: int) -> int:
    """Output room per rank for n local keys: balanced output is about the mean count plus the
    sampling error (~0.1 %); 5/4 n + 64 Ki covers uneven per-rank n up to that."""
    return int(n + n // 4 + (1 << 16))


def multi_sort_device(comm, keys, k_bits=8, vals=None, capacity=None, stream=None, ws=None, out=None):
    """rsort_u32_multi (comm: RcclComm) or rsort_u32_multi_transport (comm: a Transport):
    returns (keys_out[:count], vals_out[:count] or None, global offset)."""
    n = keys.numel()
    cap = int(capacity if capacity is not None else default_capacity(n))
    pairs = vals is not None
    kout, vout = out if out is not None else (empty_u32(cap, keys.device), empty_u32(cap, keys.device) if pairs
                                               else None)
    world = comm.world
    wsb = int(_lib().rsort_multi_workspace_size(n, cap, k_bits, 1 if pairs else 0, world))
    if ws is None or ws.numel() < wsb:
        ws = workspace(wsb, keys.device)
    cnt, off = ctypes.c_int64(), ctypes.c_int64()
    if isinstance(comm, Transport):
        st = _lib().rsort_u32_multi_transport(_ptr(keys), _ptr(vals), n, _ptr(kout), _ptr(vout), cap,
                                              ctypes.byref(cnt), ctypes.byref(off), int(k_bits), ctypes.byref(comm),
                                              _ptr(ws), ws.numel(), _stream(stream))
        _check(st, "rsort_u32_multi_transport")
    else:
        _check(_lib().rsort_u32_multi(_ptr(keys), _ptr(vals), n, _ptr(kout), _ptr(vout), cap, ctypes.byref(cnt),
                                      ctypes.byref(off), int(k_bits), comm.handle, _ptr(ws), ws.numel(),
                                      _stream(stream)), "rsort_u32_multi")
    c = cnt.value
    return kout[:c], (vout[:c] if pairs else None), off.value


MULTI_OVERLAP, MULTI_FULL, MULTI_NO_OVERLAP = 1, 2, 4
MULTI_AUTO_OVERLAP_MAX_WORLD = 8  # neither overlap flag: the overlap runs for 2 <= world <= this (rsort.h)


def set_multi_options(flags: int) -> int:
    """rsort_set_multi_options: MULTI_OVERLAP (sort the lower half of each rank's range while the
    upper half is exchanged) or MULTI_NO_OVERLAP (never; neither flag: the overlap runs for 2 <= world <=
    MULTI_AUTO_OVERLAP_MAX_WORLD), MULTI_FULL (the whole protocol also at world 1); returns the old flags."""
    return int(_lib().rsort_set_multi_options(int(flags)))


@contextmanager
def multi_options(flags: int):
    old = set_multi_options(flags)
    try:
        yield
    finally:
        set_multi_options(old)


def set_exchange_piece(keys: int) -> int:
    """Largest exchange message per round of rsort_u32_multi* (keys); returns the old value."""
    return int(_lib().rsort_set_exchange_piece(int(keys)))


def multi_set_profiling(enable: bool) -> bool:
    """rsort_multi_set_profiling: per-phase hipEvents in every multi-GPU sort (which then syncs)."""
    return bool(_lib().rsort_multi_set_profiling(1 if enable else 0))


def multi_last_stats() -> dict:
    """rsort_multi_last_stats: the calling thread's last profiled multi-GPU sort."""
    st = MultiStats()
    _check(_lib().rsort_multi_last_stats(ctypes.byref(st)), "rsort_multi_last_stats")
    return st.as_dict()


class HostTransport:
    """rsort_host_transport_wrap over two Python callables working on host (numpy) buffers:
    allgather(send: np.uint8 array) -> bytes-like of world * len(send) bytes in rank order, and
    exchange(sends: list of np.uint8 arrays, recv_sizes: list of int) -> list of bytes-like. The
    C wrapper stages the device bytes; `.transport` is the rsort_transport to pass as `comm`."""

    def __init__(self, world: int, rank: int, allgather, exchange):
        self.world, self.rank = world, rank
        self._errors = []

        def ag(ctx, h_send, h_recv, nbytes):
            try:
                send = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, nbytes)).from_address(h_send))[:nbytes]
                got = np.frombuffer(allgather(send.copy()), dtype=np.uint8)
                if got.size != world * nbytes:
                    raise ValueError(f"allgather returned {got.size} bytes, expected {world * nbytes}")
                if got.size:
                    ctypes.memmove(h_recv, got.ctypes.data, got.size)
                return 0
            except Exception as e:  # noqa: BLE001 -- any failure is a communication error to the C side
                self._errors.append(e)
                return 10  # RSORT_ERR_COMM

        def ex(ctx, h_send, send_bytes, h_recv, recv_bytes):
            try:
                sends = [np.ctypeslib.as_array((ctypes.c_uint8 * send_bytes[p]).from_address(h_send[p])).copy()
                         if send_bytes[p] else np.empty(0, np.uint8) for p in range(world)]
                outs = exchange(sends, [int(recv_bytes[p]) for p in range(world)])
                for p in range(world):
                    o = np.frombuffer(outs[p], dtype=np.uint8)
                    if o.size != recv_bytes[p]:
                        raise ValueError(f"exchange: {o.size} bytes from rank {p}, expected {recv_bytes[p]}")
                    if o.size:
                        ctypes.memmove(h_recv[p], o.ctypes.data, o.size)
                return 0
            except Exception as e:  # noqa: BLE001
                self._errors.append(e)
                return 10

        self._fns = HostTransportFns(None, world, rank, _HAG_FN(ag), _HEX_FN(ex))  # keeps the callbacks alive
        self.transport = Transport()
        _check(_lib().rsort_host_transport_wrap(ctypes.byref(self._fns), ctypes.byref(self.transport)),
               "rsort_host_transport_wrap")
        self.transport.world, self.transport.rank = world, rank

    @property
    def errors(self):
        return list(self._errors)

    def close(self):
        if self.transport.ctx:
            _lib().rsort_host_transport_free(ctypes.byref(self.transport))


class LoopbackGroup:
    """rsort_loopback_*: `world` in-process ranks (one thread each) for the multi-GPU sort."""

    def __init__(self, world: int):
        self.handle = ctypes.c_void_p()
        _check(_lib().rsort_loopback_create(int(world), ctypes.byref(self.handle)), "rsort_loopback_create")
        self.world = world

    def transport(self, rank: int) -> Transport:
        t = Transport()
        _check(_lib().rsort_loopback_transport(self.handle, int(rank), ctypes.byref(t)), "rsort_loopback_transport")
        return t

    def close(self):
        if self.handle:
            _lib().rsort_loopback_destroy(self.handle)
            self.handle = ctypes.c_void_p()


# ---------------------------------------------------------------- multi-GPU planning (host only)
def multi_sample_plan(n_per_rank, samples_per_rank: int) -> SamplePlan:
    world = len(n_per_rank)
    arr = (ctypes.c_int64 * max(1, world))(*[int(x) for x in n_per_rank])
    sp = SamplePlan()
    _check(_lib().rsort_multi_sample_plan(world, arr, int(samples_per_rank), ctypes.byref(sp)),
           "rsort_multi_sample_plan")
    return sp


def sample_device(keys, stride: int, count: int, row_len: int, out=None, stream=None):
    """rsort_sample_device: the regular splitter sample of the multi-GPU sort (row_len u32)."""
    out = out if out is not None else empty_u32(row_len, keys.device)
    _check(_lib().rsort_sample_device(_ptr(keys), keys.numel(), int(stride), int(count), int(row_len), _ptr(out),
                                      _stream(stream)), "rsort_sample_device")
    return out


def multi_exchange_rounds(max_message: int, limit: int) -> tuple[int, int]:
    """rsort_multi_exchange_rounds: (rounds, piece) of the exchange for messages of up to max_message
    keys, at most `limit` keys each."""
    r, p = ctypes.c_int64(), ctypes.c_int64()
    _check(_lib().rsort_multi_exchange_rounds(int(max_message), int(limit), ctypes.byref(r), ctypes.byref(p)),
           "rsort_multi_exchange_rounds")
    return int(r.value), int(p.value)


def multi_quantile_index(sp: SamplePlan, i: int) -> int:
    return int(_lib().rsort_multi_quantile_index(ctypes.byref(sp), int(i)))


def multi_splitters(world: int, quantile_keys, hot=None) -> MultiSplitters:
    """rsort_multi_splitters_make (hot None: every quantile key gets its equal-keys bucket) or
    rsort_multi_splitters_make_hot (hot: one flag per quantile key)."""
    q = (ctypes.c_uint32 * max(1, world - 1))(*[int(x) & 0xFFFFFFFF for x in quantile_keys])
    out = MultiSplitters()
    if hot is None:
        _check(_lib().rsort_multi_splitters_make(int(world), q, ctypes.byref(out)), "rsort_multi_splitters_make")
    else:
        h = (ctypes.c_int * max(1, world - 1))(*[1 if x else 0 for x in hot])
        _check(_lib().rsort_multi_splitters_make_hot(int(world), q, h, ctypes.byref(out)),
               "rsort_multi_splitters_make_hot")
    return out


def hot_reach(world: int, total_samples: int) -> int:
    """How far (in samples) a quantile key's run must reach on one side of its quantile position to count
    as hot (rsort_u32_multi* and multi.py alike): ~1/128 of a rank's share of the sample."""
    return max(1, int(total_samples) // (int(world) * 128))


def hot_flags(sorted_sample, quantile_positions, world: int) -> list[int]:
    """The hot flag of each quantile key from the sorted sample (numpy): its value also sits hot_reach
    samples below or above its position."""
    s = sorted_sample
    L = hot_reach(world, s.size)
    out = []
    for qi in quantile_positions:
        v = s[qi]
        out.append(int((qi - L >= 0 and s[qi - L] == v) or (qi + L < s.size and s[qi + L] == v)))
    return out


def multi_exchange_plan(world: int, me: int, counts, spl: MultiSplitters, capacity) -> ExchangePlan:
    """counts: world x buckets (rows = source ranks); capacity: world entries. Raises RSortError
    (status 9, RSORT_ERR_CAPACITY) on every rank alike when any rank's output would overflow."""
    c = np.ascontiguousarray(counts, dtype=np.int64)
    buckets = c.shape[1]
    cap = np.ascontiguousarray(capacity, dtype=np.int64)
    out = ExchangePlan()
    st = _lib().rsort_multi_exchange_plan(int(world), int(me), int(buckets),
                                          c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(spl),
                                          cap.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(out))
    _check(st, "rsort_multi_exchange_plan")
    return out


def lane_order_probe() -> int:
    """1 if the current device serves same-address LDS atomic lanes in lane order (the default
    ranking then uses one returning LDS add per key), 0 if not (ballot ranking)."""
    r = int(_lib().rsort_lane_order_probe())
    if r < 0:
        raise RSortError(-r if r < -1 else 5, "rsort_lane_order_probe")
    return r


@contextmanager
def rank_algo(algo: int):
    old = get_rank_algo()
    set_rank_algo(algo)
    try:
        yield
    finally:
        set_rank_algo(old)


@contextmanager
def group_chunks(enable: bool):
    old = get_group_chunks()
    set_group_chunks(enable)
    try:
        yield
    finally:
        set_group_chunks(old)


class Profile:
    """with Profile() as prof: ...  -> prof.times = {phase: {ms, launches, keys}}"""

    def __enter__(self):
        _check(_lib().rsort_profile_begin(), "rsort_profile_begin")
        self.times = None
        return self

    def __exit__(self, *exc):
        pt = PhaseTimes()
        st = _lib().rsort_profile_end(ctypes.byref(pt))
        self.times = pt.as_dict()
        if exc[0] is None:
            _check(st, "rsort_profile_end")
        return False


def partition_device(keys_in, keys_out, splitters, bucket_starts, vals_in=None, vals_out=None, ws=None,
                     stream=None):
    """Stable key-range partition into len(splitters)+1 buckets (multi-GPU exchange step)."""
    n = keys_in.numel()
    nb = len(splitters) + 1
    sp = (ctypes.c_uint32 * max(1, len(splitters)))(*[int(s) for s in splitters])
    need = int(_lib().rsort_partition_workspace_size(n, nb, 1 if vals_in is not None else 0))
    if ws is None or ws.numel() < need:
        ws = workspace(need, keys_in.device)
    _check(_lib().rsort_partition_device(_ptr(keys_in), _ptr(vals_in), _ptr(keys_out), _ptr(vals_out), n, sp, nb,
                                         _ptr(bucket_starts), _ptr(ws), ws.numel(), _stream(stream)),
           "rsort_partition_device")


def partition_check(n: int, num_buckets: int, pairs: bool, ws, stream=None) -> int:
    """rsort_partition_check: the last partition's on-device self-check in `ws` (0 = passed)."""
    f = ctypes.c_int()
    _check(_lib().rsort_partition_check(int(n), int(num_buckets), 1 if pairs else 0, _ptr(ws), ctypes.byref(f),
                                        _stream(stream)), "rsort_partition_check")
    return int(f.value)


def top_histogram_sampled(keys, top_bits, stride, hist, stream=None):
    """Top-bits histogram of every `stride`-th 256-key block (rsort_top_histogram_sampled)."""
    _check(_lib().rsort_top_histogram_sampled(_ptr(keys), keys.numel(), int(top_bits), int(stride), _ptr(hist),
                                              _stream(stream)), "rsort_top_histogram_sampled")


def top_histogram(keys, top_bits, hist, ws=None, stream=None):
    n = keys.numel()
    need = workspace_size(n, top_bits, False)
    if ws is None or ws.numel() < need:
        ws = workspace(need, keys.device)
    _check(_lib().rsort_top_histogram(_ptr(keys), n, int(top_bits), _ptr(hist), _ptr(ws), ws.numel(),
                                      _stream(stream)), "rsort_top_histogram")


def vendor_sort_device(keys_in, keys_out, ws=None, stream=None):
    n = keys_in.numel()
    need = int(_lib().rsort_vendor_workspace_size(n))
    if ws is None or ws.numel() < need:
        ws = workspace(need, keys_in.device)
    _check(_lib().rsort_u32_vendor_device(_ptr(keys_in), _ptr(keys_out), n, _ptr(ws), ws.numel(),
                                          _stream(stream)), "rsort_u32_vendor_device")


def fingerprint(keys, vals=None, stream=None) -> tuple[int, int]:
    """rsort_fingerprint_device: (multiset fingerprint, adjacent descents) of keys (+ values)."""
    out = torch.zeros(2, dtype=torch.int64, device=keys.device)
    _check(_lib().rsort_fingerprint_device(_ptr(keys), _ptr(vals), keys.numel(), _ptr(out), _stream(stream)),
           "rsort_fingerprint_device")
    h, d = out.cpu().tolist()
    return h & 0xFFFFFFFFFFFFFFFF, d


def gen_uniform(out, seed=0x5EED, stream=None):
    _check(_lib().rsort_gen_uniform(_ptr(out), out.numel(), int(seed), _stream(stream)), "rsort_gen_uniform")


def gen_zipf(out, cdf, seed=0x5EED, stream=None):
    _check(_lib().rsort_gen_zipf(_ptr(out), out.numel(), int(seed), _ptr(cdf), cdf.numel(), _stream(stream)),
           "rsort_gen_zipf")


def gen_iota(out, base=0, stream=None):
    _check(_lib().rsort_gen_iota(_ptr(out), out.numel(), int(base), _stream(stream)), "rsort_gen_iota")


def to_numpy_u32(t) -> np.ndarray:
    """Device/host int32 tensor -> numpy uint32 view of the same bits."""
    return t.detach().cpu().numpy().view(np.uint32)


def from_numpy_u32(a: np.ndarray, device="cuda"):
    _need_torch()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(device)
