"""Multi-GPU sort: key-range (MSD bucket) partition with ONE exchange, then a local LSD sort.

No reference counterpart (the reference is single-GPU, Parallel7.cu:10/:697); this is
BASELINE config 5 / SURVEY §8e. One process per GPU, torch.distributed over RCCL ("nccl"):

  1. top-bits histogram of a 1/16 block sample       (HIP: rsort_top_histogram_sampled)
  2. all_reduce(SUM) of the 2^top_bits counts        (RCCL, 16 KiB)
  3. splitters on bin edges balancing ~n/world keys per rank (host, 4096 values)
  4. stable partition of the local keys into world buckets (HIP: rsort_partition_device)
  5. all_to_all of the per-destination counts        (RCCL, world x i64)
  6. all_to_all of the keys (and values)             (RCCL over xGMI: one peer per link;
                                                      messages cut to <= 512 MiB pieces)
  7. local LSD sort of what arrived                   (HIP: the single-GPU sort)

Rank r ends with the keys of global ranks [offset_r, offset_r + count_r); concatenating the
ranks' outputs in rank order gives exactly Baseline1's sorted array. Received chunks are
concatenated in source-rank order, so with values the whole sort stays stable.

`LocalOps` carries the three per-device steps; GpuOps (the product) calls librsort.so. Tests
substitute a numpy implementation to exercise the distributed logic on CPU with gloo.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import radixsort as rs

# Keys per RCCL message (512 MiB of u32): the RCCL of this image (2.26, ROCm 7; torch 2.10)
# silently leaves the second half of an all_to_all message of >= 2 GiB unwritten
# (dev/a2a_lab.py: 1 GiB arrives whole, 2 GiB - 4 B does not), and two ranks holding 2^30 keys
# each exchange ~2 GiB each way. Larger exchanges go in rounds of pieces this size.
MAX_MESSAGE = 1 << 27
# Splitters come from the top-bits histogram of every 16th block of 256 keys (all ranks sample
# alike, so the global histogram keeps its proportions; a 2^30-key rank reads 256 MiB, not 4 GiB).
SAMPLE_STRIDE = 16


class GpuOps:
    """Per-rank steps on the local MI355X through the C ABI."""

    def __init__(self, device):
        self.device = device
        self._ws = None

    def _workspace(self, nbytes):
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = rs.workspace(nbytes, self.device)
        return self._ws

    def top_histogram(self, keys, top_bits, stride=1):
        h = torch.empty(1 << top_bits, dtype=torch.int32, device=self.device)
        if stride > 1:
            rs.top_histogram_sampled(keys, top_bits, stride, h)
        else:
            rs.top_histogram(keys, top_bits, h, ws=self._workspace(rs.workspace_size(keys.numel(), top_bits)))
        return h

    def partition(self, keys, vals, splitters):
        n = keys.numel()
        nb = len(splitters) + 1
        ko = torch.empty_like(keys)
        vo = torch.empty_like(vals) if vals is not None else None
        starts = torch.empty(nb + 1, dtype=torch.int32, device=self.device)
        need = int(rs._lib().rsort_partition_workspace_size(n, nb, 1 if vals is not None else 0))
        rs.partition_device(keys, ko, splitters, starts, vals_in=vals, vals_out=vo, ws=self._workspace(need))
        return ko, vo, starts

    def sort(self, keys, vals, k_bits, out_keys=None, out_vals=None):
        n = keys.numel()
        ko = out_keys if out_keys is not None else torch.empty_like(keys)
        vo = None
        if vals is not None:
            vo = out_vals if out_vals is not None else torch.empty_like(vals)
        p = rs.plan(n, k_bits, vals is not None)
        rs.sort_device(keys, ko, k_bits, vals_in=vals, vals_out=vo, ws=self._workspace(p.workspace_bytes), plan_=p)
        return ko, vo


def choose_splitters(hist: np.ndarray, world: int, top_bits: int) -> list[int]:
    """world-1 ascending u32 splitters on bin edges of the global top-bits histogram so each
    rank receives about total/world keys. Bucket i takes the bins up to and including the
    first bin whose inclusive prefix count reaches (i+1)*total/world."""
    hist = np.asarray(hist, dtype=np.int64)
    nbins = hist.size
    cum = np.cumsum(hist)
    total = int(cum[-1])
    shift = 32 - top_bits
    out: list[int] = []
    for i in range(1, world):
        b = int(np.searchsorted(cum, (total * i) // world, side="left"))
        edge = b + 1
        s = (edge << shift) if edge < nbins else 0xFFFFFFFF
        out.append(max(s, out[-1]) if out else s)
    return out


def dist_sort(keys, k_bits=8, vals=None, ops=None, group=None, top_bits=12):
    """Sort the union of every rank's `keys` (and `vals`); return this rank's slice of the
    global sorted order as (keys, vals, global_offset).

    Collectives run on the tensors' device with RCCL ("nccl"); with the gloo backend (tests:
    several ranks sharing one GPU, or CPU-only ranks) they run on host copies."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if ops is None:
        ops = GpuOps(keys.device)
    dev = keys.device
    gloo = dist.get_backend(group) == "gloo"
    host_comm = gloo and dev.type != "cpu"
    cdev = torch.device("cpu") if host_comm else dev

    def a2a(out, inp, out_splits, in_splits, pieces):
        """all_to_all of `inp` (segments in_splits, one per destination) into `out` (segments
        out_splits, one per source), every message cut into `pieces` rounds of <= MAX_MESSAGE."""
        so = np.concatenate([[0], np.cumsum(in_splits)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(out_splits)]).astype(np.int64)
        for q in range(pieces):
            lo, hi = q * MAX_MESSAGE, (q + 1) * MAX_MESSAGE
            ins = [inp[so[i] + min(lo, in_splits[i]):so[i] + min(hi, in_splits[i])] for i in range(world)]
            outs = [out[ro[j] + min(lo, out_splits[j]):ro[j] + min(hi, out_splits[j])] for j in range(world)]
            if not gloo:
                dist.all_to_all(outs, ins, group=group)  # RCCL: grouped send/recv of the pieces
                continue
            # gloo (tests): one all_to_all_single of the round's pieces on host copies
            o = torch.empty(sum(int(x.numel()) for x in outs), dtype=out.dtype)
            dist.all_to_all_single(o, torch.cat([x.cpu() for x in ins]), output_split_sizes=[int(x.numel()) for x in outs],
                                   input_split_sizes=[int(x.numel()) for x in ins], group=group)
            off = 0
            for x in outs:
                x.copy_(o[off:off + x.numel()])
                off += x.numel()
        return out

    # 1-3: global histogram of the top bits (of a 1/SAMPLE_STRIDE block sample: the splitters
    # only set each rank's load) -> splitters
    h = ops.top_histogram(keys, top_bits, SAMPLE_STRIDE).to(torch.int64).to(cdev)
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    hist = h.cpu().numpy()
    splitters = choose_splitters(hist, world, top_bits)

    # 4: stable partition into `world` key ranges
    pk, pv, starts = ops.partition(keys, vals, splitters)
    st = starts.to(torch.int64).cpu().numpy()
    send = (st[1:] - st[:-1]).astype(np.int64)

    # 5: exchange counts
    send_t = torch.from_numpy(send).to(cdev)
    recv_t = torch.empty_like(send_t)
    dist.all_to_all_single(recv_t, send_t, group=group)
    recv = recv_t.cpu().numpy()

    # 6: exchange keys (and values); chunks arrive in source-rank order (stability). Every rank
    # needs the same number of rounds: the largest message anywhere, by one small all_reduce.
    n_recv = int(recv.sum())
    big = torch.tensor([int(max(send.max(), recv.max()))], dtype=torch.int64, device=cdev)
    dist.all_reduce(big, op=dist.ReduceOp.MAX, group=group)
    pieces = max(1, -(-int(big.item()) // MAX_MESSAGE))
    rk = torch.empty(n_recv, dtype=keys.dtype, device=dev)
    a2a(rk, pk, recv.tolist(), send.tolist(), pieces)
    rv = None
    if vals is not None:
        rv = torch.empty(n_recv, dtype=vals.dtype, device=dev)
        a2a(rv, pv, recv.tolist(), send.tolist(), pieces)

    # 7: local LSD sort of the received bucket
    ok, ov = ops.sort(rk, rv, k_bits)

    # global offset of this rank's slice = keys owned by lower ranks
    counts = torch.tensor([n_recv], dtype=torch.int64, device=cdev)
    allc = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(allc, counts, group=group)
    offset = int(sum(int(c.item()) for c in allc[:rank]))
    return ok, ov, offset
