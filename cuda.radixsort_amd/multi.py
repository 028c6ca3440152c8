"""Multi-GPU sort over torch.distributed: key-range partition with ONE exchange, then a local LSD sort.

No reference counterpart (the reference is single-GPU, Parallel7.cu:10/:697); this is BASELINE
config 5 / SURVEY §8e, the same protocol as the C ABI's rsort_u32_multi (rsort_multi.cpp), and it
takes every host-side decision from the same pure C planning functions (rsort_multi_sample_plan,
rsort_multi_splitters_make, rsort_multi_exchange_plan), so both paths split and place keys alike:

  1. all_gather of the key counts                      -> the sampling plan (one stride for all)
  2. a regular sample of the local keys (HIP), all_gather, sort (HIP) -> world-1 quantile KEYS
  3. splitters with an equal-keys bucket per hot quantile key: a run of equal keys --
     a hot key, duplicate-heavy input -- is split across ranks in (source rank, position) order
  4. stable partition into those buckets (HIP: rsort_partition_device)
  5. all_gather of the bucket counts and capacities    -> the exchange plan, the same on every
     rank (a capacity overflow raises on ALL ranks before any key moves)
  6. the exchange: own range by a device copy, every other message by all_to_all (RCCL over
     xGMI: grouped send/recv), in equal rounds of <= 2^28 keys per message
  7. local LSD sort of what arrived (HIP)

Rank r ends with the keys of global ranks [offset_r, offset_r + count_r); concatenating the
ranks' outputs in rank order gives exactly Baseline1's sorted array. Received chunks are placed
in source-rank order, so with values the whole sort stays stable.

The per-device steps go through an `ops` object: GpuOps (the product) calls librsort.so; the CPU
tests substitute a numpy restatement to exercise the distributed logic with gloo.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import radixsort as rs

# total sample budget over all ranks (rsort_multi.cpp kSampleBudget)
SAMPLE_BUDGET = 1 << 20
# keys per message of one exchange round (1 GiB of u32): the RCCL of this image (2.26, ROCm 7;
# torch 2.10) silently leaves the second half of an all_to_all message of >= 2 GiB unwritten
# (dev/a2a_lab.py: 1 GiB arrives whole, 2 GiB - 4 B does not)
MAX_PIECE = 1 << 28
NO_LIMIT = (1 << 62)


class GpuOps:
    """Per-rank steps on the local MI355X through the C ABI."""

    def __init__(self, device):
        self.device = device
        self._ws = None

    def _workspace(self, nbytes):
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = rs.workspace(nbytes, self.device)
        return self._ws

    def sample(self, keys, stride, count, row_len):
        return rs.sample_device(keys, stride, count, row_len)

    def sort_keys(self, keys):
        p = rs.plan(keys.numel(), 8, False)
        rs.sort_device(keys, keys, 8, ws=self._workspace(p.workspace_bytes), plan_=p)
        return keys

    def partition(self, keys, vals, splitters):
        n = keys.numel()
        nb = len(splitters) + 1
        ko = torch.empty_like(keys)
        vo = torch.empty_like(vals) if vals is not None else None
        starts = torch.empty(nb + 1, dtype=torch.int32, device=self.device)
        need = int(rs._lib().rsort_partition_workspace_size(n, nb, 1 if vals is not None else 0))
        rs.partition_device(keys, ko, splitters, starts, vals_in=vals, vals_out=vo, ws=self._workspace(need))
        return ko, vo, starts

    def sort(self, keys, vals, k_bits):
        """In place."""
        n = keys.numel()
        p = rs.plan(n, k_bits, vals is not None)
        rs.sort_device(keys, keys, k_bits, vals_in=vals, vals_out=vals, ws=self._workspace(p.workspace_bytes),
                       plan_=p)
        return keys, vals


def host_transport(group=None) -> "rs.HostTransport":
    """The C multi-GPU sort (rsort_u32_multi_transport) over a torch.distributed group whose
    collectives run on HOST tensors (gloo): rsort_host_transport_wrap stages the device bytes, these
    callbacks move them. For rehearsing the N-rank C protocol with several ranks on one card (RCCL
    refuses two ranks on one GPU) and in CPU-side tests; the product path on a node is RCCL."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)

    def allgather(send):
        t = torch.from_numpy(send)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return torch.cat(out).numpy().tobytes()

    def exchange(sends, recv_sizes):
        inp = torch.from_numpy(np.concatenate(sends) if sends else np.empty(0, np.uint8))
        out = torch.empty(sum(recv_sizes), dtype=torch.uint8)
        dist.all_to_all_single(out, inp, output_split_sizes=list(recv_sizes),
                               input_split_sizes=[int(x.size) for x in sends], group=group)
        o = out.numpy()
        offs = np.concatenate([[0], np.cumsum(recv_sizes)]).astype(np.int64)
        return [o[offs[p]:offs[p + 1]].tobytes() for p in range(world)]

    return rs.HostTransport(world, rank, allgather, exchange)


def exchange_rounds(max_message: int, limit: int) -> tuple[int, int]:
    """(rounds, piece) for messages of up to max_message keys, <= limit keys each: the C planning
    function rsort_multi_exchange_rounds (pieces a multiple of 64 keys, never above the limit)."""
    return rs.multi_exchange_rounds(max_message, limit)


def dist_sort(keys, k_bits=8, vals=None, ops=None, group=None, capacity=None):
    """Sort the union of every rank's `keys` (and `vals`); return this rank's slice of the
    global sorted order as (keys, vals, global_offset).

    Collectives run on the tensors' device with RCCL ("nccl"); with the gloo backend (tests:
    several ranks sharing one GPU, or CPU-only ranks) they run on host copies. capacity: the
    most keys this rank may receive (None: no limit); rs.RSortError(RSORT_ERR_CAPACITY) on every
    rank alike when any rank's limit would be exceeded."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if ops is None:
        ops = GpuOps(keys.device)
    dev = keys.device
    gloo = dist.get_backend(group) == "gloo"
    cdev = torch.device("cpu") if gloo else dev

    def all_gather(t):
        t = t.to(cdev)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return torch.stack(out)

    n = keys.numel()
    # 1. key counts -> sampling plan
    n_all = all_gather(torch.tensor([n], dtype=torch.int64)).cpu().numpy().reshape(-1)
    sp = rs.multi_sample_plan(n_all.tolist(), max(1, SAMPLE_BUDGET // world))

    # 2. sample, gather, sort: the quantile keys
    row = ops.sample(keys, sp.stride, sp.count[rank], sp.row_len)
    q = [0] * (world - 1)
    hot = None
    gathered = all_gather(row).reshape(-1)
    if world > 1 and sp.total > 0:
        srt = ops.sort_keys(gathered.to(dev))
        srt = srt.cpu().numpy().view(np.uint32)[:sp.total]  # (the rows' padding sorts after the samples)
        qpos = [rs.multi_quantile_index(sp, i) for i in range(1, world)]
        q = [int(srt[i]) for i in qpos]
        hot = rs.hot_flags(srt, qpos, world)
    spl = rs.multi_splitters(world, q, hot)

    # 3-4. stable partition into the splitters' buckets
    pk, pv, starts = ops.partition(keys, vals, spl.splitters)
    st = starts.to(torch.int64).cpu().numpy()
    cnt = (st[1:] - st[:-1]).astype(np.int64)
    cap = NO_LIMIT if capacity is None else int(capacity)

    # 5. count matrix + capacities -> the exchange plan (identical on every rank)
    rows = all_gather(torch.from_numpy(np.concatenate([cnt, [cap]]).astype(np.int64))).cpu().numpy()
    xp = rs.multi_exchange_plan(world, rank, rows[:, :-1], spl, rows[:, -1])

    # 6. the exchange into source-rank order (stability)
    send_off, send_cnt = list(xp.send_off)[:world], list(xp.send_cnt)[:world]
    recv_off, recv_cnt = list(xp.recv_off)[:world], list(xp.recv_cnt)[:world]
    rk = torch.empty(xp.n_recv, dtype=keys.dtype, device=dev)
    rv = torch.empty(xp.n_recv, dtype=vals.dtype, device=dev) if vals is not None else None
    rounds, piece = exchange_rounds(xp.max_message, MAX_PIECE)
    for src, dst in ((pk, rk), (pv, rv)):
        if src is None:
            continue
        if send_cnt[rank]:
            dst[recv_off[rank]:recv_off[rank] + recv_cnt[rank]].copy_(src[send_off[rank]:send_off[rank] + send_cnt[rank]])
        for rd in range(rounds):
            lo, hi = rd * piece, (rd + 1) * piece
            ins = [src[send_off[p] + min(lo, send_cnt[p]):send_off[p] + min(hi, send_cnt[p])] if p != rank
                   else src[:0] for p in range(world)]
            outs = [dst[recv_off[p] + min(lo, recv_cnt[p]):recv_off[p] + min(hi, recv_cnt[p])] if p != rank
                    else dst[:0] for p in range(world)]
            if not gloo:
                dist.all_to_all(outs, ins, group=group)  # RCCL: grouped send/recv of this round
                continue
            # gloo: one all_to_all_single of the round's pieces on host copies
            o = torch.empty(sum(int(x.numel()) for x in outs), dtype=dst.dtype)
            dist.all_to_all_single(o, torch.cat([x.cpu() for x in ins]),
                                   output_split_sizes=[int(x.numel()) for x in outs],
                                   input_split_sizes=[int(x.numel()) for x in ins], group=group)
            off = 0
            for x in outs:
                x.copy_(o[off:off + x.numel()])
                off += x.numel()

    # 7. local LSD sort of the received keys
    ok, ov = ops.sort(rk, rv, k_bits)
    return ok, ov, int(xp.offset)
