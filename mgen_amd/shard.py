"""Sharded stream framing (BASELINE config 5 over N GPUs): one TCP / SINK byte stream split
into contiguous byte ranges, one per rank, with no data-path collective.

The reference frames a socket sequentially (MgenTcpTransport::OnRecvMsg,
src/common/mgenTransport.cpp:1683-1760; MgenAppSinkTransport::OnInputReady,
src/common/mgenAppSinkTransport.cpp:369-434): record i+1 starts where record i ends, so a
rank cannot know where the chain enters its range without its predecessors.  The protocol
(include/mgenx.h, "sharded framing"):

  rank r owns records starting in [a_r, b_r) and holds bytes [a_r, min(b_r + HALO, N));
  1. mgenx_stream_scan_exits: for each candidate entry below a_r + HALO, the position where
     its chain first reaches b_r (or "unknown" when it leaves the candidate set);
  2. all-gather of those fixed-size tables (EXIT_CAP rows x 16 B per rank), then every rank
     stitches e_0 = 0, e_{r+1} = exit_r(e_r) identically; an entry missing from the table or
     an unknown exit is settled by that rank's sequential range scan and one more all-gather
     of 3 words (rare: bad version bytes, SINK garbage, TCP errors near a boundary);
  3. mgenx_stream_scan_range from e_r on the tables of step 1: the rank's records.
A final all-gather of (records, consumed, status) gives every rank the whole-stream summary
that mgenx_stream_scan would report.  Exact for every input: the tests compare the union
with the whole-stream scan (tests/test_gpu_scan.py single-GPU over simulated ranks,
tests/test_shard_cpu.py over gloo world 2).
"""
from __future__ import annotations

import threading

import numpy as np

from ._abi import SCAN_HALO

HALO = SCAN_HALO
EXIT_CAP = 4096                       # table rows exchanged per rank
UNKNOWN = np.uint64(1) << np.uint64(63)
NONE = np.uint64(0xFFFFFFFFFFFFFFFF)


def shard_bounds(nbytes: int, world: int, rank: int):
    """(a, b, hi): rank owns record starts in [a, b) and holds bytes [a, hi)."""
    a = nbytes * rank // world
    b = nbytes * (rank + 1) // world
    return a, b, min(b + HALO, nbytes)


def local_limit(nbytes, world, rank):
    a, b, hi = shard_bounds(nbytes, world, rank)
    return (hi - a) if rank == world - 1 else (b - a)


def stitch(tables, bounds, settled):
    """Entries of every rank from the gathered exit tables.  tables[r] = (2, EXIT_CAP)
    uint64 (local entry offsets, local exits | UNKNOWN bit); bounds[r] = (a, b);
    settled[r] = (exit_global, stopped) from a range scan.  Returns (entries, need):
    entries[r] = global entry position or None (the chain stopped before rank r);
    need = the first rank whose exit must be settled by a range scan, or None."""
    world = len(bounds)
    entries = [None] * world
    entries[0] = 0
    for r in range(world):
        e = entries[r]
        if e is None:
            break
        a, b = bounds[r]
        last = r == world - 1
        if r in settled:
            ex, stopped = settled[r]
            if stopped or last:
                break
        elif e >= b and not last:
            ex = e                          # a record spans the whole range
        elif last:
            break
        else:
            ent, exi = tables[r]
            k = int(np.searchsorted(ent, np.uint64(e - a)))
            if k >= len(ent) or int(ent[k]) != e - a or (exi[k] & UNKNOWN):
                return entries, r
            ex = a + int(exi[k])
        entries[r + 1] = ex
    return entries, None


class EngineScanner:
    """The device side of the protocol on one Engine (one context = one rank's tables)."""

    def __init__(self, eng):
        self.eng = eng

    def exits(self, local, mode, window, limit):
        ent, ext, _ = self.eng.stream_scan_exits(local, mode, window, limit, cap=EXIT_CAP)
        return np.stack([ent.cpu().numpy().view(np.uint64), ext.cpu().numpy().view(np.uint64)])

    def range(self, local, mode, entry, limit, reuse):
        offs, lens, info = self.eng.stream_scan_range(local, mode, entry, limit, reuse=reuse)
        return offs, lens, int(info.n_records), int(info.consumed), int(info.status)


class TorchComm:
    """all_gather of small int64 vectors over torch.distributed (gloo: CPU tensors; nccl =
    RCCL: device tensors)."""

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.device = device
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()

    def all_gather(self, arr: np.ndarray):
        torch = self.torch
        t = torch.from_numpy(np.ascontiguousarray(arr).view(np.int64).copy())
        if self.device is not None:
            t = t.to(self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().numpy().view(np.uint64).reshape(arr.shape) for o in out]


class ThreadComm:
    """all_gather among `world` threads of one process (simulated ranks on one GPU)."""

    def __init__(self, world):
        self.world = world
        self._bar = threading.Barrier(world)
        self._slots = [None] * world

    def rank_view(self, rank):
        parent = self

        class _V:
            world = parent.world

            def __init__(self):
                self.rank = rank

            def all_gather(self, arr):
                parent._slots[rank] = np.array(arr, copy=True)
                parent._bar.wait()
                out = list(parent._slots)
                parent._bar.wait()
                return out
        return _V()


def scan_sharded(scanner, comm, local, nbytes, mode):
    """Run the protocol on this rank.  local = this rank's bytes [a, hi) (device tensor for
    EngineScanner); nbytes = the whole stream's size.  Returns (rec_off, rec_len, summary):
    this rank's records with LOCAL offsets (add a = shard_bounds(...)[0] for global ones)
    and the whole-stream (n_records, consumed, status)."""
    world, rank = comm.world, comm.rank
    bounds = [shard_bounds(nbytes, world, r)[:2] for r in range(world)]
    a, b = bounds[rank]
    limit = local_limit(nbytes, world, rank)
    table = scanner.exits(local, mode, HALO, limit)
    tables = comm.all_gather(table)
    settled = {}
    mine = None
    while True:
        entries, need = stitch(tables, bounds, settled)
        if need is None:
            break
        msg = np.zeros(3, np.uint64)
        if rank == need:
            mine = scanner.range(local, mode, entries[rank] - a, limit, True)
            _, _, _, consumed, _ = mine
            stopped = consumed < limit or rank == world - 1
            msg[:] = (a + consumed, 1 if stopped else 0, 1)
        msgs = comm.all_gather(msg)
        settled[need] = (int(msgs[need][0]), bool(msgs[need][1]))
    e = entries[rank]
    if mine is None:
        if e is None or (e >= b and rank != world - 1):
            mine = (None, None, 0, (e - a) if e is not None else 0, 0)
        else:
            mine = scanner.range(local, mode, e - a, limit, True)
    offs, lens, n, consumed, status = mine
    summ = comm.all_gather(np.array([n, a + consumed, status, 1 if e is not None else 0],
                                    np.uint64))
    total = sum(int(s[0]) for s in summ)
    # the chain stops at the last rank it reached
    last = max(r for r in range(world) if int(summ[r][3]))
    return offs, lens, (total, int(summ[last][1]), int(summ[last][2]))
