"""Test double of the device side of the sharded framing protocol (mgen_amd/shard.py):
the same candidate rule and exit semantics as mgenx_scan.hip, written as plain Python over
bytes, so the host protocol can run on CPU under gloo.  Test infrastructure only.

Candidate rule (mgenx_scan.hip scan_detect_kernel): p + 4 <= n, byte p+2 == 2 (version),
L = be16(p) in [min, max] (TCP [4, 65535], SINK [MIN_SIZE 28, MAX_SIZE 8192]), p + L <= n.
Range rule: the reference framing loops (mgenTransport.cpp:1683-1760 TCP,
mgenAppSinkTransport.cpp:369-434 SINK) started at `entry`, stopping at the first position
>= limit."""
import numpy as np

from mgen_amd.shard import EXIT_CAP, NONE, UNKNOWN

SINK_MIN, SINK_MAX = 28, 8192


def _bounds(mode):
    return (SINK_MIN, SINK_MAX) if mode == 1 else (4, 65535)


def candidates(s: bytes, mode):
    lo, hi = _bounds(mode)
    n = len(s)
    out = []
    for p in range(0, max(n - 3, 0)):
        if s[p + 2] != 2:
            continue
        L = (s[p] << 8) | s[p + 1]
        if lo <= L <= hi and p + L <= n:
            out.append(p)
    return out


def walk(s: bytes, mode, entry, limit):
    """(offs, lens, consumed, status) of the reference rule from entry below limit."""
    n = len(s)
    lo, hi = _bounds(mode)
    p, offs, lens, status = entry, [], [], 0
    while True:
        if p >= limit or p + 2 > n:
            break
        L = (s[p] << 8) | s[p + 1]
        if mode == 1:
            if L < lo or L > hi:
                p += 2
                continue
        elif L < 4:
            status = 1
            break
        if p + L > n:
            break
        offs.append(p)
        lens.append(L)
        p += L
    return offs, lens, p, status


class RefScanner:
    def __init__(self, s: bytes):
        self.s = s

    def exits(self, local, mode, window, limit):
        s = self.s
        cs = candidates(s, mode)
        cset = set(cs)
        ent = np.full(EXIT_CAP, NONE, np.uint64)
        ext = np.full(EXIT_CAP, NONE, np.uint64)
        k = 0
        for c in cs:
            if c >= window or c >= limit or k >= EXIT_CAP:
                break
            p = c
            while True:
                nx = p + ((s[p] << 8) | s[p + 1])
                if nx >= limit:
                    e = nx
                    break
                if nx not in cset:
                    e = int(np.uint64(nx) | UNKNOWN)
                    break
                p = nx
            ent[k], ext[k] = c, e
            k += 1
        return np.stack([ent, ext])

    def range(self, local, mode, entry, limit, reuse):
        offs, lens, consumed, status = walk(self.s, mode, entry, limit)
        return (np.array(offs, np.int64), np.array(lens, np.int32), len(offs), consumed, status)
