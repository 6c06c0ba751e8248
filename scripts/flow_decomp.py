#!/usr/bin/env python3
"""CPU model of the window-parallel MgenAnalytic::Update (mgenAnalytic.cpp:74-258) that
mgenx_analytic.hip's skeleton / window / sum kernels implement, checked against the oracle's
record-by-record restatement (or_flow_reduce_batch).  Not product code: it validates the
decomposition before the HIP kernels are changed.

The decomposition:
  skeleton (sequential per flow, scalar state only): window closes depend on receive times
    alone; the mask's span (first, last) and seq_start evolve without its bit contents (an
    out-of-span Set fails whatever the bits hold: a failed Set in the counted branch clears the
    mask to {seq}, an "epoch start").  Per record: flags; per window: its records, the epoch
    its first record lies in, seqMax and seq_start at the close.
  window (independent per window): the duplicate test of a record = an earlier record of the
    same epoch set the same sequence number (within an epoch every set index lies in one
    1024-wide span, so seq mod 1024 is a perfect hash); then the counters of the window.
  sum (per flow, a lane per window): each window's in-order FP64 latency sum.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

INS, DUPT, CE, ESTART, FA, INIT0, CLOSE = 1, 2, 4, 8, 16, 32, 64
M32 = 0xFFFFFFFF


def i32(x):
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def tadd(t, w):  # ProtoTime += double (the oracle's time_add)
    import math
    whole = math.floor(w)
    us = int((w - whole) * 1.0e06 + 0.5)
    s, u = t[0] + int(whole), t[1] + us
    while u >= 1000000:
        u -= 1000000
        s += 1
    return (s, u)


def tdelta(a, b):
    return float(a[0] - b[0]) + 1.0e-06 * float(a[1] - b[1])


def skeleton(recs, st, chunk=64):
    """recs: list of (seq, len, rx(sec,usec), lat).  st: dict state (modified).  Returns
    (flags per record, windows).  Chunked like the kernel: a chunk's plain records take their
    span test from inclusive prefix min / max of seq - F; the first record that fails it,
    closes, or needs the special paths is done alone, then the chunk resumes after it."""
    n = len(recs)
    flags = [0] * n
    wins = []
    win_a, win_r = 0, -1          # -1: the call's initial epoch
    cur_estart = -1
    valid, hasm = st["valid"], st["hasmask"]
    F, L, sst = st["first"], st["last"], st["seq_start"]
    ws, we = st["ws"], st["we"]
    W = st["window"]
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        pos = c0
        while pos < c1:
            # plain run from pos: inclusive span test against the running (F, L)
            ev = c1
            mn, mx = 0, i32(L - F)
            for j in range(pos, c1):
                seq, ln, rx, _ = recs[j]
                special = (not valid) or (ln != 0 and not hasm)
                closeh = valid and rx >= we
                fail = False
                if valid and hasm and ln != 0:
                    r = i32(seq - F)
                    mn2, mx2 = min(mn, r), max(mx, r)
                    fail = (mx2 - mn2) >= 1024
                if special or closeh or fail:
                    ev = j
                    break
                if ln != 0:
                    mn, mx = mn2, mx2
                    flags[j] = INS | DUPT | (CE if i32(seq - sst) >= 0 else 0)
            # commit the plain run
            if ev > pos and hasm:
                F2 = (F + mn) & M32
                L = (F + mx) & M32
                F = F2
            if ev >= c1:
                break
            seq, ln, rx, _ = recs[ev]
            fl = 0
            if not valid:
                valid = True
                ws, we = rx, tadd(rx, W)
                if ln != 0:
                    hasm = True
                    F = L = seq
                    sst = seq
                    fl = ESTART | FA | INS
                    cur_estart = ev
                else:
                    fl = INIT0
                flags[ev] = fl
                pos = ev + 1
                continue
            if ln != 0:
                if not hasm:
                    hasm = True
                    F = L = seq
                    sst = seq
                    fl = ESTART | FA | INS
                    cur_estart = ev
                else:
                    r = i32(seq - F)
                    mn2, mx2 = min(0, r), max(i32(L - F), r)
                    if mx2 - mn2 < 1024:
                        fl = INS | DUPT | (CE if i32(seq - sst) >= 0 else 0)
                        F2 = (F + mn2) & M32
                        L = (F + mx2) & M32
                        F = F2
                    elif i32(seq - sst) >= 0:
                        F = L = seq
                        fl = ESTART | INS | CE
                        cur_estart = ev
                    else:
                        fl = 0
            if rx >= we:
                seqmax = L if hasm else sst
                wins.append(dict(a=win_a, c=ev, r=win_r, zr=bool(fl & FA), seqmax=seqmax,
                                 sst=sst, ws=ws, rx=rx))
                sst = seqmax
                ws, we = rx, tadd(rx, W)
                win_a, win_r = ev + 1, cur_estart
                fl |= CLOSE
            flags[ev] = fl
            pos = ev + 1
    wins.append(dict(a=win_a, c=n, r=win_r, open=True, ws=ws))
    st.update(valid=valid, hasmask=hasm, first=F, last=L, seq_start=sst, ws=ws, we=we)
    return flags, wins


def window_pass(recs, flags, w, st0, init_bits):
    """One window: dups through the epoch table, counters, lat' per record, the report."""
    table = {}

    def insert(j, pos):
        h = recs[j][0] & 1023
        if h not in table or pos < table[h]:
            table[h] = pos
    if w["r"] < 0:
        for s in init_bits:
            table[s & 1023] = 0
        start = 0
    else:
        start = w["r"]
    for j in range(start, w["a"]):
        if flags[j] & ESTART:
            table.clear()
        if flags[j] & INS:
            insert(j, j + 1)

    def is_dup(j):
        return bool(flags[j] & DUPT) and table.get(recs[j][0] & 1023, 1 << 62) < j + 1
    # entering state
    if w["a"] == 0:
        mc, bc, lmin, lmax = st0["mc"], st0["bc"], st0["lmin"], st0["lmax"]
    else:
        c = w["a"] - 1
        seq, ln, rx, lat = recs[c]
        counted = bool(flags[c] & CE) and not is_dup(c)
        mc = 1 if ln else 0
        bc = 0
        lmin = lmax = (lat if counted else 0.0) if ln else 0.0
    dups = 0
    latp = {}
    k, s1, ssum = 0, None, 0
    cmin, cmax = None, None
    end = w["c"] + 1 if not w.get("open") else w["c"]
    for j in range(w["a"], end):
        seq, ln, rx, lat = recs[j]
        fl = flags[j]
        if fl & ESTART:
            table.clear()
        d = is_dup(j)
        if fl & INS:
            insert(j, j + 1)
        if d:
            dups += 1
        counted = bool(fl & CE) and not d and ln != 0
        if fl & FA:
            mc, bc, lmin, lmax = 1, ln, lat, lat
            latp[j] = lat
        elif fl & INIT0:
            mc, bc, lmin, lmax = 0, 0, 0.0, 0.0
            latp[j] = 0.0
        elif counted:
            latp[j] = lat
            k += 1
            if s1 is None:
                s1 = ln
            ssum += ln
            cmin = lat if cmin is None else min(cmin, lat)
            cmax = lat if cmax is None else max(cmax, lat)
        else:
            latp[j] = 0.0
    # fold the counted records into the entering state (FA / INIT0 precede every counted one)
    if k:
        if mc >= 2:
            bc = bc + ssum
        elif mc == 1:
            bc = ssum
        else:
            bc = s1 if k == 1 else ssum - s1
        if mc == 0:
            lmin, lmax = cmin, cmax
        else:
            lmin, lmax = min(lmin, cmin), max(lmax, cmax)
        mc += k
    out = dict(mc=mc, bc=bc, lmin=lmin, lmax=lmax, dups=dups, latp=latp, table=table)
    if not w.get("open"):
        rx = w["rx"]
        dur = tdelta(rx, w["ws"])
        if mc == 0:
            rep = (0, 0.0, 1.0, -1.0, -1.0)
        elif mc == 1:
            rep = (1, bc / dur, 0.0, lmin, lmax)
        else:
            delta = (w["seqmax"] - w["sst"]) & M32
            loss = 0.0 if delta <= 1 else 1.0 - mc / float((delta + 1) & M32)
            rep = (mc - 1, bc / dur, loss, lmin, lmax)
        out["report"] = dict(start=w["ws"], duration=dur, count=rep[0], rate=rep[1],
                             loss=rep[2], lmin=rep[3], lmax=rep[4], rx=rx, mc=mc)
    return out


def reduce_flow(recs, st):
    """One call's records of one flow from state st (dict).  Returns reports (with
    latency_ave) and updates st."""
    st0 = dict(mc=st["mc"], bc=st["bc"], lmin=st["lmin"], lmax=st["lmax"])
    init_bits = list(st["bits"])
    lsum0 = st["lsum"]
    flags, wins = skeleton(recs, st)
    outs = [window_pass(recs, flags, w, st0, init_bits) for w in wins]
    latp = {}
    for o in outs:
        latp.update(o["latp"])
    reps = []
    # sums: window t covers (close_{t-1} (+1 if zr), close_t]; window 0 from lsum0
    for t, (w, o) in enumerate(zip(wins, outs)):
        if t == 0:
            s, lo = lsum0, 0
        else:
            pw = wins[t - 1]
            s, lo = 0.0, pw["c"] + (1 if pw["zr"] else 0)
        hi = w["c"] if not w.get("open") else len(recs) - 1
        for j in range(lo, hi + 1):
            s = s + latp[j]
        if w.get("open"):
            st["lsum"] = s
        else:
            r = o["report"]
            r["lat_ave"] = -1.0 if r["mc"] == 0 else (s if r["mc"] == 1 else s / r["mc"])
            reps.append(r)
    last = outs[-1]
    st.update(mc=last["mc"], bc=last["bc"], lmin=last["lmin"], lmax=last["lmax"])
    st["dups"] += sum(o["dups"] for o in outs)
    st["nrep"] += len(wins) - 1
    if st["hasmask"]:
        F = st["first"]
        st["bits"] = {(F + ((h - F) & 1023)) & M32 for h in last["table"]}
    return reps


def fresh_state(window):
    from oracle import oracle as O
    return dict(valid=False, hasmask=False, first=0, last=0, seq_start=0, ws=(0, 0),
                we=(0, 0), window=O.quantized_window(window), mc=0, bc=0, lmin=0.0,
                lmax=0.0, lsum=0.0, dups=0, nrep=0, bits=set())


def check(d, n_flows, window, per_flow, splits=(0,)):
    from oracle import oracle as O
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    n = len(d["seq"])
    lat = (d["rx_sec"].astype(np.float64) - d["tx_sec"]) + 1.0e-06 * (
        d["rx_usec"].astype(np.float64) - d["tx_usec"])
    states = [fresh_state(window) for _ in range(n_flows)]
    reports = [[] for _ in range(n_flows)]
    bounds = list(splits) + [n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        fid = d["flow_id"][a:b] - 1
        for f in range(n_flows):
            ix = np.nonzero(fid == f)[0] + a
            if not len(ix):
                continue
            recs = [(int(d["seq"][i]), int(d["msg_len"][i]),
                     (int(d["rx_sec"][i]), int(d["rx_usec"][i])), float(lat[i])) for i in ix]
            reports[f] += reduce_flow(recs, states[f])
    bad = 0
    for f in range(n_flows):
        a, s = of[f], states[f]
        got = (s["mc"], s["bc"], s["dups"], s["nrep"], s["seq_start"], s["lsum"], s["lmin"],
               s["lmax"], s["ws"], s["we"], len(s["bits"]) if s["hasmask"] else 0)
        want = (a.msg_count, a.byte_count, a.dup_msg_count, a.n_reports, a.seq_start,
                a.latency_sum, a.latency_min, a.latency_max,
                (a.window_start.sec, a.window_start.usec), (a.window_end.sec, a.window_end.usec),
                a.nset)
        if got != want:
            bad += 1
            if bad < 4:
                print("state", f, got, want)
            continue
        if a.nset:
            wb = {(a.first + i) & M32 for i in range(1024) if (a.bits[i >> 3] >> (i & 7)) & 1}
            if wb != s["bits"] or a.first != s["first"]:
                bad += 1
                print("mask", f)
                continue
        k = min(int(ocnt[f]), per_flow)
        for r in range(k):
            o, g = orep[f, r], reports[f][r]
            gw = (g["start"][0], g["start"][1], g["duration"], g["count"], g["rate"], g["loss"],
                  g["lat_ave"], g["lmin"], g["lmax"], g["rx"][0], g["rx"][1])
            ww = (o["start_sec"], o["start_usec"], o["duration"], o["msg_count"], o["rate"],
                  o["loss"], o["latency_ave"], o["latency_min"], o["latency_max"], o["rx_sec"],
                  o["rx_usec"])
            if tuple(gw) != tuple(ww):
                bad += 1
                if bad < 4:
                    print("report", f, r, gw, ww)
                break
    return bad


def main():
    from mgen_amd.workloads import poisson_flows
    from test_gpu_analytics import _jumpy_flows, _mixed_lengths
    cases = [
        ("poisson 64", poisson_flows(60_000, 64, mean_gap_us=1000, seed=64), 64, 0.25, 32, (0,)),
        ("poisson lossy", poisson_flows(40_000, 48, mean_gap_us=500, seed=5, loss=0.05,
                                        dup=0.01, reorder=30), 48, 0.1, 16, (0, 1, 777, 20_000)),
        ("jumpy 0.02", _jumpy_flows(12, 3000, seed=23), 12, 0.02, 64, (0, 5000)),
        ("jumpy 0.5", _jumpy_flows(12, 3000, seed=503), 12, 0.5, 64, (0, 5000)),
        ("jumpy 30", _jumpy_flows(12, 3000, seed=30003), 12, 30.0, 64, (0, 5000)),
        ("mixed 0.001", _mixed_lengths(), 8, 0.001, 4096, (0, 30000)),
        ("mixed 0.3", _mixed_lengths(), 8, 0.3, 4096, (0, 30000)),
    ]
    tot = 0
    for name, d, nf, w, pf, sp in cases:
        bad = check(d, nf, w, pf, sp)
        print(f"{name}: {len(d['seq'])} records, {'OK' if not bad else f'{bad} BAD'}", flush=True)
        tot += bad
    sys.exit(1 if tot else 0)


if __name__ == "__main__":
    main()
