#!/usr/bin/env python3
"""Benchmark: device-resident MgenMsg unpack (+ receive CRC-32 check) on MI355X.

Headline (BASELINE.json configs[1]): 1,048,576 pre-generated 1024-B UDP MgenMsg records
(flow = 1 + i mod 64, per-flow seq, tx = 1.7e9 s + i us, dst 127.0.0.1/5000, checksum on:
flags 0x0C), packed on the GPU by mgenx_pack_batch, resident in HBM.  One step = one
mgenx_unpack_batch over the whole batch (CRC-validating decode into 32-B mgenx_rec rows; the
SoA column layout is timed beside it in extra.columns_layout).

Algorithmic bytes per step: read 1,073,741,824 B of records + write
N x 32 B rows = 1,107,296,256 B.  The metric names pack and unpack: `value` is the unpack
(the receive path), `extra.pack_unpack_config2` the two together.  value = whole-job GB/s over all ranks (weak
scaling: each rank owns its own 1M-record slab; no data-path collective).

Extras (same JSON line, "extra"): header-only decode, pack (config 2), config 3 (mixed-size
pack + unpack with DATA payload), config 4 (per-flow analytics + the RCCL all-reduce of the
per-flow counters across ranks), config 5 (TCP stream scan + TCP-rule unpack), and the
PCIe-inclusive rate (pinned host slab -> H2D -> unpack -> columns D2H).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N > 1: launched by torch.distributed.run, one rank per GPU.)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_REC = 1 << 20
REC = 1024
ALGO_BYTES = N_REC * REC + N_REC * 32
PACK_BYTES = N_REC * REC + N_REC * 20   # records written + 20-B descriptors read
PEAK_HBM_GBPS = 8000.0   # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
ROUND = "r06"


def cpu_baseline(budget_s=6.0):
    """Oracle (C restatement, byte-table CRC as in mgenMsg.cpp:538-539) on the host cores of
    this box: the MgenUdpTransport receive path (Unpack + CRC check per record) over a
    bounded sample of the config-2 workload.  One thread (the reference's ProtoDispatcher
    is single-threaded) is the reported value; all available cores (one contiguous shard per
    thread) beside it.  Median of 5 timed runs each, after a warm-up run."""
    from oracle import oracle as O
    from mgen_amd.workloads import udp_fixed
    nproc = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    threads = max(1, min(avail, 16))   # the box's CPU share per GPU is 16
    n0 = 4096
    tmpl, pool, desc = udp_fixed(n0, REC)
    slab, _ = O.udp_pack_batch(tmpl, desc, pool, n0 * REC, stride=REC, checksum=True)

    def run(n_rec, sl, nt):
        t = time.perf_counter()
        f = O.udp_recv_batch(sl, n_rec, stride=REC, fixed_len=REC, nthreads=nt)
        dt = time.perf_counter() - t
        assert int(f["err"].sum()) == 0
        return dt
    run(n0, slab, 1)
    one = sorted(run(n0, slab, 1) for _ in range(5))[2]
    reps = max(1, int(budget_s / 10 / max(one, 1e-6)))   # ~budget_s / 2 for the 5 runs
    n1 = n0 * reps
    slab1 = np.tile(slab, reps)
    t1 = sorted(run(n1, slab1, 1) for _ in range(5))[2]
    nall = n0 * reps * threads // 4 if threads > 4 else n1
    slab_all = np.tile(slab, nall // n0)
    run(nall, slab_all, threads)
    tall = sorted(run(nall, slab_all, threads) for _ in range(5))[2]
    gbps1 = n1 * (REC + 32) / t1 / 1e9
    gbps_all = nall * (REC + 32) / tall / 1e9
    return {"value": round(gbps1, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{n1} x 1024-B checksummed UDP records of config 2 per run, oracle "
                      f"or_udp_recv (Unpack + CRC check), 1 thread, median of 5 "
                      f"({t1 * 1e3:.0f} ms each)",
            "mmsg_per_s": round(n1 / t1 / 1e6, 4),
            "nproc": nproc, "cores_available": avail,
            "all_cores": {"threads": threads, "value": round(gbps_all, 3), "unit": "GB/s",
                          "records": nall, "ms_median_of_5": round(tall * 1e3, 1),
                          "note": "threads = min(cores available, 16): a one-GPU box's CPU "
                                  "share is 16 (nproc counts the whole host)"},
            "configs": cpu_baseline_configs(threads)}


def _med5(fn):
    fn()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return sorted(ts)[2]


def cpu_baseline_configs(threads):
    """The oracle (C restatement, byte-table CRC as mgenMsg.cpp:538-539) on the configs the GPU
    extras run, 1 thread and `threads` threads, median of 5 each, on bounded samples:
      config 3: UDP send sequence (Pack + checksum, 16-B DATA payload, zero fill) and the
                receive path (Unpack + CRC check) over U{64..1472} records packed back to back;
      config 4: MgenAnalytic::Update over POISSON flows (1024 flows, 256-B messages);
      config 5: TCP framing (GetRxNumBytes / OnRecvMsg: sequential by construction) with
                Unpack + CRC per record, then the framed records' Unpack + CRC spread over
                the threads (framing stays one thread)."""
    from oracle import oracle as O
    from mgen_amd.workloads import poisson_flows, udp_mixed, make_templates
    out = {}
    # ---- config 3
    n = 131072
    tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64,
                                              payload_hex="00112233445566778899aabbccddeeff")
    total = int(offs[-1] + sizes[-1])
    pack_b, unpack_b = n * 20 + n * 16 + total, total + n * 32
    res = {}
    for nt in (1, threads):
        tp = _med5(lambda: O.udp_pack_batch_mt(tmpl, desc, pool, total, rec_off=offs, nthreads=nt))
        slab, _ = O.udp_pack_batch_mt(tmpl, desc, pool, total, rec_off=offs, nthreads=nt)
        tu = _med5(lambda: O.udp_recv_batch(slab, n, rec_off=offs, rec_len=sizes, nthreads=nt))
        res[nt] = {"pack_gbps": round(pack_b / tp / 1e9, 3), "unpack_gbps": round(unpack_b / tu / 1e9, 3),
                   "combined_gbps": round((pack_b + unpack_b) / (tp + tu) / 1e9, 3)}
    out["config3_pack_unpack"] = {"records": n, "bytes": total, "threads_1": res[1],
                                  f"threads_{threads}": res[threads]}
    # ---- config 4
    d = poisson_flows(1 << 20, 1024, mean_gap_us=1000)
    idx = (d["flow_id"] - 1).astype(np.uint32)
    nr = len(idx)
    res = {}
    for nt in (1, threads):
        t = _med5(lambda: O.flow_reduce_batch_mt(1024, idx, d["seq"], d["tx_sec"], d["tx_usec"],
                                                 d["msg_len"], d["rx_sec"], d["rx_usec"],
                                                 nthreads=nt))
        res[nt] = {"mrec_per_s": round(nr / t / 1e6, 2), "ms": round(t * 1e3, 1)}
    out["config4_flow_reduce"] = {"records": nr, "flows": 1024, "threads_1": res[1],
                                  f"threads_{threads}": res[threads]}
    # ---- config 5: 4096 x 16 KiB TCP records (checksum on), built by the oracle's TCP send path
    m = 4096
    tm, pl = make_templates(64)
    dsc = np.zeros(m, O.DESC_DTYPE)
    dsc["tmpl"] = np.arange(m) % 64
    dsc["seq_num"] = np.arange(m)
    dsc["tx_sec"] = 1_700_000_000
    dsc["tx_usec"] = np.arange(m)
    dsc["flags"] = 4
    stream = O.tcp_tx_batch(tm, dsc, np.full(m, 16384, np.uint32), pl, checksum=True)
    L = O.lib()
    P = ctypes.c_void_p
    st_offs = np.zeros(m + 1, np.uint64)
    st_lens = np.zeros(m + 1, np.uint32)
    fields = np.zeros(m + 1, O.FIELDS_DTYPE)
    cons, stat = ctypes.c_uint64(0), ctypes.c_int(0)

    def scan(cap):
        return L.or_tcp_scan(P(stream.ctypes.data), stream.size, 0, P(st_offs.ctypes.data),
                             P(st_lens.ctypes.data), P(fields.ctypes.data), cap,
                             ctypes.byref(cons), ctypes.byref(stat))
    assert scan(m + 1) == m and int(fields["err"][:m].sum()) == 0
    t1 = _med5(lambda: scan(m + 1))   # framing + Unpack + CRC, one thread (the reference)
    tf = _med5(lambda: scan(0))       # framing alone
    so, sl = st_offs[:m].copy(), st_lens[:m].copy()
    tu = _med5(lambda: O.udp_recv_batch(stream, m, rec_off=so, rec_len=sl, tcp=True,
                                        nthreads=threads))
    b = stream.size
    out["config5_tcp_scan_unpack"] = {
        "records": m, "bytes": int(b),
        "threads_1": {"gbps": round(b / t1 / 1e9, 3), "ms": round(t1 * 1e3, 1)},
        f"threads_{threads}": {"gbps": round(b / (tf + tu) / 1e9, 3),
                               "ms": round((tf + tu) * 1e3, 1),
                               "note": "framing on one thread, Unpack + CRC on all"}}
    return out


def load_traffic():
    """HBM bytes per launch of the headline kernel from the PMC passes of this round
    (FETCH_SIZE / WRITE_SIZE, calibrated; scripts/pmc.sh -> profiles/traffic_<round>.json).
    rocprofv3 counters cannot be collected inside this process, so the figure is read from
    that file and labelled with its source."""
    path = None
    for rnd in (ROUND, "r05", "r04", "r03"):   # this round's PMC passes, else the latest earlier
        p = os.path.join(ROOT, "profiles", f"traffic_{rnd}.json")
        if os.path.exists(p):
            path = p
            break
    if path is None:
        return None, None
    try:
        d = json.load(open(path))
        return d.get("unpack_crc_1M_x_1024B", {}).get("hbm_bytes_per_launch"), path
    except Exception:
        return None, None


def timed(torch, fn, reps=10, warm=3):
    """Mean time (ms) of fn() on the current stream, HIP events around reps calls, after
    `warm` untimed calls (an extra follows host-side input generation that leaves the GPU
    idle; its first launches run slow -- scripts/var_shapes.py's interleaved rounds show it)."""
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


# ------------------------------------------------------------------------ extras
def extra_config3(torch, eng, dev):
    """64 flows, sizes U{64..1472}, 16-B DATA payload, checksum on: pack + unpack."""
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd.workloads import udp_mixed
    n = N_REC
    tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64,
                                              payload_hex="00112233445566778899aabbccddeeff")
    total = int(offs[-1] + sizes[-1])
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    d_offs = to_device(offs).view(torch.int64)
    d_len = to_device(sizes).view(torch.int32)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    slab = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    cols = {"rows": eng.alloc_rows(n)}   # the product output layout (as the headline)
    pack = lambda: eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=d_offs,  # noqa
                            opts=PACK_CHECKSUM, out_len=out_len)
    unpack = lambda: eng.unpack(slab, n, rec_off=d_offs, rec_len=d_len, cols=cols)  # noqa
    pms, ums = timed(torch, pack), timed(torch, unpack)
    assert int(((cols["rows"].view(torch.int32).view(n, 8)[:, 6] >> 24) & 0xFF).sum()) == 0
    pack_b = n * 20 + n * 16 + total
    unpack_b = total + n * 32
    return {"records": n, "bytes": total, "output": "mgenx_rec rows (32 B)",
            "pack_ms": round(pms, 4), "unpack_ms": round(ums, 4),
            "pack_gbps": round(pack_b / pms / 1e6, 1), "unpack_gbps": round(unpack_b / ums / 1e6, 1),
            "combined_gbps": round((pack_b + unpack_b) / (pms + ums) / 1e6, 1)}


N4_TOTAL = 8 * N_REC   # config 4: 8,388,608 records in total at every N


def extra_config4(torch, eng, dev, world, rank, dist, rehearse=False):
    """1024 POISSON flows of 256-B messages, 8,388,608 records in total: rank r receives the
    records of the flows it owns (flow_id mod world == r), in receive order, and runs
    MgenAnalytic::Update over them (mgenx_flow_reduce: sort by flow, one wave per flow);
    the per-flow counters are exported and merged with ONE mgenx_allreduce_flows (RCCL) of
    1024 x 64 B.  Also timed: device FindFlow (mgenx_flow_lookup) over the rank's records."""
    from mgen_amd.workloads import poisson_flows
    n_flows = 1024
    d = poisson_flows(N4_TOTAL, n_flows, mean_gap_us=1000)
    own = (d["flow_id"] % world) == rank
    d = {k: np.ascontiguousarray(v[own]) for k, v in d.items()}
    n = int(own.sum())
    idx = (d["flow_id"] - 1).astype(np.uint32)   # synthetic flow ids are the global index
    t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
    t_idx = torch.from_numpy(idx).to(dev)
    state = {}

    def run():
        flows = eng.flow_init(n_flows, 1.0)
        state["flows"] = flows
        eng.flow_reduce(flows, n_flows, t_idx, t["seq"], t["tx_sec"], t["tx_usec"],
                        t["msg_len"], t["rx_sec"], t["rx_usec"], n=n)
    ms = timed(torch, run, reps=5)
    counters = eng.flow_export(state["flows"], n_flows)
    # FindFlow: (dst 127.0.0.1/5000, src 10.0.x.y/5001, flow id) -> dense index, per record
    src = torch.zeros(n, 20, dtype=torch.uint8, device=dev)
    fid = t["flow_id"]
    f64 = fid.to(torch.int64)
    src[:, 0], src[:, 1], src[:, 2], src[:, 3] = 1, 4, 0x89, 0x13
    src[:, 4], src[:, 6], src[:, 7] = 10, ((f64 >> 8) & 255).to(torch.uint8), (f64 & 255).to(torch.uint8)
    dst_addr = torch.zeros(n, 16, dtype=torch.uint8, device=dev)
    dst_addr[:, 0], dst_addr[:, 3] = 127, 1
    cols = {"dst_addr": dst_addr.reshape(-1), "flow_id": fid.view(torch.int32),
            "dst_len": torch.full((n,), 4, dtype=torch.uint8, device=dev),
            "dst_port": torch.full((n,), 5000, dtype=torch.int16, device=dev)}
    table = eng.flow_table(2 * n_flows)
    try:
        fidx, nf = eng.flow_lookup(table, cols, src.reshape(-1), n)
        torch.cuda.synchronize()
        assert int(nf.cpu()[0]) == len(np.unique(d["flow_id"]))
        lk_ms = timed(torch, lambda: eng.flow_lookup(table, cols, src.reshape(-1), n,
                                                     flow_idx=fidx, n_flows=nf), reps=5)
    finally:
        eng.flow_table_destroy(table)
    pipe = pipeline_config4(torch, eng, dev, d, idx, src, state["flows"], n_flows, n)
    # one rank's share at N = 8 (flows f with f mod 8 == 0: 128 flows, 1/8 of the records),
    # timed here at N = 1: the per-flow update does not shrink with N
    share8 = None
    if world == 1:
        own8 = (d["flow_id"] % 8) == 0
        t8 = {k: torch.from_numpy(np.ascontiguousarray(v[own8])).to(dev) for k, v in d.items()}
        i8 = torch.from_numpy(np.ascontiguousarray(idx[own8])).to(dev)
        n8 = int(own8.sum())

        def run8():
            f8 = eng.flow_init(n_flows, 1.0)
            eng.flow_reduce(f8, n_flows, i8, t8["seq"], t8["tx_sec"], t8["tx_usec"],
                            t8["msg_len"], t8["rx_sec"], t8["rx_usec"], n=n8)
        ms8 = timed(torch, run8, reps=5)
        share8 = {"records": n8, "flows": n_flows // 8, "reduce_ms": round(ms8, 4),
                  "mrec_per_s": round(n8 / ms8 / 1e3, 1),
                  "note": "rank 0's share of config 4 at N = 8, timed on one GPU"}
    ar_ms = None
    merge = "mgenx_allreduce_flows (RCCL ncclAllReduce sum, 1024 x 64 B)"
    if world > 1 and rehearse:
        # dry run: the same sum over gloo (ranks may share one GPU, which RCCL refuses)
        merge = "rehearsal: gloo all-reduce of the exported counters (not RCCL)"
        host = torch.from_numpy(counters.cpu().numpy().view(np.int64).copy())
        dist.all_reduce(host)
        ar_ms = None
    elif world > 1:
        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(eng.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        comm = eng.comm_init(world, rank, bytes(uid.cpu().numpy()))
        try:
            eng.allreduce_flows(comm, counters, n_flows)   # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                eng.allreduce_flows(comm, counters, n_flows)
            torch.cuda.synchronize()
            ar_ms = (time.perf_counter() - t0) / 20 * 1e3
        finally:
            eng.comm_destroy(comm)
    return {"records_total": N4_TOTAL, "records_this_rank": n, "flows": n_flows,
            "reduce_ms": round(ms, 4), "mrec_per_s": round(n / ms / 1e3, 2),
            "findflow_ms": round(lk_ms, 4), "findflow_mrec_per_s": round(n / lk_ms / 1e3, 1),
            "rows_pipeline": pipe, "rank_share_at_8": share8, "allreduce_bytes": n_flows * 64,
            "allreduce_ms": None if ar_ms is None else round(ar_ms, 4),
            "merge": merge}


def pipeline_config4(torch, eng, dev, d, idx, src, want_flows, n_flows, n):
    """The receive path of config 4 on the unpack's 32-B rows, no column layout: the rank's
    records as 256-B datagrams (GPU-packed), mgenx_unpack_batch -> rows, FindFlow keyed from
    the rows (mgenx_flow_lookup, cols.rows), MgenAnalytic::Update reading the rows
    (mgenx_flow_reduce_rows).  Checked: every flow's state equals the column path's
    (`want_flows`, flow ids are the global index there, first-appearance order here)."""
    from mgen_amd import DESC_DTYPE, FLOW_STATE_BYTES, to_device
    from mgen_amd.workloads import make_templates
    msg = 256
    tmpl, pool = make_templates(n_flows)
    desc = np.zeros(n, DESC_DTYPE)
    desc["tmpl"], desc["seq_num"] = idx, d["seq"]
    desc["tx_sec"], desc["tx_usec"], desc["msg_len"] = d["tx_sec"], d["tx_usec"], msg
    dt, dp = to_device(tmpl, eng.device), to_device(pool, eng.device)
    crc = torch.empty(n_flows, dtype=torch.int32, device=dev)
    eng.pack_prepare(dt, n_flows, dp, crc)
    slab = torch.empty(n * msg, dtype=torch.uint8, device=dev)
    eng.pack(dt, crc, to_device(desc, eng.device), n, dp, slab, stride=msg)
    rows = {"rows": eng.alloc_rows(n)}
    rx_s = torch.from_numpy(d["rx_sec"]).to(dev)
    rx_u = torch.from_numpy(d["rx_usec"]).to(dev)
    fidx = torch.empty(n, dtype=torch.int32, device=dev)
    nf = torch.zeros(1, dtype=torch.int32, device=dev)
    table = eng.flow_table(2 * n_flows)
    box = {}
    unpack = lambda: eng.unpack(slab, n, stride=msg, fixed_len=msg, cols=rows)  # noqa: E731
    lookup = lambda: eng.flow_lookup(table, rows, src.reshape(-1), n, flow_idx=fidx,  # noqa
                                     n_flows=nf)

    def reduce():
        box["flows"] = eng.flow_init(n_flows, 1.0)
        eng.flow_reduce_rows(box["flows"], n_flows, fidx, rows["rows"], rx_s, rx_u, n=n)

    def whole():
        unpack()
        lookup()
        reduce()
    try:
        whole()
        torch.cuda.synchronize()
        assert int(nf.cpu()[0]) == len(np.unique(d["flow_id"]))
        _, first = np.unique(d["flow_id"], return_index=True)
        order = d["flow_id"][np.sort(first)] - 1          # dense index -> global flow index
        got = box["flows"].cpu().numpy().reshape(n_flows, FLOW_STATE_BYTES)
        want = want_flows.cpu().numpy().reshape(n_flows, FLOW_STATE_BYTES)
        assert np.array_equal(got[:len(order)], want[order]), "rows pipeline != column path"
        u_ms, l_ms, r_ms = timed(torch, unpack, 5), timed(torch, lookup, 5), timed(torch, reduce, 5)
        w_ms = timed(torch, whole, 5)
    finally:
        eng.flow_table_destroy(table)
    return {"datagram_bytes": msg,
            "unpack": ("header-only decode: the datagrams carry no CHECKSUM flag, so Unpack "
                       "reads each record's 64-B header row and no CRC (algorithmic bytes "
                       "n x (64 read + 32 row written))"),
            "unpack_ms": round(u_ms, 4), "findflow_ms": round(l_ms, 4),
            "reduce_ms": round(r_ms, 4), "end_to_end_ms": round(w_ms, 4),
            "end_to_end_mrec_per_s": round(n / w_ms / 1e3, 1),
            "checked": "per-flow state == column-path state (bit-exact)"}


def extra_config5(torch, eng, dev, world=1, rank=0, dist=None, rehearse=False):
    """TCP stream of 16 KiB records (checksum on): boundary scan + TCP-rule unpack over
    1 GiB per rank, the stream built by the GPU TCP transmit path (mgenx_pack_tcp).
    N > 1: one stream of N GiB split into 1-GiB shards (+ 64 KiB halo) framed with the
    sharded protocol (mgen_amd/shard.py: exits table all-gather over RCCL, then the rank's
    range); weak scaling, time = max over ranks."""
    from mgen_amd import OPT_TCP, PACK_CHECKSUM, SCAN_TCP, to_device
    from mgen_amd._abi import DESC_DTYPE
    from mgen_amd.shard import HALO, EngineScanner, TorchComm, scan_sharded
    from mgen_amd.workloads import make_templates
    n = 65536                       # 16 KiB records per rank: 1 GiB
    extra_n = HALO // 16384 if rank < world - 1 else 0   # the next rank's first records
    tmpl, pool = make_templates(64)
    desc = np.zeros(n + extra_n, DESC_DTYPE)
    seq = rank * n + np.arange(n + extra_n)
    desc["tmpl"] = seq % 64
    desc["seq_num"] = seq
    desc["tx_sec"] = 1_700_000_000 + seq // 1_000_000
    desc["tx_usec"] = seq % 1_000_000
    desc["flags"] = 4
    tm, pl = to_device(tmpl, dev.index), to_device(pool, dev.index)
    tcrc = torch.empty(64, dtype=torch.int32, device=dev)
    eng.pack_prepare(tm, 64, pl, tcrc)
    d_desc = to_device(desc, dev.index)
    d_total = torch.full((n + extra_n,), 16384, dtype=torch.int32, device=dev)
    # the TCP transmit stream built on the GPU (mgenx_pack_tcp), timed
    local, toffs = eng.pack_tcp(tm, tcrc, d_desc, d_total, n + extra_n, pl, opts=PACK_CHECKSUM)
    tx_ms = timed(torch, lambda: eng.pack_tcp(tm, tcrc, d_desc, d_total, n + extra_n, pl,
                                              opts=PACK_CHECKSUM, out=local, offs=toffs), reps=3)
    shard = local[:n * 16384]
    total_bytes = shard.numel() * world
    state = {}
    if world > 1:
        comm = TorchComm(None if rehearse else dev)
        scanner = EngineScanner(eng)

        def scan():
            state["r"] = scan_sharded(scanner, comm, local, total_bytes, SCAN_TCP)
    else:
        scan_out = (torch.empty(n + 1, dtype=torch.int64, device=dev),
                    torch.empty(n + 1, dtype=torch.int32, device=dev))

        def scan():
            offs, lens, info = eng.stream_scan(local, SCAN_TCP, out=scan_out)
            state["r"] = (offs, lens, (int(info.n_records), int(info.consumed),
                                       int(info.status)))
    scan()
    reps = 20
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        scan()
    torch.cuda.synchronize()
    scan_ms = (time.perf_counter() - t0) / reps * 1e3
    if world > 1:
        t = torch.tensor([scan_ms], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        scan_ms = float(t.item())
    offs, lens, summ = state["r"]
    assert summ == (n * world, total_bytes, 0), summ
    assert offs.numel() == n and int(offs[0]) == 0
    cols = eng.alloc_cols(n)
    ums = timed(torch, lambda: eng.unpack(local, n, rec_off=offs, rec_len=lens, opts=OPT_TCP,
                                          cols=cols), reps=10)
    assert int((cols["err"] != 0).sum()) == 0
    b = shard.numel()
    return {"records_per_rank": n, "bytes_per_rank": b, "ranks": world,
            "scan_ms": round(scan_ms, 4),
            "scan_gbps_total": round(world * b / scan_ms / 1e6, 1),
            "scan_frac_of_peak_per_gpu": round(b / scan_ms / 1e6 / PEAK_HBM_GBPS, 4),
            "unpack_ms": round(ums, 4),
            "unpack_gbps": round((b + n * 32) / ums / 1e6, 1),
            "tcp_tx_ms": round(tx_ms, 4), "tcp_tx_gbps": round(b / tx_ms / 1e6, 1),
            "stream_source": "mgenx_pack_tcp (GPU TCP transmit, timed as tcp_tx_*)",
            "framing": "sharded (exits all-gather + range)" if world > 1 else "whole stream"}


def extra_log(torch, eng, dev, slab):
    """RECV event log lines (mgenx_log_recv_text) for the config-2 batch: the decoded records
    (rows + extended columns) formatted as the reference's text log, GPU-resident."""
    from mgen_amd._abi import COLS_EXT
    full = eng.alloc_cols(N_REC, ext=True)
    cols = {name: full[name] for name, _, _ in COLS_EXT}
    cols["rows"] = eng.alloc_rows(N_REC)
    eng.unpack(slab, N_REC, stride=REC, fixed_len=REC, cols=cols)
    src = torch.zeros(N_REC, 20, dtype=torch.uint8, device=dev)
    src[:, 0], src[:, 1], src[:, 2], src[:, 3] = 1, 4, 0x89, 0xE7    # IPv4 127.0.0.1/59273
    src[:, 4], src[:, 7] = 127, 1
    rx_s = torch.full((N_REC,), 1_700_000_001, dtype=torch.int32, device=dev)
    rx_u = torch.arange(N_REC, dtype=torch.int32, device=dev) % 1_000_000
    text, line_off = eng.log_recv_text(slab, N_REC, cols, src, rx_s, rx_u, stride=REC)
    cap = text.numel()
    ms = timed(torch, lambda: eng.log_recv_text(slab, N_REC, cols, src, rx_s, rx_u, stride=REC,
                                                text_cap=cap), reps=5)
    return {"records": N_REC, "text_bytes": cap, "ms": round(ms, 4),
            "mlines_per_s": round(N_REC / ms / 1e3, 1),
            "note": "two passes (length, write) + scan; includes one D2H read of the total"}


def extra_pcap(torch, eng, dev):
    """pcap2mgen (pcap2mgen.cpp:252-482, analytics on) over a device-resident capture of
    1,048,576 packets (Ethernet / IPv4 / UDP, 262-B checksummed MGEN messages, 1024 flows,
    1 us apart): frame parse, Unpack, FindFlow + Update, the analytic REPORT lines, the RECV
    lines, received REPORT items, per-packet interleave.  Host round trips between stages
    (flow count, text sizes) included; the capture file's H2D is not."""
    from mgen_amd.pcap import Pcap2Mgen
    from mgen_amd.workloads import pcap_capture
    n = N_REC
    buf, pkt_off, rec_bytes = pcap_capture(eng, n)
    p = Pcap2Mgen(eng, analytics=True, window=0.25)
    text, _ = p.run_device(buf, pkt_off, n, 1, 0)
    torch.cuda.synchronize()
    body = text.cpu().numpy().tobytes()
    assert body.count(b" RECV ") == n, body[:300]
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        p.run_device(buf, pkt_off, n, 1, 0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    return {"packets": n, "capture_bytes": buf.numel(), "log_bytes": len(body),
            "report_lines": body.count(b" REPORT "), "ms": round(ms, 3),
            "mpkt_per_s": round(n / ms / 1e3, 1),
            "capture_gbps": round(buf.numel() / ms / 1e6, 1),
            "note": "device-resident capture; whole pipeline incl. its host size round trips"}


def extra_convert(torch, eng, dev, slab):
    """ConvertBinaryLog (mgenMsg.cpp:1417-1900) of the binary RECV log of the config-2 batch
    (1,048,576 records written on the GPU by mgenx_log_recv_binary): host record walk
    (mgenx_binlog_index) and the device conversion timed separately."""
    import mgen_amd
    from mgen_amd._abi import COLS_EXT
    full = eng.alloc_cols(N_REC, ext=True)
    cols = {name: full[name] for name, _, _ in COLS_EXT}
    cols["rows"] = eng.alloc_rows(N_REC)
    eng.unpack(slab, N_REC, stride=REC, fixed_len=REC, cols=cols)
    src = torch.zeros(N_REC, 20, dtype=torch.uint8, device=dev)
    src[:, 0], src[:, 1], src[:, 2], src[:, 3] = 1, 4, 0x89, 0xE7
    src[:, 4], src[:, 7] = 127, 1
    rx_s = torch.full((N_REC,), 1_700_000_001, dtype=torch.int32, device=dev)
    rx_u = torch.arange(N_REC, dtype=torch.int32, device=dev) % 1_000_000
    binrec, _ = eng.log_recv_binary(slab, N_REC, cols, src, rx_s, rx_u, stride=REC)
    hdr = b"mgen version=5.1.1 type=binary_log\n\0"
    log = torch.cat([torch.tensor(list(hdr), dtype=torch.uint8, device=dev), binrec])
    host = log.cpu().numpy()
    t0 = time.perf_counter()
    offs, info = mgen_amd.binlog_index(host)
    idx_ms = (time.perf_counter() - t0) * 1e3
    assert info.status == 0 and info.n_records == N_REC
    ro = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    text, _ = eng.convert_binary_log(log, ro, N_REC)
    cap = text.numel()
    reps = 3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.convert_binary_log(log, ro, N_REC, cap=cap)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    return {"records": N_REC, "binary_bytes": log.numel(), "text_bytes": cap,
            "ms": round(ms, 3), "mrec_per_s": round(N_REC / ms / 1e3, 1),
            "host_index_ms": round(idx_ms, 3),
            "note": "device conversion incl. its host size round trips; host index separate"}


def extra_pcie(torch, eng, dev, slab):
    """Config 2 from pinned host memory: 8 chunks of 128 MiB, two streams (copy of chunk
    k+1 overlaps the unpack of chunk k), core columns copied back.  Wall-clock GB/s of
    record bytes: the rate of a path that starts and ends in host memory."""
    host = torch.empty(slab.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(slab)
    chunks = 8
    per = N_REC // chunks
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    dbuf = [torch.empty(per * REC, dtype=torch.uint8, device=dev) for _ in range(2)]
    cols = [{"rows": eng.alloc_rows(per)} for _ in range(2)]
    hcols = [{k: torch.empty(v.numel(), dtype=v.dtype, pin_memory=True) for k, v in c.items()}
             for c in cols]

    def run():
        for c in range(chunks):
            j = c % 2
            with torch.cuda.stream(streams[j]):
                dbuf[j].copy_(host[c * per * REC:(c + 1) * per * REC], non_blocking=True)
                eng.unpack(dbuf[j], per, stride=REC, fixed_len=REC, cols=cols[j])
                for k, v in cols[j].items():
                    hcols[j][k].copy_(v, non_blocking=True)
        torch.cuda.synchronize()
    run()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    err = (hcols[0]["rows"].view(torch.int32).view(per, 8)[:, 6] >> 24) & 0xFF
    assert int((err != 0).sum()) == 0
    return {"gbps": round(N_REC * REC / dt / 1e9, 2), "ms": round(dt * 1e3, 3),
            "chunks": chunks, "note": "pinned H2D + unpack + 32-B rows D2H, 2 streams"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    args = ap.parse_args()

    # MGENX_BENCH_REHEARSE=1: the N-rank protocol on however many GPUs are visible (ranks
    # share them), torch.distributed over gloo, the RCCL counter merge replaced by a gloo
    # all-reduce -- a dry run of every collective's order on a one-GPU box; its numbers
    # mean nothing
    rehearse = os.environ.get("MGENX_BENCH_REHEARSE") == "1"
    from mgen_amd import launch
    if launch.needs_launch(args.gpus):
        # `python bench.py --gpus N` outside torch.distributed.run: start the N ranks as a
        # child launcher before anything touches the GPU; rank 0 prints the line
        sys.exit(launch.relaunch(__file__, sys.argv[1:], args.gpus, check_gpus=not rehearse))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")
    # collectives of host-side values: device tensors over RCCL, CPU tensors over gloo
    cdev = torch.device("cpu") if rehearse else dev

    from mgen_amd import OPT_SKIP_CRC, PACK_CHECKSUM, UNPACK_K_FIXED_RING, Engine, to_device
    from mgen_amd.workloads import udp_fixed

    eng = Engine(local)
    tmpl, pool, desc = udp_fixed(N_REC, REC)
    d_tmpl, d_pool, d_desc = (to_device(a, local) for a in (tmpl, pool, desc))
    tcrc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, tcrc)
    slab = torch.empty(N_REC * REC, dtype=torch.uint8, device=dev)
    out_len = torch.empty(N_REC, dtype=torch.int32, device=dev)

    def do_pack():
        eng.pack(d_tmpl, tcrc, d_desc, N_REC, d_pool, slab, stride=REC, opts=PACK_CHECKSUM,
                 out_len=out_len)

    do_pack()
    torch.cuda.synchronize()
    # Headline output layout: mgenx_rec rows (the 32-B core record, written as whole lines --
    # 512 contiguous bytes per wave store).  The SoA column layout carries the same 32 B per
    # record in 14 arrays of 1-4 B elements and is timed beside it (extra.columns_layout).
    rows = eng.alloc_rows(N_REC)
    cols = {"rows": rows}
    cs = eng._cols_struct(cols)
    lib, ctx = eng.lib, eng.ctx
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    slab_p = ctypes.c_void_p(slab.data_ptr())

    def step(opts=0):
        rc = lib.mgenx_unpack_batch(ctx, slab_p, slab.numel(), None, REC, None, REC, N_REC,
                                    ctypes.byref(cs), opts, stream)
        if rc != 0:
            raise RuntimeError(f"mgenx_unpack_batch rc={rc}")

    def rows_ok():
        r = rows.view(torch.int32).view(N_REC, 8)
        err = (r[:, 6] >> 24) & 0xFF            # mgenx_rec.err
        seq = r[:, 1]                           # mgenx_rec.seq_num
        want = torch.arange(N_REC, device=dev, dtype=torch.int32) // 64
        return int((err != 0).sum()) == 0 and bool(torch.equal(seq, want))

    # correctness gate before timing
    step()
    torch.cuda.synchronize()
    if not rows_ok() or int((out_len != REC).sum()):
        raise RuntimeError("unpack found bad records in a freshly packed slab")

    which = eng.last_unpack_kernel()      # the kernel the timed steps launch
    kernel_name = {UNPACK_K_FIXED_RING: "mgenx::unpack_fixed_ring_kernel<16, 4, 16>"}.get(
        which, f"UNPACK_K_{which} (not the ring kernel)")
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-launch kernel duration with HIP events on the launch stream
    n_ev = max(10, min(args.steps, 50))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(n_ev)]
    for a, b in evs:
        a.record()
        step()
        b.record()
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))

    hdr_ms = timed(torch, lambda: step(OPT_SKIP_CRC), reps=20)
    pack_ms = timed(torch, do_pack, reps=20)
    step()
    torch.cuda.synchronize()
    assert rows_ok()
    # the same decode into the 14 SoA core columns
    ccols = eng.alloc_cols(N_REC)
    col_ms = timed(torch, lambda: eng.unpack(slab, N_REC, stride=REC, fixed_len=REC,
                                             cols=ccols), reps=20)
    assert int((ccols["err"] != 0).sum()) == 0
    # memory-system probes on this box: the unpack's read pattern alone, and with 512-B
    # row stores per 16-KiB group (mgenx_diag_group_rw)
    probe_out = torch.empty(N_REC * 32, dtype=torch.uint8, device=dev)
    probe = Engine(local, diag=True)   # libmgenx_diag.so: the memory-pattern probes
    rd_ms = timed(torch, lambda: probe.group_rw(slab, probe_out, 0), reps=20)
    rw_ms = timed(torch, lambda: probe.group_rw(slab, probe_out, 1), reps=20)
    probe.close()
    del probe_out, ccols

    extra = {"columns_layout": {"unpack_ms": round(col_ms, 4),
                                "gbps": round(ALGO_BYTES / (col_ms * 1e-3) / 1e9, 1)},
             "probe_read_pattern_gbps": round(N_REC * REC / (rd_ms * 1e-3) / 1e9, 1),
             "probe_read_plus_row_stores_gbps": round(ALGO_BYTES / (rw_ms * 1e-3) / 1e9, 1),
             "header_only_unpack_ms": round(hdr_ms, 4),
             "header_only_mmsg_per_s": round(N_REC / (hdr_ms * 1e-3) / 1e6, 1),
             "pack_ms": round(pack_ms, 4),
             "pack_gbps": round(PACK_BYTES / (pack_ms * 1e-3) / 1e9, 1),
             # the metric's "pack+unpack": one pack of the batch and one unpack of it
             "pack_unpack_config2": {
                 "gbps": round((PACK_BYTES + ALGO_BYTES) / ((pack_ms + kern_ms) * 1e-3) / 1e9, 1),
                 "ms": round(pack_ms + kern_ms, 4),
                 "frac_of_peak": round((PACK_BYTES + ALGO_BYTES) / ((pack_ms + kern_ms) * 1e-3)
                                       / 1e9 / PEAK_HBM_GBPS, 4),
                 "bytes": PACK_BYTES + ALGO_BYTES,
                 "note": "pack: 1 GiB written + 20-B descriptors read; unpack: 1 GiB read + rows"}}
    if not args.no_extras:
        def guard(name, fn):
            try:
                extra[name] = fn()
            except Exception as e:  # an extra never hides the headline line
                extra[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
        # configs 4 and 5 on every rank (they have collectives); the rest on rank 0 only
        guard("config4_flow_reduce",
              lambda: extra_config4(torch, eng, dev, world, rank, dist, rehearse))
        guard("config5_tcp_scan_unpack",
              lambda: extra_config5(torch, eng, dev, world, rank, dist, rehearse))
        if rank == 0:
            guard("config3_mixed_pack_unpack", lambda: extra_config3(torch, eng, dev))
            guard("pcie_inclusive_config2", lambda: extra_pcie(torch, eng, dev, slab))
            guard("recv_log_text", lambda: extra_log(torch, eng, dev, slab))
            guard("pcap2mgen_1M_packets", lambda: extra_pcap(torch, eng, dev))
            guard("convert_binary_log_1M", lambda: extra_convert(torch, eng, dev, slab))

    traffic_b, traffic_src = load_traffic()
    ms_per_step = elapsed / args.steps * 1e3
    value = world * ALGO_BYTES * args.steps / elapsed / 1e9
    achieved = ALGO_BYTES / (kern_ms * 1e-3) / 1e9
    if rank == 0:
        line = {
            "metric": "device-resident MgenMsg pack+unpack GB/s and Mmsg/s at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (GPU-packed MgenMsg records, reference Pack semantics)",
            "config": {"workload": "udp_unpack_crc_1M_x_1024B",
                       "value_is": "unpack + receive CRC check of config 2 (pack: extra.pack_*)",
                       "records_per_gpu": N_REC,
                       "record_bytes": REC, "checksum": True, "output": "mgenx_rec rows (32 B)",
                       "algorithmic_bytes_per_step_per_gpu": ALGO_BYTES,
                       "parallelism": f"flow-sharded x{world} (independent slabs)",
                       **({"rehearsal": "ranks share GPUs over gloo: numbers invalid"}
                          if rehearse else {})},
            "mmsg_per_s": round(world * N_REC * args.steps / elapsed / 1e6, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS,
                         "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 4),
                         "traffic": traffic_b,
                         "traffic_source": traffic_src and os.path.relpath(traffic_src, ROOT),
                         "kernel": kernel_name,
                         "kernel_ms": round(kern_ms, 4)},
            "extra": extra,
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
