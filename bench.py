#!/usr/bin/env python3
"""Benchmark: device-resident MgenMsg unpack (+ receive CRC-32 check) on MI355X.

Workload (BASELINE.json configs[1]): 1,048,576 pre-generated 1024-B UDP MgenMsg records
(flow = 1 + i mod 64, per-flow seq, tx = 1.7e9 s + i us, dst 127.0.0.1/5000, checksum
on: flags 0x0C), packed on the GPU by mgenx_pack_batch, resident in HBM.  One step =
one mgenx_unpack_batch over the whole batch (CRC-validating decode into SoA columns).

Algorithmic bytes per step: read 1,073,741,824 B of records + write
N x 32 B core columns = 1,107,296,256 B.  value = whole-job GB/s over all ranks (weak
scaling: each rank owns its own 1M-record slab; no data-path collective).

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
PEAK_HBM_GBPS = 8000.0   # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
ROUND = "r01"


def cpu_baseline(budget_s=8.0):
    """Oracle (C restatement, byte-table CRC as in mgenMsg.cpp:538-539) on host cores:
    MgenUdpTransport receive path = Unpack + CRC check per record, single thread."""
    from oracle import oracle as O
    from mgen_amd.workloads import udp_fixed
    # pack a sample with the oracle itself (CPU-side inputs for the CPU baseline)
    n0 = 4096
    tmpl, pool, desc = udp_fixed(n0, REC)
    slab, _ = O.udp_pack_batch(tmpl, desc, pool, n0 * REC, stride=REC, checksum=True)
    t = time.perf_counter()
    O.udp_recv_batch(slab, n0, stride=REC, fixed_len=REC, nthreads=1)
    dt = time.perf_counter() - t
    reps = max(1, int(budget_s / max(dt, 1e-6)))
    reps = min(reps, 400)
    t = time.perf_counter()
    for _ in range(reps):
        f = O.udp_recv_batch(slab, n0, stride=REC, fixed_len=REC, nthreads=1)
    dt = time.perf_counter() - t
    assert int(f["err"].sum()) == 0
    n = n0 * reps
    gbps = n * (REC + 32) / dt / 1e9
    return {"value": round(gbps, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{n} x 1024-B checksummed UDP records ({reps} passes over a "
                      f"{n0}-record slab), oracle or_udp_recv, 1 thread, {dt:.1f} s",
            "mmsg_per_s": round(n / dt / 1e6, 4)}


def load_traffic():
    path = os.path.join(ROOT, "profiles", f"traffic_{ROUND}.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get("unpack_crc_1M_x_1024B", {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    from mgen_amd import PACK_CHECKSUM, OPT_SKIP_CRC, Engine, MgenxCols, to_device
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
    cols = eng.alloc_cols(N_REC)
    cs = eng._cols_struct(cols)
    lib, ctx = eng.lib, eng.ctx
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    slab_p = ctypes.c_void_p(slab.data_ptr())

    def step(opts=0):
        rc = lib.mgenx_unpack_batch(ctx, slab_p, slab.numel(), None, REC, None, REC, N_REC,
                                    ctypes.byref(cs), opts, stream)
        if rc != 0:
            raise RuntimeError(f"mgenx_unpack_batch rc={rc}")

    # correctness gate before timing
    step()
    torch.cuda.synchronize()
    bad = int((cols["err"] != 0).sum())
    if bad or int((out_len != REC).sum()):
        raise RuntimeError(f"unpack found {bad} bad records in a freshly packed slab")

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
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
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

    # secondary measurements (same stream, same events): header-only decode and pack
    def timed(fn, reps=20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps
    hdr_ms = timed(lambda: step(OPT_SKIP_CRC))
    pack_ms = timed(do_pack)
    step()
    torch.cuda.synchronize()
    assert int((cols["err"] != 0).sum()) == 0

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
            "config": {"workload": "udp_unpack_crc_1M_x_1024B", "records_per_gpu": N_REC,
                       "record_bytes": REC, "checksum": True,
                       "algorithmic_bytes_per_step_per_gpu": ALGO_BYTES,
                       "parallelism": f"flow-sharded x{world} (independent slabs)"},
            "mmsg_per_s": round(world * N_REC * args.steps / elapsed / 1e6, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS,
                         "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 4),
                         "traffic": load_traffic(), "kernel": "mgenx::unpack_kernel",
                         "kernel_ms": round(kern_ms, 4)},
            "extra": {"header_only_unpack_ms": round(hdr_ms, 4),
                      "header_only_mmsg_per_s": round(N_REC / (hdr_ms * 1e-3) / 1e6, 1),
                      "pack_ms": round(pack_ms, 4),
                      "pack_gbps": round((N_REC * REC + N_REC * 20) / (pack_ms * 1e-3) / 1e9,
                                         1)},
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
