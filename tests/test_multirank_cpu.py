"""World-size-2 gloo rehearsal of the multi-GPU merge: flows are owned by
rank flow_id mod G, each rank reduces its own flows' records, and one all-reduce(sum) of the
packed per-flow counters (mgenx_flow_counters, 64 B per flow) reproduces the single-rank
table exactly (non-owners contribute zeros).  The per-rank reduction here is the oracle
(CPU); on GPUs the same table comes from mgenx_flow_export and RCCL."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_FLOWS = 16
WORLD = 2


def counters(flows):
    from mgen_amd._abi import FLOW_COUNTERS_DTYPE
    c = np.zeros(len(flows), FLOW_COUNTERS_DTYPE)
    for f, a in enumerate(flows):
        c[f] = (a.msg_count, a.byte_count, a.dup_msg_count, a.n_reports, a.latency_sum,
                a.latency_min, a.latency_max, a.seq_start)
    return c


def data():
    from mgen_amd.workloads import poisson_flows
    return poisson_flows(30000, N_FLOWS, mean_gap_us=3000, seed=11)


def reduce_flows(d, owned):
    from oracle import oracle as O
    idx = np.where(owned[d["flow_id"] - 1], d["flow_id"] - 1, N_FLOWS).astype(np.uint32)
    flows, _, _ = O.flow_reduce_batch(N_FLOWS, idx, d["seq"], d["tx_sec"], d["tx_usec"],
                                      d["msg_len"], d["rx_sec"], d["rx_usec"], window=0.5,
                                      per_flow=0)
    return counters(flows)


def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    d = data()
    owned = (np.arange(N_FLOWS) % WORLD) == rank
    c = reduce_flows(d, owned)
    t = torch.from_numpy(c.view(np.uint8).copy())
    # all-reduce(sum) over 64-bit lanes: integer counters as int64, doubles as float64
    as_i64 = torch.from_numpy(c.view(np.int64).copy())
    dist.all_reduce(as_i64)
    merged = as_i64.numpy().view(c.dtype)
    # the float fields summed as integers are only valid because exactly one rank is
    # nonzero per flow; check that too with a float64 all-reduce
    f64 = torch.from_numpy(np.stack([c["latency_sum"], c["latency_min"], c["latency_max"]],
                                    axis=1).copy())
    dist.all_reduce(f64)
    if rank == 0:
        q.put((merged.tobytes(), f64.numpy().tobytes(), t.numel()))
    dist.destroy_process_group()


def test_flow_counter_merge_gloo():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    merged_b, f64_b, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = reduce_flows(data(), np.ones(N_FLOWS, bool))
    from mgen_amd._abi import FLOW_COUNTERS_DTYPE
    merged = np.frombuffer(merged_b, FLOW_COUNTERS_DTYPE)
    assert merged.tobytes() == want.tobytes()
    f64 = np.frombuffer(f64_b, np.float64).reshape(N_FLOWS, 3)
    assert np.array_equal(f64[:, 0], want["latency_sum"])
