"""GPU: the multi-GPU merge of flow-sharded analytics.

  * ownership property on one GPU: G virtual ranks each run mgenx_flow_reduce over the
    records of the flows they own (flow_id mod G, the others masked out), export their
    counters, and the SUM of the G exports (the all-reduce mgenx_allreduce_flows performs)
    equals the export of one rank owning every flow -- FP64 fields bit for bit;
  * mgenx_allreduce_flows / mgenx_allgather_u64 through a real RCCL communicator (one rank:
    this box has one GPU; rank counts > 1 run in bench.py on the 8-GPU node).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def eng(torch):
    from mgen_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def _reduce(torch, eng, d, n_flows, own):
    flows = eng.flow_init(n_flows, 1.0)
    idx = np.where(own, d["flow_id"] - 1, n_flows).astype(np.uint32)
    t = {k: torch.from_numpy(np.ascontiguousarray(v).copy()).cuda() for k, v in d.items()}
    eng.flow_reduce(flows, n_flows, torch.from_numpy(idx).cuda(), t["seq"], t["tx_sec"],
                    t["tx_usec"], t["msg_len"], t["rx_sec"], t["rx_usec"])
    return eng.flow_export(flows, n_flows)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_owner_partitioned_exports_sum_to_single_owner(torch, eng, G):
    from mgen_amd.workloads import poisson_flows
    n_flows = 256
    d = poisson_flows(200_000, n_flows=n_flows, mean_gap_us=1000)
    full = _reduce(torch, eng, d, n_flows, np.ones(len(d["seq"]), bool))
    acc = torch.zeros(n_flows * 8, dtype=torch.int64, device="cuda")
    for r in range(G):
        part = _reduce(torch, eng, d, n_flows, (d["flow_id"] % G) == r)
        acc += part.view(torch.int64)          # what the RCCL SUM computes, rank by rank
    torch.cuda.synchronize()
    assert torch.equal(acc, full.view(torch.int64))
    c = full.cpu().numpy().view(np.uint64).reshape(n_flows, 8)
    assert (c[:, 0] > 0).all()                 # every flow saw records


def test_rccl_allreduce_and_allgather_one_rank(torch, eng):
    from mgen_amd.workloads import poisson_flows
    n_flows = 64
    d = poisson_flows(20_000, n_flows=n_flows, mean_gap_us=1000)
    counters = _reduce(torch, eng, d, n_flows, np.ones(len(d["seq"]), bool))
    before = counters.clone()
    comm = eng.comm_init(1, 0, eng.comm_unique_id())
    try:
        eng.allreduce_flows(comm, counters, n_flows)
        src = torch.arange(5, dtype=torch.int64, device="cuda") * 7 + 3
        dst = torch.zeros(5, dtype=torch.int64, device="cuda")
        eng.allgather_u64(comm, src, dst, 5)
        torch.cuda.synchronize()
        assert torch.equal(counters, before)
        assert torch.equal(dst, src)
    finally:
        eng.comm_destroy(comm)
