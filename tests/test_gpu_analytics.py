"""GPU parity of mgenx_flow_reduce (MgenAnalytic::Update per flow) with the oracle's
or_flow_reduce_batch: per-flow state (counters, FP64 latency sums, the 1024-bit duplicate
mask) and every report, bit-exact; one call == the same records in several calls."""
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


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()


def run_gpu(torch, eng, d, n_flows, window, per_flow, splits=(0,)):
    from mgen_amd import FLOW_REPORT_DTYPE
    flows = eng.flow_init(n_flows, window)
    reports = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
    count = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
    n = len(d["seq"])
    bounds = list(splits) + [n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        cols = {k: dev(torch, v[a:b]) for k, v in d.items()}
        idx = dev(torch, (d["flow_id"][a:b] - 1).astype(np.uint32))
        eng.flow_reduce(flows, n_flows, idx, cols["seq"], cols["tx_sec"], cols["tx_usec"],
                        cols["msg_len"], cols["rx_sec"], cols["rx_usec"], reports=reports,
                        per_flow=per_flow, report_count=count)
    torch.cuda.synchronize()
    from mgen_amd import FLOW_STATE_DTYPE
    st = flows.cpu().numpy().view(FLOW_STATE_DTYPE)
    rep = reports.cpu().numpy().view(FLOW_REPORT_DTYPE).reshape(n_flows, per_flow)
    return st, rep, count.cpu().numpy().view(np.uint32), flows


def compare(st, rep, cnt, oflows, orep, ocnt, per_flow):
    assert np.array_equal(cnt, ocnt)
    for f, a in enumerate(oflows):
        s = st[f]
        assert s["msg_count"] == a.msg_count and s["byte_count"] == a.byte_count, f
        assert s["dup_count"] == a.dup_msg_count and s["n_reports"] == a.n_reports, f
        assert s["seq_start"] == a.seq_start and s["window_valid"] == a.window_valid, f
        assert s["latency_sum"] == a.latency_sum, (f, s["latency_sum"], a.latency_sum)
        assert s["latency_min"] == a.latency_min and s["latency_max"] == a.latency_max, f
        assert (s["win_start_sec"], s["win_start_usec"]) == (a.window_start.sec,
                                                             a.window_start.usec), f
        assert (s["win_end_sec"], s["win_end_usec"]) == (a.window_end.sec, a.window_end.usec)
        assert s["mask_n"] == a.nset, f
        if a.nset:
            assert s["mask_first"] == a.first, f
            assert s["mask"].tobytes() == bytes(a.bits), f
        k = min(int(ocnt[f]), per_flow)
        assert rep[f, :k].tobytes() == orep[f, :k].tobytes(), f


@pytest.mark.parametrize("n_flows,window", [(64, 0.25), (1024, 0.05)])
def test_flow_reduce_vs_oracle(torch, eng, n_flows, window):
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    per_flow = 32
    d = poisson_flows(300_000, n_flows, mean_gap_us=1000, seed=n_flows)
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, window, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    assert int(ocnt.sum()) > n_flows           # windows closed
    assert sum(a.dup_msg_count for a in of) > 0
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


def test_flow_reduce_streaming_batches(torch, eng):
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    d = poisson_flows(120_000, 48, mean_gap_us=500, seed=5, loss=0.05, dup=0.01, reorder=30)
    st, rep, cnt, _ = run_gpu(torch, eng, d, 48, 0.1, 16, splits=(0, 1, 777, 50_000))
    of, orep, ocnt = O.flow_reduce_batch(48, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=0.1, per_flow=16)
    compare(st, rep, cnt, of, orep, ocnt, 16)


def test_flow_export_counters(torch, eng):
    from mgen_amd import FLOW_COUNTERS_DTYPE
    from mgen_amd.workloads import poisson_flows
    d = poisson_flows(50_000, 32, seed=9)
    st, _, _, flows = run_gpu(torch, eng, d, 32, 0.5, 4)
    c = eng.flow_export(flows, 32).cpu().numpy().view(FLOW_COUNTERS_DTYPE)
    assert np.array_equal(c["msg_count"], st["msg_count"])
    assert np.array_equal(c["latency_sum"], st["latency_sum"])
    assert np.array_equal(c["n_reports"], st["n_reports"])


def _jumpy_flows(n_flows, per, seed):
    """Receive-order records whose per-flow sequence increments stress the fast segments:
    mostly +1, runs of losses, jumps past the 1024-bit mask span (clear and restart inside a
    segment), increments near 2^24 and 2^31 (int32 wrap of seq - first), zero-length
    messages, duplicates and local reordering."""
    rng = np.random.default_rng(seed)
    cols = {k: [] for k in ("flow_id", "seq", "tx_sec", "tx_usec", "rx_sec", "rx_usec",
                            "msg_len")}
    t0 = 1_700_000_000 * 10**6
    for f in range(n_flows):
        inc = np.ones(per, np.uint64)
        u = rng.random(per)
        inc[u < 0.05] = rng.integers(2, 12, int((u < 0.05).sum()))
        inc[u < 0.01] = rng.integers(1024, 3000, int((u < 0.01).sum()))
        inc[u < 0.002] = (1 << 24) + rng.integers(-3, 3, int((u < 0.002).sum()))
        inc[u < 0.0005] = (1 << 31) + 7
        seq = (np.cumsum(inc) + np.uint64(rng.integers(0, 1 << 32))) & np.uint64(0xFFFFFFFF)
        tx = t0 + np.cumsum(rng.exponential(700, per)).astype(np.int64)
        rx = tx + rng.integers(50, 500, per)
        ln = np.full(per, 200, np.uint16)
        ln[rng.random(per) < 0.003] = 0
        dup = rng.random(per) < 0.004
        seq = np.concatenate([seq, seq[dup]])
        tx = np.concatenate([tx, tx[dup]])
        rx = np.concatenate([rx, rx[dup] + 3])
        ln = np.concatenate([ln, ln[dup]])
        o = np.argsort(rx + rng.uniform(-900, 900, rx.size), kind="stable")
        for k, v in (("seq", seq[o]), ("tx_sec", tx[o] // 10**6), ("tx_usec", tx[o] % 10**6),
                     ("rx_sec", rx[o] // 10**6), ("rx_usec", rx[o] % 10**6),
                     ("msg_len", ln[o])):
            cols[k].append(v)
        cols["flow_id"].append(np.full(o.size, f + 1))
    rx_all = np.concatenate([np.asarray(a, np.int64) * 10**6 + b
                             for a, b in zip(cols["rx_sec"], cols["rx_usec"])])
    order = np.argsort(rx_all, kind="stable")
    dt = {"flow_id": np.uint32, "seq": np.uint32, "tx_sec": np.uint32, "tx_usec": np.uint32,
          "rx_sec": np.uint32, "rx_usec": np.uint32, "msg_len": np.uint16}
    return {k: np.concatenate(v).astype(dt[k])[order] for k, v in cols.items()}


@pytest.mark.parametrize("window", [0.02, 0.5, 30.0])
def test_flow_reduce_fast_segments_edge_cases(torch, eng, window):
    """The closed-form runs of plain records (fast segments) against the oracle's
    record-by-record Update, on sequences built to hit every boundary of the fast path."""
    from oracle import oracle as O
    n_flows, per_flow = 40, 64
    d = _jumpy_flows(n_flows, 6000, seed=int(window * 1000) + 3)
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, window, per_flow, splits=(0, 5000))
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


def test_flow_reduce_rows_equals_columns(torch, eng):
    """mgenx_flow_reduce_rows (seq / tx time / msg_len from the 32-B unpack rows) leaves the
    same flow state, reports and report records as the column form, which the tests above
    pin to the oracle."""
    from mgen_amd import FLOW_REPORT_DTYPE, FLOW_STATE_DTYPE, REC_DTYPE
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    n_flows, per_flow, window = 96, 8, 0.1
    d = poisson_flows(150_000, n_flows, mean_gap_us=700, seed=21, loss=0.02, dup=0.01,
                      reorder=20)
    n = len(d["seq"])
    rows = np.zeros(n, REC_DTYPE)
    rows["flow_id"], rows["seq_num"] = d["flow_id"], d["seq"]
    rows["tx_sec"], rows["tx_usec"], rows["msg_len"] = d["tx_sec"], d["tx_usec"], d["msg_len"]
    rows["dst_len"], rows["payload_len"] = 4, 7     # fields the reduction does not read
    idx = dev(torch, (d["flow_id"] - 1).astype(np.uint32))
    out = []
    for use_rows in (False, True):
        flows = eng.flow_init(n_flows, window)
        reports = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
        count = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
        rrec = torch.zeros(n_flows * per_flow, dtype=torch.int32, device="cuda")
        if use_rows:
            eng.flow_reduce_rows(flows, n_flows, idx, dev(torch, rows.view(np.uint8)),
                                 dev(torch, d["rx_sec"]), dev(torch, d["rx_usec"]),
                                 reports=reports, per_flow=per_flow, report_count=count,
                                 report_rec=rrec)
        else:
            c = {k: dev(torch, v) for k, v in d.items()}
            eng.flow_reduce(flows, n_flows, idx, c["seq"], c["tx_sec"], c["tx_usec"],
                            c["msg_len"], c["rx_sec"], c["rx_usec"], reports=reports,
                            per_flow=per_flow, report_count=count, report_rec=rrec)
        torch.cuda.synchronize()
        out.append((flows.cpu().numpy(), reports.cpu().numpy(), count.cpu().numpy(),
                    rrec.cpu().numpy()))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    st = out[1][0].view(FLOW_STATE_DTYPE)
    rep = out[1][1].view(FLOW_REPORT_DTYPE).reshape(n_flows, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    compare(st, rep, out[1][2].view(np.uint32), of, orep, ocnt, per_flow)


def test_flow_reduce_many_flows_radix_path(torch, eng):
    """More than 2047 flows: the radix-sort ordering instead of the counting sort (same
    update kernel), against the oracle."""
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    n_flows, per_flow = 5000, 4
    d = poisson_flows(200_000, n_flows, mean_gap_us=20_000, seed=33, reorder=40)
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, 0.2, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=0.2, per_flow=per_flow)
    assert int(ocnt.sum()) > n_flows
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


@pytest.mark.parametrize("n_flows", [1535, 1040])
def test_flow_reduce_single_pass_scan_many_blocks(torch, eng, n_flows):
    """The counting sort's single-pass column scan (<= 512 tiles) at the largest flow counts:
    96 and 65 blocks of 16 flows, so the look-back spans more than one 64-lane window and a
    ragged last block -- against the oracle."""
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    per_flow = 4
    d = poisson_flows(400_000, n_flows, mean_gap_us=5_000, seed=n_flows, reorder=20)
    assert (len(d["seq"]) + 4095) // 4096 <= 512
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, 0.2, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=0.2, per_flow=per_flow)
    assert int(ocnt.sum()) > n_flows
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


def test_flow_reduce_flow_none_and_tile_edges(torch, eng):
    """Records with MGENX_FLOW_NONE or an index >= n_flows are skipped; batch sizes around the
    counting sort's 8192-record tile (one short tile, exact tiles, one record past)."""
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    d = poisson_flows(40_000, 40, mean_gap_us=300, seed=8)
    n = len(d["seq"])
    rng = np.random.default_rng(3)
    idx = (d["flow_id"] - 1).astype(np.uint32)
    junk = rng.random(n) < 0.1
    idx[junk] = np.where(rng.random(int(junk.sum())) < 0.5, 0xFFFFFFFF, 40 + 7).astype(np.uint32)
    keep = ~junk
    for m in (100, 8192, 16384, 8193, n):
        flows = eng.flow_init(40, 0.05)
        reports = torch.zeros(40 * 8 * 96, dtype=torch.uint8, device="cuda")
        count = torch.zeros(40, dtype=torch.int32, device="cuda")
        c = {k: dev(torch, v[:m]) for k, v in d.items()}
        eng.flow_reduce(flows, 40, dev(torch, idx[:m]), c["seq"], c["tx_sec"], c["tx_usec"],
                        c["msg_len"], c["rx_sec"], c["rx_usec"], reports=reports, per_flow=8,
                        report_count=count)
        torch.cuda.synchronize()
        from mgen_amd import FLOW_REPORT_DTYPE, FLOW_STATE_DTYPE
        st = flows.cpu().numpy().view(FLOW_STATE_DTYPE)
        rep = reports.cpu().numpy().view(FLOW_REPORT_DTYPE).reshape(40, 8)
        k = keep[:m]
        sub = {key: v[:m][k] for key, v in d.items()}
        of, orep, ocnt = O.flow_reduce_batch(40, sub["flow_id"] - 1, sub["seq"], sub["tx_sec"],
                                             sub["tx_usec"], sub["msg_len"], sub["rx_sec"],
                                             sub["rx_usec"], window=0.05, per_flow=8)
        compare(st, rep, count.cpu().numpy().view(np.uint32), of, orep, ocnt, 8)


def test_flow_reduce_skewed_flows_tile_runs(torch, eng):
    """The one-pass tile ordering's record supply: one flow holding most records (runs of
    thousands per 8192-record tile, windows of 64 tiles far larger than the slot queue), flows
    absent from whole tiles, a flow with a single record, report_rec pointing at the closing
    record -- against the oracle."""
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    big = poisson_flows(420_000, 1, mean_gap_us=50, seed=21, reorder=3)
    small = poisson_flows(30_000, 6, mean_gap_us=400, seed=22)
    rng = np.random.default_rng(5)
    d = {k: np.concatenate([big[k], small[k]]) for k in big}
    d["flow_id"] = np.concatenate([big["flow_id"], small["flow_id"] + 1])  # flows 1, 2..7
    perm = np.argsort(rng.random(len(d["seq"])) + np.arange(len(d["seq"])) / 2e4, kind="stable")
    d = {k: np.ascontiguousarray(v[perm]) for k, v in d.items()}
    single = {k: v[:1].copy() for k, v in d.items()}
    single["flow_id"][:] = 8
    d = {k: np.concatenate([d[k], single[k]]) for k in d}
    n_flows, per_flow = 8, 64
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, 0.02, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=0.02, per_flow=per_flow)
    assert int(ocnt[0]) > 5 and of[7].msg_count == 1
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


def _mixed_lengths():
    sets = []
    for i, per in enumerate((1, 700, 2040, 2048, 2100, 5000, 9000, 20000)):
        d = _jumpy_flows(1, per, seed=100 + i)
        d["flow_id"] = d["flow_id"] + i
        sets.append(d)
    d = {k: np.concatenate([s[k] for s in sets]) for k in sets[0]}
    rx = d["rx_sec"].astype(np.int64) * 10**6 + d["rx_usec"]
    o = np.argsort(rx, kind="stable")
    return {k: np.ascontiguousarray(v[o]) for k, v in d.items()}


@pytest.mark.parametrize("window", [0.001, 0.3])
def test_flow_reduce_mixed_lengths(torch, eng, window):
    """Flows of 1 to 20000 records in one call with jumpy sequences (mask restarts, records
    below `first`, wraps, duplicates, reordering) and, at 1 ms, a window closing every record
    or two (more reports than per_flow keeps); a second call continues from the first's
    state.  Against the oracle."""
    from oracle import oracle as O
    d = _mixed_lengths()
    n_flows, per_flow = 8, 4096
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, window, per_flow,
                              splits=(0, len(d["seq"]) * 3 // 4))
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    assert sum(a.dup_msg_count for a in of) > 0
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


@pytest.mark.parametrize("window", [0.001, 0.3])
def test_flow_reduce_long_and_jumpy_flows(torch, eng, window):
    """Few long flows (one flow of many thousand records beside short ones) and flows whose
    sequence numbers jump past the mask span and back: every event kind inside long runs of
    simple records, split across two calls.  Bit-exact against the oracle."""
    from oracle import oracle as O
    d = _mixed_lengths()
    n_flows, per_flow = 8, 4096
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, window, per_flow,
                              splits=(0, len(d["seq"]) * 3 // 4))
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    compare(st, rep, cnt, of, orep, ocnt, per_flow)
    d = _jumpy_flows(40, 6000, seed=int(window * 1000) + 3)
    st, rep, cnt, _ = run_gpu(torch, eng, d, 40, window, 64, splits=(0, 5000))
    of, orep, ocnt = O.flow_reduce_batch(40, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=64)
    compare(st, rep, cnt, of, orep, ocnt, 64)


def test_flow_reduce_config4_full_size_vs_oracle(torch, eng):
    """Config 4 at its full size (8,388,608 records, 1024 POISSON flows): 2048 tiles, so every
    persistent order block walks several tiles (the next tile's loads in flight while the
    current one is written), for the column and the row form with report_rec, against the
    oracle."""
    from mgen_amd import FLOW_REPORT_DTYPE, FLOW_STATE_DTYPE, REC_DTYPE
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    n_flows, per_flow, window = 1024, 4, 1.0
    d = poisson_flows(8_388_608, n_flows, mean_gap_us=1000, seed=44, loss=0.01, dup=0.005,
                      reorder=10)
    n = len(d["seq"])
    assert n > 256 * 4096  # more tiles than one pass of the persistent grid
    idx = dev(torch, (d["flow_id"] - 1).astype(np.uint32))
    rows = np.zeros(n, REC_DTYPE)
    rows["flow_id"], rows["seq_num"] = d["flow_id"], d["seq"]
    rows["tx_sec"], rows["tx_usec"], rows["msg_len"] = d["tx_sec"], d["tx_usec"], d["msg_len"]
    out = []
    for use_rows in (False, True):
        flows = eng.flow_init(n_flows, window)
        reports = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
        count = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
        rrec = torch.zeros(n_flows * per_flow, dtype=torch.int32, device="cuda")
        if use_rows:
            eng.flow_reduce_rows(flows, n_flows, idx, dev(torch, rows.view(np.uint8)),
                                 dev(torch, d["rx_sec"]), dev(torch, d["rx_usec"]),
                                 reports=reports, per_flow=per_flow, report_count=count,
                                 report_rec=rrec)
        else:
            c = {k: dev(torch, v) for k, v in d.items()}
            eng.flow_reduce(flows, n_flows, idx, c["seq"], c["tx_sec"], c["tx_usec"],
                            c["msg_len"], c["rx_sec"], c["rx_usec"], reports=reports,
                            per_flow=per_flow, report_count=count, report_rec=rrec)
        torch.cuda.synchronize()
        out.append((flows.cpu().numpy(), reports.cpu().numpy(), count.cpu().numpy(),
                    rrec.cpu().numpy()))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    st = out[0][0].view(FLOW_STATE_DTYPE)
    rep = out[0][1].view(FLOW_REPORT_DTYPE).reshape(n_flows, per_flow)
    cnt = out[0][2].view(np.uint32)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    assert int(ocnt.sum()) > n_flows
    compare(st, rep, cnt, of, orep, ocnt, per_flow)
    # report_rec: the input index of each kept report's closing record -- its receive time
    rrec = out[0][3].view(np.uint32).reshape(n_flows, per_flow)
    for f in range(0, n_flows, 97):
        for r in range(min(int(cnt[f]), per_flow)):
            i = int(rrec[f, r])
            assert d["flow_id"][i] - 1 == f
            assert (int(d["rx_sec"][i]), int(d["rx_usec"][i])) == (int(rep[f, r]["rx_sec"]),
                                                                  int(rep[f, r]["rx_usec"]))


def test_flow_reduce_big_tiles_vs_oracle(torch, eng):
    """1,100,000 records: on a 256-CU part 4096-record tiles would take the persistent order
    grid two rounds (269 tiles), so the ordering takes 4608-record tiles (239, the last one
    ragged) -- column and row forms with report_rec against the oracle; then the same records
    with per_flow = 0 and no report counts (NULL dev_report_count) give the same states."""
    from mgen_amd import FLOW_REPORT_DTYPE, FLOW_STATE_DTYPE, REC_DTYPE
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    n_flows, per_flow, window = 200, 8, 0.5
    d = poisson_flows(1_100_000, n_flows, mean_gap_us=400, seed=46, loss=0.01, dup=0.005,
                      reorder=10)
    n = len(d["seq"])
    assert 256 * 4096 < n <= 256 * 4608
    idx = dev(torch, (d["flow_id"] - 1).astype(np.uint32))
    rows = np.zeros(n, REC_DTYPE)
    rows["flow_id"], rows["seq_num"] = d["flow_id"], d["seq"]
    rows["tx_sec"], rows["tx_usec"], rows["msg_len"] = d["tx_sec"], d["tx_usec"], d["msg_len"]
    c = {k: dev(torch, v) for k, v in d.items()}
    out = []
    for use_rows in (False, True):
        flows = eng.flow_init(n_flows, window)
        reports = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
        count = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
        rrec = torch.zeros(n_flows * per_flow, dtype=torch.int32, device="cuda")
        if use_rows:
            eng.flow_reduce_rows(flows, n_flows, idx, dev(torch, rows.view(np.uint8)),
                                 c["rx_sec"], c["rx_usec"], reports=reports, per_flow=per_flow,
                                 report_count=count, report_rec=rrec)
        else:
            eng.flow_reduce(flows, n_flows, idx, c["seq"], c["tx_sec"], c["tx_usec"],
                            c["msg_len"], c["rx_sec"], c["rx_usec"], reports=reports,
                            per_flow=per_flow, report_count=count, report_rec=rrec)
        torch.cuda.synchronize()
        out.append((flows.cpu().numpy(), reports.cpu().numpy(), count.cpu().numpy(),
                    rrec.cpu().numpy()))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    st = out[0][0].view(FLOW_STATE_DTYPE)
    rep = out[0][1].view(FLOW_REPORT_DTYPE).reshape(n_flows, per_flow)
    cnt = out[0][2].view(np.uint32)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    assert int(ocnt.sum()) > n_flows
    compare(st, rep, cnt, of, orep, ocnt, per_flow)
    rrec = out[0][3].view(np.uint32).reshape(n_flows, per_flow)
    for f in range(0, n_flows, 13):
        for r in range(min(int(cnt[f]), per_flow)):
            i = int(rrec[f, r])
            assert d["flow_id"][i] - 1 == f
            assert (int(d["rx_sec"][i]), int(d["rx_usec"][i])) == (int(rep[f, r]["rx_sec"]),
                                                                  int(rep[f, r]["rx_usec"]))
    flows = eng.flow_init(n_flows, window)
    assert eng.flow_reduce(flows, n_flows, idx, c["seq"], c["tx_sec"], c["tx_usec"],
                           c["msg_len"], c["rx_sec"], c["rx_usec"]) is None
    torch.cuda.synchronize()
    assert np.array_equal(flows.cpu().numpy(), out[0][0])


def _epoch_fuzz(n_flows, per, seed, window_us):
    """Per-flow sequences aimed at the window-parallel update's seams: epoch starts (failed
    Sets in the counted branch) on closing records and right after them, duplicates of closing
    records and across epochs, late records below `first` inside the span (first moves down)
    and far below it (silent failures below seq_start, and restarts when seq_start is older),
    int32 wraps of seq - first, messages of size 0 (a flow's first record, then the first
    actual message -- in one window, and closing one), windows of one record and of thousands,
    rx times out of order."""
    rng = np.random.default_rng(seed)
    cols = {k: [] for k in ("flow_id", "seq", "tx_sec", "tx_usec", "rx_sec", "rx_usec",
                            "msg_len")}
    t0 = 1_700_000_000 * 10**6
    for f in range(n_flows):
        seq = np.zeros(per, np.int64)
        s = int(rng.integers(0, 1 << 32))
        hist = []
        for i in range(per):
            u = rng.random()
            if u < 0.05 and hist:
                s2 = hist[-int(rng.integers(1, min(len(hist), 40) + 1))]  # duplicate
            elif u < 0.09:
                s2 = s - int(rng.integers(1, 40))                          # late, in span
            elif u < 0.11:
                s2 = s - int(rng.integers(1024, 4000))                     # far below first
            elif u < 0.14:
                s = s + int(rng.integers(1024, 3000))                      # restart ahead
                s2 = s
            elif u < 0.145:
                s = s + (1 << 31) + int(rng.integers(-5, 5))               # int32 wrap
                s2 = s
            else:
                s = s + int(rng.integers(1, 3))
                s2 = s
            seq[i] = s2
            hist.append(s2)
        gaps = rng.exponential(window_us / 40.0, per)
        big = rng.random(per) < 0.03
        gaps[big] = rng.uniform(window_us, 3 * window_us, int(big.sum()))   # one-record windows
        tx = t0 + np.cumsum(gaps).astype(np.int64) + int(rng.integers(0, 10**6))
        rx = tx + rng.integers(50, 500, per)
        swap = rng.random(per) < 0.02                                        # rx out of order
        rx[swap] -= rng.integers(1000, 50_000, int(swap.sum()))
        ln = np.full(per, 300, np.int64)
        ln[rng.random(per) < 0.03] = 0
        if f % 3 == 0:
            ln[:int(rng.integers(1, 30))] = 0   # first message(s) of size 0, then the first actual
        for k, v in (("seq", seq & 0xFFFFFFFF), ("tx_sec", tx // 10**6), ("tx_usec", tx % 10**6),
                     ("rx_sec", rx // 10**6), ("rx_usec", rx % 10**6), ("msg_len", ln)):
            cols[k].append(v)
        cols["flow_id"].append(np.full(per, f + 1))
    # interleave the flows in a receive-like order, each flow's own order kept
    key = np.concatenate([np.arange(per) + rng.uniform(0, 3, per) for _ in range(n_flows)])
    order = np.argsort(key, kind="stable")
    dt = {"flow_id": np.uint32, "seq": np.uint32, "tx_sec": np.uint32, "tx_usec": np.uint32,
          "rx_sec": np.uint32, "rx_usec": np.uint32, "msg_len": np.uint16}
    return {k: np.concatenate(v).astype(dt[k])[order] for k, v in cols.items()}


@pytest.mark.parametrize("window", [0.01, 0.2, 2.0])
def test_flow_reduce_epoch_and_window_seams(torch, eng, window):
    """The window-parallel update against the oracle on sequences built for its seams (epoch
    starts on and after closing records, duplicates across epochs and of closing records,
    records below `first`, size-0 first messages, one-record windows), streamed in four calls
    whose splits fall inside windows and epochs."""
    from oracle import oracle as O
    n_flows, per_flow = 24, 512
    d = _epoch_fuzz(n_flows, 4000, seed=int(window * 100) + 7, window_us=window * 1e6)
    n = len(d["seq"])
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, window, per_flow,
                              splits=(0, 1, n // 3, n // 3 + 5))
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=window, per_flow=per_flow)
    assert sum(a.dup_msg_count for a in of) > 0 and int(ocnt.sum()) > n_flows
    compare(st, rep, cnt, of, orep, ocnt, per_flow)


def test_flow_reduce_rank_share_vs_oracle(torch, eng):
    """Rank 0's share of config 4 at N = 8 (flows f with f mod 8 == 0: 128 of 1024 flows, 1/8
    of the records; the other flows untouched) against the oracle."""
    from mgen_amd.workloads import poisson_flows
    from oracle import oracle as O
    n_flows, per_flow = 1024, 16
    d = poisson_flows(1_048_576, n_flows, mean_gap_us=1000, seed=77)
    own = (d["flow_id"] % 8) == 0
    d = {k: np.ascontiguousarray(v[own]) for k, v in d.items()}
    st, rep, cnt, _ = run_gpu(torch, eng, d, n_flows, 1.0, per_flow)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"],
                                         d["rx_usec"], window=1.0, per_flow=per_flow)
    assert sum(1 for a in of if a.msg_count > 0) == 128 and int(ocnt.sum()) > 0
    compare(st, rep, cnt, of, orep, ocnt, per_flow)
