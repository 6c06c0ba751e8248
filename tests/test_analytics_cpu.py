"""MgenAnalytic restatement (oracle) against hand-derived sequences, from the rules of
src/common/mgenAnalytic.cpp:74-258 (parity unpinned at protolib: SURVEY.md 8(c)):
the window opens at the first receive, the first message's bytes are not counted
(:136-139), a report fires when rx >= window_end and reports msg_count - 1 messages,
loss = 1 - msg_count / (seqMax - seq_start + 1), duplicates are counted, not reported."""
import numpy as np
import pytest

from oracle import oracle as O

SIZE = 256


def run(events, window=0.5):
    """events: (seq, tx_seconds, rx_seconds) in receive order -> (oracle, [reports])."""
    a = O.AnalyticOracle(window)
    reps = []
    for seq, tx, rx in events:
        txs, txu = int(tx), int(round((tx - int(tx)) * 1e6))
        rxs, rxu = int(rx), int(round((rx - int(rx)) * 1e6))
        if a.update(rxs, rxu, SIZE, txs, txu, seq):
            r = a.a
            reps.append(dict(msg_count=r.report_msg_count, loss=r.report_loss_ave,
                             rate=r.report_rate_ave, lat=r.report_latency_ave,
                             dur=r.report_duration, lmin=r.report_latency_min,
                             lmax=r.report_latency_max))
    return a, reps


def periodic(seqs, t0=1000.0, gap=0.1, lat=0.001):
    return [(s, t0 + gap * k, t0 + gap * k + lat) for k, s in enumerate(seqs)]


def test_window_quantization():
    w = O.quantized_window(0.5)
    assert 0.45 < w < 0.55 and O.quantized_window(0.5) == w


def test_in_order():
    w = O.quantized_window(0.5)
    k_rep = int(np.ceil(w / 0.1))                 # first k with 0.1 k >= w
    a, reps = run(periodic(range(12)))
    r = reps[0]
    assert r["msg_count"] == k_rep                # msgs 0..k_rep counted, minus one
    assert r["loss"] == 0.0
    assert r["dur"] == pytest.approx(0.1 * k_rep, abs=1e-9)
    assert r["rate"] == pytest.approx(k_rep * SIZE / (0.1 * k_rep), rel=1e-9)
    assert r["lat"] == pytest.approx(0.001, abs=1e-9) and r["lmin"] == r["lmax"]


def test_lossy():
    w = O.quantized_window(0.5)
    k_rep = int(np.ceil(w / 0.1))
    seqs = [s for s in range(14) if s != 3]       # seq 3 lost
    a, reps = run(periodic(seqs))
    r = reps[0]
    received = k_rep + 1                          # messages up to the report, incl. it
    seq_max = seqs[k_rep]
    assert r["msg_count"] == received - 1
    assert r["loss"] == pytest.approx(1.0 - received / (seq_max - 0 + 1), abs=1e-12)


def test_duplicate_counted_not_reported():
    seqs = [0, 1, 2, 2, 3, 4, 5, 6, 7, 8, 9]
    a, reps = run(periodic(seqs))
    assert a.a.dup_msg_count == 1
    assert reps[0]["loss"] == 0.0


def test_reordered_is_not_loss():
    seqs = [0, 1, 3, 2, 4, 5, 6, 7, 8, 9, 10]
    a, reps = run(periodic(seqs))
    assert a.a.dup_msg_count == 0
    assert reps[0]["loss"] == 0.0


def test_batch_equals_per_record():
    from mgen_amd.workloads import poisson_flows
    d = poisson_flows(20000, 8, mean_gap_us=2000)
    f = d["flow_id"] - 1
    flows, reps, counts = O.flow_reduce_batch(8, f, d["seq"], d["tx_sec"], d["tx_usec"],
                                              d["msg_len"], d["rx_sec"], d["rx_usec"],
                                              window=0.25, per_flow=64)
    for fl in range(8):
        m = f == fl
        a = O.AnalyticOracle(0.25)
        n_rep = 0
        for i in np.nonzero(m)[0]:
            n_rep += a.update(int(d["rx_sec"][i]), int(d["rx_usec"][i]), int(d["msg_len"][i]),
                              int(d["tx_sec"][i]), int(d["tx_usec"][i]), int(d["seq"][i]))
        assert n_rep == counts[fl]
        assert a.a.msg_count == flows[fl].msg_count
        assert a.a.latency_sum == flows[fl].latency_sum
        assert bytes(a.a.bits) == bytes(flows[fl].bits)
