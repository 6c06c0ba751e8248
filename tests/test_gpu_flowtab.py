"""GPU: mgenx_flow_lookup (MgenAnalyticTable::FindFlow for batches, mgenAnalytic.cpp:312-328)
against a Python dict keyed exactly like the reference key (dst addr, dst port, src addr,
src port, flowId): dense indices in order of first appearance, records with an error
skipped, keys persisting across calls, IPv4 and IPv6 addresses."""
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


def _batch(rng, n, n_src, n_dst, n_fid):
    srcs = []
    for k in range(n_src):
        if k % 3 == 2:
            srcs.append((2, 16, 7000 + k, bytes(rng.integers(0, 256, 16, dtype=np.uint8))))
        else:
            srcs.append((1, 4, 7000 + k, bytes([10, 0, k >> 8, k & 255])))
    dsts = [(1, 4, 5000 + k, bytes([127, 0, 0, 1 + k])) for k in range(n_dst)]
    dsts.append((2, 16, 5999, bytes(range(16))))
    si = rng.integers(0, len(srcs), n)
    di = rng.integers(0, len(dsts), n)
    fid = rng.integers(1, n_fid + 1, n).astype(np.uint32)
    err = (rng.random(n) < 0.05).astype(np.uint8)
    return srcs, dsts, si, di, fid, err


def _device_inputs(torch, srcs, dsts, si, di, fid, err):
    n = len(si)
    src = np.zeros((n, 20), np.uint8)
    dst_addr = np.zeros((n, 16), np.uint8)
    dst_len = np.zeros(n, np.uint8)
    dst_port = np.zeros(n, np.uint16)
    for i in range(n):
        t, ln, port, a = srcs[si[i]]
        src[i, 0], src[i, 1] = t, ln
        src[i, 2:4] = np.frombuffer(np.uint16(port).tobytes(), np.uint8)
        src[i, 4:4 + ln] = np.frombuffer(a, np.uint8)
        t, ln, port, a = dsts[di[i]]
        dst_addr[i, :ln] = np.frombuffer(a, np.uint8)
        dst_len[i], dst_port[i] = ln, port
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    cols = {"dst_addr": t(dst_addr.reshape(-1)), "dst_len": t(dst_len),
            "dst_port": t(dst_port.view(np.int16)), "flow_id": t(fid.view(np.int32)),
            "err": t(err)}
    return cols, t(src.reshape(-1))


@pytest.mark.parametrize("max_flows,n_src,calls", [(8192, 40, 4), (2048, 12, 3)])
def test_flow_lookup_matches_reference_key(torch, eng, max_flows, n_src, calls):
    """max_flows 8192: the large-table path (flag / scan / number kernels); 2048 (4096 slots):
    the small-table path (keys staged in LDS, the last workgroup numbers the new keys)."""
    table = eng.flow_table(max_flows)
    ref = {}
    try:
        for call in range(calls):   # keys persist across batches; later batches add a few new keys
            srcs, dsts, si, di, fid, err = _batch(np.random.default_rng(100 + call), 50_000,
                                                  n_src, 6, 12)
            cols, src = _device_inputs(torch, srcs, dsts, si, di, fid, err)
            idx, nf = eng.flow_lookup(table, cols, src, len(si))
            torch.cuda.synchronize()
            idx = idx.cpu().numpy().view(np.uint32)
            want = np.zeros(len(si), np.uint32)
            for i in range(len(si)):
                if err[i]:
                    want[i] = 0xFFFFFFFF
                    continue
                s, d = srcs[si[i]], dsts[di[i]]
                key = (d[3][:d[1]], d[2], s[3][:s[1]], s[2], int(fid[i]))
                want[i] = ref.setdefault(key, len(ref))
            assert np.array_equal(idx, want), call
            assert int(nf.cpu()[0]) == len(ref)
    finally:
        eng.flow_table_destroy(table)
    assert 1000 < len(ref) < max_flows


@pytest.mark.parametrize("max_flows", [8192, 2048])
def test_flow_lookup_from_rows(torch, eng, max_flows):
    """FindFlow keyed from the 32-B mgenx_rec rows: IPv4 destinations from dst_addr4 give
    the column form's indices; an IPv6 destination without the dst_addr column is unkeyed
    (MGENX_FLOW_NONE), with it the rows form equals the columns form again."""
    from mgen_amd import REC_DTYPE
    rng = np.random.default_rng(7)
    srcs, dsts, si, di, fid, err = _batch(rng, 40_000, 30, 5, 9)
    n = len(si)
    cols, src = _device_inputs(torch, srcs, dsts, si, di, fid, err)
    rows = np.zeros(n, REC_DTYPE)
    for i in range(n):
        t, ln, port, a = dsts[di[i]]
        rows[i]["dst_addr4"] = np.frombuffer(a[:4], "<u4")[0]
        rows[i]["dst_len"], rows[i]["dst_type"], rows[i]["dst_port"] = ln, t, port
    rows["flow_id"], rows["err"] = fid, err
    rows["seq_num"] = rng.integers(0, 2**32, n, dtype=np.uint64)   # not part of the key
    drows = torch.from_numpy(rows.view(np.uint8).copy()).cuda()
    v6 = np.array([dsts[d][1] > 4 for d in di])
    want_tab, t_rows, t_both = (eng.flow_table(max_flows), eng.flow_table(max_flows),
                                eng.flow_table(max_flows))
    try:
        want, _ = eng.flow_lookup(want_tab, cols, src, n)
        got, nf = eng.flow_lookup(t_rows, {"rows": drows}, src, n)
        both, _ = eng.flow_lookup(t_both, {"rows": drows, "dst_addr": cols["dst_addr"]}, src, n)
        torch.cuda.synchronize()
        want = want.cpu().numpy().view(np.uint32)
        got = got.cpu().numpy().view(np.uint32)
        assert np.array_equal(both.cpu().numpy().view(np.uint32), want)
        assert v6.any() and (~v6 & (err == 0)).any()
        assert np.all(got[v6] == 0xFFFFFFFF)
        # IPv4-only records: same partition (dense order differs when IPv6 keys are skipped)
        keep = ~v6 & (err == 0)
        pairs = {(int(a), int(b)) for a, b in zip(want[keep], got[keep])}
        assert len(pairs) == len(set(want[keep].tolist())) == len(set(got[keep].tolist()))
        assert int(nf.cpu()[0]) == len(set(got[keep].tolist()))
    finally:
        for t in (want_tab, t_rows, t_both):
            eng.flow_table_destroy(t)


def test_flow_lookup_undersized_table_is_bounded(torch, eng):
    """More distinct keys than a table holds: a table for 64 flows (128 slots)
    takes about 64 keys (a soft bound: keys created together may pass it) and maps the rest to
    MGENX_FLOW_NONE, promptly -- no record walks the whole table -- and the keys it took keep
    their indices in a second call."""
    import time
    n, n_keys = 400_000, 150_000       # more than 2 x pcap2mgen's first table (65,536 flows)
    fid = (np.arange(n) % n_keys + 1).astype(np.uint32)
    src = np.zeros((n, 20), np.uint8)
    src[:, 0], src[:, 1], src[:, 4] = 1, 4, 10
    d = {"dst_addr": np.tile(np.array([127, 0, 0, 1] + [0] * 12, np.uint8), n),
         "dst_len": np.full(n, 4, np.uint8), "dst_port": np.full(n, 5000, np.int16),
         "flow_id": fid.view(np.int32), "err": np.zeros(n, np.uint8)}
    cols = {k: torch.from_numpy(v.copy()).cuda() for k, v in d.items()}
    s = torch.from_numpy(src.reshape(-1).copy()).cuda()
    table = eng.flow_table(64)
    try:
        eng.flow_lookup(table, cols, s, n)       # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx, nf = eng.flow_lookup(table, cols, s, n)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        got = idx.cpu().numpy().view(np.uint32)
        held = got != 0xFFFFFFFF
        k = int(nf.cpu()[0])
        assert 64 <= k <= 128
        assert len(np.unique(fid[held])) == k and got[held].max() == k - 1
        # every record of a held key resolves to that key's index
        first = {}
        for f, k in zip(fid[held], got[held]):
            assert first.setdefault(int(f), int(k)) == int(k)
        assert dt < 0.05, dt
    finally:
        eng.flow_table_destroy(table)


def test_flow_span_matches_numpy(torch, eng):
    """mgenx_flow_span (pcap2mgen's report-slot sizing): the most records of any flow index
    < n_flows and the receive-time range over those records, against numpy; records with an
    index past n_flows (MGENX_FLOW_NONE among them) do not count."""
    rng = np.random.default_rng(5)
    n, n_flows = 300_000, 777
    f = rng.integers(0, n_flows + 40, n).astype(np.uint32)
    f[rng.random(n) < 0.01] = 0xFFFFFFFF
    sec = rng.integers(1_700_000_000, 1_700_000_900, n).astype(np.uint32)
    usec = rng.integers(0, 1_000_000, n).astype(np.uint32)
    t = lambda a: torch.from_numpy(a.view(np.int32).copy()).cuda()  # noqa: E731
    most, lo, hi = eng.flow_span(t(f), t(sec), t(usec), n, n_flows)
    ok = f < n_flows
    tt = sec[ok].astype(np.int64) * 1_000_000 + usec[ok]
    assert most == int(np.bincount(f[ok], minlength=n_flows).max())
    assert (lo, hi) == (int(tt.min()), int(tt.max()))
    most, lo, hi = eng.flow_span(t(f), t(sec), t(usec), n, 0)   # no flow index is < 0
    assert (most, lo, hi) == (0, 2**64 - 1, 0)
