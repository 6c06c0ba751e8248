"""GPU parity of the MGEN_DATA items: mgenx_report_build (MgenAnalytic's report_msg with the
host-libm quantizers), mgenx_log_report_text (MgenAnalytic::Log REPORT lines),
mgenx_data_walk (ProcessRecvMessage's TLV walk: flow commands, reports, generic items,
invalid and zero-length items) and mgenx_log_report_recv_text (Report::Log), each against
the oracle restatement (tests/test_report_cpu.py), byte-exact."""
import numpy as np
import pytest

from report_util import addr, flow_command, random_values

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
    return torch.from_numpy(np.ascontiguousarray(a).copy().view(np.uint8)).cuda()


def _keys(oracle, n, rng):
    from mgen_amd import REPORT_KEY_DTYPE
    k = np.zeros(n, REPORT_KEY_DTYPE)
    for f in range(n):
        v6 = f % 4 == 3
        s, d = addr(rng, v6), addr(rng, v6)
        if f % 11 == 5:                                          # unknown address type
            s["type"] = d["type"] = 0
        k["src"][f], k["dst"][f] = s[0], d[0]
        k["flow_id"][f] = [0, 1, 7, 40, 0xFFFFFFFF, int(rng.integers(2, 1 << 31))][f % 6]
        k["protocol"][f] = [1, 2, 3, 0][f % 4]
    return k


def _reports(n_flows, per_flow, rng):
    from mgen_amd import FLOW_REPORT_DTYPE
    r = np.zeros((n_flows, per_flow), FLOW_REPORT_DTYPE)
    for f in range(n_flows):
        for j in range(per_flow):
            dur, ave, mn, mx, rate, loss = random_values(rng)
            x = r[f, j]
            x["flow"], x["index"] = f, j
            x["duration"], x["latency_ave"], x["latency_min"], x["latency_max"] = dur, ave, mn, mx
            x["rate"], x["loss"] = rate, loss
            x["msg_count"] = int(rng.integers(0, 1 << 40))
            x["rx_sec"] = int(rng.integers(1_600_000_000, 1_800_000_000))
            x["rx_usec"] = int(rng.integers(0, 1_000_000))
            r[f, j] = x
    return r


def _oracle_items(oracle, keys, reps, count, per_flow, sign0, offset=None):
    O = oracle
    out, lens, signs = {}, {}, []
    for f in range(len(keys)):
        s = np.frombuffer(keys["src"][f].tobytes(), O.ADDR_DTYPE)
        d = np.frombuffer(keys["dst"][f].tobytes(), O.ADDR_DTYPE)
        sg = int(sign0[f])
        for j in range(min(int(count[f]), per_flow)):
            w = reps[f, j]
            off = 0.0 if offset is None else float(offset[f * per_flow + j])
            b, sg = O.report_build(s, d, int(keys["flow_id"][f]), int(keys["protocol"][f]),
                                   float(w["duration"]), float(w["latency_ave"]),
                                   float(w["latency_min"]), float(w["latency_max"]),
                                   float(w["rate"]), float(w["loss"]), offset=off, sign=sg)
            out[(f, j)], lens[(f, j)] = b, len(b)
        signs.append(sg)
    return out, lens, np.array(signs, np.uint8)


def test_report_build_and_lines(torch, eng, oracle):
    O = oracle
    rng = np.random.default_rng(0x5e9)
    n_flows, per_flow = 96, 6
    keys = _keys(O, n_flows, rng)
    reps = _reports(n_flows, per_flow, rng)
    count = rng.integers(0, per_flow + 3, n_flows).astype(np.uint32)
    sign0 = (rng.random(n_flows) < 0.2).astype(np.uint8)
    offset = rng.choice([0.0, 1e-6, 0.25, 3.7, 700.0], n_flows * per_flow)
    for off in (None, offset):
        sign = dev(torch, sign0)
        items, ilen = eng.report_build(dev(torch, reps), n_flows, per_flow, dev(torch, count),
                                       dev(torch, keys), sign,
                                       None if off is None else dev(torch, off))
        items = items.cpu().numpy().reshape(-1, 52)
        ilen = ilen.cpu().numpy()
        want, wlen, wsign = _oracle_items(O, keys, reps, count, per_flow, sign0, off)
        for (f, j), b in want.items():
            k = f * per_flow + j
            assert ilen[k] == wlen[(f, j)], (f, j)
            assert items[k, :len(b)].tobytes() == b, (f, j, items[k, :len(b)].tobytes(), b)
        assert np.array_equal(sign.cpu().numpy(), wsign)
    # REPORT lines (from the last build), every option
    for opts in (0, 1):
        text, lo = eng.log_report_text(torch.from_numpy(items.reshape(-1)).cuda(),
                                       dev(torch, reps), n_flows, per_flow, dev(torch, count),
                                       opts=opts)
        got = text.cpu().numpy().tobytes()
        exp = []
        for f in range(n_flows):
            for j in range(min(int(count[f]), per_flow)):
                w = reps[f, j]
                exp.append(O.log_report(want[(f, j)], float(w["duration"]), float(w["rate"]),
                                        float(w["loss"]), float(w["latency_ave"]),
                                        float(w["latency_min"]), float(w["latency_max"]),
                                        int(w["msg_count"]) & 0xFFFFFFFF, int(w["rx_sec"]),
                                        int(w["rx_usec"]), opts))
        exp = b"".join(exp)
        if got != exp:
            gl, el = got.split(b"\n"), exp.split(b"\n")
            bad = next(i for i in range(min(len(gl), len(el))) if gl[i] != el[i])
            raise AssertionError((bad, gl[bad], el[bad]))
        assert int(lo[-1]) == len(exp)


def test_flow_reduce_to_reports(torch, eng, oracle):
    """End to end: records -> mgenx_flow_reduce -> mgenx_report_build == the oracle's
    analytics -> report_msg."""
    from mgen_amd import FLOW_REPORT_DTYPE
    from mgen_amd.workloads import poisson_flows
    O = oracle
    n_flows, per_flow = 40, 8
    d = poisson_flows(60_000, n_flows, mean_gap_us=700, seed=3, loss=0.03, dup=0.01)
    flows = eng.flow_init(n_flows, 0.2)
    reports = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
    count = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
    c = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in d.items()}
    idx = torch.from_numpy((d["flow_id"] - 1).astype(np.uint32)).cuda()
    eng.flow_reduce(flows, n_flows, idx, c["seq"], c["tx_sec"], c["tx_usec"], c["msg_len"],
                    c["rx_sec"], c["rx_usec"], reports=reports, per_flow=per_flow,
                    report_count=count)
    rng = np.random.default_rng(8)
    keys = _keys(O, n_flows, rng)
    sign = torch.zeros(n_flows, dtype=torch.uint8, device="cuda")
    items, ilen = eng.report_build(reports, n_flows, per_flow, count, dev(torch, keys), sign)
    _, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                        d["tx_usec"], d["msg_len"], d["rx_sec"], d["rx_usec"],
                                        window=0.2, per_flow=per_flow)
    assert np.array_equal(count.cpu().numpy().view(np.uint32), ocnt)
    want, wlen, _ = _oracle_items(O, keys, orep, ocnt, per_flow, np.zeros(n_flows, np.uint8))
    assert len(want) > n_flows
    items = items.cpu().numpy().reshape(-1, 52)
    for (f, j), b in want.items():
        assert items[f * per_flow + j, :len(b)].tobytes() == b, (f, j)
    assert reports.cpu().numpy().view(FLOW_REPORT_DTYPE).size == n_flows * per_flow


def _walk_corpus(oracle, rng, n):
    """MGEN_DATA payloads mixing flow commands, reports, generic items and broken items,
    packed as UDP records; also non-MGEN_DATA and corrupted records."""
    O = oracle
    pays, recs = [], []
    for i in range(n):
        items = []
        for _ in range(int(rng.integers(0, 5))):
            kind = rng.integers(0, 6)
            if kind == 0:
                st = {int(f): int(rng.integers(0, 4)) for f in
                      rng.integers(1, 48, int(rng.integers(1, 6)))}
                items.append(flow_command(st))
            elif kind in (1, 2):
                v6 = rng.random() < 0.3
                b, _ = O.report_build(addr(rng, v6), addr(rng, v6), int(rng.integers(0, 9)),
                                      int(rng.integers(0, 4)), *random_values(rng),
                                      offset=float(rng.choice([0.0, 0.5, 9.0])))
                items.append(b + bytes((-len(b)) % 4))
            elif kind == 3:
                L = int(rng.integers(1, 9)) * 4
                items.append(bytes([int(rng.integers(2, 16)), L]) + bytes(L - 2))
            elif kind == 4 and rng.random() < 0.3:
                items.append(bytes([int(rng.choice([0x07, 1, 0x12])), 0, 0, 0]))     # zero length
            elif kind == 5 and rng.random() < 0.3:
                b, _ = O.report_build(addr(rng, False), addr(rng, False), 3, 1, *random_values(rng))
                items.append(bytes([b[0], 20]) + b[2:])                                # bad length
        if rng.random() < 0.04:                                   # command longer than the rest
            items.append(flow_command({int(rng.integers(20, 41)): 1})[:-4])
        pay = b"".join(items)
        ptype = 1 if rng.random() < 0.85 else 2
        m = O.make_msg(msg_len=120 + len(pay) + int(rng.integers(0, 9)), flow_id=i + 1, seq=i,
                       payload_type=ptype, payload=pay if pay else None)
        r = bytearray(O.udp_pack(m, checksum=True))
        if i % 29 == 7:
            r[-1] ^= 0x40                                                       # bad checksum
        pays.append((ptype, pay))
        recs.append(bytes(r))
    return pays, recs


@pytest.mark.parametrize("opts", [0, 1])
def test_data_walk_and_report_recv_lines(torch, eng, oracle, opts):
    from mgen_amd import to_device
    O = oracle
    rng = np.random.default_rng(31 + opts)
    n = 600
    pays, recs = _walk_corpus(O, rng, n)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum([len(r) for r in recs])[:-1]
    slab_np = np.frombuffer(b"".join(recs) + bytes(64), np.uint8)
    slab = to_device(slab_np).view(torch.uint8)
    doffs = to_device(offs).view(torch.int64)
    dlens = to_device(np.array([len(r) for r in recs], np.int32)).view(torch.int32)
    cols = eng.unpack(slab, n, rec_off=doffs, rec_len=dlens, ext=True)
    status, nh, cmds, reps, totals = eng.data_walk(slab, n, cols, rec_off=doffs, opts=opts)
    status, nh = status.cpu().numpy(), nh.cpu().numpy()
    cmds = cmds.cpu().numpy().view(np.uint32).reshape(-1, 2)
    reps = reps.cpu().numpy().view(np.uint64).reshape(-1, 2)
    err = cols["err"].cpu().numpy()
    poff = cols["payload_off"].cpu().numpy()
    ecmd, erep = [], []
    for i, (ptype, pay) in enumerate(pays):
        if err[i] != 0 or ptype != 1:
            assert status[i] == 0xFF and nh[i] == 0, i
            continue
        st, c, r = O.data_walk(pay, controller=bool(opts))
        assert status[i] == st, (i, status[i], st, pay.hex())
        assert nh[i] == (1 if (c or r) else 0), i
        ecmd += [(i, f << 2 | s) for f, s in c]
        erep += [(i, int(offs[i]) + int(poff[i]) + o) for o in r]
    t = totals.cpu().numpy()
    assert (t[0], t[1]) == (len(ecmd), len(erep))
    assert len(ecmd) > 50 and (opts == 0 or len(erep) > 50)
    assert [tuple(map(int, x)) for x in cmds[:len(ecmd)]] == ecmd
    assert [tuple(map(int, x)) for x in reps[:len(erep)]] == erep
    assert set(status[status != 0xFF]) >= ({0, 1, 2, 3} if opts else {0, 1, 3})
    if not erep:
        return
    src = np.zeros(n, O.ADDR_DTYPE)
    for i in range(n):
        src[i] = addr(rng)[0]
    rx_sec = rng.integers(1_600_000_000, 1_800_000_000, n, dtype=np.int64).astype(np.uint32)
    rx_usec = rng.integers(0, 1_000_000, n).astype(np.uint32)
    for lopts in (0, 1):
        text, lo = eng.log_report_recv_text(slab, torch.from_numpy(reps.view(np.int64).reshape(-1)
                                                                   ).cuda(), len(erep),
                                            to_device(src.view(np.uint8)), to_device(rx_sec),
                                            to_device(rx_usec), opts=lopts)
        got = text.cpu().numpy().tobytes()
        exp = b"".join(O.log_report_recv(slab_np[o:o + 52].tobytes(), src[i], int(rx_sec[i]),
                                         int(rx_usec[i]), lopts) for i, o in erep)
        assert got == exp


def test_log_workspaces_per_stream(torch, eng, oracle):
    """Two streams formatting on one context at once (per-stream workspaces)."""
    rng = np.random.default_rng(77)
    n_flows, per_flow = 512, 4
    keys = _keys(oracle, n_flows, rng)
    reps = _reports(n_flows, per_flow, rng)
    count = np.full(n_flows, per_flow, np.uint32)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    args = (dev(torch, reps), n_flows, per_flow, dev(torch, count), dev(torch, keys))
    torch.cuda.synchronize()
    for s in (s1, s2):
        with torch.cuda.stream(s):
            sign = torch.zeros(n_flows, dtype=torch.uint8, device="cuda")
            items, _ = eng.report_build(*args, sign)
            outs.append(eng.log_report_text(items, args[0], n_flows, per_flow, args[3],
                                            opts=len(outs)))
    torch.cuda.synchronize()
    (t0, _), (t1, _) = outs
    ref0, _ = eng.log_report_text(items, args[0], n_flows, per_flow, args[3], opts=0)
    ref1, _ = eng.log_report_text(items, args[0], n_flows, per_flow, args[3], opts=1)
    assert torch.equal(t0, ref0) and torch.equal(t1, ref1)
