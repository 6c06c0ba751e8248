"""GPU parity of pcap2mgen (src/common/pcap2mgen.cpp:252-482): the device pipeline
(mgen_amd.pcap: mgenx_pcap_parse -> unpack -> FindFlow / Update -> report / RECV / received
REPORT lines -> mgenx_text_interleave) against the oracle's sequential main loop, byte for
byte, over mixed captures (Ethernet / 802.1Q / Linux SLL, IPv4 / IPv6, nanosecond and
byte-swapped files, skipped frames, MGEN_DATA reports, analytics on / off, rxlog on / off).
Also the building blocks on their own: the frame walk per record, mgenx_text_interleave over
every source kind, and mgenx_flow_reduce_ex's closing-record index."""
import numpy as np
import pytest

import pcap_util as P

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


def _diff(got: bytes, want: bytes):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    for k, (a, b) in enumerate(zip(gl, wl)):
        if a != b:
            return f"line {k}:\n got  {a!r}\n want {b!r}"
    return f"line counts {len(gl)} vs {len(wl)}"


@pytest.mark.parametrize("link,nsec,swapped", [(1, False, False), (113, False, False),
                                               (1, True, True)])
def test_frame_walk_matches_oracle(eng, torch, oracle, link, nsec, swapped):
    import mgen_amd
    f = P.capture(oracle, seed=21 + link, n=400, link=link, nsec=nsec, swapped=swapped)
    offs, info = mgen_amd.pcap_index(f)
    buf = torch.from_numpy(np.frombuffer(f, np.uint8).copy()).cuda()
    po = torch.from_numpy(offs.view(np.int64).copy()).cuda()
    n = len(offs)
    p = eng.pcap_parse(buf, po, n, info.link_type, info.flags)
    torch.cuda.synchronize()
    src = p["src"].cpu().numpy().view(mgen_amd.ADDR_DTYPE)
    for i, o in enumerate(offs):
        st, uo, ul, s, ttl, sec, usec = oracle.pcap_frame(f[int(o):], link, info.flags)
        assert int(p["status"][i]) == st, i
        assert int(p["rx_sec"][i]) == sec and int(p["rx_usec"][i]) == usec
        if st == 0:
            assert int(p["udp_off"][i]) == int(o) + uo and int(p["udp_len"][i]) == ul
            assert int(p["ttl"][i]) == ttl
            assert src[i]["type"] == s["type"] and src[i]["port"] == s["port"]
            assert bytes(src[i]["addr"][:s["len"]]) == bytes(s["addr"][:s["len"]])
        else:
            assert int(p["udp_len"][i]) == 0


@pytest.mark.parametrize("case", [
    dict(seed=1), dict(seed=2, analytics=True), dict(seed=3, analytics=True, window=0.05),
    dict(seed=4, link=113, analytics=True), dict(seed=5, nsec=True, swapped=True),
    dict(seed=6, analytics=True, log_rx=False), dict(seed=7, epoch=True, analytics=True,
                                                    window=0.02)])
def test_pcap2mgen_matches_oracle(eng, oracle, case):
    from mgen_amd.pcap import Pcap2Mgen
    c = dict(case)
    seed = c.pop("seed")
    link, nsec, sw = c.pop("link", 1), c.pop("nsec", False), c.pop("swapped", False)
    f = P.capture(oracle, seed=seed, n=700, link=link, nsec=nsec, swapped=sw)
    an, rx, w, ep = (c.get("analytics", False), c.get("log_rx", True), c.get("window", 1.0),
                     c.get("epoch", False))
    want, _ = oracle.pcap2mgen(f, analytics=an, log_rx=rx, window=w,
                               opts=oracle.LOG_EPOCH if ep else 0)
    got = Pcap2Mgen(eng, analytics=an, log_rx=rx, window=w, epoch=ep).run(f)
    assert len(want) > 0
    assert got == want, _diff(got, want)


def test_pcap2mgen_many_flows_windows(eng, oracle):
    """Hundreds of flows over 40 s of capture with a 0.5 s window: many reports per flow."""
    from mgen_amd.pcap import Pcap2Mgen
    rng = np.random.default_rng(99)
    recs, seqs = [], {}
    t = 1_650_000_000 * 1_000_000
    src = [bytes([10, 1, k // 256, k % 256]) for k in range(300)]
    for i in range(6000):
        t += int(rng.integers(1000, 12000))
        k = int(rng.integers(0, 300))
        s = seqs.get(k, 0)
        seqs[k] = s + (1 if rng.random() > 0.02 else 2)
        pay = P.mgen_payload(oracle, 1 + k % 7, s, divmod(t - int(rng.integers(50, 900)),
                                                          1_000_000), int(rng.integers(64, 300)))
        fr = P.eth(P.ipv4(P.udp(pay, 20000 + k, 5000), src[k], bytes([10, 0, 0, 2])))
        recs.append((*divmod(t, 1_000_000), fr))
    f = P.pcap(recs)
    want, _ = oracle.pcap2mgen(f, analytics=True, window=0.5)
    got = Pcap2Mgen(eng, analytics=True, window=0.5).run(f)
    assert want.count(b" REPORT ") > 500
    assert got == want, _diff(got, want)
    # the first flow table too small for the 300 flows (it holds 2 x 64 slots): the lookup
    # overflows and is redone on a table for every packet -- same log
    small = Pcap2Mgen(eng, analytics=True, window=0.5)
    small.FIRST_FLOWS = 40
    assert small.run(f) == want


def test_pcap2mgen_empty_and_nothing_mgen(eng, oracle):
    from mgen_amd.pcap import Pcap2Mgen
    empty = P.pcap([])
    assert Pcap2Mgen(eng, analytics=True).run(empty) == b""
    junk = P.pcap([(1, 2, P.eth(bytes(28), etype=0x0806))] * 5)
    assert Pcap2Mgen(eng, analytics=True).run(junk) == oracle.pcap2mgen(junk, analytics=True)[0]


def test_text_interleave_kinds(eng, torch):
    """Every source kind against a Python concatenation: per-record lines (some empty), sorted
    owners with gaps and repeats (stride 4, as the data walk's u64 pairs), a record->line map
    and a scattered line->record list."""
    from mgen_amd import TEXT_MAP, TEXT_OWNER, TEXT_PER_RECORD, TEXT_SCATTER
    rng = np.random.default_rng(5)
    n = 3000

    def src(lines):
        text = b"".join(lines)
        off = np.concatenate([[0], np.cumsum([len(x) for x in lines])]).astype(np.int64)
        t = torch.from_numpy(np.frombuffer(text + b"\0", np.uint8).copy()).cuda()
        return t, torch.from_numpy(off).cuda()

    per = [b"" if rng.random() < 0.2 else b"r%d:%s\n" % (i, b"x" * int(rng.integers(0, 90)))
           for i in range(n)]
    owners = np.sort(rng.integers(0, n, 1500))
    own_lines = [b"o%d.%d\n" % (o, k) for k, o in enumerate(owners)]
    pairs = np.zeros((1500, 2), np.int64)
    pairs[:, 0] = owners
    map_rec = rng.choice(n, 400, replace=False)
    map_lines = [b"m%d\n" % r for r in map_rec]
    rec_to_line = np.full(n, -1, np.int32)
    rec_to_line[map_rec] = np.arange(400)
    sc_rec = rng.choice(n, 300, replace=False).astype(np.int32)
    sc_rec[::7] = -1                                           # dropped lines
    sc_lines = [b"s%d\n" % k for k in range(300)]
    s0, s1, s2, s3 = src(per), src(own_lines), src(map_lines), src(sc_lines)
    pt = torch.from_numpy(pairs.reshape(-1).copy()).cuda()
    out, rec_off = eng.text_interleave([
        (TEXT_SCATTER, s3[0], s3[1], 300, torch.from_numpy(sc_rec).cuda(), 1),
        (TEXT_PER_RECORD, s0[0], s0[1], n, None, 1),
        (TEXT_OWNER, s1[0], s1[1], 1500, pt.view(torch.int32), 4),
        (TEXT_MAP, s2[0], s2[1], 400, torch.from_numpy(rec_to_line).cuda(), 1)], n)
    want = []
    for i in range(n):
        w = b""
        for k in np.nonzero(sc_rec == i)[0]:
            w += sc_lines[k]
        w += per[i]
        for k in np.nonzero(owners == i)[0]:
            w += own_lines[k]
        if rec_to_line[i] >= 0:
            w += map_lines[rec_to_line[i]]
        want.append(w)
    assert out.cpu().numpy().tobytes() == b"".join(want)
    ro = rec_off.cpu().numpy()
    assert (np.diff(ro) == [len(w) for w in want]).all()


def test_flow_reduce_report_record(eng, torch, oracle):
    """mgenx_flow_reduce_ex: each kept report's closing record is the record whose Update
    returned true in the oracle (records interleaved over flows)."""
    rng = np.random.default_rng(8)
    n, nf = 20000, 37
    fidx = rng.integers(0, nf, n).astype(np.uint32)
    t = 1_700_000_000_000_000 + np.cumsum(rng.integers(100, 3000, n))
    rx_sec, rx_usec = (t // 1_000_000).astype(np.uint32), (t % 1_000_000).astype(np.uint32)
    tx = t - rng.integers(10, 900, n)
    tx_sec, tx_usec = (tx // 1_000_000).astype(np.uint32), (tx % 1_000_000).astype(np.uint32)
    seq = np.zeros(n, np.uint32)
    cnt = np.zeros(nf, np.int64)
    for i in range(n):
        seq[i] = cnt[fidx[i]]
        cnt[fidx[i]] += 1
    ml = rng.integers(28, 1400, n).astype(np.uint16)
    a = [oracle.AnalyticOracle(0.2) for _ in range(nf)]
    closing = [[] for _ in range(nf)]
    for i in range(n):
        f = int(fidx[i])
        if a[f].update(int(rx_sec[i]), int(rx_usec[i]), int(ml[i]), int(tx_sec[i]),
                       int(tx_usec[i]), int(seq[i])):
            closing[f].append(i)
    from mgen_amd import FLOW_REPORT_DTYPE
    per = 64
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x).copy()).cuda()  # noqa: E731
    flows = eng.flow_init(nf, 0.2)
    reps = torch.zeros(nf * per * FLOW_REPORT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    rr = torch.full((nf * per,), -1, dtype=torch.int32, device="cuda")
    count = eng.flow_reduce(flows, nf, d(fidx.view(np.int32)), d(seq.view(np.int32)),
                            d(tx_sec.view(np.int32)), d(tx_usec.view(np.int32)),
                            d(ml.view(np.int16)), d(rx_sec.view(np.int32)),
                            d(rx_usec.view(np.int32)), n=n, reports=reps, per_flow=per,
                            report_rec=rr)
    torch.cuda.synchronize()
    c = count.cpu().numpy()
    r = rr.cpu().numpy().reshape(nf, per)
    for f in range(nf):
        assert c[f] == len(closing[f])
        k = min(per, len(closing[f]))
        assert list(r[f, :k]) == closing[f][:k]
        assert (r[f, k:] == -1).all()


def test_pcap2mgen_cli(oracle, tmp_path):
    """tools/pcap2mgen (the reference's command line over include/mgenx_pcap.hpp): infile /
    outfile, -analytic, +window, +rxlog, stdin / stdout."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "pcap2mgen")
    f = P.capture(oracle, seed=31, n=900)
    pin = tmp_path / "in.pcap"
    pin.write_bytes(f)
    out = tmp_path / "out.log"
    r = subprocess.run([exe, "infile", str(pin), "outfile", str(out), "ANALYTIC",
                        "win", "0.1"], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    want, _ = oracle.pcap2mgen(f, analytics=True, window=0.1)
    assert out.read_bytes() == want, _diff(out.read_bytes(), want)
    r = subprocess.run([exe, "rxlog", "OFF", "rep"], input=f, capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == oracle.pcap2mgen(f, analytics=True, log_rx=False)[0]


@pytest.mark.parametrize("snaplen,analytics", [(128, True), (96, False), (70, True)])
def test_snaplen_capture_matches_oracle(eng, oracle, snaplen, analytics):
    """A capture taken with a snapshot length (tcpdump -s N): the reference parses each frame
    by its wire length and Unpacks the UDP payload from the captured bytes, so every packet
    whose UDP header and MIN_SIZE payload bytes were captured still logs its RECV line
    (payload bytes past the capture read as zero here: mgenx_pcap_snap); shorter captures
    are skipped.  Device pipeline == oracle, byte for byte."""
    import mgen_amd
    from mgen_amd.pcap import Pcap2Mgen
    f = P.snap(P.capture(oracle, seed=40 + snaplen, n=600), snaplen)
    _, info = mgen_amd.pcap_index(f)
    assert info.snap_bytes > 0
    want, st = oracle.pcap2mgen(f, analytics=analytics, window=0.05)
    assert (st == 7).sum() > 100, np.bincount(st)
    got = Pcap2Mgen(eng, analytics=analytics, window=0.05).run(f)
    assert got == want, _diff(got, want)
    if snaplen == 128:
        assert want.count(b" RECV ") > 300
