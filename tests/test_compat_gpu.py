"""GPU: the drop-in MgenMsg / MgenPayload / MgenAnalytic shim (include/mgenx_compat), driven
in the reference's own call shapes by tests/cpp/compat_shapes (C++, links libmgenx):

  * UDP send (mgenTransport.cpp:1011-1031): LAST_BUFFER, Pack, WriteChecksum -- message by
    message with checksum off and on, and as one MgenMsg::PackBatch -- against the golden
    pack slabs (tests/golden/udp_matrix.npz) byte for byte;
  * UDP receive (mgenTransport.cpp:955-975): Unpack, ComputeCRC32 over len-4, compare with
    the BE trailer, SetChecksumError -- per datagram (force off / on) and as one
    UnpackBatch + ComputeCRC32Batch -- against the golden decoded fields (8213 vectors);
  * Mgen::UpdateRecvAnalytics (mgen.cpp:1034-1067): FindFlow / Init / Insert / Update /
    GetReport per record and as one MgenAnalytic::UpdateBatch, against the oracle's
    MgenAnalytic restatement (parity unpinned at protolib: see oracle/mgen_oracle.h);
  * MgenPayload hex strings and MgenFlowCommand status bits.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "compat_shapes")
BIN_PL = BIN + "_pl"   # the shim's MGENX_WITH_PROTOLIB branch (protolib-shaped test headers)
GOLD = os.path.join(ROOT, "tests", "golden", "udp_matrix.npz")

OUT_DTYPE = np.dtype([
    ("ok", "u1"), ("err", "u1"), ("version", "u1"), ("flags", "u1"), ("msg_len", "<u2"),
    ("hdr_len", "<u2"), ("flow_id", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"),
    ("tx_usec", "<u4"), ("dst_port", "<u2"), ("dst_type", "u1"), ("dst_len", "u1"),
    ("dst_addr", "u1", 16), ("host_port", "<u2"), ("host_type", "u1"), ("host_len", "u1"),
    ("host_addr", "u1", 16), ("latitude", "<f8"), ("longitude", "<f8"), ("alt", "<i4"),
    ("gps_status", "u1"), ("payload_type", "u1"), ("payload_len", "<u2"),
    ("payload_off", "<u4")])
REPORT_MAX = 4 + 2 * 16 + 4 * 4
LOCAL_TZ, LOCAL_OFFSET = "XYZ3", -3 * 3600   # POSIX TZ: local time = UTC - 3 h
REP_DTYPE = np.dtype([
    ("updated", "u1"), ("rsv", "u1", 7), ("duration", "<f8"), ("rate", "<f8"), ("loss", "<f8"),
    ("latency_ave", "<f8"), ("latency_min", "<f8"), ("latency_max", "<f8"),
    ("msg_count", "<u8"), ("item", "u1", REPORT_MAX)])
SAME = ("ok", "err", "version", "flags", "msg_len", "hdr_len", "flow_id", "seq_num", "tx_sec",
        "tx_usec", "dst_port", "dst_type", "dst_len", "dst_addr", "host_port", "host_type",
        "host_len", "host_addr", "alt", "gps_status", "payload_type", "payload_len",
        "payload_off")


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    from mgen_amd.workloads import poisson_flows
    assert os.path.exists(BIN), "tests/cpp/compat_shapes not built (__graft_entry__.build())"
    g = dict(np.load(GOLD, allow_pickle=False))
    a = poisson_flows(6000, n_flows=12, mean_gap_us=20000, reorder=4)
    window = 1.0
    parts = [struct.pack("<IIIIQQ", len(g["tmpl"]), len(g["pool"]), len(g["desc"]),
                         len(g["unpack_lens"]), int(g["slab_bytes"][0]), len(g["unpack_slab"])),
             g["tmpl"].tobytes(), g["pool"].tobytes(), g["desc"].tobytes(),
             g["offs"].astype(np.uint64).tobytes(), g["unpack_offs"].astype(np.uint64).tobytes(),
             g["unpack_lens"].astype(np.uint32).tobytes(), g["unpack_slab"].tobytes(),
             struct.pack("<Id", len(a["seq"]), window)]
    for k in ("flow_id", "seq", "tx_sec", "tx_usec", "rx_sec", "rx_usec"):
        parts.append(a[k].astype(np.uint32).tobytes())
    parts.append(a["msg_len"].astype(np.uint16).tobytes())
    d = tmp_path_factory.mktemp("compat")
    fin, fout = d / "in.bin", d / "out.bin"
    logs = d / "logs"
    logs.mkdir()
    fin.write_bytes(b"".join(parts))
    env = dict(os.environ, TZ=LOCAL_TZ)
    p = subprocess.run([BIN, str(fin), str(fout), str(logs)], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    raw = fout.read_bytes()
    nd, sb, nu, na = len(g["desc"]), int(g["slab_bytes"][0]), len(g["unpack_lens"]), len(a["seq"])
    out, pos = {}, 0

    def take(key, nbytes, dtype):
        nonlocal pos
        out[key] = np.frombuffer(raw[pos:pos + nbytes], dtype).copy()
        pos += nbytes
    for name in ("ck0", "ck1", "batch"):
        take(f"lens_{name}", nd * 4, np.uint32)
        take(f"slab_{name}", sb, np.uint8)
    for name in ("udp", "udp_force", "batch"):
        take(f"recv_{name}", nu * OUT_DTYPE.itemsize, OUT_DTYPE)
    for name in ("seq", "batch"):
        take(f"an_{name}", na * REP_DTYPE.itemsize, REP_DTYPE)
    out["tail"] = raw[pos:].decode()
    out["logs"] = {f.name: f.read_bytes() for f in logs.iterdir()}
    # the protolib branch: the same program, the same input
    logs_pl = d / "logs_pl"
    logs_pl.mkdir()
    fout_pl = d / "out_pl.bin"
    p = subprocess.run([BIN_PL, str(fin), str(fout_pl), str(logs_pl)], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    out["pl_raw"] = fout_pl.read_bytes()
    out["pl_logs"] = {f.name: f.read_bytes() for f in logs_pl.iterdir()}
    out["raw"] = raw
    return g, a, window, out


def test_send_shape_matches_golden(run):
    g, _, _, out = run
    for ck in (0, 1):
        assert np.array_equal(out[f"lens_ck{ck}"], g[f"pack_lens_ck{ck}_rf0"]), ck
        assert np.array_equal(out[f"slab_ck{ck}"], g[f"pack_slab_ck{ck}_rf0"]), ck


def test_pack_batch_matches_golden(run):
    g, _, _, out = run
    assert np.array_equal(out["lens_batch"], g["pack_lens_ck1_rf0"])
    assert np.array_equal(out["slab_batch"], g["pack_slab_ck1_rf0"])


def _check_fields(got, want, label):
    for k in SAME:
        bad = np.nonzero(got[k] != want[k])[0] if got[k].ndim == 1 else \
            np.nonzero((got[k] != want[k]).any(axis=1))[0]
        assert bad.size == 0, (label, k, bad[:8], got[k][bad[:3]], want[k][bad[:3]])
    # Unpack's GPS decode, ntohl(word) / 60000.0 - 180.0 (mgenMsg.cpp:453,457), as doubles
    for k, r in (("latitude", "lat_raw"), ("longitude", "lon_raw")):
        exp = want[r].astype(np.float64) / 60000.0 - 180.0
        assert np.array_equal(got[k].view(np.uint64), exp.view(np.uint64)), (label, k)


def test_receive_shape_matches_golden(run):
    g, _, _, out = run
    _check_fields(out["recv_udp"], g["unpack_fields_udp"], "udp")
    _check_fields(out["recv_udp_force"], g["unpack_fields_udp_force"], "udp_force")


def test_unpack_batch_matches_golden(run):
    g, _, _, out = run
    _check_fields(out["recv_batch"], g["unpack_fields_udp"], "batch")


def test_analytics_shape_matches_oracle(run, oracle):
    _, a, window, out = run
    flows = {}
    seq_rep, batch_rep = out["an_seq"], out["an_batch"]
    n_upd = 0
    for i in range(len(a["seq"])):
        f = int(a["flow_id"][i])
        if f not in flows:
            flows[f] = oracle.AnalyticOracle(window)
        o = flows[f]
        upd = o.update(int(a["rx_sec"][i]), int(a["rx_usec"][i]), int(a["msg_len"][i]),
                       int(a["tx_sec"][i]), int(a["tx_usec"][i]), int(a["seq"][i]))
        assert bool(seq_rep["updated"][i]) == upd, i
        assert bool(batch_rep["updated"][i]) == upd, i
        if not upd:
            continue
        n_upd += 1
        r, s = seq_rep[i], o.a
        assert r["duration"] == s.report_duration and r["msg_count"] == s.report_msg_count, i
        assert r["rate"] == s.report_rate_ave and r["loss"] == s.report_loss_ave, i
        assert r["latency_ave"] == s.report_latency_ave, i
        assert r["latency_min"] == s.report_latency_min, i
        assert r["latency_max"] == s.report_latency_max, i
        item = r["item"]
        assert item[0] >> 4 == 1 and item[0] & 0x0F == 1        # REPORT_FLOW_IPv4, UDP
        assert item[1] == (24 if f == 1 else 28)                   # len (flowId field iff != 1)
    assert n_upd > 50


def test_payload_and_flow_command(run):
    from mgen_amd._abi import hex_payload
    out = run[3]
    s1, s2, cmd, _ = out["tail"].split("|")
    assert s1 == hex_payload("abc").hex().upper() == "ABC0"
    assert s2 == "FFFEFFFF"
    assert cmd == "1 3 2 0 40"


# ---------------------------------------------------------------- logging shapes
def _recv_inputs(g):
    from oracle.oracle import ADDR_DTYPE
    n = len(g["unpack_lens"])
    src = np.zeros(n, ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 59273
    src["addr"][:, :4] = [127, 0, 0, 1]
    i = np.arange(n)
    return src, (1700000001 + i // 1000).astype(np.uint32), ((i * 37) % 1000000).astype(np.uint32)


def test_send_log_matches_oracle(run, oracle):
    """LogSendEvent (text and binary) after each UDP send == the oracle's SEND events."""
    g, _, _, out = run
    sp = np.full(len(g["tmpl"]), 5001, np.uint16)
    for name, binary in (("send.txt", False), ("send.bin", True)):
        want = oracle.log_send_batch(g["tmpl"], g["desc"], g["pool"], sp, protocol=1,
                                     checksum=True, binary=binary)
        assert out["logs"][name] == want, name


def test_recv_log_matches_oracle(run, oracle):
    """LogRecvEvent / LogRecvError as MgenUdpTransport::OnEvent calls them (text and binary)
    == the oracle's RECV / RERR events for the same received records."""
    g, _, _, out = run
    f = g["unpack_fields_udp"]
    src, rs, ru = _recv_inputs(g)
    want = oracle.log_recv_text(f, g["unpack_slab"], g["unpack_offs"], src, rs, ru, protocol=1)
    got = out["logs"]["recv.txt"]
    if got != want:
        gl, wl = got.split(b"\n"), want.split(b"\n")
        k = next(j for j in range(min(len(gl), len(wl))) if gl[j] != wl[j])
        pytest.fail(f"line {k}: {gl[k][:300]!r} != {wl[k][:300]!r}")
    wantb = oracle.log_recv_binary(f, g["unpack_slab"], g["unpack_offs"], src, rs, ru, protocol=1,
                                   rec_len=g["unpack_lens"])
    assert out["logs"]["recv.bin"] == wantb


def test_recv_log_local_time_and_epoch(run, oracle):
    g, _, _, out = run
    f = g["unpack_fields_udp"]
    src, rs, ru = _recv_inputs(g)
    ok = np.nonzero(f["err"][:64] == 0)[0]
    fl = f[ok].copy()
    fl["tx_sec"] = (fl["tx_sec"].astype(np.int64) + LOCAL_OFFSET).astype(np.uint32)
    want = oracle.log_recv_text(fl, g["unpack_slab"], g["unpack_offs"][ok], src[ok],
                                (rs[ok].astype(np.int64) + LOCAL_OFFSET).astype(np.uint32), ru[ok],
                                protocol=1)
    assert out["logs"]["recv_local.txt"] == want
    want = oracle.log_recv_text(f[ok], g["unpack_slab"], g["unpack_offs"][ok], src[ok], rs[ok],
                                ru[ok], protocol=1, opts=oracle.LOG_EPOCH)
    assert out["logs"]["recv_epoch.txt"] == want


def test_convert_binary_log_of_shim_log(run, oracle):
    """The shim's binary RECV log, converted back by MgenMsg::ConvertBinaryLog, == the
    oracle's conversion of the same file (and the file == the oracle's binary records)."""
    g, _, _, out = run
    f = g["unpack_fields_udp"]
    src, rs, ru = _recv_inputs(g)
    ok = np.nonzero(f["err"] == 0)[0]
    log = out["logs"]["recv_ok.bin"]
    hdr = b"mgen version=5.1.1 type=binary_log\n\0"
    assert log == hdr + oracle.log_recv_binary(f[ok], g["unpack_slab"], g["unpack_offs"][ok],
                                               src[ok], rs[ok], ru[ok], protocol=1,
                                               rec_len=g["unpack_lens"][ok])
    text, status, nrec = oracle.convert_binary_log(log)
    assert nrec == ok.size
    assert out["logs"]["convert.txt"] == text + (b"#1\n" if status == 0 else b"#0\n")


def test_update_recv_analytics_log_lines(run, oracle):
    """Mgen::UpdateRecvAnalytics' analytic->Log after each window close == the oracle's
    REPORT line of that report (MgenAnalytic::Log), and GetWindowEnd == the oracle's."""
    _, a, window, out = run
    rep = out["an_seq"]
    lines = []
    flows = {}
    for i in np.nonzero(rep["updated"])[0]:
        r = rep[i]
        lines.append(oracle.log_report(bytes(r["item"]), r["duration"], r["rate"], r["loss"],
                                       r["latency_ave"], r["latency_min"], r["latency_max"],
                                       int(r["msg_count"]), int(a["rx_sec"][i]),
                                       int(a["rx_usec"][i])))
    assert out["logs"]["analytic.txt"] == b"".join(lines)
    order = []
    for i in range(len(a["seq"])):
        fid = int(a["flow_id"][i])
        if fid not in flows:
            flows[fid] = oracle.AnalyticOracle(window)
            order.append(fid)
        flows[fid].update(int(a["rx_sec"][i]), int(a["rx_usec"][i]), int(a["msg_len"][i]),
                          int(a["tx_sec"][i]), int(a["tx_usec"][i]), int(a["seq"][i]))
    ends = np.frombuffer(out["logs"]["window_end.bin"], np.int64).reshape(-1, 2)
    want = [(flows[fid].a.window_end.sec, flows[fid].a.window_end.usec) for fid in order]
    assert [tuple(x) for x in ends.tolist()] == want


def _conn_expected():
    """LogTcpConnectionEvent (mgenMsg.cpp:741-944) for the events compat_shapes logs."""
    names = ["ACCEPT", "ON", "CONNECT", "DISCONNECT", "RECONNECT", "SHUTDOWN", "OFF"]
    codes = [11, 10, 13, 12, 16, 15, 14]
    txt, binv = [], []
    for host in (0, 1):
        for client in (0, 1):
            for name, code in zip(names, codes):
                flow = 7 + host
                ts = "22:15:23.004567 "   # 1700000123 s, GMT (localTime false)
                if name == "ACCEPT":
                    line = "ACCEPT src>10.0.0.1/5000 dstPort>5001"
                elif name in ("ON", "CONNECT") or client:
                    line = f"{name} flow>{flow} srcPort>5001 dst>10.0.0.1/5000 "
                elif name == "SHUTDOWN":
                    line = "SHUTDOWN src>10.0.0.1/5000 dstPort>5001"
                else:
                    line = f"{name} src>10.0.0.1/5000 dstPort>5001 "
                line += " host>2001:db8::1/6000\n" if host else "\n"
                txt.append(ts + line)
                rl = 12 + 4 + 2 + 4 + (16 + 4 if host else 0)
                b = bytes([code, 2]) + rl.to_bytes(2, "big") + (1700000123).to_bytes(4, "big")
                b += (4567).to_bytes(4, "big") + (5000).to_bytes(2, "big") + bytes([1, 4, 10, 0, 0, 1])
                b += (5001).to_bytes(2, "big") + flow.to_bytes(4, "big")
                if host:
                    b += (6000).to_bytes(2, "big") + bytes([2, 16, 0x20, 1, 0x0d, 0xb8] + [0] * 11 + [1])
                binv.append(b)
    return "".join(txt).encode(), b"".join(binv)


def test_tcp_connection_and_drec_events(run):
    out = run[3]
    t, b = _conn_expected()
    assert out["logs"]["conn.txt"] == t
    assert out["logs"]["conn.bin"] == b
    # DREC events carry the wall-clock time: compare with the time fields masked
    lines = out["logs"]["drec.txt"].decode().splitlines()
    assert [ln.split(" ", 1)[1] for ln in lines] == [
        "LISTEN proto>UDP port>5000", "IGNORE proto>TCP port>5001",
        "JOIN group>224.1.2.3 interface>eth0 port>5002", "LEAVE group>224.1.2.3 source>10.0.0.9"]
    d = out["logs"]["drec.bin"]
    recs, p = [], 0
    while p < len(d):
        rl = int.from_bytes(d[p + 2:p + 4], "big")
        recs.append(d[p:p + 2] + d[p + 12:p + 4 + rl])
        p += 4 + rl
    assert recs == [bytes([4, 0, 1, 0]) + (5000).to_bytes(2, "big"),
                    bytes([5, 0, 2, 0]) + (5001).to_bytes(2, "big"),
                    bytes([6, 0]) + (5002).to_bytes(2, "little") + bytes([1, 4, 224, 1, 2, 3, 4]) + b"eth0",
                    bytes([7, 0]) + bytes([0, 0]) + bytes([1, 4, 224, 1, 2, 3, 0])]


def test_protolib_branch_same_results(run):
    """compat_shapes built through the shim's MGENX_WITH_PROTOLIB branch (what an MGEN build
    compiles, with protolib / Mgen / DrecEvent-shaped test headers) writes the same bytes:
    sends, receives, analytics and every log but the wall-clock DREC times."""
    out = run[3]
    assert out["pl_raw"] == out["raw"]
    for name, data in out["logs"].items():
        if name.startswith("drec"):
            continue
        assert out["pl_logs"][name] == data, name


def test_shim_single_call_latency():
    """The shim's single-message calls are synchronous batches of one: measure them (and the
    batch forms) so the cost a one-at-a-time transport pays is on record."""
    import json
    exe = os.path.join(ROOT, "tests", "cpp", "shim_latency")
    p = subprocess.run([exe, "1000"], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    print("shim latency:", json.dumps(d))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "shim_latency.json"), "w") as f:
        json.dump(d, f)
    s = d["single_call_median_us"]
    assert all(v > 0 for v in s.values())
    # a batch amortises the round trip: per message far below one single call
    assert d["batch_per_msg_us"]["unpack_4096"] < s["unpack"] / 10
