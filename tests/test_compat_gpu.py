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
    fin.write_bytes(b"".join(parts))
    p = subprocess.run([BIN, str(fin), str(fout)], capture_output=True, text=True, timeout=300)
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
