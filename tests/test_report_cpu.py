"""The oracle's MGEN_DATA restatements (MgenAnalytic::Report quantizers / build / parse,
REPORT lines, ProcessRecvMessage's TLV walk with MgenFlowCommand) against the reference's
documented shapes and encodings."""
import re

import numpy as np

from report_util import addr, flow_command


def test_quantizer_round_trips(oracle):
    O = oracle
    qs = [O.q_time(v) for v in np.geomspace(1e-6, 660, 500)]
    assert qs == sorted(qs) and qs[0] == 1 and qs[-1] == 255
    assert O.q_time(1e-7) == 0 and O.q_time(7e-7) == 1 and O.q_time(1000.0) == 255
    for q in (1, 10, 100, 200, 254):
        assert O.q_time(O.uq_time(q)) == q                       # quantized values are fixed
    assert O.q_rate(0.0) == 1 and O.q_rate(-5.0) == 1
    assert O.uq_rate(O.q_rate(1250.0)) == 1250.0                 # 0.3125 * 4096: exact
    assert O.q_loss(0.0) == 0 and O.q_loss(1e-9) == 1 and O.q_loss(2.0) == 65535
    assert abs(O.uq_loss(O.q_loss(0.25)) - 0.25) < 1e-5


def test_report_wire_layout(oracle):
    """include/mgenAnalytic.h:14-57: type|proto, len, flags|offset, dst, src, ports, flowId,
    windowSize, latency ave/min/max, rate, loss."""
    O = oracle
    rng = np.random.default_rng(1)
    s, d = addr(rng, False), addr(rng, False)
    b, _ = O.report_build(s, d, 7, 2, 1.0, 0.001, 0.0005, 0.002, 1000.0, 0.1)
    assert len(b) == 28 and b[0] == (1 << 4 | 2) and b[1] == 28 and (b[2] >> 5) == 1
    assert b[4:8] == bytes(d["addr"][0, :4]) and b[8:12] == bytes(s["addr"][0, :4])
    assert int.from_bytes(b[12:14], "big") == int(d["port"][0])
    assert int.from_bytes(b[16:20], "big") == 7
    b1, _ = O.report_build(s, d, 1, 1, 1.0, 0.001, 0.0005, 0.002, 1000.0, 0.1)
    assert len(b1) == 24 and (b1[2] >> 5) == 0                   # flow 1: no flow id field
    b6, _ = O.report_build(addr(rng, True), addr(rng, True), 9, 1, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0)
    assert len(b6) == 52 and b6[0] >> 4 == 2
    _, sign = O.report_build(s, d, 7, 1, 1.0, -0.5, -0.6, -0.4, 10.0, 0.0)
    b2, sign2 = O.report_build(s, d, 7, 1, 1.0, 0.5, 0.4, 0.6, 10.0, 0.0, sign=sign)
    assert sign == 1 and sign2 == 1 and (b2[2] >> 5) & 2          # the sign flag sticks


# doc/mgen.xml:2015 (local) and :3228 (remote) REPORT lines; the code adds ", count>" to the
# local form and "reporter>" to the remote one and prints no "offset>" in the local one
DOC_LOCAL = ("01:17:01.983235 REPORT proto>UDP flow>3 src>127.0.0.1/63684 dst>127.0.0.1/5002 "
             "offset>0.000000 window>1.970563 rate>10.000000 kbps loss>0.000000 latency "
             "ave>0.000119 min>0.000109 max>0.000129")
DOC_REMOTE = ("01:17:01.983235 REPORT proto>UDP flow>3 src>127.0.0.1/63684 dst>127.0.0.1/5002 "
              "sent>01:16.58.675309 offset>0.000000 window>1.970563 rate>10.000000 kbps "
              "loss>0.000000 latency ave>0.000119 min>0.000109 max>0.000129")
F = r"-?\d+\.\d{6}"
TS = r"\d\d:\d\d:\d\d\.\d{6}"
HEAD = r"(?P<ts>" + TS + r") REPORT proto>(UDP|TCP|SINK|\?\?\?) flow>\d+ src>[0-9a-f.:]+/\d+ dst>[0-9a-f.:]+/\d+ "
VALS = (r"window>" + F + r" rate>" + F + r" kbps loss>" + F + r" latency ave>" + F + r" min>" + F
        + r" max>" + F)


def test_report_lines_follow_the_doc_shape(oracle):
    O = oracle
    # the doc's own lines, with the documented differences
    assert re.fullmatch(HEAD + r"offset>" + F + " " + VALS, DOC_LOCAL)
    assert re.fullmatch(HEAD + r"sent>\S+ offset>" + F + " " + VALS, DOC_REMOTE)
    src = np.zeros(1, O.ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 63684
    src["addr"][0, :4] = [127, 0, 0, 1]
    dst = src.copy()
    dst["port"] = 5002
    b, _ = O.report_build(src, dst, 3, 1, 1.970563, 0.000119, 0.000109, 0.000129, 1250.0, 0.0)
    t = 1_700_000_000 - 1_700_000_000 % 86400 + 3600 + 17 * 60 + 1   # 01:17:01
    local = O.log_report(b, 1.970563, 1250.0, 0.0, 0.000119, 0.000109, 0.000129, 20, t,
                         983235).decode()
    assert local.endswith("\n")
    assert re.fullmatch(HEAD + VALS + r", count>\d+", local[:-1]), local
    assert local.startswith("01:17:01.983235 REPORT proto>UDP flow>3 src>127.0.0.1/63684 "
                            "dst>127.0.0.1/5002 window>1.970563 rate>10.000000 kbps loss>"
                            "0.000000 latency ave>0.000119 min>0.000109 max>0.000129")
    remote = O.log_report_recv(b, src, t, 983235).decode()
    assert re.fullmatch(HEAD + r"reporter>\S+ sent>" + TS + r" offset>" + F + " " + VALS,
                        remote[:-1]), remote


def test_data_walk_items(oracle):
    O = oracle
    rng = np.random.default_rng(4)
    s, d = addr(rng, False), addr(rng, False)
    rep, _ = O.report_build(s, d, 5, 1, 1.0, 0.001, 0.0, 0.002, 100.0, 0.0)
    cmd = flow_command({1: 1, 3: 2, 17: 3, 40: 1})
    generic = bytes([0x07, 8, 1, 2, 3, 4, 5, 6])
    st, cmds, reps = O.data_walk(cmd + rep + generic + cmd)
    assert st == 0 and cmds == [(1, 1), (3, 2), (17, 3), (40, 1)] * 2
    assert reps == [len(cmd)]
    st, cmds, reps = O.data_walk(cmd + rep, controller=False)      # reports skipped
    assert st == 0 and reps == [] and len(cmds) == 4
    assert O.data_walk(cmd[:-1])[0] == 1                          # command longer than the rest
    bad = bytearray(rep)
    bad[1] = 20
    assert O.data_walk(bytes(bad))[0] == 2                        # invalid report length
    assert O.data_walk(bytes([0x07, 0, 1]))[0] == 3               # zero length: no progress
    assert O.data_walk(flow_command({45: 1}))[1] == []            # beyond MAX_FLOW
