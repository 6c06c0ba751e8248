"""ConvertBinaryLog on the CPU side (mgenMsg.cpp:1417-1900): the oracle's restatement on
hand-built records (exact expected lines from the reference's format strings), a round trip
through the binary RECV / SEND writers, the header and stop rules, and libmgenx's host index
walk (mgenx_binlog_index: host code, no GPU) against the oracle's stops."""
import numpy as np
import pytest

from oracle import oracle as O
import binlog_util as B


def _conv(parts, **kw):
    return O.convert_binary_log(B.binlog(parts), **kw)


def test_event_lines_exact():
    v6 = bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [5])
    parts = [B.start(3661, 7), B.listen(3662, 8, 1, 5000), B.listen(3662, 9, 2, 80, ignore=True),
             B.join(3663, 10, bytes([224, 1, 2, 3]), 5000, b"eth0"),
             B.join(3663, 11, v6, 0, b"", leave=True),
             B.conn(10, 3664, 12, bytes([10, 0, 0, 9]), 5001, 4000, 3),
             B.conn(12, 3664, 13, bytes([10, 0, 0, 9]), 5001, 4000, 0,
                    host=(bytes([1, 2, 3, 4]), 99)),
             B.conn(14, 3664, 14, bytes([10, 0, 0, 9]), 5001, 4000, 3), B.stop(3665, 15)]
    text, st, n = _conv(parts)
    assert st == 0 and n == len(parts)
    assert text.decode().split("\n") == [
        "01:01:01.000007 START",
        "01:01:02.000008 LISTEN proto>UDP port>5000",
        "01:01:02.000009 IGNORE proto>TCP port>80",
        "01:01:03.000010 JOIN group>224.1.2.3 interface>eth0 port>5000",
        "01:01:03.000011 LEAVE group>2001:db8::5",
        "01:01:04.000012 ON flow>3 srcPort>4000 dst>10.0.0.9/5001",
        "01:01:04.000013 DISCONNECT src>10.0.0.9/5001 dstPort>4000host>1.2.3.4/99",
        "01:01:04.000014 OFF flow>3 srcPort>4000 dst>10.0.0.9/5001",
        "01:01:05.000015 STOP", ""]
    text, *_ = _conv(parts[:2], opts=O.LOG_EPOCH)
    assert text == b"3661.000007 START\n3662.000008 LISTEN proto>UDP port>5000\n"


def test_recv_send_round_trip():
    """Binary RECV records -> text == the direct RECV text of the same receptions with the
    converter's ttl (log_flush) and srcPort 0 / tx-time SEND lines."""
    recs = B.recv_records(O, n=120)
    text, st, n = _conv(recs)
    assert st == 0 and n == 120
    lines = text.split(b"\n")[:-1]
    recv = [l for l in lines if b" RECV " in l]
    assert len(recv) == 120 and all(b" ttl>0 " in l for l in recv)
    t2, *_ = _conv(recs, flush=True)
    assert t2 == text.replace(b" ttl>0 ", b" ttl>1 ")
    t3, *_ = _conv(recs, log_rx=False)
    assert b" RECV " not in t3 and t3 == b"".join(l + b"\n" for l in lines if b" REPORT " in l)
    sends = B.send_records(O, n=40)
    t4, st, n = _conv(sends)
    assert st == 0 and n == len(sends) and t4.count(b" SEND ") == len(sends)
    assert all(b" srcPort>0 dst>" in l for l in t4.split(b"\n")[:-1])
    t5, st, n = _conv(B.data_recv_records(O, n=10))
    assert st == 0 and n == 10 and t5.count(b" RECV ") == 10 and t5.count(b" REPORT ") >= 10


@pytest.mark.parametrize("case,status,keep", [
    ("rerr", 3, 2), ("unknown", 3, 2), ("badaddr", 3, 2), ("toolong", 2, 2), ("short", 4, 2)])
def test_stops(case, status, keep):
    import struct
    parts = [B.start(1, 2), B.listen(1, 3, 1, 7)]
    if case == "rerr":
        bad = struct.pack(">BBH", 2, 0, 20) + bytes(20)
    elif case == "unknown":
        bad = B.ev_time(40, 1, 1)
    elif case == "badaddr":
        bad = bytearray(B.conn(10, 1, 1, bytes(4), 1, 1, 1))
        bad[14] = 7
        bad = bytes(bad)
    elif case == "toolong":
        bad = struct.pack(">BBH", 8, 0, 1025) + bytes(1025)
    else:
        bad = B.stop(5, 5)[:-2]
    tail = [] if case == "short" else [B.stop(9, 9)]    # a short record ends the file
    text, st, n = _conv(parts + [bad] + tail)
    assert st == status and n == keep and text.count(b"\n") == keep
    import mgen_amd
    offs, info = mgen_amd.binlog_index(B.binlog(parts + [bad] + tail))
    assert info.status == status and info.n_records == keep and len(offs) == keep


def test_header_rules():
    import mgen_amd
    for hdr, ok in [(B.HEADER, True), (b"mgen version=4.2 type=binary_log\n\0", True),
                    (b"mgen version=3.0 type=binary_log\n\0", False),
                    (b"mgen version=5.1.1 type=text_log\n\0", False),
                    (b"MGEN version=5 type=binary_log\n\0", False),
                    (b"mgen type=binary_log\n\0", False), (b"mgen version=5 type=binary_log", False)]:
        log = hdr + B.start(1, 1)
        text, st, _ = O.convert_binary_log(log)
        _, info = mgen_amd.binlog_index(log)
        assert (st == 0) == ok and (info.status == 0) == ok, hdr
        assert (text == b"00:00:01.000001 START\n") == ok


def test_index_matches_oracle_on_mixed_logs():
    import mgen_amd
    rng = np.random.default_rng(2)
    parts = B.recv_records(O, n=60) + B.send_records(O, n=20) + B.events(rng)
    order = rng.permutation(len(parts))
    log = B.binlog([parts[i] for i in order])
    offs, info = mgen_amd.binlog_index(log)
    _, st, n = O.convert_binary_log(log)
    assert info.status == st == 0 and info.n_records == n == len(parts)
    assert info.consumed == len(log)


def _cut(rec: bytes, rl: int) -> bytes:
    """A record whose recordLength says rl (body truncated to rl bytes)."""
    import struct
    return rec[:2] + struct.pack(">H", rl) + rec[4:4 + rl]


def short_for_type_cases():
    """Records too short for the fields their type reads (the device formatters
    must never read past a record): (label, record)."""
    v4 = bytes([10, 0, 0, 9])
    recv = B.recv_records(O, n=1)[0]
    alen = recv[4 + 11]
    join = B.join(3, 4, bytes([224, 1, 2, 3]), 5000, b"eth0")
    conn = B.conn(10, 5, 6, v4, 5001, 4000, 3)
    return [("recv_addr", _cut(recv, 12 + alen - 1)), ("recv_hdr", _cut(recv, 11)),
            ("join_name", _cut(join, len(join) - 4 - 2)), ("join_len", _cut(join, 12 + 4)),
            ("conn", _cut(conn, 18 + 4 - 1)), ("listen", _cut(B.listen(1, 2, 1, 7), 11)),
            ("start", _cut(B.start(1, 1), 7))]


@pytest.mark.parametrize("label", [c[0] for c in short_for_type_cases()])
def test_short_for_type_records_stop(label):
    import mgen_amd
    bad = dict(short_for_type_cases())[label]
    parts = [B.start(1, 2), B.listen(1, 3, 1, 7)]
    log = B.binlog(parts + [bad, B.stop(9, 9)])
    text, st, n = O.convert_binary_log(log)
    assert st == 4 and n == 2 and text.count(b"\n") == 2
    offs, info = mgen_amd.binlog_index(log)
    assert info.status == 4 and info.n_records == 2 and len(offs) == 2
