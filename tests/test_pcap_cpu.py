"""pcap2mgen on the CPU side: the oracle's frame walk on hand-built frames, the host index walk
of libmgenx (mgenx_pcap_index: host code, no GPU), and the oracle's whole main loop on small
captures (pcap2mgen.cpp:252-482).  The Ethernet / IP / UDP layer restates protolib, which is
not vendored: parity unpinned there; the log lines are the pinned formatters."""
import re
import struct

import numpy as np
import pytest

from oracle import oracle as O
import pcap_util as P


def _rec(frame, sec=1_700_000_000, frac=123456, cap=None, wire=None):
    cap = len(frame) if cap is None else cap
    wire = len(frame) if wire is None else wire
    return struct.pack("<IIII", sec, frac, cap, wire) + frame[:cap]


SRC4, DST4 = bytes([10, 0, 0, 5]), bytes([10, 0, 0, 2])
SRC6 = bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [1])
DST6 = bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [0x99])


def test_frame_ipv4_udp():
    pay = bytes(range(40))
    fr = P.eth(P.ipv4(P.udp(pay, 30001, 5001), SRC4, DST4, ttl=17))
    st, uo, ul, src, ttl, sec, usec = O.pcap_frame(_rec(fr))
    assert st == 0 and ul == 40 and uo == 16 + 14 + 20 + 8
    assert src["type"] == 1 and src["len"] == 4 and src["port"] == 30001
    assert bytes(src["addr"][:4]) == SRC4 and ttl == 17
    assert (sec, usec) == (1_700_000_000, 123456)


def test_frame_ipv6_vlan_sll_and_options():
    pay = bytes(100)
    fr = P.eth(P.ipv6(P.udp(pay, 40001, 6001), SRC6, DST6, hops=3), vlan=42)
    st, uo, ul, src, ttl, *_ = O.pcap_frame(_rec(fr))
    assert (st, uo, ul, ttl) == (0, 16 + 18 + 40 + 8, 100, 3)
    assert src["type"] == 2 and bytes(src["addr"]) == SRC6 and src["port"] == 40001
    fr = P.sll(P.ipv4(P.udp(pay, 1, 2), SRC4, DST4, ihl=6))       # IPv4 options
    st, uo, ul, *_ = O.pcap_frame(_rec(fr), link_type=113)
    assert (st, uo, ul) == (0, 16 + 16 + 24 + 8, 100)


@pytest.mark.parametrize("case,status", [
    ("arp", 2), ("tcp", 4), ("bad_total", 3), ("ver5", 3), ("trunc", 7), ("trunc_hdr", 5),
    ("oversize", 1), ("udp_len_big", 4), ("runt", 1)])
def test_frame_skips(case, status):
    pay = bytes(64)
    ip = P.ipv4(P.udp(pay, 1, 2), SRC4, DST4)
    cap = wire = None
    if case == "arp":
        fr = P.eth(bytes(28), etype=0x0806)
    elif case == "tcp":
        fr = P.eth(P.ipv4(bytes(40), SRC4, DST4, proto=6))
    elif case == "bad_total":
        fr = P.eth(P.ipv4(P.udp(pay, 1, 2), SRC4, DST4, total=3000))
    elif case == "ver5":
        fr = P.eth(bytes([0x50]) + ip[1:], etype=0x0800)
    elif case == "trunc":          # snapped: UDP header + >= 28 payload bytes captured
        fr = P.eth(ip)
        cap = len(fr) - 5
        wire = len(fr)
    elif case == "trunc_hdr":      # cut inside the first 28 payload bytes: skipped
        fr = P.eth(ip)
        cap = 14 + 20 + 8 + 27
        wire = len(fr)
    elif case == "oversize":
        fr = P.eth(P.ipv4(P.udp(bytes(4100), 1, 2), SRC4, DST4))
    elif case == "udp_len_big":
        u = bytearray(P.udp(pay, 1, 2))
        u[4:6] = struct.pack(">H", 500)
        fr = P.eth(P.ipv4(bytes(u), SRC4, DST4))
    else:
        fr = bytes(10)
    assert O.pcap_frame(_rec(fr, cap=cap, wire=wire))[0] == status


def test_frame_nsec_and_swapped():
    fr = P.eth(P.ipv4(P.udp(bytes(30), 7, 8), SRC4, DST4))
    rec = struct.pack(">IIII", 5, 999_999_999, len(fr), len(fr)) + fr
    st, *_, sec, usec = O.pcap_frame(rec, flags=3)
    assert st == 0 and (sec, usec) == (5, 999_999)


def test_pcap_index_host_walk():
    import mgen_amd
    f = P.capture(O, seed=3, n=120)
    offs, info = mgen_amd.pcap_index(f)
    # the record chain, walked in Python
    want, o = [], 24
    while o + 16 <= len(f):
        cap = struct.unpack_from("<I", f, o + 8)[0]
        if o + 16 + cap > len(f):
            break
        want.append(o)
        o += 16 + cap
    assert list(offs) == want and info.n_records == 120 and info.consumed == len(f)
    assert info.link_type == 1 and info.flags == 0
    # a cut-short last record ends the walk (pcap_next returns NULL)
    offs2, info2 = mgen_amd.pcap_index(f[:-3])
    assert list(offs2) == want[:-1] and info2.consumed == want[-1]
    g = P.capture(O, seed=3, n=10, nsec=True, swapped=True, link=113)
    _, info3 = mgen_amd.pcap_index(g)
    assert info3.flags == 3 and info3.link_type == 113 and info3.n_records == 10
    with pytest.raises(mgen_amd.MgenxError):
        mgen_amd.pcap_index(b"\x00" * 40)


LINE = re.compile(rb"^\d\d:\d\d:\d\d\.\d{6} (RECV|REPORT) ")


def test_oracle_main_loop_shapes():
    f = P.capture(O, seed=11, n=300)
    text, st = O.pcap2mgen(f)
    lines = text.split(b"\n")[:-1]
    assert all(LINE.match(l) for l in lines)
    recv = [l for l in lines if b" RECV " in l]
    # one RECV line per UDP packet (snapped ones included) whose payload Unpack accepts
    n_udp = int(((st == 0) | (st == 7)).sum())
    assert 0 < len(recv) <= n_udp
    assert all(b" ttl>" in l and b" gps>" in l and b" data>" not in l for l in recv)
    # rxlog off: only the REPORT lines of carried reports remain
    t2, _ = O.pcap2mgen(f, log_rx=False)
    assert t2 == b"".join(l + b"\n" for l in lines if b" REPORT " in l)


def test_oracle_analytic_reports():
    # one flow, 1 message every 0.25 s for 3 s: a window closes on the first message at or
    # after its end (the quantized 1 s window is slightly over 1 s), and the REPORT line comes
    # right before that message's RECV line
    recs = []
    for k in range(13):
        t = 1_700_000_000_000_000 + k * 250_000
        sec, usec = divmod(t, 1_000_000)
        pay = P.mgen_payload(O, 1, k, divmod(t - 1500, 1_000_000), 200)
        recs.append((sec, usec, P.eth(P.ipv4(P.udp(pay, 30001, 5001), SRC4, DST4))))
    f = P.pcap(recs)
    a = O.AnalyticOracle(1.0)
    closes = [k for k in range(13)
              if a.update(1_700_000_000 + k // 4, (k % 4) * 250_000, 200,
                          *divmod(1_700_000_000_000_000 + k * 250_000 - 1500, 1_000_000), k)]
    assert closes == [5, 10]
    text, _ = O.pcap2mgen(f, analytics=True, window=1.0)
    lines = text.split(b"\n")[:-1]
    kinds = b"".join(b"R" if b" REPORT " in l else b"v" for l in lines)
    assert kinds == b"".join((b"Rv" if k in closes else b"v") for k in range(13))
    rep = lines[5]
    assert rep.startswith(b"22:13:21.250000 REPORT proto>UDP flow>1 src>10.0.0.5/30001 "
                          b"dst>10.0.0.2/5000 window>1.250000 ")
    assert rep.endswith(b", count>5")


def test_cli_command_errors():
    """tools/pcap2mgen's command matching (pcap2mgen.cpp:71-248): invalid or ambiguous commands,
    missing arguments and bad rxlog values fail before any device work."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "pcap2mgen")
    if not os.path.exists(exe):
        pytest.skip("tools/pcap2mgen not built")
    for args, msg in [(["bogus"], b"invalid command"), (["infile"], b"missing argument"),
                      (["+infile", "x"], b"invalid command"),   # names are given bare
                      (["rxlog", "maybe"], b"wrong argument to rxlog"),
                      (["trace"], b"not supported"), (["r"], b"invalid command"),  # ambiguous
                      (["infile", "/nonexistent/x.pcap"], b"error opening input file")]:
        r = subprocess.run([exe] + args, capture_output=True, timeout=60, input=b"")
        assert r.returncode != 0 and msg in r.stderr, (args, r.stderr)


def test_overflow_redo_create_failure_frees_once():
    """run_device's flow-table redo: when the full-size table cannot be created,
    the first table is freed once -- not again by the cleanup.  A stand-in engine on CPU tensors
    drives the host logic up to the failing create."""
    import torch
    from mgen_amd.pcap import Pcap2Mgen

    n = 8
    freed, made = [], []

    class FakeEngine:
        device = 0

        def __init__(self):
            self.torch = torch

        def pcap_parse(self, buf, pkt_off, n_, link_type, flags):
            z = torch.zeros(n_, dtype=torch.int64)
            return {"udp_off": z, "udp_len": z, "src": z, "rx_sec": z, "rx_usec": z, "ttl": z}

        def unpack(self, buf, n_, **kw):
            return {"err": torch.zeros(n_, dtype=torch.uint8)}

        def flow_table(self, cap):
            if made:
                raise MemoryError("second table")
            made.append(cap)
            return "table0"

        def flow_lookup(self, table, cols, src, n_):
            # every record lost: the first table overflowed
            return torch.full((n_,), -1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)

        def flow_table_destroy(self, table):
            freed.append(table)

    p = Pcap2Mgen(FakeEngine(), analytics=True)
    p.FIRST_FLOWS = 2
    with pytest.raises(MemoryError):
        p.run_device(torch.zeros(16, dtype=torch.uint8), torch.zeros(n, dtype=torch.int64), n,
                     1, 0)
    assert made == [2] and freed == ["table0"]
