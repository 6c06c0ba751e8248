"""Synthetic pcap captures for the pcap2mgen tests (test infrastructure).

Frames are built byte by byte from the wire formats (Ethernet II / 802.1Q, Linux cooked
SLL, IPv4 / IPv6, UDP); MGEN payloads come from the oracle's restatement of the reference's
UDP send path (MgenMsg::Pack + WriteChecksum).  The capture mixes what pcap2mgen skips (ARP,
TCP, bad IP headers, oversize frames, truncated captures, non-MGEN UDP, bad versions) with
MGEN flows over IPv4 and IPv6, MGEN_DATA payloads carrying REPORT items, reordering and loss.
"""
import struct

import numpy as np

MAC_A = bytes([0x02, 0, 0, 0, 0, 1])
MAC_B = bytes([0x02, 0, 0, 0, 0, 2])


def udp(payload: bytes, sport: int, dport: int) -> bytes:
    return struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload


def ipv4(l4: bytes, src: bytes, dst: bytes, proto=17, ttl=64, ihl=5, total=None) -> bytes:
    opts = bytes(4 * (ihl - 5))
    tot = 4 * ihl + len(l4) if total is None else total
    hdr = struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, tot, 0x1234, 0x4000, ttl, proto, 0,
                      src, dst)
    return hdr + opts + l4


def ipv6(l4: bytes, src: bytes, dst: bytes, nh=17, hops=255, plen=None) -> bytes:
    pl = len(l4) if plen is None else plen
    return struct.pack(">IHBB16s16s", 0x60000000, pl, nh, hops, src, dst) + l4


def eth(ip: bytes, etype=None, vlan=None, pad_to=60) -> bytes:
    if etype is None:
        etype = 0x0800 if (ip[0] >> 4) == 4 else 0x86DD
    tag = struct.pack(">HH", 0x8100, vlan) if vlan is not None else b""
    f = MAC_A + MAC_B + tag + struct.pack(">H", etype) + ip
    return f + bytes(max(0, pad_to - len(f)))   # Ethernet minimum frame padding


def sll(ip: bytes, etype=None) -> bytes:
    if etype is None:
        etype = 0x0800 if (ip[0] >> 4) == 4 else 0x86DD
    return struct.pack(">HHH8sH", 0, 1, 6, MAC_A + b"\0\0", etype) + ip


def pcap(records, link=1, nsec=False, swapped=False, snaplen=65535) -> bytes:
    """records: (ts_sec, ts_frac, frame[, caplen[, wirelen]]) -> a pcap file image."""
    e = ">" if swapped else "<"
    magic = 0xA1B23C4D if nsec else 0xA1B2C3D4
    out = [struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, snaplen, link)]
    for r in records:
        sec, frac, frame = r[0], r[1], r[2]
        wire = r[4] if len(r) > 4 else len(frame)
        cap = r[3] if len(r) > 3 else len(frame)
        out.append(struct.pack(e + "IIII", sec, frac, cap, wire) + frame[:cap])
    return b"".join(out)


def mgen_payload(O, flow, seq, tx, msg_len=256, dst=None, checksum=True, payload_type=0,
                 payload=None, gps=False):
    dst = dst or ("4", bytes([10, 0, 0, 2]), 5000)
    kw = dict(lat=38.5, lon=-77.25, alt=120, gps_status=2) if gps else {}
    m = O.make_msg(msg_len=msg_len, flow_id=flow, seq=seq, tx_sec=tx[0], tx_usec=tx[1],
                   dst=dst, payload_type=payload_type, payload=payload, **kw)
    return O.udp_pack(m, checksum=checksum)


def report_item(O, rng):
    from report_util import addr, random_values
    dur, ave, mn, mx, rate, loss = random_values(rng)
    b, _ = O.report_build(addr(rng), addr(rng), int(rng.choice([1, 2, 77])), 1, dur, ave, mn, mx,
                          rate, loss, offset=float(rng.uniform(0, 3)))
    return b


def capture(O, seed=7, n=600, link=1, nsec=False, swapped=False, v6_frac=0.3):
    """A mixed capture of about n records -> (file bytes, list of notes per record)."""
    rng = np.random.default_rng(seed)
    src4 = [bytes([10, 0, 0, k]) for k in (5, 6, 7)]
    dst4 = bytes([10, 0, 0, 2])
    src6 = [bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [k]) for k in (1, 2)]
    dst6 = bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [0x99])
    seqs = {}
    recs = []
    t_us = 1_700_000_000 * 1_000_000 + 250_000
    for i in range(n):
        t_us += int(rng.integers(200, 9000))
        sec, usec = divmod(t_us, 1_000_000)
        frac = usec * 1000 + int(rng.integers(0, 1000)) if nsec else usec
        kind = rng.random()
        v6 = rng.random() < v6_frac
        flow = int(rng.integers(1, 5))
        key = (v6, flow)
        seq = seqs.get(key, 0)
        r = rng.random()
        seqs[key] = seq + (2 if r < 0.03 else 1)       # loss
        if r > 0.98:
            seq = max(0, seq - 3)                       # late / duplicate
        tx = divmod(t_us - int(rng.integers(100, 5000)), 1_000_000)
        ptype, pl = 0, None
        if rng.random() < 0.08:                         # MGEN_DATA with REPORT items
            ptype = 1
            pl = b"".join(report_item(O, rng) for _ in range(int(rng.integers(1, 3))))
        size = int(rng.integers(64, 1200))
        if v6:
            dst = ("6", dst6, 6000 + flow)
            pay = mgen_payload(O, flow, seq, tx, size, dst, payload_type=ptype, payload=pl,
                               gps=rng.random() < 0.5)
            ip = ipv6(udp(pay, 40000 + flow, 6000 + flow), src6[flow % 2], dst6,
                      hops=int(rng.integers(1, 256)))
        else:
            dst = ("4", dst4, 5000 + flow)
            pay = mgen_payload(O, flow, seq, tx, size, dst, payload_type=ptype, payload=pl,
                               gps=rng.random() < 0.5)
            ip = ipv4(udp(pay, 30000 + flow, 5000 + flow), src4[flow % 3], dst4,
                      ttl=int(rng.integers(1, 256)))
        caplen = None
        if kind < 0.02:                                 # ARP
            frame = eth(bytes(28), etype=0x0806) if link != 113 else sll(bytes(28), 0x0806)
        elif kind < 0.04:                               # TCP
            ip = ipv4(bytes(40), src4[0], dst4, proto=6)
            frame = eth(ip) if link != 113 else sll(ip)
        elif kind < 0.05:                               # bad IPv4 (total length past frame)
            ip = ipv4(udp(pay, 1, 2), src4[0], dst4, total=4000)
            frame = eth(ip) if link != 113 else sll(ip)
        elif kind < 0.06:                               # non-MGEN UDP (Unpack fails)
            ip = ipv4(udp(bytes([0, 40, 9]) + bytes(40), 53, 53), src4[1], dst4)
            frame = eth(ip) if link != 113 else sll(ip)
        elif kind < 0.07:                               # truncated capture
            frame = eth(ip) if link != 113 else sll(ip)
            caplen = max(20, len(frame) - int(rng.integers(1, 60)))
        elif kind < 0.08 and link != 113:               # 802.1Q tagged
            frame = eth(ip, vlan=int(rng.integers(1, 4095)))
        elif kind < 0.085:                              # IP version 5
            ip = bytes([0x50]) + ip[1:]
            frame = eth(ip, etype=0x0800) if link != 113 else sll(ip, 0x0800)
        elif kind < 0.09 and link != 113:               # over the 4094-byte parse buffer
            big = mgen_payload(O, flow, seq, tx, 4200, ("4", dst4, 5000 + flow))
            frame = eth(ipv4(udp(big, 30000 + flow, 5000 + flow), src4[0], dst4))
        else:
            frame = eth(ip) if link != 113 else sll(ip)
        rec = (sec, frac, frame) if caplen is None else (sec, frac, frame, caplen, len(frame))
        recs.append(rec)
    return pcap(recs, link=link, nsec=nsec, swapped=swapped)


def snap(file: bytes, snaplen: int) -> bytes:
    """The same capture as `tcpdump -s snaplen` would have written it: every record's data
    cut to snaplen bytes, its wire length kept (native-order, microsecond files)."""
    out = [file[:16] + struct.pack("<I", snaplen) + file[20:24]]
    off = 24
    while off + 16 <= len(file):
        sec, frac, cap, wire = struct.unpack("<IIII", file[off:off + 16])
        data = file[off + 16:off + 16 + cap]
        c = min(cap, snaplen)
        out.append(struct.pack("<IIII", sec, frac, c, wire) + data[:c])
        off += 16 + cap
    return b"".join(out)
