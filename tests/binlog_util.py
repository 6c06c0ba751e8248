"""Binary MGEN logs for the ConvertBinaryLog tests (test infrastructure).

RECV and SEND records come from the oracle's restatements of the reference's binary log
writers (LogRecvEvent / LogSendEvent binary branches, over the golden matrix's received
records and the send descriptors); the other events are written byte by byte in the layouts
the converter reads (mgenMsg.cpp:1628-1891; Mgen::Start for START, mgen.cpp:169-197)."""
import struct

import numpy as np

HEADER = b"mgen version=5.1.1 type=binary_log\n\0"


def ev_time(ev, sec, usec, body=b"", proto=0):
    b = struct.pack(">II", sec, usec) + body
    return struct.pack(">BBH", ev, proto, len(b)) + b


def start(sec, usec):
    return ev_time(8, sec, usec)


def stop(sec, usec):
    return ev_time(9, sec, usec)


def listen(sec, usec, proto, port, ignore=False):
    return ev_time(5 if ignore else 4, sec, usec, struct.pack(">BBH", proto, 0, port))


def join(sec, usec, group, port=0, iface=b"", leave=False):
    at = 1 if len(group) == 4 else 2
    body = struct.pack(">HBB", port, at, len(group)) + group + bytes([len(iface)]) + iface
    return ev_time(7 if leave else 6, sec, usec, body)


def conn(ev, sec, usec, addr, port, dst_port, flow_id, host=None, proto=2):
    """ON 10, ACCEPT 11, DISCONNECT 12, CONNECT 13, OFF 14, SHUTDOWN 15, RECONNECT 16."""
    at = 1 if len(addr) == 4 else 2
    body = struct.pack(">HBB", port, at, len(addr)) + addr + struct.pack(">HI", dst_port, flow_id)
    if host is not None:
        ha, hp = host
        ht = 1 if len(ha) == 4 else 2
        body += struct.pack(">HBB", hp, ht, len(ha)) + ha
    return ev_time(ev, sec, usec, body, proto)


def recv_records(O, seed=3, n=400, ok_only=True):
    """Binary RECV records of golden-matrix messages (receive path: Unpack + CRC check)."""
    from streams import golden
    gold = golden()
    rng = np.random.default_rng(seed)
    f = gold["unpack_fields_udp"]
    idx = np.nonzero((f["err"] == 0) & (f["ok"] == 1))[0] if ok_only else np.arange(len(f))
    idx = np.sort(rng.choice(idx, min(n, len(idx)), replace=False))
    src = np.zeros(len(idx), O.ADDR_DTYPE)
    for k in range(len(idx)):
        v6 = rng.random() < 0.3
        src[k]["type"], src[k]["len"] = (2, 16) if v6 else (1, 4)
        src[k]["port"] = int(rng.integers(1, 65536))
        src[k]["addr"][:16 if v6 else 4] = rng.integers(0, 256, 16 if v6 else 4)
    rx_s = rng.integers(1_600_000_000, 1_800_000_000, len(idx)).astype(np.uint32)
    rx_u = rng.integers(0, 1_000_000, len(idx)).astype(np.uint32)
    recs = []
    for k, i in enumerate(idx):
        recs.append(O.log_recv_binary(f[i:i + 1], gold["unpack_slab"],
                                      gold["unpack_offs"][i:i + 1], src[k:k + 1], rx_s[k:k + 1],
                                      rx_u[k:k + 1], protocol=int(rng.choice([1, 2, 3]))))
    return recs


def send_records(O, seed=4, n=200):
    from streams import golden
    gold = golden()
    rng = np.random.default_rng(seed)
    d = np.zeros(n, gold["desc"].dtype)
    d["tmpl"] = rng.integers(0, len(gold["tmpl"]), n)
    d["seq_num"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    d["tx_sec"] = rng.integers(1_600_000_000, 1_800_000_000, n).astype(np.uint32)
    d["tx_usec"] = rng.integers(0, 1_000_000, n).astype(np.uint32)
    d["msg_len"] = rng.integers(60, 1500, n)
    d["flags"] = 4
    out = []
    for proto in (1, 3):
        b = O.log_send_batch(gold["tmpl"], d, gold["pool"],
                             rng.integers(1, 65536, len(gold["tmpl"])).astype(np.uint16),
                             protocol=proto, binary=True)
        # split into records by their length fields
        o = 0
        while o < len(b):
            rl = struct.unpack_from(">H", b, o + 2)[0]
            out.append(b[o:o + 4 + rl])
            o += 4 + rl
    return out


def events(rng, t0=1_700_000_000):
    v4 = lambda: bytes(rng.integers(0, 256, 4).tolist())     # noqa: E731
    v6 = lambda: bytes(rng.integers(0, 256, 16).tolist())    # noqa: E731
    t = lambda: (t0 + int(rng.integers(0, 1000)), int(rng.integers(0, 1_000_000)))  # noqa: E731
    ev = [start(*t()), stop(*t()), listen(*t(), 1, 5000), listen(*t(), 2, 5001, ignore=True),
          listen(*t(), 9, 7), join(*t(), bytes([224, 1, 2, 3]), 5000, b"eth0"),
          join(*t(), bytes([239, 0, 0, 1])), join(*t(), v6(), 0, b"ib0\0junk", leave=True),
          join(*t(), bytes([224, 9, 9, 9]), 1234, leave=True)]
    for e in range(10, 17):
        for fid in (0, 7):
            ev.append(conn(e, *t(), v4(), int(rng.integers(1, 65536)), 5000, fid))
            ev.append(conn(e, *t(), v6(), 4000, int(rng.integers(1, 65536)), fid,
                           host=(v4(), 6000)))
    ev.append(conn(10, *t(), v4(), 1, 2, 3, host=(v6(), 7)))
    return ev


def binlog(parts, header=HEADER):
    return header + b"".join(parts)


def data_recv_records(O, seed=5, n=60):
    """Binary RECV records of messages whose MGEN_DATA payload carries REPORT items."""
    from report_util import addr, random_values
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        items = b""
        for _ in range(int(rng.integers(1, 4))):
            dur, ave, mn, mx, rate, loss = random_values(rng)
            b, _ = O.report_build(addr(rng), addr(rng), int(rng.choice([1, 2, 77])), 1, dur, ave,
                                  mn, mx, rate, loss, offset=float(rng.uniform(0, 3)))
            items += b
        m = O.make_msg(msg_len=int(rng.integers(len(items) + 60, 900)), flow_id=k + 1, seq=k,
                       tx_sec=1_700_000_000 + k, tx_usec=k, payload_type=1, payload=items)
        rec = O.udp_pack(m, checksum=True)
        f = O.udp_recv(rec)
        src = addr(rng)
        out.append(O.log_recv_binary(np.array([f]), np.frombuffer(rec, np.uint8), [0], src,
                                     [1_700_000_100 + k], [k * 3], protocol=1))
    return out
