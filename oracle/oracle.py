"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the C restatement (mgen_oracle.c).

This module is the parity CHECKER.  Only tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg may import it; the product (``mgen_amd`` and
libmgenx.so) never does.  Parity status: see mgen_oracle.h / DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

# ---- numpy mirrors of the C structs (aligned like the C compiler lays them out) ----
TMPL_DTYPE = np.dtype([
    ("flow_id", "<u4"),
    ("dst_type", "u1"), ("dst_len", "u1"), ("dst_port", "<u2"),
    ("dst_addr", "u1", 16),
    ("host_type", "u1"), ("host_len", "u1"), ("host_port", "<u2"),
    ("host_addr", "u1", 16),
    ("lat_raw", "<u4"), ("lon_raw", "<u4"), ("alt", "<i4"),
    ("gps_status", "u1"), ("payload_type", "u1"), ("payload_len", "<u2"),
    ("payload_off", "<u4"),
    ("has_payload", "u1"), ("rsv0", "u1"), ("rsv1", "<u2"),
], align=True)

DESC_DTYPE = np.dtype([
    ("tmpl", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"), ("tx_usec", "<u4"),
    ("msg_len", "<u2"), ("flags", "u1"), ("rsv", "u1"),
], align=True)

FIELDS_DTYPE = np.dtype([
    ("ok", "u1"), ("err", "u1"), ("version", "u1"), ("flags", "u1"),
    ("msg_len", "<u2"), ("hdr_len", "<u2"),
    ("flow_id", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"), ("tx_usec", "<u4"),
    ("dst_port", "<u2"), ("dst_type", "u1"), ("dst_len", "u1"), ("dst_addr", "u1", 16),
    ("host_port", "<u2"), ("host_type", "u1"), ("host_len", "u1"), ("host_addr", "u1", 16),
    ("lat_raw", "<u4"), ("lon_raw", "<u4"), ("alt", "<i4"),
    ("gps_status", "u1"), ("payload_type", "u1"), ("payload_len", "<u2"),
    ("payload_off", "<u4"),
], align=True)


class _Addr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint8), ("len", ctypes.c_uint8), ("port", ctypes.c_uint16),
                ("addr", ctypes.c_uint8 * 16)]


class Msg(ctypes.Structure):
    """or_msg: the MgenMsg members Pack() serialises."""
    _fields_ = [("msg_len", ctypes.c_uint16), ("mgen_msg_len", ctypes.c_uint32),
                ("version", ctypes.c_uint8), ("flags", ctypes.c_uint8),
                ("flow_id", ctypes.c_uint32), ("seq_num", ctypes.c_uint32),
                ("tx_sec", ctypes.c_uint32), ("tx_usec", ctypes.c_uint32),
                ("dst", _Addr), ("host", _Addr),
                ("latitude", ctypes.c_double), ("longitude", ctypes.c_double),
                ("altitude", ctypes.c_int32), ("gps_status", ctypes.c_uint8),
                ("payload_type", ctypes.c_uint8), ("payload_len", ctypes.c_uint16),
                ("payload_data", ctypes.c_void_p)]


class Time(ctypes.Structure):
    _fields_ = [("sec", ctypes.c_int64), ("usec", ctypes.c_int64)]


class Analytic(ctypes.Structure):
    _fields_ = [("depth", ctypes.c_uint32), ("first", ctypes.c_uint32), ("nset", ctypes.c_uint32),
                ("bits", ctypes.c_uint8 * 128),
                ("window_size", ctypes.c_double), ("window_valid", ctypes.c_int),
                ("window_start", Time), ("window_end", Time), ("seq_start", ctypes.c_uint32),
                ("msg_count", ctypes.c_uint64), ("byte_count", ctypes.c_uint64),
                ("dup_msg_count", ctypes.c_uint64),
                ("latency_sum", ctypes.c_double), ("latency_min", ctypes.c_double),
                ("latency_max", ctypes.c_double),
                ("report_valid", ctypes.c_int), ("n_reports", ctypes.c_uint64),
                ("report_start", Time), ("report_duration", ctypes.c_double),
                ("report_msg_count", ctypes.c_uint64),
                ("report_rate_ave", ctypes.c_double), ("report_loss_ave", ctypes.c_double),
                ("report_latency_ave", ctypes.c_double), ("report_latency_min", ctypes.c_double),
                ("report_latency_max", ctypes.c_double)]


_lib = None


def build():
    """Compile the restatement (gcc) into oracle/build/liboracle.so."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.or_crc32_update.argtypes = [ctypes.POINTER(u32), P, u32]
        L.or_crc32_table.argtypes = [P]
        L.or_glibc_rand_bytes.argtypes = [u32, u32, P]
        L.or_pack.argtypes = [ctypes.POINTER(Msg), P, ctypes.c_uint16, i32, ctypes.POINTER(u32),
                              i32, u32, ctypes.POINTER(ctypes.c_uint16)]
        L.or_pack.restype = ctypes.c_uint16
        L.or_udp_pack.argtypes = [ctypes.POINTER(Msg), P, i32, i32, u32]
        L.or_udp_pack.restype = u32
        L.or_tcp_tx.argtypes = [ctypes.POINTER(Msg), P, i32, i32, u32]
        L.or_tcp_tx.restype = u32
        L.or_unpack.argtypes = [P, u32, P]
        L.or_unpack_persist.argtypes = [P, u32, P]
        L.or_unpack_persist.restype = u32
        L.or_tcp_rx_persist.argtypes = [P, P, P, u32, i32, i32, P, ctypes.POINTER(u32), P, P]
        L.or_udp_recv.argtypes = [P, u32, i32, P]
        L.or_tcp_recv.argtypes = [P, u32, i32, P]
        L.or_tcp_scan.argtypes = [P, u64, i32, P, P, P, u32, ctypes.POINTER(u64),
                                  ctypes.POINTER(i32)]
        L.or_tcp_scan.restype = u32
        L.or_sink_scan.argtypes = [P, u64, i32, P, P, P, u32, ctypes.POINTER(u64)]
        L.or_sink_scan.restype = u32
        L.or_payload_from_hex.argtypes = [ctypes.c_char_p, P, u32]
        L.or_payload_from_hex.restype = u32
        L.or_udp_pack_batch.argtypes = [P, P, u32, P, P, P, u64, i32, i32, u32, P]
        L.or_udp_recv_batch.argtypes = [P, P, u64, P, u32, u32, i32, P, i32]
        L.or_tcp_tx_batch.argtypes = [P, P, P, u32, P, P, i32, i32, u32]
        L.or_tcp_tx_batch.restype = u64
        L.or_quantized_window.argtypes = [ctypes.c_double]
        L.or_quantized_window.restype = ctypes.c_double
        L.or_analytic_init.argtypes = [ctypes.POINTER(Analytic), ctypes.c_double]
        L.or_analytic_update.argtypes = [ctypes.POINTER(Analytic), Time, u32, Time, u32]
        L.or_analytic_update.restype = i32
        L.or_time_delta.argtypes = [Time, Time]
        L.or_time_delta.restype = ctypes.c_double
        L.or_flow_reduce_batch.argtypes = [P, u32, P, P, P, P, P, P, P, u32, P, u32, P]
        L.or_log_recv_text.argtypes = [P, P, P, u32, u32, i32, i32, u32, P]
        L.or_log_recv_text.restype = u32
        L.or_log_recv_binary.argtypes = [P, P, u64, P, u32, u32, i32, P]
        L.or_log_recv_binary.restype = u32
        L.or_udp_pack_batch_mt.argtypes = [P, P, u32, P, P, P, u64, i32, P, i32]
        L.or_flow_reduce_batch_mt.argtypes = [P, u32, P, P, P, P, P, P, P, u32, P, i32]
        L.or_sizeof.argtypes = [i32]
        L.or_sizeof.restype = u32
        assert L.or_sizeof(0) == TMPL_DTYPE.itemsize, "or_tmpl layout mismatch"
        assert L.or_sizeof(1) == DESC_DTYPE.itemsize, "or_desc layout mismatch"
        assert L.or_sizeof(2) == FIELDS_DTYPE.itemsize, "or_fields layout mismatch"
        assert L.or_sizeof(3) == ctypes.sizeof(Analytic), "or_analytic layout mismatch"
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- CRC
def crc_table():
    t = np.zeros(256, np.uint32)
    lib().or_crc32_table(_ptr(t))
    return t


def crc32_update(state: int, data: bytes) -> int:
    """MgenMsg::ComputeCRC32 (incremental, reset-on-zero)."""
    c = ctypes.c_uint32(state)
    buf = np.frombuffer(bytes(data), np.uint8)
    lib().or_crc32_update(ctypes.byref(c), _ptr(buf) if len(buf) else None, len(buf))
    return c.value


def glibc_rand_bytes(seed: int, n: int) -> bytes:
    out = np.zeros(max(n, 1), np.uint8)
    lib().or_glibc_rand_bytes(seed, n, _ptr(out))
    return out[:n].tobytes()


# ---------------------------------------------------------------- messages
def make_msg(*, msg_len, flow_id=1, seq=0, tx_sec=0, tx_usec=0, flags=0, version=2,
             dst=("4", bytes([127, 0, 0, 1]), 5000), host=None, lat=999.0, lon=999.0, alt=-999,
             gps_status=0, payload_type=0, payload=None, payload_len=None, mgen_msg_len=None):
    """Build an or_msg the way MgenFlow::SendMessage does (mgenFlow.cpp:946-983)."""
    m = Msg()
    keep = []
    m.msg_len = msg_len & 0xFFFF
    m.mgen_msg_len = msg_len if mgen_msg_len is None else mgen_msg_len
    m.version = version
    m.flags = flags
    m.flow_id, m.seq_num, m.tx_sec, m.tx_usec = flow_id, seq, tx_sec, tx_usec

    def fill(a, spec):
        if spec is None:
            a.type = 0
            return
        kind, raw, port = spec
        a.type = {"4": 1, "6": 2, "x": 7}[kind]
        a.len = len(raw)
        a.port = port
        for i, b in enumerate(raw[:16]):
            a.addr[i] = b
    fill(m.dst, dst)
    fill(m.host, host)
    m.latitude, m.longitude, m.altitude, m.gps_status = lat, lon, alt, gps_status
    m.payload_type = payload_type
    if payload is not None:
        pb = ctypes.create_string_buffer(bytes(payload), max(len(payload), 1))
        keep.append(pb)
        m.payload_data = ctypes.cast(pb, ctypes.c_void_p)
        m.payload_len = len(payload) if payload_len is None else payload_len
    else:
        m.payload_data = None
        m.payload_len = payload_len or 0
    m._keep = keep
    return m


def udp_pack(m: Msg, checksum=True, random_fill=False, fill_time=0) -> bytes:
    cap = max(m.msg_len, 64) + 64
    out = np.zeros(cap, np.uint8)
    n = lib().or_udp_pack(ctypes.byref(m), _ptr(out), int(checksum), int(random_fill), fill_time)
    return out[:n].tobytes()


def pack(m: Msg, buffer_len, checksum=False, tx_checksum=0, random_fill=False, fill_time=0):
    """Raw MgenMsg::Pack; returns (ret, bytes[:buffer_len], tx_checksum, flags, hdr_len)."""
    out = np.zeros(max(buffer_len, 64) + 64, np.uint8)
    ck = ctypes.c_uint32(tx_checksum)
    hl = ctypes.c_uint16(0)
    r = lib().or_pack(ctypes.byref(m), _ptr(out), buffer_len, int(checksum), ctypes.byref(ck),
                      int(random_fill), fill_time, ctypes.byref(hl))
    return r, out[:buffer_len].tobytes(), ck.value, m.flags, hl.value


def tcp_tx(m: Msg, checksum=True, random_fill=False, fill_time=0) -> bytes:
    out = np.zeros(m.mgen_msg_len + 16, np.uint8)
    n = lib().or_tcp_tx(ctypes.byref(m), _ptr(out), int(checksum), int(random_fill), fill_time)
    return out[:n].tobytes()


def _fields_one(fn, rec, *args):
    buf = np.frombuffer(bytes(rec), np.uint8).copy() if len(rec) else np.zeros(1, np.uint8)
    f = np.zeros(1, FIELDS_DTYPE)
    fn(_ptr(buf), len(rec), *args, _ptr(f))
    return f[0]


def unpack(rec: bytes):
    return _fields_one(lib().or_unpack, rec)


def udp_recv(rec: bytes, force=False):
    return _fields_one(lib().or_udp_recv, rec, int(force))


def _scan(fn, stream, force, extra_status):
    buf = np.frombuffer(bytes(stream), np.uint8).copy() if len(stream) else np.zeros(1, np.uint8)
    cap = len(stream) // 2 + 1
    offs = np.zeros(cap, np.uint64)
    lens = np.zeros(cap, np.uint32)
    f = np.zeros(cap, FIELDS_DTYPE)
    consumed = ctypes.c_uint64(0)
    if extra_status:
        st = ctypes.c_int(0)
        n = fn(_ptr(buf), len(stream), int(force), _ptr(offs), _ptr(lens), _ptr(f), cap,
               ctypes.byref(consumed), ctypes.byref(st))
        return offs[:n], lens[:n], f[:n], consumed.value, st.value
    n = fn(_ptr(buf), len(stream), int(force), _ptr(offs), _ptr(lens), _ptr(f), cap,
           ctypes.byref(consumed))
    return offs[:n], lens[:n], f[:n], consumed.value


def fresh_fields():
    """or_fields of a fresh MgenMsg (constructor defaults, mgenMsg.cpp:38-49)."""
    f = np.zeros(1, FIELDS_DTYPE)
    f["version"] = 2
    f["lat_raw"] = f["lon_raw"] = 10800000
    return f


def tcp_rx_persist(stream, offs, lens, log_open=True, force=False, state=None, pay_src=None):
    """The TCP receiver's persistent rx_msg over consecutive records (or_tcp_rx_persist):
    returns (fields per record, payload_rec per record, state after, pay_src after)."""
    stream = np.ascontiguousarray(stream, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    n = len(offs)
    st = fresh_fields() if state is None else np.array(state, FIELDS_DTYPE).reshape(1).copy()
    ps = ctypes.c_uint32(0xFFFFFFFF if pay_src is None else pay_src)
    out = np.zeros(n, FIELDS_DTYPE)
    prec = np.zeros(n, np.uint32)
    lib().or_tcp_rx_persist(_ptr(stream), _ptr(offs), _ptr(lens), n, int(log_open), int(force),
                            _ptr(st), ctypes.byref(ps), _ptr(out), _ptr(prec))
    return out, prec, st, ps.value


def tcp_scan(stream: bytes, force=False):
    return _scan(lib().or_tcp_scan, stream, force, True)


def sink_scan(stream: bytes, force=False):
    return _scan(lib().or_sink_scan, stream, force, False)


def payload_from_hex(hexstr: str) -> bytes:
    out = np.zeros(len(hexstr) // 2 + 2, np.uint8)
    n = lib().or_payload_from_hex(hexstr.encode(), _ptr(out), len(out))
    return out[:n].tobytes()


# ---------------------------------------------------------------- batches
def udp_pack_batch(tmpl, desc, pool, slab_bytes, rec_off=None, stride=0, checksum=True,
                   random_fill=False, fill_time=0):
    n = len(desc)
    slab = np.zeros(slab_bytes, np.uint8)
    lens = np.zeros(n, np.uint32)
    pool = np.ascontiguousarray(pool if pool is not None and len(pool) else np.zeros(1, np.uint8))
    lib().or_udp_pack_batch(_ptr(tmpl), _ptr(desc), n, _ptr(pool), _ptr(slab),
                            _ptr(rec_off), stride, int(checksum), int(random_fill), fill_time,
                            _ptr(lens))
    return slab, lens


def udp_recv_batch(slab, n, rec_off=None, stride=0, rec_len=None, fixed_len=0, force=False,
                   nthreads=1, tcp=False):
    out = np.zeros(n, FIELDS_DTYPE)
    lib().or_udp_recv_batch(_ptr(slab), _ptr(rec_off), stride, _ptr(rec_len), fixed_len, n,
                            int(force) | (2 if tcp else 0), _ptr(out), nthreads)
    return out


def tcp_recv(rec: bytes, force=False):
    return _fields_one(lib().or_tcp_recv, rec, int(force))


def tcp_tx_batch(tmpl, desc, msg_total, pool, checksum=True, random_fill=False, fill_time=0):
    total = int(np.asarray(msg_total, np.uint64).sum())
    stream = np.zeros(total + 16, np.uint8)
    pool = np.ascontiguousarray(pool if pool is not None and len(pool) else np.zeros(1, np.uint8))
    mt = np.ascontiguousarray(msg_total, np.uint32)
    n = lib().or_tcp_tx_batch(_ptr(tmpl), _ptr(desc), _ptr(mt), len(desc), _ptr(pool),
                              _ptr(stream), int(checksum), int(random_fill), fill_time)
    return stream[:n]


# ---------------------------------------------------------------- analytics
def quantized_window(w=1.0):
    return lib().or_quantized_window(w)


class AnalyticOracle:
    """MgenAnalytic restated (parity unpinned at the protolib boundary)."""

    def __init__(self, window=1.0):
        self.a = Analytic()
        lib().or_analytic_init(ctypes.byref(self.a), window)

    def update(self, rx_sec, rx_usec, msg_size, tx_sec, tx_usec, seq):
        return bool(lib().or_analytic_update(ctypes.byref(self.a), Time(rx_sec, rx_usec),
                                             msg_size, Time(tx_sec, tx_usec), seq))


REPORT_DTYPE = np.dtype([
    ("flow", "<u4"), ("index", "<u4"), ("start_sec", "<i8"), ("start_usec", "<i8"),
    ("duration", "<f8"), ("msg_count", "<u8"), ("rate", "<f8"), ("loss", "<f8"),
    ("latency_ave", "<f8"), ("latency_min", "<f8"), ("latency_max", "<f8"),
    ("rx_sec", "<i8"), ("rx_usec", "<i8")])


def flow_reduce_batch(n_flows, flow_idx, seq, tx_sec, tx_usec, msg_len, rx_sec, rx_usec,
                      window=1.0, per_flow=64, flows=None):
    """or_flow_reduce_batch: MgenAnalytic::Update per record (receive order) over n_flows
    flows.  Returns (flows ctypes array, reports[n_flows, per_flow], counts[n_flows])."""
    assert lib().or_sizeof(100) == REPORT_DTYPE.itemsize
    if flows is None:
        flows = (Analytic * n_flows)()
        for f in range(n_flows):
            lib().or_analytic_init(ctypes.byref(flows[f]), window)
    n = len(flow_idx)
    cols = [np.ascontiguousarray(x, dt) for x, dt in
            ((flow_idx, np.uint32), (seq, np.uint32), (tx_sec, np.uint32), (tx_usec, np.uint32),
             (msg_len, np.uint16), (rx_sec, np.uint32), (rx_usec, np.uint32))]
    reports = np.zeros(n_flows * max(per_flow, 1), REPORT_DTYPE)
    counts = np.zeros(n_flows, np.uint32)
    lib().or_flow_reduce_batch(flows, n_flows, *[_ptr(c) for c in cols], n, _ptr(reports),
                               per_flow, _ptr(counts))
    return flows, reports.reshape(n_flows, max(per_flow, 1)), counts


# ---------------------------------------------------------------- event log
ADDR_DTYPE = np.dtype([("type", "u1"), ("len", "u1"), ("port", "<u2"), ("addr", "u1", 16)])
LOG_EPOCH, LOG_NO_DATA, LOG_NO_GPS = 0x1, 0x2, 0x4


def log_recv_text(fields, slab, rec_off, src, rx_sec, rx_usec, protocol=1, ttl=None, opts=0):
    """MgenMsg::LogRecvEvent / LogRecvError text lines for n received records (or_fields
    array `fields`, record i at slab[rec_off[i]:]); src: ADDR_DTYPE array; ttl: int array
    or None (unknown).  Returns the concatenated log bytes."""
    L = lib()
    slab = np.ascontiguousarray(slab, np.uint8)
    fields = np.ascontiguousarray(fields)
    src = np.ascontiguousarray(src, ADDR_DTYPE)
    out = []
    buf = np.zeros(65536 * 2 + 1024, np.uint8)
    base = slab.ctypes.data
    for i in range(len(fields)):
        n = L.or_log_recv_text(ctypes.c_void_p(fields.ctypes.data + i * fields.itemsize),
                               ctypes.c_void_p(base + int(rec_off[i])),
                               ctypes.c_void_p(src.ctypes.data + i * src.itemsize),
                               int(rx_sec[i]), int(rx_usec[i]), protocol,
                               -1 if ttl is None else int(ttl[i]), opts, _ptr(buf))
        out.append(buf[:n].tobytes())
    return b"".join(out)


def log_recv_binary(fields, slab, rec_off, src, rx_sec, rx_usec, protocol=1, rec_len=None):
    """Binary RECV / RERR log records for n received records: record i's message bytes are
    its rec_len[i] received bytes (its msg_len field when rec_len is None), zeros after."""
    L = lib()
    slab = np.ascontiguousarray(slab, np.uint8)
    fields = np.ascontiguousarray(fields)
    src = np.ascontiguousarray(src, ADDR_DTYPE)
    out = []
    buf = np.zeros(65536 + 256, np.uint8)
    for i in range(len(fields)):
        off = int(rec_off[i])
        have = int(rec_len[i]) if rec_len is not None else int(fields["msg_len"][i])
        n = L.or_log_recv_binary(ctypes.c_void_p(fields.ctypes.data + i * fields.itemsize),
                                 ctypes.c_void_p(slab.ctypes.data + off),
                                 max(0, min(len(slab) - off, have)),
                                 ctypes.c_void_p(src.ctypes.data + i * src.itemsize),
                                 int(rx_sec[i]), int(rx_usec[i]), protocol, _ptr(buf))
        out.append(buf[:n].tobytes())
    return b"".join(out)


def log_send_text(tmpl1, desc1, src_port, protocol=1, mgen_msg_len=None, opts=0):
    """or_log_send_text for one template / descriptor record (numpy structured scalars)."""
    L = lib()
    P, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.or_log_send_text.argtypes = [P, P, ctypes.c_uint16, i32, u32, u32, P]
    L.or_log_send_text.restype = u32
    t = np.ascontiguousarray(np.asarray(tmpl1).reshape(1))
    d = np.ascontiguousarray(np.asarray(desc1).reshape(1))
    out = np.zeros(512, np.uint8)
    mml = int(d["msg_len"][0]) if mgen_msg_len is None else mgen_msg_len
    n = L.or_log_send_text(_ptr(t), _ptr(d), src_port, protocol, mml, opts, _ptr(out))
    return out[:n].tobytes()


def log_send_batch(tmpl, desc, pool, src_port, protocol=1, checksum=True, opts=0,
                   binary=False):
    """SEND log events (text or binary) of n records sent by the UDP / SINK path."""
    L = lib()
    if not getattr(L, "_send_protos", False):
        P, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.or_log_send_batch.argtypes = [P, P, u32, P, P, i32, i32, u32, i32, P]
        L.or_log_send_batch.restype = ctypes.c_uint64
        L._send_protos = True
    tmpl = np.ascontiguousarray(tmpl)
    desc = np.ascontiguousarray(desc)
    pool = np.ascontiguousarray(pool if pool is not None and len(pool) else np.zeros(1, np.uint8))
    sp = np.ascontiguousarray(src_port, np.uint16)
    out = np.zeros(len(desc) * 400 + 1024, np.uint8)
    n = L.or_log_send_batch(_ptr(tmpl), _ptr(desc), len(desc), _ptr(pool), _ptr(sp), protocol,
                            int(checksum), opts, int(binary), _ptr(out))
    return out[:n].tobytes()


# ---------------------------------------------------------------- MGEN_DATA items
def _report_protos():
    L = lib()
    if getattr(L, "_rep_ready", False):
        return L
    P, u32, i32, d = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_double
    L.or_q_time.argtypes, L.or_q_time.restype = [d], ctypes.c_uint8
    L.or_uq_time.argtypes, L.or_uq_time.restype = [ctypes.c_uint8], d
    L.or_q_rate.argtypes, L.or_q_rate.restype = [d], ctypes.c_uint16
    L.or_uq_rate.argtypes, L.or_uq_rate.restype = [ctypes.c_uint16], d
    L.or_q_loss.argtypes, L.or_q_loss.restype = [d], ctypes.c_uint16
    L.or_uq_loss.argtypes, L.or_uq_loss.restype = [ctypes.c_uint16], d
    L.or_report_build.argtypes = [P, P, u32, i32, d, d, d, d, d, d, d, ctypes.POINTER(i32), P]
    L.or_report_build.restype = u32
    L.or_log_report.argtypes = [P, d, d, d, d, d, d, ctypes.c_uint64, u32, u32, u32, P]
    L.or_log_report.restype = u32
    L.or_log_report_recv.argtypes = [P, P, u32, u32, u32, P]
    L.or_log_report_recv.restype = u32
    L.or_data_walk.argtypes = [P, u32, i32, P, ctypes.POINTER(u32), u32, P, ctypes.POINTER(u32),
                               u32]
    L.or_data_walk.restype = i32
    L._rep_ready = True
    return L


def q_time(v): return int(_report_protos().or_q_time(float(v)))
def uq_time(q): return float(_report_protos().or_uq_time(int(q)))
def q_rate(v): return int(_report_protos().or_q_rate(float(v)))
def uq_rate(q): return float(_report_protos().or_uq_rate(int(q)))
def q_loss(v): return int(_report_protos().or_q_loss(float(v)))
def uq_loss(q): return float(_report_protos().or_uq_loss(int(q)))


def report_build(src, dst, flow_id, protocol, duration, lat_ave, lat_min, lat_max, rate, loss,
                 offset=0.0, sign=0):
    """report_msg bytes after a window close (+ GetReport): returns (bytes, sign after)."""
    L = _report_protos()
    s = np.ascontiguousarray(np.asarray(src, ADDR_DTYPE).reshape(1))
    t = np.ascontiguousarray(np.asarray(dst, ADDR_DTYPE).reshape(1))
    b = np.zeros(52, np.uint8)
    sg = ctypes.c_int(sign)
    n = L.or_report_build(_ptr(s), _ptr(t), flow_id, protocol, duration, lat_ave, lat_min,
                          lat_max, rate, loss, offset, ctypes.byref(sg), _ptr(b))
    return b[:n].tobytes(), sg.value


def log_report(report, duration, rate, loss, lat_ave, lat_min, lat_max, count, sec, usec,
               opts=0):
    L = _report_protos()
    r = np.zeros(52, np.uint8)
    r[:len(report)] = np.frombuffer(report, np.uint8)
    out = np.zeros(512, np.uint8)
    n = L.or_log_report(_ptr(r), duration, rate, loss, lat_ave, lat_min, lat_max, count, sec,
                        usec, opts, _ptr(out))
    return out[:n].tobytes()


def log_report_recv(report, reporter, sec, usec, opts=0):
    L = _report_protos()
    r = np.zeros(52, np.uint8)
    r[:len(report)] = np.frombuffer(report, np.uint8)
    a = np.ascontiguousarray(np.asarray(reporter, ADDR_DTYPE).reshape(1))
    out = np.zeros(512, np.uint8)
    n = L.or_log_report_recv(_ptr(r), _ptr(a), sec, usec, opts, _ptr(out))
    return out[:n].tobytes()


def data_walk(payload: bytes, controller=True, cap=4096):
    """ProcessRecvMessage over one MGEN_DATA payload: (status, [(flow, status)], [offsets])."""
    L = _report_protos()
    p = np.frombuffer(bytes(payload) + b"\0" * 4, np.uint8).copy()
    cmds = np.zeros(cap, np.uint32)
    reps = np.zeros(cap, np.uint32)
    nc, nr = ctypes.c_uint32(0), ctypes.c_uint32(0)
    st = L.or_data_walk(_ptr(p), len(payload), int(controller), _ptr(cmds), ctypes.byref(nc), cap,
                        _ptr(reps), ctypes.byref(nr), cap)
    c = [(int(x) >> 2, int(x) & 3) for x in cmds[:min(nc.value, cap)]]
    return st, c, [int(x) for x in reps[:min(nr.value, cap)]]


# ---------------------------------------------------------------- pcap2mgen
def _pcap_protos():
    L = lib()
    if getattr(L, "_pcap_ready", False):
        return L
    P, u32, u64, i32, d = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                           ctypes.c_double)
    L.or_pcap_frame.argtypes = [P, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32), P,
                                ctypes.POINTER(i32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.or_pcap_frame.restype = i32
    L.or_pcap2mgen.argtypes = [P, u64, i32, i32, d, u32, P, u64, ctypes.POINTER(u64), P]
    L.or_pcap2mgen.restype = u64
    L._pcap_ready = True
    return L


def pcap_frame(rec: bytes, link_type=1, flags=0):
    """One pcap record (16-byte header + data): (status, udp_off, udp_len, src, ttl, sec, usec)."""
    L = _pcap_protos()
    b = np.frombuffer(bytes(rec) + b"\0" * 8, np.uint8).copy()
    uo, ul, ttl = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
    sec, usec = ctypes.c_uint32(0), ctypes.c_uint32(0)
    src = np.zeros(1, ADDR_DTYPE)
    st = L.or_pcap_frame(_ptr(b), link_type, flags, ctypes.byref(uo), ctypes.byref(ul),
                         _ptr(src), ctypes.byref(ttl), ctypes.byref(sec), ctypes.byref(usec))
    return st, uo.value, ul.value, src[0], ttl.value, sec.value, usec.value


def pcap2mgen(file: bytes, analytics=False, log_rx=True, window=1.0, opts=0):
    """pcap2mgen's whole main loop: (log text, per-record frame status)."""
    L = _pcap_protos()
    f = np.frombuffer(bytes(file), np.uint8)
    npk = ctypes.c_uint64(0)
    st = np.zeros(max(1, len(file) // 16), np.uint8)
    need = L.or_pcap2mgen(_ptr(f), len(f), int(analytics), int(log_rx), float(window), opts,
                          None, 0, ctypes.byref(npk), _ptr(st))
    out = np.zeros(max(1, need), np.uint8)
    n = L.or_pcap2mgen(_ptr(f), len(f), int(analytics), int(log_rx), float(window), opts,
                       _ptr(out), len(out), ctypes.byref(npk), _ptr(st))
    assert n == need
    return out[:n].tobytes(), st[:npk.value].copy()


# ---------------------------------------------------------------- ConvertBinaryLog
def convert_binary_log(log: bytes, log_rx=True, flush=False, opts=0):
    """MgenMsg::ConvertBinaryLog over a binary log image: (text, status, records)."""
    L = lib()
    if not getattr(L, "_bl_ready", False):
        P, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
        L.or_convert_binary_log.argtypes = [P, u64, i32, i32, u32, P, u64, ctypes.POINTER(i32),
                                            ctypes.POINTER(u64)]
        L.or_convert_binary_log.restype = u64
        L._bl_ready = True
    f = np.frombuffer(bytes(log) + b"\0" * 8, np.uint8)
    st, nr = ctypes.c_int(0), ctypes.c_uint64(0)
    need = L.or_convert_binary_log(_ptr(f), len(log), int(log_rx), int(flush), opts, None, 0,
                                   ctypes.byref(st), ctypes.byref(nr))
    out = np.zeros(max(1, need), np.uint8)
    L.or_convert_binary_log(_ptr(f), len(log), int(log_rx), int(flush), opts, _ptr(out), len(out),
                            ctypes.byref(st), ctypes.byref(nr))
    return out[:need].tobytes(), st.value, nr.value


# ---------------------------------------------------------------- CPU baselines (bench.py)
def udp_pack_batch_mt(tmpl, desc, pool, slab_bytes, rec_off=None, stride=0, checksum=True,
                      nthreads=1):
    """or_udp_pack_batch over nthreads host threads (zero fill)."""
    n = len(desc)
    slab = np.zeros(slab_bytes, np.uint8)
    lens = np.zeros(n, np.uint32)
    pool = np.ascontiguousarray(pool if pool is not None and len(pool) else np.zeros(1, np.uint8))
    lib().or_udp_pack_batch_mt(_ptr(tmpl), _ptr(desc), n, _ptr(pool), _ptr(slab), _ptr(rec_off),
                               stride, int(checksum), _ptr(lens), nthreads)
    return slab, lens


def flow_reduce_batch_mt(n_flows, flow_idx, seq, tx_sec, tx_usec, msg_len, rx_sec, rx_usec,
                         window=1.0, nthreads=1):
    """MgenAnalytic::Update per record over n_flows flows on nthreads threads (flows split by
    index); returns the per-flow report counts."""
    flows = (Analytic * n_flows)()
    for f in range(n_flows):
        lib().or_analytic_init(ctypes.byref(flows[f]), window)
    cols = [np.ascontiguousarray(x, dt) for x, dt in
            ((flow_idx, np.uint32), (seq, np.uint32), (tx_sec, np.uint32), (tx_usec, np.uint32),
             (msg_len, np.uint16), (rx_sec, np.uint32), (rx_usec, np.uint32))]
    counts = np.zeros(n_flows, np.uint32)
    lib().or_flow_reduce_batch_mt(flows, n_flows, *[_ptr(c) for c in cols], len(flow_idx),
                                  _ptr(counts), nthreads)
    return counts
