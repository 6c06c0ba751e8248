"""Python mirror of the C ABI layouts in include/mgenx.h (no torch, no HIP needed)."""
from __future__ import annotations

import ctypes

import numpy as np

# MgenMsg::Error (include/mgenMsg.h:63-70) and flags (:89-97)
ERROR_NONE, ERROR_VERSION, ERROR_CHECKSUM, ERROR_LENGTH, ERROR_DSTADDR = 0, 1, 2, 3, 4
ERROR_OOB = 0x80
FLAG_CONTINUES, FLAG_END_OF_MSG, FLAG_CHECKSUM, FLAG_LAST_BUFFER, FLAG_CHECKSUM_ERROR = (
    0x01, 0x02, 0x04, 0x08, 0x10)
OPT_CHECKSUM_FORCE, OPT_TCP, OPT_SKIP_CRC = 0x1, 0x2, 0x4
# mgenx_unpack_last_kernel: which kernel the dispatch chose (include/mgenx.h)
(UNPACK_K_HEADER, UNPACK_K_GENERAL, UNPACK_K_VAR, UNPACK_K_FIXED, UNPACK_K_FIXED_RING,
 UNPACK_K_OTHER, UNPACK_K_LONG) = 1, 2, 3, 4, 5, 6, 7
PACK_CHECKSUM, PACK_RANDOM_FILL, PACK_RAW = 0x1, 0x2, 0x4
# MGENX_DEC_*: members an Unpack assigned (mgenx_cols.decoded)
DEC_MSGLEN, DEC_BASE, DEC_DST, DEC_HDRLEN = 0x01, 0x02, 0x04, 0x08
DEC_HOST, DEC_GPS, DEC_PTYPE, DEC_PLEN = 0x10, 0x20, 0x40, 0x80
SCAN_TCP, SCAN_SINK = 0, 1

# mgenx_flow_tmpl (68 bytes) and mgenx_pack_desc (20 bytes)
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
assert TMPL_DTYPE.itemsize == 68

DESC_DTYPE = np.dtype([
    ("tmpl", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"), ("tx_usec", "<u4"),
    ("msg_len", "<u2"), ("flags", "u1"), ("rsv", "u1"),
], align=True)
assert DESC_DTYPE.itemsize == 20

# (name, torch dtype name, elements per record)
COLS_CORE = (
    ("flow_id", "int32", 1), ("seq_num", "int32", 1), ("tx_sec", "int32", 1),
    ("tx_usec", "int32", 1), ("msg_len", "int16", 1), ("dst_port", "int16", 1),
    ("flags", "uint8", 1), ("err", "uint8", 1), ("dst_type", "uint8", 1),
    ("dst_len", "uint8", 1), ("dst_addr4", "int32", 1), ("payload_len", "int16", 1),
    ("payload_type", "uint8", 1), ("gps_status", "uint8", 1),
)
COLS_EXT = (
    ("hdr_len", "int16", 1), ("payload_off", "int32", 1), ("host_port", "int16", 1),
    ("host_type", "uint8", 1), ("host_len", "uint8", 1), ("host_addr", "uint8", 16),
    ("dst_addr", "uint8", 16), ("lat_raw", "int32", 1), ("lon_raw", "int32", 1),
    ("alt", "int32", 1),
)
COLS_DEC = (("decoded", "uint8", 1),)   # after `rows` in the struct
CORE_BYTES_PER_RECORD = 32


class MgenxCols(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name, _, _ in COLS_CORE + COLS_EXT] + \
        [("rows", ctypes.c_void_p), ("decoded", ctypes.c_void_p)]


# mgenx_rec: one decoded record's core fields (32 B, row-major alternative to the columns)
REC_DTYPE = np.dtype([
    ("flow_id", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"), ("tx_usec", "<u4"),
    ("dst_addr4", "<u4"), ("msg_len", "<u2"), ("dst_port", "<u2"), ("payload_len", "<u2"),
    ("flags", "u1"), ("err", "u1"), ("dst_type", "u1"), ("dst_len", "u1"),
    ("payload_type", "u1"), ("gps_status", "u1")])
assert REC_DTYPE.itemsize == 32


def gps_raw(deg: float) -> int:
    """(UINT32)((deg + 180.0) * 60000.0) as MgenMsg::Pack computes it (mgenMsg.cpp:221,225)."""
    v = (deg + 180.0) * 60000.0
    return int(v) & 0xFFFFFFFF


def hex_payload(hexstr: str) -> bytes:
    """MgenPayload::SetPayloadString (mgenPayload.cpp:24-55): odd length reads the NUL as 0,
    non-hex characters decode as 0."""
    def nib(c):
        c = c.upper()
        return int(c, 16) if c in "0123456789ABCDEF" else 0
    n = len(hexstr) // 2 + len(hexstr) % 2
    out = bytearray(n)
    for i in range(n):
        hi = nib(hexstr[2 * i])
        lo = nib(hexstr[2 * i + 1]) if 2 * i + 1 < len(hexstr) else 0
        out[i] = (hi << 4) | lo
    return bytes(out)


# stream framing (mgenx_stream_scan)
SCAN_TCP = 0
SCAN_SINK = 1
ADDR_DTYPE = np.dtype([("type", "u1"), ("len", "u1"), ("port", "<u2"), ("addr", "u1", 16)])
REPORT_KEY_DTYPE = np.dtype([("src", ADDR_DTYPE), ("dst", ADDR_DTYPE), ("flow_id", "<u4"),
                             ("protocol", "u1"), ("rsv", "u1", 3)])   # mgenx_report_key
REPORT_MAX = 52
DATA_CONTROLLER = 0x1
RX_NOLOG = 0x1        # MGENX_RX_NOLOG
RX_FORCE = 0x2        # MGENX_RX_FORCE
RX_PREV = 0xFFFFFFFF  # MGENX_RX_PREV
RX_STATE_DTYPE = np.dtype([
    ("tx_sec", "<u4"), ("tx_usec", "<u4"), ("lat_raw", "<u4"), ("lon_raw", "<u4"),
    ("alt", "<i4"), ("payload_off", "<u4"), ("dst_port", "<u2"), ("hdr_len", "<u2"),
    ("payload_len", "<u2"), ("flags", "u1"), ("dst_type", "u1"), ("dst_len", "u1"),
    ("payload_type", "u1"), ("rsv", "u1", 2), ("dst_addr", "u1", 16)])   # mgenx_rx_state
SCAN_HALO = 65536     # MGENX_SCAN_HALO: bytes past a shard a record may extend into
SCAN_REUSE = 1        # MGENX_SCAN_REUSE


class ScanInfo(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
                ("status", ctypes.c_int32), ("candidates", ctypes.c_uint32),
                ("resolved", ctypes.c_uint64), ("path", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


# per-flow analytics (mgenx_flow_*): layouts of include/mgenx.h
FLOW_STATE_BYTES = 256
FLOW_REPORT_DTYPE = np.dtype([
    ("flow", "<u4"), ("index", "<u4"), ("start_sec", "<i8"), ("start_usec", "<i8"),
    ("duration", "<f8"), ("msg_count", "<u8"), ("rate", "<f8"), ("loss", "<f8"),
    ("latency_ave", "<f8"), ("latency_min", "<f8"), ("latency_max", "<f8"),
    ("rx_sec", "<i8"), ("rx_usec", "<i8")])
FLOW_COUNTERS_DTYPE = np.dtype([
    ("msg_count", "<u8"), ("byte_count", "<u8"), ("dup_count", "<u8"), ("n_reports", "<u8"),
    ("latency_sum", "<f8"), ("latency_min", "<f8"), ("latency_max", "<f8"),
    ("seq_start", "<u8")])
FLOW_STATE_DTYPE = np.dtype([
    ("mask", "<u4", (32,)), ("mask_first", "<u4"), ("mask_n", "<u4"), ("seq_start", "<u4"),
    ("window_valid", "<u4"), ("win_start_sec", "<i8"), ("win_start_usec", "<i8"),
    ("win_end_sec", "<i8"), ("win_end_usec", "<i8"), ("window_size", "<f8"),
    ("msg_count", "<u8"), ("byte_count", "<u8"), ("dup_count", "<u8"),
    ("latency_sum", "<f8"), ("latency_min", "<f8"), ("latency_max", "<f8"),
    ("n_reports", "<u8"), ("rsv", "<u8", (2,))])
assert FLOW_STATE_DTYPE.itemsize == FLOW_STATE_BYTES
assert FLOW_REPORT_DTYPE.itemsize == 96 and FLOW_COUNTERS_DTYPE.itemsize == 64


# ---- pcap2mgen / text interleave (include/mgenx.h) ----
class PcapInfo(ctypes.Structure):      # mgenx_pcap_info
    _fields_ = [("link_type", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("snaplen", ctypes.c_uint32), ("rsv", ctypes.c_uint32),
                ("n_records", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
                ("snap_bytes", ctypes.c_uint64)]


class TextSrc(ctypes.Structure):       # mgenx_text_src
    _fields_ = [("text", ctypes.c_void_p), ("line_off", ctypes.c_void_p),
                ("n_lines", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("index", ctypes.c_void_p), ("index_stride", ctypes.c_uint32),
                ("rsv", ctypes.c_uint32)]


TEXT_PER_RECORD, TEXT_OWNER, TEXT_MAP, TEXT_SCATTER = 0, 1, 2, 3
LOG_EPOCH, LOG_NO_DATA, LOG_NO_GPS, LOG_SKIP_ERR = 0x1, 0x2, 0x4, 0x8
FLOW_NONE = 0xFFFFFFFF
DLT_EN10MB, DLT_LINUX_SLL = 1, 113
PCAP_NSEC, PCAP_SWAPPED = 0x1, 0x2


class BinlogInfo(ctypes.Structure):    # mgenx_binlog_info
    _fields_ = [("n_records", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
                ("status", ctypes.c_int32), ("version", ctypes.c_uint32)]


BINLOG_OK, BINLOG_HEADER, BINLOG_TOO_LONG, BINLOG_EVENT, BINLOG_SHORT = 0, 1, 2, 3, 4
BINLOG_NO_RX, BINLOG_FLUSH = 0x1, 0x2


# mgenx_unpacked (include/mgenx.h): one message decoded by the resident worker
UNPACKED_DTYPE = np.dtype([
    ("flow_id", "<u4"), ("seq_num", "<u4"), ("tx_sec", "<u4"), ("tx_usec", "<u4"),
    ("payload_off", "<u4"), ("lat_raw", "<u4"), ("lon_raw", "<u4"), ("alt", "<i4"),
    ("msg_len", "<u2"), ("dst_port", "<u2"), ("payload_len", "<u2"), ("hdr_len", "<u2"),
    ("host_port", "<u2"), ("flags", "u1"), ("err", "u1"), ("dst_type", "u1"), ("dst_len", "u1"),
    ("payload_type", "u1"), ("gps_status", "u1"), ("host_type", "u1"), ("host_len", "u1"),
    ("decoded", "u1"), ("version", "u1"), ("rsv", "u1", 2),
    ("dst_addr", "u1", 16), ("host_addr", "u1", 16),
], align=True)
assert UNPACKED_DTYPE.itemsize == 88
