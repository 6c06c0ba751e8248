"""mgen_amd -- MI355X-native MgenMsg pack/parse engine (host binding).

Thin ctypes binding of the C ABI in ``include/mgenx.h`` (libmgenx.so, built from
``mgen_amd/csrc`` for gfx950).  PyTorch is used only for device memory and streams.
There is no CPU fallback: if the HIP library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._abi import (  # noqa: F401
    COLS_CORE, COLS_DEC, COLS_EXT, DESC_DTYPE, TMPL_DTYPE, MgenxCols, ERROR_CHECKSUM, ERROR_DSTADDR,
    ERROR_LENGTH, ERROR_NONE, ERROR_OOB, ERROR_VERSION, FLAG_CHECKSUM, FLAG_CHECKSUM_ERROR,
    FLAG_LAST_BUFFER, OPT_CHECKSUM_FORCE, OPT_SKIP_CRC, OPT_TCP, PACK_CHECKSUM,
    PACK_RANDOM_FILL, SCAN_SINK, SCAN_TCP, ScanInfo, FLOW_COUNTERS_DTYPE, FLOW_REPORT_DTYPE,
    FLOW_STATE_BYTES, FLOW_STATE_DTYPE, REC_DTYPE, PACK_RAW, DEC_MSGLEN, DEC_BASE, DEC_DST,
    DEC_HDRLEN, DEC_HOST, DEC_GPS, DEC_PTYPE, DEC_PLEN, RX_NOLOG, RX_FORCE, RX_PREV,
    RX_STATE_DTYPE, SCAN_HALO, SCAN_REUSE, ADDR_DTYPE, REPORT_KEY_DTYPE, DATA_CONTROLLER,
    PcapInfo, TextSrc, TEXT_PER_RECORD, TEXT_OWNER, TEXT_MAP, TEXT_SCATTER, PCAP_NSEC, PCAP_SWAPPED, LOG_EPOCH, LOG_NO_DATA, LOG_NO_GPS,
    LOG_SKIP_ERR, FLOW_NONE, DLT_EN10MB, DLT_LINUX_SLL, BinlogInfo, BINLOG_NO_RX, BINLOG_FLUSH,
    UNPACK_K_HEADER, UNPACK_K_GENERAL, UNPACK_K_VAR, UNPACK_K_FIXED, UNPACK_K_FIXED_RING,
    UNPACK_K_OTHER, UNPACK_K_LONG, UNPACKED_DTYPE,
)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmgenx.so")
DIAG_LIB_PATH = os.path.join(HERE, "libmgenx_diag.so")   # + include/mgenx_diag.h

# every function include/mgenx.h declares (tests/test_abi_cpu.py checks the header agrees)
EXPORTED_SYMBOLS = (
    "mgenx_abi_version", "mgenx_ctx_create", "mgenx_ctx_destroy", "mgenx_last_error",
    "mgenx_ctx_device", "mgenx_unpack_batch", "mgenx_pack_prepare", "mgenx_set_fill_time",
    "mgenx_pack_batch", "mgenx_pack_msgs", "mgenx_pack_tcp", "mgenx_crc32_update", "mgenx_crc32_batch",
    "mgenx_tcp_rx_persist", "mgenx_report_build", "mgenx_log_report_text", "mgenx_data_walk",
    "mgenx_log_report_recv_text", "mgenx_log_send_text", "mgenx_log_send_binary",
    "mgenx_stream_scan", "mgenx_stream_scan_exits", "mgenx_stream_scan_range", "mgenx_flow_init", "mgenx_flow_reduce", "mgenx_flow_export",
    "mgenx_log_recv_text", "mgenx_log_recv_binary", "mgenx_comm_unique_id", "mgenx_comm_init",
    "mgenx_comm_destroy", "mgenx_allreduce_flows", "mgenx_allgather_u64",
    "mgenx_flow_table_create", "mgenx_flow_table_destroy", "mgenx_flow_lookup",
    "mgenx_flow_reduce_ex", "mgenx_flow_keys", "mgenx_flow_span", "mgenx_text_interleave",
    "mgenx_pcap_index",
    "mgenx_pcap_parse", "mgenx_binlog_index", "mgenx_convert_binary_log",
    "mgenx_unpack_last_kernel", "mgenx_pcap_snap", "mgenx_flow_reduce_rows",
    "mgenx_worker_create", "mgenx_worker_destroy", "mgenx_worker_unpack", "mgenx_worker_crc32",
    "mgenx_worker_pack", "mgenx_worker_stop", "mgenx_worker_info", "mgenx_worker_recv",
    "mgenx_worker_flow_update",
)
DIAG_SYMBOLS = ("mgenx_set_tuning", "mgenx_diag_stream_read", "mgenx_diag_group_rw",
                "mgenx_diag_seg_prof", "mgenx_diag_stream_read_w", "mgenx_diag_worker_stamps",
                "mgenx_diag_chain_prof")


class MgenxError(RuntimeError):
    pass


_libs = {}


def load(diag: bool = False):
    """Load libmgenx.so (or the diagnostics build libmgenx_diag.so); fails loudly when the
    HIP build is missing."""
    path = DIAG_LIB_PATH if diag else LIB_PATH
    # geometry experiments (scripts/*_exp.sh): another build of the same sources
    path = os.environ.get("MGENX_LIB_OVERRIDE", path)
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise MgenxError(f"{path} not built: run __graft_entry__.build() "
                         "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(path)
    P, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.mgenx_abi_version.restype = i32
    L.mgenx_ctx_create.argtypes = [i32, ctypes.POINTER(P)]
    L.mgenx_ctx_destroy.argtypes = [P]
    L.mgenx_last_error.argtypes = [P]
    L.mgenx_last_error.restype = ctypes.c_char_p
    L.mgenx_unpack_batch.argtypes = [P, P, u64, P, u64, P, u32, u32,
                                     ctypes.POINTER(MgenxCols), u32, P]
    L.mgenx_unpack_last_kernel.argtypes = [P]
    L.mgenx_unpack_last_kernel.restype = i32
    L.mgenx_pack_prepare.argtypes = [P, P, u32, P, P, P]
    L.mgenx_set_fill_time.argtypes = [P, u32]
    L.mgenx_pack_batch.argtypes = [P, P, P, P, u32, P, P, u64, P, u64, P, u32, u32, P]
    L.mgenx_pack_msgs.argtypes = [P, P, P, P, u32, P, P, u64, P, u64, P, P, P, P, P, u32, u32,
                                  P]
    L.mgenx_pack_tcp.argtypes = [P, P, P, P, P, u32, P, P, u64, P, ctypes.POINTER(u64), u32,
                                 u32, P]
    L.mgenx_crc32_batch.argtypes = [P, P, P, P, u32, P, P]
    L.mgenx_crc32_update.argtypes = [P, P, P, P, u32, P, P, P]
    L.mgenx_ctx_device.argtypes = [P]
    L.mgenx_comm_unique_id.argtypes = [P]
    L.mgenx_comm_init.argtypes = [P, i32, i32, P, ctypes.POINTER(P)]
    L.mgenx_comm_destroy.argtypes = [P]
    L.mgenx_allreduce_flows.argtypes = [P, P, P, u32, P]
    L.mgenx_allgather_u64.argtypes = [P, P, P, P, u32, P]
    L.mgenx_flow_table_create.argtypes = [P, u32, ctypes.POINTER(P)]
    L.mgenx_flow_table_destroy.argtypes = [P]
    L.mgenx_flow_lookup.argtypes = [P, P, ctypes.POINTER(MgenxCols), P, u32, P, P, P]
    L.mgenx_flow_reduce_ex.argtypes = [P, P, P, P, P, P, P, P, u32, P, u32, P, u32, P, P, P]
    L.mgenx_flow_keys.argtypes = [P, P, i32, P, u32, P]
    L.mgenx_flow_span.argtypes = [P, P, P, P, u32, u32, P, P, P]
    L.mgenx_text_interleave.argtypes = [P, P, u32, u32, P, u64, P, P]
    L.mgenx_pcap_index.argtypes = [P, u64, P, u64, ctypes.POINTER(PcapInfo)]
    L.mgenx_pcap_parse.argtypes = [P, P, u64, P, u32, u32, u32, P, P, P, P, P, P, P, P]
    L.mgenx_pcap_snap.argtypes = [P, P, u64, u64, P, u32, u32, P, P, P, P]
    L.mgenx_binlog_index.argtypes = [P, u64, P, u64, ctypes.POINTER(BinlogInfo)]
    L.mgenx_convert_binary_log.argtypes = [P, P, u64, P, u32, u32, u32, P, u64, P, P]
    if diag:
        L.mgenx_set_tuning.argtypes = [P, i32, i32]
        L.mgenx_diag_stream_read.argtypes = [P, P, u64, P, i32, P]
        L.mgenx_diag_group_rw.argtypes = [P, P, u64, P, i32, P]
        L.mgenx_diag_seg_prof.argtypes = [P, i32]
        L.mgenx_diag_stream_read_w.argtypes = [P, P, u64, P, i32, i32, P]
        L.mgenx_diag_worker_stamps.argtypes = [P, P]
        L.mgenx_diag_chain_prof.argtypes = [P]
    L.mgenx_stream_scan.argtypes = [P, P, u64, i32, P, P, u64, ctypes.POINTER(ScanInfo), P]
    L.mgenx_tcp_rx_persist.argtypes = [P, P, P, P, u32, P, P, P, u32, P]
    L.mgenx_report_build.argtypes = [P, P, u32, u32, P, P, P, P, P, P, P]
    L.mgenx_log_report_text.argtypes = [P, P, P, u32, u32, P, u32, P, u64, P, P]
    L.mgenx_data_walk.argtypes = [P, P, P, u64, P, u32, u32, P, P, P, u32, P, u32, P, P]
    L.mgenx_log_report_recv_text.argtypes = [P, P, P, u32, P, P, P, u32, P, u64, P, P]
    L.mgenx_log_send_text.argtypes = [P, P, P, P, P, P, u32, i32, u32, P, u64, P, P]
    L.mgenx_log_send_binary.argtypes = [P, P, P, P, P, P, u64, P, u64, u32, i32, P, u64, P, P]
    L.mgenx_stream_scan_exits.argtypes = [P, P, u64, i32, u64, u64, P, P, u32,
                                          ctypes.POINTER(u32), P]
    L.mgenx_stream_scan_range.argtypes = [P, P, u64, i32, u64, u64, i32, P, P, u64,
                                          ctypes.POINTER(ScanInfo), P]
    L.mgenx_flow_init.argtypes = [P, P, u32, ctypes.c_double, P]
    L.mgenx_flow_reduce.argtypes = [P, P, P, P, P, P, P, P, u32, P, u32, P, u32, P, P]
    L.mgenx_flow_reduce_rows.argtypes = [P, P, P, P, P, u32, P, u32, P, u32, P, P, P]
    L.mgenx_flow_export.argtypes = [P, P, u32, P, P]
    L.mgenx_log_recv_text.argtypes = [P, P, P, u64, ctypes.POINTER(MgenxCols), P, P, P, P, u32,
                                      i32, u32, P, u64, P, P]
    L.mgenx_log_recv_binary.argtypes = [P, P, u64, P, u64, P, ctypes.POINTER(MgenxCols), P, P,
                                        P, u32, i32, P, u64, P, P]
    L.mgenx_worker_create.argtypes = [P, u32, ctypes.POINTER(P)]
    L.mgenx_worker_destroy.argtypes = [P]
    L.mgenx_worker_stop.argtypes = [P]
    L.mgenx_worker_info.argtypes = [P, ctypes.POINTER(u32)]
    L.mgenx_worker_recv.argtypes = [P, ctypes.c_char_p, u32, u32, P, ctypes.POINTER(u32),
                                    ctypes.POINTER(u32)]
    L.mgenx_worker_flow_update.argtypes = [P, P, u32, u32, u32, u32, u32, u32, u32,
                                           ctypes.POINTER(u32), P]
    L.mgenx_worker_unpack.argtypes = [P, ctypes.c_char_p, u32, P]
    L.mgenx_worker_crc32.argtypes = [P, ctypes.c_char_p, u32, u32, ctypes.POINTER(u32)]
    L.mgenx_worker_pack.argtypes = [P, P, ctypes.c_char_p, P, u32, u32, u32, u32, P,
                                    ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    _libs[path] = L
    return L


def _ptr(t):
    """Raw device pointer of a torch tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device):
    import torch
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(device))


class Engine:
    """One mgenx context on one GPU (``mgenx_ctx``)."""

    def __init__(self, device: int = 0, diag: bool = False):
        import torch
        self.torch = torch
        self.device = device
        self.lib = load(diag)
        self.ctx = ctypes.c_void_p()
        rc = self.lib.mgenx_ctx_create(device, ctypes.byref(self.ctx))
        if rc != 0:
            raise MgenxError(f"mgenx_ctx_create({device}) failed: {rc}")

    def close(self):
        if self.ctx:
            self.lib.mgenx_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.mgenx_last_error(self.ctx)
            raise MgenxError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    # ------------------------------------------------------------ single messages
    def worker(self, idle_ms: int = 200):
        """A resident single-message worker on this engine's device (mgenx_worker_*)."""
        return Worker(self, idle_ms)

    # ------------------------------------------------------------ columns
    def alloc_cols(self, n: int, ext: bool = False):
        torch = self.torch
        dev = f"cuda:{self.device}"
        cols = {name: torch.empty(n * w if w > 1 else n, dtype=getattr(torch, dt), device=dev)
                for name, dt, w in COLS_CORE}
        if ext:
            for name, dt, w in COLS_EXT + COLS_DEC:
                cols[name] = torch.empty(n * w if w > 1 else n, dtype=getattr(torch, dt),
                                         device=dev)
        return cols

    def alloc_rows(self, n: int):
        """mgenx_rec rows (32 B per record) as a uint8 tensor; pass as cols={"rows": t}."""
        return self.torch.empty(n * 32, dtype=self.torch.uint8, device=f"cuda:{self.device}")

    @staticmethod
    def _cols_struct(cols):
        s = MgenxCols()
        for name, _ in MgenxCols._fields_:
            t = cols.get(name)
            setattr(s, name, t.data_ptr() if t is not None else None)
        return s

    # ------------------------------------------------------------ unpack
    def unpack(self, slab, n, *, rec_off=None, stride=0, rec_len=None, fixed_len=0, opts=0,
               cols=None, ext=False, slab_bytes=None):
        """MgenMsg::Unpack + receive CRC check over n records (async on the current stream)."""
        if cols is None:
            cols = self.alloc_cols(n, ext)
        cs = self._cols_struct(cols)
        nbytes = slab.numel() if slab_bytes is None else slab_bytes
        rc = self.lib.mgenx_unpack_batch(self.ctx, _ptr(slab), nbytes, _ptr(rec_off), stride,
                                         _ptr(rec_len), fixed_len, n, ctypes.byref(cs), opts,
                                         _stream(self.device))
        self._check(rc, "mgenx_unpack_batch")
        return cols

    def last_unpack_kernel(self):
        """UNPACK_K_* of the kernel the last unpack() launched (mgenx_unpack_last_kernel)."""
        return int(self.lib.mgenx_unpack_last_kernel(self.ctx))

    def rx_state_init(self):
        """mgenx_rx_state of a fresh MgenMsg (GPS words 10800000 = 0 degrees), on the device."""
        from ._abi import RX_STATE_DTYPE
        st = np.zeros(1, RX_STATE_DTYPE)
        st["lat_raw"] = st["lon_raw"] = 10800000
        return self.torch.from_numpy(st.view(np.uint8).copy()).to(f"cuda:{self.device}")

    def tcp_rx_persist(self, slab, rec_off, rec_len, n, cols, state, *, payload_rec=None,
                       opts=0):
        """The TCP receiver's persistent rx_msg view of n decoded records, in place
        (mgenx_tcp_rx_persist); state: the 48-B mgenx_rx_state tensor (updated)."""
        cs = self._cols_struct(cols)
        rc = self.lib.mgenx_tcp_rx_persist(self.ctx, _ptr(slab), _ptr(rec_off), _ptr(rec_len), n,
                                           ctypes.byref(cs), _ptr(state), _ptr(payload_rec), opts,
                                           _stream(self.device))
        self._check(rc, "mgenx_tcp_rx_persist")
        return cols

    # ------------------------------------------------------------ event log
    def log_recv_text(self, slab, n, cols, src, rx_sec, rx_usec, *, rec_off=None, stride=0,
                      ttl=None, protocol=1, opts=0, text_cap=None):
        """RECV / RERR text log lines of n decoded records (mgenx_log_recv_text).  cols: the
        unpack outputs with the extended columns; src: uint8 tensor of n x 20 (mgenx_addr).
        Returns (text tensor, line offsets tensor of n + 1)."""
        torch = self.torch
        dev = slab.device
        line_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap = text_cap if text_cap is not None else max(1, n) * 160
        for _ in range(2):
            text = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
            cs = self._cols_struct(cols)
            rc = self.lib.mgenx_log_recv_text(self.ctx, _ptr(slab), _ptr(rec_off), stride,
                                              ctypes.byref(cs), _ptr(src), _ptr(rx_sec),
                                              _ptr(rx_usec), _ptr(ttl), n, protocol, opts,
                                              _ptr(text), cap, _ptr(line_off),
                                              _stream(self.device))
            self._check(rc, "mgenx_log_recv_text")
            total = int(line_off[n].item())
            if total <= cap:
                return text[:total], line_off
            cap = total
        raise MgenxError("mgenx_log_recv_text: text did not fit")

    def log_recv_binary(self, slab, n, cols, src, rx_sec, rx_usec, *, rec_off=None, stride=0,
                        rec_len=None, protocol=1, slab_bytes=None, cap=None):
        """Binary RECV / RERR log records (mgenx_log_recv_binary; rec_len: the received
        lengths, else each record's msg_len bounds its bytes).  Returns (bytes tensor,
        record positions tensor of n + 1)."""
        torch = self.torch
        dev = slab.device
        pos = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap = cap if cap is not None else max(1, n) * 128
        sb = slab.numel() if slab_bytes is None else slab_bytes
        for _ in range(2):
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
            cs = self._cols_struct(cols)
            rc = self.lib.mgenx_log_recv_binary(self.ctx, _ptr(slab), sb, _ptr(rec_off), stride,
                                                _ptr(rec_len), ctypes.byref(cs), _ptr(src),
                                                _ptr(rx_sec),
                                                _ptr(rx_usec), n, protocol, _ptr(out), cap,
                                                _ptr(pos), _stream(self.device))
            self._check(rc, "mgenx_log_recv_binary")
            total = int(pos[n].item())
            if total <= cap:
                return out[:total], pos
            cap = total
        raise MgenxError("mgenx_log_recv_binary: output did not fit")

    # ------------------------------------------------------------ pack
    def pack_prepare(self, tmpl, n_tmpl, pool, tmpl_crc):
        rc = self.lib.mgenx_pack_prepare(self.ctx, _ptr(tmpl), n_tmpl, _ptr(pool),
                                         _ptr(tmpl_crc), _stream(self.device))
        self._check(rc, "mgenx_pack_prepare")

    def set_fill_time(self, fill_time: int):
        self._check(self.lib.mgenx_set_fill_time(self.ctx, fill_time), "mgenx_set_fill_time")

    def pack(self, tmpl, tmpl_crc, desc, n, pool, slab, *, rec_off=None, stride=0, opts=0,
             fill_time=0, out_len=None):
        if out_len is None:
            out_len = self.torch.empty(n, dtype=self.torch.int32, device=slab.device)
        rc = self.lib.mgenx_pack_batch(self.ctx, _ptr(tmpl), _ptr(tmpl_crc), _ptr(desc), n,
                                       _ptr(pool), _ptr(slab), slab.numel(), _ptr(rec_off),
                                       stride, _ptr(out_len), opts, fill_time,
                                       _stream(self.device))
        self._check(rc, "mgenx_pack_batch")
        return out_len

    def pack_msgs(self, tmpl, tmpl_crc, desc, n, pool, slab, *, rec_off=None, stride=0,
                  buf_len=None, crc_in=None, opts=0, fill_time=0):
        """MgenMsg::Pack alone (mgenx_pack_msgs): returns (out_len, tx_crc, state) tensors."""
        torch = self.torch
        out_len = torch.empty(n, dtype=torch.int32, device=slab.device)
        tx_crc = torch.empty(n, dtype=torch.int32, device=slab.device)
        state = torch.empty(n, dtype=torch.int32, device=slab.device)
        rc = self.lib.mgenx_pack_msgs(self.ctx, _ptr(tmpl), _ptr(tmpl_crc), _ptr(desc), n,
                                      _ptr(pool), _ptr(slab), slab.numel(), _ptr(rec_off), stride,
                                      _ptr(buf_len), _ptr(crc_in), _ptr(out_len), _ptr(tx_crc),
                                      _ptr(state), opts, fill_time, _stream(self.device))
        self._check(rc, "mgenx_pack_msgs")
        return out_len, tx_crc, state

    def pack_tcp(self, tmpl, tmpl_crc, desc, msg_total, n, pool, *, opts=0, fill_time=0,
                 out=None, offs=None):
        """The MgenTcpTransport transmit stream of n messages (mgenx_pack_tcp): returns
        (stream uint8 tensor, message offsets int64 tensor).  out: a stream buffer to fill
        (else one is sized by a first call)."""
        torch = self.torch
        dev = msg_total.device
        if offs is None:
            offs = torch.empty(n, dtype=torch.int64, device=dev)
        total = ctypes.c_uint64(0)
        cap = None if out is None else out.numel()
        if cap is None:  # size query: a first call with no room reports the length
            rc = self.lib.mgenx_pack_tcp(self.ctx, _ptr(tmpl), _ptr(tmpl_crc), _ptr(desc),
                                         _ptr(msg_total), n, _ptr(pool), None, 0, _ptr(offs),
                                         ctypes.byref(total), opts, fill_time,
                                         _stream(self.device))
            if rc not in (0, -1):
                self._check(rc, "mgenx_pack_tcp")
            cap = int(total.value)
            out = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        rc = self.lib.mgenx_pack_tcp(self.ctx, _ptr(tmpl), _ptr(tmpl_crc), _ptr(desc),
                                     _ptr(msg_total), n, _ptr(pool), _ptr(out), cap, _ptr(offs),
                                     ctypes.byref(total), opts, fill_time, _stream(self.device))
        self._check(rc, "mgenx_pack_tcp")
        return out[:int(total.value)], offs

    def crc32_update(self, data, off, length, n, state_in, out=None):
        """MgenMsg::ComputeCRC32 running states (mgenx_crc32_update)."""
        if out is None:
            out = self.torch.empty(n, dtype=self.torch.int32, device=data.device)
        rc = self.lib.mgenx_crc32_update(self.ctx, _ptr(data), _ptr(off), _ptr(length), n,
                                         _ptr(state_in), _ptr(out), _stream(self.device))
        self._check(rc, "mgenx_crc32_update")
        return out

    def set_pack_variant(self, v: int):
        self._check(self.lib.mgenx_set_tuning(self.ctx, 2, v), "mgenx_set_tuning")

    def set_unpack_variant(self, v: int):
        self._check(self.lib.mgenx_set_tuning(self.ctx, 1, v), "mgenx_set_tuning")

    def stream_read(self, data, grid=2048, scratch=None):
        if scratch is None:
            scratch = self.torch.empty(grid, dtype=self.torch.int32, device=data.device)
        rc = self.lib.mgenx_diag_stream_read(self.ctx, _ptr(data), data.numel(), _ptr(scratch),
                                             grid, _stream(self.device))
        self._check(rc, "mgenx_diag_stream_read")

    def stream_read_w(self, data, width, grid=2048, scratch=None):
        """Diagnostic: coalesced read at `width` (4, 8, 24) bytes per lane."""
        if scratch is None:
            scratch = self.torch.empty(grid, dtype=self.torch.int32, device=data.device)
        rc = self.lib.mgenx_diag_stream_read_w(self.ctx, _ptr(data), data.numel(), _ptr(scratch),
                                               grid, width, _stream(self.device))
        self._check(rc, "mgenx_diag_stream_read_w")

    def group_rw(self, data, out, mode=1):
        """Diagnostic: the fixed unpack's read pattern (+ 512-B stores per 16-KiB group)."""
        rc = self.lib.mgenx_diag_group_rw(self.ctx, _ptr(data), data.numel(), _ptr(out), mode,
                                          _stream(self.device))
        self._check(rc, "mgenx_diag_group_rw")

    def stream_scan(self, data, mode=SCAN_TCP, cap=None, nbytes=None, out=None):
        """TCP / SINK record framing of a device byte stream (mgenx_stream_scan).  Returns
        (rec_off int64 tensor, rec_len int32 tensor, ScanInfo); synchronous.  out: optional
        preallocated (rec_off int64, rec_len int32) tensors of equal length (the capacity)."""
        torch = self.torch
        nbytes = data.numel() if nbytes is None else nbytes
        if out is not None:
            offs, lens = out
            if offs.dtype != torch.int64 or lens.dtype != torch.int32 or \
                    offs.numel() != lens.numel():
                raise ValueError("stream_scan out: (int64, int32) tensors of one length")
            cap = offs.numel()
        else:
            if cap is None:
                cap = nbytes // 4 + 1
            offs = torch.empty(cap, dtype=torch.int64, device=data.device)
            lens = torch.empty(cap, dtype=torch.int32, device=data.device)
        info = ScanInfo()
        rc = self.lib.mgenx_stream_scan(self.ctx, _ptr(data), nbytes, mode, _ptr(offs),
                                        _ptr(lens), cap, ctypes.byref(info),
                                        _stream(self.device))
        self._check(rc, "mgenx_stream_scan")
        n = min(int(info.n_records), cap)
        return offs[:n], lens[:n], info

    def stream_scan_exits(self, data, mode, window, limit, cap=4096, nbytes=None):
        """Step 1 of the sharded framing (mgenx_stream_scan_exits): builds the candidate
        tables of `data` and returns (entries, exits) uint64 device tensors of `cap` rows
        (as int64) plus the candidate count."""
        torch = self.torch
        nbytes = data.numel() if nbytes is None else nbytes
        ent = torch.empty(cap, dtype=torch.int64, device=data.device)
        ext = torch.empty(cap, dtype=torch.int64, device=data.device)
        cands = ctypes.c_uint32(0)
        rc = self.lib.mgenx_stream_scan_exits(self.ctx, _ptr(data), nbytes, mode, window, limit,
                                              _ptr(ent), _ptr(ext), cap, ctypes.byref(cands),
                                              _stream(self.device))
        self._check(rc, "mgenx_stream_scan_exits")
        return ent, ext, int(cands.value)

    def stream_scan_range(self, data, mode, entry, limit, reuse=False, cap=None, nbytes=None):
        """Records of the chain from `entry` below `limit` (mgenx_stream_scan_range); reuse:
        the tables of the last build on this engine (same tensor, unchanged)."""
        torch = self.torch
        nbytes = data.numel() if nbytes is None else nbytes
        if cap is None:
            cap = max(limit - entry, 0) // 4 + 1
        offs = torch.empty(max(cap, 1), dtype=torch.int64, device=data.device)
        lens = torch.empty(max(cap, 1), dtype=torch.int32, device=data.device)
        info = ScanInfo()
        rc = self.lib.mgenx_stream_scan_range(self.ctx, _ptr(data), nbytes, mode, entry, limit,
                                              1 if reuse else 0, _ptr(offs), _ptr(lens), cap,
                                              ctypes.byref(info), _stream(self.device))
        self._check(rc, "mgenx_stream_scan_range")
        n = min(int(info.n_records), cap)
        return offs[:n], lens[:n], info

    # ------------------------------------------------------------ analytics
    def flow_init(self, n_flows, window=1.0):
        """Fresh MgenAnalytic state for n_flows flows (mgenx_flow_init); a uint8 tensor of
        n_flows x 256 B."""
        flows = self.torch.empty(n_flows * FLOW_STATE_BYTES, dtype=self.torch.uint8,
                                 device=f"cuda:{self.device}")
        self._check(self.lib.mgenx_flow_init(self.ctx, _ptr(flows), n_flows, window,
                                             _stream(self.device)), "mgenx_flow_init")
        return flows

    def flow_reduce(self, flows, n_flows, flow_idx, seq, tx_sec, tx_usec, msg_len, rx_sec,
                    rx_usec, n=None, reports=None, per_flow=0, report_count=None,
                    report_rec=None):
        """MgenAnalytic::Update over records in receive order (mgenx_flow_reduce; with
        report_rec, mgenx_flow_reduce_ex: the record that closed each kept report).  Returns
        report_count (None when per_flow is 0 and none was passed: nothing to count into)."""
        torch = self.torch
        n = flow_idx.numel() if n is None else n
        if report_count is None and per_flow:
            report_count = torch.zeros(n_flows, dtype=torch.int32, device=flows.device)
        if report_rec is None:
            rc = self.lib.mgenx_flow_reduce(self.ctx, _ptr(flow_idx), _ptr(seq), _ptr(tx_sec),
                                            _ptr(tx_usec), _ptr(msg_len), _ptr(rx_sec),
                                            _ptr(rx_usec), n, _ptr(flows), n_flows, _ptr(reports),
                                            per_flow, _ptr(report_count), _stream(self.device))
        else:
            rc = self.lib.mgenx_flow_reduce_ex(self.ctx, _ptr(flow_idx), _ptr(seq), _ptr(tx_sec),
                                               _ptr(tx_usec), _ptr(msg_len), _ptr(rx_sec),
                                               _ptr(rx_usec), n, _ptr(flows), n_flows,
                                               _ptr(reports), per_flow, _ptr(report_count),
                                               _ptr(report_rec), _stream(self.device))
        self._check(rc, "mgenx_flow_reduce")
        return report_count

    def flow_reduce_rows(self, flows, n_flows, flow_idx, rows, rx_sec, rx_usec, n=None,
                         reports=None, per_flow=0, report_count=None, report_rec=None):
        """flow_reduce with seq / tx time / msg_len read from the unpack's 32-B rows
        (mgenx_flow_reduce_rows): the same result as the column form."""
        torch = self.torch
        n = flow_idx.numel() if n is None else n
        if report_count is None and per_flow:
            report_count = torch.zeros(n_flows, dtype=torch.int32, device=flows.device)
        rc = self.lib.mgenx_flow_reduce_rows(self.ctx, _ptr(flow_idx), _ptr(rows), _ptr(rx_sec),
                                             _ptr(rx_usec), n, _ptr(flows), n_flows,
                                             _ptr(reports), per_flow, _ptr(report_count),
                                             _ptr(report_rec), _stream(self.device))
        self._check(rc, "mgenx_flow_reduce_rows")
        return report_count

    def flow_keys(self, table, n_flows, protocol=1, keys=None):
        """The report_msg key of every flow index < n_flows (mgenx_flow_keys): a uint8
        tensor of n_flows x 48 (mgenx_report_key)."""
        if keys is None:
            keys = self.torch.zeros(max(n_flows, 1) * REPORT_KEY_DTYPE.itemsize,
                                    dtype=self.torch.uint8, device=f"cuda:{self.device}")
        self._check(self.lib.mgenx_flow_keys(self.ctx, table, protocol, _ptr(keys), n_flows,
                                             _stream(self.device)), "mgenx_flow_keys")
        return keys

    def flow_span(self, flow_idx, rx_sec, rx_usec, n, n_flows):
        """(most records of any flow index < n_flows, lowest, highest receive time in us) over
        those records (mgenx_flow_span; (0, 2**64 - 1, 0) when there are none): one read-back."""
        torch = self.torch
        dev = flow_idx.device
        counts = torch.empty(max(n_flows, 1), dtype=torch.int32, device=dev)
        out = torch.empty(3, dtype=torch.int64, device=dev)
        self._check(self.lib.mgenx_flow_span(self.ctx, _ptr(flow_idx), _ptr(rx_sec), _ptr(rx_usec),
                                             n, n_flows, _ptr(counts), _ptr(out),
                                             _stream(self.device)), "mgenx_flow_span")
        most, lo, hi = (int(v) & 0xFFFFFFFFFFFFFFFF for v in out.cpu().tolist())
        return most, lo, hi

    def text_interleave(self, sources, n_rec, cap=None):
        """mgenx_text_interleave: sources = [(kind, text, line_off, n_lines, index,
        index_stride)] (device tensors); returns (text, record offsets of n_rec + 1)."""
        torch = self.torch
        arr = (TextSrc * max(1, len(sources)))()
        keep = []
        for k, (kind, text, line_off, n_lines, index, stride) in enumerate(sources):
            arr[k].text = text.data_ptr() if text is not None and text.numel() else None
            arr[k].line_off = line_off.data_ptr()
            arr[k].n_lines = n_lines
            arr[k].kind = kind
            arr[k].index = index.data_ptr() if index is not None else None
            arr[k].index_stride = stride
            keep.append((text, line_off, index))
        dev = f"cuda:{self.device}"
        if cap is None:
            cap = sum(int(t.numel()) for _, t, *_ in sources if t is not None)
        rec_off = torch.empty(n_rec + 1, dtype=torch.int64, device=dev)
        for _ in range(2):
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
            self._check(self.lib.mgenx_text_interleave(self.ctx, arr, len(sources), n_rec,
                                                       _ptr(out), cap, _ptr(rec_off),
                                                       _stream(self.device)),
                        "mgenx_text_interleave")
            total = int(rec_off[n_rec].item())
            if total <= cap:
                return out[:total], rec_off
            cap = total
        raise MgenxError("mgenx_text_interleave: output did not fit")

    # ------------------------------------------------------------ ConvertBinaryLog
    def convert_binary_log(self, buf, rec_off, n, flags=0, opts=0, cap=None):
        """MgenMsg::ConvertBinaryLog over records indexed by binlog_index (device tensors):
        returns (text uint8 tensor, per-record offsets of n + 1).  Synchronous."""
        torch = self.torch
        dev = buf.device
        pos = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap = cap if cap is not None else max(1, n) * 200
        for _ in range(2):
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
            self._check(self.lib.mgenx_convert_binary_log(self.ctx, _ptr(buf), buf.numel(),
                                                          _ptr(rec_off), n, flags, opts,
                                                          _ptr(out), cap, _ptr(pos),
                                                          _stream(self.device)),
                        "mgenx_convert_binary_log")
            total = int(pos[n].item())
            if total <= cap:
                return out[:total], pos
            cap = total
        raise MgenxError("mgenx_convert_binary_log: text did not fit")

    # ------------------------------------------------------------ pcap2mgen
    def pcap_parse(self, buf, pkt_off, n, link_type, flags=0):
        """pcap2mgen's frame walk per record (mgenx_pcap_parse): returns a dict of device
        tensors udp_off, udp_len, src (n x 20), ttl, rx_sec, rx_usec, status."""
        torch = self.torch
        dev = buf.device
        o = {"udp_off": torch.empty(max(n, 1), dtype=torch.int64, device=dev),
             "udp_len": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
             "src": torch.empty(max(n, 1) * 20, dtype=torch.uint8, device=dev),
             "ttl": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
             "rx_sec": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
             "rx_usec": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
             "status": torch.empty(max(n, 1), dtype=torch.uint8, device=dev)}
        self._check(self.lib.mgenx_pcap_parse(self.ctx, _ptr(buf), buf.numel(), _ptr(pkt_off), n,
                                              link_type, flags, _ptr(o["udp_off"]),
                                              _ptr(o["udp_len"]), _ptr(o["src"]), _ptr(o["ttl"]),
                                              _ptr(o["rx_sec"]), _ptr(o["rx_usec"]),
                                              _ptr(o["status"]), _stream(self.device)),
                    "mgenx_pcap_parse")
        return o

    def pcap_snap(self, buf, file_bytes, pkt_off, n, flags, parsed):
        """mgenx_pcap_snap: move the SNAPPED packets of `parsed` (pcap_parse's dict) into
        buf[file_bytes:], zero-extended, in place."""
        self._check(self.lib.mgenx_pcap_snap(self.ctx, _ptr(buf), file_bytes, buf.numel(),
                                             _ptr(pkt_off), n, flags, _ptr(parsed["status"]),
                                             _ptr(parsed["udp_off"]), _ptr(parsed["udp_len"]),
                                             _stream(self.device)), "mgenx_pcap_snap")
        return parsed

    def flow_export(self, flows, n_flows, out=None):
        if out is None:
            out = self.torch.empty(n_flows * 64, dtype=self.torch.uint8, device=flows.device)
        self._check(self.lib.mgenx_flow_export(self.ctx, _ptr(flows), n_flows, _ptr(out),
                                               _stream(self.device)), "mgenx_flow_export")
        return out

    # ------------------------------------------------------------ MGEN_DATA items
    def report_build(self, reports, n_flows, per_flow, report_count, keys, sign, offset=None):
        """MgenAnalytic report_msg bytes for the kept reports (mgenx_report_build): returns
        (items uint8 [slots*52], lengths uint8 [slots]); sign (uint8 [n_flows]) updated."""
        torch = self.torch
        slots = n_flows * per_flow
        dev = report_count.device
        items = torch.zeros(max(slots, 1) * 52, dtype=torch.uint8, device=dev)
        ilen = torch.zeros(max(slots, 1), dtype=torch.uint8, device=dev)
        self._check(self.lib.mgenx_report_build(self.ctx, _ptr(reports), n_flows, per_flow,
                                                _ptr(report_count), _ptr(keys), _ptr(sign),
                                                _ptr(offset), _ptr(items), _ptr(ilen),
                                                _stream(self.device)), "mgenx_report_build")
        return items, ilen

    def _two_pass_text(self, call, n, dev, cap):
        torch = self.torch
        line_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        for _ in range(2):
            text = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
            self._check(call(text, cap, line_off), "report text")
            total = int(line_off[-1].cpu())
            if total <= cap:
                return text[:total], line_off
            cap = total
        raise MgenxError("report text did not fit")

    def log_send(self, tmpl, desc, n, *, src_port=None, out_len=None, msg_total=None,
                 slab=None, rec_off=None, stride=0, protocol=1, opts=0, binary=False,
                 cap=None):
        """SEND events of n packed records (mgenx_log_send_text / _binary): returns (bytes
        tensor, offsets tensor of n + 1)."""
        dev = desc.device
        cap = cap if cap is not None else max(1, n) * (200 if not binary else 160)
        if binary:
            call = lambda t, c, lo: self.lib.mgenx_log_send_binary(  # noqa: E731
                self.ctx, _ptr(tmpl), _ptr(desc), _ptr(out_len), _ptr(msg_total), _ptr(slab),
                slab.numel(), _ptr(rec_off), stride, n, protocol, _ptr(t), c, _ptr(lo),
                _stream(self.device))
        else:
            call = lambda t, c, lo: self.lib.mgenx_log_send_text(  # noqa: E731
                self.ctx, _ptr(tmpl), _ptr(desc), _ptr(src_port), _ptr(out_len),
                _ptr(msg_total), n, protocol, opts, _ptr(t), c, _ptr(lo), _stream(self.device))
        return self._two_pass_text(call, n, dev, cap)

    def log_report_text(self, items, reports, n_flows, per_flow, report_count, opts=0,
                        text_cap=None):
        n = n_flows * per_flow
        cap = text_cap if text_cap is not None else max(1, n) * 220
        return self._two_pass_text(
            lambda t, c, lo: self.lib.mgenx_log_report_text(
                self.ctx, _ptr(items), _ptr(reports), n_flows, per_flow, _ptr(report_count),
                opts, _ptr(t), c, _ptr(lo), _stream(self.device)), n, items.device, cap)

    def data_walk(self, slab, n, cols, *, rec_off=None, stride=0, opts=0, cmd_cap=4096,
                  rep_cap=4096):
        """ProcessRecvMessage over MGEN_DATA payloads (mgenx_data_walk): returns (status,
        needs_host, cmds [cap x 2 u32], reps [cap x 2 u64], totals [2])."""
        torch = self.torch
        dev = slab.device
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        nh = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        cmds = torch.zeros(max(cmd_cap, 1) * 2, dtype=torch.int32, device=dev)
        reps = torch.zeros(max(rep_cap, 1) * 2, dtype=torch.int64, device=dev)
        totals = torch.zeros(2, dtype=torch.int32, device=dev)
        cs = self._cols_struct(cols)
        self._check(self.lib.mgenx_data_walk(self.ctx, _ptr(slab), _ptr(rec_off), stride,
                                             ctypes.byref(cs), n, opts, _ptr(status), _ptr(nh),
                                             _ptr(cmds), cmd_cap, _ptr(reps), rep_cap,
                                             _ptr(totals), _stream(self.device)),
                    "mgenx_data_walk")
        return status[:n], nh[:n], cmds, reps, totals

    def log_report_recv_text(self, slab, reps, n_reps, src, rx_sec, rx_usec, opts=0,
                             text_cap=None):
        cap = text_cap if text_cap is not None else max(1, n_reps) * 300
        return self._two_pass_text(
            lambda t, c, lo: self.lib.mgenx_log_report_recv_text(
                self.ctx, _ptr(slab), _ptr(reps), n_reps, _ptr(src), _ptr(rx_sec),
                _ptr(rx_usec), opts, _ptr(t), c, _ptr(lo), _stream(self.device)),
            n_reps, slab.device, cap)

    # ------------------------------------------------------------ multi-GPU (RCCL)
    def comm_unique_id(self) -> bytes:
        """mgenx_comm_unique_id: the 128-byte id rank 0 hands to every rank."""
        buf = ctypes.create_string_buffer(128)
        self._check(self.lib.mgenx_comm_unique_id(buf), "mgenx_comm_unique_id")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        comm = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        self._check(self.lib.mgenx_comm_init(self.ctx, nranks, rank, buf, ctypes.byref(comm)),
                    "mgenx_comm_init")
        return comm

    def comm_destroy(self, comm):
        self.lib.mgenx_comm_destroy(comm)

    def allreduce_flows(self, comm, counters, n_flows):
        """In-place SUM of n_flows x 64-B mgenx_flow_counters over the ranks (RCCL)."""
        self._check(self.lib.mgenx_allreduce_flows(self.ctx, comm, _ptr(counters), n_flows,
                                                   _stream(self.device)), "mgenx_allreduce_flows")

    def allgather_u64(self, comm, src, dst, count):
        self._check(self.lib.mgenx_allgather_u64(self.ctx, comm, _ptr(src), _ptr(dst), count,
                                                 _stream(self.device)), "mgenx_allgather_u64")

    # ------------------------------------------------------------ FindFlow
    def flow_table(self, max_flows: int):
        t = ctypes.c_void_p()
        self._check(self.lib.mgenx_flow_table_create(self.ctx, max_flows, ctypes.byref(t)),
                    "mgenx_flow_table_create")
        return t

    def flow_table_destroy(self, t):
        self.lib.mgenx_flow_table_destroy(t)

    def flow_lookup(self, table, cols, src, n, flow_idx=None, n_flows=None):
        """Dense flow index per record (mgenx_flow_lookup); returns (flow_idx, n_flows)."""
        torch = self.torch
        dev = src.device
        if flow_idx is None:
            flow_idx = torch.empty(n, dtype=torch.int32, device=dev)
        if n_flows is None:
            n_flows = torch.zeros(1, dtype=torch.int32, device=dev)
        cs = self._cols_struct(cols)
        self._check(self.lib.mgenx_flow_lookup(self.ctx, table, ctypes.byref(cs), _ptr(src), n,
                                               _ptr(flow_idx), _ptr(n_flows),
                                               _stream(self.device)), "mgenx_flow_lookup")
        return flow_idx, n_flows

    def crc32(self, data, off, length, n, out=None):
        if out is None:
            out = self.torch.empty(n, dtype=self.torch.int32, device=data.device)
        rc = self.lib.mgenx_crc32_batch(self.ctx, _ptr(data), _ptr(off), _ptr(length), n,
                                        _ptr(out), _stream(self.device))
        self._check(rc, "mgenx_crc32_batch")
        return out


def pcap_index(buf) -> tuple:
    """mgenx_pcap_index over a host pcap image (bytes / numpy uint8): (record header offsets
    as uint64 numpy array, PcapInfo).  Host work only (the pcap_next loop)."""
    L = load()
    b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    info = PcapInfo()
    rc = L.mgenx_pcap_index(b.ctypes.data_as(ctypes.c_void_p), b.size, None, 0,
                            ctypes.byref(info))
    if rc != 0:
        raise MgenxError("mgenx_pcap_index: not a pcap file")
    offs = np.zeros(max(1, int(info.n_records)), np.uint64)
    rc = L.mgenx_pcap_index(b.ctypes.data_as(ctypes.c_void_p), b.size,
                            offs.ctypes.data_as(ctypes.c_void_p), offs.size, ctypes.byref(info))
    if rc != 0:
        raise MgenxError("mgenx_pcap_index failed")
    return offs[:int(info.n_records)], info


def binlog_index(buf) -> tuple:
    """mgenx_binlog_index over a host binary log image: (record offsets as uint64 numpy
    array, BinlogInfo).  Host work only."""
    L = load()
    b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    info = BinlogInfo()
    p = b.ctypes.data_as(ctypes.c_void_p)
    if L.mgenx_binlog_index(p, b.size, None, 0, ctypes.byref(info)) != 0:
        raise MgenxError("mgenx_binlog_index failed")
    offs = np.zeros(max(1, int(info.n_records)), np.uint64)
    if L.mgenx_binlog_index(p, b.size, offs.ctypes.data_as(ctypes.c_void_p), offs.size,
                            ctypes.byref(info)) != 0:
        raise MgenxError("mgenx_binlog_index failed")
    return offs[:int(info.n_records)], info


def convert_binary_log(log, log_rx=True, flush=False, opts=0, device=0) -> tuple:
    """ConvertBinaryLog of a host binary log image on the GPU: (text bytes, BinlogInfo)."""
    import torch
    offs, info = binlog_index(log)
    n = int(info.n_records)
    if n == 0:
        return b"", info
    eng = Engine(device)
    try:
        dev = f"cuda:{device}"
        buf = torch.from_numpy(np.frombuffer(bytes(log), np.uint8).copy()).to(dev)
        ro = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
        flags = (0 if log_rx else BINLOG_NO_RX) | (BINLOG_FLUSH if flush else 0)
        text, _ = eng.convert_binary_log(buf, ro, n, flags, opts)
        return text.cpu().numpy().tobytes(), info
    finally:
        eng.close()


def to_device(arr: np.ndarray, device=0):
    """Copy a numpy (structured) array to the GPU as raw bytes (uint8 tensor)."""
    import torch
    b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    return torch.from_numpy(b.copy()).to(f"cuda:{device}")


class Worker:
    """mgenx_worker: MgenMsg::Unpack / ComputeCRC32 of one host message per call, served by a
    wave resident on the device (no launch or copy per call)."""

    def __init__(self, eng: Engine, idle_ms: int = 200):
        self.eng = eng
        self.w = ctypes.c_void_p()
        eng._check(eng.lib.mgenx_worker_create(eng.ctx, idle_ms, ctypes.byref(self.w)),
                   "mgenx_worker_create")

    def unpack(self, msg: bytes):
        """One record's mgenx_unpacked (numpy structured scalar, UNPACKED_DTYPE)."""
        out = np.zeros(1, UNPACKED_DTYPE)
        self.eng._check(self.eng.lib.mgenx_worker_unpack(self.w, bytes(msg), len(msg),
                                                         ctypes.c_void_p(out.ctypes.data)),
                        "mgenx_worker_unpack")
        return out[0]

    def recv(self, msg: bytes, force: bool = False):
        """The receive path's Unpack + ComputeCRC32(0, msg, len - 4) in one call
        (mgenx_worker_recv): (mgenx_unpacked, crc state or None when no checksum was due)."""
        out = np.zeros(1, UNPACKED_DTYPE)
        crc, done = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.eng._check(self.eng.lib.mgenx_worker_recv(self.w, bytes(msg), len(msg), int(force),
                                                       ctypes.c_void_p(out.ctypes.data),
                                                       ctypes.byref(crc), ctypes.byref(done)),
                        "mgenx_worker_recv")
        return out[0], (crc.value if done.value else None)

    def flow_update(self, flows, slot, seq, rx_sec, rx_usec, msg_size, tx_sec, tx_usec):
        """MgenAnalytic::Update of one record on device flow state flows[slot]
        (mgenx_worker_flow_update): the closed window's report (FLOW_REPORT_DTYPE) or None."""
        rep = np.zeros(1, FLOW_REPORT_DTYPE)
        up = ctypes.c_uint32(0)
        self.eng._check(self.eng.lib.mgenx_worker_flow_update(
            self.w, _ptr(flows), slot, seq & 0xFFFFFFFF, rx_sec, rx_usec, msg_size, tx_sec,
            tx_usec, ctypes.byref(up), ctypes.c_void_p(rep.ctypes.data)), "mgenx_worker_flow_update")
        return rep[0] if up.value else None

    def device_mailbox(self) -> bool:
        """Whether requests go to device memory written through the BAR (mgenx_worker_info)."""
        f = ctypes.c_uint32(0)
        self.eng._check(self.eng.lib.mgenx_worker_info(self.w, ctypes.byref(f)), "mgenx_worker_info")
        return bool(f.value & 1)

    def crc32(self, data: bytes, state: int = 0) -> int:
        out = ctypes.c_uint32(0)
        self.eng._check(self.eng.lib.mgenx_worker_crc32(self.w, bytes(data), len(data), state,
                                                        ctypes.byref(out)),
                        "mgenx_worker_crc32")
        return out.value

    def pack(self, tmpl, payload: bytes, desc, buf_len: int, crc_in: int = 0, opts: int = 0,
             fill_time: int = 0):
        """MgenMsg::Pack of one message (mgenx_worker_pack): (bytes, tx_crc, state).  tmpl /
        desc: one-element TMPL_DTYPE / DESC_DTYPE arrays."""
        t = np.ascontiguousarray(tmpl)
        d = np.ascontiguousarray(desc)
        out = np.zeros(max(buf_len, 1), np.uint8)
        ret, tx, st = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.eng._check(self.eng.lib.mgenx_worker_pack(
            self.w, ctypes.c_void_p(t.ctypes.data), bytes(payload), ctypes.c_void_p(d.ctypes.data),
            buf_len, crc_in, opts, fill_time, ctypes.c_void_p(out.ctypes.data), ctypes.byref(ret),
            ctypes.byref(tx), ctypes.byref(st)), "mgenx_worker_pack")
        return out[:ret.value].tobytes(), tx.value, st.value

    def stop(self):
        """End the resident wave now (the next call relaunches it)."""
        if self.w:
            self.eng._check(self.eng.lib.mgenx_worker_stop(self.w), "mgenx_worker_stop")

    def close(self):
        # (after Engine.close the handle only frees itself: mgenx_ctx_destroy stopped the wave)
        if self.w:
            self.eng.lib.mgenx_worker_destroy(self.w)
            self.w = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
