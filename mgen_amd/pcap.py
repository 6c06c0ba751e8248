"""pcap2mgen on the GPU: a capture file -> the MGEN text log (src/common/pcap2mgen.cpp:252-482).

The reference walks the capture one packet at a time: pcap_next, an Ethernet / IP / UDP parse,
``MgenMsg::Unpack`` (no CRC check), then with ``analytic`` ``FindFlow`` + ``Update`` (logging
the analytic's REPORT line when a window closes), ``LogRecvEvent`` (the RECV line, GMT
timestamps, GPS, TTL, no data), and the REPORT lines of any reports the payload carries.
Here the whole file goes to HBM once and every stage is one batch call of the C ABI:

  mgenx_pcap_index (host: the record-header chain) -> mgenx_pcap_parse -> mgenx_unpack_batch
  (MGENX_OPT_SKIP_CRC: Unpack alone) -> [mgenx_flow_lookup -> mgenx_flow_reduce_ex ->
  mgenx_flow_keys -> mgenx_report_build -> mgenx_log_report_text] -> mgenx_log_recv_text
  (MGENX_LOG_SKIP_ERR) -> mgenx_data_walk + mgenx_log_report_recv_text ->
  mgenx_text_interleave (per packet: analytic REPORT, RECV, received REPORTs).

Options mirror the reference's command line (``-analytic``/``-report``, ``+rxlog on|off``,
``+window``); ``trace`` (MAC addresses in front of each line) is not supported.
"""
from __future__ import annotations

import numpy as np

from . import (DATA_CONTROLLER, FLOW_REPORT_DTYPE, LOG_EPOCH, LOG_NO_DATA, LOG_SKIP_ERR,
               OPT_SKIP_CRC, TEXT_OWNER, TEXT_PER_RECORD, TEXT_SCATTER, Engine, MgenxError,
               pcap_index)


def _quantized_window(window: float) -> float:
    """Report::QuantizeTimeValue / UnquantizeTimeValue (mgenAnalytic.cpp:621-642)."""
    import math
    stretch, tmin, tmax = 1.1, 1.0e-06, 600.0
    scale = 1.0 / (math.pow(stretch, 254) - stretch)
    if window > stretch * tmax:
        q = 0xFF
    elif window < tmin / 2.0:
        q = 0
    elif window < tmin:
        q = 1
    else:
        q = int((math.log(stretch + (window - tmin) / (scale * (tmax - tmin))) / math.log(stretch))
                + 0.5) & 0xFF
    return 0.0 if q == 0 else (tmax - tmin) * (math.pow(stretch, q) - stretch) * scale + tmin


class Pcap2Mgen:
    """pcap2mgen with its options; ``run(file)`` returns the log bytes.  Everything after the
    host index walk runs on the engine's GPU."""

    FIRST_FLOWS = 65536  # flow-table capacity tried first (see run_device)

    def __init__(self, engine: Engine, analytics: bool = False, log_rx: bool = True,
                 window: float = 1.0, epoch: bool = False):
        self.eng = engine
        self.analytics = analytics
        self.log_rx = log_rx
        self.window = window
        self.opts = LOG_EPOCH if epoch else 0

    def upload(self, file):
        """Host index walk + one H2D copy: (device file, device record offsets, PcapInfo)."""
        torch = self.eng.torch
        b = np.frombuffer(bytes(file), np.uint8) if not isinstance(file, np.ndarray) else file
        offs, info = pcap_index(b)
        dev = f"cuda:{self.eng.device}"
        # the file image, then scratch for packets cut by the snapshot length (mgenx_pcap_snap)
        buf = torch.zeros(b.size + int(info.snap_bytes), dtype=torch.uint8, device=dev)
        buf[:b.size] = torch.from_numpy(b.copy()).to(dev)
        pkt_off = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
        return buf, pkt_off, info

    def run(self, file) -> bytes:
        buf, pkt_off, info = self.upload(file)
        file_bytes = buf.numel() - int(info.snap_bytes)
        text, _ = self.run_device(buf, pkt_off, int(info.n_records), info.link_type, info.flags,
                                  file_bytes=file_bytes)
        return text.cpu().numpy().tobytes()

    def run_device(self, buf, pkt_off, n, link_type, flags, file_bytes=None):
        """The device pipeline over a resident file: (text tensor, per-packet offsets).
        file_bytes: the file image's size when buf has scratch after it for snapped packets
        (None: no scratch; packets cut by the snapshot length are skipped)."""
        eng, torch = self.eng, self.eng.torch
        dev = buf.device
        if n == 0:
            return torch.empty(0, dtype=torch.uint8, device=dev), torch.zeros(
                1, dtype=torch.int64, device=dev)
        p = eng.pcap_parse(buf, pkt_off, n, link_type, flags)
        if file_bytes is not None and file_bytes < buf.numel():
            eng.pcap_snap(buf, file_bytes, pkt_off, n, flags, p)
        cols = eng.unpack(buf, n, rec_off=p["udp_off"], rec_len=p["udp_len"], opts=OPT_SKIP_CRC,
                          ext=True)
        sources = []
        keep = []
        if self.analytics:
            # a table for up to FIRST_FLOWS flows first (a table for n flows is 64 x 2n bytes to
            # allocate, clear and free on every run); if it overflowed -- a record of a good
            # message left without a flow -- the lookup is redone on a table for n flows
            cap_flows = min(max(n, 1), self.FIRST_FLOWS)
            table = eng.flow_table(cap_flows)
            try:
                flow_idx, nfl = eng.flow_lookup(table, cols, p["src"], n)
                if cap_flows < n:
                    lost = ((flow_idx[:n] < 0) & (cols["err"][:n] == 0)).any()
                    st = torch.stack([nfl[0].to(torch.int64), lost.to(torch.int64)]).cpu()
                    n_flows, overflow = int(st[0]), bool(st[1])
                else:
                    n_flows, overflow = int(nfl.item()), False
                if overflow:
                    eng.flow_table_destroy(table)
                    table = None    # a failing create below must not free it again
                    table = eng.flow_table(max(n, 1))
                    flow_idx, nfl = eng.flow_lookup(table, cols, p["src"], n)
                    n_flows = int(nfl.item())
                if n_flows:
                    per_flow = self._per_flow(p, flow_idx, n, n_flows)
                    flows = eng.flow_init(n_flows, self.window)
                    reports = torch.zeros(n_flows * per_flow * FLOW_REPORT_DTYPE.itemsize,
                                          dtype=torch.uint8, device=dev)
                    count = torch.zeros(n_flows, dtype=torch.int32, device=dev)
                    rep_rec = torch.full((n_flows * per_flow,), -1, dtype=torch.int32,
                                         device=dev)
                    eng.flow_reduce(flows, n_flows, flow_idx, cols["seq_num"], cols["tx_sec"],
                                    cols["tx_usec"], cols["msg_len"], p["rx_sec"], p["rx_usec"],
                                    n=n, reports=reports, per_flow=per_flow, report_count=count,
                                    report_rec=rep_rec)
                    keys = eng.flow_keys(table, n_flows, protocol=1)
                    sign = torch.zeros(n_flows, dtype=torch.uint8, device=dev)
                    items, _ = eng.report_build(reports, n_flows, per_flow, count, keys, sign)
                    rtext, rline = eng.log_report_text(items, reports, n_flows, per_flow, count,
                                                       opts=self.opts)
                    sources.append((TEXT_SCATTER, rtext, rline, n_flows * per_flow, rep_rec, 1))
                    keep += [reports, count, rep_rec, items]
            finally:
                if table is not None:
                    eng.flow_table_destroy(table)
        if self.log_rx:  # LogRecvEvent(..., logData false, logGpsData true, ttl, hdr.ts)
            text, line_off = eng.log_recv_text(buf, n, cols, p["src"], p["rx_sec"],
                                               p["rx_usec"], rec_off=p["udp_off"], ttl=p["ttl"],
                                               protocol=1,
                                               opts=self.opts | LOG_NO_DATA | LOG_SKIP_ERR)
            sources.append((TEXT_PER_RECORD, text, line_off, n, None, 1))
        # the REPORT items of MGEN_DATA payloads (LogRecvEvent, mgenMsg.cpp:1104-1137)
        cap = 1024
        for _ in range(2):
            _, _, _, reps, totals = eng.data_walk(buf, n, cols, rec_off=p["udp_off"],
                                                  opts=DATA_CONTROLLER, cmd_cap=1, rep_cap=cap)
            n_reps = int(totals[1].item())
            if n_reps <= cap:
                break
            cap = n_reps
        if n_reps:
            rr_text, rr_line = eng.log_report_recv_text(buf, reps, n_reps, p["src"], p["rx_sec"],
                                                        p["rx_usec"], opts=self.opts)
            sources.append((TEXT_OWNER, rr_text, rr_line, n_reps, reps.view(torch.int32), 4))
        if not sources:
            return torch.empty(0, dtype=torch.uint8, device=dev), torch.zeros(
                n + 1, dtype=torch.int64, device=dev)
        return eng.text_interleave(sources, n)

    def _per_flow(self, p, flow_idx, n, n_flows) -> int:
        """Report slots per flow: a window closes at most once per record and at most once
        per window length of capture time (the window restarts at the closing record).  The
        counts and the time range are reduced on the device (mgenx_flow_span, one read-back)."""
        most, lo, hi = self.eng.flow_span(flow_idx, p["rx_sec"], p["rx_usec"], n, n_flows)
        if most == 0:
            return 1
        span = float(hi - lo) * 1e-6
        w = _quantized_window(self.window)
        by_time = most if w <= 0.0 else int(span / w) + 2
        return max(1, min(most, by_time))


def pcap2mgen(file, analytics=False, log_rx=True, window=1.0, epoch=False, device=0) -> bytes:
    """One-shot helper: the log text of a pcap file image."""
    eng = Engine(device)
    try:
        return Pcap2Mgen(eng, analytics, log_rx, window, epoch).run(file)
    finally:
        eng.close()


__all__ = ["Pcap2Mgen", "pcap2mgen", "MgenxError"]
