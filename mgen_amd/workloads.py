"""Synthetic MGEN batches for the BASELINE.json configurations.

These build the *inputs* of the pack path (per-flow templates + per-record descriptors),
the way MgenFlow::SendMessage fills an MgenMsg (src/common/mgenFlow.cpp:946-983): dst
127.0.0.1/5000, GPS 999/999/-999 INVALID, optional DATA payload, per-flow sequence
numbers, microsecond tx timestamps.  Seed base 0x4D47454E ("MGEN").
"""
from __future__ import annotations

import numpy as np

from ._abi import DESC_DTYPE, TMPL_DTYPE, gps_raw

SEED = 0x4D47454E
T0 = 1_700_000_000


def make_templates(n_flows: int, *, dst=(127, 0, 0, 1), dst_port=5000, payload: bytes = b"",
                   host=None, ipv6=False):
    """One template per flow (flow ids 1..n_flows).  Returns (tmpl, pool)."""
    t = np.zeros(n_flows, TMPL_DTYPE)
    t["flow_id"] = np.arange(1, n_flows + 1, dtype=np.uint32)
    if ipv6:
        t["dst_type"], t["dst_len"] = 2, 16
        a = np.zeros(16, np.uint8)
        a[15] = 1
        t["dst_addr"][:] = a
    else:
        t["dst_type"], t["dst_len"] = 1, 4
        t["dst_addr"][:, :4] = np.array(dst, np.uint8)
    t["dst_port"] = dst_port
    if host is not None:
        kind, raw, port = host
        t["host_type"] = 1 if kind == "4" else 2
        t["host_len"] = len(raw)
        t["host_addr"][:, :len(raw)] = np.frombuffer(bytes(raw), np.uint8)
        t["host_port"] = port
    t["lat_raw"] = gps_raw(999.0)
    t["lon_raw"] = gps_raw(999.0)
    t["alt"] = -999
    t["gps_status"] = 0
    pool = np.frombuffer(bytes(payload) if payload else b"\0", np.uint8).copy()
    if payload:
        t["has_payload"] = 1
        t["payload_len"] = len(payload)
        t["payload_off"] = 0
    return t, pool


def udp_fixed(n: int, size: int = 1024, n_flows: int = 64):
    """Config 2: n records of `size` bytes, flow = 1 + (i mod n_flows), per-flow seq
    0,1,2..., tx = T0 s + i us, dst 127.0.0.1/5000, no payload, zero fill."""
    tmpl, pool = make_templates(n_flows)
    i = np.arange(n, dtype=np.uint64)
    d = np.zeros(n, DESC_DTYPE)
    d["tmpl"] = (i % n_flows).astype(np.uint32)
    d["seq_num"] = (i // n_flows).astype(np.uint32)
    t_us = i + 0
    d["tx_sec"] = (T0 + t_us // 1_000_000).astype(np.uint32)
    d["tx_usec"] = (t_us % 1_000_000).astype(np.uint32)
    d["msg_len"] = size
    return tmpl, pool, d


def udp_mixed(n: int, lo: int = 64, hi: int = 1472, n_flows: int = 64, payload_hex="",
              seed=SEED):
    """Config 3: flow = i mod n_flows, size ~ U{lo..hi}, per-flow DATA payload.
    Returns (tmpl, pool, desc, offsets, sizes) with offsets = exclusive prefix sum."""
    from ._abi import hex_payload
    payload = hex_payload(payload_hex) if payload_hex else b""
    tmpl, pool = make_templates(n_flows, payload=payload)
    rng = np.random.default_rng(seed)
    sizes = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    i = np.arange(n, dtype=np.uint64)
    d = np.zeros(n, DESC_DTYPE)
    d["tmpl"] = (i % n_flows).astype(np.uint32)
    d["seq_num"] = (i // n_flows).astype(np.uint32)
    d["tx_sec"] = (T0 + i // 1_000_000).astype(np.uint32)
    d["tx_usec"] = (i % 1_000_000).astype(np.uint32)
    d["msg_len"] = sizes.astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    return tmpl, pool, d, offs, sizes.astype(np.uint32)


def poisson_flows(n, n_flows=1024, seed=SEED, loss=0.01, dup=0.001, reorder=8,
                  mean_gap_us=1000, msg_len=256, t0=1_700_000_000):
    """BASELINE config 4 shape: n_flows flows (ids 1..n_flows), per-flow tx interarrival
    Exp(mean_gap_us) (MgenPattern POISSON, mgenPattern.h:73-77), rx = tx + U[50, 500] us,
    `loss` of the sends dropped, `dup` duplicated, and records reordered within +-`reorder`
    positions of the global receive order.  Returns dict of columns in receive order
    (about n records)."""
    rng = np.random.default_rng(seed)
    per = max(1, int(n / n_flows / (1 - loss + dup)) + 1)
    flow = np.repeat(np.arange(1, n_flows + 1, dtype=np.uint32), per)
    seq = np.tile(np.arange(per, dtype=np.uint32), n_flows)
    gaps = rng.exponential(mean_gap_us, (n_flows, per))
    tx_us = (np.cumsum(gaps, axis=1) + rng.uniform(0, 1e6, (n_flows, 1))).reshape(-1)
    keep = rng.random(flow.size) >= loss
    d = rng.random(flow.size) < dup
    idx = np.concatenate([np.nonzero(keep)[0], np.nonzero(keep & d)[0]])
    tx_us = tx_us[idx]
    rx_us = tx_us + rng.uniform(50, 500, idx.size)
    order = np.argsort(rx_us, kind="stable")
    if reorder:
        jitter = order.astype(np.float64) * 0 + rng.uniform(-reorder, reorder, order.size)
        order = order[np.argsort(np.arange(order.size) + jitter, kind="stable")]
    idx, tx_us, rx_us = idx[order][:n], tx_us[order][:n], rx_us[order][:n]
    tx_i = (t0 * 10**6 + tx_us.astype(np.int64))
    rx_i = (t0 * 10**6 + rx_us.astype(np.int64))
    return {
        "flow_id": flow[idx], "seq": seq[idx],
        "tx_sec": (tx_i // 10**6).astype(np.uint32), "tx_usec": (tx_i % 10**6).astype(np.uint32),
        "rx_sec": (rx_i // 10**6).astype(np.uint32), "rx_usec": (rx_i % 10**6).astype(np.uint32),
        "msg_len": np.full(idx.size, msg_len, np.uint16),
    }


def pcap_capture(eng, n: int, msg_len: int = 262, n_flows: int = 1024, gap_us: int = 1):
    """A pcap capture image built on the device (Ethernet / IPv4 / UDP around GPU-packed
    checksummed MGEN messages): flow f = i mod n_flows from 10.0.f>>8.f&255 port 30000 + f,
    packet i captured at T0 + i * gap_us, tx 300 us earlier.  Returns (file uint8 tensor,
    record-header offsets int64 tensor, record bytes)."""
    import torch
    from . import PACK_CHECKSUM, to_device
    dev = f"cuda:{eng.device}"
    tmpl, pool, d = udp_fixed(n, msg_len, n_flows)
    t_us = np.arange(n, dtype=np.uint64) * gap_us
    d["tx_sec"] = (T0 + (t_us + 10**6 - 300) // 10**6 - 1).astype(np.uint32)
    d["tx_usec"] = ((t_us + 10**6 - 300) % 10**6).astype(np.uint32)
    d["flags"] = 0
    dt, dp = to_device(tmpl, eng.device), to_device(pool, eng.device)
    crc = torch.empty(n_flows, dtype=torch.int32, device=dev)
    eng.pack_prepare(dt, n_flows, dp, crc)
    slab = torch.empty(n * msg_len, dtype=torch.uint8, device=dev)
    eng.pack(dt, crc, to_device(d, eng.device), n, dp, slab, stride=msg_len, opts=PACK_CHECKSUM)
    R = 16 + 14 + 20 + 8 + msg_len
    assert R % 4 == 0
    h = bytearray(58)
    h[8:12] = (R - 16).to_bytes(4, "little")
    h[12:16] = (R - 16).to_bytes(4, "little")
    h[16:22] = bytes([2, 0, 0, 0, 0, 2])
    h[22:28] = bytes([2, 0, 0, 0, 0, 1])
    h[28:30] = b"\x08\x00"
    ip = 16 + 14
    h[ip:ip + 12] = bytes([0x45, 0, (20 + 8 + msg_len) >> 8, (20 + 8 + msg_len) & 255, 0, 0, 0x40,
                           0, 64, 17, 0, 0])
    h[ip + 12:ip + 16] = bytes([10, 0, 0, 0])
    h[ip + 16:ip + 20] = bytes([127, 0, 0, 1])
    u = ip + 20
    h[u + 2:u + 4] = (5000).to_bytes(2, "big")
    h[u + 4:u + 6] = (8 + msg_len).to_bytes(2, "big")
    cap = torch.empty(n, R, dtype=torch.uint8, device=dev)
    cap[:, :58] = torch.tensor(list(h), dtype=torch.uint8, device=dev)
    cap[:, 58:] = slab.view(n, msg_len)
    i = torch.arange(n, dtype=torch.int64, device=dev)
    f = i % n_flows
    t = T0 * 10**6 + i * gap_us
    w = cap.view(torch.int32)
    w[:, 0] = (t // 10**6).to(torch.int32)
    w[:, 1] = (t % 10**6).to(torch.int32)
    cap[:, ip + 14] = (f >> 8).to(torch.uint8)
    cap[:, ip + 15] = (f & 255).to(torch.uint8)
    sp = 30000 + f
    cap[:, u] = (sp >> 8).to(torch.uint8)
    cap[:, u + 1] = (sp & 255).to(torch.uint8)
    gh = torch.tensor(list((0xA1B2C3D4).to_bytes(4, "little") + (2).to_bytes(2, "little") +
                           (4).to_bytes(2, "little") + bytes(8) + (65535).to_bytes(4, "little") +
                           (1).to_bytes(4, "little")), dtype=torch.uint8, device=dev)
    file = torch.cat([gh, cap.view(-1)])
    return file, 24 + i * R, R
