"""GPU parity of the Pack-alone entry point and the incremental CRC (include/mgenx.h):

  * mgenx_pack_msgs = MgenMsg::Pack(buffer, bufferLen, includeChecksum, tx_checksum) on
    messages set up like MgenFlow::SendMessage, against the oracle's or_pack: return value,
    every byte of the buffer, tx_checksum after the call (from a zero or a running value),
    the flags member (CHECKSUM set, LAST_BUFFER cleared) and packet_header_len -- over dst
    IPv4/IPv6, host none/IPv4/IPv6, payload none/fits/too big, every truncation boundary,
    LAST_BUFFER on/off, zero and RANDOM_FILL, and the TCP fragment case where bufferLen
    (8192 / 8188) is shorter than the msg_len written into the header
    (mgenTransport.cpp:1915-1926);
  * mgenx_crc32_update = MgenMsg::ComputeCRC32(checksum, buf, len) incl. the restart from 0;
  * the Unpack field mask (mgenx_cols.decoded) against what Unpack assigns.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FILL_TIME = 1_700_000_123
SIZES = [20, 27, 28, 31, 32, 40, 44, 45, 47, 48, 52, 53, 60, 64, 76, 77, 100, 256, 1024]
PAYLOADS = [None, bytes(range(4)), bytes((i * 5 + 1) & 0xFF for i in range(60))]
DSTS = [("4", bytes([10, 1, 2, 3]), 5000), ("6", bytes(range(0x40, 0x50)), 5001)]
HOSTS = [None, ("4", bytes([192, 168, 0, 9]), 6000), ("6", bytes(range(0x60, 0x70)), 6001)]


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def eng(torch):
    from mgen_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def _cases():
    out = []
    k = 0
    for dst in DSTS:
        for host in HOSTS:
            for pay in PAYLOADS:
                for size in SIZES:
                    for last in (True, False):
                        k += 1
                        out.append(dict(dst=dst, host=host, payload=pay, msg_len=size,
                                        buf_len=size, flags=(0x08 if last else 0) |
                                        (0x04 if k % 5 == 0 else 0), crc_in=0 if k % 3 else
                                        (0x9E3779B9 * k) & 0xFFFFFFFF, seq=k, lat=12.5 + k,
                                        lon=-77.25 - k, alt=-999 + k, gps=k % 3))
    # TCP fragments: msg_len 16384 packed into 8192 / 8188 bytes, LAST_BUFFER off
    for j, bl in enumerate((8192, 8188, 8192, 8188)):
        out.append(dict(dst=DSTS[j % 2], host=HOSTS[j % 3], payload=PAYLOADS[j % 3],
                        msg_len=16384, buf_len=bl, flags=0, crc_in=0, seq=900 + j, lat=999.0,
                        lon=999.0, alt=-999, gps=0))
    return out


def _tmpl_desc(cases):
    from mgen_amd._abi import DESC_DTYPE, TMPL_DTYPE, gps_raw
    n = len(cases)
    tmpl = np.zeros(n, TMPL_DTYPE)
    desc = np.zeros(n, DESC_DTYPE)
    pool = bytearray()
    for i, c in enumerate(cases):
        t = tmpl[i]
        t["flow_id"] = 100 + i
        kind, raw, port = c["dst"]
        t["dst_type"], t["dst_len"], t["dst_port"] = (1 if kind == "4" else 2), len(raw), port
        t["dst_addr"][:len(raw)] = list(raw)
        if c["host"]:
            kind, raw, port = c["host"]
            t["host_type"], t["host_len"], t["host_port"] = (1 if kind == "4" else 2), len(raw), port
            t["host_addr"][:len(raw)] = list(raw)
        t["lat_raw"], t["lon_raw"] = gps_raw(c["lat"]), gps_raw(c["lon"])
        t["alt"], t["gps_status"] = c["alt"], c["gps"]
        if c["payload"] is not None:
            t["has_payload"], t["payload_len"], t["payload_off"] = 1, len(c["payload"]), len(pool)
            pool += c["payload"]
        desc[i] = (i, c["seq"], 1_700_000_000 + i, 1000 * i, c["msg_len"] & 0xFFFF, c["flags"], 0)
    return tmpl, desc, np.frombuffer(bytes(pool) or b"\0", np.uint8)


@pytest.mark.parametrize("checksum,rf", [(False, False), (True, False), (True, True)])
def test_pack_msgs_vs_oracle(torch, eng, oracle, checksum, rf):
    from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL, to_device
    cases = _cases()
    tmpl, desc, pool = _tmpl_desc(cases)
    n = len(cases)
    bl = np.array([c["buf_len"] for c in cases], np.uint32)
    offs = np.concatenate([[0], np.cumsum((bl + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    cin = np.array([c["crc_in"] for c in cases], np.uint32)
    slab = torch.zeros(int(offs[-1] + bl[-1] + 64), dtype=torch.uint8, device="cuda")
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    tcrc = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, n, d_pool, tcrc)
    if rf:
        eng.set_fill_time(FILL_TIME)
    opts = (PACK_CHECKSUM if checksum else 0) | (PACK_RANDOM_FILL if rf else 0)
    ln, tx, st = eng.pack_msgs(d_tmpl, tcrc, d_desc, n, d_pool, slab,
                               rec_off=to_device(offs).view(torch.int64),
                               buf_len=to_device(bl).view(torch.int32),
                               crc_in=to_device(cin).view(torch.int32), opts=opts,
                               fill_time=FILL_TIME if rf else 0)
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    ln = ln.cpu().numpy().view(np.uint32)
    tx = tx.cpu().numpy().view(np.uint32)
    st = st.cpu().numpy().view(np.uint32)
    n_fail = 0
    for i, c in enumerate(cases):
        m = oracle.make_msg(msg_len=c["msg_len"], flow_id=100 + i, seq=c["seq"],
                            tx_sec=1_700_000_000 + i, tx_usec=1000 * i, flags=c["flags"],
                            dst=c["dst"], host=c["host"], lat=c["lat"], lon=c["lon"],
                            alt=c["alt"], gps_status=c["gps"], payload=c["payload"])
        r, buf, ck, flags, hl = oracle.pack(m, c["buf_len"], checksum=checksum,
                                            tx_checksum=c["crc_in"], random_fill=rf,
                                            fill_time=FILL_TIME)
        assert ln[i] == r, (i, c, ln[i], r)
        assert tx[i] == ck, (i, c, hex(tx[i]), hex(ck))
        if r == 0:
            n_fail += 1
            continue
        o = int(offs[i])
        assert bytes(got[o:o + r]) == buf[:r], (i, c)
        assert (st[i] >> 16) & 0xFF == flags, (i, c, st[i] >> 16, flags)
        assert st[i] & 0xFFFF == hl, (i, c, st[i] & 0xFFFF, hl)
    assert 0 < n_fail < n // 4


def test_crc32_update_vs_reference_rule(torch, eng):
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 40000, dtype=np.uint8)
    lens = np.array([0, 1, 3, 4, 17, 64, 1000, 4096, 12000, 7], np.uint32)
    offs = np.array([0, 5, 9, 100, 333, 1000, 2000, 9000, 21000, 39000], np.uint64)
    state = np.array([0, 0, 0x12345678, 0, 0xFFFFFFFF, 1, 0, 0xDEADBEEF, 0, 0], np.uint32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()  # noqa: E731
    out = eng.crc32_update(t(data), t(offs).view(torch.int64), t(lens).view(torch.int32),
                           len(lens), t(state).view(torch.int32))
    torch.cuda.synchronize()
    out = out.cpu().numpy().view(np.uint32)
    for i in range(len(lens)):
        s0 = int(state[i]) or 0xFFFFFFFF   # ComputeCRC32 restarts from XINIT on 0
        seg = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        # zlib.crc32(seg, v) runs from state ~v and returns ~state
        want = zlib.crc32(seg, s0 ^ 0xFFFFFFFF) ^ 0xFFFFFFFF
        assert int(out[i]) == want, i


def test_decoded_mask_matches_unpack_stages(torch, eng):
    """mgenx_cols.decoded against the stages the golden fields reach (mgenMsg.cpp:315-500)."""
    import os
    from mgen_amd import (DEC_BASE, DEC_DST, DEC_GPS, DEC_HDRLEN, DEC_HOST, DEC_MSGLEN,
                          DEC_PLEN, DEC_PTYPE, OPT_SKIP_CRC)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = dict(np.load(os.path.join(root, "tests", "golden", "udp_matrix.npz"), allow_pickle=False))
    f = g["unpack_fields_udp"]
    n = len(f)
    slab = torch.from_numpy(g["unpack_slab"].copy()).cuda()
    offs = torch.from_numpy(g["unpack_offs"].astype(np.int64)).cuda()
    lens = torch.from_numpy(g["unpack_lens"].astype(np.int32)).cuda()
    cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, ext=True, opts=OPT_SKIP_CRC)
    torch.cuda.synchronize()
    dec = cols["decoded"].cpu().numpy()
    # the stages Unpack reaches, walked over the record bytes (mgenMsg.cpp:323-497)
    slab_h, offs_h, L = g["unpack_slab"], g["unpack_offs"], g["unpack_lens"]
    want = np.zeros(n, np.uint8)
    for i in range(n):
        r = slab_h[int(offs_h[i]):int(offs_h[i]) + int(L[i])]
        bl = int(L[i])
        if bl < 28:
            continue
        m = DEC_MSGLEN
        if r[2] != 2:
            want[i] = m
            continue
        m |= DEC_BASE
        if r[22] not in (1, 2):
            want[i] = m
            continue
        m |= DEC_DST | DEC_HDRLEN
        ln = 24 + int(r[23])
        if ln + 4 <= bl:
            ht, hlen = r[ln + 2], int(r[ln + 3])
            ln += 4
            if ln + hlen <= bl:
                if ht in (1, 2):
                    m |= DEC_HOST
                ln += hlen
                if ln + 13 <= bl:
                    m |= DEC_GPS
                    ln += 13
                    if ln + 1 <= bl:
                        m |= DEC_PTYPE
                        if ln + 3 <= bl:
                            m |= DEC_PLEN
        want[i] = m
    bad = np.nonzero(dec != want)[0]
    assert bad.size == 0, (bad[:8], dec[bad[:8]], want[bad[:8]])
    assert (want & DEC_PLEN).any() and (want == DEC_MSGLEN).any() and not want.all()


@pytest.mark.parametrize("checksum,rf", [(False, False), (True, False), (True, True)])
def test_worker_pack_vs_oracle(torch, eng, oracle, checksum, rf):
    """The resident worker's single-message Pack (mgenx_worker_pack: what the shim's
    MgenMsg::Pack calls for one message) over the same matrix, against the oracle's or_pack:
    return value, every byte, tx_checksum, flags and packet_header_len."""
    from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL
    cases = _cases()
    tmpl, desc, pool = _tmpl_desc(cases)
    opts = (PACK_CHECKSUM if checksum else 0) | (PACK_RANDOM_FILL if rf else 0)
    w = eng.worker()
    try:
        for i, c in enumerate(cases):
            t = tmpl[i:i + 1].copy()
            po, pl = int(t["payload_off"][0]), int(t["payload_len"][0])
            payload = pool[po:po + pl].tobytes() if t["has_payload"][0] else b""
            b, tx, st = w.pack(t, payload, desc[i:i + 1], c["buf_len"], c["crc_in"], opts,
                               FILL_TIME if rf else 0)
            m = oracle.make_msg(msg_len=c["msg_len"], flow_id=100 + i, seq=c["seq"],
                                tx_sec=1_700_000_000 + i, tx_usec=1000 * i, flags=c["flags"],
                                dst=c["dst"], host=c["host"], lat=c["lat"], lon=c["lon"],
                                alt=c["alt"], gps_status=c["gps"], payload=c["payload"])
            r, buf, ck, flags, hl = oracle.pack(m, c["buf_len"], checksum=checksum,
                                                tx_checksum=c["crc_in"], random_fill=rf,
                                                fill_time=FILL_TIME)
            assert len(b) == r and tx == ck, (i, c, len(b), r, hex(tx), hex(ck))
            if r:
                assert b == buf[:r], (i, c)
                assert (st >> 16) & 0xFF == flags and st & 0xFFFF == hl, (i, c, hex(st))
    finally:
        w.close()
