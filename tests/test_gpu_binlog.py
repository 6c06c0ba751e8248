"""GPU parity of ConvertBinaryLog (mgenMsg.cpp:1417-1900): mgenx_convert_binary_log over
mixed binary logs -- RECV records of the golden matrix (IPv4 / IPv6 sources, every protocol,
MGEN_DATA reports), SEND records (UDP / SINK), every other event type -- against the oracle's
sequential restatement, byte for byte, with log_rx / log_flush / epoch / data / GPS options,
and logs that stop early (RERR, unknown types, short records)."""
import numpy as np
import pytest

import binlog_util as B

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def _diff(got: bytes, want: bytes):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    for k, (a, b) in enumerate(zip(gl, wl)):
        if a != b:
            return f"line {k}:\n got  {a!r}\n want {b!r}"
    return f"line counts {len(gl)} vs {len(wl)}"


@pytest.fixture(scope="module")
def mixed(oracle):
    rng = np.random.default_rng(12)
    parts = (B.recv_records(oracle, n=1500) + B.send_records(oracle, n=300) + B.events(rng) +
             B.data_recv_records(oracle, n=80))
    order = rng.permutation(len(parts))
    return B.binlog([parts[i] for i in order])


@pytest.mark.parametrize("log_rx,flush,opts", [(True, False, 0), (True, True, 0x1),
                                                (False, False, 0), (True, False, 0x2 | 0x4)])
def test_convert_matches_oracle(torch, oracle, mixed, log_rx, flush, opts):
    import mgen_amd
    want, st, n = oracle.convert_binary_log(mixed, log_rx=log_rx, flush=flush, opts=opts)
    got, info = mgen_amd.convert_binary_log(mixed, log_rx=log_rx, flush=flush, opts=opts)
    assert st == info.status == 0 and n == info.n_records
    assert want.count(b" REPORT ") > 0 and want.count(b" SEND ") > 0
    assert got == want, _diff(got, want)


def test_convert_stops_like_the_reference(torch, oracle):
    import struct
    import mgen_amd
    rng = np.random.default_rng(3)
    parts = B.recv_records(oracle, n=50) + B.events(rng)
    for bad in [struct.pack(">BBH", 2, 0, 20) + bytes(20), B.ev_time(99, 1, 1)]:
        log = B.binlog(parts + [bad] + parts)
        want, st, n = oracle.convert_binary_log(log)
        got, info = mgen_amd.convert_binary_log(log)
        assert st == info.status == 3 and n == info.n_records == len(parts)
        assert got == want
    log = B.binlog(parts)[:-5]
    want, st, _ = oracle.convert_binary_log(log)
    got, info = mgen_amd.convert_binary_log(log)
    assert st == info.status == 4 and got == want


def test_convert_gpu_written_binary_log(torch, oracle):
    """Binary RECV records written on the GPU (mgenx_log_recv_binary) after a header line
    convert back to the direct text log of the same records (with the converter's ttl)."""
    import mgen_amd
    from mgen_amd import Engine, to_device
    from streams import golden
    gold = golden()
    eng = Engine(0)
    try:
        f = gold["unpack_fields_udp"]
        # records whose stored hdr + payload bytes hold a whole header (>= 28 bytes): a
        # shorter stored message fails Unpack in the converter, which then logs a fresh
        # MgenMsg's fields (test_convert_logs_rejected_stored_messages)
        keep = (f["err"] == 0) & (f["hdr_len"].astype(int) + f["payload_len"] >= 28)
        idx = np.nonzero(keep)[0][:2000]
        slab = to_device(gold["unpack_slab"]).view(torch.uint8)
        offs = to_device(gold["unpack_offs"][idx]).view(torch.int64)
        lens = to_device(gold["unpack_lens"][idx]).view(torch.int32)
        n = len(idx)
        cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, ext=True)
        src = np.zeros(n, mgen_amd.ADDR_DTYPE)
        src["type"], src["len"], src["port"] = 1, 4, 4321
        src["addr"][:, :4] = [192, 168, 1, 7]
        rx_s = np.full(n, 1_700_000_123, np.uint32)
        rx_u = np.arange(n, dtype=np.uint32) * 7
        ds, dsec, dusec = to_device(src.view(np.uint8)), to_device(rx_s), to_device(rx_u)
        binrec, _ = eng.log_recv_binary(slab, n, cols, ds, dsec, dusec, rec_off=offs)
        text, _ = eng.log_recv_text(slab, n, cols, ds, dsec, dusec, rec_off=offs,
                                    ttl=to_device(np.zeros(n, np.int32)))
        log = B.HEADER + binrec.cpu().numpy().tobytes()
        got, info = mgen_amd.convert_binary_log(log)
        assert info.status == 0 and info.n_records == n
        direct = text.cpu().numpy().tobytes()
        # the direct log has no REPORT walk lines; keep the RECV lines of the conversion
        conv_recv = b"".join(l + b"\n" for l in got.split(b"\n")[:-1] if b" RECV " in l)
        assert conv_recv == direct, _diff(conv_recv, direct)
    finally:
        eng.close()


def test_convert_stops_at_records_short_for_their_type(torch, oracle):
    """A truncated final RECV / JOIN / ON record (recordLength too small for the fields its
    type reads) ends the conversion as a short read; nothing is read past the record."""
    import mgen_amd
    from test_binlog_cpu import short_for_type_cases
    rng = np.random.default_rng(4)
    parts = B.recv_records(oracle, n=40) + B.events(rng)
    for label, bad in short_for_type_cases():
        log = B.binlog(parts + [bad])
        want, st, n = oracle.convert_binary_log(log)
        got, info = mgen_amd.convert_binary_log(log)
        assert st == info.status == 4 and n == info.n_records == len(parts), label
        assert got == want, label


def test_convert_logs_rejected_stored_messages(torch, oracle):
    """RECV records whose stored message is shorter than a header (hdr + payload < 28: the
    converter's Unpack rejects it) are logged anyway, from a fresh MgenMsg's members with the
    event time as tx time (mgenMsg.cpp:1601-1607), as are SEND records whose stored message
    fails (:1612-1625).  Device == oracle, byte for byte."""
    import struct
    import mgen_amd
    from streams import golden
    gold = golden()
    f = gold["unpack_fields_udp"]
    short = np.nonzero((f["err"] == 0) & (f["hdr_len"].astype(int) + f["payload_len"] < 28))[0]
    assert short.size > 5
    src = np.zeros(short.size, mgen_amd.ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 4321
    src["addr"][:, :4] = [192, 168, 1, 7]
    rx_s = np.full(short.size, 1_700_000_123, np.uint32)
    rx_u = np.arange(short.size, dtype=np.uint32) * 11
    recs = oracle.log_recv_binary(f[short], gold["unpack_slab"], gold["unpack_offs"][short], src,
                                  rx_s, rx_u, protocol=1)
    # SEND records (UDP and TCP) whose message has a bad version / dst type / is 12 bytes
    sends = b""
    for proto, body in ((1, bytes([0, 64, 3]) + bytes(61)), (2, struct.pack(">I", 9000) +
                        bytes([0, 64, 2, 4]) + bytes(16) + bytes([0, 0, 9, 4]) + bytes(40)),
                        (3, bytes(12))):
        sends += struct.pack(">BBH", 3, proto, len(body)) + body
    rng = np.random.default_rng(9)
    log = B.binlog([recs, sends] + B.events(rng))
    want, st, n = oracle.convert_binary_log(log)
    got, info = mgen_amd.convert_binary_log(log)
    assert st == info.status == 0 and n == info.n_records
    assert want.count(b" RECV ") == short.size and want.count(b" SEND ") == 3
    assert got == want, _diff(got, want)


def test_convert_tcp_send_bounded_at_the_record(torch, oracle):
    """A TCP SEND record's stored message is Unpack-ed over the bytes the record holds.  The
    reference passes recordLength (mgenMsg.cpp:1624), 4 bytes more than follow the
    mgen_msg_len word, and those come from its uninitialised / stale read buffer (:1434): the
    choice pinned here is the record bound.  Messages cut right after the destination address,
    inside the host fields and inside the GPS fields: no host> field is read past the record,
    device == oracle byte for byte."""
    import struct
    import mgen_amd
    m = oracle.make_msg(msg_len=300, flow_id=5, seq=77, tx_sec=1_700_000_000, tx_usec=5,
                        host=("4", bytes([10, 1, 2, 3]), 6000))
    full = oracle.udp_pack(m, checksum=False)
    hdr_end = 28  # msg_len .. dst address (IPv4)
    parts = []
    for cut in (hdr_end, hdr_end + 2, hdr_end + 4, hdr_end + 8, hdr_end + 12, 60, len(full)):
        body = struct.pack(">I", 300) + full[:cut]
        parts.append(struct.pack(">BBH", 3, 2, len(body)) + body)
    log = B.binlog(parts + B.events(np.random.default_rng(2)))
    want, st, n = oracle.convert_binary_log(log)
    got, info = mgen_amd.convert_binary_log(log)
    assert st == info.status == 0 and n == info.n_records
    lines = [l for l in want.split(b"\n") if b" SEND " in l]
    assert len(lines) == 7
    assert b"host>" not in lines[0] and b"host>10.1.2.3/6000" in lines[-1], lines
    assert got == want, _diff(got, want)
