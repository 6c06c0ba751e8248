"""GPU parity of mgenx_log_recv_text (MgenMsg::LogRecvEvent / LogRecvError text lines)
against the oracle restatement, which itself reproduces the reference's printed output
(tests/test_log_cpu.py).  Inputs: the golden unpack matrix decoded on the GPU (every error
class, truncated headers, IPv4/IPv6 dst and host, GPS values, payloads), with varied source
addresses, receive times and TTLs; byte-exact, every option combination."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = "tests/golden/udp_matrix.npz"


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


@pytest.fixture(scope="module")
def gold():
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return dict(np.load(os.path.join(root, GOLD), allow_pickle=False))


def _sources(oracle, n, rng):
    src = np.zeros(n, oracle.ADDR_DTYPE)
    v6 = rng.random(n) < 0.3
    src["type"] = np.where(v6, 2, 1)
    src["len"] = np.where(v6, 16, 4)
    src["port"] = rng.integers(0, 65536, n)
    src["addr"] = rng.integers(0, 256, (n, 16))
    # IPv6 shapes inet_ntop treats specially: zero runs, ::1, IPv4-mapped / -compatible
    k = np.nonzero(v6)[0]
    for j, i in enumerate(k):
        a = src["addr"][i]
        kind = j % 6
        if kind == 0:
            a[:] = 0; a[15] = 1                               # ::1
        elif kind == 1:
            a[:10] = 0; a[10:12] = 0xFF                        # ::ffff:a.b.c.d
        elif kind == 2:
            a[:12] = 0                                        # ::a.b.c.d
        elif kind == 3:
            a[2:8] = 0                                        # x::y
        elif kind == 4:
            a[4:6] = 0; a[10:14] = 0                          # two runs
        src["addr"][i] = a
    return src


@pytest.mark.parametrize("mode,opts,proto", [("udp", 0, 1), ("udp_force", 0x1, 1),
                                             ("tcp_force", 0x6, 2), ("udp", 0x7, 3)])
def test_log_lines_match_oracle(torch, eng, gold, oracle, mode, opts, proto):
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP, to_device
    uopts = {"udp": 0, "udp_force": OPT_CHECKSUM_FORCE, "tcp_force": OPT_TCP | OPT_CHECKSUM_FORCE}
    n = len(gold["unpack_lens"])
    slab = to_device(gold["unpack_slab"]).view(torch.uint8)
    offs = to_device(gold["unpack_offs"]).view(torch.int64)
    lens = to_device(gold["unpack_lens"]).view(torch.int32)
    cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, opts=uopts[mode], ext=True)
    rng = np.random.default_rng(17 + opts)
    src = _sources(oracle, n, rng)
    rx_sec = rng.integers(1_600_000_000, 1_800_000_000, n, dtype=np.int64).astype(np.uint32)
    rx_usec = rng.integers(0, 1_000_000, n).astype(np.uint32)
    ttl = rng.integers(-1, 256, n).astype(np.int32)
    text, line_off = eng.log_recv_text(
        slab, n, cols, to_device(src.view(np.uint8)), to_device(rx_sec), to_device(rx_usec),
        rec_off=offs, ttl=to_device(ttl), protocol=proto, opts=opts)
    got = text.cpu().numpy().tobytes()
    want = oracle.log_recv_text(gold[f"unpack_fields_{mode}"], gold["unpack_slab"],
                                gold["unpack_offs"], src, rx_sec, rx_usec, protocol=proto,
                                ttl=ttl, opts=opts)
    if got != want:
        g, w = got.split(b"\n"), want.split(b"\n")
        bad = [i for i in range(min(len(g), len(w))) if g[i] != w[i]][:3]
        raise AssertionError([(g[i], w[i]) for i in bad] or (len(got), len(want)))
    offs_h = line_off.cpu().numpy()
    assert offs_h[0] == 0 and offs_h[-1] == len(want)


def test_log_rows_input_and_gps_values(torch, eng, oracle):
    """Row-major unpack output as the formatter's core input; GPS raw words across the whole
    u32 range (the exactly rounded %f)."""
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd._abi import TMPL_DTYPE, DESC_DTYPE
    rng = np.random.default_rng(5)
    n_t = 64
    t = np.zeros(n_t, TMPL_DTYPE)
    t["flow_id"] = np.arange(1, n_t + 1)
    t["dst_type"], t["dst_len"], t["dst_port"] = 1, 4, 5000
    t["dst_addr"][:, :4] = [10, 1, 2, 3]
    raws = np.concatenate([[0, 1, 10800000, 10800001, 10799999, 70740000, 0xFFFFFFFF],
                           rng.integers(0, 2**32, n_t - 7, dtype=np.uint64)]).astype(np.uint32)
    t["lat_raw"] = raws
    t["lon_raw"] = raws[::-1]
    t["alt"] = rng.integers(-2**31, 2**31, n_t, dtype=np.int64).astype(np.int32)
    t["gps_status"] = np.arange(n_t) % 3
    n = 4096
    d = np.zeros(n, DESC_DTYPE)
    d["tmpl"] = np.arange(n) % n_t
    d["seq_num"] = np.arange(n)
    d["tx_sec"] = 1_700_000_000
    d["tx_usec"] = rng.integers(0, 1_000_000, n)
    d["msg_len"] = 256
    pool = np.zeros(16, np.uint8)
    dt, dp, dd = to_device(t), to_device(pool), to_device(d)
    crc = torch.empty(n_t, dtype=torch.int32, device="cuda")
    eng.pack_prepare(dt, n_t, dp, crc)
    slab = torch.zeros(n * 256, dtype=torch.uint8, device="cuda")
    eng.pack(dt, crc, dd, n, dp, slab, stride=256, opts=PACK_CHECKSUM)
    from mgen_amd._abi import COLS_EXT
    full = eng.alloc_cols(n, ext=True)
    cols = {name: full[name] for name, _, _ in COLS_EXT}   # extended columns + core rows
    cols["rows"] = eng.alloc_rows(n)
    eng.unpack(slab, n, stride=256, fixed_len=256, cols=cols)
    src = np.zeros(n, oracle.ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 40000
    src["addr"][:, :4] = [192, 168, 0, 9]
    rx_s = np.full(n, 1_700_000_001, np.uint32)
    rx_u = np.arange(n, dtype=np.uint32)
    text, _ = eng.log_recv_text(slab, n, cols, to_device(src.view(np.uint8)), to_device(rx_s),
                                to_device(rx_u), stride=256)
    h = slab.cpu().numpy()
    f = oracle.udp_recv_batch(h, n, stride=256, fixed_len=256)
    want = oracle.log_recv_text(f, h, np.arange(n, dtype=np.uint64) * 256, src, rx_s, rx_u)
    assert text.cpu().numpy().tobytes() == want


@pytest.mark.parametrize("mode", ["udp", "tcp_force"])
def test_binary_log_matches_oracle(torch, eng, gold, oracle, mode):
    """Binary RECV / RERR records (LogRecvEvent / LogRecvError binary form) == the oracle."""
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP, to_device
    uopts = {"udp": 0, "tcp_force": OPT_TCP | OPT_CHECKSUM_FORCE}
    n = len(gold["unpack_lens"])
    slab = to_device(gold["unpack_slab"]).view(torch.uint8)
    offs = to_device(gold["unpack_offs"]).view(torch.int64)
    lens = to_device(gold["unpack_lens"]).view(torch.int32)
    cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, opts=uopts[mode], ext=True)
    rng = np.random.default_rng(23)
    src = _sources(oracle, n, rng)
    rx_sec = rng.integers(1_600_000_000, 1_800_000_000, n, dtype=np.int64).astype(np.uint32)
    rx_usec = rng.integers(0, 1_000_000, n).astype(np.uint32)
    proto = 1 if mode == "udp" else 2
    out, pos = eng.log_recv_binary(slab, n, cols, to_device(src.view(np.uint8)),
                                   to_device(rx_sec), to_device(rx_usec), rec_off=offs,
                                   protocol=proto)
    want = oracle.log_recv_binary(gold[f"unpack_fields_{mode}"], gold["unpack_slab"],
                                  gold["unpack_offs"], src, rx_sec, rx_usec, protocol=proto)
    got = out.cpu().numpy().tobytes()
    assert len(got) == len(want)
    assert got == want
    # with the received lengths: a record's bytes past its msg_len field but inside the
    # datagram are the reference's receive-buffer bytes
    lens = gold["unpack_lens"]
    out, _ = eng.log_recv_binary(slab, n, cols, to_device(src.view(np.uint8)),
                                 to_device(rx_sec), to_device(rx_usec), rec_off=offs,
                                 rec_len=to_device(lens.astype(np.uint32)).view(torch.int32),
                                 protocol=proto)
    want2 = oracle.log_recv_binary(gold[f"unpack_fields_{mode}"], gold["unpack_slab"],
                                   gold["unpack_offs"], src, rx_sec, rx_usec, protocol=proto,
                                   rec_len=lens)
    assert out.cpu().numpy().tobytes() == want2
    if mode == "udp":   # the golden corpus has records whose msg_len field is short
        assert want2 != want


def test_binary_log_message_bound_and_oob(torch, eng, oracle):
    """Records whose msg_len is exactly header + payload (no checksum, no padding) in 256-B
    slots with non-zero bytes after them: each binary RECV record is exactly 4 +
    eventRecordLength bytes (doc/mgen.xml:4212-4216) and carries hdr + payload_len message
    bytes, never a neighbour's; a record outside the slab is logged as RERR with ERROR_LENGTH
    (3) in both forms, as include/mgenx.hpp maps MGENX_ERROR_OOB."""
    from mgen_amd import ERROR_OOB, to_device
    from mgen_amd._abi import DESC_DTYPE
    from mgen_amd.workloads import make_templates
    n, slot = 64, 256
    tmpl, pool = make_templates(4, payload=b"\x11\x22\x33\x44\x55")
    d = np.zeros(n, DESC_DTYPE)
    d["tmpl"] = np.arange(n) % 4
    d["seq_num"] = np.arange(n)
    d["tx_sec"] = 1_700_000_000
    d["msg_len"] = 200
    dt, dp = to_device(tmpl), to_device(pool)
    crc = torch.empty(4, dtype=torch.int32, device="cuda")
    eng.pack_prepare(dt, 4, dp, crc)
    slab = torch.full((n * slot,), 0xAB, dtype=torch.uint8, device="cuda")
    out_len = torch.empty(n, dtype=torch.int32, device="cuda")
    # first pass: header + payload sizes; then msg_len = exactly that (no padding)
    eng.pack(dt, crc, to_device(d), n, dp, slab, stride=slot, opts=0, out_len=out_len)
    c0 = eng.unpack(slab, n, stride=slot, fixed_len=200, ext=True)
    d["msg_len"] = (c0["hdr_len"].cpu().numpy().astype(np.int64) +
                    c0["payload_len"].cpu().numpy().view(np.uint16))
    slab.fill_(0xAB)
    eng.pack(dt, crc, to_device(d), n, dp, slab, stride=slot, opts=0, out_len=out_len)
    lens_h = out_len.cpu().numpy().astype(np.int32)
    offs_h = np.arange(n, dtype=np.int64) * slot
    offs_h[-1] = n * slot + 100           # the last record lies outside the slab
    offs, lens = to_device(offs_h), to_device(lens_h)
    cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, ext=True)
    err = cols["err"].cpu().numpy()
    assert err[-1] == ERROR_OOB and (err[:-1] == 0).all()
    mlen = cols["msg_len"].cpu().numpy().view(np.uint16).astype(np.int64)
    hdr = cols["hdr_len"].cpu().numpy().astype(np.int64)
    plen = cols["payload_len"].cpu().numpy().view(np.uint16).astype(np.int64)
    assert (mlen[:-1] == hdr[:-1] + plen[:-1]).all()
    src = np.zeros(n, oracle.ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 4000
    src["addr"][:, :4] = [10, 0, 0, 7]
    rx_s = np.full(n, 1_700_000_002, np.uint32)
    rx_u = np.arange(n, dtype=np.uint32)
    out, pos = eng.log_recv_binary(slab, n, cols, to_device(src.view(np.uint8)), to_device(rx_s),
                                   to_device(rx_u), rec_off=offs, protocol=1)
    got = out.cpu().numpy().tobytes()
    pos = pos.cpu().numpy().view(np.uint64)
    h = slab.cpu().numpy()
    f = oracle.udp_recv_batch(h, n - 1, rec_off=offs_h[:-1].astype(np.uint64),
                              rec_len=lens_h[:-1].astype(np.uint32))
    want = oracle.log_recv_binary(f, h, offs_h[:-1], src[:-1], rx_s[:-1], rx_u[:-1], protocol=1)
    assert got[:int(pos[n - 1])] == want
    # every RECV record is its header + eventRecordLength bytes, ending with the message's
    # own last byte
    for i in range(n - 1):
        rec = got[int(pos[i]):int(pos[i + 1])]
        assert rec[0] == 1 and len(rec) == 4 + int.from_bytes(rec[2:4], "big"), i
        m = int(mlen[i])
        assert rec[-1] == h[offs_h[i] + m - 1] and rec[-m + 4:] == h[offs_h[i] + 4:offs_h[i] + m].tobytes(), i
    last = got[int(pos[n - 1]):int(pos[n])]
    assert last[0] == 2 and last[-4:] == (3).to_bytes(4, "big")
    text, _ = eng.log_recv_text(slab, n, cols, to_device(src.view(np.uint8)), to_device(rx_s),
                                to_device(rx_u), rec_off=offs)
    assert text.cpu().numpy().tobytes().split(b"\n")[n - 1].find(b"RERR type>length ") > 0
