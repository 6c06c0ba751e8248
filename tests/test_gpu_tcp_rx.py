"""GPU parity of mgenx_tcp_rx_persist (the TCP receiver's persistent rx_msg,
mgenTransport.cpp:1082,1501-1513,1714-1720,2016-2028, CalcRxChecksum :1516-1564) with the
oracle's or_tcp_rx_persist restatement over one connection's records: records that stop
early inherit the previous record's members, the CRC check reads the flags rx_msg holds,
and with no log file nothing is decoded."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("err", "flags", "flow_id", "seq_num", "tx_sec", "tx_usec", "msg_len", "dst_port",
          "dst_type", "dst_len", "hdr_len", "lat_raw", "lon_raw", "alt", "gps_status",
          "payload_type", "payload_len", "host_type", "host_len", "host_port")


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


def connection(seed, n=400):
    """One connection's records: oracle-built TCP messages of mixed (also truncating) sizes,
    short junk records (< MIN_SIZE), bad version bytes, corrupted CRCs, checksum on/off."""
    from oracle import oracle as O
    from streams import golden
    g = golden()
    rng = np.random.default_rng(seed)
    recs = []
    for k in range(n):
        u = rng.random()
        if u < 0.08:                                   # shorter than MIN_SIZE
            L = int(rng.integers(4, 28))
            r = rng.integers(0, 256, L, dtype=np.uint8)
            r[0], r[1] = L >> 8, L & 255
            recs.append(r)
            continue
        d = np.zeros(1, g["desc"].dtype)
        d["tmpl"] = rng.integers(0, len(g["tmpl"]))
        d["seq_num"] = k
        d["tx_sec"] = 1_700_000_000 + k
        d["tx_usec"] = rng.integers(0, 1_000_000)
        d["flags"] = 0
        size = int(rng.choice([30, 40, 52, 60, 64, 70, 80, 120, 300, 1000, 9000]))
        ck = bool(rng.random() < 0.7)
        r = np.asarray(O.tcp_tx_batch(g["tmpl"], d, np.array([size], np.uint32), g["pool"],
                                      checksum=ck), np.uint8).copy()
        if len(r) == 0:
            continue
        if u > 0.95 and len(r) > 3:
            r[2] = 3                                   # bad version
        elif u > 0.9 and len(r) > 40:
            r[len(r) // 2] ^= 0x5A                     # corrupt (CRC)
        recs.append(r)
    lens = np.array([len(r) for r in recs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    return np.concatenate(recs), offs, lens


def run_gpu(torch, eng, stream, offs, lens, opts_rx, force, splits=(0,)):
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP, RX_NOLOG, to_device
    n = len(offs)
    s = to_device(stream)
    o = to_device(offs).view(torch.int64)
    ln = to_device(lens).view(torch.int32)
    uopts = OPT_TCP | (OPT_CHECKSUM_FORCE if (force or (opts_rx & RX_NOLOG)) else 0)
    cols = eng.unpack(s, n, rec_off=o, rec_len=ln, opts=uopts, ext=True)
    state = eng.rx_state_init()
    prec = torch.empty(n, dtype=torch.int32, device="cuda")
    bounds = list(splits) + [n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        sub = {k: (v[a:b] if v.numel() == n else v[a * (v.numel() // n):b * (v.numel() // n)])
               for k, v in cols.items()}
        eng.tcp_rx_persist(s, o[a:b], ln[a:b], b - a, sub, state, payload_rec=prec[a:b],
                           opts=opts_rx)
        # payload_rec is relative to the call: make it absolute
        if b - a:
            p = prec[a:b]
            prec[a:b] = torch.where(p == -1, p, p + a)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in cols.items()}, prec.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("log_open,force", [(True, False), (True, True), (False, False),
                                            (False, True)])
def test_tcp_rx_persist_vs_oracle(torch, eng, log_open, force):
    from mgen_amd import RX_FORCE, RX_NOLOG
    from oracle import oracle as O
    stream, offs, lens = connection(11 + 2 * log_open + force)
    opts = (0 if log_open else RX_NOLOG) | (RX_FORCE if force else 0)
    got, prec = run_gpu(torch, eng, stream, offs, lens, opts, force)
    want, wprec, _, _ = O.tcp_rx_persist(stream, offs, lens, log_open=log_open, force=force)
    n = len(offs)
    for f in FIELDS:
        g = got[f].view(want[f].dtype) if got[f].dtype.itemsize == want[f].dtype.itemsize \
            else got[f].astype(want[f].dtype)
        bad = np.nonzero(g != want[f])[0]
        assert len(bad) == 0, (f, bad[:5], g[bad[:5]], want[f][bad[:5]])
    # the address bytes that are part of the address (ProtoAddress keeps dst_len of them)
    dst = got["dst_addr"].reshape(n, 16)
    keep = np.arange(16)[None, :] < np.minimum(want["dst_len"], 16)[:, None]
    assert np.array_equal(np.where(keep, dst, 0), np.where(keep, want["dst_addr"], 0))
    pl = want["payload_len"] != 0
    assert np.array_equal(got["payload_off"].view(np.uint32)[pl], want["payload_off"][pl])
    assert np.array_equal(prec, wprec)
    if log_open:   # the quirks happened: inherited members and carried-flag CRC failures
        assert (want["err"] == 2).sum() > 0 and (want["flow_id"] == 0).sum() > 0


def test_tcp_rx_persist_across_batches(torch, eng):
    """Three calls over one connection carry rx_msg through the state; the result equals one
    call (payload_rec made absolute by the caller)."""
    from oracle import oracle as O
    stream, offs, lens = connection(29)
    got, prec = run_gpu(torch, eng, stream, offs, lens, 0, False, splits=(0, 97, 250))
    want, wprec, _, _ = O.tcp_rx_persist(stream, offs, lens)
    for f in ("err", "flags", "tx_sec", "dst_port", "lat_raw", "payload_type", "hdr_len"):
        assert np.array_equal(got[f].astype(np.int64), want[f].astype(np.int64)), f
