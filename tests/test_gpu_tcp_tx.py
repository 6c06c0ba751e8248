"""GPU parity of mgenx_pack_tcp (MgenTcpTransport's transmit byte stream: fragments, 8-KiB
buffers re-sent from their start, CRC over the whole fragment; mgenTransport.cpp:1320-1400,
1818-1993) with the oracle's or_tcp_tx restatement, byte for byte; and the stream it makes
frames and checks clean through mgenx_stream_scan + the TCP-rule unpack."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [0, 10, 27, 28, 60, 76, 100, 1000, 8187, 8188, 8189, 8190, 8191, 8192, 8193, 8194,
         8195, 8196, 8200, 12000, 16380, 16384, 16385, 24576, 40000, 65535, 65536, 65540,
         65600, 65610, 131070, 140000, 200000]


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
    from streams import golden
    return golden()


def _case(gold, rng, sizes):
    n = len(sizes)
    d = np.zeros(n, gold["desc"].dtype)
    d["tmpl"] = rng.integers(0, len(gold["tmpl"]), n)
    d["seq_num"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d["tx_sec"] = 1_700_000_000
    d["tx_usec"] = rng.integers(0, 1_000_000, n)
    d["flags"] = rng.choice([0, 0, 0, 4, 2, 0x20], n)
    return d, np.asarray(sizes, np.uint32)


def _gpu(torch, eng, gold, d, total, opts, fill_time=0):
    from mgen_amd import to_device
    tm, pool = to_device(gold["tmpl"]), to_device(gold["pool"])
    crc = torch.empty(len(gold["tmpl"]), dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, len(gold["tmpl"]), pool, crc)
    out, offs = eng.pack_tcp(tm, crc, to_device(d), to_device(total), len(d), pool, opts=opts,
                             fill_time=fill_time)
    torch.cuda.synchronize()
    return out.cpu().numpy(), offs.cpu().numpy()


@pytest.mark.parametrize("checksum", [True, False])
def test_tcp_tx_stream_matches_oracle(torch, eng, gold, checksum):
    from mgen_amd import PACK_CHECKSUM
    from oracle import oracle as O
    rng = np.random.default_rng(71 + checksum)
    sizes = list(SIZES) * 3
    rng.shuffle(sizes)
    d, total = _case(gold, rng, sizes)
    got, offs = _gpu(torch, eng, gold, d, total, PACK_CHECKSUM if checksum else 0)
    want = np.asarray(O.tcp_tx_batch(gold["tmpl"], d, total, gold["pool"], checksum=checksum),
                      np.uint8)
    assert len(got) == len(want)
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        k = int(np.searchsorted(offs, bad[0], side="right")) - 1
        raise AssertionError((int(bad[0]), k, int(total[k]), int(offs[k])))
    # per-message offsets: each message's own oracle stream at its offset
    for k in range(0, len(d), 7):
        one = np.asarray(O.tcp_tx_batch(gold["tmpl"], d[k:k + 1], total[k:k + 1], gold["pool"],
                                        checksum=checksum), np.uint8)
        assert np.array_equal(got[offs[k]:offs[k] + len(one)], one), k


def test_tcp_tx_random_fill(torch, eng, gold):
    from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    d, total = _case(gold, rng, [100, 8192, 8194, 16384, 70000, 30])
    eng.set_fill_time(1_700_000_123)
    got, _ = _gpu(torch, eng, gold, d, total, PACK_CHECKSUM | PACK_RANDOM_FILL, 1_700_000_123)
    want = np.asarray(O.tcp_tx_batch(gold["tmpl"], d, total, gold["pool"], checksum=True,
                                     random_fill=True, fill_time=1_700_000_123), np.uint8)
    assert np.array_equal(got, want)


def test_tcp_tx_config5_frames_and_checks(torch, eng, gold):
    """Config 5 records (16 KiB, checksum on) built on the GPU: the stream scan finds every
    record and the TCP-rule unpack verifies every CRC."""
    from mgen_amd import OPT_TCP, PACK_CHECKSUM, SCAN_TCP, to_device
    from mgen_amd.workloads import make_templates
    from mgen_amd._abi import DESC_DTYPE
    n = 2048
    tmpl, pool = make_templates(64)
    d = np.zeros(n, DESC_DTYPE)
    d["tmpl"] = np.arange(n) % 64
    d["seq_num"] = np.arange(n)
    d["tx_sec"] = 1_700_000_000
    d["flags"] = 4
    tm, pl = to_device(tmpl), to_device(pool)
    crc = torch.empty(64, dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, 64, pl, crc)
    total = to_device(np.full(n, 16384, np.uint32))
    out, offs = eng.pack_tcp(tm, crc, to_device(d), total, n, pl, opts=PACK_CHECKSUM)
    assert out.numel() == n * 16384
    so, sl, info = eng.stream_scan(out, SCAN_TCP)
    assert int(info.n_records) == n and torch.equal(so, offs)
    cols = eng.unpack(out, n, rec_off=so, rec_len=sl, opts=OPT_TCP)
    torch.cuda.synchronize()
    assert int((cols["err"] != 0).sum()) == 0
    assert np.array_equal(cols["seq_num"].cpu().numpy().view(np.uint32), np.arange(n))


def test_tcp_tx_short_buffer_no_store_past_it(torch, eng, gold):
    """mgenx_pack_tcp with a buffer shorter than the stream reports the length and fails, and
    stores nothing past the buffer's end (checked on a sentinel region after it); a right-sized
    call after it is exact, multi-fragment messages included."""
    import ctypes
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd import _ptr, _stream
    rng = np.random.default_rng(17)
    d, total = _case(gold, rng, [16384] * 40 + [200000] * 3)
    tm, pool = to_device(gold["tmpl"]), to_device(gold["pool"])
    crc = torch.empty(len(gold["tmpl"]), dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, len(gold["tmpl"]), pool, crc)
    dd, dt = to_device(d), to_device(total)
    # a one-fragment call first (rounds hint 1), then the multi-round case on a short buffer
    small_d, small_t = _case(gold, rng, [1000] * 8)
    eng.pack_tcp(tm, crc, to_device(small_d), to_device(small_t), 8, pool, opts=PACK_CHECKSUM)
    want, _ = eng.pack_tcp(tm, crc, dd, dt, len(d), pool, opts=PACK_CHECKSUM)
    want = want.cpu().numpy()
    n_total = len(want)
    cap = n_total // 2
    buf = torch.full((n_total + 65536,), 0xAB, dtype=torch.uint8, device="cuda")
    offs = torch.empty(len(d), dtype=torch.int64, device="cuda")
    tot = ctypes.c_uint64(0)
    rc = eng.lib.mgenx_pack_tcp(eng.ctx, _ptr(tm), _ptr(crc), _ptr(dd), _ptr(dt), len(d),
                                _ptr(pool), _ptr(buf), cap, _ptr(offs), ctypes.byref(tot),
                                PACK_CHECKSUM, 0, _stream(eng.device))
    torch.cuda.synchronize()
    assert rc != 0 and tot.value == n_total
    assert bool((buf[cap:] == 0xAB).all())
    got, _ = eng.pack_tcp(tm, crc, dd, dt, len(d), pool, opts=PACK_CHECKSUM)
    assert np.array_equal(got.cpu().numpy(), want)


def test_tcp_tx_plan_overflow_takes_exact_path(torch, eng, gold):
    """A stream past the one-launch plan's 2^46-byte running totals (16,385 messages of
    2^32 - 1 bytes) sends mgenx_pack_tcp to its exact path (plan kernel, device-wide scan):
    the reported length and the message offsets are still exact (uint64), and with no
    stream buffer the call fails with that length set."""
    import ctypes
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd import _ptr, _stream
    rng = np.random.default_rng(23)
    n = 16385
    d, total = _case(gold, rng, [0xFFFFFFFF] * n)
    ok = np.isin(gold["tmpl"]["dst_type"][d["tmpl"]], [1, 2])
    bytes_ = np.where(ok, np.uint64(0xFFFFFFFF), np.uint64(0))
    want_total = int(bytes_.sum())
    assert want_total >= 1 << 46
    tm, pool = to_device(gold["tmpl"]), to_device(gold["pool"])
    crc = torch.empty(len(gold["tmpl"]), dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, len(gold["tmpl"]), pool, crc)
    dd, dt = to_device(d), to_device(total)
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    tot = ctypes.c_uint64(0)
    rc = eng.lib.mgenx_pack_tcp(eng.ctx, _ptr(tm), _ptr(crc), _ptr(dd), _ptr(dt), n,
                                _ptr(pool), None, 0, _ptr(offs), ctypes.byref(tot),
                                PACK_CHECKSUM, 0, _stream(eng.device))
    torch.cuda.synchronize()
    assert rc != 0 and tot.value == want_total
    got = offs.cpu().numpy().view(np.uint64)
    want = np.concatenate([[0], np.cumsum(bytes_)[:-1]]).astype(np.uint64)
    assert np.array_equal(got, want)
    # and the one-launch path is back for the next (small) call
    small_d, small_t = _case(gold, rng, [1000, 20000, 70000])
    out, offs2 = _gpu(torch, eng, gold, small_d, small_t, PACK_CHECKSUM)
    from oracle import oracle as O
    want2 = np.asarray(O.tcp_tx_batch(gold["tmpl"], small_d, small_t, gold["pool"], checksum=True),
                       np.uint8)
    assert np.array_equal(out, want2)


def test_tcp_tx_plan_epoch_wrap(torch, eng, gold):
    """The one-launch plan tags its look-back words and verdict with a 16-bit epoch, cleared
    when it wraps: 65,540 back-to-back calls on one context (past the wrap) stay byte-exact,
    multi-fragment messages included."""
    import ctypes
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd import _ptr, _stream
    from oracle import oracle as O
    rng = np.random.default_rng(31)
    d, total = _case(gold, rng, [100, 20000, 70000, 9000])
    want = np.asarray(O.tcp_tx_batch(gold["tmpl"], d, total, gold["pool"], checksum=True),
                      np.uint8)
    tm, pool = to_device(gold["tmpl"]), to_device(gold["pool"])
    crc = torch.empty(len(gold["tmpl"]), dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, len(gold["tmpl"]), pool, crc)
    dd, dt = to_device(d), to_device(total)
    buf = torch.zeros(len(want), dtype=torch.uint8, device="cuda")
    offs = torch.empty(len(d), dtype=torch.int64, device="cuda")
    tot = ctypes.c_uint64(0)
    args = (eng.ctx, _ptr(tm), _ptr(crc), _ptr(dd), _ptr(dt), len(d), _ptr(pool), _ptr(buf),
            len(want), _ptr(offs), ctypes.byref(tot), PACK_CHECKSUM, 0, _stream(eng.device))
    fn = eng.lib.mgenx_pack_tcp
    for k in range(65540):
        if k == 65530:  # (the last calls write into a cleared buffer)
            torch.cuda.synchronize()
            buf.zero_()
        assert fn(*args) == 0 and tot.value == len(want), k
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), want)


@pytest.mark.parametrize("checksum", [False, True])
def test_doc_tcp_fragment_example_on_gpu(torch, eng, oracle, checksum):
    """doc/mgen.xml:3644-3662 on the device: mgenx_pack_tcp of the 66,559-B message equals
    or_tcp_tx (a 65,535-B CONTINUES fragment and a 1,024-B END_OF_MSG one, same seq), the TCP
    framing scan frames exactly those two records, and the RECV log of the TCP-rule unpack
    prints the doc's two lines (as the code prints them: test_oracle_pins)."""
    from mgen_amd import OPT_TCP, PACK_CHECKSUM, SCAN_TCP, to_device
    from mgen_amd._abi import DESC_DTYPE, TMPL_DTYPE
    from test_oracle_pins import (DOC_DAY, doc_tcp_expected_lines, doc_tcp_msg,
                                  doc_tcp_recv_inputs)
    t = np.zeros(1, TMPL_DTYPE)
    t["flow_id"], t["dst_type"], t["dst_len"], t["dst_port"] = 1, 1, 4, 5000
    t["dst_addr"][0, :4] = [10, 0, 0, 2]
    t["lat_raw"] = t["lon_raw"] = 70740000        # (999 + 180) * 60000
    t["alt"] = -999
    d = np.zeros(1, DESC_DTYPE)
    d["seq_num"], d["tx_sec"], d["tx_usec"] = 1, DOC_DAY + 36 * 60 + 11, 377105
    pool = np.zeros(16, np.uint8)
    tm, pl = to_device(t), to_device(pool)
    crc = torch.empty(1, dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, 1, pl, crc)
    out, offs = eng.pack_tcp(tm, crc, to_device(d), to_device(np.array([66559], np.uint32)), 1,
                             pl, opts=PACK_CHECKSUM if checksum else 0)
    want = oracle.tcp_tx(doc_tcp_msg(oracle), checksum=checksum)
    got = out.cpu().numpy().tobytes()
    assert len(got) == 66559 and got == want
    so, sl, info = eng.stream_scan(out, SCAN_TCP)
    assert int(info.n_records) == 2
    assert so.cpu().numpy().tolist() == [0, 65535] and sl.cpu().numpy().tolist() == [65535, 1024]
    cols = eng.unpack(out, 2, rec_off=so, rec_len=sl, opts=OPT_TCP, ext=True)
    torch.cuda.synchronize()
    assert cols["err"].cpu().numpy().tolist() == [0, 0]
    src, rx_sec, rx_usec = doc_tcp_recv_inputs(oracle, 2)
    text, _ = eng.log_recv_text(out, 2, cols, to_device(src.view(np.uint8)), to_device(rx_sec),
                                to_device(rx_usec), rec_off=so, protocol=2)
    lines = text.cpu().numpy().tobytes().decode().splitlines(keepends=True)
    assert lines == doc_tcp_expected_lines()
