"""GPU parity of mgenx_stream_scan (TCP / SINK record framing) against the oracle's
sequential restatement (or_tcp_scan / or_sink_scan, which follow mgenTransport.cpp:1683-1760
and mgenAppSinkTransport.cpp:369-434), plus full-size properties for BASELINE config 5."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x4D47454E


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


from streams import sink_stream, tcp_stream  # noqa: E402


def check(torch, eng, stream, mode):
    from mgen_amd import SCAN_SINK, to_device
    from oracle import oracle as O
    if mode == SCAN_SINK:
        wo, wl, _, wc = O.sink_scan(stream.tobytes())
        ws = 0
    else:
        wo, wl, _, wc, ws = O.tcp_scan(stream.tobytes())
    d = to_device(stream) if len(stream) else torch.zeros(1, dtype=torch.uint8, device="cuda")
    offs, lens, info = eng.stream_scan(d, mode, nbytes=len(stream))
    go = offs.cpu().numpy().view(np.uint64)
    gl = lens.cpu().numpy().view(np.uint32)
    assert int(info.n_records) == len(wo)
    assert np.array_equal(go, wo), (go[:8], wo[:8])
    assert np.array_equal(gl, wl)
    assert int(info.consumed) == wc
    assert int(info.status) == ws
    return info


def test_tcp_valid_mixed_sizes(torch, eng, gold):
    from mgen_amd import SCAN_TCP
    rng = np.random.default_rng(SEED)
    sizes = rng.integers(76, 40000, 300)
    sizes[::7] = 16384
    s = tcp_stream(gold, sizes, rng)
    info = check(torch, eng, s, SCAN_TCP)
    assert info.resolved == 0          # valid stream: no sequential fallback


def test_tcp_truncated_tail(torch, eng, gold):
    from mgen_amd import SCAN_TCP
    rng = np.random.default_rng(SEED + 1)
    s = tcp_stream(gold, rng.integers(76, 20000, 100), rng)
    for cut in (1, 2, 3, 100, 9000):
        check(torch, eng, s[:-cut], SCAN_TCP)


def test_tcp_bad_version_and_short_length(torch, eng, gold):
    from mgen_amd import SCAN_TCP
    from oracle import oracle as O
    rng = np.random.default_rng(SEED + 2)
    s = tcp_stream(gold, rng.integers(76, 5000, 200), rng).copy()
    offs, _, _, _, _ = O.tcp_scan(s.tobytes())
    for k in (0, 17, 50, 51, 120):
        s[int(offs[k]) + 2] = 7            # version byte: framing continues through it
    info = check(torch, eng, s, SCAN_TCP)
    assert info.resolved >= 5
    s2 = s.copy()
    s2[int(offs[150])] = 0
    s2[int(offs[150]) + 1] = 3              # msg_len 3 < 4: stream error, scan stops
    info = check(torch, eng, s2, SCAN_TCP)
    assert info.status == 1


def test_sink_with_garbage(torch, eng, gold):
    from mgen_amd import SCAN_SINK
    rng = np.random.default_rng(SEED + 3)
    sizes = rng.integers(28, 8193, 400)
    check(torch, eng, sink_stream(gold, sizes, rng), SCAN_SINK)
    check(torch, eng, sink_stream(gold, sizes, rng, garbage_every=5), SCAN_SINK)


@pytest.mark.parametrize("mode", [0, 1])
def test_random_bytes(torch, eng, mode):
    rng = np.random.default_rng(SEED + 4 + mode)
    for n in (0, 1, 3, 1000, 300_000):
        check(torch, eng, rng.integers(0, 256, n, dtype=np.uint8), mode)


@pytest.mark.parametrize("mode", [0, 1])
def test_candidate_overflow_path(torch, eng, mode):
    """A stream of 0x02 bytes makes every position plausible (beyond the candidate budget of
    one per 16 bytes): the scan falls back to the sequential resolver and still matches."""
    s = np.full(200_000, 2, np.uint8)
    info = check(torch, eng, s, mode)
    assert info.candidates == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_block_slot_overflow_second_pass(torch, eng, gold, mode):
    """A 64 KiB run of 0x02 bytes inside a valid stream: that block has more candidates than
    its slots (second detect pass writes them with exact offsets), the stream stays within
    the candidate budget, and the framing still equals the oracle's."""
    rng = np.random.default_rng(SEED + 70 + mode)
    if mode == 0:
        a = tcp_stream(gold, rng.integers(76, 5000, 400), rng)
        b = tcp_stream(gold, rng.integers(76, 5000, 400), rng)
    else:
        a = sink_stream(gold, rng.integers(28, 8193, 250), rng)
        b = sink_stream(gold, rng.integers(28, 8193, 250), rng)
    s = np.concatenate([a, np.full(70_000, 2, np.uint8), b])
    info = check(torch, eng, s, mode)
    assert info.candidates > 65536


def test_config5_stream_scan_then_unpack(torch, eng, gold):
    """BASELINE config 5 shape (16 KiB TCP records, checksum on) at 64 MiB: the scan finds
    every record at k * 16384 and the TCP-rule unpack over its output validates them all."""
    from mgen_amd import OPT_TCP, SCAN_TCP, to_device
    n = 4096
    rng = np.random.default_rng(SEED + 5)
    s = tcp_stream(gold, np.full(n, 16384), rng)
    assert len(s) == n * 16384
    d = to_device(s)
    offs, lens, info = eng.stream_scan(d, SCAN_TCP)
    assert int(info.n_records) == n and int(info.consumed) == len(s) and info.resolved == 0
    assert np.array_equal(offs.cpu().numpy(), np.arange(n, dtype=np.int64) * 16384)
    cols = eng.unpack(d, n, rec_off=offs, rec_len=lens, opts=OPT_TCP)
    torch.cuda.synchronize()
    assert int((cols["err"] != 0).sum()) == 0
    assert np.array_equal(cols["seq_num"].cpu().numpy().view(np.uint32), np.arange(n))
    # the same scan into caller-preallocated outputs, on a fresh engine (the shared one may be
    # backing off the chain hypothesis after the error streams above): the first call builds
    # exactly, the next ones take the successor-marked chain
    from mgen_amd import Engine
    e2 = Engine(0)
    out = (torch.full((n + 8,), -1, dtype=torch.int64, device="cuda"),
           torch.full((n + 8,), -1, dtype=torch.int32, device="cuda"))
    e2.stream_scan(d, SCAN_TCP, out=out)
    for _ in range(2):
        o2, l2, i2 = e2.stream_scan(d, SCAN_TCP, out=out)
        assert int(i2.n_records) == n and int(i2.consumed) == len(s)
        assert torch.equal(o2, offs) and torch.equal(l2, lens)
        assert int(i2.path) == 2  # the successor-marked chain (no lifting)
    e2.close()


# ---- sharded framing (mgenx_stream_scan_exits / _range, mgen_amd/shard.py) ----

def _corpus():
    from streams import corpus
    return corpus()


@pytest.mark.parametrize("case", range(7))
def test_scan_range_vs_sequential(torch, eng, case):
    """mgenx_stream_scan_range from arbitrary entries below arbitrary limits equals the
    reference rule started there (tests/shard_ref.walk)."""
    from mgen_amd import to_device
    from shard_ref import walk
    _, s, mode = _corpus()[case]
    d = to_device(s)
    rng = np.random.default_rng(SEED + 40 + case)
    b = s.tobytes()
    reuse = False
    for _ in range(6):
        entry = int(rng.integers(0, len(s) // 2))
        limit = int(rng.integers(entry, len(s) + 1))
        offs, lens, info = eng.stream_scan_range(d, mode, entry, limit, reuse=reuse)
        reuse = True
        wo, wl, wc, ws = walk(b, mode, entry, limit)
        assert np.array_equal(offs.cpu().numpy(), np.asarray(wo, np.int64))
        assert np.array_equal(lens.cpu().numpy(), np.asarray(wl, np.int32))
        assert (int(info.consumed), int(info.status)) == (wc, ws)
    # offset 0 to the end is the whole-stream scan
    offs, lens, info = eng.stream_scan_range(d, mode, 0, len(s))
    wo, wl, wc, ws = walk(b, mode, 0, len(s))
    assert np.array_equal(offs.cpu().numpy(), np.asarray(wo, np.int64))


def test_scan_range_reuse_needs_tables(torch, eng):
    from mgen_amd import MgenxError, to_device
    d = to_device(np.zeros(1000, np.uint8))
    eng.stream_scan(d, 0)
    d2 = to_device(np.zeros(1000, np.uint8))
    with pytest.raises(MgenxError):
        eng.stream_scan_range(d2, 0, 0, 1000, reuse=True)


@pytest.mark.parametrize("case", range(7))
def test_scan_exits_vs_reference(torch, eng, case):
    from mgen_amd import to_device
    from mgen_amd.shard import HALO
    from shard_ref import RefScanner
    _, s, mode = _corpus()[case]
    for a, limit in ((0, len(s) // 2), (len(s) // 3, len(s) // 4)):
        local = s[a:a + limit + HALO]
        ent, ext, _ = eng.stream_scan_exits(to_device(local), mode, HALO, limit, cap=4096)
        want = RefScanner(local.tobytes()).exits(None, mode, HALO, limit)
        assert np.array_equal(ent.cpu().numpy().view(np.uint64), want[0])
        assert np.array_equal(ext.cpu().numpy().view(np.uint64), want[1])


def _sharded_gpu(s, mode, world):
    import threading

    from mgen_amd import Engine, to_device
    from mgen_amd.shard import EngineScanner, ThreadComm, scan_sharded, shard_bounds
    tc = ThreadComm(world)
    res, err = [None] * world, []

    def go(r):
        try:
            e = Engine(0)
            a, _, hi = shard_bounds(len(s), world, r)
            local = to_device(s[a:hi])
            offs, lens, summ = scan_sharded(EngineScanner(e), tc.rank_view(r), local, len(s),
                                            mode)
            o = np.zeros(0, np.int64) if offs is None else offs.cpu().numpy() + a
            ln = np.zeros(0, np.int32) if lens is None else lens.cpu().numpy()
            res[r] = (o, ln, summ)
            e.close()
        except BaseException as ex:  # noqa: BLE001
            err.append(ex)
            tc._bar.abort()
    th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not err, err
    return res


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_scan_gpu_equals_whole(torch, eng, world):
    """Simulated ranks (threads, one context each) on one GPU: the union of the shards'
    records and the stitched summary equal the whole-stream scan, on every corpus case."""
    from mgen_amd import to_device
    for name, s, mode in _corpus():
        offs, lens, info = eng.stream_scan(to_device(s), mode)
        res = _sharded_gpu(s, mode, world)
        assert np.array_equal(np.concatenate([r[0] for r in res]), offs.cpu().numpy()), name
        assert np.array_equal(np.concatenate([r[1] for r in res]), lens.cpu().numpy()), name
        for r in res:
            assert r[2] == (int(info.n_records), int(info.consumed), int(info.status)), name


def test_sharded_scan_config5_shape(torch, eng, gold):
    """Config 5 records (16 KiB, TCP, checksum on) over a 64 MiB stream in 4 shards."""
    from mgen_amd import to_device
    n = 4096
    rng = np.random.default_rng(SEED + 50)
    s = tcp_stream(gold, np.full(n, 16384), rng)
    res = _sharded_gpu(s, 0, 4)
    assert np.array_equal(np.concatenate([r[0] for r in res]), np.arange(n) * 16384)
    assert all(r[2] == (n, len(s), 0) for r in res)
    del to_device


def test_scan_beyond_4gib_device_scan_path(torch, eng, gold):
    """A stream of more than 36864 detect blocks (> 1.125 GiB of 32-KiB blocks; this one is
    past 4 GiB, so offsets need 64 bits) takes the multi-workgroup exclusive scan of the block
    counts: a valid prefix followed by zero bytes frames as the oracle frames the prefix plus
    the zero-length error after it."""
    from oracle import oracle as O
    rng = np.random.default_rng(SEED + 60)
    pre = tcp_stream(gold, rng.integers(76, 3000, 50), rng)
    n = (4 << 30) + 3 * 65536 + 123
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d[:len(pre)] = torch.from_numpy(pre).cuda()
    tail = 5 << 20                                  # records planted near the end too
    d[n - tail:n - tail + len(pre)] = torch.from_numpy(pre).cuda()
    offs, lens, info = eng.stream_scan(d, 0, cap=1000)
    wo, wl, _, wc, ws = O.tcp_scan(np.concatenate([pre, np.zeros(16, np.uint8)]).tobytes())
    assert np.array_equal(offs.cpu().numpy(), np.asarray(wo, np.int64))
    assert (int(info.consumed), int(info.status)) == (wc, 1)
    assert int(info.candidates) >= 2 * len(wo)
    del d
    torch.cuda.empty_cache()


# ---- TCP header-copy pruning (speculative whole-stream scans, mgenx_scan.hip kPrune) ----

def test_pruned_scan_tcp_transmit_stream(torch, gold):
    """The TCP transmit form of 12-KiB and 20-KiB messages (each re-sends its 8-KiB Pack
    buffer, so headers repeat 8192 bytes on): repeated scans on one engine -- the first exact,
    the later ones speculative with the copies pruned -- all equal the oracle's framing."""
    from mgen_amd import Engine, SCAN_TCP, to_device
    from oracle import oracle as O
    rng = np.random.default_rng(SEED + 70)
    s = tcp_stream(gold, rng.choice([12288, 20480, 16384, 900], 600), rng)
    wo, wl, _, wc, ws = O.tcp_scan(s.tobytes())
    e = Engine(0)
    d = to_device(s)
    cands = []
    for k in range(3):
        offs, lens, info = e.stream_scan(d, SCAN_TCP)
        assert np.array_equal(offs.cpu().numpy(), np.asarray(wo, np.int64)), k
        assert np.array_equal(lens.cpu().numpy().view(np.uint32), np.asarray(wl, np.uint32))
        assert (int(info.consumed), int(info.status)) == (wc, ws)
        cands.append(int(info.path))
    # the first call builds exactly; calls 2 and 3 take the successor-marked hypothesis
    assert cands == [0, 2, 2], cands
    e.close()


def test_pruned_scan_falls_back_on_repeated_records(torch, gold):
    """Records whose first 16 bytes repeat exactly 8192 bytes later (identical 8-KiB records):
    pruning drops real record starts, the pruned set is not the chain, and the scan rebuilds
    without pruning -- the framing still equals the oracle's, on every call."""
    from mgen_amd import Engine, SCAN_TCP, to_device
    from oracle import oracle as O
    rng = np.random.default_rng(SEED + 71)
    one = tcp_stream(gold, np.array([8192]), rng)
    s = np.concatenate([tcp_stream(gold, np.array([5000]), rng)] + [one] * 40 +
                       [tcp_stream(gold, np.array([3000, 700]), rng)])
    wo, wl, _, wc, ws = O.tcp_scan(s.tobytes())
    e = Engine(0)
    d = to_device(s)
    paths = []
    for k in range(3):
        offs, lens, info = e.stream_scan(d, SCAN_TCP)
        assert np.array_equal(offs.cpu().numpy(), np.asarray(wo, np.int64)), k
        assert (int(info.consumed), int(info.status)) == (wc, ws)
        paths.append(int(info.path))
    # the hypothesis failed on call 2 (exact rebuild, path 0) and backs off on call 3
    assert paths[:2] == [0, 0] and paths[2] != 2, paths
    e.close()


# ---- config 5 at its real size (tests had stopped at 64 MiB) ----

def _tcp_tx_stream(torch, eng, n, msg=16384):
    """n messages of `msg` bytes through the GPU TCP transmit path (mgenx_pack_tcp), as the
    bench builds config 5: 64 templates, checksum on."""
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd._abi import DESC_DTYPE
    from mgen_amd.workloads import make_templates
    tmpl, pool = make_templates(64)
    desc = np.zeros(n, DESC_DTYPE)
    seq = np.arange(n)
    desc["tmpl"], desc["seq_num"] = seq % 64, seq
    desc["tx_sec"], desc["tx_usec"] = 1_700_000_000 + seq // 1_000_000, seq % 1_000_000
    desc["flags"] = 4
    tm, pl = to_device(tmpl), to_device(pool)
    tcrc = torch.empty(64, dtype=torch.int32, device="cuda")
    eng.pack_prepare(tm, 64, pl, tcrc)
    total = torch.full((n,), msg, dtype=torch.int32, device="cuda")
    stream, _ = eng.pack_tcp(tm, tcrc, to_device(desc), total, n, pl, opts=PACK_CHECKSUM)
    torch.cuda.synchronize()
    return stream


@pytest.mark.parametrize("n", [65536, 73728, 73730])
def test_config5_full_size_vs_oracle(torch, eng, n):
    """BASELINE config 5 at full size: 65,536 x 16 KiB (1 GiB, 32,768 detect blocks), and
    streams on (36,864 blocks = 1.125 GiB) and just past (36,865) the LDS block-count path's
    bound (mgenx_scan.hip kScanSmall).  The oracle's sequential framing + Unpack + CRC
    (or_tcp_scan, mgenTransport.cpp:1683-1760) against mgenx_stream_scan on a fresh engine:
    the first call (exact build) and the second (the successor-marked chain, path 2)."""
    import ctypes
    from mgen_amd import Engine, OPT_TCP, SCAN_TCP, UNPACK_K_LONG
    from oracle import oracle as O
    stream = _tcp_tx_stream(torch, eng, n)
    host = stream.cpu().numpy()
    assert host.size == n * 16384
    cap = n + 8
    wo = np.zeros(cap, np.uint64)
    wl = np.zeros(cap, np.uint32)
    wf = np.zeros(cap, O.FIELDS_DTYPE)
    cons, st = ctypes.c_uint64(0), ctypes.c_int(0)
    P = ctypes.c_void_p
    k = O.lib().or_tcp_scan(P(host.ctypes.data), host.size, 0, P(wo.ctypes.data),
                            P(wl.ctypes.data), P(wf.ctypes.data), cap, ctypes.byref(cons),
                            ctypes.byref(st))
    assert k == n and cons.value == host.size and st.value == 0
    assert int(wf["err"][:n].sum()) == 0
    e2 = Engine(0)
    try:
        paths = []
        for call in range(2):
            offs, lens, info = e2.stream_scan(stream, SCAN_TCP)
            assert int(info.n_records) == n and int(info.consumed) == host.size, call
            assert int(info.status) == 0
            assert np.array_equal(offs.cpu().numpy().view(np.uint64), wo[:n]), call
            assert np.array_equal(lens.cpu().numpy().view(np.uint32), wl[:n]), call
            paths.append(int(info.path))
        assert paths == [0, 2], paths
        cols = e2.unpack(stream, n, rec_off=offs, rec_len=lens, opts=OPT_TCP)
        torch.cuda.synchronize()
        assert e2.last_unpack_kernel() == UNPACK_K_LONG   # one wave per 16-KiB record
        for key in ("err", "seq_num", "flow_id", "tx_sec", "tx_usec", "msg_len", "flags",
                    "dst_port", "payload_len"):
            got = cols[key].cpu().numpy().view(wf[key].dtype)
            assert np.array_equal(got, wf[key][:n]), key
    finally:
        e2.close()
    del stream
    torch.cuda.empty_cache()


# ---- the chain kernel (scan_chain_kernel, path 2) at its edges ----

def _scan_calls(torch, s, calls=3, mode=0):
    """`calls` whole-stream scans of s on a fresh engine, each against the oracle; the paths."""
    from mgen_amd import Engine, to_device
    from oracle import oracle as O
    wo, wl, _, wc, ws = O.tcp_scan(s.tobytes())
    e = Engine(0)
    d = to_device(s)
    paths = []
    try:
        for k in range(calls):
            offs, lens, info = e.stream_scan(d, mode)
            assert np.array_equal(offs.cpu().numpy().view(np.uint64), np.asarray(wo, np.uint64)), k
            assert np.array_equal(lens.cpu().numpy().view(np.uint32), np.asarray(wl, np.uint32)), k
            assert (int(info.consumed), int(info.status)) == (wc, ws), k
            paths.append(int(info.path))
    finally:
        e.close()
    return paths


def test_chain_dense_small_records(torch, gold):
    """~64K records of 28..200 B (thousands of candidates per detect block group): the chain
    groups hold more than kChainCands candidates, the hypothesis is not proved there and the
    exact path frames the stream -- every call equals the oracle."""
    rng = np.random.default_rng(SEED + 80)
    s = tcp_stream(gold, rng.integers(76, 200, 40000), rng)
    paths = _scan_calls(torch, s, 4)
    assert paths[0] == 0


def test_chain_bad_record_mid_stream(torch, gold):
    """A config-5-like stream (16-KiB TCP transmit records) with one record's length field
    broken in the middle: the second call's chain check fails (or proves a shorter chain) and
    the framing still equals the oracle's -- the zero-length error stops it there."""
    from mgen_amd import Engine
    e = Engine(0)
    try:
        st = _tcp_tx_stream(torch, e, 512)
    finally:
        e.close()
    s = st.cpu().numpy().copy()
    k = 300 * 16384
    s[k] = 0
    s[k + 1] = 2  # msg_len 2 < 4: the reference's stream error
    paths = _scan_calls(torch, s, 3)
    assert paths[0] == 0


def test_chain_junk_tail_after_valid_records(torch, gold):
    """Valid 16-KiB transmit records followed by 100 KiB of random bytes: the chain from 0 ends
    at the junk, the resolver walks the rest exactly, on the chain path's second call too."""
    from mgen_amd import Engine
    e = Engine(0)
    try:
        st = _tcp_tx_stream(torch, e, 256)
    finally:
        e.close()
    rng = np.random.default_rng(SEED + 81)
    s = np.concatenate([st.cpu().numpy(), rng.integers(0, 256, 100 * 1024, dtype=np.uint8)])
    _scan_calls(torch, s, 3)


def test_chain_streams_alternate(torch, gold):
    """One engine scanning two different transmit streams in turn (the chain path's epochs and
    group summaries are reused across scans): each call equals the oracle for its stream."""
    from mgen_amd import Engine, SCAN_TCP
    from oracle import oracle as O
    e = Engine(0)
    try:
        a = _tcp_tx_stream(torch, e, 384)
        b = _tcp_tx_stream(torch, e, 200, msg=20480)
        want = {}
        for name, st in (("a", a), ("b", b)):
            wo, wl, _, wc, ws = O.tcp_scan(st.cpu().numpy().tobytes())
            want[name] = (np.asarray(wo, np.uint64), wc, ws)
        paths = []
        for k in range(6):
            name, st = ("a", a) if k % 2 == 0 else ("b", b)
            offs, lens, info = e.stream_scan(st, SCAN_TCP)
            wo, wc, ws = want[name]
            assert np.array_equal(offs.cpu().numpy().view(np.uint64), wo), k
            assert (int(info.consumed), int(info.status)) == (wc, ws), k
            paths.append(int(info.path))
        assert 2 in paths, paths
    finally:
        e.close()
