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
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return dict(np.load(os.path.join(root, "tests", "golden", "udp_matrix.npz"),
                        allow_pickle=False))


def _desc(gold, n, rng):
    d = np.zeros(n, gold["desc"].dtype)
    d["tmpl"] = rng.integers(0, len(gold["tmpl"]), n)
    d["seq_num"] = np.arange(n)
    d["tx_sec"] = 1_700_000_000
    d["tx_usec"] = rng.integers(0, 1_000_000, n)
    d["flags"] = 4
    return d


def tcp_stream(gold, sizes, rng, checksum=True):
    from oracle import oracle as O
    d = _desc(gold, len(sizes), rng)
    d["msg_len"] = np.minimum(sizes, 65535)
    return np.asarray(O.tcp_tx_batch(gold["tmpl"], d, np.asarray(sizes, np.uint32), gold["pool"],
                                      checksum=checksum), np.uint8)


def sink_stream(gold, sizes, rng, garbage_every=0):
    """UDP-packed records back to back (the SINK framing input), optionally with short runs
    of bytes whose length field is invalid (resynchronisation)."""
    from oracle import oracle as O
    d = _desc(gold, len(sizes), rng)
    d["msg_len"] = sizes
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    slab, lens = O.udp_pack_batch(gold["tmpl"], d, gold["pool"], int(np.sum(sizes)),
                                  rec_off=offs, checksum=True)
    parts = []
    for i, (o, s) in enumerate(zip(offs, sizes)):
        if garbage_every and i % garbage_every == 3:
            parts.append(np.array([0x00, 0x05, 0xAB, 0xFF, 0x7F, 0xFF][: 2 * (1 + i % 3)],
                                  np.uint8))
        if lens[i]:
            parts.append(slab[int(o):int(o) + int(lens[i])])
    return np.concatenate(parts)


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
    """A stream of 0x02 bytes makes every position plausible (slot overflow): the scan
    falls back to the sequential resolver and still matches."""
    s = np.full(200_000, 2, np.uint8)
    info = check(torch, eng, s, mode)
    assert info.candidates == 0


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
