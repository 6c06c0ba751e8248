"""GPU: the C++ sharded framing (mgenx::ShardedScan, include/mgenx.hpp) -- the stitch
protocol of mgen_amd/shard.py in the host layer an MGEN transport links -- run by
tests/cpp/shard_scan with 2 / 3 / 5 simulated ranks (threads, one context each) and with one
rank over a real RCCL communicator (RcclShardComm): the union of the ranks' records and every
rank's summary equal one mgenx_stream_scan of the whole stream, on every corpus case
(valid, truncated, bad version bytes, a TCP error, SINK garbage, random bytes) and on config
5's shape.  Reference framing: src/common/mgenTransport.cpp:1683-1760,
src/common/mgenAppSinkTransport.cpp:369-434."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "shard_scan")


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available()
    from mgen_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def _run(tmp_path, s, mode, world):
    f = tmp_path / "stream.bin"
    o = tmp_path / "out.bin"
    f.write_bytes(np.ascontiguousarray(s, np.uint8).tobytes())
    p = subprocess.run([BIN, str(f), str(mode), str(world), str(o)], capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    raw = o.read_bytes()
    n = int(np.frombuffer(raw[:8], np.uint64)[0])
    offs = np.frombuffer(raw[8:8 + 8 * n], np.uint64).astype(np.int64)
    lens = np.frombuffer(raw[8 + 8 * n:8 + 12 * n], np.uint32).astype(np.int32)
    summ = np.frombuffer(raw[8 + 12 * n:], np.uint64).reshape(world, 3)
    return offs, lens, [tuple(int(x) for x in row) for row in summ]


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_cpp_sharded_scan_equals_whole(eng, tmp_path, world):
    from mgen_amd import to_device
    from streams import corpus
    for name, s, mode in corpus():
        offs, lens, info = eng.stream_scan(to_device(s), mode)
        want = (int(info.n_records), int(info.consumed), int(info.status))
        go, gl, summ = _run(tmp_path, s, mode, world)
        assert np.array_equal(go, offs.cpu().numpy()), (name, world)
        assert np.array_equal(gl, lens.cpu().numpy()), (name, world)
        assert all(x == want for x in summ), (name, world, summ, want)


def test_cpp_sharded_scan_config5_shape(eng, tmp_path):
    """16-KiB TCP records (checksum on) over a 64 MiB stream in 4 shards."""
    from streams import golden, tcp_stream
    n = 4096
    s = tcp_stream(golden(), np.full(n, 16384), np.random.default_rng(55))
    go, gl, summ = _run(tmp_path, s, 0, 4)
    assert np.array_equal(go, np.arange(n) * 16384) and np.all(gl == 16384)
    assert all(x == (n, len(s), 0) for x in summ)
