"""The sharded framing protocol (mgen_amd/shard.py) on CPU: the device side replaced by its
Python test double (tests/shard_ref.py), ranks as threads (ThreadComm) for world sizes 1-5
and as gloo processes for world size 2.  The union of the ranks' records must equal the
whole-stream framing of the oracle (or_tcp_scan / or_sink_scan)."""
import os
import threading

import numpy as np
import pytest
import torch.multiprocessing as mp

from shard_ref import RefScanner
from streams import corpus

CASES = corpus()


def whole(s, mode):
    from oracle import oracle as O
    if mode == 1:
        wo, wl, _, wc = O.sink_scan(s.tobytes())
        ws = 0
    else:
        wo, wl, _, wc, ws = O.tcp_scan(s.tobytes())
    return np.asarray(wo, np.int64), np.asarray(wl, np.int64), wc, ws


def run_rank(comm, s, mode):
    from mgen_amd.shard import scan_sharded, shard_bounds
    a, _, hi = shard_bounds(len(s), comm.world, comm.rank)
    local = s[a:hi].tobytes()
    offs, lens, summ = scan_sharded(RefScanner(local), comm, local, len(s), mode)
    offs = np.zeros(0, np.int64) if offs is None else np.asarray(offs, np.int64) + a
    lens = np.zeros(0, np.int64) if lens is None else np.asarray(lens, np.int64)
    return offs, lens, summ


def threaded(s, mode, world):
    from mgen_amd.shard import ThreadComm
    tc = ThreadComm(world)
    res = [None] * world
    err = []

    def go(r):
        try:
            res[r] = run_rank(tc.rank_view(r), s, mode)
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            tc._bar.abort()
    th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not err, err
    return res


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
def test_sharded_equals_whole_threads(case, world):
    _, s, mode = CASES[case]
    wo, wl, wc, ws = whole(s, mode)
    res = threaded(s, mode, world)
    go = np.concatenate([r[0] for r in res])
    gl = np.concatenate([r[1] for r in res])
    assert np.array_equal(go, wo)
    assert np.array_equal(gl, wl)
    for r in res:
        assert r[2] == (len(wo), wc, ws)


def test_stitch_settles_unknown_exits():
    """A table with an unknown exit, or without the entry, asks for that rank's range scan;
    a settled stop ends the chain."""
    from mgen_amd.shard import EXIT_CAP, NONE, UNKNOWN, stitch
    ent = np.full(EXIT_CAP, NONE, np.uint64)
    ext = np.full(EXIT_CAP, NONE, np.uint64)
    ent[:2] = (0, 10)
    ext[:2] = (1000, np.uint64(500) | UNKNOWN)
    t0 = np.stack([ent, ext])
    bounds = [(0, 1000), (1000, 2000), (2000, 3000)]
    e1 = np.full(EXIT_CAP, NONE, np.uint64)
    x1 = np.full(EXIT_CAP, NONE, np.uint64)
    e1[0], x1[0] = 0, 1010
    t1 = np.stack([e1, x1])
    entries, need = stitch([t0, t1, t1], bounds, {})
    assert entries == [0, 1000, 2010] and need is None
    t0[0][0] = 5                                  # entry 0 missing from rank 0's table
    entries, need = stitch([t0, t1, t1], bounds, {})
    assert need == 0
    entries, need = stitch([t0, t1, t1], bounds, {0: (1000, False)})
    assert entries == [0, 1000, 2010] and need is None
    entries, need = stitch([t0, t1, t1], bounds, {0: (700, True)})
    assert entries == [0, None, None] and need is None


WORLD = 2


def gloo_worker(rank, port, case, q):
    import torch.distributed as dist
    from mgen_amd.shard import TorchComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    _, s, mode = CASES[case]
    offs, lens, summ = run_rank(TorchComm(), s, mode)
    q.put((rank, offs.tobytes(), lens.tobytes(), summ))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [0, 2, 3, 5], ids=[CASES[i][0] for i in (0, 2, 3, 5)])
def test_sharded_gloo_world2(case):
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=gloo_worker, args=(r, port, case, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict()
    for _ in range(WORLD):
        r, o, ln, summ = q.get(timeout=180)
        got[r] = (np.frombuffer(o, np.int64), np.frombuffer(ln, np.int64), summ)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, s, mode = CASES[case]
    wo, wl, wc, ws = whole(s, mode)
    assert np.array_equal(np.concatenate([got[0][0], got[1][0]]), wo)
    assert np.array_equal(np.concatenate([got[0][1], got[1][1]]), wl)
    assert got[0][2] == got[1][2] == (len(wo), wc, ws)
