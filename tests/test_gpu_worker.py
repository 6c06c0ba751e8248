"""GPU: the resident single-message worker (mgenx_worker_*) -- MgenMsg::Unpack and
ComputeCRC32 of one host message per call, served by a wave kept on the device.  Parity:
every unpack vector of the golden matrix equals the batch kernels' decode of the same bytes
(mgenx_unpack_batch, MGENX_OPT_SKIP_CRC: Unpack alone, every column); CRC-32 running states
equal zlib's; the wave's idle exit and relaunch keep answering."""
import os
import time
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "udp_matrix.npz")


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


FIELDS = ("flow_id", "seq_num", "tx_sec", "tx_usec", "msg_len", "dst_port", "payload_len",
          "hdr_len", "host_port", "flags", "err", "dst_type", "dst_len", "payload_type",
          "gps_status", "host_type", "host_len", "decoded", "lat_raw", "lon_raw", "alt",
          "payload_off")


def test_worker_unpack_equals_batch_on_golden_matrix(torch, eng):
    from mgen_amd import OPT_SKIP_CRC
    g = dict(np.load(GOLD, allow_pickle=False))
    slab, offs, lens = g["unpack_slab"], g["unpack_offs"], g["unpack_lens"]
    n = len(offs)
    d = torch.from_numpy(slab.copy()).cuda()
    cols = eng.unpack(d, n, rec_off=torch.from_numpy(offs.view(np.int64).copy()).cuda(),
                      rec_len=torch.from_numpy(lens.view(np.int32).copy()).cuda(),
                      opts=OPT_SKIP_CRC, ext=True)
    torch.cuda.synchronize()
    from mgen_amd import UNPACKED_DTYPE
    # the batch columns as the worker's field types (same widths, unsigned where it is)
    want = {k: cols[k].cpu().numpy().view(UNPACKED_DTYPE[k]) for k in FIELDS}
    want["dst_addr"] = cols["dst_addr"].cpu().numpy()
    want["host_addr"] = cols["host_addr"].cpu().numpy()
    w = eng.worker()
    try:
        for i in range(n):
            msg = slab[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
            u = w.unpack(msg)
            for k in FIELDS:
                assert u[k] == want[k][i], (i, k, u[k], want[k][i])
            da = want["dst_addr"].reshape(n, 16)[i]
            ha = want["host_addr"].reshape(n, 16)[i]
            assert bytes(u["dst_addr"]) == da.tobytes(), i
            assert bytes(u["host_addr"]) == ha.tobytes(), i
    finally:
        w.close()


def _crc_state(data: bytes, state: int) -> int:
    """MgenMsg::ComputeCRC32(checksum, buf, len) (mgenMsg.cpp:524-541) through zlib: the
    running register starts from ~0 when checksum == 0, and is not finally inverted."""
    v = zlib.crc32(data, (~state) & 0xFFFFFFFF if state else 0)
    return (~v) & 0xFFFFFFFF


def test_worker_crc32_vs_zlib(torch, eng):
    rng = np.random.default_rng(7)
    w = eng.worker()
    try:
        for L in (0, 1, 3, 4, 15, 16, 17, 63, 64, 65, 1020, 1024, 8188, 8192, 16383, 16384,
                  16385, 40000, 65535, 65536):
            data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            for st in (0, int(rng.integers(1, 1 << 32))):
                assert w.crc32(data, st) == _crc_state(data, st), (L, st)
    finally:
        w.close()


def test_worker_idle_exit_and_relaunch(torch, eng):
    """A wave with a 2 ms idle timeout ends between calls; the next call relaunches it and is
    answered correctly, many times over, with unpack and crc32 interleaved."""
    g = dict(np.load(GOLD, allow_pickle=False))
    slab, offs, lens = g["unpack_slab"], g["unpack_offs"], g["unpack_lens"]
    w = eng.worker(idle_ms=2)
    try:
        first = None
        for k in range(12):
            msg = slab[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
            u = w.unpack(msg)
            if first is None:
                first = (k, u.copy())
            assert w.crc32(msg, 0) == _crc_state(msg, 0)
            time.sleep(0.004 if k % 2 else 0.0)
        k, u0 = first
        msg = slab[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
        assert w.unpack(msg).tobytes() == u0.tobytes()
    finally:
        w.close()


def test_worker_latency_report(torch, eng):
    """Median per-call time of worker unpack / crc32 of a 1024-B record (printed; the bound
    is loose: the shim_latency program reports the numbers)."""
    from mgen_amd.workloads import udp_fixed
    from oracle import oracle as O
    tmpl, pool, desc = udp_fixed(4, 1024)
    slab, _ = O.udp_pack_batch(tmpl, desc, pool, 4 * 1024, stride=1024, checksum=True)
    msg = slab[:1024].tobytes()
    w = eng.worker()
    try:
        for _ in range(100):
            w.unpack(msg)
        ts = []
        for _ in range(2000):
            t = time.perf_counter()
            w.unpack(msg)
            ts.append(time.perf_counter() - t)
        tc = []
        for _ in range(2000):
            t = time.perf_counter()
            w.crc32(msg[:1020], 0)
            tc.append(time.perf_counter() - t)
        um, cm = np.median(ts) * 1e6, np.median(tc) * 1e6
        print(f"worker unpack median {um:.2f} us, crc32 median {cm:.2f} us (Python call included)")
        assert um < 200 and cm < 200
    finally:
        w.close()


def _long_header_records():
    """Records whose header runs past the worker's 180 polled bytes (dst_len / host_len bytes
    up to 255: Unpack does not bound them, mgenMsg.cpp:394-398, 425-431), so the worker reads
    them from the mailbox's data area; plus short and junk records around the boundary."""
    from mgen_amd.workloads import udp_fixed
    from oracle import oracle as O
    tmpl, pool, desc = udp_fixed(2, 1024)
    slab, _ = O.udp_pack_batch(tmpl, desc, pool, 2 * 1024, stride=1024, checksum=True)
    base = slab[:1024].copy()
    rng = np.random.default_rng(11)
    recs = []
    for dl in (4, 16, 100, 130, 150, 152, 153, 156, 157, 160, 200, 255):
        for hl in (0, 4, 16, 40, 255):
            r = base.copy()
            r[23] = dl
            r[24:24 + dl] = rng.integers(0, 256, dl, dtype=np.uint8)
            h = 24 + dl
            r[h:h + 2] = (5001 >> 8, 5001 & 255)
            r[h + 2] = 1 if hl in (4, 40) else 2
            r[h + 3] = hl
            r[h + 4:h + 4 + hl] = rng.integers(0, 256, hl, dtype=np.uint8)
            for L in (1024, min(1024, h + 4 + hl + 16), max(28, h + 10)):
                recs.append(r[:L].tobytes())
    for L in (0, 1, 27, 28, 29, 47, 48, 179, 180, 181, 183, 184):
        recs.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
    return recs


def test_worker_unpack_vs_oracle(torch, eng):
    """mgenx_worker_unpack straight against the oracle's Unpack alone (or_unpack: a fresh
    MgenMsg, Unpack(buf, len, false, false), no caller CRC -- mgenMsg.cpp:315-500) on every
    unpack vector of the golden matrix and on headers longer than the polled bytes."""
    from oracle import oracle as O
    g = dict(np.load(GOLD, allow_pickle=False))
    slab, offs, lens = g["unpack_slab"], g["unpack_offs"], g["unpack_lens"]
    msgs = [slab[int(o):int(o) + int(L)].tobytes() for o, L in zip(offs, lens)]
    longs = _long_header_records()
    # which records take the data-area path: the header (24 + dst + 4 + host + 16) past the
    # 180 bytes that travel with the doorbell
    def hdr_need(m):
        if len(m) < 24:
            return 0
        need = 24 + m[23]
        if need + 4 <= min(len(m), 180):
            need += 4 + m[need + 3] + 16
        else:
            need += 4
        return min(len(m), need)
    assert sum(hdr_need(m) > 180 for m in longs) >= 20
    w = eng.worker()
    try:
        for i, m in enumerate(msgs + longs):
            u = w.unpack(m)
            f = O.unpack(m)
            for k in FIELDS:
                if k == "decoded":
                    continue
                assert int(u[k]) == int(f[k]), (i, len(m), k, int(u[k]), int(f[k]))
            assert int(u["err"] == 0) == int(f["ok"]), i
            assert bytes(u["dst_addr"]) == f["dst_addr"].tobytes(), i
            assert bytes(u["host_addr"]) == f["host_addr"].tobytes(), i
    finally:
        w.close()


def test_worker_after_engine_close(torch):
    """mgenx_ctx_destroy stops and frees the workers made on it; their handles then refuse
    calls (MgenxError) and still free cleanly."""
    from mgen_amd import Engine, MgenxError
    e = Engine(0)
    w = e.worker(idle_ms=5000)
    msg = bytes(64)
    w.unpack(msg)
    e.close()
    with pytest.raises(MgenxError):
        w.unpack(msg)
    w.close()


def test_batch_growth_after_worker_call(torch):
    """A batch call that grows a workspace (hipFree) right after a worker call: the library ends
    the resident wave first, so the call does not wait out the wave's idle timeout (5 s here),
    and the next worker call relaunches it.  A device-wide synchronisation after
    mgenx_worker_stop does not wait either."""
    from mgen_amd import Engine
    from mgen_amd.workloads import poisson_flows
    e = Engine(0)
    try:
        w = e.worker(idle_ms=5000)
        msg = bytes(64)
        u0 = w.unpack(msg)
        d = poisson_flows(4096, 8)
        t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
        idx = torch.from_numpy((d["flow_id"] - 1).astype(np.uint32)).cuda()
        for n in (1024, 4096):  # the second call grows the flow-reduce workspace
            w.unpack(msg)
            t0 = time.perf_counter()
            flows = e.flow_init(8, 1.0)
            e.flow_reduce(flows, 8, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                          t["rx_sec"], t["rx_usec"], n=n)
            # (the stream alone: a device-wide synchronisation would wait for the live wave,
            # as mgenx.h says -- mgenx_worker_stop first)
            torch.cuda.current_stream().synchronize()
            assert time.perf_counter() - t0 < 2.0, n
        assert w.unpack(msg).tobytes() == u0.tobytes()
        w.stop()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 2.0
        w.close()
    finally:
        e.close()


@pytest.mark.parametrize("force", [False, True])
def test_worker_recv_vs_oracle(torch, eng, force):
    """mgenx_worker_recv = the UDP receive path (mgenTransport.cpp:958-975): Unpack, then
    ComputeCRC32(0, buf, len - 4) when forced or CHECKSUM is set, compared by the caller with the
    big-endian trailer -- against the oracle's or_udp_recv on every golden unpack vector
    (corrupted CRCs, every error class).  The checksum is returned exactly when the oracle
    computes one, and equals zlib's."""
    from oracle import oracle as O
    g = dict(np.load(GOLD, allow_pickle=False))
    slab, offs, lens = g["unpack_slab"], g["unpack_offs"], g["unpack_lens"]
    w = eng.worker()
    computed = 0
    try:
        for i, (o, L) in enumerate(zip(offs, lens)):
            m = slab[int(o):int(o) + int(L)].tobytes()
            u, crc = w.recv(m, force)
            f = O.udp_recv(m, force)
            ok = int(u["err"]) == 0
            due = ok and (force or (int(u["flags"]) & 0x04) != 0)
            assert (crc is not None) == due, i
            err = int(u["err"])
            if crc is not None:
                computed += 1
                assert crc == _crc_state(m[:-4], 0), i
                if (crc ^ 0xFFFFFFFF) != int.from_bytes(m[-4:], "big"):
                    err = 2  # ERROR_CHECKSUM, as the caller sets it (:970-974)
            assert err == int(f["err"]), (i, err, int(f["err"]))
            for k in ("flow_id", "seq_num", "msg_len", "flags", "hdr_len", "payload_len"):
                assert int(u[k]) == int(f[k]), (i, k)
    finally:
        w.close()
    assert computed > 100


def test_worker_flow_update_vs_oracle(torch, eng):
    """mgenx_worker_flow_update, one record per call, equals the oracle's Update over the same
    records (or_flow_reduce_batch): final states (mask, FP64 latency sum / min / max) and every
    report, on lossy, reordered, duplicated flows with mask restarts, sequence jumps and
    zero-length messages; records alternate between the worker and batch calls of
    mgenx_flow_reduce on the same state array."""
    from mgen_amd import FLOW_STATE_DTYPE
    from oracle import oracle as O
    d = _jumpy_flows_small()
    n_flows, window = 6, 0.05
    n = len(d["seq"])
    flows = eng.flow_init(n_flows, window)
    w = eng.worker()
    reps = [[] for _ in range(n_flows)]
    try:
        i = 0
        while i < n:
            if (i // 700) % 3 == 2:  # a stretch through the batch kernels
                j = min(n, i + 700)
                cols = {k: torch.from_numpy(np.ascontiguousarray(v[i:j])).cuda() for k, v in d.items()}
                idx = torch.from_numpy((d["flow_id"][i:j] - 1).astype(np.uint32)).cuda()
                per_flow = 64
                rp = torch.zeros(n_flows * per_flow * 96, dtype=torch.uint8, device="cuda")
                cnt = torch.zeros(n_flows, dtype=torch.int32, device="cuda")
                eng.flow_reduce(flows, n_flows, idx, cols["seq"], cols["tx_sec"], cols["tx_usec"],
                                cols["msg_len"], cols["rx_sec"], cols["rx_usec"], reports=rp,
                                per_flow=per_flow, report_count=cnt)
                torch.cuda.synchronize()
                from mgen_amd import FLOW_REPORT_DTYPE
                r = rp.cpu().numpy().view(FLOW_REPORT_DTYPE).reshape(n_flows, per_flow)
                c = cnt.cpu().numpy()
                for f in range(n_flows):
                    assert c[f] <= per_flow
                    reps[f].extend(r[f, :c[f]])
                i = j
                continue
            f = int(d["flow_id"][i]) - 1
            rep = w.flow_update(flows, f, int(d["seq"][i]), int(d["rx_sec"][i]),
                                int(d["rx_usec"][i]), int(d["msg_len"][i]), int(d["tx_sec"][i]),
                                int(d["tx_usec"][i]))
            if rep is not None:
                reps[f].append(rep)
            i += 1
        torch.cuda.synchronize()
    finally:
        w.close()
    st = flows.cpu().numpy().view(FLOW_STATE_DTYPE)
    of, orep, ocnt = O.flow_reduce_batch(n_flows, d["flow_id"] - 1, d["seq"], d["tx_sec"],
                                         d["tx_usec"], d["msg_len"], d["rx_sec"], d["rx_usec"],
                                         window=window, per_flow=4096)
    assert int(ocnt.sum()) > 20
    for f, a in enumerate(of):
        s = st[f]
        assert s["msg_count"] == a.msg_count and s["byte_count"] == a.byte_count, f
        assert s["dup_count"] == a.dup_msg_count and s["n_reports"] == a.n_reports, f
        assert s["seq_start"] == a.seq_start, f
        assert s["latency_sum"] == a.latency_sum, (f, s["latency_sum"], a.latency_sum)
        assert s["latency_min"] == a.latency_min and s["latency_max"] == a.latency_max, f
        assert s["mask_n"] == a.nset, f
        if a.nset:
            assert s["mask_first"] == a.first, f
            assert s["mask"].tobytes() == bytes(a.bits), f
        assert len(reps[f]) == int(ocnt[f]), f
        for k, r in enumerate(reps[f]):
            o = orep[f, k]
            for name in ("start_sec", "start_usec", "duration", "msg_count", "rate", "loss",
                         "latency_ave", "latency_min", "latency_max", "rx_sec", "rx_usec"):
                assert r[name] == o[name], (f, k, name, r[name], o[name])


def _jumpy_flows_small():
    """~4000 receive-order records over 6 flows: losses, duplicates, reordering, sequence jumps
    past the mask span and near 2^31, zero-length messages (tests/test_gpu_analytics.py's
    _jumpy_flows, smaller)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "gpu_analytics_helpers", os.path.join(ROOT, "tests", "test_gpu_analytics.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod._jumpy_flows(6, 700, seed=21)
