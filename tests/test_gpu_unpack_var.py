"""GPU parity for unpack_var_kernel -- the kernel config 3's unpack runs (per-record lengths,
at least two 64-record tiles per wave: n >= 524,288 on a 256-CU part).

Config 3 exactly: 1,048,576 records of sizes U{64..1472} packed back to back, built by the
oracle's UDP send sequence over every golden template layout (IPv4/IPv6 dst, host address,
DATA payloads that fit and that do not), checksum on and off mixed per record, then
corrupted: bit flips anywhere, bad version bytes, bad dst types.  Every core field of every
record is compared with the oracle's MgenUdpTransport receive path (Unpack + CRC check,
src/common/mgenMsg.cpp:315-500, src/common/mgenTransport.cpp:960-975) under the UDP, forced
and TCP receive rules, for the row and the column outputs, and the dispatch is checked to
have launched the var kernel (mgenx_unpack_last_kernel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 20

CORE = [
    ("flow_id", np.uint32), ("seq_num", np.uint32), ("tx_sec", np.uint32),
    ("tx_usec", np.uint32), ("msg_len", np.uint16), ("dst_port", np.uint16),
    ("flags", np.uint8), ("err", np.uint8), ("dst_type", np.uint8), ("dst_len", np.uint8),
    ("payload_len", np.uint16), ("payload_type", np.uint8), ("gps_status", np.uint8),
]
EXT = [("hdr_len", np.uint16), ("payload_off", np.uint32), ("host_port", np.uint16),
       ("host_type", np.uint8), ("host_len", np.uint8), ("lat_raw", np.uint32),
       ("lon_raw", np.uint32), ("alt", np.int32)]


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
def corpus(oracle):
    """(slab bytes, offsets, lengths, {mode: oracle fields}) of the corrupted config-3 batch."""
    import os
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gold = dict(np.load(os.path.join(ROOT, "tests", "golden", "udp_matrix.npz"),
                        allow_pickle=False))
    tmpl, pool = gold["tmpl"], gold["pool"]
    rng = np.random.default_rng(0xC3)
    sizes = rng.integers(64, 1473, N).astype(np.int64)
    offs = np.zeros(N, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1]).astype(np.uint64)
    total = int(offs[-1]) + int(sizes[-1])
    desc = np.zeros(N, gold["desc"].dtype)
    desc["tmpl"] = rng.integers(0, len(tmpl), N)
    desc["seq_num"] = rng.integers(0, 1 << 32, N, dtype=np.uint64).astype(np.uint32)
    desc["tx_sec"] = 1_700_000_000 + np.arange(N) // 1000
    desc["tx_usec"] = rng.integers(0, 1_000_000, N)
    desc["msg_len"] = sizes
    desc["flags"] = rng.choice([0, 4], N)
    a, _ = oracle.udp_pack_batch(tmpl, desc, pool, total, rec_off=offs, checksum=True)
    b, _ = oracle.udp_pack_batch(tmpl, desc, pool, total, rec_off=offs, checksum=False)
    ck = rng.random(N) < 0.7
    host = np.where(np.repeat(ck, sizes), a, b)
    del a, b
    flip = np.nonzero(rng.random(N) < 0.05)[0]
    pos = (rng.random(flip.size) * sizes[flip]).astype(np.int64)
    host[offs[flip].astype(np.int64) + pos] ^= (1 << rng.integers(0, 8, flip.size)).astype(np.uint8)
    ver = np.nonzero(rng.random(N) < 0.01)[0]
    host[offs[ver].astype(np.int64) + 2] = 3
    dst = np.nonzero(rng.random(N) < 0.01)[0]
    host[offs[dst].astype(np.int64) + 22] = rng.choice([0, 3, 255], dst.size).astype(np.uint8)
    lens = sizes.astype(np.uint32)
    fields = {}
    for mode, force, tcp in (("udp", False, False), ("udp_force", True, False),
                             ("tcp_force", True, True)):
        fields[mode] = oracle.udp_recv_batch(host, N, rec_off=offs, rec_len=lens, force=force,
                                             tcp=tcp, nthreads=16)
    # the corpus must exercise every outcome
    f = fields["udp"]
    for e in (0, 1, 2, 4):
        assert int((f["err"] == e).sum()) > 1000, e
    return host, offs, lens, fields


def _opts(mode):
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP
    return {"udp": 0, "udp_force": OPT_CHECKSUM_FORCE, "tcp_force": OPT_TCP | OPT_CHECKSUM_FORCE}[mode]


def _rows(rows, n):
    from mgen_amd import REC_DTYPE
    r = rows.cpu().numpy().view(REC_DTYPE)[:n]
    return {name: np.ascontiguousarray(r[name]) for name in REC_DTYPE.names}


def _check(got, f, n, what, fields=CORE):
    for name, dt in fields:
        g = np.asarray(got[name]).view(dt)[:n]
        w = f[name][:n].astype(dt)
        bad = np.nonzero(g != w)[0]
        assert bad.size == 0, (what, name, bad.size, bad[:8], g[bad[:4]], w[bad[:4]])
    g4 = np.asarray(got["dst_addr4"]).view(np.uint8).reshape(-1, 4)[:n]
    assert np.array_equal(g4, f["dst_addr"][:n, :4]), (what, "dst_addr4")


@pytest.mark.parametrize("n", [N, 600_001])
@pytest.mark.parametrize("mode", ["udp", "udp_force", "tcp_force"])
def test_var_kernel_config3_vs_oracle(torch, eng, corpus, mode, n):
    """Rows and core columns from unpack_var_kernel == the oracle, every record (n = 600,001:
    a partial last tile; its last record also straddles slab_bytes -> ERROR_OOB)."""
    from mgen_amd import ERROR_OOB, UNPACK_K_VAR, to_device
    host, offs, lens, fields = corpus
    f = fields[mode]
    end = int(offs[n - 1]) + int(lens[n - 1])
    cut = 0 if n == N else 100           # the last record runs past the slab: OOB
    slab = to_device(host[:end])
    d_off = to_device(offs[:n]).view(torch.int64)
    d_len = to_device(lens[:n]).view(torch.int32)
    live = n - (1 if cut else 0)
    rows = eng.alloc_rows(n)
    eng.unpack(slab, n, rec_off=d_off, rec_len=d_len, opts=_opts(mode), cols={"rows": rows},
               slab_bytes=end - cut)
    assert eng.last_unpack_kernel() == UNPACK_K_VAR
    r = _rows(rows, n)
    _check(r, f, live, (mode, n, "rows"))
    cols = eng.unpack(slab, n, rec_off=d_off, rec_len=d_len, opts=_opts(mode),
                      slab_bytes=end - cut)
    assert eng.last_unpack_kernel() == UNPACK_K_VAR
    c = {k: v.cpu().numpy() for k, v in cols.items()}
    _check(c, f, live, (mode, n, "cols"))
    if cut:
        assert r["err"][n - 1] == ERROR_OOB and c["err"][n - 1] == ERROR_OOB


def test_var_kernel_extended_columns(torch, eng, corpus):
    """The extended columns (header length, payload offset, host address, GPS words, the
    16-byte addresses) from the var kernel == the oracle, UDP rule."""
    from mgen_amd import UNPACK_K_VAR, to_device
    host, offs, lens, fields = corpus
    f = fields["udp"]
    slab = to_device(host)
    cols = eng.unpack(slab, N, rec_off=to_device(offs).view(torch.int64),
                      rec_len=to_device(lens).view(torch.int32), ext=True)
    assert eng.last_unpack_kernel() == UNPACK_K_VAR
    c = {k: v.cpu().numpy() for k, v in cols.items()}
    _check(c, f, N, "ext", CORE + EXT)
    assert np.array_equal(c["dst_addr"].reshape(-1, 16), f["dst_addr"])
    assert np.array_equal(c["host_addr"].reshape(-1, 16), f["host_addr"])


def test_small_batches_use_general_kernel(torch, eng, corpus):
    """Below two tiles per wave the dispatch keeps the general kernel (same results)."""
    from mgen_amd import UNPACK_K_GENERAL, to_device
    host, offs, lens, fields = corpus
    n = 100_000
    end = int(offs[n - 1]) + int(lens[n - 1])
    rows = eng.alloc_rows(n)
    eng.unpack(to_device(host[:end]), n, rec_off=to_device(offs[:n]).view(torch.int64),
               rec_len=to_device(lens[:n]).view(torch.int32), cols={"rows": rows})
    assert eng.last_unpack_kernel() == UNPACK_K_GENERAL
    _check(_rows(rows, n), fields["udp"], n, "general")
