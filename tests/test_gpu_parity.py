"""GPU parity: the HIP path (through the C ABI) against the oracle's golden vectors, plus
size-independent properties at BASELINE.json's full sizes.  Bit-exact everywhere."""
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "udp_matrix.npz")

# GPU column -> (oracle field, numpy view dtype)
COLMAP = [
    ("flow_id", "flow_id", np.uint32), ("seq_num", "seq_num", np.uint32),
    ("tx_sec", "tx_sec", np.uint32), ("tx_usec", "tx_usec", np.uint32),
    ("msg_len", "msg_len", np.uint16), ("dst_port", "dst_port", np.uint16),
    ("flags", "flags", np.uint8), ("err", "err", np.uint8), ("dst_type", "dst_type", np.uint8),
    ("dst_len", "dst_len", np.uint8), ("payload_len", "payload_len", np.uint16),
    ("payload_type", "payload_type", np.uint8), ("gps_status", "gps_status", np.uint8),
    ("hdr_len", "hdr_len", np.uint16), ("payload_off", "payload_off", np.uint32),
    ("host_port", "host_port", np.uint16), ("host_type", "host_type", np.uint8),
    ("host_len", "host_len", np.uint8), ("lat_raw", "lat_raw", np.uint32),
    ("lon_raw", "lon_raw", np.uint32), ("alt", "alt", np.int32),
]


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
    return dict(np.load(GOLD, allow_pickle=False))


def dev(torch, a):
    from mgen_amd import to_device
    return to_device(np.asarray(a))


def host_cols(cols, n):
    out = {}
    for name, t in cols.items():
        a = t.cpu().numpy()
        out[name] = a
    return out


def compare_cols(cols, f, n, what):
    c = host_cols(cols, n)
    for gname, oname, dt in COLMAP:
        got = c[gname].view(dt)[:n]
        want = f[oname].astype(dt)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (what, gname, bad[:10], got[bad[:5]], want[bad[:5]])
    got4 = c["dst_addr4"].view(np.uint8).reshape(-1, 4)[:n]
    assert np.array_equal(got4, f["dst_addr"][:, :4]), (what, "dst_addr4")
    assert np.array_equal(c["dst_addr"].reshape(-1, 16)[:n], f["dst_addr"]), (what, "dst_addr")
    assert np.array_equal(c["host_addr"].reshape(-1, 16)[:n], f["host_addr"]), (what, "host_addr")


def test_unpack_matrix_all_receive_rules(torch, eng, gold):
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP
    n = len(gold["unpack_lens"])
    slab = dev(torch, gold["unpack_slab"]).view(torch.uint8)
    offs = dev(torch, gold["unpack_offs"]).view(torch.int64)
    lens = dev(torch, gold["unpack_lens"]).view(torch.int32)
    for mode, opts in (("udp", 0), ("udp_force", OPT_CHECKSUM_FORCE),
                       ("tcp_force", OPT_TCP | OPT_CHECKSUM_FORCE)):
        cols = eng.unpack(slab, n, rec_off=offs, rec_len=lens, opts=opts, ext=True)
        torch.cuda.synchronize()
        compare_cols(cols, gold[f"unpack_fields_{mode}"], n, mode)


def test_unpack_core_only_matches_ext(torch, eng, gold):
    """Core-column path (no extended pointers) decodes the same as the full path."""
    n = len(gold["unpack_lens"])
    slab = dev(torch, gold["unpack_slab"]).view(torch.uint8)
    offs = dev(torch, gold["unpack_offs"]).view(torch.int64)
    lens = dev(torch, gold["unpack_lens"]).view(torch.int32)
    a = host_cols(eng.unpack(slab, n, rec_off=offs, rec_len=lens, ext=False), n)
    f = gold["unpack_fields_udp"]
    for gname, oname, dt in COLMAP[:13]:
        assert np.array_equal(a[gname].view(dt)[:n], f[oname].astype(dt)), gname
    assert np.array_equal(a["dst_addr4"].view(np.uint8).reshape(-1, 4), f["dst_addr"][:, :4])


@pytest.mark.parametrize("ck,rf", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_pack_matrix(torch, eng, gold, ck, rf):
    from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL
    desc, tmpl = gold["desc"], gold["tmpl"]
    n = len(desc)
    d_tmpl = dev(torch, tmpl)
    d_pool = dev(torch, gold["pool"])
    d_desc = dev(torch, desc)
    d_offs = dev(torch, gold["offs"]).view(torch.int64)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    ft = int(gold["fill_time"][0])
    if rf:
        eng.set_fill_time(ft)
    slab = torch.zeros(int(gold["slab_bytes"][0]), dtype=torch.uint8, device="cuda")
    opts = (PACK_CHECKSUM if ck else 0) | (PACK_RANDOM_FILL if rf else 0)
    out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=d_offs, opts=opts,
                       fill_time=ft)
    torch.cuda.synchronize()
    want = gold[f"pack_slab_ck{ck}_rf{rf}"]
    got = slab.cpu().numpy()
    lens = out_len.cpu().numpy().view(np.uint32)
    assert np.array_equal(lens, gold[f"pack_lens_ck{ck}_rf{rf}"])
    bad = np.nonzero(got != want)[0]
    if bad.size:
        offs = gold["offs"]
        rec = np.searchsorted(offs, bad[0], side="right") - 1
        pytest.fail(f"pack mismatch ck={ck} rf={rf}: {bad.size} bytes, first at {bad[0]} "
                    f"(record {rec}, size {desc['msg_len'][rec]}, tmpl {desc['tmpl'][rec]}, "
                    f"pos {bad[0] - offs[rec]})")


def _config2(torch, eng, n, size=1024):
    from mgen_amd import PACK_CHECKSUM
    from mgen_amd.workloads import udp_fixed
    tmpl, pool, desc = udp_fixed(n, size)
    d_tmpl, d_pool, d_desc = dev(torch, tmpl), dev(torch, pool), dev(torch, desc)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    slab = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, stride=size, opts=PACK_CHECKSUM)
    return desc, slab, out_len


def test_config2_full_size_roundtrip(torch, eng):
    """1M x 1024-B UDP records: pack -> unpack recovers every descriptor; flipping one bit
    in sampled records is caught as ERROR_CHECKSUM exactly there (size-independent)."""
    n, size = 1 << 20, 1024
    desc, slab, out_len = _config2(torch, eng, n, size)
    assert int((out_len != size).sum()) == 0
    cols = eng.unpack(slab, n, stride=size, fixed_len=size)
    c = host_cols(cols, n)
    assert int(c["err"].astype(np.int64).sum()) == 0
    assert np.array_equal(c["seq_num"].view(np.uint32), desc["seq_num"])
    assert np.array_equal(c["flow_id"].view(np.uint32), desc["tmpl"] + 1)
    assert np.array_equal(c["tx_sec"].view(np.uint32), desc["tx_sec"])
    assert np.array_equal(c["tx_usec"].view(np.uint32), desc["tx_usec"])
    assert np.all(c["flags"] == 0x0C) and np.all(c["msg_len"].view(np.uint16) == size)
    # spot-check bytes against zlib for a few records
    host = slab[: 8 * size].cpu().numpy()
    for i in range(8):
        r = host[i * size:(i + 1) * size].tobytes()
        assert int.from_bytes(r[-4:], "big") == zlib.crc32(r[:-4])
    # corruption property
    rng = np.random.default_rng(7)
    victims = np.unique(rng.integers(0, n, 4096))
    pos = rng.integers(0, size, victims.size)
    bits = rng.integers(0, 8, victims.size)
    idx = torch.from_numpy((victims * size + pos).astype(np.int64)).cuda()
    flip = torch.from_numpy((1 << bits).astype(np.uint8)).cuda()
    slab[idx] ^= flip
    cols = eng.unpack(slab, n, stride=size, fixed_len=size)
    c = host_cols(cols, n)
    err = c["err"]
    # a flip in the version byte / dst type turns into that error instead
    # clearing the CHECKSUM flag bit (byte 3, bit 2) disables the check (mgenTransport.cpp:960)
    unchecked = (pos == 3) & (bits == 2)
    expect_bad = set(victims[~unchecked].tolist())
    assert set(np.nonzero(err != 0)[0].tolist()) == expect_bad
    assert np.all(err[victims[pos == 2]] == 1)          # version byte
    assert np.all(err[victims[pos == 22]] == 4)         # dst type byte
    crc_class = (pos != 2) & (pos != 22) & ~unchecked
    assert np.all(err[victims[crc_class]] == 2)


@pytest.mark.parametrize("size", [1024, 512])
def test_full_size_rows_ring_kernel(torch, eng, size):
    """The headline row-output kernel (unpack_fixed_ring_kernel: 8-row load ring, row output
    held per wave and stored in bursts) at full size, where every wave runs 16+ groups and
    bursts: rows == the column kernel's output field by field, with sampled bit flips and
    runs of groups whose CHECKSUM flag is cleared (the header-only mode and the switch back)."""
    n = (1 << 20) if size == 1024 else (3 << 19)
    desc, slab, out_len = _config2(torch, eng, n, size)
    assert int((out_len != size).sum()) == 0
    rng = np.random.default_rng(size)
    victims = np.unique(rng.integers(0, n, 8192))
    pos = rng.integers(0, size, victims.size)
    bits = rng.integers(0, 8, victims.size)
    idx = torch.from_numpy((victims * size + pos).astype(np.int64)).cuda()
    slab[idx] ^= torch.from_numpy((1 << bits).astype(np.uint8)).cuda()
    # groups (16 records) 1000..1299 and every 7th group after 5000: CHECKSUM flag cleared
    groups = np.concatenate([np.arange(1000, 1300), np.arange(5000, n // 16, 7)])
    recs = (groups[:, None] * 16 + np.arange(16)[None, :]).reshape(-1)
    flag_at = torch.from_numpy((recs * size + 3).astype(np.int64)).cuda()
    slab[flag_at] &= 0xFB
    from oracle import oracle as O
    cols = eng.unpack(slab, n, stride=size, fixed_len=size)
    c = host_cols(cols, n)
    rows = eng.alloc_rows(n)
    eng.unpack(slab, n, stride=size, fixed_len=size, cols={"rows": rows})
    from mgen_amd import UNPACK_K_FIXED_RING
    assert eng.last_unpack_kernel() == UNPACK_K_FIXED_RING   # the kernel under test ran
    torch.cuda.synchronize()
    r = rows_to_cols(rows, n)
    # every record the flips or the flag clears touched, against the oracle; the rest
    # against the descriptors they were packed from
    touched = np.unique(np.concatenate([victims, recs]))
    host = slab.cpu().numpy()
    sub = np.ascontiguousarray(host.reshape(n, size)[touched]).reshape(-1)
    f = O.udp_recv_batch(sub, touched.size, stride=size, fixed_len=size)
    for out, label in ((r, "rows"), (c, "cols")):
        for gname, oname, dt in COLMAP[:13]:
            got = out[gname].view(dt)[touched]
            want = f[oname].astype(dt)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (size, label, gname, touched[bad[:8]], got[bad[:4]], want[bad[:4]])
        rest = np.setdiff1d(np.arange(n), touched)
        assert np.all(out["err"][rest] == 0), label
        assert np.array_equal(out["seq_num"].view(np.uint32)[rest], desc["seq_num"][rest]), label
        assert np.array_equal(out["flow_id"].view(np.uint32)[rest], desc["tmpl"][rest] + 1), label
    assert (c["err"] == 2).sum() > 1000 and (c["flags"] & 0x04 == 0).sum() >= 16 * 300


def test_unpack_stride_matches_offsets(torch, eng):
    """Fixed-stride addressing == explicit offsets (same records)."""
    n, size = 4096, 256
    desc, slab, _ = _config2(torch, eng, n, size)
    a = host_cols(eng.unpack(slab, n, stride=size, fixed_len=size), n)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    b = host_cols(eng.unpack(slab, n, rec_off=offs, rec_len=lens), n)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_crc32_batch_vs_zlib(torch, eng):
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 100000, dtype=np.uint8)
    lens = rng.integers(0, 3000, 64).astype(np.uint32)
    offs = rng.integers(0, 100000 - 3000, 64).astype(np.uint64)
    out = eng.crc32(dev(torch, data), dev(torch, offs).view(torch.int64),
                    dev(torch, lens).view(torch.int32), 64)
    got = out.cpu().numpy().view(np.uint32)
    for i in range(64):
        assert got[i] == zlib.crc32(data[offs[i]:offs[i] + lens[i]].tobytes())


def test_oob_records_are_flagged_not_read(torch, eng):
    from mgen_amd import ERROR_OOB
    slab = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    offs = torch.tensor([0, 4000, 5000], dtype=torch.int64, device="cuda")
    lens = torch.tensor([64, 200, 10], dtype=torch.int32, device="cuda")
    c = host_cols(eng.unpack(slab, 3, rec_off=offs, rec_len=lens), 3)
    assert c["err"].tolist() == [1, ERROR_OOB, ERROR_OOB]


FIXED_SIZES = [65, 100, 127, 128, 200, 255, 256, 511, 777, 1000, 1023, 1024]


@pytest.mark.parametrize("out", ["cols", "rows"])
@pytest.mark.parametrize("size", FIXED_SIZES)
def test_fixed_len_pipelined_vs_oracle(torch, eng, gold, size, out):
    """The pipelined fixed-length kernel (fixed stride, one length, core columns) against the
    oracle: every golden template layout, checksum on/off and caller CHECKSUM flag mixed,
    bit flips / bad version / bad dst type, a partial last group and records past the end
    of the slab (ERROR_OOB), under the UDP, forced-UDP and TCP receive rules."""
    from mgen_amd import ERROR_OOB, OPT_CHECKSUM_FORCE, OPT_TCP
    from oracle import oracle as O
    tmpl, pool = gold["tmpl"], gold["pool"]
    n = 16 * 37 + 7
    rng = np.random.default_rng(size)
    desc = np.zeros(n, gold["desc"].dtype)
    desc["tmpl"] = rng.integers(0, len(tmpl), n)
    desc["seq_num"] = np.arange(n) * 3 + 1
    desc["tx_sec"] = 1_700_000_000 + np.arange(n) // 100
    desc["tx_usec"] = rng.integers(0, 1_000_000, n)
    desc["msg_len"] = size
    desc["flags"] = rng.choice([0, 4], n)
    a, _ = O.udp_pack_batch(tmpl, desc, pool, n * size, stride=size, checksum=True)
    b, _ = O.udp_pack_batch(tmpl, desc, pool, n * size, stride=size, checksum=False)
    recs = np.where((rng.random(n) < 0.7)[:, None], a.reshape(n, size), b.reshape(n, size))
    flip = np.nonzero(rng.random(n) < 0.1)[0]
    pos = rng.integers(0, size, flip.size)
    recs[flip, pos] ^= (1 << rng.integers(0, 8, flip.size)).astype(np.uint8)
    recs[rng.random(n) < 0.02, 2] = 3          # version
    recs[rng.random(n) < 0.02, 22] = 7         # dst type
    host = np.ascontiguousarray(recs).reshape(-1)
    n_oob = 3
    slab_bytes = (n - n_oob) * size + size // 2   # last record straddles the end
    slab = dev(torch, host).view(torch.uint8)
    for opts in (0, OPT_CHECKSUM_FORCE, OPT_TCP | OPT_CHECKSUM_FORCE):
        f = O.udp_recv_batch(host, n, stride=size, fixed_len=size,
                             force=bool(opts & OPT_CHECKSUM_FORCE), tcp=bool(opts & OPT_TCP))
        if out == "rows":  # mgenx_rec output (256/512/1024: the aligned kernel)
            rows = eng.alloc_rows(n)
            eng.unpack(slab, n, stride=size, fixed_len=size, opts=opts, slab_bytes=slab_bytes,
                       cols={"rows": rows})
            torch.cuda.synchronize()
            c = rows_to_cols(rows, n)
        else:
            cols = eng.unpack(slab, n, stride=size, fixed_len=size, opts=opts,
                              slab_bytes=slab_bytes)
            c = host_cols(cols, n)
        live = n - n_oob
        for gname, oname, dt in COLMAP[:13]:
            got = c[gname].view(dt)[:live]
            want = f[oname].astype(dt)[:live]
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (size, opts, gname, bad[:8], got[bad[:4]], want[bad[:4]])
        assert np.array_equal(c["dst_addr4"].view(np.uint8).reshape(-1, 4)[:live],
                              f["dst_addr"][:live, :4])
        assert np.all(c["err"][live:] == ERROR_OOB)
        assert np.all(c["msg_len"].view(np.uint16)[live:] == 0)


def rows_to_cols(rows, n):
    """mgenx_rec rows -> the core-column dict shape host_cols() returns."""
    from mgen_amd import REC_DTYPE
    r = rows.cpu().numpy().view(REC_DTYPE)[:n]
    out = {name: np.ascontiguousarray(r[name]) for name in REC_DTYPE.names}
    out["dst_addr4"] = np.ascontiguousarray(r["dst_addr4"])
    return out


@pytest.mark.parametrize("mode", ["udp", "udp_force", "tcp_force"])
def test_unpack_matrix_rows_output(torch, eng, gold, mode):
    """Row-major output (mgenx_rec) of the general kernel == the golden fields."""
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP
    opts = {"udp": 0, "udp_force": OPT_CHECKSUM_FORCE, "tcp_force": OPT_TCP | OPT_CHECKSUM_FORCE}
    n = len(gold["unpack_lens"])
    slab = dev(torch, gold["unpack_slab"]).view(torch.uint8)
    offs = dev(torch, gold["unpack_offs"]).view(torch.int64)
    lens = dev(torch, gold["unpack_lens"]).view(torch.int32)
    rows = eng.alloc_rows(n)
    eng.unpack(slab, n, rec_off=offs, rec_len=lens, opts=opts[mode], cols={"rows": rows})
    torch.cuda.synchronize()
    c = rows_to_cols(rows, n)
    f = gold[f"unpack_fields_{mode}"]
    for gname, oname, dt in COLMAP[:13]:
        got = c[gname].view(dt)
        want = f[oname].astype(dt)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, gname, bad[:10], got[bad[:5]], want[bad[:5]])
    assert np.array_equal(c["dst_addr4"].view(np.uint8).reshape(-1, 4), f["dst_addr"][:, :4])


@pytest.mark.parametrize("size", [65, 300, 1000, 1024])
def test_fixed_len_rows_output(torch, eng, gold, size):
    """Row-major output of the pipelined fixed-length kernel == its column output."""
    n = 16 * 29 + 5
    rng = np.random.default_rng(size + 7)
    from oracle import oracle as O
    desc = np.zeros(n, gold["desc"].dtype)
    desc["tmpl"] = rng.integers(0, len(gold["tmpl"]), n)
    desc["seq_num"] = np.arange(n)
    desc["msg_len"] = size
    desc["flags"] = 4
    a, _ = O.udp_pack_batch(gold["tmpl"], desc, gold["pool"], n * size, stride=size)
    a = a.copy()
    a[rng.integers(0, n * size, 50)] ^= 0x40
    slab = dev(torch, a).view(torch.uint8)
    sb = (n - 2) * size
    cols = eng.unpack(slab, n, stride=size, fixed_len=size, slab_bytes=sb)
    rows = eng.alloc_rows(n)
    eng.unpack(slab, n, stride=size, fixed_len=size, slab_bytes=sb, cols={"rows": rows})
    torch.cuda.synchronize()
    c = host_cols(cols, n)
    r = rows_to_cols(rows, n)
    for gname, _, dt in COLMAP[:13]:
        assert np.array_equal(c[gname].view(dt)[:n], r[gname].view(dt)), gname
    assert np.array_equal(c["dst_addr4"][:n], r["dst_addr4"])


def test_crc32_batch_long_ranges(torch, eng):
    """Ranges past the 65536-entry shift table (x^(8n) by square-and-multiply), unaligned
    starts and lengths not a multiple of 4 or 64."""
    rng = np.random.default_rng(31)
    data = rng.integers(0, 256, 3_000_000, dtype=np.uint8)
    lens = np.array([65535, 65536, 65537, 200_001, 1_048_579, 2_900_000, 63, 5], np.uint32)
    offs = np.array([1, 7, 100_003, 5, 333, 99_999, 2_999_000, 2_999_990], np.uint64)
    out = eng.crc32(dev(torch, data), dev(torch, offs).view(torch.int64),
                    dev(torch, lens).view(torch.int32), len(lens))
    got = out.cpu().numpy().view(np.uint32)
    for i in range(len(lens)):
        assert got[i] == zlib.crc32(data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()), i
