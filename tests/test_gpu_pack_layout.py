"""GPU pack over variable-length slab layouts against the oracle's batch pack: packed back to
back (the aligned-unit path with boundary units composed from two records), with gaps
and odd offsets (per-record units), and with failing records inside a packed run (the
fallback); bytes outside the records must stay untouched."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


PAYLOADS = ["00112233445566778899aabbccddeeff", "", "ab" * 100]


@pytest.mark.parametrize("layout", ["packed", "gaps", "packed_failing"])
@pytest.mark.parametrize("ck,rf,pay", [(1, 0, 0), (0, 0, 1), (1, 1, 2), (1, 0, 2)])
def test_pack_layouts_vs_oracle(torch, eng, oracle, layout, ck, rf, pay):
    from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL, to_device
    from mgen_amd.workloads import udp_mixed
    n = 3000
    tmpl, pool, desc, _, sizes = udp_mixed(n, 30, 1600, 7, payload_hex=PAYLOADS[pay],
                                           seed=n + ck + 2 * rf + 4 * pay)
    rng = np.random.default_rng(len(layout) + pay)
    sizes = sizes.astype(np.int64)
    if layout == "packed_failing":
        bad = rng.random(n) < 0.02
        sizes[bad] = rng.integers(1, 27, int(bad.sum()))     # Pack fails: nothing written
    desc["msg_len"] = sizes.astype(np.uint16)
    gap = rng.integers(0, 40, n) if layout == "gaps" else np.zeros(n, np.int64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1] + gap[:-1])
    offs += 3                                                # odd start
    total = int(offs[-1] + sizes[-1]) + 64
    ft = 1_700_000_123
    want, wlen = oracle.udp_pack_batch(tmpl, desc, pool, total, rec_off=offs, checksum=bool(ck),
                                       random_fill=bool(rf), fill_time=ft)
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    if rf:
        eng.set_fill_time(ft)
    slab = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    opts = (PACK_CHECKSUM if ck else 0) | (PACK_RANDOM_FILL if rf else 0)
    out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=to_device(offs).view(torch.int64),
                       opts=opts, fill_time=ft)
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    lens = out_len.cpu().numpy().view(np.uint32)
    assert np.array_equal(lens, wlen)
    if layout == "packed_failing":
        assert (lens == 0).sum() > 10
    cover = np.zeros(total, bool)
    for o, ln in zip(offs, lens):
        cover[int(o):int(o) + int(ln)] = True
    assert np.all(got[~cover] == 0xA5), np.nonzero(got[~cover] != 0xA5)[0][:5]
    bad = np.nonzero(cover & (got != want))[0]
    if bad.size:
        rec = np.searchsorted(offs, bad[0], side="right") - 1
        pytest.fail(f"{bad.size} bytes differ, first at {bad[0]} (record {rec}, size "
                    f"{sizes[rec]}, pos {bad[0] - offs[rec]})")


@pytest.mark.parametrize("ck", [1, 0])
def test_pack_packed_large_vs_oracle(torch, eng, oracle, ck):
    """Config 3's layout (records back to back, sizes U{64..1472}) at 262,144 records: the
    fill and the overwritten head / tail units of every wave, byte for byte, on two launches
    into fresh slabs (the overwrites rely on a wave's same-address store order)."""
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd.workloads import udp_mixed
    n = 262_144
    tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64,
                                              payload_hex="00112233445566778899aabbccddeeff")
    offs = offs.astype(np.uint64)
    total = int(offs[-1] + sizes[-1])
    want, wlen = oracle.udp_pack_batch(tmpl, desc, pool, total, rec_off=offs, checksum=bool(ck))
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    d_off = to_device(offs).view(torch.int64)
    for _ in range(2):
        slab = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
        out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=d_off,
                           opts=PACK_CHECKSUM if ck else 0)
        torch.cuda.synchronize()
        assert np.array_equal(out_len.cpu().numpy().view(np.uint32), wlen)
        got = slab.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (bad.size, bad[:5])


@pytest.mark.parametrize("n", [1, 3, 64, 65, 300, 1025, 5000])
@pytest.mark.parametrize("layout", ["stride", "packed"])
def test_pack_batch_counts_vs_oracle(torch, eng, oracle, n, layout):
    """Batch counts around the pack kernel's geometry (64-record batches, groups of 4
    batches per meta/store stage, partial last group): stride slots and back-to-back
    records, byte for byte with the oracle, bytes outside the records untouched."""
    from mgen_amd import PACK_CHECKSUM, to_device
    from mgen_amd.workloads import udp_fixed, udp_mixed
    if layout == "stride":
        tmpl, pool, desc = udp_fixed(n, 512)
        offs = np.arange(n, dtype=np.uint64) * 512
        sizes = np.full(n, 512, np.int64)
    else:
        tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 16, seed=n)
        offs = offs.astype(np.uint64)
    total = int(offs[-1] + sizes[-1]) + 32
    want, wlen = oracle.udp_pack_batch(tmpl, desc, pool, total, rec_off=offs, checksum=True)
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    slab = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    if layout == "stride":
        out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, stride=512, opts=PACK_CHECKSUM)
    else:
        out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab,
                           rec_off=to_device(offs).view(torch.int64), opts=PACK_CHECKSUM)
    torch.cuda.synchronize()
    assert np.array_equal(out_len.cpu().numpy().view(np.uint32), wlen)
    got = slab.cpu().numpy()
    end = int(offs[-1] + sizes[-1])
    assert np.array_equal(got[:end], want[:end])
    assert np.all(got[end:] == 0xA5)
