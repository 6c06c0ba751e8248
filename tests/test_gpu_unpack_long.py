"""GPU parity of the long-record unpack (unpack_long_kernel: one wave per record, 1-KiB rows;
dispatched when the mean record length is >= 4 KiB, as in a TCP stream of 16-KiB messages)
against the oracle's Unpack + receive check (mgenMsg.cpp:315-500, mgenTransport.cpp:960-975,
1516-1564): long records of every length class mixed with the golden matrix's short and
corrupted ones, at unaligned offsets, under the UDP, forced and TCP rules; and fixed strides."""
import numpy as np
import pytest

from test_gpu_parity import GOLD, compare_cols

pytestmark = pytest.mark.gpu

LONG_SIZES = [4096, 4097, 4099, 5000, 8188, 8191, 8192, 8193, 8200, 12345, 16383, 16384,
              16385, 16400, 30000, 65535]


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


def _long_records(oracle, rng, k):
    """k packed records of 4 KiB .. 64 KiB: IPv4 / IPv6 destinations, host addresses, DATA
    payloads, checksum on or off, some with a flipped byte (a CRC mismatch)."""
    out = []
    for j in range(k):
        L = LONG_SIZES[j % len(LONG_SIZES)] if j < 2 * len(LONG_SIZES) else int(rng.integers(4096, 65536))
        ip6 = rng.random() < 0.3
        dst = ("6", bytes(range(1, 17)), 7000) if ip6 else ("4", bytes([10, 1, 2, 3]), 5000)
        host = ("4", bytes([192, 168, 0, 9]), 4000) if rng.random() < 0.3 else None
        pay = bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
        m = oracle.make_msg(msg_len=L, flow_id=int(rng.integers(1, 99)), seq=j,
                            tx_sec=1_700_000_000, tx_usec=j, dst=dst, host=host,
                            payload=pay if pay else None)
        rec = bytearray(oracle.udp_pack(m, checksum=bool(rng.random() < 0.85)))
        assert len(rec) == L
        if rng.random() < 0.2:
            rec[int(rng.integers(0, L))] ^= 0x40
        out.append(bytes(rec))
    return out


@pytest.mark.parametrize("mode", ["udp", "udp_force", "tcp_force", "tcp"])
def test_long_kernel_mixed_vs_oracle(torch, eng, oracle, mode):
    from mgen_amd import OPT_CHECKSUM_FORCE, OPT_TCP, UNPACK_K_LONG, to_device
    g = dict(np.load(GOLD, allow_pickle=False))
    rng = np.random.default_rng(11 + len(mode))
    shorts = [bytes(g["unpack_slab"][o:o + n]) for o, n in zip(g["unpack_offs"], g["unpack_lens"])]
    longs = _long_records(oracle, rng, 160)
    recs = shorts[::4] + longs
    order = rng.permutation(len(recs))
    recs = [recs[i] for i in order]
    n = len(recs)
    offs, lens, parts, pos = [], [], [], 0
    for r in recs:
        pad = int(rng.integers(0, 16))
        parts.append(bytes(pad))
        pos += pad
        offs.append(pos)
        lens.append(len(r))
        parts.append(r)
        pos += len(r)
    body = b"".join(parts)
    slab = np.zeros(max(len(body) + 64, 4096 * n + 64), np.uint8)   # mean >= 4 KiB: long kernel
    slab[:len(body)] = np.frombuffer(body, np.uint8)
    offs = np.asarray(offs, np.uint64)
    lens = np.asarray(lens, np.uint32)
    opts = {"udp": 0, "udp_force": OPT_CHECKSUM_FORCE, "tcp_force": OPT_TCP | OPT_CHECKSUM_FORCE,
            "tcp": OPT_TCP}[mode]
    cols = eng.unpack(to_device(slab), n, rec_off=to_device(offs).view(torch.int64),
                      rec_len=to_device(lens).view(torch.int32), opts=opts, ext=True)
    torch.cuda.synchronize()
    assert eng.last_unpack_kernel() == UNPACK_K_LONG
    want = oracle.udp_recv_batch(slab, n, rec_off=offs, rec_len=lens,
                                 force=bool(opts & OPT_CHECKSUM_FORCE), tcp=bool(opts & OPT_TCP))
    assert int((want["err"] == 2).sum()) > 10
    compare_cols(cols, want, n, mode)


@pytest.mark.parametrize("size,stride,rows", [(16384, 16384, False), (16384, 16384, True),
                                              (5000, 5008, False), (65535, 65552, True)])
def test_long_kernel_fixed_stride_vs_oracle(torch, eng, oracle, size, stride, rows):
    """Fixed-length long records (fixed_len >= 4 KiB) at a stride, columns or 32-B rows."""
    from mgen_amd import OPT_TCP, REC_DTYPE, UNPACK_K_LONG, to_device
    rng = np.random.default_rng(size)
    n = 300
    slab = np.zeros(n * stride + 64, np.uint8)
    for i in range(n):
        m = oracle.make_msg(msg_len=size, flow_id=i + 1, seq=i, tx_sec=1_700_000_000, tx_usec=i)
        r = bytearray(oracle.udp_pack(m, checksum=True))
        if i % 7 == 3:
            r[int(rng.integers(0, size))] ^= 1
        slab[i * stride:i * stride + size] = np.frombuffer(bytes(r), np.uint8)
    d = to_device(slab)
    if rows:
        out = {"rows": eng.alloc_rows(n)}
        eng.unpack(d, n, stride=stride, fixed_len=size, opts=OPT_TCP, cols=out)
    else:
        out = eng.unpack(d, n, stride=stride, fixed_len=size, opts=OPT_TCP, ext=True)
    torch.cuda.synchronize()
    assert eng.last_unpack_kernel() == UNPACK_K_LONG
    want = oracle.udp_recv_batch(slab, n, stride=stride, fixed_len=size, tcp=True)
    assert int((want["err"] == 2).sum()) > 10
    if rows:
        r = out["rows"].cpu().numpy().view(REC_DTYPE)
        for key, wk in (("flow_id", "flow_id"), ("seq_num", "seq_num"), ("msg_len", "msg_len"),
                        ("err", "err"), ("flags", "flags"), ("tx_usec", "tx_usec")):
            assert np.array_equal(r[key].astype(np.int64), want[wk].astype(np.int64)), key
    else:
        compare_cols(out, want, n, f"stride {stride}")
