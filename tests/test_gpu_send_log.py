"""GPU parity of the SEND events (mgenx_log_send_text / _binary, MgenMsg::LogSendEvent)
against the oracle restatement: the golden pack matrix (every dst / host layout, truncated
and failing Packs -- which are never sent, so never logged), UDP / SINK / TCP forms, GMT and
epoch timestamps, byte-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = "tests/golden/udp_matrix.npz"


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
    return dict(np.load(os.path.join(root, GOLD), allow_pickle=False))


@pytest.mark.parametrize("protocol,opts,binary", [(1, 0, False), (3, 1, False), (2, 0, False),
                                                  (1, 0, True), (3, 0, True), (2, 0, True)])
def test_send_events_match_oracle(torch, eng, gold, oracle, protocol, opts, binary):
    from mgen_amd import PACK_CHECKSUM, to_device
    tmpl, desc, pool = gold["tmpl"], gold["desc"], gold["pool"]
    n = len(desc)
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    d_offs = to_device(gold["offs"]).view(torch.int64)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    slab = torch.zeros(int(gold["slab_bytes"][0]), dtype=torch.uint8, device="cuda")
    out_len = eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=d_offs, opts=PACK_CHECKSUM)
    rng = np.random.default_rng(protocol * 7 + opts)
    src_port = rng.integers(0, 65536, len(tmpl)).astype(np.uint16)
    msg_total = desc["msg_len"].astype(np.uint32)
    got, off = eng.log_send(d_tmpl, d_desc, n, src_port=to_device(src_port), out_len=out_len,
                            msg_total=to_device(msg_total), slab=slab, rec_off=d_offs,
                            protocol=protocol, opts=opts, binary=binary)
    got = got.cpu().numpy().tobytes()
    want = oracle.log_send_batch(tmpl, desc, pool, src_port, protocol=protocol, checksum=True,
                                 opts=opts, binary=binary)
    lens = out_len.cpu().numpy().view(np.uint32)
    assert 0 < int((lens == 0).sum()) < n          # failing Packs are in the matrix
    assert len(got) == len(want)
    if got != want:
        bad = next(i for i in range(len(got)) if got[i] != want[i])
        pytest.fail(f"first difference at byte {bad}: {got[max(0, bad - 60):bad + 40]!r} vs "
                    f"{want[max(0, bad - 60):bad + 40]!r}")
    if not binary:
        assert got.count(b"\n") == int((lens != 0).sum())
