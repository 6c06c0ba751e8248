"""Synthetic TCP / SINK byte streams for the framing tests, built with the oracle's
restatement of the reference's TX path (test infrastructure)."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def golden():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "udp_matrix.npz"),
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


def corpus(seed=0x5348):
    """(name, stream, mode) cases covering the protocol's paths: valid streams, records
    longer than a shard, bad version bytes (chains leave the candidate set), a TCP error,
    SINK garbage, a truncated tail, random bytes."""
    from oracle import oracle as O
    gold = golden()
    rng = np.random.default_rng(seed)
    out = []
    s = tcp_stream(gold, rng.integers(76, 40000, 40), rng)
    out.append(("tcp_mixed", s, 0))
    out.append(("tcp_truncated", s[:-777], 0))
    bad = s.copy()
    offs = O.tcp_scan(bad.tobytes())[0]
    for k in (0, 5, 11, 12, 30):
        bad[int(offs[k]) + 2] = 7
    out.append(("tcp_bad_version", bad, 0))
    err = bad.copy()
    err[int(offs[25])], err[int(offs[25]) + 1] = 0, 3
    out.append(("tcp_error", err, 0))
    out.append(("tcp_small", tcp_stream(gold, rng.integers(76, 300, 1500), rng), 0))
    out.append(("sink_garbage", sink_stream(gold, rng.integers(28, 8193, 120), rng,
                                            garbage_every=5), 1))
    out.append(("random", rng.integers(0, 256, 200_000, dtype=np.uint8), 0))
    return out
