"""Generate the committed golden vectors (tests/golden/*.npz) with the oracle.

Edge matrix: record sizes across every Pack truncation boundary,
dst IPv4/IPv6, host none/IPv4/IPv6, payload none / DATA fits / DATA too big / odd-hex
DATA, checksum off/on, zero fill / RANDOM_FILL (time fixed), caller flags 0 / CHECKSUM
preset; records placed at unaligned slab offsets.  Unpack vectors add every error
class (version, length, dst type, flipped CRC byte, short receive length) and are
evaluated under the UDP, UDP+force and TCP+force receive rules.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mgen_amd._abi import DESC_DTYPE, TMPL_DTYPE, gps_raw, hex_payload  # noqa: E402

SIZES = [28, 29, 31, 32, 40, 44, 45, 46, 47, 48, 49, 51, 52, 53, 56, 57, 60, 64, 65, 76, 77,
         79, 80, 81, 95, 96, 97, 100, 127, 128, 129, 255, 256, 257, 1024, 1472]
BIG_SIZES = [4093, 8192]
PAYLOADS = [b"", hex_payload("fffeffff"), hex_payload("abc"),
            bytes(range(16)), bytes((i * 7 + 3) & 0xFF for i in range(200))]
FILL_TIME = 1_700_000_000


def build_inputs():
    pool = b"".join(PAYLOADS)
    poffs = np.cumsum([0] + [len(p) for p in PAYLOADS])[:-1]
    tmpls = []
    for dst6 in (False, True):
        for host in (None, "4", "6"):
            for pi, p in enumerate(PAYLOADS):
                t = np.zeros((), TMPL_DTYPE)
                t["flow_id"] = 1 + len(tmpls)
                if dst6:
                    t["dst_type"], t["dst_len"] = 2, 16
                    t["dst_addr"] = np.frombuffer(bytes.fromhex("fe80" + "00" * 12 + "1234"),
                                                  np.uint8)
                else:
                    t["dst_type"], t["dst_len"] = 1, 4
                    t["dst_addr"][:4] = [127, 0, 0, 1]
                t["dst_port"] = 5000 + len(tmpls)
                if host == "4":
                    t["host_type"], t["host_len"], t["host_port"] = 1, 4, 6001
                    t["host_addr"][:4] = [192, 168, 1, 77]
                elif host == "6":
                    t["host_type"], t["host_len"], t["host_port"] = 2, 16, 6002
                    t["host_addr"] = np.arange(16, dtype=np.uint8) + 0x20
                t["lat_raw"] = gps_raw(999.0)
                t["lon_raw"] = gps_raw(-12.5 + len(tmpls))
                t["alt"] = -999 + len(tmpls)
                t["gps_status"] = len(tmpls) % 3
                t["payload_type"] = 0
                if p:
                    t["has_payload"] = 1
                    t["payload_len"] = len(p)
                    t["payload_off"] = poffs[pi]
                tmpls.append(t)
    tmpl = np.array(tmpls, TMPL_DTYPE)
    descs = []
    for ti in range(len(tmpl)):
        sizes = SIZES + (BIG_SIZES if ti in (0, 7, 29) else [])
        for si, s in enumerate(sizes):
            for flags in (0, 4):
                d = np.zeros((), DESC_DTYPE)
                d["tmpl"] = ti
                d["seq_num"] = 1000 * ti + 2 * si + (flags >> 2)
                d["tx_sec"] = 1_700_000_000 + ti
                d["tx_usec"] = (si * 7919 + flags) % 1_000_000
                d["msg_len"] = s
                d["flags"] = flags
                descs.append(d)
    desc = np.array(descs, DESC_DTYPE)
    sizes = desc["msg_len"].astype(np.uint64)
    gaps = (np.arange(len(desc)) % 7).astype(np.uint64)  # unaligned placement
    offs = np.zeros(len(desc), np.uint64)
    offs[1:] = np.cumsum(sizes[:-1] + gaps[:-1])
    offs += 3
    slab_bytes = int(offs[-1] + sizes[-1] + 64)
    return tmpl, np.frombuffer(pool, np.uint8).copy(), desc, offs, slab_bytes


def corrupt_records(rec_bytes, rng):
    """Error-class variants: (bytes, recv_len) pairs."""
    out = []
    for r in rec_bytes:
        r = bytearray(r)
        L = len(r)
        k = rng.integers(0, 6)
        if k == 0 and L > 8:       # flipped payload/fill/CRC byte
            j = int(rng.integers(0, L))
            r[j] ^= 1 << int(rng.integers(0, 8))
        elif k == 1:               # bad version
            r[2] = 3
        elif k == 2:               # bad dst type
            r[22] = int(rng.choice([0, 3, 255]))
        elif k == 3:               # short receive length
            L = int(rng.integers(1, L))
        elif k == 4:               # trailer flipped
            r[-1] ^= 0x80
        out.append((bytes(r[:L]), L))
    return out


def main():
    from oracle import oracle as O
    tmpl, pool, desc, offs, slab_bytes = build_inputs()
    out = {"tmpl": tmpl, "pool": pool, "desc": desc, "offs": offs,
           "slab_bytes": np.array([slab_bytes], np.uint64), "fill_time": np.array([FILL_TIME])}
    for ck in (0, 1):
        for rf in (0, 1):
            slab, lens = O.udp_pack_batch(tmpl, desc, pool, slab_bytes, rec_off=offs,
                                          checksum=bool(ck), random_fill=bool(rf),
                                          fill_time=FILL_TIME)
            out[f"pack_slab_ck{ck}_rf{rf}"] = slab
            out[f"pack_lens_ck{ck}_rf{rf}"] = lens
    # unpack vectors: good records (ck1 rf0/rf1) + corrupted copies
    rng = np.random.default_rng(0x4D47454E)
    recs = []
    for rf in (0, 1):
        slab, lens = out[f"pack_slab_ck1_rf{rf}"], out[f"pack_lens_ck1_rf{rf}"]
        for i in range(len(desc)):
            if lens[i]:
                recs.append((slab[offs[i]:offs[i] + lens[i]].tobytes(), int(lens[i])))
    good = [r for r, _ in recs]
    recs += corrupt_records(good, rng)
    recs += [(bytes(rng.integers(0, 256, n, dtype=np.uint8)), n) for n in (0, 1, 4, 20, 27)]
    u_lens = np.array([L for _, L in recs], np.uint32)
    u_offs = np.zeros(len(recs), np.uint64)
    pad = (np.arange(len(recs)) % 5).astype(np.uint64)
    u_offs[1:] = np.cumsum(u_lens[:-1].astype(np.uint64) + pad[:-1])
    u_offs += 1
    u_slab = np.zeros(int(u_offs[-1] + u_lens[-1] + 64), np.uint8)
    for (b, L), o in zip(recs, u_offs):
        u_slab[o:o + L] = np.frombuffer(b, np.uint8)[:L]
    out.update({"unpack_slab": u_slab, "unpack_offs": u_offs, "unpack_lens": u_lens})
    for mode in ("udp", "udp_force"):
        out[f"unpack_fields_{mode}"] = O.udp_recv_batch(
            u_slab, len(recs), rec_off=u_offs, rec_len=u_lens, force=(mode == "udp_force"))
    # TCP per-record rules (Unpack sees min(L, 8192) bytes; CHECKSUM_ERROR flag)
    out["unpack_fields_tcp_force"] = O.udp_recv_batch(u_slab, len(recs), rec_off=u_offs,
                                                      rec_len=u_lens, force=True, tcp=True)
    np.savez_compressed(os.path.join(HERE, "udp_matrix.npz"), **out)
    print("records:", len(desc), "unpack vectors:", len(recs), "pack slab bytes:", slab_bytes)


if __name__ == "__main__":
    main()
