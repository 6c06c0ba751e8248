"""Pin the oracle (the CPU restatement) to the reference's own known-answer material.

The reference ships no tests or golden vectors; what it does hold:
  * the CRC-32 table text, src/common/mgenMsg.cpp:576-642 (read as text when present);
  * the decoded DATA example, doc/mgen.xml:2943-2950;
  * the wire diagram, doc/mgen.xml:4619-4839;
  * the header bytes of a 1024-B record recorded in SURVEY.md 8(a) (survey session probe);
  * libc's srand/rand, the RANDOM_FILL source (mgenMsg.cpp:277-292).
"""
import ctypes
import os
import re
import zlib

import numpy as np
import pytest

REF = "/root/reference"


def test_crc_check_value(oracle):
    # CRC-32/ISO-HDLC check value; the reference table (mgenMsg.cpp:576-642) is this CRC.
    assert oracle.crc32_update(0, b"123456789") ^ 0xFFFFFFFF == 0xCBF43926


def test_crc_matches_zlib_random(oracle):
    rng = np.random.default_rng(1)
    for n in [0, 1, 3, 4, 5, 63, 64, 65, 1020, 8188]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        if n == 0:
            continue
        assert oracle.crc32_update(0, data) ^ 0xFFFFFFFF == zlib.crc32(data)


def test_crc_reset_on_zero_quirk(oracle):
    # mgenMsg.cpp:530-533: a running value of exactly 0 restarts at CRC32_XINIT.
    a = oracle.crc32_update(0, b"")
    assert a == 0xFFFFFFFF
    assert oracle.crc32_update(0, b"abc") == oracle.crc32_update(0xFFFFFFFF, b"abc")


@pytest.mark.skipif(not os.path.exists(f"{REF}/src/common/mgenMsg.cpp"),
                    reason="reference sources not mounted (GPU box)")
def test_crc_table_equals_reference_text(oracle):
    text = open(f"{REF}/src/common/mgenMsg.cpp").read()
    body = text[text.index("CRC32_TABLE[256] ="):]
    vals = [int(v, 16) for v in re.findall(r"0x([0-9A-Fa-f]{8})L", body)[:256]]
    assert len(vals) == 256
    assert list(oracle.crc_table()) == vals


def test_glibc_rand_stream_matches_libc(oracle):
    libc = ctypes.CDLL("libc.so.6")
    for seed in [1, 0, 1700000000, 2**31 - 1]:
        libc.srand(seed)
        ref = bytes([libc.rand() & 0xFF for _ in range(3000)])
        assert oracle.glibc_rand_bytes(seed, 3000) == ref


def test_survey_recorded_header(oracle):
    # flow 1, seq 7, t=1700000000.123456, dst 127.0.0.1/5000, checksum on
    m = oracle.make_msg(msg_len=1024, flow_id=1, seq=7, tx_sec=1700000000, tx_usec=123456)
    rec = oracle.udp_pack(m, checksum=True)
    want = ("0400 02 0c 00000001 00000007 6553f100 0001e240 1388 01 04 7f000001 0000 00 00 "
            "04376820 04376820 fffffc19 00 00 0000").replace(" ", "")
    assert rec[:48].hex() == want
    assert len(rec) == 1024
    assert int.from_bytes(rec[-4:], "big") == zlib.crc32(rec[:-4])
    assert rec[48:-4] == bytes(1024 - 52)


def test_doc_data_example_decodes(oracle):
    # doc/mgen.xml:2938-2950: DATA [fffeffff], 1024-B UDP, logged as
    # size>1024 gps>INVALID,999.000000,999.000000,4294966297 data>4:FFFEFFFF
    payload = oracle.payload_from_hex("fffeffff")
    assert payload == bytes.fromhex("fffeffff")
    m = oracle.make_msg(msg_len=1024, flow_id=1, seq=0, tx_sec=1, tx_usec=618199,
                        payload=payload)
    rec = oracle.udp_pack(m, checksum=False)
    f = oracle.udp_recv(rec)
    assert f["ok"] == 1 and f["err"] == 0
    assert f["msg_len"] == 1024 and f["flow_id"] == 1 and f["seq_num"] == 0
    assert f["gps_status"] == 0                              # INVALID
    assert f["lat_raw"] / 60000.0 - 180.0 == 999.0
    assert f["lon_raw"] / 60000.0 - 180.0 == 999.0
    assert int(f["alt"]) & 0xFFFFFFFF == 4294966297
    assert f["payload_len"] == 4
    off = int(f["payload_off"])
    assert rec[off:off + 4].hex().upper() == "FFFEFFFF"
    assert f["dst_port"] == 5000 and bytes(f["dst_addr"][:4]) == bytes([127, 0, 0, 1])


def test_doc_wire_diagram_offsets(oracle):
    # doc/mgen.xml:4619-4680: messageSize, version, flags, flowId, seq, txSec, txUsec,
    # dstPort/dstAddrType/dstAddrLen, dstAddr, hostPort/type/len, lat, lon, alt, gpsStatus,
    # (code: payloadType, doc: reserved), payloadLen -- all big-endian.
    m = oracle.make_msg(msg_len=100, flow_id=0x11223344, seq=0x55667788, tx_sec=0x01020304,
                        tx_usec=0x0A0B0C0D, dst=("4", bytes([10, 1, 2, 3]), 0x1234),
                        host=("4", bytes([192, 168, 0, 9]), 0x4321), lat=0.0, lon=0.0, alt=7,
                        gps_status=2, payload_type=1, payload=b"\xAA\xBB")
    rec = oracle.udp_pack(m, checksum=False)
    assert rec[0:2] == (100).to_bytes(2, "big") and rec[2] == 2
    assert rec[4:8] == bytes.fromhex("11223344") and rec[8:12] == bytes.fromhex("55667788")
    assert rec[12:16] == bytes.fromhex("01020304") and rec[16:20] == bytes.fromhex("0a0b0c0d")
    assert rec[20:24] == bytes.fromhex("1234 01 04".replace(" ", ""))
    assert rec[24:28] == bytes([10, 1, 2, 3])
    assert rec[28:32] == bytes.fromhex("4321 01 04".replace(" ", ""))
    assert rec[32:36] == bytes([192, 168, 0, 9])
    assert rec[36:40] == (10800000).to_bytes(4, "big")      # (0 + 180) * 60000
    assert rec[44:48] == (7).to_bytes(4, "big") and rec[48] == 2
    assert rec[49] == 1 and rec[50:52] == (2).to_bytes(2, "big")
    assert rec[52:54] == b"\xAA\xBB" and rec[54:] == bytes(46)


def test_hex_payload_rules(oracle):
    from mgen_amd._abi import hex_payload
    for s in ["", "a", "ABC", "fffeffff", "zz12", "0", "123456789abcdef"]:
        assert oracle.payload_from_hex(s) == hex_payload(s), s
    assert oracle.payload_from_hex("abc") == bytes([0xAB, 0xC0])


def test_quantized_default_window(oracle):
    # MgenAnalytic ctor quantises DEFAULT_WINDOW = 1.0 (mgenAnalytic.cpp:8-16,621-642)
    assert abs(oracle.quantized_window(1.0) - 1.0112109525687343) < 1e-15


# doc/mgen.xml:3644-3662: "a TCP mgen message of size 66559 will be received and logged by the
# receiving node as two messages" -- the fragment rule of MgenTcpTransport::GetNextTxFragmentSize
# (mgenTransport.cpp:1960-1993: MAX_FRAG_SIZE 65535, MIN_FRAG_SIZE 76, mgenGlobals.h:76-78).
DOC_TCP_RECV = [
    "00:33:36.427143 RECV proto>TCP flow>1 seq>1 src>10.0.0.1/35056 dst>10.0.0.2/5000 "
    "sent>00:36:11.377105 size>65535 gps>INVALID,999.000000,999.000000,-999 flags>0x01",
    "00:33:36.427499 RECV proto>TCP flow>1 seq>1 src>10.0.0.1/35056 dst>10.0.0.1/5000 "
    "sent>00:36:11.380137 size>1024 gps>INVALID,999.000000,999.000000,-999 flags>0x02",
]
DOC_DAY = 1_700_000_000 - 1_700_000_000 % 86400


def doc_tcp_msg(oracle):
    """The doc's message: flow 1, seq 1, dst 10.0.0.2/5000, 66,559 bytes, sent 00:36:11.377105."""
    return oracle.make_msg(msg_len=66559, flow_id=1, seq=1, tx_sec=DOC_DAY + 36 * 60 + 11,
                           tx_usec=377105, dst=("4", bytes([10, 0, 0, 2]), 5000))


def doc_tcp_expected_lines():
    """The doc's RECV lines as this code prints them (code wins):
      * the line ends with the space the format leaves before "\\n" (mgenMsg.cpp:1090-1101);
      * `%ld` of the INT32 altitude prints 4294966297 on LP64 (doc/mgen.xml:2948 shows that
        value; the -999 of :3649 is a 32-bit-long build);
      * the second fragment carries the FIRST fragment's tx time and the message's dst: the
        per-fragment SetTxTime is commented out (mgenTransport.cpp:1902-1904) and every
        fragment is packed from the one tx_msg; the doc's 10.0.0.1 / .380137 are another build.
    """
    a, b = (ln.replace(",-999", ",4294966297") + " \n" for ln in DOC_TCP_RECV)
    b = b.replace("dst>10.0.0.1/5000", "dst>10.0.0.2/5000").replace(
        "sent>00:36:11.380137", "sent>00:36:11.377105")
    return [a, b]


def doc_tcp_recv_inputs(oracle, n):
    src = np.zeros(n, oracle.ADDR_DTYPE)
    src["type"], src["len"], src["port"] = 1, 4, 35056
    src["addr"][:, :4] = [10, 0, 0, 1]
    rx_sec = np.full(n, DOC_DAY + 33 * 60 + 36, np.uint32)
    rx_usec = np.array([427143, 427499][:n], np.uint32)
    return src, rx_sec, rx_usec


@pytest.mark.parametrize("checksum", [False, True])
def test_doc_tcp_fragment_example(oracle, checksum):
    """or_tcp_tx splits the 66,559-B message into a 65,535-B fragment (CONTINUES) and a 1,024-B
    one (END_OF_MSG), same flow and seq; the TCP framing scan recovers exactly those two
    records and the RECV log prints the doc's two lines (the SEND line: test_send_log_cpu)."""
    stream = oracle.tcp_tx(doc_tcp_msg(oracle), checksum=checksum)
    assert len(stream) == 66559
    assert int.from_bytes(stream[0:2], "big") == 65535
    assert int.from_bytes(stream[65535:65537], "big") == 1024
    f0, f1 = stream[3], stream[65535 + 3]
    ck = 0x04 if checksum else 0
    # wire flags: fragment 0 is packed without LAST_BUFFER (its 8-KiB buffers are re-sent),
    # fragment 1 fits one buffer: LAST_BUFFER set before its Pack (mgenTransport.cpp:1931)
    assert f0 == 0x01 | ck and f1 == 0x02 | 0x08 | ck
    for o in (0, 65535):
        assert stream[o + 4:o + 12] == (1).to_bytes(4, "big") + (1).to_bytes(4, "big")
    if checksum:  # CRC over the whole fragment but its trailer, re-sent buffers included
        for o, L in ((0, 65535), (65535, 1024)):
            rec = stream[o:o + L]
            assert int.from_bytes(rec[-4:], "big") == zlib.crc32(rec[:-4])
    offs, lens, f, consumed, st = oracle.tcp_scan(stream)
    assert list(offs) == [0, 65535] and list(lens) == [65535, 1024] and consumed == 66559
    assert list(f["err"]) == [0, 0] and list(f["seq_num"]) == [1, 1]
    assert [int(x) & 0x03 for x in f["flags"]] == [0x01, 0x02]
    src, rx_sec, rx_usec = doc_tcp_recv_inputs(oracle, 2)
    text = oracle.log_recv_text(f, np.frombuffer(stream, np.uint8), offs, src, rx_sec, rx_usec,
                                protocol=2).decode()
    assert text.splitlines(keepends=True) == doc_tcp_expected_lines()
