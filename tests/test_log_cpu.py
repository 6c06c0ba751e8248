"""CPU: the oracle's RECV/RERR log restatement (MgenMsg::LogRecvEvent / LogRecvError text
form, src/common/mgenMsg.cpp:711-735, 1034-1102) reproduces the reference's own printed
output -- the RECV lines quoted in doc/mgen.xml:2948-2949 -- byte for byte."""
import numpy as np

# doc/mgen.xml:2948 (the same line with XML entities decoded)
DOC_LINE = (b"19:39:06.618340 RECV proto>UDP flow>1 seq>0 src>127.0.0.1/59275 "
            b"dst>127.0.0.1/5000 sent>19:39:06.618199 size>1024 "
            b"gps>INVALID,999.000000,999.000000,4294966297 data>4:FFFEFFFF \n")
DAY = 1_699_920_000            # a UTC midnight
T = DAY + 19 * 3600 + 39 * 60 + 6


def _src(oracle, a=(127, 0, 0, 1), port=59275):
    s = np.zeros(1, oracle.ADDR_DTYPE)
    s["type"], s["len"], s["port"] = 1, len(a), port
    s["addr"][0, :len(a)] = a
    return s


def _record(oracle, **kw):
    from mgen_amd._abi import hex_payload
    args = dict(msg_len=1024, flow_id=1, seq=0, tx_sec=T, tx_usec=618199,
                dst=("4", bytes([127, 0, 0, 1]), 5000), lat=999.0, lon=999.0, alt=-999,
                gps_status=0, payload=hex_payload("fffeffff"))
    args.update(kw)
    m = oracle.make_msg(**args)
    return oracle.udp_pack(m, checksum=True)


def _log(oracle, rec, rx_usec=618340, **kw):
    f = oracle.udp_recv(rec)
    fields = np.array([f])
    slab = np.frombuffer(rec, np.uint8)
    return oracle.log_recv_text(fields, slab, [0], _src(oracle), [T], [rx_usec], **kw)


def test_doc_recv_line(oracle):
    assert _log(oracle, _record(oracle)) == DOC_LINE


def test_doc_second_line(oracle):
    rec = _record(oracle, seq=1, tx_sec=T + 1, tx_usec=619975)
    want = DOC_LINE.replace(b"seq>0", b"seq>1").replace(b"19:39:06.618340", b"19:39:07.620218")
    want = want.replace(b"sent>19:39:06.618199", b"sent>19:39:07.619975")
    f = oracle.udp_recv(rec)
    got = oracle.log_recv_text(np.array([f]), np.frombuffer(rec, np.uint8), [0],
                               _src(oracle), [T + 1], [620218])
    assert got == want


def test_rerr_line_on_checksum_error(oracle):
    rec = bytearray(_record(oracle))
    rec[100] ^= 1
    got = _log(oracle, bytes(rec))
    assert got == b"19:39:06.618340 RERR type>checksum src>127.0.0.1/59275\n"


def test_options_epoch_nodata_nogps(oracle):
    rec = _record(oracle)
    got = _log(oracle, rec, opts=oracle.LOG_EPOCH | oracle.LOG_NO_DATA | oracle.LOG_NO_GPS)
    assert got == (f"{T}.618340 RECV proto>UDP flow>1 seq>0 src>127.0.0.1/59275 "
                   f"dst>127.0.0.1/5000 sent>{T}.618199 size>1024 \n").encode()
