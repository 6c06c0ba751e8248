"""The oracle's MgenMsg::LogSendEvent restatement against the reference's documented SEND
line (doc/mgen.xml:3661-3662, the TCP example, and the format at :3780-3784)."""
import numpy as np


def test_send_line_matches_doc_example(oracle):
    from mgen_amd._abi import DESC_DTYPE, TMPL_DTYPE
    t = np.zeros(1, TMPL_DTYPE)
    t["flow_id"], t["dst_type"], t["dst_len"], t["dst_port"] = 1, 1, 4, 5000
    t["dst_addr"][0, :4] = [10, 0, 0, 2]
    d = np.zeros(1, DESC_DTYPE)
    day = 1_700_000_000 - 1_700_000_000 % 86400
    d["seq_num"], d["tx_sec"], d["tx_usec"] = 1, day + 29 * 60 + 51, 396962
    line = oracle.log_send_text(t[0], d[0], 0, protocol=2, mgen_msg_len=66559).decode()
    # the code prints " size>%lu " before the optional host (mgenMsg.cpp:1221-1238): the
    # doc's paragraph drops that trailing space
    assert line == ("00:29:51.396962 SEND proto>TCP flow>1 seq>1 srcPort>0 dst>10.0.0.2/5000 "
                    "size>66559 \n")
    t["host_type"], t["host_len"], t["host_port"] = 2, 16, 4000
    t["host_addr"][0, 15] = 1
    d["msg_len"] = 1024
    line = oracle.log_send_text(t[0], d[0], 4001, protocol=1, opts=1).decode()
    assert line == (f"{day + 29 * 60 + 51}.396962 SEND proto>UDP flow>1 seq>1 srcPort>4001 "
                    "dst>10.0.0.2/5000 size>1024 host>::1/4000\n")


def test_send_binary_record_layout(oracle):
    from mgen_amd.workloads import udp_mixed
    tmpl, pool, desc, _, _ = udp_mixed(3, 100, 100, 1, payload_hex="0011")
    out = oracle.log_send_batch(tmpl, desc, pool, np.array([7], np.uint16), binary=True)
    # {SEND_EVENT 3, UDP, BE recordLength} + recordLength message bytes, CHECKSUM cleared
    rl = int.from_bytes(out[2:4], "big")
    assert out[0] == 3 and out[1] == 1 and len(out) == 3 * (4 + rl)
    assert rl == 12 + 4 + 48                       # IPv4 dst, 48-byte header, no host
    assert out[4 + 3] & 0x04 == 0 and out[4:6] == (100).to_bytes(2, "big")
