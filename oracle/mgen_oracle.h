/*
 * mgen_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference MGEN hot path (USNavalResearchLaboratory/mgen,
 * src/common/mgenMsg.cpp, mgenTransport.cpp, mgenAppSinkTransport.cpp,
 * mgenAnalytic.cpp).  Written from the reference's semantics, not copied.
 *
 * This is the CHECKER.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (libmgenx.so) never links it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - The reference cannot be built here: it needs the un-vendored protolib
 *     headers (protokit.h, protoDefs.h, protoPkt.h ...), which the image lacks.
 *   - Codec (pack/unpack/crc/framing): pinned by the reference's own known-answer
 *     material -- the CRC table text in src/common/mgenMsg.cpp:576-642 (checked
 *     against the generated table by a CPU test when /root/reference exists), the
 *     decoded DATA example in doc/mgen.xml:2943-2950 and the wire diagram in
 *     doc/mgen.xml:4619-4839 -- and by the header bytes recorded in SURVEY.md 8(a).
 *   - Analytics: parity UNPINNED at the protolib boundary (ProtoSlidingMask,
 *     ProtoTime are restated from their documented behaviour; no reference test or
 *     fixture covers them).
 */
#ifndef MGEN_ORACLE_H
#define MGEN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* include/mgenGlobals.h:70-80 */
enum { OR_MIN_SIZE = 28, OR_MAX_SIZE = 8192, OR_MSG_LEN_SIZE = 2, OR_TX_BUFFER_SIZE = 8192,
       OR_MAX_FRAG_SIZE = 65535, OR_MIN_FRAG_SIZE = 76 };
/* include/mgenMsg.h:60-103 */
enum { OR_VERSION = 2 };
enum { OR_ERROR_NONE = 0, OR_ERROR_VERSION = 1, OR_ERROR_CHECKSUM = 2, OR_ERROR_LENGTH = 3,
       OR_ERROR_DSTADDR = 4 };
enum { OR_FLAG_CONTINUES = 0x01, OR_FLAG_END_OF_MSG = 0x02, OR_FLAG_CHECKSUM = 0x04,
       OR_FLAG_LAST_BUFFER = 0x08, OR_FLAG_CHECKSUM_ERROR = 0x10 };
enum { OR_ADDR_INVALID = 0, OR_ADDR_IPV4 = 1, OR_ADDR_IPV6 = 2 };

typedef struct {
    uint8_t  type;      /* ProtoAddress type: 0 invalid, 1 IPv4, 2 IPv6 */
    uint8_t  len;       /* address length in bytes (4 / 16) */
    uint16_t port;
    uint8_t  addr[16];  /* network-order address bytes */
} or_addr;

/* The MgenMsg members that Pack() serialises (include/mgenMsg.h:207-235). */
typedef struct {
    uint16_t msg_len;
    uint32_t mgen_msg_len;
    uint8_t  version;
    uint8_t  flags;
    uint32_t flow_id, seq_num, tx_sec, tx_usec;
    or_addr  dst, host;
    double   latitude, longitude;
    int32_t  altitude;
    uint8_t  gps_status;
    uint8_t  payload_type;
    uint16_t payload_len;
    const uint8_t* payload_data;   /* NULL = no payload */
} or_msg;

/* MgenMsg state after Unpack() on a fresh MgenMsg (mgenMsg.cpp:315-500), in raw form. */
typedef struct {
    uint8_t  ok;            /* Unpack() return value */
    uint8_t  err;           /* MgenMsg::Error (caller may set ERROR_CHECKSUM) */
    uint8_t  version;
    uint8_t  flags;
    uint16_t msg_len;
    uint16_t hdr_len;       /* packet_header_len */
    uint32_t flow_id, seq_num, tx_sec, tx_usec;
    uint16_t dst_port;
    uint8_t  dst_type, dst_len;
    uint8_t  dst_addr[16];
    uint16_t host_port;
    uint8_t  host_type, host_len;
    uint8_t  host_addr[16];
    uint32_t lat_raw, lon_raw;   /* 10800000 (= 0.0 degrees) when not present */
    int32_t  alt;
    uint8_t  gps_status;
    uint8_t  payload_type;
    uint16_t payload_len;
    uint32_t payload_off;        /* byte offset of payload_data from record start */
} or_fields;

/* ---- CRC-32 (mgenMsg.cpp:524-554, table 576-642) ---- */
void     or_crc32_table(uint32_t table[256]);
void     or_crc32_update(uint32_t* checksum, const uint8_t* buf, uint32_t len);
int      or_write_checksum(uint32_t* tx_checksum, uint8_t* buf, uint32_t buflen);

/* ---- glibc TYPE_3 rand() restatement (RANDOM_FILL, mgenMsg.cpp:277-292) ---- */
void     or_glibc_rand_bytes(uint32_t seed, uint32_t n, uint8_t* out);

/* ---- Pack (mgenMsg.cpp:83-313) ----
 * Packs msg into buf (caller sizes buf >= max(bufferLen, 24+dst.len)).  msg->flags is
 * updated exactly as the member is.  random_fill != 0 selects the RANDOM_FILL build with
 * time(NULL) == fill_time.  Returns Pack()'s return value. */
uint16_t or_pack(or_msg* msg, uint8_t* buf, uint16_t bufferLen, int includeChecksum,
                 uint32_t* tx_checksum, int random_fill, uint32_t fill_time, uint16_t* hdr_len);

/* UDP / SINK transmit caller sequence (mgenTransport.cpp:1011-1031,
 * mgenAppSinkTransport.cpp:159-169): LAST_BUFFER, Pack, WriteChecksum if CHECKSUM.
 * Returns the record length (0 = MSG_SEND_FAILED). */
uint32_t or_udp_pack(const or_msg* msg, uint8_t* out, int checksum_enable, int random_fill,
                     uint32_t fill_time);

/* TCP transmit state machine (mgenTransport.cpp:1320-1400, 1762-1993) for one MgenMsg
 * with mgen_msg_len bytes, every socket Send() succeeding in full.  Writes the stream
 * bytes to out (capacity >= mgen_msg_len) and returns the bytes written. */
uint32_t or_tcp_tx(const or_msg* msg, uint8_t* out, int checksum_enable, int random_fill,
                   uint32_t fill_time);

/* ---- Unpack (mgenMsg.cpp:315-500) ---- */
void     or_unpack(const uint8_t* buf, uint32_t bufferLen, or_fields* f);
uint32_t or_unpack_persist(const uint8_t* buf, uint32_t bufferLen, or_fields* f);
void     or_tcp_rx_persist(const uint8_t* stream, const uint64_t* offs, const uint32_t* lens,
                           uint32_t n, int log_open, int checksum_force, or_fields* st,
                           uint32_t* pay_src, or_fields* out, uint32_t* payload_rec);

/* UDP receive (mgenTransport.cpp:958-975) / SINK HandleMgenMessage (2092-2112):
 * Unpack, then CRC over len-4 when forced or CHECKSUM is set. */
void     or_udp_recv(const uint8_t* rec, uint32_t len, int checksum_force, or_fields* f);

/* TCP per-record receive rules (CopyMsgBuffer :1996-2031, CalcRxChecksum :1516-1564):
 * Unpack sees min(L, 8192) bytes; CRC over L-4 vs the BE trailer when forced or CHECKSUM
 * is set; a mismatch sets ERROR_CHECKSUM and the CHECKSUM_ERROR flag. */
void     or_tcp_recv(const uint8_t* rec, uint32_t L, int checksum_force, or_fields* f);

/* TCP stream receive (mgenTransport.cpp:1194-1230, 1683-1760, 1996-2031, 1516-1564).
 * Returns the number of complete records; offsets/lengths/fields for the first `cap`.
 * *consumed = bytes of complete records; *status = 0 ok, 1 desync (msg_len < 4). */
uint32_t or_tcp_scan(const uint8_t* stream, uint64_t nbytes, int checksum_force,
                     uint64_t* offs, uint32_t* lens, or_fields* f, uint32_t cap,
                     uint64_t* consumed, int* status);

/* SINK stream receive (mgenAppSinkTransport.cpp:369-434 + HandleMgenMessage). */
uint32_t or_sink_scan(const uint8_t* stream, uint64_t nbytes, int checksum_force,
                      uint64_t* offs, uint32_t* lens, or_fields* f, uint32_t cap,
                      uint64_t* consumed);

/* ---- MgenPayload::SetPayloadString (mgenPayload.cpp:24-55, fromHex 127-166) ---- */
uint32_t or_payload_from_hex(const char* hex, uint8_t* out, uint32_t cap);

/* ---- MgenAnalytic (mgenAnalytic.cpp:28-258) over restated protolib primitives ---- */
typedef struct { int64_t sec; int64_t usec; } or_time;

typedef struct {
    /* ProtoSlidingMask restatement: set of u32 indices with span < depth */
    uint32_t depth;
    uint32_t first;          /* lowest set index (valid when nset > 0) */
    uint32_t nset;
    uint8_t  bits[1024 / 8]; /* bit i <-> index first + i */
    /* MgenAnalytic members */
    double   window_size;
    int      window_valid;
    or_time  window_start, window_end;
    uint32_t seq_start;
    uint64_t msg_count, byte_count, dup_msg_count;
    double   latency_sum, latency_min, latency_max;
    /* report */
    int      report_valid;
    uint64_t n_reports;
    or_time  report_start;
    double   report_duration;
    uint64_t report_msg_count;
    double   report_rate_ave, report_loss_ave, report_latency_ave, report_latency_min,
             report_latency_max;
} or_analytic;

double   or_quantized_window(double window);   /* Report::Quantize/UnquantizeTimeValue */
void     or_analytic_init(or_analytic* a, double window);
int      or_analytic_update(or_analytic* a, or_time rx, uint32_t msg_size, or_time tx,
                            uint32_t seq);
double   or_time_delta(or_time a, or_time b);

/* Batch analytics (Mgen::UpdateRecvAnalytics, mgen.cpp:1027-1070, over many flows):
 * records in rx order, flow_idx = dense flow index (>= n_flows: skipped); every closed
 * window is appended to reports[f * cap + k] (k < cap; counts[f] counts all). */
typedef struct {
    uint32_t flow, index;
    int64_t  start_sec, start_usec;
    double   duration;
    uint64_t msg_count;
    double   rate, loss, latency_ave, latency_min, latency_max;
    int64_t  rx_sec, rx_usec;
} or_report;
void or_flow_reduce_batch(or_analytic* flows, uint32_t n_flows, const uint32_t* flow_idx,
                          const uint32_t* seq, const uint32_t* tx_sec, const uint32_t* tx_usec,
                          const uint16_t* msg_len, const uint32_t* rx_sec,
                          const uint32_t* rx_usec, uint32_t n, or_report* reports,
                          uint32_t cap, uint32_t* counts);

/* ---- Batch layer (same descriptor layout as the product's include/mgenx.h) ---- */
/* Per-flow template: what MgenFlow::SendMessage fills from flow state
 * (mgenFlow.cpp:946-983, 1039-1129).  64 bytes. */
typedef struct {
    uint32_t flow_id;
    uint8_t  dst_type, dst_len; uint16_t dst_port;
    uint8_t  dst_addr[16];
    uint8_t  host_type, host_len; uint16_t host_port;   /* host_type 0 = invalid */
    uint8_t  host_addr[16];
    uint32_t lat_raw, lon_raw;    /* (UINT32)((deg + 180.0) * 60000.0), mgenMsg.cpp:221,225 */
    int32_t  alt;
    uint8_t  gps_status, payload_type; uint16_t payload_len;
    uint32_t payload_off;         /* offset into the payload pool */
    uint8_t  has_payload, rsv0; uint16_t rsv1;
} or_tmpl;

/* Per-record descriptor (20 bytes). */
typedef struct {
    uint32_t tmpl;                /* index into the template table */
    uint32_t seq_num, tx_sec, tx_usec;
    uint16_t msg_len;
    uint8_t  flags;               /* MgenMsg flags before the transport adds LAST_BUFFER */
    uint8_t  rsv;
} or_desc;

/* Pack n records with the UDP/SINK caller sequence.  rec_off[i] (or i*stride when
 * rec_off is NULL) gives the slab position; out_len[i] receives the length (0 = failed). */
void or_udp_pack_batch(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                       const uint8_t* pool, uint8_t* slab, const uint64_t* rec_off,
                       uint64_t stride, int checksum_enable, int random_fill, uint32_t fill_time,
                       uint32_t* out_len);

/* Receive over n records (rec_len NULL => fixed_len), nthreads host threads.
 * checksum_force bit 0 = force, bit 1 = TCP rules (or_tcp_recv) instead of UDP. */
void or_udp_recv_batch(const uint8_t* slab, const uint64_t* rec_off, uint64_t stride,
                       const uint32_t* rec_len, uint32_t fixed_len, uint32_t n,
                       int checksum_force, or_fields* out, int nthreads);

/* TCP transmit of n whole messages (desc[i].msg_len ignored; msg_total[i] bytes each)
 * back to back into stream; returns bytes written. */
uint64_t or_tcp_tx_batch(const or_tmpl* tmpl, const or_desc* desc, const uint32_t* msg_total,
                         uint32_t n, const uint8_t* pool, uint8_t* stream,
                         int checksum_enable, int random_fill, uint32_t fill_time);

uint32_t or_sizeof(int which);

/* ---- RECV / RERR text log lines (MgenMsg::LogRecvEvent / LogRecvError text form,
 * mgenMsg.cpp:711-735, 1034-1102; timestamps mgen.cpp:55-83).  f = the record after the
 * receive path (Unpack + CRC check); rec = its bytes (for the data> field); src = recvfrom's
 * source; ttl < 0 = unknown.  Writes the line(s) to out (no NUL), returns the length. ---- */
enum { OR_LOG_EPOCH = 0x1, OR_LOG_NO_DATA = 0x2, OR_LOG_NO_GPS = 0x4 };
uint32_t or_log_recv_text(const or_fields* f, const uint8_t* rec, const or_addr* src,
                          uint32_t rx_sec, uint32_t rx_usec, int protocol, int ttl,
                          uint32_t opts, char* out);
/* Binary RECV / RERR records (mgenMsg.cpp:652-710, 958-1033); avail = bytes readable at rec. */
uint32_t or_log_recv_binary(const or_fields* f, const uint8_t* rec, uint64_t avail,
                            const or_addr* src, uint32_t rx_sec, uint32_t rx_usec, int protocol,
                            uint8_t* out);

/* MgenMsg::LogSendEvent (mgenMsg.cpp:1145-1241) of the UDP / SINK / TCP send paths. */
uint32_t or_log_send_text(const or_tmpl* t, const or_desc* d, uint16_t src_port, int protocol,
                          uint32_t mgen_msg_len, uint32_t opts, char* out);
uint32_t or_log_send_binary(const or_tmpl* t, const uint8_t* packed, uint32_t packed_len,
                            uint32_t hdr_len, int protocol, uint32_t mgen_msg_len, uint8_t* out);
uint64_t or_log_send_batch(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                           const uint8_t* pool, const uint16_t* src_port, int protocol,
                           int checksum_enable, uint32_t opts, int binary, uint8_t* out);

#ifdef __cplusplus
}
#endif

/* ---- MGEN_DATA items: Report quantizers / build / parse, REPORT lines, TLV walk ---- */
uint8_t  or_q_time(double v);
double   or_uq_time(uint8_t q);
uint16_t or_q_rate(double r);
double   or_uq_rate(uint16_t q);
uint16_t or_q_loss(double l);
double   or_uq_loss(uint16_t q);
uint32_t or_report_build(const or_addr* src, const or_addr* dst, uint32_t flow_id, int protocol,
                         double duration, double lat_ave, double lat_min, double lat_max,
                         double rate, double loss, double offset, int* sign, uint8_t* b);
uint32_t or_log_report(const uint8_t* report, double duration, double rate, double loss,
                       double lat_ave, double lat_min, double lat_max, uint64_t count,
                       uint32_t sec, uint32_t usec, uint32_t opts, char* out);
uint32_t or_log_report_recv(const uint8_t* report, const or_addr* reporter, uint32_t sec,
                            uint32_t usec, uint32_t opts, char* out);
int      or_data_walk(const uint8_t* pay, uint32_t len, int controller, uint32_t* cmds,
                      uint32_t* n_cmds, uint32_t cap_cmds, uint32_t* reps, uint32_t* n_reps,
                      uint32_t cap_reps);

/* ---- CPU baselines over nthreads host threads (bench.py only) ---- */
void or_udp_pack_batch_mt(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                          const uint8_t* pool, uint8_t* slab, const uint64_t* rec_off,
                          uint64_t stride, int checksum_enable, uint32_t* out_len, int nthreads);
void or_flow_reduce_batch_mt(or_analytic* flows, uint32_t n_flows, const uint32_t* flow_idx,
                             const uint32_t* seq, const uint32_t* tx_sec, const uint32_t* tx_usec,
                             const uint16_t* msg_len, const uint32_t* rx_sec,
                             const uint32_t* rx_usec, uint32_t n, uint32_t* counts, int nthreads);

/* ---- pcap2mgen (pcap2mgen.cpp:252-482) ----
 * or_pcap_frame: one pcap record (16-byte header + data) -> the UDP payload's offset from the
 * record header and length, IP source + UDP source port, TTL / hop limit, timestamp.  Returns
 * 0 UDP, 1 bad Ethernet frame, 2 not IP, 3 bad IP, 4 not UDP, 5 truncated capture, 7 snapped
 * (a UDP datagram cut by the snapshot length with its header and >= 28 payload bytes
 * captured: or_pcap2mgen unpacks the captured bytes zero-extended to the UDP length)
 * (flags: 1 nanosecond file, 2 swapped byte order).
 * or_pcap2mgen: the whole main loop over a file image -> the log text (analytic REPORT lines,
 * RECV lines when log_rx, received REPORT lines), written to out while it fits `cap`;
 * returns the full length.  status (optional): or_pcap_frame's result per record. */
int      or_pcap_frame(const uint8_t* rec, uint32_t link_type, uint32_t flags, uint32_t* udp_off,
                       uint32_t* udp_len, or_addr* src, int* ttl, uint32_t* sec, uint32_t* usec);
uint64_t or_pcap2mgen(const uint8_t* file, uint64_t nbytes, int analytics, int log_rx,
                      double window, uint32_t opts, char* out, uint64_t cap, uint64_t* n_pkts,
                      uint8_t* status);

/* ---- ConvertBinaryLog (mgenMsg.cpp:1417-1900): a binary log file image -> text; *status
 * 0 ok, 1 bad header line, 2 record longer than 1024, 3 event the reference rejects (RERR,
 * unknown type, unknown address type), 4 file ends inside a record.  flush = Mgen's
 * log_flush (the converter passes it as the RECV lines' ttl). */
uint64_t or_convert_binary_log(const uint8_t* file, uint64_t nbytes, int log_rx, int flush,
                               uint32_t opts, char* out, uint64_t cap, int* status,
                               uint64_t* n_records);

#endif
