/*
 * mgenx.h -- C ABI of the MI355X MgenMsg pack/parse engine (libmgenx.so).
 *
 * Plain pointers and sizes only.  Every `dev_*` pointer is device (HBM) memory; the
 * caller owns every buffer (the library never allocates or frees them, matching the
 * reference's caller-owned UINT32 buffers, mgenTransport.cpp:944,1023).  Calls are
 * asynchronous on the caller's hipStream_t (passed as void*), never synchronise and
 * never allocate, so they can be captured in a hipGraph.  One mgenx_ctx per device.
 * Exceptions, each stated at its entry point: calls whose output size decides later
 * launches (the stream scans, mgenx_pack_tcp) read small results back, and calls with
 * scratch grow it (hipMalloc) the first time a larger batch arrives -- warm them up with
 * the largest batch before capturing a graph.  The log / report / walk formatters keep
 * one workspace per stream; the stream scans, mgenx_flow_reduce, mgenx_pack_tcp and
 * mgenx_tcp_rx_persist keep one per context, so those run on one stream at a time per
 * context (one context per concurrent stream).
 *
 * Return value: 0 = launched, <0 = argument/launch error (MGENX_E*).  Per-record
 * outcomes go to the `err` column with MgenMsg::Error codes (include/mgenMsg.h:63-70).
 *
 * Reference interfaces replaced (USNavalResearchLaboratory/mgen):
 *   mgenx_unpack_batch  <- MgenMsg::Unpack            include/mgenMsg.h:110
 *                          + receive CRC check        src/common/mgenTransport.cpp:958-975
 *                          (SINK 2092-2112, TCP CalcRxChecksum 1516-1564)
 *   mgenx_pack_batch    <- MgenMsg::Pack              include/mgenMsg.h:108
 *                          + MgenMsg::WriteChecksum   include/mgenMsg.h:111
 *                          + UDP/SINK send sequence   src/common/mgenTransport.cpp:1011-1031
 *   mgenx_stream_scan   <- TCP/SINK record framing    src/common/mgenTransport.cpp:1683-1760,
 *                                                     mgenAppSinkTransport.cpp:369-434
 *   mgenx_flow_reduce   <- MgenAnalytic::Update       include/mgenAnalytic.h:91-94
 *                          via Mgen::UpdateRecvAnalytics src/common/mgen.cpp:1027-1070
 *   mgenx_pack_msgs     <- MgenMsg::Pack alone (TCP fragments, the MgenMsg shim)
 *   mgenx_crc32_update  <- MgenMsg::ComputeCRC32      include/mgenMsg.h:201-203
 *   mgenx_allreduce_flows  the per-flow counter merge of flow-sharded analytics (RCCL)
 *   mgenx_flow_lookup   <- MgenAnalyticTable::FindFlow  include/mgenAnalytic.h:387
 */
#ifndef MGENX_H
#define MGENX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGENX_ABI_VERSION 1

/* ---- status codes ---- */
#define MGENX_OK          0
#define MGENX_EINVAL     -1   /* bad argument (null pointer, zero stride ...) */
#define MGENX_EDEVICE    -2   /* HIP error (no device, launch failure) */
#define MGENX_ENOMEM     -3   /* context workspace allocation failed (create only) */

/* ---- wire constants (include/mgenGlobals.h:70-80, include/mgenMsg.h:60-103) ---- */
#define MGENX_MIN_SIZE        28
#define MGENX_MAX_SIZE        8192
#define MGENX_TX_BUFFER_SIZE  8192
#define MGENX_MAX_FRAG_SIZE   65535
#define MGENX_FLAG_CONTINUES      0x01
#define MGENX_FLAG_END_OF_MSG     0x02
#define MGENX_FLAG_CHECKSUM       0x04
#define MGENX_FLAG_LAST_BUFFER    0x08
#define MGENX_FLAG_CHECKSUM_ERROR 0x10
#define MGENX_ERROR_NONE      0
#define MGENX_ERROR_VERSION   1
#define MGENX_ERROR_CHECKSUM  2
#define MGENX_ERROR_LENGTH    3
#define MGENX_ERROR_DSTADDR   4
#define MGENX_ERROR_OOB       0x80  /* record lies outside the slab: not touched */
#define MGENX_ERROR_RERR_NONE 0x40  /* log formatters only: a RERR event of a message whose
                                       error is ERROR_NONE ("type>none", mgenMsg.cpp:716) */

/* ---- unpack options ---- */
#define MGENX_OPT_CHECKSUM_FORCE  0x1  /* Mgen checksum_force (mgen.cpp:2076-2087) */
#define MGENX_OPT_TCP             0x2  /* TCP receive rules: Unpack sees min(len, 8192)
                                          bytes; a CRC mismatch also sets
                                          CHECKSUM_ERROR in flags (mgenTransport.cpp:1555) */
#define MGENX_OPT_SKIP_CRC        0x4  /* header-only decode (benchmark mode; NOT the
                                          reference receive path) */

typedef struct mgenx_ctx mgenx_ctx;

int  mgenx_abi_version(void);
int  mgenx_ctx_create(int device, mgenx_ctx** out);
int  mgenx_ctx_destroy(mgenx_ctx* ctx);
/* Last HIP error string seen by this context (static storage). */
const char* mgenx_last_error(const mgenx_ctx* ctx);
/* The HIP device of a context. */
int  mgenx_ctx_device(const mgenx_ctx* ctx);

/* One decoded record's core fields, packed (32 B): the row-major alternative to the core
 * columns -- the batch analogue of one unpacked MgenMsg object.  Written whole lines at a
 * time (16 records = 512 contiguous bytes per wave store), it is the fastest output. */
typedef struct {
    uint32_t flow_id, seq_num, tx_sec, tx_usec;
    uint32_t dst_addr4;              /* first 4 address bytes, in wire order in memory */
    uint16_t msg_len, dst_port;
    uint16_t payload_len;
    uint8_t  flags, err;             /* err: MgenMsg::Error (+ MGENX_ERROR_OOB) */
    uint8_t  dst_type, dst_len, payload_type, gps_status;
} mgenx_rec;                         /* 32 bytes */

/* ------------------------------------------------------------------ */
/* Columns written by unpack: the MgenMsg state after Unpack() on a    */
/* fresh MgenMsg (mgenMsg.cpp:315-500), one element per record.        */
/* Core columns (32 bytes per record) are required; extended columns   */
/* may be NULL (not written).                                          */
/* ------------------------------------------------------------------ */
typedef struct {
    /* core */
    uint32_t* flow_id;
    uint32_t* seq_num;
    uint32_t* tx_sec;
    uint32_t* tx_usec;
    uint16_t* msg_len;
    uint16_t* dst_port;
    uint8_t*  flags;
    uint8_t*  err;          /* MgenMsg::Error (+ MGENX_ERROR_OOB) */
    uint8_t*  dst_type;     /* ProtoAddress type (0 = not decoded, 1 IPv4, 2 IPv6) */
    uint8_t*  dst_len;      /* dst address length byte from the wire */
    uint32_t* dst_addr4;    /* first 4 address bytes, in wire order in memory */
    uint16_t* payload_len;
    uint8_t*  payload_type;
    uint8_t*  gps_status;
    /* extended (optional) */
    uint16_t* hdr_len;      /* packet_header_len */
    uint32_t* payload_off;  /* payload_data - record start = (hdr_len/4)*4 */
    uint16_t* host_port;
    uint8_t*  host_type;
    uint8_t*  host_len;
    uint8_t*  host_addr;    /* 16 bytes per record */
    uint8_t*  dst_addr;     /* 16 bytes per record */
    uint32_t* lat_raw;      /* ntohl(latitude word): degrees = raw/60000 - 180 */
    uint32_t* lon_raw;
    int32_t*  alt;
    /* row-major output: when set, unpack writes these 32-B records instead of the core
     * columns (which may then be NULL); extended columns still go to their arrays */
    mgenx_rec* rows;
    /* extended (optional): MGENX_DEC_* mask of the MgenMsg members this record's Unpack
     * assigned.  Unpack leaves the other members as they were, which matters on a reused
     * MgenMsg (the TCP receiver's rx_msg, mgenTransport.cpp:1501-1513) and for the shim. */
    uint8_t*  decoded;
} mgenx_cols;

#define MGENX_DEC_MSGLEN 0x01  /* msg_len, version (bufferLen >= MIN_SIZE, mgenMsg.cpp:323-336) */
#define MGENX_DEC_BASE   0x02  /* flags, flow_id, seq_num, tx_time (version 2, :345-366) */
#define MGENX_DEC_DST    0x04  /* dst_addr and port (dst type IPv4/IPv6, :373-398) */
#define MGENX_DEC_HDRLEN 0x08  /* packet_header_len (:437-487) */
#define MGENX_DEC_HOST   0x10  /* host_addr set (valid type, fits: :425-431) */
#define MGENX_DEC_GPS    0x20  /* latitude, longitude, altitude, gps_status (:449-465) */
#define MGENX_DEC_PTYPE  0x40  /* payload_type (:472-475) */
#define MGENX_DEC_PLEN   0x80  /* payload_len, payload_data (:482-497) */

/* Decode n records.  Record i starts at dev_slab + (dev_rec_off ? dev_rec_off[i] :
 * i*stride) and is (dev_rec_len ? dev_rec_len[i] : fixed_len) bytes long (the receive
 * length: recvfrom's len for UDP, the framed msg_len for TCP/SINK).  Records extending
 * past slab_bytes are flagged MGENX_ERROR_OOB and not read. */
int mgenx_unpack_batch(mgenx_ctx* ctx, const uint8_t* dev_slab, uint64_t slab_bytes,
                       const uint64_t* dev_rec_off, uint64_t stride,
                       const uint32_t* dev_rec_len, uint32_t fixed_len, uint32_t n,
                       const mgenx_cols* cols, uint32_t opts, void* stream);

/* Which kernel the last mgenx_unpack_batch on this context launched (host-side record of
 * the dispatch; a test and profiling aid -- the choice follows the layout, the options and
 * the batch size, never the data).  0 before the first call. */
#define MGENX_UNPACK_K_HEADER     1  /* MGENX_OPT_SKIP_CRC: header-only decode */
#define MGENX_UNPACK_K_GENERAL    2  /* any layout, one group of 16 records per wave */
#define MGENX_UNPACK_K_VAR        3  /* per-record lengths, >= 2 tiles of 64 records per
                                        wave: length-ranked groups, load ring (config 3) */
#define MGENX_UNPACK_K_FIXED      4  /* fixed stride, one length in [65, 1024] */
#define MGENX_UNPACK_K_FIXED_RING 5  /* fixed 512 / 1024-B records into rows (config 2) */
#define MGENX_UNPACK_K_OTHER      6  /* a diagnostics-build ablation */
#define MGENX_UNPACK_K_LONG       7  /* mean record >= 4 KiB (TCP streams): a wave per record */
int mgenx_unpack_last_kernel(const mgenx_ctx* ctx);

/* ------------------------------------------------------------------ */
/* Pack.  A per-flow template table holds what MgenFlow::SendMessage    */
/* takes from flow state (mgenFlow.cpp:946-983, 1039-1129); a 20-byte   */
/* descriptor per record holds the per-message fields.                 */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t flow_id;
    uint8_t  dst_type, dst_len; uint16_t dst_port;    /* dst_type: 1 IPv4, 2 IPv6 */
    uint8_t  dst_addr[16];
    uint8_t  host_type, host_len; uint16_t host_port;  /* host_type 0 = invalid (no host) */
    uint8_t  host_addr[16];
    uint32_t lat_raw, lon_raw;   /* (UINT32)((deg + 180.0) * 60000.0), mgenMsg.cpp:221,225 */
    int32_t  alt;
    uint8_t  gps_status, payload_type; uint16_t payload_len;
    uint32_t payload_off;        /* into dev_pool */
    uint8_t  has_payload, rsv0; uint16_t rsv1;
} mgenx_flow_tmpl;               /* 68 bytes */

typedef struct {
    uint32_t tmpl;               /* index into the template table */
    uint32_t seq_num, tx_sec, tx_usec;
    uint16_t msg_len;            /* MgenMsg::msg_len = the record length */
    uint8_t  flags;              /* MgenMsg flags before the transport sets LAST_BUFFER */
    uint8_t  rsv;
} mgenx_pack_desc;               /* 20 bytes */

#define MGENX_PACK_CHECKSUM    0x1   /* Mgen checksum_enable */
#define MGENX_PACK_RANDOM_FILL 0x2   /* the RANDOM_FILL build: fill = glibc rand() bytes
                                        after srand(fill_time) (mgenMsg.cpp:277-292) */
#define MGENX_PACK_RAW         0x4   /* (set by mgenx_pack_msgs) MgenMsg::Pack alone */

/* Pack n records with the UDP/SINK send sequence (LAST_BUFFER, Pack, WriteChecksum)
 * into dev_slab at dev_rec_off[i] (or i*stride).  dev_out_len[i] = Pack()'s return
 * (0 = MSG_SEND_FAILED).  Template CRCs must be prepared by mgenx_pack_prepare when
 * the template table or pool changes. */
int mgenx_pack_prepare(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl, uint32_t n_tmpl,
                       const uint8_t* dev_pool, uint32_t* dev_tmpl_crc, void* stream);
/* Select the RANDOM_FILL stream (time(NULL) value the reference would seed srand with).
 * Host-side table setup (synchronous); call when fill_time changes. */
int mgenx_set_fill_time(mgenx_ctx* ctx, uint32_t fill_time);

int mgenx_pack_batch(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                     const uint32_t* dev_tmpl_crc, const mgenx_pack_desc* dev_desc, uint32_t n,
                     const uint8_t* dev_pool, uint8_t* dev_slab, uint64_t slab_bytes,
                     const uint64_t* dev_rec_off, uint64_t stride, uint32_t* dev_out_len,
                     uint32_t opts, uint32_t fill_time, void* stream);

/* MgenMsg::Pack alone (mgenMsg.cpp:83-313), without the UDP send sequence: the
 * descriptor's flags are used as given (the caller sets LAST_BUFFER or not: with it the CRC
 * runs over bufferLen - 4 bytes, without it over bufferLen), no trailer is written
 * (MgenMsg::WriteChecksum is the caller's), and the MgenMsg state Pack leaves is returned:
 *   dev_buf_len[i]  (optional) Pack's bufferLen argument; NULL = the descriptor's msg_len
 *                   (the TCP fragment path packs msg_len 16384 into bufferLen 8192/8188,
 *                   mgenTransport.cpp:1915-1926);
 *   dev_crc_in[i]   (optional) the tx_checksum argument on entry (NULL = 0);
 *   dev_tx_crc[i]   (optional) tx_checksum after Pack (unchanged when Pack returned early);
 *   dev_state[i]    (optional) packet_header_len | flags member << 16 after Pack
 *                   (packet_header_len 0xFFFF when Pack failed: not assigned).
 * A failed Pack (return 0) writes no bytes (the reference leaves a partial header). */
int mgenx_pack_msgs(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                    const uint32_t* dev_tmpl_crc, const mgenx_pack_desc* dev_desc, uint32_t n,
                    const uint8_t* dev_pool, uint8_t* dev_slab, uint64_t slab_bytes,
                    const uint64_t* dev_rec_off, uint64_t stride, const uint32_t* dev_buf_len,
                    const uint32_t* dev_crc_in, uint32_t* dev_out_len, uint32_t* dev_tx_crc,
                    uint32_t* dev_state, uint32_t opts, uint32_t fill_time, void* stream);

/* TCP transmit: the byte stream MgenTcpTransport sends for n messages (SendMessage with
 * GetNextTxFragmentSize / GetNextTxFragment / SetupNextTxBuffer / CalcTxChecksum,
 * src/common/mgenTransport.cpp:1320-1400, 1818-1993), back to back.  dev_msg_total[i] is the
 * message's mgen_msg_len (fragments of <= 65535 bytes past that, CONTINUES / END_OF_MSG);
 * the descriptor's msg_len is ignored.  A fragment over 8192 bytes is one 8-KiB Pack whose
 * buffer is re-sent from its start, the CRC (MGENX_PACK_CHECKSUM) covering every byte
 * before the trailer.  dev_msg_off[i] = the message's offset in the stream (a message whose
 * first Pack fails, or of length 0, takes no bytes); *total_bytes = the stream length.
 * Waits for the plan only (the stream layout decides the launches): it returns once the
 * stream length is known, with the stores still running on `stream` (stream-ordered, as any
 * launch).  When the stream would exceed stream_cap nothing is written, *total_bytes is set
 * and MGENX_EINVAL returned.  A context's TCP transmit calls must all use ONE stream: the plan
 * leaves its verdict in a per-context device word that the queued Pack reads, so a call on
 * another stream could overwrite it before the first call's Pack has read it. */
int mgenx_pack_tcp(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl, const uint32_t* dev_tmpl_crc,
                   const mgenx_pack_desc* dev_desc, const uint32_t* dev_msg_total, uint32_t n,
                   const uint8_t* dev_pool, uint8_t* dev_stream, uint64_t stream_cap,
                   uint64_t* dev_msg_off, uint64_t* total_bytes, uint32_t opts,
                   uint32_t fill_time, void* stream);

/* MgenMsg::ComputeCRC32(checksum, buffer, len) (mgenMsg.cpp:524-541) over n byte ranges:
 * dev_state_out[i] = the running CRC after feeding dev_data[off[i] .. off[i]+len[i]) to
 * dev_state_in[i] (0 restarts from CRC32_XINIT; no final xor). */
int mgenx_crc32_update(mgenx_ctx* ctx, const uint8_t* dev_data, const uint64_t* dev_off,
                       const uint32_t* dev_len, uint32_t n, const uint32_t* dev_state_in,
                       uint32_t* dev_state_out, void* stream);

/* Standard CRC-32 (MgenMsg::ComputeCRC32 from a zero state + CRC32_XOROT) of n
 * byte ranges: out[i] = crc(dev_data[off[i] .. off[i]+len[i])). */
int mgenx_crc32_batch(mgenx_ctx* ctx, const uint8_t* dev_data, const uint64_t* dev_off,
                      const uint32_t* dev_len, uint32_t n, uint32_t* dev_out, void* stream);

/* ---- the resident single-message worker ----
 * For callers that stay one message at a time (an unchanged MgenUdpTransport calls
 * MgenMsg::Unpack once per datagram, mgenTransport.cpp:948-997, and ComputeCRC32 once per
 * message): a batch entry point per message costs a launch, copies and a synchronisation.
 * A worker keeps ONE wave resident on the context's device, polling a mailbox in pinned host
 * memory: a call copies the message into the mailbox, the wave decodes or checksums it and
 * writes the reply back; the call spins until it arrives.  Host buffers in, results out --
 * no device pointers.  The wave exits after idle_ms without a request (the next call
 * relaunches it), on mgenx_worker_stop / mgenx_worker_destroy, and when its context is
 * destroyed (mgenx_ctx_destroy stops and frees every worker created on it; the handle then
 * only accepts mgenx_worker_destroy, other calls return MGENX_EINVAL).  While its wave runs
 * it holds up device-wide synchronisations (hipFree, hipHostFree, hipDeviceSynchronize) until
 * it idles out: the library's own workspace growth ends every worker's wave first (the next
 * call relaunches it); a caller about to synchronise the device calls mgenx_worker_stop.
 * Calls on one worker are serialised by the worker; results equal the batch entry points' on
 * the same bytes.
 *   mgenx_worker_unpack  <- MgenMsg::Unpack (include/mgenMsg.h:110, mgenMsg.cpp:315-500) on a
 *                           fresh MgenMsg: the members it assigned (`decoded`, MGENX_DEC_*) and
 *                           err (MgenMsg::Error; 0 = Unpack returned true); no CRC check
 *   mgenx_worker_crc32   <- MgenMsg::ComputeCRC32 (include/mgenMsg.h:201-203, mgenMsg.cpp:
 *                           524-541): the running checksum in and out
 *   mgenx_worker_recv    <- Unpack + the receive path's ComputeCRC32 in one reply (below)
 *   mgenx_worker_pack    <- MgenMsg::Pack alone (below)
 *   mgenx_worker_flow_update <- MgenAnalytic::Update of one record (below) */
#define MGENX_WORKER_MAX_BYTES 65536u
#define MGENX_WORKER_PACK_MAX  16384u   /* mgenx_worker_pack's largest bufferLen */
typedef struct {
    uint32_t flow_id, seq_num, tx_sec, tx_usec, payload_off;
    uint32_t lat_raw, lon_raw;
    int32_t  alt;
    uint16_t msg_len, dst_port, payload_len, hdr_len, host_port;
    uint8_t  flags, err, dst_type, dst_len, payload_type, gps_status, host_type, host_len;
    uint8_t  decoded, version, rsv[2];
    uint8_t  dst_addr[16], host_addr[16];
} mgenx_unpacked;                    /* 88 bytes */
typedef struct mgenx_worker mgenx_worker;
int mgenx_worker_create(mgenx_ctx* ctx, uint32_t idle_ms, mgenx_worker** out);
int mgenx_worker_destroy(mgenx_worker* w);
int mgenx_worker_stop(mgenx_worker* w);  /* end the wave now (the next call relaunches it) */
/* *flags: MGENX_WORKER_DEVICE_MAILBOX when requests go to fine-grained device memory the host
 * stores into through the BAR (the runtime granted the CPU access), else pinned host memory
 * (environment MGENX_WORKER_HOST_MAILBOX=1 forces the latter). */
#define MGENX_WORKER_DEVICE_MAILBOX 0x1u
int mgenx_worker_info(const mgenx_worker* w, uint32_t* flags);
int mgenx_worker_unpack(mgenx_worker* w, const uint8_t* msg, uint32_t len, mgenx_unpacked* out);
int mgenx_worker_crc32(mgenx_worker* w, const uint8_t* data, uint32_t len, uint32_t state_in,
                       uint32_t* state_out);
/* The UDP / SINK receive path's two calls in one reply (mgenTransport.cpp:958-965,
 * 2092-2100): MgenMsg::Unpack as mgenx_worker_unpack, then -- when Unpack succeeded and `force`
 * (checksum_force) is set or the decoded flags carry CHECKSUM -- ComputeCRC32(0, msg, len - 4):
 * *crc_done = 1 and *crc_state the running CRC the caller then XORs with CRC32_XOROT and
 * compares with the trailer (no final xor here, as ComputeCRC32); else *crc_done = 0. */
int mgenx_worker_recv(mgenx_worker* w, const uint8_t* msg, uint32_t len, uint32_t force,
                      mgenx_unpacked* out, uint32_t* crc_state, uint32_t* crc_done);
/* MgenAnalytic::Update (include/mgenAnalytic.h:91-94, mgenAnalytic.cpp:74-258) of ONE record
 * on the device flow state dev_flows[slot] (mgenx_flow_init / mgenx_flow_reduce's array; the
 * worker's wave reads and writes it in place).  The wave is NOT on the caller's stream: the
 * stream that last wrote dev_flows (a queued mgenx_flow_reduce or mgenx_flow_init) must be
 * synchronised before this call, and later batch work on dev_flows enqueued only after it
 * returns.  *updated = 1 when the record closed a window, with the report in *report (index =
 * the flow's report number; latency_ave from the window's in-order latency sum).  Equal to
 * mgenx_flow_reduce of the same records one call at a time. */
struct mgenx_flow_state;
struct mgenx_flow_report;
int mgenx_worker_flow_update(mgenx_worker* w, struct mgenx_flow_state* dev_flows, uint32_t slot,
                             uint32_t seq, uint32_t rx_sec, uint32_t rx_usec, uint32_t msg_size,
                             uint32_t tx_sec, uint32_t tx_usec, uint32_t* updated,
                             struct mgenx_flow_report* report);
/* MgenMsg::Pack (include/mgenMsg.h:108, mgenMsg.cpp:83-313) of one message, as mgenx_pack_msgs
 * with n = 1: the message as a template (its payload bytes at `payload`, payload_off ignored)
 * and a descriptor; bufferLen, the tx_checksum argument, MGENX_PACK_CHECKSUM /
 * MGENX_PACK_RANDOM_FILL and the fill time.  out (bufferLen bytes) receives *ret bytes
 * (Pack's return; 0: failed, nothing written); *tx_crc the tx_checksum after; *state
 * packet_header_len | flags << 16.  bufferLen <= MGENX_WORKER_PACK_MAX. */
int mgenx_worker_pack(mgenx_worker* w, const mgenx_flow_tmpl* tmpl, const uint8_t* payload,
                      const mgenx_pack_desc* desc, uint32_t buf_len, uint32_t crc_in,
                      uint32_t opts, uint32_t fill_time, uint8_t* out, uint32_t* ret,
                      uint32_t* tx_crc, uint32_t* state);

/* ---- the TCP receiver's persistent rx_msg ----
 * MgenTcpTransport decodes every message of a connection into ONE MgenMsg (rx_msg,
 * src/common/mgenTransport.cpp:1082): ResetRxMsgState (:1501-1513) zeroes only
 * mgen_msg_len / msg_len / flow_id / seq_num / the error between messages, Unpack runs only
 * while a log file is open (:2016-2028) and assigns members stage by stage (mgenMsg.cpp:
 * 315-500), and the CRC check reads the flags rx_msg holds (:1516-1564).  So a record that
 * stops early keeps the previous record's flags, tx time, destination, header length, GPS
 * position and payload; with no log file nothing is decoded at all (flow id and sequence
 * number stay 0) and the CRC is checked only under checksum_force.
 * mgenx_tcp_rx_persist rewrites n consecutive records of one connection, decoded by
 * mgenx_unpack_batch(MGENX_OPT_TCP) into core + extended columns with `decoded`, into that
 * rx_msg view, in place: every member group a record did not assign comes from the latest
 * earlier record that did, or from *dev_state (rx_msg before the batch; updated to rx_msg
 * after it).  dev_payload_rec[i] (optional) = the record whose bytes the payload member
 * points into (MGENX_RX_PREV: before this batch).  Options:
 *   MGENX_RX_NOLOG  no log file on this connection: no record is decoded (host address
 *                   and gps_status read invalid; the caller unpacks with
 *                   MGENX_OPT_CHECKSUM_FORCE to have the CRC verdicts when it needs them);
 *   MGENX_RX_FORCE  checksum_force (the receiver's setting, for records without flags).
 * Core columns are required (not the row layout). */
#define MGENX_RX_NOLOG 0x1
#define MGENX_RX_FORCE 0x2
#define MGENX_RX_PREV  0xFFFFFFFFu
typedef struct {
    uint32_t tx_sec, tx_usec, lat_raw, lon_raw;
    int32_t  alt;
    uint32_t payload_off;
    uint16_t dst_port, hdr_len, payload_len;
    uint8_t  flags, dst_type, dst_len, payload_type, rsv[2];
    uint8_t  dst_addr[16];
} mgenx_rx_state;                /* 48 bytes; zero = a fresh MgenMsg's members */
int mgenx_tcp_rx_persist(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                         const uint32_t* dev_rec_len, uint32_t n, const mgenx_cols* cols,
                         mgenx_rx_state* dev_state, uint32_t* dev_payload_rec, uint32_t opts,
                         void* stream);

/* ---- stream framing (TCP / SINK record boundaries) ----
 * mgenx_stream_scan finds the record chain of a byte stream from offset 0 exactly as the
 * reference receivers frame it -- TCP: MgenTcpTransport::GetRxNumBytes / OnRecvMsg
 * (src/common/mgenTransport.cpp:1683-1760; msg_len < 4 is a stream error that stops the
 * scan); SINK: MgenAppSinkTransport::OnInputReady (src/common/mgenAppSinkTransport.cpp:
 * 369-434; msg_len outside [28, 8192] skips the 2 length bytes) -- and writes the records'
 * offsets and lengths in stream order (the first `cap` of them).  The output feeds
 * mgenx_unpack_batch directly (rec_off / rec_len; MGENX_OPT_TCP for TCP streams).
 * Synchronous on `stream` (the record count decides the launches); the context keeps a
 * workspace that grows with the stream (about 1/32 of its size). */
#define MGENX_SCAN_TCP  0
#define MGENX_SCAN_SINK 1
typedef struct mgenx_scan_info {
  uint64_t n_records;   /* records found (only the first `cap` are written) */
  uint64_t consumed;    /* bytes consumed: offset just past the last whole record/skip */
  int32_t  status;      /* 0 = ok, 1 = TCP record with msg_len < 4 (scan stopped there) */
  uint32_t candidates;  /* diagnostic: plausible starts found by the parallel pass */
  uint64_t resolved;    /* diagnostic: records framed by the sequential resolver */
  uint32_t path;        /* diagnostic: how the chain was found -- 0 lifting (and resolver),
                           1 every candidate a record, 2 the successor-marked hypothesis */
  uint32_t reserved;
} mgenx_scan_info;
int mgenx_stream_scan(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                      uint64_t* dev_rec_off, uint32_t* dev_rec_len, uint64_t cap,
                      mgenx_scan_info* info, void* stream);

/* ---- sharded framing (one stream split over ranks; no reference counterpart: the
 * reference frames one socket sequentially) ----
 * Rank r owns the records that START in [a_r, b_r) of the global stream and holds the
 * bytes [a_r, min(b_r + MGENX_SCAN_HALO, N)) (a record starting before b_r ends within the
 * halo).  Its chain entry e_r (the first chain position >= a_r) lies below
 * a_r + MGENX_SCAN_HALO.  Protocol (mgen_amd/shard.py):
 *   1. mgenx_stream_scan_exits on the local bytes with window = MGENX_SCAN_HALO and
 *      limit = b_r - a_r: for each candidate entry below the window, where its chain first
 *      reaches >= limit (dev_exits; bit 63 set = the chain leaves the candidate set first,
 *      exit unknown).  Unused rows are ~0.
 *   2. all-gather the (entry, exit) tables; every rank stitches e_0 = 0, e_{r+1} = exit_r(e_r)
 *      identically; a missing or unknown exit is settled by that rank's
 *      mgenx_stream_scan_range (its info.consumed is the exit) and one more all-gather.
 *   3. mgenx_stream_scan_range(entry = e_r - a_r, limit, MGENX_SCAN_REUSE): the rank's
 *      records (local offsets; add a_r for global ones), on the tables of step 1.
 * The union over ranks equals mgenx_stream_scan of the whole stream. */
#define MGENX_SCAN_HALO  65536ull
#define MGENX_SCAN_REUSE 1   /* flags: reuse the tables of the last build on this context */
int mgenx_stream_scan_exits(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                            uint64_t window, uint64_t limit, uint64_t* dev_entries,
                            uint64_t* dev_exits, uint32_t cap, uint32_t* candidates,
                            void* stream);
/* Records of the chain from `entry` over positions < limit (limit <= nbytes): the scan
 * rule of mgenx_stream_scan started at `entry`.  info->consumed is where it stopped: the
 * first chain position >= limit, or the end / error position as for the whole stream. */
int mgenx_stream_scan_range(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                            uint64_t entry, uint64_t limit, int flags, uint64_t* dev_rec_off,
                            uint32_t* dev_rec_len, uint64_t cap, mgenx_scan_info* info,
                            void* stream);

/* A socket address as recvfrom reports it (ProtoAddress type / length / port / bytes). */
typedef struct {
    uint8_t  type;      /* MgenMsg::AddressType: 1 IPv4, 2 IPv6 */
    uint8_t  len;       /* address length (4 / 16) */
    uint16_t port;
    uint8_t  addr[16];  /* network byte order */
} mgenx_addr;           /* 20 bytes */

/* ---- per-flow receive analytics (MgenAnalytic::Update) ----
 * Restates MgenAnalytic::Init/Update (src/common/mgenAnalytic.cpp:28-258) as called by
 * Mgen::UpdateRecvAnalytics (src/common/mgen.cpp:1027-1070): per flow, an order-dependent
 * window state machine with a 1024-bit ProtoSlidingMask of received sequence numbers
 * (duplicate detection), FP64 latency sum/min/max and a report when rx >= window end.
 * The caller maps its flow key (src addr, dst addr, flow id: FindFlow, mgenAnalytic.cpp:
 * 312-328) to a dense flow index; records are passed in receive order.  State persists in
 * the caller's mgenx_flow_state array across calls (streaming batches).
 * Parity: bit-exact (FP64 included, no contraction) with the oracle restatement; the
 * protolib primitives themselves are unpinned (ProtoSlidingMask, ProtoTime::Delta). */
typedef struct mgenx_flow_state {   /* 256 B; set up by mgenx_flow_init */
  uint32_t mask[32];                /* bit i <-> sequence number mask_first + i */
  uint32_t mask_first, mask_n;      /* lowest set sequence number, number of set bits */
  uint32_t seq_start, window_valid;
  int64_t  win_start_sec, win_start_usec, win_end_sec, win_end_usec;
  double   window_size;             /* quantized as Report::Quantize/UnquantizeTimeValue */
  uint64_t msg_count, byte_count, dup_count;
  double   latency_sum, latency_min, latency_max;
  uint64_t n_reports;
  uint64_t rsv[2];
} mgenx_flow_state;

typedef struct mgenx_flow_report {  /* one closed window (MgenAnalytic::Report) */
  uint32_t flow, index;             /* flow index, report number within the flow */
  int64_t  start_sec, start_usec;   /* window start */
  double   duration;
  uint64_t msg_count;
  double   rate, loss, latency_ave, latency_min, latency_max;
  int64_t  rx_sec, rx_usec;         /* receive time of the message that closed it */
} mgenx_flow_report;

/* ---- MGEN_DATA items: MgenAnalytic::Report and MgenFlowCommand ----
 * Wire format include/mgenAnalytic.h:14-57 (ProtoPkt fields network order); quantizers
 * mgenAnalytic.cpp:568-642 -- the device quantizes through tables the context builds with
 * the host's libm (log, log10, pow), so results equal the reference's host arithmetic.
 *
 * mgenx_report_build: the report_msg bytes MgenAnalytic keeps (Init :28-71, the window
 * close :245-253, GetReport :296-310) for every kept report of mgenx_flow_reduce:
 * slot f * per_flow + j (j < min(report_count[f], per_flow)) gets 52 bytes (dev_items) and
 * its length (dev_item_len: 24 / 28 IPv4, 48 / 52 IPv6, per the flow-id flag).  Keys: the
 * analytic's src / dst / flow id / protocol.  dev_sign[f] carries FLAG_LATENCY_SIGN, which
 * SetLatencyAve sets and nothing clears (in/out).  dev_offset (optional, per slot): the
 * seconds GetReport's window offset measures (the send time minus the window end; the
 * analytics caller itself reports 0). */
#define MGENX_REPORT_MAX        52
#define MGENX_PAYLOAD_MGEN_DATA 1    /* MgenMsg::MGEN_DATA payload type (mgenMsg.h:102) */
#define MGENX_MAX_FLOW          40   /* MgenEvent::FlowStatus::MAX_FLOW (mgenEvent.h:194) */
typedef struct {
    mgenx_addr src, dst;
    uint32_t flow_id;
    uint8_t  protocol;           /* Protocol: 1 UDP, 2 TCP, 3 SINK */
    uint8_t  rsv[3];
} mgenx_report_key;              /* 48 bytes */
int mgenx_report_build(mgenx_ctx* ctx, const mgenx_flow_report* dev_reports, uint32_t n_flows,
                       uint32_t per_flow, const uint32_t* dev_report_count,
                       const mgenx_report_key* dev_keys, uint8_t* dev_sign,
                       const double* dev_offset, uint8_t* dev_items, uint8_t* dev_item_len,
                       void* stream);
/* REPORT log lines of the kept reports, as Mgen::UpdateRecvAnalytics logs them at each
 * window close (MgenAnalytic::Log, mgenAnalytic.cpp:260-295: the report_msg's key fields,
 * the analytic's unquantized values, timestamp = the closing message's rx time), in slot
 * order (flow-major; each flow's lines in time order; empty slots give no line).
 * Two passes like mgenx_log_recv_text: dev_line_off[n_flows * per_flow + 1]. */
int mgenx_log_report_text(mgenx_ctx* ctx, const uint8_t* dev_items,
                          const mgenx_flow_report* dev_reports, uint32_t n_flows,
                          uint32_t per_flow, const uint32_t* dev_report_count, uint32_t opts,
                          char* dev_text, uint64_t text_cap, uint64_t* dev_line_off,
                          void* stream);
/* MgenTransport::ProcessRecvMessage (mgenTransport.cpp:2132-2191) over the MGEN_DATA
 * payloads of n decoded records (err == 0, payload_type == MGEN_DATA; columns err,
 * payload_type, payload_len, payload_off required):
 *   dev_status[i]   0 walked to the end, 1 invalid MGEN_DATA payload (a flow command
 *                   longer than the rest), 2 invalid REPORT, 3 an item of length 0 (the
 *                   reference loops forever on it; the walk stops), 0xFF not MGEN_DATA;
 *   dev_needs_host[i]  1 when the payload carries flow commands or (with a controller)
 *                   reports: the host's control plane acts on them (Mgen::ProcessFlowCommand,
 *                   MgenController::OnRecvReport);
 *   dev_cmds        pairs (record, flow_id << 2 | status) for every flow whose status is
 *                   not FLOW_UNCHANGED (MgenFlowCommand::GetStatus, flows 1..MAX_FLOW);
 *   dev_reps        pairs (record, slab offset of the report item) (MGENX_DATA_CONTROLLER:
 *                   type bytes > 0x0f are reports, else skipped as generic items);
 *   dev_totals[2]   the number of commands and reports (only the first cap are written).
 * Bytes past a payload read as 0. */
#define MGENX_DATA_CONTROLLER 0x1
int mgenx_data_walk(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                    uint64_t stride, const mgenx_cols* cols, uint32_t n, uint32_t opts,
                    uint8_t* dev_status, uint8_t* dev_needs_host, uint32_t* dev_cmds,
                    uint32_t cmd_cap, uint64_t* dev_reps, uint32_t rep_cap,
                    uint32_t* dev_totals, void* stream);
/* REPORT lines of received reports (MgenAnalytic::Report::Log, mgenAnalytic.cpp:747-786):
 * dev_reps = mgenx_data_walk's pairs; per record the source (the reporter) and rx time.
 * "sent>" prints the rx time again, as the reference does. */
int mgenx_log_report_recv_text(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_reps,
                               uint32_t n_reps, const mgenx_addr* dev_src,
                               const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec,
                               uint32_t opts, char* dev_text, uint64_t text_cap,
                               uint64_t* dev_line_off, void* stream);

/* Packed per-flow counters for the multi-GPU merge (one RCCL all-reduce(sum) of
 * n_flows x 64 B: flows are owned by one rank, the others contribute zeros). */
typedef struct mgenx_flow_counters {
  uint64_t msg_count, byte_count, dup_count, n_reports;
  double   latency_sum, latency_min, latency_max;
  uint64_t seq_start;
} mgenx_flow_counters;

int mgenx_flow_init(mgenx_ctx* ctx, mgenx_flow_state* dev_flows, uint32_t n_flows,
                    double window_sec, void* stream);
/* Records i < n with dev_flow_idx[i] < n_flows update flow dev_flow_idx[i], in order.
 * Columns: seq_num, tx_sec, tx_usec, msg_len (from mgenx_unpack_batch); rx time per
 * record in dev_rx_sec/dev_rx_usec.  Reports go to dev_reports[f * per_flow + k] for
 * k < per_flow; dev_report_count[f] (zeroed by the caller) counts all of them.  With
 * per_flow == 0, dev_reports and dev_report_count may be NULL (the states' n_reports still
 * count every report).  Synchronous on `stream` only when its workspace must grow. */
int mgenx_flow_reduce(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_seq,
                      const uint32_t* dev_tx_sec, const uint32_t* dev_tx_usec,
                      const uint16_t* dev_msg_len, const uint32_t* dev_rx_sec,
                      const uint32_t* dev_rx_usec, uint32_t n, mgenx_flow_state* dev_flows,
                      uint32_t n_flows, mgenx_flow_report* dev_reports, uint32_t per_flow,
                      uint32_t* dev_report_count, void* stream);
/* mgenx_flow_reduce plus, per kept report slot f * per_flow + k, the input record whose
 * Update closed the window (dev_report_rec, optional): the record after which the reference
 * logs the REPORT line (pcap2mgen.cpp:468-470, mgen.cpp:1055-1060). */
int mgenx_flow_reduce_ex(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_seq,
                         const uint32_t* dev_tx_sec, const uint32_t* dev_tx_usec,
                         const uint16_t* dev_msg_len, const uint32_t* dev_rx_sec,
                         const uint32_t* dev_rx_usec, uint32_t n, mgenx_flow_state* dev_flows,
                         uint32_t n_flows, mgenx_flow_report* dev_reports, uint32_t per_flow,
                         uint32_t* dev_report_count, uint32_t* dev_report_rec, void* stream);
/* The same reduction reading seq_num, tx_sec, tx_usec and msg_len from the 32-B rows
 * mgenx_unpack_batch writes (cols.rows): the unpack -> FindFlow -> Update pipeline without
 * the column layout.  dev_report_rec as mgenx_flow_reduce_ex (optional). */
int mgenx_flow_reduce_rows(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const mgenx_rec* dev_rows,
                           const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec, uint32_t n,
                           mgenx_flow_state* dev_flows, uint32_t n_flows,
                           mgenx_flow_report* dev_reports, uint32_t per_flow,
                           uint32_t* dev_report_count, uint32_t* dev_report_rec, void* stream);
int mgenx_flow_export(mgenx_ctx* ctx, const mgenx_flow_state* dev_flows, uint32_t n_flows,
                      mgenx_flow_counters* dev_out, void* stream);


/* ---- MgenAnalyticTable::FindFlow for batches (mgenAnalytic.cpp:312-328) ----
 * A device hash table from the reference's flow key -- dst addr | dst port | src addr |
 * src port | flowId -- to dense flow indices 0, 1, ... (new keys are numbered in the order
 * of their first record, so the mapping is deterministic).  mgenx_flow_lookup maps n decoded
 * records (columns dst_addr, dst_len, dst_port, flow_id, and err when given: err != 0 maps
 * to MGENX_FLOW_NONE) with their recvfrom source addresses to dev_flow_idx[i] -- the input
 * mgenx_flow_reduce takes -- and copies the table's flow count to dev_n_flows[0] (optional,
 * device memory).  Keys persist across calls (streaming batches).
 * With cols->rows (the 32-B mgenx_rec output) the key fields and err come from the rows;
 * the destination address from the dst_addr column when given, else from the rows'
 * dst_addr4 -- exact for IPv4 destinations; a record whose dst_len exceeds 4 then maps to
 * MGENX_FLOW_NONE (pass dst_addr when IPv6 destinations can occur).
 * A table takes new keys while it holds fewer than its max_flows (rounded up to half its
 * power-of-two slot count; keys created concurrently may pass that bound together) and probes
 * at most 1024 slots per lookup: a record whose key finds no room maps to MGENX_FLOW_NONE (an
 * undersized table; the caller redoes the batch on a larger one).  Near the bound that
 * refusal can be spurious (a record racing the creation of its own key, or a key past the
 * probe limit): MGENX_FLOW_NONE means "redo on a larger table", never "no such flow".
 * Performance: a table of at most 2048 flows (4096 slots) is probed from a copy of its keys
 * staged in LDS (up to 1536 keys; keys past that, and keys new in the call, take the atomic
 * path); larger tables probe HBM.  Steady state, config 4: 8.4M lookups in ~0.10 ms. */
#define MGENX_FLOW_NONE 0xFFFFFFFFu
typedef struct mgenx_flow_table mgenx_flow_table;
int mgenx_flow_table_create(mgenx_ctx* ctx, uint32_t max_flows, mgenx_flow_table** out);
int mgenx_flow_table_destroy(mgenx_flow_table* table);
int mgenx_flow_lookup(mgenx_ctx* ctx, mgenx_flow_table* table, const mgenx_cols* cols,
                      const mgenx_addr* dev_src, uint32_t n, uint32_t* dev_flow_idx,
                      uint32_t* dev_n_flows, void* stream);
/* The key of every flow index < cap (MgenAnalytic::Init's src / dst / flow id, with
 * `protocol`): the report_msg keys mgenx_report_build takes (mgenAnalytic.cpp:28-71). */
int mgenx_flow_keys(mgenx_ctx* ctx, const mgenx_flow_table* table, int protocol,
                    mgenx_report_key* dev_keys, uint32_t cap, void* stream);
/* The sizes a batch's report slots need, on the device: dev_out[0] = the most records any flow
 * index < n_flows holds, dev_out[1] / dev_out[2] = the lowest / highest receive time (sec *
 * 1e6 + usec) over those records (UINT64_MAX / 0 when there are none).  dev_counts: n_flows
 * words of scratch (cleared here).  pcap2mgen sizes its per-flow report slots from these
 * (a window closes at most once per record and once per window of capture time). */
int mgenx_flow_span(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_rx_sec,
                    const uint32_t* dev_rx_usec, uint32_t n, uint32_t n_flows,
                    uint32_t* dev_counts, uint64_t* dev_out, void* stream);

/* ---- event log (MgenMsg::LogRecvEvent / LogRecvError, text form) ----
 * One line per record, as the UDP receive path logs it (src/common/mgenTransport.cpp:
 * 976-994): "RECV proto>... flow>... seq>... src>... dst>... sent>... size>... [host>...]
 * [ttl>...] [gps>...] [data>...] [flags>...]" for a good record
 * (src/common/mgenMsg.cpp:1034-1102), "RERR type>... src>..." for a record with an error
 * (:711-735); timestamps GMT "HH:MM:SS.usec" or epoch "sec.usec" (src/common/mgen.cpp:55-83).
 * Byte-exact with the reference's fprintf output on x86-64 Linux.
 * Inputs: the unpack outputs for the same records -- core fields (rows or columns) plus the
 * extended columns dst_addr, host_addr, host_port, host_type, host_len, lat_raw, lon_raw,
 * alt, payload_off (all required) --, the slab and record placement (for the data> hex),
 * the recvfrom source address, the receive time and (optional, NULL = unknown) TTL.
 * Output: dev_line_off[i] = byte offset of record i's line, dev_line_off[n] = total bytes;
 * the lines are written to dev_text only when the total fits text_cap (read
 * dev_line_off[n] and call again with a larger buffer otherwise).  No NUL terminator. */

#define MGENX_PROTO_UDP  1   /* Protocol (include/mgenGlobals.h:61-68) */
#define MGENX_PROTO_TCP  2
#define MGENX_PROTO_SINK 3
#define MGENX_LOG_EPOCH   0x1  /* Mgen::SetEpochTimestamp(true) */
#define MGENX_LOG_NO_DATA 0x2  /* log_data off */
#define MGENX_LOG_NO_GPS  0x4  /* log_gps_data off */
#define MGENX_LOG_SKIP_ERR 0x8 /* records with err != 0 get no line (pcap2mgen.cpp:428-432
                                  skips a packet Unpack rejects instead of logging RERR) */

int mgenx_log_recv_text(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                        uint64_t stride, const mgenx_cols* cols, const mgenx_addr* dev_src,
                        const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec,
                        const int32_t* dev_ttl, uint32_t n, int protocol, uint32_t opts,
                        char* dev_text, uint64_t text_cap, uint64_t* dev_line_off, void* stream);
/* The binary log form of the same events (MgenMsg::LogRecvEvent / LogRecvError binary
 * branches, src/common/mgenMsg.cpp:652-710, 958-1033): per record an event header (type,
 * protocol, BE length, BE rx time, BE source port, source type/length/address) followed, for
 * RECV, by hdr_len + payload_len message bytes with CHECKSUM cleared in the flags byte
 * (the hdr_len extended column is also required); RERR ends with the BE error code.
 * The message bytes are the receive buffer's: the record's dev_rec_len[i] bytes (the
 * recvfrom length; when dev_rec_len is NULL, its msg_len field), then zeros where the
 * reference's buffer holds stale bytes; bytes past slab_bytes are zero too.
 * dev_rec_pos has the same meaning as dev_line_off.  The file header line the reference
 * writes once per log file is the caller's. */
int mgenx_log_recv_binary(mgenx_ctx* ctx, const uint8_t* dev_slab, uint64_t slab_bytes,
                          const uint64_t* dev_rec_off, uint64_t stride,
                          const uint32_t* dev_rec_len, const mgenx_cols* cols,
                          const mgenx_addr* dev_src, const uint32_t* dev_rx_sec,
                          const uint32_t* dev_rx_usec, uint32_t n, int protocol,
                          uint8_t* dev_out, uint64_t out_cap, uint64_t* dev_rec_pos,
                          void* stream);

/* SEND events (MgenMsg::LogSendEvent, src/common/mgenMsg.cpp:1145-1241) of records packed
 * by a send path, as the transport logs them after each successful send
 * (mgenTransport.cpp:1060, 1392, 1805: theTime = the message's tx time):
 *   text:   "<tx time> SEND proto>P flow>F seq>S srcPort>SP dst>A/port size>N [host>H/port]\n"
 *           (size = msg_len; TCP: mgen_msg_len from dev_msg_total);
 *   binary: {SEND_EVENT 3, protocol, BE recordLength [, TCP: BE mgen_msg_len]} and then
 *           recordLength bytes of the packed message (UDP / SINK) with CHECKSUM cleared,
 *           recordLength = 12 + dst length + packet_header_len (+ host length + 4 with a
 *           host); bytes past the packed message read as 0.
 * dev_src_port[t]: template t's source port (the flow transport's socket port,
 * mgenFlow.cpp:975-977).  dev_out_len (optional): Pack's return per record -- 0 means the
 * message was not sent and gets no event.  Two passes as mgenx_log_recv_text:
 * dev_pos[n + 1] = byte offsets; written only when the total fits out_cap. */
int mgenx_log_send_text(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                        const mgenx_pack_desc* dev_desc, const uint16_t* dev_src_port,
                        const uint32_t* dev_out_len, const uint32_t* dev_msg_total, uint32_t n,
                        int protocol, uint32_t opts, char* dev_text, uint64_t text_cap,
                        uint64_t* dev_line_off, void* stream);
int mgenx_log_send_binary(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                          const mgenx_pack_desc* dev_desc, const uint32_t* dev_out_len,
                          const uint32_t* dev_msg_total, const uint8_t* dev_slab,
                          uint64_t slab_bytes, const uint64_t* dev_rec_off, uint64_t stride,
                          uint32_t n, int protocol, uint8_t* dev_out, uint64_t out_cap,
                          uint64_t* dev_rec_pos, void* stream);

/* ---- one log file from several line sources, in record order ----
 * The reference writes, per received message, the lines of several loggers in turn: e.g.
 * pcap2mgen (pcap2mgen.cpp:445-476) logs the analytic's REPORT line when Update closed a
 * window, then the RECV line, then the REPORT lines of the reports the payload carries.
 * mgenx_text_interleave concatenates, for record 0, 1, ..., n_rec - 1, each source's lines
 * of that record in source order.  A source is a text with line offsets (line k =
 * text[line_off[k], line_off[k+1])) and the record each line belongs to:
 *   MGENX_TEXT_PER_RECORD  line i is record i's (n_lines = n_rec; empty lines allowed);
 *   MGENX_TEXT_OWNER       owner[k * index_stride] = line k's record, non-decreasing in k;
 *   MGENX_TEXT_MAP         index[i] = record i's line (at most one), or MGENX_FLOW_NONE;
 *   MGENX_TEXT_SCATTER     index[k] = line k's record (at most one line per record, any
 *                          order; MGENX_FLOW_NONE = no record): e.g. the slots of
 *                          mgenx_log_report_text with mgenx_flow_reduce_ex's dev_report_rec.
 * Two passes like mgenx_log_recv_text: dev_rec_off[n_rec + 1] = byte offsets of each record's
 * output; dev_out is written only when the total fits out_cap.  srcs is a HOST array. */
#define MGENX_TEXT_PER_RECORD 0
#define MGENX_TEXT_OWNER      1
#define MGENX_TEXT_MAP        2
#define MGENX_TEXT_SCATTER    3
#define MGENX_TEXT_MAX_SRC    4
typedef struct {
    const char*     text;         /* may be NULL only when every line is empty */
    const uint64_t* line_off;     /* n_lines + 1 entries */
    uint32_t        n_lines;
    uint32_t        kind;         /* MGENX_TEXT_* */
    const uint32_t* index;        /* owner (OWNER), record -> line (MAP), line -> record
                                     (SCATTER) */
    uint32_t        index_stride; /* OWNER: u32 elements between owners (1, or 4 for the
                                     (record, offset) u64 pairs of mgenx_data_walk) */
    uint32_t        rsv;
} mgenx_text_src;
int mgenx_text_interleave(mgenx_ctx* ctx, const mgenx_text_src* srcs, uint32_t n_src,
                          uint32_t n_rec, char* dev_out, uint64_t out_cap, uint64_t* dev_rec_off,
                          void* stream);

/* ---- pcap2mgen: captured packets -> MgenMsg records (src/common/pcap2mgen.cpp:252-482) ----
 * mgenx_pcap_index (HOST memory, no device work: the pcap_next loop, :344) reads the pcap
 * file header and walks the record headers: the offsets of the first `cap` records' 16-byte
 * headers go to pkt_off (host memory).  info: link type, flags, records found, bytes consumed
 * (a record cut short by the end of the buffer ends the walk, as pcap_next returns NULL).
 * Returns MGENX_EINVAL for a buffer that is not a pcap file.
 * mgenx_pcap_parse (device) restates, per record, pcap2mgen's frame walk (:346-436) over
 * protolib's ProtoPktETH / ProtoPktIP / ProtoPktUDP (restated: protolib is not vendored,
 * so this layer is parity unpinned): DLT_LINUX_SLL (16-byte header) or, for every
 * other link type as in the reference, Ethernet frames (hdr.len <= 4094 bytes, optional
 * 802.1Q tag), IPv4 / IPv6, UDP.  Per record:
 * udp_off / udp_len = the UDP payload (the Unpack buffer; udp_len 0 when status != 0, so
 * Unpack rejects it), src = IP source + UDP source port (msg.SetSrcAddr, :434-435),
 * ttl = IPv4 TTL / IPv6 hop limit, rx time = the pcap timestamp (ProtoTime(hdr.ts); a
 * nanosecond file is read at microsecond precision, as pcap_fopen_offline does). */
#define MGENX_DLT_EN10MB    1
#define MGENX_DLT_LINUX_SLL 113
#define MGENX_PCAP_NSEC    0x1  /* nanosecond timestamps (magic 0xa1b23c4d) */
#define MGENX_PCAP_SWAPPED 0x2  /* the file's byte order is not the host's */
#define MGENX_PCAP_UDP       0  /* status: a UDP datagram */
#define MGENX_PCAP_BAD_ETH   1  /* "invalid Ether frame" (:370-373) */
#define MGENX_PCAP_NOT_IP    2  /* not IPv4 / IPv6 (:422) */
#define MGENX_PCAP_BAD_IP    3  /* "bad IP packet" (:388-391) */
#define MGENX_PCAP_NOT_UDP   4  /* (:425) */
#define MGENX_PCAP_TRUNCATED 5  /* UDP payload past the captured bytes: skipped (the
                                   reference reads stale buffer bytes there) */
#define MGENX_PCAP_OOB       6  /* record past the buffer */
#define MGENX_PCAP_SNAPPED   7  /* a UDP datagram cut by the capture's snapshot length whose
                                   UDP header and >= MIN_SIZE payload bytes were captured:
                                   mgenx_pcap_snap moves it into scratch, zero-extended to the
                                   UDP length (then MGENX_PCAP_UDP); left alone it is skipped */
typedef struct {
    uint32_t link_type;   /* DLT_* */
    uint32_t flags;       /* MGENX_PCAP_NSEC | MGENX_PCAP_SWAPPED */
    uint32_t snaplen;
    uint32_t rsv;
    uint64_t n_records;   /* records found (only the first cap offsets are written) */
    uint64_t consumed;    /* bytes of whole records, file header included */
    uint64_t snap_bytes;  /* scratch mgenx_pcap_snap may need: sum over records captured
                             short of their wire length of that length, 16-byte rounded */
} mgenx_pcap_info;
int mgenx_pcap_index(const uint8_t* buf, uint64_t nbytes, uint64_t* pkt_off, uint64_t cap,
                     mgenx_pcap_info* info);
int mgenx_pcap_parse(mgenx_ctx* ctx, const uint8_t* dev_buf, uint64_t buf_bytes,
                     const uint64_t* dev_pkt_off, uint32_t n, uint32_t link_type,
                     uint32_t flags, uint64_t* dev_udp_off, uint32_t* dev_udp_len,
                     mgenx_addr* dev_src, int32_t* dev_ttl, uint32_t* dev_rx_sec,
                     uint32_t* dev_rx_usec, uint8_t* dev_status, void* stream);
/* A capture taken with a snapshot length (tcpdump -s N) cuts datagrams short; the reference
 * parses such a frame by its wire length and Unpacks the UDP payload from its parse buffer,
 * so the MGEN header comes from the captured bytes and the rest of the buffer is stale.
 * mgenx_pcap_snap copies every MGENX_PCAP_SNAPPED packet's captured UDP payload into
 * dev_buf[file_bytes, buf_bytes) (scratch after the file image; info.snap_bytes is enough)
 * zero-extended to its UDP length, points dev_udp_off / dev_udp_len there and sets its
 * status to MGENX_PCAP_UDP; a packet that does not fit stays SNAPPED.  Asynchronous. */
int mgenx_pcap_snap(mgenx_ctx* ctx, uint8_t* dev_buf, uint64_t file_bytes, uint64_t buf_bytes,
                    const uint64_t* dev_pkt_off, uint32_t n, uint32_t flags, uint8_t* dev_status,
                    uint64_t* dev_udp_off, uint32_t* dev_udp_len, void* stream);

/* ---- MgenMsg::ConvertBinaryLog: binary log -> text log (src/common/mgenMsg.cpp:1417-1900) --
 * mgenx_binlog_index (HOST memory, no device work) checks the header line ("mgen
 * version=<4|5> ... type=binary_log\n" and its NUL, :1437-1518) and walks the records
 * {type, protocol, BE recordLength <= 1024, body}: the offsets of the records the reference
 * converts go to rec_off (host memory), up to the first one it stops at -- info->status:
 * MGENX_BINLOG_OK (end of file), _HEADER (not a binary log), _TOO_LONG (recordLength > 1024),
 * _EVENT (RERR or an unknown event type, or an unknown address type: the reference returns
 * false there, :1586-1590, 1892-1895), _SHORT (the file ends inside a record, or a record is
 * too short for the fields its type reads -- the event time; RECV 12 + source length; LISTEN
 * / IGNORE 12; JOIN / LEAVE 13 + group length + name length; ON ... RECONNECT 18 + address
 * length -- which mgen never writes and the reference would parse from stale buffer bytes).
 * mgenx_convert_binary_log (device) writes the text the reference writes for those records,
 * in order: RECV (Unpack of the stored message + LogRecvEvent text with the source and event
 * time, the converter's argument order at :1607 putting log_flush in the ttl slot, then the
 * REPORT lines of MGEN_DATA items), SEND (Unpack + LogSendEvent text: tx time, srcPort 0),
 * LISTEN / IGNORE / JOIN / LEAVE / START / STOP / ON / ACCEPT / CONNECT / DISCONNECT / OFF /
 * SHUTDOWN / RECONNECT lines (:1628-1891).  A RECV / SEND record whose stored message Unpack
 * rejects (mgen never writes one) is logged all the same, as the reference ignores Unpack's
 * result: the fields a fresh MgenMsg keeps, RECV's tx time = the event time.  flags: MGENX_BINLOG_NO_RX (log_rx off),
 * MGENX_BINLOG_FLUSH (log_flush on); opts: MGENX_LOG_EPOCH / _NO_DATA / _NO_GPS.
 * dev_rec_pos[n + 1] = byte offsets of each record's text; dev_text is written only when the
 * total fits text_cap.  Synchronous (intermediate sizes are read back); the context keeps a
 * workspace that grows with the log. */
#define MGENX_BINLOG_OK       0
#define MGENX_BINLOG_HEADER   1
#define MGENX_BINLOG_TOO_LONG 2
#define MGENX_BINLOG_EVENT    3
#define MGENX_BINLOG_SHORT    4
#define MGENX_BINLOG_NO_RX  0x1
#define MGENX_BINLOG_FLUSH  0x2
typedef struct {
    uint64_t n_records;   /* records to convert (only the first cap offsets are written) */
    uint64_t consumed;    /* bytes up to the end of the last of them */
    int32_t  status;      /* MGENX_BINLOG_* */
    uint32_t version;     /* the header line's major version */
} mgenx_binlog_info;
int mgenx_binlog_index(const uint8_t* buf, uint64_t nbytes, uint64_t* rec_off, uint64_t cap,
                       mgenx_binlog_info* info);
int mgenx_convert_binary_log(mgenx_ctx* ctx, const uint8_t* dev_buf, uint64_t buf_bytes,
                             const uint64_t* dev_rec_off, uint32_t n, uint32_t flags,
                             uint32_t opts, char* dev_text, uint64_t text_cap,
                             uint64_t* dev_rec_pos, void* stream);

/* ---- multi-GPU exchange (RCCL over xGMI) ----
 * One communicator per rank (one process per GPU): rank 0 calls mgenx_comm_unique_id and
 * hands the MGENX_COMM_ID_BYTES bytes to every rank (any out-of-band channel), then every
 * rank calls mgenx_comm_init.  Collectives are asynchronous on `stream`. */
typedef struct mgenx_comm mgenx_comm;
#define MGENX_COMM_ID_BYTES 128
int mgenx_comm_unique_id(void* id_out);
int mgenx_comm_init(mgenx_ctx* ctx, int nranks, int rank, const void* id, mgenx_comm** out);
int mgenx_comm_destroy(mgenx_comm* comm);
/* The per-flow counter merge after flow-sharded mgenx_flow_reduce: in-place SUM of
 * n_flows x 64 B over the ranks (one ncclAllReduce).  Exact when every flow has one owner and
 * the other ranks export zeros for it (mgenx_flow_export of a flow never updated there):
 * integer sums of the 64-bit words leave the owner's counters, FP64 fields included, bit for
 * bit. */
int mgenx_allreduce_flows(mgenx_ctx* ctx, mgenx_comm* comm, mgenx_flow_counters* dev_counters,
                          uint32_t n_flows, void* stream);
/* dev_out[r * count + k] = rank r's dev_in[k] (the stream-shard stitch). */
int mgenx_allgather_u64(mgenx_ctx* ctx, mgenx_comm* comm, const uint64_t* dev_in,
                        uint64_t* dev_out, uint32_t count, void* stream);

#ifdef __cplusplus
}
#endif
#endif
