#define _GNU_SOURCE 1  /* gmtime_r, inet_ntop under -std=c11 */
/*
 * mgen_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of the reference MGEN hot path.  Every function cites the
 * reference file:line whose behaviour it restates.  See mgen_oracle.h for the
 * parity-pinning status.
 */
#include "mgen_oracle.h"

#include <math.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* helpers: network byte order                                         */
/* ------------------------------------------------------------------ */
static void put16(uint8_t* b, uint16_t v) { b[0] = (uint8_t)(v >> 8); b[1] = (uint8_t)v; }
static void put32(uint8_t* b, uint32_t v)
{
    b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16); b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
}
static uint16_t get16(const uint8_t* b) { return (uint16_t)((b[0] << 8) | b[1]); }
static uint32_t get32(const uint8_t* b)
{
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

/* ------------------------------------------------------------------ */
/* CRC-32: reflected poly 0x04C11DB7 (0xEDB88320), init/xorout ~0      */
/* mgenMsg.cpp:524-554 (incremental ComputeCRC32), table :576-642      */
/* ------------------------------------------------------------------ */
static uint32_t g_table[256];
static int g_table_ready = 0;

void or_crc32_table(uint32_t table[256])
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
        table[i] = c;
    }
}

static const uint32_t* table(void)
{
    if (!g_table_ready) { or_crc32_table(g_table); g_table_ready = 1; }
    return g_table;
}

/* mgenMsg.cpp:524-541: a running value of exactly 0 restarts from CRC32_XINIT. */
void or_crc32_update(uint32_t* checksum, const uint8_t* buf, uint32_t len)
{
    const uint32_t* t = table();
    uint32_t c = *checksum;
    if (c == 0) c = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < len; i++) c = t[(c ^ buf[i]) & 0xFFu] ^ (c >> 8);
    *checksum = c;
}

/* mgenMsg.cpp:502-522: xor-out, stored big-endian at buflen-4. */
int or_write_checksum(uint32_t* tx_checksum, uint8_t* buf, uint32_t buflen)
{
    if (buflen < 4) return 0;
    *tx_checksum ^= 0xFFFFFFFFu;
    put32(buf + buflen - 4, *tx_checksum);
    return 1;
}

/* ------------------------------------------------------------------ */
/* glibc random_r TYPE_3 (srand/rand) -- the RANDOM_FILL byte source   */
/* (mgenMsg.cpp:277-292: srand(time(NULL)) then (char)rand() per byte) */
/* ------------------------------------------------------------------ */
void or_glibc_rand_bytes(uint32_t seed, uint32_t n, uint8_t* out)
{
    int32_t r[34];
    int32_t word = (int32_t)(seed == 0 ? 1u : seed);
    r[0] = word;
    for (int i = 1; i < 31; i++) {
        long hi = word / 127773;
        long lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        r[i] = word;
    }
    /* ring of the last 34 values; r[i] = r[i-31] + r[i-3] (mod 2^32) */
    uint32_t ring[34];
    for (int i = 0; i < 31; i++) ring[i] = (uint32_t)r[i];
    for (int i = 31; i < 34; i++) ring[i] = ring[i - 31];
    uint64_t i = 34;
    uint32_t produced = 0;
    while (produced < n) {
        uint32_t v = ring[(i - 31) % 34] + ring[(i - 3) % 34];
        ring[i % 34] = v;
        if (i >= 344) out[produced++] = (uint8_t)((v >> 1) & 0xFFu);
        i++;
    }
}

/* ------------------------------------------------------------------ */
/* MgenMsg::Pack  (mgenMsg.cpp:83-313)                                 */
/* ------------------------------------------------------------------ */
static uint8_t wire_addr_type(uint8_t protoType)
{
    /* mgenMsg.cpp:131-149 / 161-177: ProtoAddress::IPv4 -> 1, IPv6 -> 2 */
    return (protoType == OR_ADDR_IPV4 || protoType == OR_ADDR_IPV6) ? protoType : 0;
}

uint16_t or_pack(or_msg* m, uint8_t* buf, uint16_t bufferLen, int includeChecksum,
                 uint32_t* tx_checksum, int random_fill, uint32_t fill_time, uint16_t* hdr_len)
{
    uint32_t len = 0;
    const uint32_t msgLen = bufferLen;
    uint16_t dummy;
    if (!hdr_len) hdr_len = &dummy;

    put16(buf + len, m->msg_len); len += 2;            /* :97-100 */
    buf[len++] = m->version;                          /* :103 */
    buf[len++] = m->flags;                            /* :106 */
    put32(buf + len, m->flow_id); len += 4;           /* :109-112 */
    put32(buf + len, m->seq_num); len += 4;           /* :114-117 */
    put32(buf + len, m->tx_sec); len += 4;            /* :119-122 */
    put32(buf + len, m->tx_usec); len += 4;           /* :124-127 */
    put16(buf + len, m->dst.port); len += 2;          /* :129-131 */
    uint8_t dtype = wire_addr_type(m->dst.type);
    if (!dtype) return 0;                             /* :146-148 unsupported type */
    uint8_t addrLen = m->dst.len;
    buf[len++] = dtype;
    buf[len++] = addrLen;
    memcpy(buf + len, m->dst.addr, addrLen);          /* :155-157 */
    len += addrLen;

    /* host_addr (:163-216) */
    const int hostValid = (m->host.type == OR_ADDR_IPV4 || m->host.type == OR_ADDR_IPV6);
    uint8_t htype = hostValid ? m->host.type : 0;
    addrLen = hostValid ? m->host.len : 0;
    if (msgLen >= len + addrLen + 4) {
        put16(buf + len, hostValid ? m->host.port : 0); len += 2;
        buf[len++] = htype;
        buf[len++] = addrLen;
        if (addrLen) memcpy(buf + len, m->host.addr, addrLen);
        len += addrLen;
    } else {
        if (msgLen < len) return 0;                   /* :207-210 */
        memset(buf + len, 0, msgLen - len);
        *hdr_len = (uint16_t)len;
        return (uint16_t)msgLen;
    }
    /* GPS (:219-241) */
    if (msgLen >= len + 13) {
        put32(buf + len, (uint32_t)((m->latitude + 180.0) * 60000.0)); len += 4;
        put32(buf + len, (uint32_t)((m->longitude + 180.0) * 60000.0)); len += 4;
        put32(buf + len, (uint32_t)m->altitude); len += 4;
        buf[len++] = m->gps_status;
    } else {
        memset(buf + len, 0, msgLen - len);
        *hdr_len = (uint16_t)len;
        return (uint16_t)msgLen;
    }
    /* payload_type (:243-251) */
    if (msgLen >= len + 1) {
        buf[len++] = m->payload_type;
    } else {
        *hdr_len = (uint16_t)len;
        return (uint16_t)msgLen;
    }
    /* payload_len (:252-263) */
    if (msgLen >= len + 2) {
        put16(buf + len, m->payload_len);
        len += 2;
    } else {
        memset(buf + len, 0, msgLen - len);
        *hdr_len = (uint16_t)len;
        return (uint16_t)msgLen;
    }
    *hdr_len = (uint16_t)len;
    /* payload (:264-273) */
    if (m->payload_data && msgLen >= len + m->payload_len) {
        memcpy(buf + len, m->payload_data, m->payload_len);
        len += m->payload_len;
    } else {
        buf[len - 2] = 0;
        buf[len - 1] = 0;
    }
    /* fill (:275-294) */
    if (msgLen > len) {
        if (random_fill) {
            if (msgLen >= 2 + len) {
                buf[len] = 0;
                buf[len + 1] = 0;
                or_glibc_rand_bytes(fill_time, msgLen - (len + 2), buf + len + 2);
            } else if (msgLen != len) {
                buf[len] = 0;
            }
        } else {
            memset(buf + len, 0, msgLen - len);
        }
    }
    /* checksum (:295-310) */
    if (includeChecksum) {
        if (msgLen > len + 4) {
            buf[3] |= OR_FLAG_CHECKSUM;
            m->flags |= OR_FLAG_CHECKSUM;
        }
        if (m->flags & OR_FLAG_LAST_BUFFER)
            or_crc32_update(tx_checksum, buf, msgLen - 4);
        else
            or_crc32_update(tx_checksum, buf, msgLen);
        m->flags &= (uint8_t)~OR_FLAG_LAST_BUFFER;   /* ClearFlag (mgenMsg.h:126) */
    }
    return (uint16_t)msgLen;
}

/* MgenUdpTransport::SendMessage (mgenTransport.cpp:1011-1031);
 * MgenAppSinkTransport::SendMessage (mgenAppSinkTransport.cpp:159-169). */
uint32_t or_udp_pack(const or_msg* msg, uint8_t* out, int checksum_enable, int random_fill,
                     uint32_t fill_time)
{
    or_msg m = *msg;
    uint32_t tx = 0;
    m.flags |= OR_FLAG_LAST_BUFFER;
    uint32_t len = or_pack(&m, out, m.msg_len, checksum_enable, &tx, random_fill, fill_time, NULL);
    if (len == 0) return 0;
    if (checksum_enable && (m.flags & OR_FLAG_CHECKSUM)) or_write_checksum(&tx, out, len);
    return len;
}

/* ------------------------------------------------------------------ */
/* MgenTcpTransport transmit state machine                             */
/* SendMessage :1320-1400, GetNextTxBuffer :1762-1816,                 */
/* SetupNextTxBuffer :1818-1852, CalcTxChecksum :1854-1876,            */
/* GetNextTxFragment :1878-1951, GetNextTxFragmentSize :1960-1993      */
/* ------------------------------------------------------------------ */
typedef struct {
    or_msg   tx;
    uint8_t  buf[OR_TX_BUFFER_SIZE + 4];
    uint32_t tx_checksum;
    uint32_t tx_buffer_index, tx_buffer_pending, tx_msg_offset;
    uint16_t tx_fragment_pending;
    int      ck, rf;
    uint32_t T;
} tcp_tx_state;

static uint16_t tcp_next_fragment_size(tcp_tx_state* s)
{
    s->tx.flags &= (uint8_t)~OR_FLAG_CONTINUES;
    s->tx.msg_len = 0;
    uint32_t remaining = s->tx.mgen_msg_len - s->tx_msg_offset;
    if (!remaining) return 0;
    if (remaining > OR_MAX_FRAG_SIZE) {
        if (remaining < (uint32_t)(OR_MAX_FRAG_SIZE + OR_MIN_FRAG_SIZE))
            s->tx.msg_len = OR_MAX_FRAG_SIZE - OR_MIN_FRAG_SIZE;
        else
            s->tx.msg_len = OR_MAX_FRAG_SIZE;
    } else {
        s->tx.msg_len = (uint16_t)remaining;
    }
    if (s->tx.mgen_msg_len > OR_MAX_FRAG_SIZE) {
        if ((s->tx.mgen_msg_len - s->tx_msg_offset) > s->tx.msg_len)
            s->tx.flags |= OR_FLAG_CONTINUES;
        else
            s->tx.flags |= OR_FLAG_END_OF_MSG;
    }
    return s->tx.msg_len;
}

static uint16_t tcp_next_fragment(tcp_tx_state* s)
{
    uint16_t tx_buffer_size = OR_TX_BUFFER_SIZE;
    s->buf[0] = 0;
    s->tx_checksum = 0;
    s->tx_buffer_index = 0;
    if (!tcp_next_fragment_size(s)) return 0;
    if (s->ck) {
        /* int arithmetic: (msg_len - 8192) < 4 */
        if (((int)s->tx.msg_len - OR_TX_BUFFER_SIZE) < 4 && s->tx.msg_len != OR_MIN_FRAG_SIZE)
            tx_buffer_size = OR_TX_BUFFER_SIZE - 4;
    }
    if (s->tx.msg_len > OR_TX_BUFFER_SIZE) {
        s->tx_buffer_pending = or_pack(&s->tx, s->buf, tx_buffer_size, s->ck, &s->tx_checksum,
                                       s->rf, s->T, NULL);
        s->tx_msg_offset += s->tx_buffer_pending;
    } else if (s->tx.msg_len > 0) {
        s->tx.flags |= OR_FLAG_LAST_BUFFER;
        s->tx_buffer_pending = or_pack(&s->tx, s->buf, s->tx.msg_len, s->ck, &s->tx_checksum,
                                       s->rf, s->T, NULL);
        s->tx_msg_offset += s->tx_buffer_pending;
        if (s->ck && (s->tx.flags & OR_FLAG_CHECKSUM))
            or_write_checksum(&s->tx_checksum, s->buf, s->tx.msg_len);
    } else {
        s->tx_buffer_pending = 0;
    }
    return s->tx.msg_len;
}

static void tcp_calc_tx_checksum(tcp_tx_state* s)
{
    if (s->tx.flags & OR_FLAG_LAST_BUFFER) {
        if (s->tx_buffer_pending < 4) return;
        or_crc32_update(&s->tx_checksum, s->buf, s->tx_buffer_pending - 4);
    } else {
        or_crc32_update(&s->tx_checksum, s->buf, s->tx_buffer_pending);
    }
}

static void tcp_setup_next_buffer(tcp_tx_state* s)
{
    if ((s->ck && s->tx_fragment_pending <= (OR_TX_BUFFER_SIZE - 4)) ||
        (!s->ck && s->tx_fragment_pending <= OR_TX_BUFFER_SIZE)) {
        s->tx_buffer_pending = s->tx_fragment_pending;
        s->tx.flags |= OR_FLAG_LAST_BUFFER;
        if (s->ck) tcp_calc_tx_checksum(s);
        s->tx.flags &= (uint8_t)~OR_FLAG_LAST_BUFFER;
        if (s->ck) or_write_checksum(&s->tx_checksum, s->buf, s->tx_fragment_pending);
    } else {
        if (s->ck && ((int)s->tx_fragment_pending - OR_TX_BUFFER_SIZE) < 4)
            s->tx_buffer_pending = s->tx_fragment_pending - 4u;
        else
            s->tx_buffer_pending = OR_TX_BUFFER_SIZE;
        if (s->ck) tcp_calc_tx_checksum(s);
    }
    s->tx_buffer_index = 0;
    s->tx_msg_offset += s->tx_buffer_pending;
}

uint32_t or_tcp_tx(const or_msg* msg, uint8_t* out, int checksum_enable, int random_fill,
                   uint32_t fill_time)
{
    static tcp_tx_state s;   /* 8 KB buffer; single-threaded test use */
    memset(&s, 0, sizeof(s));
    s.tx = *msg;
    s.ck = checksum_enable;
    s.rf = random_fill;
    s.T = fill_time;
    uint32_t outn = 0;
    s.tx_fragment_pending = tcp_next_fragment(&s);
    if (!s.tx_fragment_pending || !s.tx_buffer_pending) return 0;
    for (uint32_t guard = 0; guard < (1u << 24); guard++) {
        uint32_t numBytes = s.tx_buffer_pending;   /* Send() moves everything */
        memcpy(out + outn, s.buf + s.tx_buffer_index, numBytes);
        outn += numBytes;
        s.tx_buffer_index += numBytes;
        s.tx_buffer_pending -= numBytes;
        s.tx_fragment_pending = (uint16_t)(s.tx_fragment_pending - numBytes);
        if (s.tx_buffer_pending) continue;
        if (0 == s.tx_buffer_pending && s.tx_fragment_pending) {
            tcp_setup_next_buffer(&s);
            if (s.tx_buffer_pending) continue;
        }
        if (s.tx_buffer_pending == 0 && s.tx_fragment_pending == 0) {
            s.tx_fragment_pending = tcp_next_fragment(&s);
            if (s.tx_buffer_pending) continue;
        }
        if (!s.tx_fragment_pending && s.tx_msg_offset > 0) return outn;
    }
    return outn;
}

/* ------------------------------------------------------------------ */
/* MgenMsg::Unpack (mgenMsg.cpp:315-500) on a fresh MgenMsg            */
/* (defaults from the constructor, mgenMsg.cpp:38-49)                  */
/* ------------------------------------------------------------------ */
static const uint32_t GPS_RAW_ZERO = 10800000u;   /* (0.0 + 180) * 60000 */

/* MgenMsg::Unpack on a REUSED MgenMsg (the TCP receiver's rx_msg): only host_addr and
 * gps_status are reset on entry (mgenMsg.cpp:318-319); every member is assigned stage by
 * stage below and the unreached ones keep their values.  or_unpack runs it on a fresh
 * MgenMsg (constructor defaults, mgenMsg.cpp:38-49). */
uint32_t or_unpack_persist(const uint8_t* buf, uint32_t bufferLen, or_fields* f)
{
    uint32_t d = 0;   /* MGENX_DEC_* mask of the members assigned */
    f->host_type = 0; f->host_len = 0; f->host_port = 0;
    memset(f->host_addr, 0, sizeof(f->host_addr));
    f->gps_status = 0;
    f->ok = 0;
    uint32_t len = 0;
    if (bufferLen < OR_MIN_SIZE) { f->err = OR_ERROR_LENGTH; return d; }   /* :323-328 */
    f->msg_len = get16(buf); len += 2;
    f->version = buf[len++];
    d |= 0x01;
    if (f->version != OR_VERSION) { f->err = OR_ERROR_VERSION; return d; } /* :336-343 */
    f->flags = buf[len++];
    f->flow_id = get32(buf + len); len += 4;
    f->seq_num = get32(buf + len); len += 4;
    f->tx_sec = get32(buf + len); len += 4;
    f->tx_usec = get32(buf + len); len += 4;
    d |= 0x02;
    uint16_t dstPort = get16(buf + len); len += 2;
    uint8_t t = buf[len++];
    if (t != OR_ADDR_IPV4 && t != OR_ADDR_IPV6) { f->err = OR_ERROR_DSTADDR; return d; } /* :374-392 */
    uint32_t addrLen = buf[len++];
    /* :394-398 -- no bounds check in the reference; bytes past the record are
     * undefined there (stale receive buffer) and read as zero here. */
    f->dst_type = t;
    f->dst_len = (uint8_t)addrLen;
    for (uint32_t i = 0; i < addrLen && i < 16; i++)
        f->dst_addr[i] = (len + i < bufferLen) ? buf[len + i] : 0;
    f->dst_port = dstPort;
    d |= 0x04;
    len += addrLen;
    /* host (:400-443) */
    if ((len + 4) <= bufferLen) {
        uint16_t hostPort = get16(buf + len); len += 2;
        uint8_t ht = buf[len++];
        if (ht != OR_ADDR_IPV4 && ht != OR_ADDR_IPV6) ht = OR_ADDR_INVALID;
        addrLen = buf[len++];
        if ((len + addrLen) <= bufferLen) {
            if (ht != OR_ADDR_INVALID) {
                f->host_type = ht;
                f->host_len = (uint8_t)addrLen;
                for (uint32_t i = 0; i < addrLen && i < 16; i++) f->host_addr[i] = buf[len + i];
                f->host_port = hostPort;
                d |= 0x10;
            }
            len += addrLen;
        } else {
            f->hdr_len = (uint16_t)len; f->ok = 1; return d | 0x08;
        }
    } else {
        f->hdr_len = (uint16_t)len; f->ok = 1; return d | 0x08;
    }
    /* GPS (:446-465) */
    if ((len + 13) <= bufferLen) {
        f->lat_raw = get32(buf + len); len += 4;
        f->lon_raw = get32(buf + len); len += 4;
        f->alt = (int32_t)get32(buf + len); len += 4;
        f->gps_status = buf[len++];
        d |= 0x20;
    } else {
        f->hdr_len = (uint16_t)len; f->ok = 1; return d | 0x08;
    }
    /* payload_type (:467-475) */
    if ((len + 1) <= bufferLen) {
        f->payload_type = buf[len++];
        d |= 0x40;
    } else {
        f->hdr_len = (uint16_t)len; f->ok = 1; return d | 0x08;
    }
    /* payload_len + data (:477-497) */
    if ((len + 2) <= bufferLen) {
        f->payload_len = get16(buf + len);
        len += 2;
        f->hdr_len = (uint16_t)len;
        d |= 0x80 | 0x08;
        if (f->payload_len != 0 && (len + f->payload_len) <= bufferLen) {
            f->payload_off = (len / 4) * 4;   /* alignedBuffer + len/4 (word floor) */
        } else {
            f->payload_len = 0;
        }
    }
    f->ok = 1;
    return d;
}

void or_unpack(const uint8_t* buf, uint32_t bufferLen, or_fields* f)
{
    memset(f, 0, sizeof(*f));
    f->version = OR_VERSION;
    f->lat_raw = f->lon_raw = GPS_RAW_ZERO;
    (void)or_unpack_persist(buf, bufferLen, f);
}

static int crc_ok(const uint8_t* rec, uint32_t len)
{
    if (len < 4) return 0;
    uint32_t c = 0;
    or_crc32_update(&c, rec, len - 4);
    c ^= 0xFFFFFFFFu;
    return c == get32(rec + len - 4);
}

/* mgenTransport.cpp:958-975 (UDP) and :2092-2112 (SINK HandleMgenMessage) */
void or_udp_recv(const uint8_t* rec, uint32_t len, int checksum_force, or_fields* f)
{
    or_unpack(rec, len, f);
    if (f->ok && (checksum_force || (f->flags & OR_FLAG_CHECKSUM))) {
        if (!crc_ok(rec, len)) f->err = OR_ERROR_CHECKSUM;
    }
}

/* ------------------------------------------------------------------ */
/* TCP receive framing                                                 */
/* Records are [p, p + msg_len); Unpack sees min(msg_len, 8192) bytes  */
/* (CopyMsgBuffer :1996-2031); CRC over msg_len-4 vs the BE trailer   */
/* (CalcRxChecksum :1516-1564), decided on the Unpacked flags or the   */
/* force option; a mismatch sets ERROR_CHECKSUM and CHECKSUM_ERROR.    */
/* The running CRC is evaluated over the whole span at once (the       */
/* reference's read boundaries depend on partial socket reads).        */
/* ------------------------------------------------------------------ */
void or_tcp_recv(const uint8_t* rec, uint32_t L, int checksum_force, or_fields* o)
{
    or_unpack(rec, L < OR_TX_BUFFER_SIZE ? L : OR_TX_BUFFER_SIZE, o);
    if (L >= 4 && (checksum_force || (o->flags & OR_FLAG_CHECKSUM))) {
        if (!crc_ok(rec, L)) {
            o->err = OR_ERROR_CHECKSUM;
            o->flags |= OR_FLAG_CHECKSUM_ERROR;
        }
    }
}

/* The TCP receiver's persistent rx_msg over n consecutive records of one connection
 * (mgenTransport.cpp:1082 rx_msg; ResetRxMsgState :1501-1513 between messages, framing
 * sets msg_len :1714-1720; Unpack on min(len, 8192) bytes only while a log file is open
 * :2016-2028; CalcRxChecksum :1516-1564 with the flags rx_msg holds).  st: rx_msg before
 * the batch (updated); out[i]: rx_msg after record i; payload_rec[i]: the record whose
 * Unpack last assigned the payload (0xFFFFFFFF = before the batch), carried in *pay_src. */
void or_tcp_rx_persist(const uint8_t* stream, const uint64_t* offs, const uint32_t* lens,
                       uint32_t n, int log_open, int checksum_force, or_fields* st,
                       uint32_t* pay_src, or_fields* out, uint32_t* payload_rec)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t* rec = stream + offs[i];
        const uint32_t L = lens[i];
        st->flow_id = 0; st->seq_num = 0; st->err = 0; st->ok = 0;   /* ResetRxMsgState */
        st->msg_len = (uint16_t)L;                                    /* the framing's */
        if (log_open) {
            const uint32_t d = or_unpack_persist(rec, L < OR_TX_BUFFER_SIZE ? L : OR_TX_BUFFER_SIZE,
                                                 st);
            if (d & 0x80) *pay_src = i;
        }
        if ((checksum_force || (st->flags & OR_FLAG_CHECKSUM)) && L >= 4 && !crc_ok(rec, L)) {
            st->err = OR_ERROR_CHECKSUM;
            st->flags |= OR_FLAG_CHECKSUM_ERROR;
        }
        out[i] = *st;
        if (payload_rec) payload_rec[i] = *pay_src;
    }
}

uint32_t or_tcp_scan(const uint8_t* stream, uint64_t nbytes, int checksum_force,
                     uint64_t* offs, uint32_t* lens, or_fields* f, uint32_t cap,
                     uint64_t* consumed, int* status)
{
    uint64_t p = 0;
    uint32_t n = 0;
    if (status) *status = 0;
    while (p + 2 <= nbytes) {
        uint32_t L = get16(stream + p);
        if (L < 4) { if (status) *status = 1; break; }
        if (p + L > nbytes) break;
        const uint8_t* rec = stream + p;
        if (n < cap) {
            or_tcp_recv(rec, L, checksum_force, &f[n]);
            offs[n] = p;
            lens[n] = L;
        }
        n++;
        p += L;
    }
    if (consumed) *consumed = p;
    return n;
}

/* MgenAppSinkTransport::OnInputReady (mgenAppSinkTransport.cpp:369-434): a length
 * outside [MIN_SIZE, MAX_SIZE] discards the two length bytes and resynchronises. */
uint32_t or_sink_scan(const uint8_t* stream, uint64_t nbytes, int checksum_force,
                      uint64_t* offs, uint32_t* lens, or_fields* f, uint32_t cap,
                      uint64_t* consumed)
{
    uint64_t p = 0;
    uint32_t n = 0;
    while (p + 2 <= nbytes) {
        uint32_t L = get16(stream + p);
        if (L < OR_MIN_SIZE || L > OR_MAX_SIZE) { p += 2; continue; }
        if (p + L > nbytes) break;
        if (n < cap) {
            or_udp_recv(stream + p, L, checksum_force, &f[n]);
            offs[n] = p;
            lens[n] = L;
        }
        n++;
        p += L;
    }
    if (consumed) *consumed = p;
    return n;
}

/* ------------------------------------------------------------------ */
/* MgenPayload::SetPayloadString (mgenPayload.cpp:24-55, :127-166)     */
/* ------------------------------------------------------------------ */
static uint8_t from_hex(char c)
{
    if (c >= '0' && c <= '9') return (uint8_t)(c - '0');
    if (c >= 'a' && c <= 'f') return (uint8_t)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (uint8_t)(c - 'A' + 10);
    return 0;
}

uint32_t or_payload_from_hex(const char* hex, uint8_t* out, uint32_t cap)
{
    if (!hex) return 0;
    size_t sl = strlen(hex);
    uint32_t n = (uint32_t)(sl / 2 + sl % 2);
    for (uint32_t i = 0; i < n && i < cap; i++) {
        uint8_t hi = from_hex(hex[2 * i]);
        uint8_t lo = (2 * i + 1 < sl) ? from_hex(hex[2 * i + 1]) : 0;  /* odd: reads NUL */
        out[i] = (uint8_t)((hi << 4) | lo);
    }
    return n;
}

/* ------------------------------------------------------------------ */
/* protolib restatements (UNPINNED: no reference fixture covers them)  */
/* ProtoTime: struct timeval; Delta = sec diff + 1e-6 * usec diff.     */
/* ProtoSlidingMask(num_bits, range 0xffffffff): a set of indices that */
/* always spans fewer than num_bits; Set() of an index that would      */
/* break the span fails; Difference() is the signed 32-bit difference. */
/* ------------------------------------------------------------------ */
double or_time_delta(or_time a, or_time b)
{
    return (double)(a.sec - b.sec) + 1.0e-06 * (double)(a.usec - b.usec);
}

static void time_add(or_time* t, double s)
{
    double whole = floor(s);
    int64_t us = (int64_t)((s - whole) * 1.0e06 + 0.5);
    t->sec += (int64_t)whole;
    t->usec += us;
    while (t->usec >= 1000000) { t->usec -= 1000000; t->sec += 1; }
}

static int time_ge(or_time a, or_time b)
{
    return (a.sec > b.sec) || (a.sec == b.sec && a.usec >= b.usec);
}

static int32_t mask_diff(uint32_t a, uint32_t b) { return (int32_t)(a - b); }

static int mask_bit(const or_analytic* a, uint32_t i) { return (a->bits[i >> 3] >> (i & 7)) & 1; }
static void mask_setbit(or_analytic* a, uint32_t i) { a->bits[i >> 3] |= (uint8_t)(1u << (i & 7)); }
static void mask_clrbit(or_analytic* a, uint32_t i) { a->bits[i >> 3] &= (uint8_t)~(1u << (i & 7)); }

static uint32_t mask_last(const or_analytic* a)
{
    for (int32_t i = (int32_t)a->depth - 1; i >= 0; i--)
        if (mask_bit(a, (uint32_t)i)) return a->first + (uint32_t)i;
    return a->first;
}

static int mask_test(const or_analytic* a, uint32_t idx)
{
    if (!a->nset) return 0;
    int32_t d = mask_diff(idx, a->first);
    if (d < 0 || (uint32_t)d >= a->depth) return 0;
    return mask_bit(a, (uint32_t)d);
}

static void mask_clear(or_analytic* a)
{
    memset(a->bits, 0, sizeof(a->bits));
    a->nset = 0;
}

static int mask_set(or_analytic* a, uint32_t idx)
{
    if (!a->nset) {
        memset(a->bits, 0, sizeof(a->bits));
        a->first = idx;
        mask_setbit(a, 0);
        a->nset = 1;
        return 1;
    }
    int32_t d = mask_diff(idx, a->first);
    if (d >= 0) {
        if ((uint32_t)d >= a->depth) return 0;
        if (!mask_bit(a, (uint32_t)d)) { mask_setbit(a, (uint32_t)d); a->nset++; }
        return 1;
    }
    /* precedes first: allowed while the span stays < depth */
    uint32_t last = mask_last(a);
    uint32_t span = (uint32_t)mask_diff(last, idx);
    if (span >= a->depth) return 0;
    uint32_t shift = (uint32_t)(-d);
    uint8_t nb[1024 / 8];
    memset(nb, 0, sizeof(nb));
    for (uint32_t i = 0; i + shift < a->depth; i++)
        if (mask_bit(a, i)) nb[(i + shift) >> 3] |= (uint8_t)(1u << ((i + shift) & 7));
    memcpy(a->bits, nb, sizeof(nb));
    a->first = idx;
    mask_setbit(a, 0);
    a->nset++;
    return 1;
}

static void mask_unset_bits(or_analytic* a, uint32_t idx, uint32_t count)
{
    if (!a->nset) return;
    /* clear every set index x with idx <= x < idx + count (mod 2^32) */
    for (uint32_t i = 0; i < a->depth; i++) {
        if (!mask_bit(a, i)) continue;
        if ((uint32_t)(a->first + i - idx) < count) {
            mask_clrbit(a, i);
            a->nset--;
        }
    }
    if (!a->nset) { mask_clear(a); return; }
    /* re-base on the new first set bit */
    uint32_t s = 0;
    while (!mask_bit(a, s)) s++;
    if (s) {
        uint8_t nb[1024 / 8];
        memset(nb, 0, sizeof(nb));
        for (uint32_t i = s; i < a->depth; i++)
            if (mask_bit(a, i)) nb[(i - s) >> 3] |= (uint8_t)(1u << ((i - s) & 7));
        memcpy(a->bits, nb, sizeof(nb));
        a->first += s;
    }
}

/* Report::QuantizeTimeValue / UnquantizeTimeValue (mgenAnalytic.cpp:621-642) */
double or_quantized_window(double value)
{
    const double STRETCH = 1.1, TMIN = 1.0e-06, TMAX = 600.0;
    const double SCALE = 1.0 / (pow(STRETCH, 254) - STRETCH);
    unsigned q;
    if (value > STRETCH * TMAX) q = 0xff;
    else if (value < TMIN / 2.0) q = 0;
    else if (value < TMIN) q = 1;
    else q = (uint8_t)((log(STRETCH + (value - TMIN) / (SCALE * (TMAX - TMIN))) / log(STRETCH)) + 0.5);
    if (q == 0) return 0.0;
    return (TMAX - TMIN) * (pow(STRETCH, q) - STRETCH) * SCALE + TMIN;
}

/* MgenAnalytic::MgenAnalytic / Init (mgenAnalytic.cpp:8-71), DEFAULT_HISTORY 1024 */
void or_analytic_init(or_analytic* a, double window)
{
    memset(a, 0, sizeof(*a));
    a->depth = 1024;
    a->window_size = or_quantized_window(window);
}

/* MgenAnalytic::Update (mgenAnalytic.cpp:74-258) */
int or_analytic_update(or_analytic* a, or_time rx, uint32_t msgSize, or_time tx, uint32_t seq)
{
    if (!a->window_valid) {
        a->window_valid = 1;
        a->window_start = rx;
        a->window_end = rx;
        time_add(&a->window_end, a->window_size);
        if (msgSize != 0) {
            mask_set(a, seq);
            a->seq_start = seq;
            a->msg_count = 1;
            a->byte_count = msgSize;
            a->latency_sum = a->latency_min = a->latency_max = or_time_delta(rx, tx);
        } else {
            a->msg_count = a->byte_count = 0;
            a->latency_sum = a->latency_min = a->latency_max = 0.0;
        }
        return 0;
    }
    double latency = 0.0;
    if (msgSize != 0) {
        if (a->nset) {
            if (mask_test(a, seq)) {
                a->dup_msg_count++;
            } else if (mask_diff(seq, a->seq_start) < 0) {
                mask_set(a, seq);
            } else {
                if (!mask_set(a, seq)) {
                    uint32_t firstSet = a->first;
                    uint32_t numBits = (uint32_t)mask_diff(seq, firstSet);
                    mask_unset_bits(a, firstSet, numBits);
                    mask_set(a, seq);
                }
                if (1 == a->msg_count)
                    a->byte_count = msgSize;
                else
                    a->byte_count += msgSize;
                latency = or_time_delta(rx, tx);
                if (0 == a->msg_count) {
                    a->latency_sum = a->latency_min = a->latency_max = latency;
                } else {
                    a->latency_sum += latency;
                    if (latency < a->latency_min)
                        a->latency_min = latency;
                    else if (latency > a->latency_max)
                        a->latency_max = latency;
                }
                a->msg_count++;
            }
        } else {
            mask_clear(a);
            mask_set(a, seq);
            a->seq_start = seq;
            a->byte_count = msgSize;
            a->latency_sum = a->latency_min = a->latency_max = or_time_delta(rx, tx);
            a->msg_count = 1;
        }
    }
    if (time_ge(rx, a->window_end)) {
        a->report_valid = 1;
        a->n_reports++;
        a->report_start = a->window_start;
        a->report_duration = or_time_delta(rx, a->window_start);
        uint32_t seqMax = a->nset ? mask_last(a) : a->seq_start;
        switch (a->msg_count) {
            case 0:
                a->report_msg_count = 0;
                a->report_rate_ave = 0.0;
                a->report_loss_ave = 1.0;
                a->report_latency_ave = a->report_latency_min = a->report_latency_max = -1.0;
                break;
            case 1:
                a->report_msg_count = 1;
                a->report_rate_ave = (double)a->byte_count / a->report_duration;
                a->report_loss_ave = 0.0;
                a->report_latency_ave = a->latency_sum;
                a->report_latency_min = a->latency_min;
                a->report_latency_max = a->latency_max;
                break;
            default: {
                a->report_msg_count = a->msg_count - 1;
                a->report_rate_ave = (double)a->byte_count / a->report_duration;
                uint32_t seqDelta = seqMax - a->seq_start;
                if (seqDelta <= 1)
                    a->report_loss_ave = 0.0;
                else
                    a->report_loss_ave = 1.0 - (double)a->msg_count / (double)(seqDelta + 1);
                a->report_latency_ave = a->latency_sum / (double)a->msg_count;
                a->report_latency_min = a->latency_min;
                a->report_latency_max = a->latency_max;
                break;
            }
        }
        a->window_start = rx;
        a->window_end = rx;
        time_add(&a->window_end, a->window_size);
        a->seq_start = seqMax;
        if (msgSize != 0) {
            a->byte_count = 0;
            a->msg_count = 1;
            a->latency_sum = a->latency_min = a->latency_max = latency;
        } else {
            a->byte_count = a->msg_count = 0;
            a->latency_sum = a->latency_min = a->latency_max = 0.0;
        }
        return 1;
    }
    return 0;
}

void or_flow_reduce_batch(or_analytic* flows, uint32_t n_flows, const uint32_t* flow_idx,
                          const uint32_t* seq, const uint32_t* tx_sec, const uint32_t* tx_usec,
                          const uint16_t* msg_len, const uint32_t* rx_sec,
                          const uint32_t* rx_usec, uint32_t n, or_report* reports,
                          uint32_t cap, uint32_t* counts)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t f = flow_idx[i];
        if (f >= n_flows) continue;
        or_analytic* a = &flows[f];
        or_time rx = {(int64_t)rx_sec[i], (int64_t)rx_usec[i]};
        or_time tx = {(int64_t)tx_sec[i], (int64_t)tx_usec[i]};
        if (or_analytic_update(a, rx, msg_len[i], tx, seq[i])) {
            const uint32_t k = counts[f]++;
            if (k < cap) {
                or_report* r = &reports[(size_t)f * cap + k];
                r->flow = f;
                r->index = k;
                r->start_sec = a->report_start.sec;
                r->start_usec = a->report_start.usec;
                r->duration = a->report_duration;
                r->msg_count = a->report_msg_count;
                r->rate = a->report_rate_ave;
                r->loss = a->report_loss_ave;
                r->latency_ave = a->report_latency_ave;
                r->latency_min = a->report_latency_min;
                r->latency_max = a->report_latency_max;
                r->rx_sec = rx.sec;
                r->rx_usec = rx.usec;
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* Batch layer                                                         */
/* ------------------------------------------------------------------ */
#include <pthread.h>
#include <stdlib.h>

/* A double d with (UINT32)((d + 180.0) * 60000.0) == raw, so Pack's own conversion
 * (mgenMsg.cpp:221,225) reproduces the template's raw word exactly. */
static double raw_to_deg(uint32_t raw)
{
    double d = (double)raw / 60000.0 - 180.0;
    for (int k = 0; k < 64 && (uint32_t)((d + 180.0) * 60000.0) < raw; k++) d = nextafter(d, 1e300);
    for (int k = 0; k < 64 && (uint32_t)((d + 180.0) * 60000.0) > raw; k++) d = nextafter(d, -1e300);
    return d;
}

static void tmpl_to_msg(const or_tmpl* t, const or_desc* d, const uint8_t* pool, or_msg* m)
{
    memset(m, 0, sizeof(*m));
    m->msg_len = d->msg_len;
    m->mgen_msg_len = d->msg_len;
    m->version = OR_VERSION;
    m->flags = d->flags;
    m->flow_id = t->flow_id;
    m->seq_num = d->seq_num;
    m->tx_sec = d->tx_sec;
    m->tx_usec = d->tx_usec;
    m->dst.type = t->dst_type; m->dst.len = t->dst_len; m->dst.port = t->dst_port;
    memcpy(m->dst.addr, t->dst_addr, 16);
    m->host.type = t->host_type; m->host.len = t->host_len; m->host.port = t->host_port;
    memcpy(m->host.addr, t->host_addr, 16);
    /* the template carries the already-converted raw words; invert exactly:
     * raw/60000 - 180 reproduces the same (UINT32)((x+180)*60000) for raw < 2^32 */
    m->latitude = raw_to_deg(t->lat_raw);
    m->longitude = raw_to_deg(t->lon_raw);
    m->altitude = t->alt;
    m->gps_status = t->gps_status;
    m->payload_type = t->payload_type;
    m->payload_len = t->payload_len;
    m->payload_data = t->has_payload ? pool + t->payload_off : NULL;
}

void or_udp_pack_batch(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                       const uint8_t* pool, uint8_t* slab, const uint64_t* rec_off,
                       uint64_t stride, int checksum_enable, int random_fill, uint32_t fill_time,
                       uint32_t* out_len)
{
    for (uint32_t i = 0; i < n; i++) {
        or_msg m;
        tmpl_to_msg(&tmpl[desc[i].tmpl], &desc[i], pool, &m);
        uint64_t off = rec_off ? rec_off[i] : (uint64_t)i * stride;
        /* Pack works in the transport's scratch txBuffer (mgenTransport.cpp:1023); a failed
         * Pack (return 0) is never sent, so its slot in the batch slab stays untouched. */
        static uint8_t scratch[65536 + 512];
        out_len[i] = or_udp_pack(&m, scratch, checksum_enable, random_fill, fill_time);
        if (out_len[i]) memcpy(slab + off, scratch, out_len[i]);
    }
}

typedef struct {
    const uint8_t* slab; const uint64_t* rec_off; uint64_t stride;
    const uint32_t* rec_len; uint32_t fixed_len; uint32_t lo, hi; int force; or_fields* out;
} recv_job;

static void* recv_worker(void* p)
{
    recv_job* j = (recv_job*)p;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        uint64_t off = j->rec_off ? j->rec_off[i] : (uint64_t)i * j->stride;
        uint32_t len = j->rec_len ? j->rec_len[i] : j->fixed_len;
        if (j->force & 2)
            or_tcp_recv(j->slab + off, len, j->force & 1, &j->out[i]);
        else
            or_udp_recv(j->slab + off, len, j->force & 1, &j->out[i]);
    }
    return NULL;
}

void or_udp_recv_batch(const uint8_t* slab, const uint64_t* rec_off, uint64_t stride,
                       const uint32_t* rec_len, uint32_t fixed_len, uint32_t n,
                       int checksum_force, or_fields* out, int nthreads)
{
    (void)table();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    recv_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t].slab = slab; jobs[t].rec_off = rec_off; jobs[t].stride = stride;
        jobs[t].rec_len = rec_len; jobs[t].fixed_len = fixed_len;
        jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
        jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        jobs[t].force = checksum_force; jobs[t].out = out;
    }
    if (nthreads == 1) { recv_worker(&jobs[0]); return; }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, recv_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ---- CPU baselines on several cores (bench.py's cpu_baseline leg) ----
 * The reference runs one dispatcher thread; these spread the same per-record work over
 * nthreads host threads to report what all the cores of the box do: contiguous record ranges
 * for Pack (UDP send sequence, zero fill: RANDOM_FILL's rand() is process-global state) and
 * flows split by index (f mod nthreads: each thread walks the records in receive order and
 * updates only its flows, so per-flow order is kept). */
typedef struct {
    const or_tmpl* tmpl; const or_desc* desc; const uint8_t* pool; uint8_t* slab;
    const uint64_t* rec_off; uint64_t stride; int ck; uint32_t* out_len; uint32_t lo, hi;
} pack_job;

static void* pack_worker(void* p)
{
    pack_job* j = (pack_job*)p;
    uint8_t* scratch = (uint8_t*)malloc(65536 + 512);
    for (uint32_t i = j->lo; i < j->hi; i++) {
        or_msg m;
        tmpl_to_msg(&j->tmpl[j->desc[i].tmpl], &j->desc[i], j->pool, &m);
        const uint64_t off = j->rec_off ? j->rec_off[i] : (uint64_t)i * j->stride;
        j->out_len[i] = or_udp_pack(&m, scratch, j->ck, 0, 0);
        if (j->out_len[i]) memcpy(j->slab + off, scratch, j->out_len[i]);
    }
    free(scratch);
    return NULL;
}

void or_udp_pack_batch_mt(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                          const uint8_t* pool, uint8_t* slab, const uint64_t* rec_off,
                          uint64_t stride, int checksum_enable, uint32_t* out_len, int nthreads)
{
    (void)table();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pack_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        pack_job* j = &jobs[t];
        j->tmpl = tmpl; j->desc = desc; j->pool = pool; j->slab = slab; j->rec_off = rec_off;
        j->stride = stride; j->ck = checksum_enable; j->out_len = out_len;
        j->lo = (uint32_t)((uint64_t)n * t / nthreads);
        j->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
    }
    if (nthreads == 1) { pack_worker(&jobs[0]); return; }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, pack_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

typedef struct {
    or_analytic* flows; uint32_t n_flows; const uint32_t* idx; const uint32_t* seq;
    const uint32_t* txs; const uint32_t* txu; const uint16_t* len; const uint32_t* rxs;
    const uint32_t* rxu; uint32_t n, t, nt; uint32_t* counts;
} flow_job;

static void* flow_worker(void* p)
{
    flow_job* j = (flow_job*)p;
    for (uint32_t i = 0; i < j->n; i++) {
        const uint32_t f = j->idx[i];
        if (f >= j->n_flows || f % j->nt != j->t) continue;
        or_time rx = {(int64_t)j->rxs[i], (int64_t)j->rxu[i]};
        or_time tx = {(int64_t)j->txs[i], (int64_t)j->txu[i]};
        if (or_analytic_update(&j->flows[f], rx, j->len[i], tx, j->seq[i])) j->counts[f]++;
    }
    return NULL;
}

void or_flow_reduce_batch_mt(or_analytic* flows, uint32_t n_flows, const uint32_t* flow_idx,
                             const uint32_t* seq, const uint32_t* tx_sec, const uint32_t* tx_usec,
                             const uint16_t* msg_len, const uint32_t* rx_sec,
                             const uint32_t* rx_usec, uint32_t n, uint32_t* counts, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    flow_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        flow_job* j = &jobs[t];
        j->flows = flows; j->n_flows = n_flows; j->idx = flow_idx; j->seq = seq;
        j->txs = tx_sec; j->txu = tx_usec; j->len = msg_len; j->rxs = rx_sec; j->rxu = rx_usec;
        j->n = n; j->t = (uint32_t)t; j->nt = (uint32_t)nthreads; j->counts = counts;
    }
    if (nthreads == 1) { flow_worker(&jobs[0]); return; }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, flow_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

uint64_t or_tcp_tx_batch(const or_tmpl* tmpl, const or_desc* desc, const uint32_t* msg_total,
                         uint32_t n, const uint8_t* pool, uint8_t* stream,
                         int checksum_enable, int random_fill, uint32_t fill_time)
{
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; i++) {
        or_msg m;
        tmpl_to_msg(&tmpl[desc[i].tmpl], &desc[i], pool, &m);
        m.mgen_msg_len = msg_total[i];
        m.msg_len = (uint16_t)(msg_total[i] > 65535 ? 65535 : msg_total[i]);
        p += or_tcp_tx(&m, stream + p, checksum_enable, random_fill, fill_time);
    }
    return p;
}

/* layout check for the Python/ctypes mirrors */
uint32_t or_sizeof(int which)
{
    if (which == 100) return (uint32_t)sizeof(or_report);
    if (which == 101) return (uint32_t)sizeof(or_analytic);
    switch (which) {
        case 0: return (uint32_t)sizeof(or_tmpl);
        case 1: return (uint32_t)sizeof(or_desc);
        case 2: return (uint32_t)sizeof(or_fields);
        case 3: return (uint32_t)sizeof(or_analytic);
        default: return 0;
    }
}

/* ------------------------------------------------------------------ */
/* RECV / RERR text log lines                                          */
/*   MgenMsg::LogRecvEvent text branch  mgenMsg.cpp:1034-1102          */
/*   MgenMsg::LogRecvError text branch  mgenMsg.cpp:711-735            */
/*   Mgen::LogLegacyTimestamp / LogEpochTimestamp  mgen.cpp:55-83      */
/* as glibc formats the reference's fprintf calls on x86-64.  Two ABI  */
/* details are pinned by the doc's own output (doc/mgen.xml:2948):     */
/* "%ld" of the INT32 altitude receives it zero-extended (-999 prints  */
/* as 4294966297), and hex payload digits are upper case.              */
/* ProtoAddress::GetHostString (protolib, absent) is taken as          */
/* inet_ntop: "dotted decimal IPv4 addresses or colon-delimited IPv6   */
/* addresses" (doc/mgen.xml:3674-3675) -- unpinned beyond IPv4.        */
/* ------------------------------------------------------------------ */
#include <arpa/inet.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static int log_ts(char* out, uint32_t sec, uint32_t usec, int epoch)
{
    if (epoch) return sprintf(out, "%lu.%06lu ", (unsigned long)sec, (unsigned long)usec);
    time_t t = (time_t)sec;
    struct tm tmv;
    gmtime_r(&t, &tmv);
    return sprintf(out, "%02d:%02d:%02d.%06lu ", tmv.tm_hour, tmv.tm_min, tmv.tm_sec,
                   (unsigned long)usec);
}

static int log_addr(char* out, uint8_t type, uint8_t len, const uint8_t* addr)
{
    char s[64];
    if (type == OR_ADDR_IPV6 && len == 16) inet_ntop(AF_INET6, addr, s, sizeof s);
    else if (type == OR_ADDR_IPV4 && len == 4) inet_ntop(AF_INET, addr, s, sizeof s);
    else strcpy(s, "(invalid)");   /* protolib behaviour for other lengths: unpinned */
    return sprintf(out, "%s", s);
}

static const char* log_proto(int protocol)
{
    switch (protocol) {   /* MgenBaseEvent::PROTOCOL_LIST, mgenEvent.cpp:75-81, 116-126 */
        case 1: return "UDP";
        case 2: return "TCP";
        case 3: return "SINK";
        default: return "UNKNOWN";
    }
}

uint32_t or_log_recv_text(const or_fields* f, const uint8_t* rec, const or_addr* src,
                          uint32_t rx_sec, uint32_t rx_usec, int protocol, int ttl,
                          uint32_t opts, char* out)
{
    const int epoch = (opts & OR_LOG_EPOCH) != 0;
    char* p = out;
    if (!f->ok || f->err) {          /* RERR (mgenTransport.cpp:976-979, 990-994) */
        static const char* names[5] = {"none", "version", "checksum", "length", "dstAddr"};
        p += log_ts(p, rx_sec, rx_usec, epoch);
        p += sprintf(p, "RERR type>%s src>", f->err <= 4 ? names[f->err] : "");
        p += log_addr(p, src->type, src->len, src->addr);
        p += sprintf(p, "/%hu\n", src->port);
        return (uint32_t)(p - out);
    }
    p += log_ts(p, rx_sec, rx_usec, epoch);
    p += sprintf(p, "RECV proto>%s flow>%lu seq>%lu src>", log_proto(protocol),
                 (unsigned long)f->flow_id, (unsigned long)f->seq_num);
    p += log_addr(p, src->type, src->len, src->addr);
    p += sprintf(p, "/%hu dst>", src->port);
    p += log_addr(p, f->dst_type, f->dst_len, f->dst_addr);
    p += sprintf(p, "/%hu sent>", f->dst_port);
    p += log_ts(p, f->tx_sec, f->tx_usec, epoch);
    p += sprintf(p, "size>%u ", (unsigned)f->msg_len);
    if (f->host_type == OR_ADDR_IPV4 || f->host_type == OR_ADDR_IPV6) {
        p += sprintf(p, "host>");
        p += log_addr(p, f->host_type, f->host_len, f->host_addr);
        p += sprintf(p, "/%hu ", f->host_port);
    }
    if (ttl >= 0) p += sprintf(p, "ttl>%d ", ttl);
    const char* status;
    switch (f->gps_status) {
        case 0: status = "INVALID"; break;
        case 1: status = "STALE"; break;
        case 2: status = "CURRENT"; break;
        default:                      /* mgenMsg.cpp:1068-1071: newline, nothing more */
            p += sprintf(p, "\n");
            return (uint32_t)(p - out);
    }
    if (!(opts & OR_LOG_NO_GPS)) {
        const double lat = ((double)f->lat_raw) / 60000.0 - 180.0;   /* mgenMsg.cpp:453 */
        const double lon = ((double)f->lon_raw) / 60000.0 - 180.0;   /* mgenMsg.cpp:457 */
        p += sprintf(p, "gps>%s,%f,%f,%lu ", status, lat, lon,
                     (unsigned long)(uint32_t)f->alt);
    }
    if (f->payload_len && !(opts & OR_LOG_NO_DATA) && f->payload_type == 0) {  /* USER_DATA */
        static const char hx[] = "0123456789ABCDEF";   /* MgenPayload::toHex */
        p += sprintf(p, "data>%hu:", f->payload_len);
        const uint8_t* d = rec + f->payload_off;          /* payload_data (word floor) */
        for (uint32_t i = 0; i < f->payload_len; i++) {
            *p++ = hx[d[i] >> 4];
            *p++ = hx[d[i] & 15];
        }
        *p++ = ' ';
    }
    if (f->flags & OR_FLAG_CONTINUES) p += sprintf(p, "flags>0x%02x ", OR_FLAG_CONTINUES);
    if (f->flags & OR_FLAG_END_OF_MSG) p += sprintf(p, "flags>0x%02x ", OR_FLAG_END_OF_MSG);
    if (f->flags & OR_FLAG_CHECKSUM_ERROR) p += sprintf(p, "flags>0x%02x ", OR_FLAG_CHECKSUM_ERROR);
    p += sprintf(p, "\n");
    return (uint32_t)(p - out);
}

/* ------------------------------------------------------------------ */
/* Binary RECV / RERR log records                                     */
/*   MgenMsg::LogRecvEvent binary branch  mgenMsg.cpp:958-1033        */
/*   MgenMsg::LogRecvError binary branch  mgenMsg.cpp:652-710         */
/* RECV: eventType, protocol, BE recordLength = 12 + srcLen + hdr +    */
/* payload_len, BE rx sec/usec, BE src port, src type/len/address,     */
/* then recordLength - index + 4 message bytes, index = 16 + srcLen   */
/* (the 4-byte record header, 8 time, 2 port, type, length, address): */
/* hdr + payload_len bytes, as eventRecordLength counts from after the */
/* header (doc/mgen.xml:4212-4216), with CHECKSUM cleared in the flags */
/* byte (CHECKSUM_ERROR set when flagged).  avail = the received bytes */
/* of the record (the receive buffer); bytes past it read as zero here */
/* (the reference's buffer holds stale bytes there).                   */
/* ------------------------------------------------------------------ */
static uint32_t put_be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; return 2; }
static uint32_t put_be32(uint8_t* p, uint32_t v) { put32(p, v); return 4; }

uint32_t or_log_recv_binary(const or_fields* f, const uint8_t* rec, uint64_t avail,
                            const or_addr* src, uint32_t rx_sec, uint32_t rx_usec, int protocol,
                            uint8_t* out)
{
    uint8_t* p = out;
    const uint32_t alen = (src->type == OR_ADDR_IPV4 || src->type == OR_ADDR_IPV6) ? src->len : 0;
    const uint8_t atype = (src->type == OR_ADDR_IPV4 || src->type == OR_ADDR_IPV6) ? src->type : 0;
    if (!f->ok || f->err) {
        *p++ = 2;                                   /* RERR_EVENT */
        *p++ = 0;
        p += put_be16(p, 12 + alen + 4);
        p += put_be32(p, rx_sec);
        p += put_be32(p, rx_usec);
        p += put_be16(p, src->port);
        *p++ = atype;
        *p++ = (uint8_t)alen;
        memcpy(p, src->addr, alen); p += alen;
        p += put_be32(p, f->err);
        return (uint32_t)(p - out);
    }
    const uint32_t rl = (12 + alen + f->hdr_len + f->payload_len) & 0xFFFF;
    *p++ = 1;                                       /* RECV_EVENT */
    *p++ = (uint8_t)protocol;
    p += put_be16(p, rl);
    p += put_be32(p, rx_sec);
    p += put_be32(p, rx_usec);
    p += put_be16(p, src->port);
    *p++ = atype;
    *p++ = (uint8_t)alen;
    memcpy(p, src->addr, alen); p += alen;
    const uint32_t index = 16 + alen;
    const uint32_t ml = (rl - index + 4) & 0xFFFF;
    for (uint32_t i = 0; i < ml; i++) {
        uint8_t b = i < avail ? rec[i] : 0;
        if (i == 3) {
            b &= (uint8_t)~OR_FLAG_CHECKSUM;
            if (f->flags & OR_FLAG_CHECKSUM_ERROR) b |= OR_FLAG_CHECKSUM_ERROR;
        }
        *p++ = b;
    }
    return (uint32_t)(p - out);
}

/* ------------------------------------------------------------------ */
/* SEND events: MgenMsg::LogSendEvent (mgenMsg.cpp:1145-1241), as the UDP / SINK send   */
/* path logs them after a successful send (mgenTransport.cpp:1060: theTime = the        */
/* message's tx time; the message's src port = the flow transport's port,              */
/* mgenFlow.cpp:975-977).  Binary: bytes past the packed message (the transport's      */
/* stale txBuffer) read as zero here: unpinned.                                        */
/* ------------------------------------------------------------------ */
static uint32_t addr_length(uint8_t type) { return type == OR_ADDR_IPV4 ? 4u : (type == OR_ADDR_IPV6 ? 16u : 0u); }

uint32_t or_log_send_text(const or_tmpl* t, const or_desc* d, uint16_t src_port, int protocol,
                          uint32_t mgen_msg_len, uint32_t opts, char* out)
{
    char* p = out;
    p += log_ts(p, d->tx_sec, d->tx_usec, (opts & OR_LOG_EPOCH) != 0);
    p += sprintf(p, "SEND proto>%s flow>%lu seq>%lu srcPort>%hu dst>", log_proto(protocol),
                 (unsigned long)t->flow_id, (unsigned long)d->seq_num, src_port);
    p += log_addr(p, t->dst_type, t->dst_len, t->dst_addr);
    p += sprintf(p, "/%hu", t->dst_port);
    if (protocol == 2) p += sprintf(p, " size>%lu ", (unsigned long)mgen_msg_len);
    else p += sprintf(p, " size>%u ", (unsigned)d->msg_len);
    if (t->host_type == OR_ADDR_IPV4 || t->host_type == OR_ADDR_IPV6) {
        p += sprintf(p, "host>");
        p += log_addr(p, t->host_type, t->host_len, t->host_addr);
        p += sprintf(p, "/%hu\n", t->host_port);
    } else {
        p += sprintf(p, "\n");
    }
    return (uint32_t)(p - out);
}

uint32_t or_log_send_binary(const or_tmpl* t, const uint8_t* packed, uint32_t packed_len,
                            uint32_t hdr_len, int protocol, uint32_t mgen_msg_len, uint8_t* out)
{
    uint8_t* p = out;
    uint32_t rl = 12 + addr_length(t->dst_type) + hdr_len;
    if (t->host_type == OR_ADDR_IPV4 || t->host_type == OR_ADDR_IPV6) rl += addr_length(t->host_type) + 4;
    if (protocol == 2) rl += 4;
    rl &= 0xFFFF;                                   /* UINT16 recordLength */
    *p++ = 3;                                       /* SEND_EVENT */
    *p++ = (uint8_t)protocol;
    p += put_be16(p, rl);
    uint32_t index = 4;
    if (protocol == 2) { p += put_be32(p, mgen_msg_len); index += 4; }
    const uint32_t ml = (rl - index + 4) & 0xFFFF;
    for (uint32_t i = 0; i < ml; i++) {
        uint8_t b = i < packed_len ? packed[i] : 0;
        if (i == 3) b &= (uint8_t)~OR_FLAG_CHECKSUM;   /* "Clear CHECKSUM flag for binary logging" */
        *p++ = b;
    }
    return (uint32_t)(p - out);
}

/* The SEND events of n records sent by the UDP / SINK path (or_udp_pack_batch's records;
 * a failed Pack is never sent, so never logged).  binary: 0 text, 1 binary.  Returns the
 * bytes written to out. */
uint64_t or_log_send_batch(const or_tmpl* tmpl, const or_desc* desc, uint32_t n,
                           const uint8_t* pool, const uint16_t* src_port, int protocol,
                           int checksum_enable, uint32_t opts, int binary, uint8_t* out)
{
    static uint8_t buf[65536 + 512];
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
        or_msg m;
        tmpl_to_msg(&tmpl[desc[i].tmpl], &desc[i], pool, &m);
        uint32_t tx = 0;
        uint16_t hl = 0;
        m.flags |= OR_FLAG_LAST_BUFFER;
        const uint32_t len = or_pack(&m, buf, m.msg_len, checksum_enable, &tx, 0, 0, &hl);
        if (len == 0) continue;
        if (checksum_enable && (m.flags & OR_FLAG_CHECKSUM)) or_write_checksum(&tx, buf, len);
        const or_tmpl* t = &tmpl[desc[i].tmpl];
        if (binary)
            pos += or_log_send_binary(t, buf, len, hl, protocol, m.mgen_msg_len, out + pos);
        else
            pos += or_log_send_text(t, &desc[i], src_port[desc[i].tmpl], protocol, m.mgen_msg_len,
                                    opts, (char*)out + pos);
    }
    return pos;
}

/* ------------------------------------------------------------------ */
/* MGEN_DATA items: MgenAnalytic::Report and MgenFlowCommand           */
/*   quantizers          mgenAnalytic.cpp:568-642                      */
/*   Report build        Init :28-71, Update :220-254, GetReport :296-310, */
/*                       InitIntoBuffer/SetDstAddr/SetSrcAddr/SetFlowId :446-566 */
/*   Report parse        InitFromBuffer :343-373, getters mgenAnalytic.h:167-220 */
/*   REPORT log lines    MgenAnalytic::Log :260-295, Report::Log :747-786 */
/*   TLV walk            MgenTransport::ProcessRecvMessage mgenTransport.cpp:2132-2191 */
/*   flow commands       MgenFlowCommand mgenPayload.cpp:276-347, MAX_FLOW mgenEvent.h:194 */
/* ProtoPkt getters/setters are network byte order.                    */
/* ------------------------------------------------------------------ */
static const double RQ_STRETCH = 1.1, RQ_MIN = 1.0e-06, RQ_MAX = 600.0;

static double rq_scale(void) { return 1.0 / (pow(RQ_STRETCH, 254) - RQ_STRETCH); }

uint8_t or_q_time(double value)
{
    if (value > RQ_STRETCH * RQ_MAX) return 0xff;
    else if (value < RQ_MIN / 2.0) return 0;
    else if (value < RQ_MIN) return 1;
    return (uint8_t)((log(RQ_STRETCH + (value - RQ_MIN) / (rq_scale() * (RQ_MAX - RQ_MIN))) /
                      log(RQ_STRETCH)) + 0.5);
}

double or_uq_time(uint8_t q)
{
    if (0 == q) return 0.0;
    return (RQ_MAX - RQ_MIN) * (pow(RQ_STRETCH, q) - RQ_STRETCH) * rq_scale() + RQ_MIN;
}

uint16_t or_q_rate(double rate)
{
    if (rate <= 0.0) return 0x01;
    /* (UINT16)log10(rate): x86-64 gcc converts through int32, so log10 < 0 wraps */
    uint16_t exponent = (uint16_t)(int32_t)log10(rate);
    uint16_t mantissa = (uint16_t)(int32_t)((4096.0 / 10.0) * (rate / pow(10.0, (double)exponent)) + 0.5);
    return (uint16_t)((mantissa << 4) | exponent);
}

double or_uq_rate(uint16_t q)
{
    double mantissa = ((double)(q >> 4)) * (10.0 / 4096.0);
    double exponent = (double)(q & 0x000f);
    return mantissa * pow(10.0, exponent);
}

uint16_t or_q_loss(double loss)
{
    if (0.0 == loss) return 0;
    loss = loss * 65535.0 + 0.5;
    if (loss < 1.0) return 1;
    else if (loss > 65535.0) return 65535;
    return (uint16_t)loss;
}

double or_uq_loss(uint16_t q) { return ((double)q) / 65535.0; }

static void put16be(uint8_t* p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static uint16_t get16be(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

/* offsets of a report whose type byte says addrLen and whose flags say flow id */
typedef struct { uint32_t alen, src, dport, sport, fid, ws, lave, lmin, lmax, rate, loss, end; } rep_off;
static rep_off rep_offsets(const uint8_t* b)
{
    rep_off o;
    const uint8_t type = b[0] >> 4;
    o.alen = type == 1 ? 4 : (type == 2 ? 16 : 0);
    o.src = 4 * (1 + o.alen / 4);
    o.dport = o.src + o.alen;
    o.sport = o.dport + 2;
    o.fid = o.sport + 2;
    o.ws = o.fid + (((b[2] >> 5) & 0x01) ? 4 : 0);
    o.lave = o.ws + 1; o.lmin = o.lave + 1; o.lmax = o.lmin + 1;
    o.rate = o.lmax + 1; o.loss = o.rate + 2; o.end = o.loss + 2;
    return o;
}

/* report_msg of an analytic (key) after Init and one window close, then GetReport(theTime):
 * offset < 0 leaves the window offset field 0.  *sign: FLAG_LATENCY_SIGN was set before (in)
 * / is set after (out) -- SetLatencyAve never clears it.  Returns the report length. */
uint32_t or_report_build(const or_addr* src, const or_addr* dst, uint32_t flow_id, int protocol,
                         double duration, double lat_ave, double lat_min, double lat_max,
                         double rate, double loss, double offset, int* sign, uint8_t* b)
{
    memset(b, 0, 52);
    /* InitIntoBuffer(REPORT_FLOW_IPv4): memset 16, type, length 16 */
    b[0] = (uint8_t)(1 << 4);
    b[1] = 16;
    uint32_t pkt_len = 16;
    b[0] = (uint8_t)((b[0] & 0xf0) | (protocol & 0x0f));            /* SetProtocol */
    const or_addr* addrs[2] = {dst, src};
    for (int k = 0; k < 2; k++) {                                   /* SetDstAddr, SetSrcAddr */
        const or_addr* a = addrs[k];
        uint32_t alen;
        uint8_t type;
        if (a->type == OR_ADDR_IPV4) { type = 1; alen = 4; }
        else if (a->type == OR_ADDR_IPV6) { type = 2; alen = 16; }
        else continue;                                               /* error: unchanged */
        const uint32_t rl = 12 + 4 + 2 * alen;
        b[0] = (uint8_t)((b[0] & 0x0f) | (type << 4));
        b[1] = (uint8_t)rl;
        rep_off o = rep_offsets(b);
        if (k == 0) { memcpy(b + 4, a->addr, alen); put16be(b + o.dport, a->port); }
        else { memcpy(b + o.src, a->addr, alen); put16be(b + o.sport, a->port); }
        pkt_len = rl;
    }
    if (flow_id != 1) {                                              /* SetFlowId */
        rep_off o = rep_offsets(b);
        const uint32_t rl = o.src + o.alen + 12 + 4;
        b[2] |= (uint8_t)(0x01 << 5);
        o = rep_offsets(b);
        put32(b + o.fid, flow_id);
        b[1] = (uint8_t)rl;
        pkt_len = rl;
    }
    rep_off o = rep_offsets(b);
    /* window close (:245-253); SetWindowSize at Init is overwritten here */
    b[o.ws] = or_q_time(duration);
    if (lat_ave < 0.0) *sign = 1;
    if (*sign) b[2] |= (uint8_t)(0x02 << 5);
    b[o.lave] = or_q_time(fabs(lat_ave));
    b[o.lmin] = or_q_time(fabs(lat_ave - lat_min));
    b[o.lmax] = or_q_time(fabs(lat_max - lat_ave));
    put16be(b + o.rate, or_q_rate(rate));
    put16be(b + o.loss, or_q_loss(loss));
    if (offset >= 0.0 || offset < 0.0) {                            /* GetReport */
        double off = offset < 0.0 ? 0.0 : offset;
        const uint16_t q = or_q_time(off);
        const uint16_t field = (uint16_t)((get16be(b + 2) & 0xe000) | q);
        put16be(b + 2, field);
    }
    (void)pkt_len;
    return (uint32_t)b[1];
}

typedef struct {
    uint8_t  valid, type, protocol, flags;
    uint32_t length;
    or_addr  src, dst;
    uint32_t flow_id;         /* GetFlowId(): 0 when the flag is clear */
    double   window_offset, window_size, lat_ave, lat_min, lat_max, rate, loss;
} or_report_view;

/* the getters over a report buffer as it is (no length check; report type 1 or 2) */
static void report_view(const uint8_t* b, or_report_view* v)
{
    const uint8_t type = b[0] >> 4;
    rep_off o = rep_offsets(b);
    v->type = type;
    v->protocol = b[0] & 0x0f;
    v->flags = b[2] >> 5;
    v->length = b[1];
    const uint8_t at = type == 1 ? OR_ADDR_IPV4 : OR_ADDR_IPV6;
    v->dst.type = at; v->dst.len = (uint8_t)o.alen; memcpy(v->dst.addr, b + 4, o.alen);
    v->dst.port = get16be(b + o.dport);
    v->src.type = at; v->src.len = (uint8_t)o.alen; memcpy(v->src.addr, b + o.src, o.alen);
    v->src.port = get16be(b + o.sport);
    v->flow_id = (v->flags & 0x01) ? get32(b + o.fid) : 0;
    v->window_offset = or_uq_time((uint8_t)(get16be(b + 2) & 0x1fff));
    v->window_size = or_uq_time(b[o.ws]);
    const double ave = or_uq_time(b[o.lave]);
    v->lat_ave = (v->flags & 0x02) ? -ave : ave;
    v->lat_min = v->lat_ave - or_uq_time(b[o.lmin]);
    v->lat_max = v->lat_ave + or_uq_time(b[o.lmax]);
    v->rate = or_uq_rate(get16be(b + o.rate));
    v->loss = or_uq_loss(get16be(b + o.loss));
}

/* Report::InitFromBuffer(buf, avail) and the getters */
int or_report_parse(const uint8_t* b, uint32_t avail, or_report_view* v)
{
    memset(v, 0, sizeof(*v));
    if (avail < 1) return 0;                                         /* OFFSET_LEN */
    const uint32_t min_len = avail > 1 ? b[1] : 0;
    if (min_len > avail) return 0;                                   /* ProtoPkt::InitFromBuffer */
    if (avail < 2) return 0;                                         /* OFFSET_FLAGS */
    const uint8_t type = b[0] >> 4;
    if (type != 1 && type != 2) return 0;
    rep_off o = rep_offsets(b);
    if (b[1] != o.end) return 0;
    report_view(b, v);
    v->valid = 1;
    return 1;
}

static const char* rep_proto(int p)
{
    switch (p) { case 1: return "UDP"; case 2: return "TCP"; case 3: return "SINK"; default: return "???"; }
}

/* MgenAnalytic::Log: the report_msg's key fields, the analytic's report doubles */
uint32_t or_log_report(const uint8_t* report, double duration, double rate, double loss,
                       double lat_ave, double lat_min, double lat_max, uint64_t count,
                       uint32_t sec, uint32_t usec, uint32_t opts, char* out)
{
    or_report_view v;
    char* p = out;
    /* the getters read the buffer as it is: a report whose addresses were invalid keeps
     * InitIntoBuffer's IPv4 type and length 16 (mgenAnalytic.cpp:63-67) */
    memset(&v, 0, sizeof v);
    report_view(report, &v);
    p += log_ts(p, sec, usec, (opts & OR_LOG_EPOCH) != 0);
    const unsigned long fid = v.flow_id ? v.flow_id : 1;
    p += sprintf(p, "REPORT proto>%s flow>%lu src>", rep_proto(v.protocol), fid);
    p += log_addr(p, v.src.type, v.src.len, v.src.addr);
    p += sprintf(p, "/%hu dst>", v.src.port);
    p += log_addr(p, v.dst.type, v.dst.len, v.dst.addr);
    p += sprintf(p, "/%hu ", v.dst.port);
    p += sprintf(p, "window>%lf rate>%lf kbps loss>%lf latency ave>%lf min>%lf max>%lf, count>%u\n",
                 duration, rate * 8.0e-03, loss, lat_ave, lat_min, lat_max, (unsigned)count);
    return (uint32_t)(p - out);
}

/* MgenAnalytic::Report::Log (a received report): "sent>" prints theTime, as the reference
 * does (mgenAnalytic.cpp:779) */
uint32_t or_log_report_recv(const uint8_t* report, const or_addr* reporter, uint32_t sec,
                            uint32_t usec, uint32_t opts, char* out)
{
    or_report_view v;
    char* p = out;
    or_report_parse(report, 52, &v);
    const int ep = (opts & OR_LOG_EPOCH) != 0;
    p += log_ts(p, sec, usec, ep);
    const unsigned long fid = v.flow_id ? v.flow_id : 1;
    p += sprintf(p, "REPORT proto>%s flow>%lu src>", rep_proto(v.protocol), fid);
    p += log_addr(p, v.src.type, v.src.len, v.src.addr);
    p += sprintf(p, "/%hu dst>", v.src.port);
    p += log_addr(p, v.dst.type, v.dst.len, v.dst.addr);
    p += sprintf(p, "/%hu reporter>", v.dst.port);
    p += log_addr(p, reporter->type, reporter->len, reporter->addr);
    p += sprintf(p, "/%hu sent>", reporter->port);
    p += log_ts(p, sec, usec, ep);
    p += sprintf(p, "offset>%lf ", v.window_offset);
    p += sprintf(p, "window>%lf rate>%lf kbps loss>%lf latency ave>%lf min>%lf max>%lf\n",
                 v.window_size, v.rate * 8.0e-03, v.loss, v.lat_ave, v.lat_min, v.lat_max);
    return (uint32_t)(p - out);
}

/* MgenFlowCommand::GetStatus(flowId) on an item of length len */
static int flowcmd_status(const uint8_t* b, uint32_t len, uint32_t flow_id)
{
    const uint32_t N = (2 * flow_id > 16) ? (2 * flow_id - 16 - 1) / 32 + 1 : 0;
    const uint32_t need = 2 + 2 + N * 4;
    if (need > len) return 0;
    const uint32_t f = flow_id - 1;
    int st = 0;
    if (b[2 + (f >> 3)] & (0x80 >> (f & 7))) st = 1;
    if (b[2 + (len - 2) / 2 + (f >> 3)] & (0x80 >> (f & 7))) st |= 2;
    return st;
}

/* MgenTransport::ProcessRecvMessage over one MGEN_DATA payload.  Flow commands with a
 * status other than FLOW_UNCHANGED go to cmds (flow id << 2 | status); with a controller,
 * report items (type byte > 0x0f) are parsed and their payload offsets go to reps.  Returns
 * 0 = walked to the end, 1 = invalid MGEN_DATA payload, 2 = invalid REPORT, 3 = an item of
 * length 0 (the reference loops forever there; the walk stops). */
int or_data_walk(const uint8_t* pay, uint32_t len, int controller, uint32_t* cmds,
                 uint32_t* n_cmds, uint32_t cap_cmds, uint32_t* reps, uint32_t* n_reps,
                 uint32_t cap_reps)
{
    uint32_t off = 0, left = len;
    *n_cmds = 0;
    *n_reps = 0;
    while (left > 0) {
        const uint8_t* b = pay + off;
        const uint8_t type = b[0];
        const uint32_t ilen = left > 1 ? b[1] : 0;   /* MgenDataItem::InitFromBuffer */
        if (type == 1) {                              /* DATA_ITEM_FLOW_CMD */
            if (ilen > left) return 1;
            uint32_t maxf = ilen > 2 ? 8 * (ilen - 2) / 2 : 0;
            if (maxf > 40) maxf = 40;                 /* MgenEvent::FlowStatus::MAX_FLOW */
            for (uint32_t i = 1; i <= maxf; i++) {
                const int st = flowcmd_status(b, ilen, i);
                if (st && *n_cmds < cap_cmds) cmds[(*n_cmds)++] = i << 2 | (uint32_t)st;
                else if (st) (*n_cmds)++;
            }
            if (ilen == 0) return 3;
            left -= ilen;
            off += (ilen / 4) * 4;
        } else if (controller && type > 0x0f) {
            or_report_view v;
            if (!or_report_parse(b, left, &v)) return 2;
            if (*n_reps < cap_reps) reps[*n_reps] = off;
            (*n_reps)++;
            left -= v.length;
            off += (v.length / 4) * 4;
        } else {
            if (ilen > left || ilen == 0) return 3;   /* GetLength() 0: no progress */
            left -= ilen;
            off += (ilen / 4) * 4;
        }
    }
    return 0;
}

/* ==== pcap2mgen (src/common/pcap2mgen.cpp:252-482) ====================================
 * The main loop over a pcap file image.  The frame walk restates protolib's ProtoPktETH /
 * ProtoPktIP / ProtoPktUDP, which is not vendored (parity unpinned at that layer): any
 * link type other than DLT_LINUX_SLL is read as Ethernet (the reference does the same,
 * :365-367), frames with hdr.len > 4094 are "invalid Ether frame" (the 4-KiB parse buffer,
 * :337-340, 369-373), an 802.1Q tag is stepped over, IPv4 needs IHL >= 5 and a total length
 * within the frame, IPv6 a payload length within it, UDP a length field within the IP payload.
 * A packet whose UDP payload lies past the captured bytes is skipped (the reference would
 * read stale bytes of its parse buffer there). */
static uint32_t pc_u32(const uint8_t* b, int sw)
{
    uint32_t v;
    memcpy(&v, b, 4);
    return sw ? __builtin_bswap32(v) : v;
}
static uint32_t pc_be16(const uint8_t* b) { return (uint32_t)b[0] << 8 | b[1]; }

int or_pcap_frame(const uint8_t* rec, uint32_t link_type, uint32_t flags, uint32_t* udp_off,
                  uint32_t* udp_len, or_addr* src, int* ttl, uint32_t* sec, uint32_t* usec)
{
    const int sw = (flags & 2) != 0;
    memset(src, 0, sizeof(*src));
    *ttl = -1;
    *udp_off = 0;
    *udp_len = 0;
    *sec = pc_u32(rec, sw);
    const uint32_t frac = pc_u32(rec + 4, sw);
    *usec = (flags & 1) ? frac / 1000u : frac;
    const uint32_t caplen = pc_u32(rec + 8, sw), wirelen = pc_u32(rec + 12, sw);
    const uint8_t* d = rec + 16;
    const uint32_t maxBytes = 4094;
    const uint32_t num = caplen < maxBytes ? caplen : maxBytes;    /* :346-347 */
    uint32_t eth_type, ip0, ip_len;
    if (link_type == 113) {                                         /* DLT_LINUX_SLL :354-364 */
        if (num < 16) return 1;
        eth_type = pc_be16(d + 14);
        ip0 = 16;
        ip_len = num - 16;
    } else {                                                        /* ProtoPktETH :368-380 */
        if (wirelen > maxBytes || wirelen < 14) return 1;
        if (num < 14) return 5;
        eth_type = pc_be16(d + 12);
        uint32_t hl = 14;
        if (eth_type == 0x8100) {
            if (wirelen < 18) return 1;
            if (num < 18) return 5;
            eth_type = pc_be16(d + 16);
            hl = 18;
        }
        ip0 = hl;
        ip_len = wirelen - hl;
    }
    if (eth_type != 0x0800 && eth_type != 0x86DD) return 2;        /* srcAddr invalid :422 */
    if (ip_len < 1) return 3;
    if (ip0 >= num) return 5;
    const uint32_t ver = d[ip0] >> 4;
    uint32_t l4, l4_len;
    if (ver == 4) {                                                 /* ProtoPktIPv4 :395-402 */
        if (ip_len < 20) return 3;
        if (ip0 + 20 > num) return 5;
        const uint32_t ihl = (d[ip0] & 15u) * 4u, tot = pc_be16(d + ip0 + 2);
        if (ihl < 20 || tot < ihl || tot > ip_len) return 3;
        *ttl = d[ip0 + 8];
        src->type = OR_ADDR_IPV4;
        src->len = 4;
        memcpy(src->addr, d + ip0 + 12, 4);
        if (d[ip0 + 9] != 17) return 4;
        l4 = ip0 + ihl;
        l4_len = tot - ihl;
    } else if (ver == 6) {                                          /* ProtoPktIPv6 :403-410 */
        if (ip_len < 40) return 3;
        if (ip0 + 40 > num) return 5;
        const uint32_t pl = pc_be16(d + ip0 + 4);
        if (40u + pl > ip_len) return 3;
        *ttl = d[ip0 + 7];
        src->type = OR_ADDR_IPV6;
        src->len = 16;
        memcpy(src->addr, d + ip0 + 8, 16);
        if (d[ip0 + 6] != 17) return 4;
        l4 = ip0 + 40;
        l4_len = pl;
    } else {
        return 3;
    }
    if (l4_len < 8) return 4;                                       /* ProtoPktUDP :424-425 */
    if (l4 + 8 > num) return 5;
    const uint32_t ul = pc_be16(d + l4 + 4);
    if (ul < 8 || ul > l4_len) return 4;
    src->port = (uint16_t)pc_be16(d + l4);
    *udp_off = 16 + l4 + 8;
    *udp_len = ul - 8;
    if (l4 + ul > num) {
        /* cut by the snapshot length: the reference parses the frame by hdr.len and Unpacks
         * udpPkt's payload from its parse buffer, so the MGEN header comes from the captured
         * bytes.  With the UDP header and MIN_SIZE payload bytes captured the payload is
         * unpacked zero-extended to the UDP length (7, SNAPPED; the reference's buffer holds
         * stale bytes there); shorter captures are skipped (5). */
        if (l4 + 8 + 28 <= num) return 7;
        *udp_off = 0;
        *udp_len = 0;
        return 5;
    }
    return 0;
}

typedef struct {
    or_addr  src, dst;
    uint32_t flow_id;
    int      used, sign;
    or_analytic a;
} pc_flow;

static int pc_addr_eq(const or_addr* x, const or_addr* y)
{
    return x->len == y->len && x->port == y->port && memcmp(x->addr, y->addr, x->len) == 0;
}

/* MgenAnalyticTable::FindFlow / Insert (mgenAnalytic.cpp:312-328): open addressing */
static pc_flow* pc_find(pc_flow** tab, uint32_t* cap, uint32_t* n, const or_addr* src,
                        const or_addr* dst, uint32_t flow_id, double window)
{
    if (2 * (*n + 1) > *cap) {
        uint32_t nc = *cap ? 2 * *cap : 64;
        pc_flow* nt = (pc_flow*)calloc(nc, sizeof(pc_flow));
        for (uint32_t i = 0; i < *cap; i++) {
            if (!(*tab)[i].used) continue;
            uint32_t h = ((*tab)[i].flow_id * 2654435761u ^ (*tab)[i].src.port ^
                          (uint32_t)(*tab)[i].dst.port << 16) & (nc - 1);
            while (nt[h].used) h = (h + 1) & (nc - 1);
            nt[h] = (*tab)[i];
        }
        free(*tab);
        *tab = nt;
        *cap = nc;
    }
    uint32_t h = (flow_id * 2654435761u ^ src->port ^ (uint32_t)dst->port << 16) & (*cap - 1);
    while ((*tab)[h].used) {
        pc_flow* f = &(*tab)[h];
        if (f->flow_id == flow_id && pc_addr_eq(&f->src, src) && pc_addr_eq(&f->dst, dst)) return f;
        h = (h + 1) & (*cap - 1);
    }
    pc_flow* f = &(*tab)[h];
    memset(f, 0, sizeof(*f));
    f->used = 1;
    f->src = *src;
    f->dst = *dst;
    f->flow_id = flow_id;
    or_analytic_init(&f->a, window);                 /* MgenAnalytic::Init :455 */
    (*n)++;
    return f;
}

static void pc_emit(char* out, uint64_t cap, uint64_t* pos, const char* s, uint32_t len)
{
    if (out && *pos + len <= cap) memcpy(out + *pos, s, len);
    *pos += len;
}

uint64_t or_pcap2mgen(const uint8_t* file, uint64_t nbytes, int analytics, int log_rx,
                      double window, uint32_t opts, char* out, uint64_t cap, uint64_t* n_pkts,
                      uint8_t* status)
{
    uint64_t pos = 0, npk = 0;
    if (n_pkts) *n_pkts = 0;
    if (nbytes < 24) return 0;
    uint32_t magic;
    memcpy(&magic, file, 4);
    int sw = 0, ns = 0;
    if (magic == 0xa1b2c3d4u) {}
    else if (magic == 0xd4c3b2a1u) sw = 1;
    else if (magic == 0xa1b23c4du) ns = 1;
    else if (magic == 0x4d3cb2a1u) sw = ns = 1;
    else return 0;
    const uint32_t flags = (ns ? 1u : 0u) | (sw ? 2u : 0u);
    const uint32_t link = pc_u32(file + 20, sw) & 0x0FFFFFFFu;
    pc_flow* tab = NULL;
    uint32_t tcap = 0, tn = 0;
    char* line = (char*)malloc(1 << 16);
    uint8_t* snap = (uint8_t*)malloc(65536);
    uint64_t off = 24;
    while (off + 16 <= nbytes) {                                    /* pcap_next :344 */
        const uint32_t caplen = pc_u32(file + off + 8, sw);
        if (off + 16 + (uint64_t)caplen > nbytes) break;
        const uint8_t* rec = file + off;
        off += 16 + (uint64_t)caplen;
        uint32_t uo, ul, sec, usec;
        or_addr src;
        int ttl;
        const int st = or_pcap_frame(rec, link, flags, &uo, &ul, &src, &ttl, &sec, &usec);
        if (status) status[npk] = (uint8_t)st;
        npk++;
        if (st != 0 && st != 7) continue;
        const uint8_t* pay = rec + uo;
        if (st == 7) {                     /* SNAPPED: the captured bytes, zero-extended */
            memset(snap, 0, 65536);
            memcpy(snap, pay, 16 + pc_u32(rec + 8, sw) - uo);
            pay = snap;
        }
        or_fields f;
        or_unpack(pay, ul, &f);                                     /* :428-432 */
        if (!f.ok) continue;
        if (analytics) {                                            /* :445-473 */
            or_addr dst;
            memset(&dst, 0, sizeof dst);
            dst.type = f.dst_type;
            dst.len = f.dst_len;
            dst.port = f.dst_port;
            memcpy(dst.addr, f.dst_addr, 16);
            if (dst.len > 16) dst.len = 16;
            pc_flow* fl = pc_find(&tab, &tcap, &tn, &src, &dst, f.flow_id, window);
            const or_time rx = {(int64_t)sec, (int64_t)usec};
            const or_time tx = {(int64_t)f.tx_sec, (int64_t)f.tx_usec};
            if (or_analytic_update(&fl->a, rx, f.msg_len, tx, f.seq_num)) {
                uint8_t rb[52];
                or_report_build(&fl->src, &fl->dst, fl->flow_id, 1, fl->a.report_duration,
                                fl->a.report_latency_ave, fl->a.report_latency_min,
                                fl->a.report_latency_max, fl->a.report_rate_ave,
                                fl->a.report_loss_ave, -1.0, &fl->sign, rb);
                const uint32_t n = or_log_report(rb, fl->a.report_duration, fl->a.report_rate_ave,
                                                 fl->a.report_loss_ave, fl->a.report_latency_ave,
                                                 fl->a.report_latency_min, fl->a.report_latency_max,
                                                 fl->a.report_msg_count, sec, usec, opts, line);
                pc_emit(out, cap, &pos, line, n);
            }
        }
        /* msg.LogRecvEvent(outfile, false, false, log_rx, false, true, payload, flush, ttl, ts) */
        if (log_rx) {
            const uint32_t n = or_log_recv_text(&f, pay, &src, sec, usec, 1, ttl,
                                                opts | OR_LOG_NO_DATA, line);
            pc_emit(out, cap, &pos, line, n);
        }
        if (f.payload_type == 1 && f.payload_len > 0) {             /* mgenMsg.cpp:1104-1137 */
            uint32_t cmds[64], reps[256], nc = 0, nr = 0;
            (void)or_data_walk(pay + f.payload_off, f.payload_len, 1, cmds, &nc, 64, reps, &nr,
                               256);
            for (uint32_t k = 0; k < nr && k < 256; k++) {
                const uint32_t n = or_log_report_recv(pay + f.payload_off + reps[k], &src, sec,
                                                      usec, opts, line);
                pc_emit(out, cap, &pos, line, n);
            }
        }
    }
    free(line);
    free(snap);
    free(tab);
    if (n_pkts) *n_pkts = npk;
    return pos;
}

/* ==== ConvertBinaryLog (mgenMsg.cpp:1417-1900) ========================================
 * The binary log -> text log conversion over a file image.  The header line ("mgen
 * version=<4|5>... type=binary_log\n\0") is checked, then records {type, protocol, BE
 * recordLength <= 1024, recordLength bytes} are converted until the end of the file or the
 * first record the reference rejects (RERR and unknown event types, an unknown address type,
 * a short record): *status then says why (OR_BL_*), and the text so far is kept, as the
 * reference has already written it.  RECV: Unpack of the stored message (recordLength - 12 -
 * srcLen bytes) and LogRecvEvent with the reference's argument order at :1607, which puts
 * log_flush in the ttl slot ("ttl>0 " / "ttl>1 "); SEND: Unpack and LogSendEvent (srcPort 0:
 * a fresh MgenMsg's source); LISTEN / IGNORE / JOIN / LEAVE / START / STOP / ON / ACCEPT /
 * CONNECT / DISCONNECT / OFF / SHUTDOWN / RECONNECT lines as :1628-1891.  A RECV or SEND
 * record whose stored message Unpack rejects (never written by mgen) is logged all the same,
 * from the members the fresh MgenMsg keeps, as the reference ignores Unpack's result. */
enum { OR_BL_OK = 0, OR_BL_HEADER = 1, OR_BL_TOO_LONG = 2, OR_BL_EVENT = 3, OR_BL_SHORT = 4 };

/* A record too short for the fields its type reads (mgen never writes one): the reference
 * parses its fixed-size read buffer regardless (stale bytes past the record); here the walk
 * stops at it as at a short read.  Every record holds its event time (8 bytes); RECV 12 +
 * source length; LISTEN / IGNORE 12; JOIN / LEAVE 13 + group length + interface name
 * length; ON ... RECONNECT 18 + address length. */
static int bl_too_short(int ev, const uint8_t* b, uint32_t rl)
{
    if (rl < 8) return 1;
    switch (ev) {
        case 1: return rl < 12 || rl < 12u + b[11];
        case 4: case 5: return rl < 12;
        case 6: case 7: return rl < 13 || rl < 13u + b[11] || rl < 13u + b[11] + b[12 + b[11]];
        default: return ev >= 10 && ev <= 16 && (rl < 12 || rl < 18u + b[11]);
    }
}

static void bl_addr(or_addr* a, uint8_t type, const uint8_t* p, uint32_t len, uint16_t port)
{
    memset(a, 0, sizeof(*a));
    a->type = type;
    a->len = (uint8_t)(len > 16 ? 16 : len);
    memcpy(a->addr, p, a->len);
    a->port = port;
}

static uint32_t bl_send_line(const or_fields* f, int protocol, uint32_t mgen_msg_len,
                             uint32_t opts, char* out)
{
    char* p = out;
    p += log_ts(p, f->tx_sec, f->tx_usec, (opts & OR_LOG_EPOCH) != 0);
    p += sprintf(p, "SEND proto>%s flow>%lu seq>%lu srcPort>%hu dst>", log_proto(protocol),
                 (unsigned long)f->flow_id, (unsigned long)f->seq_num, (unsigned short)0);
    p += log_addr(p, f->dst_type, f->dst_len, f->dst_addr);
    p += sprintf(p, "/%hu", f->dst_port);
    if (protocol == 2) p += sprintf(p, " size>%lu ", (unsigned long)mgen_msg_len);
    else p += sprintf(p, " size>%u ", (unsigned)f->msg_len);
    if (f->host_type == OR_ADDR_IPV4 || f->host_type == OR_ADDR_IPV6) {
        p += sprintf(p, "host>");
        p += log_addr(p, f->host_type, f->host_len, f->host_addr);
        p += sprintf(p, "/%hu\n", f->host_port);
    } else {
        p += sprintf(p, "\n");
    }
    return (uint32_t)(p - out);
}

uint64_t or_convert_binary_log(const uint8_t* file, uint64_t nbytes, int log_rx, int flush,
                               uint32_t opts, char* out, uint64_t cap, int* status,
                               uint64_t* n_records)
{
    uint64_t pos = 0, nrec = 0;
    *status = OR_BL_HEADER;
    if (n_records) *n_records = 0;
    if (nbytes < 4 || memcmp(file, "mgen", 4) != 0) return 0;
    char hdr[1024];
    uint64_t k = 3;
    memcpy(hdr, file, 4);
    while (hdr[k] != '\0') {                        /* the header line and its NUL */
        if (++k >= sizeof hdr || k >= nbytes) return 0;
        hdr[k] = (char)file[k];
    }
    const char* v = strstr(hdr, "version=");
    int version;
    if (!v || 1 != sscanf(v, "version=%d", &version) || (version != 4 && version != 5)) return 0;
    const char* t = strstr(v, "type=");
    char ftype[128];
    if (!t || 1 != sscanf(t, "type=%127s", ftype) || strcmp(ftype, "binary_log")) return 0;
    const int ep = (opts & OR_LOG_EPOCH) != 0;
    char* line = (char*)malloc(1 << 16);
    uint64_t off = k + 1;
    *status = OR_BL_OK;
    while (1) {
        if (off + 4 > nbytes) break;                 /* feof: done */
        const uint8_t* h = file + off;
        const int ev = h[0], proto = h[1];
        const uint32_t rl = (uint32_t)h[2] << 8 | h[3];
        if (rl > 1024) { *status = OR_BL_TOO_LONG; break; }
        if (off + 4 + rl > nbytes) { *status = OR_BL_SHORT; break; }
        const uint8_t* b = h + 4;
        if (ev != 0 && ev != 2 && ev <= 16 && bl_too_short(ev, b, rl)) { *status = OR_BL_SHORT; break; }
        off += 4 + rl;
        uint32_t n = 0;
        const uint32_t sec = get32(b), usec = get32(b + 4);
        if (ev == 1) {                                               /* RECV :1560-1609 */
            const uint8_t at = b[10];
            if (at != 1 && at != 2) { *status = OR_BL_EVENT; break; }
            const uint32_t alen = b[11];
            or_addr src;
            bl_addr(&src, at, b + 12, alen, (uint16_t)(b[8] << 8 | b[9]));
            const uint32_t idx = 12 + alen;
            or_fields f;
            or_unpack(b + idx, rl >= idx ? rl - idx : 0, &f);
            nrec++;
            if (!f.ok) {
                /* Unpack's result is ignored (:1606-1607): the line shows the fresh MgenMsg's
                 * members, tx_time = the event time set before Unpack unless Unpack got to
                 * the base fields (every error but LENGTH / VERSION) */
                if (f.err == 3 || f.err == 1) { f.tx_sec = sec; f.tx_usec = usec; }
                f.err = 0;
                f.ok = 1;
            }
            if (log_rx) {
                n = or_log_recv_text(&f, b + idx, &src, sec, usec, proto, flush ? 1 : 0, opts,
                                     line);
                pc_emit(out, cap, &pos, line, n);
            }
            if (f.payload_type == 1 && f.payload_len > 0) {
                uint32_t cmds[64], reps[256], nc = 0, nr = 0;
                (void)or_data_walk(b + idx + f.payload_off, f.payload_len, 1, cmds, &nc, 64, reps,
                                   &nr, 256);
                for (uint32_t j = 0; j < nr && j < 256; j++) {
                    n = or_log_report_recv(b + idx + f.payload_off + reps[j], &src, sec, usec, opts,
                                           line);
                    pc_emit(out, cap, &pos, line, n);
                }
            }
            continue;
        }
        if (ev == 3) {                                               /* SEND :1610-1627 */
            uint32_t idx = 0, mml = 0;
            if (proto == 2) { mml = get32(b); idx = 4; }
            or_fields f;
            /* the reference passes recordLength (:1624), i.e. 4 bytes more than the record
             * holds after a TCP SEND's mgen_msg_len word: those come from its uninitialised
             * or stale stack buffer (:1434).  Bounded here at the stored bytes: an Unpack
             * that would reach them (a message cut before its host / GPS fields) stops at
             * the record end instead (tests/test_gpu_binlog.py pins it). */
            or_unpack(b + idx, rl - idx, &f);
            nrec++;
            if (!f.ok) { f.err = 0; f.ok = 1; }  /* logged anyway, fresh members (:1624-1625) */
            n = bl_send_line(&f, proto, mml, opts, line);
            pc_emit(out, cap, &pos, line, n);
            continue;
        }
        char* p = line;
        if (ev == 4 || ev == 5) {                                    /* LISTEN / IGNORE */
            p += log_ts(p, sec, usec, ep);
            p += sprintf(p, "%s proto>%s port>%hu\n", ev == 4 ? "LISTEN" : "IGNORE",
                         log_proto(b[8]), (unsigned short)(b[10] << 8 | b[11]));
        } else if (ev == 6 || ev == 7) {                             /* JOIN / LEAVE */
            const uint8_t at = b[10];
            if (at != 1 && at != 2) { *status = OR_BL_EVENT; break; }
            const uint32_t alen = b[11];
            const uint16_t gport = (uint16_t)(b[8] << 8 | b[9]);
            uint32_t nl = b[12 + alen];
            char iface[256];
            memcpy(iface, b + 13 + alen, nl);
            iface[nl] = '\0';
            p += log_ts(p, sec, usec, ep);
            p += sprintf(p, "%s group>", ev == 6 ? "JOIN" : "LEAVE");
            p += log_addr(p, at, (uint8_t)alen, b + 12);
            if (nl) p += sprintf(p, " interface>%s", iface);
            if (gport) p += sprintf(p, " port>%hu\n", gport);
            else p += sprintf(p, "\n");
        } else if (ev == 8 || ev == 9) {                             /* START / STOP */
            p += log_ts(p, sec, usec, ep);
            p += sprintf(p, "%s\n", ev == 8 ? "START" : "STOP");
        } else if (ev >= 10 && ev <= 16) {                           /* :1730-1891 */
            const uint8_t at = b[10];
            if (at != 1 && at != 2) { *status = OR_BL_EVENT; break; }
            const uint32_t alen = b[11];
            uint32_t i = 12 + alen;
            char a[64];
            log_addr(a, at, (uint8_t)alen, b + 12);
            const uint16_t aport = (uint16_t)(b[8] << 8 | b[9]);
            const uint16_t dport = (uint16_t)(b[i] << 8 | b[i + 1]);
            i += 2;
            const unsigned long fid = get32(b + i);
            i += 4;
            int hvalid = 0;
            uint16_t hport = 0;
            uint8_t ht = 0;
            uint32_t hl = 0;
            char hs[64];
            if (i + 4 <= rl) {
                hport = (uint16_t)(b[i] << 8 | b[i + 1]);
                i += 2;
                ht = b[i++];
                if (ht != 1 && ht != 2) ht = 0;
                hl = b[i++];
                if (i + hl <= rl && ht && hl) {
                    log_addr(hs, ht, (uint8_t)hl, b + i);
                    hvalid = 1;
                }
            }
            p += log_ts(p, sec, usec, ep);
            switch (ev) {
                case 10: p += sprintf(p, "ON flow>%lu srcPort>%hu dst>%s/%hu", fid, dport, a, aport); break;
                case 11: p += sprintf(p, "ACCEPT src>%s/%hu dstPort>%hu", a, aport, dport); break;
                case 13: p += sprintf(p, "CONNECT flow>%lu srcPort>%hu dst>%s/%hu", fid, dport, a, aport); break;
                case 12:
                    if (fid) p += sprintf(p, "DISCONNECT flow>%lu dst>%s/%hu srcPort>%hu", fid, a, aport, dport);
                    else p += sprintf(p, "DISCONNECT src>%s/%hu dstPort>%hu", a, aport, dport);
                    break;
                case 16:
                    if (fid) p += sprintf(p, "RECONNECT flow>%lu dst>%s/%hu srcPort>%hu", fid, a, aport, dport);
                    else p += sprintf(p, "RECONNECT src>%s/%hu dstPort>%hu", a, aport, dport);
                    break;
                case 15:
                    if (fid) p += sprintf(p, "SHUTDOWN flow>%lu dst>%s/%hu srcPort>%hu", fid, a, aport, dport);
                    else p += sprintf(p, "SHUTDOWN src>%s/%hu dstPort>%hu", a, aport, dport);
                    break;
                case 14:
                    if (fid) p += sprintf(p, "OFF flow>%lu srcPort>%hu dst>%s/%hu", fid, dport, a, aport);
                    else p += sprintf(p, "OFF src>%s/%hu dstPort>%hu", a, aport, dport);
                    break;
            }
            if (hvalid) p += sprintf(p, "host>%s/%hu", hs, hport);
            p += sprintf(p, "\n");
        } else {                                    /* RERR (2) and unknown types :1892-1895 */
            *status = OR_BL_EVENT;
            break;
        }
        nrec++;
        pc_emit(out, cap, &pos, line, (uint32_t)(p - line));
    }
    free(line);
    if (n_records) *n_records = nrec;
    return pos;
}
