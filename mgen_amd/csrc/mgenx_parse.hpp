// mgenx_parse.hpp -- MgenMsg::Unpack of one record by one lane (mgenMsg.cpp:315-500): the
// general-layout path of the batch kernels (mgenx_unpack.hip) and the resident single-message
// worker (mgenx_worker.hip).
#pragma once

#include "mgenx_common.hpp"

namespace mgenx {

// Bytes [p, p + min(n,16)) as 4 little-endian words; bytes at or past `avail` read as 0.
__device__ __forceinline__ void load_addr16(const uint8_t* p, uint32_t n, uint32_t avail,
                                            uint32_t out[4]) {
  const uint32_t lim = min(min(n, 16u), avail);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t b0 = 4u * j;
    uint32_t w = 0;
    if (b0 + 4 <= lim) {
      w = ldu32(p + b0);
    } else if (b0 < lim) {
      for (uint32_t b = b0; b < lim; b++) w |= (uint32_t)p[b] << (8 * (b - b0));
    }
    out[j] = w;
  }
}

struct Hdr {
  uint32_t flow, seq, sec, usec, dst4, lat, lon, poff;
  int32_t alt;
  uint32_t dst_addr[4], host_addr[4];
  uint16_t msg_len, dst_port, plen, hdr_len, host_port;
  uint8_t version, flags, err, dst_type, dst_len, ptype, gps, host_type, host_len;
  uint8_t dec;  // MGENX_DEC_* of the fields Unpack assigned
  bool ok;
};

// The first 32 bytes of a record (or 28..31 when shorter), loaded up front so the CRC
// decision costs one load latency.  w[7] (bytes 28..31) is valid only if buf_len >= 32.
__device__ __forceinline__ void load_fixed(const uint8_t* r, uint32_t buf_len, uint32_t w[8]) {
  if (buf_len >= 32) {
    const u32x4_t a = ldu128(r), b = ldu128(r + 16);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  } else if (buf_len >= MGENX_MIN_SIZE) {
    const u32x4_t a = ldu128(r);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = ldu32(r + 16); w[5] = ldu32(r + 20); w[6] = ldu32(r + 24); w[7] = 0;
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = 0;
  }
}

// Unpack()'s return value from the fixed prefix alone (mgenMsg.cpp:323-392).
__device__ __forceinline__ bool fixed_ok(uint32_t buf_len, const uint32_t w[8]) {
  const uint32_t t = (w[5] >> 16) & 0xffu;
  return buf_len >= MGENX_MIN_SIZE && ((w[0] >> 16) & 0xffu) == 2u && (t == 1u || t == 2u);
}

// MgenMsg::Unpack on a fresh MgenMsg (mgenMsg.cpp:315-500); buf_len = bufferLen,
// w = load_fixed(r, buf_len).
__device__ inline void parse_header(const uint8_t* r, uint32_t buf_len, bool want_ext,
                             const uint32_t w[8], Hdr& h) {
  h.flow = h.seq = h.sec = h.usec = h.dst4 = h.poff = 0;
  h.lat = h.lon = 10800000u;  // (0.0 + 180) * 60000: the constructor's 0.0 degrees
  h.alt = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) h.dst_addr[j] = h.host_addr[j] = 0;
  h.msg_len = h.dst_port = h.plen = h.hdr_len = h.host_port = 0;
  h.version = 2;
  h.flags = h.err = h.dst_type = h.dst_len = h.ptype = h.gps = h.host_type = h.host_len = 0;
  h.dec = 0;
  h.ok = false;
  if (buf_len < MGENX_MIN_SIZE) { h.err = MGENX_ERROR_LENGTH; return; }      // :323-328
  h.msg_len = bswap16((uint16_t)(w[0] & 0xffffu));
  h.version = (uint8_t)(w[0] >> 16);
  h.dec = MGENX_DEC_MSGLEN;
  if (h.version != 2) { h.err = MGENX_ERROR_VERSION; return; }              // :336-343
  h.dec |= MGENX_DEC_BASE;
  h.flags = (uint8_t)(w[0] >> 24);
  h.flow = bswap32(w[1]);
  h.seq = bswap32(w[2]);
  h.sec = bswap32(w[3]);
  h.usec = bswap32(w[4]);
  const uint16_t dport = bswap16((uint16_t)(w[5] & 0xffffu));
  const uint32_t t = (w[5] >> 16) & 0xffu;
  const uint32_t D = w[5] >> 24;
  if (t != 1u && t != 2u) { h.err = MGENX_ERROR_DSTADDR; return; }          // :374-392
  h.dec |= MGENX_DEC_DST | MGENX_DEC_HDRLEN;  // every later return sets packet_header_len
  h.dst_type = (uint8_t)t;
  h.dst_len = (uint8_t)D;
  h.dst_port = dport;
  // :394-398 has no bounds check; bytes past the record read as zero here.
  if (want_ext) {
    load_addr16(r + 24, D, buf_len - 24, h.dst_addr);
    h.dst4 = h.dst_addr[0];
  } else {
    h.dst4 = D >= 4 ? w[6] : (w[6] & byte_range_mask(0, (int)D));
  }
  uint32_t len = 24u + D;
  if (len + 4u <= buf_len) {                                                  // :400-443
    const uint32_t hw = (len == 28u) ? w[7] : ldu32(r + len);
    const uint16_t hport = bswap16((uint16_t)(hw & 0xffffu));
    const uint32_t ht = (hw >> 16) & 0xffu;
    const uint32_t H = hw >> 24;
    len += 4u;
    if (len + H <= buf_len) {
      if (ht == 1u || ht == 2u) {
        h.dec |= MGENX_DEC_HOST;
        h.host_type = (uint8_t)ht;
        h.host_len = (uint8_t)H;
        h.host_port = hport;
        if (want_ext) load_addr16(r + len, H, H, h.host_addr);
      }
      len += H;
    } else {
      h.hdr_len = (uint16_t)len; h.ok = true; return;
    }
  } else {
    h.hdr_len = (uint16_t)len; h.ok = true; return;
  }
  if (len + 16u <= buf_len) {                                                 // :446-497
    // GPS, payload_type and payload_len in one 16-byte load (the common case)
    const u32x4_t g = ldu128(r + len);
    h.lat = bswap32(g.x);
    h.lon = bswap32(g.y);
    h.alt = (int32_t)bswap32(g.z);
    h.gps = (uint8_t)g.w;
    h.ptype = (uint8_t)(g.w >> 8);
    h.plen = bswap16((uint16_t)(g.w >> 16));
    h.dec |= MGENX_DEC_GPS | MGENX_DEC_PTYPE | MGENX_DEC_PLEN;
    len += 16u;
    h.hdr_len = (uint16_t)len;
    if (h.plen != 0 && len + h.plen <= buf_len) h.poff = (len >> 2) << 2;
    else h.plen = 0;
    h.ok = true;
    return;
  }
  if (len + 13u <= buf_len) {                                                 // :446-465
    h.lat = bswap32(ldu32(r + len));
    h.lon = bswap32(ldu32(r + len + 4));
    h.alt = (int32_t)bswap32(ldu32(r + len + 8));
    h.gps = r[len + 12];
    h.dec |= MGENX_DEC_GPS;
    len += 13u;
  } else {
    h.hdr_len = (uint16_t)len; h.ok = true; return;
  }
  if (len + 1u <= buf_len) {                                                  // :467-475
    h.ptype = r[len];
    h.dec |= MGENX_DEC_PTYPE;
    len += 1u;
  } else {
    h.hdr_len = (uint16_t)len; h.ok = true; return;
  }
  if (len + 2u <= buf_len) {                                                  // :477-497
    h.plen = bswap16(ldu16(r + len));
    h.dec |= MGENX_DEC_PLEN;
    len += 2u;
    h.hdr_len = (uint16_t)len;
    if (h.plen != 0 && len + h.plen <= buf_len) h.poff = (len >> 2) << 2;
    else h.plen = 0;
  }
  h.ok = true;
}


}  // namespace mgenx
