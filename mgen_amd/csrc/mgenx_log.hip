// mgenx_log.hip -- RECV / RERR event log lines from decoded records, on gfx950.
//
// Reference: MgenMsg::LogRecvEvent, text branch (src/common/mgenMsg.cpp:1034-1102), and
// MgenMsg::LogRecvError, text branch (:711-735), as MgenUdpTransport::OnEvent calls them
// (src/common/mgenTransport.cpp:976-994); timestamps Mgen::LogLegacyTimestamp (GMT,
// "%02d:%02d:%02d.%06lu ") or Mgen::LogEpochTimestamp ("%lu.%06lu ") (src/common/mgen.cpp:
// 55-83).  Byte-exact with glibc's printf of the same arguments on x86-64, including the
// two ABI details the doc's own output pins (doc/mgen.xml:2948): "%ld" of the INT32
// altitude prints it zero-extended, and "%f" is the exactly rounded 6-decimal value.
//
// Two passes over the records, one lane per record: (1) each line's length, (2) after an
// exclusive scan of the lengths (hipCUB), each lane writes its line at its offset.  Both
// passes run the same formatter, once with a counting sink and once with a writing sink.
// Plumbing next to the unpack: the text is ~5-15x smaller than the records it describes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr int kLogThreads = 256;

// the fields LogRecvEvent prints, gathered from rows or core columns + extended columns
struct LogRec {
  uint32_t flow, seq, sec, usec, lat, lon, alt, poff;
  uint16_t msg_len, dport, plen, hport, hdr;
  uint8_t flags, err, dtype, dlen, ptype, gps, htype, hlen;
  uint8_t daddr[16], haddr[16];
};

struct CountSink {
  uint32_t n = 0;
  __device__ void put(uint8_t) { n++; }
};

struct WriteSink {
  uint8_t* p;
  uint32_t n = 0;
  __device__ void put(uint8_t c) { p[n++] = c; }
};

template <typename S>
__device__ __forceinline__ void put_str(S& s, const char* t) {
  while (*t) s.put((uint8_t)*t++);
}

template <typename S>
__device__ void put_u64(S& s, uint64_t v, int width = 0) {  // "%0<width>lu"
  char d[20];
  int k = 0;
  do {
    d[k++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  for (int i = k; i < width; i++) s.put('0');
  while (k) s.put((uint8_t)d[--k]);
}

template <typename S>
__device__ void put_i32(S& s, int32_t v) {  // "%d"
  if (v < 0) {
    s.put('-');
    put_u64(s, (uint64_t)(-(int64_t)v));
  } else {
    put_u64(s, (uint64_t)v);
  }
}

template <typename S>
__device__ void put_hex16(S& s, uint32_t v) {  // "%x" of a 16-bit group
  const char* hx = "0123456789abcdef";
  bool lead = true;
  for (int sh = 12; sh >= 0; sh -= 4) {
    const uint32_t d = (v >> sh) & 15u;
    if (lead && d == 0 && sh) continue;
    lead = false;
    s.put((uint8_t)hx[d]);
  }
}

// Mgen::LogLegacyTimestamp (gmtime) / Mgen::LogEpochTimestamp, trailing space included
template <typename S>
__device__ void put_ts(S& s, uint32_t sec, uint32_t usec, bool epoch) {
  if (epoch) {
    put_u64(s, sec);
    s.put('.');
  } else {
    const uint32_t sod = sec % 86400u;
    put_u64(s, sod / 3600u, 2);
    s.put(':');
    put_u64(s, (sod % 3600u) / 60u, 2);
    s.put(':');
    put_u64(s, sod % 60u, 2);
    s.put('.');
  }
  put_u64(s, usec, 6);
  s.put(' ');
}

template <typename S>
__device__ void put_ipv4(S& s, const uint8_t* a) {
  for (int i = 0; i < 4; i++) {
    if (i) s.put('.');
    put_u64(s, a[i]);
  }
}

// inet_ntop(AF_INET6) as glibc formats it (resolv/inet_ntop.c): the longest run (>= 2) of
// zero groups, first on ties, becomes "::"; an IPv4-compatible (::a.b.c.d) or IPv4-mapped
// (::ffff:a.b.c.d) address ends in dotted decimal.
template <typename S>
__device__ void put_ipv6(S& s, const uint8_t* a) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = ((uint32_t)a[2 * i] << 8) | a[2 * i + 1];
  int best = -1, best_len = 0, cur = -1, cur_len = 0;
  for (int i = 0; i < 8; i++) {
    if (w[i] == 0) {
      if (cur < 0) { cur = i; cur_len = 1; } else { cur_len++; }
    } else if (cur >= 0) {
      if (best < 0 || cur_len > best_len) { best = cur; best_len = cur_len; }
      cur = -1;
    }
  }
  if (cur >= 0 && (best < 0 || cur_len > best_len)) { best = cur; best_len = cur_len; }
  if (best >= 0 && best_len < 2) best = -1;
  for (int i = 0; i < 8; i++) {
    if (best >= 0 && i >= best && i < best + best_len) {
      if (i == best) s.put(':');
      continue;
    }
    if (i) s.put(':');
    if (i == 6 && best == 0 && (best_len == 6 || (best_len == 5 && w[5] == 0xffffu))) {
      put_ipv4(s, a + 12);
      return;
    }
    put_hex16(s, w[i]);
  }
  if (best >= 0 && best + best_len == 8) s.put(':');
}

// ProtoAddress::GetHostString of the address Unpack built (protolib; see the oracle)
template <typename S>
__device__ void put_addr(S& s, uint8_t type, uint8_t len, const uint8_t* a) {
  if (type == 2 && len == 16) put_ipv6(s, a);
  else if (type == 1 && len == 4) put_ipv4(s, a);
  else put_str(s, "(invalid)");
}

// "%f" of raw / 60000.0 - 180.0 (mgenMsg.cpp:453,457): the double is computed with the same
// IEEE operations, then its exact binary value is rounded to 6 decimals, ties to even (as
// glibc's printf_fp does in round-to-nearest mode).
template <typename S>
__device__ void put_deg(S& s, uint32_t raw) {
  const double v = __dsub_rn(__ddiv_rn((double)raw, 60000.0), 180.0);
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const bool neg = (bits >> 63) != 0;
  const uint32_t ex = (uint32_t)((bits >> 52) & 0x7ffu);
  const uint64_t mant = (bits & ((1ull << 52) - 1)) | (ex ? (1ull << 52) : 0ull);
  const int e = (ex ? (int)ex : 1) - 1075;  // |v| = mant * 2^e
  uint64_t q;                              // round(|v| * 1e6)
  const unsigned __int128 P = (unsigned __int128)mant * 1000000u;
  if (e >= 0) {
    q = (uint64_t)(P << e);  // |v| < 2^23 here: no overflow
  } else if (-e >= 80) {
    q = 0;  // |v| * 1e6 < 2^-6: rounds to zero
  } else {
    const int sh = -e;
    q = (uint64_t)(P >> sh);
    const unsigned __int128 rem = P - ((unsigned __int128)q << sh);
    const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
    if (rem > half || (rem == half && (q & 1))) q++;
  }
  if (neg) s.put('-');
  put_u64(s, q / 1000000u);
  s.put('.');
  put_u64(s, q % 1000000u, 6);
}

// A record past the end of the slab (MGENX_ERROR_OOB) is not an MgenMsg::Error: it is
// logged as ERROR_LENGTH, as include/mgenx.hpp maps it
__device__ __forceinline__ uint32_t log_error(uint32_t e) {
  return e == MGENX_ERROR_OOB ? (uint32_t)MGENX_ERROR_LENGTH : e;
}

template <typename S>
__device__ void format_line(S& s, const LogRec& r, const uint8_t* rec, const mgenx_addr& src,
                            uint32_t rx_sec, uint32_t rx_usec, int protocol, int ttl,
                            uint32_t opts) {
  const bool epoch = (opts & MGENX_LOG_EPOCH) != 0;
  if (r.err) {  // LogRecvError (mgenMsg.cpp:713-734)
    put_ts(s, rx_sec, rx_usec, epoch);
    put_str(s, "RERR type>");
    switch (log_error(r.err)) {
      case 0: put_str(s, "none"); break;
      case 1: put_str(s, "version"); break;
      case 2: put_str(s, "checksum"); break;
      case 3: put_str(s, "length"); break;
      case 4: put_str(s, "dstAddr"); break;
      default: break;
    }
    put_str(s, " src>");
    put_addr(s, src.type, src.len, src.addr);
    s.put('/');
    put_u64(s, src.port);
    s.put('\n');
    return;
  }
  put_ts(s, rx_sec, rx_usec, epoch);  // mgenMsg.cpp:1038-1045
  put_str(s, "RECV proto>");
  put_str(s, protocol == 1 ? "UDP" : protocol == 2 ? "TCP" : protocol == 3 ? "SINK" : "UNKNOWN");
  put_str(s, " flow>");
  put_u64(s, r.flow);
  put_str(s, " seq>");
  put_u64(s, r.seq);
  put_str(s, " src>");
  put_addr(s, src.type, src.len, src.addr);
  s.put('/');
  put_u64(s, src.port);
  put_str(s, " dst>");
  put_addr(s, r.dtype, r.dlen, r.daddr);
  s.put('/');
  put_u64(s, r.dport);
  put_str(s, " sent>");
  put_ts(s, r.sec, r.usec, epoch);
  put_str(s, "size>");
  put_u64(s, r.msg_len);
  s.put(' ');
  if (r.htype == 1 || r.htype == 2) {  // :1047-1050
    put_str(s, "host>");
    put_addr(s, r.htype, r.hlen, r.haddr);
    s.put('/');
    put_u64(s, r.hport);
    s.put(' ');
  }
  if (ttl >= 0) {  // :1052-1053
    put_str(s, "ttl>");
    put_i32(s, ttl);
    s.put(' ');
  }
  const char* status;  // :1056-1072
  switch (r.gps) {
    case 0: status = "INVALID"; break;
    case 1: status = "STALE"; break;
    case 2: status = "CURRENT"; break;
    default:
      s.put('\n');
      return;
  }
  if (!(opts & MGENX_LOG_NO_GPS)) {  // :1073-1075
    put_str(s, "gps>");
    put_str(s, status);
    s.put(',');
    put_deg(s, r.lat);
    s.put(',');
    put_deg(s, r.lon);
    s.put(',');
    put_u64(s, r.alt);  // INT32 through "%ld": zero-extended (doc/mgen.xml:2948)
    s.put(' ');
  }
  if (r.plen && !(opts & MGENX_LOG_NO_DATA) && r.ptype == 0) {  // :1077-1086 (USER_DATA)
    const char* hx = "0123456789ABCDEF";                        // MgenPayload::toHex
    put_str(s, "data>");
    put_u64(s, r.plen);
    s.put(':');
    const uint8_t* d = rec + r.poff;  // payload_data: the word-floored header end
    for (uint32_t i = 0; i < r.plen; i++) {
      s.put((uint8_t)hx[d[i] >> 4]);
      s.put((uint8_t)hx[d[i] & 15]);
    }
    s.put(' ');
  }
  if (r.flags & MGENX_FLAG_CONTINUES) put_str(s, "flags>0x01 ");  // :1088-1100
  if (r.flags & MGENX_FLAG_END_OF_MSG) put_str(s, "flags>0x02 ");
  if (r.flags & MGENX_FLAG_CHECKSUM_ERROR) put_str(s, "flags>0x10 ");
  s.put('\n');
}

// Binary RECV / RERR records (MgenMsg::LogRecvEvent binary branch, mgenMsg.cpp:958-1033;
// LogRecvError binary branch, :652-710): BE header fields, the source address, then for RECV
// recordLength - index + 4 = hdr + payload_len + 2 message bytes with CHECKSUM cleared in
// the flags byte.  Bytes past the slab (the reference's stale receive buffer) are written 0.
template <typename S>
__device__ void put_be(S& s, uint32_t v, int bytes) {
  for (int k = bytes - 1; k >= 0; k--) s.put((uint8_t)(v >> (8 * k)));
}

template <typename S>
__device__ void format_binary(S& s, const LogRec& r, const uint8_t* rec, uint64_t avail,
                              const mgenx_addr& src, uint32_t rx_sec, uint32_t rx_usec,
                              int protocol) {
  const bool av = src.type == 1 || src.type == 2;
  const uint32_t alen = av ? src.len : 0u;
  if (r.err) {
    s.put(2);  // RERR_EVENT
    s.put(0);
    put_be(s, 12u + alen + 4u, 2);
    put_be(s, rx_sec, 4);
    put_be(s, rx_usec, 4);
    put_be(s, src.port, 2);
    s.put(av ? src.type : 0);
    s.put((uint8_t)alen);
    for (uint32_t k = 0; k < alen && k < 16; k++) s.put(src.addr[k]);
    put_be(s, log_error(r.err), 4);  // htonl(msg_error)
    return;
  }
  const uint32_t rl = (12u + alen + r.hdr + r.plen) & 0xFFFFu;
  s.put(1);  // RECV_EVENT
  s.put((uint8_t)protocol);
  put_be(s, rl, 2);
  put_be(s, rx_sec, 4);
  put_be(s, rx_usec, 4);
  put_be(s, src.port, 2);
  s.put(av ? src.type : 0);
  s.put((uint8_t)alen);
  for (uint32_t k = 0; k < alen && k < 16; k++) s.put(src.addr[k]);
  const uint32_t ml = (rl - (14u + alen) + 4u) & 0xFFFFu;
  // hdr + payload_len + 2 bytes: past the message's own msg_len (no checksum, no padding)
  // the reference writes stale bytes of its receive buffer; here they are zero, so a record
  // never depends on its neighbour in the slab
  for (uint32_t k = 0; k < ml; k++) {
    uint8_t b = (k < avail && k < r.msg_len) ? rec[k] : (uint8_t)0;
    if (k == 3) {
      b &= (uint8_t)~MGENX_FLAG_CHECKSUM;
      if (r.flags & MGENX_FLAG_CHECKSUM_ERROR) b |= MGENX_FLAG_CHECKSUM_ERROR;
    }
    s.put(b);
  }
}

struct LogParams {
  const uint8_t* slab;
  uint64_t slab_bytes;
  const uint64_t* rec_off;
  uint64_t stride;
  mgenx_cols cols;
  const mgenx_addr* src;
  const uint32_t* rx_sec;
  const uint32_t* rx_usec;
  const int32_t* ttl;
  uint32_t n;
  int protocol;
  uint32_t opts;
  uint8_t* text;
  uint64_t text_cap;
  uint64_t* line_off;  // n + 1
  uint64_t* lens;      // n + 1 (workspace): line lengths, lens[n] = 0
};

__device__ LogRec gather(const LogParams& p, uint32_t i) {
  const mgenx_cols& c = p.cols;
  LogRec r;
  if (c.rows) {
    const mgenx_rec& w = c.rows[i];
    r.flow = w.flow_id; r.seq = w.seq_num; r.sec = w.tx_sec; r.usec = w.tx_usec;
    r.msg_len = w.msg_len; r.dport = w.dst_port; r.plen = w.payload_len; r.flags = w.flags;
    r.err = w.err; r.dtype = w.dst_type; r.dlen = w.dst_len; r.ptype = w.payload_type;
    r.gps = w.gps_status;
  } else {
    r.flow = c.flow_id[i]; r.seq = c.seq_num[i]; r.sec = c.tx_sec[i]; r.usec = c.tx_usec[i];
    r.msg_len = c.msg_len[i]; r.dport = c.dst_port[i]; r.plen = c.payload_len[i];
    r.flags = c.flags[i]; r.err = c.err[i]; r.dtype = c.dst_type[i]; r.dlen = c.dst_len[i];
    r.ptype = c.payload_type[i]; r.gps = c.gps_status[i];
  }
  for (int k = 0; k < 16; k++) {
    r.daddr[k] = c.dst_addr[(size_t)i * 16 + k];
    r.haddr[k] = c.host_addr[(size_t)i * 16 + k];
  }
  r.hport = c.host_port[i]; r.htype = c.host_type[i]; r.hlen = c.host_len[i];
  r.lat = c.lat_raw[i]; r.lon = c.lon_raw[i]; r.alt = (uint32_t)c.alt[i];
  r.poff = c.payload_off[i];
  r.hdr = c.hdr_len ? c.hdr_len[i] : 0;
  return r;
}

template <typename S, bool kBinary>
__device__ __forceinline__ void format_any(S& s, const LogParams& p, uint32_t i, const LogRec& r) {
  const uint64_t off = p.rec_off ? p.rec_off[i] : (uint64_t)i * p.stride;
  const uint8_t* rec = p.slab + off;
  if (kBinary) {
    const uint64_t avail = off < p.slab_bytes ? p.slab_bytes - off : 0u;
    format_binary(s, r, rec, avail, p.src[i], p.rx_sec[i], p.rx_usec[i], p.protocol);
  } else {
    const int ttl = p.ttl ? p.ttl[i] : -1;
    format_line(s, r, rec, p.src[i], p.rx_sec[i], p.rx_usec[i], p.protocol, ttl, p.opts);
  }
}

template <bool kWrite, bool kBinary>
__global__ void __launch_bounds__(kLogThreads) log_kernel(LogParams p) {
  const uint32_t i = blockIdx.x * kLogThreads + threadIdx.x;
  if (i >= p.n) return;
  const LogRec r = gather(p, i);
  if (!kWrite) {
    CountSink s;
    format_any<CountSink, kBinary>(s, p, i, r);
    p.lens[i] = s.n;
  } else {
    const uint64_t off = p.line_off[i], end = p.line_off[i + 1];
    if (end > p.text_cap) return;  // does not fit: the caller sees line_off[n] > capacity
    WriteSink s{p.text + off};
    format_any<WriteSink, kBinary>(s, p, i, r);
  }
}

__global__ void log_tail_kernel(uint64_t* lens, uint32_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) lens[n] = 0;
}

}  // namespace mgenx

using namespace mgenx;

struct mgenx_log_ws {
  void* mem = nullptr;
  size_t bytes = 0;
};

extern "C" void* mgenx_log_ws_new() { return new mgenx_log_ws(); }
extern "C" void mgenx_log_ws_free(void* p) {
  mgenx_log_ws* w = static_cast<mgenx_log_ws*>(p);
  if (!w) return;
  if (w->mem) (void)hipFree(w->mem);
  delete w;
}

extern "C" int mgenx_log_recv_run(void* wsp, bool binary, const uint8_t* slab,
                                  uint64_t slab_bytes, const uint64_t* rec_off,
                                       uint64_t stride, const mgenx_cols* cols,
                                       const mgenx_addr* src, const uint32_t* rx_sec,
                                       const uint32_t* rx_usec, const int32_t* ttl, uint32_t n,
                                       int protocol, uint32_t opts, char* text,
                                       uint64_t text_cap, uint64_t* line_off,
                                       hipStream_t stream, char* err, size_t errn) {
  mgenx_log_ws& ws = *static_cast<mgenx_log_ws*>(wsp);
  LogParams p;
  p.slab = slab; p.slab_bytes = slab_bytes; p.rec_off = rec_off; p.stride = stride; p.cols = *cols; p.src = src;
  p.rx_sec = rx_sec; p.rx_usec = rx_usec; p.ttl = ttl; p.n = n; p.protocol = protocol;
  p.opts = opts; p.text = reinterpret_cast<uint8_t*>(text); p.text_cap = text_cap;
  p.line_off = line_off;
  const int grid = (int)((n + kLogThreads - 1) / kLogThreads);
  // workspace: line lengths (n + 1 u64), then the scan's temporary storage
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n + 1, stream);
  const size_t len_bytes = (((size_t)n + 1) * 8 + 255) & ~(size_t)255;
  const size_t need = len_bytes + scan_bytes;
  if (ws.bytes < need) {
    if (ws.mem) (void)hipFree(ws.mem);
    ws.mem = nullptr;
    ws.bytes = 0;
    if (hipMalloc(&ws.mem, need) != hipSuccess) {
      snprintf(err, errn, "log: workspace of %zu bytes", need);
      return MGENX_EDEVICE;
    }
    ws.bytes = need;
  }
  p.lens = static_cast<uint64_t*>(ws.mem);
  // pass 1: lengths; line_off = exclusive scan of the n + 1 lengths (lens[n] = 0)
  if (binary) hipLaunchKernelGGL((log_kernel<false, true>), dim3(grid), dim3(kLogThreads), 0, stream, p);
  else hipLaunchKernelGGL((log_kernel<false, false>), dim3(grid), dim3(kLogThreads), 0, stream, p);
  hipLaunchKernelGGL(log_tail_kernel, dim3(1), dim3(64), 0, stream, p.lens, n);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(static_cast<uint8_t*>(ws.mem) + len_bytes, have, p.lens,
                                       line_off, (int)n + 1, stream) != hipSuccess) {
    snprintf(err, errn, "log: scan failed");
    return MGENX_EDEVICE;
  }
  // pass 2: the lines
  if (binary) hipLaunchKernelGGL((log_kernel<true, true>), dim3(grid), dim3(kLogThreads), 0, stream, p);
  else hipLaunchKernelGGL((log_kernel<true, false>), dim3(grid), dim3(kLogThreads), 0, stream, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err, errn, "log: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  return MGENX_OK;
}
