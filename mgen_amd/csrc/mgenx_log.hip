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
#include <string.h>

#include <mutex>

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
// logged as ERROR_LENGTH, as include/mgenx.hpp maps it; MGENX_ERROR_RERR_NONE is a RERR
// event of an error-free message (LogRecvError called on it): "none", code 0
__device__ __forceinline__ uint32_t log_error(uint32_t e) {
  return e == MGENX_ERROR_OOB ? (uint32_t)MGENX_ERROR_LENGTH
                              : e == MGENX_ERROR_RERR_NONE ? 0u : e;
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
// recordLength - index + 4 = hdr + payload_len message bytes (index = 16 + source address
// length: eventRecordLength counts from after the 4-byte record header, doc/mgen.xml:
// 4212-4216) with CHECKSUM cleared in the flags byte.  Bytes past the slab are written 0.
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
  const uint32_t ml = (rl - (16u + alen) + 4u) & 0xFFFFu;  // = hdr + payload_len
  // a byte past the received record (avail: its length, or msg_len when the caller has no
  // lengths) is written as zero, so a record never depends on its neighbour in the slab
  for (uint32_t k = 0; k < ml; k++) {
    uint8_t b = k < avail ? rec[k] : (uint8_t)0;
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
  const uint32_t* rec_len;  // binary: the received lengths (NULL: each record's msg_len)
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
    uint64_t avail = off < p.slab_bytes ? p.slab_bytes - off : 0u;
    const uint64_t len = p.rec_len ? p.rec_len[i] : r.msg_len;
    if (avail > len) avail = len;
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
  // MGENX_LOG_SKIP_ERR: a record Unpack rejected gets no line (pcap2mgen.cpp:428-432)
  if (!kBinary && (p.opts & MGENX_LOG_SKIP_ERR) && r.err) {
    if (!kWrite) p.lens[i] = 0;
    return;
  }
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

// One scratch area per stream (line lengths + scan temporaries), so log calls on one context
// but different streams never share a buffer; an area grows (hipMalloc) only when a batch
// outgrows it.
struct mgenx_log_ws {
  void* mem = nullptr;
  size_t bytes = 0;
  hipStream_t stream = nullptr;
  mgenx_log_ws* next = nullptr;
};

extern "C" void* mgenx_log_ws_new() { return new mgenx_log_ws(); }
extern "C" void mgenx_log_ws_free(void* p) {
  mgenx_log_ws* w = static_cast<mgenx_log_ws*>(p);
  while (w) {
    mgenx_log_ws* nx = w->next;
    mgenx::dev_free(w->mem);
    delete w;
    w = nx;
  }
}
// the area of `stream` (the head is the first stream's; others are chained)
static mgenx_log_ws& ws_for(void* wsp, hipStream_t stream) {
  static std::mutex mu;  // the chain is shared by the context's host threads
  std::lock_guard<std::mutex> lock(mu);
  mgenx_log_ws* head = static_cast<mgenx_log_ws*>(wsp);
  if (!head->mem && !head->next && head->bytes == 0) head->stream = stream;
  for (mgenx_log_ws* w = head; w; w = w->next)
    if (w->stream == stream) return *w;
  mgenx_log_ws* w = new mgenx_log_ws();
  w->stream = stream;
  w->next = head->next;
  head->next = w;
  return *w;
}

extern "C" int mgenx_log_recv_run(void* wsp, bool binary, const uint8_t* slab,
                                  uint64_t slab_bytes, const uint64_t* rec_off,
                                  const uint32_t* rec_len,
                                       uint64_t stride, const mgenx_cols* cols,
                                       const mgenx_addr* src, const uint32_t* rx_sec,
                                       const uint32_t* rx_usec, const int32_t* ttl, uint32_t n,
                                       int protocol, uint32_t opts, char* text,
                                       uint64_t text_cap, uint64_t* line_off,
                                       hipStream_t stream, char* err, size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  LogParams p;
  p.slab = slab; p.slab_bytes = slab_bytes; p.rec_off = rec_off; p.rec_len = rec_len;
  p.stride = stride; p.cols = *cols; p.src = src;
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
    mgenx::dev_free(ws.mem);
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

// ====================================================================================
// MGEN_DATA items: MgenAnalytic::Report (build, parse, REPORT lines) and the payload TLV
// walk with MgenFlowCommand.  References: mgenAnalytic.cpp:28-71 (Init), :220-254 (the
// report at a window close), :260-295 (MgenAnalytic::Log), :296-310 (GetReport), :343-566
// (Report parse / build), :568-642 (quantizers), :747-786 (Report::Log);
// mgenTransport.cpp:2132-2191 (ProcessRecvMessage); mgenPayload.cpp:276-347
// (MgenFlowCommand); include/mgenAnalytic.h:14-57 (wire format).  ProtoPkt fields are
// network byte order.  Restated in oracle/mgen_oracle.c (or_report_*, or_data_walk).
// ====================================================================================
namespace mgenx {

struct Rq {
  const double* t;  // the context's kRq* tables
};

__device__ __forceinline__ double mulr(double a, double b) {  // no FMA contraction
  double p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}

// QuantizeTimeValue: the host's log formula through its own thresholds
__device__ uint8_t rq_q_time(const Rq& r, double v) {
  if (v > mulr(1.1, 600.0)) return 0xff;
  if (v < 1.0e-06 / 2.0) return 0;
  if (v < 1.0e-06) return 1;
  const double* T = r.t + kRqThrTime;
  uint32_t lo = 2, hi = 256;  // first k with T[k] > v
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (T[m] <= v) lo = m + 1; else hi = m;
  }
  return (uint8_t)(lo - 1);
}
__device__ __forceinline__ double rq_uq_time(const Rq& r, uint8_t q) { return r.t[kRqUnqTime + q]; }

__device__ uint16_t rq_q_rate(const Rq& r, double rate) {
  if (rate <= 0.0) return 0x01;
  // (UINT16)(int)log10(rate) from the host's thresholds; outside them the device's log10
  const double* T = r.t + kRqThrLog10;
  int32_t e;
  if (rate < T[0] || !(rate < T[kRqLog10N - 1])) {
    e = (int32_t)log10(rate);
  } else {
    uint32_t lo = 0, hi = kRqLog10N;  // first j with T[j] > rate
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (T[m] <= rate) lo = m + 1; else hi = m;
    }
    e = kRqLog10Lo + (int32_t)lo - 1;
  }
  const uint16_t ex = (uint16_t)e;
  const double p10 = ex < kRqP10N ? r.t[kRqP10 + ex] : __builtin_huge_val();
  const uint16_t mant = (uint16_t)(int32_t)(mulr(4096.0 / 10.0, rate / p10) + 0.5);
  return (uint16_t)((mant << 4) | ex);
}
__device__ __forceinline__ double rq_uq_rate(const Rq& r, uint16_t q) {
  return mulr(mulr((double)(q >> 4), 10.0 / 4096.0), r.t[kRqP10 + (q & 0xfu)]);
}
__device__ __forceinline__ uint16_t rq_q_loss(double loss) {
  if (0.0 == loss) return 0;
  loss = mulr(loss, 65535.0) + 0.5;
  if (loss < 1.0) return 1;
  if (loss > 65535.0) return 65535;
  return (uint16_t)loss;
}
__device__ __forceinline__ double rq_uq_loss(uint16_t q) { return (double)q / 65535.0; }

__device__ __forceinline__ void p16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
__device__ __forceinline__ uint32_t g16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

struct RepOff {
  uint32_t alen, src, dport, sport, fid, ws, lave, lmin, lmax, rate, loss, end;
};
__device__ __forceinline__ RepOff rep_off(uint8_t b0, uint8_t b2) {
  RepOff o;
  const uint32_t type = b0 >> 4;
  o.alen = type == 1 ? 4u : (type == 2 ? 16u : 0u);
  o.src = 4u * (1u + o.alen / 4u);
  o.dport = o.src + o.alen;
  o.sport = o.dport + 2u;
  o.fid = o.sport + 2u;
  o.ws = o.fid + (((b2 >> 5) & 1u) ? 4u : 0u);
  o.lave = o.ws + 1u; o.lmin = o.lave + 1u; o.lmax = o.lmin + 1u;
  o.rate = o.lmax + 1u; o.loss = o.rate + 2u; o.end = o.loss + 2u;
  return o;
}

// report_msg after Init (key) and a window close, then GetReport (offset >= 0)
__device__ uint32_t rep_build(const Rq& r, const mgenx_report_key& k, const mgenx_flow_report& w,
                              double offset, bool& sign, uint8_t* b /*52*/) {
  for (int i = 0; i < 52; i++) b[i] = 0;
  b[0] = (uint8_t)(1u << 4);
  b[1] = 16;
  b[0] = (uint8_t)((b[0] & 0xf0u) | (k.protocol & 0x0fu));
  for (int j = 0; j < 2; j++) {
    const mgenx_addr& a = j == 0 ? k.dst : k.src;
    uint32_t alen, type;
    if (a.type == 1) { type = 1; alen = 4; }
    else if (a.type == 2) { type = 2; alen = 16; }
    else continue;
    b[0] = (uint8_t)((b[0] & 0x0fu) | (type << 4));
    b[1] = (uint8_t)(16u + 2u * alen);
    const RepOff o = rep_off(b[0], b[2]);
    if (j == 0) {
      for (uint32_t i = 0; i < alen; i++) b[4 + i] = a.addr[i];
      p16(b + o.dport, a.port);
    } else {
      for (uint32_t i = 0; i < alen; i++) b[o.src + i] = a.addr[i];
      p16(b + o.sport, a.port);
    }
  }
  if (k.flow_id != 1u) {
    RepOff o = rep_off(b[0], b[2]);
    const uint32_t rl = o.src + o.alen + 16u;
    b[2] |= (uint8_t)(1u << 5);
    o = rep_off(b[0], b[2]);
    b[o.fid] = (uint8_t)(k.flow_id >> 24); b[o.fid + 1] = (uint8_t)(k.flow_id >> 16);
    b[o.fid + 2] = (uint8_t)(k.flow_id >> 8); b[o.fid + 3] = (uint8_t)k.flow_id;
    b[1] = (uint8_t)rl;
  }
  const RepOff o = rep_off(b[0], b[2]);
  b[o.ws] = rq_q_time(r, w.duration);
  if (w.latency_ave < 0.0) sign = true;
  if (sign) b[2] |= (uint8_t)(2u << 5);
  b[o.lave] = rq_q_time(r, fabs(w.latency_ave));
  b[o.lmin] = rq_q_time(r, fabs(w.latency_ave - w.latency_min));
  b[o.lmax] = rq_q_time(r, fabs(w.latency_max - w.latency_ave));
  p16(b + o.rate, rq_q_rate(r, w.rate));
  p16(b + o.loss, rq_q_loss(w.loss));
  const uint32_t q = rq_q_time(r, offset < 0.0 ? 0.0 : offset);
  p16(b + 2, (g16(b + 2) & 0xe000u) | q);
  return b[1];
}

struct RepView {
  bool valid;
  uint8_t protocol, flags, length;
  mgenx_addr src, dst;
  uint32_t flow_id;
  double offset, window, ave, mn, mx, rate, loss;
};

// the getters over a report buffer as it is (report type 1 or 2; no length check)
template <typename B>
__device__ void rep_view(const Rq& r, const B& byte, RepView& v) {
  const uint8_t b0 = byte(0), b2 = byte(2);
  const uint32_t type = b0 >> 4;
  const RepOff o = rep_off(b0, b2);
  v.protocol = b0 & 0x0f;
  v.flags = b2 >> 5;
  v.length = byte(1);
  const uint8_t at = type == 1 ? 1 : 2;
  v.dst.type = at; v.dst.len = (uint8_t)o.alen;
  v.src.type = at; v.src.len = (uint8_t)o.alen;
  for (int i = 0; i < 16; i++) {
    v.dst.addr[i] = (uint32_t)i < o.alen ? byte(4 + i) : 0;
    v.src.addr[i] = (uint32_t)i < o.alen ? byte(o.src + i) : 0;
  }
  v.dst.port = (uint16_t)((uint32_t)byte(o.dport) << 8 | byte(o.dport + 1));
  v.src.port = (uint16_t)((uint32_t)byte(o.sport) << 8 | byte(o.sport + 1));
  v.flow_id = (v.flags & 1u) ? ((uint32_t)byte(o.fid) << 24 | (uint32_t)byte(o.fid + 1) << 16 |
                                (uint32_t)byte(o.fid + 2) << 8 | byte(o.fid + 3))
                             : 0u;
  v.offset = rq_uq_time(r, (uint8_t)((((uint32_t)b2 << 8) | byte(3)) & 0x1fffu));
  v.window = rq_uq_time(r, byte(o.ws));
  const double ave = rq_uq_time(r, byte(o.lave));
  v.ave = (v.flags & 2u) ? -ave : ave;
  v.mn = v.ave - rq_uq_time(r, byte(o.lmin));
  v.mx = v.ave + rq_uq_time(r, byte(o.lmax));
  v.rate = rq_uq_rate(r, (uint16_t)((uint32_t)byte(o.rate) << 8 | byte(o.rate + 1)));
  v.loss = rq_uq_loss((uint16_t)((uint32_t)byte(o.loss) << 8 | byte(o.loss + 1)));
}

// Report::InitFromBuffer(b, avail) + the getters (byte(k) reads past avail as 0)
template <typename B>
__device__ bool rep_parse(const Rq& r, const B& byte, uint32_t avail, RepView& v) {
  v.valid = false;
  if (avail < 2 || byte(1) > avail) return false;
  const uint8_t b0 = byte(0), b2 = byte(2);
  const uint32_t type = b0 >> 4;
  if (type != 1 && type != 2) return false;
  if (byte(1) != rep_off(b0, b2).end) return false;
  rep_view(r, byte, v);
  v.valid = true;
  return true;
}

// "%lf" of any double as glibc prints it: the exact binary value rounded to 6 decimals,
// ties to even; inf / nan as "inf" / "nan" with the sign
template <typename S>
__device__ void put_f6(S& s, double v) {
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const bool neg = (bits >> 63) != 0;
  const uint32_t ex = (uint32_t)((bits >> 52) & 0x7ffu);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (neg) s.put('-');
  if (ex == 0x7ffu) {
    put_str(s, frac ? "nan" : "inf");
    return;
  }
  const uint64_t mant = frac | (ex ? (1ull << 52) : 0ull);
  const int e = (ex ? (int)ex : 1) - 1075;  // |v| = mant * 2^e
  if (e <= 40) {
    // |v| * 1e6 = mant * 1e6 * 2^e < 2^113: 128-bit integer arithmetic
    const unsigned __int128 P = (unsigned __int128)mant * 1000000u;
    unsigned __int128 q;
    if (e >= 0) {
      q = P << e;
    } else if (-e >= 100) {
      q = 0;
    } else {
      const int sh = -e;
      q = P >> sh;
      const unsigned __int128 rem = P - (q << sh);
      const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
      if (rem > half || (rem == half && (q & 1))) q++;
    }
    const unsigned __int128 ip = q / 1000000u;
    const uint64_t fp = (uint64_t)(q % 1000000u);
    // integer part: up to 2^93 / 1e6 < 2^74 -- two 64-bit halves in decimal
    if (ip >> 64) {
      const uint64_t base = 10000000000000000000ull;  // 1e19
      const uint64_t hi = (uint64_t)(ip / base), lo = (uint64_t)(ip % base);
      put_u64(s, hi);
      put_u64(s, lo, 19);
    } else {
      put_u64(s, (uint64_t)ip);
    }
    s.put('.');
    put_u64(s, fp, 6);
    return;
  }
  // |v| >= 2^93: an integer; its decimal digits by long division of mant * 2^e
  uint32_t w[34];
  int nw = 0;
  for (int i = 0; i < 34; i++) w[i] = 0;
  w[e / 32] = (uint32_t)(mant << (e % 32));
  w[e / 32 + 1] = (uint32_t)(mant >> (32 - e % 32));
  w[e / 32 + 2] = (e % 32) ? (uint32_t)(mant >> (64 - e % 32)) : 0u;
  nw = e / 32 + 3;
  char dig[330];
  int nd = 0;
  for (;;) {
    while (nw > 0 && w[nw - 1] == 0) nw--;
    if (nw == 0) break;
    uint64_t rem = 0;
    for (int i = nw - 1; i >= 0; i--) {
      const uint64_t cur = (rem << 32) | w[i];
      w[i] = (uint32_t)(cur / 1000000000u);
      rem = cur % 1000000000u;
    }
    for (int k = 0; k < 9; k++) {
      dig[nd++] = (char)('0' + rem % 10);
      rem /= 10;
    }
  }
  while (nd > 1 && dig[nd - 1] == '0') nd--;
  for (int i = nd - 1; i >= 0; i--) s.put((uint8_t)dig[i]);
  put_str(s, ".000000");
}

__device__ __forceinline__ const char* rep_proto(uint32_t p) {
  return p == 1 ? "UDP" : p == 2 ? "TCP" : p == 3 ? "SINK" : "???";
}

template <typename S>
__device__ void put_rep_head(S& s, const RepView& v) {
  put_str(s, "REPORT proto>");
  put_str(s, rep_proto(v.protocol));
  put_str(s, " flow>");
  put_u64(s, v.flow_id ? v.flow_id : 1u);
  put_str(s, " src>");
  put_addr(s, v.src.type, v.src.len, v.src.addr);
  s.put('/');
  put_u64(s, v.src.port);
  put_str(s, " dst>");
  put_addr(s, v.dst.type, v.dst.len, v.dst.addr);
  s.put('/');
  put_u64(s, v.dst.port);
  s.put(' ');
}

template <typename S>
__device__ void put_rep_values(S& s, double window, double rate, double loss, double ave,
                               double mn, double mx) {
  put_str(s, "window>");
  put_f6(s, window);
  put_str(s, " rate>");
  put_f6(s, mulr(rate, 8.0e-03));
  put_str(s, " kbps loss>");
  put_f6(s, loss);
  put_str(s, " latency ave>");
  put_f6(s, ave);
  put_str(s, " min>");
  put_f6(s, mn);
  put_str(s, " max>");
  put_f6(s, mx);
}

struct ItemBytes {
  const uint8_t* p;
  uint32_t n;
  __device__ uint8_t operator()(uint32_t k) const { return k < n ? p[k] : (uint8_t)0; }
};

// ---- kernels ----
// one thread per flow, its kept reports in order (FLAG_LATENCY_SIGN is never cleared)
__global__ void report_build_kernel(const mgenx_flow_report* __restrict__ reps, uint32_t n_flows,
                                    uint32_t per_flow, const uint32_t* __restrict__ count,
                                    const mgenx_report_key* __restrict__ keys,
                                    uint8_t* __restrict__ sign, const double* __restrict__ offset,
                                    const double* rq, uint8_t* __restrict__ items,
                                    uint8_t* __restrict__ item_len) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_flows) return;
  const Rq r{rq};
  const mgenx_report_key k = keys[f];
  bool sg = sign[f] != 0;
  const uint32_t m = min(count[f], per_flow);
  for (uint32_t j = 0; j < m; j++) {
    const size_t slot = (size_t)f * per_flow + j;
    uint8_t b[52];
    item_len[slot] = (uint8_t)rep_build(r, k, reps[slot], offset ? offset[slot] : 0.0, sg, b);
    for (int i = 0; i < 52; i++) items[slot * 52 + i] = b[i];
  }
  sign[f] = sg ? 1u : 0u;
}

struct RepLineParams {
  const uint8_t* items;             // 52 B per slot (built reports / received report bytes)
  const mgenx_flow_report* reps;    // analytic lines: the doubles; NULL = received reports
  const uint32_t* count;            // analytic lines: kept reports per flow
  uint32_t per_flow;
  const uint64_t* rep_pairs;        // received: (record, slab offset of the item) pairs
  const uint8_t* slab;
  const mgenx_addr* reporter;       // received: per record, the message's source
  const uint32_t* rx_sec;           // received: per record
  const uint32_t* rx_usec;
  uint32_t n;                       // slots
  uint32_t opts;
  const double* rq;
  uint8_t* text;
  uint64_t text_cap;
  uint64_t* line_off;
  uint64_t* lens;
};

template <typename S>
__device__ void rep_line(S& s, const RepLineParams& p, uint32_t i) {
  const Rq r{p.rq};
  const bool epoch = (p.opts & MGENX_LOG_EPOCH) != 0;
  RepView v = {};  // deterministic for an invalid item handed in (both passes agree)
  if (p.reps) {  // MgenAnalytic::Log (mgenAnalytic.cpp:260-295)
    const uint32_t f = i / p.per_flow, j = i % p.per_flow;
    if (j >= min(p.count[f], p.per_flow)) return;
    const mgenx_flow_report& w = p.reps[i];
    // the getters read the buffer as it is: a report whose addresses were invalid keeps
    // InitIntoBuffer's IPv4 type and length 16 (mgenAnalytic.cpp:63-67)
    rep_view(r, ItemBytes{p.items + (size_t)i * 52, 52}, v);
    put_ts(s, (uint32_t)w.rx_sec, (uint32_t)w.rx_usec, epoch);
    put_rep_head(s, v);
    put_rep_values(s, w.duration, w.rate, w.loss, w.latency_ave, w.latency_min, w.latency_max);
    put_str(s, ", count>");
    put_u64(s, (uint32_t)w.msg_count);
    s.put('\n');
  } else {  // MgenAnalytic::Report::Log (mgenAnalytic.cpp:747-786)
    const uint64_t rec = p.rep_pairs[2 * (size_t)i];
    rep_parse(r, ItemBytes{p.slab + p.rep_pairs[2 * (size_t)i + 1], 52}, 52, v);
    put_ts(s, p.rx_sec[rec], p.rx_usec[rec], epoch);
    put_rep_head(s, v);
    put_str(s, "reporter>");
    const mgenx_addr& a = p.reporter[rec];
    put_addr(s, a.type, a.len, a.addr);
    s.put('/');
    put_u64(s, a.port);
    put_str(s, " sent>");
    put_ts(s, p.rx_sec[rec], p.rx_usec[rec], epoch);  // theTime, as the reference prints it
    put_str(s, "offset>");
    put_f6(s, v.offset);
    s.put(' ');
    put_rep_values(s, v.window, v.rate, v.loss, v.ave, v.mn, v.mx);
    s.put('\n');
  }
}

template <bool kWrite>
__global__ void __launch_bounds__(kLogThreads) rep_line_kernel(RepLineParams p) {
  const uint32_t i = blockIdx.x * kLogThreads + threadIdx.x;
  if (i >= p.n) return;
  if (!kWrite) {
    CountSink s;
    rep_line(s, p, i);
    p.lens[i] = s.n;
  } else {
    const uint64_t off = p.line_off[i], end = p.line_off[i + 1];
    if (end > p.text_cap) return;
    WriteSink s{p.text + off};
    rep_line(s, p, i);
  }
}

// MgenFlowCommand::GetStatus (mgenPayload.cpp:326-347)
template <typename B>
__device__ uint32_t flowcmd_status(const B& byte, uint32_t base, uint32_t len, uint32_t flow) {
  const uint32_t N = (2 * flow > 16) ? (2 * flow - 16 - 1) / 32 + 1 : 0;
  if (2 + 2 + N * 4 > len) return 0;
  const uint32_t f = flow - 1;
  uint32_t st = (byte(base + 2 + (f >> 3)) & (0x80u >> (f & 7))) ? 1u : 0u;
  if (byte(base + 2 + (len - 2) / 2 + (f >> 3)) & (0x80u >> (f & 7))) st |= 2u;
  return st;
}

struct WalkParams {
  const uint8_t* slab;
  const uint64_t* rec_off;
  uint64_t stride;
  mgenx_cols cols;
  uint32_t n;
  uint32_t opts;
  const double* rq;
  uint8_t* status;        // per record
  uint8_t* needs_host;    // per record
  uint32_t* n_cmd;        // per record (pass 1), n + 1
  uint32_t* n_rep;
  const uint32_t* cmd_base;  // pass 2
  const uint32_t* rep_base;
  uint32_t* cmds;         // 2 words: record, flow << 2 | status
  uint32_t cmd_cap;
  uint64_t* reps;         // 2 words: record, slab offset of the report item
  uint32_t rep_cap;
};

// MgenTransport::ProcessRecvMessage (mgenTransport.cpp:2132-2191) for record i
template <bool kWrite>
__global__ void __launch_bounds__(256) data_walk_kernel(WalkParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const mgenx_cols& c = p.cols;
  const bool mine = c.err[i] == 0 && c.payload_type[i] == MGENX_PAYLOAD_MGEN_DATA;
  if (!kWrite) {
    p.n_cmd[i] = 0;
    p.n_rep[i] = 0;
    if (i == 0) { p.n_cmd[p.n] = 0; p.n_rep[p.n] = 0; }
    p.status[i] = mine ? 0 : 0xff;
    p.needs_host[i] = 0;
  }
  if (!mine) return;
  const Rq r{p.rq};
  const uint64_t off0 = (p.rec_off ? p.rec_off[i] : (uint64_t)i * p.stride) + c.payload_off[i];
  const uint32_t plen = c.payload_len[i];
  const ItemBytes all{p.slab + off0, plen};
  uint32_t off = 0, left = plen, nc = 0, nr = 0, st = 0;
  uint32_t cw = kWrite ? p.cmd_base[i] : 0, rw = kWrite ? p.rep_base[i] : 0;
  const bool ctl = (p.opts & MGENX_DATA_CONTROLLER) != 0;
  while (left > 0) {
    const uint32_t type = all(off);
    const uint32_t ilen = left > 1 ? all(off + 1) : 0u;
    if (type == 1) {  // DATA_ITEM_FLOW_CMD
      if (ilen > left) { st = 1; break; }
      uint32_t maxf = ilen > 2 ? 8 * (ilen - 2) / 2 : 0;
      if (maxf > MGENX_MAX_FLOW) maxf = MGENX_MAX_FLOW;
      for (uint32_t fl = 1; fl <= maxf; fl++) {
        const uint32_t s2 = flowcmd_status(all, off, ilen, fl);
        if (!s2) continue;
        if (kWrite && cw < p.cmd_cap) {
          p.cmds[2 * (size_t)cw] = i;
          p.cmds[2 * (size_t)cw + 1] = fl << 2 | s2;
        }
        cw++;
        nc++;
      }
      if (ilen == 0) { st = 3; break; }
      left -= ilen;
      off += (ilen / 4) * 4;
    } else if (ctl && type > 0x0f) {
      RepView v;
      const ItemBytes it{p.slab + off0 + off, left};
      if (!rep_parse(r, it, left, v)) { st = 2; break; }
      if (kWrite && rw < p.rep_cap) {
        p.reps[2 * (size_t)rw] = i;
        p.reps[2 * (size_t)rw + 1] = off0 + off;
      }
      rw++;
      nr++;
      left -= v.length;
      off += (v.length / 4u) * 4u;
    } else {
      if (ilen > left || ilen == 0) { st = 3; break; }
      left -= ilen;
      off += (ilen / 4) * 4;
    }
  }
  if (!kWrite) {
    p.n_cmd[i] = nc;
    p.n_rep[i] = nr;
    p.status[i] = (uint8_t)st;
    p.needs_host[i] = (nc || nr) ? 1u : 0u;
  }
}

// ---- mgenx_text_interleave: several line sources -> one log in record order ----
struct TextParams {
  mgenx_text_src src[MGENX_TEXT_MAX_SRC];
  uint32_t n_src;
  uint32_t n_rec;
  uint8_t* out;
  uint64_t cap;
  uint64_t* rec_off;  // n_rec + 1
  uint64_t* lens;     // n_rec + 1 (workspace)
};

// first line k in [0, n) whose owner is >= r
__device__ __forceinline__ uint32_t owner_lb(const mgenx_text_src& t, uint32_t r) {
  uint32_t lo = 0, hi = t.n_lines;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (t.index[(size_t)mid * t.index_stride] < r) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// record i's lines of source t: [lo, hi)
__device__ __forceinline__ void text_range(const mgenx_text_src& t, uint32_t i, uint32_t& lo,
                                           uint32_t& hi) {
  lo = hi = 0;
  if (t.kind == MGENX_TEXT_PER_RECORD) {
    if (i < t.n_lines) { lo = i; hi = i + 1; }
  } else if (t.kind == MGENX_TEXT_OWNER) {
    lo = owner_lb(t, i);
    hi = owner_lb(t, i + 1);
  } else {
    const uint32_t l = t.index[i];
    if (l < t.n_lines) { lo = l; hi = l + 1; }
  }
}

// MGENX_TEXT_SCATTER -> a record -> line map (the map is pre-filled with MGENX_FLOW_NONE)
__global__ void __launch_bounds__(256) text_scatter_kernel(const uint32_t* __restrict__ rec_of_line,
                                                           uint32_t n_lines, uint32_t n_rec,
                                                           uint32_t* __restrict__ map) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_lines) return;
  const uint32_t r = rec_of_line[k];
  if (r < n_rec) map[r] = k;
}

__global__ void __launch_bounds__(256) text_len_kernel(TextParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > p.n_rec) return;
  uint64_t len = 0;
  if (i < p.n_rec) {
    for (uint32_t s = 0; s < p.n_src; s++) {
      uint32_t lo, hi;
      text_range(p.src[s], i, lo, hi);
      if (hi > lo) len += p.src[s].line_off[hi] - p.src[s].line_off[lo];
    }
  }
  p.lens[i] = len;
}

// one wave per record: each source's bytes copied with the lanes side by side
__global__ void __launch_bounds__(256) text_copy_kernel(TextParams p) {
  const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (i >= p.n_rec) return;
  uint64_t pos = p.rec_off[i];
  if (p.rec_off[i + 1] > p.cap) return;  // does not fit: the caller reads rec_off[n]
  for (uint32_t s = 0; s < p.n_src; s++) {
    uint32_t lo, hi;
    text_range(p.src[s], i, lo, hi);
    if (hi <= lo) continue;
    const uint64_t a = p.src[s].line_off[lo], b = p.src[s].line_off[hi];
    const uint8_t* src = reinterpret_cast<const uint8_t*>(p.src[s].text);
    for (uint64_t k = a + lane; k < b; k += 64) p.out[pos + (k - a)] = src[k];
    pos += b - a;
  }
}

// ---- ConvertBinaryLog (mgenMsg.cpp:1417-1900) -----------------------------------------
// Record i's header at rec_off[i] (mgenx_binlog_index found it): {type, protocol, BE
// recordLength} then the body.  binlog_parse_kernel places each RECV / SEND record's stored
// message for mgenx_unpack_batch; binlog_line_kernel writes every record's line.
struct BinParams {
  const uint8_t* buf;
  const uint64_t* rec_off;
  uint32_t n;
  uint64_t* msg_off;      // RECV / SEND: the stored message; others: the record (len 0)
  uint32_t* msg_len;
  mgenx_addr* src;        // RECV: the source address and port
  uint32_t* ev_sec;
  uint32_t* ev_usec;
  uint32_t* aux;          // SEND over TCP: mgen_msg_len
  uint8_t* kind;          // event type
  uint8_t* proto;
  mgenx_cols cols;        // the unpack outputs (core + extended)
  uint32_t log_rx, flush, opts;
  uint8_t* text;
  uint64_t text_cap;
  uint64_t* line_off;     // n + 1
  uint64_t* lens;         // n + 1 (workspace)
};

__device__ __forceinline__ uint32_t be16(const uint8_t* b) { return (uint32_t)b[0] << 8 | b[1]; }
__device__ __forceinline__ uint32_t be32(const uint8_t* b) {
  return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
}

__global__ void __launch_bounds__(256) binlog_parse_kernel(BinParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t ro = p.rec_off[i];
  const uint8_t* h = p.buf + ro;
  const uint8_t* b = h + 4;
  const uint32_t ev = h[0], proto = h[1], rl = be16(h + 2);
  p.kind[i] = (uint8_t)ev;
  p.proto[i] = (uint8_t)proto;
  p.ev_sec[i] = be32(b);
  p.ev_usec[i] = be32(b + 4);
  uint64_t mo = ro;
  uint32_t ml = 0, aux = 0;
  mgenx_addr a;
  a.type = 0; a.len = 0; a.port = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) a.addr[k] = 0;
  if (ev == 1) {  // RECV (:1560-1609): srcPort, type, length, address, then the message
    const uint32_t alen = b[11];
    a.type = b[10];
    a.len = (uint8_t)(alen < 16 ? alen : 16);
    a.port = (uint16_t)be16(b + 8);
    for (uint32_t k = 0; k < a.len; k++) a.addr[k] = b[12 + k];
    mo = ro + 4 + 12 + alen;
    ml = rl >= 12 + alen ? rl - 12 - alen : 0u;
  } else if (ev == 3) {  // SEND (:1610-1627): [BE mgen_msg_len for TCP] then the message
    const uint32_t idx = proto == 2 ? 4u : 0u;
    if (proto == 2) aux = be32(b);
    mo = ro + 4 + idx;
    // the stored bytes: the reference passes recordLength (:1624), whose last 4 bytes after
    // a TCP SEND's length word are stale read-buffer bytes (:1434); bounded at the record
    ml = rl - idx;
  }
  p.msg_off[i] = mo;
  p.msg_len[i] = ml;
  p.src[i] = a;
  p.aux[i] = aux;
}

// "host>%s/%hu" of the ON ... RECONNECT records (:1790-1824, 1887-1888)
template <typename S>
__device__ void bl_conn_line(S& s, const BinParams& p, const uint8_t* b, uint32_t ev, uint32_t rl) {
  const bool epoch = (p.opts & MGENX_LOG_EPOCH) != 0;
  const uint8_t at = b[10];
  const uint32_t alen = b[11];
  const uint8_t* a = b + 12;
  uint32_t i = 12 + alen;
  const uint32_t aport = be16(b + 8), dport = be16(b + i);
  i += 2;
  const uint32_t fid = be32(b + i);
  i += 4;
  bool hvalid = false;
  uint32_t hport = 0, ht = 0, hl = 0;
  const uint8_t* ha = nullptr;
  if (i + 4 <= rl) {
    hport = be16(b + i);
    i += 2;
    ht = b[i++];
    if (ht != 1 && ht != 2) ht = 0;
    hl = b[i++];
    if (i + hl <= rl && ht && hl) { ha = b + i; hvalid = true; }
  }
  put_ts(s, be32(b), be32(b + 4), epoch);
  auto addr = [&]() { put_addr(s, at, (uint8_t)alen, a); s.put('/'); put_u64(s, aport); };
  auto flow_first = [&](const char* name) {  // "<NAME> flow>F srcPort>P dst>A/p"
    put_str(s, name); put_str(s, " flow>"); put_u64(s, fid); put_str(s, " srcPort>");
    put_u64(s, dport); put_str(s, " dst>"); addr();
  };
  auto flow_dst = [&](const char* name) {    // "<NAME> flow>F dst>A/p srcPort>P"
    put_str(s, name); put_str(s, " flow>"); put_u64(s, fid); put_str(s, " dst>"); addr();
    put_str(s, " srcPort>"); put_u64(s, dport);
  };
  auto server = [&](const char* name) {      // "<NAME> src>A/p dstPort>P"
    put_str(s, name); put_str(s, " src>"); addr(); put_str(s, " dstPort>"); put_u64(s, dport);
  };
  switch (ev) {
    case 10: flow_first("ON"); break;
    case 11: server("ACCEPT"); break;
    case 13: flow_first("CONNECT"); break;
    case 12: if (fid) flow_dst("DISCONNECT"); else server("DISCONNECT"); break;
    case 16: if (fid) flow_dst("RECONNECT"); else server("RECONNECT"); break;
    case 15: if (fid) flow_dst("SHUTDOWN"); else server("SHUTDOWN"); break;
    case 14: if (fid) flow_first("OFF"); else server("OFF"); break;
    default: break;
  }
  if (hvalid) {
    put_str(s, "host>");
    put_addr(s, (uint8_t)ht, (uint8_t)hl, ha);
    s.put('/');
    put_u64(s, hport);
  }
  s.put('\n');
}

template <typename S>
__device__ void bl_line(S& s, const BinParams& p, uint32_t i) {
  const uint8_t* h = p.buf + p.rec_off[i];
  const uint8_t* b = h + 4;
  const uint32_t ev = h[0], rl = be16(h + 2);
  const bool epoch = (p.opts & MGENX_LOG_EPOCH) != 0;
  const mgenx_cols& c = p.cols;
  if (ev == 1 || ev == 3) {
    LogParams lp;
    lp.cols = c;
    LogRec r = gather(lp, i);
    if (r.err) {
      // a stored message Unpack rejects: the reference ignores Unpack's result and logs the
      // line from the members its fresh MgenMsg holds (:1601-1607, 1612-1625) -- the fresh
      // decode's defaults, and for RECV the event time it set as tx_time before Unpack
      if (ev == 1 && !(c.decoded[i] & MGENX_DEC_BASE)) {
        r.sec = p.ev_sec[i];
        r.usec = p.ev_usec[i];
      }
      r.err = 0;
    }
    if (ev == 1) {  // LogRecvEvent (:1607): log_flush lands in the ttl argument
      if (p.log_rx)
        format_line(s, r, p.buf + p.msg_off[i], p.src[i], p.ev_sec[i], p.ev_usec[i], p.proto[i],
                    (int)p.flush, p.opts);
      return;
    }
    // LogSendEvent text (:1211-1236) of the unpacked message; time = its tx_time
    const uint32_t proto = p.proto[i];
    put_ts(s, r.sec, r.usec, epoch);
    put_str(s, "SEND proto>");
    put_str(s, proto == 1 ? "UDP" : proto == 2 ? "TCP" : proto == 3 ? "SINK" : "UNKNOWN");
    put_str(s, " flow>"); put_u64(s, r.flow);
    put_str(s, " seq>"); put_u64(s, r.seq);
    put_str(s, " srcPort>0 dst>");  // a fresh MgenMsg's source
    put_addr(s, r.dtype, r.dlen, r.daddr);
    s.put('/'); put_u64(s, r.dport);
    put_str(s, " size>"); put_u64(s, proto == 2 ? p.aux[i] : r.msg_len); s.put(' ');
    if (r.htype == 1 || r.htype == 2) {
      put_str(s, "host>"); put_addr(s, r.htype, r.hlen, r.haddr); s.put('/'); put_u64(s, r.hport);
    }
    s.put('\n');
    return;
  }
  if (ev == 4 || ev == 5) {  // LISTEN / IGNORE (:1628-1656)
    put_ts(s, be32(b), be32(b + 4), epoch);
    put_str(s, ev == 4 ? "LISTEN proto>" : "IGNORE proto>");
    const uint32_t pr = b[8];
    put_str(s, pr == 1 ? "UDP" : pr == 2 ? "TCP" : pr == 3 ? "SINK" : "UNKNOWN");
    put_str(s, " port>"); put_u64(s, be16(b + 10)); s.put('\n');
  } else if (ev == 6 || ev == 7) {  // JOIN / LEAVE (:1657-1711)
    const uint32_t alen = b[11], gport = be16(b + 8), nl = b[12 + alen];
    put_ts(s, be32(b), be32(b + 4), epoch);
    put_str(s, ev == 6 ? "JOIN group>" : "LEAVE group>");
    put_addr(s, b[10], (uint8_t)alen, b + 12);
    if (nl) {
      put_str(s, " interface>");
      for (uint32_t k = 0; k < nl && b[13 + alen + k]; k++) s.put(b[13 + alen + k]);  // "%s"
    }
    if (gport) { put_str(s, " port>"); put_u64(s, gport); }
    s.put('\n');
  } else if (ev == 8 || ev == 9) {  // START / STOP (:1712-1729)
    put_ts(s, be32(b), be32(b + 4), epoch);
    put_str(s, ev == 8 ? "START\n" : "STOP\n");
  } else if (ev >= 10 && ev <= 16) {
    bl_conn_line(s, p, b, ev, rl);
  }
}

template <bool kWrite>
__global__ void __launch_bounds__(kLogThreads) binlog_line_kernel(BinParams p) {
  const uint32_t i = blockIdx.x * kLogThreads + threadIdx.x;
  if (i >= p.n) return;
  if (!kWrite) {
    // only RECV payloads are walked for REPORT items (LogRecvEvent, :1104-1137)
    if (p.kind[i] != 1) p.cols.payload_type[i] = 0xFF;
    CountSink s;
    bl_line(s, p, i);
    p.lens[i] = s.n;
  } else {
    const uint64_t off = p.line_off[i], end = p.line_off[i + 1];
    if (end > p.text_cap) return;
    WriteSink s{p.text + off};
    bl_line(s, p, i);
  }
}

}  // namespace mgenx

// per-stream scratch for the two-pass line formatters and the walk's scans
static int rep_ws(mgenx_log_ws& ws, size_t need, void** out, char* err, size_t errn) {
  if (ws.bytes < need) {
    mgenx::dev_free(ws.mem);
    ws.mem = nullptr;
    ws.bytes = 0;
    if (hipMalloc(&ws.mem, need) != hipSuccess) {
      snprintf(err, errn, "report: workspace of %zu bytes", need);
      return MGENX_EDEVICE;
    }
    ws.bytes = need;
  }
  *out = ws.mem;
  return MGENX_OK;
}

extern "C" int mgenx_report_build_run(const mgenx_flow_report* reps, uint32_t n_flows,
                                      uint32_t per_flow, const uint32_t* count,
                                      const mgenx_report_key* keys, uint8_t* sign,
                                      const double* offset, const double* rq, uint8_t* items,
                                      uint8_t* item_len, hipStream_t stream) {
  if (!n_flows || !per_flow) return MGENX_OK;
  hipLaunchKernelGGL(mgenx::report_build_kernel, dim3((n_flows + 127) / 128), dim3(128), 0, stream,
                     reps, n_flows, per_flow, count, keys, sign, offset, rq, items, item_len);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_report_lines_run(void* wsp, mgenx::RepLineParams* pp, hipStream_t stream,
                                      char* err, size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  mgenx::RepLineParams& p = *pp;
  const uint32_t n = p.n;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n + 1, stream);
  const size_t len_bytes = (((size_t)n + 1) * 8 + 255) & ~(size_t)255;
  void* mem;
  int rc = rep_ws(ws, len_bytes + scan_bytes, &mem, err, errn);
  if (rc != MGENX_OK) return rc;
  p.lens = static_cast<uint64_t*>(mem);
  const int grid = (int)((n + mgenx::kLogThreads - 1) / mgenx::kLogThreads);
  hipLaunchKernelGGL((mgenx::rep_line_kernel<false>), dim3(grid), dim3(mgenx::kLogThreads), 0,
                     stream, p);
  hipLaunchKernelGGL(mgenx::log_tail_kernel, dim3(1), dim3(64), 0, stream, p.lens, n);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(static_cast<uint8_t*>(mem) + len_bytes, have, p.lens,
                                       p.line_off, (int)n + 1, stream) != hipSuccess) {
    snprintf(err, errn, "report lines: scan failed");
    return MGENX_EDEVICE;
  }
  hipLaunchKernelGGL((mgenx::rep_line_kernel<true>), dim3(grid), dim3(mgenx::kLogThreads), 0,
                     stream, p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_data_walk_run(void* wsp, mgenx::WalkParams* pp, uint32_t* totals,
                                   hipStream_t stream, char* err, size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  mgenx::WalkParams& p = *pp;
  const uint32_t n = p.n;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr,
                                         (uint32_t*)nullptr, (int)n + 1, stream);
  const size_t b4 = (((size_t)n + 1) * 4 + 255) & ~(size_t)255;
  void* mem;
  int rc = rep_ws(ws, 4 * b4 + scan_bytes, &mem, err, errn);
  if (rc != MGENX_OK) return rc;
  char* m = static_cast<char*>(mem);
  p.n_cmd = reinterpret_cast<uint32_t*>(m);
  p.n_rep = reinterpret_cast<uint32_t*>(m + b4);
  uint32_t* cb = reinterpret_cast<uint32_t*>(m + 2 * b4);
  uint32_t* rb = reinterpret_cast<uint32_t*>(m + 3 * b4);
  p.cmd_base = cb;
  p.rep_base = rb;
  const dim3 g((n + 255) / 256);
  hipLaunchKernelGGL((mgenx::data_walk_kernel<false>), g, dim3(256), 0, stream, p);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(m + 4 * b4, have, p.n_cmd, cb, (int)n + 1, stream) !=
          hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(m + 4 * b4, have, p.n_rep, rb, (int)n + 1, stream) !=
          hipSuccess) {
    snprintf(err, errn, "data walk: scan failed");
    return MGENX_EDEVICE;
  }
  hipLaunchKernelGGL((mgenx::data_walk_kernel<true>), g, dim3(256), 0, stream, p);
  if (totals) {
    if (hipMemcpyAsync(totals, cb + n, 4, hipMemcpyDeviceToDevice, stream) != hipSuccess ||
        hipMemcpyAsync(totals + 1, rb + n, 4, hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return MGENX_EDEVICE;
  }
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_text_interleave_run(void* wsp, const mgenx_text_src* srcs, uint32_t n_src,
                                         uint32_t n_rec, char* out, uint64_t cap,
                                         uint64_t* rec_off, hipStream_t stream, char* err,
                                         size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  mgenx::TextParams p;
  memset(&p, 0, sizeof(p));
  for (uint32_t s = 0; s < n_src; s++) p.src[s] = srcs[s];
  p.n_src = n_src; p.n_rec = n_rec; p.out = reinterpret_cast<uint8_t*>(out); p.cap = cap;
  p.rec_off = rec_off;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n_rec + 1, stream);
  const size_t len_bytes = (((size_t)n_rec + 1) * 8 + 255) & ~(size_t)255;
  const size_t map_bytes = (((size_t)n_rec + 1) * 4 + 255) & ~(size_t)255;
  uint32_t n_scatter = 0;
  for (uint32_t s = 0; s < n_src; s++) n_scatter += srcs[s].kind == MGENX_TEXT_SCATTER;
  void* mem;
  int rc = rep_ws(ws, len_bytes + n_scatter * map_bytes + scan_bytes, &mem, err, errn);
  if (rc != MGENX_OK) return rc;
  p.lens = static_cast<uint64_t*>(mem);
  // scatter sources become record -> line maps in the workspace
  char* maps = static_cast<char*>(mem) + len_bytes;
  for (uint32_t s = 0; s < n_src; s++) {
    if (p.src[s].kind != MGENX_TEXT_SCATTER) continue;
    uint32_t* map = reinterpret_cast<uint32_t*>(maps);
    maps += map_bytes;
    if (hipMemsetAsync(map, 0xFF, (size_t)n_rec * 4 + 4, stream) != hipSuccess) {
      snprintf(err, errn, "text interleave: memset failed");
      return MGENX_EDEVICE;
    }
    if (p.src[s].n_lines)
      hipLaunchKernelGGL(mgenx::text_scatter_kernel, dim3((p.src[s].n_lines + 255) / 256),
                         dim3(256), 0, stream, p.src[s].index, p.src[s].n_lines, n_rec, map);
    p.src[s].index = map;
    p.src[s].kind = MGENX_TEXT_MAP;
  }
  hipLaunchKernelGGL(mgenx::text_len_kernel, dim3((n_rec + 1 + 255) / 256), dim3(256), 0, stream,
                     p);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(static_cast<uint8_t*>(mem) + len_bytes +
                                           n_scatter * map_bytes,
                                       have, p.lens, rec_off, (int)n_rec + 1,
                                       stream) != hipSuccess) {
    snprintf(err, errn, "text interleave: scan failed");
    return MGENX_EDEVICE;
  }
  if (n_rec)
    hipLaunchKernelGGL(mgenx::text_copy_kernel, dim3((n_rec + 3) / 4), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

static mgenx::BinParams bin_params(const uint8_t* buf, const uint64_t* rec_off, uint32_t n,
                                   uint64_t* msg_off, uint32_t* msg_len, mgenx_addr* src,
                                   uint32_t* ev_sec, uint32_t* ev_usec, uint32_t* aux,
                                   uint8_t* kind, uint8_t* proto) {
  mgenx::BinParams p;
  memset(&p, 0, sizeof(p));
  p.buf = buf; p.rec_off = rec_off; p.n = n; p.msg_off = msg_off; p.msg_len = msg_len;
  p.src = src; p.ev_sec = ev_sec; p.ev_usec = ev_usec; p.aux = aux; p.kind = kind;
  p.proto = proto;
  return p;
}

extern "C" int mgenx_binlog_parse_exec(const uint8_t* buf, const uint64_t* rec_off, uint32_t n,
                                       uint64_t* msg_off, uint32_t* msg_len, mgenx_addr* src,
                                       uint32_t* ev_sec, uint32_t* ev_usec, uint32_t* aux,
                                       uint8_t* kind, uint8_t* proto, hipStream_t stream) {
  mgenx::BinParams p = bin_params(buf, rec_off, n, msg_off, msg_len, src, ev_sec, ev_usec, aux,
                                  kind, proto);
  if (p.n)
    hipLaunchKernelGGL(mgenx::binlog_parse_kernel, dim3((p.n + 255) / 256), dim3(256), 0, stream,
                       p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_binlog_lines_exec(void* wsp, const uint8_t* buf, const uint64_t* rec_off,
                                       uint32_t n, uint64_t* msg_off, uint32_t* msg_len,
                                       mgenx_addr* src, uint32_t* ev_sec, uint32_t* ev_usec,
                                       uint32_t* aux, uint8_t* kind, uint8_t* proto,
                                       const mgenx_cols* cols, uint32_t log_rx, uint32_t flush,
                                       uint32_t opts, char* text, uint64_t cap,
                                       uint64_t* line_off, hipStream_t stream, char* err,
                                       size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  mgenx::BinParams p = bin_params(buf, rec_off, n, msg_off, msg_len, src, ev_sec, ev_usec, aux,
                                  kind, proto);
  p.cols = *cols;
  p.log_rx = log_rx; p.flush = flush; p.opts = opts;
  p.text = reinterpret_cast<uint8_t*>(text); p.text_cap = cap; p.line_off = line_off;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n + 1, stream);
  const size_t len_bytes = (((size_t)n + 1) * 8 + 255) & ~(size_t)255;
  void* mem;
  int rc = rep_ws(ws, len_bytes + scan_bytes, &mem, err, errn);
  if (rc != MGENX_OK) return rc;
  p.lens = static_cast<uint64_t*>(mem);
  const int grid = (int)((n + mgenx::kLogThreads - 1) / mgenx::kLogThreads);
  if (n)
    hipLaunchKernelGGL((mgenx::binlog_line_kernel<false>), dim3(grid), dim3(mgenx::kLogThreads),
                       0, stream, p);
  hipLaunchKernelGGL(mgenx::log_tail_kernel, dim3(1), dim3(64), 0, stream, p.lens, n);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(static_cast<uint8_t*>(mem) + len_bytes, have, p.lens,
                                       p.line_off, (int)n + 1, stream) != hipSuccess) {
    snprintf(err, errn, "binlog: scan failed");
    return MGENX_EDEVICE;
  }
  if (n)
    hipLaunchKernelGGL((mgenx::binlog_line_kernel<true>), dim3(grid), dim3(mgenx::kLogThreads),
                       0, stream, p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_report_lines(void* ws, const uint8_t* items, const mgenx_flow_report* reps,
                                  const uint32_t* count, uint32_t per_flow, const uint64_t* pairs,
                                  const uint8_t* slab, const mgenx_addr* reporter,
                                  const uint32_t* rx_sec, const uint32_t* rx_usec, uint32_t n,
                                  uint32_t opts, const double* rq, char* text, uint64_t cap,
                                  uint64_t* line_off, hipStream_t stream, char* err, size_t errn) {
  mgenx::RepLineParams p;
  p.items = items; p.reps = reps; p.count = count; p.per_flow = per_flow; p.rep_pairs = pairs;
  p.slab = slab; p.reporter = reporter; p.rx_sec = rx_sec; p.rx_usec = rx_usec; p.n = n;
  p.opts = opts; p.rq = rq; p.text = reinterpret_cast<uint8_t*>(text); p.text_cap = cap;
  p.line_off = line_off; p.lens = nullptr;
  return mgenx_report_lines_run(ws, &p, stream, err, errn);
}

extern "C" int mgenx_data_walk_exec(void* ws, const uint8_t* slab, const uint64_t* rec_off,
                                    uint64_t stride, const mgenx_cols* cols, uint32_t n,
                                    uint32_t opts, const double* rq, uint8_t* status,
                                    uint8_t* needs_host, uint32_t* cmds, uint32_t cmd_cap,
                                    uint64_t* reps, uint32_t rep_cap, uint32_t* totals,
                                    hipStream_t stream, char* err, size_t errn) {
  mgenx::WalkParams p;
  p.slab = slab; p.rec_off = rec_off; p.stride = stride; p.cols = *cols; p.n = n; p.opts = opts;
  p.rq = rq; p.status = status; p.needs_host = needs_host; p.cmds = cmds; p.cmd_cap = cmd_cap;
  p.reps = reps; p.rep_cap = rep_cap;
  return mgenx_data_walk_run(ws, &p, totals, stream, err, errn);
}

// ---------------------------------------------------------------------------------------
// SEND events: MgenMsg::LogSendEvent (mgenMsg.cpp:1145-1241) of the records a send path
// packed (mgenTransport.cpp:1060: after a successful send, theTime = the tx time; the
// message's src port = the flow transport's port, mgenFlow.cpp:975-977).  One lane per
// record, a length pass, a scan, a write pass.
namespace mgenx {

struct SendParams {
  const mgenx_flow_tmpl* tmpl;
  const mgenx_pack_desc* desc;
  const uint16_t* src_port;   // per template
  const uint32_t* out_len;    // per record: Pack's return (0 = not sent: no event); NULL = all
  const uint32_t* msg_total;  // TCP: mgen_msg_len per record (NULL = msg_len)
  const uint8_t* slab;        // binary: the packed records
  uint64_t slab_bytes;
  const uint64_t* rec_off;
  uint64_t stride;
  uint32_t n;
  int protocol;
  uint32_t opts;
  bool binary;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* pos;
  uint64_t* lens;
};

__device__ __forceinline__ uint32_t addr_length(uint32_t type) {
  return type == 1u ? 4u : (type == 2u ? 16u : 0u);  // ProtoAddress::GetLength()
}

// packet_header_len after Pack(bufferLen = msgLen) (mgenMsg.cpp:97-273, as pack_kernel)
__device__ uint32_t pack_hdr_len(const mgenx_flow_tmpl& t, uint32_t msgLen) {
  const uint32_t D = t.dst_len > 16u ? 16u : t.dst_len;
  const bool hv = t.host_type == 1u || t.host_type == 2u;
  const uint32_t H = hv ? (t.host_len > 16u ? 16u : t.host_len) : 0u;
  uint32_t len = 24u + D;
  if (msgLen < len + H + 4u) return len;
  len += 4u + H;
  if (msgLen < len + 13u) return len;
  len += 13u;
  if (msgLen < len + 1u) return len;
  len += 1u;
  if (msgLen < len + 2u) return len;
  return len + 2u;
}

template <typename S>
__device__ void send_event(S& s, const SendParams& p, uint32_t i) {
  if (p.out_len && p.out_len[i] == 0) return;  // Pack failed: never sent, never logged
  const mgenx_pack_desc d = p.desc[i];
  const mgenx_flow_tmpl& t = p.tmpl[d.tmpl];
  const bool tcp = p.protocol == MGENX_PROTO_TCP;
  const uint32_t mml = (tcp && p.msg_total) ? p.msg_total[i] : d.msg_len;
  const bool hv = t.host_type == 1u || t.host_type == 2u;
  if (!p.binary) {
    put_ts(s, d.tx_sec, d.tx_usec, (p.opts & MGENX_LOG_EPOCH) != 0);
    put_str(s, "SEND proto>");
    put_str(s, p.protocol == 1 ? "UDP" : p.protocol == 2 ? "TCP" : p.protocol == 3 ? "SINK" : "UNKNOWN");
    put_str(s, " flow>");
    put_u64(s, t.flow_id);
    put_str(s, " seq>");
    put_u64(s, d.seq_num);
    put_str(s, " srcPort>");
    put_u64(s, p.src_port[d.tmpl]);
    put_str(s, " dst>");
    put_addr(s, t.dst_type, t.dst_len, t.dst_addr);
    s.put('/');
    put_u64(s, t.dst_port);
    put_str(s, " size>");
    put_u64(s, tcp ? mml : (uint32_t)d.msg_len);
    s.put(' ');
    if (hv) {
      put_str(s, "host>");
      put_addr(s, t.host_type, t.host_len, t.host_addr);
      s.put('/');
      put_u64(s, t.host_port);
    }
    s.put('\n');
    return;
  }
  // binary: {SEND_EVENT, protocol, BE recordLength [, BE mgen_msg_len]} + message bytes
  uint32_t rl = 12u + addr_length(t.dst_type) + pack_hdr_len(t, d.msg_len);
  if (hv) rl += addr_length(t.host_type) + 4u;
  if (tcp) rl += 4u;
  rl &= 0xFFFFu;
  s.put(3);
  s.put((uint8_t)p.protocol);
  s.put((uint8_t)(rl >> 8));
  s.put((uint8_t)rl);
  uint32_t index = 4;
  if (tcp) {
    s.put((uint8_t)(mml >> 24)); s.put((uint8_t)(mml >> 16));
    s.put((uint8_t)(mml >> 8)); s.put((uint8_t)mml);
    index += 4;
  }
  const uint32_t ml = (rl - index + 4u) & 0xFFFFu;
  const uint64_t off = p.rec_off ? p.rec_off[i] : (uint64_t)i * p.stride;
  const uint64_t have = p.out_len ? p.out_len[i] : d.msg_len;
  for (uint32_t k = 0; k < ml; k++) {
    uint8_t b = (k < have && off + k < p.slab_bytes) ? p.slab[off + k] : (uint8_t)0;
    if (k == 3) b &= (uint8_t)~MGENX_FLAG_CHECKSUM;  // "Clear CHECKSUM flag for binary logging"
    s.put(b);
  }
}

template <bool kWrite>
__global__ void __launch_bounds__(kLogThreads) send_kernel(SendParams p) {
  const uint32_t i = blockIdx.x * kLogThreads + threadIdx.x;
  if (i >= p.n) return;
  if (!kWrite) {
    CountSink s;
    send_event(s, p, i);
    p.lens[i] = s.n;
  } else {
    const uint64_t off = p.pos[i], end = p.pos[i + 1];
    if (end > p.out_cap) return;
    WriteSink s{p.out + off};
    send_event(s, p, i);
  }
}

}  // namespace mgenx

extern "C" int mgenx_log_send_exec(void* wsp, const mgenx_flow_tmpl* tmpl,
                                   const mgenx_pack_desc* desc, const uint16_t* src_port,
                                   const uint32_t* out_len, const uint32_t* msg_total,
                                   const uint8_t* slab, uint64_t slab_bytes,
                                   const uint64_t* rec_off, uint64_t stride, uint32_t n,
                                   int protocol, uint32_t opts, bool binary, uint8_t* out,
                                   uint64_t out_cap, uint64_t* pos, hipStream_t stream,
                                   char* err, size_t errn) {
  mgenx_log_ws& ws = ws_for(wsp, stream);
  mgenx::SendParams p;
  p.tmpl = tmpl; p.desc = desc; p.src_port = src_port; p.out_len = out_len;
  p.msg_total = msg_total; p.slab = slab; p.slab_bytes = slab_bytes; p.rec_off = rec_off;
  p.stride = stride; p.n = n; p.protocol = protocol; p.opts = opts; p.binary = binary;
  p.out = out; p.out_cap = out_cap; p.pos = pos;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n + 1, stream);
  const size_t len_bytes = (((size_t)n + 1) * 8 + 255) & ~(size_t)255;
  void* mem;
  int rc = rep_ws(ws, len_bytes + scan_bytes, &mem, err, errn);
  if (rc != MGENX_OK) return rc;
  p.lens = static_cast<uint64_t*>(mem);
  const int grid = (int)((n + mgenx::kLogThreads - 1) / mgenx::kLogThreads);
  hipLaunchKernelGGL(mgenx::send_kernel<false>, dim3(grid), dim3(mgenx::kLogThreads), 0, stream, p);
  hipLaunchKernelGGL(mgenx::log_tail_kernel, dim3(1), dim3(64), 0, stream, p.lens, n);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(static_cast<uint8_t*>(mem) + len_bytes, have, p.lens,
                                       pos, (int)n + 1, stream) != hipSuccess) {
    snprintf(err, errn, "send log: scan failed");
    return MGENX_EDEVICE;
  }
  hipLaunchKernelGGL(mgenx::send_kernel<true>, dim3(grid), dim3(mgenx::kLogThreads), 0, stream, p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}
