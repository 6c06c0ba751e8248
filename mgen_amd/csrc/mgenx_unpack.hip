// mgenx_unpack.hip -- batched MgenMsg::Unpack + receive-side CRC-32 check on gfx950.
//
// Reference semantics: MgenMsg::Unpack (src/common/mgenMsg.cpp:315-500) on a fresh
// MgenMsg, followed by the receive CRC check of the UDP / SINK / TCP callers
// (src/common/mgenTransport.cpp:958-975, 2092-2112, 1516-1564).
//
// Work mapping (one persistent 1024-thread workgroup per CU):
//   * a quad of 4 lanes owns one record; a wave owns 16 consecutive records;
//   * the record is covered by 64-byte rows aligned to the record END, so a quad's four
//     16-byte loads per row are one contiguous (unaligned) 64-byte span: coalesced, and
//     the CRC trailer always lands in word 3 of lane 3 of the last row;
//   * CRC: residue check.  The stream Y = [zero pad][payload bytes][LE(trailer)] is
//     reduced with zero initial state; the record is intact iff crc_raw(Y) equals
//     expect[L] = A_4(A_{L-4}(~0) ^ ~0) (init handled by linearity, no per-byte masking).
//     Each lane keeps 4 independent "braid" states (one per word of its 16-byte unit),
//     advanced row to row by the 64-byte shift operator A_64 -- one conflict-free LDS
//     table lookup per input byte (the A_64 tables are replicated 32x so lane l always
//     reads bank l).  The last row folds the braids with A_4 and the quad folds its four
//     lanes with A_16 / A_32 (shuffles);
//   * lane 0 of the quad decodes the header fields and writes the SoA columns.
#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr int kUnpackThreads = 1024;
constexpr int kRep = 32;                       // A_64 replicas (one per LDS bank)
constexpr int kRepDwords = 4 * 256 * kRep;     // 32768 dwords = 128 KiB
constexpr int kSmallTabDwords = 1024;          // one shift operator: 4 x 256 dwords
constexpr size_t kUnpackLdsBytes = (size_t)(kRepDwords + 3 * kSmallTabDwords) * 4u;


// A_64(x) from the replicated tables: layout [(k*256 + v) * 32 + copy], copy = lane & 31.
__device__ __forceinline__ uint32_t shift_rep(const uint32_t* rep, uint32_t x, uint32_t copy) {
  const uint32_t i0 = ((x & 0xffu) << 5) | copy;
  const uint32_t i1 = (((x >> 8) & 0xffu) << 5) | copy;
  const uint32_t i2 = (((x >> 16) & 0xffu) << 5) | copy;
  const uint32_t i3 = ((x >> 24) << 5) | copy;
  return rep[i0] ^ rep[8192 + i1] ^ rep[16384 + i2] ^ rep[24576 + i3];
}

__device__ __forceinline__ uint32_t shift_tab(const uint32_t* t, uint32_t x) {
  return t[x & 0xffu] ^ t[256 + ((x >> 8) & 0xffu)] ^ t[512 + ((x >> 16) & 0xffu)] ^
         t[768 + (x >> 24)];
}

// 128-bit little-endian left shift by s bytes (0 < s < 16), zero fill.
__device__ __forceinline__ u32x4_t shl_bytes(u32x4_t v, int s) {
  const int a = s >> 2;
  const int c = (s & 3) * 8;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int hi_i = i - a, lo_i = i - a - 1;
    uint32_t hi = 0, lo = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      hi = (k == hi_i) ? w[k] : hi;
      lo = (k == lo_i) ? w[k] : lo;
    }
    o[i] = c ? ((hi << c) | (lo >> (32 - c))) : hi;
  }
  return u32x4_t{o[0], o[1], o[2], o[3]};
}

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
  bool ok;
};

// MgenMsg::Unpack on a fresh MgenMsg (mgenMsg.cpp:315-500); buf_len = bufferLen.
__device__ void parse_header(const uint8_t* r, uint32_t buf_len, bool want_ext, Hdr& h) {
  h.flow = h.seq = h.sec = h.usec = h.dst4 = h.poff = 0;
  h.lat = h.lon = 10800000u;  // (0.0 + 180) * 60000: the constructor's 0.0 degrees
  h.alt = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) h.dst_addr[j] = h.host_addr[j] = 0;
  h.msg_len = h.dst_port = h.plen = h.hdr_len = h.host_port = 0;
  h.version = 2;
  h.flags = h.err = h.dst_type = h.dst_len = h.ptype = h.gps = h.host_type = h.host_len = 0;
  h.ok = false;
  if (buf_len < MGENX_MIN_SIZE) { h.err = MGENX_ERROR_LENGTH; return; }      // :323-328
  const u32x4_t a = ldu128(r);
  const uint32_t w4 = ldu32(r + 16), w5 = ldu32(r + 20);
  h.msg_len = bswap16((uint16_t)(a.x & 0xffffu));
  h.version = (uint8_t)(a.x >> 16);
  if (h.version != 2) { h.err = MGENX_ERROR_VERSION; return; }              // :336-343
  h.flags = (uint8_t)(a.x >> 24);
  h.flow = bswap32(a.y);
  h.seq = bswap32(a.z);
  h.sec = bswap32(a.w);
  h.usec = bswap32(w4);
  const uint16_t dport = bswap16((uint16_t)(w5 & 0xffffu));
  const uint32_t t = (w5 >> 16) & 0xffu;
  const uint32_t D = w5 >> 24;
  if (t != 1u && t != 2u) { h.err = MGENX_ERROR_DSTADDR; return; }          // :374-392
  h.dst_type = (uint8_t)t;
  h.dst_len = (uint8_t)D;
  h.dst_port = dport;
  {
    // :394-398 has no bounds check; bytes past the record read as zero here.
    uint32_t d[4];
    if (want_ext) {
      load_addr16(r + 24, D, buf_len - 24, d);
#pragma unroll
      for (int j = 0; j < 4; j++) h.dst_addr[j] = d[j];
      h.dst4 = d[0];
    } else {
      const uint32_t w6 = ldu32(r + 24);   // 24 + 4 <= 28 <= buf_len
      h.dst4 = D >= 4 ? w6 : (w6 & byte_range_mask(0, (int)D));
    }
  }
  uint32_t len = 24u + D;
  if (len + 4u <= buf_len) {                                                  // :400-443
    const uint32_t hw = ldu32(r + len);
    const uint16_t hport = bswap16((uint16_t)(hw & 0xffffu));
    const uint32_t ht = (hw >> 16) & 0xffu;
    const uint32_t H = hw >> 24;
    len += 4u;
    if (len + H <= buf_len) {
      if (ht == 1u || ht == 2u) {
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
  if (len + 13u <= buf_len) {                                                 // :446-465
    h.lat = bswap32(ldu32(r + len));
    h.lon = bswap32(ldu32(r + len + 4));
    h.alt = (int32_t)bswap32(ldu32(r + len + 8));
    h.gps = r[len + 12];
    len += 13u;
  } else {
    h.hdr_len = (uint16_t)len; h.ok = true; return;
  }
  if (len + 1u <= buf_len) {                                                  // :467-475
    h.ptype = r[len];
    len += 1u;
  } else {
    h.hdr_len = (uint16_t)len; h.ok = true; return;
  }
  if (len + 2u <= buf_len) {                                                  // :477-497
    h.plen = bswap16(ldu16(r + len));
    len += 2u;
    h.hdr_len = (uint16_t)len;
    if (h.plen != 0 && len + h.plen <= buf_len) h.poff = (len >> 2) << 2;
    else h.plen = 0;
  }
  h.ok = true;
}

// CRC-32 (init/xorout ~0) computed bit by bit: used only for records shorter than 32 B.
__device__ bool small_crc_ok(const uint8_t* r, uint32_t L) {
  if (L < 4) return false;
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t i = 0; i < L - 4; i++) {
    c ^= r[i];
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
  }
  c ^= 0xFFFFFFFFu;
  const uint32_t t = ((uint32_t)r[L - 4] << 24) | ((uint32_t)r[L - 3] << 16) |
                     ((uint32_t)r[L - 2] << 8) | r[L - 1];
  return c == t;
}

__global__ void __launch_bounds__(kUnpackThreads)
unpack_kernel(UnpackParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* rep = lds;
  uint32_t* a4 = lds + kRepDwords;
  uint32_t* a16 = a4 + kSmallTabDwords;
  uint32_t* a32 = a16 + kSmallTabDwords;

  // ---- stage the shift-operator tables (A_64 replicated 32x) ----
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const uint32_t v = p.tabs[e];
    u32x4_t s = {v, v, v, v};
    u32x4_t* dst = reinterpret_cast<u32x4_t*>(rep + (size_t)e * kRep);
#pragma unroll
    for (int c = 0; c < kRep / 4; c++) dst[c] = s;
  }
  for (int e = threadIdx.x; e < 3 * 1024; e += blockDim.x) a4[e] = p.tabs[1024 + e];
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const uint32_t copy = (uint32_t)(lane & 31);
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint64_t wave_id = (uint64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
  const uint64_t n_waves = (uint64_t)gridDim.x * waves_per_block;
  const uint64_t n_groups = ((uint64_t)p.n + 15) >> 4;
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const bool skip_crc = (p.opts & MGENX_OPT_SKIP_CRC) != 0;
  const bool want_ext = p.cols.dst_addr || p.cols.host_addr;

  for (uint64_t g = wave_id; g < n_groups; g += n_waves) {
    const uint64_t rec_idx = (g << 4) + (uint64_t)(lane >> 2);
    const bool valid = rec_idx < p.n;
    uint64_t off = 0;
    uint32_t L = 0;
    if (valid) {
      off = p.rec_off ? p.rec_off[rec_idx] : rec_idx * p.stride;
      L = p.rec_len ? p.rec_len[rec_idx] : p.fixed_len;
    }
    const bool oob = valid && (L > 65535u || off > p.slab_bytes || L > p.slab_bytes - off);
    const bool live = valid && !oob;
    const uint8_t* rec = p.slab + off;

    // ---- header decode (quad lane 0) ----
    Hdr h;
    bool needs_crc = false;
    if (live && q == 0) {
      const uint32_t buf_len = tcp ? min(L, (uint32_t)MGENX_TX_BUFFER_SIZE) : L;
      parse_header(rec, buf_len, want_ext, h);
      const bool flagged = force || (h.flags & MGENX_FLAG_CHECKSUM);
      needs_crc = !skip_crc && flagged && (tcp ? (L >= 4) : h.ok);
    }
    needs_crc = __shfl(needs_crc, lane & ~3);

    // ---- CRC residue over end-aligned 64-byte rows (quads with L >= 32) ----
    const bool vec = needs_crc && L >= 32;
    const int R = vec ? (int)((L + 63u) >> 6) : 0;
    const int64_t row0 = (int64_t)L - 64 * (int64_t)R + 16 * q;  // position of row 0 unit
    u32x4_t w = {0u, 0u, 0u, 0u};
    if (vec) {
      if (row0 >= 0) {
        w = ldu128(rec + row0);
      } else if (row0 > -16) {
        w = shl_bytes(ldu128(rec), (int)(-row0));
      }
    }
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    int r = 0;
    while (__any(vec && r < R - 1)) {
      const bool g1 = vec && r + 1 < R, g2 = vec && r + 2 < R;
      const bool g3 = vec && r + 3 < R, g4 = vec && r + 4 < R;
      const int64_t b = row0 + 64 * (int64_t)r;
      u32x4_t d1 = w, d2 = w, d3 = w, d4 = w;
      if (g1) d1 = ldu128(rec + b + 64);
      if (g2) d2 = ldu128(rec + b + 128);
      if (g3) d3 = ldu128(rec + b + 192);
      if (g4) d4 = ldu128(rec + b + 256);
#define MGENX_ROW_STEP(DN, GN)                                   \
      if (GN) {                                                  \
        h0 = shift_rep(rep, h0 ^ w.x, copy);                     \
        h1 = shift_rep(rep, h1 ^ w.y, copy);                     \
        h2 = shift_rep(rep, h2 ^ w.z, copy);                     \
        h3 = shift_rep(rep, h3 ^ w.w, copy);                     \
        w = DN;                                                  \
        r++;                                                     \
      }
      MGENX_ROW_STEP(d1, g1)
      MGENX_ROW_STEP(d2, g2)
      MGENX_ROW_STEP(d3, g3)
      MGENX_ROW_STEP(d4, g4)
#undef MGENX_ROW_STEP
    }
    // last row: byte-swap the big-endian trailer into little-endian stream order
    if (q == 3) w.w = bswap32(w.w);
    uint32_t v = shift_tab(a4, h0 ^ w.x);
    v = shift_tab(a4, v ^ h1 ^ w.y);
    v = shift_tab(a4, v ^ h2 ^ w.z);
    v = shift_tab(a4, v ^ h3 ^ w.w);
    const uint32_t t = shift_tab(a16, v) ^ __shfl_down(v, 1);
    const uint32_t tot = shift_tab(a32, t) ^ __shfl_down(t, 2);

    if (live && q == 0) {
      bool crc_ok = true;
      if (needs_crc) crc_ok = vec ? (tot == p.expect[L]) : small_crc_ok(rec, L);
      uint8_t err = h.err;
      uint8_t flags = h.flags;
      if (!crc_ok) {
        err = MGENX_ERROR_CHECKSUM;
        if (tcp) flags |= MGENX_FLAG_CHECKSUM_ERROR;
      }
      const mgenx_cols& c = p.cols;
      c.flow_id[rec_idx] = h.flow;
      c.seq_num[rec_idx] = h.seq;
      c.tx_sec[rec_idx] = h.sec;
      c.tx_usec[rec_idx] = h.usec;
      c.msg_len[rec_idx] = h.msg_len;
      c.dst_port[rec_idx] = h.dst_port;
      c.flags[rec_idx] = flags;
      c.err[rec_idx] = err;
      c.dst_type[rec_idx] = h.dst_type;
      c.dst_len[rec_idx] = h.dst_len;
      c.dst_addr4[rec_idx] = h.dst4;
      c.payload_len[rec_idx] = h.plen;
      c.payload_type[rec_idx] = h.ptype;
      c.gps_status[rec_idx] = h.gps;
      if (c.hdr_len) c.hdr_len[rec_idx] = h.hdr_len;
      if (c.payload_off) c.payload_off[rec_idx] = h.poff;
      if (c.host_port) c.host_port[rec_idx] = h.host_port;
      if (c.host_type) c.host_type[rec_idx] = h.host_type;
      if (c.host_len) c.host_len[rec_idx] = h.host_len;
      if (c.lat_raw) c.lat_raw[rec_idx] = h.lat;
      if (c.lon_raw) c.lon_raw[rec_idx] = h.lon;
      if (c.alt) c.alt[rec_idx] = h.alt;
      if (c.host_addr) {
        u32x4_t* hp = reinterpret_cast<u32x4_t*>(c.host_addr + rec_idx * 16);
        *hp = u32x4_t{h.host_addr[0], h.host_addr[1], h.host_addr[2], h.host_addr[3]};
      }
      if (c.dst_addr) {
        u32x4_t* dp = reinterpret_cast<u32x4_t*>(c.dst_addr + rec_idx * 16);
        *dp = u32x4_t{h.dst_addr[0], h.dst_addr[1], h.dst_addr[2], h.dst_addr[3]};
      }
    } else if (oob && q == 0) {
      p.cols.err[rec_idx] = MGENX_ERROR_OOB;
      p.cols.flags[rec_idx] = 0;
      p.cols.msg_len[rec_idx] = 0;
      p.cols.flow_id[rec_idx] = 0;
      p.cols.seq_num[rec_idx] = 0;
      p.cols.tx_sec[rec_idx] = 0;
      p.cols.tx_usec[rec_idx] = 0;
      p.cols.dst_port[rec_idx] = 0;
      p.cols.dst_type[rec_idx] = 0;
      p.cols.dst_len[rec_idx] = 0;
      p.cols.dst_addr4[rec_idx] = 0;
      p.cols.payload_len[rec_idx] = 0;
      p.cols.payload_type[rec_idx] = 0;
      p.cols.gps_status[rec_idx] = 0;
    }
  }
}

hipError_t launch_unpack(const UnpackParams& p, int grid, hipStream_t stream) {
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)unpack_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kUnpackLdsBytes);
    if (e != hipSuccess) return e;
    attr_done = true;
  }
  hipLaunchKernelGGL(unpack_kernel, dim3(grid), dim3(kUnpackThreads), kUnpackLdsBytes, stream,
                     p);
  return hipGetLastError();
}

}  // namespace mgenx
