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
#include <type_traits>

#include "mgenx_kernels.hpp"
#include "mgenx_parse.hpp"

namespace mgenx {

constexpr int kUnpackThreads = 1024;
constexpr int kRep = 32;                       // A_64 replicas (one per LDS bank)
constexpr int kRepDwords = 4 * 256 * kRep;     // 32768 dwords = 128 KiB
constexpr int kSmallTabDwords = 1024;          // one shift operator: 4 x 256 dwords
// fold operators A_4, A_8, A_12, A_16, A_32, A_48 (not replicated)
constexpr int kFoldTabs = 6;
constexpr size_t kUnpackLdsBytes = (size_t)(kRepDwords + kFoldTabs * kSmallTabDwords) * 4u;


// Replicated A_64 tables.  Entry (k, v, copy) -- table k (byte k of the state), byte value v,
// replica copy = lane & 31 -- sits at LDS byte address
//     (k >> 1) * 65536 + v * 256 + (k & 1) * 128 + copy * 4,
// so lane l always reads bank l (conflict-free ds_read_b32), and ONE v_perm_b32 forms each
// address from the state word: byte 1 <- byte k of the state, byte 0 <- copy * 4 and
// byte 2 <- k >> 1 (both from the lane constant s1 = copy * 4 | 1 << 16); (k & 1) * 128 is
// the ds_read immediate.  That is one VALU op per lookup, plus one v_bitop3 (XOR3) per
// three lookups to combine them.
__device__ __forceinline__ uint32_t a64_s1(uint32_t lane) { return ((lane & 31u) << 2) | (1u << 16); }

// The tables are addressed by absolute LDS address: these kernels have no static LDS, so the
// dynamic allocation starts at 0.  (Going through the extern array pointer would cost one
// v_add of its link-time base, 0, per lookup.)
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_u32(const uint8_t*, uint32_t addr, uint32_t imm) {
  return *(const lds_u32_t*)(addr + imm);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// A_64(c) as two partial words (A_64(c) = ha ^ hb), so the caller folds them together with
// the next row's data in one XOR3.
__device__ __forceinline__ void a64_parts(const uint8_t* ldsb, uint32_t c, uint32_t s1,
                                          uint32_t& ha, uint32_t& hb) {
  const uint32_t t0 = lds_u32(ldsb, __builtin_amdgcn_perm(c, s1, 0x0c0c0400u), 0);
  const uint32_t t1 = lds_u32(ldsb, __builtin_amdgcn_perm(c, s1, 0x0c0c0500u), 128);
  const uint32_t t2 = lds_u32(ldsb, __builtin_amdgcn_perm(c, s1, 0x0c020600u), 0);
  const uint32_t t3 = lds_u32(ldsb, __builtin_amdgcn_perm(c, s1, 0x0c020700u), 128);
  ha = xor3(t0, t1, t2);
  hb = t3;
}

// Stage the replicated A_64 tables (tabs[0..1023] = table k entry v at k * 256 + v) and the
// fold tables (tabs[1024..]) into LDS, in two halves so a caller can put other loads in
// flight between them: table_loads() reads this thread's entries (1024-thread blocks:
// one A_64 entry and six fold entries), table_writes() stores them.  Caller synchronises.
struct TableRegs {
  uint32_t a64, fold[kFoldTabs];
};
__device__ __forceinline__ TableRegs table_loads(const uint32_t* tabs) {
  TableRegs r;
  r.a64 = tabs[threadIdx.x];
#pragma unroll
  for (int k = 0; k < kFoldTabs; k++) r.fold[k] = tabs[1024 + k * 1024 + threadIdx.x];
  return r;
}
__device__ __forceinline__ void table_writes(uint32_t* lds, const TableRegs& r) {
  typedef __attribute__((address_space(3))) u32x4_t lds_u32x4_t;
  const uint32_t e = threadIdx.x;
  const uint32_t k = e >> 8, val = e & 255u;
  const u32x4_t s = {r.a64, r.a64, r.a64, r.a64};
  lds_u32x4_t* dst = (lds_u32x4_t*)((k >> 1) * 65536u + val * 256u + (k & 1u) * 128u);
#pragma unroll
  for (int c = 0; c < kRep / 4; c++) dst[c] = s;
  uint32_t* fold = lds + kRepDwords;
#pragma unroll
  for (int k2 = 0; k2 < kFoldTabs; k2++) fold[k2 * 1024 + e] = r.fold[k2];
}
__device__ __forceinline__ void stage_tables(uint32_t* lds, const uint32_t* tabs) {
  table_writes(lds, table_loads(tabs));
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

// load_addr16, Hdr, load_fixed, fixed_ok, parse_header: mgenx_parse.hpp (shared with the
// resident single-message worker, mgenx_worker.hip)

// Layouts the register-only parse handles (given the first 64 bytes pw[0..15] of a record
// with buf_len >= 64): version 2, dst type IPv4/IPv6, dst and host address lengths in
// {0,4,16} (every later field is then word-aligned) and header <= 64 bytes (so not IPv6
// dst + IPv6 host).  Field meaning follows mgenMsg.cpp:323-497 as in parse_header.
__device__ __forceinline__ bool fast_layout(uint32_t w0, uint32_t w5, uint32_t hw) {
  const uint32_t t = (w5 >> 16) & 0xffu;
  const uint32_t D = w5 >> 24;
  const uint32_t H = hw >> 24;
  return ((w0 >> 16) & 0xffu) == 2u && (t == 1u || t == 2u) && (D == 4u || D == 16u) &&
         (H == 0u || H == 4u || H == 16u) && D + H <= 20u;
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

// Word k (0..15) of the quad's 64-byte header prefix, read from quad lane k/4's chunk by
// DPP at the point of use (k is a constant after inlining, so the switch folds away).
// All four lanes of the quad must be active.
__device__ __forceinline__ uint32_t prefix_word(const u32x4_t& pf, int k) {
#define MGENX_PW(K, C, LN) \
  case K: return (uint32_t)__builtin_amdgcn_mov_dpp((int)pf.C, LN * 0x55, 0xf, 0xf, false);
  switch (k) {
    MGENX_PW(0, x, 0) MGENX_PW(1, y, 0) MGENX_PW(2, z, 0) MGENX_PW(3, w, 0)
    MGENX_PW(4, x, 1) MGENX_PW(5, y, 1) MGENX_PW(6, z, 1) MGENX_PW(7, w, 1)
    MGENX_PW(8, x, 2) MGENX_PW(9, y, 2) MGENX_PW(10, z, 2) MGENX_PW(11, w, 2)
    MGENX_PW(12, x, 3) MGENX_PW(13, y, 3) MGENX_PW(14, z, 3) MGENX_PW(15, w, 3)
    default: return 0u;
  }
#undef MGENX_PW
}

// ---- column stores (quad lane 0 of the record) ----

// The caller's receive check: a CRC mismatch becomes ERROR_CHECKSUM, plus the
// CHECKSUM_ERROR flag on TCP (mgenTransport.cpp:971-975, 1552-1560).
__device__ __forceinline__ void crc_verdict(bool crc_ok, bool tcp, uint8_t& err,
                                            uint8_t& flags) {
  if (!crc_ok) {
    err = MGENX_ERROR_CHECKSUM;
    if (tcp) flags |= MGENX_FLAG_CHECKSUM_ERROR;
  }
}

// Extended columns of a fast-layout record: every word is read with all lanes active (the
// DPP reads cross the quad), then only `do_store` lanes (quad lane 0) store.
template <typename PW>
__device__ __forceinline__ void store_fast_ext(const mgenx_cols& c, uint64_t i, const PW& pw,
                                               uint32_t buf_len, bool do_store) {
  uint32_t wd[16];
#pragma unroll
  for (int k = 0; k < 16; k++) wd[k] = pw(k);
  const uint32_t D = wd[5] >> 24;
  const uint32_t hw = (D == 4u) ? wd[7] : wd[10];
  const uint32_t H = hw >> 24;
  const uint32_t ht = (hw >> 16) & 0xffu;
  const bool hv = ht == 1u || ht == 2u;
  const uint32_t gi = (28u + D + H) >> 2;  // GPS block word: 8, 9, 11 or 12
  // AND/OR masks, not selects: LLVM folds a select chain over an array back into a
  // dynamic index, which puts the array in scratch memory
  const uint32_t m8 = 0u - (uint32_t)(gi == 8u), m9 = 0u - (uint32_t)(gi == 9u);
  const uint32_t m11 = 0u - (uint32_t)(gi == 11u), m12 = 0u - (uint32_t)(gi == 12u);
  auto gword = [&](int k) {
    return (wd[8 + k] & m8) | (wd[9 + k] & m9) | (wd[11 + k] & m11) | (wd[12 + k] & m12);
  };
  const uint32_t g3 = gword(3);
  const uint32_t len = 44u + D + H;
  const uint16_t plen = bswap16((uint16_t)(g3 >> 16));
  const bool pl_ok = plen != 0 && len + plen <= buf_len;  // mgenMsg.cpp:488-497
  const uint32_t lat = bswap32(gword(0)), lon = bswap32(gword(1)), alt = bswap32(gword(2));
  const bool d16 = D == 16u;
  const u32x4_t dst = {wd[6], d16 ? wd[7] : 0u, d16 ? wd[8] : 0u, d16 ? wd[9] : 0u};
  // host address at word 8 (dst IPv4) or 11 (dst IPv6); zero unless a valid type
  const uint32_t a0 = (!hv || H == 0u) ? 0u : (D == 4u ? wd[8] : wd[11]);
  const bool h16 = hv && H == 16u;  // only with dst IPv4 (D + H <= 20)
  const u32x4_t host = {a0, h16 ? wd[9] : 0u, h16 ? wd[10] : 0u, h16 ? wd[11] : 0u};
  if (!do_store) return;
  if (c.decoded)  // a fast layout decodes every field (header <= 64 <= buf_len)
    c.decoded[i] = (uint8_t)(MGENX_DEC_MSGLEN | MGENX_DEC_BASE | MGENX_DEC_DST | MGENX_DEC_HDRLEN |
                             MGENX_DEC_GPS | MGENX_DEC_PTYPE | MGENX_DEC_PLEN |
                             (hv ? MGENX_DEC_HOST : 0));
  if (c.hdr_len) c.hdr_len[i] = (uint16_t)len;
  if (c.payload_off) c.payload_off[i] = pl_ok ? len : 0u;  // len % 4 == 0
  if (c.host_port) c.host_port[i] = hv ? bswap16((uint16_t)(hw & 0xffffu)) : 0;
  if (c.host_type) c.host_type[i] = hv ? (uint8_t)ht : 0;
  if (c.host_len) c.host_len[i] = hv ? (uint8_t)H : 0;
  if (c.lat_raw) c.lat_raw[i] = lat;
  if (c.lon_raw) c.lon_raw[i] = lon;
  if (c.alt) c.alt[i] = (int32_t)alt;
  if (c.dst_addr) *reinterpret_cast<u32x4_t*>(c.dst_addr + i * 16) = dst;
  if (c.host_addr) *reinterpret_cast<u32x4_t*>(c.host_addr + i * 16) = host;
}

// Extended columns of a record decoded by parse_header (quad lane 0).
__device__ __forceinline__ void store_hdr_ext(const mgenx_cols& c, uint64_t i, const Hdr& h) {
  if (c.decoded) c.decoded[i] = h.dec;
  if (c.hdr_len) c.hdr_len[i] = h.hdr_len;
  if (c.payload_off) c.payload_off[i] = h.poff;
  if (c.host_port) c.host_port[i] = h.host_port;
  if (c.host_type) c.host_type[i] = h.host_type;
  if (c.host_len) c.host_len[i] = h.host_len;
  if (c.lat_raw) c.lat_raw[i] = h.lat;
  if (c.lon_raw) c.lon_raw[i] = h.lon;
  if (c.alt) c.alt[i] = h.alt;
  if (c.host_addr) {
    u32x4_t* hp = reinterpret_cast<u32x4_t*>(c.host_addr + i * 16);
    *hp = u32x4_t{h.host_addr[0], h.host_addr[1], h.host_addr[2], h.host_addr[3]};
  }
  if (c.dst_addr) {
    u32x4_t* dp = reinterpret_cast<u32x4_t*>(c.dst_addr + i * 16);
    *dp = u32x4_t{h.dst_addr[0], h.dst_addr[1], h.dst_addr[2], h.dst_addr[3]};
  }
}

// A record decoded by parse_header, stored whole by quad lane 0 (the rare general
// layouts and short records): core fields as a row or as columns, then extended columns.
__device__ __forceinline__ void store_hdr_q0(const mgenx_cols& c, uint64_t i, const Hdr& h,
                                             bool crc_ok, bool tcp) {
  uint8_t err = h.err, flags = h.flags;
  crc_verdict(crc_ok, tcp, err, flags);
  if (c.rows) {
    u32x4_t* r = reinterpret_cast<u32x4_t*>(c.rows + i);
    r[0] = u32x4_t{h.flow, h.seq, h.sec, h.usec};
    r[1] = u32x4_t{h.dst4, (uint32_t)h.msg_len | ((uint32_t)h.dst_port << 16),
                   (uint32_t)h.plen | ((uint32_t)flags << 16) | ((uint32_t)err << 24),
                   (uint32_t)h.dst_type | ((uint32_t)h.dst_len << 8) |
                       ((uint32_t)h.ptype << 16) | ((uint32_t)h.gps << 24)};
  } else {
    c.flow_id[i] = h.flow;
    c.seq_num[i] = h.seq;
    c.tx_sec[i] = h.sec;
    c.tx_usec[i] = h.usec;
    c.msg_len[i] = h.msg_len;
    c.dst_port[i] = h.dst_port;
    c.flags[i] = flags;
    c.err[i] = err;
    c.dst_type[i] = h.dst_type;
    c.dst_len[i] = h.dst_len;
    c.dst_addr4[i] = h.dst4;
    c.payload_len[i] = h.plen;
    c.payload_type[i] = h.ptype;
    c.gps_status[i] = h.gps;
  }
  store_hdr_ext(c, i, h);
}

// Fast-layout record stored whole by quad lane 0 from the gathered prefix words pw[16]
// (general kernel): core fields as a row or as columns, then extended columns.
__device__ __forceinline__ void store_fast_q0(const mgenx_cols& c, uint64_t i,
                                              const uint32_t (&pw)[16], uint32_t buf_len,
                                              bool crc_ok, bool tcp) {
  const uint32_t D = pw[5] >> 24;
  const uint32_t hw = (D == 4u) ? pw[7] : pw[10];
  const uint32_t gi = (28u + D + (hw >> 24)) >> 2;
  const uint32_t g3 = (pw[11] & (0u - (uint32_t)(gi == 8u))) |
                      (pw[12] & (0u - (uint32_t)(gi == 9u))) |
                      (pw[14] & (0u - (uint32_t)(gi == 11u))) |
                      (pw[15] & (0u - (uint32_t)(gi == 12u)));
  const uint32_t len = 44u + D + (hw >> 24);
  uint32_t plen = bswap16((uint16_t)(g3 >> 16));
  if (!(plen != 0 && len + plen <= buf_len)) plen = 0;  // mgenMsg.cpp:488-497
  uint8_t flags = (uint8_t)(pw[0] >> 24), err = 0;
  crc_verdict(crc_ok, tcp, err, flags);
  const uint32_t msg_len = bswap16((uint16_t)(pw[0] & 0xffffu));
  const uint32_t dport = bswap16((uint16_t)(pw[5] & 0xffffu));
  const uint32_t dtype = (pw[5] >> 16) & 0xffu;
  if (c.rows) {
    u32x4_t* r = reinterpret_cast<u32x4_t*>(c.rows + i);
    r[0] = u32x4_t{bswap32(pw[1]), bswap32(pw[2]), bswap32(pw[3]), bswap32(pw[4])};
    r[1] = u32x4_t{pw[6], msg_len | (dport << 16), plen | ((uint32_t)flags << 16) |
                   ((uint32_t)err << 24),
                   dtype | (D << 8) | (((g3 >> 8) & 0xffu) << 16) | ((g3 & 0xffu) << 24)};
  } else {
    c.msg_len[i] = (uint16_t)msg_len;
    c.flags[i] = flags;
    c.err[i] = err;
    c.flow_id[i] = bswap32(pw[1]);
    c.seq_num[i] = bswap32(pw[2]);
    c.tx_sec[i] = bswap32(pw[3]);
    c.tx_usec[i] = bswap32(pw[4]);
    c.dst_port[i] = (uint16_t)dport;
    c.dst_type[i] = (uint8_t)dtype;
    c.dst_len[i] = (uint8_t)D;
    c.dst_addr4[i] = pw[6];
    c.payload_len[i] = (uint16_t)plen;
    c.payload_type[i] = (uint8_t)(g3 >> 8);
    c.gps_status[i] = (uint8_t)g3;
  }
}

// A descriptor outside the slab: ERROR_OOB and zeroed core fields (quad lane 0).
__device__ __forceinline__ void store_oob_q0(const mgenx_cols& c, uint64_t i) {
  if (c.decoded) c.decoded[i] = 0;
  if (c.rows) {
    u32x4_t* r = reinterpret_cast<u32x4_t*>(c.rows + i);
    r[0] = u32x4_t{0u, 0u, 0u, 0u};
    r[1] = u32x4_t{0u, 0u, (uint32_t)MGENX_ERROR_OOB << 24, 0u};
    return;
  }
  c.err[i] = MGENX_ERROR_OOB;
  c.flags[i] = 0;
  c.msg_len[i] = 0;
  c.flow_id[i] = 0;
  c.seq_num[i] = 0;
  c.tx_sec[i] = 0;
  c.tx_usec[i] = 0;
  c.dst_port[i] = 0;
  c.dst_type[i] = 0;
  c.dst_len[i] = 0;
  c.dst_addr4[i] = 0;
  c.payload_len[i] = 0;
  c.payload_type[i] = 0;
  c.gps_status[i] = 0;
}

// The core fields of one record, as every lane of its quad holds them.
struct Core {
  uint32_t flow, seq, sec, usec, dst4, msg_len, dport, plen, flags, err, dtype, dlen, ptype, gps;
};

// Branch-free core output of a quad: lane q stores column q (u32 / u16 / u8 groups, five
// store instructions), or bytes 8q..8q+7 of the record's mgenx_rec row.  Lanes whose
// record is past the batch end store to the sink.  Every lane must call it (no branch
// around the stores: see unpack_fixed_kernel on vmcnt and skipped stores).
template <bool kRows>
__device__ __forceinline__ void store_core_quad(const UnpackParams& p, uint64_t idx, bool in,
                                                int lane, int q, const Core& v) {
  const uint64_t sink = (uint64_t)p.sink + 8u * (uint32_t)lane;
  if (kRows) {
    const uint64_t x =
        q == 0 ? ((uint64_t)v.seq << 32 | v.flow)
      : q == 1 ? ((uint64_t)v.usec << 32 | v.sec)
      : q == 2 ? ((uint64_t)((v.msg_len & 0xffffu) | v.dport << 16) << 32 | v.dst4)
               : ((uint64_t)(v.dtype | v.dlen << 8 | v.ptype << 16 | v.gps << 24) << 32 |
                  ((v.plen & 0xffffu) | v.flags << 16 | v.err << 24));
    st_g64(in ? (uint64_t)p.cols.rows + idx * 32 + 8u * q : sink, x);
    return;
  }
  const mgenx_cols& c = p.cols;
  auto at = [&](uint64_t base, uint32_t size) { return in ? base + idx * size : sink; };
  const uint64_t u32 = pick4(q, (uint64_t)c.flow_id, (uint64_t)c.seq_num, (uint64_t)c.tx_sec,
                             (uint64_t)c.tx_usec);
  const uint64_t u16 = pick4(q, (uint64_t)c.msg_len, (uint64_t)c.dst_port,
                             (uint64_t)c.payload_len, (uint64_t)c.payload_len);
  const uint64_t u8a = pick4(q, (uint64_t)c.flags, (uint64_t)c.err, (uint64_t)c.dst_type,
                             (uint64_t)c.dst_len);
  const uint64_t u8b = pick4(q, (uint64_t)c.payload_type, (uint64_t)c.gps_status,
                             (uint64_t)c.payload_type, (uint64_t)c.gps_status);
  st_g32(at(u32, 4), q == 0 ? v.flow : q == 1 ? v.seq : q == 2 ? v.sec : v.usec);
  st_g32(at((uint64_t)c.dst_addr4, 4), v.dst4);
  st_g16(at(u16, 2), q == 0 ? v.msg_len : q == 1 ? v.dport : v.plen);
  st_g8(at(u8a, 1), q == 0 ? v.flags : q == 1 ? v.err : q == 2 ? v.dtype : v.dlen);
  st_g8(at(u8b, 1), (q & 1) == 0 ? v.ptype : v.gps);
}

// store_core_quad with the per-lane field picked by AND/OR masks over scalars (a select
// chain over a struct can be folded back into a dynamic index, which puts it in scratch)
__device__ __forceinline__ void store_core_quad_m(const UnpackParams& p, uint64_t idx, bool in,
                                                  int lane, int q, const Core& v) {
  const uint32_t m0 = 0u - (uint32_t)(q == 0), m1 = 0u - (uint32_t)(q == 1);
  const uint32_t m2 = 0u - (uint32_t)(q == 2), m3 = 0u - (uint32_t)(q == 3);
  auto pick = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (a & m0) | (b & m1) | (c & m2) | (d & m3);
  };
  const uint64_t sink = (uint64_t)p.sink + 8u * (uint32_t)lane;
  if (p.cols.rows) {
    const uint32_t lo = pick(v.flow, v.sec, v.dst4, (v.plen & 0xffffu) | v.flags << 16 | v.err << 24);
    const uint32_t hi = pick(v.seq, v.usec, (v.msg_len & 0xffffu) | v.dport << 16,
                             v.dtype | v.dlen << 8 | v.ptype << 16 | v.gps << 24);
    st_g64(in ? (uint64_t)p.cols.rows + idx * 32 + 8u * q : sink, (uint64_t)hi << 32 | lo);
    return;
  }
  const mgenx_cols& c = p.cols;
  const uint64_t a32 = pick4(q, (uint64_t)c.flow_id, (uint64_t)c.seq_num, (uint64_t)c.tx_sec,
                             (uint64_t)c.tx_usec);
  const uint64_t a16 = pick4(q, (uint64_t)c.msg_len, (uint64_t)c.dst_port,
                             (uint64_t)c.payload_len, (uint64_t)c.payload_len);
  const uint64_t a8a = pick4(q, (uint64_t)c.flags, (uint64_t)c.err, (uint64_t)c.dst_type,
                             (uint64_t)c.dst_len);
  const uint64_t a8b = pick4(q, (uint64_t)c.payload_type, (uint64_t)c.gps_status,
                             (uint64_t)c.payload_type, (uint64_t)c.gps_status);
  st_g32(in ? a32 + idx * 4 : sink, pick(v.flow, v.seq, v.sec, v.usec));
  st_g32(in ? (uint64_t)c.dst_addr4 + idx * 4 : sink, v.dst4);
  st_g16(in ? a16 + idx * 2 : sink, pick(v.msg_len, v.dport, v.plen, v.plen));
  st_g8(in ? a8a + idx : sink, pick(v.flags, v.err, v.dtype, v.dlen));
  st_g8(in ? a8b + idx : sink, pick(v.ptype, v.gps, v.ptype, v.gps));
}

// MODE (diagnostic ablations, never the product path): 0 = full kernel, 1 = row loads +
// XOR only (no LDS table lookups), 2 = table lookups on one L1-resident row (no streaming).
// pw[4*LN .. 4*LN+3] = quad lane LN's 16-byte prefix chunk (DPP quad_perm broadcast; all
// four lanes of the quad must be active).
template <int LN>
__device__ __forceinline__ void quad_bcast(const u32x4_t& pf, uint32_t (&pw)[16]) {
  constexpr int ctrl = LN | (LN << 2) | (LN << 4) | (LN << 6);
  pw[4 * LN + 0] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pf.x, ctrl, 0xf, 0xf, false);
  pw[4 * LN + 1] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pf.y, ctrl, 0xf, 0xf, false);
  pw[4 * LN + 2] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pf.z, ctrl, 0xf, 0xf, false);
  pw[4 * LN + 3] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pf.w, ctrl, 0xf, 0xf, false);
}

template <bool kCrc, int MODE = 0, bool kSort = false>
__global__ void __launch_bounds__(kUnpackThreads)
unpack_kernel(UnpackParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* rep = lds;
  uint32_t* fold = lds + kRepDwords;  // [A4 | A8 | A12 | A16 | A32 | A48]

  // ---- stage the shift-operator tables (A_64 replicated 32x) ----
  if (kCrc) {
    stage_tables(lds, p.tabs);
    __syncthreads();
  }
  const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(rep);

  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const uint32_t s1 = a64_s1((uint32_t)lane);
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint64_t wave_id = (uint64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
  const uint64_t n_waves = (uint64_t)gridDim.x * waves_per_block;
  const uint64_t n_groups = ((uint64_t)p.n + 15) >> 4;
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const bool want_ext = p.cols.dst_addr || p.cols.host_addr;
  const mgenx_cols& cc = p.cols;
  const bool any_ext = cc.hdr_len || cc.payload_off || cc.host_port || cc.host_type ||
                       cc.host_len || cc.lat_raw || cc.lon_raw || cc.alt || cc.dst_addr ||
                       cc.host_addr || cc.decoded;

  // Per-wave predictor: while recent groups carried checksummed records, issue the row
  // loads speculatively together with the header load (one memory round per group); a
  // group without any CRC work turns speculation off (header first, body only if needed).
  bool spec = true;
  // one group: the quad's record rec_idx (valid: < n), the wave's 16 records together
  // (off, L: its placement, read by the caller)
  auto group = [&](const uint64_t rec_idx, const bool valid, const uint64_t off, const uint32_t L) {
    const bool oob = valid && (L > 65535u || off > p.slab_bytes || L > p.slab_bytes - off);
    const bool live = valid && !oob;
    const uint8_t* rec = p.slab + off;
    const uint32_t buf_len = tcp ? min(L, (uint32_t)MGENX_TX_BUFFER_SIZE) : L;

    // Header prefix: lane q of the quad loads bytes [16q, 16q+16) (64 bytes per record,
    // enough for every layout but IPv6 dst + IPv6 host); quad lane 0 gathers the words by
    // DPP quad broadcast when it parses.  Loads are unconditional (clamped to a dummy line)
    // so no divergent branch forces a full vmcnt wait.
    const bool pfx = live && L >= 32;           // prefix words 0..7 valid
    const bool pfx64 = live && buf_len >= 64;   // prefix words 0..15 valid
    const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.tabs);
    u32x4_t pf = {0u, 0u, 0u, 0u};
    uint32_t w[8];
    uint32_t expect = 0;
    auto load_header = [&]() {
      pf = ldu128((live && L >= 16u * (q + 1)) ? rec + 16 * q : dummy);
      if (kCrc) expect = p.expect[live ? L : 0u];
    };
    // prefix words 0..15 of the quad's record, gathered by DPP with every lane active
    auto gather = [&](uint32_t (&pw)[16]) {
      quad_bcast<0>(pf, pw);
      quad_bcast<1>(pf, pw);
      quad_bcast<2>(pf, pw);
      quad_bcast<3>(pf, pw);
    };
    auto unpack_words = [&](const uint32_t (&pw)[16]) {
      if (pfx) {
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = pw[j];
      } else if (live && L >= MGENX_MIN_SIZE) {
        load_fixed(rec, buf_len, w);  // 28..31-byte records
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = 0;
      }
    };
    bool needs_crc = false;
    auto decide = [&]() {
      uint32_t pw[16];
      gather(pw);
      if (kCrc && live && q == 0) {  // quad lane 0 decides and stores
        unpack_words(pw);
        const bool flagged = force || (((w[0] >> 24) & MGENX_FLAG_CHECKSUM) != 0 &&
                                       buf_len >= MGENX_MIN_SIZE &&
                                       ((w[0] >> 16) & 0xffu) == 2u);
        needs_crc = flagged && (tcp ? (L >= 4) : fixed_ok(buf_len, w));
      }
    };

    uint32_t tot = 0;
    const bool speculate = kCrc && (spec || force);
    bool run_crc = speculate;
    if (!speculate) {
      load_header();
      if (kCrc) {
        decide();
        run_crc = __any(needs_crc);
      }
    }
    if (kCrc && run_crc) {
      // ---- braid CRC over end-aligned 64-byte rows ----
      // R depends only on L, so the row loads need nothing from the header.  Quads are
      // front-padded with zero rows to the wave-uniform count V (leading zeros leave a
      // zero-initialised CRC unchanged): all lanes run the same updates.
      const int R = (live && L >= 32) ? (int)((L + 63u) >> 6) : 0;
      const bool vec = R > 0;
      const int64_t row0 = (int64_t)L - 64 * (int64_t)R + 16 * q;  // position of row 0
      int Rmax = R;
#pragma unroll
      for (int sft = 1; sft < 64; sft <<= 1) Rmax = max(Rmax, __shfl_xor(Rmax, sft));
      const int V = __builtin_amdgcn_readfirstlane(Rmax);  // virtual rows 0..V-1 (V-1 final)
      const int pad = V - R;
      const bool multi = R >= 2;
      const uint8_t* base = multi ? rec + row0 : reinterpret_cast<const uint8_t*>(p.tabs);
      const int hi_row = multi ? R - 1 : 0;
      auto row_addr = [&](int j) {
        const int real = j - pad;
        const int rr = real < 1 ? 1 : (real > hi_row ? hi_row : real);
        return base + 64 * (multi ? (MODE == 2 ? 1 : rr) : 0);
      };
      // braid state word b = ha[b] ^ hb[b] (kept split so the next row folds in one XOR3)
      uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
      const u32x4_t zero = {0u, 0u, 0u, 0u};
      u32x4_t xr = zero, xf = zero;
      // row 0 may start before the record: it is loaded from max(row0, 0) and its bytes
      // shifted up by s0 (0 when aligned); a row entirely before the record is padding
      const int s0 = row0 >= 0 ? 0 : (int)(-row0);
      auto load_row0 = [&]() { xr = ldu128(vec ? rec + (row0 >= 0 ? row0 : 0) : dummy); };
      auto load_final = [&]() { xf = ldu128(base + 64 * hi_row); };  // unused if R < 2
      auto row0_data = [&]() { return (vec && s0 < 16) ? shl_bytes(xr, s0) : zero; };
      auto consume = [&](const u32x4_t& dv, int j) {
        const int real = j - pad;
        const u32x4_t x = (real == 0) ? row0_data() : zero;
        u32x4_t xin;
        xin.x = real > 0 ? dv.x : (real == 0 ? x.x : 0u);
        xin.y = real > 0 ? dv.y : (real == 0 ? x.y : 0u);
        xin.z = real > 0 ? dv.z : (real == 0 ? x.z : 0u);
        xin.w = real > 0 ? dv.w : (real == 0 ? x.w : 0u);
        const uint32_t xw[4] = {xin.x, xin.y, xin.z, xin.w};
        if (MODE == 1) {
#pragma unroll
          for (int b = 0; b < 4; b++) ha[b] = (ha[b] << 1) ^ xw[b];
        } else {
          // all 16 lookups of the row are independent: every address first, the 16 LDS
          // reads back to back, then the folds (one LDS round trip per row)
#pragma unroll
          for (int b = 0; b < 4; b++) a64_parts(ldsb, xor3(ha[b], hb[b], xw[b]), s1, ha[b], hb[b]);
        }
      };
      // One block of N middle rows (virtual rows j0..j0+N-1, all in 1..V-2): all loads
      // issued first (unconditional, clamped addresses), then -- first block only -- row 0,
      // the final row and the header, then consumption in order with counted waits.  The
      // empty asm with a memory clobber keeps LLVM from sinking a load into its consumer.
      auto block = [&](auto n_tag, int j0, int cnt, bool first) {
        constexpr int N = decltype(n_tag)::value;
        u32x4_t d[N];
        // issue order = consumption order: row 0, the block, then the final row + header
        if (first) load_row0();
#pragma unroll
        for (int k = 0; k < N; k++) d[k] = ldu128(row_addr(j0 + k));
        if (first) {
          load_final();
          if (speculate) load_header();
        }
        asm volatile("" ::: "memory");
        if (first && V >= 2) consume(zero, 0);  // virtual row 0: row 0 (from xr) or padding
#pragma unroll
        for (int k = 0; k < N; k++)
          if (k < cnt) consume(d[k], j0 + k);
      };
      using B14 = std::integral_constant<int, 14>;
      using B6 = std::integral_constant<int, 6>;
      using B2 = std::integral_constant<int, 2>;
      const int mid = V - 2;  // middle rows 1..V-2 (wave-uniform)
      if (mid <= 2) {
        block(B2{}, 1, mid, true);
      } else if (mid <= 6) {
        block(B6{}, 1, mid, true);
      } else {
        block(B14{}, 1, min(14, mid), true);
        for (int j0 = 15; j0 <= mid; j0 += 14) block(B14{}, j0, min(14, mid + 1 - j0), false);
      }
      u32x4_t x = multi ? xf : row0_data();
      if (speculate) decide();
      // last row: byte-swap the big-endian trailer into little-endian stream order
      if (q == 3) x.w = bswap32(x.w);
      // fold: word b of lane q sits 64-16q-4b bytes before the record end, so
      //   v_q = A16(g0) ^ A12(g1) ^ A8(g2) ^ A4(g3),  tot = XOR_q A_{48-16q}(v_q)
      // (16 independent lookups, then one per-lane lookup and a quad XOR-reduce)
      const uint32_t v = shift_tab(fold + 3 * 1024, xor3(ha[0], hb[0], x.x)) ^
                         shift_tab(fold + 2 * 1024, xor3(ha[1], hb[1], x.y)) ^
                         shift_tab(fold + 1 * 1024, xor3(ha[2], hb[2], x.z)) ^
                         shift_tab(fold, xor3(ha[3], hb[3], x.w));
      const uint32_t* lt = fold + (q == 0 ? 5 : (q == 1 ? 4 : 3)) * 1024;  // A48/A32/A16
      uint32_t s = (q == 3) ? v : shift_tab(lt, v);
      s ^= __shfl_xor(s, 1);
      s ^= __shfl_xor(s, 2);
      tot = s;
      spec = __any(needs_crc);
    } else if (kCrc) {
      spec = false;
    }
    if (!kCrc) load_header();
    const bool vec_crc = needs_crc && live && L >= 32;

    uint32_t pw[16];
    gather(pw);
    if (live && q == 0) {
      // each parse path stores its own record (no join merging two decoded headers)
      if (pfx64 && fast_layout(pw[0], pw[5], (pw[5] >> 24) == 4u ? pw[7] : pw[10])) {
        store_fast_q0(p.cols, rec_idx, pw, buf_len, !needs_crc || tot == expect, tcp);
        if (any_ext) store_fast_ext(p.cols, rec_idx, [&](int k) { return pw[k]; }, buf_len, true);
      } else {
        Hdr h;
        unpack_words(pw);
        parse_header(rec, buf_len, want_ext, w, h);
        const bool crc_ok =
            !needs_crc || (vec_crc ? (tot == expect) : small_crc_ok(rec, L));
        store_hdr_q0(p.cols, rec_idx, h, crc_ok, tcp);
      }
    } else if (oob && q == 0) {
      store_oob_q0(p.cols, rec_idx);
    }
  };

  auto place = [&](uint64_t ri, uint64_t& off, uint32_t& L) {
    off = 0;
    L = 0;
    if (ri < p.n) {
      off = p.rec_off ? p.rec_off[ri] : ri * p.stride;
      L = p.rec_len ? p.rec_len[ri] : p.fixed_len;
    }
  };
  if (!kSort) {
    for (uint64_t g = wave_id; g < n_groups; g += n_waves) {
      const uint64_t ri = (g << 4) + (uint64_t)(lane >> 2);
      uint64_t off;
      uint32_t L;
      place(ri, off, L);
      group(ri, ri < p.n, off, L);
    }
    return;
  }
  // Row-balanced order for variable lengths.  A group costs its LONGEST record's rows (the
  // quads run in lock-step, shorter records front-padded), so each wave takes a tile of 64
  // consecutive records, ranks them by row count (64 lane compares), and runs them as four
  // groups of 16 records of similar length (U{64..1472}: 83% of the rows useful instead of
  // 56%).  The tile's column stores stay within 64 consecutive records.  The placements of
  // the next tile are loaded while this one runs (lane j: record t0 + j), and reach the
  // quads by lane permutes.
  const uint64_t n_tiles = ((uint64_t)p.n + 63) >> 6;
  uint64_t off_n;
  uint32_t len_n;
  place((wave_id << 6) + (uint64_t)lane, off_n, len_n);
  for (uint64_t t = wave_id; t < n_tiles; t += n_waves) {
    const uint64_t t0 = t << 6;
    const uint64_t off_l = off_n;
    const uint32_t len_l = len_n;
    place(((t + n_waves) << 6) + (uint64_t)lane, off_n, len_n);
    const uint32_t n_valid = (uint32_t)min((uint64_t)64, (uint64_t)p.n - t0);
    const uint32_t key = (uint32_t)lane < n_valid ? (len_l + 63u) >> 6 : 0xFFFFu;
    uint32_t rank = 0;
#pragma unroll 8
    for (int j = 0; j < 64; j++) {
      const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, j);
      rank += (kj < key || (kj == key && j < lane)) ? 1u : 0u;
    }
    // sorted position r -> the tile lane holding it (lane r receives it)
    const int src = __builtin_amdgcn_ds_permute((int)(rank << 2), lane);
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
      if ((uint32_t)(16 * k) >= n_valid) break;  // wave-uniform: past-the-end sorts last
      const int li = __builtin_amdgcn_ds_bpermute((16 * k + (lane >> 2)) << 2, src);
      const int at = li << 2;
      const uint64_t off = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)(uint32_t)off_l) |
                           (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)(uint32_t)(off_l >> 32)) << 32;
      const uint32_t L = (uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)len_l);
      group(t0 + (uint64_t)li, (uint32_t)li < n_valid, off, L);
    }
  }
}


// ---------------------------------------------------------------------------------------
// Variable-length records (per-record lengths: config 3, TCP / SINK scan output), with the
// rows streamed through a load ring across groups.  The braid CRC and the column output
// are those of unpack_kernel<true>; what differs is the schedule:
//   * each wave takes tiles of 64 consecutive records, ranks them by row count R (64 lane
//     compares) and runs them as four groups of 16 records of similar length;
//   * a group's virtual rows are V = max R of its records rounded up to an even count >= 4
//     (shorter records front-padded with zero rows, which leave the zero CRC state as is);
//   * the wave's rows form ONE stream over its groups, with RS = 4 rows in flight: row
//     r + 4 of the stream is loaded as row r is consumed -- during a group's last four rows
//     that is the next group's first four rows (its header follows the group's column
//     stores) -- so the loads never drain at group boundaries (the next tile is ranked one group ahead,
//     its placements loaded one tile ahead).
// No header-first mode: every record's rows are read (for batches without checksummed
// records this reads the bodies too; the payload stays unread by the CRC work otherwise).
// Row output (r03): the rows of the last KB groups are held in registers (lo / hi word of
// the quad lane's 8 bytes and the record index) and stored in one burst every KB groups, as
// the ring kernel does, instead of one row store per group mixed into the read stream.
// Config 3 (`scripts/var_shapes.py`): per-group stores 0.250 ms, KB = 4 0.236 ms, every row
// store sent to one scratch line (MODE 1, the bound of any store schedule) 0.223 ms.  KB = 8
// spills 23 VGPRs at the 128-VGPR limit of 16 waves per CU (0.240 ms); 12 waves per CU with
// KB = 8 or 16 fit the registers but lose the loads in flight (0.245-0.253 ms); flushing at
// each tile's end with the indices recomputed from the rank permutation 0.239 ms;
// non-temporal row stores 0.241-0.246 ms; tiles handed out by an atomic ticket (dynamic
// balance) 0.32-0.44 ms; (r04) a tile's 64 rows gathered by lane permutes and stored as 2 KiB
// of whole lines (two 16-B stores per lane instead of four scattered 8-B ones) 0.2359 ms
// against 0.2361 (15 VGPRs spilled; the partial-line writes are not what costs).
// Template knobs (the product instantiation is unpack_var_kernel<kUnpackThreads, 4, 0>):
//   NT   block size (one block per CU: the LDS tables);
//   KB   groups of rows held (0: one row store per group);
//   MODE bit 1 (ablation): every core store to the sink; bit 8: non-temporal row stores;
//   bit 16: every row load 64-byte aligned (wrong data, timing only).
template <int NT, int KB, int MODE>
__global__ void __launch_bounds__(NT)
unpack_var_kernel(UnpackParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t* fold = lds + kRepDwords;  // [A4 | A8 | A12 | A16 | A32 | A48]
  stage_tables(lds, p.tabs);
  __syncthreads();
  const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(lds);

  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const uint32_t s1 = a64_s1((uint32_t)lane);
  const uint64_t wave_id = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t n_waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t n_tiles = ((uint64_t)p.n + 63) >> 6;
  if (wave_id >= n_tiles) return;  // (no barrier below)
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const bool want_ext = p.cols.dst_addr || p.cols.host_addr;
  const mgenx_cols& cc = p.cols;
  const bool any_ext = cc.hdr_len || cc.payload_off || cc.host_port || cc.host_type ||
                       cc.host_len || cc.lat_raw || cc.lon_raw || cc.alt || cc.dst_addr ||
                       cc.host_addr || cc.decoded;
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.tabs);
  const u32x4_t zero = {0u, 0u, 0u, 0u};

  // ---- tiles: placements of the 64 records (lane j: record t0 + j) and their order ----
  auto place = [&](uint64_t t, uint64_t& off, uint32_t& L) {
    const uint64_t ri = (t << 6) + (uint64_t)lane;
    off = 0;
    L = 0;
    if (t < n_tiles && ri < p.n) {
      off = p.rec_off ? p.rec_off[ri] : ri * p.stride;
      L = p.rec_len ? p.rec_len[ri] : p.fixed_len;
    }
  };
  auto n_valid_of = [&](uint64_t t) { return (uint32_t)min((uint64_t)64, (uint64_t)p.n - (t << 6)); };
  // sorted position r -> the tile lane holding it
  auto rank_tile = [&](uint64_t t, uint32_t L) {
    const uint32_t key = (uint32_t)lane < n_valid_of(t) ? (L + 63u) >> 6 : 0xFFFFu;
    uint32_t rank = 0;
#pragma unroll 8
    for (int j = 0; j < 64; j++) {
      const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, j);
      rank += (kj < key || (kj == key && j < lane)) ? 1u : 0u;
    }
    return __builtin_amdgcn_ds_permute((int)(rank << 2), lane);
  };
  // the wave's tiles: wave_id, + n_waves, ...
  uint64_t t_c = wave_id, off_c, off_p;
  uint64_t t_p = t_c + n_waves;
  uint32_t len_c, len_p;
  place(t_c, off_c, len_c);
  int src_c = rank_tile(t_c, len_c), src_p = lane;
  place(t_p, off_p, len_p);
  bool p_ranked = false;

  // ---- (KB > 0) rows held per group: lo / hi word of the quad lane's 8 bytes, record index
  // (~0: the record's row is not the burst's -- a slow-layout or out-of-bounds record, stored
  // at once by quad lane 0)
  constexpr int KH = KB > 0 ? KB : 1;
  uint32_t b0[KH], b1[KH], bi[KH];
#pragma unroll
  for (int j = 0; j < KH; j++) b0[j] = b1[j] = 0u, bi[j] = 0xFFFFFFFFu;
  uint32_t held = 0;
  const bool burst = KB > 0 && p.cols.rows != nullptr && !(MODE & 1);
  auto st_row = [&](uint64_t a, uint64_t v) {
    if (MODE & 8) st_g64_nt(a, v);
    else st_g64(a, v);
  };
  auto flush = [&]() {
#pragma unroll
    for (int j = 0; j < KH; j++) {
      const uint32_t back = (uint32_t)(KH - 1 - j);
      if (back < held)  // wave-uniform
        st_row(bi[j] != 0xFFFFFFFFu ? (uint64_t)p.cols.rows + (uint64_t)bi[j] * 32 + 8u * q
                                    : (uint64_t)p.sink + 8u * (uint32_t)lane,
               (uint64_t)b1[j] << 32 | b0[j]);
    }
    held = 0;
  };

  // ---- a group: the quad's record and its row geometry ----
  struct Grp {
    uint64_t off;
    uint32_t idx, L;
    int pos0, pad;        // row 0 position in the record (+16q), virtual rows before row 0
    bool valid, live, oob;
    uint32_t V;           // virtual rows (wave-uniform, even, >= 4)
  };
  auto make = [&](uint64_t t, int k, uint64_t offs, uint32_t lens, int src) {
    Grp g;
    const int li = __builtin_amdgcn_ds_bpermute((16 * k + (lane >> 2)) << 2, src);
    const int at = li << 2;
    g.idx = (uint32_t)(t << 6) + (uint32_t)li;
    g.off = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)(uint32_t)offs) |
            (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)(uint32_t)(offs >> 32)) << 32;
    g.L = (uint32_t)__builtin_amdgcn_ds_bpermute(at, (int)lens);
    g.valid = (uint32_t)li < n_valid_of(t);
    g.oob = g.valid && (g.L > 65535u || g.off > p.slab_bytes || g.L > p.slab_bytes - g.off);
    g.live = g.valid && !g.oob;
    const int R = (g.live && g.L >= 32) ? (int)((g.L + 63u) >> 6) : 0;
    int m = R;
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) m = max(m, __shfl_xor(m, sft));
    g.V = (uint32_t)max(4, (__builtin_amdgcn_readfirstlane(m) + 1) & ~1);
    g.pad = (int)g.V - R;
    g.pos0 = (int)g.L - 64 * R + 16 * q;
    return g;
  };
  auto row_ptr = [&](const Grp& g, int j) {
    const int real = j - g.pad;
    if (MODE & 16) {  // (ablation, timing only: every row load 64-byte aligned, wrong data)
      const uint64_t a = (g.off + (uint64_t)max(g.pos0 - 16 * q + 64 * real, 0)) & ~(uint64_t)63;
      return (real >= 0) ? p.slab + a + 16u * (uint32_t)q : dummy;
    }
    return (real >= 0) ? p.slab + g.off + (uint64_t)max(g.pos0 + 64 * real, 0) : dummy;
  };
  auto hdr_ptr = [&](const Grp& g) {
    return (g.live && g.L >= 16u * (q + 1)) ? p.slab + g.off + 16 * q : dummy;
  };
  // row j's 16 bytes as the braid consumes them: row 0 of a record that does not start on
  // a row boundary is shifted up (its bytes before the record read as zero)
  auto row_data = [&](const Grp& g, const u32x4_t& x, int j) {
    const int real = j - g.pad;
    u32x4_t y = real >= 0 ? x : zero;
    const int s0 = g.pos0 < 0 ? -g.pos0 : 0;
    if (__any(real == 0 && s0 > 0)) {
      const u32x4_t sh = s0 < 16 ? shl_bytes(x, s0 & 15) : zero;
      if (real == 0) y = sh;
    }
    return y;
  };

  // ---- the first group ----
  int k = 0;
  int rho = 0;  // ring slot of the current group's row 0
  Grp G = make(t_c, 0, off_c, len_c, src_c);
  u32x4_t d[4];
#pragma unroll
  for (int j = 0; j < 4; j++) d[j] = ldu128(row_ptr(G, j));
  u32x4_t pf = ldu128(hdr_ptr(G));
  uint32_t expect = p.expect[G.live ? G.L : 0u];

  for (;;) {
    // the next group: this tile's group k + 1, or the next tile's first (ranked here)
    bool has_next = true, next_tile = false;
    Grp N;
    if (k + 1 < 4 && (uint32_t)(16 * (k + 1)) < n_valid_of(t_c)) {
      N = make(t_c, k + 1, off_c, len_c, src_c);
    } else if (t_p < n_tiles) {
      if (!p_ranked) {
        src_p = rank_tile(t_p, len_p);
        p_ranked = true;
      }
      N = make(t_p, 0, off_p, len_p, src_p);
      next_tile = true;
    } else {
      has_next = false;
      N = G;
      N.V = 4;
      N.pad = 4;  // all padding: the ring loads the dummy line
    }

    // ---- stream G's rows: chunks of 4, the last chunk feeding N's first rows ----
    uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
    auto consume = [&](const u32x4_t& y) {
      const uint32_t xw[4] = {y.x, y.y, y.z, y.w};
      uint32_t c4[4];
#pragma unroll
      for (int b = 0; b < 4; b++) c4[b] = xor3(ha[b], hb[b], xw[b]);
#pragma unroll
      for (int b = 0; b < 4; b++) a64_parts(ldsb, c4[b], s1, ha[b], hb[b]);
    };
    // G's row r sits in ring slot (r + rho) & 3 (rho in {0, 2}: V is even, not necessarily a
    // multiple of 4, so a group may start mid-ring); each variant keeps every slot index
    // static (a register copy of an in-flight row would make LLVM drain the ring)
    auto tail = [&](auto RT, int jl) {  // the last 4 rows, reloading N's rows 0..3
      constexpr int T = decltype(RT)::value;
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const u32x4_t y = row_data(G, d[(j + T) & 3], jl + j);
        __builtin_amdgcn_sched_barrier(0);
        d[(j + T) & 3] = ldu128(row_ptr(N, j));
        __builtin_amdgcn_sched_barrier(0);
        consume(y);
      }
      u32x4_t xf = row_data(G, d[(3 + T) & 3], jl + 3);
      __builtin_amdgcn_sched_barrier(0);
      d[(3 + T) & 3] = ldu128(row_ptr(N, 3));
      __builtin_amdgcn_sched_barrier(0);
      if (q == 3) xf.w = bswap32(xf.w);  // the big-endian trailer, in stream order
      const uint32_t v = shift_tab(fold + 3 * 1024, xor3(ha[0], hb[0], xf.x)) ^
                         shift_tab(fold + 2 * 1024, xor3(ha[1], hb[1], xf.y)) ^
                         shift_tab(fold + 1 * 1024, xor3(ha[2], hb[2], xf.z)) ^
                         shift_tab(fold, xor3(ha[3], hb[3], xf.w));
      const uint32_t* lt = fold + (q == 0 ? 5 : (q == 1 ? 4 : 3)) * 1024;  // A48/A32/A16
      uint32_t t = (q == 3) ? v : shift_tab(lt, v);
      t ^= __shfl_xor(t, 1);
      t ^= __shfl_xor(t, 2);
      return t;
    };
    auto run = [&](auto RHO) {
      constexpr int R0 = decltype(RHO)::value;
      const int nc = (int)((G.V - 4) >> 2);  // whole chunks before the tail
#pragma unroll 1
      for (int c = 0; c < nc; c++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const u32x4_t y = row_data(G, d[(j + R0) & 3], 4 * c + j);
          __builtin_amdgcn_sched_barrier(0);
          d[(j + R0) & 3] = ldu128(row_ptr(G, 4 * c + 4 + j));
          __builtin_amdgcn_sched_barrier(0);
          consume(y);
        }
      }
      const int r0 = 4 * nc;
      if (G.V & 2u) {  // two rows more, then the tail two slots further round the ring
#pragma unroll
        for (int j = 0; j < 2; j++) {
          const u32x4_t y = row_data(G, d[(j + R0) & 3], r0 + j);
          __builtin_amdgcn_sched_barrier(0);
          d[(j + R0) & 3] = ldu128(row_ptr(G, r0 + 4 + j));
          __builtin_amdgcn_sched_barrier(0);
          consume(y);
        }
        return tail(std::integral_constant<int, R0 ^ 2>{}, r0 + 2);
      }
      return tail(std::integral_constant<int, R0>{}, r0);
    };
    uint32_t tot = rho ? run(std::integral_constant<int, 2>{}) : run(std::integral_constant<int, 0>{});
    rho = (rho + (int)G.V) & 3;

    // ---- G's columns (as unpack_kernel) ----
    {
      uint32_t pw[16];
      quad_bcast<0>(pf, pw);
      quad_bcast<1>(pf, pw);
      quad_bcast<2>(pf, pw);
      quad_bcast<3>(pf, pw);
      const uint8_t* rec = p.slab + G.off;
      const uint32_t buf_len = tcp ? min(G.L, (uint32_t)MGENX_TX_BUFFER_SIZE) : G.L;
      // fast layouts: every quad lane derives the fields from the prefix words and the
      // quad stores them branch-free (lane q: column group q); other records: quad lane 0
      const uint32_t D = pw[5] >> 24;
      const uint32_t hw = (D == 4u) ? pw[7] : pw[10];
      const bool fast = G.live && buf_len >= 64 && fast_layout(pw[0], pw[5], hw);
      {
        const uint32_t gi = (28u + D + (hw >> 24)) >> 2;
        const uint32_t g3 = (pw[11] & (0u - (uint32_t)(gi == 8u))) |
                            (pw[12] & (0u - (uint32_t)(gi == 9u))) |
                            (pw[14] & (0u - (uint32_t)(gi == 11u))) |
                            (pw[15] & (0u - (uint32_t)(gi == 12u)));
        const uint32_t hl = 44u + D + (hw >> 24);
        Core v;
        v.plen = bswap16((uint16_t)(g3 >> 16));
        if (!(v.plen != 0 && hl + v.plen <= buf_len)) v.plen = 0;  // mgenMsg.cpp:488-497
        const bool needs_crc = force || (((pw[0] >> 24) & MGENX_FLAG_CHECKSUM) != 0);
        uint8_t flags = (uint8_t)(pw[0] >> 24), err = 0;
        crc_verdict(!needs_crc || tot == expect, tcp, err, flags);
        v.flow = bswap32(pw[1]); v.seq = bswap32(pw[2]); v.sec = bswap32(pw[3]);
        v.usec = bswap32(pw[4]); v.dst4 = pw[6];
        v.msg_len = bswap16((uint16_t)(pw[0] & 0xffffu));
        v.dport = bswap16((uint16_t)(pw[5] & 0xffffu));
        v.flags = flags; v.err = err; v.dtype = (pw[5] >> 16) & 0xffu; v.dlen = D;
        v.ptype = (g3 >> 8) & 0xffu; v.gps = g3 & 0xffu;
        if (KB > 0 && burst) {
          const uint32_t m0 = 0u - (uint32_t)(q == 0), m1 = 0u - (uint32_t)(q == 1);
          const uint32_t m2 = 0u - (uint32_t)(q == 2), m3 = 0u - (uint32_t)(q == 3);
          auto pick = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
            return (a & m0) | (b & m1) | (c & m2) | (d & m3);
          };
#pragma unroll
          for (int j = 0; j < KH - 1; j++) b0[j] = b0[j + 1], b1[j] = b1[j + 1];
          b0[KH - 1] = pick(v.flow, v.sec, v.dst4, (v.plen & 0xffffu) | v.flags << 16 | v.err << 24);
          b1[KH - 1] = pick(v.seq, v.usec, (v.msg_len & 0xffffu) | v.dport << 16,
                            v.dtype | v.dlen << 8 | v.ptype << 16 | v.gps << 24);
#pragma unroll
          for (int j = 0; j < KH - 1; j++) bi[j] = bi[j + 1];
          bi[KH - 1] = fast ? G.idx : 0xFFFFFFFFu;
          held++;
        } else {
          store_core_quad_m(p, G.idx, fast && !(MODE & 1), lane, q, v);
        }
      }
      if (fast && any_ext) store_fast_ext(p.cols, G.idx, [&](int kk) { return pw[kk]; }, buf_len, q == 0);
      if (!fast && G.live && q == 0) {
        uint32_t w[8];
        if (G.L >= 32) {
#pragma unroll
          for (int j = 0; j < 8; j++) w[j] = pw[j];
        } else if (G.L >= MGENX_MIN_SIZE) {
          load_fixed(rec, buf_len, w);
        } else {
#pragma unroll
          for (int j = 0; j < 8; j++) w[j] = 0;
        }
        const bool flagged = force || (((w[0] >> 24) & MGENX_FLAG_CHECKSUM) != 0 &&
                                       buf_len >= MGENX_MIN_SIZE && ((w[0] >> 16) & 0xffu) == 2u);
        const bool needs_crc = flagged && (tcp ? (G.L >= 4) : fixed_ok(buf_len, w));
        const bool vec_crc = needs_crc && G.L >= 32;
        Hdr h;
        parse_header(rec, buf_len, want_ext, w, h);
        const bool crc_ok = !needs_crc || (vec_crc ? (tot == expect) : small_crc_ok(rec, G.L));
        store_hdr_q0(p.cols, G.idx, h, crc_ok, tcp);
      } else if (G.oob && q == 0) {
        store_oob_q0(p.cols, G.idx);
      }
    }

    if (KB > 0 && burst && held == (uint32_t)KH) flush();
    if (!has_next) break;
    // N's header: needed only after N's rows, so loaded after G's column stores
    pf = ldu128(hdr_ptr(N));
    expect = p.expect[N.live ? N.L : 0u];
    if (next_tile) {
      t_c = t_p;
      t_p = t_c + n_waves;
      off_c = off_p;
      len_c = len_p;
      src_c = src_p;
      place(t_p, off_p, len_p);
      p_ranked = false;
      k = 0;
    } else {
      k++;
    }
    G = N;
  }
  if (KB > 0 && burst && held) flush();
}

// ---------------------------------------------------------------------------------------
// Fixed-length records (fixed stride, one length L in [65, 1024]; BASELINE config 2 and
// the recvmmsg fixed-slot layout), software-pipelined across groups.  With one L every
// group has the same row geometry (V = ceil(L/64) rows, padded to the template's NR), so
// while a wave consumes row j of group g it reloads the register with row j of its next
// group g' = g + n_waves: the wave keeps ~NR x 1 KiB of loads in flight through its own
// LDS-bound CRC work and tail, at no register cost.  The header of g' is issued at the top
// of g (before g's reloads), so with in-order completion the CRC decision for g' waits for
// that header only, and row j of g' waits only for row j.
// Semantics are those of unpack_kernel<true> (same helpers, same column stores).
// MODE (diagnostic ablations, never the product path) is a bit mask:
//   1 = loads + XOR only (no LDS lookups)       2 = no tail (no decode, no stores)
//   4 = decode but no stores (kept alive)       8 = every store to the sink
//   16 = the other store flavour (rows: temporal; columns: non-temporal)
template <int NR, int MODE = 0, bool kRows = false, bool kAligned = false>
__global__ void __launch_bounds__(kUnpackThreads)
unpack_fixed_kernel(UnpackParams p, uint32_t expect) {
  constexpr bool kAblXor = (MODE & 1) != 0, kAblNoTail = (MODE & 2) != 0;
  constexpr bool kAblNoStore = (MODE & 4) != 0, kAblSink = (MODE & 8) != 0;
  constexpr bool kAblAltStore = (MODE & 16) != 0;
  constexpr bool kAblWrap = (MODE & 32) != 0;  // stores wrapped onto the first 16K records
  constexpr bool kAblWt = (MODE & 64) != 0;    // write-through (sc1) stores
  constexpr bool kAblNtLoad = (MODE & 128) != 0;  // non-temporal row loads
  constexpr bool kAblBurst = (MODE & 256) != 0;  // (with 4) dummy rows written at the end
  constexpr bool kAblBurstSeq = (MODE & 512) != 0;  // ... to one contiguous span per wave
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* rep = lds;
  uint32_t* fold = lds + kRepDwords;  // [A4 | A8 | A12 | A16 | A32 | A48]
  const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(rep);
  const TableRegs tab_regs = table_loads(p.tabs);  // staged below, after the first rows
  asm volatile("" ::: "memory");  // these loads issue before the rows (in-order vmcnt)

  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const uint32_t s1 = a64_s1((uint32_t)lane);
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(
      blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  const uint32_t n_groups = (p.n + 15u) >> 4;
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const uint32_t L = p.fixed_len;          // host guarantees 65 <= L <= 1024
  constexpr int V = NR;                    // rows: ceil(L / 64), 2..16 (host-checked)

  // Groups are dealt round-robin (wave w takes w, w + n_waves, ...): measured faster than
  // contiguous runs per wave (254 vs 241 us on config 2), whose 4096 concurrent 256-KiB
  // streams spread worse over the HBM channels.
  uint32_t g = wave_id;
  const uint32_t g_end = n_groups;

  // Geometry.  Every load is slab (uniform SGPR base) + 32-bit per-lane offset + constant:
  // the saddr form, one VGPR per address (host guarantees slab_bytes < 4 GiB).  A dead
  // lane (past the batch or outside the slab) reads at base offset 64 instead, inside the
  // slab (host guarantees slab_bytes >= 64 (NR + 1) + 16).
  auto rec_idx = [&](uint32_t gg) { return (gg << 4) + (uint32_t)(lane >> 2); };
  auto rec_ptr = [&](uint32_t i) { return p.slab + (uint64_t)i * p.stride; };
  auto is_live = [&](uint32_t i) {
    const uint64_t off = (uint64_t)i * p.stride;
    return i < p.n && off <= p.slab_bytes && L <= p.slab_bytes - off;
  };
  auto base_off = [&](bool lv, uint32_t i) { return lv ? i * (uint32_t)p.stride : 64u; };
  // lane's byte offset of row 0 (> -64; < 0 when row 0 starts before the record)
  const int pos0 = (int)L - 64 * V + 16 * q;
  auto ld = [&](uint32_t off, int imm) {
    if (kAblNtLoad) return ldnt128(p.slab + (uint64_t)off + imm);
    return ldu128(p.slab + (uint64_t)off + imm);
  };
  // row j of the record at boff (row 0 clamped to the record start).  Rows j >= 1 start at
  // boff + pos0 + 64 j with pos0 + 64 > 0: the 32-bit part must stay non-negative (it is
  // zero-extended), so the constant part is 64 (j - 1).
  auto ld_row = [&](uint32_t boff, int j) {
    return j == 0 ? ld(boff + (uint32_t)(pos0 > 0 ? pos0 : 0), 0)
                  : ld(boff + (uint32_t)(pos0 + 64), 64 * (j - 1));
  };
  auto ld_hdr = [&](uint32_t boff) { return ld(boff + 16u * (uint32_t)q, 0); };

  u32x4_t d[NR];
  // The tail is split in two so the aligned loop can decode a group's header as soon as its
  // row 0 arrives (then reload row 0 at once): decode() turns the quad's header into the
  // lane's store values, emit() applies the checksum verdict and stores.
  struct Out {
    uint32_t o[5];
  };
  auto decode = [&](const u32x4_t& pf, uint32_t idx, bool live) {
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = prefix_word(pf, j);
    const uint32_t w10 = prefix_word(pf, 10);
    const uint32_t D = w[5] >> 24;
    const uint32_t hw = (D == 4u) ? w[7] : w10;
    const uint32_t gi = (28u + D + (hw >> 24)) >> 2;  // GPS block word (fast layouts)
    const uint32_t g3 = (prefix_word(pf, 11) & (0u - (uint32_t)(gi == 8u))) |
                        (prefix_word(pf, 12) & (0u - (uint32_t)(gi == 9u))) |
                        (prefix_word(pf, 14) & (0u - (uint32_t)(gi == 11u))) |
                        (prefix_word(pf, 15) & (0u - (uint32_t)(gi == 12u)));
    // fast layout (mgenMsg.cpp:323-497 with every field word-aligned)
    uint32_t flow = bswap32(w[1]), seq = bswap32(w[2]), sec = bswap32(w[3]);
    uint32_t usec = bswap32(w[4]), dst4 = w[6];
    uint32_t msg_len = bswap16((uint16_t)(w[0] & 0xffffu));
    uint32_t dport = bswap16((uint16_t)(w[5] & 0xffffu));
    const uint32_t hlen = 44u + D + (hw >> 24);
    uint32_t plen = bswap16((uint16_t)(g3 >> 16));
    if (!(plen != 0 && hlen + plen <= L)) plen = 0;  // mgenMsg.cpp:488-497
    uint32_t flags = w[0] >> 24, err = 0, dtype = (w[5] >> 16) & 0xffu, dlen = D;
    uint32_t ptype = (g3 >> 8) & 0xffu, gps = g3 & 0xffu;
    // general layouts: quad lane 0 parses (with loads), then broadcasts to its quad
    const bool slow = live && !fast_layout(w[0], w[5], hw);
    if (__any(slow)) {
      Hdr h;
      if (slow && q == 0) parse_header(rec_ptr(idx), L, false, w, h);
      auto bc = [&](uint32_t& dst, uint32_t v) {
        v = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
        if (slow) dst = v;
      };
      bc(flow, h.flow); bc(seq, h.seq); bc(sec, h.sec); bc(usec, h.usec); bc(dst4, h.dst4);
      bc(msg_len, h.msg_len); bc(dport, h.dst_port); bc(plen, h.plen); bc(flags, h.flags);
      bc(err, h.err); bc(dtype, h.dst_type); bc(dlen, h.dst_len); bc(ptype, h.ptype);
      bc(gps, h.gps);
    }
    if (!live) {  // descriptor outside the slab (or past the batch end)
      flow = seq = sec = usec = dst4 = msg_len = dport = plen = flags = dtype = dlen = 0;
      ptype = gps = 0;
      err = MGENX_ERROR_OOB;
    }
    Out r;
    if (kRows) {  // mgenx_rec: lane q holds bytes 8q..8q+7 of its record
      r.o[0] = q == 0 ? flow : q == 1 ? sec : q == 2 ? dst4 : (plen | flags << 16 | err << 24);
      r.o[1] = q == 0 ? seq : q == 1 ? usec : q == 2 ? (msg_len | dport << 16)
                                                    : (dtype | dlen << 8 | ptype << 16 | gps << 24);
      r.o[2] = r.o[3] = r.o[4] = 0;
    } else {  // the lane's column values: u32 (column q), dst_addr4, u16, u8a, u8b
      r.o[0] = q == 0 ? flow : q == 1 ? seq : q == 2 ? sec : usec;
      r.o[1] = dst4;
      r.o[2] = q == 0 ? msg_len : q == 1 ? dport : plen;
      r.o[3] = q == 0 ? flags : q == 1 ? err : q == 2 ? dtype : dlen;
      r.o[4] = (q & 1) == 0 ? ptype : gps;
    }
    return r;
  };
  // Store one record per quad.  Every lane runs the same instructions: the four lanes of a
  // quad store four different columns (or the four 8-byte parts of a row), with no branch
  // around the stores.  (gfx950 counts stores in vmcnt: a store that might be skipped makes
  // LLVM's wait counts assume it was, so the next row wait would also wait for the store's
  // acknowledgement.)  Lanes past the batch end write to the sink.
  auto emit = [&](Out r, uint32_t idx, bool crc_bad) {
    if (crc_bad) {  // the caller's receive check (mgenTransport.cpp:971): err, TCP flag
      const uint32_t fl = tcp ? (uint32_t)MGENX_FLAG_CHECKSUM_ERROR : 0u;
      if (kRows) {
        if (q == 3) r.o[0] = (r.o[0] & 0x00ffffffu) | fl << 16 | (uint32_t)MGENX_ERROR_CHECKSUM << 24;
      } else {
        if (q == 0) r.o[3] |= fl;
        if (q == 1) r.o[3] = MGENX_ERROR_CHECKSUM;
      }
    }
    const bool in = idx < p.n && !kAblSink;
    const uint64_t sink = (uint64_t)p.sink + 4u * (uint32_t)lane;
    const uint32_t sidx = kAblWrap ? (idx & 0x3fffu) : idx;
    auto at = [&](uint64_t base, uint32_t size) { return in ? base + (uint64_t)sidx * size : sink; };
    const mgenx_cols& c = p.cols;
    if (kAblNoStore) {  // the tail's work without its stores (kept alive)
      const uint32_t all = r.o[0] ^ r.o[1] ^ r.o[2] ^ r.o[3] ^ r.o[4];
      if (all == 0x9E3779B9u) st_g32(sink, all);
      return;
    }
    if (kRows) {  // 16 records = 512 contiguous bytes per store instruction
      const uint64_t v = (uint64_t)r.o[1] << 32 | r.o[0];
      const uint64_t ra = in ? (uint64_t)p.cols.rows + (uint64_t)sidx * 32 + 8 * q
                             : (uint64_t)p.sink + 8u * lane;
      // non-temporal: the streamed output must not compete with the read stream in L2
      if (kAblWt) st_g64_wt(ra, v);
      else if (kAblAltStore) st_g64(ra, v);  // ablation: ordinary (temporal) row stores
      else st_g64_nt(ra, v);
      return;
    }
    const uint64_t u32 = pick4(q, (uint64_t)c.flow_id, (uint64_t)c.seq_num, (uint64_t)c.tx_sec,
                               (uint64_t)c.tx_usec);
    const uint64_t u16 = pick4(q, (uint64_t)c.msg_len, (uint64_t)c.dst_port,
                               (uint64_t)c.payload_len, (uint64_t)c.payload_len);
    const uint64_t u8a = pick4(q, (uint64_t)c.flags, (uint64_t)c.err, (uint64_t)c.dst_type,
                               (uint64_t)c.dst_len);
    const uint64_t u8b = pick4(q, (uint64_t)c.payload_type, (uint64_t)c.gps_status,
                               (uint64_t)c.payload_type, (uint64_t)c.gps_status);
    if (kAblWt) {  // ablation: write-through column stores
      st_g32_wt(at(u32, 4), r.o[0]);
      st_g32_wt(at((uint64_t)c.dst_addr4, 4), r.o[1]);
      st_g16_wt(at(u16, 2), r.o[2]);
      st_g8_wt(at(u8a, 1), r.o[3]);
      st_g8_wt(at(u8b, 1), r.o[4]);
      return;
    }
    if (kAblAltStore) {  // ablation: non-temporal column stores
      st_g32_nt(at(u32, 4), r.o[0]);
      st_g32_nt(at((uint64_t)c.dst_addr4, 4), r.o[1]);
      st_g16_nt(at(u16, 2), r.o[2]);
      st_g8_nt(at(u8a, 1), r.o[3]);
      st_g8_nt(at(u8b, 1), r.o[4]);
      return;
    }
    // u32: flow, seq, tx_sec, tx_usec (lane q -> column q); then dst_addr4 (all lanes);
    // u16: msg_len, dst_port, payload_len (lane 3 repeats lane 2's store);
    // u8: flags, err, dst_type, dst_len; then payload_type, gps_status (lanes 2,3 repeat)
    st_g32(at(u32, 4), r.o[0]);
    st_g32(at((uint64_t)c.dst_addr4, 4), r.o[1]);
    st_g16(at(u16, 2), r.o[2]);
    st_g8(at(u8a, 1), r.o[3]);
    st_g8(at(u8b, 1), r.o[4]);
  };
  // the receive-side CRC decision from words 0 and 5 (mgenTransport.cpp:960-963)
  auto decide = [&](const u32x4_t& pf, bool live) {
    const uint32_t w0 = prefix_word(pf, 0);
    const uint32_t w5 = prefix_word(pf, 5);
    const bool v2 = ((w0 >> 16) & 0xffu) == 2u;
    const bool flagged = force || ((((w0 >> 24) & MGENX_FLAG_CHECKSUM) != 0) && v2);
    const uint32_t t = (w5 >> 16) & 0xffu;
    return live && flagged && (tcp || (v2 && (t == 1u || t == 2u)));
  };

  u32x4_t pf;
  // The first group's rows go in flight before the tables are written to LDS (the staging's
  // load latency and LDS writes then overlap the first HBM round trip); a wave without a
  // group still loads (dummy rows) and joins the barrier.
  auto load_group = [&](uint32_t gg) {
    const uint32_t i = rec_idx(gg);
    const uint32_t boff = base_off(is_live(i), i);
    if (!kAligned) pf = ld_hdr(boff);
    // in row order (the loop's first wait is for row 0 alone)
#pragma unroll
    for (int j = 0; j < NR; j++) {
      d[j] = ld_row(boff, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  load_group(g);  // unconditional (a wave past the end reads the dummy rows at offset 64)
  table_writes(lds, tab_regs);
  // barrier without __syncthreads()'s fence: its vmcnt(0) would wait for the rows above
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (g >= g_end) return;
  bool first = true;
  while (g < g_end) {
    // ---- pipelined mode: rows of every group speculatively in flight one group ahead.
    // No load in this loop is conditional (a conditional reload makes LLVM copy the row
    // registers at the join, and a copy of an in-flight load drains the whole queue).
    uint32_t idx = rec_idx(g);
    bool live = is_live(idx);
    if (!first) {
      const uint32_t boff = base_off(live, idx);
      if (!kAligned) pf = ld_hdr(boff);
#pragma unroll
      for (int j = 0; j < NR; j++) {
        d[j] = ld_row(boff, j);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    first = false;
    // one pipelined group; the header registers alternate between two variables (the loop
    // is unrolled twice) so the next header never needs a register copy
    auto step = [&](const u32x4_t& pf_cur, u32x4_t& pf_nxt) {
      const uint32_t gn = g + n_waves;
      const bool has_next = gn < g_end;
      const uint32_t idx_n = rec_idx(has_next ? gn : g);
      const bool live_n = has_next && is_live(idx_n);
      // next group's header first (completes before any of its rows)
      const uint32_t boff_n = base_off(live_n, idx_n);
      if (!kAligned) pf_nxt = ld_hdr(boff_n);
      asm volatile("" ::: "memory");
      const u32x4_t hdr = kAligned ? d[0] : pf_cur;  // aligned: row 0 is the header
      const bool needs_crc = decide(hdr, live);
      const bool any = __any(needs_crc);
      // aligned: decode now, so row 0's registers are free for its reload
      Out early;
      if (kAligned && !kAblNoTail) early = decode(hdr, idx, live);

      // braid state word b = ha[b] ^ hb[b] (split so the next row folds in one XOR3)
      uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < NR - 1; j++) {
        u32x4_t x = d[j];
        if (j == 0) {
          const int s0 = -pos0;
          if (s0 > 0) {
            const u32x4_t zero = {0u, 0u, 0u, 0u};
            x = s0 < 16 ? shl_bytes(x, s0) : zero;
          }
        }
        const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
        uint32_t c4[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
          if (kAblXor)
            c4[b] = (ha[b] << 1) ^ xw[b];
          else
            c4[b] = xor3(ha[b], hb[b], xw[b]);
        }
        // row j of g is dead now: reload its register for g' (same physical register, so
        // no loop-carried copy -- a copy of an in-flight load would drain the queue)
        __builtin_amdgcn_sched_barrier(0);
        d[j] = ld_row(boff_n, j);
        __builtin_amdgcn_sched_barrier(0);
        if (kAblXor) {
#pragma unroll
          for (int b = 0; b < 4; b++) ha[b] = c4[b];
          continue;
        }
#pragma unroll
        for (int b = 0; b < 4; b++) a64_parts(ldsb, c4[b], s1, ha[b], hb[b]);
      }
      // final row (V >= 2, so never row 0): the big-endian trailer goes to stream order
      const u32x4_t xf = d[NR - 1];
      uint32_t f0 = xor3(ha[0], hb[0], xf.x), f1 = xor3(ha[1], hb[1], xf.y);
      uint32_t f2 = xor3(ha[2], hb[2], xf.z);
      uint32_t f3 = xor3(ha[3], hb[3], q == 3 ? bswap32(xf.w) : xf.w);
      // opaque: later index math must not reach back to the row registers (which would keep
      // them live across their reload and cost a loop-carried copy of the in-flight load)
      asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
      __builtin_amdgcn_sched_barrier(0);
      d[NR - 1] = ld_row(boff_n, NR - 1);
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t v = shift_tab(fold + 3 * 1024, f0) ^ shift_tab(fold + 2 * 1024, f1) ^
                         shift_tab(fold + 1 * 1024, f2) ^ shift_tab(fold, f3);
      const uint32_t* lt = fold + (q == 0 ? 5 : (q == 1 ? 4 : 3)) * 1024;  // A48/A32/A16
      uint32_t s = (q == 3) ? v : shift_tab(lt, v);
      s ^= __shfl_xor(s, 1);
      s ^= __shfl_xor(s, 2);
      if (kAblNoTail) {
        if (s == 0x9E3779B9u && lane == 0) p.cols.err[idx] = (uint8_t)needs_crc;  // keep alive
      } else {
        const Out r = kAligned ? early : decode(hdr, idx, live);
        emit(r, idx, needs_crc && s != expect);
      }
      // keep the row base of g' alive past its last reload: otherwise the register allocator
      // gives that load the dying address register as destination, and the loop needs a copy
      // of the in-flight row at its back edge (a full drain)
      asm volatile("" ::"v"(boff_n + (uint32_t)(pos0 + 64)));
      g = gn;
      idx = idx_n;
      live = live_n;
      // a group without any checksummed record: stop streaming bodies (the rows of g' in
      // flight are simply overwritten later)
      return has_next && any;
    };
    u32x4_t pf2;
    if (kAligned) {
      while (step(pf, pf2)) {
      }
    } else {
      for (;;) {
        if (!step(pf, pf2)) break;
        if (!step(pf2, pf)) break;
      }
    }
    // ---- header-only mode: header first, bodies only for groups that need the CRC
    for (; g < g_end; g += n_waves) {
      const uint32_t i = rec_idx(g);
      const bool lv = is_live(i);
      const u32x4_t ph = ld_hdr(base_off(lv, i));
      const bool nc = decide(ph, lv);
      if (__any(nc)) break;  // back to pipelined mode at this group
      emit(decode(ph, i, lv), i, false);
    }
  }
  if (kAblBurst) {  // every group's row stores in one burst after the wave's last group
    uint32_t k = 0;
    for (uint32_t gg = wave_id; gg < g_end; gg += n_waves, k++) {
      const uint32_t i = rec_idx(gg);
      const uint64_t seq = (uint64_t)wave_id * 8192u + k * 512u + 8u * (uint32_t)lane;
      const uint64_t a = (uint64_t)p.cols.rows + (kAblBurstSeq ? seq : (uint64_t)i * 32 + 8 * q);
      if (i < p.n) {
        if (kAblWt) st_g64_wt(a, (uint64_t)gg);
        else if (kAblAltStore) st_g64(a, (uint64_t)gg);
        else st_g64_nt(a, (uint64_t)gg);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Aligned fixed-length records of NR = 8 or 16 rows (512 / 1024 B) with row output -- the
// headline layout -- reading and writing in separate phases.  On the MI355X boxes where
// mixing the 32-B row stores into the 1 GiB read stream costs most (config 2): the read
// pattern alone takes 168 us, with the row stores interleaved 201 us.  So each wave keeps
// the rows of its last K = 16 groups in registers (a shift register, 2 dwords per group and
// lane) and stores them in one burst every K groups and at its end: for config 2 (16 groups
// per wave) one burst, after the wave's reads (measured 0.194 ms against 0.215 ms for the
// interleaved kernel on the same box; K = 12 with two bursts: 0.204 ms).  The registers come
// from a shorter load ring: RS = 4 rows in flight per wave (row r + 4 of the wave's row stream
// is loaded as row r is consumed; 4 KiB per wave, 64 KiB per CU).
// Semantics are those of unpack_fixed_kernel<NR, 0, true, true>.
template <int NR, int RS = 4, int K = 16>
__global__ void __launch_bounds__(kUnpackThreads)
unpack_fixed_ring_kernel(UnpackParams p, uint32_t expect) {
  static_assert(NR == 8 || NR == 16, "ring kernel: 512- or 1024-byte records");
  static_assert(NR % RS == 0, "the ring divides the record's rows");
  // RS: rows in flight per wave; K: groups of row output held per wave before a burst
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t* fold = lds + kRepDwords;  // [A4 | A8 | A12 | A16 | A32 | A48]
  const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(lds);
  const TableRegs tab_regs = table_loads(p.tabs);
  asm volatile("" ::: "memory");

  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const uint32_t s1 = a64_s1((uint32_t)lane);
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(
      blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  const uint32_t g_end = (p.n + 15u) >> 4;
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const uint32_t L = p.fixed_len;  // == 64 * NR (host-checked)

  auto rec_idx = [&](uint32_t gg) { return (gg << 4) + (uint32_t)(lane >> 2); };
  auto is_live = [&](uint32_t i) {
    const uint64_t off = (uint64_t)i * p.stride;
    return i < p.n && off <= p.slab_bytes && L <= p.slab_bytes - off;
  };
  // lane's row base (32-bit offset, saddr form); a dead lane reads inside the slab at 64
  auto row_base = [&](uint32_t gg) {
    const uint32_t i = rec_idx(gg);
    return (is_live(i) ? i * (uint32_t)p.stride : 64u) + 16u * (uint32_t)q;
  };
  auto ld = [&](uint32_t base, int j) { return ldu128(p.slab + (uint64_t)base + 64 * j); };
  auto decide = [&](const u32x4_t& pf, bool live) {
    const uint32_t w0 = prefix_word(pf, 0);
    const uint32_t w5 = prefix_word(pf, 5);
    const bool v2 = ((w0 >> 16) & 0xffu) == 2u;
    const bool flagged = force || ((((w0 >> 24) & MGENX_FLAG_CHECKSUM) != 0) && v2);
    const uint32_t t = (w5 >> 16) & 0xffu;
    return live && flagged && (tcp || (v2 && (t == 1u || t == 2u)));
  };
  // the quad's 32-B mgenx_rec: lane q holds bytes 8q .. 8q+7 (as unpack_fixed_kernel)
  auto decode = [&](const u32x4_t& pf, uint32_t idx, bool live, uint32_t& o0, uint32_t& o1) {
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = prefix_word(pf, j);
    const uint32_t w10 = prefix_word(pf, 10);
    const uint32_t D = w[5] >> 24;
    const uint32_t hw = (D == 4u) ? w[7] : w10;
    const uint32_t gi = (28u + D + (hw >> 24)) >> 2;
    const uint32_t g3 = (prefix_word(pf, 11) & (0u - (uint32_t)(gi == 8u))) |
                        (prefix_word(pf, 12) & (0u - (uint32_t)(gi == 9u))) |
                        (prefix_word(pf, 14) & (0u - (uint32_t)(gi == 11u))) |
                        (prefix_word(pf, 15) & (0u - (uint32_t)(gi == 12u)));
    uint32_t flow = bswap32(w[1]), seq = bswap32(w[2]), sec = bswap32(w[3]);
    uint32_t usec = bswap32(w[4]), dst4 = w[6];
    uint32_t msg_len = bswap16((uint16_t)(w[0] & 0xffffu));
    uint32_t dport = bswap16((uint16_t)(w[5] & 0xffffu));
    const uint32_t hlen = 44u + D + (hw >> 24);
    uint32_t plen = bswap16((uint16_t)(g3 >> 16));
    if (!(plen != 0 && hlen + plen <= L)) plen = 0;  // mgenMsg.cpp:488-497
    uint32_t flags = w[0] >> 24, err = 0, dtype = (w[5] >> 16) & 0xffu, dlen = D;
    uint32_t ptype = (g3 >> 8) & 0xffu, gps = g3 & 0xffu;
    const bool slow = live && !fast_layout(w[0], w[5], hw);
    if (__any(slow)) {
      Hdr h;
      if (slow && q == 0) parse_header(p.slab + (uint64_t)idx * p.stride, L, false, w, h);
      auto bc = [&](uint32_t& dst, uint32_t v) {
        v = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
        if (slow) dst = v;
      };
      bc(flow, h.flow); bc(seq, h.seq); bc(sec, h.sec); bc(usec, h.usec); bc(dst4, h.dst4);
      bc(msg_len, h.msg_len); bc(dport, h.dst_port); bc(plen, h.plen); bc(flags, h.flags);
      bc(err, h.err); bc(dtype, h.dst_type); bc(dlen, h.dst_len); bc(ptype, h.ptype);
      bc(gps, h.gps);
    }
    if (!live) {
      flow = seq = sec = usec = dst4 = msg_len = dport = plen = flags = dtype = dlen = 0;
      ptype = gps = 0;
      err = MGENX_ERROR_OOB;
    }
    o0 = q == 0 ? flow : q == 1 ? sec : q == 2 ? dst4 : (plen | flags << 16 | err << 24);
    o1 = q == 0 ? seq : q == 1 ? usec : q == 2 ? (msg_len | dport << 16)
                                              : (dtype | dlen << 8 | ptype << 16 | gps << 24);
  };
  // the caller's receive check (mgenTransport.cpp:971): ERROR_CHECKSUM (+ TCP flag) in word 6
  auto verdict = [&](uint32_t& o0, bool crc_bad) {
    const uint32_t fl = tcp ? (uint32_t)MGENX_FLAG_CHECKSUM_ERROR : 0u;
    if (crc_bad && q == 3) o0 = (o0 & 0x00ffffffu) | fl << 16 | (uint32_t)MGENX_ERROR_CHECKSUM << 24;
  };

  // ---- output shift register: buf[K-1] = the newest group, `held` groups pending
  uint32_t b0[K], b1[K];
#pragma unroll
  for (int k = 0; k < K; k++) b0[k] = b1[k] = 0u;
  uint32_t held = 0, last_g = 0;
  auto push = [&](uint32_t o0, uint32_t o1, uint32_t gg) {
#pragma unroll
    for (int k = 0; k < K - 1; k++) {
      b0[k] = b0[k + 1];
      b1[k] = b1[k + 1];
    }
    b0[K - 1] = o0;
    b1[K - 1] = o1;
    held++;
    last_g = gg;
  };
  auto flush = [&]() {  // buf[k] belongs to group last_g - (K - 1 - k) * n_waves
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t back = (uint32_t)(K - 1 - k);
      const uint32_t gg = last_g - back * n_waves;
      const uint32_t idx = rec_idx(gg);
      const bool in = back < held && idx < p.n;
      const uint64_t v = (uint64_t)b1[k] << 32 | b0[k];
      if (back < held)  // wave-uniform
        st_g64_nt(in ? (uint64_t)p.cols.rows + (uint64_t)idx * 32 + 8 * q
                     : (uint64_t)p.sink + 8u * (uint32_t)lane, v);
    }
    held = 0;
  };

  u32x4_t d[RS];
  uint32_t g = wave_id;
  const uint32_t base0 = row_base(g < g_end ? g : 0u);
#pragma unroll
  for (int j = 0; j < RS; j++) {
    d[j] = ld(base0, j);
    __builtin_amdgcn_sched_barrier(0);
  }
  table_writes(lds, tab_regs);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (g >= g_end) return;

  bool pipelined = true;
  while (g < g_end) {
    const uint32_t gn = g + n_waves;
    const bool has_next = gn < g_end;
    const uint32_t idx = rec_idx(g);
    const bool live = is_live(idx);
    if (pipelined) {
      const uint32_t base = row_base(g), base_n = row_base(has_next ? gn : g);
      const u32x4_t hdr = d[0];  // row 0 = the 64-byte header prefix (aligned)
      const bool needs_crc = decide(hdr, live);
      const bool any = __any(needs_crc);
      uint32_t o0, o1;
      decode(hdr, idx, live, o0, o1);
      uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < NR - 1; j++) {
        const u32x4_t x = d[j % RS];
        const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
        uint32_t c4[4];
#pragma unroll
        for (int b = 0; b < 4; b++) c4[b] = xor3(ha[b], hb[b], xw[b]);
        __builtin_amdgcn_sched_barrier(0);
        // row j + RS of the stream: this group's row, or the next group's
        d[j % RS] = (j + RS < NR) ? ld(base, j + RS) : ld(base_n, j + RS - NR);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b = 0; b < 4; b++) a64_parts(ldsb, c4[b], s1, ha[b], hb[b]);
      }
      const u32x4_t xf = d[(NR - 1) % RS];
      uint32_t f0 = xor3(ha[0], hb[0], xf.x), f1 = xor3(ha[1], hb[1], xf.y);
      uint32_t f2 = xor3(ha[2], hb[2], xf.z);
      uint32_t f3 = xor3(ha[3], hb[3], q == 3 ? bswap32(xf.w) : xf.w);
      asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
      __builtin_amdgcn_sched_barrier(0);
      d[(NR - 1) % RS] = ld(base_n, NR - 1 + RS - NR);
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t v = shift_tab(fold + 3 * 1024, f0) ^ shift_tab(fold + 2 * 1024, f1) ^
                         shift_tab(fold + 1 * 1024, f2) ^ shift_tab(fold, f3);
      const uint32_t* lt = fold + (q == 0 ? 5 : (q == 1 ? 4 : 3)) * 1024;  // A48/A32/A16
      uint32_t sum = (q == 3) ? v : shift_tab(lt, v);
      sum ^= __shfl_xor(sum, 1);
      sum ^= __shfl_xor(sum, 2);
      verdict(o0, needs_crc && sum != expect);
      push(o0, o1, g);
      asm volatile("" ::"v"(base_n));
      pipelined = has_next && any;  // a group without checksummed records: header-only
    } else {
      // header-only mode: header first, body only when a record needs the CRC
      const u32x4_t ph = ld(row_base(g), 0);
      if (__any(decide(ph, live))) {
        // back to the pipelined mode at this group: its first RS rows, then re-run it
        const uint32_t bb = row_base(g);
#pragma unroll
        for (int j = 0; j < RS; j++) d[j] = ld(bb, j);
        pipelined = true;
        continue;
      }
      uint32_t o0, o1;
      decode(ph, idx, live, o0, o1);
      push(o0, o1, g);
    }
    if (held == (uint32_t)K) flush();
    g = gn;
  }
  if (held) flush();
}

// ---------------------------------------------------------------------------------------
// Long records (TCP streams: config 5's 16-KiB records), one WAVE per record.  The kernels
// above give a record to a quad, so a wave's load instruction reads 64 bytes from each of 16
// records -- 16 KiB apart here.  This one covers the record with 1-KiB rows aligned to its
// end; quad k takes bytes [64k, 64k + 64) of every row, so each load instruction reads 1 KiB
// contiguously.  The braid CRC is the quad kernels' with A_1024 in place of A_64 (staged in
// LDS replicated exactly as A_64 is above, so the same one-perm-per-lookup addressing); at the
// record end a lane folds its four words (A_4, Horner), the quad its lanes (A_16, A_32) and the
// wave its quads (A_64 .. A_512), and the residue is compared with expect[L].
// Rows stream through 8 registers: consuming row j of the wave's current 8-row block reloads
// that register with row j of its next block (the record's next block, or the first block of
// the wave's next record), so 8 KiB stay in flight per wave.  A record is front-padded with
// zero rows to whole blocks (a zero braid state stays zero through them).  Quad 0 (lanes 0-3)
// loads and decodes the header as the general kernel does, under the same receive rules
// (TCP: Unpack sees min(L, 8192) bytes, mgenTransport.cpp:2016-2031; the CRC covers L - 4).
constexpr int kLongNB = 8;                                  // rows per block
constexpr uint32_t kLongMin = 4096;                         // mean record length that picks it
constexpr int kLongFold = 7;                                // A4 A16 A32 A64 A128 A256 A512
constexpr size_t kLongLdsBytes = (size_t)(kRepDwords + kLongFold * kSmallTabDwords) * 4u;
static_assert(kLongLdsBytes <= 160u * 1024u, "long-record tables fit the CU's LDS");

template <int NB = kLongNB, int NT = kUnpackThreads>
__global__ void __launch_bounds__(NT) unpack_long_kernel(UnpackParams p) {
  static_assert(1024 % NT == 0, "table staging: whole passes");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t* fold = lds + kRepDwords;
  const uint32_t *fA4 = fold, *fA16 = fold + 1024, *fA32 = fold + 2048, *fA64 = fold + 3072,
                 *fA128 = fold + 4096, *fA256 = fold + 5120, *fA512 = fold + 6144;
  const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(lds);
  // this thread's table entries: A_1024 (replicated) and the fold operators
  constexpr int kFoldIdx[kLongFold] = {kTabA4, kTabA16, kTabA32, kTabA64, kTabA128, kTabA256,
                                       kTabA512};
  const uint32_t a1024 = p.tabs[kTabA1024 * 1024 + threadIdx.x];
  uint32_t fr[kLongFold];
#pragma unroll
  for (int k = 0; k < kLongFold; k++) fr[k] = p.tabs[kFoldIdx[k] * 1024 + threadIdx.x];
  constexpr int kNB = NB;

  const int lane = threadIdx.x & 63;
  const int q = lane & 3, quad = lane >> 2;
  const uint32_t s1 = a64_s1((uint32_t)lane);
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(
      blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  const bool force = (p.opts & MGENX_OPT_CHECKSUM_FORCE) != 0;
  const bool tcp = (p.opts & MGENX_OPT_TCP) != 0;
  const bool want_ext = p.cols.dst_addr || p.cols.host_addr;
  const mgenx_cols& cc = p.cols;
  const bool any_ext = cc.hdr_len || cc.payload_off || cc.host_port || cc.host_type ||
                       cc.host_len || cc.lat_raw || cc.lon_raw || cc.alt || cc.dst_addr ||
                       cc.host_addr || cc.decoded;
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.tabs);

  // a record's placement (wave-uniform)
  struct Rec {
    uint32_t idx;   // record index (>= n: none)
    uint64_t off;
    uint32_t L;
    bool live;      // inside the slab
    bool rows;      // its CRC runs on the rows (>= 32 bytes; shorter ones bit by bit)
    uint32_t nb;    // blocks (>= 1)
    int64_t r0;     // position of virtual row 0 (record-relative, <= 0)
  };
  auto place = [&](uint32_t ri) {
    Rec r;
    r.idx = ri;
    r.off = 0;
    r.L = 0;
    if (ri < p.n) {
      r.off = p.rec_off ? p.rec_off[ri] : (uint64_t)ri * p.stride;
      r.L = p.rec_len ? p.rec_len[ri] : p.fixed_len;
    }
    const bool oob = ri < p.n && (r.L > 65535u || r.off > p.slab_bytes || r.L > p.slab_bytes - r.off);
    r.live = ri < p.n && !oob;
    r.rows = r.live && r.L >= 32u;
    const uint32_t R = r.rows ? (r.L + 1023u) >> 10 : 0u;
    r.nb = R ? (R + kNB - 1u) / kNB : 1u;
    r.r0 = (int64_t)(r.rows ? r.L : 0u) - 1024 * (int64_t)(kNB * r.nb);
    return r;
  };
  // row j of block b of record r, this lane's 16 bytes: the address (clamped into the record;
  // lanes before its start are zeroed at consumption)
  auto row_pos = [&](const Rec& r, uint32_t b, int j) {
    return r.r0 + 1024 * (int64_t)(kNB * b + (uint32_t)j) + 16 * lane;
  };
  auto ld_row = [&](const Rec& r, uint32_t b, int j) {
    const int64_t pos = row_pos(r, b, j);
    return ldu128(r.rows && pos >= 0 ? p.slab + r.off + (uint64_t)pos
                                     : (r.rows && pos > -16 ? p.slab + r.off : dummy));
  };

  Rec cur = place(wave_id);
  uint32_t b = 0;
  u32x4_t d[kNB];
#pragma unroll
  for (int j = 0; j < kNB; j++) {
    d[j] = ld_row(cur, 0, j);
    __builtin_amdgcn_sched_barrier(0);
  }
  // stage the tables behind the first block's loads (fence-free barrier: lgkmcnt only)
  {
    typedef __attribute__((address_space(3))) u32x4_t lds_u32x4_t;
    for (uint32_t e = threadIdx.x; e < 1024u; e += NT) {
      const uint32_t k = e >> 8, val = e & 255u;
      const uint32_t av = e == threadIdx.x ? a1024 : p.tabs[kTabA1024 * 1024 + e];
      const u32x4_t s = {av, av, av, av};
      lds_u32x4_t* dst = (lds_u32x4_t*)((k >> 1) * 65536u + val * 256u + (k & 1u) * 128u);
#pragma unroll
      for (int c = 0; c < kRep / 4; c++) dst[c] = s;
      uint32_t* fl = lds + kRepDwords;
#pragma unroll
      for (int k2 = 0; k2 < kLongFold; k2++)
        fl[k2 * 1024 + e] = e == threadIdx.x ? fr[k2] : p.tabs[kFoldIdx[k2] * 1024 + e];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (cur.idx >= p.n) return;

  uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
  u32x4_t pf = {0u, 0u, 0u, 0u}, xs = {0u, 0u, 0u, 0u};
  uint32_t expect = 0;
  // header prefix (quad 0), expect[L], and the record's first 16 bytes shifted up to where
  // they sit in the lane whose chunk straddles the record start (L % 16 != 0)
  auto start_record = [&](const Rec& r) {
    pf = ldu128((r.live && quad == 0 && r.L >= 16u * (q + 1)) ? p.slab + r.off + 16 * q : dummy);
    expect = p.expect[r.live ? r.L : 0u];
    const int s = (int)(16u - (r.L & 15u)) & 15;
    const u32x4_t x0 = ldu128(r.rows ? p.slab + r.off : dummy);
    xs = s ? shl_bytes(x0, s) : x0;
  };
  start_record(cur);
  while (true) {
    // the next block of the wave's stream
    const bool last = b + 1u == cur.nb;
    const Rec nx = last ? place(cur.idx + n_waves) : cur;
    const uint32_t bn = last ? 0u : b + 1u;
    const bool has_next = nx.idx < p.n;
    // the first real row may start before the record (or the block is padding): zero the
    // lanes' bytes before the record start (uniform test: rows at or past the start need none)
    const bool fix = cur.r0 + 1024 * (int64_t)(kNB * b) < 0;
    u32x4_t xf = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < kNB; j++) {
      u32x4_t x = d[j];
      if (fix) {  // lanes before the record: zeros; the straddling lane: xs
        const int64_t pos = row_pos(cur, b, j);
        const bool zero = pos <= -16, strad = pos < 0 && pos > -16;
        x.x = zero ? 0u : (strad ? xs.x : x.x);
        x.y = zero ? 0u : (strad ? xs.y : x.y);
        x.z = zero ? 0u : (strad ? xs.z : x.z);
        x.w = zero ? 0u : (strad ? xs.w : x.w);
      }
      if (last && j == kNB - 1) {
        // the record's final row: folded below, not advanced
        uint32_t f0 = xor3(ha[0], hb[0], x.x), f1 = xor3(ha[1], hb[1], x.y);
        uint32_t f2 = xor3(ha[2], hb[2], x.z);
        uint32_t f3 = xor3(ha[3], hb[3], lane == 63 ? bswap32(x.w) : x.w);
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
        xf = u32x4_t{f0, f1, f2, f3};
        __builtin_amdgcn_sched_barrier(0);
        d[j] = has_next ? ld_row(nx, bn, j) : ldu128(dummy);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
        uint32_t c4[4];
#pragma unroll
        for (int k = 0; k < 4; k++) c4[k] = xor3(ha[k], hb[k], xw[k]);
        __builtin_amdgcn_sched_barrier(0);
        d[j] = has_next ? ld_row(nx, bn, j) : ldu128(dummy);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 4; k++) a64_parts(ldsb, c4[k], s1, ha[k], hb[k]);
      }
    }
    if (last) {
      // ---- the record's CRC residue: lane, quad and wave folds ----
      uint32_t v = shift_tab(fA4, xf.x) ^ xf.y;
      v = shift_tab(fA4, v) ^ xf.z;
      v = shift_tab(fA4, v) ^ xf.w;
      v = shift_tab(fA4, v);  // at the end of the lane's 16 bytes
      v = (q & 1) ? v : shift_tab(fA16, v);
      v ^= __shfl_xor(v, 1);
      v = (q & 2) ? v : shift_tab(fA32, v);
      v ^= __shfl_xor(v, 2);  // at the end of the quad's 64 bytes
      v = (quad & 1) ? v : shift_tab(fA64, v);
      v ^= __shfl_xor(v, 4);
      v = (quad & 2) ? v : shift_tab(fA128, v);
      v ^= __shfl_xor(v, 8);
      v = (quad & 4) ? v : shift_tab(fA256, v);
      v ^= __shfl_xor(v, 16);
      v = (quad & 8) ? v : shift_tab(fA512, v);
      v ^= __shfl_xor(v, 32);  // at the record end, in every lane
      const uint32_t tot = v;
      // ---- the header (quad 0) and the outputs, as unpack_kernel's group ----
      const uint32_t L = cur.L;
      const bool live = cur.live;
      const uint8_t* rec = p.slab + cur.off;
      const uint32_t buf_len = tcp ? min(L, (uint32_t)MGENX_TX_BUFFER_SIZE) : L;
      uint32_t pw[16];
      quad_bcast<0>(pf, pw);
      quad_bcast<1>(pf, pw);
      quad_bcast<2>(pf, pw);
      quad_bcast<3>(pf, pw);
      if (lane == 0) {
        if (live) {
          uint32_t w[8];
          const bool pfx = L >= 32;
          if (pfx) {
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] = pw[j];
          } else if (L >= MGENX_MIN_SIZE) {
            load_fixed(rec, buf_len, w);
          } else {
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] = 0;
          }
          const bool flagged = force || (((w[0] >> 24) & MGENX_FLAG_CHECKSUM) != 0 &&
                                         buf_len >= MGENX_MIN_SIZE && ((w[0] >> 16) & 0xffu) == 2u);
          const bool needs_crc = flagged && (tcp ? (L >= 4) : fixed_ok(buf_len, w));
          const bool crc_ok = !needs_crc || (cur.rows ? tot == expect : small_crc_ok(rec, L));
          if (buf_len >= 64 && fast_layout(pw[0], pw[5], (pw[5] >> 24) == 4u ? pw[7] : pw[10])) {
            store_fast_q0(p.cols, cur.idx, pw, buf_len, crc_ok, tcp);
            if (any_ext) store_fast_ext(p.cols, cur.idx, [&](int k) { return pw[k]; }, buf_len, true);
          } else {
            Hdr h;
            parse_header(rec, buf_len, want_ext, w, h);
            store_hdr_q0(p.cols, cur.idx, h, crc_ok, tcp);
          }
        } else {
          store_oob_q0(p.cols, cur.idx);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; k++) ha[k] = hb[k] = 0u;
      if (!has_next) break;
      start_record(nx);
    }
    cur = nx;
    b = bn;
  }
}

template <typename K>
static hipError_t launch_lds(K kernel, const UnpackParams& p, int grid, hipStream_t stream) {
  hipError_t e = set_max_lds((const void*)kernel, (int)kUnpackLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kUnpackThreads), kUnpackLdsBytes, stream, p);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_mode(const UnpackParams& p, int grid, hipStream_t stream) {
  return launch_lds(unpack_kernel<true, MODE>, p, grid, stream);
}

template <int NT = kUnpackThreads, int KB = 4, int MODE = 0>
static hipError_t launch_var(const UnpackParams& p, int grid, hipStream_t stream) {
  hipError_t e = set_max_lds((const void*)unpack_var_kernel<NT, KB, MODE>, (int)kUnpackLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((unpack_var_kernel<NT, KB, MODE>), dim3(grid), dim3(NT), kUnpackLdsBytes,
                     stream, p);
  return hipGetLastError();
}

template <int NB = kLongNB, int NT = kUnpackThreads>
static hipError_t launch_long_t(const UnpackParams& p, int grid, hipStream_t stream) {
  hipError_t e = set_max_lds((const void*)unpack_long_kernel<NB, NT>, (int)kLongLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((unpack_long_kernel<NB, NT>), dim3(grid), dim3(NT), kLongLdsBytes, stream, p);
  return hipGetLastError();
}
static hipError_t launch_long(const UnpackParams& p, int grid, hipStream_t stream) {
#if MGENX_DIAG
  // (diagnostics) shapes: rows per block x threads per workgroup
  switch (p.variant) {
    case 40: return launch_long_t<16, 512>(p, grid, stream);
    case 41: return launch_long_t<8, 512>(p, grid, stream);
    case 42: return launch_long_t<4, 1024>(p, grid, stream);
    case 43: return launch_long_t<12, 512>(p, grid, stream);
    case 44: return launch_long_t<2, 1024>(p, grid, stream);
    case 45: return launch_long_t<16, 1024>(p, grid, stream);
    default: break;
  }
#endif
  return launch_long_t<>(p, grid, stream);
}

#if MGENX_DIAG
static hipError_t launch_sorted(const UnpackParams& p, int grid, hipStream_t stream) {
  return launch_lds(unpack_kernel<true, 0, true>, p, grid, stream);
}
#endif

template <int NR, int MODE = 0, bool kRows = false, bool kAligned = false>
static hipError_t launch_fixed(const UnpackParams& p, int grid, hipStream_t stream) {
  hipError_t e = set_max_lds((const void*)unpack_fixed_kernel<NR, MODE, kRows, kAligned>, (int)kUnpackLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((unpack_fixed_kernel<NR, MODE, kRows, kAligned>), dim3(grid),
                     dim3(kUnpackThreads), kUnpackLdsBytes, stream, p, p.expect_fixed);
  return hipGetLastError();
}

template <int NR, int RS = 4, int K = 16>
static hipError_t launch_ring(const UnpackParams& p, int grid, hipStream_t stream) {
  hipError_t e = set_max_lds((const void*)unpack_fixed_ring_kernel<NR, RS, K>, (int)kUnpackLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((unpack_fixed_ring_kernel<NR, RS, K>), dim3(grid), dim3(kUnpackThreads),
                     kUnpackLdsBytes, stream, p, p.expect_fixed);
  return hipGetLastError();
}

typedef hipError_t (*fixed_launcher)(const UnpackParams&, int, hipStream_t);
#define MGENX_FIXED_TABLE(R)                                                              \
  {nullptr, nullptr, launch_fixed<2, 0, R>, launch_fixed<3, 0, R>, launch_fixed<4, 0, R>,    \
   launch_fixed<5, 0, R>, launch_fixed<6, 0, R>, launch_fixed<7, 0, R>, launch_fixed<8, 0, R>, \
   launch_fixed<9, 0, R>, launch_fixed<10, 0, R>, launch_fixed<11, 0, R>,                    \
   launch_fixed<12, 0, R>, launch_fixed<13, 0, R>, launch_fixed<14, 0, R>,                   \
   launch_fixed<15, 0, R>, launch_fixed<16, 0, R>}
static const fixed_launcher kFixedLaunch[17] = MGENX_FIXED_TABLE(false);
static const fixed_launcher kFixedLaunchRows[17] = MGENX_FIXED_TABLE(true);
#undef MGENX_FIXED_TABLE

hipError_t launch_unpack(const UnpackParams& p, int grid, hipStream_t stream, int* which) {
  const int unpack_variant = p.variant;
  *which = MGENX_UNPACK_K_OTHER;
  if (p.opts & MGENX_OPT_SKIP_CRC) {
    *which = MGENX_UNPACK_K_HEADER;
    hipLaunchKernelGGL((unpack_kernel<false>), dim3(grid), dim3(kUnpackThreads), 0, stream, p);
    return hipGetLastError();
  }
  // fixed stride + one length in [65, 1024] + core columns: the pipelined kernel
  const mgenx_cols& c = p.cols;
  const bool ext = c.hdr_len || c.payload_off || c.host_port || c.host_type || c.host_len ||
                   c.lat_raw || c.lon_raw || c.alt || c.dst_addr || c.host_addr || c.decoded;
  const uint32_t nr = (p.fixed_len + 63) / 64;
  const bool fixed = !p.rec_off && !p.rec_len && p.fixed_len >= 65 && p.fixed_len <= 1024 &&
                     p.stride > 0 && p.n <= 0xFFFFFFF0u && !ext &&
                     p.slab_bytes < 0xFFFF0000ull && p.slab_bytes >= 64ull * (nr + 1) + 16 &&
                     p.slab_bytes >= p.fixed_len;
  if (unpack_variant == 0 && fixed) {
    // 256 / 512 / 1024-byte records: the aligned variant (header = row 0)
    *which = (c.rows && (p.fixed_len == 512 || p.fixed_len == 1024)) ? MGENX_UNPACK_K_FIXED_RING
                                                                    : MGENX_UNPACK_K_FIXED;
    switch (p.fixed_len) {
      case 256: return c.rows ? launch_fixed<4, 0, true, true>(p, grid, stream)
                              : launch_fixed<4, 0, false, true>(p, grid, stream);
      case 512: return c.rows ? launch_ring<8>(p, grid, stream)
                              : launch_fixed<8, 0, false, true>(p, grid, stream);
      case 1024: return c.rows ? launch_ring<16>(p, grid, stream)
                               : launch_fixed<16, 0, false, true>(p, grid, stream);
      default: break;
    }
    return (c.rows ? kFixedLaunchRows : kFixedLaunch)[(p.fixed_len + 63) / 64](p, grid, stream);
  }
#if MGENX_DIAG
  // ablation 13: the interleaved-store aligned kernel (before the ring kernel)
  if (unpack_variant == 13 && fixed && p.fixed_len == 1024)
    return c.rows ? launch_fixed<16, 0, true, true>(p, grid, stream)
                  : launch_fixed<16, 0, false, true>(p, grid, stream);
  // ring-kernel shapes (rows in flight, groups held): 14 = (8, 12), 15 = (8, 8), 16 = (4, 12)
  if (unpack_variant >= 14 && unpack_variant <= 16 && fixed && p.fixed_len == 1024 && c.rows) {
    if (unpack_variant == 14) return launch_ring<16, 8, 12>(p, grid, stream);
    if (unpack_variant == 15) return launch_ring<16, 8, 8>(p, grid, stream);
    return launch_ring<16, 4, 12>(p, grid, stream);
  }
  // ablation 12: the unaligned (separate header load) path on 1024-B records
  if (unpack_variant == 12 && fixed && p.fixed_len == 1024)
    return c.rows ? launch_fixed<16, 0, true>(p, grid, stream) : launch_fixed<16, 0>(p, grid, stream);
  // ablations of the aligned 1024-B kernel: variant 1024 + MODE (see unpack_fixed_kernel)
  if (unpack_variant >= 1024 && fixed && p.fixed_len == 1024) {
    switch (unpack_variant - 1024) {
#define MGENX_ABL(M) \
  case M: return c.rows ? launch_fixed<16, M, true, true>(p, grid, stream) \
                        : launch_fixed<16, M, false, true>(p, grid, stream);
      MGENX_ABL(1) MGENX_ABL(2) MGENX_ABL(3) MGENX_ABL(4) MGENX_ABL(5) MGENX_ABL(8)
      MGENX_ABL(16) MGENX_ABL(32) MGENX_ABL(64)
      MGENX_ABL(128) MGENX_ABL(144) MGENX_ABL(130) MGENX_ABL(136) MGENX_ABL(260) MGENX_ABL(772)
      MGENX_ABL(276) MGENX_ABL(324) MGENX_ABL(788)
#undef MGENX_ABL
      default: break;
    }
  }
  switch (unpack_variant) {
    case 1: return launch_mode<1>(p, grid, stream);
    case 2: return launch_mode<2>(p, grid, stream);
    case 3: return launch_mode<0>(p, grid, stream);  // variable lengths, unsorted
    case 4: return launch_sorted(p, grid, stream);   // sorted groups, no load ring
    default: break;
  }
  // var-kernel shapes (20..39): block size, rows held, the store ablation
  if (p.rec_len && unpack_variant >= 20 && unpack_variant < 40) {
    *which = MGENX_UNPACK_K_VAR;
    switch (unpack_variant) {
      case 20: return launch_var<1024, 0, 1>(p, grid, stream);  // every row store to the sink
      case 21: return launch_var<1024, 0, 0>(p, grid, stream);  // one row store per group
      case 22: return launch_var<768, 8, 0>(p, grid, stream);
      case 23: return launch_var<768, 16, 0>(p, grid, stream);
      case 27: return launch_var<1024, 8, 0>(p, grid, stream);
      case 32: return launch_var<1024, 4, 8>(p, grid, stream);  // non-temporal row stores
      case 33: return launch_var<1024, 4, 16>(p, grid, stream);  // 64-B-aligned row loads (timing)
      default: break;
    }
  }
#endif  // MGENX_DIAG
  // long records (a TCP stream of 16-KiB records: the mean length from the slab) -- one wave
  // per record, 1-KiB contiguous loads
  const uint64_t mean = p.rec_len ? (p.n ? p.slab_bytes / p.n : 0) : p.fixed_len;
  if (mean >= kLongMin) {
    *which = MGENX_UNPACK_K_LONG;
    return launch_long(p, grid, stream);
  }
  // per-record lengths: sorted groups with the rows in a load ring -- when every wave gets
  // at least two 64-record tiles; fewer, larger records (a 1 GiB stream of 16-KiB TCP
  // records is 1024 tiles for 4096 waves) keep the general kernel's one group per wave and
  // its 14-row load blocks, which keep more bytes in flight per record
  const uint64_t tiles = ((uint64_t)p.n + 63) / 64;
  const uint64_t waves = (uint64_t)grid * (kUnpackThreads / 64);
  if (p.rec_len && tiles >= 2 * waves) {
    *which = MGENX_UNPACK_K_VAR;
    return launch_var(p, grid, stream);
  }
  *which = MGENX_UNPACK_K_GENERAL;
  return launch_mode<0>(p, grid, stream);
}

#if MGENX_DIAG
// Diagnostic: streaming read of `bytes` (16 B per lane per load, grid-stride), XOR-folded
// into one word per block so the loads are not dead.  Reference for achievable HBM rate.
__global__ void __launch_bounds__(256) stream_read_kernel(const u32x4_t* p, uint64_t n16,
                                                          uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4_t a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^
           d.z ^ d.w;
  }
  for (; i < n16; i += stride) {
    const u32x4_t a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;  // practically never taken
}

// Diagnostic: unpack_fixed_kernel's memory pattern alone (groups of 16 x 1 KiB dealt to waves
// round-robin, rows reloaded one group ahead, 512 B stored per group when MODE & 1).
template <int MODE>
__global__ void __launch_bounds__(1024) group_rw_kernel(const uint8_t* p, uint32_t n_groups,
                                                        uint8_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * 16;
  uint32_t g = wave_id;
  if (g >= n_groups) return;
  // lane l of row j: record l/4 of the group, bytes 64 j + 16 (l & 3)
  const uint32_t lo = (uint32_t)(lane >> 2) * 1024u + 16u * (lane & 3);
  u32x4_t d[16];
#pragma unroll
  for (int j = 0; j < 16; j++) d[j] = ldu128(p + (uint64_t)g * 16384u + lo + 64 * j);
  uint32_t acc = 0;
  while (g < n_groups) {
    const uint32_t gn = g + n_waves;
    const uint32_t gl = gn < n_groups ? gn : g;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      acc = (acc << 1) ^ d[j].x ^ d[j].y ^ d[j].z ^ d[j].w;
      __builtin_amdgcn_sched_barrier(0);
      d[j] = ldu128(p + (uint64_t)gl * 16384u + lo + 64 * j);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE & 4) {  // 16-B stores from half the lanes
      if (lane < 32) {
        u32x4_t v = {acc, g, acc, g};
        *reinterpret_cast<u32x4_t*>(out + (uint64_t)g * 512u + 16u * lane) = v;
      }
    } else if (MODE & 1) {
      const uint64_t a = (uint64_t)out + (uint64_t)g * 512u + 8u * lane;
      const uint64_t v = (uint64_t)acc << 32 | g;
      if (MODE & 2) st_g64_wt(a, v); else st_g64(a, v);
    }
    g = gn;
  }
  if (!(MODE & 1) && acc == 0x9E3779B9u) out[lane] = 1;
}

// Diagnostic: group_rw with the row stores held back in registers and issued K groups at a
// time (K = 1 << LK), at each group's own row position; POL 0 = non-temporal, 1 = temporal,
// 2 = write-through stores.
template <int LK, int POL>
__global__ void __launch_bounds__(1024) group_rw_buf_kernel(const uint8_t* p, uint32_t n_groups,
                                                            uint8_t* out) {
  constexpr int K = 1 << LK;
  const int lane = threadIdx.x & 63;
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * 16;
  uint32_t g = wave_id;
  if (g >= n_groups) return;
  const uint32_t lo = (uint32_t)(lane >> 2) * 1024u + 16u * (lane & 3);
  u32x4_t d[16];
#pragma unroll
  for (int j = 0; j < 16; j++) d[j] = ldu128(p + (uint64_t)g * 16384u + lo + 64 * j);
  uint32_t acc = 0;
  while (g < n_groups) {
    uint64_t buf[K];
    uint32_t gs[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t gn = g + n_waves;
      const uint32_t gl = gn < n_groups ? gn : g;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        acc = (acc << 1) ^ d[j].x ^ d[j].y ^ d[j].z ^ d[j].w;
        __builtin_amdgcn_sched_barrier(0);
        d[j] = ldu128(p + (uint64_t)gl * 16384u + lo + 64 * j);
        __builtin_amdgcn_sched_barrier(0);
      }
      buf[k] = (uint64_t)acc << 32 | g;
      gs[k] = g;
      g = gn;
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint64_t a = (uint64_t)out + (uint64_t)(gs[k] < n_groups ? gs[k] : 0u) * 512u + 8u * lane;
      if (POL == 0) st_g64_nt(a, buf[k]);
      else if (POL == 1) st_g64(a, buf[k]);
      else st_g64_wt(a, buf[k]);
    }
  }
}

// Diagnostic: every wave keeps the row stores of its (<= 16) groups in registers; RING rows
// in flight per wave (16 = one group ahead, 8 = half a group); BAR: a grid-wide arrival
// barrier (bounded spin) between the last read and the stores, so the chip reads, then
// writes.  POL as group_rw_buf_kernel.
template <int RING, bool BAR, int POL>
__global__ void __launch_bounds__(1024) group_rw_phase_kernel(const uint8_t* p, uint32_t n_groups,
                                                              uint8_t* out, uint32_t* counter) {
  constexpr int K = 16;
  const int lane = threadIdx.x & 63;
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
  const uint32_t n_waves = gridDim.x * 16;
  const uint32_t lo = (uint32_t)(lane >> 2) * 1024u + 16u * (lane & 3);
  const uint32_t my_groups = wave_id < n_groups ? (n_groups - wave_id + n_waves - 1) / n_waves : 0;
  // 32-bit byte offsets (slab < 4 GiB); group k of this wave, clamped to its last group
  auto goff = [&](int k) {
    const uint32_t kk = (uint32_t)k < my_groups ? (uint32_t)k : (my_groups ? my_groups - 1 : 0);
    const uint32_t g = wave_id + kk * n_waves;
    return (g < n_groups ? g : 0u) * 16384u + lo;
  };
  u32x4_t d[RING];
  uint32_t cur = goff(0), nxt = goff(1);
#pragma unroll
  for (int j = 0; j < RING; j++) d[j] = ldu128(p + (uint64_t)(cur + 64u * j));
  // a shift register of the last K groups' row words: buf[K-1] = the newest group
  uint64_t buf[K];
#pragma unroll
  for (int k = 0; k < K; k++) buf[k] = 0;
  uint32_t acc = 0;
  // two groups per trip keep the ring index static when RING does not divide 16
  for (uint32_t k = 0; k < my_groups; k++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      u32x4_t& x = d[j % RING];
      acc = (acc << 1) ^ x.x ^ x.y ^ x.z ^ x.w;
      __builtin_amdgcn_sched_barrier(0);
      const int jn = j + RING;  // row r + RING: this group or the next
      x = ldu128(p + (uint64_t)(jn < 16 ? cur + 64u * jn : nxt + 64u * (jn - 16)));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < K - 1; q++) buf[q] = buf[q + 1];
    buf[K - 1] = (uint64_t)acc << 32 | k;
    cur = nxt;
    nxt = goff((int)k + 2);
  }
#pragma unroll
  for (int k = 0; k < K; k++) {  // buf[k] holds group my_groups - K + k
    const int kg = (int)my_groups - K + k;
    const uint32_t g = wave_id + (uint32_t)kg * n_waves;
    if (kg >= 0 && g < n_groups) {
      const uint64_t a = (uint64_t)out + (uint64_t)g * 512u + 8u * lane;
      if (POL == 0) st_g64_nt(a, buf[k]);
      else if (POL == 1) st_g64(a, buf[k]);
      else st_g64_wt(a, buf[k]);
    }
  }
}

hipError_t launch_group_rw(const uint8_t* p, uint64_t bytes, uint8_t* out, int mode, int grid,
                           hipStream_t stream) {
  const uint32_t ng = (uint32_t)(bytes / 16384);
  if (mode >= 4096) {  // 4096 + 16 * ring_sel + 4 * bar + pol
    static uint32_t* counter = nullptr;
    if (!counter && hipMalloc((void**)&counter, 256) != hipSuccess) return hipErrorOutOfMemory;
    hipError_t e = hipMemsetAsync(counter, 0, 16, stream);
    if (e != hipSuccess) return e;
    const int m = mode - 4096;
#define MGENX_GPH(RING, BAR, POL, CODE)                                                         \
  if (m == CODE) {                                                                              \
    hipLaunchKernelGGL((group_rw_phase_kernel<RING, BAR, POL>), dim3(grid), dim3(1024), 0, stream, \
                       p, ng, out, counter);                                                    \
    return hipGetLastError();                                                                   \
  }
    MGENX_GPH(16, false, 0, 0) MGENX_GPH(16, true, 0, 4) MGENX_GPH(8, false, 0, 16)
    MGENX_GPH(8, true, 0, 20) MGENX_GPH(16, true, 1, 5) MGENX_GPH(8, true, 1, 21)
#undef MGENX_GPH
    return hipErrorInvalidValue;
  }
  if (mode >= 16) {
    const int lk = ((mode >> 4) & 7) - 1, pol = (mode >> 8) & 3;
#define MGENX_GRB(LK, POL)                                                                   \
  if (lk == LK && pol == POL) {                                                              \
    hipLaunchKernelGGL((group_rw_buf_kernel<LK, POL>), dim3(grid), dim3(1024), 0, stream, p, ng, \
                       out);                                                                 \
    return hipGetLastError();                                                                \
  }
    MGENX_GRB(0, 0) MGENX_GRB(1, 0) MGENX_GRB(2, 0) MGENX_GRB(3, 0) MGENX_GRB(4, 0)
    MGENX_GRB(2, 1) MGENX_GRB(4, 1) MGENX_GRB(2, 2) MGENX_GRB(4, 2)
#undef MGENX_GRB
    return hipErrorInvalidValue;
  }
  switch (mode & 7) {
    case 4: hipLaunchKernelGGL(group_rw_kernel<4>, dim3(grid), dim3(1024), 0, stream, p, ng, out); break;
    case 0: hipLaunchKernelGGL(group_rw_kernel<0>, dim3(grid), dim3(1024), 0, stream, p, ng, out); break;
    case 1: hipLaunchKernelGGL(group_rw_kernel<1>, dim3(grid), dim3(1024), 0, stream, p, ng, out); break;
    default: hipLaunchKernelGGL(group_rw_kernel<3>, dim3(grid), dim3(1024), 0, stream, p, ng, out); break;
  }
  return hipGetLastError();
}

// Diagnostic: a coalesced read of `bytes` at W bytes per lane (4, 8 or 24: the access shapes of
// the config-4 kernels' column loads and 24-B record loads) -- FETCH_SIZE calibration per shape.
struct alignas(8) SrW24 {
  uint32_t w[6];
};
__device__ __forceinline__ uint32_t sr_fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t sr_fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t sr_fold(const SrW24& v) {
  return v.w[0] ^ v.w[1] ^ v.w[2] ^ v.w[3] ^ v.w[4] ^ v.w[5];
}
template <typename T>
__global__ void __launch_bounds__(256) stream_read_w_kernel(const T* p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const T a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= sr_fold(a) ^ sr_fold(b) ^ sr_fold(c) ^ sr_fold(d);
  }
  for (; i < n; i += stride) acc ^= sr_fold(p[i]);
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;  // practically never taken
}
hipError_t launch_stream_read_w(const uint8_t* p, uint64_t bytes, uint32_t* out, int grid,
                                int width, hipStream_t stream) {
  if (width == 4)
    hipLaunchKernelGGL(stream_read_w_kernel<uint32_t>, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const uint32_t*>(p), bytes / 4, out);
  else if (width == 8)
    hipLaunchKernelGGL(stream_read_w_kernel<uint2>, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const uint2*>(p), bytes / 8, out);
  else if (width == 24)
    hipLaunchKernelGGL(stream_read_w_kernel<SrW24>, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const SrW24*>(p), bytes / 24, out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_stream_read(const uint8_t* p, uint64_t bytes, uint32_t* out, int grid,
                              hipStream_t stream) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4_t*>(p), bytes / 16, out);
  return hipGetLastError();
}

#endif  // MGENX_DIAG

int unpack_threads() { return kUnpackThreads; }

}  // namespace mgenx
