// mgenx_tcp.hip -- MgenTcpTransport's transmit byte stream on gfx950.
//
// Reference (restated in oracle/mgen_oracle.c or_tcp_tx): MgenTcpTransport::SendMessage
// (src/common/mgenTransport.cpp:1320-1400) with GetNextTxFragmentSize :1960-1993,
// GetNextTxFragment :1878-1951, SetupNextTxBuffer :1818-1852, CalcTxChecksum :1854-1876.
// A message of mgen_msg_len M goes out as fragments of at most 65535 bytes (65459 when the
// remainder would leave less than a minimum fragment); a fragment F <= 8192 is one packed
// buffer with LAST_BUFFER and its checksum; a larger one is ONE 8-KiB Pack (8188 bytes when
// F - 8192 < 4) whose buffer is then re-sent from its start until F bytes have gone out
// (8192 per buffer, the last one carrying the CRC over everything before it).
//
// GPU form, per round r (fragment r of every message; one round unless M > 65535):
//   tcp_frag_kernel   fragment descriptors: msg_len = F, Pack's bufferLen B, flags, offset;
//   raw Pack          (mgenx_pack.hip, MGENX_PACK_RAW) the B-byte buffer P at the fragment
//                     start, its running CRC and the MgenMsg flags it leaves -- and, as each
//                     16-byte unit of P is stored, its copies P[0 .. s_k) in every later
//                     buffer k of the fragment (PackParams.frag_len: no copy pass);
//   tcp_prefix_kernel raw(s) = the CRC register over P[0 .. s) from zero for the (at most
//                     three) distinct buffer lengths of the fragment, from one pass over P's
//                     header and payload bytes and the fill algebra (no re-read of the buffer);
//   tcp_finish_kernel the running CRC chained through the buffers algebraically,
//                     c' = raw(s) ^ x^(8s) * c  (c = 0 restarts from ~0, as ComputeCRC32 does),
//                     and the big-endian trailer.
#include <hip/hip_runtime.h>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr uint32_t kTxBuf = MGENX_TX_BUFFER_SIZE;  // 8192
constexpr uint32_t kMaxFrag = MGENX_MAX_FRAG_SIZE;  // 65535
constexpr uint32_t kMinFrag = 76;                   // MIN_FRAG_SIZE (mgenTransport.h)

// fragment r of a message of M bytes: size, offset within the message, flags bits
__device__ __forceinline__ bool tcp_fragment(uint32_t M, uint32_t r, uint32_t& F, uint32_t& at,
                                             bool& more) {
  uint32_t off = 0;
  for (uint32_t k = 0;; k++) {
    const uint32_t rem = M - off;
    if (rem == 0) return false;
    uint32_t f;
    if (rem > kMaxFrag) f = rem < kMaxFrag + kMinFrag ? kMaxFrag - kMinFrag : kMaxFrag;
    else f = rem;
    if (k == r) {
      F = f;
      at = off;
      more = rem > f;
      return true;
    }
    off += f;
  }
}

// per message: stream bytes (0 when the first Pack fails -- no destination, or a first
// fragment shorter than the address part of the header -- or M == 0) and fragment count
__global__ void tcp_plan_kernel(const mgenx_flow_tmpl* __restrict__ tmpl,
                                const mgenx_pack_desc* __restrict__ desc,
                                const uint32_t* __restrict__ msg_total, uint32_t n,
                                uint64_t* __restrict__ bytes, uint32_t* __restrict__ nfrag,
                                uint32_t* __restrict__ max_frag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c = 0;  // fragments (no early return: the block maximum below has a barrier)
  if (i == n) bytes[n] = 0;  // exclusive-scan tail
  if (i < n) {
    const uint32_t M = msg_total[i];
    const mgenx_flow_tmpl& t = tmpl[desc[i].tmpl];
    const bool dst_ok = t.dst_type == 1u || t.dst_type == 2u;
    const uint32_t D = t.dst_len > 16u ? 16u : t.dst_len;
    uint32_t F0 = 0, at;
    bool more, ok = false;
    if (M && tcp_fragment(M, 0, F0, at, more)) {
      const uint32_t B0 = F0 > kTxBuf ? kTxBuf - 4u : F0;  // smallest bufferLen it can get
      ok = dst_ok && B0 >= 24u + D;
    }
    if (ok) {
      uint32_t F, a;
      while (tcp_fragment(M, c, F, a, more)) c++;
    }
    bytes[i] = c ? (uint64_t)M : 0ull;
    nfrag[i] = c;
  }
  // the round count: a block maximum, one atomic per block (max_frag zeroed by the caller)
  __shared__ uint32_t wmax[4];
  uint32_t mx = c;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
  if ((threadIdx.x & 63u) == 0u) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0u) {
    mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (mx) atomicMax(max_frag, mx);
  }
}

// round r: the pack descriptor of fragment r of each message (msg_len 0 = none this round)
__global__ void tcp_frag_kernel(const mgenx_pack_desc* __restrict__ desc,
                                const uint32_t* __restrict__ msg_total,
                                const uint32_t* __restrict__ nfrag,
                                const uint64_t* __restrict__ msg_off, uint32_t n, uint32_t r,
                                int ck, const uint32_t* __restrict__ prev_state,
                                mgenx_pack_desc* __restrict__ fd, uint64_t* __restrict__ foff,
                                uint32_t* __restrict__ fbuf, uint32_t* __restrict__ ff) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mgenx_pack_desc d = desc[i];
  uint32_t F = 0, at = 0;
  bool more = false;
  if (r < nfrag[i]) (void)tcp_fragment(msg_total[i], r, F, at, more);
  uint32_t B = 0;
  if (F) {
    // the MgenMsg flags member: the descriptor's on the first fragment, what the previous
    // fragment's Pack left afterwards (GetNextTxFragmentSize, :1960-1993)
    uint32_t fl = r == 0 ? d.flags : (prev_state[i] >> 16) & 0xffu;
    fl &= ~(uint32_t)MGENX_FLAG_CONTINUES;
    if (msg_total[i] > kMaxFrag) fl |= more ? MGENX_FLAG_CONTINUES : MGENX_FLAG_END_OF_MSG;
    if (F > kTxBuf) {  // GetNextTxFragment: Pack into the 8-KiB buffer (:1915-1926)
      B = (ck && (int32_t)F - (int32_t)kTxBuf < 4 && F != kMinFrag) ? kTxBuf - 4u : kTxBuf;
    } else {
      fl |= MGENX_FLAG_LAST_BUFFER;
      B = F;
    }
    d.flags = (uint8_t)fl;
  }
  d.msg_len = (uint16_t)F;
  fd[i] = d;
  foff[i] = msg_off[i] + at;
  fbuf[i] = B;
  ff[i] = F;
}

// buffer k >= 1 of a fragment of F bytes whose first buffer holds B: (start, size)
// (SetupNextTxBuffer, :1818-1852); returns false past the last
__device__ __forceinline__ bool tcp_buffer(uint32_t F, uint32_t B, int ck, uint32_t k,
                                           uint32_t& start, uint32_t& size, bool& last) {
  uint32_t pos = B;
  for (uint32_t j = 1;; j++) {
    const uint32_t pend = F - pos;
    if (pend == 0) return false;
    uint32_t s;
    bool l = false;
    if ((ck && pend <= kTxBuf - 4u) || (!ck && pend <= kTxBuf)) {
      s = pend;
      l = true;
    } else {
      s = (ck && (int32_t)pend - (int32_t)kTxBuf < 4) ? pend - 4u : kTxBuf;
    }
    if (j == k) {
      start = pos;
      size = s;
      last = l;
      return true;
    }
    pos += s;
  }
}

// raw(s) = the CRC register after P[0 .. s) from a zero start (no init, no final xor), for
// the (at most three) distinct CRC lengths of a fragment's later buffers (full 8192, one
// SetupNextTxBuffer-shortened buffer, the last one's size - 4), without re-reading the
// 8-KiB buffer: P is Pack's image -- header (packet_header_len h bytes), the payload it
// copied (p bytes, read back from the payload_len field that ends a complete header), then
// fill -- so one pass over the h + p body bytes (four at a time, slicing tables in LDS)
// serves every length, extended over the fill algebraically: zeros are the shift x^(8q);
// RANDOM_FILL's fill is two zero bytes and the rand stream, raw CRC rcrc[q - 2]
// (mgenMsg.cpp:274-293).  A length inside the body (a short fragment) walks its bytes.
__global__ void __launch_bounds__(256)
tcp_prefix_kernel(const uint8_t* __restrict__ out, const uint64_t* __restrict__ foff,
                  const uint32_t* __restrict__ fbuf, const uint32_t* __restrict__ ff,
                  const uint32_t* __restrict__ plen, const uint32_t* __restrict__ state,
                  uint32_t n, int ck, int rnd, const uint32_t* __restrict__ byte_tab,
                  const uint32_t* __restrict__ a4_tab, const uint32_t* __restrict__ xpow,
                  const uint32_t* __restrict__ rcrc, uint32_t* __restrict__ acrc) {
  __shared__ uint32_t s_a4[1024];
  __shared__ uint32_t s_tab[256];
  for (uint32_t k = threadIdx.x; k < 1024u; k += blockDim.x) s_a4[k] = a4_tab[k];
  for (uint32_t k = threadIdx.x; k < 256u; k += blockDim.x) s_tab[k] = byte_tab[k];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t F = ff[i], B = fbuf[i];
  uint32_t L[3] = {0u, 0u, 0u};
  if (!(ck && F > B && plen[i])) return;
  uint32_t start, size;
  bool last;
  for (uint32_t k = 1; tcp_buffer(F, B, ck, k, start, size, last); k++) {
    const uint32_t c = last ? size - 4u : size;
    L[last ? 2 : (size == kTxBuf ? 0 : 1)] = c;
  }
  const uint8_t* P = out + foff[i];
  const uint32_t h = state[i] & 0xffffu;
  uint32_t p = 0;  // payload bytes Pack copied
  const uint32_t D = P[23];
  if (24u + D + 4u <= h) {
    const uint32_t H = P[24u + D + 3u];
    if (h == 24u + D + 4u + H + 16u) p = (uint32_t)P[h - 2u] << 8 | P[h - 1u];
  }
  const uint32_t body = h + p;
  auto walk = [&](uint32_t len) {  // raw CRC of P[0 .. len)
    uint32_t c = 0;
    const uint32_t nw = len >> 2;
    for (uint32_t k = 0; k < nw; k++) {
      const uint32_t x = c ^ ldu32(P + 4u * k);
      c = s_a4[x & 0xffu] ^ s_a4[256 + ((x >> 8) & 0xffu)] ^ s_a4[512 + ((x >> 16) & 0xffu)] ^
          s_a4[768 + (x >> 24)];
    }
    for (uint32_t k = nw << 2; k < len; k++) c = s_tab[(c ^ P[k]) & 0xffu] ^ (c >> 8);
    return c;
  };
  const uint32_t cb = walk(body);
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const uint32_t len = L[j];
    if (!len) continue;
    uint32_t c;
    if (len >= body) {
      const uint32_t q = len - body;
      c = multmodp(xpow[q], cb);
      if (rnd && q >= 3u) c ^= rcrc[q - 2u];
    } else {
      c = walk(len);
    }
    acrc[3 * i + j] = c;
  }
}

// the fragment's CRC through its later buffers and the trailer
__global__ void tcp_finish_kernel(uint8_t* __restrict__ out, const uint64_t* __restrict__ foff,
                                  const uint32_t* __restrict__ fbuf, const uint32_t* __restrict__ ff,
                                  const uint32_t* __restrict__ plen, const uint32_t* __restrict__ tx_crc,
                                  const uint32_t* __restrict__ state, const uint32_t* __restrict__ acrc,
                                  const uint32_t* __restrict__ xpow, const uint32_t* __restrict__ ia,
                                  uint32_t n, int ck, uint64_t cap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t F = ff[i], B = fbuf[i];
  if (!ck || !F || plen[i] == 0) return;
  // (defensive only: mgenx_pack_tcp refuses a stream past its capacity before any round runs)
  if (foff[i] > cap || F > cap - foff[i]) return;
  uint32_t c = tx_crc[i];
  bool write = true;
  if (F <= B) {
    // one buffer: Pack ran with LAST_BUFFER; WriteChecksum only when Pack set CHECKSUM
    write = ((state[i] >> 16) & MGENX_FLAG_CHECKSUM) != 0u;
  } else {
    uint32_t start, size;
    bool last;
    for (uint32_t k = 1; tcp_buffer(F, B, ck, k, start, size, last); k++) {
      const uint32_t s = last ? size - 4u : size;
      const uint32_t a = acrc[3 * i + (last ? 2 : (size == kTxBuf ? 0 : 1))];  // raw(P[0..s))
      // ComputeCRC32(c, P, s): a zero running value restarts (from ~0)
      const uint32_t cr = c == 0u ? 0xFFFFFFFFu : c;
      if (s) c = a ^ multmodp(xpow[s], cr);
      else c = cr;
    }
  }
  if (write) {
    const uint32_t v = c ^ 0xFFFFFFFFu;
    uint8_t* p = out + foff[i] + F - 4u;
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
  }
}

hipError_t launch_tcp_plan(const mgenx_flow_tmpl* tmpl, const mgenx_pack_desc* desc,
                           const uint32_t* msg_total, uint32_t n, uint64_t* bytes,
                           uint32_t* nfrag, uint32_t* max_frag, hipStream_t s) {
  hipLaunchKernelGGL(tcp_plan_kernel, dim3((n + 256) / 256), dim3(256), 0, s, tmpl, desc, msg_total,
                     n, bytes, nfrag, max_frag);
  return hipGetLastError();
}

hipError_t launch_tcp_frag(const mgenx_pack_desc* desc, const uint32_t* msg_total,
                           const uint32_t* nfrag, const uint64_t* msg_off, uint32_t n, uint32_t r,
                           int ck, const uint32_t* prev_state, mgenx_pack_desc* fd, uint64_t* foff,
                           uint32_t* fbuf, uint32_t* ff, hipStream_t s) {
  hipLaunchKernelGGL(tcp_frag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, desc, msg_total, nfrag,
                     msg_off, n, r, ck, prev_state, fd, foff, fbuf, ff);
  return hipGetLastError();
}

hipError_t launch_tcp_tail(uint8_t* out, const uint64_t* foff, const uint32_t* fbuf,
                           const uint32_t* ff, const uint32_t* plen, const uint32_t* tx_crc,
                           const uint32_t* state, uint32_t n, int ck, int rnd, uint32_t* acrc,
                           const uint32_t* byte_tab, const uint32_t* a4_tab, const uint32_t* xpow,
                           const uint32_t* ia, const uint32_t* rcrc, uint64_t cap, hipStream_t s) {
  if (ck) {
    hipLaunchKernelGGL(tcp_prefix_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, foff, fbuf,
                       ff, plen, state, n, ck, rnd, byte_tab, a4_tab, xpow, rcrc, acrc);
    hipLaunchKernelGGL(tcp_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, foff, fbuf,
                       ff, plen, tx_crc, state, acrc, xpow, ia, n, ck, cap);
  }
  return hipGetLastError();
}

}  // namespace mgenx
