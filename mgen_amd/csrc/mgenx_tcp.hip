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
// GPU form: round 0 (the first fragment of every message) and, only when some M > 65535,
// one more round per further fragment:
//   tcp_plan0_kernel  (round 0) the plan, the message offsets (a scan with a decoupled
//                     look-back) and the fragment descriptors in one launch, its verdict to
//                     a device word that gates round 0's Pack and to host memory;
//   tcp_frag_kernel   (round r > 0) fragment descriptors: msg_len = F, Pack's bufferLen B,
//                     flags, offset;
//   raw Pack          (mgenx_pack.hip, MGENX_PACK_RAW, PackParams.frag_len) the B-byte buffer
//                     P at the fragment start and, as each 16-byte unit of P is stored, its
//                     copies P[0 .. s_k) in every later buffer k of the fragment (no copy
//                     pass); its meta phase runs the CRC on through the later buffers
//                     algebraically -- raw(s_k) = x^(8(s_k - pend)) raw(P[0 .. pend)) over
//                     the fill, c' = raw(s) ^ x^(8s) c (c = 0 restarts from ~0, as
//                     ComputeCRC32 does) -- and writes the big-endian trailer.
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

// the size of the fragment that starts with rem bytes of the message left
__device__ __forceinline__ uint32_t tcp_frag_size(uint32_t rem) {
  if (rem > kMaxFrag) return rem < kMaxFrag + kMinFrag ? kMaxFrag - kMinFrag : kMaxFrag;
  return rem;
}

// a message of M bytes: its fragment count -- 0 when the first Pack fails (no destination, or
// a first fragment shorter than the address part of the header) or M == 0 -- and its first
// fragment's size F0
__device__ __forceinline__ uint32_t tcp_count(const mgenx_flow_tmpl& t, uint32_t M, uint32_t& F0) {
  F0 = 0;
  if (!M) return 0u;
  const bool dst_ok = t.dst_type == 1u || t.dst_type == 2u;
  const uint32_t D = t.dst_len > 16u ? 16u : t.dst_len;
  const uint32_t f0 = tcp_frag_size(M);
  const uint32_t B0 = f0 > kTxBuf ? kTxBuf - 4u : f0;  // smallest bufferLen it can get
  if (!(dst_ok && B0 >= 24u + D)) return 0u;
  uint32_t c = 0;
  for (uint32_t off = 0; off < M; c++) off += tcp_frag_size(M - off);
  F0 = f0;
  return c;
}

// per message: stream bytes (0 when the first Pack fails, see tcp_count) and fragment count
// (the exact path's plan: mgenx_pack_tcp falls back to it when tcp_plan0_kernel cannot vouch
// for its own result)
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
    uint32_t F0;
    c = tcp_count(tmpl[desc[i].tmpl], M, F0);
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

// fragment F of a message of M bytes (more: fragments follow; F == 0: none), whose MgenMsg
// flags member is fl before it: the pack descriptor's flags and msg_len; returns Pack's
// bufferLen (GetNextTxFragmentSize :1960-1993, GetNextTxFragment :1915-1926)
__device__ __forceinline__ uint32_t tcp_frag_desc(mgenx_pack_desc& d, uint32_t fl, uint32_t M,
                                                  uint32_t F, bool more, int ck) {
  uint32_t B = 0;
  if (F) {
    fl &= ~(uint32_t)MGENX_FLAG_CONTINUES;
    if (M > kMaxFrag) fl |= more ? MGENX_FLAG_CONTINUES : MGENX_FLAG_END_OF_MSG;
    if (F > kTxBuf) {  // Pack into the 8-KiB buffer
      B = (ck && (int32_t)F - (int32_t)kTxBuf < 4 && F != kMinFrag) ? kTxBuf - 4u : kTxBuf;
    } else {
      fl |= MGENX_FLAG_LAST_BUFFER;
      B = F;
    }
    d.flags = (uint8_t)fl;
  }
  d.msg_len = (uint16_t)F;
  return B;
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
  // the MgenMsg flags member: the descriptor's on the first fragment, what the previous
  // fragment's Pack left afterwards
  const uint32_t fl = r == 0 || !F ? d.flags : (prev_state[i] >> 16) & 0xffu;
  fbuf[i] = tcp_frag_desc(d, fl, msg_total[i], F, more, ck);
  fd[i] = d;
  foff[i] = msg_off[i] + at;
  ff[i] = F;
}

// The plan, the message offsets and round 0's fragment descriptors in one launch: block g
// plans messages [g kTcpPlanMsgs, (g + 1) kTcpPlanMsgs) (message u 256 + t of the block on
// thread t, coalesced), scans their stream bytes in LDS and takes its first offset from a
// decoupled look-back over the earlier blocks' epoch-tagged words (epoch << 48 | kind << 46 |
// bytes; kind 1 aggregate, 2 inclusive).  Before its inclusive word a block stores its
// fragment maximum and a failure bit (epoch << 32 | fail << 31 | fragments) in a word of its
// own; the last block waits for every inclusive word, takes the maximum over those words and
// writes the verdict:
//   skip[0]  for the launches queued behind this one (round 0's pack and tail): non-zero when
//            the stream exceeds cap or the plan failed -- they then store nothing;
//   host     one 16-byte write-through store the host spins on: the stream bytes, and epoch
//            << 48 | fail << 32 | rounds.
// It fails (the host redoes the plan on the exact path) when a look-back gives up (dispatch
// order is not promised: the wait is bounded) or a running total passes 2^46 bytes.
constexpr uint32_t kPlanThreads = 256;
constexpr uint32_t kPlanPer = kTcpPlanMsgs / kPlanThreads;
constexpr uint64_t kPlanMax = (1ull << 46) - 1;
constexpr uint32_t kPlanSpin = 1u << 20;

__device__ __forceinline__ uint64_t plan_word(uint32_t epoch, uint32_t kind, uint64_t v) {
  return ((uint64_t)epoch << 48) | ((uint64_t)kind << 46) | v;
}

__global__ void __launch_bounds__(kPlanThreads)
tcp_plan0_kernel(const mgenx_flow_tmpl* __restrict__ tmpl, const mgenx_pack_desc* __restrict__ desc,
                 const uint32_t* __restrict__ msg_total, uint32_t n, int ck, uint64_t cap,
                 uint32_t epoch, uint64_t* __restrict__ status, uint64_t* __restrict__ fmax,
                 uint64_t* __restrict__ msg_off, uint32_t* __restrict__ nfrag,
                 mgenx_pack_desc* __restrict__ fd, uint32_t* __restrict__ fbuf,
                 uint32_t* __restrict__ ff, uint32_t* __restrict__ skip,
                 uint64_t* __restrict__ host) {
  __shared__ uint32_t s_bytes[kTcpPlanMsgs];
  __shared__ uint64_t s_off[kTcpPlanMsgs];
  __shared__ uint64_t wsum[kPlanThreads / 64];
  __shared__ uint32_t wmax[kPlanThreads / 64];
  __shared__ uint64_t s_prefix;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t g = blockIdx.x;
  const uint32_t base = g * kTcpPlanMsgs;
  // 1. plan (every load issued before the dependent template reads)
  uint32_t M[kPlanPer], tix[kPlanPer];
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; u++) {
    const uint32_t i = base + u * kPlanThreads + tid;
    M[u] = i < n ? msg_total[i] : 0u;
    tix[u] = i < n ? desc[i].tmpl : 0u;
  }
  uint32_t c[kPlanPer], F0[kPlanPer], mx = 0;
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; u++) {
    c[u] = M[u] ? tcp_count(tmpl[tix[u]], M[u], F0[u]) : 0u;
    if (!M[u]) F0[u] = 0u;
    s_bytes[u * kPlanThreads + tid] = c[u] ? M[u] : 0u;
    mx = max(mx, c[u]);
  }
  // 2. fragment counts and round 0's descriptors (independent of the offsets: out before the
  // look-back)
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; u++) {
    const uint32_t i = base + u * kPlanThreads + tid;
    if (i >= n) continue;
    mgenx_pack_desc d = desc[i];
    const uint32_t F = c[u] ? F0[u] : 0u;
    fbuf[i] = tcp_frag_desc(d, d.flags, M[u], F, M[u] > F, ck);
    fd[i] = d;
    ff[i] = F;
    nfrag[i] = c[u];
  }
  __syncthreads();
  // 3. the block's exclusive offsets (thread t: entries 4t .. 4t+3) and its aggregate
  uint64_t loc[kPlanPer], tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPlanPer; k++) {
    loc[k] = tot;
    tot += s_bytes[kPlanPer * tid + k];
  }
  uint64_t incl = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint64_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
  if (lane == 63u) wsum[wv] = incl;
  if (lane == 0u) wmax[wv] = mx;
  __syncthreads();
  uint64_t run = incl - tot, agg = 0;
  uint32_t bmax = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPlanThreads / 64; k++) {
    run += k < wv ? wsum[k] : 0ull;
    agg += wsum[k];
    bmax = max(bmax, wmax[k]);
  }
#pragma unroll
  for (uint32_t k = 0; k < kPlanPer; k++) s_off[kPlanPer * tid + k] = run + loc[k];
  // 4. the block's first offset: aggregate, look-back (wave 0), its fragment maximum (and
  // failure bit), inclusive
  if (wv == 0) {
    if (lane == 0)  // (an aggregate even for block 0: its inclusive word must follow its maximum)
      __hip_atomic_store(&status[g], plan_word(epoch, 1u, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t acc = 0;
    bool gave_up = false;
    for (int64_t top = (int64_t)g - 1; top >= 0 && !gave_up; top -= 64) {
      const int64_t q = top - (int64_t)lane;
      uint64_t w = 0;
      if (q >= 0) {
        uint32_t polls = 0;
        do {
          w = __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } while ((uint32_t)(w >> 48) != epoch && ++polls < kPlanSpin);
      }
      const bool here = q < 0 || (uint32_t)(w >> 48) == epoch;
      gave_up = __ballot(!here) != 0;
      const uint32_t kind = q >= 0 ? (uint32_t)(w >> 46) & 3u : 2u;
      const uint64_t v = q >= 0 && here ? (w & kPlanMax) : 0ull;
      const uint64_t done = __ballot(kind == 2u);  // lanes holding an inclusive word
      const uint32_t stop = done ? (uint32_t)__ffsll((long long)done) - 1u : 64u;
      uint64_t mine = lane <= stop ? v : 0ull;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mine += __shfl_xor(mine, o);
      acc += mine;
      if (done) break;
    }
    const bool fail = gave_up || acc + agg > kPlanMax;  // (wave-uniform)
    if (lane == 0) {
      // the maximum word before the inclusive word (release): whoever sees the one sees the other
      __hip_atomic_store(&fmax[g], ((uint64_t)epoch << 32) | (fail ? 0x80000000ull : 0ull) | bmax,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&status[g], plan_word(epoch, 2u, min(acc + agg, kPlanMax)),
                         __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      s_prefix = acc;
    }
    if (g + 1 == gridDim.x) {
      // the verdict waits for every block's inclusive word, then takes the maximum over their
      // maximum words (no atomics: one word a block, read where it was published)
      bool all = true;
      uint64_t m = ((uint64_t)epoch << 32) | (fail ? 0x80000000ull : 0ull) | bmax;
      for (uint32_t q0 = 0; q0 < g && all; q0 += 64) {
        const uint32_t q = q0 + lane;
        bool ok = true;
        if (q < g) {
          uint32_t polls = 0;
          uint64_t w;
          do {
            w = __hip_atomic_load(&status[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(w >> 48) == epoch && ((w >> 46) & 3u) == 2u;
          } while (!ok && ++polls < kPlanSpin);
          const uint64_t f = __hip_atomic_load(&fmax[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((uint32_t)(f >> 32) != epoch) ok = false;
          m = max(m, f);
        }
        all = __ballot(!ok) == 0;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint64_t)__shfl_xor(m, o));
      if (lane == 0) {  // the verdict
        const uint64_t total = acc + agg;
        const bool bad = fail || !all || (m & 0x80000000ull) != 0;
        skip[0] = bad || total > cap ? 1u : 0u;
        const uint64_t hi = ((uint64_t)epoch << 48) | ((uint64_t)bad << 32) | (m & 0x7FFFFFFFull);
        const u32x4_t w = {(uint32_t)total, (uint32_t)(total >> 32), (uint32_t)hi,
                           (uint32_t)(hi >> 32)};
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(host), "v"(w)
                     : "memory");  // (system coherent: one write to host memory)
      }
    }
  }
  __syncthreads();
  // 5. the offsets (round 0's fragments start at them: Pack reads msg_off as its record offsets)
  const uint64_t first = s_prefix;
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; u++) {
    const uint32_t i = base + u * kPlanThreads + tid;
    if (i < n) msg_off[i] = first + s_off[u * kPlanThreads + tid];
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

hipError_t launch_tcp_plan0(const mgenx_flow_tmpl* tmpl, const mgenx_pack_desc* desc,
                            const uint32_t* msg_total, uint32_t n, int ck, uint64_t cap,
                            uint32_t epoch, uint64_t* status, uint64_t* fmax, uint64_t* msg_off,
                            uint32_t* nfrag, mgenx_pack_desc* fd, uint32_t* fbuf, uint32_t* ff,
                            uint32_t* skip, uint64_t* host, hipStream_t s) {
  hipLaunchKernelGGL(tcp_plan0_kernel, dim3((n + kTcpPlanMsgs - 1) / kTcpPlanMsgs),
                     dim3(kPlanThreads), 0, s, tmpl, desc, msg_total, n, ck, cap, epoch, status,
                     fmax, msg_off, nfrag, fd, fbuf, ff, skip, host);
  return hipGetLastError();
}

}  // namespace mgenx
