// mgenx_analytic.hip -- per-flow receive analytics (MgenAnalytic::Update) on gfx950.
//
// Reference: MgenAnalytic::Init / Update (src/common/mgenAnalytic.cpp:28-258) called per
// received message by Mgen::UpdateRecvAnalytics (src/common/mgen.cpp:1027-1070), over the
// protolib primitives ProtoSlidingMask (1024-bit duplicate window) and ProtoTime::Delta
// (restated in oracle/mgen_oracle.c; parity unpinned at protolib).
//
// The state machine is sequential per flow and independent across flows, so:
//   1. every record is written as the 24-B record the update reads (latency precomputed), and
//      the records are ordered by flow, stably (receive order kept): `order`, a counting sort
//      (per-tile flow histograms, one scan, a per-tile LDS sort written run by run) for up
//      to 2047 flows, else a hipCUB radix sort of (flow, record) pairs;
//   2. one wave per flow runs Update over its records, read through `order` (see WRing and
//      the fast segments below).
// FP64: every product that feeds an add goes through mul_rounded (an empty asm keeps the
// backend from fusing them into an FMA: neither __dadd_rn/__dmul_rn nor `#pragma clang fp
// contract(off)` prevented it -- a 1-ulp difference in a report's duration was the
// symptom), so results are bit-identical to the oracle built for x86-64.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mgenx_kernels.hpp"
#include "mgenx_flowsm.hpp"

namespace mgenx {

// One received record as the update kernel reads it: 24 B, written flow-sorted by the ordering
// step, so the update streams its flow's records instead of gathering them.  The receive time
// is one 64-bit key, sec << 32 | usec (ProtoTime's >= is the key's >=); the latency
// ProtoTime::Delta(rx, tx) depends on the record alone, so it is computed there, off the
// per-flow chain.
struct FRec {
  uint64_t rxk;
  uint32_t seq, len;
  double latency;
};

// Where a record's fields come from: the columns, or the unpack's 32-B rows when `rows` is set.
struct RecSrc {
  const uint32_t *seq, *txs, *txu;
  const uint16_t* len;
  const mgenx_rec* rows;
  const uint32_t *rxs, *rxu;
};
// a record's raw fields as loaded (the order kernel keeps the next tile's in registers while it
// writes the current one: the latency math waits for the loads, so it runs at placement)
struct RawRec {
  uint32_t seq, ts, tu, len, rs, ru;
};
template <bool kRows>
// (the column loads are non-temporal: read once, they would otherwise push out of L2 the
// partly written lines where the runs of adjacent tiles meet -- the ordering 0.183 -> 0.175 ms)
__device__ __forceinline__ RawRec load_rec_t(const RecSrc& src, uint32_t i) {
  RawRec r;
  if (kRows) {
    // flow, seq, tx_sec, tx_usec
    const u32x4_t h = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src.rows + i));
    r.seq = h.y;
    r.ts = h.z;
    r.tu = h.w;
    r.len = __builtin_nontemporal_load(&src.rows[i].msg_len);
  } else {
    r.seq = __builtin_nontemporal_load(src.seq + i);
    r.ts = __builtin_nontemporal_load(src.txs + i);
    r.tu = __builtin_nontemporal_load(src.txu + i);
    r.len = __builtin_nontemporal_load(src.len + i);
  }
  r.rs = __builtin_nontemporal_load(src.rxs + i);
  r.ru = __builtin_nontemporal_load(src.rxu + i);
  return r;
}
__device__ __forceinline__ RawRec load_rec(const RecSrc& src, uint32_t i) {
  return src.rows ? load_rec_t<true>(src, i) : load_rec_t<false>(src, i);
}
__device__ __forceinline__ FRec build_frec(const RawRec& w) {
  FRec r;
  r.seq = w.seq;
  r.len = w.len;
  r.rxk = (uint64_t)w.rs << 32 | w.ru;
  r.latency = tdelta(Tm{(int64_t)w.rs, (int64_t)w.ru}, Tm{(int64_t)w.ts, (int64_t)w.tu});
  return r;
}
__device__ __forceinline__ FRec make_frec(const RecSrc& src, uint32_t i) {
  return build_frec(load_rec(src, i));
}

// ---- MgenAnalytic::Update, window-parallel (mgenAnalytic.cpp:74-258) ----
// The state machine is sequential per flow, but its order-dependent parts separate:
//   * window closes depend on receive times alone (rxTime >= window_end, :168; the end moves to
//     rxTime + window_size at each close, :228-230);
//   * the mask's span (first, last) and seq_start evolve without the mask's bit contents: a Set
//     fails exactly when it would widen the span to 1024 or more, whatever the bits hold, and a
//     failed Set in the counted branch (:118-127) clears every set index -- the mask becomes
//     {seq} (an "epoch start"; so does the first message of a flow, :80-99, and the first actual
//     message, :156-165);
//   * within an epoch nothing is cleared and every set index stays inside one 1024-wide span,
//     so seq mod 1024 names a set index uniquely: a record is a duplicate (:109) exactly when an
//     earlier record of its epoch set the same sequence number;
//   * the counters restart at every close (:228-242), so each window's msg_count, byte_count
//     and latency min / max are reductions over its own records, from a start state that only
//     the closing record of the window before decides.
// Two kernels:
//   flow_skel_kernel  one wave per flow walks its records 256 at a time, scalar state only:
//                     a run of records whose span stays below 1024 (a wave min / max) and holds
//                     no close and no first message is plain; otherwise inclusive prefix scans
//                     of seq - first find the first record that fails its Set, and it, a close
//                     or a first message is done alone.  Out: a flag byte per record and the
//                     flow's windows (records, epoch of the first record, seqMax and seq_start
//                     at the close);
//   flow_win_kernel   one wave per window (8 waves per flow): the epoch table of the window's
//                     first record rebuilt in LDS (seq mod 1024 -> first position), the
//                     duplicate test of each record, the window's counters and report, lat' per
//                     record;
//                     the window's in-order FP64 latency sum (the one chain whose rounding
//                     depends on record order), and -- the open window's wave -- the flow's
//                     state.
// scripts/flow_decomp.py is the same decomposition on the CPU, checked against the oracle.
constexpr uint8_t kFIns = 1;      // the record's seq is in the mask after it (Set succeeded)
constexpr uint8_t kFDupT = 2;     // it takes the duplicate test with its seq inside the span
constexpr uint8_t kFCe = 4;       // counted unless a duplicate (:121-154; a restart included)
constexpr uint8_t kFEstart = 8;   // epoch start: the mask is {seq} after it
constexpr uint8_t kFFa = 16;      // first message / first actual message: counters restart at it
constexpr uint8_t kFInit0 = 32;   // first message of the flow, size 0 (:94-98)
constexpr uint8_t kFClose = 64;   // closes a window
constexpr uint32_t kNoEpoch = 0xFFFFFFFFu, kWinOpen = 1u, kWinZr = 2u;
constexpr uint32_t kWinWaves = 8;  // flow_win_kernel: waves (windows in flight) per flow
constexpr uint32_t kTabEmpty = 0xFFFFFFFFu;

struct WinItem {       // one window of a flow (flow f's k-th at wins[bnd[f] + f + k])
  uint32_t a, c;       // records [a, c] (c closes it) / open: [a, c) with c = the flow's end
  uint32_t r;          // the epoch start at record a (kNoEpoch: the call's initial epoch)
  uint32_t fl;         // kWinOpen, kWinZr (the closing record restarted the sum: :156-165)
  uint32_t seqmax, sst;  // seqMax at the close, the seq_start it is measured from (:174-219)
  uint64_t ws;         // window start, receive-time key
};
struct FlowFin {       // per flow: the state before the call (flow_skel_kernel copies it, so
                       // the window waves read it while the open window's wave rewrites the
                       // flow state), and the skeleton's results
  uint32_t mask0[32];  // the mask before the call, relative to first0
  uint32_t first0, n0, F, hasmask;
  uint32_t nwin, ncl, rc0, rsv;
  uint64_t mc0, bc0;
  double lmin0, lmax0, lsum0;
};
static_assert(sizeof(WinItem) == 32, "window item");


__device__ __forceinline__ uint64_t tm_key(Tm t) { return (uint64_t)t.sec << 32 | (uint64_t)t.usec; }
__device__ __forceinline__ Tm key_tm(uint64_t k) { return Tm{(int64_t)(k >> 32), (int64_t)(uint32_t)k}; }

// inclusive min / max scan over the wave (DPP rows of 16 by shifts, then the row broadcasts;
// lanes a step does not reach keep their value: `old` is the identity)
template <bool kMax>
__device__ __forceinline__ int32_t wave_incl_minmax(int32_t v) {
  const int32_t id = kMax ? INT32_MIN : INT32_MAX;
  auto op = [](int32_t a, int32_t c) { return kMax ? max(a, c) : min(a, c); };
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return v;
}
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
  return (int32_t)WRing::wave_reduce((uint32_t)v, (uint32_t)INT32_MAX, [](uint32_t a, uint32_t c) {
    return (uint32_t)min((int32_t)a, (int32_t)c); });
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
  return (int32_t)WRing::wave_reduce((uint32_t)v, (uint32_t)INT32_MIN, [](uint32_t a, uint32_t c) {
    return (uint32_t)max((int32_t)a, (int32_t)c); });
}

#if MGENX_DIAG
__device__ unsigned long long g_skel_prof[8];
__device__ unsigned int g_skel_claim;
#endif
// ---- the skeleton: one workgroup per flow, its walk on one wave ----
// The walk is sequential and runs on one wave, so what it costs per record is what counts
// (measured on config 4: ~2.5 k cycles per 256-record chunk for the per-record span test --
// about 250 dependent instructions on a lone wave -- whether the records came from registers
// or LDS).  So the workgroup's four waves do the per-record work in parallel around the walk:
//   1. stage the flow's records -- the first 16 bytes of each FRec: receive key, seq, length --
//      into LDS by direct global->LDS loads (kSkSeg records a segment, all in flight at once);
//   2. summarize each 256-record chunk: its largest receive key, and the lowest / highest
//      seq - base over its set attempts (base: the chunk's first seq), any non-zero length;
//   3. wave 0 walks the summaries: a chunk with no close (largest key below the window end), no
//      first message and a span below 1024 after it (the summary's min / max against first /
//      last) is plain -- O(1) scalar work; any other chunk takes the per-record path (prefix
//      scans, the first event alone, as before) on wave 0;
//   4. the four waves write the plain chunks' flag bytes (the seq_start of each is recorded).
// The summary test is exact when it passes: every record's seq - first then lies inside the
// span, where the chunk-relative value plus the chunk base's offset equals it.
constexpr uint32_t kSkQ = 4;
constexpr uint32_t kSkChunk = 64u * kSkQ;
constexpr uint32_t kSkSeg = 4096;  // records staged per segment (64 KiB: two workgroups per CU)
constexpr uint32_t kSkChunks = kSkSeg / kSkChunk;
struct SkSum {  // one chunk's summary
  uint32_t rx_lo, rx_hi, base;
  int32_t dmin, dmax;
  uint32_t nz, rsv0, rsv1;
};
constexpr size_t kSkLds = (size_t)kSkSeg * 16u + kSkChunks * sizeof(SkSum) + kSkChunks * 8u;
struct SkLd {
  uint32_t seq[kSkQ], len[kSkQ];
  uint64_t rxk[kSkQ];
};
typedef __attribute__((address_space(3))) void lds_void_t;
__global__ void __launch_bounds__(256)
flow_skel_kernel(mgenx_flow_state* __restrict__ flows, uint32_t n_flows, uint32_t fmul,
                 const uint32_t* __restrict__ bnd, const FRec* __restrict__ recs,
                 uint8_t* __restrict__ rflags, WinItem* __restrict__ wins,
                 FlowFin* __restrict__ fin, uint32_t* __restrict__ report_count) {
  extern __shared__ u32x4_t skl[];  // kSkSeg staged records {rxk, seq, len}, then summaries
  SkSum* sums = reinterpret_cast<SkSum*>(skl + kSkSeg);
  uint32_t* cst = reinterpret_cast<uint32_t*>(sums + kSkChunks);  // [c]: plain, [kSkChunks + c]: sst
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  // flows to blocks by a multiplicative permutation (fmul coprime with n_flows): blocks go to
  // the XCDs round robin, and a rank's flows (every 8th) would otherwise all land on one XCD
  const uint32_t f = (uint32_t)(((uint64_t)blockIdx.x * fmul) % n_flows);
  const uint32_t b = bnd[f], e = bnd[f + 1u];
  if (b >= e) return;
  // stage records [s, s + kSkSeg) of the flow (every wave), then wait for them (all threads)
  auto stage = [&](uint32_t s) {
    const uint32_t ninst = (min(kSkSeg, e - s) + 63u) / 64u;
    for (uint32_t k = wv; k < ninst; k += 4u) {
      const FRec* src = recs + min(s + 64u * k + lane, e - 1u);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(skl + 64u * k), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  // chunk c of the segment at s: its summary (one wave)
  auto summarize = [&](uint32_t s, uint32_t c) {
    const uint32_t i0 = s + c * kSkChunk, se = min(e, s + kSkSeg);
    const uint32_t base = skl[c * kSkChunk].z;  // the chunk's first seq
    uint32_t rhi = 0, rlo = 0;
    int32_t dmn = INT32_MAX, dmx = INT32_MIN;
    bool nz = false;
#pragma unroll
    for (uint32_t q = 0; q < kSkQ; q++) {
      const uint32_t o = 64u * q + lane;
      const u32x4_t v = skl[c * kSkChunk + o];
      const bool in = i0 + o < se;
      const bool hi_gt = v.y > rhi || (v.y == rhi && v.x > rlo);
      rlo = (in && hi_gt) ? v.x : rlo;
      rhi = (in && hi_gt) ? v.y : rhi;
      const bool att = in && v.w != 0u;
      const int32_t d = (int32_t)(v.z - base);
      dmn = att ? min(dmn, d) : dmn;
      dmx = att ? max(dmx, d) : dmx;
      nz |= att;
    }
    const uint32_t RH = WRing::wave_max(rhi);
    const uint32_t RL = WRing::wave_max(rhi == RH ? rlo : 0u);
    const int32_t DMN = wave_min_i32(dmn), DMX = wave_max_i32(dmx);
    const bool NZ = __ballot(nz) != 0ull;
    if (lane == 0) {
      SkSum sm;
      sm.rx_lo = RL;
      sm.rx_hi = RH;
      sm.base = base;
      sm.dmin = DMN;
      sm.dmax = DMX;
      sm.nz = NZ ? 1u : 0u;
      sm.rsv0 = sm.rsv1 = 0u;
      sums[c] = sm;
    }
  };
  // the plain chunks' flag bytes (every wave): set attempts, counted at or past seq_start
  auto plain_flags = [&](uint32_t s, uint32_t c) {
    const uint32_t i0 = s + c * kSkChunk, se = min(e, s + kSkSeg), sst_c = cst[kSkChunks + c];
#pragma unroll
    for (uint32_t q = 0; q < kSkQ; q++) {
      const uint32_t o = 64u * q + lane;
      const u32x4_t v = skl[c * kSkChunk + o];
      const uint32_t ce = (int32_t)(v.z - sst_c) >= 0 ? (uint32_t)kFCe : 0u;
      if (i0 + o < se) rflags[i0 + o] = (uint8_t)(v.w != 0u ? (uint32_t)(kFIns | kFDupT) | ce : 0u);
    }
  };
  if (wv != 0) {  // the helper waves: stage, summarize, write the plain chunks' flags
    for (uint32_t s = b; s < e; s += kSkSeg) {
      stage(s);
      const uint32_t nch = (min(kSkSeg, e - s) + kSkChunk - 1u) / kSkChunk;
      for (uint32_t c = wv; c < nch; c += 4u) summarize(s, c);
      __syncthreads();  // summaries ready
      __syncthreads();  // wave 0 has walked the segment
      for (uint32_t c = wv; c < nch; c += 4u)
        if (cst[c]) plain_flags(s, c);
      __syncthreads();  // the segment's LDS may be restaged
    }
    return;
  }
  mgenx_flow_state* sp = flows + f;
  const TAdd window = tadd_of(sp->window_size);
  bool valid = sp->window_valid != 0, hasm = sp->mask_n != 0;
  uint32_t F = sp->mask_first, L = F;
  if (hasm) {  // last = first + the highest set relative bit
    const uint32_t w = lane < 32u ? sp->mask[lane] : 0u;
    const uint32_t top = w ? lane * 32u + (31u - __clz(w)) : 0u;
    L = F + (uint32_t)__builtin_amdgcn_readfirstlane((int)WRing::wave_max(top));
  }
  uint32_t sst = sp->seq_start;
  Tm ws = {sp->win_start_sec, sp->win_start_usec}, we = {sp->win_end_sec, sp->win_end_usec};
  uint64_t wek = tkey(we);
  const uint32_t rc0 = report_count[f];
  uint32_t nwin = 0, ncl = 0;
  uint32_t win_a = b, win_r = kNoEpoch, cur_es = kNoEpoch;
  WinItem* wl = wins + ((size_t)b + f);
  FlowFin* fp = fin + f;
  if (lane < 32u) fp->mask0[lane] = sp->mask[lane];
  if (lane == 0) {
    fp->first0 = sp->mask_first;
    fp->n0 = sp->mask_n;
    fp->mc0 = sp->msg_count;
    fp->bc0 = sp->byte_count;
    fp->lmin0 = sp->latency_min;
    fp->lmax0 = sp->latency_max;
    fp->lsum0 = sp->latency_sum;
  }
#if MGENX_DIAG
  // (diagnostics) cycles of the first walk to finish: fast runs, prefix scans, event records,
  // total, staging (incl. its wait); counts of fast runs, slow runs, events
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memtime();
  const unsigned long long prof_t0 = prof_t;
#define SK_T(slot)                                                         \
  do {                                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
    prof[slot] += now_ - prof_t;                                           \
    prof_t = now_;                                                         \
  } while (0)
#define SK_N(slot) prof[slot]++
#else
#define SK_T(slot) do {} while (0)
#define SK_N(slot) do {} while (0)
#endif

  uint32_t seg = b;  // the staged segment's first record
  auto ld = [&](uint32_t i0, SkLd& r) {  // from LDS (lanes past the flow read stale slots)
#pragma unroll
    for (uint32_t q = 0; q < kSkQ; q++) {
      const u32x4_t v = skl[i0 - seg + 64u * q + lane];
      r.rxk[q] = (uint64_t)v.y << 32 | v.x;
      r.seq[q] = v.z;
      r.len[q] = v.w;
    }
  };
  auto chunk = [&](const uint32_t i0, const SkLd& cur) {
    const uint32_t cnt = min(kSkChunk, e - i0);
    uint32_t fl[kSkQ];
#pragma unroll
    for (uint32_t q = 0; q < kSkQ; q++) fl[q] = 0u;
    uint32_t pos = 0;
    while (pos < cnt) {
      const int32_t Lr = (int32_t)(L - F);
      int32_t rel[kSkQ];
      bool inr[kSkQ], att[kSkQ];
      int32_t lmn = INT32_MAX, lmx = INT32_MIN;
      uint64_t evb[kSkQ];  // closes and first messages, per q
      bool anyev = false;
#pragma unroll
      for (uint32_t q = 0; q < kSkQ; q++) {
        const uint32_t o = 64u * q + lane;
        inr[q] = (o >= pos) & (o < cnt);
        att[q] = inr[q] & (cur.len[q] != 0u);
        rel[q] = (int32_t)(cur.seq[q] - F);
        lmn = att[q] ? min(lmn, rel[q]) : lmn;
        lmx = att[q] ? max(lmx, rel[q]) : lmx;
        const bool spec = inr[q] & (!valid | ((cur.len[q] != 0u) & !hasm));
        const bool clo = inr[q] & valid & (cur.rxk[q] >= wek);
        evb[q] = __ballot(spec | clo);
        anyev |= evb[q] != 0ull;
      }
      const bool mask_ops = valid & hasm;
      const int32_t tmn = min(0, wave_min_i32(lmn)), tmx = max(Lr, wave_max_i32(lmx));
      if (!anyev && (!mask_ops || (int64_t)tmx - (int64_t)tmn < 1024)) {
        // the whole run [pos, cnt) is plain: every Set succeeds
#pragma unroll
        for (uint32_t q = 0; q < kSkQ; q++) {
          const uint32_t ce = (int32_t)(cur.seq[q] - sst) >= 0 ? (uint32_t)kFCe : 0u;
          fl[q] = att[q] ? (uint32_t)(kFIns | kFDupT) | ce : fl[q];
        }
        if (mask_ops) {
          const uint32_t F2 = F + (uint32_t)tmn;
          L = F + (uint32_t)tmx;
          F = F2;
        }
        SK_T(0);
        SK_N(5);
        break;
      }
      SK_T(0);
      SK_N(6);
      // each record's span from inclusive prefixes (q-major order: the scans of the four
      // groups, chained by their totals); the first failing Set, close or first message
      int32_t imn[kSkQ], imx[kSkQ];
#pragma unroll
      for (uint32_t q = 0; q < kSkQ; q++) {
        imn[q] = wave_incl_minmax<false>(att[q] ? rel[q] : INT32_MAX);
        imx[q] = wave_incl_minmax<true>(att[q] ? rel[q] : INT32_MIN);
      }
      int32_t cmn = 0, cmx = Lr;
      uint32_t ev = kSkChunk;
#pragma unroll
      for (uint32_t q = 0; q < kSkQ; q++) {
        imn[q] = min(cmn, imn[q]);
        imx[q] = max(cmx, imx[q]);
        cmn = __builtin_amdgcn_readlane(imn[q], 63);
        cmx = __builtin_amdgcn_readlane(imx[q], 63);
        const bool fail = att[q] & mask_ops & ((int64_t)imx[q] - (int64_t)imn[q] >= 1024);
        const uint64_t eb = evb[q] | __ballot(fail);
        if (eb && ev == kSkChunk) ev = 64u * q + (uint32_t)__builtin_ctzll(eb);
      }
      // the run [pos, ev): plain records
#pragma unroll
      for (uint32_t q = 0; q < kSkQ; q++) {
        const uint32_t o = 64u * q + lane;
        const uint32_t ce = (int32_t)(cur.seq[q] - sst) >= 0 ? (uint32_t)kFCe : 0u;
        fl[q] = (att[q] & (o < ev)) ? (uint32_t)(kFIns | kFDupT) | ce : fl[q];
      }
      if (ev > pos && mask_ops) {  // the span after the run
        const uint32_t o1 = ev - 1u, l1 = o1 & 63u, q1 = o1 >> 6;
        int32_t vmn = imn[0], vmx = imx[0];
#pragma unroll
        for (uint32_t q = 1; q < kSkQ; q++) {
          vmn = q1 == q ? imn[q] : vmn;
          vmx = q1 == q ? imx[q] : vmx;
        }
        const int32_t mn = __builtin_amdgcn_readlane(vmn, (int)l1);
        const int32_t mx = __builtin_amdgcn_readlane(vmx, (int)l1);
        const uint32_t F2 = F + (uint32_t)mn;
        L = F + (uint32_t)mx;
        F = F2;
      }
      SK_T(1);
      if (ev >= cnt) break;
      SK_N(7);
      // the event record, alone (wave-uniform)
      const uint32_t le = ev & 63u, qe = ev >> 6;
      uint32_t vs = cur.seq[0], vl = cur.len[0];
      uint64_t vr = cur.rxk[0];
#pragma unroll
      for (uint32_t q = 1; q < kSkQ; q++) {
        vs = qe == q ? cur.seq[q] : vs;
        vl = qe == q ? cur.len[q] : vl;
        vr = qe == q ? cur.rxk[q] : vr;
      }
      const uint32_t seq = (uint32_t)__builtin_amdgcn_readlane((int)vs, (int)le);
      const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)vl, (int)le);
      const uint64_t rxk = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vr, (int)le) |
                           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vr >> 32), (int)le) << 32;
      const uint32_t p = i0 + ev;
      const Tm rx = key_tm(rxk);
      uint32_t fe = 0;
      if (!valid) {  // :79-100 (no close test)
        valid = true;
        ws = rx;
        we = uni_t(tadd(rx, window));
        wek = tkey(we);
        if (len != 0u) {
          hasm = true;
          F = L = seq;
          sst = seq;
          fe = kFEstart | kFFa | kFIns;
          cur_es = p;
        } else {
          fe = kFInit0;
        }
      } else {
        if (len != 0u) {
          if (!hasm) {  // the first actual message (:156-165)
            hasm = true;
            F = L = seq;
            sst = seq;
            fe = kFEstart | kFFa | kFIns;
            cur_es = p;
          } else {
            const int32_t r = (int32_t)(seq - F);
            const int32_t mn = min(0, r), mx = max((int32_t)(L - F), r);
            if ((int64_t)mx - (int64_t)mn < 1024) {  // Set succeeds
              fe = kFIns | kFDupT | ((int32_t)(seq - sst) >= 0 ? kFCe : 0u);
              const uint32_t F2 = F + (uint32_t)mn;
              L = F + (uint32_t)mx;
              F = F2;
            } else if ((int32_t)(seq - sst) >= 0) {  // counted, Set fails: UnsetBits, Set
              F = L = seq;
              fe = kFEstart | kFIns | kFCe;
              cur_es = p;
            }  // else precedes the window and Set fails: nothing changes
          }
        }
        if (rxk >= wek) {  // :168-255
          const uint32_t seqmax = hasm ? L : sst;
          if (lane == 0) {
            WinItem it;
            it.a = win_a;
            it.c = p;
            it.r = win_r;
            it.fl = (fe & kFFa) ? kWinZr : 0u;
            it.seqmax = seqmax;
            it.sst = sst;
            it.ws = tm_key(ws);
            wl[nwin] = it;
          }
          nwin++;
          ncl++;
          sst = seqmax;
          ws = rx;
          we = uni_t(tadd(rx, window));
          wek = tkey(we);
          win_a = p + 1u;
          win_r = cur_es;
          fe |= kFClose;
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kSkQ; q++) fl[q] = (lane == le && q == qe) ? fe : fl[q];
      pos = ev + 1u;
      SK_T(2);
    }
#pragma unroll
    for (uint32_t q = 0; q < kSkQ; q++)
      if (64u * q + lane < cnt) rflags[i0 + 64u * q + lane] = (uint8_t)fl[q];
  };
  for (; seg < e; seg += kSkSeg) {
    stage(seg);
    const uint32_t nch = (min(kSkSeg, e - seg) + kSkChunk - 1u) / kSkChunk;
    for (uint32_t c = 0; c < nch; c += 4u) summarize(seg, c);
    __syncthreads();  // summaries ready
    SK_T(4);
    for (uint32_t c = 0; c < nch; c++) {
      const uint32_t i0 = seg + c * kSkChunk;
      const SkSum sm = sums[c];  // (every lane reads the same: broadcast)
      const uint64_t mx_rx = (uint64_t)__builtin_amdgcn_readfirstlane((int)sm.rx_hi) << 32 |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)sm.rx_lo);
      const bool nz = __builtin_amdgcn_readfirstlane((int)sm.nz) != 0;
      bool plain = valid && mx_rx < wek && (!nz || hasm);
      int64_t mn = 0, mx = (int32_t)(L - F);
      if (plain && nz) {
        const int64_t r0 = (int32_t)((uint32_t)__builtin_amdgcn_readfirstlane((int)sm.base) - F);
        mn = min((int64_t)0, r0 + __builtin_amdgcn_readfirstlane(sm.dmin));
        mx = max(mx, r0 + __builtin_amdgcn_readfirstlane(sm.dmax));
        plain = mx - mn < 1024;
      }
      if (lane == 0) {
        cst[c] = plain ? 1u : 0u;
        cst[kSkChunks + c] = sst;
      }
      if (plain) {
        if (nz) {
          const uint32_t F2 = F + (uint32_t)mn;
          L = F + (uint32_t)mx;
          F = F2;
        }
        SK_T(0);
        SK_N(5);
      } else {
        SkLd B;
        ld(i0, B);
        chunk(i0, B);
      }
    }
    __syncthreads();  // the segment is walked
    for (uint32_t c = 0; c < nch; c += 4u)
      if (cst[c]) plain_flags(seg, c);
    __syncthreads();  // the segment's LDS may be restaged
  }
  if (lane == 0) {
    WinItem it;
    it.a = win_a;
    it.c = e;
    it.r = win_r;
    it.fl = kWinOpen;
    it.seqmax = it.sst = 0u;
    it.ws = tm_key(ws);
    wl[nwin] = it;
    fp->F = F;
    fp->hasmask = hasm ? 1u : 0u;
    fp->nwin = nwin + 1u;
    fp->ncl = ncl;
    fp->rc0 = rc0;
    sp->window_valid = valid ? 1u : 0u;
    sp->win_start_sec = ws.sec;
    sp->win_start_usec = ws.usec;
    sp->win_end_sec = we.sec;
    sp->win_end_usec = we.usec;
    sp->seq_start = sst;
    sp->n_reports += ncl;
    report_count[f] = rc0 + ncl;
  }
#if MGENX_DIAG
  prof[3] = __builtin_amdgcn_s_memtime() - prof_t0;
  if (lane == 0 && atomicCAS(&g_skel_claim, 0u, 1u) == 0u)
    for (int k2 = 0; k2 < 8; k2++) g_skel_prof[k2] = prof[k2];
#endif
#undef SK_T
#undef SK_N
}

#if MGENX_DIAG
__device__ unsigned long long g_win_prof[8];
__device__ unsigned int g_win_claim;
#endif
// ---- the windows: one wave (a workgroup of its own) per window, kWinWaves per flow ----
// The wave walks its window's epoch from the epoch's start (records before the window only
// insert), chunks of 256 records q-major, two chunks in flight in two register sets.  The
// window's latency sum -- the one FP64 chain whose rounding depends on record order -- is the
// wave's, in order, over each chunk's lat' read out lane by lane.  The open window's wave writes
// the flow's state (the others read the state before the call from FlowFin).
constexpr uint32_t kWQ = 4;
constexpr uint32_t kWChunk = 64u * kWQ;
struct WLd {
  FRec r[kWQ];
  uint32_t fl[kWQ];
};
__global__ void __launch_bounds__(64)
flow_win_kernel(mgenx_flow_state* __restrict__ flows, uint32_t n_flows,
                const uint32_t* __restrict__ bnd, const FRec* __restrict__ recs,
                const uint8_t* __restrict__ rflags, const WinItem* __restrict__ wins,
                const FlowFin* __restrict__ fin, mgenx_flow_report* __restrict__ reports,
                uint32_t per_flow, uint32_t* __restrict__ report_rec,
                const uint32_t* __restrict__ order) {
  __shared__ uint32_t T[1024];
  const uint32_t lane = threadIdx.x;
  const uint32_t f = blockIdx.x / kWinWaves, wv = blockIdx.x % kWinWaves;
  if (f >= n_flows) return;
  const uint32_t b = bnd[f], e = bnd[f + 1u];
  if (b >= e) return;
  mgenx_flow_state* sp = flows + f;
  const FlowFin* fp = fin + f;
  const uint32_t nwin = fp->nwin, rc0 = fp->rc0;
  auto wsync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto clear_tab = [&] {
#pragma unroll
    for (uint32_t j = 0; j < 1024u / 64u; j++) T[64u * j + lane] = kTabEmpty;
  };
  const double inf = __builtin_huge_val();
#if MGENX_DIAG
  // (diagnostics) cycles of one middle window (k = 1) by phase: setup, insert-only chunks,
  // duplicate passes, counters, sums, tail, total; chunks
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = 0, prof_t0 = 0;
#define WN_T(slot)                                                         \
  do {                                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
    prof[slot] += now_ - prof_t;                                           \
    prof_t = now_;                                                         \
  } while (0)
#else
#define WN_T(slot) do {} while (0)
#endif
  for (uint32_t k = wv; k < nwin; k += kWinWaves) {
#if MGENX_DIAG
    prof_t = prof_t0 = __builtin_amdgcn_s_memtime();
#endif
    const WinItem it = wins[(size_t)b + f + k];
    const bool open = (it.fl & kWinOpen) != 0u;
    const uint32_t a = it.a, end = open ? it.c : it.c + 1u;
    clear_tab();
    wsync();
    uint32_t s0 = it.r;
    if (it.r == kNoEpoch) {  // the call's initial epoch: the stored mask's indices, position 0
      s0 = b;
      if (fp->n0) {
        const uint32_t F0 = fp->first0;
        uint32_t w = lane < 32u ? fp->mask0[lane] : 0u;
        while (w) {
          const uint32_t j = (uint32_t)__builtin_ctz(w);
          w &= w - 1u;
          T[(F0 + lane * 32u + j) & 1023u] = 0u;
        }
        wsync();
      }
    }
    // the start state: the stored one, or (below) the one the record before the window leaves
    uint64_t mc = 0, bc = 0;
    double lmin = 0.0, lmax = 0.0, sum = 0.0;
    if (a == b) {
      mc = fp->mc0;
      bc = fp->bc0;
      lmin = fp->lmin0;
      lmax = fp->lmax0;
      sum = fp->lsum0;
    }
    const uint32_t tfrom = a > b ? a - 1u : a;  // records from here take the duplicate test
    uint32_t kc = 0, ndup = 0, fpos = 0xFFFFFFFFu, fsize = 0;
    uint64_t ssum = 0;
    double cmn = inf, cmx = -inf;
    auto ld = [&](uint32_t i0, WLd& w) {
#pragma unroll
      for (uint32_t q = 0; q < kWQ; q++) {
        const uint32_t p = min(i0 + 64u * q + lane, end - 1u);
        w.r[q] = recs[p];
        w.fl[q] = rflags[p];
      }
    };
    auto chunk = [&](const uint32_t i0, const WLd& w) {
      const uint32_t cnt = min(kWChunk, end - i0);
      uint32_t fl[kWQ];
#pragma unroll
      for (uint32_t q = 0; q < kWQ; q++) fl[q] = 64u * q + lane < cnt ? w.fl[q] : 0u;
#if MGENX_DIAG
      prof[7]++;
#endif
      if (i0 + cnt <= tfrom) {  // before the tested records: inserts only
#pragma unroll
        for (uint32_t q = 0; q < kWQ; q++)
          if (fl[q] & kFIns) atomicMin(&T[w.r[q].seq & 1023u], i0 + 64u * q + lane + 1u);
        WN_T(1);
        return;
      }
      bool dup[kWQ] = {false, false, false, false};
      uint32_t lo = 0;
      while (lo < cnt) {
        // the sub-range [lo, hi): up to the next epoch start after lo
        uint32_t hi = cnt;
        bool at_es = false;
#pragma unroll
        for (uint32_t q = 0; q < kWQ; q++) {
          const uint32_t o = 64u * q + lane;
          const bool es = (fl[q] & kFEstart) != 0u;
          const uint64_t eb = __ballot((o > lo) & es);
          if (eb) hi = min(hi, 64u * q + (uint32_t)__builtin_ctzll(eb));
          at_es |= __ballot((o == lo) & es) != 0ull;
        }
        if (at_es) {  // an epoch start at lo: the mask is {seq} after it
          clear_tab();
          wsync();
        }
#pragma unroll
        for (uint32_t q = 0; q < kWQ; q++) {
          const uint32_t o = 64u * q + lane;
          if ((o >= lo) & (o < hi) & ((fl[q] & kFIns) != 0u))
            atomicMin(&T[w.r[q].seq & 1023u], i0 + o + 1u);
        }
        wsync();
#pragma unroll
        for (uint32_t q = 0; q < kWQ; q++) {
          const uint32_t o = 64u * q + lane;
          const uint32_t tv = T[w.r[q].seq & 1023u];
          const bool mine = (o >= lo) & (o < hi);
          dup[q] = mine ? ((fl[q] & kFDupT) != 0u) & (tv < i0 + o + 1u) : dup[q];
        }
        wsync();
        lo = hi;
      }
      WN_T(2);
      // the record before the window: the start state it leaves (:228-242)
      if (a > b && tfrom >= i0 && tfrom < i0 + cnt) {
        const uint32_t o = tfrom - i0, l = o & 63u, qq = o >> 6;
        uint32_t vl = w.r[0].len, vf = fl[0], vd = dup[0];
        double vt = w.r[0].latency;
#pragma unroll
        for (uint32_t q = 1; q < kWQ; q++) {
          vl = qq == q ? w.r[q].len : vl;
          vf = qq == q ? fl[q] : vf;
          vd = qq == q ? (uint32_t)dup[q] : vd;
          vt = qq == q ? w.r[q].latency : vt;
        }
        const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)vl, (int)l);
        const uint32_t fc = (uint32_t)__builtin_amdgcn_readlane((int)vf, (int)l);
        const bool dc = __builtin_amdgcn_readlane((int)vd, (int)l) != 0;
        const uint64_t lb = __builtin_bit_cast(uint64_t, vt);
        const double lat = __builtin_bit_cast(
            double, (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(lb >> 32), (int)l) << 32 |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lb, (int)l));
        const bool counted = (fc & kFCe) && !dc;
        mc = len ? 1u : 0u;
        bc = 0u;
        lmin = lmax = (len != 0u && counted) ? lat : 0.0;
        sum = counted ? lat : 0.0;  // latency_sum = latency (:236): the record's lat'
      }
      // the window's records: counters; a counter restart (first message / first actual
      // message) precedes every counted record of the window (the mask is empty before it)
      double lp[kWQ];
#pragma unroll
      for (uint32_t q = 0; q < kWQ; q++) {
        const uint32_t o = 64u * q + lane;
        const uint32_t p = i0 + o;
        const bool live = (o < cnt) & (p >= a);
        const bool counted = live & ((fl[q] & kFCe) != 0u) & !dup[q];
        const bool fa = live & ((fl[q] & kFFa) != 0u);
        ndup += (live & dup[q]) ? 1u : 0u;
        kc += counted ? 1u : 0u;
        ssum += counted ? w.r[q].len : 0u;
        fsize = (counted & (p < fpos)) ? w.r[q].len : fsize;
        fpos = (counted & (p < fpos)) ? p : fpos;
        cmn = vmin64(cmn, counted ? w.r[q].latency : inf);
        cmx = vmax64(cmx, counted ? w.r[q].latency : -inf);
        lp[q] = (counted | fa) ? w.r[q].latency : 0.0;
      }
#pragma unroll
      for (uint32_t q = 0; q < kWQ; q++) {
        const uint32_t o = 64u * q + lane;
        const uint64_t rs = __ballot((o < cnt) & (i0 + o >= a) & ((fl[q] & (kFFa | kFInit0)) != 0u));
        if (rs) {
          // the last one (a size-0 first message, then the first actual message: one window)
          const uint32_t l = 63u - (uint32_t)__builtin_clzll(rs);
          const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)w.r[q].len, (int)l);
          const uint64_t lb = __builtin_bit_cast(uint64_t, w.r[q].latency);
          const uint32_t llo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lb, (int)l);
          const uint32_t lhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(lb >> 32), (int)l);
          const double lat = __builtin_bit_cast(double, (uint64_t)lhi << 32 | llo);
          const uint32_t fv = (uint32_t)__builtin_amdgcn_readlane((int)fl[q], (int)l);
          const bool fa = (fv & kFFa) != 0u;
          mc = fa ? 1u : 0u;
          bc = fa ? len : 0u;
          lmin = lmax = fa ? lat : 0.0;
        }
      }
      WN_T(3);
      // the sum, in record order: lane l's lat' of group q is record i0 + 64q + l, read out
      // lane by lane (the reads do not wait for the sum: only the adds form the chain); the
      // records outside the window add 0.0, exactly (a latency sum is never -0.0)
#pragma unroll
      for (uint32_t q = 0; q < kWQ; q++) {
        const uint64_t bits = __builtin_bit_cast(uint64_t, lp[q]);
        const int lo = (int)(uint32_t)bits, hi = (int)(uint32_t)(bits >> 32);
#pragma unroll
        for (int l = 0; l < 64; l++) {
          const double x = __builtin_bit_cast(
              double, (uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, l) << 32 |
                          (uint32_t)__builtin_amdgcn_readlane(lo, l));
          sum = __dadd_rn(sum, x);
        }
      }
      WN_T(4);
    };
    WN_T(0);
    WLd A, B;
    ld(s0, A);
    ld(s0 + kWChunk, B);
    for (uint32_t i0 = s0; i0 < end; i0 += 2u * kWChunk) {
      chunk(i0, A);
      ld(i0 + 2u * kWChunk, A);
      if (i0 + kWChunk >= end) break;
      chunk(i0 + kWChunk, B);
      ld(i0 + 3u * kWChunk, B);
    }
    // fold the counted records into the start state (:132-153)
    const uint32_t K = (uint32_t)__builtin_amdgcn_readfirstlane((int)WRing::wave_sum(kc));
    const uint32_t D = (uint32_t)__builtin_amdgcn_readfirstlane((int)WRing::wave_sum(ndup));
    if (K) {
      const uint32_t slo32 = (uint32_t)ssum;
      const uint64_t S = (uint64_t)WRing::wave_sum(slo32 & 0xFFFFu) +
                         ((uint64_t)WRing::wave_sum(slo32 >> 16) << 16) +
                         ((uint64_t)WRing::wave_sum((uint32_t)(ssum >> 32)) << 32);
      const uint32_t fmin = WRing::wave_min(fpos);
      const uint64_t who = __ballot(fpos == fmin);
      const uint32_t s1 = (uint32_t)__builtin_amdgcn_readlane((int)fsize, (int)__builtin_ctzll(who));
      const double rmin = WRing::wave_reduce_f64(cmn, inf, [](double x, double y) { return y < x ? y : x; });
      const double rmax = WRing::wave_reduce_f64(cmx, -inf, [](double x, double y) { return y > x ? y : x; });
      if (mc >= 2u) bc += S;
      else if (mc == 1u) bc = S;
      else bc = K == 1u ? (uint64_t)s1 : S - s1;
      if (mc == 0u) {
        lmin = rmin;
        lmax = rmax;
      } else {
        lmin = rmin < lmin ? rmin : lmin;
        lmax = rmax > lmax ? rmax : lmax;
      }
      mc += K;
    }
    sum = __builtin_bit_cast(double, (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(
                                         (int)(uint32_t)__builtin_bit_cast(uint64_t, sum)) |
                                     (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(
                                         (int)(uint32_t)(__builtin_bit_cast(uint64_t, sum) >> 32)) << 32);
    if (D && lane == 0) atomicAdd((unsigned long long*)&sp->dup_count, (unsigned long long)D);
    if (!open) {
      const uint32_t slot = rc0 + k;
      if (slot < per_flow && lane == 0) {
        const Tm rx = key_tm(recs[it.c].rxk), ws = key_tm(it.ws);
        const double duration = tdelta(rx, ws);
        uint64_t r_count;
        double r_rate, r_loss, r_min, r_max;
        if (mc == 0) {
          r_count = 0;
          r_rate = 0.0;
          r_loss = 1.0;
          r_min = r_max = -1.0;
        } else if (mc == 1) {
          r_count = 1;
          r_rate = __ddiv_rn((double)bc, duration);
          r_loss = 0.0;
          r_min = lmin;
          r_max = lmax;
        } else {
          r_count = mc - 1;
          r_rate = __ddiv_rn((double)bc, duration);
          const uint32_t delta = it.seqmax - it.sst;
          r_loss = delta <= 1 ? 0.0 : __dsub_rn(1.0, __ddiv_rn((double)mc, (double)(uint32_t)(delta + 1u)));
          r_min = lmin;
          r_max = lmax;
        }
        const size_t s = (size_t)f * per_flow + slot;
        mgenx_flow_report* rp = reports + s;
        rp->flow = f;
        rp->index = slot;
        rp->start_sec = ws.sec;
        rp->start_usec = ws.usec;
        rp->duration = duration;
        rp->msg_count = r_count;
        rp->rate = r_rate;
        rp->loss = r_loss;
        rp->latency_ave = mc == 0 ? -1.0 : mc == 1 ? sum : __ddiv_rn(sum, (double)mc);
        rp->latency_min = r_min;
        rp->latency_max = r_max;
        rp->rx_sec = rx.sec;
        rp->rx_usec = rx.usec;
        if (report_rec) report_rec[s] = order[it.c];
      }
    } else {  // the flow's state after the call: counters and the mask (bit i <-> F + i)
      const uint32_t F = fp->F;
      uint32_t word = 0;
      if (lane < 32u && fp->hasmask) {
#pragma unroll 8
        for (uint32_t j = 0; j < 32u; j++)
          word |= T[(F + lane * 32u + j) & 1023u] != kTabEmpty ? 1u << j : 0u;
      }
      const uint32_t nset = (uint32_t)__builtin_amdgcn_readfirstlane((int)WRing::wave_sum((uint32_t)__popc(word)));
      if (lane < 32u) sp->mask[lane] = word;
      if (lane == 0) {
        if (fp->hasmask) sp->mask_first = F;
        sp->mask_n = nset;
        sp->msg_count = mc;
        sp->byte_count = bc;
        sp->latency_min = lmin;
        sp->latency_max = lmax;
        sp->latency_sum = sum;
      }
    }
    wsync();
#if MGENX_DIAG
    WN_T(5);
    prof[6] = __builtin_amdgcn_s_memtime() - prof_t0;
    if (k == 1 && lane == 0 && atomicCAS(&g_win_claim, 0u, 1u) == 0u)
      for (int k2 = 0; k2 < 8; k2++) g_win_prof[k2] = prof[k2];
    for (int k2 = 0; k2 < 8; k2++) prof[k2] = 0;
#endif
  }
#undef WN_T
}

// ---- ordering the records by flow, stably: a counting sort (flow count < kCountBins) --
// The output is every record as the 24-B FRec the update reads, flow after flow, receive order
// kept within a flow (and, for report_rec, `order`: the input index at each sorted position).
//   hist:  per-tile flow histogram (kTile records per tile), stored tile-major
//          (hist[tile * bins + flow]);
//   scan:  the exclusive prefix of hist in flow-major order = where each (flow, tile) run
//          starts, also stored tile-major (flow_col* kernels below);
//   order: each record's position in its flow-sorted tile (stable: waves own contiguous
//          eighths, ranks inside a 64-record step from ballots on the key bits); the records are
//          then built from the caller's columns (or rows) read in input order -- coalesced --
//          into their sorted slots of the tile in LDS, and written out run by run, consecutive
//          lanes to consecutive slots.  (Gathering them in sorted order fetched a line per 4-B
//          column element: 405 us for config 4; scattering them from their input positions
//          wrote partial lines: 258 us.)  Tiles go to XCDs in contiguous ranges (blockIdx mod
//          8 = XCD), so the runs of one flow from neighbouring tiles meet in the same L2 and
//          leave it as whole lines.
// Records whose flow index is >= n_flows (MGENX_FLOW_NONE) go to the extra last bin and are
// not written.
constexpr uint32_t kSortWaves = 8;
constexpr uint32_t kTile = 4096;
constexpr uint32_t kPart = kTile / kSortWaves;
// LDS of the order kernel: 9 x bins x 4 bytes of counts and bases, the tile's records (24 B
// each) and their flows (2 B each) -- within 160 KiB up to 1536 bins
constexpr uint32_t kCountBins = 1536;
constexpr uint32_t kOrderLds = kCountBins * 9u * 4u + kTile * (uint32_t)sizeof(FRec) + kTile * 2u;

__global__ void __launch_bounds__(512)
flow_hist_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows, uint32_t n_tiles,
                 uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h[];
  const uint32_t bins = n_flows + 1u;
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) h[k] = 0u;
  __syncthreads();
  const uint32_t a = blockIdx.x * kTile, e = min(n, a + kTile);
  // kHistU keys per thread and pass, all loads issued before any is used
  constexpr uint32_t kHistU = 8;
  for (uint32_t i0 = a + threadIdx.x; i0 < e; i0 += kHistU * blockDim.x) {
    uint32_t fi[kHistU];
#pragma unroll
    for (uint32_t u = 0; u < kHistU; u++) fi[u] = idx[min(i0 + u * blockDim.x, e - 1u)];
#pragma unroll
    for (uint32_t u = 0; u < kHistU; u++)
      if (i0 + u * blockDim.x < e) atomicAdd(&h[min(fi[u], n_flows)], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) hist[(size_t)blockIdx.x * bins + k] = h[k];
}

// inclusive prefix sum over the wave's 64 lanes in DPP steps (rows of 16 by shifts, then the
// row broadcasts) -- no LDS round trips, unlike __shfl_up
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// LDS-only block barrier: the block's LDS accesses before it are complete after it, while its
// global loads and stores stay in flight (__syncthreads' workgroup fence waits for every
// outstanding global access too, which would drain the next tile's prefetch)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr uint32_t kOrdStart = (kCountBins + 511u) / 512u;  // start entries per thread
#if MGENX_DIAG
// (diagnostics) cycles of flow_order_kernel's block 0, wave 0 by phase: zero, scan (incl. the
// count barrier), ranks + placement, prefetch issue, writes, tiles, count (incl. the key wait),
// total
__device__ unsigned long long g_ord_prof[8];
#define ORD_T(slot)                                                        \
  do {                                                                     \
    if (prof_on) {                                                         \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();        \
      prof[slot] += now_ - prof_t;                                         \
      prof_t = now_;                                                       \
    }                                                                      \
  } while (0)
#else
#define ORD_T(slot) \
  do {              \
  } while (0)
#endif

// Persistent: one block per CU walks its tiles, and the next tile's keys, start row and raw
// records are loaded while the current tile's runs are written, so the reads of one tile and
// the writes of the one before share the memory system (one tile per block and phase after
// phase left the chip reading, then writing: 190 us for config 4).
template <bool kRows>
__global__ void __launch_bounds__(512)
flow_order_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows,
                  uint32_t n_tiles, const uint32_t* __restrict__ start, RecSrc src,
                  FRec* __restrict__ recs, uint32_t* __restrict__ order, uint32_t key_bits,
                  uint32_t seqw) {  // diagnostics timing only (tile-contiguous writes, wrong)
  extern __shared__ uint32_t lds[];
  const uint32_t bins = n_flows + 1u;
  uint32_t* cnt = lds;                                // [wave][bin]: counts, then run bases
  uint32_t* sbase = lds + kSortWaves * bins;          // [bin]: start - tile offset
  FRec* lrec = reinterpret_cast<FRec*>(sbase + bins + (bins & 1u));  // 8-byte aligned
  uint16_t* lkey = reinterpret_cast<uint16_t*>(lrec + kTile);
  __shared__ uint32_t wsum[kSortWaves];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  // tiles: XCD x (block b runs on XCD b % 8) owns tiles [x * per, (x + 1) * per), its nb blocks
  // take them nb apart, so the tiles in flight on one XCD are neighbours and the runs of one
  // flow from adjacent tiles meet in that XCD's L2
  const uint32_t per = (n_tiles + 7u) / 8u, nb = gridDim.x >> 3;
  const uint32_t xb = (blockIdx.x & 7u) * per;
  uint32_t ci = blockIdx.x >> 3;
  if (ci >= per || xb + ci >= n_tiles) return;  // whole block: no barrier is reached by anyone
  uint32_t t = xb + ci;
  uint32_t* my = cnt + w * bins;
  uint64_t* tab = reinterpret_cast<uint64_t*>(lrec) + (size_t)w * kCountBins;
  constexpr uint32_t kKeys = kPart / 64u;
  // scan ownership: thread tid owns bins [k0, k1)
  const uint32_t B = (bins + blockDim.x - 1u) / blockDim.x;
  const uint32_t k0 = min(tid * B, bins), k1 = min(k0 + B, bins);
  uint32_t keys[kKeys], st[kOrdStart];
  RawRec raw[kKeys];
  // the wave's kPart keys, the tile's start row (this thread's bins) and its raw records, all
  // issued together (clamped indices: no branch, nothing waits here)
  // (live == false: the last pass's prefetch, every lane on element 0 -- one line, so the
  // loads still land in the loop's registers without re-reading a tile)
  auto fetch = [&](uint32_t tt, bool live) {
    const uint32_t a = tt * kTile + w * kPart;
    uint32_t ii[kKeys];
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) ii[j] = live ? min(a + 64u * j + lane, n - 1u) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) keys[j] = __builtin_nontemporal_load(idx + ii[j]);
#pragma unroll
    for (uint32_t q = 0; q < kOrdStart; q++)
      st[q] = start[live ? (size_t)tt * bins + min(k0 + q, bins - 1u) : 0];
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) raw[j] = load_rec_t<kRows>(src, ii[j]);
  };
  fetch(t, true);
  for (uint32_t k = tid; k < kSortWaves * bins; k += blockDim.x) cnt[k] = 0u;
  const uint64_t lt = (1ull << lane) - 1ull;
#if MGENX_DIAG
  const bool prof_on = blockIdx.x == 0 && w == 0;
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memtime();
  const unsigned long long prof_t0 = prof_t;
#endif
  while (true) {
    const uint32_t t0 = t * kTile;
    const uint32_t a = t0 + w * kPart, e = min(n, a + kPart);
    lds_barrier();  // (every wave is past the last tile's writes, which read lrec, and zeroing)
    ORD_T(0);
    // the wave's peer table (in lrec, free until the placement): tab[key] collects the lanes
    // of one 64-record step holding that key
    for (uint32_t k = lane; k < bins; k += 64u) tab[k] = 0ull;
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) {
      keys[j] = a + 64u * j + lane < e ? min(keys[j], n_flows) : 0xFFFFFFFFu;
      if (keys[j] != 0xFFFFFFFFu) atomicAdd(&my[keys[j]], 1u);
    }
    ORD_T(6);
    lds_barrier();
    // tile offsets: exclusive scan over bins of the tile's counts
    uint32_t local = 0;
    for (uint32_t k = k0; k < k1; k++)
#pragma unroll
      for (uint32_t v = 0; v < kSortWaves; v++) local += cnt[v * bins + k];
    const uint32_t incl = wave_incl_scan(local);
    if (lane == 63u) wsum[w] = incl;
    lds_barrier();
    uint32_t run = incl - local;
    for (uint32_t v = 0; v < w; v++) run += wsum[v];
#pragma unroll
    for (uint32_t q = 0; q < kOrdStart; q++) {
      const uint32_t k = k0 + q;
      if (k < k1) {
        sbase[k] = st[q] - run;
#pragma unroll
        for (uint32_t v = 0; v < kSortWaves; v++) {
          const uint32_t c = cnt[v * bins + k];
          cnt[v * bins + k] = run;
          run += c;
        }
      }
    }
    lds_barrier();
    ORD_T(1);
    // each record's position in the flow-sorted tile, stable: waves own contiguous eighths,
    // and inside a 64-record step a record's rank is the number of lower lanes with its key.
    // The lanes with one key (`peers`) come from the wave's table (OR in the lane bits, read,
    // clear: same-wave LDS operations complete in order, and these relaxed atomics on
    // possibly-equal addresses keep program order); the last lane of each group adds the
    // group's size to the key's running base and the group reads the old base from it.
    uint64_t peers[kKeys];
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) {
      peers[j] = 0ull;
      if (keys[j] != 0xFFFFFFFFu) {
        uint64_t* slot = &tab[keys[j]];
        __hip_atomic_fetch_or(slot, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        peers[j] = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
    }
    uint32_t pos[kKeys], old[kKeys];
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) {  // all the adds in flight together ...
      const uint32_t rank = (uint32_t)__popcll(peers[j] & lt);
      const uint32_t size = (uint32_t)__popcll(peers[j]);
      old[j] = 0u;
      if (keys[j] != 0xFFFFFFFFu && rank + 1u == size)
        old[j] = __hip_atomic_fetch_add(&my[keys[j]], size, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_WAVEFRONT);
      pos[j] = rank;
    }
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) {  // ... then the bases to the groups
      const uint32_t last = 63u - (uint32_t)__builtin_clzll(peers[j] | 1ull);
      pos[j] += (uint32_t)__shfl((int)old[j], (int)last);
    }
    // the peer table's slots are about to be overwritten by the records: every lane of the
    // wave is past its last table access once its own ops have completed (in order), but other
    // waves' tables overlap this wave's record slots
    lds_barrier();
    // the records built (latency, input index - t0 in the high half of `len`, for `order`)
    // into their slots
#pragma unroll
    for (uint32_t j = 0; j < kKeys; j++) {
      if (keys[j] != 0xFFFFFFFFu) {
        const uint32_t i = a + 64u * j + lane;
        FRec r = build_frec(raw[j]);
        r.len |= (i - t0) << 16;
        lrec[pos[j]] = r;
        lkey[pos[j]] = (uint16_t)keys[j];
      }
    }
    lds_barrier();
    ORD_T(2);
    // the next tile's loads go out before this tile's stores (unconditionally, so the loads
    // land in the loop's registers with no copy, which would wait for them)
    ci += nb;
    const bool more = ci < per && xb + ci < n_tiles;
    fetch(more ? xb + ci : t, more);
    ORD_T(3);
    // the counts of the next tile start from zero (the ranks above were the last use)
    for (uint32_t k = tid; k < kSortWaves * bins; k += blockDim.x) cnt[k] = 0u;
    // this tile's runs: consecutive lanes, consecutive slots (whole lines but at the runs'
    // ends; runs of one flow from neighbouring tiles meet in L2).  (As 8-B words, consecutive
    // lanes on consecutive words, the stores cover contiguous 512 B each but take 24 per
    // thread and three LDS reads a word: slower, 134 vs 130 us for config 4.)
    const uint32_t tn = min(n - t0, kTile);
#pragma unroll
    for (uint32_t u = 0; u < kTile / 512u; u++) {
      const uint32_t j = tid + 512u * u;
      const uint32_t k = j < tn ? lkey[j] : 0xFFFFu;
      if (k < n_flows) {
        FRec r = lrec[j];
        const uint32_t g = seqw ? t0 + j : sbase[k] + j;
        if (order) order[g] = t0 + (r.len >> 16);
        r.len &= 0xFFFFu;
        recs[g] = r;
      }
    }
    ORD_T(4);
#if MGENX_DIAG
    prof[5]++;
#endif
    if (!more) break;
    t = xb + ci;
  }
#if MGENX_DIAG
  if (prof_on && lane == 0) {
    prof[7] = __builtin_amdgcn_s_memtime() - prof_t0;
    for (int k2 = 0; k2 < 8; k2++) g_ord_prof[k2] = prof[k2];
  }
#endif
}

// scan: start[t * bins + k] = where flow k's records of tile t go -- the exclusive prefix of
// the tile-major histogram hist[t * bins + k] taken in flow-major order (flow k's runs tile
// after tile, flows one after another).  Tile-major, so the histogram kernel writes and the
// order kernel reads one tile's bins contiguously (flow-major arrays made both of them
// strided: one line per 4-B entry), and start[k] (tile 0) is flow k's first sorted position:
// the bounds the update kernels read (stride 1).  Three small kernels over chunks of
// kColTiles tiles: chunk partial sums per flow; one block for the flow totals and their
// exclusive scan; the chunk scans (each from its flow's base plus the earlier chunks).
constexpr uint32_t kColTiles = 64;
__global__ void __launch_bounds__(256)
flow_colpart_kernel(const uint32_t* __restrict__ hist, uint32_t bins, uint32_t n_tiles,
                    uint32_t* __restrict__ part) {
  const uint32_t k = blockIdx.x * 256u + threadIdx.x, c = blockIdx.y;
  if (k >= bins) return;
  const uint32_t t0 = c * kColTiles, t1 = min(n_tiles, t0 + kColTiles);
  uint32_t s = 0;
  uint32_t t = t0;
  for (; t + 8u <= t1; t += 8u) {
    uint32_t x[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) x[u] = hist[(size_t)(t + u) * bins + k];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) s += x[u];
  }
  for (; t < t1; t++) s += hist[(size_t)t * bins + k];
  part[(size_t)c * bins + k] = s;
}

// one block: base[k] = records of the flows before k (all chunks' partials summed, then an
// exclusive scan over the flows; bins <= 2048, two per thread)
__global__ void __launch_bounds__(1024)
flow_colbase_kernel(const uint32_t* __restrict__ part, uint32_t bins, uint32_t n_chunks,
                    uint32_t* __restrict__ base) {
  __shared__ uint32_t ws[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  uint32_t tot[2] = {0u, 0u};
#pragma unroll
  for (uint32_t j = 0; j < 2; j++) {
    const uint32_t k = 2u * tid + j;
    if (k < bins) {
      uint32_t c = 0;
      for (; c + 8u <= n_chunks; c += 8u) {
        uint32_t x[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) x[u] = part[(size_t)(c + u) * bins + k];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) tot[j] += x[u];
      }
      for (; c < n_chunks; c++) tot[j] += part[(size_t)c * bins + k];
    }
  }
  const uint32_t mine = tot[0] + tot[1];
  uint32_t incl = mine;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63u) ws[w] = incl;
  __syncthreads();
  uint32_t b = incl - mine;
  for (uint32_t v = 0; v < w; v++) b += ws[v];
  if (2u * tid < bins) base[2u * tid] = b;
  if (2u * tid + 1u < bins) base[2u * tid + 1u] = b + tot[0];
}

__global__ void __launch_bounds__(256)
flow_colscan_kernel(const uint32_t* __restrict__ hist, const uint32_t* __restrict__ part,
                    const uint32_t* __restrict__ base, uint32_t bins, uint32_t n_tiles,
                    uint32_t* __restrict__ start) {
  const uint32_t k = blockIdx.x * 256u + threadIdx.x, c = blockIdx.y;
  if (k >= bins) return;
  const uint32_t t0 = c * kColTiles, t1 = min(n_tiles, t0 + kColTiles);
  uint32_t run = base[k];  // + flow k's records in the chunks before c
  {
    uint32_t c2 = 0;
    for (; c2 + 8u <= c; c2 += 8u) {
      uint32_t x[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) x[u] = part[(size_t)(c2 + u) * bins + k];
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) run += x[u];
    }
    for (; c2 < c; c2++) run += part[(size_t)c2 * bins + k];
  }
  uint32_t t = t0;
  for (; t + 8u <= t1; t += 8u) {
    uint32_t x[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) x[u] = hist[(size_t)(t + u) * bins + k];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) {
      start[(size_t)(t + u) * bins + k] = run;
      run += x[u];
    }
  }
  for (; t < t1; t++) {
    start[(size_t)t * bins + k] = run;
    run += hist[(size_t)t * bins + k];
  }
}

// ---- the general ordering (any flow count): hipCUB radix sort of (flow, record) pairs ----
// keys: flow index clamped to n_flows (records to skip sort last); vals: record index
__global__ void flow_keys_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows,
                                 uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = min(idx[i], n_flows);
  vals[i] = i;
}

// the sorted records of the radix path: position p < bnd[n_flows] gets record order[p]
__global__ void flow_gather_kernel(const uint32_t* __restrict__ order, const uint32_t* __restrict__ bnd,
                                   uint32_t n_flows, RecSrc src, FRec* __restrict__ recs) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= bnd[n_flows]) return;
  recs[p] = make_frec(src, order[p]);
}

// run starts: bnd[f] = first sorted position with flow >= f (f = 0..n_flows)
__global__ void flow_bounds_kernel(const uint32_t* __restrict__ keys, uint32_t n, uint32_t n_flows,
                                   uint32_t* __restrict__ bnd) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f > n_flows) return;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2u;
    if (keys[mid] < f) lo = mid + 1u;
    else hi = mid;
  }
  bnd[f] = lo;
}

// fresh states: zero but window_size, written as 16-B units by consecutive lanes (one lane per
// state stored a 256-B struct per lane: 64 lines per store instruction)
static_assert(sizeof(mgenx_flow_state) % 16 == 0, "flow state in 16-B units");
static_assert(offsetof(mgenx_flow_state, window_size) % 8 == 0, "window_size 8-B aligned");
__global__ void flow_init_kernel(mgenx_flow_state* flows, uint32_t n_flows, double window) {
  constexpr uint32_t kUnits = sizeof(mgenx_flow_state) / 16u;
  constexpr uint32_t kWin = offsetof(mgenx_flow_state, window_size);
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (uint64_t)n_flows * kUnits) return;
  const uint32_t b = (uint32_t)(u % kUnits) * 16u;  // byte offset of this unit in its state
  const uint64_t w = __builtin_bit_cast(uint64_t, window);
  u32x4_t v = {0u, 0u, 0u, 0u};
  if (b == (kWin & ~15u)) {
    if (kWin % 16u == 0u) {
      v.x = (uint32_t)w;
      v.y = (uint32_t)(w >> 32);
    } else {
      v.z = (uint32_t)w;
      v.w = (uint32_t)(w >> 32);
    }
  }
  reinterpret_cast<u32x4_t*>(flows)[u] = v;
}

__global__ void flow_export_kernel(const mgenx_flow_state* __restrict__ flows, uint32_t n_flows,
                                   mgenx_flow_counters* __restrict__ out) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_flows) return;
  const mgenx_flow_state& s = flows[f];
  mgenx_flow_counters c;
  c.msg_count = s.msg_count;
  c.byte_count = s.byte_count;
  c.dup_count = s.dup_count;
  c.n_reports = s.n_reports;
  c.latency_sum = s.latency_sum;
  c.latency_min = s.latency_min;
  c.latency_max = s.latency_max;
  c.seq_start = s.seq_start;
  out[f] = c;
}

}  // namespace mgenx

// ------------------------------------------------------------------------------------
// host side (workspace owned by the context; see mgenx_api.hip)
// ------------------------------------------------------------------------------------
using namespace mgenx;

struct mgenx_flow_ws {
  void* mem = nullptr;
  size_t bytes = 0;
  uint32_t cu = 0;  // the device's CU count (the order kernel's persistent grid)
};

extern "C" void* mgenx_flow_ws_new() { return new mgenx_flow_ws(); }
extern "C" void mgenx_flow_ws_free(void* p) {
  mgenx_flow_ws* w = static_cast<mgenx_flow_ws*>(p);
  if (!w) return;
  mgenx::dev_free(w->mem);
  delete w;
}

// Report::QuantizeTimeValue / UnquantizeTimeValue round trip (mgenAnalytic.cpp:621-642),
// as the oracle's or_quantized_window.
static double quantized_window(double value) {
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

#if MGENX_DIAG
extern "C" int mgenx_diag_seg_prof(unsigned long long* out, int n) {
  if (out && n == 8) {  // flow_skel_kernel's phase cycles (g_skel_prof; the claim reset)
    const unsigned int zero = 0;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_skel_prof), 64) != hipSuccess) return MGENX_EDEVICE;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_skel_claim), &zero, 4) == hipSuccess ? MGENX_OK
                                                                               : MGENX_EDEVICE;
  }
  if (out && n == 12) {  // flow_win_kernel's phase cycles (g_win_prof; the claim reset)
    const unsigned int zero = 0;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_win_prof), 64) != hipSuccess) return MGENX_EDEVICE;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_win_claim), &zero, 4) == hipSuccess ? MGENX_OK
                                                                              : MGENX_EDEVICE;
  }
  if (out && n == 16)  // flow_order_kernel's phase cycles (g_ord_prof, 8 entries)
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ord_prof), 64) == hipSuccess ? MGENX_OK
                                                                              : MGENX_EDEVICE;
  return MGENX_EINVAL;
}
#endif

extern "C" int mgenx_flow_init_run(mgenx_flow_state* flows, uint32_t n_flows, double window,
                                   hipStream_t stream) {
  if (!n_flows) return MGENX_OK;
  const uint64_t units = (uint64_t)n_flows * (sizeof(mgenx_flow_state) / 16u);
  hipLaunchKernelGGL(flow_init_kernel, dim3((uint32_t)((units + 255) / 256)), dim3(256), 0, stream, flows,
                     n_flows, quantized_window(window));
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

extern "C" int mgenx_flow_export_run(const mgenx_flow_state* flows, uint32_t n_flows,
                                     mgenx_flow_counters* out, hipStream_t stream) {
  if (!n_flows) return MGENX_OK;
  hipLaunchKernelGGL(flow_export_kernel, dim3((n_flows + 255) / 256), dim3(256), 0, stream,
                     flows, n_flows, out);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" int mgenx_flow_reduce_run(void* wsp, const uint32_t* flow_idx, const uint32_t* seq,
                                     const uint32_t* txs, const uint32_t* txu, const uint16_t* len,
                                     const mgenx_rec* rows, const uint32_t* rxs, const uint32_t* rxu, uint32_t n,
                                     mgenx_flow_state* flows, uint32_t n_flows,
                                     mgenx_flow_report* reports, uint32_t per_flow,
                                     uint32_t* report_count, uint32_t* report_rec,
                                     hipStream_t stream, char* err, size_t errn) {
  mgenx_flow_ws& ws = *static_cast<mgenx_flow_ws*>(wsp);
  if (n == 0 || n_flows == 0) return MGENX_OK;
  const RecSrc src = {seq, txs, txu, len, rows, rxs, rxu};
  int sort_path = (uint64_t)n_flows + 1 <= kCountBins ? 0 : 1;  // 0 counting, 1 radix
  int sabl = 0;      // diagnostics build only: ordering-only timing (MGENX_AN_SABL)
  uint32_t oseqw = 0;  // diagnostics build only: order kernel writes tile-contiguous (MGENX_AN_SEQW)
#if MGENX_DIAG
  if (const char* sp = getenv("MGENX_AN_RADIX")) sort_path = atoi(sp) ? 1 : sort_path;
  if (const char* sa = getenv("MGENX_AN_SABL")) sabl = atoi(sa);
  if (const char* sw = getenv("MGENX_AN_SEQW")) oseqw = (uint32_t)atoi(sw);
#endif
  const uint32_t bins = n_flows + 1u;
  uint32_t key_bits = 1;
  while (key_bits < 32 && (1ull << key_bits) <= n_flows) key_bits++;
  const uint32_t n_tiles = (n + kTile - 1) / kTile;
  const size_t n_hist = (size_t)bins * n_tiles;
  size_t cub_bytes = 0;
  if (sort_path == 0)  // the chunk partials and their prefixes
    cub_bytes = (size_t)2u * ((n + kTile - 1) / kTile + kColTiles - 1u) / kColTiles * bins * 4u;
  else
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (int)n, 0, (int)key_bits, stream);
  const bool want_order = report_rec != nullptr;
  const size_t nb = a256((size_t)n * 4), rb = a256((size_t)n * sizeof(FRec));
  const size_t hb = a256(n_hist * 4), bb = a256((size_t)bins * 4);
  const size_t fb = a256((size_t)n + 256), wb = a256(((size_t)n + n_flows) * sizeof(WinItem));
  const size_t xb = a256((size_t)n_flows * sizeof(FlowFin));
  // both: records (sorted), record flags, windows, per-flow results
  // counting: hist, start, order (report_rec only), row totals
  // radix:    keys_in, keys_out, vals_in, order, bounds, cub
  const size_t common = rb + fb + wb + xb;
  const size_t need = common + (sort_path == 0 ? 2 * hb + (want_order ? nb : 0) + a256(cub_bytes)
                                               : 4 * nb + bb + a256(cub_bytes));
  if (ws.bytes < need) {
    mgenx::dev_free(ws.mem);
    ws.mem = nullptr;
    ws.bytes = 0;
    if (hipMalloc(&ws.mem, need) != hipSuccess) {
      snprintf(err, errn, "flow_reduce: workspace of %zu bytes", need);
      return MGENX_EDEVICE;
    }
    ws.bytes = need;
  }
  char* p = static_cast<char*>(ws.mem);
  auto take = [&](size_t b) { char* q = p; p += b; return q; };
  FRec* recs = (FRec*)take(rb);
  uint8_t* rflags = (uint8_t*)take(fb);
  WinItem* wins = (WinItem*)take(wb);
  FlowFin* fin = (FlowFin*)take(xb);
  const uint32_t* bnd;
  uint32_t* order = nullptr;
  hipError_t e;
  if (sort_path == 0) {
    uint32_t* hist = (uint32_t*)take(hb);
    uint32_t* start = (uint32_t*)take(hb);
    if (want_order) order = (uint32_t*)take(nb);
    uint32_t* totals = (uint32_t*)take(a256(cub_bytes));
    hipLaunchKernelGGL(flow_hist_kernel, dim3(n_tiles), dim3(512), bins * 4u, stream, flow_idx, n,
                       n_flows, n_tiles, hist);
    const uint32_t n_chunks = (n_tiles + kColTiles - 1u) / kColTiles;
    const dim3 cg((bins + 255u) / 256u, n_chunks);
    hipLaunchKernelGGL(flow_colpart_kernel, cg, dim3(256), 0, stream, hist, bins, n_tiles, totals);
    hipLaunchKernelGGL(flow_colbase_kernel, dim3(1), dim3(1024), 0, stream, totals, bins, n_chunks,
                       totals + (size_t)n_chunks * bins);
    hipLaunchKernelGGL(flow_colscan_kernel, cg, dim3(256), 0, stream, hist, totals,
                       totals + (size_t)n_chunks * bins, bins, n_tiles, start);
    e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(err, errn, "flow_reduce scan: %s", hipGetErrorString(e));
      return MGENX_EDEVICE;
    }
    // LDS: per-wave counts, the run bases, the tile's records and their flows
    const uint32_t lds = (kSortWaves * bins + bins + (bins & 1u)) * 4u +
                         kTile * (uint32_t)sizeof(FRec) + kTile * 2u;
    const void* okern = src.rows ? (const void*)flow_order_kernel<true>
                                 : (const void*)flow_order_kernel<false>;
    e = set_max_lds(okern, (int)kOrderLds + 8);
    if (e != hipSuccess) {
      snprintf(err, errn, "flow_reduce order: %s", hipGetErrorString(e));
      return MGENX_EDEVICE;
    }
    // persistent: one block per CU (LDS allows one), a multiple of 8 (one set per XCD)
    if (!ws.cu) {
      int dev = 0, cu = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cu = 256;
      ws.cu = (uint32_t)max(8, cu);
    }
    const uint32_t grid = 8u * min((n_tiles + 7u) / 8u, ws.cu / 8u);
    if (src.rows)
      hipLaunchKernelGGL(flow_order_kernel<true>, dim3(grid), dim3(64 * kSortWaves), lds, stream,
                         flow_idx, n, n_flows, n_tiles, start, src, recs, order, key_bits, oseqw);
    else
      hipLaunchKernelGGL(flow_order_kernel<false>, dim3(grid), dim3(64 * kSortWaves), lds, stream,
                         flow_idx, n, n_flows, n_tiles, start, src, recs, order, key_bits, oseqw);
    bnd = start;  // tile 0's row: flow k starts at start[k]
  } else {
    uint32_t* keys_in = (uint32_t*)take(nb);
    uint32_t* keys_out = (uint32_t*)take(nb);
    uint32_t* vals_in = (uint32_t*)take(nb);
    order = (uint32_t*)take(nb);
    uint32_t* d_bnd = (uint32_t*)take(bb);
    void* cub_tmp = take(a256(cub_bytes));
    hipLaunchKernelGGL(flow_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, flow_idx, n,
                       n_flows, keys_in, vals_in);
    e = hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, keys_in, keys_out, vals_in, order,
                                           (int)n, 0, (int)key_bits, stream);
    if (e != hipSuccess) {
      snprintf(err, errn, "flow_reduce sort: %s", hipGetErrorString(e));
      return MGENX_EDEVICE;
    }
    hipLaunchKernelGGL(flow_bounds_kernel, dim3((bins + 255) / 256), dim3(256), 0, stream, keys_out,
                       n, n_flows, d_bnd);
    hipLaunchKernelGGL(flow_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, order,
                       d_bnd, n_flows, src, recs);
    bnd = d_bnd;
  }
  if (sabl) return MGENX_OK;  // timing study: ordering only
  e = set_max_lds((const void*)flow_skel_kernel, (int)kSkLds);
  if (e != hipSuccess) {
    snprintf(err, errn, "flow_reduce skeleton: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  // block -> flow multiplier: odd, near 0.618 n_flows, coprime with n_flows (a permutation)
  uint32_t fmul = n_flows > 2 ? (uint32_t)(0.6180339887 * n_flows) | 1u : 1u;
  auto gcd = [](uint32_t x, uint32_t y) { while (y) { const uint32_t t = x % y; x = y; y = t; } return x; };
  while (fmul > 1 && gcd(fmul, n_flows) != 1) fmul -= 2;
  if (fmul == 0) fmul = 1;
  hipLaunchKernelGGL(flow_skel_kernel, dim3(n_flows), dim3(256), kSkLds, stream, flows, n_flows,
                     fmul, bnd, recs, rflags, wins, fin, report_count);
  hipLaunchKernelGGL(flow_win_kernel, dim3(n_flows * kWinWaves), dim3(64), 0, stream, flows,
                     n_flows, bnd, recs, rflags, wins, fin, reports, per_flow, report_rec, order);
  e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err, errn, "flow_reduce: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  return MGENX_OK;
}
