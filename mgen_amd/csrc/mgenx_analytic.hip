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
// a copy the compiler cannot see through (one v_mov per dword)
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x) {
  uint32_t y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
__device__ __forceinline__ FRec opaque_frec(const FRec& a) {
  FRec r;
  r.rxk = (uint64_t)opaque_u32((uint32_t)(a.rxk >> 32)) << 32 | opaque_u32((uint32_t)a.rxk);
  r.seq = opaque_u32(a.seq);
  r.len = opaque_u32(a.len);
  const uint64_t lb = __builtin_bit_cast(uint64_t, a.latency);
  r.latency = __builtin_bit_cast(double, (uint64_t)opaque_u32((uint32_t)(lb >> 32)) << 32 |
                                             opaque_u32((uint32_t)lb));
  return r;
}
__device__ __forceinline__ FRec make_frec(const RecSrc& src, uint32_t i) {
  return build_frec(load_rec(src, i));
}

// What the latency sums (the update's tail) need per kept report closed in this call
struct CloseRec {
  uint32_t pos, zr;     // the closing record (sorted position); zero restart
  uint64_t mc;          // msg_count at the close: latency_ave's divisor
};

// ---- MgenAnalytic::Update, one WAVE per flow (mgenAnalytic.cpp:74-258) ----
// The latency sum is the one FP64 chain whose rounding depends on record order; everything
// else here is integer bookkeeping and order-free min / max.  So the update walks its flow's
// records 256 at a time (4 per lane, coalesced) and leaves the sum to its tail: each
// record's contribution to latency_sum ("lat'": its latency when Update adds or assigns it, else
// 0.0) goes to lat2[], the closing records and the window msg_counts to CloseRec.  Since
// latency_sum is 0.0 whenever msg_count is 0, every assignment of a latency to it is an add to
// 0.0 (exact), and a window's sum is the in-order sum of its records' lat' values -- a window
// restarts at its closing record's lat' (0.0 for the closing "first actual message" of
// :165-173, whose local `latency` stays 0.0).
//
// Bulk runs: from the current state, a record is "simple" when it does not reach the window end
// and, if msg != 0, lies inside the mask span (0 <= seq - first < 1024: Set takes its in-span
// branch and never clears, `first` does not move).  A run of simple records changes the state in
// closed form: a record is a duplicate when its ring bit is set or an earlier record of the run
// has its sequence number (an LDS scatter finds clashes; then an LDS table of first positions
// orders them), else it sets its bit; those at or past seq_start are counted.  Counts move by
// ballots, bytes / min / max / last by per-lane partials folded before an exact step (flush).
// The first non-simple record (window end, mask restart, a record below `first`, an empty mask,
// the first record of a flow) takes the exact update below, and the run restarts after it.
#if MGENX_DIAG
// (diagnostics) cycles of flow_update_kernel's first wave by phase: detect, bulk, exact, lat'
// store, rounds, exact steps, bulk runs, total
__device__ unsigned long long g_upd_prof[10];  // + [8] restart cycles, [9] restarts
#define UPD_T(slot)                                                        \
  do {                                                                     \
    if (prof_on) {                                                         \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();        \
      prof[slot] += now_ - prof_t;                                         \
      prof_t = now_;                                                       \
    }                                                                      \
  } while (0)
#else
#define UPD_T(slot) \
  do {              \
  } while (0)
#endif
constexpr uint32_t kUR = 4;             // records per lane and round
constexpr uint32_t kRound = 64u * kUR;  // records per round
constexpr uint32_t kPiece = 4u * kRound;  // lat' staged in LDS per step of the tail's sums

__global__ void __launch_bounds__(256)
flow_update_kernel(mgenx_flow_state* __restrict__ flows, uint32_t n_flows,
                   const uint32_t* __restrict__ bnd, uint32_t bstride, const FRec* __restrict__ recs,
                   const uint32_t* __restrict__ order, double* __restrict__ lat2,
                   mgenx_flow_report* __restrict__ reports, uint32_t per_flow,
                   uint32_t* __restrict__ report_count, uint32_t* __restrict__ report_rec,
                   CloseRec* __restrict__ closes,
                   uint32_t lat2_sink) {
  __shared__ uint32_t scat[4][32];
  __shared__ uint32_t fo[4][1024];
  __shared__ double lbuf[4][kPiece];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t f = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + wv);
  if (f >= n_flows) return;
  const uint32_t b = bnd[(size_t)f * bstride], e = bnd[(size_t)(f + 1u) * bstride];
  if (b >= e) return;
  for (uint32_t j = lane; j < 1024u; j += 64u) fo[wv][j] = 0xFFFFFFFFu;
  mgenx_flow_state* sp = flows + f;
  const TAdd window = tadd_of(sp->window_size);
  WRing m;
  m.lane = lane;
  m.first = sp->mask_first;
  m.n = sp->mask_n;
  m.load_relative(sp->mask);
  if (!m.n) m.w = 0;
  bool valid = sp->window_valid != 0;
  Tm ws = {sp->win_start_sec, sp->win_start_usec}, we = {sp->win_end_sec, sp->win_end_usec};
  uint64_t wek = tkey(we);
  uint32_t seq_start = sp->seq_start;
  uint64_t msg_count = sp->msg_count, byte_count = sp->byte_count, dups = sp->dup_count;
  double lmin = sp->latency_min, lmax = sp->latency_max;
  uint64_t nrep = sp->n_reports;
  const double lsum0 = sp->latency_sum;
  const uint32_t rc0 = report_count ? report_count[f] : 0u;  // (null: per_flow == 0)
  uint32_t rcount = rc0, ncl = 0, last_close = 0, last_zr = 0;

  // the exact Update of one record (arguments wave-uniform); returns the record's lat'
  auto update = [&](uint32_t seq, uint64_t rxk, uint32_t msg, double lat, uint32_t pos) -> double {
    const Tm rx = {(int64_t)(rxk >> 32), (int64_t)(uint32_t)rxk};
    if (!valid) {  // mgenAnalytic.cpp:80-99
      valid = true;
      ws = rx;
      we = uni_t(tadd(rx, window));
      wek = tkey(we);
      if (msg != 0) {
        m.set(seq);
        seq_start = seq;
        msg_count = 1;
        byte_count = msg;
        lmin = lmax = lat;
        return lat;
      }
      msg_count = byte_count = 0;
      lmin = lmax = 0.0;
      return 0.0;
    }
    double latency = 0.0, contrib = 0.0;
    uint32_t zr = 0;
    if (msg != 0) {  // :102-178
      if (m.n) {
        if (m.test(seq)) {
          dups++;
        } else if ((int32_t)(seq - seq_start) < 0) {
          m.set(seq);
        } else {
          if (!m.set(seq)) {  // UnsetBits(first, seq - first), then Set (:120-127)
            m.unset_from_first(seq - m.first);
            m.set(seq);
          }
          if (1 == msg_count) byte_count = msg;
          else byte_count += msg;
          latency = contrib = lat;
          if (0 == msg_count) {
            lmin = lmax = latency;
          } else {
            // as value selects (a branch here lets LLVM fold the two stores into one store
            // through a selected pointer, which sends lmin/lmax to scratch memory)
            const bool lo = latency < lmin;
            const bool hi = !lo && latency > lmax;
            lmin = lo ? latency : lmin;
            lmax = hi ? latency : lmax;
          }
          msg_count++;
        }
      } else {  // the first actual message (:165-173): sets the sum, `latency` stays 0.0
        m.clear();
        m.set(seq);
        seq_start = seq;
        byte_count = msg;
        lmin = lmax = lat;
        msg_count = 1;
        contrib = lat;
        zr = 1;
      }
    }
    if (tge(rx, we)) {  // :180-256: report and restart the window
      const uint32_t seq_max = m.n ? m.get_last() : seq_start;
      if (rcount < per_flow) {  // a kept report (latency_ave: the tail below)
      const double duration = tdelta(rx, ws);
      uint64_t r_count;
      double r_rate, r_loss, r_min, r_max;
      if (msg_count == 0) {
        r_count = 0;
        r_rate = 0.0;
        r_loss = 1.0;
        r_min = r_max = -1.0;
      } else if (msg_count == 1) {
        r_count = 1;
        r_rate = __ddiv_rn((double)byte_count, duration);
        r_loss = 0.0;
        r_min = lmin;
        r_max = lmax;
      } else {
        r_count = msg_count - 1;
        r_rate = __ddiv_rn((double)byte_count, duration);
        const uint32_t delta = seq_max - seq_start;
        r_loss = delta <= 1 ? 0.0
                            : __dsub_rn(1.0, __ddiv_rn((double)msg_count, (double)(delta + 1)));
        r_min = lmin;
        r_max = lmax;
      }
      if (lane == 0) {
        const size_t slot = (size_t)f * per_flow + rcount;
        mgenx_flow_report* rp = reports + slot;
        rp->flow = f;
        rp->index = rcount;
        rp->start_sec = ws.sec;
        rp->start_usec = ws.usec;
        rp->duration = duration;
        rp->msg_count = r_count;
        rp->rate = r_rate;
        rp->loss = r_loss;
        rp->latency_min = r_min;
        rp->latency_max = r_max;
        rp->rx_sec = rx.sec;
        rp->rx_usec = rx.usec;
        CloseRec c;
        c.pos = pos;
        c.zr = zr;
        c.mc = msg_count;
        closes[slot] = c;
        if (report_rec) report_rec[slot] = order[pos];
      }
      }
      rcount++;
      nrep++;
      ncl++;
      last_close = pos;
      last_zr = zr;
      ws = rx;
      we = uni_t(tadd(rx, window));
      wek = tkey(we);
      seq_start = seq_max;
      if (msg != 0) {
        byte_count = 0;
        msg_count = 1;
        lmin = lmax = latency;
      } else {
        byte_count = msg_count = 0;
        lmin = lmax = 0.0;
      }
    }
    return contrib;
  };

  // Per-lane partials of the bulk runs, folded into the wave-uniform state by flush() before
  // every exact update and at the end: latency min / max, bytes, and the highest seq - first
  // (for `last`).  msg_count == 0 (min / max set by the first counted latency, :132-133) means
  // no counted record is pending.  msg_count == 1 (the byte restart of :128-129) also arises
  // from a run that counted one record from 0, its size pending: a run or a cheap restart
  // that meets msg_count == 1 with partials pending flushes first.
  const double inf = __builtin_huge_val();
  double pmin = inf, pmax = -inf;
  uint32_t pbytes = 0, pdmax = 0, prounds = 0;
  bool dirty = false;
  auto flush = [&]() {
    if (!dirty) return;
    const double rmin = WRing::wave_reduce_f64(pmin, inf, [](double a, double c) {
      return c < a ? c : a; });
    const double rmax = WRing::wave_reduce_f64(pmax, -inf, [](double a, double c) {
      return c > a ? c : a; });
    lmin = rmin < lmin ? rmin : lmin;
    lmax = rmax > lmax ? rmax : lmax;
    const uint64_t lo = WRing::wave_sum(pbytes & 0xFFFFu), hi = WRing::wave_sum(pbytes >> 16);
    byte_count += lo + (hi << 16);
    m.last = m.first + max(WRing::wave_max(pdmax), m.last - m.first);
    pmin = inf;
    pmax = -inf;
    pbytes = pdmax = prounds = 0;
    dirty = false;
  };

  FRec ra[kUR], rb[kUR];  // the records of two rounds (ping-pong: see the loop below)
  double latp[kUR];
  auto ld = [&](uint32_t base, FRec (&r)[kUR]) {  // clamped: lanes past the flow reload its last
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) r[q] = recs[min(base + 64u * q + lane, e - 1u)];
  };

  // records [k, ev) of the round: a bulk run (every one simple, valid && m.n)
  auto bulk = [&](const FRec (&cur)[kUR], uint32_t k, uint32_t ev) {
    // a run at msg_count == 1 replaces byte_count (:128-129), pending bytes included: a run
    // before it (the previous round's, or one before a cheap restart) that took msg_count
    // from 0 to 1 left its one record's size pending -- fold it first
    if (msg_count == 1 && dirty) flush();
    if (lane < 32u) scat[wv][lane] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // every lane issues every LDS op (non-candidates with a zero bit / the identity), so the
    // four lookups and the four atomics go out back to back under one wait each, with no
    // branch per record group
    bool cand[kUR], inring[kUR], clash = false;
    uint32_t bit[kUR], word[kUR], old[kUR];
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) {
      const uint32_t p = 64u * q + lane;
      cand[q] = p >= k && p < ev && cur[q].len != 0u;
      bit[q] = cand[q] ? 1u << (cur[q].seq & 31u) : 0u;
    }
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++)
      word[q] = (uint32_t)__shfl((int)m.w, (int)((cur[q].seq >> 5) & 31u));
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) old[q] = atomicOr(&scat[wv][(cur[q].seq >> 5) & 31u], bit[q]);
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) {
      inring[q] = (word[q] >> (cur[q].seq & 31u)) & 1u;
      clash |= (old[q] & bit[q]) != 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    bool indup[kUR];
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) indup[q] = false;
    if (__ballot(clash)) {  // two records of the run share a sequence number: the first is new
#pragma unroll
      for (uint32_t q = 0; q < kUR; q++)
        atomicMin(&fo[wv][cur[q].seq & 1023u], cand[q] ? 64u * q + lane : 0xFFFFFFFFu);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      uint32_t fv[kUR];
#pragma unroll
      for (uint32_t q = 0; q < kUR; q++) fv[q] = fo[wv][cur[q].seq & 1023u];
#pragma unroll
      for (uint32_t q = 0; q < kUR; q++) indup[q] = cand[q] && fv[q] < 64u * q + lane;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t q = 0; q < kUR; q++)
        if (cand[q]) fo[wv][cur[q].seq & 1023u] = 0xFFFFFFFFu;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // per record group: three ballots and branch-free per-lane partials (no branch per group:
    // a select the compiler turns into an exec-mask branch costs more than the select)
    uint32_t n_cnt = 0, n_cand = 0, n_new = 0;
    uint64_t cms[kUR];
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) {
      // (bitwise: && evaluates its right side under an exec mask, a branch)
      const bool nw = cand[q] & !inring[q] & !indup[q];
      const bool counted = nw & ((int32_t)(cur[q].seq - seq_start) >= 0);
      cms[q] = __ballot(counted);
      n_cnt += (uint32_t)__popcll(cms[q]);
      n_new += (uint32_t)__popcll(__ballot(nw));
      n_cand += (uint32_t)__popcll(__ballot(cand[q]));
      const double lat = cur[q].latency;
      pbytes += counted ? cur[q].len : 0u;
      // min / max (latencies are never NaN or -0, so v_min / v_max equal the compare-selects;
      // fmin would canonicalise its operands first)
      pmin = vmin64(pmin, counted ? lat : inf);
      pmax = vmax64(pmax, counted ? lat : -inf);
      pdmax = max(pdmax, cand[q] ? cur[q].seq - m.first : 0u);
      latp[q] = counted ? lat : latp[q];
    }
    const uint32_t n_dup = n_cand - n_new;
    if (n_cnt) {
      // :128-129: a counted record arriving at msg_count == 1 replaces byte_count by its size
      // (nothing is pending then, see above): at 1 the run's bytes replace it; at 0 the first
      // counted record adds and the second replaces, so the first one's size drops out
      if (msg_count == 1) byte_count = 0;
      if (msg_count == 0) {
        if (n_cnt >= 2) {  // the run's first counted record: its size
          uint32_t len1 = 0;
          bool got = false;
#pragma unroll
          for (uint32_t q = 0; q < kUR; q++) {
            if (!got && cms[q]) {
              len1 = (uint32_t)__builtin_amdgcn_readlane((int)cur[q].len, (int)__builtin_ctzll(cms[q]));
              got = true;
            }
          }
          byte_count -= len1;  // byte_count is 0 here; the flush adds it back
        }
        lmin = inf;  // :132-133: the first counted latency sets both
        lmax = -inf;
      }
      msg_count += n_cnt;
    }
    dups += n_dup;
    m.n += n_new;
    if (lane < 32u) m.w |= scat[wv][lane];
    __builtin_amdgcn_wave_barrier();
    dirty = true;
  };

  // each set's loads followed by 4 stores (to the sink slots), as every round ends: the loop
  // head's wait for ra then has the same 16 operations after it on entry as around the loop
  // (with fewer on entry, the compiler's count would make every pass drain rb's loads too)
  auto sink4 = [&]() {
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) lat2[lat2_sink + 64u * q + lane] = 0.0;  // (4 x 64 slots)
  };
  ld(b, ra);
  __builtin_amdgcn_sched_barrier(0);
  sink4();
  __builtin_amdgcn_sched_barrier(0);
  ld(b + kRound, rb);
  __builtin_amdgcn_sched_barrier(0);
  sink4();
  __builtin_amdgcn_sched_barrier(0);
#if MGENX_DIAG
  const bool prof_on = blockIdx.x == 0 && wv == 0;
  unsigned long long prof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
                     prof_t = __builtin_amdgcn_s_memtime();
  const unsigned long long prof_t0 = prof_t;
  bool was_rst = false;
#endif
  // one round: records [i0, i0 + kRound) from cur, whose registers then take the round two
  // ahead.  The loop runs it twice per pass with the two register sets swapped, so no
  // register copy waits on a load issued a round earlier (a rotating cur / nxt / next-next
  // triple in one loop body made the loop head wait for the previous round's loads, and for
  // the lat' stores issued after them)
  auto round = [&](FRec (&set)[kUR], uint32_t i0) {
    const uint32_t cnt = i0 < e ? min(kRound, e - i0) : 0u;  // (0: a pass's empty second round)
    // the round's records moved out of the load registers through an opaque move: the waits
    // for set's loads happen here (vmcnt: only the other set's loads and this round's stores
    // after them), and the round's inner loop reads no register loaded outside it -- otherwise
    // the compiler flushes vmcnt(0) before that loop, waiting for the other set's loads too
    FRec cur[kUR];
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) cur[q] = opaque_frec(set[q]);
#if MGENX_DIAG
    prof[4]++;
#endif
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) latp[q] = 0.0;
    uint32_t k = 0;
    while (k < cnt) {
      uint32_t ev = k;  // the first record from k that takes the exact update
      if (valid && m.n) {
        ev = cnt;
#pragma unroll
        for (uint32_t q = 0; q < kUR; q++) {
          const uint32_t p = 64u * q + lane;
          const bool simple = (cur[q].rxk < wek) & ((cur[q].len == 0u) | (cur[q].seq - m.first < kDepth));
          const uint64_t ns = __ballot((p >= k) & (p < cnt) & !simple);  // (bitwise: no exec branches)
          if (ns) ev = min(ev, 64u * q + (uint32_t)__builtin_ctzll(ns));
        }
        UPD_T(0);
        if (ev > k) {
          bulk(cur, k, ev);
#if MGENX_DIAG
          prof[6]++;
#endif
        }
        UPD_T(1);
      }
      if (ev >= cnt) break;
#if MGENX_DIAG
      prof[5]++;
#endif
      const uint32_t q = ev >> 6, l = ev & 63u;
      uint32_t seq = 0, len = 0, rlo = 0, rhi = 0, llo = 0, lhi = 0;
#pragma unroll
      for (uint32_t qq = 0; qq < kUR; qq++) {  // static indices (a dynamic one goes to scratch)
        const uint32_t s_ = (uint32_t)__builtin_amdgcn_readlane((int)cur[qq].seq, (int)l);
        const uint32_t n_ = (uint32_t)__builtin_amdgcn_readlane((int)cur[qq].len, (int)l);
        const uint32_t a_ = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cur[qq].rxk, (int)l);
        const uint32_t b_ = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cur[qq].rxk >> 32), (int)l);
        const uint64_t lb = __builtin_bit_cast(uint64_t, cur[qq].latency);
        const uint32_t c_ = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lb, (int)l);
        const uint32_t d_ = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(lb >> 32), (int)l);
        seq = qq == q ? s_ : seq;
        len = qq == q ? n_ : len;
        rlo = qq == q ? a_ : rlo;
        rhi = qq == q ? b_ : rhi;
        llo = qq == q ? c_ : llo;
        lhi = qq == q ? d_ : lhi;
      }
      const uint64_t rxk = (uint64_t)rhi << 32 | rlo;
      const double lat = __builtin_bit_cast(double, (uint64_t)lhi << 32 | llo);
      double lp;
      if (valid && m.n && len != 0u && rxk < wek && (int32_t)(seq - m.first) >= (int32_t)kDepth &&
          (int32_t)(seq - seq_start) >= 0) {
        // a mask restart, the common exact step (:118-127): not a duplicate (outside the span),
        // counted, Set fails, UnsetBits clears every set index (all below seq) -> mask {seq}.
        // No flush: the pending bytes / min / max stay pending (order-free); only the pending
        // `last` partials, relative to the old first, are dropped (last = seq now).
        if (msg_count <= 1 && dirty) flush();  // (the replace at 1 covers pending bytes)
        pdmax = 0;
        m.w = lane == ((seq >> 5) & 31u) ? (1u << (seq & 31u)) : 0u;
        m.first = m.last = seq;
        m.n = 1;
        if (msg_count == 1) byte_count = len;  // (flushed above: nothing pending)
        else byte_count += len;
        if (msg_count == 0) {
          lmin = lmax = lat;
        } else {
          lmin = lat < lmin ? lat : lmin;
          lmax = lat > lmax ? lat : lmax;
        }
        msg_count++;
        lp = lat;
#if MGENX_DIAG
        was_rst = true;
#endif
      } else {
        flush();
        lp = update(seq, rxk, len, lat, i0 + ev);
#if MGENX_DIAG
        was_rst = false;
#endif
      }
#pragma unroll
      for (uint32_t qq = 0; qq < kUR; qq++) latp[qq] = (qq == q && lane == l) ? lp : latp[qq];
      k = ev + 1u;
#if MGENX_DIAG
      if (prof_on) {
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();
        prof[was_rst ? 8 : 2] += now_ - prof_t;
        prof[9] += was_rst ? 1 : 0;
        prof_t = now_;
      }
#endif
    }
    // this round's lat' straight from registers, then the loads of the round two ahead into
    // cur: every round issues 4 stores and 8 loads in that order, so the wait for a round's
    // records (vmcnt: 12, the next round's stores and loads) never waits on a store
#pragma unroll
    for (uint32_t q = 0; q < kUR; q++) {
      const uint32_t p = 64u * q + lane;  // branch-free: lanes past the round write sink slots
      lat2[p < cnt ? i0 + p : lat2_sink + lane] = latp[q];
    }
    ld(i0 + 2u * kRound, set);
    if (++prounds == 4096u) flush();  // per-lane bytes stay below 2^32
    UPD_T(3);
  };
  // (no exit between the two rounds: a path from the first round's end back to the loop head
  // would leave only its own stores after its loads, and the head's waits would drain them)
  for (uint32_t i0 = b; i0 < e; i0 += 2u * kRound) {
    round(ra, i0);
    round(rb, i0 + kRound);
  }
#if MGENX_DIAG
  if (prof_on && lane == 0) {
    prof[7] = __builtin_amdgcn_s_memtime() - prof_t0;
    for (int k2 = 0; k2 < 10; k2++) g_upd_prof[k2] = prof[k2];
  }
#endif

  flush();
  m.store_relative(sp->mask);
  if (lane == 0) {
    sp->mask_first = m.first;
    sp->mask_n = m.n;
    sp->window_valid = valid ? 1u : 0u;
    sp->win_start_sec = ws.sec;
    sp->win_start_usec = ws.usec;
    sp->win_end_sec = we.sec;
    sp->win_end_usec = we.usec;
    sp->seq_start = seq_start;
    sp->msg_count = msg_count;
    sp->byte_count = byte_count;
    sp->dup_count = dups;
    sp->latency_min = lmin;
    sp->latency_max = lmax;
    sp->n_reports = nrep;
    if (report_count) report_count[f] = rcount;
  }

  // ---- the latency sums, on this wave: each window's in-order FP64 sum of lat' (lane t takes
  // window t: [lo, hi] below), staged through this
  // wave's lbuf.  The flow's lat' and closes were just written by this wave: every store is
  // waited for, and the loads read past L1 (agent scope) from the XCD's L2, where they sit --
  // no separate pass re-reading lat' from HBM.
  __builtin_amdgcn_s_waitcnt(0);
  double* piece = &lbuf[wv][0];
  const uint32_t kept = min(rcount, per_flow);
  const uint32_t nslots = kept > rc0 ? kept - rc0 : 0u;
  const uint32_t nwin = nslots + 1u;  // + the open window
  const CloseRec* cl = closes + (size_t)f * per_flow;
  auto ld32 = [](const uint32_t* q) {
    return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (uint32_t w0 = 0; w0 < nwin; w0 += 64u) {
    const uint32_t t = w0 + lane;
    const bool has = t < nwin;
    uint32_t lo = 0, hi = 0;
    double sum = 0.0;
    if (has) {
      if (t < nslots) {
        const uint32_t slot = rc0 + t;
        hi = ld32(&cl[slot].pos);
        if (t == 0) {
          lo = b;
          sum = lsum0;
        } else {
          lo = ld32(&cl[slot - 1u].pos) + (ld32(&cl[slot - 1u].zr) ? 1u : 0u);
        }
      } else {
        hi = e - 1u;
        if (ncl) {
          lo = last_close + (last_zr ? 1u : 0u);
        } else {
          lo = b;
          sum = lsum0;
        }
      }
    }
    const uint32_t nl = min(nwin - w0, 64u);
    const uint32_t a0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
    const uint32_t z0 = (uint32_t)__builtin_amdgcn_readlane((int)hi, (int)(nl - 1u));
    for (uint32_t p0 = a0; p0 <= z0 && p0 >= a0; p0 += kPiece) {
      const uint32_t pend = min(z0 + 1u, p0 + kPiece);
      const bool mine = has && lo <= hi && lo < pend && hi >= p0;
      if (!__ballot(mine)) continue;
      {  // the piece's 16 loads per lane issued together, then staged (one load, wait, LDS
         // write per step made 16 serial L2 round trips per 1024 records); branch-free: lanes
         // past the piece reload its last value into slots nobody reads
        double x[kPiece / 64u];
#pragma unroll
        for (uint32_t u = 0; u < kPiece / 64u; u++)
          x[u] = __hip_atomic_load(&lat2[min(p0 + lane + 64u * u, pend - 1u)], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (uint32_t u = 0; u < kPiece / 64u; u++) piece[lane + 64u * u] = x[u];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (mine) {
        const uint32_t ja = max(lo, p0) - p0, jz = min(hi + 1u, pend) - p0;
        uint32_t j = ja;
        for (; j + 8u <= jz; j += 8u) {
          double x[8];
#pragma unroll
          for (int u = 0; u < 8; u++) x[u] = piece[j + u];
#pragma unroll
          for (int u = 0; u < 8; u++) sum = __dadd_rn(sum, x[u]);
        }
        for (; j < jz; j++) sum = __dadd_rn(sum, piece[j]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (has) {
      if (t < nslots) {
        const uint32_t slot = rc0 + t;
        const uint64_t mc = __hip_atomic_load(&cl[slot].mc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        reports[(size_t)f * per_flow + slot].latency_ave =
            mc == 0 ? -1.0 : mc == 1 ? sum : __ddiv_rn(sum, (double)mc);
      } else {
        sp->latency_sum = sum;
      }
    }
  }
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
// Tiles of 512 x kK records (kK keys per lane of each of the 8 waves): 4096 normally; 4608
// when that takes the persistent grid's walk one round of tiles fewer (rank 0's share of
// config 4 at N = 8 is 1,048,662 records: 257 tiles of 4096 on 256 blocks put two tiles on
// one block of every XCD; 228 of 4608 take one round)
constexpr uint32_t kTile = 4096;
constexpr uint32_t kTileBig = 4608;
// LDS of the order kernel: 9 x bins x 4 bytes of counts and bases, the tile's records (24 B
// each) and their flows (2 B each) -- within 160 KiB up to 1536 bins at 4096 records, 1223 at
// 4608
constexpr uint32_t kCountBins = 1536;
constexpr uint32_t order_lds(uint32_t bins, uint32_t tile) {
  return (kSortWaves * bins + bins + (bins & 1u)) * 4u + tile * ((uint32_t)sizeof(FRec) + 2u);
}
constexpr uint32_t kLdsCap = 160u * 1024u - 64u;  // (+ the kernel's static wsum[])
static_assert(order_lds(kCountBins - 1u, kTile) <= kLdsCap, "order kernel LDS at 4096 records");

__global__ void __launch_bounds__(512)
flow_hist_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows, uint32_t tile,
                 uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h[];
  const uint32_t bins = n_flows + 1u;
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) h[k] = 0u;
  __syncthreads();
  const uint32_t a = blockIdx.x * tile, e = min(n, a + tile);
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
template <bool kRows, uint32_t kK>
__global__ void __launch_bounds__(512)
flow_order_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows,
                  uint32_t n_tiles, const uint32_t* __restrict__ start, RecSrc src,
                  FRec* __restrict__ recs, uint32_t* __restrict__ order, uint32_t key_bits,
                  uint32_t seqw) {  // diagnostics timing only (tile-contiguous writes, wrong)
  constexpr uint32_t kT = 512u * kK, kPart = kT / kSortWaves;  // tile, records per wave
  extern __shared__ uint32_t lds[];
  const uint32_t bins = n_flows + 1u;
  uint32_t* cnt = lds;                                // [wave][bin]: counts, then run bases
  uint32_t* sbase = lds + kSortWaves * bins;          // [bin]: start - tile offset
  FRec* lrec = reinterpret_cast<FRec*>(sbase + bins + (bins & 1u));  // 8-byte aligned
  uint16_t* lkey = reinterpret_cast<uint16_t*>(lrec + kT);
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
  constexpr uint32_t kKeys = kK;
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
    const uint32_t a = tt * kT + w * kPart;
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
    const uint32_t t0 = t * kT;
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
    const uint32_t tn = min(n - t0, kT);
#pragma unroll
    for (uint32_t u = 0; u < kK; u++) {
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

// The same scan in one kernel: block j owns flows [16 j, 16 j + 16) down all tiles (16 tile
// segments x 16 flows = 256 threads): segment sums, the flows' exclusive prefixes inside the
// block, one decoupled look-back over the blocks before it for the records of all lower flows
// (epoch-tagged words: epoch << 40 | kind << 38 | count, kind 1 = the block's own total, 2 =
// inclusive of every block before it), then start[] written down each segment.  Blocks wait
// only on lower blocks, all resident (<= 96 blocks); a poll count bounds every wait anyway.
constexpr uint32_t kC1Flows = 16, kC1Segs = 16;
constexpr uint32_t kC1Epochs = 1u << 22;
constexpr uint32_t kC1Spin = 1u << 20;
__global__ void __launch_bounds__(256)
flow_colscan1_kernel(const uint32_t* __restrict__ hist, uint32_t bins, uint32_t n_tiles,
                     uint32_t* __restrict__ start, uint64_t* __restrict__ status, uint32_t epoch) {
  __shared__ uint32_t part[kC1Segs][kC1Flows];
  __shared__ uint32_t fpre[kC1Flows];
  __shared__ uint64_t s_excl;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, kk = tid % kC1Flows, sg = tid / kC1Flows;
  const uint32_t j = blockIdx.x, k = j * kC1Flows + kk;
  const uint32_t per = (n_tiles + kC1Segs - 1u) / kC1Segs;
  const uint32_t t0 = min(n_tiles, sg * per), t1 = min(n_tiles, t0 + per);
  // 1. this thread's segment of its flow
  uint32_t sum = 0;
  if (k < bins) {
    uint32_t t = t0;
    for (; t + 8u <= t1; t += 8u) {
      uint32_t x[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) x[u] = hist[(size_t)(t + u) * bins + k];
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) sum += x[u];
    }
    for (; t < t1; t++) sum += hist[(size_t)t * bins + k];
  }
  part[sg][kk] = sum;
  __syncthreads();
  // 2. per flow: the segments' exclusive prefixes (in place) and the flow's total; then the
  // block's flows in order
  if (tid < kC1Flows) {
    uint32_t run = 0;
    for (uint32_t q = 0; q < kC1Segs; q++) {
      const uint32_t v = part[q][tid];
      part[q][tid] = run;
      run += v;
    }
    fpre[tid] = run;
  }
  __syncthreads();
  if (tid < 64u) {
    // 3. wave 0: the block's total, its flows' exclusive prefixes, the look-back
    const uint32_t ft = lane < kC1Flows ? fpre[lane] : 0u;
    uint32_t incl = ft;
#pragma unroll
    for (uint32_t d = 1; d < kC1Flows; d <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)incl, d);
      if (lane >= d) incl += o;
    }
    const uint32_t agg = (uint32_t)__shfl((int)incl, (int)kC1Flows - 1);
    if (lane < kC1Flows) fpre[lane] = incl - ft;
    if (lane == 0)
      __hip_atomic_store(&status[j], ((uint64_t)epoch << 40) | ((uint64_t)(j == 0 ? 2u : 1u) << 38) | agg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t acc = 0;
    bool gave_up = false;
    for (int64_t top = (int64_t)j - 1; top >= 0 && !gave_up; top -= 64) {
      const int64_t q = top - (int64_t)lane;
      uint64_t w = 0;
      if (q >= 0) {
        uint32_t polls = 0;
        do {
          w = __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } while ((uint32_t)(w >> 40) != epoch && ++polls < kC1Spin);
      }
      const bool here = q < 0 || (uint32_t)(w >> 40) == epoch;
      gave_up = __ballot(!here) != 0;
      const uint32_t kind = q >= 0 ? (uint32_t)(w >> 38) & 3u : 2u;
      const uint64_t v = q >= 0 && here ? (w & ((1ull << 38) - 1)) : 0ull;
      const uint64_t done = __ballot(kind == 2u);
      const uint32_t stop = done ? (uint32_t)__ffsll((long long)done) - 1u : 64u;
      uint64_t mine = lane <= stop ? v : 0ull;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mine += __shfl_xor(mine, o);
      acc += mine;
      if (done) break;
    }
    if (lane == 0) {
      if (j != 0)
        __hip_atomic_store(&status[j], ((uint64_t)epoch << 40) | (2ull << 38) | (acc + agg),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_excl = acc;
    }
  }
  __syncthreads();
  // 4. start[] down this thread's segment
  if (k < bins) {
    uint32_t run = (uint32_t)s_excl + fpre[kk] + part[sg][kk];
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
  uint64_t* c1_status = nullptr;  // flow_colscan1_kernel's look-back words (epoch-tagged)
  uint32_t c1_epoch = 0;
};

extern "C" void* mgenx_flow_ws_new() { return new mgenx_flow_ws(); }
extern "C" void mgenx_flow_ws_free(void* p) {
  mgenx_flow_ws* w = static_cast<mgenx_flow_ws*>(p);
  if (!w) return;
  mgenx::dev_free(w->mem);
  mgenx::dev_free(w->c1_status);
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
  if (out && n == 16)  // flow_order_kernel's phase cycles (g_ord_prof, 8 entries)
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ord_prof), 64) == hipSuccess ? MGENX_OK
                                                                              : MGENX_EDEVICE;
  if (out && n == 10)  // flow_update_kernel's phase cycles (g_upd_prof)
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_upd_prof), 80) == hipSuccess ? MGENX_OK
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
  // persistent order grid: one block per CU (LDS allows one), a multiple of 8 (one set per XCD)
  if (!ws.cu) {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cu = 256;
    ws.cu = (uint32_t)max(8, cu);
  }
  // the tile size: 4608 records when its walk is shorter (rounds of tiles per block x records
  // per tile) and its LDS fits, else 4096
  auto walk = [&](uint32_t tile) {
    const uint32_t tiles = (n + tile - 1u) / tile, per = (tiles + 7u) / 8u;
    const uint32_t nbk = min(per, ws.cu / 8u);
    return (uint64_t)((per + nbk - 1u) / nbk) * tile;
  };
  bool big = order_lds(bins, kTileBig) <= kLdsCap && walk(kTileBig) < walk(kTile);
#if MGENX_DIAG
  if (const char* tt = getenv("MGENX_AN_TILE"))  // 4096 / 4608: the tile size forced (A/B)
    big = atoi(tt) == (int)kTileBig && order_lds(bins, kTileBig) <= kLdsCap;
#endif
  const uint32_t tile = big ? kTileBig : kTile;
  const uint32_t n_tiles = (n + tile - 1) / tile;
  const size_t n_hist = (size_t)bins * n_tiles;
  size_t cub_bytes = 0;
  if (sort_path == 0)  // the chunk partials and their prefixes
    cub_bytes = (size_t)2u * ((n_tiles + kColTiles - 1u) / kColTiles) * bins * 4u;
  else
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (int)n, 0, (int)key_bits, stream);
  const bool want_order = report_rec != nullptr;
  const size_t nb = a256((size_t)n * 4), rb = a256((size_t)n * sizeof(FRec));
  const size_t hb = a256(n_hist * 4), bb = a256((size_t)bins * 4);
  const size_t lb = a256((size_t)(n + 256) * 8);  // lat' + the update's 256 sink slots
  const size_t cb = a256((size_t)n_flows * per_flow * sizeof(CloseRec));
  // both: records (sorted), lat', closes
  // counting: hist, start, order (report_rec only), row totals
  // radix:    keys_in, keys_out, vals_in, order, bounds, cub
  const size_t common = rb + lb + cb;
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
  double* lat2 = (double*)take(lb);
  CloseRec* closes = (CloseRec*)take(cb);
  const uint32_t* bnd;
  uint32_t bstride;
  uint32_t* order = nullptr;
  hipError_t e;
  if (sort_path == 0) {
    uint32_t* hist = (uint32_t*)take(hb);
    uint32_t* start = (uint32_t*)take(hb);
    if (want_order) order = (uint32_t*)take(nb);
    uint32_t* totals = (uint32_t*)take(a256(cub_bytes));
    hipLaunchKernelGGL(flow_hist_kernel, dim3(n_tiles), dim3(512), bins * 4u, stream, flow_idx, n,
                       n_flows, tile, hist);
    // the single-pass scan (flow_colscan1_kernel) up to 512 tiles: each of its blocks reads
    // every tile for its 16 flows, which beats three launches for rank 0's share at N = 8
    // (228 tiles: 0.1259 vs 0.1287 ms, three A/B pairs) but not config 4's 2048 tiles (0.2620
    // vs 0.2587)
    bool one = n_tiles <= 512u;
#if MGENX_DIAG
    if (const char* c1 = getenv("MGENX_AN_SCAN1")) one = atoi(c1) != 0;  // (A/B)
#endif
    if (one) {
      if (!ws.c1_status) {
        if (hipMalloc(&ws.c1_status, (kCountBins / kC1Flows + 1) * 8) != hipSuccess) {
          ws.c1_status = nullptr;
          snprintf(err, errn, "flow_reduce: scan words");
          return MGENX_EDEVICE;
        }
        ws.c1_epoch = 0;
      }
      if (ws.c1_epoch == 0 || ++ws.c1_epoch >= kC1Epochs) {  // (re)start the epochs from zeros
        if (hipMemsetAsync(ws.c1_status, 0, (kCountBins / kC1Flows + 1) * 8, stream) != hipSuccess) {
          snprintf(err, errn, "flow_reduce: scan words");
          return MGENX_EDEVICE;
        }
        ws.c1_epoch = 1;
      }
      hipLaunchKernelGGL(flow_colscan1_kernel, dim3((bins + kC1Flows - 1u) / kC1Flows), dim3(256), 0,
                         stream, hist, bins, n_tiles, start, ws.c1_status, ws.c1_epoch);
    } else {
      const uint32_t n_chunks = (n_tiles + kColTiles - 1u) / kColTiles;
      const dim3 cg((bins + 255u) / 256u, n_chunks);
      hipLaunchKernelGGL(flow_colpart_kernel, cg, dim3(256), 0, stream, hist, bins, n_tiles, totals);
      hipLaunchKernelGGL(flow_colbase_kernel, dim3(1), dim3(1024), 0, stream, totals, bins, n_chunks,
                         totals + (size_t)n_chunks * bins);
      hipLaunchKernelGGL(flow_colscan_kernel, cg, dim3(256), 0, stream, hist, totals,
                         totals + (size_t)n_chunks * bins, bins, n_tiles, start);
    }
    e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(err, errn, "flow_reduce scan: %s", hipGetErrorString(e));
      return MGENX_EDEVICE;
    }
    // LDS: per-wave counts, the run bases, the tile's records and their flows
    const uint32_t lds = order_lds(bins, tile);
    const uint32_t grid = 8u * min((n_tiles + 7u) / 8u, ws.cu / 8u);
    auto launch = [&](auto kern) {
      hipError_t le = set_max_lds((const void*)kern, (int)kLdsCap);
      if (le != hipSuccess) return le;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kSortWaves), lds, stream, flow_idx, n, n_flows,
                         n_tiles, start, src, recs, order, key_bits, oseqw);
      return hipGetLastError();
    };
    if (src.rows)
      e = big ? launch(flow_order_kernel<true, 9>) : launch(flow_order_kernel<true, 8>);
    else
      e = big ? launch(flow_order_kernel<false, 9>) : launch(flow_order_kernel<false, 8>);
    if (e != hipSuccess) {
      snprintf(err, errn, "flow_reduce order: %s", hipGetErrorString(e));
      return MGENX_EDEVICE;
    }
    bnd = start;  // tile 0's row: flow k starts at start[k]
    bstride = 1;
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
    bstride = 1;
  }
  if (sabl) return MGENX_OK;  // timing study: ordering only
  hipLaunchKernelGGL(flow_update_kernel, dim3((n_flows + 3) / 4), dim3(256), 0, stream, flows,
                     n_flows, bnd, bstride, recs, order, lat2, reports, per_flow, report_count,
                     report_rec, closes, n);
  e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err, errn, "flow_reduce: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  return MGENX_OK;
}
