// mgenx_flowsm.hpp -- MgenAnalytic::Update's per-flow state machine on one wave (gfx950),
// shared by the batch update kernel (mgenx_analytic.hip) and the resident worker
// (mgenx_worker.hip).
//
// Reference: MgenAnalytic::Update (src/common/mgenAnalytic.cpp:74-258) over the protolib
// primitives ProtoSlidingMask (1024-bit duplicate window) and ProtoTime (Delta, +=), restated
// in oracle/mgen_oracle.c (parity unpinned at protolib).
// FP64: every product that feeds an add goes through mul_rounded (an empty asm keeps the
// backend from fusing them into an FMA), so results are bit-identical to the x86-64 oracle.
#pragma once
#pragma clang fp contract(off)

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr uint32_t kDepth = 1024;

struct Tm {
  int64_t sec, usec;
};

// a rounded product the following add cannot fuse with (an FMA would round once)
__device__ __forceinline__ double mul_rounded(double a, double b) {
  double p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}
__device__ __forceinline__ double tdelta(Tm a, Tm b) {  // ProtoTime::Delta(a, b)
  return (double)(a.sec - b.sec) + mul_rounded(1.0e-06, (double)(a.usec - b.usec));
}
// ProtoTime += double, split: the double's whole seconds and rounded microseconds depend on the
// window size alone, so a kernel computes them once per flow (TAdd) and each window close only
// adds and normalises (no FP64 floor / conversion on the per-flow critical path)
struct TAdd {
  int64_t sec, usec;
};
__device__ __forceinline__ TAdd tadd_of(double s) {
  const double whole = floor(s);
  return TAdd{(int64_t)whole, (int64_t)(mul_rounded(s - whole, 1.0e06) + 0.5)};
}
__device__ __forceinline__ Tm tadd(Tm t, TAdd a) {
  t.sec += a.sec;
  t.usec += a.usec;
  while (t.usec >= 1000000) { t.usec -= 1000000; t.sec += 1; }
  return t;
}
__device__ __forceinline__ bool tge(Tm a, Tm b) {
  return a.sec > b.sec || (a.sec == b.sec && a.usec >= b.usec);
}

// ProtoSlidingMask(1024) with the semantics of oracle/mgen_oracle.c (mask_*): a set of u32
// indices with span < 1024.  Kept as a 1024-bit RING (index s at bit s mod 1024) plus the
// lowest (first) and highest (last) set index, so set / test are O(1) and nothing shifts;
// the state array stores it relative to `first` (bit i <-> first + i), converted on entry
// and exit.  (The shifting form scanned and moved 32 words whenever an index arrived below
// `first` -- every reordered message after a window slide -- and dominated the kernel.)
// The same ring with one WAVE per flow: ring word w (0..31) lives in lane w's register, every
// scalar of the state machine is wave-uniform (SGPRs, scalar branches), a bit is read with
// one v_readlane and set with one masked VALU op, and the rare range clears and searches
// are lane-parallel with a wave reduction.  Records of the flow are loaded 64 at a time
// (lane k holds record i0 + k, coalesced) and walked in order through v_readlane.
struct WRing {
  uint32_t w;           // this lane's ring word (lanes 32..63 hold 0)
  uint32_t first, last, n;
  uint32_t lane;
  __device__ uint32_t word(uint32_t k) const {  // k uniform
    return (uint32_t)__builtin_amdgcn_readlane((int)w, (int)(k & 31u));
  }
  __device__ bool bit(uint32_t s) const { return (word(s >> 5) >> (s & 31u)) & 1u; }
  __device__ void setbit(uint32_t s) {
    w |= (lane == ((s >> 5) & 31u)) ? (1u << (s & 31u)) : 0u;
  }
  __device__ void clear() {
    w = 0;
    n = 0;
  }
  __device__ uint32_t get_last() const { return n ? last : first; }
  __device__ bool test(uint32_t idx) const {
    if (!n) return false;
    const int32_t d = (int32_t)(idx - first);
    if (d < 0 || (uint32_t)d >= kDepth) return false;
    return bit(idx);
  }
  __device__ bool set(uint32_t idx) {
    if (!n) {
      clear();
      first = last = idx;
      setbit(idx);
      n = 1;
      return true;
    }
    const int32_t d = (int32_t)(idx - first);
    if (d >= 0) {
      if ((uint32_t)d >= kDepth) return false;
      if (!bit(idx)) {
        setbit(idx);
        n++;
        if ((uint32_t)d > last - first) last = idx;
      }
      return true;
    }
    if (last - idx >= kDepth) return false;
    setbit(idx);
    first = idx;
    n++;
    return true;
  }
  // lane mask of ring positions p with (p - a) mod 1024 < len (len < 1024) in this lane's
  // word: bit j has distance d0 + j, which wraps to 0 at j = 1024 - d0 when d0 > 992
  __device__ uint32_t range_mask(uint32_t a, uint32_t len) const {
    auto low = [](uint32_t k) { return k >= 32u ? 0xFFFFFFFFu : ((1u << k) - 1u); };
    const uint32_t d0 = (lane * 32u - a) & 1023u;
    uint32_t m = len > d0 ? low(min(min(32u, 1024u - d0), len - d0)) : 0u;
    if (d0 > 992u) {
      const uint32_t w0 = 1024u - d0;
      m |= low(min(32u - w0, len)) << w0;
    }
    return lane < 32u ? m : 0u;
  }
  // whole-wave reductions through DPP (quad swaps, half-row and row mirrors, row
  // broadcasts 15 / 31): the result is complete in lane 63 and returned wave-uniform
  template <typename Op>
  __device__ static uint32_t wave_reduce(uint32_t v, uint32_t identity, Op op) {
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0xB1, 0xF, 0xF, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0x4E, 0xF, 0xF, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0x141, 0xF, 0xF, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0x140, 0xF, 0xF, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0x142, 0xA, 0xF, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  }
  // the same reduction over doubles (both 32-bit halves moved by the same DPP pattern)
  template <int CTRL, int RMASK, typename Op>
  __device__ static double dpp_step_f64(double x, double identity, Op op) {
    const uint64_t xb = __builtin_bit_cast(uint64_t, x), ib = __builtin_bit_cast(uint64_t, identity);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)ib, (int)(uint32_t)xb,
                                                              CTRL, RMASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(ib >> 32),
                                                              (int)(uint32_t)(xb >> 32), CTRL,
                                                              RMASK, 0xF, false);
    return op(x, __builtin_bit_cast(double, (uint64_t)hi << 32 | lo));
  }
  template <typename Op>
  __device__ static double wave_reduce_f64(double v, double identity, Op op) {
    v = dpp_step_f64<0xB1, 0xF>(v, identity, op);
    v = dpp_step_f64<0x4E, 0xF>(v, identity, op);
    v = dpp_step_f64<0x141, 0xF>(v, identity, op);
    v = dpp_step_f64<0x140, 0xF>(v, identity, op);
    v = dpp_step_f64<0x142, 0xA>(v, identity, op);
    v = dpp_step_f64<0x143, 0xC>(v, identity, op);
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
  }
  __device__ static uint32_t wave_sum(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
  }
  __device__ static uint32_t wave_max(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t a, uint32_t b) { return max(a, b); });
  }
  __device__ static uint32_t wave_min(uint32_t v) {
    return wave_reduce(v, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return min(a, b); });
  }
  // clear indices first .. first + count - 1, then re-base `first` on the lowest left
  __device__ void unset_from_first(uint32_t count) {
    if (!n) return;
    if ((uint64_t)count > (uint64_t)(last - first)) {
      clear();
      return;
    }
    w &= ~range_mask(first & 1023u, count);
    n = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_sum((uint32_t)__popc(w)));
    // lowest set index at or after s = first + count, in ring order from s (last is set)
    const uint32_t s = first + count;
    const uint32_t a = s & 1023u;
    uint32_t best = 0xFFFFFFFFu;
    if (w) {
      // the set bit of this word with the smallest distance from a (mod 1024)
      const uint32_t lo = lane * 32u;
      const uint32_t sh = (a >= lo && a < lo + 32u) ? (a - lo) : 0u;
      const uint32_t hi_part = w & (0xFFFFFFFFu << sh);  // bits at/after a in this word
      if (a >= lo && a < lo + 32u && hi_part) best = (uint32_t)(__ffs(hi_part) - 1) + lo - a;
      else if (a >= lo && a < lo + 32u) best = (uint32_t)(__ffs(w) - 1) + lo + 1024u - a;
      else best = ((uint32_t)(__ffs(w) - 1) + lo - a) & 1023u;
    }
    first = s + (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_min(best));
  }
  __device__ void load_relative(const uint32_t* rel) {  // bit i of rel <-> first + i
    const uint32_t fs = first & 1023u, fw = fs >> 5, bs = fs & 31u;
    const uint32_t k = (lane - fw) & 31u;
    const uint32_t a = rel[k], b = rel[(k - 1u) & 31u];
    // ring word = this relative word shifted up by bs, plus the previous relative word's top
    // bits (relative word 31's land in ring word fw: relative indices wrap at 1024)
    uint32_t v = a << bs;
    if (bs) v |= b >> (32u - bs);
    w = lane < 32u ? v : 0u;
    last = first;
    // highest set relative bit
    uint32_t top = 0;
    const uint32_t rk = lane < 32u ? rel[lane] : 0u;
    const uint32_t cand = rk ? lane * 32u + (31u - __clz(rk)) + 1u : 0u;  // +1: 0 = none
    uint32_t mx = cand;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    top = (uint32_t)__builtin_amdgcn_readfirstlane((int)mx);
    if (top) last = first + top - 1u;
  }
  __device__ void store_relative(uint32_t* rel) const {
    const uint32_t fs = first & 1023u, fw = fs >> 5, bs = fs & 31u;
    const uint32_t src0 = (fw + lane) & 31u, src1 = (fw + lane + 1u) & 31u;
    const uint32_t x0 = (uint32_t)__shfl((int)w, (int)src0), x1 = (uint32_t)__shfl((int)w, (int)src1);
    uint32_t v = x0 >> bs;
    if (bs) v |= x1 << (32u - bs);
    if (lane < 32u) rel[lane] = n ? v : 0u;
  }
};

// Wave-uniform values: the window times come out of FP64 arithmetic (VALU), so without
// these the compiler treats every later compare and branch on them as divergent.
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ Tm uni_t(Tm t) { return Tm{uni64(t.sec), uni64(t.usec)}; }
// the window end as a receive-time key (usec < 10^6 after tadd); an end past the 32-bit seconds
// range gets the largest key, which only sends records to the exact path (it compares times)
__device__ __forceinline__ uint64_t tkey(Tm t) {
  return t.sec > 0xFFFFFFFFll ? ~0ull : ((uint64_t)t.sec << 32 | (uint64_t)t.usec);
}

__device__ __forceinline__ double vmin64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmax64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// One flow's Update state on one wave: every scalar wave-uniform, the mask a WRing.  exact()
// is MgenAnalytic::Update for one record (arguments wave-uniform); a window close hands the
// report's values to `on_close`.  The latency sum is kept as the batch kernels keep it -- not
// here: exact() returns the record's contribution lat' (its latency when Update adds or
// assigns it to latency_sum, else 0.0) and reports whether the close restarted the sum at 0.0
// (zr: the closing "first actual message", :156-165, whose local `latency` stays 0.0) -- the
// caller sums lat' in record order.
struct FlowClose {
  Tm rx, ws;           // the closing record's receive time, the window start
  double duration;     // ProtoTime::Delta(rx, window_start)
  uint64_t r_count;    // report_msg_count
  double r_rate, r_loss, r_min, r_max;
  uint64_t mc;         // msg_count at the close (latency_ave's divisor)
  uint32_t zr;
};
struct FlowSM {
  WRing m;
  bool valid;
  Tm ws, we;
  uint64_t wek;
  TAdd window;
  uint32_t seq_start;
  uint64_t msg_count, byte_count, dups, nrep;
  double lmin, lmax;

  __device__ void load(const mgenx_flow_state* sp, uint32_t lane) {
    window = tadd_of(sp->window_size);
    m.lane = lane;
    m.first = sp->mask_first;
    m.n = sp->mask_n;
    m.load_relative(sp->mask);
    if (!m.n) m.w = 0;
    valid = sp->window_valid != 0;
    ws = Tm{sp->win_start_sec, sp->win_start_usec};
    we = Tm{sp->win_end_sec, sp->win_end_usec};
    wek = tkey(we);
    seq_start = sp->seq_start;
    msg_count = sp->msg_count;
    byte_count = sp->byte_count;
    dups = sp->dup_count;
    lmin = sp->latency_min;
    lmax = sp->latency_max;
    nrep = sp->n_reports;
  }
  // every field but latency_sum (the caller's)
  __device__ void store(mgenx_flow_state* sp, uint32_t lane) const {
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
    }
  }
  template <typename OnClose>
  __device__ double exact(uint32_t seq, uint64_t rxk, uint32_t msg, double lat, OnClose on_close) {
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
            const bool lo = latency < lmin;
            const bool hi = !lo && latency > lmax;
            lmin = lo ? latency : lmin;
            lmax = hi ? latency : lmax;
          }
          msg_count++;
        }
      } else {  // the first actual message (:156-165): sets the sum, `latency` stays 0.0
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
    if (tge(rx, we)) {  // :168-255: report and restart the window
      const uint32_t seq_max = m.n ? m.get_last() : seq_start;
      FlowClose c;
      c.rx = rx;
      c.ws = ws;
      c.duration = tdelta(rx, ws);
      c.mc = msg_count;
      c.zr = zr;
      if (msg_count == 0) {
        c.r_count = 0;
        c.r_rate = 0.0;
        c.r_loss = 1.0;
        c.r_min = c.r_max = -1.0;
      } else if (msg_count == 1) {
        c.r_count = 1;
        c.r_rate = __ddiv_rn((double)byte_count, c.duration);
        c.r_loss = 0.0;
        c.r_min = lmin;
        c.r_max = lmax;
      } else {
        c.r_count = msg_count - 1;
        c.r_rate = __ddiv_rn((double)byte_count, c.duration);
        const uint32_t delta = seq_max - seq_start;
        c.r_loss = delta <= 1 ? 0.0 : __dsub_rn(1.0, __ddiv_rn((double)msg_count, (double)(delta + 1)));
        c.r_min = lmin;
        c.r_max = lmax;
      }
      on_close(c);
      nrep++;
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
  }
};

}  // namespace mgenx
