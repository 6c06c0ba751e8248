// mgenx_analytic.hip -- per-flow receive analytics (MgenAnalytic::Update) on gfx950.
//
// Reference: MgenAnalytic::Init / Update (src/common/mgenAnalytic.cpp:28-258) called per
// received message by Mgen::UpdateRecvAnalytics (src/common/mgen.cpp:1027-1070), over the
// protolib primitives ProtoSlidingMask (1024-bit duplicate window) and ProtoTime::Delta
// (restated in oracle/mgen_oracle.c; parity unpinned at protolib).
//
// The state machine is sequential per flow and independent across flows, so:
//   1. records are ordered by flow, stably (receive order kept): hipCUB radix sort of
//      (flow index, record index) -- plumbing, not the hot path;
//   2. their fields are gathered flow-contiguous (24 B per record);
//   3. one lane per flow runs Update over its records (prefetched 8 at a time), its
//      1024-bit mask in LDS, transposed (word k of lane t at k * 64 + t: conflict-free).
// FP64: every product that feeds an add goes through mul_rounded (an empty asm keeps the
// backend from fusing them into an FMA: neither __dadd_rn/__dmul_rn nor `#pragma clang fp
// contract(off)` prevented it -- a 1-ulp difference in a report's duration was the
// symptom), so results are bit-identical to the oracle built for x86-64.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>
#include <string.h>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr int kFlowThreads = 64;
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
__device__ __forceinline__ Tm tadd(Tm t, double s) {  // ProtoTime += double
  const double whole = floor(s);
  const int64_t us = (int64_t)(mul_rounded(s - whole, 1.0e06) + 0.5);
  t.sec += (int64_t)whole;
  t.usec += us;
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
struct Ring {
  uint32_t* w;  // word k at w[k * kFlowThreads]
  uint32_t first, last, n;
  __device__ uint32_t& word(uint32_t k) { return w[(k & 31u) * kFlowThreads]; }
  __device__ bool bit(uint32_t s) { return (word(s >> 5 & 31u) >> (s & 31u)) & 1u; }
  __device__ void setbit(uint32_t s) { word(s >> 5 & 31u) |= 1u << (s & 31u); }
  __device__ void clear() {  // `first` is kept (stale), as the restatement keeps it
    for (int k = 0; k < 32; k++) word(k) = 0;
    n = 0;
  }
  __device__ uint32_t get_last() { return n ? last : first; }
  __device__ bool test(uint32_t idx) {
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
    if (last - idx >= kDepth) return false;  // precedes first: allowed while span < depth
    setbit(idx);
    first = idx;
    n++;
    return true;
  }
  // clear indices first .. first + count - 1, then re-base `first` on the lowest left
  __device__ void unset_from_first(uint32_t count) {
    if (!n) return;
    if ((uint64_t)count > (uint64_t)(last - first)) {
      clear();
      return;
    }
    uint32_t s = first;
    uint32_t left = count;
    while (left) {
      const uint32_t b = s & 31u, take = min(32u - b, left);
      const uint32_t m = (take == 32u ? 0xFFFFFFFFu : ((1u << take) - 1u)) << b;
      uint32_t& x = word(s >> 5 & 31u);
      n -= __popc(x & m);
      x &= ~m;
      s += take;
      left -= take;
    }
    // lowest set index at or after s (last is still set)
    for (;;) {
      const uint32_t b = s & 31u;
      const uint32_t x = word(s >> 5 & 31u) >> b;
      if (x) {
        first = s + (uint32_t)(__ffs(x) - 1);
        return;
      }
      s += 32u - b;
    }
  }
  // relative form (bit i of words rel <-> first + i) <-> ring
  __device__ void load_relative(const uint32_t* rel) {
    for (int k = 0; k < 32; k++) word(k) = 0;
    const uint32_t fs = first & 1023u, fw = fs >> 5, bs = fs & 31u;
    for (uint32_t k = 0; k < 32; k++) {
      const uint32_t v = rel[k];
      word(fw + k) |= v << bs;
      if (bs) word(fw + k + 1) |= v >> (32u - bs);
    }
    last = first;
    for (int k = 31; k >= 0; k--)
      if (rel[k]) { last = first + 32u * k + (31u - __clz(rel[k])); break; }
  }
  __device__ void store_relative(uint32_t* rel) {
    const uint32_t fs = first & 1023u, fw = fs >> 5, bs = fs & 31u;
    for (uint32_t k = 0; k < 32; k++) {
      uint32_t v = word(fw + k) >> bs;
      if (bs) v |= word(fw + k + 1) << (32u - bs);
      rel[k] = n ? v : 0u;
    }
    if (!n) return;
    // bits of the ring that lie past `last` (none: the span is < 1024) stay zero
  }
};

struct Rec {
  uint32_t seq, txs, txu, rxs, rxu, len;
};

__global__ void __launch_bounds__(kFlowThreads)
flow_update_kernel(mgenx_flow_state* __restrict__ flows, uint32_t n_flows,
                   const uint32_t* __restrict__ begin, const uint32_t* __restrict__ end,
                   const uint32_t* __restrict__ s_seq, const uint32_t* __restrict__ s_txs,
                   const uint32_t* __restrict__ s_txu, const uint32_t* __restrict__ s_rxs,
                   const uint32_t* __restrict__ s_rxu, const uint16_t* __restrict__ s_len,
                   mgenx_flow_report* __restrict__ reports, uint32_t per_flow,
                   uint32_t* __restrict__ report_count) {
  __shared__ uint32_t lds[32 * kFlowThreads];
  const uint32_t f = blockIdx.x * kFlowThreads + threadIdx.x;
  if (f >= n_flows) return;
  const uint32_t b = begin[f], e = end[f];
  if (b >= e) return;
  mgenx_flow_state st = flows[f];
  Ring m;
  m.w = lds + threadIdx.x;
  m.first = st.mask_first;
  m.n = st.mask_n;
  m.load_relative(flows[f].mask);  // straight from memory: no 128-B local copy
  bool valid = st.window_valid != 0;
  Tm ws = {st.win_start_sec, st.win_start_usec}, we = {st.win_end_sec, st.win_end_usec};
  uint32_t seq_start = st.seq_start;
  uint64_t msg_count = st.msg_count, byte_count = st.byte_count, dups = st.dup_count;
  double lsum = st.latency_sum, lmin = st.latency_min, lmax = st.latency_max;
  uint64_t nrep = st.n_reports;
  uint32_t rcount = report_count[f];

  auto update = [&](const Rec& r) {
    const Tm rx = {(int64_t)r.rxs, (int64_t)r.rxu}, tx = {(int64_t)r.txs, (int64_t)r.txu};
    const uint32_t msg = r.len;
    if (!valid) {  // mgenAnalytic.cpp:80-99
      valid = true;
      ws = rx;
      we = tadd(rx, st.window_size);
      if (msg != 0) {
        m.set(r.seq);
        seq_start = r.seq;
        msg_count = 1;
        byte_count = msg;
        lsum = lmin = lmax = tdelta(rx, tx);
      } else {
        msg_count = byte_count = 0;
        lsum = lmin = lmax = 0.0;
      }
      return;
    }
    double latency = 0.0;
    if (msg != 0) {  // :102-178
      if (m.n) {
        if (m.test(r.seq)) {
          dups++;
        } else if ((int32_t)(r.seq - seq_start) < 0) {
          m.set(r.seq);
        } else {
          if (!m.set(r.seq)) {  // UnsetBits(first, seq - first), then Set (:120-127)
            m.unset_from_first(r.seq - m.first);
            m.set(r.seq);
          }
          if (1 == msg_count) byte_count = msg;
          else byte_count += msg;
          latency = tdelta(rx, tx);
          if (0 == msg_count) {
            lsum = lmin = lmax = latency;
          } else {
            lsum = __dadd_rn(lsum, latency);
            if (latency < lmin) lmin = latency;
            else if (latency > lmax) lmax = latency;
          }
          msg_count++;
        }
      } else {
        m.clear();
        m.set(r.seq);
        seq_start = r.seq;
        byte_count = msg;
        lsum = lmin = lmax = tdelta(rx, tx);
        msg_count = 1;
      }
    }
    if (tge(rx, we)) {  // :180-256: report and restart the window
      mgenx_flow_report rep;
      rep.flow = f;
      rep.index = rcount;
      rep.start_sec = ws.sec;
      rep.start_usec = ws.usec;
      rep.duration = tdelta(rx, ws);
      rep.rx_sec = rx.sec;
      rep.rx_usec = rx.usec;
      const uint32_t seq_max = m.n ? m.get_last() : seq_start;
      if (msg_count == 0) {
        rep.msg_count = 0;
        rep.rate = 0.0;
        rep.loss = 1.0;
        rep.latency_ave = rep.latency_min = rep.latency_max = -1.0;
      } else if (msg_count == 1) {
        rep.msg_count = 1;
        rep.rate = __ddiv_rn((double)byte_count, rep.duration);
        rep.loss = 0.0;
        rep.latency_ave = lsum;
        rep.latency_min = lmin;
        rep.latency_max = lmax;
      } else {
        rep.msg_count = msg_count - 1;
        rep.rate = __ddiv_rn((double)byte_count, rep.duration);
        const uint32_t delta = seq_max - seq_start;
        rep.loss = delta <= 1 ? 0.0
                              : __dsub_rn(1.0, __ddiv_rn((double)msg_count, (double)(delta + 1)));
        rep.latency_ave = __ddiv_rn(lsum, (double)msg_count);
        rep.latency_min = lmin;
        rep.latency_max = lmax;
      }
      if (rcount < per_flow) reports[(size_t)f * per_flow + rcount] = rep;
      rcount++;
      nrep++;
      ws = rx;
      we = tadd(rx, st.window_size);
      seq_start = seq_max;
      if (msg != 0) {
        byte_count = 0;
        msg_count = 1;
        lsum = lmin = lmax = latency;
      } else {
        byte_count = msg_count = 0;
        lsum = lmin = lmax = 0.0;
      }
    }
  };

  constexpr int kPre = 8;
  for (uint32_t i0 = b; i0 < e; i0 += kPre) {
    Rec r[kPre];
#pragma unroll
    for (int k = 0; k < kPre; k++) {
      const uint32_t i = min(i0 + k, e - 1);  // clamped: no divergent loads
      r[k] = {s_seq[i], s_txs[i], s_txu[i], s_rxs[i], s_rxu[i], (uint32_t)s_len[i]};
    }
#pragma unroll
    for (int k = 0; k < kPre; k++)
      if (i0 + k < e) update(r[k]);
  }

  m.store_relative(flows[f].mask);
  st.mask_first = m.first;
  st.mask_n = m.n;
  st.window_valid = valid ? 1u : 0u;
  st.win_start_sec = ws.sec;
  st.win_start_usec = ws.usec;
  st.win_end_sec = we.sec;
  st.win_end_usec = we.usec;
  st.seq_start = seq_start;
  st.msg_count = msg_count;
  st.byte_count = byte_count;
  st.dup_count = dups;
  st.latency_sum = lsum;
  st.latency_min = lmin;
  st.latency_max = lmax;
  st.n_reports = nrep;
  // scalar fields back (the mask words were written in place above)
  mgenx_flow_state& o = flows[f];
  o.mask_first = st.mask_first; o.mask_n = st.mask_n; o.seq_start = st.seq_start;
  o.window_valid = st.window_valid; o.win_start_sec = st.win_start_sec;
  o.win_start_usec = st.win_start_usec; o.win_end_sec = st.win_end_sec;
  o.win_end_usec = st.win_end_usec; o.msg_count = st.msg_count; o.byte_count = st.byte_count;
  o.dup_count = st.dup_count; o.latency_sum = st.latency_sum; o.latency_min = st.latency_min;
  o.latency_max = st.latency_max; o.n_reports = st.n_reports;
  report_count[f] = rcount;
}

// keys: flow index clamped to n_flows (records to skip sort last); vals: record index
__global__ void flow_keys_kernel(const uint32_t* __restrict__ idx, uint32_t n, uint32_t n_flows,
                                 uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = min(idx[i], n_flows);
  vals[i] = i;
}

// segment bounds of each flow in the sorted keys, and the flow-contiguous record fields
__global__ void flow_gather_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ order,
                                   uint32_t n, uint32_t n_flows, uint32_t* __restrict__ begin,
                                   uint32_t* __restrict__ end, const uint32_t* __restrict__ seq,
                                   const uint32_t* __restrict__ txs, const uint32_t* __restrict__ txu,
                                   const uint16_t* __restrict__ len, const uint32_t* __restrict__ rxs,
                                   const uint32_t* __restrict__ rxu, uint32_t* __restrict__ o_seq,
                                   uint32_t* __restrict__ o_txs, uint32_t* __restrict__ o_txu,
                                   uint16_t* __restrict__ o_len, uint32_t* __restrict__ o_rxs,
                                   uint32_t* __restrict__ o_rxu) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (k < n_flows) {
    if (i == 0 || keys[i - 1] != k) begin[k] = i;
    if (i + 1 == n || keys[i + 1] != k) end[k] = i + 1;
  }
  const uint32_t r = order[i];
  o_seq[i] = seq[r];
  o_txs[i] = txs[r];
  o_txu[i] = txu[r];
  o_len[i] = len[r];
  o_rxs[i] = rxs[r];
  o_rxu[i] = rxu[r];
}

__global__ void flow_init_kernel(mgenx_flow_state* flows, uint32_t n_flows, double window) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_flows) return;
  mgenx_flow_state s;
  memset(&s, 0, sizeof(s));
  s.window_size = window;
  flows[f] = s;
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
};

extern "C" void* mgenx_flow_ws_new() { return new mgenx_flow_ws(); }
extern "C" void mgenx_flow_ws_free(void* p) {
  mgenx_flow_ws* w = static_cast<mgenx_flow_ws*>(p);
  if (!w) return;
  if (w->mem) (void)hipFree(w->mem);
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

extern "C" int mgenx_flow_init_run(mgenx_flow_state* flows, uint32_t n_flows, double window,
                                   hipStream_t stream) {
  if (!n_flows) return MGENX_OK;
  hipLaunchKernelGGL(flow_init_kernel, dim3((n_flows + 255) / 256), dim3(256), 0, stream, flows,
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
                                     const uint32_t* rxs, const uint32_t* rxu, uint32_t n,
                                     mgenx_flow_state* flows, uint32_t n_flows,
                                     mgenx_flow_report* reports, uint32_t per_flow,
                                     uint32_t* report_count, hipStream_t stream, char* err,
                                     size_t errn) {
  mgenx_flow_ws& ws = *static_cast<mgenx_flow_ws*>(wsp);
  if (n == 0 || n_flows == 0) return MGENX_OK;
  int end_bit = 1;
  while (end_bit < 32 && (1ull << end_bit) <= n_flows) end_bit++;
  size_t cub_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)n, 0, end_bit, stream);
  // layout: keys_in, keys_out, vals_in, vals_out, begin, end, 5 x u32 fields, u16 len, cub
  const size_t nb = a256((size_t)n * 4), fb = a256((size_t)n_flows * 4);
  const size_t need = 4 * nb + 2 * fb + 5 * nb + a256((size_t)n * 2) + a256(cub_bytes);
  if (ws.bytes < need) {
    if (ws.mem) (void)hipFree(ws.mem);
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
  uint32_t* keys_in = (uint32_t*)take(nb);
  uint32_t* keys_out = (uint32_t*)take(nb);
  uint32_t* vals_in = (uint32_t*)take(nb);
  uint32_t* vals_out = (uint32_t*)take(nb);
  uint32_t* d_begin = (uint32_t*)take(fb);
  uint32_t* d_end = (uint32_t*)take(fb);
  uint32_t* o_seq = (uint32_t*)take(nb);
  uint32_t* o_txs = (uint32_t*)take(nb);
  uint32_t* o_txu = (uint32_t*)take(nb);
  uint32_t* o_rxs = (uint32_t*)take(nb);
  uint32_t* o_rxu = (uint32_t*)take(nb);
  uint16_t* o_len = (uint16_t*)take(a256((size_t)n * 2));
  void* cub_tmp = take(a256(cub_bytes));
  const dim3 g((n + 255) / 256);
  hipLaunchKernelGGL(flow_keys_kernel, g, dim3(256), 0, stream, flow_idx, n, n_flows, keys_in,
                     vals_in);
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, keys_in, keys_out,
                                                    vals_in, vals_out, (int)n, 0, end_bit, stream);
  if (e != hipSuccess) {
    snprintf(err, errn, "flow_reduce sort: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  (void)hipMemsetAsync(d_begin, 0, fb, stream);
  (void)hipMemsetAsync(d_end, 0, fb, stream);
  hipLaunchKernelGGL(flow_gather_kernel, g, dim3(256), 0, stream, keys_out, vals_out, n, n_flows,
                     d_begin, d_end, seq, txs, txu, len, rxs, rxu, o_seq, o_txs, o_txu, o_len,
                     o_rxs, o_rxu);
  hipLaunchKernelGGL(flow_update_kernel, dim3((n_flows + kFlowThreads - 1) / kFlowThreads),
                     dim3(kFlowThreads), 0, stream, flows, n_flows, d_begin, d_end, o_seq, o_txs,
                     o_txu, o_rxs, o_rxu, o_len, reports, per_flow, report_count);
  e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err, errn, "flow_reduce: %s", hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
  return MGENX_OK;
}
