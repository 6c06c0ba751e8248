// mgenx_scan.hip -- record-boundary scan of TCP / SINK byte streams on gfx950.
//
// Reference semantics (the oracle restates them in or_tcp_scan / or_sink_scan):
//   TCP   MgenTcpTransport::GetRxNumBytes / OnRecvMsg (src/common/mgenTransport.cpp:1683-1760):
//         a record starts with its big-endian u16 msg_len; msg_len < 4 is a stream error
//         (scan stops); an incomplete last record stays unconsumed.
//   SINK  MgenAppSinkTransport::OnInputReady (src/common/mgenAppSinkTransport.cpp:369-434):
//         msg_len outside [MIN_SIZE, MAX_SIZE] discards the two length bytes (resync).
// The framing is a sequential chain p_{i+1} = p_i + L(p_i).  On the GPU:
//   1. detect: one streaming pass flags plausible starts (L in range, record inside the
//      stream, version byte == 2) per 64 KiB block into ordered slots (1 B/byte of input);
//   2. compact + link: candidates in stream order, successor = candidate at p + L
//      (binary search), or a terminal (stream end / position that is not a candidate);
//   3. binary lifting (pointer doubling) gives the chain from any candidate in log2 steps,
//      and the chain from the current start is enumerated in parallel;
//   4. where the chain leaves the candidate set (a record with a bad version, SINK garbage,
//      a partial tail, TCP msg_len < 4) a single-thread resolver walks the reference rule
//      exactly until it re-enters the set.  Valid streams never need step 4 mid-stream.
// Bit-exact with the sequential rule for every input: candidates only shortcut positions
// the chain would compute anyway.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include <vector>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr uint32_t kScanBlockBytes = 65536;  // detect block (one workgroup)
constexpr uint32_t kScanThreads = 256;       // 256 B per thread
constexpr uint32_t kScanSlots = 2048;        // candidates per block before overflow
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct ScanMode {
  uint32_t min_len, max_len;
};

__device__ __forceinline__ uint32_t be16_at(const uint8_t* s, uint64_t p) {
  return ((uint32_t)s[p] << 8) | s[p + 1];
}

// 1. detect.  Thread t of block b owns positions [b*64K + 256 t, +256); it needs bytes up
// to 258 past its start (length + version byte of its last position).
__global__ void __launch_bounds__(kScanThreads)
scan_detect_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, ScanMode m,
                   uint16_t* __restrict__ slots, uint32_t* __restrict__ counts) {
  __shared__ uint32_t warp_sum[kScanThreads / 64];
  const uint64_t start = (uint64_t)blockIdx.x * kScanBlockBytes + 256ull * threadIdx.x;
  // a candidate p needs p + 3 <= nbytes (p + L <= nbytes with L >= 4 implies it)
  auto is_cand = [&](uint64_t p) -> bool {
    if (p + 4 > nbytes) return false;
    if (s[p + 2] != 2) return false;
    const uint32_t L = be16_at(s, p);
    return L >= m.min_len && L <= m.max_len && p + L <= nbytes;
  };
  // fast screen: positions whose version byte (p + 2) is 0x02, found 4 bytes at a time
  uint32_t cnt = 0;
  const bool full = start + 256 + 4 <= nbytes;
  uint32_t w[65];
  if (full) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const u32x4_t v = ldu128(s + start + 16 * k);
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    w[64] = ldu32(s + start + 256);
  } else {
#pragma unroll
    for (int k = 0; k < 65; k++) {
      uint32_t x = 0;
      for (int b = 0; b < 4; b++) {
        const uint64_t q = start + 4 * k + b;
        if (q < nbytes) x |= (uint32_t)s[q] << (8 * b);
      }
      w[k] = x;
    }
  }
  // Window byte j (0..259) = byte start + j; position start + i has its version byte at
  // j = i + 2.  Words without a 0x02 byte are skipped with one SWAR test; the rare others
  // are checked exactly (static indices: the window stays in registers).
  auto visit = [&](auto&& emit) {
#pragma unroll
    for (int k = 0; k < 65; k++) {
      const uint32_t x = w[k];
      const uint32_t t = x ^ 0x02020202u;
      if (((t - 0x01010101u) & ~t & 0x80808080u) != 0) {
        for (int b = 0; b < 4; b++) {
          const int i = 4 * k + b - 2;
          if (i < 0 || i >= 256 || ((x >> (8 * b)) & 0xffu) != 2u) continue;
          if (is_cand(start + (uint64_t)i)) emit(i);
        }
      }
    }
  };
  visit([&](int) { cnt++; });
  // block exclusive scan of the per-thread counts (stream order = thread order)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) warp_sum[wv] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int k = 0; k < wv; k++) wbase += warp_sum[k];
  const uint32_t total = warp_sum[0] + warp_sum[1] + warp_sum[2] + warp_sum[3];
  uint32_t pos = wbase + incl - cnt;
  if (threadIdx.x == 0) counts[blockIdx.x] = total > kScanSlots ? kNone : total;
  if (total > kScanSlots) return;  // overflow: the host resolves this stream sequentially
  uint16_t* out = slots + (size_t)blockIdx.x * kScanSlots;
  const uint32_t tofs = 256u * threadIdx.x;
  visit([&](int i) { out[pos++] = (uint16_t)(tofs + (uint32_t)i); });
}

// exclusive scan of block counts (single workgroup; n_blocks is small: 16 K per GiB)
__global__ void __launch_bounds__(1024)
scan_offsets_kernel(const uint32_t* __restrict__ counts, uint32_t n_blocks,
                    uint32_t* __restrict__ base, uint32_t* __restrict__ total_out) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  bool overflow = false;
  for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    uint32_t c = b < n_blocks ? counts[b] : 0u;
    if (c == kNone) { overflow = true; c = 0; }
    part[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (b < n_blocks) base[b] = carry + part[threadIdx.x] - c;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  const int any_ovf = __syncthreads_or(overflow);
  if (threadIdx.x == 0) total_out[0] = any_ovf ? kNone : carry;
}

__global__ void __launch_bounds__(256)
scan_compact_kernel(const uint16_t* __restrict__ slots, const uint32_t* __restrict__ counts,
                    const uint32_t* __restrict__ base, uint64_t* __restrict__ cand) {
  const uint32_t b = blockIdx.x;
  const uint32_t c = counts[b];
  const uint32_t o = base[b];
  for (uint32_t k = threadIdx.x; k < c; k += blockDim.x)
    cand[o + k] = (uint64_t)b * kScanBlockBytes + slots[(size_t)b * kScanSlots + k];
}

__device__ uint32_t find_cand(const uint64_t* cand, uint32_t n, uint64_t p) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cand[mid] < p) lo = mid + 1; else hi = mid;
  }
  return (lo < n && cand[lo] == p) ? lo : kNone;
}

// 2. link: up0 = successor (self for a terminal), dist0 = 1 if linked
__global__ void __launch_bounds__(256)
scan_link_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, const uint64_t* __restrict__ cand,
                 uint32_t n, uint32_t* __restrict__ up, uint32_t* __restrict__ dist) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint64_t p = cand[c];
  const uint64_t nx = p + be16_at(s, p);
  const uint32_t t = (nx + 2 <= nbytes) ? find_cand(cand, n, nx) : kNone;
  up[c] = t == kNone ? c : t;
  dist[c] = t == kNone ? 0u : 1u;
}

// 3. one doubling level: up_k = up_{k-1} o up_{k-1}, dist_k = dist_{k-1} + dist_{k-1} o up
__global__ void __launch_bounds__(256)
scan_double_kernel(const uint32_t* __restrict__ up0, const uint32_t* __restrict__ d0,
                   uint32_t* __restrict__ up1, uint32_t* __restrict__ d1, uint32_t n) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint32_t u = up0[c];
  up1[c] = up0[u];
  d1[c] = d0[c] + d0[u];
}

// enumerate the chain from candidate s: record i = lift(s, i), i < count
__global__ void __launch_bounds__(256)
scan_enum_kernel(const uint8_t* __restrict__ s, const uint64_t* __restrict__ cand,
                 const uint32_t* __restrict__ ups, uint32_t n, int levels, uint32_t start,
                 uint64_t count, uint64_t out_base, uint64_t cap, uint64_t* __restrict__ rec_off,
                 uint32_t* __restrict__ rec_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count || out_base + i >= cap) return;
  uint32_t node = start;
  for (int k = 0; k < levels; k++)
    if ((i >> k) & 1) node = ups[(size_t)k * n + node];
  const uint64_t p = cand[node];
  rec_off[out_base + i] = p;
  rec_len[out_base + i] = be16_at(s, p);
}

// 4. sequential resolver (one thread): the reference rule from position p until the chain
// re-enters the candidate set, ends, errors, or max_steps records were emitted.
struct ResolveState {
  uint64_t pos;        // in: start position; out: where it stopped
  uint64_t emitted;    // out: records written
  uint32_t next_cand;  // out: candidate index at `pos` (kNone if none)
  int32_t reason;      // out: 0 = candidate reached, 1 = end of stream, 2 = TCP error, 3 = steps
};

__global__ void scan_resolve_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, int sink,
                                    const uint64_t* __restrict__ cand, uint32_t n,
                                    uint64_t out_base, uint64_t cap, uint64_t max_steps,
                                    uint64_t* __restrict__ rec_off, uint32_t* __restrict__ rec_len,
                                    ResolveState* st) {
  uint64_t p = st->pos;
  uint64_t k = 0;
  int reason = 3;
  uint32_t nc = kNone;
  bool first = true;
  while (k < max_steps) {
    if (!first && n) {
      nc = find_cand(cand, n, p);
      if (nc != kNone) { reason = 0; break; }
    }
    first = false;
    if (p + 2 > nbytes) { reason = 1; break; }
    const uint32_t L = be16_at(s, p);
    if (sink) {
      if (L < MGENX_MIN_SIZE || L > MGENX_MAX_SIZE) { p += 2; continue; }  // resync
    } else if (L < 4) {
      reason = 2;
      break;
    }
    if (p + L > nbytes) { reason = 1; break; }
    if (out_base + k < cap) {
      rec_off[out_base + k] = p;
      rec_len[out_base + k] = L;
    }
    k++;
    p += L;
  }
  st->pos = p;
  st->emitted = k;
  st->next_cand = nc;
  st->reason = reason;
}

}  // namespace mgenx

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
using namespace mgenx;

namespace {

struct ScanWork {
  void* mem = nullptr;
  size_t bytes = 0;
};

hipError_t ensure(ScanWork& w, size_t need) {
  if (w.bytes >= need) return hipSuccess;
  if (w.mem) hipFree(w.mem);
  w.mem = nullptr;
  w.bytes = 0;
  hipError_t e = hipMalloc(&w.mem, need);
  if (e == hipSuccess) w.bytes = need;
  return e;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// The workspace lives with the context (grown on demand, freed by mgenx_ctx_destroy via
// mgenx_scan_release).
struct mgenx_scan_ws {
  ScanWork slots, cand, tabs, small;
};

extern "C" void* mgenx_scan_ws_new() { return new mgenx_scan_ws(); }
extern "C" void mgenx_scan_ws_free(void* p) {
  mgenx_scan_ws* w = static_cast<mgenx_scan_ws*>(p);
  if (!w) return;
  for (ScanWork* x : {&w->slots, &w->cand, &w->tabs, &w->small})
    if (x->mem) hipFree(x->mem);
  delete w;
}

// Runs the whole scan (synchronous on `stream`: the record count decides later launches).
extern "C" int mgenx_scan_run(void* wsp, const uint8_t* s, uint64_t nbytes, int mode,
                              uint64_t* rec_off, uint32_t* rec_len, uint64_t cap,
                              mgenx_scan_info* info, hipStream_t stream, char* err, size_t errn) {
  mgenx_scan_ws& ws = *static_cast<mgenx_scan_ws*>(wsp);
  const bool sink = mode == MGENX_SCAN_SINK;
  const ScanMode m = sink ? ScanMode{MGENX_MIN_SIZE, MGENX_MAX_SIZE} : ScanMode{4u, 65535u};
  mgenx_scan_info out;
  memset(&out, 0, sizeof(out));
  auto fail = [&](hipError_t e, const char* what) {
    snprintf(err, errn, "%s: %s", what, hipGetErrorString(e));
    return MGENX_EDEVICE;
  };
  hipError_t e;
  // small scratch: resolver state, total
  if ((e = ensure(ws.small, 4096)) != hipSuccess) return fail(e, "scan workspace");
  ResolveState* d_st = reinterpret_cast<ResolveState*>(ws.small.mem);
  uint32_t* d_total = reinterpret_cast<uint32_t*>(static_cast<char*>(ws.small.mem) + 256);

  uint32_t n = 0;  // candidates
  const uint64_t n_blocks64 = (nbytes + kScanBlockBytes - 1) / kScanBlockBytes;
  bool overflow = n_blocks64 == 0 || n_blocks64 > 0xFFFFFFull;
  uint64_t* d_cand = nullptr;
  uint32_t* d_up = nullptr;
  uint32_t* d_dist = nullptr;
  int levels = 1;
  if (!overflow) {
    const uint32_t nb = (uint32_t)n_blocks64;
    const size_t slot_b = align256((size_t)nb * kScanSlots * 2);
    const size_t cnt_b = align256((size_t)nb * 4);
    if ((e = ensure(ws.slots, slot_b + 2 * cnt_b)) != hipSuccess) return fail(e, "scan workspace");
    uint16_t* d_slots = static_cast<uint16_t*>(ws.slots.mem);
    uint32_t* d_counts = reinterpret_cast<uint32_t*>(static_cast<char*>(ws.slots.mem) + slot_b);
    uint32_t* d_base = d_counts + cnt_b / 4;
    hipLaunchKernelGGL(scan_detect_kernel, dim3(nb), dim3(kScanThreads), 0, stream, s, nbytes, m,
                       d_slots, d_counts);
    hipLaunchKernelGGL(scan_offsets_kernel, dim3(1), dim3(1024), 0, stream, d_counts, nb, d_base,
                       d_total);
    if ((e = hipMemcpyAsync(&n, d_total, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return fail(e, "scan detect");
    if (n == kNone) {
      overflow = true;
      n = 0;
    } else if (n > 0) {
      while ((1ull << (levels - 1)) < n) levels++;
      levels++;  // 2^(levels-1) >= n + 1 > any chain length
      if ((e = ensure(ws.cand, (size_t)n * 8)) != hipSuccess) return fail(e, "scan workspace");
      if ((e = ensure(ws.tabs, (size_t)n * 4 * (levels + 2))) != hipSuccess)
        return fail(e, "scan workspace");
      d_cand = static_cast<uint64_t*>(ws.cand.mem);
      d_up = static_cast<uint32_t*>(ws.tabs.mem);                 // [levels][n]
      d_dist = d_up + (size_t)levels * n;                          // 2 x [n] ping-pong
      hipLaunchKernelGGL(scan_compact_kernel, dim3(nb), dim3(256), 0, stream, d_slots, d_counts,
                         d_base, d_cand);
      const dim3 g((n + 255) / 256);
      hipLaunchKernelGGL(scan_link_kernel, g, dim3(256), 0, stream, s, nbytes, d_cand, n, d_up,
                         d_dist);
      for (int k = 1; k < levels; k++) {
        uint32_t* d0 = d_dist + (size_t)((k - 1) & 1) * n;
        uint32_t* d1 = d_dist + (size_t)(k & 1) * n;
        hipLaunchKernelGGL(scan_double_kernel, g, dim3(256), 0, stream, d_up + (size_t)(k - 1) * n,
                           d0, d_up + (size_t)k * n, d1, n);
      }
    }
  }
  if (overflow) n = 0;  // pathological stream: the resolver walks all of it
  uint32_t* d_dtop = d_dist ? d_dist + (size_t)((levels - 1) & 1) * n : nullptr;

  // chain walk: from position 0, alternating parallel enumeration and the resolver
  uint64_t pos = 0, total = 0;
  uint32_t at = kNone;  // candidate index at pos (if any)
  if (n) {
    uint64_t c0 = 0;
    if ((e = hipMemcpyAsync(&c0, d_cand, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return fail(e, "scan");
    if (c0 == 0) at = 0;
  }
  int reason = 1;
  for (int rounds = 0; rounds < (1 << 30); rounds++) {
    if (at != kNone) {
      // enumerate the candidate chain from `at`
      uint32_t steps = 0, term = 0;
      if ((e = hipMemcpyAsync(&steps, d_dtop + at, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&term, d_up + (size_t)(levels - 1) * n + at, 4,
                              hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipStreamSynchronize(stream)) != hipSuccess)
        return fail(e, "scan");
      const uint64_t count = (uint64_t)steps + 1;
      hipLaunchKernelGGL(scan_enum_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                         stream, s, d_cand, d_up, n, levels, at, count, total, cap, rec_off,
                         rec_len);
      total += count;
      // continue after the terminal candidate's record
      uint64_t tp = 0;
      if ((e = hipMemcpyAsync(&tp, d_cand + term, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return fail(e, "scan");
      uint8_t lb[2];
      if ((e = hipMemcpyAsync(lb, s + tp, 2, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipStreamSynchronize(stream)) != hipSuccess)
        return fail(e, "scan");
      pos = tp + (((uint32_t)lb[0] << 8) | lb[1]);
      at = kNone;
      if (pos + 2 > nbytes) { reason = 1; break; }
    }
    // resolver from pos (pos is not a candidate)
    ResolveState st;
    st.pos = pos;
    st.emitted = 0;
    st.next_cand = kNone;
    st.reason = 3;
    if ((e = hipMemcpyAsync(d_st, &st, sizeof(st), hipMemcpyHostToDevice, stream)) != hipSuccess)
      return fail(e, "scan");
    hipLaunchKernelGGL(scan_resolve_kernel, dim3(1), dim3(1), 0, stream, s, nbytes, (int)sink,
                       d_cand, n, total, cap, (uint64_t)1 << 20, rec_off, rec_len, d_st);
    if ((e = hipMemcpyAsync(&st, d_st, sizeof(st), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return fail(e, "scan resolve");
    total += st.emitted;
    out.resolved += st.emitted;
    pos = st.pos;
    if (st.reason == 0) { at = st.next_cand; continue; }
    if (st.reason == 3) continue;
    reason = st.reason;
    break;
  }
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "scan launch");
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan");
  out.n_records = total;
  out.consumed = pos;
  out.status = reason == 2 ? 1 : 0;
  out.candidates = n;
  if (info) *info = out;
  return MGENX_OK;
}
