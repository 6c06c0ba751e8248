// mgenx_flowtab.hip -- MgenAnalyticTable::FindFlow for whole batches on gfx950.
//
// Reference: MgenAnalyticTable::FindFlow (src/common/mgenAnalytic.cpp:312-328) looks a flow
// up by the key dst addr | dst port | src addr | src port | flowId (ProtoIndexedQueue over
// at most 320 bits), and Mgen::UpdateRecvAnalytics (src/common/mgen.cpp:1034-1053) creates
// the MgenAnalytic on first sight.  Here one call maps n records to dense flow indices:
//   1. insert: open addressing (linear probing) over 64-byte slots in HBM; a slot is claimed
//      by CAS on its state word, the claimant writes the key, then publishes it; lookups of
//      the same key spin (bounded) until it is published.  The first record of each new key
//      is kept with atomicMin;
//   2. number: new keys get the next dense indices in the order of their first record (an
//      exclusive scan over the "first record of a new key" flags), so the mapping does not
//      depend on thread timing;
//   3. resolve: every record reads its slot's index.
// Steady state (every key already numbered by an earlier call): the insert kernel writes each
// record's index itself from the probe's line, counts the keys it creates, and steps 2-3 return
// at once when that count is zero -- 0.30 ms -> ~0.18 ms for config 4's 8.4M lookups (the
// device-library scan of the flags alone took 48 us per call).
// Records with an error (err != 0) map to MGENX_FLOW_NONE, as the reference only updates
// analytics for good messages (mgenTransport.cpp:976-985).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>
#include <string.h>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr uint32_t kSlotEmpty = 0u, kSlotBusy = 0xFFFFFFFFu;

struct FlowKey {  // 48 bytes: the reference key's fields, zero-padded
  uint32_t w[12];
};

struct __attribute__((aligned(64))) FlowSlot {  // 64 bytes: one slot never spans two lines
  FlowKey key;
  uint32_t state;      // 0 empty, kSlotBusy being written, else 1 + slot tag
  uint32_t index;      // dense flow index (kSlotBusy until numbered)
  uint32_t first_rec;  // first record of this call that inserted/looked it up when new
  uint32_t is_new;     // created by the current call
};

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

// key of record i: dst (len, port, 16 addr bytes), src (mgenx_addr), flow id
// (the 32-B rows of mgenx_unpack_batch carry dst_addr4, the first 4 address bytes: with rows
// and no dst_addr column an IPv4 destination is keyed exactly; a longer one is not keyed --
// the caller passes the dst_addr column when IPv6 destinations can occur, see mgenx.h)
__device__ __forceinline__ FlowKey make_key(const mgenx_cols& c, const mgenx_addr* src, uint32_t i) {
  FlowKey k;
  uint32_t da[4] = {0u, 0u, 0u, 0u};
  uint32_t dl, dport, fid;
  if (c.rows) {
    const mgenx_rec& r = c.rows[i];
    dl = r.dst_len;
    dport = r.dst_port;
    fid = r.flow_id;
    da[0] = r.dst_addr4;
  } else {
    dl = c.dst_len[i];
    dport = c.dst_port[i];
    fid = c.flow_id[i];
  }
  if (c.dst_addr) {
    const uint32_t* dp = reinterpret_cast<const uint32_t*>(c.dst_addr + (size_t)i * 16);
#pragma unroll
    for (int j = 0; j < 4; j++) da[j] = dp[j];
  }
  const uint32_t* sa = reinterpret_cast<const uint32_t*>(src[i].addr);
  const uint32_t sl = src[i].len;
  // bytes past an address's length are not part of the reference key: masked to zero
  auto mask_to = [](uint32_t word, uint32_t wi, uint32_t len) {
    const uint32_t lo = 4u * wi;
    if (len >= lo + 4u) return word;
    if (len <= lo) return 0u;
    return word & ((1u << (8u * (len - lo))) - 1u);
  };
#pragma unroll
  for (int j = 0; j < 4; j++) k.w[j] = mask_to(da[j], j, dl);
#pragma unroll
  for (int j = 0; j < 4; j++) k.w[4 + j] = mask_to(sa[j], j, sl);
  k.w[8] = dl | dport << 16;
  k.w[9] = sl | (uint32_t)src[i].port << 16;
  k.w[10] = fid;
  k.w[11] = 0x4D47u;
  return k;
}

__device__ __forceinline__ uint32_t key_hash(const FlowKey& k) {
  uint32_t h = 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 11; j++) h = mix32(h ^ k.w[j]) + (uint32_t)j;
  return h;
}

// a published slot's key never changes: after the acquire load of its state, plain
// (vector) loads of the key words are safe
__device__ __forceinline__ bool key_eq(const FlowKey& a, const FlowSlot& s) {
  const u32x4_t* kw = reinterpret_cast<const u32x4_t*>(s.key.w);
  bool eq = true;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const u32x4_t v = kw[j];
    eq &= a.w[4 * j] == v.x && a.w[4 * j + 1] == v.y && a.w[4 * j + 2] == v.z &&
          a.w[4 * j + 3] == v.w;
  }
  return eq;
}

// Probes per lookup are bounded, and a table takes at most half its slots in keys (its
// max_flows, rounded up): past that a new key counts as overflow (MGENX_FLOW_NONE) instead of
// filling the table, whose probe runs would then grow towards the whole table per record.  At
// load <= 1/2 linear probing's runs stay far below the bound.
constexpr uint32_t kMaxProbe = 1024;

__global__ void flowtab_insert_kernel(FlowSlot* __restrict__ tab, uint32_t cap_mask, mgenx_cols c,
                                      const mgenx_addr* __restrict__ src, uint32_t n,
                                      uint32_t* __restrict__ rec_slot, uint32_t* __restrict__ overflow,
                                      uint32_t* __restrict__ flow_idx, uint32_t* __restrict__ n_new,
                                      const uint32_t* __restrict__ n_flows_before) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t err = c.rows ? c.rows[i].err : (c.err ? c.err[i] : 0u);
  const bool unkeyed = c.rows && !c.dst_addr && c.rows[i].dst_len > 4u;
  if (err != 0 || unkeyed) {
    rec_slot[i] = kSlotBusy;
    flow_idx[i] = MGENX_FLOW_NONE;
    return;
  }
  const FlowKey k = make_key(c, src, i);
  uint32_t s = key_hash(k) & cap_mask;
  // 0. read-only probe with plain loads: the common case, a key published by an earlier call
  //    (is_new clear).  A slot is 64 B inside one cache line and its key is written before
  //    its state is released, so a stale view of the line is at worst "not there yet" -- the
  //    atomic path below then decides.  (Acquire loads here would invalidate the caches on
  //    every probe.)
  const uint32_t max_probe = min(cap_mask + 1u, kMaxProbe);
  for (uint32_t probe = 0, s0 = s; probe < max_probe; probe++, s0 = (s0 + 1) & cap_mask) {
    const u32x4_t* q = reinterpret_cast<const u32x4_t*>(tab + s0);
    const u32x4_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
    if (q3.x == kSlotEmpty || q3.x == kSlotBusy) break;
    const bool eq = k.w[0] == q0.x && k.w[1] == q0.y && k.w[2] == q0.z && k.w[3] == q0.w &&
                    k.w[4] == q1.x && k.w[5] == q1.y && k.w[6] == q1.z && k.w[7] == q1.w &&
                    k.w[8] == q2.x && k.w[9] == q2.y && k.w[10] == q2.z && k.w[11] == q2.w;
    if (eq) {
      if (q3.w == 0u) {  // not new in this call: numbered by an earlier one
        rec_slot[i] = s0;
        flow_idx[i] = q3.y;
        return;
      }
      break;
    }
  }
  for (uint32_t probe = 0; probe < max_probe; probe++, s = (s + 1) & cap_mask) {
    FlowSlot& sl = tab[s];
    uint32_t st = __hip_atomic_load(&sl.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (st == kSlotEmpty) {
      // the key is not in the table: a new key, if the table has room for one.  (A soft
      // bound: keys created concurrently may pass it together.  A reservation before the
      // claim would also count the records of one new key that race for its slot, and refuse
      // some of them -- the first record among them, which numbers the key.)
      const uint32_t held = *n_flows_before +
          __hip_atomic_load(n_new, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t exp = kSlotEmpty;
      if (held >= (cap_mask + 1u) / 2u) {
        // at the bound only a record that would CREATE its key is refused: a record of a key
        // another record is creating in this slot right now (it read n_new after that one's
        // add) sees the claim after a short wait and compares keys below.  A claim later than
        // the wait still gets a spurious refusal (mgenx.h: the caller redoes the batch).
        for (int spin = 0; spin < 64 && exp == kSlotEmpty; spin++) {
          __builtin_amdgcn_s_sleep(1);
          exp = __hip_atomic_load(&sl.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (exp == kSlotEmpty) break;
        st = exp;
      } else if (__hip_atomic_compare_exchange_strong(&sl.state, &exp, kSlotBusy, __ATOMIC_ACQ_REL,
                                                      __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) {
#pragma unroll
        for (int j = 0; j < 12; j++)
          __hip_atomic_store(&sl.key.w[j], k.w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sl.first_rec, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sl.is_new, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sl.index, kSlotBusy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sl.state, 1u + s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(n_new, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rec_slot[i] = s;
        return;
      } else {
        st = exp;
      }
    }
    // a slot being written: wait (bounded) until its key is published
    for (int spin = 0; st == kSlotBusy && spin < 1 << 20; spin++) {
      __builtin_amdgcn_s_sleep(1);
      st = __hip_atomic_load(&sl.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (st == kSlotBusy) break;  // never published: report and give up on this record
    if (key_eq(k, sl)) {
      // a key new in this call keeps its first record (most lookups see a smaller one
      // already and skip the atomic)
      const uint32_t nw = __hip_atomic_load(&sl.is_new, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nw && __hip_atomic_load(&sl.first_rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > i)
        __hip_atomic_fetch_min(&sl.first_rec, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // (a key new in this call is numbered and resolved by the later steps)
      if (!nw) flow_idx[i] = __hip_atomic_load(&sl.index, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      rec_slot[i] = s;
      return;
    }
  }
  rec_slot[i] = kSlotBusy;
  flow_idx[i] = MGENX_FLOW_NONE;
  __hip_atomic_fetch_add(overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Steps 2-3, each returning at once when the insert created no key (n_new == 0: every
// record's index was written by the insert).  1024-record blocks:
//   first:   flag[i] = record i is the first record of a key created by this call; the
//            block's flag count;
//   offsets: one workgroup scans the block counts (blk_base) and sets the new flow total;
//   number:  the flagged records' slots get n_flows + their rank among the flags;
//   resolve: every record reads its slot's index;  commit: the new keys are numbered.
constexpr uint32_t kFtBlock = 1024;
__global__ void __launch_bounds__(1024)
flowtab_first_kernel(const FlowSlot* __restrict__ tab, const uint32_t* __restrict__ rec_slot,
                     uint32_t n, uint32_t* __restrict__ flag, uint32_t* __restrict__ blk_cnt,
                     const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  __shared__ uint32_t ws[16];
  const uint32_t t = threadIdx.x, i = blockIdx.x * kFtBlock + t;
  bool f = false;
  if (i < n) {
    const uint32_t s = rec_slot[i];
    f = s != kSlotBusy && tab[s].is_new && tab[s].first_rec == i;
    flag[i] = f ? 1u : 0u;
  }
  const uint64_t b = __ballot(f);
  if ((t & 63u) == 0u) ws[t >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  if (t == 0) {
    uint32_t x = 0;
    for (int k = 0; k < 16; k++) x += ws[k];
    blk_cnt[blockIdx.x] = x;
  }
}

__global__ void __launch_bounds__(1024)
flowtab_offsets_kernel(const uint32_t* __restrict__ blk_cnt, uint32_t nblk,
                       uint32_t* __restrict__ blk_base, uint32_t* __restrict__ n_flows,
                       const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry_s;
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  if (t == 0) carry_s = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nblk; c0 += 1024u) {
    const uint32_t k = c0 + t;
    const uint32_t v = k < nblk ? blk_cnt[k] : 0u;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63u) ws[w] = incl;
    __syncthreads();
    uint32_t before = carry_s + incl - v, tot = 0;
    for (uint32_t q = 0; q < 16u; q++) {
      before += q < w ? ws[q] : 0u;
      tot += ws[q];
    }
    if (k < nblk) blk_base[k] = before;
    __syncthreads();
    if (t == 0) carry_s += tot;
    __syncthreads();
  }
  if (t == 0) n_flows[1] = n_flows[0] + carry_s;  // new total (published by commit)
}

__global__ void __launch_bounds__(1024)
flowtab_number_kernel(FlowSlot* __restrict__ tab, const uint32_t* __restrict__ rec_slot,
                      const uint32_t* __restrict__ flag, const uint32_t* __restrict__ blk_base,
                      uint32_t n, const uint32_t* __restrict__ n_flows,
                      const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  __shared__ uint32_t ws[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6, i = blockIdx.x * kFtBlock + t;
  const bool f = i < n && flag[i];
  const uint64_t b = __ballot(f);
  if (lane == 0) ws[w] = (uint32_t)__popcll(b);
  __syncthreads();
  uint32_t r = blk_base[blockIdx.x] +
               __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
  for (uint32_t q = 0; q < w; q++) r += ws[q];
  if (f) tab[rec_slot[i]].index = n_flows[0] + r;
}

__global__ void flowtab_resolve_kernel(const FlowSlot* __restrict__ tab,
                                       const uint32_t* __restrict__ rec_slot, uint32_t n,
                                       uint32_t* __restrict__ flow_idx,
                                       const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = rec_slot[i];
  flow_idx[i] = s == kSlotBusy ? MGENX_FLOW_NONE : tab[s].index;
}

__global__ void flowtab_commit_kernel(FlowSlot* __restrict__ tab, const uint32_t* __restrict__ rec_slot,
                                      const uint32_t* __restrict__ flag, uint32_t n,
                                      uint32_t* __restrict__ n_flows,
                                      const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) tab[rec_slot[i]].is_new = 0u;
  if (i == 0) n_flows[0] = n_flows[1];
}

// MgenAnalytic::Init's key fields (mgenAnalytic.cpp:28-71) of every numbered slot: the flow's
// report_msg key, at its dense index
__global__ void flowtab_keys_kernel(const FlowSlot* __restrict__ tab, uint32_t cap_slots,
                                    int protocol, mgenx_report_key* __restrict__ keys,
                                    uint32_t cap) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap_slots) return;
  const FlowSlot& sl = tab[s];
  if (sl.state == kSlotEmpty || sl.state == kSlotBusy || sl.index >= cap) return;
  const FlowKey& k = sl.key;
  mgenx_report_key o;
  const uint32_t dl = k.w[8] & 0xFFu, sl_ = k.w[9] & 0xFFu;
  o.dst.len = (uint8_t)dl;
  o.dst.type = dl == 4 ? 1 : dl == 16 ? 2 : 0;
  o.dst.port = (uint16_t)(k.w[8] >> 16);
  o.src.len = (uint8_t)sl_;
  o.src.type = sl_ == 4 ? 1 : sl_ == 16 ? 2 : 0;
  o.src.port = (uint16_t)(k.w[9] >> 16);
#pragma unroll
  for (int j = 0; j < 4; j++) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
      o.dst.addr[4 * j + b] = (uint8_t)(k.w[j] >> (8 * b));
      o.src.addr[4 * j + b] = (uint8_t)(k.w[4 + j] >> (8 * b));
    }
  }
  o.flow_id = k.w[10];
  o.protocol = (uint8_t)protocol;
  o.rsv[0] = o.rsv[1] = o.rsv[2] = 0;
  keys[sl.index] = o;
}

}  // namespace mgenx

using namespace mgenx;

struct mgenx_flow_table {
  int device = 0;
  uint32_t cap = 0;          // slots (power of two)
  FlowSlot* slots = nullptr;
  uint32_t* counters = nullptr;  // [0] = flows, [1] = scratch, [2] = overflow, [3] = keys created
  void* ws = nullptr;        // per-call scratch: rec_slot, flag, pos, cub temp
  size_t ws_bytes = 0;
};

extern "C" {

int mgenx_flow_table_create(mgenx_ctx* ctx, uint32_t max_flows, mgenx_flow_table** out) {
  if (!ctx || !out || max_flows == 0 || max_flows > (1u << 28)) return MGENX_EINVAL;
  *out = nullptr;
  mgenx_flow_table* t = new mgenx_flow_table();
  t->device = mgenx_ctx_device(ctx);
  uint32_t cap = 64;
  while (cap < 2u * max_flows) cap <<= 1;
  t->cap = cap;
  if (hipSetDevice(t->device) != hipSuccess ||
      hipMalloc((void**)&t->slots, (size_t)cap * sizeof(FlowSlot)) != hipSuccess ||
      hipMalloc((void**)&t->counters, 256) != hipSuccess ||
      hipMemset(t->slots, 0, (size_t)cap * sizeof(FlowSlot)) != hipSuccess ||
      hipMemset(t->counters, 0, 256) != hipSuccess) {
    mgenx_flow_table_destroy(t);
    return MGENX_ENOMEM;
  }
  *out = t;
  return MGENX_OK;
}

int mgenx_flow_table_destroy(mgenx_flow_table* t) {
  if (!t) return MGENX_EINVAL;
  mgenx::dev_free(t->slots);
  mgenx::dev_free(t->counters);
  mgenx::dev_free(t->ws);
  delete t;
  return MGENX_OK;
}

int mgenx_flow_lookup(mgenx_ctx* ctx, mgenx_flow_table* t, const mgenx_cols* cols,
                      const mgenx_addr* dev_src, uint32_t n, uint32_t* dev_flow_idx,
                      uint32_t* dev_n_flows, void* stream) {
  if (!ctx || !t || !cols) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  const mgenx_cols& c = *cols;
  if (!c.rows && (!c.dst_addr || !c.dst_len || !c.dst_port || !c.flow_id)) return MGENX_EINVAL;
  if (!dev_src || !dev_flow_idx) return MGENX_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nblk = (n + kFtBlock - 1) / kFtBlock;
  const size_t nb = ((size_t)n * 4 + 255) & ~(size_t)255;
  const size_t bb = ((size_t)nblk * 4 + 255) & ~(size_t)255;
  const size_t need = 2 * nb + 2 * bb + 256;
  if (t->ws_bytes < need) {
    mgenx::dev_free(t->ws);
    t->ws = nullptr;
    t->ws_bytes = 0;
    if (hipMalloc(&t->ws, need) != hipSuccess) return MGENX_ENOMEM;
    t->ws_bytes = need;
  }
  uint32_t* rec_slot = (uint32_t*)t->ws;
  uint32_t* flag = (uint32_t*)((char*)t->ws + nb);
  uint32_t* blk_cnt = (uint32_t*)((char*)t->ws + 2 * nb);
  uint32_t* blk_base = (uint32_t*)((char*)t->ws + 2 * nb + bb);
  uint32_t* n_new = t->counters + 3;
  const dim3 g((n + 255) / 256), b(256), gk(nblk), bk(kFtBlock);
  if (hipMemsetAsync(n_new, 0, 4, s) != hipSuccess) return MGENX_EDEVICE;
  hipLaunchKernelGGL(flowtab_insert_kernel, g, b, 0, s, t->slots, t->cap - 1, c, dev_src, n,
                     rec_slot, t->counters + 2, dev_flow_idx, n_new, t->counters);
  hipLaunchKernelGGL(flowtab_first_kernel, gk, bk, 0, s, t->slots, rec_slot, n, flag, blk_cnt,
                     n_new);
  hipLaunchKernelGGL(flowtab_offsets_kernel, dim3(1), dim3(1024), 0, s, blk_cnt, nblk, blk_base,
                     t->counters, n_new);
  hipLaunchKernelGGL(flowtab_number_kernel, gk, bk, 0, s, t->slots, rec_slot, flag, blk_base, n,
                     t->counters, n_new);
  hipLaunchKernelGGL(flowtab_resolve_kernel, g, b, 0, s, t->slots, rec_slot, n, dev_flow_idx,
                     n_new);
  hipLaunchKernelGGL(flowtab_commit_kernel, g, b, 0, s, t->slots, rec_slot, flag, n, t->counters,
                     n_new);
  if (dev_n_flows &&
      hipMemcpyAsync(dev_n_flows, t->counters, 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return MGENX_EDEVICE;
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

int mgenx_flow_keys(mgenx_ctx* ctx, const mgenx_flow_table* t, int protocol,
                    mgenx_report_key* dev_keys, uint32_t cap, void* stream) {
  if (!ctx || !t || (cap && !dev_keys)) return MGENX_EINVAL;
  if (cap == 0) return MGENX_OK;
  hipLaunchKernelGGL(flowtab_keys_kernel, dim3((t->cap + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, t->slots, t->cap, protocol, dev_keys, cap);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

}  // extern "C"
