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
#include <stdlib.h>
#include <algorithm>
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
__device__ __forceinline__ FlowKey make_key(const mgenx_cols& c, const mgenx_addr* src, uint32_t i,
                                            bool& keyed) {
  FlowKey k;
  uint32_t da[4] = {0u, 0u, 0u, 0u};
  uint32_t dl, dport, fid, err;
  if (c.rows) {  // the row's words 0 and 4..7: one 4-B and one 16-B load
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(c.rows + i);
    const u32x4_t h = *reinterpret_cast<const u32x4_t*>(rb + 16);
    fid = *reinterpret_cast<const uint32_t*>(rb);
    da[0] = h.x;                   // dst_addr4
    dport = h.y >> 16;             // dst_port (bytes 22-23)
    err = h.z >> 24;               // err (byte 27)
    dl = (h.w >> 8) & 0xffu;       // dst_len (byte 29)
  } else {
    dl = c.dst_len[i];
    dport = c.dst_port[i];
    fid = c.flow_id[i];
    err = c.err ? c.err[i] : 0u;
  }
  // an error, or (rows without dst_addr) a destination longer than the rows' 4 address bytes
  keyed = err == 0u && !(c.rows && !c.dst_addr && dl > 4u);
  if (c.dst_addr) {
    const u32x4_t d = *reinterpret_cast<const u32x4_t*>(c.dst_addr + (size_t)i * 16);
    da[0] = d.x;
    da[1] = d.y;
    da[2] = d.z;
    da[3] = d.w;
  }
  // mgenx_addr: type, len, port (word 0), 16 address bytes (words 1-4)
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(src + i);
  const uint32_t s0 = sw[0];
  const uint32_t sa[4] = {sw[1], sw[2], sw[3], sw[4]};
  const uint32_t sl = (s0 >> 8) & 0xffu, sport = s0 >> 16;
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
  k.w[9] = sl | sport << 16;
  k.w[10] = fid;
  k.w[11] = 0x4D47u;
  return k;
}

// The slot hash: add-rotate-xor steps over the 11 key words (one full-rate multiply-free step
// each; v_mul_lo_u32 runs at a quarter of the VALU rate, and the former 11 mix32 rounds were
// 22 of them per record), then one mix32 for the avalanche into the low bits the mask keeps.
// Each step is a bijection of h for a fixed word, so keys that differ in one word never
// collide.  (Any hash gives the same dense indices: they follow first-record order.)
__device__ __forceinline__ uint32_t key_hash(const FlowKey& k) {
  uint32_t h = 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 11; j++) {
    h ^= k.w[j];
    h = __builtin_rotateleft32(h, 13);
    h = h * 5u + 0xE6546B64u;
  }
  return mix32(h);
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

constexpr uint32_t kPend = 0xFFFFFFFEu;  // flow_idx of a record whose key this call created

// The table's atomic path for one record (key k, home slot s): a key published by an earlier
// call (found with plain loads first), or claimed / created here.  A record of a key created
// in this call gets rec_slot = its slot and flow_idx = kPend (numbered later); kFull: also the
// slot of a found key (the large-table resolve reads rec_slot of every record).
template <bool kFull>
__device__ __forceinline__ void insert_global(FlowSlot* __restrict__ tab, uint32_t cap_mask,
                                              const FlowKey& k, uint32_t i, uint32_t s,
                                              uint32_t* __restrict__ rec_slot,
                                              uint32_t* __restrict__ overflow,
                                              uint32_t* __restrict__ flow_idx,
                                              uint32_t* __restrict__ n_new, uint32_t nf_before) {
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
        if (kFull) rec_slot[i] = s0;
        flow_idx[i] = q3.y;
        return;
      }
      // created in this call (is_new is written before the state is released, and only the
      // numbering after the call clears it): the record takes the slot and keeps the key's
      // first record -- a stale first_rec is never below the current one, so the plain view
      // only skips atomics that would not lower it.  (The acquire path below invalidates
      // caches per probe: a fresh table's first call ran 4 ms for config 4 through it.)
      if (q3.z > i)
        __hip_atomic_fetch_min(&tab[s0].first_rec, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      rec_slot[i] = s0;
      flow_idx[i] = kPend;
      return;
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
      const uint32_t held = nf_before + __hip_atomic_load(n_new, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
        flow_idx[i] = kPend;
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
      flow_idx[i] = nw ? kPend : __hip_atomic_load(&sl.index, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (kFull || nw) rec_slot[i] = s;
      return;
    }
  }
  rec_slot[i] = kSlotBusy;
  flow_idx[i] = MGENX_FLOW_NONE;
  __hip_atomic_fetch_add(overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Large tables (more than kFtSmallCap slots): one record per thread, then steps 2-3 below.
__global__ void flowtab_insert_kernel(FlowSlot* __restrict__ tab, uint32_t cap_mask, mgenx_cols c,
                                      const mgenx_addr* __restrict__ src, uint32_t n,
                                      uint32_t* __restrict__ rec_slot, uint32_t* __restrict__ overflow,
                                      uint32_t* __restrict__ flow_idx, uint32_t* __restrict__ n_new,
                                      const uint32_t* __restrict__ n_flows_before) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool keyed;
  const FlowKey k = make_key(c, src, i, keyed);
  if (!keyed) {
    rec_slot[i] = kSlotBusy;
    flow_idx[i] = MGENX_FLOW_NONE;
    return;
  }
  insert_global<true>(tab, cap_mask, k, i, key_hash(k) & cap_mask, rec_slot, overflow, flow_idx,
                      n_new, *n_flows_before);
}

// Tables of at most kFtSmallCap slots (config 4: 1024 flows, 4096 slots): persistent
// workgroups, each first staging the table's published keys in LDS -- a slot map (dense index
// + 1, 0: not staged) and the 48-B keys by dense index, up to kFtKeys of them (80 KB with the
// map: two workgroups per CU) -- and probing there; a key not found in LDS (new in this call,
// or past the staged range) takes the atomic path.  Between calls every published slot is
// numbered, so the LDS copy is the table as this call found it, and its probe runs are the
// table's own.  The global probe this replaces reads a 64-B slot per record with four 16-B
// loads, each touching 64 different lines per wave instruction: ~100 us of config 4's
// lookups.  (Ablation, diagnostics build: mode 1 = the key loads and the hash only.)
constexpr uint32_t kFtSmallCap = 4096;
constexpr uint32_t kFtKeys = 1536;
constexpr uint32_t kFtLdsBytes = kFtSmallCap * 2u + kFtSmallCap / 2u * 48u;
__global__ void __launch_bounds__(1024)
flowtab_probe_kernel(FlowSlot* __restrict__ tab, uint32_t cap_mask, mgenx_cols c,
                     const mgenx_addr* __restrict__ src, uint32_t n,
                     uint32_t* __restrict__ rec_slot, uint32_t* __restrict__ overflow,
                     uint32_t* __restrict__ flow_idx, const uint32_t* __restrict__ n_flows,
                     uint32_t* __restrict__ n_new, uint32_t kcap, int mode) {
  extern __shared__ __attribute__((aligned(16))) uint32_t fsm[];
  const uint32_t cap = cap_mask + 1u, tid = threadIdx.x;
  uint16_t* map = reinterpret_cast<uint16_t*>(fsm);
  u32x4_t* keys = reinterpret_cast<u32x4_t*>(fsm + cap / 2u);  // kcap keys
  const uint32_t nf0 = *n_flows;  // keys numbered before this call
  for (uint32_t s = tid; s < cap; s += blockDim.x) {
    const u32x4_t* q = reinterpret_cast<const u32x4_t*>(tab + s);
    const u32x4_t q3 = q[3];
    const bool pub = q3.x != kSlotEmpty && q3.x != kSlotBusy && q3.y < kcap;
    map[s] = pub ? (uint16_t)(q3.y + 1u) : (uint16_t)0u;
    if (pub) {
      keys[3u * q3.y] = q[0];
      keys[3u * q3.y + 1u] = q[1];
      keys[3u * q3.y + 2u] = q[2];
    }
  }
  __syncthreads();
  const uint32_t max_probe = min(cap, kMaxProbe);
  // one record: the LDS probe, else the atomic path
  auto probe = [&](uint32_t i, const FlowKey& k) {
    const uint32_t h = key_hash(k) & cap_mask;
#if MGENX_DIAG
    if (mode == 1) { flow_idx[i] = h; return; }
#endif
    uint32_t s = h;
    for (uint32_t pr = 0; pr < max_probe; pr++, s = (s + 1u) & cap_mask) {
      const uint32_t e = map[s];
      if (e == 0u) break;
      const u32x4_t a = keys[3u * (e - 1u)], b = keys[3u * (e - 1u) + 1u], d = keys[3u * (e - 1u) + 2u];
      if (k.w[0] == a.x && k.w[1] == a.y && k.w[2] == a.z && k.w[3] == a.w && k.w[4] == b.x &&
          k.w[5] == b.y && k.w[6] == b.z && k.w[7] == b.w && k.w[8] == d.x && k.w[9] == d.y &&
          k.w[10] == d.z && k.w[11] == d.w) {
        flow_idx[i] = e - 1u;
        return;
      }
    }
    insert_global<false>(tab, cap_mask, k, i, h, rec_slot, overflow, flow_idx, n_new, nf0);
  };
  // two records per thread and step, their key loads issued together
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + tid; i < n; i += 2u * stride) {
    const uint32_t i2 = i + stride;
    const bool has2 = i2 < n;
    bool key1, key2;
    const FlowKey k1 = make_key(c, src, i, key1);
    const FlowKey k2 = make_key(c, src, has2 ? i2 : i, key2);
    if (!key1) flow_idx[i] = MGENX_FLOW_NONE;
    else probe(i, k1);
    if (has2) {
      if (!key2) flow_idx[i2] = MGENX_FLOW_NONE;
      else probe(i2, k2);
    }
  }
}

// Small tables, after the probe: one workgroup numbers the keys this call created, in order of
// their first record -- it collects them from the slots (at most kFtSmallCap) and sorts them in
// LDS -- so the large tables' flag / scan / number kernels are not needed; it also hands the
// flow count to the caller and clears the n_new word the next call counts in.  (A ticket for
// the probe kernel's last workgroup would need an agent-scope release per workgroup: on gfx950
// that writes back the XCD's L2, measured at ~1/4 ms per call.)
__global__ void __launch_bounds__(1024)
flowtab_number_small_kernel(FlowSlot* __restrict__ tab, uint32_t cap, uint32_t* __restrict__ n_flows,
                            const uint32_t* __restrict__ n_new, uint32_t* __restrict__ n_new_next,
                            uint32_t* __restrict__ out_n_flows) {
  __shared__ unsigned long long lst[kFtSmallCap];
  __shared__ uint32_t cnt_s;
  const uint32_t tid = threadIdx.x, nf0 = n_flows[0];
  uint32_t K = 0;
  if (*n_new != 0u) {
    if (tid == 0) cnt_s = 0u;
    __syncthreads();
    // (first record, slot) of every slot created by this call, sorted by first record
    for (uint32_t s = tid; s < cap; s += blockDim.x) {
      const FlowSlot& sl = tab[s];
      if (sl.state == kSlotEmpty || sl.state == kSlotBusy || !sl.is_new) continue;
      lst[atomicAdd(&cnt_s, 1u)] = (unsigned long long)sl.first_rec << 32 | s;
    }
    __syncthreads();
    K = cnt_s;
    uint32_t P = 1;
    while (P < K) P <<= 1;
    for (uint32_t j = K + tid; j < P; j += blockDim.x) lst[j] = ~0ull;
    __syncthreads();
    for (uint32_t kk = 2; kk <= P; kk <<= 1) {  // bitonic sort, ascending
      for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
        for (uint32_t x = tid; x < P; x += blockDim.x) {
          const uint32_t y = x ^ jj;
          if (y > x) {
            const unsigned long long u = lst[x], v = lst[y];
            if (((x & kk) == 0u) ? u > v : u < v) {
              lst[x] = v;
              lst[y] = u;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t j = tid; j < K; j += blockDim.x) {
      FlowSlot& sl = tab[(uint32_t)lst[j]];
      sl.index = nf0 + j;
      sl.is_new = 0u;
    }
  }
  if (tid == 0) {
    n_flows[0] = nf0 + K;
    if (out_n_flows) *out_n_flows = nf0 + K;
    *n_new_next = 0u;  // the word the next call counts in
  }
}

// Small tables: the records of keys created in this call read their index (none: return)
__global__ void flowtab_pending_kernel(const FlowSlot* __restrict__ tab,
                                       const uint32_t* __restrict__ rec_slot, uint32_t n,
                                       uint32_t* __restrict__ flow_idx,
                                       const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (flow_idx[i] == kPend) flow_idx[i] = tab[rec_slot[i]].index;
}

// Steps 2-3, each returning at once when the insert created no key (n_new == 0: every
// record's index was written by the insert), on grids of at most kFtGrid blocks looping over
// the 1024-record chunks (an early exit then costs little more than the launch):
//   first:   flag[i] = record i is the first record of a key created by this call; each
//            chunk's flag count;
//   offsets: one workgroup scans the chunk counts (blk_base) and sets the new flow total;
//   number:  the flagged records' slots get n_flows + their rank among the flags;
//   finish:  every record reads its slot's index, the new keys are committed, the flow count
//            goes to the caller, and the other n_new word is cleared for the next call (so no
//            memset or copy launches remain around the kernels).
constexpr uint32_t kFtBlock = 1024;
constexpr uint32_t kFtGrid = 512;
__global__ void __launch_bounds__(1024)
flowtab_first_kernel(const FlowSlot* __restrict__ tab, const uint32_t* __restrict__ rec_slot,
                     uint32_t n, uint32_t* __restrict__ flag, uint32_t* __restrict__ blk_cnt,
                     const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  __shared__ uint32_t ws[16];
  const uint32_t t = threadIdx.x, nblk = (n + kFtBlock - 1u) / kFtBlock;
  for (uint32_t cb = blockIdx.x; cb < nblk; cb += gridDim.x) {
    const uint32_t i = cb * kFtBlock + t;
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
      blk_cnt[cb] = x;
    }
    __syncthreads();
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
  if (t == 0) n_flows[1] = n_flows[0] + carry_s;  // new total (published by finish)
}

__global__ void __launch_bounds__(1024)
flowtab_number_kernel(FlowSlot* __restrict__ tab, const uint32_t* __restrict__ rec_slot,
                      const uint32_t* __restrict__ flag, const uint32_t* __restrict__ blk_base,
                      uint32_t n, const uint32_t* __restrict__ n_flows,
                      const uint32_t* __restrict__ n_new) {
  if (*n_new == 0u) return;
  __shared__ uint32_t ws[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6, nblk = (n + kFtBlock - 1u) / kFtBlock;
  for (uint32_t cb = blockIdx.x; cb < nblk; cb += gridDim.x) {
    const uint32_t i = cb * kFtBlock + t;
    const bool f = i < n && flag[i];
    const uint64_t b = __ballot(f);
    if (lane == 0) ws[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t r = blk_base[cb] +
                 __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    for (uint32_t q = 0; q < w; q++) r += ws[q];
    if (f) tab[rec_slot[i]].index = n_flows[0] + r;
    __syncthreads();
  }
}

__global__ void flowtab_finish_kernel(FlowSlot* __restrict__ tab,
                                      const uint32_t* __restrict__ rec_slot,
                                      const uint32_t* __restrict__ flag, uint32_t n,
                                      uint32_t* __restrict__ flow_idx, uint32_t* __restrict__ n_flows,
                                      const uint32_t* __restrict__ n_new, uint32_t* __restrict__ n_new_next,
                                      uint32_t* __restrict__ out_n_flows) {
  const bool created = *n_new != 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t nf = created ? n_flows[1] : n_flows[0];
    n_flows[0] = nf;
    *n_new_next = 0u;
    if (out_n_flows) *out_n_flows = nf;
  }
  if (!created) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = rec_slot[i];
    flow_idx[i] = s == kSlotBusy ? MGENX_FLOW_NONE : tab[s].index;  // (index: not is_new's word)
    if (flag[i]) tab[s].is_new = 0u;
  }
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

// mgenx_flow_span: per-flow record counts (global atomics), then the largest count and the
// receive-time range, each block folding its part first
__global__ void __launch_bounds__(256)
flow_span_count_kernel(const uint32_t* __restrict__ fidx, const uint32_t* __restrict__ sec,
                       const uint32_t* __restrict__ usec, uint32_t n, uint32_t n_flows,
                       uint32_t* __restrict__ counts, unsigned long long* __restrict__ out) {
  __shared__ unsigned long long lo_s[4], hi_s[4];
  unsigned long long lo = ~0ull, hi = 0ull;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t f = fidx[i];
    if (f >= n_flows) continue;
    atomicAdd(&counts[f], 1u);
    const unsigned long long t = (unsigned long long)sec[i] * 1000000ull + usec[i];
    lo = t < lo ? t : lo;
    hi = t > hi ? t : hi;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 0u) {
    lo_s[w] = lo;
    hi_s[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; k++) {
      lo = lo_s[k] < lo ? lo_s[k] : lo;
      hi = hi_s[k] > hi ? hi_s[k] : hi;
    }
    if (lo != ~0ull) atomicMin(&out[1], lo);
    if (hi != 0ull) atomicMax(&out[2], hi);
  }
}

__global__ void __launch_bounds__(256)
flow_span_max_kernel(const uint32_t* __restrict__ counts, uint32_t n_flows,
                     unsigned long long* __restrict__ out) {
  uint32_t m = 0;
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < n_flows; f += gridDim.x * blockDim.x)
    m = max(m, counts[f]);
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63u) == 0u && m) atomicMax(&out[0], (unsigned long long)m);
}

__global__ void flow_span_init_kernel(unsigned long long* out) {
  out[0] = 0ull;
  out[1] = ~0ull;
  out[2] = 0ull;
}

}  // namespace mgenx

using namespace mgenx;

struct mgenx_flow_table {
  int device = 0;
  uint32_t cap = 0;          // slots (power of two)
  FlowSlot* slots = nullptr;
  uint32_t* counters = nullptr;  // [0] = flows, [1] = scratch, [2] = overflow, [3] / [4] = keys
                                 // created (alternate calls)
  uint32_t parity = 0;
  int cu = 256;              // compute units (the small-table path's grid)
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
  int cu = 0;
  if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, t->device) == hipSuccess && cu > 0)
    t->cu = cu;
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
  // n_new alternates between counters[3] and [4]: each call clears the word the next call
  // counts in
  uint32_t* n_new = t->counters + 3 + (t->parity & 1u);
  uint32_t* n_new_next = t->counters + 3 + ((t->parity + 1u) & 1u);
  t->parity++;
  int mode = 0;
#if MGENX_DIAG
  if (const char* m = getenv("MGENX_FT_MODE")) mode = atoi(m);
#endif
  const dim3 b(256), bk(kFtBlock);
  if (t->cap <= kFtSmallCap) {
    hipError_t e = set_max_lds((const void*)flowtab_probe_kernel, (int)kFtLdsBytes);
    if (e != hipSuccess) return MGENX_EDEVICE;
    // keys staged: up to kFtKeys (80 KB of LDS with the map: two workgroups per CU)
    uint32_t kcap = std::min(t->cap / 2u, kFtKeys), gmul = 2;
#if MGENX_DIAG
    if (const char* v = getenv("MGENX_FT_KCAP")) kcap = std::min(t->cap / 2u, (uint32_t)atoi(v));
    if (const char* v = getenv("MGENX_FT_GMUL")) gmul = (uint32_t)std::max(1, atoi(v));
#endif
    const uint32_t grid = std::max(1u, std::min((uint32_t)t->cu * gmul, (n + 2047u) / 2048u));
    hipLaunchKernelGGL(flowtab_probe_kernel, dim3(grid), dim3(1024), t->cap * 2u + kcap * 48u, s,
                       t->slots, t->cap - 1, c, dev_src, n, rec_slot, t->counters + 2,
                       dev_flow_idx, t->counters, n_new, kcap, mode);
    hipLaunchKernelGGL(flowtab_number_small_kernel, dim3(1), dim3(1024), 0, s, t->slots, t->cap,
                       t->counters, n_new, n_new_next, dev_n_flows);
    hipLaunchKernelGGL(flowtab_pending_kernel, dim3(std::min((n + 255u) / 256u, 4u * kFtGrid)), b,
                       0, s, t->slots, rec_slot, n, dev_flow_idx, n_new);
    return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
  }
  const uint32_t gs = std::min(nblk, kFtGrid), gf = std::min((n + 255u) / 256u, 4u * kFtGrid);
  hipLaunchKernelGGL(flowtab_insert_kernel, dim3((n + 255) / 256), b, 0, s, t->slots, t->cap - 1,
                     c, dev_src, n, rec_slot, t->counters + 2, dev_flow_idx, n_new, t->counters);
  hipLaunchKernelGGL(flowtab_first_kernel, dim3(gs), bk, 0, s, t->slots, rec_slot, n, flag,
                     blk_cnt, n_new);
  hipLaunchKernelGGL(flowtab_offsets_kernel, dim3(1), dim3(1024), 0, s, blk_cnt, nblk, blk_base,
                     t->counters, n_new);
  hipLaunchKernelGGL(flowtab_number_kernel, dim3(gs), bk, 0, s, t->slots, rec_slot, flag, blk_base,
                     n, t->counters, n_new);
  hipLaunchKernelGGL(flowtab_finish_kernel, dim3(gf), b, 0, s, t->slots, rec_slot, flag, n,
                     dev_flow_idx, t->counters, n_new, n_new_next, dev_n_flows);
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

int mgenx_flow_span(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_rx_sec,
                    const uint32_t* dev_rx_usec, uint32_t n, uint32_t n_flows,
                    uint32_t* dev_counts, uint64_t* dev_out, void* stream) {
  if (!ctx || !dev_out || (n && (!dev_flow_idx || !dev_rx_sec || !dev_rx_usec)) ||
      (n_flows && !dev_counts))
    return MGENX_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* out = reinterpret_cast<unsigned long long*>(dev_out);
  hipLaunchKernelGGL(flow_span_init_kernel, dim3(1), dim3(1), 0, s, out);
  if (n && n_flows) {
    if (hipMemsetAsync(dev_counts, 0, (size_t)n_flows * 4, s) != hipSuccess) return MGENX_EDEVICE;
    const uint32_t g = std::min((n + 255u) / 256u, 2048u);
    hipLaunchKernelGGL(flow_span_count_kernel, dim3(g), dim3(256), 0, s, dev_flow_idx, dev_rx_sec,
                       dev_rx_usec, n, n_flows, dev_counts, out);
    hipLaunchKernelGGL(flow_span_max_kernel, dim3(std::min((n_flows + 255u) / 256u, 256u)),
                       dim3(256), 0, s, dev_counts, n_flows, out);
  }
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

}  // extern "C"
