// mgenx_scan.hip -- record-boundary scan of TCP / SINK byte streams on gfx950.
//
// Reference semantics (the oracle restates them in or_tcp_scan / or_sink_scan):
//   TCP   MgenTcpTransport::GetRxNumBytes / OnRecvMsg (src/common/mgenTransport.cpp:1683-1760):
//         a record starts with its big-endian u16 msg_len; msg_len < 4 is a stream error
//         (scan stops); an incomplete last record stays unconsumed.
//   SINK  MgenAppSinkTransport::OnInputReady (src/common/mgenAppSinkTransport.cpp:369-434):
//         msg_len outside [MIN_SIZE, MAX_SIZE] discards the two length bytes (resync).
// The framing is a sequential chain p_{i+1} = p_i + L(p_i).  On the GPU:
//   1. detect: one coalesced streaming pass (each workgroup a 32 KiB block, 4 KiB per step
//      through LDS so every position sees its 3 following bytes) flags plausible starts
//      (L in range, record inside the stream, version byte == 2) into ordered per-block slots;
//   2. compact (device scan of the block counts) + link: successor = the candidate at p + L,
//      searched in the target block's own slot list, or a terminal;
//   3. base-4 lifting (pointer jumping, ceil(log4 n) levels) gives the chain from any
//      candidate; the chain from offset 0 is enumerated in parallel and reports where it
//      ends -- with the candidate total, the only device-to-host copies of the common path.
//      A whole-stream scan first checks the regular case (link: every candidate's successor
//      is the next candidate): the records are then the candidates, and no lifting runs;
//   4. where the chain leaves the candidate set (a record with a bad version, SINK garbage,
//      a partial tail before the end, TCP msg_len < 4, or a block with more plausible starts
//      than slots) a single-thread resolver walks the reference rule exactly until it
//      re-enters the set.  Valid streams never need step 4.
// Bit-exact with the sequential rule for every input: candidates only shortcut positions
// the chain would compute anyway.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "mgenx_kernels.hpp"

namespace mgenx {

// (MGENX_SCAN_BLOCK / MGENX_SCAN_THREADS: build-time overrides for geometry experiments)
#ifndef MGENX_SCAN_BLOCK
#define MGENX_SCAN_BLOCK 32768
#endif
#ifndef MGENX_SCAN_THREADS
#define MGENX_SCAN_THREADS 256
#endif
constexpr uint32_t kScanBlockBytes = MGENX_SCAN_BLOCK;  // detect block (one workgroup)
constexpr uint32_t kScanThreads = MGENX_SCAN_THREADS;   // 16 B per thread and step
constexpr uint32_t kScanSlots = 4096;        // candidates per block before overflow
// a slot: in-block offset (bits 0-14) | header copy (bit 15, is_copy) | length << 16
constexpr uint32_t kSlotOff = 0x7FFFu, kSlotCopy = 0x8000u;
static_assert(kScanBlockBytes <= 32768, "slot offsets are 15 bits");
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct ScanMode {
  uint32_t min_len, max_len;
};

__device__ __forceinline__ uint32_t be16_at(const uint8_t* s, uint64_t p) {
  return ((uint32_t)s[p] << 8) | s[p + 1];
}

constexpr uint32_t kScanSteps = kScanBlockBytes / (kScanThreads * 16);  // 16

// candidate mask of the 16 positions of one lane's 16-byte chunk w[0..3] (w[4] = the 4 bytes
// after it); `mine` = stream offset of the chunk
__device__ __forceinline__ uint32_t detect_hits(const uint32_t (&w)[5], uint64_t mine,
                                                uint64_t nbytes, ScanMode m) {
  uint32_t hits = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t x = w[k];
    const uint32_t z = x ^ 0x02020202u;
    uint32_t mb = (z - 0x01010101u) & ~z & 0x80808080u;  // bytes == 0x02 (may over-flag)
    if (k == 0) mb &= 0x80800000u;                       // positions -2, -1 are not ours
    if (k == 4) mb &= 0x00008080u;                       // positions 16, 17 neither
    while (mb) {
      const int bb = __ffs(mb) / 8 - 1;  // byte index in the word
      mb &= mb - 1;
      if (((x >> (8 * bb)) & 0xffu) != 2u) continue;
      const int i = 4 * k + bb - 2;      // position whose version byte this is
      const uint64_t p = mine + (uint64_t)i;
      if (p + 4 > nbytes) continue;
      const uint32_t b0 = (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
      const int j = i + 1;
      const uint32_t b1 = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
      const uint32_t L = (b0 << 8) | b1;
      if (L >= m.min_len && L <= m.max_len && p + L <= nbytes) hits |= 1u << i;
    }
  }
  return hits;
}

// Copies of a header inside a TCP message: MgenTcpTransport sends a fragment over 8192 bytes
// as its 8-KiB Pack buffer re-sent from the start (mgenTransport.cpp:1818-1876), so such a
// message carries its own header again at +8192, +16384, ... -- plausible starts that are not
// records (config 5's stream has 2 candidates per record, and the chain then needs the
// lifting).  A candidate whose first 16 bytes equal the 16 bytes 8192 earlier is taken for a
// copy by the chain hypothesis of scan_chain_* (checked there: a wrong guess only costs the
// exact path).  Detect sets that bit in the candidate's slot from two loads side by side (its
// length re-read is one of them).  (Dropping the copies in detect instead cost detect 172 ->
// 201 us in round 3: the extra dependent loads lengthened every block.)
constexpr uint64_t kCopyDist = 8192;

// exclusive prefix over the lanes of the wave and the wave total of c (0..16), by ballots
__device__ __forceinline__ uint32_t wave_excl(uint32_t c, uint32_t& wtot) {
  uint32_t excl = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < 5; b++) {
    const uint64_t mk = __ballot((c >> b) & 1u);
    excl += __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u)) << b;
    tot += (uint32_t)__popcll(mk) << b;
  }
  wtot = tot;
  return excl;
}

// 1. detect.  Workgroup b scans block b (32 KiB) as 8 steps of 4 KiB; lane t of the
// workgroup owns bytes [16 t, 16 t + 16) of every step, so each wave load instruction reads
// 1 KiB contiguously.  All 8 loads are issued up front (32 KiB in flight per workgroup;
// 52 VGPRs, 8 waves per SIMD.  64-KiB blocks (16 loads, 84 VGPRs, 5 waves per SIMD) ran the
// config-5 scan in 0.304 ms, 32 KiB in 0.280-0.285 ms; 512- and 1024-thread blocks were
// slower: scripts/scan_geom_build.sh + scan_time.py).
// A position needs the 3 bytes after it: the next lane's first word comes by a lane shift,
// across waves through LDS.  Candidates go to the block's slots in stream order (step-major,
// then lane): per-step wave prefixes by ballot, one workgroup barrier for the wave totals.
// Writes counts[b] = candidates (low word) | overflowed << 32 (a block with more candidates
// than slots writes none), and block 0 zeroes counts[n_blocks]: the exclusive scan's last
// entry then holds the candidate total and the number of overflowing blocks in one word.
// kRedo: the second pass over the overflowing blocks only, once the offsets are known:
// positions go straight to cand[base[b] ...] with no slot limit.
// kPlain (diagnostics build, MGENX_SCAN_PLAIN=1): plain instead of non-temporal loads
template <bool kRedo, bool kPlain = false>
__global__ void __launch_bounds__(kScanThreads)
scan_detect_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, ScanMode m,
                   uint32_t* __restrict__ slots, uint64_t* __restrict__ counts,
                   const uint64_t* __restrict__ base, uint64_t* __restrict__ cand,
                   uint32_t* __restrict__ irregular) {
  constexpr uint32_t kW = kScanThreads / 64;
  if (kRedo && !(counts[blockIdx.x] >> 32)) return;
  __shared__ uint32_t first[kScanSteps + 1][kW];  // first word of each wave's chunk per step
  __shared__ uint32_t wsum[kScanSteps][kW];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t block0 = (uint64_t)blockIdx.x * kScanBlockBytes;
  u32x4_t v[kScanSteps];
  if (block0 + kScanBlockBytes <= nbytes) {
#pragma unroll
    for (uint32_t st = 0; st < kScanSteps; st++)
      v[st] = kPlain ? ldu128(s + block0 + st * (kScanThreads * 16) + 16u * t)
                     : ldnt128(s + block0 + st * (kScanThreads * 16) + 16u * t);  // read once
  } else {
#pragma unroll
    for (uint32_t st = 0; st < kScanSteps; st++) {
      const uint64_t mine = block0 + st * (kScanThreads * 16) + 16u * t;
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      if (mine + 16 <= nbytes) {
        const u32x4_t x = ldu128(s + mine);
        w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
      } else {
        for (uint32_t k = 0; k < 16 && mine + k < nbytes; k++)
          w[k >> 2] |= (uint32_t)s[mine + k] << (8 * (k & 3));
      }
      v[st] = u32x4_t{w[0], w[1], w[2], w[3]};
    }
  }
  if (lane == 0) {
#pragma unroll
    for (uint32_t st = 0; st < kScanSteps; st++) first[st][wv] = v[st].x;
  }
  if (t == 0) {  // the 4 bytes after the block
    const uint64_t q = block0 + kScanBlockBytes;
    uint32_t x = 0;
    for (uint32_t k = 0; k < 4; k++)
      if (q + k < nbytes) x |= (uint32_t)s[q + k] << (8 * k);
    first[kScanSteps][0] = x;
  }
  __syncthreads();
  uint32_t hits[kScanSteps];
#pragma unroll
  for (uint32_t st = 0; st < kScanSteps; st++) {
    uint32_t nxt = __shfl_down(v[st].x, 1);
    if (lane == 63) nxt = wv + 1 < kW ? first[st][wv + 1] : first[st + 1][0];
    const uint32_t w[5] = {v[st].x, v[st].y, v[st].z, v[st].w, nxt};
    const uint64_t mine = block0 + st * (kScanThreads * 16) + 16u * t;
    hits[st] = detect_hits(w, mine, nbytes, m);
    const uint64_t any = __ballot(hits[st] != 0u);
    uint32_t wt = 0;
    if (any) (void)wave_excl(__popc(hits[st]), wt);
    if (lane == 0) wsum[st][wv] = wt;
  }
  __syncthreads();
  uint32_t total = 0;
#pragma unroll
  for (uint32_t st = 0; st < kScanSteps; st++)
#pragma unroll
    for (uint32_t k = 0; k < kW; k++) total += wsum[st][k];
  const bool ovf = !kRedo && total > kScanSlots;
  if (!ovf && total) {
    uint32_t* out = slots + (size_t)blockIdx.x * kScanSlots;
    uint64_t* outc = kRedo ? cand + (uint32_t)base[blockIdx.x] : nullptr;
    uint32_t run = 0;
#pragma unroll
    for (uint32_t st = 0; st < kScanSteps; st++) {
      uint32_t before = 0, stot = 0;
#pragma unroll
      for (uint32_t k = 0; k < kW; k++) {
        before += k < wv ? wsum[st][k] : 0u;
        stot += wsum[st][k];
      }
      if (stot) {
        uint32_t h = hits[st], wt;
        uint32_t pos = run + before + wave_excl(__popc(h), wt);
        while (h) {
          const int i = __ffs(h) - 1;
          h &= h - 1;
          const uint32_t off = 16u * (st * kScanThreads + t) + (uint32_t)i;
          if (kRedo) {
            outc[pos++] = block0 + off;
          } else {
            // the slot keeps the candidate's length field too, so the link step reads no
            // stream bytes: re-read here, where the block's bytes were just loaded (keeping
            // the 16 loaded rows live until this loop instead costs 32 VGPRs and occupancy);
            // beside it the 16 bytes 8192 earlier, for the header-copy bit (is_copy: two
            // loads side by side, no extra round trip)
            const uint64_t p = block0 + off;
            uint32_t L, cp = 0u;
            if (p + 16 <= nbytes) {
              const u32x4_t a = ldu128(s + p);
              const u32x4_t c = ldu128(s + (p >= kCopyDist ? p - kCopyDist : p));
              L = ((a.x & 0xFFu) << 8) | ((a.x >> 8) & 0xFFu);
              cp = p >= kCopyDist && a.x == c.x && a.y == c.y && a.z == c.z && a.w == c.w
                       ? kSlotCopy : 0u;
            } else {
              L = be16_at(s, p);
            }
            out[pos++] = off | cp | (L << 16);
          }
        }
      }
      run += stot;
    }
  }
  if (!kRedo && t == 0) {
    counts[blockIdx.x] = (uint64_t)total | (ovf ? (1ull << 32) : 0ull);
    if (blockIdx.x == 0) {
      counts[gridDim.x] = 0u;
      if (irregular) *irregular = 0u;  // the link step's flag (it runs after this kernel)
    }
  }
}

// the lifting tables of one build: ups / dists [levels + 1][stride], the 2- and 3-jump tables
// [levels][stride]
struct LiftTabs {
  const uint32_t *ups, *dists, *ups2, *ups3, *dists2, *dists3;
  uint32_t stride;
  int levels;
};

// where an enumerated chain stops: its record count and the position after its last record
struct ChainEnd {
  uint64_t count, next_pos;
  uint64_t more;  // the last node has a successor candidate (the descent hit its depth)
};

// 2. compact + link, one wave per block: candidate positions into the global sorted
// array, and each candidate's successor p + L searched in the target block's own slots
// (sorted, usually a handful) -- or, for a block that overflowed its slots, in its range of
// cand, written by the second detect pass.  up0 = successor (self for a terminal),
// dist0 = 1 if linked.
constexpr uint32_t kLinkPerWave = 4;  // detect blocks per link wave
__global__ void __launch_bounds__(256)
scan_link_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, const uint32_t* __restrict__ slots,
                 const uint64_t* __restrict__ counts, const uint64_t* __restrict__ base,
                 uint32_t n_blocks, uint64_t* __restrict__ cand, uint32_t* __restrict__ up,
                 uint32_t* __restrict__ dist, uint64_t spec_cap, uint32_t* __restrict__ irregular) {
  // 16 lanes per detect block, 4 blocks per wave (a block holds a handful of candidates)
  const uint32_t b =
      (blockIdx.x * 4 + (threadIdx.x >> 6)) * kLinkPerWave + ((threadIdx.x & 63u) >> 4);
  const uint32_t sub = threadIdx.x & 15u;
  const bool live = b < n_blocks;
  // irregular (optional): set unless every candidate's successor is the next candidate and
  // the last one is terminal -- then the chain from candidate 0 is the whole candidate list
  const uint64_t n_tot = base[n_blocks];
  bool odd = false;
  // speculative build (tables sized before the candidate total was known): nothing when the
  // total exceeds them; an overflowing block (its candidates need the second detect pass)
  // gets terminal entries -- the host sees either case and rebuilds exactly
  if (spec_cap && base[n_blocks] > spec_cap) return;
  const uint64_t cw = live ? counts[b] : 0ull;
  const uint32_t c = (uint32_t)cw;
  const uint32_t o = live ? (uint32_t)base[b] : 0u;
  if (spec_cap && (cw >> 32)) {
    for (uint32_t k = sub; k < c; k += 16) {
      up[o + k] = o + k;
      dist[o + k] = 0u;
    }
    if (irregular && c && sub == 0u) *irregular = 1u;
  }
  for (uint32_t k = sub; k < c && !(spec_cap && (cw >> 32)); k += 16) {
    uint64_t p, nx;
    if (cw >> 32) {
      p = cand[o + k];
      nx = p + be16_at(s, p);
    } else {
      const uint32_t sl = slots[(size_t)b * kScanSlots + k];  // offset | length << 16
      p = (uint64_t)b * kScanBlockBytes + (sl & kSlotOff);
      nx = p + (sl >> 16);
      cand[o + k] = p;
    }
    uint32_t tgt = kNone;
    if (nx + 2 <= nbytes) {
      const uint64_t bl = nx / kScanBlockBytes;
      if (bl < n_blocks) {
        const uint64_t cbw = counts[bl];
        const uint32_t cb = (uint32_t)cbw, ob = (uint32_t)base[bl];
        uint32_t lo = 0, hi = cb;
        if (cbw >> 32) {
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (cand[ob + mid] < nx) lo = mid + 1; else hi = mid;
          }
          if (lo < cb && cand[ob + lo] == nx) tgt = ob + lo;
        } else {
          const uint32_t* ts = slots + (size_t)bl * kScanSlots;
          const uint32_t key = (uint32_t)(nx % kScanBlockBytes);
          if (cb <= 8) {  // the usual handful: all loads side by side, one compare each
            uint32_t w[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) w[j] = j < cb ? ts[j] : 0xFFFFFFFFu;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++)
              if (tgt == kNone && (w[j] & kSlotOff) == key && j < cb) tgt = ob + j;
          } else {
            while (lo < hi) {
              const uint32_t mid = (lo + hi) >> 1;
              if ((ts[mid] & kSlotOff) < key) lo = mid + 1; else hi = mid;
            }
            if (lo < cb && (ts[lo] & kSlotOff) == key) tgt = ob + lo;
          }
        }
      }
    }
    up[o + k] = tgt == kNone ? o + k : tgt;
    dist[o + k] = tgt == kNone ? 0u : 1u;
    const uint64_t ci = (uint64_t)o + k;
    odd = odd || (ci + 1 < n_tot ? tgt != o + k + 1 : tgt != kNone);
  }
  // a plain store of the same value by every irregular wave: no read-modify-write to
  // serialise on one word (an atomic per wave cost 180 us on a 1-GiB stream)
  if (irregular && __ballot(odd) && (threadIdx.x & 63u) == 0u) *irregular = 1u;
}

// The regular case of the chain from offset 0 (no lifting): when the link step found every
// candidate's successor to be the next candidate (and candidate 0 at offset 0), the records
// are the candidates themselves.  Otherwise thread 0 reports `more` = 2: the caller lifts.
__global__ void __launch_bounds__(256)
scan_enum_regular_kernel(const uint8_t* __restrict__ s, const uint64_t* __restrict__ cand,
                         const uint64_t* __restrict__ total, const uint32_t* __restrict__ irregular,
                         uint32_t stride, uint64_t cap, uint64_t* __restrict__ rec_off,
                         uint32_t* __restrict__ rec_len, ChainEnd* __restrict__ end,
                         uint32_t* __restrict__ done, uint64_t* __restrict__ host_regular) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n = *total;
  const bool ok = *irregular == 0u && n != 0 && n <= stride && cand[0] == 0;
  if (i == 0) {
    *done = ok ? 1u : 0u;  // read by the lifting and enumeration launches that follow
    if (host_regular) *host_regular = ok ? 1u : 0u;
    if (ok) {
      const uint64_t tp = cand[n - 1];
      end->count = n;
      end->next_pos = tp + be16_at(s, tp);
      end->more = 0;
    } else {
      end->count = 0;
      end->next_pos = 0;
      end->more = 2;
    }
  }
  if (!ok || i >= n || i >= cap) return;
  const uint64_t p = cand[i];
  rec_off[i] = p;
  rec_len[i] = be16_at(s, p);
}

// The chain from offset 0 on a speculative whole-stream TCP scan, with no candidate table, no
// link and no lifting.  (Config 5's stream is not regular: the TCP sender re-sends each
// message's 8-KiB Pack buffer, so every message carries a copy of its header 8192 bytes on.)
// A hypothesis H is guessed from successor marks and then PROVED:
//   marks: every candidate p that is not a header copy (the slot's copy bit) marks its
//   successor q = p + L when q is a candidate (a candidate marked by two keeps no marker);
//   H = {0} and every marked candidate whose marker is 0 or itself marked (or is not known).
//   (Junk starts inside headers chain in short runs -- seq 0x802 reads as a length-8 record at
//   header offset 9 whose successor at 17 is tx_usec's same bytes -- and nothing marks the
//   junk start, so its successor stays out.)
// H is the chain from offset 0 exactly when 0 is in H, each member's successor is the next
// member in position order and the last member's successor is not a candidate: the kernel
// checks the first two within each group while it writes H out in order, the host the joins
// between groups and the last successor; otherwise the host rebuilds exactly.
// A record is shorter than 64 KiB = 2 detect blocks, so every mark that decides H for a group's
// candidates comes from its own detect blocks or the 4 before them: each group loads those
// candidates into LDS and marks there -- no candidate numbering across groups, no table in
// memory, no wait on other groups except the ranks (one decoupled look-back).
// one group's summary for the host, ONE 16-byte granule written by one store (its epoch word
// comes with it: no ordering between two stores to wait for):
//   bits   0..39  position of its first H member     66..78  H members (nh)
//          40..65 last member's successor - first     79..91  own candidates (saturating)
//          92     not proved here (fail)              93      last successor is a candidate
//          94..115 epoch
struct ChainAux {
  uint64_t lo, hi;
};
__host__ __device__ inline uint32_t aux_bits(const ChainAux& a, int at, int n) {
  const unsigned __int128 v = ((unsigned __int128)a.hi << 64) | a.lo;
  return (uint32_t)((v >> at) & (((unsigned __int128)1 << n) - 1));
}
constexpr uint32_t kChainEpochs = 1u << 22;  // look-back words: epoch << 40 | kind << 38 | count
constexpr uint32_t kChainThreads = 1024;
constexpr uint32_t kChainBlocks = 1024;  // detect blocks per group at most (4 more are loaded)
constexpr uint32_t kChainCands = 4096;   // candidates per group at most, incl. the 4 blocks before
constexpr uint32_t kChainPer = kChainCands / kChainThreads;
constexpr uint32_t kChainBack = 4;       // detect blocks before a group's own whose marks count
constexpr uint32_t kChainAhead = 2;      // and after them (the last member's successor)
constexpr uint32_t kChainGroups = 1024;
constexpr uint32_t kChainSpin = 1u << 18;  // polls of another group's word before giving up
constexpr uint32_t kMarkMulti = 0xFFFFFFFFu;  // marked by two candidates

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t chain_word(uint32_t epoch, uint32_t kind, uint64_t v) {
  return ((uint64_t)epoch << 40) | ((uint64_t)kind << 38) | v;
}

#if MGENX_DIAG
// s_memtime at the phase ends of scan_chain_kernel, thread 0 of groups 0..63 (diagnostics)
__device__ unsigned long long g_chain_prof[64 * 8];
#define CHAIN_STAMP(k)                                                                 \
  do {                                                                                 \
    if (tid == 0 && g < 64) g_chain_prof[g * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define CHAIN_STAMP(k) \
  do {                 \
  } while (0)
#endif

// One kernel after detect.  Group g owns detect blocks [g per_group, (g + 1) per_group) and
// loads the candidates of those and the kChainBack blocks before them into LDS (positions
// relative to the first loaded block, copy bit in bit 31, lengths):
//  1. the loaded blocks' candidate counts -> an exclusive prefix; candidate j -> (block, slot)
//     by a binary search of it;
//  2. marks: each non-copy candidate finds its successor among the loaded positions (binary
//     search) and marks it with its own index (an LDS CAS; a second marker leaves kMarkMulti);
//  3. the H members among its own candidates -> an LDS index list by ballot ranks;
//  4. its H count as an aggregate, a decoupled look-back over the earlier groups for its first
//     rank (bounded: dispatch order is not promised -- a group that gives up fails the scan,
//     which the host then redoes on the exact path), the list out to rec_off / rec_len, each
//     member's successor compared with the next;
//  5. its summary to host memory.
__global__ void __launch_bounds__(kChainThreads)
scan_chain_kernel(const uint32_t* __restrict__ slots, const uint64_t* __restrict__ counts,
                  uint64_t nbytes, uint32_t n_blocks, uint32_t per_group, uint32_t epoch,
                  uint64_t* __restrict__ status, uint64_t cap, uint64_t* __restrict__ rec_off,
                  uint32_t* __restrict__ rec_len, ChainAux* __restrict__ host_aux) {
  __shared__ uint32_t pre[kChainBlocks + kChainBack + kChainAhead + 1];
  __shared__ uint32_t cpos[kChainCands];   // position - bx * block bytes | copy << 31
  __shared__ uint16_t clen[kChainCands];
  __shared__ uint32_t cmark[kChainCands];  // 0: unmarked; marker index + 1; kMarkMulti
  __shared__ uint16_t hlist[kChainCands];  // H members (indices), in order
  __shared__ uint16_t cblk[kChainCands];   // candidate -> loaded block
  __shared__ uint32_t wsum[kChainThreads / 64];
  __shared__ uint32_t wsum4[kChainPer][kChainThreads / 64];
  __shared__ uint32_t sh[2];  // fail, tail candidate
  __shared__ uint64_t s_prefix;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  constexpr uint32_t kW = kChainThreads / 64;
  const uint32_t g = blockIdx.x;
  const uint32_t b0 = min(g * per_group, n_blocks), b1 = min(b0 + per_group, n_blocks);
  const uint32_t bx = b0 >= kChainBack ? b0 - kChainBack : 0u;  // first loaded block
  const uint32_t nblk = min(b1 + kChainAhead, n_blocks) - bx;     // loaded blocks
  const uint64_t base_pos = (uint64_t)bx * kScanBlockBytes;
  CHAIN_STAMP(0);
  if (tid == 0) {
    sh[0] = 0u;
    sh[1] = 0u;
  }
  // 1. candidate counts -> exclusive prefix (thread t owns K <= 3 consecutive entries)
  bool fail = false;
  for (uint32_t i = tid; i < nblk; i += kChainThreads) {
    const uint64_t w = counts[bx + i];
    pre[i] = (uint32_t)w;
    fail = fail || (w >> 32) != 0u;  // an overflowed block has no slots
  }
  for (uint32_t i = tid; i < kChainCands; i += kChainThreads) cmark[i] = 0u;
  __syncthreads();
  const uint32_t K = (nblk + kChainThreads - 1) / kChainThreads;
  const uint32_t i0 = min(tid * K, nblk), i1 = min(i0 + K, nblk);
  uint32_t tot = 0;
  for (uint32_t i = i0; i < i1; i++) tot += pre[i];
  uint32_t incl = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63u) wsum[wv] = incl;
  __syncthreads();
  uint32_t run = incl - tot, C = 0;
#pragma unroll
  for (uint32_t k = 0; k < kW; k++) {
    run += k < wv ? wsum[k] : 0u;
    C += wsum[k];
  }
  __syncthreads();  // (wsum is reused below)
  for (uint32_t i = i0; i < i1; i++) {
    const uint32_t v = pre[i];
    pre[i] = run;
    run += v;
  }
  if (tid == 0) pre[nblk] = C;
  __syncthreads();
  const uint32_t own0 = pre[b0 - bx], own1 = pre[b1 - bx];  // the own candidates
  CHAIN_STAMP(1);
  if (C > kChainCands) {
    fail = true;  // (a denser group than planned for: not proved here)
    C = 0;
  }
  // candidate -> its loaded block (thread t writes block t's run of indices)
  for (uint32_t i = tid; i < nblk && C; i += kChainThreads)
    for (uint32_t j = pre[i]; j < pre[i + 1]; j++) cblk[j] = (uint16_t)i;
  __syncthreads();
  // candidates -> LDS (candidate j = u 1024 + tid; every round's addresses first, then the
  // loads side by side)
  uint32_t pos[kChainPer], len[kChainPer];
  {
    size_t at[kChainPer];
    uint32_t blk[kChainPer];
#pragma unroll
    for (uint32_t u = 0; u < kChainPer; u++) {
      const uint32_t j = min(u * kChainThreads + tid, C ? C - 1u : 0u);
      blk[u] = C ? cblk[j] : 0u;
      at[u] = (size_t)(bx + blk[u]) * kScanSlots + (j - pre[blk[u]]);
    }
    uint32_t sl[kChainPer];
#pragma unroll
    for (uint32_t u = 0; u < kChainPer; u++) sl[u] = C ? slots[at[u]] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < kChainPer; u++) {
      const uint32_t j = u * kChainThreads + tid;
      pos[u] = blk[u] * kScanBlockBytes + (sl[u] & kSlotOff);
      len[u] = sl[u] >> 16;
      if (j < C) {
        cpos[j] = pos[u] | ((sl[u] & kSlotCopy) ? 0x80000000u : 0u);
        clen[j] = (uint16_t)len[u];
      }
      if (j >= C || (sl[u] & kSlotCopy)) len[u] = 0u;  // (a copy marks nothing)
    }
  }
  __syncthreads();
  // the index of loaded position q (relative), or kNone: its block's run of candidates, the
  // first 8 compared side by side, a binary search past them
  auto find = [&](uint32_t q) -> uint32_t {
    const uint32_t qb = q / kScanBlockBytes;
    if (qb >= nblk) return kNone;
    const uint32_t lo = pre[qb], hi = pre[qb + 1];
    uint32_t hit = kNone;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
      const uint32_t i = min(lo + k, kChainCands - 1u);
      if (lo + k < hi && (cpos[i] & 0x7FFFFFFFu) == q) hit = lo + k;
    }
    if (hit == kNone && hi - lo > 8u) {
      uint32_t a = lo + 8, b = hi;
      while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        if ((cpos[mid] & 0x7FFFFFFFu) < q) a = mid + 1; else b = mid;
      }
      if (a < hi && (cpos[a] & 0x7FFFFFFFu) == q) hit = a;
    }
    return hit;
  };
  // 2. marks: the successor among the loaded candidates
  uint32_t tgt[kChainPer];
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) tgt[u] = len[u] ? find(pos[u] + len[u]) : kNone;
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) {
    if (tgt[u] == kNone) continue;
    const uint32_t me = u * kChainThreads + tid + 1u;
    const uint32_t prev = atomicCAS(&cmark[tgt[u]], 0u, me);
    if (prev != 0u && prev != me) cmark[tgt[u]] = kMarkMulti;
  }
  __syncthreads();
  CHAIN_STAMP(2);
  // 3. the H members among the own candidates, in order (rank of candidate u 1024 + tid: the
  // members of the rounds before u, of the waves before, of the lanes before)
  uint32_t m[kChainPer], kp[kChainPer], km[kChainPer];
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) m[u] = cmark[u * kChainThreads + tid];
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) {  // the marker: at 0, or marked itself
    const uint32_t k = m[u] != 0u && m[u] != kMarkMulti ? m[u] - 1u : 0u;
    kp[u] = cpos[k];
    km[u] = cmark[k];
  }
  uint64_t bal[kChainPer];
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) {
    const uint32_t j = u * kChainThreads + tid;
    bool h = false;
    if (j >= own0 && j < own1)
      h = base_pos + pos[u] == 0 || m[u] == kMarkMulti ||
          (m[u] != 0u && (base_pos + (kp[u] & 0x7FFFFFFFu) == 0 || km[u] != 0u));
    bal[u] = __ballot(h);
    if (lane == 0) wsum4[u][wv] = (uint32_t)__popcll(bal[u]);
  }
  __syncthreads();
  uint32_t nh = 0;
#pragma unroll
  for (uint32_t u = 0; u < kChainPer; u++) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < kW; k++) {
      before += k < wv ? wsum4[u][k] : 0u;
      all += wsum4[u][k];
    }
    if ((bal[u] >> lane) & 1u)
      hlist[nh + before +
            __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[u] >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bal[u], 0u))] =
          (uint16_t)(u * kChainThreads + tid);
    nh += all;
  }
  __syncthreads();
  const uint32_t nl = nh;
  auto hpos = [&](uint32_t i) { return base_pos + (cpos[hlist[i]] & 0x7FFFFFFFu); };
  CHAIN_STAMP(3);
  // 4. this group's first rank: aggregate out, decoupled look-back (wave 0), inclusive out;
  // meanwhile wave 1 asks whether the last member's successor is a candidate (it lies in the
  // loaded blocks; that only matters for the last nonempty group: there it must not be)
  if (wv == 1 && lane == 0 && nl) {
    const uint64_t q = hpos(nl - 1) + clen[hlist[nl - 1]];  // in the loaded blocks, or past the end
    sh[1] = q < nbytes && find((uint32_t)(q - base_pos)) != kNone ? 1u : 0u;
  }
  if (wv == 0) {
    if (lane == 0)
      __hip_atomic_store(&status[g], chain_word(epoch, g == 0 ? 2u : 1u, nh), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t acc = 0;
    bool gave_up = false;
    for (int64_t top = (int64_t)g - 1; top >= 0 && !gave_up; top -= 64) {
      const int64_t q = top - (int64_t)lane;
      uint64_t w = 0;
      if (q >= 0) {
        uint32_t polls = 0;
        do {
          w = ld_agent(&status[q]);
        } while ((uint32_t)(w >> 40) != epoch && ++polls < kChainSpin);
      }
      const bool here = q < 0 || (uint32_t)(w >> 40) == epoch;
      gave_up = __ballot(!here) != 0;
      const uint32_t kind = q >= 0 ? (uint32_t)(w >> 38) & 3u : 2u;
      const uint64_t v = q >= 0 && here ? (w & ((1ull << 38) - 1)) : 0ull;
      const uint64_t done = __ballot(kind == 2u);  // lanes holding an inclusive word
      const uint32_t stop = done ? (uint32_t)__ffsll((long long)done) - 1u : 64u;
      uint64_t mine = lane <= stop ? v : 0ull;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mine += __shfl_xor(mine, o);
      acc += mine;
      if (done) break;
    }
    if (lane == 0) {
      if (g != 0 && !gave_up)
        __hip_atomic_store(&status[g], chain_word(epoch, 2u, acc + nh), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (gave_up) sh[0] = 1u;
      s_prefix = acc;
    }
  }
  __syncthreads();
  CHAIN_STAMP(4);
  const uint64_t rank0 = s_prefix;
  // H out in order; each member's successor must be the next member
  for (uint32_t i = tid; i < nl; i += kChainThreads) {
    const uint64_t r = rank0 + i;
    const uint64_t q = hpos(i);
    const uint32_t L = clen[hlist[i]];
    if (r < cap) {
      rec_off[r] = q;
      rec_len[r] = L;
    }
    if (i + 1 < nl && q + L != hpos(i + 1)) fail = true;
  }
  if (__ballot(fail) && lane == 0) atomicOr(&sh[0], 1u);
  __syncthreads();
  if (tid == 0) {  // 5. the summary to host memory: one 16-byte write-through store (the host
    // reads it while the kernel may still run; the barrier above waited for the record stores)
    const uint64_t first = nl ? hpos(0) : 0ull;
    const uint64_t span = nl ? hpos(nl - 1) + clen[hlist[nl - 1]] - first : 0ull;
    const unsigned __int128 v =
        (unsigned __int128)(first & ((1ull << 40) - 1)) |
        ((unsigned __int128)(span & ((1ull << 26) - 1)) << 40) |
        ((unsigned __int128)min(nh, 8191u) << 66) |
        ((unsigned __int128)min(own1 - own0, 8191u) << 79) |
        ((unsigned __int128)(sh[0] != 0u) << 92) | ((unsigned __int128)(sh[1] != 0u) << 93) |
        ((unsigned __int128)epoch << 94);
    const u32x4_t w = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96)};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(host_aux + g), "v"(w)
                 : "memory");  // (system coherent: one write to host memory)
  }
  CHAIN_STAMP(5);
}

// the candidate total / overflow word (exclusive scan's last entry) to host-mapped memory
__global__ void scan_total_kernel(const uint64_t* __restrict__ last, uint64_t* __restrict__ host) {
  *host = *last;
}

// exclusive scan of the block counts in one workgroup, for up to kScanSmall blocks (a 1 GiB
// stream is 32768 detect blocks): the low words go through LDS -- coalesced loads in,
// thread t then owns the K = ceil(nb / 1024) consecutive entries [t K, t K + K) (one
// sequential pass, one lane-shift scan of the thread totals per wave, one barrier for the
// wave totals), writes their prefixes back in place, and the prefixes leave in coalesced
// rows.  LDS index i sits at i + i / 32, so the K-strided accesses of a wave fall on
// distinct banks.  (Rows of 64 per wave with a lane-shift scan per row took 23 us for
// 32768 blocks; reading the K entries straight from global memory, 57 us.)  base[nb] and the
// host-mapped total word (candidates | overflowing blocks << 32) come from thread 0.
constexpr uint32_t kScanSmall = 36864;  // 1.125 GiB of 32-KiB blocks (a 1-GiB shard + its halo)
constexpr uint32_t kOffLds = (kScanSmall + kScanSmall / 32) * 4;
__device__ __forceinline__ uint32_t off_pad(uint32_t i) { return i + (i >> 5); }
__global__ void __launch_bounds__(1024)
scan_offsets_kernel(const uint64_t* __restrict__ counts, uint32_t nb, uint64_t* __restrict__ base,
                    uint64_t* __restrict__ host) {
  extern __shared__ uint32_t sv[];
  __shared__ uint32_t wsum[16], wovf[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  uint32_t ovf = 0;
  constexpr uint32_t kU = 8;  // coalesced rows of 1024 in flight per pass
  for (uint32_t r0 = 0; r0 < nb; r0 += kU * 1024u) {
    uint64_t c[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) c[u] = counts[min(r0 + u * 1024u + t, nb - 1u)];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t i = r0 + u * 1024u + t;
      if (i < nb) {
        sv[off_pad(i)] = (uint32_t)c[u];
        ovf += (uint32_t)(c[u] >> 32);
      }
    }
  }
  __syncthreads();
  const uint32_t K = (nb + 1023u) / 1024u;
  const uint32_t i0 = min(t * K, nb), i1 = min(i0 + K, nb);
  uint32_t tot = 0;
  for (uint32_t i = i0; i < i1; i++) tot += sv[off_pad(i)];
  uint32_t incl = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += o;
  }
  uint32_t wo = ovf;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) wo += (uint32_t)__shfl_xor((int)wo, d);
  if (lane == 63u) wsum[wv] = incl;
  if (lane == 0u) wovf[wv] = wo;
  __syncthreads();
  uint32_t run = incl - tot, total = 0, novf = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) {
    run += k < wv ? wsum[k] : 0u;
    total += wsum[k];
    novf += wovf[k];
  }
  for (uint32_t i = i0; i < i1; i++) {
    const uint32_t v = sv[off_pad(i)];
    sv[off_pad(i)] = run;
    run += v;
  }
  __syncthreads();
  for (uint32_t i = t; i < nb; i += 1024u) base[i] = sv[off_pad(i)];
  if (t == 0) {
    base[nb] = total;
    *host = (uint64_t)total | ((uint64_t)novf << 32);
  }
}

__device__ uint32_t find_cand(const uint64_t* cand, uint32_t n, uint64_t p) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cand[mid] < p) lo = mid + 1; else hi = mid;
  }
  return (lo < n && cand[lo] == p) ? lo : kNone;
}

// 3. one lifting level (base 4): up_k = up_{k-1}^4, dist_k = the 4 partial distances
// (a terminal points at itself with distance 0, so both saturate there).  The 2- and 3-jump
// tables of level k-1 (up2 / up3, d2 / d3) fall out of the same gathers: with them a walk
// takes one jump per level (enumeration, chain_descend) instead of up to three.
__global__ void __launch_bounds__(256)
scan_lift_kernel(const uint32_t* __restrict__ up0, const uint32_t* __restrict__ d0,
                 uint32_t* __restrict__ up1, uint32_t* __restrict__ d1,
                 uint32_t* __restrict__ up2, uint32_t* __restrict__ up3,
                 uint32_t* __restrict__ d2, uint32_t* __restrict__ d3, uint32_t n,
                 const uint64_t* __restrict__ spec_total, const uint32_t* __restrict__ regular) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  if (regular && *regular) return;  // the regular chain needs no lifting
  // speculative build: n is the capacity and the candidate count is on the device; its
  // load goes out beside the first gather (up0 has `n` readable entries either way)
  const uint64_t t = spec_total ? *spec_total : 0ull;
  const uint32_t u1 = up0[c];
  const uint32_t dc = d0[c];
  if (spec_total && (t > n || c >= (uint32_t)t)) return;
  const uint32_t u2 = up0[u1];
  const uint32_t e1 = d0[u1];
  const uint32_t u3 = up0[u2];
  const uint32_t e2 = d0[u2];
  const uint32_t u4 = up0[u3];
  const uint32_t e3 = d0[u3];
  up1[c] = u4;
  d1[c] = dc + e1 + e2 + e3;
  up2[c] = u2;
  up3[c] = u3;
  d2[c] = dc + e1;
  d3[c] = dc + e1 + e2;
}

// the last chain node from candidate c whose position is < limit (pos(c) < limit), and the
// number of records from c to it: greedy descent over the lifting levels -- at each level the
// furthest of 1, 2, 3 jumps that stays below the limit (positions grow along the chain and a
// terminal repeats itself with distance 0), the three candidates loaded side by side
__device__ __forceinline__ uint32_t chain_descend(const uint64_t* __restrict__ cand,
                                                  const LiftTabs& t, uint32_t c, uint64_t limit,
                                                  uint64_t& count) {
  uint32_t node = c;
  uint64_t cnt = 1;
  for (int k = t.levels - 1; k >= 0; k--) {
    const size_t o = (size_t)k * t.stride + node;
    const uint32_t n1 = t.ups[o], n2 = t.ups2[o], n3 = t.ups3[o];
    const uint32_t e1 = t.dists[o], e2 = t.dists2[o], e3 = t.dists3[o];
    const uint64_t p1 = cand[n1], p2 = cand[n2], p3 = cand[n3];
    if (p3 < limit) { node = n3; cnt += e3; }
    else if (p2 < limit) { node = n2; cnt += e2; }
    else if (p1 < limit) { node = n1; cnt += e1; }
  }
  count = cnt;
  return node;
}

// enumerate the chain from candidate `start` up to (excluding) position `limit`: record i
// (i <= dtop[start]) is `start` lifted by the base-4 digits of i; positions grow along the
// chain, so the records below the limit are a prefix.  With at_zero, only if that candidate
// sits at offset 0 (else nothing is written and end->count = 0).  Thread 0 reports where the
// enumeration stops.
__global__ void __launch_bounds__(256)
scan_enum_kernel(const uint8_t* __restrict__ s, const uint64_t* __restrict__ cand,
                 LiftTabs t, const uint64_t* __restrict__ spec_total,
                 uint32_t start, int at_zero, uint64_t limit, uint64_t out_base,
                 uint64_t cap, uint64_t* __restrict__ rec_off, uint32_t* __restrict__ rec_len,
                 ChainEnd* __restrict__ end, const uint32_t* __restrict__ regular) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // after scan_enum_regular_kernel: nothing to do when it found the regular chain
  if (regular && *regular) return;
  // speculative build: tables of `stride` entries, valid only when the total fits them
  const bool built = !spec_total || (*spec_total != 0 && *spec_total <= t.stride);
  const bool ok = built && !(at_zero && cand[start] != 0);
  if (i == 0) {
    uint64_t cnt = 0, nx = 0, more = 0;
    if (ok) {
      const uint32_t last = chain_descend(cand, t, start, limit, cnt);
      const uint64_t tp = cand[last];
      nx = tp + be16_at(s, tp);
      more = t.dists[last] != 0u;
    }
    end->count = cnt;
    end->next_pos = nx;
    end->more = more;
  }
  if (!ok || i > t.dists[(size_t)t.levels * t.stride + start] || out_base + i >= cap) return;
  uint32_t node = start;
  for (int k = 0; k < t.levels; k++) {  // one jump per non-zero base-4 digit of i
    const uint32_t d = (uint32_t)(i >> (2 * k)) & 3u;
    const uint32_t* tab = d == 1 ? t.ups : d == 2 ? t.ups2 : t.ups3;
    if (d) node = tab[(size_t)k * t.stride + node];
  }
  const uint64_t p = cand[node];
  if (p >= limit) return;
  rec_off[out_base + i] = p;
  rec_len[out_base + i] = be16_at(s, p);
}

// exits of the shard protocol: for each candidate c below `window` (the first ones: cand is
// sorted), the position where its chain first reaches >= limit; bit 63 set when the chain
// leaves the candidate set before (the exit then needs the sequential walk).  Entries past
// the window are ~0.
__global__ void __launch_bounds__(256)
scan_exits_kernel(const uint8_t* __restrict__ s, const uint64_t* __restrict__ cand,
                  LiftTabs t, uint32_t n, uint64_t window, uint64_t limit, uint32_t cap,
                  uint64_t* __restrict__ entries, uint64_t* __restrict__ exits) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cap) return;
  if (c >= n || cand[c] >= window || cand[c] >= limit) {
    entries[c] = ~0ull;
    exits[c] = ~0ull;
    return;
  }
  uint64_t cnt;
  const uint64_t tp = cand[chain_descend(cand, t, c, limit, cnt)];
  const uint64_t nx = tp + be16_at(s, tp);
  entries[c] = cand[c];
  exits[c] = nx | (nx < limit ? (1ull << 63) : 0ull);
}

// 4. sequential resolver (one thread): the reference rule from position p until the chain
// re-enters the candidate set, ends, errors, or max_steps records were emitted.
struct ResolveState {
  uint64_t pos;        // in: start position; out: where it stopped
  uint64_t emitted;    // out: records written
  uint32_t next_cand;  // out: candidate index at `pos` (kNone if none)
  int32_t reason;      // out: 0 = candidate reached, 1 = end of stream, 2 = TCP error, 3 = steps,
                       //      4 = position >= limit
};

__global__ void scan_resolve_kernel(const uint8_t* __restrict__ s, uint64_t nbytes, uint64_t limit,
                                    int sink,
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
    if (p >= limit) { reason = 4; break; }
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
  mgenx::dev_free(w.mem);
  w.mem = nullptr;
  w.bytes = 0;
  hipError_t e = hipMalloc(&w.mem, need);
  if (e == hipSuccess) w.bytes = need;
  return e;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// The workspace lives with the context (grown on demand, freed by mgenx_ctx_destroy via
// mgenx_scan_ws_free).  It also keeps the candidate tables of the last stream built, which
// mgenx_stream_scan_range may reuse on request.
struct mgenx_scan_ws {
  ScanWork slots, cands, tabs, small;
  // host-mapped (fine-grained) words the kernels write their results to: [0] candidate
  // total, [2..3] chain end -- no copy operations on the common path
  uint64_t* host = nullptr;
  uint64_t* host_dev = nullptr;
  // tables of the last build
  const uint8_t* key_s = nullptr;
  uint64_t key_n = 0;
  int key_mode = -1;
  uint32_t n = 0;      // candidates (0: resolver only -- none, or a pathologically dense stream)
  int levels = 0;      // lifting levels: ups / dists hold levels + 1 tables of `stride`
  uint32_t stride = 0; // table stride (n, or the capacity of a speculative build)
  uint64_t* cand = nullptr;
  uint32_t* ups = nullptr;
  uint32_t* dists = nullptr;
  uint32_t* ups2 = nullptr;   // [levels][stride] 2- and 3-jump tables
  uint32_t* ups3 = nullptr;
  uint32_t* dists2 = nullptr;
  uint32_t* dists3 = nullptr;
  uint64_t last_records = 0;  // the last whole-stream chain's record count (spec levels)
  // speculative builds: the next whole-stream scan sizes its tables by spec_cap (from the
  // last exact build) and runs detect -> link -> lifting -> enumeration without waiting for
  // the candidate total; spec_total is that total on the device, spec_pending says the
  // current tables are speculative (the host checks the total after the one sync)
  uint32_t spec_cap = 0;
  const uint64_t* spec_total = nullptr;
  bool spec_pending = false;
  // the chain hypothesis (scan_chain_*) in whole-stream TCP scans once an exact build has
  // sized spec_cap.  After a stream where it was not the chain the next prune_skip scans do not
  // try it (backoff 2, 4, ... 64 scans; reset on success)
  uint32_t prune_skip = 0, prune_backoff = 0;
  ScanWork chain;        // the chain kernel's look-back words
  uint32_t chain_epoch = 0;
  ChainAux* chain_host = nullptr;      // [kChainGroups] group summaries (host-mapped)
  ChainAux* chain_host_dev = nullptr;
  std::vector<ChainAux> chain_seen;    // the summaries as read
};

extern "C" void* mgenx_scan_ws_new() { return new mgenx_scan_ws(); }
extern "C" void mgenx_scan_ws_free(void* p) {
  mgenx_scan_ws* w = static_cast<mgenx_scan_ws*>(p);
  if (!w) return;
  for (ScanWork* x : {&w->slots, &w->cands, &w->tabs, &w->small, &w->chain})
    mgenx::dev_free(x->mem);
  mgenx::host_free(w->host);
  mgenx::host_free(w->chain_host);
  delete w;
}

namespace {

struct Fail {
  char* err;
  size_t errn;
  int operator()(hipError_t e, const char* what) const {
    snprintf(err, errn, "%s: %s", what, hipGetErrorString(e));
    return MGENX_EDEVICE;
  }
};

// detect -> device scan of the block counts -> (one copy back: the candidate total) ->
// compact + link -> lifting levels.  Leaves the tables in ws (async after the copy).
int levels_for(uint64_t n) {
  int levels = 1;
  while ((1ull << (2 * levels)) < n) levels++;  // 4^levels >= n > any chain length
  return levels;
}

// bytes of the lifting tables for `stride` candidates and `levels` levels
size_t tab_bytes(uint32_t stride, int levels) {
  return (size_t)stride * 4 * (2 * (size_t)(levels + 1) + 4 * (size_t)levels);
}

// the small device area and the host-mapped result words
int ensure_small(mgenx_scan_ws& ws, const Fail& fail) {
  hipError_t e;
  if ((e = ensure(ws.small, 4096)) != hipSuccess) return fail(e, "scan workspace");
  if (!ws.host) {
    void* hp = nullptr;
    if ((e = hipHostMalloc(&hp, 64, hipHostMallocMapped)) != hipSuccess)
      return fail(e, "scan workspace");
    ws.host = static_cast<uint64_t*>(hp);
    void* dp = nullptr;
    if ((e = hipHostGetDevicePointer(&dp, hp, 0)) != hipSuccess) return fail(e, "scan workspace");
    ws.host_dev = static_cast<uint64_t*>(dp);
  }
  return MGENX_OK;
}

uint32_t link_grid(uint32_t nb) { return (nb + 4 * kLinkPerWave - 1) / (4 * kLinkPerWave); }

// carve ws.tabs into the lifting tables; launch the link and the lifting levels
void lay_tables(mgenx_scan_ws& ws, uint32_t stride, int levels) {
  ws.stride = stride;
  ws.levels = levels;
  ws.cand = static_cast<uint64_t*>(ws.cands.mem);
  ws.ups = static_cast<uint32_t*>(ws.tabs.mem);
  ws.dists = ws.ups + (size_t)(levels + 1) * stride;
  ws.ups2 = ws.dists + (size_t)(levels + 1) * stride;
  ws.ups3 = ws.ups2 + (size_t)levels * stride;
  ws.dists2 = ws.ups3 + (size_t)levels * stride;
  ws.dists3 = ws.dists2 + (size_t)levels * stride;
}

LiftTabs lift_tabs(const mgenx_scan_ws& ws) {
  LiftTabs t;
  t.ups = ws.ups; t.dists = ws.dists; t.ups2 = ws.ups2; t.ups3 = ws.ups3;
  t.dists2 = ws.dists2; t.dists3 = ws.dists3; t.stride = ws.stride; t.levels = ws.levels;
  return t;
}

void launch_lifts(const mgenx_scan_ws& ws, const uint64_t* spec_total, hipStream_t stream,
                  const uint32_t* regular = nullptr) {
  const uint32_t st = ws.stride;
  const dim3 g((st + 255) / 256);
  for (int k = 1; k <= ws.levels; k++) {
    const size_t a = (size_t)(k - 1) * st, b = (size_t)k * st;
    hipLaunchKernelGGL(scan_lift_kernel, g, dim3(256), 0, stream, ws.ups + a, ws.dists + a,
                       ws.ups + b, ws.dists + b, ws.ups2 + a, ws.ups3 + a, ws.dists2 + a,
                       ws.dists3 + a, st, spec_total, regular);
  }
}

int scan_build(mgenx_scan_ws& ws, const uint8_t* s, uint64_t nbytes, int mode, hipStream_t stream,
               const Fail& fail, bool spec = false) {
  const bool sink = mode == MGENX_SCAN_SINK;
  const ScanMode m = sink ? ScanMode{MGENX_MIN_SIZE, MGENX_MAX_SIZE} : ScanMode{4u, 65535u};
  hipError_t e;
  ws.key_s = nullptr;
  ws.n = 0;
  ws.levels = 0;
  ws.cand = nullptr;
  ws.ups = ws.dists = nullptr;
  ws.stride = 0;
  ws.spec_pending = false;
  ws.spec_total = nullptr;
  if (int rc = ensure_small(ws, fail)) return rc;
  const uint64_t n_blocks64 = (nbytes + kScanBlockBytes - 1) / kScanBlockBytes;
  if (n_blocks64 == 0 || n_blocks64 > 0xFFFFFFull) {  // nothing to index: resolver only
    ws.key_s = s;
    ws.key_n = nbytes;
    ws.key_mode = mode;
    return MGENX_OK;
  }
  const uint32_t nb = (uint32_t)n_blocks64;
  const size_t slot_b = align256((size_t)nb * kScanSlots * 4);
  const size_t cnt_b = align256((size_t)(nb + 1) * 8);
  size_t cub_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, (const uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)(nb + 1), stream);
  if ((e = ensure(ws.slots, slot_b + 2 * cnt_b + align256(cub_bytes))) != hipSuccess)
    return fail(e, "scan workspace");
  uint32_t* d_slots = static_cast<uint32_t*>(ws.slots.mem);
  uint64_t* d_counts = reinterpret_cast<uint64_t*>(static_cast<char*>(ws.slots.mem) + slot_b);
  uint64_t* d_base = d_counts + cnt_b / 8;
  void* d_cub = static_cast<char*>(ws.slots.mem) + slot_b + 2 * cnt_b;
  uint32_t* irregular = reinterpret_cast<uint32_t*>(static_cast<char*>(ws.small.mem) + 2048);
  auto detect = scan_detect_kernel<false>;
#if MGENX_DIAG
  if (const char* v = getenv("MGENX_SCAN_PLAIN"))
    if (atoi(v)) detect = scan_detect_kernel<false, true>;
#endif
  hipLaunchKernelGGL(detect, dim3(nb), dim3(kScanThreads), 0, stream, s,
                     nbytes, m, d_slots, d_counts, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                     spec && ws.spec_cap ? irregular : (uint32_t*)nullptr);
  if (nb <= kScanSmall) {
    if ((e = set_max_lds((const void*)scan_offsets_kernel, (int)kOffLds)) != hipSuccess)
      return fail(e, "scan offsets");
    hipLaunchKernelGGL(scan_offsets_kernel, dim3(1), dim3(1024), kOffLds, stream, d_counts, nb,
                       d_base, ws.host_dev);
  } else {
    if ((e = hipcub::DeviceScan::ExclusiveSum(d_cub, cub_bytes, (const uint64_t*)d_counts, d_base,
                                              (int)(nb + 1), stream)) != hipSuccess)
      return fail(e, "scan offsets");
    hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, stream, d_base + nb, ws.host_dev);
  }
  if (spec && ws.spec_cap) {
    // speculative: tables for spec_cap candidates, linked and lifted with the total read on
    // the device; the caller enumerates and then checks the total (one sync for the scan)
    const uint32_t cap = ws.spec_cap;
    // levels for the last chain's length (a longer chain costs another enumeration round
    // in scan_walk, not correctness)
    const uint64_t want = ws.last_records ? ws.last_records : cap;  // 4^levels + 1 records
    const int levels = levels_for(std::min<uint64_t>(want, cap));
    if ((e = ensure(ws.cands, (size_t)cap * 8)) != hipSuccess ||
        (e = ensure(ws.tabs, tab_bytes(cap, levels))) != hipSuccess)
      return fail(e, "scan workspace");
    ws.key_s = s;
    ws.key_n = nbytes;
    ws.key_mode = mode;
    lay_tables(ws, cap, levels);
    ws.spec_total = d_base + nb;
    ws.spec_pending = true;
    hipLaunchKernelGGL(scan_link_kernel, dim3(link_grid(nb)), dim3(256), 0, stream, s, nbytes,
                       d_slots, d_counts, d_base, nb, ws.cand, ws.ups, ws.dists, (uint64_t)cap,
                       irregular);
    // (the lifting levels follow only when the chain is not the candidate list itself:
    // mgenx_scan_run, after its one sync)
    if ((e = hipGetLastError()) != hipSuccess) return fail(e, "scan launch");
    return MGENX_OK;
  }
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan detect");
  struct {
    uint32_t total, overflowed;  // candidates, overflowing blocks
  } h_tot;
  memcpy(&h_tot, (const void*)ws.host, 8);
  ws.key_s = s;
  ws.key_n = nbytes;
  ws.key_mode = mode;
  // candidate budget: a stream denser than one plausible start per 16 bytes is left to
  // the sequential resolver (no valid MGEN stream comes near it: records are >= 28 B)
  const uint64_t max_cand = nbytes / 16 + 65536;
  if (h_tot.total == 0 || h_tot.total > max_cand) return MGENX_OK;  // resolver only
  const uint32_t n = h_tot.total;
  const int levels = levels_for(n);
  // the next whole-stream scan speculates on about this many candidates
  ws.spec_cap = (uint32_t)std::min<uint64_t>((uint64_t)n + n / 8 + 1024, 0xFFFFFFF0u);
  if ((e = ensure(ws.cands, (size_t)n * 8)) != hipSuccess) return fail(e, "scan workspace");
  if ((e = ensure(ws.tabs, tab_bytes(n, levels))) != hipSuccess)
    return fail(e, "scan workspace");
  ws.n = n;
  lay_tables(ws, n, levels);
  if (h_tot.overflowed)  // blocks with more candidates than slots: second pass, exact sizes
    hipLaunchKernelGGL(scan_detect_kernel<true>, dim3(nb), dim3(kScanThreads), 0, stream, s,
                       nbytes, m, d_slots, d_counts, (const uint64_t*)d_base, ws.cand,
                       (uint32_t*)nullptr);
  hipLaunchKernelGGL(scan_link_kernel, dim3(link_grid(nb)), dim3(256), 0, stream, s, nbytes,
                     d_slots, d_counts, d_base, nb, ws.cand, ws.ups, ws.dists, (uint64_t)0,
                     (uint32_t*)nullptr);
  launch_lifts(ws, nullptr, stream);
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "scan launch");
  return MGENX_OK;
}

// the chain from `entry` over positions < limit, on the tables of ws.  The common case
// (entry is candidate 0 at offset 0, or any candidate: at_zero) is one enumeration and one
// copy back; positions off the candidate set go through the sequential resolver.
int scan_walk(mgenx_scan_ws& ws, const uint8_t* s, uint64_t nbytes, int mode, uint64_t entry,
              uint64_t limit, uint64_t* rec_off, uint32_t* rec_len, uint64_t cap,
              mgenx_scan_info* info, hipStream_t stream, const Fail& fail,
              const ChainEnd* first = nullptr) {
  const bool sink = mode == MGENX_SCAN_SINK;
  const uint32_t n = ws.n;
  const LiftTabs tabs = lift_tabs(ws);
  hipError_t e;
  mgenx_scan_info out;
  memset(&out, 0, sizeof(out));
  ResolveState* d_st = reinterpret_cast<ResolveState*>(ws.small.mem);
  ChainEnd* d_end = reinterpret_cast<ChainEnd*>(ws.host_dev + 2);
  const volatile uint64_t* h_end = ws.host + 2;
  uint64_t pos = entry, total = 0;
  uint32_t at = kNone;  // candidate index at pos, when known
  bool done = false;
  int reason = 1;
  if (first) {  // the speculative scan's enumeration from offset 0, already done
    if (first->count) {
      total = first->count;
      pos = first->next_pos;
      if (pos >= limit) { reason = 4; done = true; }
      else if (pos + 2 > nbytes) { reason = 1; done = true; }
    }
  } else if (n && entry == 0 && entry < limit) {
    // candidate 0 is offset 0 when offset 0 is a candidate: enumerate speculatively
    hipLaunchKernelGGL(scan_enum_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, s, ws.cand,
                       tabs, (const uint64_t*)nullptr, 0u, 1, limit, (uint64_t)0, cap, rec_off,
                       rec_len, d_end, (const uint32_t*)nullptr);
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan");
    const ChainEnd h = {h_end[0], h_end[1], h_end[2]};
    if (h.count) {
      total = h.count;
      pos = h.next_pos;
      if (pos >= limit) { reason = 4; done = true; }
      else if (pos + 2 > nbytes) { reason = 1; done = true; }
    }
  }
  for (int rounds = 0; !done && rounds < (1 << 30); rounds++) {
    if (at != kNone) {
      // enumerate the candidate chain from `at` (grid sized by n >= its length)
      hipLaunchKernelGGL(scan_enum_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, s,
                         ws.cand, tabs, (const uint64_t*)nullptr, at, 0, limit, total, cap,
                         rec_off, rec_len, d_end, (const uint32_t*)nullptr);
      if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan");
      const ChainEnd h = {h_end[0], h_end[1], h_end[2]};
      total += h.count;
      pos = h.next_pos;
      at = kNone;
      if (pos >= limit) { reason = 4; break; }
      if (pos + 2 > nbytes) { reason = 1; break; }
    }
    // resolver from pos (pos is not a candidate, or is the entry itself)
    ResolveState st;
    st.pos = pos;
    st.emitted = 0;
    st.next_cand = kNone;
    st.reason = 3;
    if ((e = hipMemcpyAsync(d_st, &st, sizeof(st), hipMemcpyHostToDevice, stream)) != hipSuccess)
      return fail(e, "scan");
    hipLaunchKernelGGL(scan_resolve_kernel, dim3(1), dim3(1), 0, stream, s, nbytes, limit,
                       (int)sink, ws.cand, n, total, cap, (uint64_t)1 << 20, rec_off, rec_len, d_st);
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
  out.n_records = total;
  if (entry == 0 && limit == nbytes) ws.last_records = total;
  out.consumed = pos;
  out.status = reason == 2 ? 1 : 0;
  out.candidates = n;
  if (info) *info = out;
  return MGENX_OK;
}


// The chain hypothesis (scan_chain_kernel) on a whole TCP stream: detect and one kernel, one
// sync.  ok = false: H was not the chain (nothing is left to reuse; the
// caller builds exactly).  Groups: enough that each holds about 2048 candidates of the last
// exact build (spec_cap; kChainCands is twice that) and at most kChainBlocks detect blocks.
bool chain_fits(const mgenx_scan_ws& ws, uint64_t nbytes) {
  const uint64_t nb = (nbytes + kScanBlockBytes - 1) / kScanBlockBytes;
  return ws.spec_cap != 0 && nb != 0 && nb <= (uint64_t)kChainGroups * kChainBlocks &&
         nbytes < (1ull << 40);
}

int scan_chain(mgenx_scan_ws& ws, const uint8_t* s, uint64_t nbytes, uint64_t* rec_off,
               uint32_t* rec_len, uint64_t cap, mgenx_scan_info* info, hipStream_t stream,
               const Fail& fail, bool& ok) {
  ok = false;
  ws.key_s = nullptr;  // no candidate tables on this path
  ws.n = 0;
  ws.levels = 0;
  ws.cand = nullptr;
  ws.ups = ws.dists = nullptr;
  ws.stride = 0;
  ws.spec_pending = false;
  ws.spec_total = nullptr;
  if (int rc = ensure_small(ws, fail)) return rc;
  hipError_t e;
  if (!ws.chain_host) {
    void* hp = nullptr;
    // (the kernel writes it with write-through stores: the host spins on it while the kernel
    // runs; a coherent allocation made each scan ~18 us slower on the host side)
    if ((e = hipHostMalloc(&hp, kChainGroups * sizeof(ChainAux), hipHostMallocMapped)) !=
        hipSuccess)
      return fail(e, "scan workspace");
    ws.chain_host = static_cast<ChainAux*>(hp);
    memset(hp, 0, kChainGroups * sizeof(ChainAux));
    void* dp = nullptr;
    if ((e = hipHostGetDevicePointer(&dp, hp, 0)) != hipSuccess) return fail(e, "scan workspace");
    ws.chain_host_dev = static_cast<ChainAux*>(dp);
  }
  const uint32_t nb = (uint32_t)((nbytes + kScanBlockBytes - 1) / kScanBlockBytes);
  const size_t slot_b = align256((size_t)nb * kScanSlots * 4);
  const size_t cnt_b = align256((size_t)(nb + 1) * 8);
  if ((e = ensure(ws.slots, slot_b + 2 * cnt_b)) != hipSuccess) return fail(e, "scan workspace");
  uint32_t* d_slots = static_cast<uint32_t*>(ws.slots.mem);
  uint64_t* d_counts = reinterpret_cast<uint64_t*>(static_cast<char*>(ws.slots.mem) + slot_b);
  uint32_t groups = std::max<uint32_t>((nb + kChainBlocks - 1) / kChainBlocks,
                                       (ws.spec_cap + 2047) / 2048);
  groups = std::min(std::max(groups, 1u), kChainGroups);
  const uint32_t per_group = (nb + groups - 1) / groups;
  groups = (nb + per_group - 1) / per_group;
  // the look-back words (epoch-tagged: cleared only when the 22-bit epoch wraps)
  if (!ws.chain.mem) {
    if ((e = ensure(ws.chain, (size_t)kChainGroups * 8)) != hipSuccess ||
        (e = hipMemsetAsync(ws.chain.mem, 0, ws.chain.bytes, stream)) != hipSuccess)
      return fail(e, "scan workspace");
    ws.chain_epoch = 0;
  }
  if (++ws.chain_epoch >= kChainEpochs) {
    if ((e = hipMemsetAsync(ws.chain.mem, 0, ws.chain.bytes, stream)) != hipSuccess)
      return fail(e, "scan workspace");
    memset(ws.chain_host, 0, kChainGroups * sizeof(ChainAux));  // (no kernel of ours runs now)
    ws.chain_epoch = 1;
  }
  const ScanMode m{4u, 65535u};
  hipLaunchKernelGGL(scan_detect_kernel<false>, dim3(nb), dim3(kScanThreads), 0, stream, s,
                     nbytes, m, d_slots, d_counts, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                     (uint32_t*)nullptr);
  hipLaunchKernelGGL(scan_chain_kernel, dim3(groups), dim3(kChainThreads), 0, stream,
                     (const uint32_t*)d_slots, (const uint64_t*)d_counts, nbytes, nb, per_group,
                     ws.chain_epoch, static_cast<uint64_t*>(ws.chain.mem), cap, rec_off, rec_len,
                     ws.chain_host_dev);
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "scan launch");
  // done when every group's summary carries this scan's epoch (each group writes it after its
  // records and summary are out): a spin on host memory instead of the stream's completion
  // signal.  After a second without them, the stream sync (a fault is reported there).
  // a summary: one aligned 16-byte load (one granule, as the kernel wrote it)
  auto aux_at = [&](uint32_t g) {
    const __m128i x = _mm_load_si128(reinterpret_cast<const __m128i*>(ws.chain_host + g));
    ChainAux a;
    a.lo = (uint64_t)_mm_cvtsi128_si64(x);
    a.hi = (uint64_t)_mm_extract_epi64(x, 1);
    return a;
  };
  std::vector<ChainAux>& ha = ws.chain_seen;
  ha.resize(groups);
  {
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t g = 0;
    for (uint64_t spins = 0; g < groups;) {
      std::atomic_signal_fence(std::memory_order_seq_cst);  // (a fresh load every poll)
      ha[g] = aux_at(g);
      if (aux_bits(ha[g], 94, 22) == ws.chain_epoch) {
        g++;
        continue;
      }
      _mm_pause();
      if ((++spins & 0xFFFF) == 0 &&
          std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan");
        for (; g < groups; g++) {
          ha[g] = aux_at(g);
          if (aux_bits(ha[g], 94, 22) != ws.chain_epoch) break;
        }
        if (g < groups) {
          snprintf(fail.err, fail.errn, "scan: chain kernel ended without its summaries");
          return MGENX_EDEVICE;
        }
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  // the joins between groups: each nonempty group starts where the previous one's last member
  // ends, the first starts at 0, the last one's successor is not a candidate
  uint64_t th = 0, tc = 0, next = 0;
  bool bad = false, any = false, tail = false;
  for (uint32_t g = 0; g < groups; g++) {
    const ChainAux& a = ha[g];
    const uint32_t nh = aux_bits(a, 66, 13);
    tc += aux_bits(a, 79, 13);
    bad = bad || aux_bits(a, 92, 1) != 0u || nh >= 8191u;
    if (!nh) continue;
    const uint64_t first = a.lo & ((1ull << 40) - 1);
    bad = bad || first != next;  // (next = 0 before the first nonempty group)
    any = true;
    th += nh;
    next = first + aux_bits(a, 40, 26);
    tail = aux_bits(a, 93, 1) != 0u;
  }
  if (bad || !any || tail) return MGENX_OK;
  ok = true;
  const uint64_t cands = tc;
  const ChainEnd h = {th, next, 0};
  // H is the chain from 0; what follows its terminal goes to the sequential resolver
  const int rc = scan_walk(ws, s, nbytes, MGENX_SCAN_TCP, 0, nbytes, rec_off, rec_len, cap, info,
                           stream, fail, &h);
  if (info) {
    info->candidates = (uint32_t)std::min<uint64_t>(cands, 0xFFFFFFFFu);
    info->path = 2;
  }
  return rc;
}

}  // namespace

#if MGENX_DIAG
extern "C" int mgenx_diag_chain_prof(unsigned long long* out) {
  return out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_prof), sizeof(g_chain_prof)) ==
                    hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}
#endif

// Whole-stream scan from offset 0 (synchronous on `stream`).
extern "C" int mgenx_scan_run(void* wsp, const uint8_t* s, uint64_t nbytes, int mode,
                              uint64_t* rec_off, uint32_t* rec_len, uint64_t cap,
                              mgenx_scan_info* info, hipStream_t stream, char* err, size_t errn) {
  mgenx_scan_ws& ws = *static_cast<mgenx_scan_ws*>(wsp);
  const Fail fail{err, errn};
  const bool try_chain = ws.prune_skip == 0;
  if (ws.prune_skip) ws.prune_skip--;
  int rc;
  if (try_chain && mode != MGENX_SCAN_SINK && chain_fits(ws, nbytes)) {
    bool ok = false;
    rc = scan_chain(ws, s, nbytes, rec_off, rec_len, cap, info, stream, fail, ok);
    if (rc != MGENX_OK || ok) {
      if (ok) ws.prune_backoff = 0;
      return rc;
    }
    // the hypothesis is not the chain (or not provably): exact build, and a backoff
    ws.prune_backoff = std::min(std::max(2u * ws.prune_backoff, 2u), 64u);
    ws.prune_skip = ws.prune_backoff;
    rc = scan_build(ws, s, nbytes, mode, stream, fail, false);
    if (rc != MGENX_OK) return rc;
    return scan_walk(ws, s, nbytes, mode, 0, nbytes, rec_off, rec_len, cap, info, stream, fail);
  }
  rc = scan_build(ws, s, nbytes, mode, stream, fail, /*spec=*/true);
  if (rc != MGENX_OK) return rc;
  if (ws.spec_pending) {
    // one sync for the whole scan: the chain from offset 0 enumerated on the speculative
    // tables; then the total and overflow word says whether they held every candidate
    const uint32_t scap = ws.stride;
    ChainEnd* d_end = reinterpret_cast<ChainEnd*>(ws.host_dev + 2);
    const volatile uint64_t* h_end = ws.host + 2;
    const uint32_t* irregular =
        reinterpret_cast<const uint32_t*>(static_cast<char*>(ws.small.mem) + 2048);
    uint32_t* regular = reinterpret_cast<uint32_t*>(static_cast<char*>(ws.small.mem) + 2052);
    hipLaunchKernelGGL(scan_enum_regular_kernel, dim3((scap + 255) / 256), dim3(256), 0, stream,
                       s, ws.cand, ws.spec_total, irregular, scap, cap, rec_off, rec_len, d_end,
                       regular, ws.host_dev + 5);
    // not the regular chain: the lifting levels on the speculative tables, then the
    // enumeration from offset 0 -- launched regardless, each returning at once when the
    // regular kernel already reported the chain.  (Deciding on the host instead costs a
    // second round trip whenever payloads hold plausible record starts -- the TCP transmit
    // stream's repeated 8-KiB buffers each begin with a header -- 0.306 -> 0.323 ms on
    // config 5.)
    launch_lifts(ws, ws.spec_total, stream, regular);
    hipLaunchKernelGGL(scan_enum_kernel, dim3((scap + 255) / 256), dim3(256), 0, stream, s,
                       ws.cand, lift_tabs(ws), ws.spec_total, 0u, 1, nbytes, (uint64_t)0, cap,
                       rec_off, rec_len, d_end, (const uint32_t*)regular);
    hipError_t e;
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return fail(e, "scan");
    uint32_t tot[2];
    memcpy(tot, (const void*)ws.host, 8);  // candidates, overflowing blocks
    const uint64_t max_cand = nbytes / 16 + 65536;
    ws.spec_pending = false;
    const bool regular_chain = ((const volatile uint64_t*)ws.host)[5] != 0;
    // the regular chain skipped the lifting: these tables are not for mgenx_scan_range reuse
    if (regular_chain) ws.key_s = nullptr;
    if (tot[1] || tot[0] > scap || tot[0] > max_cand) {
      // the tables did not hold the stream: exact build (sizes the next speculation)
      rc = scan_build(ws, s, nbytes, mode, stream, fail, false);
      if (rc != MGENX_OK) return rc;
      return scan_walk(ws, s, nbytes, mode, 0, nbytes, rec_off, rec_len, cap, info, stream, fail);
    }
    ws.n = tot[0];
    if (ws.n) {
      const ChainEnd h = {h_end[0], h_end[1], h_end[2]};
      // a chain as long as the levels reach (the descent covers 4^levels - 1 jumps) may go
      // on: rebuild with levels for n instead of continuing round by round on too few levels
      if (h.count >= (1ull << (2 * ws.levels)) && h.more) {
        rc = scan_build(ws, s, nbytes, mode, stream, fail, false);
        if (rc != MGENX_OK) return rc;
        return scan_walk(ws, s, nbytes, mode, 0, nbytes, rec_off, rec_len, cap, info, stream,
                         fail);
      }
      rc = scan_walk(ws, s, nbytes, mode, 0, nbytes, rec_off, rec_len, cap, info, stream, fail,
                     &h);
      if (info && regular_chain) info->path = 1;
      return rc;
    }
  }
  return scan_walk(ws, s, nbytes, mode, 0, nbytes, rec_off, rec_len, cap, info, stream, fail);
}

// One shard of a stream split over ranks: builds the tables and reports, for each candidate
// below `window`, where its chain leaves [.., limit).
extern "C" int mgenx_scan_exits_run(void* wsp, const uint8_t* s, uint64_t nbytes, int mode,
                                    uint64_t window, uint64_t limit, uint64_t* entries,
                                    uint64_t* exits, uint32_t cap, uint32_t* candidates,
                                    hipStream_t stream, char* err, size_t errn) {
  mgenx_scan_ws& ws = *static_cast<mgenx_scan_ws*>(wsp);
  const Fail fail{err, errn};
  int rc = scan_build(ws, s, nbytes, mode, stream, fail);
  if (rc != MGENX_OK) return rc;
  if (cap)
    hipLaunchKernelGGL(scan_exits_kernel, dim3((cap + 255) / 256), dim3(256), 0, stream, s,
                       ws.cand, lift_tabs(ws), ws.n, window, limit, cap, entries, exits);
  hipError_t e;
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "scan launch");
  if (candidates) *candidates = ws.n;
  return MGENX_OK;
}

// The records of [entry, limit) (synchronous).  reuse: the tables of the previous build on
// this workspace are for this same stream (pointer, size, mode; the caller vouches that the
// bytes are unchanged).
extern "C" int mgenx_scan_range_run(void* wsp, const uint8_t* s, uint64_t nbytes, int mode,
                                    uint64_t entry, uint64_t limit, int reuse, uint64_t* rec_off,
                                    uint32_t* rec_len, uint64_t cap, mgenx_scan_info* info,
                                    hipStream_t stream, char* err, size_t errn) {
  mgenx_scan_ws& ws = *static_cast<mgenx_scan_ws*>(wsp);
  const Fail fail{err, errn};
  if (reuse) {
    if (ws.key_s != s || ws.key_n != nbytes || ws.key_mode != mode) {
      snprintf(err, errn, "scan range: no tables built for this stream to reuse");
      return MGENX_EINVAL;
    }
  } else {
    int rc = scan_build(ws, s, nbytes, mode, stream, fail);
    if (rc != MGENX_OK) return rc;
  }
  return scan_walk(ws, s, nbytes, mode, entry, limit, rec_off, rec_len, cap, info, stream, fail);
}
