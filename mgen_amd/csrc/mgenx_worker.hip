// mgenx_worker.hip -- the resident single-message worker on gfx950.
//
// An unchanged MGEN build calls MgenMsg::Unpack once per datagram inside its RecvFrom loop,
// MgenMsg::ComputeCRC32 once per checksummed message and MgenAnalytic::Update once per received
// message (src/common/mgenTransport.cpp:948-997, 1011-1063; src/common/mgen.cpp:1027-1070).
// Through the batch entry points each such call is a launch, two copies and a synchronisation.
// Here ONE wave stays on the device and polls a request block the host writes (WReq: in device
// memory the host stores into through the BAR when it may, else in pinned host memory): the
// caller writes the message and a request number, the wave reads the message once (every lane a
// 16-byte part of it, all in flight together), serves it, writes the reply to pinned host
// memory (WRep) with tags; the caller spins on that.  No launch and no copy per call.
//   unpack: MgenMsg::Unpack on a fresh MgenMsg (mgenMsg.cpp:315-500) -- parse_header, the
//           general-layout path of the batch kernels, over an LDS copy of the header bytes;
//   recv:   Unpack, then the receive path's checksum when forced or CHECKSUM is set
//           (mgenTransport.cpp:958-965): ComputeCRC32(0, buf, len - 4) in the same reply;
//   crc32:  MgenMsg::ComputeCRC32 (mgenMsg.cpp:524-541) -- the wave CRC of crc32_kernel
//           (lane partials through the A_4 tables, combined by x^(8n) shifts) over LDS pieces;
//   pack:   MgenMsg::Pack alone, built in LDS;
//   update: MgenAnalytic::Update (mgenAnalytic.cpp:74-258) of one record on a device flow state
//           (FlowSM, the batch kernels' state machine), the report of a closed window back.
// The wave always ends: on a stop request, and after `idle_ticks` of wall clock
// (s_memrealtime, 100 MHz) without a request; the host relaunches it on the next call (the
// request then pending is served first).  Every store to host memory is a vector store.
#include "mgenx_kernels.hpp"
#include "mgenx_parse.hpp"
#include "mgenx_flowsm.hpp"

namespace mgenx {

static_assert(sizeof(mgenx_unpacked) == 88, "mgenx_unpacked is 88 bytes (include/mgenx.h)");
static_assert(sizeof(mgenx_unpacked) <= 88, "the reply's words 0-21");
static_assert(sizeof(mgenx_flow_report) == 96, "the reply's words 24-47");

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_release(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kPiece = 16384;  // bytes of a CRC span staged in LDS at a time

// one 16-byte store that leaves for host memory as one write (system coherent, sc0 sc1): a
// reply chunk and its tag arrive together
__device__ __forceinline__ void st_chunk(uint32_t* p, u32x4_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
// the polled pieces: lane k < 16 reads piece k (one 16-byte load; volatile: every poll reaches
// host memory)
__device__ __forceinline__ u32x4_t poll_pieces(const WReq* m, uint32_t lane) {
  u32x4_t v = {0u, 0u, 0u, 0u};
  if (lane < kPollPieces) v = *reinterpret_cast<const volatile u32x4_t*>(m->poll + 4u * lane);
  return v;
}

// the 16 request-block bytes at p (message offset o), bytes at or past n as zero; the block has
// 64 bytes of slack past its largest message, so the whole 16 are always readable.  Volatile:
// the host wrote them (through the BAR, or to host memory) since any earlier read -- no cache
// may answer (sc0 sc1), so no acquire fence is needed
__device__ __forceinline__ u32x4_t load_masked(const uint8_t* p, uint32_t o, uint32_t n) {
  if (o >= n) return u32x4_t{0u, 0u, 0u, 0u};
  u32x4_t v = *reinterpret_cast<const volatile u32x4_t*>(p);
  if (o + 16u > n) {
    const int k = (int)(n - o);  // 1..15 valid bytes
    v.x &= byte_range_mask(0, k < 4 ? k : 4);
    v.y &= byte_range_mask(0, k < 4 ? 0 : (k < 8 ? k - 4 : 4));
    v.z &= byte_range_mask(0, k < 8 ? 0 : (k < 12 ? k - 8 : 4));
    v.w &= byte_range_mask(0, k < 12 ? 0 : k - 12);
  }
  return v;
}

// Within one wave: its LDS accesses before it are seen by its lanes after it (a wave's LDS
// operations complete in order; the fences keep the compiler from moving them across).  The
// worker's two waves never meet at a barrier: each runs its own loop (below).
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

static_assert(kWorkerPackMax <= kPiece, "a packed message is built in one LDS piece");
static_assert(sizeof(WPackReq) == 104, "WPackReq: template, descriptor and four words");

// The shift operators in LDS: s_op[b] = A_(2^b) for b = 2..10 (4 x 256 entries each), the byte
// table for single zero bytes.  shift(x, D) = the CRC state x after D zero bytes, D < 2048.
struct WOps {
  const uint32_t* op;   // [9][1024]: A_4, A_8, ..., A_1024
  const uint32_t* tab;  // [256]
  __device__ uint32_t apply(uint32_t b, uint32_t x) const {
    const uint32_t* t = op + (b - 2u) * 1024u;
    return t[x & 0xffu] ^ t[256 + ((x >> 8) & 0xffu)] ^ t[512 + ((x >> 16) & 0xffu)] ^ t[768 + (x >> 24)];
  }
  __device__ uint32_t byte(uint32_t c, uint32_t v) const { return tab[(c ^ v) & 0xffu] ^ (c >> 8); }
  __device__ uint32_t shift(uint32_t x, uint32_t D) const {
#pragma unroll
    for (uint32_t b = 2; b <= 10; b++)
      if ((D >> b) & 1u) x = apply(b, x);
    for (uint32_t k = 0; k < (D & 3u); k++) x = tab[x & 0xffu] ^ (x >> 8);
    return x;
  }
};

// MgenMsg::ComputeCRC32(st, M, n) (mgenMsg.cpp:524-541: st == 0 restarts from ~0; no final xor)
// on one wave, table lookups only.  Lane l takes the 16-byte blocks at 16 l + 1024 k; a block's
// raw CRC (zero register) goes through its lane's Horner chain h = A_1024(h) ^ raw(block), and
// the chain is shifted once by the distance from its last block's end to the message end; the
// message's one partial block (its last bytes) by byte steps.  The start state enters as a
// XOR into bytes 0..3 (the register processing M from st = the zero register processing M with
// LE(st) XOR-ed into its first four bytes).  load16(o) = the 16 message bytes at offset o (any
// bytes past n; o < n).
template <typename Load16>
__device__ __forceinline__ uint32_t wave_crc(uint32_t n, uint32_t st_in, uint32_t lane,
                                             const WOps& ops, Load16 load16) {
  const uint32_t st = st_in == 0u ? 0xFFFFFFFFu : st_in;
  auto word_bytes = [&](uint32_t c, uint32_t w, uint32_t nb) {
    for (uint32_t j = 0; j < nb; j++) c = ops.byte(c, w >> (8 * j));
    return c;
  };
  if (n < 16u) {  // one short block: byte steps from st on every lane (same result)
    const u32x4_t v = n ? load16(0u) : u32x4_t{0u, 0u, 0u, 0u};
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t c = st;
    for (uint32_t j = 0; j < n; j++) c = ops.byte(c, w[j >> 2] >> (8 * (j & 3)));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
  }
  const uint32_t P = (n + 1023u) >> 10;
  uint32_t h = 0, part = 0, last_end = 0;
  for (uint32_t k = 0; k < P; k++) {
    const uint32_t o = 1024u * k + 16u * lane;
    const uint32_t v = n > o ? min(16u, n - o) : 0u;
    if (v) {
      u32x4_t x = load16(o);
      if (o == 0u) x.x ^= st;  // (n >= 16: lane 0's first block is whole)
      if (v == 16u) {
        uint32_t c = ops.apply(2u, x.x);
        c = ops.apply(2u, c ^ x.y);
        c = ops.apply(2u, c ^ x.z);
        c = ops.apply(2u, c ^ x.w);
        h = (k ? ops.apply(10u, h) : 0u) ^ c;
        last_end = o + 16u;
      } else {  // the message's last bytes: whole words through A_4, the rest byte by byte
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
        uint32_t c = 0;
#pragma unroll
        for (uint32_t q = 0; q < 3; q++)
          if (4u * q + 4u <= v) c = ops.apply(2u, c ^ w[q]);
        const uint32_t qw = v >> 2;
        const uint32_t tail = qw == 0 ? w[0] : qw == 1 ? w[1] : qw == 2 ? w[2] : w[3];
        part = word_bytes(c, tail, v & 3u);
      }
    }
  }
  const uint32_t c = (last_end ? ops.shift(h, n - last_end) : 0u) ^ part;
  return WRing::wave_reduce(c, 0u, [](uint32_t a, uint32_t b) { return a ^ b; });  // (DPP)
}

__global__ void __launch_bounds__(128)
worker_kernel(const WReq* q, WRep* m, const uint32_t* __restrict__ tabs,
              const uint32_t* __restrict__ byte_tab, const uint8_t* __restrict__ rtab,
              uint32_t start, uint64_t idle_ticks) {
  __shared__ uint32_t s_op[9 * 1024], s_tab[256];
  __shared__ __attribute__((aligned(16))) uint8_t buf[kPiece];
  __shared__ __attribute__((aligned(16))) uint32_t rq[4 * kReplyChunks];
  __shared__ uint64_t s_crc;   // wave 1's last receive checksum: request number << 32 | crc
  __shared__ uint32_t s_exit;  // wave 0 ended: wave 1 ends too
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  {  // A_(2^b), b = 2..10, from the context's tables
    const uint32_t src[9] = {kTabA4, kTabA8, kTabA16, kTabA32, kTabA64, kTabA128, kTabA256,
                             kTabA512, kTabA1024};
    for (uint32_t t = 0; t < 9; t++)
      for (uint32_t e = threadIdx.x; e < 1024u; e += blockDim.x)
        s_op[t * 1024u + e] = tabs[src[t] * 1024u + e];
  }
  for (uint32_t e = threadIdx.x; e < 256u; e += blockDim.x) s_tab[e] = byte_tab[e];
  if (threadIdx.x == 0) {
    s_crc = (uint64_t)start << 32;
    s_exit = 0u;
  }
  __syncthreads();  // (the only barrier the two waves share)
  const WOps ops = {s_op, s_tab};
  uint32_t last = start;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  if (wv == 1) {
    // Wave 1: the receive path's checksum, in parallel with wave 0's Unpack of the same
    // request -- it polls the same doorbell and, for a receive request, checksums
    // len - 4 bytes from the data area and posts the value with the request number.  Wave 0
    // takes it when the decode says the caller checksums (else it is not used).  It ends when
    // wave 0 does.
    for (;;) {
      if (*reinterpret_cast<volatile uint32_t*>(&s_exit)) break;
      const u32x4_t pc = poll_pieces(q, lane);
      const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)pc.x, 0);
      if ((int32_t)(r - last) <= 0 || __ballot(lane >= 1u && lane < kPollPieces && pc.w != r)) {
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      last = r;
      const uint32_t ol = (uint32_t)__builtin_amdgcn_readlane((int)pc.y, 0);
      const uint32_t op = ol >> kWorkOpShift;
      const uint32_t len = min(ol & kWorkLenMask, (uint32_t)kWorkerMaxBytes);
      if (op == kWorkStop) break;
      if (op == kWorkRecv && len >= 4u) {
        const uint32_t cl = len - 4u;
        const uint32_t c = wave_crc(cl, 0u, lane, ops,
                                    [&](uint32_t o) { return load_masked(q->data + o, o, cl); });
        if (lane == 0) *reinterpret_cast<volatile uint64_t*>(&s_crc) = (uint64_t)r << 32 | c;
      }
    }
    return;
  }
  // MgenMsg::ComputeCRC32(st, data, cl) over the request's data area
  auto span_crc = [&](uint32_t cl, uint32_t st) -> uint32_t {
    return wave_crc(cl, st, lane, ops, [&](uint32_t o) { return load_masked(q->data + o, o, cl); });
  };
  for (;;) {
    const u32x4_t pc = poll_pieces(q, lane);
    const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)pc.x, 0);
    if ((int32_t)(r - last) <= 0) {  // (numbers only grow: an older one is not new)
      if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) break;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    // every data piece written for this request?  (else read before the host wrote it)
    if (__ballot(lane >= 1u && lane < kPollPieces && pc.w != r)) continue;
#if MGENX_DIAG
    const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();  // (stamps: chunk 8, diagnostics)
    const uint64_t tc0 = __builtin_amdgcn_s_memtime();        // (shader clocks: chunk 9)
    uint64_t ts1 = ts0, ts2 = ts0, tc1 = tc0;
#endif
    const uint32_t ol = (uint32_t)__builtin_amdgcn_readlane((int)pc.y, 0);
    const uint32_t op = ol >> kWorkOpShift;
    uint32_t len = ol & kWorkLenMask;
    const uint32_t arg = (uint32_t)__builtin_amdgcn_readlane((int)pc.z, 0);
    // the polled data bytes into LDS: piece k's 12 bytes at 12 (k - 1)
    if (lane >= 1u && lane < kPollPieces) {
      uint32_t* d = reinterpret_cast<uint32_t*>(buf + 12u * (lane - 1u));
      d[0] = pc.x;
      d[1] = pc.y;
      d[2] = pc.z;
    }
    lds_sync();
    if (op == kWorkStop) {
      if (lane == 0) st_sys_release(&m->resp, r);
      break;
    }
    len = min(len, (uint32_t)kWorkerMaxBytes);
    uint32_t status = 0, crc = 0, pk_ret = 0, pk_tx = 0, pk_state = 0;
    if (op == kWorkUnpack || op == kWorkRecv) {
      // the header bytes (at most kWorkerHdrBytes) in LDS, zero past the message: the polled
      // bytes when the header lies within them (24 + dst_len + 4 + host_len + 16 <= 180, or
      // a shorter message), else all of them from the data area
      const uint32_t n = min(len, (uint32_t)kWorkerHdrBytes);
      uint32_t need = 24u + buf[23];
      if (need + 4u <= min(n, kPollData)) need += 4u + buf[need + 3u] + 16u;
      else need += 4u;
      lds_sync();  // (every lane has read the length bytes)
      if (min(n, need) <= kPollData) {  // (the host zero-filled the polled bytes past the message)
        for (uint32_t o = kPollData + 4u * lane; o < kWorkerHdrBytes; o += 256u)
          *reinterpret_cast<uint32_t*>(buf + o) = 0u;
      } else {
        for (uint32_t o = 16u * lane; o < kWorkerHdrBytes; o += 1024u)
          *reinterpret_cast<u32x4_t*>(buf + o) = load_masked(q->data + o, o, n);
      }
      lds_sync();
      if (lane == 0) {
        uint32_t w[8];
        load_fixed(buf, len, w);
        Hdr h;
        parse_header(buf, len, true, w, h);
        mgenx_unpacked u;
        u.flow_id = h.flow;
        u.seq_num = h.seq;
        u.tx_sec = h.sec;
        u.tx_usec = h.usec;
        u.payload_off = h.poff;
        u.lat_raw = h.lat;
        u.lon_raw = h.lon;
        u.alt = h.alt;
        u.msg_len = h.msg_len;
        u.dst_port = h.dst_port;
        u.payload_len = h.plen;
        u.hdr_len = h.hdr_len;
        u.host_port = h.host_port;
        u.flags = h.flags;
        u.err = h.err;
        u.dst_type = h.dst_type;
        u.dst_len = h.dst_len;
        u.payload_type = h.ptype;
        u.gps_status = h.gps;
        u.host_type = h.host_type;
        u.host_len = h.host_len;
        u.decoded = h.dec;
        u.version = h.version;
        u.rsv[0] = u.rsv[1] = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          reinterpret_cast<uint32_t*>(u.dst_addr)[j] = h.dst_addr[j];
          reinterpret_cast<uint32_t*>(u.host_addr)[j] = h.host_addr[j];
        }
        *reinterpret_cast<mgenx_unpacked*>(rq) = u;  // staged in LDS for the lanes' stores
        static_assert(offsetof(mgenx_unpacked, host_addr) + 16 == 86, "2 bytes of tail padding");
        rq[21] &= 0xFFFFu;  // the struct's tail padding (bytes 86-87) as zeros, not stale bits
        // recv: the receive path checksums a decoded message when forced (arg bit 0) or its
        // CHECKSUM flag is set (mgenTransport.cpp:958-965): ComputeCRC32(0, buf, len - 4)
        const bool want = op == kWorkRecv && u.err == 0 && len >= 4u &&
                          ((arg & 1u) || (u.flags & MGENX_FLAG_CHECKSUM));
        rq[kReplyStatus] = want ? kStatusCrc : 0u;
        rq[kReplyCrc] = 0u;
      }
      lds_sync();
#if MGENX_DIAG
      ts1 = __builtin_amdgcn_s_memrealtime();
      tc1 = __builtin_amdgcn_s_memtime();
#endif
      if (rq[kReplyStatus] & kStatusCrc) {  // wave 1's checksum of this request
        uint64_t v;
        while (((v = *reinterpret_cast<volatile uint64_t*>(&s_crc)) >> 32) != r)
          __builtin_amdgcn_s_sleep(1);
        if (lane == 0) rq[kReplyCrc] = (uint32_t)v;
        lds_sync();
      }
#if MGENX_DIAG
      ts2 = __builtin_amdgcn_s_memrealtime();
      if (lane == 8u) {  // chunk 8: the wave's own time, 10-ns ticks from the request's poll
        const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();
        st_chunk(m->reply + 32u, u32x4_t{(uint32_t)(ts1 - ts0), (uint32_t)(ts2 - ts0),
                                         (uint32_t)(ts3 - ts0), r});
      }
      if (lane == 9u) {
        const uint64_t tc3 = __builtin_amdgcn_s_memtime();
        st_chunk(m->reply + 36u, u32x4_t{(uint32_t)(tc1 - tc0), (uint32_t)(tc3 - tc0), 0u, r});
      }
#endif
      if (lane < 8u)  // the 8 tagged chunks in one instruction
        st_chunk(m->reply + 4u * lane, u32x4_t{rq[3u * lane], rq[3u * lane + 1u], rq[3u * lane + 2u], r});
      lds_sync();
    } else if (op == kWorkCrc32) {
      crc = span_crc(len, arg);
    } else if (op == kWorkUpdate) {
      // MgenAnalytic::Update of one record on its device flow state (the request from the
      // polled bytes, WUpdReq); the state is read after an acquire (batch kernels on any XCD
      // wrote it) and written back before the reply's release, so later ones see it
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      const uint32_t* u = reinterpret_cast<const uint32_t*>(buf);
      auto uw = [&](int k) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)u[k]); };
      const uint64_t fp = (uint64_t)uw(0) | (uint64_t)uw(1) << 32;
      const uint32_t slot = uw(2), seq = uw(3), rs = uw(4), ru = uw(5), ts = uw(6), tu = uw(7);
      const uint32_t msg = uw(8);
      lds_sync();
      mgenx_flow_state* sp = reinterpret_cast<mgenx_flow_state*>(fp) + slot;
      FlowSM sm;
      sm.load(sp, lane);
      const double lsum0 = sp->latency_sum;
      const uint64_t nrep0 = sm.nrep;
      const double lat = tdelta(Tm{(int64_t)rs, (int64_t)ru}, Tm{(int64_t)ts, (int64_t)tu});
      bool closed = false;
      FlowClose cl;
      const double lp = sm.exact(seq, (uint64_t)rs << 32 | ru, msg, lat, [&](const FlowClose& c) {
        closed = true;
        cl = c;
      });
      // latency_sum in record order: the window's sum before a close, the closing record's
      // lat' after it (0.0 on a zero restart)
      const double lsum1 = __dadd_rn(lsum0, lp);
      sm.store(sp, lane);
      if (lane == 0) {
        sp->latency_sum = closed ? (cl.zr ? 0.0 : __dadd_rn(0.0, lp)) : lsum1;
        if (closed) {
          mgenx_flow_report rp;
          rp.flow = slot;
          rp.index = (uint32_t)nrep0;
          rp.start_sec = cl.ws.sec;
          rp.start_usec = cl.ws.usec;
          rp.duration = cl.duration;
          rp.msg_count = cl.r_count;
          rp.rate = cl.r_rate;
          rp.loss = cl.r_loss;
          rp.latency_ave = cl.mc == 0 ? -1.0 : cl.mc == 1 ? lsum1 : __ddiv_rn(lsum1, (double)cl.mc);
          rp.latency_min = cl.r_min;
          rp.latency_max = cl.r_max;
          rp.rx_sec = cl.rx.sec;
          rp.rx_usec = cl.rx.usec;
          *reinterpret_cast<mgenx_flow_report*>(rq + kReplyReport) = rp;
        }
      }
      status = closed ? kStatusClosed : 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the state written back before the reply
      lds_sync();
    } else if (op == kWorkPack) {
      // MgenMsg::Pack alone (mgenMsg.cpp:83-313) as the batch pack kernel's meta phase walks
      // it (mgenx_pack.hip: layout, truncation, the payload_len zeroing, RANDOM_FILL after two
      // zero bytes, CHECKSUM flag, ComputeCRC32 over msgLen - 4 with LAST_BUFFER), with the
      // message built whole in LDS and checksummed by the wave.  (Acquire: the RANDOM_FILL
      // stream in rtab may have been rebuilt for a new fill time since an earlier read.)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (lane < 8u)  // the WPackReq, from the polled bytes
        *reinterpret_cast<u32x4_t*>(rq + 4u * lane) = *reinterpret_cast<const u32x4_t*>(buf + 16u * lane);
      lds_sync();
      const uint32_t* tw = rq;  // the template, 17 words (mgenx_flow_tmpl)
      const uint32_t d_seq = rq[18], d_sec = rq[19], d_usec = rq[20];
      const uint32_t d_len = rq[21] & 0xffffu, d_flags = (rq[21] >> 16) & 0xffu;
      const uint32_t msgLen = rq[22], crc_in = rq[23], popts = rq[24];
      const bool ck = (popts & MGENX_PACK_CHECKSUM) != 0, rf = (popts & MGENX_PACK_RANDOM_FILL) != 0;
      const uint32_t t_flow = tw[0], t_dtype = tw[1] & 0xffu, t_dlen = (tw[1] >> 8) & 0xffu;
      const uint32_t t_dport = tw[1] >> 16;
      const uint32_t t_htype = tw[6] & 0xffu, t_hlen = (tw[6] >> 8) & 0xffu, t_hport = tw[6] >> 16;
      const uint32_t t_gps = tw[14] & 0xffu, t_ptype = (tw[14] >> 8) & 0xffu;
      const uint32_t t_plen = tw[14] >> 16, t_has = tw[16] & 0xffu;
      uint32_t flags = d_flags;  // Pack alone: the caller's flags (LAST_BUFFER as it set it)
      const bool dst_ok = t_dtype == 1u || t_dtype == 2u;     // :146-148
      const uint32_t D = t_dlen > 16u ? 16u : t_dlen;
      const bool hv = t_htype == 1u || t_htype == 2u;
      const uint32_t H = hv ? (t_hlen > 16u ? 16u : t_hlen) : 0u;
      uint32_t len = 24u + D;
      const bool host_in = msgLen >= len + H + 4u;              // :182-200
      const bool failed = !dst_ok || (!host_in && msgLen < len);  // :207-210
      bool trunc = !host_in;
      const uint32_t host_at = len;
      if (!trunc) len += 4u + H;
      const uint32_t gps_at = len;
      const bool gps_in = !trunc && msgLen >= len + 13u;        // :219-241
      trunc = trunc || !gps_in;
      if (!trunc) len += 13u;
      const uint32_t pt_at = len;
      const bool pt_in = !trunc && msgLen >= len + 1u;          // :243-251
      trunc = trunc || !pt_in;
      if (!trunc) len += 1u;
      const uint32_t pl_at = len;
      const bool pl_in = !trunc && msgLen >= len + 2u;          // :252-263
      trunc = trunc || !pl_in;
      if (!trunc) len += 2u;
      const bool pay = !trunc && t_has && msgLen >= len + t_plen;  // :264-273
      const uint32_t pend = pay ? len + t_plen : len;
      const uint32_t ret = failed ? 0u : msgLen;
      const bool rfill = rf && !trunc;  // truncated messages are zero-filled (:205-262)
      if (ret > kWorkerPackMax) {
        status = 2;  // too long for the LDS build: the caller takes the batch path
      } else if (ret) {
        // 1. fill [0, msgLen): zeros, or from pend two zeros then the rand() stream
        for (uint32_t o = 16u * lane; o < ret; o += 1024u) {
          uint32_t w[4] = {0u, 0u, 0u, 0u};
          if (rfill && o + 16u > pend) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
              const uint32_t b = o + (uint32_t)j;
              const uint32_t v = b >= pend ? rtab[14u + b - pend] : 0u;
              w[j >> 2] |= v << (8 * (j & 3));
            }
          }
          *reinterpret_cast<u32x4_t*>(buf + o) = u32x4_t{w[0], w[1], w[2], w[3]};
        }
        lds_sync();
        // 2. the payload [len, pend) from the mailbox
        if (pay)
          for (uint32_t o = 16u * lane; o < t_plen; o += 1024u) {
            const u32x4_t v = load_masked(q->data + o, o, t_plen);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            const uint32_t nb = min(16u, t_plen - o);
            for (uint32_t j = 0; j < nb; j++) buf[len + o + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
          }
        // 3. the header (one lane)
        if (!trunc && ck && msgLen > pend + 4u) flags |= MGENX_FLAG_CHECKSUM;  // :295-301
        if (lane == 0) {
          auto put8 = [&](uint32_t at, uint32_t v) { buf[at] = (uint8_t)v; };
          auto put16 = [&](uint32_t at, uint32_t v) { put8(at, v >> 8); put8(at + 1, v); };
          auto put32 = [&](uint32_t at, uint32_t v) {
            put8(at, v >> 24); put8(at + 1, v >> 16); put8(at + 2, v >> 8); put8(at + 3, v);
          };
          put16(0, d_len);                                       // mgenMsg.cpp:97-131
          put8(2, 2);
          put8(3, flags);
          put32(4, t_flow);
          put32(8, d_seq);
          put32(12, d_sec);
          put32(16, d_usec);
          put16(20, t_dport);
          put8(22, t_dtype);
          put8(23, D);
          for (uint32_t k = 0; k < D; k++) put8(24 + k, tw[2 + (k >> 2)] >> (8 * (k & 3)));
          if (host_in) {
            put16(host_at, hv ? t_hport : 0u);
            put8(host_at + 2, hv ? t_htype : 0u);
            put8(host_at + 3, H);
            for (uint32_t k = 0; k < H; k++) put8(host_at + 4 + k, tw[7 + (k >> 2)] >> (8 * (k & 3)));
          }
          if (gps_in) {
            put32(gps_at, tw[11]);
            put32(gps_at + 4, tw[12]);
            put32(gps_at + 8, tw[13]);
            put8(gps_at + 12, t_gps);
          }
          if (pt_in) put8(pt_at, t_ptype);
          if (pl_in) put16(pl_at, t_plen);
          if (!trunc && !pay) {                                  // payload_len zeroed
            put8(len - 2, 0);
            put8(len - 1, 0);
          }
        }
        lds_sync();
        // 4. ComputeCRC32 (checksum on, a whole header)
        uint32_t tx = crc_in;
        if (ck && !trunc) {
          const uint32_t crc_len = (flags & MGENX_FLAG_LAST_BUFFER) ? msgLen - 4u : msgLen;
          tx = wave_crc(crc_len, crc_in, lane, ops, [&](uint32_t o) {  // (:530-533 in wave_crc)
            return *reinterpret_cast<const u32x4_t*>(buf + o);
          });
          flags &= ~(uint32_t)MGENX_FLAG_LAST_BUFFER;
        }
        // 5. the message out, visible before the reply's tags (release)
        for (uint32_t o = 16u * lane; o < ret; o += 1024u)
          *reinterpret_cast<u32x4_t*>(m->out + o) = *reinterpret_cast<const u32x4_t*>(buf + o);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        pk_ret = ret;
        pk_tx = tx;
        pk_state = (uint32_t)len | (flags & 0xffu) << 16;
        lds_sync();
      } else {  // Pack failed: nothing written
        pk_ret = 0u;
        pk_tx = crc_in;
        pk_state = 0xFFFFu | (flags & 0xffu) << 16;
      }
    } else {
      status = 1;
    }
    if (op == kWorkUpdate) {  // chunks 7-15: w21-23 = 0, status, 0; w24-47 the report
      if (lane < 9u)
        st_chunk(m->reply + 4u * (7u + lane),
                 lane == 0u ? u32x4_t{0u, status, 0u, r}
                            : u32x4_t{rq[21u + 3u * lane], rq[22u + 3u * lane], rq[23u + 3u * lane], r});
    } else if (op != kWorkUnpack && op != kWorkRecv && lane < 2u) {
      // chunks 6 and 7: w18-20 = 0, ret, tx_crc; w21-23 = state, status, crc
      st_chunk(m->reply + 4u * (6u + lane), lane == 0u ? u32x4_t{0u, pk_ret, pk_tx, r}
                                                      : u32x4_t{pk_state, status, crc, r});
    }
    last = r;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (lane == 0) {
    *reinterpret_cast<volatile uint32_t*>(&s_exit) = 1u;  // wave 1 ends too
    st_sys_release(&m->alive, 0u);
  }
}

hipError_t launch_worker(const WReq* q, WRep* m, const uint32_t* tabs, const uint32_t* byte_tab,
                         const uint8_t* rtab, uint32_t start, uint64_t idle_ticks,
                         hipStream_t stream) {
  hipLaunchKernelGGL(worker_kernel, dim3(1), dim3(128), 0, stream, q, m, tabs, byte_tab, rtab,
                     start, idle_ticks);
  return hipGetLastError();
}

}  // namespace mgenx
