// mgenx_worker.hip -- the resident single-message worker on gfx950.
//
// An unchanged MGEN build calls MgenMsg::Unpack once per datagram inside its RecvFrom loop and
// MgenMsg::ComputeCRC32 once per message (src/common/mgenTransport.cpp:948-997, 1011-1063).
// Through the batch entry points each such call is a launch, two copies and a synchronisation.
// Here ONE wave stays on the device and polls a mailbox in pinned host memory (WMail): the
// caller writes the message and a request number, the wave reads the message once (every lane
// a 16-byte part of it, all in flight together), decodes or checksums it, writes the reply and
// then the reply number; the caller spins on that.  No launch and no copy per call.
//   unpack: MgenMsg::Unpack on a fresh MgenMsg (mgenMsg.cpp:315-500) -- parse_header, the
//           general-layout path of the batch kernels, over an LDS copy of the header bytes;
//   crc32:  MgenMsg::ComputeCRC32 (mgenMsg.cpp:524-541) -- the wave CRC of crc32_kernel
//           (lane partials through the A_4 tables, combined by x^(8n) shifts) over LDS pieces.
// The wave always ends: on a stop request, and after `idle_ticks` of wall clock
// (s_memrealtime, 100 MHz) without a request; the host relaunches it on the next call (the
// request then pending is served first).  Every store to the mailbox is a vector store.
#include "mgenx_kernels.hpp"
#include "mgenx_parse.hpp"

namespace mgenx {

static_assert(sizeof(mgenx_unpacked) == 88, "mgenx_unpacked is 88 bytes (include/mgenx.h)");
static_assert(sizeof(mgenx_unpacked) <= 128, "the mailbox's reply area");

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

// the 16 mailbox bytes at p (message offset o), bytes at or past n as zero; the mailbox has
// 64 bytes of slack past its largest message, so the whole 16 are always readable
__device__ __forceinline__ u32x4_t load_masked(const uint8_t* p, uint32_t o, uint32_t n) {
  if (o >= n) return u32x4_t{0u, 0u, 0u, 0u};
  u32x4_t v = *reinterpret_cast<const u32x4_t*>(p);
  if (o + 16u > n) {
    const int k = (int)(n - o);  // 1..15 valid bytes
    v.x &= byte_range_mask(0, k < 4 ? k : 4);
    v.y &= byte_range_mask(0, k < 4 ? 0 : (k < 8 ? k - 4 : 4));
    v.z &= byte_range_mask(0, k < 8 ? 0 : (k < 12 ? k - 8 : 4));
    v.w &= byte_range_mask(0, k < 12 ? 0 : k - 12);
  }
  return v;
}

__global__ void __launch_bounds__(64)
worker_kernel(WMail* m, const uint32_t* __restrict__ a4_tab, const uint32_t* __restrict__ byte_tab,
              const uint32_t* __restrict__ xpow, uint32_t start, uint64_t idle_ticks) {
  __shared__ uint32_t s_a4[1024], s_tab[256];
  __shared__ __attribute__((aligned(16))) uint8_t buf[kPiece];
  const uint32_t lane = threadIdx.x;
  for (uint32_t e = lane; e < 1024u; e += 64u) s_a4[e] = a4_tab[e];
  for (uint32_t e = lane; e < 256u; e += 64u) s_tab[e] = byte_tab[e];
  __syncthreads();
  uint32_t last = start;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint32_t r = lane == 0 ? ld_sys(&m->req) : 0u;
    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)r, 0));
    if (r == last) {
      if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) break;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    // the request's words (written before `req`, read after its acquire)
    uint32_t op = 0, len = 0, arg = 0;
    if (lane == 0) {
      op = ld_sys(&m->op);
      len = ld_sys(&m->len);
      arg = ld_sys(&m->arg);
    }
    op = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)op, 0));
    len = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)len, 0));
    arg = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)arg, 0));
    if (op == kWorkStop) {
      if (lane == 0) st_sys_release(&m->resp, r);
      break;
    }
    len = min(len, (uint32_t)kWorkerMaxBytes);
    uint32_t status = 0, crc = 0;
    if (op == kWorkUnpack) {
      // the header bytes (at most kWorkerHdrBytes) into LDS, zero past the message
      const uint32_t n = min(len, (uint32_t)kWorkerHdrBytes);
      for (uint32_t o = 16u * lane; o < kWorkerHdrBytes; o += 1024u)
        *reinterpret_cast<u32x4_t*>(buf + o) = load_masked(m->data + o, o, n);
      __syncthreads();
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
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&u);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&m->unpacked);
        for (uint32_t j = 0; j < sizeof(mgenx_unpacked) / 4u; j++) st_sys(dst + j, src[j]);
      }
      __syncthreads();
    } else if (op == kWorkCrc32) {
      // the span in LDS pieces; each piece's raw CRC from lane partials, folded into the
      // running state: crc(A || B) = x^(8|B|) crc(A) ^ crc(B)
      uint32_t acc = 0;  // raw CRC (zero register) of the bytes so far
      for (uint32_t p0 = 0; p0 < len; p0 += kPiece) {
        const uint32_t pn = min(kPiece, len - p0);
        u32x4_t v[kPiece / 1024];
#pragma unroll
        for (uint32_t k = 0; k < kPiece / 1024; k++) {  // every load issued before any store
          const uint32_t o = p0 + 1024u * k + 16u * lane;
          v[k] = load_masked(m->data + o, o, len);
        }
#pragma unroll
        for (uint32_t k = 0; k < kPiece / 1024; k++)
          *reinterpret_cast<u32x4_t*>(buf + 1024u * k + 16u * lane) = v[k];
        __syncthreads();
        const uint32_t chunk = (((pn + 63u) >> 6) + 3u) & ~3u;
        const uint32_t lo = min(lane * chunk, pn), hi = min(lo + chunk, pn);
        uint32_t c = 0;
        uint32_t k = lo;
        for (; k + 4u <= hi; k += 4u) {
          const uint32_t x = c ^ *reinterpret_cast<const uint32_t*>(buf + k);
          c = s_a4[x & 0xffu] ^ s_a4[256 + ((x >> 8) & 0xffu)] ^ s_a4[512 + ((x >> 16) & 0xffu)] ^
              s_a4[768 + (x >> 24)];
        }
        for (; k < hi; k++) c = s_tab[(c ^ buf[k]) & 0xffu] ^ (c >> 8);
        const uint32_t after = pn - hi;
        if (c && after) c = multmodp(xpow8(after, xpow), c);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o);
        acc = (acc ? multmodp(xpow8(pn, xpow), acc) : 0u) ^ c;
        __syncthreads();
      }
      uint32_t st = arg == 0u ? 0xFFFFFFFFu : arg;  // ComputeCRC32: 0 restarts from ~0
      crc = acc ^ (len ? multmodp(xpow8(len, xpow), st) : st);
    } else {
      status = 1;
    }
    if (lane == 0) {
      st_sys(&m->status, status);
      st_sys(&m->crc, crc);
      st_sys_release(&m->resp, r);
    }
    last = r;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (lane == 0) st_sys_release(&m->alive, 0u);
}

hipError_t launch_worker(WMail* m, const uint32_t* a4_tab, const uint32_t* byte_tab,
                         const uint32_t* xpow, uint32_t start, uint64_t idle_ticks,
                         hipStream_t stream) {
  hipLaunchKernelGGL(worker_kernel, dim3(1), dim3(64), 0, stream, m, a4_tab, byte_tab, xpow, start,
                     idle_ticks);
  return hipGetLastError();
}

}  // namespace mgenx
