// mgenx_pcap.hip -- pcap2mgen's packet walk (src/common/pcap2mgen.cpp:252-482) for whole
// capture files on gfx950.
//
// The reference loops pcap_next -> copy into a 4-KiB buffer -> ProtoPktETH / ProtoPktIP /
// ProtoPktUDP -> MgenMsg::Unpack -> FindFlow / Update -> LogRecvEvent, one packet at a time.
// Here the capture file sits in HBM and:
//   mgenx_pcap_index  (host) walks the 16-byte record headers -- the pcap_next chain, which is
//                     sequential by construction (each header gives the next one's offset);
//   mgenx_pcap_parse  (device, one lane per packet) finds each packet's UDP payload, source
//                     address / port, TTL and timestamp.  The payloads are then Unpack-ed in
//                     place by mgenx_unpack_batch (rec_off = udp_off, rec_len = udp_len).
// Link / IP / UDP parsing restates protolib's ProtoPktETH / ProtoPktIP(v4/v6) / ProtoPktUDP,
// which is not vendored here (parity unpinned at that layer; oracle/mgen_oracle.c
// or_pcap_frame is the same restatement).
#include <hip/hip_runtime.h>

#include <string.h>

#include <hipcub/hipcub.hpp>

#include "mgenx_kernels.hpp"

namespace mgenx {

__device__ __forceinline__ uint32_t ld_u8(const uint8_t* b, uint64_t i) { return b[i]; }
__device__ __forceinline__ uint32_t ld_be16(const uint8_t* b, uint64_t i) {
  return (uint32_t)b[i] << 8 | b[i + 1];
}
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* b, uint64_t i, bool swapped) {
  const uint32_t v = (uint32_t)b[i] | (uint32_t)b[i + 1] << 8 | (uint32_t)b[i + 2] << 16 |
                     (uint32_t)b[i + 3] << 24;
  return swapped ? __builtin_bswap32(v) : v;
}

struct PcapParams {
  const uint8_t* buf;
  uint64_t buf_bytes;
  const uint64_t* pkt_off;
  uint32_t n;
  uint32_t link_type;
  uint32_t flags;
  uint64_t* udp_off;
  uint32_t* udp_len;
  mgenx_addr* src;
  int32_t* ttl;
  uint32_t* rx_sec;
  uint32_t* rx_usec;
  uint8_t* status;
};

// The frame walk of pcap2mgen.cpp:346-436 for one packet.  Offsets are relative to the
// packet data (the pcap record header + 16).
__global__ void __launch_bounds__(256) pcap_parse_kernel(PcapParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const bool sw = (p.flags & MGENX_PCAP_SWAPPED) != 0;
  const uint64_t ro = p.pkt_off[i];
  uint32_t st = MGENX_PCAP_OOB, uoff = 0, ulen = 0, tsec = 0, tusec = 0;
  int32_t ttl = -1;
  mgenx_addr a;
  a.type = 0; a.len = 0; a.port = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) a.addr[k] = 0;
  do {
    if (ro + 16 > p.buf_bytes) break;
    tsec = ld_u32(p.buf, ro, sw);
    const uint32_t frac = ld_u32(p.buf, ro + 4, sw);
    tusec = (p.flags & MGENX_PCAP_NSEC) ? frac / 1000u : frac;
    const uint32_t caplen = ld_u32(p.buf, ro + 8, sw);
    const uint32_t wirelen = ld_u32(p.buf, ro + 12, sw);
    if (ro + 16 + (uint64_t)caplen > p.buf_bytes) break;
    const uint8_t* d = p.buf + ro + 16;
    const uint32_t kMax = 4094;  // alignedBuffer[1024] less the 2-byte offset (:337-340)
    const uint32_t num = caplen < kMax ? caplen : kMax;
    uint32_t eth_type, ip0, ip_len;
    if (p.link_type == MGENX_DLT_LINUX_SLL) {  // :354-364: 16-byte cooked header
      if (num < 16) { st = MGENX_PCAP_BAD_ETH; break; }
      eth_type = ld_be16(d, 14);
      ip0 = 16;
      ip_len = num - 16;
    } else {  // ProtoPktETH::InitFromBuffer(hdr.len) over maxBytes (:368-380)
      if (wirelen > kMax || wirelen < 14) { st = MGENX_PCAP_BAD_ETH; break; }
      if (num < 14) { st = MGENX_PCAP_TRUNCATED; break; }
      eth_type = ld_be16(d, 12);
      uint32_t hl = 14;
      if (eth_type == 0x8100u) {  // 802.1Q tag: the type after it
        if (wirelen < 18) { st = MGENX_PCAP_BAD_ETH; break; }
        if (num < 18) { st = MGENX_PCAP_TRUNCATED; break; }
        eth_type = ld_be16(d, 16);
        hl = 18;
      }
      ip0 = hl;
      ip_len = wirelen - hl;
    }
    if (eth_type != 0x0800u && eth_type != 0x86DDu) { st = MGENX_PCAP_NOT_IP; break; }
    if (ip_len < 1) { st = MGENX_PCAP_BAD_IP; break; }
    if (ip0 >= num) { st = MGENX_PCAP_TRUNCATED; break; }
    const uint32_t ver = ld_u8(d, ip0) >> 4;
    uint32_t l4, l4_len;  // UDP header offset, IP payload length
    if (ver == 4) {  // ProtoPktIPv4: IHL, total length within the frame
      if (ip_len < 20) { st = MGENX_PCAP_BAD_IP; break; }
      if (ip0 + 20 > num) { st = MGENX_PCAP_TRUNCATED; break; }
      const uint32_t ihl = (ld_u8(d, ip0) & 15u) * 4u;
      const uint32_t tot = ld_be16(d, ip0 + 2);
      if (ihl < 20 || tot < ihl || tot > ip_len) { st = MGENX_PCAP_BAD_IP; break; }
      ttl = (int32_t)ld_u8(d, ip0 + 8);
      a.type = 1; a.len = 4;
#pragma unroll
      for (int k = 0; k < 4; k++) a.addr[k] = d[ip0 + 12 + k];
      if (ld_u8(d, ip0 + 9) != 17u) { st = MGENX_PCAP_NOT_UDP; break; }
      l4 = ip0 + ihl;
      l4_len = tot - ihl;
    } else if (ver == 6) {  // ProtoPktIPv6: 40-byte header, payload length
      if (ip_len < 40) { st = MGENX_PCAP_BAD_IP; break; }
      if (ip0 + 40 > num) { st = MGENX_PCAP_TRUNCATED; break; }
      const uint32_t pl = ld_be16(d, ip0 + 4);
      if (40u + pl > ip_len) { st = MGENX_PCAP_BAD_IP; break; }
      ttl = (int32_t)ld_u8(d, ip0 + 7);
      a.type = 2; a.len = 16;
#pragma unroll
      for (int k = 0; k < 16; k++) a.addr[k] = d[ip0 + 8 + k];
      if (ld_u8(d, ip0 + 6) != 17u) { st = MGENX_PCAP_NOT_UDP; break; }
      l4 = ip0 + 40;
      l4_len = pl;
    } else {
      st = MGENX_PCAP_BAD_IP;  // "Invalid IP pkt version": no source address (:411-415, :422)
      break;
    }
    // ProtoPktUDP::InitFromPacket: the header and its length field within the IP payload
    if (l4_len < 8) { st = MGENX_PCAP_NOT_UDP; break; }
    if (l4 + 8 > num) { st = MGENX_PCAP_TRUNCATED; break; }
    const uint32_t ul = ld_be16(d, l4 + 4);
    if (ul < 8 || ul > l4_len) { st = MGENX_PCAP_NOT_UDP; break; }
    a.port = (uint16_t)ld_be16(d, l4);
    uoff = l4 + 8;
    if (l4 + ul > num) {  // cut by the snapshot length: mgenx_pcap_snap zero-extends it
      st = l4 + 8 + MGENX_MIN_SIZE <= num ? MGENX_PCAP_SNAPPED : MGENX_PCAP_TRUNCATED;
      break;
    }
    st = MGENX_PCAP_UDP;
    ulen = ul - 8;
  } while (false);
  p.status[i] = (uint8_t)st;
  p.udp_off[i] = (st == MGENX_PCAP_UDP || st == MGENX_PCAP_SNAPPED) ? ro + 16 + uoff : ro;
  p.udp_len[i] = st == MGENX_PCAP_UDP ? ulen : 0u;
  p.src[i] = a;
  p.ttl[i] = ttl;
  p.rx_sec[i] = tsec;
  p.rx_usec[i] = tusec;
}

// mgenx_pcap_snap: bytes each SNAPPED packet needs in scratch (its UDP payload length, read
// from the captured UDP header 4 bytes before the payload, 16-byte rounded)
__global__ void __launch_bounds__(256) pcap_snap_size_kernel(const uint8_t* buf, uint32_t n,
                                                             const uint8_t* status,
                                                             const uint64_t* udp_off,
                                                             uint64_t* need) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  uint64_t b = 0;
  if (i < n && status[i] == MGENX_PCAP_SNAPPED) {
    const uint32_t ul = ld_be16(buf, udp_off[i] - 4);
    b = ((uint64_t)(ul - 8) + 15) & ~15ull;
  }
  need[i] = b;
}

// one wave per packet (grid-stride): captured bytes, then zeros up to the UDP length
__global__ void __launch_bounds__(256) pcap_snap_copy_kernel(uint8_t* buf, uint64_t file_bytes,
                                                             uint64_t buf_bytes,
                                                             const uint64_t* pkt_off, uint32_t n,
                                                             uint32_t flags, uint8_t* status,
                                                             uint64_t* udp_off, uint32_t* udp_len,
                                                             const uint64_t* dst) {
  const bool sw = (flags & MGENX_PCAP_SWAPPED) != 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += waves) {
    if (status[i] != MGENX_PCAP_SNAPPED) continue;
    const uint64_t src = udp_off[i];
    const uint32_t len = ld_be16(buf, src - 4) - 8u;
    const uint64_t to = file_bytes + dst[i];
    if (to + len > buf_bytes) continue;  // no room: stays SNAPPED (skipped)
    const uint64_t ro = pkt_off[i];
    const uint64_t have = ro + 16 + ld_u32(buf, ro + 8, sw) - src;  // captured payload bytes
    for (uint32_t k = lane; k < len; k += 64) buf[to + k] = k < have ? buf[src + k] : (uint8_t)0;
    if (lane == 0) {
      udp_off[i] = to;
      udp_len[i] = len;
      status[i] = MGENX_PCAP_UDP;
    }
  }
}

}  // namespace mgenx

using namespace mgenx;

static uint32_t host_u32(const uint8_t* b, bool sw) {
  uint32_t v;
  memcpy(&v, b, 4);
  return sw ? __builtin_bswap32(v) : v;
}

extern "C" {

// the pcap_next loop (pcap2mgen.cpp:344) over a file image: global header (24 bytes), then
// records of a 16-byte header {ts_sec, ts_frac, caplen, len} + caplen bytes
int mgenx_pcap_index(const uint8_t* buf, uint64_t nbytes, uint64_t* pkt_off, uint64_t cap,
                     mgenx_pcap_info* info) {
  if (!buf || !info || (cap && !pkt_off)) return MGENX_EINVAL;
  memset(info, 0, sizeof(*info));
  if (nbytes < 24) return MGENX_EINVAL;
  uint32_t magic;
  memcpy(&magic, buf, 4);
  bool sw = false, ns = false;
  switch (magic) {
    case 0xa1b2c3d4u: break;
    case 0xd4c3b2a1u: sw = true; break;
    case 0xa1b23c4du: ns = true; break;
    case 0x4d3cb2a1u: sw = ns = true; break;
    default: return MGENX_EINVAL;
  }
  info->flags = (ns ? MGENX_PCAP_NSEC : 0u) | (sw ? MGENX_PCAP_SWAPPED : 0u);
  info->snaplen = host_u32(buf + 16, sw);
  info->link_type = host_u32(buf + 20, sw) & 0x0FFFFFFFu;  // LINKTYPE in the low 28 bits
  uint64_t off = 24, n = 0;
  while (off + 16 <= nbytes) {
    const uint32_t caplen = host_u32(buf + off + 8, sw);
    if (off + 16 + (uint64_t)caplen > nbytes) break;  // short read: pcap_next returns NULL
    const uint32_t wirelen = host_u32(buf + off + 12, sw);
    if (caplen < wirelen) info->snap_bytes += ((uint64_t)wirelen + 15) & ~15ull;
    if (n < cap) pkt_off[n] = off;
    n++;
    off += 16 + (uint64_t)caplen;
  }
  info->n_records = n;
  info->consumed = off;
  return MGENX_OK;
}

int mgenx_pcap_parse_run(const uint8_t* dev_buf, uint64_t buf_bytes, const uint64_t* dev_pkt_off,
                         uint32_t n, uint32_t link_type, uint32_t flags, uint64_t* dev_udp_off,
                         uint32_t* dev_udp_len, mgenx_addr* dev_src, int32_t* dev_ttl,
                         uint32_t* dev_rx_sec, uint32_t* dev_rx_usec, uint8_t* dev_status,
                         hipStream_t stream) {
  PcapParams p;
  p.buf = dev_buf; p.buf_bytes = buf_bytes; p.pkt_off = dev_pkt_off; p.n = n;
  p.link_type = link_type; p.flags = flags; p.udp_off = dev_udp_off; p.udp_len = dev_udp_len;
  p.src = dev_src; p.ttl = dev_ttl; p.rx_sec = dev_rx_sec; p.rx_usec = dev_rx_usec;
  p.status = dev_status;
  hipLaunchKernelGGL(pcap_parse_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

int mgenx_pcap_snap_run(uint8_t* dev_buf, uint64_t file_bytes, uint64_t buf_bytes,
                        const uint64_t* dev_pkt_off, uint32_t n, uint32_t flags,
                        uint8_t* dev_status, uint64_t* dev_udp_off, uint32_t* dev_udp_len,
                        uint64_t* need, void* scan_tmp, size_t scan_bytes, hipStream_t stream) {
  hipLaunchKernelGGL(pcap_snap_size_kernel, dim3((n + 256) / 256), dim3(256), 0, stream, dev_buf,
                     n, dev_status, dev_udp_off, need);
  size_t have = scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, have, need, need, (int)n + 1, stream) !=
      hipSuccess)
    return MGENX_EDEVICE;
  const uint32_t blocks = n < 1024u * 4u ? (n + 3) / 4 : 1024u;
  hipLaunchKernelGGL(pcap_snap_copy_kernel, dim3(blocks), dim3(256), 0, stream, dev_buf,
                     file_bytes, buf_bytes, dev_pkt_off, n, flags, dev_status, dev_udp_off,
                     dev_udp_len, need);
  return hipGetLastError() == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
}

size_t mgenx_pcap_snap_scan_bytes(uint32_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (int)n + 1, (hipStream_t)0);
  return b;
}

}  // extern "C"
