// mgenx_pack.hip -- batched MgenMsg::Pack with the UDP/SINK send sequence on gfx950.
//
// Reference semantics: MgenUdpTransport::SendMessage (src/common/mgenTransport.cpp:1011-1031)
// = SetFlag(LAST_BUFFER); Pack(buf, msg_len, checksum_enable, tx_checksum)
//   (src/common/mgenMsg.cpp:83-313); WriteChecksum if the CHECKSUM flag is set (:502-522).
//
// Two phases per wave of 64 records:
//   1. meta (lane = record): build the header image (plus the first payload bytes) in LDS,
//      walk Pack's truncation rules, and compute the CRC-32 algebraically:
//         crc_raw(H || P || F) = A_|P|+|F|(crc_raw(H)) ^ A_|F|(crc_raw(P)) ^ crc_raw(F)
//      with crc_raw(P) precomputed per template (mgenx_pack_prepare), crc_raw(zero fill)=0,
//      crc_raw(random fill prefix) from a per-fill_time table, A_n(x) = x * x^(8n) mod P.
//      Only the <= 76 header bytes are fed through the byte table.
//   2. write (lane = 16-byte unit): the wave's records are cut into 16-byte units; every
//      lane composes one unit from fill / header image / payload / trailer and stores it.
#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr int kPackThreads = 256;
constexpr int kImg = 96;  // header image bytes per record (header <= 76, + first payload)


struct PackMeta {
  uint64_t off;
  uint32_t ret;      // Pack() return (0 = failed, nothing written)
  uint32_t trailer;  // value written big-endian at ret-4 when trailer_on
  uint32_t pend;     // end of header + copied payload
  uint32_t poff;     // pool offset of the payload
  uint16_t hdr;      // packet_header_len
  uint8_t trailer_on, rf;
  uint32_t rsv;
};

__device__ __forceinline__ void img_put8(uint8_t* img, uint32_t at, uint32_t v) {
  if (at < kImg) img[at] = (uint8_t)v;
}
__device__ __forceinline__ void img_put16(uint8_t* img, uint32_t at, uint32_t v) {
  img_put8(img, at, v >> 8);
  img_put8(img, at + 1, v);
}
__device__ __forceinline__ void img_put32(uint8_t* img, uint32_t at, uint32_t v) {
  img_put8(img, at, v >> 24);
  img_put8(img, at + 1, v >> 16);
  img_put8(img, at + 2, v >> 8);
  img_put8(img, at + 3, v);
}

__global__ void __launch_bounds__(kPackThreads)
pack_kernel(PackParams p) {
  constexpr int kWaves = kPackThreads / 64;
  __shared__ __attribute__((aligned(16))) uint8_t s_img[kWaves][64 * kImg];
  __shared__ PackMeta s_meta[kWaves][64];
  __shared__ uint32_t s_pre[kWaves][65];
  __shared__ uint32_t s_tab[256];

  for (int e = threadIdx.x; e < 256; e += blockDim.x) s_tab[e] = p.byte_tab[e];
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint8_t* img = &s_img[wv][lane * kImg];
  const bool ck = (p.opts & MGENX_PACK_CHECKSUM) != 0;
  const bool rf = (p.opts & MGENX_PACK_RANDOM_FILL) != 0;
  const uint64_t n_batches = ((uint64_t)p.n + 63) >> 6;
  const uint64_t n_waves = (uint64_t)gridDim.x * kWaves;

  // block-uniform trip count: every wave reaches the same __syncthreads()
  for (uint64_t base = (uint64_t)blockIdx.x * kWaves; base < n_batches; base += n_waves) {
    const uint64_t b = base + wv;
    const uint64_t i = (b << 6) + lane;
    PackMeta m;
    m.off = 0; m.ret = 0; m.trailer = 0; m.pend = 0; m.poff = 0; m.hdr = 0;
    m.trailer_on = 0; m.rf = rf ? 1 : 0; m.rsv = 0;

    // ------------------------------ phase 1: meta ------------------------------
    if (b < n_batches && i < p.n) {
      const mgenx_pack_desc d = p.desc[i];
      const mgenx_flow_tmpl& t = p.tmpl[d.tmpl];
      m.off = p.rec_off ? p.rec_off[i] : i * p.stride;
      const uint32_t msgLen = d.msg_len;
      uint32_t flags = d.flags | MGENX_FLAG_LAST_BUFFER;      // mgenTransport.cpp:1017
      bool failed = false, trunc = false;
      uint32_t len = 0;
      img_put16(img, 0, d.msg_len);                            // mgenMsg.cpp:97-131
      img_put8(img, 2, 2);
      img_put8(img, 3, flags);
      img_put32(img, 4, t.flow_id);
      img_put32(img, 8, d.seq_num);
      img_put32(img, 12, d.tx_sec);
      img_put32(img, 16, d.tx_usec);
      img_put16(img, 20, t.dst_port);
      len = 22;
      if (t.dst_type != 1 && t.dst_type != 2) {
        failed = true;                                         // :146-148
      } else {
        const uint32_t D = t.dst_len > 16 ? 16u : t.dst_len;
        img_put8(img, 22, t.dst_type);
        img_put8(img, 23, D);
        for (uint32_t k = 0; k < D; k++) img_put8(img, 24 + k, t.dst_addr[k]);
        len = 24 + D;
        const bool hv = (t.host_type == 1 || t.host_type == 2);
        const uint32_t H = hv ? (t.host_len > 16 ? 16u : t.host_len) : 0u;
        if (msgLen >= len + H + 4) {                           // :182-200
          img_put16(img, len, hv ? t.host_port : 0);
          img_put8(img, len + 2, hv ? t.host_type : 0);
          img_put8(img, len + 3, H);
          for (uint32_t k = 0; k < H; k++) img_put8(img, len + 4 + k, t.host_addr[k]);
          len += 4 + H;
        } else if (msgLen < len) {
          failed = true;                                       // :207-210
        } else {
          trunc = true;
        }
        if (!failed && !trunc) {
          if (msgLen >= len + 13) {                            // :219-241
            img_put32(img, len, t.lat_raw);
            img_put32(img, len + 4, t.lon_raw);
            img_put32(img, len + 8, (uint32_t)t.alt);
            img_put8(img, len + 12, t.gps_status);
            len += 13;
          } else {
            trunc = true;
          }
        }
        if (!failed && !trunc) {
          if (msgLen >= len + 1) {                             // :243-251
            img_put8(img, len, t.payload_type);
            len += 1;
          } else {
            trunc = true;
          }
        }
        if (!failed && !trunc) {
          if (msgLen >= len + 2) {                             // :252-263
            img_put16(img, len, t.payload_len);
            len += 2;
          } else {
            trunc = true;
          }
        }
      }
      if (failed) {
        m.ret = 0;
      } else {
        m.ret = msgLen;
        m.rf = (rf && !trunc) ? 1 : 0;   // truncated records are zero-filled (:205-262)
        m.hdr = (uint16_t)len;
        m.pend = len;
        uint32_t tx_checksum = 0;
        if (!trunc) {
          // payload (:264-273)
          if (t.has_payload && msgLen >= len + t.payload_len) {
            m.poff = t.payload_off;
            for (uint32_t k = 0; k < t.payload_len && len + k < (uint32_t)kImg; k++)
              img_put8(img, len + k, p.pool[t.payload_off + k]);
            m.pend = len + t.payload_len;
          } else {
            img_put8(img, len - 2, 0);
            img_put8(img, len - 1, 0);
          }
          if (ck) {                                            // :295-310
            if (msgLen > m.pend + 4) {
              flags |= MGENX_FLAG_CHECKSUM;
              img_put8(img, 3, flags & 0xffu);
            }
            // ComputeCRC32 over msgLen-4 bytes (LAST_BUFFER is set)
            const uint32_t crc_len = msgLen - 4;
            const uint32_t hb = crc_len < (uint32_t)m.hdr ? crc_len : (uint32_t)m.hdr;
            uint32_t c = 0;
            for (uint32_t k = 0; k < hb; k++) c = s_tab[(c ^ img[k]) & 0xffu] ^ (c >> 8);
            if (crc_len > m.hdr) {
              const uint32_t seg_end = crc_len < m.pend ? crc_len : m.pend;
              const uint32_t seg = seg_end - m.hdr;
              if (seg == m.pend - m.hdr && seg > 0) {
                c = multmodp(p.xpow[seg], c) ^ p.tmpl_crc[d.tmpl];
              } else {
                for (uint32_t k = 0; k < seg; k++)
                  c = s_tab[(c ^ p.pool[m.poff + k]) & 0xffu] ^ (c >> 8);
              }
              if (crc_len > m.pend) {
                const uint32_t f = crc_len - m.pend;
                c = multmodp(p.xpow[f], c);
                if (rf && f >= 2) c ^= p.rcrc[f - 2];
              }
            }
            tx_checksum = c ^ p.ia[crc_len];
            flags &= ~(uint32_t)MGENX_FLAG_LAST_BUFFER;
          }
        }
        // caller: WriteChecksum when checksum_enable and the CHECKSUM member flag is set
        if (ck && (flags & MGENX_FLAG_CHECKSUM) && m.ret >= 4) {
          m.trailer_on = 1;
          m.trailer = tx_checksum ^ 0xFFFFFFFFu;
        }
      }
      if (m.off > p.slab_bytes || m.ret > p.slab_bytes - m.off) m.ret = 0;  // never write OOB
      p.out_len[i] = m.ret;
    }
    s_meta[wv][lane] = m;

    // --------------------------- phase 2: write units ---------------------------
    uint32_t units = (m.ret + 15u) >> 4;
    uint32_t incl = units;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const uint32_t o = __shfl_up(incl, s);
      if (lane >= s) incl += o;
    }
    s_pre[wv][lane + 1] = incl;
    if (lane == 0) s_pre[wv][0] = 0;
    __syncthreads();
    const uint32_t total = s_pre[wv][64];
    // Each lane walks units lane, lane+64, ...; its record index only moves forward, so
    // one LDS probe per unit replaces a binary search.
    int ri = 0;
    uint32_t next_start = s_pre[wv][1];
    PackMeta r = s_meta[wv][0];
    for (uint32_t u = lane; u < total; u += 64) {
      bool moved = false;
      while (next_start <= u) {
        ri++;
        next_start = s_pre[wv][ri + 1];
        moved = true;
      }
      if (moved) r = s_meta[wv][ri];
      const uint32_t pos = (u - s_pre[wv][ri]) << 4;
      const uint8_t* rimg = &s_img[wv][ri * kImg];
      uint32_t v[4] = {0u, 0u, 0u, 0u};
      // fill (zero, or the rand() stream after two zero bytes: mgenMsg.cpp:277-292)
      if (r.rf) {
        const int64_t fidx = (int64_t)pos - (int64_t)r.pend - 2;
        if (fidx > -16) {
          const u32x4_t f = ldu128(p.rtab + 16 + fidx);
          v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        }
      }
      // header image (+ payload bytes that fit in it)
      const uint32_t img_end = r.pend < (uint32_t)kImg ? r.pend : (uint32_t)kImg;
      if (pos < img_end) {
        const u32x4_t iv = *reinterpret_cast<const u32x4_t*>(rimg + pos);
        const uint32_t w[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int lim = (int)img_end - (int)pos - 4 * k;
          const uint32_t mk = byte_range_mask(0, lim < 0 ? 0 : (lim > 4 ? 4 : lim));
          v[k] = (v[k] & ~mk) | (w[k] & mk);
        }
      }
      // payload bytes beyond the image
      if (r.pend > (uint32_t)kImg && pos + 16 > (uint32_t)kImg && pos < r.pend) {
        for (int j = 0; j < 16; j++) {
          const uint32_t q = pos + j;
          if (q >= (uint32_t)kImg && q >= r.hdr && q < r.pend) {
            const uint32_t byte = p.pool[r.poff + (q - r.hdr)];
            const int k = j >> 2, sh = (j & 3) * 8;
            v[k] = (v[k] & ~(0xffu << sh)) | (byte << sh);
          }
        }
      }
      // trailer (big-endian CRC at ret-4)
      if (r.trailer_on && pos + 16 > r.ret - 4) {
        const uint32_t be = bswap32(r.trailer);  // memory order b0..b3 = MSB..LSB
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int64_t at = (int64_t)r.ret - 4 + j - (int64_t)pos;
          if (at >= 0 && at < 16) {
            const int k = (int)at >> 2, sh = ((int)at & 3) * 8;
            const uint32_t byte = (be >> (8 * j)) & 0xffu;
            v[k] = (v[k] & ~(0xffu << sh)) | (byte << sh);
          }
        }
      }
      uint8_t* dst = p.slab + r.off + pos;
      if (pos + 16 <= r.ret) {
        stu128(dst, u32x4_t{v[0], v[1], v[2], v[3]});
      } else {
        const uint32_t rem = r.ret - pos;
        for (uint32_t j = 0; j < rem; j++) dst[j] = (uint8_t)(v[j >> 2] >> ((j & 3) * 8));
      }
    }
    __syncthreads();
  }
}

// crc_raw of each template's payload (zero initial state), one thread per template.
__global__ void pack_prepare_kernel(const mgenx_flow_tmpl* tmpl, uint32_t n_tmpl,
                                    const uint8_t* pool, const uint32_t* byte_tab,
                                    uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tmpl) return;
  uint32_t c = 0;
  if (tmpl[t].has_payload) {
    const uint8_t* s = pool + tmpl[t].payload_off;
    for (uint32_t k = 0; k < tmpl[t].payload_len; k++)
      c = byte_tab[(c ^ s[k]) & 0xffu] ^ (c >> 8);
  }
  out[t] = c;
}

hipError_t launch_pack(const PackParams& p, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(pack_kernel, dim3(grid), dim3(kPackThreads), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_pack_prepare(const mgenx_flow_tmpl* tmpl, uint32_t n_tmpl, const uint8_t* pool,
                               const uint32_t* byte_tab, uint32_t* out, hipStream_t stream) {
  if (n_tmpl == 0) return hipSuccess;
  hipLaunchKernelGGL(pack_prepare_kernel, dim3((n_tmpl + 255) / 256), dim3(256), 0, stream, tmpl,
                     n_tmpl, pool, byte_tab, out);
  return hipGetLastError();
}

}  // namespace mgenx

// Utility: standard CRC-32 of n byte ranges, one thread per range (byte table in LDS).
namespace mgenx {
__global__ void crc32_kernel(const uint8_t* data, const uint64_t* off, const uint32_t* len,
                             uint32_t n, const uint32_t* byte_tab, uint32_t* out) {
  __shared__ uint32_t s_tab[256];
  for (int e = threadIdx.x; e < 256; e += blockDim.x) s_tab[e] = byte_tab[e];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* s = data + off[i];
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t k = 0; k < len[i]; k++) c = s_tab[(c ^ s[k]) & 0xffu] ^ (c >> 8);
  out[i] = c ^ 0xFFFFFFFFu;
}

hipError_t launch_crc32(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                        const uint32_t* byte_tab, const uint32_t* /*xpow*/, uint32_t* out,
                        hipStream_t stream) {
  hipLaunchKernelGGL(crc32_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, data, off, len, n,
                     byte_tab, out);
  return hipGetLastError();
}
}  // namespace mgenx
