// mgenx_pack.hip -- batched MgenMsg::Pack with the UDP/SINK send sequence on gfx950.
//
// Reference semantics: MgenUdpTransport::SendMessage (src/common/mgenTransport.cpp:1011-1031)
// = SetFlag(LAST_BUFFER); Pack(buf, msg_len, checksum_enable, tx_checksum)
//   (src/common/mgenMsg.cpp:83-313); WriteChecksum if the CHECKSUM flag is set (:502-522).
//
// Two phases per batch of 64 records, run by different waves of a workgroup (meta waves
// build a group of batches into one LDS buffer while store waves write the previous group
// from the other, see pack_kernel):
//   1. meta (lane = record): build the header image (plus the first payload bytes) in LDS,
//      walk Pack's truncation rules, and compute the CRC-32 algebraically:
//         crc_raw(H || P || F) = A_|P|+|F|(crc_raw(H)) ^ A_|F|(crc_raw(P)) ^ crc_raw(F)
//      with crc_raw(P) precomputed per template (mgenx_pack_prepare), crc_raw(zero fill)=0,
//      crc_raw(random fill prefix) from a per-fill_time table, A_n(x) = x * x^(8n) mod P.
//      Only the <= 76 header bytes are fed through tables, four at a time:
//      c <- A_4(c ^ word) (the <= 3 trailing bytes through the byte table).
//   2. write (lane = 16-byte unit): the batch's records are cut into 16-byte units; every
//      lane composes one unit from fill / header image / payload / trailer and stores it
//      (fast forms: aligned stride slots composed once; back-to-back records as an aligned
//      zero fill with the head/tail units written over it in slab-order windows).
#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr int kProd = 4;                      // meta (producer) waves per workgroup
constexpr int kPackThreads = 2 * kProd * 64;  // + as many store (consumer) waves
constexpr int kImg = 96;  // header image bytes per record (header <= 76, + first payload)


struct PackMeta {
  uint64_t off;
  uint32_t ret;      // Pack() return (0 = failed, nothing written)
  uint32_t trailer;  // value written big-endian at ret-4 (trailer_on 1) or frag-4 (2)
  uint32_t pend;     // end of header + copied payload
  uint32_t poff;     // pool offset of the payload
  uint16_t hdr;      // packet_header_len
  uint8_t trailer_on, rf;  // trailer_on: 0 none, 1 at ret - 4, 2 at frag - 4 (TCP)
  uint32_t tx_out;   // tx_checksum after Pack (out: tx_crc)
  uint32_t state;    // packet_header_len | flags << 16 (out: state)
  uint32_t frag;     // TCP fragment length F > ret: later buffers repeat the image (else 0)
};

// MgenTcpTransport re-sends a fragment's 8-KiB Pack buffer P until F bytes have gone out
// (SetupNextTxBuffer, mgenTransport.cpp:1818-1852): later buffer k starts at start[k] and
// carries P[0 .. cnt[k]) (the last one 4 bytes less with a checksum: its CRC trailer is
// written afterwards).  At most 8 later buffers (F <= 65535, buffers of >= 8185 bytes).
constexpr int kMaxRep = 9;
struct TcpReps {
  uint32_t start[kMaxRep], cnt[kMaxRep];
};
__device__ __forceinline__ TcpReps tcp_reps(uint32_t F, uint32_t B, bool ck) {
  TcpReps t;
  uint32_t pb = B;
  bool done = F <= B;
#pragma unroll
  for (int k = 0; k < kMaxRep; k++) {
    uint32_t st = 0, cnt = 0;
    if (!done) {
      const uint32_t pend = F - pb;
      if (pend == 0) {
        done = true;
      } else {
        uint32_t sz;
        bool last = false;
        if ((ck && pend <= MGENX_TX_BUFFER_SIZE - 4u) || (!ck && pend <= MGENX_TX_BUFFER_SIZE)) {
          sz = pend;
          last = true;
        } else {
          sz = (ck && (int32_t)pend - (int32_t)MGENX_TX_BUFFER_SIZE < 4) ? pend - 4u
                                                                          : MGENX_TX_BUFFER_SIZE;
        }
        st = pb;
        cnt = (last && ck) ? sz - 4u : sz;
        pb += sz;
        done = last;
      }
    }
    t.start[k] = st;
    t.cnt[k] = cnt < B ? cnt : B;
  }
  return t;
}

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

typedef uint32_t u32x2_u1 __attribute__((ext_vector_type(2), aligned(1)));

// the first rem (< 16) bytes of the unit v at d: at most four stores (8, 4, 2, 1 bytes), the
// words moved down as they go out (a select on the byte offset becomes an indexed scratch
// load: the compiler turns such select chains into a stack array)
__device__ __forceinline__ void st_part(uint8_t* d, const uint32_t v[4], uint32_t rem) {
  uint32_t a0 = v[0], a1 = v[1];
  const uint32_t a2 = v[2], a3 = v[3];
  if (rem & 8u) {
    *reinterpret_cast<u32x2_u1*>(d) = u32x2_u1{a0, a1};
    d += 8;
    a0 = a2;
    a1 = a3;
  }
  if (rem & 4u) {
    *reinterpret_cast<u32_u1*>(d) = a0;
    d += 4;
    a0 = a1;
  }
  if (rem & 2u) {
    *reinterpret_cast<u16_u1*>(d) = (uint16_t)a0;
    d += 2;
    a0 >>= 16;
  }
  if (rem & 1u) *d = (uint8_t)a0;
}

// the big-endian trailer word be (memory order MSB..LSB) over the 16-byte unit v at record
// position pos when it overlaps bytes [at, at + 4), merged word by word with masks (a per-lane
// register index v[at >> 2] would compile to a waterfall loop over the wave)
__device__ __forceinline__ void merge_trailer(uint32_t v[4], uint32_t pos, uint32_t at,
                                              uint32_t be) {
  const int t = (int)at - (int)pos;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int o = t - 4 * k;
    uint32_t val = 0u, msk = 0u;
    if (o >= 0 && o < 4) {
      val = be << (8 * o);
      msk = 0xFFFFFFFFu << (8 * o);
    } else if (o < 0 && o > -4) {
      val = be >> (-8 * o);
      msk = 0xFFFFFFFFu >> (-8 * o);
    }
    v[k] = (v[k] & ~msk) | val;
  }
}

// kTcp: the TCP transmit form (PackParams.frag_len: later buffers of a fragment stored from
// the same units, helper meta waves).  A separate instantiation, so the UDP / SINK paths carry
// none of its registers (with them in, config 2 pack ran 0.355 ms instead of 0.216).
template <bool kTcp>
__global__ void __launch_bounds__(kPackThreads)
pack_kernel(PackParams p) {
  // Producer / consumer waves: waves 0..kProd-1 run phase 1 (meta: loads and CRC algebra)
  // of a group of kProd batches into one of two LDS buffers while waves kProd..2kProd-1 run
  // phase 2 (the slab stores) of the previous group from the other buffer.  A wave that
  // both loads and stores stalls its next loads behind its own stores (gfx950 counts
  // stores in vmcnt, in order), so split roles keep the loads and the store stream
  // overlapped; one fence-free block barrier per stage.
  __shared__ __attribute__((aligned(16))) uint8_t s_img[2][kProd][64 * kImg];
  __shared__ PackMeta s_meta[2][kProd][64];
  __shared__ uint32_t s_pre[kProd][65];
  __shared__ uint32_t s_tw[2][kProd * 64];  // trailer words (joint store: any record's)
  __shared__ uint32_t s_joint[2][kProd];    // batch fills its slots exactly (joint store)
  __shared__ uint32_t s_tick[2];            // joint store: the next 4-KB chunk of the group
  __shared__ uint32_t s_tab[256];
  __shared__ uint32_t s_a4[1024];

  // (TCP: the plan's verdict is read first and acted on after the table loads, so its latency
  // overlaps theirs; uniform: the whole grid leaves)
  const bool skip_all = kTcp && p.skip && *p.skip;
  for (int e = threadIdx.x; e < 256; e += blockDim.x) s_tab[e] = p.byte_tab[e];
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) s_a4[e] = p.a4_tab[e];
  __syncthreads();
  if (skip_all) return;

  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const bool producer = wv < kProd;
  const int slot = wv % kProd;
  const int variant = MGENX_DIAG ? p.variant : 0;  // ablations: diagnostics build only
  const bool ck = (p.opts & MGENX_PACK_CHECKSUM) != 0 && variant != 2;
  const bool rf = (p.opts & MGENX_PACK_RANDOM_FILL) != 0;
  const bool raw = (p.opts & MGENX_PACK_RAW) != 0;  // Pack alone (no UDP send sequence)
  const uint64_t n_batches = ((uint64_t)p.n + 63) >> 6;
  const uint64_t n_groups = (n_batches + kProd - 1) / kProd;

  auto wave_sync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // The joint aligned-stride store of group g from LDS buffer jb by every wave that calls it
  // (the store waves, and the meta waves once their own group is built): 4-KB chunks handed
  // out by an LDS ticket.  Returns false, storing nothing, unless every record of the group
  // fills its slot exactly (stride layout, zero fill, image inside kImg: the producers'
  // verdict per batch).
  auto joint = [&](uint64_t g, int jb) -> bool {
    const uint32_t nw = (uint32_t)min((uint64_t)kProd, n_batches - g * kProd);  // its batches
    bool jall = !p.rec_off && !rf && (p.stride & 15u) == 0 && p.stride >= 32 &&
                p.stride <= 65536 && (variant == 0 || variant >= 7);
#pragma unroll
    for (int k = 0; k < kProd; k++)
      if ((uint32_t)k < nw && !s_joint[jb][k]) jall = false;
    if (!jall) return false;
    const uint32_t U = (uint32_t)(p.stride >> 4);        // units per record
    const uint32_t q = 64u / U, rm = 64u % U;            // unit step = q records + rm units
    const uint64_t R0 = g * (uint64_t)(kProd * 64);
    const uint32_t nrec = (uint32_t)min((uint64_t)(kProd * 64), (uint64_t)p.n - R0);
    const uint32_t units = nrec * U;
    uint8_t* const base = p.slab + R0 * p.stride;
    const uint8_t* const G_IMG = &s_img[jb][0][0];
    const uint32_t* const G_TW = s_tw[jb];
    const float invU = 1.0f / (float)U;
    constexpr uint32_t kUnroll = 4, kChunk = 64u * kUnroll;  // units: 4 KB
    for (;;) {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(&s_tick[jb], 1u);
      const uint32_t c0 = (uint32_t)__shfl((int)t, 0) * kChunk;
      if (c0 >= units) break;
      const uint32_t u = c0 + (uint32_t)lane;
      uint32_t r = (uint32_t)((float)u * invU);
      if (r * U > u) r--;
      else if ((r + 1u) * U <= u) r++;
      uint32_t pu = u - r * U;
      u32x4_t v[kUnroll];
      uint32_t tw[kUnroll], pos[kUnroll], rr[kUnroll], last[kUnroll];
#pragma unroll
      for (uint32_t k = 0; k < kUnroll; k++) {
        pos[k] = pu << 4;
        rr[k] = r;
        last[k] = pu == U - 1u;
        const uint32_t rc = min(r, (uint32_t)(kProd * 64) - 1u);
        tw[k] = G_TW[rc];
        v[k] = *reinterpret_cast<const u32x4_t*>(
            &G_IMG[rc * kImg + min(pos[k], (uint32_t)kImg - 16u)]);
        pu += rm;
        r += q;
        if (pu >= U) { pu -= U; r++; }
      }
#pragma unroll
      for (uint32_t k = 0; k < kUnroll; k++) {
        if (!(pos[k] < (uint32_t)kImg && rr[k] < nrec)) v[k] = u32x4_t{0u, 0u, 0u, 0u};
        if (last[k] && tw[k]) v[k].w = tw[k];
      }
#pragma unroll
      for (uint32_t k = 0; k < kUnroll; k++) {
        const uint32_t at = c0 + (uint32_t)lane + 64u * k;
        if (at < units) stu128(base + (uint64_t)at * 16u, v[k]);
      }
    }
    return true;
  };
  // The big-TCP-buffer walk of one record (batch kq, record rr of LDS buffer cb; bst: the
  // calling wave's boundary table in LDS): the 64 lanes walk the whole FRAGMENT [0, Fe) in
  // 16-byte units, consecutive lanes on consecutive units -- P, then each later buffer k
  // (P[0 .. cnt_k) again from its start), then the trailer.  A pass of 64 units inside one
  // buffer past its image and before the trailer is zeros, stored with no per-unit walk.
  auto big_rec = [&](int cb, uint32_t kq, uint32_t rr, uint32_t* bst) {
      const PackMeta R = s_meta[cb][kq][rr];
      if (R.ret == 0u) return;
      const TcpReps reps = tcp_reps(R.frag, R.ret, p.frag_ck != 0);
      const uint8_t* rimg = &s_img[cb][kq][rr * kImg];
      const uint32_t Fe = R.frag ? R.frag : R.ret;       // the fragment's end
      const uint32_t T = R.trailer_on ? Fe - 4u : Fe;     // where its trailer starts
      const uint32_t be = bswap32(R.trailer);             // trailer bytes in memory order
      // buffer starts: 0 (P), then each later buffer's; nb buffers, bst[nb] = Fe
      uint32_t nb = 1;
#pragma unroll
      for (int k = 0; k < kMaxRep; k++) nb += reps.start[k] ? 1u : 0u;
      if (lane == 0) bst[0] = 0u;
#pragma unroll
      for (int k = 0; k < kMaxRep; k++)
        if (lane == k + 1 && reps.start[k]) bst[k + 1] = reps.start[k];
      if (lane == 0) bst[nb] = Fe;
      wave_sync();
      uint8_t* const rbase = p.slab + R.off;
      const uint32_t nu = (Fe + 15u) >> 4;
      uint32_t kb = 0, bcur = 0, bnext = bst[1];
      // the pass's buffer (wave-uniform): a pass of 64 units that lies in one buffer past
      // its image and before the trailer is zeros -- stored as such with no per-unit walk
      // (config 5: 13 of each record's 16 passes)
      uint32_t ukb = 0, ubc = 0, ubn = bnext;
      for (uint32_t u0 = 0; u0 < nu; u0 += 64u) {
        const uint32_t x0 = u0 << 4;
        while (x0 >= ubn && ukb + 1u < nb) {
          ukb++;
          ubc = ubn;
          ubn = bst[ukb + 1];
        }
        if (x0 - ubc >= (uint32_t)kImg && x0 + 1024u <= min(ubn, T)) {
          stu128(rbase + x0 + 16u * (uint32_t)lane, u32x4_t{0u, 0u, 0u, 0u});
          continue;
        }
        const uint32_t u = u0 + (uint32_t)lane;
        if (u >= nu) continue;
        const uint32_t x = u << 4;
        while (x >= bnext && kb + 1u < nb) {
          kb++;
          bcur = bnext;
          bnext = bst[kb + 1];
        }
        const uint32_t pos = x - bcur;
        const u32x4_t iv = *reinterpret_cast<const u32x4_t*>(rimg + min(pos, (uint32_t)kImg - 16u));
        uint32_t v[4] = {iv.x, iv.y, iv.z, iv.w};
        if (pos >= (uint32_t)kImg) v[0] = v[1] = v[2] = v[3] = 0u;  // (past pend: zero fill)
        if ((pos & 15u) != 0u || x + 16u > min(bnext, T)) {
          // a unit across a boundary or off the 16-byte grid of its buffer: byte by byte
          uint32_t kk = kb, bc = bcur, bn = bnext;
#pragma unroll
          for (int j = 0; j < 16; j++) {
            const uint32_t xb = x + (uint32_t)j;
            uint32_t byte = 0u;
            if (xb >= T) {
              byte = xb < Fe ? (be >> (8u * (xb - T))) & 0xffu : 0u;
            } else {
              while (xb >= bn) {
                kk++;
                bc = bn;
                bn = bst[kk + 1];
              }
              const uint32_t q = xb - bc;
              byte = q < (uint32_t)kImg ? rimg[q] : 0u;
            }
            if ((j & 3) == 0) v[j >> 2] = 0u;
            v[j >> 2] |= byte << (8 * (j & 3));
          }
        }
        if (x + 16u <= Fe) {
          stu128(rbase + x, u32x4_t{v[0], v[1], v[2], v[3]});
        } else {
          st_part(rbase + x, v, Fe - x);
        }
      }
      wave_sync();  // (the boundary table is rewritten for the next record)
  };
  // stage s: producers build group blockIdx.x + s * gridDim.x into buffer s & 1, consumers
  // store group blockIdx.x + (s - 1) * gridDim.x from buffer (s - 1) & 1 (block-uniform)
  for (uint64_t s = 0;; s++) {
    const uint64_t gp = (uint64_t)blockIdx.x + s * gridDim.x;
    const bool prod_live = gp < n_groups;
    const bool cons_live = s > 0 && gp - gridDim.x < n_groups;
    if (!prod_live && !cons_live) break;
    // a meta wave with no group to build this stage helps its store wave (big TCP path)
    const bool helper = kTcp && producer && !prod_live;
    const bool builds = producer && !helper;
    const int buf = (int)((builds ? s : s - 1) & 1);
    const uint64_t b = (builds ? gp : gp - gridDim.x) * kProd + slot;
    uint8_t* const S_IMG = &s_img[buf][slot][0];
    PackMeta* const S_META = s_meta[buf][slot];
    const uint64_t i = (b << 6) + lane;
    if constexpr (!kTcp) {
      // a meta wave with no group to build helps store the group of the other buffer
      if (producer && !prod_live && cons_live) {
        if (!(MGENX_DIAG && variant == 10)) (void)joint(gp - gridDim.x, (int)((s - 1) & 1));
        goto stage_end;
      }
    }
    if (!(builds ? prod_live : cons_live) || b >= n_batches) goto stage_end;
    if (builds) {
    if (slot == 0 && lane == 0) s_tick[buf] = 0u;  // (this buffer's store is next stage)
    uint8_t* img = S_IMG + lane * kImg;
    // the image slot starts as zeros: the bytes past pend read as the record's zero fill, so
    // the aligned-stride store loop loads image units without masking them
#pragma unroll
    for (int k = 0; k < kImg / 16; k++)
      *reinterpret_cast<u32x4_t*>(img + 16 * k) = u32x4_t{0u, 0u, 0u, 0u};
    PackMeta m;
    m.off = 0; m.ret = 0; m.trailer = 0; m.pend = 0; m.poff = 0; m.hdr = 0;
    m.trailer_on = 0; m.rf = rf ? 1 : 0; m.tx_out = 0; m.state = 0; m.frag = 0;

    // ------------------------------ phase 1: meta ------------------------------
    if (i < p.n) {
      // Every global read of the record is issued up front, in two dependent rounds:
      // descriptor, then the template (68 B, as 17 words in registers) and the CRC tables
      // indexed by lengths the template fixes.  (Field reads through the template pointer
      // inside the layout walk would each be a serialised round trip.)
      const mgenx_pack_desc d = p.desc[i];
      // TCP: the fragment this Pack starts (F > bufferLen: later buffers re-send the image)
      const uint32_t Ft = (kTcp && p.frag_len) ? p.frag_len[i] : 0u;
      const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tmpl + d.tmpl);
      uint32_t tw[17];
#pragma unroll
      for (int k = 0; k < 17; k++) tw[k] = tp[k];
      m.off = p.rec_off ? p.rec_off[i] : i * p.stride;
      // Pack's bufferLen (= msgLen in mgenMsg.cpp:95) and the msg_len member written at
      // byte 0 differ on the TCP fragment path (mgenTransport.cpp:1924: bufferLen 8192 or
      // 8188, msg_len the fragment length)
      const uint32_t msgLen = (raw && p.buf_len) ? p.buf_len[i] : d.msg_len;
      const uint32_t crc_in = (raw && p.crc_in) ? p.crc_in[i] : 0u;
      const uint32_t t_flow = tw[0], t_dtype = tw[1] & 0xffu, t_dlen = (tw[1] >> 8) & 0xffu;
      const uint32_t t_dport = tw[1] >> 16;
      const uint32_t t_htype = tw[6] & 0xffu, t_hlen = (tw[6] >> 8) & 0xffu;
      const uint32_t t_hport = tw[6] >> 16;
      const uint32_t t_gps = tw[14] & 0xffu, t_ptype = (tw[14] >> 8) & 0xffu;
      const uint32_t t_plen = tw[14] >> 16, t_poff = tw[15], t_has = tw[16] & 0xffu;
      uint32_t flags = raw ? d.flags : (d.flags | MGENX_FLAG_LAST_BUFFER);  // mgenTransport.cpp:1017

      // ---- layout walk (mgenMsg.cpp:97-273), arithmetic only ----
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
      // ComputeCRC32 over msgLen - 4 bytes with LAST_BUFFER, else over msgLen (:305-308)
      const uint32_t crc_len = (flags & MGENX_FLAG_LAST_BUFFER) ? msgLen - 4u : msgLen;
      const bool full_pay = crc_len > len && crc_len >= pend && pend > len;
      const uint32_t f = crc_len > pend ? crc_len - pend : 0u;
      const bool crc_on = ck && !failed && !trunc;
      // ---- the CRC-side reads, independent of the image ----
      uint32_t x_seg = 0, x_f = 0, ia_v = 0, rc_v = 0, tcrc = 0;
      if (crc_on) {
        if (full_pay) { x_seg = p.xpow[pend - len]; tcrc = p.tmpl_crc[d.tmpl]; }
        if (crc_len > pend) { x_f = p.xpow[f]; if (rf && f >= 2) rc_v = p.rcrc[f - 2]; }
        // A_len(init): init = ~0 (ComputeCRC32 restarts from a zero state, :530-533) or
        // the caller's running value
        ia_v = crc_in == 0u ? p.ia[crc_len] : multmodp(p.xpow[crc_len], crc_in);
      }
      // TCP, a fragment past its first buffer: the CRC runs on through every later buffer
      // (SetupNextTxBuffer / CalcTxChecksum, mgenTransport.cpp:1818-1876) and the trailer is
      // the fragment's last 4 bytes.  Later buffer k carries P[0 .. s_k) under the CRC: s_k is
      // one of at most three lengths (full 8192, one shortened buffer, the last one's size -
      // 4), so the powers they take are read here, with the others:
      //   raw(s) = x^(8(s - pend)) raw(P[0 .. pend)) [^ rcrc[s - pend - 2] with RANDOM_FILL]
      //   c'     = raw(s) ^ x^(8s) c   (c = 0 restarts from ~0, as ComputeCRC32 does)
      bool chain = false;
      uint32_t cl[3] = {0u, 0u, 0u}, xs[3] = {0u, 0u, 0u}, xq[3] = {0u, 0u, 0u},
               rq[3] = {0u, 0u, 0u};
      if (kTcp && crc_on && Ft > msgLen && !(flags & MGENX_FLAG_LAST_BUFFER)) {
        chain = true;
        uint32_t pos = msgLen;
        for (int k = 0; k < kMaxRep && pos < Ft; k++) {
          const uint32_t pd = Ft - pos;
          const bool last = pd <= MGENX_TX_BUFFER_SIZE - 4u;
          const uint32_t sz = last ? pd
                                   : ((int32_t)pd - (int32_t)MGENX_TX_BUFFER_SIZE < 4 ? pd - 4u
                                                                                      : MGENX_TX_BUFFER_SIZE);
          cl[last ? 2 : (sz == MGENX_TX_BUFFER_SIZE ? 0 : 1)] = last ? sz - 4u : sz;
          pos += sz;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
          xs[j] = p.xpow[cl[j]];
          if (cl[j] >= pend) {
            xq[j] = p.xpow[cl[j] - pend];
            if (rf && cl[j] - pend >= 3u) rq[j] = p.rcrc[cl[j] - pend - 2u];
          }
        }
      }
      // payload bytes that land in the header image (statically unrolled: one round trip)
      const uint32_t pimg = pay ? min(t_plen, (uint32_t)kImg > len ? (uint32_t)kImg - len : 0u) : 0u;
      // (whole words by dword loads, the last partial word byte by byte: no read past it)
      uint32_t pw[(kImg - 44) / 4];  // the header is >= 44 bytes when a payload follows
#pragma unroll
      for (int k = 0; k < (kImg - 44) / 4; k++) {
        const uint8_t* src = p.pool + t_poff + 4 * k;
        uint32_t w = 0;
        if ((uint32_t)(4 * k + 4) <= pimg) {
          w = ldu32(src);
        } else if ((uint32_t)(4 * k) < pimg) {
          const uint32_t nb = pimg - 4 * k;
          w = src[0] | (nb > 1 ? (uint32_t)src[1] << 8 : 0u) | (nb > 2 ? (uint32_t)src[2] << 16 : 0u);
        }
        pw[k] = w;
      }

      // ---- header image in LDS ----
      img_put16(img, 0, d.msg_len);                            // mgenMsg.cpp:97-131
      img_put8(img, 2, 2);
      img_put8(img, 3, flags);
      img_put32(img, 4, t_flow);
      img_put32(img, 8, d.seq_num);
      img_put32(img, 12, d.tx_sec);
      img_put32(img, 16, d.tx_usec);
      img_put16(img, 20, t_dport);
      if (dst_ok) {
        img_put8(img, 22, t_dtype);
        img_put8(img, 23, D);
#pragma unroll
        for (int k = 0; k < 16; k++)
          if ((uint32_t)k < D) img_put8(img, 24 + k, tw[2 + (k >> 2)] >> (8 * (k & 3)));
        if (host_in) {
          img_put16(img, host_at, hv ? t_hport : 0u);
          img_put8(img, host_at + 2, hv ? t_htype : 0u);
          img_put8(img, host_at + 3, H);
#pragma unroll
          for (int k = 0; k < 16; k++)
            if ((uint32_t)k < H) img_put8(img, host_at + 4 + k, tw[7 + (k >> 2)] >> (8 * (k & 3)));
        }
        if (gps_in) {
          img_put32(img, gps_at, tw[11]);
          img_put32(img, gps_at + 4, tw[12]);
          img_put32(img, gps_at + 8, tw[13]);
          img_put8(img, gps_at + 12, t_gps);
        }
        if (pt_in) img_put8(img, pt_at, t_ptype);
        if (pl_in) img_put16(img, pl_at, t_plen);
      }
      uint32_t tx_out = crc_in;   // unchanged unless the CRC runs
      if (failed) {
        m.ret = 0;
      } else {
        m.ret = msgLen;
        m.rf = (rf && !trunc) ? 1 : 0;   // truncated records are zero-filled (:205-262)
        m.hdr = (uint16_t)len;
        m.pend = pend;
        uint32_t tx_checksum = 0;
        if (!trunc) {
          if (pay) {
            m.poff = t_poff;
#pragma unroll
            for (int k = 0; k < kImg - 44; k++)
              if ((uint32_t)k < pimg) img_put8(img, len + k, pw[k >> 2] >> (8 * (k & 3)));
          } else {
            img_put8(img, len - 2, 0);                           // payload_len field zeroed
            img_put8(img, len - 1, 0);
          }
          if (ck) {                                            // :295-310
            if (msgLen > pend + 4) {
              flags |= MGENX_FLAG_CHECKSUM;
              img_put8(img, 3, flags & 0xffu);
            }
            // ComputeCRC32 over msgLen-4 bytes (LAST_BUFFER is set)
            const uint32_t hb = crc_len < len ? crc_len : len;
            uint32_t c = 0;
            const uint32_t nw = hb >> 2;
            for (uint32_t k = 0; k < nw; k++) {
              const uint32_t x = c ^ *reinterpret_cast<const uint32_t*>(img + 4 * k);
              c = s_a4[x & 0xffu] ^ s_a4[256 + ((x >> 8) & 0xffu)] ^
                  s_a4[512 + ((x >> 16) & 0xffu)] ^ s_a4[768 + (x >> 24)];
            }
            for (uint32_t k = nw << 2; k < hb; k++) c = s_tab[(c ^ img[k]) & 0xffu] ^ (c >> 8);
            if (crc_len > len) {
              if (full_pay) {
                c = multmodp(x_seg, c) ^ tcrc;
              } else {  // the CRC ends inside the payload (msgLen - 4 < pend)
                const uint32_t seg = (crc_len < pend ? crc_len : pend) - len;
                for (uint32_t k = 0; k < seg; k++)
                  c = s_tab[(c ^ p.pool[t_poff + k]) & 0xffu] ^ (c >> 8);
              }
            }
            const uint32_t cb = c;  // raw(P[0 .. pend)) when crc_len >= pend
            if (crc_len > len && crc_len > pend) c = multmodp(x_f, c) ^ rc_v;
            tx_checksum = c ^ ia_v;
            tx_out = tx_checksum;
            if (chain) {  // (crc_len = msgLen >= pend: no LAST_BUFFER here)
              uint32_t a[3];
#pragma unroll
              for (int j = 0; j < 3; j++) {
                if (cl[j] >= pend) {
                  a[j] = multmodp(xq[j], cb) ^ rq[j];
                } else {  // a short last buffer: its bytes are header / payload bytes
                  uint32_t r = 0;
                  for (uint32_t k = 0; k < cl[j]; k++) {
                    const uint32_t b = k < (uint32_t)kImg ? img[k] : p.pool[t_poff + (k - len)];
                    r = s_tab[(r ^ b) & 0xffu] ^ (r >> 8);
                  }
                  a[j] = r;
                }
              }
              uint32_t cc = tx_checksum, pos = msgLen;
              for (int k = 0; k < kMaxRep && pos < Ft; k++) {
                const uint32_t pd = Ft - pos;
                const bool last = pd <= MGENX_TX_BUFFER_SIZE - 4u;
                const uint32_t sz = last ? pd
                                         : ((int32_t)pd - (int32_t)MGENX_TX_BUFFER_SIZE < 4 ? pd - 4u
                                                                                            : MGENX_TX_BUFFER_SIZE);
                const int j = last ? 2 : (sz == MGENX_TX_BUFFER_SIZE ? 0 : 1);
                const uint32_t cr = cc == 0u ? 0xFFFFFFFFu : cc;
                cc = cl[j] ? a[j] ^ multmodp(xs[j], cr) : cr;
                pos += sz;
              }
              m.trailer_on = 2;
              m.trailer = cc ^ 0xFFFFFFFFu;
            }
            flags &= ~(uint32_t)MGENX_FLAG_LAST_BUFFER;
          }
        }
        // caller: WriteChecksum when checksum_enable and the CHECKSUM member flag is set (the
        // TCP form: a one-buffer fragment, mgenTransport.cpp:1376-1385)
        if ((!raw || (kTcp && p.frag_len && Ft <= msgLen)) && ck && (flags & MGENX_FLAG_CHECKSUM) &&
            m.ret >= 4) {
          m.trailer_on = 1;
          m.trailer = tx_checksum ^ 0xFFFFFFFFu;
        }
      }
      if (m.off > p.slab_bytes || m.ret > p.slab_bytes - m.off) m.ret = 0;  // never write OOB
      if (kTcp && p.frag_len && m.ret) {
        if (Ft > m.ret && Ft <= p.slab_bytes - m.off) m.frag = Ft;
      }
      if (m.trailer_on == 2 && !m.frag) m.trailer_on = 0;
      m.tx_out = tx_out;
      // the MgenMsg members Pack leaves behind: packet_header_len (set on every return but
      // the failing ones) and the flags member (CHECKSUM set, LAST_BUFFER cleared)
      m.state = (m.ret ? (uint32_t)m.hdr : 0xFFFFu) | (flags & 0xffu) << 16;
    }
    S_META[lane] = m;
    if constexpr (kTcp) {  // the batch qualifies for the big-buffer walk (read a stage later)
      const bool tok = i >= p.n || (m.pend <= (uint32_t)kImg && (m.ret == 0u || m.ret >= 1024u));
      const bool tall = __all(tok);
      if (lane == 0) s_joint[buf][slot] = tall ? 1u : 0u;
      // then help store the previous group (its verdicts came a stage ago) from the ticket
      if (p.frag_len && !rf && s > 0 && cons_live && !(MGENX_DIAG && variant == 1)) {
        const int cb = (int)((s - 1) & 1);
        const uint64_t gc = gp - gridDim.x;
        uint32_t co_nw = (uint32_t)min((uint64_t)kProd, n_batches - gc * kProd);
#pragma unroll
        for (int k = 0; k < kProd; k++)
          if ((uint32_t)k < co_nw && !s_joint[cb][k]) co_nw = 0;
        if (co_nw) {
          const uint32_t co_n = (uint32_t)min((uint64_t)co_nw * 64u, (uint64_t)p.n - ((gc * kProd) << 6));
          for (;;) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(&s_tick[cb], 1u);
            const uint32_t gr = (uint32_t)__shfl((int)t, 0);
            if (gr >= co_n) break;
            big_rec(cb, gr >> 6, gr & 63u, &s_pre[slot][32]);
          }
        }
      }
    }
    if constexpr (!kTcp) {  // for the joint store: the trailer word, the batch's verdict
      s_tw[buf][slot * 64 + lane] = m.trailer_on == 1 ? bswap32(m.trailer) : 0u;
      const bool jok = i >= p.n || (m.ret == (uint32_t)p.stride && m.pend <= (uint32_t)kImg);
      const bool jall = __all(jok);
      if (lane == 0) s_joint[buf][slot] = jall ? 1u : 0u;
      // then help store the group of the other buffer (its verdicts came a stage ago)
      // (diagnostics: variant 10 = the meta waves never help)
      if (s > 0 && cons_live && !(MGENX_DIAG && variant == 10))
        (void)joint(gp - gridDim.x, (int)((s - 1) & 1));
    }
    goto stage_end;
    }
    {
    // consumer
    const PackMeta m = S_META[lane];
    if (i < p.n && !helper) {
      p.out_len[i] = m.ret;
      if (p.tx_crc) p.tx_crc[i] = m.tx_out;
      if (p.state) p.state[i] = m.state;
    }

    // --------------------------- phase 2: write units ---------------------------
    // Packed slab fast path: when the wave's records lie back to back (rec_off[i + 1] ==
    // rec_off[i] + ret[i]), zero filled, payloads inside the image, every 16-byte-aligned
    // unit of the whole range is first stored as zeros (aligned full-width stores: the
    // fill), then each record's image units and its last 16 bytes (trailer) are written
    // over them.  Everything else keeps one (unaligned) unit store per 16 record bytes.
    const uint32_t nv = b < n_batches ? (uint32_t)min((uint64_t)64, (uint64_t)p.n - (b << 6)) : 0u;
    const bool has = (uint32_t)lane < nv;
    // Aligned stride path (config 2, the recvmmsg slot layout): every record of the group
    // fills its 16-byte-aligned slot exactly (ret == stride), zero fill, image inside kImg.
    // Each 16-byte unit of the range is composed once -- zeros, image bytes (from the
    // zero-padded LDS image: no per-byte masks), or the trailer -- and stored once: no second
    // pass over lines already written (re-writing a record's head and tail units after the
    // fill costs 8 % more bytes but a quarter more time: the lines have left L2 by then and
    // come back as partial writes).  kUnroll units go out per lane and pass, their LDS reads
    // issued together first.  The group's range is stored jointly (joint(), above): 4-KB
    // chunks handed out by an LDS ticket to the store waves and, once their own group is
    // built, the meta waves, so the workgroup's stores march through one contiguous range
    // (instead of kProd streams 64 KB apart) with every wave that has nothing else to do.  A
    // unit's record is found by a float reciprocal (exact after one correction: units <
    // 2^24), its image bytes and trailer word come from LDS (the producers' s_tw; s_joint:
    // the batch qualifies).
    if constexpr (!kTcp) {
      if (joint(gp - gridDim.x, buf)) goto stage_end;
    }
    // Big TCP buffers (PackParams.frag_len set, every record >= 1 KiB, zero fill, image
    // holding header + payload): record by record, the wave's 64 lanes walk the whole
    // FRAGMENT (big_rec, above).  (The general walk below spends most of its instructions per
    // unit on finding the unit's record and on the fill / payload / trailer cases.)
    // When every batch of the group qualifies, the group's records are handed out in slab
    // order by an LDS ticket to its store waves, helpers, and -- once their own batch is
    // built -- the meta waves: the workgroup's stores stay inside a few neighbouring records
    // (one stream per batch, 1 MB apart, ran 0.240 ms for config 5; this 0.204).  Otherwise
    // each wave walks its own batch.
    uint32_t co_nw = 0;
    if (kTcp && p.frag_len && !rf) {
      const uint64_t gc = b / kProd;
      co_nw = (uint32_t)min((uint64_t)kProd, n_batches - gc * kProd);
#pragma unroll
      for (int k = 0; k < kProd; k++)
        if ((uint32_t)k < co_nw && !s_joint[buf][k]) co_nw = 0;
    }
    if (kTcp && p.frag_len && !rf && nv > 0 &&
        (co_nw > 0 || __all(!has || (m.pend <= (uint32_t)kImg && (m.ret == 0u || m.ret >= 1024u))))) {
      if (MGENX_DIAG && variant == 1) goto stage_end;  // (diagnostics: no store phase)
      // with a helper (no group built this stage) the two waves share the records, each with
      // its own boundary table in LDS
      const uint32_t rstep = prod_live ? 1u : 2u;
      uint32_t* const bst = &s_pre[slot][helper ? 32 : 0];
      if (co_nw) {  // the group's records by an LDS ticket (the meta waves join once built)
        const uint32_t co_n = (uint32_t)min((uint64_t)co_nw * 64u, (uint64_t)p.n - (((b / kProd) * kProd) << 6));
        for (;;) {
          uint32_t t = 0;
          if (lane == 0) t = atomicAdd(&s_tick[buf], 1u);
          const uint32_t gr = (uint32_t)__shfl((int)t, 0);
          if (gr >= co_n) break;
          big_rec(buf, gr >> 6, gr & 63u, bst);
        }
      } else {  // this wave's batch (a helper takes every other record)
        for (uint32_t rr = helper ? 1u : 0u; rr < nv; rr += rstep) big_rec(buf, (uint32_t)slot, rr, bst);
      }
      goto stage_end;
    }
    if (helper) goto stage_end;  // the other store forms stay single-wave
    const uint64_t next_off = __shfl_down(m.off, 1);
    const bool packed_ok = !has || (m.ret >= 16u && m.pend <= (uint32_t)kImg && m.frag == 0u &&
                                    ((uint32_t)lane + 1 == nv || m.off + m.ret == next_off));
    // (diagnostics: variant 3 = never the fast path, 4 = fill-then-rewrite scheme, its zero
    // fill only, 5 = that scheme without its wait, 6 = no aligned-stride path)
    const bool fast = !rf && (variant == 0 || variant >= 4) && nv > 0 &&
                      __all(packed_ok);
    const uint32_t kimg = (min(m.pend, m.ret) + 15u) >> 4;  // image units
    uint32_t units = (m.ret + 15u) >> 4;
    if (fast && (variant == 0 || variant >= 6)) {
      // The wave's range is zero-filled with aligned full-width stores, and each record's
      // special units -- its image units and its last 16 bytes (trailer), record-relative
      // and unaligned -- are stored over the fill in windows of 64 (one per lane, in slab
      // order), each window right after the fill has passed its last byte: the partial
      // overwrites meet their lines still in L2 (rewriting after the whole fill sent them
      // back to HBM as partial writes).  No wait is needed: a wave's stores to the same
      // address are performed in program order.  Image units lie wholly inside the record:
      // one reaching past ret is replaced by the last unit, which carries the image bytes
      // it overlaps.
      const uint64_t A0 = __shfl(m.off, 0), A1 = __shfl(m.off + m.ret, (int)nv - 1);
      const uint64_t ra1 = A1 & ~(uint64_t)15;
      uint64_t fill = (A0 + 15u) & ~(uint64_t)15;  // next aligned unit to zero (uniform)
      const uint32_t kin = min(kimg, m.ret >> 4);
      const uint32_t n_sp = has ? kin + (16u * kin < m.ret ? 1u : 0u) : 0u;
      uint32_t incl = n_sp;
#pragma unroll
      for (int s2 = 1; s2 < 64; s2 <<= 1) {
        const uint32_t o = __shfl_up(incl, s2);
        if (lane >= s2) incl += o;
      }
      s_pre[slot][lane + 1] = incl;
      if (lane == 0) s_pre[slot][0] = 0;
      wave_sync();
      const uint32_t total = s_pre[slot][64];
      int ri = 0;
      uint32_t rstart = 0, next_start = s_pre[slot][1];
      PackMeta r = S_META[0];
      const u32x4_t zero = {0u, 0u, 0u, 0u};
      for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t u = base + (uint32_t)lane;
        const bool act = u < total;
        uint32_t pos = 0;
        uint64_t end = 0;
        if (act) {
          if (next_start <= u) {
            do {
              ri++;
              rstart = next_start;
              next_start = s_pre[slot][ri + 1];
            } while (next_start <= u);
            r = S_META[ri];
          }
          const uint32_t k = u - rstart;
          const uint32_t rki = min((min(r.pend, r.ret) + 15u) >> 4, r.ret >> 4);
          pos = k < rki ? 16u * k : r.ret - 16u;
          end = r.off + pos + 16u;
        }
        uint64_t wend = end;  // the window's last byte + 1 (wave max)
#pragma unroll
        for (int s2 = 32; s2 >= 1; s2 >>= 1) {
          const uint64_t o = __shfl_xor(wend, s2);
          wend = o > wend ? o : wend;
        }
        const uint64_t fend = min(ra1, (wend + 15u) & ~(uint64_t)15);
        for (uint64_t a = fill + 16u * (uint32_t)lane; a < fend; a += 1024u)
          stu128(p.slab + a, zero);
        if (fend > fill) fill = fend;
        if (act) {
          const uint8_t* rimg = &S_IMG[ri * kImg];
          uint32_t v[4] = {0u, 0u, 0u, 0u};
          if (pos < r.pend) {
            const u32x4_t iv = *reinterpret_cast<const u32x4_t*>(rimg + pos);
            const uint32_t w[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
              const int lim = (int)r.pend - (int)pos - 4 * kk;
              v[kk] = w[kk] & byte_range_mask(0, lim < 0 ? 0 : (lim > 4 ? 4 : lim));
            }
          }
          if (r.trailer_on == 1 && pos + 16 > r.ret - 4)
            merge_trailer(v, pos, r.ret - 4u, bswap32(r.trailer));
          stu128(p.slab + r.off + pos, u32x4_t{v[0], v[1], v[2], v[3]});
        }
      }
      for (uint64_t a = fill + 16u * (uint32_t)lane; a < ra1; a += 1024u) stu128(p.slab + a, zero);
      goto stage_end;
    }
    if (fast) {  // (diagnostics: the fill-then-rewrite scheme)
      units = has ? kimg + (16u * kimg < m.ret ? 1u : 0u) : 0u;
      const uint64_t a0 = (__shfl(m.off, 0) + 15u) & ~(uint64_t)15;
      const uint64_t a1 = __shfl(m.off + m.ret, (int)nv - 1) & ~(uint64_t)15;
      const u32x4_t zero = {0u, 0u, 0u, 0u};
      for (uint64_t a = a0 + 16u * (uint32_t)lane; a < a1; a += 1024u) stu128(p.slab + a, zero);
      // the overwrites below must land after these stores
      if (!(MGENX_DIAG && variant == 5)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    uint32_t incl = units;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const uint32_t o = __shfl_up(incl, s);
      if (lane >= s) incl += o;
    }
    s_pre[slot][lane + 1] = incl;
    if (lane == 0) s_pre[slot][0] = 0;
    wave_sync();
    const uint32_t total = s_pre[slot][64];
    // Each lane walks units lane, lane+64, ...; its record index only moves forward, so
    // LDS is probed only when the unit leaves the current record.
    int ri = 0;
    uint32_t rstart = 0, next_start = s_pre[slot][1];
    PackMeta r = S_META[0];
    TcpReps reps;
    if constexpr (kTcp) reps = tcp_reps(r.frag, r.ret, p.frag_ck != 0);
    for (uint32_t u = lane; u < ((variant == 1 || variant == 4) ? 0u : total); u += 64) {
      if (next_start <= u) {
        do {
          ri++;
          rstart = next_start;
          next_start = s_pre[slot][ri + 1];
        } while (next_start <= u);
        r = S_META[ri];
        if constexpr (kTcp) reps = tcp_reps(r.frag, r.ret, p.frag_ck != 0);
      }
      uint32_t pos = (u - rstart) << 4;
      if (fast) {  // image units, then the record's last 16 bytes (past the image)
        const uint32_t ki = (min(r.pend, r.ret) + 15u) >> 4;
        if (pos >= (ki << 4)) pos = max(r.ret - 16u, ki << 4);
      }
      const uint8_t* rimg = &S_IMG[ri * kImg];
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
      if (r.trailer_on == 1 && pos + 16 > r.ret - 4)
        merge_trailer(v, pos, r.ret - 4u, bswap32(r.trailer));
      if (kTcp && r.trailer_on == 2 && pos == 0u) {  // TCP: the fragment's last 4 bytes
        *reinterpret_cast<u32_u1*>(p.slab + r.off + r.frag - 4u) = bswap32(r.trailer);
      }
      uint8_t* dst = p.slab + r.off + pos;
      if (pos + 16 <= r.ret) {
        stu128(dst, u32x4_t{v[0], v[1], v[2], v[3]});
      } else {
        st_part(dst, v, r.ret - pos);
      }
      // TCP: the same bytes in every later buffer of the fragment (no copy pass re-reading P)
      if constexpr (kTcp)
#pragma unroll
      for (int k = 0; k < kMaxRep; k++) {
        if (pos < reps.cnt[k]) {
          uint8_t* d2 = p.slab + r.off + reps.start[k] + pos;
          if (pos + 16u <= reps.cnt[k]) {
            stu128(d2, u32x4_t{v[0], v[1], v[2], v[3]});
          } else {
            st_part(d2, v, reps.cnt[k] - pos);
          }
        }
      }
    }
    }
  stage_end:
    // fence-free barrier: __syncthreads()'s vmcnt(0) would drain the consumers' stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
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
  if (p.frag_len)
    hipLaunchKernelGGL(pack_kernel<true>, dim3(grid), dim3(kPackThreads), 0, stream, p);
  else
    hipLaunchKernelGGL(pack_kernel<false>, dim3(grid), dim3(kPackThreads), 0, stream, p);
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

// Utility: CRC-32 of n byte ranges, one WAVE per range: lane k runs the raw CRC (zero
// register, 4 bytes per step through the A_4 tables in LDS) of its 1/64 of the range, and
// the 64 partial CRCs combine by the shift operators x^(8 len) (multmodp): crc(A || B) =
// x^(8|B|) crc(A) ^ crc(B) over GF(2).
//   state_in == NULL: the standard CRC (init ~0, xorout ~0) -- mgenx_crc32_batch;
//   state_in != NULL: MgenMsg::ComputeCRC32(checksum, buf, len) (mgenMsg.cpp:524-541): the
//   running state continues from state_in[i] (0 restarts from ~0), no final xor.
namespace mgenx {
__global__ void __launch_bounds__(256)
crc32_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
             const uint32_t* __restrict__ len, uint32_t n, const uint32_t* __restrict__ byte_tab,
             const uint32_t* __restrict__ a4_tab, const uint32_t* __restrict__ xpow,
             const uint32_t* __restrict__ state_in, uint32_t* __restrict__ out) {
  __shared__ uint32_t s_tab[256];
  __shared__ uint32_t s_a4[1024];
  for (int e = threadIdx.x; e < 256; e += blockDim.x) s_tab[e] = byte_tab[e];
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) s_a4[e] = a4_tab[e];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= n) return;
  const uint8_t* s = data + off[i];
  const uint32_t L = len[i];
  const uint32_t chunk = (((L + 63u) >> 6) + 3u) & ~3u;  // bytes per lane, a multiple of 4
  const uint32_t lo = min(lane * chunk, L), hi = min(lo + chunk, L);
  uint32_t c = 0;  // raw CRC (zero register) of this lane's bytes
  uint32_t k = lo;
  for (; k + 4u <= hi; k += 4u) {
    const uint32_t x = c ^ ldu32(s + k);
    c = s_a4[x & 0xffu] ^ s_a4[256 + ((x >> 8) & 0xffu)] ^ s_a4[512 + ((x >> 16) & 0xffu)] ^
        s_a4[768 + (x >> 24)];
  }
  for (; k < hi; k++) c = s_tab[(c ^ s[k]) & 0xffu] ^ (c >> 8);
  // shift each partial by the bytes after it, then XOR across the wave
  const uint32_t after = L - hi;
  if (c && after) c = multmodp(xpow8(after, xpow), c);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o);
  if (lane == 0) {
    uint32_t st = state_in ? state_in[i] : 0u;
    if (st == 0u) st = 0xFFFFFFFFu;
    const uint32_t r = c ^ (L ? multmodp(xpow8(L, xpow), st) : st);
    out[i] = state_in ? r : (r ^ 0xFFFFFFFFu);
  }
}

hipError_t launch_crc32(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                        const uint32_t* byte_tab, const uint32_t* a4_tab, const uint32_t* xpow,
                        const uint32_t* state_in, uint32_t* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(crc32_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, data, off, len, n,
                     byte_tab, a4_tab, xpow, state_in, out);
  return hipGetLastError();
}
}  // namespace mgenx
