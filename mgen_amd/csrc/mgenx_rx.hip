// mgenx_rx.hip -- the TCP receiver's persistent rx_msg over a decoded batch.
//
// Reference: MgenTcpTransport keeps ONE MgenMsg (rx_msg) for the connection
// (src/common/mgenTransport.cpp:1082).  After each message ResetRxMsgState (:1501-1513)
// zeroes mgen_msg_len / msg_len / flow_id / seq_num / the error -- SetFlag(CLEAR) ORs zero,
// so the flags stay -- and the framing sets msg_len (:1714-1720).  Unpack runs only while a
// log file is open (CopyMsgBuffer, :2016-2028), on at most 8192 bytes; it invalidates the
// host address and gps_status first (mgenMsg.cpp:318-319) and assigns members stage by
// stage, so a record that stops early keeps the PREVIOUS record's tx time, destination,
// header length, GPS position and payload.  The CRC check (CalcRxChecksum :1516-1564) reads
// the flags rx_msg holds -- the previous record's when this one never reached them.
//
// mgenx_unpack_batch decodes each record on a fresh MgenMsg and marks what it assigned
// (mgenx_cols.decoded); this pass turns that into the rx_msg view: every member group a
// record did not assign comes from the latest earlier record (or the carried state) that
// did -- a per-group "last assigned" max-scan in three kernels: block aggregates, a scan of
// the block aggregates, and the apply pass (which re-runs the block-local scan).
#include <hip/hip_runtime.h>

#include "mgenx_kernels.hpp"

namespace mgenx {

constexpr uint32_t kRxBlock = 256;
constexpr int kGroups = 6;  // BASE (flags, tx time), DST, HDRLEN, GPS, PTYPE, PLEN
__device__ __constant__ const uint8_t kGroupBit[kGroups] = {MGENX_DEC_BASE, MGENX_DEC_DST,
                                                            MGENX_DEC_HDRLEN, MGENX_DEC_GPS,
                                                            MGENX_DEC_PTYPE, MGENX_DEC_PLEN};

__device__ __forceinline__ int32_t block_max_scan(int32_t v, int32_t* lds /*[4]*/, int32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t o = __shfl_up(v, d);
    if (lane >= (uint32_t)d) v = max(v, o);
  }
  if (lane == 63) lds[wv] = v;
  __syncthreads();
  int32_t before = -1;
  total = -1;
  for (uint32_t k = 0; k < kRxBlock / 64; k++) {
    if (k < wv) before = max(before, lds[k]);
    total = max(total, lds[k]);
  }
  __syncthreads();
  return max(v, before);  // inclusive
}

__device__ __forceinline__ uint8_t rec_decoded(const mgenx_cols& c, uint32_t i, uint32_t opts) {
  return (opts & MGENX_RX_NOLOG) ? (uint8_t)0 : c.decoded[i];
}

// per block and group: the last record that assigned the group (-1 = none)
__global__ void __launch_bounds__(kRxBlock)
rx_agg_kernel(mgenx_cols c, uint32_t n, uint32_t opts, int32_t* __restrict__ agg) {
  __shared__ int32_t lds[4];
  const uint32_t i = blockIdx.x * kRxBlock + threadIdx.x;
  const uint8_t dec = i < n ? rec_decoded(c, i, opts) : 0;
  for (int g = 0; g < kGroups; g++) {
    int32_t tot;
    (void)block_max_scan((dec & kGroupBit[g]) ? (int32_t)i : -1, lds, tot);
    if (threadIdx.x == 0) agg[blockIdx.x * kGroups + g] = tot;
  }
}

// exclusive max-scan of per-block aggregates (ng groups): the carry into each block; one
// workgroup
__global__ void __launch_bounds__(kRxBlock)
rx_carry_kernel(const int32_t* __restrict__ agg, uint32_t nb, int ng, int32_t* __restrict__ carry) {
  __shared__ int32_t lds[4];
  __shared__ int32_t buf[kRxBlock];
  for (int g = 0; g < ng; g++) {
    int32_t run = -1;
    for (uint32_t b0 = 0; b0 < nb; b0 += kRxBlock) {
      const uint32_t b = b0 + threadIdx.x;
      int32_t tot;
      const int32_t incl = block_max_scan(b < nb ? agg[b * ng + g] : -1, lds, tot);
      buf[threadIdx.x] = incl;
      __syncthreads();
      const int32_t excl = threadIdx.x ? buf[threadIdx.x - 1] : -1;
      if (b < nb) carry[b * ng + g] = max(run, excl);
      __syncthreads();
      run = max(run, tot);
    }
  }
}

// the latest record strictly before i (or -1) with v set, from the block-local scan and the
// block's carry
__device__ __forceinline__ int32_t latest_before(bool v, uint32_t i, int32_t carry, int32_t* lds,
                                                 int32_t* buf) {
  int32_t tot;
  const int32_t incl = block_max_scan(v ? (int32_t)i : -1, lds, tot);
  buf[threadIdx.x] = incl;
  __syncthreads();
  const int32_t excl = threadIdx.x ? buf[threadIdx.x - 1] : -1;
  __syncthreads();
  return max(excl, carry);
}

__device__ uint32_t crc_span(const uint8_t* p, uint32_t len, const uint32_t* tab) {
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t k = 0; k < len; k++) c = tab[(c ^ p[k]) & 0xffu] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// CalcRxChecksum for the records that did not assign the flags: checked when checksum_force
// or the CHECKSUM flag rx_msg holds (the latest assigning record's, or the carried state's)
__global__ void __launch_bounds__(kRxBlock)
rx_verdict_kernel(mgenx_cols c, uint32_t n, uint32_t opts, const int32_t* __restrict__ carry,
                  const mgenx_rx_state* __restrict__ state, const uint8_t* __restrict__ slab,
                  const uint64_t* __restrict__ rec_off, const uint32_t* __restrict__ rec_len,
                  const uint32_t* __restrict__ byte_tab, uint8_t* __restrict__ bad,
                  int32_t* __restrict__ bad_agg) {
  __shared__ int32_t lds[4];
  __shared__ int32_t buf[kRxBlock];
  const uint32_t i = blockIdx.x * kRxBlock + threadIdx.x;
  const uint8_t dec = i < n ? rec_decoded(c, i, opts) : 0;
  const int32_t src = latest_before((dec & MGENX_DEC_BASE) != 0, i, carry[blockIdx.x * kGroups], lds,
                                    buf);
  bool b = false;
  if (i < n && !(dec & MGENX_DEC_BASE)) {
    const uint8_t fl = src >= 0 ? c.flags[src] : state->flags;
    if ((opts & MGENX_RX_FORCE) || (fl & MGENX_FLAG_CHECKSUM)) {
      if (opts & MGENX_RX_NOLOG) {
        // the caller's unpack ran with MGENX_OPT_CHECKSUM_FORCE: its verdict
        b = (c.flags[i] & MGENX_FLAG_CHECKSUM_ERROR) != 0;
      } else {
        const uint32_t L = rec_len[i];
        const uint8_t* r = slab + rec_off[i];
        if (L >= 4) {
          const uint32_t want = (uint32_t)r[L - 4] << 24 | (uint32_t)r[L - 3] << 16 |
                                (uint32_t)r[L - 2] << 8 | r[L - 1];
          b = crc_span(r, L - 4, byte_tab) != want;
        }
      }
    }
  }
  if (i < n) bad[i] = b ? 1u : 0u;
  int32_t tot;
  (void)block_max_scan(b ? (int32_t)i : -1, lds, tot);
  if (threadIdx.x == 0) bad_agg[blockIdx.x] = tot;
}

__device__ __forceinline__ void copy_group(const mgenx_cols& c, int g, uint32_t i, int32_t src,
                                           const mgenx_rx_state& st, uint32_t* payload_rec) {
  const bool fs = src < 0;
  const uint32_t j = (uint32_t)src;
  switch (g) {
    case 0:
      c.flags[i] = fs ? st.flags : c.flags[j];
      c.tx_sec[i] = fs ? st.tx_sec : c.tx_sec[j];
      c.tx_usec[i] = fs ? st.tx_usec : c.tx_usec[j];
      break;
    case 1:
      c.dst_type[i] = fs ? st.dst_type : c.dst_type[j];
      c.dst_len[i] = fs ? st.dst_len : c.dst_len[j];
      c.dst_port[i] = fs ? st.dst_port : c.dst_port[j];
      c.dst_addr4[i] = fs ? (uint32_t)st.dst_addr[0] | (uint32_t)st.dst_addr[1] << 8 |
                                (uint32_t)st.dst_addr[2] << 16 | (uint32_t)st.dst_addr[3] << 24
                          : c.dst_addr4[j];
      if (c.dst_addr)
        for (int k = 0; k < 16; k++)
          c.dst_addr[(size_t)i * 16 + k] = fs ? st.dst_addr[k] : c.dst_addr[(size_t)j * 16 + k];
      break;
    case 2:
      if (c.hdr_len) c.hdr_len[i] = fs ? st.hdr_len : c.hdr_len[j];
      break;
    case 3:
      if (c.lat_raw) c.lat_raw[i] = fs ? st.lat_raw : c.lat_raw[j];
      if (c.lon_raw) c.lon_raw[i] = fs ? st.lon_raw : c.lon_raw[j];
      if (c.alt) c.alt[i] = fs ? st.alt : c.alt[j];
      break;
    case 4:
      c.payload_type[i] = fs ? st.payload_type : c.payload_type[j];
      break;
    case 5:
      c.payload_len[i] = fs ? st.payload_len : c.payload_len[j];
      if (c.payload_off) c.payload_off[i] = fs ? st.payload_off : c.payload_off[j];
      if (payload_rec) payload_rec[i] = fs ? MGENX_RX_PREV : j;
      break;
  }
}

__global__ void __launch_bounds__(kRxBlock)
rx_apply_kernel(mgenx_cols c, uint32_t n, uint32_t opts, const int32_t* __restrict__ carry,
                const int32_t* __restrict__ bad_carry, const uint8_t* __restrict__ bad,
                const mgenx_rx_state* __restrict__ state, const uint32_t* __restrict__ rec_len,
                uint32_t* __restrict__ payload_rec) {
  __shared__ int32_t lds[4];
  __shared__ int32_t buf[kRxBlock];
  const uint32_t i = blockIdx.x * kRxBlock + threadIdx.x;
  const uint8_t dec = i < n ? rec_decoded(c, i, opts) : 0;
  int32_t src[kGroups];
  for (int g = 0; g < kGroups; g++)
    src[g] = latest_before((dec & kGroupBit[g]) != 0, i, carry[blockIdx.x * kGroups + g], lds, buf);
  const bool b = i < n && bad[i];
  // the latest checksum failure at or before i among the records that kept the flags
  const int32_t last_bad = max(latest_before(b, i, bad_carry[blockIdx.x], lds, buf),
                               b ? (int32_t)i : -1);
  if (i >= n) return;
  const mgenx_rx_state st = *state;
  const uint8_t err0 = c.err[i];
  for (int g = 0; g < kGroups; g++)
    if (!(dec & kGroupBit[g])) copy_group(c, g, i, src[g], st, payload_rec);
  if (payload_rec && (dec & MGENX_DEC_PLEN)) payload_rec[i] = i;
  if (opts & MGENX_RX_NOLOG) {
    // no Unpack on this connection: the host address and gps_status keep a fresh
    // MgenMsg's (invalid) values, whatever the caller's unpack decoded
    c.gps_status[i] = 0;
    if (c.host_type) c.host_type[i] = 0;
    if (c.host_len) c.host_len[i] = 0;
    if (c.host_port) c.host_port[i] = 0;
    if (c.host_addr)
      for (int k = 0; k < 16; k++) c.host_addr[(size_t)i * 16 + k] = 0;
  }
  if (!(dec & MGENX_DEC_MSGLEN)) c.msg_len[i] = (uint16_t)rec_len[i];  // the framing's msg_len
  if (!(dec & MGENX_DEC_BASE)) {
    c.flow_id[i] = 0;  // ResetRxMsgState
    c.seq_num[i] = 0;
    // flags: the holder's, plus CHECKSUM_ERROR when any record since then failed the CRC
    // (SetFlag ORs and nothing clears it until an Unpack assigns the flags again)
    if (last_bad > src[0]) c.flags[i] |= MGENX_FLAG_CHECKSUM_ERROR;
    c.err[i] = b ? (uint8_t)MGENX_ERROR_CHECKSUM : ((opts & MGENX_RX_NOLOG) ? (uint8_t)0 : err0);
  }
}

// rx_msg after the batch: the last record's members
__global__ void rx_state_kernel(mgenx_cols c, uint32_t n, mgenx_rx_state* __restrict__ state) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t j = n - 1;
  mgenx_rx_state st = *state;
  st.flags = c.flags[j];
  st.tx_sec = c.tx_sec[j];
  st.tx_usec = c.tx_usec[j];
  st.dst_type = c.dst_type[j];
  st.dst_len = c.dst_len[j];
  st.dst_port = c.dst_port[j];
  if (c.dst_addr)
    for (int k = 0; k < 16; k++) st.dst_addr[k] = c.dst_addr[(size_t)j * 16 + k];
  else
    for (int k = 0; k < 4; k++) st.dst_addr[k] = (uint8_t)(c.dst_addr4[j] >> (8 * k));
  if (c.hdr_len) st.hdr_len = c.hdr_len[j];
  if (c.lat_raw) st.lat_raw = c.lat_raw[j];
  if (c.lon_raw) st.lon_raw = c.lon_raw[j];
  if (c.alt) st.alt = c.alt[j];
  st.payload_type = c.payload_type[j];
  st.payload_len = c.payload_len[j];
  st.payload_off = c.payload_off ? c.payload_off[j] : 0u;
  *state = st;
}

hipError_t launch_rx_persist(const mgenx_cols& c, uint32_t n, uint32_t opts, int32_t* ws,
                             mgenx_rx_state* state, const uint8_t* slab, const uint64_t* rec_off,
                             const uint32_t* rec_len, const uint32_t* byte_tab,
                             uint32_t* payload_rec, hipStream_t s) {
  const uint32_t nb = (n + kRxBlock - 1) / kRxBlock;
  int32_t* agg = ws;
  int32_t* carry = agg + (size_t)nb * kGroups;
  int32_t* bad_agg = carry + (size_t)nb * kGroups;
  int32_t* bad_carry = bad_agg + nb;
  uint8_t* bad = reinterpret_cast<uint8_t*>(bad_carry + nb);
  hipLaunchKernelGGL(rx_agg_kernel, dim3(nb), dim3(kRxBlock), 0, s, c, n, opts, agg);
  hipLaunchKernelGGL(rx_carry_kernel, dim3(1), dim3(kRxBlock), 0, s, agg, nb, kGroups, carry);
  hipLaunchKernelGGL(rx_verdict_kernel, dim3(nb), dim3(kRxBlock), 0, s, c, n, opts, carry, state,
                     slab, rec_off, rec_len, byte_tab, bad, bad_agg);
  hipLaunchKernelGGL(rx_carry_kernel, dim3(1), dim3(kRxBlock), 0, s, bad_agg, nb, 1, bad_carry);
  hipLaunchKernelGGL(rx_apply_kernel, dim3(nb), dim3(kRxBlock), 0, s, c, n, opts, carry, bad_carry,
                     bad, state, rec_len, payload_rec);
  hipLaunchKernelGGL(rx_state_kernel, dim3(1), dim3(1), 0, s, c, n, state);
  return hipGetLastError();
}

size_t rx_persist_ws_bytes(uint32_t n) {
  const size_t nb = (n + kRxBlock - 1) / kRxBlock;
  return (2 * nb * kGroups + 2 * nb) * sizeof(int32_t) + n + 256;
}

}  // namespace mgenx
