// mgenx_compat.hpp -- the batching engine behind the MgenMsg / MgenPayload / MgenAnalytic
// shim (mgenMsg.h, mgenPayload.h, mgenAnalytic.h in this directory).
//
// Every shim call is a batch: MgenMsg::Pack / Unpack / ComputeCRC32 and MgenAnalytic::Update
// on one object are batches of one, and MgenMsg::PackBatch / UnpackBatch /
// MgenAnalyticTable::UpdateBatch hand whole batches (the recvmmsg / sendmmsg handoff of
// SURVEY.md 8(b)) to the same code.  A batch is staged in one pinned host arena, copied to
// the device in one hipMemcpyAsync, processed by libmgenx's gfx950 kernels
// (mgenx_pack_msgs, mgenx_unpack_batch, mgenx_crc32_update, mgenx_flow_reduce) and copied
// back in one more; the call returns when the results are in the caller's buffers.  A single
// Pack, Unpack, ComputeCRC32 or MgenAnalytic::Update (what an unchanged transport and
// Mgen::UpdateRecvAnalytics call per message) goes instead to the resident worker
// (mgenx_worker_*): two waves kept on the device polling a request block, so the call pays no
// launch and no copy; an Unpack also brings back the checksum the receive path computes next.
// There is no host implementation of the codec here: without a GPU the calls throw.
//
// One engine per process (device MGENX_DEVICE, default 0), serialised by a mutex: the
// reference's callers run on one dispatcher thread.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "mgenx.h"

namespace mgenx {
namespace compat {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// One message for mgenx_pack_msgs: the MgenMsg members as a template + descriptor, Pack's
// bufferLen and the tx_checksum argument.
struct PackIn {
  mgenx_flow_tmpl tmpl;
  const uint8_t* payload;  // tmpl.payload_len bytes when tmpl.has_payload
  mgenx_pack_desc desc;
  uint32_t buf_len, crc_in;
};
struct PackOut {
  uint32_t ret, tx_crc, state;  // Pack() return, tx_checksum after, hdr_len | flags << 16
};

// One decoded record: the MgenMsg members Unpack can assign, plus which it did.
struct UnpackOut {
  uint32_t flow_id, seq_num, tx_sec, tx_usec, payload_off;
  uint32_t lat_raw, lon_raw;
  int32_t alt;
  uint16_t msg_len, dst_port, payload_len, hdr_len, host_port;
  uint8_t flags, err, dst_type, dst_len, payload_type, gps_status, host_type, host_len, decoded;
  uint8_t dst_addr[16], host_addr[16];
};

// One RECV / RERR log event: an MgenMsg's members as a decoded record (core.err = 0 for
// RECV, the MgenMsg::Error for RERR, MGENX_ERROR_RERR_NONE for a RERR of ERROR_NONE), the
// message bytes the line reads (the DATA payload at payload_off; for binary, the whole
// header + payload), the source, the event time and the TTL (< 0: unknown).
struct LogRecvIn {
  mgenx_rec core;
  uint16_t hdr_len, host_port;
  uint8_t host_type, host_len;
  uint8_t dst_addr[16], host_addr[16];
  uint32_t lat_raw, lon_raw;
  int32_t alt;
  uint32_t payload_off;
  mgenx_addr src;
  uint32_t rx_sec, rx_usec;
  int32_t ttl;
  const uint8_t* msg;
  uint32_t msg_bytes;
};

class Engine {
 public:
  static Engine& Get() {
    static Engine e;
    return e;
  }
  std::mutex& Lock() { return mu_; }

  // ---- MgenMsg::Pack (mgenx_pack_msgs) over n messages -------------------------------
  // dst[i] receives out[i].ret bytes (nothing when Pack fails).
  void Pack(const PackIn* in, unsigned n, uint32_t opts, uint32_t fill_time, uint8_t* const* dst,
            PackOut* out) {
    if (n == 0) return;
    Init();
    const uint32_t blen0 = in[0].buf_len ? in[0].buf_len : in[0].desc.msg_len;
    if (n == 1 && blen0 <= MGENX_WORKER_PACK_MAX && Worker()) {  // one message: the worker
      Check(mgenx_worker_pack(worker_, &in[0].tmpl, in[0].payload, &in[0].desc, blen0,
                              in[0].crc_in, opts, fill_time, dst[0], &out[0].ret, &out[0].tx_crc,
                              &out[0].state),
            "mgenx_worker_pack");
      return;
    }
    if (opts & MGENX_PACK_RANDOM_FILL)  // (the context caches the stream of its last fill time)
      Check(mgenx_set_fill_time(ctx_, fill_time), "mgenx_set_fill_time");
    // host staging: [tmpl | desc | buf_len | crc_in | rec_off | pool]
    size_t pool = 0, slab = 0;
    for (unsigned i = 0; i < n; i++) {
      if (in[i].tmpl.has_payload) pool += in[i].tmpl.payload_len;
      slab += Align(in[i].buf_len ? in[i].buf_len : in[i].desc.msg_len, 16);
    }
    Layout L;
    const size_t o_tmpl = L.Add(n * sizeof(mgenx_flow_tmpl));
    const size_t o_desc = L.Add(n * sizeof(mgenx_pack_desc));
    const size_t o_blen = L.Add(n * 4u), o_cin = L.Add(n * 4u), o_off = L.Add(n * 8u);
    const size_t o_pool = L.Add(pool ? pool : 16);
    const size_t in_bytes = L.size;
    // device outputs: [tmpl_crc | out_len | tx_crc | state | slab]
    const size_t o_tcrc = L.Add(n * 4u), o_len = L.Add(n * 4u), o_tx = L.Add(n * 4u);
    const size_t o_state = L.Add(n * 4u), o_slab = L.Add(slab + 64);
    Reserve(L.size);
    uint8_t* h = host_;
    mgenx_flow_tmpl* t = (mgenx_flow_tmpl*)(h + o_tmpl);
    mgenx_pack_desc* d = (mgenx_pack_desc*)(h + o_desc);
    uint32_t* blen = (uint32_t*)(h + o_blen);
    uint32_t* cin = (uint32_t*)(h + o_cin);
    uint64_t* off = (uint64_t*)(h + o_off);
    size_t p = 0, s = 0;
    for (unsigned i = 0; i < n; i++) {
      t[i] = in[i].tmpl;
      if (in[i].tmpl.has_payload) {
        t[i].payload_off = (uint32_t)p;
        memcpy(h + o_pool + p, in[i].payload, in[i].tmpl.payload_len);
        p += in[i].tmpl.payload_len;
      }
      d[i] = in[i].desc;
      d[i].tmpl = i;
      blen[i] = in[i].buf_len ? in[i].buf_len : in[i].desc.msg_len;
      cin[i] = in[i].crc_in;
      off[i] = s;
      s += Align(blen[i], 16);
    }
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    Check(mgenx_pack_prepare(ctx_, (const mgenx_flow_tmpl*)(g + o_tmpl), n, g + o_pool,
                             (uint32_t*)(g + o_tcrc), stream_), "mgenx_pack_prepare");
    Check(mgenx_pack_msgs(ctx_, (const mgenx_flow_tmpl*)(g + o_tmpl), (const uint32_t*)(g + o_tcrc),
                          (const mgenx_pack_desc*)(g + o_desc), n, g + o_pool, g + o_slab,
                          slab + 64, (const uint64_t*)(g + o_off), 0, (const uint32_t*)(g + o_blen),
                          (const uint32_t*)(g + o_cin), (uint32_t*)(g + o_len),
                          (uint32_t*)(g + o_tx), (uint32_t*)(g + o_state), opts, fill_time,
                          stream_),
          "mgenx_pack_msgs");
    D2H(h + o_len, g + o_len, L.size - o_len);
    Sync();
    const uint32_t* len = (const uint32_t*)(h + o_len);
    const uint32_t* tx = (const uint32_t*)(h + o_tx);
    const uint32_t* st = (const uint32_t*)(h + o_state);
    for (unsigned i = 0; i < n; i++) {
      out[i].ret = len[i];
      out[i].tx_crc = tx[i];
      out[i].state = st[i];
      if (len[i] && dst[i]) memcpy(dst[i], h + o_slab + off[i], len[i]);
    }
  }

  // ---- MgenMsg::Unpack alone (mgenx_unpack_batch, MGENX_OPT_SKIP_CRC) ---------------
  // One message (the reference's per-datagram call): the resident worker, no launch or copy.
  // The worker also computes the checksum the receive path asks for next when `force`
  // (checksum_force, the Unpack argument the callers pass) is set or the message carries
  // CHECKSUM (mgenTransport.cpp:958-965): ComputeCRC32(0, buf, len - 4) on the same bytes then
  // returns it without a GPU call (Crc32Update).
  void Unpack(const uint8_t* const* bufs, const uint16_t* lens, unsigned n, UnpackOut* out,
              bool force = false) {
    if (n == 0) return;
    Init();
    crc_cache_.valid = false;
    if (n == 1 && Worker()) {
      mgenx_unpacked u;
      uint32_t crc = 0, done = 0;
      // the flags byte (offset 3, MgenMsg::FLAGS_OFFSET) decides whether a CRC follows: without
      // one, Unpack alone copies only the header bytes into the request
      const bool want_crc = force || (lens[0] > 3u && (bufs[0][3] & MGENX_FLAG_CHECKSUM) != 0u);
      if (want_crc)
        Check(mgenx_worker_recv(worker_, bufs[0], lens[0], force ? 1u : 0u, &u, &crc, &done),
              "mgenx_worker_recv");
      else
        Check(mgenx_worker_unpack(worker_, bufs[0], lens[0], &u), "mgenx_worker_unpack");
      if (done) {
        crc_cache_.valid = true;
        crc_cache_.ptr = bufs[0];
        crc_cache_.len = lens[0] - 4u;
        crc_cache_.bytes.assign(bufs[0], bufs[0] + crc_cache_.len);
        crc_cache_.crc = crc;
      }
      UnpackOut& r = out[0];
      r.flow_id = u.flow_id;
      r.seq_num = u.seq_num;
      r.tx_sec = u.tx_sec;
      r.tx_usec = u.tx_usec;
      r.payload_off = u.payload_off;
      r.lat_raw = u.lat_raw;
      r.lon_raw = u.lon_raw;
      r.alt = u.alt;
      r.msg_len = u.msg_len;
      r.dst_port = u.dst_port;
      r.payload_len = u.payload_len;
      r.hdr_len = u.hdr_len;
      r.host_port = u.host_port;
      r.flags = u.flags;
      r.err = u.err;
      r.dst_type = u.dst_type;
      r.dst_len = u.dst_len;
      r.payload_type = u.payload_type;
      r.gps_status = u.gps_status;
      r.host_type = u.host_type;
      r.host_len = u.host_len;
      r.decoded = u.decoded;
      memcpy(r.dst_addr, u.dst_addr, 16);
      memcpy(r.host_addr, u.host_addr, 16);
      return;
    }
    size_t slab = 0;
    for (unsigned i = 0; i < n; i++) slab += Align(lens[i], 16);
    Layout L;
    const size_t o_off = L.Add(n * 8u), o_len = L.Add(n * 4u), o_slab = L.Add(slab + 64);
    const size_t in_bytes = L.size;
    // outputs, one array per column
    struct Col {
      size_t off, w;
    };
    const size_t w4[] = {4, 4, 4, 4, 4, 4, 4, 4};  // flow seq txs txu dst4 poff lat lon
    size_t c4[8];
    for (int k = 0; k < 8; k++) c4[k] = L.Add(n * w4[k]);
    const size_t c_alt = L.Add(n * 4u);
    size_t c2[5];  // msg_len dst_port payload_len hdr_len host_port
    for (int k = 0; k < 5; k++) c2[k] = L.Add(n * 2u);
    size_t c1[9];  // flags err dst_type dst_len payload_type gps host_type host_len decoded
    for (int k = 0; k < 9; k++) c1[k] = L.Add(n * 1u);
    const size_t c_da = L.Add(n * 16u), c_ha = L.Add(n * 16u);
    Reserve(L.size);
    uint8_t* h = host_;
    uint64_t* off = (uint64_t*)(h + o_off);
    uint32_t* rl = (uint32_t*)(h + o_len);
    size_t s = 0;
    for (unsigned i = 0; i < n; i++) {
      off[i] = s;
      rl[i] = lens[i];
      memcpy(h + o_slab + s, bufs[i], lens[i]);
      s += Align(lens[i], 16);
    }
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    mgenx_cols c;
    memset(&c, 0, sizeof(c));
    c.flow_id = (uint32_t*)(g + c4[0]);
    c.seq_num = (uint32_t*)(g + c4[1]);
    c.tx_sec = (uint32_t*)(g + c4[2]);
    c.tx_usec = (uint32_t*)(g + c4[3]);
    c.dst_addr4 = (uint32_t*)(g + c4[4]);
    c.payload_off = (uint32_t*)(g + c4[5]);
    c.lat_raw = (uint32_t*)(g + c4[6]);
    c.lon_raw = (uint32_t*)(g + c4[7]);
    c.alt = (int32_t*)(g + c_alt);
    c.msg_len = (uint16_t*)(g + c2[0]);
    c.dst_port = (uint16_t*)(g + c2[1]);
    c.payload_len = (uint16_t*)(g + c2[2]);
    c.hdr_len = (uint16_t*)(g + c2[3]);
    c.host_port = (uint16_t*)(g + c2[4]);
    c.flags = g + c1[0];
    c.err = g + c1[1];
    c.dst_type = g + c1[2];
    c.dst_len = g + c1[3];
    c.payload_type = g + c1[4];
    c.gps_status = g + c1[5];
    c.host_type = g + c1[6];
    c.host_len = g + c1[7];
    c.decoded = g + c1[8];
    c.dst_addr = g + c_da;
    c.host_addr = g + c_ha;
    Check(mgenx_unpack_batch(ctx_, g + o_slab, slab + 64, (const uint64_t*)(g + o_off), 0,
                             (const uint32_t*)(g + o_len), 0, n, &c, MGENX_OPT_SKIP_CRC, stream_),
          "mgenx_unpack_batch");
    D2H(h + c4[0], g + c4[0], L.size - c4[0]);
    Sync();
    auto u32 = [&](size_t o, unsigned i) { return ((const uint32_t*)(h + o))[i]; };
    auto u16 = [&](size_t o, unsigned i) { return ((const uint16_t*)(h + o))[i]; };
    for (unsigned i = 0; i < n; i++) {
      UnpackOut& r = out[i];
      r.flow_id = u32(c4[0], i);
      r.seq_num = u32(c4[1], i);
      r.tx_sec = u32(c4[2], i);
      r.tx_usec = u32(c4[3], i);
      r.payload_off = u32(c4[5], i);
      r.lat_raw = u32(c4[6], i);
      r.lon_raw = u32(c4[7], i);
      r.alt = (int32_t)u32(c_alt, i);
      r.msg_len = u16(c2[0], i);
      r.dst_port = u16(c2[1], i);
      r.payload_len = u16(c2[2], i);
      r.hdr_len = u16(c2[3], i);
      r.host_port = u16(c2[4], i);
      r.flags = h[c1[0] + i];
      r.err = h[c1[1] + i];
      r.dst_type = h[c1[2] + i];
      r.dst_len = h[c1[3] + i];
      r.payload_type = h[c1[4] + i];
      r.gps_status = h[c1[5] + i];
      r.host_type = h[c1[6] + i];
      r.host_len = h[c1[7] + i];
      r.decoded = h[c1[8] + i];
      memcpy(r.dst_addr, h + c_da + 16u * i, 16);
      memcpy(r.host_addr, h + c_ha + 16u * i, 16);
    }
  }

  // ---- MgenMsg::ComputeCRC32 (mgenx_crc32_update) over n spans -------------------------
  void Crc32Update(const uint8_t* const* bufs, const uint32_t* lens, const uint32_t* state_in,
                   unsigned n, uint32_t* state_out) {
    if (n == 0) return;
    Init();
    if (n == 1 && crc_cache_.valid && state_in[0] == 0u && bufs[0] == crc_cache_.ptr &&
        lens[0] == crc_cache_.len && memcmp(bufs[0], crc_cache_.bytes.data(), lens[0]) == 0) {
      state_out[0] = crc_cache_.crc;  // computed with the Unpack of these bytes (above)
      crc_cache_.valid = false;
      return;
    }
    crc_cache_.valid = false;
    if (n == 1 && lens[0] <= MGENX_WORKER_MAX_BYTES && Worker()) {
      Check(mgenx_worker_crc32(worker_, bufs[0], lens[0], state_in[0], state_out),
            "mgenx_worker_crc32");
      return;
    }
    size_t bytes = 0;
    for (unsigned i = 0; i < n; i++) bytes += Align(lens[i], 16);
    Layout L;
    const size_t o_off = L.Add(n * 8u), o_len = L.Add(n * 4u), o_in = L.Add(n * 4u);
    const size_t o_data = L.Add(bytes + 16), in_bytes = L.size, o_out = L.Add(n * 4u);
    Reserve(L.size);
    uint8_t* h = host_;
    uint64_t* off = (uint64_t*)(h + o_off);
    size_t s = 0;
    for (unsigned i = 0; i < n; i++) {
      off[i] = s;
      ((uint32_t*)(h + o_len))[i] = lens[i];
      ((uint32_t*)(h + o_in))[i] = state_in[i];
      if (lens[i]) memcpy(h + o_data + s, bufs[i], lens[i]);
      s += Align(lens[i], 16);
    }
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    Check(mgenx_crc32_update(ctx_, g + o_data, (const uint64_t*)(g + o_off),
                             (const uint32_t*)(g + o_len), n, (const uint32_t*)(g + o_in),
                             (uint32_t*)(g + o_out), stream_),
          "mgenx_crc32_update");
    D2H(h + o_out, g + o_out, n * 4u);
    Sync();
    memcpy(state_out, h + o_out, n * 4u);
  }

  // ---- MgenAnalytic state slots (mgenx_flow_init / mgenx_flow_reduce) -----------------
  uint32_t FlowAlloc(double window) {
    Init();
    uint32_t slot;
    if (!free_slots_.empty()) {
      slot = free_slots_.back();
      free_slots_.pop_back();
    } else {
      slot = n_slots_++;
      if (n_slots_ > slot_cap_) GrowSlots(n_slots_ * 2 < 64 ? 64 : n_slots_ * 2);
    }
    Check(mgenx_flow_init(ctx_, flows_ + slot, 1, window, stream_), "mgenx_flow_init");
    Sync();
    return slot;
  }
  void FlowFree(uint32_t slot) { free_slots_.push_back(slot); }
  void FlowReinit(uint32_t slot, double window) {
    Init();
    Check(mgenx_flow_init(ctx_, flows_ + slot, 1, window, stream_), "mgenx_flow_init");
    Sync();
  }
  // records i < n (slot[i], rx, msgSize, tx, seq) in receive order; updated[i] = a window of
  // slot[i] closed at record i, with its report in rep[i]
  void FlowUpdate(const uint32_t* slot, const uint32_t* rx_sec, const uint32_t* rx_usec,
                  const uint16_t* msg_size, const uint32_t* tx_sec, const uint32_t* tx_usec,
                  const uint32_t* seq, unsigned n, bool* updated, mgenx_flow_report* rep) {
    if (n == 0) return;
    Init();
    if (n == 1 && Worker()) {  // one record (the per-message call): the resident worker
      uint32_t up = 0;
      Check(mgenx_worker_flow_update(worker_, flows_, slot[0], seq[0], rx_sec[0], rx_usec[0],
                                     msg_size[0], tx_sec[0], tx_usec[0], &up, &rep[0]),
            "mgenx_worker_flow_update");
      updated[0] = up != 0;
      return;
    }
    // one batch per run of distinct flows keeps "which record closed which window" exact:
    // a flow closes at most one window per record, and a chunk holds each flow once
    unsigned i0 = 0;
    while (i0 < n) {
      unsigned i1 = i0;
      std::vector<uint32_t> seen;
      while (i1 < n) {
        bool dup = false;
        for (uint32_t s2 : seen) dup |= (s2 == slot[i1]);
        if (dup) break;
        seen.push_back(slot[i1]);
        i1++;
      }
      FlowChunk(slot + i0, rx_sec + i0, rx_usec + i0, msg_size + i0, tx_sec + i0, tx_usec + i0,
                seq + i0, i1 - i0, updated + i0, rep + i0);
      i0 = i1;
    }
  }
  // the window end a flow slot holds now (MgenAnalytic::GetWindowEnd): one state read-back
  void FlowWindowEnd(uint32_t slot, int64_t* sec, int64_t* usec) {
    Init();
    Reserve(sizeof(mgenx_flow_state));
    D2H(host_, flows_ + slot, sizeof(mgenx_flow_state));
    Sync();
    const mgenx_flow_state* f = (const mgenx_flow_state*)host_;
    *sec = f->win_end_sec;
    *usec = f->win_end_usec;
  }

  // ---- event log lines through libmgenx's formatters (mgenx_log.hip) ------------------
  // RECV / RERR events (MgenMsg::LogRecvEvent / LogRecvError, mgenMsg.cpp:646-1143) of n
  // records: mgenx_log_recv_text or, binary, mgenx_log_recv_binary.  Returns the bytes.
  std::string LogRecv(const LogRecvIn* in, unsigned n, bool binary, int protocol, uint32_t opts) {
    if (n == 0) return std::string();
    Init();
    size_t slab = 0, cap = 0;
    for (unsigned i = 0; i < n; i++) {
      slab += Align(in[i].msg_bytes, 16);
      cap += 512 + 2u * in[i].msg_bytes;  // a line, or a binary record, fits this
    }
    Layout L;
    const size_t o_rows = L.Add(n * sizeof(mgenx_rec)), o_hdr = L.Add(n * 2u);
    const size_t o_hp = L.Add(n * 2u), o_ht = L.Add(n), o_hl = L.Add(n);
    const size_t o_da = L.Add(n * 16u), o_ha = L.Add(n * 16u), o_lat = L.Add(n * 4u);
    const size_t o_lon = L.Add(n * 4u), o_alt = L.Add(n * 4u), o_po = L.Add(n * 4u);
    const size_t o_src = L.Add(n * sizeof(mgenx_addr)), o_rxs = L.Add(n * 4u);
    const size_t o_rxu = L.Add(n * 4u), o_ttl = L.Add(n * 4u), o_off = L.Add(n * 8u);
    const size_t o_len = L.Add(n * 4u), o_slab = L.Add(slab + 16), in_bytes = L.size;
    const size_t o_pos = L.Add((n + 1) * 8u), o_text = L.Add(cap);
    Reserve(L.size);
    uint8_t* h = host_;
    bool any_ttl = false;
    size_t s = 0;
    for (unsigned i = 0; i < n; i++) {
      const LogRecvIn& r = in[i];
      ((mgenx_rec*)(h + o_rows))[i] = r.core;
      ((uint16_t*)(h + o_hdr))[i] = r.hdr_len;
      ((uint16_t*)(h + o_hp))[i] = r.host_port;
      h[o_ht + i] = r.host_type;
      h[o_hl + i] = r.host_len;
      memcpy(h + o_da + 16u * i, r.dst_addr, 16);
      memcpy(h + o_ha + 16u * i, r.host_addr, 16);
      ((uint32_t*)(h + o_lat))[i] = r.lat_raw;
      ((uint32_t*)(h + o_lon))[i] = r.lon_raw;
      ((int32_t*)(h + o_alt))[i] = r.alt;
      ((uint32_t*)(h + o_po))[i] = r.payload_off;
      ((mgenx_addr*)(h + o_src))[i] = r.src;
      ((uint32_t*)(h + o_rxs))[i] = r.rx_sec;
      ((uint32_t*)(h + o_rxu))[i] = r.rx_usec;
      ((int32_t*)(h + o_ttl))[i] = r.ttl;
      any_ttl |= r.ttl >= 0;
      ((uint64_t*)(h + o_off))[i] = s;
      ((uint32_t*)(h + o_len))[i] = r.msg_bytes;
      if (r.msg_bytes) memcpy(h + o_slab + s, r.msg, r.msg_bytes);
      s += Align(r.msg_bytes, 16);
    }
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    mgenx_cols c;
    memset(&c, 0, sizeof(c));
    c.rows = (mgenx_rec*)(g + o_rows);
    c.hdr_len = (uint16_t*)(g + o_hdr);
    c.host_port = (uint16_t*)(g + o_hp);
    c.host_type = g + o_ht;
    c.host_len = g + o_hl;
    c.dst_addr = g + o_da;
    c.host_addr = g + o_ha;
    c.lat_raw = (uint32_t*)(g + o_lat);
    c.lon_raw = (uint32_t*)(g + o_lon);
    c.alt = (int32_t*)(g + o_alt);
    c.payload_off = (uint32_t*)(g + o_po);
    const mgenx_addr* src = (const mgenx_addr*)(g + o_src);
    const uint32_t* rxs = (const uint32_t*)(g + o_rxs);
    const uint32_t* rxu = (const uint32_t*)(g + o_rxu);
    const uint64_t* off = (const uint64_t*)(g + o_off);
    uint64_t* pos = (uint64_t*)(g + o_pos);
    if (binary)
      Check(mgenx_log_recv_binary(ctx_, g + o_slab, slab + 16, off, 0, (const uint32_t*)(g + o_len),
                                  &c, src, rxs, rxu, n,
                                  protocol, g + o_text, cap, pos, stream_),
            "mgenx_log_recv_binary");
    else
      Check(mgenx_log_recv_text(ctx_, g + o_slab, off, 0, &c, src, rxs, rxu,
                                any_ttl ? (const int32_t*)(g + o_ttl) : nullptr, n, protocol,
                                opts, (char*)(g + o_text), cap, pos, stream_),
            "mgenx_log_recv_text");
    return ReadText(o_pos, n, o_text, cap);
  }

  // SEND events (MgenMsg::LogSendEvent, mgenMsg.cpp:1145-1241) of n messages described as a
  // pack template + descriptor each (the descriptor's tx time is the event time); binary:
  // the records carry each message's packed bytes (msg[i], msg_bytes[i]).
  std::string LogSend(const mgenx_flow_tmpl* tmpl, const mgenx_pack_desc* desc,
                      const uint16_t* src_port, const uint32_t* msg_total,
                      const uint8_t* const* msg, const uint32_t* msg_bytes, unsigned n,
                      bool binary, int protocol, uint32_t opts) {
    if (n == 0) return std::string();
    Init();
    size_t slab = 0, cap = 0;
    for (unsigned i = 0; i < n; i++) {
      const uint32_t b = binary ? msg_bytes[i] : 0u;
      slab += Align(b, 16);
      cap += 512 + b;
    }
    Layout L;
    const size_t o_t = L.Add(n * sizeof(mgenx_flow_tmpl)), o_d = L.Add(n * sizeof(mgenx_pack_desc));
    const size_t o_sp = L.Add(n * 2u), o_len = L.Add(n * 4u), o_tot = L.Add(n * 4u);
    const size_t o_off = L.Add(n * 8u), o_slab = L.Add(slab + 16), in_bytes = L.size;
    const size_t o_pos = L.Add((n + 1) * 8u), o_text = L.Add(cap);
    Reserve(L.size);
    uint8_t* h = host_;
    size_t s = 0;
    for (unsigned i = 0; i < n; i++) {
      ((mgenx_flow_tmpl*)(h + o_t))[i] = tmpl[i];
      mgenx_pack_desc d = desc[i];
      d.tmpl = i;
      ((mgenx_pack_desc*)(h + o_d))[i] = d;
      ((uint16_t*)(h + o_sp))[i] = src_port[i];
      ((uint32_t*)(h + o_len))[i] = binary ? msg_bytes[i] : 1u;  // "was sent"
      ((uint32_t*)(h + o_tot))[i] = msg_total[i];
      ((uint64_t*)(h + o_off))[i] = s;
      if (binary && msg_bytes[i]) memcpy(h + o_slab + s, msg[i], msg_bytes[i]);
      s += Align(binary ? msg_bytes[i] : 0u, 16);
    }
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    const mgenx_flow_tmpl* t = (const mgenx_flow_tmpl*)(g + o_t);
    const mgenx_pack_desc* d = (const mgenx_pack_desc*)(g + o_d);
    uint64_t* pos = (uint64_t*)(g + o_pos);
    if (binary)
      Check(mgenx_log_send_binary(ctx_, t, d, (const uint32_t*)(g + o_len),
                                  (const uint32_t*)(g + o_tot), g + o_slab, slab + 16,
                                  (const uint64_t*)(g + o_off), 0, n, protocol, g + o_text, cap,
                                  pos, stream_),
            "mgenx_log_send_binary");
    else
      Check(mgenx_log_send_text(ctx_, t, d, (const uint16_t*)(g + o_sp),
                                (const uint32_t*)(g + o_len), (const uint32_t*)(g + o_tot), n,
                                protocol, opts, (char*)(g + o_text), cap, pos, stream_),
            "mgenx_log_send_text");
    return ReadText(o_pos, n, o_text, cap);
  }

  // REPORT line of an analytic's last window (MgenAnalytic::Log, mgenAnalytic.cpp:260-295):
  // its report_msg bytes and the unquantized values; the timestamp is rep.rx_sec/usec.
  std::string LogReport(const uint8_t* item, unsigned item_len, const mgenx_flow_report& rep,
                        uint32_t opts) {
    Init();
    Layout L;
    const size_t o_item = L.Add(MGENX_REPORT_MAX), o_rep = L.Add(sizeof(mgenx_flow_report));
    const size_t o_cnt = L.Add(4), in_bytes = L.size, o_pos = L.Add(16), o_text = L.Add(1024);
    Reserve(L.size);
    uint8_t* h = host_;
    memset(h + o_item, 0, MGENX_REPORT_MAX);
    memcpy(h + o_item, item, item_len < MGENX_REPORT_MAX ? item_len : MGENX_REPORT_MAX);
    memcpy(h + o_rep, &rep, sizeof(rep));
    *(uint32_t*)(h + o_cnt) = 1;
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    Check(mgenx_log_report_text(ctx_, g + o_item, (const mgenx_flow_report*)(g + o_rep), 1, 1,
                                (const uint32_t*)(g + o_cnt), opts, (char*)(g + o_text), 1024,
                                (uint64_t*)(g + o_pos), stream_),
          "mgenx_log_report_text");
    return ReadText(o_pos, 1, o_text, 1024);
  }

  // REPORT line of a received report item (MgenAnalytic::Report::Log, mgenAnalytic.cpp:
  // 747-786): the item bytes, the reporter (the message's source) and the log time.
  std::string LogReportRecv(const uint8_t* item, unsigned item_len, const mgenx_addr& reporter,
                            uint32_t sec, uint32_t usec, uint32_t opts) {
    Init();
    Layout L;
    const size_t o_item = L.Add(MGENX_REPORT_MAX), o_pair = L.Add(16);
    const size_t o_src = L.Add(sizeof(mgenx_addr)), o_s = L.Add(4), o_u = L.Add(4);
    const size_t in_bytes = L.size, o_pos = L.Add(16), o_text = L.Add(1024);
    Reserve(L.size);
    uint8_t* h = host_;
    memset(h + o_item, 0, MGENX_REPORT_MAX);
    memcpy(h + o_item, item, item_len < MGENX_REPORT_MAX ? item_len : MGENX_REPORT_MAX);
    ((uint64_t*)(h + o_pair))[0] = 0;
    ((uint64_t*)(h + o_pair))[1] = 0;
    *(mgenx_addr*)(h + o_src) = reporter;
    *(uint32_t*)(h + o_s) = sec;
    *(uint32_t*)(h + o_u) = usec;
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    Check(mgenx_log_report_recv_text(ctx_, g + o_item, (const uint64_t*)(g + o_pair), 1,
                                     (const mgenx_addr*)(g + o_src), (const uint32_t*)(g + o_s),
                                     (const uint32_t*)(g + o_u), opts, (char*)(g + o_text), 1024,
                                     (uint64_t*)(g + o_pos), stream_),
          "mgenx_log_report_recv_text");
    return ReadText(o_pos, 1, o_text, 1024);
  }

  // MgenMsg::ConvertBinaryLog (mgenMsg.cpp:1417-1900) of a whole binary log image: the text
  // and the index status (MGENX_BINLOG_*).
  std::string ConvertBinaryLog(const uint8_t* file, size_t bytes, uint32_t flags, uint32_t opts,
                               int* status) {
    mgenx_binlog_info info;
    memset(&info, 0, sizeof(info));
    if (mgenx_binlog_index(file, bytes, nullptr, 0, &info) != MGENX_OK) {
      *status = MGENX_BINLOG_HEADER;
      return std::string();
    }
    *status = info.status;
    const uint64_t n = info.n_records;
    if (n == 0) return std::string();
    Init();
    std::vector<uint64_t> offs(n);
    mgenx_binlog_index(file, bytes, offs.data(), n, &info);
    // a converted line is at most a few hundred bytes plus twice a DATA payload (<= 1024)
    uint64_t cap = n * 2560u + 4096u;
    for (int attempt = 0;; attempt++) {
    Layout L;
    const size_t o_file = L.Add(bytes + 16), o_off = L.Add(n * 8u), in_bytes = L.size;
    const size_t o_pos = L.Add((n + 1) * 8u), o_text = L.Add(cap);
    Reserve(L.size);
    memcpy(host_ + o_file, file, bytes);
    memset(host_ + o_file + bytes, 0, 16);
    memcpy(host_ + o_off, offs.data(), n * 8u);
    uint8_t* g = dev_;
    H2D(g, host_, in_bytes);
    Check(mgenx_convert_binary_log(ctx_, g + o_file, bytes, (const uint64_t*)(g + o_off),
                                   (uint32_t)n, flags, opts, (char*)(g + o_text), cap,
                                   (uint64_t*)(g + o_pos), stream_),
          "mgenx_convert_binary_log");
    D2H(host_ + o_pos, g + o_pos, (n + 1) * 8u);
    Sync();
    const uint64_t total = ((const uint64_t*)(host_ + o_pos))[n];
    if (total > cap && attempt == 0) {  // many report lines: once more at the exact size
      cap = total;
      continue;
    }
    return ReadText(o_pos, (unsigned)n, o_text, cap);
    }
  }

  const mgenx_flow_state* DevFlows() const { return flows_; }
  mgenx_ctx* Ctx() {
    Init();
    return ctx_;
  }
  hipStream_t Stream() {
    Init();
    return stream_;
  }

 private:
  struct Layout {
    size_t size = 0;
    size_t Add(size_t bytes) {
      const size_t o = size;
      size += Align(bytes, 256);
      return o;
    }
  };
  static size_t Align(size_t v, size_t a) { return (v + a - 1) / a * a; }

  Engine() = default;
  ~Engine() {
    // process teardown: the HIP runtime may already be gone, so nothing is freed here
  }
  // the resident single-message worker (mgenx_worker_*), created on first use unless
  // MGENX_COMPAT_WORKER=0; stopped at exit (before the HIP runtime's own teardown, which
  // registered its handlers earlier)
  bool Worker() {
    if (worker_) return true;
    if (worker_off_) return false;
    const char* env = getenv("MGENX_COMPAT_WORKER");
    if ((env && atoi(env) == 0) || mgenx_worker_create(ctx_, 200, &worker_) != MGENX_OK) {
      worker_ = nullptr;
      worker_off_ = true;
      return false;
    }
    std::atexit([] { Get().StopWorker(); });
    return true;
  }
  void StopWorker() {
    if (worker_) mgenx_worker_destroy(worker_);
    worker_ = nullptr;
    worker_off_ = true;
  }
  void Init() {
    if (ctx_) return;
    const char* dv = getenv("MGENX_DEVICE");
    const int device = dv ? atoi(dv) : 0;
    if (hipSetDevice(device) != hipSuccess) throw Error("mgenx compat: no HIP device");
    if (mgenx_ctx_create(device, &ctx_) != MGENX_OK) throw Error("mgenx_ctx_create failed");
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess)
      throw Error("hipStreamCreate failed");
  }
  // a resident worker wave holds up the device-wide synchronisation of hipFree / hipHostFree
  // until it idles out: end it first (the next single-message call relaunches it)
  void QuiesceWorker() {
    if (worker_) (void)mgenx_worker_stop(worker_);
  }
  void Reserve(size_t bytes) {
    if (bytes <= cap_) return;
    size_t c = cap_ ? cap_ : (1u << 20);
    while (c < bytes) c *= 2;
    QuiesceWorker();
    if (host_) (void)hipHostFree(host_);
    if (dev_) (void)hipFree(dev_);
    host_ = nullptr;
    dev_ = nullptr;
    if (hipHostMalloc((void**)&host_, c) != hipSuccess || hipMalloc((void**)&dev_, c) != hipSuccess)
      throw Error("mgenx compat: staging allocation failed");
    cap_ = c;
  }
  void GrowSlots(uint32_t cap) {
    mgenx_flow_state* f = nullptr;
    if (hipMalloc((void**)&f, (size_t)cap * sizeof(mgenx_flow_state)) != hipSuccess)
      throw Error("mgenx compat: flow state allocation failed");
    if (flows_) {
      if (hipMemcpyAsync(f, flows_, (size_t)slot_cap_ * sizeof(mgenx_flow_state),
                         hipMemcpyDeviceToDevice, stream_) != hipSuccess)
        throw Error("mgenx compat: flow state copy failed");
      Sync();
      QuiesceWorker();
      (void)hipFree(flows_);
    }
    flows_ = f;
    slot_cap_ = cap;
  }
  void FlowChunk(const uint32_t* slot, const uint32_t* rx_sec, const uint32_t* rx_usec,
                 const uint16_t* msg_size, const uint32_t* tx_sec, const uint32_t* tx_usec,
                 const uint32_t* seq, unsigned n, bool* updated, mgenx_flow_report* rep) {
    Layout L;
    const size_t o_idx = L.Add(n * 4u), o_seq = L.Add(n * 4u), o_txs = L.Add(n * 4u);
    const size_t o_txu = L.Add(n * 4u), o_len = L.Add(n * 2u), o_rxs = L.Add(n * 4u);
    const size_t o_rxu = L.Add(n * 4u), o_cnt = L.Add((size_t)slot_cap_ * 4u);
    const size_t in_bytes = L.size;
    const size_t o_rep = L.Add((size_t)slot_cap_ * sizeof(mgenx_flow_report));
    Reserve(L.size);
    uint8_t* h = host_;
    memcpy(h + o_idx, slot, n * 4u);
    memcpy(h + o_seq, seq, n * 4u);
    memcpy(h + o_txs, tx_sec, n * 4u);
    memcpy(h + o_txu, tx_usec, n * 4u);
    memcpy(h + o_len, msg_size, n * 2u);
    memcpy(h + o_rxs, rx_sec, n * 4u);
    memcpy(h + o_rxu, rx_usec, n * 4u);
    memset(h + o_cnt, 0, (size_t)slot_cap_ * 4u);
    uint8_t* g = dev_;
    H2D(g, h, in_bytes);
    Check(mgenx_flow_reduce(ctx_, (const uint32_t*)(g + o_idx), (const uint32_t*)(g + o_seq),
                            (const uint32_t*)(g + o_txs), (const uint32_t*)(g + o_txu),
                            (const uint16_t*)(g + o_len), (const uint32_t*)(g + o_rxs),
                            (const uint32_t*)(g + o_rxu), n, flows_, slot_cap_,
                            (mgenx_flow_report*)(g + o_rep), 1, (uint32_t*)(g + o_cnt), stream_),
          "mgenx_flow_reduce");
    D2H(h + o_cnt, g + o_cnt, L.size - o_cnt);
    Sync();
    const uint32_t* cnt = (const uint32_t*)(h + o_cnt);
    const mgenx_flow_report* r = (const mgenx_flow_report*)(h + o_rep);
    for (unsigned i = 0; i < n; i++) {
      updated[i] = cnt[slot[i]] != 0;
      if (updated[i]) rep[i] = r[slot[i]];
    }
  }
  // the formatters' output: pos[n] bytes at o_text (throws when the capacity was short)
  std::string ReadText(size_t o_pos, unsigned n, size_t o_text, size_t cap) {
    D2H(host_ + o_pos, dev_ + o_pos, (n + 1) * 8u);
    Sync();
    const uint64_t total = ((const uint64_t*)(host_ + o_pos))[n];
    if (total > cap) throw Error("mgenx compat: log text larger than its staging capacity");
    D2H(host_ + o_text, dev_ + o_text, total);
    Sync();
    return std::string((const char*)host_ + o_text, total);
  }
  void H2D(void* d, const void* s, size_t b) {
    if (hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, stream_) != hipSuccess)
      throw Error("mgenx compat: H2D failed");
  }
  void D2H(void* d, const void* s, size_t b) {
    if (hipMemcpyAsync(d, s, b, hipMemcpyDeviceToHost, stream_) != hipSuccess)
      throw Error("mgenx compat: D2H failed");
  }
  void Sync() {
    if (hipStreamSynchronize(stream_) != hipSuccess) throw Error("mgenx compat: sync failed");
  }
  void Check(int rc, const char* what) {
    if (rc != MGENX_OK) {
      const char* m = mgenx_last_error(ctx_);
      throw Error(std::string(what) + " failed (" + std::to_string(rc) + ")" +
                  (m && *m ? std::string(": ") + m : std::string()));
    }
  }

  struct CrcCache {  // the receive checksum computed with the last single Unpack
    bool valid = false;
    const uint8_t* ptr = nullptr;
    uint32_t len = 0, crc = 0;
    std::vector<uint8_t> bytes;
  };

  std::mutex mu_;
  CrcCache crc_cache_;
  mgenx_ctx* ctx_ = nullptr;
  mgenx_worker* worker_ = nullptr;
  bool worker_off_ = false;
  hipStream_t stream_ = nullptr;
  uint8_t* host_ = nullptr;
  uint8_t* dev_ = nullptr;
  size_t cap_ = 0;
  mgenx_flow_state* flows_ = nullptr;
  uint32_t n_slots_ = 0, slot_cap_ = 0;
  std::vector<uint32_t> free_slots_;
};

}  // namespace compat
}  // namespace mgenx
