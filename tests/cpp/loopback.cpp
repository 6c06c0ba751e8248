// loopback.cpp -- BASELINE config 1: one UDP flow PERIODIC [rate size] over loopback.
//
// Models doc/example.mgn:9 ("0.0 ON 1 UDP SRC 5001 DST 127.0.0.1/5000 PERIODIC [1000 1024]"
// with "LISTEN UDP 5000"), 10 s => 10,000 messages: MgenFlow::SendMessage (seq
// post-increment, tx time = now; src/common/mgenFlow.cpp:924-1130) -> the UDP send sequence
// (LAST_BUFFER, Pack, WriteChecksum; mgenTransport.cpp:1011-1031) -> sendmmsg -> loopback ->
// recvmmsg -> Unpack + CRC check (mgenTransport.cpp:948-975).  Ephemeral ports (5000/5001
// may be taken on a shared box); the dst field carries the listener's real port.
//
//   loopback cpu <count> <rate> <size>   the CPU reference path: the oracle restatement packs
//                                        and unpacks (test infrastructure; no GPU touched)
//   loopback gpu <count> <rate> <size>   the product path: mgenx SendBatch (GPU pack) and
//                                        RecvBatch (GPU unpack + CRC) around the same sockets
//   loopback ring <count> <rate> <size>  GPU pack, and RecvRing: received batches decoded on
//                                        the GPU while the run goes on (pinned stages, one
//                                        stream each, H2D / unpack / D2H overlapped)
//   ... [v6]                             the same over IPv6 loopback (::1)
// Prints one summary line; exit 0 iff every message arrived once, in order, intact.
#include <sys/time.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mgen_oracle.h"
#include "mgenx.hpp"
#include "mgenx_io.hpp"

static double now_s() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

struct Check {
  uint32_t n = 0, bad_seq = 0, bad_err = 0, bad_field = 0, bad_time = 0;
  void Add(uint32_t i, uint32_t seq, uint32_t err, bool fields_ok, bool time_ok) {
    n++;
    if (seq != i) bad_seq++;
    if (err) bad_err++;
    if (!fields_ok) bad_field++;
    if (!time_ok) bad_time++;
  }
};

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s cpu|gpu|ring count rate size [v6]\n", argv[0]);
    return 2;
  }
  const bool ring = std::string(argv[1]) == "ring";
  const bool gpu = ring || std::string(argv[1]) == "gpu";
  const bool v6 = argc > 5 && std::string(argv[5]) == "v6";
  const uint32_t count = (uint32_t)atoi(argv[2]);
  const double rate = atof(argv[3]);
  const uint32_t size = (uint32_t)atoi(argv[4]);
  const uint32_t slot = MGENX_MAX_SIZE;  // the reference's receive buffer (MAX_SIZE)

  mgenx::UdpTransport listener(v6 ? "::1" : "127.0.0.1", 0);
  mgenx::UdpTransport sender(v6 ? "::1" : "127.0.0.1", 0);
  const uint16_t dport = listener.Port();
  uint8_t dst_ip[16] = {127, 0, 0, 1};
  if (v6) {
    memset(dst_ip, 0, 16);
    dst_ip[15] = 1;
  }
  const uint8_t dst_len = v6 ? 16 : 4;

  // receive side: fixed slots (recvmmsg layout) + per-datagram length / source / rx time
  std::vector<uint8_t> cpu_slab(gpu ? 0 : (size_t)(count + 64) * slot);
  std::vector<uint32_t> lens(count + 64), rxs(count + 64), rxu(count + 64);
  std::vector<mgenx_addr> src(count + 64);
  std::vector<uint32_t> txs(count), txu(count);
  mgenx::Context* ctx = nullptr;
  mgenx::RecvBatch* rb = nullptr;
  mgenx::RecvRing* rr = nullptr;
  uint32_t ring_n = 0, ring_stages = 0, ring_overlap = 0;  // rows checked, stages, stages
                                                           // done while others were in flight
  mgenx::SendBatch* sb = nullptr;
  uint32_t flow = 0;
  if (gpu) {
    ctx = new mgenx::Context(0);
    if (ring) rr = new mgenx::RecvRing(*ctx, 256, slot, 3);
    else rb = new mgenx::RecvBatch(*ctx, count + 64, slot);
    sb = new mgenx::SendBatch(*ctx);
    flow = sb->AddFlow(1, v6 ? mgenx::IPv6 : mgenx::IPv4, dst_ip, dport);  // flow 1, GPS INVALID
  }
  Check c;
  auto time_ok = [&](uint32_t i, uint32_t s, uint32_t u, uint32_t rs, uint32_t ru) {
    const uint64_t tx = (uint64_t)txs[i] * 1000000u + txu[i];
    const uint64_t rx = (uint64_t)rs * 1000000u + ru;
    return s == txs[i] && u == txu[i] && rx >= tx;
  };
  auto fields_ok = [&](uint32_t flow_id, uint32_t msg_len, uint32_t port, const void* d4,
                       uint32_t gps, bool cks, bool last, uint32_t len, uint32_t sport) {
    return flow_id == 1 && msg_len == size && port == dport && memcmp(d4, dst_ip, 4) == 0 &&
           gps == 0 && cks && last && len == size && sport == sender.Port();
  };
  // RecvRing rows, checked in arrival order as the stages complete
  auto check_row = [&](const mgenx::RecvRing::Stage* d, uint32_t i) {
    const mgenx::MgenRecView v(d->rows[i]);
    const uint32_t d4 = v.GetDstAddr4();
    const uint32_t sq = v.GetSeqNum();
    const struct timeval tx = v.GetTxTime();
    c.Add(ring_n++, sq, v.GetError(),
          fields_ok(v.GetFlowId(), v.GetMsgLen(), v.GetDstPort(), &d4, v.GetGPSStatus(),
                    v.FlagIsSet(mgenx::CHECKSUM), v.FlagIsSet(mgenx::LAST_BUFFER), d->len[i],
                    d->src[i].port) && d->src[i].type == (v6 ? 2 : 1),
          sq < count && time_ok(sq, (uint32_t)tx.tv_sec, (uint32_t)tx.tv_usec, d->rx_sec[i],
                                d->rx_usec[i]));
  };
  std::vector<uint8_t> txbuf((size_t)64 * size);
  uint32_t sent = 0, got = 0, accepted = 0;  // accepted: datagrams the socket took
  const double t0 = now_s();
  while ((sent < count || got < count) && now_s() - t0 < count / rate + 5.0) {
    // PERIODIC: message k is due at t0 + k / rate
    const double t = now_s();
    uint32_t due = (uint32_t)((t - t0) * rate) + 1;
    if (due > count) due = count;
    if (due > sent + 64) due = sent + 64;
    if (due > sent) {
      const uint32_t k = due - sent;
      struct timeval tv;
      gettimeofday(&tv, nullptr);  // MgenFlow::SendMessage: tx time = now
      std::vector<uint32_t> plen(k);
      if (gpu) {
        sb->Clear();
        for (uint32_t j = 0; j < k; j++) sb->Add(flow, sent + j, tv, (uint16_t)size);
        const std::vector<uint32_t>& l = sb->Pack(true, false, 0, size);
        accepted += sender.Send(listener.Local(), sb->Datagram(0), size, l.data(), k);
      } else {
        for (uint32_t j = 0; j < k; j++) {
          or_msg m;
          memset(&m, 0, sizeof(m));
          m.msg_len = (uint16_t)size;
          m.mgen_msg_len = size;
          m.version = 2;
          m.flow_id = 1;
          m.seq_num = sent + j;
          m.tx_sec = (uint32_t)tv.tv_sec;
          m.tx_usec = (uint32_t)tv.tv_usec;
          m.dst.type = v6 ? 2 : 1; m.dst.len = dst_len; m.dst.port = dport;
          memcpy(m.dst.addr, dst_ip, dst_len);
          m.latitude = m.longitude = 999.0;
          m.altitude = -999;
          plen[j] = or_udp_pack(&m, txbuf.data() + (size_t)j * size, 1, 0, 0);
        }
        accepted += sender.Send(listener.Local(), txbuf.data(), size, plen.data(), k);
      }
      for (uint32_t j = 0; j < k; j++) { txs[sent + j] = (uint32_t)tv.tv_sec; txu[sent + j] = (uint32_t)tv.tv_usec; }
      sent += k;
    }
    // drain the listener (MgenUdpTransport::OnEvent's while (RecvFrom) loop, batched)
    if (ring) {
      for (;;) {
        if (rr->InFlight() == 3) break;  // every stage busy: decode first
        mgenx::RecvRing::Stage& st = rr->Fill();
        st.n = listener.Recv(st.slab, slot, rr->Batch(), st.len, st.src, st.rx_sec, st.rx_usec);
        if (!st.n) break;
        got += st.n;
        rr->Submit();
      }
      while (const mgenx::RecvRing::Stage* d = rr->Poll()) {
        ring_stages++;
        if (rr->InFlight() > 1) ring_overlap++;
        for (uint32_t i = 0; i < d->n; i++) check_row(d, i);
        rr->Release();
      }
    }
    for (; !ring;) {
      const uint32_t room = count + 64 - got;
      uint8_t* base = gpu ? rb->Slot(got) : cpu_slab.data() + (size_t)got * slot;
      const uint32_t r = listener.Recv(base, slot, room < 64 ? room : 64, &lens[got], &src[got],
                                       &rxs[got], &rxu[got]);
      if (!r) break;
      got += r;
    }
    if (sent >= count && got < count) {
      struct timespec ts = {0, 200000};
      nanosleep(&ts, nullptr);
    } else if (sent < count) {
      const double next = t0 + sent / rate;
      const double wait = next - now_s();
      if (wait > 0) {
        struct timespec ts = {0, (long)(wait * 1e9)};
        nanosleep(&ts, nullptr);
      }
    }
  }
  const double elapsed = now_s() - t0;

  // decode and check: seq 0..count-1 once each, in order; no error; fields as sent
  const uint32_t n = got < count ? got : count;
  if (ring) {
    while (const mgenx::RecvRing::Stage* d = rr->Wait()) {
      ring_stages++;
      for (uint32_t i = 0; i < d->n; i++) check_row(d, i);
      rr->Release();
    }
  } else if (gpu) {
    for (uint32_t i = 0; i < got; i++) rb->SetLength(i, lens[i]);
    rb->Unpack(got);
    for (uint32_t i = 0; i < n; i++) {
      const mgenx::MgenMsgView v = (*rb)[i];
      const uint32_t d4 = v.GetDstAddr4();
      const bool fields = fields_ok(v.GetFlowId(), v.GetMsgLen(), v.GetDstPort(), &d4,
                                    v.GetGPSStatus(), v.FlagIsSet(mgenx::CHECKSUM),
                                    v.FlagIsSet(mgenx::LAST_BUFFER), lens[i], src[i].port) &&
                          src[i].type == (v6 ? 2 : 1);
      const struct timeval tx = v.GetTxTime();
      c.Add(i, v.GetSeqNum(), v.GetError(), fields,
            time_ok(v.GetSeqNum() < count ? v.GetSeqNum() : 0, (uint32_t)tx.tv_sec,
                    (uint32_t)tx.tv_usec, rxs[i], rxu[i]));
    }
  } else {
    for (uint32_t i = 0; i < n; i++) {
      or_fields f;
      or_udp_recv(cpu_slab.data() + (size_t)i * slot, lens[i], 0, &f);
      const bool fields = fields_ok(f.flow_id, f.msg_len, f.dst_port, f.dst_addr, f.gps_status,
                                    (f.flags & OR_FLAG_CHECKSUM) != 0,
                                    (f.flags & OR_FLAG_LAST_BUFFER) != 0, lens[i],
                                    src[i].port) &&
                          f.dst_len == dst_len && src[i].type == (v6 ? 2 : 1);
      c.Add(i, f.seq_num, f.err, fields,
            time_ok(f.seq_num < count ? f.seq_num : 0, f.tx_sec, f.tx_usec, rxs[i], rxu[i]));
    }
  }
  const bool ok = sent == count && accepted == count && got == count && c.n == count &&
                  c.bad_seq == 0 && c.bad_err == 0 && c.bad_field == 0 && c.bad_time == 0;
  printf("{\"mode\": \"%s\", \"sent\": %u, \"send_failed\": %d, \"received\": %u, \"lost\": %d, \"out_of_order\": %u, "
         "\"errors\": %u, \"bad_fields\": %u, \"bad_times\": %u, \"elapsed_s\": %.3f, "
         "\"rate\": %.1f, \"size\": %u, \"v6\": %s, \"ring_stages\": %u, "
         "\"ring_overlapped\": %u, \"ok\": %s}\n",
         ring ? "ring" : gpu ? "gpu" : "cpu", sent, (int)sent - (int)accepted, got, (int)accepted - (int)got,
         c.bad_seq, c.bad_err,
         c.bad_field, c.bad_time, elapsed, rate, size, v6 ? "true" : "false", ring_stages,
         ring_overlap, ok ? "true" : "false");
  delete rr;
  delete sb;
  delete rb;
  delete ctx;
  return ok ? 0 : 1;
}
