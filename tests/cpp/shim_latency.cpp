// shim_latency.cpp -- per-call latency of the drop-in MgenMsg / MgenAnalytic shim: one Pack,
// Unpack, ComputeCRC32 or Update goes to the resident worker wave (mgenx_worker_*), so this
// measures what a transport that stays one-message-at-a-time pays per message: the UDP
// receive path's Unpack + ComputeCRC32(0, buf, len - 4) pair (mgenTransport.cpp:958-975, the
// checksum checked against the trailer here), MgenAnalytic::Update, Pack -- next to the batch
// forms (the recvmmsg / sendmmsg handoff) at n = 256 and 4096 per call.
// Prints one JSON object.  usage: shim_latency [iterations]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "mgenAnalytic.h"
#include "mgenMsg.h"
#include "mgenPayload.h"

using Clock = std::chrono::steady_clock;

static double median_us(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static void setup(MgenMsg& m, uint32_t seq) {
  m.SetProtocol(UDP);
  m.SetMsgLen(1024);
  m.SetFlowId(1);
  m.SetSeqNum(seq);
  struct timeval tv = {1700000000, (suseconds_t)seq};
  m.SetTxTime(tv);
  ProtoAddress dst;
  dst.SetRawHostAddress(ProtoAddress::IPv4, "\x7f\x00\x00\x01", 4);
  dst.SetPort(5000);
  m.SetDstAddr(dst);
  m.SetGPSLatitude(999.0);
  m.SetGPSLongitude(999.0);
  m.SetGPSAltitude(-999);
  m.SetFlag(MgenMsg::LAST_BUFFER);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  UINT32 buf[MAX_SIZE / 4 + 1];
  // warm up (context, staging, kernels)
  for (int i = 0; i < 50; i++) {
    MgenMsg m;
    setup(m, i);
    UINT32 ck = 0;
    m.Pack(buf, 1024, true, ck);
    MgenMsg r;
    r.Unpack(buf, 1024, false, false);
  }
  std::vector<double> pack, unpack, crc, recv, update;
  MgenAnalytic an;
  ProtoAddress s, d;
  s.SetRawHostAddress(ProtoAddress::IPv4, "\x0a\x00\x00\x02", 4);
  d.SetRawHostAddress(ProtoAddress::IPv4, "\x0a\x00\x00\x01", 4);
  an.Init(UDP, s, d, 1, 1.0);
  for (int i = 0; i < iters; i++) {
    MgenMsg m;
    setup(m, i);
    UINT32 ck = 0;
    auto t0 = Clock::now();
    const UINT16 len = m.Pack(buf, 1024, true, ck);
    auto t1 = Clock::now();
    if (m.FlagIsSet(MgenMsg::CHECKSUM)) MgenMsg::WriteChecksum(ck, (UINT8*)buf, len);
    MgenMsg r;
    auto t2 = Clock::now();
    const bool ok = r.Unpack(buf, len, false, false);
    auto t3 = Clock::now();
    UINT32 c = 0;
    MgenMsg::ComputeCRC32(c, (const UINT8*)buf, len - 4u);
    auto t4 = Clock::now();
    struct timeval rx = {1700000000, (suseconds_t)(i + 300)};
    an.Update(ProtoTime(rx), 1024, ProtoTime(r.GetTxTime()), r.GetSeqNum());
    auto t5 = Clock::now();
    UINT32 trailer;
    memcpy(&trailer, (const UINT8*)buf + len - 4u, 4);
    if (!ok || len != 1024 || (c ^ MgenMsg::CRC32_XOROT) != ntohl(trailer)) {
      fprintf(stderr, "bad round trip at %d\n", i);
      return 1;
    }
    pack.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    unpack.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
    crc.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
    recv.push_back(std::chrono::duration<double, std::micro>(t4 - t2).count());
    update.push_back(std::chrono::duration<double, std::micro>(t5 - t4).count());
  }
  // batch forms: per-message cost at n messages per call
  double batch_pack[2], batch_unpack[2];
  const unsigned ns[2] = {256, 4096};
  for (int k = 0; k < 2; k++) {
    const unsigned n = ns[k];
    std::vector<MgenMsg> msgs(n);
    std::vector<MgenMsg*> mp(n);
    std::vector<std::vector<UINT32>> bufs(n, std::vector<UINT32>(MAX_SIZE / 4 + 1));
    std::vector<UINT32*> bp(n);
    std::vector<UINT16> blen(n, 1024), res(n);
    std::vector<UINT32> txck(n);
    for (unsigned i = 0; i < n; i++) {
      setup(msgs[i], i);
      mp[i] = &msgs[i];
      bp[i] = bufs[i].data();
    }
    bool* okb = new bool[n];
    double tp = 1e30, tu = 1e30;
    for (int rep = 0; rep < 7; rep++) {
      std::fill(txck.begin(), txck.end(), 0u);
      auto t0 = Clock::now();
      MgenMsg::PackBatch(mp.data(), bp.data(), blen.data(), true, txck.data(), res.data(), n);
      auto t1 = Clock::now();
      std::vector<MgenMsg> rx(n);
      std::vector<MgenMsg*> rp(n);
      for (unsigned i = 0; i < n; i++) rp[i] = &rx[i];
      auto t2 = Clock::now();
      MgenMsg::UnpackBatch(rp.data(), bp.data(), blen.data(), okb, n);
      auto t3 = Clock::now();
      tp = std::min(tp, std::chrono::duration<double, std::micro>(t1 - t0).count());
      tu = std::min(tu, std::chrono::duration<double, std::micro>(t3 - t2).count());
    }
    delete[] okb;
    batch_pack[k] = tp / n;
    batch_unpack[k] = tu / n;
  }
  uint32_t wflags = 0;
  {
    mgenx_worker* w = nullptr;
    if (mgenx_worker_create(mgenx::compat::Engine::Get().Ctx(), 10, &w) == MGENX_OK) {
      mgenx_worker_info(w, &wflags);
      mgenx_worker_destroy(w);
    }
  }
  printf("{\"iterations\": %d, \"request_block\": \"%s\", "
         "\"single_call_median_us\": {\"pack\": %.2f, \"unpack\": %.2f, "
         "\"compute_crc32_after_unpack\": %.2f, \"recv_path_unpack_plus_crc\": %.2f, "
         "\"analytic_update\": %.2f}, "
         "\"batch_per_msg_us\": {\"pack_256\": %.3f, \"unpack_256\": %.3f, \"pack_4096\": %.3f, "
         "\"unpack_4096\": %.3f}}\n",
         iters, (wflags & MGENX_WORKER_DEVICE_MAILBOX) ? "device memory (BAR)" : "pinned host memory",
         median_us(pack), median_us(unpack), median_us(crc), median_us(recv), median_us(update),
         batch_pack[0], batch_unpack[0], batch_pack[1], batch_unpack[1]);
  return 0;
}
