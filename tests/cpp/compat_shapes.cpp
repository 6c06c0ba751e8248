// compat_shapes.cpp -- the reference's own call shapes, compiled against the drop-in
// MgenMsg / MgenPayload / MgenAnalytic shim (include/mgenx_compat) and linked with
// libmgenx.  Driven by tests/test_compat_gpu.py, which feeds it the golden matrix and
// compares what it writes with the golden vectors and the oracle.
//
//   send     MgenUdpTransport::SendMessage   src/common/mgenTransport.cpp:1011-1031
//   receive  MgenUdpTransport::OnEvent(RECV) src/common/mgenTransport.cpp:955-975
//   analytic Mgen::UpdateRecvAnalytics        src/common/mgen.cpp:1027-1067
//   batch    the same three through MgenMsg::PackBatch / UnpackBatch and
//            MgenAnalytic::UpdateBatch (one GPU round trip per batch)
//   logging  (with <log dir>) the same sends and receives logged through the shim's
//            MgenMsg::LogSendEvent / LogRecvEvent / LogRecvError (text and binary, as
//            MgenTransport::LogEvent calls them, mgenTransport.cpp:328-482), the binary log
//            converted back by MgenMsg::ConvertBinaryLog, Mgen::UpdateRecvAnalytics' whole
//            body (mgen.cpp:1027-1068) incl. MgenAnalytic::Log and GetWindowEnd, and the TCP
//            connection / DREC events
//
// usage: compat_shapes <input file> <output file> [<log dir>]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "mgenAnalytic.h"
#include "mgenMsg.h"
#include "mgenPayload.h"
#ifdef MGENX_WITH_PROTOLIB  // inside an MGEN build these come from the application
#include "mgen.h"
#include "mgenEvent.h"
#endif

struct Reader {
  std::vector<uint8_t> buf;
  size_t pos = 0;
  template <typename T>
  T get() {
    T v;
    memcpy(&v, buf.data() + pos, sizeof(T));
    pos += sizeof(T);
    return v;
  }
  const uint8_t* take(size_t n) {
    const uint8_t* p = buf.data() + pos;
    pos += n;
    return p;
  }
};

#pragma pack(push, 1)
struct OutFields {  // numpy: tests/test_compat_gpu.py OUT_DTYPE
  uint8_t ok, err, version, flags;
  uint16_t msg_len, hdr_len;
  uint32_t flow_id, seq_num, tx_sec, tx_usec;
  uint16_t dst_port;
  uint8_t dst_type, dst_len;
  uint8_t dst_addr[16];
  uint16_t host_port;
  uint8_t host_type, host_len;
  uint8_t host_addr[16];
  double latitude, longitude;
  int32_t alt;
  uint8_t gps_status, payload_type;
  uint16_t payload_len;
  uint32_t payload_off;
};
struct OutReport {
  uint8_t updated, rsv[7];
  double duration, rate, loss, latency_ave, latency_min, latency_max;
  uint64_t msg_count;
  uint8_t report_item[MgenAnalytic::Report::MAX_LENGTH];
};
#pragma pack(pop)

static ProtoAddress make_addr(uint8_t type, uint8_t len, uint16_t port, const uint8_t* a) {
  ProtoAddress x;
  if (type == 1 || type == 2) {
    x.SetRawHostAddress(type == 1 ? ProtoAddress::IPv4 : ProtoAddress::IPv6, (const char*)a, len);
    x.SetPort(port);
  }
  return x;
}

// a double that MgenMsg::Pack turns into exactly `raw` ((UINT32)((deg + 180) * 60000))
static double degrees_for(uint32_t raw) {
  double d = (double)raw / 60000.0 - 180.0;
  for (int k = 0; k < 64 && (UINT32)((d + 180.0) * 60000.0) != raw; k++)
    d = nextafter(d, (UINT32)((d + 180.0) * 60000.0) < raw ? 1e9 : -1e9);
  return d;
}

// MgenFlow::SendMessage's per-message setup (mgenFlow.cpp:946-983, 1039-1129)
static void setup_msg(MgenMsg& m, const mgenx_flow_tmpl& t, const mgenx_pack_desc& d,
                      MgenPayload& payload, const uint8_t* pool) {
  m.SetProtocol(UDP);
  m.SetMsgLen(d.msg_len);
  m.SetFlowId(t.flow_id);
  m.SetSeqNum(d.seq_num);
  struct timeval tv;
  tv.tv_sec = d.tx_sec;
  tv.tv_usec = d.tx_usec;
  m.SetTxTime(tv);
  m.SetDstAddr(make_addr(t.dst_type, t.dst_len, t.dst_port, t.dst_addr));
  if (t.host_type) m.SetHostAddr(make_addr(t.host_type, t.host_len, t.host_port, t.host_addr));
  m.SetGPSLatitude(degrees_for(t.lat_raw));
  m.SetGPSLongitude(degrees_for(t.lon_raw));
  m.SetGPSAltitude(t.alt);
  m.SetGPSStatus((MgenMsg::GPSStatus)t.gps_status);
  if (t.has_payload) {
    payload.SetPayloadBytes((char*)pool + t.payload_off, t.payload_len);
    m.SetPayload(MgenMsg::USER_DATA, payload.AccessPayloadBuffer(), payload.GetLength());
  }
  if (d.flags) m.SetFlag((MgenMsg::Flag)d.flags);
}

static void fields_of(MgenMsg& m, bool ok, const UINT32* buffer, OutFields& o) {
  memset(&o, 0, sizeof(o));
  o.ok = ok;
  o.err = (uint8_t)m.GetError();
  o.version = m.GetVersion();
  o.flags = m.GetFlagBits();
  o.msg_len = m.GetMsgLen();
  o.hdr_len = m.GetPacketHeaderLen();
  o.flow_id = m.GetFlowId();
  o.seq_num = m.GetSeqNum();
  o.tx_sec = (uint32_t)m.GetTxTime().tv_sec;
  o.tx_usec = (uint32_t)m.GetTxTime().tv_usec;
  const ProtoAddress& dst = m.GetDstAddr();
  o.dst_port = dst.GetPort();
  o.dst_type = dst.GetType() == ProtoAddress::IPv4 ? 1 : (dst.GetType() == ProtoAddress::IPv6 ? 2 : 0);
  o.dst_len = dst.GetLength();
  memcpy(o.dst_addr, dst.GetRawHostAddress(), o.dst_len > 16 ? 16 : o.dst_len);
  const ProtoAddress& host = m.GetHostAddr();
  if (host.IsValid()) {
    o.host_port = host.GetPort();
    o.host_type = host.GetType() == ProtoAddress::IPv4 ? 1 : 2;
    o.host_len = host.GetLength();
    memcpy(o.host_addr, host.GetRawHostAddress(), o.host_len > 16 ? 16 : o.host_len);
  }
  o.latitude = m.GetGPSLatitude();
  o.longitude = m.GetGPSLongitude();
  o.alt = m.GetGPSAltitude();
  o.gps_status = (uint8_t)m.GetGPSStatus();
  o.payload_type = (uint8_t)m.GetPayloadType();
  o.payload_len = m.GetPayloadLength();
  o.payload_off = m.GetPayloadData() ? (uint32_t)((const uint8_t*)m.GetPayloadData() - (const uint8_t*)buffer) : 0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <in> <out>\n", argv[0]);
    return 2;
  }
  Reader r;
  {
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    r.buf.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(r.buf.data(), 1, r.buf.size(), f) != r.buf.size()) return 2;
    fclose(f);
  }
  const uint32_t n_tmpl = r.get<uint32_t>(), pool_len = r.get<uint32_t>(), n_desc = r.get<uint32_t>();
  const uint32_t n_unp = r.get<uint32_t>();
  const uint64_t slab_bytes = r.get<uint64_t>(), unp_bytes = r.get<uint64_t>();
  const mgenx_flow_tmpl* tmpl = (const mgenx_flow_tmpl*)r.take(n_tmpl * sizeof(mgenx_flow_tmpl));
  const uint8_t* pool = r.take(pool_len);
  const mgenx_pack_desc* desc = (const mgenx_pack_desc*)r.take(n_desc * sizeof(mgenx_pack_desc));
  const uint64_t* offs = (const uint64_t*)r.take(n_desc * 8u);
  const uint64_t* uoffs = (const uint64_t*)r.take(n_unp * 8u);
  const uint32_t* ulens = (const uint32_t*)r.take(n_unp * 4u);
  const uint8_t* uslab = r.take(unp_bytes);
  const uint32_t n_an = r.get<uint32_t>();
  const double window = r.get<double>();
  const uint32_t* a_flow = (const uint32_t*)r.take(n_an * 4u);
  const uint32_t* a_seq = (const uint32_t*)r.take(n_an * 4u);
  const uint32_t* a_txs = (const uint32_t*)r.take(n_an * 4u);
  const uint32_t* a_txu = (const uint32_t*)r.take(n_an * 4u);
  const uint32_t* a_rxs = (const uint32_t*)r.take(n_an * 4u);
  const uint32_t* a_rxu = (const uint32_t*)r.take(n_an * 4u);
  const uint16_t* a_len = (const uint16_t*)r.take(n_an * 2u);

  FILE* out = fopen(argv[2], "wb");
  if (!out) return 2;
  const std::string logdir = argc > 3 ? argv[3] : "";
  auto lopen = [&](const char* name) -> FILE* {
    return logdir.empty() ? nullptr : fopen((logdir + "/" + name).c_str(), "wb");
  };
  FILE* send_txt = lopen("send.txt");
  FILE* send_bin = lopen("send.bin");

  // ---- send shape, message by message (mgenTransport.cpp:1011-1031), checksum off / on
  for (int ck = 0; ck < 2; ck++) {
    std::vector<uint8_t> slab(slab_bytes, 0);
    std::vector<uint32_t> lens(n_desc, 0);
    for (uint32_t i = 0; i < n_desc; i++) {
      MgenMsg theMsg;
      MgenPayload payload;
      setup_msg(theMsg, tmpl[desc[i].tmpl], desc[i], payload, pool);
      const bool checksumEnable = ck != 0;
      UINT32 txChecksum = 0;
      theMsg.SetFlag(MgenMsg::LAST_BUFFER);
      UINT32 txBuffer[MAX_SIZE / 4 + 1];
      unsigned int len = theMsg.Pack(txBuffer, theMsg.GetMsgLen(), checksumEnable, txChecksum);
      if (len == 0) continue;  // MSG_SEND_FAILED
      if (checksumEnable && theMsg.FlagIsSet(MgenMsg::CHECKSUM))
        theMsg.WriteChecksum(txChecksum, (unsigned char*)txBuffer, (UINT32)len);
      memcpy(slab.data() + offs[i], txBuffer, len);  // socket.SendTo(txBuffer, len, dst)
      lens[i] = len;
      if (ck && send_txt) {  // LogEvent(SEND_EVENT, &theMsg, txTime, txBuffer) (:1060, 328-350)
        theMsg.SetSrcAddr(make_addr(1, 4, 5001, (const uint8_t*)"\x7f\x00\x00\x01"));
        theMsg.LogSendEvent(send_txt, false, false, txBuffer, false, theMsg.GetTxTime());
        theMsg.LogSendEvent(send_bin, true, false, txBuffer, false, theMsg.GetTxTime());
      }
    }
    fwrite(lens.data(), 4, n_desc, out);
    fwrite(slab.data(), 1, slab_bytes, out);
  }

  // ---- the same sends as one batch (MgenMsg::PackBatch: the batched SendPendingMessage)
  {
    std::vector<MgenMsg> msgs(n_desc);
    std::vector<MgenPayload> payloads(n_desc);
    std::vector<MgenMsg*> mp(n_desc);
    std::vector<std::vector<UINT32>> bufs(n_desc, std::vector<UINT32>(MAX_SIZE / 4 + 1));
    std::vector<UINT32*> bp(n_desc);
    std::vector<UINT16> blen(n_desc), res(n_desc);
    std::vector<UINT32> txck(n_desc, 0);
    for (uint32_t i = 0; i < n_desc; i++) {
      setup_msg(msgs[i], tmpl[desc[i].tmpl], desc[i], payloads[i], pool);
      msgs[i].SetFlag(MgenMsg::LAST_BUFFER);
      mp[i] = &msgs[i];
      bp[i] = bufs[i].data();
      blen[i] = msgs[i].GetMsgLen();
    }
    MgenMsg::PackBatch(mp.data(), bp.data(), blen.data(), true, txck.data(), res.data(), n_desc);
    std::vector<uint8_t> slab(slab_bytes, 0);
    std::vector<uint32_t> lens(n_desc, 0);
    for (uint32_t i = 0; i < n_desc; i++) {
      if (!res[i]) continue;
      if (msgs[i].FlagIsSet(MgenMsg::CHECKSUM))
        MgenMsg::WriteChecksum(txck[i], (UINT8*)bp[i], res[i]);
      memcpy(slab.data() + offs[i], bp[i], res[i]);
      lens[i] = res[i];
    }
    fwrite(lens.data(), 4, n_desc, out);
    fwrite(slab.data(), 1, slab_bytes, out);
  }

  // ---- receive shape, datagram by datagram (mgenTransport.cpp:955-975), force off / on
  FILE* recv_txt = lopen("recv.txt");
  FILE* recv_bin = lopen("recv.bin");
  FILE* recv_local = lopen("recv_local.txt");
  FILE* recv_epoch = lopen("recv_epoch.txt");
  FILE* recv_ok = lopen("recv_ok.bin");  // a binary log of the good records, for ConvertBinaryLog
  if (recv_ok) {
    const char hdr[] = "mgen version=5.1.1 type=binary_log\n";
    fwrite(hdr, 1, sizeof(hdr), recv_ok);  // with its NUL (mgenMsg.cpp:1452-1463)
  }
  for (int force = 0; force < 2; force++) {
    std::vector<OutFields> o(n_unp);
    for (uint32_t i = 0; i < n_unp; i++) {
      UINT32 alignedBuffer[65536 / 4];
      memset(alignedBuffer, 0, sizeof(alignedBuffer));
      const unsigned int len = ulens[i];
      memcpy(alignedBuffer, uslab + uoffs[i], len);
      char* buffer = (char*)alignedBuffer;
      ProtoAddress srcAddr = make_addr(1, 4, 59273, (const uint8_t*)"\x7f\x00\x00\x01");
      MgenMsg theMsg;
      theMsg.SetSrcAddr(srcAddr);
      const bool ok = theMsg.Unpack(alignedBuffer, (UINT16)len, force != 0, true);
      if (ok) {
        if (force || theMsg.FlagIsSet(MgenMsg::CHECKSUM)) {
          UINT32 checksum = 0;
          theMsg.ComputeCRC32(checksum, (unsigned char*)buffer, len - 4);
          checksum = (checksum ^ theMsg.CRC32_XOROT);
          UINT32 recvdChecksum;
          memcpy(&recvdChecksum, buffer + len - 4, 4);
          recvdChecksum = ntohl(recvdChecksum);
          if (checksum != recvdChecksum) theMsg.SetChecksumError();
        }
      }
      fields_of(theMsg, ok, alignedBuffer, o[i]);
      if (force == 0 && recv_txt) {
        // MgenUdpTransport::OnEvent's logging (mgenTransport.cpp:976-994 -> LogEvent)
        struct timeval now;
        now.tv_sec = 1700000001 + i / 1000;
        now.tv_usec = (i * 37) % 1000000;
        if (!ok || theMsg.GetError()) {
          theMsg.LogRecvError(recv_txt, false, false, false, now);
          theMsg.LogRecvError(recv_bin, true, false, false, now);
        } else {
          theMsg.SetProtocol(UDP);
          theMsg.LogRecvEvent(recv_txt, false, false, true, true, true, alignedBuffer, false, -1, now);
          if (i < 64) {  // local time (TZ of the test) and epoch timestamps
            theMsg.LogRecvEvent(recv_local, false, true, true, true, true, alignedBuffer, false, -1, now);
            Mgen::SetEpochTimestamp(true);
            theMsg.LogRecvEvent(recv_epoch, false, false, true, true, true, alignedBuffer, false, -1, now);
            Mgen::SetEpochTimestamp(false);
          }
          UINT32 copy[65536 / 4];
          memcpy(copy, alignedBuffer, sizeof(copy));
          theMsg.LogRecvEvent(recv_bin, true, false, true, true, true, alignedBuffer, false, -1, now);
          theMsg.LogRecvEvent(recv_ok, true, false, true, true, true, copy, false, -1, now);
        }
      }
    }
    fwrite(o.data(), sizeof(OutFields), n_unp, out);
  }

  // ---- the same receives as one batch (MgenMsg::UnpackBatch + ComputeCRC32Batch)
  {
    std::vector<MgenMsg> msgs(n_unp);
    std::vector<MgenMsg*> mp(n_unp);
    std::vector<std::vector<UINT32>> bufs(n_unp);
    std::vector<UINT32*> bp(n_unp);
    std::vector<UINT16> blen(n_unp);
    std::vector<uint8_t> okv(n_unp);
    bool* okb = new bool[n_unp];
    for (uint32_t i = 0; i < n_unp; i++) {
      bufs[i].resize((ulens[i] + 3) / 4 + 1);
      memcpy(bufs[i].data(), uslab + uoffs[i], ulens[i]);
      mp[i] = &msgs[i];
      bp[i] = bufs[i].data();
      blen[i] = (UINT16)ulens[i];
    }
    MgenMsg::UnpackBatch(mp.data(), bp.data(), blen.data(), okb, n_unp);
    std::vector<UINT32> ck;
    std::vector<const UINT8*> cb;
    std::vector<UINT32> cl;
    std::vector<uint32_t> who;
    for (uint32_t i = 0; i < n_unp; i++)
      if (okb[i] && msgs[i].FlagIsSet(MgenMsg::CHECKSUM)) {
        ck.push_back(0);
        cb.push_back((const UINT8*)bp[i]);
        cl.push_back(ulens[i] - 4);
        who.push_back(i);
      }
    MgenMsg::ComputeCRC32Batch(ck.data(), cb.data(), cl.data(), (unsigned)ck.size());
    for (size_t k = 0; k < who.size(); k++) {
      const uint32_t i = who[k];
      UINT32 recvd;
      memcpy(&recvd, (const uint8_t*)bp[i] + ulens[i] - 4, 4);
      if ((ck[k] ^ MgenMsg::CRC32_XOROT) != ntohl(recvd)) msgs[i].SetChecksumError();
    }
    std::vector<OutFields> o(n_unp);
    for (uint32_t i = 0; i < n_unp; i++) fields_of(msgs[i], okb[i], bp[i], o[i]);
    fwrite(o.data(), sizeof(OutFields), n_unp, out);
    delete[] okb;
  }

  // ---- analytics shape (mgen.cpp:1034-1067), record by record, then as one batch
  FILE* an_log = lopen("analytic.txt");
  FILE* an_end = lopen("window_end.bin");
  for (int batch = 0; batch < 2; batch++) {
    MgenAnalyticTable table;
    std::vector<MgenAnalytic*> owned;
    std::vector<OutReport> rep(n_an);
    memset(rep.data(), 0, rep.size() * sizeof(OutReport));
    ProtoAddress src = make_addr(1, 4, 5001, (const uint8_t*)"\x0a\x00\x00\x02");
    ProtoAddress dst = make_addr(1, 4, 5000, (const uint8_t*)"\x0a\x00\x00\x01");
    std::vector<MgenAnalytic*> items(n_an);
    for (uint32_t i = 0; i < n_an; i++) {
      MgenAnalytic* analytic = table.FindFlow(src, dst, a_flow[i]);
      if (nullptr == analytic) {
        analytic = new MgenAnalytic();
        if (!analytic->Init(UDP, src, dst, a_flow[i], window)) return 3;
        if (!table.Insert(*analytic)) return 3;
        owned.push_back(analytic);
      }
      items[i] = analytic;
    }
    std::vector<ProtoTime> rx(n_an), tx(n_an);
    std::vector<unsigned int> sz(n_an);
    for (uint32_t i = 0; i < n_an; i++) {
      struct timeval a, b;
      a.tv_sec = a_rxs[i];
      a.tv_usec = a_rxu[i];
      b.tv_sec = a_txs[i];
      b.tv_usec = a_txu[i];
      rx[i] = ProtoTime(a);
      tx[i] = ProtoTime(b);
      sz[i] = a_len[i];
    }
    std::vector<uint8_t> upd(n_an);
    if (batch) {
      bool* u = new bool[n_an];
      // reports of one batch: read each flow's report right after its own record
      MgenAnalytic::UpdateBatch(items.data(), rx.data(), sz.data(), tx.data(), a_seq, u, n_an);
      for (uint32_t i = 0; i < n_an; i++) upd[i] = u[i];
      delete[] u;
    }
    for (uint32_t i = 0; i < n_an; i++) {
      MgenAnalytic* analytic = items[i];
      const bool updated = batch ? upd[i] != 0
                                 : analytic->Update(rx[i], sz[i], tx[i], a_seq[i]);
      if (!updated) continue;
      OutReport& o = rep[i];
      if (batch) {
        // UpdateBatch applies a flow's later reports too; only its last report survives
        // in the object, so the batch run records the flags only
        o.updated = 1;
        continue;
      }
      const MgenAnalytic::Report& report = analytic->GetReport(rx[i]);
      if (an_log) analytic->Log(an_log, rx[i], rx[i], false);  // mgen.cpp:1067
      o.updated = 1;
      o.duration = analytic->GetReportDuration();
      o.rate = analytic->GetReportRateAverage();
      o.loss = analytic->GetReportLossFraction();
      o.latency_ave = analytic->GetReportLatencyAverage();
      o.latency_min = analytic->GetReportLatencyMin();
      o.latency_max = analytic->GetReportLatencyMax();
      o.msg_count = analytic->GetReportMessageCount();
      memcpy(o.report_item, report.GetBuffer(), report.GetLength() < sizeof(o.report_item) ? report.GetLength() : sizeof(o.report_item));
    }
    fwrite(rep.data(), sizeof(OutReport), n_an, out);
    if (!batch && an_end) {  // MgenAnalytic::GetWindowEnd of every flow, in creation order
      for (MgenAnalytic* a : owned) {
        const ProtoTime& e = a->GetWindowEnd();
        const int64_t v[2] = {(int64_t)e.GetTimeVal().tv_sec, (int64_t)e.GetTimeVal().tv_usec};
        fwrite(v, 8, 2, an_end);
      }
    }
    for (MgenAnalytic* a : owned) delete a;
  }

  // ---- MgenPayload / MgenFlowCommand round trips (mgenPayload.cpp:24-73, 276-347)
  {
    MgenPayload p;
    p.SetPayloadString("abc");
    char* s = MgenPayload::GetPayloadString(p.GetPayloadBytes(), p.GetLength());
    fprintf(out, "%s|", s);
    delete[] s;
    p.SetPayloadString("fffeffff");
    s = MgenPayload::GetPayloadString(p.GetPayloadBytes(), p.GetLength());
    fprintf(out, "%s|", s);
    delete[] s;
    UINT32 cbuf[64];
    MgenFlowCommand cmd;
    cmd.InitIntoBuffer(MgenDataItem::DATA_ITEM_FLOW_CMD, cbuf, sizeof(cbuf));
    cmd.SetStatus(3, MgenFlowCommand::FLOW_SUSPEND);
    cmd.SetStatus(40, MgenFlowCommand::FLOW_RESET);
    cmd.SetStatus(17, MgenFlowCommand::FLOW_RESUME);
    fprintf(out, "%u %u %u %u %u|", (unsigned)cmd.GetStatus(3), (unsigned)cmd.GetStatus(40),
            (unsigned)cmd.GetStatus(17), (unsigned)cmd.GetStatus(5), cmd.GetMaxFlowId());
  }
  fclose(out);
  if (!logdir.empty()) {
    for (FILE* f : {send_txt, send_bin, recv_txt, recv_bin, recv_local, recv_epoch, recv_ok, an_log,
                    an_end})
      fclose(f);
    // ConvertBinaryLog of the good records' binary log (mgenMsg.cpp:1417-1900)
    Mgen mgen;
    FILE* conv = lopen("convert.txt");
    mgen.SetLogFile(conv);
    const bool cok = MgenMsg().ConvertBinaryLog((logdir + "/recv_ok.bin").c_str(), mgen);
    fprintf(conv, "#%d\n", cok ? 1 : 0);
    fclose(conv);
    // TCP connection events (mgenMsg.cpp:741-944) and DREC events (:1243-1415)
    FILE* ct = lopen("conn.txt");
    FILE* cb = lopen("conn.bin");
    const LogEventType evs[] = {ACCEPT_EVENT, ON_EVENT, CONNECT_EVENT, DISCONNECT_EVENT,
                                RECONNECT_EVENT, SHUTDOWN_EVENT, OFF_EVENT};
    struct timeval t0;
    t0.tv_sec = 1700000123;
    t0.tv_usec = 4567;
    for (int host = 0; host < 2; host++)
      for (int client = 0; client < 2; client++)
        for (LogEventType ev : evs) {
          MgenMsg m;
          m.SetFlowId(7 + host);
          m.SetDstAddr(make_addr(1, 4, 5000, (const uint8_t*)"\x0a\x00\x00\x01"));
          m.SetSrcAddr(make_addr(1, 4, 5001, (const uint8_t*)"\x0a\x00\x00\x02"));
          if (host) m.SetHostAddr(make_addr(2, 16, 6000, (const uint8_t*)"\x20\x01\x0d\xb8\0\0\0\0\0\0\0\0\0\0\0\x01"));
          m.LogTcpConnectionEvent(ct, false, false, false, ev, client != 0, t0);
          m.LogTcpConnectionEvent(cb, true, false, false, ev, client != 0, t0);
        }
    fclose(ct);
    fclose(cb);
    FILE* dt = lopen("drec.txt");
    FILE* db = lopen("drec.bin");
    for (int bin = 0; bin < 2; bin++) {
      Mgen dm;
      dm.SetLogFile(bin ? db : dt);
      dm.SetLogBinary(bin != 0);
      DrecEvent ev;
      ev.SetProtocol(UDP);
      MgenMsg().LogDrecEvent(LISTEN_EVENT, &ev, 5000, dm);
      ev.SetProtocol(TCP);
      MgenMsg().LogDrecEvent(IGNORE_EVENT, &ev, 5001, dm);
      ev.SetGroupAddress(make_addr(1, 4, 0, (const uint8_t*)"\xe0\x01\x02\x03"));
      ev.SetInterface("eth0");
      MgenMsg().LogDrecEvent(JOIN_EVENT, &ev, 5002, dm);
      ev.SetSourceAddress(make_addr(1, 4, 0, (const uint8_t*)"\x0a\x00\x00\x09"));
      ev.SetInterface(nullptr);
      MgenMsg().LogDrecEvent(LEAVE_EVENT, &ev, 0, dm);
    }
    fclose(dt);
    fclose(db);
  }
  printf("compat_shapes: %u sends x 3, %u receives x 3, %u analytic updates x 2\n", n_desc, n_unp,
         n_an);
  return 0;
}
