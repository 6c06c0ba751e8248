// mgenx_compat.cpp -- the out-of-line half of the MgenMsg / MgenAnalytic shim: the logging
// members.  An MGEN build compiles this file in place of src/common/mgenMsg.cpp,
// src/common/mgenPayload.cpp and src/common/mgenAnalytic.cpp (the rest of those classes is
// inline in mgenMsg.h / mgenPayload.h / mgenAnalytic.h of this directory), with
// -DMGENX_WITH_PROTOLIB and this directory ahead of the reference's include/.
//
// The per-message events are formatted by libmgenx's gfx950 formatters -- the same kernels
// the batched transports use -- as batches of one:
//   LogRecvEvent / LogRecvError   mgenMsg.cpp:646-738, 946-1143  mgenx_log_recv_text / _binary
//   LogSendEvent                  mgenMsg.cpp:1145-1241          mgenx_log_send_text / _binary
//   MgenAnalytic::Log             mgenAnalytic.cpp:260-295       mgenx_log_report_text
//   MgenAnalytic::Report::Log     mgenAnalytic.cpp:747-786       mgenx_log_report_recv_text
//   ConvertBinaryLog              mgenMsg.cpp:1417-1900          mgenx_binlog_index + _convert
// The control-plane events (LogTcpConnectionEvent :741-944, one per TCP connection change,
// and LogDrecEvent :1243-1415, one per LISTEN / JOIN command) are host code, restated here.
//
// Timestamps: the device formatters print GMT "HH:MM:SS.usec" or, when Mgen::LogTimestamp
// is Mgen::LogEpochTimestamp, "sec.usec"; a local-time log (localTime) hands them each time
// shifted by its own UTC offset (localtime_r's tm_gmtoff), which gives localtime()'s fields.
// Text goes out through Mgen::Log (fprintf unless the application replaced it), binary
// records through fwrite, as in the reference.
#include <arpa/inet.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <functional>
#include <string>
#include <vector>

#include "mgenAnalytic.h"
#include "mgenMsg.h"
#include "mgenPayload.h"
#ifdef MGENX_WITH_PROTOLIB
#include "mgen.h"
#include "mgenEvent.h"
#endif

#ifndef MGENX_WITH_PROTOLIB
// ---- the Mgen slice of mgenx_proto.h (include/mgen.h:205-216, mgen.cpp:43-83) ----
Mgen::LogFunction Mgen::Log = fprintf;
void (*Mgen::LogTimestamp)(FILE*, const struct timeval&, bool) = Mgen::LogLegacyTimestamp;
void Mgen::LogEpochTimestamp(FILE* f, const struct timeval& t, bool) {
  Mgen::Log(f, "%lu.%06lu ", (unsigned long)t.tv_sec, (unsigned long)t.tv_usec);
}
void Mgen::LogLegacyTimestamp(FILE* f, const struct timeval& t, bool localTime) {
  const time_t secs = t.tv_sec;
  struct tm tmv;
  if (localTime) localtime_r(&secs, &tmv);
  else gmtime_r(&secs, &tmv);
  Mgen::Log(f, "%02d:%02d:%02d.%06lu ", tmv.tm_hour, tmv.tm_min, tmv.tm_sec,
            (unsigned long)(UINT32)t.tv_usec);
}
#endif

namespace {

using mgenx::compat::Engine;

bool EpochTimestamps() { return Mgen::LogTimestamp == Mgen::LogEpochTimestamp; }

// the seconds the device should print for `sec` (see the header comment)
uint32_t TsSec(time_t sec, bool localTime) {
  if (!localTime || EpochTimestamps()) return (uint32_t)sec;
  struct tm lt;
  localtime_r(&sec, &lt);
  return (uint32_t)(sec + lt.tm_gmtoff);
}

uint32_t LogOpts(bool logData, bool logGps) {
  return (EpochTimestamps() ? MGENX_LOG_EPOCH : 0u) | (logData ? 0u : MGENX_LOG_NO_DATA) |
         (logGps ? 0u : MGENX_LOG_NO_GPS);
}

void WriteText(FILE* f, const std::string& t) {
  if (!t.empty()) Mgen::Log(f, "%.*s", (int)t.size(), t.data());
}

bool WriteBinary(FILE* f, const std::string& b) {
  return b.empty() || fwrite(b.data(), 1, b.size(), f) == b.size();
}

uint8_t WireType(ProtoAddress::Type t) {
  return t == ProtoAddress::IPv4 ? 1u : (t == ProtoAddress::IPv6 ? 2u : 0u);
}

mgenx_addr AddrOf(const ProtoAddress& a) {
  mgenx_addr x;
  memset(&x, 0, sizeof(x));
  x.type = WireType(a.GetType());
  x.len = (uint8_t)a.GetLength();
  x.port = a.GetPort();
  memcpy(x.addr, a.GetRawHostAddress(), x.len > 16 ? 16 : x.len);
  return x;
}

// the wire word whose decode (raw / 60000.0 - 180.0, mgenMsg.cpp:453,457) is `deg`: exact
// for every value Unpack produced; other values print as the nearest 1/60000 degree
uint32_t RawDegrees(double deg) {
  const double x = (deg + 180.0) * 60000.0;
  uint32_t raw = (x <= 0.0) ? 0u : (x >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)llround(x));
  for (int k = -1; k <= 1; k++) {
    const uint32_t r = raw + (uint32_t)k;
    if ((double)r / 60000.0 - 180.0 == deg) return r;
  }
  return raw;
}

std::string Locked(const std::function<std::string(Engine&)>& f) {
  std::lock_guard<std::mutex> g(Engine::Get().Lock());
  return f(Engine::Get());
}

}  // namespace

// ---------------------------------------------------------------- MgenMsg
void MgenMsg::FillLogRecord(mgenx::compat::LogRecvIn& r) const {
  memset(&r, 0, sizeof(r));
  mgenx_rec& c = r.core;
  c.flow_id = flow_id;
  c.seq_num = seq_num;
  c.tx_sec = (uint32_t)tx_time.tv_sec;
  c.tx_usec = (uint32_t)tx_time.tv_usec;
  c.msg_len = msg_len;
  c.dst_port = dst_addr.GetPort();
  c.payload_len = payload_len;
  c.flags = flags;
  c.dst_type = WireType(dst_addr.GetType());
  c.dst_len = (uint8_t)dst_addr.GetLength();
  memcpy(&c.dst_addr4, dst_addr.GetRawHostAddress(), c.dst_len < 4 ? c.dst_len : 4);
  c.payload_type = (uint8_t)payload_type;
  c.gps_status = (uint8_t)gps_status;
  r.hdr_len = packet_header_len;
  memcpy(r.dst_addr, dst_addr.GetRawHostAddress(), c.dst_len > 16 ? 16 : c.dst_len);
  if (host_addr.IsValid()) {
    r.host_type = WireType(host_addr.GetType());
    r.host_len = (uint8_t)host_addr.GetLength();
    r.host_port = host_addr.GetPort();
    memcpy(r.host_addr, host_addr.GetRawHostAddress(), r.host_len > 16 ? 16 : r.host_len);
  }
  r.lat_raw = RawDegrees(latitude);
  r.lon_raw = RawDegrees(longitude);
  r.alt = altitude;
  r.src = AddrOf(src_addr);
  r.ttl = -1;
}

bool MgenMsg::LogRecvError(FILE* logFile, bool logBinary, bool localTime, bool flush,
                           const struct timeval& theTime) {
  mgenx::compat::LogRecvIn r;
  FillLogRecord(r);
  r.core.err = msg_error == ERROR_NONE ? (uint8_t)MGENX_ERROR_RERR_NONE : (uint8_t)msg_error;
  r.rx_sec = logBinary ? (uint32_t)theTime.tv_sec : TsSec(theTime.tv_sec, localTime);
  r.rx_usec = (uint32_t)theTime.tv_usec;
  const std::string out = Locked([&](Engine& e) {
    return e.LogRecv(&r, 1, logBinary, (int)protocol, LogOpts(true, true));
  });
  if (logBinary) {
    if (!WriteBinary(logFile, out)) return false;
  } else {
    WriteText(logFile, out);
  }
  if (flush) fflush(logFile);
  return true;
}

bool MgenMsg::LogRecvEvent(FILE* logFile, bool logBinary, bool localTime, bool logRx,
                           bool logData, bool logGpsData, UINT32* alignedMsgBuffer, bool flush,
                           int ttl, const struct timeval& theTime) {
  mgenx::compat::LogRecvIn r;
  FillLogRecord(r);
  r.ttl = ttl;
  if (logBinary) {
    // header + message bytes: packet_header_len + payload_len of the buffer (:968, 1016)
    r.rx_sec = (uint32_t)theTime.tv_sec;
    r.rx_usec = (uint32_t)theTime.tv_usec;
    r.core.msg_len = 0xFFFF;  // write the buffer's bytes as they are
    r.msg = (const uint8_t*)alignedMsgBuffer;
    r.msg_bytes = (uint32_t)(UINT16)(packet_header_len + payload_len);
    const std::string out = Locked([&](Engine& e) {
      return e.LogRecv(&r, 1, true, (int)protocol, 0u);
    });
    // the reference edits the caller's buffer as it writes it (:1019-1026)
    char* msgBuffer = (char*)alignedMsgBuffer;
    msgBuffer[FLAGS_OFFSET] &= ~CHECKSUM;
    if (FlagIsSet(CHECKSUM_ERROR)) msgBuffer[FLAGS_OFFSET] |= CHECKSUM_ERROR;
    if (!WriteBinary(logFile, out)) return false;
  } else {
    if (logRx) {
      r.rx_sec = TsSec(theTime.tv_sec, localTime);
      r.rx_usec = (uint32_t)theTime.tv_usec;
      r.core.tx_sec = TsSec(tx_time.tv_sec, localTime);
      if (payload_len && logData && payload_type == USER_DATA && payload_data) {
        r.msg = (const uint8_t*)payload_data;  // the DATA bytes, at offset 0 of the slab
        r.msg_bytes = payload_len;
      }
      const std::string line = Locked([&](Engine& e) {
        return e.LogRecv(&r, 1, false, (int)protocol, LogOpts(logData, logGpsData));
      });
      WriteText(logFile, line);
      if (gps_status != INVALID_GPS && gps_status != STALE && gps_status != CURRENT)
        return false;  // :1068-1071: the line ends early, nothing else is logged
    }
    if (MGEN_DATA == payload_type && payload_len > 0) {  // :1104-1137
      unsigned int bufferLen = payload_len;
      UINT32* bufferPtr = payload_data;
      while (bufferLen > 0) {
        if ((UINT8)MgenDataItem::GetItemType(bufferPtr) > 0x0f) {
          MgenAnalytic::Report report;
          if (!report.InitFromBuffer(bufferPtr, bufferLen)) break;  // invalid REPORT
          report.Log(logFile, ProtoTime(tx_time), ProtoTime(theTime), localTime, src_addr);
          const UINT8 reportLen = (UINT8)report.GetLength();
          if (0 == reportLen) break;
          bufferLen -= reportLen;
          bufferPtr += reportLen / sizeof(UINT32);
        } else {
          MgenDataItem item(bufferPtr, bufferLen);
          const UINT16 itemLen = (UINT16)item.GetLength();
          if (0 == itemLen) break;
          bufferLen -= itemLen;
          bufferPtr += itemLen / sizeof(UINT32);
        }
      }
    }
  }
  if (flush) fflush(logFile);
  return true;
}

bool MgenMsg::LogSendEvent(FILE* logFile, bool logBinary, bool localTime, UINT32* alignedMsgBuffer,
                           bool flush, const struct timeval& theTime) {
  mgenx_flow_tmpl t;
  memset(&t, 0, sizeof(t));
  t.flow_id = flow_id;
  t.dst_type = WireType(dst_addr.GetType());
  t.dst_len = (uint8_t)dst_addr.GetLength();
  t.dst_port = dst_addr.GetPort();
  memcpy(t.dst_addr, dst_addr.GetRawHostAddress(), t.dst_len > 16 ? 16 : t.dst_len);
  if (host_addr.IsValid()) {
    t.host_type = WireType(host_addr.GetType());
    t.host_len = (uint8_t)host_addr.GetLength();
    t.host_port = host_addr.GetPort();
    memcpy(t.host_addr, host_addr.GetRawHostAddress(), t.host_len > 16 ? 16 : t.host_len);
  }
  mgenx_pack_desc d;
  memset(&d, 0, sizeof(d));
  d.seq_num = seq_num;
  d.tx_sec = logBinary ? (uint32_t)theTime.tv_sec : TsSec(theTime.tv_sec, localTime);
  d.tx_usec = (uint32_t)theTime.tv_usec;
  d.msg_len = msg_len;
  d.flags = flags;
  const uint16_t sport = src_addr.GetPort();
  const uint32_t total = mgen_msg_len;
  // binary: recordLength - index + 4 message bytes (:1162-1199)
  uint32_t ml = 12u + dst_addr.GetLength() + packet_header_len;
  if (host_addr.IsValid()) ml += host_addr.GetLength() + 4u;
  ml &= 0xFFFFu;
  // the record reads past the packed message (recordLength counts the dst and host address
  // twice); those bytes are whatever the caller's buffer held -- written here as zeros, as
  // mgenx_log_send_binary writes them
  if (ml > msg_len) ml = msg_len;
  const uint8_t* mb = (const uint8_t*)alignedMsgBuffer;
  const std::string out = Locked([&](Engine& e) {
    return e.LogSend(&t, &d, &sport, &total, &mb, &ml, 1, logBinary, (int)protocol,
                     LogOpts(true, true));
  });
  if (logBinary) {
    ((char*)alignedMsgBuffer)[FLAGS_OFFSET] &= ~CHECKSUM;  // :1201-1203
    if (!WriteBinary(logFile, out)) return false;
  } else {
    WriteText(logFile, out);
  }
  if (flush) fflush(logFile);
  return true;
}

// TCP connection events (mgenMsg.cpp:741-944): host code, one per connection change
bool MgenMsg::LogTcpConnectionEvent(FILE* logFile, bool logBinary, bool localTime, bool flush,
                                    LogEventType eventType, bool isClient,
                                    const struct timeval& theTime) {
  SetProtocol(TCP);
  const ProtoAddress addr = GetDstAddr();
  if (logBinary) {
    std::vector<uint8_t> b;
    auto be16 = [&](UINT16 v) { b.push_back((uint8_t)(v >> 8)); b.push_back((uint8_t)v); };
    auto be32 = [&](UINT32 v) { be16((UINT16)(v >> 16)); be16((UINT16)v); };
    auto address = [&](const ProtoAddress& a) {
      b.push_back(WireType(a.GetType()));
      const unsigned len = a.GetLength();
      b.push_back((uint8_t)len);
      const uint8_t* raw = (const uint8_t*)a.GetRawHostAddress();
      b.insert(b.end(), raw, raw + len);
    };
    b.push_back((uint8_t)eventType);
    b.push_back((uint8_t)protocol);
    UINT16 recordLength = (UINT16)(12 + addr.GetLength() + 2 + 4);
    if (host_addr.IsValid()) recordLength = (UINT16)(recordLength + host_addr.GetLength() + 4);
    be16(recordLength);
    be32((UINT32)theTime.tv_sec);
    be32((UINT32)theTime.tv_usec);
    be16(addr.GetPort());
    address(addr);
    be16(src_addr.GetPort());  // "dstPort"
    be32(flow_id);
    if (host_addr.IsValid()) {
      be16(host_addr.GetPort());
      address(host_addr);
    }
    if (fwrite(b.data(), 1, b.size(), logFile) < b.size()) return false;
  } else {
    Mgen::LogTimestamp(logFile, theTime, localTime);
    const char* h = addr.GetHostString();
    const unsigned long fl = flow_id;
    const unsigned sp = src_addr.GetPort(), dp = addr.GetPort();
    switch (eventType) {
      case ACCEPT_EVENT:
        Mgen::Log(logFile, "ACCEPT src>%s/%hu dstPort>%hu", h, dp, sp);
        break;
      case ON_EVENT:
        Mgen::Log(logFile, "ON flow>%lu srcPort>%hu dst>%s/%hu ", fl, sp, h, dp);
        break;
      case CONNECT_EVENT:
        Mgen::Log(logFile, "CONNECT flow>%lu srcPort>%hu dst>%s/%hu ", fl, sp, h, dp);
        break;
      case DISCONNECT_EVENT:
        if (isClient) Mgen::Log(logFile, "DISCONNECT flow>%lu srcPort>%hu dst>%s/%hu ", fl, sp, h, dp);
        else Mgen::Log(logFile, "DISCONNECT src>%s/%hu dstPort>%hu ", h, dp, sp);
        break;
      case RECONNECT_EVENT:
        if (isClient) Mgen::Log(logFile, "RECONNECT flow>%lu srcPort>%hu dst>%s/%hu ", fl, sp, h, dp);
        else Mgen::Log(logFile, "RECONNECT src>%s/%hu dstPort>%hu ", h, dp, sp);
        break;
      case SHUTDOWN_EVENT:
        if (isClient) Mgen::Log(logFile, "SHUTDOWN flow>%lu srcPort>%hu dst>%s/%hu ", fl, sp, h, dp);
        else Mgen::Log(logFile, "SHUTDOWN src>%s/%hu dstPort>%hu", h, dp, sp);
        break;
      case OFF_EVENT:
        if (isClient) Mgen::Log(logFile, "OFF flow>%lu srcPort>%u dst>%s/%hu ", fl, sp, h, dp);
        else Mgen::Log(logFile, "OFF src>%s/%hu dstPort>%hu ", h, dp, sp);
        break;
      default:
        break;  // the reference asserts here
    }
    if (host_addr.IsValid())
      Mgen::Log(logFile, " host>%s/%hu\n", host_addr.GetHostString(), (unsigned)host_addr.GetPort());
    else
      Mgen::Log(logFile, "\n");
  }
  if (flush) fflush(logFile);
  return true;
}

// LISTEN / IGNORE / JOIN / LEAVE events (mgenMsg.cpp:1243-1415): host code, one per command
void MgenMsg::LogDrecEvent(LogEventType eventType, const DrecEvent* event, UINT16 portNumber,
                           Mgen& mgen) {
  FILE* logFile = mgen.GetLogFile();
  if (mgen.GetOffsetPending()) return;
  if (nullptr == logFile) return;
  struct timeval eventTime;
  ProtoSystemTime(eventTime);
  const bool localTime = mgen.GetLocalTime();
  if (mgen.GetLogBinary()) {
    std::vector<uint8_t> b(4, 0);
    b[0] = (uint8_t)eventType;
    auto be32 = [&](UINT32 v) {
      for (int k = 3; k >= 0; k--) b.push_back((uint8_t)(v >> (8 * k)));
    };
    be32((UINT32)eventTime.tv_sec);
    be32((UINT32)eventTime.tv_usec);
    switch (eventType) {
      case LISTEN_EVENT:
      case IGNORE_EVENT:
        b.push_back((uint8_t)event->GetProtocol());
        b.push_back(0);
        b.push_back((uint8_t)(portNumber >> 8));
        b.push_back((uint8_t)portNumber);
        break;
      case JOIN_EVENT:
      case LEAVE_EVENT: {
        // "groupPort" is copied in host byte order (:1294-1296)
        b.push_back((uint8_t)(portNumber & 0xff));
        b.push_back((uint8_t)(portNumber >> 8));
        const ProtoAddress& addr = event->GetGroupAddress();
        const uint8_t t = WireType(addr.GetType());
        if (!t) return;  // invalid address type: nothing is written
        b.push_back(t);
        const uint8_t len = (uint8_t)addr.GetLength();
        b.push_back(len);
        const uint8_t* raw = (const uint8_t*)addr.GetRawHostAddress();
        b.insert(b.end(), raw, raw + len);
        const char* iface = event->GetInterface();
        const uint8_t il = (uint8_t)(iface ? strlen(iface) : 0);
        b.push_back(il);
        if (il) b.insert(b.end(), iface, iface + il);
        break;
      }
      default:
        break;
    }
    const UINT16 rl = (UINT16)(b.size() - 4);
    b[2] = (uint8_t)(rl >> 8);
    b[3] = (uint8_t)rl;
    (void)fwrite(b.data(), 1, b.size(), logFile);
  } else {
    switch (eventType) {
      case LISTEN_EVENT:
      case IGNORE_EVENT:
        Mgen::LogTimestamp(logFile, eventTime, localTime);
        Mgen::Log(logFile, "%s proto>%s port>%hu\n", eventType == LISTEN_EVENT ? "LISTEN" : "IGNORE",
                  MgenBaseEvent::GetStringFromProtocol(event->GetProtocol()), (unsigned)portNumber);
        break;
      case JOIN_EVENT:
      case LEAVE_EVENT: {
        Mgen::LogTimestamp(logFile, eventTime, localTime);
        Mgen::Log(logFile, "%s group>%s", eventType == JOIN_EVENT ? "JOIN" : "LEAVE",
                  event->GetGroupAddress().GetHostString());
        if (event->GetSourceAddress().IsValid()) {  // SSM
          const char* source = event->GetSourceAddress().GetHostString();
          if (source) Mgen::Log(logFile, " source>%s", source);
        }
        const char* iface = event->GetInterface();
        if (iface) Mgen::Log(logFile, " interface>%s", iface);
        if (portNumber) Mgen::Log(logFile, " port>%hu\n", (unsigned)portNumber);
        else Mgen::Log(logFile, "\n");
        break;
      }
      default:
        break;
    }
  }
  if (mgen.GetLogFlush()) fflush(logFile);
}

bool MgenMsg::ConvertBinaryLog(const char* path, Mgen& mgen) {
  FILE* logFile = mgen.GetLogFile();
  if (nullptr == logFile) return false;
  FILE* file = fopen(path, "rb");
  if (!file) return false;
  std::vector<uint8_t> data;
  uint8_t chunk[1 << 16];
  size_t got;
  while ((got = fread(chunk, 1, sizeof(chunk), file)) > 0) data.insert(data.end(), chunk, chunk + got);
  fclose(file);
  const uint32_t flags = (mgen.GetLogRx() ? 0u : (uint32_t)MGENX_BINLOG_NO_RX) |
                         (mgen.GetLogFlush() ? (uint32_t)MGENX_BINLOG_FLUSH : 0u);
  (void)mgen.GetLocalTime();  // the converter prints GMT / epoch (localTime is not forwarded)
  int status = MGENX_BINLOG_HEADER;
  const std::string text = Locked([&](Engine& e) {
    return e.ConvertBinaryLog(data.data(), data.size(), flags,
                              LogOpts(mgen.GetLogData(), mgen.GetLogGpsData()), &status);
  });
  WriteText(logFile, text);
  if (mgen.GetLogFlush()) fflush(logFile);
  return status == MGENX_BINLOG_OK;
}

// ---------------------------------------------------------------- MgenAnalytic
void MgenAnalytic::Log(FILE* filePtr, const ProtoTime& sentTime, const ProtoTime& theTime,
                       bool localTime) const {
  (void)sentTime;
  if (nullptr == filePtr) return;
  mgenx_flow_report r;
  memset(&r, 0, sizeof(r));
  r.duration = report_duration;
  r.msg_count = report_msg_count;
  r.rate = report_rate_ave;
  r.loss = report_loss_ave;
  r.latency_ave = report_latency_ave;
  r.latency_min = report_latency_min;
  r.latency_max = report_latency_max;
  r.rx_sec = TsSec(theTime.GetTimeVal().tv_sec, localTime);
  r.rx_usec = (int64_t)theTime.GetTimeVal().tv_usec;
  const std::string line = Locked([&](Engine& e) {
    return e.LogReport((const uint8_t*)report_msg.GetBuffer(), report_msg.GetLength(), r,
                       LogOpts(true, true));
  });
  WriteText(filePtr, line);
}

const ProtoTime& MgenAnalytic::GetWindowEnd() const {
  int64_t s = 0, u = 0;
  if (slot_ != kNoSlot) {
    std::lock_guard<std::mutex> g(Engine::Get().Lock());
    Engine::Get().FlowWindowEnd(slot_, &s, &u);
  }
  struct timeval tv;
  tv.tv_sec = (time_t)s;
  tv.tv_usec = (suseconds_t)u;
  window_end_ = ProtoTime(tv);
  return window_end_;
}

void MgenAnalytic::Report::Log(FILE* filePtr, const ProtoTime& sentTime, const ProtoTime& theTime,
                               bool localTime, const ProtoAddress& reporterAddr) const {
  (void)sentTime;  // the reference prints theTime as "sent>" too (mgenAnalytic.cpp:781)
  if (nullptr == filePtr) return;
  const mgenx_addr rep = AddrOf(reporterAddr);
  const std::string line = Locked([&](Engine& e) {
    return e.LogReportRecv((const uint8_t*)GetBuffer(), GetLength(), rep,
                           TsSec(theTime.GetTimeVal().tv_sec, localTime),
                           (uint32_t)theTime.GetTimeVal().tv_usec,
                           LogOpts(true, true));
  });
  WriteText(filePtr, line);
}
