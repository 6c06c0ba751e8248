// mgenx_proto.h -- the few protolib types the MgenMsg / MgenPayload / MgenAnalytic shim's
// signatures name, for builds WITHOUT protolib (this repository's tests).
//
// Inside an MGEN build the real protolib provides ProtoAddress, ProtoTime, ProtoPkt and the
// UINT* typedefs (protokit.h), and mgenGlobals.h provides Protocol and the size constants:
// define MGENX_WITH_PROTOLIB and this header only includes those.  The shim uses nothing
// of ProtoAddress beyond what MgenMsg::Pack/Unpack use in the reference
// (src/common/mgenMsg.cpp:128-156, 396-430: GetType, GetLength, GetPort, SetPort,
// GetRawHostAddress, SetRawHostAddress, IsValid, Invalidate; GetHostString for the TCP
// connection events) and of ProtoTime beyond seconds/microseconds.
//
// Without protolib there is no Mgen either: the logging members (mgenx_compat.cpp) read the
// log file and its settings from an Mgen, so this header also carries the slice of the
// reference's Mgen (include/mgen.h:195-216) they use, plus the DrecEvent / MgenBaseEvent
// getters LogDrecEvent reads (include/mgenEvent.h).  Inside an MGEN build those are the real
// classes (mgen.h, mgenEvent.h).
#pragma once

#ifdef MGENX_WITH_PROTOLIB
#include "protokit.h"
#include "mgenGlobals.h"
#else

#include <arpa/inet.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/time.h>

typedef uint8_t UINT8;
typedef uint16_t UINT16;
typedef uint32_t UINT32;
typedef int8_t INT8;
typedef int16_t INT16;
typedef int32_t INT32;

#ifndef _MGEN_GLOBALS
#define _MGEN_GLOBALS
// the subset of include/mgenGlobals.h the shim's signatures use
enum Protocol { INVALID_PROTOCOL, UDP, TCP, SINK, SOURCE };
enum { MIN_SIZE = 28, MAX_SIZE = 8192, MSG_LEN_SIZE = 2, TX_BUFFER_SIZE = 8192,
       MAX_FRAG_SIZE = 65535, MIN_FRAG_SIZE = 76 };
enum MessageStatus { MSG_SEND_FAILED, MSG_SEND_BLOCKED, MSG_SEND_OK };
enum LogEventType {
  INVALID_EVENT = 0, RECV_EVENT, RERR_EVENT, SEND_EVENT, LISTEN_EVENT, IGNORE_EVENT, JOIN_EVENT,
  LEAVE_EVENT, START_EVENT, STOP_EVENT, ON_EVENT, ACCEPT_EVENT, DISCONNECT_EVENT, CONNECT_EVENT,
  OFF_EVENT, SHUTDOWN_EVENT, RECONNECT_EVENT
};
#endif

class ProtoAddress {
 public:
  enum Type { INVALID, IPv4, IPv6, ETH, SIM };
  ProtoAddress() { Invalidate(); }
  bool IsValid() const { return type_ != INVALID; }
  void Invalidate() {
    type_ = INVALID;
    len_ = 0;
    port_ = 0;
    memset(addr_, 0, sizeof(addr_));
  }
  Type GetType() const { return type_; }
  UINT8 GetLength() const { return len_; }
  UINT16 GetPort() const { return port_; }
  void SetPort(UINT16 p) { port_ = p; }
  const char* GetRawHostAddress() const { return (const char*)addr_; }
  // the length is kept as given (Unpack passes the wire byte, mgenMsg.cpp:394-396; how
  // protolib treats a length that does not match the type is not known here), the first
  // 16 bytes are stored
  bool SetRawHostAddress(Type t, const char* buf, unsigned len) {
    type_ = t;
    len_ = (UINT8)len;
    memset(addr_, 0, sizeof(addr_));
    if (buf && len) memcpy(addr_, buf, len > 16 ? 16 : len);
    return true;
  }
  // the text form MGEN logs (inet_ntop; "(invalid)" otherwise, as the device formatters)
  const char* GetHostString(char* buffer = nullptr, unsigned int buflen = 0) const {
    static thread_local char text[64];
    char* out = buffer ? buffer : text;
    const unsigned int cap = buffer ? buflen : (unsigned int)sizeof(text);
    const char* r = nullptr;
    if (type_ == IPv4 && len_ == 4) r = inet_ntop(AF_INET, addr_, out, cap);
    else if (type_ == IPv6 && len_ == 16) r = inet_ntop(AF_INET6, addr_, out, cap);
    if (!r && cap) snprintf(out, cap, "%s", "(invalid)");
    return out;
  }
  bool HostIsEqual(const ProtoAddress& o) const {
    return type_ == o.type_ && len_ == o.len_ && memcmp(addr_, o.addr_, len_) == 0;
  }
  bool IsEqual(const ProtoAddress& o) const { return HostIsEqual(o) && port_ == o.port_; }

 private:
  Type type_;
  UINT8 len_;
  UINT16 port_;
  UINT8 addr_[16];
};

class ProtoTime {
 public:
  ProtoTime() { tv_.tv_sec = 0; tv_.tv_usec = 0; }
  explicit ProtoTime(double seconds) {
    tv_.tv_sec = (long)seconds;
    tv_.tv_usec = (long)((seconds - (double)tv_.tv_sec) * 1.0e06 + 0.5);
  }
  ProtoTime(const struct timeval& tv) : tv_(tv) {}
  unsigned long sec() const { return (unsigned long)tv_.tv_sec; }
  unsigned long usec() const { return (unsigned long)tv_.tv_usec; }
  long GetSec() const { return tv_.tv_sec; }
  long GetUsec() const { return tv_.tv_usec; }
  const struct timeval& GetTimeVal() const { return tv_; }
  double GetValue() const { return (double)tv_.tv_sec + 1.0e-06 * (double)tv_.tv_usec; }

 private:
  struct timeval tv_;
};

inline void ProtoSystemTime(struct timeval& tv) { gettimeofday(&tv, nullptr); }

// the slice of Mgen (include/mgen.h:195-216) MgenMsg's logging members read
class Mgen {
 public:
  typedef int (*LogFunction)(FILE*, const char*, ...);
  static LogFunction Log;                                     // fprintf by default
  static void (*LogTimestamp)(FILE*, const struct timeval&, bool);
  static void SetEpochTimestamp(bool enable) {
    LogTimestamp = enable ? LogEpochTimestamp : LogLegacyTimestamp;
  }
  static void LogEpochTimestamp(FILE* f, const struct timeval& t, bool localTime);
  static void LogLegacyTimestamp(FILE* f, const struct timeval& t, bool localTime);

  FILE* GetLogFile() { return log_file; }
  bool GetLogBinary() { return log_binary; }
  bool GetLocalTime() { return local_time; }
  bool GetLogFlush() { return log_flush; }
  bool GetLogRx() { return log_rx; }
  bool GetLogData() { return log_data; }
  bool GetLogGpsData() { return log_gps_data; }
  bool GetOffsetPending() { return offset_pending; }
  // settings (the reference sets these from its commands, mgen.cpp:1545-2143)
  void SetLogFile(FILE* f) { log_file = f; }
  void SetLogBinary(bool v) { log_binary = v; }
  void SetLocalTime(bool v) { local_time = v; }
  void SetLogFlush(bool v) { log_flush = v; }
  void SetLogRx(bool v) { log_rx = v; }
  void SetLogData(bool v) { log_data = v; }
  void SetLogGpsData(bool v) { log_gps_data = v; }

 private:
  FILE* log_file = nullptr;
  bool log_binary = false, local_time = false, log_flush = false, log_rx = true;
  bool log_data = true, log_gps_data = true, offset_pending = false;
};

// the getters LogDrecEvent reads (include/mgenEvent.h: MgenBaseEvent, DrecEvent)
class MgenBaseEvent {
 public:
  static const char* GetStringFromProtocol(Protocol p) {  // mgenEvent.cpp:75-126
    return p == UDP ? "UDP" : p == TCP ? "TCP" : p == SINK ? "SINK" : "UNKNOWN";
  }
};
class DrecEvent : public MgenBaseEvent {
 public:
  Protocol GetProtocol() const { return protocol; }
  const ProtoAddress& GetGroupAddress() const { return group_addr; }
  const ProtoAddress& GetSourceAddress() const { return source_addr; }
  const char* GetInterface() const { return iface[0] ? iface : nullptr; }
  void SetProtocol(Protocol p) { protocol = p; }
  void SetGroupAddress(const ProtoAddress& a) { group_addr = a; }
  void SetSourceAddress(const ProtoAddress& a) { source_addr = a; }
  void SetInterface(const char* name) { snprintf(iface, sizeof(iface), "%s", name ? name : ""); }

 private:
  Protocol protocol = INVALID_PROTOCOL;
  ProtoAddress group_addr, source_addr;
  char iface[64] = {0};
};

// Byte-offset packet view (the ProtoPkt calls MgenDataItem and MgenAnalytic::Report make):
// Get/Set UINT8/16/32 at byte offsets, network byte order for the wider ones.
class ProtoPkt {
 public:
  ProtoPkt(UINT32* buf = nullptr, unsigned bytes = 0, bool freeOnDestruct = false)
      : buffer_(buf), buffer_bytes_(bytes), pkt_length_(0), owner_(freeOnDestruct) {}
  virtual ~ProtoPkt() {
    if (owner_ && buffer_) delete[] buffer_;
  }
  bool AttachBuffer(UINT32* buf, unsigned bytes, bool freeOnDestruct = false) {
    if (owner_ && buffer_ && buffer_ != buf) delete[] buffer_;
    buffer_ = buf;
    buffer_bytes_ = bytes;
    owner_ = freeOnDestruct;
    pkt_length_ = 0;
    return true;
  }
  bool InitFromBuffer(unsigned length, UINT32* buf = nullptr, unsigned bytes = 0,
                      bool freeOnDestruct = false) {
    if (buf) AttachBuffer(buf, bytes, freeOnDestruct);
    if (length > buffer_bytes_) {
      pkt_length_ = 0;
      return false;
    }
    pkt_length_ = length;
    return true;
  }
  unsigned GetBufferLength() const { return buffer_bytes_; }
  unsigned GetLength() const { return pkt_length_; }
  void SetLength(unsigned n) { pkt_length_ = n; }
  const UINT32* GetBuffer() const { return buffer_; }
  const char* GetBuffer(unsigned byteOffset) const { return (const char*)buffer_ + byteOffset; }
  void DetachBuffer() {
    buffer_ = nullptr;
    buffer_bytes_ = 0;
    pkt_length_ = 0;
    owner_ = false;
  }
  UINT32* AccessBuffer() { return buffer_; }
  char* AccessBuffer(unsigned byteOffset) { return (char*)buffer_ + byteOffset; }
  UINT8 GetUINT8(unsigned o) const { return ((const UINT8*)buffer_)[o]; }
  UINT16 GetUINT16(unsigned o) const {
    const UINT8* b = (const UINT8*)buffer_ + o;
    return (UINT16)((b[0] << 8) | b[1]);
  }
  UINT32 GetUINT32(unsigned o) const {
    const UINT8* b = (const UINT8*)buffer_ + o;
    return ((UINT32)b[0] << 24) | ((UINT32)b[1] << 16) | ((UINT32)b[2] << 8) | b[3];
  }
  void SetUINT8(unsigned o, UINT8 v) { ((UINT8*)buffer_)[o] = v; }
  void SetUINT16(unsigned o, UINT16 v) {
    UINT8* b = (UINT8*)buffer_ + o;
    b[0] = (UINT8)(v >> 8);
    b[1] = (UINT8)v;
  }
  void SetUINT32(unsigned o, UINT32 v) {
    UINT8* b = (UINT8*)buffer_ + o;
    b[0] = (UINT8)(v >> 24);
    b[1] = (UINT8)(v >> 16);
    b[2] = (UINT8)(v >> 8);
    b[3] = (UINT8)v;
  }

 protected:
  UINT32* buffer_;
  unsigned buffer_bytes_;
  unsigned pkt_length_;
  bool owner_;
};

#endif  // MGENX_WITH_PROTOLIB
