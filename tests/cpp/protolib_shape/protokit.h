// TEST DOUBLE -- the shape of protolib's protokit.h as the MgenMsg / MgenAnalytic shim uses
// it inside an MGEN build (-DMGENX_WITH_PROTOLIB).  protolib is not vendored in the
// reference (an empty submodule), so this header carries only the members the reference's
// own call sites use (ProtoAddress: GetType/GetLength/GetPort/SetPort/GetRawHostAddress/
// SetRawHostAddress/IsValid/Invalidate/GetHostString; ProtoTime: GetTimeVal, the timeval and
// double constructors; ProtoPkt's field accessors; ProtoSystemTime).  It exists to compile
// and run the shim's protolib branch in tests/cpp/compat_shapes_pl; nothing ships with it.
#pragma once
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

class ProtoAddress {
 public:
  enum Type { INVALID, IPv4, IPv6, ETH, SIM };
  ProtoAddress() { Invalidate(); }
  bool IsValid() const { return type != INVALID; }
  void Invalidate() { type = INVALID; length = 0; port = 0; memset(raw, 0, sizeof(raw)); }
  Type GetType() const { return type; }
  UINT8 GetLength() const { return length; }
  UINT16 GetPort() const { return port; }
  void SetPort(UINT16 p) { port = p; }
  const char* GetRawHostAddress() const { return (const char*)raw; }
  bool SetRawHostAddress(Type t, const char* b, unsigned n) {
    type = t;
    length = (UINT8)n;
    memset(raw, 0, sizeof(raw));
    if (b && n) memcpy(raw, b, n > 16 ? 16 : n);
    return true;
  }
  const char* GetHostString(char* buffer = NULL, unsigned int buflen = 0) const {
    static char text[64];
    char* out = buffer ? buffer : text;
    const unsigned cap = buffer ? buflen : sizeof(text);
    const char* r = NULL;
    if (type == IPv4) r = inet_ntop(AF_INET, raw, out, cap);
    else if (type == IPv6) r = inet_ntop(AF_INET6, raw, out, cap);
    if (!r) snprintf(out, cap, "(invalid)");
    return out;
  }

 private:
  Type type;
  UINT8 length;
  UINT16 port;
  UINT8 raw[16];
};

class ProtoTime {
 public:
  ProtoTime() { tval.tv_sec = 0; tval.tv_usec = 0; }
  ProtoTime(const struct timeval& t) : tval(t) {}
  explicit ProtoTime(double s) {
    tval.tv_sec = (long)s;
    tval.tv_usec = (long)((s - (double)tval.tv_sec) * 1.0e06 + 0.5);
  }
  const struct timeval& GetTimeVal() const { return tval; }

 private:
  struct timeval tval;
};

inline void ProtoSystemTime(struct timeval& t) { gettimeofday(&t, NULL); }

class ProtoPkt {
 public:
  ProtoPkt(UINT32* b = NULL, unsigned n = 0, bool own = false)
      : buffer_ptr(b), buffer_bytes(n), pkt_length(0), owner(own) {}
  virtual ~ProtoPkt() { if (owner && buffer_ptr) delete[] buffer_ptr; }
  bool AttachBuffer(UINT32* b, unsigned n, bool own = false) {
    buffer_ptr = b; buffer_bytes = n; owner = own; pkt_length = 0;
    return true;
  }
  bool InitFromBuffer(unsigned len, UINT32* b = NULL, unsigned n = 0, bool own = false) {
    if (b) AttachBuffer(b, n, own);
    if (len > buffer_bytes) { pkt_length = 0; return false; }
    pkt_length = len;
    return true;
  }
  unsigned GetBufferLength() const { return buffer_bytes; }
  unsigned GetLength() const { return pkt_length; }
  void SetLength(unsigned n) { pkt_length = n; }
  const UINT32* GetBuffer() const { return buffer_ptr; }
  const char* GetBuffer(unsigned o) const { return (const char*)buffer_ptr + o; }
  void DetachBuffer() { buffer_ptr = NULL; buffer_bytes = 0; pkt_length = 0; owner = false; }
  UINT32* AccessBuffer() { return buffer_ptr; }
  char* AccessBuffer(unsigned o) { return (char*)buffer_ptr + o; }
  UINT8 GetUINT8(unsigned o) const { return ((const UINT8*)buffer_ptr)[o]; }
  UINT16 GetUINT16(unsigned o) const {
    UINT16 v;
    memcpy(&v, (const char*)buffer_ptr + o, 2);
    return ntohs(v);
  }
  UINT32 GetUINT32(unsigned o) const {
    UINT32 v;
    memcpy(&v, (const char*)buffer_ptr + o, 4);
    return ntohl(v);
  }
  void SetUINT8(unsigned o, UINT8 v) { ((UINT8*)buffer_ptr)[o] = v; }
  void SetUINT16(unsigned o, UINT16 v) { v = htons(v); memcpy((char*)buffer_ptr + o, &v, 2); }
  void SetUINT32(unsigned o, UINT32 v) { v = htonl(v); memcpy((char*)buffer_ptr + o, &v, 4); }

 private:
  UINT32* buffer_ptr;
  unsigned buffer_bytes, pkt_length;
  bool owner;
};
