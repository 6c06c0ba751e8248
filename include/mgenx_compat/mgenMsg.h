// mgenMsg.h -- drop-in MgenMsg over libmgenx (the MI355X engine).
//
// Same class, enums, members and signatures as the reference's include/mgenMsg.h:54-240,
// so MgenFlow, MgenTransport and pcap2mgen compile against it unchanged; the codec runs on
// the GPU:
//   Pack(UINT32*, UINT16, bool, UINT32&)   include/mgenMsg.h:108 -> mgenx_pack_msgs
//   Unpack(UINT32*, UINT16, bool, bool)    include/mgenMsg.h:110 -> mgenx_unpack_batch
//                                                                  (MGENX_OPT_SKIP_CRC)
//   static ComputeCRC32(UINT32&, ...)      include/mgenMsg.h:201 -> mgenx_crc32_update
//   static WriteChecksum(UINT32&, ...)     include/mgenMsg.h:111    (4-byte host store)
// plus the batch forms the batched transports call (PackBatch / UnpackBatch /
// ComputeCRC32Batch): one GPU round trip for many messages, with exactly the per-message
// results.  Single-message calls are batches of one (mgenx_compat.hpp).
//
// Semantics are the reference's (src/common/mgenMsg.cpp:83-541), including the state an
// MgenMsg keeps across calls: Pack sets CHECKSUM and clears LAST_BUFFER in the flags member
// and assigns packet_header_len; Unpack assigns only the members it reaches (the
// MGENX_DEC_* mask) and leaves msg_error alone on success.  One documented difference:
// a Pack that returns 0 writes no bytes (the reference leaves a partial header behind).
//
// The logging members (LogRecvEvent ... ConvertBinaryLog, mgenMsg.cpp:646-1900) keep the
// reference's signatures and are defined in mgenx_compat.cpp (which an MGEN build compiles
// instead of src/common/mgenMsg.cpp): the per-message events through libmgenx's formatters
// (mgenx_log_recv_text / _binary, mgenx_log_send_text / _binary), the binary-log conversion
// through mgenx_convert_binary_log, the TCP connection and DREC events on the host.
#ifndef _MGEN_MESSAGE
#define _MGEN_MESSAGE

#include <arpa/inet.h>
#include <stdio.h>
#include <time.h>

#include "mgenPayload.h"
#include "mgenx_compat.hpp"
#include "mgenx_proto.h"

class Mgen;
class DrecEvent;

class MgenMsg {
  friend class MgenTcpTransport;  // for msg_len & mgen_msg_len

 public:
  enum { VERSION = 2 };
  enum Error { ERROR_NONE = 0, ERROR_VERSION, ERROR_CHECKSUM, ERROR_LENGTH, ERROR_DSTADDR };
  enum AddressType { INVALID_ADDRESS = 0, IPv4 = 1, IPv6 = 2 };
  enum GPSStatus { INVALID_GPS = 0, STALE = 1, CURRENT = 2 };
  enum Flag {
    CLEAR = 0x00, CONTINUES = 0x01, END_OF_MSG = 0x02, CHECKSUM = 0x04, LAST_BUFFER = 0x08,
    CHECKSUM_ERROR = 0x10
  };
  enum PayloadType { USER_DATA = 0, MGEN_DATA = 1 };

  MgenMsg()
      : msg_len(0), mgen_msg_len(0), version(VERSION), flags(0), packet_header_len(0),
        flow_id(0), seq_num(0), latitude(0.0), longitude(0.0), altitude(0),
        gps_status(INVALID_GPS), payload_type(USER_DATA), payload_len(0), payload_data(nullptr),
        protocol(INVALID_PROTOCOL), msg_error(ERROR_NONE), compute_crc(true) {
    tx_time.tv_sec = 0;
    tx_time.tv_usec = 0;
  }
  ~MgenMsg() {}

  UINT16 Pack(UINT32* buffer, UINT16 bufferLen, bool includeChecksum, UINT32& tx_checksum) {
    MgenMsg* self = this;
    UINT16 ret = 0;
    PackBatch(&self, &buffer, &bufferLen, includeChecksum, &tx_checksum, &ret, 1);
    return ret;
  }

  bool Unpack(UINT32* buffer, UINT16 bufferLen, bool forceChecksum, bool log_data) {
    // forceChecksum is unused by the reference's Unpack (mgenMsg.cpp:315-500); here it tells
    // the engine that the caller's receive path checksums next (mgenTransport.cpp:960-963)
    (void)log_data;
    MgenMsg* self = this;
    bool ok = false;
    UnpackBatch(&self, &buffer, &bufferLen, &ok, 1, forceChecksum);
    return ok;
  }

  static bool WriteChecksum(UINT32& tx_checksum, UINT8* buffer, UINT32 buflen) {
    if (buflen < 4) return false;  // mgenMsg.cpp:502-522
    tx_checksum ^= CRC32_XOROT;
    const UINT32 be = __builtin_bswap32(tx_checksum);
    tx_checksum = be;  // the reference leaves tx_checksum in network order
    memcpy(buffer + buflen - 4, &be, 4);
    return true;
  }

  // ---- batch forms (one GPU round trip for n messages) ----
  // results[i] = msgs[i]->Pack(buffers[i], bufferLens[i], includeChecksum, txChecksums[i])
  static void PackBatch(MgenMsg* const* msgs, UINT32* const* buffers, const UINT16* bufferLens,
                        bool includeChecksum, UINT32* txChecksums, UINT16* results, unsigned n);
  // results[i] = msgs[i]->Unpack(buffers[i], bufferLens[i], ...)
  static void UnpackBatch(MgenMsg* const* msgs, UINT32* const* buffers, const UINT16* bufferLens,
                          bool* results, unsigned n, bool forceChecksum = false);
  // checksums[i]: ComputeCRC32(checksums[i], buffers[i], lens[i])
  static void ComputeCRC32Batch(UINT32* checksums, const UINT8* const* buffers,
                                const UINT32* lens, unsigned n);

  bool FlagIsSet(MgenMsg::Flag theFlag) { return (0 != (flags & theFlag)); }
  UINT16 GetMsgLen() const { return msg_len; }
  unsigned int GetMgenMsgLen() const { return mgen_msg_len; }
  UINT32 GetFlowId() const { return flow_id; }
  unsigned int GetSeqNum() const { return seq_num; }
  const ProtoAddress& GetDstAddr() const { return dst_addr; }
  const ProtoAddress& GetHostAddr() const { return host_addr; }
  MgenMsg::Error GetError() { return msg_error; }
  void ClearError() { msg_error = ERROR_NONE; }
  void SetProtocol(Protocol theProtocol) { protocol = theProtocol; }
  Protocol GetProtocol() { return protocol; }
  void SetVersion(UINT8 value) { version = value; }
  void SetFlag(MgenMsg::Flag theFlag) { flags |= theFlag; }
  void ClearFlag(MgenMsg::Flag theFlag) {
    if (FlagIsSet(theFlag)) flags ^= theFlag;
  }
  void SetMsgLen(UINT16 msgLen) { msg_len = msgLen; }
  void SetMgenMsgLen(unsigned int mgenMsgLen) { mgen_msg_len = mgenMsgLen; }
  void SetFlowId(UINT32 flowId) { flow_id = flowId; }
  void SetSeqNum(UINT32 seqNum) { seq_num = seqNum; }
  void SetTxTime(const struct timeval& txTime) { tx_time = txTime; }
  const struct timeval& GetTxTime() { return tx_time; }
  void SetDstAddr(const ProtoAddress& dstAddr) { dst_addr = dstAddr; }
  void SetSrcAddr(const ProtoAddress& srcAddr) { src_addr = srcAddr; }
  ProtoAddress& GetSrcAddr() { return src_addr; }
  void SetHostAddr(const ProtoAddress& hostAddr) { host_addr = hostAddr; }
  void SetGPSLatitude(double value) { latitude = value; }
  void SetGPSLongitude(double value) { longitude = value; }
  void SetGPSAltitude(INT32 value) { altitude = value; }
  void SetGPSStatus(GPSStatus status) { gps_status = status; }
  void SetPayload(PayloadType type, UINT32* buffer, UINT16 len) {
    payload_type = type;
    payload_data = buffer;
    payload_len = len;
  }
  PayloadType GetPayloadType() const { return payload_type; }
  const UINT32* GetPayloadData() const { return payload_data; }
  UINT32* AccessPayloadData() const { return payload_data; }
  UINT16 GetPayloadLength() const { return payload_len; }
  void SetError(MgenMsg::Error error) { msg_error = error; }
  void SetChecksumError() { msg_error = ERROR_CHECKSUM; }
  bool ComputeCRC() { return compute_crc; }
  void ComputeCRC(bool theFlag) { compute_crc = theFlag; }

  // reference logging (mgenMsg.cpp:646-1900), unchanged signatures
  bool LogRecvEvent(FILE* logFile, bool logBinary, bool localTime, bool logRecv, bool logData,
                    bool logGpsFata, UINT32* alignedMsgBuffer, bool flush, int ttl,
                    const struct timeval& theTime);
  bool LogSendEvent(FILE* logFile, bool logBinary, bool local_time, UINT32* alignedMsgBuffer,
                    bool flush, const struct timeval& theTime);
  bool LogTcpConnectionEvent(FILE* logFile, bool logBinary, bool local_time, bool flush,
                             LogEventType eventType, bool isClient, const struct timeval& theTime);
  bool LogRecvError(FILE* logFile, bool logBinary, bool local_time, bool flush,
                    const struct timeval& theTime);
  void LogDrecEvent(LogEventType eventType, const DrecEvent* event, UINT16 portNumber, Mgen& mgen);
  bool ConvertBinaryLog(const char* path, Mgen& mgen);

  static void ComputeCRC32(UINT32& checksum, const UINT8* buffer, UINT32 buflen) {
    ComputeCRC32Batch(&checksum, &buffer, &buflen, 1);
  }
  static const UINT32 CRC32_XOROT = 0xFFFFFFFFu;

  // Extensions (not in the reference class): read access to members the reference only
  // reads inside its own logging code (mgenMsg.cpp:946-1241).
  UINT16 GetPacketHeaderLen() const { return packet_header_len; }
  UINT8 GetVersion() const { return version; }
  UINT8 GetFlagBits() const { return flags; }
  double GetGPSLatitude() const { return latitude; }
  double GetGPSLongitude() const { return longitude; }
  INT32 GetGPSAltitude() const { return altitude; }
  GPSStatus GetGPSStatus() const { return gps_status; }

 protected:
  UINT16 msg_len;
  unsigned int mgen_msg_len;

 private:
  static const UINT32 CRC32_XINIT = 0xFFFFFFFFu;

  UINT8 version;
  UINT8 flags;
  UINT16 packet_header_len;
  UINT32 flow_id;
  UINT32 seq_num;
  struct timeval tx_time;
  ProtoAddress dst_addr;
  ProtoAddress src_addr;
  ProtoAddress host_addr;
  double latitude;
  double longitude;
  INT32 altitude;
  GPSStatus gps_status;
  PayloadType payload_type;
  UINT16 payload_len;
  UINT32* payload_data;
  Protocol protocol;
  Error msg_error;
  bool compute_crc;

  enum { FLAGS_OFFSET = 3 };

  // this message's members as one log record (mgenx_compat.cpp)
  void FillLogRecord(mgenx::compat::LogRecvIn& r) const;

  static UINT8 WireType(ProtoAddress::Type t) {
    return t == ProtoAddress::IPv4 ? (UINT8)IPv4 : (t == ProtoAddress::IPv6 ? (UINT8)IPv6 : 0);
  }
  static ProtoAddress::Type AddrType(UINT8 t) {
    return t == IPv4 ? ProtoAddress::IPv4 : (t == IPv6 ? ProtoAddress::IPv6 : ProtoAddress::INVALID);
  }
};

inline void MgenMsg::PackBatch(MgenMsg* const* msgs, UINT32* const* buffers,
                               const UINT16* bufferLens, bool includeChecksum,
                               UINT32* txChecksums, UINT16* results, unsigned n) {
  using mgenx::compat::Engine;
  std::vector<mgenx::compat::PackIn> in(n);
  std::vector<mgenx::compat::PackOut> out(n);
  std::vector<uint8_t*> dst(n);
  for (unsigned i = 0; i < n; i++) {
    const MgenMsg& m = *msgs[i];
    mgenx::compat::PackIn& p = in[i];
    memset(&p, 0, sizeof(p));
    mgenx_flow_tmpl& t = p.tmpl;
    t.flow_id = m.flow_id;
    // dst (mgenMsg.cpp:127-157): an unsupported type makes the kernel return 0
    t.dst_type = WireType(m.dst_addr.GetType());
    t.dst_len = m.dst_addr.GetLength();
    t.dst_port = m.dst_addr.GetPort();
    memcpy(t.dst_addr, m.dst_addr.GetRawHostAddress(), t.dst_len > 16 ? 16 : t.dst_len);
    // host (:165-204): type IPv4/IPv6 or invalid
    if (m.host_addr.IsValid()) {
      t.host_type = WireType(m.host_addr.GetType());
      t.host_len = t.host_type ? m.host_addr.GetLength() : 0;
      t.host_port = m.host_addr.GetPort();
      memcpy(t.host_addr, m.host_addr.GetRawHostAddress(), t.host_len > 16 ? 16 : t.host_len);
    }
    // GPS words exactly as Pack computes them (:221-231)
    t.lat_raw = (UINT32)((m.latitude + 180.0) * 60000.0);
    t.lon_raw = (UINT32)((m.longitude + 180.0) * 60000.0);
    t.alt = m.altitude;
    t.gps_status = (uint8_t)m.gps_status;
    t.payload_type = (uint8_t)m.payload_type;
    t.payload_len = m.payload_len;
    t.has_payload = m.payload_data != nullptr ? 1 : 0;
    p.payload = (const uint8_t*)m.payload_data;
    p.desc.seq_num = m.seq_num;
    p.desc.tx_sec = (uint32_t)m.tx_time.tv_sec;
    p.desc.tx_usec = (uint32_t)m.tx_time.tv_usec;
    p.desc.msg_len = m.msg_len;
    p.desc.flags = m.flags;
    // version: the kernel writes VERSION; a message set to another version is packed as the
    // reference would and read back as ERROR_VERSION by any receiver
    p.buf_len = bufferLens[i];
    p.crc_in = txChecksums[i];
    dst[i] = (uint8_t*)buffers[i];
  }
  uint32_t opts = includeChecksum ? MGENX_PACK_CHECKSUM : 0u;
  uint32_t fill_time = 0;
#ifdef RANDOM_FILL
  opts |= MGENX_PACK_RANDOM_FILL;  // srand(time(NULL)) per Pack (mgenMsg.cpp:282)
  fill_time = (uint32_t)time(nullptr);
#endif
  {
    std::lock_guard<std::mutex> g(Engine::Get().Lock());
    Engine::Get().Pack(in.data(), n, opts, fill_time, dst.data(), out.data());
  }
  for (unsigned i = 0; i < n; i++) {
    MgenMsg& m = *msgs[i];
    results[i] = (UINT16)out[i].ret;
    txChecksums[i] = out[i].tx_crc;
    if (out[i].ret) {
      m.packet_header_len = (UINT16)(out[i].state & 0xffffu);
      m.flags = (UINT8)(out[i].state >> 16);
    }
  }
}

inline void MgenMsg::UnpackBatch(MgenMsg* const* msgs, UINT32* const* buffers,
                                 const UINT16* bufferLens, bool* results, unsigned n,
                                 bool forceChecksum) {
  using mgenx::compat::Engine;
  std::vector<mgenx::compat::UnpackOut> out(n);
  std::vector<const uint8_t*> bufs(n);
  for (unsigned i = 0; i < n; i++) bufs[i] = (const uint8_t*)buffers[i];
  {
    std::lock_guard<std::mutex> g(Engine::Get().Lock());
    Engine::Get().Unpack(bufs.data(), bufferLens, n, out.data(), forceChecksum);
  }
  for (unsigned i = 0; i < n; i++) {
    MgenMsg& m = *msgs[i];
    const mgenx::compat::UnpackOut& r = out[i];
    // mgenMsg.cpp:318-319: every Unpack invalidates host_addr and gps_status first
    m.host_addr.Invalidate();
    m.gps_status = INVALID_GPS;
    const UINT8 dec = r.decoded;
    if (dec & MGENX_DEC_MSGLEN) {
      m.msg_len = r.msg_len;
      m.version = ((const UINT8*)buffers[i])[2];  // byte 2 as read (2 unless ERROR_VERSION)
    }
    if (dec & MGENX_DEC_BASE) {
      m.flags = r.flags;
      m.flow_id = r.flow_id;
      m.seq_num = r.seq_num;
      m.tx_time.tv_sec = (time_t)r.tx_sec;
      m.tx_time.tv_usec = (suseconds_t)r.tx_usec;
    }
    if (dec & MGENX_DEC_DST) {
      m.dst_addr.SetRawHostAddress(AddrType(r.dst_type), (const char*)r.dst_addr, r.dst_len);
      m.dst_addr.SetPort(r.dst_port);
    }
    if (dec & MGENX_DEC_HDRLEN) m.packet_header_len = r.hdr_len;
    if (dec & MGENX_DEC_HOST) {
      m.host_addr.SetRawHostAddress(AddrType(r.host_type), (const char*)r.host_addr, r.host_len);
      m.host_addr.SetPort(r.host_port);
    }
    if (dec & MGENX_DEC_GPS) {
      m.latitude = ((double)r.lat_raw) / 60000.0 - 180.0;  // mgenMsg.cpp:453,457
      m.longitude = ((double)r.lon_raw) / 60000.0 - 180.0;
      m.altitude = r.alt;
      m.gps_status = (GPSStatus)r.gps_status;
    }
    if (dec & MGENX_DEC_PTYPE) m.payload_type = (PayloadType)r.payload_type;
    if (dec & MGENX_DEC_PLEN) {
      m.payload_len = r.payload_len;
      m.payload_data = r.payload_len ? buffers[i] + r.payload_off / 4 : nullptr;
    }
    const bool ok = r.err == MGENX_ERROR_NONE;
    if (!ok) m.msg_error = (Error)r.err;
    results[i] = ok;
  }
}

inline void MgenMsg::ComputeCRC32Batch(UINT32* checksums, const UINT8* const* buffers,
                                       const UINT32* lens, unsigned n) {
  using mgenx::compat::Engine;
  std::lock_guard<std::mutex> g(Engine::Get().Lock());
  Engine::Get().Crc32Update(buffers, lens, checksums, n, checksums);
}

#endif  // _MGEN_MESSAGE
