// mgenx.hpp -- C++ host layer over the mgenx C ABI (header-only, C++17, HIP runtime).
//
// Mirrors the reference's per-message C++ surface at batch granularity, so the batching
// points of mgenTransport / mgen read like the code they replace:
//   MgenMsgView    the getters of MgenMsg (include/mgenMsg.h:115-163) over one decoded
//                  record of a batch (GetMsgLen, GetFlowId, GetSeqNum, GetTxTime,
//                  FlagIsSet, GetError, GetPayloadLength ...), same meaning and values;
//   RecvBatch      MgenMsg::Unpack + the caller's CRC check for a recvmmsg-shaped batch
//                  (mgenTransport.cpp:948-997 UDP, :2092-2112 SINK, :1516-1564 TCP);
//   SendBatch      MgenFlow::SendMessage's fields (mgenFlow.cpp:924-1130) + MgenMsg::Pack
//                  + WriteChecksum in the UDP/SINK send order (mgenTransport.cpp:1011-1031);
//   FlowAnalytics  Mgen::UpdateRecvAnalytics (mgen.cpp:1027-1070): FindFlow by
//                  (src, dst, flow id) -> MgenAnalytic::Update per record, reports out;
//   ShardedScan    MgenTcpTransport / MgenAppSinkTransport framing (mgenTransport.cpp:
//                  1683-1760, mgenAppSinkTransport.cpp:369-434) of ONE stream split over the
//                  ranks of a job (the stitch protocol of include/mgenx.h, "sharded framing",
//                  over any ShardComm all-gather: RcclShardComm uses mgenx_allgather_u64).
// Errors: argument/launch failures throw mgenx::Error (the C ABI returns codes); per-record
// outcomes are MgenMsg::Error values, as in the reference.
#pragma once

#include <hip/hip_runtime_api.h>
#include <sys/time.h>

#include <cstdint>
#include <cstring>
#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "mgenx.h"

namespace mgenx {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}

// MgenMsg enums (include/mgenMsg.h:60-103)
enum MsgError { ERROR_NONE = 0, ERROR_VERSION, ERROR_CHECKSUM, ERROR_LENGTH, ERROR_DSTADDR };
enum MsgFlag : uint8_t {
  CONTINUES = 0x01, END_OF_MSG = 0x02, CHECKSUM = 0x04, LAST_BUFFER = 0x08,
  CHECKSUM_ERROR = 0x10
};
enum AddressType : uint8_t { INVALID_ADDRESS = 0, IPv4 = 1, IPv6 = 2 };

// ---- one mgenx context + stream per device -------------------------------------------
class Context {
 public:
  explicit Context(int device = 0) : device_(device) {
    check_hip(hipSetDevice(device), "hipSetDevice");
    if (mgenx_ctx_create(device, &ctx_) != MGENX_OK) throw Error("mgenx_ctx_create failed");
    check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  }
  ~Context() {
    if (stream_) (void)hipStreamDestroy(stream_);
    if (ctx_) mgenx_ctx_destroy(ctx_);
  }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  mgenx_ctx* get() const { return ctx_; }
  hipStream_t stream() const { return stream_; }
  int device() const { return device_; }
  void Sync() const { check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }
  void Check(int rc, const char* what) const {
    if (rc != MGENX_OK) {
      const char* m = mgenx_last_error(ctx_);
      throw Error(std::string(what) + " failed (" + std::to_string(rc) + ")" +
                  (m && *m ? std::string(": ") + m : std::string()));
    }
  }

 private:
  int device_;
  mgenx_ctx* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
};

// ---- RAII device / pinned-host arrays -------------------------------------------------
template <typename T>
class DeviceArray {
 public:
  DeviceArray() = default;
  explicit DeviceArray(size_t n) { Resize(n); }
  ~DeviceArray() { Free(); }
  DeviceArray(const DeviceArray&) = delete;
  DeviceArray& operator=(const DeviceArray&) = delete;
  DeviceArray(DeviceArray&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  void Resize(size_t n) {
    if (n == n_) return;
    Free();
    if (n) check_hip(hipMalloc((void**)&p_, n * sizeof(T)), "hipMalloc");
    n_ = n;
  }
  T* data() const { return p_; }
  size_t size() const { return n_; }

 private:
  void Free() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  T* p_ = nullptr;
  size_t n_ = 0;
};

template <typename T>
class PinnedArray {
 public:
  explicit PinnedArray(size_t n = 0) { Resize(n); }
  ~PinnedArray() {
    if (p_) (void)hipHostFree(p_);
  }
  PinnedArray(const PinnedArray&) = delete;
  PinnedArray& operator=(const PinnedArray&) = delete;
  void Resize(size_t n) {
    if (n == n_) return;
    if (p_) (void)hipHostFree(p_);
    p_ = nullptr;
    if (n) check_hip(hipHostMalloc((void**)&p_, n * sizeof(T)), "hipHostMalloc");
    n_ = n;
  }
  T* data() const { return p_; }
  T& operator[](size_t i) const { return p_[i]; }
  size_t size() const { return n_; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

// ---- decoded records ------------------------------------------------------------------
// Host copies of the core columns of one batch (32 B per record).
struct CoreColumns {
  std::vector<uint32_t> flow_id, seq_num, tx_sec, tx_usec, dst_addr4;
  std::vector<uint16_t> msg_len, dst_port, payload_len;
  std::vector<uint8_t> flags, err, dst_type, dst_len, payload_type, gps_status;
  void Resize(size_t n) {
    for (auto* v : {&flow_id, &seq_num, &tx_sec, &tx_usec, &dst_addr4}) v->resize(n);
    for (auto* v : {&msg_len, &dst_port, &payload_len}) v->resize(n);
    for (auto* v : {&flags, &err, &dst_type, &dst_len, &payload_type, &gps_status}) v->resize(n);
  }
};

// MgenMsg's getters over record i of a decoded batch (include/mgenMsg.h:115-163).
class MgenMsgView {
 public:
  MgenMsgView(const CoreColumns& c, size_t i) : c_(c), i_(i) {}
  uint16_t GetMsgLen() const { return c_.msg_len[i_]; }
  uint32_t GetFlowId() const { return c_.flow_id[i_]; }
  unsigned int GetSeqNum() const { return c_.seq_num[i_]; }
  struct timeval GetTxTime() const {
    struct timeval tv;
    tv.tv_sec = (time_t)c_.tx_sec[i_];
    tv.tv_usec = (suseconds_t)c_.tx_usec[i_];
    return tv;
  }
  bool FlagIsSet(uint8_t flag) const { return (c_.flags[i_] & flag) != 0; }
  MsgError GetError() const {  // MgenMsg::GetError; 0x80 (outside the slab) -> ERROR_LENGTH
    const uint8_t e = c_.err[i_];
    return e == MGENX_ERROR_OOB ? ERROR_LENGTH : (MsgError)e;
  }
  uint16_t GetDstPort() const { return c_.dst_port[i_]; }
  AddressType GetDstAddrType() const { return (AddressType)c_.dst_type[i_]; }
  uint8_t GetDstAddrLen() const { return c_.dst_len[i_]; }
  uint32_t GetDstAddr4() const { return c_.dst_addr4[i_]; }  // network byte order
  uint8_t GetPayloadType() const { return c_.payload_type[i_]; }
  uint16_t GetPayloadLength() const { return c_.payload_len[i_]; }
  uint8_t GetGPSStatus() const { return c_.gps_status[i_]; }

 private:
  const CoreColumns& c_;
  size_t i_;
};

// ---- receive: MgenMsg::Unpack + CRC check over a batch ---------------------------------
class RecvBatch {
 public:
  // capacity records in fixed slots of `slot` bytes (recvmmsg layout)
  RecvBatch(Context& ctx, uint32_t capacity, uint32_t slot = MGENX_MAX_SIZE)
      : ctx_(ctx), cap_(capacity), slot_(slot), h_slab_((size_t)capacity * slot),
        h_len_(capacity), d_slab_((size_t)capacity * slot), d_len_(capacity) {
    for (auto* a : {&d_flow_, &d_seq_, &d_txs_, &d_txu_, &d_dst4_}) a->Resize(capacity);
    for (auto* a : {&d_mlen_, &d_dport_, &d_plen_}) a->Resize(capacity);
    for (auto* a : {&d_flags_, &d_err_, &d_dtype_, &d_dlen_, &d_ptype_, &d_gps_}) a->Resize(capacity);
  }
  uint8_t* Slot(uint32_t i) { return h_slab_.data() + (size_t)i * slot_; }  // recv target
  void SetLength(uint32_t i, uint32_t len) { h_len_[i] = len; }
  uint32_t Capacity() const { return cap_; }

  // n received datagrams (lengths set): H2D, unpack + CRC check, core columns D2H.
  // forceChecksum = MgenTransport's checksum_force; tcp = MgenTcpTransport's rules.
  void Unpack(uint32_t n, bool forceChecksum = false, bool tcp = false) {
    if (n > cap_) throw Error("RecvBatch::Unpack: n > capacity");
    n_ = n;
    hipStream_t s = ctx_.stream();
    check_hip(hipMemcpyAsync(d_slab_.data(), h_slab_.data(), (size_t)n * slot_,
                             hipMemcpyHostToDevice, s), "H2D slab");
    check_hip(hipMemcpyAsync(d_len_.data(), h_len_.data(), (size_t)n * 4, hipMemcpyHostToDevice,
                             s), "H2D lengths");
    UnpackDevice(n, forceChecksum, tcp);
    Download();
  }
  // slab already in d_slab (device-resident path): decode only, columns stay on device
  void UnpackDevice(uint32_t n, bool forceChecksum = false, bool tcp = false) {
    n_ = n;
    mgenx_cols c;
    memset(&c, 0, sizeof(c));
    c.flow_id = d_flow_.data(); c.seq_num = d_seq_.data(); c.tx_sec = d_txs_.data();
    c.tx_usec = d_txu_.data(); c.dst_addr4 = d_dst4_.data(); c.msg_len = d_mlen_.data();
    c.dst_port = d_dport_.data(); c.payload_len = d_plen_.data(); c.flags = d_flags_.data();
    c.err = d_err_.data(); c.dst_type = d_dtype_.data(); c.dst_len = d_dlen_.data();
    c.payload_type = d_ptype_.data(); c.gps_status = d_gps_.data();
    const uint32_t opts = (forceChecksum ? MGENX_OPT_CHECKSUM_FORCE : 0) | (tcp ? MGENX_OPT_TCP : 0);
    ctx_.Check(mgenx_unpack_batch(ctx_.get(), d_slab_.data(), (uint64_t)n * slot_, nullptr, slot_,
                                  d_len_.data(), 0, n, &c, opts, ctx_.stream()),
               "mgenx_unpack_batch");
  }
  void Download() {
    cols_.Resize(n_);
    hipStream_t s = ctx_.stream();
    auto d2h = [&](auto& host, auto& dev) {
      check_hip(hipMemcpyAsync(host.data(), dev.data(), n_ * sizeof(host[0]),
                               hipMemcpyDeviceToHost, s), "D2H column");
    };
    d2h(cols_.flow_id, d_flow_); d2h(cols_.seq_num, d_seq_); d2h(cols_.tx_sec, d_txs_);
    d2h(cols_.tx_usec, d_txu_); d2h(cols_.dst_addr4, d_dst4_); d2h(cols_.msg_len, d_mlen_);
    d2h(cols_.dst_port, d_dport_); d2h(cols_.payload_len, d_plen_); d2h(cols_.flags, d_flags_);
    d2h(cols_.err, d_err_); d2h(cols_.dst_type, d_dtype_); d2h(cols_.dst_len, d_dlen_);
    d2h(cols_.payload_type, d_ptype_); d2h(cols_.gps_status, d_gps_);
    ctx_.Sync();
  }
  uint32_t Size() const { return n_; }
  MgenMsgView operator[](uint32_t i) const { return MgenMsgView(cols_, i); }
  const CoreColumns& Columns() const { return cols_; }
  // device columns for FlowAnalytics
  const uint32_t* DevSeq() const { return d_seq_.data(); }
  const uint32_t* DevTxSec() const { return d_txs_.data(); }
  const uint32_t* DevTxUsec() const { return d_txu_.data(); }
  const uint16_t* DevMsgLen() const { return d_mlen_.data(); }
  uint8_t* DevSlab() const { return d_slab_.data(); }

 private:
  Context& ctx_;
  uint32_t cap_, slot_, n_ = 0;
  PinnedArray<uint8_t> h_slab_;
  PinnedArray<uint32_t> h_len_;
  DeviceArray<uint8_t> d_slab_;
  DeviceArray<uint32_t> d_len_;
  DeviceArray<uint32_t> d_flow_, d_seq_, d_txs_, d_txu_, d_dst4_;
  DeviceArray<uint16_t> d_mlen_, d_dport_, d_plen_;
  DeviceArray<uint8_t> d_flags_, d_err_, d_dtype_, d_dlen_, d_ptype_, d_gps_;
  CoreColumns cols_;
};

// MgenMsg's getters over one decoded 32-B row (mgenx_rec), as MgenMsgView over columns.
class MgenRecView {
 public:
  explicit MgenRecView(const mgenx_rec& r) : r_(r) {}
  uint16_t GetMsgLen() const { return r_.msg_len; }
  uint32_t GetFlowId() const { return r_.flow_id; }
  unsigned int GetSeqNum() const { return r_.seq_num; }
  struct timeval GetTxTime() const {
    struct timeval tv;
    tv.tv_sec = (time_t)r_.tx_sec;
    tv.tv_usec = (suseconds_t)r_.tx_usec;
    return tv;
  }
  bool FlagIsSet(uint8_t flag) const { return (r_.flags & flag) != 0; }
  MsgError GetError() const { return r_.err == MGENX_ERROR_OOB ? ERROR_LENGTH : (MsgError)r_.err; }
  uint16_t GetDstPort() const { return r_.dst_port; }
  AddressType GetDstAddrType() const { return (AddressType)r_.dst_type; }
  uint8_t GetDstAddrLen() const { return r_.dst_len; }
  uint32_t GetDstAddr4() const { return r_.dst_addr4; }
  uint8_t GetPayloadType() const { return r_.payload_type; }
  uint16_t GetPayloadLength() const { return r_.payload_len; }
  uint8_t GetGPSStatus() const { return r_.gps_status; }

 private:
  const mgenx_rec& r_;
};

// ---- receive ring: socket batches overlapped with the GPU ------------------------------
// The reference's receive loop reads, decodes and checks one datagram at a time
// (MgenUdpTransport::OnEvent, mgenTransport.cpp:938-1000).  RecvRing keeps `depth` stages of
// pinned recvmmsg slots; while the socket layer fills stage k on the host, stage k-1's
// datagrams go H2D, through unpack + CRC check, and come back as 32-B rows, each stage on its
// own HIP stream (copies and kernels of different stages overlap):
//   Stage& s = ring.Fill();                        // the next free stage (host side)
//   s.n = sock.Recv(s.slab, ring.Slot(), ring.Batch(), s.len, s.src, s.rx_sec, s.rx_usec);
//   ring.Submit();                                 // async: H2D, unpack + CRC, rows D2H
//   while (const RecvRing::Stage* d = ring.Poll()) { ... d->rows[i] ...; ring.Release(); }
// Fill() needs a free stage: call Wait() / Release() for the oldest one when all are busy.
class RecvRing {
 public:
  struct Stage {
    uint8_t* slab = nullptr;        // pinned: Batch() slots of Slot() bytes
    uint32_t* len = nullptr;        // pinned: datagram lengths
    mgenx_addr* src = nullptr;      // pinned: recvfrom sources
    uint32_t* rx_sec = nullptr;     // pinned: receive times
    uint32_t* rx_usec = nullptr;
    mgenx_rec* rows = nullptr;      // pinned: decoded rows (valid after Poll / Wait)
    uint32_t n = 0;                 // datagrams in this stage
    uint64_t seq = 0;               // submission number
  };

  RecvRing(Context& ctx, uint32_t batch, uint32_t slot = MGENX_MAX_SIZE, uint32_t depth = 3,
           uint32_t opts = 0)
      : ctx_(ctx), batch_(batch), slot_(slot), opts_(opts), st_(depth) {
    if (depth < 2 || batch == 0) throw Error("RecvRing: depth >= 2 and batch > 0");
    for (Impl& s : st_) {
      s.h_slab.Resize((size_t)batch * slot);
      s.h_len.Resize(batch);
      s.h_src.Resize(batch);
      s.h_rxs.Resize(batch);
      s.h_rxu.Resize(batch);
      s.h_rows.Resize(batch);
      s.d_slab.Resize((size_t)batch * slot);
      s.d_len.Resize(batch);
      s.d_rows.Resize(batch);
      check_hip(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "hipStreamCreate");
      check_hip(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate");
      s.v.slab = s.h_slab.data(); s.v.len = s.h_len.data(); s.v.src = s.h_src.data();
      s.v.rx_sec = s.h_rxs.data(); s.v.rx_usec = s.h_rxu.data(); s.v.rows = s.h_rows.data();
    }
  }
  ~RecvRing() {
    for (Impl& s : st_) {
      if (s.stream) (void)hipStreamSynchronize(s.stream);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.stream) (void)hipStreamDestroy(s.stream);
    }
  }
  RecvRing(const RecvRing&) = delete;
  RecvRing& operator=(const RecvRing&) = delete;
  uint32_t Batch() const { return batch_; }
  uint32_t Slot() const { return slot_; }
  uint32_t InFlight() const { return busy_; }

  Stage& Fill() {
    if (busy_ == st_.size()) throw Error("RecvRing::Fill: every stage is busy (Wait + Release)");
    Stage& v = st_[head_].v;
    v.n = 0;
    return v;
  }
  // hand the filled stage to the GPU (asynchronous on that stage's stream)
  void Submit() {
    Impl& s = st_[head_];
    const uint32_t n = s.v.n;
    if (n > batch_) throw Error("RecvRing::Submit: n > batch");
    s.v.seq = next_seq_++;
    if (n) {
      check_hip(hipMemcpyAsync(s.d_slab.data(), s.h_slab.data(), (size_t)n * slot_,
                               hipMemcpyHostToDevice, s.stream), "H2D slab");
      check_hip(hipMemcpyAsync(s.d_len.data(), s.h_len.data(), (size_t)n * 4,
                               hipMemcpyHostToDevice, s.stream), "H2D lengths");
      mgenx_cols c;
      memset(&c, 0, sizeof(c));
      c.rows = s.d_rows.data();
      ctx_.Check(mgenx_unpack_batch(ctx_.get(), s.d_slab.data(), (uint64_t)n * slot_, nullptr,
                                    slot_, s.d_len.data(), 0, n, &c, opts_, s.stream),
                 "mgenx_unpack_batch");
      check_hip(hipMemcpyAsync(s.h_rows.data(), s.d_rows.data(), (size_t)n * sizeof(mgenx_rec),
                               hipMemcpyDeviceToHost, s.stream), "D2H rows");
    }
    check_hip(hipEventRecord(s.done, s.stream), "hipEventRecord");
    head_ = (head_ + 1) % st_.size();
    busy_++;
  }
  // the oldest submitted stage once its rows are back (nullptr: none, or not yet done)
  const Stage* Poll() {
    if (!busy_ || tail_taken_) return nullptr;
    const hipError_t e = hipEventQuery(st_[tail_].done);
    if (e == hipErrorNotReady) return nullptr;
    check_hip(e, "hipEventQuery");
    tail_taken_ = true;
    return &st_[tail_].v;
  }
  // the oldest submitted stage, waiting for it (nullptr: nothing in flight)
  const Stage* Wait() {
    if (!busy_) return nullptr;
    if (!tail_taken_) check_hip(hipEventSynchronize(st_[tail_].done), "hipEventSynchronize");
    tail_taken_ = true;
    return &st_[tail_].v;
  }
  // done with the stage Poll / Wait returned: it becomes free for Fill
  void Release() {
    if (!tail_taken_) throw Error("RecvRing::Release without Poll / Wait");
    tail_taken_ = false;
    tail_ = (tail_ + 1) % st_.size();
    busy_--;
  }

 private:
  struct Impl {
    PinnedArray<uint8_t> h_slab;
    PinnedArray<uint32_t> h_len, h_rxs, h_rxu;
    PinnedArray<mgenx_addr> h_src;
    PinnedArray<mgenx_rec> h_rows;
    DeviceArray<uint8_t> d_slab;
    DeviceArray<uint32_t> d_len;
    DeviceArray<mgenx_rec> d_rows;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    Stage v;
  };
  Context& ctx_;
  uint32_t batch_, slot_, opts_;
  std::vector<Impl> st_;
  size_t head_ = 0, tail_ = 0;
  uint32_t busy_ = 0;
  bool tail_taken_ = false;
  uint64_t next_seq_ = 0;
};

// ---- send: flows + per-message descriptors -> packed datagrams --------------------------
class SendBatch {
 public:
  explicit SendBatch(Context& ctx) : ctx_(ctx) {}
  // A flow's constant fields (what MgenFlow keeps across messages).  Addresses are raw
  // bytes in network order (ProtoAddress::GetRawHostAddress); lat/lon in degrees are
  // converted as Pack does, (UINT32)((deg + 180) * 60000) (mgenMsg.cpp:221,225).
  uint32_t AddFlow(uint32_t flowId, AddressType dstType, const uint8_t* dst, uint16_t dstPort,
                   AddressType hostType = INVALID_ADDRESS, const uint8_t* host = nullptr,
                   uint16_t hostPort = 0, double lat = 999.0, double lon = 999.0,
                   int32_t alt = -999, uint8_t gpsStatus = 0,
                   const std::vector<uint8_t>& payload = {}, uint8_t payloadType = 0) {
    mgenx_flow_tmpl t;
    memset(&t, 0, sizeof(t));
    t.flow_id = flowId;
    t.dst_type = dstType;
    t.dst_len = dstType == IPv6 ? 16 : (dstType == IPv4 ? 4 : 0);
    t.dst_port = dstPort;
    if (dst) memcpy(t.dst_addr, dst, t.dst_len);
    t.host_type = hostType;
    t.host_len = hostType == IPv6 ? 16 : (hostType == IPv4 ? 4 : 0);
    t.host_port = hostPort;
    if (host) memcpy(t.host_addr, host, t.host_len);
    t.lat_raw = (uint32_t)((lat + 180.0) * 60000.0);
    t.lon_raw = (uint32_t)((lon + 180.0) * 60000.0);
    t.alt = alt;
    t.gps_status = gpsStatus;
    t.payload_type = payloadType;
    t.payload_len = (uint16_t)payload.size();
    t.has_payload = payload.empty() ? 0 : 1;
    t.payload_off = (uint32_t)pool_.size();
    pool_.insert(pool_.end(), payload.begin(), payload.end());
    tmpl_.push_back(t);
    return (uint32_t)tmpl_.size() - 1;
  }
  // one message (MgenFlow::SendMessage: seq post-increment, tx time, msg_len, flags)
  void Add(uint32_t flow, uint32_t seq, const struct timeval& txTime, uint16_t msgLen,
           uint8_t flags = 0) {
    mgenx_pack_desc d;
    memset(&d, 0, sizeof(d));
    d.tmpl = flow;
    d.seq_num = seq;
    d.tx_sec = (uint32_t)txTime.tv_sec;
    d.tx_usec = (uint32_t)txTime.tv_usec;
    d.msg_len = msgLen;
    d.flags = flags;
    desc_.push_back(d);
  }
  // Pack every message into slots of `slot` bytes; returns the packed lengths
  // (0 = Pack failed, as MgenMsg::Pack returns 0).  fillTime: the time(NULL) the
  // reference would seed RANDOM_FILL with.
  const std::vector<uint32_t>& Pack(bool checksum, bool randomFill = false,
                                    uint32_t fillTime = 0, uint32_t slot = MGENX_MAX_SIZE) {
    const uint32_t n = (uint32_t)desc_.size();
    slot_ = slot;
    hipStream_t s = ctx_.stream();
    d_tmpl_.Resize(tmpl_.size());
    d_crc_.Resize(tmpl_.size());
    d_pool_.Resize(pool_.empty() ? 1 : pool_.size());
    d_desc_.Resize(n);
    d_slab_.Resize((size_t)n * slot);
    d_len_.Resize(n);
    check_hip(hipMemcpyAsync(d_tmpl_.data(), tmpl_.data(), tmpl_.size() * sizeof(tmpl_[0]),
                             hipMemcpyHostToDevice, s), "H2D tmpl");
    if (!pool_.empty())
      check_hip(hipMemcpyAsync(d_pool_.data(), pool_.data(), pool_.size(), hipMemcpyHostToDevice,
                               s), "H2D pool");
    check_hip(hipMemcpyAsync(d_desc_.data(), desc_.data(), n * sizeof(desc_[0]),
                             hipMemcpyHostToDevice, s), "H2D desc");
    ctx_.Check(mgenx_pack_prepare(ctx_.get(), d_tmpl_.data(), (uint32_t)tmpl_.size(),
                                  d_pool_.data(), d_crc_.data(), s), "mgenx_pack_prepare");
    if (randomFill) ctx_.Check(mgenx_set_fill_time(ctx_.get(), fillTime), "mgenx_set_fill_time");
    const uint32_t opts = (checksum ? MGENX_PACK_CHECKSUM : 0) | (randomFill ? MGENX_PACK_RANDOM_FILL : 0);
    ctx_.Check(mgenx_pack_batch(ctx_.get(), d_tmpl_.data(), d_crc_.data(), d_desc_.data(), n,
                                d_pool_.data(), d_slab_.data(), (uint64_t)n * slot, nullptr,
                                slot, d_len_.data(), opts, fillTime, s),
               "mgenx_pack_batch");
    h_slab_.Resize((size_t)n * slot);
    len_.resize(n);
    check_hip(hipMemcpyAsync(h_slab_.data(), d_slab_.data(), (size_t)n * slot,
                             hipMemcpyDeviceToHost, s), "D2H slab");
    check_hip(hipMemcpyAsync(len_.data(), d_len_.data(), n * 4, hipMemcpyDeviceToHost, s),
              "D2H lengths");
    ctx_.Sync();
    return len_;
  }
  const uint8_t* Datagram(uint32_t i) const { return h_slab_.data() + (size_t)i * slot_; }
  size_t Size() const { return desc_.size(); }
  void Clear() { desc_.clear(); }

 private:
  Context& ctx_;
  std::vector<mgenx_flow_tmpl> tmpl_;
  std::vector<uint8_t> pool_;
  std::vector<mgenx_pack_desc> desc_;
  std::vector<uint32_t> len_;
  uint32_t slot_ = MGENX_MAX_SIZE;
  DeviceArray<mgenx_flow_tmpl> d_tmpl_;
  DeviceArray<uint32_t> d_crc_;
  DeviceArray<uint8_t> d_pool_;
  DeviceArray<mgenx_pack_desc> d_desc_;
  DeviceArray<uint8_t> d_slab_;
  DeviceArray<uint32_t> d_len_;
  PinnedArray<uint8_t> h_slab_;
};

// ---- analytics: Mgen::UpdateRecvAnalytics over batches ---------------------------------
class FlowAnalytics {
 public:
  FlowAnalytics(Context& ctx, uint32_t maxFlows, double windowSec, uint32_t reportsPerFlow = 16)
      : ctx_(ctx), max_(maxFlows), per_(reportsPerFlow), flows_(maxFlows),
        reports_((size_t)maxFlows * reportsPerFlow), count_(maxFlows) {
    ctx_.Check(mgenx_flow_init(ctx_.get(), flows_.data(), maxFlows, windowSec, ctx_.stream()),
               "mgenx_flow_init");
    check_hip(hipMemsetAsync(count_.data(), 0, maxFlows * 4, ctx_.stream()), "memset");
  }
  // MgenAnalyticTable::FindFlow (mgenAnalytic.cpp:312-328): key = (src addr+port, dst
  // addr+port, flow id) -> dense index, created on first use.
  uint32_t FindFlow(const std::string& src, const std::string& dst, uint32_t flowId) {
    auto key = std::make_tuple(src, dst, flowId);
    auto it = index_.find(key);
    if (it != index_.end()) return it->second;
    if (index_.size() >= max_) throw Error("FlowAnalytics: too many flows");
    const uint32_t f = (uint32_t)index_.size();
    index_.emplace(key, f);
    return f;
  }
  // Update every record of a decoded batch, in receive order.  flowIdx[i] = FindFlow of
  // record i (>= maxFlows skips it, e.g. for records with an error); rx times per record.
  void Update(const RecvBatch& b, const std::vector<uint32_t>& flowIdx,
              const std::vector<uint32_t>& rxSec, const std::vector<uint32_t>& rxUsec) {
    const uint32_t n = b.Size();
    d_idx_.Resize(n);
    d_rxs_.Resize(n);
    d_rxu_.Resize(n);
    hipStream_t s = ctx_.stream();
    check_hip(hipMemcpyAsync(d_idx_.data(), flowIdx.data(), n * 4, hipMemcpyHostToDevice, s), "H2D");
    check_hip(hipMemcpyAsync(d_rxs_.data(), rxSec.data(), n * 4, hipMemcpyHostToDevice, s), "H2D");
    check_hip(hipMemcpyAsync(d_rxu_.data(), rxUsec.data(), n * 4, hipMemcpyHostToDevice, s), "H2D");
    ctx_.Check(mgenx_flow_reduce(ctx_.get(), d_idx_.data(), b.DevSeq(), b.DevTxSec(),
                                 b.DevTxUsec(), b.DevMsgLen(), d_rxs_.data(), d_rxu_.data(), n,
                                 flows_.data(), max_, reports_.data(), per_, count_.data(), s),
               "mgenx_flow_reduce");
  }
  // all reports so far (the first reportsPerFlow of each flow), flow by flow
  std::vector<mgenx_flow_report> Reports() {
    std::vector<uint32_t> cnt(max_);
    std::vector<mgenx_flow_report> all((size_t)max_ * per_), out;
    check_hip(hipMemcpyAsync(cnt.data(), count_.data(), max_ * 4, hipMemcpyDeviceToHost,
                             ctx_.stream()), "D2H");
    check_hip(hipMemcpyAsync(all.data(), reports_.data(), all.size() * sizeof(all[0]),
                             hipMemcpyDeviceToHost, ctx_.stream()), "D2H");
    ctx_.Sync();
    for (uint32_t f = 0; f < max_; f++)
      for (uint32_t k = 0; k < cnt[f] && k < per_; k++) out.push_back(all[(size_t)f * per_ + k]);
    return out;
  }
  // packed counters for the multi-GPU merge (all-reduce sum over ranks)
  void Export(mgenx_flow_counters* dev_out) {
    ctx_.Check(mgenx_flow_export(ctx_.get(), flows_.data(), max_, dev_out, ctx_.stream()),
               "mgenx_flow_export");
  }
  mgenx_flow_state* DevState() const { return flows_.data(); }

 private:
  Context& ctx_;
  uint32_t max_, per_;
  DeviceArray<mgenx_flow_state> flows_;
  DeviceArray<mgenx_flow_report> reports_;
  DeviceArray<uint32_t> count_;
  DeviceArray<uint32_t> d_idx_, d_rxs_, d_rxu_;
  std::map<std::tuple<std::string, std::string, uint32_t>, uint32_t> index_;
};

// ---- sharded stream framing: one TCP / SINK stream over the ranks of a job --------------
// An all-gather of fixed-size u64 vectors among the ranks (host vectors in and out):
// out[r * in.size() + k] = rank r's in[k].  The framing exchanges two kinds of message:
// every rank's exit table (2 x kExitCap words) and, rarely, 3 words that settle a chain the
// tables cannot follow.
class ShardComm {
 public:
  virtual ~ShardComm() = default;
  virtual int World() const = 0;
  virtual int Rank() const = 0;
  virtual std::vector<uint64_t> AllGather(const std::vector<uint64_t>& in) = 0;
};

// RCCL over xGMI: mgenx_allgather_u64 on the context's stream (device staging buffers).
class RcclShardComm : public ShardComm {
 public:
  RcclShardComm(Context& ctx, mgenx_comm* comm, int world, int rank)
      : ctx_(ctx), comm_(comm), world_(world), rank_(rank) {}
  int World() const override { return world_; }
  int Rank() const override { return rank_; }
  std::vector<uint64_t> AllGather(const std::vector<uint64_t>& in) override {
    const size_t n = in.size();
    d_in_.Resize(n ? n : 1);
    d_out_.Resize(std::max<size_t>(n * world_, 1));
    std::vector<uint64_t> out(n * world_);
    hipStream_t s = ctx_.stream();
    check_hip(hipMemcpyAsync(d_in_.data(), in.data(), n * 8, hipMemcpyHostToDevice, s), "H2D");
    ctx_.Check(mgenx_allgather_u64(ctx_.get(), comm_, d_in_.data(), d_out_.data(), (uint32_t)n, s),
               "mgenx_allgather_u64");
    check_hip(hipMemcpyAsync(out.data(), d_out_.data(), out.size() * 8, hipMemcpyDeviceToHost, s),
              "D2H");
    ctx_.Sync();
    return out;
  }

 private:
  Context& ctx_;
  mgenx_comm* comm_;
  int world_, rank_;
  DeviceArray<uint64_t> d_in_, d_out_;
};

struct ShardScanResult {
  uint64_t a = 0;          // this rank's first owned byte: local offsets + a = global offsets
  uint64_t n_local = 0;    // this rank's records (written to the caller's arrays, local offsets)
  uint64_t n_total = 0;    // the whole stream's summary, as mgenx_stream_scan reports it:
  uint64_t consumed = 0;   //   records, bytes consumed,
  int32_t status = 0;      //   status (1 = a TCP record with msg_len < 4 stopped the chain)
};

// The protocol of include/mgenx.h ("sharded framing"; mgen_amd/shard.py is the same steps):
// rank r owns the records starting in [a_r, b_r) and holds bytes [a_r, min(b_r + HALO, N)).
//   1. mgenx_stream_scan_exits: for each candidate entry below a_r + HALO, where its chain
//      first reaches b_r (bit 63: the chain leaves the candidate set -- exit unknown);
//   2. all-gather of the tables; every rank stitches e_0 = 0, e_{r+1} = exit_r(e_r)
//      identically; a missing entry or unknown exit is settled by that rank's sequential
//      range scan and a 3-word all-gather;
//   3. mgenx_stream_scan_range from e_r on the tables of step 1: the rank's records.
// A last all-gather gives every rank the whole-stream summary.  No stream bytes move.
class ShardedScan {
 public:
  static constexpr uint32_t kExitCap = 4096;
  static constexpr uint64_t kUnknown = 1ull << 63;
  static constexpr uint64_t kHalo = MGENX_SCAN_HALO;

  ShardedScan(Context& ctx, ShardComm& comm) : ctx_(ctx), comm_(comm) {}

  // rank `rank` owns record starts in [a, b) and holds bytes [a, hi)
  static void Bounds(uint64_t nbytes, int world, int rank, uint64_t& a, uint64_t& b,
                     uint64_t& hi) {
    a = nbytes * (uint64_t)rank / (uint64_t)world;
    b = nbytes * (uint64_t)(rank + 1) / (uint64_t)world;
    hi = std::min(b + kHalo, nbytes);
  }

  // The stitch, identical on every rank.  tables: World() x [entries(kExitCap) |
  // exits(kExitCap)] (local offsets, unused rows ~0, entries ascending); bounds[r] = (a, b);
  // settled[r] = (global exit, stopped).  entries[r] = global entry or -1 (the chain
  // stopped before rank r).  Returns the first rank whose exit a range scan must settle,
  // or -1 when every entry is known.
  static int Stitch(const std::vector<uint64_t>& tables,
                    const std::vector<std::pair<uint64_t, uint64_t>>& bounds,
                    const std::map<int, std::pair<uint64_t, bool>>& settled,
                    std::vector<int64_t>& entries) {
    const int world = (int)bounds.size();
    entries.assign(world, -1);
    entries[0] = 0;
    for (int r = 0; r < world; r++) {
      const int64_t e = entries[r];
      if (e < 0) break;
      const uint64_t a = bounds[r].first, b = bounds[r].second;
      const bool last = r == world - 1;
      uint64_t ex;
      auto it = settled.find(r);
      if (it != settled.end()) {
        if (it->second.second || last) break;
        ex = it->second.first;
      } else if ((uint64_t)e >= b && !last) {
        ex = (uint64_t)e;  // a record spans the whole range
      } else if (last) {
        break;
      } else {
        const uint64_t* ent = tables.data() + (size_t)r * 2 * kExitCap;
        const uint64_t* exi = ent + kExitCap;
        const uint64_t want = (uint64_t)e - a;
        const uint64_t* k = std::lower_bound(ent, ent + kExitCap, want);
        if (k == ent + kExitCap || *k != want || (exi[k - ent] & kUnknown)) return r;
        ex = a + exi[k - ent];
      }
      entries[r + 1] = (int64_t)ex;
    }
    return -1;
  }

  // d_local: this rank's bytes [a, hi) of a stream of nbytes; the rank's records go to
  // d_off / d_len (local offsets, at most cap).  Synchronous; collective over the ranks.
  ShardScanResult Run(const uint8_t* d_local, uint64_t nbytes, int mode, uint64_t* d_off,
                      uint32_t* d_len, uint64_t cap) {
    const int world = comm_.World(), rank = comm_.Rank();
    std::vector<std::pair<uint64_t, uint64_t>> bounds(world);
    for (int r = 0; r < world; r++) {
      uint64_t ra, rb, rh;
      Bounds(nbytes, world, r, ra, rb, rh);
      bounds[r] = {ra, rb};
    }
    uint64_t a, b, hi;
    Bounds(nbytes, world, rank, a, b, hi);
    const bool last = rank == world - 1;
    const uint64_t local = hi - a, limit = last ? local : b - a;
    mgenx_ctx* c = ctx_.get();
    hipStream_t s = ctx_.stream();
    // 1. this rank's exit table
    d_ent_.Resize(kExitCap);
    d_ext_.Resize(kExitCap);
    uint32_t cands = 0;
    ctx_.Check(mgenx_stream_scan_exits(c, d_local, local, mode, kHalo, limit, d_ent_.data(),
                                       d_ext_.data(), kExitCap, &cands, s),
               "mgenx_stream_scan_exits");
    std::vector<uint64_t> table(2 * kExitCap);
    check_hip(hipMemcpyAsync(table.data(), d_ent_.data(), kExitCap * 8, hipMemcpyDeviceToHost, s), "D2H");
    check_hip(hipMemcpyAsync(table.data() + kExitCap, d_ext_.data(), kExitCap * 8,
                             hipMemcpyDeviceToHost, s), "D2H");
    ctx_.Sync();
    // 2. gather, stitch, settle what the tables cannot
    const std::vector<uint64_t> tables = comm_.AllGather(table);
    std::map<int, std::pair<uint64_t, bool>> settled;
    std::vector<int64_t> entries;
    bool have_mine = false;
    mgenx_scan_info mine = {};
    for (;;) {
      const int need = Stitch(tables, bounds, settled, entries);
      if (need < 0) break;
      std::vector<uint64_t> msg(3, 0);
      if (rank == need) {
        mine = Range(d_local, local, mode, (uint64_t)entries[rank] - a, limit, d_off, d_len, cap);
        have_mine = true;
        const bool stopped = mine.consumed < limit || last;
        msg = {a + mine.consumed, stopped ? 1ull : 0ull, 1ull};
      }
      const std::vector<uint64_t> msgs = comm_.AllGather(msg);
      settled[need] = {msgs[3 * need], msgs[3 * need + 1] != 0};
    }
    // 3. this rank's records
    const int64_t e = entries[rank];
    if (!have_mine) {
      if (e < 0 || ((uint64_t)e >= b && !last)) {
        mine = {};
        mine.consumed = e >= 0 ? (uint64_t)e - a : 0;
      } else {
        mine = Range(d_local, local, mode, (uint64_t)e - a, limit, d_off, d_len, cap);
      }
    }
    const std::vector<uint64_t> summ =
        comm_.AllGather({mine.n_records, a + mine.consumed, (uint64_t)(uint32_t)mine.status,
                         e >= 0 ? 1ull : 0ull});
    ShardScanResult r;
    r.a = a;
    r.n_local = mine.n_records;
    int reached = 0;
    for (int q = 0; q < world; q++) {
      r.n_total += summ[4 * q];
      if (summ[4 * q + 3]) reached = q;  // the chain stops at the last rank it reached
    }
    r.consumed = summ[4 * reached + 1];
    r.status = (int32_t)summ[4 * reached + 2];
    return r;
  }

 private:
  mgenx_scan_info Range(const uint8_t* d_local, uint64_t local, int mode, uint64_t entry,
                        uint64_t limit, uint64_t* d_off, uint32_t* d_len, uint64_t cap) {
    mgenx_scan_info info = {};
    ctx_.Check(mgenx_stream_scan_range(ctx_.get(), d_local, local, mode, entry, limit,
                                       MGENX_SCAN_REUSE, d_off, d_len, cap, &info, ctx_.stream()),
               "mgenx_stream_scan_range");
    return info;
  }

  Context& ctx_;
  ShardComm& comm_;
  DeviceArray<uint64_t> d_ent_, d_ext_;
};

}  // namespace mgenx
