// mgenAnalytic.h -- drop-in MgenAnalytic / MgenAnalytic::Report / MgenAnalyticTable
// (reference include/mgenAnalytic.h:64-396, src/common/mgenAnalytic.cpp).
//
// MgenAnalytic::Update (the per-flow window state machine with its 1024-bit duplicate
// mask, mgenAnalytic.cpp:74-258) runs on the GPU: each MgenAnalytic owns a device
// mgenx_flow_state slot, Update of one record goes to the resident worker
// (mgenx_worker_flow_update), and MgenAnalyticTable::UpdateBatch hands a whole receive batch
// (in receive order) to mgenx_flow_reduce.  Report building / parsing and the quantizers (mgenAnalytic.cpp:331-642) are the
// host-side wire format of the MGEN_DATA report item, as in the reference.
#ifndef _MGEN_ANALYTIC
#define _MGEN_ANALYTIC

#include <math.h>
#include <stdio.h>

#include <map>
#include <string>
#include <vector>

#include "mgenPayload.h"
#include "mgenx_compat.hpp"
#include "mgenx_proto.h"

class MgenAnalytic {
 public:
  static constexpr double DEFAULT_WINDOW = 1.0;
  enum { DEFAULT_HISTORY = 1024 };
  enum { KEY_MAX = (16 + 2 + 16 + 2 + 4) };

  class Report : public MgenDataItem {
   public:
    Report(UINT32* bufferPtr = nullptr, unsigned int bufferBytes = 0, bool freeOnDestruct = false)
        : MgenDataItem(bufferPtr, bufferBytes, freeOnDestruct) {
      InitFromBuffer();
    }
    ~Report() {}

    enum ReportType { REPORT_INVALID = 0, REPORT_FLOW_IPv4, REPORT_FLOW_IPv6 };
    enum Flag { FLAG_FLOW_ID = 0x01, FLAG_LATENCY_SIGN = 0x02 };
    enum { MAX_LENGTH = (4 + 2 * 16 + 4 * 4) };

    // mgenAnalytic.cpp:343-376: a report item of the right type whose len byte matches
    bool InitFromBuffer(UINT32* bufferPtr = nullptr, unsigned int numBytes = 0,
                        bool freeOnDestruct = false) {
      if (MgenDataItem::InitFromBuffer(bufferPtr, numBytes, freeOnDestruct) &&
          GetBufferLength() >= OFFSET_FLAGS) {
        const ReportType t = GetReportType();
        if (t == REPORT_FLOW_IPv4 || t == REPORT_FLOW_IPv6) {
          if (GetReportLength() == OffsetLossFraction() + 2) return true;
          SetType(DATA_ITEM_INVALID);
        }
      }
      if (bufferPtr) DetachBuffer();
      return false;
    }
    ReportType GetReportType() const { return (ReportType)((GetUINT8(OFFSET_TYPE) >> 4) & 0x0f); }
    Protocol GetProtocol() const { return (Protocol)(GetUINT8(OFFSET_PROTOCOL) & 0x0f); }
    UINT8 GetReportLength() const { return GetUINT8(OFFSET_LEN); }
    bool FlagIsSet(Flag flag) const { return 0 != (flag & (GetUINT8(OFFSET_FLAGS) >> 5)); }
    bool GetDstAddr(ProtoAddress& addr) const { return GetAddr(addr, 4 * OFFSET_DST, OffsetDstPort()); }
    bool GetSrcAddr(ProtoAddress& addr) const { return GetAddr(addr, 4 * OffsetSrc(), OffsetSrcPort()); }
    UINT32 GetFlowId() const { return FlagIsSet(FLAG_FLOW_ID) ? GetUINT32(OffsetFlowId()) : 0; }
    double GetWindowOffset() const { return UnquantizeTimeValue((UINT8)(GetUINT16(OFFSET_WINDOW) & 0x1fff)); }
    double GetWindowSize() const { return UnquantizeTimeValue(GetUINT8(OffsetWindowSize())); }
    double GetLatencyAve() const {
      const double ave = UnquantizeTimeValue(GetUINT8(OffsetLatencyAve()));
      return FlagIsSet(FLAG_LATENCY_SIGN) ? -ave : ave;
    }
    double GetLatencyMin() const { return GetLatencyAve() - UnquantizeTimeValue(GetUINT8(OffsetLatencyMin())); }
    double GetLatencyMax() const { return GetLatencyAve() + UnquantizeTimeValue(GetUINT8(OffsetLatencyMax())); }
    double GetRateAve() const { return UnquantizeRate(GetUINT16(OffsetRateAve())); }
    double GetLossFraction() const { return UnquantizeLoss(GetUINT16(OffsetLossFraction())); }
    // the received-report REPORT line (mgenAnalytic.cpp:747-786; mgenx_compat.cpp)
    void Log(FILE* filePtr, const ProtoTime& sentTime, const ProtoTime& theTime, bool localTime,
             const ProtoAddress& reporterAddr) const;

    // mgenAnalytic.cpp:446-475
    bool InitIntoBuffer(ReportType reportType, UINT32* bufferPtr = nullptr,
                        unsigned int bufferBytes = 0, bool freeOnDestruct = false) {
      if (reportType != REPORT_FLOW_IPv4 && reportType != REPORT_FLOW_IPv6) return false;
      const unsigned minLength = 12 + OFFSET_DST * 4;
      if (bufferPtr) {
        if (bufferBytes < minLength) return false;
        AttachBuffer(bufferPtr, bufferBytes, freeOnDestruct);
      } else if (GetBufferLength() < minLength) {
        return false;
      }
      memset(AccessBuffer(), 0, minLength);
      SetReportType(reportType);
      SetReportLength((UINT8)minLength);
      SetLength(minLength);
      return true;
    }
    void SetProtocol(Protocol protocol) {
      SetUINT8(OFFSET_PROTOCOL, (UINT8)((0xf0 & GetUINT8(OFFSET_PROTOCOL)) | (UINT8)protocol));
    }
    bool SetDstAddr(const ProtoAddress& addr) { return SetAddr(addr, true); }
    bool SetSrcAddr(const ProtoAddress& addr) { return SetAddr(addr, false); }
    // :536-550
    bool SetFlowId(UINT32 flowId) {
      const unsigned reportLength = OffsetSrc() * 4 + GetAddrLen() + 12 + 4;
      if (reportLength > GetBufferLength()) return false;
      SetFlag(FLAG_FLOW_ID);
      SetUINT32(OffsetFlowId(), flowId);
      SetReportLength((UINT8)reportLength);
      SetLength(reportLength);
      return true;
    }
    void SetWindowOffset(double seconds) {
      const UINT16 q = QuantizeTimeValue(seconds);
      SetUINT16(OFFSET_WINDOW, (UINT16)((GetUINT16(OFFSET_WINDOW) & 0xe000) | q));
    }
    void SetWindowSize(double seconds) { SetUINT8(OffsetWindowSize(), QuantizeTimeValue(seconds)); }
    void SetLatencyAve(double seconds) {
      if (seconds < 0.0) SetFlag(FLAG_LATENCY_SIGN);  // never cleared (as in the reference)
      SetUINT8(OffsetLatencyAve(), QuantizeTimeValue(fabs(seconds)));
    }
    void SetLatencyDeltaMin(double d) { SetUINT8(OffsetLatencyMin(), QuantizeTimeValue(fabs(d))); }
    void SetLatencyDeltaMax(double d) { SetUINT8(OffsetLatencyMax(), QuantizeTimeValue(fabs(d))); }
    void SetRateAve(double rate) { SetUINT16(OffsetRateAve(), QuantizeRate(rate)); }
    void SetLossFraction(double loss) { SetUINT16(OffsetLossFraction(), QuantizeLoss(loss)); }

    // quantizers (mgenAnalytic.cpp:568-642)
    static UINT8 QuantizeTimeValue(double value) {
      if (value > TIME_STRETCH * TIME_MAX) return 0xff;
      if (value < TIME_MIN / 2.0) return 0;
      if (value < TIME_MIN) return 1;
      return (UINT8)((log(TIME_STRETCH + (value - TIME_MIN) / (TimeScale() * (TIME_MAX - TIME_MIN))) /
                      log(TIME_STRETCH)) + 0.5);
    }
    static double UnquantizeTimeValue(UINT8 q) {
      if (0 == q) return 0.0;
      return (TIME_MAX - TIME_MIN) * (pow(TIME_STRETCH, q) - TIME_STRETCH) * TimeScale() + TIME_MIN;
    }

   private:
    static UINT16 QuantizeOffset(double offset) {
      if (offset < 1.0e-03) return 0x01;
      if (offset >= 10.0e+04) return 0x1fff;
      const int exponent = (int)log10(offset);
      const UINT16 mantissa = (UINT16)((1024.0 / 10.0) * (offset / pow(10.0, (double)exponent)) + 0.5);
      return (UINT16)((mantissa << 3) | ((UINT16)exponent + 3));
    }
    static double UnquantizeOffset(UINT16 q) {
      return ((double)(q >> 3)) * (10.0 / 1024.0) * pow(10.0, (double)(q & 0x0007));
    }
    static UINT16 QuantizeRate(double rate) {
      if (rate <= 0.0) return 0x01;
      const UINT16 exponent = (UINT16)log10(rate);
      const UINT16 mantissa = (UINT16)((4096.0 / 10.0) * (rate / pow(10.0, (double)exponent)) + 0.5);
      return (UINT16)((mantissa << 4) | exponent);
    }
    static double UnquantizeRate(UINT16 rate) {
      return ((double)(rate >> 4)) * (10.0 / 4096.0) * pow(10.0, (double)(rate & 0x000f));
    }
    static UINT16 QuantizeLoss(double lossFraction) {
      if (0.0 == lossFraction) return 0;
      lossFraction = lossFraction * 65535.0 + 0.5;
      if (lossFraction < 1.0) return 1;
      if (lossFraction > 65535.0) return 65535;
      return (UINT16)lossFraction;
    }
    static double UnquantizeLoss(UINT16 q) { return ((double)q) / 65535.0; }
    static constexpr double TIME_STRETCH = 1.1;
    static constexpr double TIME_MIN = 1.0e-06;
    static constexpr double TIME_MAX = 600.0;
    static double TimeScale() {
      static const double s = 1.0 / (pow(TIME_STRETCH, 254) - TIME_STRETCH);
      return s;
    }

    enum {
      OFFSET_PROTOCOL = OFFSET_TYPE,
      OFFSET_FLAGS = OFFSET_LEN + 1,
      OFFSET_WINDOW = OFFSET_LEN + 1,
      OFFSET_DST = (OFFSET_WINDOW + 2) / 4  // UINT32 offset
    };
    unsigned GetAddrLen() const {
      switch (GetReportType()) {
        case REPORT_FLOW_IPv4: return 4;
        case REPORT_FLOW_IPv6: return 16;
        default: return 0;
      }
    }
    unsigned OffsetSrc() const { return OFFSET_DST + GetAddrLen() / 4; }
    unsigned OffsetDstPort() const { return 4 * OffsetSrc() + GetAddrLen(); }
    unsigned OffsetSrcPort() const { return OffsetDstPort() + 2; }
    unsigned OffsetFlowId() const { return OffsetSrcPort() + 2; }
    unsigned OffsetWindowSize() const { return OffsetFlowId() + (FlagIsSet(FLAG_FLOW_ID) ? 4 : 0); }
    unsigned OffsetLatencyAve() const { return OffsetWindowSize() + 1; }
    unsigned OffsetLatencyMin() const { return OffsetLatencyAve() + 1; }
    unsigned OffsetLatencyMax() const { return OffsetLatencyMin() + 1; }
    unsigned OffsetRateAve() const { return OffsetLatencyMax() + 1; }
    unsigned OffsetLossFraction() const { return OffsetRateAve() + 2; }
    void SetReportType(ReportType type) {
      SetUINT8(OFFSET_TYPE, (UINT8)((0x0f & GetUINT8(OFFSET_TYPE)) | ((UINT8)type << 4)));
    }
    void SetReportLength(UINT8 n) { SetUINT8(OFFSET_LEN, n); }
    void SetFlag(Flag flag) { SetUINT8(OFFSET_FLAGS, (UINT8)(GetUINT8(OFFSET_FLAGS) | (flag << 5))); }
    // :379-444 (an address length of 6 would be ETH; report types only give 4 or 16)
    bool GetAddr(ProtoAddress& addr, unsigned byteOff, unsigned portOff) const {
      const unsigned len = GetAddrLen();
      if (len != 4 && len != 16) return false;
      addr.SetRawHostAddress(len == 4 ? ProtoAddress::IPv4 : ProtoAddress::IPv6,
                             GetBuffer(byteOff), len);
      addr.SetPort(GetUINT16(portOff));
      return true;
    }
    // :477-534
    bool SetAddr(const ProtoAddress& addr, bool dst) {
      ReportType rt;
      unsigned len;
      switch (addr.GetType()) {
        case ProtoAddress::IPv4: rt = REPORT_FLOW_IPv4; len = 4; break;
        case ProtoAddress::IPv6: rt = REPORT_FLOW_IPv6; len = 16; break;
        default: return false;
      }
      const unsigned reportLength = 12 + OFFSET_DST * 4 + 2 * len;
      if (reportLength > GetBufferLength()) return false;
      SetReportType(rt);
      SetReportLength((UINT8)reportLength);
      memcpy(AccessBuffer(4 * (dst ? (unsigned)OFFSET_DST : OffsetSrc())), addr.GetRawHostAddress(), len);
      SetUINT16(dst ? OffsetDstPort() : OffsetSrcPort(), addr.GetPort());
      SetLength(reportLength);
      return true;
    }
  };  // class Report

  MgenAnalytic() : slot_(kNoSlot), window_size(DEFAULT_WINDOW), report_valid(false) {
    window_size = Report::UnquantizeTimeValue(Report::QuantizeTimeValue(window_size));
    ClearReport();
  }
  ~MgenAnalytic() {
    if (slot_ != kNoSlot) {
      std::lock_guard<std::mutex> g(mgenx::compat::Engine::Get().Lock());
      mgenx::compat::Engine::Get().FlowFree(slot_);
    }
  }

  // mgenAnalytic.cpp:28-71 (historyDepth: the device mask is 1024 bits, the default)
  bool Init(Protocol protocol, const ProtoAddress& srcAddr, const ProtoAddress& dstAddr,
            UINT32 flowId, double windowSize = MgenAnalytic::DEFAULT_WINDOW,
            UINT32 historyDepth = MgenAnalytic::DEFAULT_HISTORY) {
    if (historyDepth != DEFAULT_HISTORY) return false;
    window_size = Report::UnquantizeTimeValue(Report::QuantizeTimeValue(windowSize));
    key_ = MakeKey(srcAddr, dstAddr, flowId);
    {
      std::lock_guard<std::mutex> g(mgenx::compat::Engine::Get().Lock());
      auto& e = mgenx::compat::Engine::Get();
      if (slot_ == kNoSlot) slot_ = e.FlowAlloc(windowSize);
      else e.FlowReinit(slot_, windowSize);
    }
    report_msg.InitIntoBuffer(Report::REPORT_FLOW_IPv4, report_buffer, Report::MAX_LENGTH);
    report_msg.SetProtocol(protocol);
    report_msg.SetDstAddr(dstAddr);
    report_msg.SetSrcAddr(srcAddr);
    if (1 != flowId) report_msg.SetFlowId(flowId);
    report_msg.SetWindowSize(window_size);
    return true;
  }
  void SetWindowSize(double windowSize) {
    window_size = Report::UnquantizeTimeValue(Report::QuantizeTimeValue(windowSize));
  }

  // returns "true" when report values have been updated (mgenAnalytic.cpp:74-258)
  bool Update(const ProtoTime& rxTime, unsigned int msgSize = 0,
              const ProtoTime& txTime = ProtoTime(0.0), UINT32 seqNum = 0) {
    MgenAnalytic* self = this;
    bool updated = false;
    UpdateBatch(&self, &rxTime, &msgSize, &txTime, &seqNum, &updated, 1);
    return updated;
  }
  // updated[i] = items[i]->Update(rxTime[i], msgSize[i], txTime[i], seqNum[i]), in order
  static void UpdateBatch(MgenAnalytic* const* items, const ProtoTime* rxTime,
                          const unsigned int* msgSize, const ProtoTime* txTime,
                          const UINT32* seqNum, bool* updated, unsigned n) {
    std::vector<uint32_t> slot(n), rxs(n), rxu(n), txs(n), txu(n), seq(n);
    std::vector<uint16_t> len(n);
    std::vector<mgenx_flow_report> rep(n);
    bool* upd = updated;
    for (unsigned i = 0; i < n; i++) {
      slot[i] = items[i]->slot_;
      rxs[i] = (uint32_t)rxTime[i].GetTimeVal().tv_sec;
      rxu[i] = (uint32_t)rxTime[i].GetTimeVal().tv_usec;
      txs[i] = (uint32_t)txTime[i].GetTimeVal().tv_sec;
      txu[i] = (uint32_t)txTime[i].GetTimeVal().tv_usec;
      len[i] = (uint16_t)msgSize[i];
      seq[i] = seqNum[i];
    }
    {
      std::lock_guard<std::mutex> g(mgenx::compat::Engine::Get().Lock());
      mgenx::compat::Engine::Get().FlowUpdate(slot.data(), rxs.data(), rxu.data(), len.data(),
                                              txs.data(), txu.data(), seq.data(), n, upd,
                                              rep.data());
    }
    for (unsigned i = 0; i < n; i++)
      if (updated[i]) items[i]->TakeReport(rep[i]);
  }

  // the REPORT line of the last closed window (mgenAnalytic.cpp:260-295; mgenx_compat.cpp)
  void Log(FILE* filePtr, const ProtoTime& sentTime, const ProtoTime& theTime,
           bool localTime) const;
  // the current window's end (include/mgenAnalytic.h:105-106): read from the device state
  const ProtoTime& GetWindowEnd() const;

  const Report& GetReport(const ProtoTime& theTime) {
    double windowOffset = (Seconds(theTime) - Seconds(report_start)) - report_duration;
    if (windowOffset < 0.0) windowOffset = 0.0;
    report_msg.SetWindowOffset(windowOffset);
    report_time = theTime;
    return report_msg;
  }
  const ProtoTime& GetReportTime() const { return report_time; }
  const ProtoTime& GetReportStartTime() const { return report_start; }
  double GetReportDuration() const { return report_duration; }
  unsigned long GetReportMessageCount() const { return report_msg_count; }
  double GetReportRateAverage() const { return report_rate_ave; }
  double GetReportLossFraction() const { return report_loss_ave; }
  double GetReportLatencyAverage() const { return report_latency_ave; }
  double GetReportLatencyMin() const { return report_latency_min; }
  double GetReportLatencyMax() const { return report_latency_max; }
  double GetWindowSize() const { return window_size; }

  const char* GetKey() const { return key_.data(); }
  unsigned int GetKeysize() const { return (unsigned)key_.size() << 3; }

  // FindFlow's key: dst addr, dst port, src addr, src port, flowId (mgenAnalytic.cpp:312-328)
  static std::string MakeKey(const ProtoAddress& src, const ProtoAddress& dst, UINT32 flowId) {
    std::string k;
    k.append(dst.GetRawHostAddress(), dst.GetLength());
    UINT16 port = dst.GetPort();
    k.append((const char*)&port, 2);
    k.append(src.GetRawHostAddress(), src.GetLength());
    port = src.GetPort();
    k.append((const char*)&port, 2);
    k.append((const char*)&flowId, 4);
    return k;
  }

 private:
  static constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
  static double Seconds(const ProtoTime& t) {  // ProtoTime::GetValue
    return (double)t.GetTimeVal().tv_sec + 1.0e-06 * (double)t.GetTimeVal().tv_usec;
  }
  void ClearReport() {
    report_duration = report_rate_ave = report_loss_ave = 0.0;
    report_latency_ave = report_latency_min = report_latency_max = 0.0;
    report_msg_count = 0;
  }
  // the report members and report_buffer updates of mgenAnalytic.cpp:170-252
  void TakeReport(const mgenx_flow_report& r) {
    report_valid = true;
    struct timeval tv;
    tv.tv_sec = (time_t)r.start_sec;
    tv.tv_usec = (suseconds_t)r.start_usec;
    report_start = ProtoTime(tv);
    report_duration = r.duration;
    report_msg_count = (unsigned long)r.msg_count;
    report_rate_ave = r.rate;
    report_loss_ave = r.loss;
    report_latency_ave = r.latency_ave;
    report_latency_min = r.latency_min;
    report_latency_max = r.latency_max;
    report_msg.SetWindowSize(report_duration);
    report_msg.SetLatencyAve(report_latency_ave);
    report_msg.SetLatencyDeltaMin(report_latency_ave - report_latency_min);
    report_msg.SetLatencyDeltaMax(report_latency_max - report_latency_ave);
    report_msg.SetRateAve(report_rate_ave);
    report_msg.SetLossFraction(report_loss_ave);
  }

  uint32_t slot_;
  std::string key_;
  double window_size;
  bool report_valid;
  ProtoTime report_start;
  double report_duration;
  unsigned long report_msg_count;
  double report_rate_ave, report_loss_ave;
  double report_latency_ave, report_latency_min, report_latency_max;
  ProtoTime report_time;
  mutable ProtoTime window_end_;
  UINT32 report_buffer[Report::MAX_LENGTH / sizeof(UINT32)];
  Report report_msg;
};

// FindFlow by the reference's key (ProtoIndexedQueue in the reference; a map here).  The
// device-side form for whole batches is mgenx_flow_lookup (dense index per record).
class MgenAnalyticTable {
 public:
  MgenAnalytic* FindFlow(const ProtoAddress& srcAddr, const ProtoAddress& dstAddr, UINT32 flowId) {
    auto it = table_.find(MgenAnalytic::MakeKey(srcAddr, dstAddr, flowId));
    return it == table_.end() ? nullptr : it->second;
  }
  bool Insert(MgenAnalytic& item) {
    return table_.emplace(std::string(item.GetKey(), item.GetKeysize() >> 3), &item).second;
  }
  void Remove(MgenAnalytic& item) { table_.erase(std::string(item.GetKey(), item.GetKeysize() >> 3)); }
  bool IsEmpty() const { return table_.empty(); }

 private:
  std::map<std::string, MgenAnalytic*> table_;
};

#endif  // _MGEN_ANALYTIC
