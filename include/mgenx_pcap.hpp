// mgenx_pcap.hpp -- pcap2mgen over the mgenx C ABI (header-only, C++17, HIP runtime).
//
// The reference tool (src/common/pcap2mgen.cpp:252-482) turns a capture file into an MGEN
// log one packet at a time.  Pcap2Mgen::Run does it for the whole file on the GPU:
//   mgenx_pcap_index (host, the pcap_next chain) -> one H2D copy of the file ->
//   mgenx_pcap_parse -> mgenx_unpack_batch(MGENX_OPT_SKIP_CRC: Unpack alone, :428) ->
//   [analytics: mgenx_flow_lookup (FindFlow, :447) -> mgenx_flow_reduce_ex (Update, :468) ->
//    mgenx_flow_keys + mgenx_report_build + mgenx_log_report_text (analytic->Log, :470)] ->
//   mgenx_log_recv_text (LogRecvEvent, :476: GMT or epoch timestamps, GPS, TTL, no data) ->
//   mgenx_data_walk + mgenx_log_report_recv_text (the REPORT items LogRecvEvent logs) ->
//   mgenx_text_interleave (per packet: analytic REPORT, RECV, received REPORTs) -> D2H.
// A few small values come back to the host between stages (flow count, report count, text
// sizes); everything per packet stays on the device.
#pragma once

#include <cmath>
#include <string>
#include <vector>

#include "mgenx.hpp"

namespace mgenx {

struct PcapOptions {
  bool analytics = false;  // -analytic / -report
  bool log_rx = true;      // +rxlog on|off
  bool epoch = false;      // Mgen::SetEpochTimestamp
  double window = 1.0;     // +window (MgenAnalytic::DEFAULT_WINDOW)
};

class Pcap2Mgen {
 public:
  Pcap2Mgen(Context& ctx, const PcapOptions& o) : ctx_(ctx), o_(o) {}

  // The log text of a pcap file image (host memory).
  std::string Run(const uint8_t* file, size_t nbytes) {
    mgenx_pcap_info info;
    if (mgenx_pcap_index(file, nbytes, nullptr, 0, &info) != MGENX_OK)
      throw Error("pcap2mgen: not a pcap file");
    std::vector<uint64_t> offs(info.n_records ? info.n_records : 1);
    (void)mgenx_pcap_index(file, nbytes, offs.data(), offs.size(), &info);
    const uint32_t n = (uint32_t)info.n_records;
    if (n == 0) return std::string();
    hipStream_t s = ctx_.stream();
    // the file image, then scratch for the packets a snapshot length cut (mgenx_pcap_snap)
    DeviceArray<uint8_t> buf(nbytes + info.snap_bytes);
    DeviceArray<uint64_t> pkt(n);
    check_hip(hipMemcpyAsync(buf.data(), file, nbytes, hipMemcpyHostToDevice, s), "H2D file");
    check_hip(hipMemcpyAsync(pkt.data(), offs.data(), (size_t)n * 8, hipMemcpyHostToDevice, s),
              "H2D offsets");
    std::string out = RunDevice(buf.data(), nbytes, pkt.data(), n, info.link_type, info.flags,
                                nbytes + info.snap_bytes);
    return out;
  }

  // The pipeline over a resident file image (device pointers).  buf_bytes > nbytes: scratch
  // after the image for packets cut by the snapshot length (else they are skipped).
  std::string RunDevice(uint8_t* d_buf, uint64_t nbytes, const uint64_t* d_pkt, uint32_t n,
                        uint32_t link_type, uint32_t flags, uint64_t buf_bytes = 0) {
    mgenx_ctx* c = ctx_.get();
    hipStream_t s = ctx_.stream();
    DeviceArray<uint64_t> udp_off(n);
    DeviceArray<uint32_t> udp_len(n), rx_sec(n), rx_usec(n);
    DeviceArray<mgenx_addr> src(n);
    DeviceArray<int32_t> ttl(n);
    DeviceArray<uint8_t> status(n);
    ctx_.Check(mgenx_pcap_parse(c, d_buf, nbytes, d_pkt, n, link_type, flags, udp_off.data(),
                                udp_len.data(), src.data(), ttl.data(), rx_sec.data(),
                                rx_usec.data(), status.data(), s),
               "mgenx_pcap_parse");
    if (buf_bytes > nbytes) {
      ctx_.Check(mgenx_pcap_snap(c, d_buf, nbytes, buf_bytes, d_pkt, n, flags, status.data(),
                                 udp_off.data(), udp_len.data(), s),
                 "mgenx_pcap_snap");
      nbytes = buf_bytes;  // the records now reach into the scratch
    }
    Columns col(n);
    ctx_.Check(mgenx_unpack_batch(c, d_buf, nbytes, udp_off.data(), 0, udp_len.data(), 0, n,
                                  &col.cols, MGENX_OPT_SKIP_CRC, s),
               "mgenx_unpack_batch");
    const uint32_t lopts = o_.epoch ? MGENX_LOG_EPOCH : 0u;
    std::vector<mgenx_text_src> srcs;
    // analytics (pcap2mgen.cpp:445-473)
    DeviceArray<char> rtext;
    DeviceArray<uint64_t> rline;
    DeviceArray<uint32_t> rep_rec;
    if (o_.analytics) {
      mgenx_flow_table* tab = nullptr;
      ctx_.Check(mgenx_flow_table_create(c, n, &tab), "mgenx_flow_table_create");
      struct TabGuard {
        mgenx_flow_table* t;
        ~TabGuard() { mgenx_flow_table_destroy(t); }
      } guard{tab};
      DeviceArray<uint32_t> fidx(n), nfl(1);
      ctx_.Check(mgenx_flow_lookup(c, tab, &col.cols, src.data(), n, fidx.data(), nfl.data(), s),
                 "mgenx_flow_lookup");
      const uint32_t n_flows = ReadU32(nfl.data());
      if (n_flows) {
        const uint32_t per_flow = PerFlow(fidx.data(), rx_sec.data(), rx_usec.data(), n, n_flows);
        const size_t slots = (size_t)n_flows * per_flow;
        DeviceArray<mgenx_flow_state> flows(n_flows);
        DeviceArray<mgenx_flow_report> reps(slots);
        DeviceArray<uint32_t> count(n_flows);
        rep_rec.Resize(slots);
        check_hip(hipMemsetAsync(count.data(), 0, (size_t)n_flows * 4, s), "memset");
        check_hip(hipMemsetAsync(rep_rec.data(), 0xFF, slots * 4, s), "memset");
        ctx_.Check(mgenx_flow_init(c, flows.data(), n_flows, o_.window, s), "mgenx_flow_init");
        ctx_.Check(mgenx_flow_reduce_ex(c, fidx.data(), col.seq.data(), col.txs.data(),
                                        col.txu.data(), col.mlen.data(), rx_sec.data(),
                                        rx_usec.data(), n, flows.data(), n_flows, reps.data(),
                                        per_flow, count.data(), rep_rec.data(), s),
                   "mgenx_flow_reduce_ex");
        DeviceArray<mgenx_report_key> keys(n_flows);
        DeviceArray<uint8_t> sign(n_flows), items(slots * MGENX_REPORT_MAX), ilen(slots);
        check_hip(hipMemsetAsync(sign.data(), 0, n_flows, s), "memset");
        ctx_.Check(mgenx_flow_keys(c, tab, MGENX_PROTO_UDP, keys.data(), n_flows, s),
                   "mgenx_flow_keys");
        ctx_.Check(mgenx_report_build(c, reps.data(), n_flows, per_flow, count.data(),
                                      keys.data(), sign.data(), nullptr, items.data(),
                                      ilen.data(), s),
                   "mgenx_report_build");
        rline.Resize(slots + 1);
        TwoPass(rtext, rline.data(), slots, [&](char* t, uint64_t cap) {
          return mgenx_log_report_text(c, items.data(), reps.data(), n_flows, per_flow,
                                       count.data(), lopts, t, cap, rline.data(), s);
        });
        srcs.push_back(Src(MGENX_TEXT_SCATTER, rtext.data(), rline.data(), (uint32_t)slots,
                           rep_rec.data(), 1));
      }
    }
    // RECV lines (LogRecvEvent, pcap2mgen.cpp:476)
    DeviceArray<char> text;
    DeviceArray<uint64_t> line(n + 1);
    if (o_.log_rx) {
      TwoPass(text, line.data(), n, [&](char* t, uint64_t cap) {
        return mgenx_log_recv_text(c, d_buf, udp_off.data(), 0, &col.cols, src.data(),
                                   rx_sec.data(), rx_usec.data(), ttl.data(), n,
                                   MGENX_PROTO_UDP, lopts | MGENX_LOG_NO_DATA | MGENX_LOG_SKIP_ERR,
                                   t, cap, line.data(), s);
      });
      srcs.push_back(Src(MGENX_TEXT_PER_RECORD, text.data(), line.data(), n, nullptr, 1));
    }
    // REPORT items carried in MGEN_DATA payloads (mgenMsg.cpp:1104-1137)
    DeviceArray<uint8_t> wst(n), wnh(n);
    DeviceArray<uint32_t> cmds(2), totals(2);
    DeviceArray<uint64_t> pairs;
    uint32_t n_reps = 0, cap = 1024;
    for (int pass = 0; pass < 2; pass++) {
      pairs.Resize((size_t)cap * 2);
      ctx_.Check(mgenx_data_walk(c, d_buf, udp_off.data(), 0, &col.cols, n,
                                 MGENX_DATA_CONTROLLER, wst.data(), wnh.data(), cmds.data(), 1,
                                 pairs.data(), cap, totals.data(), s),
                 "mgenx_data_walk");
      n_reps = ReadU32(totals.data() + 1);
      if (n_reps <= cap) break;
      cap = n_reps;
    }
    DeviceArray<char> rrtext;
    DeviceArray<uint64_t> rrline(n_reps + 1);
    if (n_reps) {
      TwoPass(rrtext, rrline.data(), n_reps, [&](char* t, uint64_t cp) {
        return mgenx_log_report_recv_text(c, d_buf, pairs.data(), n_reps, src.data(),
                                          rx_sec.data(), rx_usec.data(), lopts, t, cp,
                                          rrline.data(), s);
      });
      srcs.push_back(Src(MGENX_TEXT_OWNER, rrtext.data(), rrline.data(), n_reps,
                         reinterpret_cast<const uint32_t*>(pairs.data()), 4));
    }
    if (srcs.empty()) return std::string();
    DeviceArray<char> all;
    DeviceArray<uint64_t> rec_off(n + 1);
    uint64_t total = TwoPass(all, rec_off.data(), n, [&](char* t, uint64_t cp) {
      return mgenx_text_interleave(c, srcs.data(), (uint32_t)srcs.size(), n, t, cp,
                                   rec_off.data(), s);
    });
    std::string out(total, '\0');
    if (total)
      check_hip(hipMemcpyAsync(&out[0], all.data(), total, hipMemcpyDeviceToHost, s), "D2H log");
    ctx_.Sync();
    return out;
  }

 private:
  // the unpack columns pcap2mgen reads (core + the extended ones the log needs)
  struct Columns {
    DeviceArray<uint32_t> flow, seq, txs, txu, dst4, payoff, lat, lon;
    DeviceArray<uint16_t> mlen, dport, plen, hlen, hport;
    DeviceArray<uint8_t> flags, err, dtype, dlen, ptype, gps, htype, hl, haddr, daddr;
    DeviceArray<int32_t> alt;
    mgenx_cols cols;
    explicit Columns(uint32_t n) {
      for (auto* a : {&flow, &seq, &txs, &txu, &dst4, &payoff, &lat, &lon}) a->Resize(n);
      for (auto* a : {&mlen, &dport, &plen, &hlen, &hport}) a->Resize(n);
      for (auto* a : {&flags, &err, &dtype, &dlen, &ptype, &gps, &htype, &hl}) a->Resize(n);
      haddr.Resize((size_t)n * 16);
      daddr.Resize((size_t)n * 16);
      alt.Resize(n);
      memset(&cols, 0, sizeof(cols));
      cols.flow_id = flow.data(); cols.seq_num = seq.data(); cols.tx_sec = txs.data();
      cols.tx_usec = txu.data(); cols.msg_len = mlen.data(); cols.dst_port = dport.data();
      cols.flags = flags.data(); cols.err = err.data(); cols.dst_type = dtype.data();
      cols.dst_len = dlen.data(); cols.dst_addr4 = dst4.data(); cols.payload_len = plen.data();
      cols.payload_type = ptype.data(); cols.gps_status = gps.data(); cols.hdr_len = hlen.data();
      cols.payload_off = payoff.data(); cols.host_port = hport.data();
      cols.host_type = htype.data(); cols.host_len = hl.data(); cols.host_addr = haddr.data();
      cols.dst_addr = daddr.data(); cols.lat_raw = lat.data(); cols.lon_raw = lon.data();
      cols.alt = alt.data();
    }
  };

  static mgenx_text_src Src(uint32_t kind, const char* t, const uint64_t* lo, uint32_t n,
                            const uint32_t* idx, uint32_t stride) {
    mgenx_text_src x;
    memset(&x, 0, sizeof(x));
    x.text = t; x.line_off = lo; x.n_lines = n; x.kind = kind; x.index = idx;
    x.index_stride = stride;
    return x;
  }

  uint32_t ReadU32(const uint32_t* d) {
    uint32_t v = 0;
    check_hip(hipMemcpyAsync(&v, d, 4, hipMemcpyDeviceToHost, ctx_.stream()), "D2H");
    ctx_.Sync();
    return v;
  }

  // a two-pass formatter: size with a guess, grow once to the reported total
  template <typename F>
  uint64_t TwoPass(DeviceArray<char>& buf, uint64_t* d_off, size_t n, F call) {
    uint64_t cap = (uint64_t)n * 200 + 64;
    for (int pass = 0; pass < 2; pass++) {
      if (buf.size() < cap) buf.Resize(cap);
      ctx_.Check(call(buf.data(), cap), "log text");
      uint64_t total = 0;
      check_hip(hipMemcpyAsync(&total, d_off + n, 8, hipMemcpyDeviceToHost, ctx_.stream()),
                "D2H");
      ctx_.Sync();
      if (total <= cap) return total;
      cap = total;
    }
    throw Error("pcap2mgen: text did not fit");
  }

  // report slots per flow: a window closes at most once per record and, since the window
  // restarts at the closing record, at most once per window length of capture time (the
  // counts and the time range reduced on the device: 24 bytes come back, not the columns)
  uint32_t PerFlow(const uint32_t* d_fidx, const uint32_t* d_sec, const uint32_t* d_usec,
                   uint32_t n, uint32_t n_flows) {
    hipStream_t s = ctx_.stream();
    DeviceArray<uint32_t> cnt(n_flows);
    DeviceArray<uint64_t> d_out(3);
    ctx_.Check(mgenx_flow_span(ctx_.get(), d_fidx, d_sec, d_usec, n, n_flows, cnt.data(),
                               d_out.data(), s),
               "mgenx_flow_span");
    uint64_t o[3] = {0, 0, 0};
    check_hip(hipMemcpyAsync(o, d_out.data(), sizeof(o), hipMemcpyDeviceToHost, s), "D2H");
    ctx_.Sync();
    const uint32_t most = o[0] > 1 ? (uint32_t)o[0] : 1u;
    const double w = o_.window;  // the quantized window is within 5% of the request
    if (w <= 0.0 || o[2] < o[1]) return most;
    const double by_time = (double)(o[2] - o[1]) * 1e-6 / (0.95 * w) + 2.0;
    return by_time < most ? (uint32_t)by_time : most;
  }

  Context& ctx_;
  PcapOptions o_;
};

}  // namespace mgenx
