// C++ host-layer test (include/mgenx.hpp): SendBatch -> RecvBatch round trip with the
// MgenMsg getters, a corrupted datagram caught as ERROR_CHECKSUM, and FlowAnalytics over
// the decoded batch.  Prints "host_roundtrip ok" and exits 0 on success.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mgenx.hpp"

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)

int main() {
  using namespace mgenx;
  Context ctx(0);
  SendBatch sb(ctx);
  const uint8_t lo[4] = {127, 0, 0, 1};
  uint8_t v6[16] = {0};
  v6[15] = 1;
  const uint32_t f1 = sb.AddFlow(1, IPv4, lo, 5000, INVALID_ADDRESS, nullptr, 0, 38.8, -77.0,
                                 12, 2, std::vector<uint8_t>{0xfe, 0xed, 0xbe, 0xef});
  const uint32_t f2 = sb.AddFlow(2, IPv6, v6, 6000);
  const uint32_t n = 1000;
  std::vector<uint16_t> size(n);
  for (uint32_t i = 0; i < n; i++) {
    struct timeval tv;
    tv.tv_sec = 1700000000 + i / 1000;
    tv.tv_usec = (i * 1000) % 1000000;
    size[i] = (uint16_t)(64 + (i * 37) % 961);
    sb.Add(i % 2 ? f2 : f1, i / 2, tv, size[i]);
  }
  const std::vector<uint32_t>& len = sb.Pack(/*checksum=*/true);
  RecvBatch rb(ctx, n, MGENX_MAX_SIZE);
  for (uint32_t i = 0; i < n; i++) {
    CHECK(len[i] == size[i]);
    std::memcpy(rb.Slot(i), sb.Datagram(i), len[i]);
    rb.SetLength(i, len[i]);
  }
  rb.Unpack(n);
  for (uint32_t i = 0; i < n; i++) {
    MgenMsgView m = rb[i];
    CHECK(m.GetError() == ERROR_NONE);
    CHECK(m.GetFlowId() == (i % 2 ? 2u : 1u));
    CHECK(m.GetSeqNum() == i / 2);
    CHECK(m.GetMsgLen() == size[i]);
    CHECK(m.GetTxTime().tv_usec == (long)((i * 1000) % 1000000));
    CHECK(m.FlagIsSet(LAST_BUFFER));
    // Pack sets CHECKSUM only when msgLen > header + 4 (mgenMsg.cpp:296-300)
    const uint32_t hdr = i % 2 ? 60 : 52;
    CHECK(m.FlagIsSet(CHECKSUM) == (size[i] > hdr + 4));
    CHECK(m.GetDstAddrType() == (i % 2 ? IPv6 : IPv4));
    CHECK(m.GetDstPort() == (i % 2 ? 6000 : 5000));
    if (i % 2 == 0 && size[i] >= 52) CHECK(m.GetPayloadLength() == 4);
  }
  rb.Slot(7)[size[7] / 2] ^= 0x10;  // one flipped bit
  rb.Unpack(n);
  CHECK(rb[7].GetError() == ERROR_CHECKSUM);
  CHECK(rb[6].GetError() == ERROR_NONE);
  rb.Slot(7)[size[7] / 2] ^= 0x10;
  rb.Unpack(n);

  FlowAnalytics fa(ctx, 8, 0.1, 64);
  std::vector<uint32_t> idx(n), rxs(n), rxu(n);
  for (uint32_t i = 0; i < n; i++) {
    idx[i] = fa.FindFlow("10.0.0.1/5001", i % 2 ? "::1/6000" : "127.0.0.1/5000", rb[i].GetFlowId());
    const struct timeval tx = rb[i].GetTxTime();
    const uint64_t us = (uint64_t)tx.tv_sec * 1000000 + tx.tv_usec + 250;
    rxs[i] = (uint32_t)(us / 1000000);
    rxu[i] = (uint32_t)(us % 1000000);
  }
  fa.Update(rb, idx, rxs, rxu);
  std::vector<mgenx_flow_report> reps = fa.Reports();
  CHECK(reps.size() >= 8);
  for (const mgenx_flow_report& r : reps) {
    CHECK(r.loss == 0.0);
    CHECK(r.latency_min > 2.4e-4 && r.latency_max < 2.6e-4);
  }
  std::printf("host_roundtrip ok: %u records, %zu reports\n", n, reps.size());
  return 0;
}
