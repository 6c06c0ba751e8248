// mgenx_api.hip -- C ABI (include/mgenx.h) over the gfx950 kernels.
//
// The context owns only constant tables (CRC shift operators, x^(8n) mod P, the random
// fill stream); every data buffer belongs to the caller.  No entry point allocates,
// synchronises or copies from host memory except mgenx_ctx_create and
// mgenx_pack_prepare (table setup), so batch calls can be captured in a hipGraph.
#include <hipcub/hipcub.hpp>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <emmintrin.h>
#include <atomic>
#include <mutex>
#include <vector>


#include "mgenx_kernels.hpp"
#if MGENX_DIAG
#include "mgenx_diag.h"
#endif

extern "C" void* mgenx_scan_ws_new();
extern "C" void mgenx_scan_ws_free(void* p);
extern "C" int mgenx_scan_run(void* ws, const uint8_t* s, uint64_t nbytes, int mode,
                              uint64_t* rec_off, uint32_t* rec_len, uint64_t cap,
                              mgenx_scan_info* info, hipStream_t stream, char* err, size_t errn);
extern "C" int mgenx_scan_exits_run(void* ws, const uint8_t* s, uint64_t nbytes, int mode,
                                    uint64_t window, uint64_t limit, uint64_t* entries,
                                    uint64_t* exits, uint32_t cap, uint32_t* candidates,
                                    hipStream_t stream, char* err, size_t errn);
extern "C" int mgenx_scan_range_run(void* ws, const uint8_t* s, uint64_t nbytes, int mode,
                                    uint64_t entry, uint64_t limit, int reuse, uint64_t* rec_off,
                                    uint32_t* rec_len, uint64_t cap, mgenx_scan_info* info,
                                    hipStream_t stream, char* err, size_t errn);

extern "C" void* mgenx_log_ws_new();
extern "C" int mgenx_report_build_run(const mgenx_flow_report* reps, uint32_t n_flows,
                                      uint32_t per_flow, const uint32_t* count,
                                      const mgenx_report_key* keys, uint8_t* sign,
                                      const double* offset, const double* rq, uint8_t* items,
                                      uint8_t* item_len, hipStream_t stream);
extern "C" int mgenx_report_lines(void* ws, const uint8_t* items, const mgenx_flow_report* reps,
                                  const uint32_t* count, uint32_t per_flow, const uint64_t* pairs,
                                  const uint8_t* slab, const mgenx_addr* reporter,
                                  const uint32_t* rx_sec, const uint32_t* rx_usec, uint32_t n,
                                  uint32_t opts, const double* rq, char* text, uint64_t cap,
                                  uint64_t* line_off, hipStream_t stream, char* err, size_t errn);
extern "C" int mgenx_log_send_exec(void* ws, const mgenx_flow_tmpl* tmpl,
                                   const mgenx_pack_desc* desc, const uint16_t* src_port,
                                   const uint32_t* out_len, const uint32_t* msg_total,
                                   const uint8_t* slab, uint64_t slab_bytes,
                                   const uint64_t* rec_off, uint64_t stride, uint32_t n,
                                   int protocol, uint32_t opts, bool binary, uint8_t* out,
                                   uint64_t out_cap, uint64_t* pos, hipStream_t stream,
                                   char* err, size_t errn);
extern "C" int mgenx_data_walk_exec(void* ws, const uint8_t* slab, const uint64_t* rec_off,
                                    uint64_t stride, const mgenx_cols* cols, uint32_t n,
                                    uint32_t opts, const double* rq, uint8_t* status,
                                    uint8_t* needs_host, uint32_t* cmds, uint32_t cmd_cap,
                                    uint64_t* reps, uint32_t rep_cap, uint32_t* totals,
                                    hipStream_t stream, char* err, size_t errn);
extern "C" void mgenx_log_ws_free(void* p);
extern "C" int mgenx_text_interleave_run(void* ws, const mgenx_text_src* srcs, uint32_t n_src,
                                         uint32_t n_rec, char* out, uint64_t cap,
                                         uint64_t* rec_off, hipStream_t stream, char* err,
                                         size_t errn);
extern "C" int mgenx_pcap_parse_run(const uint8_t* dev_buf, uint64_t buf_bytes,
                                    const uint64_t* dev_pkt_off, uint32_t n, uint32_t link_type,
                                    uint32_t flags, uint64_t* dev_udp_off, uint32_t* dev_udp_len,
                                    mgenx_addr* dev_src, int32_t* dev_ttl, uint32_t* dev_rx_sec,
                                    uint32_t* dev_rx_usec, uint8_t* dev_status,
                                    hipStream_t stream);
extern "C" int mgenx_pcap_snap_run(uint8_t* dev_buf, uint64_t file_bytes, uint64_t buf_bytes,
                                   const uint64_t* dev_pkt_off, uint32_t n, uint32_t flags,
                                   uint8_t* dev_status, uint64_t* dev_udp_off,
                                   uint32_t* dev_udp_len, uint64_t* need, void* scan_tmp,
                                   size_t scan_bytes, hipStream_t stream);
extern "C" size_t mgenx_pcap_snap_scan_bytes(uint32_t n);
extern "C" int mgenx_log_recv_run(void* ws, bool binary, const uint8_t* slab,
                                  uint64_t slab_bytes, const uint64_t* rec_off,
                                  const uint32_t* rec_len,
                                       uint64_t stride, const mgenx_cols* cols,
                                       const mgenx_addr* src, const uint32_t* rx_sec,
                                       const uint32_t* rx_usec, const int32_t* ttl, uint32_t n,
                                       int protocol, uint32_t opts, char* text,
                                       uint64_t text_cap, uint64_t* line_off,
                                       hipStream_t stream, char* err, size_t errn);
extern "C" void* mgenx_flow_ws_new();
extern "C" void mgenx_flow_ws_free(void* p);
extern "C" int mgenx_flow_init_run(mgenx_flow_state* flows, uint32_t n_flows, double window,
                                   hipStream_t stream);
extern "C" int mgenx_flow_export_run(const mgenx_flow_state* flows, uint32_t n_flows,
                                     mgenx_flow_counters* out, hipStream_t stream);
extern "C" int mgenx_flow_reduce_run(void* ws, const uint32_t* flow_idx, const uint32_t* seq,
                                     const uint32_t* txs, const uint32_t* txu, const uint16_t* len,
                                     const mgenx_rec* rows,
                                     const uint32_t* rxs, const uint32_t* rxu, uint32_t n,
                                     mgenx_flow_state* flows, uint32_t n_flows,
                                     mgenx_flow_report* reports, uint32_t per_flow,
                                     uint32_t* report_count, uint32_t* report_rec,
                                     hipStream_t stream, char* err, size_t errn);

extern "C" int mgenx_binlog_parse_exec(const uint8_t* buf, const uint64_t* rec_off, uint32_t n,
                                       uint64_t* msg_off, uint32_t* msg_len, mgenx_addr* src,
                                       uint32_t* ev_sec, uint32_t* ev_usec, uint32_t* aux,
                                       uint8_t* kind, uint8_t* proto, hipStream_t stream);
extern "C" int mgenx_binlog_lines_exec(void* wsp, const uint8_t* buf, const uint64_t* rec_off,
                                       uint32_t n, uint64_t* msg_off, uint32_t* msg_len,
                                       mgenx_addr* src, uint32_t* ev_sec, uint32_t* ev_usec,
                                       uint32_t* aux, uint8_t* kind, uint8_t* proto,
                                       const mgenx_cols* cols, uint32_t log_rx, uint32_t flush,
                                       uint32_t opts, char* text, uint64_t cap,
                                       uint64_t* line_off, hipStream_t stream, char* err,
                                       size_t errn);

// a device buffer that grows on demand (the composite calls' intermediate arrays)
struct mgenx_grow {
  void* p = nullptr;
  size_t n = 0;
  void* get(size_t need) {
    if (n < need) {
      mgenx::dev_free(p);
      p = nullptr;
      n = 0;
      if (hipMalloc(&p, need) != hipSuccess) return nullptr;
      n = need;
    }
    return p;
  }
  void release() {
    mgenx::dev_free(p);
    p = nullptr;
    n = 0;
  }
};

struct mgenx_ctx {
  int device = 0;
  int cu_count = 0;
  uint32_t* d_tabs = nullptr;     // [A64 | A4 | A8 | A12 | A16 | A32 | A48 | A128 | A256 | A512 | A1024]
  uint32_t* d_expect = nullptr;   // [65536]
  std::vector<uint32_t> h_expect;  // host copy of the expect table
  uint32_t* d_xpow = nullptr;     // [65536]
  uint32_t* d_ia = nullptr;       // [65536]
  uint32_t* d_bytetab = nullptr;  // [256]
  uint8_t* d_rtab = nullptr;      // 16 + 65536 + 32 bytes
  uint32_t* d_rcrc = nullptr;     // [65536]
  uint8_t* d_sink = nullptr;      // 1 KiB: column stores of lanes past the batch end
  double* d_rq = nullptr;         // report quantizer tables (mgenx::kRq*), built with host libm
  void* scan_ws = nullptr;        // stream-scan workspace (mgenx_scan.hip), grown on demand
  void* flow_ws = nullptr;        // flow-reduce workspace (mgenx_analytic.hip), grown on demand
  void* log_ws = nullptr;         // log-format workspace (mgenx_log.hip), grown on demand
  void* tcp_ws = nullptr;         // TCP transmit workspace (mgenx_pack_tcp), grown on demand
  size_t tcp_ws_bytes = 0;
  uint64_t* tcp_host = nullptr;   // host-mapped words: the plan's verdict (16 bytes)
  void* tcp_plan = nullptr;       // the plan's maximum word, skip word and look-back words
  uint32_t tcp_plan_blocks = 0;   // (look-back words it holds)
  uint32_t tcp_epoch = 0;         // the plan's epoch (its words are cleared when it wraps)
  void* rx_ws = nullptr;          // rx-persist workspace, grown on demand
  size_t rx_ws_bytes = 0;
  uint64_t* tcp_host_dev = nullptr;
  int unpack_variant = 0;          // diagnostic kernel ablation (mgenx_set_tuning)
  int unpack_last = 0;             // MGENX_UNPACK_K_* of the last mgenx_unpack_batch
  int pack_variant = 0;
  mgenx_grow bl[5];                // mgenx_convert_binary_log: records, lines, pairs, report text
  mgenx_grow snap;                 // mgenx_pcap_snap: per-packet sizes + scan scratch
  bool rand_ready = false;
  uint32_t rand_time = 0;
  std::vector<mgenx_worker*> workers;  // live workers on this context (stopped by ctx destroy)
  char err[256] = {0};
};
static void worker_detach(mgenx_worker* w);

namespace {

constexpr uint32_t kN = 65536;

void byte_table(uint32_t t[256]) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (mgenx::kPoly ^ (c >> 1)) : (c >> 1);
    t[i] = c;
  }
}

// A_n(s): the state after n zero bytes.
uint32_t shift_n(const uint32_t t[256], uint32_t s, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) s = t[s & 0xffu] ^ (s >> 8);
  return s;
}

// MgenAnalytic::Report quantizers (mgenAnalytic.cpp:568-642) as tables built with this
// host's libm -- the reference's own log / log10 / pow: the device quantizes by threshold
// search and unquantizes by lookup, so it matches the host bit for bit.
double rq_scale() { return 1.0 / (pow(1.1, 254) - 1.1); }
uint8_t host_q_time(double value) {
  const double S = 1.1, MN = 1.0e-06, MX = 600.0;
  if (value > S * MX) return 0xff;
  if (value < MN / 2.0) return 0;
  if (value < MN) return 1;
  return (uint8_t)((log(S + (value - MN) / (rq_scale() * (MX - MN))) / log(S)) + 0.5);
}
// smallest positive double v in [lo, hi] with pred(v) (pred monotone, false -> true)
template <typename P>
double first_true(double lo, double hi, P pred) {
  uint64_t a, b;
  memcpy(&a, &lo, 8);
  memcpy(&b, &hi, 8);
  while (a < b) {
    const uint64_t m = a + (b - a) / 2;
    double v;
    memcpy(&v, &m, 8);
    if (pred(v)) b = m; else a = m + 1;
  }
  double v;
  memcpy(&v, &a, 8);
  return v;
}
void build_report_tables(double* rq) {
  const double S = 1.1, MN = 1.0e-06, MX = 600.0;
  for (int q = 0; q < 256; q++)
    rq[mgenx::kRqUnqTime + q] = q == 0 ? 0.0 : (MX - MN) * (pow(S, q) - S) * rq_scale() + MN;
  // time: T[k] = first v >= MIN with q(v) >= k, k = 2..255 (q(MIN) = 1)
  for (int k = 0; k < 256; k++) rq[mgenx::kRqThrTime + k] = HUGE_VAL;
  for (int k = 2; k < 256; k++)
    rq[mgenx::kRqThrTime + k] = first_true(MN, S * MX, [&](double v) { return host_q_time(v) >= k; });
  // rate exponent: (int)log10(r) >= e, e = kRqLog10Lo .. kRqLog10Lo + kRqLog10N - 1
  for (int j = 0; j < mgenx::kRqLog10N; j++) {
    const int e = mgenx::kRqLog10Lo + j;
    rq[mgenx::kRqThrLog10 + j] =
        first_true(1e-300, 1e300, [&](double v) { return (int32_t)log10(v) >= e; });
  }
  for (int e = 0; e < mgenx::kRqP10N; e++) rq[mgenx::kRqP10 + e] = pow(10.0, (double)e);
}

void op_table(const uint32_t t[256], uint32_t n, uint32_t* out /*1024*/) {
  for (uint32_t k = 0; k < 4; k++)
    for (uint32_t v = 0; v < 256; v++) out[k * 256 + v] = shift_n(t, v << (8 * k), n);
}

// glibc random_r TYPE_3 after srand(seed): the RANDOM_FILL byte source
// (src/common/mgenMsg.cpp:277-292 calls srand(time(NULL)) then (char)rand()).
void glibc_rand_bytes(uint32_t seed, uint32_t n, uint8_t* out) {
  int32_t r[31];
  int32_t word = (int32_t)(seed == 0 ? 1u : seed);
  r[0] = word;
  for (int i = 1; i < 31; i++) {
    const long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    r[i] = word;
  }
  uint32_t ring[34];
  for (int i = 0; i < 31; i++) ring[i] = (uint32_t)r[i];
  for (int i = 31; i < 34; i++) ring[i] = ring[i - 31];
  uint32_t made = 0;
  for (uint64_t i = 34; made < n; i++) {
    const uint32_t v = ring[(i - 31) % 34] + ring[(i - 3) % 34];
    ring[i % 34] = v;
    if (i >= 344) out[made++] = (uint8_t)(v >> 1);
  }
}

int set_err(mgenx_ctx* c, hipError_t e, const char* where) {
  if (c) snprintf(c->err, sizeof(c->err), "%s: %s", where, hipGetErrorString(e));
  return MGENX_EDEVICE;
}

}  // namespace

extern "C" {

int mgenx_abi_version(void) { return MGENX_ABI_VERSION; }

const char* mgenx_last_error(const mgenx_ctx* ctx) { return ctx ? ctx->err : "null ctx"; }

int mgenx_ctx_create(int device, mgenx_ctx** out) {
  if (!out) return MGENX_EINVAL;
  *out = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return MGENX_EDEVICE;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return MGENX_EDEVICE;
  mgenx_ctx* c = new mgenx_ctx();
  c->device = device;
  c->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;

  uint32_t t[256];
  byte_table(t);
  // operator tables: [A64 | A4 | A8 | A12 | A16 | A32 | A48] (unpack), [A128 | A256 | A512 |
  // A1024] (the worker's shifts by any distance, mgenx::kTabA128..)
  std::vector<uint32_t> tabs(11 * 1024), xpow(kN), ia(kN), expect(kN, 0);
  const uint32_t ops[11] = {64, 4, 8, 12, 16, 32, 48, 128, 256, 512, 1024};
  for (int i = 0; i < 11; i++) op_table(t, ops[i], &tabs[1024 * i]);
  xpow[0] = 0x80000000u;  // x^0
  for (uint32_t n = 1; n < kN; n++) xpow[n] = mgenx::multmodp(xpow[n - 1], 0x00800000u);
  for (uint32_t n = 0; n < kN; n++) ia[n] = mgenx::multmodp(xpow[n], 0xFFFFFFFFu);
  // self-check: x^(8n) multiplication is the n-zero-byte shift operator
  for (uint32_t n : {1u, 3u, 64u, 1000u}) {
    if (mgenx::multmodp(xpow[n], 0x12345678u) != shift_n(t, 0x12345678u, n)) {
      delete c;
      return MGENX_EINVAL;
    }
  }
  for (uint32_t L = 4; L < kN; L++) expect[L] = shift_n(t, ia[L - 4] ^ 0xFFFFFFFFu, 4);
  c->h_expect = expect;
  std::vector<double> rq(mgenx::kRqDoubles);
  build_report_tables(rq.data());

  struct {
    void** p;
    size_t bytes;
    const void* src;
  } allocs[] = {
      {(void**)&c->d_tabs, tabs.size() * 4, tabs.data()},
      {(void**)&c->d_expect, kN * 4, expect.data()},
      {(void**)&c->d_xpow, kN * 4, xpow.data()},
      {(void**)&c->d_ia, kN * 4, ia.data()},
      {(void**)&c->d_bytetab, 256 * 4, t},
      {(void**)&c->d_rtab, 16 + kN + 32, nullptr},
      {(void**)&c->d_rcrc, kN * 4, nullptr},
      {(void**)&c->d_sink, 1024, nullptr},
      {(void**)&c->d_rq, rq.size() * 8, rq.data()},
  };
  for (auto& a : allocs) {
    if (hipMalloc(a.p, a.bytes) != hipSuccess) {
      mgenx_ctx_destroy(c);
      return MGENX_ENOMEM;
    }
    e = a.src ? hipMemcpy(*a.p, a.src, a.bytes, hipMemcpyHostToDevice)
              : hipMemset(*a.p, 0, a.bytes);
    if (e != hipSuccess) {
      mgenx_ctx_destroy(c);
      return MGENX_EDEVICE;
    }
  }
  *out = c;
  return MGENX_OK;
}

int mgenx_ctx_destroy(mgenx_ctx* c) {
  if (!c) return MGENX_EINVAL;
  hipSetDevice(c->device);
  // workers first: their waves read this context's tables.  Each is stopped and its mailbox
  // freed; the handle stays valid for mgenx_worker_destroy, and its calls return MGENX_EINVAL
  for (mgenx_worker* w : c->workers) worker_detach(w);
  c->workers.clear();
  void* ps[] = {c->d_tabs, c->d_expect, c->d_xpow, c->d_ia, c->d_bytetab, c->d_rtab, c->d_rcrc,
                c->d_sink, c->d_rq};
  if (c->scan_ws) mgenx_scan_ws_free(c->scan_ws);
  if (c->flow_ws) mgenx_flow_ws_free(c->flow_ws);
  if (c->log_ws) mgenx_log_ws_free(c->log_ws);
  mgenx::dev_free(c->tcp_ws);
  mgenx::dev_free(c->tcp_plan);
  mgenx::dev_free(c->rx_ws);
  mgenx::host_free(c->tcp_host);
  for (mgenx_grow& g : c->bl) g.release();
  c->snap.release();
  for (void* p : ps) mgenx::dev_free(p);
  delete c;
  return MGENX_OK;
}

int mgenx_unpack_batch(mgenx_ctx* ctx, const uint8_t* dev_slab, uint64_t slab_bytes,
                       const uint64_t* dev_rec_off, uint64_t stride,
                       const uint32_t* dev_rec_len, uint32_t fixed_len, uint32_t n,
                       const mgenx_cols* cols, uint32_t opts, void* stream) {
  if (!ctx || !cols) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_slab) return MGENX_EINVAL;
  if (!dev_rec_off && stride == 0 && n > 1) return MGENX_EINVAL;
  const mgenx_cols& k = *cols;
  if (!k.rows && (!k.flow_id || !k.seq_num || !k.tx_sec || !k.tx_usec || !k.msg_len ||
                  !k.dst_port || !k.flags || !k.err || !k.dst_type || !k.dst_len ||
                  !k.dst_addr4 || !k.payload_len || !k.payload_type || !k.gps_status))
    return MGENX_EINVAL;
  mgenx::UnpackParams p;
  p.slab = dev_slab;
  p.slab_bytes = slab_bytes;
  p.rec_off = dev_rec_off;
  p.stride = stride;
  p.rec_len = dev_rec_len;
  p.fixed_len = fixed_len;
  p.n = n;
  p.opts = opts;
  p.tabs = ctx->d_tabs;
  p.expect = ctx->d_expect;
  p.expect_fixed = fixed_len < ctx->h_expect.size() ? ctx->h_expect[fixed_len] : 0u;
  p.sink = ctx->d_sink;
  p.variant = MGENX_DIAG ? ctx->unpack_variant : 0;
  p.cols = k;
  const uint64_t groups = ((uint64_t)n + 15) / 16;
  const uint64_t per_block = (uint64_t)mgenx::unpack_threads() / 64;  // waves per block
  uint64_t grid = (groups + per_block - 1) / per_block;
  if (grid > (uint64_t)ctx->cu_count) grid = ctx->cu_count;
  hipError_t e = mgenx::launch_unpack(p, (int)grid, (hipStream_t)stream, &ctx->unpack_last);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "unpack");
}

int mgenx_unpack_last_kernel(const mgenx_ctx* ctx) { return ctx ? ctx->unpack_last : 0; }

int mgenx_pack_prepare(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl, uint32_t n_tmpl,
                       const uint8_t* dev_pool, uint32_t* dev_tmpl_crc, void* stream) {
  if (!ctx || (n_tmpl && (!dev_tmpl || !dev_tmpl_crc))) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_pack_prepare(dev_tmpl, n_tmpl, dev_pool, ctx->d_bytetab,
                                            dev_tmpl_crc, (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "pack_prepare");
}

int mgenx_set_fill_time(mgenx_ctx* ctx, uint32_t fill_time) {
  if (!ctx) return MGENX_EINVAL;
  if (ctx->rand_ready && ctx->rand_time == fill_time) return MGENX_OK;
  std::vector<uint8_t> rt(16 + kN + 32, 0);
  glibc_rand_bytes(fill_time, kN, &rt[16]);
  uint32_t t[256];
  byte_table(t);
  std::vector<uint32_t> rc(kN);
  uint32_t c = 0;
  for (uint32_t k = 0; k < kN; k++) {
    rc[k] = c;
    c = t[(c ^ rt[16 + k]) & 0xffu] ^ (c >> 8);
  }
  hipSetDevice(ctx->device);
  hipError_t e = hipMemcpy(ctx->d_rtab, rt.data(), rt.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(ctx->d_rcrc, rc.data(), kN * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return set_err(ctx, e, "set_fill_time");
  ctx->rand_ready = true;
  ctx->rand_time = fill_time;
  return MGENX_OK;
}

static int pack_common(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                       const uint32_t* dev_tmpl_crc, const mgenx_pack_desc* dev_desc, uint32_t n,
                       const uint8_t* dev_pool, uint8_t* dev_slab, uint64_t slab_bytes,
                       const uint64_t* dev_rec_off, uint64_t stride, const uint32_t* dev_buf_len,
                       const uint32_t* dev_crc_in, uint32_t* dev_out_len, uint32_t* dev_tx_crc,
                       uint32_t* dev_state, uint32_t opts, uint32_t fill_time, void* stream,
                       const uint32_t* dev_frag_len = nullptr, int frag_ck = 0,
                       const uint32_t* dev_skip = nullptr) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_tmpl || !dev_tmpl_crc || !dev_desc || !dev_slab || !dev_out_len) return MGENX_EINVAL;
  if (!dev_rec_off && stride == 0 && n > 1) return MGENX_EINVAL;
  if (opts & MGENX_PACK_RANDOM_FILL) {
    if (!ctx->rand_ready || ctx->rand_time != fill_time) return MGENX_EINVAL;
  }
  mgenx::PackParams p;
  p.tmpl = dev_tmpl;
  p.tmpl_crc = dev_tmpl_crc;
  p.desc = dev_desc;
  p.n = n;
  p.pool = dev_pool;
  p.slab = dev_slab;
  p.slab_bytes = slab_bytes;
  p.rec_off = dev_rec_off;
  p.stride = stride;
  p.out_len = dev_out_len;
  p.opts = opts;
  p.byte_tab = ctx->d_bytetab;
  p.a4_tab = ctx->d_tabs + 1024;  // [A_64 | A_4 | ...]
  p.variant = MGENX_DIAG ? ctx->pack_variant : 0;
  p.xpow = ctx->d_xpow;
  p.ia = ctx->d_ia;
  p.rtab = ctx->d_rtab;
  p.rcrc = ctx->d_rcrc;
  p.buf_len = dev_buf_len;
  p.crc_in = dev_crc_in;
  p.tx_crc = dev_tx_crc;
  p.state = dev_state;
  p.frag_len = dev_frag_len;
  p.frag_ck = frag_ck;
  p.skip = dev_skip;
  const uint64_t batches = ((uint64_t)n + 63) / 64;
  uint64_t grid = (batches + 3) / 4;                // groups of 4 batches (kProd)
  // 76 KB of LDS per workgroup: two per CU, except for the aligned-stride layout (the
  // recvmmsg slots, config 2), whose joint 4-KB-chunk store runs faster with one workgroup --
  // eight waves -- per CU (config 2: 0.199 against 0.211 ms; config 3's packed slab the other
  // way: 0.214 against 0.188 ms)
  const bool stride_layout = !dev_rec_off && !dev_frag_len && !(opts & MGENX_PACK_RANDOM_FILL) &&
                             (stride & 15u) == 0 && stride >= 32 && stride <= 65536;
  uint64_t cap = (uint64_t)ctx->cu_count * (stride_layout ? 1u : 2u);
  if (MGENX_DIAG && ctx->pack_variant >= 7 && ctx->pack_variant <= 9)
    cap *= (uint64_t)(ctx->pack_variant - 5);  // (diag)
#if MGENX_DIAG
  if (const char* v = getenv("MGENX_PACK_GRID")) cap = (uint64_t)std::max(1, atoi(v));  // (diag)
#endif
  if (grid > cap) grid = cap;
  hipError_t e = mgenx::launch_pack(p, (int)grid, (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "pack");
}

int mgenx_pack_batch(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                     const uint32_t* dev_tmpl_crc, const mgenx_pack_desc* dev_desc, uint32_t n,
                     const uint8_t* dev_pool, uint8_t* dev_slab, uint64_t slab_bytes,
                     const uint64_t* dev_rec_off, uint64_t stride, uint32_t* dev_out_len,
                     uint32_t opts, uint32_t fill_time, void* stream) {
  if (opts & MGENX_PACK_RAW) return MGENX_EINVAL;  // mgenx_pack_msgs is the raw form
  return pack_common(ctx, dev_tmpl, dev_tmpl_crc, dev_desc, n, dev_pool, dev_slab, slab_bytes,
                     dev_rec_off, stride, nullptr, nullptr, dev_out_len, nullptr, nullptr, opts,
                     fill_time, stream);
}

int mgenx_pack_msgs(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                    const uint32_t* dev_tmpl_crc, const mgenx_pack_desc* dev_desc, uint32_t n,
                    const uint8_t* dev_pool, uint8_t* dev_slab, uint64_t slab_bytes,
                    const uint64_t* dev_rec_off, uint64_t stride, const uint32_t* dev_buf_len,
                    const uint32_t* dev_crc_in, uint32_t* dev_out_len, uint32_t* dev_tx_crc,
                    uint32_t* dev_state, uint32_t opts, uint32_t fill_time, void* stream) {
  return pack_common(ctx, dev_tmpl, dev_tmpl_crc, dev_desc, n, dev_pool, dev_slab, slab_bytes,
                     dev_rec_off, stride, dev_buf_len, dev_crc_in, dev_out_len, dev_tx_crc,
                     dev_state, opts | MGENX_PACK_RAW, fill_time, stream);
}

// the stream length and the round count (the plan kernel's maximum fragment count) for
// the host, in one 16-byte copy (the exact path)
__global__ void tcp_totals_kernel(const uint32_t* max_frag, uint32_t n, const uint64_t* off,
                                  const uint64_t* bytes, uint64_t* out) {
  out[0] = off[n - 1] + bytes[n - 1];  // (the exclusive scan's last offset + its message)
  out[1] = *max_frag;
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

int mgenx_pack_tcp(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl, const uint32_t* dev_tmpl_crc,
                   const mgenx_pack_desc* dev_desc, const uint32_t* dev_msg_total, uint32_t n,
                   const uint8_t* dev_pool, uint8_t* dev_stream, uint64_t stream_cap,
                   uint64_t* dev_msg_off, uint64_t* total_bytes, uint32_t opts,
                   uint32_t fill_time, void* stream) {
  if (!ctx || !total_bytes || (opts & ~(uint32_t)(MGENX_PACK_CHECKSUM | MGENX_PACK_RANDOM_FILL)))
    return MGENX_EINVAL;
  *total_bytes = 0;
  if (n == 0) return MGENX_OK;
  if (!dev_tmpl || !dev_tmpl_crc || !dev_desc || !dev_msg_total || !dev_msg_off)
    return MGENX_EINVAL;
  if ((opts & MGENX_PACK_RANDOM_FILL) && (!ctx->rand_ready || ctx->rand_time != fill_time))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (!ctx->tcp_host) {
    void* hp = nullptr;
    void* dp = nullptr;
    if ((e = hipHostMalloc(&hp, 64, hipHostMallocMapped)) != hipSuccess) return set_err(ctx, e, "tcp");
    memset(hp, 0, 64);
    ctx->tcp_host = static_cast<uint64_t*>(hp);
    if ((e = hipHostGetDevicePointer(&dp, hp, 0)) != hipSuccess) return set_err(ctx, e, "tcp");
    ctx->tcp_host_dev = static_cast<uint64_t*>(dp);
  }
  // workspace: bytes[n], nfrag[n], cub (a scan of n items); per round: fd, foff, fbuf, ff,
  // plen, crc, state x2; the maximum fragment count (exact path)
  size_t cub_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, (const uint64_t*)nullptr,
                                         (uint64_t*)nullptr, (int)n, s);
  const size_t b8 = a256((size_t)n * 8), b4 = a256((size_t)n * 4);
  const size_t need = b8 + b4 + a256(cub_bytes) + a256((size_t)n * sizeof(mgenx_pack_desc)) +
                      b8 + 4 * b4 + 2 * b4 + 256;
  if (ctx->tcp_ws_bytes < need) {
    mgenx::dev_free(ctx->tcp_ws);
    ctx->tcp_ws = nullptr;
    ctx->tcp_ws_bytes = 0;
    if ((e = hipMalloc(&ctx->tcp_ws, need)) != hipSuccess) return set_err(ctx, e, "tcp workspace");
    ctx->tcp_ws_bytes = need;
  }
  char* w = static_cast<char*>(ctx->tcp_ws);
  auto take = [&](size_t b) { char* q = w; w += b; return q; };
  uint64_t* bytes = (uint64_t*)take(b8);
  uint32_t* nfrag = (uint32_t*)take(b4);
  void* cub = take(a256(cub_bytes));
  mgenx_pack_desc* fd = (mgenx_pack_desc*)take(a256((size_t)n * sizeof(mgenx_pack_desc)));
  uint64_t* foff = (uint64_t*)take(b8);
  uint32_t* fbuf = (uint32_t*)take(b4);
  uint32_t* ff = (uint32_t*)take(b4);
  uint32_t* plen = (uint32_t*)take(b4);
  uint32_t* crc = (uint32_t*)take(b4);
  uint32_t* st[2] = {(uint32_t*)take(b4), (uint32_t*)take(b4)};
  uint32_t* max_frag = (uint32_t*)take(256);
  // the plan's words, in their own allocation (epoch-tagged: they must keep their place
  // whatever n the next call brings): the skip word, then a look-back word and a maximum word
  // a block
  const uint32_t blocks = (n + mgenx::kTcpPlanMsgs - 1) / mgenx::kTcpPlanMsgs;
  if (ctx->tcp_plan_blocks < blocks) {
    mgenx::dev_free(ctx->tcp_plan);
    ctx->tcp_plan = nullptr;
    ctx->tcp_plan_blocks = 0;
    const size_t pb = 256 + (size_t)blocks * 16;
    if ((e = hipMalloc(&ctx->tcp_plan, pb)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->tcp_plan, 0, pb, s)) != hipSuccess)
      return set_err(ctx, e, "tcp workspace");
    ctx->tcp_plan_blocks = blocks;
  }
  if (++ctx->tcp_epoch >= mgenx::kTcpPlanEpochs) {  // wrap: clear the words (nothing in flight)
    if ((e = hipStreamSynchronize(s)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->tcp_plan, 0, 256 + (size_t)ctx->tcp_plan_blocks * 16, s)) !=
            hipSuccess)
      return set_err(ctx, e, "tcp plan");
    memset(ctx->tcp_host, 0, 64);
    ctx->tcp_epoch = 1;
  }
  const uint32_t epoch = ctx->tcp_epoch;
  uint32_t* skip = static_cast<uint32_t*>(ctx->tcp_plan);
  uint64_t* status = reinterpret_cast<uint64_t*>(static_cast<char*>(ctx->tcp_plan) + 256);
  uint64_t* fmax = status + ctx->tcp_plan_blocks;
  const int ck = (opts & MGENX_PACK_CHECKSUM) ? 1 : 0;
  // round r: fragment descriptors (round 0's come with the plan), then Pack -- which also
  // stores the later buffers' copies, runs the CRC on through them and writes the trailer
  auto round = [&](uint32_t r, const uint32_t* gate) -> int {
    if (r > 0 && (e = mgenx::launch_tcp_frag(dev_desc, dev_msg_total, nfrag, dev_msg_off, n, r,
                                             ck, st[(r + 1) & 1], fd, foff, fbuf, ff, s)) !=
                     hipSuccess)
      return set_err(ctx, e, "tcp fragments");
    // (round 0's fragments start at the message offsets)
    return pack_common(ctx, dev_tmpl, dev_tmpl_crc, fd, n, dev_pool, dev_stream, stream_cap,
                       r == 0 ? dev_msg_off : foff, 0, fbuf, nullptr, plen, crc, st[r & 1],
                       opts | MGENX_PACK_RAW, fill_time, stream, ff, ck, gate);
  };
  // One launch plans every message, scans the offsets straight into the caller's array and
  // writes round 0's descriptors; round 0 is queued behind it before the host has read the
  // plan (gated on the device: when the stream exceeds stream_cap, or the plan failed, it
  // stores nothing), so the GPU never waits for the host between back-to-back calls.  The
  // host then spins on the plan's 16-byte verdict in host memory (not the stream's
  // completion: round 0 keeps running), and queues any further rounds.
  if ((e = mgenx::launch_tcp_plan0(dev_tmpl, dev_desc, dev_msg_total, n, ck, stream_cap, epoch,
                                   status, fmax, dev_msg_off, nfrag, fd, fbuf, ff, skip,
                                   ctx->tcp_host_dev, s)) != hipSuccess)
    return set_err(ctx, e, "tcp plan");
  const bool spec = dev_stream != nullptr;
  if (spec) {
    const int rc = round(0, skip);
    if (rc != MGENX_OK) return rc;
  }
  auto verdict = [&]() {
    const __m128i x = _mm_load_si128(reinterpret_cast<const __m128i*>(ctx->tcp_host));
    return std::make_pair((uint64_t)_mm_cvtsi128_si64(x), (uint64_t)_mm_extract_epi64(x, 1));
  };
  std::pair<uint64_t, uint64_t> v;
  {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spins = 0;; spins++) {
      std::atomic_signal_fence(std::memory_order_seq_cst);  // (a fresh load every poll)
      v = verdict();
      if ((uint32_t)(v.second >> 48) == epoch) break;
      _mm_pause();
      if ((spins & 0xFFFF) == 0xFFFF &&
          std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return set_err(ctx, e, "tcp plan");
        v = verdict();
        if ((uint32_t)(v.second >> 48) != epoch) {
          snprintf(ctx->err, sizeof(ctx->err), "tcp plan: no verdict");
          return MGENX_EDEVICE;
        }
        break;
      }
    }
  }
  uint64_t total = v.first;
  uint32_t rounds = (uint32_t)(v.second & 0x7FFFFFFFu);
  uint32_t r0 = spec ? 1u : 0u;  // the first round still to queue
  if ((v.second >> 32) & 1u) {
    // the exact path (the plan could not vouch for its offsets; round 0 stored nothing): the
    // plan per message, the offsets by a device-wide scan, the totals read back
    if ((e = hipMemsetAsync(max_frag, 0, 4, s)) != hipSuccess ||
        (e = mgenx::launch_tcp_plan(dev_tmpl, dev_desc, dev_msg_total, n, bytes, nfrag, max_frag,
                                    s)) != hipSuccess ||
        (e = hipcub::DeviceScan::ExclusiveSum(cub, cub_bytes, (const uint64_t*)bytes, dev_msg_off,
                                              (int)n, s)) != hipSuccess)
      return set_err(ctx, e, "tcp plan");
    hipLaunchKernelGGL(tcp_totals_kernel, dim3(1), dim3(1), 0, s, max_frag, n, dev_msg_off, bytes,
                       ctx->tcp_host_dev);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return set_err(ctx, e, "tcp plan");
    total = ((volatile uint64_t*)ctx->tcp_host)[0];
    rounds = (uint32_t)((volatile uint64_t*)ctx->tcp_host)[1];
    ((volatile uint64_t*)ctx->tcp_host)[1] = 0;  // (no stale epoch for the next call)
    r0 = 0;
  }
  *total_bytes = total;
  if (total > stream_cap || (total && !dev_stream)) {
    snprintf(ctx->err, sizeof(ctx->err), "tcp: the stream needs %llu bytes",
             (unsigned long long)total);
    return MGENX_EINVAL;
  }
  for (uint32_t r = r0; r < rounds; r++) {
    if (r == 0) {  // (exact path: round 0's descriptors from the fragment kernel)
      if ((e = mgenx::launch_tcp_frag(dev_desc, dev_msg_total, nfrag, dev_msg_off, n, 0, ck,
                                      st[1], fd, foff, fbuf, ff, s)) != hipSuccess)
        return set_err(ctx, e, "tcp fragments");
    }
    const int rc = round(r, nullptr);
    if (rc != MGENX_OK) return rc;
  }
  return MGENX_OK;
}

int mgenx_tcp_rx_persist(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                         const uint32_t* dev_rec_len, uint32_t n, const mgenx_cols* cols,
                         mgenx_rx_state* dev_state, uint32_t* dev_payload_rec, uint32_t opts,
                         void* stream) {
  if (!ctx || !cols || !dev_state || (opts & ~(uint32_t)(MGENX_RX_NOLOG | MGENX_RX_FORCE)))
    return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  const mgenx_cols& c = *cols;
  if (!c.flow_id || !c.seq_num || !c.tx_sec || !c.tx_usec || !c.msg_len || !c.dst_port ||
      !c.flags || !c.err || !c.dst_type || !c.dst_len || !c.dst_addr4 || !c.payload_len ||
      !c.payload_type || !c.gps_status || !c.decoded || !dev_slab || !dev_rec_off || !dev_rec_len)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  const size_t need = mgenx::rx_persist_ws_bytes(n);
  hipError_t e;
  if (ctx->rx_ws_bytes < need) {  // grows (allocates) only when the batch outgrows it
    mgenx::dev_free(ctx->rx_ws);
    ctx->rx_ws = nullptr;
    ctx->rx_ws_bytes = 0;
    if ((e = hipMalloc(&ctx->rx_ws, need)) != hipSuccess) return set_err(ctx, e, "rx workspace");
    ctx->rx_ws_bytes = need;
  }
  e = mgenx::launch_rx_persist(c, n, opts, static_cast<int32_t*>(ctx->rx_ws), dev_state, dev_slab,
                               dev_rec_off, dev_rec_len, ctx->d_bytetab, dev_payload_rec,
                               (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "rx persist");
}

int mgenx_ctx_device(const mgenx_ctx* ctx) { return ctx ? ctx->device : -1; }

#if MGENX_DIAG
int mgenx_set_tuning(mgenx_ctx* ctx, int key, int value) {
  if (!ctx) return MGENX_EINVAL;
  if (key == MGENX_TUNE_PACK_VARIANT) {
    if (value < 0 || value > 10) return MGENX_EINVAL;
    ctx->pack_variant = value;
    return MGENX_OK;
  }
  if (key == MGENX_TUNE_UNPACK_VARIANT) {
    if (value < 0 || value > 2047) return MGENX_EINVAL;
    ctx->unpack_variant = value;
    return MGENX_OK;
  }
  return MGENX_EINVAL;
}

int mgenx_diag_stream_read(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                           uint32_t* dev_scratch, int grid, void* stream) {
  if (!ctx || !dev_data || !dev_scratch || grid <= 0) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_stream_read(dev_data, bytes, dev_scratch, grid,
                                           (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "stream_read");
}

int mgenx_diag_stream_read_w(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                             uint32_t* dev_scratch, int grid, int width, void* stream) {
  if (!ctx || !dev_data || !dev_scratch || grid <= 0) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_stream_read_w(dev_data, bytes, dev_scratch, grid, width,
                                             (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "stream_read_w");
}

int mgenx_diag_group_rw(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                        uint8_t* dev_out, int mode, void* stream) {
  if (!ctx || !dev_data || !dev_out || bytes % 16384 != 0) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_group_rw(dev_data, bytes, dev_out, mode, ctx->cu_count,
                                        (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "group_rw");
}

#endif  // MGENX_DIAG

int mgenx_stream_scan(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                      uint64_t* dev_rec_off, uint32_t* dev_rec_len, uint64_t cap,
                      mgenx_scan_info* info, void* stream) {
  if (!ctx || (nbytes && !dev_stream) || (cap && (!dev_rec_off || !dev_rec_len)) ||
      (mode != MGENX_SCAN_TCP && mode != MGENX_SCAN_SINK))
    return MGENX_EINVAL;
  if (nbytes == 0) {
    if (info) memset(info, 0, sizeof(*info));
    return MGENX_OK;
  }
  hipSetDevice(ctx->device);
  if (!ctx->scan_ws) ctx->scan_ws = mgenx_scan_ws_new();
  return mgenx_scan_run(ctx->scan_ws, dev_stream, nbytes, mode, dev_rec_off, dev_rec_len, cap,
                        info, (hipStream_t)stream, ctx->err, sizeof(ctx->err));
}

int mgenx_stream_scan_exits(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                            uint64_t window, uint64_t limit, uint64_t* dev_entries,
                            uint64_t* dev_exits, uint32_t cap, uint32_t* candidates,
                            void* stream) {
  if (!ctx || !dev_stream || nbytes == 0 || limit > nbytes || (cap && (!dev_entries || !dev_exits)) ||
      (mode != MGENX_SCAN_TCP && mode != MGENX_SCAN_SINK))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->scan_ws) ctx->scan_ws = mgenx_scan_ws_new();
  return mgenx_scan_exits_run(ctx->scan_ws, dev_stream, nbytes, mode, window, limit, dev_entries,
                              dev_exits, cap, candidates, (hipStream_t)stream, ctx->err,
                              sizeof(ctx->err));
}

int mgenx_stream_scan_range(mgenx_ctx* ctx, const uint8_t* dev_stream, uint64_t nbytes, int mode,
                            uint64_t entry, uint64_t limit, int flags, uint64_t* dev_rec_off,
                            uint32_t* dev_rec_len, uint64_t cap, mgenx_scan_info* info,
                            void* stream) {
  if (!ctx || !dev_stream || nbytes == 0 || limit > nbytes || (cap && (!dev_rec_off || !dev_rec_len)) ||
      (mode != MGENX_SCAN_TCP && mode != MGENX_SCAN_SINK) || (flags & ~MGENX_SCAN_REUSE))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->scan_ws) ctx->scan_ws = mgenx_scan_ws_new();
  return mgenx_scan_range_run(ctx->scan_ws, dev_stream, nbytes, mode, entry, limit,
                              flags & MGENX_SCAN_REUSE, dev_rec_off, dev_rec_len, cap, info,
                              (hipStream_t)stream, ctx->err, sizeof(ctx->err));
}

int mgenx_flow_init(mgenx_ctx* ctx, mgenx_flow_state* dev_flows, uint32_t n_flows,
                    double window_sec, void* stream) {
  if (!ctx || (n_flows && !dev_flows) || !(window_sec >= 0.0)) return MGENX_EINVAL;
  return mgenx_flow_init_run(dev_flows, n_flows, window_sec, (hipStream_t)stream);
}

int mgenx_flow_reduce(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_seq,
                      const uint32_t* dev_tx_sec, const uint32_t* dev_tx_usec,
                      const uint16_t* dev_msg_len, const uint32_t* dev_rx_sec,
                      const uint32_t* dev_rx_usec, uint32_t n, mgenx_flow_state* dev_flows,
                      uint32_t n_flows, mgenx_flow_report* dev_reports, uint32_t per_flow,
                      uint32_t* dev_report_count, void* stream) {
  return mgenx_flow_reduce_ex(ctx, dev_flow_idx, dev_seq, dev_tx_sec, dev_tx_usec, dev_msg_len,
                              dev_rx_sec, dev_rx_usec, n, dev_flows, n_flows, dev_reports,
                              per_flow, dev_report_count, nullptr, stream);
}

int mgenx_flow_reduce_ex(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const uint32_t* dev_seq,
                         const uint32_t* dev_tx_sec, const uint32_t* dev_tx_usec,
                         const uint16_t* dev_msg_len, const uint32_t* dev_rx_sec,
                         const uint32_t* dev_rx_usec, uint32_t n, mgenx_flow_state* dev_flows,
                         uint32_t n_flows, mgenx_flow_report* dev_reports, uint32_t per_flow,
                         uint32_t* dev_report_count, uint32_t* dev_report_rec, void* stream) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0 || n_flows == 0) return MGENX_OK;
  if (!dev_flow_idx || !dev_seq || !dev_tx_sec || !dev_tx_usec || !dev_msg_len ||
      !dev_rx_sec || !dev_rx_usec || !dev_flows ||
      (per_flow && (!dev_reports || !dev_report_count)) || n > 0x7FFFFFFFu)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->flow_ws) ctx->flow_ws = mgenx_flow_ws_new();
  return mgenx_flow_reduce_run(ctx->flow_ws, dev_flow_idx, dev_seq, dev_tx_sec, dev_tx_usec,
                               dev_msg_len, nullptr, dev_rx_sec, dev_rx_usec, n, dev_flows,
                               n_flows, dev_reports, per_flow, dev_report_count, dev_report_rec,
                               (hipStream_t)stream,
                               ctx->err, sizeof(ctx->err));
}

int mgenx_flow_reduce_rows(mgenx_ctx* ctx, const uint32_t* dev_flow_idx, const mgenx_rec* dev_rows,
                           const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec, uint32_t n,
                           mgenx_flow_state* dev_flows, uint32_t n_flows,
                           mgenx_flow_report* dev_reports, uint32_t per_flow,
                           uint32_t* dev_report_count, uint32_t* dev_report_rec, void* stream) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0 || n_flows == 0) return MGENX_OK;
  if (!dev_flow_idx || !dev_rows || !dev_rx_sec || !dev_rx_usec || !dev_flows ||
      (per_flow && (!dev_reports || !dev_report_count)) || n > 0x7FFFFFFFu)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->flow_ws) ctx->flow_ws = mgenx_flow_ws_new();
  return mgenx_flow_reduce_run(ctx->flow_ws, dev_flow_idx, nullptr, nullptr, nullptr, nullptr,
                               dev_rows, dev_rx_sec, dev_rx_usec, n, dev_flows, n_flows,
                               dev_reports, per_flow, dev_report_count, dev_report_rec,
                               (hipStream_t)stream, ctx->err, sizeof(ctx->err));
}

static int log_recv(mgenx_ctx* ctx, bool binary, const uint8_t* dev_slab, uint64_t slab_bytes,
                    const uint64_t* dev_rec_off, const uint32_t* dev_rec_len, uint64_t stride,
                    const mgenx_cols* cols,
                    const mgenx_addr* dev_src, const uint32_t* dev_rx_sec,
                    const uint32_t* dev_rx_usec, const int32_t* dev_ttl, uint32_t n,
                    int protocol, uint32_t opts, char* dev_text, uint64_t text_cap,
                    uint64_t* dev_line_off, void* stream) {
  if (!ctx || !cols || !dev_line_off) return MGENX_EINVAL;
  if (n == 0) return hipMemsetAsync(dev_line_off, 0, 8, (hipStream_t)stream) == hipSuccess
                         ? MGENX_OK : MGENX_EDEVICE;
  const mgenx_cols& k = *cols;
  const bool core = k.rows || (k.flow_id && k.seq_num && k.tx_sec && k.tx_usec && k.msg_len &&
                               k.dst_port && k.flags && k.err && k.dst_type && k.dst_len &&
                               k.payload_len && k.payload_type && k.gps_status);
  const bool ext = k.dst_addr && k.host_addr && k.host_port && k.host_type && k.host_len &&
                   k.lat_raw && k.lon_raw && k.alt && k.payload_off && (!binary || k.hdr_len);
  if (!core || !ext || !dev_slab || !dev_src || !dev_rx_sec || !dev_rx_usec ||
      (!dev_rec_off && stride == 0 && n > 1) || (text_cap && !dev_text) || n > 0x7FFFFFFEu)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_log_recv_run(ctx->log_ws, binary, dev_slab, slab_bytes, dev_rec_off, dev_rec_len,
                            stride, cols,
                            dev_src, dev_rx_sec, dev_rx_usec, dev_ttl, n, protocol, opts,
                            dev_text, text_cap, dev_line_off, (hipStream_t)stream, ctx->err,
                            sizeof(ctx->err));
}

int mgenx_log_recv_text(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                        uint64_t stride, const mgenx_cols* cols, const mgenx_addr* dev_src,
                        const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec,
                        const int32_t* dev_ttl, uint32_t n, int protocol, uint32_t opts,
                        char* dev_text, uint64_t text_cap, uint64_t* dev_line_off,
                        void* stream) {
  return log_recv(ctx, false, dev_slab, ~0ull, dev_rec_off, nullptr, stride, cols, dev_src,
                  dev_rx_sec,
                  dev_rx_usec, dev_ttl, n, protocol, opts, dev_text, text_cap, dev_line_off,
                  stream);
}

int mgenx_log_recv_binary(mgenx_ctx* ctx, const uint8_t* dev_slab, uint64_t slab_bytes,
                          const uint64_t* dev_rec_off, uint64_t stride,
                          const uint32_t* dev_rec_len, const mgenx_cols* cols,
                          const mgenx_addr* dev_src, const uint32_t* dev_rx_sec,
                          const uint32_t* dev_rx_usec, uint32_t n, int protocol,
                          uint8_t* dev_out, uint64_t out_cap, uint64_t* dev_rec_pos,
                          void* stream) {
  return log_recv(ctx, true, dev_slab, slab_bytes, dev_rec_off, dev_rec_len, stride, cols, dev_src,
                  dev_rx_sec, dev_rx_usec, nullptr, n, protocol, 0, (char*)dev_out, out_cap,
                  dev_rec_pos, stream);
}

static int log_send(mgenx_ctx* ctx, bool binary, const mgenx_flow_tmpl* dev_tmpl,
                    const mgenx_pack_desc* dev_desc, const uint16_t* dev_src_port,
                    const uint32_t* dev_out_len, const uint32_t* dev_msg_total,
                    const uint8_t* dev_slab, uint64_t slab_bytes, const uint64_t* dev_rec_off,
                    uint64_t stride, uint32_t n, int protocol, uint32_t opts, uint8_t* dev_out,
                    uint64_t out_cap, uint64_t* dev_pos, void* stream) {
  if (!ctx || !dev_pos) return MGENX_EINVAL;
  if (n == 0) return hipMemsetAsync(dev_pos, 0, 8, (hipStream_t)stream) == hipSuccess
                         ? MGENX_OK : MGENX_EDEVICE;
  if (!dev_tmpl || !dev_desc || (!binary && !dev_src_port) || (out_cap && !dev_out) ||
      (binary && (!dev_slab || (!dev_rec_off && stride == 0 && n > 1))) || n > 0x7FFFFFFEu)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_log_send_exec(ctx->log_ws, dev_tmpl, dev_desc, dev_src_port, dev_out_len,
                             dev_msg_total, dev_slab, slab_bytes, dev_rec_off, stride, n,
                             protocol, opts, binary, dev_out, out_cap, dev_pos,
                             (hipStream_t)stream, ctx->err, sizeof(ctx->err));
}

int mgenx_log_send_text(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                        const mgenx_pack_desc* dev_desc, const uint16_t* dev_src_port,
                        const uint32_t* dev_out_len, const uint32_t* dev_msg_total, uint32_t n,
                        int protocol, uint32_t opts, char* dev_text, uint64_t text_cap,
                        uint64_t* dev_line_off, void* stream) {
  return log_send(ctx, false, dev_tmpl, dev_desc, dev_src_port, dev_out_len, dev_msg_total,
                  nullptr, 0, nullptr, 0, n, protocol, opts, (uint8_t*)dev_text, text_cap,
                  dev_line_off, stream);
}

int mgenx_log_send_binary(mgenx_ctx* ctx, const mgenx_flow_tmpl* dev_tmpl,
                          const mgenx_pack_desc* dev_desc, const uint32_t* dev_out_len,
                          const uint32_t* dev_msg_total, const uint8_t* dev_slab,
                          uint64_t slab_bytes, const uint64_t* dev_rec_off, uint64_t stride,
                          uint32_t n, int protocol, uint8_t* dev_out, uint64_t out_cap,
                          uint64_t* dev_rec_pos, void* stream) {
  return log_send(ctx, true, dev_tmpl, dev_desc, nullptr, dev_out_len, dev_msg_total, dev_slab,
                  slab_bytes, dev_rec_off, stride, n, protocol, 0, dev_out, out_cap, dev_rec_pos,
                  stream);
}

int mgenx_report_build(mgenx_ctx* ctx, const mgenx_flow_report* dev_reports, uint32_t n_flows,
                       uint32_t per_flow, const uint32_t* dev_report_count,
                       const mgenx_report_key* dev_keys, uint8_t* dev_sign,
                       const double* dev_offset, uint8_t* dev_items, uint8_t* dev_item_len,
                       void* stream) {
  if (!ctx || (n_flows && per_flow && (!dev_reports || !dev_report_count || !dev_keys ||
                                       !dev_sign || !dev_items || !dev_item_len)))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  return mgenx_report_build_run(dev_reports, n_flows, per_flow, dev_report_count, dev_keys,
                                dev_sign, dev_offset, ctx->d_rq, dev_items, dev_item_len,
                                (hipStream_t)stream);
}

int mgenx_log_report_text(mgenx_ctx* ctx, const uint8_t* dev_items,
                          const mgenx_flow_report* dev_reports, uint32_t n_flows,
                          uint32_t per_flow, const uint32_t* dev_report_count, uint32_t opts,
                          char* dev_text, uint64_t text_cap, uint64_t* dev_line_off,
                          void* stream) {
  const uint64_t n = (uint64_t)n_flows * per_flow;
  if (!ctx || n > 0xFFFFFFFFull || !dev_line_off ||
      (n && (!dev_items || !dev_reports || !dev_report_count)) || (text_cap && !dev_text))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_report_lines(ctx->log_ws, dev_items, dev_reports, dev_report_count, per_flow,
                            nullptr, nullptr, nullptr, nullptr, nullptr, (uint32_t)n, opts,
                            ctx->d_rq, dev_text, text_cap, dev_line_off, (hipStream_t)stream,
                            ctx->err, sizeof(ctx->err));
}

int mgenx_data_walk(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_rec_off,
                    uint64_t stride, const mgenx_cols* cols, uint32_t n, uint32_t opts,
                    uint8_t* dev_status, uint8_t* dev_needs_host, uint32_t* dev_cmds,
                    uint32_t cmd_cap, uint64_t* dev_reps, uint32_t rep_cap,
                    uint32_t* dev_totals, void* stream) {
  if (!ctx || !cols || (opts & ~(uint32_t)MGENX_DATA_CONTROLLER)) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_slab || (!dev_rec_off && stride == 0 && n > 1) || !cols->err || !cols->payload_type ||
      !cols->payload_len || !cols->payload_off || !dev_status || !dev_needs_host ||
      (cmd_cap && !dev_cmds) || (rep_cap && !dev_reps))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_data_walk_exec(ctx->log_ws, dev_slab, dev_rec_off, stride, cols, n, opts,
                              ctx->d_rq, dev_status, dev_needs_host, dev_cmds, cmd_cap, dev_reps,
                              rep_cap, dev_totals, (hipStream_t)stream, ctx->err,
                              sizeof(ctx->err));
}

int mgenx_log_report_recv_text(mgenx_ctx* ctx, const uint8_t* dev_slab, const uint64_t* dev_reps,
                               uint32_t n_reps, const mgenx_addr* dev_src,
                               const uint32_t* dev_rx_sec, const uint32_t* dev_rx_usec,
                               uint32_t opts, char* dev_text, uint64_t text_cap,
                               uint64_t* dev_line_off, void* stream) {
  if (!ctx || !dev_line_off || (n_reps && (!dev_slab || !dev_reps || !dev_src || !dev_rx_sec ||
                                          !dev_rx_usec)) || (text_cap && !dev_text))
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_report_lines(ctx->log_ws, nullptr, nullptr, nullptr, 1, dev_reps, dev_slab,
                            dev_src, dev_rx_sec, dev_rx_usec, n_reps, opts, ctx->d_rq, dev_text,
                            text_cap, dev_line_off, (hipStream_t)stream, ctx->err,
                            sizeof(ctx->err));
}

int mgenx_flow_export(mgenx_ctx* ctx, const mgenx_flow_state* dev_flows, uint32_t n_flows,
                      mgenx_flow_counters* dev_out, void* stream) {
  if (!ctx || (n_flows && (!dev_flows || !dev_out))) return MGENX_EINVAL;
  return mgenx_flow_export_run(dev_flows, n_flows, dev_out, (hipStream_t)stream);
}

// ---- the resident single-message worker (mgenx_worker.hip) ----
struct mgenx_worker {
  mgenx_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  mgenx::WReq* req = nullptr;       // the host's view of the request block (write only)
  mgenx::WReq* req_dev = nullptr;   // the device's view of it
  bool req_in_device = false;       // fine-grained device memory (else pinned host memory)
  mgenx::WRep* rep = nullptr;       // pinned host memory (mapped, coherent)
  mgenx::WRep* rep_dev = nullptr;
  uint32_t seq = 0;                  // the last request number issued
  uint64_t idle_ticks = 0;           // s_memrealtime ticks (100 MHz)
  bool launched = false;
  std::mutex mu;                     // a call and a stop from another thread do not interleave
};

// every live worker of the process (mgenx::quiesce_workers)
static std::mutex g_workers_mu;
static std::vector<mgenx_worker*> g_workers;

static uint32_t w_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
static void w_store(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
// a reply chunk (16 bytes, one load: the worker wrote it with one store) and whether it carries tag r
struct WChunk {
  uint32_t w[4];
};
static bool w_chunk(const uint32_t* p, uint32_t r, WChunk& c) {
  const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(p));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(c.w), v);
  std::atomic_thread_fence(std::memory_order_acquire);
  return c.w[3] == r;
}

// The request block in fine-grained device memory that the CPU agent may store into (through
// the BAR): the request then reaches the wave as posted writes and the wave polls local memory,
// instead of reading pinned host memory across PCIe on every poll and again for the message
// (scripts/diag/bar_probe.hip).  Null when the runtime does not grant the CPU access.
static hsa_status_t find_cpu_agent(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
static void* device_mailbox(size_t bytes) {
  if (const char* e = getenv("MGENX_WORKER_HOST_MAILBOX"))
    if (atoi(e) != 0) return nullptr;
  static hsa_agent_t cpu = {0};
  static std::once_flag once;
  std::call_once(once, [] { (void)hsa_iterate_agents(find_cpu_agent, &cpu); });
  if (!cpu.handle) return nullptr;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) != hipSuccess) return nullptr;
  if (hsa_amd_agents_allow_access(1, &cpu, nullptr, p) != HSA_STATUS_SUCCESS) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}
// host stores into the request block: a device-memory block is written through a
// write-combining mapping, so the pieces are fenced (sfence) before the doorbell and after it
static void w_fence() { _mm_sfence(); }
static void w_copy(uint8_t* dst, const uint8_t* src, size_t n) { memcpy(dst, src, n); }

// a worker wave serving requests after `start`: the previous one (if any) has ended -- it
// clears `alive` as its last act -- so reap it and launch the next
static int worker_launch(mgenx_worker* w, uint32_t start) {
  if (w->launched && hipStreamSynchronize(w->stream) != hipSuccess) return MGENX_EDEVICE;
  w_store(&w->rep->alive, 1u);
  hipError_t e = mgenx::launch_worker(w->req_dev, w->rep_dev, w->ctx->d_tabs,
                                      w->ctx->d_bytetab, w->ctx->d_rtab, start, w->idle_ticks,
                                      w->stream);
  if (e != hipSuccess) return set_err(w->ctx, e, "worker launch");
  w->launched = true;
  return MGENX_OK;
}

// the request's polled pieces: `pd` (up to kPollData bytes, zero-filled) in pieces 1-15, then
// piece 0, each with one 16-byte store
static void w_post(mgenx::WReq* m, uint32_t r, uint32_t op, uint32_t len, uint32_t arg,
                   const uint8_t* pd, uint32_t pn) {
  alignas(16) uint8_t piece[16];
  for (uint32_t k = 1; k < mgenx::kPollPieces; k++) {
    const uint32_t o = 12u * (k - 1u);
    const uint32_t c = pn > o ? std::min(12u, pn - o) : 0u;
    memset(piece, 0, 12);
    if (c) memcpy(piece, pd + o, c);
    memcpy(piece + 12, &r, 4);
    _mm_store_si128(reinterpret_cast<__m128i*>(m->poll + 4u * k),
                    _mm_load_si128(reinterpret_cast<const __m128i*>(piece)));
  }
  w_fence();
  std::atomic_thread_fence(std::memory_order_release);
  const uint32_t p0[4] = {r, op << mgenx::kWorkOpShift | len, arg, 0u};
  _mm_store_si128(reinterpret_cast<__m128i*>(m->poll), _mm_loadu_si128(reinterpret_cast<const __m128i*>(p0)));
  w_fence();
  std::atomic_thread_fence(std::memory_order_seq_cst);
}

// post request `op` (bytes beyond the polled ones already in req->data) and wait for the
// reply: chunks first_chunk .. 7 + extra into out (3 words each); returns the status word
static int worker_call(mgenx_worker* w, uint32_t op, uint32_t len, uint32_t arg,
                       uint32_t first_chunk, uint32_t last_chunk, uint32_t* out,
                       const uint8_t* pd = nullptr, uint32_t pn = 0, uint32_t* status = nullptr) {
  // (the caller holds w->mu: the request's data area is written before this call)
  if (!w->launched || !w_load(&w->rep->alive)) {
    hipSetDevice(w->ctx->device);
    const int rc = worker_launch(w, w->seq);
    if (rc != MGENX_OK) return rc;
  }
  uint32_t r = w->seq + 1u;
  if (r == 0u) r = 1u;  // 0 is "no request yet"
  w->seq = r;
  w_post(w->req, r, op, len, arg, pd, pn);
  // spin on the reply's chunk 7; a wave that ended on its idle timeout just as this request
  // arrived is relaunched, and serves it first
  uint64_t spins = 0, relaunches = 0;
  std::chrono::steady_clock::time_point t0;
  WChunk c;
  const uint32_t* rep = w->rep->reply;
  while (!w_chunk(rep + 28, r, c)) {
    if ((++spins & 4095u) == 0u) {
      if (!w_load(&w->rep->alive) && !w_chunk(rep + 28, r, c)) {
        if (++relaunches > 3) return MGENX_EDEVICE;
        hipSetDevice(w->ctx->device);
        const int rc = worker_launch(w, r - 1u);
        if (rc != MGENX_OK) return rc;
      }
      const auto now = std::chrono::steady_clock::now();
      if (spins == 4096u) t0 = now;
      else if (now - t0 > std::chrono::seconds(10)) {  // never answered
        snprintf(w->ctx->err, sizeof(w->ctx->err), "worker: no reply to request %u", r);
        return MGENX_EDEVICE;
      }
    }
    __builtin_ia32_pause();
  }
  // the other chunks of the reply: written by the same store instruction, so at most a few
  // spins behind chunk 7
  for (uint32_t ch = first_chunk; ch <= last_chunk; ch++) {
    WChunk d = c;
    if (ch != 7u)
      while (!w_chunk(rep + 4u * ch, r, d)) __builtin_ia32_pause();
    for (int j = 0; j < 3; j++) out[3u * (ch - first_chunk) + (uint32_t)j] = d.w[j];
  }
  const uint32_t st = c.w[mgenx::kReplyStatus - 21];
  if (status) *status = st;
  return (st & 0xFFu) == 0u ? MGENX_OK : MGENX_EDEVICE;
}

int mgenx_worker_create(mgenx_ctx* ctx, uint32_t idle_ms, mgenx_worker** out) {
  if (!ctx || !out) return MGENX_EINVAL;
  *out = nullptr;
  hipSetDevice(ctx->device);
  mgenx_worker* w = new mgenx_worker();
  w->ctx = ctx;  // (not yet in ctx->workers: a failed create is freed by mgenx_worker_destroy)
  w->idle_ticks = (uint64_t)(idle_ms ? idle_ms : 1u) * 100000ull;
  bool ok = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) == hipSuccess &&
            hipHostMalloc((void**)&w->rep, sizeof(mgenx::WRep),
                          hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer((void**)&w->rep_dev, w->rep, 0) == hipSuccess;
  if (ok) {
    w->req = w->req_dev = static_cast<mgenx::WReq*>(device_mailbox(sizeof(mgenx::WReq)));
    w->req_in_device = w->req != nullptr;
    if (!w->req_in_device)
      ok = hipHostMalloc((void**)&w->req, sizeof(mgenx::WReq),
                         hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
           hipHostGetDevicePointer((void**)&w->req_dev, w->req, 0) == hipSuccess;
  }
  if (!ok) {
    mgenx_worker_destroy(w);
    return MGENX_ENOMEM;
  }
  memset(w->rep, 0, sizeof(mgenx::WRep));
  alignas(16) const uint8_t zero[16] = {0};
  for (uint32_t k = 0; k < mgenx::kPollPieces; k++)  // (16-byte stores, also to device memory)
    _mm_store_si128(reinterpret_cast<__m128i*>(w->req->poll + 4u * k),
                    _mm_load_si128(reinterpret_cast<const __m128i*>(zero)));
  w_fence();
  ctx->workers.push_back(w);
  {
    std::lock_guard<std::mutex> g(g_workers_mu);
    g_workers.push_back(w);
  }
  *out = w;
  return MGENX_OK;
}

// end the worker's wave (if one runs) and wait for it: no wave is left polling, so a later
// device-wide synchronisation (hipFree, hipDeviceSynchronize) does not wait for its idle timeout
// (the calling thread's current device is restored: growth paths allocate right after a free)
static void worker_stop(mgenx_worker* w) {
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->launched || !w->rep || !w->ctx) return;
  int prev = -1;
  const bool have_prev = hipGetDevice(&prev) == hipSuccess;
  hipSetDevice(w->ctx->device);
  if (w_load(&w->rep->alive)) {  // ask the wave to end; it may end on its own meanwhile
    uint32_t r = w->seq + 1u;
    if (r == 0u) r = 1u;
    w->seq = r;
    w_post(w->req, r, mgenx::kWorkStop, 0u, 0u, nullptr, 0u);
  }
  (void)hipStreamSynchronize(w->stream);
  w->launched = false;
  if (have_prev) hipSetDevice(prev);
}

// the wave stopped and the device resources freed; the handle stays (ctx = null)
static void worker_detach(mgenx_worker* w) {
  {
    std::lock_guard<std::mutex> g(g_workers_mu);
    g_workers.erase(std::remove(g_workers.begin(), g_workers.end(), w), g_workers.end());
  }
  worker_stop(w);
  // (the other workers' waves are ended first: the frees synchronise the device)
  if (w->req_in_device) mgenx::dev_free(w->req);
  else mgenx::host_free(w->req);
  mgenx::host_free(w->rep);
  if (w->stream) (void)hipStreamDestroy(w->stream);
  w->req = w->req_dev = nullptr;
  w->rep = w->rep_dev = nullptr;
  w->stream = nullptr;
  w->ctx = nullptr;
}

extern "C++" {
namespace mgenx {
// g_workers_mu is held for the whole loop, so no worker is destroyed while it is stopped (a
// worker call holding w->mu never takes g_workers_mu; worker_detach releases it before its stop)
void quiesce_workers(int device) {
  std::lock_guard<std::mutex> g(g_workers_mu);
  for (mgenx_worker* w : g_workers)
    if (device < 0 || (w->ctx && w->ctx->device == device)) worker_stop(w);
}
}  // namespace mgenx
}  // extern "C++"

int mgenx_worker_stop(mgenx_worker* w) {
  if (!w) return MGENX_EINVAL;
  worker_stop(w);
  return MGENX_OK;
}

int mgenx_worker_destroy(mgenx_worker* w) {
  if (!w) return MGENX_EINVAL;
  if (w->ctx) {
    std::vector<mgenx_worker*>& v = w->ctx->workers;
    v.erase(std::remove(v.begin(), v.end(), w), v.end());
    worker_detach(w);
  }
  delete w;
  return MGENX_OK;
}

int mgenx_worker_info(const mgenx_worker* w, uint32_t* flags) {
  if (!w || !flags) return MGENX_EINVAL;
  *flags = w->req_in_device ? MGENX_WORKER_DEVICE_MAILBOX : 0u;
  return MGENX_OK;
}

#if MGENX_DIAG
int mgenx_diag_worker_stamps(const mgenx_worker* w, uint32_t* out) {
  if (!w || !w->rep || !out) return MGENX_EINVAL;
  for (int k = 0; k < 8; k++) out[k] = w->rep->reply[32 + k];
  return MGENX_OK;
}
#endif

static void copy_unpacked(const uint32_t* words, mgenx_unpacked* out) { memcpy(out, words, sizeof(*out)); }

int mgenx_worker_unpack(mgenx_worker* w, const uint8_t* msg, uint32_t len, mgenx_unpacked* out) {
  if (!w) return MGENX_EINVAL;
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->ctx || !out || (len && !msg) || len > MGENX_WORKER_MAX_BYTES) return MGENX_EINVAL;
  const uint32_t n = len < mgenx::kWorkerHdrBytes ? len : mgenx::kWorkerHdrBytes;
  // Unpack reads the header bytes only: the first kPollData travel in the polled pieces, the
  // data area is for headers longer than that
  if (n > mgenx::kPollData) w_copy(w->req->data, msg, n);
  uint32_t words[24];
  const int rc = worker_call(w, mgenx::kWorkUnpack, len, 0u, 0u, 7u, words, msg,
                            n < mgenx::kPollData ? n : mgenx::kPollData);
  if (rc == MGENX_OK) copy_unpacked(words, out);
  return rc;
}

int mgenx_worker_recv(mgenx_worker* w, const uint8_t* msg, uint32_t len, uint32_t force,
                      mgenx_unpacked* out, uint32_t* crc_state, uint32_t* crc_done) {
  if (!w) return MGENX_EINVAL;
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->ctx || !out || !crc_state || !crc_done || (len && !msg) || len > MGENX_WORKER_MAX_BYTES)
    return MGENX_EINVAL;
  // the whole message in the data area (the checksum reads it), its first bytes also polled
  if (len) w_copy(w->req->data, msg, len);
  uint32_t words[24], st = 0;
  const int rc = worker_call(w, mgenx::kWorkRecv, len, force ? 1u : 0u, 0u, 7u, words, msg,
                            len < mgenx::kPollData ? len : mgenx::kPollData, &st);
  if (rc != MGENX_OK) return rc;
  copy_unpacked(words, out);
  *crc_done = (st & mgenx::kStatusCrc) ? 1u : 0u;
  *crc_state = *crc_done ? words[mgenx::kReplyCrc] : 0u;
  return MGENX_OK;
}

int mgenx_worker_pack(mgenx_worker* w, const mgenx_flow_tmpl* tmpl, const uint8_t* payload,
                      const mgenx_pack_desc* desc, uint32_t buf_len, uint32_t crc_in,
                      uint32_t opts, uint32_t fill_time, uint8_t* out, uint32_t* ret,
                      uint32_t* tx_crc, uint32_t* state) {
  if (!w) return MGENX_EINVAL;
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->ctx || !tmpl || !desc || !ret || !tx_crc || !state || buf_len > MGENX_WORKER_PACK_MAX ||
      (buf_len && !out) || (tmpl->has_payload && tmpl->payload_len && !payload))
    return MGENX_EINVAL;
  if (opts & MGENX_PACK_RANDOM_FILL) {  // the rand() stream of this fill time (cached)
    const int rc = mgenx_set_fill_time(w->ctx, fill_time);
    if (rc != MGENX_OK) return rc;
  }
  mgenx::WPackReq q;
  q.tmpl = *tmpl;
  q.tmpl.payload_off = 0;  // the payload travels in the mailbox
  q.desc = *desc;
  q.buf_len = buf_len;
  q.crc_in = crc_in;
  q.opts = opts & (MGENX_PACK_CHECKSUM | MGENX_PACK_RANDOM_FILL);
  q.rsv = 0;
  if (tmpl->has_payload && tmpl->payload_len) w_copy(w->req->data, payload, tmpl->payload_len);
  uint32_t words[6];  // reply words 18-23
  const int rc = worker_call(w, mgenx::kWorkPack, buf_len, 0u, 6u, 7u, words,
                            reinterpret_cast<const uint8_t*>(&q), (uint32_t)sizeof(q));
  if (rc != MGENX_OK) return rc;
  *ret = words[mgenx::kReplyRet - 18];
  *tx_crc = words[mgenx::kReplyTx - 18];
  *state = words[mgenx::kReplyState - 18];
  if (*ret) memcpy(out, w->rep->out, *ret);
  return MGENX_OK;
}

int mgenx_worker_crc32(mgenx_worker* w, const uint8_t* data, uint32_t len, uint32_t state_in,
                       uint32_t* state_out) {
  if (!w) return MGENX_EINVAL;
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->ctx || !state_out || (len && !data) || len > MGENX_WORKER_MAX_BYTES) return MGENX_EINVAL;
  if (len) w_copy(w->req->data, data, len);
  uint32_t words[3];  // reply words 21-23
  const int rc = worker_call(w, mgenx::kWorkCrc32, len, state_in, 7u, 7u, words);
  if (rc == MGENX_OK) *state_out = words[mgenx::kReplyCrc - 21];
  return rc;
}

int mgenx_worker_flow_update(mgenx_worker* w, mgenx_flow_state* dev_flows, uint32_t slot,
                             uint32_t seq, uint32_t rx_sec, uint32_t rx_usec, uint32_t msg_size,
                             uint32_t tx_sec, uint32_t tx_usec, uint32_t* updated,
                             mgenx_flow_report* report) {
  if (!w) return MGENX_EINVAL;
  std::lock_guard<std::mutex> g(w->mu);
  if (!w->ctx || !dev_flows || !updated || !report) return MGENX_EINVAL;
  mgenx::WUpdReq q;
  q.flows = (uint64_t)(uintptr_t)dev_flows;
  q.slot = slot;
  q.seq = seq;
  q.rx_sec = rx_sec;
  q.rx_usec = rx_usec;
  q.tx_sec = tx_sec;
  q.tx_usec = tx_usec;
  q.msg = msg_size;
  q.rsv = 0;
  uint32_t words[27], st = 0;  // reply words 21-47
  const int rc = worker_call(w, mgenx::kWorkUpdate, 0u, 0u, 7u, 15u, words,
                            reinterpret_cast<const uint8_t*>(&q), (uint32_t)sizeof(q), &st);
  if (rc != MGENX_OK) return rc;
  *updated = (st & mgenx::kStatusClosed) ? 1u : 0u;
  if (*updated) memcpy(report, words + (mgenx::kReplyReport - 21), sizeof(*report));
  return MGENX_OK;
}

int mgenx_crc32_batch(mgenx_ctx* ctx, const uint8_t* dev_data, const uint64_t* dev_off,
                      const uint32_t* dev_len, uint32_t n, uint32_t* dev_out, void* stream) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_data || !dev_off || !dev_len || !dev_out) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_crc32(dev_data, dev_off, dev_len, n, ctx->d_bytetab,
                                     ctx->d_tabs + 1024, ctx->d_xpow, nullptr,
                                     dev_out, (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "crc32");
}

int mgenx_crc32_update(mgenx_ctx* ctx, const uint8_t* dev_data, const uint64_t* dev_off,
                       const uint32_t* dev_len, uint32_t n, const uint32_t* dev_state_in,
                       uint32_t* dev_state_out, void* stream) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_data || !dev_off || !dev_len || !dev_state_in || !dev_state_out) return MGENX_EINVAL;
  hipError_t e = mgenx::launch_crc32(dev_data, dev_off, dev_len, n, ctx->d_bytetab,
                                     ctx->d_tabs + 1024, ctx->d_xpow, dev_state_in,
                                     dev_state_out, (hipStream_t)stream);
  return e == hipSuccess ? MGENX_OK : set_err(ctx, e, "crc32_update");
}

int mgenx_text_interleave(mgenx_ctx* ctx, const mgenx_text_src* srcs, uint32_t n_src,
                          uint32_t n_rec, char* dev_out, uint64_t out_cap, uint64_t* dev_rec_off,
                          void* stream) {
  if (!ctx || !dev_rec_off || n_src > MGENX_TEXT_MAX_SRC || (n_src && !srcs) ||
      (out_cap && !dev_out) || n_rec > 0x7FFFFFFEu)
    return MGENX_EINVAL;
  for (uint32_t s = 0; s < n_src; s++) {
    const mgenx_text_src& t = srcs[s];
    if (t.kind > MGENX_TEXT_SCATTER || !t.line_off ||
        (t.kind != MGENX_TEXT_PER_RECORD && !t.index) ||
        (t.kind == MGENX_TEXT_OWNER && t.index_stride == 0))
      return MGENX_EINVAL;
  }
  hipSetDevice(ctx->device);
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  return mgenx_text_interleave_run(ctx->log_ws, srcs, n_src, n_rec, dev_out, out_cap,
                                   dev_rec_off, (hipStream_t)stream, ctx->err, sizeof(ctx->err));
}

int mgenx_pcap_parse(mgenx_ctx* ctx, const uint8_t* dev_buf, uint64_t buf_bytes,
                     const uint64_t* dev_pkt_off, uint32_t n, uint32_t link_type,
                     uint32_t flags, uint64_t* dev_udp_off, uint32_t* dev_udp_len,
                     mgenx_addr* dev_src, int32_t* dev_ttl, uint32_t* dev_rx_sec,
                     uint32_t* dev_rx_usec, uint8_t* dev_status, void* stream) {
  if (!ctx) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_buf || !dev_pkt_off || !dev_udp_off || !dev_udp_len || !dev_src || !dev_ttl ||
      !dev_rx_sec || !dev_rx_usec || !dev_status)
    return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  return mgenx_pcap_parse_run(dev_buf, buf_bytes, dev_pkt_off, n, link_type, flags, dev_udp_off,
                              dev_udp_len, dev_src, dev_ttl, dev_rx_sec, dev_rx_usec, dev_status,
                              (hipStream_t)stream);
}

int mgenx_pcap_snap(mgenx_ctx* ctx, uint8_t* dev_buf, uint64_t file_bytes, uint64_t buf_bytes,
                    const uint64_t* dev_pkt_off, uint32_t n, uint32_t flags, uint8_t* dev_status,
                    uint64_t* dev_udp_off, uint32_t* dev_udp_len, void* stream) {
  if (!ctx || buf_bytes < file_bytes || n > 0x7FFFFFFEu) return MGENX_EINVAL;
  if (n == 0) return MGENX_OK;
  if (!dev_buf || !dev_pkt_off || !dev_status || !dev_udp_off || !dev_udp_len) return MGENX_EINVAL;
  hipSetDevice(ctx->device);
  const size_t need_b = (((size_t)n + 1) * 8 + 255) & ~(size_t)255;
  const size_t scan_b = mgenx_pcap_snap_scan_bytes(n);
  char* m = static_cast<char*>(ctx->snap.get(need_b + scan_b));
  if (!m) return set_err(ctx, hipErrorOutOfMemory, "pcap_snap workspace");
  const int rc = mgenx_pcap_snap_run(dev_buf, file_bytes, buf_bytes, dev_pkt_off, n, flags,
                                     dev_status, dev_udp_off, dev_udp_len, (uint64_t*)m,
                                     m + need_b, scan_b, (hipStream_t)stream);
  return rc == MGENX_OK ? MGENX_OK : set_err(ctx, hipGetLastError(), "pcap_snap");
}

// ---- ConvertBinaryLog (mgenMsg.cpp:1417-1900) ----
int mgenx_binlog_index(const uint8_t* buf, uint64_t nbytes, uint64_t* rec_off, uint64_t cap,
                       mgenx_binlog_info* info) {
  if (!buf || !info || (cap && !rec_off)) return MGENX_EINVAL;
  memset(info, 0, sizeof(*info));
  info->status = MGENX_BINLOG_HEADER;
  // "mgen ... version=<4|5> ... type=binary_log\n" and its NUL (:1437-1518)
  if (nbytes < 4 || memcmp(buf, "mgen", 4) != 0) return MGENX_OK;
  char hdr[1024];
  uint64_t k = 3;
  memcpy(hdr, buf, 4);
  while (hdr[k] != '\0') {
    if (++k >= sizeof(hdr) || k >= nbytes) return MGENX_OK;
    hdr[k] = (char)buf[k];
  }
  const char* v = strstr(hdr, "version=");
  int version = 0;
  if (!v || 1 != sscanf(v, "version=%d", &version) || (version != 4 && version != 5))
    return MGENX_OK;
  const char* t = strstr(v, "type=");
  char ftype[128];
  if (!t || 1 != sscanf(t, "type=%127s", ftype) || strcmp(ftype, "binary_log")) return MGENX_OK;
  info->version = (uint32_t)version;
  info->status = MGENX_BINLOG_OK;
  uint64_t off = k + 1, n = 0;
  // the record walk (:1521-1555) with the reference's stops: a record over 1024 bytes, a short
  // record, an event type it does not convert (RERR, unknown), an unknown address type
  while (off + 4 <= nbytes) {
    const uint8_t* h = buf + off;
    const uint32_t ev = h[0], rl = (uint32_t)h[2] << 8 | h[3];
    if (rl > 1024) { info->status = MGENX_BINLOG_TOO_LONG; break; }
    if (off + 4 + rl > nbytes) { info->status = MGENX_BINLOG_SHORT; break; }
    const bool addr_ev = ev == 1 || ev == 6 || ev == 7 || (ev >= 10 && ev <= 16);
    if (ev == 0 || ev == 2 || ev > 16) { info->status = MGENX_BINLOG_EVENT; break; }
    // a record too short for the fields its type reads (mgen never writes one; the reference
    // would parse stale bytes of its read buffer): stop as at a short read, so the device
    // formatters never read past a record -- the event time (8 bytes), RECV 12 + source
    // length, LISTEN / IGNORE 12, JOIN / LEAVE 13 + group length + interface name length,
    // ON ... RECONNECT 18 + address length
    const uint8_t* b = h + 4;
    bool shortrec = rl < 8;
    if (!shortrec) {
      if (ev == 1) shortrec = rl < 12 || rl < 12u + b[11];
      else if (ev == 4 || ev == 5) shortrec = rl < 12;
      else if (ev == 6 || ev == 7)
        shortrec = rl < 13 || rl < 13u + b[11] || rl < 13u + b[11] + b[12 + b[11]];
      else if (ev >= 10 && ev <= 16) shortrec = rl < 12 || rl < 18u + b[11];
    }
    if (shortrec) { info->status = MGENX_BINLOG_SHORT; break; }
    if (addr_ev && h[14] != 1 && h[14] != 2) { info->status = MGENX_BINLOG_EVENT; break; }
    if (n < cap) rec_off[n] = off;
    n++;
    off += 4 + rl;
  }
  info->n_records = n;
  info->consumed = off;
  return MGENX_OK;
}

int mgenx_convert_binary_log(mgenx_ctx* ctx, const uint8_t* dev_buf, uint64_t buf_bytes,
                             const uint64_t* dev_rec_off, uint32_t n, uint32_t flags,
                             uint32_t opts, char* dev_text, uint64_t text_cap,
                             uint64_t* dev_rec_pos, void* stream) {
  if (!ctx || !dev_rec_pos || (text_cap && !dev_text) || n > 0x7FFFFFFEu) return MGENX_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipSetDevice(ctx->device);
  if (n == 0) return hipMemsetAsync(dev_rec_pos, 0, 8, s) == hipSuccess ? MGENX_OK : MGENX_EDEVICE;
  if (!dev_buf || !dev_rec_off) return MGENX_EINVAL;
  if (!ctx->log_ws) ctx->log_ws = mgenx_log_ws_new();
  // per-record arrays and unpack columns in one block (bl[0])
  const size_t a8 = ((size_t)n * 8 + 255) & ~(size_t)255, a4 = ((size_t)n * 4 + 255) & ~(size_t)255;
  const size_t a2 = ((size_t)n * 2 + 255) & ~(size_t)255, a1 = ((size_t)n + 255) & ~(size_t)255;
  const size_t a16 = ((size_t)n * 16 + 255) & ~(size_t)255, a20 = ((size_t)n * 20 + 255) & ~(size_t)255;
  const size_t need = a8 + 4 * a4 + a20 + 2 * a1 +                       // parse outputs
                      8 * a4 + 5 * a2 + 9 * a1 + 2 * a16 + a4;           // columns
  char* m = static_cast<char*>(ctx->bl[0].get(need));
  if (!m) return set_err(ctx, hipErrorOutOfMemory, "convert_binary_log workspace");
  auto take = [&](size_t b) { char* q = m; m += b; return q; };
  uint64_t* msg_off = (uint64_t*)take(a8);
  uint32_t* msg_len = (uint32_t*)take(a4);
  uint32_t* ev_sec = (uint32_t*)take(a4);
  uint32_t* ev_usec = (uint32_t*)take(a4);
  uint32_t* aux = (uint32_t*)take(a4);
  mgenx_addr* src = (mgenx_addr*)take(a20);
  uint8_t* kind = (uint8_t*)take(a1);
  uint8_t* proto = (uint8_t*)take(a1);
  mgenx_cols c;
  memset(&c, 0, sizeof(c));
  c.flow_id = (uint32_t*)take(a4); c.seq_num = (uint32_t*)take(a4); c.tx_sec = (uint32_t*)take(a4);
  c.tx_usec = (uint32_t*)take(a4); c.dst_addr4 = (uint32_t*)take(a4);
  c.payload_off = (uint32_t*)take(a4); c.lat_raw = (uint32_t*)take(a4);
  c.lon_raw = (uint32_t*)take(a4); c.alt = (int32_t*)take(a4);
  c.msg_len = (uint16_t*)take(a2); c.dst_port = (uint16_t*)take(a2);
  c.payload_len = (uint16_t*)take(a2); c.hdr_len = (uint16_t*)take(a2);
  c.host_port = (uint16_t*)take(a2);
  c.flags = (uint8_t*)take(a1); c.err = (uint8_t*)take(a1); c.dst_type = (uint8_t*)take(a1);
  c.dst_len = (uint8_t*)take(a1); c.payload_type = (uint8_t*)take(a1);
  c.gps_status = (uint8_t*)take(a1); c.host_type = (uint8_t*)take(a1);
  c.host_len = (uint8_t*)take(a1);
  c.decoded = (uint8_t*)take(a1);
  c.host_addr = (uint8_t*)take(a16); c.dst_addr = (uint8_t*)take(a16);
  int rc = mgenx_binlog_parse_exec(dev_buf, dev_rec_off, n, msg_off, msg_len, src, ev_sec, ev_usec,
                                   aux, kind, proto, s);
  if (rc != MGENX_OK) return set_err(ctx, hipGetLastError(), "binlog parse");
  rc = mgenx_unpack_batch(ctx, dev_buf, buf_bytes, msg_off, 0, msg_len, 0, n, &c,
                          MGENX_OPT_SKIP_CRC, stream);
  if (rc != MGENX_OK) return rc;
  const uint32_t log_rx = (flags & MGENX_BINLOG_NO_RX) ? 0u : 1u;
  const uint32_t flush = (flags & MGENX_BINLOG_FLUSH) ? 1u : 0u;
  // one line per record: size pass, then the text (bl[1] = line offsets + text)
  const size_t off_bytes = ((size_t)n + 1) * 8;
  uint64_t* line_off = (uint64_t*)ctx->bl[1].get(off_bytes + 256);
  if (!line_off) return set_err(ctx, hipErrorOutOfMemory, "convert_binary_log lines");
  rc = mgenx_binlog_lines_exec(ctx->log_ws, dev_buf, dev_rec_off, n, msg_off, msg_len, src, ev_sec,
                               ev_usec, aux, kind, proto, &c, log_rx, flush, opts, nullptr, 0,
                               line_off, s, ctx->err, sizeof(ctx->err));
  if (rc != MGENX_OK) return rc;
  uint64_t total = 0;
  if (hipMemcpyAsync(&total, line_off + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return set_err(ctx, hipGetLastError(), "convert_binary_log sync");
  char* text = (char*)ctx->bl[2].get(total + 64);
  if (!text) return set_err(ctx, hipErrorOutOfMemory, "convert_binary_log text");
  rc = mgenx_binlog_lines_exec(ctx->log_ws, dev_buf, dev_rec_off, n, msg_off, msg_len, src, ev_sec,
                               ev_usec, aux, kind, proto, &c, log_rx, flush, opts, text, total,
                               line_off, s, ctx->err, sizeof(ctx->err));
  if (rc != MGENX_OK) return rc;
  mgenx_text_src srcs[2];
  memset(srcs, 0, sizeof(srcs));
  srcs[0].text = text; srcs[0].line_off = line_off; srcs[0].n_lines = n;
  srcs[0].kind = MGENX_TEXT_PER_RECORD;
  uint32_t n_src = 1;
  // REPORT items of MGEN_DATA payloads (LogRecvEvent, mgenMsg.cpp:1104-1137)
  uint32_t cap = 256, n_reps = 0;
  uint32_t* totals = nullptr;
  uint64_t* pairs = nullptr;
  for (int pass = 0; pass < 2; pass++) {
    char* w = (char*)ctx->bl[3].get(256 + (size_t)cap * 16 + 2 * a1);
    if (!w) return set_err(ctx, hipErrorOutOfMemory, "convert_binary_log walk");
    totals = (uint32_t*)w;
    pairs = (uint64_t*)(w + 256);
    uint8_t* wst = (uint8_t*)(w + 256 + (size_t)cap * 16);
    rc = mgenx_data_walk(ctx, dev_buf, msg_off, 0, &c, n, MGENX_DATA_CONTROLLER, wst, wst + a1,
                         totals + 8, 0, pairs, cap, totals, stream);
    if (rc != MGENX_OK) return rc;
    uint32_t tt[2] = {0, 0};
    if (hipMemcpyAsync(tt, totals, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return set_err(ctx, hipGetLastError(), "convert_binary_log sync");
    n_reps = tt[1];
    if (n_reps <= cap) break;
    cap = n_reps;
  }
  if (n_reps) {
    uint64_t* rline = (uint64_t*)ctx->bl[4].get(((size_t)n_reps + 1) * 8 + (size_t)n_reps * 320);
    if (!rline) return set_err(ctx, hipErrorOutOfMemory, "convert_binary_log reports");
    char* rtext = (char*)(rline + n_reps + 1);
    rc = mgenx_log_report_recv_text(ctx, dev_buf, pairs, n_reps, src, ev_sec, ev_usec, opts, rtext,
                                    (uint64_t)n_reps * 320, rline, stream);
    if (rc != MGENX_OK) return rc;
    srcs[1].text = rtext; srcs[1].line_off = rline; srcs[1].n_lines = n_reps;
    srcs[1].kind = MGENX_TEXT_OWNER; srcs[1].index = (const uint32_t*)pairs;
    srcs[1].index_stride = 4;
    n_src = 2;
  }
  return mgenx_text_interleave(ctx, srcs, n_src, n, dev_text, text_cap, dev_rec_pos, stream);
}

}  // extern "C"
