// mgenx_kernels.hpp -- kernel parameter blocks and launchers shared with mgenx_api.hip.
#pragma once

#include "mgenx_common.hpp"

#include <mutex>
#include <set>
#include <utility>

#ifndef MGENX_DIAG
#define MGENX_DIAG 0
#endif

namespace mgenx {

// Ends the resident worker waves (mgenx_worker_*, mgenx_api.hip) of `device` (every device when
// device < 0) and waits for them; the calling thread's current device is left as it was.
// hipFree / hipHostFree synchronise the device, so with a wave still polling its mailbox they
// would wait for its idle timeout: every workspace growth frees through these.
void quiesce_workers(int device);
inline void dev_free(void* p) {
  if (!p) return;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  quiesce_workers(dev);  // hipFree synchronises the current device only
  (void)hipFree(p);
}
inline void host_free(void* p) {
  if (!p) return;
  quiesce_workers(-1);  // pinned host memory may be mapped on every device
  (void)hipHostFree(p);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute is
// per device, and threaded multi-GPU callers (mgenx::ShardedScan) launch concurrently, so the
// "done" record is per device and guarded (every entry point sets its context's device first)
inline hipError_t set_max_lds(const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.count({fn, dev})) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

struct UnpackParams {
  const uint8_t* slab;
  uint64_t slab_bytes;
  const uint64_t* rec_off;
  uint64_t stride;
  const uint32_t* rec_len;
  uint32_t fixed_len;
  uint32_t n;
  uint32_t opts;
  const uint32_t* tabs;    // [A64 | A4 | A8 | A12 | A16 | A32 | A48], 4 x 256 each
  const uint32_t* expect;  // [65536]
  uint32_t expect_fixed;   // expect[fixed_len] (host copy, fixed-length kernel)
  uint8_t* sink;           // 1 KiB scratch: stores of lanes past the batch end
  int variant;             // diagnostic ablation (0 = product path)
  mgenx_cols cols;
};

struct PackParams {
  const mgenx_flow_tmpl* tmpl;
  const uint32_t* tmpl_crc;
  const mgenx_pack_desc* desc;
  uint32_t n;
  const uint8_t* pool;
  uint8_t* slab;
  uint64_t slab_bytes;
  const uint64_t* rec_off;
  uint64_t stride;
  uint32_t* out_len;
  uint32_t opts;
  const uint32_t* byte_tab;  // [256] reference CRC table
  const uint32_t* a4_tab;    // [4][256] A_4 (x -> x * x^32 mod P): four bytes per step
  const uint32_t* xpow;      // [65536] x^(8n) mod P
  const uint32_t* ia;        // [65536] A_n(0xFFFFFFFF)
  const uint8_t* rtab;       // 16 zero bytes + glibc rand() byte stream (random fill)
  const uint32_t* rcrc;      // [65536] crc_raw of the first k rand bytes
  const uint32_t* buf_len;   // MGENX_PACK_RAW: Pack's bufferLen per record (NULL = msg_len)
  const uint32_t* crc_in;    // MGENX_PACK_RAW: tx_checksum argument on entry (NULL = 0)
  uint32_t* tx_crc;          // optional: tx_checksum after Pack
  uint32_t* state;           // optional: packet_header_len | flags << 16 after Pack
  const uint32_t* frag_len;  // MGENX_PACK_RAW, TCP: fragment length F; when F > bufferLen the
                             // later buffers' copies of the image are stored too (NULL = none)
  int frag_ck;               // the TCP transport's checksum setting (buffer sizes depend on it)
  int variant;               // diagnostic ablation (0 = product path)
  const uint32_t* skip = nullptr;  // TCP: a device word; non-zero = store nothing (the plan's
                                   // verdict on a launch made before the host has read it)
};

hipError_t launch_unpack(const UnpackParams& p, int grid, hipStream_t stream, int* which);
// tuning knob (mgenx_set_tuning): 0 = auto (pipelined fixed-length kernel when the batch
// qualifies), 1/2 = ablations of the general kernel, 3 = general kernel only
int unpack_threads();
#if MGENX_DIAG
hipError_t launch_group_rw(const uint8_t* p, uint64_t bytes, uint8_t* out, int mode, int grid,
                           hipStream_t stream);
hipError_t launch_stream_read(const uint8_t* p, uint64_t bytes, uint32_t* out, int grid,
                              hipStream_t stream);
hipError_t launch_stream_read_w(const uint8_t* p, uint64_t bytes, uint32_t* out, int grid,
                                int width, hipStream_t stream);
#endif
hipError_t launch_pack(const PackParams& p, int grid, hipStream_t stream);
hipError_t launch_pack_prepare(const mgenx_flow_tmpl* tmpl, uint32_t n_tmpl, const uint8_t* pool,
                               const uint32_t* byte_tab, uint32_t* out, hipStream_t stream);
// MgenAnalytic::Report quantizer tables (built on the host at context creation)
constexpr int kRqUnqTime = 0;          // [256] UnquantizeTimeValue(q)
constexpr int kRqThrTime = 256;        // [256] first value with QuantizeTimeValue >= k (k >= 2)
constexpr int kRqLog10Lo = -40;        // (int)log10 thresholds for e = -40 .. 24
constexpr int kRqLog10N = 65;
constexpr int kRqThrLog10 = 512;
constexpr int kRqP10 = 512 + 65;       // [309] pow(10, e)
constexpr int kRqP10N = 309;
constexpr int kRqDoubles = 512 + 65 + 309;

// TCP receiver's persistent rx_msg (mgenx_rx.hip)
hipError_t launch_rx_persist(const mgenx_cols& c, uint32_t n, uint32_t opts, int32_t* ws,
                             mgenx_rx_state* state, const uint8_t* slab, const uint64_t* rec_off,
                             const uint32_t* rec_len, const uint32_t* byte_tab,
                             uint32_t* payload_rec, hipStream_t s);
size_t rx_persist_ws_bytes(uint32_t n);
// TCP transmit (mgenx_tcp.hip)
hipError_t launch_tcp_plan(const mgenx_flow_tmpl* tmpl, const mgenx_pack_desc* desc,
                           const uint32_t* msg_total, uint32_t n, uint64_t* bytes,
                           uint32_t* nfrag, uint32_t* max_frag, hipStream_t s);
hipError_t launch_tcp_frag(const mgenx_pack_desc* desc, const uint32_t* msg_total,
                           const uint32_t* nfrag, const uint64_t* msg_off, uint32_t n, uint32_t r,
                           int ck, const uint32_t* prev_state, mgenx_pack_desc* fd, uint64_t* foff,
                           uint32_t* fbuf, uint32_t* ff, hipStream_t s);
// the plan, offsets and round 0's descriptors in one launch (kTcpPlanMsgs messages a block),
// its verdict to *skip and, as one 16-byte write, to host-mapped memory: the stream bytes,
// then epoch << 48 | fail << 32 | rounds
constexpr uint32_t kTcpPlanMsgs = 1024;
constexpr uint32_t kTcpPlanEpochs = 1u << 16;
hipError_t launch_tcp_plan0(const mgenx_flow_tmpl* tmpl, const mgenx_pack_desc* desc,
                            const uint32_t* msg_total, uint32_t n, int ck, uint64_t cap,
                            uint32_t epoch, uint64_t* status, uint64_t* fmax, uint64_t* msg_off,
                            uint32_t* nfrag, mgenx_pack_desc* fd, uint32_t* fbuf, uint32_t* ff,
                            uint32_t* skip, uint64_t* host, hipStream_t s);
// the resident single-message worker (mgenx_worker.hip): a request block the host writes (in
// fine-grained device memory the host stores into through the BAR when the runtime grants the
// CPU access to it, else in pinned host memory) and a reply block in pinned host memory
constexpr uint32_t kWorkUnpack = 1, kWorkCrc32 = 2, kWorkPack = 3, kWorkRecv = 4, kWorkUpdate = 5,
                   kWorkStop = 15;
constexpr uint32_t kWorkerMaxBytes = MGENX_WORKER_MAX_BYTES;
constexpr uint32_t kWorkerHdrBytes = 1024;  // Unpack reads at most the first 24+255+4+255+19 B
constexpr uint32_t kWorkerPackMax = MGENX_WORKER_PACK_MAX;  // Pack's bufferLen (built in LDS)
struct WPackReq {         // mgenx_pack_msgs' inputs for one message (payload in WReq::data)
  mgenx_flow_tmpl tmpl;   // words 0..16
  mgenx_pack_desc desc;   // words 17..21
  uint32_t buf_len, crc_in, opts, rsv;
};
struct WUpdReq {          // MgenAnalytic::Update of one record on a device flow state
  uint64_t flows;         // mgenx_flow_state* (device)
  uint32_t slot, seq, rx_sec, rx_usec, tx_sec, tx_usec, msg, rsv;
};
// The request: 16 pieces of 16 bytes that the worker reads whole on every poll, each written by
// the host with one 16-byte store: piece 0 = {request number, op << 28 | len, arg, 0}, written
// last; pieces 1-15 = {12 bytes of request data, request number}.  The data are the first
// kPollData bytes of the message (Unpack: the header, in the common case all of it), the
// WPackReq (Pack) or the WUpdReq (Update), so the poll that sees a request brings its data too.
// A piece whose tag is not the request number was read before the host wrote it: the worker
// polls again.
// The reply: up to 48 words in 16 TAGGED 16-byte chunks, chunk k = {w[3k], w[3k+1], w[3k+2],
// request number}, each written by one 16-byte store, so the host reads a chunk whole and knows
// from its tag that it is this request's -- no release fence (a wait for the stores'
// acknowledgement) between the reply and the worker's next poll.  Chunk 7 ends every reply (the
// host spins on it).  Words: the mgenx_unpacked (0-21), status (22: low byte 0 = ok; 0x100 the
// receive CRC was computed, 0x200 a window closed), crc (23); pack: ret (19), tx_crc (20),
// state (21); update: the mgenx_flow_report (24-47).
constexpr uint32_t kWorkOpShift = 28, kWorkLenMask = (1u << kWorkOpShift) - 1u;
constexpr uint32_t kPollPieces = 16, kPollData = 12u * (kPollPieces - 1u);  // 180 bytes
constexpr uint32_t kReplyStatus = 22, kReplyCrc = 23, kReplyRet = 19, kReplyTx = 20, kReplyState = 21;
constexpr uint32_t kReplyReport = 24, kReplyChunks = 16;
constexpr uint32_t kStatusCrc = 0x100u, kStatusClosed = 0x200u;
struct alignas(64) WReq {
  uint32_t poll[4 * kPollPieces];
  uint8_t data[kWorkerMaxBytes + 64];  // the message (beyond the polled bytes); 64 bytes of slack
};
struct alignas(64) WRep {
  uint32_t resp;    // stop requests: the reply number
  uint32_t alive;   // 1 while a launched worker runs (it clears the word when it ends)
  uint32_t rsv1[14];
  uint32_t reply[4 * kReplyChunks];  // tagged chunks
  uint8_t out[kWorkerPackMax + 64];  // a packed message
};
static_assert(sizeof(WPackReq) <= kPollData, "Pack's request travels in the polled pieces");
static_assert(sizeof(WUpdReq) <= kPollData, "Update's request travels in the polled pieces");
// the context's operator tables (mgenx_api.hip: A_n(s) = the state after n zero bytes, as 4 x 256
// byte-indexed entries): [A64 | A4 | A8 | A12 | A16 | A32 | A48 | A128 | A256 | A512 | A1024]
constexpr uint32_t kTabA64 = 0, kTabA4 = 1, kTabA8 = 2, kTabA16 = 4, kTabA32 = 5, kTabA128 = 7,
                   kTabA256 = 8, kTabA512 = 9, kTabA1024 = 10, kTabCount = 11;
hipError_t launch_worker(const WReq* q, WRep* m, const uint32_t* tabs, const uint32_t* byte_tab,
                         const uint8_t* rtab, uint32_t start, uint64_t idle_ticks,
                         hipStream_t stream);
hipError_t launch_crc32(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                        const uint32_t* byte_tab, const uint32_t* a4_tab, const uint32_t* xpow,
                        const uint32_t* state_in, uint32_t* out, hipStream_t stream);

}  // namespace mgenx
