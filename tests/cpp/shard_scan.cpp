// shard_scan.cpp -- mgenx::ShardedScan (include/mgenx.hpp) with simulated ranks: `world`
// threads on one GPU, one mgenx context each, exchanging through an in-process all-gather
// (ThreadComm); world 1 runs over a real one-rank RCCL communicator (RcclShardComm).
// Writes, for the whole stream: the union of the ranks' records (global offsets, lengths)
// and every rank's summary, for tests/test_gpu_shard_cpp.py to compare with
// mgenx_stream_scan.
// usage: shard_scan <stream file> <mode 0 TCP | 1 SINK> <world> <out file>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "mgenx.hpp"

// all-gather among the threads of this process (a generation-counted barrier)
class ThreadComm {
 public:
  explicit ThreadComm(int world) : world_(world), slots_(world) {}
  class View : public mgenx::ShardComm {
   public:
    View(ThreadComm& p, int rank) : p_(p), rank_(rank) {}
    int World() const override { return p_.world_; }
    int Rank() const override { return rank_; }
    std::vector<uint64_t> AllGather(const std::vector<uint64_t>& in) override {
      std::unique_lock<std::mutex> lk(p_.mu_);
      p_.slots_[rank_] = in;
      Arrive(lk);
      std::vector<uint64_t> out;
      for (const auto& v : p_.slots_) out.insert(out.end(), v.begin(), v.end());
      Arrive(lk);  // nobody overwrites a slot before every rank has read them all
      return out;
    }

   private:
    void Arrive(std::unique_lock<std::mutex>& lk) {
      const uint64_t gen = p_.gen_;
      if (++p_.count_ == p_.world_) {
        p_.count_ = 0;
        p_.gen_++;
        p_.cv_.notify_all();
      } else {
        p_.cv_.wait(lk, [&] { return p_.gen_ != gen; });
      }
    }
    ThreadComm& p_;
    int rank_;
  };

 private:
  int world_;
  std::vector<std::vector<uint64_t>> slots_;
  std::mutex mu_;
  std::condition_variable cv_;
  int count_ = 0;
  uint64_t gen_ = 0;
};

struct RankOut {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  mgenx::ShardScanResult res;
  std::string err;
};

static void run_rank(const std::vector<uint8_t>& stream, int mode, mgenx::ShardComm& comm,
                     mgenx::Context& ctx, RankOut& out) {
  try {
    uint64_t a, b, hi;
    mgenx::ShardedScan::Bounds(stream.size(), comm.World(), comm.Rank(), a, b, hi);
    mgenx::DeviceArray<uint8_t> d(hi - a + 1);
    mgenx::check_hip(hipMemcpy(d.data(), stream.data() + a, hi - a, hipMemcpyHostToDevice), "H2D");
    const uint64_t cap = (hi - a) / 2 + 2;
    mgenx::DeviceArray<uint64_t> off(cap);
    mgenx::DeviceArray<uint32_t> len(cap);
    mgenx::ShardedScan sc(ctx, comm);
    out.res = sc.Run(d.data(), stream.size(), mode, off.data(), len.data(), cap);
    const uint64_t n = std::min<uint64_t>(out.res.n_local, cap);
    out.off.resize(n);
    out.len.resize(n);
    mgenx::check_hip(hipMemcpy(out.off.data(), off.data(), n * 8, hipMemcpyDeviceToHost), "D2H");
    mgenx::check_hip(hipMemcpy(out.len.data(), len.data(), n * 4, hipMemcpyDeviceToHost), "D2H");
    for (auto& o : out.off) o += out.res.a;
  } catch (const std::exception& e) {
    out.err = e.what();
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <stream> <mode> <world> <out>\n", argv[0]);
    return 2;
  }
  std::vector<uint8_t> stream;
  {
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    uint8_t buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) stream.insert(stream.end(), buf, buf + got);
    std::fclose(f);
  }
  const int mode = std::atoi(argv[2]), world = std::atoi(argv[3]);
  std::vector<RankOut> outs(world);
  if (world == 1) {  // one rank over a real RCCL communicator
    mgenx::Context ctx(0);
    uint8_t id[MGENX_COMM_ID_BYTES];
    mgenx_comm* comm = nullptr;
    if (mgenx_comm_unique_id(id) != MGENX_OK || mgenx_comm_init(ctx.get(), 1, 0, id, &comm) != MGENX_OK) {
      std::fprintf(stderr, "RCCL init failed\n");
      return 3;
    }
    mgenx::RcclShardComm rc(ctx, comm, 1, 0);
    run_rank(stream, mode, rc, ctx, outs[0]);
    mgenx_comm_destroy(comm);
  } else {
    ThreadComm tc(world);
    std::vector<std::unique_ptr<ThreadComm::View>> views;
    std::vector<std::unique_ptr<mgenx::Context>> ctxs;
    for (int r = 0; r < world; r++) {
      views.emplace_back(new ThreadComm::View(tc, r));
      ctxs.emplace_back(new mgenx::Context(0));
    }
    std::vector<std::thread> th;
    for (int r = 0; r < world; r++)
      th.emplace_back(run_rank, std::cref(stream), mode, std::ref(*views[r]), std::ref(*ctxs[r]),
                      std::ref(outs[r]));
    for (auto& t : th) t.join();
  }
  FILE* o = std::fopen(argv[4], "wb");
  uint64_t total = 0;
  for (const auto& r : outs) {
    if (!r.err.empty()) {
      std::fprintf(stderr, "rank error: %s\n", r.err.c_str());
      return 1;
    }
    total += r.off.size();
  }
  std::fwrite(&total, 8, 1, o);
  for (const auto& r : outs) std::fwrite(r.off.data(), 8, r.off.size(), o);
  for (const auto& r : outs) std::fwrite(r.len.data(), 4, r.len.size(), o);
  for (const auto& r : outs) {
    const uint64_t s[3] = {r.res.n_total, r.res.consumed, (uint64_t)(uint32_t)r.res.status};
    std::fwrite(s, 8, 3, o);
  }
  std::fclose(o);
  std::printf("shard_scan: world %d, %llu records\n", world, (unsigned long long)total);
  return 0;
}
