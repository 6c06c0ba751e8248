// mailbox_probe.hip -- round-trip latency of a resident device worker polling a host-mapped
// mailbox (the design question behind the shim's single-message path): the host writes a
// request (a 1 KiB record and a sequence number), one resident wave notices it, reads the
// record, folds it, writes a reply and its sequence number back to host memory; the host spins
// on the reply.  Variants: the record read after the doorbell (two host-memory round trips) and
// the mailbox in fine-grained device memory the host writes through the BAR (when the runtime
// gives the host a mapping of it).
// The worker always exits: on a stop request, and after kIdleTicks of wall clock with no
// request (s_memrealtime, 100 MHz), and the host waits for it before the process ends.
// usage: mailbox_probe [iterations]   prints one JSON object
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>

struct alignas(64) Mail {
  uint32_t req;        // request sequence number (host writes last); 0xFFFFFFFF = stop
  uint32_t len;
  uint32_t pad0[14];
  uint32_t resp;       // reply sequence number (worker writes last)
  uint32_t fold;       // reply payload: XOR of the record words
  uint32_t pad1[14];
  uint32_t data[256];  // the record, 1 KiB
};

constexpr uint64_t kIdleTicks = 100ull * 1000 * 1000;  // 1 s at 100 MHz

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) worker(Mail* m, uint32_t* served) {
  const uint32_t lane = threadIdx.x;
  uint32_t last = 0, n = 0;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint32_t r = 0;
    if (lane == 0) r = ld_sys(&m->req);
    r = __shfl(r, 0);
    if (r == 0xFFFFFFFFu) break;
    if (r == last) {
      if (__builtin_amdgcn_s_memrealtime() - t_last > kIdleTicks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    last = r;
    // the record: 4 words per lane, read after the doorbell (acquire above)
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) x ^= __hip_atomic_load(&m->data[lane + 64 * k], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_SYSTEM);
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (lane == 0) {
      __hip_atomic_store(&m->fold, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      st_sys(&m->resp, r);
    }
    n++;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (lane == 0) served[0] = n;
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static int run(Mail* host_view, Mail* dev_view, int iters, const char* name, bool last) {
  uint32_t* served;
  hipMalloc(&served, 4);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  memset((void*)host_view, 0, sizeof(Mail));
  std::atomic_thread_fence(std::memory_order_seq_cst);
  hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, s, dev_view, served);
  std::vector<double> us;
  std::atomic<uint32_t>* req = reinterpret_cast<std::atomic<uint32_t>*>(&host_view->req);
  std::atomic<uint32_t>* resp = reinterpret_cast<std::atomic<uint32_t>*>(&host_view->resp);
  int bad = 0;
  for (int i = 1; i <= iters; i++) {
    auto t0 = std::chrono::steady_clock::now();
    uint32_t want = 0;
    for (int k = 0; k < 256; k++) {
      host_view->data[k] = (uint32_t)(i * 2654435761u + k);
      want ^= host_view->data[k];
    }
    req->store((uint32_t)i, std::memory_order_release);
    auto tw = t0;
    while (resp->load(std::memory_order_acquire) != (uint32_t)i) {
      tw = std::chrono::steady_clock::now();
      if (std::chrono::duration<double>(tw - t0).count() > 0.5) break;  // worker gone
    }
    auto t1 = std::chrono::steady_clock::now();
    if (resp->load(std::memory_order_acquire) != (uint32_t)i || host_view->fold != want) bad++;
    us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    if (bad > 3) break;
  }
  req->store(0xFFFFFFFFu, std::memory_order_release);
  hipStreamSynchronize(s);
  uint32_t n = 0;
  hipMemcpy(&n, served, 4, hipMemcpyDeviceToHost);
  printf("\"%s\": {\"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"served\": %u, \"bad\": %d}%s\n",
         name, median(us), [&] { auto v = us; std::sort(v.begin(), v.end()); return v[v.size() / 10]; }(),
         [&] { auto v = us; std::sort(v.begin(), v.end()); return v[v.size() * 9 / 10]; }(), n, bad,
         last ? "" : ",");
  hipStreamDestroy(s);
  hipFree(served);
  return bad;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 5000;
  printf("{\n");
  int bad = 0;
  // 1. pinned host memory, mapped to the device
  Mail* h = nullptr;
  if (hipHostMalloc((void**)&h, sizeof(Mail), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    printf("\"error\": \"hipHostMalloc\"}\n");
    return 1;
  }
  Mail* hd = nullptr;
  hipHostGetDevicePointer((void**)&hd, h, 0);
  bad += run(h, hd, iters, "host_pinned_coherent", false);
  // 2. fine-grained device memory, if the host can write it
  Mail* g = nullptr;
  bool dev_ok = hipExtMallocWithFlags((void**)&g, sizeof(Mail), hipDeviceMallocFinegrained) == hipSuccess;
  hipPointerAttribute_t at;
  if (dev_ok && hipPointerGetAttributes(&at, g) == hipSuccess && at.hostPointer) {
    bad += run((Mail*)at.hostPointer, g, iters, "device_finegrained", true);
  } else {
    printf("\"device_finegrained\": \"no host mapping (%d)\"\n", (int)dev_ok);
  }
  printf("}\n");
  hipHostFree(h);
  if (g) hipFree(g);
  return bad ? 2 : 0;
}
