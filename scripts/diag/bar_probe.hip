// bar_probe.hip -- can the host write a worker's request straight into device memory?
// The resident worker (mgenx_worker.hip) polls a mailbox in pinned host memory: the poll that
// sees a request is one host-memory round trip, reading a message longer than the polled bytes
// is another, and the reply a third (3.5-3.7 us per call).  If the host can store into
// fine-grained device memory (through the PCIe BAR), the request arrives as posted writes and the
// wave polls local memory: the call becomes two one-way trips.  This probe asks the runtime for
// such a mapping (fine-grained device memory, then hsa_amd_agents_allow_access for the CPU
// agent), checks that host stores arrive intact and in order, and times request -> reply with
// a 1 KiB message against the host-memory mailbox.
// The worker always exits: on a stop request, and after kIdleTicks of wall clock with no
// request (s_memrealtime, 100 MHz); the host waits for it before the process ends.
// usage: bar_probe [iterations]   prints one JSON object
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>

struct alignas(64) Req {
  uint32_t req;        // request sequence number (host writes last); 0xFFFFFFFF = stop
  uint32_t len;
  uint32_t pad0[14];
  uint32_t data[256];  // the message, 1 KiB
};
struct alignas(64) Resp {
  uint32_t resp;  // reply sequence number (worker writes last)
  uint32_t fold;  // XOR of the message words
  uint32_t pad[14];
};

constexpr uint64_t kIdleTicks = 100ull * 1000 * 1000;  // 1 s at 100 MHz

__global__ void __launch_bounds__(64) worker(const Req* q, Resp* p, uint32_t* served) {
  const uint32_t lane = threadIdx.x;
  uint32_t last = 0, n = 0;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint32_t r = 0;
    if (lane == 0) r = __hip_atomic_load(&q->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    r = __shfl(r, 0);
    if (r == 0xFFFFFFFFu) break;
    if (r == last) {
      if (__builtin_amdgcn_s_memrealtime() - t_last > kIdleTicks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    last = r;
    uint32_t x = 0;
    for (int k = 0; k < 4; k++)
      x ^= __hip_atomic_load(&q->data[lane + 64 * k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (lane == 0) {
      __hip_atomic_store(&p->fold, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&p->resp, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    n++;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (lane == 0) served[0] = n;
}

static double pct(std::vector<double> v, double f) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(f * (v.size() - 1))];
}

// q_host: the host's view of the request block, q_dev: the device's; p_*: the reply block
static int run(Req* q_host, const Req* q_dev, Resp* p_host, Resp* p_dev, int iters,
               const char* name, bool last) {
  uint32_t* served;
  if (hipMalloc(&served, 4) != hipSuccess) return 1;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int k = 0; k < 256; k++) q_host->data[k] = 0;
  q_host->req = 0;
  memset((void*)p_host, 0, sizeof(Resp));
  _mm_sfence();
  std::atomic_thread_fence(std::memory_order_seq_cst);
  hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, s, q_dev, p_dev, served);
  std::vector<double> us;
  volatile uint32_t* resp = &p_host->resp;
  int bad = 0, lost = 0;
  for (int i = 1; i <= iters; i++) {
    auto t0 = std::chrono::steady_clock::now();
    uint32_t want = 0;
    alignas(16) uint32_t tmp[256];
    for (int k = 0; k < 256; k++) {
      tmp[k] = (uint32_t)(i * 2654435761u + k);
      want ^= tmp[k];
    }
    for (int k = 0; k < 256; k += 4)  // 16-byte stores, then a fence before the doorbell
      _mm_store_si128(reinterpret_cast<__m128i*>(&q_host->data[k]),
                      _mm_load_si128(reinterpret_cast<const __m128i*>(&tmp[k])));
    _mm_sfence();
    *reinterpret_cast<volatile uint32_t*>(&q_host->req) = (uint32_t)i;
    _mm_sfence();
    bool ok = true;
    while (*resp != (uint32_t)i) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.5) {
        ok = false;  // worker gone or the request never arrived
        break;
      }
      _mm_pause();
    }
    auto t1 = std::chrono::steady_clock::now();
    if (!ok) {
      if (++lost > 2) break;
      continue;
    }
    if (*reinterpret_cast<volatile uint32_t*>(&p_host->fold) != want) bad++;
    us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    if (bad > 3) break;
  }
  *reinterpret_cast<volatile uint32_t*>(&q_host->req) = 0xFFFFFFFFu;
  _mm_sfence();
  hipStreamSynchronize(s);
  uint32_t n = 0;
  hipMemcpy(&n, served, 4, hipMemcpyDeviceToHost);
  if (us.empty()) us.push_back(-1.0);
  printf("\"%s\": {\"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"served\": %u, "
         "\"bad\": %d, \"lost\": %d}%s\n",
         name, pct(us, 0.5), pct(us, 0.1), pct(us, 0.9), n, bad, lost, last ? "" : ",");
  hipStreamDestroy(s);
  hipFree(served);
  return bad || lost;
}

static hsa_status_t find_cpu(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 3000;
  if (hipSetDevice(0) != hipSuccess) return 1;
  printf("{\n");
  int bad = 0;
  // 1. both blocks in pinned host memory (the product's mailbox today)
  Req* qh = nullptr;
  Resp* ph = nullptr;
  if (hipHostMalloc((void**)&qh, sizeof(Req), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostMalloc((void**)&ph, sizeof(Resp), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    printf("\"error\": \"hipHostMalloc\"}\n");
    return 1;
  }
  Req* qd = nullptr;
  Resp* pd = nullptr;
  hipHostGetDevicePointer((void**)&qd, qh, 0);
  hipHostGetDevicePointer((void**)&pd, ph, 0);
  bad += run(qh, qd, ph, pd, iters, "host_mailbox", false);
  // 2. the request block in fine-grained device memory the CPU agent may access
  Req* g = nullptr;
  const bool alloc_ok = hipExtMallocWithFlags((void**)&g, sizeof(Req), hipDeviceMallocFinegrained) == hipSuccess;
  hsa_agent_t cpu;
  cpu.handle = 0;
  hsa_iterate_agents(find_cpu, &cpu);
  hsa_status_t st = HSA_STATUS_ERROR;
  if (alloc_ok && cpu.handle) st = hsa_amd_agents_allow_access(1, &cpu, nullptr, g);
  printf("\"device_request_alloc\": %d, \"cpu_agent\": %d, \"allow_access_status\": %d,\n",
         (int)alloc_ok, cpu.handle ? 1 : 0, (int)st);
  if (alloc_ok && st == HSA_STATUS_SUCCESS) {
    // host stores -> device copy -> host compare: the BAR path carries the bytes intact
    alignas(16) uint32_t pat[256], back[256];
    for (int k = 0; k < 256; k++) {
      pat[k] = 0x9E3779B9u * (uint32_t)(k + 1);
      reinterpret_cast<volatile uint32_t*>(g->data)[k] = pat[k];
    }
    _mm_sfence();
    const bool cp = hipMemcpy(back, g->data, sizeof(back), hipMemcpyDeviceToHost) == hipSuccess;
    printf("\"bar_write_roundtrip_ok\": %d,\n", (int)(cp && memcmp(pat, back, sizeof(pat)) == 0));
    bad += run(g, g, ph, pd, iters, "device_request_host_reply", true);
  } else {
    printf("\"device_request_host_reply\": \"no CPU access\"\n");
  }
  printf("}\n");
  hipHostFree(qh);
  hipHostFree(ph);
  if (g) hipFree(g);
  return bad ? 2 : 0;
}
