// Diagnostic microbenchmark (not product code): read a 1 GiB slab of 1 KiB records with
// the access shapes an unpack kernel could use, 16 waves per CU (1024-thread persistent
// blocks), every wave issuing its whole 16 KiB group as one burst before consuming it.
//   S = lanes per record segment: 4 -> 16 records x 64 B per load instruction,
//   8 -> 8 x 128 B, 16 -> 4 x 256 B, 64 -> one contiguous 1 KiB record per instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int S, int THREADS>
__global__ void __launch_bounds__(THREADS) pat(const u32x4* __restrict__ slab, uint64_t n_rec,
                                               uint32_t* out) {
  constexpr int RPI = 64 / S;            // records per load instruction
  constexpr int ROWS = 1024 / (16 * S);  // load instructions per record
  constexpr int LOADS = 16;              // per lane per group (16 KiB per wave)
  constexpr int RECS = RPI * LOADS / ROWS;  // records per group
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (THREADS / 64);
  uint32_t acc = 0;
  for (uint64_t g = wave; g * RECS < n_rec; g += nw) {
    u32x4 d[LOADS];
#pragma unroll
    for (int k = 0; k < LOADS; k++) {
      const int rec_in_group = (k / ROWS) * RPI + lane / S;
      const int row = k % ROWS;
      const uint64_t rec = g * RECS + rec_in_group;
      d[k] = slab[rec * 64 + row * S + (lane % S)];
    }
#pragma unroll
    for (int k = 0; k < LOADS; k++) acc ^= d[k].x ^ d[k].y ^ d[k].z ^ d[k].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int S, int T>
float run(const u32x4* p, uint64_t n, uint32_t* o, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  pat<S, T><<<blocks, T>>>(p, n, o);
  hipEventRecord(a);
  for (int i = 0; i < 10; i++) pat<S, T><<<blocks, T>>>(p, n, o);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const uint64_t n = 1 << 20, bytes = n * 1024;
  u32x4* p; uint32_t* o;
  hipMalloc(&p, bytes); hipMalloc(&o, 64);
  hipMemset(p, 1, bytes);
  int cu = 256;
  for (int rep = 0; rep < 3; rep++) {
    printf("S4  1024thr: %.4f ms\n", run<4, 1024>(p, n, o, cu));
    printf("S8  1024thr: %.4f ms\n", run<8, 1024>(p, n, o, cu));
    printf("S16 1024thr: %.4f ms\n", run<16, 1024>(p, n, o, cu));
    printf("S64 1024thr: %.4f ms\n", run<64, 1024>(p, n, o, cu));
    printf("S4  256thr x4/CU: %.4f ms\n", run<4, 256>(p, n, o, cu * 4));
    printf("S64 256thr x8/CU: %.4f ms\n", run<64, 256>(p, n, o, cu * 8));
  }
  return 0;
}
