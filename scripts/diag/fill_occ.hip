// Store-rate probe: zero-fill 1 GiB with 16-B stores (global_store_dwordx4, 1 KB per wave
// instruction).  Workgroups of 256 threads; resident waves per CU set by a dynamic LDS pad.
// Address orders: the slab in pieces of `piece` bytes; piece j goes to workgroup j mod grid
// (grid-stride), and inside a piece the 4 waves interleave 1-KB rows (wave w: rows w, w+4, ...).
// piece = 1 KB x 4 is a 1-KB interleave over all waves; large pieces are per-workgroup chunks.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) fill_kernel(uint8_t* buf, uint64_t n, uint64_t piece) {
  extern __shared__ uint32_t pad[];
  if (n == 0) pad[threadIdx.x] = 0;  // (keeps the LDS allocation)
  const uint64_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (uint64_t c = (uint64_t)blockIdx.x * piece; c < n; c += (uint64_t)gridDim.x * piece)
    for (uint64_t a = c + wv * 1024 + 16 * lane; a < c + piece; a += 4096) *(u32x4*)(buf + a) = z;
}

int main() {
  const uint64_t n = 1ull << 30;
  uint8_t* buf;
  if (hipMalloc(&buf, n) != hipSuccess) return 1;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipFuncSetAttribute((const void*)fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int wg_per_cu : {1, 2, 4, 8}) {
    for (uint64_t piece : {4096ull, 16384ull, 65536ull, 262144ull, 1048576ull}) {
      const size_t lds = (160 * 1024) / wg_per_cu - 1024;
      for (int grid_mul : {1, 16}) {  // resident grid, or 16x as many workgroups (retiring)
        const int grid = cus * wg_per_cu * grid_mul;
        for (int w = 0; w < 3; w++)
          hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), lds, 0, buf, n, piece);
        (void)hipEventRecord(a, 0);
        for (int r = 0; r < 20; r++)
          hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), lds, 0, buf, n, piece);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("waves/CU %2d piece %7llu grid x%-2d ms %.4f\n", wg_per_cu * 4,
               (unsigned long long)piece, grid_mul, ms / 20);
      }
    }
  }
  (void)hipFree(buf);
  return 0;
}
