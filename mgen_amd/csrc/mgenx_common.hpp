// mgenx_common.hpp -- shared device helpers for the MI355X MgenMsg engine.
//
// CRC-32 here is the reference's reflected CRC (poly 0x04C11DB7 reflected = 0xEDB88320,
// init/xorout 0xFFFFFFFF; src/common/mgenMsg.cpp:524-554, table :576-642), evaluated with
// GF(2)-linear "shift operators": A_n(s) is the CRC state after feeding n zero bytes to
// state s with the byte-table update s = T[(s ^ b) & 0xff] ^ (s >> 8).  A_n is linear, so
// it is applied as four 256-entry tables (one per state byte), and
//     crc_raw(X || Y) = A_|Y|(crc_raw(X)) ^ crc_raw(Y)       (crc_raw = zero initial state)
//     crc_init(X)     = crc_raw(X) ^ A_|X|(0xFFFFFFFF)
// which lets lanes compute disjoint pieces of one record independently.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mgenx.h"

namespace mgenx {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kWave = 64;

// ---- unaligned global access (gfx950 runs in unaligned-access mode: one dword / dwordx4
//      instruction per access, split by the TA when it straddles lines) ----
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_u1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32_u1 __attribute__((aligned(1)));
typedef uint16_t u16_u1 __attribute__((aligned(1)));

__device__ __forceinline__ u32x4_t ldu128(const uint8_t* p) {
  return *reinterpret_cast<const u32x4_u1*>(p);
}
// Same load, but pinned in program order (volatile): used for software-pipelined
// prefetches that the compiler would otherwise sink next to their first use.
__device__ __forceinline__ u32x4_t ldu128_pinned(const uint8_t* p) {
  return *reinterpret_cast<const volatile u32x4_u1*>(p);
}
// Streaming (non-temporal) 16-byte load: record bodies are read once.  gfx950 runs in
// unaligned-access mode, so the aligned vector type only fixes the instruction choice.
__device__ __forceinline__ u32x4_t ldnt128(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
}
__device__ __forceinline__ uint32_t ldu32(const uint8_t* p) {
  return *reinterpret_cast<const u32_u1*>(p);
}
__device__ __forceinline__ uint16_t ldu16(const uint8_t* p) {
  return *reinterpret_cast<const u16_u1*>(p);
}
__device__ __forceinline__ void stu128(uint8_t* p, u32x4_t v) {
  *reinterpret_cast<u32x4_u1*>(p) = v;
}

// Stores through an integer address known to be global memory (a per-lane choice of
// column base pointers is computed as integers: see unpack_fixed_kernel's tail).
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ void st_g8(uint64_t a, uint32_t v) { *(g_u8*)a = (uint8_t)v; }
__device__ __forceinline__ void st_g16(uint64_t a, uint32_t v) { *(g_u16*)a = (uint16_t)v; }
__device__ __forceinline__ void st_g32(uint64_t a, uint32_t v) { *(g_u32*)a = v; }
typedef __attribute__((address_space(1))) uint64_t g_u64;
__device__ __forceinline__ void st_g64(uint64_t a, uint64_t v) { *(g_u64*)a = v; }
__device__ __forceinline__ void st_g64_nt(uint64_t a, uint64_t v) {
  __builtin_nontemporal_store(v, (g_u64*)a);
}
__device__ __forceinline__ void st_g32_nt(uint64_t a, uint32_t v) {
  __builtin_nontemporal_store(v, (g_u32*)a);
}
__device__ __forceinline__ void st_g16_nt(uint64_t a, uint32_t v) {
  __builtin_nontemporal_store((uint16_t)v, (g_u16*)a);
}
__device__ __forceinline__ void st_g8_nt(uint64_t a, uint32_t v) {
  __builtin_nontemporal_store((uint8_t)v, (g_u8*)a);
}
// Write-through stores (`sc1`: the line leaves L2 with the store instead of staying dirty
// there; MI355X_MICROARCH.md, store flavours)
__device__ __forceinline__ void st_g64_wt(uint64_t a, uint64_t v) {
  __hip_atomic_store((g_u64*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_g32_wt(uint64_t a, uint32_t v) {
  __hip_atomic_store((g_u32*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_g16_wt(uint64_t a, uint32_t v) {
  __hip_atomic_store((g_u16*)a, (uint16_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_g8_wt(uint64_t a, uint32_t v) {
  __hip_atomic_store((g_u8*)a, (uint8_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a[k] for k = sel in 0..3, as AND/OR masks (a select chain over struct fields or arrays
// can be folded back into a dynamic index into a stack copy)
__device__ __forceinline__ uint64_t pick4(int sel, uint64_t a0, uint64_t a1, uint64_t a2,
                                          uint64_t a3) {
  const uint64_t m0 = 0ull - (uint64_t)(sel == 0), m1 = 0ull - (uint64_t)(sel == 1);
  const uint64_t m2 = 0ull - (uint64_t)(sel == 2), m3 = 0ull - (uint64_t)(sel == 3);
  return (a0 & m0) | (a1 & m1) | (a2 & m2) | (a3 & m3);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint16_t bswap16(uint16_t x) { return __builtin_bswap16(x); }

// GF(2) multiply mod P in reflected representation (bit 31 = x^0), branch-free.
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    p ^= ((a >> (31 - i)) & 1u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
  }
  return p;
}

// x^(8 n) mod P for any n from the [65536] table: low 16 bits from the table, the rest by
// square-and-multiply of x^(8 * 65536)
__device__ __forceinline__ uint32_t xpow8(uint32_t n, const uint32_t* xpow) {
  if (n < 65536u) return xpow[n];
  uint32_t r = xpow[n & 0xFFFFu];
  uint32_t sq = xpow[32768];
  sq = multmodp(sq, sq);
  for (n >>= 16; n; n >>= 1) {
    if (n & 1u) r = multmodp(r, sq);
    sq = multmodp(sq, sq);
  }
  return r;
}

// Byte-mask helpers: bytes [lo, hi) of a little-endian 32-bit word, lo/hi in [0,4].
__device__ __forceinline__ uint32_t byte_range_mask(int lo, int hi) {
  uint32_t m_hi = hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
  uint32_t m_lo = lo >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lo)) - 1u);
  return lo >= hi ? 0u : (m_hi & ~m_lo);
}

}  // namespace mgenx
