/*
 * mgenx_diag.h -- diagnostics of libmgenx_diag.so (NOT part of the product ABI).
 *
 * libmgenx_diag.so is built from the same sources as libmgenx.so with the kernel ablation
 * variants and the memory-pattern probes compiled in; benchmark and tuning scripts load it
 * (mgen_amd.Engine(diag=True)).  The product library exports none of these symbols.
 */
#ifndef MGENX_DIAG_H
#define MGENX_DIAG_H

#include "mgenx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tuning knobs (per context; for benchmarking kernel variants).  MGENX_TUNE_UNPACK_VARIANT:
 * 0 = automatic (pipelined fixed-length kernel when the batch qualifies), 1/2 = ablations
 * of the general kernel (loads+XOR only / lookups on cached rows), 3 = general kernel,
 * 12 = fixed-length kernel with a separate header load (1024-B records), 1024 + M =
 * ablation bit mask M of the aligned 1024-B kernel (1 = no LDS lookups, 2 = no decode and
 * no stores, 4 = decode without stores, 8 = stores to a scratch line, 16 = the other store
 * cache policy, 32 = stores wrapped onto the first 16K records, 64 = write-through stores,
 * 128 = non-temporal row loads, 256 (with 4) = dummy rows stored after each wave's last
 * group), 40-45 = long-record kernel shapes (rows per block x threads: 16x512, 8x512,
 * 4x1024, 12x512, 2x1024, 16x1024). */
#define MGENX_TUNE_UNPACK_VARIANT 1
/* MGENX_TUNE_PACK_VARIANT: 0 = product; ablations 1 = no unit stores, 2 = no CRC work, 3-6
 * store-scheme ablations, 7-9 = grid x2..x4, 10 = the meta waves never help the joint
 * store.  (Env MGENX_PACK_GRID: the grid, diagnostics build only.) */
#define MGENX_TUNE_PACK_VARIANT 2
int mgenx_set_tuning(mgenx_ctx* ctx, int key, int value);
/* Diagnostic: plain 16-B-per-lane streaming read of `bytes` (the achievable-HBM reference
 * next to the roofline); dev_scratch holds `grid` words. */
int mgenx_diag_stream_read(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                           uint32_t* dev_scratch, int grid, void* stream);
/* Diagnostic: the same read at `width` bytes per lane (4, 8 or 24), coalesced -- FETCH_SIZE
 * calibration for the config-4 kernels' access shapes. */
int mgenx_diag_stream_read_w(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                             uint32_t* dev_scratch, int grid, int width, void* stream);
/* Diagnostic: the fixed-length unpack's memory pattern without its compute -- waves take
 * 16-KiB groups of `data` round-robin (16 loads of 1 KiB each, consumed by XOR) and, when
 * `mode` & 1, store 512 B per group to dev_out (bytes / 32 bytes); `mode` & 2: the stores
 * are write-through (sc1). */
int mgenx_diag_group_rw(mgenx_ctx* ctx, const uint8_t* dev_data, uint64_t bytes,
                        uint8_t* dev_out, int mode, void* stream);

/* Diagnostic: s_memtime phase cycles of the analytics kernels' first wave: n == 10
 * flow_update_kernel (detect, bulk, exact, lat' stores, rounds, exact steps, bulk runs, total,
 * restart cycles, restarts); n == 16 flow_order_kernel (8 entries). */
int mgenx_diag_seg_prof(unsigned long long* out, int n);

/* Diagnostic: the resident worker's own time for its last Unpack / receive request, in 10-ns
 * ticks from the poll that saw it: header parsed, checksum done, reply stored; out[3] = the
 * request number they belong to; out[4], out[5] = shader clocks (s_memtime) to the parse and
 * to the reply (out[7] = the request number); out holds 8 words. */
int mgenx_diag_worker_stamps(const mgenx_worker* w, uint32_t* out);

/* Diagnostic: s_memtime stamps of the scan's chain kernel (scan_chain_kernel), thread 0 of
 * groups 0..63, 8 per group: start, counts prefix, marks, H list, look-back, end; out holds
 * 512 words. */
int mgenx_diag_chain_prof(unsigned long long* out);

#ifdef __cplusplus
}
#endif
#endif
