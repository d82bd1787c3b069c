// zh_launch.h — host-side entry points into the device pipeline (K1 lz, K2 entropy, K3 gather).
#pragma once
#include "zh_common.h"

// Per-item bookkeeping for frames that span several device blocks.
struct ZhItemDesc {
  u8 *dst;           // item output
  u64 cap;           // item output capacity
  u32 first_block;   // index of the item's first ZhBlockDesc
  u32 nblocks;       // number of device blocks in the frame
};

// Staging slot for one block of a multi-block frame: worst case = raw block + frame header.
#define ZH_STAGE_SLOT ((u32)ZH_BLOCK_MAX + 64u)

namespace zh {
hipError_t init_kernels();
u32 lz_lds_bytes();
u32 entropy_lds_bytes();
hipError_t launch_compress(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 window_log, u32 cfg_block_size, u64 *d_item_size,
                           u32 *d_item_status, u32 *d_blk_size, const ZhItemDesc *d_items, u32 nitems, bool gather, hipStream_t stream);
void profile_enable(bool on);
int profile_collect(double *totals);
hipError_t launch_plan(const void *const *d_in_ptrs, const size_t *d_in_sizes, u32 nitems, u32 bpi, void *const *d_out_ptrs, u64 out_cap,
                       u8 *staging, ZhBlockDesc *d_descs, ZhItemDesc *d_items, u64 *d_item_size, u32 *d_item_status, hipStream_t stream);
}  // namespace zh
