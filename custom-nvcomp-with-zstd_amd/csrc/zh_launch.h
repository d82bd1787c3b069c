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

// Decoder launch (zh_decode.hip): one workgroup per input buffer; every array is a
// device array indexed by item.  Item i's workspace slot is ws + i * slot_bytes:
// block_cap literal bytes (padded to lit_bytes), then seq_cap u64 sequence records.
struct ZhDecArgs {
  const void *const *in_ptrs;  // null: a single item given by one_in / one_in_size / one_out
  const void *one_in;
  u64 one_in_size;
  void *one_out;
  const size_t *in_sizes;
  void *const *out_ptrs;
  const size_t *out_caps;  // per-item output capacity, or null: out_cap_all for every item
  u64 out_cap_all;
  size_t *out_sizes;       // bytes produced (0 on error)
  u32 *statuses;           // optional: Status values, or nvcomp codes when nvcomp_codes
  u8 *ws;
  u64 slot_bytes;
  u32 lit_bytes, block_cap, seq_cap, nvcomp_codes;
  u32 ho_off;  // offset of the item's hand-off record inside its slot (split pipeline)
  u32 phase;   // 0: whole decode in one kernel; 1 / 3: first / last kernel of the split pipeline
  u32 item0;   // first item of this launch (launch_decompress's pipelined groups)
  const u8 *dict;  // dictionary (device, whole buffer) or null; its content precedes every frame
  u64 dict_n;      // its size
  u32 dict_off;    // content offset (formatted dictionary: after tables + repcodes; raw: 0)
  u32 dict_id;     // Dictionary_ID (formatted), 0 for raw content
};
#define ZH_DEC_HANDOFF_BYTES 5376u  // sizeof(DecHandoff), zh_decode.hip

namespace zh {
u32 dec_lds_bytes();
// Split pipeline: phase-1 kernel, lanes=frames sequence kernel, phase-3 kernel.
hipError_t launch_decompress(const ZhDecArgs &a, u32 nitems, hipStream_t stream);
hipError_t init_kernels();
u32 lz_lds_bytes();
u32 entropy_lds_bytes();
// K1 hash tables of a dictionary's content tail, built once per dictionary (zh_lz.hip):
// out = 2^15 u16, tmp32 = 2^15 u32 scratch; P = the tail length covered (0: none)
hipError_t lz_dict_tables(const u8 *content, size_t cn, u16 *out, u32 *tmp32, u32 &P, hipStream_t stream);
hipError_t lz_deep_dict_tables(const u8 *content, size_t cn, u8 *stg, u32 *dprev, u32 *dhead, u32 &P, u32 &split, hipStream_t stream);
hipError_t launch_compress(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 window_log, u32 cfg_block_size, u64 *d_item_size,
                           u32 *d_item_status, u32 *d_blk_size, const ZhItemDesc *d_items, u32 nitems, bool gather, bool checksum, int level,
                           hipStream_t stream);
void profile_enable(bool on);
int profile_collect(double *totals);
hipError_t launch_plan(const void *const *d_in_ptrs, const size_t *d_in_sizes, u32 nitems, u32 bpi, void *const *d_out_ptrs, u64 out_cap,
                       u8 *staging, ZhBlockDesc *d_descs, ZhItemDesc *d_items, u64 *d_item_size, u32 *d_item_status, u32 extra_flags,
                       const u8 *dict, u32 dict_n, u32 dict_id, u32 hist, hipStream_t stream);
}  // namespace zh
