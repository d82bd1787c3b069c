// zh_common.h — device-side types shared by the gfx950 compression kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zstd_hip_params.h"

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int16_t s16;
typedef int32_t s32;

// One device block (<= ZH_BLOCK_MAX input bytes) = one K1 workgroup = one K2 wave.
struct ZhBlockDesc {
  const u8 *src;     // first input byte of this block
  u8 *dst;           // where this block's output goes (item output if DIRECT, else staging slot)
  u64 frame_size;    // content size of the frame this block belongs to
  u32 n;             // input bytes (0 = inactive slot)
  u32 item;          // batch item index
  u32 dst_cap;       // bytes available at dst
  u32 flags;         // ZH_F_* below
};

enum : u32 {
  ZH_F_FIRST = 1u,   // first block of its frame: writes the frame header, starts with reps {1,4,8}
  ZH_F_LAST = 2u,    // last block of its frame: Last_Block bit
  ZH_F_DIRECT = 4u,  // single-block frame written straight into the item's output
};

// Per-block workspace carved from the caller's temp buffer.
//   seq   : ZH_SEQ_CAP u64 records (K1: cumLit | ml<<17 | off<<25; K2 rewrites in place)
//   lits  : ZH_BLOCK_MAX literal bytes
//   meta  : u32[4] = {nseq, nlit, rle, 0}
#define ZH_SEQ_CAP 13120u
#define ZH_SEQ_BYTES (ZH_SEQ_CAP * 8u)
#define ZH_LIT_BYTES ((u32)ZH_BLOCK_MAX)
#define ZH_META_BYTES 256u  // u32[4] counters + u32[60] diagnostic stamps (-DZH_STAMPS builds)
#define ZH_WS_BLOCK_BYTES (ZH_SEQ_BYTES + ZH_LIT_BYTES + ZH_META_BYTES)

struct ZhWorkspace {
  u8 *base;          // nblocks * ZH_WS_BLOCK_BYTES
  __device__ u64 *seq(u32 b) const { return (u64 *)(base + (size_t)b * ZH_WS_BLOCK_BYTES); }
  __device__ u8 *lits(u32 b) const { return base + (size_t)b * ZH_WS_BLOCK_BYTES + ZH_SEQ_BYTES; }
  __device__ u32 *meta(u32 b) const { return (u32 *)(base + (size_t)b * ZH_WS_BLOCK_BYTES + ZH_SEQ_BYTES + ZH_LIT_BYTES); }
  __device__ u32 *dbg(u32 b) const { return meta(b) + 4; }
};

// Status codes written per item (values of cuda_zstd::Status).
enum : u32 { ZH_ST_OK = 0, ZH_ST_INVALID = 2, ZH_ST_TOO_SMALL = 7 };
