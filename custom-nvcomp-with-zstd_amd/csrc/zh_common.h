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
  const u8 *pre;     // ZH_F_DICT first block: dictionary content tail staged before the block
  u32 pre_n;         // its length (pre_n + n <= ZH_BLOCK_MAX; ZH_F_DEEP: pre_n <= ZH_DEEP_PRE), 0 without one
  u32 dict_id;       // Dictionary_ID written to the frame header (0: none)
};

enum : u32 {
  ZH_F_FIRST = 1u,   // first block of its frame: writes the frame header, starts with reps {1,4,8}
  ZH_F_LAST = 2u,    // last block of its frame: Last_Block bit
  ZH_F_DIRECT = 4u,  // single-block frame written straight into the item's output
  ZH_F_CHECKSUM = 8u,  // frame carries a content checksum (first block: FHD bit; zh_checksum_kernel appends it)
  ZH_F_DICT = 16u,     // dictionary frame: Dictionary_ID in the header, repcodes start unknown
  ZH_F_DEEP = 32u,     // level >= ZH_DEEP_LEVEL (zh_lz_deep.hip): a dictionary frame's first block is staged
                       // behind the last ZH_DEEP_PRE content bytes
};

// Per-block workspace carved from the caller's temp buffer.
//   seq   : ZH_SEQ_CAP u64 records (K1: walk literals before the match | len << 17 | catch-up << 24 |
//           off << 36, the literal run being walk literals - catch-up; K2 rewrites them in place)
//   lits  : ZH_BLOCK_MAX literal bytes; once the literals section is written, the
//           sequences' FSE states and codes in encoding order in the segment-interleaved
//           layout of the chain kernel (below): states u16 [0, 128 L), codes u8 [128 L, 192 L),
//           L = zh_k3_seglen(nbSeq)
//   meta  : u32[4] = {nseq, nlit, rle, 0}
#define ZH_SEQ_CAP 13120u
#define ZH_SEQ_BYTES (ZH_SEQ_CAP * 8u)
// FSE chain segments (zh_entropy.hip K3): each of the three tables' chains is cut into
// ZH_K3_SEGS segments of L steps (L a multiple of ZH_K3_RUN); lane t * ZH_K3_SEGS + g of the
// chain wave runs segment g of table t.  Step e of table t is element
//   ((r / RUN) * ZH_K3_SLOTS + ZH_K3_SLOT(t, g)) * RUN + r % RUN,   g = e / L, r = e % L
// of the state (u16) and code (u8) arrays, RUN = ZH_K3_RUN: RUN consecutive steps of a
// segment are contiguous (the packing kernel's 64-step chunks are whole lines) and the 63
// segments' runs are adjacent.
// ZH_K3_W waves run one block's chains (21 segments per table and wave): the batch row of a
// layout holds ZH_K3_SLOTS = 64 ZH_K3_W segment slots.
#ifndef ZH_K3_W
#define ZH_K3_W 1u
#endif
#define ZH_K3_SEGS (21u * ZH_K3_W)
#define ZH_K3_SLOTS (64u * ZH_K3_W)
#define ZH_K3_RUN 16u
// Slot of (table t, segment g) in a batch row.  Segment-major (3 g + t, the default): a step's LL,
// OF and ML runs are adjacent, so the packing kernel's loads of one segment's 16 steps touch one or
// two 128-B lines instead of three (table-major t * SEGS + g: three lines, each used for 32 B)
#ifndef ZH_K3_SEGMAJOR
#define ZH_K3_SEGMAJOR 1
#endif
#if ZH_K3_SEGMAJOR
#define ZH_K3_SLOT(t, g) (3u * (g) + (t))
#define ZH_K3_TSTRIDE ZH_K3_RUN  // elements between a step's LL, OF and ML entries
#else
#define ZH_K3_SLOT(t, g) ((t) * ZH_K3_SEGS + (g))
#define ZH_K3_TSTRIDE (ZH_K3_SEGS * ZH_K3_RUN)
#endif
#define ZH_K3_SEGLEN(nbseq) ((((nbseq) + ZH_K3_SEGS - 1u) / ZH_K3_SEGS + ZH_K3_RUN - 1u) & ~(ZH_K3_RUN - 1u))
#define ZH_K3_CODES(L) (2u * ZH_K3_SLOTS * (L))  // byte offset of the codes (after the u16 states)
#define ZH_K3_BYTES(nbseq) (3u * ZH_K3_SLOTS * ZH_K3_SEGLEN(nbseq))
#define ZH_LIT_BYTES (ZH_K3_BYTES(ZH_SEQ_CAP) > (u32)ZH_BLOCK_MAX ? ZH_K3_BYTES(ZH_SEQ_CAP) : (u32)ZH_BLOCK_MAX)
static_assert(3u * ZH_K3_SEGS <= ZH_K3_SLOTS, "one lane per (table, segment)");
#define ZH_META_BYTES 256u  // u32[4] counters + u32[60] diagnostic stamps (-DZH_STAMPS builds)
//   fse   : hand-off from the entropy kernel to the FSE chain and packing kernels:
//           the block's three FSE tables (state tables + symbol transforms, ZH_FSE_TAB_BYTES)
//           then u32 fields at ZH_FSE_FIELDS (ZH_FF_* indices)
#define ZH_FSE_BYTES 4096u
#define ZH_FSE_TAB_BYTES 3528u  // stLL u16[512] | stOF u16[256] | stML u16[512] | symLL[36] | symOF[32] | symML[53] (8 B each)
#define ZH_FSE_FIELDS 3840u
#define ZH_WS_BLOCK_BYTES (ZH_SEQ_BYTES + ZH_LIT_BYTES + ZH_META_BYTES + ZH_FSE_BYTES)
enum : u32 {
  ZH_FT_STLL = 0, ZH_FT_STOF = 1024, ZH_FT_STML = 1536, ZH_FT_SYLL = 2560, ZH_FT_SYOF = 2848, ZH_FT_SYML = 3104,  // byte offsets
  ZH_FF_NEED = 0,   // 1: the sequence bitstream is left to the chain + packing kernels
  ZH_FF_NBSEQ = 1,  // sequences (after merging)
  ZH_FF_OP = 2,     // output offset where the sequence bitstream starts
  ZH_FF_BLK = 3,    // output offset of the block header
  ZH_FF_LOGS = 4,   // logLL | logOF << 8 | logML << 16
  ZH_FF_SLL = 5, ZH_FF_SOF = 6, ZH_FF_SML = 7,  // final FSE states (chain kernel)
};

// Deep matcher (zh_lz_deep.hip) scratch slot of one persistent workgroup: staged bytes (prefix +
// block, zero padded) | u32 prev[2 x 64 Ki] | u32 off/len per block position | u16 link distances
// (when LDS cannot hold them).  Slots per call = min(blocks, ZH_DEEP_SLOTS_MAX): the grid.
#define ZH_DEEP_STG_BYTES (2u * ZH_BLOCK_MAX + 256u)
#define ZH_DEEP_SLOT_BYTES ((size_t)ZH_DEEP_STG_BYTES + 4u * 2u * ZH_BLOCK_MAX + 4u * ZH_BLOCK_MAX + 2u * 2u * ZH_BLOCK_MAX)
#define ZH_DEEP_SLOTS_MAX 256u
// K1's per-block meta word 2: 0 normal (records + literal area), 1 RLE block, ZH_META_K1HIST: no
// sequences, the literals are the block's source bytes (16-B aligned) and K1 left the literal
// histogram as ZH_K1_HIST_WAVES 256-bin u32 sub-histograms at lits + ZH_K1_HIST_OFF
#define ZH_META_K1HIST 2u
#define ZH_K1_HIST_OFF 65536u
#define ZH_K1_HIST_WAVES 16u
static_assert(ZH_K1_HIST_OFF + ZH_K1_HIST_WAVES * 1024u <= ZH_LIT_BYTES, "K1 sub-histograms fit the literal area");

struct ZhWorkspace {
  u8 *base;          // nblocks * ZH_WS_BLOCK_BYTES
  u32 *ctr;          // K1's block counter (persistent workgroups take the next block from it)
  // K1 hash tables of the batch dictionary's content, precomputed once per dictionary
  // (zh::lz_dict_tables; null: none): 2 x 2^14 u16 entries = tail position + 1 over the last
  // dtab_P content bytes, positions [0, dtab_P - ZH_DTAB_MARGIN) inserted
  const u16 *dtab;
  u32 dtab_P;
  // The deep matcher's chains of the batch dictionary (levels >= ZH_DEEP_LEVEL; null: none):
  // links of staged positions [0, dd_split) of a first block with dd_pre staged content bytes, and
  // the head table after them (zh_lz_deep.hip zh_deep_dict_kernel)
  const u32 *dd_prev;
  const u32 *dd_head;
  u32 dd_pre, dd_split;
  // The deep matcher's per-workgroup scratch slots (ZH_DEEP_SLOT_BYTES each; levels >=
  // ZH_DEEP_LEVEL only): part of the caller's workspace, so independent calls never share them
  u8 *deep_slots;
  u32 deep_nslots;
  __device__ u64 *seq(u32 b) const { return (u64 *)(base + (size_t)b * ZH_WS_BLOCK_BYTES); }
  __device__ u8 *lits(u32 b) const { return base + (size_t)b * ZH_WS_BLOCK_BYTES + ZH_SEQ_BYTES; }
  __device__ u32 *meta(u32 b) const { return (u32 *)(base + (size_t)b * ZH_WS_BLOCK_BYTES + ZH_SEQ_BYTES + ZH_LIT_BYTES); }
  __device__ u32 *dbg(u32 b) const { return meta(b) + 4; }
  __device__ u8 *fse(u32 b) const { return base + (size_t)b * ZH_WS_BLOCK_BYTES + ZH_SEQ_BYTES + ZH_LIT_BYTES + ZH_META_BYTES; }
  __device__ u32 *fsef(u32 b) const { return (u32 *)(fse(b) + ZH_FSE_FIELDS); }
};

#define ZH_DTAB_MARGIN 256u  // tail positions a block inserts itself (>= one inserter batch)

// Element index of step e of table t in the chain layout (see ZH_K3_SEGS); m = zh_k3_magic(L)
// gives e / L as umulhi(e << 8, m) exactly for e < 2^14, L <= 1024
__host__ __device__ __forceinline__ u32 zh_k3_magic(u32 L) { return ((1u << 24) + L - 1u) / L; }
__device__ __forceinline__ u32 zh_k3_index(u32 e, u32 t, u32 L, u32 m) {
  u32 const g = __umulhi(e << 8, m), r = e - g * L;
  return ((r / ZH_K3_RUN) * ZH_K3_SLOTS + ZH_K3_SLOT(t, g)) * ZH_K3_RUN + (r & (ZH_K3_RUN - 1u));
}

// Status codes written per item (values of cuda_zstd::Status).
enum : u32 { ZH_ST_OK = 0, ZH_ST_INVALID = 2, ZH_ST_TOO_SMALL = 7 };

// ---------------- wave64 cross-lane helpers on DPP (VALU only, no LDS round trip) ----------------
// Inclusive prefix with row_shr 1/2/4/8 inside 16-lane rows, then row_bcast:15 / row_bcast:31
// across rows (GFX9 DPP); a __shfl_up scan is 6 dependent ds_bpermutes.  Lanes whose DPP
// source is outside the row read 0 (the identity of add and unsigned max).
#define ZH_DPP(v, ctrl, rmask) ((u32)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), (rmask), 0xf, false))
__device__ __forceinline__ u32 wave_scan_incl(u32 v) {
  v += ZH_DPP(v, 0x111, 0xf);  // row_shr:1
  v += ZH_DPP(v, 0x112, 0xf);  // row_shr:2
  v += ZH_DPP(v, 0x114, 0xf);  // row_shr:4
  v += ZH_DPP(v, 0x118, 0xf);  // row_shr:8
  v += ZH_DPP(v, 0x142, 0xa);  // row_bcast:15 into rows 1, 3
  v += ZH_DPP(v, 0x143, 0xc);  // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ u32 wave_scan_max_incl(u32 v) {
  v = max(v, ZH_DPP(v, 0x111, 0xf));
  v = max(v, ZH_DPP(v, 0x112, 0xf));
  v = max(v, ZH_DPP(v, 0x114, 0xf));
  v = max(v, ZH_DPP(v, 0x118, 0xf));
  v = max(v, ZH_DPP(v, 0x142, 0xa));
  v = max(v, ZH_DPP(v, 0x143, 0xc));
  return v;
}
// value of lane - 1 (lane 0 reads 0): DPP wave_shr:1
__device__ __forceinline__ u32 wave_shr1(u32 v) { return ZH_DPP(v, 0x138, 0xf); }
// value of lane + 1 (lane 63 reads 0): DPP wave_shl:1
__device__ __forceinline__ u32 wave_shl1(u32 v) { return ZH_DPP(v, 0x130, 0xf); }
// v of a wave-uniform lane (v_readlane into an SGPR)
__device__ __forceinline__ u32 lane_value(u32 v, u32 uniform_lane) { return (u32)__builtin_amdgcn_readlane((int)v, (int)uniform_lane); }
