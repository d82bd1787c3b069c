// zh_lz.hip — K1: LZ77 match finding + parse for one <=64 KiB block per workgroup.
//
// Replaces the reference's find_matches_kernel / greedy_parse_kernel /
// build_sequences_gpu_kernel<<<1,1>>> (src/lz77_parallel.cu:26-70, 177-268)
// and the literal gather kernels (src/cuda_zstd_manager.cu:602-723).
// Output is identical to oracle/zstd_oracle.c orc_lz_parse (tile-lagged hash
// insertion, longer of long/short candidate, greedy + lazy-1 parse).
//
// One workgroup of 1024 threads (16 wave64, one workgroup per CU) per block,
// everything in LDS:
//   in[]   the block, staged once with 16-B loads (64 KiB)
//   TL/TS  2 x 2^14 u16 hash tables, entry = position + 1 (0 = empty)
//   cinfo  one 4096-position window: candidates -> match info (off<<8|len) in place
//   exb    per-position exits of the 64-position parse segments
// Wave roles (wave specialisation, all synchronised with workgroup barriers):
//   waves 14, 15  inserters: one wave per hash table walks the next window's
//                 tiles of ZH_TILE positions.  A single wave needs no barrier
//                 between a tile's lookups and its inserts because LDS executes
//                 one wave's operations in order; lanes of one store that hit the
//                 same slot are resolved to the latest position by a read-back.
//                 Candidates are held in registers and dumped into cinfo at the
//                 window switch, so the next window's insertion overlaps this
//                 window's lengths.
//   waves 0..13   match lengths of the window, 5 positions per thread, with
//                 same-offset chains resolved in registers.
//   waves 0..13   the serial greedy/lazy-1 parse, lanes = positions: pointer
//                 doubling gives every position's exit from its 64-position
//                 segment, wave 0 finds the segment entries as a Jacobi fixed
//                 point, binary lifting marks the visited positions, and scans of
//                 the marks place literals and sequence records.
#include "zh_common.h"

#include <algorithm>

#ifdef ZH_STAMPS
__device__ u32 g_fixups;  // diagnostic: inserter read-back fix-up rounds (all blocks)
extern "C" __global__ void zh_read_fixups(u32 *out) { *out = g_fixups; g_fixups = 0; }
extern "C" u32 zh_fixups_host() {
  u32 *d = nullptr, h = 0;
  if (hipMalloc(&d, 4) != hipSuccess) return ~0u;
  hipLaunchKernelGGL(zh_read_fixups, dim3(1), dim3(1), 0, 0, d);
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return h;
}
#endif
namespace {

constexpr u32 K1_THREADS = 1024;
constexpr u32 NPSEG = ZH_WINDOW / 64;       // parse segments per window (64 positions = one wave)
constexpr u32 INS_TID = 896;                // first inserter thread (waves 14, 15)
#ifndef ZH_K1_SB
#define ZH_K1_SB 5
#endif
constexpr u32 SB = ZH_K1_SB;                // positions per thread in the length phase
constexpr u32 NB = (ZH_WINDOW + SB - 1) / SB;  // length-phase threads (thread NB takes position `we`)
constexpr u32 TILES = ZH_WINDOW / ZH_TILE;  // 16 tiles per window
constexpr u32 TPL = ZH_TILE / 64;           // positions per inserter lane per tile
constexpr u32 NCR = TILES * TPL / 2;        // candidate registers per inserter lane (u16 pairs)
static_assert(NPSEG == 64 && NB + 1 <= INS_TID, "thread roles");
static_assert(ZH_WINDOW % ZH_TILE == 0 && ZH_TILE % 64 == 0 && TILES * TPL % 2 == 0, "tiles tile windows");

constexpr u32 HL_SIZE = 1u << ZH_HASH_LOG_LONG;
constexpr u32 HS_SIZE = 1u << ZH_HASH_LOG_SHORT;
constexpr u32 T_PAD = 8;                    // + a junk slot (index HL/HS_SIZE) for lanes past lim
constexpr u32 OFF_IN = 0;
constexpr u32 OFF_TL = OFF_IN + ZH_BLOCK_MAX + 16;
constexpr u32 OFF_TS = OFF_TL + 2 * (HL_SIZE + T_PAD);
constexpr u32 OFF_CI = OFF_TS + 2 * (HS_SIZE + T_PAD);
constexpr u32 CI_WORDS = ZH_WINDOW + 8;  // + the lookahead slot of position `we`
__device__ __forceinline__ u32 cidx(u32 i) { return i; }
constexpr u32 OFF_EXB = OFF_CI + 4 * CI_WORDS;      // u8 per position: its parse segment exit (relative)
constexpr u32 OFF_SEG = OFF_EXB + ZH_WINDOW + 16;   // parse segment entries + the window exit (exb: + a junk byte)
constexpr u32 NWW = INS_TID / 64;                   // worker waves
constexpr u32 PR = (ZH_WINDOW + INS_TID - 1) / INS_TID;  // lane-per-position rounds over a window
constexpr u32 WP_OFF = 80, WP_TOT = 160;
static_assert(PR * NWW <= WP_OFF, "emission scan slots");
constexpr u32 OFF_WP = OFF_SEG + 4 * (NPSEG + 4);     // emission scan: wave counts, offsets, total
constexpr u32 HB_STRIDE = 65;                        // per worker wave: 64 head slots + a junk slot
constexpr u32 OFF_HB = OFF_WP + 4 * 164;
constexpr u32 OFF_MISC = OFF_HB + 4 * HB_STRIDE * (INS_TID / 64);  // [0..3] scan partials, [4..6] barrier-or words
constexpr u32 K1_LDS = OFF_MISC + 4 * 16;
constexpr u32 MISC_ARR = 12;  // misc[12]: worker-wave barrier arrivals (cumulative)
static_assert(K1_LDS <= 163840 - 256, "K1 LDS budget");
static_assert(OFF_TL % 16 == 0 && OFF_CI % 16 == 0 && OFF_SEG % 16 == 0, "alignment");

__device__ __forceinline__ u32 hash_long(u64 v) {
  return (u32)((v * ZH_PRIME_LONG) >> (64 - ZH_HASH_LOG_LONG));
}
__device__ __forceinline__ u32 hash_short(u64 v) {
  return (u32)(((v << 24) * ZH_PRIME_SHORT) >> (64 - ZH_HASH_LOG_SHORT));
}

// 8 bytes at p from LDS as (lo, hi): three aligned dwords + v_alignbyte
__device__ __forceinline__ void ld64u(const u32 *in32, u32 p, u32 &lo, u32 &hi) {
  u32 const w = p >> 2, sh = p & 3;
  u32 const w0 = in32[w], w1 = in32[w + 1], w2 = in32[w + 2];
  lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
}

// common prefix (0..8) of the 8 bytes (olo, ohi) with in[b..b+8)
__device__ __forceinline__ u32 prefix8(const u32 *in32, u32 b, u32 olo, u32 ohi) {
  u32 blo, bhi;
  ld64u(in32, b, blo, bhi);
  u32 const x = olo ^ blo, y = ohi ^ bhi;
  // branch-free (v_cndmask): divergent branches cost exec-mask work on the CU's
  // shared scalar unit
  u32 const cx = __builtin_ctzg(x, 32), cy = __builtin_ctzg(y, 32);
  return (x ? cx : 32u + cy) >> 3;
}

// Extension of a chain head (p, q) whose first 8 bytes match: E = min(common prefix,
// EXT_SPAN, n - p).  EXT_SPAN = cap 64 + SB - 1, so every later position of the
// thread's run continuing the same offset gets its exact capped length as
// min(E - i, cap) without touching the input again.  Bytes 8.. are compared as
// dwords with every load issued up front; bytes past the block end read LDS
// padding/tables and are cut off by n - p.
constexpr u32 EXT_SPAN = 8 + (ZH_MAX_MATCH + SB - 1 - 8 + 3) / 4 * 4;  // (>= cap + SB - 1, whole dwords)
static_assert((EXT_SPAN - 8) % 4 == 0, "dword span");
__device__ __forceinline__ u32 ext_head(const u32 *in32, u32 p, u32 q, u32 n) {
  constexpr u32 NW = (EXT_SPAN - 8) / 4;  // dwords compared
  constexpr u32 H = (NW + 1) / 2;         // in two halves (bounded register use)
  u32 const pa = p + 8, qa = q + 8;
  u32 const wp = pa >> 2, sp = pa & 3, wq = qa >> 2, sq = qa & 3;
  u32 l = EXT_SPAN;
#pragma unroll
  for (u32 h0 = 0; h0 < NW; h0 += H) {
    // the second half only when some lane's match reaches past the first one
    if (h0 && !__ballot(l == EXT_SPAN)) break;
    u32 A[H + 1], B[H + 1];
#pragma unroll
    for (u32 k = 0; k <= H; k++) { A[k] = in32[wp + h0 + k]; B[k] = in32[wq + h0 + k]; }
    u32 lh = EXT_SPAN;
#pragma unroll
    for (int k = (int)H - 1; k >= 0; k--) {
      if (h0 + (u32)k >= NW) continue;
      u32 const x = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sp) ^ __builtin_amdgcn_alignbyte(B[k + 1], B[k], sq);
      if (x) lh = 8 + 4 * (h0 + (u32)k) + (__builtin_ctz(x) >> 3);
    }
    l = l == EXT_SPAN ? lh : l;
  }
  return min(l, n - p);
}

template <bool LONG>
__device__ __forceinline__ u32 hash_of(u32 lo, u32 hi) {
  u64 const v = ((u64)hi << 32) | lo;
  return LONG ? hash_long(v) : hash_short(v);
}

// Inserter wave: the tiles of window [wsb, we) against one table (u16 entries = position
// + 1).  Lane l handles positions tb + l + 64k of each tile; all lookups of a tile are
// issued before its stores and after the previous tile's stores (program order = LDS
// order within a wave).  Stores of later k carry later positions and land later; lanes
// of ONE store that hit the same slot leave one of their values, so every lane reads its
// slot back and lanes that find an earlier position rewrite theirs until none does: the
// slot ends with the latest position, as in the oracle's serial loop.  Candidates
// (position + 1, 0 = none) go to creg as u16 pairs.
// Repair path of insert_window for a batch in which some lane of a ds_write_b16 lost its
// slot to a LOWER position of the same store (never observed on gfx950, where the highest
// lane of a store wins, but kept so the table semantics never depend on it).  The batch's
// lookups of tile b >= 1 were issued after the earlier tiles' unrepaired stores: the correct
// value is the max of that and every earlier-tile position of the batch hashing to the same
// slot.  Then every lost store is rewritten while its slot holds an older position (slots only
// ever move forward, so later tiles' stores are never undone).
template <bool LONG, u32 BT>
__device__ __forceinline__ void insert_repair(u16 *T, u32 tb0, u32 lane, const u32 (&h)[BT][TPL], u32 (&e)[BT][TPL]) {
  constexpr u32 JUNK = LONG ? HL_SIZE : HS_SIZE;
  // (compile-time slot loops unrolled, the lane loop kept rolled: this code never runs on
  // gfx950 and must not bloat the inserter's instruction stream)
#pragma unroll
  for (u32 b = 1; b < BT; b++)
#pragma unroll
    for (u32 bb = 0; bb < b; bb++)
#pragma unroll
      for (u32 kk = 0; kk < TPL; kk++)
#pragma unroll 1
        for (u32 j = 0; j < 64; j++) {
          u32 const hj = __builtin_amdgcn_readlane(h[bb][kk], j);
          u32 const pj = tb0 + bb * ZH_TILE + 64 * kk + j + 1;
#pragma unroll
          for (u32 k = 0; k < TPL; k++)
            if (hj != JUNK && h[b][k] == hj && e[b][k] < pj) e[b][k] = pj;
        }
  for (;;) {
    bool need = false;
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++) {
        u32 const v = tb0 + b * ZH_TILE + 64 * k + lane + 1;
        if (h[b][k] != JUNK && (u32)T[h[b][k]] < v) {
          T[h[b][k]] = (u16)v;
          need = true;
        }
      }
    if (!__ballot(need)) break;
  }
}

// Inserter wave: the tiles of window [wsb, we) against one table (u16 entries = position
// + 1).  Lane l handles positions tb + l + 64k of each tile; a tile's lookups are issued
// before its stores and after the previous tile's stores (program order = LDS order within a
// wave).  Stores of later k / later tiles carry later positions and land later; lanes of ONE
// store that hit the same slot leave one of their values (on gfx950 the highest lane's, i.e.
// the latest position, as in the oracle's serial loop), which a read-back of every lane's
// slot verifies (insert_repair otherwise).  BT tiles are issued per LDS round trip together
// with the next batch's input dwords and the workers' arrival counter.  Candidates
// (position + 1, 0 = none) go to creg as u16 pairs.
template <bool LONG, typename Hook>
__device__ __forceinline__ void insert_window(const u32 *in32, u16 *T, u32 wsb, u32 we, u32 lim, u32 lane, u32 (&creg)[NCR], u32 &cwe,
                                              const u32 *arrivals, Hook &&between_tiles, u32 pmin = 0) {
  // positions below pmin are already in T (a dictionary's precomputed tables): treated like
  // positions past lim (the junk slot, no candidate)
  constexpr u32 JUNK = LONG ? HL_SIZE : HS_SIZE;
  constexpr u32 BT = 2;  // tiles per LDS round trip
  static_assert(TILES % BT == 0, "batches tile windows");
  u32 wv[BT][TPL][3];
  auto load_in = [&](u32 tb0, u32 lim_t) {
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++) {
        u32 const q = min(tb0 + b * ZH_TILE + 64 * k + lane, lim_t) >> 2;
        wv[b][k][0] = in32[q];
        wv[b][k][1] = in32[q + 1];
        wv[b][k][2] = in32[q + 2];
      }
  };
  load_in(wsb, lim);
#pragma unroll
  for (u32 t0 = 0; t0 < TILES; t0 += BT) {
    // opaque per-batch copy of lim: keeps the compiler from hoisting every tile's
    // bounds checks (64 masks) to the top of the unrolled loop
    u32 lim_t;
    __asm__ volatile("v_mov_b32 %0, %1" : "=v"(lim_t) : "v"(lim));
    u32 const tb0 = wsb + t0 * ZH_TILE;
    u32 h[BT][TPL], e[BT][TPL], r[BT][TPL];
#pragma unroll
    for (u32 b = 0; b < BT; b++) {
      u32 const tb = tb0 + b * ZH_TILE;
#pragma unroll
      for (u32 k = 0; k < TPL; k++) {
        u32 const p = tb + 64 * k + lane, sh = min(p, lim_t) & 3u;
        u32 const lo = __builtin_amdgcn_alignbyte(wv[b][k][1], wv[b][k][0], sh), hi = __builtin_amdgcn_alignbyte(wv[b][k][2], wv[b][k][1], sh);
        u32 const hh = hash_of<LONG>(lo, hi);
        e[b][k] = T[hh];
        h[b][k] = (p < lim_t && p >= pmin) ? hh : JUNK;
      }
#pragma unroll
      for (u32 k = 0; k < TPL; k++) T[h[b][k]] = (u16)(tb + 64 * k + lane + 1);
#pragma unroll
      for (u32 k = 0; k < TPL; k++) r[b][k] = T[h[b][k]];
    }
    if (t0 + BT < TILES) load_in(tb0 + BT * ZH_TILE, lim_t);
    u32 const arr = __atomic_load_n(arrivals, __ATOMIC_RELAXED);
    bool lost = false;
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++) lost |= h[b][k] != JUNK && r[b][k] < tb0 + b * ZH_TILE + 64 * k + lane + 1;
    if (__ballot(lost)) {
#ifdef ZH_STAMPS
      if (lane == 0) atomicAdd(&g_fixups, 1u);
#endif
      insert_repair<LONG, BT>(T, tb0, lane, h, e);
    }
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k += 2) {
        u32 const c0 = h[b][k] != JUNK ? e[b][k] : 0u, c1 = h[b][k + 1] != JUNK ? e[b][k + 1] : 0u;
        u32 const ri = ((t0 + b) * TPL + k) / 2;
        creg[ri] = c0 | (c1 << 16);
        // materialise this batch's candidates now (otherwise the compiler sinks their
        // computation to the dump and keeps every tile's temporaries alive)
        __asm__ volatile("" : "+v"(creg[ri]) :: "memory");
      }
    between_tiles(arr);
  }
  // the next window's first position (lazy rule at this window's end): looked up
  // after all of this window's tiles, before any of the next window's
  cwe = 0;
  if (lane < 2 && we + lane < lim) {  // (lane 1: we + 1, the second lookahead of LAZY2)
    u32 lo, hi;
    ld64u(in32, we + lane, lo, hi);
    cwe = T[hash_of<LONG>(lo, hi)];
  }
  __asm__ volatile("" ::: "memory");
}

// Positions [s, e) into T in order (the latest position wins every slot), lookups discarded:
// the few dictionary positions between a precomputed table's end and the first tile a block
// processes.  Lanes of one store that hit the same slot leave one value; the lower positions
// that won rewrite theirs until every slot holds its latest.
template <bool LONG>
__device__ __forceinline__ void insert_span(const u32 *in32, u16 *T, u32 s, u32 e, u32 lane) {
  constexpr u32 JUNK = LONG ? HL_SIZE : HS_SIZE;
  for (u32 r = s; r < e; r += 64) {
    u32 const p = r + lane;
    bool const v = p < e;
    u32 lo, hi;
    ld64u(in32, v ? p : s, lo, hi);
    u32 const h = v ? hash_of<LONG>(lo, hi) : JUNK;
    T[h] = (u16)(p + 1);
    for (;;) {
      bool const lost = v && (u32)T[h] < p + 1;
      if (!__ballot(lost)) break;
      if (lost) T[h] = (u16)(p + 1);
    }
  }
  __asm__ volatile("" ::: "memory");
}

// Dump an inserter's candidates into its half of the cinfo words (LONG: low half).
template <bool LONG>
__device__ __forceinline__ void dump_window(u8 *ci8, u32 lane_, const u32 (&creg)[NCR], u32 cwe) {
  // opaque lane copy: stops the 64 addresses from being hoisted out of the window loop
  u32 lane;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane_));
#pragma unroll
  for (u32 t = 0; t < TILES; t++) {
#pragma unroll
    for (u32 k = 0; k < TPL; k++) {
      u32 const i = t * ZH_TILE + 64 * k + lane, j = t * TPL + k;
      u16 const v = (u16)(creg[j / 2] >> (16 * (j & 1)));
      *(u16 *)(ci8 + 4 * cidx(i) + (LONG ? 0 : 2)) = v;
    }
  }
  if (lane < 2) *(u16 *)(ci8 + 4 * cidx(ZH_WINDOW + lane) + (LONG ? 0 : 2)) = (u16)cwe;
}

// Lane-per-position parse steps for window index i (a wave's 64 lanes = one parse
// segment of 64 positions): X[k] = position reached after 2^k parse steps from i, for
// k < 6, and X[6] = the segment exit, relative to the segment start (values >= the
// segment length mean "left the segment").  Returns the match info of i if the parse
// takes a match there, else 0.
// v from lane `src` (< 64) of the wave: ds_bpermute on a byte address, no lane-base math
__device__ __forceinline__ u32 bperm(u32 v, u32 src) { return (u32)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v); }

// (wave_scan_incl, wave_shr1: DPP helpers in zh_common.h)

// Parse cost of a match: libzstd's lazy "gain" (4 per byte, minus the offset's bit length)
__device__ __forceinline__ int match_gain(u32 inf) {
  return inf ? 4 * (int)(inf & 255u) - (31 - (int)__builtin_clz((inf >> 8) + 1u)) : -1000;
}

// LAZY2 (levels >= 9): a match at i is deferred when the match at i+1 gains
// more than 4 over it or the one at i+2 more than 7 (libzstd ZSTD_compressBlock_lazy_generic,
// depth 2); otherwise (levels < 9) when the match at i+1 is longer.  la / la2: the match info
// of the next window's first two positions.
template <bool LAZY2>
__device__ __forceinline__ u32 parse_steps(const u32 *ci, u32 i, u32 wn, u32 la, u32 la2, u32 lane, u32 (&X)[7]) {
  u32 const sb = i & ~63u;
  u32 const slen = wn > sb ? min(64u, wn - sb) : 0u;
  // unconditional (clamped) loads, then selects: no exec-mask branches
  u32 const r0 = ci[min(i, (u32)ZH_WINDOW)], r1 = ci[min(i + 1, (u32)ZH_WINDOW)];
  u32 const inf = i < wn ? r0 : 0u;
  u32 const inf1 = i + 1 < wn ? r1 : la;
  u32 const l = inf & 255u;
  bool tk;
  if (LAZY2) {
    u32 const r2 = ci[min(i + 2, (u32)ZH_WINDOW + 1)];
    u32 const inf2 = i + 2 < wn ? r2 : (i + 2 == wn ? la : la2);
    int const g0 = match_gain(inf);
    tk = l != 0 && match_gain(inf1) <= g0 + 4 && match_gain(inf2) <= g0 + 7;
  } else {
    tk = l != 0 && (inf1 & 255u) <= l;
  }
  u32 x = lane + (tk ? l : 1u);
  if (__ballot(tk)) {
#pragma unroll
    for (u32 k = 0; k < 6; k++) {
      X[k] = x;
      u32 const y = bperm(x, min(x, 63u));
      x = x < slen ? y : x;
    }
  } else {  // all literals in this segment: 2^k steps are 2^k positions
#pragma unroll
    for (u32 k = 0; k < 6; k++) {
      X[k] = x;
      x = x < slen ? min(x + (1u << k), slen) : x;
    }
  }
  X[6] = x;
  return tk ? inf : 0u;
}

// Inserter wave main loop.  It mirrors the workers' barrier sequence window by window
// (P, R, X, J, E1, E2) but fills the slack: between two tiles it takes the next
// barrier only once all 14 worker waves have arrived there (an LDS arrival counter),
// so the next window's insertion spreads over the whole window step.
constexpr u32 WIN_BARRIERS = 5;  // R, X, J, E1, E2
template <bool LONG>
__device__ __forceinline__ void inserter_loop(const u32 *in32, u16 *T, u8 *ci8, u32 *misc_, u32 n, u32 lim, u32 lane, u32 *dbg, u32 wstart,
                                              u32 pmin, u32 span_s, u32 span_e) {
  u32 creg[NCR];
  u32 cwe = 0;
  if (span_s < span_e) insert_span<LONG>(in32, T, span_s, span_e, lane);
  insert_window<LONG>(in32, T, wstart, min(wstart + (u32)ZH_WINDOW, n), lim, lane, creg, cwe, &misc_[MISC_ARR], [](u32) {}, pmin);
#ifdef ZH_STAMPS
  u32 st_ins = 0;
#endif
  u32 passed = 0;  // window barriers taken so far (all windows)
  for (u32 wsb = wstart; wsb < n; wsb += ZH_WINDOW) {
    u32 const we = min(wsb + ZH_WINDOW, n);
    dump_window<LONG>(ci8, lane, creg, cwe);
    __syncthreads();  // P: candidates of this window in cinfo
    u32 const done = passed + WIN_BARRIERS;
    // arr: the arrival counter as read with the last tile's read-back; a barrier taken
    // here means the counter is re-read for the next one
    auto take_ready = [&](u32 arr) {
      while (passed < done && arr >= (INS_TID / 64) * (passed + 1)) {
        __syncthreads();
        passed++;
        arr = __atomic_load_n(&misc_[MISC_ARR], __ATOMIC_RELAXED);
      }
    };
#ifdef ZH_STAMPS
    u64 const ti0 = __builtin_amdgcn_s_memtime();
#endif
    if (we < n) insert_window<LONG>(in32, T, we, min(we + ZH_WINDOW, n), lim, lane, creg, cwe, &misc_[MISC_ARR], take_ready);
#ifdef ZH_STAMPS
    u32 const dti = (u32)(__builtin_amdgcn_s_memtime() - ti0);
    st_ins += dti;
    if (lane == 0) atomicMax(&misc_[9], dti);
#endif
    while (passed < done) { __syncthreads(); passed++; }
  }
#ifdef ZH_STAMPS
  if (LONG && lane == 0) dbg[16] = st_ins;
#endif
  (void)dbg;
}

}  // namespace

// Diagnostic build only (-DZH_STAMPS): per-phase cycle sums of wave 0 into meta[4..9].
#ifdef ZH_STAMPS
#define ZH_STAMP(acc)                                           \
  do {                                                          \
    u64 _t = __builtin_amdgcn_s_memtime();                      \
    acc += (u32)(_t - stamp_prev);                              \
    stamp_prev = _t;                                            \
  } while (0)
#else
#define ZH_STAMP(acc) do { } while (0)
#endif

// The next block's input is loaded into registers while the current one is processed
// (persistent workgroups, one per CU): 64 KiB / 1024 threads = four 16-B vectors per thread.
// Only for blocks whose staged region (history prefix + block) is one 16-B aligned run of a
// multiple of 16 bytes -- every 64 KiB chunk and every history block; others stage directly.
struct Prefetch {
  uint4 v[4];
  bool ok;
};
__device__ __forceinline__ const u8 *staged_region(const ZhBlockDesc &d, u32 &n) {
  u32 const pre = d.pre_n;
  n = pre + d.n;
  // a history block's prefix is the input right before it: one contiguous region
  const u8 *const g = (pre && d.pre + pre == d.src) ? d.pre : (pre ? nullptr : d.src);
  return (d.n && g && (((uintptr_t)g) & 15) == 0 && (pre & 15) == 0 && (n & 15) == 0) ? g : nullptr;
}
__device__ __forceinline__ void prefetch_block(const ZhBlockDesc *__restrict__ blocks, u32 b, u32 nblocks, u32 tid, Prefetch &pf) {
  pf.ok = false;
  if (b >= nblocks) return;
  ZhBlockDesc const d = blocks[b];
  u32 n;
  const u8 *const g = staged_region(d, n);
  if (!g) return;
  pf.ok = true;
#pragma unroll
  for (u32 k = 0; k < 4; k++) {
    u32 const i = tid + K1_THREADS * k;
    pf.v[k] = i < (n >> 4) ? ((const uint4 *)g)[i] : make_uint4(0, 0, 0, 0);
  }
}

// Workgroup role of a thread: virtual wave = K1_WAVE_MAP nibble of its hardware wave (the
// wave-to-SIMD assignment is wave id mod 4).  ZH_K1_PERM 1 puts both inserters (virtual 14,
// 15) on SIMD 3 with one length wave and four length waves on each other SIMD: mix 13.74 ->
// 13.68 ms, but random data (few matches, the inserters are the critical path) 10.15 -> 10.72
// ms, so the default keeps the identity (inserters on SIMDs 2 and 3).
#ifndef ZH_K1_PERM
#define ZH_K1_PERM 0
#endif
// nibble p = virtual wave of hardware wave p
constexpr u64 K1_WAVE_MAP = ZH_K1_PERM ? 0xDBA9C876F543E210ull : 0xFEDCBA9876543210ull;
__device__ __forceinline__ u32 k1_tid() {
  u32 const t = threadIdx.x;
  return (u32)((K1_WAVE_MAP >> (4 * (t >> 6))) & 15u) << 6 | (t & 63u);
}

template <bool LAZY2>
__device__ __forceinline__ u32 lz_block(const ZhBlockDesc *__restrict__ blocks, ZhWorkspace ws, u32 b, u32 nblocks, u32 *s_take, Prefetch &pf) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u8 *in = smem + OFF_IN;
  u32 *in32 = (u32 *)in;
  u16 *TL = (u16 *)(smem + OFF_TL), *TS = (u16 *)(smem + OFF_TS);
  u32 *ci = (u32 *)(smem + OFF_CI);
  u8 *ci8 = smem + OFF_CI;
  u8 *exb = smem + OFF_EXB;
  u32 *wpart = (u32 *)(smem + OFF_WP);
  u32 *hbuf = (u32 *)(smem + OFF_HB);
  u32 *segx = (u32 *)(smem + OFF_SEG);
  u32 *misc = (u32 *)(smem + OFF_MISC);

  // opaque per-block thread index: stops the compiler from hoisting LDS addresses derived
  // from it out of the persistent block loop (they would stay live, and spill, across it)
  u32 tid;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(k1_tid()));
  u32 const lane = tid & 63;
  ZhBlockDesc const d = blocks[b];
  // the next block for this workgroup (dynamic: a slow block does not hold up a fixed share)
  if (tid == 0) *s_take = atomicAdd(ws.ctr, 1u);
  if (d.n == 0) {
    __syncthreads();
    u32 const next_b = *s_take;
    prefetch_block(blocks, next_b, nblocks, tid, pf);
    return next_b;
  }
  // A dictionary frame's first block is staged behind the tail of the dictionary content
  // (SURVEY §8f F2): positions [0, pre) are history only -- hashed and matched against,
  // never parsed (the parse starts at pre) -- so matches reach into the dictionary.
  u32 const pre = d.pre_n;
  u32 const n = pre + d.n;
  u32 *meta = ws.meta(b);
#ifdef ZH_STAMPS
  u64 const rt0 = __builtin_amdgcn_s_memrealtime();
  u64 stamp_prev = __builtin_amdgcn_s_memtime();
  u64 const mt0 = stamp_prev;
  u32 st_stage = 0, st_A = 0, st_X = 0, st_E1 = 0, st_Bmax = 0, st_Imax = 0, st_Bw = 0, st_B = 0, st_J = 0, st_E = 0, st_rounds = 0;
#endif

  // ---- stage the block into LDS (16 B per lane when the source allows it) and probe RLE
  // (the probe looks at the block only, never at the history in front of it)
  const u8 *src = d.src;
  bool same = true;
  u32 nst;
  if (pf.ok && staged_region(d, nst)) {  // prefetched during the previous block
    u32 const nv = n >> 4, pv = pre >> 4;
    u32 const f4 = src[0] * 0x01010101u;
#pragma unroll
    for (u32 k = 0; k < 4; k++) {
      u32 const i = tid + K1_THREADS * k;
      uint4 const v = pf.v[k];
      if (i < nv) {
        ((uint4 *)in)[i] = v;
        same &= i < pv || ((v.x == f4) & (v.y == f4) & (v.z == f4) & (v.w == f4));
      }
    }
  } else if (const u8 *const gsrc = (pre && d.pre + pre == src) ? d.pre : (pre ? nullptr : src);
             gsrc && (((uintptr_t)gsrc) & 15) == 0 && (pre & 15) == 0) {
    u32 const nv = n >> 4, pv = pre >> 4;
    u8 const first = src[0];
    u32 const f4 = first * 0x01010101u;
    for (u32 i = tid; i < nv; i += K1_THREADS) {
      uint4 v = ((const uint4 *)gsrc)[i];
      ((uint4 *)in)[i] = v;
      same &= i < pv || ((v.x == f4) & (v.y == f4) & (v.z == f4) & (v.w == f4));
    }
    for (u32 i = (nv << 4) + tid; i < n; i += K1_THREADS) { u8 c = gsrc[i]; in[i] = c; same &= c == first; }
  } else if (pre) {  // dictionary tail + block, byte loads
    const u8 *const pp = d.pre;
    u8 const first = src[0];
    for (u32 i = tid; i < n; i += K1_THREADS) {
      u8 const c = i < pre ? pp[i] : src[i - pre];
      in[i] = c;
      same &= i < pre || c == first;
    }
  } else {
    u8 const first = src[0];
    for (u32 i = tid; i < n; i += K1_THREADS) { u8 c = src[i]; in[i] = c; same &= c == first; }
  }
  if (tid < 16) in[n + tid] = 0;
  // A dictionary frame's first block starts from the dictionary's precomputed tables when the
  // batch has them (ws.dtab): their entries (tail position + 1) move to this block's staged
  // positions (entries before the staged tail are dropped), the last tail positions up to the
  // batch of tiles holding `pre` are inserted by the inserter waves (insert_span), and the
  // window loop starts at the window holding `pre` -- the same tables, candidates and parse as
  // inserting every history position (the oracle's order), without the history windows.
  bool const use_dt = ws.dtab && (d.flags & ZH_F_DICT) && (d.flags & ZH_F_FIRST) && pre >= 2 * ZH_DTAB_MARGIN && d.n >= 16 &&
                      ws.dtab_P >= pre;
  if (use_dt) {
    u32 const delta = ws.dtab_P - pre;
    const u32 *dt32 = (const u32 *)ws.dtab;
    auto clip = [&](u32 e) { return e > delta ? e - delta : 0u; };
    for (u32 i = tid; i < (HL_SIZE + HS_SIZE) / 2; i += K1_THREADS) {
      u32 const w = dt32[i];
      u32 const v = clip(w & 0xFFFFu) | (clip(w >> 16) << 16);
      u32 const j = i < HL_SIZE / 2 ? i : i + T_PAD / 2;  // TS follows TL's pad
      ((u32 *)TL)[j] = v;
    }
    if (tid < T_PAD) ((u16 *)TL)[tid < T_PAD / 2 ? HL_SIZE + tid : HL_SIZE + T_PAD + HS_SIZE + (tid - T_PAD / 2)] = 0;
  } else {
    for (u32 i = tid; i < (HL_SIZE + HS_SIZE + 2 * T_PAD) / 2; i += K1_THREADS) ((u32 *)TL)[i] = 0;  // both tables (adjacent)
  }
  // History without precomputed tables (a frame's later blocks, stream history, dictionary
  // views): only the final table over positions [0, pmin) -- the latest position per slot --
  // matters, so every wave inserts them at once (below) instead of the inserter waves walking
  // the history windows.
  bool const par_hist = !use_dt && pre >= 2 * ZH_TILE && d.n >= 16;
  // first window / first tile processed and the tail positions the inserters add themselves
  u32 const pmin = (use_dt || par_hist) ? pre & ~(ZH_TILE - 1) : 0u;  // the tile holding pre
  u32 const wstart = (use_dt || par_hist) ? (pre & ~(ZH_WINDOW - 1)) : 0u;
  u32 const span_s = use_dt ? pre - ZH_DTAB_MARGIN : 0u, span_e = use_dt ? pmin : 0u;
  if (tid < 2) misc[8 + tid] = 0;
  if (tid == 0) misc[MISC_ARR] = 0;
  bool const rle = __syncthreads_and(same) && d.n >= 2;
  u32 const next_b = *s_take;  // (written before the barrier above)
  prefetch_block(blocks, next_b, nblocks, tid, pf);  // the next block's input, in flight from here
  if (rle) {
    if (tid == 0) { meta[0] = 0; meta[1] = 0; meta[2] = 1; }
    return next_b;
  }
  if (par_hist) {
    // store every position, then rounds of read-back: a slot holding an older position than
    // one hashing there is raised (values only grow) until no thread changes anything
    for (u32 round = 0;; round++) {
      bool ch = false;
      for (u32 p = tid; p < pmin; p += K1_THREADS) {
        u32 lo, hi;
        ld64u(in32, p, lo, hi);
        u32 const hl = hash_of<true>(lo, hi), hs = hash_of<false>(lo, hi);
        u16 const v = (u16)(p + 1);
        if (round == 0) {
          TL[hl] = v;
          TS[hs] = v;
        } else {
          if (TL[hl] < v) { TL[hl] = v; ch = true; }
          if (TS[hs] < v) { TS[hs] = v; ch = true; }
        }
      }
      if (round == 0) __syncthreads();
      else if (!__syncthreads_or(ch)) break;
    }
  }

  ZH_STAMP(st_stage);
  u64 *seq_out = ws.seq(b);
  u8 *lit_out = ws.lits(b);
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 nseq_tot = 0, nlit_tot = 0, e_in = pre;
  // ---- inserter waves: their own loop with the same barrier sequence as the workers'
  // (separate code, so their registers never add to the workers' pressure)
  if (tid >= INS_TID) {
    // The inserters are the youngest waves of the workgroup and would lose every VALU
    // issue arbitration to the 3 worker waves sharing their SIMD; the next window's tables
    // gate the workers' next window, so they take priority (MI355X_MICROARCH.md, "VALU issue
    // is arbitrated ... by priority, then age").
    __builtin_amdgcn_s_setprio(2);
    if (tid < INS_TID + 64) inserter_loop<true>(in32, TL, ci8, misc, n, lim, lane, ws.dbg(b), wstart, pmin, span_s, span_e);
    else inserter_loop<false>(in32, TS, ci8, misc, n, lim, lane, ws.dbg(b), wstart, pmin, span_s, span_e);
    __builtin_amdgcn_s_setprio(0);
    return next_b;
  }

  u32 const tid_ = tid;
  for (u32 wsb = wstart; wsb < n; wsb += ZH_WINDOW) {
    u32 const we = min(wsb + ZH_WINDOW, n);
    // opaque per-window thread index: keeps the compiler from hoisting every LDS address
    // derived from it out of the window loop (they would be spilled to scratch)
    u32 tid;
    __asm__ volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(tid_));
    u32 const lane = tid & 63;
    __syncthreads();  // P
    ZH_STAMP(st_A);
    if (we <= pre) {  // dictionary history only: nothing to parse, keep the barrier sequence
      for (u32 k = 0; k < WIN_BARRIERS; k++) {
        if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
        __syncthreads();
      }
      continue;
    }
#ifdef ZH_STAMPS
    u64 const tP = __builtin_amdgcn_s_memtime();
#endif

    // ---- match lengths (threads 0..NB), while the inserter waves build the next window
    // (a worker wave without positions skips the phase: wave-uniform)
    if ((tid & ~63u) <= NB) {
      // thread tid < NB: positions [s, se) of the window; thread NB: position `we`;
      // threads above NB take part in the wave-level steps with no positions
      u32 const s = tid < NB ? wsb + SB * tid : we;
      u32 const se = tid < NB ? min(s + SB, we) : (tid == NB ? min(we + 2, n) : s);  // (we, we+1: lookahead)
      u32 const cbase = tid < NB ? SB * tid : ZH_WINDOW;  // window index of position s
      // (1) candidates, own bytes and first-8-byte prefixes; loads unconditional
      u32 cv[SB], plp = 0, psp = 0;  // prefixes packed 4 bits per position
      // the thread's own bytes [s, s + SB + 7) from four aligned dwords, shared by its SB
      // positions (positions past lim have cv = 0: their bytes are never compared)
      static_assert(SB <= 8 && ZH_WINDOW + 2 + SB <= CI_WORDS, "heads: bit j (L) and 8 + j (S); junk slots");
      constexpr u32 NOWN = (SB + 7 + 3) / 4;  // dwords of own bytes
      u32 own[NOWN];
      {
        u32 const w = s >> 2, sh = s & 3u;
        u32 aw[NOWN + 1];
#pragma unroll
        for (u32 k = 0; k <= NOWN; k++) aw[k] = in32[w + k];
#pragma unroll
        for (u32 k = 0; k < NOWN; k++) own[k] = __builtin_amdgcn_alignbyte(aw[k + 1], aw[k], sh);
      }
#pragma unroll
      for (u32 j = 0; j < SB; j++) {
        u32 const p = s + j;
        bool const v = p < se && p < lim;
        u32 const cw = ci[cidx(cbase + j)];
        cv[j] = v ? cw : 0u;
        u32 const q = j >> 2, r = j & 3u;
        u32 const olo = r ? __builtin_amdgcn_alignbyte(own[q + 1], own[q], r) : own[q];
        u32 const ohi = r ? __builtin_amdgcn_alignbyte(own[q + 2], own[q + 1], r) : own[q + 1];
        u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16;
        // wave-uniform skips (no lane has a candidate: rare matches), branch-free inside
        u32 xL = 0, xS = 0;
        if (__ballot(cL != 0)) {
          u32 const t = prefix8(in32, cL ? cL - 1 : 0u, olo, ohi);
          xL = cL ? t : 0u;
        }
        bool const hasS = cS && cS != cL;
        if (__ballot(hasS)) {
          u32 const t = prefix8(in32, hasS ? cS - 1 : 0u, olo, ohi);
          xS = hasS ? t : 0u;
        }
        plp |= xL << (4 * j);
        psp |= xS << (4 * j);
      }
#define PL(j) ((plp >> (4 * (j))) & 15u)
#define PS(j) ((psp >> (4 * (j))) & 15u)
      // (2) chains: a candidate with 8 matching bytes that continues a previous-position
      //     candidate with the same offset (also 8 matching) is a follower; else a head
      //     Bit-parallel over the thread's SB positions (bit j = position j), no branches:
      //     e = 8 matching bytes (nibble bit 3 of the packed prefix; 0 without a
      //     candidate), continuation = candidate == previous position's candidate + 1.
      auto nib8 = [](u32 pk) {  // bit j = nibble j == 8
        u32 r = 0;
#pragma unroll
        for (u32 j = 0; j < SB; j++) r |= ((pk >> (4 * j + 3)) & 1u) << j;
        return r;
      };
      u32 const eL = nib8(plp), eS = nib8(psp);
      u32 dL = 0, dS = 0, fromSL = 0, fromSS = 0, heads = 0;  // heads: bit j = L, bit 8 + j = S
      if (__ballot((eL | eS) != 0)) {  // (wave-uniform skip: no 8-byte match in the wave)
        u32 mLL = 0, mLS = 0, mSL = 0, mSS = 0;  // bit j: cX_j == cY_{j-1} + 1
#pragma unroll
        for (u32 j = 1; j < SB; j++) {
          u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16, pL1 = (cv[j - 1] & 0xFFFFu) + 1, pS1 = (cv[j - 1] >> 16) + 1;
          mLL |= cL == pL1 ? 1u << j : 0u;
          mLS |= cL == pS1 ? 1u << j : 0u;
          mSL |= cS == pL1 ? 1u << j : 0u;
          mSS |= cS == pS1 ? 1u << j : 0u;
        }
        u32 const peL = eL << 1, peS = eS << 1;
        u32 const fLL = eL & peL & mLL, fLS = eL & ~fLL & peS & mLS;
        u32 const fSL = eS & peL & mSL, fSS = eS & ~fSL & peS & mSS;
        dL = fLL | fLS; dS = fSL | fSS; fromSL = fLS; fromSS = fSS;
        heads = (eL & ~dL) | ((eS & ~dS) << 8);
      }
      // (3) extend the heads, compacted across the wave: heads are ranked in (lane, bit)
      //     order and handed out 64 at a time, one per lane (wave-private LDS slots;
      //     a wave's LDS operations execute in order, so no barrier is needed).  The
      //     extension goes back into the head position's own cinfo word (byte 0 for L,
      //     byte 2 for S: the half that was just consumed), read back in (4).
      {
        u32 const nh = __builtin_popcount(heads);
        u32 const inc = wave_scan_incl(nh);
        u32 const hbase = inc - nh, htot = __builtin_amdgcn_readlane(inc, 63);
        u32 *hb = hbuf + (tid >> 6) * HB_STRIDE;
        for (u32 c0 = 0; c0 < htot; c0 += 64) {
          // branch-free scatter: slots not in this pass (or not heads) write the junk slot
          u32 r = hbase - c0;
#pragma unroll
          for (u32 k = 0; k < 2 * SB; k++) {
            u32 const bit = k < SB ? k : 8 + (k - SB);
            u32 const h = (heads >> bit) & 1u;
            hb[h && r < 64u ? r : 64u] = (cbase + (k < SB ? k : k - SB)) | (k < SB ? 0u : 0x8000u);
            r += h;
          }
          __asm__ volatile("" ::: "memory");
          if (c0 + lane < htot) {
            u32 const e = hb[lane];  // window index (13 bits) | S flag (bit 15)
            u32 const w = e & 0x1FFFu, sf = e >> 15;
            u32 const cw = ci[cidx(w)];
            u32 const c = sf ? cw >> 16 : cw & 0xFFFFu;
            ci8[4 * cidx(w) + 2 * sf] = (u8)ext_head(in32, wsb + w, c - 1, n);
          }
          __asm__ volatile("" ::: "memory");
        }
      }
      // (4) lengths in position order; E = exact prefix below 8, the head's extension,
      //     or the predecessor's E - 1; capped length = min(E, 64, n - p)
      u32 EL = 0, ES = 0;
#pragma unroll
      for (u32 j = 0; j < SB; j++) {
        u32 const p = s + j;
        u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16;
        u32 const capj = min((u32)ZH_MAX_MATCH, n - min(p, n));
        u32 const hx = ci[cidx(cbase + j)];  // head extensions from (3)
        // selects only (no divergent branches: exec-mask work on the scalar unit)
        u32 const eFL = ((fromSL >> j) & 1u) ? ES : EL, eFS = ((fromSS >> j) & 1u) ? ES : EL;
        u32 nL = ((heads >> j) & 1u) ? (hx & 255u) : PL(j);
        nL = ((dL >> j) & 1u) ? eFL - 1u : nL;
        u32 nS = ((heads >> (8 + j)) & 1u) ? ((hx >> 16) & 255u) : PS(j);
        nS = ((dS >> j) & 1u) ? eFS - 1u : nS;
        nS = (cS && cS == cL) ? nL : nS;
        EL = nL; ES = nS;
        u32 const rL = min(nL, capj), rS = min(nS, capj);
        u32 const lL = (cL && rL >= ZH_MIN_MATCH_LONG) ? rL : 0u;
        u32 const lS = (cS && rS >= ZH_MIN_MATCH_SHORT) ? rS : 0u;
        bool const useL = lL && lL >= lS;
        u32 const ml = useL ? lL : lS, cm = useL ? cL : cS;
        u32 const v = ml ? ((p - (cm - 1u)) << 8) | ml : 0u;
        ci[p < se ? cidx(cbase + j) : ZH_WINDOW + 2 + j] = v;  // (past the run: junk slots)
      }
      if (tid == NB && we >= n) ci[cidx(ZH_WINDOW)] = 0;          // no position after the block
      if (tid == NB && we + 1 >= n) ci[cidx(ZH_WINDOW + 1)] = 0;
#undef PL
#undef PS
    }
    ZH_STAMP(st_Bw);
#ifdef ZH_STAMPS
    if (lane == 0) atomicMax(&misc[8], (u32)(__builtin_amdgcn_s_memtime() - tP));
#endif
    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
    __syncthreads();  // R
    ZH_STAMP(st_B);
#ifdef ZH_STAMPS
    if (tid == 0) { st_Bmax += misc[8]; st_Imax += misc[9]; misc[8] = 0; misc[9] = 0; }
#endif
    u32 const info_ahead = __builtin_amdgcn_readfirstlane(ci[cidx(ZH_WINDOW)]);
    u32 const info_ahead2 = LAZY2 ? __builtin_amdgcn_readfirstlane(ci[cidx(ZH_WINDOW + 1)]) : 0u;

    // ---- parse.  Lanes = positions (PR rounds of the 896 worker lanes); each wave's 64
    // lanes are one parse segment of 64 positions.  step(p) = next position the greedy /
    // lazy-1 parse visits after p; pointer doubling inside the segment (ds_bpermute)
    // gives X_k = 2^k steps for k < 6 and the segment exit of every position.
    u32 const wn = we - wsb;
    u32 const la = info_ahead;  // match info of position `we` (lazy rule at the window end)
    u32 xk[PR][6];              // [round][k]: X_{2^k}, relative to the segment start
    u32 infr[PR];               // match info of positions where the parse takes a match
#pragma unroll
    for (u32 rr = 0; rr < PR; rr++) {
      u32 const i = INS_TID * rr + tid;
      u32 X[7];
      infr[rr] = parse_steps<LAZY2>(ci, i, wn, la, info_ahead2, lane, X);
#pragma unroll
      for (u32 k = 0; k < 6; k++) xk[rr][k] = X[k];
      exb[i < wn ? i : (u32)ZH_WINDOW] = (u8)X[6];  // (past the window: junk byte)
    }
    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
    __syncthreads();  // X: exits of all positions
    ZH_STAMP(st_X);
    // Jacobi fixed point of the 64 segment entries (wave 0, lane = segment, no barrier
    // needed): entry(t) = max(start(t), exit of segment t-1 from its entry) == the
    // serial parse once no entry changes
    if (tid < 64) {
      u32 const S = wsb + 64 * lane;
      u32 const SE = min(S + 64, we);
      u32 entry = lane == 0 ? max(wsb, e_in) : S;
      u32 ex = entry;
      for (;;) {
        ex = entry < SE ? S + exb[64 * lane + (entry - S)] : entry;
        u32 const pe = wave_shr1(ex);
        u32 const ne = lane == 0 ? max(wsb, e_in) : max(S, pe);
        bool const ch = ne != entry;
        entry = ne;
#ifdef ZH_STAMPS
        st_rounds++;
#endif
        if (!__ballot(ch)) break;
      }
      segx[lane] = entry;
      if (lane == ((wn - 1) >> 6)) segx[64] = ex;  // the window's exit = next window's entry
    }
    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
    __syncthreads();  // J: converged segment entries
    ZH_STAMP(st_J);
    u32 const e_out = __builtin_amdgcn_readfirstlane(segx[64]);

    // ---- emission, lanes = positions: a position is on the parse path iff binary
    // lifting from its segment's entry (X_32 .. X_1) lands on it; scans of the
    // take/literal flags give each record's and literal's slot
    u32 fl[PR];    // bit 0 literal, bit 1 match start
#pragma unroll
    for (u32 rr = 0; rr < PR; rr++) {
      u32 const i = INS_TID * rr + tid;
      u32 const sb = i & ~63u;
      u32 cur = segx[min(i >> 6, 63u)] - (wsb + sb);  // >= 64 when the segment is skipped
      if (__ballot(infr[rr] != 0)) {
#pragma unroll
        for (int k = 5; k >= 0; k--) {
          u32 const y = bperm(xk[rr][k], min(cur, 63u));
          if (cur <= lane && y <= lane) cur = y;
        }
      } else {  // all literals: every position from the entry on is visited
        cur = cur <= lane ? lane : cur;
      }
      bool const vis = i < wn && cur == lane;
      fl[rr] = vis ? (infr[rr] ? 2u : 1u) : 0u;
    }
    u32 lcnt[PR], scnt[PR];
#pragma unroll
    for (u32 rr = 0; rr < PR; rr++) {
      u64 const ml = __ballot(fl[rr] & 1u), ms = __ballot(fl[rr] & 2u);
      lcnt[rr] = __builtin_amdgcn_mbcnt_hi((u32)(ml >> 32), __builtin_amdgcn_mbcnt_lo((u32)ml, 0u));
      scnt[rr] = __builtin_amdgcn_mbcnt_hi((u32)(ms >> 32), __builtin_amdgcn_mbcnt_lo((u32)ms, 0u));
      if (lane == 0) wpart[rr * NWW + (tid >> 6)] = (u32)__popcll(ml) | ((u32)__popcll(ms) << 16);
    }
    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
    __syncthreads();  // E1: per-wave counts (cinfo is free for the inserters from here on)
    ZH_STAMP(st_E1);
    if (tid < 64) {   // exclusive scan of the PR*NWW (round, wave) counts, in position order
      u32 carry = 0;
#pragma unroll
      for (u32 c0 = 0; c0 < PR * NWW; c0 += 64) {
        u32 const v = c0 + lane < PR * NWW ? wpart[c0 + lane] : 0u;
        u32 const inc = wave_scan_incl(v);
        if (c0 + lane < PR * NWW) wpart[WP_OFF + c0 + lane] = carry + inc - v;
        carry += __builtin_amdgcn_readlane(inc, 63);
      }
      if (tid == 0) wpart[WP_TOT] = carry;
    }
    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
    __syncthreads();  // E2: offsets
#pragma unroll
    for (u32 rr = 0; rr < PR; rr++) {
      u32 const i = INS_TID * rr + tid;
      u32 const off = wpart[WP_OFF + rr * NWW + (tid >> 6)];
      u32 const li = (off & 0xFFFFu) + lcnt[rr], si = (off >> 16) + scnt[rr];
      if (fl[rr] & 1u) lit_out[nlit_tot + li] = in[wsb + i];
      if (fl[rr] & 2u) seq_out[nseq_tot + si] = (u64)(nlit_tot + li) | ((u64)(infr[rr] & 255u) << 17) | ((u64)(infr[rr] >> 8) << 25);
    }
    u32 const total = __builtin_amdgcn_readfirstlane(wpart[WP_TOT]);
    nseq_tot += total >> 16;
    nlit_tot += total & 0xFFFFu;
    e_in = e_out;
    ZH_STAMP(st_E);
  }
  if (tid == 0) { meta[0] = nseq_tot; meta[1] = nlit_tot; meta[2] = 0; }
#ifdef ZH_STAMPS
  if (tid == 0) {
    u32 *dbg = ws.dbg(b);
    dbg[23] = (u32)rt0; dbg[24] = (u32)__builtin_amdgcn_s_memrealtime();
    dbg[25] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    dbg[26] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    dbg[27] = (u32)(__builtin_amdgcn_s_memtime() - mt0);
    dbg[40] = st_Bmax; dbg[41] = st_Imax;
    dbg[0] = st_stage; dbg[1] = st_A; dbg[2] = st_B; dbg[3] = st_J; dbg[4] = st_E; dbg[5] = st_rounds; dbg[20] = st_Bw; dbg[21] = st_X; dbg[22] = st_E1;
  }
#endif
  return next_b;
}

// Persistent workgroups (grid = one per CU, the LDS footprint allows no second): workgroup g
// takes blocks g, g + grid, ... and stages each block from registers loaded while the previous
// one was processed, so the HBM latency of staging and the per-block launch gap overlap work.
template <bool LAZY2>
__device__ __forceinline__ void lz_blocks(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  __shared__ u32 s_take;  // block index taken from the counter, broadcast to the workgroup
  if (threadIdx.x == 0) s_take = atomicAdd(ws.ctr, 1u);
  __syncthreads();
  u32 b = s_take;
  Prefetch pf;
  prefetch_block(blocks, b, nblocks, k1_tid(), pf);
  while (b < nblocks) {
    b = lz_block<LAZY2>(blocks, ws, b, nblocks, &s_take, pf);  // returns the next block taken
    __syncthreads();  // every wave is done with this block's LDS before the next is staged
  }
}
// level < 9: greedy + lazy-1; level >= 9: LAZY2 (the same kernel body, one instantiation each)
extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  lz_blocks<false>(blocks, nblocks, ws);
}
extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_lazy2_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  lz_blocks<true>(blocks, nblocks, ws);
}

extern "C" u32 zh_lz_lds_bytes() { return K1_LDS; }

// A dictionary's K1 tables (ZhWorkspace::dtab), built once per dictionary: t32[slot] = max over
// tail positions j < B hashing there of j + 1 (the latest, as K1's in-order insertion leaves
// it), then packed to u16.  tail = the last P content bytes.
extern "C" __global__ void zh_dict_hash_kernel(const u8 *__restrict__ tail, u32 B, u32 *__restrict__ t32) {
  for (u32 j = blockIdx.x * blockDim.x + threadIdx.x; j < B; j += gridDim.x * blockDim.x) {
    u32 const lo = (u32)tail[j] | ((u32)tail[j + 1] << 8) | ((u32)tail[j + 2] << 16) | ((u32)tail[j + 3] << 24);
    u32 const hi = (u32)tail[j + 4] | ((u32)tail[j + 5] << 8) | ((u32)tail[j + 6] << 16) | ((u32)tail[j + 7] << 24);
    atomicMax(&t32[hash_of<true>(lo, hi)], j + 1);
    atomicMax(&t32[HL_SIZE + hash_of<false>(lo, hi)], j + 1);
  }
}
extern "C" __global__ void zh_dict_pack_kernel(const u32 *__restrict__ t32, u16 *__restrict__ out) {
  u32 const i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < HL_SIZE + HS_SIZE) out[i] = (u16)t32[i];
}

namespace zh {
hipError_t lz_init() {
  hipError_t e = hipFuncSetAttribute((const void *)zh_lz_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K1_LDS);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void *)zh_lz_lazy2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K1_LDS);
}
// tables for the last P = min(cn, 65535) content bytes (positions [0, P - ZH_DTAB_MARGIN));
// out: 2^15 u16 (long table, then short), tmp32: 2^15 u32 scratch.  P = 0: none (too short).
hipError_t lz_dict_tables(const u8 *content, size_t cn, u16 *out, u32 *tmp32, u32 &P, hipStream_t stream) {
  P = (u32)std::min(cn, (size_t)65535);
  if (P < 2 * ZH_DTAB_MARGIN) { P = 0; return hipSuccess; }
  u32 const B = P - ZH_DTAB_MARGIN;
  hipError_t e = hipMemsetAsync(tmp32, 0, 4 * (HL_SIZE + HS_SIZE), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(zh_dict_hash_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, content + cn - P, B, tmp32);
  hipLaunchKernelGGL(zh_dict_pack_kernel, dim3((HL_SIZE + HS_SIZE + 255) / 256), dim3(256), 0, stream, tmp32, out);
  return hipGetLastError();
}
void lz_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, bool lazy2, hipStream_t stream) {
  // one persistent workgroup per CU of the stream's device
  int dev = 0, cus = 0;
  if (stream) (void)hipStreamGetDevice(stream, &dev);
  else (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  u32 const grid = std::min(nblocks, (u32)cus);
  if (lazy2) hipLaunchKernelGGL(zh_lz_lazy2_kernel, dim3(grid), dim3(K1_THREADS), K1_LDS, stream, d_descs, nblocks, ws);
  else hipLaunchKernelGGL(zh_lz_kernel, dim3(grid), dim3(K1_THREADS), K1_LDS, stream, d_descs, nblocks, ws);
}
}  // namespace zh
