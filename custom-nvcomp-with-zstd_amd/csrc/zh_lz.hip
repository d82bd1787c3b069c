// zh_lz.hip — K1: LZ77 match finding + parse for one <=64 KiB block per workgroup.
//
// Replaces the reference's find_matches_kernel / greedy_parse_kernel /
// build_sequences_gpu_kernel<<<1,1>>> (src/lz77_parallel.cu:26-70, 177-268)
// and the literal gather kernels (src/cuda_zstd_manager.cu:602-723).
// Output is identical to oracle/zstd_oracle.c orc_lz_parse_pre (tile-lagged hash
// insertion, longer of long/short candidate, greedy + lazy-1 parse, catch-up, window-granular
// miss skip, incompressibility probe).  Three instantiations by level (ZH_K1_MODE): mode 0 (levels
// 3-4) both tables + the lazy-1 check; mode 1 (level 2) the short table only; mode 2 (level 1) the
// short table only, greedy -- the long inserter wave then only keeps the step barriers.
//
// One persistent workgroup of 1024 threads (16 wave64, one workgroup per CU), blocks taken
// from a device counter, everything in LDS:
//   in[]   the block (and its history prefix), staged once with 16-B loads (64 KiB)
//   TL/TS  2 x 2^14 u16 hash tables, entry = position + 1 (0 = empty)
//   cinfo  two 2048-position windows: candidates -> match info (off<<8|len) in place
//   tm     take masks (per 64-position round), two windows
//   lm     per window parity, per 32-position walk segment: the literal bits
//   mlist  per window parity: the window's matches in order (start, catch-up bound, length,
//          offset, the walk's literals before it)
// A three-stage window pipeline, step k:
//   waves 14, 15  inserters (s_setprio 2): one wave per hash table inserts window k+1's tiles
//                 of ZH_TILE positions, two per LDS round trip (program order = LDS order
//                 within a wave; lanes of one store that hit the same slot are checked by a
//                 read-back); candidates stay in registers and are dumped after barrier X.
//   waves 1..13   window k's match lengths, lanes = positions: each candidate's common prefix
//                 from its first 8 bytes, and along same-offset chains (the candidate of p+1
//                 is the candidate of p plus one) lcp(p) = 1 + lcp(p+1): a ballot of the chain
//                 ends and one ds_bpermute give every position its length, only chain ends
//                 past 8 bytes are extended; then the parse's take decision per position.
//   wave 0        window k-1's parse, lanes = 32-position segments: each lane walks its
//                 segment (one literal run + one match per step, from the take mask) from a
//                 guessed entry; Jacobi rounds re-walk the segments whose entry changed until
//                 the walk meets the previous one -- exactly the serial parse; then the
//                 window's match list.
//   wave 1        after its lengths: window k-2's catch-up and sequence records.
//   after X       span-top take decisions (each wave its own); window k-2's literals.
#include "zh_common.h"
#include "zh_hash.h"

#include <algorithm>
#include <vector>

#if defined(ZH_STAMPS) || defined(ZH_INS_CHECK)
__device__ u32 g_fixups;  // diagnostic: inserter read-back repairs (all blocks; tests/test_gpu_k1.py)
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
// Diagnostic build only (-DZH_TIMELINE, tools/timeline.py): per K1 wave and step phase, the
// s_memtime cycles summed over every step of every block (VERDICT r5 item 2's executed per-phase
// breakdown of the window pipeline).  Worker waves: 0 P wait, 1 lengths, 2 parse / records,
// 3 X wait, 4 span tops + literals; inserter waves: 0 P wait, 1 insertion of the next window (the X
// barrier taken between its tiles included), 3 barriers left after it, 4 candidate dump; [5] steps.
#ifdef ZH_TIMELINE
__device__ unsigned long long g_tl[16 * 8];
extern "C" __global__ void zh_read_timeline(unsigned long long *out) {
  for (u32 i = threadIdx.x; i < 16 * 8; i += blockDim.x) { out[i] = g_tl[i]; g_tl[i] = 0; }
}
extern "C" int zh_timeline_host(unsigned long long *out128) {
  unsigned long long *d = nullptr;
  if (hipMalloc(&d, 16 * 8 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(zh_read_timeline, dim3(1), dim3(128), 0, 0, d);
  hipError_t e = hipMemcpy(out128, d, 16 * 8 * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return e == hipSuccess ? 0 : 1;
}
#define TL_DECL u64 tl_[6] = {0, 0, 0, 0, 0, 0}; u64 tl_prev = __builtin_amdgcn_s_memtime()
#define TL_MARK(ph) do { u64 const _t = __builtin_amdgcn_s_memtime(); tl_[ph] += _t - tl_prev; tl_prev = _t; } while (0)
#define TL_STEP() (tl_[5]++)
#define TL_FLUSH(w, lane) do { if ((lane) == 0) for (u32 _i = 0; _i < 6; _i++) atomicAdd(&g_tl[(w) * 8 + _i], (unsigned long long)tl_[_i]); } while (0)
#else
#define TL_DECL do { } while (0)
#define TL_MARK(ph) do { } while (0)
#define TL_STEP() do { } while (0)
#define TL_FLUSH(w, lane) do { } while (0)
#endif
namespace {

#ifndef ZH_K1_PMAX
#define ZH_K1_PMAX 1  // Jacobi entries from the prefix max of exits (K1 11.53 -> 11.50 ms)
#endif
constexpr u32 K1_THREADS = 1024;
constexpr u32 K1_REDO = ~0u;      // lz_block: parse this block again without the probe
constexpr u32 NROUND = ZH_WINDOW / 64;      // 64-position length rounds per window
constexpr u32 SEGP = 32;                    // positions per walk segment (one lane of wave 0)
constexpr u32 NSEG = ZH_WINDOW / SEGP;      // walk segments per window
constexpr u32 INS_TID = 896;                // first inserter thread (waves 14, 15)
// worker rounds per wave (rounds_of below): 2 bits per wave, 0 2 3 3 3 3 3 3 3 2 2 2 2 1
constexpr u64 ROUND_TAB = 0x6abfff8ull;
constexpr u32 NWW = INS_TID / 64;           // worker waves
constexpr u32 TILES = ZH_WINDOW / ZH_TILE;  // 16 tiles per window
constexpr u32 TPL = ZH_TILE / 64;           // positions per inserter lane per tile
constexpr u32 NCR = TILES * TPL / 2;        // candidate registers per inserter lane (u16 pairs)
static_assert(NSEG == 64, "one walk lane per segment");
static_assert(INS_TID == 896 && NROUND == 32, "round split: waves 1..13 take 6 x 3 + 7 x 2 rounds");
constexpr u32 REC_WAVE = 1;  // the worker wave that writes a window's records (after its length rounds)
static_assert(ZH_WINDOW % ZH_TILE == 0 && ZH_TILE % 64 == 0 && TILES * TPL % 2 == 0, "tiles tile windows");

constexpr u32 HL_SIZE = 1u << ZH_HASH_LOG_LONG;
constexpr u32 HS_SIZE = 1u << ZH_HASH_LOG_SHORT;
constexpr u32 T_PAD = 8;                    // + a junk slot (index HL/HS_SIZE) for lanes past lim
constexpr u32 OFF_IN = 0;
constexpr u32 OFF_TL = OFF_IN + ZH_BLOCK_MAX + 16;
constexpr u32 OFF_TS = OFF_TL + 2 * (HL_SIZE + T_PAD);
constexpr u32 OFF_CI = OFF_TS + 2 * (HS_SIZE + T_PAD);
constexpr u32 CI_WORDS = ZH_WINDOW + 8;  // + the lookahead slots of positions `we`, `we + 1`
__device__ __forceinline__ u32 cidx(u32 i) { return i; }
// two cinfo buffers: window k's candidates / match info in buffer k & 1 (the parse of window k
// overlaps the lengths of window k + 1)
constexpr u32 OFF_HM = OFF_CI + 2 * 4 * CI_WORDS;    // per buffer u64 per round: take masks (see span_lengths)
// The literal bytes of a window are extracted (ZH_LIT_INS = 0) by the worker waves after barrier X
// of the step that wrote its records, or (1) one step later by the inserter waves, before X, once
// they have built the next window's tables (the step's post-X phase shrinks to the span tops).
// Round 6 (profiles/r06i_lit_ins_ab.json): level 3 K1 10.36 -> 10.12 ms, level 1 8.02 -> 7.52 ms;
// the step 11.66 k -> 10.95 k cycles (tools/timeline.py).
#ifndef ZH_LIT_INS
#define ZH_LIT_INS 1
#endif
constexpr u32 LM_BUFS = ZH_LIT_INS ? 3 : 2;         // windows whose literal bits are alive at once
constexpr u32 LB_BUFS = ZH_LIT_INS ? 2 : 1;         // literal prefix-count buffers
constexpr u32 STEPS_EXTRA = ZH_LIT_INS ? 3 : 2;     // loop steps per block: windows + STEPS_EXTRA
constexpr u32 OFF_SEGM = OFF_HM + 2 * 8 * NROUND;    // per window (mod LM_BUFS), per walk segment (u32 each):
// the literal bits left after catch-up
__device__ __forceinline__ u32 segm(u32 par) { return par * NSEG; }
constexpr u32 ML_CAP = ((ZH_WINDOW + ZH_MIN_MATCH_SHORT - 1) / ZH_MIN_MATCH_SHORT + 12 + 3) & ~3u;  // matches per window
constexpr u32 OFF_ML = OFF_SEGM + 4 * LM_BUFS * NSEG;  // per window parity: the window's matches in order (u64,
                                                     // ML_* fields) for the records one step later
constexpr u32 XQ_CAP = 196;                          // chain-end queue entries per worker wave (<= 191
                                                     // used: < 64 left + 2 x 64 per round; the last is a spare)
constexpr u32 OFF_XQ = OFF_ML + 2 * 8 * ML_CAP;      // u16 per entry: window index | S << 15
constexpr u32 OFF_MISC = OFF_XQ + 2 * XQ_CAP * NWW;  // [2 par + 0] matches, [2 par + 1] first parsed position
constexpr u32 OFF_LB = OFF_MISC + 4 * 16;            // window k - 2's literal prefix counts per walk
                                                     // segment (+ the window's total), for the literal phase
constexpr u32 LB_WORDS = NSEG + 4;
// One barrier per window step (ZH_ONE_BARRIER, needs ZH_LIT_INS): the take bits at the worker
// waves' span tops (lazy rule: they need the next span's first info) are decided by wave 0 at the
// start of the window's parse in the next step (and by every wave in the probe step), and the
// inserters dump the next window's candidates once wave 0 has read the previous window's match info
// (an LDS flag, MISC_PF) -- so nothing needs barrier X.  Measured K1 10.12 -> 9.70 ms at level 3,
// 7.52 -> 7.21 ms at level 1 (profiles/r06k_one_barrier_ab.json; the first version, every wave
// deciding its own top from an extra info, was slower: 10.50 ms)
#ifndef ZH_ONE_BARRIER
#define ZH_ONE_BARRIER 1
#endif
static_assert(!ZH_ONE_BARRIER || ZH_LIT_INS, "one barrier per step needs the literals on the inserters");
constexpr u32 K1_LDS = OFF_LB + 4 * LB_WORDS * LB_BUFS;
constexpr u32 ML_LO = 11, ML_LEN = 22, ML_OFF = 29, ML_CUM = 45;  // match-list entry: start [0, 11) | ...
constexpr u32 MISC_WNM = 0;   // misc[par]: matches of the window of that parity (its match list's length)
constexpr u32 MISC_ARR = 12;  // misc[12]: worker-wave barrier arrivals (cumulative)
constexpr u32 MISC_PF = 12;   // (ZH_ONE_BARRIER, no arrivals) misc[12]: k + 1 once wave 0 has read window k - 1's match info
constexpr u32 MISC_NM = 4;    // misc[4 + (j & 3)]: matches the parse took in window j (miss skip)
constexpr u32 MISC_ANY = 13;  // misc[13]: block_any's flag (0 between calls)
constexpr u32 MISC_SCAN = 2;  // misc[2]: the repeat scan's count
constexpr u32 MISC_XCH = 8;   // misc[8 + 2 (j & 1) + LONG]: inserter's resume check of miss-skip window j
                              // ((j + 1) << 1 | hit; 0 at the block's start)
constexpr u32 MISC_RESF = 14; // misc[14 + (j & 1)]: miss-skip window j resumed (its search is whole)
static_assert(K1_LDS <= 163840 - 256, "K1 LDS budget");
static_assert(OFF_TL % 16 == 0 && OFF_CI % 16 == 0 && OFF_HM % 16 == 0 && OFF_MISC % 4 == 0, "alignment");


// v_ffbl_b32 as the hardware computes it: the lowest set bit's index, 0xFFFFFFFF for 0 (ctz
// builtins add a select for the zero case)
__device__ __forceinline__ u32 ffbl_raw(u32 x) {
  u32 r;
  __asm__("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// K1's LDS: the dynamic area, which starts at LDS address K1_DYN (after lz_blocks' one static
// word; lz_blocks traps otherwise).  A constant base lets the compiler fold constant offsets into
// the ds instructions' offset fields (through the extern symbol every address costs a v_add of
// the symbol's link-time address).  (Address 0 is the LDS null pointer to the compiler.)
constexpr u32 K1_DYN = 16;
__device__ __forceinline__ u8 *k1_lds() { return (u8 *)(__attribute__((address_space(3))) u8 *)(uintptr_t)K1_DYN; }

// Perturbation builds only (-DZH_PAD_A/I/W=N, tools/variants.sh): N dependent VALU added to a
// phase, to see which phase's instructions set K1's time.  Never in the product build.
template <int N>
__device__ __forceinline__ void vpad(u32 x) {
  if constexpr (N > 0) {
#pragma unroll
    for (int i = 0; i < N; i++) __asm__ volatile("v_add_u32 %0, %0, %0" : "+v"(x));
  }
}
#ifndef ZH_PAD_A
#define ZH_PAD_A 0
#endif
#ifndef ZH_PAD_I
#define ZH_PAD_I 0
#endif
#ifndef ZH_PAD_W
#define ZH_PAD_W 0
#endif
#ifndef ZH_PAD_C
#define ZH_PAD_C 0
#endif
#ifndef ZH_PAD_L
#define ZH_PAD_L 0
#endif

// K1's workgroup barrier: LDS ordering only.  The waves exchange data through LDS alone; their
// global writes (records, literals, the next block's prefetch loads in flight) need no ordering
// inside the kernel, so the barrier does not wait for them (__syncthreads' workgroup fence waits
// for every outstanding global access -- the literal stores' write acknowledgements and the
// next block's prefetch -- before each barrier).
__device__ __forceinline__ void k1_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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

// Common prefix of in[p..] and in[c..], capped at ZH_MAX_MATCH, for lanes `act` whose first 8
// bytes match (other lanes: any value).  Bytes 8.. are compared as dwords, 16 bytes per step
// with the step's loads issued together, until no active lane still matches; bytes past the
// block end read LDS padding / tables and are cut off by n - p later.
__device__ __forceinline__ u32 ext8(const u32 *in32, u32 p, u32 c, bool act) {
  constexpr u32 NW = ZH_MAX_MATCH / 4;  // dwords of a capped match
  constexpr u32 H = 4;                  // dwords per step: 16 bytes, early exit (a whole-match batch
                                        // of loads costs more LDS time than it saves in latency)
  u32 const wp = p >> 2, sp = p & 3, wq = c >> 2, sq = c & 3;
  u32 l = ZH_MAX_MATCH;
#pragma unroll
  for (u32 k0 = 2; k0 < NW; k0 += H) {
    if (!__ballot(act && l == ZH_MAX_MATCH)) break;
    u32 A[H + 1], B[H + 1];
#pragma unroll
    for (u32 k = 0; k <= H; k++) { A[k] = in32[wp + k0 + k]; B[k] = in32[wq + k0 + k]; }
    // the step's first differing bit: min over its dwords of ffbl(x) | 32 k (ffbl < 32 leaves the
    // dword's bits free; an equal dword's ffbl is 0xFFFFFFFF and stays above every difference)
    u32 const HK = NW - k0 < H ? NW - k0 : H;  // dwords compared in this step (constant once unrolled)
    u32 m = ~0u;
#pragma unroll
    for (u32 k = 0; k < H; k++) {
      if (k >= HK) continue;
      u32 const x = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sp) ^ __builtin_amdgcn_alignbyte(B[k + 1], B[k], sq);
      m = min(m, ffbl_raw(x) | 32u * k);
    }
    u32 const lh = m >= 32u * HK ? (u32)ZH_MAX_MATCH : 4u * k0 + (m >> 3);
    l = l == ZH_MAX_MATCH ? lh : l;
  }
  return l;
}

template <bool LONG>
__device__ __forceinline__ u32 hash_of(u32 lo, u32 hi) {
  return LONG ? hash_long(lo, hi) : hash_short(lo, hi);
}

#ifdef ZH_INS_CHECK
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
#endif

// Inserter wave: the tiles of window [wsb, we) against one table (u16 entries = position
// + 1).  Lane l handles positions tb + l + 64k of each tile; a tile's lookups are issued
// before its stores and after the previous tile's stores (program order = LDS order within a
// wave).  Stores of later k / later tiles carry later positions and land later; lanes of ONE
// store that hit the same slot leave the highest lane's value on gfx950 (the LDS services a
// wave64 store's lanes in ascending groups, each group's same-address lanes in lane order), i.e.
// the latest position, as in the oracle's serial loop.  Every K1 parity test depends on that
// order; -DZH_INS_CHECK builds a read-back of every lane's slot and a repair path
// (insert_repair) that make the tables independent of it (measured: no repair ever taken;
// K1 11.16 ms without the read-back vs 11.27 with it, profiles/r05i_k1_perturbation.json).
// BT tiles are issued per LDS round trip together with the next batch's input dwords and the
// workers' arrival counter.  Candidates (position + 1, 0 = none) go to creg as u16 pairs.
// A lane's positions are 4-aligned apart (tiles and rows are multiples of 64), so its byte
// shift is lane & 3 and its dwords sit at one base + immediate offsets; positions past lim read
// bytes past the block (inside the staging area's pad and the tables: never inserted).
// One instantiation per table serves every window (code size: K1's hot loops compete for the
// instruction cache).  skip (a miss-skip window, orc_lz_parse_pre): after the first batch of
// ZH_SKIP_TILES tiles, on_check gets whether any of its positions has a candidate matching its
// first ZH_MIN_MATCH_LONG (long table) / ZH_MIN_MATCH_SHORT (short) bytes -- the oracle's "a match
// among the searched tiles" -- and returns whether the window's search resumes; if not, the rest
// of the window is neither looked up nor inserted and its candidates are never dumped.
template <bool LONG, typename Hook, typename Check>
__device__ __forceinline__ void insert_window(const u32 *in32, u16 *T, u32 wsb, u32 lim, u32 lane, u32 (&creg)[NCR], const u32 *arrivals,
                                              Hook &&between_tiles, Check &&on_check, bool skip, u32 pmin) {
  // positions below pmin are already in T (a dictionary's precomputed tables): treated like
  // positions past lim (the junk slot, no candidate)
  constexpr u32 JUNK = LONG ? HL_SIZE : HS_SIZE;
  constexpr u32 BT = 2;  // tiles per LDS round trip
  constexpr u32 T0 = 0, NT = TILES;
  static_assert(TILES % BT == 0 && ZH_SKIP_TILES == BT, "batches tile windows; the resume check is the first batch");
  static_assert(ZH_TILE % 64 == 0 && ZH_WINDOW % 4 == 0, "a lane's positions share lane & 3");
  u32 const sh = lane & 3u;
  u32 wv[BT][TPL][3];
  auto load_in = [&](u32 tb0) {
    const u32 *const q = in32 + (tb0 >> 2) + (lane >> 2);
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++)
#pragma unroll
        for (u32 t = 0; t < 3; t++) wv[b][k][t] = q[(b * ZH_TILE + 64 * k) / 4 + t];
  };
  load_in(wsb + T0 * ZH_TILE);
#pragma unroll
  for (u32 t0 = T0; t0 < NT; t0 += BT) {
    // opaque per-batch copy of lim: keeps the compiler from hoisting every tile's
    // bounds checks (64 masks) to the top of the unrolled loop
    u32 lim_t;
    __asm__ volatile("v_mov_b32 %0, %1" : "=v"(lim_t) : "v"(lim));
    u32 const tb0 = wsb + t0 * ZH_TILE;
    u32 const p1 = tb0 + lane + 1u;  // the lane's first position of the batch, + 1
    u32 h[BT][TPL], e[BT][TPL], sa[BT][TPL];
    bool ok[BT][TPL];
#pragma unroll
    for (u32 b = 0; b < BT; b++) {
#pragma unroll
      for (u32 k = 0; k < TPL; k++) {
        u32 const q1 = p1 + b * ZH_TILE + 64 * k;  // position + 1: the stored value too
        u32 const lo = __builtin_amdgcn_alignbyte(wv[b][k][1], wv[b][k][0], sh), hi = __builtin_amdgcn_alignbyte(wv[b][k][2], wv[b][k][1], sh);
        u32 const hh = hash_of<LONG>(lo, hi);
        // LDS addresses: the store goes to the lookup's slot or the junk slot (one select)
        u32 const a = (u32)(uintptr_t)(T + hh);
        e[b][k] = *(const __attribute__((address_space(3))) u16 *)(uintptr_t)a;
        ok[b][k] = q1 <= lim_t && q1 > pmin;
        sa[b][k] = ok[b][k] ? a : (u32)(uintptr_t)(T + JUNK);
        h[b][k] = ok[b][k] ? hh : JUNK;  // (the check build's slot index)
      }
#pragma unroll
      for (u32 k = 0; k < TPL; k++) *(__attribute__((address_space(3))) u16 *)(uintptr_t)sa[b][k] = (u16)(p1 + b * ZH_TILE + 64 * k);
    }
#ifdef ZH_INS_CHECK
    u32 r[BT][TPL];
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++) r[b][k] = T[h[b][k]];
#endif
    if (t0 + BT < NT) load_in(tb0 + BT * ZH_TILE);
    vpad<ZH_PAD_I>(h[0][0]);
    u32 const arr = __atomic_load_n(arrivals, __ATOMIC_RELAXED);
#ifdef ZH_INS_CHECK
    bool lost = false;
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k++) lost |= h[b][k] != JUNK && r[b][k] < tb0 + b * ZH_TILE + 64 * k + lane + 1;
    if (__ballot(lost)) {
      if (lane == 0) atomicAdd(&g_fixups, 1u);
      insert_repair<LONG, BT>(T, tb0, lane, h, e);
    }
#endif
#pragma unroll
    for (u32 b = 0; b < BT; b++)
#pragma unroll
      for (u32 k = 0; k < TPL; k += 2) {
        u32 const c0 = ok[b][k] ? e[b][k] : 0u, c1 = ok[b][k + 1] ? e[b][k + 1] : 0u;
        u32 const ri = ((t0 + b) * TPL + k) / 2;
        creg[ri] = c0 | (c1 << 16);
        // materialise this batch's candidates now (otherwise the compiler sinks their
        // computation to the dump and keeps every tile's temporaries alive)
        __asm__ volatile("" : "+v"(creg[ri]) :: "memory");
      }
    if (t0 == 0 && skip) {
      bool v = false;
#pragma unroll
      for (u32 b = 0; b < BT; b++)
#pragma unroll
        for (u32 k = 0; k < TPL; k++) {
          // (the position's own bytes again from LDS: wv already holds the next batch's)
          u32 const p = tb0 + b * ZH_TILE + 64 * k + lane;
          u32 const c = ok[b][k] ? e[b][k] : 0u;
          u32 lo, hi, clo, chi;
          ld64u(in32, min(p, lim_t), lo, hi);
          ld64u(in32, c ? c - 1u : 0u, clo, chi);
          u32 const dx = (lo ^ clo) | ((hi ^ chi) & (LONG ? ~0u : 0xFFu));
          v |= c != 0 && dx == 0;
        }
      if (!on_check(__ballot(v) != 0)) {
        between_tiles(arr);
        break;
      }
    }
    between_tiles(arr);
  }
  __asm__ volatile("" ::: "memory");
}
// The next window's first position (lazy rule at this window's end): looked up after all of this
// window's tiles, before any of the next window's.
template <bool LONG>
__device__ __forceinline__ u32 lookahead(const u32 *in32, const u16 *T, u32 we, u32 lim, u32 lane) {
  u32 cwe = 0;
  if (lane < 2 && we + lane < lim) {  // (lane 1: we + 1, kept for the span-top rule)
    u32 lo, hi;
    ld64u(in32, we + lane, lo, hi);
    cwe = T[hash_of<LONG>(lo, hi)];
  }
  __asm__ volatile("" ::: "memory");
  return cwe;
}
struct NoCheck {
  __device__ bool operator()(bool) const { return true; }
};

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

// Miss skip (oracle orc_lz_parse_pre): window k of the block's loop searches only its first
// ZH_SKIP_TILES tiles when the parse took no match in window k - 3; windows before kskip0 (up to
// three past the one holding `pre`) never skip.  Wave-uniform.
__device__ __forceinline__ bool skip_window(const u32 *misc, u32 k, u32 kskip0) {
  return k >= kskip0 && (u32)__builtin_amdgcn_readfirstlane(__atomic_load_n(&misc[MISC_NM + ((k - 3) & 3)], __ATOMIC_RELAXED)) == 0;
}
// ... unless its first tiles found a match and the inserters resumed the whole window's search
// (decided while window k was inserted, in step k - 1; read by the workers after barrier P of
// step k -- the next write to that parity is window k + 2's, in step k + 1).
__device__ __forceinline__ bool skip_window_eff(const u32 *misc, u32 k, u32 kskip0) {
#ifdef ZH_NO_RESUME
  return skip_window(misc, k, kskip0);  // (A/B variant without the resume; not the oracle's rule)
#endif
  return skip_window(misc, k, kskip0) && (u32)__builtin_amdgcn_readfirstlane(__atomic_load_n(&misc[MISC_RESF + (k & 1)], __ATOMIC_RELAXED)) == 0;
}
// The two inserter waves' resume checks of miss-skip window j combined (mode 0: each table's wave
// sees only its own candidates).  Both reach this after their first batch of the window and
// before any barrier of the step, so neither waits on a wave held at a barrier.
template <bool LONG, bool TWO>
__device__ __forceinline__ bool resume_exchange(u32 *misc, u32 j, bool hit, u32 lane) {
  if constexpr (TWO) {
    u32 *const x = &misc[MISC_XCH + 2 * (j & 1)];
    if (lane == 0) __atomic_store_n(&x[LONG ? 1 : 0], ((j + 1) << 1) | (hit ? 1u : 0u), __ATOMIC_RELAXED);
    u32 v;
    for (;;) {
      v = (u32)__builtin_amdgcn_readfirstlane(__atomic_load_n(&x[LONG ? 0 : 1], __ATOMIC_RELAXED));
      if ((v >> 1) == j + 1) break;
      __builtin_amdgcn_s_sleep(1);
    }
    hit = hit || (v & 1u);
  }
  if (lane == 0) __atomic_store_n(&misc[MISC_RESF + (j & 1)], hit ? 1u : 0u, __ATOMIC_RELAXED);
  return hit;
}

// Incompressibility probe (oracle orc_lz_parse_pre): at the top of loop step kprobe (the
// parses of the ZH_PROBE_WINDOWS probe windows from the one holding `pre` are done) a block
// whose parse took no match in them stops -- it takes no sequences, every byte is a literal.
// Wave-uniform; every wave (inserters too) evaluates it at the same step, before barrier P.
// With ZH_PROBE_WINDOWS = 1 the decision is taken one step earlier, from the take masks
// (probe_dead_tm below), and this check never fires.
__device__ __forceinline__ bool probe_dead(const u32 *misc, u32 k, u32 kprobe) {
  if (ZH_PROBE_WINDOWS == 1 || k != kprobe) return false;
  u32 m = 0;
#pragma unroll
  for (u32 j = 1; j <= ZH_PROBE_WINDOWS; j++) m |= __atomic_load_n(&misc[MISC_NM + ((k - 1 - j) & 3)], __ATOMIC_RELAXED);
  return (u32)__builtin_amdgcn_readfirstlane(m) == 0;
}
static_assert(ZH_PROBE_WINDOWS >= 1 && ZH_PROBE_WINDOWS <= 3, "probe windows fit the match-count ring");
// Span tops of a window's worker waves (ZH_ONE_BARRIER, modes 0-1): the last position 64 hi - 1 of
// a span whose next position belongs to another wave -- hi = r_hi of waves 1..NWW-2, or 1..RS-1 in
// a miss-skip window -- takes its match under the lazy rule only with the next position's info,
// which its own wave never sees.  Lane L (< 32) decides the top at hi = L + 1 from the window's
// match info ci (length wn).
constexpr u32 span_top_mask(u64 tab) {
  u32 m = 0, hi = 0;
  for (u32 w = 1; w + 1 < INS_TID / 64; w++) {
    hi += (u32)((tab >> (2 * w)) & 3u);
    m |= 1u << hi;
  }
  return m;
}
__device__ __forceinline__ bool span_top_dec(const u32 *ci, u32 wn, bool skip, u32 L, bool act) {
  constexpr u32 TOPS_FULL = span_top_mask(ROUND_TAB), TOPS_SKIP = ((1u << (2 * ZH_SKIP_TILES)) - 1u) & ~1u;
  u32 const hi = L + 1, i = 64 * hi - 1;
  bool const top = act && L < NROUND && (((skip ? TOPS_SKIP : TOPS_FULL) >> hi) & 1u) && i < wn;
  u32 const inf = top ? ci[cidx(i)] : 0u, inf1 = top ? ci[cidx(i + 1)] : 0u;
  return top && (inf & 255u) && (inf1 & 255u) <= (inf & 255u);  // (take_rule of modes 0-1)
}
// The one-window probe from the take masks: before any match the parse visits every position,
// so it takes a match in the probe window exactly when the window has a take bit at or after
// its first parsed position e0.  Window k - 1's masks (and their span-top bits, set after
// barrier X of step k - 1) are final at barrier P of step k = kprobe - 1, so every wave --
// inserters too -- tests them right after that P and leaves the window loop together.
__device__ __forceinline__ bool probe_dead_tm(u32 k, u32 kprobe, u32 e0, bool lazy = false, u32 wnp = 0) {
  if (ZH_PROBE_WINDOWS != 1 || k + 1 != kprobe) return false;
  u8 *const smem = k1_lds();
  u32 lane;
  __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const u64 *const tmP = (const u64 *)(smem + OFF_HM) + ((k & 1u) ^ 1u) * NROUND;
  u32 const r = lane & (NROUND - 1);
  u64 m = tmP[r];
  if (ZH_ONE_BARRIER && lazy) {
    // (the span tops of the probe window, never a miss-skip window: decided here by every wave)
    const u32 *const ciP = (const u32 *)(smem + OFF_CI) + ((k & 1u) ^ 1u) * CI_WORDS;
    m |= span_top_dec(ciP, wnp, false, r, lane < NROUND) ? 1ull << 63 : 0ull;
  }
  u32 const lo = 64 * r;
  u64 const keep = e0 <= lo ? ~0ull : e0 >= lo + 64 ? 0ull : ~0ull << (e0 - lo);
  return __ballot(lane < NROUND && (m & keep) != 0) == 0;
}

// Dump an inserter's candidates into its half of the cinfo words (LONG: low half).
template <bool LONG, u32 NT>
__device__ __forceinline__ void dump_window(u8 *ci8, u32 lane_, const u32 (&creg)[NCR], u32 cwe) {
  // opaque lane copy: stops the 64 addresses from being hoisted out of the window loop
  u32 lane;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane_));
#pragma unroll
  for (u32 t = 0; t < NT; t++) {
#pragma unroll
    for (u32 k = 0; k < TPL; k++) {
      u32 const i = t * ZH_TILE + 64 * k + lane, j = t * TPL + k;
      u16 const v = (u16)(creg[j / 2] >> (16 * (j & 1)));
      *(u16 *)(ci8 + 4 * cidx(i) + (LONG ? 0 : 2)) = v;
    }
  }
  if (lane < 2) *(u16 *)(ci8 + 4 * cidx(ZH_WINDOW + lane) + (LONG ? 0 : 2)) = (u16)cwe;
}

// v from lane `src` (< 64) of the wave: ds_bpermute on a byte address, no lane-base math
__device__ __forceinline__ u32 bperm(u32 v, u32 src) { return (u32)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v); }
__device__ __forceinline__ u32 ctz64(u64 v) { return (u32)__builtin_ctzll(v); }
// bits [a, b) of a u32, 0 <= a <= b <= 32
__device__ __forceinline__ u32 bit_range32(u32 a, u32 b) {
  u32 const hi = b >= 32 ? ~0u : (1u << b) - 1u;
  return hi & ~((1u << a) - 1u);
}

// ---- the parse step rule ---------------------------------------------------------------------
// Match info words: off << 8 | len (off < 2^16).
// The serial parse at a position with a match (inf) takes it unless the match at the next
// position is longer (modes 0, 1: the lazy-1 check of levels 2-4) -- mode 2 (level 1) is greedy.
template <u32 MODE>
__device__ __forceinline__ bool take_rule(u32 inf, u32 inf1) {
  if (MODE == 2) return true;
  return (inf1 & 255u) <= (inf & 255u);
}
// modes 1, 2 search the short table only
template <u32 MODE>
constexpr bool two_tables() { return MODE == 0; }

// The 4 bytes in[a-4, a) (a >= 1; bytes before the buffer start read as 0s shifted out)
__device__ __forceinline__ u32 ld4_before(const u32 *in32, u32 a) {
  u32 const t = a >= 4 ? a - 4 : 0u, w = t >> 2, sh = t & 3;
  u32 const v = __builtin_amdgcn_alignbyte(in32[w + 1], in32[w], sh);
  return a >= 4 ? v : v << (8 * (4 - a));
}
// ---- match lengths, lanes = positions -------------------------------------------------------
// A worker wave takes a span of consecutive 64-position rounds in three passes:
//  A  (rounds high to low) per position and candidate the common prefix of the first 8 bytes
//     and whether p+1's candidate continues p's (then lcp(p) = 1 + lcp(p+1)); chain ends
//     with 8 matching bytes go to the wave's extension queue (flushed 64 at a time);
//  B  the queued chain ends extended, lanes = queue entries, results into their cinfo byte;
//  C  (rounds high to low) lengths from the chain structure -> match info in place.
constexpr u32 MAX_RW = 3;   // rounds per worker wave
// Rounds (64-position segments) of worker wave w in a window's length phase: waves 1..13
// (wave 0 parses).  A CU's waves go to SIMDs by wave id mod 4 and the length phase saturates
// VALU issue, so every SIMD gets 8 rounds -- SIMD 0 beside wave 0's parse, SIMD 1 beside wave
// 1's records and wave 13's lookahead, SIMDs 2 and 3 beside an inserter each -- with the older
// wave of a SIMD taking 3 (issue goes to the oldest ready wave, so a SIMD's youngest wave
// finishes last).  Measured (C3 mix, K1 per launch, one box): per-SIMD 9/11/6/6 rounds 12.30 ms,
// 9/9/7/7 11.86, 8/9/8/7 11.73, 8/8/8/8 11.61, 8/7/8/9 12.29 (round 4).  Round 5, SIMD 1's waves
// 1/5/9/13 (13 also computes the window's lookahead): 2/2/2/2 10.69 ms, 2/3/2/1 10.38, 1/3/3/1
// 10.37, 2/2/3/1 10.37; moving rounds between SIMDs or 4-round waves (a larger unrolled span)
// measured slower (`profiles/r05z_round_table_ab.json`).
__device__ __forceinline__ u32 rounds_of(u32 w) {
#ifdef ZH_RTAB
  return (u32)(((unsigned long long)(ZH_RTAB) >> (2 * w)) & 3u);
#else
  return (u32)((ROUND_TAB >> (2 * w)) & 3u);
#endif
}

// Pass B: extend queue entries [0, k) (k <= 64) of xq, one per lane; the extension (<= 64)
// goes to byte 0 (long candidate) or byte 2 (short) of the position's cinfo word.
__device__ __forceinline__ void xq_flush(const u32 *in32, u32 *ci, const u16 *xq, u32 k, u32 wsb, u32 lane) {
  bool const act = lane < k;
  u32 const e = act ? xq[lane] : 0u;
  u32 const i = e & 0x1FFFu, sh = (e >> 15) * 16u;
  u32 const c = (ci[cidx(i)] >> sh) & 0xFFFFu;
  u32 const x = ext8(in32, act ? wsb + i : 0u, act && c ? c - 1u : 0u, act);
  if (act) ((u8 *)ci)[4 * cidx(i) + (sh >> 3)] = (u8)x;
}

// Flags of a position after pass A
enum : u32 { LF_FL = 1u << 8, LF_FS = 1u << 9, LF_XL = 1u << 10, LF_XS = 1u << 11, LF_SL = 1u << 12 };

// The match lengths of rounds [r_lo, r_hi) (r_hi - r_lo <= MAX_RW): candidates in cinfo ->
// match info (off << 8 | len, 0 = none) in place.  Semantics of oracle/zstd_oracle.c
// orc_lz_match_info: lcp capped at ZH_MAX_MATCH and at the block end, long candidates from 8
// bytes, short from 5, the longer (long on ties).  Then per position whether the parse takes its
// match if it gets there (take_rule on the next positions' info: DPP within the round, the
// round above by carry; la1 = the position above the span when it is the window's
// top one) -> the rounds' take masks tm.  At the top of a span that is not the window's top the next positions
// belong to another wave: those take bits stay clear until the wave decides them after barrier X.
template <u32 MODE>
__device__ __forceinline__ void span_lengths(const u32 *in32, u32 *ci, u64 *tm, u16 *xq, u32 r_lo, u32 r_hi, u32 wsb, u32 we, u32 n, u32 lim,
                                             u32 lane, bool top, u32 la1) {
  constexpr bool TWO = two_tables<MODE>();
  u32 cwr[MAX_RW], flg[MAX_RW];
  // pass A, rounds high to low: a round's candidates, own bytes and candidate bytes are loaded
  // at the top of the round (hoisting every round's loads to the top of the pass was slower:
  // the longer LDS bursts delay the inserter waves, which are on the step's critical path)
  u32 olo[MAX_RW], ohi[MAX_RW], Lw[MAX_RW][3], Sw[MAX_RW][3];
  auto loadA = [&](u32 k) {
    u32 const r = r_hi - 1 - min(k, r_hi - 1 - r_lo), i = 64 * r + lane, p = wsb + i;  // (rounds past the span: repeat the last)
    // (positions at or past lim -- which covers we -- have no candidates: the inserters left 0)
    u32 const cw = ci[cidx(i)];
    cwr[k] = cw;
    ld64u(in32, p, olo[k], ohi[k]);
    // the candidates' positions (c - 1) mod 2^16, without a select: an empty candidate reads
    // position 65535's bytes (inside the staging area and its pad), and its prefix is never used --
    // a match needs a nonempty candidate, and no chain passes through an empty one (its successor
    // would need candidate 0 + 1 to continue it ... from a candidate of -1)
    u32 const aL = ((cw - 1u) & 0xFFFFu) >> 2, aS = ((cw >> 16) + 0xFFFFu) >> 2 & 0x3FFFu;
#pragma unroll
    for (u32 t = 0; t < 3; t++) {
      if constexpr (TWO) Lw[k][t] = in32[aL + t];
      Sw[k][t] = in32[aS + t];
    }
  };
  u32 ccL = 0, ccS = 0;  // candidates of the position above the round being processed
  u32 nq = 0;            // queued entries (wave-uniform)
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) {
    flg[k] = 0;
    if (r_lo + k >= r_hi) { cwr[k] = 0; continue; }
    loadA(k);
    u32 const r = r_hi - 1 - k, i = 64 * r + lane;
    u32 const cw = cwr[k];
    u32 const cL = TWO ? cw & 0xFFFFu : 0u, cS = cw >> 16;
    // common prefix (0..8) of the position's 8 bytes with the candidate's; for an empty candidate
    // any value (see loadA): ctz64 of the difference as min(ffbl(x), min(ffbl(y), 32) + 32)
    auto pref = [&](u32 c, const u32 (&w)[3]) {
      u32 const sh = (c - 1u) & 3u;
      u32 const x = olo[k] ^ __builtin_amdgcn_alignbyte(w[1], w[0], sh), y = ohi[k] ^ __builtin_amdgcn_alignbyte(w[2], w[1], sh);
      return min(ffbl_raw(x), min(ffbl_raw(y), 32u) + 32u) >> 3;
    };
    u32 const pL = TWO ? pref(cL, Lw[k]) : 0u, pS = pref(cS, Sw[k]);
    vpad<ZH_PAD_A>(pS);
    u32 cLn = wave_shl1(cL), cSn = wave_shl1(cS);
    cLn = lane == 63 ? ccL : cLn;
    cSn = lane == 63 ? ccS : cSn;
    bool const fL = pL == 8 && cLn == cL + 1u, fS = pS == 8 && cSn == cS + 1u;
    bool const xL = pL == 8 && !fL;
    bool const sL = cS == cL && xL && pS == 8 && !fS;  // S takes L's extension
    bool const xS = pS == 8 && !fS && !sL;
    flg[k] = pL | (pS << 4) | (fL ? LF_FL : 0u) | (fS ? LF_FS : 0u) | (xL ? LF_XL : 0u) | (xS ? LF_XS : 0u) | (sL ? LF_SL : 0u);
    ccL = lane_value(cL, 0);
    ccS = lane_value(cS, 0);
    // queue the chain ends to extend (L then S), flushing 64 at a time from the top
    u64 const bL = TWO ? __ballot(xL) : 0ull, bS = __ballot(xS);
    u32 const rL = __builtin_amdgcn_mbcnt_hi((u32)(bL >> 32), __builtin_amdgcn_mbcnt_lo((u32)bL, 0u));
    u32 const rS = __builtin_amdgcn_mbcnt_hi((u32)(bS >> 32), __builtin_amdgcn_mbcnt_lo((u32)bS, 0u));
    u32 const nL = (u32)__popcll(bL);
    // branch-free stores: lanes without an entry write the wave's spare slot (never read)
    xq[xL ? nq + rL : XQ_CAP - 1] = (u16)i;
    xq[xS ? nq + nL + rS : XQ_CAP - 1] = (u16)(i | 0x8000u);
    nq = (u32)__builtin_amdgcn_readfirstlane(nq + nL + (u32)__popcll(bS));
    while (nq >= 64) {
      nq -= 64;
      xq_flush(in32, ci, xq + nq, 64, wsb, lane);
    }
  }
  if (nq) xq_flush(in32, ci, xq, nq, wsb, lane);
  // pass C.  C1: every round's chain lengths without the carry (the ds_bpermutes of all rounds
  // in flight together); C2, rounds high to low: lanes whose chain runs past the round take the
  // carry, then the match info and the take decision.
  u32 lLr[MAX_RW], lSr[MAX_RW], runs[MAX_RW];
  auto c1 = [&](u32 k) {
    u32 const r = r_hi - 1 - min(k, r_hi - 1 - r_lo), i = 64 * r + lane;
    u32 const f = flg[k];
    u32 const ce = ci[cidx(i)];
    u32 const pL = f & 15u, pS = (f >> 4) & 15u;
    u32 const eL = (f & LF_XL) ? (ce & 255u) : pL;
    u32 const eS = (f & LF_XS) ? ((ce >> 16) & 255u) : ((f & LF_SL) ? eL : pS);
    u64 const RS = __ballot(!(f & LF_FS)) >> lane;
    u32 const qS = RS ? ctz64(RS) : 64u - lane;
    u32 const vS = bperm(eS, min(lane + qS, 63u));
    lSr[k] = RS ? min((u32)ZH_MAX_MATCH, qS + vS) : qS;  // (a chain running past: + carry in C2)
    runs[k] = RS ? 0u : 2u;
    if constexpr (TWO) {
      u64 const RL = __ballot(!(f & LF_FL)) >> lane;
      u32 const qL = RL ? ctz64(RL) : 64u - lane;
      u32 const vL = bperm(eL, min(lane + qL, 63u));
      lLr[k] = RL ? min((u32)ZH_MAX_MATCH, qL + vL) : qL;
      runs[k] |= RL ? 0u : 1u;
    } else {
      lLr[k] = 0;
    }
  };
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) c1(k);
  u32 clL = 0, clS = 0;  // lcps of the position above the round
  u32 cv1 = la1;         // info of the position above the round
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) {
    if (r_lo + k >= r_hi) continue;
    u32 const r = r_hi - 1 - k, i = 64 * r + lane, p = wsb + i;
    u32 const cw = cwr[k];
    u32 const cL = TWO ? cw & 0xFFFFu : 0u, cS = cw >> 16;
    u32 const lL = (runs[k] & 1u) ? min((u32)ZH_MAX_MATCH, lLr[k] + clL) : lLr[k];
    u32 const lS = (runs[k] & 2u) ? min((u32)ZH_MAX_MATCH, lSr[k] + clS) : lSr[k];
    vpad<ZH_PAD_C>(lS);
    clL = lane_value(lL, 0);
    clS = lane_value(lS, 0);
    u32 const capj = min((u32)ZH_MAX_MATCH, n - min(p, n));
    u32 const rL = min(lL, capj), rS = min(lS, capj);
    u32 const mL = (cL && rL >= ZH_MIN_MATCH_LONG) ? rL : 0u;
    u32 const mS = (cS && rS >= ZH_MIN_MATCH_SHORT) ? rS : 0u;
    bool const useL = mL && mL >= mS;
    u32 const ml = useL ? mL : mS, cm = useL ? cL : cS;
    u32 const v = ml ? ((p - (cm - 1u)) << 8) | ml : 0u;
    u32 v1 = wave_shl1(v);
    v1 = lane == 63 ? cv1 : v1;
    cv1 = lane_value(v, 0);
    bool const unk = MODE != 2 && k == 0 && !top && lane == 63;
    bool const tk = v != 0 && !unk && take_rule<MODE>(v, v1);
    ci[cidx(i)] = v;
    u64 const tb = __ballot(tk);
    if (lane == 0) tm[r] = tb;
  }
}

// ---- level 1 (mode 2): lengths at every ZH_L1_STRIDE-th position ------------------------------
// Oracle orc_lz_parse_pre with orc_lz_mode 2: only positions p = 0 mod S of the staged buffer take
// a match (the short table still holds every position).  Round r of a window covers positions
// 64 S r + S lane; along same-offset chains (the candidate of p + S is the candidate of p plus S)
// lcp(p) = S + lcp(p + S), so pass C's chain distance counts S bytes per lane.  Greedy: the take
// mask is the nonzero match info, spread to every S-th bit of the window's 64-position mask words.
constexpr u32 L1_S = ZH_L1_STRIDE;
constexpr u32 NROUND1 = NROUND / L1_S;  // length rounds per window
static_assert(L1_S == 1 || L1_S == 2 || L1_S == 4, "level-1 stride");
// 64-bit take ballot of a round -> the S mask words of its 64 S positions (bit j -> bit S j)
__device__ __forceinline__ u64 spread_bits(u64 v, u32 s) {
  if (s == 2) {
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
  } else if (s == 4) {
    v = (v | (v << 24)) & 0x000000FF000000FFull;
    v = (v | (v << 12)) & 0x000F000F000F000Full;
    v = (v | (v << 6)) & 0x0303030303030303ull;
    v = (v | (v << 3)) & 0x1111111111111111ull;
  }
  return v;
}
__device__ __forceinline__ void span_lengths_l1(const u32 *in32, u32 *ci, u64 *tm, u16 *xq, u32 r_lo, u32 r_hi, u32 wsb, u32 n, u32 lane) {
  constexpr u32 S = L1_S;
  u32 cwr[MAX_RW], flg[MAX_RW], olo[MAX_RW], ohi[MAX_RW], Sw[MAX_RW][3];
  auto loadA = [&](u32 k) {
    u32 const r = r_hi - 1 - min(k, r_hi - 1 - r_lo), i = 64 * S * r + S * lane, p = wsb + i;
    u32 const cw = ci[cidx(i)];
    cwr[k] = cw;
    ld64u(in32, p, olo[k], ohi[k]);
    u32 const aS = ((cw >> 16) + 0xFFFFu) >> 2 & 0x3FFFu;  // (an empty candidate: see span_lengths)
#pragma unroll
    for (u32 t = 0; t < 3; t++) Sw[k][t] = in32[aS + t];
  };
  u32 ccS = 0, nq = 0;
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) {
    flg[k] = 0;
    if (r_lo + k >= r_hi) { cwr[k] = 0; continue; }
    loadA(k);
    u32 const r = r_hi - 1 - k, i = 64 * S * r + S * lane;
    u32 const cS = cwr[k] >> 16;
    u32 const sh = (cS - 1u) & 3u;
    u32 const x = olo[k] ^ __builtin_amdgcn_alignbyte(Sw[k][1], Sw[k][0], sh), y = ohi[k] ^ __builtin_amdgcn_alignbyte(Sw[k][2], Sw[k][1], sh);
    u32 const pS = min(ffbl_raw(x), min(ffbl_raw(y), 32u) + 32u) >> 3;
    u32 cSn = wave_shl1(cS);
    cSn = lane == 63 ? ccS : cSn;
    bool const fS = pS == 8 && cSn == cS + S;
    bool const xS = pS == 8 && !fS;
    flg[k] = (pS << 4) | (fS ? LF_FS : 0u) | (xS ? LF_XS : 0u);
    ccS = lane_value(cS, 0);
    u64 const bS = __ballot(xS);
    u32 const rS = __builtin_amdgcn_mbcnt_hi((u32)(bS >> 32), __builtin_amdgcn_mbcnt_lo((u32)bS, 0u));
    xq[xS ? nq + rS : XQ_CAP - 1] = (u16)(i | 0x8000u);
    nq = (u32)__builtin_amdgcn_readfirstlane(nq + (u32)__popcll(bS));
    while (nq >= 64) {
      nq -= 64;
      xq_flush(in32, ci, xq + nq, 64, wsb, lane);
    }
  }
  if (nq) xq_flush(in32, ci, xq, nq, wsb, lane);
  u32 lSr[MAX_RW], runs[MAX_RW];
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) {
    u32 const r = r_hi - 1 - min(k, r_hi - 1 - r_lo), i = 64 * S * r + S * lane;
    u32 const f = flg[k];
    u32 const ce = ci[cidx(i)];
    u32 const eS = (f & LF_XS) ? ((ce >> 16) & 255u) : ((f >> 4) & 15u);
    u64 const RS = __ballot(!(f & LF_FS)) >> lane;
    u32 const qS = RS ? ctz64(RS) : 64u - lane;
    u32 const vS = bperm(eS, min(lane + qS, 63u));
    lSr[k] = RS ? min((u32)ZH_MAX_MATCH, S * qS + vS) : S * qS;
    runs[k] = RS ? 0u : 2u;
  }
  u32 clS = 0;
#pragma unroll
  for (u32 k = 0; k < MAX_RW; k++) {
    if (r_lo + k >= r_hi) continue;
    u32 const r = r_hi - 1 - k, i = 64 * S * r + S * lane, p = wsb + i;
    u32 const cS = cwr[k] >> 16;
    u32 const lS = (runs[k] & 2u) ? min((u32)ZH_MAX_MATCH, lSr[k] + clS) : lSr[k];
    clS = lane_value(lS, 0);
    u32 const capj = min((u32)ZH_MAX_MATCH, n - min(p, n));
    u32 const rS = min(lS, capj);
    u32 const mS = (cS && rS >= ZH_MIN_MATCH_SHORT) ? rS : 0u;
    u32 const v = mS ? ((p - (cS - 1u)) << 8) | mS : 0u;
    ci[cidx(i)] = v;
    u64 const tb = __ballot(v != 0);
    if (lane == 0) {
#pragma unroll
      for (u32 s = 0; s < S; s++) tm[S * r + s] = S == 1 ? tb : spread_bits((tb >> (64 / S * s)) & ((1ull << (64 / S)) - 1ull), S);
    }
  }
}
// Rounds of worker wave w in a level-1 window (NROUND1 = 16 over waves 1..13; SIMDs 2 and 0,
// whose fourth wave is the idle long-table inserter / the parse, take the extra rounds)
constexpr u64 ROUND_TAB1 = 0x5556664ull;  // 2 bits per wave: 0 1 2 1 2 1 2 1 1 1 1 1 1 1
static_assert(L1_S != 2 || (((ROUND_TAB1 >> 2) & 3) + ((ROUND_TAB1 >> 4) & 3) + ((ROUND_TAB1 >> 6) & 3) + ((ROUND_TAB1 >> 8) & 3) +
                            ((ROUND_TAB1 >> 10) & 3) + ((ROUND_TAB1 >> 12) & 3) + ((ROUND_TAB1 >> 14) & 3) + ((ROUND_TAB1 >> 16) & 3) +
                            ((ROUND_TAB1 >> 18) & 3) + ((ROUND_TAB1 >> 20) & 3) + ((ROUND_TAB1 >> 22) & 3) + ((ROUND_TAB1 >> 24) & 3) +
                            ((ROUND_TAB1 >> 26) & 3)) == NROUND1, "level-1 round table covers the window");
template <u32 MODE>
__device__ __forceinline__ u32 rounds_of_mode(u32 w) {
  if constexpr (MODE == 2 && L1_S == 2) {
#ifdef ZH_RTAB1
    return (u32)(((unsigned long long)(ZH_RTAB1) >> (2 * w)) & 3u);
#else
    return (u32)((ROUND_TAB1 >> (2 * w)) & 3u);
#endif
  } else if constexpr (MODE == 2 && L1_S == 4) {
    return w >= 1 && w <= 8 ? 1u : 0u;
  } else {
    return rounds_of(w);
  }
}

// Match info of one position from scratch (the lookahead positions `we`, `we + 1` of the
// next window, which the next window's rounds compute again): c = candidate word.
template <u32 MODE>
__device__ __forceinline__ u32 info_one(const u32 *in32, u32 p, u32 cw, u32 n, u32 lim, bool act) {
  bool const hv = act && p < lim;
  u32 const cL = (hv && two_tables<MODE>()) ? (cw & 0xFFFFu) : 0u, cS = hv ? (cw >> 16) : 0u;
  u32 lo, hi;
  ld64u(in32, hv ? p : 0u, lo, hi);
  u32 const tL = prefix8(in32, cL ? cL - 1u : 0u, lo, hi), tS = prefix8(in32, cS ? cS - 1u : 0u, lo, hi);
  u32 const pL = cL ? tL : 0u, pS = cS ? tS : 0u;
  u32 const e1 = ext8(in32, pL == 8 ? p : 0u, pL == 8 ? cL - 1u : 0u, pL == 8);
  u32 const e2 = ext8(in32, pS == 8 ? p : 0u, pS == 8 ? cS - 1u : 0u, pS == 8);
  u32 const lL = pL == 8 ? e1 : pL, lS = pS == 8 ? e2 : pS;
  u32 const capj = min((u32)ZH_MAX_MATCH, n - min(p, n));
  u32 const rL = min(lL, capj), rS = min(lS, capj);
  u32 const mL = (cL && rL >= ZH_MIN_MATCH_LONG) ? rL : 0u;
  u32 const mS = (cS && rS >= ZH_MIN_MATCH_SHORT) ? rS : 0u;
  bool const useL = mL && mL >= mS;
  u32 const ml = useL ? mL : mS, cm = useL ? cL : cS;
  return ml ? ((p - (cm - 1u)) << 8) | ml : 0u;
}

// ---- catch-up ----------------------------------------------------------------------------------
// Bytes a match at staged position P with offset off grows backwards (oracle orc_lz_parse_pre's
// catch-up): while P - e > lo and P - e > off and in[P-e-1] == in[P-e-1-off].  Compared four
// bytes at a time from the top byte down; at most a few steps.
__device__ __forceinline__ u32 catch_up(const u32 *in32, u32 P, u32 off, u32 lo, bool act) {
  u32 maxe = (act && P > lo && P > off) ? min(P - lo, P - off) : 0u;
  u32 e = 0;
  while (__ballot(e < maxe)) {
    if (e < maxe) {
      u32 const a = P - e, x = ld4_before(in32, a) ^ ld4_before(in32, a - off);
      u32 const m = x ? (u32)__builtin_clz(x) >> 3 : 4u;
      e += min(m, maxe - e);
      maxe = m < 4 ? e : maxe;
    }
  }
  return e;
}

// ---- the parse, lanes = segments --------------------------------------------------------------
// Walk of segment [S, SE) from position p by the lanes `act`: the take mask tmk names the
// positions where the parse takes a match once it gets there, so every step is one run of
// literals (the positions before the next take bit) and the match after it.  LM / MM: the
// segment's literal and match-start bits, ex: the exit (first position >= SE).  With old
// visited bits (a Jacobi re-walk from a new entry), the walk stops where it meets a position
// the old walk visited -- from there on both are the same -- and keeps the old bits above it.
template <bool REWALK, typename LenQ>
__device__ __forceinline__ void seg_walk(LenQ &&lenq, u32 tmk, u32 S, u32 SE, u32 p, bool act0, u32 &LM, u32 &MM, u32 &ex) {
  // (the first walk has no old trajectory: REWALK = false drops the merge test from the step)
  u32 const old = (REWALK && act0) ? (LM | MM) : 0u;
  vpad<ZH_PAD_W>(p);
  u32 nl = 0, nm = 0;
  bool act = act0 && p < SE, merged = false;
  u32 mpos = 0;
  if constexpr (!REWALK) {
    // the first walk: the shortest dependent chain per step (shift, ctz, the length's LDS read,
    // add); a lane's state stops changing once it leaves the segment.  (Round 4: the first walk
    // through the re-walk's step, with its merge test, cost wave 0 191 k cycles per block for
    // walk + Jacobi, this one 161 k; K1 11.75 -> 11.50 ms.)
    while (__ballot(act)) {
      u32 const o = p - S;                          // (< 32 on active lanes)
      u32 const q = p + __builtin_ctzg(tmk >> o, 32);  // next take position (>= SE: none)
      bool const st = act && q < SE;
      u32 const len = lenq(q);                      // (q <= S + 63; used only when q < SE)
      nl |= act ? bit_range32(o, min(q, SE) - S) : 0u;
      nm |= st ? 1u << (q - S) : 0u;
      p = act ? (st ? q + len : SE) : p;
      act = act && p < SE;
    }
    if (act0) {
      LM = nl;
      MM = nm;
      ex = p;
    }
    return;
  }
  // branch-free steps (selects, no exec-mask branches): each is one literal run and the
  // position after it, or the point where the walk meets the old one
  // (as the first walk's step; no take bit left: q >= SE, no old bit: x = p + 64 > q)
  while (__ballot(act)) {
    u32 const o = p - S;
    u32 const q = p + __builtin_ctzg(tmk >> o, 32);
    u32 const x = p + __builtin_ctzg(old >> o, 64);
    bool const mg = act && x <= q;
    bool const st = act && !mg && q < SE;
    u32 const re = mg ? x : min(q, SE);
    nl |= act ? bit_range32(o, re - S) : 0u;
    u32 const len = lenq(q);
    nm |= st ? 1u << (q - S) : 0u;
    mpos = mg ? x - S : mpos;
    merged = merged || mg;
    p = (act && !mg) ? (st ? q + len : SE) : p;
    act = act && !mg && p < SE;
  }
  if (act0) {
    if (merged) {
      u32 const keep = ~((1u << mpos) - 1u);
      LM = nl | (LM & keep);
      MM = nm | (MM & keep);
    } else {
      LM = nl;
      MM = nm;
      ex = p;
    }
  }
}

// Inserter wave main loop.  Step k of the workers (the lengths of window k, the parse and
// records of window k - 1, then its literals) opens with barrier P once window k's candidates
// are dumped into cinfo buffer k & 1, and the inserters then build window k + 1's candidates in
// registers.  They take the step's barrier X only once
// all 14 worker waves have arrived there (an LDS arrival counter), between two tiles, so the
// insertion spreads over the whole step.
constexpr u32 WIN_BARRIERS = 1;  // X
// The long table's wave in modes 1, 2 (the short table only): no insertion, only the step's two
// barriers (P, X) and the probe exit, so the workgroup's barrier sequence stays the same.
// Returns whether the loop ended at the incompressibility probe.
// Literal bytes of the window at staged position wsj (ZH_LIT_INS): rounds r = r0, r0 + rs, ... of
// 64 positions; lm = its literal bits per walk segment, lb = their exclusive prefix counts (+ the
// window's total at lb[NSEG]); nlit = the literals before the window.  Four rounds' LDS reads per
// round trip.
__device__ __forceinline__ void lit_rounds(const u8 *in, const u32 *lm, const u32 *lb, u8 *lit_out, u32 nlit, u32 wsj, u32 r0, u32 rs, u32 lane) {
  constexpr u32 B = 4;
  for (u32 rb = r0; rb < NROUND; rb += B * rs) {
    u64 mw[B];
    u32 lbr[B], by[B];
#pragma unroll
    for (u32 j = 0; j < B; j++) {
      u32 const r = min(rb + rs * j, NROUND - 1u);
      mw[j] = *(const u64 *)&lm[2 * r];
      lbr[j] = (u32)__builtin_amdgcn_readfirstlane(lb[2 * r]);
      by[j] = in[wsj + 64 * r + lane];
    }
#pragma unroll
    for (u32 j = 0; j < B; j++) __asm__ volatile("" : "+v"(by[j]));
#pragma unroll
    for (u32 j = 0; j < B; j++) {
      if (rb + rs * j >= NROUND) continue;
      u64 const m = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(mw[j] >> 32)) << 32) | (u32)__builtin_amdgcn_readfirstlane((u32)mw[j]);
      if ((m >> lane) & 1ull) {
        u32 const rank = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
        lit_out[nlit + lbr[j] + rank] = (u8)by[j];
      }
    }
  }
}
// The literal work of an inserter wave in step k (ZH_LIT_INS): window k - 3's rounds r0, r0 + rs, ...
struct LitJob {
  const u8 *in;
  u32 *sgm, *lbx;
  u8 *lit_out;
  u32 wstart, n, pre, r0, rs;
  u32 nlit;  // literals of the windows before the next one (running; every inserter keeps the total)
  __device__ __forceinline__ void step(u32 k, u32 lane) {
    if constexpr (ZH_LIT_INS) {
      if (k < 3) return;
      u32 const j = k - 3, wsj = wstart + j * ZH_WINDOW;
      if (wsj >= n || min(wsj + ZH_WINDOW, n) <= pre) return;
      const u32 *const lm = sgm + segm(j % LM_BUFS);
      const u32 *const lb = lbx + (j & 1u) * LB_WORDS;
      if (rs) lit_rounds(in, lm, lb, lit_out, nlit, wsj, r0, rs, lane);
      nlit += (u32)__builtin_amdgcn_readfirstlane(lb[NSEG]);
    }
  }
};
__device__ __forceinline__ bool idle_inserter_loop(u32 *misc_, u32 n, u32 wstart, u32 kprobe, u32 e0p, LitJob &lj, u32 lane, bool lazy) {
  u32 const nwin = (n - wstart + ZH_WINDOW - 1) / ZH_WINDOW;
  for (u32 k = 0; k < nwin + STEPS_EXTRA; k++) {
    if (probe_dead(misc_, k, kprobe)) return true;
    k1_barrier();  // P
    u32 const wsb = wstart + k * ZH_WINDOW;
    if (probe_dead_tm(k, kprobe, e0p, lazy, min(wsb, n) - (wsb - ZH_WINDOW))) return true;
    lj.step(k, lane);
    if (!ZH_ONE_BARRIER) k1_barrier();  // X
  }
  return false;
}
template <bool LONG, bool TWO>
__device__ __forceinline__ bool inserter_loop(const u32 *in32, u16 *T, u8 *ci8, u32 *misc_, u32 n, u32 lim, u32 lane, u32 *dbg, u32 wstart,
                                              u32 pmin, u32 span_s, u32 span_e, u32 kskip0, u32 kprobe, u32 e0p, LitJob &lj, bool lazy) {
  u32 creg[NCR];
  if (span_s < span_e) insert_span<LONG>(in32, T, span_s, span_e, lane);
  // (the first window: its own instantiation, with pmin and no barriers to take)
  insert_window<LONG>(in32, T, wstart, lim, lane, creg, &misc_[MISC_ARR], [](u32) {}, NoCheck{}, false, pmin);
  u32 cwe = lookahead<LONG>(in32, T, min(wstart + (u32)ZH_WINDOW, n), lim, lane);
  bool skipc = false;  // the window whose candidates creg holds is a miss-skip window (not resumed)
#ifdef ZH_STAMPS
  u32 st_ins = 0;
#endif
  u32 const nwin = (n - wstart + ZH_WINDOW - 1) / ZH_WINDOW;
  u32 passed = 0;  // X barriers taken so far
  TL_DECL;
  for (u32 k = 0; k < nwin + STEPS_EXTRA; k++) {
    if (probe_dead(misc_, k, kprobe)) return true;
    u32 const wsb = wstart + k * ZH_WINDOW;
    if (k < nwin) {
      if (ZH_ONE_BARRIER) {
        // buffer k & 1 held window k - 2's match info, which wave 0 read in step k - 1
        // (bounded: wave 0 sets the flag every step; the bound only keeps a bug from hanging the GPU)
        for (u32 it = 0; it < (1u << 22) && (u32)__builtin_amdgcn_readfirstlane(__atomic_load_n(&misc_[MISC_PF], __ATOMIC_RELAXED)) < k; it++)
          __builtin_amdgcn_s_sleep(1);
      }
      if (skipc) dump_window<LONG, ZH_SKIP_TILES>(ci8 + (k & 1u) * 4 * CI_WORDS, lane, creg, cwe);
      else dump_window<LONG, TILES>(ci8 + (k & 1u) * 4 * CI_WORDS, lane, creg, cwe);
    }
    TL_MARK(4);
    k1_barrier();  // P: candidates of window k in buffer k & 1
    TL_MARK(0);
    TL_STEP();
    if (probe_dead_tm(k, kprobe, e0p, lazy, min(wsb, n) - (wsb - ZH_WINDOW))) return true;
    u32 const done = passed + WIN_BARRIERS;
    // arr: the arrival counter as read with the last tile's read-back; a barrier taken
    // here means the counter is re-read for the next one
    auto take_ready = [&](u32 arr) {
      while (!ZH_ONE_BARRIER && passed < done && arr >= NWW * (passed + 1)) {
        k1_barrier();
        passed++;
        arr = __atomic_load_n(&misc_[MISC_ARR], __ATOMIC_RELAXED);
      }
    };
#ifdef ZH_STAMPS
    u64 const ti0 = __builtin_amdgcn_s_memtime();
#endif
    u32 const nx = wsb + ZH_WINDOW;
    // window k + 1: the parse of window k - 2 ended in step k - 1 (before this step's P)
    skipc = skip_window(misc_, k + 1, kskip0);
    if (k + 1 < nwin) {
#ifdef ZH_NO_RESUME
      bool const resumed = false;
      insert_window<LONG>(in32, T, nx, lim, lane, creg, &misc_[MISC_ARR], take_ready, [](bool) { return false; }, skipc, 0u);
#else
      // a miss-skip window's first tiles, then the rest of it if any of them found a match (both
      // inserters' checks combined before either takes a barrier)
      bool resumed = false;
      insert_window<LONG>(in32, T, nx, lim, lane, creg, &misc_[MISC_ARR], take_ready,
                          [&](bool h) { return resumed = resume_exchange<LONG, TWO>(misc_, k + 1, h, lane); }, skipc, 0u);
#endif
      if (resumed) skipc = false;
      cwe = lookahead<LONG>(in32, T, min(nx + ZH_WINDOW, n), lim, lane);
    }
#ifdef ZH_STAMPS
    st_ins += (u32)(__builtin_amdgcn_s_memtime() - ti0);
#endif
    TL_MARK(1);
    // window k - 3's literal bytes (their bits and prefix counts were final at X of step k - 1;
    // the next writes to those buffers come after P of step k + 1)
    lj.step(k, lane);
    TL_MARK(2);
    while (!ZH_ONE_BARRIER && passed < done) { k1_barrier(); passed++; }
    TL_MARK(3);
  }
  TL_FLUSH(LONG ? 14u : 15u, lane);
#ifdef ZH_STAMPS
  if (LONG && lane == 0) dbg[16] = st_ins;
#endif
  (void)dbg;
  return false;
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
// __syncthreads_or for the K1 workgroup: a flag word (0 between calls) raised by one lane per
// wave, read after a barrier and cleared between two more.  (The runtime's version computes the
// flat work-item id, whose entry VGPRs would then stay live -- spilled -- across the
// persistent block loop.)
__device__ __forceinline__ bool block_any(bool v, u32 *flag, u32 tid) {
  if (__ballot(v) && (tid & 63) == 0) atomicOr(flag, 1u);
  k1_barrier();
  bool const r = *flag != 0;
  k1_barrier();
  if (tid == 0) *flag = 0;
  k1_barrier();
  return r;
}

// The K1 thread index from the wave id w (an SGPR, read once) and the lane, recomputed at each
// use (opaque mbcnt): nothing from the kernel's entry VGPRs stays live, or spilled, across the
// persistent block loop.
__device__ __forceinline__ u32 k1_tid(u32 w) {
  u32 lane;
  __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  return (u32)((K1_WAVE_MAP >> (4 * w)) & 15u) << 6 | lane;
}

// Repeat scan (ZH_SCAN_*, oracle orc_repeat_scan), all 1024 threads, after the probe found no
// match: the hash tables' 64 KiB hold 2^ZH_SCAN_LOG u32 slots; positions q = 0 mod 4 below lim
// enter min(sig16 << 16 | q) into the slot of their long hash (ds_min), then every sampled block
// position p counts when its slot holds its own sig16 with a position below p.  True: the block
// has enough repeated 8-byte strings to be parsed after all.  The insert pass reads every dword
// of the staging buffer once, so it also counts the block's bytes [pre, n) into one 256-bin
// sub-histogram per wave at hw (16 x 256 u32): the literal histogram K2 needs when the block
// stays literal-only.
__device__ __forceinline__ bool repeat_scan(const u32 *in32, u32 *E, u32 *hw, u32 *misc, u32 pre, u32 n, u32 tid) {
  static_assert(ZH_SCAN_STRIDE == 4 && (4u << ZH_SCAN_LOG) <= 2 * (HL_SIZE + HS_SIZE + 2 * T_PAD), "scan table in the hash tables' space");
  static_assert(K1_THREADS / 64 == ZH_K1_HIST_WAVES && 4 * 256 * ZH_K1_HIST_WAVES <= 2 * 4 * CI_WORDS, "sub-histograms in the cinfo space");
  // the clears below take no barrier first: with one probe window the window loop is left right
  // after barrier P, when no inserter is inside a window (with 2-3, probe_dead fires at a step's
  // top while an inserter that took X in take_ready may still write TL) -- ADVICE r5
  static_assert(ZH_PROBE_WINDOWS == 1, "repeat_scan reuses the hash tables without a barrier");
  constexpr u32 NS = 1u << ZH_SCAN_LOG;
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0u, lane = tid & 63u, wave = tid >> 6;
  // slot and signature of a position's long-hash sum t: E[t >> 18], entry (t << 14) & ~0xFFFF | q
  auto slot = [&](u32 t) -> u32 * { return E + (t >> (32 - ZH_SCAN_LOG)); };
  auto key = [](u32 t) { return (t << ZH_SCAN_LOG) & 0xFFFF0000u; };
  u32 ones;  // (opaque: a constant vector would be hoisted out of the block loop and spilled)
  __asm__ volatile("v_mov_b32 %0, -1" : "=v"(ones));
  for (u32 i = tid; i < NS / 4; i += K1_THREADS) ((uint4 *)E)[i] = make_uint4(ones, ones, ones, ones);
  u32 const zero = ones + 1u;  // (opaque as well)
  ((uint4 *)hw)[tid] = make_uint4(zero, zero, zero, zero);
  if (tid == 0) misc[MISC_SCAN] = 0;
  k1_barrier();
  // insert pass: a wave takes 256 consecutive dwords (4 per lane, 64 apart); the 8 bytes at q = 4j
  // are dwords j and j + 1, the latter the next lane's (DPP), lane 63's from the next row
  u32 *const hwv = hw + 256u * wave;
  u32 const nq = (lim + 3) >> 2, nd = (n + 3) >> 2;
  for (u32 base = 256u * wave; base < nd; base += 256u * (K1_THREADS / 64)) {
    u32 w[5];
#pragma unroll
    for (u32 u = 0; u < 4; u++) w[u] = in32[base + 64u * u + lane];
    w[4] = in32[base + 256u];  // (the buffer's zero pad at most)
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 const j = base + 64u * u + lane;
      u32 const nx = u < 3 ? (u32)__builtin_amdgcn_readlane((int)w[u < 3 ? u + 1 : 0], 0) : w[4];
      u32 const t = hash_long_sum(w[u], lane == 63u ? nx : wave_shl1(w[u]));
      if (j < nq) atomicMin(slot(t), key(t) | (4u * j));
      u32 const b0 = 4u * j;
      if (b0 >= pre && b0 + 4u <= n) {
#pragma unroll
        for (u32 i = 0; i < 4; i++) atomicAdd(&hwv[(w[u] >> (8 * i)) & 255u], 1u);
      } else {
#pragma unroll
        for (u32 i = 0; i < 4; i++)
          if (b0 + i >= pre && b0 + i < n) atomicAdd(&hwv[(w[u] >> (8 * i)) & 255u], 1u);
      }
    }
  }
  k1_barrier();
  // lookup pass: the sampled block positions p = pre + ZH_SCAN_STEP m < lim count when
  // E[slot] - key < p; a lane takes 4 consecutive samples (12 bytes apart between lanes: one
  // shift for all, 6 dword loads for the 4, lanes 3 dwords apart hit distinct banks)
  static_assert(ZH_SCAN_STEP == 3, "strides coprime; 4 samples are 12 bytes");
  u32 c = 0;
  u32 const span = lim > pre ? lim - pre : 0u, nm = (span + ZH_SCAN_STEP - 1) / ZH_SCAN_STEP, sh = pre & 3u;
  for (u32 g = tid; 4u * g < nm; g += K1_THREADS) {
    u32 const p0 = pre + 12u * g, j0 = p0 >> 2;  // (a last group's unused samples may read past
                                                 // the staging pad into the table: never counted)
    u32 w[6], v[5];
#pragma unroll
    for (u32 k = 0; k < 6; k++) w[k] = in32[j0 + k];
#pragma unroll
    for (u32 k = 0; k < 5; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
    u32 const lo[4] = {v[0], __builtin_amdgcn_alignbyte(v[1], v[0], 3), __builtin_amdgcn_alignbyte(v[2], v[1], 2), __builtin_amdgcn_alignbyte(v[3], v[2], 1)};
    u32 const hi[4] = {v[1], __builtin_amdgcn_alignbyte(v[2], v[1], 3), __builtin_amdgcn_alignbyte(v[3], v[2], 2), __builtin_amdgcn_alignbyte(v[4], v[3], 1)};
    u32 t[4], e[4];
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      t[u] = hash_long_sum(lo[u], hi[u]);
      e[u] = *slot(t[u]);
    }
#pragma unroll
    for (u32 u = 0; u < 4; u++) c += (4u * g + u < nm && e[u] - key(t[u]) < p0 + 3u * u) ? 1u : 0u;
  }
  u32 const wsum = lane_value(wave_scan_incl(c), 63);
  if (lane == 0 && wsum) atomicAdd(&misc[MISC_SCAN], wsum);
  k1_barrier();
  u32 const total = (u32)__builtin_amdgcn_readfirstlane(__atomic_load_n(&misc[MISC_SCAN], __ATOMIC_RELAXED));
  return total >= max(span >> ZH_SCAN_SHIFT, (u32)ZH_SCAN_MIN);
}

template <u32 MODE>
__device__ __forceinline__ u32 lz_block(const ZhBlockDesc *__restrict__ blocks, ZhWorkspace ws, u32 b, u32 nblocks, u32 *s_take, Prefetch &pf, u32 wv, bool redo) {
  u8 *const smem = k1_lds();
  u8 *in = smem + OFF_IN;
  u32 *in32 = (u32 *)in;
  u16 *TL = (u16 *)(smem + OFF_TL), *TS = (u16 *)(smem + OFF_TS);
  u32 *ci = (u32 *)(smem + OFF_CI);
  u8 *ci8 = smem + OFF_CI;
  u64 *hm = (u64 *)(smem + OFF_HM);
  u32 *misc = (u32 *)(smem + OFF_MISC);

  // opaque per-block thread index: stops the compiler from hoisting LDS addresses derived
  // from it out of the persistent block loop (they would stay live, and spill, across it)
  u32 tid;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(k1_tid(wv)));
  u32 const lane = tid & 63;
  ZhBlockDesc const d = blocks[b];
  // the next block for this workgroup (dynamic: a slow block does not hold up a fixed share;
  // taken once per block, not again when the block is redone without the probe)
  if (tid == 0 && !redo) *s_take = atomicAdd(ws.ctr, 1u);
  if (d.n == 0) {
    k1_barrier();
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
  u32 st_stage = 0, st_A = 0, st_X = 0, st_E1 = 0, st_Bmax = 0, st_Imax = 0, st_Bw = 0, st_B = 0, st_J = 0, st_E = 0, st_E2 = 0, st_rounds = 0, st_J1 = 0, st_J2 = 0, st_J3 = 0;
#endif

  // ---- stage the block into LDS (16 B per lane when the source allows it) and probe RLE
  // (the probe looks at the block only, never at the history in front of it)
  const u8 *src = d.src;
  bool same = true;
  u32 nst;
  if (!redo && pf.ok && staged_region(d, nst)) {  // prefetched during the previous block (a redo: pf holds the next)
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
  // History without precomputed tables (a frame's later blocks, stream history, dictionary
  // views): only the final table over positions [0, pmin) -- the latest position per slot --
  // matters, so every wave inserts them at once (below) instead of the inserter waves walking
  // the history windows.
  bool const par_hist = !use_dt && pre >= 2 * ZH_TILE && d.n >= 16;
  // first window / first tile processed and the tail positions the inserters add themselves
  u32 const pmin = (use_dt || par_hist) ? pre & ~(ZH_TILE - 1) : 0u;  // the tile holding pre
  u32 const wstart = (use_dt || par_hist) ? (pre & ~(ZH_WINDOW - 1)) : 0u;
  u32 const span_s = use_dt ? pre - ZH_DTAB_MARGIN : 0u, span_e = use_dt ? pmin : 0u;
#ifdef ZH_NO_SKIP
  u32 const kskip0 = 1u << 20;
#else
  u32 const kskip0 = pre / ZH_WINDOW + 3 - wstart / ZH_WINDOW;  // first loop window that may skip
#endif
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  // the probe's step: the oracle checks once the parse of windows [a0, a0 + ZH_PROBE_WINDOWS) is
  // done, when the block has a window past them (windows counted up to lim, as the oracle does)
  // and the probe window holds enough block positions (ZH_PROBE_MAX_E0)
  u32 const a0 = pre / ZH_WINDOW, nwl = (lim + ZH_WINDOW - 1) / ZH_WINDOW;
  u32 const e0p = pre - a0 * ZH_WINDOW;  // the probe window's first parsed position
  u32 const kprobe0 = a0 + ZH_PROBE_WINDOWS + 1 <= nwl && e0p <= ZH_PROBE_MAX_E0 ? a0 + ZH_PROBE_WINDOWS + 1 - wstart / ZH_WINDOW : ~0u;
  u32 next_b = 0;
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
  if (tid == 0) {
    misc[MISC_ARR] = 0;
#pragma unroll
    for (u32 i = 0; i < 4; i++) misc[MISC_XCH + i] = 0;
  }
  if (!redo) {
    bool const rle = !block_any(!same, &misc[MISC_ANY], tid) && d.n >= 2;
    next_b = *s_take;  // (written before the barrier above)
    prefetch_block(blocks, next_b, nblocks, tid, pf);  // the next block's input, in flight from here
    if (rle) {
      if (tid == 0) {
        u32 one;  // (opaque: a constant {0, 0, 1} vector would be hoisted out of the block loop and spilled)
        __asm__ volatile("v_mov_b32 %0, 1" : "=v"(one));
        meta[0] = one - 1u; meta[1] = one - 1u; meta[2] = one;
      }
      return next_b;
    }
  } else {
    next_b = *s_take;
    k1_barrier();  // the tables and counters
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
      if (round == 0) k1_barrier();
      else if (!block_any(ch, &misc[MISC_ANY], tid)) break;
    }
  }

  ZH_STAMP(st_stage);
  u32 const kprobe = redo ? ~0u : kprobe0;
  bool dead = false;
  // ---- inserter waves: their own loop with the same barrier sequence as the workers'
  // (separate code, so their registers never add to the workers' pressure)
  if (tid >= INS_TID) {
    // The inserters are the youngest waves of the workgroup and would lose every VALU
    // issue arbitration to the 3 worker waves sharing their SIMD; the next window's tables
    // gate the workers' next window, so they take priority (MI355X_MICROARCH.md, "VALU issue
    // is arbitrated ... by priority, then age").
    // (priority 0 or 1 measured the same, profiles/r05l_k1_priority_ab.json)
    __builtin_amdgcn_s_setprio(2);
    // literal rounds (ZH_LIT_INS): both inserters half each in mode 0, else the idle long-table wave all
    bool const lw = tid < INS_TID + 64;
    LitJob lj{in, (u32 *)(smem + OFF_SEGM), (u32 *)(smem + OFF_LB), ws.lits(b), wstart, n, pre,
              two_tables<MODE>() ? (lw ? 0u : 1u) : 0u, two_tables<MODE>() ? 2u : (lw ? 1u : 0u), 0u};
    if (tid >= INS_TID + 64)
      dead = inserter_loop<false, two_tables<MODE>()>(in32, TS, ci8, misc, n, lim, lane, ws.dbg(b), wstart, pmin, span_s, span_e, kskip0, kprobe, e0p, lj,
                                                      MODE != 2);
    else if (two_tables<MODE>())
      dead = inserter_loop<true, true>(in32, TL, ci8, misc, n, lim, lane, ws.dbg(b), wstart, pmin, span_s, span_e, kskip0, kprobe, e0p, lj, MODE != 2);
    else
      dead = idle_inserter_loop(misc, n, wstart, kprobe, e0p, lj, lane, MODE != 2);
    __builtin_amdgcn_s_setprio(0);
    if (!dead) return next_b;
  } else {
  u64 *const seq_out = ws.seq(b);
  u8 *const lit_out = ws.lits(b);
  u32 nseq_tot = 0, nlit_tot = 0, e_in = pre;
  u32 const tid_ = tid;
  u32 const wave = tid >> 6;
  u32 r_lo = 0;
  for (u32 w = 0; w < wave; w++) r_lo += rounds_of_mode<MODE>(w);
  u32 const r_hi = r_lo + rounds_of_mode<MODE>(wave);
  u32 *const ci0 = ci;
  u32 *const sgm = (u32 *)(smem + OFF_SEGM);
  u32 *const lbx = (u32 *)(smem + OFF_LB);
  u16 *const xq = (u16 *)(smem + OFF_XQ) + XQ_CAP * wave;
  u32 const nwin = (n - wstart + ZH_WINDOW - 1) / ZH_WINDOW;
  u64 *const mlist = (u64 *)(smem + OFF_ML);
  u32 nwalk_tot = 0;  // the walk's literal count before the parsed window (records carry it)
  TL_DECL;
  // Step k (window j at wstart + j * ZH_WINDOW, parity j & 1):
  //   phase A  lengths of window k (waves 1..13) | span-top take decisions and parse of window
  //            k - 1 (wave 0) | catch-up and sequence records of window k - 2 (REC_WAVE)
  //   (ZH_ONE_BARRIER=0 only: X, then the take decisions at window k's span tops, each wave its
  //   own, and without ZH_LIT_INS the literals of window k - 2, lanes = positions)
  u32 m3 = 0;  // k mod LM_BUFS
  bool skp_prev = false;  // (ZH_ONE_BARRIER) window k - 1 was a miss-skip window (its span tops)
  for (u32 k = 0; k < nwin + STEPS_EXTRA; k++, m3 = m3 + 1 == LM_BUFS ? 0u : m3 + 1) {
    if (probe_dead(misc, k, kprobe)) {
      dead = true;
      break;
    }
    u32 const wsb = wstart + k * ZH_WINDOW;
    u32 const we = min(wsb + ZH_WINDOW, n);
    u32 const kb = k & 1u;
    bool const have = k < nwin && we > pre;                    // window k: lengths
    u32 const wsp = wsb - ZH_WINDOW, wep = min(wsp + ZH_WINDOW, n);
    bool const prev = k >= 1 && k <= nwin && wep > pre;        // window k - 1: parse, match list
    u32 const wsq = wsb - 2 * ZH_WINDOW;
    bool const prev2 = k >= 2 && k - 2 < nwin && min(wsq + ZH_WINDOW, n) > pre;  // window k - 2: records, literals
    // opaque per-step thread index: keeps the compiler from hoisting every LDS address
    // derived from it out of the loop (they would be spilled to scratch)
    u32 tid;
    __asm__ volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(tid_));
    u32 const lane = tid & 63;
    u32 *const ciK = ci0 + kb * CI_WORDS, *const ciP = ci0 + (kb ^ 1u) * CI_WORDS;
    u64 *const tmK = hm + kb * NROUND, *const tmP = hm + (kb ^ 1u) * NROUND;
    // window k - 1's literal bits (the walk's), window k - 2's (after its catch-up)
    u32 *const lmP = sgm + segm(LM_BUFS == 2 ? (kb ^ 1u) : (m3 == 0 ? 2u : m3 - 1u));
    u32 *const lmQ = sgm + segm(LM_BUFS == 2 ? kb : (m3 == 0 ? 1u : m3 == 1 ? 2u : 0u));
    u32 *const lbxq = lbx + (LB_BUFS == 2 ? kb : 0u) * LB_WORDS;  // window k - 2's prefix counts
    u64 *const mlP = mlist + (kb ^ 1u) * ML_CAP, *const mlQ = mlist + kb * ML_CAP;
    k1_barrier();  // P: candidates of window k in buffer k & 1
    TL_MARK(0);
    TL_STEP();
    if (probe_dead_tm(k, kprobe, e0p, MODE != 2, wep - wsp)) {
      dead = true;
      break;
    }
    ZH_STAMP(st_A);
    // a miss-skip window has candidates in its first RS rounds only: waves 1..RS take one each
    // (the top one, wave RS, knows its next positions have none), the others clear the info and
    // take masks of the rounds above
    constexpr u32 RS = 2 * ZH_SKIP_TILES;
    static_assert(RS < NWW && (RS & 1) == 0, "miss-skip rounds");
    bool const skipk = have && skip_window_eff(misc, k, kskip0);
    if (skipk && wave != 0) {
      if constexpr (MODE == 2) {
        if (wave <= RS / L1_S) span_lengths_l1(in32, ciK, tmK, xq, wave - 1, wave, wsb, n, lane);
      } else {
        if (wave <= RS) span_lengths<MODE>(in32, ciK, tmK, xq, wave - 1, wave, wsb, we, n, lim, lane, wave == RS, 0u);
      }
      for (u32 r = RS + wave - 1; r < NROUND; r += NWW - 1) {
        ciK[cidx(64 * r + lane)] = 0;
        if (lane == 0) tmK[r] = 0;
      }
      ZH_STAMP(st_B);
    } else if (MODE == 2 && have && wave != 0) {
      if (r_lo < r_hi) span_lengths_l1(in32, ciK, tmK, xq, r_lo, r_hi, wsb, n, lane);
      ZH_STAMP(st_B);
    } else if (have && wave != 0) {
      // the window's top span (wave 13) first takes the lookahead position `we`: the take
      // decision at the window's end needs its info (not in greedy mode 2)
      u32 la1 = 0;
      if (wave == NWW - 1) {
        u32 const p = we + lane;
        u32 const cw = ciK[cidx(ZH_WINDOW + (lane & 1))];
        u32 const li = info_one<MODE>(in32, p, cw, n, lim, MODE != 2 && lane == 0 && p < n);
        if (lane < 2) ciK[cidx(ZH_WINDOW + lane)] = li;
        la1 = lane_value(li, 0);
      }
      span_lengths<MODE>(in32, ciK, tmK, xq, r_lo, r_hi, wsb, we, n, lim, lane, wave == NWW - 1, la1);
      ZH_STAMP(st_B);
    }
    TL_MARK(1);
    if (wave == 0 && prev) {
      // ---- the parse of window k - 1, lanes = 32-position segments
      u32 const wn = wep - wsp;
      u32 const S = SEGP * lane, SE = min(S + SEGP, wn);
      u32 tmk = (u32)(tmP[lane >> 1] >> (32 * (lane & 1)));
      if constexpr (ZH_ONE_BARRIER && MODE != 2) {
        // the worker waves' span tops of window k - 1 (lane L: the top ending round L): a top
        // ends the odd segment 2 hi - 1, at its bit 31
        bool const dt = span_top_dec(ciP, wn, skp_prev, lane, lane < NROUND);
        u32 const d = bperm(dt ? 1u : 0u, (lane - 1u) >> 1);
        tmk |= ((lane & 1u) && d) ? 1u << 31 : 0u;
      }
      u32 const e0 = e_in - wsp;  // first parsed position (< 64 except in the window holding `pre`)
      u32 entry = lane == 0 ? e0 : max(S, e0), ex = entry;
      u32 LM = 0, MM = 0;
      // (round 6: the segment's lengths packed into 8 VGPRs, a select tree + v_perm per step instead
      // of this LDS read, measured slower: K1 10.43 -> 10.86 ms, the parse wave 6.6 k -> 7.8 k cycles
      // per step, profiles/r06d_walk_reg_ab.json)
      auto lenq = [&](u32 q) { return ciP[cidx(q)] & 255u; };
      seg_walk<false>(lenq, tmk, S, SE, entry, true, LM, MM, ex);
      // Jacobi rounds: a segment's entry is its predecessor's exit
      for (;;) {
#if ZH_K1_PMAX
        // the largest exit before the segment (its predecessor's once consistent): a match
        // covering whole segments passes its end through them in one round
        u32 const pe = wave_shr1(wave_scan_max_incl(ex));
#else
        u32 const pe = wave_shr1(ex);
#endif
        u32 const ne = lane == 0 ? e0 : max(pe, e0);
        bool const ch = ne != entry;
#ifdef ZH_STAMPS
        st_rounds++;
#endif
        if (!__ballot(ch)) break;
        seg_walk<true>(lenq, tmk, S, SE, ne, ch, LM, MM, ex);
        entry = ne;
      }
      e_in = wsp + lane_value(ex, 63);
      ZH_STAMP(st_J1);
      // the window's matches in position order, then their entries (lanes = matches): start |
      // end of the match before it (the window's first parsed position for the first: the
      // catch-up bound) | length | offset | the walk's literals before it
      u32 const ns = (u32)__popc(MM);
      u32 const is = wave_scan_incl(ns);
      u32 const nm = lane_value(is, 63);
      lmP[lane] = LM;
      u32 const nwl = lane_value(wave_scan_incl((u32)__popc(LM)), 63);
      u32 mm = MM, q = is - ns;
      while (__ballot(mm != 0)) {
        if (mm) {
          mlP[q++] = S + (u32)__builtin_ctz(mm);
          mm &= mm - 1u;
        }
      }
      ZH_STAMP(st_J2);
      u32 covered = 0, pend = e0;  // walk lengths of the matches before this pass; end of the last one
      for (u32 j0 = 0; j0 < nm; j0 += 64) {
        u32 const j = j0 + lane;
        bool const v = j < nm;
        u32 const ms = v ? (u32)mlP[j] : 0u, inf = ciP[cidx(ms)];
        u32 const len = v ? inf & 255u : 0u, off = (inf >> 8) & 0xFFFFu;
        u32 const incl = wave_scan_incl(len);
        u32 const cum = nwalk_tot + (ms - e0) - (covered + incl - len);
        u32 lo = wave_shr1(ms + len);
        if (lane == 0) lo = pend;
        pend = lane_value(ms + len, min(63u, nm - 1u - j0));
        covered += lane_value(incl, 63);
        if (v) mlP[j] = (u64)ms | ((u64)lo << ML_LO) | ((u64)len << ML_LEN) | ((u64)off << ML_OFF) | ((u64)cum << ML_CUM);
      }
      nwalk_tot += nwl;  // the window's walk literals (its last match may run past its end)
      if (lane == 0) { misc[MISC_WNM + (kb ^ 1u)] = nm; misc[MISC_NM + ((k - 1) & 3)] = nm; }
      ZH_STAMP(st_J);
    }
    // (ZH_ONE_BARRIER) wave 0 is done with window k - 1's match info: the inserters may dump
    // window k + 1's candidates into that buffer
    if (ZH_ONE_BARRIER && wave == 0 && lane == 0) __atomic_store_n(&misc[MISC_PF], k + 1, __ATOMIC_RELAXED);
    if (wave == REC_WAVE && prev2) {
      // ---- catch-up and sequence records of window k - 2, lanes = matches.  A match grows
      // back over the literals down to the end of the match before it; it takes back e bytes of
      // the literal run.  Record: the walk's literals before the match | length | e | offset;
      // K2 takes e off the literal run (zh_entropy.hip).
      u32 const nm = (u32)__builtin_amdgcn_readfirstlane(misc[MISC_WNM + kb]);
      for (u32 j0 = 0; j0 < nm; j0 += 64) {
        u32 const j = j0 + lane;
        bool const v = j < nm;
        u64 const en = v ? mlQ[j] : 0ull;
        u32 const ms = (u32)en & 0x7FFu, lo = (u32)(en >> ML_LO) & 0x7FFu, len = (u32)(en >> ML_LEN) & 0x7Fu;
        u32 const off = (u32)(en >> ML_OFF) & 0xFFFFu, cum = (u32)(en >> ML_CUM);
        u32 const e = catch_up(in32, wsq + ms, off, wsq + lo, v);
        if (v) seq_out[nseq_tot + j] = (u64)cum | ((u64)len << 17) | ((u64)e << 24) | ((u64)off << 36);
        if (e) {
          for (u32 g = (ms - e) / SEGP; g <= (ms - 1) / SEGP; g++) {
            u32 const a = max(ms - e, SEGP * g) - SEGP * g, bnd = min(ms - SEGP * g, SEGP);
            atomicAnd(&lmQ[g], ~bit_range32(a, bnd));
          }
        }
      }
      // the window's literal bits are final now (the catch-up cleared its share): the literal
      // phase's per-segment exclusive prefix counts, once for every wave (LDS ops of a wave
      // apply in order, so the reads see this wave's atomics)
      u32 const lc = (u32)__popc(lmQ[lane]), lincl = wave_scan_incl(lc);
      lbxq[lane] = lincl - lc;
      if (lane == 63) lbxq[NSEG] = lincl;
      if (ZH_ONE_BARRIER) {  // (this wave keeps the block's totals: no barrier before the others could read them)
        nlit_tot += lane_value(lincl, 63);
        nseq_tot += nm;
      }
    }
    TL_MARK(2);
    if (!ZH_ONE_BARRIER) {
      if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);
      k1_barrier();  // X: window k's match info and take masks; window k - 1's records and literal bits
    }
    TL_MARK(3);
    ZH_STAMP(st_X);
    if (!ZH_ONE_BARRIER && MODE != 2 && have && wave != 0 && wave < (skipk ? RS : NWW - 1)) {
      // ---- take decision at this wave's span top (the next position was the next wave's):
      // every wave but the window's top one, its last position
      u32 const hi = skipk ? wave : r_hi;
      u32 const i = 64 * hi - 1;
      if (lane == 0) {
        u32 const inf = ciK[cidx(i)], inf1 = ciK[cidx(i + 1)];
        // (a 32-bit atomic on the mask's half: a hoisted 64-bit bit constant spilled)
        if (i < we - wsb && (inf & 255u) && take_rule<MODE>(inf, inf1)) atomicOr((u32 *)&tmK[i >> 6] + ((i >> 5) & 1u), 1u << (i & 31));
      }
    }
    if (ZH_ONE_BARRIER) {
      // (the records wave keeps the totals)
    } else if (ZH_LIT_INS && prev2) {
      // (the inserters extract window k - 2's literals in step k + 1)
      nlit_tot += (u32)__builtin_amdgcn_readfirstlane(lbxq[NSEG]);
      nseq_tot += __builtin_amdgcn_readfirstlane(misc[MISC_WNM + kb]);
    } else if (prev2) {
      // ---- literals of window k - 2, lanes = positions (round r = segments 2r, 2r + 1)
      u32 const nm = __builtin_amdgcn_readfirstlane(misc[MISC_WNM + kb]);
#ifdef ZH_EXP_NOLITPHASE
      if (true) { nseq_tot += nm; } else  // (experiment: the literal phase's upper bound; output wrong)
#endif
      {
      // the wave's rounds r = wave + NWW j: every LDS read of them issued first (one round trip)
      constexpr u32 LR = (NROUND + NWW - 1) / NWW;
      u64 mw[LR];
      u32 lbr[LR], by[LR];
#pragma unroll
      for (u32 j = 0; j < LR; j++) {
        u32 const r = min(wave + NWW * j, NROUND - 1u);
        mw[j] = *(const u64 *)&lmQ[2 * r];
        lbr[j] = (u32)__builtin_amdgcn_readfirstlane(lbx[2 * r]);
        by[j] = in[wsq + 64 * r + lane];  // (every lane: the loads leave before the masks are tested)
      }
#pragma unroll
      for (u32 j = 0; j < LR; j++) __asm__ volatile("" : "+v"(by[j]));  // (not sunk into the branches)
#pragma unroll
      for (u32 j = 0; j < LR; j++) {
        if (wave + NWW * j >= NROUND) continue;
        u64 const lm = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(mw[j] >> 32)) << 32) | (u32)__builtin_amdgcn_readfirstlane((u32)mw[j]);
        if ((lm >> lane) & 1ull) {
          u32 const rank = __builtin_amdgcn_mbcnt_hi((u32)(lm >> 32), __builtin_amdgcn_mbcnt_lo((u32)lm, 0u));
#ifndef ZH_EXP_NOLIT
          lit_out[nlit_tot + lbr[j] + rank] = (u8)by[j];
#endif
        }
      }
      vpad<ZH_PAD_L>(nm);
      nlit_tot += (u32)__builtin_amdgcn_readfirstlane(lbx[NSEG]);
      nseq_tot += nm;
      }
    }
    ZH_STAMP(st_E);
    TL_MARK(4);
    skp_prev = skipk;
  }
  TL_FLUSH(wave, lane);
  if (!dead) {
    if (tid_ == (ZH_ONE_BARRIER ? 64u * REC_WAVE : 0u)) { meta[0] = nseq_tot; meta[1] = nlit_tot; meta[2] = 0; }
#ifdef ZH_STAMPS
    if (tid == 0) {
      u32 *dbg = ws.dbg(b);
      dbg[23] = (u32)rt0; dbg[24] = (u32)__builtin_amdgcn_s_memrealtime();
      dbg[25] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      dbg[26] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      dbg[27] = (u32)(__builtin_amdgcn_s_memtime() - mt0);
      dbg[40] = st_Bmax; dbg[41] = st_Imax; dbg[55] = st_J1; dbg[56] = st_J2; dbg[57] = st_J3;
      dbg[0] = st_stage; dbg[1] = st_A; dbg[2] = st_B; dbg[3] = st_J; dbg[4] = st_E; dbg[5] = st_rounds; dbg[20] = st_E2; dbg[21] = st_X; dbg[22] = st_E1;
    }
    if ((tid & 63) == 0 && tid < INS_TID) {  // each worker wave's length-phase cycles
      u32 const w = tid >> 6;
#ifdef ZH_EXP_PWAIT
      ws.dbg(b)[w < 12 ? 28 + w : 53 + (w - 12)] = st_A;
#else
      ws.dbg(b)[w < 12 ? 28 + w : 53 + (w - 12)] = st_B;
#endif
    }
#endif
    return next_b;
  }
  }  // (worker waves)
  // The probe ended the window loop (every wave left it at the same step): the repeat scan
  // decides between the literal-only block and redoing the block from its staging without the
  // probe (the oracle's parse simply goes on; lz_blocks calls lz_block again with `redo`).
  u32 *const hw = (u32 *)(smem + OFF_CI);  // the scan's per-wave literal sub-histograms
#ifdef ZH_NO_SCAN
  if (false) return K1_REDO;  // (A/B variant: the probe alone decides, as in round 4)
#else
  if (repeat_scan(in32, (u32 *)TL, hw, misc, pre, n, tid)) return K1_REDO;
#endif
  ZH_STAMP(st_E1);
  u32 const wave = tid >> 6;
  u32 bo;  // (opaque: the block's workspace offset is not kept live across the window loop)
  __asm__ volatile("s_mov_b32 %0, %1" : "=s"(bo) : "s"((u32)__builtin_amdgcn_readfirstlane(b)));
  u8 *const lit_out = ws.lits(bo);
  if ((((uintptr_t)d.src) & 15) == 0) {
    // no sequences, the whole block is literals, and they are the block's own bytes -- K2 reads
    // them from the source (16-B aligned).  K1 leaves K2 the literal histogram instead: the
    // scan's 16 per-wave sub-histograms, stored after the first 64 KiB of the literal area
    // (ZH_K1_HIST_OFF).
    u32 *const gh = (u32 *)(lit_out + ZH_K1_HIST_OFF) + 256u * wave;
    for (u32 i = lane; i < 256; i += 64) gh[i] = hw[256u * wave + i];
    if (tid == 0) {
      u32 two;  // (opaque: a constant {0, n, 2} vector would be hoisted out of the block loop and spilled)
      __asm__ volatile("v_mov_b32 %0, 2" : "=v"(two));
      meta[0] = two - 2u; meta[1] = d.n; meta[2] = two;
    }
#ifdef ZH_STAMPS
    ZH_STAMP(st_E);
    if (tid == 0) {
      u32 *dbg = ws.dbg(b);
      dbg[27] = (u32)(__builtin_amdgcn_s_memtime() - mt0);
      dbg[0] = st_stage; dbg[1] = st_A; dbg[2] = st_B; dbg[3] = st_J; dbg[4] = st_E; dbg[5] = st_rounds; dbg[22] = st_E1;
    }
#endif
    return next_b;
  }
  if (tid >= INS_TID) return next_b;
  // (unaligned source) the block's bytes go out of LDS to the literal area in 16-B stores
  u32 const nv = (d.n + 15) >> 4, sh = pre & 3;
  const u32 *const src32 = in32 + (pre >> 2);
  for (u32 i = tid; i < nv; i += INS_TID) {
    u32 w[5];
#pragma unroll
    for (u32 k = 0; k < 5; k++) w[k] = src32[4 * i + k];
    uint4 v;
    v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
    v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
    v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
    v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
    ((uint4 *)lit_out)[i] = v;
  }
  if (tid == 0) { meta[0] = 0; meta[1] = d.n; meta[2] = 0; }
  return next_b;
}

// Persistent workgroups (grid = one per CU, the LDS footprint allows no second): workgroup g
// takes blocks g, g + grid, ... and stages each block from registers loaded while the previous
// one was processed, so the HBM latency of staging and the per-block launch gap overlap work.
template <u32 MODE>
__device__ __forceinline__ void lz_blocks(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  extern __shared__ __attribute__((aligned(16))) u8 smem_dyn[];
  u8 *const smem = k1_lds();
  if (threadIdx.x == 0 && (u32)(uintptr_t)smem_dyn != K1_DYN) __builtin_trap();  // (see k1_lds)
  __shared__ u32 s_take;  // block index taken from the counter, broadcast to the workgroup
  if (threadIdx.x == 0) {
    s_take = atomicAdd(ws.ctr, 1u);
    ((u32 *)(smem + OFF_MISC))[MISC_ANY] = 0;
  }
  k1_barrier();
  u32 b = s_take;
  Prefetch pf;
  u32 const wv = (u32)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  prefetch_block(blocks, b, nblocks, k1_tid(wv), pf);
  bool redo = false;
  while (b < nblocks) {
    // the next block taken, or K1_REDO (the same in every wave; readfirstlane keeps it -- and the
    // block index and descriptor fields derived from it -- in SGPRs: the function's return paths
    // join under the inserter / worker split, which the compiler takes for divergence)
    u32 const r = (u32)__builtin_amdgcn_readfirstlane(lz_block<MODE>(blocks, ws, b, nblocks, &s_take, pf, wv, redo));
    k1_barrier();  // every wave is done with this block's LDS before the next is staged
    redo = r == K1_REDO;
    b = redo ? b : r;
  }
}
// one instantiation per parse mode (ZH_K1_MODE: levels 3-4 / 2 / 1)
extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  lz_blocks<0>(blocks, nblocks, ws);
}
extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_short_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  lz_blocks<1>(blocks, nblocks, ws);
}
extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_greedy_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  lz_blocks<2>(blocks, nblocks, ws);
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
  for (const void *f : {(const void *)zh_lz_kernel, (const void *)zh_lz_short_kernel, (const void *)zh_lz_greedy_kernel}) {
    hipError_t const e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K1_LDS);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
// mode = ZH_K1_MODE(level)
void lz_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 mode, hipStream_t stream) {
  // one persistent workgroup per CU of the stream's device
  int dev = 0, cus = 0;
  if (stream) (void)hipStreamGetDevice(stream, &dev);
  else (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  u32 const grid = std::min(nblocks, (u32)cus);
  auto *const k = mode == 2 ? zh_lz_greedy_kernel : mode == 1 ? zh_lz_short_kernel : zh_lz_kernel;
  hipLaunchKernelGGL(k, dim3(grid), dim3(K1_THREADS), K1_LDS, stream, d_descs, nblocks, ws);
}
}  // namespace zh

// Test hook (tests/test_gpu_k1.py, not a product entry point): K1 alone (parse mode `mode`,
// ZH_K1_MODE) over single-block items in[i * stride, + sizes[i]) (each <= ZH_BLOCK_MAX, no
// dictionary), its raw output copied back: per item ZH_SEQ_CAP records, ZH_LIT_BYTES of the
// literal area and meta {nseq, nlit, rle}.
// The per-item sizes zh_test_lz copies back (the caller's buffers are sized from these).
extern "C" void zh_test_lz_sizes(u32 *seq_cap, u32 *lit_bytes) { *seq_cap = ZH_SEQ_CAP; *lit_bytes = ZH_LIT_BYTES; }
extern "C" int zh_test_lz(const u8 *d_in, u32 nitems, u32 stride, const u32 *h_sizes, int mode, u64 *h_recs, u8 *h_lits, u32 *h_meta) {
  if (!nitems) return 0;
  std::vector<ZhBlockDesc> descs(nitems);
  for (u32 i = 0; i < nitems; i++) {
    if (h_sizes[i] > ZH_BLOCK_MAX) return 2;
    ZhBlockDesc d{};
    d.src = d_in + (size_t)i * stride;
    d.n = h_sizes[i];
    d.frame_size = h_sizes[i];
    d.item = i;
    d.flags = ZH_F_FIRST | ZH_F_LAST | ZH_F_DIRECT;
    descs[i] = d;
  }
  ZhBlockDesc *dd = nullptr;
  u8 *base = nullptr;
  u32 *ctr = nullptr;
  int rc = 0;
  if (zh::lz_init() != hipSuccess || hipMalloc(&dd, sizeof(ZhBlockDesc) * nitems) != hipSuccess ||
      hipMalloc(&base, (size_t)ZH_WS_BLOCK_BYTES * nitems) != hipSuccess || hipMalloc(&ctr, 4) != hipSuccess) {
    rc = 1;
  } else {
    (void)hipMemcpy(dd, descs.data(), sizeof(ZhBlockDesc) * nitems, hipMemcpyHostToDevice);
    (void)hipMemset(ctr, 0, 4);
    ZhWorkspace ws{base, ctr, nullptr, 0u};
    zh::lz_launch(dd, nitems, ws, (u32)mode, nullptr);
    if (hipDeviceSynchronize() != hipSuccess) rc = 1;
    for (u32 i = 0; i < nitems && !rc; i++) {
      u8 *const b = base + (size_t)i * ZH_WS_BLOCK_BYTES;
      (void)hipMemcpy(h_recs + (size_t)i * ZH_SEQ_CAP, b, ZH_SEQ_BYTES, hipMemcpyDeviceToHost);
      (void)hipMemcpy(h_lits + (size_t)i * ZH_LIT_BYTES, b + ZH_SEQ_BYTES, ZH_LIT_BYTES, hipMemcpyDeviceToHost);
      (void)hipMemcpy(h_meta + 4 * i, b + ZH_SEQ_BYTES + ZH_LIT_BYTES, 16, hipMemcpyDeviceToHost);
    }
  }
  (void)hipFree(dd);
  (void)hipFree(base);
  (void)hipFree(ctr);
  return rc;
}
