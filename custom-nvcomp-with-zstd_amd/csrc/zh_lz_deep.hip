// zh_lz_deep.hip — K1 for levels >= ZH_DEEP_LEVEL: exact hash chains, a
// ZH_DEEP_DEPTH(level)-candidate search per position, LAZY2 parse.
//
// Replaces the reference's level >= 7 chain matcher (find_matches_kernel, src/lz77_parallel.cu:26-70,
// whose atomicExch chain insert makes its output nondeterministic; search depth from the level
// table, src/cuda_zstd_types.cpp:172-183).  Output is identical to oracle/zstd_oracle.c
// orc_lz_parse_deep: the same sequence records and literal bytes K1 (zh_lz.hip) hands to the
// entropy stage, so K2-K4 are shared.
//
// One persistent 1024-thread workgroup per CU; blocks from the device counter.  Each workgroup
// owns a slot of the deep scratch in the caller's workspace (ZhWorkspace::deep_slots): the staged
// bytes (history or dictionary prefix + block, contiguous), prev[] and the per-position offsets.
// Per block:
//   1. stage the prefix + block into the slot (and probe RLE); hash every position into prev[]
//   2. chains, wave 0: positions in order, 64 per LDS `ds_max_rtn_u32` on the head table (entry =
//      position + 1): LDS executes one wave's operations in order and a store's lanes one after
//      another, so each lane gets the latest earlier position with its hash -- checked (a lane
//      that got a position >= its own saw a later lane first) with an exact fix-up otherwise
//   3. search, lanes = block positions (all 16 waves): the chain's candidates, links as u16
//      distances and the staged bytes in LDS when they fit (else the slot, L2), the longest
//      common prefix within the cap
//   4. take mask per position (the LAZY2 rule on p, p+1, p+2), then the parse as 64-position
//      segments, one per thread, walked from a guessed entry with Jacobi rounds across the
//      workgroup until every segment's entry is its left neighbour's exit (the serial parse)
//   5. records (walk literals before the match | length | 0 | offset) and the literal bytes
#include "zh_common.h"
#include "zh_hash.h"

namespace {

constexpr u32 DT = 1024;                          // threads per workgroup
constexpr u32 HSIZE = 1u << ZH_HASH_LOG_SHORT;    // head table entries (+ a junk slot)
constexpr u32 NSEG = ZH_BLOCK_MAX / 64;           // 64-position parse segments per block
constexpr u32 HB = 8192;                          // positions per chain-building round
#ifndef ZH_DEEP_FORCE_FIXUP
#define ZH_DEEP_FORCE_FIXUP 0  // test builds: every chain step takes the out-of-order fix-up path
#endif
static_assert(NSEG == DT, "one parse segment per thread");
static_assert(ZH_DEEP_PRE <= ZH_BLOCK_MAX && ZH_HIST_BLOCK <= ZH_BLOCK_MAX, "staged prefix fits the slot");
// scratch slot of one workgroup (global memory)
constexpr u32 STG_BYTES = ZH_DEEP_STG_BYTES;                // staged bytes + zero pad
constexpr u32 SLOT_PREV = STG_BYTES;                        // u32 prev[2 * ZH_BLOCK_MAX]: q + 1, 0 = none
constexpr u32 SLOT_OFF = SLOT_PREV + 4 * 2 * ZH_BLOCK_MAX;  // u32 off << 8 | len per block position
constexpr u32 SLOT_P16 = SLOT_OFF + 4 * ZH_BLOCK_MAX;       // u16 link distances when LDS cannot hold them
constexpr size_t SLOT_BYTES = SLOT_P16 + 2 * 2 * ZH_BLOCK_MAX;
static_assert(SLOT_BYTES % 256 == 0 && SLOT_BYTES == ZH_DEEP_SLOT_BYTES, "slot alignment / host size");
// LDS
constexpr u32 L_HEAD = 0;                  // u32 head[HSIZE + 4] (chains) / u8 len[ZH_BLOCK_MAX] (search, parse)
constexpr u32 L_TM = 4 * (HSIZE + 4);      // u64 take masks per segment
constexpr u32 L_LM = L_TM + 8 * NSEG;      // u64 literal bits per segment
constexpr u32 L_MM = L_LM + 8 * NSEG;      // u64 match-start bits per segment
constexpr u32 L_EX = L_MM + 8 * NSEG;      // u32 walk exit per segment
constexpr u32 L_LP = L_EX + 4 * NSEG;      // u32 literals before the segment
constexpr u32 L_MP = L_LP + 4 * NSEG;      // u32 matches before the segment
#ifndef ZH_DEEP_WAVEQ
#define ZH_DEEP_WAVEQ 1  // per-wave demand queues (C5 no dictionary 12.9 -> 13.8 GB/s)
#endif
#ifndef ZH_DEEP_G64EARLY
#define ZH_DEEP_G64EARLY 1  // (C5 15.5 / 13.5 -> 15.8 / 14.0 GB/s without / with the COVER dictionary)
#endif
#ifndef ZH_DEEP_B64
#define ZH_DEEP_B64 1  // extension bytes by 8-byte loads (C5 12.1 -> 12.9 GB/s)
#endif
constexpr u32 DEEP_LDS = 160 * 1024;
constexpr u32 L_WS = DEEP_LDS - 256;       // u32[32] per-wave sums
constexpr u32 L_MISC = L_WS + 4 * 32;      // u32[8]: [0] block_any flag, [1] next block
constexpr u32 SEARCH_LDS = L_WS;           // search: u16 link distances, then (if they fit) the staged bytes
static_assert(L_MP + 4 * NSEG <= L_WS, "parse arrays below the scan sums");
static_assert(4 * (HSIZE + 4) >= ZH_BLOCK_MAX, "len[] reuses the head table");
static_assert(L_TM + 2 * 2 * HB <= L_WS, "chain rounds' hash buffers fit below the scan sums");

// the 8 bytes at staged position p (4-B aligned slot, zero padded)
__device__ __forceinline__ void g64(const u32 *s32, u32 p, u32 &lo, u32 &hi) {
  u32 const w = p >> 2, sh = p & 3;
  u32 const w0 = s32[w], w1 = s32[w + 1], w2 = s32[w + 2];
  lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
}

__device__ __forceinline__ bool wg_any(bool v, u32 *flag, u32 tid) {
  if (__ballot(v) && (tid & 63) == 0) atomicOr(flag, 1u);
  __syncthreads();
  bool const r = *flag != 0;
  __syncthreads();
  if (tid == 0) *flag = 0;
  __syncthreads();
  return r;
}

// exclusive prefix of v over the workgroup's threads; total = the sum
__device__ __forceinline__ u32 wg_excl_scan(u32 v, u32 *ws, u32 tid, u32 &total) {
  u32 const inc = wave_scan_incl(v);
  if ((tid & 63) == 63) ws[tid >> 6] = inc;
  __syncthreads();
  u32 base = 0, tot = 0;
  u32 const w = tid >> 6;
  for (u32 k = 0; k < DT / 64; k++) {
    u32 const s = ws[k];
    base += k < w ? s : 0u;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return base + inc - v;
}

__device__ __forceinline__ u64 bits_from(u32 a) { return a >= 64 ? 0ull : ~0ull << a; }
__device__ __forceinline__ u64 bit_range64(u32 a, u32 b) { return bits_from(a) & ~bits_from(b); }

// LAZY2 gain of a match (libzstd ZSTD_compressBlock_lazy_generic): 4 per byte minus the bit
// length of offset + 1; no match: -1000 (oracle match_gain32)
__device__ __forceinline__ int gain_of(u32 len, u32 off) { return len ? 4 * (int)len - (31 - (int)__builtin_clz(off + 1u)) : -1000; }

// Walk of segment [S, SE) (block positions) from p, as zh_lz.hip seg_walk with 64-bit masks:
// each step is one literal run (the positions before the next take bit) and the match after
// it; a re-walk (act0 with old bits) stops where it meets the old trajectory.
__device__ __forceinline__ void seg_walk64(const u8 *len, u64 tmk, u32 S, u32 SE, u32 p, bool act0, u64 &LM, u64 &MM, u32 &ex) {
  u64 const old = act0 ? (LM | MM) : 0ull;
  u64 nl = 0, nm = 0;
  bool act = act0 && p < SE, merged = false;
  u32 mpos = 0;
  while (__ballot(act)) {
    u32 const o = min(p - S, 63u);
    u64 const m = tmk >> o, ov = old >> o;
    u32 const q = m ? p + (u32)__builtin_ctzll(m) : SE;
    u32 const x = ov ? p + (u32)__builtin_ctzll(ov) : ~0u;
    bool const mg = act && x <= q;
    bool const st = act && !mg && q < SE;
    u32 const re = mg ? x : q;
    nl |= act ? bit_range64(o, re - S) : 0ull;
    u32 const l = len[st ? q : 0u];
    nm |= st ? 1ull << (q - S) : 0ull;
    mpos = mg ? x - S : mpos;
    merged = merged || mg;
    p = mg ? p : (st ? q + l : (act ? q : p));
    act = act && !mg && p < SE;
  }
  if (act0) {
    if (merged) {
      u64 const keep = bits_from(mpos);
      LM = nl | (LM & keep);
      MM = nm | (MM & keep);
    } else {
      LM = nl;
      MM = nm;
      ex = p;
    }
  }
}

#ifdef ZH_STAMPS
__device__ u32 g_deep_fix;  // diagnostic: chain steps that needed the out-of-order fix-up
#endif
// Links of the staged positions [s0, lim) (s0 % 4 == 0): prev[p] = the latest q < p with p's
// hash, + 1 (0: none), given a head table holding the latest of every position below s0.  Every
// position's hash first (all threads), then rounds of HB positions: waves 1..15 copy round r + 1's
// hashes into one LDS buffer (hb: 2 x HB u16) while wave 0 links round r from the other, 64
// positions per LDS atomic, four in flight.  Ends with a barrier.
__device__ void deep_chains(const u32 *s32, u32 *prev, u32 *head, u16 *hb, u32 s0, u32 lim, u32 tid) {
  u32 const lane = tid & 63;
  // every position's hash into prev[] (4 positions per thread from 3 dwords; overwritten by the
  // links below)
#pragma unroll 4
  for (u32 g4 = (s0 >> 2) + tid; 4 * g4 < lim; g4 += DT) {
    u32 const w0 = s32[g4], w1 = s32[g4 + 1], w2 = s32[g4 + 2];
    uint4 h4;
    u32 *hh = (u32 *)&h4;
#pragma unroll
    for (u32 k = 0; k < 4; k++) hh[k] = 4 * g4 + k < lim ? hash_short(__builtin_amdgcn_alignbyte(w1, w0, k), __builtin_amdgcn_alignbyte(w2, w1, k)) : HSIZE;
    *(uint4 *)(prev + 4 * g4) = h4;
  }
  __threadfence_block();
  __syncthreads();

  // ---- 2. chains.  Rounds of HB positions: waves 1..15 copy round r + 1's hashes into one LDS
  // buffer while wave 0 links round r from the other: 64 positions per LDS atomic, four in flight.
  {
    auto hash_round = [&](u32 r, u32 t0, u32 nt) {
      u16 *const dst = hb + (r & 1u) * HB;
#pragma unroll 4
      for (u32 j = 4 * t0; j < HB; j += 4 * nt) {
        u32 const p = s0 + r * HB + j;
        uint4 const h4 = p < lim ? *(const uint4 *)(prev + p) : make_uint4(HSIZE, HSIZE, HSIZE, HSIZE);
        u32 const a = p < lim ? h4.x : HSIZE, b = p + 1 < lim ? h4.y : HSIZE, c = p + 2 < lim ? h4.z : HSIZE, e = p + 3 < lim ? h4.w : HSIZE;
        *(uint2 *)(dst + j) = make_uint2(a | (b << 16), c | (e << 16));
      }
    };
    u32 const nr = lim > s0 ? (lim - s0 + HB - 1) / HB : 0u;
    if (nr) hash_round(0, tid, DT);
    for (u32 r = 0; r < nr; r++) {
      __syncthreads();  // round r hashed; wave 0 is done with the buffer round r + 1 reuses
      if (tid < 64) {
        const u16 *const src = hb + (r & 1u) * HB;
        constexpr u32 U = 4;
        for (u32 j0 = 0; j0 < HB && s0 + r * HB + j0 < lim; j0 += 64 * U) {
          u32 h[U], rv[U];
#pragma unroll
          for (u32 u = 0; u < U; u++) h[u] = src[j0 + 64 * u + lane];
#pragma unroll
          for (u32 u = 0; u < U; u++) rv[u] = atomicMax(&head[h[u]], s0 + r * HB + j0 + 64 * u + lane + 1);
#pragma unroll
          for (u32 u = 0; u < U; u++) {
            u32 const p = s0 + r * HB + j0 + 64 * u + lane;
            bool const v = p < lim;
            if (ZH_DEEP_FORCE_FIXUP || __ballot(v && rv[u] >= p + 1)) {
#ifdef ZH_STAMPS
              if (lane == 0) atomicAdd(&g_deep_fix, 1u);
#endif
              // lanes of one atomic applied out of lane order: prev = the latest earlier lane with
              // the same hash, else the head before the step (the smallest value any lane of the
              // group got)
              u32 mn = ~0u, pm = 0;
              for (u32 k = 0; k < 64; k++) {
                u32 const hk = (u32)__builtin_amdgcn_readlane((int)h[u], (int)k), rk = (u32)__builtin_amdgcn_readlane((int)rv[u], (int)k);
                if (hk == h[u]) {
                  mn = min(mn, rk);
                  if (k < lane) pm = p - lane + k + 1;
                }
              }
              rv[u] = pm ? pm : mn;
            }
            if (v) prev[p] = rv[u];
          }
        }
      } else if (r + 1 < nr) {
        hash_round(r + 1, tid - 64, DT - 64);
      }
    }
  }
  __threadfence_block();
  __syncthreads();

}

// The chain search of block position i (lanes `valid`; all lanes of the wave call it together):
// the longest of the chain's first `depth` candidates -> off << 8 | len (0: none).  D32: the
// staged bytes (LDS or the slot), P16: link distances of positions [s0, lim) (LDS or the slot),
// positions below s0 link through dprev.  One chain per lane, the position's own 64 bytes held in
// registers (aligned to p): a candidate's extension loads only its own 15 dwords (two chains per
// lane, both loading the whole 112 bytes per extension: C5 8.5 / 6.7 GB/s vs 9.1 / 7.3 this way).
__device__ __forceinline__ u32 deep_search_one(const u32 *D32, const u16 *P16, const u32 *dprev, u32 i, bool valid, u32 pre, u32 nb, u32 n,
                                               u32 lim, u32 s0, u32 depth) {
  // the next candidate after q (+ 1, 0 = none).  (A four-hop table of the dictionary's links, one
  // 8-byte L2 load per four candidates, measured slower: C5 with the COVER dictionary 13.5 -> 12.1 GB/s.)
  auto link = [&](u32 q) -> u32 {
    if (q < s0) return dprev[q];
    u32 const dl = P16[q - s0];
    return dl ? q + 1u - dl : 0u;
  };
  u32 const p = pre + i;
  bool act = valid && i < nb && p < lim;
  u32 c = act ? link(p) : 0u, best = 0, bo = 0, dd = 0;
  act = act && c != 0 && p - (c - 1u) <= ZH_DEEP_MAXOFF;
  u32 O[16];
  {
    u32 const w = p >> 2, sh = p & 3;
    u32 R[17];
#pragma unroll
    for (u32 j = 0; j < 17; j++) R[j] = (valid && i < nb) ? D32[w + j] : 0u;
#pragma unroll
    for (u32 j = 0; j < 16; j++) O[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], sh);
  }
  u32 ownb = 0;  // own byte at p + best (best >= 8)
  while (__ballot(act)) {
    if (act) {
      u32 const q = c - 1u;
#if ZH_DEEP_G64EARLY
      // the first 8 candidate bytes loaded with the reject byte, not after it: one dependent LDS
      // round trip per candidate instead of two once best >= 8 (the bytes are dropped on a reject)
      u32 clo, chi;
      g64(D32, q, clo, chi);
#endif
      bool w = true;
      if (best >= 8) {
        u32 const b = q + best;
        w = ownb == ((D32[b >> 2] >> (8 * (b & 3))) & 255u);
      }
      u32 const nx = link(q);
      u32 l = 0;
      if (w) {
#if !ZH_DEEP_G64EARLY
        u32 clo, chi;
        g64(D32, q, clo, chi);
#endif
        u32 const x = O[0] ^ clo, y = O[1] ^ chi;
        l = x ? (u32)__builtin_ctz(x) >> 3 : y ? 4u + ((u32)__builtin_ctz(y) >> 3) : 8u;
        if (l == 8 && p + 8 < n) {
          u32 const sq = q & 3;
          u32 e = 56;
#if ZH_DEEP_B64
          // bytes [q + 8, q + 64) from aligned 8-byte loads (half the LDS instructions of dword
          // loads), dword j of the candidate being W[odd + j]: dwords 0..6 first (five loads), the
          // rest (five more) only when those all match
          u32 const a8 = q + 8, wq8 = a8 >> 3, odd = (a8 >> 2) & 1u;
          const u64 *const D64 = (const u64 *)D32 + wq8;
          u32 W[10];
#pragma unroll
          for (u32 k = 0; k < 5; k++) {
            u64 const v = D64[k];
            W[2 * k] = (u32)v;
            W[2 * k + 1] = (u32)(v >> 32);
          }
#pragma unroll
          for (int j = 6; j >= 0; j--) {
            u32 const lo = odd ? W[j + 1] : W[j], hi = odd ? W[j + 2] : W[j + 1];
            u32 const xx = O[j + 2] ^ __builtin_amdgcn_alignbyte(hi, lo, sq);
            if (xx) e = 4 * (u32)j + ((u32)__builtin_ctz(xx) >> 3);
          }
          if (e == 56) {
#pragma unroll
            for (u32 k = 0; k < 5; k++) {  // W[m] = dword 6 + m
              u64 const v = D64[3 + k];
              W[2 * k] = (u32)v;
              W[2 * k + 1] = (u32)(v >> 32);
            }
#pragma unroll
            for (int j = 13; j >= 7; j--) {
              u32 const lo = odd ? W[j - 5] : W[j - 6], hi = odd ? W[j - 4] : W[j - 5];
              u32 const xx = O[j + 2] ^ __builtin_amdgcn_alignbyte(hi, lo, sq);
              if (xx) e = 4 * (u32)j + ((u32)__builtin_ctz(xx) >> 3);
            }
          }
#else
          u32 B[15];
          u32 const wq = (q >> 2) + 2;
#pragma unroll
          for (u32 k = 0; k < 15; k++) B[k] = D32[wq + k];
#pragma unroll
          for (int j = 13; j >= 0; j--) {
            u32 const xx = O[j + 2] ^ __builtin_amdgcn_alignbyte(B[j + 1], B[j], sq);
            if (xx) e = 4 * (u32)j + ((u32)__builtin_ctz(xx) >> 3);
          }
#endif
          l = 8 + e;
        }
      }
      l = min(l, p < n ? n - p : 0u);
      if (l >= ZH_MIN_MATCH_SHORT && l > best) {
        best = l;
        bo = p - q;
        u32 const a = p + l;  // the own byte a candidate must match to beat the new best
        ownb = (D32[a >> 2] >> (8 * (a & 3))) & 255u;
      }
      dd++;
      c = nx;
      act = best < ZH_MAX_MATCH && dd < depth && c != 0 && p - (c - 1u) <= ZH_DEEP_MAXOFF;
    }
  }
  return bo << 8 | best;
}

// Step 3 of deep_block: per block position the chain's first `depth` candidates -> offg[i] =
// off << 8 | len.  DL: the staged bytes in LDS at e16 (else gdata, the slot); PL: the link
// distances in LDS at 0 (else gP16, the slot); positions below s0 link through dprev.
template <bool DL, bool PL>
__device__ __forceinline__ void deep_search(const u32 *gdata, const u16 *gP16, u32 e16, const u32 *dprev, u32 *offg, u32 pre, u32 nb, u32 n,
                                            u32 lim, u32 s0, u32 depth, u32 tid) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  const u32 *const D32 = DL ? (const u32 *)(smem + e16) : gdata;
  const u16 *const P16 = PL ? (const u16 *)smem : gP16;
  for (u32 i = tid; i < nb + (DT - 1) - (nb + DT - 1) % DT; i += DT) {
    u32 const r = deep_search_one(D32, P16, dprev, i, true, pre, nb, n, lim, s0, depth);
    if (i < nb) offg[i] = r;
  }
}

// ---- demand-driven search + parse -------------------------------------------
// The serial LAZY2 parse reads the match at a position only when it gets there, plus the two
// after it.  So instead of searching every position and then walking (steps 3-4 of deep_block),
// the segment walks run first and search on demand: every segment's lane walks as far as the
// memo of searched positions allows; a lane that needs an unsearched position posts it and the
// next two to a queue; all threads then search the queue (lanes = entries) and the walks go on.
// Jacobi rounds as before (a re-walk stops where it meets its old trajectory).  The positions the
// walks consult are the ones the serial parse consults, so records, literals and frames are
// unchanged -- only fewer positions are searched.  Used when the link distances, staged bytes and
// the memo fit in LDS (C5's 16 KiB records with or without the 64 KiB dictionary).
//   memo[i] (u16): 0xFFFF unsearched; else len | (bit length of off + 1) << 8 (the LAZY2 gain)
constexpr u32 MEMO_UNK = 0xFFFFu;
#ifndef ZH_DEEP_DEDUP
#define ZH_DEEP_DEDUP 1  // (with the warm-up below: C5 13.8 / 12.3 -> 15.5 / 13.5 GB/s; alone no change)
#endif
// A position being searched (ZH_DEEP_DEDUP): a lane claims an unsearched position by clearing bit
// 15 of its memo entry with an LDS atomic (known entries never have bit 15 set, so the clear cannot
// touch them), and only the lane that saw MEMO_UNK come back searches it -- lanes and waves that
// need the same position in the same round wait for that one search instead of repeating it.
constexpr u32 MEMO_PEND = 0x7FFFu;
__device__ __forceinline__ bool memo_unknown(u32 m) { return ZH_DEEP_DEDUP ? m >= MEMO_PEND : m == MEMO_UNK; }
#ifndef ZH_DEEP_DQ
#define ZH_DEEP_DQ 3
#endif
constexpr u32 DQ_PER = ZH_DEEP_DQ;  // positions posted per blocked lane (the needed one + lookahead)
#ifndef ZH_DEEP_WARM
#define ZH_DEEP_WARM (-2)  // first-walk warm-up: >= 0 positions, < 0 that many segment lengths
#endif
#ifndef ZH_DEEP_SEG0
#define ZH_DEEP_SEG0 16u
#endif
__device__ __forceinline__ int memo_gain(u32 m) { return (m & 255u) ? 4 * (int)(m & 255u) - (int)(m >> 8) : -1000; }
// Segment length: 16 positions for blocks of <= 16 KiB, doubled per doubling of nb (<= 64), and
// doubled again for a dictionary's first block, whose searches (chains through the dictionary's
// links in L2) are the costly part: fewer segment boundaries, fewer positions walked from wrong
// entries (C5 level 9 with the 64 KiB dictionary 11.2 / 11.5 -> 11.7 / 12.2 GB/s; without a
// dictionary 16 stays faster, 13.8 vs 13.0, as every wave keeps a segment).
__device__ __forceinline__ u32 demand_segl(u32 nb, bool dict) {
  u32 const s = (nb <= 16384u ? ZH_DEEP_SEG0 : nb <= 32768u ? 2u * ZH_DEEP_SEG0 : 4u * ZH_DEEP_SEG0) << (dict ? 1 : 0);
  return s < 64u ? s : 64u;
}
// First-walk warm-up: a segment's first walk starts this many positions before the segment (a
// walk from a wrong position meets the serial parse within a few steps, as K3's FSE chains do),
// so its entry guess is usually the true one and fewer Jacobi iterations follow; positions before
// the segment are walked but not recorded (tools/deep_jacobi_model.c).  The warm-up walks need the
// positions the segment before also needs at the same time, hence ZH_DEEP_DEDUP.  Measured (C5
// level 9, none / COVER dictionary GB/s, tools/gpu_diag.sh c5var): no warm-up 13.8 / 12.3; 16
// positions 15.0 / 12.9; one segment 14.9 / 13.2; two 15.5 / 13.5 (Jacobi iterations 4.3 -> 2.3
// and 3.5 -> 1.5); three 15.5 / 12.9; four 15.2 / 12.1.  Without the claims: 13.1-13.3 / 12.4-12.6.
__device__ __forceinline__ u32 demand_warm(u32 segl) { return ZH_DEEP_WARM < 0 ? (u32)(-(ZH_DEEP_WARM)) * segl : (u32)ZH_DEEP_WARM; }
// LDS bytes the demand path needs above the staged bytes (memo, queue, exits), for nb positions
__device__ __forceinline__ u32 demand_lds(u32 nb) { return ((2u * nb + 15u) & ~15u) + 2u * DQ_PER * DT + 4u * DT; }

// Returns through meta / seq_out / lit_out like step 5 of deep_block.  lds = the free LDS above the
// staged bytes (demand_lds(nb) bytes); misc = deep_block's LDS scalars ([0] the wg_any flag,
// [2] the queue count).
__device__ void deep_parse_demand(const u32 *D32, const u16 *P16, const u32 *dprev, u32 *offg, u8 *lds, u32 *misc, u32 *wsum, u32 pre, u32 nb,
                                  u32 n, u32 lim, u32 s0, u32 depth, u32 tid, ZhWorkspace ws, u32 b, const u8 *stg) {
  u16 *const memo = (u16 *)lds;
  u16 *const q = (u16 *)(lds + ((2u * nb + 15u) & ~15u));
  u32 *const exL = (u32 *)((u8 *)q + 2u * DQ_PER * DT);
  u32 const SEGL = demand_segl(nb, s0 != 0), nseg = (nb + SEGL - 1) / SEGL;
  // unsearched below lim, no match at or past it (the oracle's len[] is 0 there)
  for (u32 i = tid; i < nb; i += DT) memo[i] = pre + i < lim ? (u16)MEMO_UNK : (u16)0;
  if (tid == 0) misc[2] = 0;
#ifdef ZH_STAMPS
  if (tid == 0) misc[4] = 0;
#endif
  __syncthreads();
  u32 const g = tid, S = SEGL * g, SE = min(S + SEGL, nb);
  bool const sv = g < nseg;
#ifdef ZH_STAMPS
  u64 const dm0 = __builtin_amdgcn_s_memtime();
  u32 st_rounds = 0, st_searched = 0, st_walk = 0, st_jac = 0;
  u32 st_adv = 0, st_sync1 = 0, st_srch = 0, st_sync2 = 0;  // (thread 0's wave)
  u64 tq = 0;
#define DMSTAMP(acc) do { u64 const _t = __builtin_amdgcn_s_memtime(); acc += (u32)(_t - tq); tq = _t; } while (0)
#else
#define DMSTAMP(acc) do { } while (0)
#endif
  u64 LM = 0, MM = 0;
  u32 entry = S, ex = S;
  // one walk (first or Jacobi re-walk) of every lane with act0 set; all threads take part in the
  // search rounds.  old: the visited bits of the previous walk (re-walks).
  auto walk = [&](u32 p0, bool act0, u32 warm) {
    u64 const old = act0 ? (LM | MM) : 0ull;
    u64 nl = 0, nm = 0;
    bool act = act0 && p0 < SE, merged = false;
    u32 p = p0 > warm ? p0 - warm : 0u, mpos = 0, ent = p;  // ent: the first position >= S reached
    for (;;) {
      // advance as far as the memo allows
#ifdef ZH_STAMPS
      tq = __builtin_amdgcn_s_memtime();
#endif
      u32 need = ~0u;
      bool adv = act;
      while (__ballot(adv)) {
        if (adv) {
          if (ent < S && p >= S) ent = p;  // (warm-up: below S nothing is recorded)
          if (p >= SE) {
            act = adv = false;
          } else if (p >= S && ((old >> (p - S)) & 1ull)) {  // met the old trajectory: the rest is the old walk's
            merged = true;
            mpos = p - S;
            act = adv = false;
          } else {
            u32 const m0 = memo[p];
            if (memo_unknown(m0)) {
              need = p;
              adv = false;
            } else if ((m0 & 255u) == 0) {
              if (p >= S) nl |= 1ull << (p - S);
              p++;
            } else {
              u32 const m1 = p + 1 < nb ? (u32)memo[p + 1] : 0u, m2 = p + 2 < nb ? (u32)memo[p + 2] : 0u;
              if (memo_unknown(m1) || memo_unknown(m2)) {
                need = memo_unknown(m1) ? p + 1 : p + 2;
                adv = false;
              } else {
                int const g0 = memo_gain(m0);
                if (memo_gain(m1) > g0 + 4 || memo_gain(m2) > g0 + 7) {  // deferred: p is a literal
                  if (p >= S) nl |= 1ull << (p - S);
                  p++;
                } else {
                  if (p >= S) nm |= 1ull << (p - S);
                  p += m0 & 255u;
                }
              }
            }
          }
        }
      }
#if ZH_DEEP_WAVEQ
      // post the needed position and the two after it (the lazy check's lookahead) to this
      // wave's own queue (ballot-compacted), then the wave searches it (lanes = entries): no
      // workgroup barrier, every wave walks at its own pace.  A position another wave is
      // searching at the same time may be searched twice (same result).
      DMSTAMP(st_adv);
      if (!__ballot(act)) break;  // every walk of this wave has left its segment or merged
      u16 *const wq = q + (tid & ~63u) * DQ_PER;
      u32 const lane = tid & 63u;
      u32 nq = 0;
#pragma unroll
      for (u32 t = 0; t < DQ_PER; t++) {
        u32 const x = need + t;
        bool post = need != ~0u && x < nb && memo[x] == MEMO_UNK;
#if ZH_DEEP_DEDUP
        if (post) {  // claim it: UNK -> PEND; a lane that finds it claimed leaves it to its claimant
          u32 const sh = 16u * (x & 1u);
          u32 const o = atomicAnd((u32 *)memo + (x >> 1), ~(0x8000u << sh));
          post = ((o >> sh) & 0xFFFFu) == MEMO_UNK;
        }
#endif
        u64 const bm = __ballot(post);
        u32 const rank = __builtin_amdgcn_mbcnt_hi((u32)(bm >> 32), __builtin_amdgcn_mbcnt_lo((u32)bm, 0u));
        if (post) wq[nq + rank] = (u16)x;
        nq += (u32)__popcll(bm);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#ifdef ZH_STAMPS
      st_rounds++;
      st_searched += nq;
#endif
      for (u32 j0 = 0; j0 < nq; j0 += 64) {
        u32 const j = j0 + lane;
        bool const v = j < nq;
        u32 const x = v ? wq[j] : 0u;
        u32 const r = deep_search_one(D32, P16, dprev, x, v, pre, nb, n, lim, s0, depth);
        if (v) {
          offg[x] = r;
          u32 const l = r & 255u;
          memo[x] = (u16)(l ? l | ((31u - (u32)__builtin_clz((r >> 8) + 1u)) << 8) : 0u);
        }
      }
#if ZH_DEEP_DEDUP
      // (positions this wave waits for may be another wave's: re-read the memo from LDS)
      if (nq == 0) __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
#else
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#endif
      __builtin_amdgcn_wave_barrier();
      DMSTAMP(st_srch);
#else
      // post the needed position and the two after it (the lazy check's lookahead)
      if (need != ~0u) {
#pragma unroll
        for (u32 t = 0; t < DQ_PER; t++) {
          u32 const x = need + t;
          if (x < nb && memo[x] == MEMO_UNK) q[atomicAdd(&misc[2], 1u)] = (u16)x;
        }
      }
      DMSTAMP(st_adv);
      __syncthreads();
      u32 const nq = misc[2];
      DMSTAMP(st_sync1);
      if (nq == 0) break;  // (every lane has finished: no lane needed anything)
#ifdef ZH_STAMPS
      st_rounds++;
      st_searched += nq;
#endif
      // search the queue, lanes = entries (a position queued twice is searched twice, same result)
      for (u32 j0 = 0; j0 < nq; j0 += DT) {
        u32 const j = j0 + tid;
        bool const v = j < nq;
        u32 const x = v ? q[j] : 0u;
        u32 const r = deep_search_one(D32, P16, dprev, x, v, pre, nb, n, lim, s0, depth);
        if (v) {
          offg[x] = r;
          u32 const l = r & 255u;
          memo[x] = (u16)(l ? l | ((31u - (u32)__builtin_clz((r >> 8) + 1u)) << 8) : 0u);
        }
      }
      DMSTAMP(st_srch);
      __syncthreads();
      DMSTAMP(st_sync2);
      if (tid == 0) misc[2] = 0;
      __syncthreads();
#endif
    }
    if (act0) {
      if (merged) {
        u64 const keep = bits_from(mpos);
        LM = nl | (LM & keep);
        MM = nm | (MM & keep);
      } else {
        LM = nl;
        MM = nm;
        ex = p;
      }
      if (warm) entry = ent;  // (every walk ends at or past SE or merged at or past S)
    }
  };
  walk(entry, sv, g == 0 ? 0u : demand_warm(SEGL));
#ifdef ZH_STAMPS
  st_walk = (u32)(__builtin_amdgcn_s_memtime() - dm0);
  u32 st_iter = 0;
  if ((tid & 63u) == 0) atomicMax(&misc[4], st_walk);  // the slowest wave's first walk
#endif
  for (;;) {
    if (sv) exL[g] = ex;
    __syncthreads();
    u32 const ne = g == 0 ? 0u : (sv ? exL[g - 1] : entry);
    bool const ch = sv && ne != entry;
    if (!wg_any(ch, &misc[0], tid)) break;
    walk(ne, ch, 0u);
    if (ch) entry = ne;
#ifdef ZH_STAMPS
    st_iter++;
#endif
  }
#ifdef ZH_STAMPS
  st_jac = (u32)(__builtin_amdgcn_s_memtime() - dm0) - st_walk;
  if (tid == 0) { u32 *dbg = ws.dbg(b); dbg[20] = st_rounds; dbg[21] = st_searched; dbg[22] = st_walk; dbg[23] = st_jac;
                  dbg[24] = st_iter; dbg[25] = misc[4];
                  dbg[0] = st_adv; dbg[1] = st_sync1; dbg[2] = st_srch; dbg[3] = st_sync2; }
#endif
  // ---- records and literals (step 5 of deep_block)
  u32 nm_tot, nl_tot;
  u32 const mbase = wg_excl_scan(sv ? (u32)__popcll(MM) : 0u, wsum, tid, nm_tot);
  u32 const lbase = wg_excl_scan(sv ? (u32)__popcll(LM) : 0u, wsum, tid, nl_tot);
  u64 *seq_out = ws.seq(b);
  u64 mm = MM;
  u32 j = mbase;
  while (mm) {
    u32 const o = (u32)__builtin_ctzll(mm);
    mm &= mm - 1ull;
    u32 const m = S + o;
    u32 const cum = lbase + (u32)__popcll(LM & ~bits_from(o));
    u32 const r = offg[m];
    seq_out[j++] = (u64)cum | ((u64)(r & 255u) << 17) | ((u64)(r >> 8) << 36);
  }
  // literals: every lane its segment's literal bytes (SEGL <= 64 positions)
  u8 *lit_out = ws.lits(b);
  if (sv) {
    u64 lm = LM;
    u32 k = lbase;
    while (lm) {
      u32 const o = (u32)__builtin_ctzll(lm);
      lm &= lm - 1ull;
      lit_out[k++] = stg[pre + S + o];
    }
  }
  if (tid == 0) {
    u32 *meta = ws.meta(b);
    meta[0] = nm_tot;
    meta[1] = nl_tot;
    meta[2] = 0;
  }
}

#ifdef ZH_STAMPS
#define DSTAMP(k)                                                           \
  do {                                                                      \
    u64 _t = __builtin_amdgcn_s_memtime();                                  \
    if (tid == 0) ws.dbg(b)[30 + (k)] = (u32)(_t - dst0);                   \
  } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif
__device__ void deep_block(const ZhBlockDesc &d, ZhWorkspace ws, u32 b, u8 *slot, u32 depth, u32 tid) {
#ifdef ZH_STAMPS
  u64 const dst0 = __builtin_amdgcn_s_memtime();
#endif
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u32 *head = (u32 *)(smem + L_HEAD);
  u8 *lenL = smem + L_HEAD;
  u64 *tm = (u64 *)(smem + L_TM), *lmk = (u64 *)(smem + L_LM);
  u32 *exL = (u32 *)(smem + L_EX), *lpL = (u32 *)(smem + L_LP);
  u32 *wsum = (u32 *)(smem + L_WS), *misc = (u32 *)(smem + L_MISC);
  u32 const lane = tid & 63;
  u32 const pre = d.pre_n, nb = d.n, n = pre + nb;
  u32 *meta = ws.meta(b);
  u8 *stg = slot;
  const u32 *s32 = (const u32 *)slot;
  u32 *prev = (u32 *)(slot + SLOT_PREV), *offg = (u32 *)(slot + SLOT_OFF);

  // ---- 1. stage prefix + block (4 bytes per thread and step), RLE probe, head table cleared
  u8 const first = d.src[0];
  bool same = true;
  u32 const f4 = first * 0x01010101u;
  if ((((uintptr_t)d.src | (uintptr_t)d.pre | pre) & 15) == 0) {
    // 16-B loads: prefix and block both 16-B aligned (contiguous records, dictionary content)
    u32 const nv = (n + 64 + 15) / 16;
#pragma unroll 4
    for (u32 v = tid; v < nv; v += DT) {
      u32 const i = 16 * v;
      uint4 w = make_uint4(0, 0, 0, 0);
      if (i < pre) w = *(const uint4 *)(d.pre + i);
      else if (i + 16 <= n) w = *(const uint4 *)(d.src + (i - pre));
      else {
        u32 t[4] = {0, 0, 0, 0};
        for (u32 k = 0; k < 16 && i + k < n; k++) t[k >> 2] |= (u32)d.src[i + k - pre] << (8 * (k & 3));
        w = make_uint4(t[0], t[1], t[2], t[3]);
      }
      *(uint4 *)(stg + i) = w;
      if (i >= pre && i + 16 <= n) same &= (w.x == f4) & (w.y == f4) & (w.z == f4) & (w.w == f4);
      else if (i >= pre && i < n) {
        u32 const t4[4] = {w.x, w.y, w.z, w.w};
        for (u32 k = 0; k < 16 && i + k < n; k++) same &= ((t4[k >> 2] >> (8 * (k & 3))) & 255u) == first;
      }
    }
  } else {
    for (u32 i = 4 * tid; i < n + 64; i += 4 * DT) {
      u32 w = 0;
#pragma unroll
      for (u32 k = 0; k < 4; k++) {
        u32 const j = i + k;
        u8 const c = j < pre ? d.pre[j] : j < n ? d.src[j - pre] : (u8)0;
        same &= j < pre || j >= n || c == first;
        w |= (u32)c << (8 * k);
      }
      *(u32 *)(stg + i) = w;
    }
  }
  // A dictionary frame's first block starts from the dictionary's precomputed chains (built once
  // per dictionary, zh_deep_dict_kernel): the head table after its positions [0, dd_split), whose
  // links stay in ws.dd_prev; the block links only [dd_split, lim) -- the same chains.
  bool const use_dd = ws.dd_head && (d.flags & ZH_F_DICT) && (d.flags & ZH_F_FIRST) && pre == ws.dd_pre;
  u32 const s0 = use_dd ? ws.dd_split : 0u;
  const u32 *const dprev = ws.dd_prev;
  for (u32 i = tid; i < HSIZE + 4; i += DT) head[i] = use_dd && i < HSIZE ? ws.dd_head[i] : 0u;
  if (wg_any(!same, &misc[0], tid) == false && nb >= 2) {
    if (tid == 0) { meta[0] = 0; meta[1] = 0; meta[2] = 1; }
    return;
  }
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0u;

  __syncthreads();  // staged bytes visible to every wave
  DSTAMP(0);
  // ---- 2. chains of positions [s0, lim); below s0 (a dictionary's precomputed part) the head
  // table already holds every position's latest
  deep_chains(s32, prev, head, (u16 *)(smem + L_TM), s0, lim, tid);
  DSTAMP(1);

  // ---- 3. search.  The links become u16 distances (exact: offsets <= ZH_DEEP_MAXOFF = 65535) in
  // LDS, followed by the staged bytes when both fit (C5's 16 KiB records, with or without the
  // 64 KiB dictionary: every candidate step is LDS-only); otherwise the distances in LDS or the
  // slot and the bytes from the slot (L2).  Generic pointers: one code path for both.
  u32 const E = lim > s0 ? lim - s0 : 0u;  // linked positions [s0, lim)
  u32 const e16 = (2 * E + 15) & ~15u;
  bool const p_lds = e16 <= SEARCH_LDS;
  bool const d_lds = p_lds && e16 + n + 96 <= SEARCH_LDS;
  u16 *const P16w = p_lds ? (u16 *)smem : (u16 *)(slot + SLOT_P16);
  for (u32 i = tid; i < E; i += DT) {
    u32 const c = prev[s0 + i], dl = c ? s0 + i + 1u - c : 0u;
    P16w[i] = (u16)(dl <= ZH_DEEP_MAXOFF ? dl : 0u);
  }
  if (d_lds)
    for (u32 v = tid; 16 * v < n + 80; v += DT) *(uint4 *)(smem + e16 + 16 * v) = *(const uint4 *)(stg + 16 * v);
  __threadfence_block();
  __syncthreads();
#ifndef ZH_DEEP_NO_DEMAND
  // demand-driven search + parse when the memo fits beside the links and bytes in LDS
  u32 const dbase = e16 + ((n + 96 + 15) & ~15u);
  if (d_lds && dbase + demand_lds(nb) <= SEARCH_LDS) {
    DSTAMP(2);  // (search set-up: link distances and bytes in LDS)
    deep_parse_demand((const u32 *)(smem + e16), (const u16 *)smem, dprev, offg, smem + dbase, misc, wsum, pre, nb, n, lim, s0, depth, tid, ws, b,
                      stg);
    DSTAMP(4);
    return;
  }
#endif
  // typed LDS / global variants (a generic pointer makes every access a flat one: measured slower
  // than global memory)
  if (d_lds) deep_search<true, true>(s32, (const u16 *)(slot + SLOT_P16), e16, dprev, offg, pre, nb, n, lim, s0, depth, tid);
  else if (p_lds) deep_search<false, true>(s32, (const u16 *)(slot + SLOT_P16), e16, dprev, offg, pre, nb, n, lim, s0, depth, tid);
  else deep_search<false, false>(s32, (const u16 *)(slot + SLOT_P16), e16, dprev, offg, pre, nb, n, lim, s0, depth, tid);
  __threadfence_block();
  __syncthreads();
  // lengths into LDS for the parse (over the dead search arrays)
  for (u32 i = tid; i < nb; i += DT) lenL[i] = (u8)(offg[i] & 255u);
  __syncthreads();

  DSTAMP(2);
  // ---- 4. take masks (LAZY2 rule on the positions i, i+1, i+2), then the segment walk
  for (u32 i0 = 0; i0 < nb; i0 += DT) {
    u32 const i = i0 + tid;
    u32 const l0 = i < nb ? lenL[i] : 0u, l1 = i + 1 < nb ? lenL[i + 1] : 0u, l2 = i + 2 < nb ? lenL[i + 2] : 0u;
    bool tk = false;
    if (l0) {
      int const g0 = gain_of(l0, offg[i] >> 8);
      int const g1 = l1 ? gain_of(l1, offg[i + 1] >> 8) : -1000, g2 = l2 ? gain_of(l2, offg[i + 2] >> 8) : -1000;
      tk = g1 <= g0 + 4 && g2 <= g0 + 7;
    }
    u64 const bm = __ballot(tk);
    if (lane == 0 && i < nb) tm[i >> 6] = bm;
  }
  __syncthreads();
  u32 const nseg = (nb + 63) / 64;
  u32 const g = tid, S = 64 * g, SE = min(S + 64, nb);
  bool const sv = g < nseg;
  u64 const tmk = sv ? tm[g] : 0ull;
  u64 LM = 0, MM = 0;
  u32 entry = S, ex = S;
  seg_walk64(lenL, tmk, S, SE, entry, sv, LM, MM, ex);
  for (;;) {
    if (sv) exL[g] = ex;
    __syncthreads();
    u32 const ne = g == 0 ? 0u : (sv ? exL[g - 1] : entry);
    bool const ch = sv && ne != entry;
    if (!wg_any(ch, &misc[0], tid)) break;
    if (ch) {
      seg_walk64(lenL, tmk, S, SE, ne, true, LM, MM, ex);
      entry = ne;
    }
  }

  DSTAMP(3);
  // ---- 5. records and literals
  u32 nm_tot, nl_tot;
  u32 const mbase = wg_excl_scan(sv ? (u32)__popcll(MM) : 0u, wsum, tid, nm_tot);
  u32 const lbase = wg_excl_scan(sv ? (u32)__popcll(LM) : 0u, wsum, tid, nl_tot);
  if (sv) {
    lmk[g] = LM;
    lpL[g] = lbase;
  }
  u64 *seq_out = ws.seq(b);
  u64 mm = MM;
  u32 j = mbase;
  while (mm) {
    u32 const o = (u32)__builtin_ctzll(mm);
    mm &= mm - 1ull;
    u32 const m = S + o;
    u32 const cum = lbase + (u32)__popcll(LM & ~bits_from(o));
    seq_out[j++] = (u64)cum | ((u64)lenL[m] << 17) | ((u64)(offg[m] >> 8) << 36);
  }
  __syncthreads();
  u8 *lit_out = ws.lits(b);
  for (u32 i = tid; i < nb; i += DT) {
    u64 const lm = lmk[i >> 6];
    u32 const o = i & 63;
    if ((lm >> o) & 1ull) lit_out[lpL[i >> 6] + (u32)__popcll(lm & ~bits_from(o))] = stg[pre + i];
  }
  if (tid == 0) { meta[0] = nm_tot; meta[1] = nl_tot; meta[2] = 0; }
  DSTAMP(4);
}

}  // namespace

extern "C" __global__ __launch_bounds__(DT) void zh_lz_deep_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws, u8 *scratch,
                                                                  u32 depth) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u32 *misc = (u32 *)(smem + L_MISC);
  u32 const tid = threadIdx.x;
  u8 *const slot = scratch + (size_t)blockIdx.x * SLOT_BYTES;
  if (tid == 0) misc[0] = 0;
  for (;;) {
    if (tid == 0) misc[1] = atomicAdd(ws.ctr, 1u);
    __syncthreads();
    u32 const b = misc[1];
    __syncthreads();
    if (b >= nblocks) break;
    ZhBlockDesc const d = blocks[b];
    if (d.n) deep_block(d, ws, b, slot, depth, tid);
    __syncthreads();  // the slot and LDS are free for the next block
  }
}

#ifdef ZH_STAMPS
extern "C" __global__ void zh_read_deep_fix(u32 *out) { *out = g_deep_fix; g_deep_fix = 0; }
extern "C" u32 zh_deep_fix_host() {
  u32 *d = nullptr, h = 0;
  if (hipMalloc(&d, 4) != hipSuccess) return ~0u;
  hipLaunchKernelGGL(zh_read_deep_fix, dim3(1), dim3(1), 0, 0, d);
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return h;
}
#endif
// A dictionary's deep-matcher chains, built once per dictionary (one workgroup): the last P =
// min(content, ZH_DEEP_PRE) content bytes staged as a record's first block stages them, the links
// of positions [0, split) (split = (P - ZH_HASH_READ) & ~3: every byte they hash is dictionary
// content) into dprev and the head table after them into dhead.
extern "C" __global__ __launch_bounds__(DT) void zh_deep_dict_kernel(const u8 *__restrict__ tail, u32 P, u8 *stg, u32 *dprev, u32 *dhead) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u32 *head = (u32 *)(smem + L_HEAD);
  u32 const tid = threadIdx.x;
  for (u32 i = tid; i < P + 64; i += DT) stg[i] = i < P ? tail[i] : (u8)0;
  for (u32 i = tid; i < HSIZE + 4; i += DT) head[i] = 0;
  __syncthreads();
  u32 const split = (P > ZH_HASH_READ ? P - ZH_HASH_READ : 0u) & ~3u;
  deep_chains((const u32 *)stg, dprev, head, (u16 *)(smem + L_TM), 0, split, tid);
  for (u32 i = tid; i < HSIZE; i += DT) dhead[i] = head[i];
}

namespace zh {
// chains of a dictionary's last min(cn, ZH_DEEP_PRE) content bytes: dprev u32[ZH_DEEP_PRE],
// dhead u32[2^ZH_HASH_LOG_SHORT], stg >= ZH_DEEP_PRE + 64 bytes; P = 0: none (too short)
hipError_t lz_deep_dict_tables(const u8 *content, size_t cn, u8 *stg, u32 *dprev, u32 *dhead, u32 &P, u32 &split, hipStream_t stream) {
  P = (u32)std::min(cn, (size_t)ZH_DEEP_PRE);
  split = (P > ZH_HASH_READ ? P - ZH_HASH_READ : 0u) & ~3u;
  if (split < 64) { P = split = 0; return hipSuccess; }
  hipLaunchKernelGGL(zh_deep_dict_kernel, dim3(1), dim3(DT), DEEP_LDS, stream, content + cn - P, P, stg, dprev, dhead);
  return hipGetLastError();
}

hipError_t lz_deep_init() {
  hipError_t e = hipFuncSetAttribute((const void *)zh_lz_deep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DEEP_LDS);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void *)zh_deep_dict_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DEEP_LDS);
  return e;
}

hipError_t lz_deep_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, int level, hipStream_t stream) {
  int dev = 0, cus = 0;
  if (stream) (void)hipStreamGetDevice(stream, &dev);
  else (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  // one persistent workgroup per CU, at most one per scratch slot of the caller's workspace
  if (!ws.deep_slots || !ws.deep_nslots) return hipErrorInvalidValue;
  u32 const grid = std::min(std::min(nblocks, (u32)cus), ws.deep_nslots);
  hipLaunchKernelGGL(zh_lz_deep_kernel, dim3(grid), dim3(DT), DEEP_LDS, stream, d_descs, nblocks, ws, ws.deep_slots, (u32)ZH_DEEP_DEPTH(level));
  return hipGetLastError();
}
}  // namespace zh
