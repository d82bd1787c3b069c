// zh_lz.hip — K1: LZ77 match finding + parse for one <=64 KiB block per workgroup.
//
// Replaces the reference's find_matches_kernel / greedy_parse_kernel /
// build_sequences_gpu_kernel<<<1,1>>> (src/lz77_parallel.cu:26-70, 177-268)
// and the literal gather kernels (src/cuda_zstd_manager.cu:602-723).
//
// Layout (all LDS, 256 threads = 4 wave64, one workgroup per CU):
//   in[]   the block, staged once with 16-B loads (64 KiB)
//   TL/TS  2 x 2^13 u32 hash tables (value = position+1, 0 = empty), updated
//          with ds_max so insertion order inside a tile never matters
//   info[] per-position best match (off<<8 | len) for one 4096-position window
//   lstage one window's literals, staged for coalesced global writes
//   (per-position parse exits live in registers)
// The parse is the serial greedy/lazy-1 parse of oracle/zstd_oracle.c
// (orc_lz_parse) computed as a Jacobi fixed point over 256 segments.
#include "zh_common.h"

namespace {

constexpr u32 K1_THREADS = 256;
constexpr u32 NSEG = ZH_WINDOW / ZH_SEG;  // 256 segments per window, one per thread
static_assert(NSEG == K1_THREADS, "one parse segment per thread");
static_assert(ZH_WINDOW % ZH_TILE == 0 && ZH_TILE == K1_THREADS, "tiles tile windows");

constexpr u32 HL_SIZE = 1u << ZH_HASH_LOG_LONG;
constexpr u32 HS_SIZE = 1u << ZH_HASH_LOG_SHORT;
constexpr u32 OFF_IN = 0;
constexpr u32 OFF_TL = OFF_IN + ZH_BLOCK_MAX + 16;
constexpr u32 OFF_TS = OFF_TL + 4 * HL_SIZE;
constexpr u32 OFF_INFO = OFF_TS + 4 * HS_SIZE;
// candidates per window position, one pad word per 16 so that a thread's 17-entry
// segment slice (stride 17 words across lanes) is free of bank conflicts
constexpr u32 CAND_WORDS = ZH_WINDOW + ZH_WINDOW / 16 + 8;
__device__ __forceinline__ u32 cidx(u32 i) { return i + (i >> 4); }
constexpr u32 OFF_LSTAGE = OFF_INFO + 4 * CAND_WORDS;
// per-thread results of the chain-head extensions (34 bytes used of 36)
constexpr u32 RES_STRIDE = 36;
constexpr u32 OFF_RES = OFF_LSTAGE + ZH_WINDOW;
constexpr u32 OFF_SEG = OFF_RES + RES_STRIDE * K1_THREADS;
constexpr u32 OFF_SCAN = OFF_SEG + 4 * NSEG;
constexpr u32 OFF_MISC = OFF_SCAN + 4 * 16;
constexpr u32 K1_LDS = OFF_MISC + 4 * 16;
static_assert(K1_LDS <= 163840, "K1 LDS budget");
static_assert(OFF_TL % 16 == 0 && OFF_INFO % 16 == 0 && OFF_SEG % 16 == 0, "alignment");

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


// common prefix (0..8) of the 8 own bytes (olo, ohi) with in[b..b+8)
__device__ __forceinline__ u32 prefix8(const u32 *in32, u32 b, u32 olo, u32 ohi) {
  u32 blo, bhi;
  ld64u(in32, b, blo, bhi);
  u32 const x = olo ^ blo, y = ohi ^ bhi;
  return x ? (__builtin_ctz(x) >> 3) : (y ? 4 + (__builtin_ctz(y) >> 3) : 8u);
}

// Extension of a chain head (p, q) whose first 8 bytes match: E = min(common prefix,
// 80, n - p).  80 = cap 64 + 16, so every later position of the segment continuing the
// same offset gets its exact capped length as min(E - i, cap) without touching the
// input again.  Bytes 8..79 are compared as 18 dwords with every load issued up front;
// bytes past the block end read LDS padding/tables and are cut off by n - p.
constexpr u32 EXT_SPAN = ZH_MAX_MATCH + ZH_SEG;
__device__ __forceinline__ u32 ext_head(const u32 *in32, u32 p, u32 q, u32 n) {
  constexpr u32 NW = (EXT_SPAN - 8) / 4;
  u32 const pa = p + 8, qa = q + 8;
  u32 const wp = pa >> 2, sp = pa & 3, wq = qa >> 2, sq = qa & 3;
  u32 A[NW + 1], B[NW + 1];
#pragma unroll
  for (u32 k = 0; k <= NW; k++) { A[k] = in32[wp + k]; B[k] = in32[wq + k]; }
  u32 l = EXT_SPAN;
#pragma unroll
  for (int k = (int)NW - 1; k >= 0; k--) {
    u32 const x = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sp) ^ __builtin_amdgcn_alignbyte(B[k + 1], B[k], sq);
    if (x) l = 8 + 4 * (u32)k + (__builtin_ctz(x) >> 3);
  }
  return min(l, n - p);
}

// Table entries: (position+1) << 16 | 16-bit content tag.  ds_max keeps the latest
// position (the tag only rides along); a tag mismatch proves the common prefix is
// below the table's minimum match, so the candidate is dropped without touching
// the input (same result as the oracle, fewer LDS reads).
__device__ __forceinline__ u32 tag_long(u32 lo, u32 hi) { (void)lo; return hi >> 16; }               // bytes 6..7
__device__ __forceinline__ u32 tag_short(u32 lo, u32 hi) { return (lo >> 24) | ((hi & 0xFFu) << 8); }  // bytes 3..4


// candidates of p against the current tables (tag-filtered), packed cL | cS << 16
__device__ __forceinline__ u32 lookup(const u32 *TL, const u32 *TS, u32 lo, u32 hi, u32 &hL, u32 &hS, u32 &eLnew, u32 &eSnew, u32 p) {
  u64 const v = ((u64)hi << 32) | lo;
  hL = hash_long(v);
  hS = hash_short(v);
  u32 const tL = tag_long(lo, hi), tS = tag_short(lo, hi);
  u32 const eL = TL[hL], eS = TS[hS];
  eLnew = ((p + 1) << 16) | tL;
  eSnew = ((p + 1) << 16) | tS;
  u32 const cL = (eL && (eL & 0xFFFFu) == tL) ? (eL >> 16) : 0u;
  u32 const cS = (eS && (eS & 0xFFFFu) == tS) ? (eS >> 16) : 0u;
  return cL | (cS << 16);
}

// Exclusive scan of one u32 per thread over the 256-thread workgroup.
__device__ __forceinline__ u32 wg_excl_scan(u32 v, u32 *scratch, u32 &total) {
  u32 const lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u32 incl = v;
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    u32 t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) scratch[wave] = incl;
  __syncthreads();
  u32 woff = 0, tot = 0;
#pragma unroll
  for (u32 w = 0; w < K1_THREADS / 64; w++) { u32 s = scratch[w]; woff += (w < wave) ? s : 0; tot += s; }
  total = tot;
  __syncthreads();
  return woff + incl - v;
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

extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_kernel(const ZhBlockDesc *__restrict__ blocks, ZhWorkspace ws) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u8 *in = smem + OFF_IN;
  u32 *in32 = (u32 *)in;
  u32 *TL = (u32 *)(smem + OFF_TL), *TS = (u32 *)(smem + OFF_TS);
  u32 *info = (u32 *)(smem + OFF_INFO);
  u8 *lstage = smem + OFF_LSTAGE;
  u32 *segx = (u32 *)(smem + OFF_SEG);
  u32 *scan = (u32 *)(smem + OFF_SCAN);
  u32 *misc = (u32 *)(smem + OFF_MISC);

  u32 const b = blockIdx.x, tid = threadIdx.x;
  ZhBlockDesc const d = blocks[b];
  u32 const n = d.n;
  if (n == 0) return;
  u32 *meta = ws.meta(b);
#ifdef ZH_STAMPS
  u64 stamp_prev = __builtin_amdgcn_s_memtime();
  u32 st_stage = 0, st_A = 0, st_B1 = 0, st_B = 0, st_J = 0, st_E = 0, st_rounds = 0;
#endif

  // ---- stage the block into LDS (16 B per lane when the source allows it) and probe RLE
  const u8 *src = d.src;
  bool same = true;
  if ((((uintptr_t)src) & 15) == 0) {
    u32 const nv = n >> 4;
    u8 const first = src[0];
    u32 const f4 = first * 0x01010101u;
    for (u32 i = tid; i < nv; i += K1_THREADS) {
      uint4 v = ((const uint4 *)src)[i];
      ((uint4 *)in)[i] = v;
      same &= (v.x == f4) & (v.y == f4) & (v.z == f4) & (v.w == f4);
    }
    for (u32 i = (nv << 4) + tid; i < n; i += K1_THREADS) { u8 c = src[i]; in[i] = c; same &= c == first; }
  } else {
    u8 const first = src[0];
    for (u32 i = tid; i < n; i += K1_THREADS) { u8 c = src[i]; in[i] = c; same &= c == first; }
  }
  if (tid < 16) in[n + tid] = 0;
  for (u32 i = tid; i < HL_SIZE; i += K1_THREADS) TL[i] = 0;
  for (u32 i = tid; i < HS_SIZE; i += K1_THREADS) TS[i] = 0;
  bool const rle = __syncthreads_and(same) && n >= 2;
  if (rle) {
    if (tid == 0) { meta[0] = 0; meta[1] = 0; meta[2] = 1; }
    return;
  }

  ZH_STAMP(st_stage);
  u64 *seq_out = ws.seq(b);
  u8 *lit_out = ws.lits(b);
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 nseq_tot = 0, nlit_tot = 0, e_in = 0;

  for (u32 wsb = 0; wsb < n; wsb += ZH_WINDOW) {
    u32 const we = min(wsb + ZH_WINDOW, n);

    // ---- phase A: insertion in tiles of 256 positions; lookups see earlier tiles only.
    // The next tile's bytes and hashes are computed between the two barriers (software pipeline).
    u32 *cand = info;  // candidates live in info[] until phase B overwrites them
    u32 a_lo = 0, a_hi = 0;
    if (wsb + tid < lim) ld64u(in32, wsb + tid, a_lo, a_hi);
    for (u32 tb = wsb; tb < we; tb += ZH_TILE) {
      u32 const p = tb + tid;
      bool const act = p < lim;
      u32 hL = 0, hS = 0, nL = 0, nS = 0, c = 0;
      if (act) c = lookup(TL, TS, a_lo, a_hi, hL, hS, nL, nS, p);
      if (p < we) cand[cidx(p - wsb)] = c;
      __syncthreads();
      if (act) {
        atomicMax(&TL[hL], nL);
        atomicMax(&TS[hS], nS);
      }
      u32 const pn = p + ZH_TILE;
      if (pn < lim && tb + ZH_TILE < we) ld64u(in32, pn, a_lo, a_hi);
      __syncthreads();
    }
    if (tid == 0) {  // first position of the next window (lazy check at the window end)
      u32 c = 0, hL, hS, nL, nS;
      if (we < lim) { u32 lo, hi; ld64u(in32, we, lo, hi); c = lookup(TL, TS, lo, hi, hL, hS, nL, nS, we); }
      cand[cidx(we - wsb)] = c;
    }
    __syncthreads();

    ZH_STAMP(st_A);
    // ---- phase B (no barriers): match lengths of the thread's own segment (+ the
    // next segment's first position, for the lazy rule), then per-position exits
    u32 const s = wsb + tid * ZH_SEG;
    u32 const se = min(s + ZH_SEG, we);
    u32 inf[ZH_SEG + 1];
    u32 own[ZH_SEG / 4];
    {
      // (1) candidates of the 16 own positions + the next segment's first position,
      //     own bytes, and the first-8-byte prefix of every candidate: all loads
      //     unconditional so they issue back to back
      u32 cv[ZH_SEG + 1];
#pragma unroll
      for (u32 j = 0; j <= ZH_SEG; j++) {
        u32 const p = s + j;
        cv[j] = (p <= se && p < lim) ? cand[cidx(p - wsb)] : 0u;
      }
      u32 ow[ZH_SEG / 4 + 4];
      {
        uint4 const v0 = ((const uint4 *)in)[s >> 4], v1 = ((const uint4 *)in)[(s >> 4) + 1];
        ow[0] = v0.x; ow[1] = v0.y; ow[2] = v0.z; ow[3] = v0.w;
        ow[4] = v1.x; ow[5] = v1.y; ow[6] = v1.z; ow[7] = v1.w;
      }
      u32 pl[ZH_SEG + 1], ps[ZH_SEG + 1];
#pragma unroll
      for (u32 j = 0; j <= ZH_SEG; j++) {
        u32 const olo = __builtin_amdgcn_alignbyte(ow[(j >> 2) + 1], ow[j >> 2], j & 3);
        u32 const ohi = __builtin_amdgcn_alignbyte(ow[(j >> 2) + 2], ow[(j >> 2) + 1], j & 3);
        u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16;
        u32 const xL = prefix8(in32, cL ? cL - 1 : 0u, olo, ohi);
        u32 const xS = prefix8(in32, cS ? cS - 1 : 0u, olo, ohi);
        pl[j] = cL ? xL : 0u;
        ps[j] = (cS && cS != cL) ? xS : 0u;
      }
      ZH_STAMP(st_B1);
      // (2) chains: a candidate whose first 8 bytes match and that continues a
      //     previous-position candidate with the same offset (which also had 8
      //     matching bytes) is a follower; the others with 8 matching bytes are heads
      u32 dL = 0, dS = 0;       // follower bits
      u32 fromSL = 0, fromSS = 0;  // follower whose predecessor is the previous position's S pair
      u64 heads = 0;        // bit j = L head, bit 32 + j = S head
#pragma unroll
      for (u32 j = 0; j <= ZH_SEG; j++) {
        u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16;
        bool const eL = cL && pl[j] == 8, eS = cS && cS != cL && ps[j] == 8;
        u32 const pcL = j ? (cv[j - 1] & 0xFFFFu) : 0u, pcS = j ? (cv[j - 1] >> 16) : 0u;
        bool const peL = j && pcL && pl[j - 1] == 8;
        bool const peS = j && pcS && pcS != pcL && ps[j - 1] == 8;
        if (eL) {
          if (peL && cL == pcL + 1) dL |= 1u << j;
          else if (peS && cL == pcS + 1) { dL |= 1u << j; fromSL |= 1u << j; }
          else heads |= 1ull << j;
        }
        if (eS) {
          if (peL && cS == pcL + 1) dS |= 1u << j;
          else if (peS && cS == pcS + 1) { dS |= 1u << j; fromSS |= 1u << j; }
          else heads |= 1ull << (32 + j);
        }
      }
      // (3) extend the heads, one per lane per iteration (compacted across positions)
      u8 *res = smem + OFF_RES + tid * RES_STRIDE;
      for (u64 hm = heads; hm; hm &= hm - 1) {
        u32 const k = (u32)__builtin_ctzll(hm);
        u32 const j = k & 31u;
        u32 const cw = cand[cidx(s + j - wsb)];
        u32 const c = k >= 32 ? (cw >> 16) : (cw & 0xFFFFu);
        res[k >= 32 ? ZH_SEG + 1 + j : j] = (u8)ext_head(in32, s + j, c - 1, n);
      }
      // (4) lengths in position order: E = exact prefix below 8, the head's extension,
      //     or the predecessor's E - 1; capped length = min(E, 64, n - p)
      u32 rw[(2 * (ZH_SEG + 1) + 3) / 4];
#pragma unroll
      for (u32 k = 0; k < (2 * (ZH_SEG + 1) + 3) / 4; k++) rw[k] = ((const u32 *)res)[k];
      u32 EL = 0, ES = 0;
#pragma unroll
      for (u32 j = 0; j <= ZH_SEG; j++) {
        u32 const p = s + j;
        u32 const cL = cv[j] & 0xFFFFu, cS = cv[j] >> 16;
        u32 const capj = min((u32)ZH_MAX_MATCH, n - p);
        u32 const hLr = (rw[j >> 2] >> (8 * (j & 3))) & 255u;
        u32 const jS = ZH_SEG + 1 + j;
        u32 const hSr = (rw[jS >> 2] >> (8 * (jS & 3))) & 255u;
        u32 nL = pl[j];
        if (dL & (1u << j)) nL = ((fromSL >> j) & 1u ? ES : EL) - 1;
        else if ((heads >> j) & 1u) nL = hLr;
        u32 nS = ps[j];
        if (dS & (1u << j)) nS = ((fromSS >> j) & 1u ? ES : EL) - 1;
        else if ((heads >> (32 + j)) & 1u) nS = hSr;
        if (cS && cS == cL) nS = nL;
        EL = nL; ES = nS;
        u32 const rL = min(nL, capj), rS = min(nS, capj);
        u32 const lL = (cL && rL >= ZH_MIN_MATCH_LONG) ? rL : 0u;
        u32 const lS = (cS && rS >= ZH_MIN_MATCH_SHORT) ? rS : 0u;
        u32 v = 0;
        if (lL && lL >= lS) v = ((p - (cL - 1)) << 8) | lL;
        else if (lS) v = ((p - (cS - 1)) << 8) | lS;
        inf[j] = v;
      }
#pragma unroll
      for (u32 k = 0; k < ZH_SEG / 4; k++) own[k] = ow[k];
    }
    // per-position exits of the own segment (relative to s), backward, in registers
    u32 const slen = se > s ? se - s : 0u;
    u32 ex0[ZH_SEG];
#pragma unroll
    for (int j = (int)ZH_SEG - 1; j >= 0; j--) {
      u32 const l = inf[j] & 255u;
      bool const tk = l != 0 && (inf[j + 1] & 255u) <= l;
      u32 const x = tk ? (u32)j + l : (u32)j + 1;
      u32 v = x;
#pragma unroll
      for (u32 k = j + 1; k < ZH_SEG; k++) v = (x == k && k < slen) ? ex0[k] : v;
      ex0[j] = v;
    }
    ZH_STAMP(st_B);
    u32 entry = max(s, e_in);
    for (;;) {
      u32 ex = entry;
#pragma unroll
      for (u32 k = 0; k < ZH_SEG; k++) ex = (entry == s + k && k < slen) ? s + ex0[k] : ex;
      segx[tid] = ex;
      __syncthreads();
      u32 const ne = tid == 0 ? max(s, e_in) : max(segx[tid - 1], s);
      bool const ch = ne != entry;
      entry = ne;
#ifdef ZH_STAMPS
      st_rounds++;
#endif
      if (!__syncthreads_or(ch)) break;
    }
    ZH_STAMP(st_J);
    // segx[] now holds every segment's exit for the converged entries
    u32 const e_out = segx[NSEG - 1];

    // ---- emission: one walk records match starts / literals as bit masks; literals are
    // staged in LDS and written out coalesced
    u32 tmask = 0, lmask = 0;
    {
      u32 nxt = entry - s;  // >= ZH_SEG when the segment is skipped entirely
#pragma unroll
      for (u32 j = 0; j < ZH_SEG; j++) {
        if (j == nxt && s + j < se) {
          u32 const l = inf[j] & 255u;
          bool const tk = l != 0 && (inf[j + 1] & 255u) <= l;
          if (tk) { tmask |= 1u << j; nxt = j + l; }
          else { lmask |= 1u << j; nxt = j + 1; }
        }
      }
    }
    u32 const c = __builtin_popcount(tmask), l = __builtin_popcount(lmask);
    u32 total;
    u32 const ex = wg_excl_scan((c << 16) | l, scan, total);
    u32 lit_i = ex & 0xFFFFu, seq_i = nseq_tot + (ex >> 16);
#pragma unroll
    for (u32 j = 0; j < ZH_SEG; j++) {
      if (tmask & (1u << j)) {
        seq_out[seq_i++] = (u64)(nlit_tot + lit_i) | ((u64)(inf[j] & 255u) << 17) | ((u64)(inf[j] >> 8) << 25);
      } else if (lmask & (1u << j)) {
        lstage[lit_i++] = (u8)(own[j >> 2] >> (8 * (j & 3)));
      }
    }
    __syncthreads();
    u32 const ltot = total & 0xFFFFu;
    for (u32 i = tid; i < ltot; i += K1_THREADS) lit_out[nlit_tot + i] = lstage[i];
    nseq_tot += total >> 16;
    nlit_tot += total & 0xFFFFu;
    e_in = e_out;
    __syncthreads();
    ZH_STAMP(st_E);
  }
  if (tid == 0) { meta[0] = nseq_tot; meta[1] = nlit_tot; meta[2] = 0; }
#ifdef ZH_STAMPS
  if (tid == 0) {
    u32 *dbg = ws.dbg(b);
    dbg[0] = st_stage; dbg[1] = st_A; dbg[2] = st_B; dbg[3] = st_J; dbg[4] = st_E; dbg[5] = st_rounds; dbg[16] = st_B1;
  }
#endif
  (void)misc;
}

extern "C" u32 zh_lz_lds_bytes() { return K1_LDS; }

namespace zh {
hipError_t lz_init() { return hipFuncSetAttribute((const void *)zh_lz_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K1_LDS); }
void lz_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, hipStream_t stream) {
  hipLaunchKernelGGL(zh_lz_kernel, dim3(nblocks), dim3(K1_THREADS), K1_LDS, stream, d_descs, ws);
}
}  // namespace zh
