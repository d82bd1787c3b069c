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
// owns a slot of a library-held scratch buffer (deep_scratch below): the staged bytes (history or
// dictionary prefix + block, contiguous), prev[] and the per-position offsets.  Per block:
//   1. stage the prefix + block into the slot (and probe RLE); hash every position into prev[]
//   2. chains, wave 0: positions in order, 64 per LDS `ds_max_rtn_u32` on the head table (entry =
//      position + 1): LDS executes one wave's operations in order and a store's lanes one after
//      another, so each lane gets the latest earlier position with its hash -- checked (a lane
//      that got a position >= its own saw a later lane first) with an exact fix-up otherwise
//   3. search, lanes = block positions (all 16 waves): the chain's candidates from global memory
//      (L2: the slot is re-read by its own CU only), the longest common prefix within the cap
//   4. take mask per position (the LAZY2 rule on p, p+1, p+2), then the parse as 64-position
//      segments, one per thread, walked from a guessed entry with Jacobi rounds across the
//      workgroup until every segment's entry is its left neighbour's exit (the serial parse)
//   5. records (walk literals before the match | length | 0 | offset) and the literal bytes
#include "zh_common.h"
#include "zh_hash.h"

#include <mutex>

namespace {

constexpr u32 DT = 1024;                          // threads per workgroup
constexpr u32 HSIZE = 1u << ZH_HASH_LOG_SHORT;    // head table entries (+ a junk slot)
constexpr u32 NSEG = ZH_BLOCK_MAX / 64;           // 64-position parse segments per block
static_assert(NSEG == DT, "one parse segment per thread");
static_assert(ZH_DEEP_PRE <= ZH_BLOCK_MAX && ZH_HIST_BLOCK <= ZH_BLOCK_MAX, "staged prefix fits the slot");
// scratch slot of one workgroup (global memory)
constexpr u32 STG_BYTES = 2 * ZH_BLOCK_MAX + 256;           // staged bytes + zero pad
constexpr u32 SLOT_PREV = STG_BYTES;                        // u32 prev[2 * ZH_BLOCK_MAX]: q + 1, 0 = none
constexpr u32 SLOT_OFF = SLOT_PREV + 4 * 2 * ZH_BLOCK_MAX;  // u32 off[ZH_BLOCK_MAX] per block position
constexpr size_t SLOT_BYTES = SLOT_OFF + 4 * ZH_BLOCK_MAX;
static_assert(SLOT_BYTES % 256 == 0, "slot alignment");
// LDS
constexpr u32 L_HEAD = 0;                  // u32 head[HSIZE + 4] (chains) / u8 len[ZH_BLOCK_MAX] (search, parse)
constexpr u32 L_TM = 4 * (HSIZE + 4);      // u64 take masks per segment
constexpr u32 L_LM = L_TM + 8 * NSEG;      // u64 literal bits per segment
constexpr u32 L_MM = L_LM + 8 * NSEG;      // u64 match-start bits per segment
constexpr u32 L_EX = L_MM + 8 * NSEG;      // u32 walk exit per segment
constexpr u32 L_LP = L_EX + 4 * NSEG;      // u32 literals before the segment
constexpr u32 L_MP = L_LP + 4 * NSEG;      // u32 matches before the segment
constexpr u32 L_WS = L_MP + 4 * NSEG;      // u32[32] per-wave sums
constexpr u32 L_MISC = L_WS + 4 * 32;      // u32[8]: [0] block_any flag, [1] next block
constexpr u32 DEEP_LDS = L_MISC + 4 * 8;
static_assert(4 * (HSIZE + 4) >= ZH_BLOCK_MAX, "len[] reuses the head table");
static_assert(DEEP_LDS <= 160 * 1024, "deep LDS budget");

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

__device__ void deep_block(const ZhBlockDesc &d, ZhWorkspace ws, u32 b, u8 *slot, u32 depth, u32 tid) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u32 *head = (u32 *)(smem + L_HEAD);
  u8 *lenL = smem + L_HEAD;
  u64 *tm = (u64 *)(smem + L_TM), *lmk = (u64 *)(smem + L_LM), *mmk = (u64 *)(smem + L_MM);
  u32 *exL = (u32 *)(smem + L_EX), *lpL = (u32 *)(smem + L_LP), *mpL = (u32 *)(smem + L_MP);
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
  for (u32 i = tid; i < HSIZE + 4; i += DT) head[i] = 0;
  if (wg_any(!same, &misc[0], tid) == false && nb >= 2) {
    if (tid == 0) { meta[0] = 0; meta[1] = 0; meta[2] = 1; }
    return;
  }
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0u;
  // hashes of every position into prev[] (overwritten by the chains below)
  for (u32 p = tid; p < lim; p += DT) {
    u32 lo, hi;
    g64(s32, p, lo, hi);
    prev[p] = hash_short(lo, hi);
  }
  __syncthreads();

  // ---- 2. chains (wave 0): four 64-position steps of atomics in flight, then their checks
  if (tid < 64) {
    constexpr u32 U = 4;
    for (u32 p0 = 0; p0 < lim; p0 += 64 * U) {
      u32 h[U], r[U];
#pragma unroll
      for (u32 u = 0; u < U; u++) {
        u32 const p = p0 + 64 * u + lane;
        h[u] = p < lim ? prev[p] : HSIZE;
      }
#pragma unroll
      for (u32 u = 0; u < U; u++) r[u] = atomicMax(&head[h[u]], p0 + 64 * u + lane + 1);
#pragma unroll
      for (u32 u = 0; u < U; u++) {
        u32 const p = p0 + 64 * u + lane;
        bool const v = p < lim;
        if (__ballot(v && r[u] >= p + 1)) {
          // lanes of one atomic applied out of lane order: prev = the latest earlier lane with the
          // same hash, else the head before the step (the smallest value any lane of the group got)
          u32 mn = ~0u, pm = 0;
          for (u32 k = 0; k < 64; k++) {
            u32 const hk = (u32)__builtin_amdgcn_readlane((int)h[u], (int)k), rk = (u32)__builtin_amdgcn_readlane((int)r[u], (int)k);
            if (hk == h[u]) {
              mn = min(mn, rk);
              if (k < lane) pm = p0 + 64 * u + k + 1;
            }
          }
          r[u] = pm ? pm : mn;
        }
        if (v) prev[p] = r[u];
      }
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- 3. search, lanes = block positions: the chain's first `depth` candidates
  for (u32 i0 = 0; i0 < nb; i0 += DT) {
    u32 const i = i0 + tid, p = pre + i;
    bool act = i < nb && p < lim;
    u32 olo = 0, ohi = 0, c = 0;
    if (act) {
      g64(s32, p, olo, ohi);
      c = prev[p];
    }
    u32 best = 0, bo = 0, dd = 0;
    act = act && c != 0 && p - (c - 1u) <= ZH_DEEP_MAXOFF;
    while (__ballot(act)) {
      if (act) {
        u32 const q = c - 1u;
        u32 const cn = prev[q];
        u32 clo, chi;
        g64(s32, q, clo, chi);
        u32 const x = olo ^ clo, y = ohi ^ chi;
        u32 l = x ? (u32)__builtin_ctz(x) >> 3 : y ? 4u + ((u32)__builtin_ctz(y) >> 3) : 8u;
        if (l == 8) {
          for (u32 k = 8; k < ZH_MAX_MATCH && p + k < n; k += 8) {
            u32 alo, ahi, blo, bhi;
            g64(s32, p + k, alo, ahi);
            g64(s32, q + k, blo, bhi);
            u32 const x2 = alo ^ blo, y2 = ahi ^ bhi;
            if (x2 | y2) {
              l = k + (x2 ? (u32)__builtin_ctz(x2) >> 3 : 4u + ((u32)__builtin_ctz(y2) >> 3));
              break;
            }
            l = k + 8;
          }
        }
        l = min(min(l, (u32)ZH_MAX_MATCH), n - p);
        if (l >= ZH_MIN_MATCH_SHORT && l > best) {
          best = l;
          bo = p - q;
        }
        dd++;
        c = cn;
        act = best < ZH_MAX_MATCH && dd < depth && c != 0 && p - (c - 1u) <= ZH_DEEP_MAXOFF;
      }
    }
    if (i < nb) {
      lenL[i] = (u8)best;
      offg[i] = bo;
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- 4. take masks (LAZY2 rule on the positions i, i+1, i+2), then the segment walk
  for (u32 i0 = 0; i0 < nb; i0 += DT) {
    u32 const i = i0 + tid;
    u32 const l0 = i < nb ? lenL[i] : 0u, l1 = i + 1 < nb ? lenL[i + 1] : 0u, l2 = i + 2 < nb ? lenL[i + 2] : 0u;
    bool tk = false;
    if (l0) {
      int const g0 = gain_of(l0, offg[i]);
      int const g1 = l1 ? gain_of(l1, offg[i + 1]) : -1000, g2 = l2 ? gain_of(l2, offg[i + 2]) : -1000;
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

  // ---- 5. records and literals
  u32 nm_tot, nl_tot;
  u32 const mbase = wg_excl_scan(sv ? (u32)__popcll(MM) : 0u, wsum, tid, nm_tot);
  u32 const lbase = wg_excl_scan(sv ? (u32)__popcll(LM) : 0u, wsum, tid, nl_tot);
  if (sv) {
    lmk[g] = LM;
    lpL[g] = lbase;
    mpL[g] = mbase;
  }
  u64 *seq_out = ws.seq(b);
  u64 mm = MM;
  u32 j = mbase;
  while (mm) {
    u32 const o = (u32)__builtin_ctzll(mm);
    mm &= mm - 1ull;
    u32 const m = S + o;
    u32 const cum = lbase + (u32)__popcll(LM & ~bits_from(o));
    seq_out[j++] = (u64)cum | ((u64)lenL[m] << 17) | ((u64)offg[m] << 36);
  }
  __syncthreads();
  u8 *lit_out = ws.lits(b);
  for (u32 i = tid; i < nb; i += DT) {
    u64 const lm = lmk[i >> 6];
    u32 const o = i & 63;
    if ((lm >> o) & 1ull) lit_out[lpL[i >> 6] + (u32)__popcll(lm & ~bits_from(o))] = stg[pre + i];
  }
  if (tid == 0) { meta[0] = nm_tot; meta[1] = nl_tot; meta[2] = 0; }
  (void)mpL;
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

namespace zh {
// Library-held scratch of the deep matcher: one slot per workgroup (one per CU), allocated on a
// device's first deep launch and kept (~0.9 MB per CU).  Not part of the caller's workspace:
// the temp size of the reference API does not depend on the level.
static u8 *deep_scratch(int dev, u32 slots) {
  static std::mutex mu;
  static u8 *ptr[64] = {};
  static u32 have[64] = {};
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (have[dev] < slots) {
    if (ptr[dev]) (void)hipFree(ptr[dev]);
    ptr[dev] = nullptr;
    have[dev] = 0;
    if (hipMalloc(&ptr[dev], SLOT_BYTES * slots) != hipSuccess) return nullptr;
    have[dev] = slots;
  }
  return ptr[dev];
}

hipError_t lz_deep_init() { return hipFuncSetAttribute((const void *)zh_lz_deep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DEEP_LDS); }

hipError_t lz_deep_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, int level, hipStream_t stream) {
  int dev = 0, cus = 0;
  if (stream) (void)hipStreamGetDevice(stream, &dev);
  else (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  u32 const grid = std::min(nblocks, (u32)cus);
  u8 *scr = deep_scratch(dev, (u32)cus);
  if (!scr) return hipErrorOutOfMemory;
  hipLaunchKernelGGL(zh_lz_deep_kernel, dim3(grid), dim3(DT), DEEP_LDS, stream, d_descs, nblocks, ws, scr, (u32)ZH_DEEP_DEPTH(level));
  return hipGetLastError();
}
}  // namespace zh
