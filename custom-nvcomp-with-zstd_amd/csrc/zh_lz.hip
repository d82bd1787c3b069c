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
//   exit0  per-position exit of a 16-position parse segment
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
constexpr u32 OFF_EXIT = OFF_INFO + 4 * (ZH_WINDOW + 4);
constexpr u32 OFF_SEG = OFF_EXIT + 2 * ZH_WINDOW;
constexpr u32 OFF_SCAN = OFF_SEG + 4 * NSEG;
constexpr u32 OFF_MISC = OFF_SCAN + 4 * 16;
constexpr u32 K1_LDS = OFF_MISC + 4 * 16;
static_assert(K1_LDS <= 163840, "K1 LDS budget");
static_assert(OFF_TL % 16 == 0 && OFF_INFO % 16 == 0 && OFF_SEG % 16 == 0, "alignment");

__device__ __forceinline__ u32 ld32u(const u32 *in32, u32 p) {
  // unaligned 4-byte load from LDS: two aligned dwords + v_alignbyte
  u32 w0 = in32[p >> 2], w1 = in32[(p >> 2) + 1];
  return __builtin_amdgcn_alignbyte(w1, w0, p & 3);
}

__device__ __forceinline__ u32 hash_long(u64 v) {
  return (u32)((v * ZH_PRIME_LONG) >> (64 - ZH_HASH_LOG_LONG));
}
__device__ __forceinline__ u32 hash_short(u64 v) {
  return (u32)(((v << 24) * ZH_PRIME_SHORT) >> (64 - ZH_HASH_LOG_SHORT));
}

// Length of the common prefix of in[a..] and in[b..] (b < a), capped at
// min(cap, n - a).  lo/hi = the 8 bytes at a (already loaded).
__device__ __forceinline__ u32 match_len(const u32 *in32, u32 a, u32 b, u32 n, u32 lo, u32 hi) {
  u32 const maxl = min((u32)ZH_MAX_MATCH, n - a);
  u32 x = lo ^ ld32u(in32, b);
  if (x) return min((u32)(__builtin_ctz(x) >> 3), maxl);
  x = hi ^ ld32u(in32, b + 4);
  if (x) return min(4u + (__builtin_ctz(x) >> 3), maxl);
  u32 l = 8;
  while (l < maxl) {
    x = ld32u(in32, a + l) ^ ld32u(in32, b + l);
    if (x) { l += __builtin_ctz(x) >> 3; break; }
    l += 4;
  }
  return min(l, maxl);
}

// Best match at p (table state as seen by p's tile).  Returns off<<8 | len.
__device__ __forceinline__ u32 best_at(const u32 *in32, u32 p, u32 n, u32 qL, u32 qS, u32 lo, u32 hi) {
  u32 lL = 0, lS = 0;
  if (qL) { lL = match_len(in32, p, qL - 1, n, lo, hi); if (lL < ZH_MIN_MATCH_LONG) lL = 0; }
  if (qS) { lS = match_len(in32, p, qS - 1, n, lo, hi); if (lS < ZH_MIN_MATCH_SHORT) lS = 0; }
  if (lL && lL >= lS) return ((p - (qL - 1)) << 8) | lL;
  if (lS) return ((p - (qS - 1)) << 8) | lS;
  return 0;
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

extern "C" __global__ __launch_bounds__(K1_THREADS) void zh_lz_kernel(const ZhBlockDesc *__restrict__ blocks, ZhWorkspace ws) {
  extern __shared__ __attribute__((aligned(16))) u8 smem[];
  u8 *in = smem + OFF_IN;
  u32 *in32 = (u32 *)in;
  u32 *TL = (u32 *)(smem + OFF_TL), *TS = (u32 *)(smem + OFF_TS);
  u32 *info = (u32 *)(smem + OFF_INFO);
  u16 *exit0 = (u16 *)(smem + OFF_EXIT);
  u32 *segx = (u32 *)(smem + OFF_SEG);
  u32 *scan = (u32 *)(smem + OFF_SCAN);
  u32 *misc = (u32 *)(smem + OFF_MISC);

  u32 const b = blockIdx.x, tid = threadIdx.x;
  ZhBlockDesc const d = blocks[b];
  u32 const n = d.n;
  if (n == 0) return;
  u32 *meta = ws.meta(b);

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

  u64 *seq_out = ws.seq(b);
  u8 *lit_out = ws.lits(b);
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 nseq_tot = 0, nlit_tot = 0, e_in = 0;

  for (u32 wsb = 0; wsb < n; wsb += ZH_WINDOW) {
    u32 const we = min(wsb + ZH_WINDOW, n);

    // ---- match finding: tiles of 256 positions, lookups before ds_max updates
    for (u32 tb = wsb; tb < we; tb += ZH_TILE) {
      u32 const p = tb + tid;
      bool const act = p < lim;
      u32 hL = 0, hS = 0, qL = 0, qS = 0, lo = 0, hi = 0;
      if (act) {
        lo = ld32u(in32, p);
        hi = ld32u(in32, p + 4);
        u64 const v = ((u64)hi << 32) | lo;
        hL = hash_long(v);
        hS = hash_short(v);
        qL = TL[hL];
        qS = TS[hS];
      }
      __syncthreads();
      u32 inf = 0;
      if (act) {
        atomicMax(&TL[hL], p + 1);
        atomicMax(&TS[hS], p + 1);
        inf = best_at(in32, p, n, qL, qS, lo, hi);
      }
      if (p < we) info[p - wsb] = inf;
      __syncthreads();
    }
    // lazy check of the window's last position needs the first position of the next window
    if (tid == 0) {
      u32 inf = 0;
      if (we < lim) {
        u32 const lo = ld32u(in32, we), hi = ld32u(in32, we + 4);
        u64 const v = ((u64)hi << 32) | lo;
        inf = best_at(in32, we, n, TL[hash_long(v)], TS[hash_short(v)], lo, hi);
      }
      info[we - wsb] = inf;
    }
    __syncthreads();

    // ---- parse: per-segment exits, Jacobi fixed point on segment entries
    u32 const s = wsb + tid * ZH_SEG;
    u32 const se = min(s + ZH_SEG, we);
#define ZH_NEXT(pp, inf_out, take_out)                                  \
  ({                                                                    \
    u32 _i = info[(pp) - wsb];                                          \
    u32 _l = _i & 255u;                                                 \
    bool _t = _l != 0 && (info[(pp) + 1 - wsb] & 255u) <= _l;           \
    inf_out = _i;                                                       \
    take_out = _t;                                                      \
    _t ? (pp) + _l : (pp) + 1;                                          \
  })
    for (int j = (int)ZH_SEG - 1; j >= 0; j--) {
      u32 const p = s + (u32)j;
      if (p < se) {
        u32 inf; bool tk;
        u32 const x = ZH_NEXT(p, inf, tk);
        (void)inf; (void)tk;
        exit0[p - wsb] = (u16)((x >= se ? x : (u32)exit0[x - wsb] + wsb) - wsb);
      }
    }
    __syncthreads();
    u32 entry = max(s, e_in);
    for (;;) {
      u32 const ex = entry < se ? (u32)exit0[entry - wsb] + wsb : entry;
      segx[tid] = ex;
      __syncthreads();
      u32 const ne = tid == 0 ? max(s, e_in) : max(segx[tid - 1], s);
      bool const ch = ne != entry;
      entry = ne;
      if (!__syncthreads_or(ch)) break;
    }
    // segx[] now holds every segment's exit for the converged entries
    u32 const e_out = segx[NSEG - 1];

    // ---- emission: count, scan, write literals and sequence records
    u32 c = 0, l = 0;
    for (u32 p = entry; p < se;) {
      u32 inf; bool tk;
      u32 const x = ZH_NEXT(p, inf, tk);
      (void)inf;
      if (tk) c++; else l++;
      p = x;
    }
    u32 total;
    u32 const ex = wg_excl_scan((c << 16) | l, scan, total);
    u32 lit_i = nlit_tot + (ex & 0xFFFFu), seq_i = nseq_tot + (ex >> 16);
    for (u32 p = entry; p < se;) {
      u32 inf; bool tk;
      u32 const x = ZH_NEXT(p, inf, tk);
      if (tk) {
        seq_out[seq_i++] = (u64)lit_i | ((u64)(inf & 255u) << 17) | ((u64)(inf >> 8) << 25);
      } else {
        lit_out[lit_i++] = in[p];
      }
      p = x;
    }
#undef ZH_NEXT
    nseq_tot += total >> 16;
    nlit_tot += total & 0xFFFFu;
    e_in = e_out;
    __syncthreads();
  }
  if (tid == 0) { meta[0] = nseq_tot; meta[1] = nlit_tot; meta[2] = 0; }
  (void)misc;
}

extern "C" u32 zh_lz_lds_bytes() { return K1_LDS; }

namespace zh {
hipError_t lz_init() { return hipFuncSetAttribute((const void *)zh_lz_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K1_LDS); }
void lz_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, hipStream_t stream) {
  hipLaunchKernelGGL(zh_lz_kernel, dim3(nblocks), dim3(K1_THREADS), K1_LDS, stream, d_descs, ws);
}
}  // namespace zh
