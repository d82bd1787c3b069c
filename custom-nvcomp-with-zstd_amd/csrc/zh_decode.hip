// zh_decode.hip — gfx950 Zstandard decoder: RFC 8878 frames of any
// origin (this library's or libzstd's), one workgroup of one wave64 per input buffer.
//
// Replaces the reference's GPU decompression path (src/cuda_zstd_manager.cu:3194-3706,
// 4292-5530: block walk, literal/sequence decode, execution; Huffman decoder
// src/cuda_zstd_huffman.cu:1572-1833, 2204-2438; FSE decoder src/cuda_zstd_fse.cu:3839-4300;
// sequence execution src/cuda_zstd_sequence.cu:203-575).  The reference decodes one
// block per host round trip with ~10 launches; here a whole batch of frames is one
// launch and nothing returns to the host until the sizes/statuses are ready.
//
// Per input buffer (frames + skippable frames, concatenated), per block:
//   literals   raw / RLE are used in place; Huffman (direct or FSE-compressed weights,
//              1 or 4 streams, treeless reuse) decoded by lanes 0..3 into the item's
//              workspace slot
//   sequences  NCount / RLE / predefined / repeat tables (LDS), the interleaved FSE
//              bitstream decoded serially (the format has one state chain per table),
//              repcodes resolved on the fly, records (ll | ml-3 | offset) to the slot
//   execution  the block's output is produced through a 4 KiB LDS window: the wave
//              copies one sequence at a time with lanes = bytes (a match byte reads
//              position start - off + (i mod off), so overlapping copies need no
//              byte-serial loop); sources before the window come from the already
//              flushed output in HBM, sources inside it from LDS (a wave's LDS ops
//              execute in order); each full window is flushed with coalesced stores
//   checksum   XXH64 of the frame's output (4 lanes = the 4 accumulators), low 32 bits
//              compared with the frame's checksum field
// Error behaviour follows libzstd 1.4.9 (ZSTD_decompress): corrupt input -> ERROR_CORRUPT_DATA,
// too little output capacity -> ERROR_BUFFER_TOO_SMALL, bad magic -> ERROR_INVALID_MAGIC,
// checksum mismatch -> ERROR_CHECKSUM_FAILED, a frame naming another (or no given) dictionary ->
// ERROR_DICTIONARY_MISMATCH.  With a dictionary (RFC 8878 §5) its content precedes every frame
// and a formatted one's tables and repcodes seed the frame state.
#include "zh_common.h"
#include "zh_launch.h"
#include "zh_pipe.h"
#include "zh_xxh64.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>

typedef int64_t s64;

// 1: the quad sequence kernel (four lanes per buffer); 0: the one-lane-per-buffer kernel
#ifndef ZH_EXEC_CHASE
#define ZH_EXEC_CHASE 1  // (with the start bitmap) in-window sources followed in pass A; no pass B
#endif
#ifndef ZH_DEC_HUFPAR
#define ZH_DEC_HUFPAR 1  // segment-parallel Huffman literal streams (0: one lane per stream)
#endif
#ifndef ZH_DEC_QUAD
#define ZH_DEC_QUAD 1
#endif

namespace {

constexpr u32 DEC_THREADS = 64;
#ifndef ZH_DEC_STAGE
#define ZH_DEC_STAGE 8192
#endif
#ifndef ZH_HSTAGE
#define ZH_HSTAGE 1024
#endif
constexpr u32 DEC_STAGE = ZH_DEC_STAGE;  // output window (LDS)
constexpr u32 HSTAGE = ZH_HSTAGE;        // per-stream LDS stage of a Huffman stream
constexpr u32 SSTAGE = 4096;      // LDS stage of the sequence bitstream
constexpr u32 HUF_LOG_MAX = 11;   // RFC 8878 §4.2.1: Max_Number_of_Bits <= 11
constexpr u32 BLOCKSIZE_MAX = 128u * 1024u;
constexpr u32 OFF_LIMIT = 1u << 30;  // offsets are stored in 30 bits (windows up to 1 GiB)

enum : u32 { ST_OK = 0, ST_INVALID = 2, ST_MAGIC = 5, ST_CORRUPT = 6, ST_SMALL = 7, ST_DICT = 9, ST_CHECKSUM = 10 };

// sequence code tables (RFC 8878 §3.1.1.3.2.1.1): baseline | extra bits << 24
__constant__ u32 c_LL_info[36] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
    16 | 1u << 24, 18 | 1u << 24, 20 | 1u << 24, 22 | 1u << 24, 24 | 2u << 24, 28 | 2u << 24, 32 | 3u << 24, 40 | 3u << 24,
    48 | 4u << 24, 64 | 6u << 24, 128 | 7u << 24, 256 | 8u << 24, 512 | 9u << 24, 1024 | 10u << 24, 2048 | 11u << 24,
    4096 | 12u << 24, 8192 | 13u << 24, 16384 | 14u << 24, 32768 | 15u << 24, 65536 | 16u << 24};
__constant__ u32 c_ML_info[53] = {
    3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
    35 | 1u << 24, 37 | 1u << 24, 39 | 1u << 24, 41 | 1u << 24, 43 | 2u << 24, 47 | 2u << 24, 51 | 3u << 24, 59 | 3u << 24,
    67 | 4u << 24, 83 | 4u << 24, 99 | 5u << 24, 131 | 7u << 24, 259 | 8u << 24, 515 | 9u << 24, 1027 | 10u << 24,
    2051 | 11u << 24, 4099 | 12u << 24, 8195 | 13u << 24, 16387 | 14u << 24, 32771 | 15u << 24, 65539 | 16u << 24};
// predefined distributions (RFC 8878 §3.1.1.3.2.2.1-3)
__constant__ s16 c_LL_norm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ s16 c_ML_norm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                  1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ s16 c_OF_norm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// table slots: LL, OF, ML (the order of the Symbol_Compression_Modes fields)
constexpr u32 TAB_LL = 0, TAB_OF = 1, TAB_ML = 2;
__device__ __forceinline__ u32 tab_off(u32 t) { return t == 0 ? 0u : t == 1 ? 512u : 768u; }
__device__ __forceinline__ u32 tab_maxsv(u32 t) { return t == 0 ? 35u : t == 1 ? 31u : 52u; }
__device__ __forceinline__ u32 tab_maxlog(u32 t) { return t == 1 ? 8u : 9u; }
constexpr u32 TAB_NONE = 0xFFFFu, TAB_PREDEF = 0xFFFEu;  // tkind; else RLE symbol | 0x100, or 0 = FSE

// The union's three views are used one after the other inside a block: Huffman decode,
// sequence bitstream, execution window.  TAB = the split pipeline's tables-only pass
// (zh_dec_tables_kernel): no literals, no execution, so the union shrinks to the 320-byte stage
// of the table descriptions and the window arrays to stubs (8.5 KB instead of 16.8: twice the
// workgroups per CU).
template <bool TAB>
struct DecLdsT {
  static constexpr bool kLitStage = false;
  static constexpr bool kStartMap = false;
  static constexpr bool kTablesOnly = TAB;
  u32 fse[1280];  // LL [0,512) OF [512,768) ML [768,1280): sym | nbBits << 8 | newState << 16
  union {
    struct {
      u16 dt[TAB ? 2 : (1 << HUF_LOG_MAX)];  // Huffman decode table: sym | nbBits << 8
      u8 hs[4][TAB ? 4 : HSTAGE + 16];       // staged bytes of the 4 streams
    } h;
    u8 sstage[TAB ? 336 : SSTAGE + 16];      // staged bytes of the sequence bitstream (TAB: table descriptions)
    u8 out[TAB ? 16 : DEC_STAGE + 16];       // execution window
  } u;
  u32 wt[64];       // FSE table of the Huffman weights (log <= 6)
  u8 symlist[256];  // Huffman build: symbols grouped by weight
  s32 wvs[TAB ? 4 : 68];  // execution window: virtual start of each sequence (binary search keys)
  u32 wll[TAB ? 1 : 64], wlit[TAB ? 1 : 64], woff[TAB ? 1 : 64];  // execution window: literal length, first literal, offset
  u32 info[2][64];  // LL / ML code info (baseline | bits << 24), copied from constants
  s16 norm[256];    // NCount scratch
  u16 next[256];    // FSE build scratch (symbolNext)
  u8 hufw[256];     // Huffman weights of the last table (treeless literals rebuild from them)
  u32 tlog[3];      // table logs
  u32 tkind[3];     // TAB_NONE / TAB_PREDEF / RLE symbol | 0x100 / 0 = FSE
#ifdef ZH_STAMPS
  u64 lst_t[4];     // (-DZH_STAMPS) decode_literals: s_memtime after the header, weights, table, streams
#endif
  u32 bld[3];       // sequence tables whose build is left to build_dtable_wave (norm in norm + 64 t)
  u32 hlog, hnsym, hvalid;
  u32 err;   // serial-section status (lane 0 writes)
  u32 used;  // serial-section byte count (lane 0 writes)
};
using DecLds = DecLdsT<false>;
using DecLdsTab = DecLdsT<true>;

__device__ __forceinline__ u32 hb32(u32 v) { return 31u - (u32)__builtin_clz(v); }
__device__ __forceinline__ u32 lane_id() { return threadIdx.x; }

// ---- global reads of compressed bytes --------------------------------------------------
// 8 bytes at p, all of them inside the input: only aligned dwords that hold at least one
// of those bytes are loaded, so a read never touches a page the buffer does not reach.
__device__ __forceinline__ u64 ldg64(const u8 *p) {
  uintptr_t const a = (uintptr_t)p;
  const u32 *w = (const u32 *)(a & ~(uintptr_t)3);
  u32 const sh = (u32)(a & 3);
  u32 const w0 = w[0], w1 = w[1];
  u32 w2 = 0;
  if (sh) w2 = w[2];
  u32 const lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  u32 const hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return ((u64)hi << 32) | lo;
}
// Header fields are read as wave-uniform values (readfirstlane): every lane walks the same
// frame, so the whole control flow of the kernel runs on the scalar unit (s_cbranch on
// SCC, no exec-mask bookkeeping).  Inside lane-0-only sections the first active lane is 0.
__device__ __forceinline__ u32 uni(u32 v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ u64 uni64(u64 v) { return ((u64)uni((u32)(v >> 32)) << 32) | uni((u32)v); }
__device__ __forceinline__ u32 ub(const u8 *p) { return uni(p[0]); }
__device__ __forceinline__ u32 rd16(const u8 *p) { return uni(p[0] | (u32)p[1] << 8); }
__device__ __forceinline__ u32 rd24(const u8 *p) { return uni(p[0] | (u32)p[1] << 8 | (u32)p[2] << 16); }
__device__ __forceinline__ u32 rd32(const u8 *p) { return uni(p[0] | (u32)p[1] << 8 | (u32)p[2] << 16 | (u32)p[3] << 24); }

// Backward bit reader (RFC 8878 §4.1: streams are read from the end; the last byte's
// highest set bit marks the start).  pos = bits not yet consumed; reads past the start
// return zeros and drive pos negative (libzstd's "overflow").
struct BitRev {
  const u8 *p;
  s32 n, pos, cb;
  u64 c;  // bytes [cb, cb + 8) of the stream (zero-extended for streams under 8 bytes)
  __device__ __forceinline__ void fill(s32 b) {
    cb = b;
    if (n >= 8) {
      c = ldg64(p + b);
    } else {
      u64 v = 0;
      for (s32 i = 0; i < n; i++) v |= (u64)p[i] << (8 * i);
      c = v;
    }
  }
  __device__ __forceinline__ bool init(const u8 *s, u32 sz) {
    p = s;
    n = (s32)sz;
    pos = 0;
    cb = 0;
    c = 0;
    if (sz == 0) return false;
    u32 const last = s[sz - 1];
    if (!last) return false;
    pos = 8 * ((s32)sz - 1) + (s32)hb32(last);
    fill(n >= 8 ? n - 8 : 0);
    return true;
  }
  // the k (<= 56) bits below pos, bit pos-1 as the MSB
  __device__ __forceinline__ u64 peek(u32 k) {
    s32 const lo = pos - (s32)k;
    if (lo < 8 * cb) {
      s32 nb = ((pos + 7) >> 3) - 8;
      nb = nb < 0 ? 0 : nb;
      if (n < 8) nb = 0;
      else if (nb > n - 8) nb = n - 8;
      if (nb != cb) fill(nb);
    }
    u64 const m = k ? (~0ull >> (64 - k)) : 0ull;
    if (lo >= 8 * cb) return (c >> (lo - 8 * cb)) & m;
    s32 const sh = 8 * cb - lo;  // cb == 0 here: missing low bits are zeros
    return sh < 64 ? (c << sh) & m : 0ull;
  }
  __device__ __forceinline__ u32 read(u32 k) {
    u32 const v = (u32)peek(k);
    pos -= (s32)k;
    return v;
  }
};

// ---- LDS-staged streams: the decoders read their bitstreams from LDS; a wave copies the
// next stretch of a stream in one burst (all loads in flight), so a refill costs one HBM
// round trip per stage instead of one per 8 bytes.
// Copy stream bytes [lo, hi) of p to stage (wave-cooperative: every lane calls it).  Aligned
// dword loads only; the dword after a word is read only when it still holds a range byte.
__device__ void stage_copy(u8 *stage, const u8 *p, u32 lo, u32 hi) {
  u32 const lane = lane_id();
  const u8 *const s0 = p + lo;
  u32 const sa = (u32)((uintptr_t)s0 & 3u);
  const u32 *const s32 = (const u32 *)(s0 - sa);
  u32 const nb = hi - lo, ndw = (nb + 3) >> 2, lim = sa + nb;
  u32 *const d32 = (u32 *)stage;
  constexpr u32 U = 4;
  for (u32 w0 = 0; w0 < ndw; w0 += 64 * U) {
    u32 v[U];
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      v[u] = 0;
      if (w < ndw) {
        u32 const A = s32[w];
        u32 const B = (sa && 4 * (w + 1) < lim) ? s32[w + 1] : 0u;
        v[u] = __builtin_amdgcn_alignbyte(B, A, sa);
      }
    }
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      if (w < ndw) d32[w] = v[u];
    }
  }
}

// 8 bytes at byte offset o of a 4-aligned LDS stage (padded by 12 bytes)
__device__ __forceinline__ u64 lds64(const u8 *stage, u32 o) {
  const u32 *w = (const u32 *)(stage + (o & ~3u));
  u32 const sh = o & 3u;
  u32 const w0 = w[0], w1 = w[1], w2 = w[2];
  return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// Backward bit reader over an LDS stage holding stream bytes [slo, min(n, slo + cap)).
// peek() reports a needed restage instead of reading below slo.
struct BitRevS {
  const u8 *p;
  s32 n, pos, cb, slo;
  u64 c;  // bytes [cb, cb + 8) (zero-extended for streams under 8 bytes)
  template <bool UNI = false>
  __device__ __forceinline__ bool start(const u8 *s, u32 sz) {
    p = s;
    n = (s32)sz;
    pos = 0;
    cb = n + 1;   // no container yet
    slo = n + 1;  // nothing staged
    c = 0;
    if (sz == 0) return false;
    u32 const last = UNI ? ub(s + sz - 1) : s[sz - 1];
    if (!last) return false;
    pos = 8 * ((s32)sz - 1) + (s32)hb32(last);
    return true;
  }
  // container base the next read of k bits needs (valid when lo < 8 cb)
  __device__ __forceinline__ s32 want(u32 k) const {
    s32 nb = ((pos + 7) >> 3) - 8;
    nb = nb < 0 ? 0 : nb;
    return n < 8 ? 0 : (nb > n - 8 ? n - 8 : nb);
  }
  // stage window for a restage: [lo, hi)
  __device__ __forceinline__ void stage_range(s32 cap, u32 &lo, u32 &hi) const {
    s32 h = n < 8 ? n : want(0) + 8;
    s32 l = h - cap;
    lo = (u32)(l < 0 ? 0 : l);
    hi = (u32)h;
  }
  // refill the container if the next k bits need it; false = restage first.  UNI: every
  // lane holds the same reader (the sequence decoder): the container is made uniform too.
  template <bool UNI = false>
  __device__ __forceinline__ bool ensure(const u8 *stage, u32 k) {
    s32 const lo = pos - (s32)k;
    if (lo >= 8 * cb) return true;
    s32 const nb = want(k);
    if (nb == cb) return true;  // (reads below the stream start: zeros)
    if (nb < slo) return false;
    c = lds64(stage, (u32)(nb - slo));
    if (UNI) c = ((u64)uni((u32)(c >> 32)) << 32) | uni((u32)c);
    if (n < 8) c &= ~0ull >> (64 - 8 * n);
    cb = nb;
    return true;
  }
  __device__ __forceinline__ u64 bits(u32 k) const {
    s32 const lo = pos - (s32)k;
    u64 const m = k ? (~0ull >> (64 - k)) : 0ull;
    if (lo >= 8 * cb) return (c >> (lo - 8 * cb)) & m;
    s32 const sh = 8 * cb - lo;  // cb == 0: missing low bits are zeros
    return sh < 64 ? (c << sh) & m : 0ull;
  }
};

// Forward 32-bit window at a bit position (NCount headers), zeros past the end.
__device__ __forceinline__ u32 fwd32(const u8 *p, u32 avail, u32 bitpos) {
  u32 const b = bitpos >> 3;
  u64 v = 0;
#pragma unroll
  for (u32 i = 0; i < 5; i++)
    if (b + i < avail) v |= (u64)p[b + i] << (8 * i);
  return (u32)(v >> (bitpos & 7));
}

// FSE_readNCount (libzstd lib/common/entropy_common.c, RFC 8878 §4.1.1).  Fills
// norm[0..maxSV] (zeros past the last coded symbol).  Returns bytes used, 0 on error.
__device__ u32 read_ncount(const u8 *p, u32 avail, s16 *norm, u32 maxSV, u32 maxLog, u32 &tableLog) {
  if (avail == 0) return 0;
  u32 nbBits = (fwd32(p, avail, 0) & 15u) + 5u;
  if (nbBits > maxLog) return 0;
  tableLog = nbBits;
  u32 bitpos = 4;
  s32 remaining = (1 << nbBits) + 1;
  s32 threshold = 1 << nbBits;
  nbBits++;
  u32 sym = 0;
  bool prev0 = false;
  while (remaining > 1 && sym <= maxSV) {
    if (prev0) {
      u32 n0 = sym, r;
      do {
        r = fwd32(p, avail, bitpos) & 3u;
        bitpos += 2;
        n0 += r;
      } while (r == 3 && bitpos < 8 * avail + 32);
      if (n0 > maxSV) return 0;
      while (sym < n0) norm[sym++] = 0;
    }
    u32 const bs = fwd32(p, avail, bitpos);
    s32 const mx = (2 * threshold - 1) - remaining;
    s32 count;
    if ((s32)(bs & (u32)(threshold - 1)) < mx) {
      count = (s32)(bs & (u32)(threshold - 1));
      bitpos += nbBits - 1;
    } else {
      count = (s32)(bs & (u32)(2 * threshold - 1));
      if (count >= threshold) count -= mx;
      bitpos += nbBits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[sym++] = (s16)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      nbBits--;
      threshold >>= 1;
    }
  }
  if (remaining != 1) return 0;
  for (u32 s = sym; s <= maxSV; s++) norm[s] = 0;
  u32 const used = (bitpos + 7) >> 3;
  return used <= avail ? used : 0u;
}

// FSE_buildDTable (libzstd lib/common/fse_decompress.c): T[u] = sym | nbBits << 8 | newState << 16.
__device__ bool build_dtable(u32 *T, const s16 *norm, u32 maxSV, u32 tlog, u16 *next) {
  u32 const size = 1u << tlog, mask = size - 1;
  u32 high = size - 1;
  for (u32 s = 0; s <= maxSV; s++) {
    if (norm[s] == -1) {
      T[high--] = s;
      next[s] = 1;
    } else {
      next[s] = (u16)(norm[s] > 0 ? norm[s] : 0);
    }
  }
  u32 const step = (size >> 1) + (size >> 3) + 3;
  u32 pos = 0;
  for (u32 s = 0; s <= maxSV; s++) {
    s32 const k = norm[s];
    for (s32 i = 0; i < k; i++) {
      T[pos] = s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  }
  if (pos != 0) return false;
  for (u32 u = 0; u < size; u++) {
    u32 const s = T[u] & 0xFFu;
    u32 const ns = next[s]++;
    u32 const nb = tlog - hb32(ns);
    T[u] = s | nb << 8 | ((ns << nb) - size) << 16;
  }
  return true;
}

// m mod d for m < 2^18 (float quotient, one correction each way)
__device__ __forceinline__ u32 umod(u32 m, u32 d) {
  u32 const q = (u32)((float)m * __builtin_amdgcn_rcpf((float)d));
  s32 r = (s32)(m - q * d);
  if (r < 0) r += (s32)d;
  if ((u32)r >= d) r -= (s32)d;
  return (u32)r;
}

// ---- Huffman ------------------------------------------------------------------------------
// HUF_readStats (libzstd lib/common/entropy_common.c) on lane 0: weights -> L.hufw, L.hlog,
// L.hnsym.  Returns the header bytes consumed, 0 on error.
template <class LDS>
__device__ __noinline__ u32 huf_read_weights(LDS &L, const u8 *p, u32 avail) {
  if (avail < 1) return 0;
  u32 const hb = p[0];
  u32 nw = 0, used;
  for (u32 i = 0; i < 256; i++) L.hufw[i] = 0;
  if (hb >= 128) {
    nw = hb - 127;
    used = 1 + (nw + 1) / 2;
    if (used > avail) return 0;
    for (u32 i = 0; i < nw; i++) {
      u32 const b = p[1 + i / 2];
      L.hufw[i] = (u8)((i & 1) ? (b & 15u) : (b >> 4));
    }
  } else {
    used = 1 + hb;
    if (used > avail) return 0;
    u32 wlog;
    u32 const nc = read_ncount(p + 1, hb, L.norm, 255, 6, wlog);
    if (!nc) return 0;
    if (!build_dtable(L.wt, L.norm, 255, wlog, L.next)) return 0;
    BitRev r;
    if (!r.init(p + 1 + nc, hb - nc)) return 0;
    u32 s1 = r.read(wlog), s2 = r.read(wlog);
    // two interleaved states; the stream ends when a state update overflows
    for (;;) {
      if (nw > 253) return 0;
      u32 e = L.wt[s1];
      L.hufw[nw++] = (u8)(e & 0xFF);
      s1 = (e >> 16) + r.read((e >> 8) & 0xFF);
      if (r.pos < 0) { L.hufw[nw++] = (u8)(L.wt[s2] & 0xFF); break; }
      e = L.wt[s2];
      L.hufw[nw++] = (u8)(e & 0xFF);
      s2 = (e >> 16) + r.read((e >> 8) & 0xFF);
      if (r.pos < 0) { L.hufw[nw++] = (u8)(L.wt[s1] & 0xFF); break; }
    }
  }
  // only the count of weight-1 symbols is checked: no rank array (a dynamically indexed
  // private array lives in scratch)
  u32 sum = 0, rs1 = 0;
  for (u32 i = 0; i < nw; i++) {
    u32 const w = L.hufw[i];
    if (w >= 12) return 0;
    rs1 += w == 1;
    sum += (1u << w) >> 1;
  }
  if (sum == 0) return 0;
  u32 const tlog = hb32(sum) + 1;
  if (tlog > HUF_LOG_MAX) return 0;
  u32 const rest = (1u << tlog) - sum;
  if (rest & (rest - 1)) return 0;
  u32 const lastw = hb32(rest) + 1;
  L.hufw[nw] = (u8)lastw;
  rs1 += lastw == 1;
  if (rs1 < 2 || (rs1 & 1)) return 0;
  L.hlog = tlog;
  L.hnsym = nw + 1;
  return used;
}

// HUF_readDTableX1 fill, lane-parallel: weight classes in ascending weight order, symbols
// ascending inside a class, 2^(w-1) entries per symbol.
__device__ __forceinline__ void huf_build_dtable(DecLds &L) {
  u32 const lane = lane_id();
  u32 const tlog = uni(L.hlog);
  u32 w4[4];
#pragma unroll
  for (u32 k = 0; k < 4; k++) w4[k] = L.hufw[64 * k + lane];
  u32 cnt[12], rk[12], cs[12], run[12];
  u32 rank = 0, cls = 0;
#pragma unroll
  for (u32 w = 1; w <= 11; w++) {
    u32 c = 0;
#pragma unroll
    for (u32 k = 0; k < 4; k++) c += (u32)__popcll(__ballot(w4[k] == w));
    cnt[w] = c;
    rk[w] = rank;
    cs[w] = cls;
    run[w] = 0;
    rank += c << (w - 1);
    cls += c;
  }
#pragma unroll
  for (u32 k = 0; k < 4; k++) {
#pragma unroll
    for (u32 w = 1; w <= 11; w++) {
      u64 const m = __ballot(w4[k] == w);
      if (w4[k] == w) {
        u32 const r = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
        L.symlist[cs[w] + run[w] + r] = (u8)(64 * k + lane);
      }
      run[w] += (u32)__popcll(m);
    }
  }
  __syncthreads();
  for (u32 e = lane; e < (1u << tlog); e += 64) {
    // class of entry e by selects (rk/cs indexed only by unrolled constants: registers)
    u32 w = 1, rkw = rk[1], csw = cs[1];
#pragma unroll
    for (u32 v = 2; v <= 11; v++) {
      bool const in = cnt[v] && e >= rk[v];
      w = in ? v : w;
      rkw = in ? rk[v] : rkw;
      csw = in ? cs[v] : csw;
    }
    u32 const idx = (e - rkw) >> (w - 1);
    u32 const s = L.symlist[csw + idx];
    L.u.h.dt[e] = (u16)(s | (tlog + 1 - w) << 8);
  }
  __syncthreads();
}

// ---- block pieces ---------------------------------------------------------------------------
struct LitSrc {
  const u8 *g;  // literal bytes in HBM (input for raw literals, the slot for Huffman), or null
  u32 rle;      // RLE byte when g == null
  u32 n;        // regenerated size
};

struct Slot {
  u8 *lit;
  u64 *seq;
  u32 lit_cap, seq_cap;
};

// Wave copy of n bytes global -> global (raw blocks): dword stores, source realigned
// with alignbyte, 8 independent loads per lane in flight.
__device__ void wave_copy(u8 *dst, const u8 *src, u32 n) {
  u32 const lane = lane_id();
  u32 const h = min((u32)((4u - ((uintptr_t)dst & 3u)) & 3u), n);
  u32 const nw = (n - h) >> 2;
  const u8 *const s0 = src + h;
  u32 const sa = (u32)((uintptr_t)s0 & 3u);
  const u32 *const s32 = (const u32 *)(s0 - sa);
  u32 *const d32 = (u32 *)(dst + h);
  constexpr u32 U = 8;
  for (u32 w0 = 0; w0 < nw; w0 += 64 * U) {
    u32 v[U];
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      if (w < nw) {
        u32 const A = s32[w];
        u32 const B = sa ? s32[w + 1] : A;  // word w+1 holds a source byte when sa != 0
        v[u] = __builtin_amdgcn_alignbyte(B, A, sa);
      }
    }
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      if (w < nw) d32[w] = v[u];
    }
  }
  if (lane < h) dst[lane] = src[lane];
  for (u32 i = h + 4 * nw + lane; i < n; i += 64) dst[i] = src[i];
}

__device__ void wave_fill(u8 *dst, u32 v, u32 n) {
  u32 const lane = lane_id();
  u32 const h = min((u32)((4u - ((uintptr_t)dst & 3u)) & 3u), n);
  u32 const nw = (n - h) >> 2;
  u32 *const d32 = (u32 *)(dst + h);
  u32 const v4 = v * 0x01010101u;
  for (u32 w = lane; w < nw; w += 64) d32[w] = v4;
  if (lane < h) dst[lane] = (u8)v;
  for (u32 i = h + 4 * nw + lane; i < n; i += 64) dst[i] = (u8)v;
}

// Literals section (RFC 8878 §3.1.1.3.1).  Returns section bytes, 0 on error (status in st).
#if ZH_DEC_HUFPAR
// ---- segment-parallel Huffman streams --------------------------------------------------------
// One lane per stream (the libzstd decoder's shape) makes a block's literals a chain of
// n / 4 dependent table reads.  A Huffman code resynchronises within a few symbols when
// decoding starts at an arbitrary bit, so each stream is cut into S = 64 / streams segments of
// L bits, lane j of a stream decoding the symbols that start in (top - (j+1) L, top - j L]:
//   pass A: lane j decodes from its segment's first bit (a guess for j > 0), recording the first
//           HP_TRAJ positions of its trajectory, its symbol count and its exit (the first
//           position at or below its segment's end);
//   fix-up: while a lane's entry differs from its left neighbour's exit, it decodes again from
//           that exit until it lands on a recorded position of its pass-A trajectory (from there
//           on the two coincide: count = new steps + pass-A steps after that point) or leaves
//           its segment (Jacobi rounds: lane 0 is exact, lane j after at most j rounds);
//   pass B: each lane decodes its count of symbols from its exact entry and writes them at the
//           prefix sum of the counts before it.
// The symbols and the stream verdict equal the serial decode's: a stream is valid when the
// counts add up to its symbol count and the last segment ends exactly at bit 0.
#ifndef ZH_HP_TRAJ
#define ZH_HP_TRAJ 32
#endif
constexpr u32 HP_TRAJ = ZH_HP_TRAJ;
static_assert(HP_TRAJ * 64 * 2 <= 4 * (HSTAGE + 16), "trajectory records fit the stream stages");

// A lane's reader over one stream: dwords from the 4-aligned base ab (dwords holding no stream
// byte read as 0, so no load leaves the pages the stream touches), a 4-dword window w0..w3 at
// dword index wi and the two dwords below it prefetched.  Bits below the stream's bit 0 read
// as zeros (the serial reader's rule).
#ifndef ZH_HUF_PF2
#define ZH_HUF_PF2 1  // prefetch two slides ahead (4 dwords) instead of one
#endif
#ifndef ZH_HUF_PF3
#define ZH_HUF_PF3 0  // (with PF2) three slides ahead
#endif
struct HufReader {
  const u32 *ab;
  s32 da8, lastw, wi, p;
  u32 w0, w1, w2, w3, q0, q1;
#if ZH_HUF_PF2
  u32 q2, q3;  // dwords wi-2, wi-1 (q0, q1: wi-4, wi-3)
#endif
#if ZH_HUF_PF3
  u32 r0, r1;  // dwords wi-6, wi-5 (a third slide ahead)
#endif
  __device__ __forceinline__ u32 ld(s32 i) const { return (i >= 0 && i <= lastw) ? ab[i] : 0u; }
  __device__ __forceinline__ void init(const u8 *sp, u32 n) {
    ab = (const u32 *)((uintptr_t)sp & ~(uintptr_t)3);
    da8 = 8 * (s32)((uintptr_t)sp & 3u);
    lastw = (s32)(((uintptr_t)sp + n - 1 - (uintptr_t)ab) >> 2);
  }
  __device__ __forceinline__ void seek(s32 pos) {
    p = pos;
    wi = ((pos + da8 + 31) >> 5) - 4;  // bit pos lies in (96, 128] of the window
    w0 = ld(wi); w1 = ld(wi + 1); w2 = ld(wi + 2); w3 = ld(wi + 3);
#if ZH_HUF_PF2
    q2 = ld(wi - 2); q3 = ld(wi - 1);
    q0 = ld(wi - 4); q1 = ld(wi - 3);
#if ZH_HUF_PF3
    r0 = ld(wi - 6); r1 = ld(wi - 5);
#endif
#else
    q0 = ld(wi - 2); q1 = ld(wi - 1);
#endif
  }
  // decode one symbol: sym | nbBits << 8
  __device__ __forceinline__ u32 next(const u16 *dt, u32 tlog) {
    s32 v = p + da8 - 32 * wi - (s32)tlog;  // window bit of the peek's lowest bit
    if (v < 32) {  // slide down two dwords (v >= 21: a step consumes <= 11 bits)
#if ZH_HUF_PF2
      w3 = w1; w2 = w0; w1 = q3; w0 = q2;
      q3 = q1; q2 = q0;
      wi -= 2;
      v += 64;
#if ZH_HUF_PF3
      q1 = r1; q0 = r0;
      r0 = ld(wi - 6);
      r1 = ld(wi - 5);
#else
      q0 = ld(wi - 4);
      q1 = ld(wi - 3);
#endif
#else
      w3 = w1; w2 = w0; w1 = q1; w0 = q0;
      wi -= 2;
      v += 64;
      q0 = ld(wi - 2);
      q1 = ld(wi - 1);
#endif
    }
    u32 const k = (u32)v >> 5;  // 1..3
    // (mask selects: the compiler turns a select chain on k into a scratch-indexed array)
    u32 const m2 = 0u - ((k >> 1) & 1u), m1 = 0u - (k & 1u);
    u32 const lo = (w1 & ~m2) | (((w2 & ~m1) | (w3 & m1)) & m2), hi = (w2 & ~m2) | (w3 & ~m1 & m2);
    u32 x = __builtin_amdgcn_alignbit(hi, lo, (u32)v & 31u) & ((1u << tlog) - 1u);
    if (p < (s32)tlog) x &= (p <= 0) ? 0u : ~0u << (tlog - (u32)p);  // bits below the stream
    u32 const e = dt[x];
    p -= (s32)max(e >> 8, 1u);  // (>= 1 in any table huf_build_dtable makes; a loop bound)
    return e;
  }
};

// Decodes the ns (1 or 4) streams into o + off[k]; false = corrupt.  Every lane calls it.
// (msp, mn, mc, mo: this lane's stream -- bytes, size, symbols, output offset)
__device__ __forceinline__ bool huf_streams_par(DecLds &L, u32 ns, const u8 *msp, u32 mn, u32 mc, u32 mo, u8 *o, u32 tlog) {
  u32 const lane = lane_id();
  u32 const S = 64u / ns, k = lane / S, j = lane % S;
  u32 const last = mn ? msp[mn - 1] : 0u;
  bool bad = last == 0;
  s32 const top = bad ? 0 : 8 * (s32)(mn - 1) + (s32)hb32(last);
  s32 const Lb = max((top + (s32)S - 1) / (s32)S, 1);
  // trajectory positions are kept as u16 offsets into a segment: a stream with 2^16 bits or more
  // per segment (> 1 M bits for 4 streams) holds more bits than its <= 32 K symbols of <= 11 bits
  // can consume, so it is corrupt
  bad |= Lb >= 65536;
  s32 const hiB = top - (s32)j * Lb, lo = max(top - (s32)(j + 1) * Lb, 0);
  const u16 *const dt = L.u.h.dt;
  u16 *const traj = (u16 *)&L.u.h.hs[0][0];  // [HP_TRAJ][64]
  HufReader r;
  r.init(msp, mn);
  // pass A
  s32 const gA = max(hiB, 0);
  u32 cA = 0;
  r.seek(gA);
  if (!bad) {
    while (r.p > lo) {
      if (cA < HP_TRAJ) traj[cA * 64 + lane] = (u16)(gA - r.p);
      r.next(dt, tlog);
      cA++;
    }
  }
  s32 const xA = r.p;
  // fix-up rounds
  auto shr = [&](s32 v) -> s32 {  // the value of lane j - 1 of this stream (lane j = 0: top)
    s32 const u = ns == 1 ? (s32)wave_shr1((u32)v) : (s32)ZH_DPP((u32)v, 0x111, 0xf);
    return j == 0 ? top : u;
  };
  s32 entry = gA, x = xA;
  u32 c = cA;
  for (;;) {
    s32 const px = shr(x);
    bool const need = !bad && entry != px;
    if (!__ballot(need)) break;
    if (need) {
      r.seek(px);
      u32 n = 0, t = 0;
      u32 const tmax = min(cA, HP_TRAJ);
      s32 nx = 0;
      u32 nc = 0;
      for (;;) {
        s32 const pn = r.p;
        while (t < tmax && gA - (s32)traj[t * 64 + lane] > pn) t++;
        if (t < tmax && gA - (s32)traj[t * 64 + lane] == pn) { nc = n + (cA - t); nx = xA; break; }
        if (pn <= lo) { nc = n; nx = pn; break; }
        r.next(dt, tlog);
        n++;
      }
      entry = px;
      c = nc;
      x = nx;
    }
  }
  // counts -> output offsets; the stream's verdict
  u32 incl = c;
  if (ns == 1) {
    incl = wave_scan_incl(c);
  } else {
    incl += ZH_DPP(incl, 0x111, 0xf);
    incl += ZH_DPP(incl, 0x112, 0xf);
    incl += ZH_DPP(incl, 0x114, 0xf);
    incl += ZH_DPP(incl, 0x118, 0xf);
  }
  int const src = (int)((k * S + S - 1) << 2);  // the stream's last lane (a per-lane index)
  u32 const total = (u32)__builtin_amdgcn_ds_bpermute(src, (int)incl);
  s32 const fin = __builtin_amdgcn_ds_bpermute(src, x);
  bad |= total != mc || fin != 0;
  if (__ballot(bad)) return false;
  // pass B: c symbols from entry to o + mo + (incl - c); bytes until the dword boundary, packed
  // dwords inside, bytes for the tail
  u32 const o0 = mo + incl - c, o1 = mo + incl;
  u32 const a0 = (o0 + 3u) & ~3u, a1 = o1 & ~3u;
  r.seek(entry);
  u32 acc = 0;
  for (u32 i = o0; i < o1; i++) {
    u32 const sym = r.next(dt, tlog) & 0xFFu;
    if (i < a0 || i >= a1) {
      o[i] = (u8)sym;
    } else {
      acc |= sym << (8 * (i & 3u));
      if ((i & 3u) == 3u) {
        *(u32 *)(o + i - 3) = acc;
        acc = 0;
      }
    }
  }
  return true;
}
#endif

// The literals section's size without decoding it (the split pipeline's tables pass); 0 when
// its header is corrupt -- the literals pass then finds and reports the same error.
__device__ u32 skip_literals(const u8 *bp, u32 bsz) {
  if (bsz < 1) return 0;
  u32 const h0 = ub(bp);
  u32 const lt = h0 & 3u, sf = (h0 >> 2) & 3u;
  if (lt <= 1) {
    u32 hs, n;
    if (sf == 1) {
      if (bsz < 2) return 0;
      hs = 2;
      n = rd16(bp) >> 4;
    } else if (sf == 3) {
      if (bsz < 3) return 0;
      hs = 3;
      n = rd24(bp) >> 4;
    } else {
      hs = 1;
      n = h0 >> 3;
    }
    if (n > BLOCKSIZE_MAX) return 0;
    u32 const t = hs + (lt == 0 ? n : 1u);
    return t <= bsz ? t : 0u;
  }
  u32 const hs = sf <= 1 ? 3u : sf == 2 ? 4u : 5u;
  if (bsz < hs) return 0;
  u64 const hv = sf <= 1 ? (u64)rd24(bp) : sf == 2 ? (u64)rd32(bp) : ((u64)rd32(bp) | (u64)ub(bp + 4) << 32);
  u32 const n = sf <= 1 ? (u32)(hv >> 4) & 0x3FFu : sf == 2 ? (u32)(hv >> 4) & 0x3FFFu : (u32)(hv >> 4) & 0x3FFFFu;
  u32 const cs = sf <= 1 ? (u32)(hv >> 14) & 0x3FFu : sf == 2 ? (u32)(hv >> 18) & 0x3FFFu : (u32)(hv >> 22) & 0x3FFFFu;
  if (n > BLOCKSIZE_MAX || hs + cs > bsz) return 0;
  return hs + cs;
}

__device__ u32 decode_literals(DecLds &L, const u8 *bp, u32 bsz, const Slot &sl, LitSrc &lits, u32 &st) {
  u32 const lane = lane_id();
  if (bsz < 1) { st = ST_CORRUPT; return 0; }
  u32 const h0 = ub(bp);
  u32 const lt = h0 & 3u, sf = (h0 >> 2) & 3u;
  if (lt <= 1) {  // raw / RLE
    u32 hs, n;
    if (sf == 1) {
      if (bsz < 2) { st = ST_CORRUPT; return 0; }
      hs = 2;
      n = rd16(bp) >> 4;
    } else if (sf == 3) {
      if (bsz < 3) { st = ST_CORRUPT; return 0; }
      hs = 3;
      n = rd24(bp) >> 4;
    } else {
      hs = 1;
      n = h0 >> 3;
    }
    if (n > BLOCKSIZE_MAX) { st = ST_CORRUPT; return 0; }
    lits.n = n;
    if (lt == 0) {
      if (hs + n > bsz) { st = ST_CORRUPT; return 0; }
      lits.g = bp + hs;
      lits.rle = 0;
      return hs + n;
    }
    if (hs + 1 > bsz) { st = ST_CORRUPT; return 0; }
    lits.g = nullptr;
    lits.rle = ub(bp + hs);
    return hs + 1;
  }
  // Huffman-coded (2) or treeless (3)
  u32 const hs = sf <= 1 ? 3u : sf == 2 ? 4u : 5u;
  if (bsz < hs) { st = ST_CORRUPT; return 0; }
  u64 const hv = sf <= 1 ? (u64)rd24(bp) : sf == 2 ? (u64)rd32(bp) : ((u64)rd32(bp) | (u64)ub(bp + 4) << 32);
  u32 n, cs;
  if (sf <= 1) {
    n = (u32)(hv >> 4) & 0x3FFu;
    cs = (u32)(hv >> 14) & 0x3FFu;
  } else if (sf == 2) {
    n = (u32)(hv >> 4) & 0x3FFFu;
    cs = (u32)(hv >> 18) & 0x3FFFu;
  } else {
    n = (u32)(hv >> 4) & 0x3FFFFu;
    cs = (u32)(hv >> 22) & 0x3FFFFu;
  }
  u32 const ns = sf == 0 ? 1u : 4u;
  if (n > BLOCKSIZE_MAX || hs + cs > bsz) { st = ST_CORRUPT; return 0; }
  if (n > sl.lit_cap) { st = ST_SMALL; return 0; }
  const u8 *p = bp + hs;
  u32 rem = cs;
#ifdef ZH_STAMPS
  if (lane == 0) L.lst_t[0] = __builtin_amdgcn_s_memtime();
#endif
  if (lt == 2) {
    // the tree description (<= 128 bytes) staged in LDS first: lane 0's weight decode is a
    // serial FSE chain whose every byte read was a dependent global load
#ifndef ZH_DEC_WSTAGE
#define ZH_DEC_WSTAGE 0  // (1: 117.7 GB/s vs 119.1 without; profiles/r06u_dec_p5_reader_ab.json)
#endif
    const u8 *wp = p;
    if (ZH_DEC_WSTAGE) {
      u32 const wn = min(rem, 128u);
      u8 *const ws = L.u.h.hs[0];
      for (u32 k = lane; k < wn; k += 64) ws[k] = p[k];
      __syncthreads();
      wp = ws;
    }
    if (lane == 0) {
      u32 const used = huf_read_weights(L, wp, ZH_DEC_WSTAGE ? min(rem, 128u) : rem);
      L.err = used ? 0u : 1u;
      L.hvalid = used ? 1u : 0u;
      L.used = used;
    }
    __syncthreads();
    if (uni(L.err)) { st = ST_CORRUPT; return 0; }
    u32 const used = uni(L.used);
    p += used;
    rem -= used;
  } else if (!uni(L.hvalid)) {
    st = ST_CORRUPT;
    return 0;
  }
#ifdef ZH_STAMPS
  if (lane == 0) L.lst_t[1] = __builtin_amdgcn_s_memtime();
#endif
  huf_build_dtable(L);
#ifdef ZH_STAMPS
  if (lane == 0) L.lst_t[2] = __builtin_amdgcn_s_memtime();
#endif
  u32 const tlog = uni(L.hlog);
  // streams
  const u8 *sp[4];
  u32 ssz[4], cnt[4], off[4];
  if (ns == 1) {
    sp[0] = p;
    ssz[0] = rem;
    cnt[0] = n;
    off[0] = 0;
    for (u32 k = 1; k < 4; k++) { sp[k] = p; ssz[k] = 0; cnt[k] = 0; off[k] = 0; }
  } else {
    if (rem < 10) { st = ST_CORRUPT; return 0; }
    u32 const s1 = rd16(p), s2 = rd16(p + 2), s3 = rd16(p + 4);
    u32 const t = 6 + s1 + s2 + s3;
    if (t >= rem) { st = ST_CORRUPT; return 0; }
    u32 const seg = (n + 3) / 4;
    if (3 * seg > n) { st = ST_CORRUPT; return 0; }
    sp[0] = p + 6;
    ssz[0] = s1;
    sp[1] = sp[0] + s1;
    ssz[1] = s2;
    sp[2] = sp[1] + s2;
    ssz[2] = s3;
    sp[3] = sp[2] + s3;
    ssz[3] = rem - t;
    for (u32 k = 0; k < 4; k++) {
      cnt[k] = k < 3 ? seg : n - 3 * seg;
      off[k] = k * seg;
    }
  }
#if ZH_DEC_HUFPAR
  {
    u32 const k = lane / (64u / ns);
    const u8 *msp = sp[0];
    u32 mn = ssz[0], mc = cnt[0], mo = off[0];
    for (u32 t = 1; t < 4; t++)
      if (k == t) { msp = sp[t]; mn = ssz[t]; mc = cnt[t]; mo = off[t]; }
    if (!huf_streams_par(L, ns, msp, mn, mc, mo, sl.lit, tlog)) { st = ST_CORRUPT; return 0; }
  }
#else
  // lanes 0..ns-1 decode one stream each, reading it from an LDS stage; a lane whose
  // stage runs out stops, and the wave restages every such stream in one burst per round
  const u8 *mp = sp[0];
  u32 msz = ssz[0], mc = cnt[0], mo = off[0];
  for (u32 k = 1; k < 4; k++)
    if (lane == k) { mp = sp[k]; msz = ssz[k]; mc = cnt[k]; mo = off[k]; }
  bool const act = lane < ns;
  BitRevS r;
  bool bad = !r.start(mp, act ? msz : 0u) && act;
  u32 const mcnt = act && !bad ? mc : 0u;
  u8 *const o = sl.lit + mo;
  u8 *const stg = L.u.h.hs[lane & 3u];
  u32 i = 0;
  for (;;) {
    bool need = false;
    while (i < mcnt) {
      // one container check per 4 symbols: a refill leaves >= 57 bits and 4 x 11 fit
      if (!r.ensure(stg, 4 * tlog)) { need = true; break; }
      u32 const k4 = min(4u, mcnt - i);
      for (u32 u = 0; u < k4; u++) {
        u32 const e = L.u.h.dt[(u32)r.bits(tlog)];
        o[i + u] = (u8)e;
        r.pos -= (s32)(e >> 8);
      }
      i += k4;
    }
    u64 const nm = __ballot(need);
    if (!nm) break;
    u32 lo, hi;
    r.stage_range(HSTAGE, lo, hi);
    for (u32 k = 0; k < 4; k++) {
      if (!((nm >> k) & 1u)) continue;
      u32 const lk = __builtin_amdgcn_readlane(lo, k), hk = __builtin_amdgcn_readlane(hi, k);
      stage_copy(L.u.h.hs[k], sp[k], lk, hk);
      if (lane == k) r.slo = (s32)lk;
    }
    __syncthreads();
  }
  bad |= act && r.pos != 0;
  if (__ballot(bad)) { st = ST_CORRUPT; return 0; }
#endif
  lits.g = sl.lit;
  lits.rle = 0;
  lits.n = n;
  return hs + cs;
}

// One sequence table (mode 0 predefined, 1 RLE, 2 FSE, 3 repeat) on lane 0.
// Returns bytes consumed (>= 0) or -1 on error.
// FSE_buildDTable with the whole wave (same table as build_dtable): lanes = symbols for the
// counts, then lanes = cells.  The spread visits position k * step mod size at step k, so the
// cell placed at position u <= high is number k(u) = u * step^-1 mod size less the high
// (low-probability) positions reached before it; its symbol is the one whose range of cells
// holds that number.  A cell's state counter (symbolNext) is its symbol's count plus the cells
// of that symbol at lower positions: counted chunk by chunk with one ballot per distinct
// symbol, the running counts held by the symbols' lanes.  All lanes call it; false = invalid.
__device__ bool build_dtable_wave(u32 *T, const s16 *norm, u32 maxSV, u32 tlog) {
  u32 const lane = lane_id(), size = 1u << tlog, mask = size - 1u;
  u64 const below = (1ull << lane) - 1ull;
  s32 const c = lane <= maxSV ? (s32)norm[lane] : 0;
  u64 const lowm = __ballot(c == -1);
  u32 const nlow = (u32)__popcll(lowm), high = size - 1u - nlow;
  u32 const cp = c > 0 ? (u32)c : 0u;
  u32 const incl = wave_scan_incl(cp);
  if (lane_value(incl, 63) != high + 1u || nlow > size) return false;
  if (c == -1) T[size - 1u - (u32)__popcll(lowm & below)] = lane;  // low-probability symbols at the top
  u32 const step = (size >> 1) + (size >> 3) + 3u;
  u32 inv = step;  // step^-1 mod 2^32 (Newton: each round doubles the correct low bits)
#pragma unroll
  for (u32 r = 0; r < 5; r++) inv *= 2u - step * inv;
  u32 const kh = lane < nlow ? ((high + 1u + lane) * inv) & mask : 0xFFFFFFFFu;  // steps of the high positions
  for (u32 u = lane; u <= high; u += 64) {
    u32 const k = (u * inv) & mask;
    u32 skip = 0;
    for (u32 l = 0; l < nlow; l++) skip += lane_value(kh, l) < k ? 1u : 0u;
    u32 const r = k - skip;
    // the symbol s with incl[s - 1] <= r < incl[s]: count the symbols whose range ends at or below r
    u32 s = 0;
    for (u32 t = 0; t <= maxSV; t++) s += lane_value(incl, t) <= r ? 1u : 0u;
    T[u] = s;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // (lgkmcnt(0): the wave's LDS stores are done before the reads below)
  __builtin_amdgcn_wave_barrier();
  u32 cnt = c == -1 ? 1u : cp;  // symbolNext of symbol `lane`
  for (u32 c0 = 0; c0 < size; c0 += 64) {
    u32 const u = c0 + lane;
    bool const valid = u < size;
    u32 const s = valid ? T[u] & 0xFFu : 0xFFu;
    u64 pending = __ballot(valid);
    u32 ns = 0;
    while (pending) {
      u32 const s0 = (u32)__builtin_amdgcn_readlane((int)s, (int)__builtin_ctzll(pending));
      u64 const m = __ballot(valid && s == s0);
      u32 const base = lane_value(cnt, s0);
      if (s == s0) ns = base + (u32)__popcll(m & below);
      if (lane == s0) cnt += (u32)__popcll(m);
      pending &= ~m;
    }
    if (valid) {
      u32 const nb = tlog - hb32(ns);
      T[u] = s | nb << 8 | ((ns << nb) - size) << 16;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  return true;
}

// defer: leave the table build to build_dtable_wave (the normalised counts go to norm + 64 t,
// bld[t] is set); else build it here, serially.
template <class LDS>
__device__ __noinline__ s32 seq_table(LDS &L, u32 t, u32 mode, const u8 *p, u32 avail, bool defer = false) {
  u32 *T = L.fse + tab_off(t);
  u32 const maxSV = tab_maxsv(t);
  s16 *const nrm = defer ? L.norm + 64 * t : L.norm;
  if (mode == 0) {
    if (L.tkind[t] == TAB_PREDEF) return 0;
    u32 const nsym = t == TAB_LL ? 36u : t == TAB_ML ? 53u : 29u;
    const s16 *src = t == TAB_LL ? c_LL_norm : t == TAB_ML ? c_ML_norm : c_OF_norm;
    for (u32 s = 0; s <= maxSV; s++) nrm[s] = s < nsym ? src[s] : (s16)0;
    u32 const lg = t == TAB_OF ? 5u : 6u;
    if (defer) L.bld[t] = 1;
    else if (!build_dtable(T, nrm, maxSV, lg, L.next)) return -1;
    L.tlog[t] = lg;
    L.tkind[t] = TAB_PREDEF;
    return 0;
  }
  if (mode == 1) {
    if (avail < 1) return -1;
    u32 const s = p[0];
    if (s > maxSV) return -1;
    T[0] = s;  // nbBits 0, newState 0
    L.tlog[t] = 0;
    L.tkind[t] = 0x100u | s;
    return 1;
  }
  if (mode == 2) {
    u32 lg;
    u32 const used = read_ncount(p, avail, nrm, maxSV, tab_maxlog(t), lg);
    if (!used) return -1;
    if (defer) L.bld[t] = 1;
    else if (!build_dtable(T, nrm, maxSV, lg, L.next)) return -1;
    L.tlog[t] = lg;
    L.tkind[t] = 0;
    return (s32)used;
  }
  return L.tkind[t] == TAB_NONE ? -1 : 0;  // repeat
}

// Formatted dictionary (RFC 8878 §5): its Huffman table and OF / ML / LL FSE tables become
// the frame's previous tables (treeless literals and repeat modes use them).  Lane 0; false
// when they do not parse.  d = the dictionary, off = its content offset.
template <class LDS>
__device__ __forceinline__ bool load_dict_entropy(LDS &L, const u8 *d, u32 off) {
  if (off < 8 + 12) return false;
  const u8 *const p = d + 8;
  u32 const avail = off - 8 - 12;
  u32 o = huf_read_weights(L, p, avail);
  if (!o) return false;
  L.hvalid = 1;
  u32 const order[3] = {TAB_OF, TAB_ML, TAB_LL};
  for (u32 k = 0; k < 3; k++) {
    s32 const u = seq_table(L, order[k], 2, p + o, avail - o);
    if (u < 0) return false;
    o += (u32)u;
  }
  return true;
}

__device__ __forceinline__ u32 to_nvcomp(u32 s) {
  switch (s) {
    case ST_OK: return 0;
    case ST_INVALID: return 2;
    case ST_CORRUPT: return 6;
    case ST_SMALL: return 7;
    case ST_CHECKSUM: return 10;
    default: return 1;
  }
}

}  // namespace

// ---- execution of one block through the LDS window (see the header comment).
  // ---- execution, DEC_STAGE output bytes per window.  Lanes = the next 64 sequences
  // (prefix sums give their window positions).  Pass A, lanes = output bytes: literal
  // bytes, and match bytes whose source lies before the window (already in HBM), are
  // gathered with all loads of a round in flight.  Pass B, in sequence order, lanes =
  // bytes of one match: the match bytes whose source lies inside the window, from LDS
  // (a wave's LDS operations execute in order).  Then one coalesced flush.
// Returns false when an offset reaches before the frame start and the dictionary content
// (dlen bytes ending at dend) that precedes it.
template <class LDS>
__device__ bool execute_block(LDS &L, const Slot &sl, u8 *ob, s64 fpos, const LitSrc &lits, u32 nseq, u32 tl, const u8 *dend, s64 dlen,
                              u64 *xs = nullptr) {
  u32 const lane = lane_id();
  u32 q = 0, qd = 0, opos = 0, lcur = 0;
  bool bad = false;
#ifdef ZH_STAMPS
  // (-DZH_STAMPS, phase 3: xs[1] windows, xs[2] records + scan, [3] pass A, [4] pass B, [5] flush)
  u64 xp = __builtin_amdgcn_s_memtime();
#define XSTAMP(k)                                   \
  do {                                              \
    if (xs) {                                       \
      u64 const _t = __builtin_amdgcn_s_memtime();  \
      xs[k] += _t - xp;                             \
      xp = _t;                                      \
    }                                               \
  } while (0)
#else
#define XSTAMP(k) do { } while (0)
#endif
  while (q <= nseq) {
#ifdef ZH_STAMPS
    if (xs) xs[1]++;
#endif
    u32 const gs = opos;
    u32 const idx = q + lane;
    bool const valid = idx <= nseq;
    u32 ll = 0, ml = 0, off = 1;
    if (idx < nseq) {
      u64 const v = sl.seq[idx];
      ll = (u32)v & 0x1FFFFu;
      ml = ((u32)(v >> 17) & 0x1FFFFu) + 3u;
      off = (u32)(v >> 34);
    } else if (idx == nseq) {
      ll = tl;
    }
    u32 const span = ll + ml;
    u32 const incl = wave_scan_incl(span), linc = wave_scan_incl(ll);  // DPP (zh_common.h)
    s32 const vs = (s32)(incl - span) - (s32)qd;  // window-relative start (q: qd bytes done)
    s32 const ve = (s32)incl - (s32)qd;
    u32 const lit0 = lcur + linc - ll;
    u32 const tot = __builtin_amdgcn_readlane(incl, 63) - qd;
    u32 const wlen = min((u32)sizeof(L.u.out) - 16u, tot);
    s32 const ms = vs + (s32)ll;  // window-relative match start
    // an offset reaching before the frame start is corrupt (checked before any read)
    bool const obad = valid && ml && vs < (s32)wlen && fpos + (s64)gs + ms - (s64)off < -dlen;
    if (__ballot(obad)) { bad = true; break; }
    L.wvs[lane] = valid && vs < (s32)wlen ? vs : 0x7FFFFFFF;
    L.wll[lane] = ll;
    L.wlit[lane] = lit0;
    L.woff[lane] = off;
    // the window's literal bytes, lits [lfirst, lfirst + wlen), staged with 16-byte loads
    u32 lbase = 0, lfirst = 0;
    if constexpr (LDS::kLitStage) {
      if (lits.g) {
        lfirst = lcur + min(qd, (u32)__builtin_amdgcn_readlane(ll, 0));
        u32 const nlw = lits.n > lfirst ? min(wlen, lits.n - lfirst) : 0u;
        if (nlw) {
          uintptr_t const s0 = (uintptr_t)lits.g + lfirst, a0 = s0 & ~(uintptr_t)15;
          uintptr_t const alast = ((uintptr_t)lits.g + lits.n - 1) & ~(uintptr_t)15;  // (no chunk past the literals)
          u32 const nch = (u32)((s0 + nlw - 1 - a0) >> 4) + 1u;
          for (u32 c = lane; c < nch; c += 64) {
            uintptr_t const a = min(a0 + 16u * c, alast);
            *(uint4 *)(L.lst + 16 * c) = *(const uint4 *)a;
          }
          lbase = (u32)(s0 - a0);
        }
      }
    }
    if constexpr (LDS::kStartMap) {
      // the sequence of window byte x is the number of sequence starts at or below x, less one:
      // a start bitmap (lane 0's sequence starts at 0 or before) and its per-word prefix counts
      // (barriers between the lanes' LDS accesses: a one-wave workgroup, so an s_barrier
      // costs little, and without them the compiler may move a lane's read above the others' ORs)
      L.bm[2 * lane] = 0;
      __syncthreads();
      if (valid && vs < (s32)wlen) {
        u32 const p = vs > 0 ? (u32)vs : 0u;
        atomicOr(&L.bm[2 * (p >> 5)], 1u << (p & 31u));
      }
      __syncthreads();
      u32 const c = (u32)__popc(L.bm[2 * lane]);
      L.bm[2 * lane + 1] = wave_scan_incl(c) - c;
    }
    __syncthreads();
    XSTAMP(2);
    // pass A
#ifndef ZH_EXEC_UA
#define ZH_EXEC_UA 4  // bytes per lane per pass-A round (8: 92.8, 16: 89.2, 4: 93.6 GB/s)
#endif
    constexpr u32 UA = ZH_EXEC_UA;
    for (u32 x0 = 0; x0 < wlen; x0 += 64 * UA) {
      const u8 *ad[UA];
      bool w[UA];
      u32 li[UA];  // (staged literals: the byte's stage index, else ~0)
#pragma unroll
      for (u32 t = 0; t < UA; t++) {
        u32 const x = x0 + 64 * t + lane;
        if constexpr (LDS::kStartMap && ZH_EXEC_CHASE) {
          // every byte here: an in-window source is followed back (sequence by sequence, each
          // step to an earlier one or into a literal run) to a literal or a byte already in HBM
          u32 y = x < wlen ? x : 0u;
          bool lit = false;
          s32 swf = 0;
          u32 litidx = 0;
          for (;;) {
            u64 const e = ((const u64 *)L.bm)[y >> 5];
            u32 const m32 = (u32)e & (0xFFFFFFFFu >> (31u - (y & 31u)));
            u32 const j = min((u32)(e >> 32) + (u32)__popc(m32) - 1u, 63u);
            u32 const d = (u32)((s32)y - L.wvs[j]);
            u32 const llj = L.wll[j];
            if (d < llj) {
              lit = true;
              litidx = L.wlit[j] + d;
              break;
            }
            u32 const m = d - llj, offj = L.woff[j];
            s32 const sw = L.wvs[j] + (s32)llj - (s32)offj + (s32)(m < offj ? m : umod(m, offj));
            if (sw < 0) {
              swf = sw;
              break;
            }
            y = (u32)sw;
          }
          li[t] = ~0u;
          w[t] = x < wlen;
          if (lit) {
            ad[t] = lits.g ? lits.g + litidx : nullptr;
          } else {
            s64 const fa = fpos + (s64)gs + swf;  // frame position of the source (< 0: dictionary)
            ad[t] = fa >= 0 ? ob + (s64)gs + swf : dend + fa;
          }
          continue;
        }
        u32 j = 0;
        if constexpr (LDS::kStartMap) {
          u64 const e = ((const u64 *)L.bm)[min(x >> 5, 63u)];
          u32 const m = (u32)e & (0xFFFFFFFFu >> (31u - (x & 31u)));
          j = min((u32)(e >> 32) + (u32)__popc(m) - 1u, 63u);  // (bytes past wlen: any j, unused)
        } else {
#pragma unroll
          for (u32 stp = 32; stp; stp >>= 1) j += L.wvs[j + stp] <= (s32)x ? stp : 0u;
        }
        u32 const d = (u32)((s32)x - L.wvs[j]);
        u32 const llj = L.wll[j];
        li[t] = ~0u;
        if (d < llj) {
          if (LDS::kLitStage && lits.g) {
            li[t] = lbase + L.wlit[j] + d - lfirst;
            ad[t] = nullptr;
          } else {
            ad[t] = lits.g ? lits.g + L.wlit[j] + d : nullptr;
          }
          w[t] = x < wlen;
        } else {
          u32 const m = d - llj, offj = L.woff[j];
          s64 const sw = (s64)L.wvs[j] + llj - offj + (m < offj ? m : umod(m, offj));
          s64 const fa = fpos + (s64)gs + sw;  // frame position of the source (< 0: dictionary)
          ad[t] = fa >= 0 ? ob + (s64)gs + sw : dend + fa;
          w[t] = x < wlen && sw < 0;
        }
      }
      u8 v[UA];
#pragma unroll
      for (u32 t = 0; t < UA; t++) {
        if constexpr (LDS::kLitStage) {
          v[t] = !w[t] ? (u8)0 : li[t] != ~0u ? L.lst[min(li[t], (u32)sizeof(L.lst) - 1u)] : ad[t] ? *ad[t] : (u8)lits.rle;
        } else {
          v[t] = w[t] ? (ad[t] ? *ad[t] : (u8)lits.rle) : (u8)0;
        }
      }
#pragma unroll
      for (u32 t = 0; t < UA; t++)
        if (w[t]) L.u.out[x0 + 64 * t + lane] = v[t];
    }
    XSTAMP(3);
    // pass B: matches with a source inside the window, in order
    s32 const mlo = ms < 0 ? -ms : 0;
    s32 const mhi = min((s32)ml, (s32)wlen - ms);
    bool const nearp = !(LDS::kStartMap && ZH_EXEC_CHASE) && valid && mhi > mlo && ms - (s32)off + (s32)min(off, (u32)mhi) - 1 >= 0;
    u64 nm = __ballot(nearp);
    while (nm) {
      u32 const j = (u32)__builtin_ctzll(nm);
      nm &= nm - 1;
      s32 const msj = __builtin_amdgcn_readlane(ms, j), loj = __builtin_amdgcn_readlane(mlo, j), hij = __builtin_amdgcn_readlane(mhi, j);
      u32 const offj = __builtin_amdgcn_readlane(off, j);
      for (s32 m = loj + (s32)lane; m < hij; m += 64) {
        s32 const sw = msj - (s32)offj + (s32)((u32)m < offj ? (u32)m : umod((u32)m, offj));
        if (sw >= 0) L.u.out[msj + m] = L.u.out[sw];
      }
    }
    XSTAMP(4);
    // flush the window: head bytes to a 4-B aligned destination, then dwords
    {
      u8 *const d = ob + gs;
      u32 const h = min((u32)((4u - ((uintptr_t)d & 3u)) & 3u), wlen);
      u32 const nw = (wlen - h) >> 2;
      u32 *const d32 = (u32 *)(d + h);
      for (u32 k = lane; k < nw; k += 64) {
        u32 const o = h + 4 * k;
        const u32 *wp = (const u32 *)(L.u.out + (o & ~3u));
        d32[k] = __builtin_amdgcn_alignbyte(wp[1], wp[0], o & 3u);
      }
      if (lane < h) d[lane] = L.u.out[lane];
      for (u32 k = h + 4 * nw + lane; k < wlen; k += 64) d[k] = L.u.out[k];
    }
    __threadfence_block();  // later windows read this one back from HBM
    __syncthreads();
    XSTAMP(5);
    // advance: sequences that ended inside the window are done
    u32 const k = (u32)__popcll(__ballot(valid && ve <= (s32)wlen));
    if (k < 64) {
      lcur = __builtin_amdgcn_readlane(lit0, k);
      qd = (u32)((s32)wlen - __builtin_amdgcn_readlane(vs, k));
    } else {
      lcur = __builtin_amdgcn_readlane(lit0, 63) + __builtin_amdgcn_readlane(ll, 63);
      qd = 0;
    }
    q += k;
    opos = gs + wlen;
  }
  return !bad;
}

// ---- split pipeline.  A buffer holding one frame of one compressed block (every chunk
// of a batch) is decoded by three kernels: phase 1 (this kernel) does the headers, the
// literals and the sequence tables and leaves a hand-off record; zh_dec_seq_kernel runs
// the sequence bitstreams of 64 such buffers at once, one lane each (the serial FSE chains
// of 64 blocks interleave in one wave instead of one chain per wave); zh_dec_exec_kernel
// (phase 3) executes the block and finishes the frame.  Anything else is decoded in phase 1.
struct DecHandoff {
  u32 tabs[1280];  // DecLds::fse of the block
  u64 sp;          // sequence bitstream
  u32 rem, nseq, lg, flag;  // bytes, sequences, logLL | logOF << 8 | logML << 16, 1 = deferred
  u64 litg;        // literal bytes (null: RLE)
  u32 litrle, litn;
  u64 fcs, ipc;    // frame content size (~0: absent), checksum position (~0: none)
  u64 sumLL, sumML;
  u32 sbad;
  u32 rep[3];      // repcodes at the block start
};
static_assert(sizeof(DecHandoff) <= ZH_DEC_HANDOFF_BYTES, "hand-off record");

__device__ __forceinline__ DecHandoff *handoff(const ZhDecArgs &a, u32 item) {
  return (DecHandoff *)(a.ws + (size_t)item * a.slot_bytes + a.ho_off);
}

// Offset_Value -> offset with the repeat-offset history (RFC 8878 §3.1.1.5; libzstd
// ZSTD_decodeSequence: a zero offset is forced to 1)
__device__ __forceinline__ u32 resolve_off(u32 ofv, u32 ll, u32 &rep0, u32 &rep1, u32 &rep2) {
  u32 off;
  if (ofv > 3) {
    off = ofv - 3;
    rep2 = rep1;
    rep1 = rep0;
    rep0 = off;
  } else {
    u32 const idx = ofv - 1 + (ll == 0 ? 1u : 0u);
    if (idx == 0) {
      off = rep0;
    } else {
      off = idx == 3 ? rep0 - 1 : idx == 1 ? rep1 : rep2;
      off += off == 0 ? 1u : 0u;
      if (idx != 1) rep2 = rep1;
      rep1 = rep0;
      rep0 = off;
    }
  }
  return off;
}

// Diagnostic build only (-DZH_STAMPS): per-phase s_memtime cycles of each item, written
// to the first 64 bytes of its workspace slot when it finishes (tools/dec_stamps.py).
#ifdef ZH_STAMPS
#define DSTAMP(k)                              \
  do {                                         \
    u64 _t = __builtin_amdgcn_s_memtime();     \
    stv[k] += _t - stp;                        \
    stp = _t;                                  \
  } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif

// One workgroup (one wave) per input buffer.
template <class LDS>
__device__ __forceinline__ void decode_body(LDS &L, ZhDecArgs a) {
  u32 const item = a.item0 + blockIdx.x, lane = lane_id();
  const u8 *const src = (const u8 *)(a.in_ptrs ? a.in_ptrs[item] : a.one_in);
  u64 const srcn = a.in_ptrs ? (u64)a.in_sizes[item] : a.one_in_size;
  u8 *const dst = (u8 *)(a.in_ptrs ? a.out_ptrs[item] : a.one_out);
  u64 const cap = a.out_caps ? (u64)a.out_caps[item] : a.out_cap_all;
  Slot sl;
  sl.lit = a.ws + (size_t)item * a.slot_bytes;
  sl.lit_cap = a.block_cap;
  sl.seq = (u64 *)(sl.lit + a.lit_bytes);
  sl.seq_cap = a.seq_cap;
  // dictionary content precedes every frame: match sources before the frame start
  const u8 *const dend = a.dict ? a.dict + a.dict_n : nullptr;
  s64 const dlen = a.dict ? (s64)(a.dict_n - a.dict_off) : 0;
  if constexpr (!LDS::kTablesOnly) {
    if (lane < 4) L.wvs[64 + lane] = 0x7FFFFFFF;
  }
  if (lane < 36) L.info[0][lane] = c_LL_info[lane];
  if (lane < 53) L.info[1][lane] = c_ML_info[lane];
  __syncthreads();

  // split pipeline (launch_decompress): phase 4 = the sequence tables of deferrable buffers
  // only (no literals, no status), phase 5 = everything else (the literals of the deferred
  // buffers, whole decodes of the others)
  if ((a.phase == 1 || a.phase == 4) && lane == 0) handoff(a, item)->flag = 0;

  u32 st = ST_OK;
  u64 produced = 0, ip = 0;
  if (!src || (!dst && cap)) st = ST_INVALID;
#ifdef ZH_STAMPS
  u64 stv[8] = {}, stp = __builtin_amdgcn_s_memtime();
#endif
  while (st == ST_OK && ip < srcn) {
    // ---- frame header (RFC 8878 §3.1.1.1)
    if (srcn - ip < 4) { st = ST_CORRUPT; break; }
    u32 const magic = rd32(src + ip);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (srcn - ip < 8) { st = ST_CORRUPT; break; }
      u64 const sk = 8ull + rd32(src + ip + 4);
      if (sk > srcn - ip) { st = ST_CORRUPT; break; }
      ip += sk;
      continue;
    }
    if (magic != ZH_MAGIC) { st = ip == 0 ? ST_MAGIC : ST_CORRUPT; break; }
    ip += 4;
    if (srcn - ip < 1) { st = ST_CORRUPT; break; }
    u32 const fhd = ub(src + ip);
    u32 const fcsf = fhd >> 6, single = (fhd >> 5) & 1u, chk = (fhd >> 2) & 1u, didf = fhd & 3u;
    if (fhd & 8u) { st = ST_CORRUPT; break; }
    u32 const didn = didf == 0 ? 0u : didf == 1 ? 1u : didf == 2 ? 2u : 4u;
    u32 const fcsn = fcsf == 0 ? (single ? 1u : 0u) : fcsf == 1 ? 2u : fcsf == 2 ? 4u : 8u;
    u64 const hsz = 1ull + (single ? 0u : 1u) + didn + fcsn;
    if (srcn - ip < hsz) { st = ST_CORRUPT; break; }
    const u8 *h = src + ip + 1;
    if (!single) {
      u32 const wd = ub(h++);
      if (10 + (wd >> 3) > 30) { st = ST_CORRUPT; break; }
    }
    u32 did = 0;
    for (u32 i = 0; i < didn; i++) did |= ub(h + i) << (8 * i);
    h += didn;
    u64 fcs = ~0ull;
    if (fcsn == 1) fcs = ub(h);
    else if (fcsn == 2) fcs = rd16(h) + 256ull;
    else if (fcsn == 4) fcs = rd32(h);
    else if (fcsn == 8) fcs = (u64)rd32(h) | (u64)rd32(h + 4) << 32;
    if (did != 0 && (!a.dict || did != a.dict_id)) { st = ST_DICT; break; }  // libzstd: dictionary_wrong
    ip += hsz;
    if (fcs != ~0ull && fcs > cap - produced) { st = ST_SMALL; break; }
    u64 const fstart = produced;
    // frame state: repcodes, table kinds
    u32 rep0 = 1, rep1 = 4, rep2 = 8;
    bool const fdict = a.dict && a.dict_off;  // formatted dictionary: its tables and repcodes
    if (lane == 0) {
      L.tkind[0] = L.tkind[1] = L.tkind[2] = TAB_NONE;
      L.hvalid = 0;
      L.err = (fdict && !load_dict_entropy(L, a.dict, a.dict_off)) ? 1u : 0u;
    }
    __syncthreads();
    if (fdict) {
      if (uni(L.err)) { st = ST_DICT; break; }
      const u8 *const rp = a.dict + a.dict_off - 12;
      rep0 = rd32(rp);
      rep1 = rd32(rp + 4);
      rep2 = rd32(rp + 8);
    }
    // ---- blocks (RFC 8878 §3.1.1.2)
    for (;;) {
      if (srcn - ip < 3) { st = ST_CORRUPT; break; }
      u32 const bh = rd24(src + ip);
      u32 const last = bh & 1u, bt = (bh >> 1) & 3u, bsz = bh >> 3;
      ip += 3;
      u8 *const ob = dst + produced;  // this block's first output byte
      if (a.phase == 4 && !(bt == 2 && produced == 0 && last)) return;  // not deferrable
      if (bt == 0) {
        if (srcn - ip < bsz) { st = ST_CORRUPT; break; }
        if (bsz > cap - produced) { st = ST_SMALL; break; }
        wave_copy(ob, src + ip, bsz);
        ip += bsz;
        produced += bsz;
      } else if (bt == 1) {
        if (srcn - ip < 1) { st = ST_CORRUPT; break; }
        if (bsz > cap - produced) { st = ST_SMALL; break; }
        wave_fill(ob, ub(src + ip), bsz);
        ip += 1;
        produced += bsz;
      } else if (bt == 2) {
        if (bsz >= BLOCKSIZE_MAX || srcn - ip < bsz) { st = ST_CORRUPT; break; }
        const u8 *const bp = src + ip;
        LitSrc lits;
        DSTAMP(0);
        u32 ls;
        if constexpr (LDS::kTablesOnly) ls = skip_literals(bp, bsz);
        else ls = a.phase == 4 ? skip_literals(bp, bsz) : decode_literals(L, bp, bsz, sl, lits, st);
        DSTAMP(1);
        if (a.phase == 5 && produced == 0 && uni(handoff(a, item)->flag) == 1) {
          // deferred by phase 4: the literals are all this pass owes it (a corrupt literals
          // section takes it back: the status is written below, phase 3 skips it)
          DecHandoff *const ho = handoff(a, item);
          if (!ls) {
            if (lane == 0) ho->flag = 0;
            break;
          }
          if (lane == 0) {
            ho->litg = (u64)lits.g;
            ho->litrle = lits.rle;
            ho->litn = lits.n;
          }
#ifdef ZH_STAMPS
          // (-DZH_STAMPS: phase 5's split into the record's spare bytes, tools/p5_stamps.py)
          if (lane == 0) {
            u64 *const xs5 = (u64 *)((u8 *)ho + 5248);
            xs5[0] = stv[0];
            xs5[1] = L.lst_t[0] - (stp - stv[1]);
            xs5[2] = L.lst_t[1] - L.lst_t[0];
            xs5[3] = L.lst_t[2] - L.lst_t[1];
            xs5[4] = stp - L.lst_t[2];
            xs5[5] = lits.n;
          }
#endif
          return;  // phase 3 writes the size and status
        }
        if (!ls) {
          if (a.phase == 4) return;
          break;
        }
        // ---- sequences section header (RFC 8878 §3.1.1.3.2.1)
        const u8 *sp = bp + ls;
        u32 rem = bsz - ls;
        if (rem < 1) { st = ST_CORRUPT; break; }
        u32 nseq = ub(sp);
        if (nseq == 0) {
          if (rem != 1) { st = ST_CORRUPT; break; }
          sp += 1;
          rem -= 1;
        } else if (nseq < 128) {
          sp += 1;
          rem -= 1;
        } else if (nseq < 255) {
          if (rem < 2) { st = ST_CORRUPT; break; }
          nseq = ((nseq - 128) << 8) + ub(sp + 1);
          sp += 2;
          rem -= 2;
        } else {
          if (rem < 3) { st = ST_CORRUPT; break; }
          nseq = rd16(sp + 1) + 0x7F00u;
          sp += 3;
          rem -= 3;
        }
        u64 sumML = 0, sumLL = 0;
        if (nseq) {
          if (nseq > sl.seq_cap) { st = nseq > BLOCKSIZE_MAX / 3 + 1 ? ST_CORRUPT : ST_SMALL; break; }
          if (rem < 1) { st = ST_CORRUPT; break; }
          u32 const modes = ub(sp);
          sp += 1;
          rem -= 1;
          if (modes & 3u) { st = ST_CORRUPT; break; }
          // the table descriptions staged in LDS with one wave load: lane 0's NCount parse was a
          // chain of dependent global byte loads (three descriptions take <= ~240 bytes)
#ifndef ZH_DEC_TSTAGE
#define ZH_DEC_TSTAGE 320u
#endif
          u32 const tb = min(rem, (u32)ZH_DEC_TSTAGE);
          const u8 *tsrc = sp;
          if (ZH_DEC_TSTAGE) {
            for (u32 k = lane; k < tb; k += 64) L.u.sstage[k] = sp[k];
            __syncthreads();
            tsrc = L.u.sstage;
          }
          u32 const tavail = ZH_DEC_TSTAGE ? tb : rem;
          if (lane == 0) {
            u32 e = 0, used = 0;
            u32 const md[3] = {modes >> 6, (modes >> 4) & 3u, (modes >> 2) & 3u};
            L.bld[0] = L.bld[1] = L.bld[2] = 0;
            for (u32 t = 0; t < 3 && !e; t++) {
              s32 const u = seq_table(L, t, md[t], tsrc + used, tavail - used, true);
              if (u < 0) e = 1;
              else used += (u32)u;
            }
            L.err = e;
            L.used = used;
          }
          __syncthreads();
          if (uni(L.err)) { st = ST_CORRUPT; break; }
          {
            bool ok = true;
            for (u32 t = 0; t < 3; t++)
              if (uni(L.bld[t])) ok = ok && build_dtable_wave(L.fse + tab_off(t), L.norm + 64 * t, tab_maxsv(t), uni(L.tlog[t]));
            __syncthreads();
            if (!ok) {
              if (lane == 0) L.tkind[0] = L.tkind[1] = L.tkind[2] = TAB_NONE;  // (as the serial build left them unusable)
              st = ST_CORRUPT;
              break;
            }
          }
          DSTAMP(2);
          u32 const tused = uni(L.used);
          sp += tused;
          rem -= tused;
          if ((a.phase == 1 || a.phase == 4) && produced == 0 && last && ip + bsz + (chk ? 4ull : 0ull) == srcn) {
            // the buffer's only block: hand the sequence bitstream to zh_dec_seq_kernel
            DecHandoff *const ho = handoff(a, item);
#if ZH_DEC_QUAD
            // the quad sequence kernel's entries: newState | symbol << 9 | extra bits << 16 |
            // state bits << 24 (the extra bits of a code: LL / ML from the code tables, OF = code)
            for (u32 w = lane; w < 1280; w += 64) {
              u32 const e = L.fse[w], sym = e & 0x3Fu;
              u32 const xb = w < 512 ? L.info[0][sym] >> 24 : w < 768 ? sym : L.info[1][sym] >> 24;
              ho->tabs[w] = (e >> 16) | sym << 9 | xb << 16 | ((e >> 8) & 0xFFu) << 24;
            }
#else
            for (u32 w = lane; w < 1280; w += 64) ho->tabs[w] = L.fse[w];
#endif
            if (lane == 0) {
              ho->sp = (u64)sp;
              ho->rem = rem;
              ho->nseq = nseq;
              ho->lg = L.tlog[TAB_LL] | L.tlog[TAB_OF] << 8 | L.tlog[TAB_ML] << 16;
              if (a.phase == 1) {
                ho->litg = (u64)lits.g;
                ho->litrle = lits.rle;
                ho->litn = lits.n;
              }
              ho->fcs = fcs;
              ho->ipc = chk ? ip + bsz : ~0ull;
              ho->rep[0] = rep0;
              ho->rep[1] = rep1;
              ho->rep[2] = rep2;
              ho->flag = 1;
            }
            return;  // phase 3 writes the size and status
          }
          if (LDS::kTablesOnly || a.phase == 4) return;
          if constexpr (!LDS::kTablesOnly) {
          // ---- sequence bitstream (RFC 8878 §3.1.1.3.2.2): every lane decodes redundantly
          // (uniform control flow, no exec-mask work); lane j keeps record j of each 64
          BitRevS r;
          if (!r.start<true>(sp, rem)) { st = ST_CORRUPT; break; }
          u8 *const stg = L.u.sstage;
          // read k bits; the bitstream comes from an LDS stage refilled SSTAGE bytes at a time
          auto rd = [&](u32 k) -> u32 {
            if (!r.ensure<true>(stg, k)) {
              u32 lo, hi;
              r.stage_range(SSTAGE, lo, hi);
              stage_copy(stg, sp, lo, hi);
              __syncthreads();
              r.slo = (s32)uni(lo);
              r.ensure<true>(stg, k);
            }
            u32 const v = (u32)r.bits(k);
            r.pos -= (s32)k;
            return v;
          };
          u32 const lgLL = uni(L.tlog[TAB_LL]), lgOF = uni(L.tlog[TAB_OF]), lgML = uni(L.tlog[TAB_ML]);
          const u32 *TLL = L.fse + tab_off(TAB_LL), *TOF = L.fse + tab_off(TAB_OF), *TML = L.fse + tab_off(TAB_ML);
          u32 sLL = rd(lgLL), sOF = rd(lgOF), sML = rd(lgML);
          bool big = false;
          u64 rec = 0;
          for (u32 i = 0; i < nseq; i++) {
            // (table entries made wave-uniform: the chain runs in SGPRs)
            u32 const eLL = __builtin_amdgcn_readfirstlane(TLL[sLL]), eOF = __builtin_amdgcn_readfirstlane(TOF[sOF]),
                      eML = __builtin_amdgcn_readfirstlane(TML[sML]);
            u32 const ofc = eOF & 0xFFu;
            u32 const ofv = (1u << ofc) + rd(ofc);
            u32 const mi = __builtin_amdgcn_readfirstlane(L.info[1][eML & 0xFFu]);
            u32 const ml = (mi & 0xFFFFFFu) + rd(mi >> 24);
            u32 const li = __builtin_amdgcn_readfirstlane(L.info[0][eLL & 0xFFu]);
            u32 const ll = (li & 0xFFFFFFu) + rd(li >> 24);
            u32 const off = resolve_off(ofv, ll, rep0, rep1, rep2);
            big |= off >= OFF_LIMIT;
            sumLL += ll;
            sumML += ml;
            u64 const v = (u64)ll | (u64)(ml - 3) << 17 | (u64)off << 34;
            rec = lane == (i & 63u) ? v : rec;
            if ((i & 63u) == 63u || i + 1 == nseq) {
              if (lane <= (i & 63u)) sl.seq[(i & ~63u) + lane] = rec;
            }
            if (i + 1 < nseq) {
              sLL = (eLL >> 16) + rd((eLL >> 8) & 0xFFu);
              sML = (eML >> 16) + rd((eML >> 8) & 0xFFu);
              sOF = (eOF >> 16) + rd((eOF >> 8) & 0xFFu);
            }
          }
          if (r.pos > 0 || big) { st = ST_CORRUPT; break; }
          DSTAMP(3);
          }  // !kTablesOnly
        } else if (rem != 0) {
          st = ST_CORRUPT;
          break;
        }
        if (LDS::kTablesOnly || a.phase == 4) return;  // (no sequences: nothing deferred)
        if constexpr (!LDS::kTablesOnly) {
        if (sumLL > lits.n) { st = ST_CORRUPT; break; }
        u64 const total = lits.n + sumML;
        // RFC 8878 §3.1.1.2.4: a block regenerates at most Block_Maximum_Size (128 KiB), which
        // also keeps execute_block's u32 window arithmetic in range
        if (total > BLOCKSIZE_MAX) { st = ST_CORRUPT; break; }
        if (total > cap - produced) { st = ST_SMALL; break; }
        __threadfence_block();  // the records (and Huffman literals) are read back below
        __syncthreads();
        u32 const tl = lits.n - (u32)sumLL;
        s64 const fpos = (s64)(produced - fstart);  // frame bytes before this block
        bool const bad = !execute_block(L, sl, ob, fpos, lits, nseq, tl, dend, dlen);
        DSTAMP(4);
        if (bad) { st = ST_CORRUPT; break; }
        produced += total;
        ip += bsz;
        }  // !kTablesOnly
      } else {
        st = ST_CORRUPT;
        break;
      }
      __threadfence_block();
      if (last) break;
    }
    if (st != ST_OK) break;
    if (fcs != ~0ull && produced - fstart != fcs) { st = ST_CORRUPT; break; }
    if (chk) {
      if (srcn - ip < 4) { st = ST_CORRUPT; break; }
      u64 const hx = zh_xxh64(dst + fstart, produced - fstart);
      if ((u32)hx != rd32(src + ip)) { st = ST_CHECKSUM; break; }
      ip += 4;
    }
  }
#ifdef ZH_STAMPS
  DSTAMP(5);
  if (lane < 8) ((u64 *)sl.lit)[lane] = stv[lane];
#endif
  if (a.phase == 4) return;  // (an error met here is reported by phase 5)
  if (lane == 0) {
    a.out_sizes[item] = st == ST_OK ? produced : 0ull;
    if (a.statuses) a.statuses[item] = a.nvcomp_codes ? to_nvcomp(st) : st;
  }
}

extern "C" __global__ __launch_bounds__(DEC_THREADS) void zh_decode_kernel(ZhDecArgs a) {
  __shared__ DecLds L;
  decode_body(L, a);
}

// The split pipeline's phase 4 with the small LDS layout (a.phase == 4)
extern "C" __global__ __launch_bounds__(DEC_THREADS) void zh_dec_tables_kernel(ZhDecArgs a) {
  __shared__ DecLdsTab L;
  decode_body(L, a);
}

// Phase 3: execute the block of a buffer deferred by phase 1 (its sequence records are in
// the slot) and finish the frame.  Its own kernel with only the execution window in LDS
// (ExecLds, ~9 KB against DecLds' ~16 KB), so twice as many buffers execute per CU.
#ifndef ZH_EXEC_STAGE
#define ZH_EXEC_STAGE 2048  // (8192: 87.8 GB/s, 1024: 92.9, 2048: 92.8, 3072: 92.4; profiles/r06o_dec_exec_ab.json)
#endif
#ifndef ZH_EXEC_LSTAGE
#define ZH_EXEC_LSTAGE 0
#endif
#ifndef ZH_EXEC_BM
#define ZH_EXEC_BM 1
#endif
struct ExecLds {
  static constexpr bool kLitStage = ZH_EXEC_LSTAGE != 0;
  static constexpr bool kStartMap = ZH_EXEC_BM != 0;
  union {
    u8 out[ZH_EXEC_STAGE + 16];
  } u;
  s32 wvs[68];
  u32 wll[64], wlit[64], woff[64];
#if ZH_EXEC_BM
  static_assert(ZH_EXEC_STAGE <= 2048, "one start-map word per lane");
  alignas(8) u32 bm[128];  // word 2 w: the window bytes [32 w, 32 w + 32) where a sequence starts; 2 w + 1: starts before them
#endif
#if ZH_EXEC_LSTAGE
  __attribute__((aligned(16))) u8 lst[ZH_EXEC_STAGE + 32];  // the window's literal bytes
#endif
};

extern "C" __global__ __launch_bounds__(DEC_THREADS) void zh_dec_exec_kernel(ZhDecArgs a) {
  __shared__ ExecLds L;
  u32 const item = a.item0 + blockIdx.x, lane = lane_id();
  const u8 *const src = (const u8 *)(a.in_ptrs ? a.in_ptrs[item] : a.one_in);
  u8 *const dst = (u8 *)(a.in_ptrs ? a.out_ptrs[item] : a.one_out);
  u64 const cap = a.out_caps ? (u64)a.out_caps[item] : a.out_cap_all;
  Slot sl;
  sl.lit = a.ws + (size_t)item * a.slot_bytes;
  sl.lit_cap = a.block_cap;
  sl.seq = (u64 *)(sl.lit + a.lit_bytes);
  sl.seq_cap = a.seq_cap;
  const u8 *const dend = a.dict ? a.dict + a.dict_n : nullptr;
  s64 const dlen = a.dict ? (s64)(a.dict_n - a.dict_off) : 0;
  if (lane < 4) L.wvs[64 + lane] = 0x7FFFFFFF;
  __syncthreads();
  DecHandoff *const ho = handoff(a, item);
  if (uni(ho->flag) != 1) return;
  LitSrc lits;
  lits.g = (const u8 *)uni64(ho->litg);
  lits.rle = uni(ho->litrle);
  lits.n = uni(ho->litn);
  u32 const nseq = uni(ho->nseq);
  u64 const sumLL = uni64(ho->sumLL), sumML = uni64(ho->sumML), fcs = uni64(ho->fcs), ipc = uni64(ho->ipc);
#ifdef ZH_STAMPS
  u64 xs[8] = {};
  u64 const xt0 = __builtin_amdgcn_s_memtime();
#else
  u64 *const xs = nullptr;
#endif
  u32 st = ST_OK;
  u64 produced = 0;
  if (uni(ho->sbad) || sumLL > lits.n || lits.n + sumML > BLOCKSIZE_MAX) {
    st = ST_CORRUPT;
  } else if (lits.n + sumML > cap) {
    st = ST_SMALL;
  } else if (!execute_block(L, sl, dst, 0, lits, nseq, lits.n - (u32)sumLL, dend, dlen, xs)) {
    st = ST_CORRUPT;
  } else {
    produced = lits.n + sumML;
    if (fcs != ~0ull && produced != fcs) st = ST_CORRUPT;
  }
  if (st == ST_OK && ipc != ~0ull) {
    __threadfence_block();
    if ((u32)zh_xxh64(dst, produced) != rd32(src + ipc)) st = ST_CHECKSUM;
  }
#ifdef ZH_STAMPS
  xs[0] = __builtin_amdgcn_s_memtime() - xt0;
  xs[6] = nseq;
  xs[7] = produced;
  if (lane < 8) ((u64 *)sl.lit)[lane] = xs[lane];
#endif
  if (lane == 0) {
    a.out_sizes[item] = st == ST_OK ? produced : 0ull;
    if (a.statuses) a.statuses[item] = a.nvcomp_codes ? to_nvcomp(st) : st;
  }
  return;
}

// Sequence bitstreams of deferred buffers: lanes = buffers, 64 per wave, so the serial FSE
// state chains of 64 blocks advance under one instruction stream.  A step's only exposed
// memory latency is the three table reads (each lane's tables sit in its hand-off record);
// the bitstream window it needs was fetched one step earlier (win_fetch below), and decoded
// sequences leave through an LDS ring.  The chain is issue-latency bound: one wave per SIMD,
// ~180 dependent instructions a step.  Measured alternatives (profiles/r02m_dec_seq.json):
// 4-32 buffers per wave with the tables staged in LDS (32- or 16-bit entries) were slower,
// both isolated and pipelined -- LDS-limited occupancy, no shorter chain.
#ifndef ZH_D2_BUF
#define ZH_D2_BUF 64
#endif
[[maybe_unused]] constexpr u32 D2_BUF = ZH_D2_BUF;
// Decoded sequences go to an LDS ring and leave in 256-byte bursts every D2_RUN steps:
// CDNA's vmcnt counts stores too and retires in order, so a per-step global store would
// make every window load wait for the previous step's write acknowledgement.
[[maybe_unused]] constexpr u32 D2_RUN = 32;

// the top k (<= 31) bits of T; T <<= k
__device__ __forceinline__ u32 take(u64 &T, u32 k) {
  u32 const hi32 = (u32)(T >> 32);
  u32 const v = k ? hi32 >> (32u - k) : 0u;
  T <<= k;
  return v;
}

// resolve_off without branches (the lanes of a wave decode different blocks)
__device__ __forceinline__ u32 resolve_off_bf(u32 ofv, u32 ll, u32 &r0, u32 &r1, u32 &r2) {
  bool const lit = ofv > 3;
  u32 const idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // repeat index when !lit: 0..3
  u32 rs = idx == 1 ? r1 : idx == 2 ? r2 : r0 - 1;
  rs += rs == 0 ? 1u : 0u;
  u32 const off = lit ? ofv - 3 : idx == 0 ? r0 : rs;
  bool const upd = lit || idx != 0;
  u32 const n2 = (!lit && idx == 1) ? r2 : r1;
  r2 = upd ? n2 : r2;
  r1 = upd ? r0 : r1;
  r0 = upd ? off : r0;
  return off;
}

// a 320-bit bitstream window: the five little-endian words from an 8-aligned address
struct Win5 {
  u64 w0, w1, w2, w3, w4;
};

// 64 bits of the window ending at bit t (t < 320), bit t - 1 as the MSB; bits below the
// window read as zeros (t < 64: the stream's first bits).  Two halving selects, not a word
// index: an indexed form is lowered to a scratch array.
__device__ __forceinline__ u64 win64(const Win5 &w, u32 t) {
  u32 const b = t - 64u, r = b & 63u;
  bool const h2 = b >= 128u, h1 = (b & 64u) != 0u;
  u64 const y0 = h2 ? w.w2 : w.w0, y1 = h2 ? w.w3 : w.w1, y2 = h2 ? w.w4 : w.w2;
  u64 const lo = h1 ? y1 : y0, hi = h1 ? y2 : y1;
  u64 const v = r ? (lo >> r) | (hi << (64u - r)) : lo;
  return (s32)b < 0 ? w.w0 << ((64u - t) & 63u) : v;
}

typedef const __attribute__((address_space(1))) u64 *gptr64;

// the five words from the 8-aligned address A (global, not flat, loads: LDS waits do not
// wait for them; one address, four immediate offsets)
__device__ __forceinline__ Win5 win_fetch(uintptr_t A) {
  gptr64 const q = (gptr64)A;
  return Win5{q[0], q[1], q[2], q[3], q[4]};
}

#if ZH_DEC_QUAD
// Quad sequence kernel: FOUR lanes per buffer, 16 buffers per wave.  A block's FSE chain is
// serial (decoding from a guessed entry never rejoins the true trajectory: tools/seq_sync.py
// measured 0 of 240 guesses synchronising over whole C3 blocks), so the step itself is what
// has to get shorter.  Lane q of a quad owns one table: 0 = offsets, 1 = match lengths,
// 2 = literal lengths, 3 = the record (repcodes, ring).  A step is the same instruction stream
// for all of them: one table read each (entries repacked by phase 1 as newState | symbol << 9
// | extra bits << 16 | state bits << 24), three quad broadcasts (DPP) give every lane the
// bit offsets of its two fields (extra bits in the order OF, ML, LL from the top, then the
// states LL, ML, OF), two 64-bit reads of a 32-byte window the previous step staged in LDS
// by an LDS-DMA load, and three broadcasts more hand the values to lane 3.  About half the
// instructions of the one-lane step, and four times as many waves to share the SIMDs the
// 64-buffer waves left idle.
#ifndef ZH_DQ_XCD
#define ZH_DQ_XCD 0
#endif
#ifndef ZH_DQ_PF
#define ZH_DQ_PF 0
#endif
constexpr u32 DQ_BUF = 16;  // buffers per wave
constexpr u32 DQ_RUN = 32;  // records per ring run (256 bytes per buffer)

// resolve_off_bf with the repeat candidates picked by masks: the nested selects of the
// one-lane kernel compile to exec-mask branches here
__device__ __forceinline__ u32 resolve_off_masks(u32 ofv, u32 ll, u32 &r0, u32 &r1, u32 &r2) {
  bool const lit = ofv > 3;
  u32 const idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // repeat index when !lit: 0..3
  u32 const m1 = 0u - (u32)(idx == 1), m2 = 0u - (u32)(idx == 2), m3 = 0u - (u32)(idx == 3);
  u32 rs = (r1 & m1) | (r2 & m2) | ((r0 - 1) & m3);
  rs += rs == 0 ? 1u : 0u;
  u32 const off = lit ? ofv - 3 : idx == 0 ? r0 : rs;
  bool const upd = lit || idx != 0;
  u32 const n2 = (r2 & m1) | (r1 & ~m1);  // (a literal offset has m1 = 0)
  r2 = upd ? n2 : r2;
  r1 = upd ? r0 : r1;
  r0 = upd ? off : r0;
  return off;
}

template <u32 L>
__device__ __forceinline__ u32 quad_bcast(u32 v) {
  return ZH_DPP(v, L * 0x55u, 0xf);  // quad_perm [L, L, L, L]
}

typedef const __attribute__((address_space(1))) void *gvoid;
typedef __attribute__((address_space(3))) void *lvoid;

extern "C" __global__ __launch_bounds__(64) void zh_dec_seq_kernel(ZhDecArgs a, u32 nitems) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ u32 info[4][64];  // baselines by code: OF (1 << code), ML, LL, none
  __shared__ __attribute__((aligned(16))) u32 win[2][DQ_BUF][16];  // stream windows, 64 B per quad
  __shared__ __attribute__((aligned(16))) u64 ring[DQ_BUF][DQ_RUN];
#if ZH_DQ_PF
  __shared__ u32 pfd[64];  // (the prefetch's landing words, never read)
#endif
  u32 const lane = lane_id(), q = lane & 3u, b = lane >> 2;
  info[0][lane] = lane < 32 ? 1u << lane : 0u;
  info[1][lane] = lane < 53 ? c_ML_info[lane] & 0xFFFFFFu : 0u;
  info[2][lane] = lane < 36 ? c_LL_info[lane] & 0xFFFFFFu : 0u;
  info[3][lane] = 0u;
  __syncthreads();
#if ZH_DQ_XCD
  // the items phase 1 ran on this workgroup's XCD (blocks b and b + 8 share one): workgroup w
  // takes items w % 8 + 8 (16 (w / 8) + b), so their tables are in the local L2 (speed only)
  u32 const it = a.item0 + (blockIdx.x & 7u) + 8u * (DQ_BUF * (blockIdx.x >> 3) + b), end = a.item0 + nitems;
#else
  u32 const it = a.item0 + blockIdx.x * DQ_BUF + b, end = a.item0 + nitems;
#endif
  if (it >= end) return;  // (quad-uniform from here on: the four lanes read the same buffer)
  DecHandoff *const ho = handoff(a, it);
  if (ho->flag != 1) return;
  const u32 *const tq = ho->tabs + (q == 0 ? 512u : q == 1 ? 768u : 0u);
  const u8 *const sp = (const u8 *)ho->sp;
  u32 const nseq = ho->nseq, lg = ho->lg;
  s32 const n = (s32)ho->rem;
  u64 *const seq = (u64 *)(a.ws + (size_t)it * a.slot_bytes + a.lit_bytes);
  u32 const lastb = n > 0 ? sp[n - 1] : 0u;
  bool const bad = lastb == 0;
  s32 pos = bad ? 0 : 8 * (n - 1) + (s32)hb32(lastb);
  u32 rep0 = ho->rep[0], rep1 = ho->rep[1], rep2 = ho->rep[2];
  bool big = false;
  u64 acc = 0;  // lane 1: sum of match lengths, lane 2: of literal lengths
  if (!bad) {
    // The window of a step holds the 32 stream bytes from A = (the byte of bit pos - 89) & ~15
    // (a step reads at most 89 bits below pos): lanes 0 and 1 load its two 16-byte pieces, lanes
    // 2 and 3 the lines 128 and 256 bytes further down (a prefetch; their LDS pieces are never
    // read).  Pieces are clamped to the 16-byte chunks holding the stream's first and last byte,
    // so no load leaves the pages the stream touches; the bits a valid stream reads always lie in
    // the first 32 bytes of the window (bits below the stream start are the frame's own bytes and
    // are only read by corrupt streams, which end with pos != 0).
    uintptr_t const base = (uintptr_t)sp, wlo = base & ~(uintptr_t)15;
    s32 const bofs = (s32)(base - wlo), wspan = (s32)(((base + (u32)n - 1) & ~(uintptr_t)15) - wlo);
    s32 const qoff = q == 0 ? 0 : q == 1 ? 16 : q == 2 ? -128 : -256;
    auto fetch = [&](s32 p, u32 buf) -> s32 {  // -> the window's first stream bit
      s32 const A = max(((p - 89) >> 3) + bofs, 0) & ~15;  // byte offsets from wlo
      s32 const P = min(max(A + qoff, 0), wspan);
      __builtin_amdgcn_global_load_lds((gvoid)(wlo + (u32)P), (lvoid)&win[buf][0][0], 16, 0, 0);
      return 8 * (A - bofs);
    };
    // k bits whose lowest is window bit lo (lo within [0, 224) for valid streams)
    auto field = [&](u32 buf, s32 lo, u32 k) -> u32 {
      u32 const d = min((u32)(lo >> 5), 6u);
      u32 const w0 = win[buf][b][d], w1 = win[buf][b][d + 1];
      return __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(w1, w0, (u32)lo & 31u), 0u, k);
    };
    s32 wb = fetch(pos, 0);
    u32 s;
    {  // initial states, from the top: LL, OF, ML
      u32 const kL = lg & 0xFFu, kO = (lg >> 8) & 0xFFu, kM = lg >> 16;
      u32 const k = q == 0 ? kO : q == 1 ? kM : q == 2 ? kL : 0u;
      u32 const off = q == 0 ? kL : q == 1 ? kL + kO : 0u;
      s = field(0, pos - (s32)(off + k) - wb, k);
      pos -= (s32)(kL + kO + kM);
    }
    // software-pipelined: the table read of step i + 1 is issued as soon as its state is
    // known, before step i's record work, which then covers its latency
    u32 e = tq[s];
    for (u32 i = 0; i < nseq; i++) {
      u32 const cur = i & 1u;
      u32 const v = q == 3 ? 0u : e >> 16;  // extra bits | state bits << 8
      u32 const v0 = quad_bcast<0>(v), v1 = quad_bcast<1>(v), v2 = quad_bcast<2>(v);
      u32 const s01 = v0 + v1, S = s01 + v2;
      u32 const pre = q == 0 ? 0u : q == 1 ? v0 : s01;  // the fields of the lanes before this one
      bool const more = i + 1 < nseq;                    // the last sequence reads no states
      u32 const X = S & 0xFFu, NB = more ? S >> 8 : 0u;
      u32 const xb = v & 0xFFu, nb = more ? v >> 8 : 0u;
      u32 const xv = field(cur, pos - (s32)((pre & 0xFFu) + xb) - wb, xb);
      u32 const sv = field(cur, pos - (s32)(X + NB) + (s32)(pre >> 8) - wb, nb);
      pos -= (s32)(X + NB);
#if ZH_DQ_PF
      // the next entry lies in [newState, newState + 2^nb): one 128-byte line when nb <= 5;
      // touch it before the window read that finishes the state (an LDS-DMA load, so no
      // register waits for it)
      __builtin_amdgcn_global_load_lds((gvoid)(tq + (e & 0x1FFu)), (lvoid)&pfd[0], 4, 0, 0);
#endif
      s = q == 3 ? 0u : (e & 0x1FFu) + sv;
      u32 const en = tq[s];       // step i + 1 (after the last step: a harmless read)
      wb = fetch(pos, cur ^ 1u);  // (after the last step too: no branch; drained below)
      u32 const val = info[q][(e >> 9) & 0x3Fu] + xv;
      acc += val;
      // the record (every lane of the quad computes it; lane 3 keeps it)
      u32 const ofv = quad_bcast<0>(val), ml = quad_bcast<1>(val), ll = quad_bcast<2>(val);
      u32 const off = resolve_off_masks(ofv, ll, rep0, rep1, rep2);
      big |= off >= OFF_LIMIT;
      u32 const r = i & (DQ_RUN - 1);
      if (q == 3) ring[b][r] = (u64)ll | (u64)(ml - 3) << 17 | (u64)off << 34;
      if (r == DQ_RUN - 1) {  // a full run: 256 bytes, 64 from each lane of the quad
        uint4 *const dst = (uint4 *)(seq + (i + 1 - DQ_RUN)) + 4 * q;
        const uint4 *const srcr = (const uint4 *)ring[b] + 4 * q;
#pragma unroll
        for (u32 k = 0; k < 4; k++) dst[k] = srcr[k];
      }
      e = en;
    }
    for (u32 k = (nseq & ~(DQ_RUN - 1)) + q; k < nseq; k += 4) seq[k] = ring[b][k & (DQ_RUN - 1)];  // the partial last run
    __builtin_amdgcn_s_waitcnt(0);  // the last window load lands before the workgroup's LDS is released
  }
  if (q == 1) ho->sumML = acc;
  if (q == 2) ho->sumLL = acc;
  if (q == 3) ho->sbad = (bad || pos != 0 || big) ? 1u : 0u;
}
#else
extern "C" __global__ __launch_bounds__(D2_BUF) void zh_dec_seq_kernel(ZhDecArgs a, u32 nitems) {
  // highest issue priority: the chains are issue-latency bound and share SIMDs with the
  // phase-1 / phase-3 waves of the other groups of the pipeline
  __builtin_amdgcn_s_setprio(3);
  __shared__ u32 info[2][64];
  __shared__ u64 ring[D2_BUF][D2_RUN];
  u32 const lane = lane_id();
  for (u32 i = lane; i < 53; i += D2_BUF) {
    if (i < 36) info[0][i] = c_LL_info[i];
    info[1][i] = c_ML_info[i];
  }
  u32 const it0 = a.item0 + blockIdx.x * D2_BUF, end = a.item0 + nitems;
  __syncthreads();
  u32 const it = it0 + lane;
  if (lane >= D2_BUF || it >= end) return;
  DecHandoff *const ho = handoff(a, it);
  if (ho->flag != 1) return;
  const u32 *const TLL = ho->tabs, *const TOF = TLL + 512, *const TML = TLL + 768;
  const u8 *const sp = (const u8 *)ho->sp;
  u32 const nseq = ho->nseq, lg = ho->lg;
  s32 const n = (s32)ho->rem;
  u64 *const seq = (u64 *)(a.ws + (size_t)it * a.slot_bytes + a.lit_bytes);
  u32 const last = n > 0 ? sp[n - 1] : 0u;
  bool const bad = last == 0;
  s32 pos = bad ? 0 : 8 * (n - 1) + (s32)hb32(last);
  u32 rep0 = ho->rep[0], rep1 = ho->rep[1], rep2 = ho->rep[2];
  bool big = false;
  u64 sumLL = 0, sumML = 0;
  if (!bad) {
    // Bitstream window: w holds the 40 bytes from A, fetched one step ahead -- the window
    // a step reads was fetched at the start of the previous step for that step's position,
    // which covers the 128 bits below the current one (a step consumes <= 89 bits), so the
    // fetch latency hides behind a step of arithmetic.
    // The window start is clamped to the stream's aligned words [wlo, whi]: near the stream
    // start bits below the window read as zeros, near its end the window still covers the
    // top.  A stream of at most 33 bytes fits one window: it is fetched once, word by word.
    uintptr_t const base = (uintptr_t)sp, wlo = base & ~(uintptr_t)7, whi = (base + (u32)n - 1) & ~(uintptr_t)7;
    bool const small = whi < wlo + 32;
    uintptr_t const ahi = small ? wlo : whi - 32;
    auto wbase = [&](s32 p) {
      uintptr_t const A = (base + (uintptr_t)(intptr_t)(((p + 7) >> 3) - 32)) & ~(uintptr_t)7;
      return small ? wlo : (intptr_t)A < (intptr_t)wlo ? wlo : A > ahi ? ahi : A;
    };
    uintptr_t A = wbase(pos);
    Win5 w;
    if (small) {
      auto ld = [&](uintptr_t q) { return *(gptr64)(q > whi ? whi : q); };
      w = Win5{ld(wlo), ld(wlo + 8), ld(wlo + 16), ld(wlo + 24), ld(wlo + 32)};
    } else {
      w = win_fetch(A);
    }
    auto tpos = [&](s32 p) { return (u32)((s32)(8 * (intptr_t)(base - A)) + p); };
    u32 sLL, sOF, sML;
    {  // initial states
      u64 T = win64(w, tpos(pos));
      u32 const kL = lg & 0xFFu, kO = (lg >> 8) & 0xFFu, kM = lg >> 16;
      sLL = take(T, kL);
      sOF = take(T, kO);
      sML = take(T, kM);
      pos -= (s32)(kL + kO + kM);
    }
    for (u32 i = 1; i <= nseq; i++) {  // step i: sequence i - 1
      u32 const eLL = TLL[sLL], eOF = TOF[sOF], eML = TML[sML];
      // issued after the table reads: vmcnt retires in order, so waiting for the tables
      // leaves this fetch in flight (it is consumed by the next step)
      uintptr_t const An = wbase(pos);
      // (a small stream keeps its window; its lane fetches from its own hand-off record
      // instead, so the fetch is unconditional and the table wait can leave it in flight)
      Win5 wn = win_fetch(small ? (uintptr_t)ho : An);  // for step i + 1
      if (small) wn = w;
      u32 const ofc = eOF & 0xFFu;
      u32 const mi = info[1][eML & 0xFFu], li = info[0][eLL & 0xFFu];
      u32 const mb = mi >> 24, lb = li >> 24;
      u32 t = tpos(pos);
      u32 const t0 = t;
      u64 T = win64(w, t);
      u32 const ofv = (1u << ofc) + take(T, ofc);
      u32 const ml = (mi & 0xFFFFFFu) + take(T, mb);
      u32 const ll = (li & 0xFFFFFFu) + take(T, lb);
      t -= ofc + mb + lb;
      u32 const off = resolve_off_bf(ofv, ll, rep0, rep1, rep2);
      big |= off >= OFF_LIMIT;
      sumLL += ll;
      sumML += ml;
      u32 const r = (i - 1) & (D2_RUN - 1);
      ring[lane][r] = (u64)ll | (u64)(ml - 3) << 17 | (u64)off << 34;
      if (r == D2_RUN - 1) {  // a full run: 32 sequences, 256-byte aligned
        uint4 *const dst = (uint4 *)(seq + (i - D2_RUN));
        const uint4 *const srcr = (const uint4 *)ring[lane];
#pragma unroll
        for (u32 k = 0; k < D2_RUN / 2; k++) dst[k] = srcr[k];
      }
      if (i < nseq) {
        u32 const kL = (eLL >> 8) & 0xFFu, kM = (eML >> 8) & 0xFFu, kO = (eOF >> 8) & 0xFFu;
        u64 U = win64(w, t);
        sLL = (eLL >> 16) + take(U, kL);
        sML = (eML >> 16) + take(U, kM);
        sOF = (eOF >> 16) + take(U, kO);
        t -= kL + kM + kO;
      }
      pos -= (s32)(t0 - t);
      A = An;
      w = wn;
    }
    for (u32 k = nseq & ~(D2_RUN - 1); k < nseq; k++) seq[k] = ring[lane][k & (D2_RUN - 1)];  // the partial last run
  }
  ho->sumLL = sumLL;
  ho->sumML = sumML;
  ho->sbad = (bad || pos != 0 || big) ? 1u : 0u;
}
#endif  // ZH_DEC_QUAD

namespace {
struct DecPipeTag {};
}  // namespace

namespace zh {
u32 dec_lds_bytes() { return (u32)sizeof(DecLds); }
hipError_t launch_decompress(const ZhDecArgs &a0, u32 nitems, hipStream_t stream) {
  if (!nitems) return hipSuccess;
  // ZH_DEC_SYNC=1 (diagnostics only): synchronise and report after each of the three kernels
  static const bool dbg = getenv("ZH_DEC_SYNC") != nullptr;
  // items [first, first + cnt): phase 1, the sequence kernel, phase 3, in order on s;
  // after_p1 (optional) is recorded once phase 1 is queued
  auto group = [&](u32 first, u32 cnt, hipStream_t s, hipEvent_t after_p1) {
    auto check = [&](const char *k) {
      if (!dbg) return;
      hipError_t e = hipStreamSynchronize(s);
      fprintf(stderr, "zh_decode: %s -> %s\n", k, hipGetErrorString(e));
    };
    ZhDecArgs a = a0;
    a.item0 = first;
    a.phase = 1;
    hipLaunchKernelGGL(zh_decode_kernel, dim3(cnt), dim3(DEC_THREADS), 0, s, a);
    check("phase 1");
    if (after_p1) (void)hipEventRecord(after_p1, s);
#if ZH_DEC_QUAD
#if ZH_DQ_XCD
    hipLaunchKernelGGL(zh_dec_seq_kernel, dim3(((cnt + 8 * DQ_BUF - 1) / (8 * DQ_BUF)) * 8), dim3(64), 0, s, a, cnt);
#else
    hipLaunchKernelGGL(zh_dec_seq_kernel, dim3((cnt + DQ_BUF - 1) / DQ_BUF), dim3(64), 0, s, a, cnt);
#endif
#else
    hipLaunchKernelGGL(zh_dec_seq_kernel, dim3((cnt + D2_BUF - 1) / D2_BUF), dim3(D2_BUF), 0, s, a, cnt);
#endif
    check("sequences");
    hipLaunchKernelGGL(zh_dec_exec_kernel, dim3(cnt), dim3(DEC_THREADS), 0, s, a);
    check("phase 3");
  };
  // Large batches run as G groups on staggered streams (zh_pipe.h): group k's phase 1 starts
  // once group k-1's phase 1 is done, so the sequence kernel of a group (one wave per 64
  // buffers, a ~7 ms issue-latency-bound chain whatever the group size) overlaps the phase 1
  // of the later group and the execution of the earlier one.  The end is about phase 1 of
  // every group + one chain + the last group's execution, so the first group is the larger
  // (2 : 1).  Measured (profiles/r02m_dec_seq.json): G = 1 / 2 / 3 / 4 / 8 -> 56.8 / 59.1 /
  // 56.0 / 56.2 / 36.6 GB/s, 2 : 1 and 3 : 1 splits 59.3 / 59.7.  Re-measured in round 4 with
  // the current kernels (tools/dec_ab.sh, profiles/r04zd_decode_groups_ab.json): G = 1 / 2 / 3
  // -> 57.6 / 60.6 / 59.1 GB/s; two groups 1 : 1 / 2 : 1 / 3 : 1 -> 60.6 / 60.6 / 60.5.
  // Round 6 (quad sequence kernel ~4.3 ms, segment-parallel literals: phase 1 4.5 -> 2.5 ms;
  // profiles/r06n_dec_hufpar_ab.json): two groups 1 : 1 / 2 : 1 / 3 : 1 -> 87.9 / 85.3 / 85.7
  // GB/s, three groups 2 : 1 : 1 / 1 : 1 : 1 -> 86.9 / 81.0, four 1 : 1 : 1 : 1 80.5.
#ifndef ZH_DEC_G
#define ZH_DEC_G 2
#endif
#ifndef ZH_DEC_W0
#define ZH_DEC_W0 1
#endif
#ifndef ZH_DEC_SPLIT
#define ZH_DEC_SPLIT 1
#endif
#if ZH_DEC_SPLIT
  // Split pipeline: phase 4 (headers + sequence tables of the deferrable buffers, no literals)
  // gates the sequence kernel, which then runs every chain at once beside phase 5 (the
  // literals, and whole decodes of the other buffers) on the side stream; phase 3 waits for
  // both.  The chains no longer wait for the Huffman literals.
  if (StreamPipe<2> *const sp2 = (!dbg && nitems >= 2048) ? stream_pipe<DecPipeTag, 2>(stream) : nullptr) {
    std::lock_guard<std::mutex> lk(sp2->mu);
    hipStream_t const side = sp2->side[0];
    ZhDecArgs a = a0;
    a.item0 = 0;
    a.phase = 4;
#ifndef ZH_DEC_TABK
#define ZH_DEC_TABK 1
#endif
    if (ZH_DEC_TABK) hipLaunchKernelGGL(zh_dec_tables_kernel, dim3(nitems), dim3(DEC_THREADS), 0, stream, a);
    else hipLaunchKernelGGL(zh_decode_kernel, dim3(nitems), dim3(DEC_THREADS), 0, stream, a);
    (void)hipEventRecord(sp2->first_done[0], stream);
    (void)hipStreamWaitEvent(side, sp2->first_done[0], 0);
    a.phase = 5;
#ifndef ZH_DEC_P5_PAD
#define ZH_DEC_P5_PAD 0  // (occupancy experiments: dynamic LDS added to phase 5's workgroups)
#endif
    hipLaunchKernelGGL(zh_decode_kernel, dim3(nitems), dim3(DEC_THREADS), ZH_DEC_P5_PAD, side, a);
    (void)hipEventRecord(sp2->done[0], side);
#ifdef ZH_DEC_SERIAL_P5
    (void)hipStreamWaitEvent(stream, sp2->done[0], 0);  // (diagnostic: phase 5 and the chains one after the other)
#endif
    hipLaunchKernelGGL(zh_dec_seq_kernel, dim3((nitems + DQ_BUF - 1) / DQ_BUF), dim3(64), 0, stream, a, nitems);
    (void)hipStreamWaitEvent(stream, sp2->done[0], 0);
    a.phase = 3;
    hipLaunchKernelGGL(zh_dec_exec_kernel, dim3(nitems), dim3(DEC_THREADS), 0, stream, a);
    return hipGetLastError();
  }
#endif
  constexpr u32 G = ZH_DEC_G, W0 = ZH_DEC_W0, MIN_GROUP = 1024;
  StreamPipe<G> *p = (!dbg && nitems >= G * MIN_GROUP) ? stream_pipe<DecPipeTag, G>(stream) : nullptr;
  if (!p) {
    group(0, nitems, stream, nullptr);
    return hipGetLastError();
  }
  u32 const shares = W0 + G - 1, unit = nitems / shares;  // group 0: W0 shares, others one
  p->run(stream, [&](u32 k, hipStream_t s, hipEvent_t after_first) {
    u32 const first = k == 0 ? 0u : (W0 + k - 1) * unit;
    u32 const last = k + 1 == G ? nitems : (W0 + k) * unit;
    group(first, last - first, s, after_first);
  });
  return hipGetLastError();
}
}  // namespace zh
