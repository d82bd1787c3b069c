/*
 * zstd_oracle.c — CPU restatement of the gfx950 compression path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker.
 * The product (custom-nvcomp-with-zstd_amd/) never links or calls it.
 *
 * What it restates
 * ----------------
 *  * Frame header: the reference's write_frame_header choices
 *    (src/cuda_zstd_manager.cu:3998-4106): magic, FHD with Single_Segment iff
 *    content <= block_size, FCS 1/2(-256)/4 bytes, window descriptor
 *    (window_log-10)<<3 otherwise.
 *  * Block header / Raw / RLE / Compressed choice: write_block
 *    (src/cuda_zstd_manager.cu:4227-4286) and the RLE probe (:336-362, :2775-2823).
 *  * Sequence codes: RFC 8878 tables, as in the reference's ZstdSequence
 *    helpers (include/cuda_zstd_internal.h:235-455) and predefined norms
 *    (src/cuda_zstd_fse.cu:2507-2528).
 *  * Interleaved FSE sequence encode order: the reference's
 *    k_encode_fse_interleaved (src/cuda_zstd_fse_encoding_kernel.cu:32-195),
 *    which follows libzstd ZSTD_encodeSequences.
 *  * Entropy stage (literals Huffman, FSE normalisation / NCount / CTable,
 *    encoding-type selection): the reference routes every <1 MiB input to host
 *    libzstd (src/cuda_zstd_manager.cu:1604-1668), so the entropy coder the
 *    reference actually runs on this path is libzstd's.  This file restates the
 *    published libzstd v1.4.9 algorithms (FSE_normalizeCount, FSE_writeNCount,
 *    FSE_buildCTable, HUF_buildCTable, HUF_writeCTable, HUF_compress1X/4X,
 *    ZSTD_compressLiterals, ZSTD_selectEncodingType for strategy < lazy,
 *    ZSTD_buildCTable, ZSTD_encodeSequences).  Parity is pinned stage by stage
 *    against the library (tests/test_oracle_stages.py, tests/golden/).
 *  * LZ stage: the reference's find_matches_kernel/greedy parse
 *    (src/lz77_parallel.cu:26-70, :177-268) is nondeterministic (atomicExch hash
 *    insert), so this file defines the deterministic parse the GPU runs:
 *      - two hash tables of 2^13 positions: "long" keyed by 8 bytes, "short" by
 *        5 bytes (dfast-like, level 3),
 *      - insertion in tiles of 256 positions: a lookup sees every position of
 *        earlier tiles (latest wins), none of its own tile,
 *      - per-position best = longer of the two candidates (long needs >= 8,
 *        short >= 5), lengths capped at 64,
 *      - greedy parse with one-step lazy deferral (take p unless len[p+1] > len[p]),
 *      - a match directly followed (LL = 0) by one with the same offset is merged.
 *    Output of this stage is pinned by libzstd round-trip of every frame.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>

#include "../include/zstd_hip_params.h"

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int16_t s16;

/* ------------------------------------------------------------------------ */
/* RFC 8878 tables (reference: include/cuda_zstd_internal.h:235-455)        */
/* ------------------------------------------------------------------------ */
static const u8 LL_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const u8 ML_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
/* predefined distributions (reference src/cuda_zstd_fse.cu:2507-2528) */
static const s16 LL_defNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const s16 ML_defNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const s16 OF_defNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

static inline u32 highbit32(u32 v) { return 31u - (u32)__builtin_clz(v); }

static inline u32 ll_code(u32 ll) {
  static const u8 LL_Code[64] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 16, 17, 17, 18, 18, 19, 19,
                                 20, 20, 20, 20, 21, 21, 21, 21, 22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                                 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
  return ll > 63 ? highbit32(ll) + 19 : LL_Code[ll];
}
static inline u32 ml_code(u32 mlBase) {
  static const u8 ML_Code[128] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                  32, 32, 33, 33, 34, 34, 35, 35, 36, 36, 36, 36, 37, 37, 37, 37, 38, 38, 38, 38, 38, 38, 38, 38, 39, 39, 39, 39, 39, 39, 39, 39,
                                  40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41,
                                  42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42};
  return mlBase > 127 ? highbit32(mlBase) + 36 : ML_Code[mlBase];
}

/* ------------------------------------------------------------------------ */
/* Bit writer: fields appended LSB-first, bytes little-endian (BIT_CStream)  */
/* ------------------------------------------------------------------------ */
typedef struct { u8 *p, *start, *end; u64 acc; u32 nb; int overflow; } bitw_t;
static void bw_init(bitw_t *b, u8 *dst, size_t cap) { b->p = b->start = dst; b->end = dst + cap; b->acc = 0; b->nb = 0; b->overflow = 0; }
static inline void bw_add(bitw_t *b, u64 v, u32 n) {
  if (!n) return;
  b->acc |= (v & ((n == 64) ? ~0ull : ((1ull << n) - 1))) << b->nb;
  b->nb += n;
  while (b->nb >= 8) { if (b->p < b->end) *b->p++ = (u8)b->acc; else b->overflow = 1; b->acc >>= 8; b->nb -= 8; }
}
/* BIT_closeCStream: end mark then flush; returns byte size (0 on overflow) */
static size_t bw_close(bitw_t *b) {
  bw_add(b, 1, 1);
  if (b->nb) { if (b->p < b->end) *b->p++ = (u8)b->acc; else b->overflow = 1; b->acc = 0; b->nb = 0; }
  return b->overflow ? 0 : (size_t)(b->p - b->start);
}

/* ------------------------------------------------------------------------ */
/* FSE (libzstd v1.4.9 fse_compress.c restated)                              */
/* ------------------------------------------------------------------------ */
#define FSE_MIN_TABLELOG 5
#define FSE_MAX_TABLELOG 12

static u32 fse_min_table_log(size_t srcSize, u32 maxSymbolValue) {
  u32 minBitsSrc = highbit32((u32)srcSize) + 1;
  u32 minBitsSymbols = highbit32(maxSymbolValue) + 2;
  return minBitsSrc < minBitsSymbols ? minBitsSrc : minBitsSymbols;
}
static u32 fse_optimal_table_log_internal(u32 maxTableLog, size_t srcSize, u32 maxSymbolValue, u32 minus) {
  u32 maxBitsSrc = highbit32((u32)(srcSize - 1)) - minus;
  u32 tableLog = maxTableLog;
  u32 minBits = fse_min_table_log(srcSize, maxSymbolValue);
  if (tableLog == 0) tableLog = 11;
  if (maxBitsSrc < tableLog) tableLog = maxBitsSrc;
  if (minBits > tableLog) tableLog = minBits;
  if (tableLog < FSE_MIN_TABLELOG) tableLog = FSE_MIN_TABLELOG;
  if (tableLog > FSE_MAX_TABLELOG) tableLog = FSE_MAX_TABLELOG;
  return tableLog;
}
u32 orc_fse_optimal_table_log(u32 maxTableLog, size_t srcSize, u32 maxSymbolValue) {
  return fse_optimal_table_log_internal(maxTableLog, srcSize, maxSymbolValue, 2);
}

static int fse_normalize_m2(s16 *norm, u32 tableLog, const u32 *count, size_t total, u32 maxSV, s16 lowProbCount) {
  const s16 NOT_YET = -2;
  u32 distributed = 0, toDistribute;
  u32 lowThreshold = (u32)(total >> tableLog);
  u32 lowOne = (u32)((total * 3) >> (tableLog + 1));
  for (u32 s = 0; s <= maxSV; s++) {
    if (count[s] == 0) { norm[s] = 0; continue; }
    if (count[s] <= lowThreshold) { norm[s] = lowProbCount; distributed++; total -= count[s]; continue; }
    if (count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
    norm[s] = NOT_YET;
  }
  toDistribute = (1u << tableLog) - distributed;
  if (toDistribute == 0) return 0;
  if ((total / toDistribute) > lowOne) {
    lowOne = (u32)((total * 3) / (toDistribute * 2));
    for (u32 s = 0; s <= maxSV; s++)
      if (norm[s] == NOT_YET && count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; }
    toDistribute = (1u << tableLog) - distributed;
  }
  if (distributed == maxSV + 1) {
    u32 maxV = 0, maxC = 0;
    for (u32 s = 0; s <= maxSV; s++) if (count[s] > maxC) { maxV = s; maxC = count[s]; }
    norm[maxV] += (s16)toDistribute;
    return 0;
  }
  if (total == 0) {
    for (u32 s = 0; toDistribute > 0; s = (s + 1) % (maxSV + 1)) if (norm[s] > 0) { toDistribute--; norm[s]++; }
    return 0;
  }
  {
    u64 const vStepLog = 62 - tableLog;
    u64 const mid = (1ull << (vStepLog - 1)) - 1;
    u64 const rStep = (((1ull << vStepLog) * toDistribute) + mid) / (u32)total;
    u64 tmpTotal = mid;
    for (u32 s = 0; s <= maxSV; s++) {
      if (norm[s] == NOT_YET) {
        u64 const end = tmpTotal + (count[s] * rStep);
        u32 const sStart = (u32)(tmpTotal >> vStepLog);
        u32 const sEnd = (u32)(end >> vStepLog);
        u32 const weight = sEnd - sStart;
        if (weight < 1) return -1;
        norm[s] = (s16)weight;
        tmpTotal = end;
      }
    }
  }
  return 0;
}

/* FSE_normalizeCount(norm, tableLog, count, total, maxSymbolValue, useLowProbCount).
 * Returns tableLog, 0 for the RLE special case, -1 on error. */
int orc_fse_normalize(s16 *norm, u32 tableLog, const u32 *count, size_t total, u32 maxSV, int useLowProbCount) {
  static const u32 rtbTable[] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
  if (tableLog < FSE_MIN_TABLELOG || tableLog > FSE_MAX_TABLELOG) return -1;
  if (tableLog < fse_min_table_log(total, maxSV)) return -1;
  s16 const lowProbCount = useLowProbCount ? -1 : 1;
  u64 const scale = 62 - tableLog;
  u64 const step = (1ull << 62) / total;
  u64 const vStep = 1ull << (scale - 20);
  int stillToDistribute = 1 << tableLog;
  u32 largest = 0;
  s16 largestP = 0;
  u32 lowThreshold = (u32)(total >> tableLog);
  for (u32 s = 0; s <= maxSV; s++) {
    if (count[s] == total) return 0;
    if (count[s] == 0) { norm[s] = 0; continue; }
    if (count[s] <= lowThreshold) { norm[s] = lowProbCount; stillToDistribute--; }
    else {
      s16 proba = (s16)((count[s] * step) >> scale);
      if (proba < 8) {
        u64 restToBeat = vStep * rtbTable[proba];
        proba += (count[s] * step) - ((u64)proba << scale) > restToBeat;
      }
      if (proba > largestP) { largestP = proba; largest = s; }
      norm[s] = proba;
      stillToDistribute -= proba;
    }
  }
  if (-stillToDistribute >= (norm[largest] >> 1)) {
    if (fse_normalize_m2(norm, tableLog, count, total, maxSV, lowProbCount)) return -1;
  } else norm[largest] += (s16)stillToDistribute;
  return (int)tableLog;
}

/* FSE_writeNCount; returns size or 0 on error */
size_t orc_fse_write_ncount(u8 *out, size_t cap, const s16 *norm, u32 maxSV, u32 tableLog) {
  u8 *const ostart = out, *const oend = out + cap;
  int const tableSize = 1 << tableLog;
  int remaining = tableSize + 1, threshold = tableSize, nbBits = (int)tableLog + 1;
  u32 bitStream = 0;
  int bitCount = 0;
  u32 symbol = 0;
  u32 const alphabetSize = maxSV + 1;
  int previousIs0 = 0;
  bitStream += (tableLog - FSE_MIN_TABLELOG) << bitCount;
  bitCount += 4;
#define NC_FLUSH16()                                   \
  do {                                                 \
    if (out + 2 > oend) return 0;                      \
    out[0] = (u8)bitStream; out[1] = (u8)(bitStream >> 8); \
    out += 2; bitStream >>= 16;                        \
  } while (0)
  while (symbol < alphabetSize && remaining > 1) {
    if (previousIs0) {
      u32 start = symbol;
      while (symbol < alphabetSize && !norm[symbol]) symbol++;
      if (symbol == alphabetSize) break;
      while (symbol >= start + 24) { start += 24; bitStream += 0xFFFFu << bitCount; NC_FLUSH16(); }
      while (symbol >= start + 3) { start += 3; bitStream += 3u << bitCount; bitCount += 2; }
      bitStream += (symbol - start) << bitCount;
      bitCount += 2;
      if (bitCount > 16) { NC_FLUSH16(); bitCount -= 16; }
    }
    {
      int count = norm[symbol++];
      int const max = (2 * threshold - 1) - remaining;
      remaining -= count < 0 ? -count : count;
      count++;
      if (count >= threshold) count += max;
      bitStream += (u32)count << bitCount;
      bitCount += nbBits;
      bitCount -= (count < max);
      previousIs0 = (count == 1);
      if (remaining < 1) return 0;
      while (remaining < threshold) { nbBits--; threshold >>= 1; }
    }
    if (bitCount > 16) { NC_FLUSH16(); bitCount -= 16; }
  }
#undef NC_FLUSH16
  if (remaining != 1) return 0;
  if (out + 2 > oend) return 0;
  out[0] = (u8)bitStream;
  out[1] = (u8)(bitStream >> 8);
  out += (bitCount + 7) / 8;
  return (size_t)(out - ostart);
}

/* FSE compression table: stateTable + symbol transforms (FSE_buildCTable_wksp) */
typedef struct { int deltaFindState; u32 deltaNbBits; } fse_sym_t;
typedef struct { u32 tableLog; u16 stateTable[1 << FSE_MAX_TABLELOG]; fse_sym_t sym[256]; } fse_ctable_t;

int orc_fse_build_ctable(fse_ctable_t *ct, const s16 *norm, u32 maxSV, u32 tableLog) {
  u32 const tableSize = 1u << tableLog, tableMask = tableSize - 1;
  u32 const step = (tableSize >> 1) + (tableSize >> 3) + 3;
  u32 cumul[257];
  u8 tableSymbol[1 << FSE_MAX_TABLELOG];
  u32 highThreshold = tableSize - 1;
  ct->tableLog = tableLog;
  cumul[0] = 0;
  for (u32 u = 1; u <= maxSV + 1; u++) {
    if (norm[u - 1] == -1) { cumul[u] = cumul[u - 1] + 1; tableSymbol[highThreshold--] = (u8)(u - 1); }
    else cumul[u] = cumul[u - 1] + (u32)norm[u - 1];
  }
  cumul[maxSV + 1] = tableSize + 1;
  {
    u32 position = 0;
    for (u32 s = 0; s <= maxSV; s++) {
      for (int k = 0; k < norm[s]; k++) {
        tableSymbol[position] = (u8)s;
        position = (position + step) & tableMask;
        while (position > highThreshold) position = (position + step) & tableMask;
      }
    }
    if (position != 0) return -1;
  }
  for (u32 u = 0; u < tableSize; u++) { u8 s = tableSymbol[u]; ct->stateTable[cumul[s]++] = (u16)(tableSize + u); }
  {
    u32 total = 0;
    for (u32 s = 0; s <= maxSV; s++) {
      switch (norm[s]) {
      case 0: ct->sym[s].deltaNbBits = ((tableLog + 1) << 16) - (1u << tableLog); ct->sym[s].deltaFindState = 0; break;
      case -1:
      case 1: ct->sym[s].deltaNbBits = (tableLog << 16) - (1u << tableLog); ct->sym[s].deltaFindState = (int)total - 1; total++; break;
      default: {
        u32 const maxBitsOut = tableLog - highbit32((u32)norm[s] - 1);
        u32 const minStatePlus = (u32)norm[s] << maxBitsOut;
        ct->sym[s].deltaNbBits = (maxBitsOut << 16) - minStatePlus;
        ct->sym[s].deltaFindState = (int)total - norm[s];
        total += (u32)norm[s];
      }
      }
    }
  }
  return 0;
}

typedef struct { u32 value; const fse_ctable_t *ct; } fse_state_t;
static inline void fse_init_state2(fse_state_t *st, const fse_ctable_t *ct, u32 symbol) {
  fse_sym_t const tt = ct->sym[symbol];
  u32 nbBitsOut = (tt.deltaNbBits + (1u << 15)) >> 16;
  st->ct = ct;
  st->value = (nbBitsOut << 16) - tt.deltaNbBits;
  st->value = ct->stateTable[(st->value >> nbBitsOut) + tt.deltaFindState];
}
static inline void fse_encode(bitw_t *b, fse_state_t *st, u32 symbol) {
  fse_sym_t const tt = st->ct->sym[symbol];
  u32 const nbBitsOut = (st->value + tt.deltaNbBits) >> 16;
  bw_add(b, st->value, nbBitsOut);
  st->value = st->ct->stateTable[(st->value >> nbBitsOut) + tt.deltaFindState];
}
static inline void fse_flush_state(bitw_t *b, fse_state_t *st) { bw_add(b, st->value, st->ct->tableLog); }

/* ------------------------------------------------------------------------ */
/* Huffman (libzstd v1.4.9 huf_compress.c restated)                          */
/* ------------------------------------------------------------------------ */
#define HUF_TABLELOG_MAX 12
#define HUF_TABLELOG_DEFAULT 11
typedef struct { u16 val; u8 nbBits; } huf_celt_t;
typedef struct { u32 count; u16 parent; u8 byte; u8 nbBits; } huf_node_t;

static u32 huf_set_max_height(huf_node_t *huffNode, u32 lastNonNull, u32 maxNbBits) {
  u32 const largestBits = huffNode[lastNonNull].nbBits;
  if (largestBits <= maxNbBits) return largestBits;
  {
    int totalCost = 0;
    u32 const baseCost = 1u << (largestBits - maxNbBits);
    int n = (int)lastNonNull;
    while (huffNode[n].nbBits > maxNbBits) {
      totalCost += (int)(baseCost - (1u << (largestBits - huffNode[n].nbBits)));
      huffNode[n].nbBits = (u8)maxNbBits;
      n--;
    }
    while (huffNode[n].nbBits == maxNbBits) n--;
    totalCost >>= (largestBits - maxNbBits);
    {
      u32 const noSymbol = 0xF0F0F0F0;
      u32 rankLast[HUF_TABLELOG_MAX + 2];
      memset(rankLast, 0xF0, sizeof(rankLast));
      {
        u32 currentNbBits = maxNbBits;
        for (int pos = n; pos >= 0; pos--) {
          if (huffNode[pos].nbBits >= currentNbBits) continue;
          currentNbBits = huffNode[pos].nbBits;
          rankLast[maxNbBits - currentNbBits] = (u32)pos;
        }
      }
      while (totalCost > 0) {
        u32 nBitsToDecrease = highbit32((u32)totalCost) + 1;
        for (; nBitsToDecrease > 1; nBitsToDecrease--) {
          u32 const highPos = rankLast[nBitsToDecrease];
          u32 const lowPos = rankLast[nBitsToDecrease - 1];
          if (highPos == noSymbol) continue;
          if (lowPos == noSymbol) break;
          {
            u32 const highTotal = huffNode[highPos].count;
            u32 const lowTotal = 2 * huffNode[lowPos].count;
            if (highTotal <= lowTotal) break;
          }
        }
        while ((nBitsToDecrease <= HUF_TABLELOG_MAX) && (rankLast[nBitsToDecrease] == noSymbol)) nBitsToDecrease++;
        totalCost -= 1 << (nBitsToDecrease - 1);
        if (rankLast[nBitsToDecrease - 1] == noSymbol) rankLast[nBitsToDecrease - 1] = rankLast[nBitsToDecrease];
        huffNode[rankLast[nBitsToDecrease]].nbBits++;
        if (rankLast[nBitsToDecrease] == 0) rankLast[nBitsToDecrease] = noSymbol;
        else {
          rankLast[nBitsToDecrease]--;
          if (huffNode[rankLast[nBitsToDecrease]].nbBits != maxNbBits - nBitsToDecrease) rankLast[nBitsToDecrease] = noSymbol;
        }
      }
      while (totalCost < 0) {
        if (rankLast[1] == noSymbol) {
          while (huffNode[n].nbBits == maxNbBits) n--;
          huffNode[n + 1].nbBits--;
          rankLast[1] = (u32)(n + 1);
          totalCost++;
          continue;
        }
        huffNode[rankLast[1] + 1].nbBits--;
        rankLast[1]++;
        totalCost++;
      }
    }
  }
  return maxNbBits;
}

static void huf_sort(huf_node_t *huffNode, const u32 *count, u32 maxSV) {
  struct { u32 base, curr; } rankPosition[32];
  memset(rankPosition, 0, sizeof(rankPosition));
  for (u32 n = 0; n <= maxSV; n++) { u32 r = highbit32(count[n] + 1); rankPosition[r].base++; }
  for (u32 n = 30; n > 0; n--) rankPosition[n - 1].base += rankPosition[n].base;
  for (u32 n = 0; n < 32; n++) rankPosition[n].curr = rankPosition[n].base;
  for (u32 n = 0; n <= maxSV; n++) {
    u32 const c = count[n];
    u32 const r = highbit32(c + 1) + 1;
    u32 pos = rankPosition[r].curr++;
    while ((pos > rankPosition[r].base) && (c > huffNode[pos - 1].count)) { huffNode[pos] = huffNode[pos - 1]; pos--; }
    huffNode[pos].count = c;
    huffNode[pos].byte = (u8)n;
  }
}

/* HUF_buildCTable_wksp; returns maxNbBits actually used, 0 on error */
u32 orc_huf_build_ctable(huf_celt_t *tree, const u32 *count, u32 maxSV, u32 maxNbBits) {
  huf_node_t huffNode0[2 * 256 + 2];
  huf_node_t *const huffNode = huffNode0 + 1;
  int const STARTNODE = 256;
  int nonNullRank, lowS, lowN, nodeNb = STARTNODE, n, nodeRoot;
  if (maxNbBits == 0) maxNbBits = HUF_TABLELOG_DEFAULT;
  memset(huffNode0, 0, sizeof(huffNode0));
  huf_sort(huffNode, count, maxSV);
  nonNullRank = (int)maxSV;
  while (huffNode[nonNullRank].count == 0) nonNullRank--;
  lowS = nonNullRank; nodeRoot = nodeNb + lowS - 1; lowN = nodeNb;
  huffNode[nodeNb].count = huffNode[lowS].count + huffNode[lowS - 1].count;
  huffNode[lowS].parent = huffNode[lowS - 1].parent = (u16)nodeNb;
  nodeNb++; lowS -= 2;
  for (n = nodeNb; n <= nodeRoot; n++) huffNode[n].count = 1u << 30;
  huffNode0[0].count = 1u << 31;
  while (nodeNb <= nodeRoot) {
    int const n1 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
    int const n2 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
    huffNode[nodeNb].count = huffNode[n1].count + huffNode[n2].count;
    huffNode[n1].parent = huffNode[n2].parent = (u16)nodeNb;
    nodeNb++;
  }
  huffNode[nodeRoot].nbBits = 0;
  for (n = nodeRoot - 1; n >= STARTNODE; n--) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
  for (n = 0; n <= nonNullRank; n++) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
  maxNbBits = huf_set_max_height(huffNode, (u32)nonNullRank, maxNbBits);
  if (maxNbBits > HUF_TABLELOG_MAX) return 0;
  {
    u16 nbPerRank[HUF_TABLELOG_MAX + 1] = {0}, valPerRank[HUF_TABLELOG_MAX + 1] = {0};
    int const alphabetSize = (int)(maxSV + 1);
    for (n = 0; n <= nonNullRank; n++) nbPerRank[huffNode[n].nbBits]++;
    {
      u16 min = 0;
      for (n = (int)maxNbBits; n > 0; n--) { valPerRank[n] = min; min += nbPerRank[n]; min >>= 1; }
    }
    for (n = 0; n < alphabetSize; n++) tree[huffNode[n].byte].nbBits = huffNode[n].nbBits;
    for (n = 0; n < alphabetSize; n++) tree[n].val = valPerRank[tree[n].nbBits]++;
  }
  return maxNbBits;
}

/* FSE_compress_usingCTable (two interleaved states); returns 0 if not compressible */
static size_t fse_compress_using_ctable(u8 *dst, size_t cap, const u8 *src, size_t n, const fse_ctable_t *ct) {
  bitw_t b;
  fse_state_t s1, s2;
  const u8 *ip = src + n;
  if (n <= 2) return 0;
  bw_init(&b, dst, cap);
  if (n & 1) {
    fse_init_state2(&s1, ct, *--ip);
    fse_init_state2(&s2, ct, *--ip);
    fse_encode(&b, &s1, *--ip);
  } else {
    fse_init_state2(&s2, ct, *--ip);
    fse_init_state2(&s1, ct, *--ip);
  }
  while (ip > src) {
    fse_encode(&b, &s2, *--ip);
    fse_encode(&b, &s1, *--ip);
  }
  fse_flush_state(&b, &s2);
  fse_flush_state(&b, &s1);
  return bw_close(&b);
}

/* HUF_compressWeights */
static size_t huf_compress_weights(u8 *dst, size_t cap, const u8 *w, size_t wtSize) {
  u32 maxSV = HUF_TABLELOG_MAX, count[HUF_TABLELOG_MAX + 1];
  s16 norm[HUF_TABLELOG_MAX + 1];
  fse_ctable_t ct;
  u8 *op = dst;
  if (wtSize <= 1) return 0;
  {
    u32 maxCount = 0;
    memset(count, 0, sizeof(count));
    for (size_t i = 0; i < wtSize; i++) count[w[i]]++;
    while (!count[maxSV]) maxSV--;
    for (u32 s = 0; s <= maxSV; s++) if (count[s] > maxCount) maxCount = count[s];
    if (maxCount == wtSize) return 1;
    if (maxCount == 1) return 0;
  }
  {
    u32 tableLog = orc_fse_optimal_table_log(6, wtSize, maxSV);
    if (orc_fse_normalize(norm, tableLog, count, wtSize, maxSV, 0) < 0) return 0;
    size_t h = orc_fse_write_ncount(op, cap, norm, maxSV, tableLog);
    if (!h) return 0;
    op += h;
    orc_fse_build_ctable(&ct, norm, maxSV, tableLog);
    size_t c = fse_compress_using_ctable(op, (size_t)(dst + cap - op), w, wtSize, &ct);
    if (c == 0) return 0;
    op += c;
  }
  return (size_t)(op - dst);
}

/* HUF_writeCTable; returns header size or 0 on error */
size_t orc_huf_write_ctable(u8 *dst, size_t cap, const huf_celt_t *tree, u32 maxSV, u32 huffLog) {
  u8 bitsToWeight[HUF_TABLELOG_MAX + 1], w[256];
  memset(w, 0, sizeof(w));
  bitsToWeight[0] = 0;
  for (u32 n = 1; n < huffLog + 1; n++) bitsToWeight[n] = (u8)(huffLog + 1 - n);
  for (u32 n = 0; n < maxSV; n++) w[n] = bitsToWeight[tree[n].nbBits];
  {
    size_t h = huf_compress_weights(dst + 1, cap - 1, w, maxSV);
    if ((h > 1) & (h < maxSV / 2)) { dst[0] = (u8)h; return h + 1; }
  }
  if (maxSV > (256 - 128)) return 0;
  if (((maxSV + 1) / 2) + 1 > cap) return 0;
  dst[0] = (u8)(128 + (maxSV - 1));
  w[maxSV] = 0;
  for (u32 n = 0; n < maxSV; n += 2) dst[(n / 2) + 1] = (u8)((w[n] << 4) + w[n + 1]);
  return ((maxSV + 1) / 2) + 1;
}

static size_t huf_compress1x(u8 *dst, size_t cap, const u8 *src, size_t n, const huf_celt_t *ct) {
  bitw_t b;
  bw_init(&b, dst, cap);
  for (size_t i = n; i > 0; i--) bw_add(&b, ct[src[i - 1]].val, ct[src[i - 1]].nbBits);
  return bw_close(&b);
}
static size_t huf_compress4x(u8 *dst, size_t cap, const u8 *src, size_t n, const huf_celt_t *ct) {
  size_t const seg = (n + 3) / 4;
  u8 *op = dst + 6;
  if (cap < 6 + 1 + 1 + 1 + 8) return 0;
  if (n < 12) return 0;
  for (int k = 0; k < 4; k++) {
    size_t len = k < 3 ? seg : n - 3 * seg;
    size_t c = huf_compress1x(op, (size_t)(dst + cap - op), src + k * seg, len, ct);
    if (c == 0) return 0;
    if (k < 3) { dst[2 * k] = (u8)c; dst[2 * k + 1] = (u8)(c >> 8); }
    op += c;
  }
  return (size_t)(op - dst);
}

/* ZSTD_compressLiterals (no previous table). Returns section size. */
size_t orc_compress_literals(u8 *dst, size_t cap, const u8 *src, size_t n) {
  size_t const minGain = (n >> 6) + 2;
  size_t const lhSize = 3 + (n >= 1024) + (n >= 16384);
  int singleStream = n < 256;
  size_t cLitSize = 0;
  if (n > ZH_COMPRESS_LITERALS_SIZE_MIN) {
    /* HUF_compress_internal */
    u32 count[256], maxSV = 255, largest = 0;
    memset(count, 0, sizeof(count));
    for (size_t i = 0; i < n; i++) count[src[i]]++;
    while (!count[maxSV]) maxSV--;
    for (u32 s = 0; s <= maxSV; s++) if (count[s] > largest) largest = count[s];
    if (largest == n) cLitSize = 1;
    else if (largest <= (n >> 7) + 4) cLitSize = 0;
    else {
      huf_celt_t tree[256];
      u8 *op = dst + lhSize;
      u8 *const oend = dst + cap;
      memset(tree, 0, sizeof(tree));
      u32 huffLog = fse_optimal_table_log_internal(HUF_TABLELOG_DEFAULT, n, maxSV, 1);
      huffLog = orc_huf_build_ctable(tree, count, maxSV, huffLog);
      size_t h = huffLog ? orc_huf_write_ctable(op, (size_t)(oend - op), tree, maxSV, huffLog) : 0;
      if (h && h + 12 < n) {
        op += h;
        size_t c = singleStream ? huf_compress1x(op, (size_t)(oend - op), src, n, tree) : huf_compress4x(op, (size_t)(oend - op), src, n, tree);
        if (c) { op += c; cLitSize = (size_t)(op - (dst + lhSize)); if (cLitSize >= n - 1) cLitSize = 0; }
      }
    }
  }
  if (cLitSize == 0 || cLitSize >= n - minGain) {
    /* ZSTD_noCompressLiterals */
    size_t const fl = 1 + (n > 31) + (n > 4095);
    if (n + fl > cap) return 0;
    switch (fl) {
    case 1: dst[0] = (u8)(0 + (n << 3)); break;
    case 2: { u32 v = (u32)(0 + (1 << 2) + (n << 4)); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); break; }
    default: { u32 v = (u32)(0 + (3 << 2) + (n << 4)); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); }
    }
    memcpy(dst + fl, src, n);
    return n + fl;
  }
  if (cLitSize == 1) {
    /* ZSTD_compressRleLiteralsBlock */
    size_t const fl = 1 + (n > 31) + (n > 4095);
    switch (fl) {
    case 1: dst[0] = (u8)(1 + (n << 3)); break;
    case 2: { u32 v = (u32)(1 + (1 << 2) + (n << 4)); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); break; }
    default: { u32 v = (u32)(1 + (3 << 2) + (n << 4)); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); }
    }
    dst[fl] = src[0];
    return fl + 1;
  }
  {
    u32 const hType = 2; /* set_compressed */
    switch (lhSize) {
    case 3: { u32 lhc = hType + ((u32)(!singleStream) << 2) + ((u32)n << 4) + ((u32)cLitSize << 14);
              dst[0] = (u8)lhc; dst[1] = (u8)(lhc >> 8); dst[2] = (u8)(lhc >> 16); break; }
    case 4: { u32 lhc = hType + (2 << 2) + ((u32)n << 4) + ((u32)cLitSize << 18);
              dst[0] = (u8)lhc; dst[1] = (u8)(lhc >> 8); dst[2] = (u8)(lhc >> 16); dst[3] = (u8)(lhc >> 24); break; }
    default: { u32 lhc = hType + (3 << 2) + ((u32)n << 4) + ((u32)cLitSize << 22);
               dst[0] = (u8)lhc; dst[1] = (u8)(lhc >> 8); dst[2] = (u8)(lhc >> 16); dst[3] = (u8)(lhc >> 24); dst[4] = (u8)(cLitSize >> 10); }
    }
    return lhSize + cLitSize;
  }
}

/* ------------------------------------------------------------------------ */
/* Sequences section                                                        */
/* ------------------------------------------------------------------------ */
/* one raw sequence: literal length, match length, match offset (distance) */
typedef struct { u32 ll, ml, off; } orc_seq_t;

enum { SET_BASIC = 0, SET_RLE = 1, SET_COMPRESSED = 2 };

static int select_encoding_type(const u32 *count, u32 max, size_t mostFrequent, size_t nbSeq, u32 defaultNormLog, int defaultAllowed) {
  if (mostFrequent == nbSeq) {
    if (defaultAllowed && nbSeq <= 2) return SET_BASIC;
    return SET_RLE;
  }
  /* strategy < ZSTD_lazy branch, strategy = dfast (2): mult = 8, baseLog = 3 */
  if (defaultAllowed) {
    size_t const dynamicFse_nbSeq_min = (((size_t)1 << defaultNormLog) * 8) >> 3;
    if ((nbSeq < dynamicFse_nbSeq_min) || (mostFrequent < (nbSeq >> (defaultNormLog - 1)))) return SET_BASIC;
  }
  (void)count; (void)max;
  return SET_COMPRESSED;
}

/* ZSTD_buildCTable; returns header bytes written or (size_t)-1 on error */
static size_t build_ctable(u8 *dst, size_t cap, fse_ctable_t *ct, u32 fseLog, int type, u32 *count, u32 max,
                           const u8 *codeTable, size_t nbSeq, const s16 *defNorm, u32 defNormLog, u32 defMax) {
  switch (type) {
  case SET_RLE: {
    /* FSE_buildCTable_rle: tableLog 0, single state */
    ct->tableLog = 0;
    ct->stateTable[0] = 0; ct->stateTable[1] = 0;
    memset(ct->sym, 0, sizeof(ct->sym));
    ct->sym[codeTable[0]].deltaNbBits = 0; ct->sym[codeTable[0]].deltaFindState = 0;
    if (!cap) return (size_t)-1;
    dst[0] = codeTable[0];
    return 1;
  }
  case SET_BASIC:
    orc_fse_build_ctable(ct, defNorm, defMax, defNormLog);
    return 0;
  default: {
    s16 norm[53];
    size_t nbSeq_1 = nbSeq;
    u32 const tableLog = orc_fse_optimal_table_log(fseLog, nbSeq, max);
    if (count[codeTable[nbSeq - 1]] > 1) { count[codeTable[nbSeq - 1]]--; nbSeq_1--; }
    if (orc_fse_normalize(norm, tableLog, count, nbSeq_1, max, nbSeq_1 >= 2048) < 0) return (size_t)-1;
    size_t h = orc_fse_write_ncount(dst, cap, norm, max, tableLog);
    if (!h) return (size_t)-1;
    orc_fse_build_ctable(ct, norm, max, tableLog);
    return h;
  }
  }
}

/* Encode a sequences section from (already repcode-resolved) codes.
 * Returns size or (size_t)-1. */
static size_t encode_sequences_section(u8 *dst, size_t cap, const u32 *llv, const u32 *mlb, const u32 *ofb, size_t nbSeq) {
  u8 *op = dst, *const oend = dst + cap;
  if (cap < 4) return (size_t)-1;
  if (nbSeq < 128) *op++ = (u8)nbSeq;
  else if (nbSeq < ZH_LONGNBSEQ) { op[0] = (u8)((nbSeq >> 8) + 0x80); op[1] = (u8)nbSeq; op += 2; }
  else { op[0] = 0xFF; op[1] = (u8)(nbSeq - ZH_LONGNBSEQ); op[2] = (u8)((nbSeq - ZH_LONGNBSEQ) >> 8); op += 3; }
  if (nbSeq == 0) return (size_t)(op - dst);
  u8 *llC = malloc(nbSeq), *mlC = malloc(nbSeq), *ofC = malloc(nbSeq);
  for (size_t i = 0; i < nbSeq; i++) { llC[i] = (u8)ll_code(llv[i]); mlC[i] = (u8)ml_code(mlb[i]); ofC[i] = (u8)highbit32(ofb[i]); }
  u8 *seqHead = op++;
  fse_ctable_t ctLL, ctOF, ctML;
  u32 count[53];
  int types[3];
  const u8 *codes[3] = {llC, ofC, mlC};
  fse_ctable_t *cts[3] = {&ctLL, &ctOF, &ctML};
  u32 const maxSym[3] = {35, 31, 52}, fseLogs[3] = {9, 8, 9}, defLogs[3] = {6, 5, 6}, defMax[3] = {35, 28, 52};
  const s16 *defNorms[3] = {LL_defNorm, OF_defNorm, ML_defNorm};
  for (int t = 0; t < 3; t++) {
    u32 max = maxSym[t];
    size_t mostFrequent = 0;
    memset(count, 0, sizeof(count));
    for (size_t i = 0; i < nbSeq; i++) count[codes[t][i]]++;
    while (max && !count[max]) max--;
    for (u32 s = 0; s <= max; s++) if (count[s] > mostFrequent) mostFrequent = count[s];
    int defaultAllowed = (t == 1) ? (max <= 28) : 1;
    types[t] = select_encoding_type(count, max, mostFrequent, nbSeq, defLogs[t], defaultAllowed);
    size_t h = build_ctable(op, (size_t)(oend - op), cts[t], fseLogs[t], types[t], count, max, codes[t], nbSeq, defNorms[t], defLogs[t], defMax[t]);
    if (h == (size_t)-1) { free(llC); free(mlC); free(ofC); return (size_t)-1; }
    op += h;
  }
  *seqHead = (u8)((types[0] << 6) + (types[1] << 4) + (types[2] << 2));
  {
    /* ZSTD_encodeSequences */
    bitw_t b;
    fse_state_t sML, sOF, sLL;
    size_t n = nbSeq - 1;
    bw_init(&b, op, (size_t)(oend - op));
    fse_init_state2(&sML, &ctML, mlC[n]);
    fse_init_state2(&sOF, &ctOF, ofC[n]);
    fse_init_state2(&sLL, &ctLL, llC[n]);
    bw_add(&b, llv[n], LL_bits[llC[n]]);
    bw_add(&b, mlb[n], ML_bits[mlC[n]]);
    bw_add(&b, ofb[n], ofC[n]);
    for (n = nbSeq - 1; n-- > 0;) {
      fse_encode(&b, &sOF, ofC[n]);
      fse_encode(&b, &sML, mlC[n]);
      fse_encode(&b, &sLL, llC[n]);
      bw_add(&b, llv[n], LL_bits[llC[n]]);
      bw_add(&b, mlb[n], ML_bits[mlC[n]]);
      bw_add(&b, ofb[n], ofC[n]);
    }
    fse_flush_state(&b, &sML);
    fse_flush_state(&b, &sOF);
    fse_flush_state(&b, &sLL);
    size_t s = bw_close(&b);
    free(llC); free(mlC); free(ofC);
    if (!s) return (size_t)-1;
    op += s;
  }
  return (size_t)(op - dst);
}

/* Repcode resolution (encoder side of RFC 8878 §3.1.2.5).  rep[] entries of 0
 * are "unknown" (inherited from an earlier block compressed independently) and
 * are never referenced.  Produces offBase (Offset_Value) per sequence. */
void orc_resolve_repcodes(const orc_seq_t *seq, size_t nbSeq, u32 rep_in[3], u32 *offBase) {
  u32 r0 = rep_in[0], r1 = rep_in[1], r2 = rep_in[2];
  for (size_t i = 0; i < nbSeq; i++) {
    u32 o = seq[i].off, ll0 = seq[i].ll == 0, ob;
    if (!ll0) ob = (o == r0 && r0) ? 1 : (o == r1 && r1) ? 2 : (o == r2 && r2) ? 3 : o + 3;
    else ob = (o == r1 && r1) ? 1 : (o == r2 && r2) ? 2 : (r0 > 1 && o == r0 - 1) ? 3 : o + 3;
    offBase[i] = ob;
    /* decoder update */
    if (ob > 3) { r2 = r1; r1 = r0; r0 = o; }
    else {
      u32 idx = ob - 1 + ll0; /* 0: rep0, 1: rep1, 2: rep2, 3: rep0-1 */
      if (idx == 0) {}
      else if (idx == 1) { u32 t = r1; r1 = r0; r0 = t; }
      else if (idx == 2) { u32 t = r2; r2 = r1; r1 = r0; r0 = t; }
      else { r2 = r1; r1 = r0; r0 = o; }
    }
  }
  rep_in[0] = r0; rep_in[1] = r1; rep_in[2] = r2;
}

/* Build a compressed block body (literals + sequences sections) from raw
 * sequences.  Returns body size, or 0 if the caller should emit a raw block
 * (body >= n - minGain), or (size_t)-1 on error. */
size_t orc_encode_block_body(u8 *dst, size_t cap, const u8 *src, size_t n, const orc_seq_t *seq, size_t nbSeq, u32 rep[3]) {
  u8 *lits = malloc(n + 1);
  u32 *llv = malloc(sizeof(u32) * (nbSeq + 1)), *mlb = malloc(sizeof(u32) * (nbSeq + 1)), *ofb = malloc(sizeof(u32) * (nbSeq + 1));
  size_t nl = 0, pos = 0;
  for (size_t i = 0; i < nbSeq; i++) {
    memcpy(lits + nl, src + pos, seq[i].ll); nl += seq[i].ll;
    pos += seq[i].ll + seq[i].ml;
    llv[i] = seq[i].ll; mlb[i] = seq[i].ml - 3;
  }
  memcpy(lits + nl, src + pos, n - pos); nl += n - pos;
  orc_resolve_repcodes(seq, nbSeq, rep, ofb);
  size_t r = (size_t)-1;
  size_t ls = orc_compress_literals(dst, cap, lits, nl);
  if (ls) {
    size_t ss = encode_sequences_section(dst + ls, cap - ls, llv, mlb, ofb, nbSeq);
    if (ss != (size_t)-1) {
      size_t const minGain = (n >> 6) + 2;
      size_t const maxC = n > minGain ? n - minGain : 0;
      r = (ls + ss >= maxC) ? 0 : ls + ss;
    } else if (n <= cap) r = 0; /* dstSize_tooSmall & srcSize <= capacity -> raw */
  }
  free(lits); free(llv); free(mlb); free(ofb);
  return r;
}

/* ------------------------------------------------------------------------ */
/* LZ stage (deterministic tile-lagged dual hash, lazy-1 greedy parse)       */
/* ------------------------------------------------------------------------ */
static inline u64 rd64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }
/* hashes of include/zstd_hip_params.h (24 x 24-bit products, low 32 bits, top bits) */
static inline u32 mul24(u32 a, u32 b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
static inline u32 zh_hash_long(u64 v) {
  u32 const t = mul24((u32)v, ZH_HK_L0) + mul24((u32)(v >> 24), ZH_HK_L1) + mul24((u32)(v >> 48), ZH_HK_L2);
  return t >> (32 - ZH_HASH_LOG_LONG);
}
static inline u32 zh_hash_short(u64 v) {
  u32 const t = mul24((u32)v, ZH_HK_S0) + mul24((u32)(v >> 24) & 0xFFFFu, ZH_HK_S1);
  return t >> (32 - ZH_HASH_LOG_SHORT);
}

static u32 common_prefix(const u8 *src, u32 a, u32 b, u32 n, u32 cap) {
  u32 l = 0;
  while (l < cap && a + l < n && src[a + l] == src[b + l]) l++;
  return l;
}

/* Per-position best match over the tiles [t0, t1) of src[0, n) (tile-aligned, t1 <= lim):
 * len[p] (0 or >= ZH_MIN_MATCH_*), off[p].  Each tile's lookups see the tables after every
 * earlier tile's insertions (K1's inserter waves: zh_lz.hip insert_window).  `skip_from`:
 * tiles at or above it are neither looked up nor inserted (len 0), see orc_lz_parse_pre. */
/* per thread: oracle frames may run on a thread pool (test_c5_full_workload_vs_oracle's pattern) */
static _Thread_local u32 g_TL[1 << ZH_HASH_LOG_LONG], g_TS[1 << ZH_HASH_LOG_SHORT];
/* K1's parse mode of the level (ZH_K1_MODE): 0 = both tables, lazy-1 check (levels 3-4);
 * 1 = the short (5-byte) table only, lazy-1 (level 2); 2 = the short table only, greedy (level 1).
 * Set by orc_compress_frame_lv. */
static _Thread_local int orc_lz_mode = 0; /* per thread: callers may run frames on a thread pool */
static void match_info_tiles(const u8 *src, u32 n, u32 t0, u32 t1, u32 skip_from, u8 *len, u16 *off) {
  const u32 EMPTY = 0xFFFFFFFFu;
  u32 const lim = n - ZH_HASH_READ;
  for (u32 t = t0; t < t1 && t < skip_from; t += ZH_TILE) {
    u32 e = t + ZH_TILE < lim ? t + ZH_TILE : lim;
    for (u32 p = t; p < e; p++) {
      u64 v = rd64(src + p);
      u32 qL = g_TL[zh_hash_long(v)], qS = g_TS[zh_hash_short(v)];
      u32 lL = (qL != EMPTY && orc_lz_mode == 0) ? common_prefix(src, p, qL, n, ZH_MAX_MATCH) : 0;
      u32 lS = qS != EMPTY ? common_prefix(src, p, qS, n, ZH_MAX_MATCH) : 0;
      if (lL < ZH_MIN_MATCH_LONG) lL = 0;
      if (lS < ZH_MIN_MATCH_SHORT) lS = 0;
      if (lL && lL >= lS) { len[p] = (u8)lL; off[p] = (u16)(p - qL); }
      else if (lS) { len[p] = (u8)lS; off[p] = (u16)(p - qS); }
    }
    for (u32 p = t; p < e; p++) { u64 v = rd64(src + p); g_TL[zh_hash_long(v)] = p; g_TS[zh_hash_short(v)] = p; }
  }
}
static void match_info_reset(u32 n, u8 *len, u16 *off) {
  for (u32 i = 0; i < (1u << ZH_HASH_LOG_LONG); i++) g_TL[i] = 0xFFFFFFFFu;
  for (u32 i = 0; i < (1u << ZH_HASH_LOG_SHORT); i++) g_TS[i] = 0xFFFFFFFFu;
  memset(len, 0, n + 1);
  memset(off, 0, sizeof(u16) * (n + 1));
}

/* Per-position best match of every tile (no skipping). Arrays sized n+1. */
void orc_lz_match_info(const u8 *src, u32 n, u8 *len, u16 *off) {
  match_info_reset(n, len, off);
  if (n <= ZH_HASH_READ) return;
  u32 const lim = n - ZH_HASH_READ;
  match_info_tiles(src, n, 0, (lim + ZH_TILE - 1) / ZH_TILE * ZH_TILE, 0xFFFFFFFFu, len, off);
}

/* Parse + merge over src[0, n).  Positions [0, pre) are dictionary history:
 * hashed and matched against like any other, but the parse starts at pre.
 * Returns number of sequences; *last_lits = trailing literals. */
/* Parse strategy: 0 = greedy with a one-position lazy check (levels < 9); 1 = LAZY2 (levels
 * >= 9; the reference maps level 9 to LAZY, src/cuda_zstd_types.cpp:172-182):
 * libzstd ZSTD_compressBlock_lazy_generic's depth-2 rule on this matcher's candidates -- the
 * match at p is deferred when the match at p+1 gains more than 4, or the one at p+2 more than 7,
 * with gain = 4 x length - bit length of (offset + 1).  Set by orc_compress_frame_lv. */
static _Thread_local int orc_parse_lazy2 = 0;
static _Thread_local int orc_parse_level = 3; /* levels >= ZH_DEEP_LEVEL: the deep matcher (orc_lz_parse_deep) */
static int match_gain(const u8 *len, const u16 *off, u32 p) {
  return len[p] ? 4 * (int)len[p] - (31 - __builtin_clz((u32)off[p] + 1u)) : -1000;
}
static int match_gain32(const u8 *len, const u32 *off, u32 p) {
  return len[p] ? 4 * (int)len[p] - (31 - __builtin_clz(off[p] + 1u)) : -1000;
}

/* Deep matcher (levels >= ZH_DEEP_LEVEL; the reference's level table gives level 9
 * a 32-candidate chain search, src/cuda_zstd_types.cpp:172-183, walked per position by
 * find_matches_kernel, src/lz77_parallel.cu:26-70, whose atomicExch chain insert makes it
 * nondeterministic).  Deterministic restatement, what zh_lz_deep_kernel computes:
 *   - exact hash chains over the whole staged buffer buf[0, n) (history/dictionary prefix
 *     [0, pre) + block): prev[p] = the latest q < p with the same 5-byte short hash, positions
 *     [0, lim) with lim = n - ZH_HASH_READ;
 *   - per block position p in [pre, lim): the first `depth` chain candidates at offsets up to
 *     ZH_DEEP_MAXOFF (the walk ends at the first one further away), each's common
 *     prefix with p (capped at ZH_MAX_MATCH and at n); the longest with >= ZH_MIN_MATCH_SHORT
 *     bytes wins, the nearest on ties; the walk stops early at a capped match;
 *   - LAZY2 parse from pre (libzstd ZSTD_compressBlock_lazy_generic's depth-2 rule, as
 *     orc_lz_parse_pre), no catch-up, a directly following same-offset match merged. */
size_t orc_lz_parse_deep(const u8 *buf, u32 pre, u32 n, u32 depth, orc_seq_t *seq, u32 *last_lits) {
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 *prev = malloc(sizeof(u32) * (lim + 1));
  u32 *head = calloc((size_t)1 << ZH_HASH_LOG_SHORT, sizeof(u32));
  u8 *len = calloc(n + 3, 1);
  u32 *off = calloc(n + 3, sizeof(u32));
  for (u32 p = 0; p < lim; p++) {
    u32 const h = zh_hash_short(rd64(buf + p));
    prev[p] = head[h]; /* q + 1, 0 = none */
    head[h] = p + 1;
  }
  for (u32 p = pre; p < lim; p++) {
    u32 best = 0, bo = 0, c = prev[p];
    for (u32 d = 0; d < depth && c && p - (c - 1) <= ZH_DEEP_MAXOFF; d++) {
      u32 const q = c - 1, l = common_prefix(buf, p, q, n, ZH_MAX_MATCH);
      if (l >= ZH_MIN_MATCH_SHORT && l > best) {
        best = l;
        bo = p - q;
        if (best >= ZH_MAX_MATCH) break;
      }
      c = prev[q];
    }
    len[p] = (u8)best;
    off[p] = bo;
  }
  size_t ns = 0;
  u32 p = pre, anchor = pre;
  while (p < lim) {
    if (len[p] == 0) { p++; continue; }
    int const g0 = match_gain32(len, off, p);
    if (match_gain32(len, off, p + 1) > g0 + 4 || match_gain32(len, off, p + 2) > g0 + 7) { p++; continue; }
    u32 const ll = p - anchor, of = off[p];
    if (ns && ll == 0 && seq[ns - 1].off == of) seq[ns - 1].ml += len[p];
    else { seq[ns].ll = ll; seq[ns].ml = len[p]; seq[ns].off = of; ns++; }
    p += len[p];
    anchor = p;
  }
  *last_lits = n - anchor;
  free(prev); free(head); free(len); free(off);
  return ns;
}
/* Miss skip (libzstd dfast's kSearchStrength idea at window granularity): the matcher and the
 * parse run window by window (ZH_WINDOW positions, aligned in the staged buffer, as K1's
 * pipeline does), and a window whose window three before it -- the newest one K1's parse has
 * finished when its insertion starts -- took no match (counted at the match position before
 * catch-up) searches and inserts only its first ZH_SKIP_TILES tiles; the rest of it has no
 * candidates.  Windows up to three past the one holding `pre` never skip. */
/* Repeat scan (ZH_SCAN_*, include/zstd_hip_params.h; K1 zh_lz.hip repeat_scan): the number of
 * sampled block positions p = pre + ZH_SCAN_STEP m < lim whose 8 bytes repeat an earlier sampled position, as seen
 * through a 2^ZH_SCAN_LOG-slot table of min(sig16 << 16 | q) over q = 0 mod ZH_SCAN_STRIDE in
 * [0, lim) -- slot and sig16 from the long hash's sum (top 14 bits, the 16 below them). */
static inline u32 scan_sum(u64 v) {
  return mul24((u32)v, ZH_HK_L0) + mul24((u32)(v >> 24), ZH_HK_L1) + mul24((u32)(v >> 48), ZH_HK_L2);
}
u32 orc_repeat_scan(const u8 *src, u32 pre, u32 n) {
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 *E = malloc(sizeof(u32) << ZH_SCAN_LOG);
  memset(E, 0xFF, sizeof(u32) << ZH_SCAN_LOG);
  for (u32 q = 0; q < lim; q += ZH_SCAN_STRIDE) {
    u32 const t = scan_sum(rd64(src + q)), s = t >> (32 - ZH_SCAN_LOG), e = ((t << ZH_SCAN_LOG) & 0xFFFF0000u) | q;
    if (e < E[s]) E[s] = e;
  }
  u32 c = 0;
  for (u32 p = pre; p < lim; p += ZH_SCAN_STEP) {
    u32 const t = scan_sum(rd64(src + p)), s = t >> (32 - ZH_SCAN_LOG);
    c += E[s] - ((t << ZH_SCAN_LOG) & 0xFFFF0000u) < p;
  }
  free(E);
  return c;
}
static int repeat_scan_alive(const u8 *src, u32 pre, u32 n) {
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 const need = lim > pre ? (lim - pre) >> ZH_SCAN_SHIFT : 0;
  return orc_repeat_scan(src, pre, n) >= (need > ZH_SCAN_MIN ? need : ZH_SCAN_MIN);
}

size_t orc_lz_parse_pre(const u8 *src, u32 pre, u32 n, orc_seq_t *seq, u32 *last_lits) {
  if (orc_parse_level >= ZH_DEEP_LEVEL) return orc_lz_parse_deep(src, pre, n, ZH_DEEP_DEPTH(orc_parse_level), seq, last_lits);
  u8 *len = malloc(n + 2);
  u16 *off = malloc(sizeof(u16) * (n + 2));
  match_info_reset(n, len, off);
  len[n + 1] = 0; off[n + 1] = 0;
  size_t ns = 0;
  u32 p = pre, anchor = pre, lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 const nwin = (lim + ZH_WINDOW - 1) / ZH_WINDOW, a0 = pre / ZH_WINDOW;
  u32 *mcount = calloc(nwin + 1, sizeof(u32));
  for (u32 a = 0; a <= nwin; a++) {
    if (a < nwin) {
      u32 const t0 = a * ZH_WINDOW, t1 = (a + 1) * ZH_WINDOW;
      int const skip = a >= a0 + 3 && mcount[a - 3] == 0;
      if (skip) {
        /* a miss-skip window searches its first ZH_SKIP_TILES tiles; a match among them (any
         * position with a candidate of at least the minimum length) resumes the search of the
         * rest of the window, as if it had not skipped (K1: the inserter waves check their
         * candidates after the first batch of tiles) */
        u32 const ts = t0 + ZH_SKIP_TILES * ZH_TILE;
        match_info_tiles(src, n, t0, ts, 0xFFFFFFFFu, len, off);
        int hit = 0;
        for (u32 q = t0; q < ts && q < lim; q++) hit |= len[q] != 0;
        if (hit) match_info_tiles(src, n, ts, t1, 0xFFFFFFFFu, len, off);
      } else {
        match_info_tiles(src, n, t0, t1, 0xFFFFFFFFu, len, off);
      }
    }
    /* incompressibility probe: once the parse of the probe windows [a0, a0 + ZH_PROBE_WINDOWS)
     * is done (in the iteration after the one that inserted window a0 + ZH_PROBE_WINDOWS) and
     * it took no match there, and the repeat scan of the whole block finds (almost) no repeated
     * 8-byte string, the block takes no sequences at all -- the whole block is literals (K1
     * stops; K2 reads them from the source, orc_compress_block_pre).  Otherwise the parse goes
     * on as if there were no probe (K1 restarts the block without it).  Blocks whose `pre` lies
     * past ZH_PROBE_MAX_E0 in its window are not probed. */
    if (a == a0 + ZH_PROBE_WINDOWS + 1 && a <= nwin && pre - a0 * ZH_WINDOW <= ZH_PROBE_MAX_E0) {
      u32 m = 0;
      for (u32 j = a0; j < a0 + ZH_PROBE_WINDOWS; j++) m += mcount[j];
      if (m == 0 && !repeat_scan_alive(src, pre, n)) {
        ns = 0;
        anchor = pre;
        break;
      }
    }
    /* the parse of every window before a (its lookahead p + 1, p + 2 is in window a's first tile) */
    u32 const pe = a < nwin ? a * ZH_WINDOW : lim;
    while (p < lim && p < pe) {
      int defer;
      /* level 1 (mode 2) looks matches up at positions p = 0 mod ZH_L1_STRIDE only (K1
       * span_lengths_l1); the skip windows' resume check above still sees every position's
       * candidate, as K1's inserter waves do */
      if (len[p] == 0 || (orc_lz_mode == 2 && p % ZH_L1_STRIDE)) defer = 1;
      else if (orc_parse_lazy2) {
        int const g0 = match_gain(len, off, p);
        defer = match_gain(len, off, p + 1) > g0 + 4 || match_gain(len, off, p + 2) > g0 + 7;
      } else defer = orc_lz_mode != 2 && len[p + 1] > len[p];
      if (defer) { p++; continue; }
      /* catch-up (libzstd 1.4.9 ZSTD_compressBlock_doubleFast_generic / lazy_generic "catch
       * up"): the match grows backwards over the literals since the last sequence while the
       * bytes before it equal the bytes before its source, bounded by the start of the
       * ZH_WINDOW-position parse window holding p (the device parses window by window; windows
       * start at multiples of ZH_WINDOW of the staged buffer).  The parse itself continues at
       * p + len[p] either way. */
      mcount[p / ZH_WINDOW]++;
      u32 ms = p, ml = len[p];
      u32 const of = off[p], wlo = p & ~(u32)(ZH_WINDOW - 1), lo = anchor > wlo ? anchor : wlo;
      while (ms > lo && ms > of && src[ms - 1] == src[ms - 1 - of]) { ms--; ml++; }
      u32 ll = ms - anchor;
      if (ns && ll == 0 && seq[ns - 1].off == of) seq[ns - 1].ml += ml; /* continuation merge */
      else { seq[ns].ll = ll; seq[ns].ml = ml; seq[ns].off = of; ns++; }
      p += len[p];
      anchor = p;
    }
  }
  *last_lits = n - anchor;
  free(len); free(off); free(mcount);
  return ns;
}
size_t orc_lz_parse(const u8 *src, u32 n, orc_seq_t *seq, u32 *last_lits) { return orc_lz_parse_pre(src, 0, n, seq, last_lits); }

/* ------------------------------------------------------------------------ */
/* Block + frame                                                            */
/* ------------------------------------------------------------------------ */
static int is_rle(const u8 *src, size_t n) {
  for (size_t i = 1; i < n; i++) if (src[i] != src[0]) return 0;
  return 1;
}

/* Compress one block (<= ZH_BLOCK_MAX) with its block header.  rep[] in/out.
 * Returns bytes written or 0 on insufficient capacity. */
size_t orc_compress_block_pre(u8 *dst, size_t cap, const u8 *buf, u32 pre, u32 n, int last, u32 rep[3]) {
  const u8 *src = buf + pre;  /* the block; buf[0, pre) = dictionary history staged before it */
  u32 hdr;
  if (n >= 2 && is_rle(src, n)) {
    if (cap < 4) return 0;
    hdr = (u32)last + (1u << 1) + (n << 3);
    dst[0] = (u8)hdr; dst[1] = (u8)(hdr >> 8); dst[2] = (u8)(hdr >> 16); dst[3] = src[0];
    return 4;
  }
  orc_seq_t *seq = malloc(sizeof(orc_seq_t) * (n / ZH_MIN_MATCH_SHORT + 2));
  u32 lastLits;
  size_t ns = orc_lz_parse_pre(buf, pre, pre + n, seq, &lastLits);
  u32 repSave[3] = {rep[0], rep[1], rep[2]};
  size_t body = (cap > 3) ? orc_encode_block_body(dst + 3, cap - 3, src, n, seq, ns, rep) : (size_t)-1;
  free(seq);
  if (body == (size_t)-1 || body == 0) {
    /* raw block; the decoder sees no sequences, so its repcodes are unchanged */
    rep[0] = repSave[0]; rep[1] = repSave[1]; rep[2] = repSave[2];
    if (cap < 3 + (size_t)n) return 0;
    hdr = (u32)last + (0u << 1) + (n << 3);
    dst[0] = (u8)hdr; dst[1] = (u8)(hdr >> 8); dst[2] = (u8)(hdr >> 16);
    memcpy(dst + 3, src, n);
    return 3 + (size_t)n;
  }
  hdr = (u32)last + (2u << 1) + ((u32)body << 3);
  dst[0] = (u8)hdr; dst[1] = (u8)(hdr >> 8); dst[2] = (u8)(hdr >> 16);
  return 3 + body;
}
size_t orc_compress_block(u8 *dst, size_t cap, const u8 *src, u32 n, int last, u32 rep[3]) {
  return orc_compress_block_pre(dst, cap, src, 0, n, last, rep);
}

/* Frame header (reference write_frame_header, src/cuda_zstd_manager.cu:3998-4106,
 * without dictionary / checksum).  Returns header size. */
size_t orc_frame_header_dict(u8 *dst, u64 content, u32 block_size, u32 window_log, u32 dict_id);
size_t orc_frame_header(u8 *dst, u64 content, u32 block_size, u32 window_log) { return orc_frame_header_dict(dst, content, block_size, window_log, 0); }
/* dict_id != 0: Dictionary_ID field of libzstd's minimal size (the reference writes a 1-byte
 * XXH32 of the buffer, :4020-4026, which libzstd rejects). */
size_t orc_frame_header_dict(u8 *dst, u64 content, u32 block_size, u32 window_log, u32 dict_id) {
  size_t o = 0;
  u32 const didf = dict_id == 0 ? 0 : dict_id < 256 ? 1 : dict_id < 65536 ? 2 : 3;
  u32 magic = 0xFD2FB528u;
  memcpy(dst, &magic, 4); o = 4;
  int ss = content <= block_size;
  u32 fcs_flag, fcs_size;
  if (ss) { if (content < 256) { fcs_flag = 0; fcs_size = 1; } else if (content < 65536 + 256) { fcs_flag = 1; fcs_size = 2; } else if (content <= 0xFFFFFFFFull) { fcs_flag = 2; fcs_size = 4; } else { fcs_flag = 3; fcs_size = 8; } }
  else { if (content >= 256 && content < 65536 + 256) { fcs_flag = 1; fcs_size = 2; } else if (content <= 0xFFFFFFFFull) { fcs_flag = 2; fcs_size = 4; } else { fcs_flag = 3; fcs_size = 8; } }
  dst[o++] = (u8)((fcs_flag << 6) | (ss ? 0x20 : 0) | didf);
  if (!ss) dst[o++] = (u8)((window_log - 10) << 3);
  for (u32 k = 0; k < (didf == 3 ? 4u : didf); k++) dst[o++] = (u8)(dict_id >> (8 * k));
  if (fcs_size == 1) dst[o++] = (u8)content;
  else if (fcs_size == 2) { u32 v = (u32)content - 256; dst[o++] = (u8)v; dst[o++] = (u8)(v >> 8); }
  else if (fcs_size == 4) { u32 v = (u32)content; memcpy(dst + o, &v, 4); o += 4; }
  else { memcpy(dst + o, &content, 8); o += 8; }
  return o;
}

/* XXH64, seed 0 (the published xxHash algorithm, which the reference runs in
 * src/cuda_zstd_xxhash.cu:72-228 for the frame content checksum; pinned against the
 * python xxhash module in tests/test_oracle_stages.py). */
static u64 xx_rotl(u64 x, int r) { return (x << r) | (x >> (64 - r)); }
static u64 xx_round(u64 acc, u64 in) { return xx_rotl(acc + in * 0xC2B2AE3D27D4EB4Full, 31) * 0x9E3779B185EBCA87ull; }
u64 orc_xxh64(const u8 *p, u64 n) {
  const u64 P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull, P4 = 0x85EBCA77C2B2AE63ull,
            P5 = 0x27D4EB2F165667C5ull;
  u64 h, i = 0;
  if (n >= 32) {
    u64 v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1, w;
    for (; i + 32 <= n; i += 32) {
      memcpy(&w, p + i, 8); v1 = xx_round(v1, w);
      memcpy(&w, p + i + 8, 8); v2 = xx_round(v2, w);
      memcpy(&w, p + i + 16, 8); v3 = xx_round(v3, w);
      memcpy(&w, p + i + 24, 8); v4 = xx_round(v4, w);
    }
    h = xx_rotl(v1, 1) + xx_rotl(v2, 7) + xx_rotl(v3, 12) + xx_rotl(v4, 18);
    h = (h ^ xx_round(0, v1)) * P1 + P4;
    h = (h ^ xx_round(0, v2)) * P1 + P4;
    h = (h ^ xx_round(0, v3)) * P1 + P4;
    h = (h ^ xx_round(0, v4)) * P1 + P4;
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) {
    u64 w;
    memcpy(&w, p + i, 8);
    h ^= xx_round(0, w);
    h = xx_rotl(h, 27) * P1 + P4;
  }
  if (i + 4 <= n) {
    u32 w;
    memcpy(&w, p + i, 4);
    h ^= (u64)w * P1;
    h = xx_rotl(h, 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; i++) {
    h ^= (u64)p[i] * P5;
    h = xx_rotl(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

/* Whole frame.  block_size = reference CompressionConfig.block_size (frame
 * header single-segment rule); internal blocks are ZH_BLOCK_MAX bytes.  Blocks
 * after the first start with unknown repcodes (they are compressed
 * independently on the GPU).  Returns frame size or 0. */
size_t orc_compress_frame_ck(u8 *dst, size_t cap, const u8 *src, u64 n, u32 block_size, u32 window_log, int checksum);
size_t orc_compress_frame(u8 *dst, size_t cap, const u8 *src, u64 n, u32 block_size, u32 window_log) {
  return orc_compress_frame_ck(dst, cap, src, n, block_size, window_log, 0);
}

/* checksum != 0: Content_Checksum_Flag set and the low 32 bits of XXH64 of the input
 * appended (reference src/cuda_zstd_manager.cu:3037-3056 when checksum is computed). */
/* ------------------------------------------------------------------------ */
/* Dictionaries (RFC 8878 §5)                                */
/* ------------------------------------------------------------------------ */
static u32 dict_fwd32(const u8 *p, size_t avail, size_t bitpos) {
  size_t b = bitpos >> 3; u64 v = 0;
  for (size_t i = 0; i < 5; i++) if (b + i < avail) v |= (u64)p[b + i] << (8 * i);
  return (u32)(v >> (bitpos & 7));
}
/* bytes of an FSE table description (FSE_readNCount restated for sizing); 0 if malformed */
static size_t dict_ncount_size(const u8 *p, size_t avail, u32 maxSV, u32 maxLog) {
  if (!avail) return 0;
  u32 nb = (dict_fwd32(p, avail, 0) & 15u) + 5u;
  if (nb > maxLog) return 0;
  size_t bp = 4; int rem = (1 << nb) + 1, thr = 1 << nb; nb++;
  u32 sym = 0; int prev0 = 0;
  while (rem > 1 && sym <= maxSV) {
    if (prev0) {
      u32 n0 = sym, r;
      do { r = dict_fwd32(p, avail, bp) & 3u; bp += 2; n0 += r; } while (r == 3 && bp < 8 * avail + 32);
      if (n0 > maxSV) return 0;
      sym = n0;
    }
    u32 bs = dict_fwd32(p, avail, bp); int mx = (2 * thr - 1) - rem, c;
    if ((int)(bs & (u32)(thr - 1)) < mx) { c = (int)(bs & (u32)(thr - 1)); bp += nb - 1; }
    else { c = (int)(bs & (u32)(2 * thr - 1)); if (c >= thr) c -= mx; bp += nb; }
    c--; rem -= c < 0 ? -c : c; sym++; prev0 = c == 0;
    while (rem < thr) { nb--; thr >>= 1; }
  }
  if (rem != 1) return 0;
  size_t used = (bp + 7) >> 3;
  return used <= avail ? used : 0;
}
/* Raw content (no 0xEC30A437 magic): *id = 0, content at 0.  Formatted: Dictionary_ID, Huffman
 * table description, OF / ML / LL FSE table descriptions, three repcodes (each in [1, content
 * size], libzstd ZSTD_loadDEntropy), content.  Returns 0, or -1 if malformed. */
int orc_dict_layout(const u8 *d, size_t n, u32 *id, size_t *content_off) {
  u32 magic = 0;
  *id = 0; *content_off = 0;
  if (n >= 4) memcpy(&magic, d, 4);
  if (n < 8 || magic != 0xEC30A437u) return 0;
  memcpy(id, d + 4, 4);
  size_t o = 8;
  u32 hb = d[o];
  size_t hsz = hb >= 128 ? 1 + ((size_t)(hb - 127) + 1) / 2 : 1 + (size_t)hb;
  if (hb == 0 || o + hsz > n) return -1;
  o += hsz;
  static const u32 msv[3] = {31, 52, 35}, mlg[3] = {8, 9, 9};
  for (int t = 0; t < 3; t++) {
    size_t u = o < n ? dict_ncount_size(d + o, n - o, msv[t], mlg[t]) : 0;
    if (!u) return -1;
    o += u;
  }
  if (o + 12 > n) return -1;
  for (int k = 0; k < 3; k++) {
    u32 r; memcpy(&r, d + o + 4 * k, 4);
    if (r == 0 || r > n - o - 12) return -1;
  }
  *content_off = o + 12;
  return 0;
}

/* Whole frame with an optional dictionary (dict_n == 0: none).  The first block is compressed
 * behind the last min(content, ZH_BLOCK_MAX - block) bytes of the dictionary content; blocks of
 * a dictionary frame start with unknown repcodes (the dictionary's are never referenced). */
size_t orc_compress_frame_dict(u8 *dst, size_t cap, const u8 *src, u64 n, u32 block_size, u32 window_log, int checksum, const u8 *dict,
                               size_t dict_n) {
  u32 did = 0;
  size_t co = 0;
  if (dict_n && orc_dict_layout(dict, dict_n, &did, &co)) return 0;
  if (cap < (dict_n ? 26u : 22u)) return 0;
  size_t o = orc_frame_header_dict(dst, n, block_size, window_log, did);
  if (checksum) dst[4] |= 0x04;
  u64 pos = 0;
  u32 b = 0;
  u32 const bs = ZH_FRAME_BLOCK(n, dict_n != 0 && orc_parse_level < ZH_DEEP_LEVEL);
  do {
    u32 bn = (u32)((n - pos) < bs ? (n - pos) : bs);
    u32 rep[3] = {1, 4, 8};
    if (b > 0 || dict_n) { rep[0] = rep[1] = rep[2] = 0; }
    size_t w;
    if (b == 0 && dict_n) {
      size_t cn = dict_n - co;
      size_t const room = orc_parse_level >= ZH_DEEP_LEVEL ? (size_t)ZH_DEEP_PRE : (size_t)(ZH_BLOCK_MAX - bn);
      u32 pre = (u32)(cn < room ? cn : room);
      u8 *buf = malloc((size_t)pre + bn + 16);
      memcpy(buf, dict + dict_n - pre, pre);
      memcpy(buf + pre, src, bn);
      w = orc_compress_block_pre(dst + o, cap - o, buf, pre, bn, pos + bn >= n, rep);
      free(buf);
    } else if (b > 0 && window_log >= ZH_HIST_WINDOW_LOG) {
      /* history: the previous 32 KiB block is hashed and matched against, never parsed */
      w = orc_compress_block_pre(dst + o, cap - o, src + pos - ZH_HIST_BLOCK, ZH_HIST_BLOCK, bn, pos + bn >= n, rep);
    } else {
      w = orc_compress_block(dst + o, cap - o, src + pos, bn, pos + bn >= n, rep);
    }
    if (!w) return 0;
    o += w; pos += bn; b++;
  } while (pos < n);
  if (checksum) {
    if (o + 4 > cap) return 0;
    u32 h = (u32)orc_xxh64(src, n);
    memcpy(dst + o, &h, 4);
    o += 4;
  }
  return o;
}
size_t orc_compress_frame_ck(u8 *dst, size_t cap, const u8 *src, u64 n, u32 block_size, u32 window_log, int checksum) {
  return orc_compress_frame_dict(dst, cap, src, n, block_size, window_log, checksum, NULL, 0);
}
/* The frame at a compression level: levels >= ZH_DEEP_LEVEL run the deep matcher (the device's
 * zh_lz_deep_kernel); the dual-hash LAZY2 parse (orc_parse_lazy2) stays for the study tools. */
size_t orc_compress_frame_lv(u8 *dst, size_t cap, const u8 *src, u64 n, u32 block_size, u32 window_log, int checksum, const u8 *dict,
                             size_t dict_n, int level) {
  int const save = orc_parse_lazy2, save_lv = orc_parse_level, save_m = orc_lz_mode;
  orc_parse_lazy2 = level >= 9;
  orc_parse_level = level;
  orc_lz_mode = ZH_K1_MODE(level);
  size_t const r = orc_compress_frame_dict(dst, cap, src, n, block_size, window_log, checksum, dict, dict_n);
  orc_parse_lazy2 = save;
  orc_parse_level = save_lv;
  orc_lz_mode = save_m;
  return r;
}

size_t orc_max_compressed_size(u64 n) {
  /* reference estimate_compressed_size (src/cuda_zstd_types.cpp:831-853) */
  u64 nb = (n + (128 * 1024 - 1)) / (128 * 1024);
  if (nb == 0) nb = 1;
  return (size_t)(n + n / 255 + nb * 3 + 512);
}
