// zh_entropy.hip — K2: entropy coding + block/frame assembly, one wave64 per block.
//
// Replaces the reference's compress_literals (Raw only, src/cuda_zstd_manager.cu:4406-4484),
// encode_sequences_with_predefined_fse / k_build_ctable / k_encode_fse_interleaved
// (src/cuda_zstd_manager.cu:4493-4661, src/cuda_zstd_fse_encoding_kernel.cu:32-325),
// write_block (:4227-4286) and write_frame_header (:3998-4106).
// Bit-for-bit the same stream as oracle/zstd_oracle.c (orc_compress_block), whose
// entropy stage is pinned byte-identical to libzstd 1.4.9.
//
// Work split: everything data-parallel (histograms, code computation, sequence
// merge, Huffman stream packing, FSE bit packing) runs on the 64 lanes; the
// inherently serial parts (repcode history, table builds, FSE state chain)
// run as wave-uniform loops.  Many blocks are resident per CU (small LDS), so
// one block's serial chain overlaps other blocks' parallel phases.
#include "zh_common.h"

namespace {

#ifndef ZH_K2_PAIR
#define ZH_K2_PAIR 1  // the record pass two chunks per iteration
#endif
#ifndef ZH_HIST_PF
#define ZH_HIST_PF 1  // literal histogram: next step's loads before this step's atomics
#endif
constexpr u32 K2_THREADS = 128;  // wave 0: literals section; wave 1: frame/sequences section, finish
constexpr u32 SW_WORDS = 184;  // >= 512 literal codes of <= 11 bits per append (+ pending bits)

// ---------------- LDS layout (bytes) ----------------
// The literals-only regions come first: wave 1's copy of the layout starts early enough that
// its (unused) SW / HVAL / HNB overlap the end of wave 0's copy.
constexpr u32 OFF_SW = 0;                          // bit sink words
constexpr u32 OFF_HVAL = OFF_SW + 4 * SW_WORDS;    // u16[256] Huffman code values
constexpr u32 OFF_HNB = OFF_HVAL + 2 * 256;        // u8[256] Huffman code lengths
constexpr u32 OFF_MISC = OFF_HNB + 256;            // 64 u32 scalars / broadcast
constexpr u32 OFF_HIST = OFF_MISC + 4 * 64;        // 256 u32 literal histogram; later 121 code counts
constexpr u32 OFF_HBUF = OFF_HIST + 4 * 256;       // u8[768] header scratch (weights / NCount)
constexpr u32 OFF_SCR = OFF_HBUF + 768;            // serial-helper scratch (lane 0)
constexpr u32 OFF_U = OFF_SCR + 1024;              // union: Huffman nodes | FSE tables
static_assert(OFF_U % 16 == 0, "alignment");
// Huffman build view
constexpr u32 OFF_NODES = OFF_U;                   // 514 nodes x 8 B
constexpr u32 U_HUF_END = OFF_NODES + 8 * 516;
// FSE view
constexpr u32 OFF_ST_LL = OFF_U;                   // u16[512]
constexpr u32 OFF_ST_OF = OFF_ST_LL + 1024;        // u16[256]
constexpr u32 OFF_ST_ML = OFF_ST_OF + 512;         // u16[512]
constexpr u32 OFF_SYM = OFF_ST_ML + 1024;          // (u32 dNb, s32 dFS): LL [0, 36), OF [36, 68), ML [68, 121)
constexpr u32 SYM_OF = 36, SYM_ML = 68;
constexpr u32 OFF_TSYM = OFF_SYM + 976;            // u8[512] spread scratch
constexpr u32 OFF_NORM = OFF_TSYM + 512;           // s16[64]
constexpr u32 U_FSE_END = OFF_NORM + 128;
// the Huffman weights' FSE table (tableLog <= 6, <= 13 symbols) and the weights, in the nodes'
// region once the tree is built (wave 0 only)
constexpr u32 OFF_W_ST = OFF_U, OFF_W_SYM = OFF_U + 128, OFF_W_TSYM = OFF_U + 256, OFF_W_NORM = OFF_U + 320;
constexpr u32 OFF_WTS = OFF_U + 352;               // u8[256] Huffman weights
static_assert(OFF_WTS + 256 <= U_HUF_END, "weights inside the nodes' region");
// wave 0 (literals) uses [0, U_HUF_END), wave 1 (sequences) [OFF_MISC, U_FSE_END) of its copy:
// wave 1's copy starts where wave 0's ends, less the literal-only head it never touches
constexpr u32 K2_WAVE_LDS = (U_HUF_END > U_FSE_END ? U_HUF_END : U_FSE_END);  // one wave's layout
static_assert(K2_WAVE_LDS < 16384, "K2 LDS budget");
constexpr u32 K2_W1 = (U_HUF_END - OFF_MISC + 15) & ~15u;  // wave 1's layout base
#ifndef ZH_K2_LDS_PAD
#define ZH_K2_LDS_PAD 0  // (occupancy experiments: extra LDS per block)
#endif
constexpr u32 K2_LDS = K2_W1 + U_FSE_END + ZH_K2_LDS_PAD;  // 15,952 B: 10 blocks per CU (was 17,632: 9)

__constant__ u8 c_LL_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ u8 c_ML_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ s16 c_LL_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ s16 c_ML_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ s16 c_OF_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ u8 c_LL_code[64] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 16, 17, 17, 18, 18, 19, 19,
                                 20, 20, 20, 20, 21, 21, 21, 21, 22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                                 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
__constant__ u8 c_ML_code[128] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                  32, 32, 33, 33, 34, 34, 35, 35, 36, 36, 36, 36, 37, 37, 37, 37, 38, 38, 38, 38, 38, 38, 38, 38, 39, 39, 39, 39, 39, 39, 39, 39,
                                  40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41,
                                  42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42};

__constant__ u32 c_rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};

// LDS scratch for the lane-0 serial helpers (keeps them out of scratch memory)
struct SerialScratch {
  u32 cumul[64];
  u32 rankLast[16];
  u32 base[32];
  u32 curr[32];
  u32 wcount[16];
  u16 nbPerRank[16];
  u16 valPerRank[16];
  u32 khigh[64];   // parallel FSE spread: step index of each high (low-probability) cell
  u8 lowsym[64];   // ... and the symbol stored there
};
static_assert(sizeof(SerialScratch) <= 1024, "scratch");

__device__ __forceinline__ u32 highbit32(u32 v) { return 31u - (u32)__builtin_clz(v); }
__device__ __forceinline__ u32 ll_code(u32 ll) { return ll > 63 ? highbit32(ll) + 19 : c_LL_code[ll]; }
__device__ __forceinline__ u32 ml_code(u32 mlBase) { return mlBase > 127 ? highbit32(mlBase) + 36 : c_ML_code[mlBase]; }
__device__ __forceinline__ u32 lane_id() { return threadIdx.x & 63u; }
// Code tables held across the wave (lane x holds entry x), looked up with ds_bpermute
// instead of a constant-memory load per lookup.  All lanes must execute the lookups.
struct CodeTabs {
  u32 llc, mlc0, mlc1, llb, mlb;
  __device__ __forceinline__ void load() {
    u32 const l = lane_id();
    llc = c_LL_code[l]; mlc0 = c_ML_code[l]; mlc1 = c_ML_code[64 + l];
    llb = l < 36 ? c_LL_bits[l] : 0u; mlb = l < 53 ? c_ML_bits[l] : 0u;
  }
  __device__ __forceinline__ u32 ll_code(u32 ll) const {
    u32 const c = (u32)__shfl((int)llc, (int)(ll & 63u), 64);
    return ll > 63 ? highbit32(ll) + 19 : c;
  }
  __device__ __forceinline__ u32 ml_code(u32 m) const {
    u32 const a = (u32)__shfl((int)mlc0, (int)(m & 63u), 64), b = (u32)__shfl((int)mlc1, (int)(m & 63u), 64);
    return m > 127 ? highbit32(m) + 36 : (m < 64 ? a : b);
  }
  __device__ __forceinline__ u32 ll_bits(u32 c) const { return (u32)__shfl((int)llb, (int)(c & 63u), 64); }
  __device__ __forceinline__ u32 ml_bits(u32 c) const { return (u32)__shfl((int)mlb, (int)(c & 63u), 64); }
};
// Orders a wave's LDS accesses around it (the data is the wave's own: LDS executes one wave's
// operations in order, so a compiler fence is all that is needed; kernels with several waves
// per workgroup give each wave its own LDS slice)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ u32 wave_excl_scan(u32 v, u32 &total) {
  u32 const incl = wave_scan_incl(v);  // DPP (zh_common.h)
  total = lane_value(incl, 63);
  return incl - v;
}
__device__ __forceinline__ u32 wave_sum(u32 v) { return lane_value(wave_scan_incl(v), 63); }
__device__ __forceinline__ u32 wave_max(u32 v) { return lane_value(wave_scan_max_incl(v), 63); }

// ---------------- output: bytes at dst[pos..] guarded by cap ----------------
struct Out {
  u8 *dst;
  u32 cap;
  __device__ __forceinline__ void put(u32 pos, u8 v) const { if (pos < cap) dst[pos] = v; }
};

// ---------------- bit sink: LSB-first fields, little-endian bytes (BIT_CStream) ----------------
// Wave-uniform state; sw[] holds the pending partial byte in sw[0] bits [0, pend).
struct BitSink {
  u32 pos;   // next byte to write in Out
  u32 pend;  // pending bits in sw[0] (0..7)
};

#ifndef ZH_SINK_BF
#define ZH_SINK_BF 1
#endif
template <int K>
__device__ __forceinline__ void sink_append(BitSink &bs, const Out &o, u32 *sw, const u32 (&val)[K], const u32 (&nb)[K]) {
  u32 const lane = lane_id();
  u32 tot = 0;
#pragma unroll
  for (int k = 0; k < K; k++) tot += nb[k];
  u32 all;
  u32 bit = wave_excl_scan(tot, all) + bs.pend;
  u32 const end = bs.pend + all;
  u32 const nwords = (end + 31) >> 5;
  for (u32 w = 1 + lane; w < nwords + 1; w += 64) sw[w] = 0;
  wave_sync();
#if ZH_SINK_BF
  // branch-free: every field ORs its low part into word bit >> 5 and its high part (0 unless it
  // straddles) into the next word, which lies inside [1, nwords] (zeroed above) since bit < end;
  // a field of 0 bits ORs 0.  Field widths are <= 31 (codes, states, extra bits), so v_bfe masks.
  u32 *const swa = sw;
#pragma unroll
  for (int k = 0; k < K; k++) {
    u32 const v = __builtin_amdgcn_ubfe(val[k], 0u, nb[k]);
    u32 *const wp = swa + (bit >> 5);
    u32 const sh = bit & 31u;
    __hip_atomic_fetch_or(wp, v << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(wp + 1, (v >> 1) >> (31u - sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    bit += nb[k];
  }
#else
#pragma unroll
  for (int k = 0; k < K; k++) {
    if (nb[k]) {
      u32 const v = val[k] & ((nb[k] >= 32) ? 0xFFFFFFFFu : ((1u << nb[k]) - 1u));
      u32 const w = bit >> 5, sh = bit & 31;
      atomicOr(&sw[w], v << sh);
      if (sh + nb[k] > 32) atomicOr(&sw[w + 1], v >> (32 - sh));
      bit += nb[k];
    }
  }
#endif
  wave_sync();
  u32 const full = end >> 3;
  const u8 *sb = (const u8 *)sw;
  for (u32 i = lane; i < full; i += 64) o.put(bs.pos + i, sb[i]);
  u8 const part = sb[full];
  wave_sync();
  if (lane == 0) sw[0] = (end & 7) ? part : 0;
  bs.pos += full;
  bs.pend = end & 7;
  wave_sync();
}

// BIT_closeCStream: end mark + flush of the partial byte
__device__ __forceinline__ void sink_close(BitSink &bs, const Out &o, u32 *sw) {
  u32 v[1] = {1u}, nb[1] = {lane_id() == 0 ? 1u : 0u};
  sink_append<1>(bs, o, sw, v, nb);
  if (bs.pend) {
    if (lane_id() == 0) o.put(bs.pos, (u8)sw[0]);
    bs.pos += 1;
    bs.pend = 0;
  }
  if (lane_id() == 0) sw[0] = 0;
  wave_sync();
}

// ---------------- FSE (libzstd v1.4.9 algorithms; lane-0 serial) ----------------
__device__ u32 fse_min_table_log(u32 srcSize, u32 maxSV) {
  u32 a = highbit32(srcSize) + 1, b = highbit32(maxSV) + 2;
  return a < b ? a : b;
}
__device__ u32 fse_optimal_table_log(u32 maxTableLog, u32 srcSize, u32 maxSV, u32 minus) {
  u32 maxBitsSrc = highbit32(srcSize - 1) - minus;
  u32 tableLog = maxTableLog;
  u32 minBits = fse_min_table_log(srcSize, maxSV);
  if (maxBitsSrc < tableLog) tableLog = maxBitsSrc;
  if (minBits > tableLog) tableLog = minBits;
  if (tableLog < 5) tableLog = 5;
  if (tableLog > 12) tableLog = 12;
  return tableLog;
}

__device__ bool fse_normalize_m2(s16 *norm, u32 tableLog, const u32 *count, u32 total, u32 maxSV, s16 lowProbCount) {
  const s16 NOT_YET = -2;
  u32 distributed = 0, toDistribute;
  u32 lowThreshold = total >> tableLog;
  u32 lowOne = (u32)(((u64)total * 3) >> (tableLog + 1));
  for (u32 s = 0; s <= maxSV; s++) {
    if (count[s] == 0) { norm[s] = 0; continue; }
    if (count[s] <= lowThreshold) { norm[s] = lowProbCount; distributed++; total -= count[s]; continue; }
    if (count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
    norm[s] = NOT_YET;
  }
  toDistribute = (1u << tableLog) - distributed;
  if (toDistribute == 0) return true;
  if ((total / toDistribute) > lowOne) {
    lowOne = (u32)(((u64)total * 3) / (toDistribute * 2));
    for (u32 s = 0; s <= maxSV; s++)
      if (norm[s] == NOT_YET && count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; }
    toDistribute = (1u << tableLog) - distributed;
  }
  if (distributed == maxSV + 1) {
    u32 maxV = 0, maxC = 0;
    for (u32 s = 0; s <= maxSV; s++) if (count[s] > maxC) { maxV = s; maxC = count[s]; }
    norm[maxV] += (s16)toDistribute;
    return true;
  }
  if (total == 0) {
    for (u32 s = 0; toDistribute > 0; s = (s + 1) % (maxSV + 1)) if (norm[s] > 0) { toDistribute--; norm[s]++; }
    return true;
  }
  u64 const vStepLog = 62 - tableLog;
  u64 const mid = (1ull << (vStepLog - 1)) - 1;
  u64 const rStep = (((1ull << vStepLog) * toDistribute) + mid) / (u64)total;
  u64 tmpTotal = mid;
  for (u32 s = 0; s <= maxSV; s++) {
    if (norm[s] == NOT_YET) {
      u64 const end = tmpTotal + (count[s] * rStep);
      u32 const weight = (u32)(end >> vStepLog) - (u32)(tmpTotal >> vStepLog);
      if (weight < 1) return false;
      norm[s] = (s16)weight;
      tmpTotal = end;
    }
  }
  return true;
}

// ---------------- FSE normalisation + NCount, wave-parallel (lane = symbol, maxSV < 64) ----------------
// FSE_normalizeCount (libzstd v1.4.9) with the per-symbol probabilities on the lanes and the
// two reductions (sum, first-maximum) on DPP; the rare "m2" redistribution falls back to the
// serial fse_normalize_m2 on lane 0.  c = this lane's count (0 past maxSV).  The result is
// returned per lane (lane s: norm[s]) and stored to norm[] in LDS.
__device__ int fse_normalize_wave(s16 *norm, u32 tableLog, u32 c, u32 total, u32 maxSV, bool useLowProbCount, u32 lane, u32 *cnt_scratch) {
  s16 const lowProbCount = useLowProbCount ? -1 : 1;
  u32 const scale = 62 - tableLog;
  u64 const step = (1ull << 62) / total;
  u64 const vStep = 1ull << (scale - 20);
  u32 const lowThreshold = total >> tableLog;
  int n = 0, contrib = 0;
  u32 key = 0;  // proba * 256 + (255 - s): the first symbol of maximal probability wins, as in the serial loop
  if (lane <= maxSV && c != 0) {
    if (c <= lowThreshold) {
      n = lowProbCount;
      contrib = 1;
    } else {
      u64 const cs = (u64)c * step;
      int proba = (int)(cs >> scale);
      if (proba < 8) proba += cs - ((u64)proba << scale) > vStep * c_rtb[proba];
      n = proba;
      contrib = proba;
      key = ((u32)proba << 8) | (255u - lane);
    }
  }
  int const still = (int)(1u << tableLog) - (int)wave_sum((u32)contrib);
  u32 const kmax = wave_max(key);
  u32 const largest = kmax ? 255u - (kmax & 255u) : 0u;
  int const nl = (int)lane_value((u32)n, largest);
  if (-still >= (nl >> 1)) {  // libzstd's FSE_normalizeM2 (rare): serial, from LDS
    if (lane <= maxSV) cnt_scratch[lane] = c;
    wave_sync();
    if (lane == 0) fse_normalize_m2(norm, tableLog, cnt_scratch, total, maxSV, lowProbCount);
    wave_sync();
    return lane <= maxSV ? norm[lane] : 0;
  }
  if (lane == largest) n += still;
  if (lane <= maxSV) norm[lane] = (s16)n;
  return n;
}

// FSE_writeNCount with every lane running the same (wave-uniform, scalar) loop; the counts
// come from the lanes of normv (v_readlane), lane 0 stores the bytes.  Returns the size.
__device__ u32 fse_write_ncount_wave(u8 *out, int normv, u32 maxSV, u32 tableLog, u32 lane) {
  u32 o = 0;
  auto put2 = [&](u32 bs) {
    if (lane == 0) { out[o] = (u8)bs; out[o + 1] = (u8)(bs >> 8); }
    o += 2;
  };
  int const tableSize = 1 << tableLog;
  int remaining = tableSize + 1, threshold = tableSize, nbBits = (int)tableLog + 1;
  u32 bitStream = tableLog - 5;
  int bitCount = 4;
  u32 symbol = 0;
  u32 const alphabetSize = maxSV + 1;
  bool previousIs0 = false;
  while (symbol < alphabetSize && remaining > 1) {
    if (previousIs0) {
      u32 start = symbol;
      while (symbol < alphabetSize && !lane_value((u32)normv, symbol)) symbol++;
      if (symbol == alphabetSize) break;
      while (symbol >= start + 24) {
        start += 24;
        bitStream += 0xFFFFu << bitCount;
        put2(bitStream);
        bitStream >>= 16;
      }
      while (symbol >= start + 3) { start += 3; bitStream += 3u << bitCount; bitCount += 2; }
      bitStream += (symbol - start) << bitCount;
      bitCount += 2;
      if (bitCount > 16) { put2(bitStream); bitStream >>= 16; bitCount -= 16; }
    }
    int count = (int)lane_value((u32)normv, symbol++);
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
    if (bitCount > 16) { put2(bitStream); bitStream >>= 16; bitCount -= 16; }
  }
  if (remaining != 1) return 0;
  if (lane == 0) { out[o] = (u8)bitStream; out[o + 1] = (u8)(bitStream >> 8); }
  return o + (u32)(bitCount + 7) / 8;
}

struct FseSym { u32 dNb; s32 dFS; };

// Wave-parallel FSE_buildCTable (libzstd 1.4.9's FSE_buildCTable_wksp tables).  Symbols <= 63.
// Spread: the i-th positive-count cell in symbol order goes to the i-th position of
// (k * step) & mask, k = 0, 1, ... skipping positions above highThreshold; with
// step odd, position u is reached at k(u) = u * step^-1 mod tableSize, so its rank is
// k(u) minus the number of skipped (high) positions reached earlier.
__device__ void fse_build_ctable_par(u16 *st, FseSym *sym, u8 *tableSymbol, const s16 *norm, u32 maxSV, u32 tableLog, SerialScratch *scr) {
  u32 const lane = lane_id();
  u32 const T = 1u << tableLog, mask = T - 1;
  u32 const step = (T >> 1) + (T >> 3) + 3;
  u32 inv = step;
#pragma unroll
  for (int it = 0; it < 5; it++) inv *= 2u - step * inv;
  inv &= mask;
  int const nv = lane <= maxSV ? (int)norm[lane] : 0;
  bool const isLow = nv == -1;
  u32 tot;
  u32 const cum = wave_excl_scan(isLow ? 1u : (u32)max(nv, 0), tot);   // first state slot of the symbol
  u32 const pst = wave_excl_scan(nv > 0 ? (u32)nv : 0u, tot);           // first spread rank of the symbol
  u64 const lowm = __ballot(isLow);
  u32 const nLow = (u32)__popcll(lowm);
  u32 const highThreshold = T - 1 - nLow;
  if (isLow) {
    u32 const i = (u32)__popcll(lowm & ((1ull << lane) - 1ull));  // low symbols fill the top, in symbol order
    scr->lowsym[i] = (u8)lane;
    scr->khigh[i] = ((T - 1 - i) * inv) & mask;
  }
  wave_sync();
  u32 *pstart = scr->base;   // base[32] + curr[32] = 64 entries
  pstart[lane] = lane <= maxSV ? pst : 0xFFFFFFFFu;
  wave_sync();
  for (u32 u = lane; u < T; u += 64) {
    u32 sy;
    if (u > highThreshold) {
      sy = scr->lowsym[T - 1 - u];
    } else {
      u32 const k = (u * inv) & mask;
      u32 before = 0;
      for (u32 i = 0; i < nLow; i++) before += scr->khigh[i] < k ? 1u : 0u;
      u32 const rank = k - before;
      // last symbol whose first rank <= rank (symbols with no positive cells share a
      // start with their successor and are skipped by the <=)
      u32 lo = 0, hi = maxSV;
      while (lo < hi) {
        u32 const mid = (lo + hi + 1) >> 1;
        if (pstart[mid] <= rank) lo = mid; else hi = mid - 1;
      }
      sy = lo;
    }
    tableSymbol[u] = (u8)sy;
  }
  wave_sync();
  // state table: st[cum[s] + j] = T + (j-th smallest position holding s)
  u32 run = 0;  // lane s: positions of symbol s placed so far
  for (u32 u0 = 0; u0 < T; u0 += 64) {
    u32 const u = u0 + lane;
    u32 const sy = u < T ? tableSymbol[u] : 0xFFu;
    u64 pend = __ballot(u < T);
    while (pend) {
      u32 const s0 = __builtin_amdgcn_readlane(sy, (u32)__builtin_ctzll(pend));
      u64 const m = __ballot(sy == s0) & pend;
      u32 const b0 = __builtin_amdgcn_readlane(run, s0) + __builtin_amdgcn_readlane(cum, s0);
      if ((m >> lane) & 1ull) st[b0 + (u32)__popcll(m & ((1ull << lane) - 1ull))] = (u16)(T + u);
      run += lane == s0 ? (u32)__popcll(m) : 0u;
      pend &= ~m;
    }
  }
  // symbol transforms
  if (lane <= maxSV) {
    if (nv == 0) { sym[lane].dNb = ((tableLog + 1) << 16) - T; sym[lane].dFS = 0; }
    else if (nv == -1 || nv == 1) { sym[lane].dNb = (tableLog << 16) - T; sym[lane].dFS = (s32)cum - 1; }
    else {
      u32 const maxBitsOut = tableLog - highbit32((u32)nv - 1);
      u32 const minStatePlus = (u32)nv << maxBitsOut;
      sym[lane].dNb = (maxBitsOut << 16) - minStatePlus;
      sym[lane].dFS = (s32)cum - nv;
    }
  }
  wave_sync();
}

// ---------------- Huffman (libzstd v1.4.9 HUF_buildCTable) ----------------
struct HufNode { u32 count; u16 parent; u8 byte; u8 nbBits; };

__device__ u32 huf_set_max_height(HufNode *huffNode, u32 lastNonNull, u32 maxNbBits, SerialScratch *scr) {
  u32 const largestBits = huffNode[lastNonNull].nbBits;
  if (largestBits <= maxNbBits) return largestBits;
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
  u32 const noSymbol = 0xF0F0F0F0u;
  u32 *rankLast = scr->rankLast;
  for (int i = 0; i < 14; i++) rankLast[i] = noSymbol;
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
      if (huffNode[highPos].count <= 2 * huffNode[lowPos].count) break;
    }
    while ((nBitsToDecrease <= 12) && (rankLast[nBitsToDecrease] == noSymbol)) nBitsToDecrease++;
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
  return maxNbBits;
}


// --- wave-parallel HUF_buildCTable (same tree and code lengths as libzstd's serial build) ---
// element e of a 256-key array lives in lane e/4, slot e%4
__device__ __forceinline__ void bitonic_sort_desc_256(u32 (&key)[4]) {
  u32 const lane = lane_id();
#pragma unroll
  for (u32 size = 2; size <= 256; size <<= 1) {
#pragma unroll
    for (u32 d = size >> 1; d > 0; d >>= 1) {
      u32 part[4];
#pragma unroll
      for (u32 k = 0; k < 4; k++) part[k] = d >= 4 ? (u32)__shfl_xor((int)key[k], (int)(d >> 2), 64) : key[k ^ d];
#pragma unroll
      for (u32 k = 0; k < 4; k++) {
        u32 const e = 4 * lane + k;
        bool const desc = (e & size) == 0;
        bool const lo = (e & d) == 0;  // e is the lower index of its pair
        u32 const mx = max(key[k], part[k]), mn = min(key[k], part[k]);
        key[k] = (desc == lo) ? mx : mn;
      }
    }
  }
}

// value of slot i (0..255) of a 4-register lane-major array (i = 64 r + lane), wave-uniform i
__device__ __forceinline__ u32 wave_get(const u32 (&a)[4], u32 i) {
  u32 const l = i & 63u, r = i >> 6;
  u32 const v0 = __builtin_amdgcn_readlane(a[0], l), v1 = __builtin_amdgcn_readlane(a[1], l);
  u32 const v2 = __builtin_amdgcn_readlane(a[2], l), v3 = __builtin_amdgcn_readlane(a[3], l);
  return r == 0 ? v0 : r == 1 ? v1 : r == 2 ? v2 : v3;
}
__device__ __forceinline__ void wave_set(u32 (&a)[4], u32 i, u32 v) {
  u32 const l = i & 63u, r = i >> 6;
  bool const me = lane_id() == l;
#pragma unroll
  for (u32 k = 0; k < 4; k++) a[k] = (me && r == k) ? v : a[k];
}

#ifdef ZH_STAMPS
__device__ u32 g_hst[6];  // diagnostic: Huffman build phase cycles (all blocks)
#define HSTAMP(k)                                                     \
  do {                                                                \
    u64 const t_ = __builtin_amdgcn_s_memtime();                      \
    if ((k) >= 0 && lane == 0) atomicAdd(&g_hst[(k) < 0 ? 0 : (k)], (u32)(t_ - hst_prev)); \
    hst_prev = t_;                                                    \
  } while (0)
#else
#define HSTAMP(k) do { } while (0)
#endif
__device__ u32 huf_build_ctable_par(HufNode *huffNode0, u16 *hval, u8 *hnb, const u32 *count, u32 maxSV, u32 maxNbBits, SerialScratch *scr) {
  u32 const lane = lane_id();
#ifdef ZH_STAMPS
  u64 hst_prev = 0;
#endif
  HufNode *const huffNode = huffNode0 + 1;
  u32 const STARTNODE = 256;
  for (u32 i = lane; i < 2 * 256 + 2; i += 64) { huffNode0[i].count = 0; huffNode0[i].parent = 0; huffNode0[i].byte = 0; huffNode0[i].nbBits = 0; }
  // HUF_sort order = count descending, symbol ascending among equal counts
  u32 key[4];
#pragma unroll
  for (u32 k = 0; k < 4; k++) {
    u32 const sym = 4 * lane + k;
    key[k] = sym <= maxSV ? (count[sym] << 8) | (255u - sym) : 0u;
  }
  HSTAMP(-1);
  bitonic_sort_desc_256(key);
  wave_sync();
  u32 nz = 0;
#pragma unroll
  for (u32 k = 0; k < 4; k++) {
    u32 const e = 4 * lane + k;
    if (e <= maxSV) { huffNode[e].count = key[k] >> 8; huffNode[e].byte = (u8)(255u - (key[k] & 255u)); }
    nz += (e <= maxSV && (key[k] >> 8) != 0) ? 1u : 0u;
  }
  int const nonNullRank = (int)wave_sum(nz) - 1;
  wave_sync();
  HSTAMP(0);
  // Two-queue merge (HUF_buildCTable's order and tie-break: a leaf only when strictly smaller)
  // with the counts in registers (leaf i / internal node m at lane i%64, reg i/64).  The loop
  // keeps each queue's head count and fetches only the next entry of the queue it advanced;
  // it records one bit per pick (1 = internal node), and the parents are written afterwards,
  // lane-parallel: pick k goes to node 256 + k/2, and its source is leaf
  // nonNullRank - (leaf picks before k) or internal node 256 + (internal picks before k).
  u32 L[4], I[4] = {0, 0, 0, 0};
#pragma unroll
  for (u32 r = 0; r < 4; r++) L[r] = huffNode[64 * r + lane].count;
  u32 const nodeRoot = STARTNODE + (u32)nonNullRank - 1;
  {
    int lowS = nonNullRank;
    u32 lowN = STARTNODE;
    u32 cs = wave_get(L, (u32)lowS), cn = 1u << 30;  // queue heads (internal queue empty)
    u64 bits = 0;
    u32 pwlo = 0, pwhi = 0, npick = 0;  // lane w: pick bits [64 w, 64 w + 64)
    for (u32 m = STARTNODE; m <= nodeRoot; m++) {
      u32 c = 0;
#pragma unroll
      for (u32 q = 0; q < 2; q++) {
        bool const internal = !(cs < cn);
        if (internal) {
          c += cn;
          lowN++;
          cn = lowN < m ? wave_get(I, lowN - STARTNODE) : (1u << 30);
        } else {
          c += cs;
          lowS--;
          cs = lowS >= 0 ? wave_get(L, (u32)lowS) : (1u << 31);
        }
        bits |= (u64)(internal ? 1u : 0u) << (npick & 63u);
        npick++;
      }
      wave_set(I, m - STARTNODE, c);
      if (lowN == m) cn = c;  // the queue was empty: the new node is its head
      if ((npick & 63u) == 0) {
        u32 const w = (npick >> 6) - 1;
        if (lane == w) { pwlo = (u32)bits; pwhi = (u32)(bits >> 32); }
        bits = 0;
      }
    }
    if (npick & 63u) {
      u32 const w = npick >> 6;
      if (lane == w) { pwlo = (u32)bits; pwhi = (u32)(bits >> 32); }
    }
    u32 const nw = (npick + 63u) >> 6;
    u32 const pcw = lane < nw ? (u32)__popcll(((u64)pwhi << 32) | pwlo) : 0u;
    u32 const ibw = wave_scan_incl(pcw) - pcw;  // internal picks before word w
    u64 const below = (1ull << lane) - 1ull;
    for (u32 q = 0; q < nw; q++) {
      u64 const word = ((u64)lane_value(pwhi, q) << 32) | lane_value(pwlo, q);
      u32 const k = 64u * q + lane;
      if (k < npick) {
        u32 const ib = lane_value(ibw, q) + (u32)__popcll(word & below);
        u32 const node = ((word >> lane) & 1u) ? STARTNODE + ib : (u32)nonNullRank - (k - ib);
        huffNode[node].parent = (u16)(STARTNODE + (k >> 1));
      }
    }
  }
  wave_sync();
  HSTAMP(1);
  // depths by pointer doubling over leaves 0..nonNull and internal nodes 256..root:
  // jump = parent (root: itself), dist = 1 (root: 0); nbBits of a leaf = its depth
  u32 const nLeaf = (u32)nonNullRank + 1, nInt = (u32)nonNullRank;
  for (u32 x = lane; x < nLeaf + nInt; x += 64) {
    u32 const nd = x < nLeaf ? x : STARTNODE + (x - nLeaf);
    huffNode[nd].nbBits = nd == nodeRoot ? 0 : 1;
    if (nd == nodeRoot) huffNode[nd].parent = (u16)nodeRoot;
  }
  wave_sync();
  for (u32 round = 0; (1u << round) < nLeaf; round++) {
    u32 jd[8], jj[8];
#pragma unroll
    for (u32 k = 0; k < 8; k++) {
      u32 const x = lane + 64 * k;
      jd[k] = 0; jj[k] = 0;
      if (x < nLeaf + nInt) {
        u32 const nd = x < nLeaf ? x : STARTNODE + (x - nLeaf);
        u32 const j = huffNode[nd].parent;
        jd[k] = huffNode[j].nbBits;
        jj[k] = huffNode[j].parent;
      }
    }
    wave_sync();
#pragma unroll
    for (u32 k = 0; k < 8; k++) {
      u32 const x = lane + 64 * k;
      if (x < nLeaf + nInt) {
        u32 const nd = x < nLeaf ? x : STARTNODE + (x - nLeaf);
        huffNode[nd].nbBits = (u8)(huffNode[nd].nbBits + jd[k]);
        huffNode[nd].parent = (u16)jj[k];
      }
    }
    wave_sync();
  }
  HSTAMP(2);
  if (lane == 0) maxNbBits = huf_set_max_height(huffNode, (u32)nonNullRank, maxNbBits, scr);
  maxNbBits = __builtin_amdgcn_readfirstlane(maxNbBits);
  if (maxNbBits > 12) return 0;
  HSTAMP(3);
  // nbPerRank / valPerRank, then codes in symbol order within each rank
  for (u32 i = lane; i < 256; i += 64) hnb[i] = 0;
  wave_sync();
  for (u32 nn = lane; nn <= maxSV; nn += 64) hnb[huffNode[nn].byte] = huffNode[nn].nbBits;
  wave_sync();
  // nbPerRank on lane r (ballots over the code lengths), then valPerRank as a uniform loop
  u32 nbr = 0;
  for (u32 n0 = 0; n0 <= maxSV; n0 += 64) {
    u32 const v = n0 + lane <= maxSV ? hnb[n0 + lane] : 0u;
    for (u32 r = 1; r <= maxNbBits; r++) {
      u32 const c = (u32)__popcll(__ballot(v == r));
      nbr += lane == r ? c : 0u;
    }
  }
  u32 base = 0;  // lane r holds the next code of rank r
  {
    u32 mn = 0;
    for (int r = (int)maxNbBits; r > 0; r--) {
      if (lane == (u32)r) base = mn;
      mn += lane_value(nbr, (u32)r);
      mn = (mn >> 1) & 0xFFFFu;
    }
  }
  for (u32 n0 = 0; n0 <= maxSV; n0 += 64) {
    u32 const nn = n0 + lane;
    u32 const v = nn <= maxSV ? hnb[nn] : 255u;
    u32 code = 0;
    for (u32 r = 0; r <= maxNbBits; r++) {
      u64 const m = __ballot(v == r);
      if (!m) continue;
      u32 const b0 = __builtin_amdgcn_readlane(base, r);
      if (v == r) code = b0 + (u32)__popcll(m & ((1ull << lane) - 1ull));
      base += lane == r ? (u32)__popcll(m) : 0u;
    }
    if (nn <= maxSV) hval[nn] = (u16)code;
  }
  wave_sync();
  HSTAMP(4);
  return maxNbBits;
}

// HUF_writeCTable with the whole wave: weights and their histogram lane-parallel, the weights'
// FSE table by the wave-parallel normalisation / NCount / table build, and the two-state
// FSE_compress_usingCTable of the weights as a wave-uniform loop whose table lookups are
// v_readlane from lane-held copies (weights <= 12, table <= 64 cells).  Same bytes as
// libzstd 1.4.9's HUF_writeCTable; returns the size (0 = raw literals), uniform.
__device__ u32 huf_write_ctable_wave(u8 *hbuf, u8 *w, const u8 *hnb, u32 maxSV, u32 huffLog, u16 *st, FseSym *sym, u8 *tsym, s16 *norm,
                                    SerialScratch *scr) {
  u32 const lane = lane_id();
  for (u32 n = lane; n <= maxSV; n += 64) w[n] = (n < maxSV && hnb[n]) ? (u8)(huffLog + 1 - hnb[n]) : 0;
  wave_sync();
  u32 h = 0;
  if (maxSV > 1) {
    // count[v] on lane v (v <= 12): one ballot per weight value per 64 weights
    u32 cnt = 0;
    for (u32 n0 = 0; n0 < maxSV; n0 += 64) {
      u32 const wv = n0 + lane < maxSV ? w[n0 + lane] : 255u;
#pragma unroll
      for (u32 v = 0; v <= 12; v++) {
        u32 const c = (u32)__popcll(__ballot(wv == v));
        cnt += lane == v ? c : 0u;
      }
    }
    u64 const nzm = __ballot(lane <= 12 && cnt != 0);
    u32 const mx = 63u - (u32)__builtin_clzll(nzm);
    u32 const maxCount = wave_max(lane <= 12 ? cnt : 0u);
    if (maxCount == maxSV) h = 1;
    else if (maxCount == 1) h = 0;
    else {
      u32 const tableLog = fse_optimal_table_log(6, maxSV, mx, 2);
      int const nv = fse_normalize_wave(norm, tableLog, lane <= mx ? cnt : 0u, maxSV, mx, false, lane, scr->cumul);
      u32 const hs = fse_write_ncount_wave(hbuf + 1, nv, mx, tableLog, lane);
      if (hs) {
        wave_sync();
        fse_build_ctable_par(st, sym, tsym, norm, mx, tableLog, scr);
        wave_sync();
        u32 cs = 0;
        if (maxSV > 2) {
          // lane-held copies: st (<= 64 cells), the symbol transforms, the weights (4 per lane)
          u32 const stv = lane < (1u << tableLog) ? (u32)st[lane] : 0u;
          u32 const dnbv = lane <= mx ? sym[lane].dNb : 0u;
          u32 const dfsv = lane <= mx ? (u32)sym[lane].dFS : 0u;
          u32 wl[4];
#pragma unroll
          for (u32 k = 0; k < 4; k++) wl[k] = 64 * k + lane < maxSV ? w[64 * k + lane] : 0u;
          auto wat = [&](u32 i) {  // w[i], i uniform
            u32 const l = i & 63u, r = i >> 6;
            u32 const a0 = lane_value(wl[0], l), a1 = lane_value(wl[1], l), a2 = lane_value(wl[2], l), a3 = lane_value(wl[3], l);
            return r == 0 ? a0 : r == 1 ? a1 : r == 2 ? a2 : a3;
          };
          auto init = [&](u32 sy) {
            u32 const dnb = lane_value(dnbv, sy), dfs = lane_value(dfsv, sy);
            u32 const nbo = (dnb + (1u << 15)) >> 16;
            return lane_value(stv, (((nbo << 16) - dnb) >> nbo) + dfs);
          };
          u8 *const out = hbuf + 1 + hs;
          u64 acc = 0;
          u32 nbits = 0, o = 0;
          auto add = [&](u32 v, u32 nb) {
            acc |= ((u64)v & ((1ull << nb) - 1ull)) << nbits;
            nbits += nb;
            while (nbits >= 8) {
              if (lane == 0) out[o] = (u8)acc;
              o++;
              acc >>= 8;
              nbits -= 8;
            }
          };
          auto step = [&](u32 &state, u32 sy) {
            u32 const dnb = lane_value(dnbv, sy), dfs = lane_value(dfsv, sy);
            u32 const nb = (state + dnb) >> 16;
            u32 const v = state & ((1u << nb) - 1u);
            state = lane_value(stv, (state >> nb) + dfs);
            add(v, nb);
          };
          int ip = (int)maxSV;
          u32 s1, s2;
          if (maxSV & 1) {
            s1 = init(wat((u32)--ip));
            s2 = init(wat((u32)--ip));
            step(s1, wat((u32)--ip));
          } else {
            s2 = init(wat((u32)--ip));
            s1 = init(wat((u32)--ip));
          }
          while (ip > 0) {
            step(s2, wat((u32)--ip));
            step(s1, wat((u32)--ip));
          }
          add(s2, tableLog);
          add(s1, tableLog);
          add(1, 1);
          if (nbits) {
            if (lane == 0) out[o] = (u8)acc;
            o++;
          }
          cs = o;
        }
        h = cs ? hs + cs : 0;
      }
    }
  }
  u32 ret;
  if ((h > 1) & (h < maxSV / 2)) {
    if (lane == 0) hbuf[0] = (u8)h;
    ret = h + 1;
  } else if (maxSV > 128) {
    ret = 0;
  } else {
    if (lane == 0) hbuf[0] = (u8)(128 + (maxSV - 1));
    for (u32 n = 2 * lane; n < maxSV; n += 128) hbuf[(n / 2) + 1] = (u8)((w[n] << 4) + w[n + 1]);
    ret = ((maxSV + 1) / 2) + 1;
  }
  wave_sync();
  return ret;
}

// byte copy global -> Out (wave-parallel)
// Wave copy of n bytes to o[pos..]: byte head up to a 4-B aligned destination, then
// dword stores (source realigned with alignbyte, 8 independent loads per lane in
// flight), byte tail; bytes at or past o.cap are dropped like Out::put does.
__device__ __forceinline__ void copy_bytes4(const Out &o, u32 pos, const u8 *src, u32 n) {
  u32 const lane = lane_id();
  u8 *const d0 = o.dst + pos;
  u32 const h = min((u32)((4u - ((uintptr_t)d0 & 3u)) & 3u), n);
  u32 const nw = (n - h) >> 2;
  u32 const capw = o.cap > pos + h ? (o.cap - pos - h) >> 2 : 0u;
  u32 const lim = min(nw, capw);
  const u8 *const s0 = src + h;
  u32 const sa = (u32)((uintptr_t)s0 & 3u);
  const u32 *const s32 = (const u32 *)(s0 - sa);
  u32 *const d32 = (u32 *)(d0 + h);
#ifndef ZH_COPY_U
#define ZH_COPY_U 8
#endif
  constexpr u32 U = ZH_COPY_U;  // dwords per lane in flight (16: no change on random data, 1.33 ms)
  for (u32 w0 = 0; w0 < lim; w0 += 64 * U) {
    u32 v[U];
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      if (w < lim) {
        u32 const A = s32[w];
        u32 const B = sa ? s32[w + 1] : A;  // word w+1 holds an in-range byte when sa != 0
        v[u] = __builtin_amdgcn_alignbyte(B, A, sa);
      }
    }
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const w = w0 + 64 * u + lane;
      if (w < lim) d32[w] = v[u];
    }
  }
  if (lane < h) o.put(pos + lane, src[lane]);
  for (u32 i = h + 4 * lim + lane; i < n; i += 64) o.put(pos + i, src[i]);
}

// Large copies (raw blocks, raw literals): 16-B aligned stores, each from the one or two
// aligned 16-B source chunks holding its bytes (a chunk holding a needed byte never crosses a
// page), funnel-shifted by the source's offset; CP16_U stores per lane in flight.
#ifndef ZH_CP16_U
#define ZH_CP16_U 4
#endif
__device__ __forceinline__ uint4 funnel16(uint4 a, uint4 b, u32 sa) {
  // bytes [sa, sa + 16) of the 32-byte a:b (sa wave-uniform; selects, no indexed array)
  u32 const q = sa >> 2, r = sa & 3u;
  u32 const w0 = q == 0 ? a.x : q == 1 ? a.y : q == 2 ? a.z : a.w;
  u32 const w1 = q == 0 ? a.y : q == 1 ? a.z : q == 2 ? a.w : b.x;
  u32 const w2 = q == 0 ? a.z : q == 1 ? a.w : q == 2 ? b.x : b.y;
  u32 const w3 = q == 0 ? a.w : q == 1 ? b.x : q == 2 ? b.y : b.z;
  u32 const w4 = q == 0 ? b.x : q == 1 ? b.y : q == 2 ? b.z : b.w;
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r), __builtin_amdgcn_alignbyte(w3, w2, r),
                    __builtin_amdgcn_alignbyte(w4, w3, r));
}
__device__ __forceinline__ void copy_bytes16(const Out &o, u32 pos, const u8 *src, u32 n) {
  u32 const lane = lane_id();
  u8 *const d0 = o.dst + pos;
  u32 const hb = min((u32)((16u - ((uintptr_t)d0 & 15u)) & 15u), n);  // bytes before a 16-B boundary
  u32 const nc = (n - hb) >> 4;
  u32 const capc = o.cap > pos + hb ? (o.cap - pos - hb) >> 4 : 0u;
  u32 const lim = min(nc, capc);
  const u8 *const s = src + hb;
  u32 const sa = (u32)((uintptr_t)s & 15u);
  const uint4 *const s16 = (const uint4 *)(s - sa);
  uint4 *const dd = (uint4 *)(d0 + hb);
  constexpr u32 U = ZH_CP16_U;
  for (u32 c0 = 0; c0 < lim; c0 += 64 * U) {
    uint4 a[U], b2[U];
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const c = c0 + 64 * u + lane;
      if (c < lim) {
        a[u] = s16[c];
        b2[u] = sa ? s16[c + 1] : a[u];
      }
    }
#pragma unroll
    for (u32 u = 0; u < U; u++) {
      u32 const c = c0 + 64 * u + lane;
      if (c < lim) dd[c] = sa ? funnel16(a[u], b2[u], sa) : a[u];
    }
  }
  if (lane < hb) o.put(pos + lane, src[lane]);
  for (u32 i = hb + 16 * lim + lane; i < n; i += 64) o.put(pos + i, src[i]);
}
#ifndef ZH_COPY16
#define ZH_COPY16 1
#endif
__device__ __forceinline__ void copy_bytes(const Out &o, u32 pos, const u8 *src, u32 n) {
  if (ZH_COPY16) copy_bytes16(o, pos, src, n);
  else copy_bytes4(o, pos, src, n);
}

}  // namespace

#ifdef ZH_STAMPS
#define ZH_STAMP(k)                                     \
  do {                                                  \
    u64 _t = __builtin_amdgcn_s_memtime();              \
    st[k] += (u32)(_t - stamp_prev);                    \
    stamp_prev = _t;                                    \
  } while (0)
#else
#define ZH_STAMP(k) do { } while (0)
#endif

// ============================================================================
// Raw fallback (ZSTD_compressBlock_internal: a compressed body of >= n - minGain bytes is
// replaced by the raw block) and the block header; returns the block's end offset.
// A 64-lane sweep over u64 records: lane l of chunk c gets record 64 c + l, loaded
// RING_DEPTH chunks ahead (global-memory latency at 4 waves per SIMD is several chunks' work)
constexpr u32 RING_DEPTH = 4;
struct RecRing {
  u64 r[RING_DEPTH];
  __device__ __forceinline__ void init(const u64 *seq, u32 n, u32 lane) {
#pragma unroll
    for (u32 k = 0; k < RING_DEPTH; k++) r[k] = lane + 64 * k < n ? seq[lane + 64 * k] : 0;
  }
  __device__ __forceinline__ u64 next(const u64 *seq, u32 n, u32 i) {
    u64 const v = r[0];
#pragma unroll
    for (u32 k = 0; k + 1 < RING_DEPTH; k++) r[k] = r[k + 1];
    u32 const j = i + 64 * RING_DEPTH;
    r[RING_DEPTH - 1] = j < n ? seq[j] : 0;
    return v;
  }
};

__device__ u32 finish_block(const ZhBlockDesc &d, const Out &o, u32 blk, u32 op, bool early_raw) {
  u32 const lane = lane_id(), n = d.n, last = (d.flags & ZH_F_LAST) ? 1u : 0u, body0 = blk + 3;
  u32 const body = op - body0;
  u32 const minGain = (n >> 6) + 2;
  u32 const maxC = n > minGain ? n - minGain : 0;
  if (!early_raw && body < maxC) {
    u32 const hdr = last + (2u << 1) + (body << 3);
    if (lane == 0) { o.put(blk, (u8)hdr); o.put(blk + 1, (u8)(hdr >> 8)); o.put(blk + 2, (u8)(hdr >> 16)); }
    return op;
  }
  u32 const hdr = last + (n << 3);
  wave_sync();
  if (lane == 0) { o.put(blk, (u8)hdr); o.put(blk + 1, (u8)(hdr >> 8)); o.put(blk + 2, (u8)(hdr >> 16)); }
  copy_bytes(o, body0, d.src, n);
  return body0 + n;
}

__device__ __forceinline__ void write_status(const ZhBlockDesc &d, u32 b, u32 total, u64 *item_size, u32 *item_status, u32 *blk_size) {
  if (lane_id() == 0) {
    if (d.flags & ZH_F_DIRECT) {
      item_size[d.item] = total;
      item_status[d.item] = total <= d.dst_cap ? ZH_ST_OK : ZH_ST_TOO_SMALL;
    } else {
      blk_size[b] = total <= d.dst_cap ? total : 0xFFFFFFFFu;
    }
  }
}

extern "C" __global__ __launch_bounds__(K2_THREADS) void zh_entropy_kernel(const ZhBlockDesc *__restrict__ blocks, ZhWorkspace ws, u32 window_log,
                                                                             u32 cfg_block_size, u64 *__restrict__ item_size,
                                                                             u32 *__restrict__ item_status, u32 *__restrict__ blk_size) {
  extern __shared__ __attribute__((aligned(16))) u8 smem_all[];
  // Two waves per block, each with its own copy of the LDS layout: wave 0 builds the literals
  // section, wave 1 (concurrently) the sequences section's merge / repcodes / codes / FSE
  // tables; after one barrier wave 1 places the sequence headers behind the literals and
  // finishes the block.  A block's latency is the longer of the two halves, not their sum.
  u32 const wave = threadIdx.x >> 6;
  u8 *const smem = smem_all + wave * K2_W1;
  u32 *const xch = (u32 *)(smem_all + OFF_MISC) + 56;  // wave 0 -> wave 1: literals end, early_raw
  u32 *sw = (u32 *)(smem + OFF_SW);
  u32 *misc = (u32 *)(smem + OFF_MISC);
  u32 *hist = (u32 *)(smem + OFF_HIST);
  u16 *hval = (u16 *)(smem + OFF_HVAL);
  u8 *hnb = smem + OFF_HNB;
  u8 *hbuf = smem + OFF_HBUF;
  HufNode *nodes = (HufNode *)(smem + OFF_NODES);
  u16 *stLL = (u16 *)(smem + OFF_ST_LL), *stOF = (u16 *)(smem + OFF_ST_OF), *stML = (u16 *)(smem + OFF_ST_ML);
  FseSym *symLL = (FseSym *)(smem + OFF_SYM), *symOF = symLL + SYM_OF, *symML = symLL + SYM_ML;
  u8 *tsym = smem + OFF_TSYM;
  s16 *norm = (s16 *)(smem + OFF_NORM);
  u8 *wts = smem + OFF_WTS;
  SerialScratch *scr = (SerialScratch *)(smem + OFF_SCR);

  u32 const b = blockIdx.x, lane = lane_id();
  ZhBlockDesc const d = blocks[b];
  u32 const n = d.n;
  if (n == 0) return;
  const u32 *meta = ws.meta(b);
  u32 const nseq_raw = meta[0], nlit = meta[1], rle = meta[2] == 1u, k1hist = meta[2] == ZH_META_K1HIST;
  Out const o{d.dst, d.dst_cap};
  if (wave == 0 && lane == 0) sw[0] = 0;  // (wave 1's SW overlaps wave 0's layout: never touched)
#ifdef ZH_STAMPS
  u64 stamp_prev = __builtin_amdgcn_s_memtime();
  u32 st[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif

  // ---- frame header (reference write_frame_header choices, no dict; checksum flag when asked)
  u32 pos = 0;
  if (d.flags & ZH_F_FIRST) {
    u64 const content = d.frame_size;
    bool const ss = content <= cfg_block_size;
    u32 fcs_flag, fcs_size;
    if (ss) {
      if (content < 256) { fcs_flag = 0; fcs_size = 1; }
      else if (content < 65536 + 256) { fcs_flag = 1; fcs_size = 2; }
      else if (content <= 0xFFFFFFFFull) { fcs_flag = 2; fcs_size = 4; }
      else { fcs_flag = 3; fcs_size = 8; }
    } else {
      if (content >= 256 && content < 65536 + 256) { fcs_flag = 1; fcs_size = 2; }
      else if (content <= 0xFFFFFFFFull) { fcs_flag = 2; fcs_size = 4; }
      else { fcs_flag = 3; fcs_size = 8; }
    }
    // Dictionary_ID of a formatted dictionary (raw content: none), libzstd's minimal size
    u32 const did = (d.flags & ZH_F_DICT) ? d.dict_id : 0u;
    u32 const didf = did == 0 ? 0u : did < 256 ? 1u : did < 65536 ? 2u : 3u;
    u32 const didn = didf == 3 ? 4u : didf;
    if (wave == 1 && lane == 0) {
      u32 p = 0;
      o.put(p++, 0x28); o.put(p++, 0xB5); o.put(p++, 0x2F); o.put(p++, 0xFD);
      o.put(p++, (u8)((fcs_flag << 6) | (ss ? 0x20 : 0) | ((d.flags & ZH_F_CHECKSUM) ? 0x04 : 0) | didf));
      if (!ss) o.put(p++, (u8)((window_log - 10) << 3));
      for (u32 k = 0; k < didn; k++) o.put(p++, (u8)(did >> (8 * k)));
      u64 v = fcs_size == 2 ? content - 256 : content;
      for (u32 k = 0; k < fcs_size; k++) o.put(p++, (u8)(v >> (8 * k)));
    }
    pos = 5 + (ss ? 0 : 1) + didn + fcs_size;
  }
  u32 const blk = pos;
  u32 const body0 = blk + 3;
  u32 const last = (d.flags & ZH_F_LAST) ? 1u : 0u;
  u32 total;
  bool early_raw = false, handoff = false;
  if (wave == 1 && lane == 0) ws.fsef(b)[ZH_FF_NEED] = 0;

  if (rle) {
    u32 const hdr = last + (1u << 1) + (n << 3);
    if (wave == 1 && lane == 0) { o.put(blk, (u8)hdr); o.put(blk + 1, (u8)(hdr >> 8)); o.put(blk + 2, (u8)(hdr >> 16)); o.put(blk + 3, d.src[0]); }
    total = blk + 4;
  } else {
    // (ZH_META_K1HIST: no sequences, the literals are the block's own bytes -- read from the
    // source -- and K1 counted their histogram)
    const u8 *lits = k1hist ? d.src : ws.lits(b);
    u64 *seq = ws.seq(b);
    u32 op = body0;
    // the literal histogram, both waves (wave 1 before its sequence work), into wave 0's hist
    if (nlit > ZH_COMPRESS_LITERALS_SIZE_MIN) {
      u32 *const hist0 = (u32 *)(smem_all + OFF_HIST);
      u32 const nl = nlit;
      if (k1hist) {
        // the sum of K1's per-wave sub-histograms, both waves (two bins per lane)
        const u32 *const kh = (const u32 *)(ws.lits(b) + ZH_K1_HIST_OFF);
        u32 const i = lane + 64u * wave, i2 = i + 128u;
        u32 s1 = 0, s2 = 0;
#pragma unroll
        for (u32 w = 0; w < ZH_K1_HIST_WAVES; w++) { s1 += kh[256u * w + i]; s2 += kh[256u * w + i2]; }
        hist0[i] = s1;
        hist0[i2] = s2;
      } else if (wave == 0) {
        for (u32 i = lane; i < 256; i += 64) hist0[i] = 0;
      }
      __syncthreads();
      // 16 literals per lane per load (lits is 16-B aligned), two loads per step, the next step's
      // loads issued before this step's LDS atomics
      auto load2 = [&](u32 i0, uint4 (&q)[2]) {
#pragma unroll
        for (u32 g = 0; g < 2; g++) {
          u32 const i = i0 + 16 * g;
          if (i + 16 <= nl) q[g] = *(const uint4 *)(lits + i);
          else {
            u32 t[4] = {0, 0, 0, 0};
            for (u32 k = 0; i + k < nl && k < 16; k++) t[k >> 2] |= (u32)lits[i + k] << (8 * (k & 3));
            q[g] = make_uint4(t[0], t[1], t[2], t[3]);
          }
        }
      };
      u32 const i00 = k1hist ? nl : 32 * lane + 2048 * wave;  // (K1's histogram: nothing to count)
      uint4 q[2];
      if (i00 < nl) load2(i00, q);
      for (u32 i0 = i00; i0 < nl; i0 += 4096) {
        uint4 qn[2];
#if ZH_HIST_PF
        if (i0 + 4096 < nl) load2(i0 + 4096, qn);
#endif
#pragma unroll
        for (u32 g = 0; g < 2; g++) {
          u32 const i = i0 + 16 * g;
          u32 const cnt = i < nl ? min(16u, nl - i) : 0u;
          u32 const w[4] = {q[g].x, q[g].y, q[g].z, q[g].w};
#pragma unroll
          for (u32 k = 0; k < 16; k++)
            if (k < cnt) atomicAdd(&hist0[(w[k >> 2] >> (8 * (k & 3))) & 255u], 1u);
        }
#if !ZH_HIST_PF
        if (i0 + 4096 < nl) load2(i0 + 4096, qn);
#endif
        q[0] = qn[0];
        q[1] = qn[1];
      }
      __syncthreads();
    }
    // ======================= literals section (ZSTD_compressLiterals), wave 0 =======================
    if (wave == 0) {
      u32 const nl = nlit;
      u32 const minGain = (nl >> 6) + 2;
      u32 const lhSize = 3 + (nl >= 1024) + (nl >= 16384);
      bool const single = nl < 256;
      u32 cLit = 0, hsz = 0, huffLog = 0;
      u32 *ssz = misc + 8;  // per-stream byte sizes (LDS, wave-uniform)
      if (nl > ZH_COMPRESS_LITERALS_SIZE_MIN) {
        u32 mx = 0, lg = 0;
        for (u32 i = lane; i < 256; i += 64) { u32 c = hist[i]; if (c) mx = max(mx, i); lg = max(lg, c); }
        u32 const maxSV = wave_max(mx), largest = wave_max(lg);
        if (largest == nl) cLit = 1;
        else if (largest <= (nl >> 7) + 4) cLit = 0;
        else {
          ZH_STAMP(0);  // literal histogram
          u32 hl = fse_optimal_table_log(11, nl, maxSV, 1);
          hl = huf_build_ctable_par(nodes, hval, hnb, hist, maxSV, hl, scr);
          ZH_STAMP(11);  // Huffman tree (parallel part)
          huffLog = hl;
          hsz = hl ? huf_write_ctable_wave(hbuf, wts, hnb, maxSV, hl, (u16 *)(smem + OFF_W_ST), (FseSym *)(smem + OFF_W_SYM), smem + OFF_W_TSYM,
                                           (s16 *)(smem + OFF_W_NORM), scr)
                   : 0;
          ZH_STAMP(1);  // Huffman tree + header (serial)
          if (hsz && hsz + 12 < nl) {
            // stream sizes: sum of code lengths per stream (+ end mark)
            u32 const seg = (nl + 3) / 4;
            u32 ns = single ? 1 : 4;
            if (!single && nl < 12) ns = 0;
            u32 cs = single ? 0 : 6;
            for (u32 k = 0; k < ns; k++) {
              u32 a = single ? 0 : k * seg, e = single ? nl : (k < 3 ? (k + 1) * seg : nl);
              u32 bits = 0;
              for (u32 i = a + lane; i < e; i += 64) bits += hnb[lits[i]];
              bits = wave_sum(bits);
              ssz[k] = (bits + 1 + 7) >> 3;
              cs += ssz[k];
            }
            if (ns) {
              u32 const tot = hsz + cs;
              cLit = (tot >= nl - 1) ? 0 : tot;
            }
          }
        }
      }
      ZH_STAMP(2);  // stream sizes
      if (cLit == 0 || cLit >= nl - minGain) {
        // raw literals
        u32 const fl = 1 + (nl > 31) + (nl > 4095);
        u32 v = fl == 1 ? (nl << 3) : fl == 2 ? ((1u << 2) + (nl << 4)) : ((3u << 2) + (nl << 4));
        // the sequences section adds >= 1 byte: past the block's minGain the block is
        // emitted raw whatever the sequences cost, so skip writing this body at all
        u32 const bmaxC = n > (n >> 6) + 2 ? n - ((n >> 6) + 2) : 0u;
        early_raw = fl + nl + 1 >= bmaxC;
        if (!early_raw) {
          if (lane < fl) o.put(op + lane, (u8)(v >> (8 * lane)));
          copy_bytes(o, op + fl, lits, nl);
        }
        op += fl + nl;
      } else if (cLit == 1) {
        u32 const fl = 1 + (nl > 31) + (nl > 4095);
        u32 v = fl == 1 ? (1 + (nl << 3)) : fl == 2 ? (1 + (1u << 2) + (nl << 4)) : (1 + (3u << 2) + (nl << 4));
        if (lane < fl) o.put(op + lane, (u8)(v >> (8 * lane)));
        if (lane == 0) o.put(op + fl, lits[0]);
        op += fl + 1;
      } else {
        u64 lhc;
        if (lhSize == 3) lhc = 2 + ((u64)(!single) << 2) + ((u64)nl << 4) + ((u64)cLit << 14);
        else if (lhSize == 4) lhc = 2 + (2u << 2) + ((u64)nl << 4) + ((u64)cLit << 18);
        else lhc = 2 + (3u << 2) + ((u64)nl << 4) + ((u64)cLit << 22);
        if (lane < lhSize) o.put(op + lane, (u8)(lhc >> (8 * lane)));
        op += lhSize;
        for (u32 i = lane; i < hsz; i += 64) o.put(op + i, hbuf[i]);
        op += hsz;
        u32 const seg = (nl + 3) / 4;
        u32 const ns = single ? 1 : 4;
        if (!single) {
          if (lane < 6) { u32 k = lane >> 1; o.put(op + lane, (u8)(ssz[k] >> (8 * (lane & 1)))); }
          op += 6;
        }
        for (u32 k = 0; k < ns; k++) {
          u32 a = single ? 0 : k * seg, e = single ? nl : (k < 3 ? (k + 1) * seg : nl);
          BitSink bs{op, 0};
          // symbols from e-1 down to a, 8 per lane per append (codes paired into <= 22-bit fields);
          // a lane's 8 symbols are the bytes [A, A + 8), A = e - 8 - base - 8 lane, read as three
          // aligned dwords, the next append's in flight while this one is encoded
          const u32 *l32 = (const u32 *)lits;
          auto ld3 = [&](u32 base_, u32 (&dw)[3]) {
            int const A = (int)e - 8 - (int)base_ - 8 * (int)lane;
            u32 const w0 = A > (int)a ? (u32)A >> 2 : a >> 2;
            dw[0] = l32[w0]; dw[1] = l32[w0 + 1]; dw[2] = l32[w0 + 2];
          };
          u32 dn[3];
          ld3(0, dn);
          for (u32 base = 0; base < e - a; base += 512) {
            u32 const dw[3] = {dn[0], dn[1], dn[2]};
            if (base + 512 < e - a) ld3(base + 512, dn);
            int const A = (int)e - 8 - (int)base - 8 * (int)lane;
            u32 const sh = (u32)A & 3u;
            u32 const lo = __builtin_amdgcn_alignbyte(dw[1], dw[0], sh), hi = __builtin_amdgcn_alignbyte(dw[2], dw[1], sh);
            bool const full = A >= (int)a;  // all 8 bytes inside the stream (else: byte loads)
            u32 v[4], nb[4];
#pragma unroll
            for (u32 f = 0; f < 4; f++) {
              u32 const j0 = base + 8 * lane + 2 * f, j1 = j0 + 1;
              u32 c0 = 0, n0 = 0, c1 = 0, n1 = 0;
              // symbol jj = 2f (+1) of the lane is byte 7 - jj of (lo, hi)
              u32 const b0 = full ? ((f < 2 ? hi : lo) >> (8 * (3 - 2 * (f & 1)))) & 255u : 0u;
              u32 const b1 = full ? ((f < 2 ? hi : lo) >> (8 * (2 - 2 * (f & 1)))) & 255u : 0u;
              if (j0 < e - a) { u32 const c = full ? b0 : lits[e - 1 - j0]; c0 = hval[c]; n0 = hnb[c]; }
              if (j1 < e - a) { u32 const c = full ? b1 : lits[e - 1 - j1]; c1 = hval[c]; n1 = hnb[c]; }
              v[f] = c0 | (c1 << n0);
              nb[f] = n0 + n1;
            }
            sink_append<4>(bs, o, sw, v, nb);
          }
          sink_close(bs, o, sw);
          op = bs.pos;
        }
      }
      (void)huffLog;
      ZH_STAMP(3);  // literal streams
      if (lane == 0) { xch[0] = op; xch[1] = early_raw ? 1u : 0u; }
    }

    // ======================= sequences section, wave 1 =======================
    u32 nbSeq = 0, hpos = 0, typesw_ = 0, logLL = 0, logOF = 0, logML = 0;
    if (wave == 1) {
    // One pass over K1's records: literal lengths from the cumulative counts, same-offset
    // continuations merged into their run head (DPP scan), and each closed run handed on as
    // a sequence (ds_permute compaction, a chunk's runs + the one left open by the chunk
    // before) to the repcode / code / histogram step, which writes the merged records in
    // place (record = ll | mlBase << 17 | offBase << 34 | llCode << 51 | mlCode << 57).
    u32 *hLL = hist, *hOF = hist + 64, *hML = hist + 128;
    for (u32 i = lane; i < 192; i += 64) hist[i] = 0;
    wave_sync();
    {
      // Repcode resolution, lane-parallel.  With o_i the offset of sequence i:
      //  - r0 before i is o_{i-1} (every zstd repcode update leaves the used offset in rep[0]);
      //  - rep[1] survives sequence j only when j repeats rep[0] with LL > 0, otherwise it
      //    becomes rep[0]-before-j: r1_i = r0_m for the last such m < i;
      //  - rep[2] survives j when j used rep[0] (LL > 0) or rep[1], otherwise it becomes
      //    rep[1]-before-j: r2_i = r1_m for the last such m < i.
      // (oracle/zstd_oracle.c orc_resolve_repcodes is the serial form.)
      u32 cr0 = 1, cr1 = 4, cr2 = 8;  // reps before the batch's first sequence
      if (!(d.flags & ZH_F_FIRST) || (d.flags & ZH_F_DICT)) { cr0 = cr1 = cr2 = 0; }  // dictionary frames: its repcodes never referenced
      u64 const below = (1ull << lane) - 1ull;
      CodeTabs ct;
      ct.load();
      // sequences nbSeq + [0, m) in lanes [0, m)
      auto sequences_c = [&](u32 m, u32 ll, u32 ml, u32 off, u32 llc, u32 mlc) {
        u32 const i = nbSeq + lane;
        bool const valid = lane < m;
        u32 r0 = wave_shr1(off);
        if (lane == 0) r0 = cr0;
        bool const keep1 = ll > 0 && off == r0;
        u64 const nk1 = __ballot(valid && !keep1);
        u64 const m1 = nk1 & below;
        u32 const src1 = m1 ? 63u - (u32)__builtin_clzll(m1) : 0u;
        u32 const t1 = __shfl(r0, src1, 64);
        u32 const r1 = m1 ? t1 : cr1;
        bool const keep2 = (ll > 0 && off == r0) || off == r1;
        u64 const nk2 = __ballot(valid && !keep2);
        u64 const m2 = nk2 & below;
        u32 const src2 = m2 ? 63u - (u32)__builtin_clzll(m2) : 0u;
        u32 const t2 = __shfl(r1, src2, 64);
        u32 const r2 = m2 ? t2 : cr2;
        u32 ob;
        if (ll) ob = off == r0 ? 1u : off == r1 ? 2u : off == r2 ? 3u : off + 3;
        else ob = off == r1 ? 1u : off == r2 ? 2u : (r0 > 1 && off == r0 - 1) ? 3u : off + 3;
        // reps after the last sequence
        u32 const lastLane = m - 1;
        u32 const n1 = keep1 ? r1 : r0, n2 = keep2 ? r2 : r1;
        cr0 = lane_value(off, lastLane);
        cr1 = lane_value(n1, lastLane);
        cr2 = lane_value(n2, lastLane);
        u32 const mlb = ml - 3;
        if (valid) {
          atomicAdd(&hLL[llc], 1u);
          atomicAdd(&hML[mlc], 1u);
          atomicAdd(&hOF[highbit32(ob)], 1u);
          // + the LL / ML codes in the spare top bits (ob < 2^17: offsets stay inside the block)
          seq[i] = (u64)ll | ((u64)mlb << 17) | ((u64)ob << 34) | ((u64)llc << 51) | ((u64)mlc << 57);
        }
        nbSeq += m;
      };
      auto sequences = [&](u32 m, u32 ll, u32 ml, u32 off) { sequences_c(m, ll, ml, off, ct.ll_code(ll), ct.ml_code(ml - 3)); };
      u32 carryCum = 0, carryOff = 0, openLL = 0, openMl = 0, openOff = 0;
      bool open = false;
      RecRing ring;  // records loaded RING_DEPTH chunks ahead (a chunk writes only indices < its end)
      ring.init(seq, nseq_raw, lane);
#if ZH_K2_PAIR
      // Two chunks per iteration: the second chunk's run analysis, its permutes and both
      // chunks' code lookups depend only on records (not on the first chunk's results), so
      // their LDS round trips overlap; the open run and the repcodes pass on in order.
      // fast: every record of the chunk opens its own run (no same-offset continuation, the
      // common case): the run sums, their scan and the permutes reduce to the records themselves
      // and a shift by the open run (DPP)
      struct Chunk { u32 ll, off, runMl, incl, cum; u64 hm; bool head, fast; };
      auto analyse = [&](u64 rec, u32 i, u32 pc0, u32 po0, Chunk &c) {
        bool const valid = i < nseq_raw;
        u32 const cum = (u32)(rec & 0x1FFFFu), ce = (u32)((rec >> 24) & 0xFFFu);
        u32 const ml = (u32)((rec >> 17) & 0x7Fu) + ce, off = (u32)((rec >> 36) & 0x1FFFFu);
        u32 pc = wave_shr1(cum), po = wave_shr1(off);
        if (lane == 0) { pc = pc0; po = po0; }
        u32 const ll = cum - pc - ce;
        bool const flag = valid && i > 0 && ll == 0 && off == po;
        bool const head = valid && !flag;
        u64 const hm = __ballot(head);
        u32 const mlv = valid ? ml : 0u;
        c.fast = hm == __ballot(valid);
        if (c.fast) {
          c.runMl = mlv;
          c.incl = 0;  // (advance reads it only before the first head: lane 0 is one)
        } else {
          u32 const incl = wave_scan_incl(mlv);
          u64 const headBitsAfter = hm & ~((lane == 63) ? ~0ull : ((2ull << lane) - 1));
          u32 const runEnd = headBitsAfter ? (u32)__builtin_ctzll(headBitsAfter) - 1u : 63u;
          u32 const inclEnd = (u32)__builtin_amdgcn_ds_bpermute((int)(runEnd << 2), (int)incl);
          c.runMl = inclEnd - (incl - mlv);
          c.incl = incl;
        }
        c.ll = ll; c.off = off; c.cum = cum; c.hm = hm; c.head = head;
      };
      // the chunk's runs to lanes hp + rank (ds_permute, as in the single-chunk step below)
      auto gather = [&](const Chunk &c, u32 hp, u32 &sll, u32 &sml, u32 &soff) {
        if (c.fast) {  // lane + hp (lane 0 takes the open run in advance)
          sll = hp ? wave_shr1(c.ll) : c.ll;
          sml = hp ? wave_shr1(c.runMl) : c.runMl;
          soff = hp ? wave_shr1(c.off) : c.off;
          return;
        }
        u32 const hcount = (u32)__popcll(c.hm), rank = (u32)__popcll(c.hm & below);
        u32 const dest = c.head ? rank + hp : (hcount + hp + (lane - rank)) & 63u;
        sll = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)c.ll);
        sml = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)c.runMl);
        soff = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)c.off);
      };
      // open-run state through the chunk; returns the sequences it closes (lanes [0, m))
      auto advance = [&](const Chunk &c, u32 &sll, u32 &sml, u32 &soff) {
        u32 const hcount = (u32)__popcll(c.hm);
        u32 const firstH = c.hm ? (u32)__builtin_ctzll(c.hm) : 64u;
        openMl += firstH ? lane_value(c.incl, firstH - 1u) : 0u;
        if (!hcount) return 0u;
        u32 const hp = open ? 1u : 0u;
        if (hp && lane == 0) { sll = openLL; sml = openMl; soff = openOff; }
        int const lastH = 63 - __builtin_clzll(c.hm);
        openLL = lane_value(c.ll, (u32)lastH);
        openOff = lane_value(c.off, (u32)lastH);
        openMl = lane_value(c.runMl, (u32)lastH);
        open = true;
        return hp + hcount - 1;
      };
      for (u32 base = 0; base < nseq_raw; base += 128) {
        bool const two = base + 64 < nseq_raw;  // (then chunk A is full)
        u64 const recA = ring.next(seq, nseq_raw, base + lane);
        u64 const recB = two ? ring.next(seq, nseq_raw, base + 64 + lane) : 0ull;
        Chunk A, B;
        analyse(recA, base + lane, carryCum, carryOff, A);
        u32 const cA = lane_value(A.cum, 63), oA = lane_value(A.off, 63);
        if (two) analyse(recB, base + 64 + lane, cA, oA, B);
        u32 const lastLane = two ? min(63u, nseq_raw - 1 - (base + 64)) : min(63u, nseq_raw - 1 - base);
        carryCum = two ? lane_value(B.cum, lastLane) : lane_value(A.cum, lastLane);
        carryOff = two ? lane_value(B.off, lastLane) : lane_value(A.off, lastLane);
        u32 const hpA = open ? 1u : 0u, hpB = (open || A.hm) ? 1u : 0u;
        u32 aL = 0, aM = 0, aO = 0, bL = 0, bM = 0, bO = 0;
        if (A.hm) gather(A, hpA, aL, aM, aO);
        if (two && B.hm) gather(B, hpB, bL, bM, bO);
        u32 const mA = advance(A, aL, aM, aO);
        u32 const aLc = ct.ll_code(aL), aMc = ct.ml_code(aM - 3);
        u32 mB = 0, bLc = 0, bMc = 0;
        if (two) {
          mB = advance(B, bL, bM, bO);
          bLc = ct.ll_code(bL);
          bMc = ct.ml_code(bM - 3);
        }
        if (mA) sequences_c(mA, aL, aM, aO, aLc, aMc);
        if (mB) sequences_c(mB, bL, bM, bO, bLc, bMc);
      }
#else
      for (u32 base = 0; base < nseq_raw; base += 64) {
        u32 const i = base + lane;
        bool const valid = i < nseq_raw;
        u64 const rec = ring.next(seq, nseq_raw, i);
        // K1 record: the walk's literals before the match | length | catch-up | offset; the
        // catch-up e moves e bytes of the literal run into the match (zh_lz.hip)
        u32 const cum = (u32)(rec & 0x1FFFFu), ce = (u32)((rec >> 24) & 0xFFFu);
        u32 const ml = (u32)((rec >> 17) & 0x7Fu) + ce, off = (u32)((rec >> 36) & 0x1FFFFu);
        u32 pc = wave_shr1(cum), po = wave_shr1(off);
        if (lane == 0) { pc = carryCum; po = carryOff; }
        u32 const ll = cum - pc - ce;
        bool const flag = valid && i > 0 && ll == 0 && off == po;
        bool const head = valid && !flag;
        u64 const hm = __ballot(head);
        // run sums of ml: inclusive DPP scan, each head reads the scan at its run's last lane in
        // this chunk (one ds_bpermute); lanes before the first head extend the open run
        u32 const mlv = valid ? ml : 0u;
        u32 const incl = wave_scan_incl(mlv);
        u64 const headBitsAfter = hm & ~((lane == 63) ? ~0ull : ((2ull << lane) - 1));
        u32 const runEnd = headBitsAfter ? (u32)__builtin_ctzll(headBitsAfter) - 1u : 63u;
        u32 const inclEnd = (u32)__builtin_amdgcn_ds_bpermute((int)(runEnd << 2), (int)incl);
        u32 const runMl = inclEnd - (incl - mlv);  // (heads: the run's ml within this chunk)
        u32 const hcount = (u32)__popcll(hm);
        u32 const firstH = hm ? (u32)__builtin_ctzll(hm) : 64u;
        openMl += firstH ? lane_value(incl, firstH - 1u) : 0u;
        if (hcount) {
          // sequences of this step: the run left open before (if any), then this chunk's runs
          // but its last (which stays open); heads go to lanes hp + rank, the other lanes to
          // the lanes above (a bijection, as ds_permute needs)
          u32 const hp = open ? 1u : 0u;
          u32 const rank = (u32)__popcll(hm & below);
          u32 const dest = head ? rank + hp : (hcount + hp + (lane - rank)) & 63u;
          u32 sll = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)ll);
          u32 sml = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)runMl);
          u32 soff = (u32)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)off);
          if (hp && lane == 0) { sll = openLL; sml = openMl; soff = openOff; }
          int const lastH = 63 - __builtin_clzll(hm);
          openLL = lane_value(ll, (u32)lastH);
          openOff = lane_value(off, (u32)lastH);
          openMl = lane_value(runMl, (u32)lastH);
          open = true;
          u32 const m = hp + hcount - 1;
          if (m) sequences(m, sll, sml, soff);
        }
        u32 const lastLane = min(63u, nseq_raw - 1 - base);
        carryCum = lane_value(cum, lastLane);
        carryOff = lane_value(off, lastLane);
      }
#endif
      if (open) sequences(1, openLL, openMl, openOff);
      wave_sync();
    }
    ZH_STAMP(4);  // merge + repcodes + codes + histograms
    if (nbSeq > 0) {
      ZH_STAMP(5);
      // tables: LL, OF, ML (ZSTD_selectEncodingType for strategy dfast + ZSTD_buildCTable)
      u64 const rec0 = seq[0], recL = seq[nbSeq - 1];
      u32 hposw = 0, typesw = 0, logsw[3];
      {
        // ZSTD_selectEncodingType (dfast) + normalisation + NCount header, wave-parallel
        // (lane = symbol; every value below is wave-uniform)
        u32 const first_code[3] = {ll_code((u32)(rec0 & 0x1FFFFu)), highbit32((u32)(rec0 >> 34) & 0x1FFFFu), ml_code((u32)((rec0 >> 17) & 0x1FFFFu))};
        u32 const last_code[3] = {ll_code((u32)(recL & 0x1FFFFu)), highbit32((u32)(recL >> 34) & 0x1FFFFu), ml_code((u32)((recL >> 17) & 0x1FFFFu))};
        for (int t = 0; t < 3; t++) {
          u16 *st = t == 0 ? stLL : t == 1 ? stOF : stML;
          FseSym *sy = t == 0 ? symLL : t == 1 ? symOF : symML;
          u32 *cnt = hist + 64 * t;
          u32 const maxSym = t == 0 ? 35 : t == 1 ? 31 : 52;
          u32 const fseLog = t == 1 ? 8 : 9, defLog = t == 1 ? 5 : 6, defMax = t == 0 ? 35 : t == 1 ? 28 : 52;
          const s16 *defNorm = t == 0 ? c_LL_def : t == 1 ? c_OF_def : c_ML_def;
          u32 c = lane <= maxSym ? cnt[lane] : 0u;
          u64 const nz = __ballot(c != 0);
          u32 const mx = nz ? 63u - (u32)__builtin_clzll(nz) : 0u;
          u32 const mostFrequent = wave_max(c);
          bool const defAllowed = (t == 1) ? (mx <= 28) : true;
          u32 type;
          if (mostFrequent == nbSeq) type = (defAllowed && nbSeq <= 2) ? 0 : 1;
          else if (defAllowed && ((nbSeq < (1u << defLog)) || (mostFrequent < (nbSeq >> (defLog - 1))))) type = 0;
          else type = 2;
          u32 bmax = 0, blog = 0;
          if (type == 1) {
            u32 const fc = first_code[t];
            if (lane == 0) {
              st[0] = 0; st[1] = 0;
              sy[fc].dNb = 0; sy[fc].dFS = 0;
              hbuf[hposw] = (u8)fc;
            }
            hposw++;
            logsw[t] = 0;
          } else if (type == 0) {
            if (lane <= defMax) norm[lane] = defNorm[lane];
            bmax = defMax; blog = defLog;
            logsw[t] = defLog;
          } else {
            u32 nb1 = nbSeq;
            u32 const tl = fse_optimal_table_log(fseLog, nbSeq, mx, 2);
            u32 const lc = last_code[t];
            if (lane_value(c, lc) > 1) {
              if (lane == lc) c--;
              nb1--;
            }
            int const nv = fse_normalize_wave(norm, tl, c, nb1, mx, nb1 >= 2048, lane, scr->cumul);
            hposw += fse_write_ncount_wave(hbuf + hposw, nv, mx, tl, lane);
            bmax = mx; blog = tl;
            logsw[t] = tl;
          }
          typesw |= type << (6 - 2 * t);
          wave_sync();
          if (type != 1) fse_build_ctable_par(st, sy, tsym, norm, bmax, blog, scr);
          wave_sync();
        }
        if (lane == 0) {
          misc[0] = hposw;
          misc[1] = typesw;
          misc[2] = logsw[0]; misc[3] = logsw[1]; misc[4] = logsw[2];
        }
      }
      wave_sync();
      hpos = misc[0];
      typesw_ = misc[1];
      logLL = misc[2]; logOF = misc[3]; logML = misc[4];
      ZH_STAMP(6);  // FSE tables (serial)

      // hand-off: the FSE state chains run in zh_fse_chain_kernel (lanes = blocks x
      // tables, so many serial chains share a wave) and the bitstream is packed by
      // zh_seq_pack_kernel, which also finishes the block
      u8 *fz = ws.fse(b);
      {
        const u32 *sL = (const u32 *)stLL, *sO = (const u32 *)stOF, *sM = (const u32 *)stML;
        for (u32 i = lane; i < 256; i += 64) ((u32 *)(fz + ZH_FT_STLL))[i] = sL[i];
        for (u32 i = lane; i < 128; i += 64) ((u32 *)(fz + ZH_FT_STOF))[i] = sO[i];
        for (u32 i = lane; i < 256; i += 64) ((u32 *)(fz + ZH_FT_STML))[i] = sM[i];
        if (lane < 36) ((FseSym *)(fz + ZH_FT_SYLL))[lane] = symLL[lane];
        if (lane < 32) ((FseSym *)(fz + ZH_FT_SYOF))[lane] = symOF[lane];
        if (lane < 53) ((FseSym *)(fz + ZH_FT_SYML))[lane] = symML[lane];
      }
    }
    if (wave == 1 && lane == 0) xch[2] = nbSeq;
    }  // wave 1
    __syncthreads();  // the literals section is written; its end and early_raw are in xch
    if (xch[1] != 0) {  // raw block (the literals alone pass its minGain): both waves copy half
      u32 const h = (n / 2) & ~63u;
      if (wave == 0) copy_bytes(o, body0, d.src, h);
      else copy_bytes(o, body0 + h, d.src + h, n - h);
    } else if (u32 const ns = xch[2]; ns > 0) {
      // the codes in encoding order (step k = ns-1-i) in the chain layout (zh_common.h), both
      // waves (wave 0 is otherwise idle here): a lane per 16-step run (contiguous in the
      // layout), its 16 records, three 16-byte stores
      u32 const k3L = ZH_K3_SEGLEN(ns), k3m = zh_k3_magic(k3L);
      u8 *const cb = ws.lits(b) + ZH_K3_CODES(k3L);
      for (u32 k0 = 16u * (lane + 64u * wave); k0 < ns; k0 += 16u * K2_THREADS) {
        u64 r[16];
#pragma unroll
        for (u32 q = 0; q < 16; q++) r[q] = k0 + q < ns ? seq[ns - 1 - (k0 + q)] : 0ull;
        u32 wl[4] = {0, 0, 0, 0}, wo[4] = {0, 0, 0, 0}, wm[4] = {0, 0, 0, 0};
#pragma unroll
        for (u32 q = 0; q < 16; q++) {
          u32 const ob = (u32)(r[q] >> 34) & 0x1FFFFu;
          wl[q >> 2] |= ((u32)(r[q] >> 51) & 63u) << (8 * (q & 3));
          wo[q >> 2] |= (ob ? highbit32(ob) : 0u) << (8 * (q & 3));
          wm[q >> 2] |= ((u32)(r[q] >> 57)) << (8 * (q & 3));
        }
        u32 const x0 = zh_k3_index(k0, 0, k3L, k3m);
        *(uint4 *)(cb + x0) = make_uint4(wl[0], wl[1], wl[2], wl[3]);
        *(uint4 *)(cb + x0 + ZH_K3_TSTRIDE) = make_uint4(wo[0], wo[1], wo[2], wo[3]);
        *(uint4 *)(cb + x0 + 2u * ZH_K3_TSTRIDE) = make_uint4(wm[0], wm[1], wm[2], wm[3]);
      }
    }
    if (wave == 1) {
      op = xch[0];
      early_raw = xch[1] != 0;
      if (!early_raw) {
        // nbSeq header, then (with sequences) the table types and NCount headers
        if (nbSeq < 128) { if (lane == 0) o.put(op, (u8)nbSeq); op += 1; }
        else if (nbSeq < ZH_LONGNBSEQ) { if (lane == 0) { o.put(op, (u8)((nbSeq >> 8) + 0x80)); o.put(op + 1, (u8)nbSeq); } op += 2; }
        else { if (lane == 0) { o.put(op, 0xFF); o.put(op + 1, (u8)(nbSeq - ZH_LONGNBSEQ)); o.put(op + 2, (u8)((nbSeq - ZH_LONGNBSEQ) >> 8)); } op += 3; }
        if (nbSeq > 0) {
          if (lane == 0) o.put(op, (u8)typesw_);
          op += 1;
          for (u32 i = lane; i < hpos; i += 64) o.put(op + i, hbuf[i]);
          op += hpos;
          // (the codes in encoding order: both waves, above)
          // hand-off: the FSE state chains run in zh_fse_chain_kernel and the bitstream is
          // packed by zh_seq_pack_kernel, which also finishes the block
          u32 *ff = ws.fsef(b);
          if (lane == 0) {
            ff[ZH_FF_NBSEQ] = nbSeq; ff[ZH_FF_OP] = op; ff[ZH_FF_BLK] = blk;
            ff[ZH_FF_LOGS] = logLL | (logOF << 8) | (logML << 16);
            ff[ZH_FF_NEED] = 1;
          }
          handoff = true;
        }
      }
      if (early_raw) {
        u32 const hdr = last + (n << 3);
        if (lane == 0) { o.put(blk, (u8)hdr); o.put(blk + 1, (u8)(hdr >> 8)); o.put(blk + 2, (u8)(hdr >> 16)); }
        total = body0 + n;
      } else if (!handoff) {
        total = finish_block(d, o, blk, op, false);
      }
    }
  }
  ZH_STAMP(8);  // tail (raw copy etc.)
#ifdef ZH_STAMPS
  if (lane == 0) {  // wave 0: the literal phases, wave 1: the rest
    u32 *dbg = ws.dbg(b);
    if (wave == 0) { for (int k = 0; k < 4; k++) dbg[6 + k] = st[k]; dbg[42] = st[11]; }
    else { for (int k = 4; k < 9; k++) dbg[6 + k] = st[k]; dbg[17] = st[9]; dbg[18] = st[10]; dbg[19] = nseq_raw; }
  }
#endif
  if (wave == 1 && !handoff) write_status(d, b, total, item_size, item_status, blk_size);
}

// ======================= FSE state chains (K3) =======================
// One wave per block (K3_WAVES per workgroup).  Lane t * K3_SEGS + g runs segment g of table
// t's (LL, OF, ML) chain: encoding step e (e >= 1) encodes sequence nbSeq-1-e from the state
// the previous step left (step 0 is FSE_initCState2 with the last sequence's code).  The state
// before each step goes to the block's literal area (free by now) as u16, the codes come from
// pass B of the entropy kernel, both in the segment-interleaved chain layout (zh_common.h:
// each 16-step batch of the 63 segments is one contiguous run); the final states go to the
// fse fields.
//
// A chain is serial, but its step map s -> stT[(s >> nb) + dFS] is many-to-one (a symbol with
// normalised count c leaves at most c states), so two trajectories that start apart merge
// within a few dozen steps and then never part.  Segment g > 0 therefore starts from a guess
// (its first state after K3_WARM warm-up steps from an arbitrary state) and the segments run
// in parallel; then, in Jacobi rounds, every segment whose entry differs from its left
// neighbour's exit reruns from the right entry until its new trajectory meets the stored one
// (from there on every state is already right).  The states written are exactly the serial
// chain's.  The kernel's time is a block's longest segment, not its whole chain.
constexpr u32 K3_SEGS = ZH_K3_SEGS;  // 3 x 21 x ZH_K3_W lanes
constexpr u32 K3_W = ZH_K3_W;        // waves per block
#ifndef ZH_K3_OCC
#define ZH_K3_OCC 8  // minimum waves per SIMD the chain kernel is compiled for (8: <= 64 VGPRs)
#endif
#ifndef ZH_K3_WARM
#define ZH_K3_WARM 128
#endif
constexpr u32 K3_WARM = ZH_K3_WARM;  // warm-up steps before a segment's first step (64 -> 128: entropy
                                     // 3.05 -> 3.02 ms at 16,384 blocks, 0.775 -> 0.75 at 2,048)
constexpr u32 K3_WAVES = K3_W == 1 ? 4 : K3_W;  // waves per workgroup (the CU holds at most 16 workgroups)
constexpr u32 K3_BPW = K3_WAVES / K3_W;          // blocks per workgroup
constexpr u32 K3_TAB_STRIDE = (ZH_FSE_TAB_BYTES + 15) & ~15u;
constexpr u32 K3_LDS = K3_BPW * K3_TAB_STRIDE + 64;  // + the workgroup's exchange words (K3_W > 1)
constexpr u32 K3_BATCH = 16;   // steps per code load / state store
constexpr u32 K3_TABW = ZH_FSE_TAB_BYTES / 4;

// K3 of block bb (K3_W waves; the caller checked that the block needs it); smem = the block's
// K3_TAB_STRIDE bytes of LDS, xw = the workgroup's exchange words (K3_W > 1); lane = the
// thread's index among the block's K3_W * 64 (lane t * K3_SEGS + g runs segment g of table t)
__device__ __forceinline__ void k3_chain(ZhWorkspace ws, u32 bb, u8 *smem, u32 lane, u32 *xw) {
#ifdef ZH_STAMPS
  u64 const k3pre = __builtin_amdgcn_s_memtime();
  u64 const k3rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  u32 *ff = ws.fsef(bb);
  {
    const u32 *src = (const u32 *)ws.fse(bb);
    constexpr u32 NT = 64 * K3_W;
    u32 v[(K3_TABW + NT - 1) / NT];
#pragma unroll
    for (u32 q = 0; q < (K3_TABW + NT - 1) / NT; q++) v[q] = NT * q + lane < K3_TABW ? src[NT * q + lane] : 0u;
#pragma unroll
    for (u32 q = 0; q < (K3_TABW + NT - 1) / NT; q++)
      if (NT * q + lane < K3_TABW) ((u32 *)smem)[NT * q + lane] = v[q];
  }
  if constexpr (K3_W == 1) {
    // the tables are this wave's own: LDS executes one wave's operations in order
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
  u32 const t = min(lane / K3_SEGS, 2u), g = lane - K3_SEGS * t;  // lanes >= 3 K3_SEGS: an empty segment
  u32 const nbSeq = ff[ZH_FF_NBSEQ];
  const u16 *stT = (const u16 *)(smem + (t == 0 ? ZH_FT_STLL : t == 1 ? ZH_FT_STOF : ZH_FT_STML));
  const FseSym *syT = (const FseSym *)(smem + (t == 0 ? ZH_FT_SYLL : t == 1 ? ZH_FT_SYOF : ZH_FT_SYML));
  // chain layout (zh_common.h): batch k of this lane's segment at element (SLOTS k + slot) * 16
  u32 const seglen = ZH_K3_SEGLEN(nbSeq), nk = seglen / K3_BATCH;
  u16 *const gst = (u16 *)ws.lits(bb);                          // states
  const u8 *const cbase = ws.lits(bb) + ZH_K3_CODES(seglen);    // codes
  // this lane's slot and the slot of the segment before (warm-up codes); slots past 3 K3_SEGS exist
  // in the layout and are never read by the packing kernel
  u32 const ln = lane < 3 * K3_SEGS ? ZH_K3_SLOT(t, g) : lane, lnp = ZH_K3_SLOT(t, g - 1u);
  // element of batch k (16 steps) of a slot's segment
  auto at = [&](u32 k, u32 slot) { return ((k * K3_BATCH / ZH_K3_RUN) * ZH_K3_SLOTS + slot) * ZH_K3_RUN + (k * K3_BATCH) % ZH_K3_RUN; };
  auto codes_at = [&](u32 k, u32 slot) { return *(const uint4 *)(cbase + at(k, slot)); };  // batch k's 16 codes
  u32 const a = lane < 3 * K3_SEGS ? g * seglen : 3u * K3_SEGS * seglen;  // first step (lane 63: none)
  auto init_state = [&](u32 code) {  // FSE_initCState2
    FseSym const tr = syT[code];
    u32 const nb = (tr.dNb + (1u << 15)) >> 16;
    return (u32)stT[(((nb << 16) - tr.dNb) >> nb) + tr.dFS];
  };
  auto step = [&](u32 s, u32 code, bool live) {
    FseSym const tr = syT[code];
    u32 const nb = (s + tr.dNb) >> 16;
    u32 const nx = stT[min((s >> nb) + (u32)tr.dFS, 1023u)];
    return live ? nx : s;
  };
  // entry guess: segment 0 the exact initial state, others the state after the last K3_WARM
  // steps of the segment before, run from an arbitrary state (their codes: K3_WARM / 16
  // 16-byte loads issued together)
  u32 entry;
  if (a == 0) {
    entry = init_state(codes_at(0, ln).x & 63u);
  } else {
    constexpr u32 NW = K3_WARM / K3_BATCH;
    constexpr u32 CH = NW < 8u ? NW : 8u;  // batches per group of loads (8 x 16 B in flight)
    static_assert(NW % CH == 0, "warm-up groups");
    u32 const kw = nk > NW ? nk - NW : 0u, ep = a - seglen;  // first warm-up batch, first step of segment g-1
    u32 s = stT[0];
#pragma unroll
    for (u32 j0 = 0; j0 < NW; j0 += CH) {
      uint4 cw[CH];
#pragma unroll
      for (u32 j = 0; j < CH; j++) cw[j] = kw + j0 + j < nk ? codes_at(kw + j0 + j, lnp) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (u32 j = 0; j < CH; j++) {
        u32 const w[4] = {cw[j].x, cw[j].y, cw[j].z, cw[j].w};
#pragma unroll
        for (u32 q = 0; q < K3_BATCH; q++) {
          u32 const e = ep + K3_BATCH * (kw + j0 + j) + q;
          s = step(s, (w[q >> 2] >> (8 * (q & 3))) & 63u, kw + j0 + j < nk && e >= 1 && e < nbSeq);
        }
      }
    }
    entry = s;
  }
#ifdef ZH_STAMPS
  u64 const k3t0 = __builtin_amdgcn_s_memtime();
  u32 k3rounds = 0, k3rerun = 0;
#endif
  // A pass over the segment from state s: batches of K3_BATCH steps, the next batch's codes
  // (and, with check, its first stored state) loaded while this one runs; with check, stops
  // at the first batch whose stored first state equals the new trajectory's (returns true:
  // merged, everything from there on and the exit are already right).  s ends as the exit
  // state when the pass runs to the end.
  auto pass = [&](u32 &s, bool check) {
    uint4 cn = codes_at(0, ln);
    u32 on = check ? (u32)gst[at(0, ln)] : 0u;
    for (u32 k = 0; k < nk; k++) {
      uint4 const c4 = cn;
      u32 const o = on;
      if (k + 1 < nk) {
        cn = codes_at(k + 1, ln);
        if (check) on = gst[at(k + 1, ln)];
      }
      if (check && s == o) return true;  // met the stored trajectory: the rest is stored
      u32 const w[4] = {c4.x, c4.y, c4.z, c4.w};
      u32 sv[K3_BATCH];
#pragma unroll
      for (u32 q = 0; q < K3_BATCH; q++) {
        sv[q] = s;
        u32 const e = a + K3_BATCH * k + q;
        s = step(s, (w[q >> 2] >> (8 * (q & 3))) & 63u, e >= 1 && e < nbSeq);
      }
      uint4 *dst = (uint4 *)(gst + at(k, ln));
      dst[0] = make_uint4(sv[0] | (sv[1] << 16), sv[2] | (sv[3] << 16), sv[4] | (sv[5] << 16), sv[6] | (sv[7] << 16));
      dst[1] = make_uint4(sv[8] | (sv[9] << 16), sv[10] | (sv[11] << 16), sv[12] | (sv[13] << 16), sv[14] | (sv[15] << 16));
    }
    return false;
  };
  // first pass: every segment from its entry guess
  u32 x = entry;
  (void)pass(x, false);
  // Jacobi rounds: entry(g) = exit(g - 1); a changed entry reruns its segment until the new
  // trajectory merges with the stored one (exit then unchanged) or the segment ends
  for (;;) {
    u32 pe = wave_shr1(x);
    if constexpr (K3_W > 1) {
      // the first lane of a wave takes the last lane of the wave before (LDS, one barrier)
      if ((lane & 63u) == 63u) xw[lane >> 6] = x;
      __syncthreads();
      if ((lane & 63u) == 0u && lane) pe = xw[(lane >> 6) - 1u];
    }
    u32 const ne = (g == 0 || lane >= 3 * K3_SEGS) ? entry : pe;
    bool const active = ne != entry;
    if constexpr (K3_W > 1) {
      // any segment of the block to rerun: flag word xw[K3_W], cleared for the next round
      if (__ballot(active) && (lane & 63u) == 0u) atomicOr(&xw[K3_W], 1u);
      __syncthreads();
      bool const any = xw[K3_W] != 0u;
      __syncthreads();
      if (lane == 0) xw[K3_W] = 0u;
      if (!any) break;
    } else {
      if (!__ballot(active)) break;
    }
#ifdef ZH_STAMPS
    k3rounds++;
    k3rerun += __builtin_popcountll(__ballot(active));
#endif
    if (active) {
      entry = ne;
      u32 s = ne;
      if (!pass(s, true)) x = s;  // ran to the segment's end without merging: a new exit
    }
  }
  if (g == K3_SEGS - 1 && lane < 3 * K3_SEGS) ff[ZH_FF_SLL + t] = x;
#ifdef ZH_STAMPS
  if (lane == 0) { u32 *dbg = ws.dbg(bb); dbg[46] = (u32)(__builtin_amdgcn_s_memtime() - k3t0); dbg[47] = k3rounds; dbg[48] = k3rerun; dbg[49] = nbSeq;
                   dbg[50] = (u32)(k3t0 - k3pre); dbg[51] = (u32)k3rt0; dbg[52] = (u32)__builtin_amdgcn_s_memrealtime(); }
#endif
}

extern "C" __global__ __launch_bounds__(64 * K3_WAVES) __attribute__((amdgpu_waves_per_eu(ZH_K3_OCC, 8))) void zh_fse_chain_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws) {
  extern __shared__ __attribute__((aligned(16))) u8 smem_all[];
  u32 const bw = threadIdx.x / (64 * K3_W), lane = threadIdx.x % (64 * K3_W);  // block of the workgroup, lane in it
  u32 const bb = blockIdx.x * K3_BPW + bw;
  if (bb >= nblocks || blocks[bb].n == 0) return;  // (block-uniform: all K3_W waves return)
  if (ws.fsef(bb)[ZH_FF_NEED] == 0) return;
  k3_chain(ws, bb, smem_all + bw * K3_TAB_STRIDE, lane, (u32 *)(smem_all + K3_BPW * K3_TAB_STRIDE));  // this block's tables
}

// ======================= sequence bitstream packing (K2b) =======================
// One wave per block left by the entropy kernel: FSE state bits and extra bits of 64
// encode steps per bit-sink append, final state flush, then the block is finished
// (raw fallback, header, status) exactly as the entropy kernel does for other blocks.
// K4_WAVES blocks (one per wave, each with its own LDS slice) per workgroup: a CU holds at
// most 16 workgroups.
constexpr u32 KP_SW = 0, KP_DNB = 4 * SW_WORDS, KP_LDS = (KP_DNB + 4 * 128 + 15) & ~15u;
constexpr u32 K4_WAVES = 4;
#ifndef ZH_K4_PF
#define ZH_K4_PF 1
#endif
constexpr u32 K4_PF = ZH_K4_PF;  // chunks in flight (3 measured slower: entropy 3.05 -> 3.20 ms at 16,384
                                 // blocks, no change at 2,048)

// K4 of block b (one wave; the caller checked that the block needs it); smem = KP_LDS bytes
__device__ __forceinline__ void k4_pack(const ZhBlockDesc &d, ZhWorkspace ws, u32 b, u8 *smem, u32 lane, u64 *__restrict__ item_size,
                                        u32 *__restrict__ item_status, u32 *__restrict__ blk_size) {
  const u32 *ff = ws.fsef(b);
  u32 *sw = (u32 *)(smem + KP_SW);
  u32 *dNb = (u32 *)(smem + KP_DNB);  // LL [0, 36), OF [40, 72), ML [72, 125)
  const u8 *fz = ws.fse(b);
  if (lane < 36) dNb[lane] = ((const FseSym *)(fz + ZH_FT_SYLL))[lane].dNb;
  if (lane < 32) dNb[40 + lane] = ((const FseSym *)(fz + ZH_FT_SYOF))[lane].dNb;
  if (lane < 53) dNb[72 + lane] = ((const FseSym *)(fz + ZH_FT_SYML))[lane].dNb;
  if (lane == 0) sw[0] = 0;
  u32 const nbSeq = ff[ZH_FF_NBSEQ], logs = ff[ZH_FF_LOGS], blk = ff[ZH_FF_BLK];
  u32 const logLL = logs & 255u, logOF = (logs >> 8) & 255u, logML = logs >> 16;
  u32 const sLL = ff[ZH_FF_SLL], sOF = ff[ZH_FF_SOF], sML = ff[ZH_FF_SML];
  Out const o{d.dst, d.dst_cap};
  const u64 *seq = ws.seq(b);
  u32 const k3L = ZH_K3_SEGLEN(nbSeq), k3m = zh_k3_magic(k3L);
  // K3's states in the chain layout (a step-linear layout, whole lines here but 32-B pieces for
  // K3's stores, measured slower: entropy stage 3.05 -> 3.30 ms)
  const u16 *gLL = (const u16 *)ws.lits(b), *gOF = gLL + ZH_K3_TSTRIDE, *gML = gOF + ZH_K3_TSTRIDE;  // chain layout
  CodeTabs ct;
  ct.load();
  wave_sync();
  BitSink bs{ff[ZH_FF_OP], 0};
  // K4_PF 64-step chunks of records and states in flight
  u64 rq[K4_PF];
  u32 lq[K4_PF], mq[K4_PF], oq[K4_PF];
  auto fetch = [&](u32 e, u64 &r, u32 &sl, u32 &sm, u32 &so) {
    r = e < nbSeq ? seq[nbSeq - 1 - e] : 0;
    sl = sm = so = 0;
    if (0 < e && e < nbSeq) {
      u32 const x = zh_k3_index(e, 0, k3L, k3m);
      sl = gLL[x]; sm = gML[x]; so = gOF[x];
    }
  };
#pragma unroll
  for (u32 j = 0; j < K4_PF; j++) fetch(64 * j + lane, rq[j], lq[j], mq[j], oq[j]);
  for (u32 e0 = 0; e0 < nbSeq; e0 += 64) {
    u32 const e = e0 + lane;
    bool const valid = e < nbSeq;
    u64 const rec = rq[0];
    u32 const s_L = lq[0], s_M = mq[0], s_O = oq[0];
#pragma unroll
    for (u32 j = 0; j + 1 < K4_PF; j++) { rq[j] = rq[j + 1]; lq[j] = lq[j + 1]; mq[j] = mq[j + 1]; oq[j] = oq[j + 1]; }
    fetch(e + 64 * K4_PF, rq[K4_PF - 1], lq[K4_PF - 1], mq[K4_PF - 1], oq[K4_PF - 1]);
    u32 const ll = (u32)(rec & 0x1FFFFu), mlb = (u32)((rec >> 17) & 0x1FFFFu), ob = (u32)(rec >> 34) & 0x1FFFFu;
    u32 const llc = valid ? (u32)(rec >> 51) & 63u : 0, mlc = valid ? (u32)(rec >> 57) & 63u : 0, ofc = valid ? highbit32(ob) : 0;
    u32 const llbits = ct.ll_bits(llc), mlbits = ct.ml_bits(mlc);
    u32 vOF = 0, nOF = 0, vML = 0, nML = 0, vLL = 0, nLL = 0;
    if (valid && e > 0) {
      nOF = (s_O + dNb[40 + ofc]) >> 16; vOF = s_O;
      nML = (s_M + dNb[72 + mlc]) >> 16; vML = s_M;
      nLL = (s_L + dNb[llc]) >> 16; vLL = s_L;
    }
    u32 v6[6] = {vOF, vML, vLL, ll, mlb, ob};
    u32 n6[6] = {nOF, nML, nLL, valid ? llbits : 0u, valid ? mlbits : 0u, ofc};
    sink_append<6>(bs, o, sw, v6, n6);
  }
  {
    u32 v3[3] = {sML, sOF, sLL};
    u32 n3[3] = {lane == 0 ? logML : 0u, lane == 0 ? logOF : 0u, lane == 0 ? logLL : 0u};
    sink_append<3>(bs, o, sw, v3, n3);
  }
  sink_close(bs, o, sw);
  u32 const total = finish_block(d, o, blk, bs.pos, false);
  write_status(d, b, total, item_size, item_status, blk_size);
}

extern "C" __global__ __launch_bounds__(64 * K4_WAVES) void zh_seq_pack_kernel(const ZhBlockDesc *__restrict__ blocks, u32 nblocks, ZhWorkspace ws,
                                                                               u64 *__restrict__ item_size, u32 *__restrict__ item_status,
                                                                               u32 *__restrict__ blk_size) {
  extern __shared__ __attribute__((aligned(16))) u8 smem_all[];
  u32 const wv = threadIdx.x >> 6, b = blockIdx.x * K4_WAVES + wv;
  if (b >= nblocks) return;
  ZhBlockDesc const d = blocks[b];
  if (d.n == 0 || ws.fsef(b)[ZH_FF_NEED] == 0) return;
  k4_pack(d, ws, b, smem_all + wv * KP_LDS, lane_id(), item_size, item_status, blk_size);
}

extern "C" u32 zh_entropy_lds_bytes() { return K2_LDS; }
#ifdef ZH_STAMPS
extern "C" __global__ void zh_read_hst(u32 *out) { for (int k = 0; k < 6; k++) { out[k] = g_hst[k]; g_hst[k] = 0; } }
extern "C" void zh_hst_host(u32 *out6) {
  u32 *d = nullptr;
  if (hipMalloc(&d, 24) != hipSuccess) return;
  hipLaunchKernelGGL(zh_read_hst, dim3(1), dim3(1), 0, 0, d);
  (void)hipMemcpy(out6, d, 24, hipMemcpyDeviceToHost);
  (void)hipFree(d);
}
#endif

namespace zh {
hipError_t entropy_init() {
  hipError_t e = hipFuncSetAttribute((const void *)zh_entropy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K2_LDS);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void *)zh_fse_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)K3_LDS);
  return e;
}
void entropy_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 window_log, u32 cfg_block_size, u64 *d_item_size,
                    u32 *d_item_status, u32 *d_blk_size, hipStream_t stream) {
  hipLaunchKernelGGL(zh_entropy_kernel, dim3(nblocks), dim3(K2_THREADS), K2_LDS, stream, d_descs, ws, window_log, cfg_block_size, d_item_size,
                     d_item_status, d_blk_size);
  // (persistent K3 / K4 waves taking blocks from a counter measured slower: entropy stage
  // 3.04 -> 3.22 ms at 16,384 blocks, 0.75 -> 0.80 ms at 2,048)
  u32 const g3 = (nblocks + K3_BPW - 1) / K3_BPW, g4 = (nblocks + K4_WAVES - 1) / K4_WAVES;
  hipLaunchKernelGGL(zh_fse_chain_kernel, dim3(g3), dim3(64 * K3_WAVES), K3_LDS, stream, d_descs, nblocks, ws);
#ifndef ZH_K4_LDS_PAD
#define ZH_K4_LDS_PAD 0  // (occupancy experiments: LDS padding per K4 workgroup)
#endif
  hipLaunchKernelGGL(zh_seq_pack_kernel, dim3(g4), dim3(64 * K4_WAVES), K4_WAVES * KP_LDS + ZH_K4_LDS_PAD, stream, d_descs, nblocks, ws, d_item_size,
                     d_item_status, d_blk_size);
}
}  // namespace zh
