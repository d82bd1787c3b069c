// zh_hash.h — the match finders' position hashes (include/zstd_hip_params.h), shared by K1
// (zh_lz.hip) and the deep matcher (zh_lz_deep.hip); oracle/zstd_oracle.c zh_hash_long/short.
#pragma once
#include "zh_common.h"

// Full-rate v_mad_u32_u24 sums (the 24-bit multiplies take the low 24 bits of each operand, so
// byte groups need no masking but the short hash's bytes 3-4); (lo, hi) = the 8 bytes at p.
// the long hash's 32-bit sum (also the repeat scan's slot and signature, zh_lz.hip repeat_scan)
__device__ __forceinline__ u32 hash_long_sum(u32 lo, u32 hi) {
  u32 t = __umul24(lo, ZH_HK_L0);
  t += __umul24(__builtin_amdgcn_alignbyte(hi, lo, 3), ZH_HK_L1);
  t += __umul24(hi >> 16, ZH_HK_L2);
  return t;
}
__device__ __forceinline__ u32 hash_long(u32 lo, u32 hi) { return hash_long_sum(lo, hi) >> (32 - ZH_HASH_LOG_LONG); }
__device__ __forceinline__ u32 hash_short(u32 lo, u32 hi) {
  u32 t = __umul24(lo, ZH_HK_S0);
  t += __umul24(__builtin_amdgcn_alignbyte(hi, lo, 3) & 0xFFFFu, ZH_HK_S1);
  return t >> (32 - ZH_HASH_LOG_SHORT);
}
