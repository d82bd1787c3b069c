// zh_xxh64.h — XXH64 (seed 0) for the frame content checksum (RFC 8878 §3.1.1: the low
// 32 bits of XXH64 of the decompressed content).  Used by the compressor's checksum
// kernel and by the decoder.  One wave: lanes 0..3 run the four accumulators over the
// 32-byte stripes; the tail and the merge are done redundantly on every lane.
#pragma once
#include "zh_common.h"

// 8 bytes at p, all inside the buffer: aligned dword loads only (never a page the buffer
// does not reach)
__device__ __forceinline__ u64 zh_ld64(const u8 *p) {
  uintptr_t const a = (uintptr_t)p;
  const u32 *w = (const u32 *)(a & ~(uintptr_t)3);
  u32 const sh = (u32)(a & 3);
  u32 const w0 = w[0], w1 = w[1];
  u32 w2 = 0;
  if (sh) w2 = w[2];
  return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

__device__ __noinline__ u64 zh_xxh64(const u8 *p, u64 n) {
  constexpr u64 P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull, P4 = 0x85EBCA77C2B2AE63ull,
                P5 = 0x27D4EB2F165667C5ull;
  auto rotl = [](u64 x, u32 r) { return (x << r) | (x >> (64 - r)); };
  auto round = [&](u64 acc, u64 in) { return rotl(acc + in * P2, 31) * P1; };
  u32 const lane = threadIdx.x & 63u;
  u64 h;
  u64 const nst = n / 32;
  if (n >= 32) {
    u64 v = lane == 0 ? P1 + P2 : lane == 1 ? P2 : lane == 2 ? 0ull : (u64)0 - P1;
    if (lane < 4) {
      u64 k = 0;
      for (; k + 4 <= nst; k += 4) {
        u64 a[4];
#pragma unroll
        for (u32 j = 0; j < 4; j++) a[j] = zh_ld64(p + 32 * (k + j) + 8 * lane);
#pragma unroll
        for (u32 j = 0; j < 4; j++) v = round(v, a[j]);
      }
      for (; k < nst; k++) v = round(v, zh_ld64(p + 32 * k + 8 * lane));
    }
    u64 const v1 = __shfl(v, 0, 64), v2 = __shfl(v, 1, 64), v3 = __shfl(v, 2, 64), v4 = __shfl(v, 3, 64);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = (h ^ round(0, v1)) * P1 + P4;
    h = (h ^ round(0, v2)) * P1 + P4;
    h = (h ^ round(0, v3)) * P1 + P4;
    h = (h ^ round(0, v4)) * P1 + P4;
  } else {
    h = P5;
  }
  h += n;
  const u8 *q = p + 32 * nst;
  u64 r = n - 32 * nst;
  while (r >= 8) {
    h ^= round(0, zh_ld64(q));
    h = rotl(h, 27) * P1 + P4;
    q += 8;
    r -= 8;
  }
  if (r >= 4) {
    h ^= (u64)((u32)q[0] | (u32)q[1] << 8 | (u32)q[2] << 16 | (u32)q[3] << 24) * P1;
    h = rotl(h, 23) * P2 + P3;
    q += 4;
    r -= 4;
  }
  while (r) {
    h ^= (u64)(*q) * P5;
    h = rotl(h, 11) * P1;
    q++;
    r--;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// XXH64 (seed 0) of one buffer by a whole wave, for long inputs: every lane loads one 32-byte
// stripe of a 64-stripe chunk and pre-multiplies its four words by P2 into LDS (double
// buffered; the next chunk's loads are in flight while this chunk's rounds run), and lanes
// 0..3 run the four accumulator chains acc = rotl(acc + t, 31) * P1 from LDS -- the only
// serial part of XXH64.  lds: 2 x 256 u64 of the caller's LDS.  Same value as zh_xxh64.
__device__ __noinline__ u64 zh_xxh64_wave(const u8 *p, u64 n, u64 *lds) {
  constexpr u64 P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full;
  u32 const lane = threadIdx.x & 63u;
  u64 const nst = n / 32, nch = nst / 64;
  if (nch == 0) return zh_xxh64(p, n);
  auto rotl = [](u64 x, u32 r) { return (x << r) | (x >> (64 - r)); };
  u64 v = lane == 0 ? P1 + P2 : lane == 1 ? P2 : lane == 2 ? 0ull : (u64)0 - P1;
  u64 w[4];
#pragma unroll
  for (u32 j = 0; j < 4; j++) w[j] = zh_ld64(p + 32 * (u64)lane + 8 * j);
  for (u64 c = 0; c < nch; c++) {
    u64 *const b = lds + 256 * (c & 1);
#pragma unroll
    for (u32 j = 0; j < 4; j++) b[4 * lane + j] = w[j] * P2;
    if (c + 1 < nch) {
#pragma unroll
      for (u32 j = 0; j < 4; j++) w[j] = zh_ld64(p + 32 * (64 * (c + 1) + lane) + 8 * j);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < 4) {
      for (u32 s0 = 0; s0 < 64; s0 += 8) {
        u64 t[8];
#pragma unroll
        for (u32 s = 0; s < 8; s++) t[s] = b[4 * (s0 + s) + lane];
#pragma unroll
        for (u32 s = 0; s < 8; s++) v = rotl(v + t[s], 31) * P1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // remaining stripes (< 64): lanes 0..3 directly
  if (lane < 4) {
    for (u64 k = 64 * nch; k < nst; k++) v = rotl(v + zh_ld64(p + 32 * k + 8 * lane) * P2, 31) * P1;
  }
  auto round = [&](u64 acc, u64 in) { return rotl(acc + in * P2, 31) * P1; };
  constexpr u64 P3 = 0x165667B19E3779F9ull, P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
  u64 const v1 = __shfl(v, 0, 64), v2 = __shfl(v, 1, 64), v3 = __shfl(v, 2, 64), v4 = __shfl(v, 3, 64);
  u64 h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  h = (h ^ round(0, v1)) * P1 + P4;
  h = (h ^ round(0, v2)) * P1 + P4;
  h = (h ^ round(0, v3)) * P1 + P4;
  h = (h ^ round(0, v4)) * P1 + P4;
  h += n;
  const u8 *q = p + 32 * nst;
  u64 r = n - 32 * nst;
  while (r >= 8) {
    h ^= round(0, zh_ld64(q));
    h = rotl(h, 27) * P1 + P4;
    q += 8;
    r -= 8;
  }
  if (r >= 4) {
    h ^= (u64)((u32)q[0] | (u32)q[1] << 8 | (u32)q[2] << 16 | (u32)q[3] << 24) * P1;
    h = rotl(h, 23) * P2 + P3;
    q += 4;
    r -= 4;
  }
  while (r) {
    h ^= (u64)(*q) * P5;
    h = rotl(h, 11) * P1;
    q++;
    r--;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}
