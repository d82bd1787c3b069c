// zh_dict.cpp — host side of dictionaries (RFC 8878 §5).
//
//   dict_layout  raw content (any buffer not starting with the dictionary magic: ID 0, all of
//                it content) or a formatted dictionary: magic, Dictionary_ID, Huffman table
//                description, OF / ML / LL FSE table descriptions, three repcodes (each in
//                [1, content size], libzstd ZSTD_loadDEntropy's check), content
//   cover_train  COVER training (Liao, Petri, Moffat, Wirth, WWW 2016 — the algorithm of
//                libzstd's ZDICT_trainFromBuffer_cover) producing raw-content dictionaries;
//                replaces the reference's byte / 4-gram frequency fill
//                (src/cuda_zstd_dictionary.cu:179-415, train_dictionary_gpu)
#include "zh_dict.h"

#include <algorithm>
#include <cstring>

namespace zh {
namespace {
typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

u32 rd32le(const u8 *p) {
  u32 v;
  memcpy(&v, p, 4);
  return v;
}

// 32 bits starting at bit `bitpos` (LSB first), zeros past `avail` bytes
u32 fwd32(const u8 *p, size_t avail, size_t bitpos) {
  size_t const b = bitpos >> 3;
  u64 v = 0;
  for (size_t i = 0; i < 5; i++)
    if (b + i < avail) v |= (u64)p[b + i] << (8 * i);
  return (u32)(v >> (bitpos & 7));
}

// bytes used by an FSE table description (FSE_readNCount, RFC 8878 §4.1.1); 0 if malformed
size_t ncount_size(const u8 *p, size_t avail, u32 maxSV, u32 maxLog) {
  if (!avail) return 0;
  u32 nb = (fwd32(p, avail, 0) & 15u) + 5u;
  if (nb > maxLog) return 0;
  size_t bp = 4;
  int rem = (1 << nb) + 1, thr = 1 << nb;
  nb++;
  u32 sym = 0;
  bool prev0 = false;
  while (rem > 1 && sym <= maxSV) {
    if (prev0) {
      u32 n0 = sym, r;
      do {
        r = fwd32(p, avail, bp) & 3u;
        bp += 2;
        n0 += r;
      } while (r == 3 && bp < 8 * avail + 32);
      if (n0 > maxSV) return 0;
      sym = n0;
    }
    u32 const bs = fwd32(p, avail, bp);
    int const mx = (2 * thr - 1) - rem;
    int c;
    if ((int)(bs & (u32)(thr - 1)) < mx) {
      c = (int)(bs & (u32)(thr - 1));
      bp += nb - 1;
    } else {
      c = (int)(bs & (u32)(2 * thr - 1));
      if (c >= thr) c -= mx;
      bp += nb;
    }
    c--;
    rem -= c < 0 ? -c : c;
    sym++;
    prev0 = c == 0;
    while (rem < thr) {
      nb--;
      thr >>= 1;
    }
  }
  if (rem != 1) return 0;
  size_t const used = (bp + 7) >> 3;
  return used <= avail ? used : 0;
}
}  // namespace

bool dict_layout(const u8 *d, size_t n, u32 &id, size_t &content_off) {
  id = 0;
  content_off = 0;
  if (n < 8 || rd32le(d) != kDictMagic) return true;  // raw content
  id = rd32le(d + 4);
  size_t o = 8;
  u32 const hb = d[o];
  size_t const hsz = hb >= 128 ? 1 + ((size_t)(hb - 127) + 1) / 2 : 1 + (size_t)hb;
  if (hb == 0 || o + hsz > n) return false;
  o += hsz;
  static const u32 msv[3] = {31, 52, 35}, mlg[3] = {8, 9, 9};  // OF, ML, LL
  for (int t = 0; t < 3; t++) {
    size_t const u = o < n ? ncount_size(d + o, n - o, msv[t], mlg[t]) : 0;
    if (!u) return false;
    o += u;
  }
  if (o + 12 > n) return false;
  size_t const cn = n - o - 12;
  for (int k = 0; k < 3; k++) {
    u32 const r = rd32le(d + o + 4 * k);
    if (r == 0 || r > cn) return false;
  }
  content_off = o + 12;
  return true;
}

std::vector<u8> cover_train(const std::vector<std::pair<const u8 *, size_t>> &samples, size_t dict_size, u32 k, u32 d) {
  d = std::min<u32>(std::max<u32>(d, 4), 8);
  k = std::max<u32>(k, 2 * d);
  std::vector<u8> corpus;
  std::vector<size_t> ends;
  for (auto const &s : samples) {
    if (s.second) corpus.insert(corpus.end(), s.first, s.first + s.second);
    ends.push_back(corpus.size());
  }
  size_t const N = corpus.size();
  if (N < (size_t)k || dict_size < d) return {};
  corpus.resize(N + 8, 0);  // padding for the 8-byte reads
  constexpr u32 HB = 20, NONE = ~0u;
  u64 const mask = d >= 8 ? ~0ull : ((1ull << (8 * d)) - 1);
  size_t const nd = N - d + 1;  // d-mer start positions
  // hashed d-mer id of every position; NONE where the d-mer crosses a sample end
  std::vector<u32> dm(nd, NONE);
  size_t si = 0;
  for (size_t i = 0; i < nd; i++) {
    while (ends[si] <= i) si++;
    if (i + d > ends[si]) continue;
    u64 v;
    memcpy(&v, corpus.data() + i, 8);
    dm[i] = (u32)(((v & mask) * 0x9E3779B185EBCA87ull) >> (64 - HB));
  }
  // frequency of a d-mer = number of samples containing it
  std::vector<u32> freq(1u << HB, 0), seen(1u << HB, NONE);
  si = 0;
  for (size_t i = 0; i < nd; i++) {
    while (ends[si] <= i) si++;
    u32 const h = dm[i];
    if (h != NONE && seen[h] != (u32)si) {
      seen[h] = (u32)si;
      freq[h]++;
    }
  }
  // epochs (libzstd COVER_computeEpochs): about dict_size / k / 4 of them, each >= 10 k
  size_t const seg = k - d + 1;  // d-mers per segment
  size_t epochs = std::max<size_t>(1, dict_size / k / 4), esz = nd / epochs;
  if (esz < 10 * (size_t)k) {
    esz = std::min(nd, 10 * (size_t)k);
    epochs = std::max<size_t>(1, nd / esz);
  }
  std::vector<u32> active(1u << HB, 0);
  std::vector<u8> dict(dict_size);
  size_t tail = dict_size;
  u32 zero_run = 0;
  u32 const max_zero = std::max<u32>(10, std::min<u32>(100, (u32)(epochs >> 3)));
  for (size_t e = 0; tail > 0; e = (e + 1) % epochs) {
    size_t const b = e * esz, end = std::min(nd, b + esz);
    // best window of `seg` d-mers in [b, end): score = sum of the frequencies of its distinct d-mers
    u64 score = 0, best = 0;
    size_t best_b = b, wb = b;
    for (size_t i = b; i < end; i++) {
      u32 const h = dm[i];
      if (h != NONE && active[h]++ == 0) score += freq[h];
      if (i + 1 - wb > seg) {
        u32 const g = dm[wb++];
        if (g != NONE && --active[g] == 0) score -= freq[g];
      }
      if (score > best) {
        best = score;
        best_b = wb;
      }
    }
    for (size_t i = wb; i < end; i++)
      if (dm[i] != NONE) active[dm[i]] = 0;
    if (best == 0) {
      if (++zero_run >= max_zero) break;
      continue;
    }
    zero_run = 0;
    size_t sb = best_b, se = std::min(end, best_b + seg);
    while (sb < se && (dm[sb] == NONE || freq[dm[sb]] == 0)) sb++;
    while (se > sb && (dm[se - 1] == NONE || freq[dm[se - 1]] == 0)) se--;
    for (size_t i = sb; i < se; i++)
      if (dm[i] != NONE) freq[dm[i]] = 0;
    size_t const bytes = std::min(se - sb + d - 1, tail);
    if (bytes < d) break;
    tail -= bytes;
    memcpy(dict.data() + tail, corpus.data() + sb, bytes);
  }
  dict.erase(dict.begin(), dict.begin() + (ptrdiff_t)tail);
  return dict;
}
}  // namespace zh
