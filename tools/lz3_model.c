/* Design-space experiment (not product code): ratio and walk statistics of LZ parse
 * semantics for the round-3 K1, entropy-coded by libzstd's ZSTD_compressSequences (the
 * device entropy stage is byte-identical to it), vs ZSTD_compress level 3.
 *   gcc -O2 -fopenmp -I/opt/conda/include tools/lz3_model.c tools/datagen.c \
 *       -L/opt/conda/lib -l:libzstd.so.1 -lm -o /tmp/lz3 && /tmp/lz3 */
#define ZSTD_STATIC_LINKING_ONLY
#include <zstd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void dg_fill(uint8_t *dst, size_t n_chunks, size_t chunk_size, uint64_t seed, int kind, uint64_t first);

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static int g_hash = 0;  /* 0: 64-bit multiply (r02), 1: 24-bit multiply-adds (full-rate v_mad_u32_u24) */
static inline uint32_t mu24(uint32_t a, uint32_t b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
static inline uint32_t hashL(uint64_t v, int hl) {
  if (g_hash) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32), b = (uint32_t)(v >> 24);
    uint32_t t = mu24(lo, 0x9E3779u) + mu24(b, 0x85EBCAu) + mu24(hi >> 16, 0xC2B2AEu);
    return t >> (32 - hl);
  }
  return (uint32_t)((v * 0xCF1BBCDCB7A56463ull) >> (64 - hl));
}
static inline uint32_t hashS(uint64_t v, int hl) {
  if (g_hash) {
    uint32_t lo = (uint32_t)v, b = (uint32_t)(v >> 24) & 0xFFFFu;
    uint32_t t = mu24(lo, 0x27D4EBu) + mu24(b, 0x165667u);
    return t >> (32 - hl);
  }
  return (uint32_t)(((v << 24) * 0x9E3779B185EBCA87ull) >> (64 - hl));
}
static int cnt(const uint8_t *a, const uint8_t *b, const uint8_t *end) { int n = 0; while (a + n < end && a[n] == b[n]) n++; return n; }

typedef struct {
  int tile, hl, hs;
  int mode;     /* 0 cur (lazy-1 best-of-two), 1 dfast rule */
  int cap;      /* per-step length cap (cur) */
  int skip;     /* dfast: kSearchStrength (0 = none) */
  int catchup, imm, rep1;  /* dfast options: backward catch-up, immediate rep, rep check at p+1 */
  int lazyL;    /* dfast: long check at p+1 when only the short matched */
  int repcap;   /* dfast: step cap for matches (0 none) */
  const char *name;
} cfg_t;

typedef struct { long steps, visited; long simt; } stats_t;

static int *g_cL, *g_cS;
static void candidates(const uint8_t *src, int n, const cfg_t *c) {
  static int TL[1 << 18], TS[1 << 18];
  for (int i = 0; i < (1 << c->hl); i++) TL[i] = -1;
  for (int i = 0; i < (1 << c->hs); i++) TS[i] = -1;
  int lim = n - 8;
  for (int p = 0; p < n; p++) { g_cL[p] = -1; g_cS[p] = -1; }
  for (int t = 0; t < lim; t += c->tile) {
    int e = t + c->tile < lim ? t + c->tile : lim;
    for (int p = t; p < e; p++) { uint64_t v = rd64(src + p); g_cL[p] = TL[hashL(v, c->hl)]; g_cS[p] = TS[hashS(v, c->hs)]; }
    for (int p = t; p < e; p++) { uint64_t v = rd64(src + p); TL[hashL(v, c->hl)] = p; TS[hashS(v, c->hs)] = p; }
  }
}

static int len[70000], off[70000];
static size_t parse_cur(const uint8_t *src, int n, const cfg_t *c, ZSTD_Sequence *sq, int *steps_at) {
  const uint8_t *end = src + n;
  int lim = n - 8;
  for (int p = 0; p <= n + 1; p++) { len[p] = 0; off[p] = 0; }
  for (int p = 0; p < lim; p++) {
    int qL = g_cL[p], qS = g_cS[p];
    int lL = qL >= 0 ? cnt(src + p, src + qL, end) : 0, lS = qS >= 0 ? cnt(src + p, src + qS, end) : 0;
    if (lL > c->cap) lL = c->cap;
    if (lS > c->cap) lS = c->cap;
    if (lL < 8) lL = 0;
    if (lS < 5) lS = 0;
    if (lL && lL >= lS) { len[p] = lL; off[p] = p - qL; } else if (lS) { len[p] = lS; off[p] = p - qS; }
  }
  int p = 0, anchor = 0; size_t ns = 0;
  while (p < lim) {
    steps_at[p] = 1;
    if (len[p] == 0 || len[p + 1] > len[p]) { p++; continue; }
    int ms = p, ml = len[p], of = off[p];
    if (c->catchup) while (ms > anchor && ms - of > 0 && src[ms - 1] == src[ms - 1 - of]) { ms--; ml++; }
    if (ns && ms == anchor && sq[ns - 1].offset == (unsigned)of) sq[ns - 1].matchLength += ml;
    else { sq[ns].litLength = ms - anchor; sq[ns].offset = of; sq[ns].matchLength = ml; sq[ns].rep = 0; ns++; }
    p += len[p]; anchor = p;
  }
  sq[ns].litLength = n - anchor; sq[ns].offset = 0; sq[ns].matchLength = 0; sq[ns].rep = 0; ns++;
  return ns;
}


/* SIMT cost of the lane-per-segment walk over windows of W positions, segments of S (lanes =
 * W / S), literal runs skipped by a "has match" mask: one iteration per visited position with a
 * match candidate.  Jacobi: guessed entries = segment starts, re-walk until the trajectory meets
 * the previous one.  Returns wave-iterations (sum over rounds of the max over lanes). */
static long g_rounds, g_windows, g_maxr;
static int walk_iters(int s0, int e, int se, int n, int lim, int *vis, int mark, int *merged) {
  int p = s0, it = 0; *merged = 0;
  while (p < se) {
    if (p >= lim || len[p] == 0) { if (mark) vis[p] = mark; p++; continue; }
    if (vis[p] && vis[p] != mark) { *merged = 1; break; }
    it++;
    vis[p] = mark;
    if (len[p + 1] > len[p]) p++; else p += len[p];
  }
  (void)e; (void)n;
  return it;
}
static long walk_cost(int n, int W, int S) {
  int lim = n - 8; long cost = 0;
  static int vis[70000], ent[4096], ext[4096];
  int e_in = 0;
  for (int ws = 0; ws < n; ws += W) {
    int we = ws + W < n ? ws + W : n;
    int ns = (we - ws + S - 1) / S;
    for (int p = ws; p < we + 64; p++) vis[p < 70000 ? p : 69999] = 0;
    /* round 1 */
    int mx = 0;
    for (int g = 0; g < ns; g++) {
      int s = ws + g * S, se = s + S < we ? s + S : we, m;
      ent[g] = g == 0 ? (e_in > s ? e_in : s) : s;
      int it = walk_iters(ent[g], 0, se, n, lim, vis, g + 1, &m);
      /* exit */
      int p = ent[g];
      while (p < se) { if (p >= lim || len[p] == 0 || len[p + 1] > len[p]) p++; else p += len[p]; }
      ext[g] = p;
      if (it > mx) mx = it;
    }
    cost += mx;
    int rounds = 1;
    for (;;) {
      int ch = 0; mx = 0;
      int nent[4096];
      for (int g = 1; g < ns; g++) nent[g] = ext[g - 1];
      for (int g = 1; g < ns; g++) {
        if (nent[g] == ent[g]) continue;
        ch = 1;
        int s = ws + g * S, se = s + S < we ? s + S : we, m;
        /* re-walk until merge with the old trajectory of this lane */
        int it = 0, p = nent[g];
        while (p < se) {
          if (p >= lim || len[p] == 0) { p++; continue; }
          if (vis[p] == g + 1) break; /* merged */
          it++;
          if (len[p + 1] > len[p]) p++; else p += len[p];
        }
        (void)m;
        /* true new trajectory & marks */
        for (int q = s; q < se; q++) if (vis[q] == g + 1) vis[q] = 0;
        p = nent[g];
        while (p < se) { vis[p] = g + 1; if (p >= lim || len[p] == 0 || len[p + 1] > len[p]) p++; else p += len[p]; }
        ent[g] = nent[g];
        ext[g] = p;
        if (it > mx) mx = it;
      }
      if (!ch) break;
      cost += mx + 2; rounds++;
    }
    g_rounds += rounds; g_windows++; if (rounds > g_maxr) g_maxr = rounds;
    e_in = ext[ns - 1];
  }
  return cost;
}

static size_t parse_dfast(const uint8_t *src, int n, const cfg_t *c, ZSTD_Sequence *sq, int *steps_at) {
  const uint8_t *end = src + n;
  int lim = n - 8;
  int p = 0, anchor = 0, rep0 = 0, rep1 = 0; size_t ns = 0;
  while (p < lim) {
    steps_at[p] = 1;
    int ms = -1, ml = 0, off = 0, isrep = 0;
    if (c->rep1 && rep0 && p + 1 - rep0 >= 0 && p + 1 < lim && rd32(src + p + 1) == rd32(src + p + 1 - rep0)) {
      ms = p + 1; off = rep0; ml = 4 + cnt(src + p + 5, src + p + 5 - rep0, end); isrep = 1;
    } else {
      int q = g_cL[p];
      if (q >= 0 && rd64(src + q) == rd64(src + p)) { ms = p; off = p - q; ml = 8 + cnt(src + p + 8, src + q + 8, end); }
      else {
        q = g_cS[p];
        if (q >= 0 && rd32(src + q) == rd32(src + p)) {
          int q3 = c->lazyL && p + 1 < lim ? g_cL[p + 1] : -1;
          if (q3 >= 0 && rd64(src + q3) == rd64(src + p + 1)) { ms = p + 1; off = p + 1 - q3; ml = 8 + cnt(src + p + 9, src + q3 + 8, end); }
          else { ms = p; off = p - q; ml = 4 + cnt(src + p + 4, src + q + 4, end); }
        }
      }
      if (ms >= 0 && c->catchup) while (ms > anchor && ms - off > 0 && src[ms - 1] == src[ms - 1 - off]) { ms--; ml++; }
    }
    if (ms < 0) { p += (c->skip ? ((p - anchor) >> c->skip) : 0) + 1; continue; }
    if (!isrep) { rep1 = rep0; rep0 = off; }
    sq[ns].litLength = ms - anchor; sq[ns].offset = off; sq[ns].matchLength = ml; sq[ns].rep = 0; ns++;
    p = anchor = ms + ml;
    if (c->imm) while (p < lim && rep1 && p >= rep1 && rd32(src + p) == rd32(src + p - rep1)) {
      int l = 4 + cnt(src + p + 4, src + p + 4 - rep1, end);
      int t = rep0; rep0 = rep1; rep1 = t;
      sq[ns].litLength = 0; sq[ns].offset = rep0; sq[ns].matchLength = l; sq[ns].rep = 0; ns++;
      p = anchor = p + l;
    }
  }
  sq[ns].litLength = n - anchor; sq[ns].offset = 0; sq[ns].matchLength = 0; sq[ns].rep = 0; ns++;
  return ns;
}

int main(int argc, char **argv) {
  if (argc > 2) g_hash = atoi(argv[2]);
  int nch = argc > 1 ? atoi(argv[1]) : 128, cs = 65536;
  uint8_t *buf = malloc((size_t)nch * cs), *out = malloc(200000);
  ZSTD_Sequence *seqs = malloc(sizeof(ZSTD_Sequence) * (cs + 8));
  int *steps = malloc(sizeof(int) * (cs + 8));
  g_cL = malloc(sizeof(int) * (cs + 8)); g_cS = malloc(sizeof(int) * (cs + 8));
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  int kinds[] = {0, 1, 3, 5, 6, 7, 8};
  const char *kn[] = {"mix", "random", "sym16", "text", "json", "source", "csv", "exe", "sensor"};
  cfg_t cfgs[] = {
    {128, 14, 14, 0, 64, 0, 0, 0, 0, 0, 0, "cur (r02)"},
    {128, 14, 14, 0, 64, 0, 1, 0, 0, 0, 0, "cur+catch"},
    {128, 14, 14, 0, 32, 0, 1, 0, 0, 0, 0, "cur+catch cap32"},
    {128, 14, 14, 0, 16, 0, 1, 0, 0, 0, 0, "cur+catch cap16"},
    {128, 14, 14, 0, 1000, 0, 1, 0, 0, 0, 0, "cur+catch nocap"},
    {64, 14, 14, 0, 64, 0, 1, 0, 0, 0, 0, "cur+catch t64"},
    {32, 14, 14, 0, 64, 0, 1, 0, 0, 0, 0, "cur+catch t32"},
    {128, 14, 14, 1, 0, 8, 1, 1, 1, 1, 0, "dfast full"},
    {64, 14, 14, 1, 0, 8, 1, 1, 1, 1, 0, "dfast tile64"},
  };
  int ncfg = sizeof(cfgs) / sizeof(cfgs[0]);
  for (int ki = 0; ki < (int)(sizeof(kinds) / sizeof(kinds[0])); ki++) {
    dg_fill(buf, nch, cs, kinds[ki] == 1 ? 0x5EED0004 : 0x5EED0003, kinds[ki], 0);
    size_t ref = 0;
    for (int i = 0; i < nch; i++) ref += ZSTD_compress(out, 200000, buf + (size_t)i * cs, cs, 3);
    printf("%-7s libzstd-L3 %.4f\n", kn[kinds[ki]], (double)nch * cs / ref);
    for (int ci = 0; ci < ncfg; ci++) {
      size_t tot = 0, nseq = 0; long vis = 0;
      for (int i = 0; i < nch; i++) {
        const uint8_t *src = buf + (size_t)i * cs;
        candidates(src, cs, &cfgs[ci]);
        memset(steps, 0, sizeof(int) * cs);
        size_t ns = cfgs[ci].mode ? parse_dfast(src, cs, &cfgs[ci], seqs, steps) : parse_cur(src, cs, &cfgs[ci], seqs, steps);
        for (int p = 0; p < cs; p++) vis += steps[p];
        nseq += ns;
        ZSTD_CCtx_reset(cc, ZSTD_reset_session_and_parameters);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_compressionLevel, 3);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_blockDelimiters, ZSTD_sf_explicitBlockDelimiters);
        size_t r = ZSTD_compressSequences(cc, out, 200000, seqs, ns, src, cs);
        if (ZSTD_isError(r)) { printf("err %s\n", ZSTD_getErrorName(r)); return 1; }
        tot += r;
      }
      if (!cfgs[ci].mode && cfgs[ci].catchup && cfgs[ci].tile == 128) {
        long w1 = 0, w2 = 0, w3 = 0; g_rounds = g_windows = g_maxr = 0;
        for (int i = 0; i < nch; i++) { const uint8_t *src = buf + (size_t)i * cs; candidates(src, cs, &cfgs[ci]); memset(steps, 0, sizeof(int) * cs); parse_cur(src, cs, &cfgs[ci], seqs, steps);
          w1 += walk_cost(cs, 2048, 32); }
        long r1 = g_rounds, wn1 = g_windows, m1 = g_maxr; g_rounds = g_windows = g_maxr = 0;
        for (int i = 0; i < nch; i++) { const uint8_t *src = buf + (size_t)i * cs; candidates(src, cs, &cfgs[ci]); memset(steps, 0, sizeof(int) * cs); parse_cur(src, cs, &cfgs[ci], seqs, steps);
          w2 += walk_cost(cs, 2048, 16); w3 += walk_cost(cs, 4096, 64); }
        printf("      walk iters/block: W2048 S32 %ld (rounds avg %.2f max %ld) | W2048 S16 %ld | W4096 S64 %ld\n", w1 / nch, (double)r1 / wn1, m1, w2 / nch, w3 / nch);
      }
      printf("   %-16s ratio %.4f (%.4f of L3)  seq/chunk %6zu  steps/chunk %6ld\n", cfgs[ci].name, (double)nch * cs / tot, (double)ref / tot, nseq / nch, vis / nch);
    }
  }
  return 0;
}
