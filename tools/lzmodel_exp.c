/* Design-space experiment (not product code): ratio of GPU-friendly LZ parse
 * variants, entropy-coded by libzstd's ZSTD_compressSequences, vs ZSTD_compress L3. */
#define ZSTD_STATIC_LINKING_ONLY
#include <zstd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void dg_fill(uint8_t *dst, size_t n_chunks, size_t chunk_size, uint64_t seed, int kind, uint64_t first);

typedef struct { int tile, hl, hs, mins, rep, lazy, catchup, imm, hl8; } cfg_t;

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t hash8(uint64_t v, int hl) { return (uint32_t)((v * 0xCF1BBCDCB7A56463ull) >> (64 - hl)); }
static inline uint32_t hash5(uint64_t v, int hl, int mins) {
  uint64_t m = mins >= 8 ? v : (v << (64 - 8 * mins));
  return (uint32_t)((m * 0x9E3779B185EBCA87ull) >> (64 - hl));
}
static int cnt(const uint8_t *a, const uint8_t *b, const uint8_t *end) {
  int n = 0; while (a + n < end && a[n] == b[n]) n++; return n;
}

static size_t model2(const uint8_t *src, int n, cfg_t c, ZSTD_Sequence *seqs);
static int main2(void);
static size_t model(const uint8_t *src, int n, cfg_t c, ZSTD_Sequence *seqs) {
  int *TL = malloc(sizeof(int) << c.hl), *TS = malloc(sizeof(int) << c.hs);
  int *cL = malloc(sizeof(int) * n), *cS = malloc(sizeof(int) * n);
  for (int i = 0; i < (1 << c.hl); i++) TL[i] = -1;
  for (int i = 0; i < (1 << c.hs); i++) TS[i] = -1;
  int lim = n - 8;
  for (int t = 0; t < lim; t += c.tile) {
    int e = t + c.tile < lim ? t + c.tile : lim;
    for (int p = t; p < e; p++) { uint64_t v = rd64(src + p); cL[p] = TL[hash8(v, c.hl)]; cS[p] = TS[hash5(v, c.hs, c.mins)]; }
    for (int p = t; p < e; p++) { uint64_t v = rd64(src + p); TL[hash8(v, c.hl)] = p; TS[hash5(v, c.hs, c.mins)] = p; }
  }
  const uint8_t *end = src + n;
  int anchor = 0, p = 0, rep0 = 1, rep1 = 4, rep2 = 8; size_t ns = 0;
  (void)rep2;
  while (p < lim) {
    int ms = -1, ml = 0, off = 0;
    if (c.rep && p >= rep0 && rd32(src + p) == rd32(src + p - rep0)) { ms = p; off = rep0; ml = 4 + cnt(src + p + 4, src + p + 4 - rep0, end); }
    else {
      int q = cL[p];
      if (q >= 0 && rd64(src + q) == rd64(src + p)) { ms = p; off = p - q; ml = 8 + cnt(src + p + 8, src + q + 8, end); }
      else {
        q = cS[p];
        int l = q >= 0 ? cnt(src + p, src + q, end) : 0;
        if (l >= c.mins) {
          ms = p; off = p - q; ml = l;
          if (c.lazy && p + 1 < lim) {
            int q1 = cL[p + 1];
            if (q1 >= 0 && rd64(src + q1) == rd64(src + p + 1)) {
              int l1 = 8 + cnt(src + p + 9, src + q1 + 8, end);
              if (l1 > ml) { ms = p + 1; off = p + 1 - q1; ml = l1; }
            }
          }
        }
      }
    }
    if (ms < 0) { p++; continue; }
    if (c.catchup) while (ms > anchor && ms - off > 0 && src[ms - 1] == src[ms - 1 - off]) { ms--; ml++; }
    seqs[ns].litLength = ms - anchor; seqs[ns].offset = off; seqs[ns].matchLength = ml; seqs[ns].rep = 0; ns++;
    if (off != rep0) { rep2 = rep1; rep1 = rep0; rep0 = off; }
    p = anchor = ms + ml;
    if (c.imm) while (p < lim && p >= rep1 && rd32(src + p) == rd32(src + p - rep1)) {
      int l = 4 + cnt(src + p + 4, src + p + 4 - rep1, end);
      seqs[ns].litLength = 0; seqs[ns].offset = rep1; seqs[ns].matchLength = l; seqs[ns].rep = 0; ns++;
      int t = rep0; rep0 = rep1; rep1 = t; p = anchor = p + l;
    }
  }
  seqs[ns].litLength = n - anchor; seqs[ns].offset = 0; seqs[ns].matchLength = 0; seqs[ns].rep = 0; ns++;
  free(TL); free(TS); free(cL); free(cS);
  return ns;
}

int g_bl[70000]; extern int g_maxml;
int main(int argc, char **argv) {
  if (argc > 1) return main2();
  int nch = 128, cs = 65536;
  uint8_t *buf = malloc((size_t)nch * cs), *out = malloc(200000);
  ZSTD_Sequence *seqs = malloc(sizeof(ZSTD_Sequence) * cs);
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  int kinds[] = {0, 3, 5, 6, 7, 8, 2};
  cfg_t cfgs[] = {
    {1, 16, 15, 5, 1, 1, 1, 1, 8},
    {64, 14, 14, 5, 1, 1, 0, 1, 8},
    {64, 14, 14, 5, 2, 1, 0, 0, 8},
    {64, 14, 14, 5, 2, 2, 0, 0, 8},
    {64, 14, 14, 5, 2, 0, 0, 0, 8},
    {128, 14, 14, 5, 2, 1, 0, 0, 8},
    {256, 14, 14, 5, 2, 1, 0, 0, 8},
    {512, 14, 14, 5, 2, 1, 0, 0, 8},
    {256, 13, 13, 5, 2, 1, 0, 0, 8},
    {256, 14, 13, 5, 2, 1, 0, 0, 8},
    {256, 13, 14, 5, 2, 1, 0, 0, 8},
    {256, 14, 14, 5, 2, 1, 0, 0, 6},
    {256, 14, 14, 4, 2, 1, 0, 0, 8},
    {256, 15, 14, 5, 2, 1, 0, 0, 8},
  };
  int ncfg = sizeof(cfgs) / sizeof(cfgs[0]);
  for (int ki = 0; ki < 7; ki++) {
    dg_fill(buf, nch, cs, 0x5EED0003, kinds[ki], 0);
    size_t ref = 0;
    for (int i = 0; i < nch; i++) ref += ZSTD_compress(out, 200000, buf + (size_t)i * cs, cs, 3);
    printf("kind %d libzstd-L3 ratio %.4f\n", kinds[ki], (double)nch * cs / ref);
    for (int ci = 0; ci < ncfg; ci++) {
      size_t tot = 0, nseq = 0;
      for (int i = 0; i < nch; i++) {
        size_t ns = cfgs[ci].rep == 2 ? model2(buf + (size_t)i * cs, cs, cfgs[ci], seqs) : model(buf + (size_t)i * cs, cs, cfgs[ci], seqs);
        nseq += ns;
        ZSTD_CCtx_reset(cc, ZSTD_reset_session_and_parameters);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_compressionLevel, 3);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_blockDelimiters, ZSTD_sf_explicitBlockDelimiters);
        size_t r = ZSTD_compressSequences(cc, out, 200000, seqs, ns, buf + (size_t)i * cs, cs);
        if (ZSTD_isError(r)) { printf("err %s\n", ZSTD_getErrorName(r)); return 1; }
        tot += r;
      }
      cfg_t c = cfgs[ci];
      printf("  tile%3d hl%d hs%d mins%d rep%d lazy%d catch%d imm%d : ratio %.4f (%.3f of L3) seq/chunk %zu\n", c.tile, c.hl, c.hs, c.mins, c.rep, c.lazy, c.catchup, c.imm,
             (double)nch * cs / tot, (double)ref / tot, nseq / nch);
    }
  }
  return 0;
}

int g_maxml = 1 << 30;
int model3_rounds(const int *bl, int n, int lazy, int W, int S, int *maxr);
static size_t model2(const uint8_t *src, int n, cfg_t c, ZSTD_Sequence *seqs) {
  int *TL = malloc(sizeof(int) << c.hl), *TS = malloc(sizeof(int) << c.hs);
  int *bl = malloc(sizeof(int) * (n + 1)), *bo = malloc(sizeof(int) * (n + 1));
  for (int i = 0; i < (1 << c.hl); i++) TL[i] = -1;
  for (int i = 0; i < (1 << c.hs); i++) TS[i] = -1;
  int lim = n - 8; const uint8_t *end = src + n;
  for (int p = 0; p <= n; p++) { bl[p] = 0; bo[p] = 0; }
  for (int t = 0; t < lim; t += c.tile) {
    int e = t + c.tile < lim ? t + c.tile : lim;
    for (int p = t; p < e; p++) {
      uint64_t v = rd64(src + p); int qL = TL[hash8(v, c.hl)], qS = TS[hash5(v, c.hs, c.mins)];
      int lL = qL >= 0 ? cnt(src + p, src + qL, end) : 0, lS = qS >= 0 ? cnt(src + p, src + qS, end) : 0;
      if (lL > g_maxml) lL = g_maxml; if (lS > g_maxml) lS = g_maxml;
      if (lL < c.hl8) lL = 0;
      if (lS < c.mins) lS = 0;
      if (lL >= lS && lL) { bl[p] = lL; bo[p] = p - qL; } else if (lS) { bl[p] = lS; bo[p] = p - qS; }
    }
    for (int p = t; p < e; p++) { uint64_t v = rd64(src + p); TL[hash8(v, c.hl)] = p; TS[hash5(v, c.hs, c.mins)] = p; }
  }
  memcpy(g_bl, bl, sizeof(int) * (n + 1));
  int anchor = 0, p = 0; size_t ns = 0;
  while (p < lim) {
    if (bl[p] == 0 || (c.lazy && bl[p + 1] > bl[p] + c.lazy - 1)) { p++; continue; }
    seqs[ns].litLength = p - anchor; seqs[ns].offset = bo[p]; seqs[ns].matchLength = bl[p]; seqs[ns].rep = 0; ns++;
    p = anchor = p + bl[p];
  }
  seqs[ns].litLength = n - anchor; seqs[ns].offset = 0; seqs[ns].matchLength = 0; seqs[ns].rep = 0; ns++;
  free(TL); free(TS); free(bl); free(bo);
  return ns;
}

/* rounds needed by a Jacobi segment-parallel parse: window W, segment S */
int model3_rounds(const int *bl, int n, int lazy, int W, int S, int *maxr) {
  int lim = n - 8, tot = 0, nw = 0;
  int *nx = malloc(sizeof(int) * (n + 1)), *ex = malloc(sizeof(int) * (n + 1));
  for (int p = 0; p < n; p++) nx[p] = (p >= lim) ? p + 1 : (bl[p] == 0 || (lazy && bl[p + 1] > bl[p])) ? p + 1 : p + bl[p];
  int e = 0; *maxr = 0;
  for (int ws = 0; ws < n; ws += W) {
    int we = ws + W < n ? ws + W : n;
    for (int s = ws; s < we; s += S) { int se = s + S < we ? s + S : we; for (int p = se - 1; p >= s; p--) ex[p] = nx[p] >= se ? nx[p] : ex[nx[p]]; }
    int ns = (we - ws + S - 1) / S; int *ent = malloc(sizeof(int) * ns), *xt = malloc(sizeof(int) * ns);
    for (int k = 0; k < ns; k++) ent[k] = ws + k * S;
    int r = 0;
    for (;;) {
      r++;
      for (int k = 0; k < ns; k++) { int se = ws + (k + 1) * S; xt[k] = ent[k] < se && ent[k] < we ? ex[ent[k]] : ent[k]; }
      int ch = 0;
      for (int k = 0; k < ns; k++) { int ne = k == 0 ? e : xt[k - 1]; if (k == 0 && ne < ws) ne = ws; if (ne != ent[k]) { ch = 1; ent[k] = ne; } }
      if (!ch) break;
    }
    e = xt[ns - 1]; tot += r; nw++; if (r > *maxr) *maxr = r;
    free(ent); free(xt);
  }
  free(nx); free(ex);
  return tot / nw;
}

static int main2(void) {
  int nch = 64, cs = 65536;
  uint8_t *buf = malloc((size_t)nch * cs), *out = malloc(200000);
  ZSTD_Sequence *seqs = malloc(sizeof(ZSTD_Sequence) * cs);
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  int kinds[] = {0, 3, 6, 7, 8, 4};
  cfg_t c = {256, 14, 14, 5, 2, 1, 0, 0, 8};
  int caps[] = {1 << 30, 255, 128, 64};
  for (int ki = 0; ki < 6; ki++) {
    dg_fill(buf, nch, cs, 0x5EED0003, kinds[ki], 0);
    for (int ci = 0; ci < 4; ci++) {
      g_maxml = caps[ci];
      size_t tot = 0; long r16 = 0, r32 = 0, r64 = 0; int m16 = 0, m32 = 0, m64 = 0, mx;
      for (int i = 0; i < nch; i++) {
        size_t ns = model2(buf + (size_t)i * cs, cs, c, seqs);
        r16 += model3_rounds(g_bl, cs, 1, 4096, 16, &mx); if (mx > m16) m16 = mx;
        r32 += model3_rounds(g_bl, cs, 1, 8192, 32, &mx); if (mx > m32) m32 = mx;
        r64 += model3_rounds(g_bl, cs, 1, 16384, 64, &mx); if (mx > m64) m64 = mx;
        ZSTD_CCtx_reset(cc, ZSTD_reset_session_and_parameters);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_compressionLevel, 3);
        ZSTD_CCtx_setParameter(cc, ZSTD_c_blockDelimiters, ZSTD_sf_explicitBlockDelimiters);
        tot += ZSTD_compressSequences(cc, out, 200000, seqs, ns, buf + (size_t)i * cs, cs);
      }
      printf("kind %d cap %d ratio %.4f rounds(avg/max) S16 %ld/%d S32 %ld/%d S64 %ld/%d\n", kinds[ki], caps[ci], (double)nch * cs / tot, r16 / nch, m16, r32 / nch, m32, r64 / nch, m64);
    }
  }
  return 0;
}
