/* CPU model of the deep matcher's demand-driven walk (zh_lz_deep.hip deep_parse_demand): the
 * segment walks, the per-wave search rounds and the Jacobi iterations, on the oracle's per-position
 * matches (orc_lz_parse_deep's len/off).  Counts what costs time on the GPU -- search rounds per
 * wave (a round lasts as long as its slowest search) and Jacobi iterations (one workgroup barrier
 * each) -- for entry rules and queue widths, and checks that every variant's parse equals the
 * serial LAZY2 parse.  Diagnostic tool, not part of the product.
 *   gcc -O2 -o /tmp/deepsim tools/deep_jacobi_model.c && /tmp/deepsim records.bin 16384 [dict.bin]
 * On 64 C5 records (no dictionary, 16-position segments) it reproduces the GPU's 10.9 search rounds
 * and 37.6 % of positions searched; a prefix-max entry rule and speculative posting at p + len
 * change nothing, a warm-up walk before each segment cuts the Jacobi iterations (4.2 -> 2.2 at 32
 * positions), which the GPU confirmed once duplicate searches were claimed away;
 * dealing segments to waves round-robin instead of in 64-segment runs needs more passes (the
 * slowest wave's first walk 13.7 -> 18.7 at 16 positions + 32 warm-up; runs of 32: 12.9), and so
 * does posting 4-8 positions after a literal step (13.4-13.8).  The slowest wave is the one over
 * the record's first KiB (few matches yet: almost every position searched, PERWAVE=1 prints the
 * per-wave passes), about 1.65 x the mean wave.
 */
#include "../oracle/zstd_oracle.c"
#include <stdio.h>

#define DEPTH 32
static u8 *LEN;
static u32 *OFF;
static u16 *MEMO; /* 1 = known */
static u32 NB, PRE, N, LIM;

static int gain(u32 p) { return (p < NB && LEN[p]) ? 4 * (int)LEN[p] - (31 - __builtin_clz(OFF[p] + 1u)) : -1000; }

static void matches(const u8 *buf, u32 pre, u32 n) {
  u32 const lim = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  u32 *prev = malloc(sizeof(u32) * (lim + 1));
  u32 *head = calloc((size_t)1 << ZH_HASH_LOG_SHORT, sizeof(u32));
  for (u32 p = 0; p < lim; p++) {
    u32 const h = zh_hash_short(rd64(buf + p));
    prev[p] = head[h];
    head[h] = p + 1;
  }
  for (u32 i = 0; i + pre < n + 3; i++) { LEN[i] = 0; OFF[i] = 0; }
  for (u32 p = pre; p < lim; p++) {
    u32 best = 0, bo = 0, c = prev[p];
    for (u32 d = 0; d < DEPTH && c && p - (c - 1) <= ZH_DEEP_MAXOFF; d++) {
      u32 const q = c - 1, l = common_prefix(buf, p, q, n, ZH_MAX_MATCH);
      if (l >= ZH_MIN_MATCH_SHORT && l > best) { best = l; bo = p - q; if (best >= ZH_MAX_MATCH) break; }
      c = prev[q];
    }
    LEN[p - pre] = (u8)best;
    OFF[p - pre] = bo;
  }
  free(prev); free(head);
}

/* one lane's walk state */
typedef struct { u32 S, SE, p, need, spec, ent; int lit; int act, adv, merged; u32 mpos; u64 nl, nm, old; } Lane;

static int DQ = 3, SEGL = 16, RULE = 0, SPEC = 0, WARM = 0, INTER = 0, DQL = 0; /* INTER: segments dealt to waves in runs of INTER (0: 64); DQL: posts after a literal step */ /* INTER: wave w takes segments w, w + nw, ... */
static u32 NW = 16; /* RULE 0: predecessor's exit, 1: prefix max of exits */
static long searched;

/* walk of the lanes [w*64, w*64+64) with act0 set, from p0[]; returns the wave's search passes */
static int walk_wave(u32 w, u32 nseg, const u32 *p0, const int *act0, u64 *LM, u64 *MM, u32 *ex, u32 *entry_out, u32 warm) {
  Lane L[64];
  for (int l = 0; l < 64; l++) {
    u32 g = INTER ? ((l / INTER) * NW + w) * INTER + l % INTER : w * 64 + l;
    Lane *x = &L[l];
    memset(x, 0, sizeof *x);
    if (g >= nseg) continue;
    x->S = SEGL * g; x->SE = x->S + SEGL < NB ? x->S + SEGL : NB;
    x->old = act0[g] ? (LM[g] | MM[g]) : 0;
    x->act = act0[g] && p0[g] < x->SE;
    x->p = p0[g] >= warm ? p0[g] - warm : 0;
    x->ent = x->p >= x->S ? x->p : ~0u;
  }
  int rounds = 0;
  for (;;) {
    int any = 0;
    for (int l = 0; l < 64; l++) {
      Lane *x = &L[l];
      x->need = ~0u;
      x->spec = ~0u;
      x->adv = x->act;
      while (x->adv) {
        u32 p = x->p;
        if (p >= x->SE) { x->act = x->adv = 0; if (x->ent == ~0u) x->ent = p; break; }
        if (p >= x->S && x->ent == ~0u) x->ent = p;
        if (p >= x->S && ((x->old >> (p - x->S)) & 1)) { x->merged = 1; x->mpos = p - x->S; x->act = x->adv = 0; break; }
        if (!MEMO[p]) { x->need = p; x->adv = 0; break; }
        if (!LEN[p]) { if (p >= x->S) x->nl |= 1ull << (p - x->S); x->p++; x->lit = 1; continue; }
        int k1 = p + 1 < NB && !MEMO[p + 1], k2 = p + 2 < NB && !MEMO[p + 2];
        if (k1 || k2) {
          x->need = k1 ? p + 1 : p + 2;
          x->adv = 0;
          if (SPEC && p + LEN[p] < x->SE) x->spec = p + LEN[p];  /* where the walk goes if it takes p's match */
          break;
        }
        int g0 = gain(p);
        if (gain(p + 1) > g0 + 4 || gain(p + 2) > g0 + 7) { if (p >= x->S) x->nl |= 1ull << (p - x->S); x->p++; x->lit = 1; }
        else { if (p >= x->S) x->nm |= 1ull << (p - x->S); x->p += LEN[p]; x->lit = 0; }
      }
      any |= x->act;
    }
    if (!any) break;
    int nq = 0;
    for (int l = 0; l < 64; l++) {
      if (L[l].need == ~0u) continue;
      for (int t = 0; t < ((DQL && L[l].lit) ? DQL : DQ); t++) {
        u32 xx = L[l].need + t;
        if (xx < NB && !MEMO[xx]) { MEMO[xx] = 1; searched++; nq++; }
      }
      if (L[l].spec != ~0u)
        for (int t = 0; t < SPEC; t++) {
          u32 xx = L[l].spec + t;
          if (xx < NB && !MEMO[xx]) { MEMO[xx] = 1; searched++; nq++; }
        }
    }
    rounds += (nq + 63) / 64; /* search passes: lanes = queue entries, 64 at a time */
  }
  for (int l = 0; l < 64; l++) {
    u32 g = INTER ? ((l / INTER) * NW + w) * INTER + l % INTER : w * 64 + l;
    if (g >= nseg || !act0[g]) continue;
    Lane *x = &L[l];
    if (x->merged) {
      u64 keep = x->mpos >= 64 ? 0 : ~0ull << x->mpos;
      LM[g] = x->nl | (LM[g] & keep);
      MM[g] = x->nm | (MM[g] & keep);
    } else {
      LM[g] = x->nl; MM[g] = x->nm; ex[g] = x->p;
    }
    if (entry_out) entry_out[g] = x->ent;
  }
  return rounds;
}

/* returns the parse's match count; prints the cost figures */
static void model(const u8 *buf, u32 pre, u32 n, long *acc) {
  PRE = pre; N = n; NB = n - pre; LIM = n > ZH_HASH_READ ? n - ZH_HASH_READ : 0;
  matches(buf, pre, n);
  for (u32 i = 0; i < NB; i++) MEMO[i] = pre + i < LIM ? 0 : 1;
  u32 const nseg = (NB + SEGL - 1) / SEGL, nw = (nseg + 63) / 64;
  NW = nw;
  u32 *entry = calloc(nseg, 4), *ex = calloc(nseg, 4), *ne = calloc(nseg, 4);
  u64 *LM = calloc(nseg, 8), *MM = calloc(nseg, 8);
  int *act = calloc(nseg, sizeof(int));
  searched = 0;
  for (u32 g = 0; g < nseg; g++) { entry[g] = SEGL * g; ex[g] = entry[g]; act[g] = 1; }
  int r0 = 0, rsum = 0;
  for (u32 w = 0; w < nw; w++) { int r = walk_wave(w, nseg, entry, act, LM, MM, ex, WARM ? entry : NULL, WARM); if (r > r0) r0 = r; rsum += r; }
  acc[7] += rsum; acc[8] += nw;
  if (getenv("PERWAVE") && WARM == 32 && !INTER) {  /* per-wave first-walk passes (fresh memo) */
    static int once = 0;
    if (once++ < 3) {
      for (u32 i = 0; i < NB; i++) MEMO[i] = pre + i < LIM ? 0 : 1;
      for (u32 g = 0; g < nseg; g++) { entry[g] = SEGL * g; ex[g] = entry[g]; act[g] = 1; LM[g] = MM[g] = 0; }
      fprintf(stderr, "per-wave:");
      for (u32 w = nw; w-- > 0;) fprintf(stderr, " %d", walk_wave(w, nseg, entry, act, LM, MM, ex, entry, WARM));
      fprintf(stderr, "  (waves %u..0, walked last to first)\n", nw - 1);
    }
  }
  entry[0] = 0;
  int iters = 0, rj = 0;
  for (;;) {
    int anych = 0;
    u32 run = 0;
    for (u32 g = 0; g < nseg; g++) {
      u32 e = g == 0 ? 0 : (RULE ? run : ex[g - 1]);
      if (RULE) run = run > ex[g] ? run : ex[g];
      ne[g] = e;
      act[g] = e != entry[g];
      anych |= act[g];
    }
    if (!anych) break;
    iters++;
    int rm = 0;
    for (u32 w = 0; w < nw; w++) { int r = walk_wave(w, nseg, ne, act, LM, MM, ex, NULL, 0); if (r > rm) rm = r; }
    rj += rm;
    for (u32 g = 0; g < nseg; g++) if (act[g]) entry[g] = ne[g];
  }
  /* the walk's parse vs the serial LAZY2 parse */
  u32 p = 0, ok = 1, nmatch = 0;
  while (p < NB && pre + p < LIM) {
    int take = LEN[p] && !(gain(p + 1) > gain(p) + 4 || gain(p + 2) > gain(p) + 7);
    u32 g = p / SEGL, o = p - SEGL * g;
    int bit = take ? (int)((MM[g] >> o) & 1) : (int)((LM[g] >> o) & 1);
    if (!bit) { ok = 0; break; }
    if (take) { nmatch++; p += LEN[p]; } else p++;
  }
  acc[0] += r0; acc[1] += iters; acc[2] += rj; acc[3] += searched; acc[4] += ok; acc[5] += nmatch; acc[6] += NB;
  free(entry); free(ex); free(ne); free(LM); free(MM); free(act);
}

int main(int argc, char **argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s records.bin recsize [dict.bin]\n", argv[0]); return 2; }
  FILE *f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  u8 *data = malloc(sz);
  if (fread(data, 1, sz, f) != (size_t)sz) return 1;
  fclose(f);
  u32 rec = (u32)atoi(argv[2]), nrec = (u32)(sz / rec);
  u8 *dict = NULL;
  u32 dn = 0;
  if (argc > 3) {
    f = fopen(argv[3], "rb");
    fseek(f, 0, SEEK_END);
    dn = (u32)ftell(f);
    fseek(f, 0, SEEK_SET);
    dict = malloc(dn);
    if (fread(dict, 1, dn, f) != dn) return 1;
    fclose(f);
  }
  u8 *buf = malloc(dn + rec + 64);
  LEN = malloc(rec + 64);
  OFF = malloc(4 * (rec + 64));
  MEMO = malloc(2 * (rec + 64));
  static const int cfg[][7] = {{3, 16, 0, 0, 0, 0, 0}, {3, 16, 1, 0, 0, 0, 0}, {3, 16, 0, 3, 0, 0, 0}, {3, 16, 0, 0, 32, 0, 0}, {3, 16, 0, 0, 32, 1, 0},
                               {3, 16, 0, 0, 32, 32, 0}, {3, 16, 0, 0, 32, 0, 6}, {3, 32, 0, 0, 0, 0, 0}, {3, 32, 0, 0, 64, 0, 0}};
  /* DQ, SEGL, rule, spec, warm-up, run of segments per wave (0: 64), posts after a literal */  /* DQ, SEGL, rule, spec, warm-up, run of segments per wave (0: 64), posts after a literal */  /* DQ, SEGL, rule, spec, warm-up, interleave, posts after a literal */  /* DQ, SEGL, rule, spec, warm-up, interleave */  /* DQ, SEGL, rule, spec, warm-up */
  for (u32 c = 0; c < sizeof cfg / sizeof cfg[0]; c++) {
    DQ = cfg[c][0]; SEGL = cfg[c][1]; RULE = cfg[c][2]; SPEC = cfg[c][3]; WARM = cfg[c][4]; INTER = cfg[c][5]; DQL = cfg[c][6];
    long acc[9] = {0};
    for (u32 r = 0; r < nrec; r++) {
      if (dn) memcpy(buf, dict, dn);
      memcpy(buf + dn, data + (size_t)r * rec, rec);
      memset(buf + dn + rec, 0, 64);
      model(buf, dn, dn + rec, acc);
    }
    printf("DQ %d/%d spec %d warm %d inter %d SEGL %d rule %s: first-walk passes %.2f (wave mean %.2f), Jacobi iterations %.2f, Jacobi passes %.2f, total passes %.2f, "
           "searched %.1f%%, parse ok %ld/%u\n",
           DQ, DQL, SPEC, WARM, INTER, SEGL, RULE ? "prefix-max" : "predecessor", (double)acc[0] / nrec, (double)acc[7] / acc[8], (double)acc[1] / nrec, (double)acc[2] / nrec,
           (double)(acc[0] + acc[2]) / nrec, 100.0 * acc[3] / acc[6], acc[4], nrec);
  }
  return 0;
}
