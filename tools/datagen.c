/*
 * datagen.c — seeded synthetic corpora for tests and bench (test/bench
 * infrastructure, not part of the compression product).
 *
 * BASELINE.md §2 / SURVEY.md §8(d) name the inputs:
 *   C1  1 MiB "dickens-like" English text           (kind DG_TEXT,   seed 0x5EED0001)
 *   C2  iid bytes over a seeded 16-symbol alphabet  (kind DG_SYM16,  seed 0x5EED0002)
 *   C3a Silesia-like per-chunk mix                  (kind DG_MIX,    seed 0x5EED0003)
 *   C3b uniform random bytes                        (kind DG_RANDOM, seed 0x5EED0004)
 *   C5  JSON-like records (template of the reference's
 *       tests/test_compressible_data.cu:40-62)      (kind DG_JSON,   seed 0x5EED0005)
 * Every chunk is generated from its own PRNG stream (seed, chunk index), so
 * the output does not depend on the thread count.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdio.h>

enum { DG_MIX = 0, DG_RANDOM = 1, DG_SYM16 = 2, DG_TEXT = 3, DG_JSON = 4,
       DG_SOURCE = 5, DG_CSV = 6, DG_EXE = 7, DG_SENSOR = 8 };

typedef struct { uint64_t s; } rng_t;
static inline uint64_t splitmix(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t rnext(rng_t *r) { return splitmix(&r->s); }
static inline uint32_t rbelow(rng_t *r, uint32_t n) {
  return (uint32_t)(((rnext(r) >> 32) * (uint64_t)n) >> 32);
}

/* ---------------- vocabulary (fixed, independent of the data seed) ------- */
#define VOCAB 4096
static char g_words[VOCAB][16];
static uint8_t g_wlen[VOCAB];
static uint32_t g_zipf_cdf[VOCAB]; /* scaled to 2^32-1 */
static int g_init = 0;

static const char k_letters[] = "eeeeeeeeeeeetttttttttaaaaaaaaooooooooiiiiiiinnnnnnnsssssshhhhhhrrrrrrddddllllcccuuummmwwffggyyppbbvk";

static void vocab_init(void) {
  if (g_init) return;
  rng_t r = {0xC0FFEE123ull};
  for (int i = 0; i < VOCAB; i++) {
    /* frequent words are short */
    int len = 1 + (int)rbelow(&r, 3) + (int)rbelow(&r, 3 + (i < 64 ? 0 : (i < 512 ? 3 : 7)));
    if (len > 14) len = 14;
    for (int k = 0; k < len; k++) g_words[i][k] = k_letters[rbelow(&r, sizeof(k_letters) - 1)];
    g_wlen[i] = (uint8_t)len;
  }
  double h = 0, acc = 0;
  for (int i = 0; i < VOCAB; i++) h += 1.0 / __builtin_pow(i + 1.0, 1.15);
  for (int i = 0; i < VOCAB; i++) {
    acc += 1.0 / __builtin_pow(i + 1.0, 1.15) / h;
    double v = acc * 4294967295.0;
    g_zipf_cdf[i] = v > 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
  }
  g_zipf_cdf[VOCAB - 1] = 0xFFFFFFFFu;
  g_init = 1;
}

static inline int zipf_word(rng_t *r) {
  uint32_t u = (uint32_t)(rnext(r) >> 32);
  int lo = 0, hi = VOCAB - 1;
  while (lo < hi) { int mid = (lo + hi) >> 1; if (g_zipf_cdf[mid] < u) lo = mid + 1; else hi = mid; }
  return lo;
}

typedef struct { uint8_t *p; size_t n, cap; } out_t;
static inline void put(out_t *o, const void *s, size_t k) {
  if (o->n >= o->cap) return;
  if (k > o->cap - o->n) k = o->cap - o->n;
  memcpy(o->p + o->n, s, k); o->n += k;
}
static inline void putc1(out_t *o, char c) { if (o->n < o->cap) o->p[o->n++] = (uint8_t)c; }
static void putnum(out_t *o, uint64_t v) { char b[24]; int k = 0; do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v); while (k) putc1(o, b[--k]); }

static void gen_text(out_t *o, rng_t *r) {
  while (o->n < o->cap) {
    int nsent = 3 + (int)rbelow(r, 6);
    for (int s = 0; s < nsent && o->n < o->cap; s++) {
      int nw = 5 + (int)rbelow(r, 16);
      if (o->n > 2048 && rbelow(r, 3) == 0) { /* re-use an earlier phrase */
        size_t from = (size_t)rbelow(r, (uint32_t)(o->n - 64)), k = 16 + rbelow(r, 48);
        put(o, o->p + from, k); putc1(o, ' ');
      }
      for (int w = 0; w < nw; w++) {
        int id = zipf_word(r);
        if (w == 0) { putc1(o, (char)(g_words[id][0] - 32)); put(o, g_words[id] + 1, g_wlen[id] - 1); }
        else put(o, g_words[id], g_wlen[id]);
        if (w + 1 < nw) { if (rbelow(r, 12) == 0) putc1(o, ','); putc1(o, ' '); }
      }
      putc1(o, rbelow(r, 10) == 0 ? '?' : '.');
      putc1(o, ' ');
    }
    put(o, "\n\n", 2);
  }
}

static const char *k_tags[] = {"record", "item", "entry", "node", "value", "field", "name", "data"};
static const char *k_kw[] = {"if", "for", "while", "return", "int", "static", "const", "void", "struct", "else"};
static void gen_source(out_t *o, rng_t *r) {
  int depth = 1;
  while (o->n < o->cap) {
    int kind = (int)rbelow(r, 3);
    for (int d = 0; d < depth; d++) put(o, "  ", 2);
    if (kind == 0) {
      const char *t = k_tags[rbelow(r, 8)];
      putc1(o, '<'); put(o, t, strlen(t)); put(o, " id=\"", 5); putnum(o, rbelow(r, 5000));
      put(o, "\" type=\"", 8); int w = zipf_word(r); put(o, g_words[w], g_wlen[w]); put(o, "\">", 2);
      int nw = 1 + (int)rbelow(r, 4);
      for (int k = 0; k < nw; k++) { int x = zipf_word(r); put(o, g_words[x], g_wlen[x]); if (k + 1 < nw) putc1(o, ' '); }
      put(o, "</", 2); put(o, t, strlen(t)); put(o, ">\n", 2);
    } else if (kind == 1) {
      const char *k = k_kw[rbelow(r, 10)]; put(o, k, strlen(k)); put(o, " (", 2);
      int a = zipf_word(r); put(o, g_words[a], g_wlen[a]); put(o, "_", 1); putnum(o, rbelow(r, 32));
      put(o, " > ", 3); putnum(o, rbelow(r, 100)); put(o, ") {\n", 4);
      if (depth < 6) depth++;
    } else {
      int a = zipf_word(r), b = zipf_word(r);
      put(o, g_words[a], g_wlen[a]); put(o, " = ", 3); put(o, g_words[b], g_wlen[b]); put(o, "(", 1);
      putnum(o, rbelow(r, 64)); put(o, ", ", 2); int c = zipf_word(r); put(o, g_words[c], g_wlen[c]); put(o, ");\n", 3);
      if (depth > 1 && rbelow(r, 3) == 0) { depth--; for (int d = 0; d < depth; d++) put(o, "  ", 2); put(o, "}\n", 2); }
    }
  }
}

static const char *k_first[] = {"James", "Mary", "John", "Linda", "Robert", "Susan", "Michael", "Karen", "David", "Lisa", "Maria", "Wei", "Ahmed", "Yuki", "Olga", "Pierre"};
static const char *k_last[] = {"Smith", "Jones", "Brown", "Garcia", "Miller", "Davis", "Wilson", "Lee", "Martin", "Clark", "Lewis", "Walker", "Young", "King", "Wright", "Scott"};
static const char *k_cat[] = {"books", "garden", "tools", "toys", "music", "sports", "food", "health"};
static void gen_csv(out_t *o, rng_t *r, uint64_t base_id) {
  uint64_t id = base_id;
  while (o->n < o->cap) {
    const char *f = k_first[rbelow(r, 16)], *l = k_last[rbelow(r, 16)];
    putnum(o, id++); putc1(o, ','); put(o, f, strlen(f)); putc1(o, ' '); put(o, l, strlen(l)); putc1(o, ',');
    for (const char *c = f; *c; c++) putc1(o, (char)(*c | 32)); putc1(o, '.');
    for (const char *c = l; *c; c++) putc1(o, (char)(*c | 32)); put(o, "@example.com,", 13);
    put(o, "2023-", 5); int m = 1 + (int)rbelow(r, 12); putc1(o, (char)('0' + m / 10)); putc1(o, (char)('0' + m % 10));
    putc1(o, '-'); int d = 1 + (int)rbelow(r, 28); putc1(o, (char)('0' + d / 10)); putc1(o, (char)('0' + d % 10));
    putc1(o, ','); putnum(o, rbelow(r, 100000)); putc1(o, '.'); putnum(o, 10 + rbelow(r, 90)); putc1(o, ',');
    const char *c = k_cat[rbelow(r, 8)]; put(o, c, strlen(c)); putc1(o, ',');
    { int t = (int)rbelow(r, 2); put(o, t ? "true" : "false", t ? 4 : 5); } putc1(o, '\n');
  }
}

static void gen_exe(out_t *o, rng_t *r) {
  /* fixed idiom table + skewed single-byte opcode distribution */
  uint8_t idioms[64][8]; uint8_t ilen[64];
  rng_t ir = {0xE7Eull};
  for (int i = 0; i < 64; i++) { ilen[i] = (uint8_t)(2 + rbelow(&ir, 7)); for (int k = 0; k < ilen[i]; k++) idioms[i][k] = (uint8_t)(rnext(&ir) >> 56); }
  uint32_t base = 0x00401000u + (uint32_t)rbelow(r, 0x10000) * 16;
  while (o->n < o->cap) {
    uint32_t c = rbelow(r, 100);
    if (c < 52) { int i = (int)(rbelow(r, 64) * rbelow(r, 64) / 64); put(o, idioms[i], ilen[i]); }
    else if (c < 64) { uint32_t a = base + rbelow(r, 512) * 4; putc1(o, (char)0xE8); put(o, &a, 4); }
    else if (c < 67) { int z = 4 + (int)rbelow(r, 24); for (int k = 0; k < z; k++) putc1(o, 0); }
    else { uint32_t g = rbelow(r, 256); g = (g * g) >> 8; g = (g * 0x9Du + 0x3B) & 0xFF; putc1(o, (char)g); }
  }
}

static void gen_sensor(out_t *o, rng_t *r) {
  int32_t v = 20000 + (int32_t)rbelow(r, 20000);
  while (o->n + 2 <= o->cap) {
    int32_t d = (int32_t)rbelow(r, 9) - 4 + ((int32_t)rbelow(r, 5) - 2) * (rbelow(r, 8) == 0);
    v += d; if (v < 0) v = 0; if (v > 65535) v = 65535;
    uint16_t u = (uint16_t)v; put(o, &u, 2);
  }
  if (o->n < o->cap) putc1(o, 0);
}

static void gen_json(out_t *o, rng_t *r, uint64_t base_id) {
  uint64_t id = base_id;
  while (o->n < o->cap) {
    const char *f = k_first[rbelow(r, 16)], *l = k_last[rbelow(r, 16)];
    put(o, "{\"id\":", 6); putnum(o, id++); put(o, ",\"name\":\"", 9); put(o, f, strlen(f)); putc1(o, ' ');
    put(o, l, strlen(l)); put(o, "\",\"email\":\"", 11);
    for (const char *c = f; *c; c++) putc1(o, (char)(*c | 32)); putnum(o, rbelow(r, 1000));
    put(o, "@example.com\",\"active\":", 23); { int t = (int)rbelow(r, 2); put(o, t ? "true" : "false", t ? 4 : 5); }
    put(o, ",\"score\":", 9); putnum(o, rbelow(r, 1000)); put(o, ",\"tags\":[\"", 10);
    const char *c = k_cat[rbelow(r, 8)]; put(o, c, strlen(c)); put(o, "\"]}\n", 4);
  }
}

static void gen_chunk(uint8_t *dst, size_t n, uint64_t seed, uint64_t idx, int kind) {
  rng_t r; r.s = seed * 0x100000001B3ull ^ (idx + 1) * 0x9E3779B97F4A7C15ull; rnext(&r);
  out_t o = {dst, 0, n};
  if (kind == DG_MIX) {
    uint32_t c = rbelow(&r, 100);
    kind = c < 27 ? DG_TEXT : c < 39 ? DG_SOURCE : c < 59 ? DG_CSV : c < 86 ? DG_EXE : DG_SENSOR;
  }
  switch (kind) {
  case DG_RANDOM: { size_t i = 0; for (; i + 8 <= n; i += 8) { uint64_t v = rnext(&r); memcpy(dst + i, &v, 8); }
                    for (; i < n; i++) dst[i] = (uint8_t)rnext(&r); break; }
  case DG_SYM16: { uint8_t alpha[16]; rng_t ar = {seed ^ 0xA1FAull}; for (int k = 0; k < 16; k++) alpha[k] = (uint8_t)(rnext(&ar) >> 56);
                   for (size_t i = 0; i < n; i += 16) { uint64_t v = rnext(&r); for (int k = 0; k < 16 && i + k < n; k++) dst[i + k] = alpha[(v >> (4 * k)) & 15]; } break; }
  case DG_TEXT: gen_text(&o, &r); break;
  case DG_SOURCE: gen_source(&o, &r); break;
  case DG_CSV: gen_csv(&o, &r, idx * 700 + 1000); break;
  case DG_EXE: gen_exe(&o, &r); break;
  case DG_SENSOR: gen_sensor(&o, &r); break;
  case DG_JSON: gen_json(&o, &r, idx * 200 + 1); break;
  default: memset(dst, 0, n);
  }
}

/* Fill n_chunks × chunk_size bytes; chunk i comes from stream (seed, first_chunk + i). */
void dg_fill(uint8_t *dst, size_t n_chunks, size_t chunk_size, uint64_t seed, int kind, uint64_t first_chunk) {
  vocab_init();
#pragma omp parallel for schedule(dynamic, 16)
  for (long i = 0; i < (long)n_chunks; i++) gen_chunk(dst + (size_t)i * chunk_size, chunk_size, seed, first_chunk + (uint64_t)i, kind);
}
