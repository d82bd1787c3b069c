/*
 * cpubench.c — host libzstd baseline (BASELINE.md §2 "CPU baseline"): one ZSTD_CCtx (or
 * ZSTD_DCtx) per POSIX thread, ZSTD_compressCCtx / ZSTD_decompressDCtx over the same
 * 64 KiB chunks the GPU compresses, chunks handed out by an atomic counter.  libzstd is
 * the reference's own CPU route (src/cuda_zstd_manager.cu:1604-1668,
 * src/cuda_zstd_hybrid.cu:402-458); it is loaded with dlopen so this library has no link
 * dependency.  Bench infrastructure only (bench.py's cpu_baseline leg).
 *
 *   cpub_run(mode, data, nchunks, chunk, level, threads, passes, secs[], comp_bytes)
 *     mode 0: compress `nchunks` chunks of `chunk` bytes at `data`;
 *     mode 1: decompress frames (data = slot-strided frames, sizes[] their lengths).
 *   Each pass is one whole sweep of the sample; secs[p] is its wall time.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
/* AddressSanitizer refuses RTLD_DEEPBIND dlopens: sanitizer builds open libzstd without it */
#if defined(__SANITIZE_ADDRESS__)
#define CPB_DEEPBIND 0
#elif defined(__has_feature)
#if __has_feature(address_sanitizer)
#define CPB_DEEPBIND 0
#endif
#endif
#ifndef CPB_DEEPBIND
#define CPB_DEEPBIND RTLD_DEEPBIND
#endif
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef void *(*create_fn)(void);
typedef size_t (*free_fn)(void *);
typedef size_t (*cctx_fn)(void *, void *, size_t, const void *, size_t, int);
typedef size_t (*dctx_fn)(void *, void *, size_t, const void *, size_t);
typedef unsigned (*iserr_fn)(size_t);
typedef size_t (*bound_fn)(size_t);

static struct {
  create_fn create_c, create_d;
  free_fn free_c, free_d;
  cctx_fn comp;
  dctx_fn decomp;
  iserr_fn is_error;
  bound_fn bound;
  unsigned (*version)(void);
  int ok;
} Z;

static int load(void) {
  if (Z.ok) return 0;
  const char *names[] = {"libzstd.so.1", "/opt/conda/lib/libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1", "libzstd.so"};
  for (unsigned i = 0; i < sizeof(names) / sizeof(names[0]); i++) {
    void *h = dlopen(names[i], RTLD_NOW | RTLD_LOCAL | CPB_DEEPBIND);  /* (one image, see tests/zh_testlib.py) */
    if (!h) continue;
    Z.create_c = (create_fn)dlsym(h, "ZSTD_createCCtx");
    Z.create_d = (create_fn)dlsym(h, "ZSTD_createDCtx");
    Z.free_c = (free_fn)dlsym(h, "ZSTD_freeCCtx");
    Z.free_d = (free_fn)dlsym(h, "ZSTD_freeDCtx");
    Z.comp = (cctx_fn)dlsym(h, "ZSTD_compressCCtx");
    Z.decomp = (dctx_fn)dlsym(h, "ZSTD_decompressDCtx");
    Z.is_error = (iserr_fn)dlsym(h, "ZSTD_isError");
    Z.bound = (bound_fn)dlsym(h, "ZSTD_compressBound");
    Z.version = (unsigned (*)(void))dlsym(h, "ZSTD_versionNumber");
    if (Z.create_c && Z.create_d && Z.free_c && Z.free_d && Z.comp && Z.decomp && Z.is_error && Z.bound && Z.version) {
      Z.ok = 1;
      return 0;
    }
  }
  return -1;
}

unsigned cpub_zstd_version(void) { return load() ? 0 : Z.version(); }

typedef struct {
  int mode, level;
  const uint8_t *data;
  const size_t *sizes;  /* mode 1: frame sizes */
  size_t nchunks, chunk, slot;
  atomic_size_t next;
  atomic_size_t out_bytes;
  atomic_int err;
} Job;

static void *worker(void *arg) {
  Job *j = (Job *)arg;
  size_t const cap = j->mode == 0 ? Z.bound(j->chunk) : j->chunk;
  uint8_t *buf = (uint8_t *)malloc(cap);
  void *ctx = j->mode == 0 ? Z.create_c() : Z.create_d();
  size_t tot = 0;
  if (buf && ctx) {
    for (;;) {
      size_t const i = atomic_fetch_add(&j->next, 1);
      if (i >= j->nchunks) break;
      size_t r;
      if (j->mode == 0)
        r = Z.comp(ctx, buf, cap, j->data + i * j->chunk, j->chunk, j->level);
      else
        r = Z.decomp(ctx, buf, cap, j->data + i * j->slot, j->sizes[i]);
      if (Z.is_error(r)) { atomic_store(&j->err, 1); break; }
      tot += r;
    }
  } else {
    atomic_store(&j->err, 1);
  }
  atomic_fetch_add(&j->out_bytes, tot);
  if (ctx) { if (j->mode == 0) Z.free_c(ctx); else Z.free_d(ctx); }
  free(buf);
  return NULL;
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

/* Returns 0 on success; secs[0..passes) = wall time of each pass, *out_bytes = bytes one
 * pass produced (compressed bytes for mode 0, decompressed bytes for mode 1). */
/* cpus (optional, `threads` entries): thread t runs pinned to CPU cpus[t] (bench.py's SMT
 * measurement: one core's two hardware threads against one thread alone). */
int cpub_run_pinned(int mode, const uint8_t *data, const size_t *sizes, size_t nchunks, size_t chunk, size_t slot, int level, int threads,
                    int passes, double *secs, size_t *out_bytes, const int *cpus);
int cpub_run(int mode, const uint8_t *data, const size_t *sizes, size_t nchunks, size_t chunk, size_t slot, int level, int threads, int passes,
             double *secs, size_t *out_bytes) {
  return cpub_run_pinned(mode, data, sizes, nchunks, chunk, slot, level, threads, passes, secs, out_bytes, NULL);
}
int cpub_run_pinned(int mode, const uint8_t *data, const size_t *sizes, size_t nchunks, size_t chunk, size_t slot, int level, int threads,
                    int passes, double *secs, size_t *out_bytes, const int *cpus) {
  if (load() || threads < 1 || passes < 1 || (mode == 1 && !sizes)) return -1;
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  if (!th) return -1;
  int rc = 0;
  for (int p = 0; p < passes && !rc; p++) {
    Job j;
    memset(&j, 0, sizeof(j));
    j.mode = mode;
    j.level = level;
    j.data = data;
    j.sizes = sizes;
    j.nchunks = nchunks;
    j.chunk = chunk;
    j.slot = slot;
    double const t0 = now();
    int started = 0;
    for (int t = 0; t < threads; t++, started++) {
      pthread_attr_t at;
      pthread_attr_init(&at);
      if (cpus) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(cpus[t], &cs);
        pthread_attr_setaffinity_np(&at, sizeof(cs), &cs);
      }
      int const e = pthread_create(&th[t], &at, worker, &j);
      pthread_attr_destroy(&at);
      if (e) { rc = -1; break; }
    }
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    secs[p] = now() - t0;
    if (atomic_load(&j.err)) rc = -2;
    *out_bytes = atomic_load(&j.out_bytes);
  }
  free(th);
  return rc;
}
