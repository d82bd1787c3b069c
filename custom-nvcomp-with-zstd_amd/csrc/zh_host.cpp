// zh_host.cpp — C++17 host runtime: managers, workspace planning, C ABI.
//
// Host side of the reference's L3/L4: ZstdBatchManager /
// NvcompV5BatchManager / HybridEngine / C API, redesigned around one batched
// device pipeline (K1 zh_lz_kernel -> K2 zh_entropy_kernel -> [K3 gather]) with a
// single host synchronisation per call instead of the reference's ~13 per block
// (src/cuda_zstd_manager.cu:2328-3112).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
// AddressSanitizer refuses RTLD_DEEPBIND dlopens: sanitizer builds of the host code
// open libzstd without it
#if defined(__SANITIZE_ADDRESS__)
#define ZH_DLOPEN_DEEPBIND 0
#elif defined(__has_feature)
#if __has_feature(address_sanitizer)
#define ZH_DLOPEN_DEEPBIND 0
#endif
#endif
#ifndef ZH_DLOPEN_DEEPBIND
#define ZH_DLOPEN_DEEPBIND RTLD_DEEPBIND
#endif

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "cuda_zstd_hybrid.h"
#include "cuda_zstd_manager.h"
#include "cuda_zstd_nvcomp.h"
#include "zh_dict.h"
#include "zh_launch.h"

namespace cuda_zstd {

// ============================================================================
// status strings (reference src/cuda_zstd_types.cpp:36-79)
// ============================================================================
const char *status_to_string(Status s) {
  switch (s) {
    case Status::SUCCESS: return "Success";
    case Status::ERROR_GENERIC: return "Generic error";
    case Status::ERROR_INVALID_PARAMETER: return "Invalid parameter";
    case Status::ERROR_OUT_OF_MEMORY: return "Out of memory";
    case Status::ERROR_CUDA_ERROR: return "HIP runtime error";
    case Status::ERROR_INVALID_MAGIC: return "Invalid magic number";
    case Status::ERROR_CORRUPT_DATA: return "Corrupt data";
    case Status::ERROR_BUFFER_TOO_SMALL: return "Buffer too small";
    case Status::ERROR_UNSUPPORTED_VERSION: return "Unsupported version";
    case Status::ERROR_DICTIONARY_MISMATCH: return "Dictionary mismatch";
    case Status::ERROR_CHECKSUM_FAILED: return "Checksum failed";
    case Status::ERROR_IO: return "I/O error";
    case Status::ERROR_COMPRESSION: return "Compression error";
    case Status::ERROR_DECOMPRESSION: return "Decompression error";
    case Status::ERROR_WORKSPACE_INVALID: return "Workspace invalid";
    case Status::ERROR_STREAM_ERROR: return "Stream error";
    case Status::ERROR_ALLOCATION_FAILED: return "Allocation failed";
    case Status::ERROR_HASH_TABLE_FULL: return "Hash table full";
    case Status::ERROR_SEQUENCE_ERROR: return "Sequence error";
    case Status::ERROR_NOT_INITIALIZED: return "Not initialized";
    case Status::ERROR_ALREADY_INITIALIZED: return "Already initialized";
    case Status::ERROR_INVALID_STATE: return "Invalid state";
    case Status::ERROR_TIMEOUT: return "Timeout";
    case Status::ERROR_CANCELLED: return "Cancelled";
    case Status::ERROR_NOT_IMPLEMENTED: return "Not implemented";
    case Status::ERROR_INTERNAL: return "Internal error";
    case Status::ERROR_UNKNOWN: return "Unknown error";
    case Status::ERROR_DICTIONARY_FAILED: return "Dictionary failed";
    case Status::ERROR_UNSUPPORTED_FORMAT: return "Unsupported format";
  }
  return "Unknown error";
}

// ============================================================================
// error context / last error (reference src/cuda_zstd_types.cpp:81-141)
// ============================================================================
namespace {
std::recursive_mutex &error_mutex() {
  static std::recursive_mutex m;
  return m;
}
ErrorContext g_last_error;
ErrorCallback g_error_callback = nullptr;
}  // namespace
const char *get_detailed_error_message(const ErrorContext &ctx) {
  static thread_local char buf[512];
  const char *const file = ctx.file ? ctx.file : "unknown", *const fn = ctx.function ? ctx.function : "unknown";
  const char *const sep = ctx.message ? " - " : "", *const msg = ctx.message ? ctx.message : "";
  if (ctx.cuda_error != hipSuccess)
    snprintf(buf, sizeof(buf), "%s at %s:%d in %s() - HIP Error: %s (%d)%s%s", status_to_string(ctx.status), file, ctx.line, fn,
             hipGetErrorString(ctx.cuda_error), (int)ctx.cuda_error, sep, msg);
  else
    snprintf(buf, sizeof(buf), "%s at %s:%d in %s()%s%s", status_to_string(ctx.status), file, ctx.line, fn, sep, msg);
  return buf;
}
void set_error_callback(ErrorCallback cb) {
  std::lock_guard<std::recursive_mutex> g(error_mutex());
  g_error_callback = cb;
}
void log_error(const ErrorContext &ctx) {
  std::lock_guard<std::recursive_mutex> g(error_mutex());
  g_last_error = ctx;
  if (g_error_callback) g_error_callback(ctx);
}
ErrorContext get_last_error() {
  std::lock_guard<std::recursive_mutex> g(error_mutex());
  return g_last_error;
}
void clear_last_error() {
  std::lock_guard<std::recursive_mutex> g(error_mutex());
  g_last_error = ErrorContext();
}
namespace {
// a public entry point's result: failures go to the last-error slot (and the callback)
inline Status noted(Status s, const char *fn, int line) {
  if (s != Status::SUCCESS) log_error(ErrorContext(s, __FILE__, line, fn));
  return s;
}
}  // namespace
#define ZH_NOTED(s) noted((s), __func__, __LINE__)

// ============================================================================
// CompressionConfig (reference src/cuda_zstd_types.cpp:147-210, 860-950)
// ============================================================================
Strategy CompressionConfig::level_to_strategy(int level) {
  if (level <= 1) return Strategy::FAST;
  if (level <= 3) return Strategy::DFAST;
  if (level <= 6) return Strategy::GREEDY;
  if (level <= 12) return Strategy::LAZY;
  if (level <= 15) return Strategy::LAZY2;
  if (level <= 18) return Strategy::BTLAZY2;
  if (level <= 20) return Strategy::BTOPT;
  return Strategy::BTULTRA;
}
int CompressionConfig::strategy_to_default_level(Strategy s) {
  switch (s) {
    case Strategy::FAST: return 1;
    case Strategy::DFAST: return 3;
    case Strategy::GREEDY: return 5;
    case Strategy::LAZY: return 9;
    case Strategy::LAZY2: return 14;
    case Strategy::BTLAZY2: return 17;
    case Strategy::BTOPT: return 19;
    default: return 22;
  }
}
void apply_level_parameters(CompressionConfig &c) {
  int level = std::min(std::max(c.level, (int)MIN_COMPRESSION_LEVEL), (int)MAX_COMPRESSION_LEVEL);
  c.strategy = CompressionConfig::level_to_strategy(level);
  c.min_match = 3;
  if (level <= 1) { c.window_log = 18; c.hash_log = 15; c.chain_log = 15; c.search_log = 1; c.target_length = 0; }
  else if (level <= 3) { c.window_log = 19; c.hash_log = 17; c.chain_log = 17; c.search_log = 1; c.target_length = 0; }
  else if (level <= 6) { c.window_log = 20; c.hash_log = 17; c.chain_log = 17; c.search_log = level == 4 ? 2 : level == 5 ? 4 : 8; c.target_length = level <= 5 ? 0 : 8; }
  else if (level <= 9) { c.window_log = 22; c.hash_log = 18; c.chain_log = 18; c.search_log = level == 7 ? 8 : level == 8 ? 16 : 32; c.target_length = level <= 8 ? 16 : 32; }
  else if (level <= 12) { c.window_log = 23; c.hash_log = 19; c.chain_log = 19; c.search_log = level == 10 ? 64 : level == 11 ? 128 : 256; c.target_length = 64; }
  else if (level <= 15) { c.window_log = 23; c.hash_log = level <= 14 ? 19 : 20; c.chain_log = 19; c.search_log = level <= 14 ? 256 : 512; c.target_length = 128; }
  else if (level <= 18) { c.window_log = 23; c.hash_log = 20; c.chain_log = 20; c.search_log = level <= 17 ? 512 : 999; c.target_length = 256; }
  else { c.window_log = 23; c.hash_log = 20; c.chain_log = 20; c.search_log = 999; c.target_length = 999; }
}
CompressionConfig CompressionConfig::from_level(int level) {
  CompressionConfig c;
  c.compression_mode = CompressionMode::LEVEL_BASED;
  c.level = level;
  c.use_exact_level = true;
  apply_level_parameters(c);
  return c;
}
CompressionConfig CompressionConfig::optimal(size_t) { return from_level(3); }
CompressionConfig CompressionConfig::get_default() { return from_level(3); }
Status CompressionConfig::validate() const {
  if (!is_valid_compression_level(level)) return Status::ERROR_INVALID_PARAMETER;
  if (window_log < MIN_WINDOW_LOG || window_log > MAX_WINDOW_LOG) return Status::ERROR_INVALID_PARAMETER;
  if (block_size == 0) return Status::ERROR_INVALID_PARAMETER;
  return Status::SUCCESS;
}
Status validate_config(const CompressionConfig &c) { return c.validate(); }

// reference src/cuda_zstd_types.cpp:831-853 (callers size outputs with it)
size_t estimate_compressed_size(size_t n, int) {
  size_t nb = (n + (128 * 1024 - 1)) / (128 * 1024);
  if (nb == 0) nb = 1;
  return n + n / 255 + nb * 3 + 512;
}
u32 get_optimal_block_size(u32 input_size, u32) {
  (void)input_size;
  return ZH_BLOCK_MAX;
}

ZstdManager::ExecutionPath ZstdManager::select_execution_path(size_t size, int cpu_threshold) {
  return (cpu_threshold > 0 && size < (size_t)cpu_threshold) ? ExecutionPath::CPU : ExecutionPath::GPU_BATCH;
}

// ============================================================================
// host libzstd bridge (the reference's CPU route; FORCE_CPU + decompress)
// ============================================================================
namespace {
constexpr u32 kSkippableMagic = 0x184D2A50u;  // RFC 8878 skippable frames 0x184D2A50..5F
constexpr u32 kMetadataMagic = 0x444D5A43u;   // "CZMD": this library's metadata frame
constexpr size_t kMetadataFrameBytes = 16;
struct LibZstd {
  size_t (*compress)(void *, size_t, const void *, size_t, int) = nullptr;
  size_t (*decompress)(void *, size_t, const void *, size_t) = nullptr;
  unsigned (*isError)(size_t) = nullptr;
  unsigned long long (*frameContentSize)(const void *, size_t) = nullptr;
  size_t (*compressBound)(size_t) = nullptr;
  bool ok = false;
  LibZstd() {
    const char *names[] = {"libzstd.so.1", "libzstd.so", "/opt/conda/lib/libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1"};
    for (const char *nm : names) {
      // RTLD_DEEPBIND: a libzstd opened here binds its own calls inside itself even when another
      // libzstd image sits in the global scope (a preloaded tool's), never mixing two versions
      void *h = dlopen(nm, RTLD_NOW | RTLD_LOCAL | ZH_DLOPEN_DEEPBIND);
      if (!h) continue;
      compress = (decltype(compress))dlsym(h, "ZSTD_compress");
      decompress = (decltype(decompress))dlsym(h, "ZSTD_decompress");
      isError = (decltype(isError))dlsym(h, "ZSTD_isError");
      frameContentSize = (decltype(frameContentSize))dlsym(h, "ZSTD_getFrameContentSize");
      compressBound = (decltype(compressBound))dlsym(h, "ZSTD_compressBound");
      ok = compress && decompress && isError && frameContentSize && compressBound;
      if (ok) break;
    }
  }
};
LibZstd &libzstd() {
  static LibZstd z;
  return z;
}

bool is_device_ptr(const void *p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

Status copy_any(void *dst, const void *src, size_t n, hipStream_t stream) {
  if (!n) return Status::SUCCESS;
  if (!is_device_ptr(dst) && !is_device_ptr(src)) {  // host to host (FORCE_CPU on host buffers): no HIP call
    memmove(dst, src, n);
    return Status::SUCCESS;
  }
  if (hipMemcpyAsync(dst, src, n, hipMemcpyDefault, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
  if (hipStreamSynchronize(stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
  return Status::SUCCESS;
}

// reference CPU route: D2H, ZSTD_compress(level), H2D (src/cuda_zstd_manager.cu:1607-1668)
Status cpu_compress(const void *in, size_t n, void *out, size_t *out_size, int level, hipStream_t stream) {
  LibZstd &z = libzstd();
  if (!z.ok) return Status::ERROR_NOT_IMPLEMENTED;
  std::vector<u8> h_in(n), h_out(z.compressBound(n));
  Status s = copy_any(h_in.data(), in, n, stream);
  if (s != Status::SUCCESS) return s;
  size_t c = z.compress(h_out.data(), h_out.size(), h_in.data(), n, level);
  if (z.isError(c)) return Status::ERROR_COMPRESSION;
  if (c > *out_size) return Status::ERROR_BUFFER_TOO_SMALL;
  s = copy_any(out, h_out.data(), c, stream);
  if (s != Status::SUCCESS) return s;
  *out_size = c;
  return Status::SUCCESS;
}

// reference decompress CPU route (src/cuda_zstd_manager.cu:3219-3344)
Status cpu_decompress(const void *in, size_t n, void *out, size_t *out_size, hipStream_t stream) {
  LibZstd &z = libzstd();
  if (!z.ok) return Status::ERROR_NOT_IMPLEMENTED;
  if (!in || !out || !out_size || n < 4) return Status::ERROR_INVALID_PARAMETER;
  std::vector<u8> h_in(n);
  Status s = copy_any(h_in.data(), in, n, stream);
  if (s != Status::SUCCESS) return s;
  u32 magic;
  memcpy(&magic, h_in.data(), 4);
  if (magic != ZSTD_MAGIC) return Status::ERROR_INVALID_MAGIC;
  unsigned long long fcs = z.frameContentSize(h_in.data(), n);
  if (fcs == (unsigned long long)-2) return Status::ERROR_CORRUPT_DATA;
  size_t cap = *out_size;
  if (fcs != (unsigned long long)-1 && fcs > cap) return Status::ERROR_BUFFER_TOO_SMALL;
  std::vector<u8> h_out(fcs != (unsigned long long)-1 ? (size_t)fcs : cap);
  size_t d = z.decompress(h_out.data(), h_out.size(), h_in.data(), n);
  if (z.isError(d)) return Status::ERROR_CORRUPT_DATA;
  if (d > cap) return Status::ERROR_BUFFER_TOO_SMALL;
  s = copy_any(out, h_out.data(), d, stream);
  if (s != Status::SUCCESS) return s;
  *out_size = d;
  return Status::SUCCESS;
}

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Workspace layout inside the caller's temp buffer
struct WsLayout {
  size_t descs, items, blk_size, item_size, item_status, staging, counter, blocks, deep, deep_slots, total;
  // deep: a level >= ZH_DEEP_LEVEL call (the deep matcher's scratch slots, one per persistent
  // workgroup, follow the block areas)
  static WsLayout make(size_t nblocks, size_t nitems, bool staged, bool deep = false) {
    WsLayout L{};
    size_t o = 0;
    L.descs = o; o = align256(o + nblocks * sizeof(ZhBlockDesc));
    L.items = o; o = align256(o + nitems * sizeof(ZhItemDesc));
    L.blk_size = o; o = align256(o + nblocks * 4);
    L.item_size = o; o = align256(o + nitems * 8);
    L.item_status = o; o = align256(o + nitems * 4);
    L.staging = o; o = align256(o + (staged ? nblocks * (size_t)ZH_STAGE_SLOT : 0));
    L.counter = o; o = align256(o + 4);
    L.blocks = o; o = align256(o + nblocks * (size_t)ZH_WS_BLOCK_BYTES);
    L.deep_slots = deep ? std::min(nblocks, (size_t)ZH_DEEP_SLOTS_MAX) : 0;
    L.deep = o; o = align256(o + L.deep_slots * ZH_DEEP_SLOT_BYTES);
    L.total = o + 256;  // slack for base alignment
    return L;
  }
};

// Device blocks of a frame of n bytes (ZH_FRAME_BLOCK: 64 KiB, or 32 KiB history blocks for
// larger frames and for dictionary frames over 32 KiB below ZH_DEEP_LEVEL: split_dict)
inline size_t block_size_of(size_t n, bool split_dict) { return ZH_FRAME_BLOCK(n, split_dict); }
inline bool split_dict_of(bool has_dict, int level) { return has_dict && level < ZH_DEEP_LEVEL; }
inline size_t blocks_of(size_t n, bool split_dict = false) {
  size_t const bs = block_size_of(n, split_dict);
  return (n + bs - 1) / bs;
}

// Decoder workspace (zh_decode.hip): per-item arrays (host-array entry points upload
// them), then one slot per item holding the literals and sequence records of the block
// being decoded.  A slot is sized for blocks of block_cap regenerated bytes: 128 KiB
// (the format's maximum) unless every output capacity is smaller.
struct DecLayout {
  size_t in_ptrs, in_sizes, out_ptrs, caps, out_sizes, statuses, slots, total;
  u32 block_cap, lit_bytes, seq_cap, ho_off;
  u64 slot_bytes;
  static constexpr size_t kBlockMax = 128 * 1024;
  static DecLayout make(size_t n, size_t max_block) {
    DecLayout L{};
    L.block_cap = (u32)std::min(std::max<size_t>(max_block, 64), kBlockMax);
    L.lit_bytes = (u32)align256(L.block_cap + 64);
    L.seq_cap = L.block_cap / 3 + 2;
    L.ho_off = (u32)(L.lit_bytes + align256((size_t)L.seq_cap * 8));
    L.slot_bytes = L.ho_off + align256(ZH_DEC_HANDOFF_BYTES);
    size_t o = 0;
    L.in_ptrs = o; o = align256(o + n * 8);
    L.in_sizes = o; o = align256(o + n * 8);
    L.out_ptrs = o; o = align256(o + n * 8);
    L.caps = o; o = align256(o + n * 8);
    L.out_sizes = o; o = align256(o + n * 8);
    L.statuses = o; o = align256(o + n * 4);
    L.slots = o; o = align256(o + n * L.slot_bytes);
    L.total = o + 256;  // slack for base alignment
    return L;
  }
  ZhDecArgs args(u8 *base) const {
    ZhDecArgs a{};
    a.ws = base + slots;
    a.slot_bytes = slot_bytes;
    a.lit_bytes = lit_bytes;
    a.block_cap = block_cap;
    a.seq_cap = seq_cap;
    a.ho_off = ho_off;
    return a;
  }
};

Status from_dec_status(u32 s) {
  switch (s) {
    case 0: return Status::SUCCESS;
    case 2: return Status::ERROR_INVALID_PARAMETER;
    case 5: return Status::ERROR_INVALID_MAGIC;
    case 6: return Status::ERROR_CORRUPT_DATA;
    case 7: return Status::ERROR_BUFFER_TOO_SMALL;
    case 9: return Status::ERROR_DICTIONARY_MISMATCH;
    case 10: return Status::ERROR_CHECKSUM_FAILED;
    default: return Status::ERROR_DECOMPRESSION;
  }
}

std::once_flag g_init_flag;
hipError_t g_init_err = hipSuccess;
Status ensure_kernels() {
  std::call_once(g_init_flag, [] { g_init_err = zh::init_kernels(); });
  return g_init_err == hipSuccess ? Status::SUCCESS : Status::ERROR_CUDA_ERROR;
}

// A dictionary on the device: the whole buffer (the decoder reads a formatted
// dictionary's tables and repcodes from it) and its content offset.
struct DevDict {
  u8 *d = nullptr;
  size_t cap = 0, n = 0, off = 0;
  u32 id = 0;
  bool owned = true;  // false: a view of caller memory (streaming history)
  // K1's hash tables of the content tail, built at load (owned dictionaries only): every
  // record's first block starts from them instead of hashing the dictionary again
  u16 *tabs = nullptr;
  u32 *tabs_tmp = nullptr;
  u32 tabs_P = 0;
  // the deep matcher's chains of the content tail (levels >= ZH_DEEP_LEVEL), built at load
  u32 *deep_prev = nullptr, *deep_head = nullptr;
  u8 *deep_stg = nullptr;
  u32 deep_P = 0, deep_split = 0;
  std::vector<u8> host;  // the loaded bytes (a reload of the same dictionary keeps everything)
  // stream-ordered launches that may still read the buffers: one event per stream, recorded
  // after each launch (the blocking entry points have finished reading when they return)
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
  DevDict() = default;
  DevDict(const DevDict &) = delete;
  DevDict &operator=(const DevDict &) = delete;
  ~DevDict() {
    wait_uses();
    for (auto &u : uses) (void)hipEventDestroy(u.second);
    if (d && owned) (void)hipFree(d);
    if (tabs) (void)hipFree(tabs);
    if (tabs_tmp) (void)hipFree(tabs_tmp);
    if (deep_prev) (void)hipFree(deep_prev);
    if (deep_head) (void)hipFree(deep_head);
    if (deep_stg) (void)hipFree(deep_stg);
  }
  // raw-content view of device-resident history (never freed here)
  static void view(DevDict &v, const void *p, size_t bytes) {
    v.owned = false;
    v.d = (u8 *)p;
    v.cap = v.n = bytes;
    v.off = 0;
    v.id = 0;
    v.tabs_P = 0;  // (a moving history window: hashed by every block)
    v.deep_P = 0;
  }
  const u8 *content() const { return d + off; }
  size_t content_n() const { return n - off; }
  // a stream-ordered launch on `stream` reads this dictionary
  Status note_use(hipStream_t stream) const {
    auto *self = const_cast<DevDict *>(this);
    for (auto &u : self->uses)
      if (u.first == stream) return hipEventRecord(u.second, stream) == hipSuccess ? Status::SUCCESS : Status::ERROR_CUDA_ERROR;
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    self->uses.emplace_back(stream, e);
    return hipEventRecord(e, stream) == hipSuccess ? Status::SUCCESS : Status::ERROR_CUDA_ERROR;
  }
  // every stream-ordered launch that read the dictionary has finished (before it is replaced)
  Status wait_uses() {
    Status s = Status::SUCCESS;
    for (auto &u : uses)
      if (hipEventSynchronize(u.second) != hipSuccess) s = Status::ERROR_CUDA_ERROR;
    return s;
  }
  // raw content or a formatted dictionary (host or device buffer); replaces the previous one
  Status load(const void *p, size_t bytes, hipStream_t stream) {
    if (!p || !bytes || bytes > zh::kDictMaxBytes) return Status::ERROR_INVALID_PARAMETER;
    std::vector<u8> h(bytes);
    Status s = copy_any(h.data(), p, bytes, stream);
    if (s != Status::SUCCESS) return s;
    if (owned && d && n == bytes && host == h) return Status::SUCCESS;  // the same dictionary: tables kept
    u32 did = 0;
    size_t co = 0;
    if (!zh::dict_layout(h.data(), bytes, did, co)) return Status::ERROR_DICTIONARY_FAILED;
    if (d && wait_uses() != Status::SUCCESS) return Status::ERROR_CUDA_ERROR;  // stream-ordered launches still reading it
    if (bytes > cap) {
      if (d) (void)hipFree(d);
      d = nullptr;
      cap = 0;
      n = 0;
      if (hipMalloc(&d, bytes) != hipSuccess) { d = nullptr; return Status::ERROR_OUT_OF_MEMORY; }
      cap = bytes;
    }
    if (hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    n = bytes;
    off = co;
    id = did;
    tabs_P = 0;
    if (!tabs && hipMalloc(&tabs, 2u * (1u << ZH_HASH_LOG_LONG) + 2u * (1u << ZH_HASH_LOG_SHORT)) != hipSuccess) tabs = nullptr;
    if (!tabs_tmp && hipMalloc(&tabs_tmp, 4u * ((1u << ZH_HASH_LOG_LONG) + (1u << ZH_HASH_LOG_SHORT))) != hipSuccess) tabs_tmp = nullptr;
    if (tabs && tabs_tmp) {
      u32 P = 0;
      if (zh::lz_dict_tables(content(), content_n(), tabs, tabs_tmp, P, stream) == hipSuccess && hipStreamSynchronize(stream) == hipSuccess)
        tabs_P = P;
    }
    deep_P = deep_split = 0;
    if (!deep_prev && hipMalloc(&deep_prev, 4u * ZH_DEEP_PRE) != hipSuccess) deep_prev = nullptr;
    if (!deep_head && hipMalloc(&deep_head, 4u << ZH_HASH_LOG_SHORT) != hipSuccess) deep_head = nullptr;
    if (!deep_stg && hipMalloc(&deep_stg, ZH_DEEP_PRE + 256) != hipSuccess) deep_stg = nullptr;
    if (deep_prev && deep_head && deep_stg) {
      u32 P = 0, sp = 0;
      if (zh::lz_deep_dict_tables(content(), content_n(), deep_stg, deep_prev, deep_head, P, sp, stream) == hipSuccess &&
          hipStreamSynchronize(stream) == hipSuccess) {
        deep_P = P;
        deep_split = sp;
      }
    }
    host.swap(h);
    return Status::SUCCESS;
  }
  void fill(ZhDecArgs &a) const {
    if (!n) return;
    a.dict = d;
    a.dict_n = n;
    a.dict_off = (u32)off;
    a.dict_id = id;
  }
};

// Descriptor fields of a block: a dictionary frame's first block gets the content tail that
// fits in front of it in K1's 64 KiB of LDS; a later block of a history frame gets the 32 KiB
// of input before it (when the window reaches that far)
void set_dict_block(ZhBlockDesc &d, const DevDict *dd, bool first, bool hist, bool deep) {
  d.pre = nullptr;
  d.pre_n = 0;
  d.dict_id = 0;
  if (!first && hist) {
    d.pre = d.src - ZH_HIST_BLOCK;
    d.pre_n = ZH_HIST_BLOCK;
  }
  if (!dd || !dd->n) return;
  d.flags |= ZH_F_DICT;
  d.dict_id = dd->id;
  if (!first) return;
  size_t const cn = dd->content_n();
  // (the deep matcher of levels >= ZH_DEEP_LEVEL stages up to ZH_DEEP_PRE content bytes: it keeps
  // the staged bytes in global memory, not in K1's 64 KiB of LDS)
  d.pre_n = (u32)std::min(cn, deep ? (size_t)ZH_DEEP_PRE : (size_t)ZH_BLOCK_MAX - d.n);
  d.pre = dd->content() + cn - d.pre_n;
}

// the deep matcher's precomputed dictionary chains, when the dictionary has them
void set_deep_dict(ZhWorkspace &ws, const DevDict *dd) {
  ws.dd_prev = ws.dd_head = nullptr;
  ws.dd_pre = ws.dd_split = 0;
  if (!dd || !dd->deep_P) return;
  ws.dd_prev = dd->deep_prev;
  ws.dd_head = dd->deep_head;
  ws.dd_pre = dd->deep_P;
  ws.dd_split = dd->deep_split;
}

Status from_item_status(u32 s) {
  return s == ZH_ST_OK ? Status::SUCCESS : s == ZH_ST_TOO_SMALL ? Status::ERROR_BUFFER_TOO_SMALL : Status::ERROR_INVALID_PARAMETER;
}
}  // namespace

// ============================================================================
// ZstdBatchManager
// ============================================================================
class ZstdBatchManager::Impl {
 public:
  CompressionConfig config;
  CompressionStats stats;
  dictionary::DictionaryHeader dict_hdr{};  // set_dictionary's header (dictionary_id: the frames' RFC ID)
  bool has_dict = false;
  std::mutex api_mutex;  // one manager serialises calls (reference src/cuda_zstd_manager.cu:1542)
  void *pinned = nullptr;
  size_t pinned_bytes = 0;
  DevDict mgr_dict, call_dict;  // set_dictionary()'s / compress()'s per-call dictionary
  const DevDict *active() const { return mgr_dict.n ? &mgr_dict : nullptr; }

  explicit Impl(const CompressionConfig &c) : config(c) {}
  ~Impl() { if (pinned) (void)hipHostFree(pinned); }

  void *host_scratch(size_t bytes) {
    if (bytes > pinned_bytes) {
      if (pinned) (void)hipHostFree(pinned);
      pinned = nullptr;
      pinned_bytes = 0;
      if (hipHostMalloc(&pinned, bytes, hipHostMallocDefault) != hipSuccess) { pinned = nullptr; return nullptr; }
      pinned_bytes = bytes;
    }
    return pinned;
  }

  // Run the device pipeline over a list of frames given as host arrays.
  // out_sizes: in = capacity, out = bytes; statuses out.
  Status run(const void *const *in_ptrs, const size_t *in_sizes, size_t count, void *const *out_ptrs, size_t *out_sizes, Status *statuses,
             void *temp, size_t temp_size, hipStream_t stream, const DevDict *dd = nullptr) {
    Status s = ensure_kernels();
    if (s != Status::SUCCESS) return s;
    size_t nblocks = 0;
    bool staged = false;
    bool const has_dict = dd && dd->n;
    bool const hist = config.window_log >= ZH_HIST_WINDOW_LOG;
    for (size_t i = 0; i < count; i++) {
      size_t nb = blocks_of(in_sizes[i], split_dict_of(has_dict, config.level));
      nblocks += nb;
      staged |= nb > 1;
    }
    WsLayout L = WsLayout::make(nblocks, count, staged, config.level >= ZH_DEEP_LEVEL);
    if (!temp || temp_size < L.total) return Status::ERROR_BUFFER_TOO_SMALL;
    u8 *base = (u8 *)(((uintptr_t)temp + 255) & ~(uintptr_t)255);

    // host plan -> one pinned upload
    size_t const up_bytes = L.blk_size;  // descs + items
    u8 *h = (u8 *)host_scratch(up_bytes + count * 12);
    if (!h) return Status::ERROR_OUT_OF_MEMORY;
    ZhBlockDesc *hd = (ZhBlockDesc *)(h + L.descs);
    ZhItemDesc *hi = (ZhItemDesc *)(h + L.items);
    u8 *staging = base + L.staging;
    size_t b = 0;
    for (size_t i = 0; i < count; i++) {
      bool const sd = split_dict_of(has_dict, config.level);
      size_t const n = in_sizes[i], nb = blocks_of(n, sd), bs = block_size_of(n, sd);
      hi[i].dst = (u8 *)out_ptrs[i];
      hi[i].cap = out_sizes[i];
      hi[i].first_block = (u32)b;
      hi[i].nblocks = (u32)nb;
      for (size_t k = 0; k < nb; k++, b++) {
        ZhBlockDesc &d = hd[b];
        d.src = (const u8 *)in_ptrs[i] + k * bs;
        d.frame_size = n;
        d.n = (u32)std::min(bs, n - k * bs);
        d.item = (u32)i;
        d.flags = (k == 0 ? ZH_F_FIRST : 0u) | (k + 1 == nb ? ZH_F_LAST : 0u) | (nb == 1 ? ZH_F_DIRECT : 0u) |
                  (config.checksum != ChecksumPolicy::NO_COMPUTE_NO_VERIFY ? ZH_F_CHECKSUM : 0u) |
                  (config.level >= ZH_DEEP_LEVEL ? ZH_F_DEEP : 0u);
        set_dict_block(d, dd, k == 0, hist, config.level >= ZH_DEEP_LEVEL);
        if (nb == 1) {
          d.dst = (u8 *)out_ptrs[i];
          d.dst_cap = (u32)std::min(out_sizes[i], (size_t)0xFFFFFFFFu);
        } else {
          d.dst = staging + b * (size_t)ZH_STAGE_SLOT;
          d.dst_cap = ZH_STAGE_SLOT;
        }
      }
    }
    if (hipMemcpyAsync(base, h, up_bytes, hipMemcpyHostToDevice, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    ZhWorkspace ws{base + L.blocks, (u32 *)(base + L.counter), dd && dd->tabs_P ? dd->tabs : nullptr, dd ? dd->tabs_P : 0u};
    set_deep_dict(ws, dd);
    ws.deep_slots = L.deep_slots ? base + L.deep : nullptr;
    ws.deep_nslots = (u32)L.deep_slots;
    hipError_t e = zh::launch_compress((const ZhBlockDesc *)(base + L.descs), (u32)nblocks, ws, config.window_log, config.block_size,
                                       (u64 *)(base + L.item_size), (u32 *)(base + L.item_status), (u32 *)(base + L.blk_size),
                                       (const ZhItemDesc *)(base + L.items), (u32)count, staged,
                                       config.checksum != ChecksumPolicy::NO_COMPUTE_NO_VERIFY, config.level, stream);
    if (e != hipSuccess) return Status::ERROR_CUDA_ERROR;
    u64 *h_size = (u64 *)(h + up_bytes);
    u32 *h_status = (u32 *)(h_size + count);
    if (hipMemcpyAsync(h_size, base + L.item_size, count * 8, hipMemcpyDeviceToHost, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipMemcpyAsync(h_status, base + L.item_status, count * 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipStreamSynchronize(stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    bool all_ok = true;
    for (size_t i = 0; i < count; i++) {
      Status st = from_item_status(h_status[i]);
      statuses[i] = st;
      if (st == Status::SUCCESS) out_sizes[i] = (size_t)h_size[i];
      else all_ok = false;
      stats.input_bytes += in_sizes[i];
      if (st == Status::SUCCESS) stats.output_bytes += h_size[i];
    }
    stats.blocks_processed += nblocks;
    stats.num_blocks += nblocks;
    return all_ok ? Status::SUCCESS : Status::ERROR_GENERIC;
  }

  // Decode a list of buffers given as host arrays of device pointers (one launch of
  // zh_decode_kernel, one host synchronisation).  out_sizes: in = capacity, out = bytes.
  Status run_decompress(const void *const *in_ptrs, const size_t *in_sizes, size_t count, void *const *out_ptrs, size_t *out_sizes,
                        Status *statuses, void *temp, size_t temp_size, hipStream_t stream) {
    Status s = ensure_kernels();
    if (s != Status::SUCCESS) return s;
    size_t maxcap = 0;
    for (size_t i = 0; i < count; i++) maxcap = std::max(maxcap, out_sizes[i]);
    DecLayout L = DecLayout::make(count, maxcap);
    if (!temp || temp_size < L.total) return Status::ERROR_BUFFER_TOO_SMALL;
    u8 *base = (u8 *)(((uintptr_t)temp + 255) & ~(uintptr_t)255);
    size_t const up = L.out_sizes, down = L.slots - L.out_sizes;
    u8 *h = (u8 *)host_scratch(up + down);
    if (!h) return Status::ERROR_OUT_OF_MEMORY;
    for (size_t i = 0; i < count; i++) {
      ((const void **)(h + L.in_ptrs))[i] = in_ptrs[i];
      ((size_t *)(h + L.in_sizes))[i] = in_sizes[i];
      ((void **)(h + L.out_ptrs))[i] = out_ptrs[i];
      ((size_t *)(h + L.caps))[i] = out_sizes[i];
    }
    if (hipMemcpyAsync(base, h, up, hipMemcpyHostToDevice, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    ZhDecArgs a = L.args(base);
    mgr_dict.fill(a);
    a.in_ptrs = (const void *const *)(base + L.in_ptrs);
    a.in_sizes = (const size_t *)(base + L.in_sizes);
    a.out_ptrs = (void *const *)(base + L.out_ptrs);
    a.out_caps = (const size_t *)(base + L.caps);
    a.out_sizes = (size_t *)(base + L.out_sizes);
    a.statuses = (u32 *)(base + L.statuses);
    if (zh::launch_decompress(a, (u32)count, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipMemcpyAsync(h + up, base + L.out_sizes, down, hipMemcpyDeviceToHost, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipStreamSynchronize(stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    const size_t *hsz = (const size_t *)(h + up);
    const u32 *hst = (const u32 *)(h + up + (L.statuses - L.out_sizes));
    bool all_ok = true;
    for (size_t i = 0; i < count; i++) {
      Status st = from_dec_status(hst[i]);
      statuses[i] = st;
      if (st == Status::SUCCESS) {
        out_sizes[i] = hsz[i];
        stats.bytes_decompressed += hsz[i];
      } else {
        all_ok = false;
      }
    }
    return all_ok ? Status::SUCCESS : Status::ERROR_GENERIC;
  }

  // One buffer, no pointer-array upload (ZhDecArgs single-item fields).  Synchronous
  // unless d_actual is given (then the size lands there, stream-ordered, 0 on error).
  Status run_decompress_one(const void *in, size_t n, void *out, size_t cap, size_t *h_actual, size_t *d_actual, void *temp, size_t temp_size,
                            hipStream_t stream, const DevDict *dd = nullptr) {
    Status s = ensure_kernels();
    if (s != Status::SUCCESS) return s;
    DecLayout L = DecLayout::make(1, cap);
    if (!temp || temp_size < L.total) return Status::ERROR_BUFFER_TOO_SMALL;
    u8 *base = (u8 *)(((uintptr_t)temp + 255) & ~(uintptr_t)255);
    ZhDecArgs a = L.args(base);
    (dd ? *dd : mgr_dict).fill(a);
    a.one_in = in;
    a.one_in_size = n;
    a.one_out = out;
    a.out_cap_all = cap;
    a.out_sizes = d_actual ? d_actual : (size_t *)(base + L.out_sizes);
    a.statuses = (u32 *)(base + L.statuses);
    if (zh::launch_decompress(a, 1, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (d_actual) return Status::SUCCESS;
    u8 *h = (u8 *)host_scratch(16);
    if (!h) return Status::ERROR_OUT_OF_MEMORY;
    if (hipMemcpyAsync(h, base + L.out_sizes, 8, hipMemcpyDeviceToHost, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipMemcpyAsync(h + 8, base + L.statuses, 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipStreamSynchronize(stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    Status st = from_dec_status(*(const u32 *)(h + 8));
    if (st == Status::SUCCESS) {
      *h_actual = *(const size_t *)h;
      stats.bytes_decompressed += *h_actual;
    }
    return st;
  }
};

ZstdBatchManager::ZstdBatchManager() : pimpl_(new Impl(CompressionConfig::from_level(3))) {}
ZstdBatchManager::ZstdBatchManager(const CompressionConfig &c) : pimpl_(new Impl(c)) {}
ZstdBatchManager::~ZstdBatchManager() = default;

Status ZstdBatchManager::configure(const CompressionConfig &c) {
  Status s = c.validate();
  if (s != Status::SUCCESS) return s;
  pimpl_->config = c;
  return Status::SUCCESS;
}
CompressionConfig ZstdBatchManager::get_config() const { return pimpl_->config; }

// sized for the dictionary layout as well (a per-call dictionary is only known at compress())
size_t ZstdBatchManager::get_compress_temp_size(size_t n) const {
  size_t nb = std::max<size_t>(1, blocks_of(n, true));
  return WsLayout::make(nb, 1, nb > 1, pimpl_->config.level >= ZH_DEEP_LEVEL).total;
}
// one slot for 128 KiB blocks (reference src/cuda_zstd_manager.cu:1373-1408 also sizes for one block)
size_t ZstdBatchManager::get_decompress_temp_size(size_t) const { return DecLayout::make(1, DecLayout::kBlockMax).total; }
size_t ZstdBatchManager::get_max_compressed_size(size_t n) const { return estimate_compressed_size(n, pimpl_->config.level); }

Status ZstdBatchManager::compress(const void *in, size_t n, void *out, size_t *out_size, void *temp, size_t temp_size, const void *dict_buffer,
                                  size_t dict_size, hipStream_t stream, void *) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  // reference validation order (src/cuda_zstd_manager.cu:1549-1565)
  if (!in || !out || !out_size || !temp) return Status::ERROR_INVALID_PARAMETER;
  if (n == 0) { *out_size = 0; return Status::ERROR_INVALID_PARAMETER; }
  if (temp_size < get_compress_temp_size(n)) return Status::ERROR_BUFFER_TOO_SMALL;
  // a per-call dictionary (host or device buffer) overrides the manager's set_dictionary()
  const DevDict *dd = pimpl_->active();
  if (dict_buffer && dict_size) {
    Status s = pimpl_->call_dict.load(dict_buffer, dict_size, stream);
    if (s != Status::SUCCESS) return s;
    dd = &pimpl_->call_dict;
  }
  auto t0 = std::chrono::steady_clock::now();
  Status st;
  if (!dd && select_execution_path(n, (int)pimpl_->config.cpu_threshold) == ExecutionPath::CPU) {
    st = cpu_compress(in, n, out, out_size, pimpl_->config.level, stream);
    if (st == Status::SUCCESS) { pimpl_->stats.input_bytes += n; pimpl_->stats.output_bytes += *out_size; }
  } else {
    Status item;
    const void *ip[1] = {in};
    void *opv[1] = {out};
    size_t sz[1] = {n};
    st = pimpl_->run(ip, sz, 1, opv, out_size, &item, temp, temp_size, stream, dd);
    if (st == Status::ERROR_GENERIC) st = item;
  }
  pimpl_->stats.compression_time_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return st;
}

// GPU decode (zh_decode.hip) of device-resident frames; validation order of the
// reference (src/cuda_zstd_manager.cu:3203-3212).  *out_size: capacity in, bytes out.
Status ZstdBatchManager::decompress(const void *in, size_t n, void *out, size_t *out_size, void *temp, size_t temp_size, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (!in || !out || !out_size || !temp || n < 4) return Status::ERROR_INVALID_PARAMETER;
  // the slot the decode actually uses: sized by the output capacity, so a workspace from
  // allocate_inference_workspace(max_out) is enough (reference tests/test_inference_api.cu:398-410)
  if (temp_size < DecLayout::make(1, *out_size).total) return Status::ERROR_BUFFER_TOO_SMALL;
  if (!is_device_ptr(in) || !is_device_ptr(out)) return Status::ERROR_INVALID_PARAMETER;  // device-resident API
  auto t0 = std::chrono::steady_clock::now();
  size_t got = 0;
  Status s = pimpl_->run_decompress_one(in, n, out, *out_size, &got, nullptr, temp, temp_size, stream);
  if (s == Status::SUCCESS) *out_size = got;
  pimpl_->stats.decompression_time_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return s;
}

Status ZstdBatchManager::compress_with_history(const void *in, size_t n, void *out, size_t *out_size, void *temp, size_t temp_size,
                                               const void *hist, size_t hist_n, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (!in || !out || !out_size || !temp || (hist_n && !hist)) return Status::ERROR_INVALID_PARAMETER;
  if (n == 0) { *out_size = 0; return Status::ERROR_INVALID_PARAMETER; }
  if (temp_size < get_compress_temp_size(n)) return Status::ERROR_BUFFER_TOO_SMALL;
  DevDict view;
  if (hist_n) DevDict::view(view, hist, hist_n);
  Status item;
  const void *ip[1] = {in};
  void *opv[1] = {out};
  size_t sz[1] = {n};
  auto t0 = std::chrono::steady_clock::now();
  Status st = pimpl_->run(ip, sz, 1, opv, out_size, &item, temp, temp_size, stream, hist_n ? &view : pimpl_->active());
  if (st == Status::ERROR_GENERIC) st = item;
  pimpl_->stats.compression_time_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return st;
}
Status ZstdBatchManager::decompress_with_history(const void *in, size_t n, void *out, size_t *out_size, void *temp, size_t temp_size,
                                                 const void *hist, size_t hist_n, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (!in || !out || !out_size || !temp || n < 4 || (hist_n && !hist)) return Status::ERROR_INVALID_PARAMETER;
  if (temp_size < DecLayout::make(1, *out_size).total) return Status::ERROR_BUFFER_TOO_SMALL;
  DevDict view;
  if (hist_n) DevDict::view(view, hist, hist_n);
  size_t got = 0;
  Status s = pimpl_->run_decompress_one(in, n, out, *out_size, &got, nullptr, temp, temp_size, stream, hist_n ? &view : nullptr);
  if (s == Status::SUCCESS) *out_size = got;
  return s;
}

// Dictionary compression and decompression: raw content or a formatted RFC 8878
// dictionary; copied to the device once (the reference keeps a shallow pointer and copies it
// into the workspace per call, src/cuda_zstd_manager.cu:1699-1775, 3711-3764)
// The reference's checks (src/cuda_zstd_manager.cu:3711-3736): content present, MIN_DICT_SIZE ..
// MAX_DICT_SIZE bytes.  raw_content may be host or device memory (copied once, DevDict::load).
Status ZstdBatchManager::set_dictionary(const dictionary::Dictionary &d) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (!d.raw_content || d.raw_size == 0) return Status::ERROR_INVALID_PARAMETER;
  if (d.raw_size < dictionary::MIN_DICT_SIZE || d.raw_size > dictionary::MAX_DICT_SIZE) return Status::ERROR_INVALID_PARAMETER;
  Status s = pimpl_->mgr_dict.load(d.raw_content, d.raw_size, 0);
  if (s != Status::SUCCESS) return s;
  pimpl_->dict_hdr = d.header;
  pimpl_->dict_hdr.dictionary_id = pimpl_->mgr_dict.id;
  pimpl_->dict_hdr.raw_content_size = d.raw_size;
  pimpl_->has_dict = true;
  return Status::SUCCESS;
}
// reference :3858-3863: no dictionary -> ERROR_INVALID_PARAMETER; else a deep copy (the caller
// frees dict.raw_content with free(), Dictionary's copy semantics)
Status ZstdBatchManager::get_dictionary(dictionary::Dictionary &d) const {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);  // set_dictionary swaps mgr_dict under it
  if (!pimpl_->has_dict) return Status::ERROR_INVALID_PARAMETER;
  dictionary::Dictionary view;
  view.header = pimpl_->dict_hdr;
  view.raw_content = pimpl_->mgr_dict.host.data();
  view.raw_size = (u32)pimpl_->mgr_dict.host.size();
  d = view;
  return d.raw_content ? Status::SUCCESS : Status::ERROR_OUT_OF_MEMORY;
}
Status ZstdBatchManager::clear_dictionary() {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  pimpl_->has_dict = false;
  pimpl_->dict_hdr = dictionary::DictionaryHeader{};
  pimpl_->mgr_dict.n = 0;
  return Status::SUCCESS;
}
const CompressionStats &ZstdBatchManager::get_stats() const { return pimpl_->stats; }
Status ZstdBatchManager::set_compression_level(int level) {
  if (!is_valid_compression_level(level)) return Status::ERROR_INVALID_PARAMETER;
  CompressionConfig c = pimpl_->config;
  c.level = level;
  apply_level_parameters(c);
  pimpl_->config = c;
  return Status::SUCCESS;
}
int ZstdBatchManager::get_compression_level() const { return pimpl_->config.level; }
void ZstdBatchManager::reset_stats() { pimpl_->stats = CompressionStats{}; }

size_t ZstdBatchManager::get_batch_compress_temp_size(const std::vector<size_t> &sizes) const {
  size_t nb = 0;
  bool staged = false;
  // (for the manager's dictionary as set now -- compress_batch takes no per-call dictionary; a
  // dictionary set later may need more: ZH_FRAME_BLOCK, and the call then fails with
  // ERROR_BUFFER_TOO_SMALL)
  bool const sd = split_dict_of(pimpl_->active() != nullptr, pimpl_->config.level);
  for (size_t s : sizes) { size_t k = blocks_of(s, sd); nb += k; staged |= k > 1; }
  return WsLayout::make(nb, sizes.size(), staged, pimpl_->config.level >= ZH_DEEP_LEVEL).total;
}
size_t ZstdBatchManager::get_batch_decompress_temp_size(const std::vector<size_t> &sizes) const {
  return DecLayout::make(std::max<size_t>(1, sizes.size()), DecLayout::kBlockMax).total;
}

Status ZstdBatchManager::compress_batch(const std::vector<BatchItem> &items, void *temp, size_t temp_size, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  reset_stats();
  if (items.empty()) return Status::SUCCESS;
  auto &mut = const_cast<std::vector<BatchItem> &>(items);  // reference writes sizes/status through const (:5745)
  std::vector<size_t> sizes(items.size());
  for (size_t i = 0; i < items.size(); i++) sizes[i] = items[i].input_size;
  if (temp_size < get_batch_compress_temp_size(sizes)) return Status::ERROR_BUFFER_TOO_SMALL;
  // items with invalid arguments never reach the device; the reference's batch loop calls
  // compress() per item (src/cuda_zstd_manager.cu:5744-5768), so an item below cpu_threshold
  // takes compress()'s libzstd route (without a dictionary, as compress() decides) and the rest
  // share one device launch
  const DevDict *dd = pimpl_->active();
  std::vector<const void *> ip;
  std::vector<void *> op;
  std::vector<size_t> isz, osz, idx;
  bool any_bad = false;
  auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < items.size(); i++) {
    if (!items[i].input_ptr || !items[i].output_ptr || items[i].input_size == 0) {
      mut[i].status = Status::ERROR_INVALID_PARAMETER;
      any_bad = true;
      continue;
    }
    if (!dd && select_execution_path(items[i].input_size, (int)pimpl_->config.cpu_threshold) == ExecutionPath::CPU) {
      size_t o = items[i].output_size;
      mut[i].status = cpu_compress(items[i].input_ptr, items[i].input_size, items[i].output_ptr, &o, pimpl_->config.level, stream);
      if (mut[i].status == Status::SUCCESS) {
        mut[i].output_size = o;
        pimpl_->stats.input_bytes += items[i].input_size;
        pimpl_->stats.output_bytes += o;
      } else {
        any_bad = true;
      }
      continue;
    }
    ip.push_back(items[i].input_ptr);
    op.push_back(items[i].output_ptr);
    isz.push_back(items[i].input_size);
    osz.push_back(items[i].output_size);
    idx.push_back(i);
  }
  std::vector<Status> st(idx.size());
  Status r = idx.empty() ? Status::SUCCESS : pimpl_->run(ip.data(), isz.data(), idx.size(), op.data(), osz.data(), st.data(), temp, temp_size, stream, dd);
  pimpl_->stats.compression_time_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (r != Status::SUCCESS && r != Status::ERROR_GENERIC) return r;
  for (size_t j = 0; j < idx.size(); j++) {
    mut[idx[j]].status = st[j];
    if (st[j] == Status::SUCCESS) mut[idx[j]].output_size = osz[j];
    else any_bad = true;
  }
  return any_bad ? Status::ERROR_GENERIC : Status::SUCCESS;
}

// ZstdBatchManager::decompress_batch (reference src/cuda_zstd_manager.cu:5799-5885): every
// item decoded by one launch; output_size in = capacity, out = bytes; per-item status.
Status ZstdBatchManager::decompress_batch(const std::vector<BatchItem> &items, void *temp, size_t temp_size, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (items.empty()) return Status::SUCCESS;
  auto &mut = const_cast<std::vector<BatchItem> &>(items);  // the reference writes sizes/status through const
  std::vector<const void *> ip;
  std::vector<void *> op;
  std::vector<size_t> isz, osz, idx;
  bool any_bad = false;
  for (size_t i = 0; i < items.size(); i++) {
    if (!items[i].input_ptr || !items[i].output_ptr || items[i].input_size < 4) {
      mut[i].status = Status::ERROR_INVALID_PARAMETER;
      any_bad = true;
      continue;
    }
    ip.push_back(items[i].input_ptr);
    op.push_back(items[i].output_ptr);
    isz.push_back(items[i].input_size);
    osz.push_back(items[i].output_size);
    idx.push_back(i);
  }
  if (idx.empty()) return Status::ERROR_GENERIC;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<Status> st(idx.size());
  Status r = pimpl_->run_decompress(ip.data(), isz.data(), idx.size(), op.data(), osz.data(), st.data(), temp, temp_size, stream);
  pimpl_->stats.decompression_time_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (r != Status::SUCCESS && r != Status::ERROR_GENERIC) return r;
  for (size_t j = 0; j < idx.size(); j++) {
    mut[idx[j]].status = st[j];
    if (st[j] == Status::SUCCESS) mut[idx[j]].output_size = osz[j];
    else any_bad = true;
  }
  return any_bad ? Status::ERROR_GENERIC : Status::SUCCESS;
}

Status ZstdBatchManager::decompress_to_preallocated(const void *in, size_t n, void *out, size_t cap, size_t *actual, void *temp, size_t temp_size,
                                                    hipStream_t stream) {
  if (!in || !out || !actual) return Status::ERROR_INVALID_PARAMETER;
  if (cap == 0) return Status::ERROR_BUFFER_TOO_SMALL;  // reference tests/test_inference_api.cu:581-586
  *actual = cap;
  return decompress(in, n, out, actual, temp, temp_size, stream);
}
Status ZstdBatchManager::decompress_batch_preallocated(std::vector<BatchItem> &items, void *t, size_t ts, hipStream_t stream) {
  return decompress_batch(items, t, ts, stream);
}
// stream-ordered: nothing is synchronised; *d_actual (device) receives the size, 0 on error
Status ZstdBatchManager::decompress_async_no_sync(const void *in, size_t n, void *out, size_t cap, size_t *d_actual, void *temp, size_t temp_size,
                                                  hipStream_t stream) {
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  if (!in || !out || !d_actual || !temp || n < 4) return Status::ERROR_INVALID_PARAMETER;
  if (temp_size < DecLayout::make(1, cap).total) return Status::ERROR_BUFFER_TOO_SMALL;
  return pimpl_->run_decompress_one(in, n, out, cap, nullptr, d_actual, temp, temp_size, stream);
}
size_t ZstdBatchManager::get_inference_workspace_size(size_t, size_t max_out) const { return DecLayout::make(1, max_out).total; }
Status ZstdBatchManager::allocate_inference_workspace(size_t a, size_t b, void **ptr, size_t *size) {
  if (!ptr || !size) return Status::ERROR_INVALID_PARAMETER;
  *size = std::max<size_t>(256, get_inference_workspace_size(a, b));
  return hipMalloc(ptr, *size) == hipSuccess ? Status::SUCCESS : Status::ERROR_OUT_OF_MEMORY;
}
Status ZstdBatchManager::free_inference_workspace(void *ptr) { return hipFree(ptr) == hipSuccess ? Status::SUCCESS : Status::ERROR_CUDA_ERROR; }

// (static: no dictionary, levels below ZH_DEEP_LEVEL; get_batch_device_temp_size_for covers the
// manager's level and dictionary)
// levels below ZH_DEEP_LEVEL without a dictionary (the deep matcher's scratch slots of levels >=
// ZH_DEEP_LEVEL, up to ZH_DEEP_SLOTS_MAX x ZH_DEEP_SLOT_BYTES, are in get_batch_device_temp_size_for)
size_t ZstdBatchManager::get_batch_device_temp_size(size_t count, size_t max_chunk) {
  size_t const bpi = std::max<size_t>(1, blocks_of(max_chunk));
  return WsLayout::make(count * bpi, count, bpi > 1).total;
}
size_t ZstdBatchManager::get_batch_device_temp_size_for(size_t count, size_t max_chunk) const {
  size_t const bpi = std::max<size_t>(1, blocks_of(max_chunk, split_dict_of(pimpl_->active() != nullptr, pimpl_->config.level)));
  return WsLayout::make(count * bpi, count, bpi > 1, pimpl_->config.level >= ZH_DEEP_LEVEL).total;
}

Status ZstdBatchManager::compress_batch_device(const void *const *d_in_ptrs, const size_t *d_in_sizes, size_t max_chunk, size_t count,
                                               void *const *d_out_ptrs, size_t *d_out_sizes, int *d_statuses, void *temp, size_t temp_size,
                                               hipStream_t stream) {
  // one manager serialises calls (the dictionary's use events: set_dictionary waits on them)
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  Status s = ensure_kernels();
  if (s != Status::SUCCESS) return s;
  if (!count) return Status::SUCCESS;
  if (!d_in_ptrs || !d_in_sizes || !d_out_ptrs || !d_out_sizes || max_chunk == 0) return Status::ERROR_INVALID_PARAMETER;
  const DevDict *dd = pimpl_->active();
  // (with a dictionary set, chunks over 32 KiB take two history blocks: a larger workspace
  // than get_batch_device_temp_size's, from nvcomp_zstd_batch_get_compress_temp_size_v5)
  size_t const bpi = blocks_of(max_chunk, split_dict_of(dd != nullptr, pimpl_->config.level)), nblocks = count * bpi;
  WsLayout L = WsLayout::make(nblocks, count, bpi > 1, pimpl_->config.level >= ZH_DEEP_LEVEL);
  if (!temp || temp_size < L.total) return Status::ERROR_BUFFER_TOO_SMALL;
  u8 *base = (u8 *)(((uintptr_t)temp + 255) & ~(uintptr_t)255);
  u64 const cap = estimate_compressed_size(max_chunk, pimpl_->config.level);
  u64 *item_size = (u64 *)d_out_sizes;
  u32 *item_status = d_statuses ? (u32 *)d_statuses : (u32 *)(base + L.item_status);
  bool const ck = pimpl_->config.checksum != ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  u32 const hist = pimpl_->config.window_log >= ZH_HIST_WINDOW_LOG ? 1u : 0u;
  hipError_t e = zh::launch_plan(d_in_ptrs, d_in_sizes, (u32)count, (u32)bpi, d_out_ptrs, cap, base + L.staging, (ZhBlockDesc *)(base + L.descs),
                                 (ZhItemDesc *)(base + L.items), item_size, item_status,
                                 (ck ? ZH_F_CHECKSUM : 0u) | (pimpl_->config.level >= ZH_DEEP_LEVEL ? ZH_F_DEEP : 0u),
                                 dd ? dd->content() : nullptr, dd ? (u32)dd->content_n() : 0u, dd ? dd->id : 0u, hist, stream);
  if (e != hipSuccess) return Status::ERROR_CUDA_ERROR;
  ZhWorkspace ws{base + L.blocks, (u32 *)(base + L.counter), dd && dd->tabs_P ? dd->tabs : nullptr, dd ? dd->tabs_P : 0u};
  set_deep_dict(ws, dd);
  ws.deep_slots = L.deep_slots ? base + L.deep : nullptr;
  ws.deep_nslots = (u32)L.deep_slots;
  e = zh::launch_compress((const ZhBlockDesc *)(base + L.descs), (u32)nblocks, ws, pimpl_->config.window_log, pimpl_->config.block_size, item_size,
                          item_status, (u32 *)(base + L.blk_size), (const ZhItemDesc *)(base + L.items), (u32)count, bpi > 1, ck,
                          pimpl_->config.level, stream);
  if (e != hipSuccess) return Status::ERROR_CUDA_ERROR;
  return dd ? dd->note_use(stream) : Status::SUCCESS;
}

size_t ZstdBatchManager::get_batch_device_decompress_temp_size(size_t count, size_t max_out) {
  return DecLayout::make(std::max<size_t>(1, count), max_out).total;
}

Status ZstdBatchManager::decompress_batch_device(const void *const *d_in_ptrs, const size_t *d_in_sizes, const size_t *d_out_caps, size_t max_out,
                                                 size_t count, void *const *d_out_ptrs, size_t *d_out_sizes, int *d_statuses, void *temp,
                                                 size_t temp_size, hipStream_t stream) {
  // one manager serialises calls (the dictionary's use events: set_dictionary waits on them)
  std::lock_guard<std::mutex> lock(pimpl_->api_mutex);
  Status s = ensure_kernels();
  if (s != Status::SUCCESS) return s;
  if (!count) return Status::SUCCESS;
  if (!d_in_ptrs || !d_in_sizes || !d_out_ptrs || !d_out_sizes || max_out == 0) return Status::ERROR_INVALID_PARAMETER;
  DecLayout L = DecLayout::make(count, max_out);
  if (!temp || temp_size < L.total) return Status::ERROR_BUFFER_TOO_SMALL;
  u8 *base = (u8 *)(((uintptr_t)temp + 255) & ~(uintptr_t)255);
  ZhDecArgs a = L.args(base);
  pimpl_->mgr_dict.fill(a);
  a.in_ptrs = d_in_ptrs;
  a.in_sizes = d_in_sizes;
  a.out_ptrs = d_out_ptrs;
  a.out_caps = d_out_caps;
  a.out_cap_all = max_out;
  a.out_sizes = d_out_sizes;
  a.statuses = d_statuses ? (u32 *)d_statuses : (u32 *)(base + L.statuses);
  a.nvcomp_codes = 1;
  if (zh::launch_decompress(a, (u32)count, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
  return pimpl_->mgr_dict.n ? pimpl_->mgr_dict.note_use(stream) : Status::SUCCESS;
}

// ============================================================================
// Streaming manager (reference src/cuda_zstd_manager.cu:6043-6455).  compress_chunk: each chunk
// an independent frame (:6306-6310).  compress_chunk_with_history: the chunk is compressed with
// the preceding stream bytes (a 64 KiB device window, the most K1 can stage) as raw-content
// history, as the reference passes its window to compress() as a dictionary (:6327-6418).
// decompress_chunk keeps the same window of decoded bytes and hands it to the decoder, so
// chunks of either kind decode in stream order.
// ============================================================================
namespace {
struct FrameProbe {
  u64 content = 0;
  bool has_content = false, checksum = false;
  u32 dict_id = 0, window_log = 0;
  int meta_level = -1;
  size_t frame_offset = 0;
};
Status probe_frame(const void *data, size_t n, FrameProbe &f);
constexpr size_t kStreamWindow = 64 * 1024;
// a device window of the last kStreamWindow stream bytes (double-buffered: no overlapping copies)
struct HistWindow {
  u8 *buf[2] = {nullptr, nullptr};
  int cur = 0;
  size_t n = 0;
  ~HistWindow() {
    for (u8 *b : buf)
      if (b) (void)hipFree(b);
  }
  Status ensure() {
    for (u8 *&b : buf)
      if (!b && hipMalloc(&b, kStreamWindow) != hipSuccess) { b = nullptr; return Status::ERROR_OUT_OF_MEMORY; }
    return Status::SUCCESS;
  }
  const u8 *data() const { return buf[cur]; }
  // Enqueue the window's next state (its last bytes + src) into the other buffer on `stream`,
  // without waiting: the chunk call's own stream synchronisation (its compress / decompress,
  // which is blocking on return) covers it.  The current buffer stays valid until commit().
  size_t pend_n = 0;
  Status stage(const void *src, size_t len, hipStream_t stream) {
    Status s = ensure();
    if (s != Status::SUCCESS) return s;
    u8 *const dst = buf[cur ^ 1];
    size_t const take = std::min(len, kStreamWindow), keep = std::min(n, kStreamWindow - take);
    if (keep && hipMemcpyAsync(dst, buf[cur] + n - keep, keep, hipMemcpyDeviceToDevice, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    if (hipMemcpyAsync(dst + keep, (const u8 *)src + len - take, take, hipMemcpyDefault, stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    pend_n = keep + take;
    return Status::SUCCESS;
  }
  void commit() {
    cur ^= 1;
    n = pend_n;
  }
  // stage + a wait of its own (decompress_chunk: the window takes the decoded bytes, which exist
  // only after the call's synchronisation)
  Status append(const void *src, size_t len, hipStream_t stream) {
    Status s = stage(src, len, stream);
    if (s != Status::SUCCESS) return s;
    if (hipStreamSynchronize(stream) != hipSuccess) return Status::ERROR_CUDA_ERROR;
    commit();
    return Status::SUCCESS;
  }
  void clear() { n = 0; }
};
}  // namespace

class ZstdStreamingManager::Impl {
 public:
  CompressionConfig config;
  ZstdBatchManager mgr;
  void *ws = nullptr;
  size_t ws_size = 0;
  bool comp = false, decomp = false;
  HistWindow chist, dhist;  // compressor's and decompressor's stream windows
  // the session compresses chunks against the stream history (init_compression_with_history /
  // compress_chunk_with_history): decompress_chunk then decodes against the decoded window;
  // otherwise chunks are frames of their own and decode with the manager's dictionary, if any
  bool hist_mode = false;
  bool has_dict = false;  // set_dictionary succeeded (frames with its Dictionary_ID decode with it)
  explicit Impl(const CompressionConfig &c) : config(c), mgr(c) {}
  ~Impl() { if (ws) (void)hipFree(ws); }
  Status ensure_ws(size_t need) {
    if (need <= ws_size) return Status::SUCCESS;
    if (ws) (void)hipFree(ws);
    ws = nullptr;
    ws_size = 0;
    if (hipMalloc(&ws, need) != hipSuccess) return Status::ERROR_OUT_OF_MEMORY;
    ws_size = need;
    return Status::SUCCESS;
  }
};
ZstdStreamingManager::ZstdStreamingManager() : pimpl_(new Impl(CompressionConfig::from_level(3))) {}
ZstdStreamingManager::ZstdStreamingManager(const CompressionConfig &c) : pimpl_(new Impl(c)) {}
ZstdStreamingManager::~ZstdStreamingManager() = default;
Status ZstdStreamingManager::init_compression(hipStream_t, size_t max_chunk) {
  Status s = pimpl_->ensure_ws(pimpl_->mgr.get_compress_temp_size(max_chunk ? max_chunk : (size_t)ZH_BLOCK_MAX));
  if (s != Status::SUCCESS) return s;
  pimpl_->comp = true;
  return Status::SUCCESS;
}
Status ZstdStreamingManager::init_compression_with_history(hipStream_t st, size_t m) {
  Status s = init_compression(st, m);
  if (s == Status::SUCCESS) s = pimpl_->chist.ensure();
  if (s == Status::SUCCESS) pimpl_->hist_mode = true;
  return s;
}
Status ZstdStreamingManager::init_decompression_with_history(hipStream_t st) {
  Status s = init_decompression(st);
  if (s == Status::SUCCESS) pimpl_->hist_mode = true;
  return s;
}
Status ZstdStreamingManager::init_decompression(hipStream_t) {
  Status s = pimpl_->ensure_ws(pimpl_->mgr.get_decompress_temp_size(0));
  if (s == Status::SUCCESS) s = pimpl_->dhist.ensure();
  if (s != Status::SUCCESS) return s;
  pimpl_->decomp = true;
  return Status::SUCCESS;
}
Status ZstdStreamingManager::compress_chunk(const void *in, size_t n, void *out, size_t *out_size, bool, hipStream_t stream) {
  if (!pimpl_->comp) return Status::ERROR_NOT_INITIALIZED;
  Status s = pimpl_->ensure_ws(pimpl_->mgr.get_compress_temp_size(n));
  if (s != Status::SUCCESS) return s;
  // the stream window follows every chunk, so a later chunk_with_history sees these bytes (the
  // window copy is enqueued first: compress()'s final synchronisation covers it)
  bool const win = pimpl_->chist.buf[0] != nullptr;
  if (win) {
    s = pimpl_->chist.stage(in, n, stream);
    if (s != Status::SUCCESS) return s;
  }
  s = pimpl_->mgr.compress(in, n, out, out_size, pimpl_->ws, pimpl_->ws_size, nullptr, 0, stream);
  if (s == Status::SUCCESS && win) pimpl_->chist.commit();
  else if (win) (void)hipStreamSynchronize(stream);  // (an early error return: the copy still reads `in`)
  return s;
}
Status ZstdStreamingManager::compress_chunk_with_history(const void *in, size_t n, void *out, size_t *out_size, bool, hipStream_t stream) {
  if (!in || !out || !out_size) return Status::ERROR_INVALID_PARAMETER;
  if (!pimpl_->comp || !pimpl_->chist.buf[0]) {  // auto-initialise, as the reference does
    Status s = init_compression_with_history(stream, n);
    if (s != Status::SUCCESS) return s;
  }
  Status s = pimpl_->ensure_ws(pimpl_->mgr.get_compress_temp_size(n));
  if (s != Status::SUCCESS) return s;
  // the next window state goes to the other buffer while this chunk reads the current one;
  // compress_with_history's synchronisation covers the copy
  s = pimpl_->chist.stage(in, n, stream);
  if (s != Status::SUCCESS) return s;
  s = pimpl_->mgr.compress_with_history(in, n, out, out_size, pimpl_->ws, pimpl_->ws_size, pimpl_->chist.data(), pimpl_->chist.n, stream);
  if (s == Status::SUCCESS) pimpl_->chist.commit();
  else (void)hipStreamSynchronize(stream);  // (an early error return: the copy still reads `in`)
  return s;
}
Status ZstdStreamingManager::decompress_chunk(const void *in, size_t n, void *out, size_t *out_size, bool *is_last, hipStream_t stream) {
  if (!in || !out || !out_size) return Status::ERROR_INVALID_PARAMETER;
  if (!pimpl_->decomp) {
    Status s = init_decompression(stream);
    if (s != Status::SUCCESS) return s;
  }
  if (is_last) *is_last = true;  // every chunk is a complete frame
  Status s = pimpl_->ensure_ws(pimpl_->mgr.get_decompress_temp_size(n));
  if (s != Status::SUCCESS) return s;
  // Per frame: the decoded window is the frame's history unless the frame was compressed with
  // the manager's dictionary.  Without a dictionary the window is harmless (a frame of its own
  // never reaches before its start).  With one, only a history session (compression with history
  // in this manager, or init_decompression_with_history) has history frames, and those carry no
  // Dictionary_ID: a frame naming the dictionary, or any frame outside a history session -- a
  // formatted dictionary's frame written without its ID (libzstd dictIDFlag 0) included -- decodes
  // with the dictionary.  History frames therefore need init_decompression_with_history (ADVICE
  // r5): outside a history session an ID-less frame that fails against the dictionary (corrupt, or
  // its content checksum does not hold) is decoded once more against the window; an ID-less frame
  // without a checksum that decodes against the dictionary cannot be told apart and is kept.
  bool hist_frame = true, retry_hist = false;
  if (pimpl_->has_dict) {
    FrameProbe fp;
    bool const probed = probe_frame(in, n, fp) == Status::SUCCESS;
    hist_frame = pimpl_->hist_mode && probed && fp.dict_id == 0;
    retry_hist = !pimpl_->hist_mode && probed && fp.dict_id == 0 && pimpl_->dhist.n;
  }
  bool const use_hist = pimpl_->dhist.n && hist_frame;
  size_t const cap = *out_size;
  s = pimpl_->mgr.decompress_with_history(in, n, out, out_size, pimpl_->ws, pimpl_->ws_size, use_hist ? pimpl_->dhist.data() : nullptr,
                                          use_hist ? pimpl_->dhist.n : 0, stream);
  if ((s == Status::ERROR_CHECKSUM_FAILED || s == Status::ERROR_CORRUPT_DATA) && retry_hist) {
    *out_size = cap;
    s = pimpl_->mgr.decompress_with_history(in, n, out, out_size, pimpl_->ws, pimpl_->ws_size, pimpl_->dhist.data(), pimpl_->dhist.n, stream);
  }
  if (s == Status::SUCCESS) s = pimpl_->dhist.append(out, *out_size, stream);
  return s;
}
Status ZstdStreamingManager::reset() {
  pimpl_->comp = pimpl_->decomp = false;
  pimpl_->hist_mode = false;
  pimpl_->chist.clear();
  pimpl_->dhist.clear();
  return Status::SUCCESS;
}
Status ZstdStreamingManager::reset_streaming() {
  pimpl_->chist.clear();
  pimpl_->dhist.clear();
  return Status::SUCCESS;
}
Status ZstdStreamingManager::flush(hipStream_t s) { return hipStreamSynchronize(s) == hipSuccess ? Status::SUCCESS : Status::ERROR_CUDA_ERROR; }
Status ZstdStreamingManager::flush_streaming(hipStream_t s) { return flush(s); }
Status ZstdStreamingManager::set_config(const CompressionConfig &c) { pimpl_->config = c; return pimpl_->mgr.configure(c); }
Status ZstdStreamingManager::set_dictionary(const dictionary::Dictionary &d) {
  Status const s = pimpl_->mgr.set_dictionary(d);
  if (s == Status::SUCCESS) pimpl_->has_dict = true;
  return s;
}
CompressionConfig ZstdStreamingManager::get_config() const { return pimpl_->config; }
size_t ZstdStreamingManager::get_temp_size() const { return pimpl_->ws_size; }
bool ZstdStreamingManager::is_compression_initialized() const { return pimpl_->comp; }
bool ZstdStreamingManager::is_decompression_initialized() const { return pimpl_->decomp; }

// ============================================================================
// dictionary training API (reference include/cuda_zstd_dictionary.h:176-210,
// src/cuda_zstd_dictionary.cu:421-520): COVER (zh_dict.cpp) instead of the reference's
// byte-frequency / 4-gram fill, same validation and buffer contract
// ============================================================================
namespace dictionary {
Status train_dictionary(const std::vector<const void *> &samples, const std::vector<size_t> &sample_sizes, void *dict_buffer,
                        size_t dict_size, const DictionaryTrainingParams *params, hipStream_t stream) {
  (void)params;
  (void)stream;
  if (samples.empty() || sample_sizes.empty() || !dict_buffer || samples.size() != sample_sizes.size()) return Status::ERROR_INVALID_PARAMETER;
  if (!is_valid_dictionary_size(dict_size)) return Status::ERROR_INVALID_PARAMETER;
  std::vector<std::pair<const u8 *, size_t>> s;
  size_t total = 0;
  for (size_t i = 0; i < samples.size(); i++) {
    if (!samples[i] && sample_sizes[i]) return Status::ERROR_INVALID_PARAMETER;
    s.emplace_back((const u8 *)samples[i], sample_sizes[i]);
    total += sample_sizes[i];
  }
  if (total == 0) return Status::ERROR_INVALID_PARAMETER;
  std::vector<u8> c;
  try {
    c = zh::cover_train(s, dict_size);
  } catch (...) {
    return Status::ERROR_OUT_OF_MEMORY;
  }
  if (c.empty() || c.size() > dict_size) return Status::ERROR_DICTIONARY_FAILED;
  // the buffer holds dict_size bytes: the trained content at its end (the most useful segments
  // nearest the data, as ZDICT lays them out), zeros before it when the samples gave less
  u8 *const out = (u8 *)dict_buffer;
  memset(out, 0, dict_size - c.size());
  memcpy(out + dict_size - c.size(), c.data(), c.size());
  return Status::SUCCESS;
}
Status create_dictionary_from_samples(const void *samples_buffer, const size_t *sample_offsets, size_t num_samples, void *dict_buffer,
                                      size_t dict_size, const DictionaryTrainingParams *params, hipStream_t stream) {
  if (!samples_buffer || !sample_offsets || !dict_buffer || num_samples == 0) return Status::ERROR_INVALID_PARAMETER;
  std::vector<const void *> samples;
  std::vector<size_t> sizes;
  const u8 *const base = (const u8 *)samples_buffer;
  for (size_t i = 0; i < num_samples; i++) {
    size_t const a = sample_offsets[i], e = i + 1 < num_samples ? sample_offsets[i + 1] : a + 8 * 1024;
    if (e < a) return Status::ERROR_INVALID_PARAMETER;
    samples.push_back(base + a);
    sizes.push_back(e - a);
  }
  return train_dictionary(samples, sizes, dict_buffer, dict_size, params, stream);
}
u32 get_optimal_dict_size(size_t total) {
  size_t const s = total / 100;
  if (s < MIN_DICT_SIZE) return MIN_DICT_SIZE;
  if (s > MAX_DICT_SIZE) return MAX_DICT_SIZE;
  return (u32)((s + 1023) / 1024 * 1024);
}
bool is_valid_dictionary_size(size_t size) { return size >= MIN_DICT_SIZE && size <= MAX_DICT_SIZE; }
}  // namespace dictionary

// ============================================================================
// factories / convenience (reference include/cuda_zstd_manager.h:358-386)
// ============================================================================
std::unique_ptr<ZstdManager> create_manager(int level) {
  if (!is_valid_compression_level(level)) throw std::invalid_argument("compression level");
  return std::unique_ptr<ZstdManager>(new ZstdBatchManager(CompressionConfig::from_level(level)));
}
std::unique_ptr<ZstdManager> create_manager(const CompressionConfig &c) { return std::unique_ptr<ZstdManager>(new ZstdBatchManager(c)); }
std::unique_ptr<ZstdBatchManager> create_batch_manager(int level) {
  return std::unique_ptr<ZstdBatchManager>(new ZstdBatchManager(CompressionConfig::from_level(level)));
}
std::unique_ptr<ZstdStreamingManager> create_streaming_manager(int level) {
  return std::unique_ptr<ZstdStreamingManager>(new ZstdStreamingManager(CompressionConfig::from_level(level)));
}
namespace {
// one frame through a temporary manager (level, optional dictionary), workspace allocated here
Status oneshot_compress(const void *in, size_t n, void *out, size_t *out_size, int level, const dictionary::Dictionary *dict, hipStream_t stream) {
  if (!is_valid_compression_level(level)) return Status::ERROR_INVALID_PARAMETER;
  ZstdBatchManager m(CompressionConfig::from_level(level));
  if (dict) {
    Status const sd = m.set_dictionary(*dict);
    if (sd != Status::SUCCESS) return sd;
  }
  size_t need = m.get_compress_temp_size(n);
  void *ws = nullptr;
  if (hipMalloc(&ws, need) != hipSuccess) return Status::ERROR_OUT_OF_MEMORY;
  Status s = m.compress(in, n, out, out_size, ws, need, nullptr, 0, stream);
  (void)hipFree(ws);
  return s;
}
Status oneshot_decompress(const void *in, size_t n, void *out, size_t *out_size, const dictionary::Dictionary *dict, hipStream_t stream) {
  ZstdBatchManager m;
  if (dict) {
    Status const sd = m.set_dictionary(*dict);
    if (sd != Status::SUCCESS) return sd;
  }
  size_t need = m.get_decompress_temp_size(n);
  void *ws = nullptr;
  if (hipMalloc(&ws, need) != hipSuccess) return Status::ERROR_OUT_OF_MEMORY;
  Status s = m.decompress(in, n, out, out_size, ws, need, stream);
  (void)hipFree(ws);
  return s;
}
}  // namespace
Status compress_simple(const void *in, size_t n, void *out, size_t *out_size, int level, hipStream_t stream) {
  return ZH_NOTED(oneshot_compress(in, n, out, out_size, level, nullptr, stream));
}
Status decompress_simple(const void *in, size_t n, void *out, size_t *out_size, hipStream_t stream) {
  return ZH_NOTED(oneshot_decompress(in, n, out, out_size, nullptr, stream));
}
Status compress_with_dict(const void *in, size_t n, void *out, size_t *out_size, const dictionary::Dictionary &dict, int level, hipStream_t stream) {
  return ZH_NOTED(oneshot_compress(in, n, out, out_size, level, &dict, stream));
}
Status decompress_with_dict(const void *in, size_t n, void *out, size_t *out_size, const dictionary::Dictionary &dict, hipStream_t stream) {
  return ZH_NOTED(oneshot_decompress(in, n, out, out_size, &dict, stream));
}

// reference src/cuda_zstd_types.cpp:271-560 (per-stage pool buffers) -> one region here
Status allocate_compression_workspace(CompressionWorkspace &w, size_t max_block_size, const CompressionConfig &config) {
  if (w.is_allocated || max_block_size == 0) return ZH_NOTED(Status::ERROR_INVALID_PARAMETER);
  Status const sv = config.validate();
  if (sv != Status::SUCCESS) return ZH_NOTED(sv);
  ZstdBatchManager m(config);
  size_t const need = m.get_compress_temp_size(max_block_size);
  void *p = nullptr;
  if (hipMalloc(&p, need) != hipSuccess) return ZH_NOTED(Status::ERROR_OUT_OF_MEMORY);
  w = CompressionWorkspace{};
  w.d_workspace = p;
  w.total_size = w.total_size_bytes = need;
  w.is_allocated = true;
  w.hash_table_size = 1u << config.hash_log;
  w.chain_table_size = 1u << config.chain_log;
  w.max_matches = (u32)std::min<size_t>(max_block_size, 0xFFFFFFFFu);
  w.max_costs = w.max_matches + 1;
  w.max_sequences = w.max_matches / 3;
  w.num_blocks = (u32)((max_block_size + ZH_BLOCK_MAX - 1) / ZH_BLOCK_MAX);
  return Status::SUCCESS;
}
Status free_compression_workspace(CompressionWorkspace &w) {
  Status s = Status::SUCCESS;
  if (w.d_workspace && hipFree(w.d_workspace) != hipSuccess) s = Status::ERROR_CUDA_ERROR;
  w = CompressionWorkspace{};
  return ZH_NOTED(s);
}

// Frame header fields of the first zstd frame in a buffer, after any skippable frames (the
// reference parse_zstd_frame_header skips them the same way, src/cuda_zstd_manager.cu:875-900);
// *meta_level = the level of a metadata frame written by write_metadata_frame, else -1.
namespace {
Status probe_frame(const void *data, size_t n, FrameProbe &f) {
  if (!data || n < 4) return Status::ERROR_INVALID_PARAMETER;
  size_t off = 0;
  for (int guard = 0; guard < 64; guard++) {  // (bounded number of leading skippable frames)
    u8 h[18] = {0};
    size_t const take = std::min<size_t>(n - off, sizeof(h));
    if (take < 4) return Status::ERROR_CORRUPT_DATA;
    if (copy_any(h, (const u8 *)data + off, take, 0) != Status::SUCCESS) return Status::ERROR_CUDA_ERROR;
    u32 magic;
    memcpy(&magic, h, 4);
    if ((magic & 0xFFFFFFF0u) == kSkippableMagic) {
      if (take < 8) return Status::ERROR_CORRUPT_DATA;
      u32 fs;
      memcpy(&fs, h + 4, 4);
      if (fs == 8 && take >= 16) {
        u32 cm, lv;
        memcpy(&cm, h + 8, 4);
        memcpy(&lv, h + 12, 4);
        if (cm == kMetadataMagic) f.meta_level = (int)lv;
      }
      if (n - off < 8 + (size_t)fs) return Status::ERROR_CORRUPT_DATA;
      off += 8 + (size_t)fs;
      continue;
    }
    if (magic != ZSTD_MAGIC) return Status::ERROR_INVALID_MAGIC;
    if (take < 5) return Status::ERROR_CORRUPT_DATA;
    u8 const fhd = h[4];
    u32 const fcs_flag = fhd >> 6, ss = (fhd >> 5) & 1, did = fhd & 3;
    size_t o = 5;
    if (!ss) f.window_log = 10 + (h[o++] >> 3);
    u32 const dsz = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
    if (o + dsz > take) return Status::ERROR_CORRUPT_DATA;
    for (u32 k = 0; k < dsz; k++) f.dict_id |= (u32)h[o + k] << (8 * k);
    o += dsz;
    u32 const fsz = fcs_flag == 0 ? (ss ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (o + fsz > take) return Status::ERROR_CORRUPT_DATA;
    u64 v = 0;
    for (u32 k = 0; k < fsz; k++) v |= (u64)h[o + k] << (8 * k);
    if (fsz == 2) v += 256;
    f.content = v;
    f.has_content = fsz != 0;
    f.checksum = (fhd >> 2) & 1;
    f.frame_offset = off;
    return Status::SUCCESS;
  }
  return Status::ERROR_CORRUPT_DATA;
}
}  // namespace

Status get_decompressed_size(const void *data, size_t n, size_t *out) {
  if (!data || !out || n < 4) return Status::ERROR_INVALID_PARAMETER;
  FrameProbe f;
  Status s = probe_frame(data, n, f);
  if (s != Status::SUCCESS) return s;
  if (!f.has_content) return Status::ERROR_UNSUPPORTED_FORMAT;
  *out = (size_t)f.content;
  return Status::SUCCESS;
}
Status validate_compressed_data(const void *data, size_t n, bool) {
  FrameProbe f;
  return probe_frame(data, n, f);
}

// Skippable metadata frame (RFC 8878 §3.1.2): the reference declares SkippableFrameHeader +
// CustomMetadataFrame {custom magic, compression level} and a device writer
// (src/cuda_zstd_manager.cu:309-318, 391-412) but never calls it.  Here it is a utility: 16
// bytes [0x184D2A50][8][kMetadataMagic][level] in front of frames; every zstd decoder (libzstd,
// zh_decode.hip) skips it, extract_metadata reads the level back.
Status write_metadata_frame(void *out, size_t capacity, int level, size_t *written, hipStream_t stream) {
  if (!out || !written) return Status::ERROR_INVALID_PARAMETER;
  if (capacity < kMetadataFrameBytes) return Status::ERROR_BUFFER_TOO_SMALL;
  u32 const w[4] = {kSkippableMagic, 8u, kMetadataMagic, (u32)level};
  Status s = copy_any(out, w, sizeof(w), stream);
  if (s == Status::SUCCESS) *written = kMetadataFrameBytes;
  return s;
}

// reference is_nvcomp_zstd_format / extract_metadata (include/cuda_zstd_manager.h:415-419,
// src/cuda_zstd_manager.cu:992-1030): frame header fields after any skippable frames; the
// level comes from a metadata frame (3 when there is none, as the reference reports)
bool is_nvcomp_zstd_format(const void *data, size_t n) {
  FrameProbe f;
  return probe_frame(data, n, f) == Status::SUCCESS;
}
Status extract_metadata(const void *data, size_t n, NvcompMetadata &m) {
  FrameProbe f;
  Status s = probe_frame(data, n, f);
  if (s != Status::SUCCESS) return s;
  m.format_version = get_format_version();
  m.compression_level = f.meta_level >= 0 ? (u32)f.meta_level : 3u;
  m.uncompressed_size = f.has_content ? f.content : 0;
  m.dictionary_id = f.dict_id;
  m.checksum_policy = f.checksum ? ChecksumPolicy::COMPUTE_AND_VERIFY : ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  m.chunk_size = 128 * 1024;
  m.num_chunks = f.has_content ? (u32)((f.content + m.chunk_size - 1) / m.chunk_size) : 0;
  return Status::SUCCESS;
}

// ============================================================================
// NVCOMP v5 layer (reference src/cuda_zstd_nvcomp.cpp)
// ============================================================================
namespace nvcomp_v5 {
int status_to_nvcomp_error(Status s) {
  switch (s) {
    case Status::SUCCESS: return 0;
    case Status::ERROR_INVALID_PARAMETER: return 2;
    case Status::ERROR_OUT_OF_MEMORY: return 3;
    case Status::ERROR_CUDA_ERROR: return 4;
    case Status::ERROR_CORRUPT_DATA: return 6;
    case Status::ERROR_BUFFER_TOO_SMALL: return 7;
    case Status::ERROR_CHECKSUM_FAILED: return 10;
    case Status::ERROR_COMPRESSION: return 12;
    default: return 1;
  }
}
Status nvcomp_error_to_status(int e) {
  switch (e) {
    case 0: return Status::SUCCESS;
    case 2: return Status::ERROR_INVALID_PARAMETER;
    case 3: return Status::ERROR_OUT_OF_MEMORY;
    case 4: return Status::ERROR_CUDA_ERROR;
    case 6: return Status::ERROR_CORRUPT_DATA;
    case 7: return Status::ERROR_BUFFER_TOO_SMALL;
    case 10: return Status::ERROR_CHECKSUM_FAILED;
    case 12: return Status::ERROR_COMPRESSION;
    default: return Status::ERROR_GENERIC;
  }
}
const char *get_nvcomp_v5_error_string(int e) { return status_to_string(nvcomp_error_to_status(e)); }
bool is_nvcomp_v5_zstd_format(const void *data, size_t n) {
  if (!data || n < 4) return false;
  u32 m = 0;
  if (copy_any(&m, data, 4, 0) != Status::SUCCESS) return false;
  return m == ZSTD_MAGIC;
}
bool is_compatible_with_nvcomp_v5(u32 v) { return (v >> 16) == 5; }
NvcompV5Options to_nvcomp_v5_opts(const CompressionConfig &c) {
  NvcompV5Options o;
  o.level = c.level;
  o.chunk_size = c.block_size;
  o.enable_checksum = c.checksum != ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  return o;
}
CompressionConfig from_nvcomp_v5_opts(const NvcompV5Options &o) {
  CompressionConfig c = CompressionConfig::from_level(o.level);
  c.block_size = o.chunk_size;
  c.checksum = o.enable_checksum ? ChecksumPolicy::COMPUTE_NO_VERIFY : ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  return c;
}
std::unique_ptr<ZstdManager> create_nvcomp_v5_manager(const NvcompV5Options &o) { return create_manager(from_nvcomp_v5_opts(o)); }

class NvcompV5BatchManager::Impl {
 public:
  NvcompV5Options opts;
  ZstdBatchManager mgr;
  explicit Impl(const NvcompV5Options &o) : opts(o), mgr(config_of(o)) {}
  static CompressionConfig config_of(const NvcompV5Options &o) {  // level + checksum option
    CompressionConfig c = CompressionConfig::from_level(o.level);
    c.checksum = o.enable_checksum ? ChecksumPolicy::COMPUTE_NO_VERIFY : ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
    return c;
  }
};
NvcompV5BatchManager::NvcompV5BatchManager(const NvcompV5Options &o) : pimpl_(new Impl(o)) {}
NvcompV5BatchManager::~NvcompV5BatchManager() = default;
ZstdBatchManager &NvcompV5BatchManager::batch_manager() { return pimpl_->mgr; }

template <typename T>
static Status fetch_array(std::vector<T> &dst, const T *src, size_t n, hipStream_t stream) {
  dst.resize(n);
  if (!n) return Status::SUCCESS;
  if (is_device_ptr(src)) return copy_any(dst.data(), src, n * sizeof(T), stream);
  memcpy(dst.data(), src, n * sizeof(T));
  return Status::SUCCESS;
}

size_t NvcompV5BatchManager::get_compress_temp_size(const size_t *sizes, size_t n, hipStream_t stream) const {
  if (!n || !sizes) return 0;
  std::vector<size_t> h;
  if (fetch_array(h, sizes, n, stream) != Status::SUCCESS) return 0;
  return pimpl_->mgr.get_batch_compress_temp_size(h);
}
size_t NvcompV5BatchManager::get_decompress_temp_size(const size_t *, size_t n, hipStream_t) const {
  return pimpl_->mgr.get_batch_decompress_temp_size(std::vector<size_t>(n));
}
size_t NvcompV5BatchManager::get_max_compressed_chunk_size(size_t n) const { return pimpl_->mgr.get_max_compressed_size(n); }
const CompressionStats &NvcompV5BatchManager::get_stats() const { return pimpl_->mgr.get_stats(); }

Status NvcompV5BatchManager::compress_async(const void *const *d_in, const size_t *in_sizes, size_t n, void *const *d_out, size_t *out_sizes,
                                            void *temp, size_t temp_bytes, hipStream_t stream) {
  if (!n) return Status::SUCCESS;
  if (!d_in || !in_sizes || !d_out || !out_sizes) return Status::ERROR_INVALID_PARAMETER;
  std::vector<const void *> hin;
  std::vector<void *> hout;
  std::vector<size_t> hsz, hcap;
  Status s = fetch_array(hin, (const void *const *)d_in, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hout, (void *const *)d_out, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hsz, in_sizes, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hcap, (const size_t *)out_sizes, n, stream);
  if (s != Status::SUCCESS) return s;
  std::vector<BatchItem> items(n);
  for (size_t i = 0; i < n; i++) {
    items[i].input_ptr = (void *)hin[i];
    items[i].output_ptr = hout[i];
    items[i].input_size = hsz[i];
    // reference callers pass the compressed-size array uninitialised; treat 0 as "sized with the bound"
    items[i].output_size = hcap[i] ? hcap[i] : get_max_compressed_chunk_size(hsz[i]);
  }
  Status r = pimpl_->mgr.compress_batch(items, temp, temp_bytes, stream);
  for (size_t i = 0; i < n; i++) hcap[i] = items[i].status == Status::SUCCESS ? items[i].output_size : 0;
  Status w = is_device_ptr(out_sizes) ? copy_any(out_sizes, hcap.data(), n * sizeof(size_t), stream) : (memcpy(out_sizes, hcap.data(), n * sizeof(size_t)), Status::SUCCESS);
  return r != Status::SUCCESS ? r : w;
}

// NvcompV5BatchManager::decompress_async (reference src/cuda_zstd_nvcomp.cpp:540-610): arrays on
// the host or the device; uncompressed_sizes in = capacity, out = bytes (0 for a failed item).
Status NvcompV5BatchManager::decompress_async(const void *const *d_in, const size_t *in_sizes, size_t n, void *const *d_out, size_t *out_sizes,
                                              void *temp, size_t temp_bytes, hipStream_t stream) {
  if (!n) return Status::SUCCESS;
  if (!d_in || !in_sizes || !d_out || !out_sizes) return Status::ERROR_INVALID_PARAMETER;
  std::vector<const void *> hin;
  std::vector<void *> hout;
  std::vector<size_t> hsz, hcap;
  Status s = fetch_array(hin, (const void *const *)d_in, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hout, (void *const *)d_out, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hsz, in_sizes, n, stream);
  if (s == Status::SUCCESS) s = fetch_array(hcap, (const size_t *)out_sizes, n, stream);
  if (s != Status::SUCCESS) return s;
  std::vector<BatchItem> items(n);
  for (size_t i = 0; i < n; i++) {
    items[i].input_ptr = (void *)hin[i];
    items[i].output_ptr = hout[i];
    items[i].input_size = hsz[i];
    items[i].output_size = hcap[i];
  }
  Status r = pimpl_->mgr.decompress_batch(items, temp, temp_bytes, stream);
  for (size_t i = 0; i < n; i++) hcap[i] = items[i].status == Status::SUCCESS ? items[i].output_size : 0;
  Status w = is_device_ptr(out_sizes) ? copy_any(out_sizes, hcap.data(), n * sizeof(size_t), stream) : (memcpy(out_sizes, hcap.data(), n * sizeof(size_t)), Status::SUCCESS);
  return r != Status::SUCCESS ? r : w;
}

Status get_metadata_async(const void *d, size_t n, NvcompV5Metadata *m, hipStream_t) {
  if (!m) return Status::ERROR_INVALID_PARAMETER;
  size_t s;
  Status st = get_decompressed_size(d, n, &s);
  if (st != Status::SUCCESS) return st;
  m->uncompressed_size = s;
  m->compressed_size = n;
  m->num_chunks = 1;
  m->chunk_size = (u32)std::min<size_t>(s, 0xFFFFFFFFu);
  return Status::SUCCESS;
}
Status get_metadata(const void *d, size_t n, NvcompV5Metadata &m) { return get_metadata_async(d, n, &m, 0); }
bool validate_metadata(const NvcompV5Metadata &m) { return is_compatible_with_nvcomp_v5(m.format_version); }
Status get_decompressed_size_async(const void *d, size_t n, size_t *out, hipStream_t) { return get_decompressed_size(d, n, out); }
Status get_num_chunks(const void *d, size_t n, size_t *out) {
  size_t s;
  Status st = get_decompressed_size(d, n, &s);
  if (st == Status::SUCCESS && out) *out = 1;
  return st;
}
Status get_chunk_sizes(const void *d, size_t n, size_t *sizes, size_t max_chunks) {
  if (!sizes || !max_chunks) return Status::ERROR_INVALID_PARAMETER;
  return get_decompressed_size(d, n, sizes);
}
}  // namespace nvcomp_v5

// ============================================================================
// HybridEngine (reference src/cuda_zstd_hybrid.cu)
// ============================================================================
// Throughput history for ADAPTIVE routing (reference src/cuda_zstd_hybrid.cu:46-136): a
// 64-sample ring per (CPU | GPU, compress | decompress), MB/s = MiB of input (compress) or of
// output (decompress) per second of the call.
struct ThroughputHistory {
  static constexpr size_t kMax = 64;
  double ring[4][kMax] = {};
  size_t count[4] = {};
  static size_t slot(ExecutionBackend b, bool comp) {
    bool const cpu = b == ExecutionBackend::CPU_LIBZSTD || b == ExecutionBackend::CPU_PARALLEL;
    return (cpu ? 0u : 2u) + (comp ? 0u : 1u);
  }
  void record(ExecutionBackend b, bool comp, double mbps) {
    size_t const k = slot(b, comp);
    ring[k][count[k] % kMax] = mbps;
    count[k]++;
  }
  double average(ExecutionBackend b, bool comp) const {
    size_t const k = slot(b, comp), n = std::min(count[k], kMax);
    if (!n) return 0.0;
    double s = 0;
    for (size_t i = 0; i < n; i++) s += ring[k][i];
    return s / (double)n;
  }
  void reset() { for (size_t &c : count) c = 0; }
};

class HybridEngine::Impl {
 public:
  HybridConfig config;
  CompressionStats stats;
  ThroughputHistory prof;
  mutable std::mutex mu;  // guards prof (get_observed_throughput may run beside a call)
  ZstdBatchManager mgr;
  explicit Impl(const HybridConfig &c) : config(c), mgr(CompressionConfig::from_level(c.compression_level)) {}
  void profile(ExecutionBackend b, bool comp, size_t bytes, double ms) {
    if (!config.enable_profiling) return;
    std::lock_guard<std::mutex> g(mu);
    prof.record(b, comp, ms > 0 ? ((double)bytes / (1024.0 * 1024.0)) / (ms / 1000.0) : 0.0);
  }
};
HybridEngine::HybridEngine() : pimpl_(new Impl(HybridConfig{})) {}
HybridEngine::HybridEngine(const HybridConfig &c) : pimpl_(new Impl(c)) {}
HybridEngine::~HybridEngine() = default;
HybridEngine::HybridEngine(HybridEngine &&) noexcept = default;
HybridEngine &HybridEngine::operator=(HybridEngine &&) noexcept = default;
double HybridEngine::get_observed_throughput(ExecutionBackend b, bool comp) const {
  std::lock_guard<std::mutex> g(pimpl_->mu);
  return pimpl_->prof.average(b, comp);
}
void HybridEngine::reset_profiling() {
  std::lock_guard<std::mutex> g(pimpl_->mu);
  pimpl_->prof.reset();
}
Status HybridEngine::configure(const HybridConfig &c) {
  if (!is_valid_compression_level(c.compression_level)) return Status::ERROR_INVALID_PARAMETER;
  pimpl_->config = c;
  return pimpl_->mgr.set_compression_level(c.compression_level);
}
HybridConfig HybridEngine::get_config() const { return pimpl_->config; }
Status HybridEngine::set_compression_level(int level) {
  if (!is_valid_compression_level(level)) return Status::ERROR_INVALID_PARAMETER;
  pimpl_->config.compression_level = level;
  return pimpl_->mgr.set_compression_level(level);
}
DataLocation HybridEngine::detect_location(const void *p) { return is_device_ptr(p) ? DataLocation::DEVICE : DataLocation::HOST; }
ExecutionBackend HybridEngine::query_routing(size_t n, DataLocation il, DataLocation ol, bool is_compression) const {
  HybridMode m = pimpl_->config.mode;
  if (m == HybridMode::FORCE_CPU) return ExecutionBackend::CPU_LIBZSTD;
  if (m == HybridMode::FORCE_GPU) return ExecutionBackend::GPU_KERNELS;
  bool const dev = il == DataLocation::DEVICE && ol == DataLocation::DEVICE;
  if (m == HybridMode::PREFER_GPU) return (il == DataLocation::HOST && ol == DataLocation::HOST) ? ExecutionBackend::CPU_LIBZSTD : ExecutionBackend::GPU_KERNELS;
  if (m == HybridMode::PREFER_CPU) return dev ? ExecutionBackend::GPU_KERNELS : ExecutionBackend::CPU_LIBZSTD;
  if (m == HybridMode::ADAPTIVE) {
    // reference src/cuda_zstd_hybrid.cu:215-240: with samples of both, the GPU when > 1.2x the CPU
    double const cpu = get_observed_throughput(ExecutionBackend::CPU_LIBZSTD, is_compression);
    double const gpu = get_observed_throughput(ExecutionBackend::GPU_KERNELS, is_compression);
    if (cpu > 0.0 && gpu > 0.0) return gpu > 1.2 * cpu ? ExecutionBackend::GPU_KERNELS : ExecutionBackend::CPU_LIBZSTD;
  }
  // AUTO (and ADAPTIVE without history): device-resident data stays on the device; host data
  // goes to libzstd
  (void)n;
  return dev ? ExecutionBackend::GPU_KERNELS : ExecutionBackend::CPU_LIBZSTD;
}
size_t HybridEngine::get_max_compressed_size(size_t n) const {
  LibZstd &z = libzstd();
  size_t a = estimate_compressed_size(n, pimpl_->config.compression_level);
  return z.ok ? std::max(a, z.compressBound(n)) : a;
}
CompressionStats HybridEngine::get_stats() const { return pimpl_->stats; }
void HybridEngine::reset_stats() { pimpl_->stats = CompressionStats{}; }

Status HybridEngine::compress(const void *in, size_t n, void *out, size_t *out_size, DataLocation il, DataLocation ol, HybridResult *res,
                              hipStream_t stream) {
  if (!in || !out || !out_size || n == 0) return Status::ERROR_INVALID_PARAMETER;
  if (il == DataLocation::UNKNOWN) il = detect_location(in);
  if (ol == DataLocation::UNKNOWN) ol = detect_location(out);
  auto t0 = std::chrono::steady_clock::now();
  ExecutionBackend be = query_routing(n, il, ol, true);
  Status s;
  if (be == ExecutionBackend::CPU_LIBZSTD) {
    s = cpu_compress(in, n, out, out_size, pimpl_->config.compression_level, stream);
  } else {
    // device pipeline: stage host buffers through device memory when needed
    const void *din = in;
    void *dout = out, *tmp_in = nullptr, *tmp_out = nullptr, *ws = nullptr;
    size_t const cap = *out_size;
    s = Status::SUCCESS;
    if (il != DataLocation::DEVICE) {
      if (hipMalloc(&tmp_in, n) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
      else s = copy_any(tmp_in, in, n, stream);
      din = tmp_in;
    }
    if (s == Status::SUCCESS && ol != DataLocation::DEVICE) {
      if (hipMalloc(&tmp_out, cap) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
      dout = tmp_out;
    }
    size_t need = pimpl_->mgr.get_compress_temp_size(n);
    if (s == Status::SUCCESS && hipMalloc(&ws, need) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
    if (s == Status::SUCCESS) s = pimpl_->mgr.compress(din, n, dout, out_size, ws, need, nullptr, 0, stream);
    if (s == Status::SUCCESS && tmp_out) s = copy_any(out, tmp_out, *out_size, stream);
    if (tmp_in) (void)hipFree(tmp_in);
    if (tmp_out) (void)hipFree(tmp_out);
    if (ws) (void)hipFree(ws);
  }
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (s == Status::SUCCESS) {
    pimpl_->stats.input_bytes += n;
    pimpl_->stats.output_bytes += *out_size;
    pimpl_->stats.compression_time_ms += ms;
    pimpl_->profile(be, true, n, ms);
  }
  if (res) {
    res->backend_used = be;
    res->input_location = il;
    res->output_location = ol;
    res->total_time_ms = ms;
    res->compute_time_ms = ms;
    res->input_bytes = n;
    res->output_bytes = s == Status::SUCCESS ? *out_size : 0;
    res->compression_ratio = (s == Status::SUCCESS && *out_size) ? (float)n / *out_size : 0.f;
    res->throughput_mbps = ms > 0 ? n / 1e6 / (ms / 1e3) : 0;
    res->routing_reason = be == ExecutionBackend::CPU_LIBZSTD ? "cpu (libzstd)" : "gpu (gfx950 kernels)";
  }
  return ZH_NOTED(s);
}

// same routing as compress (reference src/cuda_zstd_hybrid.cu:836-905): libzstd for host data /
// FORCE_CPU, the gfx950 decoder for device data (host buffers staged through HBM when forced)
Status HybridEngine::decompress(const void *in, size_t n, void *out, size_t *out_size, DataLocation il, DataLocation ol, HybridResult *res,
                                hipStream_t stream) {
  if (!in || !out || !out_size || n < 4) return Status::ERROR_INVALID_PARAMETER;
  if (il == DataLocation::UNKNOWN) il = detect_location(in);
  if (ol == DataLocation::UNKNOWN) ol = detect_location(out);
  auto t0 = std::chrono::steady_clock::now();
  ExecutionBackend be = query_routing(n, il, ol, false);
  Status s;
  if (be == ExecutionBackend::CPU_LIBZSTD) {
    s = cpu_decompress(in, n, out, out_size, stream);
  } else {
    const void *din = in;
    void *dout = out, *tmp_in = nullptr, *tmp_out = nullptr, *ws = nullptr;
    size_t const cap = *out_size;
    s = Status::SUCCESS;
    if (il != DataLocation::DEVICE) {
      if (hipMalloc(&tmp_in, n) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
      else s = copy_any(tmp_in, in, n, stream);
      din = tmp_in;
    }
    if (s == Status::SUCCESS && ol != DataLocation::DEVICE) {
      if (hipMalloc(&tmp_out, std::max<size_t>(cap, 1)) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
      dout = tmp_out;
    }
    size_t need = pimpl_->mgr.get_decompress_temp_size(n);
    if (s == Status::SUCCESS && hipMalloc(&ws, need) != hipSuccess) s = Status::ERROR_OUT_OF_MEMORY;
    if (s == Status::SUCCESS) s = pimpl_->mgr.decompress(din, n, dout, out_size, ws, need, stream);
    if (s == Status::SUCCESS && tmp_out) s = copy_any(out, tmp_out, *out_size, stream);
    if (tmp_in) (void)hipFree(tmp_in);
    if (tmp_out) (void)hipFree(tmp_out);
    if (ws) (void)hipFree(ws);
  }
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (s == Status::SUCCESS) {
    pimpl_->stats.bytes_decompressed += *out_size;
    pimpl_->stats.decompression_time_ms += ms;
    pimpl_->profile(be, false, *out_size, ms);
  }
  if (res) {
    res->backend_used = be;
    res->input_location = il;
    res->output_location = ol;
    res->total_time_ms = ms;
    res->compute_time_ms = ms;
    res->input_bytes = n;
    res->output_bytes = s == Status::SUCCESS ? *out_size : 0;
  }
  return ZH_NOTED(s);
}

// reference src/cuda_zstd_hybrid.cu:912-992: items one by one through the routing; per-item
// BatchRoutingResult; ERROR_COMPRESSION / ERROR_DECOMPRESSION when any item failed
Status HybridEngine::compress_batch(const void *const *inputs, const size_t *sizes, void **outputs, size_t *out_sizes, size_t count,
                                    DataLocation il, DataLocation ol, BatchRoutingResult *results, hipStream_t stream) {
  if (!inputs || !sizes || !outputs || !out_sizes || count == 0) return ZH_NOTED(Status::ERROR_INVALID_PARAMETER);
  bool ok = true;
  for (size_t i = 0; i < count; i++) {
    HybridResult r;
    Status s = compress(inputs[i], sizes[i], outputs[i], &out_sizes[i], il, ol, &r, stream);
    if (results) {
      results[i].item_index = i;
      results[i].backend_used = r.backend_used;
      results[i].status = s;
      results[i].input_bytes = sizes[i];
      results[i].output_bytes = out_sizes[i];
      results[i].compute_time_ms = r.compute_time_ms;
    }
    ok &= s == Status::SUCCESS;
  }
  return ok ? Status::SUCCESS : ZH_NOTED(Status::ERROR_COMPRESSION);
}
Status HybridEngine::decompress_batch(const void *const *inputs, const size_t *sizes, void **outputs, size_t *out_sizes, size_t count,
                                      DataLocation il, DataLocation ol, BatchRoutingResult *results, hipStream_t stream) {
  if (!inputs || !sizes || !outputs || !out_sizes || count == 0) return ZH_NOTED(Status::ERROR_INVALID_PARAMETER);
  bool ok = true;
  for (size_t i = 0; i < count; i++) {
    HybridResult r;
    Status s = decompress(inputs[i], sizes[i], outputs[i], &out_sizes[i], il, ol, &r, stream);
    if (results) {
      results[i].item_index = i;
      results[i].backend_used = r.backend_used;
      results[i].status = s;
      results[i].input_bytes = sizes[i];
      results[i].output_bytes = out_sizes[i];
      results[i].compute_time_ms = r.compute_time_ms;
    }
    ok &= s == Status::SUCCESS;
  }
  return ok ? Status::SUCCESS : ZH_NOTED(Status::ERROR_DECOMPRESSION);
}

Status hybrid_decompress(const void *in, size_t n, void *out, size_t *out_size, DataLocation il, DataLocation ol, HybridResult *res, hipStream_t stream) {
  HybridEngine e;
  return e.decompress(in, n, out, out_size, il, ol, res, stream);
}
Status hybrid_compress(const void *in, size_t n, void *out, size_t *out_size, DataLocation il, DataLocation ol, int level, HybridResult *res,
                       hipStream_t stream) {
  HybridConfig c;
  c.compression_level = level;
  HybridEngine e(c);
  return e.compress(in, n, out, out_size, il, ol, res, stream);
}
std::unique_ptr<HybridEngine> create_hybrid_engine(const HybridConfig &c) { return std::unique_ptr<HybridEngine>(new HybridEngine(c)); }
std::unique_ptr<HybridEngine> create_hybrid_engine(int level) {
  HybridConfig c;
  c.compression_level = level;
  return create_hybrid_engine(c);
}

}  // namespace cuda_zstd

// ============================================================================
// C ABI (reference src/cuda_zstd_c_api.cpp:10-209, src/cuda_zstd_nvcomp.cpp:766-840)
// ============================================================================
using namespace cuda_zstd;
using nvcomp_v5::status_to_nvcomp_error;

struct cuda_zstd_manager_t { std::unique_ptr<ZstdBatchManager> manager; };
// the handle owns the bytes; `dict` is the reference-shaped view of them (its copy operations
// would malloc, so it is never copied here)
struct cuda_zstd_dict_t {
  std::vector<u8> bytes;
  std::unique_ptr<dictionary::Dictionary> dict;
  void set(std::vector<u8> &&b, u32 id) {
    bytes = std::move(b);
    dict.reset(new dictionary::Dictionary);
    dict->raw_content = bytes.data();
    dict->raw_size = (u32)bytes.size();
    dict->header.dictionary_id = id;
    dict->header.raw_content_size = (u32)bytes.size();
  }
};
struct nvcomp_zstd_batch_manager_t { std::unique_ptr<nvcomp_v5::NvcompV5BatchManager> mgr; };
struct cuda_zstd_hybrid_engine_t { std::unique_ptr<HybridEngine> engine; };

// every C entry's Status -> the reference's int codes; failures also go to the last-error slot
static int c_err(Status s) { return status_to_nvcomp_error(s == Status::SUCCESS ? s : noted(s, "C API", 0)); }

extern "C" {

cuda_zstd_manager_t *cuda_zstd_create_manager(int level) {
  try {
    if (!is_valid_compression_level(level)) return nullptr;
    auto *m = new cuda_zstd_manager_t;
    m->manager.reset(new ZstdBatchManager(CompressionConfig::from_level(level)));
    return m;
  } catch (...) {
    return nullptr;
  }
}
void cuda_zstd_destroy_manager(cuda_zstd_manager_t *m) { delete m; }

int cuda_zstd_compress(cuda_zstd_manager_t *m, const void *src, size_t n, void *dst, size_t *dst_size, void *ws, size_t ws_size, hipStream_t stream) {
  if (!m || !m->manager) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->manager->compress(src, n, dst, dst_size, ws, ws_size, nullptr, 0, stream));
}
int cuda_zstd_decompress(cuda_zstd_manager_t *m, const void *src, size_t n, void *dst, size_t *dst_size, void *ws, size_t ws_size, hipStream_t stream) {
  if (!m || !m->manager) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->manager->decompress(src, n, dst, dst_size, ws, ws_size, stream));
}
size_t cuda_zstd_get_compress_workspace_size(cuda_zstd_manager_t *m, size_t n) { return (m && m->manager) ? m->manager->get_compress_temp_size(n) : 0; }
size_t cuda_zstd_get_decompress_workspace_size(cuda_zstd_manager_t *m, size_t n) { return (m && m->manager) ? m->manager->get_decompress_temp_size(n) : 0; }
size_t cuda_zstd_get_max_compressed_size(cuda_zstd_manager_t *m, size_t n) { return (m && m->manager) ? m->manager->get_max_compressed_size(n) : 0; }

cuda_zstd_dict_t *cuda_zstd_train_dictionary(const void **samples, const size_t *sizes, size_t num, size_t dict_size) {
  if (!samples || !sizes || num == 0 || dict_size == 0) return nullptr;
  try {
    // COVER-trained raw content (zh_dict.cpp), replacing the reference's n-gram fill
    // (src/cuda_zstd_dictionary.cu:179-415); samples are host buffers
    std::vector<std::pair<const u8 *, size_t>> s;
    for (size_t i = 0; i < num; i++) {
      if (!samples[i] || sizes[i] == 0) return nullptr;  // (reference src/cuda_zstd_c_api.cpp:142-145)
      s.emplace_back((const u8 *)samples[i], sizes[i]);
    }
    std::vector<u8> c = zh::cover_train(s, std::min(dict_size, zh::kDictMaxBytes));
    if (c.size() < dictionary::MIN_DICT_SIZE) return nullptr;  // (set_dictionary would refuse it)
    auto *d = new cuda_zstd_dict_t;
    d->set(std::move(c), 0);
    return d;
  } catch (...) {
    return nullptr;
  }
}
void cuda_zstd_destroy_dictionary(cuda_zstd_dict_t *d) { delete d; }
// reference DictionaryManager::load_dictionary (include/cuda_zstd_dictionary.h:292-310): a host
// buffer with raw content or a formatted dictionary (e.g. ZDICT_trainFromBuffer's)
cuda_zstd_dict_t *cuda_zstd_load_dictionary(const void *buffer, size_t size) {
  // the managers' set_dictionary limits (MIN_DICT_SIZE .. MAX_DICT_SIZE, reference
  // src/cuda_zstd_manager.cu:3711-3736) apply here already, so a handle is always settable
  if (!buffer || size < dictionary::MIN_DICT_SIZE || size > zh::kDictMaxBytes) return nullptr;
  u32 id = 0;
  size_t off = 0;
  if (!zh::dict_layout((const u8 *)buffer, size, id, off)) return nullptr;
  try {
    auto *d = new cuda_zstd_dict_t;
    d->set(std::vector<u8>((const u8 *)buffer, (const u8 *)buffer + size), id);
    return d;
  } catch (...) {
    return nullptr;
  }
}
size_t cuda_zstd_get_dictionary_content(const cuda_zstd_dict_t *d, void *out, size_t capacity) {
  if (!d || !d->dict) return 0;
  size_t const n = d->bytes.size();
  if (out && capacity >= n) memcpy(out, d->bytes.data(), n);
  return n;
}
int cuda_zstd_get_dictionary_layout(const cuda_zstd_dict_t *d, unsigned int *dict_id, size_t *content_offset) {
  if (!d || !d->dict) return c_err(Status::ERROR_INVALID_PARAMETER);
  u32 id = 0;
  size_t off = 0;
  if (!zh::dict_layout(d->bytes.data(), d->bytes.size(), id, off)) return c_err(Status::ERROR_DICTIONARY_FAILED);
  if (dict_id) *dict_id = id;
  if (content_offset) *content_offset = off;
  return 0;
}
int cuda_zstd_clear_dictionary(cuda_zstd_manager_t *m) {
  if (!m || !m->manager) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->manager->clear_dictionary());
}
int cuda_zstd_set_dictionary(cuda_zstd_manager_t *m, cuda_zstd_dict_t *d) {
  if (!m || !m->manager || !d || !d->dict) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->manager->set_dictionary(*d->dict));
}
const char *cuda_zstd_get_error_string(int code) { return status_to_string(nvcomp_v5::nvcomp_error_to_status(code)); }
int cuda_zstd_is_error(int code) { return code != 0; }

size_t cuda_zstd_get_batch_compress_workspace_size(cuda_zstd_manager_t *m, const size_t *sizes, size_t count) {
  if (!m || !m->manager || (!sizes && count)) return 0;
  return m->manager->get_batch_compress_temp_size(std::vector<size_t>(sizes, sizes + count));
}
int cuda_zstd_compress_batch(cuda_zstd_manager_t *m, const void *const *in_ptrs, const size_t *in_sizes, size_t count, void *const *out_ptrs,
                             size_t *out_sizes, int *statuses, void *ws, size_t ws_size, hipStream_t stream) {
  if (!m || !m->manager || (count && (!in_ptrs || !in_sizes || !out_ptrs || !out_sizes))) return c_err(Status::ERROR_INVALID_PARAMETER);
  std::vector<BatchItem> items(count);
  for (size_t i = 0; i < count; i++) {
    items[i].input_ptr = (void *)in_ptrs[i];
    items[i].output_ptr = out_ptrs[i];
    items[i].input_size = in_sizes[i];
    items[i].output_size = out_sizes[i];
  }
  Status s = m->manager->compress_batch(items, ws, ws_size, stream);
  for (size_t i = 0; i < count; i++) {
    if (items[i].status == Status::SUCCESS) out_sizes[i] = items[i].output_size;
    if (statuses) statuses[i] = c_err(items[i].status);
  }
  return c_err(s);
}
size_t cuda_zstd_get_batch_decompress_workspace_size(cuda_zstd_manager_t *m, const size_t *sizes, size_t count) {
  if (!m || !m->manager || (!sizes && count)) return 0;
  return m->manager->get_batch_decompress_temp_size(std::vector<size_t>(sizes, sizes + count));
}
int cuda_zstd_decompress_batch(cuda_zstd_manager_t *m, const void *const *in_ptrs, const size_t *in_sizes, size_t count, void *const *out_ptrs,
                               size_t *out_sizes, int *statuses, void *ws, size_t ws_size, hipStream_t stream) {
  if (!m || !m->manager || (count && (!in_ptrs || !in_sizes || !out_ptrs || !out_sizes))) return c_err(Status::ERROR_INVALID_PARAMETER);
  std::vector<BatchItem> items(count);
  for (size_t i = 0; i < count; i++) {
    items[i].input_ptr = (void *)in_ptrs[i];
    items[i].output_ptr = out_ptrs[i];
    items[i].input_size = in_sizes[i];
    items[i].output_size = out_sizes[i];
  }
  Status s = m->manager->decompress_batch(items, ws, ws_size, stream);
  for (size_t i = 0; i < count; i++) {
    out_sizes[i] = items[i].status == Status::SUCCESS ? items[i].output_size : 0;
    if (statuses) statuses[i] = c_err(items[i].status);
  }
  return c_err(s);
}

nvcompZstdManagerHandle nvcomp_zstd_create_manager_v5(int level) {
  try {
    if (!is_valid_compression_level(level)) return nullptr;
    return (nvcompZstdManagerHandle) new ZstdBatchManager(CompressionConfig::from_level(level));
  } catch (...) {
    return nullptr;
  }
}
void nvcomp_zstd_destroy_manager_v5(nvcompZstdManagerHandle h) { delete static_cast<ZstdBatchManager *>(h); }
int nvcomp_zstd_compress_async_v5(nvcompZstdManagerHandle h, const void *in, size_t n, void *out, size_t *out_size, void *t, size_t ts, hipStream_t s) {
  auto *m = static_cast<ZstdBatchManager *>(h);
  if (!m) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->compress(in, n, out, out_size, t, ts, nullptr, 0, s));
}
int nvcomp_zstd_decompress_async_v5(nvcompZstdManagerHandle h, const void *in, size_t n, void *out, size_t *out_size, void *t, size_t ts, hipStream_t s) {
  auto *m = static_cast<ZstdBatchManager *>(h);
  if (!m) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->decompress(in, n, out, out_size, t, ts, s));
}
size_t nvcomp_zstd_get_compress_temp_size_v5(nvcompZstdManagerHandle h, size_t n) { return h ? static_cast<ZstdBatchManager *>(h)->get_compress_temp_size(n) : 0; }
size_t nvcomp_zstd_get_decompress_temp_size_v5(nvcompZstdManagerHandle h, size_t n) { return h ? static_cast<ZstdBatchManager *>(h)->get_decompress_temp_size(n) : 0; }
int nvcomp_zstd_get_metadata_v5(const void *d, size_t n, nvcomp_v5::NvcompV5Metadata *m, hipStream_t s) {
  return c_err(nvcomp_v5::get_metadata_async(d, n, m, s));
}

nvcomp_zstd_batch_manager_t *nvcomp_zstd_batch_create_v5(int level, unsigned int chunk_size, int enable_checksum) {
  try {
    if (!is_valid_compression_level(level)) return nullptr;
    nvcomp_v5::NvcompV5Options o;
    o.level = level;
    o.chunk_size = chunk_size ? chunk_size : 64 * 1024;
    o.enable_checksum = enable_checksum != 0;
    auto *m = new nvcomp_zstd_batch_manager_t;
    m->mgr.reset(new nvcomp_v5::NvcompV5BatchManager(o));
    return m;
  } catch (...) {
    return nullptr;
  }
}
void nvcomp_zstd_batch_destroy_v5(nvcomp_zstd_batch_manager_t *m) { delete m; }
size_t nvcomp_zstd_batch_get_compress_temp_size_v5(nvcomp_zstd_batch_manager_t *m, const size_t *sizes, size_t n) {
  return (m && m->mgr) ? m->mgr->get_compress_temp_size(sizes, n) : 0;
}
size_t nvcomp_zstd_batch_get_max_compressed_chunk_size_v5(nvcomp_zstd_batch_manager_t *m, size_t n) {
  return (m && m->mgr) ? m->mgr->get_max_compressed_chunk_size(n) : 0;
}
int nvcomp_zstd_batch_compress_async_v5(nvcomp_zstd_batch_manager_t *m, const void *const *in, const size_t *in_sizes, size_t n, void *const *out,
                                        size_t *out_sizes, void *t, size_t tb, hipStream_t s) {
  if (!m || !m->mgr) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->mgr->compress_async(in, in_sizes, n, out, out_sizes, t, tb, s));
}
size_t nvcomp_zstd_batched_compress_get_temp_size_v5(size_t n, size_t max_chunk) { return ZstdBatchManager::get_batch_device_temp_size(n, max_chunk); }
size_t nvcomp_zstd_batch_get_batched_temp_size_v5(nvcomp_zstd_batch_manager_t *m, size_t n, size_t max_chunk) {
  return (m && m->mgr) ? m->mgr->batch_manager().get_batch_device_temp_size_for(n, max_chunk) : 0;
}
int nvcomp_zstd_batch_set_dictionary_v5(nvcomp_zstd_batch_manager_t *m, cuda_zstd_dict_t *d) {
  if (!m || !m->mgr || !d || !d->dict) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->mgr->batch_manager().set_dictionary(*d->dict));
}
int nvcomp_zstd_batched_compress_async_v5(nvcomp_zstd_batch_manager_t *m, const void *const *d_in, const size_t *d_in_sizes, size_t max_chunk,
                                          size_t n, void *const *d_out, size_t *d_out_sizes, int *d_statuses, void *t, size_t tb, hipStream_t s) {
  if (!m || !m->mgr) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->mgr->batch_manager().compress_batch_device(d_in, d_in_sizes, max_chunk, n, d_out, d_out_sizes, d_statuses, t, tb, s));
}
size_t nvcomp_zstd_batch_get_decompress_temp_size_v5(nvcomp_zstd_batch_manager_t *m, const size_t *sizes, size_t n) {
  return (m && m->mgr) ? m->mgr->get_decompress_temp_size(sizes, n) : 0;
}
int nvcomp_zstd_batch_decompress_async_v5(nvcomp_zstd_batch_manager_t *m, const void *const *in, const size_t *in_sizes, size_t n, void *const *out,
                                          size_t *out_sizes, void *t, size_t tb, hipStream_t s) {
  if (!m || !m->mgr) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(m->mgr->decompress_async(in, in_sizes, n, out, out_sizes, t, tb, s));
}
size_t nvcomp_zstd_batched_decompress_get_temp_size_v5(size_t n, size_t max_out) {
  return ZstdBatchManager::get_batch_device_decompress_temp_size(n, max_out);
}
int nvcomp_zstd_batched_decompress_async_v5(nvcomp_zstd_batch_manager_t *m, const void *const *d_in, const size_t *d_in_sizes,
                                            const size_t *d_out_caps, size_t max_out, size_t n, void *const *d_out, size_t *d_out_sizes,
                                            int *d_statuses, void *t, size_t tb, hipStream_t s) {
  if (!m || !m->mgr) return c_err(Status::ERROR_INVALID_PARAMETER);
  return c_err(
      m->mgr->batch_manager().decompress_batch_device(d_in, d_in_sizes, d_out_caps, max_out, n, d_out, d_out_sizes, d_statuses, t, tb, s));
}

cuda_zstd_hybrid_engine_t *cuda_zstd_hybrid_create(const cuda_zstd_hybrid_config_t *c) {
  try {
    HybridConfig hc;
    if (c) {
      hc.mode = (HybridMode)c->mode;
      hc.cpu_size_threshold = c->cpu_size_threshold;
      hc.gpu_device_threshold = c->gpu_device_threshold;
      hc.compression_level = c->compression_level;
      hc.enable_profiling = c->enable_profiling != 0;
      hc.cpu_thread_count = c->cpu_thread_count;
      if (!is_valid_compression_level(hc.compression_level) || c->mode > 5) return nullptr;
    }
    auto *e = new cuda_zstd_hybrid_engine_t;
    e->engine.reset(new HybridEngine(hc));
    return e;
  } catch (...) {
    return nullptr;
  }
}
cuda_zstd_hybrid_engine_t *cuda_zstd_hybrid_create_default(void) { return cuda_zstd_hybrid_create(nullptr); }
void cuda_zstd_hybrid_destroy(cuda_zstd_hybrid_engine_t *e) { delete e; }
static void fill_result(cuda_zstd_hybrid_result_t *r, const HybridResult &h) {
  if (!r) return;
  r->backend_used = (unsigned)h.backend_used;
  r->input_location = (unsigned)h.input_location;
  r->output_location = (unsigned)h.output_location;
  r->total_time_ms = h.total_time_ms;
  r->transfer_time_ms = h.transfer_time_ms;
  r->compute_time_ms = h.compute_time_ms;
  r->throughput_mbps = h.throughput_mbps;
  r->input_bytes = h.input_bytes;
  r->output_bytes = h.output_bytes;
  r->compression_ratio = h.compression_ratio;
}
int cuda_zstd_hybrid_compress(cuda_zstd_hybrid_engine_t *e, const void *in, size_t n, void *out, size_t *out_size, unsigned il, unsigned ol,
                              cuda_zstd_hybrid_result_t *r, hipStream_t s) {
  if (!e || !e->engine || il > 3 || ol > 3) return c_err(Status::ERROR_INVALID_PARAMETER);
  HybridResult h;
  Status st = e->engine->compress(in, n, out, out_size, (DataLocation)il, (DataLocation)ol, &h, s);
  fill_result(r, h);
  return c_err(st);
}
int cuda_zstd_hybrid_decompress(cuda_zstd_hybrid_engine_t *e, const void *in, size_t n, void *out, size_t *out_size, unsigned il, unsigned ol,
                                cuda_zstd_hybrid_result_t *r, hipStream_t s) {
  if (!e || !e->engine || il > 3 || ol > 3) return c_err(Status::ERROR_INVALID_PARAMETER);
  HybridResult h;
  Status st = e->engine->decompress(in, n, out, out_size, (DataLocation)il, (DataLocation)ol, &h, s);
  fill_result(r, h);
  return c_err(st);
}
size_t cuda_zstd_hybrid_max_compressed_size(cuda_zstd_hybrid_engine_t *e, size_t n) { return (e && e->engine) ? e->engine->get_max_compressed_size(n) : 0; }
unsigned int cuda_zstd_hybrid_query_routing(cuda_zstd_hybrid_engine_t *e, size_t n, unsigned il, unsigned ol, int is_c) {
  if (!e || !e->engine) return 0;
  return (unsigned)e->engine->query_routing(n, (DataLocation)il, (DataLocation)ol, is_c != 0);
}

void cuda_zstd_hip_profile_enable(int on) { zh::profile_enable(on != 0); }
int cuda_zstd_hip_profile_collect(double *ms3) { return zh::profile_collect(ms3); }

struct cuda_zstd_stream_t {
  std::unique_ptr<ZstdStreamingManager> m;
};
cuda_zstd_stream_t *cuda_zstd_stream_create(int level) {
  if (!is_valid_compression_level(level)) return nullptr;
  try {
    auto *h = new cuda_zstd_stream_t;
    h->m.reset(new ZstdStreamingManager(CompressionConfig::from_level(level)));
    return h;
  } catch (...) {
    return nullptr;
  }
}
void cuda_zstd_stream_destroy(cuda_zstd_stream_t *s) { delete s; }
int cuda_zstd_stream_compress_chunk(cuda_zstd_stream_t *s, const void *src, size_t n, void *dst, size_t *dst_size, int with_history, int last,
                                    hipStream_t stream) {
  if (!s || !s->m) return c_err(Status::ERROR_INVALID_PARAMETER);
  if (!with_history && !s->m->is_compression_initialized()) {
    Status st = s->m->init_compression(stream, n);
    if (st != Status::SUCCESS) return c_err(st);
  }
  return c_err(with_history ? s->m->compress_chunk_with_history(src, n, dst, dst_size, last != 0, stream)
                                             : s->m->compress_chunk(src, n, dst, dst_size, last != 0, stream));
}
int cuda_zstd_stream_decompress_chunk(cuda_zstd_stream_t *s, const void *src, size_t n, void *dst, size_t *dst_size, int *is_last,
                                      hipStream_t stream) {
  if (!s || !s->m) return c_err(Status::ERROR_INVALID_PARAMETER);
  bool l = false;
  Status st = s->m->decompress_chunk(src, n, dst, dst_size, &l, stream);
  if (is_last) *is_last = l ? 1 : 0;
  return c_err(st);
}
int cuda_zstd_stream_reset(cuda_zstd_stream_t *s) { return s && s->m ? c_err(s->m->reset()) : 2; }

int cuda_zstd_write_metadata_frame(void *dst, size_t capacity, int level, size_t *written, hipStream_t stream) {
  return c_err(write_metadata_frame(dst, capacity, level, written, stream));
}
int cuda_zstd_extract_metadata(const void *src, size_t size, unsigned int *level, unsigned long long *usize, unsigned int *dict_id, int *has_ck) {
  NvcompMetadata m;
  Status s = extract_metadata(src, size, m);
  if (s == Status::SUCCESS) {
    if (level) *level = m.compression_level;
    if (usize) *usize = m.uncompressed_size;
    if (dict_id) *dict_id = m.dictionary_id;
    if (has_ck) *has_ck = m.checksum_policy != ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  }
  return c_err(s);
}

const char *cuda_zstd_hip_version(void) { return "cuda_zstd_hip 0.2.0 (gfx950)"; }
unsigned int cuda_zstd_hip_kernel_lds_bytes(int which) { return which == 0 ? zh::lz_lds_bytes() : zh::entropy_lds_bytes(); }

}  // extern "C"
