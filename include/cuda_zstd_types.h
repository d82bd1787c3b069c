// cuda_zstd_types.h — core types of the gfx950 Zstandard compressor.
//
// Drop-in counterpart of the reference's include/cuda_zstd_types.h:
//   Status                      include/cuda_zstd_types.h:92-128 (same values)
//   Strategy / CompressionMode  :133-160
//   ChecksumPolicy              :166-170
//   CompressionConfig           :196-232 (same fields; cpu_threshold default 0, see below)
//   CompressionStats            :238-262
//   BatchItem                   :268-274
//   DictionaryContent           :280-284
//   BatchRoutingResult          :430-437
//   Hybrid enums / structs      :312-430
// Streams are hipStream_t (same pointer ABI as cudaStream_t).
#ifndef CUDA_ZSTD_TYPES_H_
#define CUDA_ZSTD_TYPES_H_

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
namespace cuda_zstd {

typedef uint8_t byte_t;
typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int32_t i32;
typedef int64_t i64;

enum class Status : u32 {
  SUCCESS = 0,
  ERROR_GENERIC = 1,
  ERROR_INVALID_PARAMETER = 2,
  ERROR_OUT_OF_MEMORY = 3,
  ERROR_CUDA_ERROR = 4,  // HIP runtime error
  ERROR_INVALID_MAGIC = 5,
  ERROR_CORRUPT_DATA = 6,
  ERROR_CORRUPTED_DATA [[deprecated("Use ERROR_CORRUPT_DATA instead")]] = 6,  // reference :101
  ERROR_BUFFER_TOO_SMALL = 7,
  ERROR_UNSUPPORTED_VERSION = 8,
  ERROR_DICTIONARY_MISMATCH = 9,
  ERROR_CHECKSUM_FAILED = 10,
  ERROR_IO = 11,
  ERROR_COMPRESSION = 12,
  ERROR_COMPRESSION_FAILED [[deprecated("Use ERROR_COMPRESSION instead")]] = 12,  // reference :109
  ERROR_DECOMPRESSION = 13,
  ERROR_DECOMPRESSION_FAILED [[deprecated("Use ERROR_DECOMPRESSION instead")]] = 13,  // reference :112
  ERROR_WORKSPACE_INVALID = 14,
  ERROR_STREAM_ERROR = 15,
  ERROR_ALLOCATION_FAILED = 16,
  ERROR_HASH_TABLE_FULL = 17,
  ERROR_SEQUENCE_ERROR = 18,
  ERROR_NOT_INITIALIZED = 19,
  ERROR_ALREADY_INITIALIZED = 20,
  ERROR_INVALID_STATE = 21,
  ERROR_TIMEOUT = 22,
  ERROR_CANCELLED = 23,
  ERROR_NOT_IMPLEMENTED = 24,
  ERROR_INTERNAL = 25,
  ERROR_UNKNOWN = 26,
  ERROR_DICTIONARY_FAILED = 27,
  ERROR_UNSUPPORTED_FORMAT = 28
};

const char *status_to_string(Status status);

// Error context and the process-wide last-error slot (reference include/cuda_zstd_types.h:132-156,
// src/cuda_zstd_types.cpp:81-141).  The library records every failing Status of its public
// entry points here (log_error) and hands it to the callback, if one is set.
struct ErrorContext {
  Status status = Status::SUCCESS;
  const char *file = nullptr;
  int line = 0;
  const char *function = nullptr;
  const char *message = nullptr;
  hipError_t cuda_error = hipSuccess;  // HIP runtime error (the reference's cudaError_t field)

  ErrorContext() = default;
  ErrorContext(Status s, const char *f, int l, const char *fn, const char *msg = nullptr)
      : status(s), file(f), line(l), function(fn), message(msg) {}
};
// "<status> at <file>:<line> in <function>()[ - HIP Error: ...][ - message]", thread-local buffer
const char *get_detailed_error_message(const ErrorContext &ctx);
typedef void (*ErrorCallback)(const ErrorContext &ctx);
void set_error_callback(ErrorCallback callback);
void log_error(const ErrorContext &ctx);
ErrorContext get_last_error();
void clear_last_error();

enum class Strategy : u32 { FAST = 0, DFAST = 1, GREEDY = 2, LAZY = 3, LAZY2 = 4, BTLAZY2 = 5, BTOPT = 6, BTULTRA = 7 };
enum class CompressionMode : u32 { LEVEL_BASED = 0, STRATEGY_BASED = 1 };
enum class ChecksumPolicy : u32 { NO_COMPUTE_NO_VERIFY = 0, COMPUTE_NO_VERIFY = 1, COMPUTE_AND_VERIFY = 2 };

constexpr u32 ZSTD_MAGIC = 0xFD2FB528;
constexpr u32 MIN_COMPRESSION_LEVEL = 1;
constexpr u32 MAX_COMPRESSION_LEVEL = 22;
constexpr u32 DEFAULT_COMPRESSION_LEVEL = 3;
constexpr u32 MIN_WINDOW_LOG = 10;
constexpr u32 MAX_WINDOW_LOG = 31;
constexpr u32 DEFAULT_BLOCK_SIZE = 128 * 1024;

struct CompressionConfig {
  CompressionMode compression_mode = CompressionMode::LEVEL_BASED;
  int level = 3;
  bool use_exact_level = true;
  Strategy strategy = Strategy::GREEDY;
  u32 window_log = 20;
  u32 hash_log = 17;
  u32 chain_log = 17;
  u32 search_log = 8;
  u32 min_match = 3;
  u32 target_length = 0;
  u32 block_size = 128 * 1024;  // frame-header single-segment rule; device blocks are 64 KiB
  bool enable_ldm = false;
  u32 ldm_hash_log = 20;
  ChecksumPolicy checksum = ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
  // Reference default is 1 MiB (every <1 MiB input went to host libzstd).  Here the
  // device path is the default at every size; a caller that sets a threshold gets the
  // reference's host-libzstd route below it.
  u32 cpu_threshold = 0;

  static CompressionConfig from_level(int level);
  static CompressionConfig optimal(size_t input_size);
  static int strategy_to_default_level(Strategy s);
  static Strategy level_to_strategy(int level);
  Status validate() const;
  static CompressionConfig get_default();
};

// reference include/cuda_zstd_types.h:290-298
struct NvcompMetadata {
  u32 format_version = 0;
  u32 compression_level = 0;
  u64 uncompressed_size = 0;
  u32 num_chunks = 0;
  u32 chunk_size = 0;
  u32 dictionary_id = 0;
  ChecksumPolicy checksum_policy = ChecksumPolicy::NO_COMPUTE_NO_VERIFY;
};

struct CompressionStats {
  uint64_t input_bytes = 0;
  uint64_t output_bytes = 0;
  uint64_t num_blocks = 0;
  uint64_t num_sequences = 0;
  uint64_t num_literals = 0;
  uint64_t matches_found = 0;
  uint64_t bytes_compressed = 0;
  uint64_t bytes_produced = 0;
  uint64_t bytes_decompressed = 0;
  uint64_t blocks_processed = 0;
  double compression_time_ms = 0.0;
  double decompression_time_ms = 0.0;
  float get_ratio() const { return output_bytes > 0 ? (float)input_bytes / output_bytes : 0.0f; }
  double get_compression_throughput_gbps() const {
    return compression_time_ms > 0 ? (input_bytes / 1e9) / (compression_time_ms / 1000.0) : 0.0;
  }
};

struct BatchItem {
  void *input_ptr = nullptr;
  void *output_ptr = nullptr;
  size_t input_size = 0;
  size_t output_size = 0;  // in: capacity, out: compressed bytes
  Status status = Status::SUCCESS;
};

// a dictionary's device-resident content (reference include/cuda_zstd_types.h:280-284)
struct DictionaryContent {
  const unsigned char *d_buffer = nullptr;
  size_t size = 0;
  u32 dict_id = 0;
};

// ---- hybrid CPU/GPU routing (reference include/cuda_zstd_types.h:312-430) ----
enum class HybridMode : u32 { AUTO = 0, PREFER_CPU = 1, PREFER_GPU = 2, FORCE_CPU = 3, FORCE_GPU = 4, ADAPTIVE = 5 };
enum class DataLocation : u32 { HOST = 0, DEVICE = 1, MANAGED = 2, UNKNOWN = 3 };
enum class ExecutionBackend : u32 { CPU_LIBZSTD = 0, GPU_KERNELS = 1, CPU_PARALLEL = 2, GPU_BATCH = 3 };

struct HybridConfig {
  HybridMode mode = HybridMode::AUTO;
  size_t cpu_size_threshold = 1024 * 1024;
  size_t gpu_device_threshold = 64 * 1024;
  bool enable_profiling = false;
  int compression_level = 3;
  u32 cpu_thread_count = 0;
  bool use_pinned_memory = true;
  bool overlap_transfers = true;
};

struct HybridResult {
  ExecutionBackend backend_used = ExecutionBackend::CPU_LIBZSTD;
  DataLocation input_location = DataLocation::HOST;
  DataLocation output_location = DataLocation::HOST;
  double total_time_ms = 0.0;
  double transfer_time_ms = 0.0;
  double compute_time_ms = 0.0;
  double throughput_mbps = 0.0;
  size_t input_bytes = 0;
  size_t output_bytes = 0;
  float compression_ratio = 1.0f;
  const char *routing_reason = nullptr;
};

// per-item result of HybridEngine's batch calls (reference include/cuda_zstd_types.h:430-437)
struct BatchRoutingResult {
  size_t item_index = 0;
  ExecutionBackend backend_used = ExecutionBackend::CPU_LIBZSTD;
  Status status = Status::SUCCESS;
  size_t input_bytes = 0;
  size_t output_bytes = 0;
  double compute_time_ms = 0.0;
};

inline bool is_valid_compression_level(int level) {
  return level >= (int)MIN_COMPRESSION_LEVEL && level <= (int)MAX_COMPRESSION_LEVEL;
}
inline float get_compression_ratio(size_t uncompressed, size_t compressed) {
  return compressed > 0 ? static_cast<float>(uncompressed) / compressed : 0.0f;
}

// Pre-sized compression workspace (reference include/cuda_zstd_types.h:456-499, 523-527).  The
// reference carves ~20 per-stage buffers out of a memory pool; this library's kernels use one
// contiguous region (`d_workspace`, `total_size` bytes = ZstdBatchManager::get_compress_temp_size
// of max_block_size, which covers every level and the dictionary layout) that is passed as the
// temp workspace of compress().  The per-stage pointer fields are kept for source compatibility
// and stay null; the size fields report the configured search parameters.
struct CompressionWorkspace {
  u32 *d_hash_table = nullptr;
  u32 hash_table_size = 0;
  u32 *d_chain_table = nullptr;
  u32 chain_table_size = 0;
  void *d_matches = nullptr;
  u32 max_matches = 0;
  void *d_costs = nullptr;
  u32 max_costs = 0;
  u32 *d_literal_lengths_reverse = nullptr;
  u32 *d_match_lengths_reverse = nullptr;
  u32 *d_offsets_reverse = nullptr;
  u32 max_sequences = 0;
  u32 *d_frequencies = nullptr;
  u32 *d_code_lengths = nullptr;
  u32 *d_bit_offsets = nullptr;
  u32 *d_block_sums = nullptr;
  u32 *d_scanned_block_sums = nullptr;
  u32 num_blocks = 0;
  void *d_workspace = nullptr;
  size_t total_size = 0;
  size_t total_size_bytes = 0;
  bool is_allocated = false;
  hipStream_t stream = nullptr;
  hipEvent_t event_complete = nullptr;
  u32 *d_lz77_temp = nullptr;
  void *d_sequences = nullptr;
  void *d_fse_tables = nullptr;
  void *d_huffman_table = nullptr;
  void *d_bitstream = nullptr;
};
// hipMalloc of the whole region (ERROR_OUT_OF_MEMORY on failure, ERROR_INVALID_PARAMETER for a
// size of 0 or an already allocated workspace); free releases it and resets the struct.
Status allocate_compression_workspace(CompressionWorkspace &workspace, size_t max_block_size, const CompressionConfig &config);
Status free_compression_workspace(CompressionWorkspace &workspace);

}  // namespace cuda_zstd
#endif  // __cplusplus
#endif  // CUDA_ZSTD_TYPES_H_
