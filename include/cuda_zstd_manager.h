// cuda_zstd_manager.h — manager interface of the gfx950 Zstandard compressor.
//
// Same class names, virtual signatures and semantics as the reference's
// include/cuda_zstd_manager.h:
//   ZstdManager          :45-100   (pure-virtual interface)
//   ZstdBatchManager     :113-278  (compress_batch, inference decompress API)
//   ZstdStreamingManager :300-352  (each chunk an independent frame, as in the reference)
//   factories            :358-363, convenience :369-386, utilities :392-419
// The C ABI of the same header (:433-479) lives in cuda_zstd_capi.h.
#ifndef CUDA_ZSTD_MANAGER_H_
#define CUDA_ZSTD_MANAGER_H_

#include "cuda_zstd_types.h"
#include "cuda_zstd_capi.h"
#include "cuda_zstd_dictionary.h"

#ifdef __cplusplus
#include <memory>
#include <vector>

namespace cuda_zstd {

class ZstdManager {
 public:
  virtual ~ZstdManager() = default;
  virtual Status configure(const CompressionConfig &config) = 0;
  virtual CompressionConfig get_config() const = 0;
  virtual size_t get_compress_temp_size(size_t uncompressed_size) const = 0;
  virtual size_t get_decompress_temp_size(size_t compressed_size) const = 0;
  virtual size_t get_max_compressed_size(size_t uncompressed_size) const = 0;
  virtual Status compress(const void *uncompressed_data, size_t uncompressed_size, void *compressed_data, size_t *compressed_size,
                          void *temp_workspace, size_t temp_size, const void *dict_buffer, size_t dict_size, hipStream_t stream,
                          void *streaming_context = nullptr) = 0;
  virtual Status decompress(const void *compressed_data, size_t compressed_size, void *uncompressed_data, size_t *uncompressed_size,
                            void *temp_workspace, size_t temp_size, hipStream_t stream = 0) = 0;
  virtual Status set_dictionary(const dictionary::Dictionary &dict) = 0;
  virtual Status get_dictionary(dictionary::Dictionary &dict) const = 0;
  virtual Status clear_dictionary() = 0;
  virtual const CompressionStats &get_stats() const = 0;
  virtual Status set_compression_level(int level) = 0;
  virtual int get_compression_level() const = 0;
  virtual void reset_stats() = 0;

  enum class ExecutionPath { CPU, GPU_BATCH, GPU_CHUNK };
  // reference src/cuda_zstd_manager.cu:6465-6471: size < threshold -> CPU
  static ExecutionPath select_execution_path(size_t size, int cpu_threshold = 0);
  virtual Status preallocate_tables(hipStream_t stream = 0) { (void)stream; return Status::SUCCESS; }
  virtual Status free_tables(hipStream_t stream = 0) { (void)stream; return Status::SUCCESS; }
};

class ZstdBatchManager : public ZstdManager {
 public:
  ZstdBatchManager();
  explicit ZstdBatchManager(const CompressionConfig &config);
  ~ZstdBatchManager() override;

  Status configure(const CompressionConfig &config) override;
  CompressionConfig get_config() const override;
  size_t get_compress_temp_size(size_t uncompressed_size) const override;
  size_t get_decompress_temp_size(size_t compressed_size) const override;
  size_t get_max_compressed_size(size_t uncompressed_size) const override;
  Status compress(const void *uncompressed_data, size_t uncompressed_size, void *compressed_data, size_t *compressed_size,
                  void *temp_workspace, size_t temp_size, const void *dict_buffer, size_t dict_size, hipStream_t stream = 0,
                  void *streaming_context = nullptr) override;
  Status decompress(const void *compressed_data, size_t compressed_size, void *uncompressed_data, size_t *uncompressed_size,
                    void *temp_workspace, size_t temp_size, hipStream_t stream = 0) override;
  Status set_dictionary(const dictionary::Dictionary &dict) override;
  Status get_dictionary(dictionary::Dictionary &dict) const override;
  Status clear_dictionary() override;
  const CompressionStats &get_stats() const override;
  Status set_compression_level(int level) override;
  int get_compression_level() const override;
  void reset_stats() override;

  Status compress_batch(const std::vector<BatchItem> &items, void *temp_workspace, size_t temp_size, hipStream_t stream = 0);
  Status decompress_batch(const std::vector<BatchItem> &items, void *temp_workspace, size_t temp_size, hipStream_t stream = 0);
  size_t get_batch_compress_temp_size(const std::vector<size_t> &uncompressed_sizes) const;
  size_t get_batch_decompress_temp_size(const std::vector<size_t> &compressed_sizes) const;

  Status decompress_to_preallocated(const void *compressed_data, size_t compressed_size, void *preallocated_output,
                                    size_t output_capacity, size_t *actual_output_size, void *temp_workspace, size_t temp_size,
                                    hipStream_t stream = 0);
  Status decompress_batch_preallocated(std::vector<BatchItem> &items, void *temp_workspace, size_t temp_size, hipStream_t stream = 0);
  Status decompress_async_no_sync(const void *compressed_data, size_t compressed_size, void *preallocated_output,
                                  size_t output_capacity, size_t *d_actual_size, void *temp_workspace, size_t temp_size,
                                  hipStream_t stream);
  size_t get_inference_workspace_size(size_t max_compressed_size, size_t max_output_size) const;
  Status allocate_inference_workspace(size_t max_compressed_size, size_t max_output_size, void **workspace_ptr, size_t *workspace_size);
  Status free_inference_workspace(void *workspace_ptr);

  // Stream-ordered batched compression over device arrays (no host sync); used by the
  // nvcomp_zstd_batched_compress_async_v5 C entry.
  Status compress_batch_device(const void *const *d_in_ptrs, const size_t *d_in_sizes, size_t max_chunk_bytes, size_t count,
                               void *const *d_out_ptrs, size_t *d_out_sizes, int *d_statuses, void *temp_workspace, size_t temp_size,
                               hipStream_t stream);
  // levels below 5 (ZH_DEEP_LEVEL) without a dictionary; otherwise get_batch_device_temp_size_for
  static size_t get_batch_device_temp_size(size_t count, size_t max_chunk_bytes);
  // the same for this manager's level and dictionary (levels >= 5 add the deep matcher's scratch
  // slots, ~1.2 MB per persistent workgroup; a dictionary over 32 KiB chunks adds history blocks)
  size_t get_batch_device_temp_size_for(size_t count, size_t max_chunk_bytes) const;

  // Stream-ordered batched decompression over device arrays (no host sync; GPU decoder,
  // any RFC 8878 frames); used by nvcomp_zstd_batched_decompress_async_v5.
  // d_out_caps[i] = output capacity (every capacity <= max_uncompressed_chunk_bytes, or null:
  // max_uncompressed_chunk_bytes for all); d_out_sizes[i] = bytes produced (0 on error);
  // d_statuses[i] (optional) = nvcomp-style code.
  Status decompress_batch_device(const void *const *d_in_ptrs, const size_t *d_in_sizes, const size_t *d_out_caps,
                                 size_t max_uncompressed_chunk_bytes, size_t count, void *const *d_out_ptrs, size_t *d_out_sizes,
                                 int *d_statuses, void *temp_workspace, size_t temp_size, hipStream_t stream);
  static size_t get_batch_device_decompress_temp_size(size_t count, size_t max_uncompressed_chunk_bytes);

  // Streaming history (what the reference's compress_chunk_with_history does by
  // passing its device window as a raw-content dictionary, src/cuda_zstd_manager.cu:6327-6418):
  // d_history = device-resident preceding bytes (no copy), used as the frame's history; frames
  // decode with that history as a raw-content dictionary (libzstd ZSTD_decompress_usingDict too).
  Status compress_with_history(const void *uncompressed_data, size_t uncompressed_size, void *compressed_data, size_t *compressed_size,
                               void *temp_workspace, size_t temp_size, const void *d_history, size_t history_size, hipStream_t stream = 0);
  Status decompress_with_history(const void *compressed_data, size_t compressed_size, void *uncompressed_data, size_t *uncompressed_size,
                                 void *temp_workspace, size_t temp_size, const void *d_history, size_t history_size, hipStream_t stream = 0);

 private:
  class Impl;
  std::unique_ptr<Impl> pimpl_;
};

class ZstdStreamingManager {
 public:
  ZstdStreamingManager();
  explicit ZstdStreamingManager(const CompressionConfig &config);
  ~ZstdStreamingManager();
  Status init_compression(hipStream_t stream = 0, size_t max_chunk_size = 0);
  Status init_compression_with_history(hipStream_t stream = 0, size_t max_chunk_size = 0);
  Status init_decompression(hipStream_t stream = 0);
  // (not in the reference) a decode-only session whose frames came from
  // compress_chunk_with_history: with a raw-content dictionary set, decompress_chunk cannot tell
  // a history frame from a dictionary frame by its header (both carry Dictionary_ID 0)
  Status init_decompression_with_history(hipStream_t stream = 0);
  Status compress_chunk(const void *input, size_t input_size, void *output, size_t *output_size, bool is_last_chunk, hipStream_t stream = 0);
  Status compress_chunk_with_history(const void *input, size_t input_size, void *output, size_t *output_size, bool is_last_chunk,
                                     hipStream_t stream = 0);
  Status decompress_chunk(const void *input, size_t input_size, void *output, size_t *output_size, bool *is_last_chunk,
                          hipStream_t stream = 0);
  Status reset();
  Status reset_streaming();
  Status flush(hipStream_t stream = 0);
  Status flush_streaming(hipStream_t stream = 0);
  Status set_config(const CompressionConfig &config);
  Status set_dictionary(const dictionary::Dictionary &dict);
  CompressionConfig get_config() const;
  size_t get_temp_size() const;
  bool is_compression_initialized() const;
  bool is_decompression_initialized() const;

 private:
  class Impl;
  std::unique_ptr<Impl> pimpl_;
};

std::unique_ptr<ZstdManager> create_manager(int compression_level = 3);
std::unique_ptr<ZstdManager> create_manager(const CompressionConfig &config);
std::unique_ptr<ZstdBatchManager> create_batch_manager(int compression_level = 3);
std::unique_ptr<ZstdStreamingManager> create_streaming_manager(int compression_level = 3);

Status compress_simple(const void *uncompressed_data, size_t uncompressed_size, void *compressed_data, size_t *compressed_size,
                       int compression_level = 3, hipStream_t stream = 0);
Status decompress_simple(const void *compressed_data, size_t compressed_size, void *uncompressed_data, size_t *uncompressed_size,
                         hipStream_t stream = 0);
// reference include/cuda_zstd_manager.h:377-386 (declared there, never defined): one frame
// compressed against / decompressed with `dict` (raw content or RFC 8878 §5 formatted), the
// workspace allocated and freed inside the call, output valid on return
Status compress_with_dict(const void *uncompressed_data, size_t uncompressed_size, void *compressed_data, size_t *compressed_size,
                          const dictionary::Dictionary &dict, int compression_level = 3, hipStream_t stream = 0);
Status decompress_with_dict(const void *compressed_data, size_t compressed_size, void *uncompressed_data, size_t *uncompressed_size,
                            const dictionary::Dictionary &dict, hipStream_t stream = 0);

Status get_decompressed_size(const void *compressed_data, size_t compressed_size, size_t *decompressed_size);
Status validate_compressed_data(const void *compressed_data, size_t compressed_size, bool check_checksum = true);
size_t estimate_compressed_size(size_t uncompressed_size, int compression_level);
Status validate_config(const CompressionConfig &config);
void apply_level_parameters(CompressionConfig &config);
u32 get_optimal_block_size(u32 input_size, u32 compression_level);

constexpr const char *get_format_name() { return "cuda_zstd"; }
constexpr u32 get_format_version() { return 0x00010000; }
// reference include/cuda_zstd_manager.h:415-419 (skips leading skippable frames)
bool is_nvcomp_zstd_format(const void *compressed_data, size_t compressed_size);
Status extract_metadata(const void *compressed_data, size_t compressed_size, NvcompMetadata &metadata);
// 16-byte skippable metadata frame (reference SkippableFrameHeader + CustomMetadataFrame,
// src/cuda_zstd_manager.cu:309-318, 391-412) written to a host or device buffer
Status write_metadata_frame(void *output, size_t capacity, int compression_level, size_t *written, hipStream_t stream = 0);

}  // namespace cuda_zstd
#endif  // __cplusplus
#endif  // CUDA_ZSTD_MANAGER_H_
