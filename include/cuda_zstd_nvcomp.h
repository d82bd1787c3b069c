// cuda_zstd_nvcomp.h — nvCOMP v5 compatibility layer (C++ side).
//
// Mirrors the reference's include/cuda_zstd_nvcomp.h:
//   NvcompV5Options      :41-51
//   NvcompV5BatchManager :85-137  (compress_async/decompress_async: blocking on return, as in the reference)
//   NvcompV5Metadata     :144-169 and metadata helpers :172-227
//   status <-> int       :209-216 (src/cuda_zstd_nvcomp.cpp:75-119)
// The C ABI of this header (:272-336) lives in cuda_zstd_capi.h.
#ifndef CUDA_ZSTD_NVCOMP_H_
#define CUDA_ZSTD_NVCOMP_H_

#include "cuda_zstd_manager.h"

#ifdef __cplusplus
namespace cuda_zstd {
namespace nvcomp_v5 {

bool is_nvcomp_v5_zstd_format(const void *compressed_data, size_t compressed_size);
constexpr u32 get_nvcomp_v5_format_version() { return 0x00050000; }
bool is_compatible_with_nvcomp_v5(u32 format_version);

struct NvcompV5Options {
  int level;
  int algorithm;
  u32 chunk_size;
  bool enable_checksum;
  NvcompV5Options() : level(3), algorithm(0), chunk_size(64 * 1024), enable_checksum(false) {}
};

NvcompV5Options to_nvcomp_v5_opts(const CompressionConfig &config);
CompressionConfig from_nvcomp_v5_opts(const NvcompV5Options &opts);
std::unique_ptr<ZstdManager> create_nvcomp_v5_manager(const NvcompV5Options &opts);

class NvcompV5BatchManager {
 public:
  explicit NvcompV5BatchManager(const NvcompV5Options &opts);
  ~NvcompV5BatchManager();
  size_t get_compress_temp_size(const size_t *chunk_sizes, size_t num_chunks, hipStream_t stream = 0) const;
  size_t get_decompress_temp_size(const size_t *compressed_sizes, size_t num_chunks, hipStream_t stream = 0) const;
  size_t get_max_compressed_chunk_size(size_t uncompressed_chunk_size) const;
  Status compress_async(const void *const *d_uncompressed_ptrs, const size_t *uncompressed_sizes, size_t num_chunks,
                        void *const *d_compressed_ptrs, size_t *compressed_sizes, void *d_temp_storage, size_t temp_storage_bytes,
                        hipStream_t stream = 0);
  Status decompress_async(const void *const *d_compressed_ptrs, const size_t *compressed_sizes, size_t num_chunks,
                          void *const *d_uncompressed_ptrs, size_t *uncompressed_sizes, void *d_temp_storage,
                          size_t temp_storage_bytes, hipStream_t stream = 0);
  const CompressionStats &get_stats() const;
  ZstdBatchManager &batch_manager();

 private:
  class Impl;
  std::unique_ptr<Impl> pimpl_;
};

struct NvcompV5Metadata {
  u32 format_version;
  u32 library_version;
  int compression_level;
  u64 uncompressed_size;
  u64 compressed_size;
  u32 num_chunks;
  u32 chunk_size;
  u32 dictionary_id;
  ChecksumPolicy checksum_policy;
  bool has_dictionary;
  u64 checksum;
  NvcompV5Metadata()
      : format_version(get_nvcomp_v5_format_version()), library_version(0x00010000), compression_level(3), uncompressed_size(0),
        compressed_size(0), num_chunks(0), chunk_size(0), dictionary_id(0), checksum_policy(ChecksumPolicy::NO_COMPUTE_NO_VERIFY),
        has_dictionary(false), checksum(0) {}
};

Status get_metadata_async(const void *d_compressed_data, size_t compressed_size, NvcompV5Metadata *h_metadata, hipStream_t stream = 0);
Status get_metadata(const void *d_compressed_data, size_t compressed_size, NvcompV5Metadata &metadata);
bool validate_metadata(const NvcompV5Metadata &metadata);
Status get_decompressed_size_async(const void *d_compressed_data, size_t compressed_size, size_t *h_decompressed_size,
                                   hipStream_t stream = 0);
Status get_num_chunks(const void *d_compressed_data, size_t compressed_size, size_t *num_chunks);
Status get_chunk_sizes(const void *d_compressed_data, size_t compressed_size, size_t *chunk_sizes, size_t max_chunks);

int status_to_nvcomp_error(Status status);
Status nvcomp_error_to_status(int nvcomp_error);
const char *get_nvcomp_v5_error_string(int error_code);

}  // namespace nvcomp_v5
}  // namespace cuda_zstd

extern "C" int nvcomp_zstd_get_metadata_v5(const void *d_compressed_data, size_t compressed_size,
                                           cuda_zstd::nvcomp_v5::NvcompV5Metadata *h_metadata, hipStream_t stream);
#endif  // __cplusplus
#endif  // CUDA_ZSTD_NVCOMP_H_
