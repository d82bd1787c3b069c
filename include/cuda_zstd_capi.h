/*
 * cuda_zstd_capi.h — the C ABI of libcuda_zstd_hip.so (plain C, for cgo/ctypes/JNI).
 *
 * Every entry point keeps the reference's name, argument order and error
 * behaviour; only cudaStream_t became hipStream_t (same pointer ABI).
 *
 *  manager API   reference include/cuda_zstd_manager.h:433-479, src/cuda_zstd_c_api.cpp:10-209
 *  nvCOMP v5 API reference include/cuda_zstd_nvcomp.h:272-336, src/cuda_zstd_nvcomp.cpp:766-840
 *  hybrid API    reference include/cuda_zstd_hybrid.h:292-363
 *  batch API     NEW C counterparts of ZstdBatchManager::compress_batch
 *                (include/cuda_zstd_manager.h:148-150) and NvcompV5BatchManager::compress_async
 *                (include/cuda_zstd_nvcomp.h:112-121), which the reference exposes only in C++,
 *                plus one stream-ordered device-array entry (nvcomp_zstd_batched_compress_async_v5).
 *
 * Return codes of the int-returning functions are the reference's
 * status_to_nvcomp_error mapping (src/cuda_zstd_nvcomp.cpp:75-96):
 * 0 OK, 2 invalid parameter, 3 out of memory, 4 device error, 6 corrupt data,
 * 7 buffer too small, 10 checksum, 12 compression, everything else 1.
 */
#ifndef CUDA_ZSTD_CAPI_H_
#define CUDA_ZSTD_CAPI_H_

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- manager API (reference include/cuda_zstd_manager.h:437-475) ---------------- */
typedef struct cuda_zstd_manager_t cuda_zstd_manager_t;
typedef struct cuda_zstd_dict_t cuda_zstd_dict_t;

cuda_zstd_manager_t *cuda_zstd_create_manager(int compression_level);
void cuda_zstd_destroy_manager(cuda_zstd_manager_t *manager);
int cuda_zstd_compress(cuda_zstd_manager_t *manager, const void *src, size_t src_size, void *dst, size_t *dst_size,
                       void *workspace, size_t workspace_size, hipStream_t stream);
int cuda_zstd_decompress(cuda_zstd_manager_t *manager, const void *src, size_t src_size, void *dst, size_t *dst_size,
                         void *workspace, size_t workspace_size, hipStream_t stream);
size_t cuda_zstd_get_compress_workspace_size(cuda_zstd_manager_t *manager, size_t src_size);
size_t cuda_zstd_get_decompress_workspace_size(cuda_zstd_manager_t *manager, size_t compressed_size);
cuda_zstd_dict_t *cuda_zstd_train_dictionary(const void **samples, const size_t *sample_sizes, size_t num_samples, size_t dict_size);
void cuda_zstd_destroy_dictionary(cuda_zstd_dict_t *dict);
int cuda_zstd_set_dictionary(cuda_zstd_manager_t *manager, cuda_zstd_dict_t *dict);
/* dictionaries: cuda_zstd_train_dictionary is COVER training (raw content);
 * load = raw content or a formatted RFC 8878 §5 dictionary from a host buffer (reference
 * DictionaryManager::load_dictionary, include/cuda_zstd_dictionary.h:292); content copies the
 * bytes out (returns the size); layout gives the Dictionary_ID and content offset (0, 0 for raw).
 * Both return NULL for a dictionary outside 256 B .. 128 KiB (MIN/MAX_DICT_SIZE, the limits
 * cuda_zstd_set_dictionary enforces), so every handle they return can be set on a manager */
cuda_zstd_dict_t *cuda_zstd_load_dictionary(const void *buffer, size_t size);
size_t cuda_zstd_get_dictionary_content(const cuda_zstd_dict_t *dict, void *out, size_t capacity);
int cuda_zstd_get_dictionary_layout(const cuda_zstd_dict_t *dict, unsigned int *dict_id, size_t *content_offset);
int cuda_zstd_clear_dictionary(cuda_zstd_manager_t *manager);
const char *cuda_zstd_get_error_string(int error_code);
int cuda_zstd_is_error(int code);

/* batch (C counterpart of ZstdBatchManager::compress_batch, src/cuda_zstd_manager.cu:5715-5797).
 * Host arrays of device pointers; out_sizes[i] is capacity on entry, bytes on exit;
 * statuses (optional) receives each item's nvcomp-style code.  Blocking, like the reference. */
size_t cuda_zstd_get_batch_compress_workspace_size(cuda_zstd_manager_t *manager, const size_t *input_sizes, size_t count);
int cuda_zstd_compress_batch(cuda_zstd_manager_t *manager, const void *const *input_ptrs, const size_t *input_sizes, size_t count,
                             void *const *output_ptrs, size_t *output_sizes, int *statuses, void *workspace,
                             size_t workspace_size, hipStream_t stream);
size_t cuda_zstd_get_max_compressed_size(cuda_zstd_manager_t *manager, size_t src_size);
/* batch decompression (C counterpart of ZstdBatchManager::decompress_batch,
 * reference include/cuda_zstd_manager.h:153-158, src/cuda_zstd_manager.cu:5799-5885): the GPU
 * decoder, one launch for all items; out_sizes[i] capacity in, bytes out (0 on error). */
size_t cuda_zstd_get_batch_decompress_workspace_size(cuda_zstd_manager_t *manager, const size_t *compressed_sizes, size_t count);
int cuda_zstd_decompress_batch(cuda_zstd_manager_t *manager, const void *const *input_ptrs, const size_t *input_sizes, size_t count,
                               void *const *output_ptrs, size_t *output_sizes, int *statuses, void *workspace, size_t workspace_size,
                               hipStream_t stream);

/* ---------------- nvCOMP v5 API (reference include/cuda_zstd_nvcomp.h:277-331) ---------------- */
typedef void *nvcompZstdManagerHandle;
nvcompZstdManagerHandle nvcomp_zstd_create_manager_v5(int compression_level);
void nvcomp_zstd_destroy_manager_v5(nvcompZstdManagerHandle handle);
int nvcomp_zstd_compress_async_v5(nvcompZstdManagerHandle handle, const void *d_uncompressed, size_t uncompressed_size,
                                  void *d_compressed, size_t *compressed_size, void *d_temp, size_t temp_size, hipStream_t stream);
int nvcomp_zstd_decompress_async_v5(nvcompZstdManagerHandle handle, const void *d_compressed, size_t compressed_size,
                                    void *d_uncompressed, size_t *uncompressed_size, void *d_temp, size_t temp_size,
                                    hipStream_t stream);
size_t nvcomp_zstd_get_compress_temp_size_v5(nvcompZstdManagerHandle handle, size_t uncompressed_size);
size_t nvcomp_zstd_get_decompress_temp_size_v5(nvcompZstdManagerHandle handle, size_t compressed_size);

/* NvcompV5BatchManager as a C handle (reference include/cuda_zstd_nvcomp.h:85-137,
 * src/cuda_zstd_nvcomp.cpp:300-484).  Pointer and size arrays may live on the host or
 * the device (probed like the reference); blocking on return. */
typedef struct nvcomp_zstd_batch_manager_t nvcomp_zstd_batch_manager_t;
nvcomp_zstd_batch_manager_t *nvcomp_zstd_batch_create_v5(int compression_level, unsigned int chunk_size, int enable_checksum);
void nvcomp_zstd_batch_destroy_v5(nvcomp_zstd_batch_manager_t *mgr);
size_t nvcomp_zstd_batch_get_compress_temp_size_v5(nvcomp_zstd_batch_manager_t *mgr, const size_t *chunk_sizes, size_t num_chunks);
size_t nvcomp_zstd_batch_get_max_compressed_chunk_size_v5(nvcomp_zstd_batch_manager_t *mgr, size_t uncompressed_chunk_size);
int nvcomp_zstd_batch_compress_async_v5(nvcomp_zstd_batch_manager_t *mgr, const void *const *d_uncompressed_ptrs,
                                        const size_t *uncompressed_sizes, size_t num_chunks, void *const *d_compressed_ptrs,
                                        size_t *compressed_sizes, void *d_temp_storage, size_t temp_storage_bytes,
                                        hipStream_t stream);

/* Stream-ordered batched compression (nvCOMP nvcompBatchedZstdCompressAsync shape).
 * All arrays are DEVICE arrays; nothing is synchronised; results are valid once
 * `stream` reaches this point.  d_compressed_sizes[i] receives bytes written;
 * d_statuses[i] (optional) the item's nvcomp-style code.  Every chunk must be
 * <= max_uncompressed_chunk_bytes and every output buffer must hold
 * nvcomp_zstd_batch_get_max_compressed_chunk_size_v5(max_uncompressed_chunk_bytes). */
size_t nvcomp_zstd_batched_compress_get_temp_size_v5(size_t num_chunks, size_t max_uncompressed_chunk_bytes);
/* The same for the handle's level and dictionary (levels >= 5, ZH_DEEP_LEVEL, add the deep
 * matcher's scratch slots; a dictionary over 32 KiB chunks adds history blocks): what a handle at
 * its level, with or without a dictionary, needs for nvcomp_zstd_batched_compress_async_v5.  (The
 * static size above covers levels below 5 without a dictionary; at levels >= 5, or with a
 * dictionary, a workspace of that size fails loudly with 7 and nothing is launched.) */
size_t nvcomp_zstd_batch_get_batched_temp_size_v5(nvcomp_zstd_batch_manager_t *mgr, size_t num_chunks, size_t max_uncompressed_chunk_bytes);
/* A dictionary for the batch handle's compress/decompress calls (the C++
 * manager's set_dictionary).  With a dictionary, chunks over 32 KiB take two history blocks:
 * size the workspace with nvcomp_zstd_batch_get_batched_temp_size_v5 after setting it. */
int nvcomp_zstd_batch_set_dictionary_v5(nvcomp_zstd_batch_manager_t *mgr, cuda_zstd_dict_t *dict);
int nvcomp_zstd_batched_compress_async_v5(nvcomp_zstd_batch_manager_t *mgr, const void *const *d_uncompressed_ptrs,
                                          const size_t *d_uncompressed_sizes, size_t max_uncompressed_chunk_bytes,
                                          size_t num_chunks, void *const *d_compressed_ptrs, size_t *d_compressed_sizes,
                                          int *d_statuses, void *d_temp_storage, size_t temp_storage_bytes,
                                          hipStream_t stream);

/* NvcompV5BatchManager::decompress_async as a C handle call (reference include/cuda_zstd_nvcomp.h:97-99,
 * 119-125): host or device arrays, uncompressed_sizes[i] capacity in, bytes out; blocking on return. */
size_t nvcomp_zstd_batch_get_decompress_temp_size_v5(nvcomp_zstd_batch_manager_t *mgr, const size_t *compressed_sizes, size_t num_chunks);
int nvcomp_zstd_batch_decompress_async_v5(nvcomp_zstd_batch_manager_t *mgr, const void *const *d_compressed_ptrs,
                                          const size_t *compressed_sizes, size_t num_chunks, void *const *d_uncompressed_ptrs,
                                          size_t *uncompressed_sizes, void *d_temp_storage, size_t temp_storage_bytes, hipStream_t stream);

/* Stream-ordered batched decompression (nvCOMP nvcompBatchedZstdDecompressAsync shape).
 * All arrays are DEVICE arrays; nothing is synchronised.  d_uncompressed_caps[i] = output
 * capacity (null: max_uncompressed_chunk_bytes for every chunk); d_actual_sizes[i] receives
 * the bytes produced (0 on error); d_statuses[i] (optional) the nvcomp-style code.
 * Decodes any RFC 8878 frame (concatenated and skippable frames included) whose blocks
 * regenerate at most min(128 KiB, max_uncompressed_chunk_bytes) bytes of literals. */
size_t nvcomp_zstd_batched_decompress_get_temp_size_v5(size_t num_chunks, size_t max_uncompressed_chunk_bytes);
int nvcomp_zstd_batched_decompress_async_v5(nvcomp_zstd_batch_manager_t *mgr, const void *const *d_compressed_ptrs,
                                            const size_t *d_compressed_sizes, const size_t *d_uncompressed_caps,
                                            size_t max_uncompressed_chunk_bytes, size_t num_chunks, void *const *d_uncompressed_ptrs,
                                            size_t *d_actual_sizes, int *d_statuses, void *d_temp_storage, size_t temp_storage_bytes,
                                            hipStream_t stream);

/* ---------------- hybrid API (reference include/cuda_zstd_hybrid.h:296-359) ---------------- */
typedef struct cuda_zstd_hybrid_engine_t cuda_zstd_hybrid_engine_t;
typedef struct {
  unsigned int mode;
  size_t cpu_size_threshold;
  size_t gpu_device_threshold;
  int compression_level;
  int enable_profiling;
  unsigned int cpu_thread_count;
} cuda_zstd_hybrid_config_t;
typedef struct {
  unsigned int backend_used;
  unsigned int input_location;
  unsigned int output_location;
  double total_time_ms;
  double transfer_time_ms;
  double compute_time_ms;
  double throughput_mbps;
  size_t input_bytes;
  size_t output_bytes;
  float compression_ratio;
} cuda_zstd_hybrid_result_t;
cuda_zstd_hybrid_engine_t *cuda_zstd_hybrid_create(const cuda_zstd_hybrid_config_t *config);
cuda_zstd_hybrid_engine_t *cuda_zstd_hybrid_create_default(void);
void cuda_zstd_hybrid_destroy(cuda_zstd_hybrid_engine_t *engine);
int cuda_zstd_hybrid_compress(cuda_zstd_hybrid_engine_t *engine, const void *input, size_t input_size, void *output,
                              size_t *output_size, unsigned int input_loc, unsigned int output_loc,
                              cuda_zstd_hybrid_result_t *result, hipStream_t stream);
int cuda_zstd_hybrid_decompress(cuda_zstd_hybrid_engine_t *engine, const void *input, size_t input_size, void *output,
                                size_t *output_size, unsigned int input_loc, unsigned int output_loc,
                                cuda_zstd_hybrid_result_t *result, hipStream_t stream);
size_t cuda_zstd_hybrid_max_compressed_size(cuda_zstd_hybrid_engine_t *engine, size_t input_size);
unsigned int cuda_zstd_hybrid_query_routing(cuda_zstd_hybrid_engine_t *engine, size_t data_size, unsigned int input_loc,
                                            unsigned int output_loc, int is_compression);

/* ---------------- streaming (reference ZstdStreamingManager, include/cuda_zstd_manager.h:300-352) ----
 * No C binding in the reference; added so the streaming path is reachable from C/ctypes.  Every
 * chunk is a complete frame; with_history = compress_chunk_with_history (the preceding <= 64 KiB
 * of the stream as raw-content history); decompress_chunk keeps the decoded window, so chunks
 * decode in stream order.  Device buffers; blocking on return. */
typedef struct cuda_zstd_stream_t cuda_zstd_stream_t;
cuda_zstd_stream_t *cuda_zstd_stream_create(int compression_level);
void cuda_zstd_stream_destroy(cuda_zstd_stream_t *s);
int cuda_zstd_stream_compress_chunk(cuda_zstd_stream_t *s, const void *src, size_t src_size, void *dst, size_t *dst_size, int with_history,
                                    int is_last_chunk, hipStream_t stream);
int cuda_zstd_stream_decompress_chunk(cuda_zstd_stream_t *s, const void *src, size_t src_size, void *dst, size_t *dst_size,
                                      int *is_last_chunk, hipStream_t stream);
int cuda_zstd_stream_reset(cuda_zstd_stream_t *s);

/* ---------------- frame metadata (skippable frames) ----------------
 * A 16-byte skippable frame [0x184D2A50][8][0x444D5A43 "CZMD"][level] in front of frames: the
 * reference's SkippableFrameHeader + CustomMetadataFrame (src/cuda_zstd_manager.cu:309-318,
 * writer :391-412).  dst: host or device.  extract: the first zstd frame's header fields after
 * any skippable frames (reference extract_metadata, src/cuda_zstd_manager.cu:992-1030); level 3
 * when no metadata frame is present.  Return nvcomp-style codes. */
int cuda_zstd_write_metadata_frame(void *dst, size_t capacity, int compression_level, size_t *written, hipStream_t stream);
int cuda_zstd_extract_metadata(const void *src, size_t size, unsigned int *compression_level, unsigned long long *uncompressed_size,
                               unsigned int *dictionary_id, int *has_checksum);

/* ---------------- library info ---------------- */
const char *cuda_zstd_hip_version(void);
/* Per-kernel timing with HIP events recorded on the launch stream (bench.py roofline).
 * collect() waits for the recorded launches and returns their count; ms3[0..2] = summed
 * milliseconds of K1 (zh_lz_kernel), the entropy stage (zh_entropy_kernel +
 * zh_fse_chain_kernel + zh_seq_pack_kernel) and the frame tail (zh_gather_kernel +
 * zh_checksum_kernel). */
void cuda_zstd_hip_profile_enable(int on);
int cuda_zstd_hip_profile_collect(double *ms3);
/* LDS bytes requested by K1 (which = 0) and the entropy kernel (1), for launch-bound checks. */
unsigned int cuda_zstd_hip_kernel_lds_bytes(int which);

#ifdef __cplusplus
}
#endif
#endif /* CUDA_ZSTD_CAPI_H_ */
