// cuda_zstd_hybrid.h — CPU/GPU routing engine (reference include/cuda_zstd_hybrid.h:73-240).
//
// Routing here is explicit: FORCE_CPU runs host libzstd (the reference's
// cpu_compress, src/cuda_zstd_hybrid.cu:402-458); FORCE_GPU / PREFER_GPU run the
// gfx950 kernels; AUTO / PREFER_CPU / ADAPTIVE follow the reference's simple
// size/location rules (decide_route, :196-328) without its profiling heuristics.
// The C ABI (:292-363) lives in cuda_zstd_capi.h.
#ifndef CUDA_ZSTD_HYBRID_H_
#define CUDA_ZSTD_HYBRID_H_

#include "cuda_zstd_manager.h"

#ifdef __cplusplus
namespace cuda_zstd {

class HybridEngine {
 public:
  HybridEngine();
  explicit HybridEngine(const HybridConfig &config);
  ~HybridEngine();
  HybridEngine(const HybridEngine &) = delete;
  HybridEngine &operator=(const HybridEngine &) = delete;
  HybridEngine(HybridEngine &&) noexcept;             // reference :82-83
  HybridEngine &operator=(HybridEngine &&) noexcept;

  Status configure(const HybridConfig &config);
  HybridConfig get_config() const;
  Status set_compression_level(int level);

  Status compress(const void *input, size_t input_size, void *output, size_t *output_size, DataLocation input_loc = DataLocation::HOST,
                  DataLocation output_loc = DataLocation::HOST, HybridResult *result = nullptr, hipStream_t stream = 0);
  Status decompress(const void *input, size_t input_size, void *output, size_t *output_size, DataLocation input_loc = DataLocation::HOST,
                    DataLocation output_loc = DataLocation::HOST, HybridResult *result = nullptr, hipStream_t stream = 0);
  Status compress_batch(const void *const *inputs, const size_t *input_sizes, void **outputs, size_t *output_sizes, size_t count,
                        DataLocation input_loc = DataLocation::HOST, DataLocation output_loc = DataLocation::HOST,
                        BatchRoutingResult *results = nullptr, hipStream_t stream = 0);
  // reference :180-186: each item routed like decompress(); output_sizes in = capacity, out = bytes
  Status decompress_batch(const void *const *inputs, const size_t *input_sizes, void **outputs, size_t *output_sizes, size_t count,
                          DataLocation input_loc = DataLocation::HOST, DataLocation output_loc = DataLocation::HOST,
                          BatchRoutingResult *results = nullptr, hipStream_t stream = 0);

  size_t get_max_compressed_size(size_t input_size) const;
  ExecutionBackend query_routing(size_t data_size, DataLocation input_loc, DataLocation output_loc, bool is_compression) const;
  CompressionStats get_stats() const;
  void reset_stats();
  static DataLocation detect_location(const void *ptr);

  // reference :229-235 (src/cuda_zstd_hybrid.cu:46-136, 1029-1038): the mean of the last 64
  // MB/s samples of a backend (CPU_* share one history, GPU_* the other), recorded by
  // compress/decompress when HybridConfig::enable_profiling is set; ADAPTIVE routing picks the
  // GPU once both have samples and it is > 1.2x the CPU's. 0 = no samples.
  double get_observed_throughput(ExecutionBackend backend, bool is_compression) const;
  void reset_profiling();

 private:
  class Impl;
  std::unique_ptr<Impl> pimpl_;
};

Status hybrid_compress(const void *input, size_t input_size, void *output, size_t *output_size, DataLocation input_loc = DataLocation::HOST,
                       DataLocation output_loc = DataLocation::HOST, int compression_level = 3, HybridResult *result = nullptr,
                       hipStream_t stream = 0);
// reference :263-268: a temporary engine with the default configuration
Status hybrid_decompress(const void *input, size_t input_size, void *output, size_t *output_size, DataLocation input_loc = DataLocation::HOST,
                         DataLocation output_loc = DataLocation::HOST, HybridResult *result = nullptr, hipStream_t stream = 0);
std::unique_ptr<HybridEngine> create_hybrid_engine(const HybridConfig &config = HybridConfig{});
std::unique_ptr<HybridEngine> create_hybrid_engine(int compression_level);

}  // namespace cuda_zstd
#endif  // __cplusplus
#endif  // CUDA_ZSTD_HYBRID_H_
