// cuda_zstd_dictionary.h — dictionary types and training API of the gfx950 Zstandard compressor.
//
// Drop-in counterpart of the reference's include/cuda_zstd_dictionary.h (same names, fields and
// semantics, so a reference caller compiles unchanged):
//   DICT_MAGIC_NUMBER / MIN_DICT_SIZE / MAX_DICT_SIZE          :28-30
//   DictionaryTrainingParams, CoverParams                       :36-50
//   DictionaryHeader, DictionaryContent                         :56-71
//   Dictionary {header, raw_content, raw_size}                  :72-159 (deep-copying copy
//                                                               operations, no-op destructor)
//   train_dictionary / create_dictionary_from_samples           :176-196
//   get_optimal_dict_size / is_valid_dictionary_size            :198-210
//   compat::DictionaryTrainerWrapper / DictionaryManagerWrapper  :216-310, and their aliases
//
// What differs (documented, not an ABI change): training is COVER (Liao et al., libzstd's
// ZDICT_trainFromBuffer_cover algorithm, csrc/zh_dict.cpp) producing raw content, where the
// reference fills the buffer with a byte-frequency / 4-gram heuristic
// (src/cuda_zstd_dictionary.cu:179-415); a manager copies the bytes at set_dictionary (the
// reference keeps the caller's pointer, src/cuda_zstd_manager.cu:3743-3745), and frames name the
// dictionary by its RFC 8878 Dictionary_ID (a formatted dictionary's, none for raw content), not
// by header.dictionary_id.
#ifndef CUDA_ZSTD_DICTIONARY_H_
#define CUDA_ZSTD_DICTIONARY_H_

#include "cuda_zstd_types.h"

#ifdef __cplusplus
#include <cstdlib>
#include <cstring>
#include <vector>

namespace cuda_zstd {
namespace dictionary {

constexpr u32 DICT_MAGIC_NUMBER = 0xEC30A437;  // RFC 8878 §5 dictionary magic
constexpr u32 MIN_DICT_SIZE = 256;
constexpr u32 MAX_DICT_SIZE = 128 * 1024;

struct DictionaryTrainingParams {
  u32 optimization_level = 0;  // accepted for source compatibility; COVER's own parameters apply
  bool use_gpu = true;
  u32 max_threads = 256;
  u32 reserved[5] = {0};
};

// legacy parameters of the compat trainer (reference :44-50)
struct CoverParams {
  u32 k = 0;
  u32 d = 0;
  u32 steps = 0;
  u32 splitPoint = 0;
  double accel = 0.0;
};

struct DictionaryHeader {
  u32 magic_number;
  u32 dictionary_id;
  u32 entropy_tables_size;
  u32 offsets_size;
  u32 match_lengths_size;
  u32 literal_lengths_size;
  u32 huffman_table_size;
  u32 raw_content_size;
};

struct DictionaryContent {
  unsigned char *d_buffer;
  u32 size;
  u32 dict_id;
};

// The reference's ownership rules: the destructor never frees raw_content (it may be the caller's
// memory); a copy (constructor or assignment) owns a malloc'd host copy of the bytes that its
// holder releases with free().  set_dictionary reads raw_content (host or device memory) once and
// keeps its own copy; get_dictionary hands back such a malloc'd copy.
struct Dictionary {
  DictionaryHeader header;
  unsigned char *raw_content;
  u32 raw_size;

  Dictionary() : header{DICT_MAGIC_NUMBER, 0, 0, 0, 0, 0, 0, 0}, raw_content(nullptr), raw_size(0) {}
  ~Dictionary() = default;
  Dictionary(const Dictionary &o) : header(o.header), raw_content(nullptr), raw_size(o.raw_size) { take_copy(o); }
  Dictionary &operator=(const Dictionary &o) {
    if (this == &o) return *this;
    std::free(raw_content);
    raw_content = nullptr;
    header = o.header;
    raw_size = o.raw_size;
    take_copy(o);
    return *this;
  }

 private:
  void take_copy(const Dictionary &o) {
    if (!o.raw_content || !raw_size) return;
    raw_content = static_cast<unsigned char *>(std::malloc(raw_size));
    if (raw_content) std::memcpy(raw_content, o.raw_content, raw_size);
  }
};

// COVER training over host samples into dict_buffer (dict_size bytes, MIN..MAX_DICT_SIZE); the
// trained content fills the buffer from its end (ZDICT's layout: the most useful segments last)
// and any unused head is zero.
Status train_dictionary(const std::vector<const void *> &samples, const std::vector<size_t> &sample_sizes, void *dict_buffer,
                        size_t dict_size, const DictionaryTrainingParams *params = nullptr, hipStream_t stream = 0);
// samples as one buffer with start offsets; sample i ends where i + 1 starts, the last one after
// 8 KiB (reference src/cuda_zstd_dictionary.cu:475-503): the caller's buffer must hold at least
// sample_offsets[num_samples - 1] + 8192 bytes, whatever the last sample's real length
Status create_dictionary_from_samples(const void *samples_buffer, const size_t *sample_offsets, size_t num_samples, void *dict_buffer,
                                      size_t dict_size, const DictionaryTrainingParams *params = nullptr, hipStream_t stream = 0);
// ~1 % of the data, clamped to [MIN_DICT_SIZE, MAX_DICT_SIZE], rounded up to a KiB
u32 get_optimal_dict_size(size_t total_data_size);
bool is_valid_dictionary_size(size_t size);

namespace compat {

// DictionaryTrainer::train_dictionary(samples, sizes, dict_out, size): dict_out.raw_content is a
// new malloc'd buffer (free() it), header.dictionary_id the reference's 31-multiplier hash of the
// first 256 bytes.
class DictionaryTrainerWrapper {
 public:
  static Status train_dictionary(const std::vector<const void *> &samples, const std::vector<size_t> &sample_sizes, Dictionary &dict_out,
                                 size_t dict_size, const CoverParams *params = nullptr, hipStream_t stream = 0) {
    unsigned char *buf = static_cast<unsigned char *>(std::malloc(dict_size ? dict_size : 1));
    if (!buf) return Status::ERROR_OUT_OF_MEMORY;
    DictionaryTrainingParams tp;
    if (params) tp.optimization_level = params->k;
    Status const s = ::cuda_zstd::dictionary::train_dictionary(samples, sample_sizes, buf, dict_size, &tp, stream);
    if (s != Status::SUCCESS) {
      std::free(buf);
      return s;
    }
    dict_out.raw_content = buf;
    dict_out.raw_size = (u32)dict_size;
    dict_out.header.dictionary_id = id_hash(buf, dict_size);
    return s;
  }
  static u32 id_hash(const unsigned char *p, size_t n) {
    u32 h = 0;
    for (size_t i = 0; i < n && i < 256; i++) h = h * 31u + p[i];
    return h;
  }
};

// DictionaryManager: host-side allocation helpers of the reference's tests (the "gpu" in the names
// is the reference's; it allocates with malloc as well).
class DictionaryManagerWrapper {
 public:
  static Status allocate_dictionary_gpu(Dictionary &dict, size_t size, hipStream_t stream = 0) {
    (void)stream;
    dict.raw_content = static_cast<unsigned char *>(std::malloc(size ? size : 1));
    if (!dict.raw_content) return Status::ERROR_OUT_OF_MEMORY;
    dict.raw_size = (u32)size;
    return Status::SUCCESS;
  }
  static Status free_dictionary_gpu(Dictionary &dict, hipStream_t stream = 0) {
    (void)stream;
    std::free(dict.raw_content);
    dict.raw_content = nullptr;
    dict.raw_size = 0;
    dict.header.dictionary_id = 0;
    return Status::SUCCESS;
  }
  static Status load_dictionary(const void *dict_buffer, size_t dict_size, Dictionary &dict_out) {
    unsigned char *buf = static_cast<unsigned char *>(std::malloc(dict_size ? dict_size : 1));
    if (!buf) return Status::ERROR_OUT_OF_MEMORY;
    if (dict_size) std::memcpy(buf, dict_buffer, dict_size);
    dict_out.raw_content = buf;
    dict_out.raw_size = (u32)dict_size;
    dict_out.header.dictionary_id = DictionaryTrainerWrapper::id_hash(buf, dict_size);
    return Status::SUCCESS;
  }
};

}  // namespace compat

using DictionaryTrainer = compat::DictionaryTrainerWrapper;
using DictionaryManager = compat::DictionaryManagerWrapper;

}  // namespace dictionary
}  // namespace cuda_zstd
#endif  // __cplusplus

#endif  // CUDA_ZSTD_DICTIONARY_H_
