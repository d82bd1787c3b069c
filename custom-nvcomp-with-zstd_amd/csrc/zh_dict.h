// zh_dict.h — host side of dictionaries (zh_dict.cpp; SURVEY.md §8f F2, RFC 8878 §5).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <utility>
#include <vector>

namespace zh {
constexpr uint32_t kDictMagic = 0xEC30A437u;
constexpr size_t kDictMaxBytes = 128 * 1024;  // reference dictionary::MAX_DICT_SIZE (include/cuda_zstd_dictionary.h:30)

// Raw content (no dictionary magic): id 0, content at 0.  Formatted: its Dictionary_ID and the
// offset of its content.  false when a formatted dictionary is malformed.
bool dict_layout(const uint8_t *d, size_t n, uint32_t &id, size_t &content_off);

// COVER training over host samples -> raw-content dictionary of at most dict_size bytes
// (segments of k bytes scored by their d-byte d-mers); empty when the samples are too small.
std::vector<uint8_t> cover_train(const std::vector<std::pair<const uint8_t *, size_t>> &samples, size_t dict_size, uint32_t k = 1024,
                                 uint32_t d = 8);
}  // namespace zh
