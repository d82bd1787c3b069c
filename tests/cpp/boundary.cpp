// boundary.cpp — the reference's own C++ call shapes on the drop-in boundary, driven by
// tests/test_gpu_boundary.py (-m gpu).  Built by __graft_entry__.build() (tests/cpp/Makefile)
// against libcuda_zstd_hip.so; test infrastructure only.
//
//   boundary nvcomp <dir>          NvcompV5BatchManager::compress_async with DEVICE pointer
//                                  arrays, HOST input sizes and DEVICE in/out size array, as
//                                  reference tests/test_nvcomp_batch.cu:132-134 calls it; then
//                                  decompress_async of the frames (device arrays) back
//   boundary threshold <dir> <T>   ZstdBatchManager with CompressionConfig::cpu_threshold = T:
//                                  ZstdManager::compress of every chunk (device buffers); chunks
//                                  below T take the libzstd route (reference
//                                  src/cuda_zstd_manager.cu:1604-1668), the rest the GPU
//   boundary batch_threshold <dir> <T>  ZstdBatchManager::compress_batch of every chunk as one
//                                  BatchItem vector with cpu_threshold = T: items below T take
//                                  libzstd (the reference's per-item compress() loop,
//                                  src/cuda_zstd_manager.cu:5744-5768), the rest one GPU launch
//   boundary inference <dir>       GPU compress of every chunk, then the inference flow of
//                                  reference tests/test_inference_api.cu:398-410: a workspace
//                                  from allocate_inference_workspace(frame, chunk) and
//                                  decompress_to_preallocated into an exactly-sized output
//   boundary stream_dict <dir> <h>  ZstdStreamingManager with set_dictionary(<dir>/dict.bin)
//                                  (raw content or a formatted dictionary): every chunk through
//                                  compress_chunk (h = 0) or compress_chunk_with_history (h = 1),
//                                  then every frame through decompress_chunk in order
//
// <dir>/in.bin = the chunks back to back, <dir>/sizes.bin = u64 sizes.  Writes
// <dir>/frames.bin (frames back to back), <dir>/fsizes.bin (u64), and for `nvcomp`
// <dir>/back.bin (decoded chunks back to back).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "cuda_zstd_manager.h"
#include "cuda_zstd_nvcomp.h"

using namespace cuda_zstd;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 2;                                                                \
    }                                                                          \
  } while (0)

static std::vector<char> slurp(const std::string &p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<char>(std::istreambuf_iterator<char>(f), {});
}
static void dump(const std::string &p, const void *d, size_t n) {
  std::ofstream f(p, std::ios::binary);
  f.write((const char *)d, (std::streamsize)n);
}

int main(int argc, char **argv) {
  if (argc < 3) return 1;
  std::string const mode = argv[1], dir = argv[2];
  std::vector<char> in = slurp(dir + "/in.bin"), szb = slurp(dir + "/sizes.bin");
  size_t const n = szb.size() / 8;
  std::vector<size_t> sizes(n);
  memcpy(sizes.data(), szb.data(), n * 8);
  std::vector<size_t> offs(n + 1, 0);
  for (size_t i = 0; i < n; i++) offs[i + 1] = offs[i] + sizes[i];
  if (offs[n] != in.size()) return 1;

  // device chunks (one allocation each, as the reference test does)
  std::vector<void *> d_in(n), d_out(n);
  size_t const cap = estimate_compressed_size(*std::max_element(sizes.begin(), sizes.end()), 3);
  for (size_t i = 0; i < n; i++) {
    CK(hipMalloc(&d_in[i], std::max<size_t>(sizes[i], 1)));
    CK(hipMemcpy(d_in[i], in.data() + offs[i], sizes[i], hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out[i], cap));
  }
  std::vector<size_t> fsz(n, 0);
  std::vector<char> frames;

  if (mode == "nvcomp") {
    nvcomp_v5::NvcompV5Options opts;
    opts.level = 3;
    nvcomp_v5::NvcompV5BatchManager bm(opts);
    void **d_in_ptrs, **d_out_ptrs;
    size_t *d_out_sizes;
    CK(hipMalloc(&d_in_ptrs, n * sizeof(void *)));
    CK(hipMalloc(&d_out_ptrs, n * sizeof(void *)));
    CK(hipMalloc(&d_out_sizes, n * sizeof(size_t)));
    CK(hipMemcpy(d_in_ptrs, d_in.data(), n * sizeof(void *), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_out_ptrs, d_out.data(), n * sizeof(void *), hipMemcpyHostToDevice));
    std::vector<size_t> caps(n, cap);
    CK(hipMemcpy(d_out_sizes, caps.data(), n * sizeof(size_t), hipMemcpyHostToDevice));
    size_t const temp_size = bm.get_compress_temp_size(sizes.data(), n);
    void *d_temp;
    CK(hipMalloc(&d_temp, temp_size));
    Status st = bm.compress_async((const void *const *)d_in_ptrs, sizes.data(), n, d_out_ptrs, d_out_sizes, d_temp, temp_size);
    CK(hipDeviceSynchronize());
    if (st != Status::SUCCESS) {
      fprintf(stderr, "compress_async: %s\n", status_to_string(st));
      return 3;
    }
    CK(hipMemcpy(fsz.data(), d_out_sizes, n * 8, hipMemcpyDeviceToHost));
    // decompress_async: device arrays of frames and outputs, device size array (capacity in)
    std::vector<void *> d_back(n);
    for (size_t i = 0; i < n; i++) CK(hipMalloc(&d_back[i], std::max<size_t>(sizes[i], 1)));
    void **d_back_ptrs;
    size_t *d_fsz, *d_back_sizes;
    CK(hipMalloc(&d_back_ptrs, n * sizeof(void *)));
    CK(hipMalloc(&d_fsz, n * 8));
    CK(hipMalloc(&d_back_sizes, n * 8));
    CK(hipMemcpy(d_back_ptrs, d_back.data(), n * sizeof(void *), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_fsz, fsz.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_back_sizes, sizes.data(), n * 8, hipMemcpyHostToDevice));
    size_t const dts = bm.get_decompress_temp_size(fsz.data(), n);
    void *d_dtemp;
    CK(hipMalloc(&d_dtemp, dts));
    st = bm.decompress_async((const void *const *)d_out_ptrs, d_fsz, n, d_back_ptrs, d_back_sizes, d_dtemp, dts);
    CK(hipDeviceSynchronize());
    if (st != Status::SUCCESS) {
      fprintf(stderr, "decompress_async: %s\n", status_to_string(st));
      return 4;
    }
    std::vector<size_t> bsz(n);
    CK(hipMemcpy(bsz.data(), d_back_sizes, n * 8, hipMemcpyDeviceToHost));
    std::vector<char> back(in.size());
    for (size_t i = 0; i < n; i++) {
      if (bsz[i] != sizes[i]) { fprintf(stderr, "chunk %zu: decoded %zu of %zu bytes\n", i, bsz[i], sizes[i]); return 5; }
      CK(hipMemcpy(back.data() + offs[i], d_back[i], sizes[i], hipMemcpyDeviceToHost));
    }
    dump(dir + "/back.bin", back.data(), back.size());
  } else if (mode == "threshold") {
    if (argc < 4) return 1;
    CompressionConfig c = CompressionConfig::from_level(3);
    c.cpu_threshold = (u32)std::stoul(argv[3]);
    ZstdBatchManager m(c);
    size_t const ts = m.get_compress_temp_size(*std::max_element(sizes.begin(), sizes.end()));
    void *d_temp;
    CK(hipMalloc(&d_temp, ts));
    for (size_t i = 0; i < n; i++) {
      fsz[i] = cap;
      Status st = m.compress(d_in[i], sizes[i], d_out[i], &fsz[i], d_temp, ts, nullptr, 0, 0);
      if (st != Status::SUCCESS) {
        fprintf(stderr, "compress %zu: %s\n", i, status_to_string(st));
        return 3;
      }
    }
  } else if (mode == "batch_threshold") {
    if (argc < 4) return 1;
    CompressionConfig c = CompressionConfig::from_level(3);
    c.cpu_threshold = (u32)std::stoul(argv[3]);
    ZstdBatchManager m(c);
    std::vector<BatchItem> items(n);
    for (size_t i = 0; i < n; i++) {
      items[i].input_ptr = d_in[i];
      items[i].input_size = sizes[i];
      items[i].output_ptr = d_out[i];
      items[i].output_size = cap;
    }
    size_t const ts = m.get_batch_compress_temp_size(sizes);
    void *d_temp;
    CK(hipMalloc(&d_temp, ts));
    Status st = m.compress_batch(items, d_temp, ts, 0);
    if (st != Status::SUCCESS) {
      fprintf(stderr, "compress_batch: %s\n", status_to_string(st));
      return 3;
    }
    for (size_t i = 0; i < n; i++) fsz[i] = items[i].output_size;
  } else if (mode == "inference") {
    ZstdBatchManager m(CompressionConfig::from_level(3));
    size_t const ts = m.get_compress_temp_size(*std::max_element(sizes.begin(), sizes.end()));
    void *d_temp;
    CK(hipMalloc(&d_temp, ts));
    std::vector<char> back(in.size());
    for (size_t i = 0; i < n; i++) {
      fsz[i] = cap;
      Status st = m.compress(d_in[i], sizes[i], d_out[i], &fsz[i], d_temp, ts, nullptr, 0, 0);
      if (st != Status::SUCCESS) { fprintf(stderr, "compress %zu: %s\n", i, status_to_string(st)); return 3; }
      void *ws = nullptr;
      size_t ws_size = 0;
      st = m.allocate_inference_workspace(fsz[i], sizes[i], &ws, &ws_size);
      if (st != Status::SUCCESS) { fprintf(stderr, "allocate_inference_workspace: %s\n", status_to_string(st)); return 3; }
      void *d_o;
      CK(hipMalloc(&d_o, sizes[i]));
      size_t actual = 0;
      st = m.decompress_to_preallocated(d_out[i], fsz[i], d_o, sizes[i], &actual, ws, ws_size, 0);
      if (st != Status::SUCCESS || actual != sizes[i]) {
        fprintf(stderr, "decompress_to_preallocated %zu (ws %zu B): %s, %zu B\n", i, ws_size, status_to_string(st), actual);
        return 4;
      }
      CK(hipMemcpy(back.data() + offs[i], d_o, sizes[i], hipMemcpyDeviceToHost));
      (void)m.free_inference_workspace(ws);
      CK(hipFree(d_o));
    }
    dump(dir + "/back.bin", back.data(), back.size());
  } else if (mode == "stream_dict") {
    if (argc < 4) return 1;
    bool const hist = std::stoul(argv[3]) != 0;
    std::vector<char> db = slurp(dir + "/dict.bin");
    dictionary::Dictionary dct;
    dct.raw_content.assign(db.begin(), db.end());
    ZstdStreamingManager sm(CompressionConfig::from_level(3));
    Status st = sm.set_dictionary(dct);
    if (st == Status::SUCCESS) st = hist ? sm.init_compression_with_history(0, 0) : sm.init_compression(0, 0);
    if (st != Status::SUCCESS) { fprintf(stderr, "init: %s\n", status_to_string(st)); return 3; }
    for (size_t i = 0; i < n; i++) {
      fsz[i] = cap;
      st = hist ? sm.compress_chunk_with_history(d_in[i], sizes[i], d_out[i], &fsz[i], i + 1 == n, 0)
                : sm.compress_chunk(d_in[i], sizes[i], d_out[i], &fsz[i], i + 1 == n, 0);
      if (st != Status::SUCCESS) { fprintf(stderr, "compress_chunk %zu: %s\n", i, status_to_string(st)); return 3; }
    }
    std::vector<char> back(in.size());
    void *d_o;
    CK(hipMalloc(&d_o, std::max<size_t>(*std::max_element(sizes.begin(), sizes.end()), 1)));
    for (size_t i = 0; i < n; i++) {
      size_t got = sizes[i];
      bool last = false;
      st = sm.decompress_chunk(d_out[i], fsz[i], d_o, &got, &last, 0);
      if (st != Status::SUCCESS || got != sizes[i]) { fprintf(stderr, "decompress_chunk %zu: %s, %zu B\n", i, status_to_string(st), got); return 4; }
      CK(hipMemcpy(back.data() + offs[i], d_o, sizes[i], hipMemcpyDeviceToHost));
    }
    dump(dir + "/back.bin", back.data(), back.size());
  } else {
    return 1;
  }
  for (size_t i = 0; i < n; i++) {
    size_t const o = frames.size();
    frames.resize(o + fsz[i]);
    CK(hipMemcpy(frames.data() + o, d_out[i], fsz[i], hipMemcpyDeviceToHost));
  }
  dump(dir + "/frames.bin", frames.data(), frames.size());
  dump(dir + "/fsizes.bin", fsz.data(), n * 8);
  printf("ok %zu\n", n);
  return 0;
}
