// zh_pipe.h — side streams + events for the staggered group pipelines (host code).
//
// The entropy stage (zh_entropy.hip) and the decoder (zh_decode.hip) split large batches into
// G groups of consecutive blocks/items on G streams: group k's first, throughput-bound kernel
// starts once group k-1's first kernel is done, so the latency-bound kernels after it (one
// wave per few blocks) overlap the next groups' first kernel.  One set per device and per
// pipeline (Tag), created on the device of the caller's stream at its first large call and
// kept; a call holds the set's mutex while it enqueues its groups.
#ifndef ZH_PIPE_H_
#define ZH_PIPE_H_

#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>

namespace zh {

template <unsigned G>
struct StreamPipe {
  std::mutex mu;
  hipStream_t side[G - 1] = {};
  hipEvent_t start = nullptr, first_done[G - 1] = {}, done[G - 1] = {};
  bool ok = true;
  explicit StreamPipe(int dev) {
    int cur = -1;
    ok = hipGetDevice(&cur) == hipSuccess && hipSetDevice(dev) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&start, hipEventDisableTiming) == hipSuccess;
    for (unsigned k = 0; k + 1 < G; k++) {
      ok = ok && hipStreamCreateWithFlags(&side[k], hipStreamNonBlocking) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&first_done[k], hipEventDisableTiming) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&done[k], hipEventDisableTiming) == hipSuccess;
    }
    if (cur >= 0) (void)hipSetDevice(cur);
  }

  // Enqueue group(k, s, after_first) for k = 0..G-1: group 0 on the caller's stream, the others
  // on side streams ordered after everything already on it; group(...) records after_first
  // (when non-null) once its first kernel is queued.  The caller's stream then waits for all.
  template <class F>
  void run(hipStream_t stream, F &&group) {
    std::lock_guard<std::mutex> lk(mu);
    (void)hipEventRecord(start, stream);
    for (unsigned k = 0; k < G; k++) {
      hipStream_t const s = k ? side[k - 1] : stream;
      if (k) {
        (void)hipStreamWaitEvent(s, start, 0);
        (void)hipStreamWaitEvent(s, first_done[k - 1], 0);
      }
      group(k, s, k + 1 < G ? first_done[k] : nullptr);
      if (k) (void)hipEventRecord(done[k - 1], s);
    }
    for (unsigned k = 1; k < G; k++) (void)hipStreamWaitEvent(stream, done[k - 1], 0);
  }
};

// The device a stream belongs to (the null stream: the current device)
inline int stream_device(hipStream_t s) {
  int dev = -1;
  if (s && hipStreamGetDevice(s, &dev) == hipSuccess) return dev;
  (void)hipGetLastError();
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return dev;
}

// The pipe of (Tag, device of s); null if its streams could not be created
template <class Tag, unsigned G>
StreamPipe<G> *stream_pipe(hipStream_t s) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<StreamPipe<G>>> pipes;
  int const dev = stream_device(s);
  std::lock_guard<std::mutex> lk(mu);
  auto &p = pipes[dev];
  if (!p) p.reset(new StreamPipe<G>(dev));
  return p->ok ? p.get() : nullptr;
}

}  // namespace zh
#endif  // ZH_PIPE_H_
