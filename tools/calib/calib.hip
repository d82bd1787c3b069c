// tools/calib/calib.hip — FETCH_SIZE / WRITE_SIZE calibration for the access widths the entropy
// kernels use (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").  Each kernel streams 1 GiB (past the 256 MiB
// Infinity Cache) with one access width, coalesced across lanes; run under rocprofv3 --pmc.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ void rd(const T *__restrict__ p, size_t n, unsigned *out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v = p[i];
    acc ^= *(const unsigned *)&v;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads
}
template <typename T>
__global__ void wr(T *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (T)i;
}
struct u128 { unsigned a, b, c, d; __device__ u128() {} __device__ u128(size_t i) : a((unsigned)i), b(1), c(2), d(3) {} };

int main() {
  size_t const B = 1ull << 30;
  void *buf = nullptr;
  unsigned *out = nullptr;
  if (hipMalloc(&buf, B) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, B);
  dim3 g(4096), t(256);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(rd<uint8_t>, g, t, 0, 0, (const uint8_t *)buf, B, out);
    hipLaunchKernelGGL(rd<uint32_t>, g, t, 0, 0, (const uint32_t *)buf, B / 4, out);
    hipLaunchKernelGGL(rd<uint64_t>, g, t, 0, 0, (const uint64_t *)buf, B / 8, out);
    hipLaunchKernelGGL(rd<uint4>, g, t, 0, 0, (const uint4 *)buf, B / 16, out);
    hipLaunchKernelGGL(wr<uint8_t>, g, t, 0, 0, (uint8_t *)buf, B);
    hipLaunchKernelGGL(wr<uint32_t>, g, t, 0, 0, (uint32_t *)buf, B / 4);
    hipLaunchKernelGGL(wr<uint64_t>, g, t, 0, 0, (uint64_t *)buf, B / 8);
    hipLaunchKernelGGL(wr<u128>, g, t, 0, 0, (u128 *)buf, B / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("calib done: each kernel moves %zu bytes\n", B);
  return 0;
}
