// zh_plan.hip — batch planning, multi-block frame gather, and launch wrappers.
//
// zh_plan_kernel : builds one ZhBlockDesc per (item, 64 KiB sub-block) from device
//                  pointer/size arrays, for the stream-ordered batched entry point
//                  (no host round trip, unlike the reference's compress_async,
//                  src/cuda_zstd_nvcomp.cpp:319-437).
// zh_gather_kernel: concatenates the staged blocks of multi-block frames (the
//                  reference assembles them on the host with blocking copies,
//                  src/cuda_zstd_manager.cu:2765-3027).
#include "zh_common.h"
#include "zh_launch.h"
#include "zh_xxh64.h"

#include <mutex>
#include <vector>

extern "C" u32 zh_lz_lds_bytes();
extern "C" u32 zh_entropy_lds_bytes();
namespace zh {
hipError_t lz_init();
void lz_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 mode, hipStream_t stream);
hipError_t lz_deep_init();
hipError_t lz_deep_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, int level, hipStream_t stream);
hipError_t entropy_init();
void entropy_launch(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 window_log, u32 cfg_block_size, u64 *d_item_size,
                    u32 *d_item_status, u32 *d_blk_size, hipStream_t stream);
}  // namespace zh

extern "C" __global__ void zh_plan_kernel(const void *const *__restrict__ in_ptrs, const size_t *__restrict__ in_sizes, u32 nitems,
                                          u32 bpi, void *const *__restrict__ out_ptrs, u64 out_cap, u8 *staging, ZhBlockDesc *descs,
                                          ZhItemDesc *items, u64 *item_size, u32 *item_status, u32 extra_flags,
                                          const u8 *dict, u32 dict_n, u32 dict_id, u32 hist) {
  u32 const b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nitems * bpi) return;
  u32 const it = b / bpi, k = b % bpi;
  u64 const size = in_sizes[it];
  u64 const bs = ZH_FRAME_BLOCK(size, dict != nullptr && !(extra_flags & ZH_F_DEEP));
  u64 const nb = (size + bs - 1) / bs;
  ZhBlockDesc d;
  d.src = (const u8 *)in_ptrs[it] + (u64)k * bs;
  d.frame_size = size;
  d.item = it;
  d.n = (k < nb) ? (u32)min(bs, size - (u64)k * bs) : 0u;
  d.flags = (k == 0 ? ZH_F_FIRST : 0u) | (k + 1 == nb ? ZH_F_LAST : 0u) | (nb == 1 ? ZH_F_DIRECT : 0u) | extra_flags;
  d.pre = nullptr;
  d.pre_n = 0;
  d.dict_id = 0;
  if (k > 0 && hist) {  // history frame: the previous 32 KiB block is staged in front
    d.pre = d.src - ZH_HIST_BLOCK;
    d.pre_n = ZH_HIST_BLOCK;
  }
  if (dict) {  // dictionary frame: the first block is compressed behind the content's tail
    d.flags |= ZH_F_DICT;
    d.dict_id = dict_id;
    if (k == 0) {
      d.pre_n = (extra_flags & ZH_F_DEEP) ? min(dict_n, (u32)ZH_DEEP_PRE) : min(dict_n, (u32)ZH_BLOCK_MAX - d.n);
      d.pre = dict + dict_n - d.pre_n;
    }
  }
  if (nb == 1) {
    d.dst = (u8 *)out_ptrs[it];
    d.dst_cap = (u32)min(out_cap, (u64)0xFFFFFFFFu);
  } else {
    d.dst = staging + (size_t)b * ZH_STAGE_SLOT;
    d.dst_cap = ZH_STAGE_SLOT;
  }
  descs[b] = d;
  if (k == 0) {
    ZhItemDesc id;
    id.dst = (u8 *)out_ptrs[it];
    id.cap = out_cap;
    id.first_block = b;
    id.nblocks = (u32)nb;
    items[it] = id;
    if (size == 0) { item_size[it] = 0; item_status[it] = ZH_ST_INVALID; }
  }
}

// One workgroup per block: a block of a multi-block frame sums the staged sizes of its
// frame's blocks (its output offset and the frame's total), the frame's first block sets the
// item's size and status, and every block copies its own staged bytes (a 64 MiB frame is
// 1024 workgroups, not one).
extern "C" __global__ __launch_bounds__(256) void zh_gather_kernel(const ZhItemDesc *__restrict__ items, const ZhBlockDesc *__restrict__ descs,
                                                                    const u32 *__restrict__ blk_size, u64 *item_size, u32 *item_status) {
  u32 const b = blockIdx.x, tid = threadIdx.x;
  ZhBlockDesc const d = descs[b];
  if (d.n == 0) return;
  ZhItemDesc const id = items[d.item];
  if (id.nblocks <= 1) return;
  u32 const k = b - id.first_block;
  __shared__ u64 part[2][4];
  __shared__ u32 badp[4];
  u64 pre = 0, tot = 0;
  u32 bad = 0;
  for (u32 j = tid; j < id.nblocks; j += 256) {
    u32 const s = blk_size[id.first_block + j];
    bad |= s == 0xFFFFFFFFu;
    u64 const v = s == 0xFFFFFFFFu ? 0u : s;
    tot += v;
    pre += j < k ? v : 0u;
  }
  for (u32 o = 32; o; o >>= 1) {
    pre += __shfl_down(pre, o, 64);
    tot += __shfl_down(tot, o, 64);
    bad |= __shfl_down(bad, o, 64);
  }
  if ((tid & 63) == 0) { part[0][tid >> 6] = pre; part[1][tid >> 6] = tot; badp[tid >> 6] = bad; }
  __syncthreads();
  pre = part[0][0] + part[0][1] + part[0][2] + part[0][3];
  tot = part[1][0] + part[1][1] + part[1][2] + part[1][3];
  bad = badp[0] | badp[1] | badp[2] | badp[3];
  bool const fail = bad || tot > id.cap;
  if (k == 0 && tid == 0) {
    item_size[d.item] = tot;
    item_status[d.item] = fail ? ZH_ST_TOO_SMALL : ZH_ST_OK;
  }
  if (fail) return;
  u32 const s = blk_size[b];
  const u8 *src = d.dst;
  u8 *dst = id.dst + pre;
  for (u32 i = tid; i < s; i += 256) dst[i] = src[i];
}

// Content checksum (reference src/cuda_zstd_manager.cu:3037-3056): one wave per
// finished frame appends the low 32 bits of XXH64 of the item's input (the first block
// already set the FHD checksum flag).
extern "C" __global__ __launch_bounds__(64) void zh_checksum_kernel(const ZhItemDesc *__restrict__ items, const ZhBlockDesc *__restrict__ descs,
                                                                   u64 *item_size, u32 *item_status) {
  u32 const it = blockIdx.x, lane = threadIdx.x;
  if (item_status[it] != ZH_ST_OK) return;
  ZhItemDesc const id = items[it];
  ZhBlockDesc const d = descs[id.first_block];
  __shared__ u64 xb[512];
  u64 const h = zh_xxh64_wave(d.src, d.frame_size, xb);
  u64 const size = item_size[it];
  __syncthreads();
  if (size + 4 > id.cap) {
    if (lane == 0) item_status[it] = ZH_ST_TOO_SMALL;
    return;
  }
  if (lane < 4) id.dst[size + lane] = (u8)(h >> (8 * lane));
  if (lane == 0) item_size[it] = size + 4;
}

namespace zh {

hipError_t init_kernels() {
  hipError_t e = lz_init();
  if (e != hipSuccess) return e;
  e = lz_deep_init();
  if (e != hipSuccess) return e;
  return entropy_init();
}

u32 lz_lds_bytes() { return zh_lz_lds_bytes(); }
u32 entropy_lds_bytes() { return zh_entropy_lds_bytes(); }

// ---- optional per-kernel event timing (bench.py roofline): events recorded on the launch stream
namespace {
struct ProfState {
  std::mutex mu;
  bool on = false;
  std::vector<hipEvent_t> pool;           // free events
  std::vector<std::vector<hipEvent_t>> pending;  // per launch: e0 (pre-K1), e1 (K1 done), e2 (K2 done), e3 (K3 done)
};
ProfState &prof() {
  static ProfState p;
  return p;
}
hipEvent_t prof_event() {
  ProfState &p = prof();
  if (!p.pool.empty()) { hipEvent_t e = p.pool.back(); p.pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
}  // namespace

void profile_enable(bool on) {
  std::lock_guard<std::mutex> g(prof().mu);
  prof().on = on;
}

// totals[0..2] = summed ms of K1, K2, K3 over the recorded launches; returns launch count
int profile_collect(double *totals) {
  ProfState &p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  totals[0] = totals[1] = totals[2] = 0;
  int n = 0;
  for (auto &ev : p.pending) {
    (void)hipEventSynchronize(ev[3]);
    float a = 0, b = 0, c = 0;
    (void)hipEventElapsedTime(&a, ev[0], ev[1]);
    (void)hipEventElapsedTime(&b, ev[1], ev[2]);
    (void)hipEventElapsedTime(&c, ev[2], ev[3]);
    totals[0] += a; totals[1] += b; totals[2] += c;
    for (auto e : ev) p.pool.push_back(e);
    n++;
  }
  p.pending.clear();
  return n;
}

hipError_t launch_compress(const ZhBlockDesc *d_descs, u32 nblocks, ZhWorkspace ws, u32 window_log, u32 cfg_block_size, u64 *d_item_size,
                           u32 *d_item_status, u32 *d_blk_size, const ZhItemDesc *d_items, u32 nitems, bool gather, bool checksum, int level,
                           hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  std::vector<hipEvent_t> ev;
  {
    std::lock_guard<std::mutex> g(prof().mu);
    if (prof().on) for (int k = 0; k < 4; k++) ev.push_back(prof_event());
  }
  if (!ev.empty()) (void)hipEventRecord(ev[0], stream);
  (void)hipMemsetAsync(ws.ctr, 0, 4, stream);  // K1's block counter
  // levels >= ZH_DEEP_LEVEL: the deep chain matcher; below: K1's dual-hash parse
  if (level >= ZH_DEEP_LEVEL) {
    hipError_t const e = lz_deep_launch(d_descs, nblocks, ws, level, stream);
    if (e != hipSuccess) return e;
  } else {
    lz_launch(d_descs, nblocks, ws, (u32)ZH_K1_MODE(level), stream);
  }
  if (!ev.empty()) (void)hipEventRecord(ev[1], stream);
  entropy_launch(d_descs, nblocks, ws, window_log, cfg_block_size, d_item_size, d_item_status, d_blk_size, stream);
  if (!ev.empty()) (void)hipEventRecord(ev[2], stream);
  if (gather && nitems) hipLaunchKernelGGL(zh_gather_kernel, dim3(nblocks), dim3(256), 0, stream, d_items, d_descs, d_blk_size, d_item_size, d_item_status);
  if (checksum && nitems) hipLaunchKernelGGL(zh_checksum_kernel, dim3(nitems), dim3(64), 0, stream, d_items, d_descs, d_item_size, d_item_status);
  if (!ev.empty()) {
    (void)hipEventRecord(ev[3], stream);
    std::lock_guard<std::mutex> g(prof().mu);
    prof().pending.push_back(ev);
  }
  return hipGetLastError();
}

hipError_t launch_plan(const void *const *d_in_ptrs, const size_t *d_in_sizes, u32 nitems, u32 bpi, void *const *d_out_ptrs, u64 out_cap,
                       u8 *staging, ZhBlockDesc *d_descs, ZhItemDesc *d_items, u64 *d_item_size, u32 *d_item_status, u32 extra_flags,
                       const u8 *dict, u32 dict_n, u32 dict_id, u32 hist, hipStream_t stream) {
  u32 const total = nitems * bpi;
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(zh_plan_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, d_in_ptrs, d_in_sizes, nitems, bpi, d_out_ptrs, out_cap,
                     staging, d_descs, d_items, d_item_size, d_item_status, extra_flags, dict, dict_n, dict_id, hist);
  return hipGetLastError();
}

}  // namespace zh
