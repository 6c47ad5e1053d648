// n-way sum-reduce: dst = scale * sum_i src_i   (fp32 accumulation).
//
// This is the local SUM that the reference's backends run on the host inside every
// all-reduce / reduce (mpi4py pickle path applies numpy `a+b` in Python:
// collectives/1d/openmpi.py:63,148; oneCCL/Gloo reduce loops: collectives/1d/dsccl.py:65).
// Here it is one HBM-streaming kernel over up to 16 source buffers (local copies, or peer
// buffers mapped over xGMI by the IPC all-reduce), 16-byte vector I/O, grid-stride.
// HBM roofline: (nsrc + 1) * bytes / 6.3 TB/s.
#include <vector>

#include "common.h"

namespace dlbb {

constexpr int kMaxSrc = 16;

struct ReduceArgs {
  const void* src[kMaxSrc];
  void* dst;
  int64_t n;       // elements
  int nsrc;
  float scale;
  uint64_t* stamps;  // per-workgroup start/end records (diagnostic), usually null
};

// Runtime source count, one source per loop trip. Round 5 measured a templated count with every
// source's load in flight equal within noise (1-3 % behind), round 6 block-contiguous tiles of
// 1-4 vectors per lane with and without non-temporal source loads: within +-10 % of this at
// 64 MiB-1 GiB in both directions (profiles/r06_kernels/memroof_variants.jsonl) — the hardware
// already overlaps the loop trips' loads.
template <int DTI, int DTO>
__global__ void __launch_bounds__(256) reduce_sum_kernel(ReduceArgs a) {
  uint64_t t0 = 0;
  if (a.stamps) t0 = stamp_now();
  const int64_t nvec = a.n / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec;
       i += stride) {
    float acc[8];
    load8<DTI>(a.src[0], i, acc);
    for (int s = 1; s < a.nsrc; ++s) {
      float v[8];
      load8<DTI>(a.src[s], i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    if (a.scale != 1.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
    }
    store8<DTO>(a.dst, i, acc);
  }
  // scalar tail (n % 8 elements), handled by block 0
  if (blockIdx.x == 0) {
    const int64_t t = nvec * 8 + threadIdx.x;
    if (t < a.n) {
      float acc = 0.f;
      for (int s = 0; s < a.nsrc; ++s)
        acc += Elem<DTI>::ld(static_cast<const typename Elem<DTI>::T*>(a.src[s]), t);
      Elem<DTO>::st(static_cast<typename Elem<DTO>::T*>(a.dst), t, acc * a.scale);
    }
  }
  if (a.stamps) {
    __syncthreads();
    if (threadIdx.x == 0) stamp_write(a.stamps, t0);
  }
}

// Stand-in for a link-bound transfer (DDP overlap studies on one GPU): each workgroup holds
// its CU slot for `ns` nanoseconds of wall time (s_memrealtime, 100 MHz), sleeping between
// polls — the occupancy and duration of a collective's workgroups without its traffic.
__global__ void __launch_bounds__(64) spin_kernel(uint64_t ticks, uint64_t* stamps) {
  const uint64_t t0 = stamp_now();
  uint64_t t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    t = stamp_now();
  }
  if (stamps && threadIdx.x == 0) stamp_write(stamps, t0);
}

// ---- stamp registry (host)
static uint64_t* g_stamp_buf = nullptr;
static int64_t g_stamp_cap = 0, g_stamp_next = 0;
struct StampEntry {
  int kind;
  int64_t first, count;
};
static std::vector<StampEntry> g_stamp_log;

uint64_t* stamp_acquire(int kind, int64_t nrec) {
  if (!g_stamp_buf || nrec <= 0 || g_stamp_next + nrec > g_stamp_cap) return nullptr;
  uint64_t* p = g_stamp_buf + 4 * g_stamp_next;
  g_stamp_log.push_back({kind, g_stamp_next, nrec});
  g_stamp_next += nrec;
  return p;
}

template <int DTI, int DTO>
static hipError_t launch_reduce(const ReduceArgs& a, int nblocks, hipStream_t s) {
  const int block = 256;
  const int grid = nblocks > 0 ? nblocks : stream_grid((a.n + 7) / 8, block);
  hipLaunchKernelGGL((reduce_sum_kernel<DTI, DTO>), dim3(grid), dim3(block), 0, s, a);
  return hipGetLastError();
}

}  // namespace dlbb

using namespace dlbb;

// srcs: host array of nsrc device pointers (passed by value in the kernel argument block).
// nblocks > 0 caps the grid (a CU budget, e.g. for a reduction running beside compute);
// 0 = enough workgroups to fill the chip.
DLBB_API int dlbb_reduce_sum_grid(const void* const* srcs, int nsrc, void* dst, int64_t n,
                                  int dtype_in, int dtype_out, float scale, int nblocks,
                                  hipStream_t stream) {
  if (nsrc < 1 || nsrc > kMaxSrc || n < 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  ReduceArgs a{};
  for (int i = 0; i < nsrc; ++i) a.src[i] = srcs[i];
  a.dst = dst;
  a.n = n;
  a.nsrc = nsrc;
  a.scale = scale;
  const int grid = nblocks > 0 ? nblocks : stream_grid((n + 7) / 8, 256);
  a.stamps = stamp_acquire(STAMP_REDUCE, grid);
#define DLBB_R(I, O) \
  if (dtype_in == I && dtype_out == O) return launch_reduce<I, O>(a, grid, stream);
  DLBB_R(DT_BF16, DT_BF16) DLBB_R(DT_BF16, DT_F32) DLBB_R(DT_F16, DT_F16)
  DLBB_R(DT_F16, DT_F32) DLBB_R(DT_F32, DT_F32) DLBB_R(DT_F32, DT_BF16)
  DLBB_R(DT_F32, DT_F16)
#undef DLBB_R
  return hipErrorInvalidValue;
}

DLBB_API int dlbb_reduce_sum(const void* const* srcs, int nsrc, void* dst, int64_t n,
                             int dtype_in, int dtype_out, float scale, hipStream_t stream) {
  return dlbb_reduce_sum_grid(srcs, nsrc, dst, n, dtype_in, dtype_out, scale, 0, stream);
}

// Hold `nblocks` workgroup slots for `ns` nanoseconds on `stream` (see spin_kernel).
DLBB_API int dlbb_spin_ns(int64_t ns, int nblocks, hipStream_t stream) {
  if (ns < 0 || nblocks < 1 || nblocks > 65535) return hipErrorInvalidValue;
  uint64_t* st = stamp_acquire(STAMP_SPIN, nblocks);
  hipLaunchKernelGGL(spin_kernel, dim3(nblocks), dim3(64), 0, stream,
                     static_cast<uint64_t>((ns + 9) / 10), st);
  return hipGetLastError();
}

// Stamp buffer: `buf` holds `cap_records` 32-byte records (null disables stamping); resets the
// launch log. Not thread-safe; a diagnostic for one process at a time.
DLBB_API void dlbb_stamps_set(void* buf, int64_t cap_records) {
  g_stamp_buf = static_cast<uint64_t*>(buf);
  g_stamp_cap = buf ? cap_records : 0;
  g_stamp_next = 0;
  g_stamp_log.clear();
}

DLBB_API int64_t dlbb_stamps_launches() { return static_cast<int64_t>(g_stamp_log.size()); }

DLBB_API int dlbb_stamps_entry(int64_t i, int* kind, int64_t* first, int64_t* count) {
  if (i < 0 || i >= static_cast<int64_t>(g_stamp_log.size())) return hipErrorInvalidValue;
  *kind = g_stamp_log[i].kind;
  *first = g_stamp_log[i].first;
  *count = g_stamp_log[i].count;
  return hipSuccess;
}
