// Streams restricted to a subset of the CUs (hipExtStreamCreateWithCUMask).
//
// The DDP step runs the weight-gradient GEMMs on a side stream beside the backward's critical
// path. Unrestricted, their LDS-heavy workgroups (3 x 48 KiB per CU) spread over every CU, and a
// main-stream ping-pong GEMM workgroup (one per CU, ~130 KiB of LDS) cannot start on a CU until
// they leave: the main stream's kernels run 1.1-3x slower inside the step than alone
// (profiles/r05_step/SUMMARY.md §2). A CU mask confines the side stream to a fixed share of every
// XCD, so the rest of the chip is always free for the critical path.
#include "common.h"

#include <vector>

// Mask of `ncu` CUs keeping CU i when (i / 8) % den < num: the same share of every XCD whether
// the mask bits map to CUs XCD-interleaved (XCD = i % 8) or XCD-contiguous (XCD = i / 32).
// Returns the number of CUs kept; writes the stream handle to *out.
DLBB_API int dlbb_stream_create_cu_share(int ncu, int num, int den, hipStream_t* out,
                                         int* kept) {
  if (ncu <= 0 || num <= 0 || den <= 0 || num > den || !out) return hipErrorInvalidValue;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  int n = 0;
  for (int i = 0; i < ncu; ++i)
    if ((i / 8) % den < num) {
      mask[i / 32] |= 1u << (i % 32);
      ++n;
    }
  if (kept) *kept = n;
  return hipExtStreamCreateWithCUMask(out, static_cast<uint32_t>(mask.size()), mask.data());
}

// Active CUs of a stream's mask (-1 on error).
DLBB_API int dlbb_stream_cu_count(hipStream_t s, int ncu) {
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  if (hipExtStreamGetCUMask(s, static_cast<uint32_t>(mask.size()), mask.data()) != hipSuccess)
    return -1;
  int n = 0;
  for (uint32_t w : mask) n += __builtin_popcount(w);
  return n;
}

// Fork `to` after the work queued on `from` so far, with an event that skips the system-scope
// fence a default HIP event's record performs (L2 writeback and invalidate, for host
// visibility). Ordering between two streams of one device needs no system fence: every kernel
// dispatch already releases its writes at device scope at the end of the kernel.
// mode 1: hipEventDisableSystemFence, 2: hipEventReleaseToDevice. Events come from a per-device
// ring (a wait binds to the record that precedes it, so a slot is reusable once re-recorded).
namespace {
constexpr int kForkRing = 64;
struct ForkRing {
  hipEvent_t ev[kForkRing] = {};
  int next = 0;
  int mode = 0;
};
ForkRing g_fork[64];
}  // namespace

DLBB_API int dlbb_stream_fork(hipStream_t from, hipStream_t to, int mode) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64 || (mode != 1 && mode != 2)) return hipErrorInvalidValue;
  ForkRing& r = g_fork[dev];
  if (r.mode != mode) {                     // (re)create the ring for this flag set
    for (auto& x : r.ev)
      if (x) { hipEventDestroy(x); x = nullptr; }
    const unsigned flags = hipEventDisableTiming |
                           (mode == 1 ? hipEventDisableSystemFence : hipEventReleaseToDevice);
    for (auto& x : r.ev)
      if ((e = hipEventCreateWithFlags(&x, flags)) != hipSuccess) return e;
    r.mode = mode;
    r.next = 0;
  }
  hipEvent_t ev = r.ev[r.next];
  r.next = (r.next + 1) % kForkRing;
  if ((e = hipEventRecord(ev, from)) != hipSuccess) return e;
  return hipStreamWaitEvent(to, ev, 0);
}
