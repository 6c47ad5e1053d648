// Stream ordering without the system-scope fence of a default HIP event (parallel/streams.py).
// (Round 5's CU-masked side streams, hipExtStreamCreateWithCUMask, measured 2.7-3x slower for
// the weight gradients and were removed in round 6.)
#include "common.h"

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
