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
