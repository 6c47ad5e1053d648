// Cast / pack kernels.
//
// Replaces the reference's host staging chain bf16 -> fp32 -> numpy -> MPI -> numpy -> bf16
// (models.py:84-98; collectives/3d/openmpi.py:43) with on-device conversion:
//   dlbb_cast        : contiguous dtype conversion (bf16/fp16/fp32 in any direction)
//   dlbb_pack_rows   : strided 2-D gather + cast into a dense buffer — e.g. the QKV
//                      column slice `qkv[:, :, :H/P]` (models.py:166-167) or any [rows, cols]
//                      view with a row stride, in one pass.
#include "common.h"

namespace dlbb {

template <int DTI, int DTO>
__global__ void __launch_bounds__(256) cast_kernel(const void* __restrict__ src,
                                                   void* __restrict__ dst, int64_t n) {
  const int64_t nvec = n / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < nvec; i += 4 * stride) {   // 4 loads in flight before any store
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8<DTI>(src, i + u * stride, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) store8<DTO>(dst, i + u * stride, v[u]);
  }
  for (; i < nvec; i += stride) {
    float v[8];
    load8<DTI>(src, i, v);
    store8<DTO>(dst, i, v);
  }
  if (blockIdx.x == 0) {
    const int64_t t = nvec * 8 + threadIdx.x;
    if (t < n)
      Elem<DTO>::st(static_cast<typename Elem<DTO>::T*>(dst), t,
                    Elem<DTI>::ld(static_cast<const typename Elem<DTI>::T*>(src), t));
  }
}

// One wave-row loop: rows x cols, source row stride ld_src (elements), dense-or-strided dest.
template <int DTI, int DTO>
__global__ void __launch_bounds__(256) pack_rows_kernel(const void* __restrict__ src,
                                                        void* __restrict__ dst, int64_t rows,
                                                        int64_t cols, int64_t ld_src,
                                                        int64_t ld_dst, int vec_ok) {
  using TI = typename Elem<DTI>::T;
  using TO = typename Elem<DTO>::T;
  const int64_t per_row = vec_ok ? cols / 8 : cols;
  const int64_t total = rows * per_row;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += stride) {
    const int64_t r = i / per_row, c = i - r * per_row;
    if (vec_ok) {
      float v[8];
      load8<DTI>(static_cast<const TI*>(src) + r * ld_src, c, v);
      store8<DTO>(static_cast<TO*>(dst) + r * ld_dst, c, v);
    } else {
      Elem<DTO>::st(static_cast<TO*>(dst), r * ld_dst + c,
                    Elem<DTI>::ld(static_cast<const TI*>(src), r * ld_src + c));
    }
  }
}

template <int DTI, int DTO>
static hipError_t launch_cast(const void* s, void* d, int64_t n, hipStream_t st) {
  const int block = 256;
  hipLaunchKernelGGL((cast_kernel<DTI, DTO>), dim3(stream_grid((n + 7) / 8, block)),
                     dim3(block), 0, st, s, d, n);
  return hipGetLastError();
}

template <int DTI, int DTO>
static hipError_t launch_pack(const void* s, void* d, int64_t rows, int64_t cols,
                              int64_t lds, int64_t ldd, hipStream_t st) {
  const int ei = Elem<DTI>::kBytes, eo = Elem<DTO>::kBytes;
  const bool vec_ok = (cols % 8 == 0) && (lds % 8 == 0) && (ldd % 8 == 0) &&
                      (reinterpret_cast<uintptr_t>(s) % (8 * ei) == 0) &&
                      (reinterpret_cast<uintptr_t>(d) % (8 * eo) == 0);
  const int64_t work = rows * (vec_ok ? cols / 8 : cols);
  const int block = 256;
  hipLaunchKernelGGL((pack_rows_kernel<DTI, DTO>), dim3(stream_grid(work, block)), dim3(block),
                     0, st, s, d, rows, cols, lds, ldd, vec_ok ? 1 : 0);
  return hipGetLastError();
}

}  // namespace dlbb

using namespace dlbb;


DLBB_API int dlbb_cast(const void* src, int dtype_in, void* dst, int dtype_out, int64_t n,
                       hipStream_t stream) {
  if (n <= 0) return n == 0 ? hipSuccess : hipErrorInvalidValue;
#define CALLC(a, b) launch_cast<a, b>(src, dst, n, stream)
  if (dtype_in == DT_BF16 && dtype_out == DT_F32) return CALLC(DT_BF16, DT_F32);
  if (dtype_in == DT_F32 && dtype_out == DT_BF16) return CALLC(DT_F32, DT_BF16);
  if (dtype_in == DT_F16 && dtype_out == DT_F32) return CALLC(DT_F16, DT_F32);
  if (dtype_in == DT_F32 && dtype_out == DT_F16) return CALLC(DT_F32, DT_F16);
  if (dtype_in == DT_BF16 && dtype_out == DT_F16) return CALLC(DT_BF16, DT_F16);
  if (dtype_in == DT_F16 && dtype_out == DT_BF16) return CALLC(DT_F16, DT_BF16);
  if (dtype_in == DT_BF16 && dtype_out == DT_BF16) return CALLC(DT_BF16, DT_BF16);
  if (dtype_in == DT_F16 && dtype_out == DT_F16) return CALLC(DT_F16, DT_F16);
  if (dtype_in == DT_F32 && dtype_out == DT_F32) return CALLC(DT_F32, DT_F32);
#undef CALLC
  return hipErrorInvalidValue;
}

DLBB_API int dlbb_pack_rows(const void* src, int dtype_in, int64_t ld_src, void* dst,
                            int dtype_out, int64_t ld_dst, int64_t rows, int64_t cols,
                            hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
#define CALLP(a, b) launch_pack<a, b>(src, dst, rows, cols, ld_src, ld_dst, stream)
  if (dtype_in == DT_BF16 && dtype_out == DT_F32) return CALLP(DT_BF16, DT_F32);
  if (dtype_in == DT_F32 && dtype_out == DT_BF16) return CALLP(DT_F32, DT_BF16);
  if (dtype_in == DT_F16 && dtype_out == DT_F32) return CALLP(DT_F16, DT_F32);
  if (dtype_in == DT_F32 && dtype_out == DT_F16) return CALLP(DT_F32, DT_F16);
  if (dtype_in == DT_BF16 && dtype_out == DT_BF16) return CALLP(DT_BF16, DT_BF16);
  if (dtype_in == DT_F16 && dtype_out == DT_F16) return CALLP(DT_F16, DT_F16);
  if (dtype_in == DT_F32 && dtype_out == DT_F32) return CALLP(DT_F32, DT_F32);
#undef CALLP
  return hipErrorInvalidValue;
}
