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

// Cast v2 (default). The kernel above measured 4.10 TB/s bf16 -> fp32 against 5.49 for torch's
// copy (profiles/r01_initial/kernel_microbench.jsonl:14): it moves 8 elements per lane, so
// one of its two sides is a 32-B-per-lane access split over two instructions that each touch
// every other 16 B of a wave's span. Here a lane moves E elements with E chosen so the WIDER side
// is exactly one 16-B access per lane (bf16 <-> fp32: 8 B in, 16 B out; 16-bit <-> 16-bit: 16 B
// both): every wave instruction covers one contiguous 512 B / 1 KiB span. U such vectors per
// lane are loaded before any is stored (U x 16 B in flight per lane), block-contiguous tiles of
// 256 x U vectors, grid-stride over tiles. NT: non-temporal stores (a streaming destination is
// not re-read by this kernel; A/B via dlbb_cast_set_variant).
template <int DT, int E>
struct VecIO;
template <>
struct VecIO<DT_F32, 4> {
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[4]) {
    const f32x4 t = reinterpret_cast<const f32x4*>(p)[i];
    v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
  }
  template <bool NT>
  __device__ __forceinline__ static void st(void* p, int64_t i, const float (&v)[4]) {
    const f32x4 t = {v[0], v[1], v[2], v[3]};
    f32x4* q = reinterpret_cast<f32x4*>(p) + i;
    if constexpr (NT) __builtin_nontemporal_store(t, q); else *q = t;
  }
};
template <int DT>
struct VecIO16_4 {
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[4]) {
    const u16x4 t = reinterpret_cast<const u16x4*>(p)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = DT == DT_BF16 ? bf16_to_f32(t[j]) : f16_to_f32(t[j]);
  }
  template <bool NT>
  __device__ __forceinline__ static void st(void* p, int64_t i, const float (&v)[4]) {
    u16x4 t;
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = DT == DT_BF16 ? f32_to_bf16(v[j]) : f32_to_f16(v[j]);
    u16x4* q = reinterpret_cast<u16x4*>(p) + i;
    if constexpr (NT) __builtin_nontemporal_store(t, q); else *q = t;
  }
};
template <int DT>
struct VecIO16_8 {
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[8]) {
    const u16x8 t = reinterpret_cast<const u16x8*>(p)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = DT == DT_BF16 ? bf16_to_f32(t[j]) : f16_to_f32(t[j]);
  }
  template <bool NT>
  __device__ __forceinline__ static void st(void* p, int64_t i, const float (&v)[8]) {
    u16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = DT == DT_BF16 ? f32_to_bf16(v[j]) : f32_to_f16(v[j]);
    u16x8* q = reinterpret_cast<u16x8*>(p) + i;
    if constexpr (NT) __builtin_nontemporal_store(t, q); else *q = t;
  }
};
template <> struct VecIO<DT_BF16, 4> : VecIO16_4<DT_BF16> {};
template <> struct VecIO<DT_F16, 4> : VecIO16_4<DT_F16> {};
template <> struct VecIO<DT_BF16, 8> : VecIO16_8<DT_BF16> {};
template <> struct VecIO<DT_F16, 8> : VecIO16_8<DT_F16> {};

template <int DTI, int DTO>
constexpr int cast_vec() {   // elements per lane-vector: the wider side is one 16-B access
  return (Elem<DTI>::kBytes == 4 || Elem<DTO>::kBytes == 4) ? 4 : 8;
}

template <int DTI, int DTO, int U, bool NT>
__global__ void __launch_bounds__(256) cast2_kernel(const void* __restrict__ src,
                                                    void* __restrict__ dst, int64_t n) {
  constexpr int E = cast_vec<DTI, DTO>();
  const int64_t nvec = n / E;
  const int64_t tile = 256 * U;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * tile; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * tile) {
    float v[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256 + threadIdx.x;
      if (i < nvec) VecIO<DTI, E>::ld(src, i, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256 + threadIdx.x;
      if (i < nvec) VecIO<DTO, E>::template st<NT>(dst, i, v[u]);
    }
  }
  if (blockIdx.x == 0) {
    const int64_t t = nvec * E + threadIdx.x;
    if (t < n)
      Elem<DTO>::st(static_cast<typename Elem<DTO>::T*>(dst), t,
                    Elem<DTI>::ld(static_cast<const typename Elem<DTI>::T*>(src), t));
  }
}

// 0: 8-element kernel above, 1: cast2, 2: cast2 + nt stores, 3: 2 with one tile per block,
// 4: 1 with one tile per block, 5 (default): 1 while source + destination fit the 256 MiB MALL,
// else 2 — measured (profiles/r05_kernels/memroof_pass1.jsonl, TB/s v1 / v2): bf16->fp32 64 MiB
// 5.54 / 5.43, 256 MiB 5.15 / 6.56, 1 GiB 5.36 / 5.49; fp32->bf16 256 MiB 4.65 / 5.72
static int g_cast_variant = 5;

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
  constexpr int E = cast_vec<DTI, DTO>(), U = 8;
  const uintptr_t align = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d);
  if (g_cast_variant == 0 || (align & 15)) {
    hipLaunchKernelGGL((cast_kernel<DTI, DTO>), dim3(stream_grid((n + 7) / 8, block)),
                       dim3(block), 0, st, s, d, n);
    return hipGetLastError();
  }
  int v = g_cast_variant;
  if (v == 5)
    v = n * (Elem<DTI>::kBytes + Elem<DTO>::kBytes) > (int64_t{256} << 20) ? 2 : 1;
  int64_t g = (n / E + 256 * U - 1) / (256 * U);
  // variants 3/4: one tile per block (no grid-stride loop), as torch's elementwise launch
  const int64_t cap = v >= 3 ? (int64_t{1} << 30) : 4096;
  g = g < 1 ? 1 : (g > cap ? cap : g);
  if (v == 2 || v == 3)
    hipLaunchKernelGGL((cast2_kernel<DTI, DTO, U, true>), dim3(g), dim3(block), 0, st, s, d, n);
  else
    hipLaunchKernelGGL((cast2_kernel<DTI, DTO, U, false>), dim3(g), dim3(block), 0, st, s, d, n);
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


// A/B switch: 0 = 8-element kernel, 1 = one 16-B wide side per lane, 2 = 1 + nt stores,
// 3 = 2 without the grid-stride cap, 4 = 1 without it, 5 = 1 or 2 by size (default)
DLBB_API void dlbb_cast_set_variant(int v) { g_cast_variant = v < 0 || v > 5 ? 5 : v; }

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
