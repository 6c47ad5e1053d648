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

// Cast. An 8-elements-per-lane kernel measured 4.10 TB/s bf16 -> fp32 against 5.49 for torch's
// copy (profiles/r01_initial/kernel_microbench.jsonl:14): one of its two sides is a
// 32-B-per-lane access split over two instructions that each touch every other 16 B of a
// wave's span. Here a lane moves E elements with E chosen so the WIDER side
// is exactly one 16-B access per lane (bf16 <-> fp32: 8 B in, 16 B out; 16-bit <-> 16-bit: 16 B
// both): every wave instruction covers one contiguous 512 B / 1 KiB span. U such vectors per
// lane are loaded before any is stored (U x 16 B in flight per lane), block-contiguous tiles of
// 256 x U vectors, grid-stride over tiles. NT: non-temporal stores (a streaming destination is
// not re-read by this kernel). U, NT and the grid cap per dtype pair and size: launch_cast.
template <int DT, int E>
struct VecIO;
template <>
struct VecIO<DT_F32, 4> {
  template <bool NT = false>
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[4]) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p) + i;
    f32x4 t;
    if constexpr (NT) t = __builtin_nontemporal_load(q); else t = *q;
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
  template <bool NT = false>
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[4]) {
    const u16x4* q = reinterpret_cast<const u16x4*>(p) + i;
    u16x4 t;
    if constexpr (NT) t = __builtin_nontemporal_load(q); else t = *q;
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
  template <bool NT = false>
  __device__ __forceinline__ static void ld(const void* p, int64_t i, float (&v)[8]) {
    const u16x8* q = reinterpret_cast<const u16x8*>(p) + i;
    u16x8 t;
    if constexpr (NT) t = __builtin_nontemporal_load(q); else t = *q;
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

template <int DTI, int DTO>
__global__ void __launch_bounds__(256) cast_scalar_kernel(const void* __restrict__ src,
                                                          void* __restrict__ dst, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    Elem<DTO>::st(static_cast<typename Elem<DTO>::T*>(dst), i,
                  Elem<DTI>::ld(static_cast<const typename Elem<DTI>::T*>(src), i));
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

// Round-6 pack: a 2-D grid — x over 16-B column vectors of a row,
// y over groups of R rows (grid-stride) — so a lane never divides a flat index by the row
// length (the 64-bit division per vector of pack_rows_kernel), and R rows' loads are in flight
// before the first store.
template <int DTI, int DTO, int R, bool NT>
__global__ void __launch_bounds__(256) pack2_kernel(const void* __restrict__ src,
                                                    void* __restrict__ dst, int64_t rows,
                                                    int64_t cols, int64_t ld_src, int64_t ld_dst) {
  using TI = typename Elem<DTI>::T;
  using TO = typename Elem<DTO>::T;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= cols / 8) return;
  for (int64_t r0 = static_cast<int64_t>(blockIdx.y) * R; r0 < rows;
       r0 += static_cast<int64_t>(gridDim.y) * R) {
    float v[R][8];
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (r0 + u < rows) load8<DTI>(static_cast<const TI*>(src) + (r0 + u) * ld_src, c, v[u]);
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (r0 + u >= rows) continue;
      TO* q = static_cast<TO*>(dst) + (r0 + u) * ld_dst;
      if constexpr (NT && DTO != DT_F32) {
        u16x8 t;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          t[j] = DTO == DT_BF16 ? f32_to_bf16(v[u][j]) : f32_to_f16(v[u][j]);
        __builtin_nontemporal_store(t, reinterpret_cast<u16x8*>(q) + c);
      } else {
        store8<DTO>(q, c, v[u]);
      }
    }
  }
}
// Launch policy from the grid-shape A/B of these kernels (profiles/r06_kernels/
// memroof_grid_ab.jsonl, TB/s at 64 MiB / 1 GiB of source): past the MALL a one-tile-per-
// workgroup grid beats the 4096-workgroup grid-stride form by 5-17 % (bf16 -> fp32 6.48 vs 5.55,
// torch's copy 5.83); widening casts take non-temporal stores at every size (U = 2: 6.93 / 6.48),
// narrowing ones U = 8 + NT below the MALL (6.67) and U = 2 plain above it (5.94 vs torch 5.87),
// same-width copies U = 2 plain (6.70 / 5.84) except between 128 and 256 MiB (U = 8 + NT).
template <int DTI, int DTO, int U, bool NT>
static void launch_cast2(const void* s, void* d, int64_t n, int64_t cap, hipStream_t st) {
  constexpr int E = cast_vec<DTI, DTO>();
  int64_t g = (n / E + 256 * U - 1) / (256 * U);
  g = g < 1 ? 1 : g;
  if (cap > 0 && g > cap) g = cap;
  if (g > (int64_t{1} << 30)) g = int64_t{1} << 30;    // grid-stride beyond
  hipLaunchKernelGGL((cast2_kernel<DTI, DTO, U, NT>), dim3(static_cast<unsigned>(g)), dim3(256),
                     0, st, s, d, n);
}

template <int DTI, int DTO>
static hipError_t launch_cast(const void* s, void* d, int64_t n, hipStream_t st) {
  const int block = 256;
  const uintptr_t align = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d);
  if (align & 15) {       // a view not 16-B aligned: one element per lane
    hipLaunchKernelGGL((cast_scalar_kernel<DTI, DTO>), dim3(stream_grid(n, block)), dim3(block),
                       0, st, s, d, n);
    return hipGetLastError();
  }
  constexpr int ei = Elem<DTI>::kBytes, eo = Elem<DTO>::kBytes;
  const bool big = n * ei > (int64_t{256} << 20);       // past the 256-MB MALL
  if constexpr (eo > ei) {
    launch_cast2<DTI, DTO, 2, true>(s, d, n, big ? 0 : 16384, st);
  } else if constexpr (eo < ei) {
    if (big) launch_cast2<DTI, DTO, 2, false>(s, d, n, 0, st);
    else launch_cast2<DTI, DTO, 8, true>(s, d, n, 4096, st);
  } else if (n * ei > (int64_t{128} << 20) && !big) {
    // same width, source + destination past the MALL but the source within it: NT stores
    // (256 MiB: 6.94 TB/s vs 5.50 plain, memroof_batched_*.jsonl)
    launch_cast2<DTI, DTO, 8, true>(s, d, n, 4096, st);
  } else {
    launch_cast2<DTI, DTO, 2, false>(s, d, n, big ? 0 : 4096, st);
  }
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
  if (vec_ok) {
    // grid-shape A/B (profiles/r06_kernels/memroof_grid_ab.jsonl, QKV column slice): one row
    // per lane-group and one tile per workgroup below 128 MiB of destination (64 MiB: 6.84 TB/s
    // vs torch's strided copy 6.21), 4 rows in flight + non-temporal stores past it (1 GiB:
    // 5.68 vs 5.79 — the one size torch's copy still leads); both on the uncapped grid
    const int64_t gx = (cols / 8 + 255) / 256;
    const bool big = rows * cols * eo >= (int64_t{128} << 20);
    const int R = big ? 4 : 1;
    const int64_t gy = (rows + R - 1) / R;
    const dim3 gd(static_cast<unsigned>(gx), static_cast<unsigned>(gy < 65535 ? gy : 65535));
    if (big)
      hipLaunchKernelGGL((pack2_kernel<DTI, DTO, 4, true>), gd, dim3(block), 0, st, s, d, rows,
                         cols, lds, ldd);
    else
      hipLaunchKernelGGL((pack2_kernel<DTI, DTO, 1, false>), gd, dim3(block), 0, st, s, d, rows,
                         cols, lds, ldd);
    return hipGetLastError();
  }
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
