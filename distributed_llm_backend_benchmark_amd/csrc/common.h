// Shared helpers for the gfx950 (MI355X, CDNA4) kernels of this package.
//
// Conventions used by every kernel file:
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * bf16/fp16 move as 16-byte vectors (8 elements / lane) — hipcc does not vectorise
//     scalar 16-bit loads (CDNA guide, Guideline 13).
//   * accumulation is fp32; bf16 rounding uses the native v_cvt_pk_bf16_f32 (RNE, NaN-safe),
//     which hipcc emits for a plain (__bf16) cast on gfx950.
//   * every launcher is a plain C ABI function taking raw device pointers and a hipStream_t,
//     returns hipError_t as int, allocates nothing and never synchronises (graph-capturable).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DLBB_API extern "C" __attribute__((visibility("default")))

namespace dlbb {

enum DType : int { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

constexpr int kWave = 64;

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));   // MFMA operand fragment
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(3))) i16x4* lds_i16x4_ptr;

// Transposed LDS read (ds_read_b64_tr_b16) issued through inline asm, at byte address
// `lds` + OFF (OFF: the instruction's 16-bit immediate). The builtin form carries an LDS memory
// operand that the compiler's wait-count pass cannot separate from LDS-DMA still in flight into
// ANOTHER buffer of a multi-buffered loop, so it put `s_waitcnt vmcnt(0)` before the first such
// read of every iteration — draining the very prefetch the loop overlaps (NN / TN ping-pong
// GEMMs, the weight-gradient kernel, all attention kernels; tools/isa_check.py reports it).
// The asm read is invisible to that pass in both directions: the compiler never waits for its
// RESULT either, so every caller issues `s_waitcnt lgkmcnt(0)` before any use of the returned
// registers (tr_wait below ties the wait to them). tools/isa_check.py checks the compiled code:
// no instruction may touch a destination register of such a read before an lgkmcnt(0).
template <int OFF = 0>
__device__ __forceinline__ i16x4 ds_read_tr16(const void* lds) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is a 16-bit immediate");
  i16x4 t;
  const uint32_t addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_i16x4_ptr)(lds)));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t) : "v"(addr), "n"(OFF));
  return t;
}

// 16-byte LDS read through inline asm at `lds` + OFF, for reads of a region that LDS-DMA also
// fills (same reason and same contract as ds_read_tr16: wait lgkmcnt(0) before use)
template <int OFF = 0>
__device__ __forceinline__ f32x4 ds_read_b128_asm(const void* lds) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is a 16-bit immediate");
  f32x4 t;
  const uint32_t addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_vptr_t)(lds)));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(t) : "v"(addr), "n"(OFF));
  return t;
}

// s_waitcnt lgkmcnt(0) that the fragments passed in depend on, so no use of them can be
// scheduled before it (see ds_read_tr16); later arguments are tied by empty asm statements
// ordered after the wait
template <typename F>
__device__ __forceinline__ void tr_tie(F& f) {
  asm volatile("" : "+v"(f));
}
template <typename F, typename... R>
__device__ __forceinline__ void tr_wait(F& f, R&... r) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f));
  (tr_tie(r), ...);
}
// Counted form: the reads issued BEFORE the last N LDS operations have landed (LDS returns in
// order; any other LDS op issued in between only makes the wait stricter). The arguments are
// those reads' destinations.
template <int N, typename F, typename... R>
__device__ __forceinline__ void lgk_wait(F& f, R&... r) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f) : "n"(N));
  (tr_tie(r), ...);
}

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
__device__ __forceinline__ float f16_to_f32(uint16_t v) {
  return static_cast<float>(__builtin_bit_cast(_Float16, v));
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}

// Element traits: load/store one element as fp32.
template <int DT> struct Elem;
template <> struct Elem<DT_F32> {
  using T = float;
  static constexpr int kBytes = 4;
  __device__ __forceinline__ static float ld(const T* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void st(T* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<DT_BF16> {
  using T = uint16_t;
  static constexpr int kBytes = 2;
  __device__ __forceinline__ static float ld(const T* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ __forceinline__ static void st(T* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};
template <> struct Elem<DT_F16> {
  using T = uint16_t;
  static constexpr int kBytes = 2;
  __device__ __forceinline__ static float ld(const T* p, int64_t i) { return f16_to_f32(p[i]); }
  __device__ __forceinline__ static void st(T* p, int64_t i, float v) { p[i] = f32_to_f16(v); }
};

// 8 consecutive elements <-> 8 floats (one 16 B load for 16-bit types, two for fp32).
template <int DT>
__device__ __forceinline__ void load8(const void* base, int64_t i8, float (&v)[8]) {
  if constexpr (DT == DT_F32) {
    const float4* p = reinterpret_cast<const float4*>(base) + 2 * i8;
    float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    u16x8 r = reinterpret_cast<const u16x8*>(base)[i8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (DT == DT_BF16) ? bf16_to_f32(r[j]) : f16_to_f32(r[j]);
  }
}

template <int DT>
__device__ __forceinline__ void store8(void* base, int64_t i8, const float (&v)[8]) {
  if constexpr (DT == DT_F32) {
    float4* p = reinterpret_cast<float4*>(base) + 2 * i8;
    p[0] = make_float4(v[0], v[1], v[2], v[3]);
    p[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      r[j] = (DT == DT_BF16) ? f32_to_bf16(v[j]) : f32_to_f16(v[j]);
    reinterpret_cast<u16x8*>(base)[i8] = r;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// erf(z) on v_exp_f32 + v_rcp_f32 (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7): ~14 VALU ops,
// branch-free, instead of libm erff — the GELU epilogue of the 7B FFN-up GEMM (4096 x 16384
// outputs per call) was VALU-bound on it.
__device__ __forceinline__ float fast_erf(float z) {
  const float az = __builtin_fabsf(z);
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, az, 1.0f));
  float p = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  p = __builtin_fmaf(p, t, 1.421413741f);
  p = __builtin_fmaf(p, t, -0.284496736f);
  p = __builtin_fmaf(p, t, 0.254829592f);
  const float r = 1.0f - p * t * __expf(-az * az);
  return __builtin_copysignf(r, z);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + fast_erf(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + fast_erf(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// tanh(u) = 1 - 2 / (exp(2u) + 1) on v_exp_f32 + v_rcp_f32 (a handful of VALU ops instead of
// the branchy libm tanhf, which made the bias-GELU passes VALU-bound); saturates correctly
// (exp -> inf gives 1, exp -> 0 gives -1); ~1e-6 relative error, far below bf16 resolution.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * u) + 1.0f);
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + fast_tanh(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float t = fast_tanh(k0 * (x + k1 * x2 * x));
  return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * k1 * x2);
}

// ---------------------------------------------------------------------------------------
// Per-workgroup start / end stamps (opt-in diagnostic, dlbb_stamps_set): a stamped launch
// writes one 32-byte record per workgroup, [t_start, t_end, HW_ID | XCC_ID << 32,
// blockIdx.x | blockIdx.y << 32], times from s_memrealtime (100 MHz, shared by every CU).
// Only thread 0 of a workgroup stores, once, after the workgroup's last barrier — nothing the
// kernel computes reads a stamp. Host registry in csrc/reduce.hip; unstamped launches (the
// default) run kernels without any stamp code.
enum StampKind { STAMP_GEMM_NT = 1, STAMP_GEMM_NN = 2, STAMP_GEMM_TN = 3, STAMP_REDUCE = 4,
                 STAMP_SPIN = 5 };
// host: `nrec` records for one launch of `kind`, or nullptr (stamps off / buffer full)
uint64_t* stamp_acquire(int kind, int64_t nrec);

__device__ __forceinline__ uint64_t stamp_now() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// thread 0 of the workgroup, after its final barrier
__device__ __forceinline__ void stamp_write(uint64_t* recs, uint64_t t0) {
  const uint64_t t1 = stamp_now();
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
  const uint64_t wg = blockIdx.x + static_cast<uint64_t>(blockIdx.y) * gridDim.x;
  uint64_t* r = recs + 4 * wg;
  r[0] = t0;
  r[1] = t1;
  r[2] = hw | (static_cast<uint64_t>(xcc) << 32);
  r[3] = blockIdx.x | (static_cast<uint64_t>(blockIdx.y) << 32);
}

// Grid size for memory-bound grid-stride kernels: enough blocks to fill 256 CUs several
// times over, capped (CDNA guide, Guideline 11).
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return static_cast<int>(g);
}

}  // namespace dlbb
