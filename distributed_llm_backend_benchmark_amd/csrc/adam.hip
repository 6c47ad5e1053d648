// Fused AdamW over flat buffers (one launch for the whole model).
//
// The reference's only optimizer step is DeepSpeed's Adam inside `model_engine.step()`
// (test/ccl.py:114-115). The DDP microbenchmark keeps parameters, gradients and optimizer state
// as single flat device buffers (gradient buckets are views of the flat gradient buffer), so the
// optimizer is one HBM-streaming pass:
//   reads  fp32 master p, m, v, and the bf16|fp32 reduced gradient g (scaled by grad_scale,
//          e.g. 1/world for averaging — fused here instead of a separate pass)
//   writes fp32 p, m, v and the bf16 working copy used by the next forward.
#include "common.h"

namespace dlbb {

struct AdamArgs {
  float* p;
  float* m;
  float* v;
  const void* g;
  uint16_t* p_bf16;   // optional bf16 shadow of p
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2;     // 1 - beta^t
  float grad_scale;
  const int* step_dev;   // optional: step count read on the device (HIP-graph replayable)
  // optional row filter: update only the elements of rows r (row_len elements each, row_len %
  // 8 == 0) with row_mask[r] == row_sel — one table's rows split between two AdamW calls
  const uint8_t* row_mask;
  int64_t row_len;
  int row_sel;
};

// fp32 state streamed once per step (p, m, v: 12 B/param in, 12 B out — past the 256 MiB MALL
// for any real model): NT = non-temporal loads/stores for them (A/B, DLBB_ADAMW_NT)
template <bool NT>
__device__ __forceinline__ void ld8f(const float* base, int64_t i8, float (&v)[8]) {
  const f32x4* q = reinterpret_cast<const f32x4*>(base) + 2 * i8;
  f32x4 x, y;
  if constexpr (NT) { x = __builtin_nontemporal_load(q); y = __builtin_nontemporal_load(q + 1); }
  else { x = q[0]; y = q[1]; }
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = x[j]; v[4 + j] = y[j]; }
}
template <bool NT>
__device__ __forceinline__ void st8f(float* base, int64_t i8, const float (&v)[8]) {
  f32x4* q = reinterpret_cast<f32x4*>(base) + 2 * i8;
  const f32x4 x = {v[0], v[1], v[2], v[3]}, y = {v[4], v[5], v[6], v[7]};
  if constexpr (NT) { __builtin_nontemporal_store(x, q); __builtin_nontemporal_store(y, q + 1); }
  else { q[0] = x; q[1] = y; }
}

template <int GDT, bool NT = false>
__global__ void __launch_bounds__(256) adamw_kernel(AdamArgs a) {
  const int64_t nvec = a.n / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  float bc1 = a.bc1, bc2 = a.bc2;
  if (a.step_dev) {            // graph replay: the step advances in device memory
    const float t = static_cast<float>(*a.step_dev);
    bc1 = 1.f - powf(a.beta1, t);
    bc2 = 1.f - powf(a.beta2, t);
  }
  const float step = a.lr / bc1;
  const float inv_bc2 = 1.0f / bc2;
  auto body = [&](float& p, float& m, float& v, float g) {
    g *= a.grad_scale;
    m = a.beta1 * m + (1.f - a.beta1) * g;
    v = a.beta2 * v + (1.f - a.beta2) * g * g;
    const float denom = sqrtf(v * inv_bc2) + a.eps;
    p = p * (1.f - a.lr * a.weight_decay) - step * m / denom;
  };
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec;
       i += stride) {
    if (a.row_mask && a.row_mask[i * 8 / a.row_len] != a.row_sel) continue;
    float p[8], m[8], v[8], g[8];
    ld8f<NT>(a.p, i, p);
    ld8f<NT>(a.m, i, m);
    ld8f<NT>(a.v, i, v);
    load8<GDT>(a.g, i, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) body(p[j], m[j], v[j], g[j]);
    st8f<NT>(a.p, i, p);
    st8f<NT>(a.m, i, m);
    st8f<NT>(a.v, i, v);
    if (a.p_bf16) store8<DT_BF16>(a.p_bf16, i, p);
  }
  if (blockIdx.x == 0) {
    const int64_t t = nvec * 8 + threadIdx.x;
    if (t < a.n && !(a.row_mask && a.row_mask[t / a.row_len] != a.row_sel)) {
      float p = a.p[t], m = a.m[t], v = a.v[t];
      const float g = Elem<GDT>::ld(static_cast<const typename Elem<GDT>::T*>(a.g), t);
      body(p, m, v, g);
      a.p[t] = p; a.m[t] = m; a.v[t] = v;
      if (a.p_bf16) a.p_bf16[t] = f32_to_bf16(p);
    }
  }
}

}  // namespace dlbb

using namespace dlbb;

static int g_adamw_nt = 0;   // non-temporal fp32 state traffic (A/B: dlbb_adamw_set_nt)
DLBB_API void dlbb_adamw_set_nt(int on) { g_adamw_nt = on ? 1 : 0; }

static int launch_adamw(const AdamArgs& a, int grad_dtype, hipStream_t stream) {
  const int grid = stream_grid((a.n + 7) / 8, 256);
  // 32-byte alignment of the fp32 arrays for the two float4 halves of an 8-vector
  const bool nt = g_adamw_nt && !((reinterpret_cast<uintptr_t>(a.p) | reinterpret_cast<uintptr_t>(a.m) |
                                   reinterpret_cast<uintptr_t>(a.v)) & 15);
  if (grad_dtype == DT_BF16) {
    if (nt) hipLaunchKernelGGL((adamw_kernel<DT_BF16, true>), dim3(grid), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((adamw_kernel<DT_BF16, false>), dim3(grid), dim3(256), 0, stream, a);
  } else if (grad_dtype == DT_F32) {
    if (nt) hipLaunchKernelGGL((adamw_kernel<DT_F32, true>), dim3(grid), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((adamw_kernel<DT_F32, false>), dim3(grid), dim3(256), 0, stream, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

DLBB_API int dlbb_adamw(float* p, float* m, float* v, const void* g, int grad_dtype,
                        void* p_bf16, int64_t n, float lr, float beta1, float beta2, float eps,
                        float weight_decay, int step, float grad_scale, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (step < 1) return hipErrorInvalidValue;
  AdamArgs a{p, m, v, g, static_cast<uint16_t*>(p_bf16), n, lr, beta1, beta2, eps,
             weight_decay, 1.f - powf(beta1, static_cast<float>(step)),
             1.f - powf(beta2, static_cast<float>(step)), grad_scale, nullptr, nullptr, 1, 0};
  return launch_adamw(a, grad_dtype, stream);
}

// Same update with the step count (>= 1) read from device memory `step_dev` — the form a HIP
// graph can replay (the caller advances the counter on the stream before each update).
DLBB_API int dlbb_adamw_devstep(float* p, float* m, float* v, const void* g, int grad_dtype,
                                void* p_bf16, int64_t n, float lr, float beta1, float beta2,
                                float eps, float weight_decay, const int* step_dev,
                                float grad_scale, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (!step_dev) return hipErrorInvalidValue;
  AdamArgs a{p, m, v, g, static_cast<uint16_t*>(p_bf16), n, lr, beta1, beta2, eps,
             weight_decay, 1.f, 1.f, grad_scale, step_dev, nullptr, 1, 0};
  return launch_adamw(a, grad_dtype, stream);
}

// Row-filtered update (either step form: step_dev non-null = device step count, else `step`):
// only rows r of the [n / row_len, row_len] range with row_mask[r] == row_sel.
DLBB_API int dlbb_adamw_rows(float* p, float* m, float* v, const void* g, int grad_dtype,
                             void* p_bf16, int64_t n, float lr, float beta1, float beta2,
                             float eps, float weight_decay, int step, const int* step_dev,
                             float grad_scale, const uint8_t* row_mask, int64_t row_len,
                             int row_sel, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (!row_mask || row_len <= 0 || row_len % 8 || n % row_len) return hipErrorInvalidValue;
  if (!step_dev && step < 1) return hipErrorInvalidValue;
  const float b1 = step_dev ? 1.f : 1.f - powf(beta1, static_cast<float>(step));
  const float b2 = step_dev ? 1.f : 1.f - powf(beta2, static_cast<float>(step));
  AdamArgs a{p, m, v, g, static_cast<uint16_t*>(p_bf16), n, lr, beta1, beta2, eps,
             weight_decay, b1, b2, grad_scale, step_dev, row_mask, row_len, row_sel};
  return launch_adamw(a, grad_dtype, stream);
}
