// Bias + GELU, forward and backward.
//
// Reference: `torch.nn.functional.gelu(x)` after the column-parallel FFN-up GEMM
// (models.py:181-182; erf form). GPT-2 uses the tanh form. Forward: y = gelu(x + b) in one
// 16-byte-vector pass (the same epilogue is also fused into the MFMA GEMM, gemm.hip).
// Backward: dx = dy * gelu'(x + b), with db = colsum(dx) accumulated in fp32 registers per
// block over a row strip and flushed with one float atomic per (column, block) into an fp32
// workspace (few atomics: rows / strip per column; CDNA guide Guideline 12), then cast.
#include "common.h"

namespace dlbb {

template <int APPROX>
__device__ __forceinline__ float act(float x) { return APPROX ? gelu_tanh(x) : gelu_erf(x); }
template <int APPROX>
__device__ __forceinline__ float act_grad(float x) {
  return APPROX ? gelu_tanh_grad(x) : gelu_erf_grad(x);
}

// cols % 8 == 0. grid-stride over 8-element vectors.
template <int APPROX>
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ b,
                                                            uint16_t* __restrict__ y,
                                                            int64_t rows, int cols) {
  const int64_t cv = cols / 8;
  const int64_t total = rows * cv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += stride) {
    float v[8];
    load8<DT_BF16>(x, i, v);
    if (b) {
      float bb[8];
      load8<DT_BF16>(b, i % cv, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bb[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act<APPROX>(v[j]);
    store8<DT_BF16>(y, i, v);
  }
}

// Backward tiling: a 256-thread block owns 64 column-vectors (512 columns) x kStripRows rows;
// its 4 waves take interleaved rows (wave w: r0 + w, r0 + w + 4, ...), keep fp32 column sums in
// registers, reduce them across the waves through LDS and flush ONE float atomic per column per
// block. (A thread-per-column layout over 32-row strips issued 16x more atomics — 512 per
// column for 16 K rows — which serialised at the memory-side atomic unit: 172 us for GPT-2's
// 16384 x 3072 at 3x the traffic time.)
constexpr int kStripRows = 64;
constexpr int kColVecs = 64;

// grid: (ceil(cv / 64), ceil(rows / kStripRows)); block 256.
template <int APPROX>
__global__ void __launch_bounds__(256) bias_gelu_bwd_kernel(const uint16_t* __restrict__ dy,
                                                            const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ b,
                                                            uint16_t* __restrict__ dx,
                                                            float* __restrict__ db_ws,
                                                            int64_t rows, int cols) {
  __shared__ float red[3][kColVecs][8 + 1];
  const int64_t cv = cols / 8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kColVecs + lane;
  const bool live = c < cv;
  float bb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (b && live) load8<DT_BF16>(b, c, bb);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kStripRows;
  const int64_t r1 = r0 + kStripRows < rows ? r0 + kStripRows : rows;
  if (live) {
    int64_t r = r0 + w;
    for (; r + 12 < r1; r += 16) {   // 8 independent 16-B loads in flight per thread
      float v[4][8], g[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        load8<DT_BF16>(x, (r + 4 * u) * cv + c, v[u]);
        load8<DT_BF16>(dy, (r + 4 * u) * cv + c, g[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g[u][j] *= act_grad<APPROX>(v[u][j] + bb[j]);
          acc[j] += g[u][j];
        }
        store8<DT_BF16>(dx, (r + 4 * u) * cv + c, g[u]);
      }
    }
    for (; r < r1; r += 4) {
      float v[8], g[8];
      load8<DT_BF16>(x, r * cv + c, v);
      load8<DT_BF16>(dy, r * cv + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[j] *= act_grad<APPROX>(v[j] + bb[j]);
        acc[j] += g[j];
      }
      store8<DT_BF16>(dx, r * cv + c, g);
    }
  }
  if (!db_ws) return;
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w - 1][lane][j] = acc[j];
  }
  __syncthreads();
  if (w == 0 && live) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = acc[j] + red[0][lane][j] + red[1][lane][j] + red[2][lane][j];
      atomicAdd(db_ws + c * 8 + j, t);
    }
  }
}

}  // namespace dlbb

using namespace dlbb;

// approx: 0 = erf (torch default, reference models.py:182), 1 = tanh (GPT-2).
DLBB_API int dlbb_bias_gelu_fwd(const void* x, const void* bias, void* y, int64_t rows, int cols,
                                int approx, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (cols % 8 != 0) return hipErrorInvalidValue;
  const int grid = stream_grid(rows * (cols / 8), 256);
  const uint16_t* xp = static_cast<const uint16_t*>(x);
  const uint16_t* bp = static_cast<const uint16_t*>(bias);
  uint16_t* yp = static_cast<uint16_t*>(y);
  if (approx)
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<1>, dim3(grid), dim3(256), 0, stream, xp, bp, yp,
                       rows, cols);
  else
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<0>, dim3(grid), dim3(256), 0, stream, xp, bp, yp,
                       rows, cols);
  return hipGetLastError();
}

// db_ws: fp32 [cols] workspace, ZEROED by the caller on the same stream (or null: no dbias).
DLBB_API int dlbb_bias_gelu_bwd(const void* dy, const void* x, const void* bias, void* dx,
                                float* db_ws, int64_t rows, int cols, int approx,
                                hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (cols % 8 != 0) return hipErrorInvalidValue;
  const int64_t cv = cols / 8;
  const dim3 grid((cv + kColVecs - 1) / kColVecs, (rows + kStripRows - 1) / kStripRows);
  auto* g = static_cast<const uint16_t*>(dy);
  auto* xp = static_cast<const uint16_t*>(x);
  auto* bp = static_cast<const uint16_t*>(bias);
  auto* o = static_cast<uint16_t*>(dx);
  if (approx)
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<1>, grid, dim3(256), 0, stream, g, xp, bp, o, db_ws,
                       rows, cols);
  else
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<0>, grid, dim3(256), 0, stream, g, xp, bp, o, db_ws,
                       rows, cols);
  return hipGetLastError();
}
