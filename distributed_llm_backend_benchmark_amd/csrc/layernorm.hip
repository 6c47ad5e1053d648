// Fused residual-add + LayerNorm, forward and backward.
//
// Reference: nn.LayerNorm(hidden, dtype=bf16) at models.py:122,135,222 applied at
// models.py:156,177,236, with the residual adds at models.py:173,188. Per transformer block the
// reference reads/writes the [B,S,H] activation once for the add and twice more for the LN;
// here h = x + r, y = LN(h) is ONE pass: one wave owns a row, keeps it in registers
// (NV x 4 elements per lane, 8-byte vector I/O), computes two-pass fp32 statistics with wave
// shuffles, and writes both y and the new residual stream h.
//
// Backward recomputes x_hat from (h, mean, rstd), adds the incoming residual-stream gradient
// (fusing the residual branch), and produces dgamma/dbeta through per-workgroup fp32 partials
// + a column reduction (no float atomics, bitwise reproducible).
#include "common.h"

namespace dlbb {

struct LnFwdArgs {
  const uint16_t* x;      // [rows, cols] bf16
  const uint16_t* r;      // optional residual [rows, cols] bf16
  const void* gamma;      // [cols] bf16 or fp32 (param dtype)
  const void* beta;       // optional [cols]
  uint16_t* y;            // [rows, cols] bf16
  uint16_t* h_out;        // optional: x + r (bf16)
  float* mean;            // optional [rows]
  float* rstd;            // optional [rows]
  int64_t rows;
  int cols;
  float eps;
};

template <int PDT>
__device__ __forceinline__ float ldp(const void* p, int i) {
  return PDT == DT_F32 ? static_cast<const float*>(p)[i]
                       : bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
}

__device__ __forceinline__ void ld4(const uint16_t* p, int64_t i4, float (&v)[4]) {
  u16x4 r = reinterpret_cast<const u16x4*>(p)[i4];
  v[0] = bf16_to_f32(r[0]); v[1] = bf16_to_f32(r[1]);
  v[2] = bf16_to_f32(r[2]); v[3] = bf16_to_f32(r[3]);
}
__device__ __forceinline__ void st4(uint16_t* p, int64_t i4, const float (&v)[4]) {
  u16x4 r;
  r[0] = f32_to_bf16(v[0]); r[1] = f32_to_bf16(v[1]);
  r[2] = f32_to_bf16(v[2]); r[3] = f32_to_bf16(v[3]);
  reinterpret_cast<u16x4*>(p)[i4] = r;
}
__device__ __forceinline__ float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }

template <int PDT>
__device__ __forceinline__ void ldp4(const void* p, int c4, float (&v)[4]) {
  if constexpr (PDT == DT_F32) {
    const float4 t = reinterpret_cast<const float4*>(p)[c4];
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    ld4(static_cast<const uint16_t*>(p), c4, v);
  }
}

// NV = number of 4-element vectors per lane; cols == NV * 256. All loads of the row (x and r)
// are issued before any store (restrict-qualified: a store to h_out cannot alias the next
// loads, which had serialised the row into NV load round trips).
template <int NV, int PDT>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const uint16_t* __restrict__ xp = a.x;
  const uint16_t* __restrict__ rp = a.r;
  uint16_t* __restrict__ hp = a.h_out;
  uint16_t* __restrict__ yp = a.y;
  const int64_t base4 = row * (a.cols / 4);
  float v[NV][4], rr[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    ld4(xp, base4 + i * 64 + lane, v[i]);
    if (rp) ld4(rp, base4 + i * 64 + lane, rr[i]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (rp) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i][j] = round_bf16(v[i][j] + rr[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[i][j];
  }
  if (rp && hp) {
#pragma unroll
    for (int i = 0; i < NV; ++i) st4(hp, base4 + i * 64 + lane, v[i]);
  }
  const float inv_c = 1.0f / static_cast<float>(a.cols);
  const float mean = wave_sum(s) * inv_c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[i][j] - mean;
      ss += d * d;
    }
  const float rstd = rsqrtf(wave_sum(ss) * inv_c + a.eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float g[4], b[4] = {0.f, 0.f, 0.f, 0.f}, o[4];
    ldp4<PDT>(a.gamma, i * 64 + lane, g);
    if (a.beta) ldp4<PDT>(a.beta, i * 64 + lane, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + b[j];
    st4(yp, base4 + i * 64 + lane, o);
  }
  if (lane == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
}

// Generic fallback for any cols (two passes over global memory, scalar).
template <int PDT>
__global__ void __launch_bounds__(256) ln_fwd_generic(LnFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int64_t base = row * a.cols;
  float s = 0.f;
  for (int c = lane; c < a.cols; c += 64) {
    float v = bf16_to_f32(a.x[base + c]);
    if (a.r) {
      v = round_bf16(v + bf16_to_f32(a.r[base + c]));
      if (a.h_out) a.h_out[base + c] = f32_to_bf16(v);
    }
    s += v;
  }
  const float inv_c = 1.0f / static_cast<float>(a.cols);
  const float mean = wave_sum(s) * inv_c;
  float ss = 0.f;
  for (int c = lane; c < a.cols; c += 64) {
    float v = bf16_to_f32(a.x[base + c]);
    if (a.r) v = round_bf16(v + bf16_to_f32(a.r[base + c]));
    ss += (v - mean) * (v - mean);
  }
  const float rstd = rsqrtf(wave_sum(ss) * inv_c + a.eps);
  for (int c = lane; c < a.cols; c += 64) {
    float v = bf16_to_f32(a.x[base + c]);
    if (a.r) v = round_bf16(v + bf16_to_f32(a.r[base + c]));
    const float b = a.beta ? ldp<PDT>(a.beta, c) : 0.f;
    a.y[base + c] = f32_to_bf16((v - mean) * rstd * ldp<PDT>(a.gamma, c) + b);
  }
  if (lane == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
}

struct LnBwdArgs {
  const uint16_t* dy;     // [rows, cols]
  const uint16_t* h;      // LN input (x, or x + r) [rows, cols]
  const void* gamma;
  const float* mean;
  const float* rstd;
  const uint16_t* dres;   // optional gradient already flowing into h (residual stream)
  uint16_t* dx;           // [rows, cols]: d(LN input) (+ dres)
  float* dgamma_part;     // [gridDim.x, cols]
  float* dbeta_part;      // [gridDim.x, cols] (may be null)
  int64_t rows;
  int cols;
};

template <int NV, int PDT>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdArgs a) {
  __shared__ float red[2][4][NV * 256];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float dg[NV][4], db[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[i][j] = db[i][j] = 0.f;
  float gam[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gam[i][j] = ldp<PDT>(a.gamma, (i * 64 + lane) * 4 + j);
  const float inv_c = 1.0f / static_cast<float>(a.cols);
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
  const uint16_t* __restrict__ hp = a.h;
  const uint16_t* __restrict__ dyp = a.dy;
  const uint16_t* __restrict__ drp = a.dres;
  uint16_t* __restrict__ dxp = a.dx;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + w; row < a.rows; row += nwaves) {
    const int64_t base4 = row * (a.cols / 4);
    const float mu = a.mean[row], rs = a.rstd[row];
    float xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float hv[4], dyv[4];
      ld4(hp, base4 + i * 64 + lane, hv);
      ld4(dyp, base4 + i * 64 + lane, dyv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[i][j] = (hv[j] - mu) * rs;
        g[i][j] = dyv[j] * gam[i][j];
        s1 += g[i][j] * xh[i][j];
        s2 += g[i][j];
        dg[i][j] += dyv[j] * xh[i][j];
        db[i][j] += dyv[j];
      }
    }
    float dr[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i) {           // every load of the row before any store
      if (drp) {
        ld4(drp, base4 + i * 64 + lane, dr[i]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) dr[i][j] = 0.f;
      }
    }
    const float c1 = wave_sum(s1) * inv_c, c2 = wave_sum(s2) * inv_c;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] - xh[i][j] * c1 - c2) + dr[i][j];
      st4(dxp, base4 + i * 64 + lane, o);
    }
  }
  // cross-wave reduction of the dgamma/dbeta partials through LDS
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[0][w][(i * 64 + lane) * 4 + j] = dg[i][j];
      red[1][w][(i * 64 + lane) * 4 + j] = db[i][j];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < a.cols; c += 256) {
    const float sg = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    const float sb = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    a.dgamma_part[static_cast<int64_t>(blockIdx.x) * a.cols + c] = sg;
    if (a.dbeta_part) a.dbeta_part[static_cast<int64_t>(blockIdx.x) * a.cols + c] = sb;
  }
}

// Backward, pipelined (default). The kernel above is latency-bound at the GPT-2 shape (16384 x
// 768: 59 us per call, ~1.7 TB/s; profiles/r04_final/gpt2_kernel_stats_steady.csv:6): each wave
// owns 8 rows in sequence and every row is load -> wait -> two wave reductions -> store, with
// only 2 waves per SIMD to hide it. Here:
//   * WPB = 8 waves per block, so the same 512 partial rows of dgamma/dbeta come with twice the
//     resident waves (rows up to 1024 wide: wider rows keep the kernel above, whose register
//     footprint already limits it to 1-2 waves / SIMD);
//   * a two-deep register pipeline per wave: row r + stride's h / dy / dres / mean / rstd loads
//     are issued BEFORE row r's reductions and stores, so one row is always in flight while the
//     previous one is reduced (restrict pointers: the dx store of row r cannot alias them);
//   * the cross-wave dgamma / dbeta reduction reuses ONE [WPB][cols] LDS array (dgamma, then
//     dbeta); operands stay packed bf16 in registers until used (2 rows in flight <= 128 VGPRs).
template <int NV>
struct LnRow {                    // one row's operands, still packed bf16 (2 VGPRs per 4 values)
  u16x4 h[NV], dy[NV], dr[NV];
  float mu, rs;
};

template <int NV>
__device__ __forceinline__ void ln_row_load(const LnBwdArgs& a, const uint16_t* __restrict__ hp,
                                            const uint16_t* __restrict__ dyp,
                                            const uint16_t* __restrict__ drp, int64_t row,
                                            int lane, LnRow<NV>& r) {
  const int64_t base4 = row * (a.cols / 4);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    r.h[i] = reinterpret_cast<const u16x4*>(hp)[base4 + i * 64 + lane];
    r.dy[i] = reinterpret_cast<const u16x4*>(dyp)[base4 + i * 64 + lane];
  }
  if (drp) {
#pragma unroll
    for (int i = 0; i < NV; ++i) r.dr[i] = reinterpret_cast<const u16x4*>(drp)[base4 + i * 64 + lane];
  }
  r.mu = a.mean[row];
  r.rs = a.rstd[row];
}

template <int NV, int PDT, int WPB>
__global__ void __launch_bounds__(64 * WPB) ln_bwd_pipe_kernel(LnBwdArgs a) {
  __shared__ float red[WPB][NV * 256];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float dg[NV][4], db[NV][4], gam[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    ldp4<PDT>(a.gamma, i * 64 + lane, gam[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[i][j] = db[i][j] = 0.f;
  }
  const float inv_c = 1.0f / static_cast<float>(a.cols);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * WPB;
  const uint16_t* __restrict__ hp = a.h;
  const uint16_t* __restrict__ dyp = a.dy;
  const uint16_t* __restrict__ drp = a.dres;
  uint16_t* __restrict__ dxp = a.dx;
  int64_t row = static_cast<int64_t>(blockIdx.x) * WPB + w;
  LnRow<NV> cur;
  if (row < a.rows) ln_row_load<NV>(a, hp, dyp, drp, row, lane, cur);
  for (; row < a.rows; row += stride) {
    LnRow<NV> nxt;
    const bool more = row + stride < a.rows;
    if (more) ln_row_load<NV>(a, hp, dyp, drp, row + stride, lane, nxt);
    float xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float dyv = bf16_to_f32(cur.dy[i][j]);
        xh[i][j] = (bf16_to_f32(cur.h[i][j]) - cur.mu) * cur.rs;
        g[i][j] = dyv * gam[i][j];
        s1 += g[i][j] * xh[i][j];
        s2 += g[i][j];
        dg[i][j] += dyv * xh[i][j];
        db[i][j] += dyv;
      }
    const float c1 = wave_sum(s1) * inv_c, c2 = wave_sum(s2) * inv_c;
    const int64_t base4 = row * (a.cols / 4);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = cur.rs * (g[i][j] - xh[i][j] * c1 - c2) + (drp ? bf16_to_f32(cur.dr[i][j]) : 0.f);
      st4(dxp, base4 + i * 64 + lane, o);
    }
    if (more) cur = nxt;
  }
  // cross-wave reduction of the partials: dgamma, then dbeta through the same LDS array
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1 && !a.dbeta_part) break;
    if (pass == 1) __syncthreads();          // every wave has read the dgamma pass
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[w][(i * 64 + lane) * 4 + j] = pass ? db[i][j] : dg[i][j];
    __syncthreads();
    float* dst = (pass ? a.dbeta_part : a.dgamma_part) + static_cast<int64_t>(blockIdx.x) * a.cols;
    for (int c = threadIdx.x; c < a.cols; c += 64 * WPB) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < WPB; ++k) s += red[k][c];
      dst[c] = s;
    }
  }
}

// out[c] = sum_b part[b, c]  (fp32 accumulate, out in bf16 or fp32).
// 256 threads = 8 row groups x 32 columns: every wave reads 2 x 128 contiguous bytes per
// partial row, and each thread keeps 8 independent loads in flight (the naive
// one-thread-per-column loop was latency-bound: 118 us for 512 x 768 partials).
template <int DTO>
__global__ void __launch_bounds__(256) col_reduce_kernel(const float* __restrict__ part_g,
                                                         const float* __restrict__ part_b,
                                                         int nparts, int cols, void* out_g,
                                                         void* out_b, int accumulate) {
  // blockIdx.y: 0 = dgamma, 1 = dbeta (one launch for both)
  const float* part = blockIdx.y ? part_b : part_g;
  void* out = blockIdx.y ? out_b : out_g;
  __shared__ float red[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  float s = 0.f;
  if (c < cols) {
    int b = ty;
    for (; b + 56 < nparts; b += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[static_cast<int64_t>(b + 8 * u) * cols + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nparts; b += 8) s += part[static_cast<int64_t>(b) * cols + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][tx];
    auto* o = static_cast<typename Elem<DTO>::T*>(out);
    if (accumulate) t += Elem<DTO>::ld(o, c);     // into an existing gradient (grad sinks)
    Elem<DTO>::st(o, c, t);
  }
}

// Block-per-row forward for wide rows (cols = T * 8 * VPT): 16-byte vectors, the row held in
// registers, statistics reduced across the block's waves through LDS. Gives rows x T/64 waves
// of parallelism where the wave-per-row kernel only has `rows` waves.
template <int T, int VPT, int PDT>
__global__ void __launch_bounds__(T) ln_fwd_row_kernel(LnFwdArgs a) {
  __shared__ float red[2][T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = blockIdx.x;
  const int64_t base8 = row * (a.cols / 8);
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int64_t c8 = i * T + threadIdx.x;
    load8<DT_BF16>(a.x, base8 + c8, v[i]);
    if (a.r) {
      float rr[8];
      load8<DT_BF16>(a.r, base8 + c8, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = round_bf16(v[i][j] + rr[j]);
      if (a.h_out) store8<DT_BF16>(a.h_out, base8 + c8, v[i]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[i][j];
  }
  s = wave_sum(s);
  if (lane == 0) red[0][w] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < T / 64; ++k) tot += red[0][k];
  const float inv_c = 1.0f / static_cast<float>(a.cols);
  const float mean = tot * inv_c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[i][j] - mean;
      ss += d * d;
    }
  ss = wave_sum(ss);
  if (lane == 0) red[1][w] = ss;
  __syncthreads();
  float vt = 0.f;
#pragma unroll
  for (int k = 0; k < T / 64; ++k) vt += red[1][k];
  const float rstd = rsqrtf(vt * inv_c + a.eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c8 = i * T + threadIdx.x;
    float g[8], b[8], o[8];
    if constexpr (PDT == DT_F32) {
      load8<DT_F32>(a.gamma, c8, g);
      if (a.beta) load8<DT_F32>(a.beta, c8, b);
    } else {
      load8<DT_BF16>(a.gamma, c8, g);
      if (a.beta) load8<DT_BF16>(a.beta, c8, b);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + (a.beta ? b[j] : 0.f);
    store8<DT_BF16>(a.y, base8 + c8, o);
  }
  if (threadIdx.x == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
}

template <int T, int VPT, int PDT>
static hipError_t fwd_row(const LnFwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((ln_fwd_row_kernel<T, VPT, PDT>), dim3(a.rows), dim3(T), 0, s, a);
  return hipGetLastError();
}

// returns hipErrorNotSupported when no (T, VPT) instance fits
template <int PDT>
static hipError_t fwd_row_dispatch(const LnFwdArgs& a, hipStream_t s) {
  if (a.cols % 8 != 0) return hipErrorNotSupported;
  const int nv = a.cols / 8;
#define ROW(T, V) if (nv == T * V) return fwd_row<T, V, PDT>(a, s);
  ROW(256, 1) ROW(256, 2) ROW(256, 3) ROW(256, 4) ROW(256, 5) ROW(256, 6) ROW(256, 8)
  ROW(128, 3) ROW(128, 5) ROW(128, 7) ROW(64, 5) ROW(64, 7)
#undef ROW
  return hipErrorNotSupported;
}

template <int NV, int PDT>
static hipError_t fwd_nv(const LnFwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((ln_fwd_kernel<NV, PDT>), dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int PDT>
static hipError_t fwd_dispatch(const LnFwdArgs& a, hipStream_t s) {
  if (a.cols >= 2048) {
    hipError_t e = fwd_row_dispatch<PDT>(a, s);
    if (e != hipErrorNotSupported) return e;
  }
  if (a.cols % 256 == 0) {
    switch (a.cols / 256) {
      case 1: return fwd_nv<1, PDT>(a, s);
      case 2: return fwd_nv<2, PDT>(a, s);
      case 3: return fwd_nv<3, PDT>(a, s);
      case 4: return fwd_nv<4, PDT>(a, s);
      case 5: return fwd_nv<5, PDT>(a, s);
      case 6: return fwd_nv<6, PDT>(a, s);
      case 8: return fwd_nv<8, PDT>(a, s);
      case 10: return fwd_nv<10, PDT>(a, s);
      case 12: return fwd_nv<12, PDT>(a, s);
      case 16: return fwd_nv<16, PDT>(a, s);
      case 20: return fwd_nv<20, PDT>(a, s);
      case 24: return fwd_nv<24, PDT>(a, s);
      case 32: return fwd_nv<32, PDT>(a, s);
      default: break;
    }
  }
  hipLaunchKernelGGL((ln_fwd_generic<PDT>), dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Partial rows of the pipelined backward: one block per WPB rows, at most 512 blocks (one
// resident round at <= 128 VGPRs: 4 waves / SIMD).
static inline int bwd_pipe_grid(int64_t rows, int wpb) {
  int64_t g = (rows + wpb - 1) / wpb;
  if (g > 512) g = 512;
  return static_cast<int>(g < 1 ? 1 : g);
}

template <int NV, int PDT>
static hipError_t bwd_nv(const LnBwdArgs& a, int grid, hipStream_t s) {
  if constexpr (NV <= 4) {        // the pipelined kernel (rows up to 1024 wide)
    hipLaunchKernelGGL((ln_bwd_pipe_kernel<NV, PDT, 8>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((ln_bwd_kernel<NV, PDT>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dlbb

using namespace dlbb;

DLBB_API int dlbb_layernorm_fwd(const void* x, const void* residual, const void* gamma,
                                const void* beta, int param_dtype, void* y, void* h_out,
                                float* mean, float* rstd, int64_t rows, int cols, float eps,
                                hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (cols <= 0 || cols % 4 != 0) return hipErrorInvalidValue;
  LnFwdArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(residual), gamma,
              beta, static_cast<uint16_t*>(y), static_cast<uint16_t*>(h_out), mean, rstd,
              rows, cols, eps};
  return param_dtype == DT_F32 ? fwd_dispatch<DT_F32>(a, stream)
                               : fwd_dispatch<DT_BF16>(a, stream);
}

// Supported widths for the backward: cols in {256,512,768,1024,1536,2048,3072,4096}
// (LDS: 2 x 4 x cols floats <= 128 KiB). Returns the number of partial rows the caller
// must provide via `max_parts` query: call with dx == nullptr to get the grid size.
DLBB_API int dlbb_layernorm_bwd_grid(int64_t rows) {
  int64_t g = (rows + 3) / 4;
  if (g > 512) g = 512;
  return static_cast<int>(g < 1 ? 1 : g);
}

DLBB_API int dlbb_layernorm_bwd(const void* dy, const void* h, const void* gamma, int param_dtype,
                                const float* mean, const float* rstd, const void* dres, void* dx,
                                float* part_ws, void* dgamma, void* dbeta, int64_t rows,
                                int cols, int accumulate, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (cols % 256 != 0) return hipErrorInvalidValue;
  // partial rows actually used (<= dlbb_layernorm_bwd_grid(rows), the caller's ws size)
  const int grid = cols <= 1024 ? bwd_pipe_grid(rows, 8)
                                                         : dlbb_layernorm_bwd_grid(rows);
  float* pg = part_ws;
  float* pb = dbeta ? part_ws + static_cast<int64_t>(grid) * cols : nullptr;
  LnBwdArgs a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(h), gamma, mean,
              rstd, static_cast<const uint16_t*>(dres), static_cast<uint16_t*>(dx), pg, pb,
              rows, cols};
  hipError_t e = hipErrorInvalidValue;
#define LB(NV)                                                                   \
  case NV:                                                                       \
    e = param_dtype == DT_F32 ? bwd_nv<NV, DT_F32>(a, grid, stream)              \
                              : bwd_nv<NV, DT_BF16>(a, grid, stream);            \
    break;
  switch (cols / 256) {
    LB(1) LB(2) LB(3) LB(4) LB(6) LB(8) LB(12) LB(16)
    default: return hipErrorInvalidValue;
  }
#undef LB
  if (e != hipSuccess) return e;
  const dim3 cg((cols + 31) / 32, dbeta ? 2 : 1), cb(256);
  if (param_dtype == DT_F32)
    hipLaunchKernelGGL((col_reduce_kernel<DT_F32>), cg, cb, 0, stream, pg, pb, grid, cols, dgamma,
                       dbeta, accumulate);
  else
    hipLaunchKernelGGL((col_reduce_kernel<DT_BF16>), cg, cb, 0, stream, pg, pb, grid, cols,
                       dgamma, dbeta, accumulate);
  return hipGetLastError();
}
