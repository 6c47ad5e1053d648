// MFMA bf16 GEMM with fused epilogues, gfx950.
//
//   C[M,N] = epilogue( A[M,K] · B[N,K]^T )      A, B bf16 row-major (K contiguous), fp32 acc
//   epilogue: (+ bias[N]) -> (GELU erf | GELU tanh) -> (+ residual[M,N]) -> bf16 | fp32 store,
//             optional second store of the pre-activation (needed by the GELU backward).
//
// Replaces the reference's CPU `torch.matmul` for every tensor-parallel linear
// (ColumnParallelLinear models.py:47 — QKV and FFN-up, RowParallelLinear models.py:81 —
// attention-out and FFN-down) with the GELU (models.py:182) fused into the FFN-up epilogue and
// an fp32-output option that feeds an fp32 all-reduce directly (models.py:84).
// Weights are stored [out_features, in_features] (K-contiguous) so both MFMA operands are read
// row-wise: the natural layout for v_mfma_f32_16x16x32_bf16 (lane l holds A[l&15][8(l>>4)+j]
// and B[8(l>>4)+j][l&15]).
//
// Structure (CDNA guide §5 "standard MFMA GEMM main loop" + T1 + T2, 2-phase minimum of T3):
//   * 128x128x64 block tile, 256 threads = 4 waves in 2x2, 64x64 per wave = 4x4 MFMA tiles.
//   * global -> LDS with global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear LDS
//     destination); bank-conflict XOR swizzle applied on the SOURCE address and on the
//     ds_read (rule 21): LDS slot s of row r holds k-chunk s ^ (r & 7).
//   * two LDS buffers: the next K-tile streams in while the current one feeds the MFMAs;
//     one vmcnt(0) + barrier per K-tile.
//   * XCD-aware bijective workgroup remap (T1) + GROUP_M tile grouping for L2 reuse.
//   * M and N may be ragged (source rows clamped, stores masked); K % 64 == 0.
#include "common.h"

namespace dlbb {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = BM * BK * 2;            // 16 KiB per operand per buffer
constexpr int kGroupM = 8;

enum Epi : int {
  EPI_BIAS = 1,
  EPI_GELU_ERF = 2,
  EPI_GELU_TANH = 4,
  EPI_RESIDUAL = 8,
};

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const uint16_t* bias;
  const uint16_t* residual;
  uint16_t* preact;        // optional bf16 pre-activation output [M, N] (ldc)
  int64_t M, N, K;
  int64_t lda, ldb, ldc, ldr;
  int epi;
  int out_f32;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds16(const void* g, char* lds_base_wave_uniform) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(lds_base_wave_uniform), 16, 0,
                                   0);
}

// Stage a 128 x 64 bf16 tile of a K-contiguous matrix into LDS (16 KiB).
// Wave w issues 4 instructions; instruction i covers tile rows [w*32 + i*8, +8).
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ X, int64_t ld,
                                           int64_t row0, int64_t rows, int64_t k0, char* lds,
                                           int wave, int lane) {
  const int r_in = lane >> 3;                    // 0..7
  const int slot = lane & 7;                     // LDS 16 B slot
  const int chunk = slot ^ r_in;                 // source k-chunk (swizzle, rule 21)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int trow = wave * 32 + i * 8;
    int64_t gr = row0 + trow + r_in;
    gr = gr < rows ? gr : rows - 1;              // ragged edge: clamp (stores are masked)
    const uint16_t* src = X + gr * ld + k0 + chunk * 8;
    glds16(src, lds + trow * (BK * 2));
  }
}

__device__ __forceinline__ bf16x8 read_frag(const char* lds, int row, int chunk) {
  const int off = row * (BK * 2) + ((chunk ^ (row & 7)) << 4);
  return *reinterpret_cast<const bf16x8*>(lds + off);
}

__device__ __forceinline__ float apply_act(float v, int epi) {
  if (epi & EPI_GELU_ERF) return gelu_erf(v);
  if (epi & EPI_GELU_TANH) return gelu_tanh(v);
  return v;
}

__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_nt_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- workgroup -> tile: XCD-aware bijective remap, then GROUP_M swizzle
  const int64_t tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int64_t nwg = tiles_m * tiles_n;
  int64_t wid = blockIdx.x;
  {
    const int64_t q = nwg / 8, r = nwg % 8, x = wid % 8;
    wid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wid / 8;
  }
  const int64_t group_size = kGroupM * tiles_n;
  const int64_t group = wid / group_size;
  const int64_t first_m = group * kGroupM;
  const int64_t gm = (tiles_m - first_m) < kGroupM ? (tiles_m - first_m) : kGroupM;
  const int64_t tm = first_m + (wid % group_size) % gm;
  const int64_t tn = (wid % group_size) / gm;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  // buffer c: A at smem + c * 2 * kTileBytes, B right after it
  auto bufA = [&](int c) { return smem + c * 2 * kTileBytes; };
  auto bufB = [&](int c) { return smem + c * 2 * kTileBytes + kTileBytes; };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = a.K / BK;
  stage_tile(a.A, a.lda, m0, a.M, 0, bufA(0), wave, lane);
  stage_tile(a.B, a.ldb, n0, a.N, 0, bufB(0), wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage_tile(a.A, a.lda, m0, a.M, (kt + 1) * BK, bufA(cur ^ 1), wave, lane);
      stage_tile(a.B, a.ldb, n0, a.N, (kt + 1) * BK, bufB(cur ^ 1), wave, lane);
    }
    const char* la = bufA(cur);
    const char* lb = bufB(cur);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag(la, wm * 64 + i * 16 + fr, ks * 4 + fq);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag(lb, wn * 64 + j * 16 + fr, ks * 4 + fq);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: C/D map of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + reg
  const int epi = a.epi;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + fr;
    if (col >= a.N) continue;
    const float bias = (epi & EPI_BIAS) ? bf16_to_f32(a.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + fq * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] + bias;
        if (a.preact) a.preact[row * a.ldc + col] = f32_to_bf16(v);
        v = apply_act(v, epi);
        if (epi & EPI_RESIDUAL) v += bf16_to_f32(a.residual[row * a.ldr + col]);
        if (a.out_f32)
          static_cast<float*>(a.C)[row * a.ldc + col] = v;
        else
          static_cast<uint16_t*>(a.C)[row * a.ldc + col] = f32_to_bf16(v);
      }
    }
  }
}

}  // namespace dlbb

using namespace dlbb;

DLBB_API int dlbb_gemm_bf16_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                               const void* residual, int64_t ldr, void* preact, int epi,
                               int out_f32, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % BK != 0) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8) return hipErrorInvalidValue;          // 16-byte rows for glds
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    return hipErrorInvalidValue;
  if ((epi & EPI_BIAS) && !bias) return hipErrorInvalidValue;
  if ((epi & EPI_RESIDUAL) && !residual) return hipErrorInvalidValue;
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C,
             static_cast<const uint16_t*>(bias), static_cast<const uint16_t*>(residual),
             static_cast<uint16_t*>(preact), M, N, K, lda, ldb, ldc, ldr, epi, out_f32};
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm_bf16_nt_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kThreads),
                     4 * kTileBytes, stream, a);
  return hipGetLastError();
}
