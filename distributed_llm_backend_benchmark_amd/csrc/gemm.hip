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
#include <cstdlib>
#include <utility>

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
  // dgrad through a GELU: C = (A · B) * gelu'(u), u = the forward pre-activation [M, N] passed
  // in `residual` / ldr (the GELU backward fused into the producing GEMM's epilogue)
  EPI_DGELU_ERF = 16,
  EPI_DGELU_TANH = 32,
};
constexpr int EPI_READS_R = EPI_RESIDUAL | EPI_DGELU_ERF | EPI_DGELU_TANH;

__device__ __forceinline__ float apply_r(float v, float r, int epi) {
  if (epi & EPI_DGELU_TANH) return v * gelu_tanh_grad(r);
  if (epi & EPI_DGELU_ERF) return v * gelu_erf_grad(r);
  return v + r;
}

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
  int vec_ok;              // 16-B aligned C / residual / preact / bias rows (vector epilogue)
  int kt_split;            // NN split-K (gridDim.y > 1): K-tiles per split; split s writes fp32
                           // partials to C + s * M * ldc
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds16(const void* g, char* lds_base_wave_uniform) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(lds_base_wave_uniform), 16, 0,
                                   0);
}

// Stage a 128 x 64 bf16 tile of a K-contiguous matrix into LDS (16 KiB).
// Wave w issues 4 instructions; instruction i covers tile rows [w*32 + i*8, +8).
__device__ __forceinline__ int perm_brow(int x) {
  return (x & ~63) | (((x >> 2) & 3) << 4) | (((x >> 4) & 3) << 2) | (x & 3);
}

template <bool PERM>   // PERM: B rows in the perm_brow order (swapped-operand epilogue)
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ X, int64_t ld,
                                           int64_t row0, int64_t rows, int64_t k0, char* lds,
                                           int wave, int lane) {
  const int r_in = lane >> 3;                    // 0..7
  const int slot = lane & 7;                     // LDS 16 B slot
  const int chunk = slot ^ r_in;                 // source k-chunk (swizzle, rule 21)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int trow = wave * 32 + i * 8;
    int64_t gr = row0 + (PERM ? perm_brow(trow + r_in) : trow + r_in);
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


// ---------------------------------------------------------------------------------------
// 256 x 256 x 64 tile, 512 threads (8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave),
// one workgroup per CU (2 x 64 KiB LDS buffers). Each K-tile is computed in 4 phases, one
// 64 x 32 output quadrant per wave per phase (16 MFMA 16x16x32). LDS is staged in 4 sections
// of 128 rows x 64 k (16 KiB = 2 global_load_lds_dwordx4 per wave) cut along what the phases
// read: SA0 = A rows of m-quadrant 0 of both wave rows, SB0 / SB1 = B rows of n-quadrant 0 / 1
// of all four wave columns, SA1 = A rows of m-quadrant 1. Phase p of tile t issues section p of
// tile t+1, so sections stay 3-4 phases in flight; the waits are COUNTED (vmcnt(4): two
// sections may stay outstanding) and the barrier is a raw s_barrier so hipcc does not drain the
// LDS-DMA queue (CDNA guide §5 "Pipelining across barriers", T3/T4, T5).
//   phase 1: issue SA0' | read A(mq0), B(nq0) | 16 MFMA (mq0,nq0) | vmcnt(4) (SB1 landed)
//   phase 2: issue SB0' | read B(nq1)         | 16 MFMA (mq0,nq1) | vmcnt(4) (SA1 landed)
//   phase 3: issue SB1' | read A(mq1)         | 16 MFMA (mq1,nq1) |
//   phase 4: issue SA1' | (no reads)          | 16 MFMA (mq1,nq0) | vmcnt(4) (SA0',SB0' landed)
// WAR: tile t+1 overwrites the buffer tile t-1 read; its last reads (phase 3) precede the
// phase-4 barrier every wave has passed before issuing tile t+1's sections.
constexpr int BM2 = 256, BN2 = 256;
constexpr int kThreads2 = 512;
constexpr int kTile2Bytes = BM2 * BK * 2;      // 32 KiB per operand
constexpr int kBuf2Bytes = 2 * kTile2Bytes;    // A + B = 64 KiB

// tile row of 8-row group g (0..15) of section `sec` (0 = SA0, 1 = SB0, 2 = SB1, 3 = SA1)
__device__ __forceinline__ int section_row(int sec, int g) {
  if (sec == 0) return g < 8 ? g * 8 : 128 + (g - 8) * 8;
  if (sec == 3) return 64 + (g < 8 ? g * 8 : 128 + (g - 8) * 8);
  return (sec == 2 ? 32 : 0) + (g >> 2) * 64 + (g & 3) * 8;
}

// B rows are staged PERMUTED inside each 64-row block: LDS row (j*16 + t) holds output column
// (t>>2)*16 + j*4 + (t&3) (bits [3:2] and [5:4] of the row index swapped). With the MFMA
// operands swapped (D = W_rows x X_rows^T, so each lane holds 4 consecutive columns of one
// output row) the four n-tiles j of a wave then give every lane 16 CONSECUTIVE columns of one
// row: the epilogue stores 2 x 16 B per lane and row block instead of 16 scattered 2-B stores.

template <bool PERM>
__device__ __forceinline__ void stage_section(const uint16_t* __restrict__ X, int64_t ld,
                                              int64_t row0, int64_t rows, int64_t k0,
                                              char* tile, int sec, int wave, int lane) {
  const int r_in = lane >> 3;
  const int chunk = (lane & 7) ^ r_in;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int trow = section_row(sec, wave * 2 + i);
    int64_t gr = row0 + (PERM ? perm_brow(trow + r_in) : trow + r_in);
    gr = gr < rows ? gr : rows - 1;
    glds16(X + gr * ld + k0 + chunk * 8, tile + trow * (BK * 2));
  }
}

__device__ __forceinline__ void stage_next(const GemmArgs& a, int64_t m0, int64_t n0,
                                           int64_t k0, char* buf, int sec, int wave, int lane) {
  if (sec == 0 || sec == 3)
    stage_section<false>(a.A, a.lda, m0, a.M, k0, buf, sec, wave, lane);
  else
    stage_section<true>(a.B, a.ldb, n0, a.N, k0, buf + kTile2Bytes, sec, wave, lane);
}

#define DLBB_WAIT_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
#define DLBB_BARRIER()                                       \
  do {                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       \
    __builtin_amdgcn_s_barrier();                            \
  } while (0)

template <int MQ, int NQ>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[8][4], const bf16x8 (&af)[2][4],
                                              const bf16x8 (&bf)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[MQ * 4 + i][NQ * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            bf[ks][j], af[ks][i], acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void read_a(const char* tileA, int wr, int mq, int fr, int fq,
                                       bf16x8 (&af)[2][4]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[ks][i] = read_frag(tileA, wr * 128 + mq * 64 + i * 16 + fr, ks * 4 + fq);
}

__device__ __forceinline__ void read_b(const char* tileB, int wc, int nq, int fr, int fq,
                                       bf16x8 (&bf)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bf[ks][j] = read_frag(tileB, wc * 64 + nq * 32 + j * 16 + fr, ks * 4 + fq);
}

struct Tile256 {
  int64_t m0, n0;
};

// virtual workgroup id -> output tile: XCD-aware bijective remap (T1), then GROUP_M ordering
// (BNT: tile width, 256 or 192)
template <int BNT = BN2>
__device__ __forceinline__ Tile256 tile_of(const GemmArgs& a, int vb) {
  // 32-bit index math (tile counts < 2^31): 64-bit divisions cost SGPRs and SALU time
  const int tiles_m = static_cast<int>((a.M + BM2 - 1) / BM2);
  const int tiles_n = static_cast<int>((a.N + BNT - 1) / BNT);
  const int nwg = tiles_m * tiles_n;
  const int q = nwg >> 3, r = nwg & 7, x = vb & 7;
  const int wid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (vb >> 3);
  const int gmx = kGroupM;
  const int group_size = gmx * tiles_n;
  const int group = wid / group_size;
  const int first_m = group * gmx;
  const int gm = (tiles_m - first_m) < gmx ? (tiles_m - first_m) : gmx;
  const int in_group = wid - group * group_size;
  return Tile256{static_cast<int64_t>(first_m + in_group % gm) * BM2,
                 static_cast<int64_t>(in_group / gm) * BNT};
}

// Deep-pipeline prologue: all four sections of K-tile 0 and S0, S1 of K-tile 1 (6 sections).
__device__ __forceinline__ void deep_prologue(const GemmArgs& a, int64_t m0, int64_t n0,
                                              int64_t nk, char* smem, int wave, int lane) {
  stage_next(a, m0, n0, 0, smem, 0, wave, lane);
  stage_next(a, m0, n0, 0, smem, 1, wave, lane);
  stage_next(a, m0, n0, 0, smem, 2, wave, lane);
  stage_next(a, m0, n0, 0, smem, 3, wave, lane);
  if (nk > 1) {
    stage_next(a, m0, n0, BK, smem + kBuf2Bytes, 0, wave, lane);
    stage_next(a, m0, n0, BK, smem + kBuf2Bytes, 1, wave, lane);
  }
}

  // Deep pipeline: a section is restaged for tile t+2 into the CURRENT buffer as soon as
  // tile t's last read of it is two phases old, so four sections (one whole K-tile) stay in
  // flight instead of two, with the same 128 KiB of LDS. Issue schedule in tile t:
  //   ph1: S2(t+1)  ph2: S3(t+1)  ph3: S0(t+2)  ph4: S1(t+2)
  // (S0 = A mq0, S1 = B nq0, S2 = B nq1, S3 = A mq1; last reads of tile t: S0,S1 @ph1,
  // S2 @ph2, S3 @ph3.) Each phase: ds_reads first, then the section issue, the counted wait
  // for the section read NEXT phase (retired before this phase's first barrier: with the
  // wave rows staggered by one barrier that is the latest safe point), barrier, lgkmcnt(0),
  // 16 MFMA, barrier.
// Entry: the prologue's S0(0), S1(0) retired and a barrier passed; the lagging wave row has
// taken its extra barrier. Exit: every LDS read done; the wave rows are still staggered.
__device__ __forceinline__ void deep_mainloop(const GemmArgs& a, f32x4 (&acc)[8][4], int64_t m0,
                                              int64_t n0, int64_t nk, char* smem, int wave,
                                              int lane) {
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[2][4], b0[2][2], b1[2][2];
  for (int64_t t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * kBuf2Bytes;
    char* nxt = smem + ((t + 1) & 1) * kBuf2Bytes;
    const bool m1 = t + 1 < nk, m2 = t + 2 < nk;
    // phase 1: MFMA (mq0, nq0); wait S2(t)
    read_a(cur, wr, 0, fr, fq, af);
    read_b(cur + kTile2Bytes, wc, 0, fr, fq, b0);
    if (m1) { stage_next(a, m0, n0, (t + 1) * BK, nxt, 2, wave, lane); DLBB_WAIT_VM(8); }
    else DLBB_WAIT_VM(2);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma_quadrant<0, 0>(acc, af, b0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // phase 2: MFMA (mq0, nq1); wait S3(t)
    read_b(cur + kTile2Bytes, wc, 1, fr, fq, b1);
    if (m1) { stage_next(a, m0, n0, (t + 1) * BK, nxt, 3, wave, lane); DLBB_WAIT_VM(8); }
    else DLBB_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma_quadrant<0, 1>(acc, af, b1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // phase 3: MFMA (mq1, nq1); restage S0 for tile t+2
    read_a(cur, wr, 1, fr, fq, af);
    if (m2) stage_next(a, m0, n0, (t + 2) * BK, cur, 0, wave, lane);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma_quadrant<1, 1>(acc, af, b1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // phase 4: MFMA (mq1, nq0); restage S1 for tile t+2; wait S0(t+1), S1(t+1)
    if (m2) { stage_next(a, m0, n0, (t + 2) * BK, cur, 1, wave, lane); DLBB_WAIT_VM(8); }
    else if (m1) DLBB_WAIT_VM(4);
    else DLBB_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_quadrant<1, 0>(acc, af, b0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
}

// Epilogue of one 256^2 tile (global stores from registers; no LDS, no barriers).
// Epilogue of one wave's MI*16 x 64 output block at (row0, col0) — global stores from
// registers (no LDS, no barriers). Requires the swapped-operand MFMA + perm_brow B staging.
// JSWAP (NN kernel, transposed-read B image): lanes with fq odd hold column (j ^ 1)*4 + r in
// acc[i][j][r] (see read_b_nn), so the 4-column groups are swapped pairwise back into order.
template <int MI, bool JSWAP = false>
__device__ __forceinline__ void store_tile(const GemmArgs& a, const f32x4 (&acc)[MI][4],
                                           int64_t row0, int64_t col0, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  const bool odd = JSWAP && (fq & 1);
  // epilogue. Lane (fr, fq) holds output row rbase + i*16 + fr, columns cbase .. cbase+15
  // (acc[i][j][r] = column j*4 + r, see perm_brow).
  const int epi = a.epi;
  const int64_t cbase = col0 + fq * 16;
  const int cols_left = static_cast<int>(a.N - cbase < 16 ? a.N - cbase : 16);
  if (cols_left <= 0) return;
  const int64_t rbase = row0 + fr;
  const int rows_left = static_cast<int>(a.M - rbase);     // rows i*16 < rows_left are valid
  const bool vec = a.vec_ok && cols_left == 16;
  float bias[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) bias[c] = 0.f;
  if (epi & EPI_BIAS) {
    if (vec) {
      const u16x8* bp = reinterpret_cast<const u16x8*>(a.bias + cbase);
      const u16x8 b0v = bp[0], b1v = bp[1];
#pragma unroll
      for (int c = 0; c < 8; ++c) { bias[c] = bf16_to_f32(b0v[c]); bias[8 + c] = bf16_to_f32(b1v[c]); }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) if (c < cols_left) bias[c] = bf16_to_f32(a.bias[cbase + c]);
    }
  }
  const int ldc = static_cast<int>(a.ldc), ldr = static_cast<int>(a.ldr);
  float* cf = static_cast<float*>(a.C) + rbase * a.ldc + cbase;
  uint16_t* cb = static_cast<uint16_t*>(a.C) + rbase * a.ldc + cbase;
  uint16_t* pb = a.preact ? a.preact + rbase * a.ldc + cbase : nullptr;
  const uint16_t* rb = (epi & EPI_READS_R) ? a.residual + rbase * a.ldr + cbase : nullptr;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    if (i * 16 >= rows_left) break;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[j * 4 + r] = (odd ? acc[i][j ^ 1][r] : acc[i][j][r]) + bias[j * 4 + r];
    const int oc = i * 16 * ldc, orr = i * 16 * ldr;
    if (vec) {
      if (pb) {
        u16x8 p0, p1;
#pragma unroll
        for (int c = 0; c < 8; ++c) { p0[c] = f32_to_bf16(v[c]); p1[c] = f32_to_bf16(v[8 + c]); }
        reinterpret_cast<u16x8*>(pb + oc)[0] = p0;
        reinterpret_cast<u16x8*>(pb + oc)[1] = p1;
      }
      if (epi & (EPI_GELU_ERF | EPI_GELU_TANH)) {
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = apply_act(v[c], epi);
      }
      if (rb) {
        const u16x8 r0 = reinterpret_cast<const u16x8*>(rb + orr)[0];
        const u16x8 r1 = reinterpret_cast<const u16x8*>(rb + orr)[1];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = apply_r(v[c], bf16_to_f32(r0[c]), epi);
          v[8 + c] = apply_r(v[8 + c], bf16_to_f32(r1[c]), epi);
        }
      }
      if (a.out_f32) {
        float4* o = reinterpret_cast<float4*>(cf + oc);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      } else {
        u16x8 o0, o1;
#pragma unroll
        for (int c = 0; c < 8; ++c) { o0[c] = f32_to_bf16(v[c]); o1[c] = f32_to_bf16(v[8 + c]); }
        reinterpret_cast<u16x8*>(cb + oc)[0] = o0;
        reinterpret_cast<u16x8*>(cb + oc)[1] = o1;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (c >= cols_left) break;
        float x = v[c];
        if (pb) pb[oc + c] = f32_to_bf16(x);
        x = apply_act(x, epi);
        if (rb) x = apply_r(x, bf16_to_f32(rb[orr + c]), epi);
        if (a.out_f32) cf[oc + c] = x; else cb[oc + c] = f32_to_bf16(x);
      }
    }
  }
}
template <bool JSWAP = false>
__device__ __forceinline__ void store_tile_256(const GemmArgs& a, const f32x4 (&acc)[8][4],
                                               int64_t m0, int64_t n0, int wave, int lane) {
  store_tile<8, JSWAP>(a, acc, m0 + (wave >> 2) * 128, n0 + (wave & 3) * 64, lane);
}

// 128 x 128 x 64 tile, 4 waves (2 x 2, 64 x 64 each), two LDS buffers, 2 workgroups per CU:
// the small-grid path (fewer than ~192 256^2 tiles).
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
  stage_tile<false>(a.A, a.lda, m0, a.M, 0, bufA(0), wave, lane);
  stage_tile<true>(a.B, a.ldb, n0, a.N, 0, bufB(0), wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage_tile<false>(a.A, a.lda, m0, a.M, (kt + 1) * BK, bufA(cur ^ 1), wave, lane);
      stage_tile<true>(a.B, a.ldb, n0, a.N, (kt + 1) * BK, bufB(cur ^ 1), wave, lane);
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: swapped operands + permuted B rows -> 16 consecutive columns per lane
  store_tile<4>(a, acc, m0 + wm * 64, n0 + wn * 64, lane);
}


// 256^2 tile on the deep pipeline (deep_prologue / deep_mainloop, wave rows staggered by one
// barrier): the general-contract fallback of the 256^2 grid (ragged N % 64 / M % 8, 64-bit
// panel offsets) where the ping-pong's buffer-resource staging does not apply. (Round-1/2
// lock-step / staggered / early-issue schedules and the persistent deep form were removed in
// round 6: never faster than this or the ping-pong.)
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_deep(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2;
  const Tile256 tl = tile_of(a, static_cast<int>(blockIdx.x));
  const int64_t m0 = tl.m0, n0 = tl.n0;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = a.K / BK;
  const bool lag = wr == 1;
  deep_prologue(a, m0, n0, nk, smem, wave, lane);
  if (nk > 1) DLBB_WAIT_VM(8); else DLBB_WAIT_VM(4);   // retire S0(0), S1(0)
  __builtin_amdgcn_s_barrier();
  if (lag) __builtin_amdgcn_s_barrier();
  deep_mainloop(a, acc, m0, n0, nk, smem, wave, lane);
  if (!lag) __builtin_amdgcn_s_barrier();
  store_tile_256(a, acc, m0, n0, wave, lane);
}

// ---------------------------------------------------------------------------------------
// Row clamping is per 8-row group and wave-uniform (host contract: M % 8 == 0, N % 64 == 0),
// so each load is buffer_load_dwordx4 ... lds with the tile's operand base in a buffer
// resource (SGPRs), the group's row + k offset in soffset (SGPR) and one per-lane 32-bit
// offset (aoff / boff: the lane's row within the group and its swizzled k-chunk) — two VGPRs
// of addressing for all sixteen loads, nothing 64-bit per load for hipcc to hoist into VGPRs.
// perm_brow(trow + r) == perm_brow(trow) | perm_brow(r) for trow % 8 == 0 (the bits it swaps
// are split between the two), and a 64-row block of B is wholly in or out. Every access is in
// bounds by construction (clamped rows), so the resource carries no range limit.
__device__ __forceinline__ void bldsx4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                       char* lds_base_wave_uniform) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(lds_base_wave_uniform), 16, voff, soff,
                                           0, 0);
}

// Ping-pong with all 160 KiB of LDS (set_stagger(6)): A double-buffered (2 x 32 KiB), B triple-
// buffered (3 x 32 KiB), and each A buffer refilled in halves as soon as the wave row that reads
// that half is done with it. The A rows [0,128) are read only by wave row 0 (intervals 2u) and
// rows [128,256) only by wave row 1 (intervals 2u+1), so every load gets 3-4 intervals to land
// instead of 2:
//   interval 2u   (row 0 reads tile u):  row 0 issues A-hi(u+1) and B(u+2)
//   interval 2u+1 (row 1 reads tile u):  row 1 issues A-lo(u+2)
// Waits (counted, oldest first): row 0 ends interval 2u with A-hi(u) retired (row 1 reads it
// next) and interval 2u+1 with B(u+1) retired; row 1 ends 2u+1 with A-lo(u+1) retired.
// WAR: A-hi(u+1) replaces A-hi(u-1) (last read by row 1 in 2u-1), B(u+2) replaces B(u-1)
// (2u-1), A-lo(u+2) replaces A-lo(u) (row 0, 2u) — each behind the barrier that closes the read.
constexpr int kPP6Lds = 2 * kTile2Bytes + 3 * kTile2Bytes;  // 160 KiB

__device__ __forceinline__ void stage_a_half(__amdgpu_buffer_rsrc_t ra, uint32_t lda2, int rows_a,
                                             uint32_t k2, char* abuf, int half, int w4,
                                             uint32_t aoff) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {            // 16 groups of 8 rows, 4 per wave
    const int trow = half * 128 + (i * 4 + w4) * 8;
    const int g = trow < rows_a - 8 ? trow : rows_a - 8;
    bldsx4(ra, aoff, static_cast<uint32_t>(g) * lda2 + k2, abuf + trow * (BK * 2));
  }
}

// piece I (0..3) of stage_a_half: one wave-instruction (8 rows x 128 B)
template <int I>
__device__ __forceinline__ void stage_a_piece(__amdgpu_buffer_rsrc_t ra, uint32_t lda2,
                                              int rows_a, uint32_t k2, char* abuf, int half,
                                              int w4, uint32_t aoff) {
  const int trow = half * 128 + (I * 4 + w4) * 8;
  const int g = trow < rows_a - 8 ? trow : rows_a - 8;
  bldsx4(ra, aoff, static_cast<uint32_t>(g) * lda2 + k2, abuf + trow * (BK * 2));
}

// I0 / I1: the slice [I0, I1) of the 8 instructions (0..3 = tile rows [0, 128), 4..7 = rows
// [128, 256)) — the balanced ping-pong splits a B tile between the two wave rows
template <int I0 = 0, int I1 = 8>
__device__ __forceinline__ void stage_b(__amdgpu_buffer_rsrc_t rb, uint32_t ldb2, int rows_b,
                                        uint32_t k2, char* bbuf, int w4, uint32_t boff) {
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int trow = (i * 4 + w4) * 8;
    const int g = (trow & ~63) < rows_b ? perm_brow(trow) : (perm_brow(trow) & 63);
    bldsx4(rb, boff, static_cast<uint32_t>(g) * ldb2 + k2, bbuf + trow * (BK * 2));
  }
}

__device__ __forceinline__ void read_split(const char* abuf, const char* bbuf, int wr, int wc,
                                           int fr, int fq, bf16x8 (&af)[2][8],
                                           bf16x8 (&bf)[2][4]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int i = 0; i < 8; ++i) af[ks][i] = read_frag(abuf, wr * 128 + i * 16 + fr, ks * 4 + fq);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[ks][j] = read_frag(bbuf, wc * 64 + j * 16 + fr, ks * 4 + fq);
  }
}

// all 64 MFMAs of one wave's 128 x 64 outputs for one K-tile (k outer, so the two MFMAs into
// one accumulator are 32 instructions apart)
__device__ __forceinline__ void mfma_full(f32x4 (&acc)[8][4], const bf16x8 (&af)[2][8],
                                          const bf16x8 (&bf)[2][4]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[i][j], 0,
                                                            0, 0);
}

// ---------------------------------------------------------------------------------------
// NN operand B (dgrad: dX[M, N] = dY[M, K] · W[K, N], W stored [K][N] row-major — the reduction
// runs along W's ROWS). One K-tile of B = 64 k-rows x 256 columns, staged as two [64][128]
// images (256-B rows, 16 KiB each: image c holds tile columns [128c, 128c + 128)) by the same
// buffer_load ... lds DMA (one instruction = 4 k-rows x 256 B), and read as MFMA fragments with
// ds_read_b64_tr_b16 (CDNA guide T10), so no transposed copy of W is ever made.
// Fragment (ks, j) of wave column wc, lane (fq, fr = 4q + p): k-rows ks*32 + 8 fq + 4h + q,
// columns (wc & 1)*64 + 16 p + 4 (j ^ (p & 1)) + 0..3 — the perm_brow column order (each lane
// ends with 16 consecutive output columns), with the 4-column groups of odd p swapped pairwise
// so the 32 lanes of a half read both 8-B halves of the 16-B slots (JSWAP epilogue undoes it).
// Image swizzle: 16-B chunk c of k-row r lives in slot c ^ nnf(r), nnf(r) = (r & 3) | ((r >> 3)
// & 1) << 3: with the half-slot alternation every 32-lane half of a transposed read hits 32
// distinct (slot, half) bank pairs — conflict-free (the bank of byte a is (a/4) mod 64).
__device__ __forceinline__ int nnf(int row) { return (row & 3) | (((row >> 3) & 1) << 3); }

// rows [64u, 64u + 64) of the B panel (columns n0 .. n0 + 255): 32 wave-instructions, 8 per
// wave of the staging wave row (w4 = its wave column). Instruction s = 4i + w4: image s >> 4,
// row group rg = s & 15; nnf's bit 3 for its rows is (rg >> 1) & 1 = (w4 >> 1) & 1, fixed per
// wave, so one per-lane offset (boff) serves all eight loads.
template <int I0 = 0, int I1 = 8>
__device__ __forceinline__ void stage_b_nn(__amdgpu_buffer_rsrc_t rb, uint32_t ldb2, int u,
                                           char* bbuf, int w4, uint32_t boff) {
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int s = i * 4 + w4, img = s >> 4, rg = s & 15;
    bldsx4(rb, boff, static_cast<uint32_t>(u * BK + rg * 4) * ldb2 + img * 256,
           bbuf + img * (kTile2Bytes / 2) + rg * 1024);
  }
}


__device__ __forceinline__ void read_b_nn(const char* bbuf, int wc, int fr, int fq,
                                          bf16x8 (&bf)[2][4]) {
  const int q = fr >> 2, p = fr & 3;
  const char* img = bbuf + (wc >> 1) * (kTile2Bytes / 2);
  // rows ks * 32 + 8 fq + 4 h + q all have nnf(row) = nnf(8 fq + q): the address is a per-lane
  // base per column block j plus the immediate (ks * 32 + 4 h) * 256 (asm reads: common.h)
  const int r0 = 8 * fq + q;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (wc & 1) * 64 + 16 * p + 4 * (j ^ (p & 1));
    const char* base = img + r0 * 256 + (((col >> 3) ^ nnf(r0)) << 4) + (col & 7) * 2;
    const i16x4 t00 = ds_read_tr16<0>(base), t01 = ds_read_tr16<1024>(base);
    const i16x4 t10 = ds_read_tr16<8192>(base), t11 = ds_read_tr16<9216>(base);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bf[0][j][e] = t00[e];
      bf[0][j][4 + e] = t01[e];
      bf[1][j][e] = t10[e];
      bf[1][j][4 + e] = t11[e];
    }
  }
}

// ---------------------------------------------------------------------------------------
// TN operand A (weight gradient: dW[N_out, K_out] = dY[T, N_out]^T · X[T, K_out], both operands
// row-major over the reduction T). One K-tile of A = 64 t-rows x 256 dY columns, staged as two
// [64][128] images exactly like the NN B tile; image h holds output rows [128h, 128h + 128), so
// the A halves of the ping-pong ("A-lo" read by wave row 0, "A-hi" by row 1) are the two images
// and keep their 16-instruction staging (the counted waits are unchanged). Fragments come from
// ds_read_b64_tr_b16 in PLAIN column order (the A side of the epilogue is not permuted): lane
// (fq, fr = 4q + p) reads t-rows ks*32 + 8 fq + 4h + q, columns i*16 + 4p .. +3, with the
// csrc/gemm_tn.hip image swizzle — 16-B chunk c of row r in slot c ^ swz_tn(r), swz_tn(r) =
// 2 ((r & 3) | ((r >> 3) & 1) << 2), which makes every half-wave hit disjoint bank groups.
__device__ __forceinline__ int swz_tn(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }

// image `half` of A K-tile u: 16 wave-instructions, 4 per wave of the staging wave row
// (w4 = its wave column): instruction s = 4i + w4 loads t-rows 4s .. 4s + 3. An image wholly
// past the last output row (rows_a <= 128) re-stages image 0 (its rows are never stored).
__device__ __forceinline__ void stage_a_half_tn(__amdgpu_buffer_rsrc_t ra, uint32_t lda2,
                                                int rows_a, int u, char* abuf, int half, int w4,
                                                uint32_t aoff) {
  const uint32_t col = rows_a > 128 * half ? static_cast<uint32_t>(half) * 256 : 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rg = i * 4 + w4;
    bldsx4(ra, aoff, static_cast<uint32_t>(u * BK + rg * 4) * lda2 + col,
           abuf + half * (kTile2Bytes / 2) + rg * 1024);
  }
}

__device__ __forceinline__ void read_a_tn(const char* abuf, int wr, int fr, int fq,
                                          bf16x8 (&af)[2][8]) {
  // row = ks*32 + 8 fq + 4h + q has row & 3 = q and (row >> 3) & 1 = fq & 1, so swz_tn(row) is
  // one per-lane constant S (even): chunk (2i + (p >> 1)) ^ S = (2i ^ S) + (p >> 1), and the
  // byte offset is lane base + ((32 i) ^ 16 S) + immediate (ks, h). The 8 per-i addresses are
  // recomputed at every call (the empty asm hides S's invariance) rather than held in VGPRs
  // across the main loop, where the 256-register budget has no room for them.
  const int q = fr >> 2, p = fr & 3;
  int sx = swz_tn(q | ((fq & 1) << 3)) << 4;
  asm volatile("" : "+v"(sx));
  const char* lb = abuf + wr * (kTile2Bytes / 2) + (8 * fq + q) * 256 + (p >> 1) * 16 +
                   (p & 1) * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const char* ai = lb + (sx ^ (32 * i));
    // rows (ks * 32 + 4 h): immediates (asm reads, common.h)
    const i16x4 t00 = ds_read_tr16<0>(ai), t01 = ds_read_tr16<1024>(ai);
    const i16x4 t10 = ds_read_tr16<8192>(ai), t11 = ds_read_tr16<9216>(ai);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      af[0][i][e] = t00[e];
      af[0][i][4 + e] = t01[e];
      af[1][i][e] = t10[e];
      af[1][i][4 + e] = t11[e];
    }
  }
}

template <bool NN, int I0 = 0, int I1 = 8>
__device__ __forceinline__ void stage_b_any(__amdgpu_buffer_rsrc_t rb, uint32_t ldb2, int rows_b,
                                            int u, char* bbuf, int w4, uint32_t boff) {
  if constexpr (NN)
    stage_b_nn<I0, I1>(rb, ldb2, u, bbuf, w4, boff);
  else
    stage_b<I0, I1>(rb, ldb2, rows_b, static_cast<uint32_t>(u) * (BK * 2), bbuf, w4, boff);
}

template <bool NN, bool TN = false>
__device__ __forceinline__ void read_split_any(const char* abuf, const char* bbuf, int wr, int wc,
                                               int fr, int fq, bf16x8 (&af)[2][8],
                                               bf16x8 (&bf)[2][4]) {
  if constexpr (TN) {
    read_a_tn(abuf, wr, fr, fq, af);
    read_b_nn(bbuf, wc, fr, fq, bf);
  } else if constexpr (NN) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[ks][i] = read_frag(abuf, wr * 128 + i * 16 + fr, ks * 4 + fq);
    read_b_nn(bbuf, wc, fr, fq, bf);
  } else {
    read_split(abuf, bbuf, wr, wc, fr, fq, af, bf);
  }
}

// ---------------------------------------------------------------------------------------
// 256 x 192 output tiles (NJ = 3 MFMA column fragments per wave instead of 4: each of the 4 wave
// columns owns 48 output columns). For grids whose 256² form ends in a partial round of the
// 256 CUs — the GPT-2 projections N = 768 (192 tiles of 256², 0.75 round -> 256 tiles, one full
// round), QKV N = 2304 (576 tiles, 2.25 rounds -> 768, 3 full rounds) — the same work fills every
// CU. Host contract: N % 192 == 0 (every 48-row B block wholly in bounds).
// B row order inside a wave column's 48-row block (the perm_brow analogue): LDS image row
// L = 16 j + 4 fq + r (fragment j, lane quad fq, accumulator r) holds B row 12 fq + 4 j + r, so
// lane (fr, fq) ends with 12 consecutive output columns, acc[i][j][r] = column 4 j + r. In the
// 8-row DMA groups L = 8 g + r_in this is separable: row = g48_base(g) + g48_lane(r_in).
__device__ __forceinline__ int g48_base(int g) { return 24 * (g & 1) + 4 * (g >> 1); }
__device__ __forceinline__ int g48_lane(int r_in) { return 12 * (r_in >> 2) + (r_in & 3); }

// B tile of 192 rows = 24 groups of 8: instruction s = 4 i + w4 stages group s (wave column
// block s / 6, group g = s % 6) — 6 per wave of the staging row. [I0, I1) slices as stage_b.
template <int I0 = 0, int I1 = 6>
__device__ __forceinline__ void stage_b192(__amdgpu_buffer_rsrc_t rb, uint32_t ldb2, uint32_t k2,
                                           char* bbuf, int w4, uint32_t boff) {
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int s = i * 4 + w4;
    const int blk = s / 6, g = s - blk * 6;
    bldsx4(rb, boff, static_cast<uint32_t>(blk * 48 + g48_base(g)) * ldb2 + k2,
           bbuf + s * 8 * (BK * 2));
  }
}

// Epilogue of one wave's 128 x 48 block: lane (fr, fq) holds rows row0 + 16 i + fr, columns
// col0 + 12 fq + 4 j + r. The 12 columns are 24 B of bf16 (8-B aligned): three 8-B stores per
// row; fp32 output three 16-B stores. Host contract N % 192 == 0: every column group is whole.
template <int MI>
__device__ __forceinline__ void store_tile12(const GemmArgs& a, const f32x4 (&acc)[MI][3],
                                             int64_t row0, int64_t col0, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  const int epi = a.epi;
  const int64_t cbase = col0 + fq * 12;
  const int64_t rbase = row0 + fr;
  const int rows_left = static_cast<int>(a.M - rbase);
  const bool vec = a.vec_ok != 0;
  float bias[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) bias[c] = 0.f;
  if (epi & EPI_BIAS) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const u16x4 bv = vec ? reinterpret_cast<const u16x4*>(a.bias + cbase)[q]
                           : u16x4{a.bias[cbase + 4 * q], a.bias[cbase + 4 * q + 1],
                                   a.bias[cbase + 4 * q + 2], a.bias[cbase + 4 * q + 3]};
#pragma unroll
      for (int c = 0; c < 4; ++c) bias[4 * q + c] = bf16_to_f32(bv[c]);
    }
  }
  float* cf = static_cast<float*>(a.C) + rbase * a.ldc + cbase;
  uint16_t* cb = static_cast<uint16_t*>(a.C) + rbase * a.ldc + cbase;
  uint16_t* pb = a.preact ? a.preact + rbase * a.ldc + cbase : nullptr;
  const uint16_t* rb = (epi & EPI_READS_R) ? a.residual + rbase * a.ldr + cbase : nullptr;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    if (i * 16 >= rows_left) break;
    float v[12];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j * 4 + r] = acc[i][j][r] + bias[j * 4 + r];
    const int64_t oc = static_cast<int64_t>(i) * 16 * a.ldc, orr = static_cast<int64_t>(i) * 16 * a.ldr;
    if (vec) {
      if (pb) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          reinterpret_cast<u16x4*>(pb + oc)[q] =
              u16x4{f32_to_bf16(v[4 * q]), f32_to_bf16(v[4 * q + 1]), f32_to_bf16(v[4 * q + 2]),
                    f32_to_bf16(v[4 * q + 3])};
      }
      if (epi & (EPI_GELU_ERF | EPI_GELU_TANH)) {
#pragma unroll
        for (int c = 0; c < 12; ++c) v[c] = apply_act(v[c], epi);
      }
      if (rb) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const u16x4 rv = reinterpret_cast<const u16x4*>(rb + orr)[q];
#pragma unroll
          for (int c = 0; c < 4; ++c) v[4 * q + c] = apply_r(v[4 * q + c], bf16_to_f32(rv[c]), epi);
        }
      }
      if (a.out_f32) {
        float4* o = reinterpret_cast<float4*>(cf + oc);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          reinterpret_cast<u16x4*>(cb + oc)[q] =
              u16x4{f32_to_bf16(v[4 * q]), f32_to_bf16(v[4 * q + 1]), f32_to_bf16(v[4 * q + 2]),
                    f32_to_bf16(v[4 * q + 3])};
      }
    } else {
#pragma unroll
      for (int c = 0; c < 12; ++c) {
        float x = v[c];
        if (pb) pb[oc + c] = f32_to_bf16(x);
        x = apply_act(x, epi);
        if (rb) x = apply_r(x, bf16_to_f32(rb[orr + c]), epi);
        if (a.out_f32) cf[oc + c] = x; else cb[oc + c] = f32_to_bf16(x);
      }
    }
  }
}

// counted LDS-DMA wait with a compile-time count (the 192-wide tile changes every count)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The ping-pong schedule, for B stored [N][K] (NT: forward, C = A · B^T) or [K][N] (NN: dgrad).
// Both B layouts stage 32 wave-instructions per K-tile from wave row 0, so the counted waits
// are identical.
// BAL (balanced DMA issue): LDS-DMA instructions are expensive to ISSUE (~60-185 cycles each
// beside a phase's ds_reads, MI355X_MICROARCH.md), and the plain schedule has wave row 0 issue
// 12 of the 16 per K-tile (A-hi + all of B) in its memory interval against row 1's 4 (A-lo).
// BAL moves the second half of every B tile from tile 2 on (rows [128, 256) / the second
// image) to wave row 1, issued in interval 2u+1 next to A-lo(u+2) — 8 per row per K-tile:
//   interval 2u   (row 0): A-hi(u+1), B0(u+2)    interval 2u+1 (row 1): A-lo(u+2), B1(u+2)
// B1(u+2) replaces B(u-1), last read by row 1 in interval 2u-1; row 1 retires A-lo(u+1) and
// B1(u+1) together before the barrier ending 2u+1 (row 0 reads tile u+1 in 2u+2). B(1) stays
// whole in row 0's prologue, so the counted waits below also hold for u = 0.
// TN (weight gradient, implies NN for B): A [K][lda] row-major over the reduction, staged and
// read as transposed images (stage_a_half_tn / read_a_tn); split-K as for NN.
// STAMP (diagnostic variants only): per-workgroup start / end records into `st` (common.h).
// NJ: MFMA column fragments per wave — 4 (256-wide tile) or 3 (256 x 192, NT only; see
// stage_b192). NBI = B DMA instructions per staging wave per K-tile (2 NJ): every counted wait
// below is written in it (NJ = 4 gives the original literals).
// PHASES (diagnostic only, dlbb_gemm_nt_phase_probe): thread 0 stamps start / first MFMA (after
// the prologue waits) / end of the K-loop / end of the stores: 4 u64 per workgroup into `st`.
template <bool NN, bool BAL = false, bool TN = false, bool STAMP = false, int NJ = 4,
          bool PHASES = false>
__device__ __forceinline__ void pingpong_body(GemmArgs a, char* smem, uint64_t* st = nullptr) {
  static_assert(NJ == 4 || (NJ == 3 && !NN && !TN), "192-wide tiles: NT only");
  constexpr int NBI = 2 * NJ;                 // B DMA instructions per staging wave per K-tile
  constexpr int kTileB = NJ * 64 * BK * 2;    // bytes of one B tile buffer
  uint64_t t_start = 0;
  if constexpr (STAMP || PHASES) t_start = stamp_now();
  uint64_t t_first = 0, t_loop = 0;
  if (gridDim.y > 1) {               // split-K slice blockIdx.y (wave-uniform, SGPR math)
    const int s = blockIdx.y, nkt = static_cast<int>(a.K / BK);
    const int kt0 = s * a.kt_split, kt1 = kt0 + a.kt_split < nkt ? kt0 + a.kt_split : nkt;
    if constexpr (TN)                  // TN: A is row-major over the reduction too
      a.A += static_cast<int64_t>(kt0) * BK * a.lda;
    else
      a.A += static_cast<int64_t>(kt0) * BK;
    if constexpr (NN)                  // NN / TN: B row-major over the reduction
      a.B += static_cast<int64_t>(kt0) * BK * a.ldb;
    else                               // NT: B [N][K], the slice is a column offset
      a.B += static_cast<int64_t>(kt0) * BK;
    a.K = static_cast<int64_t>(kt1 - kt0) * BK;
    a.C = static_cast<float*>(a.C) + static_cast<int64_t>(s) * a.M * a.ldc;
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const Tile256 tl = tile_of<NJ * 64>(a, static_cast<int>(blockIdx.x));
  const int64_t m0 = tl.m0, n0 = tl.n0;
  const int nk = static_cast<int>(a.K / BK);
  char* const abuf0 = smem;
  char* const bbuf0 = smem + 2 * kTile2Bytes;

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], bf[2][NJ];
  const int r_in = lane >> 3, chunk = (lane & 7) ^ (lane >> 3);
  const uint32_t lda2 = static_cast<uint32_t>(a.lda) * 2, ldb2 = static_cast<uint32_t>(a.ldb) * 2;
  // TN: image rows 4s + rq, so swz_tn needs rq and bit 1 of the wave column
  const uint32_t aoff =
      TN ? static_cast<uint32_t>(lane >> 4) * lda2 +
               static_cast<uint32_t>((lane & 15) ^ (2 * ((lane >> 4) | (((wc >> 1) & 1) << 2)))) * 16
         : static_cast<uint32_t>(r_in) * lda2 + chunk * 16;
  uint32_t boff;
  if constexpr (NN) {
    const int rq = lane >> 4, slot = lane & 15;
    boff = static_cast<uint32_t>(rq) * ldb2 +
           static_cast<uint32_t>(slot ^ rq ^ (((wc >> 1) & 1) << 3)) * 16;
  } else if constexpr (NJ == 3) {
    boff = static_cast<uint32_t>(g48_lane(r_in)) * ldb2 + chunk * 16;
  } else {
    boff = static_cast<uint32_t>(perm_brow(r_in)) * ldb2 + chunk * 16;
  }
  const int rows_a = static_cast<int>(a.M - m0), rows_b = static_cast<int>(a.N - n0);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(TN ? a.A + m0 : a.A + m0 * a.lda), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(NN ? a.B + n0 : a.B + n0 * a.ldb), 0, 0x7fffffff, 0x00020000);
  constexpr uint32_t kStep = BK * 2;
  // B tile u into buffer `bb`, instruction slice [I0, I1) of the staging wave
  auto stage_bt = [&](auto i0, auto i1, int u, char* bb) {
    constexpr int I0 = decltype(i0)::value, I1 = decltype(i1)::value;
    if constexpr (NJ == 3)
      stage_b192<I0, I1>(rb, ldb2, static_cast<uint32_t>(u) * kStep, bb, wc, boff);
    else
      stage_b_any<NN, I0, I1>(rb, ldb2, rows_b, u, bb, wc, boff);
  };
  using Z = std::integral_constant<int, 0>;
  using H = std::integral_constant<int, NBI / 2>;
  using F = std::integral_constant<int, NBI>;
  auto read_frags = [&](const char* ab, const char* bb, int row) {
    if constexpr (NJ == 3) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < 8; ++i) af[ks][i] = read_frag(ab, row * 128 + i * 16 + fr, ks * 4 + fq);
#pragma unroll
        for (int j = 0; j < 3; ++j) bf[ks][j] = read_frag(bb, wc * 48 + j * 16 + fr, ks * 4 + fq);
      }
    } else {
      read_split_any<NN, TN>(ab, bb, row, wc, fr, fq, af, bf);
    }
  };
  auto mfma_all = [&]() {
    if constexpr (NJ == 3) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[i][j],
                                                                0, 0, 0);
    } else {
      mfma_full(acc, af, bf);
    }
  };
  // TN: A half `half` of K-tile u staged as a transposed image (4 wave-instructions per wave,
  // as stage_a_half); the NT / NN call sites below are kept verbatim (identical ISA)
#define DLBB_STAGE_A(U, BUF, HALF, NT_CALL)                                       \
  do {                                                                            \
    if constexpr (TN) stage_a_half_tn(ra, lda2, rows_a, (U), (BUF), (HALF), wc, aoff); \
    else NT_CALL;                                                                 \
  } while (0)

  if (wr == 0) {
    // prologue, row 0: A-lo(0), B(0), B(1); retire the first two
    DLBB_STAGE_A(0, abuf0, 0, stage_a_half(ra, lda2, rows_a, 0, abuf0, 0, wc, aoff));
    stage_bt(Z{}, F{}, 0, bbuf0);
    if (nk > 1) {
      stage_bt(Z{}, F{}, 1, bbuf0 + kTileB);
      wait_vm<NBI>();
    } else {
      DLBB_WAIT_VM(0);
    }
    __builtin_amdgcn_s_barrier();
    if constexpr (PHASES) t_first = stamp_now();
    int cb = 0;                                       // B buffer of tile u
    for (int u = 0; u < nk; ++u) {
      const char* ab = abuf0 + (u & 1) * kTile2Bytes;
      read_frags(ab, bbuf0 + cb * kTileB, 0);
      const bool h1 = u + 1 < nk, b2 = u + 2 < nk;
      if (h1)
        DLBB_STAGE_A(u + 1, abuf0 + ((u + 1) & 1) * kTile2Bytes, 1,
                     stage_a_half(ra, lda2, rows_a, (u + 1) * kStep,
                                  abuf0 + ((u + 1) & 1) * kTile2Bytes, 1, wc, aoff));
      auto stage_b2 = [&]() {
        const int cb2 = cb == 0 ? 2 : cb - 1;         // (u + 2) % 3
        if (BAL)
          stage_bt(Z{}, H{}, u + 2, bbuf0 + cb2 * kTileB);
        else
          stage_bt(Z{}, F{}, u + 2, bbuf0 + cb2 * kTileB);
      };
      if (b2) stage_b2();
      // retire A-hi(u) (issued two intervals ago; tile 0's came from row 1)
      constexpr int kB2 = BAL ? NBI / 2 : NBI;         // B(u+2) instructions issued
      if constexpr (BAL) {
        if (b2) wait_vm<NBI / 2 + 4 + kB2>();
        else if (h1) wait_vm<NBI / 2 + 4>();
        else wait_vm<0>();
      } else {
        if (b2) wait_vm<NBI + 4 + kB2>();
        else if (h1) wait_vm<NBI + 4>();
        else wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();                   // end of interval 2u
      __builtin_amdgcn_sched_barrier(0);
      mfma_all();

      __builtin_amdgcn_sched_barrier(0);
      if (h1) {                                       // retire B(u+1) (BAL: its first half)
        if (b2) { if (BAL) wait_vm<4 + NBI / 2>(); else wait_vm<4 + NBI>(); }
        else wait_vm<4>();
      }
      __builtin_amdgcn_s_barrier();                   // end of interval 2u+1
      cb = cb == 2 ? 0 : cb + 1;
    }
    if constexpr (PHASES) t_loop = stamp_now();
  } else {
    // prologue, row 1: A-hi(0), A-lo(1)
    DLBB_STAGE_A(0, abuf0, 1, stage_a_half(ra, lda2, rows_a, 0, abuf0, 1, wc, aoff));
    if (nk > 1)
      DLBB_STAGE_A(1, abuf0 + kTile2Bytes, 0,
                   stage_a_half(ra, lda2, rows_a, kStep, abuf0 + kTile2Bytes, 0, wc, aoff));
    __builtin_amdgcn_s_barrier();                     // prologue barrier
    if (nk > 1) DLBB_WAIT_VM(4); else DLBB_WAIT_VM(0);  // A-hi(0)
    __builtin_amdgcn_s_barrier();                     // end of interval 0
    int cb = 0;
    for (int u = 0; u < nk; ++u) {
      const char* ab = abuf0 + (u & 1) * kTile2Bytes;
      read_frags(ab, bbuf0 + cb * kTileB, 1);
      const bool l2 = u + 2 < nk;
      if (l2)
        DLBB_STAGE_A(u + 2, abuf0 + (u & 1) * kTile2Bytes, 0,
                     stage_a_half(ra, lda2, rows_a, (u + 2) * kStep,
                                  abuf0 + (u & 1) * kTile2Bytes, 0, wc, aoff));
      if (BAL && l2) {
        const int cb2 = cb == 0 ? 2 : cb - 1;         // (u + 2) % 3
        stage_bt(H{}, F{}, u + 2, bbuf0 + cb2 * kTileB);
      }
      if (u + 1 < nk) {                               // retire A-lo(u+1) (BAL: and B1(u+1))
        if (l2) { if (BAL) wait_vm<4 + NBI / 2>(); else wait_vm<4>(); }
        else wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();                   // end of interval 2u+1
      __builtin_amdgcn_sched_barrier(0);
      mfma_all();
      __builtin_amdgcn_sched_barrier(0);
      if (u + 1 < nk) __builtin_amdgcn_s_barrier();   // end of interval 2u+2
      cb = cb == 2 ? 0 : cb + 1;
    }
  }
  if constexpr (NJ == 3)
    store_tile12<8>(a, acc, m0 + (wave >> 2) * 128, n0 + (wave & 3) * 48, lane);
  else
    store_tile_256<NN>(a, acc, m0, n0, wave, lane);
  if constexpr (STAMP) {
    __syncthreads();
    if (threadIdx.x == 0) stamp_write(st, t_start);
  }
  if constexpr (PHASES) {
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t* r = st + 4 * (blockIdx.x + static_cast<uint64_t>(blockIdx.y) * gridDim.x);
      // s_memrealtime (100 MHz) needs < 48 bits for days: the XCD id and HW_ID ride in the
      // top 16 bits of the start stamp (xcc << 13 | se << 10 | cu << 6)
      const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
      const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
      const uint64_t tag = ((xcc & 7u) << 13) | (((hw >> 13) & 7u) << 10) | (((hw >> 8) & 15u) << 6);
      r[0] = (t_start & ((1ull << 48) - 1)) | (tag << 48);
      r[1] = t_first;
      r[2] = t_loop;
      r[3] = stamp_now();
    }
  }
#undef DLBB_STAGE_A
}

__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_pingpong3(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false>(a, smem);
}

// A/B variant (set_stagger(7)): the balanced DMA issue (BAL above).
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_pingpong3_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false, true>(a, smem);
}
// 256 x 192 tiles (N % 192 == 0): grids that end in a partial round of 256² tiles
constexpr int kPP192Lds = 2 * kTile2Bytes + 3 * (3 * 64 * BK * 2);   // 136 KiB
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_192_pingpong3(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false, false, false, false, 3>(a, smem);
}
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_192_pingpong3_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false, true, false, false, 3>(a, smem);
}

// phase-stamped twins (diagnostic): tools/diag/pp_phases.py
__global__ void __launch_bounds__(kThreads2, 1) gemm_nt_pp_phases(GemmArgs a, uint64_t* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false, true, false, false, 4, true>(a, smem, st);
}
__global__ void __launch_bounds__(kThreads2, 1) gemm_nt_pp192_phases(GemmArgs a, uint64_t* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<false, true, false, false, 3, true>(a, smem, st);
}

// dgrad: C[M, N] = A[M, K] · B[K, N] (B row-major over the reduction); host contract
// N % 256 == 0, M % 8 == 0, K % 64 == 0.
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nn_256_pingpong3(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<true>(a, smem);
}
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nn_256_pingpong3_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<true, true>(a, smem);
}

// weight gradient: C[M, N] = A[K, M]^T · B[K, N] (both row-major over the reduction K); host
// contract M % 128 == 0, N % 256 == 0, K % 64 == 0.
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_tn_256_pingpong3(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<true, false, true>(a, smem);
}
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_tn_256_pingpong3_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pingpong_body<true, true, true>(a, smem);
}

// Stamped diagnostic twins of the six ping-pong kernels (dlbb_stamps_set): identical schedule,
// plus one start / end record per workgroup.
#define DLBB_PP_STAMPED(NAME, NN_, BAL_, TN_)                                          \
  __global__ void __launch_bounds__(kThreads2, 1) NAME##_st(GemmArgs a, uint64_t* st) { \
    extern __shared__ __attribute__((aligned(16))) char smem[];                        \
    pingpong_body<NN_, BAL_, TN_, true>(a, smem, st);                                  \
  }
DLBB_PP_STAMPED(gemm_bf16_nt_256_pingpong3, false, false, false)
DLBB_PP_STAMPED(gemm_bf16_nt_256_pingpong3_bal, false, true, false)
DLBB_PP_STAMPED(gemm_bf16_nn_256_pingpong3, true, false, false)
DLBB_PP_STAMPED(gemm_bf16_nn_256_pingpong3_bal, true, true, false)
DLBB_PP_STAMPED(gemm_bf16_tn_256_pingpong3, true, false, true)
DLBB_PP_STAMPED(gemm_bf16_tn_256_pingpong3_bal, true, true, true)
#undef DLBB_PP_STAMPED

// ---------------------------------------------------------------------------------------
// Persistent ping-pong (set_stagger(10), NT): one workgroup per CU walks the output tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... as ONE continuous stream of K-tiles g = 0 .. G-1
// (tile i = g / nk, K-tile g % nk). The non-persistent kernel pays a fixed cost per tile —
// prologue DMA latency, the pipeline fill (row 1 idle in interval 0) and drain (row 0 idle in
// the last interval), the epilogue with the matrix pipe idle, workgroup launch: ~6.5 us per
// 256² tile in multi-round grids, ~7 % at K = 4096 and far more at short K
// (tools/diag/pp_tile_overhead.py: median workgroup time = 10.6 us + 1.37 us per K-tile in one
// round). Here the schedule of pingpong_body<false, BAL> simply continues across tiles: the DMA
// of g + 1 / g + 2 already targets the next tile while the current one finishes, and each wave
// row stores its finished accumulators at the START of its first memory interval of the next
// tile (before that interval's ds_reads, so the epilogue's temporaries never coexist with the
// fragments), then zeroes them.
// Counted waits with stores in flight: every count below is the number of LOADS (DMA) issued
// after the one being retired. Loads return in order; a store may complete earlier or later
// than a load, but it only ever ADDS to the outstanding count — so vmcnt <= (younger loads)
// still implies the target load is done (stores can only make a wait longer, never unsafe).
// Host contract as the ping-pong (M % 8, N % 64, 32-bit panel offsets) plus nk >= 2.
// Lean epilogue of one wave's 128 x 64 block for the persistent kernel: plain bf16 output, vector
// stores only (host contract: no bias / activation / residual / pre-activation, bf16 C, vec_ok;
// N % 64 == 0 makes every 16-column lane group whole). The general epilogue (store_tile) inside
// the tile loop measured 7-15 % slower on the same shapes (persistent_ab_general_epilogue.jsonl).
// LEAN epilogue kinds of the persistent kernel, bf16 output with vector stores: NT plain, + bias,
// + bias -> GELU (tanh / erf) with an optional bf16 pre-activation store (the GPT-2 QKV / FC
// forwards on multi-round grids of 12 K-tiles); NN plain and the GELU backward C = (A·B)·gelu'(u)
// (the GPT-2 MLP-proj dgrad). Each kind is its own instantiation, so the tile loop carries only
// the code its shape needs (the general store_tile in the loop measured 7-15 % slower).
enum PpLean : int {
  PP_PLAIN = 0, PP_BIAS = 1, PP_BIAS_GELU_TANH = 2, PP_BIAS_GELU_ERF = 3,
  PP_DGELU_TANH = 4, PP_DGELU_ERF = 5,
};

// What the epilogue reads (the bias of the lane's 16 columns, or its 8 x 16 values of u) is loaded
// by the caller BEFORE the wave drains its DMA with vmcnt(0), so the load latency hides in that
// drain instead of stalling the flush. The fragments are dead there, so u's 64 VGPRs fit.
#ifndef DLBB_UPRE
#define DLBB_UPRE 1
#endif
struct LeanPre { u16x8 v[8]; };   // bias: v[0..1]; GELU backward: u of row blocks 0..3

template <int LEAN>
__device__ __forceinline__ void lean_pre(const GemmArgs& a, LeanPre& p, int64_t row0,
                                         int64_t col0, int lane) {
  const int64_t cbase = col0 + (lane >> 4) * 16;
  if (cbase >= a.N) return;
  if constexpr (LEAN == PP_BIAS || LEAN == PP_BIAS_GELU_TANH || LEAN == PP_BIAS_GELU_ERF) {
    const u16x8* bp = reinterpret_cast<const u16x8*>(a.bias + cbase);
    p.v[0] = bp[0];
    p.v[1] = bp[1];
  } else if constexpr (LEAN == PP_DGELU_TANH || LEAN == PP_DGELU_ERF) {
    const int64_t rbase = row0 + (lane & 15);
    const int rows_left = static_cast<int>(a.M - rbase);
    const uint16_t* up = a.residual + rbase * a.ldr + cbase;
#pragma unroll
    for (int i = 0; i < DLBB_UPRE; ++i) {    // (all eight blocks' 64 VGPRs beside the accumulators spill)
      if (i * 16 >= rows_left) break;
      const u16x8* q = reinterpret_cast<const u16x8*>(up + static_cast<int64_t>(i) * 16 * a.ldr);
      p.v[2 * i] = q[0];
      p.v[2 * i + 1] = q[1];
    }
  }
}

template <bool NN, int LEAN>
__device__ __forceinline__ void store_lean_bf16(const GemmArgs& a, const f32x4 (&acc)[8][4],
                                                int64_t row0, int64_t col0, int lane,
                                                const LeanPre& p) {
  constexpr bool kBias = LEAN == PP_BIAS || LEAN == PP_BIAS_GELU_TANH || LEAN == PP_BIAS_GELU_ERF;
  constexpr bool kDgelu = LEAN == PP_DGELU_TANH || LEAN == PP_DGELU_ERF;
  const int fr = lane & 15, fq = lane >> 4;
  const bool odd = NN && (fq & 1);      // NN fragments: 4-column groups swapped (read_b_nn)
  const int64_t cbase = col0 + fq * 16;
  if (cbase >= a.N) return;
  const int64_t rbase = row0 + fr;
  const int rows_left = static_cast<int>(a.M - rbase);
  uint16_t* cb = static_cast<uint16_t*>(a.C) + rbase * a.ldc + cbase;
  float bias[16];
  if constexpr (kBias) {
#pragma unroll
    for (int c = 0; c < 8; ++c) { bias[c] = bf16_to_f32(p.v[0][c]); bias[8 + c] = bf16_to_f32(p.v[1][c]); }
  }
  uint16_t* pb = ((LEAN == PP_BIAS_GELU_TANH || LEAN == PP_BIAS_GELU_ERF) && a.preact)
                     ? a.preact + rbase * a.ldc + cbase : nullptr;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i * 16 >= rows_left) break;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = odd ? acc[i][j ^ 1][r] : acc[i][j][r];
        v[j * 4 + r] = kBias ? x + bias[j * 4 + r] : x;
      }
    const int64_t oc = static_cast<int64_t>(i) * 16 * a.ldc;
    if (pb) {
      u16x8 p0, p1;
#pragma unroll
      for (int c = 0; c < 8; ++c) { p0[c] = f32_to_bf16(v[c]); p1[c] = f32_to_bf16(v[8 + c]); }
      reinterpret_cast<u16x8*>(pb + oc)[0] = p0;
      reinterpret_cast<u16x8*>(pb + oc)[1] = p1;
    }
    if constexpr (LEAN == PP_BIAS_GELU_TANH) {
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = gelu_tanh(v[c]);
    } else if constexpr (LEAN == PP_BIAS_GELU_ERF) {
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = gelu_erf(v[c]);
    } else if constexpr (kDgelu) {
      u16x8 ua, ub;
      if (i < DLBB_UPRE) {
        ua = p.v[2 * i];
        ub = p.v[2 * i + 1];
      } else {                          // blocks 4..7: loaded here (latency exposed)
        const u16x8* q = reinterpret_cast<const u16x8*>(a.residual + (rbase + i * 16) * a.ldr +
                                                        cbase);
        ua = q[0];
        ub = q[1];
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float u0 = bf16_to_f32(ua[c]), u1 = bf16_to_f32(ub[c]);
        v[c] *= LEAN == PP_DGELU_TANH ? gelu_tanh_grad(u0) : gelu_erf_grad(u0);
        v[8 + c] *= LEAN == PP_DGELU_TANH ? gelu_tanh_grad(u1) : gelu_erf_grad(u1);
      }
    }
    u16x8 o0, o1;
#pragma unroll
    for (int c = 0; c < 8; ++c) { o0[c] = f32_to_bf16(v[c]); o1[c] = f32_to_bf16(v[8 + c]); }
    u16x8* o = reinterpret_cast<u16x8*>(cb + oc);
    o[0] = o0;
    o[1] = o1;
  }
}

template <bool NN, bool BAL, int LEAN = PP_PLAIN>
__device__ __forceinline__ void pp_persist_body(GemmArgs a, char* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = static_cast<int>(a.K / BK);
  const int tiles = static_cast<int>(((a.M + BM2 - 1) / BM2) * ((a.N + BN2 - 1) / BN2));
  const int nwg = static_cast<int>(gridDim.x), wg = static_cast<int>(blockIdx.x);
  const int mine = wg < tiles ? (tiles - wg + nwg - 1) / nwg : 0;
  if (mine == 0) return;
  const int G = mine * nk;                      // this workgroup's virtual K-tiles
  char* const abuf0 = smem;
  char* const bbuf0 = smem + 2 * kTile2Bytes;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], bf[2][4];
  const int r_in = lane >> 3, chunk = (lane & 7) ^ (lane >> 3);
  const uint32_t lda2 = static_cast<uint32_t>(a.lda) * 2, ldb2 = static_cast<uint32_t>(a.ldb) * 2;
  const uint32_t aoff = static_cast<uint32_t>(r_in) * lda2 + chunk * 16;
  uint32_t boff;
  if constexpr (NN) {                           // as pingpong_body: transposed-read B images
    const int rq = lane >> 4, slot = lane & 15;
    boff = static_cast<uint32_t>(rq) * ldb2 +
           static_cast<uint32_t>(slot ^ rq ^ (((wc >> 1) & 1) << 3)) * 16;
  } else {
    boff = static_cast<uint32_t>(perm_brow(r_in)) * ldb2 + chunk * 16;
  }
  constexpr uint32_t kStep = BK * 2;
#define DLBB_RSRC(P) \
  __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(P), 0, 0x7fffffff, 0x00020000)

  Tile256 tc = tile_of(a, wg);                  // the tile being multiplied
  // bias kinds: the bias of the tile being multiplied is loaded one tile ahead (8 VGPRs held
  // across the K loop) — loaded at the flush it stalled every tile boundary (+6 us on the GPT-2
  // QKV forward); the GELU backward's u is too large to hold and is loaded at the boundary
  constexpr bool kBiasAhead =
      LEAN == PP_BIAS || LEAN == PP_BIAS_GELU_TANH || LEAN == PP_BIAS_GELU_ERF;
  LeanPre bias_ahead;
  if constexpr (kBiasAhead)
    lean_pre<LEAN>(a, bias_ahead, tc.m0 + (wave >> 2) * 128, tc.n0 + (wave & 3) * 64, lane);
  {
    const __amdgpu_buffer_rsrc_t ra = DLBB_RSRC(a.A + tc.m0 * a.lda);
    const __amdgpu_buffer_rsrc_t rb = DLBB_RSRC(NN ? a.B + tc.n0 : a.B + tc.n0 * a.ldb);
    const int rows_a = static_cast<int>(a.M - tc.m0), rows_b = static_cast<int>(a.N - tc.n0);
    if (wr == 0) {                              // prologue (nk >= 2): A-lo(0), B(0), B(1)
      stage_a_half(ra, lda2, rows_a, 0, abuf0, 0, wc, aoff);
      stage_b_any<NN>(rb, ldb2, rows_b, 0, bbuf0, wc, boff);
      stage_b_any<NN>(rb, ldb2, rows_b, 1, bbuf0 + kTile2Bytes, wc, boff);
      DLBB_WAIT_VM(8);
      __builtin_amdgcn_s_barrier();
    } else {                                    // A-hi(0), A-lo(1)
      stage_a_half(ra, lda2, rows_a, 0, abuf0, 1, wc, aoff);
      stage_a_half(ra, lda2, rows_a, kStep, abuf0 + kTile2Bytes, 0, wc, aoff);
      __builtin_amdgcn_s_barrier();
      DLBB_WAIT_VM(4);
      __builtin_amdgcn_s_barrier();             // end of interval 0
    }
  }
  // A wave row stores its part of finished tile T at the start of its FIRST memory interval of
  // tile T + 1 (before the ds_reads: the fragments are dead there, so the epilogue fits beside
  // the accumulators). It first retires its own outstanding DMA (vmcnt(0)) — the loads that
  // interval's and the next interval's counted waits would otherwise retire with the stores
  // queued behind them — and those two waits are skipped at the boundary. The lane-dependent
  // epilogue addresses are recomputed here (the empty asm), not hoisted into the K loop.
#define DLBB_PP_FLUSH(T)                                                           \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    int ln_ = lane;                                                                \
    asm volatile("" : "+v"(ln_));                                                  \
    store_lean_bf16<NN, LEAN>(                                                     \
          a, acc, (T).m0 + (wave >> 2) * 128, (T).n0 + (wave & 3) * 64, ln_, pre_);  \
    _Pragma("unroll") for (int x_ = 0; x_ < 8; ++x_)                                \
      _Pragma("unroll") for (int y_ = 0; y_ < 4; ++y_)                              \
        acc[x_][y_] = f32x4{0.f, 0.f, 0.f, 0.f};                                    \
    __builtin_amdgcn_sched_barrier(0);                                             \
  } while (0)
  int cb = 0;                                   // B buffer of virtual K-tile g (g % 3)
  for (int i = 0; i < mine; ++i) {
    const Tile256 tn = i + 1 < mine ? tile_of(a, wg + (i + 1) * nwg) : tc;   // next tile
    const __amdgpu_buffer_rsrc_t ra = DLBB_RSRC(a.A + tc.m0 * a.lda);
    const __amdgpu_buffer_rsrc_t rb = DLBB_RSRC(NN ? a.B + tc.n0 : a.B + tc.n0 * a.ldb);
    const __amdgpu_buffer_rsrc_t ran = DLBB_RSRC(a.A + tn.m0 * a.lda);
    const __amdgpu_buffer_rsrc_t rbn = DLBB_RSRC(NN ? a.B + tn.n0 : a.B + tn.n0 * a.ldb);
    const int rows_a = static_cast<int>(a.M - tc.m0), rows_b = static_cast<int>(a.N - tc.n0);
    const int rows_an = static_cast<int>(a.M - tn.m0), rows_bn = static_cast<int>(a.N - tn.n0);
    if (wr == 0) {
      for (int k = 0; k < nk; ++k) {
        const int g = i * nk + k;
        const bool bnd = k == 0 && i > 0;       // first K-tile of a new output tile
        read_split_any<NN>(abuf0 + (g & 1) * kTile2Bytes, bbuf0 + cb * kTile2Bytes, 0, wc, fr, fq, af,
                           bf);
        const bool h1 = g + 1 < G, b2 = g + 2 < G;
        char* const an = abuf0 + ((g + 1) & 1) * kTile2Bytes;
        if (h1) {                               // A-hi(g+1): this tile's K-tile or the next's 0
          if (k + 1 < nk) stage_a_half(ra, lda2, rows_a, (k + 1) * kStep, an, 1, wc, aoff);
          else stage_a_half(ran, lda2, rows_an, 0, an, 1, wc, aoff);
        }
        if (b2) {                               // B(g+2) (BAL: its first half)
          char* const bn = bbuf0 + (cb == 0 ? 2 : cb - 1) * kTile2Bytes;
          const bool here = k + 2 < nk;
          const int ub = here ? k + 2 : k + 2 - nk;       // K-tile index within its tile
          if (BAL)
            stage_b_any<NN, 0, 4>(here ? rb : rbn, ldb2, here ? rows_b : rows_bn, ub, bn, wc, boff);
          else
            stage_b_any<NN, 0, 8>(here ? rb : rbn, ldb2, here ? rows_b : rows_bn, ub, bn, wc, boff);
        }
        if (bnd) {
          // A-hi(g) retired at the top: no wait, so the stores are never drained here
        } else if (BAL) {
          if (b2) DLBB_WAIT_VM(12);
          else if (h1) DLBB_WAIT_VM(8);
          else DLBB_WAIT_VM(0);
        } else {
          if (b2) DLBB_WAIT_VM(20);
          else if (h1) DLBB_WAIT_VM(12);
          else DLBB_WAIT_VM(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();           // end of interval 2g
        __builtin_amdgcn_sched_barrier(0);
        mfma_full(acc, af, bf);
        __builtin_amdgcn_sched_barrier(0);
        if (h1 && !bnd) {                       // (boundary: B(g+1) retired at the top)
          if (b2) { if (BAL) DLBB_WAIT_VM(8); else DLBB_WAIT_VM(12); }
          else DLBB_WAIT_VM(4);
        }
        __builtin_amdgcn_s_barrier();           // end of interval 2g+1
        cb = cb == 2 ? 0 : cb + 1;
      }
    } else {
      for (int k = 0; k < nk; ++k) {
        const int g = i * nk + k;
        const bool bnd = k == 0 && i > 0;
        read_split_any<NN>(abuf0 + (g & 1) * kTile2Bytes, bbuf0 + cb * kTile2Bytes, 1, wc, fr, fq, af,
                           bf);
        const bool l2 = g + 2 < G;
        if (l2) {                               // A-lo(g+2) (BAL: and B1(g+2))
          const bool here = k + 2 < nk;
          const int ub = here ? k + 2 : k + 2 - nk;
          stage_a_half(here ? ra : ran, lda2, here ? rows_a : rows_an,
                       static_cast<uint32_t>(ub) * kStep, abuf0 + (g & 1) * kTile2Bytes, 0, wc,
                       aoff);
          if (BAL)
            stage_b_any<NN, 4, 8>(here ? rb : rbn, ldb2, here ? rows_b : rows_bn, ub,
                                  bbuf0 + (cb == 0 ? 2 : cb - 1) * kTile2Bytes, wc, boff);
        }
        if (g + 1 < G && !bnd) {               // (boundary: A-lo(g+1) retired at the top)
          if (l2) { if (BAL) DLBB_WAIT_VM(8); else DLBB_WAIT_VM(4); }
          else DLBB_WAIT_VM(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();           // end of interval 2g+1
        __builtin_amdgcn_sched_barrier(0);
        mfma_full(acc, af, bf);
        __builtin_amdgcn_sched_barrier(0);
        if (g + 1 < G) __builtin_amdgcn_s_barrier();   // end of interval 2g+2
        cb = cb == 2 ? 0 : cb + 1;
      }
    }
    // this row's part of tile i, at the start of its first memory interval of tile i + 1
    LeanPre pre_;
    if constexpr (kBiasAhead) pre_ = bias_ahead;
    else lean_pre<LEAN>(a, pre_, tc.m0 + (wave >> 2) * 128, tc.n0 + (wave & 3) * 64, lane);
    DLBB_WAIT_VM(0);
    DLBB_PP_FLUSH(tc);
    if constexpr (kBiasAhead)   // issued after the stores: older than every later counted load
      if (i + 1 < mine)
        lean_pre<LEAN>(a, bias_ahead, tn.m0 + (wave >> 2) * 128, tn.n0 + (wave & 3) * 64, lane);
    tc = tn;
  }
#undef DLBB_PP_FLUSH
#undef DLBB_RSRC
}

template <int LEAN>
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_pp_persist(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_persist_body<false, false, LEAN>(a, smem);
}
template <int LEAN>
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_pp_persist_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_persist_body<false, true, LEAN>(a, smem);
}
// NN (dgrad) persistent form: balanced DMA issue (NN's measured default at every K)
template <int LEAN>
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nn_256_pp_persist_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_persist_body<true, true, LEAN>(a, smem);
}

// ---------------------------------------------------------------------------------------
// Stream-K NT GEMM (256² tiles, the balanced / plain ping-pong schedule of pp_persist_body) for
// grids below one round of the CUs — the 7B TP shard projections (models.py:47,81 at
// baseline_config.yaml:17 P = 4 / 8: 96-128 tiles on 256 CUs). The output
// tiles' K-loops are laid end to end as ONE stream of tiles * nk K-tile iterations; workgroup v
// (one per CU) runs the contiguous range [v L, v L + L) of it, so every CU gets the same work
// whatever the tile count. With tiles < workgroups a range is at most nk long, so it touches at
// most two tiles: the tail of tile P and the head of tile P + 1. A tile covered by ONE range is
// stored directly (full epilogue); a tile split between ranges is combined in the launch, per
// WAVE (each wave owns a 128 x 64 block of every tile, so no workgroup barrier is needed, and
// the staggered wave rows of the ping-pong keep their barrier pairing):
//   poll the (tile, wave) arrival counter; unless every other contributor has already arrived,
//   store the 32 fp32 accumulators write-through (sc1, 1 KiB per wave-instruction), drain them
//   (s_waitcnt vmcnt(0)) and add 1 to the counter. The wave that sees the last arrival (its poll
//   or the value its add returned) reads the other contributors' blocks with sc1 loads, adds
//   them in registers, resets the counter to 0 and runs the whole epilogue (bias, GELU,
//   pre-activation, residual, bf16 | fp32 store). MI355X_MICROARCH.md 'Valid forms' row 1: sc1
//   stores, vmcnt(0) before the add, one workgroup per CU, loads after the add returned, sc1
//   loads — no release / acquire fences (a release writes back the whole XCD L2). Nobody waits
//   for anybody, so the launch cannot deadlock beside other kernels holding CUs.
// Partial block of (slot, wave): ws + (slot * 8 + wave) * 32 KiB, register r of lane l at
// r * 1 KiB + 16 l. Slots: workgroup v's first segment (its range starts inside the tile) uses
// slot 2 v, its second segment slot 2 v + 1; a contributor u of tile t used slot 2 u iff
// u L >= t nk. Counters: tiles * 8 ints, zero on entry and left zero.
typedef unsigned sk_u32v4 __attribute__((vector_size(16)));   // the buffer builtins' b128 type

struct SkArgs {
  float* ws;
  int* cnt;
  int L;       // K-tile iterations per workgroup
  int nk;      // K-tiles per output tile
};

// tile index -> 256² output tile, GROUP_M order without the XCD remap (consecutive stream
// ranges are placed on one XCD instead, see pp_streamk_body)
__device__ __forceinline__ Tile256 tile_linear(const GemmArgs& a, int wid) {
  const int tiles_m = static_cast<int>((a.M + BM2 - 1) / BM2);
  const int tiles_n = static_cast<int>((a.N + BN2 - 1) / BN2);
  const int group_size = kGroupM * tiles_n;
  const int group = wid / group_size;
  const int first_m = group * kGroupM;
  const int gm = (tiles_m - first_m) < kGroupM ? (tiles_m - first_m) : kGroupM;
  const int in_group = wid - group * group_size;
  return Tile256{static_cast<int64_t>(first_m + in_group % gm) * BM2,
                 static_cast<int64_t>(in_group / gm) * BN2};
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// One wave's end of a segment of tile t (see above). `full`: the segment is the whole K range.
__device__ __forceinline__ void sk_finish(const GemmArgs& a, const SkArgs& s, f32x4 (&acc)[8][4],
                                          int t, bool full, int v, int slot, int wave, int lane) {
  const Tile256 T = tile_linear(a, t);
  if (!full) {
    int* cnt = s.cnt + t * 8 + wave;
    const int first = (t * s.nk) / s.L, last = ((t + 1) * s.nk - 1) / s.L;
    const int others = last - first;                  // contributors besides this one
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(s.ws);
    const uint32_t lo = static_cast<uint32_t>(lane) * 16;
    int seen = 0;
    if (lane == 0) seen = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    seen = __builtin_amdgcn_readfirstlane(seen);
    bool is_last = seen == others;
    if (!is_last) {
      const uint32_t base = static_cast<uint32_t>(slot * 8 + wave) * 32768u;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u32v4, acc[i][j]), rw, lo,
                                                 base + (i * 4 + j) * 1024, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int prev = 0;
      if (lane == 0)
        prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prev = __builtin_amdgcn_readfirstlane(prev);
      is_last = prev == others;
    }
    if (!is_last) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    for (int u = first; u <= last; ++u) {
      if (u == v) continue;
      const int su = u * s.L >= t * s.nk ? 2 * u : 2 * u + 1;
      const uint32_t base = static_cast<uint32_t>(su * 8 + wave) * 32768u;
#pragma unroll
      for (int h = 0; h < 2; ++h) {                   // 16 loads in flight, then 16 adds
        f32x4 p[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            p[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rw, lo, base + ((4 * h + i) * 4 + j) * 1024, 16));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 * h + i][j] += p[i][j];
      }
    }
    if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  store_tile_256(a, acc, T.m0, T.n0, wave, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <bool BAL>
__device__ __forceinline__ void pp_streamk_body(GemmArgs a, SkArgs s, char* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = s.nk;
  // stream position v of this workgroup: consecutive ranges (which share tiles, so their
  // partial blocks and A / B panels) on one XCD (blockIdx % 8 under round-robin dispatch —
  // speed only, never correctness); the same bijective remap as tile_of
  const int nwg = static_cast<int>(gridDim.x), bx = static_cast<int>(blockIdx.x);
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bx & 7;
  const int v = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bx >> 3);
  const int tiles = static_cast<int>(((a.M + BM2 - 1) / BM2) * ((a.N + BN2 - 1) / BN2));
  const int it0 = v * s.L;
  const int itend = it0 + s.L < tiles * nk ? it0 + s.L : tiles * nk;
  if (it0 >= itend) return;                          // (host: never; whole workgroup)
  const int G = itend - it0;                          // this range's K-tiles (host: >= 2)
  const int tP = it0 / nk, kP = it0 - tP * nk;        // first tile and its first K-tile
  const int gb = nk - kP;                             // first iteration of tile P + 1
  const Tile256 TP = tile_linear(a, tP);
  const Tile256 TQ = gb < G ? tile_linear(a, tP + 1) : TP;
  char* const abuf0 = smem;
  char* const bbuf0 = smem + 2 * kTile2Bytes;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], bf[2][4];
  const int r_in = lane >> 3, chunk = (lane & 7) ^ (lane >> 3);
  const uint32_t lda2 = static_cast<uint32_t>(a.lda) * 2, ldb2 = static_cast<uint32_t>(a.ldb) * 2;
  const uint32_t aoff = static_cast<uint32_t>(r_in) * lda2 + chunk * 16;
  const uint32_t boff = static_cast<uint32_t>(perm_brow(r_in)) * ldb2 + chunk * 16;
  constexpr uint32_t kStep = BK * 2;
  const __amdgpu_buffer_rsrc_t raP = rsrc_of(a.A + TP.m0 * a.lda);
  const __amdgpu_buffer_rsrc_t rbP = rsrc_of(a.B + TP.n0 * a.ldb);
  const __amdgpu_buffer_rsrc_t raQ = rsrc_of(a.A + TQ.m0 * a.lda);
  const __amdgpu_buffer_rsrc_t rbQ = rsrc_of(a.B + TQ.n0 * a.ldb);
  const int rows_aP = static_cast<int>(a.M - TP.m0), rows_bP = static_cast<int>(a.N - TP.n0);
  const int rows_aQ = static_cast<int>(a.M - TQ.m0), rows_bQ = static_cast<int>(a.N - TQ.n0);
  // iteration g -> (tile P or Q, K-tile index inside it)
  auto in_q = [&](int g) __attribute__((always_inline)) { return g >= gb; };
  auto kt = [&](int g) __attribute__((always_inline)) { return g >= gb ? g - gb : kP + g; };
  auto stage_a = [&](int g, char* buf, int half) __attribute__((always_inline)) {
    const bool q = in_q(g);
    stage_a_half(q ? raQ : raP, lda2, q ? rows_aQ : rows_aP, static_cast<uint32_t>(kt(g)) * kStep,
                 buf, half, wc, aoff);
  };
  auto stage_bh = [&](auto i0, auto i1, int g, char* buf) __attribute__((always_inline)) {
    constexpr int I0 = decltype(i0)::value, I1 = decltype(i1)::value;
    const bool q = in_q(g);
    stage_b<I0, I1>(q ? rbQ : rbP, ldb2, q ? rows_bQ : rows_bP,
                    static_cast<uint32_t>(kt(g)) * kStep, buf, wc, boff);
  };
  using Z = std::integral_constant<int, 0>;
  using H = std::integral_constant<int, 4>;
  using F = std::integral_constant<int, 8>;
  // end of a segment: tile P after iteration gb - 1 (when Q follows), the last tile after G - 1
  auto finish = [&](int g) __attribute__((always_inline)) {
    const bool q = in_q(g);
    const int kb = q ? 0 : kP, ke = kt(g) + 1;
    int ln = lane;
    asm volatile("" : "+v"(ln));                    // epilogue addresses not hoisted
    sk_finish(a, s, acc, q ? tP + 1 : tP, kb == 0 && ke == nk, v, q ? 2 * v + 1 : 2 * v, wave, ln);
  };

  if (wr == 0) {                                    // prologue: A-lo(0), B(0), B(1)
    stage_a(0, abuf0, 0);
    stage_bh(Z{}, F{}, 0, bbuf0);
    stage_bh(Z{}, F{}, 1, bbuf0 + kTile2Bytes);
    DLBB_WAIT_VM(8);
    __builtin_amdgcn_s_barrier();
  } else {                                          // A-hi(0), A-lo(1)
    stage_a(0, abuf0, 1);
    stage_a(1, abuf0 + kTile2Bytes, 0);
    __builtin_amdgcn_s_barrier();
    DLBB_WAIT_VM(4);
    __builtin_amdgcn_s_barrier();                   // end of interval 0
  }
  int cb = 0;                                       // B buffer of iteration g (g % 3)
  if (wr == 0) {
    for (int g = 0; g < G; ++g) {
      const bool bnd = g == gb && g > 0;            // first K-tile of tile Q
      read_split_any<false>(abuf0 + (g & 1) * kTile2Bytes, bbuf0 + cb * kTile2Bytes, 0, wc, fr,
                            fq, af, bf);
      const bool h1 = g + 1 < G, b2 = g + 2 < G;
      if (h1) stage_a(g + 1, abuf0 + ((g + 1) & 1) * kTile2Bytes, 1);   // A-hi(g+1)
      if (b2) {                                     // B(g+2) (BAL: its first half)
        char* const bn = bbuf0 + (cb == 0 ? 2 : cb - 1) * kTile2Bytes;
        if (BAL) stage_bh(Z{}, H{}, g + 2, bn);
        else stage_bh(Z{}, F{}, g + 2, bn);
      }
      if (bnd) {
        // A-hi(g) retired by the segment end's drain
      } else if (BAL) {
        if (b2) DLBB_WAIT_VM(12);
        else if (h1) DLBB_WAIT_VM(8);
        else DLBB_WAIT_VM(0);
      } else {
        if (b2) DLBB_WAIT_VM(20);
        else if (h1) DLBB_WAIT_VM(12);
        else DLBB_WAIT_VM(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();                 // end of interval 2g
      __builtin_amdgcn_sched_barrier(0);
      mfma_full(acc, af, bf);
      __builtin_amdgcn_sched_barrier(0);
      if (h1 && !bnd) {
        if (b2) { if (BAL) DLBB_WAIT_VM(8); else DLBB_WAIT_VM(12); }
        else DLBB_WAIT_VM(4);
      }
      __builtin_amdgcn_s_barrier();                 // end of interval 2g+1
      cb = cb == 2 ? 0 : cb + 1;
      if (g == gb - 1 || g == G - 1) {
        DLBB_WAIT_VM(0);
        __builtin_amdgcn_sched_barrier(0);
        finish(g);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    for (int g = 0; g < G; ++g) {
      const bool bnd = g == gb && g > 0;
      read_split_any<false>(abuf0 + (g & 1) * kTile2Bytes, bbuf0 + cb * kTile2Bytes, 1, wc, fr,
                            fq, af, bf);
      const bool l2 = g + 2 < G;
      if (l2) {                                     // A-lo(g+2) (BAL: and B1(g+2))
        stage_a(g + 2, abuf0 + (g & 1) * kTile2Bytes, 0);
        if (BAL) stage_bh(H{}, F{}, g + 2, bbuf0 + (cb == 0 ? 2 : cb - 1) * kTile2Bytes);
      }
      if (g + 1 < G && !bnd) {
        if (l2) { if (BAL) DLBB_WAIT_VM(8); else DLBB_WAIT_VM(4); }
        else DLBB_WAIT_VM(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();                 // end of interval 2g+1
      __builtin_amdgcn_sched_barrier(0);
      mfma_full(acc, af, bf);
      __builtin_amdgcn_sched_barrier(0);
      if (g + 1 < G) __builtin_amdgcn_s_barrier();  // end of interval 2g+2
      cb = cb == 2 ? 0 : cb + 1;
      if (g == gb - 1 || g == G - 1) {
        DLBB_WAIT_VM(0);
        __builtin_amdgcn_sched_barrier(0);
        finish(g);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_streamk(GemmArgs a, SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_streamk_body<false>(a, s, smem);
}
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_256_streamk_bal(GemmArgs a, SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_streamk_body<true>(a, s, smem);
}

// ---------------------------------------------------------------------------------------
// Persistent 256 x 192 ping-pong with the C stores SPREAD under the next tile's K-loop (plain
// bf16 output; autotune candidate `mfma192p`). Built to test whether a tile's C stores, flushed in
// one burst by pp_persist_body at the next tile's first memory interval, cost the GPT-2 LM head
// (16384 x 50304 x 768: 1.65 GB of logits) because they serialise with the counted DMA waits
// (stores and loads share vmcnt). They do not: the K-loop alone takes 0.83 ms and the stores add
// 0.25 ms burst or spread alike (profiles/r04_gemm/SUMMARY.md) — kept as a correct candidate.
// At a tile boundary each lane packs its 96 fp32 accumulators to bf16 pairs and zeroes them;
// EARLY (12 or 18) of its 24 eight-byte stores go out right there (before that iteration's
// loads), the rest (24 / 12 parked VGPRs) kSpi per iteration AFTER that iteration's DMA. Every
// counted wait adds the stores younger than the load it retires (template arguments: one
// immediate per wait; a runtime count measured 13-17 % slower); a spread batch is retired one
// iteration later. 6 or 0 early (36 / 48 parked) spill once the spread iterations are unrolled
// (249 VGPRs at 12). Host contract: N % 192 == 0, M % 16 == 0, K / 64 > the spread iterations.
constexpr int kSpi = 3;
constexpr int spread_iters(int early) { return (24 - early) / kSpi; }

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {   // f(integral_constant<int, B .. E-1>)
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmc() {   // any compile-time count
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool BAL, int EARLY_>
__device__ __forceinline__ void pp192_spread_body(GemmArgs a, char* smem) {
  constexpr int kEarly = EARLY_;
  constexpr int kSpreadIters = spread_iters(kEarly);
  constexpr int NJ = 3, NBI = 6;
  constexpr int NBx = BAL ? NBI / 2 : NBI;      // B instructions of wave row 0 per iteration
  constexpr int kTileB = NJ * 64 * BK * 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = static_cast<int>(a.K / BK);
  const int tiles = static_cast<int>(((a.M + BM2 - 1) / BM2) * (a.N / 192));
  const int nwg = static_cast<int>(gridDim.x), wg = static_cast<int>(blockIdx.x);
  const int mine = wg < tiles ? (tiles - wg + nwg - 1) / nwg : 0;
  if (mine == 0) return;
  const int G = mine * nk;
  char* const abuf0 = smem;
  char* const bbuf0 = smem + 2 * kTile2Bytes;

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], bf[2][NJ];
  const int r_in = lane >> 3, chunk = (lane & 7) ^ (lane >> 3);
  const uint32_t lda2 = static_cast<uint32_t>(a.lda) * 2, ldb2 = static_cast<uint32_t>(a.ldb) * 2;
  const uint32_t aoff = static_cast<uint32_t>(r_in) * lda2 + chunk * 16;
  const uint32_t boff = static_cast<uint32_t>(g48_lane(r_in)) * ldb2 + chunk * 16;
  constexpr uint32_t kStep = BK * 2;
#define DLBB_RSRC(P) \
  __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(P), 0, 0x7fffffff, 0x00020000)
  Tile256 tc = tile_of<192>(a, wg);
  Tile256 tp = tc;                              // the tile whose C is in pk
  Tile256 tprev = tc;                           // the tile finished last
  {
    const __amdgpu_buffer_rsrc_t ra = DLBB_RSRC(a.A + tc.m0 * a.lda);
    const __amdgpu_buffer_rsrc_t rb = DLBB_RSRC(a.B + tc.n0 * a.ldb);
    const int rows_a = static_cast<int>(a.M - tc.m0);
    if (wr == 0) {                              // prologue: A-lo(0), B(0), B(1)
      stage_a_half(ra, lda2, rows_a, 0, abuf0, 0, wc, aoff);
      stage_b192(rb, ldb2, 0, bbuf0, wc, boff);
      stage_b192(rb, ldb2, kStep, bbuf0 + kTileB, wc, boff);
      wait_vm<NBI>();
      __builtin_amdgcn_s_barrier();
    } else {                                    // A-hi(0), A-lo(1)
      stage_a_half(ra, lda2, rows_a, 0, abuf0, 1, wc, aoff);
      stage_a_half(ra, lda2, rows_a, kStep, abuf0 + kTile2Bytes, 0, wc, aoff);
      __builtin_amdgcn_s_barrier();
      DLBB_WAIT_VM(4);
      __builtin_amdgcn_s_barrier();             // end of interval 0
    }
  }
  // lane's C rows / columns within a tile: rows wr*128 + 16 i + fr, columns wc*48 + 12 fq + 4 j;
  // buffer stores from the tile origin: lane offset in one VGPR, the (i, j) part in SGPRs, and a
  // wave-uniform row-block guard (host contract M % 16 == 0)
  const uint32_t ldc2 = static_cast<uint32_t>(a.ldc) * 2;
  const uint32_t c_lane = static_cast<uint32_t>(wr * 128 + fr) * ldc2 + (wc * 48 + fq * 12) * 2;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  // per batch: the tile's resource and the row pitch are re-derived behind empty asm, so the
  // compiler cannot hoist 24 per-store offsets out of the K-loop (that spilled)
  struct CDst { __amdgpu_buffer_rsrc_t rc; uint32_t ld, cl; int64_t rows; };
  auto cdst = [&]() {
    CDst d;
    uint16_t* base = static_cast<uint16_t*>(a.C) + tp.m0 * a.ldc + tp.n0;
    asm volatile("" : "+s"(base));
    d.rc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    d.ld = ldc2;
    asm volatile("" : "+s"(d.ld));
    d.cl = c_lane;
    d.rows = a.M - tp.m0 - wr * 128;
    return d;
  };
  auto store_q = [&](const CDst& d, int q, u32x2 v) {   // q compile-time after unrolling
    const int i = q / 3, j = q % 3;
    if (i * 16 < d.rows)
      __builtin_amdgcn_raw_buffer_store_b64(v, d.rc, d.cl + static_cast<uint32_t>(i * 16) * d.ld + j * 8,
                                            0, 0);
  };
  auto pack = [&](int i, int j) {
    return u32x2{static_cast<uint32_t>(f32_to_bf16(acc[i][j][0])) |
                     (static_cast<uint32_t>(f32_to_bf16(acc[i][j][1])) << 16),
                 static_cast<uint32_t>(f32_to_bf16(acc[i][j][2])) |
                     (static_cast<uint32_t>(f32_to_bf16(acc[i][j][3])) << 16)};
  };
  u32x2 pk[24 - kEarly];                        // the previous tile's spread part, bf16 pairs
  // finished tile tp: store its first kEarly fragments now, park the rest in pk, zero acc
  auto park = [&]() {
    const CDst d = cdst();
#pragma unroll
    for (int q = 0; q < 24; ++q) {
      const u32x2 v = pack(q / 3, q % 3);
      if (q < kEarly) store_q(d, q, v);
      else pk[q - kEarly] = v;
      acc[q / 3][q % 3] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_batch = [&](int it) {              // it: a constant after inlining
    const CDst d = cdst();
#pragma unroll
    for (int q = kEarly; q < 24; ++q)
      if ((q - kEarly) / kSpi == it) store_q(d, q, pk[q - kEarly]);
  };
  auto mfma_all = [&]() {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[x][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][x], acc[x][j], 0,
                                                              0, 0);
  };
  // One K-loop per wave row (as pp_persist_body: a row test inside the loop keeps both rows'
  // temporaries live together and spills). Every store count is a template argument of the
  // iteration, so each counted wait is one immediate (a runtime count measured 13-17 % slower:
  // the compare-and-branch chain sits between the ds_reads and the barrier):
  //   E  = boundary stores issued at the top of this iteration (older than its loads)
  //   SP = spread stores issued in the previous iteration (after its loads)
  //   SC = spread stores issued in this iteration (after its loads), batch IT
  using std::integral_constant;
  auto run = [&](auto row_c) {
    constexpr int ROW = decltype(row_c)::value;
    int cb = 0;
    for (int i = 0; i < mine; ++i) {
      const Tile256 tn = i + 1 < mine ? tile_of<192>(a, wg + (i + 1) * nwg) : tc;
      const __amdgpu_buffer_rsrc_t ra = DLBB_RSRC(a.A + tc.m0 * a.lda);
      const __amdgpu_buffer_rsrc_t rb = DLBB_RSRC(a.B + tc.n0 * a.ldb);
      const __amdgpu_buffer_rsrc_t ran = DLBB_RSRC(a.A + tn.m0 * a.lda);
      const __amdgpu_buffer_rsrc_t rbn = DLBB_RSRC(a.B + tn.n0 * a.ldb);
      const int rows_a = static_cast<int>(a.M - tc.m0), rows_an = static_cast<int>(a.M - tn.m0);
      auto iter = [&](int k, auto e_c, auto sp_c, auto sc_c, auto it_c) {
        constexpr int E = decltype(e_c)::value, SP = decltype(sp_c)::value;
        constexpr int SC = decltype(sc_c)::value, IT = decltype(it_c)::value;
        constexpr int X = E + SP + SC;          // stores younger than every awaited load
        const int g = i * nk + k;
        {
          const char* ab = abuf0 + (g & 1) * kTile2Bytes;
          const char* bb = bbuf0 + cb * kTileB;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int x = 0; x < 8; ++x)
              af[ks][x] = read_frag(ab, ROW * 128 + x * 16 + fr, ks * 4 + fq);
#pragma unroll
            for (int j = 0; j < 3; ++j) bf[ks][j] = read_frag(bb, wc * 48 + j * 16 + fr, ks * 4 + fq);
          }
        }
        if constexpr (ROW == 0) {
          const bool h1 = g + 1 < G, b2 = g + 2 < G;
          if (h1) {                             // A-hi(g+1)
            char* const an = abuf0 + ((g + 1) & 1) * kTile2Bytes;
            if (k + 1 < nk) stage_a_half(ra, lda2, rows_a, (k + 1) * kStep, an, 1, wc, aoff);
            else stage_a_half(ran, lda2, rows_an, 0, an, 1, wc, aoff);
          }
          if (b2) {                             // B(g+2) (BAL: its first half)
            char* const bn = bbuf0 + (cb == 0 ? 2 : cb - 1) * kTileB;
            const bool here = k + 2 < nk;
            const uint32_t k2 = static_cast<uint32_t>(here ? k + 2 : k + 2 - nk) * kStep;
            if (BAL) stage_b192<0, 3>(here ? rb : rbn, ldb2, k2, bn, wc, boff);
            else stage_b192<0, 6>(here ? rb : rbn, ldb2, k2, bn, wc, boff);
          }
          if constexpr (SC > 0) store_batch(IT);   // after the loads: younger than all of them
          // retire A-hi(g): younger = B(g+1), the stores, A-hi(g+1), B(g+2) (g = 0: B(1) is
          // whole, so BAL over-retires its second half there, as pingpong_body)
          if (b2) wait_vmc<2 * NBx + 4 + X>();
          else if (h1) wait_vmc<NBx + 4 + X>();
          else wait_vmc<X>();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();         // end of interval 2g
          __builtin_amdgcn_sched_barrier(0);
          mfma_all();
          __builtin_amdgcn_sched_barrier(0);
          if (h1) {                             // retire B(g+1) (BAL: its first half)
            if (b2) wait_vmc<4 + NBx + X>();
            else wait_vmc<4 + X>();
          }
          __builtin_amdgcn_s_barrier();         // end of interval 2g+1
        } else {
          const bool l2 = g + 2 < G;
          if (l2) {                             // A-lo(g+2) (BAL: and B1(g+2))
            const bool here = k + 2 < nk;
            const int ub = here ? k + 2 : k + 2 - nk;
            stage_a_half(here ? ra : ran, lda2, here ? rows_a : rows_an,
                         static_cast<uint32_t>(ub) * kStep, abuf0 + (g & 1) * kTile2Bytes, 0, wc,
                         aoff);
            if (BAL)
              stage_b192<3, 6>(here ? rb : rbn, ldb2, static_cast<uint32_t>(ub) * kStep,
                               bbuf0 + (cb == 0 ? 2 : cb - 1) * kTileB, wc, boff);
          }
          if constexpr (SC > 0) store_batch(IT);
          if (g + 1 < G) {                      // retire A-lo(g+1) (BAL: and B1(g+1))
            if (l2) wait_vmc<4 + (BAL ? NBI / 2 : 0) + X>();
            else wait_vmc<X>();
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();         // end of interval 2g+1
          __builtin_amdgcn_sched_barrier(0);
          mfma_all();
          __builtin_amdgcn_sched_barrier(0);
          if (g + 1 < G) __builtin_amdgcn_s_barrier();   // end of interval 2g+2
        }
        cb = cb == 2 ? 0 : cb + 1;
      };
      using Z = integral_constant<int, 0>;
      using S = integral_constant<int, kSpi>;
      int k = 0;
      if (i > 0) {                              // boundary + spread iterations (host: nk > them)
        tp = tprev;                             // the finished tile: E early stores,
        __builtin_amdgcn_sched_barrier(0);      // the rest parked in pk (fenced: the next
        park();                                 // ds_reads must not rise above the packing)
        __builtin_amdgcn_sched_barrier(0);
        iter(0, integral_constant<int, kEarly>{}, Z{}, S{}, Z{});
        static_for<1, kSpreadIters>([&](auto it_c) {
          iter(decltype(it_c)::value, Z{}, S{}, S{}, it_c);
        });
        iter(kSpreadIters, Z{}, S{}, Z{}, Z{});
        k = kSpreadIters + 1;
      }
      for (; k < nk; ++k) iter(k, Z{}, Z{}, Z{}, Z{});
      tprev = tc;
      tc = tn;
    }
  };
  if (wr == 0) run(integral_constant<int, 0>{});
  else run(integral_constant<int, 1>{});
  // the last tile: plain epilogue (nothing left to hide it under)
  DLBB_WAIT_VM(0);
  tp = tprev;
  park();
#pragma unroll
  for (int it = 0; it < kSpreadIters; ++it) store_batch(it);
#undef DLBB_RSRC
}

template <int EARLY>
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_192_pp_spread(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp192_spread_body<false, EARLY>(a, smem);
}
template <int EARLY>
__global__ void __launch_bounds__(kThreads2, 1) gemm_bf16_nt_192_pp_spread_bal(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp192_spread_body<true, EARLY>(a, smem);
}


}  // namespace dlbb

using namespace dlbb;

// Launch a ping-pong kernel, or its stamped twin when stamping is on (dlbb_stamps_set).
#define DLBB_PP_LAUNCH(KERNEL, KIND, GRID, ARGS)                                          \
  do {                                                                                   \
    const dim3 g_(GRID);                                                                 \
    uint64_t* st_ = stamp_acquire(KIND, static_cast<int64_t>(g_.x) * g_.y);              \
    if (st_)                                                                             \
      hipLaunchKernelGGL(KERNEL##_st, g_, dim3(kThreads2), kPP6Lds, stream, ARGS, st_);  \
    else                                                                                 \
      hipLaunchKernelGGL(KERNEL, g_, dim3(kThreads2), kPP6Lds, stream, ARGS);            \
  } while (0)

static int dlbb_gemm_force_tile = 0;   // 0 = heuristic, 128 or 256 = force (A/B testing)

// compute units of the current device (cached per device): persistent grids
static int num_cus() {
  static int ncu[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (ncu[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    ncu[dev] = n;
  }
  return ncu[dev];
}

// 256^2 schedule (set_stagger): 6 = ping-pong (160 KiB LDS, measured fastest; the default),
// 10 = its persistent form on multi-round grids (the default's upgrade, see below), 3 = the
// deep-pipeline general-contract kernel (forced for A/B; also every ragged shape's fallback)
static int dlbb_gemm_stagger = 6;
// Balanced DMA issue (BAL) for the ping-pong kernels: 0 never, 1 always, 2 (default) = always
// for NN (dgrad: +1-5 % on every measured shape, K 768 .. 50304) and for NT when the reduction
// has >= kBalMinKTiles K-tiles (NT: +1-5 % at K >= 2048, -1.5 % at K = 768)
// (profiles/r02_gemm/gemm_ab_pingpong_bal.jsonl, dgrad_ab_nn_bal.jsonl)
static int dlbb_gemm_bal = 2;
constexpr int64_t kBalMinKTiles = 32;
constexpr int64_t kPersistMaxKTiles = 48;
// > 0 while GEMMs share the chip with communication kernels on another stream (the overlapped TP
// forward, ops.gemm.concurrent_comm): the persistent forms assume all num_cus workgroups are
// co-resident, and comm workgroups holding CUs push part of such a grid into a second round
// (the same slowdown as hipBLASLt's persistent Stream-K there), so they are off meanwhile
static int dlbb_gemm_concurrent = 0;
static bool persist_enabled() { return dlbb_gemm_concurrent <= 0; }
// dlbb_gemm_set_persist_epi(0): keep bias / bias-GELU epilogues on the non-persistent
// ping-pong (A/B)
static int dlbb_persist_epi = 1;
static bool persist_epi_enabled() { return dlbb_persist_epi != 0; }
static bool use_bal(int64_t k_tiles, bool nn) {
  return dlbb_gemm_bal == 1 || (dlbb_gemm_bal == 2 && (nn || k_tiles >= kBalMinKTiles));
}

DLBB_API void dlbb_gemm_set_tile(int tile) { dlbb_gemm_force_tile = tile; }
DLBB_API void dlbb_gemm_set_stagger(int on) { dlbb_gemm_stagger = on; }
DLBB_API int dlbb_gemm_get_stagger() { return dlbb_gemm_stagger; }
DLBB_API void dlbb_gemm_set_persist_epi(int on) { dlbb_persist_epi = on ? 1 : 0; }
DLBB_API void dlbb_gemm_set_concurrent(int on) { dlbb_gemm_concurrent = on; }
DLBB_API int dlbb_gemm_get_concurrent() { return dlbb_gemm_concurrent; }
DLBB_API void dlbb_gemm_set_bal(int mode) { dlbb_gemm_bal = mode >= 0 && mode <= 2 ? mode : 2; }

// ---------------------------------------------------------------------------------------
// Stream-K plan (pp_streamk_body) for an NT shape on `ncu` CUs: out = {grid, L, ws bytes,
// counters}; returns 0 when the shape is outside the Stream-K contract (256² tiles below one
// round of the CUs, >= 8 K-tiles per tile). Every range is >= kSkMinL K-tiles long (the
// combine of a split tile costs about a tile's partial block per extra contributor, so very
// short ranges do not pay) and no range is a single K-tile (the prologue stages two).
constexpr int kSkMinL = 8;
DLBB_API int dlbb_gemm_streamk_plan(int64_t M, int64_t N, int64_t K, int ncu, int64_t* out) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0 || ncu <= 0) return 0;
  const int64_t tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
  const int64_t nk = K / BK;
  if (nk < kSkMinL || tiles >= ncu) return 0;
  const int64_t iters = tiles * nk;
  int64_t grid = iters / kSkMinL < ncu ? iters / kSkMinL : ncu;
  if (grid < 2) return 0;
  int64_t L = (iters + grid - 1) / grid;
  while (iters % L == 1) ++L;          // no one-K-tile range
  if (L > nk) return 0;                // (cannot happen for tiles < ncu) a range spans <= 2 tiles
  grid = (iters + L - 1) / L;
  out[0] = grid;
  out[1] = L;
  out[2] = 2 * grid * 8 * 32768;       // two partial slots per workgroup, 8 waves x 32 KiB
  out[3] = tiles * 8;                  // (tile, wave) arrival counters
  return 1;
}

// Stream-K NT GEMM, the same result contract as dlbb_gemm_bf16_nt (every epilogue); `ws` /
// `cnt` as planned by dlbb_gemm_streamk_plan(..., ncu = grid owner's CU count), cnt ZERO on
// entry (left zero). Host contract as the ping-pong: M % 8 == 0, N % 64 == 0, 16-B aligned
// A / B / ws rows, 32-bit offsets within a 256-row panel.
DLBB_API int dlbb_gemm_bf16_nt_streamk(const void* A, int64_t lda, const void* B, int64_t ldb,
                                       void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                       const void* bias, const void* residual, int64_t ldr,
                                       void* preact, int epi, int out_f32, int ncu, void* ws,
                                       int64_t ws_bytes, int* cnt, int64_t ncnt,
                                       hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  int64_t plan[4];
  if (!dlbb_gemm_streamk_plan(M, N, K, ncu, plan)) return hipErrorInvalidValue;
  if (!ws || !cnt || ws_bytes < plan[2] || ncnt < plan[3]) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || M % 8 || N % 64 || M < 8) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) |
       reinterpret_cast<uintptr_t>(ws)) & 15)
    return hipErrorInvalidValue;
  if (lda * 2 * 256 + K * 2 >= (1LL << 31) || ldb * 2 * 256 + K * 2 >= (1LL << 31) ||
      plan[2] >= (1LL << 32))
    return hipErrorInvalidValue;
  if ((epi & EPI_BIAS) && !bias) return hipErrorInvalidValue;
  if ((epi & EPI_READS_R) && !residual) return hipErrorInvalidValue;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec_ok = (ldc % 8 == 0) && al16(C) && (!preact || al16(preact)) &&
                     (!(epi & EPI_READS_R) || (ldr % 8 == 0 && al16(residual))) &&
                     (!(epi & EPI_BIAS) || al16(bias));
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C,
             static_cast<const uint16_t*>(bias), static_cast<const uint16_t*>(residual),
             static_cast<uint16_t*>(preact), M, N, K, lda, ldb, ldc, ldr, epi, out_f32,
             vec_ok, 0};
  SkArgs s{static_cast<float*>(ws), cnt, static_cast<int>(plan[1]), static_cast<int>(K / BK)};
  const dim3 g(static_cast<unsigned>(plan[0])), b(kThreads2);
  if (use_bal(plan[1], false))
    hipLaunchKernelGGL(gemm_bf16_nt_256_streamk_bal, g, b, kPP6Lds, stream, a, s);
  else
    hipLaunchKernelGGL(gemm_bf16_nt_256_streamk, g, b, kPP6Lds, stream, a, s);
  return hipGetLastError();
}

// Diagnostic: one plain bf16 NT GEMM on the balanced ping-pong (nj = 4: 256², 3: 256 x 192) with
// per-workgroup phase stamps (4 u64 each: start, first MFMA, K-loop end, stores end) into recs
// (gridDim.x records). Contract as the ping-pong; no autotuning, no epilogue.
DLBB_API int dlbb_gemm_nt_phase_probe(const void* A, int64_t lda, const void* B, int64_t ldb,
                                      void* C, int64_t M, int64_t N, int64_t K, int nj,
                                      uint64_t* recs, hipStream_t stream) {
  if (M % 8 || (nj == 3 ? N % 192 : N % 64) || K % BK || K < 2 * BK || !recs)
    return hipErrorInvalidValue;
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C, nullptr,
             nullptr, nullptr, M, N, K, lda, ldb, N, 0, 0, 0, 1, 0};
  const int64_t tiles = ((M + BM2 - 1) / BM2) * ((N + 64 * nj - 1) / (64 * nj));
  if (nj == 3)
    hipLaunchKernelGGL(gemm_nt_pp192_phases, dim3(static_cast<unsigned>(tiles)), dim3(kThreads2),
                       kPP192Lds, stream, a, recs);
  else
    hipLaunchKernelGGL(gemm_nt_pp_phases, dim3(static_cast<unsigned>(tiles)), dim3(kThreads2),
                       kPP6Lds, stream, a, recs);
  return hipGetLastError();
}

// NT GEMM with an explicit kernel variant (the autotuner's candidates, ops/gemm.py):
//   0 = the size heuristic below (256² ping-pong / persistent / 128² small grids)
//   1 = 256 x 192 ping-pong tiles (N % 192 == 0, M % 8 == 0; otherwise variant 0)
//   2 = persistent 256 x 192 with the C stores spread under the next tile (plain bf16 output;
//       otherwise variant 1)
DLBB_API int dlbb_gemm_bf16_nt_v(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                                 const void* residual, int64_t ldr, void* preact, int epi,
                                 int out_f32, int variant, hipStream_t stream);

DLBB_API int dlbb_gemm_bf16_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                               const void* residual, int64_t ldr, void* preact, int epi,
                               int out_f32, hipStream_t stream) {
  return dlbb_gemm_bf16_nt_v(A, lda, B, ldb, C, ldc, M, N, K, bias, residual, ldr, preact, epi,
                             out_f32, 0, stream);
}

DLBB_API int dlbb_gemm_bf16_nt_v(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                                 const void* residual, int64_t ldr, void* preact, int epi,
                                 int out_f32, int variant, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % BK != 0) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8) return hipErrorInvalidValue;          // 16-byte rows for glds
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    return hipErrorInvalidValue;
  if ((epi & EPI_BIAS) && !bias) return hipErrorInvalidValue;
  if ((epi & EPI_READS_R) && !residual) return hipErrorInvalidValue;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec_ok = (ldc % 8 == 0) && al16(C) && (!preact || al16(preact)) &&
                     (!(epi & EPI_READS_R) || (ldr % 8 == 0 && al16(residual))) &&
                     (!(epi & EPI_BIAS) || al16(bias));
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C,
             static_cast<const uint16_t*>(bias), static_cast<const uint16_t*>(residual),
             static_cast<uint16_t*>(preact), M, N, K, lda, ldb, ldc, ldr, epi, out_f32,
             vec_ok, 0};
  const int64_t tiles256 = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
  // variant 2: persistent 256 x 192 with spread C stores (plain bf16 output only, >= 9 K-tiles,
  // 8-byte aligned rows; pp192_spread_body); anything else falls back to variant 1
  if (variant == 2 && epi == 0 && !preact && !out_f32 && vec_ok && persist_enabled() &&
      N % 192 == 0 && M % 16 == 0 && M >= 16 && K / BK >= spread_iters(12) + 2 &&
      lda * 2 * 256 + K * 2 < (1LL << 31) && ldb * 2 * 192 + K * 2 < (1LL << 31)) {
    const int64_t tiles = ((M + BM2 - 1) / BM2) * (N / 192);
    const int64_t grid = tiles < num_cus() ? tiles : num_cus();
    const dim3 g(static_cast<unsigned>(grid)), b(kThreads2);
    const bool bal = use_bal(K / BK, false);
    if (bal) hipLaunchKernelGGL(gemm_bf16_nt_192_pp_spread_bal<12>, g, b, kPP192Lds, stream, a);
    else hipLaunchKernelGGL(gemm_bf16_nt_192_pp_spread<12>, g, b, kPP192Lds, stream, a);
    return hipGetLastError();
  }
  if (variant == 2) variant = 1;
  if (variant == 1 && N % 192 == 0 && M % 8 == 0 && M >= 8 &&
      lda * 2 * 256 + K * 2 < (1LL << 31) && ldb * 2 * 192 + K * 2 < (1LL << 31)) {
    const dim3 g(static_cast<unsigned>(((M + BM2 - 1) / BM2) * (N / 192))), b(kThreads2);
    if (use_bal(K / BK, false))
      hipLaunchKernelGGL(gemm_bf16_nt_192_pingpong3_bal, g, b, kPP192Lds, stream, a);
    else
      hipLaunchKernelGGL(gemm_bf16_nt_192_pingpong3, g, b, kPP192Lds, stream, a);
    return hipGetLastError();
  }
  // the 256^2 schedule needs >= ~1 workgroup per CU to fill the chip; otherwise 128^2 tiles
  const int force = dlbb_gemm_force_tile;
  if (force == 256 || (force != 128 && tiles256 >= 192)) {
    const dim3 g(static_cast<unsigned>(tiles256)), b(kThreads2);
    int mode = dlbb_gemm_stagger == 10 || dlbb_gemm_stagger == 3 ? dlbb_gemm_stagger : 6;
    // default ping-pong on a multi-round grid with a short reduction: the persistent form
    // (tools/gemm_ab.py, profiles/r03_gemm/persistent_ab.jsonl, plain bf16: +6.6 % at
    // 16384 x 3072 x 768, +10.6 % GPT-2 LM head; neutral at K = 4096 over 3 rounds; -2 % on
    // one-round grids)
    // lean epilogue kinds (bf16 output, vector stores, nothing read but the bias): plain, bias,
    // bias -> GELU with an optional pre-activation store; -1 = the general epilogue only
    int lean = -1;
    if (!out_f32 && vec_ok) {
      if (epi == 0 && !preact) lean = PP_PLAIN;
      else if (epi == EPI_BIAS && !preact) lean = PP_BIAS;
      else if (epi == (EPI_BIAS | EPI_GELU_TANH)) lean = PP_BIAS_GELU_TANH;
      else if (epi == (EPI_BIAS | EPI_GELU_ERF)) lean = PP_BIAS_GELU_ERF;
    }
    if (lean > PP_PLAIN && !persist_epi_enabled()) lean = -1;
    if (mode == 6 && lean >= 0 && persist_enabled() && tiles256 > num_cus() &&
        K / BK <= kPersistMaxKTiles)
      mode = 10;
    // persistent ping-pong (mode 10): the ping-pong contract, at least two K-tiles and a lean
    // epilogue
    if (mode == 10 && (K < 2 * BK || lean < 0)) mode = 6;
    // ping-pong contract: 8-row A groups and 64-row B blocks wholly in or out (uniform clamps),
    // 32-bit buffer offsets within a 256-row panel; otherwise the deep-pipeline kernel
    if ((mode == 6 || mode == 10) &&
        !(M % 8 == 0 && N % 64 == 0 && M >= 8 && lda * 2 * 256 + K * 2 < (1LL << 31) &&
          ldb * 2 * 256 + K * 2 < (1LL << 31)))
      mode = 3;
    if (mode == 10) {
      const int64_t grid = tiles256 < num_cus() ? tiles256 : num_cus();
      const dim3 gp(static_cast<unsigned>(grid)), bp(kThreads2);
      const bool bal = use_bal(K / BK, false);
#define DLBB_PP_PERSIST_LAUNCH(L)                                                          \
  do {                                                                                     \
    if (bal) hipLaunchKernelGGL(gemm_bf16_nt_256_pp_persist_bal<L>, gp, bp, kPP6Lds, stream, a); \
    else hipLaunchKernelGGL(gemm_bf16_nt_256_pp_persist<L>, gp, bp, kPP6Lds, stream, a);   \
  } while (0)
      switch (lean) {
        case PP_BIAS: DLBB_PP_PERSIST_LAUNCH(PP_BIAS); break;
        case PP_BIAS_GELU_TANH: DLBB_PP_PERSIST_LAUNCH(PP_BIAS_GELU_TANH); break;
        case PP_BIAS_GELU_ERF: DLBB_PP_PERSIST_LAUNCH(PP_BIAS_GELU_ERF); break;
        default: DLBB_PP_PERSIST_LAUNCH(PP_PLAIN); break;
      }
#undef DLBB_PP_PERSIST_LAUNCH
      return hipGetLastError();
    }
    if (mode == 6 && use_bal(K / BK, false))
      DLBB_PP_LAUNCH(gemm_bf16_nt_256_pingpong3_bal, STAMP_GEMM_NT, g, a);
    else if (mode == 6)
      DLBB_PP_LAUNCH(gemm_bf16_nt_256_pingpong3, STAMP_GEMM_NT, g, a);
    else
      hipLaunchKernelGGL(gemm_bf16_nt_256_deep, g, b, 2 * kBuf2Bytes, stream, a);
    return hipGetLastError();
  }
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm_bf16_nt_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kThreads),
                     4 * kTileBytes, stream, a);
  return hipGetLastError();
}

// split-K partial reduce + cast (csrc/gemm_tn.hip): out[i] = sum_s ws[s * n + i]
int dlbb_split_reduce_launch(const float* ws, void* out, int dt_f32, int64_t n, int split,
                             hipStream_t stream);

// dgrad GEMM: C[M, N] = epilogue(A[M, K] · B[K, N]), B row-major [K][N] (a Linear weight
// [out, in] is exactly this for dX = dY · W). Ping-pong 256^2 schedule with transposed-read B.
DLBB_API int dlbb_gemm_bf16_nn(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                               const void* residual, int64_t ldr, void* preact, int epi,
                               int out_f32, int split, float* ws, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % BK != 0 || N % BN2 != 0 || M % 8 != 0) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || ldb < N || lda < K) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    return hipErrorInvalidValue;
  // 32-bit buffer offsets: a 256-row panel of A, all K rows of B
  if (lda * 2 * 256 + K * 2 >= (1LL << 31) || K * ldb * 2 >= (1LL << 31))
    return hipErrorInvalidValue;
  if ((epi & EPI_BIAS) && !bias) return hipErrorInvalidValue;
  if ((epi & EPI_READS_R) && !residual) return hipErrorInvalidValue;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec_ok = (ldc % 8 == 0) && al16(C) && (!preact || al16(preact)) &&
                     (!(epi & EPI_READS_R) || (ldr % 8 == 0 && al16(residual))) &&
                     (!(epi & EPI_BIAS) || al16(bias));
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C,
             static_cast<const uint16_t*>(bias), static_cast<const uint16_t*>(residual),
             static_cast<uint16_t*>(preact), M, N, K, lda, ldb, ldc, ldr, epi, out_f32,
             vec_ok, 0};
  const int64_t tiles256 = ((M + BM2 - 1) / BM2) * (N / BN2);
  const int nkt = static_cast<int>(K / BK);
  if (split > 1) {
    // split-K for grids below one workgroup per CU (the LM-head dX: 192 tiles, 786 K-tiles):
    // fp32 partials [split][M][N] in ws, then one reduce + bf16 cast pass. Plain product only.
    if (!ws || epi != 0 || out_f32 || ldc != N || split > nkt) return hipErrorInvalidValue;
    a.kt_split = (nkt + split - 1) / split;
    split = (nkt + a.kt_split - 1) / a.kt_split;   // every slice starts inside the reduction
    a.C = ws;
    a.out_f32 = 1;
    a.vec_ok = (reinterpret_cast<uintptr_t>(ws) & 15) == 0 && N % 8 == 0;
    if (use_bal(a.kt_split, true))
      DLBB_PP_LAUNCH(gemm_bf16_nn_256_pingpong3_bal, STAMP_GEMM_NN,
                     dim3(static_cast<unsigned>(tiles256), split), a);
    else
      DLBB_PP_LAUNCH(gemm_bf16_nn_256_pingpong3, STAMP_GEMM_NN,
                     dim3(static_cast<unsigned>(tiles256), split), a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return dlbb_split_reduce_launch(ws, C, 0, M * N, split, stream);
  }
  // multi-round grid with a short reduction: the persistent form (plain bf16 or the GELU
  // backward, operands of the epilogue prefetched before the DMA drain; the GPT-2 MLP-proj dX,
  // 768 tiles x 12 K-tiles)
  if (persist_enabled() && persist_epi_enabled() && tiles256 > num_cus() && nkt >= 2 &&
      nkt <= kPersistMaxKTiles && use_bal(nkt, true) && !out_f32 && vec_ok && !preact) {
    const int lean = epi == 0 ? PP_PLAIN
                     : epi == EPI_DGELU_TANH ? PP_DGELU_TANH
                     : epi == EPI_DGELU_ERF ? PP_DGELU_ERF : -1;
    const dim3 gp(static_cast<unsigned>(num_cus())), bp(kThreads2);
    switch (lean) {
      case PP_PLAIN:
        hipLaunchKernelGGL(gemm_bf16_nn_256_pp_persist_bal<PP_PLAIN>, gp, bp, kPP6Lds, stream, a);
        return hipGetLastError();
      case PP_DGELU_TANH:
        hipLaunchKernelGGL(gemm_bf16_nn_256_pp_persist_bal<PP_DGELU_TANH>, gp, bp, kPP6Lds,
                           stream, a);
        return hipGetLastError();
      case PP_DGELU_ERF:
        hipLaunchKernelGGL(gemm_bf16_nn_256_pp_persist_bal<PP_DGELU_ERF>, gp, bp, kPP6Lds,
                           stream, a);
        return hipGetLastError();
      default:
        break;
    }
  }
  if (use_bal(nkt, true))
    DLBB_PP_LAUNCH(gemm_bf16_nn_256_pingpong3_bal, STAMP_GEMM_NN,
                   dim3(static_cast<unsigned>(tiles256)), a);
  else
    DLBB_PP_LAUNCH(gemm_bf16_nn_256_pingpong3, STAMP_GEMM_NN,
                   dim3(static_cast<unsigned>(tiles256)), a);
  return hipGetLastError();
}

// Split-K NT GEMM, plain product to bf16 (C = A · B^T, ldc == N): the ping-pong on
// (tiles, split) with fp32 partials [split][M][N] in ws, then one reduce + cast pass
// (dlbb_split_reduce_launch). For grids below one round of the CUs — the TP-7B shard
// projections (4096 x 1536 x 4096 at P = 8: 128 tiles of 256 x 192 -> 256 workgroups at
// split 2) — where a whole-K tile per workgroup leaves half the chip idle and the in-launch
// Stream-K combine measured slower (profiles/r06_kernels/tp_gemm_table_streamk.jsonl).
// tile192: 256 x 192 tiles (N % 192 == 0), else 256^2. ws: >= split * M * N fp32, 16-B aligned.
DLBB_API int dlbb_gemm_bf16_nt_split(const void* A, int64_t lda, const void* B, int64_t ldb,
                                     void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                     int split, int tile192, float* ws, int64_t ws_bytes,
                                     hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % BK != 0 || split < 2 || ldc != N) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || M % 8 || M < 8 || N % 64) return hipErrorInvalidValue;
  if (tile192 && N % 192) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) |
       reinterpret_cast<uintptr_t>(ws)) & 15)
    return hipErrorInvalidValue;
  const int bn = tile192 ? 192 : BN2;
  if (lda * 2 * 256 + K * 2 >= (1LL << 31) || ldb * 2 * bn + K * 2 >= (1LL << 31))
    return hipErrorInvalidValue;
  const int nkt = static_cast<int>(K / BK);
  if (split > nkt) return hipErrorInvalidValue;
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), ws, nullptr,
             nullptr, nullptr, M, N, K, lda, ldb, N, 0, 0, 1, N % 8 == 0 ? 1 : 0, 0};
  a.kt_split = (nkt + split - 1) / split;
  split = (nkt + a.kt_split - 1) / a.kt_split;   // every slice starts inside the reduction
  if (!ws || ws_bytes < static_cast<int64_t>(split) * M * N * 4) return hipErrorInvalidValue;
  const int64_t tiles = ((M + BM2 - 1) / BM2) * ((N + bn - 1) / bn);
  const dim3 g(static_cast<unsigned>(tiles), static_cast<unsigned>(split)), b(kThreads2);
  const bool bal = use_bal(a.kt_split, false);
  if (tile192) {
    if (bal) hipLaunchKernelGGL(gemm_bf16_nt_192_pingpong3_bal, g, b, kPP192Lds, stream, a);
    else hipLaunchKernelGGL(gemm_bf16_nt_192_pingpong3, g, b, kPP192Lds, stream, a);
  } else {
    if (bal) DLBB_PP_LAUNCH(gemm_bf16_nt_256_pingpong3_bal, STAMP_GEMM_NT, g, a);
    else DLBB_PP_LAUNCH(gemm_bf16_nt_256_pingpong3, STAMP_GEMM_NT, g, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return dlbb_split_reduce_launch(ws, C, 0, M * N, split, stream);
}

// weight-gradient GEMM on the 256^2 ping-pong: C[M, N] = epilogue(A[K, M]^T · B[K, N]) with
// A = dY [tokens][lda] and B = X [tokens][ldb], both read as transposed LDS images (no transpose
// pass). epi: 0 or EPI_RESIDUAL (accumulate: residual = the bf16 output itself). One workgroup
// per 256^2 output tile, the whole reduction in-kernel (dW stored directly, no fp32 partials).
// split > 1: fp32 partials [split][M][N] in ws + one reduce/cast pass (plain product, ldc == N) —
// for grids that leave a partial last round (the LM-head dW's tail rows).
DLBB_API int dlbb_gemm_bf16_tn(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, const void* residual,
                               int64_t ldr, int epi, int out_f32, int split, float* ws,
                               hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % BK != 0 || M % 128 != 0 || N % BN2 != 0) return hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    return hipErrorInvalidValue;
  // 32-bit buffer offsets over all K rows of both operands
  if (K * lda * 2 >= (1LL << 31) || K * ldb * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  if (epi != 0 && epi != EPI_RESIDUAL) return hipErrorInvalidValue;
  if (epi == EPI_RESIDUAL && (!residual || out_f32)) return hipErrorInvalidValue;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec_ok = (ldc % 8 == 0) && al16(C) && (epi == 0 || (ldr % 8 == 0 && al16(residual)));
  GemmArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C, nullptr,
             static_cast<const uint16_t*>(residual), nullptr, M, N, K, lda, ldb, ldc, ldr, epi,
             out_f32, vec_ok, 0};
  const int64_t tiles256 = ((M + BM2 - 1) / BM2) * (N / BN2);
  const int nkt = static_cast<int>(K / BK);
  if (split > 1) {
    if (!ws || epi != 0 || ldc != N || split > nkt || (reinterpret_cast<uintptr_t>(ws) & 15))
      return hipErrorInvalidValue;
    const int dt_f32 = out_f32;
    a.kt_split = (nkt + split - 1) / split;
    split = (nkt + a.kt_split - 1) / a.kt_split;   // every slice starts inside the reduction
    a.C = ws;
    a.out_f32 = 1;
    a.vec_ok = N % 8 == 0;
    const dim3 g(static_cast<unsigned>(tiles256), static_cast<unsigned>(split));
    if (use_bal(a.kt_split, true))
      DLBB_PP_LAUNCH(gemm_bf16_tn_256_pingpong3_bal, STAMP_GEMM_TN, g, a);
    else
      DLBB_PP_LAUNCH(gemm_bf16_tn_256_pingpong3, STAMP_GEMM_TN, g, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return dlbb_split_reduce_launch(ws, C, dt_f32, M * N, split, stream);
  }
  if (use_bal(nkt, true))
    DLBB_PP_LAUNCH(gemm_bf16_tn_256_pingpong3_bal, STAMP_GEMM_TN,
                   dim3(static_cast<unsigned>(tiles256)), a);
  else
    DLBB_PP_LAUNCH(gemm_bf16_tn_256_pingpong3, STAMP_GEMM_TN,
                   dim3(static_cast<unsigned>(tiles256)), a);
  return hipGetLastError();
}
