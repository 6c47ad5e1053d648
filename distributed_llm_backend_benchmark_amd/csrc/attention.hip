// Causal flash-attention forward for gfx950 (bf16 in/out, fp32 softmax), head dim 64.
//
// Used by the GPT-2 DDP microbenchmark (models/gpt2.py); the reference model has no real
// attention (models.py:162-167 slices QKV), so this kernel goes beyond parity: it replaces the
// library flash kernel on the training path's second-largest cost (profiles/r01_gpt2).
//
// Inputs are read straight out of the fused QKV activation [B, T, 3, H, D] (row stride ld
// elements); the output is written as [B, T, H, D] (row stride ldo) so it feeds the
// projection GEMM without a transpose, and the per-row log-sum-exp (natural log, [B, H, T] fp32)
// is what the backward consumes.
//
// Structure (CDNA guide §B "Fused attention prefill", §3 "An accumulator tile as the next
// MFMA's operand", T10):
//   * workgroup = 4 waves = 128 queries of one (b, h); wave w owns 32 queries. Query blocks are
//     launched heaviest first (causal work grows with the block index).
//   * K/V tiles of 64 keys are staged by LDS-DMA (global_load_lds 16 B), double buffered; the
//     K image is XOR-swizzled for the ds_read_b128 row reads, the V image for the
//     ds_read_b64_tr_b16 transposed reads (both conflict-free: see kswz / vswz).
//   * swapped scores: S^T = K Q^T with v_mfma_f32_32x32x16_bf16, so a lane owns ONE query
//     (lane & 31) and 16 keys per 32-key tile; the row max / sum are lane-local plus one
//     exchange with lane ^ 32. exp2 with log2(e)/sqrt(D) folded into the scale.
//   * O^T = V^T P^T: P^T (the S^T accumulator, cvt to bf16) is directly the B operand (keys are
//     the k index); V^T comes from the transposed LDS read. O^T stays in 32 fp32 registers.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace dlbb {

constexpr int kAttnD = 64;
constexpr int kQB = 128;        // queries per workgroup
constexpr int kKB = 64;         // keys per tile
constexpr int kAttnThreads = 256;
constexpr int kTileKV = kKB * kAttnD * 2;   // 8 KiB

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16-B chunk c (0..7) of LDS row r is stored in slot c ^ swz(r)
__device__ __forceinline__ int kswz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int vswz(int r) { return ((r >> 1) & 1) << 2; }

__device__ __forceinline__ void attn_glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_vptr_t)(lds), 16, 0, 0);
}

struct AttnArgs {
  const uint16_t* qkv;   // [B, T, 3, H, D]
  uint16_t* out;         // [B, T, H, D] with row stride ldo
  float* lse;            // [B, H, T]
  int64_t ld, ldo;       // token row strides (elements)
  int B, T, H;
  float scale_log2;      // log2(e) / sqrt(D)
  int xcd;               // 1: XCD-aware head-contiguous block order (head_block)
  uint64_t* stamps;      // diagnostic, normally null: wg_stamp per workgroup
};

// Block -> (block-in-head, h, b) for a (blocks-per-head, H, B) grid. xcd = 1: XCD-aware
// bijective remap (guide T1; blockIdx % 8 labels the blocks that share an L2) so each XCD's
// eighth of the grid is a contiguous run of WHOLE heads — a head's K/V (forward, dQ) or Q/dO
// (dK/dV) tiles are then fetched into one L2 instead of into all eight (the default dispatch
// sends the consecutive blocks of one head to eight different XCDs). Order inside a head kept.
__device__ __forceinline__ void head_block(int xcd_on, int& blk, int& h, int& b) {
  const int nb = gridDim.x, H = gridDim.y;
  if (!xcd_on) {
    blk = blockIdx.x;
    h = blockIdx.y;
    b = blockIdx.z;
    return;
  }
  const int nwg = nb * H * gridDim.z;
  const int L = blockIdx.x + nb * (blockIdx.y + H * blockIdx.z);
  const int x = L % 8, q = nwg / 8, r = nwg % 8;
  const int wid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / 8;
  blk = wid % nb;
  const int hh = wid / nb;
  h = hh % H;
  b = hh / H;
}

// lane ^ 32 half exchange of a per-lane value by v_permlane32_swap (a VALU op) instead of a
// ds_bpermute LDS round trip; max over both halves ends in every lane
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Diagnostic workgroup timeline (dlbb_attn_set_stamps; null in production): slot k of the
// launch-order workgroup's 4 words gets the 100 MHz wall clock (k = 0 start, 1 end of the first
// causal pass, 2 end) and, with k = 0, word 3 = XCC id << 16 | HW_ID's SE / SH / CU fields —
// the residency and balance of the grid on the chip, without PMC (tools/attn_timeline.py).
// A vector store from thread 0.
__device__ __forceinline__ void wg_stamp(uint64_t* st, int k) {
  if (!st) return;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  uint64_t* p = st + 4 * static_cast<int64_t>(L);
  p[k] = static_cast<uint64_t>(wall_clock64());
  if (k == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    p[3] = (static_cast<uint64_t>(xcc & 0xf) << 16) | ((hw >> 8) & 0xffff);
  }
}

// Forward tile geometry per head dim: one 8-KiB image per K / V tile — 64 keys x 128 B at
// D = 64, 32 keys x 256 B at D = 128 (the TP model's heads, models/tp_transformer.py) — so both
// keep 32 KiB of LDS per workgroup (double-buffered K and V) and 2 DMA wave-instructions per
// wave per image.
template <int D>
struct FwdGeo {
  static constexpr int KB = 8192 / (2 * D);   // keys per tile
  static constexpr int NKK = KB / 32;         // 32-key halves per tile
  static constexpr int NKS = D / 16;          // k-steps of S^T = K Q^T
  static constexpr int NDT = D / 32;          // 32-dim blocks of O^T
  static constexpr int ROW = 2 * D;           // image row bytes
  static constexpr int RPI = 1024 / ROW;      // rows per DMA wave-instruction
  static constexpr int TILE = KB * ROW;       // 8 KiB
};
// K image (ds_read_b128 row reads) and V image (ds_read_b64_tr_b16) swizzles: 16-B chunk c of
// row r in slot c ^ swz(r). D = 64 (128-B rows): kswz / vswz above. D = 128 (256-B rows: every
// row covers all 64 banks): r & 15 makes the 16 rows of each ds_read_b128 lane group hit 16
// distinct bank quads; (r & 3) << 2 puts the 4 rows of a transposed read's 32-lane group in 4
// distinct 64-B bank segments.
template <int D>
__device__ __forceinline__ int kswz_d(int r) { return D == 64 ? kswz(r) : (r & 15); }
template <int D>
__device__ __forceinline__ int vswz_d(int r) { return D == 64 ? vswz(r) : ((r & 3) << 2); }

// Causal forward, head dim D (64 or 128). Round-5 schedule (variant 6 of its A/B: row-max
// exchange by v_permlane32_swap, incremental DMA sources; 128 VGPRs at D = 64 then, 139 since
// the round-6 pairing and deferred max = 3 waves per SIMD: the paired GPT-2 grid of 768
// workgroups is exactly one round of 3 per CU). Round 6 measured a software-pipelined body (QK^T of tile j+1 and PV of tile j-1 beside
// the softmax of tile j in one straight block): 75.1 vs 56.5 us at the GPT-2 shape — its 212
// VGPRs left 2 waves per SIMD, and the hardware's interleave of 4 waves beat the compiler's
// in-wave interleave (profiles/r06_kernels/attn_fwd_pipelined_ab.jsonl); removed. Also measured
// and removed (commit 62e38ff, profiles/r06_kernels/attn_fwd_shape_ab.jsonl, bit-identical
// outputs): 8 waves / 256 queries per workgroup sharing each K/V tile (55.97 vs 50.81 us at the
// GPT-2 shape; 84 vs 58 at D = 128) and a 3-deep K/V ring with asm LDS reads and counted waits,
// so no DMA drain at the first V read (59.3 us): this loop is not DMA-latency bound.
template <int D>
__global__ void __launch_bounds__(kAttnThreads, 2) attn_fwd_kernel(AttnArgs a) {
  using G = FwdGeo<D>;
  constexpr int KB = G::KB, ROW = G::ROW, RPI = G::RPI, TILE = G::TILE;
  constexpr int WROWS = KB / 4;                   // image rows staged per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nqb = (a.T + kQB - 1) / kQB;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  // causal pairing: workgroup blk of a head runs query block nqb-1-blk (the heaviest) and then
  // block blk (the lightest), so every workgroup does about the same 2 (nqb + 1) tiles. The
  // heavy-first single-block grid left its second round of workgroups half the chip's slots:
  // 1.7 of 4 waves resident per SIMD on average (PMC SQ_WAVE_CYCLES vs kernel cycles,
  // profiles/r06_kernels/pmc_attn_summary.jsonl).
  const int npass = nqb - 1 - blk != blk ? 2 : 1;
  wg_stamp(a.stamps, 0);
  for (int pass = 0; pass < npass; ++pass) {
    if (pass) wg_stamp(a.stamps, 1);
    if (pass) __syncthreads();                    // every wave done with the LDS ring
    const int qb = pass == 0 ? nqb - 1 - blk : blk;
    const int q0 = qb * kQB;
    const int qw = q0 + wave * 32;                  // this wave's first query
    const int r = lane & 31, hi = lane >> 5;
    const uint16_t* base_bt = a.qkv + static_cast<int64_t>(b) * a.T * a.ld;
    const int hoff = h * D;

    // Q fragments (B operand of S^T = K Q^T): lane holds Q[qw + r][16 ks + 8 hi + j]
    bf16x8 qf[G::NKS];
    {
      int q = qw + r;
      q = q < a.T ? q : a.T - 1;
      const uint16_t* qp = base_bt + static_cast<int64_t>(q) * a.ld + hoff + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < G::NKS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
    }

    f32x16 o[G::NDT];
#pragma unroll
    for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[dt][e] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int qme = qw + r;                          // this lane's query
    const int q_hi = qw + 31;                        // wave's last query
    const int last_key = (q0 + kQB - 1) < (a.T - 1) ? (q0 + kQB - 1) : (a.T - 1);
    const int nt = last_key / KB + 1;

    auto tileK = [&](int c) { return smem + c * 2 * TILE; };
    auto tileV = [&](int c) { return smem + c * 2 * TILE + TILE; };

    // DMA: this lane's sources of image rows wave * WROWS + i * RPI + lane / (ROW / 16) of key
    // tile 0 (K and V sections, swizzled chunk); tile kt adds kt * KB rows, uniform
    const int r_in = lane / (ROW / 16), slot = lane % (ROW / 16);
    const uint16_t* dsrc[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wave * WROWS + i * RPI + r_in;
      const uint16_t* src = base_bt + static_cast<int64_t>(row) * a.ld + hoff;
      dsrc[2 * i] = src + D * a.H + (slot ^ kswz_d<D>(row)) * 8;
      dsrc[2 * i + 1] = src + 2 * D * a.H + (slot ^ vswz_d<D>(row)) * 8;
    }
    auto stage = [&](int k0, char* tk, char* tv) {
      if (k0 + KB <= a.T) {                          // wave-uniform: no row past T
        const int64_t off = static_cast<int64_t>(k0) * a.ld;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          attn_glds16(dsrc[2 * i] + off, tk + (wave * WROWS + i * RPI) * ROW);
          attn_glds16(dsrc[2 * i + 1] + off, tv + (wave * WROWS + i * RPI) * ROW);
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {                  // rows past T clamped (scores masked)
        const int row = wave * WROWS + i * RPI + r_in;
        int key = k0 + row;
        key = key < a.T ? key : a.T - 1;
        const uint16_t* src = base_bt + static_cast<int64_t>(key) * a.ld + hoff;
        attn_glds16(src + D * a.H + (slot ^ kswz_d<D>(row)) * 8,
                    tk + (wave * WROWS + i * RPI) * ROW);
        attn_glds16(src + 2 * D * a.H + (slot ^ vswz_d<D>(row)) * 8,
                    tv + (wave * WROWS + i * RPI) * ROW);
      }
    };
    stage(0, tileK(0), tileV(0));
    for (int kt = 0; kt < nt; ++kt) {
      const int cur = kt & 1;
      // one barrier per tile: it both publishes tile kt (every wave's DMA retired) and frees
      // buffer cur^1 (every wave finished tile kt-1), so the restage goes right after it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 1 < nt) stage((kt + 1) * KB, tileK(cur ^ 1), tileV(cur ^ 1));
      const int k0 = kt * KB;
      if (k0 <= q_hi) {                               // wave-uniform: tile has keys <= a query
        const char* tk = tileK(cur);
        const char* tv = tileV(cur);
        // ---- S^T for the 32-key halves
        f32x16 s[G::NKK];
#pragma unroll
        for (int kk = 0; kk < G::NKK; ++kk) {
#pragma unroll
          for (int e = 0; e < 16; ++e) s[kk][e] = 0.f;
          const int row = kk * 32 + r;
#pragma unroll
          for (int ks = 0; ks < G::NKS; ++ks) {
            const int c = 2 * ks + hi;
            const bf16x8 kf =
                *reinterpret_cast<const bf16x8*>(tk + row * ROW + ((c ^ kswz_d<D>(row)) << 4));
            s[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kk], 0, 0, 0);
          }
        }
        // ---- scale, causal mask, online softmax (lane = one query; keys in registers)
        const bool diag = k0 + KB - 1 > qw;           // some key of this tile beyond some query
        if (diag) {
          // key(kk, e) = k0 + 4 hi + kk*32 + (e & 3) + 8 (e >> 2): one per-lane threshold
          const int th = qme - k0 - 4 * hi;
#pragma unroll
          for (int kk = 0; kk < G::NKK; ++kk)
#pragma unroll
            for (int e = 0; e < 16; ++e)
              if (kk * 32 + (e & 3) + 8 * (e >> 2) > th) s[kk][e] = -INFINITY;
        }
        float mx = -INFINITY;                          // max of the RAW scores (scale > 0)
#pragma unroll
        for (int kk = 0; kk < G::NKK; ++kk)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[kk][e]);
        mx = xhalf_max(mx);
        // deferred max (CDNA guide §B "defer-max RESCALE_THRESHOLD"): the running max moves only
        // when some lane's tile max exceeds it by more than 2^8 in probability, so after the
        // first tiles p = exp2(s - m) stays <= 256 (bf16 / fp32 safe) and the O rescale and its
        // exp are skipped; the normaliser l and LSE use the same m, so the result is unchanged
        const float mc = mx * a.scale_log2;
        const float mn = __any(mc > m + 8.f) ? fmaxf(m, mc) : m;   // m = -inf first: moves
        const float alpha = __builtin_amdgcn_exp2f(m - mn);   // m = -inf on the first tile -> 0
        const bool rescale = m != mn;
        m = mn;
        float ls = 0.f;
#pragma unroll
        for (int kk = 0; kk < G::NKK; ++kk)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            s[kk][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kk][e], a.scale_log2, -mn));
            ls += s[kk][e];
          }
        l = l * alpha + ls;
        if (__any(rescale)) {                          // wave-uniform skip when no max moved
#pragma unroll
          for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[dt][e] *= alpha;
        }
        // ---- O^T += V^T P^T: k-step = 16 keys;
        //      P^T element j <-> key 16 s + 8 (j>>2) + 4 hi + (j&3)
        const int g = lane >> 4, i16 = lane & 15;
        const int tq = i16 >> 2, tp = i16 & 3;        // tr-read lane role: block row / col group
#pragma unroll
        for (int kk = 0; kk < G::NKK; ++kk)
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            bf16x8 pf;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              pf[j] = __builtin_bit_cast(short, static_cast<__bf16>(s[kk][8 * st + j]));
#pragma unroll
            for (int dt = 0; dt < G::NDT; ++dt) {
              bf16x8 vf;
#pragma unroll
              for (int half = 0; half < 2; ++half) {
                const int row = kk * 32 + 16 * st + 8 * half + 4 * (g >> 1) + tq;
                const int col = dt * 32 + 16 * (g & 1) + 4 * tp;
                const int off = row * ROW + (((col >> 3) ^ vswz_d<D>(row)) << 4) + (col & 7) * 2;
                // builtin read, kept on purpose: the compiler drains the next tile's K/V DMA
                // (vmcnt(0)) before the first of these, but that DMA has had the S MFMAs and the
                // softmax to land, and the builtin lets it interleave the reads with the MFMAs
                // under counted lgkmcnt waits (the asm form measured 3-4 % slower here,
                // profiles/r05_attention/). tools/isa_check.py allows this kernel.
                const i16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_ptr)(tv + off));
#pragma unroll
                for (int u = 0; u < 4; ++u) vf[4 * half + u] = t[u];
              }
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
            }
          }
      }
    }

    // ---- finalize: l over both lane halves, O / l, store O [B,T,H,D] and LSE
    const float lt = l + __shfl_xor(l, 32, 64);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    if (qme < a.T) {
      uint16_t* op = a.out + (static_cast<int64_t>(b) * a.T + qme) * a.ldo + hoff;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          u16x4 w;
#pragma unroll
          for (int u = 0; u < 4; ++u) w[u] = f32_to_bf16(o[dt][4 * gg + u] * inv);
          *reinterpret_cast<u16x4*>(op + dt * 32 + 8 * gg + 4 * hi) = w;
        }
      if (hi == 0 && a.lse)
        a.lse[(static_cast<int64_t>(b) * a.H + h) * a.T + qme] =
            (m + __builtin_amdgcn_logf(lt)) * 0.69314718055994531f;
    }
  }
  wg_stamp(a.stamps, 2);
}


// ===================================================================================== backward
// dS = P * (dP - delta), delta = rowsum(dO * O), P recomputed from Q, K and the forward's LSE.
// Two kernels, no atomics (CDNA guide §B "Attention backward": a dQ sum across key blocks by
// float atomics would cost dQ-bytes / 1.3 TB/s — ~100+ us at GPT-2's shape):
//   dkdv: a workgroup owns 128 keys (wave: 32, key on the MFMA lane) and sweeps 32-query
//         slices; S = Q K^T and dP = dO V^T come out with the key on the lane, so P and dS are
//         directly the B operands of dV^T += dO^T P and dK^T += Q^T dS (Q / dO slice images
//         read by rows AND transposed: one swizzle serves both, bswz).
//   dq:   a workgroup owns 128 queries (wave: 32, query on the lane) and sweeps 64-key tiles
//         like the forward: S^T = K Q^T, dP^T = V dO^T, then dQ^T += K^T dS^T (K image read
//         transposed).
// Both write straight into the fused dQKV gradient [B, T, 3, H, D].

// one swizzle for row reads (ds_read_b128, 32x32x16 A operand) and transposed reads
// (ds_read_b64_tr_b16) of a [rows][64 x bf16] image: t = pair index, bit 2 flipped on odd t
__device__ __forceinline__ int bswz(int r) {
  const int t = (r >> 1) & 7;
  return t ^ ((t & 1) << 2);
}

struct AttnBwdArgs {
  const uint16_t* qkv;     // [B, T, 3, H, D]
  const uint16_t* dout;    // [B, T, H, D] (row stride ldo)
  const float* lse;        // [B, H, T] natural log
  float* delta;            // [B, H, T]: -rowsum(dO * O) (negated: the dP accumulator's start)
  float* nls;              // [B, H, T]: -LSE * sqrt(D) (the S accumulator's start: S' = S - LSE
                           // sqrt(D), p = exp2(S' * scale_log2))
  const uint16_t* out;     // [B, T, H, D] forward output O (row stride ldo): fuse_delta only
  int fuse_delta;          // 1: the dQ kernel computes delta / nls for its queries and writes
                           // them for the dK/dV kernel launched after it (no delta kernel)
  uint16_t* dqkv;          // [B, T, 3, H, D] (row stride ld)
  int64_t ld, ldo;
  int B, T, H;
  float scale_log2;        // log2(e) / sqrt(D)
  float scale;             // 1 / sqrt(D)
  int xcd;                 // see head_block
  uint64_t* stamps;        // diagnostic, normally null: wg_stamp per workgroup
};

// transposed operand read of a [rows][64] bf16 image (bswz): A operand of a 32x32x16 MFMA whose
// k index is the image row: lane (col = colbase + (lane & 31), hi) gets rows
// rowbase + 8 (j>>2) + 4 hi + (j&3), j = 0..7 — matching an accumulator reused as B operand.
__device__ __forceinline__ bf16x8 tr_operand(const char* img, int rowbase, int colbase, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  bf16x8 f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int row = rowbase + 8 * half + 4 * (g >> 1) + tq;
    const int col = colbase + 16 * (g & 1) + 4 * tp;
    const int off = row * 128 + (((col >> 3) ^ bswz(row)) << 4) + (col & 7) * 2;
    const i16x4 t = ds_read_tr16(img + off);   // asm read: the caller waits (tr_wait)
#pragma unroll
    for (int u = 0; u < 4; ++u) f[4 * half + u] = t[u];
  }
  return f;
}

// tr_operand with the row offset as the reads' immediate: rows rowbase + 8 half + 4 (g>>1) + tq
// of column block dt. For rowbase % 16 == 0 the bswz chunk is (lane bits) | ((dt ^ half ^
// lane bit) << 2), so the address is one of two per-lane values (tr_lane_off(P), P = dt ^
// half) plus (rowbase + 8 half) * 128 — `same` = image + tr_lane_off(dt), `flip` = image +
// tr_lane_off(dt ^ 1). Equal to tr_operand for every lane / rowbase / dt (checked offline
// over all combinations when written); asm reads: the caller waits (tr_wait).
__device__ __forceinline__ uint32_t tr_lane_off(int lane, int P) {
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int L = 2 * (g >> 1) + (tq >> 1);
  const int chunk = (((2 * (g & 1) + (tp >> 1)) ^ L) & 3) | (((P ^ (L & 1)) & 1) << 2);
  return static_cast<uint32_t>((4 * (g >> 1) + tq) * 128 + chunk * 16 + ((4 * tp) & 7) * 2);
}
template <int ROWBASE, int IMG = 0>   // IMG: byte offset of the image from `same` / `flip`'s one
__device__ __forceinline__ bf16x8 tr_operand_at(const char* same, const char* flip) {
  static_assert(ROWBASE % 16 == 0, "row base");
  const i16x4 t0 = ds_read_tr16<IMG + ROWBASE * 128>(same);
  const i16x4 t1 = ds_read_tr16<IMG + (ROWBASE + 8) * 128>(flip);
  bf16x8 f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f[u] = t0[u];
    f[4 + u] = t1[u];
  }
  return f;
}

__device__ __forceinline__ bf16x8 row_operand(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((chunk ^ bswz(row)) << 4));
}

__device__ __forceinline__ bf16x8 acc_to_bf16(const f32x16& x, int st) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = __builtin_bit_cast(short, static_cast<__bf16>(x[8 * st + j]));
  return f;
}

// stage 64 rows x 128 B of a [T, ...] bf16 matrix (row stride ld) into an image with the bswz
// layout; wave w issues rows [16w, 16w + 16) (2 instructions). Rows >= T are clamped.
__device__ __forceinline__ void stage64(const uint16_t* base, int64_t ld, int row0, int T,
                                        char* img, int wave, int lane) {
  const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + r_in;
    int t = row0 + row;
    t = t < T ? t : T - 1;
    attn_glds16(base + static_cast<int64_t>(t) * ld + (slot ^ bswz(row)) * 8,
                img + (wave * 16 + i * 8) * 128);
  }
}

constexpr int kBwdKeys = 128;
constexpr int kSlice = 64;                   // queries staged per barrier pair (2 x 32)
constexpr int kSliceImg = kSlice * 128;      // 8 KiB

// INC: DMA sources of the Q / dO slice images from per-lane base pointers + one uniform offset
// per slice (the clamped per-row 64-bit address arithmetic only on a slice that crosses T); the
// forward's variant bit 4, measured 3 % there (A/B: dlbb_attn_set_bwd_incr)
template <bool INC>
__global__ void __launch_bounds__(kAttnThreads, 3) attn_bwd_dkdv_d64_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hi = lane >> 5;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  // causal pairing: key blocks blk (more query slices) and nkb-1-blk, equal work per workgroup
  const int nkb = (a.T + kBwdKeys - 1) / kBwdKeys;
  const int npass = nkb - 1 - blk != blk ? 2 : 1;
  wg_stamp(a.stamps, 0);
  for (int pass = 0; pass < npass; ++pass) {
    if (pass) wg_stamp(a.stamps, 1);
    if (pass) __syncthreads();                    // every wave done with the LDS ring
    const int kb0 = (pass == 0 ? blk : nkb - 1 - blk) * kBwdKeys;   // heaviest (block 0) first
    const int kw = kb0 + wave * 32;
    const int mykey = kw + r;
    const uint16_t* base_bt = a.qkv + static_cast<int64_t>(b) * a.T * a.ld;
    const uint16_t* dout_bt = a.dout + static_cast<int64_t>(b) * a.T * a.ldo;
    const int hoff = h * kAttnD;
    const int64_t bh = static_cast<int64_t>(b) * a.H + h;
    const float* lrow = a.nls + bh * a.T;            // -LSE * sqrt(D)
    const float* drow = a.delta + bh * a.T;          // -delta

    bf16x8 kf[4], vf[4];
    {
      const int kk = mykey < a.T ? mykey : a.T - 1;
      const uint16_t* kp = base_bt + static_cast<int64_t>(kk) * a.ld + kAttnD * a.H + hoff + 8 * hi;
      const uint16_t* vp = kp + kAttnD * a.H;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        kf[ks] = *reinterpret_cast<const bf16x8*>(kp + 16 * ks);
        vf[ks] = *reinterpret_cast<const bf16x8*>(vp + 16 * ks);
      }
    }
    f32x16 dv[2], dk[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) { dv[dt][e] = 0.f; dk[dt][e] = 0.f; }

    const int ns = (a.T - kb0 + kSlice - 1) / kSlice;
    auto imgQ = [&](int c) { return smem + c * 2 * kSliceImg; };
    auto imgG = [&](int c) { return smem + c * 2 * kSliceImg + kSliceImg; };
    // per-slice row constants (LSE, delta of the slice's 64 queries) ride the same LDS-DMA
    // double buffer as the Q / dO images instead of being loaded from global memory right
    // before use: waves 0 / 1 stage one 256-B row each (rows past T clamped, as for Q / dO)
    auto rowv = [&](int c) { return reinterpret_cast<float*>(smem + 4 * kSliceImg + c * 512); };
    auto stage_rows = [&](int q0, int c) {
      if (wave < 2) {
        int t = q0 + lane;
        t = t < a.T ? t : a.T - 1;
        __builtin_amdgcn_global_load_lds((wave == 0 ? lrow : drow) + t,
                                         (lds_vptr_t)(rowv(c) + 64 * wave), 4, 0, 0);
      }
    };
    // INC: this lane's Q / dO sources for image rows wave * 16 + i * 8 + lane / 8 of slice 0
    const uint16_t* qsrc[2];
    const uint16_t* gsrc[2];
    if constexpr (INC) {
      const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wave * 16 + i * 8 + r_in;
        qsrc[i] = base_bt + hoff + static_cast<int64_t>(kb0 + row) * a.ld + (slot ^ bswz(row)) * 8;
        gsrc[i] = dout_bt + hoff + static_cast<int64_t>(kb0 + row) * a.ldo + (slot ^ bswz(row)) * 8;
      }
    }
    auto stage_slice = [&](int q0, int c) {
      if constexpr (INC) {
        if (q0 + kSlice <= a.T) {                     // wave-uniform: no row past T
          const int d = q0 - kb0;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            attn_glds16(qsrc[i] + static_cast<int64_t>(d) * a.ld,
                        imgQ(c) + (wave * 16 + i * 8) * 128);
            attn_glds16(gsrc[i] + static_cast<int64_t>(d) * a.ldo,
                        imgG(c) + (wave * 16 + i * 8) * 128);
          }
          return;
        }
      }
      stage64(base_bt + hoff, a.ld, q0, a.T, imgQ(c), wave, lane);
      stage64(dout_bt + hoff, a.ldo, q0, a.T, imgG(c), wave, lane);
    };
    stage_slice(kb0, 0);
    stage_rows(kb0, 0);
    for (int i = 0; i < ns; ++i) {
      const int cur = i & 1;
      const int qs = kb0 + i * kSlice;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                   // publishes slice i, frees buffer cur^1
      if (i + 1 < ns) {
        stage_slice(qs + kSlice, cur ^ 1);
        stage_rows(qs + kSlice, cur ^ 1);
      }
      const char* iq = imgQ(cur);
      const char* ig = imgG(cur);
      const float* rv = rowv(cur);
      // transposed-read lane addresses of this slice's images (parity 0 / 1, tr_operand_at)
      const char* gq0 = iq + tr_lane_off(lane, 0);
      const char* gq1 = iq + tr_lane_off(lane, 1);
      const char* gg0 = ig + tr_lane_off(lane, 0);
      const char* gg1 = ig + tr_lane_off(lane, 1);
      auto sub_body = [&](auto subc) __attribute__((always_inline)) {
        constexpr int sub = decltype(subc)::value;
        const int qsub = qs + 32 * sub;
        if (qsub + 31 < kw) return;                   // wave-uniform: every query < every key
        constexpr int rb = 32 * sub;                  // image row base of this 32-query block
        // per-row constants for rows q = qsub + 8 g + 4 hi + u (register e = 4 g + u) as the
        // accumulators' starting values: S' = Q K^T - LSE sqrt(D), dP' = dO V^T - delta
        // (asm reads: rowv is filled by LDS-DMA, and a compiler-visible read of it drained every
        // DMA in flight — the next slice's Q / dO included; common.h ds_read_b128_asm)
        f32x16 s, dp;
        f32x4 lv[4], dv4[4];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          lv[g4] = ds_read_b128_asm(rv + rb + 8 * g4 + 4 * hi);
          dv4[g4] = ds_read_b128_asm(rv + 64 + rb + 8 * g4 + 4 * hi);
        }
        tr_wait(lv[0], lv[1], lv[2], lv[3], dv4[0], dv4[1], dv4[2], dv4[3]);
        s = __builtin_shufflevector(__builtin_shufflevector(lv[0], lv[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                    __builtin_shufflevector(lv[2], lv[3], 0, 1, 2, 3, 4, 5, 6, 7),
                                    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        dp = __builtin_shufflevector(
            __builtin_shufflevector(dv4[0], dv4[1], 0, 1, 2, 3, 4, 5, 6, 7),
            __builtin_shufflevector(dv4[2], dv4[3], 0, 1, 2, 3, 4, 5, 6, 7),
            0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_operand(iq, rb + r, 2 * ks + hi), kf[ks],
                                                      s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_operand(ig, rb + r, 2 * ks + hi), vf[ks],
                                                       dp, 0, 0, 0);
        }
        // mask the raw scores (exp2(-inf) = 0) only where a query of the block can precede a key
        // of the wave (the diagonal) or lies past T: a wave-uniform branch, so interior blocks run
        // no per-element index compares
        const bool diag = qsub < kw + 31;
        if (diag || qsub + 31 >= a.T) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int q = qsub + (e & 3) + 8 * (e >> 2) + 4 * hi;
            if ((diag && mykey > q) || q >= a.T) s[e] = -INFINITY;
          }
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = __builtin_amdgcn_exp2f(s[e] * a.scale_log2);
          s[e] = p;
          dp[e] = p * dp[e];
        }
        auto st_body = [&](auto stc) __attribute__((always_inline)) {
          constexpr int st = decltype(stc)::value;
          const bf16x8 pb = acc_to_bf16(s, st);
          const bf16x8 db = acc_to_bf16(dp, st);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            // dO^T, Q^T (asm reads; row offset in the immediate)
            bf16x8 gt = tr_operand_at<rb + 16 * st>(dt ? gg1 : gg0, dt ? gg0 : gg1);
            bf16x8 qt = tr_operand_at<rb + 16 * st>(dt ? gq1 : gq0, dt ? gq0 : gq1);
            tr_wait(gt, qt);
            dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gt, pb, dv[dt], 0, 0, 0);
            dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qt, db, dk[dt], 0, 0, 0);
          }
        };
        st_body(std::integral_constant<int, 0>{});
        st_body(std::integral_constant<int, 1>{});
      };
      sub_body(std::integral_constant<int, 0>{});
      sub_body(std::integral_constant<int, 1>{});
    }
    if (mykey < a.T) {
      uint16_t* dkp = a.dqkv + (static_cast<int64_t>(b) * a.T + mykey) * a.ld + kAttnD * a.H + hoff;
      uint16_t* dvp = dkp + kAttnD * a.H;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          u16x4 wk, wv;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            wk[u] = f32_to_bf16(dk[dt][4 * gg + u] * a.scale);
            wv[u] = f32_to_bf16(dv[dt][4 * gg + u]);
          }
          *reinterpret_cast<u16x4*>(dkp + dt * 32 + 8 * gg + 4 * hi) = wk;
          *reinterpret_cast<u16x4*>(dvp + dt * 32 + 8 * gg + 4 * hi) = wv;
        }
    }
  }
  wg_stamp(a.stamps, 2);
}

// K and V tiles of 64 keys in the bswz layout (both read by rows; K also transposed)
__device__ __forceinline__ void stage_kv64(const AttnBwdArgs& a, const uint16_t* base_bt, int k0,
                                           int hoff, char* tk, char* tv, int wave, int lane) {
  const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + r_in;
    int key = k0 + row;
    key = key < a.T ? key : a.T - 1;
    const uint16_t* src =
        base_bt + static_cast<int64_t>(key) * a.ld + hoff + (slot ^ bswz(row)) * 8;
    attn_glds16(src + kAttnD * a.H, tk + (wave * 16 + i * 8) * 128);
    attn_glds16(src + 2 * kAttnD * a.H, tv + (wave * 16 + i * 8) * 128);
  }
}

template <bool INC>   // as the dK/dV kernel: incremental K / V tile DMA sources
__global__ void __launch_bounds__(kAttnThreads, 2) attn_bwd_dq_d64_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nqb = (a.T + kQB - 1) / kQB;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  // causal pairing as the forward: query blocks nqb-1-blk then blk, equal work per workgroup
  const int npass = nqb - 1 - blk != blk ? 2 : 1;
  wg_stamp(a.stamps, 0);
  for (int pass = 0; pass < npass; ++pass) {
    if (pass) wg_stamp(a.stamps, 1);
    if (pass) __syncthreads();                    // every wave done with the LDS ring
    const int qb = pass == 0 ? nqb - 1 - blk : blk;
    const int q0 = qb * kQB;
    const int qw = q0 + wave * 32;
    const int r = lane & 31, hi = lane >> 5;
    const uint16_t* base_bt = a.qkv + static_cast<int64_t>(b) * a.T * a.ld;
    const int hoff = h * kAttnD;
    const int64_t bh = static_cast<int64_t>(b) * a.H + h;
    const int qme = qw + r;
    const int qc = qme < a.T ? qme : a.T - 1;

    bf16x8 qf[4], gf[4];
    {
      const uint16_t* qp = base_bt + static_cast<int64_t>(qc) * a.ld + hoff + 8 * hi;
      const uint16_t* gp = a.dout + (static_cast<int64_t>(b) * a.T + qc) * a.ldo + hoff + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
        gf[ks] = *reinterpret_cast<const bf16x8*>(gp + 16 * ks);
      }
    }
    float nl2, nd;                                   // -LSE * log2(e), -delta
    if (a.fuse_delta) {
      // the row constants of this lane's query, here instead of a separate pass over dO and O:
      // delta = dO . O over the 64 dims (8 per (ks, hi) fragment, halves joined by lane ^ 32)
      const uint16_t* op = a.out + (static_cast<int64_t>(b) * a.T + qc) * a.ldo + hoff + 8 * hi;
      float acc = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 of = *reinterpret_cast<const bf16x8*>(op + 16 * ks);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc += bf16_to_f32(static_cast<uint16_t>(gf[ks][j])) *
                 bf16_to_f32(static_cast<uint16_t>(of[j]));
      }
      const float other = __shfl_xor(acc, 32, 64);
      nd = -(hi == 0 ? acc + other : other + acc);   // (even chunks) + (odd chunks), as the kernel
      const float nls = -a.lse[bh * a.T + qc] / a.scale;   // -LSE * sqrt(D)
      nl2 = nls * a.scale_log2;
      if (hi == 0 && qme < a.T) {
        a.delta[bh * a.T + qme] = nd;
        a.nls[bh * a.T + qme] = nls;
      }
    } else {
      nl2 = a.nls[bh * a.T + qc] * a.scale_log2;
      nd = a.delta[bh * a.T + qc];
    }
    f32x16 dq[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) dq[dt][e] = 0.f;
    const int q_hi = qw + 31;
    const int last_key = (q0 + kQB - 1) < (a.T - 1) ? (q0 + kQB - 1) : (a.T - 1);
    const int nt = last_key / kKB + 1;
    auto tileK = [&](int c) { return smem + c * 2 * kTileKV; };
    auto tileV = [&](int c) { return smem + c * 2 * kTileKV + kTileKV; };
    const uint16_t* ksrc[2];
    if constexpr (INC) {
      const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wave * 16 + i * 8 + r_in;
        ksrc[i] = base_bt + static_cast<int64_t>(row) * a.ld + hoff + (slot ^ bswz(row)) * 8 +
                  kAttnD * a.H;
      }
    }
    auto stage = [&](int k0, char* tk, char* tv) {
      if constexpr (INC) {
        if (k0 + kKB <= a.T) {                        // wave-uniform: no row past T
          const int64_t off = static_cast<int64_t>(k0) * a.ld;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            attn_glds16(ksrc[i] + off, tk + (wave * 16 + i * 8) * 128);
            attn_glds16(ksrc[i] + off + kAttnD * a.H, tv + (wave * 16 + i * 8) * 128);
          }
          return;
        }
      }
      stage_kv64(a, base_bt, k0, hoff, tk, tv, wave, lane);
    };
    stage(0, tileK(0), tileV(0));
    for (int kt = 0; kt < nt; ++kt) {
      const int cur = kt & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                   // publishes tile kt, frees buffer cur^1
      if (kt + 1 < nt) stage((kt + 1) * kKB, tileK(cur ^ 1), tileV(cur ^ 1));
      const int k0 = kt * kKB;
      if (k0 <= q_hi) {
        const char* tk = tileK(cur);
        // K^T transposed-read lane addresses (parity 0 / 1) and the row offset as the immediate
        const char* tk0 = tk + tr_lane_off(lane, 0);
        const char* tk1 = tk + tr_lane_off(lane, 1);
        auto trk = [&](int sel, const char* same, const char* flip) __attribute__((always_inline)) {
          switch (sel) {                              // (compile-time after unrolling)
            case 0: return tr_operand_at<0>(same, flip);
            case 1: return tr_operand_at<16>(same, flip);
            case 2: return tr_operand_at<32>(same, flip);
            default: return tr_operand_at<48>(same, flip);
          }
        };
        const char* tv = tileV(cur);
        const bool diag = k0 + kKB - 1 > qw;           // wave-uniform: a key beyond a query
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          f32x16 s, dp;
#pragma unroll
          for (int e = 0; e < 16; ++e) { s[e] = 0.f; dp[e] = 0.f; }
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_operand(tk, kk * 32 + r, 2 * ks + hi),
                                                        qf[ks], s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_operand(tv, kk * 32 + r, 2 * ks + hi),
                                                         gf[ks], dp, 0, 0, 0);
          }
          // causal mask on the raw scores of diagonal tiles only (a branch, as in the forward:
          // exp2 of -inf is the zero probability); interior tiles run no per-element compares
          if (diag) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int key = k0 + kk * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
              if (key > qme) s[e] = -INFINITY;
            }
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[e], a.scale_log2, nl2));
            dp[e] = p * (dp[e] + nd);
          }
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            bf16x8 kt2[2];                            // K^T operands (asm reads)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
              kt2[dt] = trk(kk * 2 + st, dt ? tk1 : tk0, dt ? tk0 : tk1);
            const bf16x8 db = acc_to_bf16(dp, st);
            tr_wait(kt2[0], kt2[1]);
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
              dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt2[dt], db, dq[dt], 0, 0, 0);
          }
        }
      }
    }
    if (qme < a.T) {
      uint16_t* dqp = a.dqkv + (static_cast<int64_t>(b) * a.T + qme) * a.ld + hoff;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          u16x4 w;
#pragma unroll
          for (int u = 0; u < 4; ++u) w[u] = f32_to_bf16(dq[dt][4 * gg + u] * a.scale);
          *reinterpret_cast<u16x4*>(dqp + dt * 32 + 8 * gg + 4 * hi) = w;
        }
    }
  }
  wg_stamp(a.stamps, 2);
}

}  // namespace dlbb

using namespace dlbb;

static int g_attn_xcd = 1;   // A/B switch for the XCD-aware block order (dlbb_attn_set_xcd)
DLBB_API void dlbb_attn_set_xcd(int on) { g_attn_xcd = on ? 1 : 0; }
// diagnostic workgroup timeline buffers (wg_stamp; 4 uint64 per workgroup), null = off
static uint64_t* g_stamps_fwd = nullptr;
static uint64_t* g_stamps_dq = nullptr;
static uint64_t* g_stamps_dkdv = nullptr;
DLBB_API void dlbb_attn_set_stamps(void* fwd, void* dq, void* dkdv) {
  g_stamps_fwd = static_cast<uint64_t*>(fwd);
  g_stamps_dq = static_cast<uint64_t*>(dq);
  g_stamps_dkdv = static_cast<uint64_t*>(dkdv);
}

// qkv: [B, T, 3, H, D] bf16, D = 64 or 128 (token row stride ld elements, 16-B aligned rows);
// out: [B, T, H, D] bf16 (row stride ldo); lse: [B, H, T] fp32 (may be null). Causal only.
DLBB_API int dlbb_attn_fwd(const void* qkv, int64_t ld, void* out, int64_t ldo, float* lse,
                           int B, int T, int H, int D, float scale, hipStream_t stream) {
  if (B <= 0 || T <= 0 || H <= 0) return hipSuccess;
  if (D != 64 && D != 128) return hipErrorInvalidValue;
  if (ld % 8 || ldo % 4 || (reinterpret_cast<uintptr_t>(qkv) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 7))
    return hipErrorInvalidValue;
  if (ld < 3 * H * D || ldo < H * D) return hipErrorInvalidValue;
  AttnArgs a{static_cast<const uint16_t*>(qkv), static_cast<uint16_t*>(out), lse, ld, ldo,
             B, T, H, scale * 1.4426950408889634f, g_attn_xcd, g_stamps_fwd};
  const dim3 grid(((T + kQB - 1) / kQB + 1) / 2, H, B);   // query blocks paired (causal)
  if (D == 64)
    hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(kAttnThreads), 4 * FwdGeo<64>::TILE,
                       stream, a);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(kAttnThreads), 4 * FwdGeo<128>::TILE,
                       stream, a);
  return hipGetLastError();
}

// Backward of dlbb_attn_fwd (D = 64). dout / out: [B, T, H, 64] (row stride ldo); lse:
// forward's; delta: [2, B, H, T] fp32 workspace (-delta, -LSE sqrt(D), produced by the dQ
// kernel for the dK/dV kernel after it); dqkv: [B, T, 3, H, 64] (row stride ld, written fully).
// (Round-5 A/B forms removed in round 6: the dK/dV kernel concurrently on a side stream — its
// backward 5 % faster alone, the GPT-2 step 0.25 ms slower; a separate delta pass; per-row DMA
// addresses in dQ / incremental ones in dK/dV — each measured slower.)
DLBB_API int dlbb_attn_bwd(const void* qkv, int64_t ld, const void* out, const void* dout,
                           int64_t ldo, const float* lse, float* delta, void* dqkv, int B, int T,
                           int H, int D, float scale, hipStream_t stream) {
  if (B <= 0 || T <= 0 || H <= 0) return hipSuccess;
  if (D != kAttnD) return hipErrorInvalidValue;
  if (ld % 8 || ldo % 8 || ld < 3 * H * D || ldo < H * D) return hipErrorInvalidValue;
  auto mis16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) != 0; };
  if (mis16(qkv) || mis16(out) || mis16(dout) || mis16(dqkv)) return hipErrorInvalidValue;
  if (!lse || !delta || !out || !dout) return hipErrorInvalidValue;
  const int64_t rows = static_cast<int64_t>(B) * T * H;
  AttnBwdArgs a{static_cast<const uint16_t*>(qkv), static_cast<const uint16_t*>(dout), lse, delta,
                delta + rows, static_cast<const uint16_t*>(out), 1,
                static_cast<uint16_t*>(dqkv), ld, ldo, B, T, H,
                scale * 1.4426950408889634f, scale, g_attn_xcd, g_stamps_dq};
  // both kernels pair a heavy and a light causal block per workgroup (see the forward)
  const dim3 gq(((T + kQB - 1) / kQB + 1) / 2, H, B),
      gk(((T + kBwdKeys - 1) / kBwdKeys + 1) / 2, H, B);
  hipLaunchKernelGGL(attn_bwd_dq_d64_kernel<true>, gq, dim3(kAttnThreads), 4 * kTileKV, stream,
                     a);
  a.stamps = g_stamps_dkdv;
  hipLaunchKernelGGL(attn_bwd_dkdv_d64_kernel<false>, gk, dim3(kAttnThreads),
                     4 * kSliceImg + 1024, stream, a);
  return hipGetLastError();
}
