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

// Stage keys [k0, k0 + 64) of head h: K (section 1 of the row) and V (section 2) tiles.
// 64 rows x 128 B per image = 8 KiB = 8 wave-instructions; wave w issues rows [16w, 16w + 16)
// of each (2 + 2 instructions). Rows past T are clamped (their scores are masked).
__device__ __forceinline__ void attn_stage(const AttnArgs& a, const uint16_t* base_bt, int k0,
                                           int hoff, char* tk, char* tv, int wave, int lane) {
  const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + r_in;
    int key = k0 + row;
    key = key < a.T ? key : a.T - 1;
    const uint16_t* src = base_bt + static_cast<int64_t>(key) * a.ld + hoff;
    attn_glds16(src + kAttnD * a.H + (slot ^ kswz(row)) * 8, tk + (wave * 16 + i * 8) * 128);
    attn_glds16(src + 2 * kAttnD * a.H + (slot ^ vswz(row)) * 8, tv + (wave * 16 + i * 8) * 128);
  }
}

// lane ^ 32 half exchange of a per-lane value by v_permlane32_swap (a VALU op) instead of a
// ds_bpermute LDS round trip; max over both halves ends in every lane
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// v_max3_f32 as one instruction (fmaxf on MFMA outputs gets canonicalising v_max first)
__device__ __forceinline__ float max3_asm(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Forward variants (bit mask, A/B via dlbb_attn_set_fwd_variant):
//   1: the tile's 8 K fragments read up front (asm ds_read_b128, one counted lgkmcnt wait per
//      32-key half) — the compiler's schedule re-used one register quad and waited for each read
//      in front of its MFMA (8 LDS round trips per tile);
//   2: the row-max exchange with the other lane half by v_permlane32_swap (no LDS round trip);
//   4: K/V DMA sources from per-lane base pointers + one uniform offset per tile (the clamped
//      per-row 64-bit address arithmetic only on a tile that crosses T);
//   8: row max and row sum as pairwise trees (depth 5) instead of 32-long dependent chains
//      (instantiated as 14 = 2 | 4 | 8 only).
template <int V>
__global__ void __launch_bounds__(kAttnThreads, 2) attn_fwd_d64_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nqb = (a.T + kQB - 1) / kQB;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  const int qb = nqb - 1 - blk;                   // heaviest first
  const int q0 = qb * kQB;
  const int qw = q0 + wave * 32;                  // this wave's first query
  const int r = lane & 31, hi = lane >> 5;
  const uint16_t* base_bt = a.qkv + static_cast<int64_t>(b) * a.T * a.ld;
  const int hoff = h * kAttnD;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[qw + r][16 ks + 8 hi + j]
  bf16x8 qf[4];
  {
    int q = qw + r;
    q = q < a.T ? q : a.T - 1;
    const uint16_t* qp = base_bt + static_cast<int64_t>(q) * a.ld + hoff + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }

  f32x16 o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[dt][e] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int qme = qw + r;                          // this lane's query
  const int q_hi = qw + 31;                        // wave's last query
  const int last_key = (q0 + kQB - 1) < (a.T - 1) ? (q0 + kQB - 1) : (a.T - 1);
  const int nt = last_key / kKB + 1;

  auto tileK = [&](int c) { return smem + c * 2 * kTileKV; };
  auto tileV = [&](int c) { return smem + c * 2 * kTileKV + kTileKV; };

  // V & 4: this lane's 4 DMA sources of key-tile 0 (rows wave * 16 + i * 8 + lane / 8, K and V
  // sections); tile kt adds kt * 64 rows, uniform
  const uint16_t* dsrc[4];
  if constexpr ((V & 4) != 0) {
    const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wave * 16 + i * 8 + r_in;
      const uint16_t* src = base_bt + static_cast<int64_t>(row) * a.ld + hoff;
      dsrc[2 * i] = src + kAttnD * a.H + (slot ^ kswz(row)) * 8;
      dsrc[2 * i + 1] = src + 2 * kAttnD * a.H + (slot ^ vswz(row)) * 8;
    }
  }
  auto stage = [&](int k0, char* tk, char* tv) {
    if constexpr ((V & 4) != 0) {
      if (k0 + kKB <= a.T) {                        // wave-uniform: no row past T
        const int64_t off = static_cast<int64_t>(k0) * a.ld;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          attn_glds16(dsrc[2 * i] + off, tk + (wave * 16 + i * 8) * 128);
          attn_glds16(dsrc[2 * i + 1] + off, tv + (wave * 16 + i * 8) * 128);
        }
        return;
      }
    }
    attn_stage(a, base_bt, k0, hoff, tk, tv, wave, lane);
  };
  stage(0, tileK(0), tileV(0));
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    // one barrier per tile: it both publishes tile kt (every wave's DMA retired) and frees
    // buffer cur^1 (every wave finished tile kt-1), so the restage goes right after it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nt) stage((kt + 1) * kKB, tileK(cur ^ 1), tileV(cur ^ 1));
    const int k0 = kt * kKB;
    if (k0 <= q_hi) {                               // wave-uniform: tile has keys <= a query
      const char* tk = tileK(cur);
      const char* tv = tileV(cur);
      // ---- S^T for the two 32-key halves
      f32x16 s[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 16; ++e) s[kk][e] = 0.f;
      if constexpr ((V & 1) != 0) {
        // rows r and 32 + r share kswz (it depends on row bits 1..3): the second half is the
        // first's addresses + 4 KiB (read immediate)
        f32x4 kr[2][4];
        const char* krow = tk + r * 128;
        const int sw = kswz(r);
        const char* kp[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kp[ks] = krow + (((2 * ks + hi) ^ sw) << 4);
        // issue order = wait order: half 0's four reads, then half 1's (asm volatile keeps it)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kr[0][ks] = ds_read_b128_asm<0>(kp[ks]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kr[1][ks] = ds_read_b128_asm<4096>(kp[ks]);
        lgk_wait<4>(kr[0][0], kr[0][1], kr[0][2], kr[0][3]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kr[0][ks]),
                                                         qf[ks], s[0], 0, 0, 0);
        lgk_wait<0>(kr[1][0], kr[1][1], kr[1][2], kr[1][3]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kr[1][ks]),
                                                         qf[ks], s[1], 0, 0, 0);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int row = kk * 32 + r;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const int c = 2 * ks + hi;
            const bf16x8 kf =
                *reinterpret_cast<const bf16x8*>(tk + row * 128 + ((c ^ kswz(row)) << 4));
            s[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kk], 0, 0, 0);
          }
        }
      }
      // ---- scale, causal mask, online softmax (lane = one query; keys in registers)
      const bool diag = k0 + kKB - 1 > qw;          // some key of this tile beyond some query
      float mx = -INFINITY;                          // max of the RAW scores (scale > 0)
      if (diag) {
        // key(kk, e) = k0 + 4 hi + const(kk, e): one per-lane threshold, compile-time offsets
        const int th = qme - k0 - 4 * hi;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (kk * 32 + (e & 3) + 8 * (e >> 2) > th) s[kk][e] = -INFINITY;
      }
      if constexpr ((V & 8) != 0) {
        // 3-ary tree of v_max3 (depth 4: 32 -> 11 -> 4 -> 2 -> 1) instead of a 16-long
        // dependent v_max3 chain
        float v[32], t[11];
#pragma unroll
        for (int e = 0; e < 16; ++e) { v[e] = s[0][e]; v[16 + e] = s[1][e]; }
#pragma unroll
        for (int j = 0; j < 10; ++j) t[j] = max3_asm(v[3 * j], v[3 * j + 1], v[3 * j + 2]);
        t[10] = max3_asm(v[30], v[31], v[31]);
        const float u0 = max3_asm(t[0], t[1], t[2]), u1 = max3_asm(t[3], t[4], t[5]);
        const float u2 = max3_asm(t[6], t[7], t[8]), u3 = max3_asm(t[9], t[10], t[10]);
        mx = max3_asm(max3_asm(u0, u1, u2), u3, u3);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[kk][e]);
      }
      if constexpr ((V & 2) != 0)
        mx = xhalf_max(mx);
      else
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx * a.scale_log2);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);   // m = -inf on the first tile -> 0
      const bool rescale = m != mn;
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          s[kk][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kk][e], a.scale_log2, -mn));
      if constexpr ((V & 8) != 0) {
        float t[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = s[0][e] + s[1][e];
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
          for (int e = 0; e < w; ++e) t[e] += t[e + w];
        ls = t[0];
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int e = 0; e < 16; ++e) ls += s[kk][e];
      }
      l = l * alpha + ls;
      if (__any(rescale)) {                          // wave-uniform skip when no max moved
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) o[dt][e] *= alpha;
      }
      // ---- O^T += V^T P^T: k-step = 16 keys; P^T element j <-> key 16 s + 8 (j>>2) + 4 hi + (j&3)
      const int g = lane >> 4, i16 = lane & 15;
      const int tq = i16 >> 2, tp = i16 & 3;        // tr-read lane role: block row / col group
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 pf;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pf[j] = __builtin_bit_cast(short, static_cast<__bf16>(s[kk][8 * st + j]));
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            bf16x8 vf;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              const int row = kk * 32 + 16 * st + 8 * half + 4 * (g >> 1) + tq;
              const int col = dt * 32 + 16 * (g & 1) + 4 * tp;
              const int off = row * 128 + (((col >> 3) ^ vswz(row)) << 4) + (col & 7) * 2;
              // builtin read, kept on purpose: the compiler drains the next tile's K/V DMA
              // (vmcnt(0)) before the first of these, but that DMA has had the S MFMAs and the
              // softmax to land, and the builtin lets it interleave the reads with the MFMAs
              // under counted lgkmcnt waits. The asm form (common.h ds_read_tr16, grouped
              // waits; also software-pipelined) measured 3-4 % SLOWER here (61-62 vs 58-60 us
              // at the GPT-2 shape, profiles/r05_attention/), unlike dQ / dK/dV where the
              // drain sat right behind the DMA issue. tools/isa_check.py allows this kernel.
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
    for (int dt = 0; dt < 2; ++dt)
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
};

// ndelta[b, h, t] = -sum_d dO[b, t, h, d] * O[b, t, h, d] and nls[b, h, t] = -LSE * sqrt(D): the
// row constants of the backward, pre-negated / pre-scaled once per row here so the dK/dV loop
// starts its S and dP accumulators at them (guide: 'row constants as the initial accumulator'):
// p = exp2(S' * scale_log2) and dS = P * dP' with no subtraction, and no constant held in
// registers across the MFMA chains; one thread per (b, t, h) row of 64
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(const uint16_t* __restrict__ dout,
                                                             const uint16_t* __restrict__ out,
                                                             int64_t ldo, const float* __restrict__ lse,
                                                             float* __restrict__ delta,
                                                             float* __restrict__ nls,
                                                             float scale, int B, int T, int H) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nrows = static_cast<int64_t>(B) * T * H;
  if (row >= nrows) return;
  const int h = static_cast<int>(row % H);
  const int64_t bt = row / H;
  const uint16_t* g = dout + bt * ldo + h * kAttnD;
  const uint16_t* o = out + bt * ldo + h * kAttnD;
  // even / odd 8-dim chunks summed separately, then added: the order of the dQ kernel's fused
  // form (lane halves hi = 0 / 1, joined by lane ^ 32), so both give bitwise the same constants
  float acc2[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kAttnD / 8; ++c) {
    float x[8], y[8];
    load8<DT_BF16>(g, c, x);
    load8<DT_BF16>(o, c, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc2[c & 1] += x[j] * y[j];
  }
  const int64_t b = bt / T, t = bt % T;
  const int64_t i = (b * H + h) * T + t;
  delta[i] = -(acc2[0] + acc2[1]);
  nls[i] = -lse[i] / scale;
}

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
__global__ void __launch_bounds__(kAttnThreads, 2) attn_bwd_dkdv_d64_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hi = lane >> 5;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  const int kb0 = blk * kBwdKeys;                   // block 0 = most query slices: first
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
          attn_glds16(qsrc[i] + static_cast<int64_t>(d) * a.ld, imgQ(c) + (wave * 16 + i * 8) * 128);
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
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qsub = qs + 32 * sub;
      if (qsub + 31 < kw) continue;                 // wave-uniform: every query < every key
      const int rb = 32 * sub;                      // image row base of this 32-query block
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
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s[4 * g4 + u] = lv[g4][u];
          dp[4 * g4 + u] = dv4[g4][u];
        }
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
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pb = acc_to_bf16(s, st);
        const bf16x8 db = acc_to_bf16(dp, st);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          bf16x8 gt = tr_operand(ig, rb + 16 * st, 32 * dt, lane);   // dO^T, Q^T (asm reads)
          bf16x8 qt = tr_operand(iq, rb + 16 * st, 32 * dt, lane);
          tr_wait(gt, qt);
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gt, pb, dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qt, db, dk[dt], 0, 0, 0);
        }
      }
    }
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

// K and V tiles of 64 keys in the bswz layout (both read by rows; K also transposed)
__device__ __forceinline__ void stage_kv64(const AttnBwdArgs& a, const uint16_t* base_bt, int k0,
                                           int hoff, char* tk, char* tv, int wave, int lane) {
  const int r_in = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + r_in;
    int key = k0 + row;
    key = key < a.T ? key : a.T - 1;
    const uint16_t* src = base_bt + static_cast<int64_t>(key) * a.ld + hoff + (slot ^ bswz(row)) * 8;
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
  const int qb = nqb - 1 - blk;
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
          for (int dt = 0; dt < 2; ++dt) kt2[dt] = tr_operand(tk, kk * 32 + 16 * st, 32 * dt, lane);
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

// ============================================================================ pipelined forward
// Round-6 forward body (the round-5 kernel ran QK^T -> softmax -> PV of a tile back to back in
// one wave: MFMA busy 19 %, the VALU softmax never beside the matrix work). Each wave now runs
// a software pipeline over its key tiles: iteration `it` issues the QK^T MFMAs of tile it + 1,
// the softmax (VALU) of tile it and the PV MFMAs of tile it - 1 as ONE straight-line block, so
// the softmax's exps / max / sums fill the issue gaps of 16 independent MFMAs instead of
// waiting for their own (CDNA guide §B "Fused attention prefill": P of tile j beside PV of
// tile j - 1).
//   * K and V are staged in rings of 4 x 8 KiB (64 KiB per workgroup, 2 workgroups per CU):
//     at the top of iteration it (after the one barrier) K_{it+3} and V_{it+2} are issued, so a
//     K tile has two iterations to land and a V tile three; the counted wait vmcnt(6) retires
//     exactly K_{it+1} (and everything older: V_{it-1}). Past the last tile the loads repeat
//     the last tile (uniform instruction counts keep the count constant).
//   * lazy rescaling: a row's reference max m moves only when a tile's max exceeds it by more
//     than 2^8 (p = exp2(s c - m) <= 256 otherwise, exact in bf16 / fp32 sums); the O
//     rescale (32 multiplies, wave-uniformly skipped when no lane moved) is applied one
//     iteration late, right before the PV of the tile whose softmax moved m.
//   * only a wave's LAST key tile meets the diagonal (queries qw .. qw + 31, qw % 32 == 0, tiles
//     of 64): it is the one masked softmax.
//   * layouts as the round-5 kernel: swapped scores S^T = K Q^T (lane = query), K image kswz
//     (ds_read_b128 rows), V image vswz (ds_read_b64_tr_b16), O^T = V^T P^T in registers.
constexpr int kRing = 4;
constexpr float kLazyLog2 = 8.f;

struct FwdRegs {
  bf16x8 qf[4];
  f32x16 o[2];
  float m, l, alpha;      // reference max (log2 units), row sum, pending O rescale
};

// K fragments of the key tile in image `tk` (8 row reads, issued in wait order: half 0 first)
__device__ __forceinline__ void fwd_kreads(const char* tk, f32x4 (&kr)[2][4], int lane) {
  const int r = lane & 31, hi = lane >> 5;
  const char* krow = tk + r * 128;
  const int sw = kswz(r);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) kr[0][ks] = ds_read_b128_asm<0>(krow + (((2 * ks + hi) ^ sw) << 4));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) kr[1][ks] = ds_read_b128_asm<4096>(krow + (((2 * ks + hi) ^ sw) << 4));
}

// S^T half KK (32 keys) = K Q^T; the caller has waited for kr[KK]
template <int KK>
__device__ __forceinline__ void fwd_scores_half(const f32x4 (&kr)[2][4], const bf16x8 (&qf)[4],
                                                f32x16 (&s)[2]) {
#pragma unroll
  for (int e = 0; e < 16; ++e) s[KK][e] = 0.f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    s[KK] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kr[KK][ks]), qf[ks],
                                                    s[KK], 0, 0, 0);
}

// V^T fragments of keys [32 KK, 32 KK + 32) of the tile in image `tv` (8 transposed reads;
// the caller waits). row = KK*32 + 16 st + 8 half + 4 (g >> 1) + tq: vswz(row) depends on bit 1
// of tq only, so the address is a per-lane base per dt plus an immediate.
template <int KK>
__device__ __forceinline__ void fwd_vreads(const char* tv, i16x4 (&vt)[2][2][2], int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  const int row0 = 4 * (g >> 1) + tq;
  const int sw = vswz(row0);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const int col = dt * 32 + 16 * (g & 1) + 4 * tp;
    const char* b = tv + row0 * 128 + (((col >> 3) ^ sw) << 4) + (col & 7) * 2;
    vt[0][dt][0] = ds_read_tr16<(KK * 32 + 0) * 128>(b);
    vt[0][dt][1] = ds_read_tr16<(KK * 32 + 8) * 128>(b);
    vt[1][dt][0] = ds_read_tr16<(KK * 32 + 16) * 128>(b);
    vt[1][dt][1] = ds_read_tr16<(KK * 32 + 24) * 128>(b);
  }
}

template <int N>
__device__ __forceinline__ void vt_wait(i16x4 (&vt)[2][2][2]) {
  lgk_wait<N>(vt[0][0][0], vt[0][0][1], vt[0][1][0], vt[0][1][1], vt[1][0][0], vt[1][0][1],
              vt[1][1][0], vt[1][1][1]);
}

// O^T += V^T P^T for keys half KK of a tile (4 MFMA)
template <int KK>
__device__ __forceinline__ void fwd_pv_half(f32x16 (&o)[2], const i16x4 (&vt)[2][2][2],
                                            const bf16x8 (&p)[2][2]) {
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      bf16x8 vf;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vf[u] = vt[st][dt][0][u];
        vf[4 + u] = vt[st][dt][1][u];
      }
      o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, p[KK][st], o[dt], 0, 0, 0);
    }
}

__device__ __forceinline__ void fwd_rescale(FwdRegs& R) {
  if (__builtin_amdgcn_ballot_w64(R.alpha != 1.f) != 0) {   // wave-uniform skip
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) R.o[dt][e] *= R.alpha;
  }
}

// softmax part 1 of the scores `s` of key tile k0 (in place: s becomes p in fp32), updating
// m / l; returns the tile's O rescale factor (applied before the PV of this tile)
template <bool DIAG>
__device__ __forceinline__ float fwd_softmax(FwdRegs& R, f32x16 (&s)[2], int k0, int qme,
                                             float c, int lane) {
  const int hi = lane >> 5;
  if constexpr (DIAG) {
    // key(kk, e) = k0 + 4 hi + kk*32 + (e & 3) + 8 (e >> 2): one per-lane threshold
    const int th = qme - k0 - 4 * hi;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (kk * 32 + (e & 3) + 8 * (e >> 2) > th) s[kk][e] = -INFINITY;
  }
  float mx = max3_asm(s[0][0], s[0][1], s[0][2]);
#pragma unroll
  for (int e = 3; e < 15; e += 2) mx = max3_asm(mx, s[0][e], s[0][e + 1]);
  mx = max3_asm(mx, s[0][15], s[1][0]);
#pragma unroll
  for (int e = 1; e < 15; e += 2) mx = max3_asm(mx, s[1][e], s[1][e + 1]);
  mx = fmaxf(mx, s[1][15]);
  mx = xhalf_max(mx) * c;
  const float mn = mx > R.m + kLazyLog2 ? mx : R.m;     // m = -inf on the first tile
  const float alpha = __builtin_amdgcn_exp2f(R.m - mn);
  R.m = mn;
  float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float v = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kk][e], c, -mn));
      s[kk][e] = v;
      if (kk == 0) ls0 += v; else ls1 += v;
    }
  R.l = R.l * alpha + (ls0 + ls1);
  return alpha;
}

// softmax part 2: the probabilities to bf16 MFMA operands
__device__ __forceinline__ void fwd_pack(const f32x16 (&s)[2], bf16x8 (&p)[2][2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        p[kk][st][j] = __builtin_bit_cast(short, static_cast<__bf16>(s[kk][8 * st + j]));
}

__global__ void __launch_bounds__(kAttnThreads, 2) attn_fwd_pipe_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nqb = (a.T + kQB - 1) / kQB;
  int blk, h, b;
  head_block(a.xcd, blk, h, b);
  const int qb = nqb - 1 - blk;                   // heaviest first
  const int q0 = qb * kQB;
  const int qw = q0 + wave * 32;
  const int r = lane & 31, hi = lane >> 5;
  const uint16_t* base_bt = a.qkv + static_cast<int64_t>(b) * a.T * a.ld;
  const int hoff = h * kAttnD;
  const int qme = qw + r;
  const float c = a.scale_log2;
  // key tiles of the workgroup (barriers) and of this wave (work); nt_w = 0: no query < T
  const int last_key = (q0 + kQB - 1) < (a.T - 1) ? (q0 + kQB - 1) : (a.T - 1);
  const int nt = last_key / kKB + 1;
  const int q_hi = (qw + 31) < (a.T - 1) ? (qw + 31) : (a.T - 1);
  const int nt_w = qw < a.T ? q_hi / kKB + 1 : 0;

  FwdRegs R;
  {
    const int q = qme < a.T ? qme : a.T - 1;
    const uint16_t* qp = base_bt + static_cast<int64_t>(q) * a.ld + hoff + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) R.qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) R.o[dt][e] = 0.f;
  R.m = -INFINITY;
  R.l = 0.f;
  R.alpha = 1.f;

  auto ringK = [&](int t) { return smem + (t & (kRing - 1)) * kTileKV; };
  auto ringV = [&](int t) { return smem + (kRing + (t & (kRing - 1))) * kTileKV; };
  // K / V staging by buffer_load ... lds: the (b, h) section bases in buffer resources
  // (SGPRs), this lane's row-in-tile + swizzled chunk as a 32-bit offset (rows wave * 16 +
  // i * 8 + lane / 8), a tile's rows as a uniform offset; a tile crossing T clamps its rows
  const int r_in = lane >> 3, slot = lane & 7;
  const uint32_t ld2 = static_cast<uint32_t>(a.ld) * 2;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(base_bt + hoff + kAttnD * a.H), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(base_bt + hoff + 2 * kAttnD * a.H), 0, 0x7fffffff, 0x00020000);
  uint32_t koff[2], voff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + r_in;
    koff[i] = static_cast<uint32_t>(row) * ld2 + ((slot ^ kswz(row)) << 4);
    voff[i] = static_cast<uint32_t>(row) * ld2 + ((slot ^ vswz(row)) << 4);
  }
  // stage K (sec 1) or V (sec 2) of key index ts into its ring slot (tile min(ts, nt - 1))
  auto stage = [&](int ts, int sec) __attribute__((always_inline)) {
    char* dst = sec == 1 ? ringK(ts) : ringV(ts);
    const int t = ts < nt - 1 ? ts : nt - 1;
    const int k0 = t * kKB;
    const __amdgpu_buffer_rsrc_t rs = sec == 1 ? rk : rv;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t off;
      if (k0 + kKB <= a.T) {                       // wave-uniform: no row past T
        off = (sec == 1 ? koff[i] : voff[i]) + static_cast<uint32_t>(k0) * ld2;
      } else {
        const int row = wave * 16 + i * 8 + r_in;
        const int key = k0 + row < a.T ? k0 + row : a.T - 1;
        off = static_cast<uint32_t>(key) * ld2 +
              ((slot ^ (sec == 1 ? kswz(row) : vswz(row))) << 4);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr_t)(dst + (wave * 16 + i * 8) * 128), 16,
                                               off, 0, 0, 0);
    }
  };

  f32x16 s[2];
  bf16x8 p[2][2];
  // prologue: K_0 | K_1, V_0 -> K_0 landed; iteration -1: K_2, V_1 issued, S_0
  stage(0, 1);
  stage(1, 1);
  stage(0, 2);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  stage(2, 1);
  stage(1, 2);
  auto scores = [&](int t) __attribute__((always_inline)) {
    f32x4 kr[2][4];
    fwd_kreads(ringK(t), kr, lane);
    lgk_wait<4>(kr[0][0], kr[0][1], kr[0][2], kr[0][3]);
    fwd_scores_half<0>(kr, R.qf, s);
    lgk_wait<0>(kr[1][0], kr[1][1], kr[1][2], kr[1][3]);
    fwd_scores_half<1>(kr, R.qf, s);
  };
  auto pv = [&](int t) __attribute__((always_inline)) {
    i16x4 vt[2][2][2];
    fwd_vreads<0>(ringV(t), vt, lane);
    vt_wait<0>(vt);
    fwd_rescale(R);
    fwd_pv_half<0>(R.o, vt, p);
    fwd_vreads<1>(ringV(t), vt, lane);
    vt_wait<0>(vt);
    fwd_pv_half<1>(R.o, vt, p);
  };
  if (nt_w > 0) scores(0);
  // iteration it: [PV_{it-1} | softmax_it] then S_{it+1}. The PV MFMAs (independent of the
  // softmax) are issued between its VALU; p holds tile it - 1's probabilities until the PV
  // has read them, then tile it's.
  for (int it = 0; it <= nt; ++it) {
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // K_{it+1} (and V_{it-1}) landed
    __builtin_amdgcn_s_barrier();                      // ... for every wave; slots it-1 free
    stage(it + 3, 1);
    stage(it + 2, 2);
    const int k0 = it * kKB;
    if (it >= 1 && it + 1 < nt_w) {                    // steady state: one straight block
      i16x4 vt[2][2][2];
      fwd_vreads<0>(ringV(it - 1), vt, lane);
      const float al = fwd_softmax<false>(R, s, k0, qme, c, lane);
      vt_wait<0>(vt);
      fwd_rescale(R);
      fwd_pv_half<0>(R.o, vt, p);
      fwd_vreads<1>(ringV(it - 1), vt, lane);
      vt_wait<0>(vt);
      fwd_pv_half<1>(R.o, vt, p);
      fwd_pack(s, p);
      R.alpha = al;
      scores(it + 1);
    } else {                                           // first / diagonal / drain iterations
      if (it >= 1 && it <= nt_w) pv(it - 1);
      if (it < nt_w) {
        const float al = it == nt_w - 1 ? fwd_softmax<true>(R, s, k0, qme, c, lane)
                                        : fwd_softmax<false>(R, s, k0, qme, c, lane);
        fwd_pack(s, p);
        R.alpha = al;
      }
      if (it + 1 < nt_w) scores(it + 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA in flight at exit

  // ---- finalize: l over both lane halves, O / l, store O [B,T,H,D] and LSE
  const float lt = R.l + __shfl_xor(R.l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qme < a.T) {
    uint16_t* op = a.out + (static_cast<int64_t>(b) * a.T + qme) * a.ldo + hoff;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        u16x4 w;
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = f32_to_bf16(R.o[dt][4 * gg + u] * inv);
        *reinterpret_cast<u16x4*>(op + dt * 32 + 8 * gg + 4 * hi) = w;
      }
    if (hi == 0 && a.lse)
      a.lse[(static_cast<int64_t>(b) * a.H + h) * a.T + qme] =
          (R.m + __builtin_amdgcn_logf(lt)) * 0.69314718055994531f;
  }
}
}  // namespace dlbb

using namespace dlbb;

static int g_attn_xcd = 1;   // A/B switch for the XCD-aware block order (dlbb_attn_set_xcd)
// dK/dV and dQ kernels concurrently (fork/join side stream): opt-in, DLBB_ATTN_CONCURRENT=1.
// The backward alone is 5 % faster (195 vs 205 us at GPT-2 shape) but the GPT-2 step measured
// 0.25 ms SLOWER in an in-call A/B (20.2 vs 19.95 ms), so the default is sequential.
static int g_attn_concurrent = [] {
  const char* v = getenv("DLBB_ATTN_CONCURRENT");
  return (v && v[0] == '1') ? 1 : 0;
}();

// delta / nls computed inside the dQ kernel (1, default) or by the separate row kernel first (0);
// the concurrent form always uses the separate kernel (A/B: dlbb_attn_set_fuse_delta)
static int g_attn_fuse_delta = 1;
// forward kernel variant (attn_fwd_d64_kernel<V> bit mask; A/B: dlbb_attn_set_fwd_variant).
// 6 = permlane32 exchange + incremental DMA addresses: 49.8 vs 52.2 us at the GPT-2 shape,
// 85.6 vs 90.3 (T 2048), 197.2 vs 201.9 (T 4096); the batched K reads (bit 1) measured no gain
// (profiles/r05_attention/fwd_variants.jsonl)
static int g_attn_fwd_variant = 6;
// backward kernels with incremental DMA sources, bit mask: 1 dQ, 2 dK/dV (0: per-row clamped
// addresses). dK/dV<true> holds 174 VGPRs (occupancy 2 waves / SIMD, vs 3 at 166)
static int g_attn_bwd_incr = 1;

DLBB_API void dlbb_attn_set_xcd(int on) { g_attn_xcd = on ? 1 : 0; }
DLBB_API void dlbb_attn_set_fuse_delta(int on) { g_attn_fuse_delta = on ? 1 : 0; }
DLBB_API void dlbb_attn_set_concurrent(int on) { g_attn_concurrent = on ? 1 : 0; }
DLBB_API void dlbb_attn_set_fwd_variant(int v) {
  g_attn_fwd_variant = (v >= 0 && v <= 7) || v == 14 || v == 100 ? v : 6;
}
DLBB_API int dlbb_attn_get_fwd_variant() { return g_attn_fwd_variant; }
DLBB_API void dlbb_attn_set_bwd_incr(int m) { g_attn_bwd_incr = m & 3; }
DLBB_API int dlbb_attn_get_bwd_incr() { return g_attn_bwd_incr; }

// Per-device side stream + fork/join events for the concurrent backward (created once; a fork
// through an event recorded on the caller's stream is also how a HIP-graph capture of that
// stream picks up the side-stream work).
struct AttnSide {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static AttnSide g_side[64];

static int attn_side(AttnSide** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  AttnSide& sd = g_side[dev];
  if (!sd.s) {
    if ((e = hipStreamCreateWithFlags(&sd.s, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&sd.fork, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&sd.join, hipEventDisableTiming)) != hipSuccess) return e;
  }
  *out = &sd;
  return hipSuccess;
}

// qkv: [B, T, 3, H, 64] bf16 (token row stride ld elements, 16-B aligned rows);
// out: [B, T, H, 64] bf16 (row stride ldo); lse: [B, H, T] fp32 (may be null). Causal only.
DLBB_API int dlbb_attn_fwd(const void* qkv, int64_t ld, void* out, int64_t ldo, float* lse,
                           int B, int T, int H, int D, float scale, hipStream_t stream) {
  if (B <= 0 || T <= 0 || H <= 0) return hipSuccess;
  if (D != kAttnD) return hipErrorInvalidValue;
  if (ld % 8 || ldo % 4 || (reinterpret_cast<uintptr_t>(qkv) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 7))
    return hipErrorInvalidValue;
  if (ld < 3 * H * D || ldo < H * D) return hipErrorInvalidValue;
  AttnArgs a{static_cast<const uint16_t*>(qkv), static_cast<uint16_t*>(out), lse, ld, ldo,
             B, T, H, scale * 1.4426950408889634f, g_attn_xcd};
  const dim3 grid((T + kQB - 1) / kQB, H, B);
  if (g_attn_fwd_variant == 100) {
    hipLaunchKernelGGL(attn_fwd_pipe_kernel, grid, dim3(kAttnThreads), 2 * kRing * kTileKV, stream,
                       a);
    return hipGetLastError();
  }
  switch (g_attn_fwd_variant) {
#define FWD_V(N)                                                                           \
  case N:                                                                                  \
    hipLaunchKernelGGL(attn_fwd_d64_kernel<N>, grid, dim3(kAttnThreads), 4 * kTileKV, stream, a); \
    break;
    FWD_V(1) FWD_V(2) FWD_V(3) FWD_V(4) FWD_V(5) FWD_V(6) FWD_V(7) FWD_V(14)
#undef FWD_V
    default:
      hipLaunchKernelGGL(attn_fwd_d64_kernel<0>, grid, dim3(kAttnThreads), 4 * kTileKV, stream, a);
  }
  return hipGetLastError();
}

// Backward of dlbb_attn_fwd. dout / out: [B, T, H, 64] (row stride ldo); lse: forward's;
// delta: [2, B, H, T] fp32 workspace (-delta, -LSE sqrt(D)); dqkv: [B, T, 3, H, 64] (row stride
// ld, written fully).
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
  // sequential (default): the dQ kernel produces delta / nls for the dK/dV kernel after it;
  // concurrent: both read them, so the separate delta kernel runs first
  const int fuse = g_attn_concurrent ? 0 : g_attn_fuse_delta;
  if (!fuse)
    hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3(static_cast<unsigned>((rows + 255) / 256)),
                       dim3(256), 0, stream, static_cast<const uint16_t*>(dout),
                       static_cast<const uint16_t*>(out), ldo, lse, delta, delta + rows,
                       scale, B, T, H);
  AttnBwdArgs a{static_cast<const uint16_t*>(qkv), static_cast<const uint16_t*>(dout), lse, delta,
                delta + rows, static_cast<const uint16_t*>(out), fuse,
                static_cast<uint16_t*>(dqkv), ld, ldo, B, T, H,
                scale * 1.4426950408889634f, scale, g_attn_xcd};
  // dK/dV and dQ are independent (both read Q/K/V/dO/LSE/delta, write disjoint dQKV columns):
  // dQ runs on a side stream forked after the delta kernel and joined back, so each kernel's
  // causal tail (its last, lightest blocks) overlaps the other's work instead of idling CUs
  AttnSide* sd = nullptr;
  if (g_attn_concurrent) {
    const int e = attn_side(&sd);
    if (e != hipSuccess) return e;
  }
  hipStream_t dq_stream = stream;
  if (sd) {
    hipError_t e;
    if ((e = hipEventRecord(sd->fork, stream)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(sd->s, sd->fork, 0)) != hipSuccess) return e;
    dq_stream = sd->s;
  }
  const dim3 gq((T + kQB - 1) / kQB, H, B), gk((T + kBwdKeys - 1) / kBwdKeys, H, B);
  if (g_attn_bwd_incr & 1)
    hipLaunchKernelGGL(attn_bwd_dq_d64_kernel<true>, gq, dim3(kAttnThreads), 4 * kTileKV,
                       dq_stream, a);
  else
    hipLaunchKernelGGL(attn_bwd_dq_d64_kernel<false>, gq, dim3(kAttnThreads), 4 * kTileKV,
                       dq_stream, a);
  if (g_attn_bwd_incr & 2)
    hipLaunchKernelGGL(attn_bwd_dkdv_d64_kernel<true>, gk, dim3(kAttnThreads),
                       4 * kSliceImg + 1024, stream, a);
  else
    hipLaunchKernelGGL(attn_bwd_dkdv_d64_kernel<false>, gk, dim3(kAttnThreads),
                       4 * kSliceImg + 1024, stream, a);
  if (sd) {
    hipError_t e;
    if ((e = hipEventRecord(sd->join, sd->s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(stream, sd->join, 0)) != hipSuccess) return e;
  }
  return hipGetLastError();
}
