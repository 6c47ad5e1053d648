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

namespace dlbb {

constexpr int kAttnD = 64;
constexpr int kQB = 128;        // queries per workgroup
constexpr int kKB = 64;         // keys per tile
constexpr int kAttnThreads = 256;
constexpr int kTileKV = kKB * kAttnD * 2;   // 8 KiB

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(3))) i16x4* lds_i16x4_ptr;

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
};

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

__global__ void __launch_bounds__(kAttnThreads, 2) attn_fwd_d64_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nqb = (a.T + kQB - 1) / kQB;
  const int qb = nqb - 1 - static_cast<int>(blockIdx.x);     // heaviest first
  const int h = blockIdx.y, b = blockIdx.z;
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

  attn_stage(a, base_bt, 0, hoff, tileK(0), tileV(0), wave, lane);
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) {
      attn_stage(a, base_bt, (kt + 1) * kKB, hoff, tileK(cur ^ 1), tileV(cur ^ 1), wave, lane);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const int k0 = kt * kKB;
    if (k0 <= q_hi) {                               // wave-uniform: tile has keys <= a query
      const char* tk = tileK(cur);
      const char* tv = tileV(cur);
      // ---- S^T for the two 32-key halves
      f32x16 s[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int e = 0; e < 16; ++e) s[kk][e] = 0.f;
        const int row = kk * 32 + r;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int c = 2 * ks + hi;
          const bf16x8 kf =
              *reinterpret_cast<const bf16x8*>(tk + row * 128 + ((c ^ kswz(row)) << 4));
          s[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kk], 0, 0, 0);
        }
      }
      // ---- scale, causal mask, online softmax (lane = one query; keys in registers)
      const bool diag = k0 + kKB - 1 > qw;          // some key of this tile beyond some query
      float mx = -INFINITY;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = s[kk][e] * a.scale_log2;
          if (diag) {
            const int key = k0 + kk * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
            if (key > qme) v = -INFINITY;
          }
          s[kk][e] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);   // m = -inf on the first tile -> 0
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = __builtin_amdgcn_exp2f(s[kk][e] - mn);
          s[kk][e] = p;
          ls += p;
        }
      l = l * alpha + ls;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[dt][e] *= alpha;
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
              const i16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_ptr)(tv + off));
#pragma unroll
              for (int u = 0; u < 4; ++u) vf[4 * half + u] = t[u];
            }
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
          }
        }
    }
    __builtin_amdgcn_s_barrier();                   // buffer cur is restaged next iteration
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

}  // namespace dlbb

using namespace dlbb;

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
             B, T, H, scale * 1.4426950408889634f};
  const dim3 grid((T + kQB - 1) / kQB, H, B);
  hipLaunchKernelGGL(attn_fwd_d64_kernel, grid, dim3(kAttnThreads), 4 * kTileKV, stream, a);
  return hipGetLastError();
}
