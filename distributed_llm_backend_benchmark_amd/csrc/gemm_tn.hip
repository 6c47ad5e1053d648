// Weight-gradient GEMM, gfx950: dW[N][K] = sum_m dY[m][N] * X[m][K]   (reduction over ROWS).
//
// Training backward of every linear (GPT-2, TP model): dW = dY^T X with M = tokens (16 K) and a
// small output (768 x 768 .. 3072 x 768). The library picks 128^2..256^2 tiles without enough
// split-K and reaches 210-530 TFLOP/s on these shapes (profiles/r01_gpt2). Here:
//   * both operands are row-major over the reduction index m, so MFMA fragments (8 consecutive m
//     of one column) come from ds_read_b64_tr_b16 transposed reads of [64 m][128 col] LDS tiles
//     staged by LDS-DMA (global_load_lds 16 B) — no transpose pass over the activations;
//   * LDS image swizzle: 16-B chunk c of row m lives in slot c ^ 2 h(m), h(m) = (m & 3) |
//     ((m >> 3) & 1) << 2, which makes the 8 rows a 32-lane half reads hit 8 disjoint 32-B bank
//     groups (conflict-free; a plain 256-B-row image is 8-way);
//   * split-K over m: fp32 partials [split][N][K], then one reduce + bf16 cast kernel
//     (deterministic; no float atomics);
//   * optional fused bias gradient db[n] = sum_m dY[m][n]: the workgroups of output column
//     block 0 also multiply their dY fragments by an all-ones B operand (two extra MFMAs per
//     k-step per wave, the fragments are already in registers), partials [split][N] go through
//     the same reduce kernel — replaces a separate column-sum pass over dY.
// 128 x 128 output tile per workgroup, 4 waves in 2 x 2 (64 x 64 each = 4 x 4 MFMA 16x16x32),
// BM = 32 rows of m per stage, two LDS buffers (32 KiB: three workgroups per CU).
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace dlbb {

namespace tn {

constexpr int BKO = 128, BM = 32;                 // output cols (K) per tile, reduction rows/stage
constexpr int kTile = BM * 128 * 2;               // 8 KiB per [BM][128] image


__device__ __forceinline__ int swz(int m) { return ((m & 3) | (((m >> 3) & 1) << 2)) << 1; }

struct Args {
  const uint16_t* A;   // [M][lda]  (dY)
  const uint16_t* B;   // [M][ldb]  (X)
  float* ws;           // [split][N][K]
  int64_t lda, ldb;
  int M, N, K;
  int m_per_split;
  int nsplit;          // fused db partials (BIAS) at ws + nsplit * N * K (tk == 0 blocks)
  void* direct;        // nsplit == 1, no accumulate, no bias: store dW here (no ws, no reduce)
  int direct_bf16;     // direct / fused-reduce store dtype: bf16 (1) or fp32 (0)
  // in-launch split-K reduce (cnt != null): per-tile arrival counters (zero on entry; the last
  // arriver resets its own), the final dW / db and whether to add into them
  int* cnt;
  void* out;
  void* out_bias;
  int accumulate;
  int tile_major;      // workgroup order: 0 = split-major, 1 = a tile's splits adjacent
};

// SB16 (bf16 dW outputs): the dW partial slabs are bf16, slab s = the first half of the bytes of
// fp32 slab s of ws — half the split-K round trip's traffic; the db partials stay fp32. fp32
// outputs keep fp32 slabs (their contract is fp32 accuracy).
template <bool SB16>
__device__ __forceinline__ f32x4 slab_ld4(const float* slab, int64_t off) {
  if constexpr (SB16) {
    const u16x4 v = *reinterpret_cast<const u16x4*>(reinterpret_cast<const uint16_t*>(slab) + off);
    return f32x4{bf16_to_f32(v[0]), bf16_to_f32(v[1]), bf16_to_f32(v[2]), bf16_to_f32(v[3])};
  } else {
    return *reinterpret_cast<const f32x4*>(slab + off);
  }
}

// The last-arriving workgroup of a tile sums the `nsplit` fp32 slabs of that tile (+ the fused
// bias partials of column block 0) and writes the final bf16 / fp32 dW — replaces the separate
// split_reduce_kernel pass (profiles/r04_final/gpt2_kernel_stats_steady.csv:5: 40 us x 50 calls
// per GPT-2 step). Slab reads are 16-B, coalesced along K, 8 independent loads per thread per
// slab; NT threads cover the BNxTBK tile in TBK / 8 float4 per thread, 8 at a time.
template <int NT, int BN, int TBK, bool SB16>
__device__ __forceinline__ void wgrad_tile_reduce(const Args& a, int n0, int k0, bool bias) {
  constexpr int C4 = TBK / 4;                      // float4 per tile row
  constexpr int PER = BN * C4 / NT;                // float4 per thread
  static_assert(PER % 8 == 0, "tile must split into 8-float4 chunks per thread");
  const int64_t slab = static_cast<int64_t>(a.N) * a.K;
#pragma unroll 1
  for (int ch = 0; ch < PER / 8; ++ch) {
    f32x4 acc[8];
    int64_t off[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int f = (ch * 8 + u) * NT + static_cast<int>(threadIdx.x);
      off[u] = static_cast<int64_t>(n0 + f / C4) * a.K + k0 + (f % C4) * 4;
      acc[u] = slab_ld4<SB16>(a.ws, off[u]);
    }
#pragma unroll 2
    for (int s = 1; s < a.nsplit; ++s) {
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = slab_ld4<SB16>(a.ws + s * slab, off[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += t[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (a.direct_bf16) {
        uint16_t* o = static_cast<uint16_t*>(a.out) + off[u];
        float v[4] = {acc[u][0], acc[u][1], acc[u][2], acc[u][3]};
        if (a.accumulate) {
          const u16x4 p = *reinterpret_cast<const u16x4*>(o);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += bf16_to_f32(p[j]);
        }
        u16x4 r;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = f32_to_bf16(v[j]);
        *reinterpret_cast<u16x4*>(o) = r;
      } else {
        f32x4* o = reinterpret_cast<f32x4*>(static_cast<float*>(a.out) + off[u]);
        *o = a.accumulate ? *o + acc[u] : acc[u];
      }
    }
  }
  if (bias && static_cast<int>(threadIdx.x) < BN) {
    const float* wb = a.ws + static_cast<int64_t>(a.nsplit) * slab + n0 + threadIdx.x;
    float s0 = 0.f;
    for (int s = 0; s < a.nsplit; ++s) s0 += wb[static_cast<int64_t>(s) * a.N];
    const int n = n0 + threadIdx.x;
    if (a.direct_bf16) {
      uint16_t* o = static_cast<uint16_t*>(a.out_bias) + n;
      *o = f32_to_bf16(a.accumulate ? s0 + bf16_to_f32(*o) : s0);
    } else {
      float* o = static_cast<float*>(a.out_bias) + n;
      *o = a.accumulate ? s0 + *o : s0;
    }
  }
}

// MFMA 16x16x32 operand from a [64 m][128 col] image: lane l gets column colbase + (l & 15),
// rows 32 KS + 8 (l >> 4) + j, j = 0..7 (two transposed reads of 4 rows each). swz(row) is the
// same for every (KS, half) (row & 3 = q, bit 3 = g & 1), so the rows' offset (32 KS + 4 half)
// x 256 is the reads' immediate. Asm reads (common.h ds_read_tr16): the caller waits lgkmcnt(0)
// before using the fragment.
template <int KS>
__device__ __forceinline__ bf16x8 frag(const char* img, int colbase, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int r0 = 8 * g + q;
  const int col = colbase + 4 * p;
  const char* base = img + r0 * 256 + (((col >> 3) ^ swz(r0)) << 4) + (col & 7) * 2;
  const i16x4 t0 = ds_read_tr16<KS * 8192>(base), t1 = ds_read_tr16<KS * 8192 + 1024>(base);
  bf16x8 f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f[u] = t0[u];
    f[4 + u] = t1[u];
  }
  return f;
}

// One stage = BM rows of m of the NA = WM / 2 A sub-images ([BM][128 cols of dY] each) and the B
// image ([BM][128 cols of X]); every 4-row x 256-B wave-instruction of the stage is one slot
// j = wave * per + q of NIMG * BM / 4, spread evenly over the workgroup's waves.
// buffer_load ... lds with the split's operand bases in buffer resources (SGPRs): the lane's
// row-in-group and swizzled chunk are a loop-invariant 32-bit voffset, the stage's row the
// uniform soffset. The former global_load_lds form rebuilt a 64-bit address per load every
// stage: 78 VALU (12 v_mul_lo_u32, 6 v_mad_u64_u32) per 34 MFMAs, 3.35 VALU instructions per
// MFMA over the kernel (PMC, profiles/r06_kernels/pmc_wgradqkv_summary.jsonl) — issue slots the
// 16x16x32 MFMAs' 8 free cycles cannot hold. Host contract: every offset below 2 GiB.
template <int WM, int WJ = 4>
__device__ __forceinline__ void stage_all(__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb,
                                          uint32_t lda2, uint32_t ldb2, uint32_t mrel, int n0,
                                          int k0, char* buf, int wave, int lane) {
  constexpr int NA = WM / 2, NIMG = NA + WJ / 4, RG = BM / 4, NW = 2 * WM;
  constexpr int PER = NIMG * RG / NW;
  static_assert(NIMG * RG % NW == 0, "stage slots must divide evenly over the waves");
  const int rq = lane >> 4, slot = lane & 15;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int j = wave * PER + q;
    const int img = j / RG, rg = j % RG;
    const int row = rg * 4 + rq;
    const int chunk = slot ^ swz(row);
    const bool is_a = img < NA;
    const uint32_t ld2 = is_a ? lda2 : ldb2;
    const int c0 = is_a ? n0 + img * 128 : k0 + (img - NA) * 128;
    const uint32_t voff = static_cast<uint32_t>(rq) * ld2 + static_cast<uint32_t>(c0 + chunk * 8) * 2;
    const uint32_t soff = (mrel + static_cast<uint32_t>(rg * 4)) * ld2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(is_a ? ra : rb,
                                             (lds_vptr_t)(buf + img * kTile + rg * 4 * 256), 16,
                                             voff, soff, 0, 0);
  }
}

// BIAS: a separate instantiation (two extra accumulators + the ones operand). NB: LDS ring
// depth (stages) — NB - 1 stages of DMA in flight while one is consumed. WM: output rows (N) per
// workgroup in 64-row wave blocks — 2: 128 x 128 tile, 4 waves, three workgroups per CU;
// 4: 256 x 128 tile, 8 waves, two per CU: 1.33x the MFMA work per byte staged through L2 (the
// 128 x 128 tile needs ~64 FLOP per L2 byte, more than the L2 delivers at the MFMA rate).
// WJ: 16-column B fragments per wave — 4: 64 x 64 per wave (128 output columns per tile), 8:
// 64 x 128 per wave (256 columns per tile): 25 % fewer LDS fragment bytes per MFMA and 2/3 of the
// DMA per output of the 128 x 128 tile; the 128-column kernels are LDS-bound (GPT-2 dW shapes).
template <bool BIAS, int NB, int WM, int WJ = 4, bool SB16 = false>
__global__ void __launch_bounds__(128 * WM, WJ == 8 ? 2 : (WM == 2 ? 3 : 2))
    wgrad_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NIMG = WM / 2 + WJ / 4;
  constexpr int TBK = 32 * WJ;                    // output columns (K) per tile
  constexpr int kStage = NIMG * kTile;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // workgroup -> (split, tile): XCD-aware bijective remap (guide T1; blockIdx % 8 labels the
  // blocks that share an L2), then split-major / row-block-major order, so the ~1/8 of the grid
  // that shares an XCD is a contiguous run of tiles of one split: its dY column blocks are
  // re-read by the tiles_k workgroups of a row and its X blocks by every row — from that L2
  // instead of from the Infinity Cache / HBM (the default round-robin puts neighbours on
  // different XCDs, so every workgroup fetched its panels from beyond L2).
  const int tiles_k = a.K / TBK;
  const int tiles = (a.N / (64 * WM)) * tiles_k;
  const int nwg = gridDim.x, xcd = blockIdx.x % 8, q = nwg / 8, r = nwg % 8;
  const int wid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + blockIdx.x / 8;
  // tile_major: a tile's nsplit slices are adjacent ids, i.e. mostly on one XCD, so the
  // in-launch reducer reads its slabs from its own L2 (guide: 104-122 vs 62-70 GB/s per block)
  const int split = a.tile_major ? wid % a.nsplit : wid / tiles;
  const int t = a.tile_major ? wid / a.nsplit : wid % tiles;
  const int tn = t / tiles_k, tk = t % tiles_k;
  const int n0 = tn * 64 * WM, k0 = tk * TBK;
  const int mb = split * a.m_per_split;
  const int me = mb + a.m_per_split < a.M ? mb + a.m_per_split : a.M;
  const int nsteps = (me - mb) / BM;

  f32x4 acc[4][WJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias: wave (wm, wn) of a column-block-0 workgroup sums fragments i = 2 wn, 2 wn + 1
  const bool do_bias = BIAS && tk == 0;
  f32x4 bacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  bf16x8 ones;
#pragma unroll
  for (int u = 0; u < 8; ++u) ones[u] = static_cast<short>(0x3F80);

  auto stg = [&](int c) { return smem + c * kStage; };
  // this wave's A sub-image (128 dY columns) and the row offset of its 64 inside it
  const int asub = (wm * 64) / 128, acol = (wm * 64) % 128;
  // and its B image / column offset (WJ = 8: one whole 128-column image per wave)
  const int bsub = WM / 2 + (wn * 16 * WJ) / 128, bcol = (wn * 16 * WJ) % 128;
  constexpr int kLoadsPerStage = NIMG * (BM / 4) / (2 * WM);   // buffer_load lds per wave
  // the split's rows [mb, me) of dY and X as buffer resources (offsets < 2 GiB: host contract)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.A + static_cast<int64_t>(mb) * a.lda), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.B + static_cast<int64_t>(mb) * a.ldb), 0, 0x7fffffff, 0x00020000);
  const uint32_t lda2 = static_cast<uint32_t>(a.lda) * 2, ldb2 = static_cast<uint32_t>(a.ldb) * 2;
#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < nsteps)
      stage_all<WM, WJ>(ra, rb, lda2, ldb2, p * BM, n0, k0, stg(p), wave, lane);
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s % NB;
    // stage s landed: later stages (up to NB - 2 of them) may still be in flight
    const int ahead = nsteps - 1 - s < NB - 2 ? nsteps - 1 - s : NB - 2;
    if (NB >= 4 && ahead >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * kLoadsPerStage) : "memory");
    else if (NB >= 3 && ahead >= 1)
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kLoadsPerStage) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // one barrier per stage: it publishes stage s (every wave's DMA of it retired) and frees
    // the buffer of stage s - 1 (every wave finished it), which stage s + NB - 1 now refills
    __builtin_amdgcn_s_barrier();
    if (s + NB - 1 < nsteps)
      stage_all<WM, WJ>(ra, rb, lda2, ldb2, (s + NB - 1) * BM, n0, k0, stg((s + NB - 1) % NB),
                        wave, lane);
    const char* ia = stg(cur) + asub * kTile;
    const char* ib = stg(cur) + bsub * kTile;
    auto kstep = [&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      bf16x8 af[4], bfr[WJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<ks>(ia, acol + i * 16, lane);
#pragma unroll
      for (int j = 0; j < WJ; ++j) bfr[j] = frag<ks>(ib, bcol + j * 16, lane);
      tr_wait(af[0]);                    // the asm reads' results (frag)
#pragma unroll
      for (int i = 1; i < 4; ++i) tr_tie(af[i]);
#pragma unroll
      for (int j = 0; j < WJ; ++j) tr_tie(bfr[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (do_bias) {   // wave-uniform branches on wn (a runtime index into af[] would
                       // become v_cndmask chains over every fragment register)
        if (wn == 0) {
          bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], ones, bacc[0], 0, 0, 0);
          bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], ones, bacc[1], 0, 0, 0);
        } else {
          bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], ones, bacc[0], 0, 0, 0);
          bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[3], ones, bacc[1], 0, 0, 0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    };
    static_assert(BM == 32, "one 32-deep k-step per stage");
    kstep(std::integral_constant<int, 0>{});
  }
  // D map: col = lane & 15 (output k), row = 4 (lane >> 4) + r (output n)
  const int fr = lane & 15, fq = lane >> 4;
  if (!BIAS && a.direct) {    // one split: the tile is final — no fp32 partial round trip
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t o = static_cast<int64_t>(n0 + wm * 64 + i * 16 + fq * 4 + r) * a.K +
                            k0 + wn * 16 * WJ + j * 16 + fr;
          if (a.direct_bf16)
            static_cast<uint16_t*>(a.direct)[o] = f32_to_bf16(acc[i][j][r]);
          else
            static_cast<float*>(a.direct)[o] = acc[i][j][r];
        }
    return;
  }
  float* w = a.ws + static_cast<int64_t>(split) * a.N * a.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * 64 + i * 16 + fq * 4 + r;
        const int k = k0 + wn * 16 * WJ + j * 16 + fr;
        if constexpr (SB16)
          reinterpret_cast<uint16_t*>(w)[static_cast<int64_t>(n) * a.K + k] =
              f32_to_bf16(acc[i][j][r]);
        else
          w[static_cast<int64_t>(n) * a.K + k] = acc[i][j][r];
      }
  if (do_bias && fr == 0) {   // every D column holds the same sum; lanes 0/16/32/48 write
    float* wb = a.ws + static_cast<int64_t>(a.nsplit) * a.N * a.K +
                static_cast<int64_t>(split) * a.N;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) wb[n0 + wm * 64 + (2 * wn + h) * 16 + fq * 4 + r] = bacc[h][r];
  }
  if (!a.cnt) return;
  // in-launch split-K combine (guide §5 "In-launch split-K reduction", counter form): every
  // wave's slab stores retired -> barrier -> ONE agent release -> ticket; the workgroup drawing
  // nsplit - 1 acquires once and reduces. The explicit waits after the fences are kept on
  // purpose (ROCm 7.2 may drop the fence's own wait).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* last = reinterpret_cast<int*>(smem);        // LDS is free: the k-loop is over
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(a.cnt + t, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    const int is_last = prev == a.nsplit - 1;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // re-arm for the next launch on this stream (kernel boundary orders it)
      __hip_atomic_store(a.cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last[0] = is_last;
  }
  __syncthreads();
  if (!last[0]) return;
  wgrad_tile_reduce<128 * WM, 64 * WM, TBK, SB16>(a, n0, k0, BIAS && tk == 0);
}

// out[i] = sum_s ws[s][i] (+ out[i] if accumulate), bf16 or fp32 output; 8 elements / thread.
// Vectors past n / 8 reduce the bias partials ([split][nb] after the weight partials) into outb.
// Sum of `split` fp32 slabs (+ optional existing output), one 16-byte float4 per thread per
// item. S > 0: the split count is a template constant, so all S slab loads of an item are
// issued before the first add (S x 16 B in flight per lane); S == 0: runtime split, 8 slabs per
// load batch. The previous form (8 floats per thread, one slab per loop trip) waited for every
// slab in turn: 40 us per GPT-2 dW call, ~2 TB/s (profiles/r04_final/gpt2_kernel_stats_steady.csv:5).
template <int S, bool NT>
__device__ __forceinline__ f32x4 ld_slab(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int S, bool NT>
__device__ __forceinline__ f32x4 sum_slabs(const float* __restrict__ src, int64_t ld, int64_t vi,
                                           int split) {
  const f32x4* p = reinterpret_cast<const f32x4*>(src) + vi;
  const int64_t ld4 = ld / 4;
  if constexpr (S > 0) {
    f32x4 t[S];
#pragma unroll
    for (int s = 0; s < S; ++s) t[s] = ld_slab<S, NT>(p + s * ld4);
#pragma unroll
    for (int s = 1; s < S; ++s) t[0] += t[s];
    return t[0];
  } else {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 8 <= split; s += 8) {
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = ld_slab<S, NT>(p + (s + u) * ld4);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; s < split; ++s) acc += ld_slab<S, NT>(p + s * ld4);
    return acc;
  }
}

// sum_slabs over bf16 slabs (SB16 layout above)
template <int S, bool NT>
__device__ __forceinline__ f32x4 sum_slabs_b16(const float* __restrict__ src, int64_t ld,
                                               int64_t vi, int split) {
  auto ld16 = [&](int s) {
    const u16x4* p = reinterpret_cast<const u16x4*>(src + static_cast<int64_t>(s) * ld) + vi;
    const u16x4 v = NT ? __builtin_nontemporal_load(p) : *p;
    return f32x4{bf16_to_f32(v[0]), bf16_to_f32(v[1]), bf16_to_f32(v[2]), bf16_to_f32(v[3])};
  };
  if constexpr (S > 0) {
    f32x4 t[S];
#pragma unroll
    for (int s = 0; s < S; ++s) t[s] = ld16(s);
#pragma unroll
    for (int s = 1; s < S; ++s) t[0] += t[s];
    return t[0];
  } else {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < split; ++s) acc += ld16(s);
    return acc;
  }
}

template <int DTO, int S, bool NT, bool SB = false>
__global__ void __launch_bounds__(256) split_reduce_kernel(const float* __restrict__ ws,
                                                           void* __restrict__ out, int64_t n,
                                                           void* __restrict__ outb, int64_t nb,
                                                           int split, int accumulate) {
  const int64_t nv = n / 4, nvb = nb / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nv + nvb;
       v += stride) {
    const bool is_b = v >= nv;
    const float* src = is_b ? ws + split * n : ws;
    const int64_t ld = is_b ? nb : n, vi = is_b ? v - nv : v;
    void* dst = is_b ? outb : out;
    f32x4 acc = SB && !is_b ? sum_slabs_b16<S, NT>(src, ld, vi, split)
                            : sum_slabs<S, NT>(src, ld, vi, split);
    if constexpr (DTO == DT_F32) {
      f32x4* o = static_cast<f32x4*>(dst) + vi;
      *o = accumulate ? *o + acc : acc;
    } else {
      u16x4* o = static_cast<u16x4*>(dst) + vi;
      if (accumulate) {
        const u16x4 p = *o;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += bf16_to_f32(p[j]);
      }
      u16x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = f32_to_bf16(acc[j]);
      *o = r;
    }
  }
}

// Round-4 form (A/B variant 0): 8 floats per thread, one slab per loop trip.

// split-reduce form: every slab load in flight, non-temporal loads. Round 5 measured it against
// an 8-float form and plain loads: all three 4.5-5.4 TB/s at the GPT-2 dW shapes isolated
// (11-18 us; this one fastest by 2-5 %, profiles/r05_kernels/split_reduce.jsonl); the slabs are
// read once, so streaming loads also keep them from displacing the main stream's L2 lines.

template <int DTO, bool NT, bool SB>
static void split_reduce_dispatch_v(const float* ws, void* out, int64_t n, void* outb, int64_t nb,
                                    int split, int accumulate, hipStream_t stream) {
  const int g = stream_grid((n + nb) / 4, 256);
#define SR(SV)                                                                                   \
  case SV:                                                                                       \
    hipLaunchKernelGGL((split_reduce_kernel<DTO, SV, NT, SB>), dim3(g), dim3(256), 0, stream, ws, \
                       out, n, outb, nb, split, accumulate);                                     \
    return;
  switch (split) {
    SR(1) SR(2) SR(3) SR(4) SR(5) SR(6) SR(7) SR(8) SR(9) SR(10) SR(11) SR(12) SR(16)
    default:
      hipLaunchKernelGGL((split_reduce_kernel<DTO, 0, NT, SB>), dim3(g), dim3(256), 0, stream, ws,
                         out, n, outb, nb, split, accumulate);
  }
#undef SR
}

template <int DTO, bool SB = false>
static void split_reduce_dispatch(const float* ws, void* out, int64_t n, void* outb, int64_t nb,
                                  int split, int accumulate, hipStream_t stream) {
  split_reduce_dispatch_v<DTO, true, SB>(ws, out, n, outb, nb, split, accumulate, stream);
}

}  // namespace tn
}  // namespace dlbb

using namespace dlbb;

// LDS ring depth of the wgrad kernel (A/B: dlbb_gemm_wgrad_set_stages)
static int g_wgrad_stages = 2;

DLBB_API void dlbb_gemm_wgrad_set_stages(int nb) { g_wgrad_stages = nb >= 2 && nb <= 4 ? nb : 2; }


// dW[N][K] = A^T B with A = [M][lda] (N columns used), B = [M][ldb] (K columns used), bf16.
// Requires M % 32 == 0, N % bn == 0, K % 128 == 0, lda/ldb % 8 == 0, 16-B aligned bases;
// bn = 128 (128 x 128 tiles) or 256 (256 x 128 tiles). ws: fp32 workspace of
// split * (N * K + N) floats. out: bf16 (dt_out 1) or fp32 (0), dense [N][K]. out_bias
// (optional, same dtype as out, N elements): fused db = column sums of A.
// bk: output columns (K) per tile, 128 or 256 (the latter with bn = 128 only: 64 x 128 per wave).
// workgroup order of the fused-reduce launches (A/B: dlbb_gemm_wgrad_set_order)
static int g_wgrad_tile_major = 1;

DLBB_API void dlbb_gemm_wgrad_set_order(int tile_major) { g_wgrad_tile_major = tile_major ? 1 : 0; }

// Number of per-tile arrival counters a fused-reduce launch of this shape needs.
DLBB_API int dlbb_gemm_wgrad_counters(int N, int K, int bn, int bk) {
  return bn > 0 && bk > 0 ? (N / bn) * (K / bk) : 0;
}

static int wgrad_launch(const void* A, int64_t lda, const void* B, int64_t ldb, void* out,
                        int dt_out, int accumulate, float* ws, int M, int N, int K, int split,
                        void* out_bias, int bn, int bk, int* counters, int ncounters,
                        hipStream_t stream) {
  using namespace dlbb::tn;
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (bn != 128 && bn != 256) return hipErrorInvalidValue;
  if (bk != 128 && !(bk == 256 && bn == 128)) return hipErrorInvalidValue;
  if (M % BM || N % bn || K % bk || lda % 8 || ldb % 8 || split < 1) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) |
       reinterpret_cast<uintptr_t>(ws)) & 15)
    return hipErrorInvalidValue;
  int per = (M / split + BM - 1) / BM * BM;
  if (per <= 0) per = BM;
  split = (M + per - 1) / per;
  // buffer offsets from a split's first row stay below 2 GiB (wgrad_kernel's resources)
  if (static_cast<int64_t>(per) * (lda > ldb ? lda : ldb) * 2 >= (int64_t{1} << 31))
    return hipErrorInvalidValue;
  // one split, plain store, no bias: the kernel writes dW itself (ws may be null)
  const bool direct = split == 1 && !accumulate && !out_bias;
  if (!direct && !ws) return hipErrorInvalidValue;
  const int ntiles = (N / bn) * (K / bk);
  // in-launch combine: needs one zeroed counter per tile and 16-B aligned outputs
  const bool fused = !direct && counters && ncounters >= ntiles &&
                     !((reinterpret_cast<uintptr_t>(out) |
                        reinterpret_cast<uintptr_t>(counters)) & 15);
  if (counters && !direct && !fused) return hipErrorInvalidValue;
  Args a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), ws, lda, ldb, M, N, K,
         per, split, direct ? out : nullptr, dt_out == DT_BF16 ? 1 : 0,
         fused ? counters : nullptr, out, out_bias, accumulate,
         fused ? g_wgrad_tile_major : 0};
  const dim3 grid((N / bn) * (K / bk) * split);
  const int stages = g_wgrad_stages;
  const bool sb16 = dt_out == DT_BF16;   // bf16 partial slabs for bf16 dW (SB16)
#define WG_LAUNCH(BIASV, NBV, WMV, WJV)                                                     \
  do {                                                                                      \
    if (sb16)                                                                               \
      hipLaunchKernelGGL((wgrad_kernel<BIASV, NBV, WMV, WJV, true>), grid,                  \
                         dim3(128 * (WMV)), NBV * ((WMV) / 2 + (WJV) / 4) * kTile, stream, a); \
    else                                                                                    \
      hipLaunchKernelGGL((wgrad_kernel<BIASV, NBV, WMV, WJV, false>), grid,                 \
                         dim3(128 * (WMV)), NBV * ((WMV) / 2 + (WJV) / 4) * kTile, stream, a); \
  } while (0)
#define WG_STAGES(BIASV, WMV, WJV)                \
  if (stages == 4) WG_LAUNCH(BIASV, 4, WMV, WJV); \
  else if (stages == 3) WG_LAUNCH(BIASV, 3, WMV, WJV); \
  else WG_LAUNCH(BIASV, 2, WMV, WJV)
  if (bk == 256) {
    if (out_bias) { WG_STAGES(true, 2, 8); } else { WG_STAGES(false, 2, 8); }
  } else if (bn == 256) {
    if (out_bias) { WG_STAGES(true, 4, 4); } else { WG_STAGES(false, 4, 4); }
  } else {
    if (out_bias) { WG_STAGES(true, 2, 4); } else { WG_STAGES(false, 2, 4); }
  }
#undef WG_STAGES
#undef WG_LAUNCH
  if (direct || fused) return hipGetLastError();
  const int64_t n = static_cast<int64_t>(N) * K;
  const int64_t nb = out_bias ? N : 0;
  if (dt_out == DT_BF16)
    split_reduce_dispatch<DT_BF16, true>(ws, out, n, out_bias, nb, split, accumulate, stream);
  else
    split_reduce_dispatch<DT_F32>(ws, out, n, out_bias, nb, split, accumulate, stream);
  return hipGetLastError();
}

// The weight-gradient split-K reduce alone (microbenchmarks): out[n] (+ outb[nb]) = sum of the
// `split` fp32 slabs of ws laid out as the wgrad kernel writes them (n slabs, then nb slabs).
DLBB_API int dlbb_split_reduce(const float* ws, void* out, int dt_out, int64_t n, void* outb,
                               int64_t nb, int split, int accumulate, hipStream_t stream) {
  if (n % 8 || nb % 8 || split < 1) return hipErrorInvalidValue;
  if (dt_out == DT_BF16)
    tn::split_reduce_dispatch<DT_BF16>(ws, out, n, outb, nb, split, accumulate, stream);
  else
    tn::split_reduce_dispatch<DT_F32>(ws, out, n, outb, nb, split, accumulate, stream);
  return hipGetLastError();
}

DLBB_API int dlbb_gemm_wgrad_tile2(const void* A, int64_t lda, const void* B, int64_t ldb,
                                   void* out, int dt_out, int accumulate, float* ws, int M, int N,
                                   int K, int split, void* out_bias, int bn, int bk,
                                   hipStream_t stream) {
  return wgrad_launch(A, lda, B, ldb, out, dt_out, accumulate, ws, M, N, K, split, out_bias, bn,
                      bk, nullptr, 0, stream);
}

// As tile2, with the split-K combine done inside the launch by each tile's last-arriving
// workgroup: `counters` = dlbb_gemm_wgrad_counters(N, K, bn, bk) ints, ZERO on entry (the
// launch leaves them zero again), owned by one stream at a time. A one-split plain store still
// takes the direct path (no counters touched).
DLBB_API int dlbb_gemm_wgrad_fused(const void* A, int64_t lda, const void* B, int64_t ldb,
                                   void* out, int dt_out, int accumulate, float* ws, int M, int N,
                                   int K, int split, void* out_bias, int bn, int bk,
                                   int* counters, int ncounters, hipStream_t stream) {
  if (!counters) return hipErrorInvalidValue;
  return wgrad_launch(A, lda, B, ldb, out, dt_out, accumulate, ws, M, N, K, split, out_bias, bn,
                      bk, counters, ncounters, stream);
}

DLBB_API int dlbb_gemm_wgrad_tile(const void* A, int64_t lda, const void* B, int64_t ldb,
                                  void* out, int dt_out, int accumulate, float* ws, int M, int N,
                                  int K, int split, void* out_bias, int bn, hipStream_t stream) {
  return dlbb_gemm_wgrad_tile2(A, lda, B, ldb, out, dt_out, accumulate, ws, M, N, K, split,
                               out_bias, bn, 128, stream);
}

// out (bf16, or fp32 when dt_f32) = sum over `split` fp32 slices of n elements (n % 8 == 0);
// used by the NN dgrad's split-K (csrc/gemm.hip).
int dlbb_split_reduce_launch(const float* ws, void* out, int dt_f32, int64_t n, int split,
                             hipStream_t stream) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  if (dt_f32)
    tn::split_reduce_dispatch<DT_F32>(ws, out, n, nullptr, 0, split, 0, stream);
  else
    tn::split_reduce_dispatch<DT_BF16>(ws, out, n, nullptr, 0, split, 0, stream);
  return hipGetLastError();
}

DLBB_API int dlbb_gemm_wgrad(const void* A, int64_t lda, const void* B, int64_t ldb, void* out,
                             int dt_out, int accumulate, float* ws, int M, int N, int K,
                             int split, void* out_bias, hipStream_t stream) {
  return dlbb_gemm_wgrad_tile(A, lda, B, ldb, out, dt_out, accumulate, ws, M, N, K, split,
                              out_bias, 128, stream);
}
