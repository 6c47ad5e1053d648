// Token + position embedding of the GPT-2 microbenchmark, forward and backward, gfx950.
//
// Forward: x[b, t, :] = wte[idx[b, t], :] + wpe[t, :] in one pass (bf16 rows, 16-B vectors,
// fp32 add) instead of a gather kernel followed by a broadcast add.
//
// Backward accumulates IN PLACE into the parameters' gradient buffers (the trainer's flat bucket
// views), so no dense [vocab, C] gradient is ever materialised, zero-filled or added:
//   * wte: the token ids arrive sorted (stable sort: ``order`` = positions in sorted order).
//     A workgroup per sorted position; the one at the start of each run of equal ids sums the
//     run's dX rows in fp32 (in position order: deterministic) and does one read-modify-write
//     of that vocabulary row. No atomics, so the result is bit-reproducible run to run.
//   * wpe: a workgroup per position t sums dX[b, t, :] over the batch (fp32), then one
//     read-modify-write of wpe_grad[t, :].
// Both parts are ONE launch (workgroups [0, B*T) do wte runs, the next T do wpe rows).
// torch's path (sort, segment offsets, dense zero-fill, compute_grad_weight, sum_and_scatter,
// two AccumulateGrad adds, a batch reduction and another add) is ~20 kernels and ~0.3 ms per
// GPT-2 step (profiles/r01_gpt2/gpt2_step_timeline_787k.txt).
#include "common.h"

#include <rocprim/block/block_radix_sort.hpp>

namespace dlbb {

constexpr int kEmbThreads = 64;   // one wave per row: C / 8 vectors strided over the lanes

__global__ void __launch_bounds__(kEmbThreads) emb_fwd_kernel(
    const int64_t* __restrict__ idx, const uint16_t* __restrict__ wte,
    const uint16_t* __restrict__ wpe, uint16_t* __restrict__ out, int T, int C, int64_t V) {
  const int64_t row = blockIdx.x;                 // b * T + t
  const int t = static_cast<int>(row % T);
  int64_t id = idx[row];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);        // invalid ids: clamped reads stay in bounds
  const uint16_t* e = wte + id * C;
  const uint16_t* p = wpe + static_cast<int64_t>(t) * C;
  uint16_t* o = out + row * C;
  for (int v = threadIdx.x; v < C / 8; v += kEmbThreads) {
    float a[8], b[8];
    load8<DT_BF16>(e, v, a);
    load8<DT_BF16>(p, v, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += b[j];
    store8<DT_BF16>(o, v, a);
  }
}

// DTG: dtype of the gradient buffers (bf16 flat buckets, or fp32).
template <int DTG>
__global__ void __launch_bounds__(kEmbThreads) emb_bwd_kernel(
    const int64_t* __restrict__ sorted_ids, const int64_t* __restrict__ order,
    const uint16_t* __restrict__ dx, void* __restrict__ wte_grad, void* __restrict__ wpe_grad,
    int64_t N, int T, int C, int64_t V) {
  const int64_t blk = blockIdx.x;
  const int nv = C / 8;
  if (blk < N) {
    if (wte_grad == nullptr) return;
    const int64_t id = sorted_ids[blk];
    if (blk > 0 && sorted_ids[blk - 1] == id) return;     // not the start of this id's run
    if (id < 0 || id >= V) return;                        // invalid ids contribute nothing
    int64_t end = blk + 1;
    while (end < N && sorted_ids[end] == id) ++end;
    for (int v = threadIdx.x; v < nv; v += kEmbThreads) {
      float acc[8];
      load8<DTG>(wte_grad, id * nv + v, acc);
      for (int64_t j = blk; j < end; ++j) {
        float d[8];
        load8<DT_BF16>(dx + order[j] * C, v, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += d[k];
      }
      store8<DTG>(wte_grad, id * nv + v, acc);
    }
    return;
  }
  if (wpe_grad == nullptr) return;
  const int t = static_cast<int>(blk - N);
  const int64_t B = N / T;
  for (int v = threadIdx.x; v < nv; v += kEmbThreads) {
    float acc[8];
    load8<DTG>(wpe_grad, static_cast<int64_t>(t) * nv + v, acc);
    for (int64_t b = 0; b < B; ++b) {
      float d[8];
      load8<DT_BF16>(dx + (b * T + t) * C, v, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += d[k];
    }
    store8<DTG>(wpe_grad, static_cast<int64_t>(t) * nv + v, acc);
  }
}

// Stable sort of the token ids for the embedding backward, in ONE workgroup (the ids are at
// most kSortMax and the vocabulary below 2^18): key and position packed into one 32-bit word
// (id << 14 | position), the blocked layout already in position order, so a radix sort on the
// id bits alone is the stable sort. Replaces torch.sort (a device memcpy of the keys plus
// several rocPRIM launches, 50 us per GPT-2 step) with one launch of pure kernel work — the
// memcpy was the only non-kernel node in the captured training step.
constexpr int kSortThreads = 1024, kSortItems = 16, kSortMax = kSortThreads * kSortItems;
constexpr int kSortPosBits = 14;                         // 2^14 = kSortMax

__global__ void __launch_bounds__(kSortThreads) sort_ids_kernel(const int64_t* __restrict__ ids,
                                                                int64_t* __restrict__ sorted,
                                                                int64_t* __restrict__ order,
                                                                int n, int key_bits) {
  using Sort = rocprim::block_radix_sort<uint32_t, kSortThreads, kSortItems>;
  __shared__ typename Sort::storage_type storage;
  uint32_t k[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const int i = threadIdx.x * kSortItems + j;           // blocked: position order
    k[j] = i < n ? (static_cast<uint32_t>(ids[i]) << kSortPosBits) | static_cast<uint32_t>(i)
                 : 0xFFFFFFFFu;
  }
  Sort().sort(k, storage, kSortPosBits, kSortPosBits + key_bits);
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const int i = threadIdx.x * kSortItems + j;
    if (i < n) {
      sorted[i] = static_cast<int64_t>(k[j] >> kSortPosBits);
      order[i] = static_cast<int64_t>(k[j] & ((1u << kSortPosBits) - 1));
    }
  }
}

}  // namespace dlbb

using namespace dlbb;

// idx int64 [N = B*T] in [0, V); wte [V, C], wpe [>= T, C], out [N, C]; bf16, C % 8 == 0,
// 16-B aligned rows.
DLBB_API int dlbb_embedding_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out,
                                int64_t N, int T, int C, int64_t V, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (C % 8 || T <= 0 || N % T) return hipErrorInvalidValue;
  auto mis = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) != 0; };
  if (mis(wte) || mis(wpe) || mis(out)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3(static_cast<unsigned>(N)), dim3(kEmbThreads),
                     0, stream, idx, static_cast<const uint16_t*>(wte),
                     static_cast<const uint16_t*>(wpe), static_cast<uint16_t*>(out), T, C, V);
  return hipGetLastError();
}

// Accumulate the embedding gradients: wte_grad[sorted_ids[i]] += dx[order[i]] (runs of equal ids
// summed in order; ids outside [0, V) are skipped), wpe_grad[t] += sum_b dx[b, t]. Either grad
// pointer may be null (skipped).
// dt_grad: 1 bf16, 0 fp32 (both grads). dx bf16 [N = B*T, C].
DLBB_API int dlbb_embedding_bwd(const int64_t* sorted_ids, const int64_t* order, const void* dx,
                                void* wte_grad, void* wpe_grad, int dt_grad, int64_t N, int T,
                                int C, int64_t V, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (C % 8 || T <= 0 || N % T) return hipErrorInvalidValue;
  auto mis = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) != 0; };
  if (mis(dx) || mis(wte_grad) || mis(wpe_grad)) return hipErrorInvalidValue;
  const dim3 g(static_cast<unsigned>(N + T));
  const auto* d = static_cast<const uint16_t*>(dx);
  if (dt_grad == DT_BF16)
    hipLaunchKernelGGL(emb_bwd_kernel<DT_BF16>, g, dim3(kEmbThreads), 0, stream, sorted_ids,
                       order, d, wte_grad, wpe_grad, N, T, C, V);
  else if (dt_grad == DT_F32)
    hipLaunchKernelGGL(emb_bwd_kernel<DT_F32>, g, dim3(kEmbThreads), 0, stream, sorted_ids,
                       order, d, wte_grad, wpe_grad, N, T, C, V);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// sorted / order (int64, n each) = the stable ascending sort of ids and the positions it took.
// hipErrorNotSupported when n > 16384 or vocab > 2^18 (the caller falls back to a library sort).
DLBB_API int dlbb_sort_ids(const int64_t* ids, int64_t* sorted, int64_t* order, int64_t n,
                           int vocab, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (n > kSortMax || vocab <= 0 || vocab > (1 << 18)) return hipErrorNotSupported;
  int bits = 1;
  while ((1 << bits) < vocab) ++bits;
  hipLaunchKernelGGL(sort_ids_kernel, dim3(1), dim3(kSortThreads), 0, stream, ids, sorted, order,
                     static_cast<int>(n), bits);
  return hipGetLastError();
}
