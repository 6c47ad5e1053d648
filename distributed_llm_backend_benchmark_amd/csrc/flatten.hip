// Multi-tensor flatten / unflatten / all-to-all split packing in ONE launch.
//
// The reference stages tensor lists through Python: `dist.all_gather` into a list
// (collectives/1d/dsccl.py:72-76), all-to-all split lists built with
// `data[i*c:(i+1)*c].clone()` (collectives/1d/dsccl.py:137-138, collectives/1d/openmpi.py:161-162).
// Here any list of (src, dst, nbytes) copies is described by a device-resident chunk table
// (built once per layout on the host, ≤ kChunkBytes per entry) and executed by one
// grid-stride kernel: each workgroup walks chunks, moving 16 B per lane when src/dst/nbytes
// are 16-B aligned. Used for DDP gradient buckets (flatten grads -> bucket, unflatten
// reduced bucket -> grads with the 1/world scale fused) and for MoE token packing.
#include "common.h"

namespace dlbb {

struct CopyChunk {
  uint64_t src;
  uint64_t dst;
  uint64_t nbytes;
};

template <bool NT>
__global__ void __launch_bounds__(256) chunk_copy_kernel(const CopyChunk* __restrict__ table,
                                                         int64_t nchunks) {
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const CopyChunk ch = table[c];
    const char* s = reinterpret_cast<const char*>(ch.src);
    char* d = reinterpret_cast<char*>(ch.dst);
    const uint64_t nb = ch.nbytes;
    if (((ch.src | ch.dst) & 15) == 0) {
      const uint64_t nv = nb >> 4;
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4* __restrict__ s4 = reinterpret_cast<const u32x4*>(s);
      u32x4* __restrict__ d4 = reinterpret_cast<u32x4*>(d);
      uint64_t i = threadIdx.x;
      for (; i + 3 * 256 < nv; i += 4 * 256) {   // 4 x 16 B in flight per lane before a store
        u32x4 t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = s4[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if constexpr (NT) __builtin_nontemporal_store(t[u], d4 + i + u * 256);
          else d4[i + u * 256] = t[u];
        }
      }
      for (; i < nv; i += blockDim.x) d4[i] = s4[i];
      for (uint64_t i = (nv << 4) + threadIdx.x; i < nb; i += blockDim.x) d[i] = s[i];
    } else if (((ch.src | ch.dst | nb) & 1) == 0) {
      const uint16_t* s2 = reinterpret_cast<const uint16_t*>(s);
      uint16_t* d2 = reinterpret_cast<uint16_t*>(d);
      for (uint64_t i = threadIdx.x; i < (nb >> 1); i += blockDim.x) d2[i] = s2[i];
    } else {
      for (uint64_t i = threadIdx.x; i < nb; i += blockDim.x) d[i] = s[i];
    }
  }
}

// Same walk, element-typed with a fused scale (bf16/fp16/fp32 -> same or fp32/bf16 dst):
// used to unflatten an all-reduced gradient bucket with the 1/world averaging applied.
template <int DTI, int DTO>
__global__ void __launch_bounds__(256) chunk_scale_kernel(const CopyChunk* __restrict__ table,
                                                          int64_t nchunks, float scale) {
  using TI = typename Elem<DTI>::T;
  using TO = typename Elem<DTO>::T;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const CopyChunk ch = table[c];
    const TI* s = reinterpret_cast<const TI*>(ch.src);
    TO* d = reinterpret_cast<TO*>(ch.dst);
    const int64_t n = static_cast<int64_t>(ch.nbytes / Elem<DTI>::kBytes);
    const bool vec = ((ch.src & 15) == 0) && ((ch.dst & (8 * Elem<DTO>::kBytes - 1)) == 0);
    int64_t done = 0;
    if (vec) {
      const int64_t nv = n / 8;
      for (int64_t i = threadIdx.x; i < nv; i += blockDim.x) {
        float v[8];
        load8<DTI>(s, i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= scale;
        store8<DTO>(d, i, v);
      }
      done = nv * 8;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += blockDim.x)
      Elem<DTO>::st(d, i, Elem<DTI>::ld(s, i) * scale);
  }
}

static int grid_for(int64_t nchunks) {
  int64_t g = nchunks < 1 ? 1 : nchunks;
  return static_cast<int>(g > 4096 ? 4096 : g);
}

}  // namespace dlbb

using namespace dlbb;

// table: DEVICE pointer to nchunks CopyChunk entries (3 x uint64 each).
// Destination stores: 0 plain, 1 non-temporal, 2 auto (default) = non-temporal once the copy's
// source + destination bytes exceed the 256 MiB MALL — measured (profiles/r05_kernels/
// memroof_pass1.jsonl): 8-way list unpack of 256 MiB 4.82 -> 6.12 TB/s with nt stores, 64 MiB
// (everything cache-resident) 4.89 plain vs 4.86 nt.
static int g_chunk_nt = 2;
constexpr int64_t kNtBytes = int64_t{256} << 20;

DLBB_API void dlbb_chunk_copy_set_nt(int nt) { g_chunk_nt = nt < 0 || nt > 2 ? 2 : nt; }

// total_bytes: bytes the table moves (0 = unknown: plain stores under auto)
DLBB_API int dlbb_chunk_copy2(const void* table, int64_t nchunks, int64_t total_bytes,
                              hipStream_t stream) {
  if (nchunks <= 0) return hipSuccess;
  const bool nt = g_chunk_nt == 1 || (g_chunk_nt == 2 && 2 * total_bytes > kNtBytes);
  if (nt)
    hipLaunchKernelGGL(chunk_copy_kernel<true>, dim3(grid_for(nchunks)), dim3(256), 0, stream,
                       static_cast<const CopyChunk*>(table), nchunks);
  else
    hipLaunchKernelGGL(chunk_copy_kernel<false>, dim3(grid_for(nchunks)), dim3(256), 0, stream,
                       static_cast<const CopyChunk*>(table), nchunks);
  return hipGetLastError();
}

DLBB_API int dlbb_chunk_copy(const void* table, int64_t nchunks, hipStream_t stream) {
  return dlbb_chunk_copy2(table, nchunks, 0, stream);
}

DLBB_API int dlbb_chunk_copy_scale(const void* table, int64_t nchunks, int dtype_in,
                                   int dtype_out, float scale, hipStream_t stream) {
  if (nchunks <= 0) return hipSuccess;
  const CopyChunk* t = static_cast<const CopyChunk*>(table);
  const dim3 g(grid_for(nchunks)), b(256);
#define CS(I, O)                                                                        \
  if (dtype_in == I && dtype_out == O) {                                               \
    hipLaunchKernelGGL((chunk_scale_kernel<I, O>), g, b, 0, stream, t, nchunks, scale); \
    return hipGetLastError();                                                          \
  }
  CS(DT_BF16, DT_BF16) CS(DT_BF16, DT_F32) CS(DT_F32, DT_F32) CS(DT_F32, DT_BF16)
  CS(DT_F16, DT_F16) CS(DT_F16, DT_F32)
#undef CS
  return hipErrorInvalidValue;
}
