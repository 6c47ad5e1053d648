// IPC one-shot / two-shot all-reduce over xGMI (single node, up to 8 GPUs).
//
// What it replaces: the reference's all-reduce paths are host collectives — mpi4py
// `comm.allreduce` / `comm.Allreduce` (collectives/1d/openmpi.py:63, models.py:95) and
// oneCCL/Gloo `dist.all_reduce` (collectives/1d/dsccl.py:65) with oneCCL's algorithm menu
// (direct / ring / 2d / ... selected by CCL_ALLREDUCE, collectives/3d/launch_dsccl.sh:46-47).
// On MI355X every GPU has a dedicated xGMI link to each of its 7 peers (fully connected), so a
// "direct" algorithm that reads all peers at once uses all 7 links concurrently, where a ring
// uses one. RCCL stays the default; this kernel is the low-latency / all-links path.
//
// Protocol (per call, per workgroup b; `e` = per-workgroup epoch counter kept in device memory,
// so the kernel is HIP-graph replayable):
//   one-shot : copy my input range b -> my IPC buffer[e&1] ; signal(phase 0, e) to all peers ;
//              wait all peers' phase-0 flag >= e ; out[b] = sum_p peer_buf[p][e&1][b]
//   two-shot : copy sub-range b of every shard -> buffer[e&1] ; signal/wait phase 0 ;
//              reduce sub-range b of MY shard from all peers -> my tmp[e&1] and out ;
//              signal/wait phase 1 ; gather sub-range b of every peer shard from peer tmp -> out
//   two-shot, registered (in place on a user buffer every rank IPC-mapped once with
//   dlbb_car_reg_open — no copy-in, no tmp): signal/wait phase 0 (inputs ready) ; reduce
//              sub-range b of MY shard from every rank's buffer into my buffer ; signal/wait
//              phase 1 ; gather sub-range b of every peer shard from its owner's buffer ;
//              signal/wait phase 2 (no peer still reads my buffer when my stream moves on)
// Epochs: every call advances the epoch of ALL kMaxBlocks workgroup slots by one (block 0 also
// bumps the slots beyond this call's grid), so the epoch - and with it the buffer half - is the
// same in every workgroup of a call even when consecutive calls use different grid sizes.
// Double buffering by epoch parity + the ">= e" wait makes one barrier per phase sufficient:
// a rank reaches epoch e+2 (and overwrites buffer[e&1]) only after every peer signalled e+1,
// i.e. finished reading epoch e.
// Memory ordering (CDNA guide §6 G16, system scope because readers are other GPUs): payload
// plain stores -> each wave `s_waitcnt vmcnt(0)` -> barrier -> one lane per peer:
// release fence (buffer_wbl2 sc0 sc1) -> `s_waitcnt vmcnt(0)` (ROCm 7.2 pitfall 12) -> relaxed
// system-scope flag store into the peer's uncached signal page. Consumer: relaxed system-scope
// poll (sc0 sc1, bypasses caches) with s_sleep, ONE acquire fence (buffer_inv sc0 sc1), barrier,
// then plain loads of peer memory. Every spin is bounded: on timeout the kernel records an error
// code and exits, so a broken peer cannot hang the GPU.
#include "common.h"

#include <string.h>

#include <new>
#include <vector>

namespace dlbb {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;
constexpr int kCarThreads = 512;
constexpr unsigned kSpinLimit = 1u << 26;   // ~ seconds of polling, then give up
constexpr uint32_t kMagic = 0xD1BB0000u;

struct Signal {
  uint32_t flags[3][kMaxBlocks][kMaxRanks];   // written by peers (remote stores)
  uint32_t epoch[kMaxBlocks];                 // local per-workgroup call counter
  uint32_t error;                             // nonzero: a wait timed out
  uint32_t pad[3];
};

struct CarKernelArgs {
  char* data[kMaxRanks];        // each rank's IPC data region: 2 x cap bytes
  char* tmp[kMaxRanks];         // each rank's IPC tmp region (two-shot): 2 x cap bytes
  Signal* sig[kMaxRanks];
  const void* inp;
  void* out;
  int64_t nbytes;               // message bytes, multiple of 16 * world (two-shot) / 16
  int64_t cap;                  // capacity per buffer half
  int rank;
  int world;
};

__device__ __forceinline__ void signal_peers(const CarKernelArgs& a, int phase, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(a.world)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&a.sig[threadIdx.x]->flags[phase][blockIdx.x][a.rank], e,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ bool wait_peers(const CarKernelArgs& a, int phase, uint32_t e) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(a.world)) {
    uint32_t* f = &a.sig[a.rank]->flags[phase][blockIdx.x][threadIdx.x];
    unsigned spins = 0;
    while (static_cast<int32_t>(
               __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        timed_out = 1;
        __hip_atomic_store(&a.sig[a.rank]->error, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return timed_out == 0;
}

// Advance this call's epoch (see header): each workgroup bumps its own slot, block 0 also the
// slots no workgroup of this grid owns. Returns the epoch of the calling workgroup.
__device__ __forceinline__ uint32_t begin_epoch(const CarKernelArgs& a) {
  __shared__ uint32_t s_epoch;
  Signal* s = a.sig[a.rank];
  if (threadIdx.x == 0) s_epoch = ++s->epoch[blockIdx.x];
  if (blockIdx.x == 0)
    for (unsigned b = gridDim.x + threadIdx.x; b < static_cast<unsigned>(kMaxBlocks);
         b += blockDim.x)
      ++s->epoch[b];
  __syncthreads();
  return s_epoch;
}

// W = world size as a compile-time constant (2, 4, 8: every peer load issued before the adds,
// fully unrolled) or 0 (runtime world). Peer pointers come straight from the kernel-argument
// block with wave-uniform indices (scalar loads), never from a runtime-indexed local array.
template <int DT, int W>
__device__ __forceinline__ void sum_vec(const CarKernelArgs& a, int64_t half, int64_t off,
                                        float (&acc)[8]) {
  if constexpr (W > 0) {
    float v[W][8];
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int p = (a.rank + k) & (W - 1);   // rotate so ranks start on different links
      load8<DT>(a.data[p] + half + off, 0, v[k]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = v[0][j];
#pragma unroll
    for (int k = 1; k < W; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[k][j];
  } else {
    load8<DT>(a.data[a.rank] + half + off, 0, acc);
    for (int k = 1; k < a.world; ++k) {
      const int p = (a.rank + k) % a.world;
      float v[8];
      load8<DT>(a.data[p] + half + off, 0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
}

template <int DT, int W>
__global__ void __launch_bounds__(kCarThreads) car_oneshot_kernel(CarKernelArgs a) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  const uint32_t e = begin_epoch(a);
  const int64_t half = (e & 1) * a.cap;
  const int64_t nvec = a.nbytes / kVecBytes;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = blockIdx.x * per;
  const int64_t v1 = v0 + per < nvec ? v0 + per : nvec;
  char* mine = a.data[a.rank] + half;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
#pragma unroll
    for (int q = 0; q < kVecBytes / 16; ++q)
      reinterpret_cast<u16x8*>(mine + v * kVecBytes)[q] =
          reinterpret_cast<const u16x8*>(static_cast<const char*>(a.inp) + v * kVecBytes)[q];
  }
  signal_peers(a, 0, e);
  if (!wait_peers(a, 0, e)) return;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, half, v * kVecBytes, acc);
    store8<DT>(a.out, v, acc);
  }
}

template <int DT, int W>
__global__ void __launch_bounds__(kCarThreads) car_twoshot_kernel(CarKernelArgs a) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  const uint32_t e = begin_epoch(a);
  const int64_t half = (e & 1) * a.cap;
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;      // vectors per shard
  const int64_t per = (shard_vec + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = blockIdx.x * per;
  const int64_t s1 = s0 + per < shard_vec ? s0 + per : shard_vec;
  char* mine = a.data[a.rank] + half;
  constexpr int kQ = kVecBytes / 16;
  // publish sub-range [s0, s1) of every shard (W > 0: all W loads in flight per thread)
  if constexpr (W > 0) {
    for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
      u16x8 t[W][kQ];
#pragma unroll
      for (int p = 0; p < W; ++p)
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          t[p][q] = reinterpret_cast<const u16x8*>(
              static_cast<const char*>(a.inp) + (p * shard_vec + v) * kVecBytes)[q];
#pragma unroll
      for (int p = 0; p < W; ++p)
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(mine + (p * shard_vec + v) * kVecBytes)[q] = t[p][q];
    }
  } else {
    for (int p = 0; p < a.world; ++p) {
      const int64_t base = p * shard_vec;
      for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
        const int64_t off = (base + v) * kVecBytes;
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(mine + off)[q] =
              reinterpret_cast<const u16x8*>(static_cast<const char*>(a.inp) + off)[q];
      }
    }
  }
  signal_peers(a, 0, e);
  if (!wait_peers(a, 0, e)) return;
  // reduce-scatter: my shard, sub-range b
  char* my_tmp = a.tmp[a.rank] + half;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, half, (mybase + v) * kVecBytes, acc);
    store8<DT>(my_tmp, mybase + v, acc);
    store8<DT>(a.out, mybase + v, acc);
  }
  signal_peers(a, 1, e);
  if (!wait_peers(a, 1, e)) return;
  // all-gather: every other shard's sub-range b from its owner's tmp. W > 0: the W-1 remote
  // loads of a thread are all in flight before its stores (one per xGMI link), instead of one
  // peer at a time.
  if constexpr (W > 0) {
    for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
      u16x8 t[W - 1][kQ];
#pragma unroll
      for (int k = 1; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          t[k - 1][q] = reinterpret_cast<const u16x8*>(a.tmp[p] + half +
                                                       (p * shard_vec + v) * kVecBytes)[q];
      }
#pragma unroll
      for (int k = 1; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(static_cast<char*>(a.out) +
                                   (p * shard_vec + v) * kVecBytes)[q] = t[k - 1][q];
      }
    }
  } else {
    for (int k = 1; k < a.world; ++k) {
      const int p = (a.rank + k) % a.world;
      const char* src = a.tmp[p] + half;
      const int64_t base = p * shard_vec;
      for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
        const int64_t off = (base + v) * kVecBytes;
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(static_cast<char*>(a.out) + off)[q] =
              reinterpret_cast<const u16x8*>(src + off)[q];
      }
    }
  }
}

// Registered two-shot, in place (see header). a.data[p] = rank p's registered buffer (no halves).
// Disjointness: in phase 1 a rank writes only shard `rank` of its own buffer, which peers do not
// read in phase 1 (peer q reads shard q); in phase 2 it writes shards p != rank of its own buffer,
// and peers only read shard `rank` of it. Workgroup b of every rank owns sub-range b of every
// shard, so the per-workgroup flags order exactly the producer/consumer pairs.
template <int DT, int W>
__global__ void __launch_bounds__(kCarThreads) car_twoshot_reg_kernel(CarKernelArgs a) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  constexpr int kQ = kVecBytes / 16;
  const uint32_t e = begin_epoch(a);
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  const int64_t per = (shard_vec + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = blockIdx.x * per;
  const int64_t s1 = s0 + per < shard_vec ? s0 + per : shard_vec;
  char* mine = a.data[a.rank];
  signal_peers(a, 0, e);                       // my input is complete (stream order)
  if (!wait_peers(a, 0, e)) return;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, 0, (mybase + v) * kVecBytes, acc);
    store8<DT>(mine, mybase + v, acc);
  }
  signal_peers(a, 1, e);
  if (!wait_peers(a, 1, e)) return;
  if constexpr (W > 0) {
    for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
      u16x8 t[W - 1][kQ];
#pragma unroll
      for (int k = 1; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          t[k - 1][q] = reinterpret_cast<const u16x8*>(a.data[p] +
                                                       (p * shard_vec + v) * kVecBytes)[q];
      }
#pragma unroll
      for (int k = 1; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(mine + (p * shard_vec + v) * kVecBytes)[q] = t[k - 1][q];
      }
    }
  } else {
    for (int k = 1; k < a.world; ++k) {
      const int p = (a.rank + k) % a.world;
      for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
        const int64_t off = (p * shard_vec + v) * kVecBytes;
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(mine + off)[q] =
              reinterpret_cast<const u16x8*>(a.data[p] + off)[q];
      }
    }
  }
  signal_peers(a, 2, e);                       // done reading every peer's buffer
  wait_peers(a, 2, e);
}

// Registered two-shot, PUSH form (in place): the same traffic per link as the pull form, but
// every byte crosses xGMI as a posted remote WRITE instead of a read round trip.
//   reduce-scatter push: shard p of my buffer -> slot `rank` of rank p's staging half (tmp[e&1])
//   flag barrier 0 ; reduce the world slots of my staging half (local reads) and push the result
//   into shard `rank` of every rank's buffer (mine included) ; flag barrier 1 (my buffer is
//   complete once every peer's pushes into it have landed).
// Staging halves alternate by epoch parity: a rank writes half e&1 of a peer in call e only
// after passing barrier 1 of call e-1, i.e. after that peer finished reducing call e-2's half.
// Requires nbytes <= cap (world slots of nbytes / world each).
template <int DT, int W>
__global__ void __launch_bounds__(kCarThreads) car_twoshot_push_kernel(CarKernelArgs a) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  constexpr int kQ = kVecBytes / 16;
  const uint32_t e = begin_epoch(a);
  const int64_t half = (e & 1) * a.cap;
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  const int64_t shard_bytes = shard_vec * kVecBytes;
  const int64_t per = (shard_vec + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = blockIdx.x * per;
  const int64_t s1 = s0 + per < shard_vec ? s0 + per : shard_vec;
  const char* mine = a.data[a.rank];
  const int64_t my_slot = half + a.rank * shard_bytes;
  if constexpr (W > 0) {
    for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
      u16x8 t[W][kQ];
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          t[k][q] = reinterpret_cast<const u16x8*>(mine + (p * shard_vec + v) * kVecBytes)[q];
      }
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(a.tmp[p] + my_slot + v * kVecBytes)[q] = t[k][q];
      }
    }
  } else {
    for (int k = 0; k < a.world; ++k) {
      const int p = (a.rank + k) % a.world;
      for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x)
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          reinterpret_cast<u16x8*>(a.tmp[p] + my_slot + v * kVecBytes)[q] =
              reinterpret_cast<const u16x8*>(mine + (p * shard_vec + v) * kVecBytes)[q];
    }
  }
  signal_peers(a, 0, e);
  if (!wait_peers(a, 0, e)) return;
  const char* stage = a.tmp[a.rank] + half;
  const int64_t out_off = a.rank * shard_bytes;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    load8<DT>(stage, v, acc);
    if constexpr (W > 0) {
      float x[W - 1][8];
#pragma unroll
      for (int k = 1; k < W; ++k) load8<DT>(stage + k * shard_bytes, v, x[k - 1]);
#pragma unroll
      for (int k = 1; k < W; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[k - 1][j];
    } else {
      for (int k = 1; k < a.world; ++k) {
        float x[8];
        load8<DT>(stage + k * shard_bytes, v, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      }
    }
    if constexpr (W > 0) {
#pragma unroll
      for (int k = 0; k < W; ++k)
        store8<DT>(a.data[(a.rank + k) & (W - 1)] + out_off, v, acc);
    } else {
      for (int k = 0; k < a.world; ++k)
        store8<DT>(a.data[(a.rank + k) % a.world] + out_off, v, acc);
    }
  }
  signal_peers(a, 1, e);
  wait_peers(a, 1, e);
}

// ---- direct (one-hop) collectives on registered inputs --------------------------------------
// Every GPU reads its peers' registered input buffers over its own xGMI link to each of them, so
// all 7 links of a GPU carry traffic at once (an RCCL ring uses one link in and one out per
// channel). Entry barrier: every rank's input is complete; exit barrier: no peer still reads my
// input when my stream moves on (the caller may overwrite it). Workgroup b moves sub-range b of
// every peer's chunk with the loads from all peers in flight together.
//   all-gather : out[p * chunk .. ] = in_p[0 .. chunk)
//   all-to-all : out[p * chunk .. ] = in_p[rank * chunk .. ]   (equal splits)
template <int W, bool A2A>
__global__ void __launch_bounds__(kCarThreads) car_pull_kernel(CarKernelArgs a) {
  const uint32_t e = begin_epoch(a);
  const int64_t chunk = a.nbytes;                    // bytes per peer chunk, multiple of 16
  const int64_t nvec = chunk / 16;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = blockIdx.x * per;
  const int64_t v1 = v0 + per < nvec ? v0 + per : nvec;
  const int64_t src_off = A2A ? a.rank * chunk : 0;
  char* out = static_cast<char*>(a.out);
  signal_peers(a, 0, e);
  if (!wait_peers(a, 0, e)) return;
  if constexpr (W > 0) {
    for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      u16x8 t[W];
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
        t[k] = reinterpret_cast<const u16x8*>(a.data[p] + src_off)[v];
      }
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int p = (a.rank + k) & (W - 1);
        reinterpret_cast<u16x8*>(out + p * chunk)[v] = t[k];
      }
    }
  } else {
    for (int k = 0; k < a.world; ++k) {
      const int p = (a.rank + k) % a.world;
      for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x)
        reinterpret_cast<u16x8*>(out + p * chunk)[v] =
            reinterpret_cast<const u16x8*>(a.data[p] + src_off)[v];
    }
  }
  signal_peers(a, 2, e);
  wait_peers(a, 2, e);
}

//   reduce-scatter : out[0 .. n/P) = sum_p in_p[rank * n/P .. ]   (fp32 accumulation)
template <int DT, int W>
__global__ void __launch_bounds__(kCarThreads) car_rs_kernel(CarKernelArgs a) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  const uint32_t e = begin_epoch(a);
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  const int64_t per = (shard_vec + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = blockIdx.x * per;
  const int64_t s1 = s0 + per < shard_vec ? s0 + per : shard_vec;
  signal_peers(a, 0, e);
  if (!wait_peers(a, 0, e)) return;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, 0, (mybase + v) * kVecBytes, acc);
    store8<DT>(a.out, v, acc);
  }
  signal_peers(a, 2, e);
  wait_peers(a, 2, e);
}

template <int W>
void launch_direct(int kind, int dtype, dim3 g, dim3 b, hipStream_t st, const CarKernelArgs& a) {
  if (kind == 0) hipLaunchKernelGGL((car_pull_kernel<W, false>), g, b, 0, st, a);
  else if (kind == 1) hipLaunchKernelGGL((car_pull_kernel<W, true>), g, b, 0, st, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL((car_rs_kernel<DT_BF16, W>), g, b, 0, st, a);
  else if (dtype == DT_F16) hipLaunchKernelGGL((car_rs_kernel<DT_F16, W>), g, b, 0, st, a);
  else hipLaunchKernelGGL((car_rs_kernel<DT_F32, W>), g, b, 0, st, a);
}

template <int DT>
void launch_push(int w, dim3 g, dim3 b, hipStream_t st, const CarKernelArgs& a) {
  if (w == 2) hipLaunchKernelGGL((car_twoshot_push_kernel<DT, 2>), g, b, 0, st, a);
  else if (w == 4) hipLaunchKernelGGL((car_twoshot_push_kernel<DT, 4>), g, b, 0, st, a);
  else if (w == 8) hipLaunchKernelGGL((car_twoshot_push_kernel<DT, 8>), g, b, 0, st, a);
  else hipLaunchKernelGGL((car_twoshot_push_kernel<DT, 0>), g, b, 0, st, a);
}

struct RegBuf {
  char* ptr[kMaxRanks] = {};    // every rank's registered buffer (mine at [rank])
  int64_t bytes = 0;
};

struct OpenedMap {               // one hipIpcOpenMemHandle per (peer, allocation)
  int peer;
  hipIpcMemHandle_t handle;
  char* base;
};

struct CarState {
  int rank = 0, world = 1, device = 0;
  int64_t cap = 0;
  char* data = nullptr;       // 2 * cap (coarse-grained, IPC)
  char* tmp = nullptr;        // 2 * cap
  Signal* sig = nullptr;      // uncached, IPC
  bool opened = false;
  CarKernelArgs args{};
  char* peer_data[kMaxRanks] = {};
  char* peer_tmp[kMaxRanks] = {};
  Signal* peer_sig[kMaxRanks] = {};
  std::vector<RegBuf> regs;
  std::vector<OpenedMap> opened_maps;
};

}  // namespace dlbb

using namespace dlbb;

#define CAR_CHECK(x)                         \
  do {                                       \
    hipError_t _e = (x);                     \
    if (_e != hipSuccess) return (int)_e;    \
  } while (0)

DLBB_API int dlbb_car_create(int rank, int world, int64_t cap_bytes, void** out) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || cap_bytes <= 0)
    return hipErrorInvalidValue;
  cap_bytes = (cap_bytes + 255) / 256 * 256;
  CarState* s = new (std::nothrow) CarState();
  if (!s) return hipErrorOutOfMemory;
  s->rank = rank;
  s->world = world;
  s->cap = cap_bytes;
  hipError_t e = hipGetDevice(&s->device);   // (no early return: s must not leak)
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->data), 2 * cap_bytes);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->tmp), 2 * cap_bytes);
  if (e == hipSuccess)
    e = hipExtMallocWithFlags(reinterpret_cast<void**>(&s->sig), sizeof(Signal),
                              hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(s->sig, 0, sizeof(Signal));
  if (e == hipSuccess) {
    // magic word identifying this rank's signal page: peers verify their IPC mapping with a
    // copy-engine read before any kernel touches it (a bad mapping must not fault a kernel)
    const uint32_t magic = kMagic | static_cast<uint32_t>(rank);
    e = hipMemcpy(&s->sig->pad[0], &magic, sizeof(magic), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (s->data) (void)hipFree(s->data);
    if (s->tmp) (void)hipFree(s->tmp);
    if (s->sig) (void)hipFree(s->sig);
    delete s;
    return (int)e;
  }
  *out = s;
  return hipSuccess;
}

// Writes 3 x 64-byte IPC handles (data, tmp, signal) into out_handles (192 bytes).
DLBB_API int dlbb_car_ipc_handles(void* h, void* out_handles) {
  CarState* s = static_cast<CarState*>(h);
  hipIpcMemHandle_t hd, ht, hs;
  CAR_CHECK(hipIpcGetMemHandle(&hd, s->data));
  CAR_CHECK(hipIpcGetMemHandle(&ht, s->tmp));
  CAR_CHECK(hipIpcGetMemHandle(&hs, s->sig));
  char* o = static_cast<char*>(out_handles);
  memcpy(o, &hd, 64);
  memcpy(o + 64, &ht, 64);
  memcpy(o + 128, &hs, 64);
  return hipSuccess;
}

DLBB_API int dlbb_car_handle_bytes() { return 3 * 64; }

// all_handles: world x 192 bytes in rank order; peer_devices: each rank's device ordinal
// (used to decide whether peer access must be enabled; same device -> plain IPC mapping).
DLBB_API int dlbb_car_open(void* h, const void* all_handles, const int* peer_devices) {
  CarState* s = static_cast<CarState*>(h);
  if (s->opened) return hipSuccess;
  const char* hs = static_cast<const char*>(all_handles);
  for (int p = 0; p < s->world; ++p) {
    if (p == s->rank) {
      s->peer_data[p] = s->data;
      s->peer_tmp[p] = s->tmp;
      s->peer_sig[p] = s->sig;
      continue;
    }
    if (peer_devices && peer_devices[p] != s->device) {
      int can = 0;
      CAR_CHECK(hipDeviceCanAccessPeer(&can, s->device, peer_devices[p]));
      if (!can) return hipErrorPeerAccessUnsupported;
      hipError_t e = hipDeviceEnablePeerAccess(peer_devices[p], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return (int)e;
      (void)hipGetLastError();
    }
    hipIpcMemHandle_t hd, ht, hsg;
    memcpy(&hd, hs + p * 192, 64);
    memcpy(&ht, hs + p * 192 + 64, 64);
    memcpy(&hsg, hs + p * 192 + 128, 64);
    void *pd = nullptr, *pt = nullptr, *ps = nullptr;
    CAR_CHECK(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess));
    CAR_CHECK(hipIpcOpenMemHandle(&pt, ht, hipIpcMemLazyEnablePeerAccess));
    CAR_CHECK(hipIpcOpenMemHandle(&ps, hsg, hipIpcMemLazyEnablePeerAccess));
    s->peer_data[p] = static_cast<char*>(pd);
    s->peer_tmp[p] = static_cast<char*>(pt);
    s->peer_sig[p] = static_cast<Signal*>(ps);
    uint32_t magic = 0;
    CAR_CHECK(hipMemcpy(&magic, &s->peer_sig[p]->pad[0], sizeof(magic), hipMemcpyDeviceToHost));
    if (magic != (kMagic | static_cast<uint32_t>(p))) return hipErrorInvalidHandle;
  }
  for (int p = 0; p < kMaxRanks; ++p) {
    s->args.data[p] = s->peer_data[p];
    s->args.tmp[p] = s->peer_tmp[p];
    s->args.sig[p] = s->peer_sig[p];
  }
  s->args.rank = s->rank;
  s->args.world = s->world;
  s->args.cap = s->cap;
  s->opened = true;
  return hipSuccess;
}

DLBB_API int64_t dlbb_car_capacity(void* h) { return static_cast<CarState*>(h)->cap; }

// algo: 1 = one-shot, 2 = two-shot. nblocks <= 128. dtype: bf16 | f16 | f32.
// Requirements (checked): nbytes <= cap; nbytes % 16 == 0 (one-shot) or
// nbytes % (vec_bytes * world) == 0 (two-shot).
DLBB_API int dlbb_car_allreduce(void* h, const void* inp, void* out, int64_t n, int dtype,
                                int algo, int nblocks, hipStream_t stream) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened) return hipErrorNotInitialized;
  const int64_t esz = dtype == DT_F32 ? 4 : 2;
  const int64_t vec = 8 * esz;
  const int64_t nbytes = n * esz;
  if (nbytes <= 0) return hipSuccess;
  if (nbytes > s->cap || nbytes % vec != 0) return hipErrorInvalidValue;
  if (algo == 2 && nbytes % (vec * s->world) != 0) return hipErrorInvalidValue;
  if (nblocks < 1) nblocks = 1;
  if (nblocks > kMaxBlocks) nblocks = kMaxBlocks;
  if (s->world == 1) {
    if (out != inp) CAR_CHECK(hipMemcpyAsync(out, inp, nbytes, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }
  CarKernelArgs a = s->args;
  a.inp = inp;
  a.out = out;
  a.nbytes = nbytes;
  const dim3 g(nblocks), b(kCarThreads);
#define CAR_W(KERN, D)                                                                  \
  do {                                                                                  \
    if (s->world == 2) hipLaunchKernelGGL((KERN<D, 2>), g, b, 0, stream, a);            \
    else if (s->world == 4) hipLaunchKernelGGL((KERN<D, 4>), g, b, 0, stream, a);       \
    else if (s->world == 8) hipLaunchKernelGGL((KERN<D, 8>), g, b, 0, stream, a);       \
    else hipLaunchKernelGGL((KERN<D, 0>), g, b, 0, stream, a);                          \
  } while (0)
#define CAR_L(KERN, D) CAR_W(KERN, D)
  if (algo == 2) {
    if (dtype == DT_BF16) CAR_L(car_twoshot_kernel, DT_BF16);
    else if (dtype == DT_F16) CAR_L(car_twoshot_kernel, DT_F16);
    else CAR_L(car_twoshot_kernel, DT_F32);
  } else {
    if (dtype == DT_BF16) CAR_L(car_oneshot_kernel, DT_BF16);
    else if (dtype == DT_F16) CAR_L(car_oneshot_kernel, DT_F16);
    else CAR_L(car_oneshot_kernel, DT_F32);
  }
#undef CAR_W
#undef CAR_L
  return hipGetLastError();
}

// ---- registered buffers -----------------------------------------------------------------------
// Export the IPC handle of the allocation that contains `ptr` (e.g. a torch caching-allocator
// segment) and ptr's offset in it.
DLBB_API int dlbb_car_reg_export(void* h, const void* ptr, void* out_handle, int64_t* out_offset) {
  (void)h;
  void* base = nullptr;
  size_t size = 0;
  CAR_CHECK(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
  hipIpcMemHandle_t hd;
  CAR_CHECK(hipIpcGetMemHandle(&hd, base));
  memcpy(out_handle, &hd, 64);
  *out_offset = static_cast<const char*>(ptr) - static_cast<char*>(base);
  return hipSuccess;
}

// Map every peer's exported buffer (all_handles: world x 64 bytes, offsets: world) and record
// the registration; *out_id indexes it for dlbb_car_allreduce_reg. A peer allocation already
// mapped by an earlier registration is reused (one open per allocation and peer).
DLBB_API int dlbb_car_reg_open(void* h, const void* ptr, int64_t nbytes, const void* all_handles,
                               const int64_t* offsets, int* out_id) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened) return hipErrorNotInitialized;
  RegBuf r;
  r.bytes = nbytes;
  const char* hs = static_cast<const char*>(all_handles);
  for (int p = 0; p < s->world; ++p) {
    if (p == s->rank) {
      r.ptr[p] = static_cast<char*>(const_cast<void*>(ptr));
      continue;
    }
    hipIpcMemHandle_t hd;
    memcpy(&hd, hs + p * 64, 64);
    char* base = nullptr;
    for (const OpenedMap& m : s->opened_maps)
      if (m.peer == p && memcmp(&m.handle, &hd, sizeof(hd)) == 0) base = m.base;
    if (!base) {
      void* pd = nullptr;
      CAR_CHECK(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess));
      base = static_cast<char*>(pd);
      s->opened_maps.push_back(OpenedMap{p, hd, base});
    }
    r.ptr[p] = base + offsets[p];
    // copy-engine read of the first and last byte: a bad mapping fails here, not in a kernel
    char probe[2];
    CAR_CHECK(hipMemcpy(&probe[0], r.ptr[p], 1, hipMemcpyDeviceToHost));
    CAR_CHECK(hipMemcpy(&probe[1], r.ptr[p] + nbytes - 1, 1, hipMemcpyDeviceToHost));
  }
  s->regs.push_back(r);
  *out_id = static_cast<int>(s->regs.size()) - 1;
  return hipSuccess;
}

// In-place all-reduce of registration `id` (n elements from its start; n * esize must be a
// multiple of 16 * world and at most the registered size).
DLBB_API int dlbb_car_allreduce_reg(void* h, int id, int64_t n, int dtype, int nblocks,
                                    hipStream_t stream) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened || id < 0 || id >= static_cast<int>(s->regs.size())) return hipErrorInvalidValue;
  const RegBuf& r = s->regs[id];
  const int64_t esz = dtype == DT_F32 ? 4 : 2;
  const int64_t nbytes = n * esz;
  if (nbytes <= 0) return hipSuccess;
  if (nbytes > r.bytes || nbytes % (8 * esz * s->world) != 0) return hipErrorInvalidValue;
  if (s->world == 1) return hipSuccess;
  if (nblocks < 1) nblocks = 1;
  if (nblocks > kMaxBlocks) nblocks = kMaxBlocks;
  CarKernelArgs a = s->args;
  for (int p = 0; p < kMaxRanks; ++p) a.data[p] = r.ptr[p];
  a.inp = r.ptr[s->rank];
  a.out = r.ptr[s->rank];
  a.nbytes = nbytes;
  const dim3 g(nblocks), b(kCarThreads);
#define CAR_RW(D)                                                                            \
  do {                                                                                       \
    if (s->world == 2) hipLaunchKernelGGL((car_twoshot_reg_kernel<D, 2>), g, b, 0, stream, a); \
    else if (s->world == 4) hipLaunchKernelGGL((car_twoshot_reg_kernel<D, 4>), g, b, 0, stream, a); \
    else if (s->world == 8) hipLaunchKernelGGL((car_twoshot_reg_kernel<D, 8>), g, b, 0, stream, a); \
    else hipLaunchKernelGGL((car_twoshot_reg_kernel<D, 0>), g, b, 0, stream, a);            \
  } while (0)
  if (dtype == DT_BF16) CAR_RW(DT_BF16);
  else if (dtype == DT_F16) CAR_RW(DT_F16);
  else CAR_RW(DT_F32);
#undef CAR_RW
  return hipGetLastError();
}

// Push form of the registered two-shot (see car_twoshot_push_kernel); nbytes <= capacity.
DLBB_API int dlbb_car_allreduce_reg_push(void* h, int id, int64_t n, int dtype, int nblocks,
                                         hipStream_t stream) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened || id < 0 || id >= static_cast<int>(s->regs.size())) return hipErrorInvalidValue;
  const RegBuf& r = s->regs[id];
  const int64_t esz = dtype == DT_F32 ? 4 : 2;
  const int64_t nbytes = n * esz;
  if (nbytes <= 0) return hipSuccess;
  if (nbytes > r.bytes || nbytes > s->cap || nbytes % (8 * esz * s->world) != 0)
    return hipErrorInvalidValue;
  if (s->world == 1) return hipSuccess;
  if (nblocks < 1) nblocks = 1;
  if (nblocks > kMaxBlocks) nblocks = kMaxBlocks;
  CarKernelArgs a = s->args;               // tmp[] = every rank's staging region
  for (int p = 0; p < kMaxRanks; ++p) a.data[p] = r.ptr[p];
  a.inp = r.ptr[s->rank];
  a.out = r.ptr[s->rank];
  a.nbytes = nbytes;
  const dim3 g(nblocks), b(kCarThreads);
  const int w = s->world == 2 || s->world == 4 || s->world == 8 ? s->world : 0;
  if (dtype == DT_BF16) launch_push<DT_BF16>(w, g, b, stream, a);
  else if (dtype == DT_F16) launch_push<DT_F16>(w, g, b, stream, a);
  else launch_push<DT_F32>(w, g, b, stream, a);
  return hipGetLastError();
}

// Direct collectives on registration `id` (this rank's registered input; out is local).
//   kind 0 = all-gather  : bytes = chunk bytes per rank (<= registered), out = world x chunk
//   kind 1 = all-to-all  : bytes = chunk bytes per peer (world x chunk <= registered)
//   kind 2 = reduce-scatter (dtype): bytes = whole input (multiple of 16 x world), out = bytes/world
DLBB_API int dlbb_car_direct_reg(void* h, int id, int kind, int64_t bytes, int dtype, void* out,
                                 int nblocks, hipStream_t stream) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened || id < 0 || id >= static_cast<int>(s->regs.size()) || !out)
    return hipErrorInvalidValue;
  const RegBuf& r = s->regs[id];
  if (bytes <= 0) return hipSuccess;
  if (kind == 0 && (bytes % 16 || bytes > r.bytes)) return hipErrorInvalidValue;
  if (kind == 1 && (bytes % 16 || bytes * s->world > r.bytes)) return hipErrorInvalidValue;
  if (kind == 2 && (bytes % (16 * s->world) || bytes > r.bytes)) return hipErrorInvalidValue;
  if (kind < 0 || kind > 2) return hipErrorInvalidValue;
  if (nblocks < 1) nblocks = 1;
  if (nblocks > kMaxBlocks) nblocks = kMaxBlocks;
  CarKernelArgs a = s->args;
  for (int p = 0; p < kMaxRanks; ++p) a.data[p] = r.ptr[p];
  a.inp = r.ptr[s->rank];
  a.out = out;
  a.nbytes = bytes;
  const dim3 g(nblocks), b(kCarThreads);
  const int w = s->world == 2 || s->world == 4 || s->world == 8 ? s->world : 0;
  if (w == 2) launch_direct<2>(kind, dtype, g, b, stream, a);
  else if (w == 4) launch_direct<4>(kind, dtype, g, b, stream, a);
  else if (w == 8) launch_direct<8>(kind, dtype, g, b, stream, a);
  else launch_direct<0>(kind, dtype, g, b, stream, a);
  return hipGetLastError();
}

// Reads (and clears) the device-side timeout flag. Synchronous: call outside timed regions.
DLBB_API int dlbb_car_error(void* h) {
  CarState* s = static_cast<CarState*>(h);
  uint32_t err = 0;
  CAR_CHECK(hipMemcpy(&err, &s->sig->error, sizeof(err), hipMemcpyDeviceToHost));
  if (err) {
    const uint32_t z = 0;
    CAR_CHECK(hipMemcpy(&s->sig->error, &z, sizeof(z), hipMemcpyHostToDevice));
  }
  return static_cast<int>(err);
}

DLBB_API int dlbb_car_destroy(void* h) {
  CarState* s = static_cast<CarState*>(h);
  if (!s) return hipSuccess;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < s->world; ++p) {
    if (p == s->rank || !s->opened) continue;
    if (s->peer_data[p]) (void)hipIpcCloseMemHandle(s->peer_data[p]);
    if (s->peer_tmp[p]) (void)hipIpcCloseMemHandle(s->peer_tmp[p]);
    if (s->peer_sig[p]) (void)hipIpcCloseMemHandle(s->peer_sig[p]);
  }
  for (const OpenedMap& m : s->opened_maps) (void)hipIpcCloseMemHandle(m.base);
  (void)hipFree(s->data);
  (void)hipFree(s->tmp);
  (void)hipFree(s->sig);
  delete s;
  return hipSuccess;
}
