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
// Every wait is bounded in WALL time (s_memrealtime, the 100 MHz constant clock), not in polls:
// a poll of a peer's flag over xGMI costs ~1 us, so a poll count would stretch to a minute.
constexpr uint64_t kRealtimeHz = 100000000ull;
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
  uint64_t timeout_ticks;       // wait bound, s_memrealtime ticks (dlbb_car_set_timeout_ms)
  // uneven all-to-all (K_A2AV, MoE dispatch): bytes this rank pulls from peer p, at v_src[p] in
  // p's registered input, landing at v_dst[p] in out (all multiples of 16)
  int64_t v_src[kMaxRanks];
  int64_t v_cnt[kMaxRanks];
  int64_t v_dst[kMaxRanks];
};

// Every kernel body takes its workgroup index `bid` and workgroup count `nb` explicitly instead of
// reading blockIdx / gridDim, so the same device code runs in two launch forms:
//   * per rank (production): one grid of nb workgroups per GPU, bid = blockIdx.x;
//   * virtual ranks (single-GPU harness, dlbb_car_vr_launch): ONE grid of world x nb workgroups
//     on one GPU, workgroup g plays rank g / nb with bid = g % nb against the sibling ranks'
//     buffers in the same HBM. Same loads, stores, flags and fences as production; only the
//     transport differs (local HBM instead of xGMI).
__device__ __forceinline__ void signal_peers(const CarKernelArgs& a, int phase, uint32_t e,
                                             unsigned bid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(a.world)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&a.sig[threadIdx.x]->flags[phase][bid][a.rank], e,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ bool wait_peers(const CarKernelArgs& a, int phase, uint32_t e,
                                           unsigned bid) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(a.world)) {
    uint32_t* f = &a.sig[a.rank]->flags[phase][bid][threadIdx.x];
    // fail fast: after one timed-out wait on this rank the instance is dead (raise_if_error
    // raises on every rank); later calls skip their waits instead of each waiting out the bound
    if (__hip_atomic_load(&a.sig[a.rank]->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
      timed_out = 1;
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      unsigned spins = 0;
      while (static_cast<int32_t>(
                 __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if ((++spins & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
          timed_out = 1;
          __hip_atomic_store(&a.sig[a.rank]->error, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return timed_out == 0;
}

// Advance this call's epoch (see header): each workgroup bumps its own slot, workgroup 0 also the
// slots no workgroup of this call owns. Returns the epoch of the calling workgroup.
__device__ __forceinline__ uint32_t begin_epoch(const CarKernelArgs& a, unsigned bid,
                                                unsigned nb) {
  __shared__ uint32_t s_epoch;
  Signal* s = a.sig[a.rank];
  if (threadIdx.x == 0) s_epoch = ++s->epoch[bid];
  if (bid == 0)
    for (unsigned b = nb + threadIdx.x; b < static_cast<unsigned>(kMaxBlocks); b += blockDim.x)
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

// Sub-range [r0, r1) of n items owned by workgroup bid of nb.
__device__ __forceinline__ void split_range(int64_t n, unsigned bid, unsigned nb, int64_t& r0,
                                            int64_t& r1) {
  const int64_t per = (n + nb - 1) / nb;
  r0 = bid * per;
  r1 = r0 + per < n ? r0 + per : n;
}

template <int DT, int W>
__device__ __forceinline__ void oneshot_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  constexpr int kQ = kVecBytes / 16;
  int64_t v0, v1;
  split_range(a.nbytes / kVecBytes, bid, nb, v0, v1);
  // the thread's first input vector is loaded BEFORE the epoch read-modify-write (uncached
  // signal page), so the two memory round trips overlap instead of running back to back — the
  // latency floor of a small message (one vector per thread)
  const int64_t vf = v0 + threadIdx.x;
  u16x8 first[kQ];
  if (vf < v1) {
#pragma unroll
    for (int q = 0; q < kQ; ++q)
      first[q] = reinterpret_cast<const u16x8*>(static_cast<const char*>(a.inp) +
                                                vf * kVecBytes)[q];
  }
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t half = (e & 1) * a.cap;
  char* mine = a.data[a.rank] + half;
  if (vf < v1) {
#pragma unroll
    for (int q = 0; q < kQ; ++q) reinterpret_cast<u16x8*>(mine + vf * kVecBytes)[q] = first[q];
  }
  for (int64_t v = vf + blockDim.x; v < v1; v += blockDim.x) {
#pragma unroll
    for (int q = 0; q < kQ; ++q)
      reinterpret_cast<u16x8*>(mine + v * kVecBytes)[q] =
          reinterpret_cast<const u16x8*>(static_cast<const char*>(a.inp) + v * kVecBytes)[q];
  }
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, half, v * kVecBytes, acc);
    store8<DT>(a.out, v, acc);
  }
}

template <int DT, int W>
__device__ __forceinline__ void twoshot_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t half = (e & 1) * a.cap;
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;      // vectors per shard
  int64_t s0, s1;
  split_range(shard_vec, bid, nb, s0, s1);
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
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
  // reduce-scatter: my shard, sub-range b
  char* my_tmp = a.tmp[a.rank] + half;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, half, (mybase + v) * kVecBytes, acc);
    store8<DT>(my_tmp, mybase + v, acc);
    store8<DT>(a.out, mybase + v, acc);
  }
  signal_peers(a, 1, e, bid);
  if (!wait_peers(a, 1, e, bid)) return;
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
__device__ __forceinline__ void twoshot_reg_body(const CarKernelArgs& a, unsigned bid,
                                                 unsigned nb) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  constexpr int kQ = kVecBytes / 16;
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  int64_t s0, s1;
  split_range(shard_vec, bid, nb, s0, s1);
  char* mine = a.data[a.rank];
  signal_peers(a, 0, e, bid);                  // my input is complete (stream order)
  if (!wait_peers(a, 0, e, bid)) return;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, 0, (mybase + v) * kVecBytes, acc);
    store8<DT>(mine, mybase + v, acc);
  }
  signal_peers(a, 1, e, bid);
  if (!wait_peers(a, 1, e, bid)) return;
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
  signal_peers(a, 2, e, bid);                  // done reading every peer's buffer
  wait_peers(a, 2, e, bid);
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
__device__ __forceinline__ void twoshot_push_body(const CarKernelArgs& a, unsigned bid,
                                                  unsigned nb) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  constexpr int kQ = kVecBytes / 16;
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t half = (e & 1) * a.cap;
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  const int64_t shard_bytes = shard_vec * kVecBytes;
  int64_t s0, s1;
  split_range(shard_vec, bid, nb, s0, s1);
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
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
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
  signal_peers(a, 1, e, bid);
  wait_peers(a, 1, e, bid);
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
__device__ __forceinline__ void pull_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t chunk = a.nbytes;                    // bytes per peer chunk, multiple of 16
  int64_t v0, v1;
  split_range(chunk / 16, bid, nb, v0, v1);
  const int64_t src_off = A2A ? a.rank * chunk : 0;
  char* out = static_cast<char*>(a.out);
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
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
  signal_peers(a, 2, e, bid);
  wait_peers(a, 2, e, bid);
}

template <int DT, int W>
__device__ __forceinline__ void ag_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  pull_body<W, false>(a, bid, nb);
}
template <int DT, int W>
__device__ __forceinline__ void a2a_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  pull_body<W, true>(a, bid, nb);
}

//   uneven all-to-all (MoE expert-parallel dispatch, top-k router splits): from every peer p
//   out[v_dst[p] .. + v_cnt[p]) = in_p[v_src[p] .. + v_cnt[p]) — each GPU pulls its own tokens
//   from all 7 peers at once, one hop per link (RCCL's all-to-all-v moves them peer by peer).
//   Peers are visited from rank + 1 on so the 7 links start loaded evenly; 4 independent 16-B
//   loads per thread and peer keep enough bytes in flight per link.
template <int DT, int W>
__device__ __forceinline__ void a2av_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  const uint32_t e = begin_epoch(a, bid, nb);
  char* out = static_cast<char*>(a.out);
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
  const int world = W > 0 ? W : a.world;
#pragma unroll
  for (int k = 0; k < (W > 0 ? W : kMaxRanks); ++k) {
    if (W == 0 && k >= world) break;
    const int p = W > 0 ? (a.rank + k) & (W - 1) : (a.rank + k) % world;
    int64_t v0, v1;
    split_range(a.v_cnt[p] / 16, bid, nb, v0, v1);
    const u16x8* src = reinterpret_cast<const u16x8*>(a.data[p] + a.v_src[p]);
    u16x8* dst = reinterpret_cast<u16x8*>(out + a.v_dst[p]);
    const int64_t bs = blockDim.x;
    int64_t v = v0 + threadIdx.x;
    for (; v + 3 * bs < v1; v += 4 * bs) {
      const u16x8 t0 = src[v], t1 = src[v + bs], t2 = src[v + 2 * bs], t3 = src[v + 3 * bs];
      dst[v] = t0;
      dst[v + bs] = t1;
      dst[v + 2 * bs] = t2;
      dst[v + 3 * bs] = t3;
    }
    for (; v < v1; v += bs) dst[v] = src[v];
  }
  signal_peers(a, 2, e, bid);
  wait_peers(a, 2, e, bid);
}

//   reduce-scatter : out[0 .. n/P) = sum_p in_p[rank * n/P .. ]   (fp32 accumulation)
template <int DT, int W>
__device__ __forceinline__ void rs_body(const CarKernelArgs& a, unsigned bid, unsigned nb) {
  constexpr int64_t kVecBytes = 8 * Elem<DT>::kBytes;
  const uint32_t e = begin_epoch(a, bid, nb);
  const int64_t shard_vec = a.nbytes / kVecBytes / a.world;
  int64_t s0, s1;
  split_range(shard_vec, bid, nb, s0, s1);
  signal_peers(a, 0, e, bid);
  if (!wait_peers(a, 0, e, bid)) return;
  const int64_t mybase = a.rank * shard_vec;
  for (int64_t v = s0 + threadIdx.x; v < s1; v += blockDim.x) {
    float acc[8];
    sum_vec<DT, W>(a, 0, (mybase + v) * kVecBytes, acc);
    store8<DT>(a.out, v, acc);
  }
  signal_peers(a, 2, e, bid);
  wait_peers(a, 2, e, bid);
}

// Kernel-argument block of the virtual-rank launch: every rank's own argument block.
struct CarVirtArgs {
  CarKernelArgs r[kMaxRanks];
};

// NAME<DT, W>: production per-rank grid. NAME##_vr<DT, W>: world x nb workgroups on one GPU,
// workgroup g runs rank g / nb (wave-uniform, so the argument block is read with scalar loads).
#define DLBB_CAR_KERNELS(NAME, BODY)                                                          \
  template <int DT, int W>                                                                    \
  __global__ void __launch_bounds__(kCarThreads) NAME(CarKernelArgs a) {                     \
    BODY<DT, W>(a, blockIdx.x, gridDim.x);                                                    \
  }                                                                                           \
  template <int DT, int W>                                                                    \
  __global__ void __launch_bounds__(kCarThreads) NAME##_vr(CarVirtArgs v, unsigned nb) {     \
    const unsigned r = blockIdx.x / nb;                                                       \
    BODY<DT, W>(v.r[r], blockIdx.x - r * nb, nb);                                             \
  }

DLBB_CAR_KERNELS(car_oneshot_kernel, oneshot_body)
DLBB_CAR_KERNELS(car_twoshot_kernel, twoshot_body)
DLBB_CAR_KERNELS(car_twoshot_reg_kernel, twoshot_reg_body)
DLBB_CAR_KERNELS(car_twoshot_push_kernel, twoshot_push_body)
DLBB_CAR_KERNELS(car_ag_kernel, ag_body)
DLBB_CAR_KERNELS(car_a2a_kernel, a2a_body)
DLBB_CAR_KERNELS(car_rs_kernel, rs_body)
DLBB_CAR_KERNELS(car_a2av_kernel, a2av_body)
#undef DLBB_CAR_KERNELS

enum CarKind : int {
  K_ONESHOT = 1, K_TWOSHOT = 2, K_REG = 3, K_PUSH = 4, K_AG = 5, K_A2A = 6, K_RS = 7, K_A2AV = 8
};

// Resolves (kind, DT, W) to the kernel symbol: per-rank form (VR = false) or virtual form.
template <int DT, int W, bool VR>
const void* car_kernel_ptr(int kind) {
#define DLBB_CAR_PTR(NAME)                                                        \
  (VR ? reinterpret_cast<const void*>(&NAME##_vr<DT, W>)                          \
      : reinterpret_cast<const void*>(&NAME<DT, W>))
  switch (kind) {
    case K_ONESHOT: return DLBB_CAR_PTR(car_oneshot_kernel);
    case K_TWOSHOT: return DLBB_CAR_PTR(car_twoshot_kernel);
    case K_REG: return DLBB_CAR_PTR(car_twoshot_reg_kernel);
    case K_PUSH: return DLBB_CAR_PTR(car_twoshot_push_kernel);
    case K_RS: return DLBB_CAR_PTR(car_rs_kernel);
    default: break;
  }
  if constexpr (DT == DT_BF16) {     // byte movers: one instantiation (dtype-free)
    if (kind == K_AG) return DLBB_CAR_PTR(car_ag_kernel);
    if (kind == K_A2A) return DLBB_CAR_PTR(car_a2a_kernel);
    if (kind == K_A2AV) return DLBB_CAR_PTR(car_a2av_kernel);
  }
#undef DLBB_CAR_PTR
  return nullptr;
}

template <bool VR>
const void* car_kernel(int kind, int dtype, int world) {
  if (kind == K_AG || kind == K_A2A || kind == K_A2AV) dtype = DT_BF16;
  const int w = world == 2 || world == 4 || world == 8 ? world : 0;
#define DLBB_CAR_W(D)                                        \
  switch (w) {                                               \
    case 2: return car_kernel_ptr<D, 2, VR>(kind);           \
    case 4: return car_kernel_ptr<D, 4, VR>(kind);           \
    case 8: return car_kernel_ptr<D, 8, VR>(kind);           \
    default: return car_kernel_ptr<D, 0, VR>(kind);          \
  }
  if (dtype == DT_BF16) DLBB_CAR_W(DT_BF16)
  if (dtype == DT_F16) DLBB_CAR_W(DT_F16)
  DLBB_CAR_W(DT_F32)
#undef DLBB_CAR_W
}

struct RegBuf {
  char* ptr[kMaxRanks] = {};    // every rank's registered buffer (mine at [rank])
  char* map[kMaxRanks] = {};    // base of the opened peer mapping it lives in (null: own / local)
  int64_t bytes = 0;            // 0: released (dlbb_car_reg_close); ids are never reused
};

struct OpenedMap {               // one hipIpcOpenMemHandle per (peer, allocation)
  int peer;
  hipIpcMemHandle_t handle;
  char* base;
  int refs;                      // live registrations inside this mapping
};

struct CarState {
  int rank = 0, world = 1, device = 0;
  int64_t cap = 0;
  char* data = nullptr;       // 2 * cap (coarse-grained, IPC)
  char* tmp = nullptr;        // 2 * cap
  Signal* sig = nullptr;      // uncached, IPC
  bool opened = false;
  bool local = false;         // virtual rank: peers are sibling states in this process (no IPC)
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

static void car_finish_open(CarState* s) {
  for (int p = 0; p < kMaxRanks; ++p) {
    s->args.data[p] = s->peer_data[p];
    s->args.tmp[p] = s->peer_tmp[p];
    s->args.sig[p] = s->peer_sig[p];
  }
  s->args.rank = s->rank;
  s->args.world = s->world;
  s->args.cap = s->cap;
  s->opened = true;
}

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
  car_finish_open(s);
  return hipSuccess;
}

// Virtual ranks (single-GPU harness): states[r] was created with dlbb_car_create(r, world, ...)
// in THIS process on the same device; every state's peers become its siblings' own allocations
// (no IPC handles). The kernels then run unchanged against buffers in one HBM.
DLBB_API int dlbb_car_open_local(void* const* states, int world) {
  if (world < 1 || world > kMaxRanks) return hipErrorInvalidValue;
  for (int r = 0; r < world; ++r) {
    const CarState* s = static_cast<const CarState*>(states[r]);
    if (!s || s->rank != r || s->world != world || s->opened ||
        s->cap != static_cast<const CarState*>(states[0])->cap ||
        s->device != static_cast<const CarState*>(states[0])->device)
      return hipErrorInvalidValue;
  }
  for (int r = 0; r < world; ++r) {
    CarState* s = static_cast<CarState*>(states[r]);
    for (int p = 0; p < world; ++p) {
      const CarState* q = static_cast<const CarState*>(states[p]);
      s->peer_data[p] = q->data;
      s->peer_tmp[p] = q->tmp;
      s->peer_sig[p] = q->sig;
    }
    s->local = true;
    car_finish_open(s);
  }
  return hipSuccess;
}

DLBB_API int64_t dlbb_car_capacity(void* h) { return static_cast<CarState*>(h)->cap; }

static const RegBuf* car_reg(const CarState* s, int id) {
  if (id < 0 || id >= static_cast<int>(s->regs.size()) || s->regs[id].bytes <= 0) return nullptr;
  return &s->regs[id];
}

// Validates one rank's call and fills its kernel-argument block. `count` is in elements for the
// all-reduce kinds and in bytes for the direct kinds (as the public entry points take them).
// *noop: nothing to launch (empty message, or a registered all-reduce at world 1).
// wait bound of every IPC kernel launched from now on. Default 60 s: ranks can enter a
// collective seconds apart (a peer still autotuning its first GEMMs; 8 processes time-sliced on
// one GPU in the rehearsal tests measured > 5 s), and a wrong timeout kills the instance; with
// fail-fast a dead peer costs one bound per rank, not one per call.
static uint64_t g_car_timeout_ticks = 60 * kRealtimeHz;

DLBB_API void dlbb_car_set_timeout_ms(int ms) {
  g_car_timeout_ticks = static_cast<uint64_t>(ms < 1 ? 1 : ms) * (kRealtimeHz / 1000);
}

static int car_prepare(const CarState* s, int kind, const void* inp, void* out, int64_t count,
                       int dtype, int id, CarKernelArgs* a, bool* noop) {
  *noop = false;
  if (!s->opened) return hipErrorNotInitialized;
  if (dtype != DT_BF16 && dtype != DT_F16 && dtype != DT_F32) return hipErrorInvalidValue;
  const int64_t esz = dtype == DT_F32 ? 4 : 2;
  const int64_t vec = 8 * esz;
  const int64_t W = s->world;
  *a = s->args;
  a->timeout_ticks = g_car_timeout_ticks;
  if (kind == K_ONESHOT || kind == K_TWOSHOT) {
    const int64_t nbytes = count * esz;
    if (nbytes < 0 || nbytes > s->cap || nbytes % vec != 0) return hipErrorInvalidValue;
    if (kind == K_TWOSHOT && nbytes % (vec * W) != 0) return hipErrorInvalidValue;
    a->inp = inp;
    a->out = out;
    a->nbytes = nbytes;
    *noop = nbytes == 0 || W == 1;
    return hipSuccess;
  }
  const RegBuf* r = car_reg(s, id);
  if (!r) return hipErrorInvalidValue;
  for (int p = 0; p < kMaxRanks; ++p) a->data[p] = r->ptr[p];
  a->inp = r->ptr[s->rank];
  if (kind == K_REG || kind == K_PUSH) {
    const int64_t nbytes = count * esz;
    if (nbytes < 0 || nbytes > r->bytes || nbytes % (vec * W) != 0) return hipErrorInvalidValue;
    if (kind == K_PUSH && nbytes > s->cap) return hipErrorInvalidValue;
    a->out = r->ptr[s->rank];
    a->nbytes = nbytes;
    *noop = nbytes == 0 || W == 1;
    return hipSuccess;
  }
  if (!out || count < 0) return hipErrorInvalidValue;
  if (kind == K_AG && (count % 16 || count > r->bytes)) return hipErrorInvalidValue;
  if (kind == K_A2A && (count % 16 || count * W > r->bytes)) return hipErrorInvalidValue;
  if (kind == K_RS && (count % (vec * W) || count > r->bytes)) return hipErrorInvalidValue;
  if (kind != K_AG && kind != K_A2A && kind != K_RS) return hipErrorInvalidValue;
  a->out = out;
  a->nbytes = count;
  *noop = count == 0;
  return hipSuccess;
}

static int clamp_blocks(int nblocks) {
  return nblocks < 1 ? 1 : nblocks > kMaxBlocks ? kMaxBlocks : nblocks;
}

static int car_launch_rank(CarState* s, int kind, const void* inp, void* out, int64_t count,
                           int dtype, int id, int nblocks, hipStream_t stream) {
  CarKernelArgs a;
  bool noop = false;
  const int rc = car_prepare(s, kind, inp, out, count, dtype, id, &a, &noop);
  if (rc != hipSuccess) return rc;
  if (noop) {
    if ((kind == K_ONESHOT || kind == K_TWOSHOT) && a.nbytes > 0 && out != inp)
      CAR_CHECK(hipMemcpyAsync(out, inp, a.nbytes, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }
  const void* fn = car_kernel<false>(kind, dtype, s->world);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {&a};
  CAR_CHECK(hipLaunchKernel(fn, dim3(clamp_blocks(nblocks)), dim3(kCarThreads), args, 0, stream));
  return hipSuccess;
}

// algo: 1 = one-shot, 2 = two-shot. nblocks <= 256. dtype: bf16 | f16 | f32.
// Requirements (checked): nbytes <= cap; nbytes % 16 == 0 (one-shot) or
// nbytes % (vec_bytes * world) == 0 (two-shot).
DLBB_API int dlbb_car_allreduce(void* h, const void* inp, void* out, int64_t n, int dtype,
                                int algo, int nblocks, hipStream_t stream) {
  return car_launch_rank(static_cast<CarState*>(h), algo == 2 ? K_TWOSHOT : K_ONESHOT, inp, out,
                         n, dtype, -1, nblocks, stream);
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
// the registration; *out_id indexes it for the registered launches. A peer allocation already
// mapped by a live registration is reused (one open per allocation and peer, reference counted).
DLBB_API int dlbb_car_reg_open(void* h, const void* ptr, int64_t nbytes, const void* all_handles,
                               const int64_t* offsets, int* out_id) {
  CarState* s = static_cast<CarState*>(h);
  if (!s->opened || s->local || nbytes <= 0) return hipErrorInvalidValue;
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
    OpenedMap* m = nullptr;
    for (OpenedMap& o : s->opened_maps)
      if (o.peer == p && memcmp(&o.handle, &hd, sizeof(hd)) == 0) m = &o;
    if (!m) {
      void* pd = nullptr;
      CAR_CHECK(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess));
      s->opened_maps.push_back(OpenedMap{p, hd, static_cast<char*>(pd), 0});
      m = &s->opened_maps.back();
    }
    r.ptr[p] = m->base + offsets[p];
    r.map[p] = m->base;
    // copy-engine read of the first and last byte: a bad mapping fails here, not in a kernel
    char probe[2];
    hipError_t e = hipMemcpy(&probe[0], r.ptr[p], 1, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&probe[1], r.ptr[p] + nbytes - 1, 1, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      if (m->refs == 0) {          // drop the mapping this call opened
        (void)hipIpcCloseMemHandle(m->base);
        s->opened_maps.pop_back();
      }
      for (int q = 0; q < p; ++q)  // and the references taken for the earlier peers
        for (OpenedMap& o : s->opened_maps)
          if (r.map[q] && o.peer == q && o.base == r.map[q]) --o.refs;
      return (int)e;
    }
    ++m->refs;
  }
  s->regs.push_back(r);
  *out_id = static_cast<int>(s->regs.size()) - 1;
  return hipSuccess;
}

// Virtual ranks: register ptrs[r] (one buffer per virtual rank, nbytes each) in every sibling
// state under the same id.
DLBB_API int dlbb_car_reg_local(void* const* states, int world, void* const* ptrs, int64_t nbytes,
                                int* out_id) {
  if (world < 1 || world > kMaxRanks || nbytes <= 0) return hipErrorInvalidValue;
  const size_t id = static_cast<CarState*>(states[0])->regs.size();
  for (int r = 0; r < world; ++r) {
    const CarState* s = static_cast<const CarState*>(states[r]);
    if (!s->local || s->world != world || s->regs.size() != id || !ptrs[r])
      return hipErrorInvalidValue;
  }
  RegBuf reg;
  reg.bytes = nbytes;
  for (int p = 0; p < world; ++p) reg.ptr[p] = static_cast<char*>(ptrs[p]);
  for (int r = 0; r < world; ++r) static_cast<CarState*>(states[r])->regs.push_back(reg);
  *out_id = static_cast<int>(id);
  return hipSuccess;
}

// Release registration `id`: peer mappings no other live registration uses are closed. The caller
// guarantees that no launch on it is in flight on ANY rank (synchronize + barrier first).
DLBB_API int dlbb_car_reg_close(void* h, int id) {
  CarState* s = static_cast<CarState*>(h);
  if (id < 0 || id >= static_cast<int>(s->regs.size()) || s->regs[id].bytes <= 0)
    return hipErrorInvalidValue;
  RegBuf& r = s->regs[id];
  for (int p = 0; p < s->world; ++p) {
    if (!r.map[p]) continue;
    for (size_t i = 0; i < s->opened_maps.size(); ++i) {
      OpenedMap& m = s->opened_maps[i];
      if (m.peer != p || m.base != r.map[p]) continue;
      if (--m.refs <= 0) {
        CAR_CHECK(hipIpcCloseMemHandle(m.base));
        s->opened_maps.erase(s->opened_maps.begin() + i);
      }
      break;
    }
  }
  r = RegBuf();
  return hipSuccess;
}

// Live registrations and opened peer mappings (lifecycle tests).
DLBB_API int dlbb_car_reg_counts(void* h, int* live_regs, int* open_maps) {
  const CarState* s = static_cast<const CarState*>(h);
  int live = 0;
  for (const RegBuf& r : s->regs) live += r.bytes > 0;
  *live_regs = live;
  *open_maps = static_cast<int>(s->opened_maps.size());
  return hipSuccess;
}

// In-place all-reduce of registration `id` (n elements from its start; n * esize must be a
// multiple of 16 * world and at most the registered size).
DLBB_API int dlbb_car_allreduce_reg(void* h, int id, int64_t n, int dtype, int nblocks,
                                    hipStream_t stream) {
  return car_launch_rank(static_cast<CarState*>(h), K_REG, nullptr, nullptr, n, dtype, id,
                         nblocks, stream);
}

// Push form of the registered two-shot (see twoshot_push_body); nbytes <= capacity.
DLBB_API int dlbb_car_allreduce_reg_push(void* h, int id, int64_t n, int dtype, int nblocks,
                                         hipStream_t stream) {
  return car_launch_rank(static_cast<CarState*>(h), K_PUSH, nullptr, nullptr, n, dtype, id,
                         nblocks, stream);
}

// Uneven all-to-all on registration `id` (every rank registered its input, the same number of
// bytes everywhere): pull cnt[p] bytes at src_off[p] of peer p's input into out + dst_off[p],
// for every p (all multiples of 16, within the registration). Collective, like every direct kind.
DLBB_API int dlbb_car_alltoallv_reg(void* h, int id, const int64_t* src_off, const int64_t* cnt,
                                    const int64_t* dst_off, void* out, int nblocks,
                                    hipStream_t stream) {
  CarState* s = static_cast<CarState*>(h);
  if (!s || !s->opened || !out || !src_off || !cnt || !dst_off) return hipErrorInvalidValue;
  const RegBuf* r = car_reg(s, id);
  if (!r) return hipErrorInvalidValue;
  CarKernelArgs a = s->args;
  a.timeout_ticks = g_car_timeout_ticks;
  for (int p = 0; p < kMaxRanks; ++p) {
    a.data[p] = r->ptr[p];
    a.v_src[p] = a.v_cnt[p] = a.v_dst[p] = 0;
  }
  int64_t total = 0;
  for (int p = 0; p < s->world; ++p) {
    if (cnt[p] < 0 || src_off[p] < 0 || dst_off[p] < 0 || cnt[p] % 16 || src_off[p] % 16 ||
        dst_off[p] % 16 || src_off[p] + cnt[p] > r->bytes)
      return hipErrorInvalidValue;
    a.v_src[p] = src_off[p];
    a.v_cnt[p] = cnt[p];
    a.v_dst[p] = dst_off[p];
    total += cnt[p];
  }
  a.inp = r->ptr[s->rank];
  a.out = out;
  a.nbytes = total;
  const void* fn = car_kernel<false>(K_A2AV, DT_BF16, s->world);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {&a};
  CAR_CHECK(hipLaunchKernel(fn, dim3(clamp_blocks(nblocks)), dim3(kCarThreads), args, 0, stream));
  return hipSuccess;
}

// Direct collectives on registration `id` (this rank's registered input; out is local).
//   kind 0 = all-gather  : bytes = chunk bytes per rank (<= registered), out = world x chunk
//   kind 1 = all-to-all  : bytes = chunk bytes per peer (world x chunk <= registered)
//   kind 2 = reduce-scatter (dtype): bytes = whole input (multiple of vec x world), out = bytes/world
DLBB_API int dlbb_car_direct_reg(void* h, int id, int kind, int64_t bytes, int dtype, void* out,
                                 int nblocks, hipStream_t stream) {
  if (kind < 0 || kind > 2) return hipErrorInvalidValue;
  static const int kKinds[3] = {K_AG, K_A2A, K_RS};
  return car_launch_rank(static_cast<CarState*>(h), kKinds[kind], nullptr, out, bytes, dtype, id,
                         nblocks, stream);
}

// ---- virtual-rank launch (single-GPU harness) -------------------------------------------------
// Resident workgroups of the virtual form of (kind, dtype, world) on this device: one launch of
// world x nblocks workgroups must fit entirely (every rank's workgroups spin on the others'), so
// dlbb_car_vr_launch refuses a larger grid instead of letting it wait out its timeout.
DLBB_API int dlbb_car_vr_max_blocks(int kind, int dtype, int world) {
  const void* fn = car_kernel<true>(kind, dtype, world);
  if (!fn) return -1;
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kCarThreads, 0) != hipSuccess)
    return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  return per_cu * cus;
}

// One launch of world x nblocks workgroups: every virtual rank r of the states opened with
// dlbb_car_open_local runs its part of collective `kind` (1 one-shot, 2 two-shot, 3 registered
// pull, 4 registered push, 5 all-gather, 6 all-to-all, 7 reduce-scatter) with inputs inp[r] /
// outputs out[r] (all-reduce kinds; direct kinds read registration `id` and write out[r]).
DLBB_API int dlbb_car_vr_launch(void* const* states, int world, int kind, const void* const* inp,
                                void* const* out, int64_t count, int dtype, int id, int nblocks,
                                hipStream_t stream) {
  if (world < 2 || world > kMaxRanks) return hipErrorInvalidValue;
  const int nb = clamp_blocks(nblocks);
  const int cap = dlbb_car_vr_max_blocks(kind, dtype, world);
  if (cap < 0) return hipErrorInvalidValue;
  if (nb * world > cap) return hipErrorInvalidConfiguration;
  CarVirtArgs v;
  bool noop = false;
  for (int r = 0; r < world; ++r) {
    const CarState* s = static_cast<const CarState*>(states[r]);
    if (!s || !s->local || s->rank != r || s->world != world) return hipErrorInvalidValue;
    const int rc = car_prepare(s, kind, inp ? inp[r] : nullptr, out ? out[r] : nullptr, count,
                               dtype, id, &v.r[r], &noop);
    if (rc != hipSuccess) return rc;
    if (noop) return hipSuccess;
  }
  const void* fn = car_kernel<true>(kind, dtype, world);
  unsigned nbu = static_cast<unsigned>(nb);
  void* args[] = {&v, &nbu};
  CAR_CHECK(hipLaunchKernel(fn, dim3(nb * world), dim3(kCarThreads), args, 0, stream));
  return hipSuccess;
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
    if (p == s->rank || !s->opened || s->local) continue;
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
