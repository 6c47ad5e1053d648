// Native RCCL collective engine: communicator + timing loops in C++ (nccl-tests methodology).
//
// The reference times every collective from Python around a blocking backend call
// (collectives/1d/openmpi.py:60-65; collectives/1d/dsccl.py:61-67). Through torch's
// ProcessGroupNCCL an RCCL call also pays a cross-stream hop (caller stream -> internal NCCL
// stream -> caller stream) that is not part of the collective. This engine owns its own RCCL
// communicator (unique id broadcast over the torch process group by the Python side), enqueues
// the collective on ONE stream bracketed by HIP events, and runs the warmup / per-iteration
// (device barrier before every timed iteration) / back-to-back loops entirely in C++, so the
// reported latency is the collective's own.
//
// Links librccl.so.1 — resolved at load time to the RCCL torch already mapped (same SONAME),
// so both communicators come from one library instance.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <string.h>

#include <new>
#include <vector>

#define DLBB_API extern "C" __attribute__((visibility("default")))

namespace {

enum Op : int {
  OP_ALLREDUCE = 0,
  OP_ALLGATHER = 1,
  OP_REDUCE_SCATTER = 2,
  OP_BROADCAST = 3,
  OP_REDUCE = 4,
  OP_ALLTOALL = 5,
  OP_SENDRECV = 6,
  OP_GATHER = 7,
  OP_SCATTER = 8,
};

struct Engine {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
  float* barrier_buf = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    default: return ncclFloat32;
  }
}

size_t elem_size(int dt) { return dt == 0 ? 4 : 2; }

// count = elements of the per-rank message (the op's "N"): see bench/schema.py conventions.
ncclResult_t enqueue_on(Engine* e, int op, const void* send, void* recv, size_t count, int dt,
                        int root, hipStream_t st) {
  const ncclDataType_t t = to_nccl(dt);
  if (e->nranks == 1) {
    // One rank: every collective is the identity, i.e. a device copy when out of place
    // (hipMemcpyAsync on st: 5.3 TB/s at 1 GiB vs 4.6 for a vector-copy kernel).
    if (send == recv || count == 0) return ncclSuccess;
    return hipMemcpyAsync(recv, send, count * elem_size(dt), hipMemcpyDeviceToDevice, st) ==
                   hipSuccess
               ? ncclSuccess
               : ncclUnhandledCudaError;
  }
  switch (op) {
    case OP_ALLREDUCE:
      return ncclAllReduce(send, recv, count, t, ncclSum, e->comm, st);
    case OP_ALLGATHER:   // send: count, recv: nranks * count
      return ncclAllGather(send, recv, count, t, e->comm, st);
    case OP_REDUCE_SCATTER:   // send: count (multiple of nranks), recv: count / nranks
      return ncclReduceScatter(send, recv, count / e->nranks, t, ncclSum, e->comm, st);
    case OP_BROADCAST:
      return ncclBroadcast(send, recv, count, t, root, e->comm, st);
    case OP_REDUCE:
      return ncclReduce(send, recv, count, t, ncclSum, root, e->comm, st);
    case OP_ALLTOALL:   // count elements per rank, count / nranks to each peer
      return ncclAllToAll(send, recv, count / e->nranks, t, e->comm, st);
    case OP_GATHER:   // send: count, recv (root): nranks * count
      return ncclGather(send, recv, count, t, root, e->comm, st);
    case OP_SCATTER:   // send (root): nranks * count, recv: count
      return ncclScatter(send, recv, count, t, root, e->comm, st);
    case OP_SENDRECV: {   // ring: send to rank+1, receive from rank-1
      const int nxt = (e->rank + 1) % e->nranks, prv = (e->rank - 1 + e->nranks) % e->nranks;
      ncclResult_t r = ncclGroupStart();
      if (r != ncclSuccess) return r;
      r = ncclSend(send, count, t, nxt, e->comm, st);
      if (r == ncclSuccess) r = ncclRecv(recv, count, t, prv, e->comm, st);
      ncclResult_t r2 = ncclGroupEnd();
      return r != ncclSuccess ? r : r2;
    }
    default:
      return ncclInvalidArgument;
  }
}

ncclResult_t enqueue(Engine* e, int op, const void* send, void* recv, size_t count, int dt,
                     int root) {
  return enqueue_on(e, op, send, recv, count, dt, root, e->stream);
}

// device-side barrier: 1-element all-reduce on the engine stream, then host sync
int barrier(Engine* e) {
  if (ncclAllReduce(e->barrier_buf, e->barrier_buf, 1, ncclFloat32, ncclSum, e->comm,
                    e->stream) != ncclSuccess)
    return -1;
  return hipStreamSynchronize(e->stream) == hipSuccess ? 0 : -2;
}

}  // namespace

DLBB_API int dlbb_rccl_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

DLBB_API int dlbb_rccl_get_unique_id(void* out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return 1000 + static_cast<int>(r);
  memcpy(out, &id, sizeof(id));
  return 0;
}

DLBB_API int dlbb_rccl_init(const void* id_bytes, int nranks, int rank, void** out) {
  Engine* e = new (std::nothrow) Engine();
  if (!e) return 2;
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&e->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete e;
    return 1000 + static_cast<int>(r);
  }
  e->rank = rank;
  e->nranks = nranks;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&e->barrier_buf), 256) != hipSuccess ||
      hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) {
    ncclCommDestroy(e->comm);
    delete e;
    return 2;
  }
  (void)hipMemset(e->barrier_buf, 0, 256);
  *out = e;
  return 0;
}

DLBB_API int dlbb_rccl_run(void* h, int op, const void* send, void* recv, int64_t count, int dt,
                           int root) {
  Engine* e = static_cast<Engine*>(h);
  const ncclResult_t r = enqueue(e, op, send, recv, static_cast<size_t>(count), dt, root);
  if (r != ncclSuccess) return 1000 + static_cast<int>(r);
  return hipStreamSynchronize(e->stream) == hipSuccess ? 0 : 3;
}

// Enqueue on the CALLER's stream (e.g. torch's current stream) without synchronising: no
// cross-stream hop, and capturable into a HIP graph (RCCL kernels are graph-safe; only torch's
// ProcessGroupNCCL watchdog was not).
// `stream` is used as given — a null handle is the (legacy) default stream, a valid target;
// pass own_stream = 1 to use the engine's private stream instead.
DLBB_API int dlbb_rccl_enqueue(void* h, int op, const void* send, void* recv, int64_t count,
                               int dt, int root, void* stream, int own_stream) {
  Engine* e = static_cast<Engine*>(h);
  hipStream_t st = own_stream ? e->stream : static_cast<hipStream_t>(stream);
  const ncclResult_t r = enqueue_on(e, op, send, recv, static_cast<size_t>(count), dt, root, st);
  return r == ncclSuccess ? 0 : 1000 + static_cast<int>(r);
}

// Uneven all-to-all (MoE token dispatch): counts / displacements in elements, one entry per
// peer (host arrays of nranks size_t). Single rank: the self block is a stream-ordered copy.
DLBB_API int dlbb_rccl_alltoallv(void* h, const void* send, const int64_t* sendcounts,
                                 const int64_t* sdispls, void* recv, const int64_t* recvcounts,
                                 const int64_t* rdispls, int dt, void* stream) {
  Engine* e = static_cast<Engine*>(h);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t es = elem_size(dt);
  if (e->nranks == 1) {
    if (sendcounts[0] == 0) return 0;
    return hipMemcpyAsync(static_cast<char*>(recv) + rdispls[0] * es,
                          static_cast<const char*>(send) + sdispls[0] * es, sendcounts[0] * es,
                          hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : 3;
  }
  std::vector<size_t> sc(e->nranks), sd(e->nranks), rc(e->nranks), rd(e->nranks);
  for (int p = 0; p < e->nranks; ++p) {
    sc[p] = static_cast<size_t>(sendcounts[p]);
    sd[p] = static_cast<size_t>(sdispls[p]);
    rc[p] = static_cast<size_t>(recvcounts[p]);
    rd[p] = static_cast<size_t>(rdispls[p]);
  }
  const ncclResult_t r = ncclAllToAllv(send, sc.data(), sd.data(), recv, rc.data(), rd.data(),
                                       to_nccl(dt), e->comm, st);
  return r == ncclSuccess ? 0 : 1000 + static_cast<int>(r);
}

// Per-iteration timing, reference methodology: [device barrier + sync] -> event -> op -> event
// -> sync; times_us[i] = device time of iteration i. `warmup` untimed iterations first.
DLBB_API int dlbb_rccl_time_iters(void* h, int op, const void* send, void* recv, int64_t count,
                                  int dt, int root, int warmup, int iters, float* times_us) {
  Engine* e = static_cast<Engine*>(h);
  for (int i = 0; i < warmup; ++i) {
    if (enqueue(e, op, send, recv, static_cast<size_t>(count), dt, root) != ncclSuccess) return 4;
  }
  if (hipStreamSynchronize(e->stream) != hipSuccess) return 3;
  for (int i = 0; i < iters; ++i) {
    if (barrier(e) != 0) return 5;
    (void)hipEventRecord(e->ev0, e->stream);
    if (enqueue(e, op, send, recv, static_cast<size_t>(count), dt, root) != ncclSuccess) return 4;
    (void)hipEventRecord(e->ev1, e->stream);
    if (hipEventSynchronize(e->ev1) != hipSuccess) return 3;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e->ev0, e->ev1);
    times_us[i] = ms * 1000.f;
  }
  return 0;
}

// Back-to-back timing (nccl-tests): one event pair around `iters` enqueued ops; returns the mean
// microseconds per op in *mean_us.
DLBB_API int dlbb_rccl_time_batched(void* h, int op, const void* send, void* recv, int64_t count,
                                    int dt, int root, int warmup, int iters, float* mean_us) {
  Engine* e = static_cast<Engine*>(h);
  for (int i = 0; i < warmup; ++i)
    if (enqueue(e, op, send, recv, static_cast<size_t>(count), dt, root) != ncclSuccess) return 4;
  if (barrier(e) != 0) return 5;
  (void)hipEventRecord(e->ev0, e->stream);
  for (int i = 0; i < iters; ++i)
    if (enqueue(e, op, send, recv, static_cast<size_t>(count), dt, root) != ncclSuccess) return 4;
  (void)hipEventRecord(e->ev1, e->stream);
  if (hipEventSynchronize(e->ev1) != hipSuccess) return 3;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e->ev0, e->ev1);
  *mean_us = ms * 1000.f / static_cast<float>(iters > 0 ? iters : 1);
  return 0;
}

DLBB_API int dlbb_rccl_destroy(void* h) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return 0;
  (void)hipStreamSynchronize(e->stream);
  ncclCommDestroy(e->comm);
  (void)hipEventDestroy(e->ev0);
  (void)hipEventDestroy(e->ev1);
  (void)hipFree(e->barrier_buf);
  (void)hipStreamDestroy(e->stream);
  delete e;
  return 0;
}
