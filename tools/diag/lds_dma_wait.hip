// Minimal reproduction of the compiler behaviour behind csrc/common.h ds_read_tr16 (round 5):
// LDS-DMA into one half of a dynamic LDS array, then a transposed read of the OTHER half.
//   k_builtin : __builtin_amdgcn_ds_read_tr16_b64 -> the compiler emits s_waitcnt vmcnt(0)
//               before the read (waits for the DMA it cannot prove disjoint)
//   k_plain   : a plain 16-byte LDS load of the same address -> no wait
//   k_asm     : the inline-asm read of csrc/common.h -> no wait (caller waits lgkmcnt itself)
// tests/test_isa_cpu.py compiles this for gfx950 and checks all three.
#include "../../distributed_llm_backend_benchmark_amd/csrc/common.h"
using namespace dlbb;

extern __shared__ char dyn_smem[];

extern "C" __global__ void k_builtin(const int* __restrict__ g, i16x4* out, int n) {
  i16x4 acc = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    __builtin_amdgcn_global_load_lds(g + i * 256 + threadIdx.x,
                                     (lds_vptr_t)(dyn_smem + ((i + 1) & 1) * 4096), 4, 0, 0);
    acc += __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_i16x4_ptr)(dyn_smem + (i & 1) * 4096 + threadIdx.x * 8));
    __builtin_amdgcn_s_barrier();
  }
  out[threadIdx.x] = acc;
}

extern "C" __global__ void k_plain(const int* __restrict__ g, bf16x8* out, int n) {
  bf16x8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    __builtin_amdgcn_global_load_lds(g + i * 256 + threadIdx.x,
                                     (lds_vptr_t)(dyn_smem + ((i + 1) & 1) * 4096), 4, 0, 0);
    acc += *reinterpret_cast<const bf16x8*>(dyn_smem + (i & 1) * 4096 + threadIdx.x * 16);
    __builtin_amdgcn_s_barrier();
  }
  out[threadIdx.x] = acc;
}

extern "C" __global__ void k_asm(const int* __restrict__ g, i16x4* out, int n) {
  i16x4 acc = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    __builtin_amdgcn_global_load_lds(g + i * 256 + threadIdx.x,
                                     (lds_vptr_t)(dyn_smem + ((i + 1) & 1) * 4096), 4, 0, 0);
    i16x4 t = ds_read_tr16(dyn_smem + (i & 1) * 4096 + threadIdx.x * 8);
    tr_wait(t);
    acc += t;
    __builtin_amdgcn_s_barrier();
  }
  out[threadIdx.x] = acc;
}
