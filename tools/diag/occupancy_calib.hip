// Calibration of the PMC occupancy estimate (waves per SIMD = SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE
// / 8) / 1024): spin kernels whose residency is known by construction. 256-thread workgroups
// (one wave per SIMD each) that spin ~200 us; `wgs` = 256 / 512 / 768 / 1024 -> 1 / 2 / 3 / 4
// waves per SIMD when every workgroup is resident at once (tiny register / LDS use).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/occ tools/diag/occupancy_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) spin(long long cycles, int* out) {
  const long long t0 = wall_clock64();
  long long t = t0;
  int acc = 0;
  while (t - t0 < cycles) {
    t = wall_clock64();
    acc += static_cast<int>(t);
  }
  if (acc == 0x7fffffff) out[threadIdx.x] = acc;   // keeps the loop; never true in practice
}

int main() {
  int* out;
  if (hipMalloc(&out, 1024 * sizeof(int)) != hipSuccess) return 1;
  // wall_clock64 runs at 100 MHz on this part: 20000 ticks = 200 us
  for (int wgs : {256, 512, 768, 1024}) {
    for (int rep = 0; rep < 3; ++rep) spin<<<wgs, 256>>>(20000, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("wgs %d done\n", wgs);
  }
  hipFree(out);
  return 0;
}
