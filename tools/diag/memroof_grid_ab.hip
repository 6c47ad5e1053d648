// Grid-shape A/B of the production cast / pack kernels (csrc/cast.hip, included as is) at the
// collective-path sizes, VERDICT r05 item 6: torch's copy stays ~4 % ahead of the capped
// grid-stride cast at 1 GiB (profiles/r06_kernels/memroof_batched.jsonl). Variants: the
// production cap (4096 workgroups, grid-stride) vs larger caps and the uncapped one-tile-per-
// workgroup grid, U = 1 / 2 / 4 / 8 vectors per lane, plain vs non-temporal stores.
// Build + run (box):  hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//   -I distributed_llm_backend_benchmark_amd/csrc tools/diag/memroof_grid_ab.hip -o /tmp/mr_ab
//   && /tmp/mr_ab > gpurun_out/.../memroof_grid_ab.jsonl
#include <cstdio>
#include <vector>

#include "cast.hip"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <class F>
static float time_us(F f, int batch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  (void)hipDeviceSynchronize();
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < batch; ++i) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ts.push_back(ms * 1e3f / batch);
  }
  std::sort(ts.begin(), ts.end());
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ts[ts.size() / 2];
}

template <int DTI, int DTO, int U, bool NT>
static void cast_row(const char* name, const void* s, void* d, int64_t n, int batch) {
  constexpr int E = dlbb::cast_vec<DTI, DTO>();
  const int64_t tiles = (n / E + 256 * U - 1) / (256 * U);
  const double bytes = double(n) * (dlbb::Elem<DTI>::kBytes + dlbb::Elem<DTO>::kBytes);
  for (int64_t cap : {int64_t{4096}, int64_t{16384}, int64_t{65536}, int64_t{0}}) {
    const int64_t g = cap ? (tiles < cap ? tiles : cap) : tiles;
    if (g > 2147483647) continue;
    const float us = time_us([&] {
      hipLaunchKernelGGL((dlbb::cast2_kernel<DTI, DTO, U, NT>), dim3(unsigned(g)), dim3(256), 0,
                         0, s, d, n);
    }, batch, 15);
    printf("{\"kernel\": \"cast2\", \"pair\": \"%s\", \"src_MiB\": %lld, \"U\": %d, \"nt\": %d, "
           "\"cap\": %lld, \"grid\": %lld, \"us\": %.2f, \"TBps\": %.3f}\n",
           name, (long long)((n * dlbb::Elem<DTI>::kBytes) >> 20), U, int(NT), (long long)cap,
           (long long)g, us, bytes / us * 1e-6);
  }
}

template <int R, bool NT>
static void pack_row(const void* s, void* d, int64_t rows, int64_t cols, int batch) {
  const int64_t gx = (cols / 8 + 255) / 256;
  for (int64_t cap : {int64_t{4096}, int64_t{16384}, int64_t{0}}) {
    int64_t gy = (rows + R - 1) / R;
    if (cap) {
      const int64_t gyc = (cap + gx - 1) / gx;
      gy = gy < gyc ? gy : gyc;
    }
    gy = gy < 65535 ? gy : 65535;
    const float us = time_us([&] {
      hipLaunchKernelGGL((dlbb::pack2_kernel<dlbb::DT_BF16, dlbb::DT_BF16, R, NT>),
                         dim3(unsigned(gx), unsigned(gy)), dim3(256), 0, 0, s, d, rows, cols,
                         3 * cols, cols);
    }, batch, 15);
    const double bytes = double(rows) * cols * 4;
    printf("{\"kernel\": \"pack2\", \"src_MiB\": %lld, \"R\": %d, \"nt\": %d, \"cap\": %lld, "
           "\"grid\": [%lld, %lld], \"us\": %.2f, \"TBps\": %.3f}\n",
           (long long)((rows * cols * 2) >> 20), R, int(NT), (long long)cap, (long long)gx,
           (long long)gy, us, bytes / us * 1e-6);
  }
}

int main() {
  const int64_t max_bytes = int64_t{1} << 30;
  void *s = nullptr, *d = nullptr, *p = nullptr;
  CK(hipMalloc(&s, max_bytes));
  CK(hipMalloc(&d, 2 * max_bytes));
  CK(hipMalloc(&p, 3 * max_bytes));
  CK(hipMemset(s, 0x3c, max_bytes));
  CK(hipMemset(p, 0x3c, 3 * max_bytes));
  for (int64_t mib : {int64_t{64}, int64_t{1024}}) {
    const int batch = mib <= 256 ? 10 : 4;
    const int64_t nb = (mib << 20) / 2, nf = (mib << 20) / 4;
    using namespace dlbb;
    cast_row<DT_BF16, DT_F32, 8, true>("bf16->fp32", s, d, nb, batch);
    cast_row<DT_BF16, DT_F32, 8, false>("bf16->fp32", s, d, nb, batch);
    cast_row<DT_BF16, DT_F32, 4, true>("bf16->fp32", s, d, nb, batch);
    cast_row<DT_BF16, DT_F32, 2, true>("bf16->fp32", s, d, nb, batch);
    cast_row<DT_BF16, DT_F32, 1, true>("bf16->fp32", s, d, nb, batch);
    cast_row<DT_F32, DT_BF16, 8, true>("fp32->bf16", s, d, nf, batch);
    cast_row<DT_F32, DT_BF16, 4, true>("fp32->bf16", s, d, nf, batch);
    cast_row<DT_F32, DT_BF16, 2, false>("fp32->bf16", s, d, nf, batch);
    cast_row<DT_BF16, DT_BF16, 8, true>("bf16->bf16", s, d, nb, batch);
    cast_row<DT_BF16, DT_BF16, 2, false>("bf16->bf16", s, d, nb, batch);
    cast_row<DT_F32, DT_F32, 8, true>("fp32->fp32", s, d, nf, batch);
    cast_row<DT_F32, DT_F32, 2, false>("fp32->fp32", s, d, nf, batch);
    const float us = time_us([&] { (void)hipMemcpyAsync(d, s, mib << 20, hipMemcpyDeviceToDevice, 0); },
                             batch, 15);
    printf("{\"kernel\": \"hipMemcpyDtoD\", \"src_MiB\": %lld, \"us\": %.2f, \"TBps\": %.3f}\n",
           (long long)mib, us, 2.0 * (mib << 20) / us * 1e-6);
    const int64_t cols = 4096, rows = (mib << 20) / (2 * cols);
    pack_row<4, true>(p, d, rows, cols, batch);
    pack_row<4, false>(p, d, rows, cols, batch);
    pack_row<2, false>(p, d, rows, cols, batch);
    pack_row<1, false>(p, d, rows, cols, batch);
    pack_row<8, true>(p, d, rows, cols, batch);
    fflush(stdout);
  }
  CK(hipFree(s));
  CK(hipFree(d));
  CK(hipFree(p));
  return 0;
}
