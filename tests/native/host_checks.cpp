// Host-side checks of the kernel library's C ABI, built with AddressSanitizer + LeakSanitizer +
// UBSan on the HOST code only (hipcc -Xarch_host -fsanitize=...; device code is not
// instrumented — GPU sanitizers are not available on this pool). Run by
// tests/test_native_host_asan.py on the CPU (no device: every entry point must fail cleanly,
// without leaks) and, when a GPU is visible, the create / destroy cycles run for real.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
int dlbb_gemm_bf16_nt(const void*, int64_t, const void*, int64_t, void*, int64_t, int64_t,
                      int64_t, int64_t, const void*, const void*, int64_t, void*, int, int,
                      hipStream_t);
int dlbb_gemm_wgrad(const void*, int64_t, const void*, int64_t, void*, int, int, float*, int, int,
                    int, int, hipStream_t);
int dlbb_attn_fwd(const void*, int64_t, void*, int64_t, float*, int, int, int, int, float,
                  hipStream_t);
int dlbb_attn_bwd(const void*, int64_t, const void*, const void*, int64_t, const float*, float*,
                  void*, int, int, int, int, float, hipStream_t);
int dlbb_car_create(int, int, int64_t, void**);
int dlbb_car_destroy(void*);
int dlbb_car_handle_bytes();
int dlbb_rccl_unique_id_bytes();
int dlbb_bias_gelu_fwd(const void*, const void*, void*, int64_t, int, int, hipStream_t);
int dlbb_pack_rows(const void*, int, int64_t, void*, int, int64_t, int64_t, int64_t, hipStream_t);
}

static int failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

int main() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const int bad = static_cast<int>(hipErrorInvalidValue);
  alignas(16) static uint16_t buf[4096];

  // ---- argument validation: rejected before any device work
  EXPECT(dlbb_gemm_bf16_nt(buf, 64, buf, 64, buf, 64, 8, 8, 100, nullptr, nullptr, 0, nullptr, 0,
                           0, nullptr) == bad);                        // K % 64
  EXPECT(dlbb_gemm_bf16_nt(buf + 1, 64, buf, 64, buf, 64, 8, 8, 64, nullptr, nullptr, 0, nullptr,
                           0, 0, nullptr) == bad);                     // misaligned A
  EXPECT(dlbb_gemm_bf16_nt(buf, 64, buf, 64, buf, 64, 8, 8, 64, nullptr, nullptr, 0, nullptr, 1,
                           0, nullptr) == bad);                        // bias flag, no bias
  EXPECT(dlbb_gemm_bf16_nt(buf, 64, buf, 64, buf, 64, 0, 8, 64, nullptr, nullptr, 0, nullptr, 0,
                           0, nullptr) == 0);                          // empty: no-op
  float ws[64];
  EXPECT(dlbb_gemm_wgrad(buf, 128, buf, 128, buf, 1, 0, ws, 100, 128, 128, 1, nullptr) == bad);
  EXPECT(dlbb_attn_fwd(buf, 192, buf, 64, nullptr, 1, 16, 1, 128, 0.1f, nullptr) == bad);  // D
  EXPECT(dlbb_attn_fwd(buf, 100, buf, 64, nullptr, 1, 16, 1, 64, 0.1f, nullptr) == bad);   // ld
  EXPECT(dlbb_attn_bwd(buf, 192, buf, buf, 64, nullptr, nullptr, buf, 1, 16, 1, 32, 0.1f,
                       nullptr) == bad);
  EXPECT(dlbb_bias_gelu_fwd(buf, nullptr, buf, 4, 12, 0, nullptr) == bad);                 // cols%8
  EXPECT(dlbb_pack_rows(buf, 7, 8, buf, 1, 8, 2, 8, nullptr) == bad);                      // dtype
  EXPECT(dlbb_car_handle_bytes() == 192);
  EXPECT(dlbb_rccl_unique_id_bytes() == 128);

  // ---- custom all-reduce state: invalid arguments, and create/destroy (no device: clean
  // failure; with a device: 3 full cycles) — LeakSanitizer checks both paths at exit
  void* h = nullptr;
  EXPECT(dlbb_car_create(0, 9, 1 << 20, &h) == bad);
  EXPECT(dlbb_car_create(2, 2, 1 << 20, &h) == bad);
  EXPECT(dlbb_car_create(0, 1, 0, &h) == bad);
  for (int i = 0; i < 3; ++i) {
    h = nullptr;
    const int rc = dlbb_car_create(0, 1, 1 << 20, &h);
    if (ndev > 0) {
      EXPECT(rc == 0 && h != nullptr);
    } else {
      EXPECT(rc != 0);
    }
    if (rc == 0) EXPECT(dlbb_car_destroy(h) == 0);
  }
  EXPECT(dlbb_car_destroy(nullptr) == 0);
  std::printf("host checks: devices=%d failures=%d\n", ndev, failures);
  return failures == 0 ? 0 : 1;
}
