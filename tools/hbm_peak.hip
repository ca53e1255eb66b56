// hbm_peak.hip — the measured HBM copy peak that bench.py reports beside the 8 TB/s spec figure (tools only, not
// part of libsbam): a streaming copy with 16-B global loads and stores (global_load_dwordx4 / global_store_dwordx4),
// four independent 16-B loads in flight per lane, grid-stride over a buffer far larger than the 256 MB Infinity
// Cache, launched with enough workgroups to fill 256 CUs several times over.  Read + write bytes / kernel time.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_copy16(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto ld = [](const u32x4 *p) { return NT ? __builtin_nontemporal_load(p) : *p; };
  auto st = [](u32x4 v, u32x4 *p) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
  };
  for (; i + 3 * stride < n; i += 4 * stride) {
    const u32x4 a = ld(src + i), b = ld(src + i + stride), c = ld(src + i + 2 * stride), d = ld(src + i + 3 * stride);
    st(a, dst + i);
    st(b, dst + i + stride);
    st(c, dst + i + 2 * stride);
    st(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) st(ld(src + i), dst + i);
}

// Copy `bytes` (multiple of 16) device to device `reps` times after one warm-up (nt: nontemporal loads and
// stores); *ms = average kernel time.
// Returns 0 or the HIP error code.
extern "C" int hbm_copy_peak(int device, int64_t bytes, int reps, int grid, int nt, double *ms) {
  if (hipSetDevice(device) != hipSuccess) return 1;
  void *a = nullptr, *b = nullptr;
  hipError_t e = hipMalloc(&a, bytes);
  if (e == hipSuccess) e = hipMalloc(&b, bytes);
  if (e == hipSuccess) e = hipMemset(a, 1, bytes);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  const int64_t n = bytes / 16;
  if (e == hipSuccess) {
    auto launch = [&]() {
      if (nt) hipLaunchKernelGGL(k_copy16<true>, dim3(grid), dim3(256), 0, 0, (const u32x4 *)a, (u32x4 *)b, n);
      else hipLaunchKernelGGL(k_copy16<false>, dim3(grid), dim3(256), 0, 0, (const u32x4 *)a, (u32x4 *)b, n);
    };
    launch();
    e = hipEventRecord(e0, 0);
    for (int r = 0; r < reps && e == hipSuccess; r++) {
      launch();
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(e1, 0);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    if (e == hipSuccess) *ms = (double)t / reps;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  return e == hipSuccess ? 0 : (int)e;
}
