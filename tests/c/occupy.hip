// Test helper (not part of libntt): a kernel that holds CUs for a given time, so that a GPU test can
// take part of the device away from a library launch deterministically (tests/test_gpu_fused_order.py).
// Each workgroup reserves `lds_bytes` of LDS (dynamic) and sleeps until `ms` milliseconds of the
// 100 MHz wall clock have passed since it started.  Built by tests/occupy_build.py.
#include <hip/hip_runtime.h>

__global__ void occ_spin(long long ticks) {
  extern __shared__ unsigned int occ_lds[];
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0) occ_lds[0] = 1u;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

extern "C" int occ_launch(int workgroups, int lds_bytes, double ms, void* stream) {
  if (workgroups <= 0 || lds_bytes < 4 || lds_bytes > 160 * 1024 || ms <= 0) return -1;
  const long long ticks = (long long)(ms * 1e5);  // wall_clock64: 100 MHz
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&occ_spin), hipFuncAttributeMaxDynamicSharedMemorySize,
                          lds_bytes) != hipSuccess)
    return -2;
  hipLaunchKernelGGL(occ_spin, dim3(workgroups), dim3(64), lds_bytes, static_cast<hipStream_t>(stream), ticks);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
