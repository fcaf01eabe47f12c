// Shader-clock probe for bench diagnostics (not part of the product library).
//
// One wave samples the 64-bit shader-clock counter (s_memtime) and the constant
// 100 MHz counter (s_memrealtime) every `interval` real-time ticks, `n` times,
// and stores the pairs with ordinary vector stores: out[2i] = memtime,
// out[2i+1] = memrealtime.  The shader clock over a sample interval is
// d(memtime) / d(memrealtime) * 100 MHz.  Launched on a side stream while the
// timed steps run, it records the clock the kernels saw.
//
// Build: hipcc -O3 -shared -fPIC --offload-arch=gfx950 scripts/diag_clock.hip -o scripts/libdxr_diag.so
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(64) clock_probe_kernel(unsigned long long* out, int n,
                                                          unsigned long long interval) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    const unsigned long long target = r0 + (unsigned long long)i * interval;
    while (__builtin_amdgcn_s_memrealtime() < target) __builtin_amdgcn_s_sleep(2);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 2) out[2 * i + threadIdx.x] = threadIdx.x == 0 ? t : r;
  }
}

extern "C" int dxr_diag_clock_probe(unsigned long long* out, int n, unsigned long long interval,
                                    hipStream_t stream) {
  if (n <= 0 || !out) return 1;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, stream, out, n, interval);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
