// Latency of the two stamp sources on gfx950, in shader cycles (s_memtime):
// s_memtime back to back, and an s_memrealtime whose result is waited for.
//   hipcc --offload-arch=gfx950 -O3 tools/clock_probe.hip -o tools/clock_probe_bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned long long* o) {
  unsigned long long a, b, c, d, r;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(a)::"memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(b)::"memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r)::"memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(d)::"memory");
  unsigned long long e;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e)::"memory");
  if (threadIdx.x == 0) {
    o[blockIdx.x * 4 + 0] = b - a;   // memtime -> memtime
    o[blockIdx.x * 4 + 1] = c - b;   // memtime -> memrealtime (waited) -> memtime
    o[blockIdx.x * 4 + 2] = e - c;   // again
    o[blockIdx.x * 4 + 3] = d - r;   // realtime ticks between the two realtime stamps
  }
}

int main() {
  unsigned long long* o;
  hipMalloc(&o, 256 * 4 * 8);
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(256), dim3(64), 0, 0, o);
  hipDeviceSynchronize();
  unsigned long long h[256 * 4];
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  double s[4] = {0, 0, 0, 0};
  for (int b = 0; b < 256; ++b)
    for (int i = 0; i < 4; ++i) s[i] += h[b * 4 + i];
  printf("mean over 256 wgs (shader cycles): memtime->memtime %.1f, memtime->realtime(waited)->memtime %.1f, %.1f; "
         "realtime ticks between two realtime stamps %.2f\n", s[0] / 256, s[1] / 256, s[2] / 256, s[3] / 256);
  hipFree(o);
  return 0;
}
