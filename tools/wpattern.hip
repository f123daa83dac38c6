// wpattern.hip -- per-CU load rate of the gradient kernels' weight-fragment
// access patterns on gfx950 (measurement tool, not part of the library).
// 256 workgroups x 1024 threads (one per CU), every workgroup reading the SAME
// `kb` KiB of row-major weight matrices W[K][128], as the 16-row tiles do:
//   0 contig   f32x4 per lane, 1 KiB contiguous per wave instruction (wstream)
//   1 tile16   load_wchunk: lane (r, kq) reads the f32 W[k0 + 4 s + kq][16 t + r]
//              (a 16-column MFMA tile: 4 rows x 64 B per instruction)
//   2 group64  rg_load: f32x4 at W[k0 + 4 s + kq][64 g + 4 r] (4 rows x 256 B)
//   3 tcrow    load_wchunk_tc (round 2): f32x4 at W[16 t + r][c0 + 16 kq + 4 m]
//   4 tcrow2   f32x4 at W[16 t + r][c0 + 16 m + 4 kq]: the four kq lanes of a row
//              read 64 contiguous bytes per instruction
// Loads in flight per lane: 16 (f32) or 8 (f32x4) -- one 64-deep chunk.
//   hipcc -O3 --offload-arch=gfx950 tools/wpattern.hip -o /tmp/wpattern && /tmp/wpattern 512
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void k_pat(const float* __restrict__ w, int nmat, int mode, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, kq = lane >> 4;
  const int N = 128, K = 128;  // each matrix 64 KiB
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // work item = (matrix, 16-column tile or 64-column group, 64-deep chunk)
  if (mode == 0) {
    const f32x4* w4 = reinterpret_cast<const f32x4*>(w);
    const int n4 = nmat * K * N / 4;
    for (int i0 = 0; i0 < n4; i0 += 8 * 1024) {
      f32x4 v[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) v[d] = w4[i0 + d * 1024 + threadIdx.x];
#pragma unroll
      for (int d = 0; d < 8; ++d) acc += v[d];
    }
  } else if (mode == 1) {
    const int items = nmat * (N / 16) * (K / 64);
    for (int it = wave; it < items; it += 16) {
      const int m = it / ((N / 16) * (K / 64)), rem = it % ((N / 16) * (K / 64)), t = rem / (K / 64), c = rem % (K / 64);
      const float* W = w + (size_t)m * K * N;
      float v[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) v[s] = W[(64 * c + 4 * s + kq) * N + 16 * t + r];
#pragma unroll
      for (int s = 0; s < 16; ++s) acc[s & 3] += v[s];
    }
  } else if (mode == 2) {
    const int items = nmat * (N / 64) * (K / 32);
    for (int it = wave; it < items; it += 16) {
      const int m = it / ((N / 64) * (K / 32)), rem = it % ((N / 64) * (K / 32)), g = rem / (K / 32), c = rem % (K / 32);
      const float* W = w + (size_t)m * K * N;
      f32x4 v[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = *reinterpret_cast<const f32x4*>(W + (32 * c + 4 * s + kq) * N + 64 * g + 4 * r);
#pragma unroll
      for (int s = 0; s < 8; ++s) acc += v[s];
    }
  } else {
    const bool two = mode == 4;
    const int items = nmat * (K / 16) * (N / 64);
    for (int it = wave; it < items; it += 16) {
      const int m = it / ((K / 16) * (N / 64)), rem = it % ((K / 16) * (N / 64)), t = rem / (N / 64), c = rem % (N / 64);
      const float* W = w + (size_t)m * K * N;
      f32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[q] = *reinterpret_cast<const f32x4*>(W + (16 * t + r) * N + 64 * c + (two ? 16 * q + 4 * kq : 16 * kq + 4 * q));
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += v[q];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[blockIdx.x] = 1.f;
}

int main(int argc, char** argv) {
  const int kb = argc > 1 ? atoi(argv[1]) : 512;
  const int grid = argc > 2 ? atoi(argv[2]) : 256;
  const int nmat = kb / 64;
  float* w;
  float* out;
  if (hipMalloc(&w, (size_t)nmat * 64 * 1024) != hipSuccess || hipMalloc(&out, 4 * grid) != hipSuccess) return 1;
  (void)hipMemset(w, 0, (size_t)nmat * 64 * 1024);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[5] = {"contig", "tile16", "group64", "tcrow", "tcrow2"};
  for (int mode = 0; mode < 5; ++mode) {
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_pat, dim3(grid), dim3(1024), 0, 0, w, nmat, mode, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it >= 2 && ms < best) best = ms;
    }
    const double bytes = (double)nmat * 64 * 1024;
    printf("%-8s %d KiB x %d WGs: %7.2f us  %6.1f GB/s per CU  %5.1f B/clk@2.4GHz\n", names[mode], nmat * 64, grid,
           best * 1e3, bytes / (best * 1e-3) / 1e9, bytes / (best * 1e-3) / 2.4e9);
  }
  return 0;
}
