// wstream.hip -- per-CU weight-stream ceiling on gfx950 (measurement tool, not
// part of the library).  Every workgroup (1024 threads, one per CU) streams
// `kb` KiB of f32x4 through registers, the way the general gradient kernels
// stream weight chunks (16-B loads, 8 loads per lane in flight), and the
// kernel time gives bytes per CU-cycle.  Modes:
//   0 shared   every workgroup reads the SAME bytes in the same order
//   1 distinct every workgroup reads its own bytes (no sharing)
//   2 rotated  the same bytes, each workgroup starting at its own offset
//   3 xcd-rot  the same bytes, the start rotated by blockIdx / 8 (workgroups
//              of one XCD spread, the 8 XCDs in step)
//   hipcc -O3 --offload-arch=gfx950 tools/wstream.hip -o /tmp/wstream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ __launch_bounds__(1024) void k_stream(const f32x4* __restrict__ w, int n4, int mode, int reps, float* out) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const f32x4* base = mode == 1 ? w + (size_t)blockIdx.x * n4 : w;
  int rot = 0;
  if (mode == 2) rot = (int)(((size_t)blockIdx.x * 7919u) % (unsigned)(n4 / nt)) * nt;
  if (mode == 3) rot = (int)(((size_t)(blockIdx.x >> 3) * (n4 / nt) / 32u)) * nt;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r) {
    for (int i0 = 0; i0 < n4; i0 += D * nt) {
      f32x4 v[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        int i = i0 + d * nt + tid + rot;
        if (i >= n4) i -= n4;
        v[d] = base[i];
      }
#pragma unroll
      for (int d = 0; d < D; ++d) acc += v[d];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[blockIdx.x] = 1.f;
}

int main(int argc, char** argv) {
  const int kb = argc > 1 ? atoi(argv[1]) : 832;
  const int grid = argc > 2 ? atoi(argv[2]) : 256;
  const int reps = argc > 3 ? atoi(argv[3]) : 1;
  const int n4 = kb * 1024 / 16;
  f32x4* w;
  float* out;
  if (hipMalloc(&w, (size_t)n4 * 16 * grid) != hipSuccess || hipMalloc(&out, 4 * grid) != hipSuccess) return 1;
  (void)hipMemset(w, 0, (size_t)n4 * 16 * grid);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[4] = {"shared", "distinct", "rotated", "xcd-rot"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int depth = 0; depth < 2; ++depth) {
      float best = 1e30f;
      for (int it = 0; it < 12; ++it) {
        (void)hipEventRecord(e0);
        if (depth == 0) hipLaunchKernelGGL(k_stream<8>, dim3(grid), dim3(1024), 0, 0, w, n4, mode, reps, out);
        else hipLaunchKernelGGL(k_stream<2>, dim3(grid), dim3(1024), 0, 0, w, n4, mode, reps, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2 && ms < best) best = ms;
      }
      const double bytes = (double)n4 * 16 * reps;
      printf("mode %-8s depth %d  %d KiB x %d reps x %d WGs: %.2f us  %.1f GB/s per CU  %.1f B/clk@2.4GHz  chip %.2f TB/s\n",
             names[mode], depth == 0 ? 8 : 2, kb, reps, grid, best * 1e3, bytes / (best * 1e-3) / 1e9,
             bytes / (best * 1e-3) / 2.4e9, bytes * grid / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
