// What a launch costs outside its workgroups, by bytes written: the packet's
// begin -> first workgroup start and last wave end -> packet end, for the S2
// gradient launches' shape (129 workgroups x 512 threads, one per CU) writing
// 0 .. 4 MB with plain 16-B stores (the partial slabs and hand-off blocks are
// ~3.3 MB per critic launch), each launch stamping its first start / last end
// on s_memrealtime.  Run under rocprofv3 --kernel-trace for the packet times:
//   hipcc --offload-arch=gfx950 -O3 tools/outside_probe.hip -o tools/outside_probe_bin
//   rocprofv3 --kernel-trace --stats -d <dir> -o run --output-format csv -- tools/outside_probe_bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

struct Span {
  unsigned long long t0, t1;
};

// per-workgroup start / end stamps with plain stores (a first version used
// one global atomicMin / atomicMax per workgroup: 129 device-scope atomics on
// one address serialised and added ~3 us to every boundary)
__global__ __launch_bounds__(512) void k_write(float4* buf, int per_wg, Span* span, int slot) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  float4* p = buf + (size_t)blockIdx.x * per_wg;
  const float v = (float)(blockIdx.x + slot);
  for (int i = threadIdx.x; i < per_wg; i += blockDim.x) p[i] = make_float4(v, v, v, v);
  __syncthreads();
  if (threadIdx.x == 0) span[(size_t)slot * gridDim.x + blockIdx.x] = Span{t, __builtin_amdgcn_s_memrealtime()};
}

int main() {
  const int grid = 129, reps = 60;
  const int sizes_kb[] = {0, 256, 1024, 2048, 3392, 4096};  // bytes written per launch
  float4* buf = nullptr;
  Span* span = nullptr;
  (void)hipMalloc(&buf, (size_t)8 << 20);
  (void)hipMalloc(&span, sizeof(Span) * reps * grid);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int kb : sizes_kb) {
    const int per_wg = (int)(((size_t)kb << 10) / 16 / grid);
    std::vector<Span> init((size_t)reps * grid, Span{0ull, 0ull});
    (void)hipMemcpy(span, init.data(), sizeof(Span) * reps * grid, hipMemcpyHostToDevice);
    // a captured chain of launches, as the training step's graph replays them
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_write, dim3(grid), dim3(512), 0, s, buf, per_wg, span, r);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s);   // warm
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(span, init.data(), sizeof(Span) * reps * grid, hipMemcpyHostToDevice);
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    std::vector<Span> w((size_t)reps * grid), h(reps, Span{~0ull, 0ull});
    (void)hipMemcpy(w.data(), span, sizeof(Span) * reps * grid, hipMemcpyDeviceToHost);
    for (int r = 0; r < reps; ++r)
      for (int b = 0; b < grid; ++b) {
        const Span& x = w[(size_t)r * grid + b];
        h[r].t0 = x.t0 < h[r].t0 ? x.t0 : h[r].t0;
        h[r].t1 = x.t1 > h[r].t1 ? x.t1 : h[r].t1;
      }
    double body = 0, gap = 0;
    for (int r = 2; r < reps; ++r) {
      body += (h[r].t1 - h[r].t0) * 0.01;
      gap += (h[r].t0 - h[r - 1].t1) * 0.01;
    }
    std::printf("written %5d KB per launch: in-kernel span %.2f us, last end -> next first start %.2f us\n", kb,
                body / (reps - 2), gap / (reps - 2));
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  (void)hipFree(buf);
  (void)hipFree(span);
  return 0;
}
