// overlap_probe.hip -- can a dependent kernel of a hipGraph start before its
// predecessor ends on gfx950?  (measurement tool, not part of the library)
//
// A chain of N kernels alternating a small grid (40 WGs x 256 threads, ~w0 us
// of work, like an optimizer launch) and a large one (128 WGs x 512 threads,
// ~w1 us, like a gradient launch).  Each WG writes `kb` KiB (dirty lines at
// the boundary), then thread 0 fences (agent-scope release) and adds 1 to
// ctr[pos]; with `wait`, a WG first spins until ctr[pos - 1] == grid of the
// previous kernel (bounded: records a fault instead of hanging), then acquires.
// Modes, one graph each (replayed `reps` times, event-timed):
//   0 serial  one stream, no device waits (the kernel boundary orders them)
//   1 serial  one stream + the device waits (their cost when already satisfied)
//   2 fork    kernels alternate two captured streams (A: even, B: odd), each
//             stream's own order kept by the graph, the cross-stream order only
//             by the device waits -- kernel i+1 may be dispatched while i runs
// Per boundary it prints (last WG end of kernel i) -> (first WG start of
// kernel i+1) and (first WG start of i+1) -> (its wait satisfied).
//   hipcc -O3 --offload-arch=gfx950 tools/overlap_probe.hip -o tools/overlap_probe_bin
//   tools/overlap_probe_bin [N=12] [w0_us=3] [w1_us=7] [kb=16] [reps=200]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr int MAXK = 64, MAXWG = 128;

struct KArgs {
  uint32_t* ctr;            // [MAXK]
  uint32_t* fault;
  unsigned long long* t;    // [MAXK][MAXWG][3]: start, wait satisfied, end
  float* scratch;           // per-WG dirty bytes
  int pos, wait, nprev, kb;
  unsigned long long work_ticks;  // 100 MHz ticks
};

__global__ __launch_bounds__(512) void k_chain(KArgs a) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  __shared__ unsigned long long tw;
  if (threadIdx.x == 0) {
    unsigned long long tsat = t0;
    if (a.wait) {
      uint32_t it = 0;
      while (__hip_atomic_load(a.ctr + a.pos - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)a.nprev) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1u << 16)) {  // ~2 ms: a wait that is never satisfied costs little
          __hip_atomic_store(a.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __atomic_thread_fence(__ATOMIC_ACQUIRE);  // agent scope by default in HIP device code
      tsat = __builtin_amdgcn_s_memrealtime();
    }
    tw = tsat;
  }
  __syncthreads();
  // busy work
  const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
  float acc = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - tb < a.work_ticks) acc = acc * 1.0000001f + 1.0f;
  // dirty lines
  float* s = a.scratch + (size_t)blockIdx.x * (a.kb * 256);
  for (int i = threadIdx.x; i < a.kb * 256; i += blockDim.x) s[i] = acc + (float)i;
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __hip_atomic_fetch_add(a.ctr + a.pos, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long* t = a.t + ((size_t)a.pos * MAXWG + blockIdx.x) * 3;
    t[0] = t0;
    t[1] = tw;
    t[2] = __builtin_amdgcn_s_memrealtime();
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 12;
  const double w0 = argc > 2 ? atof(argv[2]) : 3.0, w1 = argc > 3 ? atof(argv[3]) : 7.0;
  const int kb = argc > 4 ? atoi(argv[4]) : 16;
  const int reps = argc > 5 ? atoi(argv[5]) : 200;
  if (N < 2 || N > MAXK) return 1;
  uint32_t *ctr, *fault;
  unsigned long long* t;
  float* scratch;
  CHK(hipMalloc(&ctr, MAXK * 4));
  CHK(hipMalloc(&fault, 4));
  CHK(hipMalloc(&t, sizeof(unsigned long long) * MAXK * MAXWG * 3));
  CHK(hipMalloc(&scratch, sizeof(float) * MAXWG * kb * 256 * 2));
  CHK(hipMemset(fault, 0, 4));
  hipStream_t sa, sb;
  CHK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CHK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  // grid / block of the odd (large) kernels: argv[6] argv[7] (default 128 x 512)
  const int g1 = argc > 6 ? atoi(argv[6]) : 128, b1 = argc > 7 ? atoi(argv[7]) : 512;
  const int nmodes = argc > 8 ? atoi(argv[8]) : 3;
  if (g1 > MAXWG || b1 > 512) return 1;
  auto grid = [&](int i) { return i % 2 ? g1 : 40; };
  auto block = [&](int i) { return i % 2 ? b1 : 256; };
  const char* names[3] = {"serial", "serial+wait", "fork"};
  for (int mode = 0; mode < nmodes; ++mode) {
    hipGraph_t g;
    hipGraphExec_t x;
    CHK(hipStreamBeginCapture(sa, hipStreamCaptureModeThreadLocal));
    CHK(hipMemsetAsync(ctr, 0, MAXK * 4, sa));
    hipEvent_t fk, jn;
    std::vector<hipEvent_t> evs;
    if (mode == 2) {
      CHK(hipEventCreateWithFlags(&fk, hipEventDisableTiming));
      CHK(hipEventRecord(fk, sa));
      CHK(hipStreamWaitEvent(sb, fk, 0));
    }
    for (int i = 0; i < N; ++i) {
      KArgs a;
      a.ctr = ctr;
      a.fault = fault;
      a.t = t;
      a.scratch = scratch + (size_t)(i % 2) * MAXWG * kb * 256;
      a.pos = i;
      a.wait = (mode >= 1 && i > 0) ? 1 : 0;
      a.nprev = i > 0 ? grid(i - 1) : 0;
      a.kb = kb;
      a.work_ticks = (unsigned long long)((i % 2 ? w1 : w0) * 100.0);
      hipStream_t s = (mode == 2 && i % 2) ? sb : sa;
      hipLaunchKernelGGL(k_chain, dim3(grid(i)), dim3(block(i)), 0, s, a);
      CHK(hipGetLastError());
    }
    if (mode == 2) {
      CHK(hipEventCreateWithFlags(&jn, hipEventDisableTiming));
      CHK(hipEventRecord(jn, sb));
      CHK(hipStreamWaitEvent(sa, jn, 0));
    }
    CHK(hipStreamEndCapture(sa, &g));
    CHK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    for (int r = 0; r < (mode == 2 ? 2 : 10); ++r) CHK(hipGraphLaunch(x, sa));
    CHK(hipStreamSynchronize(sa));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, sa));
    const int nrep = mode == 2 ? std::min(reps, 20) : reps;
    for (int r = 0; r < nrep; ++r) CHK(hipGraphLaunch(x, sa));
    CHK(hipEventRecord(e1, sa));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t hf = 0;
    CHK(hipMemcpy(&hf, fault, 4, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> h((size_t)MAXK * MAXWG * 3);
    CHK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
    printf("mode %-12s N=%d w0=%.1f w1=%.1f kb=%d: %.2f us per graph (%.2f us of work), fault=%u\n", names[mode], N, w0,
           w1, kb, 1000.0 * ms / nrep, (N / 2) * (w0 + w1) + (N % 2) * w0, hf);
    // per boundary, last replay: end(i) -> first start(i+1), first start(i+1) -> wait satisfied
    double sum_gap = 0;
    printf("  boundary: end(i)->start(i+1) us | start(i+1)->satisfied us\n  ");
    for (int i = 0; i + 1 < N; ++i) {
      unsigned long long end_i = 0, st_n = ~0ull, sat_n = 0;
      for (int b = 0; b < grid(i); ++b) end_i = std::max(end_i, h[((size_t)i * MAXWG + b) * 3 + 2]);
      for (int b = 0; b < grid(i + 1); ++b) {
        st_n = std::min(st_n, h[((size_t)(i + 1) * MAXWG + b) * 3 + 0]);
        sat_n = std::max(sat_n, h[((size_t)(i + 1) * MAXWG + b) * 3 + 1]);
      }
      const double gap = ((double)st_n - (double)end_i) / 100.0;
      sum_gap += gap;
      printf("%.2f|%.2f ", gap, ((double)sat_n - (double)st_n) / 100.0);
    }
    printf("\n  mean end->start %.2f us\n", sum_gap / (N - 1));
    // dispatch ramp: last WG start - first WG start, and last end - first end, per kernel
    printf("  start spread | end spread us per kernel:\n  ");
    for (int i = 0; i < N; ++i) {
      unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
      for (int b = 0; b < grid(i); ++b) {
        const unsigned long long* q = &h[((size_t)i * MAXWG + b) * 3];
        s0 = std::min(s0, q[0]);
        s1 = std::max(s1, q[0]);
        e0 = std::min(e0, q[2]);
        e1 = std::max(e1, q[2]);
      }
      printf("%.2f|%.2f ", (s1 - s0) / 100.0, (e1 - e0) / 100.0);
    }
    printf("\n");
    fflush(stdout);
    CHK(hipMemset(fault, 0, 4));
    CHK(hipGraphExecDestroy(x));
    CHK(hipGraphDestroy(g));
  }
  return 0;
}
