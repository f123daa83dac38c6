// overlap_branch_probe.hip -- do two independent launches on two streams (and
// as two branches of one captured graph) share the MI355X, i.e. can compute
// work hide in the CUs an optimizer-shaped launch leaves idle?  (tools only;
// not part of the library)
//
// A: the S5 critic optimizer's slab read (145 workgroups x 1,024 threads, each
//    summing 256 partials of 256 parameters: 37.9 MB);
// C: an MFMA chain kernel of nc workgroups x 1,024 threads (each wave a chain
//    of fp32 16x16x4 MFMAs on register operands), the shape of a target-actor
//    forward pass with no memory traffic.
// Timed: A alone, C alone, A then C on one stream, A || C on two streams, and
// A || C as two branches of one graph (replayed), by events on the first
// stream with the second joined into it.
//   hipcc -O3 --offload-arch=gfx950 tools/overlap_branch_probe.hip -o tools/overlap_branch_probe_bin
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)(i & 1023) * 1e-3f;
}

__global__ __launch_bounds__(1024) void k_read(const float* __restrict__ slab, int nwg, int64_t stride_w, float* out) {
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6, c = blockIdx.x;
  const float* base = slab + (int64_t)c * 256 + 4 * lane;
  f32x4 v[16];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = *reinterpret_cast<const f32x4*>(base + (int64_t)(g + 16 * k) * stride_w);
#pragma unroll
  for (int k = 0; k < 16; ++k) s += v[k];
  __shared__ f32x4 red[16][64];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0) {
    for (int q = 1; q < 16; ++q) s += red[q][lane];
    *reinterpret_cast<f32x4*>(out + (int64_t)c * 256 + 4 * lane) = s;
  }
}

__global__ __launch_bounds__(1024) void k_chain(int steps, float* out) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float a = 1e-3f * (threadIdx.x & 15), b = 1e-3f * (threadIdx.x >> 4);
  for (int s = 0; s < steps; ++s) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    a += 1e-7f;
  }
  if (acc[0] == 12345.f) out[threadIdx.x] = acc[1];
}

int main() {
  const int nch = 145, nwg = 256, reps = 21;
  const int64_t P = (int64_t)nch * 256;
  float *slab, *out;
  (void)hipMalloc(&slab, sizeof(float) * P * nwg);
  (void)hipMalloc(&out, sizeof(float) * P + 4096);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1, fork, join;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&join, hipEventDisableTiming);
  const int steps = 256;  // ~4 us of MFMA chain per wave at 4 waves per SIMD
  for (int nc : {64, 110, 256}) {
    auto A = [&](hipStream_t s) { hipLaunchKernelGGL(k_read, dim3(nch), dim3(1024), 0, s, slab, nwg, P, out); };
    auto C = [&](hipStream_t s) { hipLaunchKernelGGL(k_chain, dim3(nc), dim3(1024), 0, s, steps, out + P); };
    auto timed = [&](auto body) {
      float tot = 0.f;
      for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s1, slab, P * nwg);
        (void)hipEventRecord(e0, s1);
        body();
        (void)hipEventRecord(e1, s1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r > 0) tot += ms;
      }
      return tot / (reps - 1) * 1e3f;
    };
    const float ta = timed([&] { A(s1); });
    const float tc = timed([&] { C(s1); });
    const float tser = timed([&] {
      A(s1);
      C(s1);
    });
    const float tpar = timed([&] {
      (void)hipEventRecord(fork, s1);
      (void)hipStreamWaitEvent(s2, fork, 0);
      C(s2);
      A(s1);
      (void)hipEventRecord(join, s2);
      (void)hipStreamWaitEvent(s1, join, 0);
    });
    // the same fork/join captured as one graph with two branches
    hipGraph_t g;
    hipGraphExec_t x;
    (void)hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
    (void)hipEventRecord(fork, s1);
    (void)hipStreamWaitEvent(s2, fork, 0);
    C(s2);
    A(s1);
    (void)hipEventRecord(join, s2);
    (void)hipStreamWaitEvent(s1, join, 0);
    (void)hipStreamEndCapture(s1, &g);
    (void)hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    const float tgr = timed([&] { (void)hipGraphLaunch(x, s1); });
    (void)hipGraphExecDestroy(x);
    (void)hipGraphDestroy(g);
    printf("chain grid %3d: A alone %6.2f us, C alone %6.2f, A;C %6.2f, A||C streams %6.2f, A||C graph %6.2f\n", nc, ta,
           tc, tser, tpar, tgr);
  }
  return 0;
}
