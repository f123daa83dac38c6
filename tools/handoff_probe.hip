// handoff_probe.hip -- how fast can workgroups of ONE launch hand a freshly
// written parameter block to other workgroups of the same launch on gfx950?
// (measurement tool, not part of the library)
//
// The question behind it: an optimizer launch (~40 workgroups reduce, clip and
// Adam-step a net) followed by a gradient launch whose workgroups need only a
// small part of the stepped net (the updated target actor, 5.6K floats at S2)
// costs a kernel boundary (~1.7 us measured, tools/timeline.py) plus the
// consumer's load prologue.  Merged into one launch, the consumers could
// prefetch everything else while the producers work, then wait on a counter.
//
// One launch: P producer workgroups spin `work` us (the optimizer's body), then
// each writes its 256-float slice of the block, waits for its stores, and adds
// 1 to a counter; C consumer workgroups first stream `pre` KiB of unrelated
// data (their own prologue), then poll the counter until all P arrived, then
// load the WHOLE block and check it.  Memory flavours (mode):
//   0  stores and loads both sc0 sc1 (__hip_atomic_*, system scope)
//   1  plain stores + agent release fence on the producer; agent acquire
//      fence + plain loads on the consumer
//   2  stores sc0 sc1, loads sc1 (agent-scope atomic loads)
// Printed (medians over reps, us, from the launch's first workgroup start):
// last producer add, consumers' counter seen (median / max), block loaded
// (median / max), and mismatches (stale reads).
//   hipcc -O3 --offload-arch=gfx950 tools/handoff_probe.hip -o tools/handoff_probe_bin
//   tools/handoff_probe_bin [mode=0] [P=40] [C=64] [work_us=3] [pre_kib=48] [reps=50]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Args {
  float* block;                 // [P * 256]
  const float* pre;             // consumers' unrelated prologue data
  uint32_t* ctr;
  uint32_t* bad;
  uint32_t* fault;
  unsigned long long* t;        // [grid][3]
  int P, C, mode, pre_floats;
  uint32_t epoch;
  unsigned long long work_ticks;
};

__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(512) void k_handoff(Args a) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int b = blockIdx.x, tid = threadIdx.x;
  unsigned long long t1 = 0, t2 = 0;
  if (b < a.P) {
    // producer: the optimizer's body, then this workgroup's slice
    while (__builtin_amdgcn_s_memrealtime() - t0 < a.work_ticks) __builtin_amdgcn_s_sleep(1);
    if (tid < 256) {
      const float v = (float)(a.epoch * 1000u + (uint32_t)(b * 256 + tid) % 1000u);
      float* p = a.block + b * 256 + tid;
      if (a.mode == 1) *p = v;
      else st_sys(p, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      if (a.mode == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t1 = __builtin_amdgcn_s_memrealtime();
    }
  } else {
    // consumer: its own prologue (unrelated data), then the wait and the block
    float acc = 0.f;
    for (int i = tid; i < a.pre_floats; i += 512) acc += a.pre[i];
    __shared__ int seen;
    if (tid == 0) {
      uint32_t it = 0;
      const uint32_t want = (uint32_t)a.P * a.epoch;
      while (__hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1u << 20)) {
          __hip_atomic_store(a.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (a.mode == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      t1 = __builtin_amdgcn_s_memrealtime();
      seen = 1;
    }
    __syncthreads();
    (void)seen;
    uint32_t nbad = 0;
    for (int i = tid; i < a.P * 256; i += 512) {
      float v;
      if (a.mode == 0) v = __hip_atomic_load(a.block + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else if (a.mode == 2) v = __hip_atomic_load(a.block + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else v = a.block[i];
      const float want = (float)(a.epoch * 1000u + (uint32_t)i % 1000u);
      nbad += v != want ? 1u : 0u;
      acc += v;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    t2 = __builtin_amdgcn_s_memrealtime();
    if (nbad) atomicAdd(a.bad, nbad);
    if (acc == 12345.f) a.bad[1] = 1;  // keep the prologue loads
  }
  if (tid == 0) {
    a.t[b * 3 + 0] = t0;
    a.t[b * 3 + 1] = t1;
    a.t[b * 3 + 2] = t2;
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int P = argc > 2 ? atoi(argv[2]) : 40;
  const int C = argc > 3 ? atoi(argv[3]) : 64;
  const double work_us = argc > 4 ? atof(argv[4]) : 3.0;
  const int pre_kib = argc > 5 ? atoi(argv[5]) : 48;
  const int reps = argc > 6 ? atoi(argv[6]) : 50;
  const int grid = P + C;
  Args a{};
  CHK(hipMalloc(&a.block, sizeof(float) * P * 256));
  float* pre;
  const int pre_floats = pre_kib * 256;
  CHK(hipMalloc(&pre, sizeof(float) * std::max(pre_floats, 1)));
  CHK(hipMemset(pre, 0, sizeof(float) * std::max(pre_floats, 1)));
  a.pre = pre;
  CHK(hipMalloc(&a.ctr, 4));
  CHK(hipMalloc(&a.bad, 8));
  CHK(hipMalloc(&a.fault, 4));
  CHK(hipMalloc(&a.t, sizeof(unsigned long long) * grid * 3));
  CHK(hipMemset(a.ctr, 0, 4));
  CHK(hipMemset(a.bad, 0, 8));
  CHK(hipMemset(a.fault, 0, 4));
  a.P = P;
  a.C = C;
  a.mode = mode;
  a.pre_floats = pre_floats;
  a.work_ticks = (unsigned long long)(work_us * 100.0);
  std::vector<double> last_add, seen_med, seen_max, load_med, load_max;
  std::vector<unsigned long long> h(grid * 3);
  for (int r = 0; r < reps; ++r) {
    a.epoch = (uint32_t)(r + 1);
    hipLaunchKernelGGL(k_handoff, dim3(grid), dim3(512), 0, 0, a);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h.data(), a.t, sizeof(unsigned long long) * grid * 3, hipMemcpyDeviceToHost));
    unsigned long long s0 = ~0ull, la = 0;
    for (int b = 0; b < grid; ++b) s0 = std::min(s0, h[b * 3]);
    for (int b = 0; b < P; ++b) la = std::max(la, h[b * 3 + 1]);
    std::vector<double> sn, ld;
    for (int b = P; b < grid; ++b) {
      sn.push_back((h[b * 3 + 1] - s0) / 100.0);
      ld.push_back((h[b * 3 + 2] - s0) / 100.0);
    }
    last_add.push_back((la - s0) / 100.0);
    seen_med.push_back(med(sn));
    seen_max.push_back(*std::max_element(sn.begin(), sn.end()));
    load_med.push_back(med(ld));
    load_max.push_back(*std::max_element(ld.begin(), ld.end()));
  }
  uint32_t bad[2], fault;
  CHK(hipMemcpy(bad, a.bad, 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&fault, a.fault, 4, hipMemcpyDeviceToHost));
  printf("mode %d P %d C %d work %.1f us pre %d KiB: last producer add %.2f | counter seen med %.2f max %.2f | "
         "block loaded med %.2f max %.2f | stale %u fault %u\n",
         mode, P, C, work_us, pre_kib, med(last_add), med(seen_med), med(seen_max), med(load_med), med(load_max),
         bad[0], fault);
  return 0;
}
