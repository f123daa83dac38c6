// mdp_apply_fused.hip -- one launch for the batch reduction + optimizer step
// of one net (single-GPU path; with world_size > 1 the reduced gradient must
// be materialised for the RCCL all-reduce, so k_reduce -> all-reduce -> k_apply
// stay separate).
//
// Workgroup (tensor t, chunk c) of 256 parameters, 1024 threads: 16 groups of
// 64 threads each sum a quarter-ish of the per-workgroup partial gradients of
// the chunk (float4 columns), combined in LDS in a fixed order (deterministic).
// clip_by_norm needs the norm of the WHOLE tensor (tf_util.py:177-182): every
// chunk publishes its fp64 sum of squares with an agent-scope store, drains it
// and bumps the tensor's counter; all chunks of the tensor wait for the counter
// and sum the published partials in chunk order, so every chunk derives the
// identical norm.  Counters grow monotonically (target = next multiple of the
// chunk count, from the value the add returned), so they never need a reset.
// The grid (<= a few dozen workgroups) is always co-resident; every spin is
// bounded and records a fault in Ctl instead of hanging.
//
// Then TF1 ApplyAdam on the chunk (+ Polyak of the chunk for the actor step),
// Polyak workgroups of the other net, the stats workgroup -- exactly as k_apply
// -- and the last workgroup to finish advances the beta powers (the
// AdamOptimizer._finish update) and, for the actor step, the noise counter.
#include "mdp_device.h"
#include "mdp_kernels.h"
#include "mdp_ra.h"

__global__ __launch_bounds__(1024) void k_reduce_apply(FusedApplyArgs f) {
  ra_block<1024>(f, blockIdx.x, gridDim.x, 0, nullptr);
}

hipError_t mdp_launch_reduce_apply(const FusedApplyArgs& f, hipStream_t s) {
  const ApplyArgs& a = f.ap;
  const int grid = f.rblk[6] + (a.polyak ? a.oblk[6] : 0) + (a.stats_mode ? 1 : 0);
  hipLaunchKernelGGL(k_reduce_apply, dim3(grid), dim3(1024), 0, s, f);
  return hipGetLastError();
}
