// mdp_queue.h -- the weight-chunk stream of the general (H >= 64) layer phases:
// TileJob, rg_load / rg_acc (one 16-B load per lane and k-row feeding 4 MFMA
// tiles) and fwd_phase_l12 (layer 1 + layer 2 of independent nets as one
// work-queue phase), used by mdp_grads.hip (the gradient kernels).
#pragma once
#include "mdp_device.h"

#ifndef MDP_GKS
#define MDP_GKS 8  // k-steps (of 4) per weight chunk of the grouped layer phases
#endif

namespace {
// A layer phase: several dense layers Y = relu(X W + b) (all N = H wide) of
// independent nets, dealt over the waves (fwd_phase_grouped).  Job q -> (X, K,
// W, b, Y) comes from `job`, as LDS offsets and global pointers.
struct TileJob {
  int xoff, ldx, K;   // X = lds + xoff; k rows k0 .. K-1 of X and W (a split-K slice: k0 > 0 or K short)
  int k0;
  const float* W;     // [K][N] global
  const float* b;     // null: store the raw accumulator (a partial sum over K, no bias / ReLU)
  int yoff;           // Y = lds + yoff (row stride ldy)
};
// Unit (job, g) owns output columns
// 64 g .. 64 g + 63 as 4 MFMA tiles with a permuted column map (tile t, lane
// column r <-> column 64 g + 4 r + t), so ONE 16-byte load per lane and k-row
// feeds all 4 tiles: 4x fewer load instructions and 4x the MFMAs per byte in
// flight of the 16-column version.  Units are dealt round-robin over the
// waves; each walks its 4 KS-deep k-steps per chunk with the next chunk (of
// this unit or of the wave's next unit) in flight.
// rows k >= K: the clamped (finite) row K-1 is loaded and the A operand of
// that row is zeroed in rg_acc -- no select on the loaded value, which would
// make the wave wait for the prefetch right where it is issued
template <int KS>
__device__ __forceinline__ void rg_load(f32x4 (&w)[KS], const float* __restrict__ W, int N, int col4, int c0, int K,
                                        int kq) {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = c0 + 4 * s + kq;
    w[s] = *reinterpret_cast<const f32x4*>(W + (int64_t)min(k, K - 1) * N + col4);
  }
}
template <int KS>
__device__ __forceinline__ void rg_acc(f32x4 (&acc)[4], const float* X, int ldx, int r, int c0, int K, int kq,
                                       const f32x4 (&w)[KS]) {
  float x[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = X[r * ldx + min(k, K - 1)];
    x[s] = k < K ? v : 0.f;
  }
  __builtin_amdgcn_sched_barrier(0);  // every A read ahead of the MFMA chain
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (c0 + 4 * s < K) {  // wave-uniform
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], w[s][t], acc[t], 0, 0, 0);
    }
  }
}

// Layer 1 and layer 2 of independent nets as ONE phase fed by a work queue.
// Waves take 64-column units from an LDS counter in the order
//   layer 1 of the long jobs (listed first by the caller: the critic, K = cin,
//   and the target critic's obs' part, K = sum_obs), layer 1 of the target
//   actors, layer 2 of the target actors, layer 2 of the critic,
// and a layer-2 unit of net q waits only for net q's layer-1 units (cnt[q]
// reaches `want`), not for a workgroup barrier.  Stamped at tag N=6, H=128:
// with the two layers as separate barrier phases, 12 waves finished layer 1 at
// ~3.5 us while the long chains ran to 8.4 us; with a static deal of the fused
// phase the waves holding the long chains still carried 9 of the 88 chunks
// (5.5 per wave on average) -- every chunk costs ~2 us once all 16 waves
// stream (the per-CU weight-stream ceiling), so the phase is set by the most
// loaded wave.  No deadlock: layer-1 units wait for nothing and every one is
// taken before any layer-2 unit.  job(layer, j) -> TileJob; L1 job j1(q) and
// net index net1(q) come from the caller's order.  Ping-pong chunk stream as
// fwd_phase_grouped.
template <class JobFn, class OrdFn>
__device__ __forceinline__ void fwd_phase_l12(float* lds, int nj1, int nj2, int N, int ldy, int* cnt, int* qctr,
                                              int want, JobFn job, OrdFn ord) {
  constexpr int KS = MDP_GKS;
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, kq = lane >> 4, ngr = N >> 6, t1 = nj1 * ngr, tot = t1 + nj2 * ngr;
  struct It {
    int layer, net, g, c0;
    TileJob j;
#if defined(MDP_STAMPS) && defined(MDP_QUEUE_TRACE)
    unsigned long long t0;
#endif
  };
  // next unit from the queue (one LDS atomic per unit, lane 0, broadcast)
  auto take = [&](It& it) -> bool {
    int q = 0;
    if (lane == 0) q = __hip_atomic_fetch_add(qctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    q = __builtin_amdgcn_readfirstlane(q);
    if (q >= tot) return false;
    it.layer = q < t1 ? 0 : 1;
    const int qq = q < t1 ? q : q - t1;
    const int jb = it.layer == 0 ? ord(qq / ngr) : qq / ngr;  // layer 2: the caller's job order (actors, critic)
    it.net = jb;
    it.j = job(it.layer, jb);
    it.g = qq % ngr;
    it.c0 = it.j.k0;
#if defined(MDP_STAMPS) && defined(MDP_QUEUE_TRACE)
    it.t0 = __builtin_amdgcn_s_memrealtime();
#endif
    return true;
  };
  auto next = [&](It& it) -> bool {
    const int c2 = it.c0 + 4 * KS;
    if (c2 < it.j.K) {
      it.c0 = c2;
      return true;
    }
    return take(it);
  };
  It a;
  if (!take(a)) return;
  f32x4 wa[KS], wb[KS], ba = {0.f, 0.f, 0.f, 0.f}, bb = ba;
  auto load = [&](f32x4(&w)[KS], f32x4& bias, const It& it) {
    rg_load<KS>(w, it.j.W, N, 64 * it.g + 4 * r, it.c0, it.j.K, kq);
    if (it.j.b) bias = *reinterpret_cast<const f32x4*>(it.j.b + 64 * it.g + 4 * r);
  };
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](const It& it, const f32x4(&w)[KS], const f32x4& bias) {
    if (it.layer == 1 && it.c0 == it.j.k0) lds_wait(cnt + it.net, want);
    rg_acc<KS>(acc, lds + it.j.xoff, it.j.ldx, r, it.c0, it.j.K, kq, w);
    if (it.c0 + 4 * KS >= it.j.K) {  // unit done: bias, ReLU, scatter the 4 tiles' columns
      float* Y = lds + it.j.yoff + 64 * it.g + 4 * r;
      if (it.j.b) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int t = 0; t < 4; ++t) Y[(kq * 4 + i) * ldy + t] = fmaxf(acc[t][i] + bias[t], 0.f);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int t = 0; t < 4; ++t) Y[(kq * 4 + i) * ldy + t] = acc[t][i];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (it.layer == 0) lds_signal(cnt + it.net);
#if defined(MDP_STAMPS) && defined(MDP_QUEUE_TRACE)
      if (blockIdx.x == 0 && lane == 0) {
        const unsigned q = atomicAdd(&g_q_n, 1u);
        if (q < 160) {
          g_q_trace[q][0] = threadIdx.x >> 6;
          g_q_trace[q][1] = (unsigned long long)(it.layer << 8 | it.net);
          g_q_trace[q][2] = it.g;
          g_q_trace[q][3] = it.t0;
          g_q_trace[q][4] = __builtin_amdgcn_s_memrealtime();
        }
      }
#endif
    }
  };
  load(wa, ba, a);
  while (true) {
    It b = a;
    const bool hb = next(b);
    if (hb) load(wb, bb, b);
    step(a, wa, ba);
    if (!hb) break;
    It c = b;
    const bool hc = next(c);
    if (hc) load(wa, ba, c);
    step(b, wb, bb);
    if (!hc) break;
    a = c;
  }
}

}  // namespace
