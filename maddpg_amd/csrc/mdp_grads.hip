// mdp_grads.hip -- per-agent critic-step and actor-step gradient kernels (gfx950),
// general topology: H = 64 or 128, up to 8 agents, wide critic inputs (BASELINE
// configs[4]: simple_tag N=6, H=128, B=4096).  The register-resident kernels
// of mdp_grads_r.hip serve H = 64 with <= 3 target actors.
//
// One 1024-thread workgroup (16 waves) owns 16 batch rows; the reduction over
// the batch happens in k_reduce_apply from per-workgroup partials
// (deterministic).  Every dense layer is spread over ALL 16 waves as MFMA
// tiles with the next weight chunk in flight: single-net layers as 16-column
// tiles (fwd_tile / dgrad_tile_relu), the phases of independent nets (target
// actors + critic) as 64-column groups fed by 16-byte weight loads
// (fwd_phase_grouped), dealt round-robin over the waves with no barrier
// between nets, so a wave's load latency is covered by the other waves on its
// SIMD (4 per SIMD at 1024 threads).  (The
// earlier design ran one whole net per wave: at H = 128 a wave then waited on
// ~600 MFMAs and every weight chunk in turn -- the target critic alone took
// 21 us of a 98 us critic step.)
//
// k_critic_grad (maddpg.py:180-188):
//   gather | L1 tiles of the target actors (+ critic) || L2 tiles || heads, Gumbel a~
//   || target critic L1 || L2 || wave 0: head, fp64 TD, loss, dL/dq
//   || dW3, db3, d2 || dh1 tiles + dW2 tiles || dW1, db1
// k_actor_grad (maddpg.py:37-58):
//   gather | actor L1 || L2 || head, Gumbel a_i, critic input || critic L1 || L2
//   || head q, d2 || dh1c tiles || da, softmax backward + reg (wave 0)
//   || dW3a, db3a, d2a || dh1a tiles + dW2a tiles || dW1a, db1a
#include "mdp_device.h"
#include "mdp_kernels.h"

#ifndef MDP_SPLITK
#define MDP_SPLITK 1  // max k-slices of the long layer-1 jobs of the critic kernel (<= 1: off; 3 measured: no gain)
#endif
#ifndef MDP_GEN_THREADS
#define MDP_GEN_THREADS 1024  // 16 waves: 4 per SIMD to cover the weight-chunk latency
#endif

#ifdef MDP_STAMPS
// diagnostic: the layer work queue's units of workgroup 0 (critic kernel, first
// pass): [unit][wave, layer << 8 | net, g, t_take, t_done] (s_memrealtime)
__device__ unsigned long long g_q_trace[160][5];
__device__ unsigned int g_q_n;
#define MDP_QUEUE_TRACE 1
#endif
#include "mdp_queue.h"
namespace {
// Y[16][col tile nt] = act(X[16][K] @ W[K][N] + b), weights in 64-deep chunks, the next in flight
template <bool RELU>
__device__ __forceinline__ void fwd_tile(const float* X, int ldx, int K, const float* __restrict__ W,
                                         const float* __restrict__ b, int N, float* Y, int ldy, int nt) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int col = nt * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float wa[MDP_KC], wb[MDP_KC];
  load_wchunk(wa, W, N, col, 0, K, kq);
  const float bias = b[col];
  for (int c0 = 0; c0 < K; c0 += 4 * MDP_KC) {
    const bool more = c0 + 4 * MDP_KC < K;
    if (more) load_wchunk(wb, W, N, col, c0 + 4 * MDP_KC, K, kq);
    acc = mfma_chunk(acc, wa, X, ldx, r, c0, K, kq);
    if (more) {
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s) wa[s] = wb[s];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = acc[i] + bias;
    if (RELU) v = fmaxf(v, 0.f);
    Y[(kq * 4 + i) * ldy + col] = v;
  }
}

// The chunks ping-pong between two register sets with the loop unrolled by
// two: the next chunk's loads are issued before the wait for the current one,
// so two chunks are in flight during a wait, and the compiler waits for exactly
// the chunk it is about to use.  (A copy wa = wb of the prefetch buffer at the
// end of each iteration made the wave wait there for every load in flight:
// one chunk in flight at a time.)  Each chunk load also fetches the unit's
// bias, so the store at a unit's end does not wait behind the prefetch.
template <class JobFn>
__device__ __forceinline__ void fwd_phase_grouped(float* lds, int njobs, int N, int ldy, JobFn job) {
  constexpr int KS = MDP_GKS;  // k-steps (of 4) per chunk
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int r = lane & 15, kq = lane >> 4, ngr = N >> 6, total = njobs * ngr;
  struct It {
    int u, g, c0;
    TileJob j;
  };
  It a;
  a.u = wave;
  if (a.u >= total) return;
  a.j = job(a.u / ngr);
  a.g = a.u % ngr;
  a.c0 = a.j.k0;
  auto next = [&](It& it) -> bool {
    const int c2 = it.c0 + 4 * KS;
    if (c2 < it.j.K) {
      it.c0 = c2;
      return true;
    }
    it.u += nw;
    if (it.u >= total) return false;
    it.j = job(it.u / ngr);
    it.g = it.u % ngr;
    it.c0 = it.j.k0;
    return true;
  };
  f32x4 wa[KS], wb[KS], ba = {0.f, 0.f, 0.f, 0.f}, bb = ba;
  auto load = [&](f32x4(&w)[KS], f32x4& bias, const It& it) {
    rg_load<KS>(w, it.j.W, N, 64 * it.g + 4 * r, it.c0, it.j.K, kq);
    if (it.j.b) bias = *reinterpret_cast<const f32x4*>(it.j.b + 64 * it.g + 4 * r);
  };
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](const It& it, const f32x4(&w)[KS], const f32x4& bias) {
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

// fwd_tile continued from a partial: Y tile = act(init + X[:, k0:K] W[k0:K, :] + b),
// init[16][ldi] the raw accumulator of X[:, 0:k0] W[0:k0, :] (same MFMA k order as
// one chain over 0..K, so the result is bit-identical to fwd_tile)
template <bool RELU>
__device__ __forceinline__ void fwd_tile_from(const float* X, int ldx, int k0, int K, const float* __restrict__ W,
                                              const float* __restrict__ b, int N, const float* init, int ldi,
                                              float* Y, int ldy, int nt) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int col = nt * 16 + r;
  f32x4 acc;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = init[(kq * 4 + i) * ldi + col];
  float wa[MDP_KC], wb[MDP_KC];
  load_wchunk(wa, W, N, col, k0, K, kq);
  const float bias = b[col];
  for (int c0 = k0; c0 < K; c0 += 4 * MDP_KC) {
    const bool more = c0 + 4 * MDP_KC < K;
    if (more) load_wchunk(wb, W, N, col, c0 + 4 * MDP_KC, K, kq);
    acc = mfma_chunk(acc, wa, X, ldx, r, c0, K, kq);
    if (more) {
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s) wa[s] = wb[s];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = acc[i] + bias;
    if (RELU) v = fmaxf(v, 0.f);
    Y[(kq * 4 + i) * ldy + col] = v;
  }
}

// Prefetched single-net layers: `wa` holds the first 64-deep weight chunk of
// this wave's tile (nt), issued by the caller AHEAD -- before the barrier that
// precedes the layer, behind heads, Gumbel sampling and TD on other waves -- so
// the layer starts on weights already in registers instead of paying a round
// trip after the barrier.  One tile per wave (nt = wave < N / 16).
__device__ __forceinline__ void pf_load(float (&wa)[MDP_KC], const float* __restrict__ W, int N, int nt, int k0, int K) {
  const int lane = threadIdx.x & 63;
  load_wchunk(wa, W, N, nt * 16 + (lane & 15), k0, K, lane >> 4);
}
// Transposed operand of dX = dY @ W^T (W[K][N] row-major, N a multiple of 64):
// output column kk = row kk of W, contraction order n = c0 + 16 kq + s within a
// 64-deep chunk, so a lane's 16 fragments are 64 contiguous bytes of row kk --
// four 16-B loads instead of sixteen strided 4-B ones (n = c0 + 4 s + kq)
__device__ __forceinline__ void load_wchunk_tc(f32x4 (&w)[4], const float* __restrict__ W, int N, int kk, int c0,
                                               int kq) {
#pragma unroll
  for (int m = 0; m < 4; ++m) w[m] = *reinterpret_cast<const f32x4*>(W + (int64_t)kk * N + c0 + 16 * kq + 4 * m);
}
__device__ __forceinline__ f32x4 mfma_chunk_tc(f32x4 acc, const f32x4 (&w)[4], const float* A, int lda, int r, int c0,
                                               int kq) {
  float x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = A[r * lda + c0 + 16 * kq + q];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 16; ++q) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[q], w[q >> 2][q & 3], acc, 0, 0, 0);
  return acc;
}
__device__ __forceinline__ void pf_load_t(f32x4 (&wa)[4], const float* __restrict__ W, int N, int nt) {
  const int lane = threadIdx.x & 63;
  load_wchunk_tc(wa, W, N, nt * 16 + (lane & 15), 0, lane >> 4);
}
// Y tile = act([init +] X[:, k0:K] W[k0:K, :] + b); init (raw accumulator of the
// rows before k0, same MFMA k order as one chain) may be null.  DEEP: with at
// most three 64-deep chunks, the second and third are requested together at
// entry (one round trip after the prefetched first, not two); same chain.
template <bool RELU, bool DEEP = false>
__device__ __forceinline__ void fwd_tile_pf(const float* X, int ldx, int k0, int K, const float* __restrict__ W,
                                            const float* __restrict__ b, int N, const float* init, int ldi, float* Y,
                                            int ldy, int nt, float (&wa)[MDP_KC]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int col = nt * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (init) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = init[(kq * 4 + i) * ldi + col];
  }
  const float bias = b[col];
  float wb[MDP_KC];
  constexpr int D = 4 * MDP_KC;
  if (DEEP && K - k0 <= 3 * D) {
    float wc[MDP_KC];
    if (k0 + D < K) load_wchunk(wb, W, N, col, k0 + D, K, kq);
    if (k0 + 2 * D < K) load_wchunk(wc, W, N, col, k0 + 2 * D, K, kq);
    acc = mfma_chunk(acc, wa, X, ldx, r, k0, K, kq);
    if (k0 + D < K) acc = mfma_chunk(acc, wb, X, ldx, r, k0 + D, K, kq);
    if (k0 + 2 * D < K) acc = mfma_chunk(acc, wc, X, ldx, r, k0 + 2 * D, K, kq);
  } else
  for (int c0 = k0; c0 < K; c0 += 4 * MDP_KC) {
    const bool more = c0 + 4 * MDP_KC < K;
    if (more) load_wchunk(wb, W, N, col, c0 + 4 * MDP_KC, K, kq);
    acc = mfma_chunk(acc, wa, X, ldx, r, c0, K, kq);
    if (more) {
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s) wa[s] = wb[s];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = acc[i] + bias;
    if (RELU) v = fmaxf(v, 0.f);
    Y[(kq * 4 + i) * ldy + col] = v;
  }
}
// mfma_chunk with the columns [z_lo, z_hi) of A read as zero (the actor
// step's critic layer 1 before its a_i input exists)
__device__ __forceinline__ f32x4 mfma_chunk_zc(f32x4 acc, const float (&w)[MDP_KC], const float* A, int lda, int r,
                                               int c0, int K, int kq, int z_lo, int z_hi) {
  const int kmax = K > 0 ? K - 1 : 0;
  float x[MDP_KC];
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = A[r * lda + min(k, kmax)];
    x[s] = (k < K && (k < z_lo || k >= z_hi)) ? v : 0.f;
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    if (c0 + 4 * s < K)  // wave-uniform
      acc = MDP_MFMA(x[s], w[s], acc);
  }
  return acc;
}

// dX tile nt = (dY[16][N] @ W^T) masked by Hin > 0 (N a multiple of 64), first
// chunk of W^T in wa (pf_load_t); contiguous transposed fragments (load_wchunk_tc)
__device__ __forceinline__ void dgrad_tile_relu_pf(const float* dY, int ldy, int N, const float* __restrict__ W,
                                                   const float* Hin, int ldh, float* dX, int ldx, int nt,
                                                   f32x4 (&wa)[4]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int kk = nt * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 wb[4];
  for (int c0 = 0; c0 < N; c0 += 64) {
    const bool more = c0 + 64 < N;
    if (more) load_wchunk_tc(wb, W, N, kk, c0 + 64, kq);
    acc = mfma_chunk_tc(acc, wa, dY, ldy, r, c0, kq);
    if (more) {
#pragma unroll
      for (int m = 0; m < 4; ++m) wa[m] = wb[m];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = kq * 4 + i;
    dX[row * ldx + kk] = Hin[row * ldh + kk] > 0.f ? acc[i] : 0.f;
  }
}

// dX[16][tile nt of K] = (dY[16][N] @ W^T) masked by Hin > 0, W[K][N] global
__device__ __forceinline__ void dgrad_tile_relu(const float* dY, int ldy, int N, const float* __restrict__ W,
                                                const float* Hin, int ldh, float* dX, int ldx, int nt) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int kk = nt * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float wa[MDP_KC], wb[MDP_KC];
  load_wchunk_t(wa, W, N, kk, 0, N, kq, true);
  for (int c0 = 0; c0 < N; c0 += 4 * MDP_KC) {
    const bool more = c0 + 4 * MDP_KC < N;
    if (more) load_wchunk_t(wb, W, N, kk, c0 + 4 * MDP_KC, N, kq, true);
    acc = mfma_chunk(acc, wa, dY, ldy, r, c0, N, kq);
    if (more) {
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s) wa[s] = wb[s];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = kq * 4 + i;
    dX[row * ldx + kk] = Hin[row * ldh + kk] > 0.f ? acc[i] : 0.f;
  }
}

// dW[K][N] tile t = (mt, nt) of X^T[K][16] @ dY[16][N], to global (stride N); rows >= K not written
__device__ __forceinline__ void wgrad_tile(const float* X, int ldx, int K, const float* dY, int ldy, int N,
                                           float* __restrict__ dW, int t) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int nnt = N >> 4, mt = t / nnt, nt = t - mt * nnt;
  const int feat = mt * 16 + r;
  const int fc = min(feat, K - 1);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r0 = 0; r0 < MDP_R; r0 += 4) {
    const int row = r0 + kq;
    const float xv = X[row * ldx + fc];
    const float a = feat < K ? xv : 0.f;
    const float g = dY[row * ldy + nt * 16 + r];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(g, a, acc, 0, 0, 0);  // transposed tile (slab_st4)
  }
  if (feat < K) slab_st4(dW + feat * N + nt * 16 + kq * 4, acc);
}
}  // namespace

static_assert(MDP_GEN_THREADS / 64 >= MDP_MAX_UNITS / 16, "one single-net layer tile per wave (pf_load / *_pf)");

// blk: this workgroup's row tile (blockIdx.x, or its index inside the
// critic half of a gradient-pair launch)
template <int H>
__device__ __forceinline__ void critic_body(const CriticArgs& a, const Topo& T, const int blk) {
  // (no MDP_KARG_TOUCH here: at H = 128 it turned the kernel's 47 spilled
  // SGPRs into 91 spilled VGPRs)
  constexpr int NT = H / 16;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const ADesc& ag = T.ag[a.agent];
  const int G = a.group;
  const int ldr = lds_ld(T.row_stride), ldc = lds_ld(T.cin_max), ldh = H + 1;
  const int S = MDP_R * ldh;  // one activation slot
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* xt = cv.take(MDP_R * ldc);
  float* xl = cv.take(MDP_R * ldc);
  float* hA = cv.take((G + 1) * S);
  float* hB = cv.take((G + 1) * S);
  float* lg = cv.take((G + 1) * MDP_R * 8);
  float* dq = cv.take(MDP_R);
  int* cnt = reinterpret_cast<int*>(cv.take(MDP_MAX_AGENTS + 4));  // layer-1 units done per net, then the
                                                                    // work-queue counter (fwd_phase_l12)

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = blockDim.x >> 6;
  const int r0 = blk * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const bool lq = ag.local_q != 0;
  // throughput mode (multi > 1: one launch per agent, every agent from the
  // round-start parameters) draws agent i's noise at upd_ctr + i, as the fast kernels
  const uint32_t ctr = a.ctl->upd_ctr + (a.multi > 1 ? (uint32_t)a.agent : 0u);
  const NDesc& nd = ag.critic;
  float* h1c = hA + G * S;
  float* h2c = hB + G * S;
  float* qv = lg + G * MDP_R * 8;
  float pf[MDP_KC];  // this wave's next single-net layer chunk, issued ahead (wave < NT)
  f32x4 pft[4];      // the backward's first W^T chunk, issued ahead
  constexpr int HKS = H / 4 <= 32 ? H / 4 : 1;  // head fragments per lane (the target critic's, issued ahead)
  MDP_STAMP(0);

  gather_rows16(a.replay, T.row_stride, a.idx, r0, nvalid, rowbuf, ldr);
  __syncthreads();
  // target critic input: [obs'_all | a~_all] (global) or [obs'_i | a~_i] (local, maddpg.py:86-87)
  if (lq) {
    copy_cols16(rowbuf, ldr, ag.nobs_off, xt, ldc, 0, ag.obs_dim);
    copy_cols16(rowbuf, ldr, ag.obs_off, xl, ldc, 0, ag.obs_dim);
    copy_cols16(rowbuf, ldr, ag.act_off, xl, ldc, ag.obs_dim, MDP_ACT_DIM);
  } else {
    copy_cols16(rowbuf, ldr, T.ag[0].nobs_off, xt, ldc, 0, T.sum_obs);
  }
  if (tid < MDP_MAX_AGENTS + 4) cnt[tid] = 0;
  __syncthreads();
  const float* Xc = lq ? xl : rowbuf;  // critic input: the row prefix (global) or [obs_i | act_i]
  const int ldX = lq ? ldc : ldr;
  MDP_STAMP(1);

  // target actors of the group (+ the critic forward with the first group): each
  // layer phase deals every net's 16-column tiles over all waves
  const int nact = lq ? 1 : T.n;
  const int npass = (nact + G - 1) / G;
  // the target critic's obs' part of layer 1 (maddpg.py:86) does not depend on
  // the target actions: with the first layer-1 phase, raw, into xl (unused by a
  // MADDPG critic); only the a~ rows remain after the Gumbel sample
  const bool tpre = !lq && T.sum_obs % 4 == 0 && ldc >= ldh && MDP_R * ldc >= MDP_R * ldh;
  // Split-K of the first layer-1 phase: the two long-K jobs -- the critic (K =
  // cin, 158 at tag N=6) and the target critic's obs' part (K = sum_obs) -- ran
  // as one unit per 64-column group, a serial chain of ~5 weight chunks (one
  // round trip each) while the short target-actor units were done at 40 % of
  // the phase (stamped).  Here each is cut into sc / st slices of its k-steps,
  // dealt FIRST so they start at t = 0, with raw partials into hB (unused until
  // the layer-2 phase); the slices are summed in slice order (+ bias, ReLU for
  // the critic) right after the phase.
  int sc = 0, st = 0;
#if MDP_SPLITK > 1
  {
    const int kc = (ag.cin + 3) / 4, kt = (T.sum_obs + 3) / 4;  // k-steps
    sc = min(MDP_SPLITK, (kc + 2 * MDP_GKS - 1) / (2 * MDP_GKS));  // >= 2 chunks per slice
    st = tpre ? min(MDP_SPLITK, (kt + 2 * MDP_GKS - 1) / (2 * MDP_GKS)) : 0;
    while (sc + st > G + 1 && sc + st > 0) {
      if (sc >= st) --sc;
      else --st;
    }
    if (sc + st < 3 || sc < 1 || (tpre && st < 1)) sc = st = 0;  // nothing to gain
  }
#endif
  const bool split = sc > 0;
  for (int pass = 0; pass < npass; ++pass) {
    const int g0 = pass * G;
    const int ng = min(G, nact - g0);
    const int nj = ng + (g0 == 0 ? 1 : 0);
    const bool sp = split && g0 == 0;
    const int nj1 = sp ? sc + st + ng : nj + (g0 == 0 && tpre ? 1 : 0);  // layer-1 jobs
    const int o_row = (int)(rowbuf - lds), o_xc = (int)(Xc - lds), o_ha = (int)(hA - lds), o_hb = (int)(hB - lds);
    auto jobf = [&](int layer, int jb) -> TileJob {
        if (sp && layer == 0 && jb < sc + st) {  // a split-K slice, raw into hB slot jb
          const bool crit = jb < sc;
          const int q = crit ? jb : jb - sc, ns = crit ? sc : st;
          const int K = crit ? ag.cin : T.sum_obs, ks = (K + 3) / 4;
          TileJob j;
          j.xoff = crit ? o_xc : (int)(xt - lds);
          j.ldx = crit ? ldX : ldc;
          j.k0 = 4 * (q * ks / ns);
          j.K = min(K, 4 * ((q + 1) * ks / ns));
          j.W = crit ? a.theta + nd.t[0].off : a.target + nd.t[0].off;
          j.b = nullptr;
          j.yoff = o_hb + jb * S;
          return j;
        }
        if (sp && layer == 0) jb -= sc + st;  // then the target actors
        if (jb == nj) {  // layer 1 only: the target critic's obs' part
          TileJob j;
          j.xoff = (int)(xt - lds);
          j.ldx = ldc;
          j.k0 = 0;
          j.K = T.sum_obs;
          j.W = a.target + nd.t[0].off;
          j.b = nullptr;
          j.yoff = (int)(xl - lds);
          return j;
        }
        const bool actor = jb < ng;
        const ADesc& aj = T.ag[lq ? a.agent : g0 + jb];
        const NDesc& net = actor ? aj.actor : nd;
        const float* P = actor ? a.target : a.theta;
        const int slot = (actor ? jb : G) * S;
        TileJob j;
        j.k0 = 0;
        if (layer == 0) {
          j.xoff = actor ? o_row + aj.nobs_off : o_xc;
          j.ldx = actor ? ldr : ldX;
          j.K = actor ? aj.obs_dim : ag.cin;
          j.W = P + net.t[0].off;
          j.b = P + net.t[1].off;
          j.yoff = o_ha + slot;
        } else {
          j.xoff = o_ha + slot;
          j.ldx = ldh;
          j.K = H;
          j.W = P + net.t[2].off;
          j.b = P + net.t[3].off;
          j.yoff = o_hb + slot;
        }
        return j;
    };
    if (!sp && H >= 128) {  // layer 1 + layer 2 as one phase, per-net hand-off (fwd_phase_l12; at H = 64 it spills)
      // layer-1 order: the long jobs first (critic, the target critic's obs' part), then the actors
      const int nlong = nj1 - ng;
      fwd_phase_l12(lds, nj1, nj, H, ldh, cnt, cnt + MDP_MAX_AGENTS + 3, (H >> 6) * (pass + 1), jobf,
                    [&](int q) { return q < nlong ? ng + q : q - nlong; });
      if (g0 == 0) MDP_STAMPW(16 + wave);  // per-wave phase end (diagnostic build)
      __syncthreads();
      if (tid == 0) cnt[MDP_MAX_AGENTS + 3] = 0;  // the queue of the next group (barriers follow)
      if (g0 == 0) {
        MDP_STAMP(6);
        MDP_STAMP(7);
      }
    } else {
    for (int layer = 0; layer < 2; ++layer) {
      fwd_phase_grouped(lds, layer == 0 ? nj1 : nj, H, ldh, [&](int jb) { return jobf(layer, jb); });
      if (g0 == 0) MDP_STAMPW((layer == 0 ? 16 : 40) + wave);  // per-wave phase end (diagnostic build)
      __syncthreads();
      if (sp && layer == 0) {  // sum the slices in slice order: critic h1 = relu(sum + b1), obs' part raw
        const float* b1 = a.theta + nd.t[1].off;
        for (int e = tid; e < MDP_R * H; e += blockDim.x) {
          const int r = e / H, c = e - r * H, o = r * ldh + c;
          float v = hB[o];
          for (int q = 1; q < sc; ++q) v += hB[q * S + o];
          h1c[o] = fmaxf(v + b1[c], 0.f);
          if (st) {
            float w = hB[sc * S + o];
            for (int q = 1; q < st; ++q) w += hB[(sc + q) * S + o];
            xl[o] = w;
          }
        }
        __syncthreads();
      }
      if (g0 == 0) MDP_STAMP(6 + layer);
    }
    }
    // heads: net jb on wave jb % nw, then the Gumbel-softmax target actions
    for (int jb = wave; jb < nj; jb += nw) {
      if (jb < ng) {
        const NDesc& an = T.ag[lq ? a.agent : g0 + jb].actor;
        head_mfma<H / 4>(hB + jb * S, ldh, H, a.target + an.t[4].off, a.target + an.t[5].off, MDP_ACT_DIM,
                         lg + jb * MDP_R * 8, 8);
      } else {
        head_mfma<H / 4>(h2c, ldh, H, a.theta + nd.t[4].off, a.theta + nd.t[5].off, 1, qv, 8);
      }
    }
    __syncthreads();
    if (g0 == 0) MDP_STAMP(8);
    for (int e = tid; e < ng * MDP_R; e += blockDim.x) {  // distributions.py:264-266
      const int jb = e / MDP_R, row = e - jb * MDP_R;
      const int j = lq ? a.agent : g0 + jb;
      float u[MDP_ACT_DIM], act[MDP_ACT_DIM];
      if (a.u_tgt) {
        for (int k = 0; k < MDP_ACT_DIM; ++k)
          u[k] = row < nvalid ? a.u_tgt[((int64_t)j * a.B + r0 + row) * MDP_ACT_DIM + k] : 0.5f;
      } else {
        uniforms5(a.seed, (uint32_t)((a.agent << 8) | (j + 1)), ctr, (uint32_t)(r0 + row), u);
      }
      gumbel_softmax5(lg + jb * MDP_R * 8 + row * 8, u, act);
      const int dst = lq ? ag.obs_dim : T.sum_obs + MDP_ACT_DIM * j;
      for (int k = 0; k < MDP_ACT_DIM; ++k) xt[row * ldc + dst + k] = act[k];
    }
    __syncthreads();
  }
  MDP_STAMP(2);

  // target critic Q'(o', a~) over all waves; wave 0: head, fp64 TD target
  // (maddpg.py:186), loss partials, dL/dq = 2(q-y)/B
  float thw[HKS], thb = 0.f;  // the target critic's head fragments, issued with its layer 2 (wave 0)
  {
    const float* P = a.target;
    if (wave < NT) {  // (a prefetch of this layer across the layer phases would spill)
      pf_load(pf, P + nd.t[0].off, H, wave, tpre ? T.sum_obs : 0, ag.cin);
      fwd_tile_pf<true>(xt, ldc, tpre ? T.sum_obs : 0, ag.cin, P + nd.t[0].off, P + nd.t[1].off, H,
                        tpre ? xl : nullptr, ldh, hA, ldh, wave, pf);
      pf_load(pf, P + nd.t[2].off, H, wave, 0, H);
    }
    __syncthreads();
    if (wave < NT) {
      if (H / 4 <= 32 && wave == 0) head_load<HKS>(thw, thb, P + nd.t[4].off, P + nd.t[5].off, 1);
      fwd_tile_pf<true>(hA, ldh, 0, H, P + nd.t[2].off, P + nd.t[3].off, H, nullptr, 0, hB, ldh, wave, pf);
      pf_load_t(pft, a.theta + nd.t[2].off, H, wave);  // the backward's dh1 = d2 W2^T
    }
    __syncthreads();
  }
  // the dq * W3 backward below reads one W3 column per thread (the block is a
  // multiple of H wide): requested here, ahead of the TD-error phase, instead
  // of one dependent load per row pass after it
  static_assert(MDP_GEN_THREADS % H == 0, "d2 pass: fixed column per thread");
  const float w3h = a.theta[nd.t[4].off + tid % H];
  if (wave == 0) {
    const float* P = a.target;
    if constexpr (H / 4 <= 32) head_acc<HKS>(thw, thb, hB, ldh, 1, lg, 8);
    else head_mfma<H / 4>(hB, ldh, H, P + nd.t[4].off, P + nd.t[5].off, 1, lg, 8);
    wave_sync();
    double s_l = 0.0, s_y = 0.0, s_r = 0.0, s_q = 0.0;
    float g = 0.f;
    if (lane < nvalid) {
      const double rew = (double)rowbuf[lane * ldr + ag.rew_off];
      const double done = (double)rowbuf[lane * ldr + ag.done_off];
      const double qn = (double)lg[lane * 8];
      const double y64 = rew + a.gamma * (1.0 - done) * qn;
      const float y = (float)y64;
      const float diff = qv[lane * 8] - y;
      g = (2.0f * diff) * a.inv_b;
      s_l = (double)diff * (double)diff;
      s_y = y64;
      s_r = rew;
      s_q = qn;
      a.y_out[r0 + lane] = y64;
    }
    if (lane < MDP_R) dq[lane] = g;
    s_l = sum16(s_l);
    s_y = sum16(s_y);
    s_r = sum16(s_r);
    s_q = sum16(s_q);
    if (lane == 0) {
      double* st = a.slab_stat + (int64_t)blk * 8;
      st[0] = s_l;
      st[1] = s_y;
      st[2] = s_r;
      st[3] = s_q;
    }
  }
  __syncthreads();
  MDP_STAMP(3);

  // backward through the critic (tf.gradients of q_loss w.r.t. q_func vars)
  float* slab = a.slab + (int64_t)blk * a.slab_stride - nd.off;
  float* d2 = hA;
  float* d1 = hB;
  if (tid < H) {
    float s = 0.f;
    for (int r = 0; r < MDP_R; ++r) s = fmaf(h2c[r * ldh + tid], dq[r], s);
    slab[nd.t[4].off + tid] = s;
  }
  if (tid == H) {
    float s = 0.f;
    for (int r = 0; r < MDP_R; ++r) s += dq[r];
    slab[nd.t[5].off] = s;
  }
  for (int r = tid / H, h = tid % H; r < MDP_R; r += MDP_GEN_THREADS / H)
    d2[r * ldh + h] = h2c[r * ldh + h] > 0.f ? dq[r] * w3h : 0.f;
  __syncthreads();
  MDP_STAMP(4);
  // dh1 tiles then dW2 tiles, dealt over all waves
  for (int t = wave; t < NT + NT * NT; t += nw) {
    if (t < NT) dgrad_tile_relu_pf(d2, ldh, H, a.theta + nd.t[2].off, h1c, ldh, d1, ldh, t, pft);
    else wgrad_tile(h1c, ldh, H, d2, ldh, H, slab + nd.t[2].off, t - NT);
  }
  colsum16(d2, ldh, H, slab + nd.t[3].off);
  __syncthreads();
  wgrad_waves(Xc, ldX, ag.cin, d1, ldh, H, slab + nd.t[0].off, 0, nw);
  colsum16(d1, ldh, H, slab + nd.t[1].off);
  MDP_STAMP(5);
}

template <int H>
__global__ __launch_bounds__(MDP_GEN_THREADS) void k_critic_grad(CriticArgs a) {
  critic_body<H>(a, a.topo, blockIdx.x);
}

// AA: ActorArgs, or the Topo-less ActorArgsHead of a gradient-pair launch
template <int H, class AA>
__device__ __forceinline__ void actor_body(const AA& a, const Topo& T, const int blk) {
  constexpr int NT = H / 16;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const ADesc& ag = T.ag[a.agent];
  const int ldr = lds_ld(T.row_stride), ldc = lds_ld(T.cin_max), ldh = H + 1;
  const int S = MDP_R * ldh;
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* x = cv.take(MDP_R * ldc);
  float* h1a = cv.take(S);
  float* h2a = cv.take(S);
  float* h1c = cv.take(S);
  float* h2c = cv.take(S);
  float* d2 = cv.take(S);
  float* d1 = cv.take(S);
  float* lg = cv.take(MDP_R * 8);
  float* av = cv.take(MDP_R * 8);
  float* da = cv.take(MDP_R * 8);
  float* dl = cv.take(MDP_R * 8);
  float* qv = cv.take(MDP_R * 8);
  float* w1ai = cv.take(MDP_ACT_DIM * H);  // the critic's layer-1 rows of the a_i input (for da)

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = blockDim.x >> 6;
  const int r0 = blk * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const bool lq = ag.local_q != 0;
  // throughput mode (multi > 1: one launch per agent, every agent from the
  // round-start parameters) draws agent i's noise at upd_ctr + i, as the fast kernels
  const uint32_t ctr = a.ctl->upd_ctr + (a.multi > 1 ? (uint32_t)a.agent : 0u);
  const NDesc& na = ag.actor;
  const NDesc& nc = ag.critic;
  const float* P = a.theta;
  const int cin = ag.cin;

  float pf[MDP_KC];  // this wave's next layer chunk, issued ahead (wave < NT)
  f32x4 pft[4];      // the next transposed (backward) chunk, issued ahead
  // Critic layer 1 beside the actor forward (par, a MADDPG critic at H <= 128):
  // its input is the replay row prefix except the a_i columns, which the
  // Gumbel sample fills only after the actor head.  Waves NT .. 2 NT - 1 (idle
  // during the single-net actor layers) run tile wave - NT of it over the row
  // with a_i read as zero, one 64-deep weight chunk per phase of the actor
  // forward (actor L1, actor L2, head + Gumbel), then add the a_i k-steps from
  // the sample: the 3.8 us critic layer-1 phase (S5, stamped) becomes a
  // two-k-step phase.  (The MFMA k order differs from one chain over the row:
  // a_i's k-steps come last.)
  constexpr bool kPar = 2 * NT <= MDP_GEN_THREADS / 64;
  const bool par = kPar && !lq && ag.a_in_off + MDP_ACT_DIM <= cin;
  const bool pw = par && wave >= NT && wave < 2 * NT;  // a partial wave (uniform)
  const int a_lo = ag.a_in_off, a4 = a_lo & ~3;
  f32x4 pacc = {0.f, 0.f, 0.f, 0.f};
  float paw[2] = {0.f, 0.f};  // W1c rows a4 + 4 s + kq of this lane's column (the a_i k-steps)
  MDP_STAMP(32);
  if (wave < NT) pf_load(pf, P + na.t[0].off, H, wave, 0, ag.obs_dim);
  if (pw) pf_load(pf, P + nc.t[0].off, H, wave - NT, 0, cin);
  gather_rows16(a.replay, T.row_stride, a.idx, r0, nvalid, rowbuf, ldr);
  for (int e = tid; e < MDP_ACT_DIM * H; e += blockDim.x) w1ai[e] = P[nc.t[0].off + (int64_t)ag.a_in_off * H + e];
  __syncthreads();
  MDP_STAMP(33);
  // actor forward on obs_i -> logits p (maddpg.py:39)
  if (wave < NT) {
    fwd_tile_pf<true>(rowbuf + ag.obs_off, ldr, 0, ag.obs_dim, P + na.t[0].off, P + na.t[1].off, H, nullptr, 0, h1a,
                      ldh, wave, pf);
    pf_load(pf, P + na.t[2].off, H, wave, 0, H);
  }
  const int pcol = (wave - NT) * 16 + (lane & 15);  // the partial wave's column
  if (pw) {
    const float* W1c = P + nc.t[0].off;
    pacc = mfma_chunk_zc(pacc, pf, rowbuf, ldr, lane & 15, 0, cin, lane >> 4, a_lo, a_lo + MDP_ACT_DIM);
    if (4 * MDP_KC < cin) load_wchunk(pf, W1c, H, pcol, 4 * MDP_KC, cin, lane >> 4);
  } else if (!par) {
    // critic input with act_input_n[i] = the sample (maddpg.py:48-52): the replay part now
    for (int e = tid; e < MDP_R * cin; e += blockDim.x) {
      const int r = e / cin, c = e - r * cin;
      const int src = lq ? (c < ag.obs_dim ? ag.obs_off + c : ag.act_off + c - ag.obs_dim) : c;
      x[r * ldc + c] = rowbuf[r * ldr + src];
    }
  }
  __syncthreads();
  MDP_STAMP(34);
  // the actor head's fragments (wave 0), issued ahead of the layer-2 tile
  constexpr int HKS = H / 4 <= 32 ? H / 4 : 1;
  float hw[HKS], hb = 0.f;
  if (H / 4 <= 32 && wave == 0) head_load<HKS>(hw, hb, P + na.t[4].off, P + na.t[5].off, MDP_ACT_DIM);
  if (wave < NT) {
    fwd_tile_pf<true>(h1a, ldh, 0, H, P + na.t[2].off, P + na.t[3].off, H, nullptr, 0, h2a, ldh, wave, pf);
    if (par) pf_load(pf, P + nc.t[2].off, H, wave, 0, H);  // critic L2 follows the a_i step
    else pf_load(pf, P + nc.t[0].off, H, wave, 0, cin);
  } else if (pw && 4 * MDP_KC < cin) {
    const float* W1c = P + nc.t[0].off;
    pacc = mfma_chunk_zc(pacc, pf, rowbuf, ldr, lane & 15, 4 * MDP_KC, cin, lane >> 4, a_lo, a_lo + MDP_ACT_DIM);
    if (8 * MDP_KC < cin) load_wchunk(pf, W1c, H, pcol, 8 * MDP_KC, cin, lane >> 4);
  }
  __syncthreads();
  MDP_STAMP(35);
  if (wave == 0) {
    if constexpr (H / 4 <= 32) head_acc<HKS>(hw, hb, h2a, ldh, MDP_ACT_DIM, lg, 8);
    else head_mfma<H / 4>(h2a, ldh, H, P + na.t[4].off, P + na.t[5].off, MDP_ACT_DIM, lg, 8);
    wave_sync();
    if (lane < MDP_R) {  // fresh Gumbel sample (maddpg.py:49)
      float u[MDP_ACT_DIM];
      if (a.u_act) {
        for (int k = 0; k < MDP_ACT_DIM; ++k)
          u[k] = lane < nvalid ? a.u_act[(int64_t)(r0 + lane) * MDP_ACT_DIM + k] : 0.5f;
      } else {
        uniforms5(a.seed, (uint32_t)((a.agent << 8) | 0x80), ctr, (uint32_t)(r0 + lane), u);
      }
      gumbel_softmax5(lg + lane * 8, u, av + lane * 8);
      if (!par)
        for (int k = 0; k < MDP_ACT_DIM; ++k) x[lane * ldc + ag.a_in_off + k] = av[lane * 8 + k];
    }
  } else if (pw) {
    const float* W1c = P + nc.t[0].off;
    for (int c0 = 8 * MDP_KC; c0 < cin; c0 += 4 * MDP_KC) {  // the rest of the row (cin > 128)
      pacc = mfma_chunk_zc(pacc, pf, rowbuf, ldr, lane & 15, c0, cin, lane >> 4, a_lo, a_lo + MDP_ACT_DIM);
      if (c0 + 4 * MDP_KC < cin) load_wchunk(pf, W1c, H, pcol, c0 + 4 * MDP_KC, cin, lane >> 4);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) paw[q] = W1c[min(a4 + 4 * q + (lane >> 4), cin - 1) * H + pcol];
  }
  __syncthreads();
  MDP_STAMP(36);
  // critic (post-step weights) forward
  if (par) {
    if (pw) {  // + the a_i k-steps (rows a4 .. a4 + 7 of W1c; a_i's columns from the sample) + b1, ReLU
      const int r = lane & 15, kq = lane >> 4;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int k = a4 + 4 * q + kq;
        const float xa = (k >= a_lo && k < a_lo + MDP_ACT_DIM) ? av[r * 8 + (k - a_lo)] : 0.f;
        if (a4 + 4 * q < cin) pacc = MDP_MFMA(xa, paw[q], pacc);
      }
      const float bias = P[nc.t[1].off + pcol];
#pragma unroll
      for (int i = 0; i < 4; ++i) h1c[(kq * 4 + i) * ldh + pcol] = fmaxf(pacc[i] + bias, 0.f);
    }
  } else if (wave < NT) {
    fwd_tile_pf<true, true>(x, ldc, 0, cin, P + nc.t[0].off, P + nc.t[1].off, H, nullptr, 0, h1c, ldh, wave, pf);
    pf_load(pf, P + nc.t[2].off, H, wave, 0, H);
  }
  __syncthreads();
  MDP_STAMP(37);
  float qw[HKS], qb = 0.f;  // the critic head's fragments (q), issued ahead on an idle wave
  const float w3h = P[nc.t[4].off + tid % H];  // d2 pass below: one W3c column per thread
  if (wave < NT) {
    fwd_tile_pf<true>(h1c, ldh, 0, H, P + nc.t[2].off, P + nc.t[3].off, H, nullptr, 0, h2c, ldh, wave, pf);
    pf_load_t(pft, P + nc.t[2].off, H, wave);  // dh1c = d2 W2c^T
  } else if (H / 4 <= 32 && wave == nw - 1) {
    head_load<HKS>(qw, qb, P + nc.t[4].off, P + nc.t[5].off, 1);
  }
  __syncthreads();
  MDP_STAMP(38);
  // dL/dq = -1/B ; d2 = dq * W3c masked by h2c > 0.  q (the loss value only)
  // waits for the next phase, on a wave the dh1c tiles leave idle
  const bool q_late = NT < nw;
  if (!q_late && wave == 0) head_mfma<H / 4>(h2c, ldh, H, P + nc.t[4].off, P + nc.t[5].off, 1, qv, 8);
  for (int r = tid / H, h = tid % H; r < MDP_R; r += MDP_GEN_THREADS / H)
    d2[r * ldh + h] = (r < nvalid && h2c[r * ldh + h] > 0.f) ? a.neg_inv_b * w3h : 0.f;
  __syncthreads();
  MDP_STAMP(39);
  // dh1c = d2 @ W2c^T masked by h1c > 0
  if (wave < NT) {
    dgrad_tile_relu_pf(d2, ldh, H, P + nc.t[2].off, h1c, ldh, d1, ldh, wave, pft);
    pf_load_t(pft, P + na.t[2].off, H, wave);  // dh1a = d2a W2a^T, after the softmax backward
  } else if (q_late && wave == nw - 1) {
    if constexpr (H / 4 <= 32) head_acc<HKS>(qw, qb, h2c, ldh, 1, qv, 8);
    else head_mfma<H / 4>(h2c, ldh, H, P + nc.t[4].off, P + nc.t[5].off, 1, qv, 8);
  }
  __syncthreads();
  MDP_STAMP(56);
  if (wave == 0) {
    // da[r][k] = sum_h d1[r][h] * W1c[a_in_off + k][h] (only the a_i input
    // columns): one MFMA tile, column k < 5 of it, the W1c rows staged in LDS
    // at the start.  (A VALU loop reading W1c from global memory took 14 us
    // of the 45 us S5 actor step.)
    {
      const int r = lane & 15, kq = lane >> 4, c = min(r, MDP_ACT_DIM - 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int s4 = 0; s4 < H / 4; ++s4) {
        const int k = 4 * s4 + kq;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(d1[r * ldh + k], w1ai[c * H + k], acc, 0, 0, 0);
      }
      if (r < MDP_ACT_DIM) {
#pragma unroll
        for (int i = 0; i < 4; ++i) da[(kq * 4 + i) * 8 + r] = acc[i];
      }
    }
    wave_sync();
    // softmax backward + regulariser: dlogits = (da - sum(a*da)) * a + reg*2*p/(B*A); loss partials
    double s_q = 0.0, s_p = 0.0;
    if (lane < MDP_R) {
      float dot = 0.f;
      for (int k = 0; k < MDP_ACT_DIM; ++k) dot += da[lane * 8 + k] * av[lane * 8 + k];
      for (int k = 0; k < MDP_ACT_DIM; ++k) {
        const float g = (da[lane * 8 + k] - dot) * av[lane * 8 + k] + lg[lane * 8 + k] * a.reg_scale;
        dl[lane * 8 + k] = lane < nvalid ? g : 0.f;
      }
      if (lane < nvalid) {
        s_q = (double)qv[lane * 8];
        for (int k = 0; k < MDP_ACT_DIM; ++k) {
          const double p = (double)lg[lane * 8 + k];
          s_p += p * p;
        }
      }
    }
    s_q = sum16(s_q);
    s_p = sum16(s_p);
    if (lane == 0) {
      double* st = a.slab_stat + (int64_t)blk * 8;
      st[0] = s_q;
      st[1] = s_p;
    }
  }
  __syncthreads();
  MDP_STAMP(57);
  // actor backward: dW3a, db3a, d2a = (dl @ W3a^T) masked by h2a > 0
  float* slab = a.slab + (int64_t)blk * a.slab_stride - na.off;
  const float* W3a = P + na.t[4].off;
  for (int e = tid; e < H * MDP_ACT_DIM; e += blockDim.x) {
    const int h = e / MDP_ACT_DIM, k = e - h * MDP_ACT_DIM;
    float s = 0.f;
    for (int r = 0; r < MDP_R; ++r) s = fmaf(h2a[r * ldh + h], dl[r * 8 + k], s);
    slab[na.t[4].off + e] = s;
  }
  if (tid < MDP_ACT_DIM) {
    float s = 0.f;
    for (int r = 0; r < MDP_R; ++r) s += dl[r * 8 + tid];
    slab[na.t[5].off + tid] = s;
  }
  for (int e = tid; e < MDP_R * H; e += blockDim.x) {
    const int r = e / H, h = e - r * H;
    float s = 0.f;
    for (int k = 0; k < MDP_ACT_DIM; ++k) s = fmaf(dl[r * 8 + k], W3a[h * MDP_ACT_DIM + k], s);
    d2[r * ldh + h] = h2a[r * ldh + h] > 0.f ? s : 0.f;
  }
  __syncthreads();
  MDP_STAMP(58);
  // dh1a tiles then dW2a tiles, dealt over all waves
  for (int t = wave; t < NT + NT * NT; t += nw) {
    if (t < NT) dgrad_tile_relu_pf(d2, ldh, H, P + na.t[2].off, h1a, ldh, d1, ldh, t, pft);
    else wgrad_tile(h1a, ldh, H, d2, ldh, H, slab + na.t[2].off, t - NT);
  }
  colsum16(d2, ldh, H, slab + na.t[3].off);
  __syncthreads();
  MDP_STAMP(59);
  wgrad_waves(rowbuf + ag.obs_off, ldr, ag.obs_dim, d1, ldh, H, slab + na.t[0].off, 0, nw);
  colsum16(d1, ldh, H, slab + na.t[1].off);
  MDP_STAMP(60);
}

template <int H>
__global__ __launch_bounds__(MDP_GEN_THREADS) void k_actor_grad(ActorArgs a) {
  MDP_KARG_TOUCH("s"(a.agent), "s"(a.slab_stride), "s"(a.cpre_agent), "s"(a.topo.n));
  MDP_KARG_TOUCH(MDP_KARG_ADESC(a.topo.ag[a.agent]));
  actor_body<H>(a, a.topo, blockIdx.x);
}

// throughput mode: agent i's critic step (workgroups [0, B/16)) and actor step
// (the rest) in one launch -- no kernel boundary between them, and the actor
// step's workgroups start on the CUs the critic step's finished ones free
template <int H>
__global__ __launch_bounds__(MDP_GEN_THREADS) void k_grad_pair(GradPairArgs p) {
  const int nc = (p.c.B + MDP_R - 1) / MDP_R;
  if ((int)blockIdx.x < nc) critic_body<H>(p.c, p.c.topo, blockIdx.x);
  else actor_body<H>(p.x, p.c.topo, (int)blockIdx.x - nc);
}

// ---------------------------------------------------------------- launchers
namespace {
template <int H>
hipError_t launch_critic(const CriticArgs& a, int lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_critic_grad<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MDP_LDS_BUDGET);
    (void)hipGetLastError();
    attr = true;
  }
  mdp_launch(k_critic_grad<H>, dim3((a.B + MDP_R - 1) / MDP_R), dim3(MDP_GEN_THREADS), lds, s, a);
  return hipGetLastError();
}
template <int H>
hipError_t launch_actor(const ActorArgs& a, int lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_actor_grad<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MDP_LDS_BUDGET);
    (void)hipGetLastError();
    attr = true;
  }
  mdp_launch(k_actor_grad<H>, dim3((a.B + MDP_R - 1) / MDP_R), dim3(MDP_GEN_THREADS), lds, s, a);
  return hipGetLastError();
}
}  // namespace

template <int H>
hipError_t launch_pair(const GradPairArgs& a, int lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_grad_pair<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MDP_LDS_BUDGET);
    (void)hipGetLastError();
    attr = true;
  }
  mdp_launch(k_grad_pair<H>, dim3(2 * ((a.c.B + MDP_R - 1) / MDP_R)), dim3(MDP_GEN_THREADS), lds, s, a);
  return hipGetLastError();
}

hipError_t mdp_launch_grad_pair(const GradPairArgs& a, int H, int lds_bytes, hipStream_t s) {
  switch (H) {
    case 64: return launch_pair<64>(a, lds_bytes, s);
    case 128: return launch_pair<128>(a, lds_bytes, s);
    case 256: return launch_pair<256>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t mdp_launch_critic_grad(const CriticArgs& a, int H, int lds_bytes, hipStream_t s) {
  switch (H) {
    case 64: return launch_critic<64>(a, lds_bytes, s);
    case 128: return launch_critic<128>(a, lds_bytes, s);
    case 256: return launch_critic<256>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}
hipError_t mdp_launch_actor_grad(const ActorArgs& a, int H, int lds_bytes, hipStream_t s) {
  switch (H) {
    case 64: return launch_actor<64>(a, lds_bytes, s);
    case 128: return launch_actor<128>(a, lds_bytes, s);
    case 256: return launch_actor<256>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}

#ifdef MDP_STAMPS
// diagnostic build: stamps of this translation unit's kernels (own code object)
// the queue trace of the last critic launch (reset = 1: clear it)
extern "C" int mdp_debug_q_trace(unsigned long long* out, int reset) {
  if (reset) {
    unsigned z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_q_n), &z, sizeof(z)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_q_trace), sizeof(unsigned long long) * 160 * 5) == hipSuccess ? 0 : -1;
}
extern "C" int mdp_debug_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif
