// mdp_grads_r.hip -- fast critic-step / actor-step gradient kernels for H = 64.
//
// Same contract and outputs as k_critic_grad / k_actor_grad (mdp_grads.hip;
// per-workgroup partial gradients of 16 batch rows, reduced by k_reduce), for
// the topologies grads_r_ok() admits (every S1-S3 configuration at H = 64).
//
// What is different: every wave loads ALL the weights it will use into its
// registers at kernel start (mdp_device.h "register-resident layers"), so the
// kernel pays one memory round trip, overlapped with the replay gather,
// instead of one per layer; and each phase is given to the waves whose SIMDs
// are free (waves w and w + 4 share a SIMD).  Workgroup barriers B1..B6 are
// executed by every wave the same number of times, each role at its own point
// of its program (a wave arrives late at a barrier when its own work there is
// not needed by the others until the next one).  The replay rows are handed
// over through an LDS counter instead of a barrier (B0 only zeroes it): the
// waves with the heaviest weight loads never wait for the others to finish
// ISSUING theirs (the per-CU load path is the prologue's bottleneck).
//
// k_critic_grad_r (maddpg.py:180-188):
//   waves 0..na-1  target actor j -> Gumbel a~_j                 | B2
//   wave 3         critic forward L1, L2                        | B2 | head q | B3
//   waves 4..7     target-critic L1 column tile on obs' | B2 | + a~ part | B3 | L2 tile | B4
//                  wave 4: head q', fp64 TD, dL/dq (-> LDS flag), d2, dW3, db3 | B5
//   waves 0..3     v = W3 o [h2 > 0] rows | B3 | u tile = (v W2^T) o [h1 > 0] | B4 |
//                  wait for dq, dh1 tile = dq o u | B5   (the backward is linear in dq)
//   all            dW2, db2, dW1, db1 (one phase)
// k_actor_grad_r (maddpg.py:37-58):
//   wave 0  actor forward, Gumbel a_i                              | B2
//   waves 1..3  critic L1 on the replay part (a_i rows masked), one third of
//           the contraction each (waves 2, 3 after their share of the gather) | B2
//   wave 1  sum of the thirds + a_i part -> h1c                    | B2b
//   waves 0..3  one 16-column tile each of critic L2, d2c, q partials | B3
//   waves 4..7  dh1c tiles                                         | B4
//   wave 0  da = dh1c W1c[a_i]^T, softmax backward + reg -> dlogits, d2a, dW3a, db3a | B5
//   waves 0..3 dW2a (four tiles each, interleaved), db2a  ||  waves 4..7 dh1a tiles | B6
//   all     dW1a, db1a
#include "mdp_device.h"
#include "mdp_kernels.h"
#include "mdp_mt.h"

// row tiles per workgroup for the grid: 16 rows (MDP_R)
#define MDP_RW MDP_R

// diagnostic build (make budget; tools/grad_budget.py): the phase points of
// EVERY workgroup of agent MDP_BUDGET_AGENT's critic (kind 0) and actor (kind 1)
// launches -- lane 0 of the wave that reaches a point stamps it into
// g_bud[kind][wg][pt]: the MDP_STAMP / MDP_STAMPW points below, 62 the
// workgroup's start (wave 0), 63 its end (the last wave), 28..32 the critic
// step's CRIT_T points and 33..38 critic_pre's CPRE_T points (the latest wave)
#ifdef MDP_BUDGET
#ifndef MDP_BUDGET_AGENT
#define MDP_BUDGET_AGENT 1
#endif
// The points are kept in LDS during the launch (a global store mid-kernel would
// count in vmcnt and delay the kernel's own later load waits until its ack) and
// written out by the workgroup's last wave at its end.  A point is one s_memtime
// (the shader clock, ~40 cycles) with its lgkmcnt(0) and one LDS store from lane
// 0; the workgroup's start and end also read s_memrealtime (100 MHz, one clock
// for the GPU: slots 64, 65), which places it in the launch and calibrates the
// shader clock.
#define MDP_BUD_N 72
__device__ unsigned long long g_bud[2][160][MDP_BUD_N];
__shared__ int s_bud;  // this launch records into g_bud[s_bud] (-1: not the chosen agent's launch)
__shared__ unsigned long long s_bud_t[MDP_BUD_N];
__shared__ unsigned s_bud_cnt;
// MDP_BUDGET_REP = 2: every point stamped twice (the first value kept), so the
// stamps' own cost can be extrapolated away (tools/grad_budget.py: t0 = 2 t1 - t2)
#ifndef MDP_BUDGET_REP
#define MDP_BUDGET_REP 1
#endif
// (the builtin, not an asm statement with a memory clobber: that clobber is a
// compiler barrier at every point and cost the launch ~1.4 us of lost load /
// LDS overlap, measured -- r06f; the builtin leaves the schedule to the
// compiler, which places the stamp's wait at its LDS store)
__device__ __forceinline__ unsigned long long bud_now() {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
#if MDP_BUDGET_REP > 1
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  asm volatile("" ::"s"(t2));
#endif
  return t;
}
__device__ __forceinline__ unsigned long long bud_real() { return __builtin_amdgcn_s_memrealtime(); }
#define BUD(i)                                           \
  do {                                                   \
    const unsigned long long t__ = bud_now();            \
    if ((threadIdx.x & 63) == 0) s_bud_t[i] = t__;       \
  } while (0)
#define BUDMAX(i)                                        \
  do {                                                   \
    const unsigned long long t__ = bud_now();            \
    if ((threadIdx.x & 63) == 0) atomicMax(&s_bud_t[i], t__); \
  } while (0)
// wave 0 clears the points and stamps the start before anything else
#define BUD_BEGIN(k, agent_, multi_)                                          \
  do {                                                                        \
    s_bud = ((agent_) == MDP_BUDGET_AGENT && (multi_) <= 1) ? (k) : -1;       \
    if (threadIdx.x < 64) {                                                   \
      s_bud_t[threadIdx.x] = 0ull;                                            \
      if (threadIdx.x < MDP_BUD_N - 64) s_bud_t[64 + threadIdx.x] = 0ull;     \
      if (threadIdx.x == 0) s_bud_cnt = 0u;                                   \
      const unsigned long long r__ = bud_real();                              \
      if (threadIdx.x == 0) s_bud_t[64] = r__;                                \
      BUD(62);                                                                \
    }                                                                         \
  } while (0)
// every wave at its end; the last one writes the workgroup's points out
#define MDP_WG_END(k)                                                                     \
  do {                                                                                    \
    BUDMAX(63);                                                                           \
    {                                                                                     \
      const unsigned long long r__ = bud_real();                                          \
      if ((threadIdx.x & 63) == 0) atomicMax(&s_bud_t[65], r__);                          \
    }                                                                                     \
    unsigned c__ = 0u;                                                                    \
    if ((threadIdx.x & 63) == 0) c__ = atomicAdd(&s_bud_cnt, 1u);                         \
    c__ = __builtin_amdgcn_readfirstlane(c__);                                            \
    if (c__ + 1u == (blockDim.x >> 6) && s_bud >= 0 && blockIdx.x < 160) {                \
      const int l__ = threadIdx.x & 63;                                                   \
      g_bud[s_bud][blockIdx.x][l__] = s_bud_t[l__];                                       \
      if (l__ < MDP_BUD_N - 64) g_bud[s_bud][blockIdx.x][64 + l__] = s_bud_t[64 + l__];   \
    }                                                                                     \
  } while (0)
#undef MDP_STAMP
#undef MDP_STAMPW
#define MDP_WG_START(k) \
  do {                  \
  } while (0)
#ifdef MDP_BUDGET_MIN  // only the workgroups' start and end (what the points themselves cost)
#define MDP_STAMP(i) (void)0
#define MDP_STAMPW(i) (void)0
#define CRIT_T(i) (void)0
#define CPRE_T(i) (void)0
#else
#define MDP_STAMP(i) BUD(i)
#define MDP_STAMPW(i) BUD(i)
#define CRIT_T(i) BUDMAX(28 + (i))
#define CPRE_T(i) BUDMAX(33 + (i))
#endif
#else
#define BUD_BEGIN(k, agent_, multi_) (void)0
#endif

// diagnostic build: every workgroup's start (wave 0) and per-wave end of the
// last critic (k = 0) / actor (k = 1) launch -- which role ends the launch
#if defined(MDP_BUDGET)
#elif defined(MDP_STAMPS)
__device__ unsigned long long g_wg_t0[2][512];
__device__ unsigned long long g_wg_t1[2][512][8];
// critic_pre's per-wave phase points (row tile < 64, wave, point)
__device__ unsigned long long g_cpre_t[64][8][6];
// the critic step's per-wave points after B5 (row tile < 64, wave, point)
__device__ unsigned long long g_crit_t[64][8][6];
#define CRIT_T(i)                                                                                   \
  do {                                                                                              \
    if ((threadIdx.x & 63) == 0 && bx < 64) g_crit_t[bx][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define CPRE_T(i)                                                                                   \
  do {                                                                                              \
    if ((threadIdx.x & 63) == 0 && bx < 64) g_cpre_t[bx][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define MDP_WG_START(k)                                                               \
  do {                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 512) g_wg_t0[k][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define MDP_WG_END(k)                                                                 \
  do {                                                                                \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 512)                                  \
      g_wg_t1[k][blockIdx.x][threadIdx.x >> 6] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define MDP_WG_START(k) \
  do {                  \
  } while (0)
#define MDP_WG_END(k) \
  do {                \
  } while (0)
#define CPRE_T(i) \
  do {            \
  } while (0)
#define CRIT_T(i) \
  do {            \
  } while (0)
#endif

namespace {
constexpr int RH = MDP_RH, LH = MDP_RLH, LD = MDP_RLD;

// column sums of a [16][ld] LDS block over the 64 columns, by the 64 lanes of one wave
__device__ __forceinline__ void colsum64(const float* X, int ldx, float* __restrict__ out) {
  const int c = threadIdx.x & 63;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < MDP_R; ++r) s += X[r * ldx + c];
  slab_st(out + c, s);
}

// dX tile (columns 16 tt .. 16 tt + 15) = (dY @ W^T) masked by Hin > 0
__device__ __forceinline__ void dgrad_tile(const float* dY, const f32x4 (&w)[4], const float* Hin, float* dX, int tt) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const f32x4 acc = rdg_acc(dY, LD, w);
  const int col = 16 * tt + r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = kq * 4 + i;
    dX[row * LD + col] = Hin[row * LH + col] > 0.f ? acc[i] : 0.f;
  }
}
// critic L2 column tile tt (columns 16 tt .. 16 tt + 15) for the actor step:
// h2 = relu(h1 W2 + b2); d2c = dq W3 masked by h2 > 0 with dq = -1/B (rows past
// the batch zero); q partial = sum over the tile's columns of h2 W3
__device__ __forceinline__ void critic_l2_tile(const float* h1, const float (&w2t)[16], float b2t, float w3t, int tt,
                                               int nvalid, float dq, float* d2, float* qpart) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  rt_acc<16>(acc, h1, LH, RH, w2t);
  const int col = 16 * tt + r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = kq * 4 + i;
    const float h = fmaxf(acc[i] + b2t, 0.f);
    d2[row * LD + col] = (row < nvalid && h > 0.f) ? dq * w3t : 0.f;
    float s = h * w3t;  // sum over the 16 columns (lanes r of this kq group), fixed order
    s = row_sum(s);
    if (r == 0) qpart[tt * MDP_R + row] = s;
  }
}
// rows 4 q .. 4 q + 3 of d2a = (dl W3a^T) o [h2a > 0] and their share of
// dW3a = h2a^T dl (lane = hidden unit), one row quarter per wave 0..3
__device__ __forceinline__ void d2a_rows(const float* h2a, const float* dl, const float (&w3a)[MDP_ACT_DIM], float* d2a,
                                         float* gwpart, int q) {
  const int lane = threadIdx.x & 63;
  float gw[MDP_ACT_DIM] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = 4 * q + i;
    const float h = h2a[rr * LH + lane];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MDP_ACT_DIM; ++k) {
      const float d = dl[rr * 8 + k];
      s = fmaf(d, w3a[k], s);
      gw[k] = fmaf(h, d, gw[k]);
    }
    d2a[rr * LD + lane] = h > 0.f ? s : 0.f;
  }
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) gwpart[(q * MDP_ACT_DIM + k) * 64 + lane] = gw[k];
}
// dW3a (sum of the four quarters, fixed order) and db3a = column sums of dl
__device__ __forceinline__ void dw3a_store(const float* gwpart, const float* dl, float* dw3, float* db3) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) {
    const float g = ((gwpart[k * 64 + lane] + gwpart[(MDP_ACT_DIM + k) * 64 + lane]) +
                     gwpart[(2 * MDP_ACT_DIM + k) * 64 + lane]) + gwpart[(3 * MDP_ACT_DIM + k) * 64 + lane];
    slab_st(dw3 + lane * MDP_ACT_DIM + k, g);
  }
  if (lane < MDP_ACT_DIM) {
    float s = 0.f;
    for (int rr = 0; rr < MDP_R; ++rr) s += dl[rr * 8 + lane];
    slab_st(db3 + lane, s);
  }
}
// actor forward of 16 rows on ONE wave (maddpg.py:39) and the fresh policy
// sample a_i (:49): h1a, h2a (LDS, stride LH), logits lg and sample av (stride
// 8).  Weights and the Gumbel noise are requested before waiting for the
// replay rows (nsig gather waves signal rows_ready).
__device__ __forceinline__ void actor_fwd_wave(const float* __restrict__ P, const NDesc& na, const ADesc& ag,
                                               const float* rowbuf, int ldr, const float* u_act, int nvalid, int r0,
                                               uint64_t seed, int agent, uint32_t ctr, int* rows_ready, int nsig,
                                               float* h1a, float* h2a, float* lg, float* av) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  f32x4 w1[16], w2[16];
  float w3[16];
  rf_load<16>(w1, P + na.t[0].off, ag.obs_dim);
  rf_load<16>(w2, P + na.t[2].off, RH);
  rh_load(w3, P + na.t[4].off, MDP_ACT_DIM);
  const f32x4 b1 = ld4(P + na.t[1].off + 4 * r), b2 = ld4(P + na.t[3].off + 4 * r);
  const float b3 = P[na.t[5].off + min(r, MDP_ACT_DIM - 1)];
  float gn[MDP_ACT_DIM];  // Gumbel noise of the policy sample, while the weights are in flight
  {
    float u[MDP_ACT_DIM];
    if (u_act) {
      for (int k = 0; k < MDP_ACT_DIM; ++k) u[k] = lane < nvalid ? u_act[(int64_t)(r0 + lane) * MDP_ACT_DIM + k] : 0.5f;
    } else {
      uniforms5(seed, (uint32_t)((agent << 8) | 0x80), ctr_use(ctr), (uint32_t)(r0 + (lane & 15)), u);
    }
    gumbel_noise5(u, gn);
  }
  lds_wait(rows_ready, nsig);
  MDP_STAMP(17);
  {
    f32x4 acc[4];
    rf_zero(acc);
    rf_acc<16>(acc, rowbuf + ag.obs_off, ldr, ag.obs_dim, w1);
    rf_store<true>(acc, b1, h1a, LH);
  }
  wave_sync();
  {
    f32x4 acc[4];
    rf_zero(acc);
    rf_acc<16>(acc, h1a, LH, RH, w2);
    rf_store<true>(acc, b2, h2a, LH);
  }
  wave_sync();
  {
    const f32x4 acc = rh_acc(h2a, LH, w3);
    if (r < MDP_ACT_DIM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) lg[(kq * 4 + i) * 8 + r] = acc[i] + b3;
    }
  }
  wave_sync();
  if (lane < MDP_R) gumbel_softmax5_pre(lg + lane * 8, gn, av + lane * 8);
}

// float4 q of a row block [16][MDP_APRE_W] <-> its LDS home (h1a | h2a | lg | av)
__device__ __forceinline__ float* apre_lds(int q, float* h1a, float* h2a, float* lg, float* av) {
  const int row = q / (MDP_APRE_W / 4), c = 4 * (q - row * (MDP_APRE_W / 4));
  return c < 64 ? h1a + row * LH + c : c < 128 ? h2a + row * LH + c - 64 : c < 136 ? lg + row * 8 + c - 128
                                                                                  : av + row * 8 + c - 136;
}

// extra workgroup of k_critic_grad_r: the actor forward + sample of row tile bx
// for the actor step that follows (same agent, same indices, same noise)
__device__ __forceinline__ void actor_pre_tile(const CriticArgs& a, float* lds, int* rows_ready, int bx) {
  const Topo& T = a.topo;
  const ADesc& ag = T.ag[a.agent];
  const int ldr = lds_ld(T.row_stride);
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* h1a = cv.take(MDP_R * LH);
  float* h2a = cv.take(MDP_R * LH);
  float* lg = cv.take(MDP_R * 8);
  float* av = cv.take(MDP_R * 8);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = bx * MDP_R, nvalid = min(MDP_R, a.B - r0);
  if (threadIdx.x == 0) *rows_ready = 0;
  __syncthreads();
  if (wave == 0) {
    actor_fwd_wave(a.theta, ag.actor, ag, rowbuf, ldr, a.u_act, nvalid, r0, a.seed, a.agent, ctr_load(a.ctl),
                   rows_ready, 7, h1a, h2a, lg, av);
  } else {
    gather_rows16_part(a.replay, T.row_stride, a.idx, r0, nvalid, rowbuf, ldr, 64, 448);
    lds_signal(rows_ready);
  }
  __syncthreads();
  float* dst = a.apre + (int64_t)r0 * MDP_APRE_W;
  for (int q = threadIdx.x; q < MDP_R * MDP_APRE_W / 4; q += blockDim.x)
    handoff_st4(dst + 4 * q, *reinterpret_cast<const f32x4*>(apre_lds(q, h1a, h2a, lg, av)));
  store_rows16(rowbuf, ldr, T.row_stride, a.apre_rows + (int64_t)r0 * T.row_stride);
}
// one wave stores 16 rows x ncols (a multiple of 4) of an LDS tile into the
// row block dst [16][MDP_CPRE_W] at column c0
__device__ __forceinline__ void wave_store_cols16(const float* src, int ld, float* dst, int c0, int ncols) {
  const int lane = threadIdx.x & 63, n4 = ncols >> 2;
  for (int e = lane; e < MDP_R * n4; e += 64) {
    const int r = e / n4, c = 4 * (e - r * n4);
    handoff_st4(dst + r * MDP_CPRE_W + c0 + c, *reinterpret_cast<const f32x4*>(src + r * ld + c));
  }
}
// first MFMA k-step (of 4 inputs) of the target critic's a~ part that holds a
// target action of agent p (columns 5 p .. 5 p + 4)
__device__ __forceinline__ int cpre_split(int p) { return (MDP_ACT_DIM * p) / 4; }

// extra workgroup of k_actor_grad_r (agent p's actor step): the next critic
// step's (agent k, MADDPG critic) work that p's coming update does not touch,
// for row tile bx -- target actors j != p with their Gumbel samples (maddpg.py:
// 183), the critic forward q(o, a) (:85-88), and the target critic's layer-1
// accumulator over obs' and a~_j, j != p (:104; p's weight rows read as zero)
// -- into cpre.  Roles as k_critic_grad_r: waves 0..2 target actors, wave 3
// the critic, waves 4..7 gather and one target-critic column tile each.
__device__ __forceinline__ void critic_pre_tile(const ActorArgs& a, float* lds, int* rows_ready, int bx) {
  const Topo& T = a.topo;
  const int k = a.cpre_agent, p = a.agent;
  const ADesc& ag = T.ag[k];
  const NDesc& nd = ag.critic;
  const int na = T.n;
  const int ldr = lds_ld(T.row_stride);
  const int kb = MDP_ACT_DIM * na, ldA = lds_ld(kb);
  const int ka_t = T.sum_obs, xo_t = T.ag[0].nobs_off, ka_c = ag.cin;
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* xa = cv.take(MDP_R * ldA);
  float* lg = cv.take(3 * MDP_R * 8);
  float* h1a = cv.take(3 * MDP_R * LH);
  float* h2a = cv.take(3 * MDP_R * LH);
  float* h1c = cv.take(MDP_R * LH);
  float* h2c = cv.take(MDP_R * LH);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int r0 = bx * MDP_R, nvalid = min(MDP_R, a.B - r0);
  // the cpre block [16][MDP_CPRE_W]: h1c | h2c | target-critic accumulator |
  // q + pad | a~ [16]; after B2 every wave stores its own part (no second
  // barrier and workgroup-wide copy: that tail was ~1.7 µs of ~7 µs)
  float* dst = a.cpre + (int64_t)r0 * MDP_CPRE_W;
  const uint32_t ctr = ctr_load(a.ctl) + 1u;  // critic k runs after p's actor step advanced the counter
  const float* Pc = a.theta;
  const float* Pt = a.target;
  if (threadIdx.x == 0) *rows_ready = 0;
  __syncthreads();
  CPRE_T(0);
  if (wave < 3) {
    if (wave < na && wave != p) {
      const int j = wave;
      const ADesc& aj = T.ag[j];
      const NDesc& an = aj.actor;
      f32x4 w1[16], w2[16];
      float w3[16];
      rf_load<16>(w1, Pt + an.t[0].off, aj.obs_dim);
      rf_load<16>(w2, Pt + an.t[2].off, RH);
      rh_load(w3, Pt + an.t[4].off, MDP_ACT_DIM);
      const f32x4 b1 = ld4(Pt + an.t[1].off + 4 * r), b2 = ld4(Pt + an.t[3].off + 4 * r);
      const float b3 = Pt[an.t[5].off + min(r, MDP_ACT_DIM - 1)];
      float gn[MDP_ACT_DIM];
      {
        float u[MDP_ACT_DIM];
        uniforms5(a.seed, (uint32_t)((k << 8) | (j + 1)), ctr_use(ctr), (uint32_t)(r0 + (lane & 15)), u);
        gumbel_noise5(u, gn);
      }
      lds_wait(rows_ready, 4);
      CPRE_T(1);
      float* h1 = h1a + wave * MDP_R * LH;
      float* h2 = h2a + wave * MDP_R * LH;
      float* lgj = lg + wave * MDP_R * 8;
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<16>(acc, rowbuf + aj.nobs_off, ldr, aj.obs_dim, w1);
        rf_store<true>(acc, b1, h1, LH);
      }
      wave_sync();
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<16>(acc, h1, LH, RH, w2);
        rf_store<true>(acc, b2, h2, LH);
      }
      wave_sync();
      {
        const f32x4 acc = rh_acc(h2, LH, w3);
        if (r < MDP_ACT_DIM) {
#pragma unroll
          for (int i = 0; i < 4; ++i) lgj[(kq * 4 + i) * 8 + r] = acc[i] + b3;
        }
      }
      wave_sync();
      if (lane < MDP_R) {
        float act[MDP_ACT_DIM];
        gumbel_softmax5_pre(lgj + lane * 8, gn, act);
        for (int q = 0; q < MDP_ACT_DIM; ++q) xa[lane * ldA + MDP_ACT_DIM * j + q] = act[q];
      }
    } else if (wave == p && lane < MDP_R) {  // p's slot: zero weights meet zeros (not stale LDS, e.g. NaN)
      for (int q = 0; q < MDP_ACT_DIM; ++q) xa[lane * ldA + MDP_ACT_DIM * p + q] = 0.f;
    }
    CPRE_T(2);
    __syncthreads();  // B2: a~_j (j != p) ready
    CPRE_T(3);
    // the gathered rows -> cpre_rows, by the three target-actor waves
    {
      const int v4 = T.row_stride >> 2;
      float* rb = a.cpre_rows + (int64_t)r0 * T.row_stride;
      for (int e = threadIdx.x; e < MDP_R * v4; e += 3 * 64) {
        const int rr = e / v4, c4 = e - rr * v4;
        const float* sp = rowbuf + rr * ldr + c4 * 4;
        handoff_st4(rb + (int64_t)rr * T.row_stride + c4 * 4, f32x4{sp[0], sp[1], sp[2], sp[3]});
      }
    }
  } else if (wave == 3) {
    f32x4 w1[20], w2[16];
    float w3[16];
    rf_load<20>(w1, Pc + nd.t[0].off, ka_c);
    rf_load<16>(w2, Pc + nd.t[2].off, RH);
    rq_load(w3, Pc + nd.t[4].off);
    const f32x4 b1 = ld4(Pc + nd.t[1].off + 4 * r), b2 = ld4(Pc + nd.t[3].off + 4 * r);
    const float b3 = Pc[nd.t[5].off];
    lds_wait(rows_ready, 4);
    CPRE_T(1);
    {
      f32x4 acc[4];
      rf_zero(acc);
      rf_acc<20>(acc, rowbuf, ldr, ka_c, w1);
      rf_store<true>(acc, b1, h1c, LH);
    }
    wave_sync();
    {
      f32x4 acc[4];
      rf_zero(acc);
      rf_acc<16>(acc, h1c, LH, RH, w2);
      rf_store<true>(acc, b2, h2c, LH);
    }
    wave_sync();
    const float q = rq_head(h2c, LH, w3) + b3;
    CPRE_T(2);
    __syncthreads();  // B2
    CPRE_T(3);
    wave_store_cols16(h1c, LH, dst, 0, RH);
    wave_store_cols16(h2c, LH, dst, RH, RH);
    if ((lane & 3) == 0) handoff_st4(dst + (lane >> 2) * MDP_CPRE_W + 3 * RH, f32x4{q, 0.f, 0.f, 0.f});
  } else {
    const int tt = wave - 4, col = 16 * tt + r;
    gather_rows16_part(a.replay, T.row_stride, a.cpre_idx, r0, nvalid, rowbuf, ldr, 256, 256);
    lds_signal(rows_ready);
    // the k-steps of the a~ part before p's first target action (rows 0 .. 4 ks - 1)
    const int ks = cpre_split(p);
    float wa[16], wb[5];
    rt_load<16>(wa, Pt + nd.t[0].off, RH, col, ka_t);
    rt_load_k<5>(wb, Pt + nd.t[0].off + ka_t * RH, RH, col, 4 * ks);
    lds_wait(rows_ready, 4);
    CPRE_T(1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    rt_acc<16>(acc, rowbuf + xo_t, ldr, ka_t, wa);
    CPRE_T(2);
    __syncthreads();  // B2: a~ ready
    CPRE_T(3);
    // every a~_j (p's slot zero: the critic step writes it), one per lane of waves 4..7
    {
      const int e = 64 * tt + lane, rr = e >> 4, c = e & 15;
      dst[rr * MDP_CPRE_W + 3 * RH + 4 + c] = c < kb ? xa[rr * ldA + c] : 0.f;
    }
    if (ks > 0) rt_acc<5>(acc, xa, ldA, 4 * ks, wb);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[(kq * 4 + i) * MDP_CPRE_W + 2 * RH + col] = acc[i];
    CPRE_T(4);
  }
  CPRE_T(5);
}
}  // namespace

__global__ __launch_bounds__(512) void k_critic_grad_r(CriticArgs a) {
  MDP_KARG_TOUCH("s"(a.agent), "s"(a.inv_b), "s"(a.pf_count), "s"(a.cpre_prev), "s"(a.topo.n), "s"(gridDim.x));
  BUD_BEGIN(0, a.agent, a.multi);
  MDP_WG_START(0);
  MDP_TL(a.ctl, 0, 0);
  if (a.pf_count > 0 && blockIdx.x == gridDim.x - 1) {
    MDP_TL_ROLE(0, 2);
    // the next round's index draw (same ring length, the MT stream continues):
    // one workgroup beside the B/16 of this kernel, so it costs no time of its own
    make_index_block<512>(a.pf_ctl, a.pf_count, a.pf_out);
    MDP_WG_END(0);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ int rows_ready;  // gather waves done (LDS hand-off, replaces a barrier)
  __shared__ int post_sync[2];  // critic_post: target-actor L1, L2 tiles of waves 0..3 done
  __shared__ int dq_ready;      // wave 4 wrote dL/dq (the dh1 tiles of waves 0..3 wait for it)
  int agent = a.agent, bx = blockIdx.x;
  if (a.apre) {  // workgroups [B/16, 2 B/16): the actor step's forward (strict mode only)
    const int nwg = (a.B + MDP_RW - 1) / MDP_RW;
    if (bx >= nwg) {
      MDP_TL_ROLE(0, 1);
      actor_pre_tile(a, lds, &rows_ready, bx - nwg);
      MDP_WG_END(0);
      return;
    }
  }
  if (a.multi > 1) {  // throughput mode: every agent's critic step in this launch
    const int nwg = (a.B + MDP_RW - 1) / MDP_RW;
    agent = bx / nwg;
    bx -= agent * nwg;
  }
  const int32_t* idx = a.multi > 1 ? a.idx + (int64_t)agent * a.B : a.idx;
  const float* u_tgt = (a.multi > 1 && a.u_tgt) ? a.u_tgt + (int64_t)agent * a.topo.n * a.B * MDP_ACT_DIM : a.u_tgt;
  const Topo& T = a.topo;
  MDP_KARG_TOUCH(MDP_KARG_ADESC(T.ag[agent]), MDP_KARG_ADESC(T.ag[max(a.cpre_prev, 0)]));
  const ADesc& ag = T.ag[agent];
  const NDesc& nd = ag.critic;
  const bool lq = ag.local_q != 0;
  const int na = lq ? 1 : T.n;
  const int ldr = lds_ld(T.row_stride);
  const int kb = MDP_ACT_DIM * na, ldA = lds_ld(kb);
  const int ka_t = lq ? ag.obs_dim : T.sum_obs;  // target critic input part A: obs' (maddpg.py:86-87)
  const int xo_t = lq ? ag.nobs_off : T.ag[0].nobs_off;
  const int ka_c = lq ? ag.obs_dim : ag.cin;     // online critic input: the row prefix, or obs_i | act_i
  const int xo_c = lq ? ag.obs_off : 0;
  const int kb_c = lq ? MDP_ACT_DIM : 0;
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* xa = cv.take(MDP_R * ldA);
  float* lg = cv.take(3 * MDP_R * 8);
  float* h1a = cv.take(3 * MDP_R * LH);
  float* h2a = cv.take(3 * MDP_R * LH);
  float* h1c = cv.take(MDP_R * LH);
  float* h2c = cv.take(MDP_R * LH);
  float* h1t = cv.take(MDP_R * LH);
  float* h2t = cv.take(MDP_R * LH);
  float* qv = cv.take(MDP_R);
  float* qn = cv.take(MDP_R);
  float* dq = cv.take(MDP_R);
  float* d2 = cv.take(MDP_R * LD);
  float* d1 = cv.take(MDP_R * LD);

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int r0 = bx * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const uint32_t ctr = ctr_load(a.ctl) + (a.multi > 1 ? (uint32_t)agent : 0u);
  const float* Pc = a.theta;
  const float* Pt = a.target;
  // critic_post: target actor pprev is the only one left (see CriticArgs::cpre)
  const bool post = a.cpre != nullptr;
  const int pprev = a.cpre_prev;
  const int64_t ao = a.multi > 1 ? (int64_t)agent : 0;  // per-agent output blocks (throughput mode)
  float* slab = a.slab + ao * a.slab_agent_stride + (int64_t)bx * a.slab_stride - nd.off;
  double* slab_stat = a.slab_stat + ao * (int64_t)((a.B + MDP_R - 1) / MDP_R) * 8;
  double* y_out = a.y_out + ao * a.B;
  MDP_STAMP(0);
  if (threadIdx.x == 0) rows_ready = 0;
  if (threadIdx.x < 2) post_sync[threadIdx.x] = 0;
  if (threadIdx.x == 2) dq_ready = 0;
  __syncthreads();  // B0 (nothing in flight yet)

  if (wave < 4) {
    f32x4 wt[4];  // W2^T tile of the critic for u (requested after B2, off the prologue's load burst)
    float w3v;    // W3 of the critic at column `lane` (v = W3 o [h2c > 0], below)
    if (post) {
      // ---------------- critic_post: target actor pprev (Polyak-updated since the
      // critic_pre) over waves 0..3, one 16-column tile of L1 and L2 each, the
      // head as split-K partials over the tiles; wave 3 also loads h1c, h2c, q
      const ADesc& aj = T.ag[pprev];
      const NDesc& an = aj.actor;
      const int col = 16 * wave + r;
      // the cpre block, issued first (wave 1 h1c, wave 2 h2c, wave 3 q and the
      // a~ except pprev's) but written to LDS only after this wave's L2 tile:
      // written here, each wave waited for its block before issuing its
      // target-actor weights, which then landed ~1 us after wave 0's
      const int c0 = wave == 1 ? 0 : (wave == 2 ? 64 : 192), nc4 = wave == 3 ? 5 : 16;
      f32x4 cv4[4];
      if (wave > 0) {
        const float* src = a.cpre + (int64_t)r0 * MDP_CPRE_W;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int q = min(lane + 64 * it, MDP_R * nc4 - 1), row = q / nc4;
          cv4[it] = ld4(src + (int64_t)row * MDP_CPRE_W + c0 + 4 * (q - row * nc4));
        }
      }
      float w1t[16], w2t[16], w3[16];
      rt_load_k<16>(w1t, Pt + an.t[0].off, RH, col, aj.obs_dim);
      rt_load<16>(w2t, Pt + an.t[2].off, RH, col, RH);
      const float b1 = Pt[an.t[1].off + col], b2 = Pt[an.t[3].off + col];
      float gn[MDP_ACT_DIM], b3 = 0.f;
      if (wave == 0) {  // the head (one MFMA chain, as the unsplit step) and the Gumbel noise
        rh_load(w3, Pt + an.t[4].off, MDP_ACT_DIM);
        b3 = Pt[an.t[5].off + min(r, MDP_ACT_DIM - 1)];
        float u[MDP_ACT_DIM];
        uniforms5(a.seed, (uint32_t)((agent << 8) | (pprev + 1)), ctr_use(ctr), (uint32_t)(r0 + (lane & 15)), u);
        gumbel_noise5(u, gn);
      }
      w3v = Pc[nd.t[4].off + lane];
      float* h1 = h1a;
      float* h2 = h2a;
      if (wave == 0) MDP_STAMPW(48);
      if (wave == 3) MDP_STAMPW(54);
      lds_wait(&rows_ready, 4);
      if (wave == 0) MDP_STAMPW(49);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      rt_acc<16>(acc, rowbuf + aj.nobs_off, ldr, aj.obs_dim, w1t);
#pragma unroll
      for (int i = 0; i < 4; ++i) h1[(kq * 4 + i) * LH + col] = fmaxf(acc[i] + b1, 0.f);
      lds_signal(&post_sync[0]);
      lds_wait(&post_sync[0], 4);
      acc = f32x4{0.f, 0.f, 0.f, 0.f};
      rt_acc<16>(acc, h1, LH, RH, w2t);
#pragma unroll
      for (int i = 0; i < 4; ++i) h2[(kq * 4 + i) * LH + col] = fmaxf(acc[i] + b2, 0.f);
      lds_signal(&post_sync[1]);
      if (wave == 0) MDP_STAMPW(50);
      if (wave == 3) MDP_STAMPW(55);
      if (wave > 0) {  // the cpre block into LDS (landed with the weights: loads complete in order)
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int q = lane + 64 * it, row = q / nc4, c = c0 + 4 * (q - row * nc4);
          if (q < MDP_R * nc4) {
            if (c < 64) *reinterpret_cast<f32x4*>(h1c + row * LH + c) = cv4[it];
            else if (c < 128) *reinterpret_cast<f32x4*>(h2c + row * LH + c - 64) = cv4[it];
            else if (c == 192) qv[row] = cv4[it][0];
            else {  // the stored target actions (not pprev's slot: wave 0 writes it)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int cc = c - 196 + e;
                if (cc < kb && (cc < MDP_ACT_DIM * pprev || cc >= MDP_ACT_DIM * (pprev + 1)))
                  xa[row * ldA + cc] = cv4[it][e];
              }
            }
          }
        }
      }
      if (wave == 0) {
        lds_wait(&post_sync[1], 4);
        MDP_STAMPW(51);
        float* lgj = lg;
        {
          const f32x4 hacc = rh_acc(h2, LH, w3);
          if (r < MDP_ACT_DIM) {
#pragma unroll
            for (int i = 0; i < 4; ++i) lgj[(kq * 4 + i) * 8 + r] = hacc[i] + b3;
          }
        }
        wave_sync();
        if (lane < MDP_R) {  // distributions.py:264-266
          float act[MDP_ACT_DIM];
          gumbel_softmax5_pre(lgj + lane * 8, gn, act);
          for (int c = 0; c < MDP_ACT_DIM; ++c) xa[lane * ldA + MDP_ACT_DIM * pprev + c] = act[c];
        }
        MDP_STAMPW(52);
      }
      __syncthreads();  // B2
      if (wave == 0) MDP_STAMPW(53);
    } else if (wave < na) {
      // ---------------- target actor j on obs'_j, Gumbel-softmax target action (maddpg.py:183)
      const int j = lq ? agent : wave;
      const ADesc& aj = T.ag[j];
      const NDesc& an = aj.actor;
#ifdef MDP_STAMPS
      MDP_STAMP(11);
      {
        volatile int sink = an.t[0].off + an.t[2].off;
        (void)sink;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      MDP_STAMP(12);
#endif
      f32x4 w1[16], w2[16];
      float w3[16];
      rf_load<16>(w1, Pt + an.t[0].off, aj.obs_dim);
      rf_load<16>(w2, Pt + an.t[2].off, RH);
      rh_load(w3, Pt + an.t[4].off, MDP_ACT_DIM);
      const f32x4 b1 = ld4(Pt + an.t[1].off + 4 * r), b2 = ld4(Pt + an.t[3].off + 4 * r);
      const float b3 = Pt[an.t[5].off + min(r, MDP_ACT_DIM - 1)];
      // Gumbel noise of the target action, computed while the weights are in flight
      float gn[MDP_ACT_DIM];
      {
        float u[MDP_ACT_DIM];
        if (u_tgt) {
          for (int k = 0; k < MDP_ACT_DIM; ++k)
            u[k] = lane < nvalid ? u_tgt[((int64_t)j * a.B + r0 + lane) * MDP_ACT_DIM + k] : 0.5f;
        } else {
          uniforms5(a.seed, (uint32_t)((agent << 8) | (j + 1)), ctr_use(ctr), (uint32_t)(r0 + (lane & 15)), u);
        }
        gumbel_noise5(u, gn);
      }
#ifdef MDP_STAMPS
      MDP_STAMP(13);
      {
        float sink = w1[0][0] + w2[15][3] + w3[15] + b1[0] + b2[0] + b3;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        volatile float vs = sink;
        (void)vs;
      }
      MDP_STAMP(14);
#endif
      lds_wait(&rows_ready, 4);
      MDP_STAMP(1);
      MDP_CLK(40);
      float* h1 = h1a + wave * MDP_R * LH;
      float* h2 = h2a + wave * MDP_R * LH;
      float* lgj = lg + wave * MDP_R * 8;
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<16>(acc, rowbuf + aj.nobs_off, ldr, aj.obs_dim, w1);
        rf_store<true>(acc, b1, h1, LH);
      }
      wave_sync();
      MDP_STAMP(41);
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<16>(acc, h1, LH, RH, w2);
        rf_store<true>(acc, b2, h2, LH);
      }
      wave_sync();
      MDP_STAMP(42);
      {
        const f32x4 acc = rh_acc(h2, LH, w3);
        if (r < MDP_ACT_DIM) {
#pragma unroll
          for (int i = 0; i < 4; ++i) lgj[(kq * 4 + i) * 8 + r] = acc[i] + b3;
        }
      }
      wave_sync();
      MDP_STAMP(43);
      if (lane < MDP_R) {  // distributions.py:264-266
        const int row = lane;
        float act[MDP_ACT_DIM];
        gumbel_softmax5_pre(lgj + row * 8, gn, act);
        const int dst = lq ? 0 : MDP_ACT_DIM * j;
        for (int k = 0; k < MDP_ACT_DIM; ++k) xa[row * ldA + dst + k] = act[k];
      }
      MDP_STAMP(2);
      MDP_CLK(44);
      w3v = Pc[nd.t[4].off + lane];
      __syncthreads();  // B2
    } else if (wave == 3) {
      // ---------------- online critic forward q(o, a) (maddpg.py:85-88, 104)
      f32x4 w1[20], w1b[2], w2[16];
      float w3[16];
      rf_load<20>(w1, Pc + nd.t[0].off, ka_c);
      rf_load<2>(w1b, Pc + nd.t[0].off + ka_c * RH, kb_c);
      rf_load<16>(w2, Pc + nd.t[2].off, RH);
      rq_load(w3, Pc + nd.t[4].off);
      const f32x4 b1 = ld4(Pc + nd.t[1].off + 4 * r), b2 = ld4(Pc + nd.t[3].off + 4 * r);
      const float b3 = Pc[nd.t[5].off];
      lds_wait(&rows_ready, 4);
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<20>(acc, rowbuf + xo_c, ldr, ka_c, w1);
        if (kb_c) rf_acc<2>(acc, rowbuf + ag.act_off, ldr, kb_c, w1b);
        rf_store<true>(acc, b1, h1c, LH);
      }
      wave_sync();
      {
        f32x4 acc[4];
        rf_zero(acc);
        rf_acc<16>(acc, h1c, LH, RH, w2);
        rf_store<true>(acc, b2, h2c, LH);
      }
      wave_sync();
      MDP_STAMPW(3);
      w3v = Pc[nd.t[4].off + lane];
      __syncthreads();  // B2
      const float q = rq_head(h2c, LH, w3) + b3;
      if ((lane & 3) == 0) qv[lane >> 2] = q;
    } else {
      w3v = Pc[nd.t[4].off + lane];
      __syncthreads();  // B2
    }
    // The critic backward is linear in the per-row dL/dq (maddpg.py:91):
    // d2 = dq o v with v = W3 o [h2c > 0], dh1 = dq o u with u = (v W2^T) o
    // [h1c > 0].  u needs no TD target, so waves 0..3 compute it while waves
    // 4..7 run the target critic and the TD error, and scale it by dq once wave
    // 4 has it: the dh1 tiles leave the critical path and dW2, dW1 run as one
    // phase after B5.  v (rows 4 wave .. 4 wave + 3) in the d2 buffer until
    // wave 4 overwrites it with dq o v after B4.
    // The W2^T tile is requested only here: issued with the prologue's loads it
    // competed with the target actor's weights on the critical path, and u is
    // needed only once wave 4 has dq (after B4).
    rdg_load(wt, Pc + nd.t[2].off, 16 * wave + r, true);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 4 * wave + i;
      d2[rr * LD + lane] = h2c[rr * LH + lane] > 0.f ? w3v : 0.f;
    }
    __syncthreads();  // B3
    float vx[16];  // this lane's v fragments (row lane & 15), read before wave 4 overwrites d2
    {
      const float* yr = d2 + r * LD + 16 * kq;
#pragma unroll
      for (int q = 0; q < 16; ++q) vx[q] = yr[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // B4
    f32x4 u = {0.f, 0.f, 0.f, 0.f};  // u tile `wave` (columns 16 wave .. 16 wave + 15), rdg_acc's chain
#pragma unroll
    for (int q = 0; q < 16; ++q) u = MDP_MFMA(vx[q], wt[q >> 2][q & 3], u);
    lds_wait(&dq_ready, 1);
    {
      const int col = 16 * wave + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i;
        d1[row * LD + col] = h1c[row * LH + col] > 0.f ? dq[row] * u[i] : 0.f;
      }
    }
    __syncthreads();  // B5: d2, d1 ready
  } else {
    // ---------------- target critic Q'(o', a~), one 16-column tile per wave
    const int tt = wave - 4, col = 16 * tt + r;
    // the replay gather is issued first, by these waves only (their own weights are few
    // and needed late); waves 0..3 start on their weight loads at once
    if (post) load_rows16_part(a.cpre_rows + (int64_t)r0 * T.row_stride, T.row_stride, rowbuf, ldr, 256, 256);
    else gather_rows16_part(a.replay, T.row_stride, idx, r0, nvalid, rowbuf, ldr, 256, 256);
    lds_signal(&rows_ready);
#ifdef MDP_STAMPS
    if (tt == 0) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      MDP_STAMPW(15);
    }
#endif
    float wa[16], wb[5], w2[16], w3[16];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ks = post ? cpre_split(pprev) : 0;
    if (post) {  // the accumulator up to k-step ks from cpre; W1 rows of the a~ k-steps from ks on
      rt_load_k<5>(wb, Pt + nd.t[0].off + (ka_t + 4 * ks) * RH, RH, col, kb - 4 * ks);
      const float* src = a.cpre + (int64_t)r0 * MDP_CPRE_W + 128 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = src[(kq * 4 + i) * MDP_CPRE_W];
    } else {
      rt_load<16>(wa, Pt + nd.t[0].off, RH, col, ka_t);
      rt_load<5>(wb, Pt + nd.t[0].off + ka_t * RH, RH, col, kb);
    }
    rt_load<16>(w2, Pt + nd.t[2].off, RH, col, RH);
    const float b1 = Pt[nd.t[1].off + col], b2 = Pt[nd.t[3].off + col];
    if (tt == 0) rq_load(w3, Pt + nd.t[4].off);
    const float b3 = Pt[nd.t[5].off];
    const float w3c = Pc[nd.t[4].off + lane];  // d2 = dq * W3 of the online critic
    lds_wait(&rows_ready, 4);
    if (!post) rt_acc<16>(acc, rowbuf + xo_t, ldr, ka_t, wa);
    __syncthreads();  // B2: a~ ready
    if (tt == 0) MDP_STAMPW(4);
    if (post) rt_acc<5>(acc, xa + 4 * ks, ldA, kb - 4 * ks, wb);
    else rt_acc<5>(acc, xa, ldA, kb, wb);
#pragma unroll
    for (int i = 0; i < 4; ++i) h1t[(kq * 4 + i) * LH + col] = fmaxf(acc[i] + b1, 0.f);
    __syncthreads();  // B3
    if (tt == 0) MDP_STAMPW(5);
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    rt_acc<16>(acc, h1t, LH, RH, w2);
#pragma unroll
    for (int i = 0; i < 4; ++i) h2t[(kq * 4 + i) * LH + col] = fmaxf(acc[i] + b2, 0.f);
    __syncthreads();  // B4
    if (tt == 0) MDP_STAMPW(6);
    double s_l = 0.0, s_y = 0.0, s_r = 0.0, s_q = 0.0;  // wave 4's loss / stat partials (rows = lanes)
    if (tt == 0) {
      // fp64 TD target (maddpg.py:186), loss partials, dL/dq = 2 (q - y) / B
      const float qt = rq_head(h2t, LH, w3) + b3;
      if ((lane & 3) == 0) qn[lane >> 2] = qt;
      wave_sync();
      float g = 0.f;
      if (lane < nvalid) {
        const double rew = (double)rowbuf[lane * ldr + ag.rew_off];
        const double done = (double)rowbuf[lane * ldr + ag.done_off];
        const double qnv = (double)qn[lane];
        const double y64 = rew + a.gamma * (1.0 - done) * qnv;
        const float y = (float)y64;
        const float diff = qv[lane] - y;
        g = (2.0f * diff) * a.inv_b;
        s_l = (double)diff * (double)diff;
        s_y = y64;
        s_r = rew;
        s_q = qnv;
        y_out[r0 + lane] = y64;
      }
      if (lane < MDP_R) dq[lane] = g;
      lds_signal(&dq_ready);
      MDP_STAMPW(60);
      wave_sync();
      // dW3 = h2^T dq, db3 = sum dq, d2 = (dq W3^T) o [h2 > 0]   (lane = hidden unit)
      float s = 0.f, sb = 0.f;
#pragma unroll
      for (int rr = 0; rr < MDP_R; ++rr) {
        const float h = h2c[rr * LH + lane], dqr = dq[rr];
        s = fmaf(h, dqr, s);
        sb += dqr;
        d2[rr * LD + lane] = h > 0.f ? dqr * w3c : 0.f;
      }
      MDP_STAMPW(61);
      slab_st(slab + nd.t[4].off + lane, s);
      if (lane == 0) slab_st(slab + nd.t[5].off, sb);
      MDP_STAMPW(7);
    }
    __syncthreads();  // B5
    if (tt == 0) {
      MDP_STAMPW(8);
      // the update's stats (maddpg.py:196): partial sums of this tile, beside the backward
      s_l = sum16(s_l);
      s_y = sum16(s_y);
      s_r = sum16(s_r);
      s_q = sum16(s_q);
      if (lane == 0) {
        double* st = slab_stat + (int64_t)bx * 8;
        st[0] = s_l;
        st[1] = s_y;
        st[2] = s_r;
        st[3] = s_q;
      }
    }
  }
  // one phase: dW2 = h1^T d2, dW1 = x^T dh1, db2 and db1 = column sums of d2, dh1
  // (wgrad_multi here -- every tile's operands read first, the chains
  // interleaved, stores last -- measured slower: S2 1.074M -> 1.048M with all
  // five tiles of a wave at once, 1.064M as 2 + 3: the stores of the first
  // tiles no longer drain behind the later tiles' work)
  CRIT_T(0);
  wgrad_waves(h1c, LH, RH, d2, LD, RH, slab + nd.t[2].off, 0, 8);
  CRIT_T(1);
  wgrad_waves(rowbuf + xo_c, ldr, ka_c, d1, LD, RH, slab + nd.t[0].off, 0, 8);
  CRIT_T(2);
  if (kb_c) wgrad_waves(rowbuf + ag.act_off, ldr, kb_c, d1, LD, RH, slab + nd.t[0].off + ka_c * RH, 0, 8);
  CRIT_T(3);
  if (wave == 4) MDP_STAMPW(9);
  if (wave == 5) colsum64(d2, LD, slab + nd.t[3].off);
  if (wave == 7) colsum64(d1, LD, slab + nd.t[1].off);
  CRIT_T(4);
  MDP_STAMP(10);
  MDP_WG_END(0);
}

__global__ __launch_bounds__(512) void k_actor_grad_r(ActorArgs a) {
  MDP_KARG_TOUCH("s"(a.agent), "s"(a.slab_stride), "s"(a.cpre_agent), "s"(a.topo.n), "s"(gridDim.x));
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ int rows_ready;
  __shared__ int fwd_issued;  // waves 0..3 issued the loads the critic forward needs first
  BUD_BEGIN(1, a.agent, a.multi);
  MDP_WG_START(1);
  MDP_TL(a.ctl, 2, 0);
  int agent = a.agent, bx = blockIdx.x;
  if (a.cpre) {  // workgroups [B/16, 2 B/16): the next critic step's independent work (strict mode)
    const int nwg = (a.B + MDP_RW - 1) / MDP_RW;
    if (bx >= nwg) {
      MDP_TL_ROLE(2, 1);
      critic_pre_tile(a, lds, &rows_ready, bx - nwg);
      MDP_WG_END(1);
      return;
    }
  }
  if (a.multi > 1) {  // throughput mode: every agent's actor step in this launch
    const int nwg = (a.B + MDP_RW - 1) / MDP_RW;
    agent = bx / nwg;
    bx -= agent * nwg;
  }
  const int32_t* idx = a.multi > 1 ? a.idx + (int64_t)agent * a.B : a.idx;
  const float* u_act = (a.multi > 1 && a.u_act) ? a.u_act + (int64_t)agent * a.B * MDP_ACT_DIM : a.u_act;
  const Topo& T = a.topo;
  MDP_KARG_TOUCH(MDP_KARG_ADESC(T.ag[agent]));
  const ADesc& ag = T.ag[agent];
  const NDesc& na = ag.actor;
  const NDesc& nc = ag.critic;
  const bool lq = ag.local_q != 0;
  const int ldr = lds_ld(T.row_stride);
  const int ka_c = lq ? ag.obs_dim : ag.cin;  // critic input from the replay row (a_i rows masked)
  const int xo_c = lq ? ag.obs_off : 0;
  LdsCarve cv(lds);
  float* rowbuf = cv.take(MDP_R * ldr);
  float* av = cv.take(MDP_R * 8);
  float* lg = cv.take(MDP_R * 8);
  float* da = cv.take(MDP_R * 8);
  float* dl = cv.take(MDP_R * 8);
  float* qv = cv.take(MDP_R);
  float* h1a = cv.take(MDP_R * LH);
  float* h2a = cv.take(MDP_R * LH);
  float* h1c = cv.take(MDP_R * LH);
  float* d2c = cv.take(MDP_R * LD);
  float* d1c = cv.take(MDP_R * LD);
  float* d2a = cv.take(MDP_R * LD);
  float* d1a = cv.take(MDP_R * LD);
  float* l1part = cv.take(2 * 64 * 16);  // critic L1 partial accumulators of waves 2, 3
  float* gwpart = cv.take(4 * MDP_ACT_DIM * 64);  // dW3a partials of the four row quarters
  float* qpart = cv.take(4 * MDP_R);     // critic head partials of the four L2 column tiles

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int r0 = bx * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const uint32_t ctr = ctr_load(a.ctl) + (a.multi > 1 ? (uint32_t)agent : 0u);
  const float* P = a.theta;
  // critic L1 replay-part contraction split over waves 1..3 (KC rows each)
  constexpr int KC = 28, KSC = KC / 4;
  const int64_t ao = a.multi > 1 ? (int64_t)agent : 0;
  float* slab = a.slab + ao * a.slab_agent_stride + (int64_t)bx * a.slab_stride - na.off;
  double* slab_stat = a.slab_stat + ao * (int64_t)((a.B + MDP_R - 1) / MDP_R) * 8;
  MDP_STAMP(16);
  if (threadIdx.x == 0) rows_ready = 0;
  if (threadIdx.x == 1) fwd_issued = 0;
  __syncthreads();  // B0

  // wave 0's loss / stat terms (rows = lanes 0..15), summed at the end, off the path to B4b
  double s_q = 0.0, s_p = 0.0;
  if (wave < 4) {
    if (wave == 0) {
      // ---------------- actor forward on obs_i -> logits p (maddpg.py:39), sample a_i (:49)
      f32x4 wda[4];
      float w3a[MDP_ACT_DIM];
      float w2t[16];  // critic L2 column tile 0
      float b2t, w3t;
      if (a.apre) {  // computed by the critic launch's extra workgroups: load the block
        // issue order: the block (the sample a_i is on the path to B2), the
        // critic L2 tile, then -- after fwd_issued -- the backward's weights
        const float* src = a.apre + (int64_t)r0 * MDP_APRE_W;
        f32x4 v[MDP_APRE_W / 16];
#pragma unroll
        for (int k = 0; k < MDP_APRE_W / 16; ++k) v[k] = ld4(src + 4 * (lane + 64 * k));
        rt_load<16>(w2t, P + nc.t[2].off, RH, r, RH);
        b2t = P[nc.t[3].off + r];
        w3t = P[nc.t[4].off + r];
        lds_signal(&fwd_issued);
        rdg_load(wda, P + nc.t[0].off + ag.a_in_off * RH, min(r, MDP_ACT_DIM - 1), r < MDP_ACT_DIM);
#pragma unroll
        for (int k = 0; k < MDP_ACT_DIM; ++k) w3a[k] = P[na.t[4].off + lane * MDP_ACT_DIM + k];
#pragma unroll
        for (int k = 0; k < MDP_APRE_W / 16; ++k)
          *reinterpret_cast<f32x4*>(apre_lds(lane + 64 * k, h1a, h2a, lg, av)) = v[k];
        wave_sync();
      } else {
        lds_signal(&fwd_issued);
        actor_fwd_wave(P, na, ag, rowbuf, ldr, u_act, nvalid, r0, a.seed, agent, ctr, &rows_ready, 6, h1a, h2a, lg,
                       av);
        // backward-phase weights: W1c rows of the a_i input (for da) and W3 of the actor (for d2a)
        rdg_load(wda, P + nc.t[0].off + ag.a_in_off * RH, min(r, MDP_ACT_DIM - 1), r < MDP_ACT_DIM);
#pragma unroll
        for (int k = 0; k < MDP_ACT_DIM; ++k) w3a[k] = P[na.t[4].off + lane * MDP_ACT_DIM + k];
        rt_load<16>(w2t, P + nc.t[2].off, RH, r, RH);
        b2t = P[nc.t[3].off + r];
        w3t = P[nc.t[4].off + r];
      }
      MDP_STAMP(18);
      __syncthreads();  // B2: a_i and the L1 thirds ready
      __syncthreads();  // B2b: h1c ready
      critic_l2_tile(h1c, w2t, b2t, w3t, 0, nvalid, a.neg_inv_b, d2c, qpart);
      __syncthreads();  // B3: critic forward, d2c ready
      if (lane < MDP_R) qv[lane] = ((qpart[lane] + qpart[MDP_R + lane]) + qpart[2 * MDP_R + lane]) +
                                   qpart[3 * MDP_R + lane] + P[nc.t[5].off];
      __syncthreads();  // B4: dh1c ready
      MDP_STAMP(23);
      // da[r][k] = sum_h dh1c[r][h] W1c[a_in_off + k][h]
      {
        const f32x4 acc = rdg_acc(d1c, LD, wda);
        if (r < MDP_ACT_DIM) {
#pragma unroll
          for (int i = 0; i < 4; ++i) da[(kq * 4 + i) * 8 + r] = acc[i];
        }
      }
      wave_sync();
      // softmax backward + regulariser: dlogits = (da - sum(a da)) a + reg 2 p / (B A); loss terms
      if (lane < MDP_R) {
        float dot = 0.f;
        for (int k = 0; k < MDP_ACT_DIM; ++k) dot += da[lane * 8 + k] * av[lane * 8 + k];
        for (int k = 0; k < MDP_ACT_DIM; ++k) {
          const float g = (da[lane * 8 + k] - dot) * av[lane * 8 + k] + lg[lane * 8 + k] * a.reg_scale;
          dl[lane * 8 + k] = lane < nvalid ? g : 0.f;
        }
        if (lane < nvalid) {
          s_q = (double)qv[lane];
          for (int k = 0; k < MDP_ACT_DIM; ++k) {
            const double p = (double)lg[lane * 8 + k];
            s_p += p * p;
          }
        }
      }
      __syncthreads();  // B4b: dlogits ready
      d2a_rows(h2a, dl, w3a, d2a, gwpart, 0);
      MDP_STAMP(24);
      __syncthreads();  // B5: d2a ready
      dw3a_store(gwpart, dl, slab + na.t[4].off, slab + na.t[5].off);
    } else {
      // ---------------- critic (post-step weights) forward with a_i = the sample (maddpg.py:48-52)
      // waves 2, 3 gather their share of the replay rows first
      if (wave > 1) {
        if (a.apre) load_rows16_part(a.apre_rows + (int64_t)r0 * T.row_stride, T.row_stride, rowbuf, ldr, 128, 384);
        else gather_rows16_part(a.replay, T.row_stride, idx, r0, nvalid, rowbuf, ldr, 128, 384);
      }
      if (wave > 1) lds_signal(&rows_ready);
      const int k0 = KC * (wave - 1);  // this wave's third of the replay-part contraction
      f32x4 w1[KSC];
      rf_load<KSC>(w1, P + nc.t[0].off + k0 * RH, max(min(ka_c - k0, KC), 0));  // a_i rows: zeroed in rf_acc
      f32x4 w1b[2], b1;
      if (wave == 1) {
        rf_load<2>(w1b, P + nc.t[0].off + ag.a_in_off * RH, MDP_ACT_DIM);
        b1 = ld4(P + nc.t[1].off + 4 * r);
      }
      float w2t[16];  // critic L2 column tile `wave`
      rt_load<16>(w2t, P + nc.t[2].off, RH, 16 * wave + r, RH);
      const float b2t = P[nc.t[3].off + 16 * wave + r], w3t = P[nc.t[4].off + 16 * wave + r];
      lds_signal(&fwd_issued);
      lds_wait(&rows_ready, 6);
      if (wave == 1) MDP_STAMPW(56);
      f32x4 acc[4];
      rf_zero(acc);
      if (k0 < ka_c)
        rf_acc<KSC>(acc, rowbuf + xo_c + k0, ldr, min(ka_c - k0, KC), w1, ag.a_in_off - k0,
                    ag.a_in_off + MDP_ACT_DIM - k0);
      if (wave == 1) MDP_STAMPW(57);
      if (wave == 3) MDP_STAMPW(58);
      if (wave > 1) {  // hand the partial accumulators to wave 1 (lane-major, 16 floats each)
        float* pp = l1part + ((wave - 2) * 64 + lane) * 16;
#pragma unroll
        for (int t = 0; t < 4; ++t) *reinterpret_cast<f32x4*>(pp + 4 * t) = acc[t];
      }
      __syncthreads();  // B2
      if (wave == 1) {
        MDP_STAMPW(19);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          acc[t] += *reinterpret_cast<const f32x4*>(l1part + lane * 16 + 4 * t);
          acc[t] += *reinterpret_cast<const f32x4*>(l1part + (64 + lane) * 16 + 4 * t);
        }
        rf_acc<2>(acc, av, 8, MDP_ACT_DIM, w1b);
        rf_store<true>(acc, b1, h1c, LH);
      }
      __syncthreads();  // B2b: h1c ready
      critic_l2_tile(h1c, w2t, b2t, w3t, wave, nvalid, a.neg_inv_b, d2c, qpart);
      if (wave == 1) MDP_STAMPW(20);
      float w3a[MDP_ACT_DIM];
#pragma unroll
      for (int k = 0; k < MDP_ACT_DIM; ++k) w3a[k] = P[na.t[4].off + lane * MDP_ACT_DIM + k];
      __syncthreads();  // B3
      __syncthreads();  // B4
      __syncthreads();  // B4b
      d2a_rows(h2a, dl, w3a, d2a, gwpart, wave);
      __syncthreads();  // B5
    }
    // dW2a = h1a^T d2a (waves 0..3, four tiles each, interleaved), db2a
    wgrad_multi<4>(WgJob{h1a, d2a, slab + na.t[2].off, LH, RH, LD, RH}, WgJob{nullptr, nullptr, nullptr, 0, 0, 0, 64},
                   WgJob{nullptr, nullptr, nullptr, 0, 0, 0, 64}, 0, 4);
    if (wave == 3) colsum64(d2a, LD, slab + na.t[3].off);
    __syncthreads();  // B6
  } else {
    // ---------------- dgrad tiles: dh1c through the critic, dh1a through the actor
    const int tt = wave - 4;
    // waves 2..7 gather the replay rows (first); waves 0, 1 start on their weights at once
    if (a.apre) load_rows16_part(a.apre_rows + (int64_t)r0 * T.row_stride, T.row_stride, rowbuf, ldr, 128, 384);
    else gather_rows16_part(a.replay, T.row_stride, idx, r0, nvalid, rowbuf, ldr, 128, 384);
    lds_signal(&rows_ready);
    f32x4 wc[4], wa[4];
    lds_wait(&fwd_issued, 4);  // the critic forward's loads go first
    rdg_load(wc, P + nc.t[2].off, 16 * tt + r, true);
    rdg_load(wa, P + na.t[2].off, 16 * tt + r, true);
    __syncthreads();  // B2
    __syncthreads();  // B2b
    __syncthreads();  // B3
    if (tt == 0) MDP_STAMPW(21);
    dgrad_tile(d2c, wc, h1c, d1c, tt);
    __syncthreads();  // B4
    if (tt == 0) MDP_STAMPW(22);
    __syncthreads();  // B4b
    __syncthreads();  // B5
    if (tt == 0) MDP_STAMPW(25);
    dgrad_tile(d2a, wa, h1a, d1a, tt);
    __syncthreads();  // B6
    if (tt == 0) MDP_STAMPW(26);
  }
  // dW1a = obs_i^T dh1a over all waves, db1a
  wgrad_waves(rowbuf + ag.obs_off, ldr, ag.obs_dim, d1a, LD, RH, slab + na.t[0].off, 0, 8);
  if (wave == 7) colsum64(d1a, LD, slab + na.t[1].off);
  if (wave == 0) {  // the update's stats: this tile's partial sums
    s_q = sum16(s_q);
    s_p = sum16(s_p);
    if (lane == 0) {
      double* st = slab_stat + (int64_t)bx * 8;
      st[0] = s_q;
      st[1] = s_p;
    }
  }
  MDP_STAMP(27);
  MDP_WG_END(1);
}

namespace {
template <typename K, typename A>
hipError_t launch_r(K kern, const A& a, int lds, hipStream_t s, bool& attr, int extra = 0) {
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, MDP_LDS_BUDGET);
    (void)hipGetLastError();
    attr = true;
  }
  const int per = (a.B + MDP_RW - 1) / MDP_RW;
  mdp_launch(kern, dim3(per * (a.multi > 1 ? a.multi : 1) + extra), dim3(512), lds, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t mdp_launch_critic_grad_r(const CriticArgs& a, int lds_bytes, hipStream_t s) {
  static bool attr = false;
  const int per = (a.B + MDP_RW - 1) / MDP_RW;
  // grid: critic row tiles | actor-forward row tiles (a.apre) | the index draw (pf_count; last)
  return launch_r(k_critic_grad_r, a, lds_bytes, s, attr, (a.apre ? per : 0) + (a.pf_count > 0 ? 1 : 0));
}
hipError_t mdp_launch_actor_grad_r(const ActorArgs& a, int lds_bytes, hipStream_t s) {
  static bool attr = false;
  // grid: actor row tiles | the next critic step's row tiles (a.cpre)
  return launch_r(k_actor_grad_r, a, lds_bytes, s, attr, a.cpre ? (a.B + MDP_RW - 1) / MDP_RW : 0);
}

#ifdef MDP_TIMELINE
extern "C" int mdp_debug_tl_r(unsigned long long* out, int reset) {
  const size_t n = sizeof(unsigned long long) * MDP_TL_SLOTS * MDP_TL_WG * 2;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_mdp_tl)) != hipSuccess) return -1;
    return hipMemset(p, 0, n) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_tl), n) == hipSuccess ? 0 : -1;
}
#endif

#ifdef MDP_BUDGET
// [2][160][MDP_BUD_N] phase points of the chosen agent's last critic / actor launch; reset: zero them
extern "C" int mdp_debug_budget(unsigned long long* out, int reset) {
  const size_t n = sizeof(unsigned long long) * 2 * 160 * MDP_BUD_N;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_bud)) != hipSuccess) return -1;
    return hipMemset(p, 0, n) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bud), n) == hipSuccess ? 0 : -1;
}
#endif
#ifdef MDP_STAMPS
// diagnostic build: stamps of this translation unit's kernels (own code object)
extern "C" int mdp_debug_stamps_r(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
// the critic step's per-wave points after B5 [64][8][6] (CRIT_T)
extern "C" int mdp_debug_crit_times(unsigned long long* t) {
  return hipMemcpyFromSymbol(t, HIP_SYMBOL(g_crit_t), sizeof(unsigned long long) * 64 * 8 * 6) == hipSuccess ? 0 : -1;
}
// critic_pre's per-wave phase points [64][8][6] (CPRE_T)
extern "C" int mdp_debug_cpre_times(unsigned long long* t) {
  return hipMemcpyFromSymbol(t, HIP_SYMBOL(g_cpre_t), sizeof(unsigned long long) * 64 * 8 * 6) == hipSuccess ? 0 : -1;
}
// [2][512] starts, then [2][512][8] per-wave ends
extern "C" int mdp_debug_wg_times(unsigned long long* t0, unsigned long long* t1) {
  if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_wg_t0), sizeof(unsigned long long) * 2 * 512) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_wg_t1), sizeof(unsigned long long) * 2 * 512 * 8) == hipSuccess ? 0 : -1;
}
#endif
