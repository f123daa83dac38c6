// mdp_grads_pair.hip -- the general critic step (maddpg.py:180-188) as PAIRS of
// workgroups per 32 batch rows (gfx950).
//
// Why pairs.  The single-workgroup general kernel (mdp_grads.hip) runs every
// net of the step on 16 rows per CU.  A 16-row MFMA tile turns each 4-byte
// weight into 8 flops, so one CU needs ~32 B/clk of weights to keep its four
// SIMDs' fp32 MFMA busy -- the ceiling a CU reaches when every CU streams the
// same weights (tools/wstream.hip: 31-33 B/clk).  At S5 (tag N=6, H=128) the
// step streams ~830 KB of weights per 16 rows and ran at 28-32 % MFMA busy.
// Here each weight fragment feeds TWO row tiles (32 rows), and the nets are
// split between the two workgroups of a pair so the grid still covers the
// chip (B = 4096: 128 pairs = 256 workgroups):
//   A (blockIdx < P):  obs' rows -> every target actor (maddpg.py:184, the
//                      Gumbel sample distributions.py:264-266) -> a~ to pair_xa
//   B (blockIdx >= P): rows -> critic forward h1, h2, q and the target critic's
//                      obs' part of layer 1 (independent of a~) || wait for A
//                      -> target critic on a~, fp64 TD target, loss partials,
//                      backward, one partial-gradient slab per 32 rows.
// A never waits, and every A workgroup precedes every B workgroup in dispatch
// order, so B's wait always ends (the hand-off is bounded by a spin limit that
// records Ctl::fault like the optimizer's handshakes).  Hand-off protocol
// (MI355X_MICROARCH.md, inter-workgroup visibility): A's a~ stores are
// agent-scope (sc1) stores, every storing wave drains them (vmcnt(0)), then
// one lane adds 1 to pair_prod[p]; B's lane 0 polls pair_prod[p] until it
// passes B's own count pair_cons[p], bumps that count, and every a~ load is an
// agent-scope (sc1) load behind a workgroup barrier.  The counters need no
// reset: each launch adds exactly one to both.
//
// The MFMA k order per output element is one chain over the layer's inputs as
// in the single-workgroup kernel; the batch sum of each weight gradient runs
// over 32 rows inside the workgroup instead of two 16-row partials, so results
// agree with it (and the oracle) to fp32 rounding, not bitwise.
#include "mdp_device.h"
#include "mdp_kernels.h"

#ifndef MDP_PKS
#define MDP_PKS 8  // k-steps (of 4) per weight chunk of the pair phases
#endif

// diagnostic build (-DMDP_STAMPS): wall-clock stamps of pair 0 -- slots 0..31
// the actor workgroup (block 0), 32..63 the critic workgroup (block P)
#ifdef MDP_STAMPS
__device__ unsigned long long g_pair_stamps[64];
#define PSTAMP(i)                                                                            \
  do {                                                                                       \
    if ((blockIdx.x == 0 || (int)blockIdx.x == (a.B + MDP_PAIR_R - 1) / MDP_PAIR_R) && threadIdx.x == 0) \
      g_pair_stamps[(blockIdx.x ? 32 : 0) + (i)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
extern "C" int mdp_debug_stamps_pair(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pair_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#else
#define PSTAMP(i) \
  do {            \
  } while (0)
#endif

namespace {
constexpr int PR = MDP_PAIR_R;  // 32 rows: two 16-row MFMA tiles
constexpr uint32_t kPairSpin = 1u << 22;

// One dense layer of one net over 32 rows: Y[32][N] = act([init +] X[:, k0:K] W[k0:K, :] + b).
// X = lds + xoff, row r at X[r * ldx + k] with k the ABSOLUTE input index
// (a continuation over k0..K-1 points xoff at k = 0 of its buffer).
struct PJob {
  int xoff, ldx, k0, K;
  const float* W;  // [K][N] global
  const float* b;  // null: store the raw accumulator
  int ioff;        // >= 0: start from the raw accumulator lds[ioff + row * ldy + col]
  int yoff;        // Y = lds + yoff (row stride ldy)
};

// Units (job, g) own output columns 16 g .. 16 g + 15 over both 16-row tiles;
// a unit's k rows run in PIECES of up to 128 (32 MFMA k-steps).  A piece's
// weights are loaded whole into registers (32 floats per lane, one memory
// round trip) and each fragment feeds the two row tiles.  Pieces ping-pong
// between two register sets with the loop unrolled by two, so the next
// piece's loads are in flight during this piece's MFMAs and the compiler's
// wait is for exactly the piece it is about to use (a register copy of a
// prefetch buffer at the end of each iteration would wait for every load in
// flight -- the stamped cause of 2.5 us per 32-row chunk in a first version).
// The first piece of a phase is issued by phase_prime BEFORE the barrier that
// precedes the phase.  Units are dealt round-robin over waves [w0, w0 + nw).
struct Piece {
  float w[32];
  float bias;
};
struct PItem {
  int u, pc, g;
  PJob j;
};

template <class JobFn>
__device__ __forceinline__ bool item_first(PItem& it, int njobs, int N, int w0, int nw, JobFn& job) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ngr = N >> 4;
  it.u = wave - w0;
  it.pc = 0;
  if (wave < w0 || it.u >= nw || it.u >= njobs * ngr) return false;
  it.j = job(it.u / ngr);
  it.g = it.u % ngr;
  return true;
}
template <class JobFn>
__device__ __forceinline__ bool item_next(PItem& it, int njobs, int N, int nw, JobFn& job) {
  const int ngr = N >> 4;
  if (it.j.k0 + 128 * (it.pc + 1) < it.j.K) {
    ++it.pc;
    return true;
  }
  it.u += nw;
  it.pc = 0;
  if (it.u >= njobs * ngr) return false;
  it.j = job(it.u / ngr);
  it.g = it.u % ngr;
  return true;
}
__device__ __forceinline__ void piece_load(Piece& P, const PItem& it, int N) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int kb = it.j.k0 + 128 * it.pc, col = 16 * it.g + r;
  const float* W = it.j.W + col;
#pragma unroll
  for (int s = 0; s < 32; ++s)
    if (kb + 4 * s < it.j.K) P.w[s] = W[(int64_t)min(kb + 4 * s + kq, it.j.K - 1) * N];  // wave-uniform test
  P.bias = it.j.b ? it.j.b[col] : 0.f;
}
__device__ __forceinline__ void piece_run(float* lds, f32x4 (&acc)[2], const Piece& P, const PItem& it, int ldy) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const PJob& j = it.j;
  const int col = 16 * it.g + r;
  if (it.pc == 0) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      if (j.ioff >= 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[rt][i] = lds[j.ioff + (16 * rt + 4 * kq + i) * ldy + col];
      } else {
        acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  const float* X = lds + j.xoff;
  const int kb = j.k0 + 128 * it.pc;
#pragma unroll
  for (int s0 = 0; s0 < 32; s0 += 4) {
    if (kb + 4 * s0 >= j.K) break;  // wave-uniform
    float x[2][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = kb + 4 * (s0 + s) + kq, kc = min(k, j.K - 1);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const float v = X[(16 * rt + r) * j.ldx + kc];
        x[rt][s] = k < j.K ? v : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (kb + 4 * (s0 + s) < j.K) {
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[rt][s], P.w[s0 + s], acc[rt], 0, 0, 0);
      }
  }
  if (kb + 128 >= j.K) {  // last piece: bias, ReLU, store
    float* Y = lds + j.yoff + col;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[rt][i];
        Y[(16 * rt + 4 * kq + i) * ldy] = j.b ? fmaxf(v + P.bias, 0.f) : v;
      }
  }
}
template <class JobFn>
__device__ __forceinline__ void phase_prime(Piece& P0, int njobs, int N, int w0, int nw, JobFn job) {
  PItem it;
  if (item_first(it, njobs, N, w0, nw, job)) piece_load(P0, it, N);
}
// P0 holds this wave's first piece (phase_prime)
template <class JobFn>
__device__ __forceinline__ void phase_run(float* lds, Piece& P0, Piece& P1, int njobs, int N, int ldy, int w0, int nw,
                                          JobFn job) {
  PItem a;
  if (!item_first(a, njobs, N, w0, nw, job)) return;
  f32x4 acc[2];
  while (true) {
    PItem b = a;
    const bool hb = item_next(b, njobs, N, nw, job);
    if (hb) piece_load(P1, b, N);
    piece_run(lds, acc, P0, a, ldy);
    if (!hb) break;
    PItem c = b;
    const bool hc = item_next(c, njobs, N, nw, job);
    if (hc) piece_load(P0, c, N);
    piece_run(lds, acc, P1, b, ldy);
    if (!hc) break;
    a = c;
  }
}

// head over 32 rows on one wave: out[32][nout] = X[32][K] @ W[K][nout] + b,
// K = 4 KS, the fragments loaded ahead by head_load (both row tiles share them)
template <int KS>
__device__ __forceinline__ void head2_acc(const float (&w)[KS], float bias, const float* X, int ldx, int nout,
                                          float* out, int ldo) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s0 = 0; s0 < KS; s0 += 8) {
    float x[2][8];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) x[rt][s] = X[(16 * rt + r) * ldx + 4 * (s0 + s) + kq];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[rt][s], w[s0 + s], acc[rt], 0, 0, 0);
  }
  if (r < nout) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(16 * rt + kq * 4 + i) * ldo + r] = acc[rt][i] + bias;
  }
}

// rows [r0, r0 + 32) of the replay ring, float4 columns [c4a, c4b) -> buf[r][4 c4 - 4 c4a ..]
__device__ __forceinline__ void gather32(const float* __restrict__ replay, int stride, const int32_t* __restrict__ idx,
                                         int r0, int nvalid, int c4a, int c4b, float* buf, int ld) {
  const int w4 = c4b - c4a;
  for (int e = threadIdx.x; e < PR * w4; e += blockDim.x) {
    const int r = e / w4, c4 = e - r * w4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < nvalid) v = *reinterpret_cast<const float4*>(replay + (int64_t)idx[r0 + r] * stride + 4 * (c4a + c4));
    float* d = buf + r * ld + 4 * c4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}

// dW[K][N] tiles of X^T[K][32] @ dY[32][N] over waves [w0, w0 + wn) -> global (stride N)
__device__ __forceinline__ void wgrad32(const float* X, int ldx, int K, const float* dY, int ldy, int N,
                                        float* __restrict__ dW, int w0, int wn) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < w0 || wave >= w0 + wn) return;
  const int r = lane & 15, kq = lane >> 4;
  const int nmt = (K + 15) >> 4, nnt = N >> 4;
  for (int t = wave - w0; t < nmt * nnt; t += wn) {
    const int mt = t / nnt, nt = t - mt * nnt;
    const int feat = mt * 16 + r;
    const int fc = min(feat, K - 1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < PR; q += 4) {
      const int row = q + kq;
      const float xv = X[row * ldx + fc];
      const float a = feat < K ? xv : 0.f;
      const float g = dY[row * ldy + nt * 16 + r];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, g, acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = mt * 16 + kq * 4 + i;
      if (k < K) slab_st(dW + k * N + nt * 16 + r, acc[i]);
    }
  }
}

// dX[32][16-col tile nt] = (dY[32][N] @ W^T) masked by Hin > 0 (N a multiple of
// 64): contiguous transposed fragments (contraction order n = c0 + 16 kq + s),
// each fragment feeding both row tiles
__device__ __forceinline__ void dgrad32(const float* dY, int ldy, int N, const float* __restrict__ W, const float* Hin,
                                        int ldh, float* dX, int ldx, int nt) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int kk = nt * 16 + r;
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  f32x4 wa[4], wb[4];
  auto load = [&](f32x4(&w)[4], int c0) {
#pragma unroll
    for (int m = 0; m < 4; ++m) w[m] = *reinterpret_cast<const f32x4*>(W + (int64_t)kk * N + c0 + 16 * kq + 4 * m);
  };
  load(wa, 0);
  for (int c0 = 0; c0 < N; c0 += 64) {
    const bool more = c0 + 64 < N;
    if (more) load(wb, c0 + 64);
    float x[2][16];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int q = 0; q < 16; ++q) x[rt][q] = dY[(16 * rt + r) * ldy + c0 + 16 * kq + q];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[rt][q], wa[q >> 2][q & 3], acc[rt], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int m = 0; m < 4; ++m) wa[m] = wb[m];
    }
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * rt + kq * 4 + i;
      dX[row * ldx + kk] = Hin[row * ldh + kk] > 0.f ? acc[rt][i] : 0.f;
    }
}

__device__ __forceinline__ void colsum32(const float* X, int ldx, int ncols, float* __restrict__ out) {
  for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < PR; ++r) s += X[r * ldx + c];
    slab_st(out + c, s);
  }
}

// lanes 0..31 hold one value each; the sum in every lane (fixed order)
__device__ __forceinline__ double sum32(double v) {
  const int lane = threadIdx.x & 63;
  v = lane < PR ? v : 0.0;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint32_t ld_agent32(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agentf(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agentf(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

// ------------------------------------------------------- A: the target actors
template <int H>
__device__ __forceinline__ void pair_actors(const CriticArgs& a, float* lds, int p, int r0, int nvalid) {
  const Topo& T = a.topo;
  const int G = a.group, n = T.n, ldh = H + 1, S = PR * ldh;
  const int lo4 = T.ag[0].nobs_off & ~3, c4b = (T.ag[0].nobs_off + T.sum_obs + 3) >> 2;
  const int ldo = lds_ld(4 * c4b - lo4);
  LdsCarve cv(lds);
  float* ob = cv.take(PR * ldo);
  float* h1 = cv.take(G * S);
  float* h2 = cv.take(G * S);
  float* lg = cv.take(G * PR * 8);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const uint32_t ctr = a.ctl->upd_ctr + (a.multi > 1 ? (uint32_t)a.agent : 0u);
  const int o_ob = (int)(ob - lds), o_h1 = (int)(h1 - lds), o_h2 = (int)(h2 - lds);
  // layer `layer` of the target actors g0 .. g0 + ng - 1
  auto jobs = [&](int g0, int layer) {
    return [=, &T, &a](int jb) {
      const NDesc& an = T.ag[g0 + jb].actor;
      PJob j;
      j.k0 = 0;
      j.ioff = -1;
      if (layer == 0) {
        j.xoff = o_ob + T.ag[g0 + jb].nobs_off - lo4;
        j.ldx = ldo;
        j.K = T.ag[g0 + jb].obs_dim;
        j.W = a.target + an.t[0].off;
        j.b = a.target + an.t[1].off;
        j.yoff = o_h1 + jb * S;
      } else {
        j.xoff = o_h1 + jb * S;
        j.ldx = ldh;
        j.K = H;
        j.W = a.target + an.t[2].off;
        j.b = a.target + an.t[3].off;
        j.yoff = o_h2 + jb * S;
      }
      return j;
    };
  };
  constexpr int HKS = H / 4;
  Piece P0, P1;
  PSTAMP(0);
  phase_prime(P0, min(G, n), H, 0, nw, jobs(0, 0));
  gather32(a.replay, T.row_stride, a.idx, r0, nvalid, lo4 >> 2, c4b, ob, ldo);
  __syncthreads();
  PSTAMP(1);
  for (int g0 = 0; g0 < n; g0 += G) {
    const int ng = min(G, n - g0);
    phase_run(lds, P0, P1, ng, H, ldh, 0, nw, jobs(g0, 0));
    phase_prime(P0, ng, H, 0, nw, jobs(g0, 1));
    __syncthreads();
    PSTAMP(2 + 4 * (g0 / G));
    phase_run(lds, P0, P1, ng, H, ldh, 0, nw, jobs(g0, 1));
    // heads: actor jb on wave nw - 1 - jb (the waves with the fewest layer units),
    // both row tiles; fragments in P1's registers (free once the phase is done)
    float(&hw)[HKS] = *reinterpret_cast<float(*)[HKS]>(P1.w);
    float& hb = P1.bias;
    const int hj = nw - 1 - wave;
    if (hj < ng) head_load<HKS>(hw, hb, a.target + T.ag[g0 + hj].actor.t[4].off,
                                a.target + T.ag[g0 + hj].actor.t[5].off, MDP_ACT_DIM);
    __syncthreads();
    PSTAMP(3 + 4 * (g0 / G));
    if (hj < ng) head2_acc<HKS>(hw, hb, h2 + hj * S, ldh, MDP_ACT_DIM, lg + hj * PR * 8, 8);
    __syncthreads();
    PSTAMP(4 + 4 * (g0 / G));
    if (g0 + G < n) phase_prime(P0, min(G, n - g0 - G), H, 0, nw, jobs(g0 + G, 0));
    // Gumbel-softmax target actions (distributions.py:264-266) -> pair_xa
    for (int e = tid; e < ng * PR; e += blockDim.x) {
      const int jb = e / PR, row = e - jb * PR, j = g0 + jb;
      float u[MDP_ACT_DIM], act[MDP_ACT_DIM];
      if (a.u_tgt) {
        for (int k = 0; k < MDP_ACT_DIM; ++k)
          u[k] = row < nvalid ? a.u_tgt[((int64_t)j * a.B + r0 + row) * MDP_ACT_DIM + k] : 0.5f;
      } else {
        uniforms5(a.seed, (uint32_t)((a.agent << 8) | (j + 1)), ctr, (uint32_t)(r0 + row), u);
      }
      gumbel_softmax5(lg + (jb * PR + row) * 8, u, act);
      float* dst = a.pair_xa + (int64_t)(r0 + row) * (MDP_ACT_DIM * n) + MDP_ACT_DIM * j;
      for (int k = 0; k < MDP_ACT_DIM; ++k) st_agentf(dst + k, act[k]);
    }
    PSTAMP(5 + 4 * (g0 / G));
  }
  // publish: every storing wave drains its sc1 stores, then one add
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_fetch_add(a.pair_prod + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  PSTAMP(15);
}

// ------------------------------------------- B: critic, target critic, backward
template <int H>
__device__ __forceinline__ void pair_critic(const CriticArgs& a, float* lds, int p, int r0, int nvalid) {
  constexpr int NT = H / 16, HKS = H / 4;
  const Topo& T = a.topo;
  const ADesc& ag = T.ag[a.agent];
  const NDesc& nd = ag.critic;
  const int n = T.n, ldh = H + 1, S = PR * ldh, ldr = lds_ld(T.row_stride), nax = MDP_ACT_DIM * n;
  const int ldx = lds_ld(nax);
  LdsCarve cv(lds);
  float* rowbuf = cv.take(PR * ldr);
  float* h1c = cv.take(S);
  float* h2c = cv.take(S);
  float* xl = cv.take(S);  // target critic layer 1: raw accumulator over obs'
  float* hA = cv.take(S);
  float* hB = cv.take(S);
  float* xa = cv.take(PR * ldx);  // a~ of every agent
  float* qv = cv.take(PR * 8);
  float* qn = cv.take(PR * 8);
  float* spare = cv.take(PR * 8);
  float* dq = cv.take(PR);
  (void)spare;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = blockDim.x >> 6;
  const int o_row = (int)(rowbuf - lds), o_h1c = (int)(h1c - lds), o_h2c = (int)(h2c - lds), o_xl = (int)(xl - lds);
  const int o_hA = (int)(hA - lds), o_hB = (int)(hB - lds), o_xa = (int)(xa - lds);
  const float* Pt = a.target;
  // critic layer 1 on [obs_all | act_all] (the row prefix) and the target
  // critic's obs' part of layer 1 (raw, maddpg.py:86) -- neither needs a~
  auto l1 = [&](int jb) {
    PJob j;
    j.k0 = 0;
    j.ioff = -1;
    j.ldx = ldr;
    if (jb == 0) {
      j.xoff = o_row;
      j.K = ag.cin;
      j.W = a.theta + nd.t[0].off;
      j.b = a.theta + nd.t[1].off;
      j.yoff = o_h1c;
    } else {
      j.xoff = o_row + T.ag[0].nobs_off;
      j.K = T.sum_obs;
      j.W = Pt + nd.t[0].off;
      j.b = nullptr;
      j.yoff = o_xl;
    }
    return j;
  };
  auto dense = [&](int xoff, int ldxx, int k0, int K, const float* W, const float* b, int ioff, int yoff) {
    return [=](int) {
      PJob j;
      j.xoff = xoff;
      j.ldx = ldxx;
      j.k0 = k0;
      j.K = K;
      j.W = W;
      j.b = b;
      j.ioff = ioff;
      j.yoff = yoff;
      return j;
    };
  };
  auto l2 = dense(o_h1c, ldh, 0, H, a.theta + nd.t[2].off, a.theta + nd.t[3].off, -1, o_h2c);
  // target critic: layer 1 continued over the a~ inputs k = sum_obs .. cin-1
  // from the stored raw obs' accumulator, then layer 2
  auto t1 = dense(o_xa - T.sum_obs, ldx, T.sum_obs, ag.cin, Pt + nd.t[0].off, Pt + nd.t[1].off, o_xl, o_hA);
  auto t2 = dense(o_hA, ldh, 0, H, Pt + nd.t[2].off, Pt + nd.t[3].off, -1, o_hB);
  Piece P0, P1;
  float(&hw)[HKS] = *reinterpret_cast<float(*)[HKS]>(P1.w);  // head fragments: P1's registers
  float& hb = P1.bias;
  PSTAMP(0);
  phase_prime(P0, 2, H, 0, nw, l1);
  gather32(a.replay, T.row_stride, a.idx, r0, nvalid, 0, T.row_stride >> 2, rowbuf, ldr);
  __syncthreads();
  PSTAMP(1);
  phase_run(lds, P0, P1, 2, H, ldh, 0, nw, l1);
  phase_prime(P0, 1, H, 0, NT, l2);
  __syncthreads();
  PSTAMP(2);
  phase_run(lds, P0, P1, 1, H, ldh, 0, NT, l2);
  if (wave == NT) head_load<HKS>(hw, hb, a.theta + nd.t[4].off, a.theta + nd.t[5].off, 1);
  phase_prime(P0, 1, H, 0, NT, t1);
  __syncthreads();
  PSTAMP(3);
  // q head || wait for the target actions
  if (wave == NT) {
    head2_acc<HKS>(hw, hb, h2c, ldh, 1, qv, 8);
  } else if (wave == nw - 1 && lane == 0) {
    const uint32_t want = ld_agent32(a.pair_cons + p) + 1u;
    uint32_t it = 0;
    while ((int32_t)(ld_agent32(a.pair_prod + p) - want) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > kPairSpin) {
        __hip_atomic_store(const_cast<uint32_t*>(&a.ctl->fault), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    st_agent32(a.pair_cons + p, want);
  }
  __syncthreads();
  PSTAMP(4);
  for (int e = tid; e < PR * nax; e += blockDim.x) {
    const int r = e / nax, c = e - r * nax;
    xa[r * ldx + c] = ld_agentf(a.pair_xa + (int64_t)(r0 + r) * nax + c);
  }
  __syncthreads();
  PSTAMP(5);
  phase_run(lds, P0, P1, 1, H, ldh, 0, NT, t1);
  phase_prime(P0, 1, H, 0, NT, t2);
  __syncthreads();
  PSTAMP(6);
  phase_run(lds, P0, P1, 1, H, ldh, 0, NT, t2);
  if (wave == NT) head_load<HKS>(hw, hb, Pt + nd.t[4].off, Pt + nd.t[5].off, 1);
  __syncthreads();
  PSTAMP(7);
  if (wave == NT) head2_acc<HKS>(hw, hb, hB, ldh, 1, qn, 8);
  __syncthreads();
  PSTAMP(8);
  // fp64 TD target (maddpg.py:186), loss partials, dL/dq = 2 (q - y) / B
  if (wave == 0) {
    double s_l = 0.0, s_y = 0.0, s_r = 0.0, s_q = 0.0;
    float g = 0.f;
    if (lane < nvalid) {
      const double rew = (double)rowbuf[lane * ldr + ag.rew_off];
      const double done = (double)rowbuf[lane * ldr + ag.done_off];
      const double qnx = (double)qn[lane * 8];
      const double y64 = rew + a.gamma * (1.0 - done) * qnx;
      const float y = (float)y64;
      const float diff = qv[lane * 8] - y;
      g = (2.0f * diff) * a.inv_b;
      s_l = (double)diff * (double)diff;
      s_y = y64;
      s_r = rew;
      s_q = qnx;
      a.y_out[r0 + lane] = y64;
    }
    if (lane < PR) dq[lane] = g;
    s_l = sum32(s_l);
    s_y = sum32(s_y);
    s_r = sum32(s_r);
    s_q = sum32(s_q);
    if (lane == 0) {
      double* st = a.slab_stat + (int64_t)p * 8;
      st[0] = s_l;
      st[1] = s_y;
      st[2] = s_r;
      st[3] = s_q;
    }
  }
  __syncthreads();
  PSTAMP(9);
  // backward through the critic (tf.gradients of q_loss w.r.t. q_func vars)
  float* slab = a.slab + (int64_t)p * a.slab_stride - nd.off;
  const float* W3 = a.theta + nd.t[4].off;
  float* d2 = hA;
  float* d1 = hB;
  if (tid < H) {
    float s = 0.f;
    for (int r = 0; r < PR; ++r) s = fmaf(h2c[r * ldh + tid], dq[r], s);
    slab_st(slab + nd.t[4].off + tid, s);
  }
  if (tid == H) {
    float s = 0.f;
    for (int r = 0; r < PR; ++r) s += dq[r];
    slab_st(slab + nd.t[5].off, s);
  }
  for (int e = tid; e < PR * H; e += blockDim.x) {
    const int r = e / H, h = e - r * H;
    d2[r * ldh + h] = h2c[r * ldh + h] > 0.f ? dq[r] * W3[h] : 0.f;
  }
  __syncthreads();
  PSTAMP(10);
  // dh1 tiles on waves 0..NT-1, dW2 tiles on the rest
  if (wave < NT) dgrad32(d2, ldh, H, a.theta + nd.t[2].off, h1c, ldh, d1, ldh, wave);
  wgrad32(h1c, ldh, H, d2, ldh, H, slab + nd.t[2].off, NT < nw ? NT : 0, NT < nw ? nw - NT : nw);
  colsum32(d2, ldh, H, slab + nd.t[3].off);
  __syncthreads();
  PSTAMP(11);
  wgrad32(rowbuf, ldr, ag.cin, d1, ldh, H, slab + nd.t[0].off, 0, nw);
  colsum32(d1, ldh, H, slab + nd.t[1].off);
  __syncthreads();
  PSTAMP(12);
}

template <int H>
__global__ __launch_bounds__(1024) void k_critic_pair(CriticArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int P = (a.B + PR - 1) / PR;
  const bool is_a = (int)blockIdx.x < P;
  const int p = is_a ? (int)blockIdx.x : (int)blockIdx.x - P;
  const int r0 = p * PR, nvalid = min(PR, a.B - r0);
  if (is_a) pair_actors<H>(a, lds, p, r0, nvalid);
  else pair_critic<H>(a, lds, p, r0, nvalid);
}

namespace {
template <int H>
hipError_t launch_pair(const CriticArgs& a, int lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_critic_pair<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MDP_LDS_BUDGET);
    (void)hipGetLastError();
    attr = true;
  }
  const int P = (a.B + PR - 1) / PR;
  hipLaunchKernelGGL(k_critic_pair<H>, dim3(2 * P), dim3(1024), lds, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t mdp_launch_critic_pair(const CriticArgs& a, int H, int lds_bytes, hipStream_t s) {
  switch (H) {
    case 64: return launch_pair<64>(a, lds_bytes, s);
    case 128: return launch_pair<128>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}
