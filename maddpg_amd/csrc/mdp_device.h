// mdp_device.h -- device-side building blocks of libmaddpg_hip (gfx950 / CDNA4).
//
// * Philox4x32-10 counter RNG (Gumbel uniforms, env resets) with TF1's
//   23-bit RandomUniform float conversion.
// * 16-row MLP tiles on the fp32 MFMA v_mfma_f32_16x16x4_f32: one wave owns a
//   16x16 output tile; A fragment lane l = X[l&15][k0 + (l>>4)], B fragment
//   lane l = W[k0 + (l>>4)][l&15], C/D lane l reg i = Y[(l>>4)*4+i][l&15].
//   The instruction is a k-ordered fmaf chain (exact fp32, no reduced
//   precision), so layer outputs are bitwise deterministic.
// * workgroup reductions over 64-wide wavefronts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mdp_topo.h"

#define MDP_NT 256          // threads per workgroup (4 waves)
#define MDP_NW 4            // waves per workgroup
#define MDP_R 16            // batch rows per workgroup tile

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one fp32 MFMA step, D = A x B + C over a 16x16 tile with k = 4 (exact fp32:
// the bitwise fmaf chain, MI355X_MICROARCH.md).  (Timing-only variants of
// this step live in tools/variants/mdp_exp.patch, not in the product.)
#define MDP_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// diagnostic build only (-DMDP_STAMPS): wall-clock stamps of workgroup 0
#ifdef MDP_STAMPS
__device__ unsigned long long g_mdp_stamps[64];
#define MDP_STAMP(i)                                                                     \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_mdp_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// shader-clock stamp (s_memtime) next to the wall-clock ones, for the in-kernel clock
#define MDP_CLK(i)                                                                      \
  do {                                                                                  \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_mdp_stamps[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// stamp from lane 0 of whichever wave executes it (workgroup 0)
#define MDP_STAMPW(i)                                                                              \
  do {                                                                                             \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_mdp_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MDP_STAMP(i) \
  do {               \
  } while (0)
#define MDP_STAMPW(i) \
  do {                \
  } while (0)
#define MDP_CLK(i) \
  do {             \
  } while (0)
#endif

// diagnostic build only (-DMDP_TIMELINE, `make timeline`): per launch of a
// round, the first workgroup start and the last wave end (s_memrealtime, 100
// MHz), keyed by the update counter at entry (one agent update: critic launch,
// its optimizer, actor launch, its optimizer) and the workgroup's role -- the
// graph-replayed round's launch bodies and the gaps between them
// (tools/timeline.py).  Slot = (upd_ctr & 255) * 16 + 4 * kind + role.
#ifdef MDP_TIMELINE
// per (slot, workgroup): start (thread 0, plain store) and end (max over the
// workgroup's waves: an atomic on a per-workgroup word, so at most 16 waves
// contend -- one word per slot made ~1000 waves queue on one address)
#define MDP_TL_SLOTS 1024
#define MDP_TL_WG 512
__device__ unsigned long long g_mdp_tl[MDP_TL_SLOTS][MDP_TL_WG][2];
struct MdpTl {
  unsigned long long t0;
  uint32_t ctr;
  int kr;
  __device__ MdpTl(const uint32_t* upd_ctr, int kind, int role)
      : t0(__builtin_amdgcn_s_memrealtime()),
        ctr(__hip_atomic_load(const_cast<uint32_t*>(upd_ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
        kr(4 * kind + role) {}
  __device__ void set_role(int kind, int role) { kr = 4 * kind + role; }
  __device__ ~MdpTl() {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t slot = (ctr & 63u) * 16u + (uint32_t)kr;
    if (blockIdx.x < MDP_TL_WG) {
      if (threadIdx.x == 0) g_mdp_tl[slot][blockIdx.x][0] = t0;
      if ((threadIdx.x & 63) == 0) atomicMax(&g_mdp_tl[slot][blockIdx.x][1], t1);
    }
  }
};
#define MDP_TL(ctl, kind, role) MdpTl mdp_tl_(&(ctl)->upd_ctr, kind, role)
#define MDP_TL_ROLE(kind, role) mdp_tl_.set_role(kind, role)
// the last rollout launch's per-workgroup start / end (k_rollout, mdp_kernels.hip)
__device__ unsigned long long g_mdp_tl_roll[MDP_TL_WG][2];
struct MdpTlRoll {
  unsigned long long t0;
  __device__ MdpTlRoll() : t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~MdpTlRoll() {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < MDP_TL_WG) {
      if (threadIdx.x == 0) g_mdp_tl_roll[blockIdx.x][0] = t0;
      if ((threadIdx.x & 63) == 0) atomicMax(&g_mdp_tl_roll[blockIdx.x][1], t1);
    }
  }
};
#define MDP_TL_ROLLOUT() MdpTlRoll mdp_tlr_
#else
#define MDP_TL_ROLLOUT() \
  do {                   \
  } while (0)
#define MDP_TL(ctl, kind, role) \
  do {                          \
  } while (0)
#define MDP_TL_ROLE(kind, role) \
  do {                          \
  } while (0)
#endif

// A kernel's first branches each read a kernarg field, and the compiler issues
// each read behind the previous branch: a chain of scalar-cache misses (ISA:
// five s_load / s_waitcnt pairs before the first global load).  Naming one
// field per 64-B line of the argument block here makes them one round trip;
// the later reads hit the scalar cache.
#define MDP_KARG_TOUCH(...) asm volatile("" ::__VA_ARGS__)
// every 64-B line of two agents' descriptors (212 B each: fields at most 56 B
// apart), once the kernel knows which agents it serves -- one round trip
#define MDP_KARG_ADESC(d) "s"((d).actor.t[0].off), "s"((d).actor.t[3].rows), "s"((d).actor.in), \
                          "s"((d).critic.t[2].off), "s"((d).critic.in), "s"((d).cin)

// The training-noise counter (Ctl::upd_ctr, advanced by the previous
// optimizer launch) is a uniform load from memory another kernel wrote: the
// compiler turned it into an SGPR with v_readfirstlane right after the load and
// waited for it there -- every wave stalled a memory round trip (ISA:
// global_load + s_waitcnt vmcnt(0) in front of B0) before issuing its weight
// loads.  ctr_load issues the load where it stands; ctr_use makes the VGPR
// opaque where the noise is made, so the wait moves there (behind the weight
// loads, which are still in flight).
__device__ __forceinline__ uint32_t ctr_load(const Ctl* ctl) { return ctl->upd_ctr; }
__device__ __forceinline__ uint32_t ctr_use(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// ------------------------------------------------------------------ RNG
struct Philox {
  __device__ static inline uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ static inline uint4 gen(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

// TF1 random_uniform float: mantissa from 23 random bits, value in [0, 1).
__device__ __forceinline__ float u01(uint32_t x) {
  return __uint_as_float((x >> 9) | 0x3f800000u) - 1.0f;
}

// five uniforms for one (stream, counter, row) triple
__device__ __forceinline__ void uniforms5(uint64_t seed, uint32_t stream, uint32_t ctr, uint32_t row, float u[5]) {
  uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  uint4 a = Philox::gen(make_uint4(row, ctr, stream, 0u), key);
  uint4 b = Philox::gen(make_uint4(row, ctr, stream, 1u), key);
  u[0] = u01(a.x); u[1] = u01(a.y); u[2] = u01(a.z); u[3] = u01(a.w); u[4] = u01(b.x);
}

// -------------------------------------------------------------- helpers
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sums over lane groups on DPP moves (VALU ops on the lane crossbar) instead of
// __shfl_xor, which lowers to ds_bpermute round trips through the LDS
// crossbar.  quad_perm [1,0,3,2] / [2,3,0,1] are exactly xor 1 / xor 2; once
// every quad holds its sum, the half-row and row mirrors pair the same partial
// sums as xor 4 / xor 8, so quad_sum / row_sum are bit-identical to those
// butterflies.  Every lane of the wave must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float quad_sum(float s) {  // = s + shfl_xor 1, then + shfl_xor 2
  s += dpp_f<0xB1>(s);
  s += dpp_f<0x4E>(s);
  return s;
}
__device__ __forceinline__ float half_row_sum(float s) {  // ... then + shfl_xor 4
  s = quad_sum(s);
  s += dpp_f<0x141>(s);
  return s;
}
__device__ __forceinline__ float row_sum(float s) {  // ... then + shfl_xor 8
  s = half_row_sum(s);
  s += dpp_f<0x140>(s);
  return s;
}

// fp64 wave sum on DPP moves (each a VALU op on the lane crossbar) instead of
// six ds_bpermute round trips through the LDS crossbar (stamped 0.4 us of the
// optimizer's critical path): xor 1, xor 2, half-row mirror, row mirror (every
// lane holds its row's sum), row_bcast15 / row_bcast31 fold the rows into lane
// 63, read back to every lane.  A fixed tree: deterministic.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_d<0x140, 0xf>(v);  // row_mirror
  v += dpp_d<0x142, 0xa>(v);  // row_bcast15 into rows 1, 3
  v += dpp_d<0x143, 0xc>(v);  // row_bcast31 into rows 2, 3
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// workgroup-wide sum (all threads get the result); scratch >= MDP_NW doubles
__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// odd leading dimension so the 16 row-reads of one fragment land on distinct banks
__host__ __device__ __forceinline__ int lds_ld(int cols) { return (cols | 1); }

// ------------------------------------------------------ MFMA layer tiles
// Y[16][N] = act(X[16][K] @ W[K][N] + b)   X,Y in LDS; W,b global row-major [K][N]
// N multiple of 16.  Column tiles are dealt round-robin over the 4 waves.
// B fragments of one 64-deep K chunk (16 MFMA k-steps) for one column: all 16
// global loads are issued together so the chunk pays one L2 latency, not 16.
// Rows k >= K load the (finite) row K-1 and are NOT zeroed here: the consumer
// zeroes the A operand of those rows (mfma_chunk / load_afrag).  A select on
// the loaded value would make the wave wait for the load right where it is
// issued -- the prefetch of the next chunk would not overlap the current one.
#define MDP_KC 16
__device__ __forceinline__ void load_wchunk(float (&w)[MDP_KC], const float* __restrict__ W, int ldw, int col, int c0,
                                   int K, int kq) {
  const int kmax = K > 0 ? K - 1 : 0;
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    w[s] = W[min(k, kmax) * ldw + col];
  }
}
// same for a transposed operand: element (k, col) at W[col * ldw + k]
__device__ __forceinline__ void load_wchunk_t(float (&w)[MDP_KC], const float* __restrict__ W, int ldw, int col, int c0,
                                     int K, int kq, bool colok) {
  const int kmax = K > 0 ? K - 1 : 0;
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = W[col * ldw + min(k, kmax)];
    w[s] = colok ? v : 0.f;
  }
}
// acc += A[r][c0 .. c0+63] . w  with A from LDS (row r = lane&15)
__device__ __forceinline__ f32x4 mfma_chunk(f32x4 acc, const float (&w)[MDP_KC], const float* A, int lda, int r, int c0,
                                   int K, int kq) {
  const int kmax = K > 0 ? K - 1 : 0;
  float x[MDP_KC];
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = A[r * lda + min(k, kmax)];
    x[s] = k < K ? v : 0.f;
  }
  __builtin_amdgcn_sched_barrier(0);  // every A read ahead of the MFMA chain
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    if (c0 + 4 * s < K)  // wave-uniform
      acc = MDP_MFMA(x[s], w[s], acc);
  }
  return acc;
}

template <bool RELU>
__device__ __forceinline__ void tile_fwd(const float* X, int ldx, int K, const float* __restrict__ W,
                                const float* __restrict__ b, int N, float* Y, int ldy) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, kq = lane >> 4;
  for (int nt = wave; nt < (N >> 4); nt += MDP_NW) {
    const int col = nt * 16 + r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float wa[MDP_KC], wb[MDP_KC];
    load_wchunk(wa, W, N, col, 0, K, kq);
    for (int c0 = 0; c0 < K; c0 += 4 * MDP_KC) {
      const bool more = c0 + 4 * MDP_KC < K;
      if (more) load_wchunk(wb, W, N, col, c0 + 4 * MDP_KC, K, kq);
      acc = mfma_chunk(acc, wa, X, ldx, r, c0, K, kq);
      if (more) {
#pragma unroll
        for (int s = 0; s < MDP_KC; ++s) wa[s] = wb[s];
      }
    }
    const float bias = b[col];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = acc[i] + bias;
      if (RELU) v = fmaxf(v, 0.f);
      Y[(kq * 4 + i) * ldy + col] = v;
    }
  }
}

// dX[16][K] = (dY[16][N] @ W^T) masked by (H > 0) where H is the layer input
// (post-ReLU activations of the previous layer); K multiple of 16.
__device__ __forceinline__ void tile_dgrad_relu(const float* dY, int ldy, int N, const float* __restrict__ W, int K,
                                       const float* Hin, int ldh, float* dX, int ldx) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, kq = lane >> 4;
  for (int nt = wave; nt < (K >> 4); nt += MDP_NW) {
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
      const float h = Hin[row * ldh + kk];
      dX[row * ldx + kk] = h > 0.f ? acc[i] : 0.f;
    }
  }
}

// ONE wave: out[16][nout] = X[16][K] @ W[K][nout] + b for nout <= 16 as a single
// MFMA column tile (column r = lane & 15): every weight of the lane is requested
// up front (one memory round trip), then KS = K/4 dependent MFMAs.  Replaces
// the VALU heads whose k-loop waited on one global load per iteration.
// K is a multiple of 4 (every caller passes H), so a k-step is either wholly
// inside K or skipped, and columns r >= nout are computed but never stored: the
// weight loads need no select.  (A select on the loaded value made the compiler
// branch around each load and wait for it there, one round trip per k-step.)
template <int KS>
__device__ __forceinline__ void head_mfma(const float* X, int ldx, int K, const float* __restrict__ W,
                                          const float* __restrict__ b, int nout, float* out, int ldo) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int c = min(r, nout - 1), kmax = K - 1;
  if constexpr (KS > 32) {
    // wide heads (H = 256): 64-deep chunks, one round trip each, so the
    // fragments fit the register budget of a 1024-thread workgroup.  Same
    // accumulator and k order as the one-shot form.
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < K; c0 += 4 * MDP_KC) {
      float w[MDP_KC], x[MDP_KC];
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s) {
        const int k = c0 + 4 * s + kq;
        w[s] = W[min(k, kmax) * nout + c];
        x[s] = X[r * ldx + min(k, kmax)];
      }
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s)
        if (c0 + 4 * s < K) acc = MDP_MFMA(x[s], w[s], acc);
    }
    const float bias = b[c];
    if (r < nout) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(kq * 4 + i) * ldo + r] = acc[i] + bias;
    }
    return;
  }
  float w[KS], x[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + kq;
    w[s] = W[min(k, kmax) * nout + c];
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) x[s] = X[r * ldx + min(4 * s + kq, kmax)];
  const float bias = b[c];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
    if (4 * s < K) acc = MDP_MFMA(x[s], w[s], acc);
  if (r < nout) {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(kq * 4 + i) * ldo + r] = acc[i] + bias;
  }
}

// head_mfma in two steps, so the head's weight fragments can be issued ahead
// (K = 4 KS; columns r >= nout are computed but never stored, so the loads need
// no select -- a select on the loaded value would wait for it at the load)
template <int KS>
__device__ __forceinline__ void head_load(float (&w)[KS], float& bias, const float* __restrict__ W,
                                          const float* __restrict__ b, int nout) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int c = min(r, nout - 1);
#pragma unroll
  for (int s = 0; s < KS; ++s) w[s] = W[(4 * s + kq) * nout + c];
  bias = b[c];
}
template <int KS>
__device__ __forceinline__ void head_acc(const float (&w)[KS], float bias, const float* X, int ldx, int nout,
                                         float* out, int ldo) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  float x[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) x[s] = X[r * ldx + 4 * s + kq];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) acc = MDP_MFMA(x[s], w[s], acc);
  if (r < nout) {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(kq * 4 + i) * ldo + r] = acc[i] + bias;
  }
}

// out[16][nout] = X[16][K] @ W[K][nout] + b  (small heads, VALU; 4 lanes per output)
__device__ __forceinline__ void tile_head(const float* X, int ldx, int K, const float* __restrict__ W,
                                 const float* __restrict__ b, int nout, float* out, int ldo) {
  const int total = MDP_R * nout;
  for (int base = 0; base < total * 4; base += MDP_NT) {
    const int t = base + threadIdx.x;
    const int o = t >> 2, q = t & 3;
    float s = 0.f;
    if (o < total) {
      const int row = o / nout, c = o - row * nout;
      for (int k = q; k < K; k += 4) s = fmaf(X[row * ldx + k], W[k * nout + c], s);
    }
    s = quad_sum(s);
    if (o < total && q == 0) {
      const int row = o / nout, c = o - row * nout;
      out[row * ldo + c] = s + b[c];
    }
  }
}

// softmax(logits - log(-log(u))) on one row of 5 (distributions.py:264-266)
// Gumbel noise g = log(-log(u)) (distributions.py:235) -- independent of the
// logits, so the fast kernels compute it while their weights are in flight
// The noise and the softmax use the hardware transcendentals (v_log_f32 /
// v_exp_f32 / v_rcp_f32, a few ulp): the precise libm forms cost ~1 us of VALU
// in the gradient kernels' prologue, on the critical path.  Parity with the
// oracle is within the tests' fp32 tolerances either way.
__device__ __forceinline__ void gumbel_noise5(const float* u, float* gn) {
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) gn[k] = __logf(-__logf(u[k]));
}
// softmax(logits - g): the same operations in the same order as gumbel_softmax5
__device__ __forceinline__ void gumbel_softmax5_pre(const float* logits, const float* gn, float* a) {
  float z[MDP_ACT_DIM];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) {
    z[k] = logits[k] - gn[k];
    m = fmaxf(m, z[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) {
    z[k] = __expf(z[k] - m);
    s += z[k];
  }
  const float inv = __builtin_amdgcn_rcpf(s);
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) a[k] = z[k] * inv;
}
__device__ __forceinline__ void gumbel_softmax5(const float* logits, const float* u, float* a) {
  float gn[MDP_ACT_DIM];
  gumbel_noise5(u, gn);
  gumbel_softmax5_pre(logits, gn, a);
}

// ------------------------------------------------------ phase-parallel tiles
// (k_critic_grad / k_actor_grad, 512-thread workgroups)  A "job" is one dense
// layer Y[16][N] = act(X[16][K] @ W[K][N] + b) of one net; all jobs of a
// phase are independent, their 16x16 output tiles are dealt over the waves
// and each wave runs two tiles' MFMA chains interleaved (the 40-cycle
// dependent latency of one chain is covered by the other's issue).  Every
// weight fragment of both tiles is requested before the first MFMA, so a
// phase pays one global-load latency instead of one per chunk.
//
// Job records live in LDS and hold OFFSETS, not pointers: X/Y index the
// dynamic LDS segment, W/b index one of two global bases (online / target
// parameters).  A pointer reloaded from LDS would be a generic address and
// every access would become a FLAT load with a full vmcnt+lgkmcnt wait.
struct FJob {
  int xoff, ldx, K, woff, boff, yoff, ldy, wsel;
};
struct HJob {  // output head: out[16][nout] = X[16][K] @ W3[K][nout] + b3 (VALU)
  int xoff, ldx, woff, boff, nout, ooff, ldo, wsel;
};

// unconditional (clamped, in-bounds) load + select: no branch per element
__device__ __forceinline__ void load_wfrag(float (&w)[MDP_KC], const float* __restrict__ W, int ldw, int col, int c0,
                                           int K, int kq) {
  const int kmax = K > 0 ? K - 1 : 0;
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = W[min(k, kmax) * ldw + col];
    w[s] = k < K ? v : 0.f;
  }
}
__device__ __forceinline__ void load_afrag(float (&a)[MDP_KC], const float* X, int ldx, int r, int c0, int K, int kq) {
  const int kmax = K > 0 ? K - 1 : 0;
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    const float v = X[r * ldx + min(k, kmax)];
    a[s] = k < K ? v : 0.f;
  }
}

// acc_a += A_a . w_a and acc_b += A_b . w_b over one 64-deep chunk, alternating chains
__device__ __forceinline__ void mfma_chunk2(f32x4& acc_a, const float (&xa)[MDP_KC], const float (&wa)[MDP_KC], int na,
                                            f32x4& acc_b, const float (&xb)[MDP_KC], const float (&wb)[MDP_KC], int nb) {
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    if (s < na) acc_a = MDP_MFMA(xa[s], wa[s], acc_a);
    if (s < nb) acc_b = MDP_MFMA(xb[s], wb[s], acc_b);
  }
}

__device__ __forceinline__ int ksteps(int K, int c0) {
  const int left = K - c0;
  return left <= 0 ? 0 : (left >= 4 * MDP_KC ? MDP_KC : (left + 3) >> 2);
}

// all jobs have N output columns (N multiple of 16); ReLU on every job
__device__ __forceinline__ void fwd_phase(const FJob* jobs, int njobs, int N, float* lds, const float* __restrict__ P0,
                                          const float* __restrict__ P1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int ntl = N >> 4, total = njobs * ntl;
  for (int t0 = wave; t0 < total; t0 += 2 * nw) {
    const int t1 = t0 + nw;
    const bool two = t1 < total;
    const FJob ja = jobs[t0 / ntl];
    const FJob jb = jobs[two ? t1 / ntl : t0 / ntl];
    const int ca = (t0 % ntl) * 16 + r;
    const int cb = two ? (t1 % ntl) * 16 + r : ca;
    const int Kb = two ? jb.K : 0;
    const float* Wa = (ja.wsel ? P1 : P0) + ja.woff;
    const float* Wb = (jb.wsel ? P1 : P0) + jb.woff;
    const float* Xa = lds + ja.xoff;
    const float* Xb = lds + jb.xoff;
    float wa0[MDP_KC], wa1[MDP_KC], wb0[MDP_KC], wb1[MDP_KC], xa[MDP_KC], xb[MDP_KC];
    load_wfrag(wa0, Wa, N, ca, 0, ja.K, kq);
    load_wfrag(wb0, Wb, N, cb, 0, Kb, kq);
    const bool second = ja.K > 4 * MDP_KC || Kb > 4 * MDP_KC;
    if (second) {
      load_wfrag(wa1, Wa, N, ca, 4 * MDP_KC, ja.K, kq);
      load_wfrag(wb1, Wb, N, cb, 4 * MDP_KC, Kb, kq);
    }
    const float biasa = (ja.wsel ? P1 : P0)[ja.boff + ca];
    const float biasb = (jb.wsel ? P1 : P0)[jb.boff + cb];
    f32x4 acc_a = {0.f, 0.f, 0.f, 0.f}, acc_b = {0.f, 0.f, 0.f, 0.f};
    load_afrag(xa, Xa, ja.ldx, r, 0, ja.K, kq);
    load_afrag(xb, Xb, jb.ldx, r, 0, Kb, kq);
    mfma_chunk2(acc_a, xa, wa0, ksteps(ja.K, 0), acc_b, xb, wb0, ksteps(Kb, 0));
    if (second) {
      load_afrag(xa, Xa, ja.ldx, r, 4 * MDP_KC, ja.K, kq);
      load_afrag(xb, Xb, jb.ldx, r, 4 * MDP_KC, Kb, kq);
      mfma_chunk2(acc_a, xa, wa1, ksteps(ja.K, 4 * MDP_KC), acc_b, xb, wb1, ksteps(Kb, 4 * MDP_KC));
      for (int c0 = 8 * MDP_KC; c0 < ja.K || c0 < Kb; c0 += 4 * MDP_KC) {   // K > 128: stream
        load_wfrag(wa0, Wa, N, ca, c0, ja.K, kq);
        load_wfrag(wb0, Wb, N, cb, c0, Kb, kq);
        load_afrag(xa, Xa, ja.ldx, r, c0, ja.K, kq);
        load_afrag(xb, Xb, jb.ldx, r, c0, Kb, kq);
        mfma_chunk2(acc_a, xa, wa0, ksteps(ja.K, c0), acc_b, xb, wb0, ksteps(Kb, c0));
      }
    }
    float* Ya = lds + ja.yoff;
    float* Yb = lds + jb.yoff;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Ya[(kq * 4 + i) * ja.ldy + ca] = fmaxf(acc_a[i] + biasa, 0.f);
      if (two) Yb[(kq * 4 + i) * jb.ldy + cb] = fmaxf(acc_b[i] + biasb, 0.f);
    }
  }
}

// heads of several nets, 4 lanes per output, nout <= 8
__device__ __forceinline__ void head_phase(const HJob* jobs, int njobs, int K, float* lds, const float* __restrict__ P0,
                                           const float* __restrict__ P1) {
  int total = 0;
  for (int j = 0; j < njobs; ++j) total += MDP_R * jobs[j].nout;
  for (int base = 0; base < total * 4; base += blockDim.x) {
    const int t = base + threadIdx.x;
    const int o = t >> 2, q = t & 3;
    float s = 0.f;
    int jj = 0, oo = o;
    const bool ok = o < total;
    if (ok) {
      while (oo >= MDP_R * jobs[jj].nout) {
        oo -= MDP_R * jobs[jj].nout;
        ++jj;
      }
    }
    const HJob h = jobs[ok ? jj : 0];
    const int row = ok ? oo / h.nout : 0, c = ok ? oo - row * h.nout : 0;
    const float* X = lds + h.xoff;
    const float* W = (h.wsel ? P1 : P0) + h.woff;
    if (ok)
      for (int k = q; k < K; k += 4) s = fmaf(X[row * h.ldx + k], W[k * h.nout + c], s);
    s = quad_sum(s);
    if (ok && q == 0) lds[h.ooff + row * h.ldo + c] = s + (h.wsel ? P1 : P0)[h.boff + c];
  }
}


// ---------------------------------------------------------- wave-local nets
// LDS ordering between lanes of ONE wave (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One wave computes a whole layer Y[16][N] = act(X[16][K] @ W[K][N] + b) for
// N = 16*NT: the NT column tiles' MFMA chains are interleaved (NT independent
// accumulators), all weight fragments of a 64-deep chunk are loaded together.
template <int NT, bool RELU>
__device__ __forceinline__ void wave_layer(const float* X, int ldx, int K, const float* __restrict__ W,
                                           const float* __restrict__ b, float* Y, int ldy) {
  constexpr int N = NT * 16;
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < K; c0 += 4 * MDP_KC) {
    float w[NT][MDP_KC], x[MDP_KC];
#pragma unroll
    for (int t = 0; t < NT; ++t) load_wfrag(w[t], W, N, t * 16 + r, c0, K, kq);
    load_afrag(x, X, ldx, r, c0, K, kq);
    const int ns = ksteps(K, c0);
#pragma unroll
    for (int s = 0; s < MDP_KC; ++s) {
      if (s < ns) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = MDP_MFMA(x[s], w[t][s], acc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float bias = b[t * 16 + r];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = acc[t][i] + bias;
      if (RELU) v = fmaxf(v, 0.f);
      Y[(kq * 4 + i) * ldy + t * 16 + r] = v;
    }
  }
  wave_sync();
}

// one wave: out[16][nout] = X[16][K] @ W[K][nout] + b, nout <= 8 (4 lanes per output, passes of 16)
__device__ __forceinline__ void wave_head(const float* X, int ldx, int K, const float* __restrict__ W,
                                          const float* __restrict__ b, int nout, float* out, int ldo) {
  const int lane = threadIdx.x & 63;
  const int total = MDP_R * nout;
  for (int base = 0; base < total; base += 16) {
    const int o = base + (lane >> 2), q = lane & 3;
    const bool ok = o < total;
    const int row = ok ? o / nout : 0, c = ok ? o - row * nout : 0;
    float s = 0.f;
    for (int k = q; k < K; k += 4) s = fmaf(X[row * ldx + k], W[k * nout + c], s);
    s = quad_sum(s);
    if (ok && q == 0) out[row * ldo + c] = s + b[c];
  }
  wave_sync();
}

// one wave: dX[16][K] = (dY[16][N] @ W^T) masked by Hin > 0, W global [K][N], K = 16*NT
template <int NT>
__device__ __forceinline__ void wave_dgrad(const float* dY, int ldy, int N, const float* __restrict__ W,
                                           const float* Hin, int ldh, float* dX, int ldx) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < N; c0 += 4 * MDP_KC) {
    float w[NT][MDP_KC], x[MDP_KC];
#pragma unroll
    for (int t = 0; t < NT; ++t) load_wchunk_t(w[t], W, N, t * 16 + r, c0, N, kq, true);
    load_afrag(x, dY, ldy, r, c0, N, kq);
#pragma unroll
    for (int s = 0; s < MDP_KC; ++s) {
      if (c0 + 4 * s < N) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = MDP_MFMA(x[s], w[t][s], acc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kq * 4 + i, kk = t * 16 + r;
      dX[row * ldx + kk] = Hin[row * ldh + kk] > 0.f ? acc[t][i] : 0.f;
    }
  }
  wave_sync();
}

// dX[16][K] = (dY[16][N] @ W^T) masked by Hin > 0, tiles over waves 0..K/16-1
// (the caller keeps those waves free of other work); W global [K][N].
__device__ __forceinline__ void dgrad_tiles(const float* dY, int ldy, int N, const float* __restrict__ W, int K,
                                   const float* Hin, int ldh, float* dX, int ldx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  for (int nt = wave; nt < (K >> 4); nt += nw) {
    const int kk = nt * 16 + r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < N; c0 += 4 * MDP_KC) {
      float w[MDP_KC], x[MDP_KC];
      load_wchunk_t(w, W, N, kk, c0, N, kq, true);
      load_afrag(x, dY, ldy, r, c0, N, kq);
#pragma unroll
      for (int s = 0; s < MDP_KC; ++s)
        if (c0 + 4 * s < N) acc = MDP_MFMA(x[s], w[s], acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kq * 4 + i;
      const float h = Hin[row * ldh + kk];
      dX[row * ldx + kk] = h > 0.f ? acc[i] : 0.f;
    }
  }
}

__device__ __forceinline__ void gather_rows16(const float* __restrict__ replay, int stride, const int32_t* __restrict__ idx,
                                     int r0, int nvalid, float* rowbuf, int ldr) {
  const int v4 = stride >> 2;
  for (int e = threadIdx.x; e < MDP_R * v4; e += blockDim.x) {
    const int r = e / v4, c4 = e - r * v4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < nvalid) v = *reinterpret_cast<const float4*>(replay + (int64_t)idx[r0 + r] * stride + c4 * 4);
    float* d = rowbuf + r * ldr + c4 * 4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}

// the same over the threads [t0, t0 + nt) of the workgroup only
__device__ __forceinline__ void gather_rows16_part(const float* __restrict__ replay, int stride,
                                                   const int32_t* __restrict__ idx, int r0, int nvalid, float* rowbuf,
                                                   int ldr, int t0, int nt) {
  const int v4 = stride >> 2;
  for (int e = (int)threadIdx.x - t0; e < MDP_R * v4; e += nt) {
    const int r = e / v4, c4 = e - r * v4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < nvalid) v = *reinterpret_cast<const float4*>(replay + (int64_t)idx[r0 + r] * stride + c4 * 4);
    float* d = rowbuf + r * ldr + c4 * 4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}

// the 16 rows of a contiguous [16][stride] block (stored by an earlier launch's
// gather) into rowbuf, over the threads [t0, t0 + nt): one round trip, no index load
__device__ __forceinline__ void load_rows16_part(const float* __restrict__ block, int stride, float* rowbuf, int ldr,
                                                 int t0, int nt) {
  const int v4 = stride >> 2;
  for (int e = (int)threadIdx.x - t0; e < MDP_R * v4; e += nt) {
    const int r = e / v4, c4 = e - r * v4;
    const float4 v = *reinterpret_cast<const float4*>(block + (int64_t)r * stride + c4 * 4);
    float* d = rowbuf + r * ldr + c4 * 4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}
// rowbuf's 16 rows -> a contiguous [16][stride] block (all threads)
// 16-B store of a split-step hand-off block (apre / cpre and their row
// blocks, read by the next launch); MDP_WT_HANDOFF: write-through (sc1)
__device__ __forceinline__ void handoff_st4(float* p, f32x4 v) {
#ifdef MDP_WT_HANDOFF
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#else
  *reinterpret_cast<f32x4*>(p) = v;
#endif
}

__device__ __forceinline__ void store_rows16(const float* rowbuf, int ldr, int stride, float* __restrict__ block) {
  const int v4 = stride >> 2;
  for (int e = threadIdx.x; e < MDP_R * v4; e += blockDim.x) {
    const int r = e / v4, c4 = e - r * v4;
    const float* sp = rowbuf + r * ldr + c4 * 4;
    handoff_st4(block + (int64_t)r * stride + c4 * 4, f32x4{sp[0], sp[1], sp[2], sp[3]});
  }
}

__device__ __forceinline__ void copy_cols16(const float* src, int lds_src, int src_off, float* dst, int lds_dst, int dst_off,
                                   int ncols) {
  for (int e = threadIdx.x; e < MDP_R * ncols; e += blockDim.x) {
    const int r = e / ncols, c = e - r * ncols;
    dst[r * lds_dst + dst_off + c] = src[r * lds_src + src_off + c];
  }
}

__device__ __forceinline__ void colsum16(const float* X, int ldx, int ncols, float* __restrict__ out) {
  for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < MDP_R; ++r) s += X[r * ldx + c];
    out[c] = s;
  }
}

// Arena-relative LDS carving for the dynamic shared segment.
struct LdsCarve {
  float* base;
  int off;
  __device__ LdsCarve(float* p) : base(p), off(0) {}
  __device__ float* take(int n) {
    float* p = base + off;
    off += (n + 3) & ~3;
    return p;
  }
};

// ------------------------------------------- register-resident layers (H = 64)
// Used by the fast gradient kernels (mdp_grads_r.hip).  Every weight a wave
// needs is loaded into its registers at kernel start -- one memory round trip
// for the whole kernel, overlapped with the replay gather -- instead of one
// per layer.  Forward layers keep all four 16-column tiles in one wave with a
// PERMUTED column map: tile t, lane (r = lane & 15, kq = lane >> 4) produces
// column 4r + t, so a lane's B fragments at one k-step are 4 consecutive
// floats of a weight row (one 16-B load).  Contraction index k = 4s + kq.
#define MDP_RH 64   // hidden width of the register-resident path
#define MDP_RLH 68  // LDS row stride of forward activations (4r + kq: 64 distinct banks)
#define MDP_RLD 65  // LDS row stride of backward deltas (r + 16 kq + s: 64 distinct banks)

__device__ __forceinline__ f32x4 ld4(const float* __restrict__ p) { return *reinterpret_cast<const f32x4*>(p); }

// w[s] = W[4s+kq][4r .. 4r+3] of W[K][64] for the k-steps below K (others 0).
// Rows >= K hold the clamped row K-1 and rows the caller excludes stay as
// loaded: rf_acc zeroes the A operand of those rows.  (A select on the loaded
// value inside the per-k-step branch made the wave wait for each load before
// issuing the next: serialised round trips.)
template <int KS>
__device__ __forceinline__ void rf_load(f32x4 (&w)[KS], const float* __restrict__ W, int K) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  const int kq = lane >> 4;
  // Unconditional, clamped to row K - 1: rf_acc skips the k-steps past K (and
  // zeroes the A operand of rows >= K).  A per-k-step branch merged the loaded
  // value with a zero into one register, and the copy made the wave wait for
  // the load right where it was issued (ISA: global_load_dwordx4 + vmcnt(0) +
  // v_mov in rf_load<2>); the clamped extra loads hit the same row's lines.
#pragma unroll
  for (int s = 0; s < KS; ++s) w[s] = ld4(W + min(4 * s + kq, K - 1) * MDP_RH + 4 * r);
}

// acc[t] += X[16][K] @ W (the fragments of rf_load); X in LDS; input rows >= K
// and rows inside [mlo, mhi) contribute zero.  All A fragments are read first
// (clamped, unconditional) so the MFMA chain never waits on LDS.
template <int KS>
__device__ __forceinline__ void rf_acc(f32x4 (&acc)[4], const float* X, int ldx, int K, const f32x4 (&w)[KS],
                                       int mlo = 0, int mhi = 0) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const float* xr = X + r * ldx;
  float x[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + kq;
    const float v = xr[min(k, K - 1)];
    x[s] = (k < K && (k < mlo || k >= mhi)) ? v : 0.f;
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every read ahead of the MFMA chain
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (4 * s < K) {
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = MDP_MFMA(x[s], w[s][t], acc[t]);
    }
  }
}

__device__ __forceinline__ void rf_zero(f32x4 (&acc)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Y[16][64] = act(acc + b), b = bias[4r .. 4r+3]; Y row stride a multiple of 4 (16-B stores)
template <bool RELU>
__device__ __forceinline__ void rf_store(const f32x4 (&acc)[4], f32x4 b, float* Y, int ldy) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 v;
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = RELU ? fmaxf(acc[t][i] + b[t], 0.f) : acc[t][i] + b[t];
    *reinterpret_cast<f32x4*>(Y + (kq * 4 + i) * ldy + 4 * r) = v;
  }
}

// output head with nout <= 16 columns on one MFMA tile (column r), K = 64
__device__ __forceinline__ void rh_load(float (&w)[16], const float* __restrict__ W, int nout) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int c = min(r, nout - 1);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float v = W[(4 * s + kq) * nout + c];
    w[s] = r < nout ? v : 0.f;
  }
}
__device__ __forceinline__ f32x4 rh_acc(const float* X, int ldx, const float (&w)[16]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  float x[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) x[s] = X[r * ldx + 4 * s + kq];
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = MDP_MFMA(x[s], w[s], acc);
  return acc;
}

// scalar head (nout = 1) on the VALU: lane (row = lane >> 2, q = lane & 3), w[j] = W3[4j + q]
__device__ __forceinline__ void rq_load(float (&w)[16], const float* __restrict__ W) {
  const int q = threadIdx.x & 3;
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = W[4 * j + q];
}
// returns sum_k X[row][k] W3[k] in all 4 lanes of the row
__device__ __forceinline__ float rq_head(const float* X, int ldx, const float (&w)[16]) {
  const int lane = threadIdx.x & 63, row = lane >> 2, q = lane & 3;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s = fmaf(X[row * ldx + 4 * j + q], w[j], s);
  return quad_sum(s);
}

// one 16-column tile per wave (column col = 16 tt + r of W[K][ldw]), k = 4s + kq;
// unconditional clamped loads (straight-line code, exact vmcnt accounting); K >= 1.
// Rows >= K hold the clamped row K-1: rt_acc zeroes their A operand.
template <int KS>
__device__ __forceinline__ void rt_load(float (&w)[KS], const float* __restrict__ W, int ldw, int col, int K) {
  const int kq = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int s = 0; s < KS; ++s) w[s] = W[min(4 * s + kq, K - 1) * ldw + col];
}
// rt_load for a runtime K <= 4 KS: only the k-steps below K issue loads (no
// select on the loaded value: it would serialise the loads, see rf_load)
template <int KS>
__device__ __forceinline__ void rt_load_k(float (&w)[KS], const float* __restrict__ W, int ldw, int col, int K) {
  const int kq = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    w[s] = 0.f;
    if (4 * s < K) w[s] = W[min(4 * s + kq, K - 1) * ldw + col];  // wave-uniform branch
  }
}
template <int KS>
__device__ __forceinline__ void rt_acc(f32x4& acc, const float* X, int ldx, int K, const float (&w)[KS]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const float* xr = X + r * ldx;
  float x[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + kq;
    const float v = xr[min(k, K - 1)];
    x[s] = k < K ? v : 0.f;
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every read ahead of the MFMA chain
#pragma unroll
  for (int s = 0; s < KS; ++s)
    if (4 * s < K) acc = MDP_MFMA(x[s], w[s], acc);
}

// transposed tile for dX = dY @ W^T (W[K][64] row-major): output column kk = W row,
// contraction n = 16 kq + s, so a lane's 16 fragments are one contiguous 64-B run
// of row kk: w[m] = W[kk][16 kq + 4m .. +3]; ok = false zeroes the fragment
__device__ __forceinline__ void rdg_load(f32x4 (&w)[4], const float* __restrict__ W, int kk, bool ok) {
  const int kq = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const f32x4 v = ld4(W + kk * MDP_RH + 16 * kq + 4 * m);
    w[m] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}
__device__ __forceinline__ f32x4 rdg_acc(const float* dY, int ldy, const f32x4 (&w)[4]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const float* yr = dY + r * ldy + 16 * kq;
  float x[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) x[s] = yr[s];
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = MDP_MFMA(x[s], w[s >> 2][s & 3], acc);
  return acc;
}

// LDS hand-off without a workgroup barrier: the producing waves signal after
// their LDS writes completed; consumers spin (s_sleep) until every producer
// has.  The counter must be zeroed before a barrier that precedes any signal.
__device__ __forceinline__ void lds_signal(int* flag) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait(int* flag, int n) {
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < n) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}

// ------------------------------------------------ shared by the grad kernels
// lanes 0..15 hold one value each; returns the sum in every lane (fixed order)
__device__ __forceinline__ double sum16(double v) {  // lanes 0..15 (every lane of row 0 gets it)
  const int lane = threadIdx.x & 63;
  v = lane < MDP_R ? v : 0.0;
  v += dpp_d<0xB1, 0xf>(v);
  v += dpp_d<0x4E, 0xf>(v);
  v += dpp_d<0x141, 0xf>(v);
  v += dpp_d<0x140, 0xf>(v);
  return v;
}

// weight-gradient tiles over waves [w0, w0 + wn)
// partial-gradient slab store (read once by k_reduce_apply on another CU).
// MDP_NT_SLAB=1 (nontemporal) measured: gradient kernels -0.2 us, k_reduce_apply
// 4.94 -> 5.33 us, S2 1.3 % slower end to end -- off.
#ifndef MDP_NT_SLAB
#define MDP_NT_SLAB 0
#endif
__device__ __forceinline__ void slab_st(float* p, float v) {
#if MDP_NT_SLAB == 3  // write-through vector store (global_store_dword sc1): no dirty L2 line at the kernel end
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#elif MDP_NT_SLAB == 2
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through (sc1)
#elif MDP_NT_SLAB
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void slab_st4(float* p, f32x4 v) {
#if MDP_NT_SLAB == 3  // one 16-B write-through store (the round-3 "sc1" variant was four 4-B ones)
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#elif MDP_NT_SLAB == 2
#pragma unroll
  for (int j = 0; j < 4; ++j) __hip_atomic_store(p + j, v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif MDP_NT_SLAB
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
#else
  *reinterpret_cast<f32x4*>(p) = v;
#endif
}
// Weight-gradient tiles are computed TRANSPOSED, dW^T tile = dY^T X (the
// MFMA's A operand from dY, B from X -- the same products in the same k
// order, so every element is bit-identical to the X^T dY form): a lane then
// holds dW[k][n .. n + 3] for one k, written as ONE 16-byte store instead of
// four 4-byte stores to four rows (N and the tensor offsets are multiples of 4).
// One weight-gradient job of wgrad_multi: dW[K][N] (global, stride N) of
// X^T[K][16] dY[16][N] (LDS operands); K = 0: no job
struct WgJob {
  const float* X;
  const float* dY;
  float* dW;
  int ldx, K, ldy, N;
};
// The tiles of up to three jobs, concatenated and dealt round-robin over waves
// [w0, w0 + wn).  A wave reads the LDS operands of T tiles at once and runs
// their MFMA chains interleaved before storing: one tile at a time, each
// 4-step chain waited on its LDS reads and on itself (40-cycle dependent MFMA
// latency), ~0.3 us per tile.  Each tile's chain is wgrad_waves' (same k
// order), so the result is bit-identical.  Tiles past the end re-read a valid
// tile (clamped) and store nothing.
template <int T>
__device__ __forceinline__ void wgrad_multi(const WgJob& j0, const WgJob& j1, const WgJob& j2, int w0, int wn) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < w0 || wave >= w0 + wn) return;
  const int r = lane & 15, kq = lane >> 4;
  const int n0 = ((j0.K + 15) >> 4) * (j0.N >> 4);
  const int n1 = j1.K > 0 ? ((j1.K + 15) >> 4) * (j1.N >> 4) : 0;
  const int n2 = j2.K > 0 ? ((j2.K + 15) >> 4) * (j2.N >> 4) : 0;
  const int total = n0 + n1 + n2;
  for (int base = wave - w0; base < total; base += T * wn) {
    float a[T][4], g[T][4];
    float* dst[T];
    bool krem[T];
#pragma unroll
    for (int s = 0; s < T; ++s) {
      const int tv = base + s * wn;
      const int t = min(tv, total - 1);
      const bool in0 = t < n0, in1 = !in0 && t < n0 + n1;
      const float* X = in0 ? j0.X : (in1 ? j1.X : j2.X);
      const float* dY = in0 ? j0.dY : (in1 ? j1.dY : j2.dY);
      float* dW = in0 ? j0.dW : (in1 ? j1.dW : j2.dW);
      const int ldx = in0 ? j0.ldx : (in1 ? j1.ldx : j2.ldx);
      const int K = in0 ? j0.K : (in1 ? j1.K : j2.K);
      const int ldy = in0 ? j0.ldy : (in1 ? j1.ldy : j2.ldy);
      const int N = in0 ? j0.N : (in1 ? j1.N : j2.N);
      const int tl = in0 ? t : (in1 ? t - n0 : t - n0 - n1);
      const int nnt = N >> 4, mt = tl / nnt, nt = tl - mt * nnt;
      const int feat = mt * 16 + r, fc = min(feat, K - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * i + kq;
        const float xv = X[row * ldx + fc];
        a[s][i] = feat < K ? xv : 0.f;
        g[s][i] = dY[row * ldy + nt * 16 + r];
      }
      dst[s] = dW + feat * N + nt * 16 + kq * 4;
      krem[s] = tv < total && feat < K;
    }
    __builtin_amdgcn_sched_barrier(0);  // every LDS read ahead of the MFMA chains
    f32x4 acc[T];
#pragma unroll
    for (int s = 0; s < T; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < T; ++s) acc[s] = MDP_MFMA(g[s][i], a[s][i], acc[s]);
#pragma unroll
    for (int s = 0; s < T; ++s)
      if (krem[s]) slab_st4(dst[s], acc[s]);
  }
}
__device__ __forceinline__ void wgrad_waves(const float* X, int ldx, int K, const float* dY, int ldy, int N,
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
    for (int r0 = 0; r0 < MDP_R; r0 += 4) {
      const int row = r0 + kq;
      const float xv = X[row * ldx + fc];
      const float a = feat < K ? xv : 0.f;
      const float g = dY[row * ldy + nt * 16 + r];
      acc = MDP_MFMA(g, a, acc);  // transposed tile
    }
    if (feat < K) slab_st4(dW + feat * N + nt * 16 + kq * 4, acc);
  }
}

