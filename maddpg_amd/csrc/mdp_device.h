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

// diagnostic build only (-DMDP_STAMPS): wall-clock stamps of workgroup 0
#ifdef MDP_STAMPS
__device__ unsigned long long g_mdp_stamps[64];
#define MDP_STAMP(i)                                                                     \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_mdp_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MDP_STAMP(i) \
  do {               \
  } while (0)
#endif

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
__device__ inline float u01(uint32_t x) {
  return __uint_as_float((x >> 9) | 0x3f800000u) - 1.0f;
}

// five uniforms for one (stream, counter, row) triple
__device__ inline void uniforms5(uint64_t seed, uint32_t stream, uint32_t ctr, uint32_t row, float u[5]) {
  uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  uint4 a = Philox::gen(make_uint4(row, ctr, stream, 0u), key);
  uint4 b = Philox::gen(make_uint4(row, ctr, stream, 1u), key);
  u[0] = u01(a.x); u[1] = u01(a.y); u[2] = u01(a.z); u[3] = u01(a.w); u[4] = u01(b.x);
}

// -------------------------------------------------------------- helpers
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// workgroup-wide sum (all threads get the result); scratch >= MDP_NW doubles
__device__ inline double block_sum_d(double v, double* scratch) {
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
__host__ __device__ inline int lds_ld(int cols) { return (cols | 1); }

// ------------------------------------------------------ MFMA layer tiles
// Y[16][N] = act(X[16][K] @ W[K][N] + b)   X,Y in LDS; W,b global row-major [K][N]
// N multiple of 16.  Column tiles are dealt round-robin over the 4 waves.
// B fragments of one 64-deep K chunk (16 MFMA k-steps) for one column: all 16
// global loads are issued together so the chunk pays one L2 latency, not 16.
#define MDP_KC 16
__device__ inline void load_wchunk(float (&w)[MDP_KC], const float* __restrict__ W, int ldw, int col, int c0,
                                   int K, int kq) {
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    w[s] = k < K ? W[k * ldw + col] : 0.f;
  }
}
// same for a transposed operand: element (k, col) at W[col * ldw + k]
__device__ inline void load_wchunk_t(float (&w)[MDP_KC], const float* __restrict__ W, int ldw, int col, int c0,
                                     int K, int kq, bool colok) {
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k = c0 + 4 * s + kq;
    w[s] = (k < K && colok) ? W[col * ldw + k] : 0.f;
  }
}
// acc += A[r][c0 .. c0+63] . w  with A from LDS (row r = lane&15)
__device__ inline f32x4 mfma_chunk(f32x4 acc, const float (&w)[MDP_KC], const float* A, int lda, int r, int c0,
                                   int K, int kq) {
#pragma unroll
  for (int s = 0; s < MDP_KC; ++s) {
    const int k0 = c0 + 4 * s;
    if (k0 < K) {  // wave-uniform
      const int k = k0 + kq;
      const float a = k < K ? A[r * lda + k] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[s], acc, 0, 0, 0);
    }
  }
  return acc;
}

template <bool RELU>
__device__ inline void tile_fwd(const float* X, int ldx, int K, const float* __restrict__ W,
                                const float* __restrict__ b, int N, float* Y, int ldy) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

// dW[K][N] = X^T[K][16] @ dY[16][N], written to global (row-major, stride N).
// Rows >= K are not written.
__device__ inline void tile_wgrad(const float* X, int ldx, int K, const float* dY, int ldy, int N,
                                  float* __restrict__ dW) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int nmt = (K + 15) >> 4, nnt = N >> 4;
  for (int t = wave; t < nmt * nnt; t += MDP_NW) {
    const int mt = t / nnt, nt = t - mt * nnt;
    const int feat = mt * 16 + r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r0 = 0; r0 < MDP_R; r0 += 4) {
      const int row = r0 + kq;
      const float a = feat < K ? X[row * ldx + feat] : 0.f;
      const float g = dY[row * ldy + nt * 16 + r];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, g, acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = mt * 16 + kq * 4 + i;
      if (k < K) dW[k * N + nt * 16 + r] = acc[i];
    }
  }
}

// dX[16][K] = (dY[16][N] @ W^T) masked by (H > 0) where H is the layer input
// (post-ReLU activations of the previous layer); K multiple of 16.
__device__ inline void tile_dgrad_relu(const float* dY, int ldy, int N, const float* __restrict__ W, int K,
                                       const float* Hin, int ldh, float* dX, int ldx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

// out[16][nout] = X[16][K] @ W[K][nout] + b  (small heads, VALU; 4 lanes per output)
__device__ inline void tile_head(const float* X, int ldx, int K, const float* __restrict__ W,
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
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (o < total && q == 0) {
      const int row = o / nout, c = o - row * nout;
      out[row * ldo + c] = s + b[c];
    }
  }
}

// softmax(logits - log(-log(u))) on one row of 5 (distributions.py:264-266)
__device__ inline void gumbel_softmax5(const float* logits, const float* u, float* a) {
  float z[MDP_ACT_DIM];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) {
    z[k] = logits[k] - logf(-logf(u[k]));
    m = fmaxf(m, z[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) {
    z[k] = expf(z[k] - m);
    s += z[k];
  }
#pragma unroll
  for (int k = 0; k < MDP_ACT_DIM; ++k) a[k] = z[k] / s;
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
