// mdp_kernels.hip -- HIP kernels of the MADDPG hot path for gfx950 (MI355X).
//
// Kernel map (reference site -> kernel):
//   replay_buffer.py:46-47  make_index        -> k_make_index   (CPython MT19937, 1 workgroup)
//   replay_buffer.py:34-44  _encode_sample    -> k_gather_rows  (+ fused into the grad kernels)
//   replay_buffer.py:25-32  add               -> k_put_rows / k_put_agent (+ fused into k_rollout)
//   maddpg.py:184-188       target_act + target_q + TD + q_train grads -> k_critic_grad
//   maddpg.py:46-61         p_train grads (through the critic's a_i input) -> k_actor_grad
//   tf_util.py:177-182 + TF ApplyAdam + maddpg.py:20-26 -> k_apply (clip, Adam, Polyak)
//   train.py:112-128 + MPE World.step -> k_rollout (actors + Gumbel + physics + obs/reward
//                                        + replay append + episode reset), k_env_reset
#include "mdp_device.h"
#include "mdp_kernels.h"
#include "mdp_mt.h"

// ================================================================ index
// count x randint(0, len-1): r = getrandbits(k) = temper(next) >> (32-k),
// k = len.bit_length(), rejected while r >= len (Lib/random.py _randbelow).
// Accepted draws are compacted with a workgroup prefix sum; the stream
// position after the count-th accepted draw is stored back (mdp_mt.h).
__global__ __launch_bounds__(1024) void k_make_index(Ctl* ctl, int count, int32_t* __restrict__ out) {
  make_index_block<1024>(ctl, count, out);
}

// ================================================================ replay
// out[b][:] = replay[idx[b]][:]   (float4 elements, rows contiguous).  32-bit
// element arithmetic (the host splits launches so count * stride / 4 < 2^31);
// each thread keeps 4 elements' index and row loads in flight before it stores,
// and the gathered rows are streamed out with nontemporal stores (measured
// 4M rows of 528 B: 5.25 -> 6.0 TB/s; bench.py gather_stage).
__device__ __forceinline__ void st_nt4(float* o, float4 v) {
  __builtin_nontemporal_store(v.x, o);
  __builtin_nontemporal_store(v.y, o + 1);
  __builtin_nontemporal_store(v.z, o + 2);
  __builtin_nontemporal_store(v.w, o + 3);
}

__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ replay, int stride,
                                                     const int32_t* __restrict__ idx, int count,
                                                     float* __restrict__ out) {
  const uint32_t v4 = (uint32_t)stride >> 2;
  const uint32_t total = (uint32_t)count * v4;
  const uint32_t step = gridDim.x * blockDim.x;
  uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  for (; e + 3u * step < total; e += 4u * step) {
    uint32_t b[4], c[4];
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t ee = e + (uint32_t)k * step;
      b[k] = ee / v4;
      c[k] = ee - b[k] * v4;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = *reinterpret_cast<const float4*>(replay + (int64_t)idx[b[k]] * stride + c[k] * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) st_nt4(out + (int64_t)b[k] * stride + c[k] * 4, v[k]);
  }
  for (; e < total; e += step) {
    const uint32_t b = e / v4, c = e - b * v4;
    st_nt4(out + (int64_t)b * stride + c * 4, *reinterpret_cast<const float4*>(replay + (int64_t)idx[b] * stride + c * 4));
  }
}

// ============================================================= check_nan
// non-finite entries of a float span -- the reference's _Function(check_nan)
// (tf_util.py:322,366-368) as an opt-in debug check (mdp_check_finite):
// grid-stride; a thread that saw any adds its count with one integer atomic
// (exact and order-independent; none at all on finite data)
__global__ __launch_bounds__(256) void k_count_nonfinite(const float* __restrict__ p, int64_t n, uint32_t* cnt) {
  uint32_t c = 0u;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += isfinite(p[i]) ? 0u : 1u;
  if (c) atomicAdd(cnt, c);
}

// ring append of whole rows: replay[(next + r) % cap] = src[r]
__global__ __launch_bounds__(256) void k_put_rows(float* __restrict__ replay, int stride, int64_t cap,
                                                  int64_t next, const float* __restrict__ src, int64_t rows) {
  const int v4 = stride >> 2;
  const int64_t total = rows * v4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / v4;
    const int c = (int)(e - r * v4);
    const int64_t dst = (next + r) % cap;
    *reinterpret_cast<float4*>(replay + dst * stride + c * 4) =
        *reinterpret_cast<const float4*>(src + r * stride + c * 4);
  }
}

// per-agent add (facade): cols = [obs(o) | act(5) | obs'(o) | rew | done] written at pos[r]
__global__ __launch_bounds__(256) void k_put_agent(float* __restrict__ replay, int stride, int obs_off,
                                                   int act_off, int nobs_off, int rew_off, int done_off,
                                                   int o, const int64_t* __restrict__ pos,
                                                   const float* __restrict__ cols, int64_t rows) {
  const int w = 2 * o + MDP_ACT_DIM + 2;
  const int64_t total = rows * w;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / w;
    const int c = (int)(e - r * w);
    int dc;
    if (c < o) dc = obs_off + c;
    else if (c < o + MDP_ACT_DIM) dc = act_off + (c - o);
    else if (c < 2 * o + MDP_ACT_DIM) dc = nobs_off + (c - o - MDP_ACT_DIM);
    else if (c == 2 * o + MDP_ACT_DIM) dc = rew_off;
    else dc = done_off;
    replay[pos[r] * stride + dc] = cols[e];
  }
}

// ================================================================ grads
namespace {

__device__ inline void gather_tile(const float* __restrict__ replay, int stride, const int32_t* __restrict__ idx,
                                   int r0, int nvalid, float* rowbuf, int ldr) {
  const int v4 = stride >> 2;
  for (int e = threadIdx.x; e < MDP_R * v4; e += MDP_NT) {
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

// copy ncols columns of a 16-row LDS tile
__device__ inline void copy_cols(const float* src, int lds_src, int src_off, float* dst, int lds_dst, int dst_off,
                                 int ncols) {
  for (int e = threadIdx.x; e < MDP_R * ncols; e += MDP_NT) {
    const int r = e / ncols, c = e - r * ncols;
    dst[r * lds_dst + dst_off + c] = src[r * lds_src + src_off + c];
  }
}

// column sums of a 16-row tile -> global
__device__ inline void colsum_store(const float* X, int ldx, int ncols, float* __restrict__ out) {
  for (int c = threadIdx.x; c < ncols; c += MDP_NT) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < MDP_R; ++r) s += X[r * ldx + c];
    out[c] = s;
  }
}

// mlp_fwd_tile for H = 64 / 128 with in <= 64 (one 64-deep weight chunk for
// layer 1): every fragment of the wave's column tiles -- both layers, and the
// head's on wave 0 -- is requested before the first MFMA, one memory round
// trip per net instead of one per layer and tile (at H = 128 the rollout ran
// about seven per agent).  Same tiles, chunk order and head as mlp_fwd_tile<H>:
// bit-identical.
template <int H>
__device__ inline void mlp_fwd_tile_pf(const float* X, int ldx, int K, const float* P, const NDesc& nd, float* h1,
                                       float* h2, int ldh, float* out, int ldo) {
  static_assert(H == 64 || H == 128, "register budget: H <= 128");
  constexpr int TW = H / (16 * MDP_NW);  // column tiles per wave (tile_fwd deals nt = wave + t * MDP_NW)
  constexpr int KC2 = H / (4 * MDP_KC);  // 64-deep chunks of layer 2
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, kq = lane >> 4;
  float w1[TW][MDP_KC], w2[TW][KC2][MDP_KC], w3[H / 4], b3 = 0.f, b1[TW], b2[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int col = (wave + t * MDP_NW) * 16 + r;
    load_wchunk(w1[t], P + nd.t[0].off, H, col, 0, K, kq);
#pragma unroll
    for (int c = 0; c < KC2; ++c) load_wchunk(w2[t][c], P + nd.t[2].off, H, col, c * 4 * MDP_KC, H, kq);
  }
  if (wave == 0) head_load<H / 4>(w3, b3, P + nd.t[4].off, P + nd.t[5].off, nd.out);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int col = (wave + t * MDP_NW) * 16 + r;
    b1[t] = P[nd.t[1].off + col];
    b2[t] = P[nd.t[3].off + col];
  }
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int col = (wave + t * MDP_NW) * 16 + r;
    const f32x4 acc = mfma_chunk(f32x4{0.f, 0.f, 0.f, 0.f}, w1[t], X, ldx, r, 0, K, kq);
#pragma unroll
    for (int i = 0; i < 4; ++i) h1[(kq * 4 + i) * ldh + col] = fmaxf(acc[i] + b1[t], 0.f);
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int col = (wave + t * MDP_NW) * 16 + r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC2; ++c) acc = mfma_chunk(acc, w2[t][c], h1, ldh, r, c * 4 * MDP_KC, H, kq);
#pragma unroll
    for (int i = 0; i < 4; ++i) h2[(kq * 4 + i) * ldh + col] = fmaxf(acc[i] + b2[t], 0.f);
  }
  __syncthreads();
  if (wave == 0) head_acc<H / 4>(w3, b3, h2, ldh, nd.out, out, ldo);
  __syncthreads();
}

template <int H>
__device__ inline void mlp_fwd_tile(const float* X, int ldx, int K, const float* P, const NDesc& nd, float* h1,
                                    float* h2, int ldh, float* out, int ldo) {
  tile_fwd<true>(X, ldx, K, P + nd.t[0].off, P + nd.t[1].off, H, h1, ldh);
  __syncthreads();
  tile_fwd<true>(h1, ldh, H, P + nd.t[2].off, P + nd.t[3].off, H, h2, ldh);
  __syncthreads();
  if (threadIdx.x < 64) head_mfma<H / 4>(h2, ldh, H, P + nd.t[4].off, P + nd.t[5].off, nd.out, out, ldo);
  __syncthreads();
}

}  // namespace

// ================================================================ apply
namespace {
// true in every thread of the last workgroup to arrive (no static LDS: keeps
// the dynamic LDS base 16-B aligned)
__device__ inline bool last_block(uint32_t* ticket) {
  int last = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t old = atomicAdd(ticket, 1u);
    last = (old == gridDim.x - 1) ? 1 : 0;
  }
  return __syncthreads_or(last) != 0;
}
}  // namespace

// grad[e] = sum_w slab[w][e] in fixed w order (deterministic); one element per
// thread, the nwg partial loads unrolled 8-wide so they are in flight together.
// Thread 0 also advances the optimizer step (replaces the AdamOptimizer._finish
// beta-power update): beta[2..3] <- beta[0..1] (powers this step's ApplyAdam
// uses), beta[0..1] *= (b1, b2) in fp32.  k_reduce always precedes k_apply in
// stream order, so no cross-workgroup protocol is needed.
__global__ __launch_bounds__(256) void k_reduce(ReduceArgs a) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e == 0 && a.beta) {
    const float p1 = a.beta[0], p2 = a.beta[1];
    a.beta[2] = p1;
    a.beta[3] = p2;
    a.beta[0] = p1 * a.b1;
    a.beta[1] = p2 * a.b2;
    if (a.bump_ctr) a.ctl->upd_ctr += 1u;
  }
  // 8 lanes per element: lane q sums partials w = q, q+8, ... (all loads in
  // flight at once), then a fixed xor-tree over the 8 lanes -> deterministic
  const int64_t el = e >> 3;
  const int q = (int)(e & 7);
  float s = 0.f;
  if (el < a.size) {
    const float* p = a.slab + el;
    float v[8], t[24];  // up to 32 partials per lane (B <= 4096) in flight at once
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int w = q + 8 * k;
      v[k] = w < a.nwg ? p[(int64_t)w * a.slab_stride] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 24; ++k) {
      const int w = q + 64 + 8 * k;
      t[k] = w < a.nwg ? p[(int64_t)w * a.slab_stride] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 24; ++k)
      if (q + 64 + 8 * k < a.nwg) s += t[k];
    for (int w = q + 256; w < a.nwg; w += 8) s += p[(int64_t)w * a.slab_stride];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  s = half_row_sum(s);
  if (el < a.size && q == 0) a.grad[a.off + el] = s;
}

// Workgroup (tensor t, chunk c) of `net`: per-tensor clip_by_norm (norm of the
// whole scaled tensor, recomputed by every chunk from the reduced gradient),
// TF1 ApplyAdam on the chunk, optional Polyak of the chunk; then Polyak chunks
// of `other` (actor step only) and one stats workgroup.  The last workgroup to
// finish advances this optimizer's beta powers.
__global__ __launch_bounds__(256) void k_apply(ApplyArgs a) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float b1p = a.beta[2], b2p = a.beta[3];  // powers for this step, latched by k_reduce
  if (b < a.blk[6]) {
    int t = 0;
    while (b >= a.blk[t + 1]) ++t;
    const TDesc td = a.net.t[t];
    const int n = td.rows * td.cols;
    const float* g = a.grad + td.off;
    // this block's chunk of grad / m / v / theta / target is requested together with
    // the whole-tensor norm loads, so the block pays ONE memory round trip
    constexpr int PT = MDP_APPLY_CHUNK / 256;  // parameters per thread
    const int e0 = (b - a.blk[t]) * MDP_APPLY_CHUNK;
    const int e1 = min(n, e0 + MDP_APPLY_CHUNK);
    float cg[PT], cm[PT], cv[PT], cth[PT], ctg[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int e = min(e0 + tid + q * 256, e1 - 1);
      const int64_t i = td.off + e;
      cg[q] = g[e];
      cm[q] = a.m[i];
      cv[q] = a.v[i];
      cth[q] = a.theta[i];
      ctg[q] = a.polyak ? a.target[i] : 0.f;
    }
    double ss = 0.0;
    for (int f0 = tid; f0 < n; f0 += 8 * blockDim.x) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int e = f0 + q * blockDim.x;
        v[q] = e < n ? g[min(e, n - 1)] * a.scale : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += (double)v[q] * (double)v[q];
    }
    ss = block_sum_d(ss, red);
    const float norm = (float)sqrt(ss);
    const float clip = a.clip;
    const float denom = fmaxf(norm, clip);
    const float one = 1.0f;
    const float alpha = a.lr * sqrtf(one - b2p) / (one - b1p);
    const float c1 = one - a.b1, c2 = one - a.b2;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int e = e0 + tid + q * 256;
      if (e < e1) {
        const int64_t i = td.off + e;
        const float gc = ((cg[q] * a.scale) * clip) / denom;
        const float m = cm[q] + (gc - cm[q]) * c1;
        const float v = cv[q] + (gc * gc - cv[q]) * c2;
        const float th = cth[q] - (m * alpha) / (sqrtf(v) + a.eps);
        a.m[i] = m;
        a.v[i] = v;
        a.theta[i] = th;
        if (a.polyak) a.target[i] = a.pa * ctg[q] + a.pb * th;
      }
    }
  } else if (a.polyak && b < a.blk[6] + a.oblk[6]) {
    const int bb = b - a.blk[6];
    int t = 0;
    while (bb >= a.oblk[t + 1]) ++t;
    const TDesc td = a.other.t[t];
    const int n = td.rows * td.cols;
    const int e0 = (bb - a.oblk[t]) * MDP_APPLY_CHUNK;
    const int e1 = min(n, e0 + MDP_APPLY_CHUNK);
    for (int e = e0 + tid; e < e1; e += blockDim.x) {
      const int64_t i = td.off + e;
      a.target[i] = a.pa * a.target[i] + a.pb * a.theta[i];
    }
  } else if (a.stats_mode) {
    // stats workgroup (maddpg.py:196): critic fills 0,2,3,4,5; actor fills 1
    // one wave, lane-strided partial sums + fixed xor trees (deterministic, no barriers)
    if (tid < 64) {
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      for (int w = tid; w < a.nwg; w += 64) {
        const double* st = a.slab_stat + (int64_t)w * 8;
        s0 += st[0];
        s1 += st[1];
        s2 += st[2];
        s3 += st[3];
      }
      s0 = wave_sum_d(s0);
      s1 = wave_sum_d(s1);
      if (a.stats_mode == 1) {
        s2 = wave_sum_d(s2);
        s3 = wave_sum_d(s3);
        const double mean_y = s1 / a.B;
        double dv = 0.0;
        for (int i = tid; i < a.B; i += 64) {
          const double d = a.y[i] - mean_y;
          dv += d * d;
        }
        dv = wave_sum_d(dv);
        if (tid == 0) {
          a.stats_out[0] = s0 / a.B;
          a.stats_out[2] = mean_y;
          a.stats_out[3] = s2 / a.B;
          a.stats_out[4] = s3 / a.B;
          a.stats_out[5] = sqrt(dv / a.B);
        }
      } else if (tid == 0) {
        a.stats_out[1] = -s0 / a.B + (double)a.reg * (s1 / ((double)a.B * MDP_ACT_DIM));
      }
    }
  }
}

// ================================================================ env
namespace {

struct EnvTile {
  float* pos;  // [16][ne][2]
  float* vel;
};

__device__ inline float softplus_f(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }

__device__ inline float dist2(const float* p, int a, int b) {
  const float dx = p[2 * a] - p[2 * b], dy = p[2 * a + 1] - p[2 * b + 1];
  return sqrtf(dx * dx + dy * dy);
}

// observation of agent i into o[] (scenario observation(), see oracle/mpe.py)
__device__ inline void env_obs(const EnvDesc& E, const float* p, const float* v, int goal, int i, float* o) {
  const int n = E.n_agents, L = E.n_landmarks;
  int c = 0;
  switch (E.scenario) {
    case MDP_SCN_SIMPLE:
      o[c++] = v[2 * i];
      o[c++] = v[2 * i + 1];
      for (int l = 0; l < L; ++l) {
        o[c++] = p[2 * (n + l)] - p[2 * i];
        o[c++] = p[2 * (n + l) + 1] - p[2 * i + 1];
      }
      break;
    case MDP_SCN_SPREAD:
      o[c++] = v[2 * i];
      o[c++] = v[2 * i + 1];
      o[c++] = p[2 * i];
      o[c++] = p[2 * i + 1];
      for (int l = 0; l < L; ++l) {
        o[c++] = p[2 * (n + l)] - p[2 * i];
        o[c++] = p[2 * (n + l) + 1] - p[2 * i + 1];
      }
      for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        o[c++] = p[2 * j] - p[2 * i];
        o[c++] = p[2 * j + 1] - p[2 * i + 1];
      }
      for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        o[c++] = 0.f;  // other.state.c (silent agents)
        o[c++] = 0.f;
      }
      break;
    case MDP_SCN_ADVERSARY:
      if (!E.adversary[i]) {
        o[c++] = p[2 * (n + goal)] - p[2 * i];
        o[c++] = p[2 * (n + goal) + 1] - p[2 * i + 1];
      }
      for (int l = 0; l < L; ++l) {
        o[c++] = p[2 * (n + l)] - p[2 * i];
        o[c++] = p[2 * (n + l) + 1] - p[2 * i + 1];
      }
      for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        o[c++] = p[2 * j] - p[2 * i];
        o[c++] = p[2 * j + 1] - p[2 * i + 1];
      }
      break;
    case MDP_SCN_TAG:
      o[c++] = v[2 * i];
      o[c++] = v[2 * i + 1];
      o[c++] = p[2 * i];
      o[c++] = p[2 * i + 1];
      for (int l = 0; l < L; ++l) {
        o[c++] = p[2 * (n + l)] - p[2 * i];
        o[c++] = p[2 * (n + l) + 1] - p[2 * i + 1];
      }
      for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        o[c++] = p[2 * j] - p[2 * i];
        o[c++] = p[2 * j + 1] - p[2 * i + 1];
      }
      for (int j = 0; j < n; ++j) {
        if (j == i || E.adversary[j]) continue;
        o[c++] = v[2 * j];
        o[c++] = v[2 * j + 1];
      }
      break;
    default:
      break;
  }
}

// rewards of all agents (scenario reward() + shared reward for collaborative worlds)
__device__ inline void env_reward(const EnvDesc& E, const float* p, int goal, float* rew) {
  const int n = E.n_agents, L = E.n_landmarks;
  switch (E.scenario) {
    case MDP_SCN_SIMPLE: {
      const float dx = p[0] - p[2 * n], dy = p[1] - p[2 * n + 1];
      rew[0] = -(dx * dx + dy * dy);
      break;
    }
    case MDP_SCN_SPREAD: {
      float base = 0.f;
      for (int l = 0; l < L; ++l) {
        float m = INFINITY;
        for (int a = 0; a < n; ++a) m = fminf(m, dist2(p, a, n + l));
        base -= m;
      }
      float tot = 0.f;
      for (int i = 0; i < n; ++i) {
        float r = base;
        for (int a = 0; a < n; ++a)
          if (dist2(p, a, i) < E.size[a] + E.size[i]) r -= 1.f;
        tot += r;
      }
      for (int i = 0; i < n; ++i) rew[i] = tot;  // world.collaborative: reward_n = [sum] * n
      break;
    }
    case MDP_SCN_ADVERSARY: {
      const int g = n + goal;
      float adv = 0.f, mg = INFINITY;
      for (int a = 0; a < n; ++a) {
        if (E.adversary[a]) adv += dist2(p, a, g);
        else mg = fminf(mg, dist2(p, a, g));
      }
      for (int i = 0; i < n; ++i) {
        if (E.adversary[i]) {
          const float dx = p[2 * i] - p[2 * g], dy = p[2 * i + 1] - p[2 * g + 1];
          rew[i] = -(dx * dx + dy * dy);
        } else {
          rew[i] = -mg + adv;
        }
      }
      break;
    }
    case MDP_SCN_TAG: {
      float caught = 0.f;
      for (int g = 0; g < n; ++g) {
        if (E.adversary[g]) continue;
        for (int a = 0; a < n; ++a)
          if (E.adversary[a] && dist2(p, g, a) < E.size[g] + E.size[a]) caught += 1.f;
      }
      for (int i = 0; i < n; ++i) {
        if (E.adversary[i]) {
          rew[i] = 10.f * caught;
        } else {
          float r = 0.f;
          for (int a = 0; a < n; ++a)
            if (E.adversary[a] && dist2(p, a, i) < E.size[a] + E.size[i]) r -= 10.f;
          for (int d = 0; d < 2; ++d) {
            const float x = fabsf(p[2 * i + d]);
            float bnd = 0.f;
            if (x < 0.9f) bnd = 0.f;
            else if (x < 1.0f) bnd = (x - 0.9f) * 10.f;
            else bnd = fminf(expf(2.f * x - 2.f), 10.f);
            r -= bnd;
          }
          rew[i] = r;
        }
      }
      break;
    }
    default:
      break;
  }
}

// scenario benchmark_data() of every agent (MPE environment._get_info with
// info_callback = scenario.benchmark_data, train.py:57-60,139-141) into
// out[n][MDP_BENCH_W], zero-padded.  Same post-physics state as env_reward.
__device__ inline void env_bench(const EnvDesc& E, const float* p, int goal, float* out) {
  const int n = E.n_agents, L = E.n_landmarks;
  for (int q = 0; q < n * MDP_BENCH_W; ++q) out[q] = 0.f;
  switch (E.scenario) {
    case MDP_SCN_SPREAD: {
      float min_dists = 0.f, occupied = 0.f;
      for (int l = 0; l < L; ++l) {
        float m = INFINITY;
        for (int a = 0; a < n; ++a) m = fminf(m, dist2(p, a, n + l));
        min_dists += m;
        if (m < 0.1f) occupied += 1.f;
      }
      for (int i = 0; i < n; ++i) {
        float coll = 0.f;
        for (int a = 0; a < n; ++a)
          if (dist2(p, a, i) < E.size[a] + E.size[i]) coll += 1.f;  // includes self
        float* o = out + i * MDP_BENCH_W;
        o[0] = -min_dists - coll;
        o[1] = coll;
        o[2] = min_dists;
        o[3] = occupied;
      }
      break;
    }
    case MDP_SCN_ADVERSARY: {
      const int g = n + goal;
      for (int i = 0; i < n; ++i) {
        float* o = out + i * MDP_BENCH_W;
        auto sq = [&](int b) {
          const float dx = p[2 * i] - p[2 * b], dy = p[2 * i + 1] - p[2 * b + 1];
          return dx * dx + dy * dy;
        };
        if (E.adversary[i]) {
          o[0] = sq(g);
        } else {
          for (int l = 0; l < L; ++l) o[l] = sq(n + l);
          o[L] = sq(g);
        }
      }
      break;
    }
    case MDP_SCN_TAG: {
      for (int i = 0; i < n; ++i) {
        if (!E.adversary[i]) continue;
        float c = 0.f;
        for (int a = 0; a < n; ++a)
          if (!E.adversary[a] && dist2(p, a, i) < E.size[a] + E.size[i]) c += 1.f;
        out[i * MDP_BENCH_W] = c;
      }
      break;
    }
    default:
      break;
  }
}

// World.step (core.py) for a tile of envs: action force, pairwise soft contact,
// damping, integration with max_speed clamp.  One thread per (env, entity)
// (one thread per env ran 33 of the 98 us S5 rollout): the force on entity e is
// summed over its contacts in the order the pair loop of core.py adds them --
// pairs (o, e) for o < e, then (e, o) for o > e -- with each pair's force
// computed in the same (a < b) orientation, so the result is bit-identical to
// the one-thread-per-env loop (and the oracle's); then damping and integration,
// after a barrier (they move the positions the contacts read).  sp / sv: the
// tile's [R][2 MDP_MAX_ENT] state; f: [R][3 MDP_MAX_ENT] force scratch; act:
// row r's actions at act + r * ldr.  Every thread of the workgroup calls it.
__device__ inline void env_physics_tile(const EnvDesc& E, float* sp, float* sv, const float* act, int ldr, float* f,
                                        int nvalid) {
  const int n = E.n_agents, ne = E.n_agents + E.n_landmarks;
  const float k = 1e-3f;  // contact_margin
  for (int q = threadIdx.x; q < nvalid * ne; q += MDP_NT) {
    const int r = q / ne, e = q - r * ne;
    const float* p = sp + r * 2 * MDP_MAX_ENT;
    float fx = 0.f, fy = 0.f, has = 0.f;
    if (e < n) {  // environment._set_action, discrete action space
      const float* a = act + r * ldr + e * MDP_ACT_DIM;
      fx = (a[1] - a[2]) * E.accel[e];
      fy = (a[3] - a[4]) * E.accel[e];
      has = 1.f;
    }
    if (E.collide[e] && E.movable[e]) {
      for (int o = 0; o < ne; ++o) {
        if (o == e || !E.collide[o]) continue;
        const int a = min(o, e), b = max(o, e);
        const float dx = p[2 * a] - p[2 * b], dy = p[2 * a + 1] - p[2 * b + 1];
        const float dist = sqrtf(dx * dx + dy * dy);
        const float dmin = E.size[a] + E.size[b];
        const float pen = softplus_f(-(dist - dmin) / k) * k;
        const float sx = 1e2f * dx / dist * pen, sy = 1e2f * dy / dist * pen;
        if (e == a) {
          fx = sx + fx;
          fy = sy + fy;
        } else {
          fx = -sx + fx;
          fy = -sy + fy;
        }
        has = 1.f;
      }
    }
    float* fr = f + r * 3 * MDP_MAX_ENT;
    fr[e] = fx;
    fr[MDP_MAX_ENT + e] = fy;
    fr[2 * MDP_MAX_ENT + e] = has;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < nvalid * ne; q += MDP_NT) {
    const int r = q / ne, e = q - r * ne;
    if (!E.movable[e]) continue;
    float* p = sp + r * 2 * MDP_MAX_ENT;
    float* v = sv + r * 2 * MDP_MAX_ENT;
    const float* fr = f + r * 3 * MDP_MAX_ENT;
    float vx = v[2 * e] * (1.f - 0.25f), vy = v[2 * e + 1] * (1.f - 0.25f);
    if (fr[2 * MDP_MAX_ENT + e] != 0.f) {
      vx += (fr[e] / 1.f) * 0.1f;
      vy += (fr[MDP_MAX_ENT + e] / 1.f) * 0.1f;
    }
    const float ms = E.max_speed[e];
    if (ms >= 0.f) {
      const float spd = sqrtf(vx * vx + vy * vy);
      if (spd > ms) {
        const float s = sqrtf(vx * vx + vy * vy);
        vx = vx / s * ms;
        vy = vy / s * ms;
      }
    }
    v[2 * e] = vx;
    v[2 * e + 1] = vy;
    p[2 * e] += vx * 0.1f;
    p[2 * e + 1] += vy * 0.1f;
  }
  __syncthreads();
}

// reset_world of one env from Philox uniforms.  Uniform slot c (2 per entity in
// entity order, then the adversary goal) is word c % 4 of the Philox block at
// counter (env, ctr, stream, c / 4); the slots are consumed in order, so each
// block is generated when its first word is needed -- up to 2 MDP_MAX_ENT + 1
// slots (an earlier revision kept a fixed 20 and read past it beyond 10 entities)
__device__ inline void env_reset_one(const EnvDesc& E, uint64_t seed, uint32_t stream, uint32_t ctr, uint32_t env,
                                     float* p, float* v, int32_t* goal) {
  const int n = E.n_agents, ne = E.n_agents + E.n_landmarks;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  uint4 blk = make_uint4(0u, 0u, 0u, 0u);
  int c = 0;
  auto next_u = [&]() -> float {
    const int w = c & 3;
    if (w == 0) blk = Philox::gen(make_uint4(env, ctr, stream, (uint32_t)(c >> 2)), key);
    ++c;
    return u01(w == 0 ? blk.x : w == 1 ? blk.y : w == 2 ? blk.z : blk.w);
  };
  for (int e = 0; e < ne; ++e) {
    float lo = -1.f, hi = 1.f, sc = 1.f;
    if (e >= n) {
      if (E.scenario == MDP_SCN_SPREAD || E.scenario == MDP_SCN_ADVERSARY) sc = 0.8f;
      if (E.scenario == MDP_SCN_TAG) {
        lo = -0.9f;
        hi = 0.9f;
      }
    }
    const float ux = next_u();
    const float uy = next_u();
    p[2 * e] = sc * (lo + (hi - lo) * ux);
    p[2 * e + 1] = sc * (lo + (hi - lo) * uy);
    v[2 * e] = 0.f;
    v[2 * e + 1] = 0.f;
  }
  if (E.scenario == MDP_SCN_ADVERSARY) {
    int g = (int)(next_u() * E.n_landmarks);
    *goal = g < E.n_landmarks ? g : E.n_landmarks - 1;
  } else {
    *goal = 0;
  }
}

}  // namespace

__global__ __launch_bounds__(256) void k_env_reset(EnvResetArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.E) return;
  const int ne = a.env.n_agents + a.env.n_landmarks;
  float p[2 * MDP_MAX_ENT], v[2 * MDP_MAX_ENT];
  int32_t g;
  env_reset_one(a.env, a.seed, 0x30000u, a.ctr, (uint32_t)(a.env_base + e), p, v, &g);
  for (int q = 0; q < 2 * ne; ++q) {
    a.pos[(int64_t)e * 2 * ne + q] = p[q];
    a.vel[(int64_t)e * 2 * ne + q] = v[q];
  }
  a.goal[e] = g;
  a.ep_step[e] = 0;
  for (int j = 0; j < a.env.n_agents; ++j) a.ep_rew[(int64_t)e * a.env.n_agents + j] = 0.f;
}

// current observations [E][sum_obs]
__global__ __launch_bounds__(256) void k_env_obs(EnvObsArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.E) return;
  const int ne = a.env.n_agents + a.env.n_landmarks;
  const float* p = a.pos + (int64_t)e * 2 * ne;
  const float* v = a.vel + (int64_t)e * 2 * ne;
  float* o = a.obs + (int64_t)e * a.topo.sum_obs;
  for (int j = 0; j < a.env.n_agents; ++j) env_obs(a.env, p, v, a.goal[e], j, o + a.topo.ag[j].obs_off);
}

// One vector env step for 16 env copies per workgroup (train.py:112-128).
// the last workgroup to arrive advances the ring and the env step counter
__device__ __forceinline__ void rollout_finish(const RolloutArgs& a, int64_t next, int64_t len) {
  if (last_block(a.ticket) && threadIdx.x == 0) {
    const int64_t moved = (int64_t)a.nsteps * a.E;  // a.nsteps env steps in this launch
    a.ctl->next = (next + moved) % a.cap;
    a.ctl->len = len + moved < a.cap ? len + moved : a.cap;
    a.ctl->env_steps += (uint64_t)a.nsteps;
    a.ctl->episodes += atomicExch(&a.ctl->ep_pending, 0u);
    *a.ticket = 0u;
  }
}

// MULTI: the a.nsteps > 1 instantiation (the one-step launch keeps its
// straight-line schedule: a run-time loop around the body cost it 1.3 us)
template <int H, bool MULTI>
__global__ __launch_bounds__(MDP_NT) void k_rollout(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  MDP_TL_ROLLOUT();
  const Topo& T = a.topo;
  const EnvDesc& E = a.env;
  const int n = E.n_agents, ne = E.n_agents + E.n_landmarks;
  const int ldr = lds_ld(T.row_stride), ldh = H + 1;
  LdsCarve cv(lds);
  float* rowt = cv.take(MDP_R * ldr);
  float* h1 = cv.take(MDP_R * ldh);
  float* h2 = cv.take(MDP_R * ldh);
  float* lg = cv.take(MDP_R * 8);
  // H = 64: every agent's policy forward on its own wave (rollout_par), h1 | h2 | logits per agent
  constexpr int PAR_W = H == 64 ? MDP_NW * (2 * MDP_R * MDP_RLH + MDP_R * 8) : 0;
  float* hpar = cv.take(PAR_W);
  float* sp = cv.take(MDP_R * 2 * MDP_MAX_ENT);
  float* sv = cv.take(MDP_R * 2 * MDP_MAX_ENT);
  float* sfo = cv.take(MDP_R * 3 * MDP_MAX_ENT);  // per-env force scratch of env_physics
  float* epr = cv.take(MDP_R * MDP_MAX_AGENTS);    // the envs' running episode rewards
  int* sgoal = reinterpret_cast<int*>(cv.take(MDP_R));  // the envs' goal landmarks

  const int tid = threadIdx.x;
  // with a draw workgroup it is block 0 (dispatched first: at tag6 B=4096 the
  // draw is 24,576 indices) and the env copies start at block 1
  const int e0 = ((int)blockIdx.x - (a.pf_count > 0 ? 1 : 0)) * MDP_R;
  const int nvalid = min(MDP_R, a.E - e0);
  // Ctl fields written by earlier launches: issued here, consumed as opaque
  // VGPRs where they are used (ctr_use) -- made SGPRs at the load, they were
  // waited for in front of the state loads
  // (through a VGPR copy of the pointer: as scalar loads they shared lgkmcnt
  // with the kernarg reads, and the first kernarg wait waited for them too)
  const Ctl* ctlv = a.ctl;
  asm volatile("" : "+v"(ctlv));
  typedef __attribute__((address_space(1))) const Ctl gCtl;  // global, not FLAT
  const gCtl* gc = (const gCtl*)ctlv;
  if (a.pf_count > 0 && blockIdx.x == 0) {
    const int64_t next = gc->next, len = gc->len;
    // the index draw of the step's first round, off the critical path: the
    // MT state is untouched by the env workgroups, and the length is the one
    // the last workgroup below will store (every workgroup read ctl->len
    // before arriving at the ticket)
    MDP_STAMP(48);
    make_index_block<MDP_NT>(a.ctl, a.pf_count, a.pf_out, (uint32_t)(len + a.E < a.cap ? len + a.E : a.cap));
    MDP_STAMP(49);
    rollout_finish(a, next, len);
    return;
  }

  MDP_STAMP(40);
  // every env-state load of the step issued up front (the episode bookkeeping
  // read ep_rew / ep_step from memory in the physics phase: a round trip there)
  // (all loads first, then the LDS stores: a load-store loop waited for each
  // load before the next loop's loads issued; goal / ep_step stay opaque
  // VGPRs until used, or the compiler waits for them right here)
  int goal = 0, ep_st = 0;
  if (tid < MDP_R && tid < nvalid) {
    goal = a.goal[e0 + tid];
    ep_st = a.ep_step[e0 + tid];
  }
  static_assert(MDP_R * 2 * MDP_MAX_ENT <= 2 * MDP_NT && MDP_R * MDP_MAX_AGENTS <= MDP_NT, "rollout prologue");
  float pv[2] = {0.f, 0.f}, vv[2] = {0.f, 0.f}, er = 0.f;
  const int er_r = tid / n, er_j = tid - er_r * n;
  if (tid < MDP_R * n && er_r < nvalid) er = a.ep_rew[(int64_t)(e0 + er_r) * n + er_j];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + u * MDP_NT, r = q / (2 * ne), c = q - r * 2 * ne;
    if (q < MDP_R * 2 * ne && r < nvalid) {
      pv[u] = a.pos[(int64_t)(e0 + r) * 2 * ne + c];
      vv[u] = a.vel[(int64_t)(e0 + r) * 2 * ne + c];
    }
  }
  // (issued after the state loads: a register reused behind them made an
  // earlier wait for this one)
  const int64_t next_raw = gc->next, len_raw = gc->len;
  const uint32_t step_raw = (uint32_t)gc->env_steps;
  const int64_t ep_base_raw = gc->episodes;  // advanced only by this launch's last workgroup
  if (tid < MDP_R * n) epr[er_r * MDP_MAX_AGENTS + er_j] = er;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + u * MDP_NT, r = q / (2 * ne), c = q - r * 2 * ne;
    if (q < MDP_R * 2 * ne) {
      sp[r * 2 * MDP_MAX_ENT + c] = pv[u];
      sv[r * 2 * MDP_MAX_ENT + c] = vv[u];
    }
  }
  if (tid < MDP_R) sgoal[tid] = (int)ctr_use((uint32_t)goal);
  // a.nsteps > 1 (one env workgroup, no draw, no injected actions: the host's
  // mdp_rollout_steps_ok) runs that many consecutive env steps of a stretch
  // without update rounds, the env state kept in LDS and registers between
  // them; each step is exactly the launch's one step (same counters, same order)
  __shared__ int s_nterm;  // this step's finished episodes (lockstep log slots)
  int ep_done = 0;         // episodes finished in this launch's earlier steps
  const int nsteps = MULTI ? a.nsteps : 1;
  for (int sidx = 0; sidx < nsteps; ++sidx) {
  if (MULTI && sidx > 0) __syncthreads();  // the previous step's replay rows are out of rowt
  // this step's counter, read where it is used (an opaque VGPR, as the Ctl fields above)
  auto step_s = [&]() { return ctr_use(step_raw) + (uint32_t)sidx; };
  const int64_t next_s = next_raw + (int64_t)sidx * a.E;
  for (int q = tid; q < MDP_R * ldr; q += MDP_NT) rowt[q] = 0.f;
  if (MULTI && tid == 0) s_nterm = 0;
  __syncthreads();
  // observations, one thread per (env, agent)
  static_assert(MDP_R * MDP_MAX_AGENTS <= MDP_NT, "rollout obs: one pass");
  if (tid < MDP_R * n) {
    const int r = tid / n, j = tid - r * n;
    env_obs(E, sp + r * 2 * MDP_MAX_ENT, sv + r * 2 * MDP_MAX_ENT, sgoal[r], j, rowt + r * ldr + T.ag[j].obs_off);
  }
  __syncthreads();

  MDP_STAMP(41);
  // policies: act_j = gumbel_softmax(actor_j(obs_j))  (MADDPGAgentTrainer.action).
  // H = 64, n <= 4 agents: wave j runs agent j's whole forward from registers
  // (all its fragments requested at once, the register kernels' one-wave net),
  // the agents in parallel -- one after another over all four waves they took
  // ~3 us each (stamped); the same MFMA k order per output, so the same values
  bool par = false;
  if constexpr (H == 64) {
    par = !a.act_in && n <= MDP_NW;
    for (int j = 0; j < n; ++j) par = par && T.ag[j].obs_dim <= 64;
  }
  if (par) {
    if constexpr (H == 64) {
      const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 15, kq = lane >> 4;
      if (wave < n) {
        const int j = wave;
        const ADesc& aj = T.ag[j];
        const NDesc& an = aj.actor;
        const float* P = a.theta;
        f32x4 w1[16], w2[16];
        float w3[16];
        rf_load<16>(w1, P + an.t[0].off, aj.obs_dim);
        rf_load<16>(w2, P + an.t[2].off, MDP_RH);
        rh_load(w3, P + an.t[4].off, MDP_ACT_DIM);
        const f32x4 b1 = ld4(P + an.t[1].off + 4 * r), b2 = ld4(P + an.t[3].off + 4 * r);
        const float b3 = P[an.t[5].off + min(r, MDP_ACT_DIM - 1)];
        float u[MDP_ACT_DIM];  // the sample's uniforms, while the weights are in flight
        if (lane < MDP_R) {
          if (a.u_in) {
            for (int k = 0; k < MDP_ACT_DIM; ++k)
              u[k] = lane < nvalid ? a.u_in[((int64_t)(e0 + lane) * n + j) * MDP_ACT_DIM + k] : 0.5f;
          } else {
            uniforms5(a.seed, 0x10000u | (uint32_t)j, step_s(), (uint32_t)(a.env_base + e0 + lane), u);
          }
        }
        float* h1j = hpar + j * (2 * MDP_R * MDP_RLH + MDP_R * 8);
        float* h2j = h1j + MDP_R * MDP_RLH;
        float* lgj = h2j + MDP_R * MDP_RLH;
        {
          f32x4 acc[4];
          rf_zero(acc);
          rf_acc<16>(acc, rowt + aj.obs_off, ldr, aj.obs_dim, w1);
          rf_store<true>(acc, b1, h1j, MDP_RLH);
        }
        wave_sync();
        {
          f32x4 acc[4];
          rf_zero(acc);
          rf_acc<16>(acc, h1j, MDP_RLH, MDP_RH, w2);
          rf_store<true>(acc, b2, h2j, MDP_RLH);
        }
        wave_sync();
        {
          const f32x4 acc = rh_acc(h2j, MDP_RLH, w3);
          if (r < MDP_ACT_DIM) {
#pragma unroll
            for (int i = 0; i < 4; ++i) lgj[(kq * 4 + i) * 8 + r] = acc[i] + b3;
          }
        }
        wave_sync();
        if (lane < MDP_R) gumbel_softmax5(lgj + lane * 8, u, rowt + lane * ldr + aj.act_off);
      }
      __syncthreads();
      MDP_STAMP(42);
    }
  }
  for (int j = 0; j < (par ? 0 : n); ++j) {
    const ADesc& aj = T.ag[j];
    if (!a.act_in) {
      bool pf = false;
      // (H = 64 only: at H = 128 the fragments take the kernel to 256 VGPRs, one
      // workgroup per CU, for 0.3 of the 6 us per agent)
      if constexpr (H == 64 && MDP_NW == 4) {
        if (aj.obs_dim <= 4 * MDP_KC) {
          mlp_fwd_tile_pf<H>(rowt + aj.obs_off, ldr, aj.obs_dim, a.theta, aj.actor, h1, h2, ldh, lg, 8);
          pf = true;
        }
      }
      if (!pf) mlp_fwd_tile<H>(rowt + aj.obs_off, ldr, aj.obs_dim, a.theta, aj.actor, h1, h2, ldh, lg, 8);
    }
    if (tid < MDP_R) {
      float* dst = rowt + tid * ldr + aj.act_off;
      if (a.act_in) {
        for (int k = 0; k < MDP_ACT_DIM; ++k)
          dst[k] = tid < nvalid ? a.act_in[((int64_t)(e0 + tid) * n + j) * MDP_ACT_DIM + k] : 0.f;
      } else {
        float u[MDP_ACT_DIM];
        if (a.u_in) {
          for (int k = 0; k < MDP_ACT_DIM; ++k)
            u[k] = tid < nvalid ? a.u_in[((int64_t)(e0 + tid) * n + j) * MDP_ACT_DIM + k] : 0.5f;
        } else {
          uniforms5(a.seed, 0x10000u | (uint32_t)j, step_s(), (uint32_t)(a.env_base + e0 + tid), u);
        }
        gumbel_softmax5(lg + tid * 8, u, dst);
      }
    }
    __syncthreads();
    if (j < 4) MDP_STAMP(42 + j);
  }

  // physics (one thread per (env, entity)), then rewards and bookkeeping (one
  // thread per env, wave 0) beside the next observations (one thread per
  // (env, agent), the other waves); terminal envs reset after both
  env_physics_tile(E, sp, sv, rowt + T.ag[0].act_off, ldr, sfo, nvalid);
  bool term = false;
  if (tid < nvalid) {
    const float* p = sp + tid * 2 * MDP_MAX_ENT;
    float* row = rowt + tid * ldr;
    // the row's rewards rew_0 .. rew_{n-1} are contiguous (mdp_topo.h): written
    // in place, not through a private array (scratch memory)
    float* rew = row + T.ag[0].rew_off;
    env_reward(E, p, goal, rew);
    if (a.bench) env_bench(E, p, goal, a.bench + (int64_t)(e0 + tid) * n * MDP_BENCH_W);
    for (int j = 0; j < n; ++j) row[T.ag[j].done_off] = 0.f;  // done_callback is None (environment.py _get_done)
    const int e = e0 + tid;
    float tot = 0.f;
    for (int j = 0; j < n; ++j) {
      const float r = epr[tid * MDP_MAX_AGENTS + j] + rew[j];
      epr[tid * MDP_MAX_AGENTS + j] = r;
      a.ep_rew[(int64_t)e * n + j] = r;
      tot += r;
    }
    const int st = (int)ctr_use((uint32_t)ep_st) + 1;
    term = st >= E.max_ep_len;
    if (term) {  // terminal -> log episode, env.reset() (train.py:127-133)
      const uint32_t q = atomicAdd(&a.ctl->ep_pending, 1u);
      const int64_t slot = ep_base_raw + (a.eplog_by_env ? (int64_t)(ep_done + e) : (int64_t)q);
      float* lgp = a.eplog + (slot % a.eplog_cap) * (1 + n);
      lgp[0] = tot;
      for (int j = 0; j < n; ++j) {
        lgp[1 + j] = epr[tid * MDP_MAX_AGENTS + j];
        a.ep_rew[(int64_t)e * n + j] = 0.f;
        if (MULTI) epr[tid * MDP_MAX_AGENTS + j] = 0.f;
      }
      if (MULTI) {
        atomicAdd(&s_nterm, 1);
        ep_st = 0;
      }
    } else {
      a.ep_step[e] = st;
      if (MULTI) ep_st = st;
    }
  } else if (tid >= 64 && tid - 64 < nvalid * n) {
    const int q = tid - 64, r = q / n, j = q - r * n;
    env_obs(E, sp + r * 2 * MDP_MAX_ENT, sv + r * 2 * MDP_MAX_ENT, sgoal[r], j, rowt + r * ldr + T.ag[j].nobs_off);
  }
  static_assert(64 + MDP_R * MDP_MAX_AGENTS <= MDP_NT, "rollout obs': one pass on waves 1..");
  __syncthreads();
  if (MULTI) ep_done += s_nterm;
  if (term) {
    const int e = e0 + tid;
    int32_t g;
    env_reset_one(E, a.seed, 0x20000u, step_s(), (uint32_t)(a.env_base + e), sp + tid * 2 * MDP_MAX_ENT,
                  sv + tid * 2 * MDP_MAX_ENT, &g);
    a.goal[e] = g;
    a.ep_step[e] = 0;
    if (MULTI) {
      goal = g;
      sgoal[tid] = g;
    }
  }
  __syncthreads();
  MDP_STAMP(46);
  // replay append of the 16 rows + env state store
  const int v4 = T.row_stride >> 2;
  for (int q = tid; q < nvalid * v4; q += MDP_NT) {
    const int r = q / v4, c4 = q - r * v4;
    const float* s = rowt + r * ldr + c4 * 4;
    const int64_t dst = (next_s + e0 + r) % a.cap;
    *reinterpret_cast<float4*>(a.replay + dst * T.row_stride + c4 * 4) = make_float4(s[0], s[1], s[2], s[3]);
  }
  }  // steps of the launch
  for (int q = tid; q < nvalid * 2 * ne; q += MDP_NT) {
    const int r = q / (2 * ne), c = q - r * 2 * ne;
    a.pos[(int64_t)(e0 + r) * 2 * ne + c] = sp[r * 2 * MDP_MAX_ENT + c];
    a.vel[(int64_t)(e0 + r) * 2 * ne + c] = sv[r * 2 * MDP_MAX_ENT + c];
  }
  MDP_STAMP(47);
  rollout_finish(a, next_raw, len_raw);
}

// batched policy / critic evaluation for the facade (action, target_act, q_values)
template <int H>
__global__ __launch_bounds__(MDP_NT) void k_mlp_eval(EvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ldx = lds_ld(a.in), ldh = H + 1;
  LdsCarve cv(lds);
  float* x = cv.take(MDP_R * ldx);
  float* h1 = cv.take(MDP_R * ldh);
  float* h2 = cv.take(MDP_R * ldh);
  float* lg = cv.take(MDP_R * 8);
  const int r0 = blockIdx.x * MDP_R;
  const int nvalid = min(MDP_R, a.rows - r0);
  for (int q = threadIdx.x; q < MDP_R * a.in; q += MDP_NT) {
    const int r = q / a.in, c = q - r * a.in;
    x[r * ldx + c] = r < nvalid ? a.x[(int64_t)(r0 + r) * a.in + c] : 0.f;
  }
  __syncthreads();
  mlp_fwd_tile<H>(x, ldx, a.in, a.P, a.net, h1, h2, ldh, lg, 8);
  const int tid = threadIdx.x;
  if (tid < nvalid) {
    const int row = r0 + tid;
    if (a.gumbel) {
      float u[MDP_ACT_DIM], act[MDP_ACT_DIM];
      if (a.u) {
        for (int k = 0; k < MDP_ACT_DIM; ++k) u[k] = a.u[(int64_t)row * MDP_ACT_DIM + k];
      } else {
        uniforms5(a.seed, a.stream, a.ctr, (uint32_t)row, u);
      }
      gumbel_softmax5(lg + tid * 8, u, act);
      for (int k = 0; k < MDP_ACT_DIM; ++k) a.out[(int64_t)row * MDP_ACT_DIM + k] = act[k];
    } else {
      for (int k = 0; k < a.net.out; ++k) a.out[(int64_t)row * a.net.out + k] = lg[tid * 8 + k];
    }
  }
}

// ================================================================ launchers
#define MDP_CHECK_LAUNCH() \
  do {                     \
    hipError_t e_ = hipGetLastError(); \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

template <int H>
static hipError_t launch_rollout_t(const RolloutArgs& a, int lds_bytes, hipStream_t s) {
  const int grid = (a.E + MDP_R - 1) / MDP_R + (a.pf_count > 0 ? 1 : 0);
  if (a.nsteps > 1)
    mdp_launch(k_rollout<H, true>, dim3(grid), dim3(MDP_NT), lds_bytes, s, a);
  else
    mdp_launch(k_rollout<H, false>, dim3(grid), dim3(MDP_NT), lds_bytes, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
template <int H>
static hipError_t launch_eval_t(const EvalArgs& a, int lds_bytes, hipStream_t s) {
  const int grid = (a.rows + MDP_R - 1) / MDP_R;
  hipLaunchKernelGGL(k_mlp_eval<H>, dim3(grid), dim3(MDP_NT), lds_bytes, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}

static int set_lds_limit_done = 0;
template <int H>
static void raise_lds_limits() {
  (void)hipFuncSetAttribute((const void*)k_rollout<H, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
  (void)hipFuncSetAttribute((const void*)k_rollout<H, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
  (void)hipFuncSetAttribute((const void*)k_mlp_eval<H>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
}
static void ensure_lds_limits() {
  if (!set_lds_limit_done) {
    raise_lds_limits<64>();
    raise_lds_limits<128>();
    raise_lds_limits<256>();
    (void)hipGetLastError();  // an unsupported opt-in must not poison the next launch check
    set_lds_limit_done = 1;
  }
}

hipError_t mdp_launch_rollout(const RolloutArgs& a, int H, int lds_bytes, hipStream_t s) {
  ensure_lds_limits();
  switch (H) {
    case 64: return launch_rollout_t<64>(a, lds_bytes, s);
    case 128: return launch_rollout_t<128>(a, lds_bytes, s);
    case 256: return launch_rollout_t<256>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}
hipError_t mdp_launch_eval(const EvalArgs& a, int H, int lds_bytes, hipStream_t s) {
  ensure_lds_limits();
  switch (H) {
    case 64: return launch_eval_t<64>(a, lds_bytes, s);
    case 128: return launch_eval_t<128>(a, lds_bytes, s);
    case 256: return launch_eval_t<256>(a, lds_bytes, s);
    default: return hipErrorInvalidValue;
  }
}
hipError_t mdp_launch_apply(const ApplyArgs& a, hipStream_t s) {
  const int grid = a.blk[6] + (a.polyak ? a.oblk[6] : 0) + (a.stats_mode ? 1 : 0);
  mdp_launch(k_apply, dim3(grid), dim3(256), 0, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_reduce(const ReduceArgs& a, hipStream_t s) {
  const int grid = (int)((a.size * 8 + 255) / 256);
  mdp_launch(k_reduce, dim3(grid), dim3(256), 0, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_make_index(Ctl* ctl, int count, int32_t* out, hipStream_t s) {
  mdp_launch(k_make_index, dim3(1), dim3(1024), 0, s, ctl, count, out);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
// Polyak of every target net in one pass (throughput mode: after the round's
// last optimizer step, so no gradient of the round reads a stepped target)
__global__ __launch_bounds__(256) void k_polyak(float* __restrict__ target, const float* __restrict__ theta,
                                                int64_t n4, float pa, float pb, const Ctl* ctl) {
  if (__hip_atomic_load(&ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 tg = reinterpret_cast<const f32x4*>(target)[i];
    const f32x4 th = reinterpret_cast<const f32x4*>(theta)[i];
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pa * tg[j] + pb * th[j];  // the fused kernels' expression
    reinterpret_cast<f32x4*>(target)[i] = o;
  }
}
hipError_t mdp_launch_polyak(float* target, const float* theta, int64_t n, float pa, float pb, const Ctl* ctl,
                             hipStream_t s) {
  const int64_t n4 = n / 4;
  const int grid = (int)std::min<int64_t>(1024, (n4 + 255) / 256);
  mdp_launch(k_polyak, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, target, theta, n4, pa, pb, ctl);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_gather(const float* replay, int stride, const int32_t* idx, int count, float* out,
                             hipStream_t s) {
  const int v4 = stride >> 2;
  const int per = (int)((((int64_t)1 << 31) - 1) / v4);  // rows per launch: elements < 2^31
  for (int b0 = 0; b0 < count; b0 += per) {
    const int n = count - b0 < per ? count - b0 : per;
    const int64_t total = (int64_t)n * v4;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_gather_rows, dim3(grid), dim3(256), 0, s, replay, stride, idx + b0, n,
                       out + (int64_t)b0 * stride);
    MDP_CHECK_LAUNCH();
  }
  return hipSuccess;
}
hipError_t mdp_launch_count_nonfinite(const float* p, int64_t n, uint32_t* cnt, hipStream_t s) {
  int grid = (int)((n + 255) / 256);
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_count_nonfinite, dim3(grid), dim3(256), 0, s, p, n, cnt);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_put_rows(float* replay, int stride, int64_t cap, int64_t next, const float* src, int64_t rows,
                               hipStream_t s) {
  const int64_t total = rows * (stride >> 2);
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_put_rows, dim3(grid), dim3(256), 0, s, replay, stride, cap, next, src, rows);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_put_agent(float* replay, int stride, const ADesc& ag, const int64_t* pos, const float* cols,
                                int64_t rows, hipStream_t s) {
  const int64_t total = rows * (2 * ag.obs_dim + MDP_ACT_DIM + 2);
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_put_agent, dim3(grid), dim3(256), 0, s, replay, stride, ag.obs_off, ag.act_off, ag.nobs_off,
                     ag.rew_off, ag.done_off, ag.obs_dim, pos, cols, rows);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_env_reset(const EnvResetArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_env_reset, dim3((a.E + 255) / 256), dim3(256), 0, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}
hipError_t mdp_launch_env_obs(const EnvObsArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_env_obs, dim3((a.E + 255) / 256), dim3(256), 0, s, a);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}

// ring head / length written in stream order (facade adds and resets)
__global__ void k_set_ring(Ctl* ctl, int64_t len, int64_t next) {
  ctl->len = len;
  ctl->next = next;
}
hipError_t mdp_launch_set_ring(Ctl* ctl, int64_t len, int64_t next, hipStream_t s) {
  hipLaunchKernelGGL(k_set_ring, dim3(1), dim3(1), 0, s, ctl, len, next);
  MDP_CHECK_LAUNCH();
  return hipSuccess;
}

#ifdef MDP_TIMELINE
// diagnostic build: the last rollout's per-workgroup start / end (tools/step_boundary.py)
extern "C" int mdp_debug_tl_roll(unsigned long long* out, int reset) {
  const size_t n = sizeof(unsigned long long) * MDP_TL_WG * 2;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_mdp_tl_roll)) != hipSuccess) return -1;
    return hipMemset(p, 0, n) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_tl_roll), n) == hipSuccess ? 0 : -1;
}
#endif

#ifdef MDP_STAMPS
// diagnostic build: stamps of this translation unit's kernels (k_rollout: 40..47)
extern "C" int mdp_debug_stamps_k(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif
