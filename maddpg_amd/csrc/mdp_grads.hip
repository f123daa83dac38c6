// mdp_grads.hip -- per-agent critic-step and actor-step gradient kernels (gfx950).
//
// One 512-thread workgroup (8 waves) owns 16 batch rows; the reduction over
// the batch happens in k_reduce from per-workgroup partials (deterministic).
//
// Forward passes are WAVE-LOCAL: one wave runs a whole net (L1 -> L2 -> head)
// with its H/16 column tiles' fp32-MFMA chains interleaved (wave_layer in
// mdp_device.h) and only wave-scope LDS ordering between layers, so
// independent nets (every agent's target actor and the critic) run
// concurrently on different waves with no workgroup barrier between their
// layers.  Workgroup barriers remain only where data crosses nets or rows
// meet columns (weight gradients, spread over all waves).
//
// k_critic_grad (maddpg.py:180-188):
//   gather rows | waves: target actor j (+Gumbel a~_j), critic fwd  || barrier
//   | wave 0: target critic -> fp64 TD target, loss, dL/dq             || barrier
//   | dW3, db3, d2                                                     || barrier
//   | wave 0: dh1 ; waves 1..7: dW2 ; db2                              || barrier
//   | dW1, db1
// k_actor_grad (maddpg.py:37-58):
//   gather | wave 0: actor fwd, Gumbel a_i, critic(a_i) fwd, d2, dh1, da_i,
//   softmax backward + reg -> dlogits                                  || barrier
//   | dW3a, db3a, d2a || wave 0: d1a ; waves 1..7: dW2a || dW1a, db1a
#include "mdp_device.h"
#include "mdp_kernels.h"


template <int H>
__global__ __launch_bounds__(512) void k_critic_grad(CriticArgs a) {
  constexpr int NT = H / 16;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Topo& T = a.topo;
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

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  const int r0 = blockIdx.x * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const bool lq = ag.local_q != 0;
  const uint32_t ctr = a.ctl->upd_ctr;
  const NDesc& nd = ag.critic;
  float* h1c = hA + G * S;
  float* h2c = hB + G * S;
  float* qv = lg + G * MDP_R * 8;
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
  __syncthreads();
  const float* Xc = lq ? xl : rowbuf;  // critic input: the row prefix (global) or [obs_i | act_i]
  const int ldX = lq ? ldc : ldr;
  MDP_STAMP(1);

  // one wave per net: target actors of the group (+ the critic forward with the first group)
  const int nact = lq ? 1 : T.n;
  for (int g0 = 0; g0 < nact; g0 += G) {
    const int ng = min(G, nact - g0);
    const int nj = ng + (g0 == 0 ? 1 : 0);
    for (int jb = wave; jb < nj; jb += nw) {
      if (jb < ng) {
        const int j = lq ? a.agent : g0 + jb;
        const ADesc& aj = T.ag[j];
        const float* P = a.target;
        float* h1 = hA + jb * S;
        float* h2 = hB + jb * S;
        float* lgj = lg + jb * MDP_R * 8;
        wave_layer<NT, true>(rowbuf + aj.nobs_off, ldr, aj.obs_dim, P + aj.actor.t[0].off, P + aj.actor.t[1].off, h1,
                             ldh);
        wave_layer<NT, true>(h1, ldh, H, P + aj.actor.t[2].off, P + aj.actor.t[3].off, h2, ldh);
        wave_head(h2, ldh, H, P + aj.actor.t[4].off, P + aj.actor.t[5].off, MDP_ACT_DIM, lgj, 8);
        if (lane < MDP_R) {  // Gumbel-softmax target action (distributions.py:264-266)
          const int row = lane;
          float u[MDP_ACT_DIM], act[MDP_ACT_DIM];
          if (a.u_tgt) {
            for (int k = 0; k < MDP_ACT_DIM; ++k)
              u[k] = row < nvalid ? a.u_tgt[((int64_t)j * a.B + r0 + row) * MDP_ACT_DIM + k] : 0.5f;
          } else {
            uniforms5(a.seed, (uint32_t)((a.agent << 8) | (j + 1)), ctr, (uint32_t)(r0 + row), u);
          }
          gumbel_softmax5(lgj + row * 8, u, act);
          const int dst = lq ? ag.obs_dim : T.sum_obs + MDP_ACT_DIM * j;
          for (int k = 0; k < MDP_ACT_DIM; ++k) xt[row * ldc + dst + k] = act[k];
        }
      } else {
        const float* P = a.theta;
        wave_layer<NT, true>(Xc, ldX, ag.cin, P + nd.t[0].off, P + nd.t[1].off, h1c, ldh);
        wave_layer<NT, true>(h1c, ldh, H, P + nd.t[2].off, P + nd.t[3].off, h2c, ldh);
        wave_head(h2c, ldh, H, P + nd.t[4].off, P + nd.t[5].off, 1, qv, 8);
      }
    }
    __syncthreads();
  }
  MDP_STAMP(2);

  // wave 0: target critic Q'(o', a~), fp64 TD target (maddpg.py:186), loss partials, dL/dq = 2(q-y)/B
  if (wave == 0) {
    const float* P = a.target;
    wave_layer<NT, true>(xt, ldc, ag.cin, P + nd.t[0].off, P + nd.t[1].off, hA, ldh);
    wave_layer<NT, true>(hA, ldh, H, P + nd.t[2].off, P + nd.t[3].off, hB, ldh);
    wave_head(hB, ldh, H, P + nd.t[4].off, P + nd.t[5].off, 1, lg, 8);
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
      double* st = a.slab_stat + (int64_t)blockIdx.x * 8;
      st[0] = s_l;
      st[1] = s_y;
      st[2] = s_r;
      st[3] = s_q;
    }
  }
  __syncthreads();
  MDP_STAMP(3);

  // backward through the critic (tf.gradients of q_loss w.r.t. q_func vars)
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride - nd.off;
  const float* W3 = a.theta + nd.t[4].off;
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
  for (int e = tid; e < MDP_R * H; e += blockDim.x) {
    const int r = e / H, h = e - r * H;
    d2[r * ldh + h] = h2c[r * ldh + h] > 0.f ? dq[r] * W3[h] : 0.f;
  }
  __syncthreads();
  MDP_STAMP(4);
  if (wave == 0) wave_dgrad<NT>(d2, ldh, H, a.theta + nd.t[2].off, h1c, ldh, d1, ldh);
  wgrad_waves(h1c, ldh, H, d2, ldh, H, slab + nd.t[2].off, 1, nw - 1);
  colsum16(d2, ldh, H, slab + nd.t[3].off);
  __syncthreads();
  wgrad_waves(Xc, ldX, ag.cin, d1, ldh, H, slab + nd.t[0].off, 0, nw);
  colsum16(d1, ldh, H, slab + nd.t[1].off);
  MDP_STAMP(5);
}

template <int H>
__global__ __launch_bounds__(512) void k_actor_grad(ActorArgs a) {
  constexpr int NT = H / 16;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Topo& T = a.topo;
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

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  const int r0 = blockIdx.x * MDP_R;
  const int nvalid = min(MDP_R, a.B - r0);
  const bool lq = ag.local_q != 0;
  const uint32_t ctr = a.ctl->upd_ctr;
  const NDesc& na = ag.actor;
  const NDesc& nc = ag.critic;
  const float* P = a.theta;

  gather_rows16(a.replay, T.row_stride, a.idx, r0, nvalid, rowbuf, ldr);
  __syncthreads();
  if (wave == 0) {
    // actor forward on obs_i -> logits p (maddpg.py:39), fresh Gumbel sample (:49)
    wave_layer<NT, true>(rowbuf + ag.obs_off, ldr, ag.obs_dim, P + na.t[0].off, P + na.t[1].off, h1a, ldh);
    wave_layer<NT, true>(h1a, ldh, H, P + na.t[2].off, P + na.t[3].off, h2a, ldh);
    wave_head(h2a, ldh, H, P + na.t[4].off, P + na.t[5].off, MDP_ACT_DIM, lg, 8);
    // critic input with act_input_n[i] = the sample (maddpg.py:48-52)
    const int cin = ag.cin;
    for (int e = lane; e < MDP_R * cin; e += 64) {
      const int r = e / cin, c = e - r * cin;
      const int src = lq ? (c < ag.obs_dim ? ag.obs_off + c : ag.act_off + c - ag.obs_dim) : c;
      x[r * ldc + c] = rowbuf[r * ldr + src];
    }
    wave_sync();
    if (lane < MDP_R) {
      float u[MDP_ACT_DIM];
      if (a.u_act) {
        for (int k = 0; k < MDP_ACT_DIM; ++k)
          u[k] = lane < nvalid ? a.u_act[(int64_t)(r0 + lane) * MDP_ACT_DIM + k] : 0.5f;
      } else {
        uniforms5(a.seed, (uint32_t)((a.agent << 8) | 0x80), ctr, (uint32_t)(r0 + lane), u);
      }
      gumbel_softmax5(lg + lane * 8, u, av + lane * 8);
      for (int k = 0; k < MDP_ACT_DIM; ++k) x[lane * ldc + ag.a_in_off + k] = av[lane * 8 + k];
    }
    wave_sync();
    // critic (post-step weights) forward, q for the loss value
    wave_layer<NT, true>(x, ldc, cin, P + nc.t[0].off, P + nc.t[1].off, h1c, ldh);
    wave_layer<NT, true>(h1c, ldh, H, P + nc.t[2].off, P + nc.t[3].off, h2c, ldh);
    wave_head(h2c, ldh, H, P + nc.t[4].off, P + nc.t[5].off, 1, qv, 8);
    // dL/dq = -1/B ; d2 = dq * W3c masked by h2c > 0 ; dh1 = d2 @ W2c^T masked by h1c > 0
    const float* W3c = P + nc.t[4].off;
    for (int e = lane; e < MDP_R * H; e += 64) {
      const int r = e / H, h = e - r * H;
      d2[r * ldh + h] = (r < nvalid && h2c[r * ldh + h] > 0.f) ? a.neg_inv_b * W3c[h] : 0.f;
    }
    wave_sync();
    wave_dgrad<NT>(d2, ldh, H, P + nc.t[2].off, h1c, ldh, d1, ldh);
    // da[r][k] = sum_h d1[r][h] * W1c[a_in_off + k][h]   (only the a_i input columns)
    {
      const float* W1c = P + nc.t[0].off + (int64_t)ag.a_in_off * H;
      for (int base = 0; base < MDP_R * MDP_ACT_DIM; base += 16) {
        const int o = base + (lane >> 2), q = lane & 3;
        const int r = o / MDP_ACT_DIM, k = o - r * MDP_ACT_DIM;
        float s = 0.f;
        for (int h = q; h < H; h += 4) s = fmaf(d1[r * ldh + h], W1c[k * H + h], s);
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if (q == 0) da[r * 8 + k] = s;
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
      double* st = a.slab_stat + (int64_t)blockIdx.x * 8;
      st[0] = s_q;
      st[1] = s_p;
    }
  }
  __syncthreads();
  // actor backward: dW3a, db3a, d2a = (dl @ W3a^T) masked by h2a > 0
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride - na.off;
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
  if (wave == 0) wave_dgrad<NT>(d2, ldh, H, P + na.t[2].off, h1a, ldh, d1, ldh);
  wgrad_waves(h1a, ldh, H, d2, ldh, H, slab + na.t[2].off, 1, nw - 1);
  colsum16(d2, ldh, H, slab + na.t[3].off);
  __syncthreads();
  wgrad_waves(rowbuf + ag.obs_off, ldr, ag.obs_dim, d1, ldh, H, slab + na.t[0].off, 0, nw);
  colsum16(d1, ldh, H, slab + na.t[1].off);
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
  hipLaunchKernelGGL(k_critic_grad<H>, dim3((a.B + MDP_R - 1) / MDP_R), dim3(512), lds, s, a);
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
  hipLaunchKernelGGL(k_actor_grad<H>, dim3((a.B + MDP_R - 1) / MDP_R), dim3(512), lds, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t mdp_launch_critic_grad(const CriticArgs& a, int H, int lds_bytes, hipStream_t s) {
  return H == 64 ? launch_critic<64>(a, lds_bytes, s) : launch_critic<128>(a, lds_bytes, s);
}
hipError_t mdp_launch_actor_grad(const ActorArgs& a, int H, int lds_bytes, hipStream_t s) {
  return H == 64 ? launch_actor<64>(a, lds_bytes, s) : launch_actor<128>(a, lds_bytes, s);
}

#ifdef MDP_STAMPS
// diagnostic build: stamps of this translation unit's kernels (own code object)
extern "C" int mdp_debug_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif
