// mdp_kernels.h -- kernel argument blocks and host-side launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "mdp_topo.h"

// Argument blocks: the scalars and pointers a kernel reads first come first and
// the (1.7 KB) Topo last, so a kernel's opening kernarg reads share a few 64-B
// scalar-cache lines (its early branches otherwise chained one miss each).
struct CriticArgs {
  int agent, B;
  const float* theta;
  const float* target;
  const float* replay;
  const int32_t* idx;
  const float* u_tgt;   // [n][B][5] or null
  uint64_t seed;
  const Ctl* ctl;
  double gamma;
  float inv_b;
  float* slab;          // [nwg][slab_stride] partial critic grads (net-relative)
  int slab_stride;
  double* slab_stat;    // [nwg][8]
  double* y_out;        // [B]
  int group;            // target actors run concurrently per pass (LDS budget)
  // k_critic_grad_r only: one extra workgroup draws the NEXT round's indices
  // (pf_count draws into pf_out) while this kernel runs (0: none)
  Ctl* pf_ctl;
  int32_t* pf_out;
  int pf_count;
  // throughput mode (fast kernels): `multi` agents in one launch, agent =
  // workgroup / (B/16); idx, u_tgt, slab, slab_stat, y_out are then bases with
  // per-agent strides and the noise counter is upd_ctr + agent
  int multi;
  int64_t slab_agent_stride;
  // k_critic_grad_r only: B/16 extra workgroups run the SAME agent's actor
  // forward + policy sample of the coming actor step (it needs only the actor
  // weights, which the critic step does not touch) into apre [B][MDP_APRE_W];
  // u_act: injected uniforms of that sample or null (0: no extra workgroups)
  float* apre;
  float* apre_rows;     // the replay rows it gathered, [B][row_stride] (the actor step reads them contiguously)
  const float* u_act;
  // critic_post mode (k_critic_grad_r): the work of this critic step that does
  // not depend on the previous agent's update (target actors j != cpre_prev,
  // the critic forward, the target critic's layer-1 accumulator over obs' and
  // those target actions) was done by extra workgroups of that agent's actor
  // launch into cpre [B][MDP_CPRE_W]; only target actor cpre_prev (Polyak-
  // updated since) and the rest of the step remain (null: the full step)
  const float* cpre;
  const float* cpre_rows;  // the replay rows the critic_pre gathered, [B][row_stride]
  int cpre_prev;
  Topo topo;
};

// precomputed critic-step work of one batch row (k_actor_grad_r's extra
// workgroups -> k_critic_grad_r in critic_post mode):
//   h1 [64] | h2 [64] (critic forward) | target-critic L1 accumulator [64] | q | pad 3 | a~ [16]
// The accumulator stops at the first MFMA k-step holding a target action of
// the previous agent; critic_post resumes the chain there with every a~ (the
// stored ones + the fresh one), so the result is bit-identical to the
// unsplit critic step
#define MDP_CPRE_W 212

// precomputed actor forward of one batch row (k_critic_grad_r's extra
// workgroups -> k_actor_grad_r): h1 [64] | h2 [64] | logits [8] | sample [8]
#define MDP_APRE_W 144

// (the fields without the Topo: the gradient-pair launch passes ONE Topo for both steps)
struct ActorArgsHead {
  int agent, B;
  const float* theta;
  const float* replay;
  const int32_t* idx;
  const float* u_act;   // [B][5] or null
  uint64_t seed;
  const Ctl* ctl;
  float neg_inv_b;      // dL/dq = -1/B
  float reg_scale;      // 2 * actor_reg / (B * 5)
  float* slab;
  int slab_stride;
  double* slab_stat;
  int multi;                  // throughput mode, as CriticArgs
  int64_t slab_agent_stride;
  const float* apre;          // k_actor_grad_r: the forward precomputed by the critic launch, or null
  const float* apre_rows;     // ... and its replay rows [B][row_stride] (read instead of a gather)
  // k_actor_grad_r: B/16 extra workgroups run the NEXT critic step's
  // independent work (agent cpre_agent, indices cpre_idx) into cpre (null: none)
  float* cpre;
  float* cpre_rows;
  int cpre_agent;
  const int32_t* cpre_idx;
  const float* target;        // target nets (the critic_pre role's target actors / critic)
};
struct ActorArgs : ActorArgsHead {
  Topo topo;
};

// throughput mode on the general kernels: agent i's critic step and actor step
// (independent there: both read the round-start parameters) as ONE launch --
// workgroups [0, B/16) the critic step, [B/16, 2 B/16) the actor step
struct GradPairArgs {
  CriticArgs c;
  ActorArgsHead x;
};

struct ReduceArgs {
  const float* slab;
  int nwg, slab_stride;
  float* grad;
  int64_t off, size;
  float* beta;          // [4] of this optimizer: next powers (TF variables), this step's powers
  float b1, b2;
  Ctl* ctl;
  int bump_ctr;         // actor phase: advance the training-noise counter
};

#define MDP_APPLY_CHUNK 1024  // parameters per apply workgroup

struct ApplyArgs {
  int blk[7], oblk[7];  // prefix counts of chunk workgroups per tensor (net / other)
  float* theta;
  float* target;
  float* m;
  float* v;
  float* grad;
  const float* slab;    // null: read grad[] (already reduced / all-reduced)
  int slab_stride, nwg;
  float scale, clip, lr, b1, b2, eps;
  float* beta;          // [2] beta1^t, beta2^t of this optimizer
  int polyak;
  float pa, pb;         // fp32(1 - tau), fp32(1 - (1 - tau))
  int stats_mode;       // 0 none, 1 critic, 2 actor
  const double* slab_stat;
  const double* y;
  int B;
  float reg;
  double* stats_out;
  uint32_t* ticket;
  Ctl* ctl;
  int bump_ctr;         // the last workgroup advances Ctl::upd_ctr by this much
  NDesc net, other;
};

// k_reduce_apply (mdp_apply_fused.hip): batch reduction + optimizer step in one launch
#define MDP_RA_CHUNK 256   // parameters per workgroup
#define MDP_RA_MAXCH 256   // chunks per tensor the sync area holds
// Direct xGMI gradient exchange of the data-parallel step (phase 3 below):
// every rank owns one exchange buffer (uncached device memory, IPC-exported)
// of 64-bit words laid out as
//   [2 slots][world][PT + MDP_XCH_PROBE]   word = epoch << 32 | fp32 bits
// (slot = exchange epoch & 1; the last MDP_XCH_PROBE words of a row belong
// to the connection probe) and holds every peer's buffer mapped
// (hipIpcOpenMemHandle).  Rank r stores each value of its reduced chunk, tagged
// with the epoch, into row [slot][r] of every peer with ONE 64-bit
// system-scope store; the receiver polls each word of its peers' rows until
// the tag equals the epoch (data and flag arrive together: no fences, no
// separate flag round trip -- the LL protocol) and sums the world's values in
// rank order, so every rank computes the identical sum and replicas stay
// bit-equal.  Epoch 0 never occurs (the buffer starts zeroed).
#define MDP_XCH_MAXW 8
#define MDP_XCH_PROBE 2048   // probe words per row (8 chunks)
struct XchgDesc {
  int world, rank;
  int64_t pt;                        // words per row: param-space length + MDP_XCH_PROBE
  uint64_t* data[MDP_XCH_MAXW];      // rank q's exchange buffer in this process (data[rank] local)
};
inline int64_t mdp_xch_bytes(int world, int64_t param_floats) {
  return 8 * (2 * (int64_t)world * (param_floats + MDP_XCH_PROBE));
}

struct FusedApplyArgs {
  int pf_count;         // (below)
  int phase;            // 0 reduce + step; 1 reduce into grad[] only; 2 step from grad[] (all-reduced);
                        // 3 reduce, xGMI exchange with every rank (xd), step x ap.scale
  int rblk[7];          // prefix counts of MDP_RA_CHUNK workgroups per tensor of ap.net
  uint32_t* sync_ctr;   // 6 tensor counters of this (agent, net), 32 words apart
  uint64_t* sync_part;  // [6][MDP_RA_MAXCH][2] published sums of squares (epoch-tagged halves)
  uint32_t* done_ctr;   // workgroups finished (last one advances beta)
  const XchgDesc* xd;   // phase 3: device copy of the exchange descriptor
  int net_id;           // phase 3: 2 * agent + net (epoch counter)
  uint32_t* xstep;      // phase 3: Ctl::xstep[net_id], exchanges done for this net
  uint64_t* wstat;      // phase 3: Ctl::xw_ticks when the exchange waits are stamped, else null
  // pf_count > 0: one extra (last) workgroup draws pf_count indices of the NEXT
  // round into pf_out, continuing the MT19937 stream (a piece of the draw the
  // fast kernels make beside the critic step; general-kernel configurations)
  int32_t* pf_out;
  Ctl* pf_ctl;
  ApplyArgs ap;         // ap.slab / nwg / slab_stride: the partial gradients
};
// sync area: per (agent, net) 8 counters x 128 B (6 done, 7 norm epoch), then [6][MAXCH][2] tagged words
inline int64_t mdp_ra_sync_bytes() {
  return (int64_t)MDP_MAX_AGENTS * 2 * 8 * 128 + (int64_t)MDP_MAX_AGENTS * 2 * 6 * MDP_RA_MAXCH * 16;
}

struct RolloutArgs {
  Topo topo;
  EnvDesc env;
  const float* theta;
  float* replay;
  int64_t cap;
  float* pos;
  float* vel;
  int32_t* goal;
  int32_t* ep_step;
  float* ep_rew;
  float* eplog;
  int64_t eplog_cap;
  // env copies in lockstep (all terminate on the same step): episode e of a
  // step is logged at slot episodes + e -- env order, deterministic; otherwise
  // in arrival order
  int eplog_by_env;
  Ctl* ctl;
  uint64_t seed;
  int E, env_base;
  const float* act_in;
  const float* u_in;
  uint32_t* ticket;
  float* bench;  // benchmark_data records [E][n][MDP_BENCH_W] or null
  // > 0: one extra workgroup draws the step's first-round indices (pf_count
  // randint draws against the ring length after this step) beside the envs
  int pf_count;
  int32_t* pf_out;
  // consecutive env steps in this launch (1; > 1 only with one env workgroup,
  // no draw, no bench records and the policies' own actions)
  int nsteps;
};

struct EnvResetArgs {
  EnvDesc env;
  uint64_t seed;
  uint32_t ctr;
  int env_base, E;
  float* pos;
  float* vel;
  int32_t* goal;
  int32_t* ep_step;
  float* ep_rew;
};

struct EnvObsArgs {
  Topo topo;
  EnvDesc env;
  int E;
  const float* pos;
  const float* vel;
  const int32_t* goal;
  float* obs;
};

struct EvalArgs {
  const float* P;
  NDesc net;
  int in, rows;
  const float* x;
  float* out;
  int gumbel;
  const float* u;
  uint64_t seed;
  uint32_t stream, ctr;
};

// kernel width that serves --num-units u: the gradient / rollout / eval kernels
// are instantiated for H = 64, 128, 256 (the fast register-resident ones for 64)
inline int mdp_device_units(int u) { return u <= 64 ? 64 : (u <= 128 ? 128 : 256); }

// ---- dynamic LDS sizes (must mirror the LdsCarve order in the kernels)
inline int mdp_r4(int n) { return (n + 3) & ~3; }
inline int mdp_ld(int c) { return c | 1; }
// k_critic_grad / k_actor_grad (mdp_grads.hip); FJob/HJob are 48-byte LDS job records
inline int lds_critic_bytes(const Topo& t, int G) {
  const int R = 16, ldr = mdp_ld(t.row_stride), ldc = mdp_ld(t.cin_max), S = R * (t.H + 1);
  return 4 * (mdp_r4(R * ldr) + 2 * mdp_r4(R * ldc) + 2 * mdp_r4((G + 1) * S) + mdp_r4((G + 1) * R * 8) +
              mdp_r4(R) + mdp_r4(MDP_MAX_AGENTS + 4));
}
inline int lds_actor_bytes(const Topo& t) {
  const int R = 16, ldr = mdp_ld(t.row_stride), ldc = mdp_ld(t.cin_max), S = R * (t.H + 1);
  return 4 * (mdp_r4(R * ldr) + mdp_r4(R * ldc) + 6 * mdp_r4(S) + 5 * mdp_r4(R * 8) + mdp_r4(5 * t.H));
}
#define MDP_LDS_BUDGET (160 * 1024)
// fast (register-resident, H = 64) variants in mdp_grads_r.hip
inline int lds_critic_r_bytes(const Topo& t, int agent) {
  const int R = 16, ldr = mdp_ld(t.row_stride), LH = 68, LD = 65;
  const int na = t.ag[agent].local_q ? 1 : t.n, ldA = mdp_ld(5 * na);
  return 4 * (mdp_r4(R * ldr) + mdp_r4(R * ldA) + 3 * R * 8 + 6 * R * LH + 4 * R * LH + 3 * R + 2 * mdp_r4(R * LD));
}
inline int lds_actor_r_bytes(const Topo& t) {
  const int R = 16, ldr = mdp_ld(t.row_stride), LH = 68, LD = 65;
  return 4 * (mdp_r4(R * ldr) + 4 * R * 8 + R + 3 * R * LH + 4 * mdp_r4(R * LD) + 2 * 64 * 16 + 4 * R + 4 * 5 * 64);
}
// critic_pre role of k_actor_grad_r (mirrors critic_pre_tile's carve)
inline int lds_critic_pre_bytes(const Topo& t) {
  const int R = 16, ldr = mdp_ld(t.row_stride), LH = 68, ldA = mdp_ld(5 * t.n);
  return 4 * (mdp_r4(R * ldr) + mdp_r4(R * ldA) + 3 * R * 8 + 6 * R * LH + 3 * R * LH + 4 * R + 16 * R);
}
// the fast kernels hold every weight of a wave in registers: H = 64, at most 3
// target actors, actor inputs <= 64, critic inputs <= 80, target-critic action part <= 20
inline bool grads_r_ok(const Topo& t, int agent) {
  if (t.H != 64) return false;
  const ADesc& ag = t.ag[agent];
  const int na = ag.local_q ? 1 : t.n;
  if (na > 3) return false;
  for (int j = 0; j < t.n; ++j)
    if (t.ag[j].obs_dim > 64) return false;
  if (ag.cin > 80) return false;
  if ((ag.local_q ? ag.obs_dim : t.sum_obs) > 64) return false;
  return 5 * na <= 20;
}
inline int lds_rollout_bytes(const Topo& t) {
  const int R = 16, ldr = mdp_ld(t.row_stride), ldh = t.H + 1;
  const int par = t.H == 64 ? 4 * (2 * R * 68 + R * 8) : 0;  // k_rollout's per-agent forward slots (H = 64)
  return 4 * (mdp_r4(R * ldr) + 2 * mdp_r4(R * ldh) + mdp_r4(R * 8) + par + 2 * mdp_r4(R * 2 * MDP_MAX_ENT) +
              mdp_r4(R * 3 * MDP_MAX_ENT) + mdp_r4(R * MDP_MAX_AGENTS) + mdp_r4(R));
}
inline int lds_eval_bytes(int in, int H) {
  const int R = 16, ldx = mdp_ld(in), ldh = H + 1;
  return 4 * (mdp_r4(R * ldx) + 2 * mdp_r4(R * ldh) + mdp_r4(R * 8));
}

// ---- per-launch timing (bench.py's kernel pass): when the host armed a
// start/stop event pair for the next launch, that launch carries them on its
// own dispatch packet (hipExtLaunchKernel), so their elapsed time is the
// packet's begin -> end -- the interval rocprofv3 --kernel-trace reports --
// with no marker packets of their own in between
struct MdpLaunchEv {
  hipEvent_t start = nullptr, stop = nullptr;
};
MdpLaunchEv& mdp_launch_ev();  // this host thread's armed pair (mdp_api.cpp)
template <typename F, typename... Args>
inline void mdp_launch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t s, Args... args) {
  MdpLaunchEv& e = mdp_launch_ev();
  if (e.start) {
    const hipEvent_t a = e.start, z = e.stop;
    e.start = e.stop = nullptr;
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, a, z, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
  }
}

hipError_t mdp_launch_critic_grad(const CriticArgs& a, int H, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_actor_grad(const ActorArgs& a, int H, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_grad_pair(const GradPairArgs& a, int H, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_critic_grad_r(const CriticArgs& a, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_actor_grad_r(const ActorArgs& a, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_rollout(const RolloutArgs& a, int H, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_eval(const EvalArgs& a, int H, int lds_bytes, hipStream_t s);
hipError_t mdp_launch_apply(const ApplyArgs& a, hipStream_t s);
hipError_t mdp_launch_reduce(const ReduceArgs& a, hipStream_t s);
hipError_t mdp_launch_reduce_apply(const FusedApplyArgs& f, hipStream_t s);
// throughput mode: the optimizer steps of `count` nets in one launch; list[]
// lives in device memory (written once), wg_start[q] = first workgroup of net q
#define MDP_RA_BATCH_MAX (2 * MDP_MAX_AGENTS)
struct RaBatch {
  const FusedApplyArgs* list = nullptr;
  int count = 0;
  int narrow = 0;       // fan-in <= 64 partials: 256-thread workgroups (mdp_ra_narrow)
  int wg_start[MDP_RA_BATCH_MAX + 1] = {};
  // pf_count > 0: one extra (last) workgroup draws pf_count indices of the next
  // round into pf_out, continuing the MT19937 stream in pf_ctl (as FusedApplyArgs)
  int pf_count = 0;
  int32_t* pf_out = nullptr;
  Ctl* pf_ctl = nullptr;
};
int mdp_ra_grid(const FusedApplyArgs& f);
hipError_t mdp_ra_occupancy(int* per_cu);   // co-resident k_reduce_apply workgroups per CU
hipError_t mdp_spin_kernels_scratch(int* bytes);  // largest scratch per lane of the spinning kernels
// grid of the fused optimizer launch of (agent, net): the 256-parameter chunks
// of the net, for the actor step the Polyak workgroups of the critic, one stats
// workgroup (mirrors fused_args_for / apply_args / mdp_ra_grid)
inline int mdp_ra_grid_of(const Topo& t, int agent, int net) {
  const NDesc& d = net ? t.ag[agent].critic : t.ag[agent].actor;
  const NDesc& o = net ? t.ag[agent].actor : t.ag[agent].critic;
  int g = 2;  // + the stats workgroup and a slot for an index-draw workgroup
  for (int k = 0; k < 6; ++k) {
    g += (d.t[k].rows * d.t[k].cols + MDP_RA_CHUNK - 1) / MDP_RA_CHUNK;
    if (!net) g += (o.t[k].rows * o.t[k].cols + MDP_APPLY_CHUNK - 1) / MDP_APPLY_CHUNK;
  }
  return g;
}
// the fused launch is safe: every tensor's chunks fit the sync area and the
// whole grid is co-resident on `capacity` workgroup slots
inline bool mdp_ra_fits(const Topo& t, int agent, int net, int capacity) {
  const NDesc& d = net ? t.ag[agent].critic : t.ag[agent].actor;
  for (int k = 0; k < 6; ++k)
    if ((d.t[k].rows * d.t[k].cols + MDP_RA_CHUNK - 1) / MDP_RA_CHUNK > MDP_RA_MAXCH) return false;
  return mdp_ra_grid_of(t, agent, net) <= capacity;
}
hipError_t mdp_launch_reduce_apply_batch(const RaBatch& b, hipStream_t s);
hipError_t mdp_ra_batch_occupancy(int* per_cu);
// connection probe of the xGMI exchange: nchunk chunks of a rank-tagged
// pattern through the same exchange code, *bad += mismatching parameters,
// *fault = 2 when a peer's flag did not arrive in time
hipError_t mdp_launch_xchg_probe(const XchgDesc* xd, uint32_t ep, int nchunk, uint32_t* bad, uint32_t* fault,
                                 hipStream_t s);
hipError_t mdp_launch_make_index(Ctl* ctl, int count, int32_t* out, hipStream_t s);
// target <- pa target + pb theta over n floats (make_update_exp, maddpg.py:20-26),
// skipped once Ctl::fault is set; n a multiple of 4
hipError_t mdp_launch_polyak(float* target, const float* theta, int64_t n, float pa, float pb, const Ctl* ctl,
                             hipStream_t s);
hipError_t mdp_launch_gather(const float* replay, int stride, const int32_t* idx, int count, float* out,
                             hipStream_t s);
hipError_t mdp_launch_count_nonfinite(const float* p, int64_t n, uint32_t* cnt, hipStream_t s);
hipError_t mdp_launch_put_rows(float* replay, int stride, int64_t cap, int64_t next, const float* src, int64_t rows,
                               hipStream_t s);
hipError_t mdp_launch_put_agent(float* replay, int stride, const ADesc& ag, const int64_t* pos, const float* cols,
                                int64_t rows, hipStream_t s);
hipError_t mdp_launch_env_reset(const EnvResetArgs& a, hipStream_t s);
hipError_t mdp_launch_env_obs(const EnvObsArgs& a, hipStream_t s);
hipError_t mdp_launch_set_ring(Ctl* ctl, int64_t len, int64_t next, hipStream_t s);
