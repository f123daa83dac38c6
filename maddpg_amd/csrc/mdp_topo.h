// mdp_topo.h -- problem topology shared by host launch code and kernels.
//
// Param space (one region each for theta, target, Adam m, Adam v, grad):
//   [agent 0: actor | critic][agent 1: actor | critic] ...
// each net = W1[in][H] b1[H] W2[H][H] b2[H] W3[H][out] b3[out]
// (experiments/train.py:43-45, TF fully_connected stores W as [in, out]),
// every tensor padded to a multiple of 4 floats (16-B aligned).
//
// Joint replay row (one row per transition, shared by all agents, because the
// reference draws ONE index set and gathers it from every agent's buffer,
// maddpg.py:167-178):
//   [obs_0 .. obs_{N-1} | act_0 .. act_{N-1} | obs'_0 .. obs'_{N-1} | rew_0..rew_{N-1} | done_0..done_{N-1} | pad]
// so the MADDPG critic input concat(obs_n + act_n) (maddpg.py:85) is the row's
// contiguous prefix.
#pragma once
#include <stdint.h>

#include "../../include/maddpg_hip.h"

#define MDP_MAX_ENT 16

struct TDesc {
  int off, rows, cols;
};
struct NDesc {
  TDesc t[6];  // W1 b1 W2 b2 W3 b3
  int off, size, in, out;
};
struct ADesc {
  NDesc actor, critic;
  int obs_dim, obs_off, act_off, nobs_off, rew_off, done_off;
  int local_q, cin, a_in_off;  // critic input width; offset of a_i inside it
};
struct Topo {
  int n, H, row_stride, sum_obs, cin_max, obs_max;
  ADesc ag[MDP_MAX_AGENTS];
};

// MPE entity table for the device env (multiagent/core.py Entity/Agent fields)
struct EnvDesc {
  int scenario, n_agents, n_landmarks, n_adv, max_ep_len;
  float size[MDP_MAX_ENT];
  float accel[MDP_MAX_AGENTS];       // sensitivity (5.0 when agent.accel is None)
  float max_speed[MDP_MAX_ENT];      // <0: None
  int collide[MDP_MAX_ENT];
  int movable[MDP_MAX_ENT];
  int adversary[MDP_MAX_AGENTS];
};

// device control block (one per handle, in the arena)
struct Ctl {
  uint32_t mt[624];
  int32_t mt_pos;
  int32_t pad0;
  int64_t len;          // replay rows valid
  int64_t next;         // ring head
  int64_t env_steps;    // vector steps taken (RNG counter for rollouts)
  int64_t episodes;     // finished episodes logged
  uint32_t ticket[8];   // last-workgroup tickets
  uint32_t upd_ctr;     // RNG counter for training noise
  uint32_t fault;       // set by a bounded spin that timed out (1 norm handshake, 2 xGMI exchange)
  uint32_t xstep[16];   // xGMI exchanges completed per net (2 * agent + net): the epoch counter
  uint32_t ep_pending;  // episodes finished in the running rollout (the last workgroup folds it in)
  uint32_t pad1;
  // xGMI exchange diagnostics (mdp_dp_exchange_stats): per chunk workgroup,
  // the s_memrealtime ticks (100 MHz) from its own chunk's stores to the
  // arrival of every peer's chunk -- peer skew + fabric latency
  uint64_t xw_ticks;    // summed over chunk exchanges
  uint64_t xw_count;    // chunk exchanges counted
  uint64_t xw_max;      // the longest single wait
  uint32_t nonfinite;   // mdp_check_finite's count of non-finite parameters / Adam state
  uint32_t pad2;
};
