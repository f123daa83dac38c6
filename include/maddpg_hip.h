/*
 * maddpg_hip.h -- C ABI of libmaddpg_hip.so, the MI355X-native MADDPG hot path.
 *
 * The reference (adolfogonzalez3/maddpg) is pure Python over TensorFlow 1.x;
 * its "plugin" boundary for this path is the Python surface of
 *   maddpg/__init__.py:1-15               AgentTrainer
 *   maddpg/trainer/maddpg.py:112-196      MADDPGAgentTrainer(action/experience/preupdate/update)
 *   maddpg/trainer/replay_buffer.py:5-85  ReplayBuffer(add/make_index/sample_index/__len__)
 *   experiments/train.py:78-189           the training loop (env step + updates)
 * There is no reference FFI; the binding a maintainer adds is the ctypes stub
 * in maddpg_amd/_lib.py (shown in INTEGRATION.md).  Each entry point below
 * names the reference call it replaces.
 *
 * Conventions
 *  - All compute state lives in ONE device arena the caller allocates (a
 *    PyTorch uint8 CUDA tensor in practice) of mdp_arena_bytes() bytes.  The
 *    library's one device allocation of its own is the direct xGMI exchange
 *    buffer (mdp_dp_xgmi_open: hipExtMallocWithFlags, uncached, IPC-exported,
 *    [2 slots][world][params + probe] 64-bit words; freed by
 *    mdp_dp_xgmi_close / mdp_destroy).
 *  - "_dev" pointers are device pointers on the handle's device; "_host"
 *    pointers are host memory.  Device-pointer calls are asynchronous on the
 *    handle's stream unless stated; host-pointer calls synchronise.  Every
 *    non-NULL "_dev" argument (and mdp_create's arena) is checked at entry
 *    with hipPointerGetAttributes / hipMemGetAddressRange: host memory
 *    (malloc, the stack, pinned hipHostMalloc), another device's memory or an
 *    allocation shorter than the call reads or writes returns < 0 with a
 *    message, before anything is launched.
 *  - Return 0 on success, 1 for "skipped" (update gates), <0 on error; the
 *    message is in mdp_last_error(h).  No C++ exception crosses the ABI.
 *  - One handle per GPU process; calls on one handle are not thread-safe.
 */
#ifndef MADDPG_HIP_H
#define MADDPG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDP_MAX_AGENTS 8
#define MDP_ACT_DIM 5          /* MPE Discrete(dim_p*2+1) action spaces */
#define MDP_MAX_UNITS 256      /* largest --num-units (train.py:24) */
/* Besides these bounds, a configuration must fit the kernels' LDS envelope (a
   16-row tile of every launch in a CU's 160 KB: the sum of obs dims up to
   ~530 / ~470 / ~270 at 64 / 128 / 256 units); mdp_arena_bytes returns -1 and
   mdp_create's handle carries the reason otherwise. */
#define MDP_ABI_VERSION 5

enum mdp_scenario {
    MDP_SCN_NONE = 0,          /* trainer only (no device env) */
    MDP_SCN_SIMPLE = 1,
    MDP_SCN_SPREAD = 2,
    MDP_SCN_ADVERSARY = 3,
    MDP_SCN_TAG = 4
};

/* which parameter set of one agent (mdp_set_params / mdp_get_params) */
enum mdp_which {
    MDP_ACTOR = 0, MDP_CRITIC = 1, MDP_TGT_ACTOR = 2, MDP_TGT_CRITIC = 3,
    MDP_M_ACTOR = 4, MDP_V_ACTOR = 5, MDP_M_CRITIC = 6, MDP_V_CRITIC = 7,
    MDP_G_ACTOR = 8, MDP_G_CRITIC = 9
};

/* arena regions (mdp_region) */
enum mdp_region_id {
    MDP_R_THETA = 0, MDP_R_TARGET = 1, MDP_R_ADAM_M = 2, MDP_R_ADAM_V = 3,
    MDP_R_GRAD = 4, MDP_R_REPLAY = 5, MDP_R_INDEX = 6, MDP_R_STATS = 7,
    MDP_R_ENV = 8, MDP_R_EPLOG = 9, MDP_R_BETA = 10, MDP_R_SLAB = 11,
    MDP_R_CTL = 12, MDP_R_COUNT = 13
};

typedef struct mdp_config {
    int32_t n_agents;                 /* env.n (train.py:83) */
    int32_t obs_dim[MDP_MAX_AGENTS];  /* obs_shape_n (maddpg.py:113) */
    int32_t local_q[MDP_MAX_AGENTS];  /* local_q_func = ddpg (train.py:67-74) */
    int32_t act_dim;                  /* must be MDP_ACT_DIM */
    int32_t num_units;                /* --num-units, 1..MDP_MAX_UNITS (train.py:24) */
    int32_t batch_size;               /* --batch-size */
    int32_t max_episode_len;          /* --max-episode-len */
    int64_t capacity;                 /* ReplayBuffer(1e6) (maddpg.py:147) */
    int32_t num_envs;                 /* vector env copies on this rank (0: no env) */
    int32_t scenario;                 /* enum mdp_scenario */
    int32_t num_adversaries;          /* simple_tag / simple_adversary split */
    int32_t world_size, rank;         /* data-parallel group (grads scaled by 1/world) */
    float lr;                         /* --lr (Adam) */
    float tau;                        /* Polyak 1e-2 (maddpg.py:21) */
    float grad_clip;                  /* 0.5 (maddpg.py:130,142) */
    float actor_reg;                  /* 1e-3 (maddpg.py:56) */
    float adam_b1, adam_b2, adam_eps; /* TF1 AdamOptimizer defaults */
    double gamma;                     /* --gamma (TD target in fp64, maddpg.py:186) */
    uint64_t seed;                    /* device Philox key (Gumbel noise, env resets) */
    int32_t episode_log_rows;         /* finished-episode log ring (0: max(4096, 4 num_envs));
                                         otherwise >= 2 num_envs (mdp_create fails below);
                                         train.py sizes it save_rate + 2 num_envs */
    int32_t reserved;
} mdp_config;

typedef struct mdp_tensor_info {      /* one fully_connected{,_1,_2}/{weights,biases} */
    int64_t offset;                   /* floats from the start of a param-space region */
    int32_t rows, cols;               /* the TF variable's shape ([in, num_units] ...) */
    int32_t dev_rows, dev_cols;       /* its block in the arena: num_units padded to the
                                         kernel width (64/128/256), extra entries zero */
} mdp_tensor_info;

typedef struct mdp_handle mdp_handle;

/* ---- lifecycle ------------------------------------------------------- */
int32_t mdp_abi_version(void);
/* arena size for cfg; fills *param_floats with the param-space length (may be NULL) */
int64_t mdp_arena_bytes(const mdp_config* cfg, int64_t* param_floats);
/* U.initialize() / MADDPGAgentTrainer.__init__ (maddpg.py:113-149): binds the
 * arena, zeroes it, sets Adam beta powers, seeds the index RNG with seed. */
int mdp_create(const mdp_config* cfg, void* arena_dev, int64_t arena_bytes,
               void* hip_stream, mdp_handle** out);
int mdp_destroy(mdp_handle* h);
const char* mdp_last_error(const mdp_handle* h);
void* mdp_stream(mdp_handle* h);
int mdp_synchronize(mdp_handle* h);
/* byte offset + size of a region inside the arena */
int mdp_region(const mdp_handle* h, int32_t region, int64_t* offset, int64_t* bytes);
/* layout of tensor t (0..5 = W1,b1,W2,b2,W3,b3) of agent's actor (net=0) or critic (net=1) */
int mdp_tensor(const mdp_handle* h, int32_t agent, int32_t net, int32_t t, mdp_tensor_info* out);
/* joint replay row layout: offsets (floats) of agent's obs/act/obs_next/rew/done, row stride */
int mdp_row_layout(const mdp_handle* h, int32_t agent, int32_t out6[6]);

/* ---- parameters (golden injection, checkpoint; tf_util.py:259-273) --- */
int mdp_set_params(mdp_handle* h, int32_t agent, int32_t which, const float* src_host, int64_t n);
int mdp_get_params(mdp_handle* h, int32_t agent, int32_t which, float* dst_host, int64_t n);
/* beta1^t, beta2^t of agent's actor (net=0) / critic (net=1) Adam */
int mdp_get_beta_powers(mdp_handle* h, int32_t agent, int32_t net, float out2[2]);
int mdp_set_beta_powers(mdp_handle* h, int32_t agent, int32_t net, const float in2[2]);

/* ---- replay buffer (replay_buffer.py) -------------------------------- */
int64_t mdp_buffer_len(mdp_handle* h);                     /* __len__ :18-19 */
/* add `rows` whole joint rows [rows][row_stride] (device) at the ring head (:25-32) */
int mdp_buffer_add_rows(mdp_handle* h, const float* rows_dev, int64_t rows);
/* write agent's columns of arbitrary ring positions (per-agent add of the facade) */
int mdp_buffer_put_agent(mdp_handle* h, int32_t agent, const int64_t* pos_dev,
                         const float* cols_dev, int64_t rows);
/* host-tracked ring state after put_agent (len/next are per agent in the reference) */
int mdp_buffer_set_len(mdp_handle* h, int64_t len, int64_t next_idx);
/* random.seed(seed) on the device MT19937 (CPython init_by_array) */
int mdp_seed_py_random(mdp_handle* h, uint64_t seed);
/* random.setstate/getstate: 624 words + position (random.getstate()[1]) */
int mdp_set_rng_state(mdp_handle* h, const uint32_t* state625_host);
int mdp_get_rng_state(mdp_handle* h, uint32_t* state625_host);
/* make_index (:46-47): count x randint(0, len-1), bit-exact CPython stream */
int mdp_make_index(mdp_handle* h, int32_t count, int32_t* idx_dev);
/* sample_index (:55-56) fused gather: out[b] = joint row idx[b] */
int mdp_sample_rows(mdp_handle* h, const int32_t* idx_dev, int32_t count, float* out_dev);

/* ---- policies (maddpg.py:151-152, p_debug / q_debug) ------------------ */
/* act[rows][5] = gumbel_softmax(actor_or_target(obs)); u_dev: injected uniforms or NULL */
int mdp_act(mdp_handle* h, int32_t agent, int32_t target, const float* obs_dev,
            float* act_dev, int32_t rows, const float* u_dev);
/* logits[rows][5] = actor_or_target(obs) (p_debug['p_values'], maddpg.py:63) */
int mdp_actor_logits(mdp_handle* h, int32_t agent, int32_t target, const float* obs_dev,
                     float* logits_dev, int32_t rows);
/* q[rows] = critic_or_target(x[rows][cin]) with x already concatenated */
int mdp_q_values(mdp_handle* h, int32_t agent, int32_t target, const float* x_dev,
                 float* q_dev, int32_t rows);

/* ---- training (maddpg.py:161-196) ------------------------------------ */
/* One agent's update past the gates, strict reference order.
 * idx_dev: B indices or NULL (draw from the device MT stream);
 * u_tgt_dev: [n_agents][B][5] uniforms for the target actors or NULL;
 * u_act_dev: [B][5] uniforms for the actor-loss sample or NULL. */
int mdp_update(mdp_handle* h, int32_t agent, const int32_t* idx_dev,
               const float* u_tgt_dev, const float* u_act_dev);
/* gates of maddpg.py:162-165; returns 1 (skip) or 0 (train) */
int mdp_update_gate(mdp_handle* h, int64_t t);
/* MADDPGAgentTrainer.update(agents, t) as one call (maddpg.py:161-196), the
 * signature SURVEY.md 8b sketches: the gates at train step t (1 = skipped,
 * the reference's `return None`, nothing drawn), else the update on idx_dev
 * (B indices, or NULL: drawn from the device MT stream, replay_buffer.py:46-47)
 * with u_dev (NULL, or [n_agents][B][5] target-actor uniforms followed by
 * [B][5] actor-loss uniforms) and the 6 stats [q_loss, p_loss, mean y,
 * mean r, mean Q', std y] in stats_out (synchronous); 0 = trained, <0 error */
int mdp_agent_update(mdp_handle* h, int32_t agent, int64_t t, const int32_t* idx_dev, const float* u_dev,
                     double stats_out[6]);
/* update round: all agents in order (train.py:158-161), indices from the MT stream.
 * Replayed from a captured hipGraph after the first round (see mdp_set_graphs). */
int mdp_update_round(mdp_handle* h);
/* enable (default) / disable hipGraph replay of mdp_update_round / mdp_train_step */
int mdp_set_graphs(mdp_handle* h, int32_t on);
/* One vector step of the training loop (train.py:110-161 for num_envs env
 * copies): mdp_env_step with the policy's own actions, then `rounds` update
 * rounds (the rounds the update cadence makes due; 0..64).  Replayed as ONE
 * hipGraph per distinct `rounds` (per-round graph launches leave the GPU idle
 * between rounds).  Single-GPU path; data-parallel ranks use the phase entry
 * points below with an all-reduce between them. */
int mdp_train_step(mdp_handle* h, int32_t rounds);
/* n consecutive training steps (rounds[i] update rounds after step i's
 * rollout, exactly as n mdp_train_step calls) replayed as ONE graph, keyed
 * by the round counts: saves the graph-launch boundary between steps.  A step
 * with 0 rounds is its rollout launch alone inside the graph (a stretch of
 * them one k_rollout launch of that many steps when num_envs <= 16); before the first
 * (eager) training step, with profiling or eager collectives the steps run
 * one by one.  launch = 0:
 * only capture and instantiate the graph (nothing runs), so a timed region
 * replays graphs made ahead of it. */
int mdp_train_steps(mdp_handle* h, int32_t n, const int32_t* rounds, int32_t launch);

/* ---- native data parallelism (one process per GPU, RCCL over xGMI) ------
 * Replaces the reference's single-process update (maddpg.py:161-196) on G
 * ranks: each rank owns its env copies / replay shard / index stream; every
 * optimizer phase sums the reduced gradient with one ncclAllReduce on the
 * engine stream and applies it x 1/G (SURVEY §8e strict mode).  Rank 0 makes
 * the id, the caller broadcasts it (e.g. torch.distributed), every rank calls
 * mdp_dp_init; afterwards mdp_update / mdp_update_round / mdp_train_step run
 * the data-parallel update (collectives launched eagerly; MDP_DP_GRAPHS=1 in
 * the environment captures them in the step graph). RCCL is dlopen'ed. */
int mdp_dp_unique_id(uint8_t* out128);
int mdp_dp_init(mdp_handle* h, const uint8_t* id128, int32_t world, int32_t rank);

/* ---- direct xGMI gradient exchange (alternative to mdp_dp_init) ---------
 * Same semantics as the RCCL path (sum over ranks in rank order, x 1/G, every
 * replica bit-identical), but the exchange runs INSIDE the fused optimizer
 * kernel: each 256-parameter chunk workgroup stores its reduced chunk straight
 * into every peer's IPC-mapped buffer over xGMI, raises a per-chunk flag and
 * sums the world's chunks -- no collective launch, so a data-parallel update
 * has the single-GPU launch count (4 per agent strict, 3 per round
 * throughput).  Handshake (every rank, in order):
 *   open(world, rank) -> its 64-byte IPC handle; the caller all-gathers the
 *   handles; connect(handles[world][64]); probe() exchanges a known pattern
 *   (0 = every value arrived; fails after 30 s without a peer); the caller
 *   agrees on success across ranks, then enable() -- or close() everywhere and
 *   fall back to mdp_dp_init.  world 2..8. */
#define MDP_XGMI_HANDLE_BYTES 64
int mdp_dp_xgmi_open(mdp_handle* h, int32_t world, int32_t rank, uint8_t* handle_out);
int mdp_dp_xgmi_connect(mdp_handle* h, const uint8_t* handles);
int mdp_dp_xgmi_probe(mdp_handle* h, int32_t* mismatches);
int mdp_dp_xgmi_enable(mdp_handle* h);
int mdp_dp_xgmi_close(mdp_handle* h);
/* what this rank's data parallelism is wired to: out4 = {kind (0 none, 1 RCCL,
 * 2 direct xGMI), ranks in the communicator (ncclCommCount / exchange world),
 * this rank, peers reached (RCCL: ranks - 1; xGMI: peer buffers mapped)} */
int mdp_dp_info(mdp_handle* h, int32_t out4[4]);
/* what the direct xGMI exchange cost this rank (in-kernel s_memrealtime stamps
 * of k_reduce_apply's chunk workgroups: from a chunk's own stores to the
 * arrival of every peer's copy -- peer skew plus fabric latency): out4 =
 * {chunk exchanges counted, mean wait us, longest wait us, total wait us}
 * since the last reset; reset != 0 zeroes the counters.  The RCCL path's cost
 * is event-timed instead (mdp_prof_enable(MDP_K_ALLREDUCE)). */
int mdp_dp_exchange_stats(mdp_handle* h, double out4[4], int32_t reset);
/* collect those stamps (on != 0) in the optimizer launches issued from now on
 * while enabled -- eager launches and graphs captured meanwhile; graphs
 * captured with it off carry no stamping code path (default off: the three
 * counter atomics per chunk stay out of the exchange's critical path) */
int mdp_dp_exchange_stats_enable(mdp_handle* h, int32_t on);
/* Co-residency plan of the spin-waiting optimizer launch (k_reduce_apply: the
 * chunk workgroups of a tensor wait for each other's norm partials, the xGMI
 * exchange for the peers' chunks).  For cfg on a device with `cus` CUs that
 * hold `per_cu` of its 1024-thread workgroups each, out[2 agent + net] = the
 * launch's grid when the one-launch step is used (grid <= cus x per_cu), or
 * -grid when that net falls back to k_reduce + k_apply (no spin).  Returns the
 * number of nets that fall back, < 0 for an invalid cfg.  Needs no GPU. */
int mdp_ra_plan(const mdp_config* cfg, int32_t cus, int32_t per_cu, int32_t* out);
/* phase entry points for data parallelism (grad -> all-reduce -> apply) */
int mdp_critic_grad(mdp_handle* h, int32_t agent, const int32_t* idx_dev, const float* u_tgt_dev);
int mdp_actor_grad(mdp_handle* h, int32_t agent, const int32_t* idx_dev, const float* u_act_dev);
/* reduce the per-workgroup partials of net (0 actor, 1 critic) into MDP_R_GRAD */
int mdp_reduce_grad(mdp_handle* h, int32_t agent, int32_t net);
/* clip + Adam (+ Polyak of both nets when net==0) reading MDP_R_GRAD scaled by `scale` */
int mdp_apply_grad(mdp_handle* h, int32_t agent, int32_t net, float scale);
/* the 6 values update() returns (maddpg.py:196), fp64, synchronises */
int mdp_get_stats(mdp_handle* h, int32_t agent, double out6[6]);
/* debug check (the reference's _Function(check_nan), tf_util.py:322,366-368):
 * *nonfinite_out = the number of NaN / Inf values in every parameter set
 * (weights, targets, Adam m and v of every agent) and in the agents' update
 * stats; counted on the device, synchronous (ABI 5) */
int mdp_check_finite(mdp_handle* h, int64_t* nonfinite_out);

/* ---- update mode of the round paths (mdp_update_round, mdp_train_step) ----
 * 0 strict (default): the reference's order -- agents in turn, each critic
 *   step before its actor step, later agents' TD targets see the earlier
 *   agents' Polyak-updated target actors (maddpg.py:180-194, train.py:160-161).
 * 1 throughput (opt-in, NOT the reference's semantics): every
 *   agent's critic and actor gradients from the round-start parameters, then
 *   every clip + Adam + Polyak -- 3 launches per round.  With data parallelism
 *   (mdp_dp_init BEFORE this call): gradients, a reduce pass, ONE all-reduce
 *   of the whole gradient region per round, the step pass (x 1/world).  Needs
 *   the fused optimizer step for every net (mdp_create's co-residency plan)
 *   and <= 8 agents; the fast H=64 kernels batch every agent's gradients in
 *   one launch, the general kernels (H=128/256, > 3 target actors) run one
 *   gradient launch per agent and step kind. */
int mdp_set_update_mode(mdp_handle* h, int32_t mode);
/* one throughput-mode round with injected randomness (the parity entry point,
 * like mdp_update): idx_dev [n][B] (NULL: drawn from the index stream),
 * u_tgt_dev [n][n][B][5] (agent, target actor j, row), u_act_dev [n][B][5]
 * (NULL: device Philox noise, counter upd_ctr + agent) */
int mdp_update_all(mdp_handle* h, const int32_t* idx_dev, const float* u_tgt_dev, const float* u_act_dev);

/* ---- device environments (MPE World.step, train.py:104-128) ---------- */
int mdp_env_reset(mdp_handle* h);
/* one vector step: actions from the actors (or act_in_dev [E][n][5]), physics,
 * replay append, episode bookkeeping and resets at max_episode_len.
 * u_dev: injected Gumbel uniforms [E][n][5] or NULL. */
int mdp_env_step(mdp_handle* h, const float* act_in_dev, const float* u_dev);
/* env state: pos/vel [E][n_entities][2] fp32, goal [E] int32, ep_step [E] int32 */
int mdp_env_get_state(mdp_handle* h, float* pos_host, float* vel_host, int32_t* goal_host, int32_t* ep_step_host);
int mdp_env_set_state(mdp_handle* h, const float* pos_host, const float* vel_host, const int32_t* goal_host, const int32_t* ep_step_host);
int mdp_env_obs(mdp_handle* h, float* obs_dev);   /* current obs [E][sum obs] */
/* --benchmark mode (train.py:139-148): mdp_env_step that also writes every
 * agent's scenario benchmark_data() of the post-physics state (MPE
 * environment._get_info -> info_n['n']) to info_dev [E][n][MDP_BENCH_W] fp32,
 * before the episode reset.  Record per scenario (zero-padded):
 *   simple_spread    (rew_i, collisions_i, sum_l min_a dist, occupied landmarks)
 *   simple_adversary adversary: (|pos - goal|^2); good: (|pos - lm_l|^2 ..., |pos - goal|^2)
 *   simple_tag       adversary: (good agents in contact); good: (0)
 *   simple           has no benchmark_data (the reference's make_env raises): error */
#define MDP_BENCH_W 8
int mdp_env_step_bench(mdp_handle* h, float* info_dev);
/* finished-episode log: total entries written so far, copy last `n` [n][1+n_agents] */
int64_t mdp_episode_count(mdp_handle* h);
int mdp_episode_log(mdp_handle* h, int64_t first, int64_t n, float* out_host);

/* ---- profiling: HIP events bracketing every launch of one kernel kind -- */
enum mdp_kernel_kind {
    MDP_K_INDEX = 0, MDP_K_GATHER = 1, MDP_K_CRITIC_GRAD = 2, MDP_K_ACTOR_GRAD = 3,
    MDP_K_APPLY = 4, MDP_K_ROLLOUT = 5, MDP_K_REDUCE = 6, MDP_K_REDUCE_APPLY = 7,
    MDP_K_ALLREDUCE = 8,   /* the RCCL data-parallel all-reduces (not a kernel of this library) */
    MDP_K_COUNT = 9
};
int mdp_prof_enable(mdp_handle* h, int32_t kind, int32_t on);
/* which grad kernels serve `agent`: 1 = register-resident k_*_grad_r (H = 64
 * envelope), 0 = general k_*_grad */
int mdp_grad_variant(mdp_handle* h, int32_t agent);
/* sum of event-measured durations (ms) and launch count since enable; synchronises */
int mdp_prof_read(mdp_handle* h, int32_t kind, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* MADDPG_HIP_H */
