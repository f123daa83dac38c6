// mdp_api.cpp -- C ABI of libmaddpg_hip.so (declared in include/maddpg_hip.h).
//
// Owns the handle: arena carving, parameter/replay layout, the device MT19937
// control block, launch sequencing for the reference's per-agent update
// order (maddpg.py:161-196, train.py:158-161), the device env loop and the
// HIP-event kernel timers used by bench.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <map>
#include <vector>

#include "mdp_kernels.h"

namespace {

inline int64_t r4(int64_t n) { return (n + 3) & ~int64_t(3); }
inline int64_t a256(int64_t n) { return (n + 255) & ~int64_t(255); }

NDesc make_net(int64_t& off, int in, int H, int out) {
  NDesc d;
  d.off = (int)off;
  d.in = in;
  d.out = out;
  const int shp[6][2] = {{in, H}, {1, H}, {H, H}, {1, H}, {H, out}, {1, out}};
  for (int t = 0; t < 6; ++t) {
    d.t[t].off = (int)off;
    d.t[t].rows = shp[t][0];
    d.t[t].cols = shp[t][1];
    off += r4((int64_t)shp[t][0] * shp[t][1]);
  }
  d.size = (int)(off - d.off);
  return d;
}

// scenario entity tables (multiagent/scenarios/*.py make_world)
bool make_env(const mdp_config& c, EnvDesc& e, std::vector<int>& obs_dims, std::string& err) {
  std::memset(&e, 0, sizeof(e));
  e.scenario = c.scenario;
  e.max_ep_len = c.max_episode_len;
  const int n = c.n_agents;
  e.n_agents = n;
  for (int i = 0; i < MDP_MAX_ENT; ++i) e.max_speed[i] = -1.f;
  for (int i = 0; i < MDP_MAX_AGENTS; ++i) e.accel[i] = 5.0f;
  obs_dims.assign(n, 0);
  switch (c.scenario) {
    case MDP_SCN_SIMPLE:
      if (n != 1) { err = "simple has exactly 1 agent"; return false; }
      e.n_landmarks = 1;
      e.size[0] = e.size[1] = 0.05f;
      e.movable[0] = 1;
      obs_dims[0] = 4;
      break;
    case MDP_SCN_SPREAD:
      e.n_landmarks = n;
      for (int i = 0; i < n; ++i) {
        e.size[i] = 0.15f;
        e.collide[i] = 1;
        e.movable[i] = 1;
        e.size[n + i] = 0.05f;
        obs_dims[i] = 4 + 2 * n + 4 * (n - 1);
      }
      break;
    case MDP_SCN_ADVERSARY: {
      const int na = c.num_adversaries;
      if (na < 1 || na >= n) { err = "simple_adversary needs 1 <= adversaries < agents"; return false; }
      e.n_landmarks = n - 1;
      e.n_adv = na;
      for (int i = 0; i < n; ++i) {
        e.size[i] = 0.15f;
        e.movable[i] = 1;
        e.adversary[i] = i < na;
        obs_dims[i] = (i < na ? 0 : 2) + 2 * (n - 1) + 2 * (n - 1);
      }
      for (int l = 0; l < n - 1; ++l) e.size[n + l] = 0.08f;
      break;
    }
    case MDP_SCN_TAG: {
      const int na = c.num_adversaries, ng = n - na, L = 2;
      if (na < 1 || ng < 1) { err = "simple_tag needs >=1 adversary and >=1 good agent"; return false; }
      e.n_landmarks = L;
      e.n_adv = na;
      for (int i = 0; i < n; ++i) {
        const bool adv = i < na;
        e.adversary[i] = adv;
        e.size[i] = adv ? 0.075f : 0.05f;
        e.accel[i] = adv ? 3.0f : 4.0f;
        e.max_speed[i] = adv ? 1.0f : 1.3f;
        e.collide[i] = 1;
        e.movable[i] = 1;
        obs_dims[i] = 4 + 2 * L + 2 * (n - 1) + 2 * (adv ? ng : ng - 1);
      }
      for (int l = 0; l < L; ++l) {
        e.size[n + l] = 0.2f;
        e.collide[n + l] = 1;
      }
      break;
    }
    default:
      err = "unknown scenario";
      return false;
  }
  if (n + e.n_landmarks > MDP_MAX_ENT) { err = "too many entities"; return false; }
  return true;
}

struct Layout {
  Topo topo;
  EnvDesc env;
  int64_t PT = 0;
  int nwg = 0, slab_c = 0, slab_a = 0, eplog_rows = 0, n_ent = 0;
  int H_log = 0;  // --num-units (topo.H is the padded device width)
  int64_t off[MDP_R_COUNT];
  int64_t bytes[MDP_R_COUNT];
  int64_t total = 0;
};

bool build_layout(const mdp_config* c, Layout& L, std::string& err) {
  if (!c) { err = "null config"; return false; }
  if (c->n_agents < 1 || c->n_agents > MDP_MAX_AGENTS) { err = "n_agents out of range"; return false; }
  if (c->act_dim != MDP_ACT_DIM) { err = "act_dim must be 5 (MPE Discrete(5))"; return false; }
  if (c->num_units < 1 || c->num_units > MDP_MAX_UNITS) { err = "num_units must be in [1, 256]"; return false; }
  // upper bounds keep every row / index count of a launch inside int32
  if (c->batch_size < 1 || c->batch_size > (1 << 20)) { err = "batch_size must be in [1, 2^20]"; return false; }
  if (c->capacity < 1 || c->capacity > (int64_t(1) << 31) - 1) { err = "capacity out of range"; return false; }
  if (c->num_envs < 0 || c->num_envs > (1 << 24)) { err = "num_envs must be in [0, 2^24]"; return false; }
  // --num-units is any width (train.py:24); the device nets are H wide with H
  // the kernel width that holds it.  The extra hidden units have zero weights
  // and biases: relu(0) = 0 feeds nothing forward, their gradients are exactly
  // zero (ReLU mask / zero input activations), so Adam and Polyak keep them at
  // zero and every logical output is bit-identical to an unpadded net.
  const int n = c->n_agents, H = mdp_device_units(c->num_units);
  Topo& T = L.topo;
  std::memset(&T, 0, sizeof(T));
  T.n = n;
  T.H = H;
  L.H_log = c->num_units;
  int sum_obs = 0, obs_max = 0;
  for (int i = 0; i < n; ++i) {
    if (c->obs_dim[i] < 1 || c->obs_dim[i] > 256) { err = "obs_dim out of range"; return false; }
    sum_obs += c->obs_dim[i];
    obs_max = std::max(obs_max, (int)c->obs_dim[i]);
  }
  T.sum_obs = sum_obs;
  T.obs_max = obs_max;
  T.row_stride = (int)r4(2 * sum_obs + (MDP_ACT_DIM + 2) * n);
  int64_t off = 0;
  int acc = 0, cin_max = 0;
  for (int i = 0; i < n; ++i) {
    ADesc& a = T.ag[i];
    a.obs_dim = c->obs_dim[i];
    a.local_q = c->local_q[i] ? 1 : 0;
    a.obs_off = acc;
    a.act_off = sum_obs + MDP_ACT_DIM * i;
    a.nobs_off = sum_obs + MDP_ACT_DIM * n + acc;
    a.rew_off = 2 * sum_obs + MDP_ACT_DIM * n + i;
    a.done_off = 2 * sum_obs + MDP_ACT_DIM * n + n + i;
    acc += a.obs_dim;
    a.cin = a.local_q ? a.obs_dim + MDP_ACT_DIM : sum_obs + MDP_ACT_DIM * n;
    a.a_in_off = a.local_q ? a.obs_dim : sum_obs + MDP_ACT_DIM * i;
    cin_max = std::max(cin_max, a.cin);
    a.actor = make_net(off, a.obs_dim, H, MDP_ACT_DIM);
    a.critic = make_net(off, a.cin, H, 1);
  }
  T.cin_max = cin_max;
  L.PT = off;
  L.nwg = (c->batch_size + 15) / 16;
  for (int i = 0; i < n; ++i) {
    L.slab_c = std::max(L.slab_c, T.ag[i].critic.size);
    L.slab_a = std::max(L.slab_a, T.ag[i].actor.size);
  }
  const int E = c->num_envs;
  std::vector<int> dims;
  if (c->scenario != MDP_SCN_NONE) {
    if (!make_env(*c, L.env, dims, err)) return false;
    for (int i = 0; i < n; ++i)
      if (dims[i] != c->obs_dim[i]) {
        char b[160];
        std::snprintf(b, sizeof(b), "obs_dim[%d]=%d does not match scenario (%d)", i, c->obs_dim[i], dims[i]);
        err = b;
        return false;
      }
    if ((int64_t)E > c->capacity) { err = "num_envs exceeds replay capacity"; return false; }
  } else {
    std::memset(&L.env, 0, sizeof(L.env));
  }
  L.n_ent = n + L.env.n_landmarks;
  // The kernels' envelope: one 16-row tile of every launch keeps its rows and
  // activations in the CU's 160 KB of LDS.  The reference (TF1) has no such
  // limit; its largest MPE case (simple_tag N=6, H=128) needs 66 KB.  A larger
  // configuration is refused here, at create, not by its first update.
  {
    int need = std::max(lds_critic_bytes(T, 1), lds_actor_bytes(T));
    need = std::max(need, lds_eval_bytes(std::max(cin_max, obs_max), H));
    if (c->scenario != MDP_SCN_NONE) need = std::max(need, lds_rollout_bytes(T));
    if (need > MDP_LDS_BUDGET) {
      char b[200];
      std::snprintf(b, sizeof(b),
                    "configuration outside the kernels' LDS envelope: a 16-row tile needs %d bytes, a CU has %d "
                    "(sum of obs dims %d, %d units)", need, MDP_LDS_BUDGET, sum_obs, c->num_units);
      err = b;
      return false;
    }
  }
  if (c->episode_log_rows < 0) { err = "episode_log_rows < 0"; return false; }
  // lockstep logging writes slot ep_base + e for every env finishing in one
  // step: a ring shorter than two steps' worth would overwrite records of the
  // same or the previous step before a reader (LearningCurve) sees them
  if (c->episode_log_rows > 0 && (int64_t)c->episode_log_rows < 2 * (int64_t)E) {
    err = "episode_log_rows must be 0 (default) or at least 2 * num_envs";
    return false;
  }
  L.eplog_rows = c->episode_log_rows > 0 ? c->episode_log_rows : std::max(4096, 4 * E);
  int64_t sz[MDP_R_COUNT];
  sz[MDP_R_THETA] = sz[MDP_R_TARGET] = sz[MDP_R_ADAM_M] = sz[MDP_R_ADAM_V] = sz[MDP_R_GRAD] = 4 * L.PT;
  sz[MDP_R_REPLAY] = 4 * c->capacity * T.row_stride;
  sz[MDP_R_INDEX] = 2 * 4 * (int64_t)n * c->batch_size;  // two slots: round r draws round r+1's
  sz[MDP_R_STATS] = 8 * 8 * (int64_t)n;
  sz[MDP_R_ENV] = (int64_t)E * (4 * 4 * L.n_ent + 4 + 4 + 4 * n) + 64;
  sz[MDP_R_EPLOG] = 4 * (int64_t)L.eplog_rows * (1 + n);
  sz[MDP_R_BETA] = 4 * 8 * (int64_t)n;  // per optimizer: next powers (TF vars), powers of this step
  // per-agent blocks of partial gradients / stats / TD targets (throughput mode
  // computes every agent's gradients in one launch; strict mode uses block 0)
  sz[MDP_R_SLAB] = (int64_t)n * (4 * (int64_t)L.nwg * (L.slab_c + L.slab_a) + 2 * 8 * 8 * (int64_t)L.nwg +
                                  8 * (int64_t)c->batch_size) + 256 + 256 + mdp_ra_sync_bytes() +
                   4 * (int64_t)L.nwg * 16 * (MDP_APRE_W + MDP_CPRE_W + 2 * T.row_stride) +  // precomputed work + rows
                   512;  // counters
  sz[MDP_R_CTL] = sizeof(Ctl);
  int64_t o = 0;
  for (int r = 0; r < MDP_R_COUNT; ++r) {
    L.off[r] = o;
    L.bytes[r] = sz[r];
    o += a256(sz[r]);
  }
  L.total = o;
  return true;
}

// CPython _randommodule.c: init_genrand + init_by_array, key = 32-bit words of |seed|
void py_seed_state(uint64_t seed, uint32_t* mt, int32_t* pos) {
  std::vector<uint32_t> key;
  uint64_t s = seed;
  while (s) {
    key.push_back((uint32_t)(s & 0xffffffffu));
    s >>= 32;
  }
  if (key.empty()) key.push_back(0);
  mt[0] = 19650218u;
  for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int i = 1, j = 0;
  const int kl = (int)key.size();
  for (int k = std::max(624, kl); k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i;
    ++j;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
    if (j >= kl) j = 0;
  }
  for (int k = 623; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
  }
  mt[0] = 0x80000000u;
  *pos = 624;
}

}  // namespace

struct mdp_handle {
  mdp_config cfg;
  Layout L;
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  char* arena = nullptr;
  float *theta, *target, *m, *v, *grad, *replay, *beta, *slab_c, *slab_a, *eplog;
  float *pos, *vel, *ep_rew;
  int32_t *index, *goal, *ep_step;
  double *stats, *stat_c, *stat_a, *y;
  Ctl* ctl;
  int64_t len = 0, next = 0;  // host mirror of the ring
  uint32_t act_ctr = 0, reset_ctr = 0;
  bool env_lockstep = true;   // every env copy at the same episode step (log in env order)
  std::string err;
  bool ready = false;  // mdp_create finished: arena, stream and layout bound
  bool prof_on[MDP_K_COUNT] = {};
  std::vector<hipEvent_t> ev[MDP_K_COUNT];
  size_t ev_used[MDP_K_COUNT] = {};
  double prof_ms[MDP_K_COUNT] = {};
  int64_t prof_n[MDP_K_COUNT] = {};
  // hipGraph of one update round (index draw + every agent's 6 kernels)
  bool graphs = true;
  bool capturing = false;
  int eager_rounds = 0;
  // MDP_GENERAL_GRADS=1 in the environment at create: always use the general
  // grad kernels (mdp_grads.hip) -- lets tests compare both paths
  bool general_grads = false;
  // single-GPU optimizer step as one k_reduce_apply launch (MDP_UNFUSED_APPLY=1: k_reduce + k_apply)
  bool fused_apply = true;
  uint32_t* ra_ctr = nullptr;
  uint64_t* ra_part = nullptr;
  // the actor forward + sample of agent i computed by extra workgroups of its
  // critic-step launch (fast kernels, strict order; MDP_ACTOR_PRE=0: off)
  float* apre = nullptr;
  bool actor_pre = true;
  // the next agent's critic-step work independent of this agent's update,
  // computed by extra workgroups of this agent's actor-step launch (critic_pre
  // -> critic_post; fast kernels, strict order; MDP_CRITIC_PRE=0: off)
  float* cpre = nullptr;
  bool critic_pre = true;
  float* apre_rows = nullptr;  // the replay rows those launches gathered (read contiguously by the step)
  float* cpre_rows = nullptr;
  hipGraph_t round_graph = nullptr;
  hipGraphExec_t round_exec = nullptr;
  // mdp_train_step graphs (rollout + k rounds), one per k
  std::map<int, hipGraphExec_t> step_exec;
  // mdp_train_steps graphs: several consecutive steps as one graph, keyed by their round counts
  std::map<std::vector<int>, hipGraphExec_t> multi_exec;
  int eager_steps = 0;
  // native data parallelism (mdp_dp_init): RCCL communicator of this rank
  ncclComm_t comm = nullptr;
  int dp_world = 1;
  bool dp_graphs = false;  // capture collectives in the step graph (MDP_DP_GRAPHS=1)
  // update mode of the round paths: 0 strict (maddpg.py order), 1 throughput
  int update_mode = 0;
  FusedApplyArgs* tp_list = nullptr;  // device copy of the 2n optimizer steps (throughput mode)
  RaBatch tp_batch;                   // single GPU: reduce + step
  RaBatch tp_reduce, tp_step;         // data parallel: reduce pass, all-reduce, step pass (x 1/G)
  // co-residency of the spin-waiting optimizer launches (k_reduce_apply's
  // norm handshake, the xGMI exchange): CUs x resident workgroups per CU of
  // k_reduce_apply / k_reduce_apply_batch, measured at create
  int ra_cap = 0, ra_batch_cap = 0;
  bool tp_fits[4] = {true, true, true, true};  // per RaBatch: whole grid co-resident
  std::vector<FusedApplyArgs> tp_host[4];     // the batches' entries, for per-net launches
  RaBatch tp_xchg;                    // data parallel over xGMI: reduce + exchange + step (x 1/G)
  // general kernels (tp_round_general): agent i's optimizer steps right after
  // its gradients, as one launch of the [critic_i, actor_i] pair reading the
  // SHARED slabs (phase 0 single GPU, 1 reduce-only before the all-reduce, 3
  // xGMI); no Polyak inside (one k_polyak after the round's last step)
  RaBatch tp_pair[3][MDP_MAX_AGENTS];
  bool tp_pair_fits[3][MDP_MAX_AGENTS] = {};
  FusedApplyArgs tp_pair_host[3][MDP_MAX_AGENTS][2];
  // the xGMI batch only when its whole grid is co-resident (every chunk
  // workgroup spins on its peers' matching chunk); otherwise one launch per net
  bool rollout_draw = true;           // step_launches: first-round draw inside k_rollout
  bool draw_ahead = true;             // step_launches: draws one agent ahead (MDP_DRAW_AHEAD=0: per round)
  bool grad_pair = true;              // throughput mode, general kernels: critic + actor step in one launch (MDP_GRAD_PAIR=0: two)
  // direct xGMI exchange (mdp_dp_p2p_*): this rank's IPC-exported buffer and
  // the device descriptor of every rank's buffer mapped here
  uint64_t* xbuf = nullptr;
  int x_world = 0, x_rank = 0;
  std::vector<void*> x_opened;        // peer buffers opened with hipIpcOpenMemHandle
  XchgDesc* xd_dev = nullptr;
  uint32_t* x_probe = nullptr;        // [0] mismatches, [1] fault of the connection probe
  uint32_t x_probe_ep = 0;
  bool p2p = false;
  bool xw_stats = false;              // stamp the exchange waits (mdp_dp_exchange_stats_enable)
};

namespace {

int fail(mdp_handle* h, const char* what, hipError_t e = hipSuccess) {
  if (h) {
    h->err = what;
    if (e != hipSuccess) {
      h->err += ": ";
      h->err += hipGetErrorString(e);
    }
  }
  return -1;
}

#define HIPCHK(h, call)                        \
  do {                                         \
    hipError_t e__ = (call);                   \
    if (e__ != hipSuccess) return fail(h, #call, e__); \
  } while (0)

// every entry point on a handle refuses a null one and one whose mdp_create
// failed (no arena or stream bound: nothing may be launched on it); the
// create error stays in mdp_last_error
bool unusable(const mdp_handle* h) { return !h || !h->ready; }
#define MDP_NEED(h)               \
  do {                            \
    if (unusable(h)) return -1;   \
  } while (0)

// A caller buffer that a kernel dereferences ("_dev" in the header) must be
// memory of the handle's device (hipMalloc, PyTorch's caching allocator,
// managed memory) and hold `bytes` from `p` to the end of its allocation.  A
// host address that reached a kernel faulted the GPU with an illegal memory
// access instead of returning < 0 (round 5's r05h), so every entry
// point checks its pointers here before anything is launched: one
// hipPointerGetAttributes (+ hipMemGetAddressRange) per pointer, host-side
// only; graph replays take no caller pointers.  null_ok: NULL means "not
// given" for this argument.  h->device is set by mdp_create before any check.
int need_dev(mdp_handle* h, const void* p, int64_t bytes, const char* fn, const char* arg, bool null_ok = true) {
  auto refuse = [&](const char* why) {
    std::string m = std::string(fn) + ": " + arg + " " + why;
    return fail(h, m.c_str());
  };
  if (!p) return null_ok ? 0 : refuse("is null");
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  const hipError_t e = hipPointerGetAttributes(&a, p);
  // an unknown (host) address may set the runtime's last error: clear it, or
  // the next launch's hipGetLastError check would report it
  if (e != hipSuccess) (void)hipGetLastError();
  // (device memory mapped with hipMemCreate + hipMemMap -- PyTorch's expandable
  // segments -- reports type Device too: tests/native/abi_host_check.cpp, r06r)
  const bool managed = a.isManaged || a.type == hipMemoryTypeManaged;
  if (e != hipSuccess || !(a.type == hipMemoryTypeDevice || managed)) {
    (void)hipGetLastError();
    return refuse("is not device memory (a host address would fault the GPU); pass a buffer of the handle's device");
  }
  if (!managed && a.device != h->device) return refuse("is memory of another device than the handle's");
  if (!managed && bytes > 0) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess) {
      if ((const char*)p + bytes > (const char*)base + size)
        return refuse("ends before the bytes this call reads or writes (allocation too small)");
    } else {
      (void)hipGetLastError();
    }
  }
  return 0;
}
#define MDP_DEV(h, p, bytes, fn, null_ok)                                   \
  do {                                                                     \
    if (need_dev(h, p, (int64_t)(bytes), fn, #p, null_ok)) return -1;     \
  } while (0)

}  // namespace

MdpLaunchEv& mdp_launch_ev() {
  static thread_local MdpLaunchEv e;
  return e;
}

namespace {

// time one launch when profiling `kind`.  packet (the kernel launchers, which
// go through mdp_launch): the pair rides on the launch's own dispatch packet,
// so the elapsed time is that packet's begin -> end, the interval rocprofv3
// reports.  Otherwise (an RCCL call, a multi-launch gather) the pair is
// recorded as markers around the scope and includes their own cost.
struct ProfScope {
  mdp_handle* h;
  int kind;
  bool packet;
  hipEvent_t stop = nullptr;
  ProfScope(mdp_handle* hh, int k, bool pk = true) : h(hh), kind(k), packet(pk) {
    if (!h->prof_on[kind] || h->capturing) return;
    auto& pool = h->ev[kind];
    size_t u = h->ev_used[kind];
    if (u + 2 > pool.size()) {
      for (int q = 0; q < 64; ++q) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        pool.push_back(e);
      }
    }
    h->ev_used[kind] = u + 2;
    stop = pool[u + 1];
    if (packet) {
      mdp_launch_ev() = MdpLaunchEv{pool[u], pool[u + 1]};
    } else {
      (void)hipEventRecord(pool[u], h->stream);
    }
  }
  ~ProfScope() {
    if (!stop) return;
    if (!packet) {
      (void)hipEventRecord(stop, h->stream);
      return;
    }
    MdpLaunchEv& e = mdp_launch_ev();
    if (e.start) {  // nothing was launched (an error path): drop the unrecorded pair
      e.start = e.stop = nullptr;
      h->ev_used[kind] -= 2;
    }
  }
};

void flush_prof(mdp_handle* h, int kind) {
  auto& pool = h->ev[kind];
  const size_t u = h->ev_used[kind];
  if (!u) return;
  (void)hipEventSynchronize(pool[u - 1]);
  for (size_t q = 0; q + 1 < u; q += 2) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pool[q], pool[q + 1]) == hipSuccess) {
      h->prof_ms[kind] += ms;
      h->prof_n[kind] += 1;
    }
  }
  h->ev_used[kind] = 0;
}

bool bad_agent(mdp_handle* h, int agent) {
  if (unusable(h)) return true;
  if (agent < 0 || agent >= h->cfg.n_agents) {
    fail(h, "agent index out of range");
    return true;
  }
  return false;
}

int region_for(int which, int* region, int* net) {
  switch (which) {
    case MDP_ACTOR: *region = MDP_R_THETA; *net = 0; return 0;
    case MDP_CRITIC: *region = MDP_R_THETA; *net = 1; return 0;
    case MDP_TGT_ACTOR: *region = MDP_R_TARGET; *net = 0; return 0;
    case MDP_TGT_CRITIC: *region = MDP_R_TARGET; *net = 1; return 0;
    case MDP_M_ACTOR: *region = MDP_R_ADAM_M; *net = 0; return 0;
    case MDP_V_ACTOR: *region = MDP_R_ADAM_V; *net = 0; return 0;
    case MDP_M_CRITIC: *region = MDP_R_ADAM_M; *net = 1; return 0;
    case MDP_V_CRITIC: *region = MDP_R_ADAM_V; *net = 1; return 0;
    case MDP_G_ACTOR: *region = MDP_R_GRAD; *net = 0; return 0;
    case MDP_G_CRITIC: *region = MDP_R_GRAD; *net = 1; return 0;
    default: return -1;
  }
}

const NDesc& net_of(mdp_handle* h, int agent, int net) {
  return net ? h->L.topo.ag[agent].critic : h->L.topo.ag[agent].actor;
}

// logical (TF variable) shape of tensor t of a net whose device width is padded:
// (W1 [in, u], b1 [u], W2 [u, u], b2 [u], W3 [u, out], b3 [out], u = --num-units)
void logical_shape(const mdp_handle* h, const NDesc& d, int t, int* rows, int* cols) {
  const int u = h->L.H_log;
  *rows = (t == 2 || t == 4) ? u : d.t[t].rows;
  *cols = t < 4 ? u : d.t[t].cols;
}

int64_t net_floats(const mdp_handle* h, const NDesc& d) {
  int64_t s = 0;
  for (int t = 0; t < 6; ++t) {
    int r, c;
    logical_shape(h, d, t, &r, &c);
    s += (int64_t)r * c;
  }
  return s;
}

int launch_make_index(mdp_handle* h, int count, int32_t* out) {
  if (h->len <= 0) return fail(h, "make_index on an empty replay buffer (randint(0, -1))");
  ProfScope p(h, MDP_K_INDEX);
  HIPCHK(h, mdp_launch_make_index(h->ctl, count, out, h->stream));
  return 0;
}

bool tp_fast(const mdp_handle* h);


// tp: throughput mode on the general kernels -- this agent's own blocks of
// partials / stats / TD targets and noise counter upd_ctr + agent (multi = 2
// marks it; the general kernels take the agent from a.agent, not the grid)
// shared: throughput mode with the strict mode's slab (consumed by this
// agent's own optimizer launch before the next agent's gradients run)
CriticArgs critic_args(mdp_handle* h, int agent, const int32_t* idx, const float* u_tgt, bool tp, int post_prev,
                       const float* u_act, bool shared) {
  CriticArgs a;
  a.apre = nullptr;
  a.u_act = u_act;
  a.cpre = nullptr;
  a.cpre_rows = h->cpre_rows;
  a.apre_rows = h->apre_rows;
  a.cpre_prev = post_prev;
  a.multi = tp ? 2 : 0;
  a.slab_agent_stride = 0;
  a.pf_ctl = h->ctl;
  a.pf_out = nullptr;
  a.pf_count = 0;
  a.topo = h->L.topo;
  a.agent = agent;
  a.B = h->cfg.batch_size;
  a.theta = h->theta;
  a.target = h->target;
  a.replay = h->replay;
  a.idx = idx;
  a.u_tgt = u_tgt;
  a.seed = h->cfg.seed;
  a.ctl = h->ctl;
  a.gamma = h->cfg.gamma;
  a.inv_b = 1.0f / (float)a.B;
  a.slab = h->slab_c;
  a.slab_stride = h->L.slab_c;
  a.slab_stat = h->stat_c;
  a.y_out = h->y;
  if (tp) {
    if (!shared) a.slab += (int64_t)agent * h->L.nwg * h->L.slab_c;
    a.slab_stat += (int64_t)agent * h->L.nwg * 8;
    a.y_out += (int64_t)agent * h->cfg.batch_size;
  }
  // as many target actors per pass as the LDS budget allows (all of them for S1-S4)
  const int nact = h->L.topo.ag[agent].local_q ? 1 : h->cfg.n_agents;
  int G = nact;
  while (G > 1 && lds_critic_bytes(h->L.topo, G) > MDP_LDS_BUDGET) --G;
  a.group = G;
  return a;
}

int do_critic_grad(mdp_handle* h, int agent, const int32_t* idx, const float* u_tgt, int32_t* pf_out = nullptr,
                   bool tp = false, bool apre = false, const float* u_act = nullptr, int post_prev = -1,
                   int pf_n = 0, bool shared = false) {
  CriticArgs a = critic_args(h, agent, idx, u_tgt, tp, post_prev, u_act, shared);
  ProfScope p(h, MDP_K_CRITIC_GRAD);
  if (!tp && !h->general_grads && grads_r_ok(h->L.topo, agent)) {
    if (pf_out) {  // pf_n indices of the next round's draw (0: all n B of them)
      a.pf_out = pf_out;
      a.pf_count = pf_n > 0 ? pf_n : h->cfg.n_agents * h->cfg.batch_size;
    }
    if (apre) a.apre = h->apre;
    if (post_prev >= 0) a.cpre = h->cpre;
    HIPCHK(h, mdp_launch_critic_grad_r(a, lds_critic_r_bytes(h->L.topo, agent), h->stream));
    return 0;
  }
  if (lds_critic_bytes(h->L.topo, a.group) > MDP_LDS_BUDGET) return fail(h, "critic step does not fit in LDS");
  HIPCHK(h, mdp_launch_critic_grad(a, h->L.topo.H, lds_critic_bytes(h->L.topo, a.group), h->stream));
  return 0;
}

ActorArgs actor_args(mdp_handle* h, int agent, const int32_t* idx, const float* u_act, bool tp, bool apre,
                     int pre_next, const int32_t* pre_idx, bool shared) {
  ActorArgs a;
  a.apre = apre ? h->apre : nullptr;
  a.apre_rows = h->apre_rows;
  a.cpre = nullptr;
  a.cpre_rows = h->cpre_rows;
  a.cpre_agent = pre_next;
  a.cpre_idx = pre_idx;
  a.target = h->target;
  a.multi = tp ? 2 : 0;
  a.slab_agent_stride = 0;
  a.topo = h->L.topo;
  a.agent = agent;
  a.B = h->cfg.batch_size;
  a.theta = h->theta;
  a.replay = h->replay;
  a.idx = idx;
  a.u_act = u_act;
  a.seed = h->cfg.seed;
  a.ctl = h->ctl;
  a.neg_inv_b = -1.0f / (float)a.B;
  a.reg_scale = (float)(2.0 * (double)h->cfg.actor_reg / ((double)a.B * MDP_ACT_DIM));
  a.slab = h->slab_a;
  a.slab_stride = h->L.slab_a;
  a.slab_stat = h->stat_a;
  if (tp) {
    if (!shared) a.slab += (int64_t)agent * h->L.nwg * h->L.slab_a;
    a.slab_stat += (int64_t)agent * h->L.nwg * 8;
  }
  return a;
}

int do_actor_grad(mdp_handle* h, int agent, const int32_t* idx, const float* u_act, bool tp = false,
                  bool apre = false, int pre_next = -1, const int32_t* pre_idx = nullptr, bool shared = false) {
  ActorArgs a = actor_args(h, agent, idx, u_act, tp, apre, pre_next, pre_idx, shared);
  ProfScope p(h, MDP_K_ACTOR_GRAD);
  if (!tp && !h->general_grads && grads_r_ok(h->L.topo, agent)) {
    int lds = lds_actor_r_bytes(h->L.topo);
    if (pre_next >= 0) {
      a.cpre = h->cpre;
      lds = std::max(lds, lds_critic_pre_bytes(h->L.topo));
    }
    HIPCHK(h, mdp_launch_actor_grad_r(a, lds, h->stream));
    return 0;
  }
  HIPCHK(h, mdp_launch_actor_grad(a, h->L.topo.H, lds_actor_bytes(h->L.topo), h->stream));
  return 0;
}

// net 1: critic Adam (+ critic stats); net 0: actor Adam + Polyak of both nets (+ actor stats)
ApplyArgs apply_args(mdp_handle* h, int agent, int net, float scale, bool tp = false) {
  const ADesc& ag = h->L.topo.ag[agent];
  ApplyArgs a;
  a.net = net ? ag.critic : ag.actor;
  a.other = net ? ag.actor : ag.critic;
  a.theta = h->theta;
  a.target = h->target;
  a.m = h->m;
  a.v = h->v;
  a.grad = h->grad;
  auto chunks = [](const NDesc& d, int* blk) {
    blk[0] = 0;
    for (int t = 0; t < 6; ++t)
      blk[t + 1] = blk[t] + (d.t[t].rows * d.t[t].cols + MDP_APPLY_CHUNK - 1) / MDP_APPLY_CHUNK;
  };
  chunks(a.net, a.blk);
  chunks(a.other, a.oblk);
  a.slab = nullptr;
  a.slab_stride = net ? h->L.slab_c : h->L.slab_a;
  a.nwg = h->L.nwg;
  a.scale = scale;
  a.clip = h->cfg.grad_clip;
  a.lr = h->cfg.lr;
  a.b1 = h->cfg.adam_b1;
  a.b2 = h->cfg.adam_b2;
  a.eps = h->cfg.adam_eps;
  a.beta = h->beta + agent * 8 + net * 4;
  a.polyak = net ? 0 : 1;
  const double tau = (double)h->cfg.tau;
  a.pa = (float)(1.0 - tau);
  a.pb = (float)(1.0 - (1.0 - tau));
  a.stats_mode = net ? 1 : 2;
  a.slab_stat = net ? h->stat_c : h->stat_a;
  a.y = h->y;
  a.B = h->cfg.batch_size;
  a.reg = h->cfg.actor_reg;
  a.stats_out = h->stats + agent * 8;
  a.ticket = &h->ctl->ticket[net];
  a.ctl = h->ctl;
  a.bump_ctr = net ? 0 : 1;
  return a;
}

int do_apply(mdp_handle* h, int agent, int net, bool from_slab, float scale) {
  (void)from_slab;
  const ApplyArgs a = apply_args(h, agent, net, scale);
  ProfScope p(h, MDP_K_APPLY);
  HIPCHK(h, mdp_launch_apply(a, h->stream));
  return 0;
}

// batch reduction + clip + Adam (+ Polyak, stats, beta advance) in one launch
// (single GPU, and the xGMI exchange).  Its chunk workgroups spin on each other
// (the per-tensor norm handshake; the exchange also on the peers' matching
// chunk), so the launch is used only when its whole grid is co-resident --
// grid <= CUs x resident workgroups per CU -- and every tensor's chunks fit the
// sync area; otherwise the step runs as k_reduce + k_apply (no spin).
bool reduce_apply_ok(const mdp_handle* h, int agent, int net) {
  return mdp_ra_fits(h->L.topo, agent, net, h->ra_cap);
}

FusedApplyArgs fused_args_for(mdp_handle* h, int agent, int net, bool tp = false) {
  FusedApplyArgs f;
  f.ap = apply_args(h, agent, net, 1.0f, tp);
  f.ap.slab = net ? h->slab_c : h->slab_a;
  f.rblk[0] = 0;
  for (int t = 0; t < 6; ++t)
    f.rblk[t + 1] = f.rblk[t] + (f.ap.net.t[t].rows * f.ap.net.t[t].cols + MDP_RA_CHUNK - 1) / MDP_RA_CHUNK;
  const int g = agent * 2 + net;
  f.sync_ctr = h->ra_ctr + (int64_t)g * 8 * 32;
  f.done_ctr = f.sync_ctr + 6 * 32;
  f.sync_part = h->ra_part + (int64_t)g * 6 * MDP_RA_MAXCH * 2;
  f.phase = 0;
  f.xd = nullptr;
  f.net_id = g;
  f.xstep = nullptr;
  f.wstat = nullptr;
  f.pf_count = 0;
  f.pf_out = nullptr;
  f.pf_ctl = h->ctl;
  return f;
}

// phase 3: reduce + xGMI exchange with every rank + step x 1/G (one launch)
void set_xchg(mdp_handle* h, FusedApplyArgs& f, int agent, int net) {
  f.phase = 3;
  f.ap.scale = 1.0f / (float)h->dp_world;
  f.xd = h->xd_dev;
  f.net_id = 2 * agent + net;
  f.xstep = h->ctl->xstep + f.net_id;
  f.wstat = h->xw_stats ? &h->ctl->xw_ticks : nullptr;
}

void xgmi_release(mdp_handle* h) {
  for (void* p : h->x_opened)
    if (p) (void)hipIpcCloseMemHandle(p);
  h->x_opened.clear();
  if (h->xd_dev) (void)hipFree(h->xd_dev);
  if (h->x_probe) (void)hipFree(h->x_probe);
  if (h->xbuf) (void)hipFree(h->xbuf);
  h->xd_dev = nullptr;
  h->x_probe = nullptr;
  h->xbuf = nullptr;
  h->p2p = false;
  h->x_world = 0;
  h->x_rank = 0;
}

// pf_out / pf_count: a piece of the next round's index draw rides in this launch
int do_reduce_apply(mdp_handle* h, int agent, int net, int32_t* pf_out = nullptr, int pf_count = 0) {
  FusedApplyArgs f = fused_args_for(h, agent, net);
  if (pf_out && pf_count > 0) {
    f.pf_out = pf_out;
    f.pf_count = pf_count;
  }
  if (h->p2p) set_xchg(h, f, agent, net);
  ProfScope p(h, MDP_K_REDUCE_APPLY);
  HIPCHK(h, mdp_launch_reduce_apply(f, h->stream));
  return 0;
}

int do_reduce(mdp_handle* h, int agent, int net) {
  const NDesc& d = net_of(h, agent, net);
  ReduceArgs a;
  a.slab = net ? h->slab_c : h->slab_a;
  a.nwg = h->L.nwg;
  a.slab_stride = net ? h->L.slab_c : h->L.slab_a;
  a.grad = h->grad;
  a.off = d.off;
  a.size = d.size;
  a.beta = h->beta + agent * 8 + net * 4;
  a.b1 = h->cfg.adam_b1;
  a.b2 = h->cfg.adam_b2;
  a.ctl = h->ctl;
  a.bump_ctr = net ? 0 : 1;
  ProfScope p(h, MDP_K_REDUCE);
  HIPCHK(h, mdp_launch_reduce(a, h->stream));
  return 0;
}

// ---- RCCL, loaded on first use (the library has no link-time RCCL dependency)
struct RcclApi {
  bool tried = false, ok = false;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  decltype(&ncclCommCount) count = nullptr;
};
RcclApi& rccl() {
  static RcclApi r;
  if (!r.tried) {
    r.tried = true;
    // MDP_RCCL_LIB: another library with RCCL's entry points (the tests'
    // one-GPU stand-in communicator, tests/rccl_standin/); no fallback then
    const char* alt = getenv("MDP_RCCL_LIB");
    void* so = nullptr;
    if (alt && alt[0]) {
      so = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
    } else {
      so = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
      if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    if (so) {
      r.get_id = (decltype(r.get_id))dlsym(so, "ncclGetUniqueId");
      r.init_rank = (decltype(r.init_rank))dlsym(so, "ncclCommInitRank");
      r.all_reduce = (decltype(r.all_reduce))dlsym(so, "ncclAllReduce");
      r.destroy = (decltype(r.destroy))dlsym(so, "ncclCommDestroy");
      r.err = (decltype(r.err))dlsym(so, "ncclGetErrorString");
      r.count = (decltype(r.count))dlsym(so, "ncclCommCount");
      r.ok = r.get_id && r.init_rank && r.all_reduce && r.destroy && r.err;
    }
  }
  return r;
}

// sum all-reduce of one net's reduced gradient (flat, in the grad region) on the engine stream
int dp_allreduce(mdp_handle* h, int agent, int net) {
  const NDesc& d = net_of(h, agent, net);
  float* g = h->grad + d.off;
  ProfScope p(h, MDP_K_ALLREDUCE, false);
  const ncclResult_t r = rccl().all_reduce(g, g, (size_t)d.size, ncclFloat32, ncclSum, h->comm, h->stream);
  if (r != ncclSuccess) {
    h->err = std::string("ncclAllReduce: ") + rccl().err(r);
    return -1;
  }
  return 0;
}

// throughput mode: the whole grad region (every agent's actor + critic) in one call
int dp_allreduce_all(mdp_handle* h) {
  ProfScope p(h, MDP_K_ALLREDUCE, false);
  const ncclResult_t r = rccl().all_reduce(h->grad, h->grad, (size_t)h->L.PT, ncclFloat32, ncclSum, h->comm, h->stream);
  if (r != ncclSuccess) {
    h->err = std::string("ncclAllReduce: ") + rccl().err(r);
    return -1;
  }
  return 0;
}

// the critic step's launch also computes the actor step's forward + sample
// (extra workgroups on the otherwise idle CUs; the actor weights are not
// touched by the critic step, the indices and noise are the actor step's own)
bool actor_pre_ok(const mdp_handle* h, int agent) {
  return h->actor_pre && !h->general_grads && grads_r_ok(h->L.topo, agent);
}

// agent k's critic step split around agent p's update (critic_pre in p's actor
// launch, critic_post for k): fast kernels for both, k's critic MADDPG-style
// (a DDPG critic needs no target actor but its own).  p != k: the pre part
// accumulates k's TARGET critic layer 1, which p's actor optimizer launch
// Polyak-updates -- with k == p (one agent, carried across rounds) that
// accumulator would be one Polyak step stale.
bool critic_pre_ok(const mdp_handle* h, int p, int k) {
  const Topo& T = h->L.topo;
  return p != k && h->critic_pre && !h->general_grads && grads_r_ok(T, p) && grads_r_ok(T, k) &&
         !T.ag[k].local_q;
}

// strict data-parallel update of one agent (maddpg.py:188-194 order):
// critic grads -> reduce -> all-reduce -> clip + Adam (x 1/G); then the actor
// the next round's draw in pieces inside the optimizer launches (general kernels)
struct DrawPieces {
  int32_t* out = nullptr;   // this agent's critic-step piece; the actor-step piece follows it
  int n_critic = 0, n_actor = 0;
  int n_grad = 0;           // the critic-gradient launch's draw into pf_out (0: the whole next round)
};

int do_update_dp(mdp_handle* h, int agent, const int32_t* idx, const float* u_tgt, const float* u_act,
                 int32_t* pf_out, int post_prev, int pre_next, const int32_t* pre_idx, const DrawPieces& dp) {
  const float scale = 1.0f / (float)h->dp_world;
  const bool pre = actor_pre_ok(h, agent);
  int rc;
  if (h->p2p) {  // the exchange lives inside the optimizer launch: same 4 launches as one GPU
    if ((rc = do_critic_grad(h, agent, idx, u_tgt, pf_out, false, pre, u_act, post_prev, dp.n_grad))) return rc;
    if ((rc = do_reduce_apply(h, agent, 1, dp.out, dp.n_critic))) return rc;
    if ((rc = do_actor_grad(h, agent, idx, u_act, false, pre, pre_next, pre_idx))) return rc;
    return do_reduce_apply(h, agent, 0, dp.out ? dp.out + dp.n_critic : nullptr, dp.n_actor);
  }
  if ((rc = do_critic_grad(h, agent, idx, u_tgt, pf_out, false, pre, u_act, post_prev, dp.n_grad))) return rc;
  if ((rc = do_reduce(h, agent, 1))) return rc;
  if ((rc = dp_allreduce(h, agent, 1))) return rc;
  if ((rc = do_apply(h, agent, 1, false, scale))) return rc;
  if ((rc = do_actor_grad(h, agent, idx, u_act, false, pre, pre_next, pre_idx))) return rc;
  if ((rc = do_reduce(h, agent, 0))) return rc;
  if ((rc = dp_allreduce(h, agent, 0))) return rc;
  return do_apply(h, agent, 0, false, scale);
}

// pf_out: the critic kernel also draws the next round's indices there (fast path only)
// post_prev >= 0: this critic step finishes the work that agent post_prev's
// actor launch started (critic_post); pre_next >= 0: this actor launch starts
// agent pre_next's next critic step on indices pre_idx (critic_pre)
int do_update(mdp_handle* h, int agent, const int32_t* idx, const float* u_tgt, const float* u_act,
              int32_t* pf_out = nullptr, int post_prev = -1, int pre_next = -1, const int32_t* pre_idx = nullptr,
              const DrawPieces& dp = DrawPieces()) {
  // data parallel: the exchange runs whatever the noise source (injected
  // uniforms included -- an update that skipped it would split the replicas)
  if (h->comm || h->p2p) return do_update_dp(h, agent, idx, u_tgt, u_act, pf_out, post_prev, pre_next, pre_idx, dp);
  int rc;
  const bool fused = h->fused_apply && reduce_apply_ok(h, agent, 0) && reduce_apply_ok(h, agent, 1);
  const bool pre = actor_pre_ok(h, agent);
  if ((rc = do_critic_grad(h, agent, idx, u_tgt, pf_out, false, pre, u_act, post_prev, dp.n_grad))) return rc;
  if (fused) {
    if ((rc = do_reduce_apply(h, agent, 1, dp.out, dp.n_critic))) return rc;
  } else {
    if ((rc = do_reduce(h, agent, 1))) return rc;
    if ((rc = do_apply(h, agent, 1, false, 1.0f))) return rc;
  }
  if ((rc = do_actor_grad(h, agent, idx, u_act, false, pre, pre_next, pre_idx))) return rc;
  if (fused) {
    if ((rc = do_reduce_apply(h, agent, 0, dp.out ? dp.out + dp.n_critic : nullptr, dp.n_actor))) return rc;
  } else {
    if ((rc = do_reduce(h, agent, 0))) return rc;
    if ((rc = do_apply(h, agent, 0, false, 1.0f))) return rc;
  }
  return 0;
}

// ---- throughput mode: every agent's critic and actor gradients
// from the round-start parameters (one launch each), then every optimizer
// step (clip + Adam + Polyak) in one launch.  NOT the reference's order
// (maddpg.py:188-194, train.py:160-161): labelled, opt-in.
// the fast kernels serve every agent: all agents' critic (actor) steps in ONE launch
bool tp_fast(const mdp_handle* h) {
  if (h->general_grads) return false;
  for (int i = 0; i < h->cfg.n_agents; ++i)
    if (!grads_r_ok(h->L.topo, i)) return false;
  return true;
}

// otherwise the general kernels run one launch per agent and step kind
bool tp_ok(const mdp_handle* h) {
  if (!h->fused_apply) return false;
  for (int i = 0; i < h->cfg.n_agents; ++i)
    if (!reduce_apply_ok(h, i, 0) || !reduce_apply_ok(h, i, 1)) return false;
  return 2 * h->cfg.n_agents <= MDP_RA_BATCH_MAX;
}

// the optimizer step of (agent, net) in throughput mode: its own block of
// partials / stats, Polyak of its own net (both nets stepped in this launch),
// agent 0's actor step advances the noise counter by n (every agent used
// upd_ctr + agent)
FusedApplyArgs tp_args(mdp_handle* h, int agent, int net) {
  const int64_t nwg = h->L.nwg;
  FusedApplyArgs f = fused_args_for(h, agent, net, true);
  f.ap.slab = net ? h->slab_c + agent * nwg * h->L.slab_c : h->slab_a + agent * nwg * h->L.slab_a;
  f.ap.slab_stat = (net ? h->stat_c : h->stat_a) + agent * nwg * 8;
  f.ap.y = h->y + (int64_t)agent * h->cfg.batch_size;
  f.ap.polyak = 1;
  for (int t = 0; t < 7; ++t) f.ap.oblk[t] = 0;
  f.ap.bump_ctr = (net == 0 && agent == 0) ? h->cfg.n_agents : 0;
  return f;
}

// four device lists of the 2n steps: [0, 2n) fused (single GPU), [2n, 4n)
// reduce-only, [4n, 6n) step from the all-reduced grad[] scaled by 1/G,
// [6n, 8n) reduce + xGMI exchange + step (phase 3)
int tp_setup(mdp_handle* h) {
  if (h->tp_list) {
    (void)hipFree(h->tp_list);
    h->tp_list = nullptr;
  }
  const int n = h->cfg.n_agents;
  std::vector<FusedApplyArgs> list;
  RaBatch* rbs[4] = {&h->tp_batch, &h->tp_reduce, &h->tp_step, &h->tp_xchg};
  for (int ph = 0; ph < 4; ++ph) {
    RaBatch& rb = *rbs[ph];
    rb.count = 2 * n;
    rb.narrow = h->L.nwg <= 64 ? 1 : 0;
    rb.wg_start[0] = 0;
    for (int i = 0; i < n; ++i)
      for (int net = 1; net >= 0; --net) {
        FusedApplyArgs f = tp_args(h, i, net);
        f.phase = ph;
        if (ph == 2) f.ap.scale = 1.0f / (float)h->dp_world;
        if (ph == 3) {
          if (h->p2p) set_xchg(h, f, i, net);
          else f.phase = 0;  // unused list
        }
        list.push_back(f);
        const int q = 2 * i + (1 - net);
        rb.wg_start[q + 1] = rb.wg_start[q] + mdp_ra_grid(f);
      }
  }
  for (int ph = 0; ph < 4; ++ph) {
    h->tp_host[ph].assign(list.begin() + 2 * n * ph, list.begin() + 2 * n * (ph + 1));
    // phase 1 (reduce only) never spins; the others need the whole batch co-resident
    h->tp_fits[ph] = ph == 1 || rbs[ph]->wg_start[2 * n] <= h->ra_batch_cap;
  }
  // the per-agent pairs of the general kernels (tp_round_general): shared
  // slabs, no Polyak, the LAST agent's actor step advancing the noise counter
  // by n (every gradient launch of the round read upd_ctr + agent before it)
  const int pair_phase[3] = {0, 1, 3};
  const size_t pair0 = list.size();
  for (int pp = 0; pp < 3; ++pp)
    for (int i = 0; i < n; ++i) {
      RaBatch& rb = h->tp_pair[pp][i];
      rb = RaBatch();
      rb.count = 2;
      rb.narrow = h->L.nwg <= 64 ? 1 : 0;
      for (int k = 0; k < 2; ++k) {
        const int net = 1 - k;  // critic, then actor
        FusedApplyArgs f = tp_args(h, i, net);
        f.ap.slab = net ? h->slab_c : h->slab_a;
        f.ap.polyak = 0;
        f.ap.bump_ctr = (net == 0 && i == n - 1) ? n : 0;
        f.phase = pair_phase[pp];
        if (pp == 2) {
          if (h->p2p) set_xchg(h, f, i, net);
          else f.phase = 0;  // unused list
        }
        list.push_back(f);
        h->tp_pair_host[pp][i][k] = f;
        rb.wg_start[k + 1] = rb.wg_start[k] + mdp_ra_grid(f);
      }
      // + the draw workgroup; a reduce-only pass never spins
      h->tp_pair_fits[pp][i] = pp == 1 || rb.wg_start[2] + 1 <= h->ra_batch_cap;
    }
  HIPCHK(h, hipMalloc((void**)&h->tp_list, sizeof(FusedApplyArgs) * list.size()));
  HIPCHK(h, hipMemcpy(h->tp_list, list.data(), sizeof(FusedApplyArgs) * list.size(), hipMemcpyHostToDevice));
  for (int ph = 0; ph < 4; ++ph) rbs[ph]->list = h->tp_list + (int64_t)ph * 2 * n;
  for (int pp = 0; pp < 3; ++pp)
    for (int i = 0; i < n; ++i) h->tp_pair[pp][i].list = h->tp_list + pair0 + (int64_t)(pp * n + i) * 2;
  return 0;
}

int dp_allreduce_all(mdp_handle* h);
int launch_tp_batch(mdp_handle* h, int ph);

// every agent's gradients + every optimizer step; idx [n][B]; optional injected
// uniforms u_tgt [n][n][B][5] (agent, target actor j, row) and u_act [n][B][5]
// throughput-mode gradients on the fast kernels: every agent's critic (actor)
// step in ONE launch, workgroup -> (agent, row tile)
int tp_grads_fast(mdp_handle* h, const int32_t* idx, const float* u_tgt, const float* u_act, int32_t* pf_out) {
  const int n = h->cfg.n_agents;
  const int64_t nwg = h->L.nwg;
  int lds_c = 0;
  for (int i = 0; i < n; ++i) lds_c = std::max(lds_c, lds_critic_r_bytes(h->L.topo, i));
  {
    CriticArgs a;
    a.apre = nullptr;
    a.apre_rows = nullptr;
    a.u_act = nullptr;
    a.cpre = nullptr;
    a.cpre_rows = nullptr;
    a.cpre_prev = -1;
    a.pf_ctl = h->ctl;
    a.pf_out = pf_out;
    a.pf_count = pf_out ? n * h->cfg.batch_size : 0;
    a.topo = h->L.topo;
    a.agent = 0;
    a.B = h->cfg.batch_size;
    a.theta = h->theta;
    a.target = h->target;
    a.replay = h->replay;
    a.idx = idx;
    a.u_tgt = u_tgt;
    a.seed = h->cfg.seed;
    a.ctl = h->ctl;
    a.gamma = h->cfg.gamma;
    a.inv_b = 1.0f / (float)a.B;
    a.slab = h->slab_c;
    a.slab_stride = h->L.slab_c;
    a.slab_stat = h->stat_c;
    a.y_out = h->y;
    a.group = 0;
    a.multi = n;
    a.slab_agent_stride = nwg * h->L.slab_c;
    ProfScope p(h, MDP_K_CRITIC_GRAD);
    HIPCHK(h, mdp_launch_critic_grad_r(a, lds_c, h->stream));
  }
  {
    ActorArgs a;
    a.apre = nullptr;
    a.apre_rows = nullptr;
    a.cpre = nullptr;
    a.cpre_rows = nullptr;
    a.cpre_agent = -1;
    a.cpre_idx = nullptr;
    a.target = h->target;
    a.topo = h->L.topo;
    a.agent = 0;
    a.B = h->cfg.batch_size;
    a.theta = h->theta;
    a.replay = h->replay;
    a.idx = idx;
    a.u_act = u_act;
    a.seed = h->cfg.seed;
    a.ctl = h->ctl;
    a.neg_inv_b = -1.0f / (float)a.B;
    a.reg_scale = (float)(2.0 * (double)h->cfg.actor_reg / ((double)a.B * MDP_ACT_DIM));
    a.slab = h->slab_a;
    a.slab_stride = h->L.slab_a;
    a.slab_stat = h->stat_a;
    a.multi = n;
    a.slab_agent_stride = nwg * h->L.slab_a;
    ProfScope p(h, MDP_K_ACTOR_GRAD);
    HIPCHK(h, mdp_launch_actor_grad_r(a, lds_actor_r_bytes(h->L.topo), h->stream));
  }
  return 0;
}

// agent i's optimizer pair (critic_i, actor_i) in one launch when its grid is
// co-resident, else one launch per net; `piece`: agent i's B indices of the
// next round drawn on the side (halves in the per-net launches)
int launch_tp_pair(mdp_handle* h, int pp, int i, int32_t* piece) {
  const int B = h->cfg.batch_size;
  const int kind = pp == 1 ? MDP_K_REDUCE : MDP_K_REDUCE_APPLY;
  if (h->tp_pair_fits[pp][i]) {
    RaBatch rb = h->tp_pair[pp][i];
    if (piece) {
      rb.pf_out = piece;
      rb.pf_count = B;
      rb.pf_ctl = h->ctl;
    }
    ProfScope p(h, kind);
    HIPCHK(h, mdp_launch_reduce_apply_batch(rb, h->stream));
    return 0;
  }
  for (int k = 0; k < 2; ++k) {
    FusedApplyArgs f = h->tp_pair_host[pp][i][k];
    if (piece) {
      f.pf_out = piece + (k ? (B + 1) / 2 : 0);
      f.pf_count = k ? B - (B + 1) / 2 : (B + 1) / 2;
      f.pf_ctl = h->ctl;
    }
    ProfScope p(h, kind);
    HIPCHK(h, mdp_launch_reduce_apply(f, h->stream));
  }
  return 0;
}

// Throughput mode on the general kernels (H = 128, wide critics): agent by
// agent, the critic and actor gradients from the round-start parameters, then
// that agent's two optimizer steps (one launch) -- the partial-gradient slabs
// are consumed before the next agent's gradients overwrite them, so they stay
// the strict mode's size (L2 / MALL resident) instead of n per-agent blocks.
// No agent's gradient reads another agent's actor or critic (the critic input
// is the replay's actions), only the target actors, so the targets' Polyak is
// the one thing held back: one k_polyak over every target net after the last
// step.  The same arithmetic as one batch of every net (update_round_throughput).
// With RCCL: reduce-only pairs, ONE all-reduce of the whole gradient region,
// then the step pass (with Polyak) as before.  draw_out: the next round's n B
// indices, agent i's B in agent i's pair launch (MT19937 stream order).
int tp_round_general(mdp_handle* h, const int32_t* idx, const float* u_tgt, const float* u_act, int32_t* draw_out) {
  const int n = h->cfg.n_agents;
  const int64_t B = h->cfg.batch_size;
  const int pp = h->comm ? 1 : h->p2p ? 2 : 0;
  int rc;
  for (int i = 0; i < n; ++i) {
    const int32_t* ix = idx + i * B;
    const float* ut = u_tgt ? u_tgt + i * n * B * MDP_ACT_DIM : nullptr;
    const float* ua = u_act ? u_act + i * B * MDP_ACT_DIM : nullptr;
    if (h->grad_pair) {  // both gradient steps of agent i in one launch
      GradPairArgs g;
      g.c = critic_args(h, i, ix, ut, true, -1, nullptr, true);
      g.x = actor_args(h, i, ix, ua, true, false, -1, nullptr, true);
      const int lds = std::max(lds_critic_bytes(h->L.topo, g.c.group), lds_actor_bytes(h->L.topo));
      if (lds > MDP_LDS_BUDGET) return fail(h, "gradient pair does not fit in LDS");
      ProfScope p(h, MDP_K_CRITIC_GRAD);
      HIPCHK(h, mdp_launch_grad_pair(g, h->L.topo.H, lds, h->stream));
    } else {
      if ((rc = do_critic_grad(h, i, ix, ut, nullptr, true, false, nullptr, -1, 0, true))) return rc;
      if ((rc = do_actor_grad(h, i, ix, ua, true, false, -1, nullptr, true))) return rc;
    }
    if ((rc = launch_tp_pair(h, pp, i, draw_out ? draw_out + i * B : nullptr))) return rc;
  }
  if (h->comm) {  // data parallel over RCCL: ONE all-reduce of every net's gradient per round
    if ((rc = dp_allreduce_all(h))) return rc;
    ProfScope p(h, MDP_K_APPLY, h->tp_fits[2]);
    return launch_tp_batch(h, 2);
  }
  const ApplyArgs a = apply_args(h, 0, 0, 1.0f);
  HIPCHK(h, mdp_launch_polyak(h->target, h->theta, h->L.PT, a.pa, a.pb, h->ctl, h->stream));
  return 0;
}

// the optimizer steps of every net in one launch when the batch grid is
// co-resident (its chunk workgroups spin), else one launch per net (e.g. tag
// N=6 at H=128: ~1,350 chunk workgroups; each net's own grid fits)
int launch_tp_batch(mdp_handle* h, int ph) {
  const RaBatch* rbs[4] = {&h->tp_batch, &h->tp_reduce, &h->tp_step, &h->tp_xchg};
  if (h->tp_fits[ph]) {
    HIPCHK(h, mdp_launch_reduce_apply_batch(*rbs[ph], h->stream));
    return 0;
  }
  for (const FusedApplyArgs& f : h->tp_host[ph]) HIPCHK(h, mdp_launch_reduce_apply(f, h->stream));
  return 0;
}

// pf_out: the next round's draw in the fast critic launch; draw_out: ... in the
// general path's optimizer launches
int do_round_tp(mdp_handle* h, const int32_t* idx, const float* u_tgt, const float* u_act, int32_t* pf_out,
                int32_t* draw_out = nullptr) {
  // the general path draws in its pair launches; a pf_out handed here anyway is
  // filled there in the same MT19937 order (agent i's B at pf_out + i B)
  if (!tp_fast(h)) return tp_round_general(h, idx, u_tgt, u_act, draw_out ? draw_out : pf_out);
  const int rc = tp_grads_fast(h, idx, u_tgt, u_act, pf_out);
  if (rc) return rc;
  if (h->p2p) {  // data parallel over xGMI: reduce + exchange + step of every net, one launch
    ProfScope p(h, MDP_K_REDUCE_APPLY, h->tp_fits[3]);
    return launch_tp_batch(h, 3);
  }
  if (h->comm) {  // data parallel: ONE all-reduce of every net's gradient per round
    {
      ProfScope p(h, MDP_K_REDUCE, h->tp_fits[1]);
      const int rc = launch_tp_batch(h, 1);
      if (rc) return rc;
    }
    const int rc = dp_allreduce_all(h);
    if (rc) return rc;
    ProfScope p(h, MDP_K_APPLY, h->tp_fits[2]);
    return launch_tp_batch(h, 2);
  }
  ProfScope p(h, MDP_K_REDUCE_APPLY, h->tp_fits[0]);
  return launch_tp_batch(h, 0);
}

int set_ring(mdp_handle* h, int64_t len, int64_t next) {
  h->len = len;
  h->next = next;
  HIPCHK(h, mdp_launch_set_ring(h->ctl, len, next, h->stream));
  return 0;
}

}  // namespace

// ======================================================================= ABI
extern "C" {

int32_t mdp_abi_version(void) { return MDP_ABI_VERSION; }

int64_t mdp_arena_bytes(const mdp_config* cfg, int64_t* param_floats) {
  Layout L;
  std::string err;
  if (!build_layout(cfg, L, err)) return -1;
  if (param_floats) *param_floats = L.PT;
  return L.total;
}

int mdp_ra_plan(const mdp_config* cfg, int32_t cus, int32_t per_cu, int32_t* out) {
  Layout L;
  std::string err;
  if (!build_layout(cfg, L, err) || cus < 0 || per_cu < 0) return -1;
  int fallback = 0;
  for (int i = 0; i < cfg->n_agents; ++i)
    for (int net = 0; net < 2; ++net) {
      const int g = mdp_ra_grid_of(L.topo, i, net);
      const bool ok = mdp_ra_fits(L.topo, i, net, cus * per_cu);
      if (out) out[2 * i + net] = ok ? g : -g;
      fallback += ok ? 0 : 1;
    }
  return fallback;
}

int mdp_create(const mdp_config* cfg, void* arena_dev, int64_t arena_bytes, void* hip_stream, mdp_handle** out) {
  if (!out) return -1;
  *out = nullptr;
  mdp_handle* h = new mdp_handle();
  std::string err;
  if (!build_layout(cfg, h->L, err)) {
    h->err = err;
    *out = h;
    return -1;
  }
  h->cfg = *cfg;
  {
    const char* g = getenv("MDP_GENERAL_GRADS");
    h->general_grads = g && g[0] == '1';
    const char* u = getenv("MDP_UNFUSED_APPLY");
    h->fused_apply = !(u && u[0] == '1');
    const char* rd = getenv("MDP_ROLLOUT_DRAW");
    h->rollout_draw = !(rd && rd[0] == '0');
    const char* da = getenv("MDP_DRAW_AHEAD");
    h->draw_ahead = !(da && da[0] == '0');
    const char* gp = getenv("MDP_GRAD_PAIR");
    h->grad_pair = !(gp && gp[0] == '0');
    const char* ap = getenv("MDP_ACTOR_PRE");
    h->actor_pre = !(ap && ap[0] == '0');
    const char* cp = getenv("MDP_CRITIC_PRE");
    h->critic_pre = !(cp && cp[0] == '0');
  }
  if (!arena_dev || arena_bytes < h->L.total) {
    h->err = "arena missing or too small";
    *out = h;
    return -1;
  }
  *out = h;
  HIPCHK(h, hipGetDevice(&h->device));
  if (need_dev(h, arena_dev, h->L.total, "mdp_create", "arena_dev", false)) return -1;
  {
    int cus = 0, per = 0, per_b = 0;
    HIPCHK(h, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
    HIPCHK(h, mdp_ra_occupancy(&per));
    HIPCHK(h, mdp_ra_batch_occupancy(&per_b));
    h->ra_cap = cus * per;
    h->ra_batch_cap = cus * per_b;
    // a spinning grid with scratch may not be co-resident (scratch-slot
    // throttling): no fused / exchanging launch then -- every step runs as the
    // non-spinning k_reduce + k_apply pair and the xGMI set-up is refused
    int scratch = 0;
    HIPCHK(h, mdp_spin_kernels_scratch(&scratch));
    if (scratch > 0) h->ra_cap = h->ra_batch_cap = 0;
  }
  if (hip_stream) {
    h->stream = (hipStream_t)hip_stream;
  } else {
    HIPCHK(h, hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->own_stream = true;
  }
  h->arena = (char*)arena_dev;
  auto R = [&](int r) { return (void*)(h->arena + h->L.off[r]); };
  h->theta = (float*)R(MDP_R_THETA);
  h->target = (float*)R(MDP_R_TARGET);
  h->m = (float*)R(MDP_R_ADAM_M);
  h->v = (float*)R(MDP_R_ADAM_V);
  h->grad = (float*)R(MDP_R_GRAD);
  h->replay = (float*)R(MDP_R_REPLAY);
  h->index = (int32_t*)R(MDP_R_INDEX);
  h->stats = (double*)R(MDP_R_STATS);
  h->eplog = (float*)R(MDP_R_EPLOG);
  h->beta = (float*)R(MDP_R_BETA);
  h->ctl = (Ctl*)R(MDP_R_CTL);
  {
    const int E = cfg->num_envs, ne = h->L.n_ent, n = cfg->n_agents;
    char* p = (char*)R(MDP_R_ENV);
    h->pos = (float*)p;
    p += 4 * (int64_t)E * ne * 2;
    h->vel = (float*)p;
    p += 4 * (int64_t)E * ne * 2;
    h->goal = (int32_t*)p;
    p += 4 * (int64_t)E;
    h->ep_step = (int32_t*)p;
    p += 4 * (int64_t)E;
    h->ep_rew = (float*)p;
    (void)n;
  }
  {
    char* p = (char*)R(MDP_R_SLAB);
    const int64_t nwg = h->L.nwg, na = cfg->n_agents;
    h->slab_c = (float*)p;
    p += 4 * na * nwg * h->L.slab_c;
    h->slab_a = (float*)p;
    p += 4 * na * nwg * h->L.slab_a;
    p = (char*)(((uintptr_t)p + 7) & ~uintptr_t(7));
    h->stat_c = (double*)p;
    p += 8 * 8 * na * nwg;
    h->stat_a = (double*)p;
    p += 8 * 8 * na * nwg;
    h->y = (double*)p;
    p += 8 * na * (int64_t)cfg->batch_size + 256;
    p = (char*)(((uintptr_t)p + 255) & ~uintptr_t(255));
    h->ra_ctr = (uint32_t*)p;
    h->ra_part = (uint64_t*)(p + (int64_t)MDP_MAX_AGENTS * 2 * 8 * 128);
    h->apre = (float*)(p + mdp_ra_sync_bytes());
    h->cpre = h->apre + (int64_t)nwg * 16 * MDP_APRE_W;
    h->apre_rows = h->cpre + (int64_t)nwg * 16 * MDP_CPRE_W;
    h->cpre_rows = h->apre_rows + (int64_t)nwg * 16 * h->L.topo.row_stride;
  }
  HIPCHK(h, hipMemsetAsync(h->arena, 0, h->L.total, h->stream));
  std::vector<float> beta(8 * cfg->n_agents);
  for (int i = 0; i < cfg->n_agents * 2; ++i) {  // TF1: beta powers start at beta
    beta[4 * i] = beta[4 * i + 2] = cfg->adam_b1;
    beta[4 * i + 1] = beta[4 * i + 3] = cfg->adam_b2;
  }
  HIPCHK(h, hipMemcpyAsync(h->beta, beta.data(), 4 * beta.size(), hipMemcpyHostToDevice, h->stream));
  Ctl c;
  std::memset(&c, 0, sizeof(c));
  py_seed_state(0, c.mt, &c.mt_pos);
  HIPCHK(h, hipMemcpyAsync(h->ctl, &c, sizeof(c), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->err.clear();
  h->ready = true;
  return 0;
}

int mdp_destroy(mdp_handle* h) {
  if (!h) return 0;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->tp_list) (void)hipFree(h->tp_list);
  for (int k = 0; k < MDP_K_COUNT; ++k)
    for (auto e : h->ev[k]) (void)hipEventDestroy(e);
  if (h->round_exec) (void)hipGraphExecDestroy(h->round_exec);
  if (h->comm) (void)rccl().destroy(h->comm);
  xgmi_release(h);
  for (auto& kv : h->step_exec) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : h->multi_exec) (void)hipGraphExecDestroy(kv.second);
  if (h->round_graph) (void)hipGraphDestroy(h->round_graph);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

const char* mdp_last_error(const mdp_handle* h) { return h ? h->err.c_str() : "null handle"; }
void* mdp_stream(mdp_handle* h) { return h ? (void*)h->stream : nullptr; }

int mdp_synchronize(mdp_handle* h) {
  MDP_NEED(h);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint32_t fault = 0;
  HIPCHK(h, hipMemcpy(&fault, &h->ctl->fault, sizeof(fault), hipMemcpyDeviceToHost));
  if (fault == 1) return fail(h, "device fault: a tensor-norm handshake timed out (k_reduce_apply)");
  if (fault == 2) return fail(h, "device fault: a data-parallel peer did not reach the xGMI exchange within 30 s");
  if (fault) return fail(h, "device fault");
  return 0;
}

int mdp_region(const mdp_handle* h, int32_t region, int64_t* offset, int64_t* bytes) {
  if (unusable(h) || region < 0 || region >= MDP_R_COUNT) return -1;
  if (offset) *offset = h->L.off[region];
  if (bytes) *bytes = h->L.bytes[region];
  return 0;
}

int mdp_tensor(const mdp_handle* h, int32_t agent, int32_t net, int32_t t, mdp_tensor_info* out) {
  if (unusable(h) || agent < 0 || agent >= h->cfg.n_agents || t < 0 || t > 5 || !out) return -1;
  const NDesc& d = net ? h->L.topo.ag[agent].critic : h->L.topo.ag[agent].actor;
  out->offset = d.t[t].off;
  logical_shape(h, d, t, &out->rows, &out->cols);
  out->dev_rows = d.t[t].rows;
  out->dev_cols = d.t[t].cols;
  return 0;
}

int mdp_row_layout(const mdp_handle* h, int32_t agent, int32_t out6[6]) {
  if (unusable(h) || agent < 0 || agent >= h->cfg.n_agents) return -1;
  const ADesc& a = h->L.topo.ag[agent];
  out6[0] = a.obs_off;
  out6[1] = a.act_off;
  out6[2] = a.nobs_off;
  out6[3] = a.rew_off;
  out6[4] = a.done_off;
  out6[5] = h->L.topo.row_stride;
  return 0;
}

int mdp_set_params(mdp_handle* h, int32_t agent, int32_t which, const float* src, int64_t n) {
  if (bad_agent(h, agent)) return -1;
  int region, net;
  if (region_for(which, &region, &net)) return fail(h, "bad param set id");
  const NDesc& d = net_of(h, agent, net);
  if (n != net_floats(h, d)) return fail(h, "param count mismatch");
  std::vector<float> buf(d.size, 0.f);  // padded entries stay zero
  int64_t s = 0;
  for (int t = 0; t < 6; ++t) {
    int rows, cols;
    logical_shape(h, d, t, &rows, &cols);
    for (int r = 0; r < rows; ++r, s += cols)
      std::memcpy(buf.data() + (d.t[t].off - d.off) + (int64_t)r * d.t[t].cols, src + s, 4 * (int64_t)cols);
  }
  float* dst = (float*)(h->arena + h->L.off[region]) + d.off;
  HIPCHK(h, hipMemcpyAsync(dst, buf.data(), 4 * buf.size(), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_get_params(mdp_handle* h, int32_t agent, int32_t which, float* dst, int64_t n) {
  if (bad_agent(h, agent)) return -1;
  int region, net;
  if (region_for(which, &region, &net)) return fail(h, "bad param set id");
  const NDesc& d = net_of(h, agent, net);
  if (n != net_floats(h, d)) return fail(h, "param count mismatch");
  std::vector<float> buf(d.size);
  const float* src = (const float*)(h->arena + h->L.off[region]) + d.off;
  HIPCHK(h, hipMemcpyAsync(buf.data(), src, 4 * buf.size(), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  int64_t s = 0;
  for (int t = 0; t < 6; ++t) {
    int rows, cols;
    logical_shape(h, d, t, &rows, &cols);
    for (int r = 0; r < rows; ++r, s += cols)
      std::memcpy(dst + s, buf.data() + (d.t[t].off - d.off) + (int64_t)r * d.t[t].cols, 4 * (int64_t)cols);
  }
  return 0;
}

int mdp_get_beta_powers(mdp_handle* h, int32_t agent, int32_t net, float out2[2]) {
  if (bad_agent(h, agent)) return -1;
  HIPCHK(h, hipMemcpyAsync(out2, h->beta + agent * 8 + (net ? 4 : 0), 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_set_beta_powers(mdp_handle* h, int32_t agent, int32_t net, const float in2[2]) {
  if (bad_agent(h, agent)) return -1;
  HIPCHK(h, hipMemcpyAsync(h->beta + agent * 8 + (net ? 4 : 0), in2, 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

// ----------------------------------------------------------------- replay
int64_t mdp_buffer_len(mdp_handle* h) { return unusable(h) ? -1 : h->len; }

int mdp_buffer_add_rows(mdp_handle* h, const float* rows_dev, int64_t rows) {
  MDP_NEED(h);
  if (rows < 0) return fail(h, "negative row count");
  if (rows == 0) return 0;
  MDP_DEV(h, rows_dev, rows * 4 * h->L.topo.row_stride, "mdp_buffer_add_rows", false);
  const int64_t cap = h->cfg.capacity;
  // more rows than the ring holds: only the last `cap` survive (earlier ones
  // would be overwritten), which also keeps every destination row unique
  const int64_t skip = rows > cap ? rows - cap : 0;
  const int64_t start = (h->next + skip) % cap;
  HIPCHK(h, mdp_launch_put_rows(h->replay, h->L.topo.row_stride, cap, start,
                                rows_dev + skip * h->L.topo.row_stride, rows - skip, h->stream));
  return set_ring(h, std::min(cap, h->len + rows), (h->next + rows) % cap);
}

int mdp_buffer_put_agent(mdp_handle* h, int32_t agent, const int64_t* pos_dev, const float* cols_dev, int64_t rows) {
  if (bad_agent(h, agent)) return -1;
  if (rows <= 0) return 0;
  MDP_DEV(h, pos_dev, rows * 8, "mdp_buffer_put_agent", false);
  MDP_DEV(h, cols_dev, rows * 4 * (2 * h->L.topo.ag[agent].obs_dim + MDP_ACT_DIM + 2), "mdp_buffer_put_agent", false);
  HIPCHK(h, mdp_launch_put_agent(h->replay, h->L.topo.row_stride, h->L.topo.ag[agent], pos_dev, cols_dev, rows,
                                 h->stream));
  return 0;
}

int mdp_buffer_set_len(mdp_handle* h, int64_t len, int64_t next_idx) {
  MDP_NEED(h);
  if (len < 0 || len > h->cfg.capacity || next_idx < 0 || next_idx >= h->cfg.capacity)
    return fail(h, "ring state out of range");
  return set_ring(h, len, next_idx);
}

int mdp_seed_py_random(mdp_handle* h, uint64_t seed) {
  MDP_NEED(h);
  Ctl c;
  py_seed_state(seed, c.mt, &c.mt_pos);
  HIPCHK(h, hipMemcpyAsync(h->ctl->mt, c.mt, sizeof(c.mt) + sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_set_rng_state(mdp_handle* h, const uint32_t* st) {
  MDP_NEED(h);
  if (!st) return fail(h, "null RNG state");
  if (st[624] > 624) return fail(h, "MT position out of range");
  uint32_t buf[625];
  std::memcpy(buf, st, sizeof(buf));
  HIPCHK(h, hipMemcpyAsync(h->ctl->mt, buf, sizeof(buf), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_get_rng_state(mdp_handle* h, uint32_t* st) {
  MDP_NEED(h);
  if (!st) return fail(h, "null RNG state");
  HIPCHK(h, hipMemcpyAsync(st, h->ctl->mt, 625 * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_make_index(mdp_handle* h, int32_t count, int32_t* idx_dev) {
  MDP_NEED(h);
  if (count < 0) return fail(h, "negative count");
  if (count == 0) return 0;
  MDP_DEV(h, idx_dev, 4 * (int64_t)count, "mdp_make_index", false);
  return launch_make_index(h, count, idx_dev);
}

int mdp_sample_rows(mdp_handle* h, const int32_t* idx_dev, int32_t count, float* out_dev) {
  MDP_NEED(h);
  if (count <= 0) return 0;
  MDP_DEV(h, idx_dev, 4 * (int64_t)count, "mdp_sample_rows", false);
  MDP_DEV(h, out_dev, 4 * (int64_t)count * h->L.topo.row_stride, "mdp_sample_rows", false);
  ProfScope p(h, MDP_K_GATHER, false);
  HIPCHK(h, mdp_launch_gather(h->replay, h->L.topo.row_stride, idx_dev, count, out_dev, h->stream));
  return 0;
}

// ---------------------------------------------------------------- policies
int mdp_act(mdp_handle* h, int32_t agent, int32_t target, const float* obs_dev, float* act_dev, int32_t rows,
            const float* u_dev) {
  if (bad_agent(h, agent)) return -1;
  if (rows <= 0) return 0;
  const ADesc& ag = h->L.topo.ag[agent];
  MDP_DEV(h, obs_dev, 4 * (int64_t)rows * ag.obs_dim, "mdp_act", false);
  MDP_DEV(h, act_dev, 4 * (int64_t)rows * MDP_ACT_DIM, "mdp_act", false);
  MDP_DEV(h, u_dev, 4 * (int64_t)rows * MDP_ACT_DIM, "mdp_act", true);
  EvalArgs a;
  a.P = target ? h->target : h->theta;
  a.net = ag.actor;
  a.in = ag.obs_dim;
  a.rows = rows;
  a.x = obs_dev;
  a.out = act_dev;
  a.gumbel = 1;
  a.u = u_dev;
  a.seed = h->cfg.seed;
  a.stream = 0x40000u | (uint32_t)(agent << 1) | (uint32_t)(target ? 1 : 0);
  a.ctr = h->act_ctr++;
  HIPCHK(h, mdp_launch_eval(a, h->L.topo.H, lds_eval_bytes(a.in, h->L.topo.H), h->stream));
  return 0;
}

int mdp_actor_logits(mdp_handle* h, int32_t agent, int32_t target, const float* obs_dev, float* logits_dev,
                     int32_t rows) {
  if (bad_agent(h, agent)) return -1;
  if (rows <= 0) return 0;
  const ADesc& ag = h->L.topo.ag[agent];
  MDP_DEV(h, obs_dev, 4 * (int64_t)rows * ag.obs_dim, "mdp_actor_logits", false);
  MDP_DEV(h, logits_dev, 4 * (int64_t)rows * MDP_ACT_DIM, "mdp_actor_logits", false);
  EvalArgs a;
  a.P = target ? h->target : h->theta;
  a.net = ag.actor;
  a.in = ag.obs_dim;
  a.rows = rows;
  a.x = obs_dev;
  a.out = logits_dev;
  a.gumbel = 0;
  a.u = nullptr;
  a.seed = h->cfg.seed;
  a.stream = 0;
  a.ctr = 0;
  HIPCHK(h, mdp_launch_eval(a, h->L.topo.H, lds_eval_bytes(a.in, h->L.topo.H), h->stream));
  return 0;
}

int mdp_q_values(mdp_handle* h, int32_t agent, int32_t target, const float* x_dev, float* q_dev, int32_t rows) {
  if (bad_agent(h, agent)) return -1;
  if (rows <= 0) return 0;
  const ADesc& ag = h->L.topo.ag[agent];
  MDP_DEV(h, x_dev, 4 * (int64_t)rows * ag.cin, "mdp_q_values", false);
  MDP_DEV(h, q_dev, 4 * (int64_t)rows, "mdp_q_values", false);
  EvalArgs a;
  a.P = target ? h->target : h->theta;
  a.net = ag.critic;
  a.in = ag.cin;
  a.rows = rows;
  a.x = x_dev;
  a.out = q_dev;
  a.gumbel = 0;
  a.u = nullptr;
  a.seed = h->cfg.seed;
  a.stream = 0;
  a.ctr = 0;
  HIPCHK(h, mdp_launch_eval(a, h->L.topo.H, lds_eval_bytes(a.in, h->L.topo.H), h->stream));
  return 0;
}

// ---------------------------------------------------------------- training
int mdp_update_gate(mdp_handle* h, int64_t t) {
  MDP_NEED(h);
  if (h->len < (int64_t)h->cfg.batch_size * h->cfg.max_episode_len) return 1;  // maddpg.py:162-163
  if (t % 100 != 0) return 1;                                                   // maddpg.py:164-165
  return 0;
}

int mdp_update(mdp_handle* h, int32_t agent, const int32_t* idx_dev, const float* u_tgt_dev, const float* u_act_dev) {
  if (bad_agent(h, agent)) return -1;
  const int64_t B = h->cfg.batch_size, n = h->cfg.n_agents;
  MDP_DEV(h, idx_dev, 4 * B, "mdp_update", true);
  MDP_DEV(h, u_tgt_dev, 4 * n * B * MDP_ACT_DIM, "mdp_update", true);
  MDP_DEV(h, u_act_dev, 4 * B * MDP_ACT_DIM, "mdp_update", true);
  const int32_t* idx = idx_dev;
  if (!idx) {
    int32_t* slot = h->index + (int64_t)agent * h->cfg.batch_size;
    int rc = launch_make_index(h, h->cfg.batch_size, slot);
    if (rc) return rc;
    idx = slot;
  }
  return do_update(h, agent, idx, u_tgt_dev, u_act_dev);
}

int mdp_agent_update(mdp_handle* h, int32_t agent, int64_t t, const int32_t* idx_dev, const float* u_dev,
                     double stats_out[6]) {
  if (unusable(h) || !stats_out) return -1;
  if (bad_agent(h, agent)) return -1;
  if (mdp_update_gate(h, t)) return 1;
  MDP_DEV(h, u_dev, 4 * (int64_t)(h->cfg.n_agents + 1) * h->cfg.batch_size * MDP_ACT_DIM, "mdp_agent_update", true);
  const float* u_tgt = u_dev;
  const float* u_act = u_dev ? u_dev + (int64_t)h->cfg.n_agents * h->cfg.batch_size * MDP_ACT_DIM : nullptr;
  const int rc = mdp_update(h, agent, idx_dev, u_tgt, u_act);
  if (rc) return rc;
  return mdp_get_stats(h, agent, stats_out);
}

// One strict round.  Agent i's critic step is split around agent i-1's update
// when critic_pre_ok: its independent part rides in i-1's actor launch.
// carry_in: the previous round's last actor launch already did agent 0's part
// (rounds of one training step, same replay contents); next_idx: the next
// round's indices, if drawn by now (the prefetch in agent 0's critic launch),
// lets this round's last actor launch do the next round's agent-0 part.
// Returns in *carry_out whether it did.
// draw_out: the next round's n*B indices drawn in 2n pieces by the round's
// optimizer launches (configurations without the fast critic kernel's
// prefetch; only where every step is the one-launch fused kind)
// ahead: the draw runs one agent ahead instead -- agent i's launches draw
// agent i+1's B indices of THIS round into idx (which the caller then owns),
// the last agent's the next round's agent 0 into pf_out (ahead 1: in the fast
// critic launches) or draw_out (ahead 2: in the optimizer launches), if any:
// the MT19937 stream order of the reference's per-agent make_index calls
// (maddpg.py:173), with only agent 0's B of a step's first round left to the
// rollout's draw workgroup
static int round_updates(mdp_handle* h, const int32_t* idx, int32_t* pf_out = nullptr, bool carry_in = false,
                         const int32_t* next_idx = nullptr, bool* carry_out = nullptr, int32_t* draw_out = nullptr,
                         int ahead = 0) {
  const int n = h->cfg.n_agents, B = h->cfg.batch_size;
  if (carry_out) *carry_out = false;
  if (h->update_mode == 1) return do_round_tp(h, idx, nullptr, nullptr, pf_out, draw_out);
  const int nb = n * B, piece = (nb + 2 * n - 1) / (2 * n);
  // the next round's draw (pf_out) in per-agent pieces, agent i's B indices in
  // agent i's critic launch -- the stream order of one n B draw (every launch
  // continues the MT19937 state in Ctl) -- when every critic launch is a fast
  // one; one n B draw in agent 0's launch made that launch the round's
  // longest (rocprof 10.1 vs 9.2 us)
  bool pieces = ahead == 1 || (ahead == 0 && pf_out != nullptr && !h->general_grads);
  for (int i = 0; i < n && pieces && ahead == 0; ++i) pieces = grads_r_ok(h->L.topo, i);
  int32_t* cur = const_cast<int32_t*>(idx);
  int rc = 0;
  for (int i = 0; i < n && !rc; ++i) {
    DrawPieces dp;
    if (pieces) dp.n_grad = B;
    if (ahead == 2) {
      dp.out = i + 1 < n ? cur + (int64_t)(i + 1) * B : draw_out;
      if (dp.out) {
        dp.n_critic = (B + 1) / 2;
        dp.n_actor = B - dp.n_critic;
      }
    } else if (draw_out) {
      const int o = std::min(nb, 2 * i * piece);
      dp.out = draw_out + o;
      dp.n_critic = std::min(piece, nb - o);
      dp.n_actor = std::min(piece, nb - o - dp.n_critic);
    }
    const int post_prev = i > 0 ? (critic_pre_ok(h, i - 1, i) ? i - 1 : -1) : (carry_in ? n - 1 : -1);
    int pre_next = -1;
    const int32_t* pre_idx = nullptr;
    if (i + 1 < n && critic_pre_ok(h, i, i + 1)) {
      pre_next = i + 1;
      pre_idx = idx + (int64_t)(i + 1) * B;
    } else if (i + 1 == n && next_idx && critic_pre_ok(h, n - 1, 0)) {
      pre_next = 0;
      pre_idx = next_idx;
      if (carry_out) *carry_out = true;
    }
    int32_t* pf_i = ahead == 1 ? (i + 1 < n ? cur + (int64_t)(i + 1) * B : pf_out)
                    : pieces        ? pf_out + (int64_t)i * B
                                    : (i == 0 ? pf_out : nullptr);
    rc = do_update(h, i, idx + (int64_t)i * B, nullptr, nullptr, pf_i, post_prev, pre_next, pre_idx, dp);
  }
  return rc;
}

// can the round's optimizer launches draw the next round's indices (all fused)?
static bool draw_in_ra_ok(const mdp_handle* h) {
  if (!h->fused_apply || h->comm) return false;
  for (int i = 0; i < h->cfg.n_agents; ++i)
    if (!reduce_apply_ok(h, i, 0) || !reduce_apply_ok(h, i, 1)) return false;
  return true;
}

// can agent 0's critic kernel draw the next round's indices on the side?
static bool prefetch_ok(const mdp_handle* h) {
  return !h->general_grads && grads_r_ok(h->L.topo, 0) && h->cfg.n_agents * h->cfg.batch_size <= 4096;
}

static int round_launches(mdp_handle* h) {
  const int n = h->cfg.n_agents, B = h->cfg.batch_size;
  int rc = launch_make_index(h, n * B, h->index);
  if (rc) return rc;
  return round_updates(h, h->index);
}

static bool any_prof(const mdp_handle* h) {
  for (int k = 0; k < MDP_K_COUNT; ++k)
    if (h->prof_on[k]) return true;
  return false;
}

// Every argument of the round's kernels is invariant (round-varying scalars --
// replay length, MT19937 state, noise counter -- are read from the device
// control block), so the round is captured once and replayed with one
// hipGraphLaunch.  Per-kernel event profiling runs the eager path.
int mdp_update_round(mdp_handle* h) {
  MDP_NEED(h);
  if (h->len <= 0) return fail(h, "update round on an empty replay buffer");
  if (!h->graphs || any_prof(h) || h->eager_rounds < 1) {
    ++h->eager_rounds;  // the first round runs eagerly (one-time kernel attribute setup)
    return round_launches(h);
  }
  if (!h->round_exec) {
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    h->capturing = true;
    const int rc = round_launches(h);
    h->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return fail(h, "hipStreamEndCapture", e);
    h->round_graph = g;
    HIPCHK(h, hipGraphInstantiate(&h->round_exec, g, nullptr, nullptr, 0));
  }
  HIPCHK(h, hipGraphLaunch(h->round_exec, h->stream));
  return 0;
}

int mdp_grad_variant(mdp_handle* h, int32_t agent) {
  if (unusable(h) || agent < 0 || agent >= h->cfg.n_agents) return -1;
  return (!h->general_grads && grads_r_ok(h->L.topo, agent)) ? 1 : 0;
}

int mdp_dp_unique_id(uint8_t* out128) {
  if (!out128 || !rccl().ok) return -1;
  ncclUniqueId id;
  if (rccl().get_id(&id) != ncclSuccess) return -1;
  std::memcpy(out128, &id, sizeof(id));
  return 0;
}

int mdp_dp_init(mdp_handle* h, const uint8_t* id128, int32_t world, int32_t rank) {
  if (unusable(h) || !id128) return -1;
  if (h->update_mode != 0) return fail(h, "join data parallelism before choosing the throughput mode");
  if (h->p2p || h->xbuf) return fail(h, "mdp_dp_init: the xGMI exchange is already set up");
  if (!rccl().ok) return fail(h, "librccl.so.1 could not be loaded");
  if (world < 1 || rank < 0 || rank >= world) return fail(h, "mdp_dp_init: bad world/rank");
  if (h->comm) return fail(h, "mdp_dp_init: already initialised");
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  HIPCHK(h, hipSetDevice(h->device));
  const ncclResult_t r = rccl().init_rank(&h->comm, world, id, rank);
  if (r != ncclSuccess) {
    h->comm = nullptr;
    h->err = std::string("ncclCommInitRank: ") + rccl().err(r);
    return -1;
  }
  h->dp_world = world;
  const char* g = getenv("MDP_DP_GRAPHS");
  h->dp_graphs = g && g[0] == '1';
  // drop graphs captured without the collectives
  for (auto& kv : h->step_exec) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : h->multi_exec) (void)hipGraphExecDestroy(kv.second);
  h->step_exec.clear();
  h->multi_exec.clear();
  if (h->round_exec) {
    (void)hipGraphExecDestroy(h->round_exec);
    h->round_exec = nullptr;
  }
  if (h->round_graph) {
    (void)hipGraphDestroy(h->round_graph);
    h->round_graph = nullptr;
  }
  return 0;
}

static void drop_graphs(mdp_handle* h);

int mdp_dp_xgmi_open(mdp_handle* h, int32_t world, int32_t rank, uint8_t* handle_out) {
  if (unusable(h) || !handle_out) return -1;
  if (h->update_mode != 0) return fail(h, "join data parallelism before choosing the throughput mode");
  if (h->comm) return fail(h, "mdp_dp_xgmi_open: an RCCL communicator is already set up");
  if (h->xbuf) return fail(h, "mdp_dp_xgmi_open: already open");
  if (world < 2 || world > MDP_XCH_MAXW || rank < 0 || rank >= world)
    return fail(h, "mdp_dp_xgmi_open: world must be 2..8 and 0 <= rank < world");
  if (h->general_grads || !h->fused_apply) return fail(h, "the xGMI exchange needs the fused optimizer kernel");
  for (int i = 0; i < h->cfg.n_agents; ++i)
    for (int net = 0; net < 2; ++net) {
      if (!reduce_apply_ok(h, i, net)) return fail(h, "the xGMI exchange needs the fused optimizer kernel");
    }
  HIPCHK(h, hipSetDevice(h->device));
  const int64_t bytes = mdp_xch_bytes(world, h->L.PT);
  void* p = nullptr;
  HIPCHK(h, hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached));
  h->xbuf = (uint64_t*)p;
  HIPCHK(h, hipMemset(p, 0, (size_t)bytes));
  HIPCHK(h, hipMalloc((void**)&h->x_probe, 2 * sizeof(uint32_t)));
  HIPCHK(h, hipDeviceSynchronize());
  hipIpcMemHandle_t mh;
  HIPCHK(h, hipIpcGetMemHandle(&mh, p));
  static_assert(sizeof(mh) == MDP_XGMI_HANDLE_BYTES, "IPC handle size");
  std::memcpy(handle_out, &mh, sizeof(mh));
  h->x_world = world;
  h->x_rank = rank;
  return 0;
}

int mdp_dp_xgmi_connect(mdp_handle* h, const uint8_t* handles) {
  if (unusable(h) || !handles) return -1;
  if (!h->xbuf) return fail(h, "mdp_dp_xgmi_connect: call mdp_dp_xgmi_open first");
  if (!h->x_opened.empty()) return fail(h, "mdp_dp_xgmi_connect: already connected");
  const int W = h->x_world, r = h->x_rank;
  XchgDesc xd;
  std::memset(&xd, 0, sizeof(xd));
  xd.world = W;
  xd.rank = r;
  xd.pt = h->L.PT + MDP_XCH_PROBE;
  h->x_opened.assign(W, nullptr);
  for (int q = 0; q < W; ++q) {
    void* base = h->xbuf;
    if (q != r) {
      hipIpcMemHandle_t mh;
      std::memcpy(&mh, handles + (int64_t)q * MDP_XGMI_HANDLE_BYTES, sizeof(mh));
      const hipError_t e = hipIpcOpenMemHandle(&base, mh, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) return fail(h, "hipIpcOpenMemHandle", e);
      h->x_opened[q] = base;
    }
    xd.data[q] = (uint64_t*)base;
  }
  HIPCHK(h, hipMalloc((void**)&h->xd_dev, sizeof(XchgDesc)));
  HIPCHK(h, hipMemcpy(h->xd_dev, &xd, sizeof(XchgDesc), hipMemcpyHostToDevice));
  return 0;
}

int mdp_dp_xgmi_probe(mdp_handle* h, int32_t* mismatches) {
  if (unusable(h)) return -1;
  if (!h->xd_dev) return fail(h, "mdp_dp_xgmi_probe: not connected");
  const int nchunk = MDP_XCH_PROBE / 256;
  HIPCHK(h, hipMemsetAsync(h->x_probe, 0, 2 * sizeof(uint32_t), h->stream));
  for (int k = 0; k < 4; ++k)  // both slots, each reused once
    HIPCHK(h, mdp_launch_xchg_probe(h->xd_dev, ++h->x_probe_ep, nchunk, h->x_probe, h->x_probe + 1, h->stream));
  uint32_t res[2] = {0, 0};
  HIPCHK(h, hipMemcpyAsync(res, h->x_probe, sizeof(res), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (mismatches) *mismatches = (int32_t)res[0];
  if (res[1]) return fail(h, "mdp_dp_xgmi_probe: a peer did not reach the exchange within 30 s");
  if (res[0]) return fail(h, "mdp_dp_xgmi_probe: exchanged values differ from the expected world sum");
  return 0;
}

int mdp_dp_xgmi_enable(mdp_handle* h) {
  if (unusable(h)) return -1;
  if (!h->xd_dev) return fail(h, "mdp_dp_xgmi_enable: not connected");
  if (h->update_mode != 0) return fail(h, "join data parallelism before choosing the throughput mode");
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->p2p = true;
  h->dp_world = h->x_world;
  drop_graphs(h);  // graphs captured without the exchange
  return 0;
}

int mdp_dp_xgmi_close(mdp_handle* h) {
  if (unusable(h)) return -1;
  (void)hipGetLastError();  // a failed open/map must not surface at the next launch check
  if (h->stream) HIPCHK(h, hipStreamSynchronize(h->stream));
  xgmi_release(h);
  if (!h->comm) h->dp_world = 1;
  drop_graphs(h);
  return 0;
}

int mdp_dp_info(mdp_handle* h, int32_t out4[4]) {
  if (unusable(h) || !out4) return -1;
  out4[0] = h->p2p ? 2 : (h->comm ? 1 : 0);
  out4[1] = 1;
  out4[2] = h->cfg.rank;
  out4[3] = 0;
  if (h->p2p) {
    out4[1] = h->x_world;
    out4[2] = h->x_rank;
    for (void* p : h->x_opened) out4[3] += p ? 1 : 0;
  } else if (h->comm) {
    int c = h->dp_world;
    if (rccl().count && rccl().count(h->comm, &c) != ncclSuccess) return fail(h, "ncclCommCount failed");
    out4[1] = c;
    out4[3] = c - 1;
  }
  return 0;
}

int mdp_dp_exchange_stats(mdp_handle* h, double out4[4], int32_t reset) {
  if (unusable(h) || !out4) return -1;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint64_t w[3] = {0, 0, 0};
  HIPCHK(h, hipMemcpy(w, &h->ctl->xw_ticks, sizeof(w), hipMemcpyDeviceToHost));
  const double us_per_tick = 0.01;  // s_memrealtime: 100 MHz
  out4[0] = (double)w[1];
  out4[1] = w[1] ? (double)w[0] * us_per_tick / (double)w[1] : 0.0;
  out4[2] = (double)w[2] * us_per_tick;
  out4[3] = (double)w[0] * us_per_tick;
  if (reset) {
    HIPCHK(h, hipMemsetAsync(&h->ctl->xw_ticks, 0, sizeof(w), h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  return 0;
}

int mdp_dp_exchange_stats_enable(mdp_handle* h, int32_t on) {
  if (unusable(h)) return -1;
  h->xw_stats = on != 0;
  return 0;
}

int mdp_set_graphs(mdp_handle* h, int32_t on) {
  MDP_NEED(h);
  h->graphs = on != 0;
  return 0;
}

static void drop_graphs(mdp_handle* h) {
  for (auto& kv : h->step_exec) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : h->multi_exec) (void)hipGraphExecDestroy(kv.second);
  h->step_exec.clear();
  h->multi_exec.clear();
  h->eager_steps = 0;
  if (h->round_exec) {
    (void)hipGraphExecDestroy(h->round_exec);
    h->round_exec = nullptr;
  }
  if (h->round_graph) {
    (void)hipGraphDestroy(h->round_graph);
    h->round_graph = nullptr;
  }
  h->eager_rounds = 0;
}

int mdp_set_update_mode(mdp_handle* h, int32_t mode) {
  if (unusable(h)) return -1;
  if (mode != 0 && mode != 1) return fail(h, "update mode must be 0 (strict) or 1 (throughput)");
  if (mode == 1) {
    if (!tp_ok(h)) return fail(h, "throughput mode needs the fused optimizer step for every net and <= 8 agents");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (tp_setup(h)) return -1;
  }
  if (mode != h->update_mode) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    drop_graphs(h);
    h->update_mode = mode;
  }
  return 0;
}

int mdp_update_all(mdp_handle* h, const int32_t* idx_dev, const float* u_tgt_dev, const float* u_act_dev) {
  if (unusable(h)) return -1;
  if (h->update_mode != 1) return fail(h, "mdp_update_all: set throughput mode first");
  if (h->len <= 0) return fail(h, "update on an empty replay buffer");
  {
    const int64_t B = h->cfg.batch_size, n = h->cfg.n_agents;
    MDP_DEV(h, idx_dev, 4 * n * B, "mdp_update_all", true);
    MDP_DEV(h, u_tgt_dev, 4 * n * n * B * MDP_ACT_DIM, "mdp_update_all", true);
    MDP_DEV(h, u_act_dev, 4 * n * B * MDP_ACT_DIM, "mdp_update_all", true);
  }
  const int32_t* idx = idx_dev;
  if (!idx) {
    const int rc = launch_make_index(h, h->cfg.n_agents * h->cfg.batch_size, h->index);
    if (rc) return rc;
    idx = h->index;
  }
  return do_round_tp(h, idx, u_tgt_dev, u_act_dev, nullptr);
}

int mdp_critic_grad(mdp_handle* h, int32_t agent, const int32_t* idx_dev, const float* u_tgt_dev) {
  if (bad_agent(h, agent)) return -1;
  if (!idx_dev) return fail(h, "critic_grad needs indices");
  MDP_DEV(h, idx_dev, 4 * (int64_t)h->cfg.batch_size, "mdp_critic_grad", false);
  MDP_DEV(h, u_tgt_dev, 4 * (int64_t)h->cfg.n_agents * h->cfg.batch_size * MDP_ACT_DIM, "mdp_critic_grad", true);
  return do_critic_grad(h, agent, idx_dev, u_tgt_dev);
}

int mdp_actor_grad(mdp_handle* h, int32_t agent, const int32_t* idx_dev, const float* u_act_dev) {
  if (bad_agent(h, agent)) return -1;
  if (!idx_dev) return fail(h, "actor_grad needs indices");
  MDP_DEV(h, idx_dev, 4 * (int64_t)h->cfg.batch_size, "mdp_actor_grad", false);
  MDP_DEV(h, u_act_dev, 4 * (int64_t)h->cfg.batch_size * MDP_ACT_DIM, "mdp_actor_grad", true);
  return do_actor_grad(h, agent, idx_dev, u_act_dev);
}

int mdp_reduce_grad(mdp_handle* h, int32_t agent, int32_t net) {
  if (bad_agent(h, agent)) return -1;
  return do_reduce(h, agent, net ? 1 : 0);
}

int mdp_apply_grad(mdp_handle* h, int32_t agent, int32_t net, float scale) {
  if (bad_agent(h, agent)) return -1;
  return do_apply(h, agent, net ? 1 : 0, false, scale);
}

int mdp_get_stats(mdp_handle* h, int32_t agent, double out6[6]) {
  if (bad_agent(h, agent)) return -1;
  double buf[8];
  HIPCHK(h, hipMemcpyAsync(buf, h->stats + agent * 8, sizeof(buf), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (int i = 0; i < 6; ++i) out6[i] = buf[i];
  return 0;
}

// -------------------------------------------------------------------- env
static int need_env(mdp_handle* h) {
  MDP_NEED(h);
  if (h->cfg.scenario == MDP_SCN_NONE || h->cfg.num_envs <= 0) return fail(h, "handle has no device env");
  return 0;
}

int mdp_env_reset(mdp_handle* h) {
  if (need_env(h)) return -1;
  EnvResetArgs a;
  a.env = h->L.env;
  a.seed = h->cfg.seed;
  a.ctr = h->reset_ctr++;
  a.env_base = h->cfg.rank * h->cfg.num_envs;
  a.E = h->cfg.num_envs;
  a.pos = h->pos;
  a.vel = h->vel;
  a.goal = h->goal;
  a.ep_step = h->ep_step;
  a.ep_rew = h->ep_rew;
  HIPCHK(h, mdp_launch_env_reset(a, h->stream));
  h->env_lockstep = true;
  return 0;
}

// pf_out: an extra rollout workgroup draws pf_count indices for the step's
// first round against the post-step ring length (the draw leaves the critical path)
// nsteps > 1: that many consecutive steps without update rounds in one launch
// (rollout_multi_ok: one env workgroup, the policies' own actions, no draw)
static int env_step_launch(mdp_handle* h, const float* act_in_dev, const float* u_dev, float* bench = nullptr,
                           int32_t* pf_out = nullptr, int pf_count = 0, int nsteps = 1) {
  RolloutArgs a;
  a.pf_out = pf_out;
  a.pf_count = pf_out ? pf_count : 0;
  a.nsteps = nsteps;
  a.topo = h->L.topo;
  a.env = h->L.env;
  a.theta = h->theta;
  a.replay = h->replay;
  a.cap = h->cfg.capacity;
  a.pos = h->pos;
  a.vel = h->vel;
  a.goal = h->goal;
  a.ep_step = h->ep_step;
  a.ep_rew = h->ep_rew;
  a.eplog = h->eplog;
  a.eplog_cap = h->L.eplog_rows;
  a.eplog_by_env = h->env_lockstep ? 1 : 0;
  a.ctl = h->ctl;
  a.seed = h->cfg.seed;
  a.E = h->cfg.num_envs;
  a.env_base = h->cfg.rank * h->cfg.num_envs;
  a.act_in = act_in_dev;
  a.u_in = u_dev;
  a.ticket = &h->ctl->ticket[2];
  a.bench = bench;
  ProfScope p(h, MDP_K_ROLLOUT);
  HIPCHK(h, mdp_launch_rollout(a, h->L.topo.H, lds_rollout_bytes(h->L.topo), h->stream));
  return 0;
}

// several env steps per k_rollout launch need every env copy in one workgroup
static bool rollout_multi_ok(const mdp_handle* h) { return h->cfg.num_envs <= 16; }  // k_rollout: 16 envs per workgroup (MDP_R)

static void advance_ring_mirror(mdp_handle* h) {
  const int64_t cap = h->cfg.capacity, E = h->cfg.num_envs;
  h->len = std::min(cap, h->len + E);
  h->next = (h->next + E) % cap;
}

int mdp_env_step(mdp_handle* h, const float* act_in_dev, const float* u_dev) {
  if (need_env(h)) return -1;
  const int64_t en5 = 4 * (int64_t)h->cfg.num_envs * h->cfg.n_agents * MDP_ACT_DIM;
  MDP_DEV(h, act_in_dev, en5, "mdp_env_step", true);
  MDP_DEV(h, u_dev, en5, "mdp_env_step", true);
  const int rc = env_step_launch(h, act_in_dev, u_dev);
  if (rc) return rc;
  advance_ring_mirror(h);
  return 0;
}

int mdp_env_step_bench(mdp_handle* h, float* info_dev) {
  if (need_env(h)) return -1;
  if (!info_dev) return fail(h, "mdp_env_step_bench: info_dev is null");
  MDP_DEV(h, info_dev, 4 * (int64_t)h->cfg.num_envs * h->cfg.n_agents * MDP_BENCH_W, "mdp_env_step_bench", false);
  if (h->cfg.scenario == MDP_SCN_SIMPLE)
    return fail(h, "scenario 'simple' has no benchmark_data (MPE Scenario attribute missing)");
  const int rc = env_step_launch(h, nullptr, nullptr, info_dev);
  if (rc) return rc;
  advance_ring_mirror(h);
  return 0;
}

// rollout, then `rounds` rounds on alternating index slots; round r's first
// critic kernel draws round r+1's indices (same ring length: the rounds of one
// step follow one rollout) in an extra workgroup -- the draw leaves the
// critical path for every round but the first
static int step_launches(mdp_handle* h, int rounds) {
  const int nb = h->cfg.n_agents * h->cfg.batch_size;
  int32_t* slot[2] = {h->index, h->index + nb};
  // the critic-launch prefetch serves throughput mode only where its one critic
  // launch covers every agent (tp_fast); a mix of fast and general agents
  // (e.g. tag with DDPG adversaries) draws in the optimizer pair launches
  const bool pf = prefetch_ok(h) && (h->update_mode == 0 || tp_fast(h));
  // (throughput mode on the general kernels: in its optimizer pair launches, RCCL included)
  const bool ra_draw = !pf && (h->update_mode == 0 ? draw_in_ra_ok(h) : !tp_fast(h));
  bool fast_all = !h->general_grads;
  for (int i = 0; i < h->cfg.n_agents && fast_all; ++i) fast_all = grads_r_ok(h->L.topo, i);
  // one agent ahead (round_updates): the step's first draw is agent 0's B only
  const int ahead = !h->draw_ahead || h->update_mode != 0 ? 0 : (pf && fast_all) ? 1 : ra_draw ? 2 : 0;
  const int first = ahead ? h->cfg.batch_size : nb;
  // the first round's draw rides in the rollout launch (MDP_ROLLOUT_DRAW=0: its own launch)
  const bool in_rollout = rounds > 0 && h->rollout_draw;
  int rc = env_step_launch(h, nullptr, nullptr, nullptr, in_rollout ? slot[0] : nullptr, first);
  if (rc || rounds == 0) return rc;
  if (!in_rollout && (rc = launch_make_index(h, first, slot[0]))) return rc;
  bool carry = false;
  for (int r = 0; r < rounds && !rc; ++r) {
    const bool more = r + 1 < rounds;
    int32_t* next = (more && pf) ? slot[(r + 1) & 1] : nullptr;  // drawn in the critic launches
    rc = round_updates(h, slot[r & 1], next, carry, next, &carry, (more && ra_draw) ? slot[(r + 1) & 1] : nullptr,
                       ahead);
    if (!rc && more && !pf && !ra_draw) rc = launch_make_index(h, nb, slot[(r + 1) & 1]);
  }
  return rc;
}

// the launches of one training step (eager, or captured once per round count and replayed)
static int train_step_body(mdp_handle* h, int rounds) {
  // RCCL collectives are launched eagerly unless asked; the xGMI exchange is
  // inside the optimizer kernels, so those steps are always captured
  const bool no_graph = h->comm && !h->dp_graphs;
  if (!h->graphs || no_graph || any_prof(h) || h->eager_steps < 1 || rounds == 0) {
    if (rounds > 0) ++h->eager_steps;  // first training step eager (one-time kernel attribute setup)
    return step_launches(h, rounds);
  }
  auto it = h->step_exec.find(rounds);
  if (it == h->step_exec.end()) {
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    h->capturing = true;
    const int rc = step_launches(h, rounds);
    h->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return fail(h, "hipStreamEndCapture", e);
    hipGraphExec_t x = nullptr;
    const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) return fail(h, "hipGraphInstantiate", ei);
    it = h->step_exec.emplace(rounds, x).first;
  }
  HIPCHK(h, hipGraphLaunch(it->second, h->stream));
  return 0;
}

// several consecutive training steps captured as ONE graph (keyed by their
// round counts): the launches are exactly those of the steps one by one, but a
// graph launch boundary costs ~6.7 us on the GPU clock against ~1.5-2 us for a
// kernel boundary inside a graph (tools/step_boundary.py)
static int multi_graph(mdp_handle* h, const std::vector<int>& ks, hipGraphExec_t* out) {
  auto it = h->multi_exec.find(ks);
  if (it != h->multi_exec.end()) {
    *out = it->second;
    return 0;
  }
  HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  h->capturing = true;
  int rc = 0;
  for (size_t i = 0; i < ks.size() && !rc;) {
    // a stretch of steps without update rounds (one env copy: 99 of every 100)
    // as one rollout launch of that many steps, when the envs fit one workgroup
    size_t j = i;
    while (j < ks.size() && ks[j] == 0 && (int)(j - i) < 64) ++j;
    if (j - i > 1 && rollout_multi_ok(h)) {
      rc = env_step_launch(h, nullptr, nullptr, nullptr, nullptr, 0, (int)(j - i));
      i = j;
    } else {
      rc = step_launches(h, ks[i]);
      ++i;
    }
  }
  h->capturing = false;
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(h->stream, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(h, "hipStreamEndCapture", e);
  hipGraphExec_t x = nullptr;
  const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ei != hipSuccess) return fail(h, "hipGraphInstantiate", ei);
  h->multi_exec.emplace(ks, x);
  *out = x;
  return 0;
}

int mdp_train_steps(mdp_handle* h, int32_t n, const int32_t* rounds, int32_t launch) {
  if (need_env(h)) return -1;
  if (n < 1 || n > 64 || !rounds) return fail(h, "mdp_train_steps: 1 <= n <= 64 steps");
  std::vector<int> ks(rounds, rounds + n);
  for (int k : ks)
    if (k < 0 || k > 64) return fail(h, "mdp_train_steps: rounds must be in [0, 64]");
  // steps without a round (replay below the gate, or fewer than train_every
  // transitions per step: E = 1 trains every 100th step) are their rollout
  // launch alone inside the group's graph
  const bool no_graph = h->comm && !h->dp_graphs;
  const bool graphable = h->graphs && !no_graph && !any_prof(h) && h->eager_steps >= 1;
  if (!launch) {  // capture and instantiate ahead of time (nothing runs)
    hipGraphExec_t x = nullptr;
    return graphable ? multi_graph(h, ks, &x) : 0;
  }
  if (!graphable) {
    for (int k : ks) {
      const int rc = mdp_train_step(h, k);
      if (rc) return rc;
    }
    return 0;
  }
  const int64_t len0 = h->len, next0 = h->next;
  for (int i = 0; i < n; ++i) advance_ring_mirror(h);
  hipGraphExec_t x = nullptr;
  int rc = multi_graph(h, ks, &x);
  if (!rc) {
    const hipError_t e = hipGraphLaunch(x, h->stream);
    if (e != hipSuccess) rc = fail(h, "hipGraphLaunch", e);
  }
  if (rc) {
    h->len = len0;
    h->next = next0;
  }
  return rc;
}

int mdp_train_step(mdp_handle* h, int32_t rounds) {
  if (need_env(h)) return -1;
  if (rounds < 0 || rounds > 64) return fail(h, "mdp_train_step: rounds must be in [0, 64]");
  if (rounds > 0 && h->len + h->cfg.num_envs <= 0) return fail(h, "update round on an empty replay buffer");
  // the index kernels read the ring length the rollout leaves (device Ctl); the
  // host mirror moves first so the empty-buffer guard sees the same state, and
  // moves back when the step could not be launched
  const int64_t len0 = h->len, next0 = h->next;
  advance_ring_mirror(h);
  const int rc = train_step_body(h, rounds);
  if (rc) {
    h->len = len0;
    h->next = next0;
  }
  return rc;
}

int mdp_env_get_state(mdp_handle* h, float* pos, float* vel, int32_t* goal, int32_t* ep_step) {
  if (need_env(h)) return -1;
  const int64_t E = h->cfg.num_envs, ne = h->L.n_ent;
  if (pos) HIPCHK(h, hipMemcpyAsync(pos, h->pos, 4 * E * ne * 2, hipMemcpyDeviceToHost, h->stream));
  if (vel) HIPCHK(h, hipMemcpyAsync(vel, h->vel, 4 * E * ne * 2, hipMemcpyDeviceToHost, h->stream));
  if (goal) HIPCHK(h, hipMemcpyAsync(goal, h->goal, 4 * E, hipMemcpyDeviceToHost, h->stream));
  if (ep_step) HIPCHK(h, hipMemcpyAsync(ep_step, h->ep_step, 4 * E, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_env_set_state(mdp_handle* h, const float* pos, const float* vel, const int32_t* goal, const int32_t* ep_step) {
  if (need_env(h)) return -1;
  const int64_t E = h->cfg.num_envs, ne = h->L.n_ent;
  if (pos) HIPCHK(h, hipMemcpyAsync(h->pos, pos, 4 * E * ne * 2, hipMemcpyHostToDevice, h->stream));
  if (vel) HIPCHK(h, hipMemcpyAsync(h->vel, vel, 4 * E * ne * 2, hipMemcpyHostToDevice, h->stream));
  if (goal) HIPCHK(h, hipMemcpyAsync(h->goal, goal, 4 * E, hipMemcpyHostToDevice, h->stream));
  if (ep_step) {
    HIPCHK(h, hipMemcpyAsync(h->ep_step, ep_step, 4 * E, hipMemcpyHostToDevice, h->stream));
    h->env_lockstep = std::all_of(ep_step, ep_step + E, [&](int32_t s) { return s == ep_step[0]; });
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

int mdp_env_obs(mdp_handle* h, float* obs_dev) {
  if (need_env(h)) return -1;
  {
    int64_t so = 0;
    for (int i = 0; i < h->cfg.n_agents; ++i) so += h->cfg.obs_dim[i];
    MDP_DEV(h, obs_dev, 4 * (int64_t)h->cfg.num_envs * so, "mdp_env_obs", false);
  }
  EnvObsArgs a;
  a.topo = h->L.topo;
  a.env = h->L.env;
  a.E = h->cfg.num_envs;
  a.pos = h->pos;
  a.vel = h->vel;
  a.goal = h->goal;
  a.obs = obs_dev;
  HIPCHK(h, mdp_launch_env_obs(a, h->stream));
  return 0;
}

// the reference's check_nan (tf_util.py:322,366-368, a debug option it never
// enables): non-finite values in every parameter set (theta, target, Adam m
// and v) and in every agent's 6 update stats, counted on the device;
// synchronous, outside any graph
int mdp_check_finite(mdp_handle* h, int64_t* nonfinite) {
  MDP_NEED(h);
  if (!nonfinite) return fail(h, "mdp_check_finite: nonfinite is null");
  HIPCHK(h, hipMemsetAsync(&h->ctl->nonfinite, 0, sizeof(uint32_t), h->stream));
  const float* sets[4] = {h->theta, h->target, h->m, h->v};
  for (const float* p : sets) HIPCHK(h, mdp_launch_count_nonfinite(p, h->L.PT, &h->ctl->nonfinite, h->stream));
  uint32_t c = 0;
  const int n = h->cfg.n_agents;
  std::vector<double> st(8 * (size_t)n);
  HIPCHK(h, hipMemcpyAsync(&c, &h->ctl->nonfinite, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(st.data(), h->stats, sizeof(double) * st.size(), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  int64_t bad = c;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 6; ++k) bad += std::isfinite(st[8 * i + k]) ? 0 : 1;
  *nonfinite = bad;
  return 0;
}

int64_t mdp_episode_count(mdp_handle* h) {
  MDP_NEED(h);
  int64_t n = 0;
  if (hipMemcpyAsync(&n, &h->ctl->episodes, 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess) return -1;
  if (hipStreamSynchronize(h->stream) != hipSuccess) return -1;
  return n;
}

int mdp_episode_log(mdp_handle* h, int64_t first, int64_t n, float* out) {
  MDP_NEED(h);
  const int64_t cap = h->L.eplog_rows, w = 1 + h->cfg.n_agents;
  if (n > cap || first < 0) return fail(h, "episode log request exceeds ring");
  int64_t done = 0;
  while (done < n) {  // at most two contiguous spans of the ring
    const int64_t slot = (first + done) % cap;
    const int64_t span = std::min(n - done, cap - slot);
    HIPCHK(h, hipMemcpyAsync(out + done * w, h->eplog + slot * w, 4 * w * span, hipMemcpyDeviceToHost, h->stream));
    done += span;
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return 0;
}

// -------------------------------------------------------------- profiling
int mdp_prof_enable(mdp_handle* h, int32_t kind, int32_t on) {
  MDP_NEED(h);
  if (kind < 0 || kind >= MDP_K_COUNT) return fail(h, "bad kernel kind");
  if (!on) flush_prof(h, kind);
  h->prof_on[kind] = on != 0;
  if (on) {
    h->prof_ms[kind] = 0.0;
    h->prof_n[kind] = 0;
    h->ev_used[kind] = 0;
  }
  return 0;
}

int mdp_prof_read(mdp_handle* h, int32_t kind, double* total_ms, int64_t* launches) {
  MDP_NEED(h);
  if (kind < 0 || kind >= MDP_K_COUNT) return fail(h, "bad kernel kind");
  flush_prof(h, kind);
  if (total_ms) *total_ms = h->prof_ms[kind];
  if (launches) *launches = h->prof_n[kind];
  return 0;
}

}  // extern "C"
