// abi_host_check -- every entry point of include/maddpg_hip.h driven from C++
// with the C-ABI shim (maddpg_amd/csrc/mdp_api.cpp) built under host
// AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race detection /
// sanitizers": the reference has none, `tf_util.py:322` check_nan off).  The
// kernels are the shipped objects; only host code is instrumented (GPU ASan is
// not available on this pool).
//
//   make -C maddpg_amd/csrc host-check         -> tests/native/abi_host_check
//   abi_host_check cpu    no GPU needed: config validation, layout, the
//                         ra plan, null / failed-create handles on every entry
//   abi_host_check gpu    device 0: the whole lifecycle of two configurations
//                         (H=64 register kernels, H=128 general kernels), strict
//                         and throughput rounds, graphs, every error path on a
//                         live handle, destroy
// Exit status 0 and a final "OK <checks>" line when every check held; any
// sanitizer report aborts the run (-fno-sanitize-recover, ASan default).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "maddpg_hip.h"

static int g_checks = 0, g_fail = 0;

#define CHECK(cond)                                                             \
  do {                                                                          \
    ++g_checks;                                                                 \
    if (!(cond)) {                                                              \
      ++g_fail;                                                                 \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);      \
    }                                                                           \
  } while (0)

// rc < 0 and a non-empty message: the ABI's error convention
#define CHECK_ERR(h, call)                                                      \
  do {                                                                          \
    const long long rc__ = (long long)(call);                                   \
    ++g_checks;                                                                 \
    if (rc__ >= 0 || std::strlen(mdp_last_error(h)) == 0) {                     \
      ++g_fail;                                                                 \
      std::fprintf(stderr, "FAIL %s:%d: %s -> %lld (%s)\n", __FILE__, __LINE__, \
                   #call, rc__, mdp_last_error(h));                             \
    }                                                                           \
  } while (0)

#define CHECK_OK(h, call)                                                       \
  do {                                                                          \
    const long long rc__ = (long long)(call);                                   \
    ++g_checks;                                                                 \
    if (rc__ != 0) {                                                            \
      ++g_fail;                                                                 \
      std::fprintf(stderr, "FAIL %s:%d: %s -> %lld (%s)\n", __FILE__, __LINE__, \
                   #call, rc__, mdp_last_error(h));                             \
    }                                                                           \
  } while (0)

#define HIP_OR_DIE(call)                                                        \
  do {                                                                          \
    const hipError_t e__ = (call);                                              \
    if (e__ != hipSuccess) {                                                    \
      std::fprintf(stderr, "HIP %s: %s\n", #call, hipGetErrorString(e__));      \
      std::exit(3);                                                             \
    }                                                                           \
  } while (0)

// the MPE scenario table of maddpg_amd/envs.py (upstream make_world defaults)
static mdp_config base_config(int scenario, int n, int na, int H, int B, int E) {
  mdp_config c;
  std::memset(&c, 0, sizeof(c));
  c.n_agents = n;
  c.act_dim = MDP_ACT_DIM;
  c.num_units = H;
  c.batch_size = B;
  c.max_episode_len = 25;
  c.capacity = 100000;
  c.num_envs = E;
  c.scenario = scenario;
  c.num_adversaries = na;
  c.world_size = 1;
  c.lr = 1e-2f;
  c.tau = 1e-2f;
  c.grad_clip = 0.5f;
  c.actor_reg = 1e-3f;
  c.adam_b1 = 0.9f;
  c.adam_b2 = 0.999f;
  c.adam_eps = 1e-8f;
  c.gamma = 0.95;
  c.seed = 7;
  for (int i = 0; i < n; ++i) {
    switch (scenario) {
      case MDP_SCN_SIMPLE: c.obs_dim[i] = 4; break;
      case MDP_SCN_SPREAD: c.obs_dim[i] = 4 + 2 * n + 4 * (n - 1); break;
      case MDP_SCN_ADVERSARY: c.obs_dim[i] = (i < na ? 0 : 2) + 4 * (n - 1); break;
      case MDP_SCN_TAG: c.obs_dim[i] = 4 + 4 + 2 * (n - 1) + 2 * ((n - na) - (i < na ? 0 : 1)); break;
      default: c.obs_dim[i] = 10 + i; break;
    }
  }
  return c;
}

// ---------------------------------------------------------------- cpu mode
static void null_handle_entries(mdp_handle* h) {
  // h is NULL or a handle whose mdp_create failed: every call is refused
  float f[64] = {};
  double d[8] = {};
  int32_t i4[8] = {}, i6[6] = {};
  int64_t off = 0, bytes = 0;
  uint32_t st[625] = {};
  uint8_t xh[MDP_XGMI_HANDLE_BYTES] = {};
  mdp_tensor_info ti;
  const int32_t rounds[2] = {1, 1};
  CHECK(mdp_synchronize(h) < 0);
  CHECK(mdp_region(h, MDP_R_THETA, &off, &bytes) < 0);
  CHECK(mdp_tensor(h, 0, 0, 0, &ti) < 0);
  CHECK(mdp_row_layout(h, 0, i6) < 0);
  CHECK(mdp_set_params(h, 0, MDP_ACTOR, f, 1) < 0);
  CHECK(mdp_get_params(h, 0, MDP_ACTOR, f, 1) < 0);
  CHECK(mdp_get_beta_powers(h, 0, 0, f) < 0);
  CHECK(mdp_set_beta_powers(h, 0, 0, f) < 0);
  CHECK(mdp_buffer_len(h) < 0);
  CHECK(mdp_buffer_add_rows(h, nullptr, 1) < 0);
  CHECK(mdp_buffer_put_agent(h, 0, nullptr, nullptr, 1) < 0);
  CHECK(mdp_buffer_set_len(h, 0, 0) < 0);
  CHECK(mdp_seed_py_random(h, 1) < 0);
  CHECK(mdp_set_rng_state(h, st) < 0);
  CHECK(mdp_get_rng_state(h, st) < 0);
  CHECK(mdp_make_index(h, 4, nullptr) < 0);
  CHECK(mdp_sample_rows(h, nullptr, 4, nullptr) < 0);
  CHECK(mdp_act(h, 0, 0, nullptr, nullptr, 1, nullptr) < 0);
  CHECK(mdp_actor_logits(h, 0, 0, nullptr, nullptr, 1) < 0);
  CHECK(mdp_q_values(h, 0, 0, nullptr, nullptr, 1) < 0);
  CHECK(mdp_update(h, 0, nullptr, nullptr, nullptr) < 0);
  CHECK(mdp_update_gate(h, 100) < 0);
  CHECK(mdp_agent_update(h, 0, 100, nullptr, nullptr, d) < 0);
  CHECK(mdp_update_round(h) < 0);
  CHECK(mdp_set_graphs(h, 1) < 0);
  CHECK(mdp_train_step(h, 1) < 0);
  CHECK(mdp_train_steps(h, 2, rounds, 1) < 0);
  CHECK(mdp_dp_init(h, xh, 2, 0) < 0);
  CHECK(mdp_dp_xgmi_open(h, 2, 0, xh) < 0);
  CHECK(mdp_dp_xgmi_connect(h, xh) < 0);
  CHECK(mdp_dp_xgmi_probe(h, i4) < 0);
  CHECK(mdp_dp_xgmi_enable(h) < 0);
  CHECK(mdp_dp_xgmi_close(h) < 0);
  CHECK(mdp_dp_info(h, i4) < 0);
  CHECK(mdp_dp_exchange_stats(h, d, 1) < 0);
  CHECK(mdp_dp_exchange_stats_enable(h, 1) < 0);
  CHECK(mdp_critic_grad(h, 0, nullptr, nullptr) < 0);
  CHECK(mdp_actor_grad(h, 0, nullptr, nullptr) < 0);
  CHECK(mdp_reduce_grad(h, 0, 0) < 0);
  CHECK(mdp_apply_grad(h, 0, 0, 1.f) < 0);
  CHECK(mdp_get_stats(h, 0, d) < 0);
  CHECK(mdp_check_finite(h, &off) < 0);
  CHECK(mdp_set_update_mode(h, 1) < 0);
  CHECK(mdp_update_all(h, nullptr, nullptr, nullptr) < 0);
  CHECK(mdp_env_reset(h) < 0);
  CHECK(mdp_env_step(h, nullptr, nullptr) < 0);
  CHECK(mdp_env_get_state(h, nullptr, nullptr, nullptr, nullptr) < 0);
  CHECK(mdp_env_set_state(h, nullptr, nullptr, nullptr, nullptr) < 0);
  CHECK(mdp_env_obs(h, nullptr) < 0);
  CHECK(mdp_env_step_bench(h, f) < 0);
  CHECK(mdp_episode_count(h) < 0);
  CHECK(mdp_episode_log(h, 0, 1, f) < 0);
  CHECK(mdp_prof_enable(h, 0, 1) < 0);
  CHECK(mdp_prof_read(h, 0, d, &off) < 0);
  CHECK(mdp_grad_variant(h, 0) < 0);
  CHECK(mdp_last_error(h) != nullptr);
}

static void cpu_mode() {
  CHECK(mdp_abi_version() == MDP_ABI_VERSION);
  int64_t pt = 0;
  CHECK(mdp_arena_bytes(nullptr, &pt) < 0);
  CHECK(mdp_ra_plan(nullptr, 256, 1, nullptr) < 0);

  // every BASELINE config and the widest nets lay out
  const mdp_config ok[] = {
      base_config(MDP_SCN_SIMPLE, 1, 0, 64, 1024, 1),
      base_config(MDP_SCN_SPREAD, 3, 0, 64, 1024, 1024),
      base_config(MDP_SCN_ADVERSARY, 3, 1, 64, 1024, 4096),
      base_config(MDP_SCN_TAG, 6, 4, 128, 4096, 4096),
      base_config(MDP_SCN_NONE, 8, 0, 256, 1 << 20, 0),
      base_config(MDP_SCN_SPREAD, 3, 0, 1, 1, 1),
  };
  for (const mdp_config& c : ok) {
    pt = 0;
    const int64_t b = mdp_arena_bytes(&c, &pt);
    CHECK(b > 0);
    CHECK(pt > 0);
    CHECK(b % 256 == 0);
    int32_t plan[2 * MDP_MAX_AGENTS];
    const int fb = mdp_ra_plan(&c, 256, 1, plan);
    CHECK(fb >= 0 && fb <= 2 * c.n_agents);
    for (int i = 0; i < 2 * c.n_agents; ++i) CHECK(plan[i] != 0);
    CHECK(mdp_ra_plan(&c, 0, 1, plan) == 2 * c.n_agents);  // nothing fits on no CUs
  }
  CHECK(mdp_ra_plan(&ok[1], -1, 1, nullptr) < 0);

  // every validation rule of build_layout refuses
  auto bad = [](void (*edit)(mdp_config&)) {
    mdp_config c = base_config(MDP_SCN_SPREAD, 3, 0, 64, 1024, 1024);
    edit(c);
    int64_t p = -5;
    CHECK(mdp_arena_bytes(&c, &p) < 0);
    CHECK(p == -5);
    mdp_handle* h = nullptr;
    char arena[16];
    CHECK(mdp_create(&c, arena, 16, nullptr, &h) < 0);
    CHECK(h != nullptr && std::strlen(mdp_last_error(h)) > 0);
    null_handle_entries(h);
    CHECK(mdp_destroy(h) == 0);
  };
  bad([](mdp_config& c) { c.n_agents = 0; });
  bad([](mdp_config& c) { c.n_agents = MDP_MAX_AGENTS + 1; });
  bad([](mdp_config& c) { c.act_dim = 4; });
  bad([](mdp_config& c) { c.num_units = 0; });
  bad([](mdp_config& c) { c.num_units = MDP_MAX_UNITS + 1; });
  bad([](mdp_config& c) { c.batch_size = 0; });
  bad([](mdp_config& c) { c.batch_size = (1 << 20) + 1; });
  bad([](mdp_config& c) { c.capacity = 0; });
  bad([](mdp_config& c) { c.capacity = int64_t(1) << 31; });
  bad([](mdp_config& c) { c.num_envs = -1; });
  bad([](mdp_config& c) { c.num_envs = (1 << 24) + 1; });
  bad([](mdp_config& c) { c.capacity = 100; });            // fewer rows than env copies
  bad([](mdp_config& c) { c.obs_dim[1] = 17; });           // not the scenario's
  bad([](mdp_config& c) { c.obs_dim[2] = 0; });
  bad([](mdp_config& c) { c.scenario = 99; });
  bad([](mdp_config& c) { c.episode_log_rows = -1; });
  bad([](mdp_config& c) { c.episode_log_rows = 2047; });   // < 2 num_envs
  bad([](mdp_config& c) {
    c = base_config(MDP_SCN_ADVERSARY, 3, 0, 64, 64, 4);   // no adversary
  });
  bad([](mdp_config& c) {
    c = base_config(MDP_SCN_TAG, 4, 4, 64, 64, 4);         // no good agent
  });

  // a null handle, a null config, no out pointer, an arena too small
  null_handle_entries(nullptr);
  CHECK(std::strcmp(mdp_last_error(nullptr), "null handle") == 0);
  CHECK(mdp_stream(nullptr) == nullptr);
  CHECK(mdp_destroy(nullptr) == 0);
  mdp_handle* h = nullptr;
  char arena[16];
  CHECK(mdp_create(nullptr, arena, 16, nullptr, &h) < 0);
  CHECK(h != nullptr);
  null_handle_entries(h);
  CHECK(mdp_destroy(h) == 0);
  CHECK(mdp_create(&ok[1], arena, 16, nullptr, nullptr) < 0);
  h = nullptr;
  CHECK(mdp_create(&ok[1], arena, 16, nullptr, &h) < 0);  // arena smaller than mdp_arena_bytes
  CHECK(std::strstr(mdp_last_error(h), "arena") != nullptr);
  null_handle_entries(h);
  CHECK(mdp_destroy(h) == 0);
}

// ---------------------------------------------------------------- gpu mode
static uint32_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(s >> 33);
}

static int64_t net_floats(mdp_handle* h, int agent, int net) {
  int64_t n = 0;
  for (int t = 0; t < 6; ++t) {
    mdp_tensor_info ti;
    if (mdp_tensor(h, agent, net, t, &ti) != 0) return -1;
    n += (int64_t)ti.rows * ti.cols;
  }
  return n;
}

static bool all_finite(const double* v, int n) {
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(v[i])) return false;
  return true;
}

// rc < 0 and the message names the refusal `why`: nothing was launched
#define CHECK_REFUSED(h, call, why)                                               \
  do {                                                                            \
    const long long rc__ = (long long)(call);                                     \
    ++g_checks;                                                                   \
    if (rc__ >= 0 || std::strstr(mdp_last_error(h), why) == nullptr) {            \
      ++g_fail;                                                                   \
      std::fprintf(stderr, "FAIL %s:%d: %s -> %lld (%s)\n", __FILE__, __LINE__,   \
                   #call, rc__, mdp_last_error(h));                               \
    }                                                                             \
  } while (0)

static int lay_stride(mdp_handle* h) {
  int32_t lay[6] = {};
  return mdp_row_layout(h, 0, lay) == 0 ? lay[5] : 0;
}

// Every "_dev" argument of every entry point refuses host memory (malloc, the
// stack, pinned hipHostMalloc) and a device buffer shorter than the call
// needs, returning < 0 with a message before any launch -- a host address that
// reached a kernel faulted the GPU in round 5 (r05h).  The handle
// stays usable: the caller's lifecycle continues on it afterwards.
static void host_pointers_refused(mdp_handle* h, const mdp_config& c, int32_t* idx, float* rows, float* obs,
                                  float* act, float* q, float* u, float* info) {
  const int n = c.n_agents, B = c.batch_size, E = c.num_envs;
  const size_t big = (size_t)64 << 20;  // larger than any buffer a call here reads or writes
  void* hb = std::malloc(big);
  CHECK(hb != nullptr);
  std::memset(hb, 0, big);
  float* hf = (float*)hb;
  int32_t* hi = (int32_t*)hb;
  int64_t* hl = (int64_t*)hb;
  const char* NDM = "not device memory";
  CHECK_REFUSED(h, mdp_buffer_add_rows(h, hf, 4), NDM);
  CHECK_REFUSED(h, mdp_buffer_put_agent(h, 0, hl, rows, 4), NDM);
  CHECK_REFUSED(h, mdp_buffer_put_agent(h, 0, (int64_t*)idx, hf, 4), NDM);
  CHECK_REFUSED(h, mdp_make_index(h, B, hi), NDM);
  CHECK_REFUSED(h, mdp_sample_rows(h, hi, B, rows), NDM);
  CHECK_REFUSED(h, mdp_sample_rows(h, idx, B, hf), NDM);
  CHECK_REFUSED(h, mdp_act(h, 0, 0, hf, act, B, nullptr), NDM);
  CHECK_REFUSED(h, mdp_act(h, 0, 0, obs, hf, B, nullptr), NDM);
  CHECK_REFUSED(h, mdp_act(h, 0, 1, obs, act, B, hf), NDM);
  CHECK_REFUSED(h, mdp_actor_logits(h, 0, 0, hf, act, B), NDM);
  CHECK_REFUSED(h, mdp_actor_logits(h, 0, 0, obs, hf, B), NDM);
  CHECK_REFUSED(h, mdp_q_values(h, 0, 0, hf, q, B), NDM);
  CHECK_REFUSED(h, mdp_q_values(h, 0, 0, rows, hf, B), NDM);
  CHECK_REFUSED(h, mdp_update(h, 0, hi, nullptr, nullptr), NDM);
  CHECK_REFUSED(h, mdp_update(h, 0, idx, hf, nullptr), NDM);
  CHECK_REFUSED(h, mdp_update(h, 0, idx, nullptr, hf), NDM);
  double st6[6];
  CHECK_REFUSED(h, mdp_agent_update(h, 0, 100, hi, u, st6), NDM);
  CHECK_REFUSED(h, mdp_agent_update(h, 0, 100, idx, hf, st6), NDM);
  CHECK_REFUSED(h, mdp_critic_grad(h, 0, hi, u), NDM);
  CHECK_REFUSED(h, mdp_critic_grad(h, 0, idx, hf), NDM);
  CHECK_REFUSED(h, mdp_actor_grad(h, 0, hi, u), NDM);
  CHECK_REFUSED(h, mdp_actor_grad(h, 0, idx, hf), NDM);
  CHECK_REFUSED(h, mdp_env_step(h, hf, nullptr), NDM);
  CHECK_REFUSED(h, mdp_env_step(h, nullptr, hf), NDM);
  CHECK_REFUSED(h, mdp_env_obs(h, hf), NDM);
  CHECK_REFUSED(h, mdp_env_step_bench(h, hf), NDM);
  // the stack and pinned host memory are host memory too
  int32_t on_stack[16] = {};
  CHECK_REFUSED(h, mdp_make_index(h, 16, on_stack), NDM);
  void* pinned = nullptr;
  HIP_OR_DIE(hipHostMalloc(&pinned, 4 * (size_t)B * 8, hipHostMallocDefault));
  CHECK_REFUSED(h, mdp_act(h, 0, 0, obs, (float*)pinned, B, nullptr), NDM);
  HIP_OR_DIE(hipHostFree(pinned));
  // device buffers shorter than the call needs: the last 4 bytes the call
  // would touch lie one float past the end of a 4 MiB allocation.  Run only
  // where the runtime reports that allocation's exact extent (the library
  // checks with the same hipMemGetAddressRange), so a runtime that rounds
  // extents can never let a kernel read past a mapping here.
  {
    const size_t FB = (size_t)4 << 20, NF = FB / 4;
    float* four = nullptr;
    HIP_OR_DIE(hipMalloc((void**)&four, FB));
    hipDeviceptr_t base = nullptr;
    size_t ext = 0;
    const bool exact = hipMemGetAddressRange(&base, &ext, (hipDeviceptr_t)four) == hipSuccess &&
                       base == (hipDeviceptr_t)four && ext == FB;
    std::printf("  short-buffer checks %s (extent %zu of %zu)\n", exact ? "on" : "skipped", ext, FB);
    if (exact) {
      const char* SHORT = "allocation too small";
      const size_t stride = (size_t)lay_stride(h);
      CHECK_REFUSED(h, mdp_make_index(h, B, (int32_t*)(four + NF - B + 1)), SHORT);
      CHECK_REFUSED(h, mdp_sample_rows(h, idx, B, four + NF - (size_t)B * stride + 1), SHORT);
      CHECK_REFUSED(h, mdp_q_values(h, 0, 0, rows, four + NF - B + 1, B), SHORT);
      CHECK_REFUSED(h, mdp_env_step_bench(h, four + NF - (size_t)E * n * MDP_BENCH_W + 1), SHORT);
      CHECK_REFUSED(h, mdp_update(h, 0, idx, four + NF - (size_t)n * B * 5 + 1, nullptr), SHORT);
      // exactly long enough is accepted (the last float of the allocation)
      CHECK_OK(h, mdp_q_values(h, 0, 0, rows, four + NF - B, B));
    }
    CHECK_OK(h, mdp_synchronize(h));
    HIP_OR_DIE(hipFree(four));
  }
  // device memory mapped through the virtual-memory API (hipMemCreate +
  // hipMemMap, what PyTorch's expandable segments use) is accepted
  {
    hipMemAllocationProp prop;
    std::memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess && gran) {
      const size_t sz = ((4 * (size_t)n * B + gran - 1) / gran) * gran;
      hipMemGenericAllocationHandle_t mh;
      void* va = nullptr;
      HIP_OR_DIE(hipMemCreate(&mh, sz, &prop, 0));
      HIP_OR_DIE(hipMemAddressReserve(&va, sz, 0, nullptr, 0));
      HIP_OR_DIE(hipMemMap(va, sz, 0, mh, 0));
      hipMemAccessDesc acc;
      acc.location = prop.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      HIP_OR_DIE(hipMemSetAccess(va, sz, &acc, 1));
      hipPointerAttribute_t pa;
      std::memset(&pa, 0, sizeof(pa));
      const hipError_t pe = hipPointerGetAttributes(&pa, va);
      (void)hipGetLastError();
      std::printf("  virtual-memory mapping: hipPointerGetAttributes %s, type %d\n", hipGetErrorString(pe), (int)pa.type);
      CHECK_OK(h, mdp_make_index(h, n * B, (int32_t*)va));
      CHECK_OK(h, mdp_sample_rows(h, (const int32_t*)va, B, rows));
      CHECK_OK(h, mdp_synchronize(h));
      HIP_OR_DIE(hipMemUnmap(va, sz));
      HIP_OR_DIE(hipMemAddressFree(va, sz));
      HIP_OR_DIE(hipMemRelease(mh));
    } else {
      (void)hipGetLastError();
      std::printf("  virtual-memory mapping: not supported here, skipped\n");
    }
  }
  // an arena in host memory: mdp_create fails, and the failed handle refuses everything
  {
    int64_t pt = 0;
    const int64_t need = mdp_arena_bytes(&c, &pt);
    if (need > 0 && (size_t)need <= big) {
      mdp_handle* hh = nullptr;
      CHECK(mdp_create(&c, hb, need, nullptr, &hh) < 0);
      CHECK(hh != nullptr && std::strstr(mdp_last_error(hh), "arena_dev") != nullptr);
      null_handle_entries(hh);
      CHECK(mdp_destroy(hh) == 0);
    }
  }
  std::free(hb);
  CHECK_OK(h, mdp_synchronize(h));  // nothing faulted, nothing was launched
}

static void lifecycle(const mdp_config& c, const char* name) {
  std::printf("gpu lifecycle: %s\n", name);
  std::fflush(stdout);
  const int n = c.n_agents, B = c.batch_size, E = c.num_envs;
  int64_t pt = 0;
  const int64_t bytes = mdp_arena_bytes(&c, &pt);
  CHECK(bytes > 0);
  void* arena = nullptr;
  HIP_OR_DIE(hipMalloc(&arena, bytes));
  hipStream_t s;
  HIP_OR_DIE(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  mdp_handle* h = nullptr;
  CHECK_OK(h, mdp_create(&c, arena, bytes, s, &h));
  if (!h || mdp_buffer_len(h) != 0) {
    std::fprintf(stderr, "create failed: %s\n", mdp_last_error(h));
    std::exit(4);
  }
  CHECK(mdp_stream(h) == (void*)s);

  // layout queries
  int64_t off = -1, rb = -1, prev_end = 0;
  for (int r = 0; r < MDP_R_COUNT; ++r) {
    CHECK_OK(h, mdp_region(h, r, &off, &rb));
    CHECK(off >= prev_end && off + rb <= bytes);
    prev_end = off + rb;
  }
  CHECK(mdp_region(h, MDP_R_COUNT, &off, &rb) < 0);
  int32_t lay[6];
  for (int i = 0; i < n; ++i) CHECK_OK(h, mdp_row_layout(h, i, lay));
  CHECK(mdp_row_layout(h, n, lay) < 0);
  mdp_tensor_info ti;
  CHECK(mdp_tensor(h, 0, 0, 6, &ti) < 0);
  CHECK(mdp_tensor(h, 0, 0, 0, nullptr) < 0);
  const int stride = lay[5];

  // parameters: deterministic small values, read back exactly
  uint64_t seed = 12345;
  for (int i = 0; i < n; ++i)
    for (int w = MDP_ACTOR; w <= MDP_TGT_CRITIC; ++w) {
      const int64_t nf = net_floats(h, i, (w == MDP_CRITIC || w == MDP_TGT_CRITIC) ? 1 : 0);
      CHECK(nf > 0);
      std::vector<float> p(nf), q(nf, -1.f);
      for (auto& x : p) x = ((float)(lcg(seed) % 20001) - 10000.f) * 1e-5f;
      CHECK_OK(h, mdp_set_params(h, i, w, p.data(), nf));
      CHECK_OK(h, mdp_get_params(h, i, w, q.data(), nf));
      CHECK(std::memcmp(p.data(), q.data(), 4 * nf) == 0);
      CHECK_ERR(h, mdp_set_params(h, i, w, p.data(), nf - 1));  // count mismatch
    }
  {
    std::vector<float> p(8);
    CHECK_ERR(h, mdp_set_params(h, 0, 10, p.data(), 8));  // bad set id
    CHECK_ERR(h, mdp_set_params(h, n, 0, p.data(), 8));   // bad agent
    float b2[2];
    CHECK_OK(h, mdp_get_beta_powers(h, 0, 1, b2));
    CHECK(b2[0] == c.adam_b1 && b2[1] == c.adam_b2);
    CHECK_OK(h, mdp_set_beta_powers(h, 0, 1, b2));
  }

  // index stream: seed, state round trip
  CHECK_OK(h, mdp_seed_py_random(h, 1234));
  std::vector<uint32_t> st(625), st2(625);
  CHECK_OK(h, mdp_get_rng_state(h, st.data()));
  CHECK(st[624] == 624);
  CHECK_OK(h, mdp_set_rng_state(h, st.data()));
  CHECK_OK(h, mdp_get_rng_state(h, st2.data()));
  CHECK(st == st2);
  st2[624] = 625;
  CHECK_ERR(h, mdp_set_rng_state(h, st2.data()));
  CHECK_ERR(h, mdp_set_rng_state(h, nullptr));

  // training loop: fill the ring to the update gate (B x max_episode_len rows)
  CHECK_OK(h, mdp_env_reset(h));
  const int64_t gate_rows = (int64_t)B * c.max_episode_len;
  while (mdp_buffer_len(h) < gate_rows) CHECK_OK(h, mdp_train_step(h, 0));
  CHECK(mdp_update_gate(h, 99) == 1);
  CHECK(mdp_update_gate(h, 100) == 0);
  for (int k = 0; k < 3; ++k) CHECK_OK(h, mdp_train_step(h, 1 + k % 2));  // eager, then captured graphs
  const int32_t ks[3] = {1, 2, 1};
  CHECK_OK(h, mdp_train_steps(h, 3, ks, 0));  // capture only
  CHECK_OK(h, mdp_train_steps(h, 3, ks, 1));
  CHECK_OK(h, mdp_synchronize(h));
  CHECK_ERR(h, mdp_train_step(h, 65));
  CHECK_ERR(h, mdp_train_steps(h, 0, ks, 1));
  const int32_t kbad[2] = {1, 70};
  CHECK_ERR(h, mdp_train_steps(h, 2, kbad, 1));
  double stats[6];
  for (int i = 0; i < n; ++i) {
    CHECK_OK(h, mdp_get_stats(h, i, stats));
    CHECK(all_finite(stats, 6));
  }
  {
    int64_t bad = -1;
    CHECK_OK(h, mdp_check_finite(h, &bad));
    CHECK(bad == 0);
    CHECK_ERR(h, mdp_check_finite(h, nullptr));
  }

  // device buffers for the per-call paths
  int32_t* idx = nullptr;
  float *rows = nullptr, *obs = nullptr, *act = nullptr, *q = nullptr, *u = nullptr, *info = nullptr;
  HIP_OR_DIE(hipMalloc((void**)&idx, 4 * (size_t)n * B));
  HIP_OR_DIE(hipMalloc((void**)&rows, 4 * (size_t)B * stride));
  HIP_OR_DIE(hipMalloc((void**)&obs, 4 * (size_t)B * 256));
  HIP_OR_DIE(hipMalloc((void**)&act, 4 * (size_t)B * 8));
  HIP_OR_DIE(hipMalloc((void**)&q, 4 * (size_t)B));
  HIP_OR_DIE(hipMalloc((void**)&u, 4 * (size_t)(n + 1) * B * 5));
  HIP_OR_DIE(hipMalloc((void**)&info, 4 * (size_t)E * n * MDP_BENCH_W));
  HIP_OR_DIE(hipMemset(obs, 0, 4 * (size_t)B * 256));
  {
    std::vector<float> hu((size_t)(n + 1) * B * 5);
    for (auto& x : hu) x = ((float)(lcg(seed) % 65535) + 1.f) / 65537.f;
    HIP_OR_DIE(hipMemcpy(u, hu.data(), 4 * hu.size(), hipMemcpyHostToDevice));
  }
  host_pointers_refused(h, c, idx, rows, obs, act, q, u, info);
  CHECK_OK(h, mdp_make_index(h, n * B, idx));
  CHECK_ERR(h, mdp_make_index(h, -1, idx));
  CHECK_OK(h, mdp_sample_rows(h, idx, B, rows));
  CHECK_OK(h, mdp_act(h, 0, 0, obs, act, B, nullptr));
  CHECK_OK(h, mdp_act(h, 0, 1, obs, act, B, u));
  CHECK_OK(h, mdp_actor_logits(h, n - 1, 1, obs, act, B));
  CHECK_OK(h, mdp_q_values(h, 0, 0, rows, q, B));
  CHECK_OK(h, mdp_update(h, 0, idx, u, u + (size_t)n * B * 5));
  CHECK_OK(h, mdp_update(h, n - 1, nullptr, nullptr, nullptr));
  CHECK(mdp_agent_update(h, 0, 99, idx, u, stats) == 1);  // gated: t % 100 != 0
  CHECK_OK(h, mdp_agent_update(h, 0, 100, idx, u, stats));
  CHECK(all_finite(stats, 6));
  CHECK_OK(h, mdp_agent_update(h, n - 1, 200, nullptr, nullptr, stats));
  CHECK(mdp_agent_update(h, 0, 100, idx, u, nullptr) < 0);
  CHECK(mdp_grad_variant(h, 0) == 0 || mdp_grad_variant(h, 0) == 1);
  // the phase entry points (data-parallel order, one replica)
  CHECK_OK(h, mdp_critic_grad(h, 0, idx, u));
  CHECK_OK(h, mdp_reduce_grad(h, 0, 1));
  CHECK_OK(h, mdp_apply_grad(h, 0, 1, 1.f));
  CHECK_OK(h, mdp_actor_grad(h, 0, idx, u + (size_t)n * B * 5));
  CHECK_OK(h, mdp_reduce_grad(h, 0, 0));
  CHECK_OK(h, mdp_apply_grad(h, 0, 0, 1.f));
  CHECK_ERR(h, mdp_critic_grad(h, 0, nullptr, u));
  CHECK_ERR(h, mdp_actor_grad(h, 0, nullptr, u));
  // rounds: graphs on / off, profiled
  CHECK_OK(h, mdp_update_round(h));
  CHECK_OK(h, mdp_update_round(h));
  CHECK_OK(h, mdp_set_graphs(h, 0));
  CHECK_OK(h, mdp_update_round(h));
  CHECK_OK(h, mdp_train_step(h, 1));
  CHECK_OK(h, mdp_set_graphs(h, 1));
  for (int k = 0; k < MDP_K_COUNT; ++k) CHECK_OK(h, mdp_prof_enable(h, k, 1));
  CHECK_OK(h, mdp_train_step(h, 2));
  double ms = -1;
  int64_t launches = -1;
  CHECK_OK(h, mdp_prof_read(h, MDP_K_ROLLOUT, &ms, &launches));
  CHECK(launches == 1 && ms > 0);
  CHECK_OK(h, mdp_prof_read(h, MDP_K_CRITIC_GRAD, &ms, &launches));
  CHECK(launches >= n);
  for (int k = 0; k < MDP_K_COUNT; ++k) CHECK_OK(h, mdp_prof_enable(h, k, 0));
  CHECK_ERR(h, mdp_prof_enable(h, MDP_K_COUNT, 1));
  CHECK_ERR(h, mdp_prof_read(h, -1, &ms, &launches));

  // env: state round trip, observations, benchmark records, the episode log
  {
    const int ne = n + (c.scenario == MDP_SCN_SPREAD ? n : c.scenario == MDP_SCN_TAG ? 2 : n - 1);
    std::vector<float> pos((size_t)E * ne * 2), vel(pos.size());
    std::vector<int32_t> goal(E), eps(E);
    CHECK_OK(h, mdp_env_get_state(h, pos.data(), vel.data(), goal.data(), eps.data()));
    CHECK_OK(h, mdp_env_set_state(h, pos.data(), vel.data(), goal.data(), eps.data()));
    CHECK_OK(h, mdp_env_get_state(h, nullptr, nullptr, nullptr, nullptr));
    float* eobs = nullptr;
    HIP_OR_DIE(hipMalloc((void**)&eobs, 4 * (size_t)E * 256 * n));
    CHECK_OK(h, mdp_env_obs(h, eobs));
    CHECK_OK(h, mdp_env_step_bench(h, info));
    CHECK_ERR(h, mdp_env_step_bench(h, nullptr));
    CHECK_OK(h, mdp_env_step(h, nullptr, nullptr));
    CHECK_OK(h, mdp_synchronize(h));
    const int64_t eps_done = mdp_episode_count(h);
    CHECK(eps_done >= E);
    std::vector<float> log((size_t)4 * (1 + n));
    CHECK_OK(h, mdp_episode_log(h, eps_done - 4, 4, log.data()));
    CHECK_ERR(h, mdp_episode_log(h, 0, int64_t(1) << 40, log.data()));
    CHECK_ERR(h, mdp_episode_log(h, -1, 1, log.data()));
    HIP_OR_DIE(hipFree(eobs));
  }
  // replay buffer entry points
  {
    CHECK_ERR(h, mdp_buffer_add_rows(h, rows, -1));
    CHECK_OK(h, mdp_buffer_add_rows(h, rows, 0));
    CHECK_OK(h, mdp_buffer_add_rows(h, rows, B));
    int64_t* pos = nullptr;
    HIP_OR_DIE(hipMalloc((void**)&pos, 8 * (size_t)B));
    std::vector<int64_t> hp(B);
    for (int b = 0; b < B; ++b) hp[b] = b;
    HIP_OR_DIE(hipMemcpy(pos, hp.data(), 8 * (size_t)B, hipMemcpyHostToDevice));
    CHECK_OK(h, mdp_buffer_put_agent(h, 0, pos, rows, B));
    CHECK_ERR(h, mdp_buffer_set_len(h, c.capacity + 1, 0));
    CHECK_ERR(h, mdp_buffer_set_len(h, 10, c.capacity));
    const int64_t len = mdp_buffer_len(h);
    CHECK_OK(h, mdp_buffer_set_len(h, len, len % c.capacity));
    CHECK_OK(h, mdp_synchronize(h));
    HIP_OR_DIE(hipFree(pos));
  }
  // data parallelism: none wired; the xGMI set-up refuses out-of-order calls
  {
    int32_t d4[4] = {-1, -1, -1, -1};
    CHECK_OK(h, mdp_dp_info(h, d4));
    CHECK(d4[0] == 0);
    uint8_t hs[MDP_XGMI_HANDLE_BYTES * 2] = {};
    CHECK_ERR(h, mdp_dp_xgmi_connect(h, hs));
    CHECK_ERR(h, mdp_dp_xgmi_probe(h, d4));
    CHECK_ERR(h, mdp_dp_xgmi_enable(h));
    double x4[4];
    CHECK_OK(h, mdp_dp_exchange_stats(h, x4, 1));
    CHECK_OK(h, mdp_dp_exchange_stats_enable(h, 0));
  }
  // throughput mode: injected and drawn rounds, graph replay
  CHECK_ERR(h, mdp_set_update_mode(h, 2));
  CHECK_ERR(h, mdp_update_all(h, nullptr, nullptr, nullptr));  // strict mode still
  CHECK_OK(h, mdp_set_update_mode(h, 1));
  {
    float* ut = nullptr;
    HIP_OR_DIE(hipMalloc((void**)&ut, 4 * (size_t)n * n * B * 5));
    HIP_OR_DIE(hipMemset(ut, 0, 4 * (size_t)n * n * B * 5));
    std::vector<float> hu((size_t)n * n * B * 5);
    for (auto& x : hu) x = ((float)(lcg(seed) % 65535) + 1.f) / 65537.f;
    HIP_OR_DIE(hipMemcpy(ut, hu.data(), 4 * hu.size(), hipMemcpyHostToDevice));
    CHECK_OK(h, mdp_update_all(h, idx, ut, u));
    CHECK_OK(h, mdp_update_all(h, nullptr, nullptr, nullptr));
    HIP_OR_DIE(hipFree(ut));
  }
  CHECK_OK(h, mdp_update_round(h));
  CHECK_OK(h, mdp_update_round(h));
  for (int k = 0; k < 3; ++k) CHECK_OK(h, mdp_train_step(h, 2));
  CHECK_OK(h, mdp_set_update_mode(h, 0));
  CHECK_OK(h, mdp_train_step(h, 1));
  CHECK_OK(h, mdp_synchronize(h));
  for (int i = 0; i < n; ++i) {
    CHECK_OK(h, mdp_get_stats(h, i, stats));
    CHECK(all_finite(stats, 6));
  }
  // a live handle survives every refused call above
  CHECK(mdp_buffer_len(h) > 0);
  CHECK_OK(h, mdp_destroy(h));
  HIP_OR_DIE(hipFree(idx));
  HIP_OR_DIE(hipFree(rows));
  HIP_OR_DIE(hipFree(obs));
  HIP_OR_DIE(hipFree(act));
  HIP_OR_DIE(hipFree(q));
  HIP_OR_DIE(hipFree(u));
  HIP_OR_DIE(hipFree(info));
  HIP_OR_DIE(hipStreamDestroy(s));
  HIP_OR_DIE(hipFree(arena));
}

static void gpu_mode() {
  int dev = 0;
  HIP_OR_DIE(hipGetDeviceCount(&dev));
  HIP_OR_DIE(hipSetDevice(0));
  std::printf("hip runtime up: %d device(s)\n", dev);
  std::fflush(stdout);
  // S2 shape at a small batch: the register-resident H=64 kernels
  lifecycle(base_config(MDP_SCN_SPREAD, 3, 0, 64, 256, 256), "simple_spread N=3 H=64 B=256 E=256");
  // S5 shape at a small batch: the general H=128 kernels, 6 agents
  lifecycle(base_config(MDP_SCN_TAG, 6, 4, 128, 256, 64), "simple_tag N=6 H=128 B=256 E=64");
  // ragged batch, a DDPG agent, --num-units padded to the kernel width
  mdp_config c = base_config(MDP_SCN_ADVERSARY, 3, 1, 50, 200, 32);
  c.local_q[0] = 1;
  lifecycle(c, "simple_adversary N=3 ddpg adversary H=50 B=200 E=32");
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "cpu";
  if (std::strcmp(mode, "cpu") == 0) {
    cpu_mode();
  } else if (std::strcmp(mode, "gpu") == 0) {
    cpu_mode();
    std::printf("cpu checks done (%d)\n", g_checks);
    std::fflush(stdout);
    gpu_mode();
  } else {
    std::fprintf(stderr, "usage: %s cpu|gpu\n", argv[0]);
    return 2;
  }
  // (flushed here: a LeakSanitizer report at exit leaves without flushing stdio)
  if (g_fail) {
    std::printf("FAILED %d of %d checks\n", g_fail, g_checks);
    std::fflush(stdout);
    return 1;
  }
  std::printf("OK %d checks (%s)\n", g_checks, mode);
  std::fflush(stdout);
  return 0;
}
