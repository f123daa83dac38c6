// mdp_apply_fused.hip -- one launch for the batch reduction + optimizer step
// of one net.  Single GPU: phase 0.  Data parallel over RCCL: phase 1 (reduce
// into grad[]) -> ncclAllReduce -> phase 2 (step).  Data parallel over the
// direct xGMI exchange: phase 3, still ONE launch -- each chunk workgroup
// pushes its reduced chunk to every peer and sums the world's chunks in rank
// order before the clip/Adam below (xchg_chunk, LL protocol).
//
// Workgroup (tensor t, chunk c) of 256 parameters, 1024 threads: 16 groups of
// 64 threads each sum a quarter-ish of the per-workgroup partial gradients of
// the chunk (float4 columns), combined in LDS in a fixed order (deterministic).
// clip_by_norm needs the norm of the WHOLE tensor (tf_util.py:177-182): every
// chunk publishes its fp64 sum of squares as two agent-scope 64-bit stores of
// (epoch << 32 | half of the bits); all chunks of the tensor poll the pairs
// until both tags carry this step's epoch and sum them in chunk order, so
// every chunk derives the identical norm.  The epoch (sync counter 7 of the
// net) is read at the start and advanced by the last workgroup, so the slots
// never need a reset and a stale pair never carries the awaited tag.
// The host launches it only when the whole grid is co-resident (grid <= CUs x
// resident workgroups per CU, mdp_ra_fits; otherwise k_reduce + k_apply);
// every spin is bounded and records a fault in Ctl instead of hanging, and
// once a fault is recorded no launch writes the optimizer state any more (a
// faulted step leaves m, v, theta, targets and the beta powers untouched).
//
// Then TF1 ApplyAdam on the chunk (+ Polyak of the chunk for the actor step),
// Polyak workgroups of the other net, the stats workgroup -- exactly as k_apply
// -- and the last workgroup to finish advances the beta powers (the
// AdamOptimizer._finish update) and, for the actor step, the noise counter.
#include "mdp_device.h"
#include "mdp_kernels.h"
#include "mdp_mt.h"

namespace {
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kSpinLimit = 1u << 22;

__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a peer that has not arrived after 30 s (s_memrealtime runs at 100 MHz)
// is taken to be gone: the wait records Ctl::fault = 2 and gives up, and later
// exchanges skip their waits (the host reports the fault at the next sync)
constexpr uint64_t kXchgTimeoutTicks = 30ull * 100000000ull;

__device__ __forceinline__ uint64_t ll_word(float v, uint32_t ep) {
  return ((uint64_t)ep << 32) | (uint64_t)__float_as_uint(v);
}

// The xGMI exchange of 4 parameters per lane at param-space offset i0 (LL
// protocol, see XchgDesc), run by ONE wave.  g: this rank's reduced values;
// returns the sum over ranks in rank order (identical on every rank).  A
// bounded wait (30 s on the 100 MHz real-time clock) records *fault = 2 and
// gives up; once a fault is recorded later exchanges do not wait.
// The descriptor is read into (uniform) registers once, before any atomic
// (re-reading it after each one serialised a round trip per peer), and the
// exchange words are addressed as global memory (not FLAT): every peer's
// stores and every word's load issue back to back, one round trip per poll.
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// wstat (optional): Ctl::xw_ticks -- lane 0 adds this chunk's wait (ticks
// from its stores to the last peer word's arrival), the count and the maximum
__device__ __forceinline__ f32x4 xchg_chunk(const XchgDesc* xdp, uint32_t* fault, f32x4 g, int64_t i0, bool act,
                                           uint32_t ep, uint64_t* wstat = nullptr) {
  const int W = __builtin_amdgcn_readfirstlane(xdp->world), r = __builtin_amdgcn_readfirstlane(xdp->rank);
  const int64_t pt = (int64_t)uni64((uint64_t)xdp->pt);
  uint64_t base[MDP_XCH_MAXW];
#pragma unroll
  for (int q = 0; q < MDP_XCH_MAXW; ++q) base[q] = uni64((uint64_t)xdp->data[q]);  // all slots: no per-slot branch
  const int64_t slot_row = (int64_t)(ep & 1u) * W;
  if (act) {
#pragma unroll
    for (int q = 0; q < MDP_XCH_MAXW; ++q) {
      if (q < W && q != r) {
        gu64* dst = reinterpret_cast<gu64*>(base[q]) + (slot_row + r) * pt + i0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __hip_atomic_store(dst + j, ll_word(g[j], ep), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  const bool gone = __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  const gu64* mine = reinterpret_cast<const gu64*>(base[r]) + slot_row * pt + i0;
  // every peer's 4 words in flight at once (one round trip for the whole
  // world, not one per peer), re-read together until all carry this epoch
  float pv[MDP_XCH_MAXW][4];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    uint64_t w[MDP_XCH_MAXW][4];
#pragma unroll
    for (int q = 0; q < MDP_XCH_MAXW; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[q][j] = (uint64_t)ep << 32;
        if (q < W && q != r && act)
          w[q][j] = __hip_atomic_load(const_cast<gu64*>(mine + q * pt + j), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    bool all = true;
#pragma unroll
    for (int q = 0; q < MDP_XCH_MAXW; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pv[q][j] = __uint_as_float((uint32_t)w[q][j]);
        all = all && (uint32_t)(w[q][j] >> 32) == ep;
      }
    }
    if (all || gone) break;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kXchgTimeoutTicks) {
      __hip_atomic_store(fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  if (wstat && act && (threadIdx.x & 63) == 0) {
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
    __hip_atomic_fetch_add(wstat, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(wstat + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(wstat + 2, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the world's sum in rank order (identical on every rank)
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < MDP_XCH_MAXW; ++q) {
    if (q < W) {
      f32x4 v = g;
      if (q != r && act) v = f32x4{pv[q][0], pv[q][1], pv[q][2], pv[q][3]};
      s = q == 0 ? v : s + v;
    }
  }
  return act ? s : g;
}
}  // namespace

// connection probe: word i of the probe area carries (q + 1) * 4096 +
// ((i + 7 ep) % 4096) from rank q (exact in fp32), so the world sum is known
// in closed form and differs between the epochs that reuse a slot
__global__ __launch_bounds__(64) void k_xchg_probe(const XchgDesc* xd, uint32_t ep, uint32_t* bad, uint32_t* fault) {
  const XchgDesc& x = *xd;
  const int64_t p0 = (int64_t)blockIdx.x * 256 + 4 * threadIdx.x;  // within the probe area
  f32x4 g, want;
  for (int j = 0; j < 4; ++j) {
    const float base = (float)((p0 + j + 7 * (int64_t)ep) % 4096);
    g[j] = (float)((x.rank + 1) * 4096) + base;
    float w = 0.f;
    for (int q = 0; q < x.world; ++q) w += (float)((q + 1) * 4096) + base;
    want[j] = w;
  }
  const f32x4 s = xchg_chunk(xd, fault, g, x.pt - MDP_XCH_PROBE + p0, true, ep);
  uint32_t nbad = 0;
  for (int j = 0; j < 4; ++j) nbad += s[j] != want[j] ? 1u : 0u;
  if (nbad) atomicAdd(bad, nbad);
}

hipError_t mdp_launch_xchg_probe(const XchgDesc* xd, uint32_t ep, int nchunk, uint32_t* bad, uint32_t* fault,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_xchg_probe, dim3(nchunk), dim3(64), 0, s, xd, ep, bad, fault);
  return hipGetLastError();
}

// diagnostic build only: per-workgroup phase stamps of the last critic-step
// (sel 0) and actor-step (sel 1) optimizer launch (tools/ra_budget.py)
#ifdef MDP_STAMPS
__device__ unsigned long long g_ra_ph[2][1024][8];
#define MDP_RA_PH(k)                                                                                     \
  do {                                                                                                   \
    if (threadIdx.x == 0 && b < 1024) g_ra_ph[a.stats_mode == 1 ? 0 : 1][b][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" int mdp_debug_ra_phases(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ra_ph), sizeof(g_ra_ph)) == hipSuccess ? 0 : -1;
}
extern "C" int mdp_debug_ra_phases_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_ra_ph)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(unsigned long long) * 2 * 1024 * 8) == hipSuccess && hipDeviceSynchronize() == hipSuccess
             ? 0 : -1;
}
#else
#define MDP_RA_PH(k) \
  do {               \
  } while (0)
#endif

// ((r0 + r1) + (r2 + r3)) + ... over rows [LO, LO + N) of the group sums
// (compile-time indices: a private array here stayed in scratch)
template <int LO, int N>
__device__ __forceinline__ f32x4 red_tree(const f32x4 (*red)[64], int col) {
  if constexpr (N == 1)
    return red[LO][col];
  else
    return red_tree<LO, N / 2>(red, col) + red_tree<LO + N / 2, N / 2>(red, col);
}

// b: this workgroup's index among the nb workgroups of this net's step;
// G waves (G = 16: 1024-thread workgroups; G = 4: 256 threads, used exactly
// when nwg <= 64 -- a launch of fewer waves dispatches sooner).  Wave q sums
// partials w = q, q + G, ..., then a fixed tree over the waves: the summation
// order is a function of nwg alone (every launch of a configuration agrees)
template <int G>
__device__ __forceinline__ void reduce_apply_body(const FusedApplyArgs& f, const int b, const uint32_t nb) {
  const ApplyArgs& a = f.ap;
  __shared__ f32x4 red[G][64];
  __shared__ f32x4 gl[64];         // the chunk's reduced gradient (wave 0 -> the Adam waves)
  __shared__ float step_l[4];      // beta1^t, beta2^t, the tensor norm, fault
  const int tid = threadIdx.x, lane = tid & 63;
  MDP_STAMP(30);
  MDP_RA_PH(0);
  if (f.phase == 1 && b >= f.rblk[6]) return;  // reduce-only pass: chunk workgroups only
  if (b < f.rblk[6]) {
    int t = 0;
    while (b >= f.rblk[t + 1]) ++t;
    const TDesc td = a.net.t[t];
    const int n = td.rows * td.cols;
    const int nch = f.rblk[t + 1] - f.rblk[t];
    const int c = b - f.rblk[t];
    const int col = tid & 63, grp = tid >> 6;
    const int p0 = c * MDP_RA_CHUNK + 4 * col;  // this thread's 4 parameters (tensor-relative)
    const bool act = p0 < n;
    const int64_t i0 = td.off + p0;             // absolute parameter index
    // The Adam step runs on waves 0..3, wave q on parameters 64 q .. 64 q + 63
    // of the chunk (one per lane, contiguous): on wave 0 alone, four parameters
    // per lane of divides and square roots took 0.7 us of VALU issue (stamped).
    // Its state is requested with the partial-gradient loads.
    const int pq = c * MDP_RA_CHUNK + 64 * grp + lane;
    const bool aact = grp < 4 && pq < n;
    const int64_t iq = td.off + pq;
    float m1 = 0.f, v1 = 0.f, th1 = 0.f, tg1 = 0.f;
    const float b1p = a.beta[0], b2p = a.beta[1];  // this step's powers (wave 0; advanced at the end)
    // exchange epoch (advanced at the end); kept opaque until the exchange --
    // the +1 here made the compiler wait for the load in front of the partials
    const uint32_t ep_raw = f.phase == 3 ? f.xstep[0] : 0u;
    const uint32_t nep = f.sync_ctr[7 * 32] + 1u;                // norm-handshake epoch (advanced at the end)
    // a fault recorded by an earlier launch, read with the first loads (not
    // after the handshake, where its round trip would sit in front of Adam)
    // (kept an opaque VGPR until the step: compared here, the compiler waited
    // for the load in front of the partial loads)
    uint32_t fault0 = 0u;
    if (grp == 0) fault0 = __hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool faulted = false;
    if (aact && f.phase != 1) {
      m1 = a.m[iq];
      v1 = a.v[iq];
      th1 = a.theta[iq];
      if (a.polyak) tg1 = a.target[iq];
    }
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if constexpr (G == 16) {
      if (f.phase == 2) {  // step from the all-reduced gradient in grad[]
        if (grp == 0 && act) s = ld4(a.grad + i0);
      } else if (act) {
        const float* base = a.slab + (td.off - a.net.off) + p0;
        // partials w = grp + 16 k: up to 16 loads (B <= 4096) in flight at
        // once, summed in the fixed order ((v0 + v1) + v2) + v3, then v4, v5, ...
        f32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int w = grp + 16 * k;
          v[k] = w < a.nwg ? ld4(base + (int64_t)w * a.slab_stride) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        s = ((v[0] + v[1]) + v[2]) + v[3];
#pragma unroll
        for (int k = 4; k < 16; ++k)
          if (grp + 16 * k < a.nwg) s += v[k];
        for (int w = grp + 256; w < a.nwg; w += 16) s += ld4(base + (int64_t)w * a.slab_stride);
      }
      red[grp][col] = s;
    } else {
      static_assert(G == 4, "narrow launch: 4 waves");
      // nwg <= 64 (host-checked): wave grp sums partials w = grp + 4 k, all 16
      // loads issued unconditionally (a partial past nwg re-reads the last one
      // and is dropped by the select: a guarded load compiled to a branch per
      // load), in the order ((v0 + v1) + v2) + v3, then v4, v5, ...
      if (f.phase == 2) {
        if (grp == 0 && act) s = ld4(a.grad + i0);
      } else if (act) {
        const float* base = a.slab + (td.off - a.net.off) + p0;
        f32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = ld4(base + (int64_t)min(grp + 4 * k, a.nwg - 1) * a.slab_stride);
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (grp + 4 * k >= a.nwg) v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        s = ((v[0] + v[1]) + v[2]) + v[3];
#pragma unroll
        for (int k = 4; k < 16; ++k)
          if (grp + 4 * k < a.nwg) s += v[k];
      }
      red[grp][col] = s;
    }
    __syncthreads();
    MDP_STAMP(31);
    MDP_RA_PH(1);
    if (grp == 0 && f.phase != 1 && a.stats_mode) {
      // arrival: this workgroup has its step's beta powers and epochs in
      // registers (loaded first, vmcnt drained), so the stats workgroup may
      // advance them -- a fire-and-forget add instead of a returning atomic at
      // the end of every workgroup
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(f.done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (grp == 0) {
      // the G group sums as a fixed pairwise tree: every LDS read issued at
      // once, log2 G dependent adds (a chain over the groups waited on each read)
      f32x4 g = red_tree<0, G>(red, col);
      MDP_STAMP(34);
      if (f.phase == 3) g = xchg_chunk(f.xd, &a.ctl->fault, g, i0, act, ctr_use(ep_raw) + 1u, f.wstat);
      double ss = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gs = g[j] * a.scale;
        if (p0 + j < n) ss += (double)gs * (double)gs;
      }
      ss = wave_sum_d(ss);
      MDP_STAMP(35);
      MDP_RA_PH(2);
      // the norm handshake's publish goes out first (its round trip is the
      // launch's longest wait), the reduced-gradient stores behind it
      uint64_t* part = f.sync_part + (int64_t)t * MDP_RA_MAXCH * 2;
      const uint64_t tag = (uint64_t)nep << 32;
      if (f.phase != 1 && nch > 1 && lane == 0) {
        // this chunk's fp64 sum of squares as two epoch-tagged 64-bit words
        // (high and low half) -- data and flag in one store, no counter RMW
        const uint64_t bits = (uint64_t)__double_as_longlong(ss);
        st_agent64(part + 2 * c, tag | (bits >> 32));
        st_agent64(part + 2 * c + 1, tag | (bits & 0xffffffffull));
      }
      if (act && f.phase != 2) {
        if (p0 + 3 < n) {
          *reinterpret_cast<f32x4*>(a.grad + i0) = g;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (p0 + j < n) a.grad[i0 + j] = g[j];
        }
      }
      MDP_STAMP(36);
      MDP_RA_PH(3);
      double tot = ss;
      if (f.phase != 1) {  // phase 1 (data parallel) stops here: the all-reduce follows
      if (nch > 1) {
        // read every chunk's pair (published above) back once both tags carry
        // this step's epoch (bounded spin -> Ctl::fault = 1)
        MDP_STAMP(32);
        tot = 0.0;
        for (int q = lane; q < nch; q += 64) {
          uint64_t hi = ld_agent64(part + 2 * q), lo = ld_agent64(part + 2 * q + 1);
          uint32_t it = 0;
          while ((uint32_t)(hi >> 32) != nep || (uint32_t)(lo >> 32) != nep) {
            __builtin_amdgcn_s_sleep(1);
            if (++it > kSpinLimit) {
              __hip_atomic_store(&a.ctl->fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              faulted = true;
              break;
            }
            hi = ld_agent64(part + 2 * q);
            lo = ld_agent64(part + 2 * q + 1);
          }
          tot += __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
        }
        tot = wave_sum_d(tot);
      }
      // a timed-out handshake of this chunk, exchange of this launch or an
      // earlier launch's fault leaves the optimizer state as it was (a chunk
      // that saw every word of its tensor has the right norm and steps)
      faulted = __ballot(faulted || ctr_use(fault0) != 0u) != 0ull;
      if (f.phase == 3)
        faulted = faulted || __hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      MDP_STAMP(37);
      MDP_RA_PH(4);
      // the chunk's gradient, this step's powers, the norm and the fault state
      // to the Adam waves
      gl[col] = g;
      if (lane == 0) {
        step_l[0] = b1p;
        step_l[1] = b2p;
        step_l[2] = (float)sqrt(tot);
        step_l[3] = faulted ? 1.f : 0.f;
      }
      }  // phase != 1
    }
    if (f.phase != 1) {
      __syncthreads();
      // TF1 ApplyAdam (+ Polyak for the actor step) of this lane's parameter
      // (a timed-out handshake of this chunk, exchange of this launch or an
      // earlier launch's fault leaves the optimizer state as it was)
      if (aact && step_l[3] == 0.f) {
        const float gq = reinterpret_cast<const float*>(gl)[64 * grp + lane];
        const float norm = step_l[2];
        const float clip = a.clip;
        const float denom = fmaxf(norm, clip);
        const float one = 1.0f;
        const float alpha = a.lr * sqrtf(one - step_l[1]) / (one - step_l[0]);
        const float c1 = one - a.b1, c2 = one - a.b2;
        const float gc = ((gq * a.scale) * clip) / denom;
        const float mo = m1 + (gc - m1) * c1;
        const float vo = v1 + (gc * gc - v1) * c2;
        const float tho = th1 - (mo * alpha) / (sqrtf(vo) + a.eps);
        a.m[iq] = mo;
        a.v[iq] = vo;
        a.theta[iq] = tho;
        if (a.polyak) a.target[iq] = a.pa * tg1 + a.pb * tho;
      }
    }
  } else if (a.polyak && b < f.rblk[6] + a.oblk[6]) {
    if (__hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const int bb = b - f.rblk[6];
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
  } else if (a.stats_mode && tid < 64) {
    // stats workgroup (maddpg.py:196), as in k_apply
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int w = tid;  // 4 workgroups' records in flight, summed in the sequential order
    for (; w + 3 * 64 < a.nwg; w += 4 * 64) {
      f64x4 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = *reinterpret_cast<const f64x4*>(a.slab_stat + (int64_t)(w + 64 * k) * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s0 += r[k][0];
        s1 += r[k][1];
        s2 += r[k][2];
        s3 += r[k][3];
      }
    }
    for (; w < a.nwg; w += 64) {
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
      int i = tid;  // 8 loads in flight, summed in the sequential order
      for (; i + 7 * 64 < a.B; i += 8 * 64) {
        double yv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) yv[k] = a.y[i + 64 * k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double d = yv[k] - mean_y;
          dv += d * d;
        }
      }
      for (; i < a.B; i += 64) {
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
  MDP_STAMP(33);
#ifdef MDP_STAMPS
  __syncthreads();  // (every wave's Adam / Polyak / stats stores issued)
#endif
  MDP_RA_PH(5);
  if (f.phase == 1) return;  // uniform: the whole grid of a reduce-only pass
  if (a.stats_mode) {
    // the stats workgroup advances the optimizer step once every chunk
    // workgroup has arrived (read this step's beta powers and epochs); the
    // grid is co-resident (mdp_ra_fits), the wait bounded
    if (b == f.rblk[6] + (a.polyak ? a.oblk[6] : 0) && tid == 0) {
      const uint32_t want = (uint32_t)f.rblk[6];
      uint32_t it = 0;
      while (__hip_atomic_load(f.done_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > kSpinLimit) {
          __hip_atomic_store(&a.ctl->fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      MDP_RA_PH(6);
      __hip_atomic_store(f.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        const float p1 = a.beta[0], p2 = a.beta[1];
        a.beta[2] = p1;
        a.beta[3] = p2;
        a.beta[0] = p1 * a.b1;
        a.beta[1] = p2 * a.b2;
      }
      if (a.bump_ctr) a.ctl->upd_ctr += (uint32_t)a.bump_ctr;
      if (f.phase == 3) f.xstep[0] += 1u;
      f.sync_ctr[7 * 32] += 1u;
      MDP_RA_PH(7);
    }
    return;
  }
  // (no stats workgroup) the last workgroup to finish advances the optimizer
  // step (every net workgroup read beta before its add)
  __syncthreads();
  if (tid == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(f.done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev % nb == nb - 1) {
      if (__hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        const float p1 = a.beta[0], p2 = a.beta[1];
        a.beta[2] = p1;
        a.beta[3] = p2;
        a.beta[0] = p1 * a.b1;
        a.beta[1] = p2 * a.b2;
      }
      if (a.bump_ctr) a.ctl->upd_ctr += (uint32_t)a.bump_ctr;
      if (f.phase == 3) f.xstep[0] += 1u;
      f.sync_ctr[7 * 32] += 1u;
    }
  }
}

// diagnostic build: every workgroup's start and end of the last launch (roles:
// chunk workgroups, Polyak, stats, the draw piece last) -- which role ends it
#ifdef MDP_STAMPS
__device__ unsigned long long g_ra_t0[1024], g_ra_t1[1024];
#define MDP_RA_WG(arr)                                                                 \
  do {                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 1024) arr[blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" int mdp_debug_ra_wg(unsigned long long* t0, unsigned long long* t1, int n) {
  if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_ra_t0), sizeof(unsigned long long) * n) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_ra_t1), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#else
#define MDP_RA_WG(arr) \
  do {                 \
  } while (0)
#endif


template <int NT>
__global__ __launch_bounds__(NT) void k_reduce_apply(FusedApplyArgs f) {
  MDP_RA_WG(g_ra_t0);
  MDP_TL(f.ap.ctl, f.ap.polyak ? 3 : 1, blockIdx.x == gridDim.x - 1 && f.pf_count > 0 ? 3 : 0);
  MDP_KARG_TOUCH("s"(f.pf_count), "s"(f.xstep), "s"(f.ap.blk[0]), "s"(f.ap.target), "s"(f.ap.clip), "s"(f.ap.stats_mode),
                 "s"(f.ap.ctl), "s"(gridDim.x), "s"(f.ap.net.t[0].off), "s"(f.ap.net.t[4].cols), "s"(f.ap.other.t[2].off),
                 "s"(f.ap.other.in));
  if (f.pf_count > 0 && blockIdx.x == gridDim.x - 1) {  // a piece of the next round's index draw
    make_index_block<NT>(f.pf_ctl, f.pf_count, f.pf_out);
    __syncthreads();
    MDP_RA_WG(g_ra_t1);
    return;
  }
  reduce_apply_body<NT / 64>(f, blockIdx.x, gridDim.x - (f.pf_count > 0 ? 1 : 0));
#ifdef MDP_STAMPS
  __syncthreads();
  MDP_RA_WG(g_ra_t1);
#endif
}

// throughput mode: the steps of several nets in one launch (each net's chunk
// workgroups handshake only among themselves; the nets are independent)
template <int NT>
__global__ __launch_bounds__(NT) void k_reduce_apply_batch(RaBatch rb) {
  if (rb.pf_count > 0 && blockIdx.x == gridDim.x - 1) {  // a piece of the next round's index draw
    make_index_block<NT>(rb.pf_ctl, rb.pf_count, rb.pf_out);
    return;
  }
  int q = 0;
  while (q + 1 < rb.count && (int)blockIdx.x >= rb.wg_start[q + 1]) ++q;
  const int b = blockIdx.x - rb.wg_start[q];
  reduce_apply_body<NT / 64>(rb.list[q], b, (uint32_t)(rb.wg_start[q + 1] - rb.wg_start[q]));
}

int mdp_ra_grid(const FusedApplyArgs& f) {
  const ApplyArgs& a = f.ap;
  return f.rblk[6] + (a.polyak ? a.oblk[6] : 0) + (a.stats_mode ? 1 : 0);
}

// 256-thread workgroups (4 waves of up to 16 partials) when the fan-in is at
// most 64 partials: S2 optimizer launch 3.88 -> 3.50 us event-timed (128
// threads: 4.17, 512: 3.64).  MDP_RA_NARROW=0 builds the 1024-thread launch
// for every fan-in (A/B only: its summation order differs)
#ifndef MDP_RA_NARROW
#define MDP_RA_NARROW 1
#endif
static bool mdp_ra_narrow(const FusedApplyArgs& f) { return MDP_RA_NARROW && f.ap.nwg <= 64; }

hipError_t mdp_launch_reduce_apply(const FusedApplyArgs& f, hipStream_t s) {
  const dim3 grid(mdp_ra_grid(f) + (f.pf_count > 0 ? 1 : 0));
  if (mdp_ra_narrow(f))
    mdp_launch(k_reduce_apply<256>, grid, dim3(256), 0, s, f);
  else
    mdp_launch(k_reduce_apply<1024>, grid, dim3(1024), 0, s, f);
  return hipGetLastError();
}

// the largest private segment (scratch bytes per lane) of the kernels whose
// workgroups spin on other workgroups of the same grid (the norm handshake, the
// xGMI exchange and its probe).  Their correctness rests on the whole grid being
// resident at once; waves that need scratch are dispatched only while the
// queue's scratch slots last, so a spinning grid must not use any (the build
// guard tools/check_scratch.py rejects it too; this is the run-time check)
hipError_t mdp_spin_kernels_scratch(int* bytes) {
  const void* ks[] = {(const void*)k_reduce_apply<256>, (const void*)k_reduce_apply<1024>,
                      (const void*)k_reduce_apply_batch<256>, (const void*)k_reduce_apply_batch<1024>,
                      (const void*)k_xchg_probe};
  *bytes = 0;
  for (const void* k : ks) {
    hipFuncAttributes at;
    const hipError_t e = hipFuncGetAttributes(&at, k);
    if (e != hipSuccess) return e;
    if ((int)at.localSizeBytes > *bytes) *bytes = (int)at.localSizeBytes;
  }
  return hipSuccess;
}

// co-resident k_reduce_apply workgroups per CU
hipError_t mdp_ra_occupancy(int* per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k_reduce_apply<1024>, 1024, 0);
}

// co-resident k_reduce_apply_batch workgroups per CU
hipError_t mdp_ra_batch_occupancy(int* per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k_reduce_apply_batch<1024>, 1024, 0);
}

hipError_t mdp_launch_reduce_apply_batch(const RaBatch& b, hipStream_t s) {
  const dim3 grid(b.wg_start[b.count] + (b.pf_count > 0 ? 1 : 0));  // + the draw piece, last
  if (MDP_RA_NARROW && b.narrow)
    mdp_launch(k_reduce_apply_batch<256>, grid, dim3(256), 0, s, b);
  else
    mdp_launch(k_reduce_apply_batch<1024>, grid, dim3(1024), 0, s, b);
  return hipGetLastError();
}

#ifdef MDP_TIMELINE
extern "C" int mdp_debug_tl_ra(unsigned long long* out, int reset) {
  const size_t n = sizeof(unsigned long long) * MDP_TL_SLOTS * MDP_TL_WG * 2;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_mdp_tl)) != hipSuccess) return -1;
    return hipMemset(p, 0, n) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_tl), n) == hipSuccess ? 0 : -1;
}
#endif

#ifdef MDP_STAMPS
// diagnostic build: stamps of this translation unit's kernels (own code object)
extern "C" int mdp_debug_stamps_ra(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mdp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif
