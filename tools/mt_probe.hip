// mt_probe.hip -- the replay index draw (mdp_mt.h) in isolation: three forms of
// the same CPython MT19937 / randint stream, checked against each other bit
// for bit (draws, final state, stream position) and timed with launch events.
//   0  make_index_block<NT> (mdp_mt.h, the library's form): the state in place
//      in LDS, one block per pass, whole workgroup, 2 barriers
//   1  probe_draw_wave (below): one wave, the state in registers, the twist
//      with cross-lane reads, no barrier
//   2  probe_draw_db<NT> (below): the state double-buffered in LDS, 1 barrier per block
// (tools only; not part of the library)
//   hipcc -O3 --offload-arch=gfx950 -I maddpg_amd/csrc tools/mt_probe.hip -o tools/mt_probe_bin
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "mdp_mt.h"

// the double-buffered form: the state in two LDS buffers, one barrier per block
// (twist as in make_index_block) Twist, sequential form: for kk in 0..623: mt[kk] = mt[(kk+397)%624] ^
// mix(mt[kk], mt[kk+1]).  kk < 227 reads old mt[kk+397]; 227 <= kk < 623
// reads new mt[kk-227]; kk = 623 reads new mt[396] and new mt[0].  So words
// t, t+227, t+454 (t < 227; the third for t <= 169) form a chain one thread
// computes in registers from old words only (thread 169 recomputes new mt[0]
// for word 623).  Reads the old block from src, writes the new one to dst and
// this thread's chain words to v[].
__device__ __forceinline__ void mt_twist_chains(const uint32_t* src, uint32_t* dst, int t, int nc, uint32_t (&v)[3]) {
  if (!nc) return;
  const uint32_t c0 = src[t], n0 = src[t + 1], f0 = src[t + 397], c1 = src[t + 227], n1 = src[t + 228];
  uint32_t c2 = 0, n2 = 0;
  if (nc == 3) {
    c2 = src[t + 454];
    n2 = t == 169 ? src[397] ^ mt_mix(src[0], src[1]) : src[t + 455];  // word 623: new mt[0]
  }
  v[0] = f0 ^ mt_mix(c0, n0);
  v[1] = v[0] ^ mt_mix(c1, n1);
  dst[t] = v[0];
  dst[t + 227] = v[1];
  if (nc == 3) {
    v[2] = v[1] ^ mt_mix(c2, n2);
    dst[t + 454] = v[2];
  }
}

template <int NT>
__device__ __forceinline__ void probe_draw_db(Ctl* ctl, int count, int32_t* __restrict__ out,
                                              uint32_t len_override = 0u) {
  static_assert(NT >= 256 && NT % 64 == 0, "the twist chains take threads 0..226 (waves 0..3)");
  __shared__ uint32_t mt[2][624];
  __shared__ int wsum[2][3][4];
  __shared__ int s_newpos;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t n = len_override ? len_override : (uint32_t)ctl->len;
  if (n == 0) {  // randint(0, -1) raises in the reference; the host refuses it too
    for (int i = t; i < count; i += NT) out[i] = 0;
    return;
  }
  if (count <= 0) return;
  for (int i = t; i < 624; i += NT) mt[0][i] = ctl->mt[i];
  const int pos0 = ctl->mt_pos;
  const int k = 32 - __clz(n);
  const int nc = t < 170 ? 3 : (t < 227 ? 2 : 0);  // chain length of this thread
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint32_t v[3] = {0u, 0u, 0u}, r[3];
  bool acc[3];
  unsigned long long bal[3];
  int b = 0, from = 0;  // the pending block: buffer b, its words >= from
  __syncthreads();
  if (pos0 < 624) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < nc) v[c] = mt[0][t + 227 * c];
    from = pos0;
  } else {
    mt_twist_chains(mt[0], mt[1], t, nc, v);
    b = 1;
  }
  // the pending block's ballots, their counts into wsum[b]
#define MDP_MT_BALLOT()                                       \
  _Pragma("unroll") for (int c = 0; c < 3; ++c) {             \
    const int i = t + 227 * c;                                \
    r[c] = mt_temper(v[c]) >> (32 - k);                       \
    acc[c] = c < nc && i >= from && r[c] < n;                 \
    bal[c] = __ballot(acc[c]);                                \
    if (lane == 0 && w < 4) wsum[b][c][w] = __popcll(bal[c]); \
  }
  MDP_MT_BALLOT();
  __syncthreads();
  int produced = 0;
  bool done = false;
  // acceptance >= 1/2 per draw, so ~2 count/624 blocks; the bound only guards a hang
  const int max_iters = 64 + 4 * count / 64;
  for (int iters = 0;; ++iters) {
    const int need = count - produced;
    int base = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      int before = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int x = wsum[b][c][q];
        before += q < w ? x : 0;
        tot += x;
      }
      const int g = base + before + __popcll(bal[c] & lt);
      if (acc[c]) {
        if (g < need) out[produced + g] = (int32_t)r[c];
        if (g == need - 1) s_newpos = t + 227 * c + 1;
      }
      base += tot;
    }
    if (base >= need) {
      done = true;
      break;
    }
    produced += base;
    if (iters >= max_iters) break;
    mt_twist_chains(mt[b], mt[b ^ 1], t, nc, v);
    b ^= 1;
    from = 0;
    MDP_MT_BALLOT();
    __syncthreads();
  }
#undef MDP_MT_BALLOT
  __syncthreads();
  const int pos = done ? s_newpos : 624;
  for (int i = t; i < 624; i += NT) ctl->mt[i] = mt[b][i];
  if (t == 0) ctl->mt_pos = pos;
}


// value of x in lane (lane + s) & 63; addr = ((lane + s) & 63) << 2
__device__ __forceinline__ uint32_t mt_lane(uint32_t x, int addr) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)x);
}

// the state as w[j] = mt[64 j + lane] (w[9] valid in lanes 0..47), twisted
// with cross-lane reads: old mt[kk+397] = lane l+13 of w[j+6] / w[j+7]; new
// mt[kk-227] = lane l+29 of new w[j-4] / w[j-3]; mt[kk+1] = lane l+1 (lane 63:
// lane 0 of w[j+1]; kk = 623: new mt[0])
__device__ __forceinline__ void mt_twist_wave(uint32_t (&w)[10], int l) {
  const int a1 = ((l + 1) & 63) << 2, a13 = ((l + 13) & 63) << 2, a29 = ((l + 29) & 63) << 2;
  uint32_t o[4], nx[10], nw[10], r[7];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = mt_lane(w[6 + i], a13);
#pragma unroll
  for (int j = 0; j < 10; ++j) nx[j] = mt_lane(w[j], a1);
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    uint32_t nxt = nx[j];
    if (j < 9) {
      const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)w[j + 1], 0);
      nxt = l == 63 ? h : nxt;
    } else {
      const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)nw[0], 0);
      nxt = l == 47 ? h : nxt;
    }
    uint32_t f;
    if (j < 3) f = l < 51 ? o[j] : o[j + 1];
    else if (j == 3) f = l < 35 ? o[3] : r[0];
    else f = l < 35 ? r[j - 4] : r[j - 3];
    nw[j] = f ^ mt_mix(w[j], nxt);
    if (j <= 6) r[j] = mt_lane(nw[j], a29);
  }
#pragma unroll
  for (int j = 0; j < 10; ++j) w[j] = nw[j];
}

// one wave (lanes of wave 0) draws; the others wait at the closing barrier
template <int NT>
__device__ __forceinline__ void probe_draw_wave(Ctl* ctl, int count, int32_t* __restrict__ out) {
  if (threadIdx.x < 64) {
    const int l = threadIdx.x & 63;
    const uint32_t n = (uint32_t)ctl->len;
    const int k = 32 - __clz(n);
    uint32_t w[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) w[j] = (j < 9 || l < 48) ? ctl->mt[64 * j + l] : 0u;
    int pos = ctl->mt_pos;
    const unsigned long long lt = (1ull << l) - 1ull;
    int produced = 0;
    const int max_iters = 64 + 4 * count / 64;
    int iters = 0;
    while (produced < count && iters++ < max_iters) {
      if (pos >= 624) {
        mt_twist_wave(w, l);
        pos = 0;
      }
      int newpos = 624;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int kk = 64 * j + l;
        const uint32_t r = mt_temper(w[j]) >> (32 - k);
        const bool acc = kk < 624 && kk >= pos && r < n;
        const unsigned long long bal = __ballot(acc);
        const int c = __popcll(bal), need = count - produced, rank = __popcll(bal & lt);
        if (acc && rank < need) out[produced + rank] = (int32_t)r;
        if (c >= need) {
          const unsigned long long last = __ballot(acc && rank == need - 1);
          newpos = 64 * j + __builtin_ctzll(last) + 1;
          produced = count;
          break;
        }
        produced += c;
      }
      pos = newpos;
    }
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (j < 9 || l < 48) ctl->mt[64 * j + l] = w[j];
    if (l == 0) ctl->mt_pos = pos;
  }
  __syncthreads();
}

template <int V, int NT>
__global__ __launch_bounds__(NT) void k_probe(Ctl* ctl, int count, int32_t* out) {
  if (V == 0) make_index_block<NT>(ctl, count, out);
  if (V == 1) probe_draw_wave<NT>(ctl, count, out);
  if (V == 2) probe_draw_db<NT>(ctl, count, out);
}

static void seed_ctl(Ctl& c, uint32_t s, int pos, int64_t len) {
  memset(&c, 0, sizeof(c));
  c.mt[0] = s;
  for (int i = 1; i < 624; ++i) c.mt[i] = 1812433253u * (c.mt[i - 1] ^ (c.mt[i - 1] >> 30)) + (uint32_t)i;
  c.mt_pos = pos;
  c.len = len;
}

struct Res {
  std::vector<int32_t> out;
  Ctl ctl;
  float us;
};

template <int V, int NT>
static Res run(const Ctl& init, int count, int reps) {
  Ctl* d_ctl;
  int32_t* d_out;
  (void)hipMalloc(&d_ctl, sizeof(Ctl));
  (void)hipMalloc(&d_out, sizeof(int32_t) * (count + 1));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float tot = 0.f;
  Res res;
  res.out.resize(count);
  for (int rep = 0; rep < reps; ++rep) {
    (void)hipMemcpy(d_ctl, &init, sizeof(Ctl), hipMemcpyHostToDevice);
    (void)hipMemset(d_out, 0xff, sizeof(int32_t) * (count + 1));
    hipExtLaunchKernelGGL((k_probe<V, NT>), dim3(1), dim3(NT), 0, 0, a, b, 0u, d_ctl, count, d_out);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep > 0) tot += ms;
  }
  (void)hipMemcpy(res.out.data(), d_out, sizeof(int32_t) * count, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&res.ctl, d_ctl, sizeof(Ctl), hipMemcpyDeviceToHost);
  res.us = tot / (reps - 1) * 1e3f;
  (void)hipFree(d_ctl);
  (void)hipFree(d_out);
  return res;
}

static bool same(const Res& x, const Res& y) {
  return x.out == y.out && x.ctl.mt_pos == y.ctl.mt_pos && !memcmp(x.ctl.mt, y.ctl.mt, sizeof(x.ctl.mt));
}

int main() {
  const int reps = 11;
  struct Case {
    int count, pos;
    int64_t len;
  } cases[] = {{1024, 624, 1000000}, {1024, 100, 524289}, {2048, 300, 50000},   {3072, 624, 1000000},
               {24576, 624, 1000000}, {24576, 5, 524289}, {1, 623, 7},          {5000, 624, 1}};
  int bad = 0;
  for (const Case& cs : cases) {
    Ctl init;
    seed_ctl(init, 12345u + cs.count, cs.pos, cs.len);
    Res r0 = run<0, 256>(init, cs.count, reps);
    Res r0b = run<0, 512>(init, cs.count, reps);
    Res r1 = run<1, 256>(init, cs.count, reps);
    Res r2 = run<2, 256>(init, cs.count, reps);
    Res r2b = run<2, 512>(init, cs.count, reps);
    Res r2c = run<2, 1024>(init, cs.count, reps);
    const bool ok = same(r0, r0b) && same(r0, r1) && same(r0, r2) && same(r0, r2b) && same(r0, r2c);
    bad += !ok;
    printf("count %5d pos %3d len %7lld: wg256 %7.2f us  wg512 %7.2f  wave %7.2f  p256 %7.2f  p512 %7.2f  p1024 %7.2f"
           "  (end pos %d)  %s\n",
           cs.count, cs.pos, (long long)cs.len, r0.us, r0b.us, r1.us, r2.us, r2b.us, r2c.us, r0.ctl.mt_pos,
           ok ? "identical" : "MISMATCH");
  }
  printf(bad ? "mt_probe: %d MISMATCH\n" : "mt_probe: all identical\n", bad);
  return bad ? 1 : 0;
}
