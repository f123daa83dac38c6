// mdp_mt.h -- CPython's MT19937 stream and random.randint on one workgroup.
//
// replay_buffer.py:46-47 draws [random.randint(0, len-1) for _ in range(B)]
// from the module-global CPython generator (_randommodule.c genrand_uint32,
// Lib/random.py _randbelow_with_getrandbits): r = getrandbits(k) =
// temper(next word) >> (32 - k), k = len.bit_length(), rejected while
// r >= len.  The 624-word state lives in Ctl; one workgroup regenerates it
// (one block of 624 words per pass, the twist as per-thread chains), tempers
// the block and compacts the accepted draws with ballots + a workgroup prefix
// sum, so the output is bit-identical to the sequential stream.  Used by
// k_make_index (1024 threads), k_rollout's draw workgroup (256), the index
// pieces of the optimizer launches (256 / 1024) and the extra workgroup of
// k_critic_grad_r (512).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mdp_topo.h"

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt) {
  const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// One workgroup draws a block of 624 words per pass with two barriers.
// Twist, sequential form: for kk in 0..623: mt[kk] = mt[(kk+397)%624] ^
// mix(mt[kk], mt[kk+1]).  kk < 227 reads old mt[kk+397]; 227 <= kk < 623
// reads new mt[kk-227]; kk = 623 reads new mt[396] and new mt[0].  So words
// t, t+227, t+454 (t < 227; the third for t <= 169) form a chain one thread
// computes in registers from old words only: every old word is read before
// the pass's first barrier, and thread 169 recomputes new mt[0] for word 623.
// The accepted draws are ranked in stream order as chunk (0: words 0..226,
// 1: 227..453, 2: 454..623), then wave, then lane -- one ballot per chunk and
// wave, summed after the second barrier.  (A pass of NT words with a
// four-stage twist took ~10 barriers per 624 words: the S5 rollout's 24,576
// draws outlasted its env workgroups by ~45 us.)
//
// count draws of randint(0, ctl->len - 1) into out[], advancing ctl's state.
// Must be called by all NT threads of the workgroup (blockDim.x == NT).
// len_override > 0: draw from randint(0, len_override - 1) instead of ctl->len
// (k_rollout's extra workgroup draws against the length its step leaves).
template <int NT>
__device__ __forceinline__ void make_index_block(Ctl* ctl, int count, int32_t* __restrict__ out,
                                                 uint32_t len_override = 0u) {
  static_assert(NT >= 256 && NT % 64 == 0, "the twist chains take threads 0..226 (waves 0..3)");
  __shared__ uint32_t mt[624];
  __shared__ int wsum[3][4];
  __shared__ int s_newpos;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = t; i < 624; i += NT) mt[i] = ctl->mt[i];
  int pos = ctl->mt_pos;
  const uint32_t n = len_override ? len_override : (uint32_t)ctl->len;
  if (n == 0) {  // randint(0, -1) raises in the reference; the host refuses it too
    for (int i = t; i < count; i += NT) out[i] = 0;
    return;
  }
  const int k = 32 - __clz(n);
  const int nc = t < 170 ? 3 : (t < 227 ? 2 : 0);  // chain length of this thread
  const unsigned long long lt = (1ull << lane) - 1ull;
  __syncthreads();
  int produced = 0;
  // acceptance >= 1/2 per draw, so ~2 count/624 passes; the bound only guards a hang
  const int max_iters = 64 + 4 * count / 64;
  int iters = 0;
  while (produced < count && iters++ < max_iters) {
    uint32_t v[3] = {0u, 0u, 0u};
    if (pos >= 624) {
      uint32_t c0 = 0, n0 = 0, f0 = 0, c1 = 0, n1 = 0, c2 = 0, n2 = 0;
      if (nc) {
        c0 = mt[t];
        n0 = mt[t + 1];
        f0 = mt[t + 397];
        c1 = mt[t + 227];
        n1 = mt[t + 228];
      }
      if (nc == 3) {
        c2 = mt[t + 454];
        n2 = t == 169 ? mt[397] ^ mt_mix(mt[0], mt[1]) : mt[t + 455];  // word 623: new mt[0]
      }
      __syncthreads();
      if (nc) {
        v[0] = f0 ^ mt_mix(c0, n0);
        v[1] = v[0] ^ mt_mix(c1, n1);
        mt[t] = v[0];
        mt[t + 227] = v[1];
        if (nc == 3) {
          v[2] = v[1] ^ mt_mix(c2, n2);
          mt[t + 454] = v[2];
        }
      }
      pos = 0;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (c < nc) v[c] = mt[t + 227 * c];
    }
    uint32_t r[3];
    bool acc[3];
    unsigned long long bal[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int i = t + 227 * c;
      r[c] = mt_temper(v[c]) >> (32 - k);
      acc[c] = c < nc && i >= pos && r[c] < n;
      bal[c] = __ballot(acc[c]);
      if (lane == 0 && w < 4) wsum[c][w] = __popcll(bal[c]);
    }
    __syncthreads();
    const int need = count - produced;
    int base = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      int before = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int x = wsum[c][q];
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
      __syncthreads();
      pos = s_newpos;
      produced = count;
    } else {
      produced += base;
      pos = 624;
    }
  }
  __syncthreads();
  for (int i = t; i < 624; i += NT) ctl->mt[i] = mt[i];
  if (t == 0) ctl->mt_pos = pos;
}
