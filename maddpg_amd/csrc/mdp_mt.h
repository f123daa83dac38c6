// mdp_mt.h -- CPython's MT19937 stream and random.randint on one workgroup.
//
// replay_buffer.py:46-47 draws [random.randint(0, len-1) for _ in range(B)]
// from the module-global CPython generator (_randommodule.c genrand_uint32,
// Lib/random.py _randbelow_with_getrandbits): r = getrandbits(k) =
// temper(next word) >> (32 - k), k = len.bit_length(), rejected while
// r >= len.  The 624-word state lives in Ctl; one workgroup regenerates it in
// LDS (4 dependency stages per twist), tempers a block of words per pass and
// compacts the accepted draws with a ballot + workgroup prefix sum, so the
// output is bit-identical to the sequential stream.  Used by k_make_index
// (1024 threads) and, for the next round's indices, by the extra workgroup of
// k_critic_grad_r (512 threads).
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

// Generation step over the 624 words in LDS.  Sequential form: for kk in
// 0..623: mt[kk] = mt[(kk+397)%624] ^ mix(mt[kk], mt[kk+1]).  kk < 227 reads
// old mt[kk+397]; 227 <= kk < 623 reads new mt[kk-227]; kk = 623 reads new
// mt[396] and new mt[0].  NT threads, word i = t + p*NT.
template <int NT>
__device__ __forceinline__ void mt_twist(uint32_t* mt) {
  constexpr int PER = (624 + NT - 1) / NT;
  const int t = threadIdx.x;
  uint32_t cur[PER], nxt[PER], far[PER];
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int i = t + p * NT;
    cur[p] = nxt[p] = far[p] = 0;
    if (i < 624) {
      cur[p] = mt[i];
      nxt[p] = mt[i + 1 < 624 ? i + 1 : 0];
    }
    if (i < 227) far[p] = mt[i + 397];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int i = t + p * NT;
    if (i < 227) mt[i] = far[p] ^ mt_mix(cur[p], nxt[p]);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int i = t + p * NT;
    if (i >= 227 && i < 454) mt[i] = mt[i - 227] ^ mt_mix(cur[p], nxt[p]);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int i = t + p * NT;
    if (i >= 454 && i < 623) mt[i] = mt[i - 227] ^ mt_mix(cur[p], nxt[p]);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int i = t + p * NT;
    if (i == 623) mt[623] = mt[396] ^ mt_mix(cur[p], mt[0]);
  }
  __syncthreads();
}

// count draws of randint(0, ctl->len - 1) into out[], advancing ctl's state.
// Must be called by all NT threads of the workgroup (blockDim.x == NT).
// len_override > 0: draw from randint(0, len_override - 1) instead of ctl->len
// (k_rollout's extra workgroup draws against the length its step leaves).
template <int NT>
__device__ __forceinline__ void make_index_block(Ctl* ctl, int count, int32_t* __restrict__ out,
                                                 uint32_t len_override = 0u) {
  __shared__ uint32_t mt[624];
  __shared__ int wsum[NT / 64];
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
  __syncthreads();
  int produced = 0;
  // acceptance >= 1/2 per draw, so ~2 count/NT passes; the bound only guards a hang
  const int max_iters = 64 + 4 * count / 64;
  int iters = 0;
  while (produced < count && iters++ < max_iters) {
    if (pos >= 624) {
      mt_twist<NT>(mt);
      pos = 0;
    }
    const int take = min(624 - pos, NT);
    bool acc = false;
    uint32_t r = 0;
    if (t < take) {
      r = mt_temper(mt[pos + t]) >> (32 - k);
      acc = r < n;
    }
    const unsigned long long bal = __ballot(acc);
    const int wrank = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
      const int c = wsum[i];
      before += (i < w) ? c : 0;
      total += c;
    }
    const int rank = before + wrank;
    const int need = count - produced;
    if (acc && rank < need) out[produced + rank] = (int32_t)r;
    if (total >= need) {
      if (acc && rank == need - 1) s_newpos = pos + t + 1;
      __syncthreads();
      pos = s_newpos;
      produced = count;
    } else {
      produced += total;
      pos += take;
    }
    __syncthreads();
  }
  for (int i = t; i < 624; i += NT) ctl->mt[i] = mt[i];
  if (t == 0) ctl->mt_pos = pos;
}
