// bf16x6_probe -- is an exact three-way bf16 split of fp32 operands (6 bf16
// MFMA products per K-slice) a faster fp32-faithful path for the gradient
// kernels' dependent MFMA chains than the fp32 MFMA (v_mfma_f32_16x16x4_f32)?
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/bf16x6_probe_bin tools/bf16x6_probe.hip
//   tools/bf16x6_probe_bin            (on the GPU box)
//
// x = h + m + l exactly (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m): 3 x 8
// significant bits = fp32's 24), so X.W = sum of the 9 plane products; the 3
// smallest (m.l, l.m, l.l: <= ~2^-25 of |x||w|) are dropped.  Reports
// 1) numerics: one 16-row layer Y = X W (K = 64 and 158, N = 64) against fp64,
//    fp32 MFMA vs bf16x6 vs bf16x3 (h.h + h.m + m.h);
// 2) cycles (s_memtime) of a dependent layer chain on one wave: 4 output tiles
//    x K = 64, repeated, with the A operand (the activations) as fp32 registers
//    split on the fly, or already split (as if the producing layer stored planes).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP %s: %s\n", #x, hipGetErrorString(e));                    \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}
// the same exact split by truncation, in integer ops on the bits: hi = the top
// 16 bits of x, r = x - hi exact (<= 16 significant bits), mid = the top 16 bits
// of r, lo = r - mid exact (<= 8 significant bits: a bf16).  Two values per call,
// packed as the MFMA operand wants them (element j in the low half).
__device__ __forceinline__ void split3_pk(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t u0 = __float_as_uint(x0) & 0xffff0000u, u1 = __float_as_uint(x1) & 0xffff0000u;
  const float r0 = x0 - __uint_as_float(u0), r1 = x1 - __uint_as_float(u1);
  const uint32_t v0 = __float_as_uint(r0) & 0xffff0000u, v1 = __float_as_uint(r1) & 0xffff0000u;
  const float s0 = r0 - __uint_as_float(v0), s1 = r1 - __uint_as_float(v1);
  h = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
  m = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
  l = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- numerics
// one wave: Y[16][64] = X[16][K] W[K][64]; out[0] fp32 MFMA, out[1] bf16x6, out[2] bf16x3
__global__ void k_layer(const float* X, const float* W, int K, float* out) {
  const int lane = threadIdx.x;
  // fp32: A[l&15][k=l>>4], B[k=l>>4][l&15]; C: col = l&15, row = (l>>4)*4 + i
  for (int t = 0; t < 4; ++t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K; k0 += 4) {
      const int k = k0 + (lane >> 4);
      const float a = k < K ? X[(lane & 15) * K + k] : 0.f;
      const float b = k < K ? W[k * 64 + 16 * t + (lane & 15)] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) out[((lane >> 4) * 4 + i) * 64 + 16 * t + (lane & 15)] = acc[i];
  }
  for (int v = 0; v < 3; ++v) {  // 0 bf16x6, 1 bf16x3, 2 bf16x6 with the truncation split
    for (int t = 0; t < 4; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < K; k0 += 32) {
        bf16x8 ah, am, al, bh, bm, bl;
        if (v < 2) {
          for (int j = 0; j < 8; ++j) {
            const int k = k0 + 8 * (lane >> 4) + j;
            const float a = k < K ? X[(lane & 15) * K + k] : 0.f;
            const float b = k < K ? W[k * 64 + 16 * t + (lane & 15)] : 0.f;
            __bf16 h, m, l;
            split3(a, h, m, l);
            ah[j] = h;
            am[j] = m;
            al[j] = l;
            split3(b, h, m, l);
            bh[j] = h;
            bm[j] = m;
            bl[j] = l;
          }
        } else {
          u32x4 a4[3], b4[3];
          for (int j = 0; j < 4; ++j) {
            const int k = k0 + 8 * (lane >> 4) + 2 * j;
            const float a0 = k < K ? X[(lane & 15) * K + k] : 0.f, a1 = k + 1 < K ? X[(lane & 15) * K + k + 1] : 0.f;
            const float b0 = k < K ? W[k * 64 + 16 * t + (lane & 15)] : 0.f;
            const float b1 = k + 1 < K ? W[(k + 1) * 64 + 16 * t + (lane & 15)] : 0.f;
            uint32_t h, m, l;
            split3_pk(a0, a1, h, m, l);
            a4[0][j] = h;
            a4[1][j] = m;
            a4[2][j] = l;
            split3_pk(b0, b1, h, m, l);
            b4[0][j] = h;
            b4[1][j] = m;
            b4[2][j] = l;
          }
          ah = __builtin_bit_cast(bf16x8, a4[0]);
          am = __builtin_bit_cast(bf16x8, a4[1]);
          al = __builtin_bit_cast(bf16x8, a4[2]);
          bh = __builtin_bit_cast(bf16x8, b4[0]);
          bm = __builtin_bit_cast(bf16x8, b4[1]);
          bl = __builtin_bit_cast(bf16x8, b4[2]);
        }
        // smallest terms first
        if (v != 1) {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
      }
      for (int i = 0; i < 4; ++i) out[(1 + v) * 1024 + ((lane >> 4) * 4 + i) * 64 + 16 * t + (lane & 15)] = acc[i];
    }
  }
}

// ---------------------------------------------------------------- timing
// R repetitions of one 16 x 64 x 64 layer on one wave, the accumulators carried
// (a dependent chain across repetitions, 4 independent tiles inside one).
// mode 0: fp32 MFMA (16 k-steps x 4 tiles = 64 MFMAs per layer)
// mode 1: bf16x6, A and B pre-split in registers (2 K-slices x 4 tiles x 6 = 48)
// mode 2: bf16x6, A split from fp32 registers every repetition (the activations)
// mode 3: bf16x3 pre-split (24 MFMAs per layer)
// mode 4: bf16x6, A split by truncation in bit operations every repetition
template <int MODE>
__global__ void k_chain(const float* seed, int R, float* out, long long* cyc) {
  const int lane = threadIdx.x & 63;
  f32x4 acc[4];
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float af[16], bf[16][4];
  for (int s = 0; s < 16; ++s) {
    af[s] = seed[(lane + s) & 63];
    for (int t = 0; t < 4; ++t) bf[s][t] = seed[(lane * 3 + s * 5 + t) & 63];
  }
  bf16x8 ah[2], am[2], al[2], bh[2][4], bm[2][4], bl[2][4];
  float a8[2][8];
  for (int q = 0; q < 2; ++q)
    for (int j = 0; j < 8; ++j) {
      a8[q][j] = af[8 * q + j];
      __bf16 h, m, l;
      split3(a8[q][j], h, m, l);
      ah[q][j] = h;
      am[q][j] = m;
      al[q][j] = l;
      for (int t = 0; t < 4; ++t) {
        split3(bf[8 * q + j][t], h, m, l);
        bh[q][t][j] = h;
        bm[q][t][j] = m;
        bl[q][t][j] = l;
      }
    }
  __syncthreads();
  const long long t0 = clock64();
  for (int r = 0; r < R; ++r) {
    if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[s][t], acc[t], 0, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bf16x8 xh = ah[q], xm = am[q], xl = al[q];
        if (MODE == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            __bf16 h, m, l;
            split3(a8[q][j] + (float)r * 1e-30f, h, m, l);  // re-split every repetition
            xh[j] = h;
            xm[j] = m;
            xl[j] = l;
          }
        }
        if (MODE == 4) {  // the truncation split in bit operations, every repetition
          u32x4 h4, m4, l4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t h, m, l;
            split3_pk(a8[q][2 * j] + (float)r * 1e-30f, a8[q][2 * j + 1], h, m, l);
            h4[j] = h;
            m4[j] = m;
            l4[j] = l;
          }
          xh = __builtin_bit_cast(bf16x8, h4);
          xm = __builtin_bit_cast(bf16x8, m4);
          xl = __builtin_bit_cast(bf16x8, l4);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (MODE != 3) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, bl[q][t], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl, bh[q][t], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xm, bm[q][t], acc[t], 0, 0, 0);
          }
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, bm[q][t], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xm, bh[q][t], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, bh[q][t], acc[t], 0, 0, 0);
        }
      }
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static double max_rel(const float* y, const std::vector<double>& ref) {
  double m = 0, s = 0;
  for (size_t i = 0; i < ref.size(); ++i) s = std::fmax(s, std::fabs(ref[i]));
  for (size_t i = 0; i < ref.size(); ++i) m = std::fmax(m, std::fabs(y[i] - ref[i]));
  return m / s;
}

int main() {
  // numerics at the gradient kernels' layer shapes
  uint64_t st = 88172645463325252ull;
  auto rnd = [&]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (double)(st >> 11) / 9007199254740992.0;
  };
  for (int K : {18, 64, 158}) {
    for (int dist = 0; dist < 2; ++dist) {
      std::vector<float> X(16 * K), W(K * 64);
      const double lim = std::sqrt(6.0 / (K + 64));  // Xavier uniform (tf_util / layers default)
      for (auto& x : X) x = dist == 0 ? (float)rnd() : (float)(rnd() * 2 - 1) * 3.f;  // ReLU outputs / raw obs
      for (auto& w : W) w = (float)((rnd() * 2 - 1) * lim);
      std::vector<double> ref(16 * 64, 0.0);
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 64; ++j) {
          double a = 0;
          for (int k = 0; k < K; ++k) a += (double)X[i * K + k] * (double)W[k * 64 + j];
          ref[i * 64 + j] = a;
        }
      float *dX, *dW, *dO;
      CK(hipMalloc(&dX, 4 * X.size()));
      CK(hipMalloc(&dW, 4 * W.size()));
      CK(hipMalloc(&dO, 4 * 4 * 1024));
      CK(hipMemcpy(dX, X.data(), 4 * X.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dW, W.data(), 4 * W.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(k_layer, dim3(1), dim3(64), 0, 0, dX, dW, K, dO);
      CK(hipDeviceSynchronize());
      std::vector<float> o(4 * 1024);
      CK(hipMemcpy(o.data(), dO, 4 * o.size(), hipMemcpyDeviceToHost));
      std::printf("numerics K=%3d %s: max|y - y64| / max|y64|  fp32 MFMA %.2e  bf16x6 %.2e  bf16x3 %.2e  "
                  "bf16x6 (truncation split) %.2e\n", K, dist == 0 ? "X in [0,1) " : "X in (-3,3)",
                  max_rel(o.data(), ref), max_rel(o.data() + 1024, ref), max_rel(o.data() + 2048, ref),
                  max_rel(o.data() + 3072, ref));
      CK(hipFree(dX));
      CK(hipFree(dW));
      CK(hipFree(dO));
    }
  }
  // timing: one wave per workgroup; 1 workgroup (one wave on the chip) and 256 x 4 waves
  std::vector<float> seed(64);
  for (auto& s : seed) s = (float)(rnd() * 0.1);
  float *dS, *dO;
  long long* dC;
  CK(hipMalloc(&dS, 4 * 64));
  CK(hipMalloc(&dO, 4 * 1024 * 256));
  CK(hipMalloc(&dC, 8 * 1024));
  CK(hipMemcpy(dS, seed.data(), 4 * 64, hipMemcpyHostToDevice));
  const int R = 2000;
  const char* names[5] = {"fp32 MFMA 16x16x4 (64 MFMA)", "bf16x6, A+B pre-split (48)", "bf16x6, A split per layer (48)",
                          "bf16x3, pre-split (24)", "bf16x6, A bit-split per layer (48)"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int wpb : {64, 256}) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_chain<0>, dim3(wpb == 64 ? 1 : 256), dim3(wpb), 0, 0, dS, R, dO, dC);
        if (mode == 1) hipLaunchKernelGGL(k_chain<1>, dim3(wpb == 64 ? 1 : 256), dim3(wpb), 0, 0, dS, R, dO, dC);
        if (mode == 2) hipLaunchKernelGGL(k_chain<2>, dim3(wpb == 64 ? 1 : 256), dim3(wpb), 0, 0, dS, R, dO, dC);
        if (mode == 3) hipLaunchKernelGGL(k_chain<3>, dim3(wpb == 64 ? 1 : 256), dim3(wpb), 0, 0, dS, R, dO, dC);
        if (mode == 4) hipLaunchKernelGGL(k_chain<4>, dim3(wpb == 64 ? 1 : 256), dim3(wpb), 0, 0, dS, R, dO, dC);
      };
      launch();
      CK(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      long long c = 0;
      CK(hipMemcpy(&c, dC, 8, hipMemcpyDeviceToHost));
      std::printf("chain %-32s %s: %7.1f cycles per 16x64x64 layer (s_memtime), %6.3f us per layer (event)\n",
                  names[mode], wpb == 64 ? "1 wave        " : "4 waves x 256 ", (double)c / R, 1e3 * ms / R);
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
    }
  }
  return 0;
}
