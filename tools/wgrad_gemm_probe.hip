// wgrad_gemm_probe.hip -- could the S5 optimizer launch compute the critic's
// weight gradients as a batch GEMM (dW = X^T D over K = B = 4,096 rows) from
// per-row factors, instead of summing 256 partial slabs?  (tools only; not
// part of the library)
//
// One workgroup per 16 x 16 tile of dW1 (158 x 128: 10 x 8 tiles, X [B][160])
// and dW2 (128 x 128: 8 x 8 tiles, X = H1 [B][128]), D [B][128]; its G waves
// split K, each a chain of K / (4 G) MFMA 16x16x4 steps with its operand
// loads issued P steps ahead; the wave tiles summed in LDS.  The factors are
// written first by a separate kernel (dirty in L2, then the boundary), as
// the gradient launch would leave them.  Timed with launch events against the
// slab read of the same outputs (slab_layout_probe: S5 critic 8.4 us).
//   hipcc -O3 --offload-arch=gfx950 tools/wgrad_gemm_probe.hip -o tools/wgrad_gemm_probe_bin
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)((i * 7) & 1023) * 1e-3f - 0.5f;
}

struct GemmArgs {
  const float* X1;  // [B][ldx1] (critic input rows)
  const float* X2;  // [B][128]  (h1)
  const float* D1;  // [B][128]
  const float* D2;  // [B][128]
  int B, K1, ldx1, t1;  // t1: tiles of dW1 (the rest are dW2)
  float* out;
};

template <int G, int P>
__global__ __launch_bounds__(64 * G) void k_gemm_tiles(GemmArgs g) {
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6, r = lane & 15, kq = lane >> 4;
  const int tile = blockIdx.x;
  const bool w1 = tile < g.t1;
  const int tt = w1 ? tile : tile - g.t1;
  const int mt = tt >> 3, nt = tt & 7;
  const float* X = w1 ? g.X1 : g.X2;
  const float* D = w1 ? g.D1 : g.D2;
  const int ldx = w1 ? g.ldx1 : 128, K = w1 ? g.K1 : 128;
  const int feat = mt * 16 + r, fc = min(feat, K - 1);
  const int rows = g.B / G, row0 = q * rows;
  const float* xp = X + (int64_t)(row0 + kq) * ldx + fc;
  const float* dp = D + (int64_t)(row0 + kq) * 128 + nt * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float a[P], b[P];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    a[s] = xp[(int64_t)4 * s * ldx];
    b[s] = dp[(int64_t)4 * s * 128];
  }
  const int steps = rows / 4;
  for (int s0 = 0; s0 < steps; s0 += P) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const float av = a[s], bv = b[s];
      const int nx = s0 + s + P;
      if (nx < steps) {
        a[s] = xp[(int64_t)4 * nx * ldx];
        b[s] = dp[(int64_t)4 * nx * 128];
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, feat < K ? av : 0.f, acc, 0, 0, 0);
    }
  }
  __shared__ f32x4 red[G][64];
  red[q][lane] = acc;
  __syncthreads();
  if (q == 0) {
    f32x4 s = red[0][lane];
    for (int w = 1; w < G; ++w) s += red[w][lane];
    *reinterpret_cast<f32x4*>(g.out + (int64_t)tile * 256 + 4 * lane) = s;
  }
}

template <int G, int P>
static float run(const GemmArgs& ga, int ntiles, float* fill, int64_t nfill, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float tot = 0.f;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, fill, nfill);
    hipExtLaunchKernelGGL((k_gemm_tiles<G, P>), dim3(ntiles), dim3(64 * G), 0, 0, a, b, 0u, ga);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 0) tot += ms;
  }
  return tot / (reps - 1) * 1e3f;
}

int main() {
  const int B = 4096, K1 = 158, ldx1 = 160, reps = 21;
  const int64_t n1 = (int64_t)B * ldx1, nh = (int64_t)B * 128;
  float* buf;
  const int64_t nfill = n1 + 3 * nh;
  (void)hipMalloc(&buf, sizeof(float) * nfill);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * 256 * 256);
  GemmArgs ga;
  ga.X1 = buf;
  ga.X2 = buf + n1;
  ga.D1 = buf + n1 + nh;
  ga.D2 = buf + n1 + 2 * nh;
  ga.B = B;
  ga.K1 = K1;
  ga.ldx1 = ldx1;
  ga.t1 = 80;
  ga.out = out;
  printf("S5 critic dW1 + dW2 as 144 GEMM tiles (K = 4096): G16 P4 %.2f  G16 P8 %.2f  G16 P16 %.2f  G8 P8 %.2f  "
         "G8 P16 %.2f us\n",
         run<16, 4>(ga, 144, buf, nfill, reps), run<16, 8>(ga, 144, buf, nfill, reps),
         run<16, 16>(ga, 144, buf, nfill, reps), run<8, 8>(ga, 144, buf, nfill, reps),
         run<8, 16>(ga, 144, buf, nfill, reps));
  ga.t1 = 0;
  printf("dW2 only (64 tiles): G16 P8 %.2f us\n", run<16, 8>(ga, 64, buf, nfill, reps));
  // check one tile against the host
  std::vector<float> h(nfill), o(256);
  (void)hipMemcpy(h.data(), buf, sizeof(float) * nfill, hipMemcpyDeviceToHost);
  ga.t1 = 80;
  run<16, 8>(ga, 144, buf, nfill, 2);
  (void)hipMemcpy(o.data(), out + 13 * 256, sizeof(float) * 256, hipMemcpyDeviceToHost);  // tile 13: mt 1, nt 5
  double maxe = 0.0;
  for (int lane = 0; lane < 64; ++lane)
    for (int j = 0; j < 4; ++j) {
      // acc[j] of lane (r, kq) = sum over rows of D[row][nt*16 + r'] X[row][feat'] in the transposed layout:
      // MFMA 16x16x4 D = A B: A = bv (16 x 4: output col x row), B = av (4 x 16: row x feature),
      // acc lane (r, kq) element j -> row index 4 kq + j of the 16 x 16 result, column r
      const int oc = 4 * (lane >> 4) + j, fr = lane & 15;
      double s = 0.0;
      for (int row = 0; row < B; ++row)
        s += (double)h[n1 + nh + (int64_t)row * 128 + 5 * 16 + oc] * (double)h[(int64_t)row * ldx1 + 16 + fr];
      maxe = std::max(maxe, std::abs(s - (double)o[4 * lane + j]));
    }
  printf("tile check (tile 13 vs fp64 host): max abs err %.3e\n", maxe);
  return 0;
}
