// slab_layout_probe.hip -- is the optimizer launch's partial-gradient read
// faster with a chunk-major slab layout?  (tools only; not part of the library)
//
// k_reduce_apply's chunk workgroup c sums the nwg partial slabs of its 256
// parameters: today the slabs are workgroup-major, [w][param] (each partial
// 1 KB, nwg of them at a stride of the net's size), so a workgroup reads nwg
// separate 1 KB pieces; chunk-major, [chunk][w][256], would make them one
// contiguous nwg KB block.  Both patterns, same bytes, same 16-B loads in
// flight (16 per lane, as the kernel), one 1024-thread (S5) or 256-thread
// (S2) workgroup per chunk; the slabs are written first by a separate kernel
// (dirty in L2, then the boundary), as in the training step.
//   hipcc -O3 --offload-arch=gfx950 tools/slab_layout_probe.hip -o tools/slab_layout_probe_bin
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)(i & 1023) * 1e-3f;
}

// G waves per workgroup; wave g sums partials w = g, g + G, ...
template <int G>
__global__ void k_read(const float* __restrict__ slab, int nwg, int64_t stride_w, int64_t chunk_stride, int cmajor,
                       float* out) {
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6, c = blockIdx.x;
  const float* base = cmajor ? slab + (int64_t)c * chunk_stride + 4 * lane : slab + (int64_t)c * 256 + 4 * lane;
  const int64_t ws = cmajor ? 256 : stride_w;
  f32x4 v[16];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int w0 = g; w0 < nwg; w0 += 16 * G) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int w = min(w0 + G * k, nwg - 1);
      v[k] = *reinterpret_cast<const f32x4*>(base + (int64_t)w * ws);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (w0 + G * k < nwg) s += v[k];
  }
  __shared__ f32x4 red[G][64];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0) {
    for (int q = 1; q < G; ++q) s += red[q][lane];
    *reinterpret_cast<f32x4*>(out + (int64_t)c * 256 + 4 * lane) = s;
  }
}

// the chunk's partials split over S workgroups: workgroup b reads part
// b % S (partials [part nwg / S, (part + 1) nwg / S)) of chunk b / S
template <int G>
__global__ void k_read_split(const float* __restrict__ slab, int nwg, int64_t stride_w, int S, float* out) {
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6, c = blockIdx.x / S, part = blockIdx.x % S;
  const float* base = slab + (int64_t)c * 256 + 4 * lane;
  const int w_lo = part * nwg / S, w_hi = (part + 1) * nwg / S;
  f32x4 v[16];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int w0 = w_lo + g; w0 < w_hi; w0 += 16 * G) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int w = min(w0 + G * k, w_hi - 1);
      v[k] = *reinterpret_cast<const f32x4*>(base + (int64_t)w * stride_w);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (w0 + G * k < w_hi) s += v[k];
  }
  __shared__ f32x4 red[G][64];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0) {
    for (int q = 1; q < G; ++q) s += red[q][lane];
    *reinterpret_cast<f32x4*>(out + (int64_t)blockIdx.x * 256 + 4 * lane) = s;
  }
}

template <int G>
static float run_split(int nchunk, int nwg, int S, int reps) {
  const int64_t P = (int64_t)nchunk * 256;
  float *slab, *out;
  (void)hipMalloc(&slab, sizeof(float) * P * nwg);
  (void)hipMalloc(&out, sizeof(float) * P * S);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float tot = 0.f;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, slab, P * nwg);
    hipExtLaunchKernelGGL(k_read_split<G>, dim3(nchunk * S), dim3(64 * G), 0, 0, a, b, 0u, (const float*)slab, nwg,
                          P, S, out);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 0) tot += ms;
  }
  (void)hipFree(slab);
  (void)hipFree(out);
  return tot / (reps - 1) * 1e3f;
}

template <int G>
static float run(int nchunk, int nwg, int cmajor, int reps) {
  const int64_t P = (int64_t)nchunk * 256;
  float *slab, *out;
  (void)hipMalloc(&slab, sizeof(float) * P * nwg);
  (void)hipMalloc(&out, sizeof(float) * P);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float tot = 0.f;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, slab, P * nwg);
    hipExtLaunchKernelGGL(k_read<G>, dim3(nchunk), dim3(64 * G), 0, 0, a, b, 0u, (const float*)slab, nwg, P,
                                (int64_t)256 * nwg, cmajor, out);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 0) tot += ms;
  }
  (void)hipFree(slab);
  (void)hipFree(out);
  return tot / (reps - 1) * 1e3f;
}

int main() {
  const int reps = 21;
  // S2: critic 8,705 params -> 35 chunks, 64 partials, 256-thread workgroups
  printf("S2 critic (35 chunks x 64 partials, 4 waves): wg-major %.2f us, chunk-major %.2f us\n",
         run<4>(35, 64, 0, reps), run<4>(35, 64, 1, reps));
  // S5: critic 36,993 params -> 145 chunks, 256 partials, 1024-thread workgroups
  printf("S5 critic (145 chunks x 256 partials, 16 waves): wg-major %.2f us, chunk-major %.2f us\n",
         run<16>(145, 256, 0, reps), run<16>(145, 256, 1, reps));
  printf("S5 actor (79 chunks x 256 partials, 16 waves): wg-major %.2f us, chunk-major %.2f us\n",
         run<16>(79, 256, 0, reps), run<16>(79, 256, 1, reps));
  // the fan-in split over S workgroups per chunk (no combine): does reading
  // from more CUs shorten the read?
  printf("S5 critic split: S1 G16 %.2f  S2 G16 %.2f  S2 G8 %.2f  S4 G4 %.2f  S4 G8 %.2f us\n",
         run_split<16>(145, 256, 1, reps), run_split<16>(145, 256, 2, reps), run_split<8>(145, 256, 2, reps),
         run_split<4>(145, 256, 4, reps), run_split<8>(145, 256, 4, reps));
  printf("S5 actor split:  S1 G16 %.2f  S2 G16 %.2f  S2 G8 %.2f  S4 G4 %.2f  S4 G8 %.2f us\n",
         run_split<16>(79, 256, 1, reps), run_split<16>(79, 256, 2, reps), run_split<8>(79, 256, 2, reps),
         run_split<4>(79, 256, 4, reps), run_split<8>(79, 256, 4, reps));
  printf("S2 critic split: S1 G4 %.2f  S2 G4 %.2f  S2 G2 %.2f  S4 G1 %.2f us\n", run_split<4>(35, 64, 1, reps),
         run_split<4>(35, 64, 2, reps), run_split<2>(35, 64, 2, reps), run_split<1>(35, 64, 4, reps));
  return 0;
}
