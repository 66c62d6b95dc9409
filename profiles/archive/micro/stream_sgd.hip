// HBM ceiling of the SGD-momentum update shape on MI355X: read p, m; write p, m (16 B/elem),
// g synthesised in registers (as in the wgrad epilogue, where g comes from the MFMA tile).
// Variants: flat grid-stride (U float4 per lane in flight, WG/CU), and 2-D tiles of a
// [4096][9216] matrix with row segments of 512 B / 1 KiB / 2 KiB (the epilogue's tile shapes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void flat_sgd(float* __restrict__ p, float* __restrict__ m, long n4, float lr, float mu) {
  f4* P = (f4*)p; f4* M = (f4*)m;
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    f4 pv[U], mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = base + (long)u * 256; if (i >= n4) i = n4 - 1;
      if (NT) { pv[u] = __builtin_nontemporal_load(P + i); mv[u] = __builtin_nontemporal_load(M + i); }
      else { pv[u] = P[i]; mv[u] = M[i]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = base + (long)u * 256; if (i >= n4) continue;
      f4 g = pv[u] * 1e-3f;
      mv[u] = mu * mv[u] + g; pv[u] = pv[u] - lr * mv[u];
      if (NT) { __builtin_nontemporal_store(pv[u], P + i); __builtin_nontemporal_store(mv[u], M + i); }
      else { P[i] = pv[u]; M[i] = mv[u]; }
    }
  }
}

// tile (TR rows x TC cols) of a row-major [R][C] matrix per workgroup iteration, persistent grid
template <int TR, int TC, int U, bool NT>
__global__ __launch_bounds__(256) void tile_sgd(float* __restrict__ p, float* __restrict__ m, int R, int C, float lr, float mu) {
  constexpr int C4 = TC / 4, IT = TR * C4 / 256;
  static_assert(IT % U == 0, "");
  const int tn = C / TC, tiles = (R / TR) * tn;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int r0 = (t / tn) * TR, c0 = (t % tn) * TC;
#pragma unroll
    for (int i0 = 0; i0 < IT; i0 += U) {
      long gi[U]; f4 pv[U], mv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = (i0 + u) * 256 + threadIdx.x;
        gi[u] = (long)(r0 + e / C4) * C + c0 + (e % C4) * 4;
        if (NT) { pv[u] = __builtin_nontemporal_load((f4*)(p + gi[u])); mv[u] = __builtin_nontemporal_load((f4*)(m + gi[u])); }
        else { pv[u] = *(f4*)(p + gi[u]); mv[u] = *(f4*)(m + gi[u]); }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f4 g = pv[u] * 1e-3f;
        mv[u] = mu * mv[u] + g; pv[u] = pv[u] - lr * mv[u];
        if (NT) { __builtin_nontemporal_store(pv[u], (f4*)(p + gi[u])); __builtin_nontemporal_store(mv[u], (f4*)(m + gi[u])); }
        else { *(f4*)(p + gi[u]) = pv[u]; *(f4*)(m + gi[u]) = mv[u]; }
      }
    }
  }
}

template <typename F>
float timeit(F f, int reps = 20) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const int R = 4096, C = 9216; const long n = (long)R * C;
  float *p, *m, *junk;
  CK(hipMalloc(&p, n * 4)); CK(hipMalloc(&m, n * 4)); CK(hipMalloc(&junk, 512l << 20));
  CK(hipMemset(p, 0, n * 4)); CK(hipMemset(m, 0, n * 4));
  const double bytes = 16.0 * n;
  // evict MALL between reps: touch 512 MiB (as the real step's other traffic does)
  auto flush = [&]() { CK(hipMemsetAsync(junk, 1, 512l << 20)); };
  float flush_us = timeit([&] { flush(); });
  printf("{\"flush_us\": %.1f}\n", flush_us);
#define RUNF(U, NT, WPC) { int g = 256 * WPC; float us = timeit([&] { flush(); hipLaunchKernelGGL((flat_sgd<U, NT>), dim3(g), dim3(256), 0, 0, p, m, n / 4, 1e-4f, 0.9f); }) - flush_us; \
    printf("{\"kind\": \"flat\", \"U\": %d, \"nt\": %d, \"wg_per_cu\": %d, \"us\": %.1f, \"TBps\": %.2f}\n", U, NT, WPC, us, bytes / us / 1e6); }
  RUNF(2, false, 4) RUNF(4, false, 4) RUNF(8, false, 4) RUNF(4, true, 4) RUNF(8, true, 4)
  RUNF(4, false, 8) RUNF(8, false, 2) RUNF(16, false, 2) RUNF(4, true, 8) RUNF(8, true, 2)
#define RUNT(TR, TC, U, NT, WPC) { int g = 256 * WPC; float us = timeit([&] { flush(); hipLaunchKernelGGL((tile_sgd<TR, TC, U, NT>), dim3(g), dim3(256), 0, 0, p, m, R, C, 1e-4f, 0.9f); }) - flush_us; \
    printf("{\"kind\": \"tile\", \"TR\": %d, \"TC\": %d, \"U\": %d, \"nt\": %d, \"wg_per_cu\": %d, \"us\": %.1f, \"TBps\": %.2f}\n", TR, TC, U, NT, WPC, us, bytes / us / 1e6); }
  RUNT(128, 128, 8, true, 2) RUNT(128, 128, 8, false, 2) RUNT(128, 128, 16, true, 2) RUNT(128, 128, 8, true, 4) RUNT(128, 128, 4, true, 4)
  RUNT(64, 256, 8, true, 2) RUNT(64, 256, 8, false, 2) RUNT(64, 256, 8, true, 4)
  RUNT(32, 512, 8, true, 2) RUNT(32, 512, 8, false, 2) RUNT(32, 512, 8, true, 4)
  RUNT(128, 128, 8, true, 1) RUNT(64, 256, 16, true, 2)
  return 0;
}
