// fma64_latency.hip -- dependent-chain latency of v_fma_f64 on one wave
// (gfx950): C independent chains of N dependent FMAs, interleaved, timed
// with s_memtime (shader clock) on a single wave; prints cycles per FMA.
// Build: hipcc --offload-arch=gfx950 -O3 fma64_latency.hip -o fma64_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int C>
__global__ void chains(double* out, long long* cyc, double a, int n) {
  double x[C];
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] = threadIdx.x * 1e-3 + c;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int c = 0; c < C; ++c) x[c] = fma(a, x[c], 0.5);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int C>
void run(double* d, long long* c, int waves) {
  const int n = 4096;
  hipLaunchKernelGGL(chains<C>, dim3(waves), dim3(64), 0, 0, d, c, 0.999, n);
  (void)hipDeviceSynchronize();
  long long cyc = 0;
  (void)hipMemcpy(&cyc, c, sizeof(cyc), hipMemcpyDeviceToHost);
  printf("chains %d waves %d: %.2f cycles per FMA, %.2f per chain link\n", C, waves,
         (double)cyc / (n * 16.0 * C), (double)cyc / (n * 16.0));
}

int main() {
  double* d;
  long long* c;
  (void)hipMalloc(&d, 64 * sizeof(double) * 4096);
  (void)hipMalloc(&c, sizeof(long long));
  for (int w = 1; w <= 2; ++w) {
    run<1>(d, c, w); run<1>(d, c, w);
    run<2>(d, c, w);
    run<3>(d, c, w);
    run<4>(d, c, w);
    run<6>(d, c, w);
    run<8>(d, c, w);
  }
  return 0;
}
