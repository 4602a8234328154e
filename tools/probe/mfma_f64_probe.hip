// Cycle probe of v_mfma_f64_16x16x4_f64 on gfx950: issue rate with 1, 2, 4, 8 independent accumulator chains
// (one wave per SIMD, operands in registers), measured with s_memtime around 1024 MFMAs.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(64) void probe(double* out, unsigned long long* cyc, double a0, double b0) {
  f64x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, (double)threadIdx.x};
  double a = a0 + threadIdx.x * 1e-3, b = b0 - threadIdx.x * 1e-3;
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 1024 / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  double s = 0.0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run(double* d_out, unsigned long long* d_cyc) {
  hipLaunchKernelGGL(probe<CH>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0, 2.0);
  hipLaunchKernelGGL(probe<CH>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0, 2.0);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("chains %d: %.1f cycles per MFMA (1024 MFMAs, one wave)\n", CH, (double)c / 1024.0);
}

int main() {
  double* d_out;
  unsigned long long* d_cyc;
  (void)hipMalloc(&d_out, 64 * 8 * 4);
  (void)hipMalloc(&d_cyc, 64);
  run<1>(d_out, d_cyc);
  run<2>(d_out, d_cyc);
  run<3>(d_out, d_cyc);
  run<4>(d_out, d_cyc);
  run<8>(d_out, d_cyc);
  return 0;
}
