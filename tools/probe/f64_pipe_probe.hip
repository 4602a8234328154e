// Probe: do FP64 VALU instructions of one wave overlap the FP64 MFMAs of the other wave on the same SIMD (gfx950)?
// One 512-thread workgroup (two waves per SIMD): waves 0-3 run `nm` v_mfma_f64_16x16x4_f64 (4 accumulator chains),
// waves 4-7 run `nv` independent v_fma_f64 (8 chains), or f32 FMAs, or integer adds; s_memtime per wave.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/f64_pipe_probe.hip -o tools/probe/f64_pipe_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int KIND>  // VALU kind of waves 4-7: 0 f64 fma, 1 f32 fma, 2 int add
__global__ __launch_bounds__(512) void probe(double* out, unsigned long long* cyc, int nm, int nv, double a0) {
  const int w = threadIdx.x >> 6;
  double s = 0.0;
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  if (w < 4) {
    f64x4 acc[4];
    for (int c = 0; c < 4; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, (double)threadIdx.x};
    const double a = a0 + threadIdx.x * 1e-3, b = a0 - threadIdx.x * 1e-3;
    for (int i = 0; i < nm; i += 4) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][3];
  } else if (KIND == 0) {
    double x[8];
    for (int c = 0; c < 8; ++c) x[c] = a0 + c + threadIdx.x;
    for (int i = 0; i < nv; i += 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = __builtin_fma(x[c], 0.999999, 1e-9);
    }
    for (int c = 0; c < 8; ++c) s += x[c];
  } else if (KIND == 1) {
    float x[8];
    for (int c = 0; c < 8; ++c) x[c] = (float)a0 + c + threadIdx.x;
    for (int i = 0; i < nv; i += 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = __builtin_fmaf(x[c], 0.999999f, 1e-9f);
    }
    for (int c = 0; c < 8; ++c) s += x[c];
  } else {
    int x[8];
    for (int c = 0; c < 8; ++c) x[c] = c + threadIdx.x;
    for (int i = 0; i < nv; i += 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = x[c] * 3 + 7;
    }
    for (int c = 0; c < 8; ++c) s += x[c];
  }
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

template <int KIND>
void run(const char* name, int nm, int nv, double* d_out, unsigned long long* d_cyc) {
  hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(512), 0, 0, d_out, d_cyc, nm, nv, 1.0);  // warm
  hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(512), 0, 0, d_out, d_cyc, nm, nv, 1.0);
  unsigned long long c[8];
  hipMemcpy(c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-10s mfma/wave %5d valu/wave %6d | mfma waves %7llu %7llu %7llu %7llu | valu waves %7llu %7llu %7llu %7llu\n",
         name, nm, nv, c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
}

int main() {
  double* d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_out, 512 * sizeof(double));
  hipMalloc(&d_cyc, 8 * sizeof(unsigned long long));
  const int NM = 1024;
  for (int nv : {0, 4096, 8192, 16384, 32768}) {
    run<0>("f64 fma", NM, nv, d_out, d_cyc);
    run<0>("f64 alone", 0, nv, d_out, d_cyc);
  }
  for (int nv : {8192, 16384}) {
    run<1>("f32 fma", NM, nv, d_out, d_cyc);
    run<1>("f32 alone", 0, nv, d_out, d_cyc);
    run<2>("int", NM, nv, d_out, d_cyc);
    run<2>("int alone", 0, nv, d_out, d_cyc);
  }
  hipDeviceSynchronize();
  return 0;
}
