// Cycle probe of the FP64 headline kernel's block loop on gfx950: one "block" = 2 dependent
// v_mfma_f64_16x16x4_f64 on one of 16 accumulators (the GW row tiles), its A operands one ds_read_b128
// issued E blocks ahead (s_waitcnt lgkmcnt(E - 1)), the B operands re-scaled once per k-pair (2 v_mul_f64) as
// in k_est_all_f64.  Variants isolate what costs MFMA issue when a SIMD holds one wave (cfg4, N = 128) vs two
// (metric, N = 64): the LDS reads, the per-k-pair VALU, the waves per SIMD.  s_memtime around 32 k-pairs x 16
// tiles (1024 MFMAs) per wave; printed: cycles per MFMA (64 = the SIMD's FP64 MFMA rate).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int E = 6;
constexpr int NT = 16;  // accumulators (row tiles)
constexpr int KPAIRS = 32;

template <int NW, bool LDSRD, bool VMUL>
__global__ __launch_bounds__(NW * 64) void probe(double* out, unsigned long long* cyc, double y0, double p0) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 1024 / 8; i += NW * 64) reinterpret_cast<double*>(lds)[i] = 1e-3 * (i & 255);
  __syncthreads();
  f64x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, (double)(lane + t)};
  double ya = y0 + lane * 1e-3, yb = y0 - lane * 1e-3, p = p0;
  double bs0 = ya * p, bs1 = yb * p;
  int roff = lane * 16;
  asm volatile("" : "+v"(roff));
  double2 areg = make_double2(0.5 + lane * 1e-4, 0.25);
  double2 buf[E + 1];
  if constexpr (LDSRD) {
#pragma unroll
    for (int i = 0; i < E; ++i) buf[i] = *reinterpret_cast<const double2*>(&lds[roff + i * 1024]);
  }
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < KPAIRS; ++s) {
    if constexpr (VMUL) {
      bs0 = ya * p;
      bs1 = yb * p;
      p = p * 0.999;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int b = s * NT + t;
      __builtin_amdgcn_sched_barrier(0);
      double2 a;
      if constexpr (LDSRD) {
        buf[(b + E) % (E + 1)] = *reinterpret_cast<const double2*>(&lds[roff + ((b + E) % 56) * 1024]);
        a = buf[b % (E + 1)];
      } else {
        a = areg;
      }
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, bs0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, bs1, acc[t], 0, 0, 0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  double sum = 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) sum += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * NW * 64 + threadIdx.x] = sum;
  if (lane == 0) {
    cyc[2 * wave] = t0;
    cyc[2 * wave + 1] = t1;
  }
}

template <int NW, bool LDSRD, bool VMUL>
void run(const char* name, double* d_out, unsigned long long* d_cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<NW, LDSRD, VMUL>), dim3(1), dim3(NW * 64), 0, 0, d_out, d_cyc, 1.0, 0.9);
  unsigned long long c[16] = {0};
  (void)hipMemcpy(c, d_cyc, 2 * NW * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  unsigned long long lo = ~0ull, hi = 0, mx = 0;
  for (int i = 0; i < NW; ++i) {
    lo = c[2 * i] < lo ? c[2 * i] : lo;
    hi = c[2 * i + 1] > hi ? c[2 * i + 1] : hi;
    mx = c[2 * i + 1] - c[2 * i] > mx ? c[2 * i + 1] - c[2 * i] : mx;
  }
  const int per = NW > 4 ? NW / 4 : 1;
  printf("%-34s waves %d (%d per SIMD): span %.1f cycles per MFMA per SIMD (longest wave %.1f per own MFMA)\n", name,
         NW, per, (double)(hi - lo) / (2.0 * KPAIRS * NT) / per, (double)mx / (2.0 * KPAIRS * NT));
}

int main() {
  double* d_out;
  unsigned long long* d_cyc;
  (void)hipMalloc(&d_out, 8 * 64 * 8);
  (void)hipMalloc(&d_cyc, 16 * 8);
  run<1, false, false>("MFMA only", d_out, d_cyc);
  run<1, false, true>("MFMA + k-pair v_mul", d_out, d_cyc);
  run<1, true, false>("MFMA + ds_read", d_out, d_cyc);
  run<1, true, true>("MFMA + ds_read + v_mul", d_out, d_cyc);
  run<4, true, true>("MFMA + ds_read + v_mul", d_out, d_cyc);
  run<8, true, true>("MFMA + ds_read + v_mul", d_out, d_cyc);
  run<8, false, false>("MFMA only", d_out, d_cyc);
  return 0;
}
