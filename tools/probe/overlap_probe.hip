// Probe: can a small kernel on a second stream run beside a persistent kernel that leaves some CUs free?
// (r06: the K-shard prepare's first kernel, launched on the prepare stream while the shard's persistent partial kernel
// holds 240 of 256 CUs, only completed when the partial kernel's workgroups began to retire.)
//
// P: G workgroups of 512 threads with 144 KB of LDS each (one per CU, like k_est_all_f64g), spinning SPIN_US.
// S: a small kernel on another stream, NS workgroups of `ts` threads, launched 100 us after P; every workgroup
//    records its start (wall clock) -- the probe prints when S's first / last workgroup started and S's event time.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe/overlap_probe tools/probe/overlap_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ __launch_bounds__(512) void k_persist(long long ticks, unsigned long long* t0out, int* sink) {
  extern __shared__ char lds[];
  const long long t0 = wall_clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) *t0out = (unsigned long long)t0;
  int acc = 0;
  while (wall_clock64() - t0 < ticks) {
    acc += lds[threadIdx.x] ;
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == 12345) sink[0] = acc;  // keep the LDS read
}

// the same with 256 VGPRs per wave (the clobber): one 8-wave workgroup then fills a CU's register file, as
// k_est_all_f64g does
__global__ __launch_bounds__(512) void k_persist_full(long long ticks, unsigned long long* t0out, int* sink) {
  extern __shared__ char lds[];
  asm volatile("" ::: "v255");
  const long long t0 = wall_clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) *t0out = (unsigned long long)t0;
  int acc = 0;
  while (wall_clock64() - t0 < ticks) {
    acc += lds[threadIdx.x];
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == 12345) sink[0] = acc;
}

__global__ void k_small(unsigned long long* starts, float* buf, int n) {
  if (threadIdx.x == 0) starts[blockIdx.x] = (unsigned long long)wall_clock64();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = buf[i] * 1.5f + 1.0f;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 240;
  const int NS = argc > 2 ? atoi(argv[2]) : 256;
  const int TS = argc > 3 ? atoi(argv[3]) : 256;
  const bool full = argc > 4 && atoi(argv[4]) != 0;
  const int spin_us = 1000;
  int rate_khz = 0;
  CHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const long long ticks = (long long)spin_us * rate_khz / 1000;
  CHK(hipFuncSetAttribute((const void*)k_persist, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
  CHK(hipFuncSetAttribute((const void*)k_persist_full, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
  hipStream_t a, b;
  CHK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CHK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  unsigned long long *t0, *starts;
  float* buf;
  int* sink;
  const int n = 16 * 64 * 64 * 2;
  CHK(hipMalloc(&t0, 8));
  CHK(hipMalloc(&starts, 8 * NS));
  CHK(hipMalloc(&buf, 4 * n));
  CHK(hipMalloc(&sink, 4));
  CHK(hipMemset(buf, 0, 4 * n));
  hipEvent_t e0, e1, e2;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventCreate(&e2));
  for (int rep = 0; rep < 3; ++rep) {
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, a));
    if (full)
      hipLaunchKernelGGL(k_persist_full, dim3(G), dim3(512), 144 * 1024, a, ticks, t0, sink);
    else
      hipLaunchKernelGGL(k_persist, dim3(G), dim3(512), 144 * 1024, a, ticks, t0, sink);
    CHK(hipGetLastError());
    // 100 us later (host side), the small kernel on the other stream
    unsigned long long dummy = 0;
    (void)dummy;
    const auto wait_host = [](double us) {
      timespec s, c;
      clock_gettime(CLOCK_MONOTONIC, &s);
      do clock_gettime(CLOCK_MONOTONIC, &c);
      while ((c.tv_sec - s.tv_sec) * 1e6 + (c.tv_nsec - s.tv_nsec) / 1e3 < us);
    };
    wait_host(100.0);
    CHK(hipEventRecord(e1, b));
    hipLaunchKernelGGL(k_small, dim3(NS), dim3(TS), 0, b, starts, buf, n);
    CHK(hipGetLastError());
    CHK(hipEventRecord(e2, b));
    CHK(hipDeviceSynchronize());
    unsigned long long h0;
    unsigned long long* hs = (unsigned long long*)malloc(8 * NS);
    CHK(hipMemcpy(&h0, t0, 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hs, starts, 8 * NS, hipMemcpyDeviceToHost));
    unsigned long long mn = ~0ull, mx = 0;
    for (int i = 0; i < NS; ++i) {
      mn = hs[i] < mn ? hs[i] : mn;
      mx = hs[i] > mx ? hs[i] : mx;
    }
    float ms_small = 0.f, ms_launch = 0.f;
    CHK(hipEventElapsedTime(&ms_small, e1, e2));
    CHK(hipEventElapsedTime(&ms_launch, e0, e2));
    const double us_per_tick = 1000.0 / rate_khz;
    printf("{\"full_vgpr\": %d, \"G\": %d, \"NS\": %d, \"TS\": %d, \"spin_us\": %d, \"small_first_start_us\": %.1f, "
           "\"small_last_start_us\": %.1f, \"small_event_ms\": %.3f, \"persist_start_to_small_end_ms\": %.3f}\n",
           (int)full, G, NS, TS, spin_us, (double)(mn - h0) * us_per_tick, (double)(mx - h0) * us_per_tick, ms_small, ms_launch);
    free(hs);
  }
  return 0;
}
