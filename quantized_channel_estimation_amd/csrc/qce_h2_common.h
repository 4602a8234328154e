// Shared device pieces of the FP16 two-term split estimate kernels (qce_estimate_h2.hip: the fused
// kernel for M, N <= 64; qce_estimate_h2x.hip: the chunk-streamed kernel for M, N up to 256).
// Table geometry, MFMA/LDS fragment helpers, the per-component scalars and the online-softmax step.
#pragma once
#include "qce_common.h"

#include <utility>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#define QCE_NEG_INF (-__builtin_inf())

template <int MP, int NP, bool HM>
struct H2Geom {
  static constexpr int R = 2 * MP, S = 2 * NP;
  static constexpr int NSL = R / 32, NSW = S / 32;
  static constexpr int KS = R / 16;  // k-steps of 16 real columns
  static constexpr int HMI = HM ? 1 : 0;
  // k-step units of 2 KB (two pieces x 64 lanes x 16 B)
  static constexpr int GL_STEPS = NSL * (NSL + 1) + HMI * NSL;  // sum_r (2r + 2 + HM)
  static constexpr int GW_STEPS = NSW * (KS + HMI);
  static constexpr int GL_BYTES = GL_STEPS * 2048;
  static constexpr int GW_BYTES = GW_STEPS * 2048;
  static constexpr int COMP_BYTES = GL_BYTES + GW_BYTES;
  static constexpr __host__ __device__ int gl_off(int r) { return r * (r + 1) + HMI * r; }  // in steps
};

QCE_DEV f16x8 lds_frag(const char* base, int byte_off, int lane) {
  return *reinterpret_cast<const f16x8*>(base + byte_off + lane * 16);
}

QCE_DEV f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }

QCE_DEV void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// The per-component scalars (slice scales, c_k) are fetched with scalar loads and waited for right
// away, before the LDS reads of a phase: an outstanding SMEM load would force every later LDS wait
// to lgkmcnt(0) (scalar loads return out of order), which serialises the fragment prefetch.
template <int NS>
struct CompScalars {
  float s[NS];
  double c;
  QCE_DEV void load(const float* __restrict__ sinv, const double* __restrict__ cconst, int k) {
    const float* sk = sinv + (long long)k * NS;
#pragma unroll
    for (int i = 0; i < NS; ++i) s[i] = sk[i];
    c = cconst[k];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};

template <int OFF>
QCE_DEV void ds_rd(f16x8& v, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
}
template <int N_>
QCE_DEV void wait_lgkm(f16x8& a, f16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N_));
}
template <typename F, int... I>
QCE_DEV void static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
constexpr int c_gl_slice(int idx, int hmi) {
  int r = 0, base = 0;
  while (idx >= base + 2 * r + 2 + hmi) {
    base += 2 * r + 2 + hmi;
    ++r;
  }
  return r;
}

QCE_DEV void softmax_step(double lp, double& m, double& ssum, float& alpha, float& p) {
  const double mnew = fmax(m, lp);
  alpha = (m == mnew) ? 1.0f : expf((float)(m - mnew));
  p = (lp == QCE_NEG_INF) ? 0.0f : expf((float)(lp - mnew));
  ssum = ssum * (double)alpha + (double)p;
  m = mnew;
}

QCE_DEV void write_final(double2* __restrict__ h, double* __restrict__ om, double* __restrict__ os,
                         float* __restrict__ oa, long long row, int N, int hh, int NSW, const f32x16* out, double m,
                         double ssum, bool partial_fmt) {
  if (partial_fmt) {
    if (hh == 0) {
      om[row] = m;
      os[row] = ssum;
    }
    float* pa = oa + row * (2LL * N);
    for (int r = 0; r < NSW; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 16 * r + 4 * q + 2 * hh;
        if (n0 < N) *reinterpret_cast<float2*>(pa + 2 * n0) = make_float2(out[r][4 * q + 0], out[r][4 * q + 1]);
        if (n0 + 1 < N)
          *reinterpret_cast<float2*>(pa + 2 * n0 + 2) = make_float2(out[r][4 * q + 2], out[r][4 * q + 3]);
      }
    return;
  }
  const double inv = 1.0 / ssum;
  double2* hp = h + row * N;
  for (int r = 0; r < NSW; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 16 * r + 4 * q + 2 * hh;
      if (n0 < N) hp[n0] = make_double2((double)out[r][4 * q + 0] * inv, (double)out[r][4 * q + 1] * inv);
      if (n0 + 1 < N) hp[n0 + 1] = make_double2((double)out[r][4 * q + 2] * inv, (double)out[r][4 * q + 3] * inv);
    }
}
