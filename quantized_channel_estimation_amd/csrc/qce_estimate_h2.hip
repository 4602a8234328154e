// Fused 'all'-mode estimate kernel on FP16 matrix cores with an exact two-term split
// (gfx950 / CDNA4).  Same math as k_est_all_f32 (qce_estimate.hip, restating
// gmm_cplx_bussgang.py:220-228, :331-332, :388-435, :632-656), different arithmetic:
//
//  * every component table (E(Linv_k) with its -q0 column, E(W_k) with its b column) is cut into
//    32-row slices; a slice is scaled by a power of two 2^e (max entry -> [2^13, 2^14)) and split
//    as a = a_hi + a_lo with a_hi = fp16(a), a_lo = fp16(a - a_hi): 22 significant bits relative to
//    the slice maximum (prepare: k_pack_h2);
//  * the observations are exact in fp16 after a per-quantiser scale (1 bit: y*sqrt(2) = +-1;
//    uniform b-bit: y*2/delta = odd integers <= 255), so a*y = a_hi*y + a_lo*y is two
//    v_mfma_f32_32x32x16_f16 with fp32 accumulation — fp32-class results at 1/8 of the fp32-MFMA
//    cycles.  Observations that are not exact (Lloyd-Max labels, n_bits = inf, or any unquantised
//    input) are split too (y = y_hi + y_lo) and the wave takes a three-product path
//    (a_hi y_hi + a_lo y_hi + a_hi y_lo); the choice is per wave, by ballot, so no input can
//    silently lose precision;
//  * one 512-thread workgroup = 8 waves x 32 samples shares each component's tables through LDS:
//    the Linv part (GL) and the W part (GW) have their own LDS slot and are streamed by
//    global_load_lds (16 B per lane) one phase ahead of the MFMAs that read them;
//  * the K loop can be split over blockIdx.y (split-K) to fill the chip when B/256 workgroups do
//    not divide evenly over the CUs; split partials (running max, sum, accumulator) are merged by
//    k_merge_splits — the same merge the K-shard multi-GPU path uses.
#include "qce_common.h"
#include "qce_kernels.h"

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

long long qce_pack_h2_stride_bytes(int MP, int NP, int has_mean) {
  const int R = 2 * MP, S = 2 * NP, NSL = R / 32, NSW = S / 32, KS = R / 16, HMI = has_mean ? 1 : 0;
  return (long long)(NSL * (NSL + 1) + HMI * NSL + NSW * (KS + HMI)) * 2048;
}

QCE_DEV f16x8 lds_frag(const char* base, int byte_off, int lane) {
  return *reinterpret_cast<const f16x8*>(base + byte_off + lane * 16);
}

QCE_DEV f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }

// global -> LDS copy of `bytes` (multiple of 1 KB) by the 8 waves, one 1 KB wave-instruction each
template <int BYTES>
QCE_DEV void stage(const char* __restrict__ src, char* dst, int wave, int lane) {
#pragma unroll
  for (int c = wave; c < BYTES / 1024; c += 8) {
    __builtin_amdgcn_global_load_lds((const void*)(src + c * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)(dst + c * 1024), 16, 0, 0);
  }
}

template <int MP, int NP, bool HM, bool Y2>
QCE_DEV void h2_kloop(int k0, int k1, const char* __restrict__ pack, long long cstride, const float* __restrict__ sinv,
                      const double* __restrict__ cconst, const f16x8* yh, const f16x8* yl, char* lds,
                      f32x16 (&out)[H2Geom<MP, NP, HM>::NSW], double& m, double& ssum, int wave, int lane) {
  using G = H2Geom<MP, NP, HM>;
  char* slotL = lds;
  char* slotW = lds + G::GL_BYTES;
  const int NSLICE = G::NSL + G::NSW;
  // prologue: both halves of component k0
  stage<G::GL_BYTES>(pack + (long long)k0 * cstride, slotL, wave, lane);
  stage<G::GW_BYTES>(pack + (long long)k0 * cstride + G::GL_BYTES, slotW, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int k = k0; k < k1; ++k) {
    const float* sk = sinv + (long long)k * NSLICE;
    // ---- GL phase: whitened residual u = E(Linv)[y;1], quad form in FP64 ----
    double quad = 0.0;
#pragma unroll
    for (int r = 0; r < G::NSL; ++r) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
      const int base = G::gl_off(r) * 2048;
#pragma unroll
      for (int s = 0; s < 2 * r + 2; ++s) {
        const f16x8 a0 = lds_frag(slotL, base + s * 2048, lane);
        const f16x8 a1 = lds_frag(slotL, base + s * 2048 + 1024, lane);
        acc = mfma_h(a0, yh[s], acc);
        acc = mfma_h(a1, yh[s], acc);
        if (Y2) acc = mfma_h(a0, yl[s], acc);
      }
      if (HM) {
        const f16x8 a0 = lds_frag(slotL, base + (2 * r + 2) * 2048, lane);
        const f16x8 a1 = lds_frag(slotL, base + (2 * r + 2) * 2048 + 1024, lane);
        acc = mfma_h(a0, yh[G::KS], acc);
        acc = mfma_h(a1, yh[G::KS], acc);
      }
      float qs = 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) qs = fmaf(acc[q], acc[q], qs);
      const double is = (double)sk[r];
      quad = fma((double)qs, is * is, quad);
    }
    quad += __shfl_xor(quad, 32);
    const double lp = cconst[k] - quad;
    const double mnew = fmax(m, lp);
    const float alpha = (m == mnew) ? 1.0f : expf((float)(m - mnew));
    const float p = (lp == QCE_NEG_INF) ? 0.0f : expf((float)(lp - mnew));
    ssum = ssum * (double)alpha + (double)p;
    m = mnew;
    // GW_k has to have landed before its phase; slotL is free once every wave passed here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (k + 1 < k1) stage<G::GL_BYTES>(pack + (long long)(k + 1) * cstride, slotL, wave, lane);
    // ---- GW phase: Z = E(W)[y;1], folded into the running accumulator ----
#pragma unroll
    for (int r = 0; r < G::NSW; ++r) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
      const int base = r * (G::KS + G::HMI) * 2048;
#pragma unroll
      for (int s = 0; s < G::KS; ++s) {
        const f16x8 a0 = lds_frag(slotW, base + s * 2048, lane);
        const f16x8 a1 = lds_frag(slotW, base + s * 2048 + 1024, lane);
        acc = mfma_h(a0, yh[s], acc);
        acc = mfma_h(a1, yh[s], acc);
        if (Y2) acc = mfma_h(a0, yl[s], acc);
      }
      if (HM) {
        const f16x8 a0 = lds_frag(slotW, base + G::KS * 2048, lane);
        const f16x8 a1 = lds_frag(slotW, base + G::KS * 2048 + 1024, lane);
        acc = mfma_h(a0, yh[G::KS], acc);
        acc = mfma_h(a1, yh[G::KS], acc);
      }
      const float ps = p * sk[G::NSL + r];
#pragma unroll
      for (int q = 0; q < 16; ++q) out[r][q] = fmaf(out[r][q], alpha, ps * acc[q]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (k + 1 < k1) stage<G::GW_BYTES>(pack + (long long)(k + 1) * cstride + G::GL_BYTES, slotW, wave, lane);
  }
}

// PARTIAL: write (m, s, acc) for split blockIdx.y (row = split * B + sample); else the final h.
template <int MP, int NP, bool HM, bool PARTIAL>
__global__ __launch_bounds__(512) void k_est_all_h2(long long B, int M, int N, int K, int nsplit, double y_scale,
                                                    const double2* __restrict__ y, const char* __restrict__ pack,
                                                    long long cstride, const float* __restrict__ sinv,
                                                    const double* __restrict__ cconst, double2* __restrict__ h,
                                                    double* __restrict__ part_m, double* __restrict__ part_s,
                                                    float* __restrict__ part_acc) {
  using G = H2Geom<MP, NP, HM>;
  __shared__ __attribute__((aligned(16))) char lds[G::COMP_BYTES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, hh = lane >> 5;
  const long long sample = (long long)blockIdx.x * 256 + wave * 32 + j;
  const bool valid = sample < B;
  // split-K range
  const int split = blockIdx.y;
  const int kb = (int)(((long long)K * split) / nsplit), ke = (int)(((long long)K * (split + 1)) / nsplit);

  // Y^T fragments: k-step s covers real features 16s + 8hh + t (t = 0..7) = complex 8s + 4hh + t/2
  f16x8 yh[G::KS + G::HMI], yl[G::KS];
  bool inexact = false;
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 8 * s + 4 * hh + t;
      double2 v = make_double2(0.0, 0.0);
      if (valid && c < M) v = y[sample * M + c];
      const double re = v.x * y_scale, im = v.y * y_scale;
      const _Float16 rh = (_Float16)re, ih = (_Float16)im;
      const _Float16 rl = (_Float16)(re - (double)rh), il = (_Float16)(im - (double)ih);
      yh[s][2 * t] = rh;
      yh[s][2 * t + 1] = ih;
      yl[s][2 * t] = rl;
      yl[s][2 * t + 1] = il;
      inexact |= (rl != (_Float16)0.0f) || (il != (_Float16)0.0f);
    }
  }
  if (HM) {
#pragma unroll
    for (int t = 0; t < 8; ++t) yh[G::KS][t] = (_Float16)0.0f;
    if (hh == 0) yh[G::KS][0] = (_Float16)1.0f;  // the [y; 1] augmentation column
  }
  f32x16 out[G::NSW];
#pragma unroll
  for (int r = 0; r < G::NSW; ++r)
#pragma unroll
    for (int q = 0; q < 16; ++q) out[r][q] = 0.0f;
  double m = QCE_NEG_INF, ssum = 0.0;
  if (__ballot(inexact) != 0ull)
    h2_kloop<MP, NP, HM, true>(kb, ke, pack, cstride, sinv, cconst, yh, yl, lds, out, m, ssum, wave, lane);
  else
    h2_kloop<MP, NP, HM, false>(kb, ke, pack, cstride, sinv, cconst, yh, yl, lds, out, m, ssum, wave, lane);

  if (!valid) return;
  if (PARTIAL) {
    const long long row = (long long)split * B + sample;
    if (hh == 0) {
      part_m[row] = m;
      part_s[row] = ssum;
    }
    float* pa = part_acc + row * (2LL * N);
#pragma unroll
    for (int r = 0; r < G::NSW; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 16 * r + 4 * q + 2 * hh;
        if (n0 < N) *reinterpret_cast<float2*>(pa + 2 * n0) = make_float2(out[r][4 * q + 0], out[r][4 * q + 1]);
        if (n0 + 1 < N) *reinterpret_cast<float2*>(pa + 2 * n0 + 2) = make_float2(out[r][4 * q + 2], out[r][4 * q + 3]);
      }
    return;
  }
  const double inv = 1.0 / ssum;
  double2* hp = h + sample * N;
#pragma unroll
  for (int r = 0; r < G::NSW; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 16 * r + 4 * q + 2 * hh;
      if (n0 < N) hp[n0] = make_double2((double)out[r][4 * q + 0] * inv, (double)out[r][4 * q + 1] * inv);
      if (n0 + 1 < N) hp[n0 + 1] = make_double2((double)out[r][4 * q + 2] * inv, (double)out[r][4 * q + 3] * inv);
    }
}

// Merge nsplit partials per sample: h = sum_j acc_j e^{m_j - M} / sum_j s_j e^{m_j - M}
// (final) or the merged partial (m, s, acc) for a further cross-GPU combine.
__global__ __launch_bounds__(256) void k_merge_splits(long long B, int N, int nsplit, const double* __restrict__ pm,
                                                      const double* __restrict__ ps, const float* __restrict__ pa,
                                                      double2* __restrict__ h, double* __restrict__ om,
                                                      double* __restrict__ os, float* __restrict__ oa) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  double mx = QCE_NEG_INF;
  for (int j = 0; j < nsplit; ++j) mx = fmax(mx, pm[(long long)j * B + b]);
  double s = 0.0;
  for (int j = 0; j < nsplit; ++j) {
    const double mj = pm[(long long)j * B + b];
    s += (mj == QCE_NEG_INF) ? 0.0 : ps[(long long)j * B + b] * exp(mj - mx);
  }
  for (int n = lane; n < N; n += 64) {
    double re = 0.0, im = 0.0;
    for (int j = 0; j < nsplit; ++j) {
      const double mj = pm[(long long)j * B + b];
      const double sc = (mj == QCE_NEG_INF) ? 0.0 : exp(mj - mx);
      const float2 v = *reinterpret_cast<const float2*>(pa + ((long long)j * B + b) * 2 * N + 2 * n);
      re += (double)v.x * sc;
      im += (double)v.y * sc;
    }
    if (h) {
      h[b * N + n] = make_double2(re / s, im / s);
    } else {
      oa[b * 2 * N + 2 * n] = (float)re;
      oa[b * 2 * N + 2 * n + 1] = (float)im;
    }
  }
  if (!h && lane == 0) {
    om[b] = mx;
    os[b] = s;
  }
}

// ---------------------------------------------------------------------------
// prepare-side packing: per (component, slice) power-of-two scale and fp16 hi/lo pieces
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack_h2(int M, int N, int MP, int NP, int has_mean, long long cstride,
                                                 double y_scale, const double2* __restrict__ Linv,
                                                 const double2* __restrict__ W, const double2* __restrict__ q0,
                                                 const double2* __restrict__ bvec, char* __restrict__ pack,
                                                 float* __restrict__ sinv) {
  const int k = blockIdx.y, sl = blockIdx.x, tid = threadIdx.x;
  const int R = 2 * MP, S = 2 * NP, NSL = R / 32, NSW = S / 32, KS = R / 16, HMI = has_mean ? 1 : 0;
  const bool isL = sl < NSL;
  const int r = isL ? sl : sl - NSL;
  const int nsteps = isL ? 2 * r + 2 : KS;
  const int rows = isL ? M : N;
  const double2* Mx = isL ? Linv + (long long)k * M * M : W + (long long)k * N * M;
  long long off;  // in k-steps
  if (isL)
    off = (long long)r * (r + 1) + (long long)HMI * r;
  else
    off = (long long)NSL * (NSL + 1) + (long long)HMI * NSL + (long long)r * (KS + HMI);
  char* dst = pack + (long long)k * cstride + off * 2048;
  auto value = [&](int row, int col) -> double {  // real-embedded, y-scale-aware entry
    int i = row >> 1;
    if (i >= rows) return 0.0;
    if (col == R) {  // augmentation column: -q0 (GL) or b (GW), times y_scale
      double2 v = isL ? q0[(long long)k * M + i] : bvec[(long long)k * N + i];
      double o = (row & 1) ? v.y : v.x;
      return (isL ? -o : o) * y_scale;
    }
    if (col > R) return 0.0;
    int jj = col >> 1;
    if (jj >= M) return 0.0;
    double2 v = Mx[(long long)i * M + jj];
    int rr = row & 1, cc = col & 1;
    return (rr == cc) ? v.x : (rr == 0 ? -v.y : v.y);
  };
  // slice maximum over the stored entries
  __shared__ double red[256];
  double mx = 0.0;
  const int ncols = nsteps * 16;
  for (int e = tid; e < 32 * ncols; e += 256) mx = fmax(mx, fabs(value(32 * r + e / ncols, e % ncols)));
  if (HMI)
    for (int e = tid; e < 32; e += 256) mx = fmax(mx, fabs(value(32 * r + e, R)));
  red[tid] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  mx = red[0];
  int e2 = 0;
  if (mx > 0.0) {
    int ex;
    frexp(mx, &ex);  // mx = f * 2^ex, f in [0.5, 1)
    e2 = 14 - ex;    // mx * 2^e2 in [2^13, 2^14)
  }
  const double scale = ldexp(1.0, e2);
  if (tid == 0) sinv[(long long)k * (NSL + NSW) + sl] = (float)ldexp(1.0, -e2) / (float)y_scale;
  // pieces: step s, piece p, lane l, element t -> E[32r + (l&31)][16s + 8(l>>5) + t]
  const int total_steps = nsteps + HMI;
  for (int e = tid; e < total_steps * 64 * 8; e += 256) {
    const int t = e & 7, l = (e >> 3) & 63, s = e >> 9;
    const int row = 32 * r + (l & 31);
    double v;
    if (s < nsteps) {
      v = value(row, 16 * s + 8 * (l >> 5) + t);
    } else {
      v = ((l >> 5) == 0 && t == 0) ? value(row, R) : 0.0;
    }
    v *= scale;
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (double)hi);
    _Float16* d = reinterpret_cast<_Float16*>(dst + (long long)s * 2048);
    d[l * 8 + t] = hi;
    d[512 + l * 8 + t] = lo;
  }
}

hipError_t qce_launch_pack_h2(int K, int M, int N, int MP, int NP, int has_mean, long long cstride, double y_scale,
                              const double2* Linv, const double2* W, const double2* q0, const double2* bvec, char* pack,
                              float* sinv, hipStream_t st) {
  const int nsl = (2 * MP) / 32 + (2 * NP) / 32;
  hipLaunchKernelGGL(k_pack_h2, dim3(nsl, K), dim3(256), 0, st, M, N, MP, NP, has_mean, cstride, y_scale, Linv, W, q0,
                     bvec, pack, sinv);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
template <int MP, int NP, bool HM>
static hipError_t launch_h2_t(const QceH2Args& a, double2* h, double* pm, double* ps, float* pa, bool partial,
                              hipStream_t st) {
  dim3 grid((unsigned)((a.B + 255) / 256), (unsigned)a.nsplit);
  if (partial)
    hipLaunchKernelGGL((k_est_all_h2<MP, NP, HM, true>), grid, dim3(512), 0, st, a.B, a.M, a.N, a.K, a.nsplit,
                       a.y_scale, a.y, a.pack, a.cstride, a.sinv, a.cconst, h, pm, ps, pa);
  else
    hipLaunchKernelGGL((k_est_all_h2<MP, NP, HM, false>), grid, dim3(512), 0, st, a.B, a.M, a.N, a.K, a.nsplit,
                       a.y_scale, a.y, a.pack, a.cstride, a.sinv, a.cconst, h, pm, ps, pa);
  return hipGetLastError();
}

hipError_t qce_launch_est_h2(const QceH2Args& a, double2* h, double* pm, double* ps, float* pa, bool partial,
                             hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_CASE(X, Y)                                                                    \
  if (a.MP == X && a.NP == Y)                                                             \
    return hm ? launch_h2_t<X, Y, true>(a, h, pm, ps, pa, partial, st)                    \
              : launch_h2_t<X, Y, false>(a, h, pm, ps, pa, partial, st);
  QCE_CASE(16, 16)
  QCE_CASE(16, 32)
  QCE_CASE(16, 64)
  QCE_CASE(32, 16)
  QCE_CASE(32, 32)
  QCE_CASE(32, 64)
  QCE_CASE(64, 16)
  QCE_CASE(64, 32)
  QCE_CASE(64, 64)
#undef QCE_CASE
  return hipErrorInvalidValue;
}

int qce_h2_blocks_per_cu(int MP, int NP, int has_mean) {
  int n = 0;
  const void* fn = nullptr;
#define QCE_OCC(X, Y)                                                                                     \
  if (MP == X && NP == Y)                                                                                 \
    fn = has_mean ? (const void*)k_est_all_h2<X, Y, true, false> : (const void*)k_est_all_h2<X, Y, false, false>;
  QCE_OCC(16, 16) QCE_OCC(16, 32) QCE_OCC(16, 64) QCE_OCC(32, 16) QCE_OCC(32, 32) QCE_OCC(32, 64) QCE_OCC(64, 16)
  QCE_OCC(64, 32) QCE_OCC(64, 64)
#undef QCE_OCC
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 512, 0) != hipSuccess || n < 1) n = 1;
  return n;
}

hipError_t qce_launch_merge_splits(long long B, int N, int nsplit, const double* pm, const double* ps, const float* pa,
                                   double2* h, double* om, double* os, float* oa, hipStream_t st) {
  hipLaunchKernelGGL(k_merge_splits, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, nsplit, pm, ps, pa, h, om,
                     os, oa);
  return hipGetLastError();
}
