// Fourier-domain estimate path for circulant / block-circulant mixtures.
//
// After a circulant fit (gmm_cplx_bussgang.py:104-117) every covariance is C_k = F^H diag(c_k) F with F
// the unitary DFT; after a block-circulant fit (:118-133) F = kron(F_n1, F_n2).  With A = I (one
// pilot, estimate_from_y :191-192) every per-SNR quantity of _prepare_for_prediction (:246-328) stays
// diagonal in that basis:
//   Cy_k = F^H diag(c_k + s2) F, diag(Cy_k) = d_k (constant), so the Bussgang gain is a scalar g_k;
//   1 bit: the arcsine law (:292-301) acts entry-wise on a (block-)circulant matrix, so Cr_k is
//          (block-)circulant: its eigenvalues r_k = DFT(first column of Cr_k);
//   multi-bit: Cr_k = b^2 Cy_k + (1 - b^2) d_k I  ->  r_k = b^2 (c_k + s2) + (1 - b^2) d_k;  inf: r = c + s2;
//   W_k = C_k g_k Cr_k^-1 = F^H diag(g c / r) F;  b_k = mu_k - W_k g mu_k;
//   lp_k = -N log(pi) - sum log r + log w_k - sum_i |y~_i - g mu~_i|^2 / r_i      (y~ = F y)
// so one estimate is: FFT(y), a (B x N)(N x K) product for lp, the softmax / selection over K, a
// (B x K)(K x N) product for the per-bin filter, and an inverse FFT:  h = F^H (y~ . f + bb).
// All FP64.  HBM-bound: 16 N bytes in and 16 N bytes out per estimate.
//
// Kernels: k_fft_struct (model creation: eigenvalues c_k, mean spectra, and the check that every C_k
// really is (block-)circulant for the candidate (n1, n2)); k_fft_prep (per SNR tables);
// k_fft_est<N, TS, OUT> (one workgroup = a tile of TS observations held in LDS as spectra).
#include "qce_common.h"
#include "qce_kernels.h"

#define QCE_NEG_INF (-__builtin_inf())

namespace {

constexpr double PI_D = 3.14159265358979323846;

QCE_DEV int ilog2(int v) { return 31 - __clz(v); }

QCE_DEV int bitrev(int j, int lg) { return (int)(__brev((unsigned)j) >> (32 - lg)) & ((1 << lg) - 1); }

// e^{-2 pi i t / 256}, t < 128, into LDS (every power-of-two length <= 256 indexes it with a stride)
QCE_DEV void twiddles(double2* tw) {
  for (int t = threadIdx.x; t < 128; t += blockDim.x) {
    double s, c;
    sincospi(-(double)t / 128.0, &s, &c);
    tw[t] = make_double2(c, s);
  }
}

// In-place radix-2 DIT FFT along one axis of every row of a TS x N tile (row stride N): the axis has
// length L and element stride st; the other index ranges over N / L lines.  inv: e^{+}, unnormalised.
// Rows sit RS = N + 1 elements apart in LDS (16-B elements: consecutive rows start 4 banks apart, so
// a wave reading one element of 16 different rows is conflict-free).
QCE_DEV void fft_axis(double2* T, int TS, int N, int L, int st, bool inv, const double2* tw) {
  if (L <= 1) return;
  const int lg = ilog2(L), lgN = ilog2(N), RS = N + 1;
  const int nthr = blockDim.x;
  auto at = [&](int s, int line, int j) -> int {  // element (line, j) of row s
    return s * RS + (st == 1 ? (line << lg) + j : line + j * st);
  };
  for (int e = threadIdx.x; e < TS * N; e += nthr) {
    const int s = e >> lgN, q = e & (N - 1);
    const int line = q >> lg, j = q & (L - 1);
    const int r = bitrev(j, lg);
    if (j < r) {
      const int a = at(s, line, j), b = at(s, line, r);
      const double2 u = T[a];
      T[a] = T[b];
      T[b] = u;
    }
  }
  __syncthreads();
  const int hN = N >> 1, lgh = lgN - 1;
  for (int len = 2; len <= L; len <<= 1) {
    const int half = len >> 1, lgl = ilog2(len), wstride = 256 >> lgl;
    for (int e = threadIdx.x; e < TS * hN; e += nthr) {
      const int s = e >> lgh, q = e & (hN - 1);
      const int line = q >> (lg - 1), bt = q & ((L >> 1) - 1);
      const int blk = bt >> (lgl - 1), t = bt & (half - 1);
      const int j0 = (blk << lgl) + t;
      const int a = at(s, line, j0), b = at(s, line, j0 + half);
      double2 w = tw[t * wstride];
      if (inv) w.y = -w.y;
      const double2 u = T[a], v = cmul(T[b], w);
      T[a] = cadd(u, v);
      T[b] = csub(u, v);
    }
    __syncthreads();
  }
}

// 2-D DFT over (n1, n2), index i = i1 n2 + i2 (kron(F_n1, F_n2) order); n1 = 1 is the 1-D DFT
QCE_DEV void fft2(double2* T, int TS, int N, int n1, int n2, bool inv, const double2* tw) {
  fft_axis(T, TS, N, n2, 1, inv, tw);
  fft_axis(T, TS, N, n1, n2, inv, tw);
}

// Bussgang gain of a diagonal entry d (same formulas as k_gain_cr, qce_prepare.hip)
QCE_DEV double bussgang_gain(double d, int kind, int n_bits, int quant_kind, double delta, const double* thr,
                             const double* lab) {
  if (kind == 0) return sqrt(2.0 / PI_D) * (1.0 / sqrt(d));
  if (kind == 2) return 1.0;
  if (quant_kind == 0) {
    const int L = 1 << n_bits;
    double dinv = 1.0 / d, acc = 0.0;
    for (int q = 1; q < L; ++q) {
      const double o = (double)q - (double)L / 2.0;
      acc += exp(-delta * delta * (o * o) * dinv);
    }
    return acc * (delta / sqrt(PI_D) / sqrt(d));
  }
  if (quant_kind == 1) {
    const int L = 1 << n_bits;
    const double dinv = 1.0 / d;
    double acc = -lab[0] * exp(-thr[0] * thr[0] * dinv);
    acc += lab[L - 1] * exp(-thr[L - 2] * thr[L - 2] * dinv);
    for (int q = 1; q < L - 1; ++q) acc += lab[q] * (exp(-thr[q - 1] * thr[q - 1] * dinv) - exp(-thr[q] * thr[q] * dinv));
    return acc / (sqrt(PI_D) * sqrt(d));
  }
  return 0.0;
}

// phase index of the 2-D DFT term e^{-2 pi i <i, m>}: (i1 m1 / n1 + i2 m2 / n2) in units of 1/N
QCE_DEV int dft_phase(int i, int m, int n1, int n2) {
  const int i1 = i / n2, i2 = i % n2, m1 = m / n2, m2 = m % n2;
  const int N = n1 * n2;
  return ((i1 * m1 % n1) * n2 + (i2 * m2 % n2) * n1) % N;  // (i1 m1/n1 + i2 m2/n2) N mod N
}

QCE_DEV double2 unit_root(int p, int N) {  // e^{-2 pi i p / N}
  double s, c;
  sincospi(-2.0 * (double)p / (double)N, &s, &c);
  return make_double2(c, s);
}

}  // namespace

// Model creation, one workgroup per component: c_k = Re DFT2(first column of C_k), mean spectrum
// mu~_k = F mu_k (unitary), and bad[k] = 1 when C_k is not (block-)circulant for (n1, n2) to a
// relative tolerance (entry (a, b) must equal entry (a - b mod, 0) in both axes).
__global__ __launch_bounds__(256) void k_fft_struct(int N, int n1, int n2, double tol, const double2* __restrict__ covs,
                                                    const double2* __restrict__ means, double* __restrict__ ceig,
                                                    double2* __restrict__ col0, double2* __restrict__ mspec,
                                                    int* __restrict__ bad) {
  const int k = blockIdx.x, tid = threadIdx.x;
  const double2* C = covs + (long long)k * N * N;
  __shared__ double red[256];
  __shared__ int s_bad;
  double mx = 0.0;
  for (int e = tid; e < N * N; e += 256) mx = fmax(mx, fmax(fabs(C[e].x), fabs(C[e].y)));
  red[tid] = mx;
  if (tid == 0) s_bad = 0;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  const double lim = tol * fmax(red[0], 1e-300);
  int b = 0;
  for (int e = tid; e < N * N; e += 256) {
    const int a = e / N, c = e % N;
    const int a1 = a / n2, a2 = a % n2, c1 = c / n2, c2 = c % n2;
    const int d = ((a1 - c1 + n1) % n1) * n2 + ((a2 - c2 + n2) % n2);
    const double2 v = C[e], w = C[(long long)d * N];
    if (fabs(v.x - w.x) > lim || fabs(v.y - w.y) > lim) b = 1;
  }
  if (b) atomicOr(&s_bad, 1);
  for (int m = tid; m < N; m += 256) col0[(long long)k * N + m] = C[(long long)m * N];
  __syncthreads();
  const double isq = 1.0 / sqrt((double)N);
  for (int i = tid; i < N; i += 256) {
    double re = 0.0;
    double2 ms = make_double2(0.0, 0.0);
    for (int m = 0; m < N; ++m) {
      const double2 w = unit_root(dft_phase(i, m, n1, n2), N);
      re += C[(long long)m * N].x * w.x - C[(long long)m * N].y * w.y;
      ms = cfma(means[(long long)k * N + m], w, ms);
    }
    ceig[(long long)k * N + i] = re;
    mspec[(long long)k * N + i] = cscale(ms, isq);
  }
  if (tid == 0) bad[k] = s_bad;
}

// Per-SNR tables, one workgroup per component (FP64):
//   rinvT[i][k] = 1 / (N r_i),  uT[i][k] = g mu~_i / (sqrt(N) r_i),
//   cprime[k] = -N log(pi) - sum log r + log w_k - sum |g mu~_i|^2 / r_i,
//   wT[k][i] = g c_i / (N r_i),  bT[k][i] = mu~_i (1 - g^2 c_i / r_i) / sqrt(N),
// status[k] = 1 when some r_i <= 0 (Cr_k not positive definite, gmm_cplx_bussgang.py:43-46).
__global__ __launch_bounds__(256) void k_fft_prep(int N, int n1, int n2, int K, double s2, int kind, int n_bits,
                                                  int quant_kind, double delta, const double* __restrict__ thr,
                                                  const double* __restrict__ lab, const double* __restrict__ logw,
                                                  const double* __restrict__ ceig, const double2* __restrict__ col0,
                                                  const double2* __restrict__ mspec, double* __restrict__ rinvT,
                                                  double2* __restrict__ uT, double* __restrict__ cprime,
                                                  double* __restrict__ wT, double2* __restrict__ bT,
                                                  double* __restrict__ gain_out, int* __restrict__ status) {
  const int k = blockIdx.x, tid = threadIdx.x;
  __shared__ double2 rho[256];
  __shared__ double red[256];
  __shared__ double redm[256];
  __shared__ int s_bad;
  const double* c = ceig + (long long)k * N;
  const double2* cc = col0 + (long long)k * N;
  const double d = cc[0].x + s2;  // the (constant) diagonal of Cy_k
  const double g = bussgang_gain(d, kind, n_bits, quant_kind, delta, thr, lab);
  const double PI2 = 2.0 / PI_D;
  if (tid == 0) s_bad = 0;
  if (kind == 0) {  // arcsine law on the first column of Cy_k = C_k + s2 I
    for (int m = tid; m < N; m += 256) {
      double2 v = cc[m];
      if (m == 0) v.x += s2;
      double re = v.x / d, im = v.y / d;
      re = re > 1.0 ? 1.0 : (re < -1.0 ? -1.0 : re);
      im = im > 1.0 ? 1.0 : (im < -1.0 ? -1.0 : im);
      rho[m] = make_double2(PI2 * asin(re), PI2 * asin(im));
    }
  }
  __syncthreads();
  double beta2 = 0.0;
  if (kind == 1) {
    const double bt = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
    beta2 = bt * bt;
  }
  const double isq = 1.0 / sqrt((double)N), invN = 1.0 / (double)N;
  double ldet = 0.0, mq = 0.0;
  for (int i = tid; i < N; i += 256) {
    double r;
    if (kind == 0) {
      r = 0.0;
      for (int m = 0; m < N; ++m) {
        const double2 w = unit_root(dft_phase(i, m, n1, n2), N);
        r += rho[m].x * w.x - rho[m].y * w.y;
      }
    } else if (kind == 2) {
      r = c[i] + s2;
    } else {
      r = beta2 * (c[i] + s2) + (1.0 - beta2) * d;
    }
    if (!(r > 0.0)) atomicOr(&s_bad, 1);
    const double2 mt = cscale(mspec[(long long)k * N + i], g);  // g mu~
    rinvT[(long long)i * K + k] = invN / r;
    uT[(long long)i * K + k] = cscale(mt, isq / r);
    wT[(long long)k * N + i] = g * c[i] * invN / r;
    bT[(long long)k * N + i] = cscale(mspec[(long long)k * N + i], (1.0 - g * g * c[i] / r) * isq);
    ldet += log(r);
    mq += (mt.x * mt.x + mt.y * mt.y) / r;
  }
  red[tid] = ldet;
  redm[tid] = mq;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[tid] += red[tid + o];
      redm[tid] += redm[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    cprime[k] = -(N * log(PI_D)) - red[0] + logw[k] - redm[0];
    gain_out[k] = g;
    status[k] = s_bad;
  }
}

// One tile of TS observations per workgroup (256 threads).  OUT: 0 = 'all' estimate h, 1 = lp only
// (B x K), 2 = weighted estimate with the selection weights wts (B x K, from k_select), 3 = K-shard
// partial (m, s, acc).  LDS: the spectra (TS x N complex) and a TS x K FP64 tile (lp, then weights).
template <int TS, int OUT>
__global__ __launch_bounds__(256) void k_fft_est(long long B, int N, int n1, int n2, int K, int has_mean,
                                                 const double2* __restrict__ y, const double* __restrict__ rinvT,
                                                 const double2* __restrict__ uT, const double* __restrict__ cprime,
                                                 const double* __restrict__ wT, const double2* __restrict__ bT,
                                                 const double* __restrict__ wts, double2* __restrict__ h,
                                                 double* __restrict__ lp_out, double* __restrict__ om,
                                                 double* __restrict__ os, float* __restrict__ oa) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);            // 128 twiddles
  double2* T = tw + 128;                                     // TS x (N + 1) spectra
  double* P = reinterpret_cast<double*>(T + TS * (N + 1));   // TS x (K + 1) lp / weights
  double* red = P + TS * (K + 1);                            // 2 x 256 reduction scratch
  constexpr int G = 256 / TS;                                // thread groups per observation
  const int tid = threadIdx.x;
  const int s = tid % TS;
  const int g = TS == 64 ? __builtin_amdgcn_readfirstlane(tid / TS) : tid / TS;  // wave-uniform at TS = 64
  const int KP = K + 1, RS = N + 1;
  const long long b0 = (long long)blockIdx.x * TS;
  const int rows = (int)((B - b0) < TS ? (B - b0) : TS);
  twiddles(tw);
  // tile of observations -> LDS (contiguous rows: coalesced 16-B loads)
  const double2* yt = y + b0 * N;
  for (int e = tid; e < TS * N; e += 256) T[(e / N) * RS + e % N] = (e / N < rows) ? yt[e] : make_double2(0.0, 0.0);
  __syncthreads();
  fft2(T, TS, N, n1, n2, false, tw);  // Y = sqrt(N) F y (unnormalised DFT)

  const int kpt = (K + G - 1) / G, k0 = g * kpt, k1 = (k0 + kpt < K) ? k0 + kpt : K;
  if (OUT != 2) {
    // lp[s][k] = c'_k - sum_i |Y_i|^2 rinv_ik + 2 sum_i Re(conj(Y_i) u_ik)
    constexpr int KC = 8;
    for (int kc = k0; kc < k1; kc += KC) {
      double acc[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) acc[j] = (kc + j < k1) ? cprime[kc + j] : 0.0;
      for (int i = 0; i < N; ++i) {
        const double2 v = T[s * RS + i];
        const double p = v.x * v.x + v.y * v.y;
        const double* ri = rinvT + (long long)i * K + kc;
#pragma unroll
        for (int j = 0; j < KC; ++j)
          if (kc + j < k1) acc[j] = fma(-p, ri[j], acc[j]);
        if (has_mean) {
          const double2* ui = uT + (long long)i * K + kc;
#pragma unroll
          for (int j = 0; j < KC; ++j)
            if (kc + j < k1) acc[j] = fma(2.0 * v.x, ui[j].x, fma(2.0 * v.y, ui[j].y, acc[j]));
        }
      }
#pragma unroll
      for (int j = 0; j < KC; ++j)
        if (kc + j < k1) P[s * KP + kc + j] = acc[j];
    }
    __syncthreads();
    if (OUT == 1) {
      for (int e = tid; e < rows * K; e += 256) lp_out[b0 * K + e] = P[(e / K) * KP + e % K];
      return;
    }
    // softmax over k: max, then e^{lp - max} and its sum; 'all' normalises, the partial keeps (m, s)
    double mx = QCE_NEG_INF;
    for (int k = k0; k < k1; ++k) mx = fmax(mx, P[s * KP + k]);
    red[g * TS + s] = mx;
    __syncthreads();
    mx = QCE_NEG_INF;
    for (int q = 0; q < G; ++q) mx = fmax(mx, red[q * TS + s]);
    __syncthreads();
    double sm = 0.0;
    for (int k = k0; k < k1; ++k) {
      const double lpv = P[s * KP + k];
      const double e = (lpv == QCE_NEG_INF) ? 0.0 : exp(lpv - mx);
      P[s * KP + k] = e;
      sm += e;
    }
    red[256 + g * TS + s] = sm;
    __syncthreads();
    sm = 0.0;
    for (int q = 0; q < G; ++q) sm += red[256 + q * TS + s];
    if (OUT == 0) {
      const double inv = 1.0 / sm;
      for (int k = k0; k < k1; ++k) P[s * KP + k] *= inv;
    } else if (g == 0 && s < rows) {
      om[b0 + s] = mx;
      os[b0 + s] = sm;
    }
  } else {
    for (int e = tid; e < TS * K; e += 256) {
      const int r = e / K, k = e % K;
      P[r * KP + k] = (r < rows) ? wts[(b0 + r) * K + k] : 0.0;
    }
  }
  __syncthreads();
  // per-bin filter f_i = sum_k gamma_k wT[k][i] and bias bb_i = sum_k gamma_k bT[k][i]; Z = Y f + bb
  {
    const int npt = N / G;  // bins per thread (N >= G for every instantiated (N, TS))
    const int i0 = g * npt;
    constexpr int NB = 16;
    for (int ic = 0; ic < npt; ic += NB) {
      double f[NB];
      double2 bb[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f[j] = 0.0;
        bb[j] = make_double2(0.0, 0.0);
      }
      for (int k = 0; k < K; ++k) {
        const double gk = P[s * KP + k];
        const double* wk = wT + (long long)k * N + i0 + ic;
#pragma unroll
        for (int j = 0; j < NB; ++j)
          if (ic + j < npt) f[j] = fma(gk, wk[j], f[j]);
        if (has_mean) {
          const double2* bk = bT + (long long)k * N + i0 + ic;
#pragma unroll
          for (int j = 0; j < NB; ++j)
            if (ic + j < npt) bb[j] = make_double2(fma(gk, bk[j].x, bb[j].x), fma(gk, bk[j].y, bb[j].y));
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j)
        if (ic + j < npt) {
          const int i = i0 + ic + j;
          const double2 v = T[s * RS + i];
          T[s * RS + i] = make_double2(fma(v.x, f[j], bb[j].x), fma(v.y, f[j], bb[j].y));
        }
    }
  }
  __syncthreads();
  fft2(T, TS, N, n1, n2, true, tw);  // h = F^H z = IFFT_unnorm(Y f / N + bb / sqrt(N)) (folded into wT, bT)
  if (OUT == 3) {
    float* at = oa + b0 * 2 * N;
    for (int e = tid; e < rows * N; e += 256) {
      const double2 v = T[(e / N) * RS + e % N];
      at[2 * e] = (float)v.x;
      at[2 * e + 1] = (float)v.y;
    }
    return;
  }
  if (OUT == 4) {  // FP64 accumulator (qce_estimate_partial_f64)
    double2* at = reinterpret_cast<double2*>(oa) + b0 * N;
    for (int e = tid; e < rows * N; e += 256) at[e] = T[(e / N) * RS + e % N];
    return;
  }
  double2* ht = h + b0 * N;
  for (int e = tid; e < rows * N; e += 256) ht[e] = T[(e / N) * RS + e % N];
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
bool qce_fft_pow2(int v) { return v >= 1 && v <= 256 && (v & (v - 1)) == 0; }

int qce_fft_tile(int N, int K) {
  // largest TS (power of two, <= 64, N / (256 / TS) >= 1) whose LDS tile fits 150 KB
  for (int ts = 64; ts >= 1; ts >>= 1) {
    const long long bytes = 128LL * 16 + (long long)ts * (N + 1) * 16 + (long long)ts * (K + 1) * 8 + 512 * 8;
    if (bytes <= 150 * 1024 && N * ts >= 256) return ts;
  }
  return 0;
}

static long long fft_lds_bytes(int TS, int N, int K) {
  return 128LL * 16 + (long long)TS * (N + 1) * 16 + (long long)TS * (K + 1) * 8 + 512 * 8;
}

hipError_t qce_launch_fft_struct(int K, int N, int n1, int n2, double tol, const double2* covs, const double2* means,
                                 double* ceig, double2* col0, double2* mspec, int* bad, hipStream_t st) {
  hipLaunchKernelGGL(k_fft_struct, dim3(K), dim3(256), 0, st, N, n1, n2, tol, covs, means, ceig, col0, mspec, bad);
  return hipGetLastError();
}

hipError_t qce_launch_fft_prep(const QceFftPrepArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_fft_prep, dim3(a.K), dim3(256), 0, st, a.N, a.n1, a.n2, a.K, a.s2, a.kind, a.n_bits,
                     a.quant_kind, a.delta, a.thr, a.lab, a.logw, a.ceig, a.col0, a.mspec, a.rinvT, a.uT, a.cprime,
                     a.wT, a.bT, a.gain, a.status);
  return hipGetLastError();
}

template <int TS, int OUT>
static hipError_t launch_fft_t(const QceFftEstArgs& a, hipStream_t st) {
  const long long lds = fft_lds_bytes(TS, a.N, a.K);
  static bool attr_set = false;  // raise the dynamic-LDS cap once per instance
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_est<TS, OUT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  dim3 grid((unsigned)((a.B + TS - 1) / TS));
  hipLaunchKernelGGL((k_fft_est<TS, OUT>), grid, dim3(256), (size_t)lds, st, a.B, a.N, a.n1, a.n2, a.K, a.has_mean,
                     a.y, a.rinvT, a.uT, a.cprime, a.wT, a.bT, a.wts, a.h, a.lp, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int OUT>
static hipError_t launch_fft_out(const QceFftEstArgs& a, hipStream_t st) {
  switch (qce_fft_tile(a.N, a.K)) {
    case 64: return launch_fft_t<64, OUT>(a, st);
    case 32: return launch_fft_t<32, OUT>(a, st);
    case 16: return launch_fft_t<16, OUT>(a, st);
    case 8: return launch_fft_t<8, OUT>(a, st);
    case 4: return launch_fft_t<4, OUT>(a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t qce_launch_fft_est(const QceFftEstArgs& a, int out, hipStream_t st) {
  if (a.B <= 0) return hipSuccess;
  switch (out) {
    case 0: return launch_fft_out<0>(a, st);
    case 1: return launch_fft_out<1>(a, st);
    case 2: return launch_fft_out<2>(a, st);
    case 3: return launch_fft_out<3>(a, st);
    case 4: return launch_fft_out<4>(a, st);
    default: return hipErrorInvalidValue;
  }
}
