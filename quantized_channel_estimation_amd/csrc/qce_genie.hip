// Per-sample ("assigned component") LMMSE: h_b = W_c y_b + b_c, c = comp[b] (or b).  Serves the genie
// Bussgang-LMMSE baseline (estimators/blmmse.py:20-62 estimate_genie: one covariance per sample, so
// the model holds one component per sample and each sample uses its own filter) and any caller
// that has already chosen the component.  FP64, like the reference.
//
// One wave per sample, lane = output row(s); y_b is broadcast from LDS; W_c rows are read with
// lane-strided addresses whose cache lines are consumed over consecutive m.  HBM-bound: the
// filter (16 N M bytes) dominates per sample.
#include "qce_common.h"
#include "qce_kernels.h"

namespace {

__global__ __launch_bounds__(256) void k_est_assigned(long long B, int N, int M, const double2* __restrict__ y,
                                                      const long long* __restrict__ comp,
                                                      const double2* __restrict__ W,
                                                      const double2* __restrict__ bvec, double2* __restrict__ h) {
  __shared__ double2 ys[4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + w;
  const bool live = b < B;
  if (live)
    for (int m = lane; m < M; m += 64) ys[w][m] = y[b * M + m];
  __syncthreads();
  if (!live) return;
  const long long c = comp ? comp[b] : b;
  const double2* Wc = W + c * (long long)N * M;
  for (int n = lane; n < N; n += 64) {
    const double2* row = Wc + (long long)n * M;
    double2 acc = bvec[c * N + n];
    for (int m = 0; m < M; ++m) acc = cfma(row[m], ys[w][m], acc);
    h[b * N + n] = acc;
  }
}

}  // namespace

hipError_t qce_launch_est_assigned(long long B, int N, int M, int K, const double2* y, const long long* comp,
                                   const double2* W, const double2* bvec, double2* h, hipStream_t st) {
  (void)K;
  hipLaunchKernelGGL(k_est_assigned, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, M, y, comp, W, bvec, h);
  return hipGetLastError();
}

// Bussgang least squares for column-orthogonal effective matrices (estimators/LS.py: lstsq(A_eff, y) with
// A_eff = G A, G diagonal, A = I or kron(x, I) as get_pilot_matrix builds it, so A_eff^H A_eff is diagonal):
// h_i = sum_m conj(A_eff[m][i]) y_m / sum_m |A_eff[m][i]|^2, the minimum-norm least-squares solution.
namespace {

__global__ __launch_bounds__(256) void k_ls_colorth(long long B, int N, int M, const double2* __restrict__ y,
                                                    const long long* __restrict__ comp,
                                                    const double2* __restrict__ Aeff, double2* __restrict__ h) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const long long c = comp ? comp[b] : b;
  const double2* Ac = Aeff + c * (long long)M * N;
  const double2* yb = y + b * M;
  for (int i = lane; i < N; i += 64) {
    double2 num = make_double2(0.0, 0.0);
    double den = 0.0;
    for (int m = 0; m < M; ++m) {
      const double2 a = Ac[(long long)m * N + i];
      num = cadd(num, cmul(cconj(a), yb[m]));
      den += a.x * a.x + a.y * a.y;
    }
    h[b * N + i] = make_double2(num.x / den, num.y / den);
  }
}

}  // namespace

hipError_t qce_launch_ls(long long B, int N, int M, const double2* y, const long long* comp, const double2* Aeff,
                         double2* h, hipStream_t st) {
  hipLaunchKernelGGL(k_ls_colorth, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, M, y, comp, Aeff, h);
  return hipGetLastError();
}

// Bussgang least squares for a general full-column-rank effective matrix (estimators/LS.py:32,47,73:
// lstsq(A_eff, y), M >= N): per component c the pseudo-inverse P_c = (A_eff^H A_eff)^{-1} A_eff^H is formed
// once by Gauss-Jordan elimination of the Hermitian positive-definite Gram matrix (no pivoting needed) on the
// augmented N x (N + M) tableau [G | A_eff^H] held in device scratch; h_b = P_c y_b then runs on
// k_est_assigned with a zero offset.  One workgroup per component; the tableau is O(K N (N + M)) bytes.
// direct = 1 eliminates [A | I] for a Hermitian positive-definite N x N A instead (A^-1 without forming A^H A,
// so the condition number is not squared: the Cq^-1 of the matched-filter rate).  A pivot that is not finite
// or whose real part falls to <= 1e-13 x the largest diagonal entry (rank-deficient / not positive definite)
// is reported through bad[c] = its index + 1; the host turns that into QCE_ECHOL.
namespace {

__global__ __launch_bounds__(256) void k_ls_pinv(int N, int M, int direct, const double2* __restrict__ Aeff,
                                                 double2* __restrict__ T, double2* __restrict__ P,
                                                 double2* __restrict__ bzero, int* __restrict__ bad) {
  __shared__ double2 f[256];
  __shared__ double dmax;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int L = N + M;
  const double2* A = Aeff + (long long)c * M * N;  // (M, N) row-major
  double2* Tc = T + (long long)c * N * L;
  for (int idx = tid; idx < N * L; idx += 256) {
    const int i = idx / L, j = idx % L;
    double2 v = make_double2(0.0, 0.0);
    if (direct) {
      v = (j < N) ? A[(long long)i * N + j] : make_double2(j - N == i ? 1.0 : 0.0, 0.0);
    } else if (j < N) {
      for (int m = 0; m < M; ++m) v = cadd(v, cmul(cconj(A[(long long)m * N + i]), A[(long long)m * N + j]));
    } else {
      v = cconj(A[(long long)(j - N) * N + i]);
    }
    Tc[idx] = v;
  }
  for (int i = tid; i < N; i += 256) bzero[(long long)c * N + i] = make_double2(0.0, 0.0);
  __syncthreads();
  if (tid == 0) {
    double d = 0.0;
    for (int i = 0; i < N; ++i) d = fmax(d, Tc[(long long)i * L + i].x);
    dmax = d;
    bad[c] = 0;
  }
  __syncthreads();
  for (int p = 0; p < N; ++p) {
    const double2 piv = Tc[(long long)p * L + p];
    if (tid == 0 && bad[c] == 0 && !(piv.x > 1e-13 * dmax && isfinite(piv.x) && isfinite(piv.y))) bad[c] = p + 1;
    const double ip = 1.0 / (piv.x * piv.x + piv.y * piv.y);
    const double2 inv = make_double2(piv.x * ip, -piv.y * ip);
    for (int r = tid; r < N; r += 256) f[r] = cmul(Tc[(long long)r * L + p], inv);
    __syncthreads();
    for (int idx = tid; idx < N * (L - p); idx += 256) {
      const int r = idx / (L - p), j = p + idx % (L - p);
      if (r == p) continue;
      Tc[(long long)r * L + j] = cadd(Tc[(long long)r * L + j], cmul(make_double2(-f[r].x, -f[r].y), Tc[(long long)p * L + j]));
    }
    __syncthreads();
    for (int j = p + tid; j < L; j += 256) Tc[(long long)p * L + j] = cmul(Tc[(long long)p * L + j], inv);
    __syncthreads();
  }
  double2* Pc = P + (long long)c * N * M;
  for (int idx = tid; idx < N * M; idx += 256) {
    const int i = idx / M, m = idx % M;
    Pc[idx] = Tc[(long long)i * L + N + m];
  }
}

}  // namespace

hipError_t qce_launch_ls_pinv(int K, int N, int M, int direct, const double2* Aeff, double2* T, double2* P,
                              double2* bzero, int* bad, hipStream_t st) {
  if (N > 256 || (direct && M != N)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_ls_pinv, dim3((unsigned)K), dim3(256), 0, st, N, M, direct, Aeff, T, P, bzero, bad);
  return hipGetLastError();
}

// Per-sample matched-filter rate of the scripts' LS branch (Bussgang_GMM.py:186-198): with v = B h_est_b,
// e = B (h_b - h_est_b), B = diag(buss) and g = v^H Cq^-1:
// rate_b = Re log2(1 + |g v|^2 / (g Cq g^H + |g e|^2)).  One wave per sample; Cq^-1 from k_ls_pinv (direct).
namespace {

__global__ __launch_bounds__(256) void k_rate_mf(long long B, int N, const double2* __restrict__ he,
                                                 const double2* __restrict__ h, const double* __restrict__ buss,
                                                 const double2* __restrict__ Cq, const double2* __restrict__ Cqi,
                                                 double* __restrict__ rate) {
  __shared__ double2 vs[4][256], gs[4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + w;
  if (b >= B) return;  // no block-wide barrier below: each wave works on its own LDS rows
  double2 ev[4];
  for (int q = 0; q < 4; ++q) {
    const int i = lane + 64 * q;
    if (i < N) {
      const double2 r = he[b * N + i], t = h[b * N + i];
      vs[w][i] = make_double2(buss[i] * r.x, buss[i] * r.y);
      ev[q] = make_double2(buss[i] * (t.x - r.x), buss[i] * (t.y - r.y));
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int q = 0; q < 4; ++q) {
    const int j = lane + 64 * q;
    if (j < N) {
      double2 g = make_double2(0.0, 0.0);
      for (int i = 0; i < N; ++i) g = cadd(g, cmul(cconj(vs[w][i]), Cqi[(long long)i * N + j]));
      gs[w][j] = g;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int q = 0; q < 4; ++q) {
    const int j = lane + 64 * q;
    if (j < N) {
      const double2 g = gs[w][j];
      const double2 a = cmul(g, vs[w][j]), c = cmul(g, ev[q]);
      double2 t = make_double2(0.0, 0.0);
      for (int k = 0; k < N; ++k) t = cadd(t, cmul(Cq[(long long)j * N + k], cconj(gs[w][k])));
      const double2 d = cmul(g, t);
      s[0] += a.x; s[1] += a.y; s[2] += d.x; s[3] += d.y; s[4] += c.x; s[5] += c.y;
    }
  }
  for (int o = 32; o > 0; o >>= 1)
    for (int u = 0; u < 6; ++u) s[u] += __shfl_xor(s[u], o, 64);
  if (lane == 0) {
    const double num = s[0] * s[0] + s[1] * s[1];
    const double dr = s[2] + s[4] * s[4] + s[5] * s[5], di = s[3];
    const double dd = dr * dr + di * di;
    const double zr = 1.0 + num * dr / dd, zi = -num * di / dd;
    rate[b] = log2(sqrt(zr * zr + zi * zi));
  }
}

__global__ __launch_bounds__(256) void k_sum_fixed(long long B, const double* __restrict__ x, double* __restrict__ out) {
  __shared__ double p[256];
  double acc = 0.0;
  for (long long i = threadIdx.x; i < B; i += 256) acc += x[i];
  p[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) p[threadIdx.x] += p[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = p[0];
}

}  // namespace

hipError_t qce_launch_rate_mf(long long B, int N, const double2* he, const double2* h, const double* buss,
                              const double2* Cq, const double2* Cqi, double* rate, double* sum, hipStream_t st) {
  if (N > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rate_mf, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, he, h, buss, Cq, Cqi, rate);
  hipLaunchKernelGGL(k_sum_fixed, dim3(1), dim3(256), 0, st, B, rate, sum);
  return hipGetLastError();
}
