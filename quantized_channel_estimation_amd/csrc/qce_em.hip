// EM training of the complex Gaussian mixture on the device:
//   E-step  resp = exp(lp - logsumexp_k lp), mean_b logsumexp      gmm_cplx_bussgang.py:612-656
//           (lp is the model's weighted log-prob, computed by the estimate path's lp kernels)
//   M-step  nk = sum_b r_bk + 10 eps; mu_k = sum_b r_bk x_b / nk    :719-723 (zero_mean -> mu = 0 :724)
//           'full': C_k = sum_b r_bk (x_b - mu_k)(x_b - mu_k)^H / nk + reg I        :739-765
//           'diag': c_k = sum r |x|^2 / nk - 2 Re(conj(mu_k) m_k) + |mu_k|^2 + reg  :767-790
//                   (m_k = sum r x / nk before the zero-mean reset, as the reference has it)
// All FP64 (the reference is complex128).  The full covariance is the hot part: K weighted
// (N x B)(B x N) Hermitian products, run on v_mfma_f64_16x16x4_f64 as four real products
// (Re = Ar Br + Ai Bi, Im = Ai Br - Ar Bi with A = r d, B = d, d = x - mu_k), 16x16 output tiles,
// one wave per row tile and four column tiles, a chunk of samples per workgroup; the chunk partials
// are summed in a fixed order (deterministic, no atomics).
//
// Roofline: MFMA (FP64).  Algorithmic flops per M-step: 8 K B N^2 (complex MAC = 8 flops).
#include "qce_common.h"
#include "qce_kernels.h"

namespace {

constexpr double EPS10 = 10.0 * 2.220446049250313e-16;  // 10 * np.finfo(float64).eps (:721)
constexpr int STAT_CHUNK = 1024;

// per (block of STAT_KB components, sample chunk): sum r, sum r x (N), sum r |x|^2 (N).
// Thread = (sample group g, feature f); each x is loaded once for STAT_KB components; the G group
// partials are added through LDS in a fixed order.
constexpr int STAT_KB = 8;

template <int NPAD>
__global__ __launch_bounds__(256) void k_em_stats(long long B, int N, int K, const double2* __restrict__ X,
                                                  const double* __restrict__ R, double* __restrict__ pnk,
                                                  double2* __restrict__ psx, double* __restrict__ psxx) {
  constexpr int G = 256 / NPAD;
  const int k0 = blockIdx.x * STAT_KB, c = blockIdx.y;
  const int f = threadIdx.x % NPAD, g = threadIdx.x / NPAD;
  const int nkb = K - k0 < STAT_KB ? K - k0 : STAT_KB;
  const long long b0 = (long long)c * STAT_CHUNK;
  const long long b1 = b0 + STAT_CHUNK < B ? b0 + STAT_CHUNK : B;
  double nk[STAT_KB], sr[STAT_KB], si[STAT_KB], sxx[STAT_KB];
#pragma unroll
  for (int j = 0; j < STAT_KB; ++j) nk[j] = sr[j] = si[j] = sxx[j] = 0.0;
  for (long long b = b0 + g; b < b1; b += G) {
    const double2 x = f < N ? X[b * N + f] : make_double2(0.0, 0.0);
    const double xx = x.x * x.x + x.y * x.y;
    const double* rb = R + b * K + k0;
#pragma unroll
    for (int j = 0; j < STAT_KB; ++j) {
      const double r = j < nkb ? rb[j] : 0.0;
      nk[j] += r;
      sr[j] += r * x.x;
      si[j] += r * x.y;
      sxx[j] += r * xx;
    }
  }
  __shared__ double red[G > 1 ? G - 1 : 1][STAT_KB][4][NPAD];
  if (G > 1 && g > 0) {
#pragma unroll
    for (int j = 0; j < STAT_KB; ++j) {
      red[g - 1][j][0][f] = nk[j];
      red[g - 1][j][1][f] = sr[j];
      red[g - 1][j][2][f] = si[j];
      red[g - 1][j][3][f] = sxx[j];
    }
  }
  __syncthreads();
  if (g != 0) return;
  for (int q = 0; q < G - 1; ++q) {
#pragma unroll
    for (int j = 0; j < STAT_KB; ++j) {
      nk[j] += red[q][j][0][f];
      sr[j] += red[q][j][1][f];
      si[j] += red[q][j][2][f];
      sxx[j] += red[q][j][3][f];
    }
  }
  for (int j = 0; j < nkb; ++j) {
    const long long o = (long long)c * K + k0 + j;
    if (f == 0) pnk[o] = nk[j];
    if (f < N) {
      psx[o * N + f] = make_double2(sr[j], si[j]);
      psxx[o * N + f] = sxx[j];
    }
  }
}

// fixed-order reduction over chunks: nk, means (or 0), m = sum r x / nk, and the diagonal variant
__global__ __launch_bounds__(256) void k_em_means(int C, int N, int K, int zero_mean, int diag, double reg,
                                                  const double* __restrict__ pnk, const double2* __restrict__ psx,
                                                  const double* __restrict__ psxx, double* __restrict__ nk_out,
                                                  double2* __restrict__ mean_out, double* __restrict__ diag_out) {
  const int k = blockIdx.x, t = threadIdx.x;
  double nk = 0.0;
  for (int c = 0; c < C; ++c) nk += pnk[(long long)c * K + k];
  nk += EPS10;
  if (t == 0) nk_out[k] = nk;
  if (t >= N) return;
  double2 sx = make_double2(0.0, 0.0);
  double sxx = 0.0;
  for (int c = 0; c < C; ++c) {
    const long long o = ((long long)c * K + k) * N + t;
    sx = cadd(sx, psx[o]);
    sxx += psxx[o];
  }
  const double2 m = make_double2(sx.x / nk, sx.y / nk);
  const double2 mu = zero_mean ? make_double2(0.0, 0.0) : m;
  mean_out[(long long)k * N + t] = mu;
  if (diag) {
    // avg_X2 - 2 Re(conj(mu) m) + |mu|^2 + reg
    const double avg_x2 = sxx / nk;
    const double re_xm = mu.x * m.x + mu.y * m.y;
    diag_out[(long long)k * N + t] = avg_x2 - 2.0 * re_xm + (mu.x * mu.x + mu.y * mu.y) + reg;
  }
}

// weighted centred covariance partials on FP64 MFMA.  Block = 4 waves; output block (blockIdx.z)
// of 4 x 4 tiles of 16 x 16; wave w owns row tile 4 rb + w and the four column tiles 4 cb + t.
__global__ __launch_bounds__(256) void k_em_cov(long long B, int N, int K, int NT, int chunk,
                                                const double2* __restrict__ X, const double* __restrict__ R,
                                                const double2* __restrict__ mean, double2* __restrict__ part) {
  const int k = blockIdx.x, c = blockIdx.y;
  const int ncb = (NT + 3) >> 2;
  const int rb = blockIdx.z / ncb, cb = blockIdx.z % ncb;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rt = rb * 4 + w;
  if (rt >= NT) return;  // no barriers below
  const int i = lane & 15, kk = lane >> 4;
  const int fr = rt * 16 + i;
  int fc[4];
  double2 muc[4];
  const double2* mk = mean + (long long)k * N;
  const double2 mur = fr < N ? mk[fr] : make_double2(0.0, 0.0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    fc[t] = (cb * 4 + t) * 16 + i;
    muc[t] = (cb * 4 + t < NT && fc[t] < N) ? mk[fc[t]] : make_double2(0.0, 0.0);
  }
  f64x4 re[4], im[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    re[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    im[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  }
  const long long b0 = (long long)c * chunk;
  const long long b1 = b0 + chunk < B ? b0 + chunk : B;
  for (long long bs = b0; bs < b1; bs += 4) {
    const long long b = bs + kk;
    const bool ok = b < b1;
    const double r = ok ? R[b * K + k] : 0.0;
    const double2* xb = X + (ok ? b : 0) * N;
    double2 dr = (ok && fr < N) ? csub(xb[fr], mur) : make_double2(0.0, 0.0);
    const double ar = r * dr.x, ai = r * dr.y;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (cb * 4 + t >= NT) continue;  // wave-uniform
      const double2 dc = (ok && fc[t] < N) ? csub(xb[fc[t]], muc[t]) : make_double2(0.0, 0.0);
      re[t] = mfma16x16x4d(ar, dc.x, re[t]);
      re[t] = mfma16x16x4d(ai, dc.y, re[t]);
      im[t] = mfma16x16x4d(ai, dc.x, im[t]);
      im[t] = mfma16x16x4d(-ar, dc.y, im[t]);
    }
  }
  double2* pk = part + ((long long)c * K + k) * N * N;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (cb * 4 + t >= NT) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = rt * 16 + kk + 4 * q, col = (cb * 4 + t) * 16 + i;
      if (row < N && col < N) pk[(long long)row * N + col] = make_double2(re[t][q], im[t][q]);
    }
  }
}

__global__ __launch_bounds__(256) void k_em_cov_final(int C, int N, int K, double reg, const double2* __restrict__ part,
                                                      const double* __restrict__ nk, double2* __restrict__ covs) {
  const long long n = (long long)K * N * N;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    double2 s = make_double2(0.0, 0.0);
    for (int c = 0; c < C; ++c) s = cadd(s, part[(long long)c * n + e]);
    const int k = (int)(e / ((long long)N * N));
    const int rc = (int)(e - (long long)k * N * N);
    const double d = nk[k];
    s = make_double2(s.x / d, s.y / d);
    if (rc / N == rc % N) s.x += reg;
    covs[e] = s;
  }
}

// E-step: one wave per sample; resp = exp(lp - lse), lse = max + log(sum exp(lp - max)) (scipy logsumexp)
__global__ __launch_bounds__(256) void k_em_resp(long long B, int K, const double* __restrict__ lp,
                                                 double* __restrict__ resp, double* __restrict__ lse) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const double* row = lp + b * K;
  double mx = -__builtin_inf();
  for (int k = lane; k < K; k += 64) mx = fmax(mx, row[k]);
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  const double sh = isinf(mx) ? 0.0 : mx;  // scipy: non-finite max -> shift 0
  double s = 0.0;
  for (int k = lane; k < K; k += 64) s += exp(row[k] - sh);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double l = log(s) + sh;
  for (int k = lane; k < K; k += 64) resp[b * K + k] = exp(row[k] - l);
  if (lane == 0) lse[b] = l;
}

constexpr int MEAN_BLOCKS = 256;

__global__ __launch_bounds__(256) void k_mean_partial(long long n, const double* __restrict__ v, double* __restrict__ part) {
  double acc = 0.0;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)MEAN_BLOCKS * 256) acc += v[e];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(64) void k_mean_final(long long n, const double* __restrict__ part, double* __restrict__ out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < MEAN_BLOCKS; i += 64) acc += part[i];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (threadIdx.x == 0) out[0] = acc / (double)n;
}

}  // namespace

namespace {

// one thread per (component, frequency p): theta = Re sum_j G[k][p][j] conj(F2[p][j])   (G = F2 Mx_k)
__global__ __launch_bounds__(256) void k_inv_em_sigma(int K, int N, int P, const double2* __restrict__ G,
                                                      const double2* __restrict__ F2, double* __restrict__ sigma,
                                                      double reg, int init) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)K * P) return;
  const int k = (int)(e / P), p = (int)(e % P);
  const double2* g = G + ((long long)k * P + p) * N;
  const double2* f = F2 + (long long)p * N;
  double th = 0.0;
  for (int j = 0; j < N; ++j) th += g[j].x * f[j].x + g[j].y * f[j].y;
  double sg = init ? th : sigma[e] + sigma[e] * th * sigma[e];  // Sigma + Sigma * Theta * Sigma (:821)
  if (sg < reg) sg = reg;                                           // (:822, and :585 at init)
  sigma[e] = sg;
}

// C_k[i][j] = sum_p conj(F2[p][i]) sigma_kp F2[p][j] + reg [i == j]   (:823-824)
__global__ __launch_bounds__(256) void k_inv_em_cov(int K, int N, int P, const double2* __restrict__ F2,
                                                    const double* __restrict__ sigma, double reg,
                                                    double2* __restrict__ C) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)K * N * N) return;
  const int k = (int)(e / ((long long)N * N));
  const int rc = (int)(e - (long long)k * N * N), i = rc / N, j = rc % N;
  const double* sg = sigma + (long long)k * P;
  double2 acc = make_double2(0.0, 0.0);
  for (int p = 0; p < P; ++p) {
    const double2 a = F2[(long long)p * N + i], b = F2[(long long)p * N + j];
    const double2 ca = make_double2(a.x * sg[p], -a.y * sg[p]);
    acc = cfma(ca, b, acc);
  }
  if (i == j) acc.x += reg;
  C[e] = acc;
}

}  // namespace

hipError_t qce_launch_inv_em_sigma(int K, int N, int P, const double2* G, const double2* F2, double* sigma, double reg,
                                   int init, hipStream_t st) {
  const long long n = (long long)K * P;
  hipLaunchKernelGGL(k_inv_em_sigma, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, K, N, P, G, F2, sigma, reg,
                     init);
  return hipGetLastError();
}

hipError_t qce_launch_inv_em_cov(int K, int N, int P, const double2* F2, const double* sigma, double reg, double2* C,
                                 hipStream_t st) {
  const long long n = (long long)K * N * N;
  hipLaunchKernelGGL(k_inv_em_cov, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, K, N, P, F2, sigma, reg, C);
  return hipGetLastError();
}

QceEmPlan qce_em_plan(long long B, int N, int K, int diag) {
  QceEmPlan p;
  p.C = (int)((B + STAT_CHUNK - 1) / STAT_CHUNK);
  p.NT = (N + 15) / 16;
  const int ncb = (p.NT + 3) / 4;
  p.nblk = ncb * ncb;
  long long c2 = (2048 + (long long)K * p.nblk - 1) / ((long long)K * p.nblk);
  const long long cmax = (B + 63) / 64;
  if (c2 > cmax) c2 = cmax;
  if (c2 < 1) c2 = 1;
  long long chunk = (B + c2 - 1) / c2;
  chunk = (chunk + 3) / 4 * 4;
  p.chunk = (int)chunk;
  p.C2 = diag ? 0 : (int)((B + chunk - 1) / chunk);
  p.stat_doubles = (size_t)p.C * K * (1 + 3 * (size_t)N);
  p.part_elems = diag ? 0 : (size_t)p.C2 * K * N * N;
  return p;
}

hipError_t qce_launch_em_mstep(const QceEmArgs& a, hipStream_t st) {
  const QceEmPlan& p = a.plan;
  const int K = a.K, N = a.N;
  double* pnk = a.stats;
  double2* psx = reinterpret_cast<double2*>(a.stats + (size_t)p.C * K);
  double* psxx = a.stats + (size_t)p.C * K * (1 + 2 * (size_t)N);
  const dim3 sg((K + STAT_KB - 1) / STAT_KB, p.C);
  if (N <= 64) hipLaunchKernelGGL(k_em_stats<64>, sg, dim3(256), 0, st, a.B, N, K, a.X, a.R, pnk, psx, psxx);
  else if (N <= 128) hipLaunchKernelGGL(k_em_stats<128>, sg, dim3(256), 0, st, a.B, N, K, a.X, a.R, pnk, psx, psxx);
  else hipLaunchKernelGGL(k_em_stats<256>, sg, dim3(256), 0, st, a.B, N, K, a.X, a.R, pnk, psx, psxx);
  hipLaunchKernelGGL(k_em_means, dim3(K), dim3(256), 0, st, p.C, N, K, a.zero_mean, a.diag, a.reg, pnk, psx, psxx,
                     a.nk, a.means, a.diag_out);
  if (!a.diag) {
    hipLaunchKernelGGL(k_em_cov, dim3(K, p.C2, p.nblk), dim3(256), 0, st, a.B, N, K, p.NT, p.chunk, a.X, a.R,
                       a.means, a.part);
    const long long n = (long long)K * N * N;
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_em_cov_final, dim3((unsigned)g), dim3(256), 0, st, p.C2, N, K, a.reg, a.part, a.nk, a.covs);
  }
  return hipGetLastError();
}

int qce_mean_scratch() { return MEAN_BLOCKS; }

hipError_t qce_launch_em_resp(long long B, int K, const double* lp, double* resp, double* lse, double* part,
                              double* mean_out, hipStream_t st) {
  hipLaunchKernelGGL(k_em_resp, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, K, lp, resp, lse);
  hipLaunchKernelGGL(k_mean_partial, dim3(MEAN_BLOCKS), dim3(256), 0, st, B, lse, part);
  hipLaunchKernelGGL(k_mean_final, dim3(1), dim3(64), 0, st, B, part, mean_out);
  return hipGetLastError();
}
