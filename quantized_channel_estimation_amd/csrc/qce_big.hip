// Dense FP64 path for channel / observation dimensions beyond the fused kernels' 256 (N or M in (256, 4096]):
// the reference runs any N (gmm_cplx_bussgang.py:197-242, :388-435), e.g. 8 pilots at N = 64 (M = 512).
//
// Per row chunk of Bc observations (Bc sized so that the K-component intermediate stays below ~512 MB):
//   lp   D_k = Y L_k^-T for all k in ONE batched FP64-MFMA complex GEMM (k_zgemm_mfma, batch K), then
//        lp_bk = c_k - || D_kb - q0_k ||^2 (one wave per (b, k)): the reference's (y - mu_y)^T conj(P_k) norm
//        (:413-417) with P_k = (L_k^-1)^H, q0 = L^-1 mu_y;
//   h    Yw[b][k][:] = w_bk y_b, then ONE complex GEMM over the stacked inner dimension K M:
//        H = Yw (Bc x KM) . Wstack^T with Wstack[n][k][m] = W_k[n][m] (transposed once per prepare), plus
//        sum_k w_bk b_k -- the responsibility-weighted LMMSE sum (:220-228, :331-332) for any weights w: proba
//        ('all'), the FP64 selection weights (modes 1 / n / p), e^{lp - m} (K-shard partial) or e^{lp - shift}.
// Work per estimate: 8 K M^2 + 8 K M N real flops on FP64 MFMA, the same count as the fused kernels'.
#include <math.h>

#include "../../include/qce.h"
#include "qce_common.h"
#include "qce_kernels.h"
#include "qce_model.h"

namespace {

unsigned grid_n(long long n) {
  long long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

// lp[b][k] = c_k - sum_i |D[k][b][i] - q0[k][i]|^2, one wave per (b, k); D chunk-local rows
__global__ __launch_bounds__(256) void k_big_lp(long long Bc, int K, int M, const double2* __restrict__ D,
                                                const double2* __restrict__ q0, const double* __restrict__ cconst,
                                                double* __restrict__ lp) {
  const int lane = threadIdx.x & 63;
  const long long item = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= Bc * K) return;
  const long long b = item / K;
  const int k = (int)(item % K);
  const double2* d = D + ((long long)k * Bc + b) * M;
  const double2* q = q0 + (long long)k * M;
  double s = 0.0;
  for (int i = lane; i < M; i += 64) {
    const double2 v = csub(d[i], q[i]);
    s = fma(v.x, v.x, fma(v.y, v.y, s));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) lp[b * K + k] = cconst[k] - s;
}

// weights of one row: mode 1: w = e^{lp - m}, om = m, os = sum w; mode 2: w = e^{lp - shift}, s -> pk[b][0];
// mode 3: the responsibilities w = e^{lp - m} / sum (the 'all' mode's proba for any K, gmm_cplx_bussgang.py:220-228)
__global__ __launch_bounds__(256) void k_big_weights(long long B, int K, const double* __restrict__ lp, int mode,
                                                     const double* __restrict__ shift, double* __restrict__ w,
                                                     double* __restrict__ om, double* __restrict__ os,
                                                     double* __restrict__ pk, long long pk_stride) {
  const int lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const double* row = lp + b * K;
  double mx = -__builtin_inf();
  if (mode != 2) {
    for (int k = lane; k < K; k += 64) mx = fmax(mx, row[k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  } else {
    mx = *shift;
  }
  double s = 0.0;
  for (int k = lane; k < K; k += 64) {
    const double e = (row[k] == -__builtin_inf() || mx == -__builtin_inf()) ? 0.0 : exp(row[k] - mx);
    w[b * K + k] = e;
    s += e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (mode == 3) {
    const double inv = 1.0 / s;
    for (int k = lane; k < K; k += 64) w[b * K + k] *= inv;
    return;
  }
  if (lane == 0) {
    if (mode == 1) {
      om[b] = mx;
      os[b] = s;
    } else {
      pk[b * pk_stride] = s;
      pk[b * pk_stride + 1] = 0.0;
    }
  }
}

// Yw[b][k][m] = w[b][k] y[b][m]
__global__ __launch_bounds__(256) void k_big_scale(long long Bc, int K, int M, const double2* __restrict__ y,
                                                   const double* __restrict__ w, double2* __restrict__ yw) {
  const long long total = Bc * K * M;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long b = e / ((long long)K * M);
    const long long r = e % ((long long)K * M);
    const int k = (int)(r / M), mm = (int)(r % M);
    yw[e] = cscale(y[b * M + mm], w[b * K + k]);
  }
}

// h[b][n] (row stride ldh, double2) += sum_k w[b][k] bvec[k][n]
__global__ __launch_bounds__(256) void k_big_bias(long long Bc, int K, int N, const double* __restrict__ w,
                                                  const double2* __restrict__ bvec, double2* __restrict__ h,
                                                  long long ldh) {
  const long long total = Bc * N;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long b = e / N;
    const int n = (int)(e % N);
    double2 acc = h[b * ldh + n];
    for (int k = 0; k < K; ++k) {
      const double wk = w[b * K + k];
      if (wk != 0.0) acc = cadd(acc, cscale(bvec[(long long)k * N + n], wk));
    }
    h[b * ldh + n] = acc;
  }
}

// Wstack[n][k][m] = W_k[n][m]
__global__ __launch_bounds__(256) void k_big_stack(int K, int N, int M, const double2* __restrict__ W,
                                                   double2* __restrict__ ws) {
  const long long total = (long long)K * N * M;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int n = (int)(e / ((long long)K * M));
    const long long r = e % ((long long)K * M);
    const int k = (int)(r / M), mm = (int)(r % M);
    ws[e] = W[((long long)k * N + n) * M + mm];
  }
}

long long chunk_rows(const qce_model* m, long long B) {
  const long long per = (long long)m->K * (m->M > m->N ? m->M : m->N) * 16;  // bytes of one row's intermediate
  long long c = ((long long)512 << 20) / (per > 0 ? per : 1);
  if (c < 16) c = 16;
  return c < B ? c : B;
}

}  // namespace

#define BIG_HIP(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t e_ = (expr);                                                                            \
    if (e_ != hipSuccess) return qce_set_error(QCE_EHIP, std::string(#expr) + " failed: " + hipGetErrorString(e_)); \
  } while (0)

// Wstack of the current prepare (lazily, once per prepare)
int qce_big_prepare_filters(qce_model* m, hipStream_t st) {
  if (m->big_ws_valid) return QCE_OK;
  BIG_HIP(m->big_ws.ensure((size_t)m->K * m->N * m->M));
  hipLaunchKernelGGL(k_big_stack, dim3(grid_n((long long)m->K * m->N * m->M)), dim3(256), 0, st, m->K, m->N, m->M,
                     m->W.p, m->big_ws.p);
  BIG_HIP(hipGetLastError());
  m->big_ws_valid = 1;
  return QCE_OK;
}

int qce_big_lp(qce_model* m, const double2* y, long long B, double* lp, hipStream_t st) {
  const int K = m->K, M = m->M;
  const long long C = chunk_rows(m, B);
  BIG_HIP(m->big_d.ensure((size_t)K * C * M));
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0);
  for (long long r0 = 0; r0 < B; r0 += C) {
    const long long n = (B - r0) < C ? (B - r0) : C;
    // D_k (n x M) = Y (n x M) . Linv_k^T
    BIG_HIP(qce_zgemm_batched(0, 1, (int)n, M, M, one, y + r0 * M, M, 0, m->Linv.p, M, (long long)M * M, zero,
                              m->big_d.p, M, n * M, K, st));
    hipLaunchKernelGGL(k_big_lp, dim3((unsigned)((n * K + 3) / 4)), dim3(256), 0, st, n, K, M, m->big_d.p, m->q0.p,
                       m->cconst.p, lp + r0 * K);
    BIG_HIP(hipGetLastError());
  }
  return QCE_OK;
}

// out (row stride ldo double2, B rows) = sum_k w[b][k] (W_k y_b + b_k)
int qce_big_wsum(qce_model* m, const double2* y, long long B, const double* w, double2* out, long long ldo,
                 hipStream_t st) {
  const int K = m->K, M = m->M, N = m->N;
  if (int rc = qce_big_prepare_filters(m, st)) return rc;
  const long long C = chunk_rows(m, B);
  BIG_HIP(m->big_d.ensure((size_t)K * C * M));
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0);
  for (long long r0 = 0; r0 < B; r0 += C) {
    const long long n = (B - r0) < C ? (B - r0) : C;
    hipLaunchKernelGGL(k_big_scale, dim3(grid_n(n * K * M)), dim3(256), 0, st, n, K, M, y + r0 * M, w + r0 * K,
                       m->big_d.p);
    BIG_HIP(hipGetLastError());
    BIG_HIP(qce_zgemm_batched(0, 1, (int)n, N, K * M, one, m->big_d.p, K * M, 0, m->big_ws.p, K * M, 0, zero,
                              out + r0 * ldo, (int)ldo, 0, 1, st));
    hipLaunchKernelGGL(k_big_bias, dim3(grid_n(n * N)), dim3(256), 0, st, n, K, N, w + r0 * K, m->bvec.p,
                       out + r0 * ldo, ldo);
    BIG_HIP(hipGetLastError());
  }
  return QCE_OK;
}

// 'all'-mode responsibilities of B rows of lp (m->lp_scr) into m->w64_scr, unbounded K (no LDS-resident row)
int qce_big_proba(qce_model* m, long long B, hipStream_t st) {
  hipLaunchKernelGGL(k_big_weights, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, m->K, m->lp_scr.p, 3, nullptr,
                     m->w64_scr.p, nullptr, nullptr, nullptr, 0LL);
  BIG_HIP(hipGetLastError());
  return QCE_OK;
}

// K-shard partials: wmode 1 -> (m, s, acc (B x 2N)); wmode 2 -> shifted packed rows (B x (2N+2))
int qce_big_partial(qce_model* m, const double2* y, long long B, int wmode, double* om, double* os, double* oa,
                    double* pk, const double* shift, hipStream_t st) {
  const int K = m->K, N = m->N;
  BIG_HIP(m->lp_scr.ensure((size_t)B * K));
  BIG_HIP(m->w64_scr.ensure((size_t)B * K));
  if (int rc = qce_big_lp(m, y, B, m->lp_scr.p, st)) return rc;
  hipLaunchKernelGGL(k_big_weights, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, K, m->lp_scr.p, wmode, shift,
                     m->w64_scr.p, om, os, pk, 2LL * N + 2);
  BIG_HIP(hipGetLastError());
  if (wmode == 1) return qce_big_wsum(m, y, B, m->w64_scr.p, reinterpret_cast<double2*>(oa), N, st);
  return qce_big_wsum(m, y, B, m->w64_scr.p, reinterpret_cast<double2*>(pk) + 1, N + 1, st);
}
