// Dispatch of the chunk-streamed large-shape estimate kernel (qce_h2x_kernel.h; one translation
// unit per padded shape, qce_h2x_s*.hip, so the fully unrolled instances compile in parallel) and
// the split-record merge.
#include "qce_h2x_kernel.h"

// Combine S split records per sample (one wave per sample):
// h = sum_s acc_s e^{m_s - M} / sum_s s_s e^{m_s - M}, or the merged (m, s, acc) partial.
__global__ __launch_bounds__(256) void k_merge_splits(long long B, int N, int S, const double* __restrict__ rm,
                                                      const double* __restrict__ rs, const float* __restrict__ ra,
                                                      double2* __restrict__ h, double* __restrict__ om,
                                                      double* __restrict__ os, float* __restrict__ oa) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  double mx = QCE_NEG_INF;
  for (int s = 0; s < S; ++s) mx = fmax(mx, rm[(long long)s * B + b]);
  double tot = 0.0;
  for (int s = 0; s < S; ++s) {
    const double ms = rm[(long long)s * B + b];
    tot += (ms == QCE_NEG_INF) ? 0.0 : rs[(long long)s * B + b] * exp(ms - mx);
  }
  for (int n = lane; n < N; n += 64) {
    double re = 0.0, im = 0.0;
    for (int s = 0; s < S; ++s) {
      const long long r = (long long)s * B + b;
      const double sc = (rm[r] == QCE_NEG_INF) ? 0.0 : exp(rm[r] - mx);
      const float2 v = *reinterpret_cast<const float2*>(ra + r * 2 * N + 2 * n);
      re += (double)v.x * sc;
      im += (double)v.y * sc;
    }
    if (h) {
      h[b * N + n] = make_double2(re / tot, im / tot);
    } else {
      oa[b * 2 * N + 2 * n] = (float)re;
      oa[b * 2 * N + 2 * n + 1] = (float)im;
    }
  }
  if (!h && lane == 0) {
    om[b] = mx;
    os[b] = tot;
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
// padded (MP, NP) pairs with an instance: {64, 128, 256}^2 without (64, 64) (qce_estimate_h2.hip)
#define QCE_H2X_SHAPES(X) X(64, 128) X(64, 256) X(128, 64) X(128, 128) X(128, 256) X(256, 64) X(256, 128) X(256, 256)

#define QCE_DECL(X, Y) hipError_t qce_h2x_launch_##X##x##Y(const QceH2XArgs& a, bool hm, int ksplit, int out_rec, hipStream_t st);
QCE_H2X_SHAPES(QCE_DECL)
#undef QCE_DECL

bool qce_h2x_shape(int MP, int NP) {
#define QCE_CASE(X, Y) \
  if (MP == X && NP == Y) return true;
  QCE_H2X_SHAPES(QCE_CASE)
#undef QCE_CASE
  return false;
}

long long qce_h2x_pad_bytes() { return (long long)X_CHB * 2; }

int qce_h2x_tile() { return X_TILE; }

int qce_h2x_row_chunks(int MP, int NP) { return ((2 * NP) / 32) / x_rsw(MP, NP, true); }

hipError_t qce_launch_est_h2x(const QceH2XArgs& a, int ksplit, bool out_partial, hipStream_t st) {
  const bool hm = a.has_mean != 0;
  hipError_t e = hipMemsetAsync(a.yflag, 0, sizeof(int), st);
  if (e != hipSuccess) return e;
  if ((e = qce_launch_y_exact(a.B * a.M * 2, reinterpret_cast<const double*>(a.y), a.y_scale, a.yflag, st)) !=
      hipSuccess)
    return e;
  const bool direct = ksplit == 1;  // no merge: final h, or the partial written straight as records
  QceH2XArgs b = a;
  if (direct && out_partial) {
    b.rm = a.om;
    b.rs = a.os;
    b.ra = a.oa;
  }
  const int out_rec = (direct && !out_partial) ? 0 : 1;
  e = hipErrorInvalidValue;
#define QCE_CASE(X, Y) \
  if (a.MP == X && a.NP == Y) e = qce_h2x_launch_##X##x##Y(b, hm, ksplit, out_rec, st);
  QCE_H2X_SHAPES(QCE_CASE)
#undef QCE_CASE
  if (e != hipSuccess || direct) return e;
  hipLaunchKernelGGL(k_merge_splits, dim3((unsigned)((a.B + 3) / 4)), dim3(256), 0, st, a.B, a.N, ksplit, a.rm, a.rs,
                     a.ra, out_partial ? nullptr : a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}
