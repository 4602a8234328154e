// Estimate-side kernels of the Bussgang-GMM estimator (gfx950 / CDNA4).
//
// Restated hot path (gmm_cplx_bussgang.py):
//   lp[b,k] = c_k - || Linv_k (y_b - mu_y,k) ||^2                (:388-435, :369-386)
//   gamma   = softmax_k lp                                        (:632-656, :351-367)
//   'all'   : h_b = sum_k gamma_bk (W_k y_b + b_k)                (:220-228, :331-332)
//   1 / n / p: selection over gamma, renormalised                 (:197-219, :229-242)
//
// k_est_all_f32 is a flash-style single pass over the K components for a tile of
// 128 samples (4 waves x 32 samples): per component the whitened residual
// u = E(Linv_k) [y;1] runs on v_mfma_f32_32x32x2_f32 (lower-triangular tiles skipped),
// its squared norm gives lp in FP64, an online softmax (running max m, sum s) rescales the
// accumulator, and Z = E(W_k) [y;1] on the same MFMA is folded in with weight e^{lp-m}.
// The samples sit on the MFMA column (lane) axis, so every per-sample scalar (quad form,
// m, s, weight) is a per-lane register and the Y^T fragments stay resident in VGPRs for
// the whole K loop; component tables stream from L2 in fragment order (16 B per lane).
#include "qce_common.h"
#include "qce_kernels.h"

#define QCE_NEG_INF (-__builtin_inf())

template <int MP, int NP, bool HAS_MEAN, bool PARTIAL>
__global__ __launch_bounds__(256, 2) void k_est_all_f32(long long B, int M, int N, int K, const double2* __restrict__ y,
                                                        const float* __restrict__ pack, long long comp_stride,
                                                        const double* __restrict__ cconst, double2* __restrict__ h,
                                                        double* __restrict__ part_m, double* __restrict__ part_s,
                                                        float* __restrict__ part_acc) {
  constexpr int R = 2 * MP, S = 2 * NP;
  constexpr int NSL = R / 32, NSW = S / 32;
  constexpr int GW = MP / 4;
  constexpr int HM = HAS_MEAN ? 1 : 0;
  constexpr int GL_TOTAL = 2 * NSL * (NSL + 1) + HM * NSL;  // sum_r (4r+4+HM)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, hh = lane >> 5;
  const long long sample = (long long)blockIdx.x * 128 + wave * 32 + j;
  const bool valid = sample < B;

  float yv[MP + HM];
#pragma unroll
  for (int s = 0; s < MP; ++s) {
    float v = 0.0f;
    if (valid && s < M) {
      const double* yp = reinterpret_cast<const double*>(y + sample * M + s);
      v = (float)yp[hh];
    }
    yv[s] = v;
  }
  if (HAS_MEAN) yv[MP] = hh ? 0.0f : 1.0f;

  f32x16 out[NSW];
#pragma unroll
  for (int r = 0; r < NSW; ++r)
#pragma unroll
    for (int q = 0; q < 16; ++q) out[r][q] = 0.0f;
  double m = QCE_NEG_INF, ssum = 0.0;

  for (int k = 0; k < K; ++k) {
    const f32x4* __restrict__ pk = reinterpret_cast<const f32x4*>(pack + (long long)k * comp_stride) + lane;
    double quad = 0.0;
    int goff = 0;
#pragma unroll
    for (int r = 0; r < NSL; ++r) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
      for (int g = 0; g < 4 * r + 4; ++g) {
        f32x4 a = pk[(goff + g) * 64];
        acc = mfma32x32x2(a[0], yv[4 * g + 0], acc);
        acc = mfma32x32x2(a[1], yv[4 * g + 1], acc);
        acc = mfma32x32x2(a[2], yv[4 * g + 2], acc);
        acc = mfma32x32x2(a[3], yv[4 * g + 3], acc);
      }
      if (HAS_MEAN) {
        f32x4 a = pk[(goff + 4 * r + 4) * 64];
        acc = mfma32x32x2(a[0], yv[MP], acc);
      }
      goff += 4 * r + 4 + HM;
#pragma unroll
      for (int q = 0; q < 16; ++q) quad = fma((double)acc[q], (double)acc[q], quad);
    }
    quad += __shfl_xor(quad, 32);
    const double lp = cconst[k] - quad;
    const double mnew = fmax(m, lp);
    const double alpha = (m == mnew) ? 1.0 : exp(m - mnew);
    const double p = (lp == QCE_NEG_INF) ? 0.0 : exp(lp - mnew);
    ssum = ssum * alpha + p;
    m = mnew;
    const float af = (float)alpha, pf = (float)p;
#pragma unroll
    for (int r = 0; r < NSW; ++r) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
      const int base = GL_TOTAL + r * (GW + HM);
#pragma unroll
      for (int g = 0; g < GW; ++g) {
        f32x4 a = pk[(base + g) * 64];
        acc = mfma32x32x2(a[0], yv[4 * g + 0], acc);
        acc = mfma32x32x2(a[1], yv[4 * g + 1], acc);
        acc = mfma32x32x2(a[2], yv[4 * g + 2], acc);
        acc = mfma32x32x2(a[3], yv[4 * g + 3], acc);
      }
      if (HAS_MEAN) {
        f32x4 a = pk[(base + GW) * 64];
        acc = mfma32x32x2(a[0], yv[MP], acc);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) out[r][q] = fmaf(out[r][q], af, pf * acc[q]);
    }
  }

  if (!valid) return;
  if (PARTIAL) {
    if (hh == 0) {
      part_m[sample] = m;
      part_s[sample] = ssum;
    }
    float* pa = part_acc + sample * (2LL * N);
#pragma unroll
    for (int r = 0; r < NSW; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 16 * r + 4 * q + 2 * hh;
        if (n0 < N) {
          pa[2 * n0] = out[r][4 * q + 0];
          pa[2 * n0 + 1] = out[r][4 * q + 1];
        }
        if (n0 + 1 < N) {
          pa[2 * n0 + 2] = out[r][4 * q + 2];
          pa[2 * n0 + 3] = out[r][4 * q + 3];
        }
      }
    return;
  }
  const double inv = 1.0 / ssum;
  double2* hp = h + sample * N;
#pragma unroll
  for (int r = 0; r < NSW; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 16 * r + 4 * q + 2 * hh;
      if (n0 < N) hp[n0] = make_double2((double)out[r][4 * q + 0] * inv, (double)out[r][4 * q + 1] * inv);
      if (n0 + 1 < N) hp[n0 + 1] = make_double2((double)out[r][4 * q + 2] * inv, (double)out[r][4 * q + 3] * inv);
    }
}

// h = sum_k w[b][k] (W_k y + b_k): the LMMSE half only, for the selective modes.  A
// component no sample of the wave selected is skipped wave-uniformly.
template <int MP, int NP, bool HAS_MEAN, int RC>
__global__ __launch_bounds__(256, (MP > 64 || NP > 64) ? 1 : 2) void k_est_weighted_f32(long long B, int M, int N, int K,
                                                             const double2* __restrict__ y,
                                                             const float* __restrict__ pack, long long comp_stride,
                                                             const float* __restrict__ wts, double2* __restrict__ h) {
  constexpr int R = 2 * MP, S = 2 * NP;
  constexpr int NSL = R / 32, NSW = S / 32;
  constexpr int GW = MP / 4;
  constexpr int HM = HAS_MEAN ? 1 : 0;
  constexpr int GL_TOTAL = 2 * NSL * (NSL + 1) + HM * NSL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, hh = lane >> 5;
  const long long sample = (long long)blockIdx.x * 128 + wave * 32 + j;
  const bool valid = sample < B;
  float yv[MP + HM];
#pragma unroll
  for (int s = 0; s < MP; ++s) {
    float v = 0.0f;
    if (valid && s < M) {
      const double* yp = reinterpret_cast<const double*>(y + sample * M + s);
      v = (float)yp[hh];
    }
    yv[s] = v;
  }
  if (HAS_MEAN) yv[MP] = hh ? 0.0f : 1.0f;
  static_assert(NSW % RC == 0, "row chunk");
  const int r0 = blockIdx.y * RC;  // first W slice of this workgroup's row chunk
  f32x16 out[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int q = 0; q < 16; ++q) out[r][q] = 0.0f;
  for (int k = 0; k < K; ++k) {
    const float w = valid ? wts[sample * K + k] : 0.0f;
    if (__ballot(w != 0.0f) == 0ull) continue;
    const f32x4* __restrict__ pk = reinterpret_cast<const f32x4*>(pack + (long long)k * comp_stride) + lane;
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
      const int base = GL_TOTAL + (r0 + r) * (GW + HM);
#pragma unroll
      for (int g = 0; g < GW; ++g) {
        f32x4 a = pk[(base + g) * 64];
        acc = mfma32x32x2(a[0], yv[4 * g + 0], acc);
        acc = mfma32x32x2(a[1], yv[4 * g + 1], acc);
        acc = mfma32x32x2(a[2], yv[4 * g + 2], acc);
        acc = mfma32x32x2(a[3], yv[4 * g + 3], acc);
      }
      if (HAS_MEAN) {
        f32x4 a = pk[(base + GW) * 64];
        acc = mfma32x32x2(a[0], yv[MP], acc);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) out[r][q] = fmaf(w, acc[q], out[r][q]);
    }
  }
  if (!valid) return;
  double2* hp = h + sample * N;
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 16 * (r0 + r) + 4 * q + 2 * hh;
      if (n0 < N) hp[n0] = make_double2((double)out[r][4 * q + 0], (double)out[r][4 * q + 1]);
      if (n0 + 1 < N) hp[n0 + 1] = make_double2((double)out[r][4 * q + 2], (double)out[r][4 * q + 3]);
    }
}

// lp[b][k] in FP64 on v_mfma_f64_16x16x4_f64 (exact argmax / ranking for the selective modes
// and for predict_proba_cplx / _predict_cplx).  4 waves x 16 samples per workgroup.
template <int MP, bool HAS_MEAN>
__global__ __launch_bounds__(256, MP > 64 ? 1 : 2) void k_lp_f64(long long B, int M, int K, const double2* __restrict__ y,
                                                   const double* __restrict__ pack, long long comp_stride,
                                                   const double* __restrict__ cconst, double* __restrict__ lp) {
  constexpr int R = 2 * MP;
  constexpr int NSL = R / 16;
  constexpr int NS = MP / 2;  // k-steps of 4 real columns
  constexpr int HM = HAS_MEAN ? 1 : 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long sample = (long long)blockIdx.x * 64 + wave * 16 + (lane & 15);
  const bool valid = sample < B;
  double yd[NS + HM];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = 2 * s + (lane >> 5), part = (lane >> 4) & 1;
    double v = 0.0;
    if (valid && c < M) v = reinterpret_cast<const double*>(y + sample * M + c)[part];
    yd[s] = v;
  }
  if (HAS_MEAN) yd[NS] = (lane >> 4) == 0 ? 1.0 : 0.0;
  for (int k = 0; k < K; ++k) {
    const double* __restrict__ pk = pack + (long long)k * comp_stride + lane;
    double quad = 0.0;
    int soff = 0;
#pragma unroll
    for (int r = 0; r < NSL; ++r) {
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4 * r + 4; ++s) acc = mfma16x16x4d(pk[(soff + s) * 64], yd[s], acc);
      if (HAS_MEAN) acc = mfma16x16x4d(pk[(soff + 4 * r + 4) * 64], yd[NS], acc);
      soff += 4 * r + 4 + HM;
#pragma unroll
      for (int q = 0; q < 4; ++q) quad = fma(acc[q], acc[q], quad);
    }
    quad += __shfl_xor(quad, 16);
    quad += __shfl_xor(quad, 32);
    if (valid && (lane >> 4) == 0) lp[sample * K + k] = cconst[k] - quad;
  }
}

// ---------------------------------------------------------------------------
// per-sample selection, one wave per sample (K <= 256: 4 values per lane)
// ---------------------------------------------------------------------------
QCE_DEV double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
QCE_DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// argmax with (value, index) ordering: larger value wins; on ties prefer_low selects the lower index
QCE_DEV void wave_argmax(double& v, int& idx, bool prefer_low) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o);
    int oi = __shfl_xor(idx, o);
    bool take = (ov > v) || (ov == v && (prefer_low ? (oi < idx) : (oi > idx)));
    if (take) {
      v = ov;
      idx = oi;
    }
  }
}

__global__ __launch_bounds__(256) void k_select(long long B, int K, const double* __restrict__ lp, int mode, int nsel,
                                                double psel, double* __restrict__ proba, long long* __restrict__ labels,
                                                float* __restrict__ wts, double* __restrict__ wts64) {
  const int lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const double* row = lp + b * K;
  double v[4];
  int taken = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = lane + 64 * i;
    v[i] = k < K ? row[k] : QCE_NEG_INF;
  }
  // labels: first index of max lp (numpy argmax)
  double bv = QCE_NEG_INF;
  int bi = 1 << 30;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = lane + 64 * i;
    if (k < K && (v[i] > bv || (v[i] == bv && k < bi) || bi == (1 << 30))) {
      bv = v[i];
      bi = k;
    }
  }
  wave_argmax(bv, bi, true);
  if (labels && lane == 0) labels[b] = bi;
  // logsumexp (scipy.special.logsumexp) -> proba = exp(lp - lse)
  const double mx = wave_max(fmax(fmax(v[0], v[1]), fmax(v[2], v[3])));
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < K) t += exp(v[i] - mx);
  const double lse = log(wave_sum(t)) + mx;
  double pr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) pr[i] = (lane + 64 * i < K) ? exp(v[i] - lse) : -1.0;
  if (proba) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (lane + 64 * i < K) proba[b * K + lane + 64 * i] = pr[i];
  }
  if (!wts && !wts64) return;
  double w[4] = {0.0, 0.0, 0.0, 0.0};
  if (mode == 3 || (mode == 1 && nsel == 1)) {  // argmax path (:200-207): h = h_label, weight exactly 1
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (lane + 64 * i == bi) w[i] = 1.0;
  } else if (mode == 1 || mode == 2) {
    // descending-proba selection (:213 / :235-236); ties broken towards the higher index,
    // matching a reversed stable ascending sort
    double cum = 0.0;
    double chosen[4] = {0.0, 0.0, 0.0, 0.0};
    const int limit = (mode == 1) ? (nsel < K ? nsel : K) : K;
    for (int it = 0; it < limit; ++it) {
      double cv = -2.0;
      int ci = -1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = lane + 64 * i;
        if (k < K && !((taken >> i) & 1) && (pr[i] > cv || (pr[i] == cv && k > ci))) {
          cv = pr[i];
          ci = k;
        }
      }
      wave_argmax(cv, ci, false);
      if (ci < 0) break;
      if ((ci & 63) == lane) {
        taken |= 1 << (ci >> 6);
        chosen[ci >> 6] = cv;
      }
      cum += cv;
      if (mode == 2 && cum >= psel) break;
    }
    // normalise by the sum of the selected probabilities (:219 / :242)
    double tot = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((taken >> i) & 1) tot += chosen[i];
    tot = wave_sum(tot);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((taken >> i) & 1) w[i] = chosen[i] / tot;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < K) {
      if (wts) wts[b * K + lane + 64 * i] = (float)w[i];
      if (wts64) wts64[b * K + lane + 64 * i] = w[i];
    }
}

// ---------------------------------------------------------------------------
// k_select for K > 256 (up to QCE_SELECT_WIDE_MAX): one 256-thread workgroup per sample, the row in LDS.
// Same results as k_select: labels = first maximum of lp (numpy argmax), proba = exp(lp - logsumexp);
// top-n / cumulative-p select in descending-proba order with ties towards the higher index (a bitonic sort of
// (proba, index) keys in LDS), the cumulative sum taken sequentially in that order (np.cumsum + searchsorted,
// gmm_cplx_bussgang.py:213, :235-236), weights renormalised by the selected sum (:219, :242).
// ---------------------------------------------------------------------------
#define QCE_SELECT_WIDE_MAX 4096

QCE_DEV bool sel_before(double va, int ia, double vb, int ib) { return va > vb || (va == vb && ia > ib); }

__global__ __launch_bounds__(256) void k_select_wide(long long B, int K, int P, const double* __restrict__ lp,
                                                     int mode, int nsel, double psel, double* __restrict__ proba,
                                                     long long* __restrict__ labels, float* __restrict__ wts,
                                                     double* __restrict__ wts64) {
  extern __shared__ double sel_lds[];
  double* v = sel_lds;                                // P values
  int* id = reinterpret_cast<int*>(sel_lds + P);      // P indices
  __shared__ double rv[4];
  __shared__ int ri[4];
  __shared__ double s_tot;
  __shared__ int s_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long b = blockIdx.x;
  const double* row = lp + b * K;
  // max and first argmax
  double bv = QCE_NEG_INF;
  int bi = 1 << 30;
  for (int k = tid; k < K; k += 256) {
    const double x = row[k];
    v[k] = x;
    if (x > bv || bi == (1 << 30)) {
      bv = x;
      bi = k;
    }
  }
  wave_argmax(bv, bi, true);
  if (lane == 0) {
    rv[wv] = bv;
    ri[wv] = bi;
  }
  __syncthreads();
  bv = rv[0];
  bi = ri[0];
  for (int w = 1; w < 4; ++w)
    if (rv[w] > bv || (rv[w] == bv && ri[w] < bi)) {
      bv = rv[w];
      bi = ri[w];
    }
  if (labels && tid == 0) labels[b] = bi;
  const double mx = bv;
  double t = 0.0;
  for (int k = tid; k < K; k += 256) t += exp(v[k] - mx);
  t = wave_sum(t);
  __syncthreads();
  if (lane == 0) rv[wv] = t;
  __syncthreads();
  const double lse = log(rv[0] + rv[1] + rv[2] + rv[3]) + mx;
  for (int k = tid; k < K; k += 256) {
    const double pr = exp(v[k] - lse);
    if (proba) proba[b * K + k] = pr;
    v[k] = pr;
    id[k] = k;
  }
  if (!wts && !wts64) return;
  if (mode == 3 || (mode == 1 && nsel == 1)) {  // argmax path: weight exactly 1 on the first maximum
    for (int k = tid; k < K; k += 256) {
      const double w = (k == bi) ? 1.0 : 0.0;
      if (wts) wts[b * K + k] = (float)w;
      if (wts64) wts64[b * K + k] = w;
    }
    return;
  }
  for (int k = K + tid; k < P; k += 256) {
    v[k] = -2.0;  // below every probability
    id[k] = -1;
  }
  __syncthreads();
  // bitonic sort, descending by (proba, index)
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const double va = v[i], vb = v[j];
          const int ia = id[i], ib = id[j];
          if (desc ? sel_before(vb, ib, va, ia) : sel_before(va, ia, vb, ib)) {
            v[i] = vb;
            v[j] = va;
            id[i] = ib;
            id[j] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0) {  // sequential prefix in the sorted order
    int cnt = (mode == 1) ? (nsel < K ? nsel : K) : K;
    double cum = 0.0;
    if (mode == 2) {
      for (int j = 0; j < K; ++j) {
        cum += v[j];
        if (cum >= psel) {
          cnt = j + 1;
          break;
        }
      }
    }
    double tot = 0.0;
    for (int j = 0; j < cnt; ++j) tot += v[j];
    s_cnt = cnt;
    s_tot = tot;
  }
  __syncthreads();
  const int cnt = s_cnt;
  const double tot = s_tot;
  for (int j = tid; j < K; j += 256) {  // every component sits at exactly one sorted position
    const double w = j < cnt ? v[j] / tot : 0.0;
    const int k = id[j];
    if (wts) wts[b * K + k] = (float)w;
    if (wts64) wts64[b * K + k] = w;
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
bool qce_shape_supported(int MP, int NP) {  // the FP32 fused 'all' kernel (k_est_all_f32)
  auto ok = [](int v) { return v == 16 || v == 32 || v == 64; };
  return ok(MP) && ok(NP);
}

bool qce_select_shape_supported(int MP, int NP) {  // lp (FP64) + weighted LMMSE kernels
  return qce_shape_supported(MP, NP) || ((MP == 64 || MP == 128 || MP == 256) && (NP == 64 || NP == 128 || NP == 256));
}

template <int MP, int NP, bool HM>
static hipError_t launch_all_t(const QceEstArgs& a, double2* h, double* pm, double* ps, float* pa, bool partial,
                               hipStream_t st) {
  dim3 grid((unsigned)((a.B + 127) / 128));
  if (partial)
    hipLaunchKernelGGL((k_est_all_f32<MP, NP, HM, true>), grid, dim3(256), 0, st, a.B, a.M, a.N, a.K, a.y, a.pack32,
                       a.stride32, a.cconst, h, pm, ps, pa);
  else
    hipLaunchKernelGGL((k_est_all_f32<MP, NP, HM, false>), grid, dim3(256), 0, st, a.B, a.M, a.N, a.K, a.y, a.pack32,
                       a.stride32, a.cconst, h, pm, ps, pa);
  return hipGetLastError();
}

template <int MP, int NP, bool HM>
static hipError_t launch_w_t(const QceEstArgs& a, const float* w, double2* h, hipStream_t st) {
  // row chunk: y (MP + 1 registers) + RC accumulator slices (16 registers each) within ~400
  constexpr int NSW = (2 * NP) / 32;
  constexpr int RC = (MP <= 64 && NP <= 64) ? NSW : ((MP + 16 * NSW <= 400) ? NSW : (MP + 128 <= 400 ? 8 : 4));
  dim3 grid((unsigned)((a.B + 127) / 128), NSW / RC);
  hipLaunchKernelGGL((k_est_weighted_f32<MP, NP, HM, RC>), grid, dim3(256), 0, st, a.B, a.M, a.N, a.K, a.y, a.pack32,
                     a.stride32, w, h);
  return hipGetLastError();
}

template <int MP, bool HM>
static hipError_t launch_lp_t(const QceEstArgs& a, double* lp, hipStream_t st) {
  dim3 grid((unsigned)((a.B + 63) / 64));
  hipLaunchKernelGGL((k_lp_f64<MP, HM>), grid, dim3(256), 0, st, a.B, a.M, a.K, a.y, a.pack64, a.stride64, a.cconst,
                     lp);
  return hipGetLastError();
}

#define QCE_FOR_SHAPES(X) \
  X(16, 16) X(16, 32) X(16, 64) X(32, 16) X(32, 32) X(32, 64) X(64, 16) X(64, 32) X(64, 64)

hipError_t qce_launch_est_all(const QceEstArgs& a, double2* h, hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_CASE(X, Y)                                                                      \
  if (a.MP == X && a.NP == Y)                                                               \
    return hm ? launch_all_t<X, Y, true>(a, h, nullptr, nullptr, nullptr, false, st)        \
              : launch_all_t<X, Y, false>(a, h, nullptr, nullptr, nullptr, false, st);
  QCE_FOR_SHAPES(QCE_CASE)
#undef QCE_CASE
  return hipErrorInvalidValue;
}

hipError_t qce_launch_est_partial(const QceEstArgs& a, double* m, double* s, float* acc, hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_CASE(X, Y)                                                                      \
  if (a.MP == X && a.NP == Y)                                                               \
    return hm ? launch_all_t<X, Y, true>(a, nullptr, m, s, acc, true, st)                   \
              : launch_all_t<X, Y, false>(a, nullptr, m, s, acc, true, st);
  QCE_FOR_SHAPES(QCE_CASE)
#undef QCE_CASE
  return hipErrorInvalidValue;
}

#define QCE_FOR_LARGE_SHAPES(X) X(64, 128) X(64, 256) X(128, 64) X(128, 128) X(128, 256) X(256, 64) X(256, 128) X(256, 256)

hipError_t qce_launch_est_weighted(const QceEstArgs& a, const float* w, double2* h, hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_CASE(X, Y) \
  if (a.MP == X && a.NP == Y) return hm ? launch_w_t<X, Y, true>(a, w, h, st) : launch_w_t<X, Y, false>(a, w, h, st);
  QCE_FOR_SHAPES(QCE_CASE)
  QCE_FOR_LARGE_SHAPES(QCE_CASE)
#undef QCE_CASE
  return hipErrorInvalidValue;
}

hipError_t qce_launch_lp(const QceEstArgs& a, double* lp, hipStream_t st) {
  const bool hm = a.has_mean != 0;
  switch (a.MP) {
    case 16: return hm ? launch_lp_t<16, true>(a, lp, st) : launch_lp_t<16, false>(a, lp, st);
    case 32: return hm ? launch_lp_t<32, true>(a, lp, st) : launch_lp_t<32, false>(a, lp, st);
    case 64: return hm ? launch_lp_t<64, true>(a, lp, st) : launch_lp_t<64, false>(a, lp, st);
    case 128: return hm ? launch_lp_t<128, true>(a, lp, st) : launch_lp_t<128, false>(a, lp, st);
    case 256: return hm ? launch_lp_t<256, true>(a, lp, st) : launch_lp_t<256, false>(a, lp, st);
    default: return hipErrorInvalidValue;
  }
}

int qce_select_max_k() { return QCE_SELECT_WIDE_MAX; }

hipError_t qce_launch_select(long long B, int K, const double* lp, int mode, int n, double p, double* proba,
                             long long* labels, float* wts, hipStream_t st, double* wts64) {
  if (K > 256) {
    if (K > QCE_SELECT_WIDE_MAX) return hipErrorInvalidValue;
    int P = 1;
    while (P < K) P <<= 1;
    const size_t lds = (size_t)P * (sizeof(double) + sizeof(int));
    hipLaunchKernelGGL(k_select_wide, dim3((unsigned)B), dim3(256), lds, st, B, K, P, lp, mode, n, p, proba, labels, wts,
                       wts64);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((B + 3) / 4));
  hipLaunchKernelGGL(k_select, grid, dim3(256), 0, st, B, K, lp, mode, n, p, proba, labels, wts, wts64);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// FP64 selective-mode LMMSE (gmm_cplx_bussgang.py:200-219, :229-242): h_b = sum_k w_bk (W_k y_b + b_k) over the
// components the selection kept (w_bk != 0, wave-uniform skip), FP64 VALU.  One wave per sample, y in LDS,
// filters transposed (WT_k = W_k^T, M x N) so the 64 lanes (output rows) read one coalesced 1 KB row per m.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_est_sparse_f64(long long B, int N, int M, int K, const double2* __restrict__ y,
                                                        const double* __restrict__ w, const double2* __restrict__ WT,
                                                        const double2* __restrict__ bvec, double2* __restrict__ h) {
  __shared__ double2 ys[4][256];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + wv;
  const bool live = b < B;
  if (live)
    for (int m = lane; m < M; m += 64) ys[wv][m] = y[b * M + m];
  __syncthreads();
  if (!live) return;
  double2 acc[4];  // rows n = lane + 64 r (N <= 256)
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = make_double2(0.0, 0.0);
  const double* wr = w + b * K;
  for (int k = 0; k < K; ++k) {
    const double wk = wr[k];
    if (wk == 0.0) continue;  // same value in every lane of the wave
    const double2* Wk = WT + (long long)k * M * N;
    double2 t[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) t[r] = (lane + 64 * r < N) ? bvec[(long long)k * N + lane + 64 * r] : make_double2(0.0, 0.0);
    for (int m = 0; m < M; ++m) {
      const double2 ym = ys[wv][m];
      const double2* row = Wk + (long long)m * N;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (lane + 64 * r < N) t[r] = cfma(row[lane + 64 * r], ym, t[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc[r].x = fma(wk, t[r].x, acc[r].x);
      acc[r].y = fma(wk, t[r].y, acc[r].y);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (lane + 64 * r < N) h[b * N + lane + 64 * r] = acc[r];
}

// WT_k[m][n] = W_k[n][m]
__global__ __launch_bounds__(256) void k_transpose_w(int K, int N, int M, const double2* __restrict__ W,
                                                     double2* __restrict__ WT) {
  const long long total = (long long)K * N * M;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long k = e / ((long long)M * N), r = e % ((long long)M * N);
    const int m = (int)(r / N), n = (int)(r % N);
    WT[e] = W[(k * N + n) * M + m];
  }
}

hipError_t qce_launch_sparse_f64(long long B, int N, int M, int K, const double2* y, const double* w, const double2* W,
                                 const double2* bvec, double2* WT, bool transpose, double2* h, hipStream_t st) {
  if (N > 256 || M > 256) return hipErrorInvalidValue;
  if (transpose) {
    long long blocks = ((long long)K * N * M + 255) / 256;
    blocks = blocks > 16384 ? 16384 : blocks;
    hipLaunchKernelGGL(k_transpose_w, dim3((unsigned)blocks), dim3(256), 0, st, K, N, M, W, WT);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_est_sparse_f64, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, M, K, y, w, WT, bvec, h);
  return hipGetLastError();
}
