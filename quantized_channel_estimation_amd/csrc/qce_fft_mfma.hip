// MFMA Fourier-domain 'all' / K-shard-partial estimate for (block-)circulant mixtures with A = I
// (the per-bin algebra is derived in qce_fft.hip's header).
//
// Per estimate (zero mean): Y = DFT(y); lp_k = c'_k - sum_i |Y_i|^2 rinv_ik; gamma = softmax(lp);
// f_i = sum_k gamma_k w_ki; h = IDFT(Y . f (+ sum_k gamma_k bb_ki)).  The two K x N products are the
// whole of the arithmetic (4 K N flops per estimate) and run here on v_mfma_f64_16x16x4_f64, so the
// result keeps the FP64 accuracy of the reference (gmm_cplx_bussgang.py computes in complex128).
//
// Kernels (dispatch in launch_mfma_out; QCE_FFT_CHUNK=0 at prepare time keeps the round-2 pair):
//   k_fft_wreg   N = 64: persistent one-wave tiles, register transform (pass 1 / LDS exchange / pass 2); <HM> means
//   k_fft_chunk  zero-mean N = 128, 256: components split over the waves for lp / softmax, bins for the filter,
//                two barriers per 128-component chunk; register transform for N = 256
//   k_fft_chunk_hm  N = 128, 256 with means: k_fft_chunk's split, spectra kept in the LDS tile, 3x the MFMAs
//   k_fft_wave   N = 16, 32 (wave-local LDS transform; N = 64 with QCE_FFT_CHUNK=0)
//   k_fft_mfma   N = 128, 256 with QCE_FFT_CHUNK=0 (the round-2 kernel, described next)
// On gfx950 FP64 VALU instructions and FP64 MFMAs share the SIMD's issue budget (tools/probe/f64_pipe_probe.hip),
// so the newer kernels are organised around fewer VALU instructions per MFMA.
//
// k_fft_mfma: workgroup = 4 waves and TS = 4096 / N observations (64 for N <= 64): the tile of spectra (TS x N
// complex128 = 64 KB) sits in LDS for the transforms, two workgroups per CU.  Wave w owns 16 observations
// (MFMA columns) and a range of NB = min(N, 64) bins, whose spectra (and |Y|^2) it keeps in registers through
// the component loop: for N > 64 the KW = N / 64 waves of one observation group split the bins and add their
// partial log-probabilities through LDS in a fixed order (every wave sees bit-identical lp), double-buffered in
// the then unused spectra tile with one barrier per block, the next block's lp MFMAs in flight behind the
// exchange and softmax of the current one.  Components stream in blocks of 16 (MFMA rows) with an online softmax:
//   lp block   D[comp][obs]  = sum_bins (-rinv)[bin][comp] * |Y|^2[bin][obs]       (A: table, B: LDS)
//   filter     F[bin][obs]  += w[comp][bin] * e^{lp - m}[comp][obs]                (B: the lp tile as is)
// The f64 D layout (row = lane/16 + 4 r, col = lane % 16) is exactly the B-operand layout of k-step r
// (k = lane / 16), so the softmax weights feed the filter product with no data movement.
//
// FFTs: radix-2 DIF in LDS grouped into radix-8/4/2 register passes (natural order in, per-axis
// bit-reversed order out), the inverse is the exact reverse (DIT, conjugate twiddles), so no
// bit-reversal pass exists: the per-bin tables are stored in that bit-reversed order (k_fft_pack).
#include "qce_common.h"
#include "qce_kernels.h"

// 1: pass-1 twiddles from the conflict-free lane table (pass1_lane_tw); 0: from the 128-entry table (A/B builds)
#ifndef QCE_FFT_LANE_TW
#define QCE_FFT_LANE_TW 1
#endif

namespace {

constexpr double SQH = 0.70710678118654752440;  // sqrt(1/2)

QCE_DEV int brev(int j, int lg) { return lg == 0 ? 0 : (int)(__brev((unsigned)j) >> (32 - lg)); }

// v * e^{-2 pi i mm / P} (INV: e^{+...}); P in {2, 4, 8}, mm < P / 2 (compile-time after unrolling)
template <bool INV>
QCE_DEV double2 rootmul(double2 v, int P, int mm) {
  if (mm == 0) return v;
  if (P == 4 || mm == 2) return INV ? make_double2(-v.y, v.x) : make_double2(v.y, -v.x);
  if (mm == 1)
    return INV ? make_double2((v.x - v.y) * SQH, (v.x + v.y) * SQH) : make_double2((v.x + v.y) * SQH, (v.y - v.x) * SQH);
  return INV ? make_double2((-v.x - v.y) * SQH, (v.x - v.y) * SQH) : make_double2((v.y - v.x) * SQH, (-v.x - v.y) * SQH);
}

// One register pass of RL radix-2 stages over every line of one axis of every observation row.
// Axis length L = 2^lgL, element stride st (1: the n2 axis, n2: the n1 axis), first half-distance
// D = 2^lgD (axis units).  A group holds R = 2^RL elements a_m = blk 2D + j + m E (E = 2D / R).
// Forward (DIF): stage s pairs (m, m + R/2^{s+1}) with twiddle W_{2D_s}^{j + (m mod half) E}.
// Inverse (DIT): the same stages in reverse order, conjugate twiddles.
template <int RL, bool INV>
QCE_DEV void fft_pass(double2* T, int lgTS, int RS, int lgN, int lgL, int st, int lgD, const double2* tw, int t0,
                      int nthr) {
  constexpr int R = 1 << RL;
  const int lgE = lgD + 1 - RL;
  const int lgnb = lgL - lgD - 1;  // blocks per line
  const int total = 1 << (lgTS + lgN - RL);
  const int TSm = (1 << lgTS) - 1;
  for (int it = t0; it < total; it += nthr) {
    const int s = it & TSm, q = it >> lgTS;
    const int j = q & ((1 << lgE) - 1), rest = q >> lgE;
    const int blk = rest & ((1 << lgnb) - 1), line = rest >> lgnb;
    double2* row = T + s * RS;
    int idx[R];
    double2 x[R];
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const int a = (blk << (lgD + 1)) + j + (m << lgE);
      idx[m] = (st == 1) ? (line << lgL) + a : a * st + line;
      x[m] = row[idx[m]];
    }
    double2 w[RL];
#pragma unroll
    for (int sI = 0; sI < RL; ++sI) {  // W_{2 D_s}^j = tw[j * 128 / D_s]
      w[sI] = tw[j << (7 - (lgD - sI))];
      if (INV) w[sI].y = -w[sI].y;
    }
    if (!INV) {
#pragma unroll
      for (int sI = 0; sI < RL; ++sI) {
        const int half = R >> (sI + 1);
#pragma unroll
        for (int m = 0; m < R; ++m) {
          if (m & half) continue;
          const double2 a = x[m], b = x[m + half];
          x[m] = cadd(a, b);
          x[m + half] = rootmul<false>(cmul(csub(a, b), w[sI]), 2 * half, m & (half - 1));
        }
      }
    } else {
#pragma unroll
      for (int sI = RL - 1; sI >= 0; --sI) {
        const int half = R >> (sI + 1);
#pragma unroll
        for (int m = 0; m < R; ++m) {
          if (m & half) continue;
          const double2 a = x[m];
          const double2 b = rootmul<true>(cmul(x[m + half], w[sI]), 2 * half, m & (half - 1));
          x[m] = cadd(a, b);
          x[m + half] = csub(a, b);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < R; ++m) row[idx[m]] = x[m];
  }
}

// Orders one wave's LDS accesses without a workgroup barrier: a wave's LDS instructions complete in
// issue order, so a compiler fence around the wave barrier is all the wave-local FFT passes need.
QCE_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// WAVE: the passes run over one wave's own tile (64 lanes, wave-local ordering); otherwise over the
// workgroup's tile (256 threads, __syncthreads between passes)
template <bool INV, bool WAVE = false>
QCE_DEV void fft_axis_passes(double2* T, int lgTS, int RS, int lgN, int lgL, int st, const double2* tw) {
  const int t0 = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x, nthr = WAVE ? 64 : 256;
  // forward: half-distances L/2 .. 1 in groups of <= 3 stages; inverse: the same passes reversed
  int rl[3], dd[3], np = 0;
  for (int rem = lgL, lgD = lgL - 1; rem > 0;) {
    const int r = rem < 3 ? rem : 3;
    rl[np] = r;
    dd[np] = lgD;
    ++np;
    lgD -= r;
    rem -= r;
  }
  for (int i = 0; i < np; ++i) {
    const int p = INV ? np - 1 - i : i;
    if (rl[p] == 3) fft_pass<3, INV>(T, lgTS, RS, lgN, lgL, st, dd[p], tw, t0, nthr);
    else if (rl[p] == 2) fft_pass<2, INV>(T, lgTS, RS, lgN, lgL, st, dd[p], tw, t0, nthr);
    else fft_pass<1, INV>(T, lgTS, RS, lgN, lgL, st, dd[p], tw, t0, nthr);
    if (WAVE) wave_lds_sync();
    else __syncthreads();
  }
}

// Diagnostic build only (-DQCE_STAMPS): per-wave cycle sums of k_fft_wave's / k_fft_mfma's segments (s_memtime) into
// g_fft_stamps (qce_debug_fft_stamps); the product kernel executes no stamp.
#ifdef QCE_STAMPS
__device__ unsigned long long* g_fft_stamps = nullptr;
#define FW_STAMP_DECL unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = __builtin_amdgcn_s_memtime();
#define FW_STAMP(i)                                             \
  do {                                                          \
    __builtin_amdgcn_sched_barrier(0);                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          \
    st_acc[(i)] += t_ - st_prev;                                \
    st_prev = t_;                                               \
    __builtin_amdgcn_sched_barrier(0);                          \
  } while (0)
#define FW_STAMP_FLUSH                                                                                  \
  if (g_fft_stamps && lane == 0 && blockIdx.x < 4096)                                                  \
    for (int i_ = 0; i_ < 8; ++i_) g_fft_stamps[((long long)blockIdx.x * 4 + wid) * 8 + i_] = st_acc[i_];
#else
#define FW_STAMP_DECL
#define FW_STAMP(i)
#define FW_STAMP_FLUSH
#endif

template <int N, int OUT, bool has_mean>
__global__ __launch_bounds__(256, has_mean ? 1 : 2) void k_fft_mfma(long long B, int lg1, int lg2, int Kp,
                                                     const double2* __restrict__ y, const double* __restrict__ pr,
                                                     const double* __restrict__ pur, const double* __restrict__ pui,
                                                     const double* __restrict__ pc, const double* __restrict__ pw,
                                                     const double* __restrict__ pbr, const double* __restrict__ pbi,
                                                     double2* __restrict__ h, double* __restrict__ om,
                                                     double* __restrict__ os, float* __restrict__ oa) {
  constexpr int KW = N >= 64 ? N / 64 : 1;  // waves splitting the bins of one observation group
  constexpr int SG = 4 / KW;                // observation groups (of 16) per workgroup
  constexpr int TS = 16 * SG;
  constexpr int NB = N / KW;  // bins per wave
  constexpr int NT = NB / 16;
  constexpr int RS = N + 1;  // padded row: consecutive rows start 4 banks apart
  constexpr int lgN = __builtin_ctz(N), lgTS = __builtin_ctz(TS);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);
  double2* T = tw + 128;
  const int tid = threadIdx.x;
  const long long b0 = (long long)blockIdx.x * TS;
  const int rows = (int)((B - b0) < TS ? (B - b0) : TS);
  FW_STAMP_DECL

  for (int t = tid; t < 128; t += 256) {
    double sn, cs;
    sincospi(-(double)t / 128.0, &sn, &cs);
    tw[t] = make_double2(cs, sn);
  }
  {  // all TS N / 256 loads per thread in flight at once: rows past the batch end read a clamped (valid)
     // row and are stored as 0
    static_assert(TS * N % 256 == 0, "tile");
    constexpr int NL = TS * N / 256;
    const double2* yt = y + b0 * N;
    double2 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i, r = e >> lgN;
      v[i] = yt[(r < rows ? r : rows - 1) * N + (e & (N - 1))];
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i, r = e >> lgN;
      T[r * RS + (e & (N - 1))] = (r < rows) ? v[i] : make_double2(0.0, 0.0);
    }
  }
  __syncthreads();
  FW_STAMP(0);
  const int n1 = 1 << lg1, n2 = 1 << lg2;
  fft_axis_passes<false>(T, lgTS, RS, lgN, lg2, 1, tw);
  if (lg1 > 0) fft_axis_passes<false>(T, lgTS, RS, lgN, lg1, n2, tw);
  FW_STAMP(1);

  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int sg = wid % SG, kw = wid / SG;
  const int col = lane & 15, hq = lane >> 4;
  const int srow = sg * 16 + col;
  double2* Trow = T + srow * RS;
  const int bin0 = kw * NB;
  // The lane's spectrum values stay in registers for the whole component loop: bins bin0 + 4 u + hq (u < NB / 4)
  // are the lp product's B operand of k-step u and, as u = 4 t + r, the filter accumulator's row hq + 4 r of
  // tile t -- so the spectra tile is free during the loop and carries the lp exchange (double-buffered).
  constexpr int NU = NB / 4;
  double2 yv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) yv[u] = Trow[bin0 + 4 * u + hq];
  constexpr int NTM = has_mean ? NT : 1;
  f64x4 F[NT], Br[NTM], Bi[NTM];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    for (int r = 0; r < 4; ++r) F[t][r] = 0.0;
#pragma unroll
  for (int t = 0; t < NTM; ++t)
    for (int r = 0; r < 4; ++r) Br[t][r] = Bi[t][r] = 0.0;
  double m = -__builtin_inf(), ssum = 0.0;
  const int ncb = Kp >> 4;
  // Table operands come straight from L2 with one block of prefetch distance: the lp operands of block cb + 2 are
  // issued in iteration cb (consumed by the lp MFMAs of cb + 2, which run in iteration cb + 1), the filter
  // operands of block cb at the top of iteration cb (consumed after the exchange and softmax).
  auto load_lp = [&](int cb, double (&a)[NU]) {
    const double* pa = pr + (long long)(bin0 + hq) * Kp + (cb << 4) + col;
#pragma unroll
    for (int u = 0; u < NU; ++u) a[u] = pa[(long long)4 * u * Kp];
  };
  // lp partial of component block cb over this wave's bins: D[comp][obs] = c'_comp (wave 0) - sum |Y|^2 rinv
  // (+ 2 Re conj(Y) u with means)
  auto lp_partial = [&](int cb, const double (&a)[NU]) -> f64x4 {
    const int c0 = cb << 4;
    f64x4 C;
#pragma unroll
    for (int r = 0; r < 4; ++r) C[r] = (kw == 0) ? pc[c0 + hq + 4 * r] : 0.0;
#pragma unroll
    for (int u = 0; u < NU; ++u) C = mfma16x16x4d(a[u], yv[u].x * yv[u].x + yv[u].y * yv[u].y, C);
    if constexpr (has_mean) {
      const long long o = (long long)(bin0 + hq) * Kp + c0 + col;
      const double *qa = pur + o, *qb = pui + o;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        C = mfma16x16x4d(qa[(long long)4 * u * Kp], yv[u].x, C);
        C = mfma16x16x4d(qb[(long long)4 * u * Kp], yv[u].y, C);
      }
    }
    return C;
  };
  double* X = reinterpret_cast<double*>(T);  // [2][SG][KW][4][64] lp partials, aliasing the spectra tile
  auto xslot = [&](int buf, int q) -> double* { return X + (((buf * SG + sg) * KW + q) * 256); };
  double la[NU];
  load_lp(0, la);
  __syncthreads();  // every wave holds its spectra: the tile may now carry the exchange
  f64x4 Cn = lp_partial(0, la);
  if (ncb > 1) load_lp(1, la);
  FW_STAMP(2);
  if constexpr (KW > 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) xslot(0, kw)[r * 64 + lane] = Cn[r];
  }
  for (int cb = 0; cb < ncb; ++cb) {
    const int c0 = cb << 4;
    f64x4 C = Cn;
    if constexpr (KW > 1) __syncthreads();  // block cb's partials are in X[cb & 1]; X[(cb + 1) & 1] is free
    double wv[4][NT];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < NT; ++t) wv[r][t] = pw[(long long)(c0 + hq + 4 * r) * N + bin0 + col + 16 * t];
    if (cb + 1 < ncb) {
      Cn = lp_partial(cb + 1, la);  // MFMAs in flight behind the exchange and softmax of block cb
      if (cb + 2 < ncb) load_lp(cb + 2, la);
    }
    if constexpr (KW > 1) {  // add the KW bin-range partials of this observation group, fixed order
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double acc = xslot(cb & 1, 0)[r * 64 + lane];
#pragma unroll
        for (int q = 1; q < KW; ++q) acc += xslot(cb & 1, q)[r * 64 + lane];
        C[r] = acc;
      }
    }
    // online softmax over this block of 16 components (rows hq + 4 r of the tile, all 4 lane groups)
    double bm = fmax(fmax(C[0], C[1]), fmax(C[2], C[3]));
    bm = fmax(bm, __shfl_xor(bm, 16));
    bm = fmax(bm, __shfl_xor(bm, 32));
    const double mn = fmax(m, bm);
    double e[4], alpha = 1.0;
    if (mn == -__builtin_inf()) {
      e[0] = e[1] = e[2] = e[3] = 0.0;
    } else {
      alpha = exp(m - mn);
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = exp(C[r] - mn);
    }
    double ls = (e[0] + e[1]) + (e[2] + e[3]);
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    ssum = ssum * alpha + ls;
    m = mn;
#pragma unroll
    for (int t = 0; t < NT; ++t) F[t] *= alpha;
    if constexpr (has_mean) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        Br[t] *= alpha;
        Bi[t] *= alpha;
      }
    }
    // filter: F[bin][obs] += w[comp][bin] e[comp][obs] (the lp D layout is the B layout of k-step r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int t = 0; t < NT; ++t) F[t] = mfma16x16x4d(wv[r][t], e[r], F[t]);
      if constexpr (has_mean) {
        const long long o = (long long)(c0 + hq + 4 * r) * N + bin0 + col;
        const double *ba = pbr + o, *bb = pbi + o;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          Br[t] = mfma16x16x4d(ba[16 * t], e[r], Br[t]);
          Bi[t] = mfma16x16x4d(bb[16 * t], e[r], Bi[t]);
        }
      }
    }
    if constexpr (KW > 1) {
      if (cb + 1 < ncb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) xslot((cb + 1) & 1, kw)[r * 64 + lane] = Cn[r];
      }
    }
  }
  FW_STAMP(3);
  if constexpr (KW > 1) __syncthreads();  // every wave is done with the exchange: the tile takes Z
  // Z = Y f + bb (each (observation, bin) of the tile belongs to exactly one lane)
  const double sc = (OUT == 0) ? 1.0 / ssum : 1.0;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = 4 * t + r;
      const int bin = bin0 + 4 * u + hq;
      const double2 v = yv[u];
      const double f = F[t][r] * sc;
      if constexpr (has_mean)
        Trow[bin] = make_double2(fma(v.x, f, Br[t][r] * sc), fma(v.y, f, Bi[t][r] * sc));
      else
        Trow[bin] = make_double2(v.x * f, v.y * f);
    }
  if ((OUT == 3 || OUT == 4) && kw == 0 && hq == 0 && srow < rows) {
    om[b0 + srow] = m;
    os[b0 + srow] = ssum;
  }
  FW_STAMP(4);
  __syncthreads();
  if (lg1 > 0) fft_axis_passes<true>(T, lgTS, RS, lgN, lg1, n2, tw);
  fft_axis_passes<true>(T, lgTS, RS, lgN, lg2, 1, tw);
  (void)n1;
  FW_STAMP(5);
  if (OUT == 3) {
    float2* at = reinterpret_cast<float2*>(oa) + b0 * N;
#pragma unroll 4
    for (int e = tid; e < rows * N; e += 256) {
      const double2 v = T[(e >> lgN) * RS + (e & (N - 1))];
      at[e] = make_float2((float)v.x, (float)v.y);
    }
  } else if (OUT == 4) {  // FP64 accumulator of the K-shard partial (qce_estimate_partial_f64)
    double2* at = reinterpret_cast<double2*>(oa) + b0 * N;
#pragma unroll 4
    for (int e = tid; e < rows * N; e += 256) at[e] = T[(e >> lgN) * RS + (e & (N - 1))];
  } else if (rows == TS) {  // whole tile: all LDS reads issued before the unguarded stores
    double2* ht = h + b0 * N;
    constexpr int NL = TS * N / 256;
    double2 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i;
      v[i] = T[(e >> lgN) * RS + (e & (N - 1))];
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) ht[tid + 256 * i] = v[i];
  } else {
    double2* ht = h + b0 * N;
#pragma unroll 4
    for (int e = tid; e < rows * N; e += 256) ht[e] = T[(e >> lgN) * RS + (e & (N - 1))];
  }
  FW_STAMP(6);
  FW_STAMP_FLUSH
}

// Reductions over the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48) on the gfx950 cross-row
// swaps (no LDS round trip): op(swap pair) = op(x[l], x[l^16]) in either operand order, so every row of a
// column gets bit-identical results.
QCE_DEV void row_pair(double v, bool r32, double& a, double& b) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  if (r32) {
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = __hiloint2double(ph[0], pl[0]);
    b = __hiloint2double(ph[1], pl[1]);
  } else {
    const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = __hiloint2double(ph[0], pl[0]);
    b = __hiloint2double(ph[1], pl[1]);
  }
}
QCE_DEV double col_max4(double v) {
  double a, b;
  row_pair(v, false, a, b);
  row_pair(fmax(a, b), true, a, b);
  return fmax(a, b);
}
QCE_DEV double col_sum4(double v) {
  double a, b;
  row_pair(v, false, a, b);
  row_pair(a + b, true, a, b);
  return a + b;
}

// N <= 64: one wave owns 16 observations end to end (load, FFT, both products, IFFT, store) with no
// workgroup barrier after the twiddle table; waves loop over 16-observation tiles (persistent grid of
// two workgroups per CU, 8 waves per CU).  The spectra stay in the wave's LDS tile through the component
// loop, |Y|^2 in registers.  Tables are in fragment order (k_fft_pack): a lane's operands for two
// consecutive MFMAs are one 16-byte load, and block cb+1's operands are fetched while block cb computes.
//   lp  table: [cb][t/2][lane][t&1] = -rinv[bin 4t + lane/16][comp 16cb + lane%16]       t < N/4
//   filter   : [cb][j/2][lane][j&1] = w[comp 16cb + lane/16 + 4r][bin 16t + lane%16]     j = r NT + t
// CIRC: one axis (n1 = 1, circulant), FFT passes resolved at compile time
template <int N, int OUT, bool HM, bool CIRC>
__global__ __launch_bounds__(256, HM ? 1 : 2) void k_fft_wave(long long B, long long ntiles, int lg1, int lg2, int Kp,
                                                     const double2* __restrict__ y, const double* __restrict__ pr,
                                                     const double* __restrict__ pur, const double* __restrict__ pui,
                                                     const double* __restrict__ pc, const double* __restrict__ pw,
                                                     const double* __restrict__ pbr, const double* __restrict__ pbi,
                                                     double2* __restrict__ h, double* __restrict__ om,
                                                     double* __restrict__ os, float* __restrict__ oa) {
  constexpr int NT = N / 16;  // 16-bin tiles of the filter product
  constexpr int NK = N / 4;   // k-steps of the lp product
  constexpr int NL = NK / 2;  // 16-byte lp operand loads per block
  constexpr int NW = 2 * NT;  // 16-byte filter operand loads per block
  constexpr int RS = N + 1;
  constexpr int lgN = __builtin_ctz(N);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  double2* T = tw + 128 + wid * (16 * RS);
  for (int t = tid; t < 128; t += 256) {
    double sn, cs;
    sincospi(-(double)t / 128.0, &sn, &cs);
    tw[t] = make_double2(cs, sn);
  }
  __syncthreads();
  const int col = lane & 15, hq = lane >> 4;
  double2* Trow = T + col * RS;
  const int ncb = Kp >> 4;
  const double2* PR = reinterpret_cast<const double2*>(pr) + lane;
  const double2* PW = reinterpret_cast<const double2*>(pw) + lane;
  FW_STAMP_DECL
  // Main phase: whole rounds of tiles, one wave per tile.  The remainder (fewer tiles than waves: the last,
  // partial round at large B, every tile at small B) is worked by the four waves of a workgroup together,
  // each on every fourth component block, with the partial (m, s, F) merged through LDS (zero-mean models)
  const long long W = (long long)gridDim.x * 4;
  const long long nmain = HM ? ntiles : (ntiles / W) * W;
  // y of the wave's next tile is fetched into registers behind the component loop of the current one
  // (N/4 16-byte loads in flight, latency hidden by the filter epilogue, inverse FFT and store); rows
  // past the batch end read a clamped (valid) row and are stored as 0
  double2 v[N / 4];
  auto load_y = [&](long long t) __attribute__((always_inline)) {
    const long long bb = t * 16;
    const int rr = (int)((B - bb) < 16 ? (B - bb) : 16);
    const double2* yt = y + bb * N;
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const int e = lane + 64 * i, r = e >> lgN;
      v[i] = yt[(r < rr ? r : rr - 1) * N + (e & (N - 1))];
    }
  };
  constexpr bool PREF = !HM;  // the mean terms' accumulators leave no registers for the prefetch
  // one tile: component blocks s0, s0 + bs, ...; next >= 0: prefetch that tile's y (main phase);
  // coop: the workgroup's four waves share the tile (bs = 4), wave 0 merges and writes
  auto run_tile = [&](long long tile, int s0, int bs, long long next, bool coop) __attribute__((always_inline)) {
    const long long b0 = tile * 16;
    const int rows = (int)((B - b0) < 16 ? (B - b0) : 16);
    if (!PREF || coop) load_y(tile);
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const int e = lane + 64 * i, r = e >> lgN;
      T[r * RS + (e & (N - 1))] = (r < rows) ? v[i] : make_double2(0.0, 0.0);
    }
    wave_lds_sync();
    FW_STAMP(0);
    if constexpr (CIRC) {
      fft_axis_passes<false, true>(T, 4, RS, lgN, lgN, 1, tw);  // compile-time passes and indices
    } else {
      fft_axis_passes<false, true>(T, 4, RS, lgN, lg2, 1, tw);
      if (lg1 > 0) fft_axis_passes<false, true>(T, 4, RS, lgN, lg1, 1 << lg2, tw);
    }
    FW_STAMP(1);
    // |Y|^2 (the lp B operand) is re-derived from the spectra in LDS per block instead of held in 2 N / 4
    // registers: those registers carry the next tile's y instead
    auto y2 = [&](int t) {
      const double2 q = Trow[4 * t + hq];
      return q.x * q.x + q.y * q.y;
    };
    f64x4 F[NT], Br[HM ? NT : 1], Bi[HM ? NT : 1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      for (int r = 0; r < 4; ++r) F[t][r] = 0.0;
    if constexpr (HM) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        for (int r = 0; r < 4; ++r) Br[t][r] = Bi[t][r] = 0.0;
    }
    double m = -__builtin_inf(), ssum = 0.0;
    // Software pipeline over component blocks: iteration j issues the lp MFMAs of block j+1 (independent
    // of block j's softmax VALU, so the two overlap), then block j's softmax and filter MFMAs.
    auto lp_block = [&](int cb, const double2* ta, const double* pcv) {
      f64x4 C;
#pragma unroll
      for (int r = 0; r < 4; ++r) C[r] = pcv[r];
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        C = mfma16x16x4d(ta[i].x, y2(2 * i), C);
        C = mfma16x16x4d(ta[i].y, y2(2 * i + 1), C);
      }
      if constexpr (HM) {
        const double2* qa = reinterpret_cast<const double2*>(pur) + lane + cb * NL * 64;
        const double2* qb = reinterpret_cast<const double2*>(pui) + lane + cb * NL * 64;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const double2 ua = qa[i * 64], ub = qb[i * 64];
          const double2 v0 = Trow[8 * i + hq], v1 = Trow[8 * i + 4 + hq];
          C = mfma16x16x4d(ua.x, v0.x, C);
          C = mfma16x16x4d(ub.x, v0.y, C);
          C = mfma16x16x4d(ua.y, v1.x, C);
          C = mfma16x16x4d(ub.y, v1.y, C);
        }
      }
      return C;
    };
    // online softmax over one block of 16 components (rows hq + 4 r, all four lane groups of a column);
    // branch-free: an all -inf prefix gives alpha = e = 0 through the 0 shift
    auto softmax = [&](const f64x4& C, double* e) {
      const double bm = col_max4(fmax(fmax(C[0], C[1]), fmax(C[2], C[3])));
      const double mn = fmax(m, bm);
      const double sh = (mn == -__builtin_inf()) ? 0.0 : mn;
      const double alpha = exp(m - sh);
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = exp(C[r] - sh);
      const double ls = col_sum4((e[0] + e[1]) + (e[2] + e[3]));
      ssum = ssum * alpha + ls;
      m = mn;
      return alpha;
    };
    auto filter_block = [&](int cb, const double2* tb, const double* e, double alpha) {
#pragma unroll
      for (int t = 0; t < NT; ++t) F[t] *= alpha;
#pragma unroll
      for (int j = 0; j < 4 * NT; ++j) {
        const int r = j / NT, t = j % NT;
        const double wv = (j & 1) ? tb[j >> 1].y : tb[j >> 1].x;
        F[t] = mfma16x16x4d(wv, e[r], F[t]);
      }
      if constexpr (HM) {
        const double2* qa = reinterpret_cast<const double2*>(pbr) + lane + cb * NW * 64;
        const double2* qb = reinterpret_cast<const double2*>(pbi) + lane + cb * NW * 64;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          Br[t] *= alpha;
          Bi[t] *= alpha;
        }
#pragma unroll
        for (int j = 0; j < 4 * NT; ++j) {
          const int r = j / NT, t = j % NT;
          const double2 ua = qa[(j >> 1) * 64], ub = qb[(j >> 1) * 64];
          Br[t] = mfma16x16x4d((j & 1) ? ua.y : ua.x, e[r], Br[t]);
          Bi[t] = mfma16x16x4d((j & 1) ? ub.y : ub.x, e[r], Bi[t]);
        }
      }
    };
    const int nb = (ncb - s0 + bs - 1) / bs;  // this wave's component blocks s0 + j bs, j < nb
    auto blk = [&](int j) { return s0 + j * bs; };
    if (nb > 0) {
      const int last = nb - 1;
      double2 ta[NL], tb[NW];
      double pcv[4];
#pragma unroll
      for (int i = 0; i < NL; ++i) ta[i] = PR[(blk(0) * NL + i) * 64];
#pragma unroll
      for (int r = 0; r < 4; ++r) pcv[r] = pc[16 * blk(0) + hq + 4 * r];
      f64x4 C = lp_block(blk(0), ta, pcv);
      {
        const int b1 = blk(last > 0 ? 1 : 0);
#pragma unroll
        for (int i = 0; i < NL; ++i) ta[i] = PR[(b1 * NL + i) * 64];
#pragma unroll
        for (int r = 0; r < 4; ++r) pcv[r] = pc[16 * b1 + hq + 4 * r];
#pragma unroll
        for (int i = 0; i < NW; ++i) tb[i] = PW[(blk(0) * NW + i) * 64];
      }
      FW_STAMP(2);
      // operand registers are refilled right after the MFMAs that read them: lp operands of block j+2
      // behind the lp MFMAs of j+1, filter operands of j+1 behind the filter MFMAs of j
      for (int j = 0; j < last; ++j) {
        const int b1 = blk(j + 1), b2 = blk(j + 2 < last ? j + 2 : last);
        const f64x4 Cn = lp_block(b1, ta, pcv);
#pragma unroll
        for (int i = 0; i < NL; ++i) ta[i] = PR[(b2 * NL + i) * 64];
#pragma unroll
        for (int r = 0; r < 4; ++r) pcv[r] = pc[16 * b2 + hq + 4 * r];
        double e[4];
        const double alpha = softmax(C, e);
        filter_block(blk(j), tb, e, alpha);
#pragma unroll
        for (int i = 0; i < NW; ++i) tb[i] = PW[(b1 * NW + i) * 64];
        C = Cn;
      }
      FW_STAMP(3);
      if (PREF && next >= 0) {
        load_y(next);
      } else {  // define v on every path, so the consumed values are dead through the component loop
#pragma unroll
        for (int i = 0; i < N / 4; ++i) v[i] = make_double2(0.0, 0.0);
      }
      {
        double e[4];
        const double alpha = softmax(C, e);
        filter_block(blk(last), tb, e, alpha);
      }
    }
    if (coop) {  // waves 1-3 hand (F, m, s) to wave 0 through their own (now free) spectra tiles
      double* Td = reinterpret_cast<double*>(T);
      if (wid != 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) Td[(t * 4 + r) * 64 + lane] = F[t][r];
        Td[4 * NT * 64 + lane] = m;
        Td[(4 * NT + 1) * 64 + lane] = ssum;
      }
      __syncthreads();
      if (wid == 0) {  // fixed order: wave 0's own partial, then waves 1, 2, 3
        double mm = m;
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const double* Tw = reinterpret_cast<const double*>(tw + 128 + w * (16 * RS));
          mm = fmax(mm, Tw[4 * NT * 64 + lane]);
        }
        const double f0 = exp(m - mm);
        ssum *= f0;
#pragma unroll
        for (int t = 0; t < NT; ++t) F[t] *= f0;
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const double* Tw = reinterpret_cast<const double*>(tw + 128 + w * (16 * RS));
          const double mw = Tw[4 * NT * 64 + lane];
          const double fw = (mw == -__builtin_inf()) ? 0.0 : exp(mw - mm);
          ssum = fma(Tw[(4 * NT + 1) * 64 + lane], fw, ssum);
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) F[t][r] = fma(Tw[(t * 4 + r) * 64 + lane], fw, F[t][r]);
        }
        m = mm;
      }
    }
    if (!coop || wid == 0) {
      // Z = Y f + bb in place (each (observation, bin) of the tile belongs to exactly one lane)
      const double sc = (OUT == 0) ? 1.0 / ssum : 1.0;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int bin = 16 * t + hq + 4 * r;
          const double2 q = Trow[bin];
          const double f = F[t][r] * sc;
          if constexpr (HM)
            Trow[bin] = make_double2(fma(q.x, f, Br[t][r] * sc), fma(q.y, f, Bi[t][r] * sc));
          else
            Trow[bin] = make_double2(q.x * f, q.y * f);
        }
      if ((OUT == 3 || OUT == 4) && hq == 0 && col < rows) {
        om[b0 + col] = m;
        os[b0 + col] = ssum;
      }
      FW_STAMP(4);
      wave_lds_sync();
      if constexpr (CIRC) {
        fft_axis_passes<true, true>(T, 4, RS, lgN, lgN, 1, tw);
      } else {
        if (lg1 > 0) fft_axis_passes<true, true>(T, 4, RS, lgN, lg1, 1 << lg2, tw);
        fft_axis_passes<true, true>(T, 4, RS, lgN, lg2, 1, tw);
      }
      FW_STAMP(5);
      if (OUT == 3) {
        float2* at = reinterpret_cast<float2*>(oa) + b0 * N;
#pragma unroll
        for (int i = 0; i < N / 4; ++i) {
          const int e = lane + 64 * i, r = e >> lgN;
          if (r < rows) {
            const double2 q = T[r * RS + (e & (N - 1))];
            at[e] = make_float2((float)q.x, (float)q.y);
          }
        }
      } else if (OUT == 4) {
        double2* at = reinterpret_cast<double2*>(oa) + b0 * N;
#pragma unroll
        for (int i = 0; i < N / 4; ++i) {
          const int e = lane + 64 * i, r = e >> lgN;
          if (r < rows) at[e] = T[r * RS + (e & (N - 1))];
        }
      } else {
        double2* ht = h + b0 * N;
        if (rows == 16) {  // whole tile: no per-element guard, all LDS reads issued before the stores
#pragma unroll
          for (int i = 0; i < N / 4; ++i) {
            const int e = lane + 64 * i;
            ht[e] = T[(e >> lgN) * RS + (e & (N - 1))];
          }
        } else {
#pragma unroll
          for (int i = 0; i < N / 4; ++i) {
            const int e = lane + 64 * i, r = e >> lgN;
            if (r < rows) ht[e] = T[r * RS + (e & (N - 1))];
          }
        }
      }
    }
    if (coop) __syncthreads();  // wave 0 has read the partials before the next tile overwrites them
    FW_STAMP(6);
    wave_lds_sync();
  };
  long long tile = (long long)blockIdx.x * 4 + wid;
  if (PREF && tile < nmain) load_y(tile);
  for (; tile < nmain; tile += W) run_tile(tile, 0, 1, tile + W < nmain ? tile + W : -1, false);
  for (long long tt = nmain + blockIdx.x; tt < ntiles; tt += gridDim.x) run_tile(tt, wid, 4, -1, true);
  FW_STAMP_FLUSH
}

// Buffer-resource memory access: a wave-uniform descriptor (base, byte extent) in scalar registers plus a 32-bit
// per-lane offset, so no 64-bit per-lane addresses occupy vector registers; loads past the extent return 0 and
// stores past it are dropped (the ragged last tile needs no guards).
typedef unsigned int qce_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int qce_u32x2 __attribute__((ext_vector_type(2)));
QCE_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
QCE_DEV double2 buf_ld2(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
QCE_DEV double buf_ld1(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
QCE_DEV void buf_st2(double2 v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(qce_u32x4, v), r, voff, soff, 0);
}
QCE_DEV void buf_st1f2(float2 v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(qce_u32x2, v), r, voff, soff, 0);
}

// e^x for x <= 700 (x = -inf and x < -708 give e^-708 = 3e-308, negligible beside the largest weight 1, which every
// use has): 2^(k/32) from a 32-entry LDS
// table (exp2_tab, 2^(j/32)) times the degree-6 Taylor polynomial of e^r, |r| <= ln2/64 (truncation 4e-18), 2^(k>>5)
// added to the exponent field: 18 VALU against ~32 for the libm exp, about 2 ulp.
QCE_DEV double exp_nonpos(double x, const double* __restrict__ tab) {
  constexpr double L32 = 46.166241308446828384;      // 32 / ln 2
  constexpr double LH = 2.1660849390173098072e-02;   // ln 2 / 32, leading bits
  constexpr double LL = 2.3251928468788740148e-12;   // ln 2 / 32 - LH
  x = fmax(x, -708.0);  // -inf and deep underflow -> e^-708 (3e-308, negligible beside the largest weight 1)
  const double kf = __builtin_rint(x * L32);
  double r = fma(kf, -LH, x);
  r = fma(kf, -LL, r);
  const int k = (int)kf;
  double p = fma(r, 1.0 / 720.0, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const double v = tab[k & 31] * p;
  return __hiloint2double(__double2hiint(v) + ((k >> 5) << 20), __double2loint(v));
}
QCE_DEV void exp2_tab_init(double* tab, int tid) {
  if (tid < 32) tab[tid] = exp2((double)tid / 32.0);
}

// ---- register-resident transform of 16 points per thread (N = 256 in two passes of four radix-2 stages) ----
// v * e^{-2 pi i mm / 16} (INV: e^{+...}), mm < 8 compile-time after unrolling
template <bool INV>
QCE_DEV double2 rootmul16(double2 v, int mm) {
  if (!(mm & 1)) return rootmul<INV>(v, 8, mm >> 1);
  constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173;  // cos, sin (pi / 8)
  const double c = (mm == 1) ? C1 : (mm == 3) ? S1 : (mm == 5) ? -S1 : -C1;
  const double s = (mm == 1) ? S1 : (mm == 3) ? C1 : (mm == 5) ? C1 : S1;  // sin(2 pi mm / 16)
  return INV ? make_double2(v.x * c - v.y * s, v.x * s + v.y * c) : make_double2(v.x * c + v.y * s, v.y * c - v.x * s);
}
template <bool INV>
QCE_DEV double2 root_any(double2 v, int P, int mm) {
  return P == 16 ? rootmul16<INV>(v, mm) : rootmul<INV>(v, P, mm);
}

// Radix-2^RL group on the registers x[S m], m < 2^RL: the stages of one contiguous bit range of one axis, first
// half-distance 2^lgD (axis units), j = the axis position bits below the range (the group twiddle W_{2D_s}^j;
// JZ: j == 0 for every thread).  Forward: DIF stages, inverse: the same stages reversed (DIT), conjugate twiddles --
// the arithmetic of fft_pass with all R elements in one thread.
// LT: tw is a pass-1 lane table (pass1_lane_tw) and j the lane's g: stage sI's twiddle is tw[16 sI + g].
template <int RL, bool INV, int S, bool JZ, bool LT = false>
QCE_DEV void reg_group(double2* x, int lgD, int j, const double2* tw) {
  constexpr int R = 1 << RL;
  double2 w[RL];
  if constexpr (!JZ) {
#pragma unroll
    for (int sI = 0; sI < RL; ++sI) {
      w[sI] = LT ? tw[16 * sI + j] : tw[j << (7 - (lgD - sI))];
      if (INV) w[sI].y = -w[sI].y;
    }
  }
  if constexpr (!INV) {
#pragma unroll
    for (int sI = 0; sI < RL; ++sI) {
      const int half = R >> (sI + 1);
#pragma unroll
      for (int m = 0; m < R; ++m) {
        if (m & half) continue;
        const double2 a = x[S * m], b = x[S * (m + half)];
        x[S * m] = cadd(a, b);
        double2 d = csub(a, b);
        if constexpr (!JZ) d = cmul(d, w[sI]);
        x[S * (m + half)] = root_any<false>(d, 2 * half, m & (half - 1));
      }
    }
  } else {
#pragma unroll
    for (int sI = RL - 1; sI >= 0; --sI) {
      const int half = R >> (sI + 1);
#pragma unroll
      for (int m = 0; m < R; ++m) {
        if (m & half) continue;
        const double2 a = x[S * m];
        double2 b = x[S * (m + half)];
        if constexpr (!JZ) b = cmul(b, w[sI]);
        b = root_any<true>(b, 2 * half, m & (half - 1));
        x[S * m] = cadd(a, b);
        x[S * (m + half)] = csub(a, b);
      }
    }
  }
}

// One pass over a thread's 2^RT points (array index = RT bits of the storage position): array bits [0, RA) are
// axis n2 (segment A), [RA, RT) axis n1 (segment B).  The axes are independent, so the segments run in either order.
template <int RT, int RA, bool INV, bool JZA, bool JZB, bool LT = false>
QCE_DEV void reg_pass(double2* x, int lgDA, int jA, int lgDB, int jB, const double2* tw) {
  constexpr int RB = RT - RA;
  if constexpr (RB > 0) {
#pragma unroll
    for (int a = 0; a < (1 << RA); ++a) reg_group<RB, INV, (1 << RA), JZB, LT>(x + a, lgDB, jB, tw);
  }
  if constexpr (RA > 0) {
#pragma unroll
    for (int b = 0; b < (1 << RB); ++b) reg_group<RA, INV, 1, JZA, LT>(x + (b << RA), lgDA, jA, tw);
  }
}
template <int RA, bool INV, bool JZA, bool JZB, bool LT = false>
QCE_DEV void reg_pass16(double2 (&x)[16], int lgDA, int jA, int lgDB, int jB, const double2* tw) {
  reg_pass<4, RA, INV, JZA, JZB, LT>(x, lgDA, jA, lgDB, jB, tw);
}

// Pass-1 lane twiddle table (64 double2): entry 16 sI + g = the stage-sI group twiddle of the lanes whose pass-1
// points have low bits g.  Pass 1 reads tw[j << (7 - (lgD - sI))] with j = g (or g >> lg2): the 16 lanes of a
// ds_read_b128 group (distinct g) land on only 2-8 of the 128-entry table's bank quads (4- to 8-way conflicts,
// a quarter of the Fourier kernels' LDS cycles); the lane table puts them on 16 consecutive 16-byte slots.  The
// entries are computed like tw (same sincospi of the same index), so both forms are bit-identical.  The non-JZ
// segment of pass 1 is n2 bits [4, lg2) (j = g, lgD = lg2 - 1) for lg2 > 4, else n1 bits [4, lgN) (j = g >> lg2,
// lgD = lgN - 1 - lg2); threads 0-63 fill it.
QCE_DEV void pass1_lane_tw(double2* tl, int lgN, int lg2, int tid) {
  if (tid >= 64) return;
  const int sI = tid >> 4, g = tid & 15;
  const int RL = lg2 > 4 ? lg2 - 4 : (lg2 == 4 ? 0 : lgN - 4);
  const int lgD = lg2 > 4 ? lg2 - 1 : lgN - 1 - lg2;
  const int j = lg2 > 4 ? g : (g >> lg2);
  double sn = 0.0, cs = 1.0;
  if (sI < RL) sincospi(-(double)(j << (7 - (lgD - sI))) / 128.0, &sn, &cs);
  tl[tid] = make_double2(cs, sn);
}

// N = 64 = n1 n2: pass 1 = storage bits 5, 4 on a group of 4 points sharing the bits 0-3 (g); segment A = n2 bits
// [4, min(lg2, 6)), B = n1 bits [max(lg2, 4), 6), j = the axis bits below the segment
// LT: tw is the pass-1 lane table (pass1_lane_tw with lgN = 6)
template <bool INV, bool LT = false>
QCE_DEV void fft64_pass1(double2* x, int lg2, int g, const double2* tw) {
  switch (lg2) {
    case 6: reg_pass<2, 2, INV, false, true, LT>(x, 5, g, 0, 0, tw); break;
    case 5: reg_pass<2, 1, INV, false, true, LT>(x, 4, g, 0, 0, tw); break;
    case 4: reg_pass<2, 0, INV, true, true, LT>(x, 0, 0, 1, 0, tw); break;
    default: reg_pass<2, 0, INV, true, false, LT>(x, 0, 0, 5 - lg2, LT ? g : g >> lg2, tw); break;
  }
}

// N = 256 = n1 n2 (lg2 = log2 n2): the forward transform's stages in descending storage bit order are bits 7..4
// (pass 1) and 3..0 (pass 2) -- per axis high bits before low bits, as DIF requires.  Pass 1: the thread's points
// share the storage bits 0-3 (g), pass 2 the bits 4-7.
template <bool INV, bool LT = false>  // LT: tw is the pass-1 lane table (pass1_lane_tw with lgN = 8)
QCE_DEV void fft256_pass1(double2 (&x)[16], int lg2, int g, const double2* tw) {
  switch (lg2) {  // segment A = n2 bits [4, lg2), B = n1 bits [max(lg2, 4), 8)
    case 8: reg_pass16<4, INV, false, true, LT>(x, 7, g, 0, 0, tw); break;
    case 7: reg_pass16<3, INV, false, true, LT>(x, 6, g, 0, 0, tw); break;
    case 6: reg_pass16<2, INV, false, true, LT>(x, 5, g, 1, 0, tw); break;
    case 5: reg_pass16<1, INV, false, true, LT>(x, 4, g, 2, 0, tw); break;
    case 4: reg_pass16<0, INV, true, true, LT>(x, 0, 0, 3, 0, tw); break;
    default:  // n1 bits 4-7, j = n1 bits < 4
      reg_pass16<0, INV, true, false, LT>(x, 0, 0, 7 - lg2, LT ? g : g >> lg2, tw);
      break;
  }
}
// pass 2 of every N >= 16 split: storage bits 3..0 of a lane's 16 points (bits >= 4 fixed)
template <bool INV>
QCE_DEV void fft_pass_low4(double2 (&x)[16], int lg2, const double2* tw) {
  switch (lg2 >= 4 ? 4 : lg2) {  // segment A = n2 bits [0, min(lg2, 4)), B = n1 bits [lg2, 4)
    case 4: reg_pass16<4, INV, true, true>(x, 3, 0, 0, 0, tw); break;
    case 3: reg_pass16<3, INV, true, true>(x, 2, 0, 0, 0, tw); break;
    case 2: reg_pass16<2, INV, true, true>(x, 1, 0, 1, 0, tw); break;
    case 1: reg_pass16<1, INV, true, true>(x, 0, 0, 2, 0, tw); break;
    default: reg_pass16<0, INV, true, true>(x, 0, 0, 3, 0, tw); break;
  }
}

// Filter-phase bin of k_fft_chunk<256>: wave w = t / 4 owns the storage positions with bits 4-7 = hq + 4 w, its tile
// t % 4 and accumulator register r (row hq + 4 r) give bits 0-3 = r + 4 (t % 4) -- exactly the 16 points a lane
// holds after pass 2, so the spectra and Z never pass through LDS between the transforms and the filter.
QCE_DEV int chunk256_bin(int t, int row) { return (((row & 3) + 4 * (t >> 2)) << 4) | ((row >> 2) + 4 * (t & 3)); }

// Zero-mean models, N = 64 (cfg3): k_fft_wave's persistent one-wave-per-tile schedule with the transform in registers.
// Pass 1 (storage bits 5, 4) runs on the prefetched y (lane: observations s0 + 4 q, positions g + 16 j), one
// wave-local LDS exchange, pass 2 (bits 3..0) leaves lane (hq, col) holding positions 16 hq + i of observation col.
// The tables are ordered so those 16 points are the lane's own operands: lp k-step u, k-index hq = position
// 16 hq + u (the B operand |Y|^2 comes from registers, computed once per tile), filter tile t, row hq + 4 r =
// position 16 hq + r + 4 t (chunk256_bin).  The spectra wait in the lane's own slots of the wave tile during the
// component loop; Z, inverse pass 2, the exchange and inverse pass 1 run the same way back, stores from registers.
// HM (models with means, gmm_cplx_bussgang.py:96-100, :256-264, :288): lp k-step u adds 2 Re(Y_u^* u_k,u) as two more
// MFMAs on the lane's own spectra (Re Y, Im Y of position 16 hq + u; a second accumulator), the filter two more
// accumulator sets (Re b, Im b) at the filter positions, Z = Y f + b: 3x the MFMAs, one wave per SIMD (512
// registers) and a larger per-wave LDS slot for the tail's partial exchange.
template <int OUT, bool HM>
__global__ __launch_bounds__(256, HM ? 1 : 2) void k_fft_wreg(long long B, long long ntiles, int lg2, int Kp,
                                                              const double2* __restrict__ y,
                                                              const double* __restrict__ pr,
                                                              const double* __restrict__ pur,
                                                              const double* __restrict__ pui,
                                                              const double* __restrict__ pc,
                                                              const double* __restrict__ pw,
                                                              const double* __restrict__ pbr,
                                                              const double* __restrict__ pbi,
                                                              double2* __restrict__ h, double* __restrict__ om,
                                                              double* __restrict__ os, float* __restrict__ oa) {
  constexpr int N = 64, NT = 4, NL = 8, NW = 8, RS = N + 1;
  constexpr int WS = HM ? 1664 : 16 * RS;  // double2 per wave slot: the tile, or the tail's (F, Br, Bi, m, s) rows
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  double* etab = reinterpret_cast<double*>(tw + 128);  // 2^(j/32), j < 32
  double2* tl = tw + 144;                               // pass-1 lane twiddles
  double2* T = tw + 208 + wid * WS;
  for (int t = tid; t < 128; t += 256) {
    double sn, cs;
    sincospi(-(double)t / 128.0, &sn, &cs);
    tw[t] = make_double2(cs, sn);
  }
  exp2_tab_init(etab, tid);
  pass1_lane_tw(tl, 6, lg2, tid);
  __syncthreads();
  const int col = lane & 15, hq = lane >> 4;
  const int g1 = lane & 15, s0 = lane >> 4;  // pass-1 lane: observations s0 + 4 q, positions g1 + 16 j
  double2* Town = T + col * RS + 16 * hq;    // the lane's pass-2 points
  const int ncb = Kp >> 4;
  // tables, y and h through buffer descriptors (scalar registers); per-lane 32-bit offsets
  const __amdgpu_buffer_rsrc_t rpr = buf_rsrc(pr, (unsigned)(Kp * N * 8)), rpw = buf_rsrc(pw, (unsigned)(Kp * N * 8));
  const __amdgpu_buffer_rsrc_t rpc = buf_rsrc(pc, (unsigned)(Kp * 8));
  const __amdgpu_buffer_rsrc_t rur = buf_rsrc(pur, HM ? (unsigned)(Kp * N * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rui = buf_rsrc(pui, HM ? (unsigned)(Kp * N * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rbr = buf_rsrc(pbr, HM ? (unsigned)(Kp * N * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rbi = buf_rsrc(pbi, HM ? (unsigned)(Kp * N * 8) : 0u);
  const unsigned ul16 = (unsigned)lane * 16;
  const unsigned yo = (unsigned)(s0 * N + g1) * 16;  // pass-1 lane: byte offset of (s0, g1) in a tile
  FW_STAMP_DECL
  const long long W = (long long)gridDim.x * 4;
  const long long nmain = (ntiles / W) * W;
  double2 v[16];  // y of a tile in the pass-1 layout: v[4 q + j] = y[s0 + 4 q][g1 + 16 j]
  auto load_y = [&](long long t) __attribute__((always_inline)) {
    const long long bb = t * 16;
    const int rr = (int)((B - bb) < 16 ? (B - bb) : 16);
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(y + bb * N, (unsigned)(rr * N * 16));  // rows past B read 0
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * q + j] = buf_ld2(ry, yo + 256 * j, 4096 * q);
  };
  auto run_tile = [&](long long tile, int s0b, int bs, long long next, bool coop) __attribute__((always_inline)) {
    const long long b0 = tile * 16;
    const int rows = (int)((B - b0) < 16 ? (B - b0) : 16);
    if (coop) load_y(tile);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      fft64_pass1<false, QCE_FFT_LANE_TW>(v + 4 * q, lg2, g1, QCE_FFT_LANE_TW ? tl : tw);
#pragma unroll
      for (int j = 0; j < 4; ++j) T[(s0 + 4 * q) * RS + g1 + 16 * j] = v[4 * q + j];
    }
    wave_lds_sync();
    FW_STAMP(0);
    {
      double2 yv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) yv[i] = Town[i];
      fft_pass_low4<false>(yv, lg2, tw);
#pragma unroll
      for (int i = 0; i < 16; ++i) Town[i] = yv[i];  // the lane's own slots: no other lane reads them
    }
    // |Y|^2 of lp k-step u is the lane's own point u, re-derived from the spectra per use (two VALU per k-step keep
    // 32 registers free for the next tile's y)
    auto y2 = [&](int u, unsigned o) {
      const double2 q = Town[u + o];
      return q.x * q.x + q.y * q.y;
    };
    FW_STAMP(1);
    f64x4 F[NT], Br[HM ? NT : 1], Bi[HM ? NT : 1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      for (int r = 0; r < 4; ++r) F[t][r] = 0.0;
    if constexpr (HM) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        for (int r = 0; r < 4; ++r) Br[t][r] = Bi[t][r] = 0.0;
    }
    double m = -__builtin_inf(), ssum = 0.0;
    // c'_comp is added after the MFMAs, so its loads have the whole product to land
    // HM: the mean tables of a block are loaded at its start and consumed after its |Y|^2 (lp) or w (filter) MFMAs,
    // which cover their latency; only the r / w tables are prefetched a block ahead (register budget)
    auto lp_block = [&](int cb, const double2* ta) {
      double pcv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) pcv[r] = buf_ld1(rpc, (unsigned)(hq + 4 * r) * 8, (unsigned)cb * 128);
      f64x4 C;
#pragma unroll
      for (int r = 0; r < 4; ++r) C[r] = 0.0;
      unsigned o = 0;  // opaque zero: the spectra reads stay in the loop instead of being hoisted into registers
      asm volatile("" : "+v"(o));
      double2 ua[HM ? NL : 1], qa[HM ? NL : 1];
      if constexpr (HM) {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          ua[i] = buf_ld2(rur, ul16, (unsigned)cb * NL * 1024 + 1024 * i);
          qa[i] = buf_ld2(rui, ul16, (unsigned)cb * NL * 1024 + 1024 * i);
        }
      }
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        C = mfma16x16x4d(ta[i].x, y2(2 * i, o), C);
        C = mfma16x16x4d(ta[i].y, y2(2 * i + 1, o), C);
      }
      if constexpr (HM) {  // + 2 Re(Y^* u): (2 Re u) Re Y + (2 Im u) Im Y on the lane's own points
        f64x4 D;
#pragma unroll
        for (int r = 0; r < 4; ++r) D[r] = 0.0;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const double2 q0 = Town[2 * i + o], q1 = Town[2 * i + 1 + o];
          D = mfma16x16x4d(ua[i].x, q0.x, D);
          D = mfma16x16x4d(qa[i].x, q0.y, D);
          D = mfma16x16x4d(ua[i].y, q1.x, D);
          D = mfma16x16x4d(qa[i].y, q1.y, D);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) C[r] += D[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) C[r] += pcv[r];
      return C;
    };
    // Softmax with a lagging shift m: the weights are e^(lp - m) with m moved (and F, s rescaled) only when a lane's
    // block maximum exceeds it by more than 32 nats -- weights stay below e^32, and after the first blocks the
    // whole wave skips the rescale (column maximum, one exp, 16 multiplies).  ssum is the lane's own partial sum
    // (its 4 components of each block); the column sum is taken once per tile.
    auto softmax = [&](const f64x4& C, double* e) {
      const double lm = fmax(fmax(C[0], C[1]), fmax(C[2], C[3]));
      if (__builtin_amdgcn_ballot_w64(lm > m + 32.0)) {
        const double bm = col_max4(lm);
        const double mn = (bm > m + 32.0) ? bm : m;  // the column's four lanes agree (same bm, same m)
        const double alpha = exp_nonpos(m - mn, etab);  // 1 where the shift stays, ~0 from -inf
        ssum *= alpha;
#pragma unroll
        for (int t = 0; t < NT; ++t) F[t] *= alpha;
        if constexpr (HM) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            Br[t] *= alpha;
            Bi[t] *= alpha;
          }
        }
        m = mn;
      }
      const double sh = (m == -__builtin_inf()) ? 0.0 : m;
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = exp_nonpos(C[r] - sh, etab);
      ssum += (e[0] + e[1]) + (e[2] + e[3]);
    };
    auto filter_block = [&](const double2* tb, int cb, const double* e) {
      double2 tr[HM ? NW : 1], ti[HM ? NW : 1];
      if constexpr (HM) {
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          tr[i] = buf_ld2(rbr, ul16, (unsigned)cb * NW * 1024 + 1024 * i);
          ti[i] = buf_ld2(rbi, ul16, (unsigned)cb * NW * 1024 + 1024 * i);
        }
      }
#pragma unroll
      for (int j = 0; j < 4 * NT; ++j) {
        const int r = j / NT, t = j % NT;
        const double wv = (j & 1) ? tb[j >> 1].y : tb[j >> 1].x;
        F[t] = mfma16x16x4d(wv, e[r], F[t]);
      }
      if constexpr (HM) {
#pragma unroll
        for (int j = 0; j < 4 * NT; ++j) {
          const int r = j / NT, t = j % NT;
          Br[t] = mfma16x16x4d((j & 1) ? tr[j >> 1].y : tr[j >> 1].x, e[r], Br[t]);
        }
#pragma unroll
        for (int j = 0; j < 4 * NT; ++j) {
          const int r = j / NT, t = j % NT;
          Bi[t] = mfma16x16x4d((j & 1) ? ti[j >> 1].y : ti[j >> 1].x, e[r], Bi[t]);
        }
      }
    };
    const int nb = (ncb - s0b + bs - 1) / bs;  // this wave's component blocks s0b + j bs, j < nb
    auto blk = [&](int j) { return s0b + j * bs; };
    if (nb > 0) {
      const int last = nb - 1;
      double2 ta[NL], tb[NW];
      auto load_lp = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NL; ++i) ta[i] = buf_ld2(rpr, ul16, (unsigned)cb * NL * 1024 + 1024 * i);
      };
      auto load_w = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NW; ++i) tb[i] = buf_ld2(rpw, ul16, (unsigned)cb * NW * 1024 + 1024 * i);
      };
      load_lp(blk(0));
      f64x4 C = lp_block(blk(0), ta);
      load_lp(blk(last > 0 ? 1 : 0));
      load_w(blk(0));
      FW_STAMP(2);
      for (int j = 0; j < last; ++j) {
        const int b1 = blk(j + 1), b2 = blk(j + 2 < last ? j + 2 : last);
        const f64x4 Cn = lp_block(b1, ta);
        load_lp(b2);
        double e[4];
        softmax(C, e);
        filter_block(tb, blk(j), e);
        load_w(b1);
        C = Cn;
      }
      FW_STAMP(3);
      if (next >= 0) load_y(next);  // behind the last block, the merge, the inverse transform and the store
      {
        double e[4];
        softmax(C, e);
        filter_block(tb, blk(last), e);
      }
    }
    ssum = col_sum4(ssum);  // the lanes' partial sums -> the column's (bit-identical in its four lanes)
    if (coop) {  // waves 1-3 hand (F, m, s) to wave 0 through their own tiles (wave 0's holds its spectra)
      double* Td = reinterpret_cast<double*>(T);
      constexpr int NA = HM ? 3 : 1;  // accumulator sets: F (, Br, Bi)
      if (wid != 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            Td[(t * 4 + r) * 64 + lane] = F[t][r];
            if constexpr (HM) {
              Td[(4 * NT + t * 4 + r) * 64 + lane] = Br[t][r];
              Td[(8 * NT + t * 4 + r) * 64 + lane] = Bi[t][r];
            }
          }
        Td[NA * 4 * NT * 64 + lane] = m;
        Td[(NA * 4 * NT + 1) * 64 + lane] = ssum;
      }
      __syncthreads();
      if (wid == 0) {  // fixed order: wave 0's own partial, then waves 1, 2, 3
        double mm = m;
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const double* Tw = reinterpret_cast<const double*>(tw + 208 + w * WS);
          mm = fmax(mm, Tw[NA * 4 * NT * 64 + lane]);
        }
        const double f0 = exp_nonpos(m - mm, etab);
        ssum *= f0;
#pragma unroll
        for (int t = 0; t < NT; ++t) F[t] *= f0;
        if constexpr (HM) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            Br[t] *= f0;
            Bi[t] *= f0;
          }
        }
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const double* Tw = reinterpret_cast<const double*>(tw + 208 + w * WS);
          const double mw = Tw[NA * 4 * NT * 64 + lane];
          const double fw = exp_nonpos(mw - mm, etab);
          ssum = fma(Tw[(NA * 4 * NT + 1) * 64 + lane], fw, ssum);
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              F[t][r] = fma(Tw[(t * 4 + r) * 64 + lane], fw, F[t][r]);
              if constexpr (HM) {
                Br[t][r] = fma(Tw[(4 * NT + t * 4 + r) * 64 + lane], fw, Br[t][r]);
                Bi[t][r] = fma(Tw[(8 * NT + t * 4 + r) * 64 + lane], fw, Bi[t][r]);
              }
            }
        }
        m = mm;
      }
    }
    if (!coop || wid == 0) {
      const double sc = (OUT == 0) ? 1.0 / ssum : 1.0;
      if ((OUT == 3 || OUT == 4) && hq == 0 && col < rows) {
        om[b0 + col] = m;
        os[b0 + col] = ssum;
      }
      double2 z[16];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double2 q = Town[r + 4 * t];
          const double f = F[t][r] * sc;
          if constexpr (HM)
            z[r + 4 * t] = make_double2(fma(q.x, f, Br[t][r] * sc), fma(q.y, f, Bi[t][r] * sc));
          else
            z[r + 4 * t] = make_double2(q.x * f, q.y * f);
        }
      FW_STAMP(4);
      fft_pass_low4<true>(z, lg2, tw);
#pragma unroll
      for (int i = 0; i < 16; ++i) Town[i] = z[i];
      wave_lds_sync();
      const unsigned ob = (unsigned)rows * N * 16;  // rows past B: stores dropped by the descriptor extent
      const __amdgpu_buffer_rsrc_t ro = (OUT == 0) ? buf_rsrc(h + b0 * N, ob)
                                      : (OUT == 3) ? buf_rsrc(reinterpret_cast<float2*>(oa) + b0 * N, ob / 2)
                                                   : buf_rsrc(reinterpret_cast<double2*>(oa) + b0 * N, ob);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double2 x[4];
        const int sr = s0 + 4 * q;
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = T[sr * RS + g1 + 16 * j];
        fft64_pass1<true, QCE_FFT_LANE_TW>(x, lg2, g1, QCE_FFT_LANE_TW ? tl : tw);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (OUT == 3)
            buf_st1f2(make_float2((float)x[j].x, (float)x[j].y), ro, yo / 2 + 128 * j, 2048 * q);
          else
            buf_st2(x[j], ro, yo + 256 * j, 4096 * q);
        }
      }
      FW_STAMP(5);
    }
    if (coop) __syncthreads();  // wave 0 has read the partials before the next tile overwrites them
    wave_lds_sync();
    FW_STAMP(6);
  };
  long long tile = (long long)blockIdx.x * 4 + wid;
  if (tile < nmain) load_y(tile);
  for (; tile < nmain; tile += W) run_tile(tile, 0, 1, tile + W < nmain ? tile + W : -1, false);
  for (long long tt = nmain + blockIdx.x; tt < ntiles; tt += gridDim.x) run_tile(tt, wid, 4, -1, true);
  FW_STAMP_FLUSH
}

// Zero-mean models, N = 128, 256: one workgroup (4 waves) per 16 observations, the components split over the waves
// for the log-probabilities and the bins split over the waves for the filter, so the softmax of every (component,
// observation) is evaluated exactly once and the waves meet at two barriers per chunk of 128 components (not per
// block of 16).  Per chunk:
//   lp    wave w: blocks w, w + 4 of the chunk over all N bins: D[comp][obs] = c'_comp + sum_bins (-rinv) |Y|^2
//         (A: fragment-order table from L2, B: |Y|^2 from LDS, both blocks share each B read)
//   max   per-wave column max -> LDS, barrier, every wave takes the chunk max (fixed order) and the running max
//   e     e = exp(lp - m) of the wave's own 32 components -> LDS (the filter's B layout), column sums -> LDS, barrier
//   F     wave w: its N/4 bins over the chunk's 128 components: F[bin][obs] = alpha F + w[comp][bin] e[comp][obs]
// Layout: the spectra tile T (16 x (N+1) complex) carries the y load and the forward FFT; the lane's filter-phase
// spectra (bins bin0 + 16 t + hq + 4 r) move to registers and the tile is reused for |Y|^2 (in the lp B layout),
// e and the per-wave column maxima / sums; after the last chunk it takes Z = Y f for the inverse FFT.
template <int N>
struct FftChunkLds {
  static constexpr int TS = 16, RS = N + 1;
  static constexpr size_t tile = (size_t)TS * RS * 16;
  static constexpr size_t y2 = (size_t)N * TS * 8, e = (size_t)128 * TS * 8, sm = (size_t)2 * 4 * TS * 8;
  static constexpr size_t body = tile > y2 + e + sm ? tile : y2 + e + sm;
  static constexpr size_t bytes = 128 * 16 + body + 32 * 8 + 64 * 16;  // + the exp table, the pass-1 lane twiddles
};

template <int N, int OUT>
__global__ __launch_bounds__(256, 2) void k_fft_chunk(long long B, int lg1, int lg2, int Kp,
                                                      const double2* __restrict__ y, const double* __restrict__ pr,
                                                      const double* __restrict__ pc, const double* __restrict__ pw,
                                                      double2* __restrict__ h, double* __restrict__ om,
                                                      double* __restrict__ os, float* __restrict__ oa) {
  constexpr int TS = 16, RS = N + 1, lgTS = 4;
  constexpr int lgN = __builtin_ctz(N);
  constexpr int NB = N / 4;    // bins per wave in the filter product
  constexpr int NTW = NB / 16;  // the wave's 16-bin filter tiles
  constexpr int NTF = N / 16;   // 16-bin tiles of the whole filter table
  constexpr int NL = N / 8;     // 16-byte lp operand loads per block (two k-steps each)
  constexpr int NWF = N / 8;    // 16-byte filter operand loads per block
  constexpr int CB = 8;         // component blocks per chunk (two per wave)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);
  double2* T = tw + 128;
  double2* Y2 = T;                                                 // [N/8][4][16] (k-steps 2i, 2i+1 of the lp B)
  double2* E = reinterpret_cast<double2*>(reinterpret_cast<double*>(T) + N * TS);  // [CB * 2][4][16]
  double* SM = reinterpret_cast<double*>(E + CB * 2 * 64);         // [2][4][16] column maxima, column sums
  double* etab = reinterpret_cast<double*>(smem) + 2 * 128 + FftChunkLds<N>::body / 8;  // 2^(j/32), after the body
  double2* tl = reinterpret_cast<double2*>(etab + 32);                                  // pass-1 lane twiddles (N = 256)
  const int tid = threadIdx.x;
  const long long b0 = (long long)blockIdx.x * TS;
  const int rows = (int)((B - b0) < TS ? (B - b0) : TS);
  FW_STAMP_DECL

  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, hq = lane >> 4;
  const int bin0 = wid * NB;
  double2 yv[NTW * 4];  // the lane's filter-phase spectra (tile t, accumulator row hq + 4 r: yv[4 t + r])
  if constexpr (N == 256) {
    // pass 1 straight from HBM: thread (s = tid / 16, g = tid % 16) holds positions g + 16 i of observation s (each
    // i a 256-byte contiguous run over 16 lanes); pass 2 thread (wave w, hq, col) the positions 16 (hq + 4 w) + i of
    // observation col, which stay in registers as yv
    const int s1 = tid >> 4, g = tid & 15;
    {
      const double2* yr = y + (b0 + (s1 < rows ? s1 : rows - 1)) * N + g;
      double2 x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = yr[16 * i];
      for (int t = tid; t < 128; t += 256) {
        double sn, cs;
        sincospi(-(double)t / 128.0, &sn, &cs);
        tw[t] = make_double2(cs, sn);
      }
      exp2_tab_init(etab, tid);
      pass1_lane_tw(tl, 8, lg2, tid);
      __syncthreads();
      FW_STAMP(0);
      if (s1 >= rows) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = make_double2(0.0, 0.0);
      }
      fft256_pass1<false, QCE_FFT_LANE_TW>(x, lg2, g, QCE_FFT_LANE_TW ? tl : tw);
#pragma unroll
      for (int i = 0; i < 16; ++i) T[s1 * RS + g + 16 * i] = x[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) yv[i] = T[col * RS + 16 * (hq + 4 * wid) + i];
    fft_pass_low4<false>(yv, lg2, tw);
    FW_STAMP(1);
    __syncthreads();  // every spectrum value is in registers: the tile takes |Y|^2, e and the column statistics
    // |Y|^2 in the lp B layout (k-step u = p / 4 covers p = 4 u + hq'): position 16 (hq + 4 w) + r + 4 t is k-step
    // u = 4 (hq + 4 w) + t, row hq' = r; the pair (t even, t odd) is one 16-byte slot
#pragma unroll
    for (int tp = 0; tp < 2; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 a = yv[r + 8 * tp], b = yv[r + 8 * tp + 4];
        Y2[((2 * (hq + 4 * wid) + tp) * 4 + r) * 16 + col] =
            make_double2(a.x * a.x + a.y * a.y, b.x * b.x + b.y * b.y);
      }
    __syncthreads();
  } else {
    for (int t = tid; t < 128; t += 256) {
      double sn, cs;
      sincospi(-(double)t / 128.0, &sn, &cs);
      tw[t] = make_double2(cs, sn);
    }
    exp2_tab_init(etab, tid);
    {  // all loads in flight at once; rows past the batch end read a clamped (valid) row and are stored as 0
      constexpr int NLY = TS * N / 256;
      const double2* yt = y + b0 * N;
      double2 v[NLY];
#pragma unroll
      for (int i = 0; i < NLY; ++i) {
        const int e = tid + 256 * i, r = e >> lgN;
        v[i] = yt[(r < rows ? r : rows - 1) * N + (e & (N - 1))];
      }
#pragma unroll
      for (int i = 0; i < NLY; ++i) {
        const int e = tid + 256 * i, r = e >> lgN;
        T[r * RS + (e & (N - 1))] = (r < rows) ? v[i] : make_double2(0.0, 0.0);
      }
    }
    __syncthreads();
    FW_STAMP(0);
    fft_axis_passes<false>(T, lgTS, RS, lgN, lg2, 1, tw);
    if (lg1 > 0) fft_axis_passes<false>(T, lgTS, RS, lgN, lg1, 1 << lg2, tw);
    FW_STAMP(1);
    // bin bin0 + 16 t + hq + 4 r, observation col
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) yv[4 * t + r] = T[col * RS + bin0 + 16 * t + hq + 4 * r];
    {  // |Y|^2 in the lp B layout: pair (k-step 2i, 2i + 1) of lane (hq, col) = bins 8 i + hq, 8 i + 4 + hq
      constexpr int NP = N * TS / 2 / 256;
      double2 q[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int p = tid + 256 * j, s = p & 15, rest = p >> 4;
        const int bq = 8 * (rest >> 2) + (rest & 3);
        const double2 a = T[s * RS + bq], b = T[s * RS + bq + 4];
        q[j] = make_double2(a.x * a.x + a.y * a.y, b.x * b.x + b.y * b.y);
      }
      __syncthreads();  // every spectrum value is in registers: the tile takes |Y|^2, e and the column statistics
#pragma unroll
      for (int j = 0; j < NP; ++j) Y2[tid + 256 * j] = q[j];  // index = (i * 4 + hq) * 16 + s
      __syncthreads();
    }
  }
  FW_STAMP(2);

  f64x4 F[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    for (int r = 0; r < 4; ++r) F[t][r] = 0.0;
  double m = -__builtin_inf(), ssum = 0.0;
  const int ncb = Kp >> 4;
  // tables through buffer descriptors: scalar block offsets, one 32-bit lane offset (no 64-bit address math)
  const __amdgpu_buffer_rsrc_t rpr = buf_rsrc(pr, (unsigned)(Kp * N * 8)), rpw = buf_rsrc(pw, (unsigned)(Kp * N * 8));
  const unsigned ul16 = (unsigned)lane * 16;
  const double2* Y2l = Y2 + hq * 16 + col;
  for (int c0 = 0; c0 < ncb; c0 += CB) {
    const int cb0 = c0 + wid, cb1 = cb0 + 4;
    const bool v0 = cb0 < ncb, v1 = cb1 < ncb;  // wave-uniform
    f64x4 C0, C1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      C0[r] = v0 ? pc[16 * cb0 + hq + 4 * r] : -__builtin_inf();
      C1[r] = v1 ? pc[16 * cb1 + hq + 4 * r] : -__builtin_inf();
    }
    if (v1) {
      const unsigned o0 = (unsigned)cb0 * NL * 1024, o1 = (unsigned)cb1 * NL * 1024;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const double2 a0 = buf_ld2(rpr, ul16, o0 + 1024 * i), a1 = buf_ld2(rpr, ul16, o1 + 1024 * i), b = Y2l[i * 64];
        C0 = mfma16x16x4d(a0.x, b.x, C0);
        C1 = mfma16x16x4d(a1.x, b.x, C1);
        C0 = mfma16x16x4d(a0.y, b.y, C0);
        C1 = mfma16x16x4d(a1.y, b.y, C1);
      }
    } else if (v0) {
      const unsigned o0 = (unsigned)cb0 * NL * 1024;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const double2 a0 = buf_ld2(rpr, ul16, o0 + 1024 * i), b = Y2l[i * 64];
        C0 = mfma16x16x4d(a0.x, b.x, C0);
        C0 = mfma16x16x4d(a0.y, b.y, C0);
      }
    }
    FW_STAMP(3);
    // chunk maximum per observation: per-wave column maxima, then all four in a fixed order
    const double lm = col_max4(fmax(fmax(fmax(C0[0], C0[1]), fmax(C0[2], C0[3])),
                                    fmax(fmax(C1[0], C1[1]), fmax(C1[2], C1[3]))));
    if (hq == 0) SM[wid * 16 + col] = lm;
    __syncthreads();
    const double mn = fmax(fmax(m, fmax(SM[col], SM[16 + col])), fmax(SM[32 + col], SM[48 + col]));
    const double sh = (mn == -__builtin_inf()) ? 0.0 : mn;
    const double alpha = exp_nonpos(m - sh, etab);
    // e of the wave's own components, in the filter's B layout: k-step ks = 4 (local block) + r covers the
    // components 4 ks + hq; pair (ks even, ks + 1) per 16-byte slot
    double ls = 0.0;
    {
      double e[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = v0 ? exp_nonpos(C0[r] - sh, etab) : 0.0;
      ls += (e[0] + e[1]) + (e[2] + e[3]);
      E[((2 * wid) * 4 + hq) * 16 + col] = make_double2(e[0], e[1]);
      E[((2 * wid + 1) * 4 + hq) * 16 + col] = make_double2(e[2], e[3]);
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = v1 ? exp_nonpos(C1[r] - sh, etab) : 0.0;
      ls += (e[0] + e[1]) + (e[2] + e[3]);
      E[((2 * (wid + 4)) * 4 + hq) * 16 + col] = make_double2(e[0], e[1]);
      E[((2 * (wid + 4) + 1) * 4 + hq) * 16 + col] = make_double2(e[2], e[3]);
    }
    ls = col_sum4(ls);
    if (hq == 0) SM[64 + wid * 16 + col] = ls;
    __syncthreads();
    ssum = ssum * alpha + ((SM[64 + col] + SM[80 + col]) + (SM[96 + col] + SM[112 + col]));
    m = mn;
    FW_STAMP(4);
#pragma unroll
    for (int t = 0; t < NTW; ++t) F[t] *= alpha;
    // filter over the chunk's blocks (padding blocks beyond ncb carry e = 0 and are skipped)
    // the operands of block bl + 1 are fetched while block bl computes; the CB blocks are unrolled (guards are
    // wave-uniform), so the two operand buffers alternate without register copies
    const int nbl = (ncb - c0) < CB ? (ncb - c0) : CB;
    constexpr int NWL = 2 * NTW;  // 16-byte filter operand loads per block and wave: (r, tile pair tp)
    const unsigned wbase = (unsigned)c0 * NWF * 1024 + (unsigned)((wid * NTW) >> 1) * 1024;
    auto load_w = [&](int bl, double2 (&wv)[NWL]) {
      const unsigned ob = wbase + (unsigned)bl * NWF * 1024;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int tp = 0; tp < NTW / 2; ++tp)
          wv[r * (NTW / 2) + tp] = buf_ld2(rpw, ul16, ob + ((r * NTF) >> 1) * 1024 + tp * 1024);
    };
    auto filter_blk = [&](int bl, const double2 (&wc)[NWL]) {
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const double2 ev = E[((2 * bl + rp) * 4 + hq) * 16 + col];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const int r = 2 * rp + rr;
          const double eb = rr ? ev.y : ev.x;
#pragma unroll
          for (int tp = 0; tp < NTW / 2; ++tp) {  // filter table pair (j, j + 1), j = r NTF + t: tiles t, t + 1
            const double2 wv = wc[r * (NTW / 2) + tp];
            F[2 * tp] = mfma16x16x4d(wv.x, eb, F[2 * tp]);
            F[2 * tp + 1] = mfma16x16x4d(wv.y, eb, F[2 * tp + 1]);
          }
        }
      }
    };
    double2 wa[NWL], wb[NWL];
    load_w(0, wa);
#pragma unroll
    for (int bl = 0; bl < CB; bl += 2) {
      if (bl < nbl) {
        if (bl + 1 < nbl) load_w(bl + 1, wb);
        filter_blk(bl, wa);
      }
      if (bl + 1 < nbl) {
        if (bl + 2 < nbl) load_w(bl + 2, wa);
        filter_blk(bl + 1, wb);
      }
    }
    FW_STAMP(5);
  }
  __syncthreads();  // every wave is done with |Y|^2 and e: the tile takes Z
  const double sc = (OUT == 0) ? 1.0 / ssum : 1.0;
  if ((OUT == 3 || OUT == 4) && wid == 0 && hq == 0 && col < rows) {
    om[b0 + col] = m;
    os[b0 + col] = ssum;
  }
  if constexpr (N == 256) {  // inverse pass 2 on the registers, one LDS exchange, inverse pass 1, store from registers
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double f = F[t][r] * sc;
        yv[4 * t + r] = make_double2(yv[4 * t + r].x * f, yv[4 * t + r].y * f);
      }
    fft_pass_low4<true>(yv, lg2, tw);
#pragma unroll
    for (int i = 0; i < 16; ++i) T[col * RS + 16 * (hq + 4 * wid) + i] = yv[i];
    __syncthreads();
    const int s1 = tid >> 4, g = tid & 15;
    double2 x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = T[s1 * RS + g + 16 * i];
    fft256_pass1<true, QCE_FFT_LANE_TW>(x, lg2, g, QCE_FFT_LANE_TW ? tl : tw);
    FW_STAMP(6);
    if (s1 < rows) {
      const long long o = (b0 + s1) * N + g;
      if (OUT == 3) {
        float2* at = reinterpret_cast<float2*>(oa) + o;
#pragma unroll
        for (int i = 0; i < 16; ++i) at[16 * i] = make_float2((float)x[i].x, (float)x[i].y);
      } else if (OUT == 4) {
        double2* at = reinterpret_cast<double2*>(oa) + o;
#pragma unroll
        for (int i = 0; i < 16; ++i) at[16 * i] = x[i];
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) h[o + 16 * i] = x[i];
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 v = yv[4 * t + r];
        const double f = F[t][r] * sc;
        T[col * RS + bin0 + 16 * t + hq + 4 * r] = make_double2(v.x * f, v.y * f);
      }
    __syncthreads();
    if (lg1 > 0) fft_axis_passes<true>(T, lgTS, RS, lgN, lg1, 1 << lg2, tw);
    fft_axis_passes<true>(T, lgTS, RS, lgN, lg2, 1, tw);
    FW_STAMP(6);
    if (OUT == 3) {
      float2* at = reinterpret_cast<float2*>(oa) + b0 * N;
#pragma unroll 4
      for (int e = tid; e < rows * N; e += 256) {
        const double2 v = T[(e >> lgN) * RS + (e & (N - 1))];
        at[e] = make_float2((float)v.x, (float)v.y);
      }
    } else if (OUT == 4) {
      double2* at = reinterpret_cast<double2*>(oa) + b0 * N;
#pragma unroll 4
      for (int e = tid; e < rows * N; e += 256) at[e] = T[(e >> lgN) * RS + (e & (N - 1))];
    } else if (rows == TS) {
      double2* ht = h + b0 * N;
      constexpr int NLY = TS * N / 256;
      double2 v[NLY];
#pragma unroll
      for (int i = 0; i < NLY; ++i) {
        const int e = tid + 256 * i;
        v[i] = T[(e >> lgN) * RS + (e & (N - 1))];
      }
#pragma unroll
      for (int i = 0; i < NLY; ++i) ht[tid + 256 * i] = v[i];
    } else {
      double2* ht = h + b0 * N;
#pragma unroll 4
      for (int e = tid; e < rows * N; e += 256) ht[e] = T[(e >> lgN) * RS + (e & (N - 1))];
    }
  }
  FW_STAMP(7);
  FW_STAMP_FLUSH
}

// Models with means, N = 128, 256 (the reference's fit default zero_mean=False, gmm_cplx_bussgang.py:96-100; the
// means enter at :256-264, :288): k_fft_chunk's split (components over the waves for lp / softmax, bins over the waves
// for the filter, two barriers per chunk of 128 components) with the mean terms of the Fourier-domain formula
//   lp_k = c'_k - sum_i |Y_i|^2 r_ik + 2 sum_i (Re Y_i Re u_ik + Im Y_i Im u_ik)    (u_ik = (mu_y)_ik / r_ik)
//   Z_i  = Y_i f_i + sum_k gamma_k b_ik                                            (f_i = sum_k gamma_k w_ik)
// i.e. two more real MFMAs per lp k-step (B = Re Y, Im Y read from the spectra tile) and two more filter accumulator
// sets (Re b, Im b): 3x the zero-mean MFMA work.  The spectra stay in the LDS tile through the component loop (Z is
// formed from it at the end), so |Y|^2, e and the column statistics get their own LDS (118 KB at N = 256: one
// workgroup per CU, one wave per SIMD with up to 512 registers, the accumulators in AGPRs).  Tables in k_fft_chunk's
// fragment order (k_fft_pack with frag, pur / pui beside pr, pbr / pbi beside pw).
template <int N>
struct FftChunkHmLds {
  static constexpr int TS = 16, RS = N + 1;
  static constexpr size_t tile = (size_t)TS * RS * 16;
  static constexpr size_t y2 = (size_t)N * TS * 8, e = (size_t)128 * TS * 8, sm = (size_t)2 * 4 * TS * 8;
  static constexpr size_t bytes = 128 * 16 + tile + y2 + e + sm + 32 * 8 + 64 * 16;
};

template <int N, int OUT>
__global__ __launch_bounds__(256, 1) void k_fft_chunk_hm(long long B, int lg1, int lg2, int Kp,
                                                         const double2* __restrict__ y, const double* __restrict__ pr,
                                                         const double* __restrict__ pur, const double* __restrict__ pui,
                                                         const double* __restrict__ pc, const double* __restrict__ pw,
                                                         const double* __restrict__ pbr,
                                                         const double* __restrict__ pbi, double2* __restrict__ h,
                                                         double* __restrict__ om, double* __restrict__ os,
                                                         float* __restrict__ oa) {
  using LD = FftChunkHmLds<N>;
  constexpr int TS = 16, RS = N + 1, lgTS = 4;
  constexpr int lgN = __builtin_ctz(N);
  constexpr int NB = N / 4, NTW = NB / 16, NTF = N / 16, NL = N / 8, NWF = N / 8, CB = 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* tw = reinterpret_cast<double2*>(smem);
  double2* T = tw + 128;                                                         // spectra, kept through the loop
  double2* Y2 = reinterpret_cast<double2*>(reinterpret_cast<char*>(T) + LD::tile);  // [N/8][4][16]
  double2* E = reinterpret_cast<double2*>(reinterpret_cast<char*>(Y2) + LD::y2);    // [CB * 2][4][16]
  double* SM = reinterpret_cast<double*>(reinterpret_cast<char*>(E) + LD::e);       // [2][4][16]
  double* etab = reinterpret_cast<double*>(reinterpret_cast<char*>(SM) + LD::sm);  // 2^(j/32)
  double2* tl = reinterpret_cast<double2*>(etab + 32);                              // pass-1 lane twiddles (N = 256)
  const int tid = threadIdx.x;
  const long long b0 = (long long)blockIdx.x * TS;
  const int rows = (int)((B - b0) < TS ? (B - b0) : TS);
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, hq = lane >> 4;
  const int bin0 = wid * NB;
  double2* Trow = T + col * RS;
  // the lane's filter-phase storage position of tile t, accumulator row hq + 4 r
  auto fpos = [&](int t, int r) -> int {
    return N == 256 ? 16 * (hq + 4 * wid) + r + 4 * t : bin0 + 16 * t + hq + 4 * r;
  };
  if constexpr (N == 256) {
    const int s1 = tid >> 4, g = tid & 15;
    const double2* yr = y + (b0 + (s1 < rows ? s1 : rows - 1)) * N + g;
    double2 x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = yr[16 * i];
    for (int t = tid; t < 128; t += 256) {
      double sn, cs;
      sincospi(-(double)t / 128.0, &sn, &cs);
      tw[t] = make_double2(cs, sn);
    }
    exp2_tab_init(etab, tid);
    pass1_lane_tw(tl, 8, lg2, tid);
    __syncthreads();
    if (s1 >= rows) {
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = make_double2(0.0, 0.0);
    }
    fft256_pass1<false, QCE_FFT_LANE_TW>(x, lg2, g, QCE_FFT_LANE_TW ? tl : tw);
#pragma unroll
    for (int i = 0; i < 16; ++i) T[s1 * RS + g + 16 * i] = x[i];
    __syncthreads();
    double2 yv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) yv[i] = Trow[16 * (hq + 4 * wid) + i];
    fft_pass_low4<false>(yv, lg2, tw);
#pragma unroll
    for (int i = 0; i < 16; ++i) Trow[16 * (hq + 4 * wid) + i] = yv[i];  // the lane's own points: no barrier needed
#pragma unroll
    for (int tp = 0; tp < 2; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 a = yv[r + 8 * tp], b = yv[r + 8 * tp + 4];
        Y2[((2 * (hq + 4 * wid) + tp) * 4 + r) * 16 + col] = make_double2(a.x * a.x + a.y * a.y, b.x * b.x + b.y * b.y);
      }
    __syncthreads();
  } else {
    for (int t = tid; t < 128; t += 256) {
      double sn, cs;
      sincospi(-(double)t / 128.0, &sn, &cs);
      tw[t] = make_double2(cs, sn);
    }
    exp2_tab_init(etab, tid);
    {
      constexpr int NLY = TS * N / 256;
      const double2* yt = y + b0 * N;
      double2 v[NLY];
#pragma unroll
      for (int i = 0; i < NLY; ++i) {
        const int e = tid + 256 * i, r = e >> lgN;
        v[i] = yt[(r < rows ? r : rows - 1) * N + (e & (N - 1))];
      }
#pragma unroll
      for (int i = 0; i < NLY; ++i) {
        const int e = tid + 256 * i, r = e >> lgN;
        T[r * RS + (e & (N - 1))] = (r < rows) ? v[i] : make_double2(0.0, 0.0);
      }
    }
    __syncthreads();
    fft_axis_passes<false>(T, lgTS, RS, lgN, lg2, 1, tw);
    if (lg1 > 0) fft_axis_passes<false>(T, lgTS, RS, lgN, lg1, 1 << lg2, tw);
    {
      constexpr int NP = N * TS / 2 / 256;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int p = tid + 256 * j, sI = p & 15, rest = p >> 4;
        const int bq = 8 * (rest >> 2) + (rest & 3);
        const double2 a = T[sI * RS + bq], b = T[sI * RS + bq + 4];
        Y2[tid + 256 * j] = make_double2(a.x * a.x + a.y * a.y, b.x * b.x + b.y * b.y);
      }
    }
    __syncthreads();
  }

  f64x4 F[NTW], Br[NTW], Bi[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    for (int r = 0; r < 4; ++r) F[t][r] = Br[t][r] = Bi[t][r] = 0.0;
  double m = -__builtin_inf(), ssum = 0.0;
  const int ncb = Kp >> 4;
  const unsigned tb = (unsigned)(Kp * N * 8);
  const __amdgpu_buffer_rsrc_t rpr = buf_rsrc(pr, tb), rpw = buf_rsrc(pw, tb);
  const __amdgpu_buffer_rsrc_t rur = buf_rsrc(pur, tb), rui = buf_rsrc(pui, tb);
  const __amdgpu_buffer_rsrc_t rbr = buf_rsrc(pbr, tb), rbi = buf_rsrc(pbi, tb);
  const unsigned ul16 = (unsigned)lane * 16;
  const double2* Y2l = Y2 + hq * 16 + col;
  for (int c0 = 0; c0 < ncb; c0 += CB) {
    const int cb0 = c0 + wid, cb1 = cb0 + 4;
    const bool v0 = cb0 < ncb, v1 = cb1 < ncb;  // wave-uniform
    f64x4 C0, C1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      C0[r] = v0 ? pc[16 * cb0 + hq + 4 * r] : -__builtin_inf();
      C1[r] = v1 ? pc[16 * cb1 + hq + 4 * r] : -__builtin_inf();
    }
    // lp k-steps 2i, 2i + 1, row hq: storage positions 8 i + hq, 8 i + 4 + hq (the Y2 pair, k_fft_pack layouts 0 / 1)
    if (v0) {
      const unsigned o0 = (unsigned)cb0 * NL * 1024, o1 = (unsigned)(v1 ? cb1 : cb0) * NL * 1024;
#pragma unroll 4
      for (int i = 0; i < NL; ++i) {
        const double2 a0 = buf_ld2(rpr, ul16, o0 + 1024 * i), a1 = buf_ld2(rpr, ul16, o1 + 1024 * i);
        const double2 u0 = buf_ld2(rur, ul16, o0 + 1024 * i), u1 = buf_ld2(rur, ul16, o1 + 1024 * i);
        const double2 q0 = buf_ld2(rui, ul16, o0 + 1024 * i), q1 = buf_ld2(rui, ul16, o1 + 1024 * i);
        const double2 b = Y2l[i * 64];
        const double2 ya = Trow[8 * i + hq], yb = Trow[8 * i + 4 + hq];
        C0 = mfma16x16x4d(a0.x, b.x, C0);
        C1 = mfma16x16x4d(a1.x, b.x, C1);
        C0 = mfma16x16x4d(a0.y, b.y, C0);
        C1 = mfma16x16x4d(a1.y, b.y, C1);
        C0 = mfma16x16x4d(u0.x, ya.x, C0);
        C1 = mfma16x16x4d(u1.x, ya.x, C1);
        C0 = mfma16x16x4d(q0.x, ya.y, C0);
        C1 = mfma16x16x4d(q1.x, ya.y, C1);
        C0 = mfma16x16x4d(u0.y, yb.x, C0);
        C1 = mfma16x16x4d(u1.y, yb.x, C1);
        C0 = mfma16x16x4d(q0.y, yb.y, C0);
        C1 = mfma16x16x4d(q1.y, yb.y, C1);
      }
      if (!v1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) C1[r] = -__builtin_inf();
      }
    }
    const double lm = col_max4(fmax(fmax(fmax(C0[0], C0[1]), fmax(C0[2], C0[3])),
                                    fmax(fmax(C1[0], C1[1]), fmax(C1[2], C1[3]))));
    if (hq == 0) SM[wid * 16 + col] = lm;
    __syncthreads();
    const double mn = fmax(fmax(m, fmax(SM[col], SM[16 + col])), fmax(SM[32 + col], SM[48 + col]));
    const double sh = (mn == -__builtin_inf()) ? 0.0 : mn;
    const double alpha = exp_nonpos(m - sh, etab);
    double ls = 0.0;
    {
      double e[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = v0 ? exp_nonpos(C0[r] - sh, etab) : 0.0;
      ls += (e[0] + e[1]) + (e[2] + e[3]);
      E[((2 * wid) * 4 + hq) * 16 + col] = make_double2(e[0], e[1]);
      E[((2 * wid + 1) * 4 + hq) * 16 + col] = make_double2(e[2], e[3]);
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = v1 ? exp_nonpos(C1[r] - sh, etab) : 0.0;
      ls += (e[0] + e[1]) + (e[2] + e[3]);
      E[((2 * (wid + 4)) * 4 + hq) * 16 + col] = make_double2(e[0], e[1]);
      E[((2 * (wid + 4) + 1) * 4 + hq) * 16 + col] = make_double2(e[2], e[3]);
    }
    ls = col_sum4(ls);
    if (hq == 0) SM[64 + wid * 16 + col] = ls;
    __syncthreads();
    ssum = ssum * alpha + ((SM[64 + col] + SM[80 + col]) + (SM[96 + col] + SM[112 + col]));
    m = mn;
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      F[t] *= alpha;
      Br[t] *= alpha;
      Bi[t] *= alpha;
    }
    const int nbl = (ncb - c0) < CB ? (ncb - c0) : CB;
    constexpr int NWL = 2 * NTW;
    const unsigned wbase = (unsigned)c0 * NWF * 1024 + (unsigned)((wid * NTW) >> 1) * 1024;
#pragma unroll 1
    for (int bl = 0; bl < nbl; ++bl) {
      const unsigned ob = wbase + (unsigned)bl * NWF * 1024;
      double2 ww[NWL], wr[NWL], wi[NWL];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int tp = 0; tp < NTW / 2; ++tp) {
          const unsigned o = ob + ((r * NTF) >> 1) * 1024 + tp * 1024;
          ww[r * (NTW / 2) + tp] = buf_ld2(rpw, ul16, o);
          wr[r * (NTW / 2) + tp] = buf_ld2(rbr, ul16, o);
          wi[r * (NTW / 2) + tp] = buf_ld2(rbi, ul16, o);
        }
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const double2 ev = E[((2 * bl + rp) * 4 + hq) * 16 + col];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const int r = 2 * rp + rr;
          const double eb = rr ? ev.y : ev.x;
#pragma unroll
          for (int tp = 0; tp < NTW / 2; ++tp) {
            const int j = r * (NTW / 2) + tp;
            F[2 * tp] = mfma16x16x4d(ww[j].x, eb, F[2 * tp]);
            F[2 * tp + 1] = mfma16x16x4d(ww[j].y, eb, F[2 * tp + 1]);
            Br[2 * tp] = mfma16x16x4d(wr[j].x, eb, Br[2 * tp]);
            Br[2 * tp + 1] = mfma16x16x4d(wr[j].y, eb, Br[2 * tp + 1]);
            Bi[2 * tp] = mfma16x16x4d(wi[j].x, eb, Bi[2 * tp]);
            Bi[2 * tp + 1] = mfma16x16x4d(wi[j].y, eb, Bi[2 * tp + 1]);
          }
        }
      }
    }
  }
  // Z = Y f + b at the lane's filter positions (every (observation, bin) of the tile belongs to exactly one lane)
  const double sc = (OUT == 0) ? 1.0 / ssum : 1.0;
  if ((OUT == 3 || OUT == 4) && wid == 0 && hq == 0 && col < rows) {
    om[b0 + col] = m;
    os[b0 + col] = ssum;
  }
  if constexpr (N == 256) {
    double2 z[16];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 v = Trow[fpos(t, r)];
        const double f = F[t][r] * sc;
        z[4 * t + r] = make_double2(fma(v.x, f, Br[t][r] * sc), fma(v.y, f, Bi[t][r] * sc));
      }
    fft_pass_low4<true>(z, lg2, tw);
#pragma unroll
    for (int i = 0; i < 16; ++i) Trow[16 * (hq + 4 * wid) + i] = z[i];
    __syncthreads();
    const int s1 = tid >> 4, g = tid & 15;
    double2 x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = T[s1 * RS + g + 16 * i];
    fft256_pass1<true, QCE_FFT_LANE_TW>(x, lg2, g, QCE_FFT_LANE_TW ? tl : tw);
    if (s1 < rows) {
      const long long o = (b0 + s1) * N + g;
      if (OUT == 3) {
        float2* at = reinterpret_cast<float2*>(oa) + o;
#pragma unroll
        for (int i = 0; i < 16; ++i) at[16 * i] = make_float2((float)x[i].x, (float)x[i].y);
      } else if (OUT == 4) {
        double2* at = reinterpret_cast<double2*>(oa) + o;
#pragma unroll
        for (int i = 0; i < 16; ++i) at[16 * i] = x[i];
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) h[o + 16 * i] = x[i];
      }
    }
  } else {
    double2 z[4 * NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 v = Trow[fpos(t, r)];
        const double f = F[t][r] * sc;
        z[4 * t + r] = make_double2(fma(v.x, f, Br[t][r] * sc), fma(v.y, f, Bi[t][r] * sc));
      }
    // a lane writes back only the positions it read (the last lp reads of the tile precede the chunk's barriers)
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) Trow[fpos(t, r)] = z[4 * t + r];
    __syncthreads();
    if (lg1 > 0) fft_axis_passes<true>(T, lgTS, RS, lgN, lg1, 1 << lg2, tw);
    fft_axis_passes<true>(T, lgTS, RS, lgN, lg2, 1, tw);
    if (OUT == 3) {
      float2* at = reinterpret_cast<float2*>(oa) + b0 * N;
      for (int e = tid; e < rows * N; e += 256) {
        const double2 v = T[(e >> lgN) * RS + (e & (N - 1))];
        at[e] = make_float2((float)v.x, (float)v.y);
      }
    } else if (OUT == 4) {
      double2* at = reinterpret_cast<double2*>(oa) + b0 * N;
      for (int e = tid; e < rows * N; e += 256) at[e] = T[(e >> lgN) * RS + (e & (N - 1))];
    } else {
      double2* ht = h + b0 * N;
      for (int e = tid; e < rows * N; e += 256) ht[e] = T[(e >> lgN) * RS + (e & (N - 1))];
    }
  }
}

// natural-order per-bin tables of k_fft_prep -> the kernel's storage order (bit-reversed per axis),
// negated rinv, components padded to Kp (padding: c' = -inf, zero tables); N <= 64: fragment order of
// k_fft_wave, otherwise the row-major N x Kp / Kp x N order of k_fft_mfma
__global__ __launch_bounds__(256) void k_fft_pack(int N, int lg1, int lg2, int K, int Kp, int has_mean, int frag,
                                                  const double* __restrict__ rinvT, const double2* __restrict__ uT,
                                                  const double* __restrict__ cprime, const double* __restrict__ wT,
                                                  const double2* __restrict__ bT, double* __restrict__ pr,
                                                  double* __restrict__ pur, double* __restrict__ pui,
                                                  double* __restrict__ pc, double* __restrict__ pw,
                                                  double* __restrict__ pbr, double* __restrict__ pbi) {
  const int n2m = (1 << lg2) - 1;
  auto bin_of = [&](int p) { return (brev(p >> lg2, lg1) << lg2) | brev(p & n2m, lg2); };
  const long long total = (long long)N * Kp;
  // fragment order, table layouts: 0 k_fft_wave (lp bins 4 t + k, filter bins 16 t + row), 1 k_fft_chunk<256> (filter
  // bins chunk256_bin), 2 k_fft_wreg (lp bins 16 k + t, filter bins chunk256_bin)
  const int layout = (N == 256) ? 1 : (N == 64 && frag) ? 2 : 0;
  if (N <= 64 || frag) {  // fragment order: e = ((cb Q + i) 64 + lane) 2 + s, Q = N / 8 16-byte loads per block and table
    const int Q = N / 8, NT = N / 16;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
      const int s = (int)(e & 1), lane = (int)((e >> 1) & 63);
      const long long g = e >> 7;
      const int i = (int)(g % Q), cb = (int)(g / Q);
      const int j = 2 * i + s;
      {  // lp: t = j, bin 4t + lane/16, comp 16cb + lane%16
        const int p = (layout == 2) ? 16 * (lane >> 4) + j : 4 * j + (lane >> 4), k = 16 * cb + (lane & 15);
        const bool ok = k < K;
        const long long src = (long long)bin_of(p) * K + k;
        pr[e] = ok ? -rinvT[src] : 0.0;
        if (has_mean) {
          pur[e] = ok ? 2.0 * uT[src].x : 0.0;
          pui[e] = ok ? 2.0 * uT[src].y : 0.0;
        }
      }
      {  // filter: r = j / NT, t = j % NT; comp 16cb + lane/16 + 4r, bin 16t + lane%16
        const int r = j / NT, t = j % NT;
        const int k = 16 * cb + (lane >> 4) + 4 * r;
        const int p = (layout != 0) ? chunk256_bin(t, lane & 15) : 16 * t + (lane & 15);
        const bool ok = k < K;
        const long long src = (long long)k * N + bin_of(p);
        pw[e] = ok ? wT[src] : 0.0;
        if (has_mean) {
          pbr[e] = ok ? bT[src].x : 0.0;
          pbi[e] = ok ? bT[src].y : 0.0;
        }
      }
      if (e < Kp) pc[e] = e < K ? cprime[e] : -__builtin_inf();
    }
    return;
  }
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    {  // N x Kp
      const int p = (int)(e / Kp), k = (int)(e % Kp);
      const bool ok = k < K;
      const long long src = (long long)bin_of(p) * K + k;
      pr[e] = ok ? -rinvT[src] : 0.0;
      if (has_mean) {
        pur[e] = ok ? 2.0 * uT[src].x : 0.0;
        pui[e] = ok ? 2.0 * uT[src].y : 0.0;
      }
    }
    {  // Kp x N
      const int k = (int)(e / N), p = (int)(e % N);
      const bool ok = k < K;
      const long long src = (long long)k * N + bin_of(p);
      pw[e] = ok ? wT[src] : 0.0;
      if (has_mean) {
        pbr[e] = ok ? bT[src].x : 0.0;
        pbi[e] = ok ? bT[src].y : 0.0;
      }
    }
    if (e < Kp) pc[e] = e < K ? cprime[e] : -__builtin_inf();
  }
}

template <int N, int OUT, bool HM>
hipError_t launch_mfma_t(const QceFftEstArgs& a, hipStream_t st) {
  constexpr int KW = N >= 64 ? N / 64 : 1;
  constexpr int TS = 16 * (4 / KW);
  // twiddles + the spectra tile (the lp exchange of the component loop aliases the tile)
  const size_t lds = 128 * 16 + (size_t)TS * (N + 1) * 16;
  static_assert(2 * 4 * 256 * 8 <= TS * (N + 1) * 16, "exchange fits the tile");
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_mfma<N, OUT, HM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int lg1 = __builtin_ctz(a.n1), lg2 = __builtin_ctz(a.n2);
  dim3 grid((unsigned)((a.B + TS - 1) / TS));
  hipLaunchKernelGGL((k_fft_mfma<N, OUT, HM>), grid, dim3(256), lds, st, a.B, lg1, lg2, a.Kp, a.y, a.pr,
                     a.pur, a.pui, a.pc, a.pw, a.pbr, a.pbi, a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int N, int OUT, bool HM, bool CIRC>
hipError_t launch_wave_c(const QceFftEstArgs& a, hipStream_t st) {
  const size_t lds = 128 * 16 + (size_t)4 * 16 * (N + 1) * 16;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_wave<N, OUT, HM, CIRC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int lg1 = __builtin_ctz(a.n1), lg2 = __builtin_ctz(a.n2);
  const long long ntiles = (a.B + 15) / 16;
  // persistent: two workgroups (8 waves) per CU; with means one (their accumulators need the registers of
  // two waves)
  const long long slots = (HM ? 1LL : 2LL) * (a.cu > 0 ? a.cu : 256);
  // zero-mean: one workgroup per tile up to the slot count (tiles beyond whole rounds of 4 waves are
  // worked cooperatively by a workgroup's four waves); with means: one wave per tile
  const long long want = HM ? (ntiles + 3) / 4 : ntiles;
  const long long wgs = want < slots ? want : slots;
  hipLaunchKernelGGL((k_fft_wave<N, OUT, HM, CIRC>), dim3((unsigned)wgs), dim3(256), lds, st, a.B, ntiles, lg1, lg2,
                     a.Kp, a.y, a.pr, a.pur, a.pui, a.pc, a.pw, a.pbr, a.pbi, a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int OUT, bool HM>
hipError_t launch_wreg(const QceFftEstArgs& a, hipStream_t st) {
  const size_t lds = 128 * 16 + 32 * 8 + 64 * 16 + (size_t)4 * (HM ? 1664 : 16 * 65) * 16;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_wreg<OUT, HM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const long long ntiles = (a.B + 15) / 16;
  // persistent: two workgroups (8 waves) per CU, one with means (a wave per SIMD)
  const long long slots = (HM ? 1LL : 2LL) * (a.cu > 0 ? a.cu : 256);
  const long long wgs = ntiles < slots ? ntiles : slots;
  hipLaunchKernelGGL((k_fft_wreg<OUT, HM>), dim3((unsigned)wgs), dim3(256), lds, st, a.B, ntiles, __builtin_ctz(a.n2),
                     a.Kp, a.y, a.pr, a.pur, a.pui, a.pc, a.pw, a.pbr, a.pbi, a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int N, int OUT, bool HM>
hipError_t launch_wave_t(const QceFftEstArgs& a, hipStream_t st) {
  if constexpr (N == 64) {
    if (a.chunk) return launch_wreg<OUT, HM>(a, st);
  }
  return a.n1 == 1 ? launch_wave_c<N, OUT, HM, true>(a, st) : launch_wave_c<N, OUT, HM, false>(a, st);
}


template <int N, int OUT>
hipError_t launch_chunk_t(const QceFftEstArgs& a, hipStream_t st) {
  constexpr size_t lds = FftChunkLds<N>::bytes;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_chunk<N, OUT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int lg1 = __builtin_ctz(a.n1), lg2 = __builtin_ctz(a.n2);
  dim3 grid((unsigned)((a.B + 15) / 16));
  hipLaunchKernelGGL((k_fft_chunk<N, OUT>), grid, dim3(256), lds, st, a.B, lg1, lg2, a.Kp, a.y, a.pr, a.pc, a.pw,
                     a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int N, int OUT>
hipError_t launch_chunk_hm(const QceFftEstArgs& a, hipStream_t st) {
  constexpr size_t lds = FftChunkHmLds<N>::bytes;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fft_chunk_hm<N, OUT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int lg1 = __builtin_ctz(a.n1), lg2 = __builtin_ctz(a.n2);
  dim3 grid((unsigned)((a.B + 15) / 16));
  hipLaunchKernelGGL((k_fft_chunk_hm<N, OUT>), grid, dim3(256), lds, st, a.B, lg1, lg2, a.Kp, a.y, a.pr, a.pur, a.pui,
                     a.pc, a.pw, a.pbr, a.pbi, a.h, a.om, a.os, a.oa);
  return hipGetLastError();
}

template <int OUT, bool HM>
hipError_t launch_mfma_out(const QceFftEstArgs& a, hipStream_t st) {
  switch (a.N) {
    case 16: return launch_wave_t<16, OUT, HM>(a, st);
    case 32: return launch_wave_t<32, OUT, HM>(a, st);
    case 64: return launch_wave_t<64, OUT, HM>(a, st);
    case 128:
      if (a.chunk) return HM ? launch_chunk_hm<128, OUT>(a, st) : launch_chunk_t<128, OUT>(a, st);
      return launch_mfma_t<128, OUT, HM>(a, st);
    case 256:
      if (a.chunk) return HM ? launch_chunk_hm<256, OUT>(a, st) : launch_chunk_t<256, OUT>(a, st);
      return launch_mfma_t<256, OUT, HM>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool qce_fft_mfma_shape(int N) { return N >= 16 && N <= 256 && (N & (N - 1)) == 0; }

int qce_fft_kpad(int K) { return (K + 15) & ~15; }

hipError_t qce_launch_fft_pack(const QceFftEstArgs& a, const double* rinvT, const double2* uT, const double* cprime,
                               const double* wT, const double2* bT, hipStream_t st) {
  const int lg1 = __builtin_ctz(a.n1), lg2 = __builtin_ctz(a.n2);
  const long long total = (long long)a.N * a.Kp;
  const int blocks = (int)((total + 255) / 256);
  hipLaunchKernelGGL(k_fft_pack, dim3(blocks), dim3(256), 0, st, a.N, lg1, lg2, a.K, a.Kp, a.has_mean,
                     a.chunk, rinvT, uT,
                     cprime, wT, bT, const_cast<double*>(a.pr), const_cast<double*>(a.pur),
                     const_cast<double*>(a.pui), const_cast<double*>(a.pc), const_cast<double*>(a.pw),
                     const_cast<double*>(a.pbr), const_cast<double*>(a.pbi));
  return hipGetLastError();
}

hipError_t qce_launch_fft_mfma(const QceFftEstArgs& a, int out, hipStream_t st) {
  if (a.B <= 0) return hipSuccess;
  if (out == 0) return a.has_mean ? launch_mfma_out<0, true>(a, st) : launch_mfma_out<0, false>(a, st);
  if (out == 3) return a.has_mean ? launch_mfma_out<3, true>(a, st) : launch_mfma_out<3, false>(a, st);
  if (out == 4) return a.has_mean ? launch_mfma_out<4, true>(a, st) : launch_mfma_out<4, false>(a, st);
  return hipErrorInvalidValue;
}

#ifdef QCE_STAMPS
// diagnostic build only: point k_fft_wave's stamp buffer at dev (8 x 64-bit per wave; nullptr = off)
hipError_t qce_fft_set_stamps(unsigned long long* dev) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fft_stamps), &dev, sizeof(dev));
}
#endif
