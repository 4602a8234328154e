// FP64 'all' mode for the padded dimensions beyond the fused kernel (max(MP, NP) = 256): the reference's own
// two-step form of estimate_from_y's 'all' branch (gmm_cplx_bussgang.py:220-228) --
//
//   proba = predict_proba_cplx(y)                  (lp on FP64 MFMA: k_lp_f64; logsumexp: k_wsum_weights)
//   h_b   = sum_k proba_bk (W_k y_b + b_k)         (k_wsum_f64, FP64 MFMA, FP64 accumulation)
//
// every product an FP64 computation of the reference's complex128 formula.  The same two kernels give the
// K-shard partials: weights e^{lp - m_b} with (m, s) per row, or e^{lp - M*} packed for one SUM collective.
//
// k_wsum_f64 is a GEMM whose reduction runs over (component, observation column): the B operand of component k is
// proba_bk * y_b, built in registers from y fragments that stay resident for one 64-column chunk of the
// observation.  Workgroup = 4 waves x (16 CT) samples sharing one stream of filter blocks through an LDS ring
// (global_load_lds, 16 B per lane, one barrier per 16 KB chunk); a workgroup owns RG row tiles (8 complex rows
// each) of the output, so accumulators + y fragments fit one wave per SIMD.  Roofline: FP64 MFMA,
// 8 M N flops per (sample, component).
#include "qce_f64_kernel.h"

namespace {

template <int MP, int NP, bool HM>
struct WsG {
  static constexpr int MC = MP < 64 ? MP : 64;   // complex observation columns per chunk
  static constexpr int NMC = MP / MC;            // chunks
  static constexpr int KPC = MC / 4;             // k-pairs (4 complex columns) per chunk
  static constexpr int NTW = NP / 8;             // output row tiles (8 complex rows each)
  static constexpr int RG = NTW < 8 ? NTW : 8;   // row tiles per workgroup
  static constexpr int NG = NTW / RG;            // row groups
  static constexpr int SL = KPC * RG + (HM ? RG : 0);  // 1 KB blocks per (component, chunk, group) stream
  static constexpr int CB = 16;                  // blocks per ring chunk (16 KB)
  static constexpr int SLP = (SL + CB - 1) / CB * CB;
  static constexpr int NCH = SLP / CB;           // ring chunks per stream
  static constexpr int NSLOT = 8;                // 128 KB of LDS
  static constexpr int NW = 4;
  static constexpr int LPW = CB / NW;            // 1 KB pieces per wave per ring chunk
};

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// weights: one lane per observation row (coalesced K x B stores)
//   mode 0: proba = exp(lp - logsumexp(lp))       ('all', gmm_cplx_bussgang.py:220-228, :351-367, :632-656)
//   mode 1: e^{lp - m_b}, m_b = max_k lp, s_b = sum_k e^{lp - m_b} -> om, os (K-shard partial)
//   mode 2: e^{lp - M*} with the shared shift M*, s -> pk[b][0], 0 -> pk[b][1] (shifted packed K-shard partial)
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wsum_weights(long long B, int K, const double* __restrict__ lp, int mode,
                                                      const double* __restrict__ shift, double* __restrict__ wT,
                                                      double* __restrict__ om, double* __restrict__ os,
                                                      double* __restrict__ pk, long long pk_stride) {
  const long long b = (long long)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const double* r = lp + b * K;
  double m = QCE_NEG_INF;
  for (int k = 0; k < K; ++k) m = fmax(m, r[k]);
  if (mode == 2) {
    const double sh = *shift;
    double tot = 0.0;
    for (int k = 0; k < K; ++k) {
      const double v = r[k] == QCE_NEG_INF ? 0.0 : exp(r[k] - sh);
      wT[(long long)k * B + b] = v;
      tot += v;
    }
    pk[b * pk_stride] = tot;
    pk[b * pk_stride + 1] = 0.0;
    return;
  }
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += r[k] == QCE_NEG_INF ? 0.0 : exp(r[k] - m);
  if (mode == 0) {
    const double lse = log(s) + m;  // scipy.special.logsumexp
    for (int k = 0; k < K; ++k) wT[(long long)k * B + b] = exp(r[k] - lse);
  } else {
    for (int k = 0; k < K; ++k) wT[(long long)k * B + b] = r[k] == QCE_NEG_INF ? 0.0 : exp(r[k] - m);
    om[b] = m;
    os[b] = s;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// filter tables: stream (k, c, rg) = blocks (k-pair s outer, row tile t inner) of E(W_k) rows 8(rg RG + t) ..
// columns c MC .. + MC, then (HM) RG blocks with the b_k column (zero for c > 0), padded to whole ring chunks.
// Block = A operand of one row tile for the two k-steps of a k-pair, lane-major (lane l: 16 B), as k_pack_f64all.
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pack_wsum(int M, int N, int MC, int NMC, int KPC, int RG, int NG, int has_mean,
                                                  int slp, const double2* __restrict__ W,
                                                  const double2* __restrict__ bvec, double* __restrict__ pack) {
  const int q = blockIdx.y, lane = threadIdx.x;
  const long long stream = blockIdx.x;  // (k NMC + c) NG + rg
  const int rg = (int)(stream % NG), c = (int)((stream / NG) % NMC);
  const long long k = stream / ((long long)NG * NMC);
  const int rho = lane & 15, gk = lane >> 4;
  double v0 = 0.0, v1 = 0.0;
  int tt = -1, s = 0, bias = 0;
  if (q < KPC * RG) {
    s = q / RG;
    tt = q % RG;
  } else if (has_mean && q < KPC * RG + RG) {
    tt = q - KPC * RG;
    bias = 1;
  }
  if (tt >= 0) {
    const int T = rg * RG + tt;
    const int i = 8 * T + 4 * (rho >> 3) + (rho & 3), a = (rho >> 2) & 1;
    if (!bias) {
      const int j = c * MC + 4 * s + gk;
      if (i < N && j < M) {
        const double2 z = W[(k * N + i) * M + j];
        v0 = a == 0 ? z.x : z.y;   // k-step 2s: multiplies Re y_j
        v1 = a == 0 ? -z.y : z.x;  // k-step 2s+1: multiplies Im y_j
      }
    } else if (c == 0 && gk == 0 && i < N) {
      const double2 z = bvec[k * N + i];
      v0 = a == 0 ? z.x : z.y;
    }
  }
  *reinterpret_cast<double2*>(pack + ((stream * slp + q) * 64 + lane) * 2) = make_double2(v0, v1);
}

// ---------------------------------------------------------------------------------------------------------------
// out[b][ooff + i] = sum_k w_kb (W_k y_b + b_k)_i   (double2 elements, row stride ostride)
// grid (ceil(B / TS), NG); TS = 64 CT samples
// ---------------------------------------------------------------------------------------------------------------
template <int MP, int NP, bool HM, int CT>
__global__ __launch_bounds__(256, 1) void k_wsum_f64(long long B, int M, int N, int K, const double2* __restrict__ y,
                                                     const char* __restrict__ pack, const double* __restrict__ wT,
                                                     double2* __restrict__ out, long long ostride, int ooff) {
  using G = WsG<MP, NP, HM>;
  constexpr int NW = G::NW, CHUNK = G::CB * 1024;
  constexpr int TS = NW * 16 * CT;
  __shared__ __attribute__((aligned(16))) char lds[G::NSLOT * CHUNK];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, col = lane & 15;
  const long long tile = blockIdx.x;
  const int rg = blockIdx.y;
  const long long sbase = tile * TS + (long long)wave * 16 * CT;
  const long long nchunks = (long long)K * G::NMC * G::NCH;

  // ring: chunk j of the stream order (chunk c outer, component k inner) -> slot j % NSLOT
  auto issue = [&](long long j) {
    // the slot follows the unclamped stream index (past the end: the slot the barrier just freed, never read);
    // only the source is clamped, to the last chunk, which keeps vmcnt uniform (a clamped slot index
    // wrote into the last real chunk's slot while other waves could still read it)
    char* dst = lds + (int)(j % G::NSLOT) * CHUNK + wave * 1024;
    if (j >= nchunks) j = nchunks - 1;
    const long long st = j / G::NCH;
    const int cc = (int)(j % G::NCH);
    const long long c = st / K, k = st % K;
    const char* src = pack + ((((k * G::NMC + c) * G::NG + rg) * G::SLP + (long long)cc * G::CB) * 1024) +
                      wave * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < G::LPW; ++i)
      lds_dma16(src + i * NW * 1024, dst + i * NW * 1024);
  };
#pragma unroll 1
  for (int j = 0; j < G::NSLOT - 1; ++j) issue(j);
  long long jc = 0;  // next chunk to consume

  f64x4 acc[G::RG][CT];
#pragma unroll
  for (int t = 0; t < G::RG; ++t)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[t][c] = f64x4{0.0, 0.0, 0.0, 0.0};
  long long srow[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const long long sm = sbase + 16 * c + col;
    srow[c] = sm < B ? sm : B - 1;  // clamped rows compute on finite data and are never stored
  }

#pragma unroll 1
  for (int ch = 0; ch < G::NMC; ++ch) {
    // y fragments of this column chunk: k-pair s, lane group g -> complex column ch MC + 4 s + g
    double2 yv[CT][G::KPC];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const double2* yr = y + srow[c] * M;
#pragma unroll
      for (int s = 0; s < G::KPC; ++s) {
        const int cc = ch * G::MC + 4 * s + g;
        yv[c][s] = yr[cc < M ? cc : M - 1];  // a padded column meets zero table entries
      }
    }
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
      double wk[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) wk[c] = wT[(long long)k * B + srow[c]];
      double bs0[CT], bs1[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) bs0[c] = bs1[c] = 0.0;
      static_for(
          [&](auto ccv) {
            constexpr int cc = decltype(ccv)::value;
            // chunk jc: every wave's pieces landed, every wave is done with chunk jc - 1 (its slot is refilled)
            wait_vmcnt<(G::NSLOT - 2) * G::LPW>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            issue(jc + G::NSLOT - 1);
            const int roff = (int)(jc % G::NSLOT) * CHUNK + lane * 16;
            ++jc;
            double2 a_next = *reinterpret_cast<const double2*>(&lds[roff]);
            static_for(
                [&](auto iv) {
                  constexpr int i = decltype(iv)::value;
                  constexpr int q = cc * G::CB + i;
                  const double2 a = a_next;
                  if constexpr (i + 1 < G::CB) a_next = *reinterpret_cast<const double2*>(&lds[roff + (i + 1) * 1024]);
                  __builtin_amdgcn_sched_barrier(0);
                  if constexpr (q < G::KPC * G::RG) {  // filter block (k-pair s, row tile t)
                    constexpr int s = q / G::RG, t = q % G::RG;
                    if constexpr (t == 0) {
#pragma unroll
                      for (int c = 0; c < CT; ++c) {
                        bs0[c] = yv[c][s].x * wk[c];
                        bs1[c] = yv[c][s].y * wk[c];
                      }
                    }
#pragma unroll
                    for (int c = 0; c < CT; ++c) acc[t][c] = mfma16x16x4d(a.x, bs0[c], acc[t][c]);
#pragma unroll
                    for (int c = 0; c < CT; ++c) acc[t][c] = mfma16x16x4d(a.y, bs1[c], acc[t][c]);
                  } else if constexpr (HM && q < G::SL) {  // b_k column: B = w in lane group 0 (chunk 0 only)
                    constexpr int t = q - G::KPC * G::RG;
                    if (ch == 0) {
#pragma unroll
                      for (int c = 0; c < CT; ++c) acc[t][c] = mfma16x16x4d(a.x, g == 0 ? wk[c] : 0.0, acc[t][c]);
                    }
                  }
                },
                std::make_integer_sequence<int, G::CB>{});
          },
          std::make_integer_sequence<int, G::NCH>{});
    }
  }
  // rows of row tile T: complex 8T + g (regs 0, 1) and 8T + 4 + g (regs 2, 3)
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const long long sm = sbase + 16 * c + col;
    if (sm >= B) continue;
    double2* o = out + sm * ostride + ooff;
#pragma unroll
    for (int t = 0; t < G::RG; ++t) {
      const int T = rg * G::RG + t;
      const int i0 = 8 * T + g, i1 = 8 * T + 4 + g;
      if (i0 < N) o[i0] = make_double2(acc[t][c][0], acc[t][c][1]);
      if (i1 < N) o[i1] = make_double2(acc[t][c][2], acc[t][c][3]);
    }
  }
  wait_vmcnt<0>();  // drain the ring's trailing (dummy) loads before the workgroup retires
}

// ---------------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------------
namespace {
constexpr int WS_CT = 2;

int ws_dims(int MP, int NP, int hm, int* mc, int* nmc, int* kpc, int* rg, int* ng, int* slp) {
  const int MC = MP < 64 ? MP : 64, NTW = NP / 8, RG = NTW < 8 ? NTW : 8;
  const int SL = (MC / 4) * RG + (hm ? RG : 0);
  *mc = MC;
  *nmc = MP / MC;
  *kpc = MC / 4;
  *rg = RG;
  *ng = NTW / RG;
  *slp = (SL + 15) / 16 * 16;
  return 0;
}

template <int MP, int NP, bool HM>
hipError_t launch_wsum_t(const QceWsumArgs& a, hipStream_t st) {
  using G = WsG<MP, NP, HM>;
  constexpr int TS = 4 * 16 * WS_CT;
  dim3 grid((unsigned)((a.B + TS - 1) / TS), (unsigned)G::NG);
  hipLaunchKernelGGL((k_wsum_f64<MP, NP, HM, WS_CT>), grid, dim3(256), 0, st, a.B, a.M, a.N, a.K, a.y, a.pack, a.wT,
                     a.out, a.ostride, a.ooff);
  return hipGetLastError();
}

template <int MP, int NP>
hipError_t launch_wsum_mn(const QceWsumArgs& a, hipStream_t st) {
  return a.has_mean ? launch_wsum_t<MP, NP, true>(a, st) : launch_wsum_t<MP, NP, false>(a, st);
}
}  // namespace

// the two-pass FP64 path covers every padded shape with a dimension of 256 (the fused kernel stops at 128)
bool qce_wsum_shape(int MP, int NP) {
  auto ok = [](int v) { return v == 16 || v == 32 || v == 64 || v == 128 || v == 256; };
  return ok(MP) && ok(NP) && (MP == 256 || NP == 256);
}

long long qce_pack_wsum_bytes(int MP, int NP, int has_mean) {
  int mc, nmc, kpc, rg, ng, slp;
  ws_dims(MP, NP, has_mean, &mc, &nmc, &kpc, &rg, &ng, &slp);
  return (long long)nmc * ng * slp * 1024;  // per component
}

hipError_t qce_launch_pack_wsum(int K, int M, int N, int MP, int NP, int has_mean, const double2* W,
                                const double2* bvec, double* pack, hipStream_t st) {
  int mc, nmc, kpc, rg, ng, slp;
  ws_dims(MP, NP, has_mean, &mc, &nmc, &kpc, &rg, &ng, &slp);
  hipLaunchKernelGGL(k_pack_wsum, dim3((unsigned)K * nmc * ng, slp), dim3(64), 0, st, M, N, mc, nmc, kpc, rg, ng,
                     has_mean, slp, W, bvec, pack);
  return hipGetLastError();
}

hipError_t qce_launch_wsum_weights(long long B, int K, const double* lp, int mode, const double* shift, double* wT,
                                   double* om, double* os, double* pk, long long pk_stride, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_wsum_weights, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, B, K, lp, mode, shift, wT, om,
                     os, pk, pk_stride);
  return hipGetLastError();
}

hipError_t qce_launch_wsum(const QceWsumArgs& a, hipStream_t st) {
  if (a.B <= 0) return hipSuccess;
#define QCE_WS(X, Y) \
  if (a.MP == X && a.NP == Y) return launch_wsum_mn<X, Y>(a, st);
  QCE_WS(256, 16) QCE_WS(256, 32) QCE_WS(256, 64) QCE_WS(256, 128) QCE_WS(256, 256)
  QCE_WS(16, 256) QCE_WS(32, 256) QCE_WS(64, 256) QCE_WS(128, 256)
#undef QCE_WS
  return hipErrorInvalidValue;
}
