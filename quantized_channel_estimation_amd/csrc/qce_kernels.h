// Internal launch interface between the C-ABI layer (qce_capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

struct QcePrepareArgs {
  int K, N, M, MP, NP, has_mean, identityA;
  int kind;        // 0: 1 bit, 1: multi-bit, 2: n_bits = inf
  int n_bits;      // multi-bit only
  int quant_kind;  // 0 uniform, 1 lloyd, 2 other (zero gain)
  int beta_first;  // multi-bit Cr: beta = gain[0] (blmmse.py) instead of clip(mean gain, 0, 1)
  double sigma2, delta;
  const double* thr;  // device, 2^b - 1 entries
  const double* lab;  // device, 2^b entries
  const double2* A;   // M x N
  const double2* covs;
  const double2* means;
  const double* logw;
  double2 *Cy, *Cr, *Lw, *Linv, *Aeff, *work, *V, *W, *means_y, *q0, *bvec;
  double *gain, *cconst;
  int* status;
  float* pack32;
  long long stride32;
  double* pack64;
  long long stride64;
};

long long qce_pack_f32_stride(int MP, int NP, int has_mean);
long long qce_pack_f64_stride(int MP, int has_mean);
hipError_t qce_launch_prepare(const QcePrepareArgs& p, hipStream_t st);
hipError_t qce_launch_pack_selective(const QcePrepareArgs& p, hipStream_t st);

struct QceEstArgs {
  long long B;
  int M, N, K, MP, NP, has_mean;
  const double2* y;  // B x M (row stride M)
  const float* pack32;
  long long stride32;
  const double* pack64;
  long long stride64;
  const double* cconst;
};

// 'all' mode, fused responsibilities + LMMSE combination; h = B x N complex128
hipError_t qce_launch_est_all(const QceEstArgs& a, double2* h, hipStream_t st);
// K-shard partial: m, s (B doubles), acc (B x 2N floats, un-normalised, interleaved re/im)
hipError_t qce_launch_est_partial(const QceEstArgs& a, double* m, double* s, float* acc, hipStream_t st);
// weighted log-probabilities lp[b][k] (FP64), row stride K
hipError_t qce_launch_lp(const QceEstArgs& a, double* lp, hipStream_t st);
// selection: mode 0 = proba only, 1 = top-n, 2 = cumulative-p, 3 = argmax(lp)
hipError_t qce_launch_select(long long B, int K, const double* lp, int mode, int n, double p, double* proba,
                             long long* labels, float* wts, hipStream_t st, double* wts64 = nullptr);
int qce_select_max_k();  // widest K qce_launch_select covers (k_select up to 256, k_select_wide beyond)
// FP64 selective-mode LMMSE h = sum_k w64[b][k] (W_k y + b_k), w64 sparse; WT (K x M x N) = transposed filters
// (built from W when transpose, else reused)
hipError_t qce_launch_sparse_f64(long long B, int N, int M, int K, const double2* y, const double* w, const double2* W,
                                 const double2* bvec, double2* WT, bool transpose, double2* h, hipStream_t st);
// h = sum_k wts[b][k] (W_k y_b + b_k)
hipError_t qce_launch_est_weighted(const QceEstArgs& a, const float* wts, double2* h, hipStream_t st);
bool qce_shape_supported(int MP, int NP);         // FP32 fused kernel (M, N <= 64)
bool qce_select_shape_supported(int MP, int NP);  // lp + weighted kernels of the selective modes

// FP16 two-term split kernel (qce_estimate_h2.hip), stream-K scheduled
struct QceH2Args {
  long long B;
  int M, N, K, MP, NP, has_mean;
  int nwg;      // persistent workgroups P
  int R;        // data-parallel rounds of whole tiles
  long long L;  // stream-K tail: work items (tile, component) per workgroup
  double y_scale;
  int* yflag;  // device int: set when some observation is not exact in fp16 (k_y_exact)
  const double2* y;
  const char* pack;
  long long cstride;  // bytes per component
  const float* sinv;  // K x (NSL + NSW) inverse slice scales (y-scale folded in)
  const double* cconst;
  double2* h;                  // final output (or nullptr with out_partial)
  double *om, *os;             // partial-format output (K-shard path)
  float* oa;
  double *pm, *ps;             // scratch for cut tiles: nwg * 2 * 256 records
  float* pa;
};
long long qce_pack_h2_stride_bytes(int MP, int NP, int has_mean);
hipError_t qce_launch_pack_h2(int K, int M, int N, int MP, int NP, int has_mean, long long cstride, double y_scale,
                              const double2* Linv, const double2* W, const double2* q0, const double2* bvec, char* pack,
                              float* sinv, hipStream_t st);
hipError_t qce_launch_est_h2(const QceH2Args& a, bool out_partial, hipStream_t st);
int qce_h2_blocks_per_cu(int MP, int NP, int has_mean);

// FP64 fused 'all' kernel (qce_estimate_f64.hip): the reference-precision path, stream-K scheduled
struct QceF64Args {
  long long B;
  int M, N, K, MP, NP, has_mean;
  int nwg;      // persistent workgroups P
  int R;        // data-parallel rounds of whole tiles
  long long L;  // stream-K tail: (tile, component) items per workgroup
  const double2* y;
  const char* pack;  // K x qce_pack_f64all_bytes
  const double* cconst;
  double2* h;           // final output (or nullptr with out_partial)
  double *om, *os, *oa;  // partial-format output (K-shard path), oa B x 2N
  double *pm, *ps, *pa;  // scratch for cut tiles: nwg * 2 * tile records
  double* pk = nullptr;   // shifted packed partial B x (2N+2): [s e^{m-shift}, 0, acc e^{m-shift}] (instead of om/os/oa)
  const double* shift = nullptr;  // device pointer: the shared shift M* of the packed partial
  unsigned long long* stamps = nullptr;  // diagnostic builds (-DQCE_STAMPS): per-wave segment cycles
  int waves = 8;  // workgroup shape where M, N <= 64: 8 waves x 1 column tile (two per SIMD), or 4 x 2 (QCE_F64_WAVES=4)
  int g3 = 0;     // 3M tables / kernel: 1 k_est_all_f64g (padded M, N <= 64; 8 waves x 16 samples), 2 k_est_all_f64h
                 // (padded M = N = 128: row halves, y in LDS; 8 waves x 64 samples)
};
// k_est_all_f64h (qce_f64h.hip): the 3M kernel for padded M = N = 128
bool qce_f64h_shape(int MP, int NP);
long long qce_pack_f64h_bytes(int has_mean);
hipError_t qce_launch_pack_f64h(int K, int M, int N, int has_mean, const double2* Linv, const double2* W,
                                const double2* q0, const double2* bvec, double* pack, hipStream_t st);
hipError_t qce_f64h_launch(const QceF64Args& a, bool out_partial, hipStream_t st);
bool qce_f64g_shape(int MP, int NP);
int qce_f64g_waves();  // waves per workgroup of k_est_all_f64g (tile = 16 x waves samples; 8 / waves workgroups per CU)
long long qce_pack_f64g_bytes(int MP, int NP, int has_mean);
hipError_t qce_launch_pack_f64g(int K, int M, int N, int MP, int NP, int has_mean, const double2* Linv,
                                const double2* W, const double2* q0, const double2* bvec, double* pack,
                                hipStream_t st);
bool qce_f64_shape(int MP, int NP);
int qce_f64_tile(int MP, int NP);  // samples per workgroup tile
long long qce_pack_f64all_bytes(int MP, int NP, int has_mean);
hipError_t qce_launch_pack_f64all(int K, int M, int N, int MP, int NP, int has_mean, const double2* Linv,
                                  const double2* W, const double2* q0, const double2* bvec, double* pack,
                                  hipStream_t st);
hipError_t qce_launch_est_f64(const QceF64Args& a, bool out_partial, hipStream_t st);
hipError_t qce_launch_pack_shifted(long long B, int N, const double* m, const double* s, const double* acc,
                                   const float* acc32, const double* shift, double* pk, hipStream_t st);
// out[0] = max_k cconst[k] (device), the local part of the K-shard shift M*
hipError_t qce_launch_cconst_max(int K, const double* cconst, const int* status, double* out, hipStream_t st);
hipError_t qce_launch_f64_to_f32(const double* a, float* b, long long n, hipStream_t st);
// FP64 'all' mode beyond the fused kernel's 128 (qce_wsum_f64.hip): lp (k_lp_f64) -> weights -> weighted filter sum
struct QceWsumArgs {
  long long B;
  int M, N, K, MP, NP, has_mean;
  const double2* y;
  const char* pack;   // K x qce_pack_wsum_bytes
  const double* wT;   // K x B weights
  double2* out;       // out[b * ostride + ooff + i]
  long long ostride;  // double2 elements per output row
  int ooff;
};
bool qce_wsum_shape(int MP, int NP);
long long qce_pack_wsum_bytes(int MP, int NP, int has_mean);  // per component
hipError_t qce_launch_pack_wsum(int K, int M, int N, int MP, int NP, int has_mean, const double2* W,
                                const double2* bvec, double* pack, hipStream_t st);
// mode 0: proba (K x B), 1: e^{lp - m} with (m, s) -> om / os, 2: e^{lp - shift} with s -> pk[b * pk_stride]
hipError_t qce_launch_wsum_weights(long long B, int K, const double* lp, int mode, const double* shift, double* wT,
                                   double* om, double* os, double* pk, long long pk_stride, hipStream_t st);
hipError_t qce_launch_wsum(const QceWsumArgs& a, hipStream_t st);

hipError_t qce_launch_f32_to_f64(const float* a, double* b, long long n, hipStream_t st);

// *flag |= (some y * y_scale is not exactly representable in fp16); n = doubles in y
hipError_t qce_launch_y_exact(long long n, const double* y, double y_scale, int* flag, hipStream_t st);

// chunk-streamed FP16 split kernel for padded M or N of 128 / 256 (qce_estimate_h2x.hip)
struct QceH2XArgs {
  long long B;
  int M, N, K, MP, NP, has_mean;
  double y_scale;
  int* yflag;
  const double2* y;
  const char* pack;
  long long cstride;
  const float* sinv;
  const double* cconst;
  double2* h;                  // final output
  double *om, *os;             // K-shard partial output
  float* oa;
  double *rm, *rs;             // split records: ksplit x B (m, s), ksplit x B x 2N acc
  float* ra;
};
bool qce_h2x_shape(int MP, int NP);
long long qce_h2x_pad_bytes();  // extra bytes the pack allocation needs (chunk overrun)
int qce_h2x_tile();
int qce_h2x_row_chunks(int MP, int NP);
hipError_t qce_launch_est_h2x(const QceH2XArgs& a, int ksplit, bool out_partial, hipStream_t st);

// Fourier-domain path for (block-)circulant mixtures with A = I (qce_fft.hip)
struct QceFftPrepArgs {
  int N, n1, n2, K;
  double s2;
  int kind, n_bits, quant_kind;
  double delta;
  const double *thr, *lab, *logw, *ceig;
  const double2 *col0, *mspec;
  double* rinvT;   // N x K
  double2* uT;     // N x K
  double* cprime;  // K
  double* wT;      // K x N
  double2* bT;     // K x N
  double* gain;    // K
  int* status;     // K
};
struct QceFftEstArgs {
  long long B;
  int N, n1, n2, K, has_mean;
  const double2* y;
  const double* rinvT;
  const double2* uT;
  const double* cprime;
  const double* wT;
  const double2* bT;
  const double* wts;  // FP64 selection weights (out = 2; k_select's wts64)
  double2* h;
  double* lp;        // out = 1
  double *om, *os;   // out = 3, 4
  float* oa;         // out = 3: f32 (B, 2N); out = 4: the same buffer holds an f64 (B, 2N) accumulator
  // MFMA kernel tables (qce_fft_mfma.hip, storage order, components padded to Kp)
  int Kp;
  const double *pr, *pur, *pui, *pc, *pw, *pbr, *pbi;
  int cu;     // compute units of the device (persistent grid of k_fft_wave)
  int chunk;  // N = 128, 256: k_fft_chunk / k_fft_chunk_hm on fragment-order tables (else k_fft_mfma, row-major)
};
bool qce_fft_pow2(int v);
int qce_fft_tile(int N, int K);  // 0: no tile fits (K too large)
hipError_t qce_launch_fft_struct(int K, int N, int n1, int n2, double tol, const double2* covs, const double2* means,
                                 double* ceig, double2* col0, double2* mspec, int* bad, hipStream_t st);
hipError_t qce_launch_fft_prep(const QceFftPrepArgs& a, hipStream_t st);
// out: 0 'all' h, 1 lp, 2 weighted h, 3 K-shard partial (f32 acc), 4 K-shard partial (f64 acc)
hipError_t qce_launch_fft_est(const QceFftEstArgs& a, int out, hipStream_t st);
// MFMA Fourier kernel (qce_fft_mfma.hip): N in {16, ..., 256}; out 0 'all' h, 3 / 4 K-shard partial (f32 / f64)
bool qce_fft_mfma_shape(int N);
int qce_fft_kpad(int K);
hipError_t qce_launch_fft_pack(const QceFftEstArgs& a, const double* rinvT, const double2* uT, const double* cprime,
                               const double* wT, const double2* bT, hipStream_t st);
hipError_t qce_launch_fft_mfma(const QceFftEstArgs& a, int out, hipStream_t st);

// Observation generation / quantisation (qce_observe.hip; utils.py:189-203, :241-251)
struct QceObserveArgs {
  long long B;
  int M, N;
  const double2* A;  // M x N, nullptr = identity (M == N)
  const double2* h;  // B x N
  const double2* w;  // B x M supplied noise (noise == 1)
  int noise;         // 0 none, 1 supplied, 2 generated (Philox, seed, element offset)
  double noise_scale;
  unsigned long long seed, offset;
  int kind;  // 0: 1 bit, 1: multi-bit (thr / lab), 2: unquantised
  const double* thr;
  const double* lab;
  int nthr;
  double2* y;  // B x M
};
hipError_t qce_launch_observe(const QceObserveArgs& a, hipStream_t st);
int qce_sq_err_scratch();
hipError_t qce_launch_sq_err(long long n, const double2* a, const double2* b, double* part, double* out,
                             hipStream_t st);

// EM training (qce_em.hip; gmm_cplx_bussgang.py:612-790)
struct QceEmPlan {
  int C = 0;      // stats chunks of 1024 samples
  int NT = 0;     // 16-wide feature tiles
  int nblk = 0;   // 64 x 64 output blocks
  int chunk = 0;  // samples per covariance workgroup
  int C2 = 0;     // covariance chunks
  size_t stat_doubles = 0, part_elems = 0;
};
QceEmPlan qce_em_plan(long long B, int N, int K, int diag);
struct QceEmArgs {
  long long B;
  int N, K, diag, zero_mean;
  double reg;
  QceEmPlan plan;
  const double2* X;  // B x N
  const double* R;   // B x K responsibilities
  double* stats;     // plan.stat_doubles
  double2* part;     // plan.part_elems
  double* nk;        // K
  double2* means;    // K x N
  double2* covs;     // K x N x N ('full')
  double* diag_out;  // K x N ('diag')
};
hipError_t qce_launch_em_mstep(const QceEmArgs& a, hipStream_t st);
int qce_mean_scratch();
hipError_t qce_launch_em_resp(long long B, int K, const double* lp, double* resp, double* lse, double* part,
                              double* mean_out, hipStream_t st);

// h_b = W_c y_b + b_c with c = comp[b] (comp == nullptr: c = b) — per-sample ("genie") filters
hipError_t qce_launch_est_assigned(long long B, int N, int M, int K, const double2* y, const long long* comp,
                                   const double2* W, const double2* bvec, double2* h, hipStream_t st);

// batched row-major complex GEMM C = alpha op(A) op(B) + beta C (op 0 = N, 1 = T, 2 = C^H); supported
// (opa, opb): (0,0) (0,2) (2,0) (0,1).  Strides sA/sB/sC per batch entry (0 = shared operand).
hipError_t qce_zgemm_batched(int opa, int opb, int m, int n, int k, double2 alpha, const double2* A, int lda,
                             long long sA, const double2* B, int ldb, long long sB, double2 beta, double2* C, int ldc,
                             long long sC, int batch, hipStream_t st);
// Toeplitz inverse-EM covariance step (qce_em.hip; gmm_cplx_bussgang.py:792-826)
//   theta_kp = Re diag(F2 Mx_k F2^H)_p; init: sigma = max(theta, reg); else sigma += sigma^2 theta, max reg
hipError_t qce_launch_inv_em_sigma(int K, int N, int P, const double2* G, const double2* F2, double* sigma, double reg,
                                   int init, hipStream_t st);
//   C_k = F2^H diag(sigma_k) F2 + reg I
hipError_t qce_launch_inv_em_cov(int K, int N, int P, const double2* F2, const double* sigma, double reg, double2* C,
                                 hipStream_t st);

// SCM channels (qce_scm.hip; scm_helper.py:17-84, SCMMulti.py:30-56)
int qce_scm_max_path();
hipError_t qce_launch_scm(long long B, int n_coh, int N, int n_path, double sigma, const double* gains,
                          const double* angles, const double2* x, unsigned long long seed, float2* h, float2* t,
                          hipStream_t st);

// statistical rate lower bound (qce_rate.hip; Bussgang_GMM.py:146-162)
int qce_rate_scratch();
hipError_t qce_launch_rate(long long B, int N, const double2* he, const double2* h, const double* buss,
                           const double2* Cq, double clip, double2* inner, double* den2, double* part, double* stat,
                           hipStream_t st);
// Bussgang LS with column-orthogonal A_eff (qce_genie.hip; estimators/LS.py)
hipError_t qce_launch_ls(long long B, int N, int M, const double2* y, const long long* comp, const double2* Aeff,
                         double2* h, hipStream_t st);
// Pseudo-inverses P_c = (A_eff^H A_eff)^{-1} A_eff^H of full-column-rank A_eff (qce_genie.hip; LS.py general A)
hipError_t qce_launch_rate_mf(long long B, int N, const double2* he, const double2* h, const double* buss,
                              const double2* Cq, const double2* Cqi, double* rate, double* sum, hipStream_t st);
// Gauss-Jordan inverse per component: direct = 0 -> (A^H A)^-1 A^H (M >= N), 1 -> A^-1 (A Hermitian PD, M == N);
// bad[c] = first failing pivot + 1 (0 = ok)
hipError_t qce_launch_ls_pinv(int K, int N, int M, int direct, const double2* Aeff, double2* T, double2* P,
                              double2* bzero, int* bad, hipStream_t st);
