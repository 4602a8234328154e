// Private layout of a qce_model (the opaque handle of include/qce.h), shared by the C-ABI units
// (qce_capi.hip: model lifetime / prepare / estimate; qce_kshard.hip: the K-shard step over a communicator).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "qce_kernels.h"

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, sizeof(T) * (count ? count : 1));
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct qce_model {
  int K = 0, N = 0, device = 0;
  int a_identity_n = 0;   // m->A holds I_N (skips the upload + sync of a repeated A = NULL prepare)
  // zero-mean model: the first q0_zeroed / bvec_zeroed elements of q0 / bvec hold zeros (the prepare then skips
  // their three launches).  Counted in elements, not remembered by address: a DevBuf::ensure that grows
  // the buffer may get the old address back from hipMalloc, and the grown tail must be zeroed again
  size_t q0_zeroed = 0, bvec_zeroed = 0;
  int packs_valid = 0;    // pack32 / pack64 built for the current prepare (lazy: 'all' mode never needs them)
  QcePrepareArgs pack_args{};
  int beta_first = 0;  // QCE_OPT_BETA_FIRST: multi-bit Cr mixes with the first gain (blmmse.py:53, :86)
  int precision = QCE_PRECISION_F64;  // QCE_OPT_PRECISION: arithmetic of the dense 'all' / partial path
  hipStream_t stream = nullptr;
  int has_mean = 0;
  std::vector<double> weights;
  DevBuf<double2> means, covs;
  DevBuf<double> logw;
  // prepared state
  int M = 0, MP = 0, NP = 0, prepared = 0;
  DevBuf<double2> A, Cy, Cr, Lw, Linv, Aeff, work, V, W, means_y, q0, bvec;
  DevBuf<double> gain, cconst, thr, lab;
  DevBuf<int> status;
  int* status_host = nullptr;  // pinned copy of the last prepare's Cholesky status (read lazily)
  hipEvent_t status_ev = nullptr;
  int status_pending = 0;
  DevBuf<float> pack32;
  DevBuf<double> pack64;
  long long stride32 = 0, stride64 = 0;
  // estimate scratch
  DevBuf<double2> y_scr, h_scr;
  DevBuf<double> lp_scr, proba_scr, m_scr, s_scr;
  DevBuf<float> w_scr, acc_scr;
  DevBuf<long long> lab_scr;
  // FP16 two-term split tables (qce_estimate_h2.hip)
  DevBuf<char> pack16;
  DevBuf<float> sinv;
  long long cstride16 = 0;
  double y_scale = 1.0;
  DevBuf<double> sp_m, sp_s;
  DevBuf<float> sp_a;
  DevBuf<int> yflag;
  // FP64 fused-kernel tables (qce_estimate_f64.hip) and its cut-tile scratch
  DevBuf<char> pack_f64;
  int f64_g3 = 0;  // pack_f64 holds the 3M layout (k_est_all_f64g)
  int f64_active = 0;  // the last dense prepare packed FP64 tables: 'all' / partial run k_est_all_f64
  DevBuf<char> pack_ws;
  int f64_wide = 0;    // ... or, beyond padded 128, the two-pass FP64 path (qce_wsum_f64.hip)
  int pack64_valid = 0;  // pack64 (the k_lp_f64 table) built without pack32
  DevBuf<double> fp_m, fp_s, fp_a;
  DevBuf<double> part_a64;  // FP64 partial accumulator behind the f32 qce_estimate_partial
  DevBuf<double> fp_pack;   // host-I/O staging of qce_estimate_partial_shifted
  DevBuf<double> w64_scr;   // FP64 selection weights (selective modes)
  DevBuf<double> shift_scr;  // one double: staged K-shard shift / cconst max
  DevBuf<double2> WT;       // transposed filters W_k^T for the FP64 selective-mode kernel (built lazily)
  int wt_valid = 0;
  int cu_count = 256;
  int reserve_cus = 0;  // QCE_OPT_RESERVE_CUS: CUs the persistent grids leave to a concurrent communication stream
  int reserve_set = 0;  // the caller set QCE_OPT_RESERVE_CUS (a K-shard step then keeps the caller's value)
  int sched_cus() const { return cu_count - reserve_cus > 8 ? cu_count - reserve_cus : 8; }
  // dimensions beyond the fused kernels' 256 (qce_big.hip): GEMM-based FP64 path
  int big = 0;
  DevBuf<double2> big_ws, big_d;  // stacked transposed filters (N x K x M); per-chunk intermediate
  int big_ws_valid = 0;
  // Fourier-domain path for (block-)circulant mixtures (qce_fft.hip): structure found at creation
  int fft_n1 = 0, fft_n2 = 0;
  int fft_active = 0;   // the last prepare took the Fourier path (dense tables computed lazily)
  int dense_valid = 0;  // dense tables match the last prepare
  DevBuf<double> f_ceig, f_rinvT, f_cprime, f_wT, f_gain;
  DevBuf<double2> f_col0, f_mspec, f_uT, f_bT;
  DevBuf<int> f_bad;
  DevBuf<double> f_pr, f_pur, f_pui, f_pc, f_pw, f_pbr, f_pbi;  // qce_fft_mfma.hip tables
  int fft_mfma = 0;                                            // the MFMA kernel serves 'all' / partial
  int fft_chunk = 1;  // N = 128, 256: k_fft_chunk / k_fft_chunk_hm (fragment-order tables); 0: k_fft_mfma (QCE_FFT_CHUNK=0)
  // host-I/O pipeline of qce_estimate: two pinned slots per direction, copy-in / copy-out streams
  struct {
    double2* pin_y[2] = {nullptr, nullptr};
    double2* pin_h[2] = {nullptr, nullptr};
    size_t cap_y = 0, cap_h = 0;  // elements per slot
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_c[2] = {nullptr, nullptr}, ev_out[2] = {nullptr, nullptr};
  } hp;
  // arguments of the last prepare (replayed for the dense tables qce_get_tables returns)
  struct {
    int M = 0, quant_kind = 0, n_levels = 0;
    double snr_db = 0.0, n_bits = 1.0;
    std::vector<double> thr, lab;
  } last;
};

// Internal entry points of qce_capi.hip used by qce_kshard.hip (C++ linkage: not part of the ABI).
int qce_set_error(int code, const std::string& msg);  // sets qce_last_error() and returns code
// h_b = sum_k w[b][k] (W_k y_b + b_k), w (B x K) FP64 selection weights on the device (dense or Fourier path)
int qce_weighted_estimate(qce_model* m, const double2* y, long long B, const double* w, double2* h, hipStream_t st);

// qce_big.hip: the GEMM-based FP64 path for N or M in (256, QCE_BIG_MAX]
#define QCE_BIG_MAX 4096
int qce_big_lp(qce_model* m, const double2* y, long long B, double* lp, hipStream_t st);
int qce_big_proba(qce_model* m, long long B, hipStream_t st);
int qce_big_wsum(qce_model* m, const double2* y, long long B, const double* w, double2* out, long long ldo,
                 hipStream_t st);
int qce_big_partial(qce_model* m, const double2* y, long long B, int wmode, double* om, double* os, double* oa,
                    double* pk, const double* shift, hipStream_t st);
