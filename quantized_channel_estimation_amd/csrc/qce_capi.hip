// C ABI of libqce.so (declared in include/qce.h): model lifetime, per-SNR prepare and the
// estimate entry points, orchestrating the kernels of qce_prepare.hip / qce_estimate.hip on one
// HIP stream per model.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/qce.h"
#include "qce_common.h"
#include "qce_kernels.h"
#include "qce_model.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return fail(QCE_EHIP, std::string(#expr) + " failed: " + hipGetErrorString(e_));             \
  } while (0)

int pad_dim(int v) {
  if (v <= 16) return 16;
  if (v <= 32) return 32;
  if (v <= 64) return 64;
  if (v <= 128) return 128;
  if (v <= 256) return 256;
  return -1;
}

}  // namespace

int qce_set_error(int code, const std::string& msg) { return fail(code, msg); }

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

hipStream_t pick_stream(qce_model* m, void* stream) { return stream ? (hipStream_t)stream : m->stream; }

QceEstArgs est_args(qce_model* m, const double2* y, long long B) {
  QceEstArgs a;
  a.B = B;
  a.M = m->M;
  a.N = m->N;
  a.K = m->K;
  a.MP = m->MP;
  a.NP = m->NP;
  a.has_mean = m->has_mean;
  a.y = y;
  a.pack32 = m->pack32.p;
  a.stride32 = m->stride32;
  a.pack64 = m->pack64.p;
  a.stride64 = m->stride64;
  a.cconst = m->cconst.p;
  return a;
}

// stage host input (io == HOST) or use the device pointer directly
int stage_input(qce_model* m, const double* y, long long B, int io, hipStream_t st, const double2** dy) {
  if (io == QCE_IO_DEVICE) {
    *dy = reinterpret_cast<const double2*>(y);
    return QCE_OK;
  }
  HIPCHK(m->y_scr.ensure((size_t)B * m->M));
  HIPCHK(hipMemcpyAsync(m->y_scr.p, y, sizeof(double2) * (size_t)B * m->M, hipMemcpyHostToDevice, st));
  *dy = m->y_scr.p;
  return QCE_OK;
}

int ensure_packs(qce_model* m, hipStream_t st) {
  if (m->packs_valid) return QCE_OK;
  QcePrepareArgs p = m->pack_args;
  if (m->pack64_valid) p.pack64 = nullptr;
  HIPCHK(qce_launch_pack_selective(p, st));
  m->packs_valid = 1;
  m->pack64_valid = 1;
  return QCE_OK;
}

// the FP64 log-prob table alone (k_lp_f64), for the two-pass FP64 'all' path
int ensure_pack64(qce_model* m, hipStream_t st) {
  if (m->packs_valid || m->pack64_valid) return QCE_OK;
  QcePrepareArgs p = m->pack_args;
  p.pack32 = nullptr;
  HIPCHK(qce_launch_pack_selective(p, st));
  m->pack64_valid = 1;
  return QCE_OK;
}

bool use_h2() {
  const char* e = getenv("QCE_KERNEL");
  return !(e && strcmp(e, "f32") == 0);
}

#ifdef QCE_STAMPS
unsigned long long* g_f64_stamps = nullptr;  // diagnostic build: segment cycles of the last FP64 launch
long long g_f64_stamp_records = 0;
#endif

// Arithmetic of the dense 'all' / partial path for this model: the model option, overridden by
// QCE_KERNEL=f64 | h2 | f32 (A/B runs).
bool want_f64(const qce_model* m) {
  const char* e = getenv("QCE_KERNEL");
  if (e && strcmp(e, "f64") == 0) return true;
  if (e && (strcmp(e, "h2") == 0 || strcmp(e, "f32") == 0)) return false;
  return m->precision == QCE_PRECISION_F64;
}

// 'all' mode in FP64 (qce_estimate_f64.hip): whole tiles data-parallel over one resident workgroup
// per CU, the remaining tiles' (tile, component) items dealt out stream-K; final h, or the FP64
// (m, s, acc) partial when h == nullptr (K-shard path)
int run_f64(qce_model* m, const double2* dy, long long B, double2* h, double* om, double* os, double* oa,
            hipStream_t st, double* pk = nullptr, const double* shift = nullptr) {
  const long long TS = m->f64_g3 == 2 ? 64LL : (m->f64_g3 ? 16LL * qce_f64g_waves() : qce_f64_tile(m->MP, m->NP));
  const long long tiles = (B + TS - 1) / TS;
  // one 8-wave workgroup per CU (its ring / y tile fills the LDS), or two 4-wave ones (3M kernel built with 4 waves)
  long long slots = (long long)m->sched_cus() * (m->f64_g3 == 1 ? 8 / qce_f64g_waves() : 1);
  const char* e = getenv("QCE_WORKGROUPS");
  if (e && atoll(e) > 0) slots = atoll(e);
  long long nwg, R, L;
  if (tiles >= slots) {
    nwg = slots;
    R = tiles / slots;
    L = ((tiles - R * slots) * m->K + nwg - 1) / nwg;
  } else {
    R = 0;
    L = (tiles * m->K + slots - 1) / slots;
    if (L < 1) L = 1;
    nwg = (tiles * m->K + L - 1) / L;
  }
  QceF64Args a;
  a.B = B;
  a.M = m->M;
  a.N = m->N;
  a.K = m->K;
  a.MP = m->MP;
  a.NP = m->NP;
  a.has_mean = m->has_mean;
  a.nwg = (int)nwg;
  a.R = (int)R;
  a.L = L;
  a.y = dy;
  a.pack = m->pack_f64.p;
  a.cconst = m->cconst.p;
  a.h = h;
  a.om = om;
  a.os = os;
  a.oa = oa;
  HIPCHK(m->fp_m.ensure((size_t)nwg * 2 * TS));
  HIPCHK(m->fp_s.ensure((size_t)nwg * 2 * TS));
  HIPCHK(m->fp_a.ensure((size_t)nwg * 2 * TS * 2 * m->N));
  a.pm = m->fp_m.p;
  a.ps = m->fp_s.p;
  a.pa = m->fp_a.p;
  a.pk = pk;
  a.shift = shift;
  {
    const char* wv = getenv("QCE_F64_WAVES");  // 8 (default): two waves per SIMD where M, N <= 64
    a.waves = (wv && atoi(wv) == 4) ? 4 : 8;
  }
  a.g3 = m->f64_g3;
  if (a.g3) a.waves = qce_f64g_waves();
#ifdef QCE_STAMPS
  static unsigned long long* g_stamps = nullptr;
  if (!g_stamps) HIPCHK(hipMalloc(&g_stamps, sizeof(unsigned long long) * 4096 * 8 * 8));
  HIPCHK(hipMemsetAsync(g_stamps, 0, sizeof(unsigned long long) * 4096 * 8 * 8, st));
  a.stamps = nwg <= 4096 ? g_stamps : nullptr;
  g_f64_stamps = g_stamps;
  g_f64_stamp_records = nwg * a.waves;
#endif
  HIPCHK(qce_launch_est_f64(a, h == nullptr, st));
  return QCE_OK;
}

// 'all' mode / K-shard partials in FP64 beyond padded 128 (qce_wsum_f64.hip): lp on FP64 MFMA, the weights of
// the requested output (wmode 0: proba -> h; 1: (m, s, acc); 2: shifted packed rows), the weighted filter sum
int run_wide(qce_model* m, const double2* dy, long long B, int wmode, double2* h, double* om, double* os, double* oa,
             double* pk, const double* shift, hipStream_t st) {
  const size_t BK = (size_t)B * m->K;
  HIPCHK(m->lp_scr.ensure(BK));
  HIPCHK(m->w64_scr.ensure(BK));
  if (int rc = ensure_pack64(m, st)) return rc;
  QceEstArgs a = est_args(m, dy, B);
  HIPCHK(qce_launch_lp(a, m->lp_scr.p, st));
  HIPCHK(qce_launch_wsum_weights(B, m->K, m->lp_scr.p, wmode, shift, m->w64_scr.p, om, os, pk, 2LL * m->N + 2, st));
  QceWsumArgs w;
  w.B = B;
  w.M = m->M;
  w.N = m->N;
  w.K = m->K;
  w.MP = m->MP;
  w.NP = m->NP;
  w.has_mean = m->has_mean;
  w.y = dy;
  w.pack = m->pack_ws.p;
  w.wT = m->w64_scr.p;
  if (wmode == 0) {
    w.out = h;
    w.ostride = m->N;
    w.ooff = 0;
  } else if (wmode == 1) {
    w.out = reinterpret_cast<double2*>(oa);
    w.ostride = m->N;
    w.ooff = 0;
  } else {
    w.out = reinterpret_cast<double2*>(pk);
    w.ostride = m->N + 1;
    w.ooff = 1;
  }
  HIPCHK(qce_launch_wsum(w, st));
  return QCE_OK;
}

int run_h2x(qce_model* m, const double2* dy, long long B, double2* h, double* om, double* os, float* oa,
            hipStream_t st);

// 'all' mode on the FP16 split kernel, stream-K scheduled over the resident workgroups: final h,
// or the (m, s, acc) partial when h == nullptr (K-shard path)

int run_h2(qce_model* m, const double2* dy, long long B, double2* h, double* om, double* os, float* oa,
           hipStream_t st) {
  if (qce_h2x_shape(m->MP, m->NP)) return run_h2x(m, dy, B, h, om, os, oa, st);
  const long long tiles = (B + 255) / 256;
  long long slots = (long long)m->sched_cus() * qce_h2_blocks_per_cu(m->MP, m->NP, m->has_mean);
  const char* e = getenv("QCE_WORKGROUPS");
  if (e && atoll(e) > 0) slots = atoll(e);
  // data-parallel rounds of whole tiles, stream-K over the remaining tiles' (tile, component) items
  long long nwg, R, L;
  if (tiles >= slots) {
    nwg = slots;
    R = tiles / slots;
    const long long tail_items = (tiles - R * slots) * m->K;
    L = (tail_items + nwg - 1) / nwg;
  } else {
    R = 0;
    L = (tiles * m->K + slots - 1) / slots;
    if (L < 1) L = 1;
    nwg = (tiles * m->K + L - 1) / L;
  }
  QceH2Args a;
  a.B = B;
  a.M = m->M;
  a.N = m->N;
  a.K = m->K;
  a.MP = m->MP;
  a.NP = m->NP;
  a.has_mean = m->has_mean;
  a.nwg = (int)nwg;
  a.R = (int)R;
  a.L = L;
  a.y_scale = m->y_scale;
  a.y = dy;
  a.pack = m->pack16.p;
  a.cstride = m->cstride16;
  a.sinv = m->sinv.p;
  a.cconst = m->cconst.p;
  a.h = h;
  a.om = om;
  a.os = os;
  a.oa = oa;
  HIPCHK(m->sp_m.ensure((size_t)nwg * 2 * 256));
  HIPCHK(m->sp_s.ensure((size_t)nwg * 2 * 256));
  HIPCHK(m->sp_a.ensure((size_t)nwg * 2 * 256 * 2 * m->N));
  HIPCHK(m->yflag.ensure(1));
  a.yflag = m->yflag.p;
  a.pm = m->sp_m.p;
  a.ps = m->sp_s.p;
  a.pa = m->sp_a.p;
  HIPCHK(qce_launch_est_h2(a, h == nullptr, st));
  return QCE_OK;
}

// 'all' mode for the large padded shapes (qce_estimate_h2x.hip): 128-sample tiles x K splits x
// row chunks, split records merged by k_merge_splits
int run_h2x(qce_model* m, const double2* dy, long long B, double2* h, double* om, double* os, float* oa,
            hipStream_t st) {
  const long long tiles = (B + qce_h2x_tile() - 1) / qce_h2x_tile();
  const long long nrc = qce_h2x_row_chunks(m->MP, m->NP);
  const long long slots = m->sched_cus();  // one 128 KB-LDS workgroup per CU
  int ksplit = 1;
  double best = 0.0;
  for (int s = 1; s <= 8 && s <= m->K; ++s) {  // fill the chip: tiles*s*nrc over whole waves of workgroups
    const long long wg = tiles * s * nrc;
    const double eff = (double)wg / (double)(slots * ((wg + slots - 1) / slots));
    if (eff > best + 0.02) {
      best = eff;
      ksplit = s;
    }
  }
  const char* e = getenv("QCE_KSPLIT");
  if (e && atoi(e) > 0) ksplit = atoi(e) < m->K ? atoi(e) : m->K;
  QceH2XArgs a;
  a.B = B;
  a.M = m->M;
  a.N = m->N;
  a.K = m->K;
  a.MP = m->MP;
  a.NP = m->NP;
  a.has_mean = m->has_mean;
  a.y_scale = m->y_scale;
  HIPCHK(m->yflag.ensure(1));
  a.yflag = m->yflag.p;
  a.y = dy;
  a.pack = m->pack16.p;
  a.cstride = m->cstride16;
  a.sinv = m->sinv.p;
  a.cconst = m->cconst.p;
  a.h = h;
  a.om = om;
  a.os = os;
  a.oa = oa;
  a.rm = a.rs = nullptr;
  a.ra = nullptr;
  if (ksplit > 1) {
    HIPCHK(m->sp_m.ensure((size_t)ksplit * B));
    HIPCHK(m->sp_s.ensure((size_t)ksplit * B));
    HIPCHK(m->sp_a.ensure((size_t)ksplit * B * 2 * m->N));
    a.rm = m->sp_m.p;
    a.rs = m->sp_s.p;
    a.ra = m->sp_a.p;
  }
  HIPCHK(qce_launch_est_h2x(a, ksplit, h == nullptr, st));
  return QCE_OK;
}

bool fft_enabled() {
  const char* e = getenv("QCE_FFT");
  return !(e && e[0] == '0');
}

// Is every C_k (block-)circulant for some power-of-two split N = n1 n2?  (circulant fit:
// gmm_cplx_bussgang.py:104-117, block-circulant fit: :118-133).  Sets fft_n1/fft_n2 and keeps the
// eigenvalues, first columns and mean spectra for the per-SNR Fourier prepare.
hipError_t detect_structure(qce_model* m) {
  const int K = m->K, N = m->N;
  m->fft_n1 = m->fft_n2 = 0;
  if (N > 256 || !qce_fft_pow2(N) || N < 4 || qce_fft_tile(N, K) == 0 || K > 256) return hipSuccess;
  hipError_t e;
  if ((e = m->f_ceig.ensure((size_t)K * N)) != hipSuccess) return e;
  if ((e = m->f_col0.ensure((size_t)K * N)) != hipSuccess) return e;
  if ((e = m->f_mspec.ensure((size_t)K * N)) != hipSuccess) return e;
  if ((e = m->f_bad.ensure(K)) != hipSuccess) return e;
  std::vector<int> bad(K);
  for (int n1 = 1; n1 < N; n1 *= 2) {
    const int n2 = N / n1;
    if ((e = qce_launch_fft_struct(K, N, n1, n2, 1e-10, m->covs.p, m->means.p, m->f_ceig.p, m->f_col0.p,
                                   m->f_mspec.p, m->f_bad.p, m->stream)) != hipSuccess)
      return e;
    if ((e = hipMemcpyAsync(bad.data(), m->f_bad.p, sizeof(int) * K, hipMemcpyDeviceToHost, m->stream)) != hipSuccess)
      return e;
    if ((e = hipStreamSynchronize(m->stream)) != hipSuccess) return e;
    bool ok = true;
    for (int k = 0; k < K; ++k) ok = ok && bad[k] == 0;
    if (ok) {
      m->fft_n1 = n1;
      m->fft_n2 = n2;
      return hipSuccess;
    }
  }
  m->f_ceig.release();
  m->f_col0.release();
  m->f_mspec.release();
  return hipSuccess;
}

QceFftEstArgs fft_args(qce_model* m, const double2* y, long long B) {
  QceFftEstArgs a;
  a.B = B;
  a.N = m->N;
  a.n1 = m->fft_n1;
  a.n2 = m->fft_n2;
  a.K = m->K;
  a.has_mean = m->has_mean;
  a.y = y;
  a.rinvT = m->f_rinvT.p;
  a.uT = m->f_uT.p;
  a.cprime = m->f_cprime.p;
  a.wT = m->f_wT.p;
  a.bT = m->f_bT.p;
  a.wts = nullptr;
  a.h = nullptr;
  a.lp = nullptr;
  a.om = a.os = nullptr;
  a.oa = nullptr;
  a.Kp = qce_fft_kpad(m->K);
  a.pr = m->f_pr.p;
  a.pur = m->f_pur.p;
  a.pui = m->f_pui.p;
  a.pc = m->f_pc.p;
  a.pw = m->f_pw.p;
  a.pbr = m->f_pbr.p;
  a.pbi = m->f_pbi.p;
  a.cu = m->sched_cus();
  a.chunk = m->fft_chunk;
  return a;
}

// QCE_FFT_KERNEL=lds keeps 'all' / partial on the LDS-tiled FP64 kernel of qce_fft.hip (A/B runs)
bool fft_mfma_enabled() {
  const char* e = getenv("QCE_FFT_KERNEL");
  return !(e && strcmp(e, "lds") == 0);
}

// Uniform quantiser step get_uniform_quant_step (uniform_quantizer.py:44-45) with standard_quantization_step
// (:6-23): J. Max's table for n_bits <= 8, the asymptote 4 sqrt(b) 2^-b of Hui & Neuhoff beyond it (:15-21).
double uniform_step(double snr_db, int nb) {
  static const double tbl[9] = {0, 1.596, 0.9957, 0.5860, 0.3352, 0.1881, 0.1041, 0.0569, 0.0308};
  const double std_step = nb <= 8 ? tbl[nb] : 4.0 * sqrt((double)nb) * pow(2.0, -nb);
  return sqrt((1.0 + pow(10.0, -snr_db / 10.0)) / 2.0) * std_step;
}

// The Cholesky status of a prepare is copied to pinned host memory behind the prepare's kernels and read only
// when a call synchronises anyway (host I/O, qce_synchronize, qce_get_tables): a prepare costs no host round
// trip.  A failed prepare surfaces as QCE_ECHOL there (device-I/O estimates in between compute on NaN tables).
int post_status(qce_model* m, hipStream_t st) {
  const int K = m->K;
  if (!m->status_host) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&m->status_host), sizeof(int) * K, hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&m->status_ev, hipEventDisableTiming));
  }
  HIPCHK(hipMemcpyAsync(m->status_host, m->status.p, sizeof(int) * K, hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(m->status_ev, st));
  m->status_pending = 1;
  return QCE_OK;
}

int check_status(qce_model* m, bool block) {
  if (!m->status_pending) return QCE_OK;
  if (!block && hipEventQuery(m->status_ev) == hipErrorNotReady) return QCE_OK;
  HIPCHK(hipEventSynchronize(m->status_ev));
  m->status_pending = 0;
  for (int k = 0; k < m->K; ++k)
    if (m->status_host[k]) {
      m->prepared = 0;
      return fail(QCE_ECHOL,
                  "Fitting the mixture model failed because some components have ill-defined empirical covariance "
                  "(for instance caused by singleton or collapsed samples). Try to decrease the number of "
                  "components, or increase reg_covar.");
    }
  return QCE_OK;
}

#define HOST_SYNC_CHECK(m, st)                      \
  do {                                              \
    HIPCHK(hipStreamSynchronize(st));               \
    if (int rc_ = check_status((m), true)) return rc_; \
  } while (0)

int check_model(qce_model* m, bool need_prepared) {
  if (!m) return fail(QCE_EARG, "null model");
  if (need_prepared && m->prepared)
    if (int rc = check_status(m, false)) return rc;  // a failure already known surfaces at once
  if (need_prepared && !m->prepared) return fail(QCE_ESTATE, "qce_prepare has not been called on this model");
  return QCE_OK;
}

}  // namespace

extern "C" {

int qce_version(void) { return 200; }

const char* qce_last_error(void) { return g_err.c_str(); }

int qce_device_count(int* count) {
  if (!count) return fail(QCE_EARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return QCE_OK;
}

int qce_model_create(int K, int N, const double* means_cplx, const double* covs_cplx, const double* weights,
                     int device, qce_model** out) {
  if (!out || !covs_cplx || !weights) return fail(QCE_EARG, "null argument");
  *out = nullptr;
  if (K <= 0 || N <= 0) return fail(QCE_EARG, "K and N must be positive");
  if (N > QCE_BIG_MAX) return fail(QCE_ENOTIMPL, "N > " + std::to_string(QCE_BIG_MAX) + " is not covered");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(QCE_EHIP, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(QCE_EARG, "device index out of range");
  DeviceGuard g(device);
  qce_model* m = new qce_model();
  m->K = K;
  m->N = N;
  m->device = device;
  m->weights.assign(weights, weights + K);
  std::vector<double> logw(K);
  for (int k = 0; k < K; ++k) logw[k] = log(weights[k]);
  std::vector<double> mz((size_t)2 * K * N, 0.0);
  if (means_cplx) {
    memcpy(mz.data(), means_cplx, sizeof(double) * 2 * (size_t)K * N);
    for (double v : mz)
      if (v != 0.0) {
        m->has_mean = 1;
        break;
      }
  }
  if (hipDeviceGetAttribute(&m->cu_count, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      m->cu_count < 1)
    m->cu_count = 256;
  hipError_t e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = m->means.ensure((size_t)K * N);
  if (e == hipSuccess) e = m->covs.ensure((size_t)K * N * N);
  if (e == hipSuccess) e = m->logw.ensure(K);
  if (e == hipSuccess) e = hipMemcpy(m->means.p, mz.data(), sizeof(double2) * (size_t)K * N, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(m->covs.p, covs_cplx, sizeof(double2) * (size_t)K * N * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(m->logw.p, logw.data(), sizeof(double) * K, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    qce_model_destroy(m);
    return fail(QCE_EHIP, std::string("model allocation failed: ") + hipGetErrorString(e));
  }
  if ((e = detect_structure(m)) != hipSuccess) {
    qce_model_destroy(m);
    return fail(QCE_EHIP, std::string("structure detection failed: ") + hipGetErrorString(e));
  }
  *out = m;
  return QCE_OK;
}

int qce_model_set_params(qce_model* m, const double* means_cplx, const double* covs_cplx, const double* weights) {
  if (!m || !covs_cplx || !weights) return fail(QCE_EARG, "null argument");
  DeviceGuard g(m->device);
  const int K = m->K, N = m->N;
  HIPCHK(hipStreamSynchronize(m->stream));
  m->weights.assign(weights, weights + K);
  std::vector<double> logw(K);
  for (int k = 0; k < K; ++k) logw[k] = log(weights[k]);
  std::vector<double> mz((size_t)2 * K * N, 0.0);
  m->has_mean = 0;
  if (means_cplx) {
    memcpy(mz.data(), means_cplx, sizeof(double) * 2 * (size_t)K * N);
    for (double v : mz)
      if (v != 0.0) {
        m->has_mean = 1;
        break;
      }
  }
  HIPCHK(hipMemcpyAsync(m->means.p, mz.data(), sizeof(double2) * (size_t)K * N, hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipMemcpyAsync(m->covs.p, covs_cplx, sizeof(double2) * (size_t)K * N * N, hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipMemcpyAsync(m->logw.p, logw.data(), sizeof(double) * K, hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  m->prepared = 0;
  HIPCHK(detect_structure(m));
  return QCE_OK;
}

int qce_model_destroy(qce_model* m) {
  if (!m) return QCE_OK;
  DeviceGuard g(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  for (auto* b : {&m->means, &m->covs, &m->A, &m->Cy, &m->Cr, &m->Lw, &m->Linv, &m->Aeff, &m->work, &m->V, &m->W,
                  &m->means_y, &m->q0, &m->bvec, &m->y_scr, &m->h_scr})
    b->release();
  for (auto* b : {&m->logw, &m->gain, &m->cconst, &m->thr, &m->lab, &m->pack64, &m->lp_scr, &m->proba_scr,
                  &m->m_scr, &m->s_scr})
    b->release();
  m->status.release();
  if (m->status_host) (void)hipHostFree(m->status_host);
  if (m->status_ev) (void)hipEventDestroy(m->status_ev);
  m->pack32.release();
  m->w_scr.release();
  m->acc_scr.release();
  m->lab_scr.release();
  m->pack16.release();
  m->sinv.release();
  m->sp_m.release();
  m->sp_s.release();
  m->sp_a.release();
  m->yflag.release();
  m->pack_f64.release();
  m->pack_ws.release();
  for (auto* b : {&m->fp_m, &m->fp_s, &m->fp_a, &m->part_a64, &m->fp_pack, &m->w64_scr, &m->shift_scr})
    b->release();
  m->WT.release();
  m->big_ws.release();
  m->big_d.release();
  for (auto* b : {&m->f_ceig, &m->f_rinvT, &m->f_cprime, &m->f_wT, &m->f_gain}) b->release();
  for (auto* b : {&m->f_col0, &m->f_mspec, &m->f_uT, &m->f_bT}) b->release();
  m->f_bad.release();
  for (int i = 0; i < 2; ++i) {
    if (m->hp.pin_y[i]) (void)hipHostFree(m->hp.pin_y[i]);
    if (m->hp.pin_h[i]) (void)hipHostFree(m->hp.pin_h[i]);
    for (hipEvent_t ev : {m->hp.ev_in[i], m->hp.ev_c[i], m->hp.ev_out[i]})
      if (ev) (void)hipEventDestroy(ev);
  }
  for (hipStream_t hs : {m->hp.s_in, m->hp.s_out})
    if (hs) {
      (void)hipStreamSynchronize(hs);
      (void)hipStreamDestroy(hs);
    }
  if (m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
  return QCE_OK;
}

static int prepare_impl(qce_model* m, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                        const double* thresholds, const double* labels, int n_levels, void* stream, bool allow_fft);

int qce_prepare(qce_model* m, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                const double* thresholds, const double* labels, int n_levels, void* stream) {
  return prepare_impl(m, A, M, snr_db, n_bits, quant_kind, thresholds, labels, n_levels, stream, true);
}

}  // extern "C"

namespace {
// The dense tables of a prepare that took the Fourier path, computed when first asked for
// (qce_get_tables: the reference's gm state mirror); the Fourier tables stay active.
int ensure_dense(qce_model* m, void* stream = nullptr) {
  if (!m->fft_active || m->dense_valid) return QCE_OK;
  const int rc = prepare_impl(m, nullptr, m->last.M, m->last.snr_db, m->last.n_bits, m->last.quant_kind,
                              m->last.thr.empty() ? nullptr : m->last.thr.data(),
                              m->last.lab.empty() ? nullptr : m->last.lab.data(), m->last.n_levels, stream, false);
  if (rc) return rc;
  m->fft_active = 1;
  m->dense_valid = 1;
  return QCE_OK;
}
}  // namespace

extern "C" {

static int prepare_impl(qce_model* m, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                        const double* thresholds, const double* labels, int n_levels, void* stream, bool allow_fft) {
  int rc = check_model(m, false);
  if (rc) return rc;
  const int N = m->N, K = m->K;
  if (!A) M = N;
  if (M <= 0) return fail(QCE_EARG, "M must be positive");
  if (M > QCE_BIG_MAX) return fail(QCE_ENOTIMPL, "M > " + std::to_string(QCE_BIG_MAX) + " is not covered");
  int kind;
  int nb = 0;
  if (n_bits == 1.0) {
    kind = 0;
  } else if (isinf(n_bits) && n_bits > 0) {
    kind = 2;
  } else {
    if (!(n_bits >= 2.0 && n_bits <= (double)QCE_MAX_UNIFORM_BITS) || n_bits != floor(n_bits))
      return fail(QCE_ENOTIMPL, "n_bits must be 1.." + std::to_string(QCE_MAX_UNIFORM_BITS) + " or inf");
    kind = 1;
    nb = (int)n_bits;
    if (quant_kind == QCE_QUANT_LLOYD && nb > 8) return fail(QCE_ENOTIMPL, "lloyd quantiser tables cover n_bits <= 8");
  }
  if (kind == 1 && quant_kind == QCE_QUANT_LLOYD) {
    if (!thresholds || !labels || n_levels != (1 << nb))
      return fail(QCE_EARG, "lloyd quantiser needs 2^b labels and 2^b-1 thresholds");
  }
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  bool idA = (A == nullptr);
  if (A && M == N) {  // an explicit identity is the same observation model
    idA = true;
    for (int i = 0; i < M && idA; ++i)
      for (int j = 0; j < N; ++j) {
        const double re = A[2 * ((size_t)i * N + j)], im = A[2 * ((size_t)i * N + j) + 1];
        if (im != 0.0 || re != (i == j ? 1.0 : 0.0)) {
          idA = false;
          break;
        }
      }
  }
  m->last.M = M;
  m->last.snr_db = snr_db;
  m->last.n_bits = n_bits;
  m->last.quant_kind = quant_kind;
  m->last.n_levels = n_levels;
  if (allow_fft) {
    m->last.thr.assign(thresholds && kind == 1 ? thresholds : nullptr,
                       thresholds && kind == 1 ? thresholds + (n_levels > 0 ? n_levels - 1 : 0) : nullptr);
    m->last.lab.assign(labels && kind == 1 ? labels : nullptr, labels && kind == 1 ? labels + n_levels : nullptr);
  }
  if (allow_fft && idA && m->fft_n1 > 0 && fft_enabled() && !m->beta_first) {
    // Fourier-domain prepare (qce_fft.hip): per-bin tables only
    HIPCHK(m->f_rinvT.ensure((size_t)N * K));
    HIPCHK(m->f_uT.ensure((size_t)N * K));
    HIPCHK(m->f_cprime.ensure(K));
    HIPCHK(m->f_wT.ensure((size_t)K * N));
    HIPCHK(m->f_bT.ensure((size_t)K * N));
    HIPCHK(m->f_gain.ensure(K));
    HIPCHK(m->status.ensure(K));
    HIPCHK(m->thr.ensure(256));
    HIPCHK(m->lab.ensure(256));
    double delta = 0.0;
    if (kind == 1 && quant_kind == QCE_QUANT_UNIFORM) delta = uniform_step(snr_db, nb);
    if (kind == 1 && quant_kind == QCE_QUANT_LLOYD) {
      HIPCHK(hipMemcpyAsync(m->thr.p, thresholds, sizeof(double) * (n_levels - 1), hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(m->lab.p, labels, sizeof(double) * n_levels, hipMemcpyHostToDevice, st));
    }
    QceFftPrepArgs fa;
    fa.N = N;
    fa.n1 = m->fft_n1;
    fa.n2 = m->fft_n2;
    fa.K = K;
    fa.s2 = pow(10.0, -snr_db / 10.0);
    fa.kind = kind;
    fa.n_bits = nb;
    fa.quant_kind = quant_kind;
    fa.delta = delta;
    fa.thr = m->thr.p;
    fa.lab = m->lab.p;
    fa.logw = m->logw.p;
    fa.ceig = m->f_ceig.p;
    fa.col0 = m->f_col0.p;
    fa.mspec = m->f_mspec.p;
    fa.rinvT = m->f_rinvT.p;
    fa.uT = m->f_uT.p;
    fa.cprime = m->f_cprime.p;
    fa.wT = m->f_wT.p;
    fa.bT = m->f_bT.p;
    fa.gain = m->f_gain.p;
    fa.status = m->status.p;
    HIPCHK(qce_launch_fft_prep(fa, st));
    m->fft_mfma = 0;
    {
      const char* e = getenv("QCE_FFT_CHUNK");  // read per prepare: the table order and the kernel go together
      m->fft_chunk = !(e && e[0] == '0');
    }
    if (qce_fft_mfma_shape(N) && fft_mfma_enabled()) {
      const size_t KpN = (size_t)qce_fft_kpad(K) * N;
      HIPCHK(m->f_pr.ensure(KpN));
      HIPCHK(m->f_pc.ensure((size_t)qce_fft_kpad(K)));
      HIPCHK(m->f_pw.ensure(KpN));
      if (m->has_mean) {
        HIPCHK(m->f_pur.ensure(KpN));
        HIPCHK(m->f_pui.ensure(KpN));
        HIPCHK(m->f_pbr.ensure(KpN));
        HIPCHK(m->f_pbi.ensure(KpN));
      }
      QceFftEstArgs pa = fft_args(m, nullptr, 0);
      HIPCHK(qce_launch_fft_pack(pa, m->f_rinvT.p, m->f_uT.p, m->f_cprime.p, m->f_wT.p, m->f_bT.p, st));
      m->fft_mfma = 1;
    }
    if ((rc = post_status(m, st))) return rc;
    m->M = N;
    m->fft_active = 1;
    m->dense_valid = 0;
    m->prepared = 1;
    return QCE_OK;
  }
  m->fft_active = 0;
  m->dense_valid = 1;
  const size_t KMM = (size_t)K * M * M, KMN = (size_t)K * M * N;
  HIPCHK(m->A.ensure((size_t)M * N));
  HIPCHK(m->Cy.ensure(KMM));
  HIPCHK(m->Cr.ensure(KMM));
  HIPCHK(m->Lw.ensure(KMM));
  HIPCHK(m->Linv.ensure(KMM));
  HIPCHK(m->Aeff.ensure(KMN));
  HIPCHK(m->work.ensure(KMN));
  HIPCHK(m->V.ensure(KMN));
  HIPCHK(m->W.ensure(KMN));
  HIPCHK(m->means_y.ensure((size_t)K * M));
  HIPCHK(m->q0.ensure((size_t)K * M));
  HIPCHK(m->bvec.ensure((size_t)K * N));
  if (m->has_mean) {
    m->q0_zeroed = m->bvec_zeroed = 0;  // the prepare writes them
  } else if (m->q0_zeroed < (size_t)K * M || m->bvec_zeroed < (size_t)K * N) {  // zero-mean: q0 = 0, b = 0 at every SNR
    m->q0_zeroed = m->bvec_zeroed = 0;
    HIPCHK(hipMemsetAsync(m->q0.p, 0, sizeof(double2) * m->q0.n, st));
    HIPCHK(hipMemsetAsync(m->bvec.p, 0, sizeof(double2) * m->bvec.n, st));
    m->q0_zeroed = m->q0.n;
    m->bvec_zeroed = m->bvec.n;
  }
  HIPCHK(m->gain.ensure((size_t)K * M));
  HIPCHK(m->cconst.ensure(K));
  HIPCHK(m->status.ensure(K));
  HIPCHK(m->thr.ensure(256));
  HIPCHK(m->lab.ensure(256));
  m->big = (pad_dim(M) < 0 || pad_dim(N) < 0);
  m->big_ws_valid = 0;
  int MP = m->big ? 0 : pad_dim(M), NP = m->big ? 0 : pad_dim(N);
  if (!m->big && (MP > 64 || NP > 64)) {  // the chunk-streamed kernel family (qce_estimate_h2x.hip) starts at 64
    MP = MP < 64 ? 64 : MP;
    NP = NP < 64 ? 64 : NP;
  }
  const long long s32 = m->big ? 0 : qce_pack_f32_stride(MP, NP, m->has_mean);
  const long long s64 = m->big ? 0 : qce_pack_f64_stride(MP, m->has_mean);
  HIPCHK(m->pack32.ensure((size_t)s32 * K));
  HIPCHK(m->pack64.ensure((size_t)s64 * K));
  int identityA = 0;
  if (A) {
    HIPCHK(hipMemcpyAsync(m->A.p, A, sizeof(double2) * (size_t)M * N, hipMemcpyHostToDevice, st));
    m->a_identity_n = 0;
  } else {
    if (m->a_identity_n != N) {
      std::vector<double> eye((size_t)2 * N * N, 0.0);
      for (int i = 0; i < N; ++i) eye[(size_t)2 * (i * N + i)] = 1.0;
      HIPCHK(hipMemcpyAsync(m->A.p, eye.data(), sizeof(double2) * (size_t)N * N, hipMemcpyHostToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
      m->a_identity_n = N;
    }
    identityA = 1;
  }
  if (A && M == N) {  // an explicit identity takes the same fast path (bitwise the same Cy)
    identityA = 1;
    for (int i = 0; i < M && identityA; ++i)
      for (int j = 0; j < N; ++j) {
        double re = A[2 * ((size_t)i * N + j)], im = A[2 * ((size_t)i * N + j) + 1];
        if (im != 0.0 || re != (i == j ? 1.0 : 0.0)) {
          identityA = 0;
          break;
        }
      }
  }
  double delta = 0.0;
  if (kind == 1 && quant_kind == QCE_QUANT_UNIFORM) delta = uniform_step(snr_db, nb);
  if (kind == 1 && quant_kind == QCE_QUANT_LLOYD) {
    HIPCHK(hipMemcpyAsync(m->thr.p, thresholds, sizeof(double) * (n_levels - 1), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->lab.p, labels, sizeof(double) * n_levels, hipMemcpyHostToDevice, st));
  }
  QcePrepareArgs p;
  p.K = K;
  p.N = N;
  p.M = M;
  p.MP = MP;
  p.NP = NP;
  p.has_mean = m->has_mean;
  p.identityA = identityA;
  p.kind = kind;
  p.n_bits = nb;
  p.quant_kind = quant_kind;
  p.beta_first = m->beta_first;
  p.sigma2 = pow(10.0, -snr_db / 10.0);
  p.delta = delta;
  p.thr = m->thr.p;
  p.lab = m->lab.p;
  p.A = m->A.p;
  p.covs = m->covs.p;
  p.means = m->means.p;
  p.logw = m->logw.p;
  p.Cy = m->Cy.p;
  p.Cr = m->Cr.p;
  p.Lw = m->Lw.p;
  p.Linv = m->Linv.p;
  p.Aeff = m->Aeff.p;
  p.work = m->work.p;
  p.V = m->V.p;
  p.W = m->W.p;
  p.means_y = m->means_y.p;
  p.q0 = m->q0.p;
  p.bvec = m->bvec.p;
  p.gain = m->gain.p;
  p.cconst = m->cconst.p;
  p.status = m->status.p;
  p.pack32 = m->pack32.p;
  p.stride32 = s32;
  p.pack64 = m->pack64.p;
  p.stride64 = s64;
  m->pack_args = p;
  m->packs_valid = 0;
  m->pack64_valid = 0;
  m->wt_valid = 0;
  p.pack32 = nullptr;  // selective-mode / log-prob tables are packed on first use (ensure_packs)
  p.pack64 = nullptr;
  HIPCHK(qce_launch_prepare(p, st));
  m->f64_active = !m->big && want_f64(m) && qce_f64_shape(MP, NP);
  m->f64_wide = !m->big && want_f64(m) && !m->f64_active && qce_wsum_shape(MP, NP);
  if (m->big) {
    // GEMM-based FP64 path (qce_big.hip): the dense tables are all it reads; the stacked filters on first use
  } else if (m->f64_wide) {
    // FP64 filter tables of the two-pass path; the log-prob table is packed on first use (ensure_pack64)
    HIPCHK(m->pack_ws.ensure((size_t)qce_pack_wsum_bytes(MP, NP, m->has_mean) * K));
    HIPCHK(qce_launch_pack_wsum(K, M, N, MP, NP, m->has_mean, m->W.p, m->bvec.p,
                                reinterpret_cast<double*>(m->pack_ws.p), st));
  } else if (m->f64_active) {
    // FP64 tables of the fused kernel (reference precision): 3M layout where the 3M kernel covers the shape
    m->f64_g3 = qce_f64g_shape(MP, NP) ? 1 : (qce_f64h_shape(MP, NP) ? 2 : 0);
    if (m->f64_g3 == 2) {
      HIPCHK(m->pack_f64.ensure((size_t)qce_pack_f64h_bytes(m->has_mean) * K));
      HIPCHK(qce_launch_pack_f64h(K, M, N, m->has_mean, m->Linv.p, m->W.p, m->q0.p, m->bvec.p,
                                  reinterpret_cast<double*>(m->pack_f64.p), st));
    } else if (m->f64_g3) {
      HIPCHK(m->pack_f64.ensure((size_t)qce_pack_f64g_bytes(MP, NP, m->has_mean) * K));
      HIPCHK(qce_launch_pack_f64g(K, M, N, MP, NP, m->has_mean, m->Linv.p, m->W.p, m->q0.p, m->bvec.p,
                                  reinterpret_cast<double*>(m->pack_f64.p), st));
    } else {
      HIPCHK(m->pack_f64.ensure((size_t)qce_pack_f64all_bytes(MP, NP, m->has_mean) * K));
      HIPCHK(qce_launch_pack_f64all(K, M, N, MP, NP, m->has_mean, m->Linv.p, m->W.p, m->q0.p, m->bvec.p,
                                    reinterpret_cast<double*>(m->pack_f64.p), st));
    }
  } else {
    // FP16 two-term split tables; the observation scale makes quantiser outputs exact in fp16
    // (1 bit: y sqrt(2) = +-1; uniform: y 2/delta = odd integers), folded into the slice scales
    double y_scale = 1.0;
    if (kind == 0) y_scale = sqrt(2.0);
    else if (kind == 1 && quant_kind == QCE_QUANT_UNIFORM && delta > 0.0) y_scale = 2.0 / delta;
    const long long cs16 = qce_pack_h2_stride_bytes(MP, NP, m->has_mean);
    const int nslices = (2 * MP) / 32 + (2 * NP) / 32;
    HIPCHK(m->pack16.ensure((size_t)cs16 * K + (size_t)qce_h2x_pad_bytes()));
    HIPCHK(m->sinv.ensure((size_t)nslices * K));
    HIPCHK(qce_launch_pack_h2(K, M, N, MP, NP, m->has_mean, cs16, y_scale, m->Linv.p, m->W.p, m->q0.p, m->bvec.p,
                              m->pack16.p, m->sinv.p, st));
    m->cstride16 = cs16;
    m->y_scale = y_scale;
  }
  if ((rc = post_status(m, st))) return rc;
  m->M = M;
  m->MP = MP;
  m->NP = NP;
  m->stride32 = s32;
  m->stride64 = s64;
  m->prepared = 1;
  return QCE_OK;
}

}  // extern "C"

namespace {

// memcpy split over a few host threads (pageable numpy buffer <-> pinned slot)
void par_memcpy(void* dst, const void* src, size_t bytes) {
  const size_t piece = (size_t)2 << 20;
  int nt = (int)((bytes + piece - 1) / piece);
  static const int cap = [] {  // QCE_HOST_THREADS (default 16: the CPU share of one GPU on an 8-GPU node)
    const char* v = getenv("QCE_HOST_THREADS");
    const int hw = (int)std::thread::hardware_concurrency();
    int c = v ? atoi(v) : 16;
    if (hw > 0 && c > hw) c = hw;
    return c < 1 ? 1 : c;
  }();
  if (nt > cap) nt = cap;
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  const size_t per = (bytes + nt - 1) / nt;
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) {
    const size_t o = per * t;
    if (o >= bytes) break;
    const size_t n = (o + per > bytes) ? bytes - o : per;
    th.emplace_back([=] { memcpy((char*)dst + o, (const char*)src + o, n); });
  }
  memcpy(dst, src, per < bytes ? per : bytes);
  for (auto& x : th) x.join();
}

// rows per host-pipeline chunk; 0 = one shot (QCE_HOST_PIPELINE=0, or too small a batch to split)
long long host_chunk_rows(const qce_model* m, long long B) {
  const char* e = getenv("QCE_HOST_PIPELINE");
  if (e && e[0] == '0') return 0;
  const long long width = m->M > m->N ? m->M : m->N;
  long long cap = ((long long)32 << 20) / (16 * width);  // <= 32 MB per slot and direction
  static const long long parts = [] {  // QCE_HOST_CHUNKS: chunks per batch (A/B runs; default 8)
    const char* v = getenv("QCE_HOST_CHUNKS");
    const long long n = v ? atoll(v) : 8;
    return n < 2 ? 2 : n;
  }();
  long long c = (B + parts - 1) / parts;
  if (c > cap) c = cap;
  c = (c + 255) / 256 * 256;
  if (c < 4096) c = 4096;
  return (B >= 2 * c) ? c : 0;
}

// Host memory the GPU can DMA directly: already page-locked (hipHostMalloc'ed, or registered by the caller), or
// registered here for the duration of one call (hipHostRegister pins the pages the caller's array already has:
// ~0.3 ms per 100 MB of touched memory, measured on the box, profiles/r05_hostreg_probe.json).
struct HostDma {
  void* p = nullptr;
  bool registered = false;  // registered by this call: unregistered at its end
  bool ok = false;
  HostDma(void* ptr, size_t bytes) : p(ptr) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, ptr) == hipSuccess && at.type == hipMemoryTypeHost) {
      ok = true;
      return;
    }
    (void)hipGetLastError();
    if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess) {
      ok = registered = true;
      return;
    }
    (void)hipGetLastError();  // e.g. a range overlapping another registration: the staged path takes it
  }
  ~HostDma() {
    if (registered) (void)hipHostUnregister(p);
  }
};

// row boundaries of the direct-DMA pipeline: chunks growing x4 from the first (whose upload is the only exposed
// transfer) to the middle and shrinking again (the last chunk's download is the other); an upload of 1 KB rows at
// ~56 GB/s is ~5x faster than the estimate of a row, so each upload hides behind the previous chunk's kernel
std::vector<long long> direct_chunks(long long B) {
  std::vector<long long> sz;
  const char* e0 = getenv("QCE_HOST_C0");  // first chunk's rows (A/B runs; default B / 24)
  const char* eg = getenv("QCE_HOST_GROW");  // growth factor of the chunks towards the middle (default 4)
  long long c0 = e0 ? atoll(e0) : B / 24;
  const long long grow = eg && atoll(eg) >= 1 ? atoll(eg) : 4;
  if (c0 < 4096) c0 = 4096;
  long long left = B;
  std::vector<long long> head, tail;
  for (long long c = c0; left > 0;) {
    if (left <= 2 * c) {
      head.push_back(left);
      left = 0;
      break;
    }
    head.push_back(c);
    tail.push_back(c);
    left -= 2 * c;
    c *= grow;
  }
  sz = head;
  for (auto it = tail.rbegin(); it != tail.rend(); ++it) sz.push_back(*it);
  std::vector<long long> bounds{0};
  for (long long v : sz) bounds.push_back(bounds.back() + v);
  return bounds;
}

}  // namespace

extern "C" {

int qce_host_alloc(size_t bytes, void** out) {
  if (!out) return fail(QCE_EARG, "null argument");
  *out = nullptr;
  HIPCHK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return QCE_OK;
}

int qce_host_free(void* p) {
  if (p) HIPCHK(hipHostFree(p));
  return QCE_OK;
}

namespace {
// Every return of a host-I/O pipeline, the error paths included, first waits for its copy streams: the
// caller's arrays are unregistered (HostDma) or handed back right after, and an async copy may still be using them.
struct CopyStreamsDrain {
  hipStream_t a, b;
  ~CopyStreamsDrain() {
    if (a) (void)hipStreamSynchronize(a);
    if (b) (void)hipStreamSynchronize(b);
  }
};
// estimate_host_direct could not get its whole-batch device scratch: the bounded staged pipeline takes the batch
constexpr int kDirectNoScratch = -1;
}  // namespace

// Host numpy I/O straight from / into the caller's arrays (both DMA-able, see HostDma): per chunk H2D on a copy
// stream, the estimate on the compute stream, D2H on a second copy stream -- no host copies, one sync at the end.
static int estimate_host_direct(qce_model* m, const double* y, long long B, int mode, double mode_param,
                                double* h_out, hipStream_t st) {
  auto& hp = m->hp;
  const size_t M = (size_t)m->M, N = (size_t)m->N;
  if (!hp.s_in) HIPCHK(hipStreamCreateWithFlags(&hp.s_in, hipStreamNonBlocking));
  if (!hp.s_out) HIPCHK(hipStreamCreateWithFlags(&hp.s_out, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) {
    if (!hp.ev_in[i]) HIPCHK(hipEventCreateWithFlags(&hp.ev_in[i], hipEventDisableTiming));
    if (!hp.ev_c[i]) HIPCHK(hipEventCreateWithFlags(&hp.ev_c[i], hipEventDisableTiming));
  }
  if (m->y_scr.ensure((size_t)B * M) != hipSuccess || m->h_scr.ensure((size_t)B * N) != hipSuccess) {
    (void)hipGetLastError();
    m->y_scr.release();  // the staged pipeline sizes its own (bounded) scratch
    m->h_scr.release();
    return kDirectNoScratch;
  }
  CopyStreamsDrain drain{hp.s_in, hp.s_out};
  const std::vector<long long> bd = direct_chunks(B);
  const double2* ys = reinterpret_cast<const double2*>(y);
  double2* hs = reinterpret_cast<double2*>(h_out);
  // the copy streams start behind the compute stream's earlier work (the scratch buffers' previous readers)
  HIPCHK(hipEventRecord(hp.ev_c[1], st));
  HIPCHK(hipStreamWaitEvent(hp.s_in, hp.ev_c[1], 0));
  int rc = QCE_OK;
  for (size_t i = 0; i + 1 < bd.size() && rc == QCE_OK; ++i) {
    const long long o = bd[i], n = bd[i + 1] - bd[i];
    HIPCHK(hipMemcpyAsync(m->y_scr.p + o * M, ys + o * M, sizeof(double2) * (size_t)n * M, hipMemcpyHostToDevice,
                          hp.s_in));
    HIPCHK(hipEventRecord(hp.ev_in[0], hp.s_in));
    HIPCHK(hipStreamWaitEvent(st, hp.ev_in[0], 0));
    rc = qce_estimate(m, reinterpret_cast<const double*>(m->y_scr.p + o * M), n, mode, mode_param,
                      reinterpret_cast<double*>(m->h_scr.p + o * N), QCE_IO_DEVICE, st);
    if (rc != QCE_OK) break;
    HIPCHK(hipEventRecord(hp.ev_c[0], st));
    HIPCHK(hipStreamWaitEvent(hp.s_out, hp.ev_c[0], 0));
    HIPCHK(hipMemcpyAsync(hs + o * N, m->h_scr.p + o * N, sizeof(double2) * (size_t)n * N, hipMemcpyDeviceToHost,
                          hp.s_out));
  }
  HIPCHK(hipStreamSynchronize(hp.s_in));
  HIPCHK(hipStreamSynchronize(hp.s_out));
  if (rc) return rc;
  HOST_SYNC_CHECK(m, st);
  return QCE_OK;
}

// Host numpy I/O split into chunks: host copies into a pinned slot, H2D on a copy stream, the estimate on
// the compute stream, D2H on a second copy stream into another pinned slot, host copy out -- chunk i's
// transfers overlap chunk i-1's and i+1's compute (results identical: every sample is independent).
static int estimate_host_pipelined(qce_model* m, const double* y, long long B, long long C, int mode,
                                   double mode_param, double* h_out, hipStream_t st) {
  auto& hp = m->hp;
  const size_t M = (size_t)m->M, N = (size_t)m->N;
  if (!hp.s_in) HIPCHK(hipStreamCreateWithFlags(&hp.s_in, hipStreamNonBlocking));
  if (!hp.s_out) HIPCHK(hipStreamCreateWithFlags(&hp.s_out, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) {
    if (!hp.ev_in[i]) HIPCHK(hipEventCreateWithFlags(&hp.ev_in[i], hipEventDisableTiming));
    if (!hp.ev_c[i]) HIPCHK(hipEventCreateWithFlags(&hp.ev_c[i], hipEventDisableTiming));
    if (!hp.ev_out[i]) HIPCHK(hipEventCreateWithFlags(&hp.ev_out[i], hipEventDisableTiming));
  }
  CopyStreamsDrain drain{hp.s_in, hp.s_out};
  if (hp.cap_y < (size_t)C * M || hp.cap_h < (size_t)C * N) {
    HIPCHK(hipStreamSynchronize(hp.s_in));
    HIPCHK(hipStreamSynchronize(hp.s_out));
    for (int i = 0; i < 2; ++i) {
      if (hp.pin_y[i]) (void)hipHostFree(hp.pin_y[i]);
      if (hp.pin_h[i]) (void)hipHostFree(hp.pin_h[i]);
      hp.pin_y[i] = hp.pin_h[i] = nullptr;
    }
    hp.cap_y = hp.cap_h = 0;
    for (int i = 0; i < 2; ++i) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&hp.pin_y[i]), sizeof(double2) * (size_t)C * M, hipHostMallocDefault));
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&hp.pin_h[i]), sizeof(double2) * (size_t)C * N, hipHostMallocDefault));
    }
    hp.cap_y = (size_t)C * M;
    hp.cap_h = (size_t)C * N;
  }
  // two device slots per direction, like the pinned ones (bounded scratch: a batch of any size streams through)
  HIPCHK(m->y_scr.ensure((size_t)2 * C * M));
  HIPCHK(m->h_scr.ensure((size_t)2 * C * N));
  const long long nc = (B + C - 1) / C;
  const double2* ys = reinterpret_cast<const double2*>(y);
  double2* hs = reinterpret_cast<double2*>(h_out);
  // the copy-in stream starts behind the compute stream's earlier work (the scratch slots' previous readers)
  HIPCHK(hipEventRecord(hp.ev_c[0], st));
  HIPCHK(hipStreamWaitEvent(hp.s_in, hp.ev_c[0], 0));
  int rc = QCE_OK;
  for (long long i = 0; i <= nc; ++i) {
    if (i < nc && rc == QCE_OK) {
      const int s = (int)(i & 1);
      const long long o = i * C, n = (B - o) < C ? (B - o) : C;
      double2* yslot = m->y_scr.p + (size_t)s * C * M;
      double2* hslot = m->h_scr.p + (size_t)s * C * N;
      if (i >= 2) HIPCHK(hipEventSynchronize(hp.ev_in[s]));  // slot s: chunk i-2's upload has read it
      par_memcpy(hp.pin_y[s], ys + o * M, sizeof(double2) * (size_t)n * M);
      if (i >= 2) HIPCHK(hipStreamWaitEvent(hp.s_in, hp.ev_c[s], 0));  // chunk i-2's estimate has read y slot s
      HIPCHK(hipMemcpyAsync(yslot, hp.pin_y[s], sizeof(double2) * (size_t)n * M, hipMemcpyHostToDevice, hp.s_in));
      HIPCHK(hipEventRecord(hp.ev_in[s], hp.s_in));
      HIPCHK(hipStreamWaitEvent(st, hp.ev_in[s], 0));
      if (i >= 2) HIPCHK(hipStreamWaitEvent(st, hp.ev_out[s], 0));  // chunk i-2's download has read h slot s
      rc = qce_estimate(m, reinterpret_cast<const double*>(yslot), n, mode, mode_param,
                        reinterpret_cast<double*>(hslot), QCE_IO_DEVICE, st);
      if (rc == QCE_OK) {
        HIPCHK(hipEventRecord(hp.ev_c[s], st));
        HIPCHK(hipStreamWaitEvent(hp.s_out, hp.ev_c[s], 0));
        HIPCHK(hipMemcpyAsync(hp.pin_h[s], hslot, sizeof(double2) * (size_t)n * N, hipMemcpyDeviceToHost,
                              hp.s_out));
        HIPCHK(hipEventRecord(hp.ev_out[s], hp.s_out));
      }
    }
    if (i >= 1 && rc == QCE_OK) {  // chunk i-1 back to the caller's array
      const long long j = i - 1, o = j * C, n = (B - o) < C ? (B - o) : C;
      const int s = (int)(j & 1);
      HIPCHK(hipEventSynchronize(hp.ev_out[s]));
      par_memcpy(hs + o * N, hp.pin_h[s], sizeof(double2) * (size_t)n * N);
    }
  }
  HIPCHK(hipStreamSynchronize(hp.s_in));
  HIPCHK(hipStreamSynchronize(hp.s_out));
  if (rc) return rc;
  HOST_SYNC_CHECK(m, st);
  return QCE_OK;
}

int qce_estimate(qce_model* m, const double* y, int64_t B, int mode, double mode_param, double* h_out, int io,
                 void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!y || !h_out))) return fail(QCE_EARG, "bad y / h_out");
  if (B == 0) return QCE_OK;
  if (!m->fft_active && !m->big && mode != QCE_MODE_ALL && !qce_select_shape_supported(m->MP, m->NP))
    return fail(QCE_ENOTIMPL, "selective modes: shape not covered");
  if (mode != QCE_MODE_ALL && m->K > qce_select_max_k())
    return fail(QCE_ENOTIMPL, "selective modes support K <= " + std::to_string(qce_select_max_k()));
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  if (io == QCE_IO_HOST)
    if (const long long C = host_chunk_rows(m, B)) {
      const char* de = getenv("QCE_HOST_DIRECT");  // QCE_HOST_DIRECT=0: the staged pipeline only (A/B runs, tests)
      if (!(de && de[0] == '0')) {
        HostDma dy(const_cast<double*>(y), sizeof(double2) * (size_t)B * m->M);
        HostDma dh(h_out, sizeof(double2) * (size_t)B * m->N);
        if (dy.ok && dh.ok) {
          const int drc = estimate_host_direct(m, y, B, mode, mode_param, h_out, st);
          if (drc != kDirectNoScratch) return drc;
        }
      }
      return estimate_host_pipelined(m, y, B, C, mode, mode_param, h_out, st);
    }
  const double2* dy = nullptr;
  if ((rc = stage_input(m, y, B, io, st, &dy))) return rc;
  double2* dh = reinterpret_cast<double2*>(h_out);
  if (io == QCE_IO_HOST) {
    HIPCHK(m->h_scr.ensure((size_t)B * m->N));
    dh = m->h_scr.p;
  }
  if (m->big) {  // N or M beyond 256: lp GEMM -> FP64 weights -> stacked-filter GEMM (qce_big.hip)
    int kmode = 0, n = 0;
    double p = 0.0;
    if (mode == QCE_MODE_TOPN) {
      if (mode_param < 1.0 || mode_param != floor(mode_param)) return fail(QCE_EARG, "top-n needs an integer n >= 1");
      n = mode_param > 1e9 ? 1000000000 : (int)mode_param;
      kmode = (n == 1) ? 3 : 1;
    } else if (mode == QCE_MODE_CUMP) {
      kmode = 2;
      p = mode_param;
    } else if (mode != QCE_MODE_ALL) {
      return fail(QCE_EARG, "unknown mode");
    }
    HIPCHK(m->lp_scr.ensure((size_t)B * m->K));
    HIPCHK(m->w64_scr.ensure((size_t)B * m->K));
    if ((rc = qce_big_lp(m, dy, B, m->lp_scr.p, st))) return rc;
    if (mode == QCE_MODE_ALL && m->K > qce_select_max_k()) {  // 'all' takes any K
      if ((rc = qce_big_proba(m, B, st))) return rc;
    } else if (mode == QCE_MODE_ALL)  // responsibilities = proba (:220-228: no renormalisation)
      HIPCHK(qce_launch_select(B, m->K, m->lp_scr.p, 0, 0, 0.0, m->w64_scr.p, nullptr, nullptr, st));
    else
      HIPCHK(qce_launch_select(B, m->K, m->lp_scr.p, kmode, n, p, nullptr, nullptr, nullptr, st, m->w64_scr.p));
    if ((rc = qce_big_wsum(m, dy, B, m->w64_scr.p, dh, m->N, st))) return rc;
    if (io == QCE_IO_HOST) {
      HIPCHK(hipMemcpyAsync(h_out, dh, sizeof(double2) * (size_t)B * m->N, hipMemcpyDeviceToHost, st));
      HOST_SYNC_CHECK(m, st);
    }
    return QCE_OK;
  }
  if (!m->fft_active && (mode != QCE_MODE_ALL || !use_h2()) && (rc = ensure_packs(m, st))) return rc;
  QceEstArgs a = est_args(m, dy, B);
  if (m->fft_active) {  // Fourier-domain path (qce_fft.hip)
    QceFftEstArgs fa = fft_args(m, dy, B);
    fa.h = dh;
    if (mode == QCE_MODE_ALL) {
      if (m->fft_mfma) HIPCHK(qce_launch_fft_mfma(fa, 0, st));
      else HIPCHK(qce_launch_fft_est(fa, 0, st));
    } else {
      int kmode, n = 0;
      double p = 0.0;
      if (mode == QCE_MODE_TOPN) {
        if (mode_param < 1.0 || mode_param != floor(mode_param)) return fail(QCE_EARG, "top-n needs an integer n >= 1");
        n = mode_param > 1e9 ? 1000000000 : (int)mode_param;
        kmode = (n == 1) ? 3 : 1;
      } else if (mode == QCE_MODE_CUMP) {
        kmode = 2;
        p = mode_param;
      } else {
        return fail(QCE_EARG, "unknown mode");
      }
      HIPCHK(m->lp_scr.ensure((size_t)B * m->K));
      HIPCHK(m->w64_scr.ensure((size_t)B * m->K));
      fa.lp = m->lp_scr.p;
      HIPCHK(qce_launch_fft_est(fa, 1, st));
      // FP64 selection weights: the reference sorts complex128-derived proba (gmm_cplx_bussgang.py:213, :235-236)
      HIPCHK(qce_launch_select(B, m->K, m->lp_scr.p, kmode, n, p, nullptr, nullptr, nullptr, st, m->w64_scr.p));
      fa.wts = m->w64_scr.p;
      HIPCHK(qce_launch_fft_est(fa, 2, st));
    }
  } else if (mode == QCE_MODE_ALL) {
    if (m->f64_active) {
      if ((rc = run_f64(m, dy, B, dh, nullptr, nullptr, nullptr, st))) return rc;
    } else if (m->f64_wide) {
      if ((rc = run_wide(m, dy, B, 0, dh, nullptr, nullptr, nullptr, nullptr, nullptr, st))) return rc;
    } else if (use_h2() || !qce_shape_supported(m->MP, m->NP)) {
      if ((rc = run_h2(m, dy, B, dh, nullptr, nullptr, nullptr, st))) return rc;
    } else {
      HIPCHK(qce_launch_est_all(a, dh, st));
    }
  } else {
    int kmode, n = 0;
    double p = 0.0;
    if (mode == QCE_MODE_TOPN) {
      if (mode_param < 1.0 || mode_param != floor(mode_param)) return fail(QCE_EARG, "top-n needs an integer n >= 1");
      n = mode_param > 1e9 ? 1000000000 : (int)mode_param;
      kmode = (n == 1) ? 3 : 1;
    } else if (mode == QCE_MODE_CUMP) {
      kmode = 2;
      p = mode_param;
    } else {
      return fail(QCE_EARG, "unknown mode");
    }
    HIPCHK(m->lp_scr.ensure((size_t)B * m->K));
    HIPCHK(m->w_scr.ensure((size_t)B * m->K));
    HIPCHK(qce_launch_lp(a, m->lp_scr.p, st));
    if (want_f64(m)) {  // FP64 selection weights and FP64 filters (the reference's complex128 arithmetic)
      HIPCHK(m->w64_scr.ensure((size_t)B * m->K));
      HIPCHK(qce_launch_select(B, m->K, m->lp_scr.p, kmode, n, p, nullptr, nullptr, nullptr, st, m->w64_scr.p));
      HIPCHK(m->WT.ensure((size_t)m->K * m->M * m->N));
      HIPCHK(qce_launch_sparse_f64(B, m->N, m->M, m->K, dy, m->w64_scr.p, m->W.p, m->bvec.p, m->WT.p, !m->wt_valid,
                                   dh, st));
      m->wt_valid = 1;
    } else {
      HIPCHK(qce_launch_select(B, m->K, m->lp_scr.p, kmode, n, p, nullptr, nullptr, m->w_scr.p, st));
      HIPCHK(qce_launch_est_weighted(a, m->w_scr.p, dh, st));
    }
  }
  if (io == QCE_IO_HOST) {
    HIPCHK(hipMemcpyAsync(h_out, dh, sizeof(double2) * (size_t)B * m->N, hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  }
  return QCE_OK;
}

int qce_log_prob(qce_model* m, const double* X, int64_t B, double* lp_out, double* proba_out, int64_t* labels_out,
                 int io, void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && !X)) return fail(QCE_EARG, "bad X");
  if (B == 0) return QCE_OK;
  if (m->K > qce_select_max_k() && (proba_out || labels_out))
    return fail(QCE_ENOTIMPL, "proba/labels support K <= " + std::to_string(qce_select_max_k()));
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dx = nullptr;
  if ((rc = stage_input(m, X, B, io, st, &dx))) return rc;
  if (!m->fft_active && !m->big && (rc = ensure_packs(m, st))) return rc;
  QceEstArgs a = est_args(m, dx, B);
  const size_t BK = (size_t)B * m->K;
  double* dlp = lp_out;
  double* dpr = proba_out;
  long long* dlab = reinterpret_cast<long long*>(labels_out);
  if (io == QCE_IO_HOST || !lp_out) {
    HIPCHK(m->lp_scr.ensure(BK));
    dlp = m->lp_scr.p;
  }
  if (io == QCE_IO_HOST && proba_out) {
    HIPCHK(m->proba_scr.ensure(BK));
    dpr = m->proba_scr.p;
  }
  if (io == QCE_IO_HOST && labels_out) {
    HIPCHK(m->lab_scr.ensure((size_t)B));
    dlab = m->lab_scr.p;
  }
  if (m->fft_active) {
    QceFftEstArgs fa = fft_args(m, dx, B);
    fa.lp = dlp;
    HIPCHK(qce_launch_fft_est(fa, 1, st));
  } else if (m->big) {
    if ((rc = qce_big_lp(m, dx, B, dlp, st))) return rc;
  } else {
    HIPCHK(qce_launch_lp(a, dlp, st));
  }
  if (proba_out || labels_out) HIPCHK(qce_launch_select(B, m->K, dlp, 0, 0, 0.0, dpr, dlab, nullptr, st));
  if (io == QCE_IO_HOST) {
    if (lp_out) HIPCHK(hipMemcpyAsync(lp_out, dlp, sizeof(double) * BK, hipMemcpyDeviceToHost, st));
    if (proba_out) HIPCHK(hipMemcpyAsync(proba_out, dpr, sizeof(double) * BK, hipMemcpyDeviceToHost, st));
    if (labels_out) HIPCHK(hipMemcpyAsync(labels_out, dlab, sizeof(int64_t) * B, hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  }
  return QCE_OK;
}

int qce_estimate_partial(qce_model* m, const double* y, int64_t B, double* m_out, double* s_out, float* acc_out,
                         int io, void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!y || !m_out || !s_out || !acc_out))) return fail(QCE_EARG, "bad arguments");
  if (B == 0) return QCE_OK;
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dy = nullptr;
  if ((rc = stage_input(m, y, B, io, st, &dy))) return rc;
  double *dm = m_out, *ds = s_out;
  float* da = acc_out;
  if (io == QCE_IO_HOST) {
    HIPCHK(m->m_scr.ensure((size_t)B));
    HIPCHK(m->s_scr.ensure((size_t)B));
    HIPCHK(m->acc_scr.ensure((size_t)B * 2 * m->N));
    dm = m->m_scr.p;
    ds = m->s_scr.p;
    da = m->acc_scr.p;
  }
  if (m->fft_active) {
    QceFftEstArgs fa = fft_args(m, dy, B);
    fa.om = dm;
    fa.os = ds;
    fa.oa = da;
    if (m->fft_mfma) HIPCHK(qce_launch_fft_mfma(fa, 3, st));
    else HIPCHK(qce_launch_fft_est(fa, 3, st));
  } else if (m->f64_active || m->f64_wide || m->big) {  // FP64 partial, rounded to this entry point's f32 accumulator
    HIPCHK(m->part_a64.ensure((size_t)B * 2 * m->N));
    if (m->big) {
      if ((rc = qce_big_partial(m, dy, B, 1, dm, ds, m->part_a64.p, nullptr, nullptr, st))) return rc;
    } else if (m->f64_active) {
      if ((rc = run_f64(m, dy, B, nullptr, dm, ds, m->part_a64.p, st))) return rc;
    } else if ((rc = run_wide(m, dy, B, 1, nullptr, dm, ds, m->part_a64.p, nullptr, nullptr, st))) {
      return rc;
    }
    HIPCHK(qce_launch_f64_to_f32(m->part_a64.p, da, (long long)B * 2 * m->N, st));
  } else if (use_h2() || !qce_shape_supported(m->MP, m->NP)) {
    if ((rc = run_h2(m, dy, B, nullptr, dm, ds, da, st))) return rc;
  } else {
    if ((rc = ensure_packs(m, st))) return rc;
    QceEstArgs a = est_args(m, dy, B);
    HIPCHK(qce_launch_est_partial(a, dm, ds, da, st));
  }
  if (io == QCE_IO_HOST) {
    HIPCHK(hipMemcpyAsync(m_out, dm, sizeof(double) * B, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s_out, ds, sizeof(double) * B, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(acc_out, da, sizeof(float) * (size_t)B * 2 * m->N, hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  }
  return QCE_OK;
}

int qce_estimate_partial_f64(qce_model* m, const double* y, int64_t B, double* m_out, double* s_out, double* acc_out,
                             int io, void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!y || !m_out || !s_out || !acc_out))) return fail(QCE_EARG, "bad arguments");
  if (B == 0) return QCE_OK;
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dy = nullptr;
  if ((rc = stage_input(m, y, B, io, st, &dy))) return rc;
  double *dm = m_out, *ds = s_out, *da = acc_out;
  if (io == QCE_IO_HOST) {
    HIPCHK(m->m_scr.ensure((size_t)B));
    HIPCHK(m->s_scr.ensure((size_t)B));
    HIPCHK(m->part_a64.ensure((size_t)B * 2 * m->N));
    dm = m->m_scr.p;
    ds = m->s_scr.p;
    da = m->part_a64.p;
  }
  if (!m->fft_active && m->big) {
    if ((rc = qce_big_partial(m, dy, B, 1, dm, ds, da, nullptr, nullptr, st))) return rc;
  } else if (!m->fft_active && m->f64_active) {
    if ((rc = run_f64(m, dy, B, nullptr, dm, ds, da, st))) return rc;
  } else if (!m->fft_active && m->f64_wide) {
    if ((rc = run_wide(m, dy, B, 1, nullptr, dm, ds, da, nullptr, nullptr, st))) return rc;
  } else if (m->fft_active) {  // Fourier path: the same kernels with an FP64 accumulator
    QceFftEstArgs fa = fft_args(m, dy, B);
    fa.om = dm;
    fa.os = ds;
    fa.oa = reinterpret_cast<float*>(da);
    if (m->fft_mfma) HIPCHK(qce_launch_fft_mfma(fa, 4, st));
    else HIPCHK(qce_launch_fft_est(fa, 4, st));
  } else {  // the fast (fp16-split) path keeps an f32 accumulator: widen it
    HIPCHK(m->acc_scr.ensure((size_t)B * 2 * m->N));
    if ((rc = qce_estimate_partial(m, reinterpret_cast<const double*>(dy), B, dm, ds, m->acc_scr.p, QCE_IO_DEVICE,
                                   st)))
      return rc;
    HIPCHK(qce_launch_f32_to_f64(m->acc_scr.p, da, (long long)B * 2 * m->N, st));
  }
  if (io == QCE_IO_HOST) {
    HIPCHK(hipMemcpyAsync(m_out, dm, sizeof(double) * B, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s_out, ds, sizeof(double) * B, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(acc_out, da, sizeof(double) * (size_t)B * 2 * m->N, hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  }
  return QCE_OK;
}

int qce_estimate_partial_shifted(qce_model* m, const double* y, int64_t B, const double* shift, double* packed_out,
                                 int io, void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!y || !packed_out || !shift))) return fail(QCE_EARG, "bad arguments");
  if (B == 0) return QCE_OK;
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dy = nullptr;
  if ((rc = stage_input(m, y, B, io, st, &dy))) return rc;
  const size_t W = (size_t)B * (2 * m->N + 2);
  double* dp = packed_out;
  const double* dshift = shift;
  if (io == QCE_IO_HOST) {
    HIPCHK(m->fp_pack.ensure(W));
    dp = m->fp_pack.p;
    HIPCHK(m->shift_scr.ensure(1));
    HIPCHK(hipMemcpyAsync(m->shift_scr.p, shift, sizeof(double), hipMemcpyHostToDevice, st));
    dshift = m->shift_scr.p;
  }
  if (!m->fft_active && m->big) {
    if ((rc = qce_big_partial(m, dy, B, 2, nullptr, nullptr, nullptr, dp, dshift, st))) return rc;
  } else if (!m->fft_active && m->f64_active) {
    if ((rc = run_f64(m, dy, B, nullptr, nullptr, nullptr, nullptr, st, dp, dshift))) return rc;
  } else if (!m->fft_active && m->f64_wide) {
    if ((rc = run_wide(m, dy, B, 2, nullptr, nullptr, nullptr, nullptr, dp, dshift, st))) return rc;
  } else {  // other paths: their (m, s, acc) partial, scaled and packed
    HIPCHK(m->m_scr.ensure((size_t)B));
    HIPCHK(m->s_scr.ensure((size_t)B));
    HIPCHK(m->part_a64.ensure((size_t)B * 2 * m->N));
    if ((rc = qce_estimate_partial_f64(m, reinterpret_cast<const double*>(dy), B, m->m_scr.p, m->s_scr.p,
                                       m->part_a64.p, QCE_IO_DEVICE, st)))
      return rc;
    HIPCHK(qce_launch_pack_shifted(B, m->N, m->m_scr.p, m->s_scr.p, m->part_a64.p, nullptr, dshift, dp, st));
  }
  if (io == QCE_IO_HOST) {
    HIPCHK(hipMemcpyAsync(packed_out, dp, sizeof(double) * W, hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  }
  return QCE_OK;
}

int qce_cconst_max(qce_model* m, double* out, int io, void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (!out) return fail(QCE_EARG, "null out");
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  if (m->fft_active && (rc = ensure_dense(m, st))) return rc;
  if (io == QCE_IO_HOST) {
    HIPCHK(m->shift_scr.ensure(1));
    HIPCHK(qce_launch_cconst_max(m->K, m->cconst.p, m->status.p, m->shift_scr.p, st));
    HIPCHK(hipMemcpyAsync(out, m->shift_scr.p, sizeof(double), hipMemcpyDeviceToHost, st));
    HOST_SYNC_CHECK(m, st);
  } else {
    HIPCHK(qce_launch_cconst_max(m->K, m->cconst.p, m->status.p, out, st));
  }
  return QCE_OK;
}

int qce_get_tables(qce_model* m, double* means_y, double* Cy, double* Cr, double* P, double* A_eff, double* W,
                   double* b, double* cconst) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if ((rc = ensure_dense(m))) return rc;
  DeviceGuard g(m->device);
  hipStream_t st = m->stream;
  const int K = m->K, M = m->M, N = m->N;
  HOST_SYNC_CHECK(m, st);
  auto cp = [&](double* dst, const void* src, size_t bytes) -> hipError_t {
    if (!dst) return hipSuccess;
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  };
  HIPCHK(cp(means_y, m->means_y.p, sizeof(double2) * (size_t)K * M));
  HIPCHK(cp(Cy, m->Cy.p, sizeof(double2) * (size_t)K * M * M));
  HIPCHK(cp(Cr, m->Cr.p, sizeof(double2) * (size_t)K * M * M));
  HIPCHK(cp(A_eff, m->Aeff.p, sizeof(double2) * (size_t)K * M * N));
  HIPCHK(cp(W, m->W.p, sizeof(double2) * (size_t)K * N * M));
  HIPCHK(cp(b, m->bvec.p, sizeof(double2) * (size_t)K * N));
  HIPCHK(cp(cconst, m->cconst.p, sizeof(double) * (size_t)K));
  if (P) {
    std::vector<double> li((size_t)2 * K * M * M);
    HIPCHK(hipMemcpy(li.data(), m->Linv.p, sizeof(double2) * (size_t)K * M * M, hipMemcpyDeviceToHost));
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
          const size_t src = ((size_t)k * M * M + (size_t)j * M + i) * 2;  // P[i][j] = conj(Linv[j][i])
          const size_t dst = ((size_t)k * M * M + (size_t)i * M + j) * 2;
          P[dst] = li[src];
          P[dst + 1] = (j >= i) ? -li[src + 1] : 0.0;
          if (j < i) P[dst] = 0.0;
        }
  }
  return QCE_OK;
}

int qce_model_info(qce_model* m, int* K, int* N, int* M, int* device) {
  if (!m) return fail(QCE_EARG, "null model");
  if (K) *K = m->K;
  if (N) *N = m->N;
  if (M) *M = m->prepared ? m->M : 0;
  if (device) *device = m->device;
  return QCE_OK;
}

int qce_model_structure(qce_model* m, int* n1, int* n2, int* fourier_active) {
  if (!m) return fail(QCE_EARG, "null model");
  if (n1) *n1 = m->fft_n1;
  if (n2) *n2 = m->fft_n2;
  if (fourier_active) *fourier_active = m->prepared ? m->fft_active : 0;
  return QCE_OK;
}

int qce_model_kernel(qce_model* m, int* kind) {
  if (!m || !kind) return fail(QCE_EARG, "null argument");
  if (!m->prepared) *kind = QCE_KERNEL_NONE;
  else if (m->fft_active) *kind = QCE_KERNEL_FOURIER;
  else if (m->big) *kind = QCE_KERNEL_BIG;
  else if (m->f64_active) *kind = m->f64_g3 ? QCE_KERNEL_F64_3M : QCE_KERNEL_F64_4M;
  else if (m->f64_wide) *kind = QCE_KERNEL_F64_WIDE;
  else *kind = QCE_KERNEL_FAST;
  return QCE_OK;
}

namespace {

// stream-ordered scratch for the model-free entry points (freed on the same stream)
struct StreamScratch {
  hipStream_t st;
  std::vector<void*> ptrs;
  explicit StreamScratch(hipStream_t s) : st(s) {}
  hipError_t get(void** p, size_t bytes) {
    hipError_t e = hipMallocAsync(p, bytes ? bytes : 1, st);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~StreamScratch() {
    for (void* p : ptrs) (void)hipFreeAsync(p, st);
  }
};

}  // namespace

int qce_observe(const double* h, int64_t B, int N, const double* A, int M, double noise_scale, int noise_kind,
                const double* noise, uint64_t seed, uint64_t offset, double n_bits, const double* thresholds,
                const double* labels, int n_levels, double* y_out, int device, int io, void* stream) {
  if (B < 0 || N < 1 || (A && M < 1) || (!A && M != N)) return fail(QCE_EARG, "observe: bad shape");
  if (noise_kind < 0 || noise_kind > 2 || (noise_kind == 1 && !noise)) return fail(QCE_EARG, "observe: bad noise");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "observe: bad io");
  if (B > 0 && (!h || !y_out)) return fail(QCE_EARG, "observe: null buffer");
  int kind;
  if (n_bits == 1.0) kind = 0;
  else if (isinf(n_bits) && n_bits > 0) kind = 2;
  else {
    kind = 1;
    if (!thresholds || !labels || n_levels < 2 || n_levels > 256)
      return fail(QCE_EARG, "observe: multi-bit quantisation needs thresholds (L-1) and labels (L), 2 <= L <= 256");
    for (int i = 1; i < n_levels - 1; ++i)
      if (!(thresholds[i] >= thresholds[i - 1])) return fail(QCE_EARG, "observe: thresholds must be increasing");
  }
  if (B == 0) return QCE_OK;
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  const size_t ny = (size_t)B * M, nh = (size_t)B * N;
  QceObserveArgs a;
  a.B = B;
  a.M = M;
  a.N = N;
  a.noise = noise_kind;
  a.noise_scale = noise_scale;
  a.seed = seed;
  a.offset = offset;
  a.kind = kind;
  a.nthr = kind == 1 ? n_levels - 1 : 0;
  {
    StreamScratch sc(st);
    void* p;
    a.A = nullptr;
    if (A) {
      HIPCHK(sc.get(&p, sizeof(double2) * (size_t)M * N));
      HIPCHK(hipMemcpyAsync(p, A, sizeof(double2) * (size_t)M * N, hipMemcpyHostToDevice, st));
      a.A = (const double2*)p;
    }
    a.thr = a.lab = nullptr;
    if (kind == 1) {
      HIPCHK(sc.get(&p, sizeof(double) * (size_t)(2 * n_levels - 1)));
      HIPCHK(hipMemcpyAsync(p, thresholds, sizeof(double) * (n_levels - 1), hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync((double*)p + n_levels - 1, labels, sizeof(double) * n_levels, hipMemcpyHostToDevice, st));
      a.thr = (const double*)p;
      a.lab = (const double*)p + n_levels - 1;
    }
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&p, sizeof(double2) * nh));
      HIPCHK(hipMemcpyAsync(p, h, sizeof(double2) * nh, hipMemcpyHostToDevice, st));
      a.h = (const double2*)p;
      a.w = nullptr;
      if (noise_kind == 1) {
        HIPCHK(sc.get(&p, sizeof(double2) * ny));
        HIPCHK(hipMemcpyAsync(p, noise, sizeof(double2) * ny, hipMemcpyHostToDevice, st));
        a.w = (const double2*)p;
      }
      HIPCHK(sc.get(&p, sizeof(double2) * ny));
      a.y = (double2*)p;
    } else {
      a.h = (const double2*)h;
      a.w = (const double2*)noise;
      a.y = (double2*)y_out;
    }
    HIPCHK(qce_launch_observe(a, st));
    if (io == QCE_IO_HOST) HIPCHK(hipMemcpyAsync(y_out, a.y, sizeof(double2) * ny, hipMemcpyDeviceToHost, st));
  }
  if (io == QCE_IO_HOST) HIPCHK(hipStreamSynchronize(st));
  return QCE_OK;
}

int qce_sq_error(const double* a, const double* b, int64_t n, double* out, int device, int io, void* stream) {
  if (n < 0 || !out || (n > 0 && (!a || !b))) return fail(QCE_EARG, "sq_error: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "sq_error: bad io");
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  {
    StreamScratch sc(st);
    void *pa, *pb, *part, *po;
    HIPCHK(sc.get(&part, sizeof(double) * qce_sq_err_scratch()));
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&pa, sizeof(double2) * (size_t)n));
      HIPCHK(sc.get(&pb, sizeof(double2) * (size_t)n));
      HIPCHK(sc.get(&po, sizeof(double)));
      HIPCHK(hipMemcpyAsync(pa, a, sizeof(double2) * (size_t)n, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(pb, b, sizeof(double2) * (size_t)n, hipMemcpyHostToDevice, st));
    } else {
      pa = (void*)a;
      pb = (void*)b;
      po = out;
    }
    HIPCHK(qce_launch_sq_err(n, (const double2*)pa, (const double2*)pb, (double*)part, (double*)po, st));
    if (io == QCE_IO_HOST) HIPCHK(hipMemcpyAsync(out, po, sizeof(double), hipMemcpyDeviceToHost, st));
  }
  if (io == QCE_IO_HOST) HIPCHK(hipStreamSynchronize(st));
  return QCE_OK;
}

int qce_em_estep(qce_model* m, const double* X, int64_t B, double* resp_out, double* mean_lse_out, int io,
                 void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 1 || !X || !resp_out || !mean_lse_out) return fail(QCE_EARG, "em_estep: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "em_estep: bad io");
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dx = nullptr;
  if ((rc = stage_input(m, X, B, io, st, &dx))) return rc;
  const size_t BK = (size_t)B * m->K;
  HIPCHK(m->lp_scr.ensure(BK));
  double* dlp = m->lp_scr.p;
  if (m->fft_active) {
    QceFftEstArgs fa = fft_args(m, dx, B);
    fa.lp = dlp;
    HIPCHK(qce_launch_fft_est(fa, 1, st));
  } else if (m->big) {
    if ((rc = qce_big_lp(m, dx, B, dlp, st))) return rc;
  } else {
    if ((rc = ensure_packs(m, st))) return rc;
    QceEstArgs a = est_args(m, dx, B);
    HIPCHK(qce_launch_lp(a, dlp, st));
  }
  {
    StreamScratch sc(st);
    void *lse, *part, *dresp = resp_out, *dmean = mean_lse_out;
    HIPCHK(sc.get(&lse, sizeof(double) * (size_t)B));
    HIPCHK(sc.get(&part, sizeof(double) * qce_mean_scratch()));
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&dresp, sizeof(double) * BK));
      HIPCHK(sc.get(&dmean, sizeof(double)));
    }
    HIPCHK(qce_launch_em_resp(B, m->K, dlp, (double*)dresp, (double*)lse, (double*)part, (double*)dmean, st));
    if (io == QCE_IO_HOST) {
      HIPCHK(hipMemcpyAsync(resp_out, dresp, sizeof(double) * BK, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(mean_lse_out, dmean, sizeof(double), hipMemcpyDeviceToHost, st));
    }
  }
  if (io == QCE_IO_HOST) HOST_SYNC_CHECK(m, st);
  return QCE_OK;
}

int qce_em_mstep(const double* X, int64_t B, int N, int K, const double* resp, double reg_covar, int diag,
                 int zero_mean, double* nk_out, double* means_out, double* covs_out, int device, int io,
                 void* stream) {
  if (B < 1 || N < 1 || N > 256 || K < 1 || !X || !resp || !nk_out || !means_out || !covs_out)
    return fail(QCE_EARG, "em_mstep: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "em_mstep: bad io");
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  QceEmArgs a;
  a.B = B;
  a.N = N;
  a.K = K;
  a.diag = diag ? 1 : 0;
  a.zero_mean = zero_mean ? 1 : 0;
  a.reg = reg_covar;
  a.plan = qce_em_plan(B, N, K, a.diag);
  const size_t nX = (size_t)B * N, nR = (size_t)B * K, nM = (size_t)K * N;
  const size_t nC = a.diag ? nM : nM * N;
  const size_t cov_bytes = a.diag ? sizeof(double) * nC : sizeof(double2) * nC;
  {
    StreamScratch sc(st);
    void* p;
    HIPCHK(sc.get(&p, sizeof(double) * a.plan.stat_doubles));
    a.stats = (double*)p;
    a.part = nullptr;
    if (!a.diag) {
      HIPCHK(sc.get(&p, sizeof(double2) * a.plan.part_elems));
      a.part = (double2*)p;
    }
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&p, sizeof(double2) * nX));
      HIPCHK(hipMemcpyAsync(p, X, sizeof(double2) * nX, hipMemcpyHostToDevice, st));
      a.X = (const double2*)p;
      HIPCHK(sc.get(&p, sizeof(double) * nR));
      HIPCHK(hipMemcpyAsync(p, resp, sizeof(double) * nR, hipMemcpyHostToDevice, st));
      a.R = (const double*)p;
      HIPCHK(sc.get(&p, sizeof(double) * K));
      a.nk = (double*)p;
      HIPCHK(sc.get(&p, sizeof(double2) * nM));
      a.means = (double2*)p;
      HIPCHK(sc.get(&p, cov_bytes));
    } else {
      a.X = (const double2*)X;
      a.R = resp;
      a.nk = nk_out;
      a.means = (double2*)means_out;
      p = covs_out;
    }
    a.covs = a.diag ? nullptr : (double2*)p;
    a.diag_out = a.diag ? (double*)p : nullptr;
    HIPCHK(qce_launch_em_mstep(a, st));
    if (io == QCE_IO_HOST) {
      HIPCHK(hipMemcpyAsync(nk_out, a.nk, sizeof(double) * K, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(means_out, a.means, sizeof(double2) * nM, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(covs_out, p, cov_bytes, hipMemcpyDeviceToHost, st));
    }
  }
  if (io == QCE_IO_HOST) HIPCHK(hipStreamSynchronize(st));
  return QCE_OK;
}

int qce_model_set_option(qce_model* m, int option, double value) {
  if (!m) return fail(QCE_EARG, "null model");
  if (option == QCE_OPT_BETA_FIRST) {
    m->beta_first = value != 0.0;
    m->prepared = 0;
    return QCE_OK;
  }
  if (option == QCE_OPT_RESERVE_CUS) {
    if (value < 0.0 || value != floor(value)) return fail(QCE_EARG, "reserve_cus must be an integer >= 0");
    m->reserve_cus = value > 1e6 ? 1000000 : (int)value;
    m->reserve_set = 1;
    return QCE_OK;
  }
  if (option == QCE_OPT_PRECISION) {
    if (value != QCE_PRECISION_F64 && value != QCE_PRECISION_FAST) return fail(QCE_EARG, "unknown precision");
    m->precision = (int)value;
    m->prepared = 0;
    return QCE_OK;
  }
  return fail(QCE_EARG, "unknown option");
}

static int assigned_impl(qce_model* m, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                         void* stream, int ls);

int qce_estimate_assigned(qce_model* m, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                          void* stream) {
  return assigned_impl(m, y, B, comp, h_out, io, stream, 0);
}

int qce_estimate_ls(qce_model* m, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                    void* stream) {
  return assigned_impl(m, y, B, comp, h_out, io, stream, 1);
}

int qce_estimate_ls_general(qce_model* m, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                            void* stream) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (m->M < m->N) return fail(QCE_ENOTIMPL, "general LS needs M >= N (full column rank A_eff)");
  return assigned_impl(m, y, B, comp, h_out, io, stream, 2);
}

static int assigned_impl(qce_model* m, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                         void* stream, int ls) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!y || !h_out))) return fail(QCE_EARG, "bad arguments");
  if (!comp && B > m->K) return fail(QCE_EARG, "without comp, sample b uses component b: B <= K");
  if (B == 0) return QCE_OK;
  if (m->big) return fail(QCE_ENOTIMPL, "per-sample filters / LS cover N, M <= 256");
  if ((rc = ensure_dense(m))) return rc;
  DeviceGuard g(m->device);
  hipStream_t st = pick_stream(m, stream);
  const double2* dy = nullptr;
  if ((rc = stage_input(m, y, B, io, st, &dy))) return rc;
  {
    StreamScratch sc(st);
    void* p;
    const long long* dc = reinterpret_cast<const long long*>(comp);
    double2* dh = reinterpret_cast<double2*>(h_out);
    if (comp && io == QCE_IO_HOST) {
      for (int64_t b = 0; b < B; ++b)
        if (comp[b] < 0 || comp[b] >= m->K) return fail(QCE_EARG, "component index out of range");
      HIPCHK(sc.get(&p, sizeof(long long) * (size_t)B));
      HIPCHK(hipMemcpyAsync(p, comp, sizeof(long long) * (size_t)B, hipMemcpyHostToDevice, st));
      dc = (const long long*)p;
    }
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&p, sizeof(double2) * (size_t)B * m->N));
      dh = (double2*)p;
    }
    if (ls == 2) {
      void *T, *P, *bz, *bad;
      HIPCHK(sc.get(&T, sizeof(double2) * (size_t)m->K * m->N * (m->N + m->M)));
      HIPCHK(sc.get(&P, sizeof(double2) * (size_t)m->K * m->N * m->M));
      HIPCHK(sc.get(&bz, sizeof(double2) * (size_t)m->K * m->N));
      HIPCHK(sc.get(&bad, sizeof(int) * (size_t)m->K));
      HIPCHK(qce_launch_ls_pinv(m->K, m->N, m->M, 0, m->Aeff.p, (double2*)T, (double2*)P, (double2*)bz, (int*)bad, st));
      std::vector<int> hb(m->K);
      HIPCHK(hipMemcpyAsync(hb.data(), bad, sizeof(int) * (size_t)m->K, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      for (int k = 0; k < m->K; ++k)
        if (hb[k])
          return fail(QCE_ECHOL, "LS: A_eff of component " + std::to_string(k) +
                                     " is not of full column rank (Gram matrix pivot " + std::to_string(hb[k] - 1) +
                                     " vanishes)");
      HIPCHK(qce_launch_est_assigned(B, m->N, m->M, m->K, dy, dc, (const double2*)P, (const double2*)bz, dh, st));
    } else if (ls) HIPCHK(qce_launch_ls(B, m->N, m->M, dy, dc, m->Aeff.p, dh, st));
    else HIPCHK(qce_launch_est_assigned(B, m->N, m->M, m->K, dy, dc, m->W.p, m->bvec.p, dh, st));
    if (io == QCE_IO_HOST)
      HIPCHK(hipMemcpyAsync(h_out, dh, sizeof(double2) * (size_t)B * m->N, hipMemcpyDeviceToHost, st));
  }
  if (io == QCE_IO_HOST) HOST_SYNC_CHECK(m, st);
  return QCE_OK;
}

int qce_em_toeplitz(qce_model* m, const double* S, int K, int N, const double* F2, int P, double* sigma, double reg,
                    int init, double* covs_out, int device, void* stream) {
  if (!S || !F2 || !sigma || K < 1 || N < 1 || P < 1 || (!init && (!m || !covs_out)))
    return fail(QCE_EARG, "em_toeplitz: bad arguments");
  int rc;
  if (!init) {
    if ((rc = check_model(m, true))) return rc;
    if (m->K != K || m->N != N || m->M != N) return fail(QCE_EARG, "em_toeplitz: model shape mismatch");
    if ((rc = ensure_dense(m))) return rc;
    device = m->device;
  }
  DeviceGuard g(device);
  hipStream_t st = (!init && !stream) ? m->stream : (hipStream_t)stream;
  const size_t nn = (size_t)N * N, KNN = (size_t)K * nn;
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0), mone = make_double2(-1.0, 0.0);
  {
    StreamScratch sc(st);
    void *dS, *dF, *dsg, *dG, *dC = nullptr, *dT = nullptr, *dM = nullptr;
    HIPCHK(sc.get(&dS, sizeof(double2) * KNN));
    HIPCHK(sc.get(&dF, sizeof(double2) * (size_t)P * N));
    HIPCHK(sc.get(&dsg, sizeof(double) * (size_t)K * P));
    HIPCHK(sc.get(&dG, sizeof(double2) * (size_t)K * P * N));
    HIPCHK(hipMemcpyAsync(dS, S, sizeof(double2) * KNN, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dF, F2, sizeof(double2) * (size_t)P * N, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dsg, sigma, sizeof(double) * (size_t)K * P, hipMemcpyHostToDevice, st));
    const double2* Mx = (const double2*)dS;
    if (!init) {
      // Cinv = Linv^H Linv (the previous covariances' inverse, :808); Mx = Cinv S Cinv - Cinv (:812)
      HIPCHK(sc.get(&dC, sizeof(double2) * KNN));
      HIPCHK(sc.get(&dT, sizeof(double2) * KNN));
      HIPCHK(sc.get(&dM, sizeof(double2) * KNN));
      HIPCHK(qce_zgemm_batched(2, 0, N, N, N, one, m->Linv.p, N, nn, m->Linv.p, N, nn, zero, (double2*)dC, N, nn, K,
                               st));
      HIPCHK(qce_zgemm_batched(0, 0, N, N, N, one, (const double2*)dC, N, nn, (const double2*)dS, N, nn, zero,
                               (double2*)dT, N, nn, K, st));
      HIPCHK(hipMemcpyAsync(dM, dC, sizeof(double2) * KNN, hipMemcpyDeviceToDevice, st));
      HIPCHK(qce_zgemm_batched(0, 0, N, N, N, one, (const double2*)dT, N, nn, (const double2*)dC, N, nn, mone,
                               (double2*)dM, N, nn, K, st));
      Mx = (const double2*)dM;
    }
    // G_k = F2 Mx_k (P x N), then theta = Re diag(G_k F2^H)
    HIPCHK(qce_zgemm_batched(0, 0, P, N, N, one, (const double2*)dF, N, 0, Mx, N, nn, zero, (double2*)dG, N,
                             (long long)P * N, K, st));
    HIPCHK(qce_launch_inv_em_sigma(K, N, P, (const double2*)dG, (const double2*)dF, (double*)dsg, reg, init, st));
    HIPCHK(hipMemcpyAsync(sigma, dsg, sizeof(double) * (size_t)K * P, hipMemcpyDeviceToHost, st));
    if (!init) {
      HIPCHK(qce_launch_inv_em_cov(K, N, P, (const double2*)dF, (const double*)dsg, reg, (double2*)dT, st));
      HIPCHK(hipMemcpyAsync(covs_out, dT, sizeof(double2) * KNN, hipMemcpyDeviceToHost, st));
    }
  }
  HIPCHK(hipStreamSynchronize(st));
  return QCE_OK;
}

int qce_scm_generate(int64_t B, int n_coherence, int N, int n_path, double path_sigma, const double* gains,
                     const double* angles, const double* x, uint64_t seed, float* h_out, float* t_out, int device,
                     int io, void* stream) {
  if (B < 0 || n_coherence < 1 || N < 1 || N > 256 || n_path < 1 || n_path > qce_scm_max_path() ||
      (B > 0 && (!h_out || !t_out)) || (!gains) != (!angles))
    return fail(QCE_EARG, "scm_generate: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "scm_generate: bad io");
  if (B == 0) return QCE_OK;
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  const size_t F = 100 * (size_t)N, nh = (size_t)B * n_coherence * N, nt = (size_t)B * N;
  {
    StreamScratch sc(st);
    void* p;
    const double *dg = gains, *da = angles;
    const double2* dx = (const double2*)x;
    float2* dh = (float2*)h_out;
    float2* dt = (float2*)t_out;
    if (io == QCE_IO_HOST) {
      if (gains) {
        HIPCHK(sc.get(&p, sizeof(double) * 2 * (size_t)B * n_path));
        HIPCHK(hipMemcpyAsync(p, gains, sizeof(double) * (size_t)B * n_path, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync((double*)p + (size_t)B * n_path, angles, sizeof(double) * (size_t)B * n_path,
                              hipMemcpyHostToDevice, st));
        dg = (const double*)p;
        da = (const double*)p + (size_t)B * n_path;
      }
      if (x) {
        HIPCHK(sc.get(&p, sizeof(double2) * (size_t)B * F * n_coherence));
        HIPCHK(hipMemcpyAsync(p, x, sizeof(double2) * (size_t)B * F * n_coherence, hipMemcpyHostToDevice, st));
        dx = (const double2*)p;
      }
      HIPCHK(sc.get(&p, sizeof(float2) * (nh + nt)));
      dh = (float2*)p;
      dt = (float2*)p + nh;
    }
    HIPCHK(qce_launch_scm(B, n_coherence, N, n_path, path_sigma, dg, da, dx, seed, dh, dt, st));
    if (io == QCE_IO_HOST) {
      HIPCHK(hipMemcpyAsync(h_out, dh, sizeof(float2) * nh, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(t_out, dt, sizeof(float2) * nt, hipMemcpyDeviceToHost, st));
    }
  }
  if (io == QCE_IO_HOST) HIPCHK(hipStreamSynchronize(st));
  return QCE_OK;
}

int qce_rate_bound(const double* h_est, const double* h, int64_t B, int N, const double* buss, const double* Cq,
                   double norm_clip, double* out, int device, int io, void* stream) {
  if (B < 1 || N < 1 || !h_est || !h || !buss || !Cq || !out) return fail(QCE_EARG, "rate_bound: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "rate_bound: bad io");
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  const size_t nb = (size_t)B * N;
  {
    StreamScratch sc(st);
    void *dhe = (void*)h_est, *dh = (void*)h, *dbuss, *dcq, *inner, *den2, *part, *stat;
    HIPCHK(sc.get(&dbuss, sizeof(double) * N));
    HIPCHK(sc.get(&dcq, sizeof(double2) * (size_t)N * N));
    HIPCHK(hipMemcpyAsync(dbuss, buss, sizeof(double) * N, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dcq, Cq, sizeof(double2) * (size_t)N * N, hipMemcpyHostToDevice, st));
    HIPCHK(sc.get(&inner, sizeof(double2) * (size_t)B));
    HIPCHK(sc.get(&den2, sizeof(double) * (size_t)B));
    HIPCHK(sc.get(&part, sizeof(double) * qce_rate_scratch()));
    HIPCHK(sc.get(&stat, sizeof(double) * 8));
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&dhe, sizeof(double2) * nb));
      HIPCHK(sc.get(&dh, sizeof(double2) * nb));
      HIPCHK(hipMemcpyAsync(dhe, h_est, sizeof(double2) * nb, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(dh, h, sizeof(double2) * nb, hipMemcpyHostToDevice, st));
    }
    HIPCHK(qce_launch_rate(B, N, (const double2*)dhe, (const double2*)dh, (const double*)dbuss, (const double2*)dcq,
                           norm_clip, (double2*)inner, (double*)den2, (double*)part, (double*)stat, st));
    double res[6];
    HIPCHK(hipMemcpyAsync(res, stat, sizeof(double) * 6, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    out[0] = res[5];  // rate
    out[1] = res[4];  // num
    out[2] = res[3];  // den1
    out[3] = res[2];  // den2
  }
  return QCE_OK;
}

int qce_rate_mf(const double* h_est, const double* h, int64_t B, int N, const double* buss, const double* Cq,
                double* out, int device, int io, void* stream) {
  if (B < 1 || N < 1 || N > 256 || !h_est || !h || !buss || !Cq || !out) return fail(QCE_EARG, "rate_mf: bad arguments");
  if (io != QCE_IO_HOST && io != QCE_IO_DEVICE) return fail(QCE_EARG, "rate_mf: bad io");
  DeviceGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  const size_t nb = (size_t)B * N, nn = (size_t)N * N;
  {
    StreamScratch sc(st);
    void *dhe = (void*)h_est, *dh = (void*)h, *dbuss, *dcq, *T, *cqi, *bz, *rate, *sum, *bad;
    HIPCHK(sc.get(&dbuss, sizeof(double) * N));
    HIPCHK(sc.get(&dcq, sizeof(double2) * nn));
    HIPCHK(sc.get(&T, sizeof(double2) * nn * 2));
    HIPCHK(sc.get(&cqi, sizeof(double2) * nn));
    HIPCHK(sc.get(&bz, sizeof(double2) * N));
    HIPCHK(sc.get(&rate, sizeof(double) * (size_t)B));
    HIPCHK(sc.get(&sum, sizeof(double)));
    HIPCHK(sc.get(&bad, sizeof(int)));
    HIPCHK(hipMemcpyAsync(dbuss, buss, sizeof(double) * N, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dcq, Cq, sizeof(double2) * nn, hipMemcpyHostToDevice, st));
    if (io == QCE_IO_HOST) {
      HIPCHK(sc.get(&dhe, sizeof(double2) * nb));
      HIPCHK(sc.get(&dh, sizeof(double2) * nb));
      HIPCHK(hipMemcpyAsync(dhe, h_est, sizeof(double2) * nb, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(dh, h, sizeof(double2) * nb, hipMemcpyHostToDevice, st));
    }
    HIPCHK(qce_launch_ls_pinv(1, N, N, 1, (const double2*)dcq, (double2*)T, (double2*)cqi, (double2*)bz, (int*)bad, st));
    HIPCHK(qce_launch_rate_mf(B, N, (const double2*)dhe, (const double2*)dh, (const double*)dbuss, (const double2*)dcq,
                              (const double2*)cqi, (double*)rate, (double*)sum, st));
    double r = 0.0;
    int hb = 0;
    HIPCHK(hipMemcpyAsync(&r, sum, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&hb, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (hb) return fail(QCE_ECHOL, "rate_mf: Cq is not positive definite (pivot " + std::to_string(hb - 1) + ")");
    out[0] = r / (double)B;
  }
  return QCE_OK;
}

}  // extern "C"

// Selective-mode LMMSE sum with weights computed elsewhere (the K-shard path's globally selected weights of
// this shard's components): h_b = sum_k w[b][k] (W_k y_b + b_k) on the FP64 sparse kernel (dense) or the Fourier
// kernel's weighted output (gmm_cplx_bussgang.py:216-218, :239-241 for one shard of the sum).
int qce_weighted_estimate(qce_model* m, const double2* y, long long B, const double* w, double2* h, hipStream_t st) {
  int rc = check_model(m, true);
  if (rc) return rc;
  if (B <= 0) return QCE_OK;
  DeviceGuard g(m->device);
  if (m->fft_active) {
    QceFftEstArgs fa = fft_args(m, y, B);
    fa.wts = w;
    fa.h = h;
    HIPCHK(qce_launch_fft_est(fa, 2, st));
    return QCE_OK;
  }
  if (m->big) return qce_big_wsum(m, y, B, w, h, m->N, st);
  HIPCHK(m->WT.ensure((size_t)m->K * m->M * m->N));
  HIPCHK(qce_launch_sparse_f64(B, m->N, m->M, m->K, y, w, m->W.p, m->bvec.p, m->WT.p, !m->wt_valid, h, st));
  m->wt_valid = 1;
  return QCE_OK;
}

extern "C" {

int qce_synchronize(qce_model* m) {
  if (!m) return fail(QCE_EARG, "null model");
  DeviceGuard g(m->device);
  HIPCHK(hipStreamSynchronize(m->stream));
  return check_status(m, true);
}

}  // extern "C"

#ifdef QCE_STAMPS
hipError_t qce_fft_set_stamps(unsigned long long* dev);
// diagnostic build only: stamp buffer of k_fft_wave (n 64-bit words on the device; n = 0 frees it) and
// its readback (8 segment cycle sums per wave of the launches since the last call with n > 0)
extern "C" int qce_debug_fft_stamps(unsigned long long* out, long long n) {
  static unsigned long long* d = nullptr;
  static long long cap = 0;
  if (n <= 0) {
    if (d) (void)hipFree(d);
    d = nullptr;
    cap = 0;
    return qce_fft_set_stamps(nullptr) == hipSuccess ? 0 : QCE_EHIP;
  }
  if (!d) {
    if (hipMalloc(&d, sizeof(unsigned long long) * n) != hipSuccess) return QCE_EHIP;
    cap = n;
    if (hipMemset(d, 0, sizeof(unsigned long long) * n) != hipSuccess) return QCE_EHIP;
    if (qce_fft_set_stamps(d) != hipSuccess) return QCE_EHIP;
    return 0;
  }
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return QCE_EHIP;
  if (hipMemcpy(out, d, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost) != hipSuccess) return QCE_EHIP;
  return (int)n;
}
// diagnostic build only: per-wave segment cycles (8 per wave) of the last k_est_all_f64 launch
extern "C" int qce_debug_f64_stamps(unsigned long long* out, long long n) {
  if (!g_f64_stamps) return QCE_ESTATE;
  if (n > g_f64_stamp_records * 8) n = g_f64_stamp_records * 8;
  if (hipDeviceSynchronize() != hipSuccess) return QCE_EHIP;
  if (hipMemcpy(out, g_f64_stamps, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost) != hipSuccess) return QCE_EHIP;
  return (int)n;
}
#endif
