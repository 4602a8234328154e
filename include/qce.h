/*
 * qce.h — C ABI of the MI355X-native Bussgang-GMM channel estimator (libqce.so).
 *
 * This is the drop-in boundary for the hot path of benediktfesl/Quantized_Channel_Estimation:
 * the per-SNR precompute and the per-batch estimate of `Gmm_nbit` (modules/gmm_cplx_bussgang.py)
 * and its twin `Gmm_quant` (modules/gmm_cplx_quant.py:190-457).  The Python host class
 * `quantized_channel_estimation_amd.Gmm_nbit` binds these entry points through ctypes
 * (INTEGRATION.md shows the binding a maintainer of the reference would add).
 *
 * Conventions
 *  - complex numbers are interleaved (re, im) doubles, numpy complex128 layout; all arrays are
 *    row-major (C order) and contiguous;
 *  - `io` selects where the caller's I/O buffers live: QCE_IO_HOST (host memory, the call is
 *    synchronous) or QCE_IO_DEVICE (device memory of the model's device, e.g. a torch tensor's
 *    data_ptr(); the call is asynchronous on `stream`, NULL = the model's own stream);
 *  - the library owns the per-model device tables; a model is bound to one device and is not
 *    thread-safe (use one model per thread/stream);
 *  - every entry point returns a status code (QCE_OK = 0); `qce_last_error()` returns the message
 *    of the last failure on the calling thread.  No C++ exception crosses the ABI.
 */
#ifndef QCE_H
#define QCE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qce_model qce_model;

/* status codes */
#define QCE_OK 0
#define QCE_EARG 1     /* invalid argument (shape, pointer, mode)            -> ValueError          */
#define QCE_ECHOL 2    /* Cr_k not positive definite (gmm_cplx_bussgang.py:43-46) -> ValueError      */
#define QCE_ENOTIMPL 3 /* configuration the kernels do not cover          -> NotImplementedError */
#define QCE_EHIP 4     /* HIP runtime failure                              -> RuntimeError        */
#define QCE_ESTATE 5   /* call order (estimate before prepare)             -> RuntimeError        */
#define QCE_ECOMM 6    /* communicator / collective failure (RCCL or host transport) -> RuntimeError */

/* estimate modes (gmm_cplx_bussgang.py:197-242) */
#define QCE_MODE_ALL 0  /* 'all': sum of all responsibility-weighted LMMSE estimates   (:220-228) */
#define QCE_MODE_TOPN 1 /* int n: top-n by responsibility, renormalised; n == 1 -> argmax (:197-219) */
#define QCE_MODE_CUMP 2 /* float p: shortest descending prefix with cumulative prob >= p (:229-242) */

/* quantiser kinds for multi-bit n_bits (gmm_cplx_bussgang.py:281-284) */
#define QCE_QUANT_UNIFORM 0
#define QCE_QUANT_LLOYD 1
#define QCE_QUANT_OTHER 2 /* any other string: the reference leaves the Bussgang gain at 0 */

/* model options (qce_model_set_option) */
#define QCE_OPT_BETA_FIRST 1 /* multi-bit Cr = g_0^2 Cy + (1 - g_0^2) diag(Cy) with the first Bussgang gain
                                (estimators/blmmse.py:53, :86) instead of clip(mean gain, 0, 1)
                                (gmm_cplx_bussgang.py:304-307); value != 0 enables */

#define QCE_OPT_PRECISION 2 /* arithmetic of the dense 'all' mode and the K-shard partial: QCE_PRECISION_F64 (default,
                               the reference's complex128 arithmetic: FP64 MFMA products, FP64 accumulation and
                               softmax) or QCE_PRECISION_FAST (fp16 two-term split products with fp32 accumulation,
                               ~1e-7 relative; an opt-in throughput mode) */
#define QCE_PRECISION_F64 0
#define QCE_PRECISION_FAST 1
#define QCE_OPT_RESERVE_CUS 3 /* CUs the persistent estimate kernels leave free (value >= 0; default 0): room for the
                                 collective kernels of a concurrent communication stream (qce_kshard_create sets it on
                                 the shard's models for RCCL at world > 1).  Keeps the prepared state. */

#define QCE_IO_HOST 0
#define QCE_IO_DEVICE 1

int qce_version(void);
/* Digest of the sources this library was built from (build.py: sha256 of the csrc .hip / .h files and qce.h). */
const char* qce_build_id(void);
const char* qce_last_error(void);
int qce_device_count(int* count);

/* Model parameters after `Gmm_nbit.fit` (gmm_cplx_bussgang.py:96-163): means_cplx (K,N) c128,
 * covs_cplx (K,N,N) c128, gm.weights_ (K,) f64.  Replaces the attribute bag the reference keeps in
 * its sklearn GaussianMixture (:86-94).  N <= 256 (padded internally to 16/32/64/128/256), K <= 4096 for
 * the selective modes and the proba / labels outputs (any K for 'all').  The structure of the covariances is
 * detected here (qce_model_structure). */
int qce_model_create(int K, int N, const double* means_cplx, const double* covs_cplx, const double* weights,
                     int device, qce_model** out);
int qce_model_destroy(qce_model* model);
/* Replace the parameters of a model in place (same K, N; e.g. between EM iterations): re-uploads
 * means / covariances / weights, re-detects the structure and drops the prepared state. */
int qce_model_set_params(qce_model* model, const double* means_cplx, const double* covs_cplx, const double* weights);

/* Per-SNR precompute: `_prepare_for_prediction` (gmm_cplx_bussgang.py:246-328).
 * A: (M,N) c128 observation matrix, or NULL for the identity (estimate_from_y :191-192).
 * n_bits: 1..16 (uniform; beyond 8 bits the step is the reference's asymptote 4 sqrt(b) 2^-b,
 * uniform_quantizer.py:15-21; lloyd: 1..8) or +INFINITY (np.inf).  thresholds (2^b-1) / labels (2^b) are the
 * quantiser tables of the lloyd kind (lloyd_max_quantizer.py:24-37); NULL otherwise.
 * Runs asynchronously on `stream` (NULL = the model's stream; pass the stream later estimates use so a prepare
 * never overwrites tables an in-flight estimate still reads); no host synchronisation.  The per-component
 * Cholesky status is copied behind the prepare's kernels and read at the next call that synchronises anyway
 * (host-I/O estimates, qce_log_prob, qce_get_tables, qce_synchronize, host-I/O qce_cconst_max), which returns
 * QCE_ECHOL if some Cr_k is not positive definite (:43-46).  Device-I/O estimates issued in between compute on
 * NaN tables; device-I/O callers read the status through qce_cconst_max (it writes +inf on a failure). */
int qce_prepare(qce_model* model, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                const double* thresholds, const double* labels, int n_levels, void* stream);

/* Channel estimates: `estimate_from_y` (gmm_cplx_bussgang.py:166-243) for y (B,M) c128 -> h (B,N) c128.
 * mode/mode_param: QCE_MODE_ALL; QCE_MODE_TOPN with n; QCE_MODE_CUMP with p. */
int qce_estimate(qce_model* model, const double* y, int64_t B, int mode, double mode_param, double* h_out, int io,
                 void* stream);

/* `_estimate_weighted_log_prob` (:369-386) -> lp (B,K) f64; `predict_proba_cplx` (:351-367) -> proba (B,K);
 * `_predict_cplx` (:335-349) -> labels (B,) int64.  Any output pointer may be NULL. */
int qce_log_prob(qce_model* model, const double* X, int64_t B, double* lp_out, double* proba_out,
                 int64_t* labels_out, int io, void* stream);

/* K-shard partial of the 'all' mode for the components this model holds: per sample the running max
 * m (B,) f64, the sum s = sum_k exp(lp_k - m) (B,) f64 and acc = sum_k exp(lp_k - m) (W_k y + b_k)
 * (B, 2N) f32 interleaved; h = (sum_g acc_g e^{m_g}) / (sum_g s_g e^{m_g}). */
int qce_estimate_partial(qce_model* model, const double* y, int64_t B, double* m_out, double* s_out, float* acc_out,
                         int io, void* stream);

/* The same partial with an FP64 accumulator acc (B, 2N) f64 interleaved — the format the K-shard combine
 * all-reduces (one SUM of (s, acc) under a shared shift, sharding.py). */
int qce_estimate_partial_f64(qce_model* model, const double* y, int64_t B, double* m_out, double* s_out, double* acc_out,
                             int io, void* stream);

/* The K-shard partial scaled to a shift shared by all shards and packed for one SUM collective:
 * packed_out (B, 2N+2) f64, row b = [s_b e^{m_b - shift}, 0, acc_b e^{m_b - shift} (2N interleaved)].
 * shift: one double where `io` says (device memory for QCE_IO_DEVICE, so the shift can come from a device-side
 * collective without a host round trip).  With shift = max over ALL components of cconst (>= every lp, the quad
 * form is >= 0) the element-wise sum over shards of these rows gives h_b = acc / s exactly (rows whose sum
 * underflows to s = 0 need the two-step combine of the unshifted partials). */
int qce_estimate_partial_shifted(qce_model* model, const double* y, int64_t B, const double* shift, double* packed_out,
                                 int io, void* stream);

/* out[0] = max_k cconst_k of the last prepare (this shard's part of the shift above; the caller reduces it over
 * shards with a MAX collective), or +INFINITY if the prepare's Cholesky factorisation failed for some component:
 * the failure then travels with the shift through the MAX collective to every shard (sharding.py raises the
 * reference's ValueError).  `out` where `io` says; device I/O is asynchronous on `stream`, host I/O synchronises
 * and returns QCE_ECHOL on a failure. */
int qce_cconst_max(qce_model* model, double* out, int io, void* stream);

/* Per-SNR tables for state mirroring (the reference mutates gm.means_, gm.covariances_,
 * gm.precisions_cholesky_, :262-313) and tests.  Host pointers, any may be NULL:
 * means_y (K,M), Cy (K,M,M), Cr (K,M,M), P (K,M,M) = (L^-1)^H, A_eff (K,M,N), W (K,N,M),
 * b (K,N), cconst (K,) = -M log(pi) + 2 log det P_k + log w_k. */
int qce_get_tables(qce_model* model, double* means_y, double* Cy, double* Cr, double* P, double* A_eff, double* W,
                   double* b, double* cconst);

/* Dimensions of the prepared state (M <= 256): M (0 before the first prepare). */
int qce_model_info(qce_model* model, int* K, int* N, int* M, int* device);

/* Structure of the mixture found at creation: every C_k is block-circulant for kron(F_n1, F_n2) (n1 = 1:
 * circulant, the fits of gmm_cplx_bussgang.py:104-133), or n1 = n2 = 0.  With A = I such a model is
 * prepared and estimated in the Fourier domain (per-bin tables; fourier_active = 1 after such a prepare).
 * Environment QCE_FFT=0 keeps every prepare on the dense path. */
int qce_model_structure(qce_model* model, int* n1, int* n2, int* fourier_active);
/* The 'all'-mode kernel family the last prepare selected (diagnostics, benchmarks): */
#define QCE_KERNEL_NONE 0     /* not prepared */
#define QCE_KERNEL_F64_4M 1   /* k_est_all_f64: real 2x2 embedding, FP64 MFMA (padded M, N up to 128) */
#define QCE_KERNEL_F64_3M 2   /* k_est_all_f64g: Gauss 3-product complex multiply, FP64 MFMA (padded M, N <= 64) */
#define QCE_KERNEL_F64_WIDE 3 /* k_lp_f64 + k_wsum_f64 (padded 256) */
#define QCE_KERNEL_BIG 4      /* GEMM path, N or M in (256, 4096] */
#define QCE_KERNEL_FOURIER 5  /* (block-)circulant models in the Fourier basis */
#define QCE_KERNEL_FAST 6     /* precision 'fast': fp16 two-term split */
int qce_model_kernel(qce_model* model, int* kind);

/* Observations on the device (model-free): `get_observation_nbit` (utils.py:241-251) with `quant`
 * (utils.py:189-203):  y = Q(A h + noise_scale * w).
 * h (B,N) c128; A (M,N) c128 host array or NULL for the identity (then M == N); y_out (B,M) c128.
 * noise_kind: 0 none (pure quantiser, `quant`), 1 w supplied in `noise` (B,M) c128 — the reference's
 * crandn draw, result bit-identical to numpy for A = NULL —, 2 generated on the device: circular
 * CN(0,1) from Philox4x32-10 keyed by `seed`, complex element e of the batch uses counter offset + e.
 * n_bits: 1 (sign law), +INFINITY (no quantisation), else labels[np.digitize(.)] with thresholds
 * (n_levels - 1, increasing) and labels (n_levels) host arrays.  h / noise / y_out live where `io` says;
 * `stream` NULL = the null stream of `device`. */
int qce_observe(const double* h, int64_t B, int N, const double* A, int M, double noise_scale, int noise_kind,
                const double* noise, uint64_t seed, uint64_t offset, double n_bits, const double* thresholds,
                const double* labels, int n_levels, double* y_out, int device, int io, void* stream);

/* out[0] = sum |a_i - b_i|^2 over n complex values (the scripts' MSE numerator, Bussgang_GMM.py:289);
 * deterministic reduction order.  `out` is host memory for QCE_IO_HOST, device memory otherwise. */
int qce_sq_error(const double* a, const double* b, int64_t n, double* out, int device, int io, void* stream);

/* EM training on the device (gmm_cplx_bussgang.py:437-790, `fit_cplx` / `_e_step` / `_m_step`).
 * E-step: the model must be prepared as the fit's channel-domain model (A = NULL, snr_db = +INFINITY,
 * n_bits = +INFINITY: Cr = C).  resp_out (B,K) f64 = exp(log_resp) (:612-656, :676);
 * mean_lse_out[0] = mean_b logsumexp_k lp (the lower bound, :629).  Both where `io` says. */
int qce_em_estep(qce_model* model, const double* X, int64_t B, double* resp_out, double* mean_lse_out, int io,
                 void* stream);

/* M-step `estimate_gaussian_parameters` (:698-737): X (B,N) c128, resp (B,K) f64 ->
 * nk_out (K,) = sum_b resp + 10 eps, means_out (K,N) c128 (zeros when zero_mean), and
 * diag == 0: covs_out (K,N,N) c128 ('full', :739-765); diag != 0: covs_out (K,N) f64 ('diag', :767-790).
 * N <= 256.  Buffers where `io` says (model-free; `stream` NULL = the null stream of `device`). */
int qce_em_mstep(const double* X, int64_t B, int N, int K, const double* resp, double reg_covar, int diag,
                 int zero_mean, double* nk_out, double* means_out, double* covs_out, int device, int io,
                 void* stream);

/* Set a model option (QCE_OPT_*); drops the prepared state. */
int qce_model_set_option(qce_model* model, int option, double value);

/* Per-sample filters: h_b = W_c y_b + b_c with c = comp[b] (int64, B entries, NULL: c = b, B <= K).
 * The genie Bussgang-LMMSE (estimators/blmmse.py:20-62) is a model with one component per sample
 * (C_b = toeplitz(t_b)^T) estimated this way.  y / comp / h_out where `io` says. */
int qce_estimate_assigned(qce_model* model, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                          void* stream);

/* Bussgang least squares (estimators/LS.py: lstsq(A_eff, y)) with the prepared A_eff of component c = comp[b]
 * (NULL: c = b).  Requires column-orthogonal A_eff (A = NULL or kron(x, I), the scripts' pilot matrices):
 * h_i = sum_m conj(A_eff[m][i]) y_m / sum_m |A_eff[m][i]|^2. */
int qce_estimate_ls(qce_model* model, const double* y, int64_t B, const int64_t* comp, double* h_out, int io,
                    void* stream);

/* Bussgang least squares for a general pilot matrix with full column rank (M >= N): h_b = pinv(A_eff_c) y_b,
 * the same solution as estimators/LS.py:32,47,73 (np.linalg.lstsq(A_eff, y)) for full-rank A_eff.  The
 * pseudo-inverses are formed on the device per call (normal equations, Gauss-Jordan).  M < N -> QCE_ENOTIMPL. */
int qce_estimate_ls_general(qce_model* model, const double* y, int64_t B, const int64_t* comp, double* h_out,
                            int io, void* stream);

/* Toeplitz / block-Toeplitz inverse-EM covariance step (gmm_cplx_bussgang.py:792-826, Barton & Fuhrmann):
 * S (K,N,N) c128 = the M-step's weighted sample covariances WITHOUT reg; F2 (P,N) c128 the partial DFT of
 * `fit` (:143-153); sigma (K,P) f64 in/out.  init != 0 (_initialize, :582-586): sigma = max(Re diag(F2 S F2^H), reg),
 * `model` unused.  init == 0: `model` is prepared on the previous covariances (A = NULL, snr = inf, n_bits = inf:
 * its L^-1 gives Cinv); sigma += sigma^2 Re diag(F2 (Cinv S Cinv - Cinv) F2^H), max reg;
 * covs_out (K,N,N) = F2^H diag(sigma) F2 + reg I.  Host buffers; synchronous. */
int qce_em_toeplitz(qce_model* model, const double* S, int K, int N, const double* F2, int P, double* sigma, double reg,
                    int init, double* covs_out, int device, void* stream);

/* SCM multi-path channels (modules/SCM3GPP/SCMMulti.py:30-56 generate_channel, scm_helper.py:17-84):
 * h_out (B, n_coherence, N) complex64, t_out (B, N) complex64 (first covariance rows).  gains / angles
 * (B, n_path) f64 (normalised gains, angles in degrees) and x (B, 100 N, n_coherence) c128 (the crandn draw)
 * may be supplied — the reference's own draws give its channels to float32 rounding — or NULL: then drawn on the
 * device from Philox4x32-10 keyed by `seed`.  N <= 256, n_path <= 16.  Buffers where `io` says. */
int qce_scm_generate(int64_t B, int n_coherence, int N, int n_path, double path_sigma, const double* gains,
                     const double* angles, const double* x, uint64_t seed, float* h_out, float* t_out, int device,
                     int io, void* stream);

/* Statistical achievable-rate lower bound of the scripts (Bussgang_GMM.py:146-162 and its copies
 * :206-216, :238-249, :291-306): g_b = h_est_b / max(||h_est_b||^2, norm_clip) (norm_clip 0: no clip; the
 * GMM branch uses 0.1), inner_b = g_b^H diag(buss) h_b, den2_b = Re g_b^H Cq g_b;
 * out[0] = log2(1 + num / (den1 + den2)), out[1] = num = |mean inner|^2, out[2] = den1 = var(inner),
 * out[3] = den2 = mean den2_b.  h_est / h (B,N) c128 where `io` says; buss (N,) f64, Cq (N,N) c128 and out
 * host; synchronous. */
int qce_rate_bound(const double* h_est, const double* h, int64_t B, int N, const double* buss, const double* Cq,
                   double norm_clip, double* out, int device, int io, void* stream);

/* Per-sample matched-filter rate of the scripts' LS branch (Bussgang_GMM.py:186-198): g = (buss o h_est_b)^H Cq^-1,
 * out[0] = mean_b Re log2(1 + |g B h_est_b|^2 / (g Cq g^H + |g B (h_b - h_est_b)|^2)), B = diag(buss).  Cq^-1 is
 * formed on the device (Cq Hermitian, full rank: equal to np.linalg.pinv to rounding).  h_est / h (B,N) c128
 * where `io` says; buss (N,) f64, Cq (N,N) c128 and out host; N <= 256; synchronous. */
int qce_rate_mf(const double* h_est, const double* h, int64_t B, int N, const double* buss, const double* Cq,
                double* out, int device, int io, void* stream);

/* Page-locked host memory (hipHostMalloc / hipHostFree).  QCE_IO_HOST calls DMA straight from / into page-locked
 * arrays (and from / into pageable ones they can register for the call): a caller that allocates its result arrays
 * here, and reuses them, saves the page faults of fresh pageable memory (the Python layer's result pool, _lib.py). */
int qce_host_alloc(size_t bytes, void** out);
int qce_host_free(void* p);

/* Device synchronisation of the model's stream (for timing and for QCE_IO_DEVICE callers). */
int qce_synchronize(qce_model* model);

/* ---------------------------------------------------------------------------------------------------------------
 * K-shard estimation over a communicator.  Replaces the reference's only parallelism,
 * a process pool over SNR points (Bussgang_GMM.py:29-32, :287), by one process per GPU, each holding a contiguous
 * slice of the mixture's components (qce_kshard_slice), with the collectives issued by the library itself:
 * RCCL (ncclAllReduce / ncclReduceScatter / ncclAllGather over xGMI) or a caller-supplied host transport.
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct qce_comm qce_comm;
typedef struct qce_kshard qce_kshard;

#define QCE_COMM_ID_BYTES 128 /* ncclUniqueId */
#define QCE_COMM_RCCL 0
#define QCE_COMM_HOST 1

/* collective ops of a host transport; all data are doubles */
#define QCE_COLL_ALLREDUCE_SUM 0 /* recv[i] = sum_r send_r[i], count elements                          */
#define QCE_COLL_ALLREDUCE_MAX 1 /* recv[i] = max_r send_r[i], count elements                          */
#define QCE_COLL_REDUCE_SCATTER_SUM 2 /* send: world * count, recv[i] = sum_r send_r[rank * count + i]  */
#define QCE_COLL_ALLGATHER 3     /* send: count, recv[r * count + i] = send_r[i]                      */

/* A host transport (MPI, gloo, ...): called synchronously with host buffers (the library has synchronised the
 * stream and staged the device data); returns 0 on success. */
typedef int (*qce_host_collective)(void* user, int op, const double* send, double* recv, int64_t count);

/* ncclGetUniqueId: called on one rank, the QCE_COMM_ID_BYTES bytes are then shared with every rank. */
int qce_comm_unique_id(void* id_out);
/* ncclCommInitRank on `device` (collective over the `world` ranks). */
int qce_comm_init(const void* unique_id, int rank, int world, int device, qce_comm** out);
/* A communicator whose collectives go through the caller's host transport `fn` (`user` passed through). */
int qce_comm_init_host(int rank, int world, int device, qce_host_collective fn, void* user, qce_comm** out);
int qce_comm_destroy(qce_comm* comm);
int qce_comm_info(qce_comm* comm, int* rank, int* world, int* device, int* kind);

/* Components [lo, hi) of rank `rank` in the balanced contiguous split of K over `world` ranks (K >= world). */
int qce_kshard_slice(int K, int world, int rank, int* lo, int* hi);
/* Rows of h_out a rank receives from qce_kshard_estimate: per pipeline chunk the global row range
 * [ranges[2i], ranges[2i+1]) (concatenated in h_out in this order); scatter = 0: every rank gets all B rows.
 * `cap` = number of ranges the array holds; *n = ranges written.  Selective modes use chunks = 1. */
int qce_kshard_rows(int64_t B, int chunks, int world, int rank, int scatter, int64_t* ranges, int cap, int* n);

/* A K-shard estimator: `shard` holds components qce_kshard_slice(K_total, world, rank) of the mixture (a model
 * created from that slice), `comm` its communicator.  Neither is owned. */
int qce_kshard_create(qce_model* shard, qce_comm* comm, int K_total, qce_kshard** out);
int qce_kshard_destroy(qce_kshard* ks);
/* Double-buffered tables: `spare` is a second model of the same shard (same parameters; not owned).  Prepares then
 * alternate between the two table sets on the library's prepare stream: prepare t+1 waits only for the last step
 * that read its set (step t-1), so it runs beside step t's partial kernels (Bussgang_GMM.py:284-287: the next SNR
 * point's tables do not depend on the current estimate).  A prepare issues no collective. */
int qce_kshard_set_spare(qce_kshard* ks, qce_model* spare);
/* Per-SNR prepare of the shard (qce_prepare) and the shard's shift M_r = max over its components of
 * c_k = -M log(pi) + 2 log det P_k + log w_k (>= every local lp: the quad form is >= 0; +inf when a Cholesky
 * factorisation failed).  No collective and no host synchronisation: the shards agree on M* = max_r M_r at the start
 * of the next qce_kshard_estimate, on the library's communication stream. */
int qce_kshard_prepare(qce_kshard* ks, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                       const double* thresholds, const double* labels, int n_levels, void* stream);
/* One estimate step over y (B, M) c128 in device memory (the same y on every rank).  Its first collective is an
 * 8-byte MAX of the shards' shifts M_r (M*); every collective of the library is issued on one communicator from its
 * communication stream, so all ranks issue them in the same order.
 * QCE_MODE_ALL (gmm_cplx_bussgang.py:220-228): per chunk the shard's FP64 partial rows [s e^{m-M_r}, 0,
 * acc e^{m-M_r}] (qce_estimate_partial_shifted) and one SUM collective of them on the communication stream
 * (reduce-scatter, scatter != 0, or all-reduce) that scales each shard's rows by e^{M_r - M*} on the way in (RCCL
 * PreMulSum, scalar in device memory), overlapped with the next chunk's kernel; h = acc / s.  QCE_MODE_TOPN / QCE_MODE_CUMP (:197-219, :229-242): n == 1 all-gathers each shard's (max lp, index)
 * and the owner of the first global maximum contributes W_j y + b_j; otherwise the shards' lp are all-gathered,
 * every rank selects the same components (k_select on the full lp) and the shards' weighted filter sums are
 * summed (one chunk).  h_out: device memory, the rows qce_kshard_rows names.  A 2-double MAX of the step's flag
 * word [rows whose shifted sum underflowed, Cholesky failure on any rank] closes the step; nothing is read on the
 * host until qce_kshard_finish.  The step's collectives and row finalisation run on the library's communication
 * stream and may still be in flight when the next step's kernels start on `stream` (the send rows alternate between
 * two buffers); h_out is complete once qce_kshard_finish returned, which also orders `stream` after the step.  y and
 * every h_out since the last finish must stay valid until then. */
int qce_kshard_estimate(qce_kshard* ks, const double* y, int64_t B, int mode, double mode_param, int chunks,
                        int scatter, double* h_out, void* stream);
/* The caller's sync point: reads the flag words (one host synchronisation).  QCE_ECHOL with the reference's
 * message (gmm_cplx_bussgang.py:43-46) if a Cholesky factorisation failed on any rank -- on every rank; rows of
 * the last step whose shifted sum underflowed are recombined exactly (collective: per-row MAX of the shards'
 * running maxima, then the SUM); QCE_ESTATE if an earlier, already superseded step had such rows. */
int qce_kshard_finish(qce_kshard* ks, void* stream);
/* The flag words the last qce_kshard_finish read: [rows of the last step recombined exactly, Cholesky failure on
 * some rank, the same two for the superseded steps before it] (diagnostics and tests). */
int qce_kshard_flags(qce_kshard* ks, double* out4);
/* Kernel timing of the shard's estimate launches (HIP events around each partial / lp launch on the compute
 * stream): enable != 0 starts recording (clears earlier records); qce_kshard_kernel_ms synchronises on the
 * recorded events, returns their summed duration and count, and clears them. */
int qce_kshard_timing(qce_kshard* ks, int enable);
int qce_kshard_kernel_ms(qce_kshard* ks, double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif
#endif /* QCE_H */
