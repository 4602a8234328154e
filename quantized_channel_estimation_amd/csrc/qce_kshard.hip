// K-shard estimation over a communicator (include/qce.h).
//
// The reference's only parallelism is a process pool over SNR points (Bussgang_GMM.py:29-32, :287); here one
// SNR point's mixture is split over the GPUs of a node by components, one process per GPU, and the library issues
// the collectives itself -- RCCL over xGMI (ncclAllReduce / ncclReduceScatter / ncclAllGather on device buffers) or
// a caller-supplied host transport (the library stages through pinned host memory).
//
// 'all' mode (gmm_cplx_bussgang.py:220-228): every shard's estimate is written scaled by its own y-independent
// shift M_r = max_{k in shard} c_k (>= every local lp_bk because the quad form is >= 0), with no collective between
// the prepare and the kernel; the step's first collective (an 8-byte MAX on the communication stream) agrees on
// M* = max_r M_r, and every SUM multiplies the shard's rows by e^{M_r - M*} on the way in (RCCL's PreMulSum with the
// scalar in device memory for all-reduces; a scaling kernel before a reduce-scatter -- RCCL 2.26.6's PreMulSum
// reduce-scatter drops tail elements, see reduce_chunks -- and before a host transport), so one SUM of the packed rows
// [s e^{m - M*}, 0, acc e^{m - M*}] over the shards gives h = acc / s.  Every collective of the library is issued on
// one communicator from one stream, so every rank issues them in the same order.  The batch is cut into chunks; chunk i's
// reduce-scatter runs on the communication stream while chunk i+1's partial kernel runs on the compute stream.
// Rows whose shifted sum leaves the normal FP64 range are counted on the device; one 2-double MAX per step agrees
// on the flag word [flagged rows, Cholesky failure], read once at qce_kshard_finish, which recombines the flagged
// step exactly with a per-row shift (MAX of the shards' running maxima, then the SUM).
//
// Selective modes (:197-219, :229-242): argmax all-gathers each shard's (max lp, index) and the owner of the first
// global maximum contributes W_j y + b_j; top-n / cumulative-p all-gather the shards' lp so that every rank runs
// the same FP64 selection (k_select) on the full row and contributes its own components' weighted filters.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "../../include/qce.h"
#include "qce_common.h"
#include "qce_model.h"

namespace {

// a row whose shifted sum is below this is recombined exactly (sharding.py UNDERFLOW_S): above it every term that
// matters is a normal double, so the shifted sums carry full FP64 precision
constexpr double kUnderflowS = 1e-290;

const char* kCholMessage =
    "Fitting the mixture model failed because some components have ill-defined empirical covariance "
    "(for instance caused by singleton or collapsed samples). Try to decrease the number of "
    "components, or increase reg_covar.";

#define KS_HIP(expr)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return qce_set_error(QCE_EHIP, std::string(#expr) + " failed: " + hipGetErrorString(e_));    \
  } while (0)

#define KS_RC(expr)             \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != QCE_OK) return rc_; \
  } while (0)

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev && hipSetDevice(dev) != hipSuccess) (void)hipGetLastError();  // no sticky error left behind
  }
  ~DevGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct Chunk {
  long long lo, hi;    // global rows of the chunk
  long long npad;      // rows of the collective's send buffer (multiple of world under reduce-scatter)
  long long r0, nv;    // this rank's rows of the chunk: [r0, r0 + nv)
  long long pk_off;    // row offset of the chunk in the send buffer
  long long rs_off;    // row offset in the receive buffer (reduce-scatter)
  long long h_off;     // row offset in h_out
};

// sharding.chunk_bounds: with scatter every chunk but the last holds a multiple of `world` rows
std::vector<Chunk> chunk_layout(long long B, int chunks, int world, int rank, bool scatter) {
  std::vector<Chunk> out;
  if (B <= 0) return out;
  long long c = chunks < 1 ? 1 : chunks;
  const long long cap = B / (world > 1 ? world : 1);
  if (c > (cap > 1 ? cap : 1)) c = cap > 1 ? cap : 1;
  long long step = (B + c - 1) / c;
  if (scatter) step = (step + world - 1) / world * world;
  long long pk = 0, rs = 0, ho = 0;
  for (long long lo = 0; lo < B;) {
    Chunk ch;
    ch.lo = lo;
    ch.hi = lo + step < B ? lo + step : B;
    const long long n = ch.hi - ch.lo;
    if (scatter) {
      ch.npad = (n + world - 1) / world * world;
      const long long q = ch.npad / world;
      ch.r0 = ch.lo + rank * q;
      const long long e = ch.r0 + q < ch.hi ? ch.r0 + q : ch.hi;
      ch.nv = e > ch.r0 ? e - ch.r0 : 0;
      ch.rs_off = rs;
      rs += q;
    } else {
      ch.npad = n;
      ch.r0 = ch.lo;
      ch.nv = n;
      ch.rs_off = 0;
    }
    ch.pk_off = pk;
    pk += ch.npad;
    ch.h_off = ho;
    ho += ch.nv;
    out.push_back(ch);
    lo = ch.hi;
  }
  return out;
}

// CUs the shard's persistent estimate kernels leave free for other streams (QCE_KSHARD_RESERVE_CUS, default 0).
// Round 6 measured that free CUs beside the persistent grid do not buy overlap: the dispatcher places a kernel's
// workgroups on the shader engines in order and a workgroup whose engine has no free CU blocks the ones behind it, so
// a kernel with more than ~2 workgroups per XCD (the prepare's, the row scaling, RCCL's channels) waits for the
// persistent grid to retire anyway (tools/probe/overlap_probe.hip, profiles/r06_overlap_probe*.jsonl), while the
// grid itself loses reserve / 256 of its CUs (emulated world-8 rank step, K = 16: 1.12 ms at 0, 1.16 ms at 16)
int kshard_reserve_cus() {
  const char* e = getenv("QCE_KSHARD_RESERVE_CUS");
  const int v = e ? atoi(e) : 0;
  return v < 0 ? 0 : v;
}

// Test hook QCE_KSHARD_EMULATE_WORLD="W[:R]" (a world-1 communicator only): lay the step's rows out as rank R of W
// ranks would -- the shard computes its components over all B rows, but its reduce-scatter takes and returns only
// the rank's B / W rows and only those are finalised -- so one GPU rehearses the per-rank work of a W-GPU step
// (the collective's wire time is the part one GPU cannot show)
bool kshard_emulated(int* world, int* rank) {
  const char* e = getenv("QCE_KSHARD_EMULATE_WORLD");
  if (!e || !*e) return false;
  char* end = nullptr;
  const long w = strtol(e, &end, 10);
  if (end == e) return false;
  long r = 0;
  if (*end == ':') {
    char* e2 = nullptr;
    r = strtol(end + 1, &e2, 10);
    if (e2 == end + 1 || *e2) return false;
  } else if (*end) {
    return false;
  }
  if (w < 2 || w > 4096 || r < 0 || r >= w) return false;
  *world = (int)w;
  *rank = (int)r;
  return true;
}

void slice_of(int K, int world, int rank, int* lo, int* hi) {
  const int base = K / world, rem = K % world;
  *lo = rank * base + (rank < rem ? rank : rem);
  *hi = *lo + base + (rank < rem ? 1 : 0);
}

// ---------------------------------------------------------------------------------------------------------------
// kernels (HBM-bound row passes; grid-stride, 256 threads)
// ---------------------------------------------------------------------------------------------------------------
unsigned grid_for(long long n) {
  long long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// the row passes that run beside the next prepare (the send rows' scaling, the finalisation): their grid capped at
// QCE_KSHARD_ROWPASS_WG workgroups (grid-stride), so they do not queue thousands of workgroups ahead of the prepare's
// kernels in the dispatcher (A/B knob; 0 or unset = grid_for)
unsigned rowpass_grid(long long n) {
  static const long cap = [] {
    const char* e = getenv("QCE_KSHARD_ROWPASS_WG");
    return e ? atol(e) : 0L;
  }();
  const unsigned g = grid_for(n);
  return (cap > 0 && (long)g > cap) ? (unsigned)cap : g;
}

// h[r] = acc[r] / s[r] from packed rows [s, 0, acc (2N)]; rows with s below the normal range are counted
__global__ __launch_bounds__(256) void k_ks_finalize(long long n, int N, const double* __restrict__ rows,
                                                     double2* __restrict__ h, double thr, unsigned* __restrict__ cnt) {
  const long long W = 2LL * N + 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n * N; i += (long long)gridDim.x * 256) {
    const long long b = i / N, j = i % N;
    const double* r = rows + b * W;
    const double s = r[0];
    const double2 a = *reinterpret_cast<const double2*>(r + 2 + 2 * j);
    h[b * N + j] = make_double2(a.x / s, a.y / s);
    if (j == 0 && s < thr) atomicAdd(cnt, 1u);
  }
}

// fl = [flagged rows, Cholesky failure on this rank (its shift slot carries +inf after the MAX)]
__global__ void k_ks_flags(const unsigned* __restrict__ cnt, const double* __restrict__ shift, int local_chol,
                           double* __restrict__ fl) {
  if (threadIdx.x == 0) {
    fl[0] = cnt ? (double)*cnt : 0.0;
    fl[1] = (local_chol || isinf(*shift) || isnan(*shift)) ? 1.0 : 0.0;
  }
}

// earlier = max(earlier, fl): a superseded step's flags (every step before the last is accounted for)
__global__ void k_ks_fold(double* __restrict__ earlier, const double* __restrict__ fl) {
  if (threadIdx.x < 2) earlier[threadIdx.x] = fmax(earlier[threadIdx.x], fl[threadIdx.x]);
}

// [m, s, acc] partial -> packed rows scaled by a per-row shift mg (the exact recombination of flagged steps)
__global__ __launch_bounds__(256) void k_ks_pack_rowshift(long long B, int N, const double* __restrict__ m,
                                                          const double* __restrict__ s, const double* __restrict__ acc,
                                                          const double* __restrict__ mg, double* __restrict__ pk) {
  const long long W = 2LL * N + 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < B * W; i += (long long)gridDim.x * 256) {
    const long long b = i / W, j = i % W;
    const double sc = (m[b] == -__builtin_inf()) ? 0.0 : exp(m[b] - mg[b]);
    const double v = j == 0 ? s[b] : (j == 1 ? 0.0 : acc[b * 2 * N + j - 2]);
    pk[i] = v * sc;
  }
}

// sh = [M_r, M_r]: the shard's shift of the step's table set, the second slot the MAX's input (on the communication
// stream, so the compute stream carries no copy between two partial kernels)
__global__ void k_ks_shift_in(const double* __restrict__ src, double* __restrict__ sh) {
  if (threadIdx.x < 2) sh[threadIdx.x] = *src;
}

// test hook of the exact recombination (QCE_KSHARD_SHIFT_BIAS): raise the agreed shift so rows leave the range
__global__ void k_ks_add(double* __restrict__ v, double d) {
  if (threadIdx.x == 0) v[0] += d;
}

// sh = [M_r, M*] (M* after the MAX): sc = e^{M_r - M*} <= 1, the factor the shard's rows enter the SUM with.  A failed
// factorisation somewhere (M* = +inf) gives 0 or NaN here; the step's flag word raises before any row is read.
// bias > 0 (test hook QCE_KSHARD_GLOBAL_BIAS) raises M* so the scaled rows leave the normal range.
__global__ void k_ks_scale_of(double* __restrict__ sh, double bias, double* __restrict__ sc) {
  if (threadIdx.x == 0) {
    sh[1] += bias;
    sc[0] = exp(sh[0] - sh[1]);
  }
}

// test hook QCE_KSHARD_CS_DELAY_US: hold the communication stream for `ticks` of the 100 MHz-class wall clock at the
// start of a step, so the steps' collectives lag far behind the compute stream (tests of the send-row hand-off)
__global__ void k_ks_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

// host transports: the PreMulSum's multiplication done in place before the rows are staged
__global__ __launch_bounds__(256) void k_ks_scale_rows(long long n, double* __restrict__ v,
                                                       const double* __restrict__ sc) {
  const double f = *sc;
  if ((reinterpret_cast<uintptr_t>(v) & 15) == 0) {  // 16-byte accesses, then the odd last element
    double2* v2 = reinterpret_cast<double2*>(v);
    const long long n2 = n >> 1;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
      const double2 a = v2[i];
      v2[i] = make_double2(a.x * f, a.y * f);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) v[n - 1] *= f;
    return;
  }
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) v[i] *= f;
}

// one-time check of RCCL's PreMulSum reduce-scatter at a given count (see reduce_chunks): send[j] = j mod P + 1 on
// every rank, scalar 0.5 in pr[0]; rank r's slice must come back as world * 0.5 * (send value at r count + i)
constexpr long long kProbeP = 1048573;
__global__ __launch_bounds__(256) void k_ks_probe_fill(double* __restrict__ send, long long n, double* __restrict__ pr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    pr[0] = 0.5;
    pr[1] = 0.0;
  }
  for (long long j = (long long)blockIdx.x * 256 + threadIdx.x; j < n; j += (long long)gridDim.x * 256)
    send[j] = (double)(j % kProbeP + 1);
}
__global__ __launch_bounds__(256) void k_ks_probe_check(const double* __restrict__ recv, long long count, int world,
                                                        int rank, double* __restrict__ bad) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < count; i += (long long)gridDim.x * 256) {
    const double want = world * 0.5 * (double)(((long long)rank * count + i) % kProbeP + 1);
    if (recv[i] != want) *bad = 1.0;  // every writer stores the same value
  }
}

// first maximum of each lp row (numpy argmax) as (value, index) doubles, one wave per row
__global__ __launch_bounds__(256) void k_ks_row_argmax(long long B, int K, const double* __restrict__ lp,
                                                       double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  double bv = -__builtin_inf();
  int bi = 1 << 30;
  for (int k = lane; k < K; k += 64) {
    const double v = lp[b * K + k];
    if (v > bv || bi == (1 << 30)) {
      bv = v;
      bi = k;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    out[2 * b] = bv;
    out[2 * b + 1] = (double)bi;
  }
}

// global winner of the gathered (value, local index) pairs: larger value, ties to the lower rank (= lower global
// index, the shards are contiguous); the owner's weight row is one-hot, every other rank's row is zero
__global__ __launch_bounds__(256) void k_ks_argmax_weights(long long B, int world, int rank, int Kl,
                                                           const double* __restrict__ g, double* __restrict__ w) {
  for (long long b = (long long)blockIdx.x * 256 + threadIdx.x; b < B; b += (long long)gridDim.x * 256) {
    double bv = -__builtin_inf();
    int br = -1, bi = 0;
    for (int r = 0; r < world; ++r) {
      const double v = g[((long long)r * B + b) * 2];
      if (br < 0 || v > bv) {
        bv = v;
        br = r;
        bi = (int)g[((long long)r * B + b) * 2 + 1];
      }
    }
    for (int k = 0; k < Kl; ++k) w[b * Kl + k] = (br == rank && k == bi) ? 1.0 : 0.0;
  }
}

// lp (B x Kl) -> (B x Kmax), padded with -inf (equal all-gather counts)
__global__ __launch_bounds__(256) void k_ks_pad(long long B, int Kl, int Kmax, const double* __restrict__ lp,
                                                double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < B * Kmax; i += (long long)gridDim.x * 256) {
    const long long b = i / Kmax;
    const int k = (int)(i % Kmax);
    out[i] = k < Kl ? lp[b * Kl + k] : -__builtin_inf();
  }
}

// gathered (world x B x Kmax) -> the full row-major lp (B x K) in global component order
__global__ __launch_bounds__(256) void k_ks_assemble(long long B, int world, int K, int Kmax,
                                                     const double* __restrict__ g, double* __restrict__ lp) {
  const int base = K / world, rem = K % world;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < B * K; i += (long long)gridDim.x * 256) {
    const long long b = i / K;
    const int kg = (int)(i % K);
    const int r = kg < rem * (base + 1) ? kg / (base + 1) : rem + (kg - rem * (base + 1)) / base;
    const int lo = r * base + (r < rem ? r : rem);
    lp[i] = g[((long long)r * B + b) * Kmax + (kg - lo)];
  }
}

// w_loc (B x Kl) = w_full[:, lo:lo+Kl]
__global__ __launch_bounds__(256) void k_ks_slice(long long B, int K, int lo, int Kl, const double* __restrict__ wf,
                                                  double* __restrict__ wl) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < B * Kl; i += (long long)gridDim.x * 256) {
    const long long b = i / Kl;
    wl[i] = wf[b * K + lo + (int)(i % Kl)];
  }
}

template <typename T>
struct KBuf {
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

}  // namespace

struct qce_comm {
  int rank = 0, world = 1, device = 0, kind = QCE_COMM_RCCL;
  ncclComm_t nc = nullptr;  // every collective of the K-shard steps, issued only from their communication stream
  qce_host_collective fn = nullptr;
  void* user = nullptr;
  double *pin_send = nullptr, *pin_recv = nullptr;  // host transport staging
  size_t pin_cap_send = 0, pin_cap_recv = 0;
};

struct qce_kshard {
  qce_model* m = nullptr;  // the model of the latest prepare (mods[cur]); not owned, never dereferenced by
  int device = 0;          // qce_kshard_destroy (the model may already be gone)
  // double-buffered tables (qce_kshard_set_spare): prepare t+1 fills the other model on the prepare stream `ps`
  // while step t's partial kernels still read this one
  qce_model* mods[2] = {nullptr, nullptr};
  int cur = 0;
  hipStream_t ps = nullptr;
  hipEvent_t ev_prep[2] = {nullptr, nullptr}, ev_used[2] = {nullptr, nullptr};
  hipEvent_t ev_shift_rd[2] = {nullptr, nullptr};  // on cs: step t's read of set [i]'s shift slot (agree_shift)
  int used_valid[2] = {0, 0};
  qce_comm* c = nullptr;
  int K = 0, lo = 0, hi = 0, Kmax = 0;
  int lw = 1, lr = 0;  // world / rank the rows are laid out for: the communicator's, or QCE_KSHARD_EMULATE_WORLD's
  int agree_first = 0;  // 'all' mode: M* agreed before the partial kernel, which then writes rows shifted by M*
                        // (no scaling pass; QCE_KSHARD_AGREE_FIRST); 2: world-1 probe that skips the scaling only
  int reserve = 0;     // CUs the step's persistent kernels leave to the communication stream (unless the caller set
                       // QCE_OPT_RESERVE_CUS on the model; applied per launch, the model is not modified)
  hipStream_t cs = nullptr;  // communication stream: the chunks' collectives and row finalisation
  std::vector<hipEvent_t> ev_chunk;
  hipEvent_t ev_done = nullptr;
  KBuf<double> shift, fl, earlier, rs;  // shift: one slot per table set
  KBuf<double> pkb[2];                  // the steps' send rows, alternating: step t+1's kernels fill one while step
  int pkp = 0;                          // t's collectives still read the other
  KBuf<double> step_shift;              // [2 parity + 0]: the shard's shift M_r the step's kernels used (copied on the
                                        // compute stream); [2 parity + 1]: the agreed M* (MAX on the comm stream)
  KBuf<double> scale;                   // [parity]: e^{M_r - M*}, the PreMulSum scalar of the step's SUMs
  KBuf<double> probe;                   // PreMulSum reduce-scatter check: [scalar, mismatch flag]
  std::vector<std::pair<long long, int>> rs_premul;  // (count, RCCL's PreMulSum reduce-scatter exact at that count)
  hipEvent_t ev_pk[2] = {nullptr, nullptr};  // recorded on cs after the last reader of pkb[p] / step_shift[p]
  int pk_valid[2] = {0, 0};
  hipEvent_t ev_st2cs = nullptr, ev_cs2st = nullptr;
  hipEvent_t ev_shift_read = nullptr;  // recorded on cs once a step has read its table set's shift slot (agree_shift)
  int shift_read_valid = 0;
  KBuf<unsigned> cnt;
  double* host_fl = nullptr;  // pinned: [fl0, fl1, earlier0, earlier1] of the last step
  double last_flags[4] = {0, 0, 0, 0};  // host_fl as the last qce_kshard_finish read it
  int local_chol = 0;         // this rank's library refused a call with the reference's Cholesky error
  // the last step, kept for finish(): exact recombination of flagged rows
  struct {
    int valid = 0;
    const double2* y = nullptr;
    long long B = 0;
    int chunks = 1, scatter = 1, mode = QCE_MODE_ALL;
    double2* h = nullptr;
    qce_model* model = nullptr;  // the table set the step read
    int stale = 0;  // a prepare ran after the step: its rows can no longer be recombined with the step's tables
  } pending;
  int any_pending_before = 0;  // a step was superseded before finish(): its flags went into `earlier`
  // repair / selective-mode scratch
  KBuf<double> rm, rsum, racc, mg, lp, lpad, gath, lpfull, wfull, wloc;
  // kernel timing
  int timing = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
  size_t tev_used = 0;
};

namespace {

int comm_error(const std::string& what, ncclResult_t r) {
  return qce_set_error(QCE_ECOMM, what + " failed: " + ncclGetErrorString(r));
}

// one collective of doubles on stream st (see the QCE_COLL_* semantics in qce.h).  premul (SUM ops only): a device
// scalar every rank's send data are multiplied by before the sum (ncclRedOpCreatePreMulSum; host transports scale
// the send buffer in place first).
int collective(qce_comm* c, int op, double* send, double* recv, long long count, hipStream_t st,
               const double* premul = nullptr) {
  if (count <= 0) return QCE_OK;
  const bool sum = op == QCE_COLL_ALLREDUCE_SUM || op == QCE_COLL_REDUCE_SCATTER_SUM;
  if (c->kind == QCE_COMM_RCCL) {
    ncclResult_t r;
    ncclComm_t nc = c->nc;
    ncclRedOp_t sop = ncclSum;
    const bool pm = premul && sum;
    if (pm) {
      // created per call and destroyed once enqueued (the op is captured at enqueue; the scalar is read on device)
      r = ncclRedOpCreatePreMulSum(&sop, const_cast<double*>(premul), ncclFloat64, ncclScalarDevice, nc);
      if (r != ncclSuccess) return comm_error("ncclRedOpCreatePreMulSum", r);
    }
    switch (op) {
      case QCE_COLL_ALLREDUCE_SUM: r = ncclAllReduce(send, recv, (size_t)count, ncclFloat64, sop, nc, st); break;
      case QCE_COLL_ALLREDUCE_MAX: r = ncclAllReduce(send, recv, (size_t)count, ncclFloat64, ncclMax, nc, st); break;
      case QCE_COLL_REDUCE_SCATTER_SUM:
        r = ncclReduceScatter(send, recv, (size_t)count, ncclFloat64, sop, nc, st);
        break;
      case QCE_COLL_ALLGATHER: r = ncclAllGather(send, recv, (size_t)count, ncclFloat64, nc, st); break;
      default: r = ncclInvalidArgument; break;
    }
    if (pm) {
      const ncclResult_t rd = ncclRedOpDestroy(sop, nc);
      if (r == ncclSuccess && rd != ncclSuccess) return comm_error("ncclRedOpDestroy", rd);
    }
    if (r != ncclSuccess) return comm_error("RCCL collective", r);
    return QCE_OK;
  }
  // host transport: synchronise, stage through pinned memory, call, copy back
  const long long ns = (op == QCE_COLL_REDUCE_SCATTER_SUM) ? count * c->world : count;
  const long long nr = (op == QCE_COLL_ALLGATHER) ? count * c->world : count;
  if (premul && sum) {
    hipLaunchKernelGGL(k_ks_scale_rows, dim3(grid_for(ns)), dim3(256), 0, st, ns, send, premul);
    KS_HIP(hipGetLastError());
  }
  if ((size_t)ns > c->pin_cap_send) {
    if (c->pin_send) (void)hipHostFree(c->pin_send);
    c->pin_send = nullptr;
    c->pin_cap_send = 0;
    KS_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->pin_send), sizeof(double) * ns, hipHostMallocDefault));
    c->pin_cap_send = (size_t)ns;
  }
  if ((size_t)nr > c->pin_cap_recv) {
    if (c->pin_recv) (void)hipHostFree(c->pin_recv);
    c->pin_recv = nullptr;
    c->pin_cap_recv = 0;
    KS_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->pin_recv), sizeof(double) * nr, hipHostMallocDefault));
    c->pin_cap_recv = (size_t)nr;
  }
  KS_HIP(hipMemcpyAsync(c->pin_send, send, sizeof(double) * ns, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  if (c->fn(c->user, op, c->pin_send, c->pin_recv, count) != 0)
    return qce_set_error(QCE_ECOMM, "host collective failed");
  KS_HIP(hipMemcpyAsync(recv, c->pin_recv, sizeof(double) * nr, hipMemcpyHostToDevice, st));
  KS_HIP(hipStreamSynchronize(st));
  return QCE_OK;
}

// the step's CU reservation for the duration of one launch call (the launches read it when they size the grid)
struct ReserveScope {
  qce_model* m;
  int prev;
  ReserveScope(qce_model* mm, int reserve) : m(mm), prev(mm->reserve_cus) {
    if (!m->reserve_set) m->reserve_cus = reserve;
  }
  ~ReserveScope() { m->reserve_cus = prev; }
};

hipStream_t ks_stream(qce_kshard* ks, void* stream) {
  if (stream) return (hipStream_t)stream;
  return ks->m->stream;
}

// device call of this rank that may report the prepare's deferred Cholesky status: recorded instead of returned,
// so the rank still joins every collective of the step and all ranks raise together at finish()
bool guarded(qce_kshard* ks, int rc, int* hard) {
  if (rc == QCE_OK) return true;
  if (rc == QCE_ECHOL || (rc == QCE_ESTATE && ks->local_chol)) {
    ks->local_chol = 1;
    return false;
  }
  *hard = rc;
  return false;
}

int timed_begin(qce_kshard* ks, hipStream_t st) {
  if (!ks->timing) return QCE_OK;
  if (ks->tev_used == ks->tev.size()) {
    hipEvent_t a, b;
    KS_HIP(hipEventCreate(&a));
    KS_HIP(hipEventCreate(&b));
    ks->tev.emplace_back(a, b);
  }
  KS_HIP(hipEventRecord(ks->tev[ks->tev_used].first, st));
  return QCE_OK;
}
int timed_end(qce_kshard* ks, hipStream_t st) {
  if (!ks->timing) return QCE_OK;
  KS_HIP(hipEventRecord(ks->tev[ks->tev_used].second, st));
  ks->tev_used++;
  return QCE_OK;
}

// RCCL's PreMulSum reduce-scatter at `count` doubles per rank: exact (1) or not (0), from the cache or, the first
// time a count is used, from one check run in the step's own buffers (before any partial kernel of the step is
// enqueued: the host waits for it) and agreed over the ranks with a MAX, so every rank takes the same path.
int rs_premul_exact(qce_kshard* ks, double* send, double* recv, long long count, int* ok) {
  for (const auto& e : ks->rs_premul)
    if (e.first == count) {
      *ok = e.second;
      return QCE_OK;
    }
  qce_comm* c = ks->c;
  KS_HIP(ks->probe.ensure(2));
  const long long n = count * c->world;
  hipLaunchKernelGGL(k_ks_probe_fill, dim3(grid_for(n)), dim3(256), 0, ks->cs, send, n, ks->probe.p);
  KS_HIP(hipGetLastError());
  KS_RC(collective(c, QCE_COLL_REDUCE_SCATTER_SUM, send, recv, count, ks->cs, ks->probe.p));
  hipLaunchKernelGGL(k_ks_probe_check, dim3(grid_for(count)), dim3(256), 0, ks->cs, recv, count, c->world, c->rank,
                     ks->probe.p + 1);
  KS_HIP(hipGetLastError());
  KS_RC(collective(c, QCE_COLL_ALLREDUCE_MAX, ks->probe.p + 1, ks->probe.p + 1, 1, ks->cs));
  double bad = 1.0;
  KS_HIP(hipMemcpyAsync(&bad, ks->probe.p + 1, sizeof(double), hipMemcpyDeviceToHost, ks->cs));
  KS_HIP(hipStreamSynchronize(ks->cs));
  *ok = bad == 0.0 ? 1 : 0;
  ks->rs_premul.emplace_back(count, *ok);
  return QCE_OK;
}

// QCE_KSHARD_RS_PREMUL=0: never use RCCL's PreMulSum reduce-scatter (always the scaling kernel + SUM)
bool rs_premul_allowed() {
  static const bool on = [] {
    const char* e = getenv("QCE_KSHARD_RS_PREMUL");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the SUM collectives of a step's packed rows (pk, W doubles per row) per chunk on the communication stream, each
// behind its own chunk's producer on `st`, and the rows' finalisation h = acc / s into h_out
int reduce_chunks(qce_kshard* ks, const std::vector<Chunk>& L, bool scatter, int W, hipStream_t st, double2* h_out,
                  bool count_flags, size_t chunk_index, const double* premul) {
  qce_comm* c = ks->c;
  const int N = ks->m->N;  // every table set has the same N
  const Chunk& ch = L[chunk_index];
  hipEvent_t ev = ks->ev_chunk[chunk_index];
  KS_HIP(hipEventRecord(ev, st));
  KS_HIP(hipStreamWaitEvent(ks->cs, ev, 0));
  double* send = ks->pkb[ks->pkp].p + ch.pk_off * W;
  const double* rows;
  if (scatter) {
    const long long q = ch.npad / ks->lw;
    // The librccl this links against (2.26.6, the one torch ships) loses the tail of some reduce-scatters with a
    // PreMulSum op: up to 16 doubles past a boundary that depends on the count (measured on the box,
    // tools/rs_tail_probe.py, profiles/r06_rs_tail_probe*.jsonl; SUM, and all-reduce with PreMulSum, are exact).  Each
    // count is therefore checked once on the real communicator (rs_premul_exact); at a count where the PreMulSum
    // reduce-scatter is not exact the chunk's rows -- every row this rank contributes -- are scaled by a kernel first
    // and the reduce-scatter is a plain SUM.
    // an emulated layout on a world-1 communicator: the rank's own q rows are the whole world-1 reduce-scatter
    double* send_rs = send + (ks->lw != c->world ? (long long)ks->lr * q * W : 0LL);
    double* recv = ks->rs.p + ch.rs_off * W;
    if (premul && c->kind == QCE_COMM_RCCL) {
      // the count's PreMulSum check ran before the step's partial kernels (step_all); where RCCL's PreMulSum
      // reduce-scatter is exact the scaling rides the collective, elsewhere a kernel scales every row first
      int ok = 0;
      for (const auto& e : ks->rs_premul)
        if (e.first == q * W) ok = e.second;
      if (!ok || !rs_premul_allowed()) {
        hipLaunchKernelGGL(k_ks_scale_rows, dim3(rowpass_grid(ch.npad * W)), dim3(256), 0, ks->cs, ch.npad * W, send,
                           premul);
        KS_HIP(hipGetLastError());
        premul = nullptr;
      }
    }
    send = send_rs;
    KS_RC(collective(c, QCE_COLL_REDUCE_SCATTER_SUM, send, recv, q * W, ks->cs, premul));
    rows = recv;
  } else {
    KS_RC(collective(c, QCE_COLL_ALLREDUCE_SUM, send, send, ch.npad * W, ks->cs, premul));
    rows = send;
  }
  if (ch.nv > 0) {
    hipLaunchKernelGGL(k_ks_finalize, dim3(rowpass_grid(ch.nv * N)), dim3(256), 0, ks->cs, ch.nv, N, rows,
                       h_out + ch.h_off * N, count_flags ? kUnderflowS : -1.0, ks->cnt.p);
    KS_HIP(hipGetLastError());
  }
  return QCE_OK;
}

int ensure_events(qce_kshard* ks, size_t n) {
  while (ks->ev_chunk.size() < n) {
    hipEvent_t e;
    KS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ks->ev_chunk.push_back(e);
  }
  return QCE_OK;
}

// close a step: flag word MAX, pinned copy of [fl, earlier], the caller's stream ordered behind the comm stream
int close_step(qce_kshard* ks) {
  hipLaunchKernelGGL(k_ks_flags, dim3(1), dim3(64), 0, ks->cs, ks->cnt.p, ks->step_shift.p + 2 * ks->pkp + 1,
                     ks->local_chol, ks->fl.p);
  KS_HIP(hipGetLastError());
  KS_RC(collective(ks->c, QCE_COLL_ALLREDUCE_MAX, ks->fl.p, ks->fl.p, 2, ks->cs));
  KS_HIP(hipMemcpyAsync(ks->host_fl, ks->fl.p, 2 * sizeof(double), hipMemcpyDeviceToHost, ks->cs));
  KS_HIP(hipMemcpyAsync(ks->host_fl + 2, ks->earlier.p, 2 * sizeof(double), hipMemcpyDeviceToHost, ks->cs));
  KS_HIP(hipEventRecord(ks->ev_done, ks->cs));  // h_out complete (the caller's stream waits for it in finish)
  // the last reader of this parity's send rows and shift slots: step t+2 (the next user of the parity) waits for it
  KS_HIP(hipEventRecord(ks->ev_pk[ks->pkp], ks->cs));
  ks->pk_valid[ks->pkp] = 1;
  return QCE_OK;
}


// stream hand-offs: every data collective is issued on the communication stream (one stream per communicator)
int st_to_cs(qce_kshard* ks, hipStream_t st) {
  if (st == ks->cs) return QCE_OK;
  KS_HIP(hipEventRecord(ks->ev_st2cs, st));
  KS_HIP(hipStreamWaitEvent(ks->cs, ks->ev_st2cs, 0));
  return QCE_OK;
}
int cs_to_st(qce_kshard* ks, hipStream_t st) {
  if (st == ks->cs) return QCE_OK;
  KS_HIP(hipEventRecord(ks->ev_cs2st, ks->cs));
  KS_HIP(hipStreamWaitEvent(st, ks->ev_cs2st, 0));
  return QCE_OK;
}

// the step's agreed shift on the communication stream: the shard's M_r of the step's table set (behind the compute
// stream's wait for that set's prepare) into step_shift[2p], [2p + 1]; M* = MAX over the shards in [2p + 1]; then the
// SUMs' scalar e^{M_r - M*}.  The table set's slot is not rewritten before this has read it: the next prepare into
// the set waits for the step's close on this stream (ev_used).
int agree_shift(qce_kshard* ks, hipStream_t st) {
  double* sh = ks->step_shift.p + 2 * ks->pkp;
  KS_RC(st_to_cs(ks, st));
  hipLaunchKernelGGL(k_ks_shift_in, dim3(1), dim3(64), 0, ks->cs, ks->shift.p + ks->cur, sh);
  KS_HIP(hipGetLastError());
  KS_HIP(hipEventRecord(ks->ev_shift_read, ks->cs));
  ks->shift_read_valid = 1;
  if (ks->mods[1]) KS_HIP(hipEventRecord(ks->ev_shift_rd[ks->cur], ks->cs));
  KS_RC(collective(ks->c, QCE_COLL_ALLREDUCE_MAX, sh + 1, sh + 1, 1, ks->cs));
  double bias = 0.0;
  if (const char* b = getenv("QCE_KSHARD_GLOBAL_BIAS")) bias = atof(b);  // tests only
  hipLaunchKernelGGL(k_ks_scale_of, dim3(1), dim3(64), 0, ks->cs, sh, bias, ks->scale.p + ks->pkp);
  KS_HIP(hipGetLastError());
  return QCE_OK;
}

// 'all' mode: per chunk the shifted partial on st (or, for the exact recombination, the per-row-shift rows of a
// whole-batch FP64 partial), its SUM collective on cs, the finalisation
int step_all(qce_kshard* ks, qce_model* m, const double2* y, long long B, int chunks, bool scatter, double2* h,
             hipStream_t st, bool rowshift) {
  qce_comm* c = ks->c;
  const int N = m->N, M = m->M, W = 2 * N + 2;
  std::vector<Chunk> L = chunk_layout(B, chunks, ks->lw, ks->lr, scatter);
  long long pk_rows = 0, rs_rows = 0;
  for (const Chunk& ch : L) {
    pk_rows += ch.npad;
    if (scatter) rs_rows += ch.npad / ks->lw;
  }
  KBuf<double>& pkbuf = ks->pkb[ks->pkp];
  KS_HIP(pkbuf.ensure((size_t)pk_rows * W));
  if (scatter) KS_HIP(ks->rs.ensure((size_t)rs_rows * W));
  KS_RC(ensure_events(ks, L.size()));
  if (scatter && !rowshift && !ks->agree_first && c->kind == QCE_COMM_RCCL && rs_premul_allowed()) {
    for (const Chunk& ch : L) {  // each new count checked once, in the rows this step is about to fill
      const long long q = ch.npad / ks->lw;
      double* send = pkbuf.p + ch.pk_off * W + (ks->lw != c->world ? (long long)ks->lr * q * W : 0LL);
      int ok;
      KS_RC(rs_premul_exact(ks, send, ks->rs.p + ch.rs_off * W, q * W, &ok));
    }
  }
  int hard = QCE_OK;
  if (rowshift) {
    // exact recombination: m (running max), s, acc of this shard for the whole batch; mg = MAX over shards of m
    KS_HIP(ks->rm.ensure((size_t)B));
    KS_HIP(ks->rsum.ensure((size_t)B));
    KS_HIP(ks->racc.ensure((size_t)B * 2 * N));
    KS_HIP(ks->mg.ensure((size_t)B));
    if (!guarded(ks, qce_estimate_partial_f64(m, reinterpret_cast<const double*>(y), B, ks->rm.p, ks->rsum.p,
                                              ks->racc.p, QCE_IO_DEVICE, st), &hard)) {
      if (hard) return hard;
      KS_HIP(hipMemsetAsync(ks->rm.p, 0xff, sizeof(double) * B, st));  // NaN rows; the Cholesky flag raises first
    }
    KS_HIP(hipMemcpyAsync(ks->mg.p, ks->rm.p, sizeof(double) * B, hipMemcpyDeviceToDevice, st));
    KS_RC(st_to_cs(ks, st));
    KS_RC(collective(c, QCE_COLL_ALLREDUCE_MAX, ks->mg.p, ks->mg.p, B, ks->cs));
    KS_RC(cs_to_st(ks, st));
  }
  for (size_t i = 0; i < L.size(); ++i) {
    const Chunk& ch = L[i];
    const long long n = ch.hi - ch.lo;
    double* pk = pkbuf.p + ch.pk_off * W;
    if (ch.npad > n) KS_HIP(hipMemsetAsync(pk + n * W, 0, sizeof(double) * (ch.npad - n) * W, st));
    if (rowshift) {
      hipLaunchKernelGGL(k_ks_pack_rowshift, dim3(grid_for(n * W)), dim3(256), 0, st, n, N, ks->rm.p + ch.lo,
                         ks->rsum.p + ch.lo, ks->racc.p + ch.lo * 2 * N, ks->mg.p + ch.lo, pk);
      KS_HIP(hipGetLastError());
    } else {
      bool ok = false;
      if (!ks->local_chol) {
        KS_RC(timed_begin(ks, st));
        ReserveScope rsv(m, ks->reserve);
        // the shard's own shift M_r, read straight from the table set's slot (final once st waited for its prepare)
        // agree-first: the agreed M* (the compute stream waited for the MAX), so the rows enter the SUM unscaled
        const double* shp = ks->agree_first == 1 ? ks->step_shift.p + 2 * ks->pkp + 1 : ks->shift.p + ks->cur;
        ok = guarded(ks, qce_estimate_partial_shifted(m, reinterpret_cast<const double*>(y + ch.lo * M), n, shp, pk,
                                                      QCE_IO_DEVICE, st), &hard);
        if (hard) return hard;
        KS_RC(timed_end(ks, st));
      }
      if (!ok) KS_HIP(hipMemsetAsync(pk, 0, sizeof(double) * n * W, st));
    }
    KS_RC(reduce_chunks(ks, L, scatter, W, st, h, !rowshift, i,
                        (rowshift || ks->agree_first) ? nullptr : ks->scale.p + ks->pkp));
  }
  return QCE_OK;
}

// selective modes: global selection from the shards' lp, this shard's weighted filter sum, one SUM collective
int step_select(qce_kshard* ks, const double2* y, long long B, int mode, double param, bool scatter, double2* h,
                hipStream_t st) {
  qce_model* m = ks->m;
  qce_comm* c = ks->c;
  const int N = m->N, Kl = m->K, W = 2 * N;
  int kmode, nsel = 0;
  double p = 0.0;
  if (ks->lw != c->world)
    return qce_set_error(QCE_ENOTIMPL, "QCE_KSHARD_EMULATE_WORLD rehearses the 'all' mode only");
  ReserveScope rsv(m, ks->reserve);
  if (mode == QCE_MODE_TOPN) {
    if (param < 1.0 || param != floor(param)) return qce_set_error(QCE_EARG, "top-n needs an integer n >= 1");
    nsel = param > 1e9 ? 1000000000 : (int)param;
    kmode = nsel == 1 ? 3 : 1;
  } else if (mode == QCE_MODE_CUMP) {
    kmode = 2;
    p = param;
  } else {
    return qce_set_error(QCE_EARG, "unknown mode");
  }
  if (kmode != 3 && ks->K > qce_select_max_k())
    return qce_set_error(QCE_ENOTIMPL, "K-shard top-n / cumulative-p support K <= " + std::to_string(qce_select_max_k()));
  std::vector<Chunk> L = chunk_layout(B, 1, c->world, c->rank, scatter);
  KS_RC(ensure_events(ks, 1));
  const long long npad = L[0].npad;
  KS_HIP(ks->lp.ensure((size_t)B * Kl));
  KS_HIP(ks->wloc.ensure((size_t)B * Kl));
  KBuf<double>& pkbuf = ks->pkb[ks->pkp];
  KS_HIP(pkbuf.ensure((size_t)npad * W));
  if (scatter) KS_HIP(ks->rs.ensure((size_t)(npad / c->world) * W));
  int hard = QCE_OK;
  bool ok = false;
  if (!ks->local_chol) {
    KS_RC(timed_begin(ks, st));
    ok = guarded(ks, qce_log_prob(m, reinterpret_cast<const double*>(y), B, ks->lp.p, nullptr, nullptr, QCE_IO_DEVICE,
                                  st), &hard);
    if (hard) return hard;
    KS_RC(timed_end(ks, st));
  }
  if (!ok) KS_HIP(hipMemsetAsync(ks->lp.p, 0, sizeof(double) * B * Kl, st));
  if (kmode == 3) {
    // argmax: (max lp, local index) per row and shard -> the owner of the first global maximum
    KS_HIP(ks->lpad.ensure((size_t)B * 2));
    KS_HIP(ks->gath.ensure((size_t)B * 2 * c->world));
    hipLaunchKernelGGL(k_ks_row_argmax, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, Kl, ks->lp.p, ks->lpad.p);
    KS_HIP(hipGetLastError());
    KS_RC(st_to_cs(ks, st));
    KS_RC(collective(c, QCE_COLL_ALLGATHER, ks->lpad.p, ks->gath.p, B * 2, ks->cs));
    KS_RC(cs_to_st(ks, st));
    hipLaunchKernelGGL(k_ks_argmax_weights, dim3(grid_for(B)), dim3(256), 0, st, B, c->world, c->rank, Kl,
                       ks->gath.p, ks->wloc.p);
    KS_HIP(hipGetLastError());
  } else {
    const int K = ks->K, Kmax = ks->Kmax;
    KS_HIP(ks->lpad.ensure((size_t)B * Kmax));
    KS_HIP(ks->gath.ensure((size_t)B * Kmax * c->world));
    KS_HIP(ks->lpfull.ensure((size_t)B * K));
    KS_HIP(ks->wfull.ensure((size_t)B * K));
    hipLaunchKernelGGL(k_ks_pad, dim3(grid_for(B * Kmax)), dim3(256), 0, st, B, Kl, Kmax, ks->lp.p, ks->lpad.p);
    KS_HIP(hipGetLastError());
    KS_RC(st_to_cs(ks, st));
    KS_RC(collective(c, QCE_COLL_ALLGATHER, ks->lpad.p, ks->gath.p, B * Kmax, ks->cs));
    KS_RC(cs_to_st(ks, st));
    hipLaunchKernelGGL(k_ks_assemble, dim3(grid_for(B * K)), dim3(256), 0, st, B, c->world, K, Kmax, ks->gath.p,
                       ks->lpfull.p);
    KS_HIP(hipGetLastError());
    // the same FP64 selection on every rank (gmm_cplx_bussgang.py:213, :235-236)
    KS_HIP(qce_launch_select(B, K, ks->lpfull.p, kmode, nsel, p, nullptr, nullptr, nullptr, st, ks->wfull.p));
    hipLaunchKernelGGL(k_ks_slice, dim3(grid_for(B * Kl)), dim3(256), 0, st, B, K, ks->lo, Kl, ks->wfull.p,
                       ks->wloc.p);
    KS_HIP(hipGetLastError());
  }
  // this shard's share of sum_k w_bk (W_k y_b + b_k), written straight into the collective's rows (a row of 2N
  // doubles is one c128 row of h)
  if (npad > B) KS_HIP(hipMemsetAsync(pkbuf.p + B * W, 0, sizeof(double) * (npad - B) * W, st));
  ok = false;
  if (!ks->local_chol) {
    ok = guarded(ks, qce_weighted_estimate(m, y, B, ks->wloc.p, reinterpret_cast<double2*>(pkbuf.p), st), &hard);
    if (hard) return hard;
  }
  if (!ok) KS_HIP(hipMemsetAsync(pkbuf.p, 0, sizeof(double) * B * W, st));
  // SUM over shards on the communication stream, rows straight into h_out
  const Chunk& ch = L[0];
  KS_HIP(hipEventRecord(ks->ev_chunk[0], st));
  KS_HIP(hipStreamWaitEvent(ks->cs, ks->ev_chunk[0], 0));
  if (scatter) {
    const long long q = npad / c->world;
    KS_RC(collective(c, QCE_COLL_REDUCE_SCATTER_SUM, pkbuf.p, ks->rs.p, q * W, ks->cs));
    if (ch.nv > 0)
      KS_HIP(hipMemcpyAsync(h, ks->rs.p, sizeof(double) * ch.nv * W, hipMemcpyDeviceToDevice, ks->cs));
  } else {
    KS_RC(collective(c, QCE_COLL_ALLREDUCE_SUM, pkbuf.p, reinterpret_cast<double*>(h), B * W, ks->cs));
  }
  return QCE_OK;
}

}  // namespace

extern "C" {

int qce_comm_unique_id(void* id_out) {
  if (!id_out) return qce_set_error(QCE_EARG, "null id");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return comm_error("ncclGetUniqueId", r);
  memcpy(id_out, &id, sizeof(id));
  return QCE_OK;
}

int qce_comm_init(const void* unique_id, int rank, int world, int device, qce_comm** out) {
  if (!unique_id || !out) return qce_set_error(QCE_EARG, "null argument");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return qce_set_error(QCE_EARG, "rank / world out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return qce_set_error(QCE_EARG, "device index out of range");
  DevGuard g(device);
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  qce_comm* c = new qce_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->kind = QCE_COMM_RCCL;
  ncclResult_t r = ncclCommInitRank(&c->nc, world, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return comm_error("ncclCommInitRank", r);
  }
  *out = c;
  return QCE_OK;
}

int qce_comm_init_host(int rank, int world, int device, qce_host_collective fn, void* user, qce_comm** out) {
  if (!fn || !out) return qce_set_error(QCE_EARG, "null argument");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return qce_set_error(QCE_EARG, "rank / world out of range");
  qce_comm* c = new qce_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->kind = QCE_COMM_HOST;
  c->fn = fn;
  c->user = user;
  *out = c;
  return QCE_OK;
}

int qce_comm_destroy(qce_comm* c) {
  if (!c) return QCE_OK;
  DevGuard g(c->device);
  if (c->nc) (void)ncclCommDestroy(c->nc);
  if (c->pin_send) (void)hipHostFree(c->pin_send);
  if (c->pin_recv) (void)hipHostFree(c->pin_recv);
  delete c;
  return QCE_OK;
}

int qce_comm_info(qce_comm* c, int* rank, int* world, int* device, int* kind) {
  if (!c) return qce_set_error(QCE_EARG, "null comm");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  if (device) *device = c->device;
  if (kind) *kind = c->kind;
  return QCE_OK;
}

int qce_kshard_slice(int K, int world, int rank, int* lo, int* hi) {
  if (!lo || !hi) return qce_set_error(QCE_EARG, "null argument");
  if (world < 1 || rank < 0 || rank >= world || K < world)
    return qce_set_error(QCE_EARG, "K-shard split needs K >= world and 0 <= rank < world");
  slice_of(K, world, rank, lo, hi);
  return QCE_OK;
}

int qce_kshard_rows(int64_t B, int chunks, int world, int rank, int scatter, int64_t* ranges, int cap, int* n) {
  if (!ranges || !n || B < 0 || world < 1 || rank < 0 || rank >= world)
    return qce_set_error(QCE_EARG, "bad arguments");
  std::vector<Chunk> L = chunk_layout(B, chunks, world, rank, scatter != 0);
  if ((int)L.size() > cap) return qce_set_error(QCE_EARG, "ranges array too small");
  for (size_t i = 0; i < L.size(); ++i) {
    ranges[2 * i] = L[i].r0;
    ranges[2 * i + 1] = L[i].r0 + L[i].nv;
  }
  *n = (int)L.size();
  return QCE_OK;
}

int qce_kshard_create(qce_model* shard, qce_comm* comm, int K_total, qce_kshard** out) {
  if (!shard || !comm || !out) return qce_set_error(QCE_EARG, "null argument");
  *out = nullptr;
  if (K_total < comm->world) return qce_set_error(QCE_EARG, "K-shard split needs K >= world");
  if (comm->kind == QCE_COMM_RCCL && comm->device != shard->device)
    return qce_set_error(QCE_EARG, "model and communicator are on different devices");
  int lo, hi;
  slice_of(K_total, comm->world, comm->rank, &lo, &hi);
  if (hi - lo != shard->K)
    return qce_set_error(QCE_EARG, "the shard model must hold components [" + std::to_string(lo) + ", " +
                                       std::to_string(hi) + ") of the balanced split (qce_kshard_slice)");
  DevGuard g(shard->device);
  qce_kshard* ks = new qce_kshard();
  ks->lw = comm->world;
  ks->lr = comm->rank;
  if (comm->world == 1) (void)kshard_emulated(&ks->lw, &ks->lr);
  if (comm->kind == QCE_COMM_RCCL && ks->lw > 1) ks->reserve = kshard_reserve_cus();
  if (const char* af = getenv("QCE_KSHARD_AGREE_FIRST")) {
    ks->agree_first = atoi(af);
    // the probe (2) leaves the rows unscaled: exact only where M* = M_r, i.e. one real rank
    if (ks->agree_first == 2 && comm->world != 1) ks->agree_first = 0;
  }
  ks->m = shard;
  ks->mods[0] = shard;
  ks->device = shard->device;
  ks->c = comm;
  ks->K = K_total;
  ks->lo = lo;
  ks->hi = hi;
  ks->Kmax = (K_total + comm->world - 1) / comm->world;
  hipError_t e = hipStreamCreateWithFlags(&ks->cs, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ks->ev_done, hipEventDisableTiming);
  if (e == hipSuccess) e = ks->shift.ensure(2);
  if (e == hipSuccess) e = ks->step_shift.ensure(4);
  if (e == hipSuccess) e = ks->scale.ensure(2);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ks->ev_pk[i], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ks->ev_st2cs, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ks->ev_cs2st, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ks->ev_shift_read, hipEventDisableTiming);
  if (e == hipSuccess) e = ks->fl.ensure(2);
  if (e == hipSuccess) e = ks->earlier.ensure(2);
  if (e == hipSuccess) e = ks->cnt.ensure(1);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&ks->host_fl), 4 * sizeof(double), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemset(ks->earlier.p, 0, 2 * sizeof(double));
  if (e == hipSuccess) e = hipMemset(ks->fl.p, 0, 2 * sizeof(double));
  if (e != hipSuccess) {
    qce_kshard_destroy(ks);
    return qce_set_error(QCE_EHIP, std::string("K-shard allocation failed: ") + hipGetErrorString(e));
  }
  *out = ks;
  return QCE_OK;
}

int qce_kshard_destroy(qce_kshard* ks) {
  if (!ks) return QCE_OK;
  DevGuard g(ks->device);
  if (ks->cs) (void)hipStreamSynchronize(ks->cs);
  for (auto* b : {&ks->shift, &ks->fl, &ks->earlier, &ks->pkb[0], &ks->pkb[1], &ks->step_shift, &ks->scale, &ks->probe, &ks->rs,
                  &ks->rm, &ks->rsum, &ks->racc, &ks->mg, &ks->lp, &ks->lpad, &ks->gath, &ks->lpfull, &ks->wfull,
                  &ks->wloc})
    b->release();
  ks->cnt.release();
  for (hipEvent_t e : ks->ev_chunk) (void)hipEventDestroy(e);
  for (auto& pr : ks->tev) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (ks->ev_done) (void)hipEventDestroy(ks->ev_done);
  if (ks->ev_st2cs) (void)hipEventDestroy(ks->ev_st2cs);
  if (ks->ev_cs2st) (void)hipEventDestroy(ks->ev_cs2st);
  if (ks->ev_shift_read) (void)hipEventDestroy(ks->ev_shift_read);
  for (int i = 0; i < 2; ++i) {
    if (ks->ev_pk[i]) (void)hipEventDestroy(ks->ev_pk[i]);
    if (ks->ev_prep[i]) (void)hipEventDestroy(ks->ev_prep[i]);
    if (ks->ev_used[i]) (void)hipEventDestroy(ks->ev_used[i]);
    if (ks->ev_shift_rd[i]) (void)hipEventDestroy(ks->ev_shift_rd[i]);
  }
  if (ks->ps) {
    (void)hipStreamSynchronize(ks->ps);
    (void)hipStreamDestroy(ks->ps);
  }
  if (ks->host_fl) (void)hipHostFree(ks->host_fl);
  if (ks->cs) (void)hipStreamDestroy(ks->cs);
  delete ks;
  return QCE_OK;
}

int qce_kshard_prepare(qce_kshard* ks, const double* A, int M, double snr_db, double n_bits, int quant_kind,
                       const double* thresholds, const double* labels, int n_levels, void* stream) {
  if (!ks) return qce_set_error(QCE_EARG, "null K-shard");
  DevGuard g(ks->device);
  hipStream_t st = ks_stream(ks, stream);
  const bool dbl = ks->mods[1] != nullptr;
  // with a spare table set the prepare fills the set the previous step did NOT read, on the prepare stream, so it
  // overlaps that step's partial kernels; it waits only for the last step that read this set
  const int j = dbl ? 1 - ks->cur : 0;
  qce_model* m = ks->mods[j];
  hipStream_t ps = dbl ? ks->ps : st;
  if (dbl && ks->used_valid[j]) {
    KS_HIP(hipStreamWaitEvent(ps, ks->ev_used[j], 0));
    KS_HIP(hipStreamWaitEvent(ps, ks->ev_shift_rd[j], 0));
  }
  // one table set: its shift slot is read on the communication stream at the start of each step (agree_shift), which
  // may lag behind the compute stream; the prepare that rewrites it waits for that read
  if (!dbl && ks->shift_read_valid) KS_HIP(hipStreamWaitEvent(ps, ks->ev_shift_read, 0));
  if (ks->pending.valid && ks->pending.model == m) ks->pending.stale = 1;  // its tables are being replaced
  ks->cur = j;
  ks->m = m;
  ks->local_chol = 0;
  KS_RC(qce_prepare(m, A, M, snr_db, n_bits, quant_kind, thresholds, labels, n_levels, ps));
  double* shift = ks->shift.p + j;
  int hard = QCE_OK;
  if (!guarded(ks, qce_cconst_max(m, shift, QCE_IO_DEVICE, ps), &hard)) {
    if (hard) return hard;
    const double inf = __builtin_inf();  // the failure rides the shift as the kernel would have written it
    KS_HIP(hipMemcpyAsync(shift, &inf, sizeof(double), hipMemcpyHostToDevice, ps));
    KS_HIP(hipStreamSynchronize(ps));
  }
  // no collective here: the shards agree on M* at the start of the step that uses these tables (agree_shift), on the
  // communication stream behind the previous step's collectives, so every rank issues its collectives in one order
  if (const char* b = getenv("QCE_KSHARD_SHIFT_BIAS")) {  // tests only: force the underflow path
    hipLaunchKernelGGL(k_ks_add, dim3(1), dim3(64), 0, ps, shift, atof(b));
    KS_HIP(hipGetLastError());
  }
  if (dbl) KS_HIP(hipEventRecord(ks->ev_prep[j], ps));
  return QCE_OK;
}

int qce_kshard_set_spare(qce_kshard* ks, qce_model* spare) {
  if (!ks || !spare) return qce_set_error(QCE_EARG, "null argument");
  const qce_model* a = ks->mods[0];
  if (spare == a || spare->K != a->K || spare->N != a->N || spare->device != a->device)
    return qce_set_error(QCE_EARG, "the spare model must be a second model of the same shard (same K, N, device)");
  DevGuard g(ks->device);
  KS_HIP(hipStreamCreateWithFlags(&ks->ps, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) {
    KS_HIP(hipEventCreateWithFlags(&ks->ev_prep[i], hipEventDisableTiming));
    KS_HIP(hipEventCreateWithFlags(&ks->ev_used[i], hipEventDisableTiming));
    KS_HIP(hipEventCreateWithFlags(&ks->ev_shift_rd[i], hipEventDisableTiming));
  }
  ks->mods[1] = spare;
  return QCE_OK;
}

int qce_kshard_estimate(qce_kshard* ks, const double* y, int64_t B, int mode, double mode_param, int chunks,
                        int scatter, double* h_out, void* stream) {
  if (!ks) return qce_set_error(QCE_EARG, "null K-shard");
  if (B < 0 || (B > 0 && (!y || !h_out))) return qce_set_error(QCE_EARG, "bad y / h_out");
  if (!ks->m->prepared && !ks->local_chol) return qce_set_error(QCE_ESTATE, "qce_kshard_prepare has not been called");
  DevGuard g(ks->device);
  hipStream_t st = ks_stream(ks, stream);
  // a step superseded before finish(): its flags fold into the running `earlier` word
  if (ks->pending.valid) {
    hipLaunchKernelGGL(k_ks_fold, dim3(1), dim3(64), 0, ks->cs, ks->earlier.p, ks->fl.p);
    KS_HIP(hipGetLastError());
    ks->any_pending_before = 1;
  }
  KS_HIP(hipMemsetAsync(ks->cnt.p, 0, sizeof(unsigned), ks->cs));
  const double2* yd = reinterpret_cast<const double2*>(y);
  double2* hd = reinterpret_cast<double2*>(h_out);
  const bool dbl = ks->mods[1] != nullptr;
  if (dbl) KS_HIP(hipStreamWaitEvent(st, ks->ev_prep[ks->cur], 0));
  // this step's send rows: the buffer the previous step's collectives do not read, once the step before that (the
  // last reader of this parity, still in flight on the comm stream) is done with it; the shard's shift, kept in the
  // parity's slot (the next prepare may overwrite the table set's slot before the comm stream gets there)
  ks->pkp ^= 1;
  if (ks->pk_valid[ks->pkp]) KS_HIP(hipStreamWaitEvent(st, ks->ev_pk[ks->pkp], 0));
  if (const char* d = getenv("QCE_KSHARD_CS_DELAY_US")) {  // tests only
    int rate_khz = 0;
    KS_HIP(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, ks->device));
    hipLaunchKernelGGL(k_ks_spin, dim3(1), dim3(64), 0, ks->cs, (long long)(atof(d) * rate_khz / 1000.0));
    KS_HIP(hipGetLastError());
  }
  KS_RC(agree_shift(ks, st));
  if (ks->agree_first == 1 && mode == QCE_MODE_ALL && B > 0) KS_RC(cs_to_st(ks, st));  // the partial reads M*
  if (B > 0) {
    if (mode == QCE_MODE_ALL) {
      KS_RC(step_all(ks, ks->m, yd, B, chunks, scatter != 0, hd, st, false));
    } else {
      KS_RC(step_select(ks, yd, B, mode, mode_param, scatter != 0, hd, st));
    }
  }
  // the table set's readers are the step's kernels on st and the read of its shift slot on cs (ev_shift_rd): the
  // next prepare into the set waits for those two only, not for the step's collectives and row finalisation
  // (round 5 waited for the step's close on cs; emulated world-8 rank step 1.107 / 1.103 -> 1.080 / 1.097 ms,
  // profiles/r06_kshard_prepare_order_ab.jsonl)
  if (dbl) {
    KS_HIP(hipEventRecord(ks->ev_used[ks->cur], st));
    ks->used_valid[ks->cur] = 1;
  }
  KS_RC(st_to_cs(ks, st));  // the flag word closes the step behind its last kernel
  KS_RC(close_step(ks));
  ks->pending.valid = 1;
  ks->pending.y = yd;
  ks->pending.B = B;
  ks->pending.chunks = mode == QCE_MODE_ALL ? chunks : 1;
  ks->pending.scatter = scatter;
  ks->pending.mode = mode;
  ks->pending.h = hd;
  ks->pending.model = ks->m;
  ks->pending.stale = 0;
  return QCE_OK;
}

int qce_kshard_finish(qce_kshard* ks, void* stream) {
  if (!ks) return qce_set_error(QCE_EARG, "null K-shard");
  if (!ks->pending.valid) return QCE_OK;
  DevGuard g(ks->device);
  hipStream_t st = ks_stream(ks, stream);
  KS_HIP(hipEventSynchronize(ks->ev_done));
  const double f0 = ks->host_fl[0], f1 = ks->host_fl[1], e0 = ks->host_fl[2], e1 = ks->host_fl[3];
  for (int i = 0; i < 4; ++i) ks->last_flags[i] = ks->host_fl[i];
  auto pend = ks->pending;
  ks->pending.valid = 0;
  ks->any_pending_before = 0;
  KS_HIP(hipMemsetAsync(ks->earlier.p, 0, 2 * sizeof(double), ks->cs));
  if (f1 > 0.0 || e1 > 0.0) return qce_set_error(QCE_ECHOL, kCholMessage);
  if (e0 > 0.0)
    return qce_set_error(QCE_ESTATE, "an earlier K-shard estimate had rows whose shifted sum underflowed; call "
                                     "qce_kshard_finish after each such step to have them recombined");
  if (f0 > 0.0 && pend.mode == QCE_MODE_ALL && pend.stale)
    return qce_set_error(QCE_ESTATE, "the last K-shard estimate had rows whose shifted sum underflowed and "
                                     "qce_kshard_prepare ran before qce_kshard_finish: they cannot be recombined");
  if (f0 > 0.0 && pend.mode == QCE_MODE_ALL) {
    // exact recombination of the last step (every rank agrees through the MAX of the flag word), all of it on the
    // communication stream (its collectives are data-communicator work)
    KS_RC(step_all(ks, pend.model, pend.y, pend.B, pend.chunks, pend.scatter != 0, pend.h, ks->cs, true));
    KS_HIP(hipEventRecord(ks->ev_done, ks->cs));
    KS_HIP(hipEventSynchronize(ks->ev_done));
  }
  KS_HIP(hipStreamWaitEvent(st, ks->ev_done, 0));  // the caller's stream sees h complete
  return QCE_OK;
}

int qce_kshard_flags(qce_kshard* ks, double* out4) {
  if (!ks || !out4) return qce_set_error(QCE_EARG, "null argument");
  for (int i = 0; i < 4; ++i) out4[i] = ks->last_flags[i];
  return QCE_OK;
}

int qce_kshard_timing(qce_kshard* ks, int enable) {
  if (!ks) return qce_set_error(QCE_EARG, "null K-shard");
  ks->timing = enable != 0;
  ks->tev_used = 0;
  return QCE_OK;
}

int qce_kshard_kernel_ms(qce_kshard* ks, double* total_ms, int* launches) {
  if (!ks || !total_ms) return qce_set_error(QCE_EARG, "null argument");
  DevGuard g(ks->device);
  double t = 0.0;
  for (size_t i = 0; i < ks->tev_used; ++i) {
    KS_HIP(hipEventSynchronize(ks->tev[i].second));
    float ms = 0.0f;
    KS_HIP(hipEventElapsedTime(&ms, ks->tev[i].first, ks->tev[i].second));
    t += ms;
  }
  *total_ms = t;
  if (launches) *launches = (int)ks->tev_used;
  ks->tev_used = 0;
  return QCE_OK;
}

}  // extern "C"
