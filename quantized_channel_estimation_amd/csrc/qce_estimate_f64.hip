// FP64 'all'-mode path, host side and the small kernels around k_est_all_f64 (qce_f64_kernel.h):
// the stream-K merge, the shifted packed partial, table packing and precision conversions.
#include "qce_f64g_kernel.h"

// Combine the stream-K pieces of tiles cut between workgroups (one wave per sample; tiles written
// whole return at once): h = sum_j acc_j e^{m_j - M} / sum_j s_j e^{m_j - M}, or the merged partial.
__global__ __launch_bounds__(256) void k_merge_f64(long long B, int N, int K, int TS, long long L,
                                                   const double* __restrict__ pm, const double* __restrict__ ps,
                                                   const double* __restrict__ pa, double2* __restrict__ h,
                                                   double* __restrict__ om, double* __restrict__ os,
                                                   double* __restrict__ oa, double* __restrict__ pk,
                                                   const double* __restrict__ shift) {
  // One wave per row.  Its lanes first take one partial record each (the row's maximum, then the record weights
  // e^{m_w - max}, staged in LDS: computed once per record instead of once per output element), then the output
  // elements n = lane, lane + 64 (N <= 128 on the fused FP64 kernel), accumulated in registers over chunks of 64
  // records.
  __shared__ double wsc[4][64];
  __shared__ long long wrec[4][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * 4 + wv;
  if (b >= B || L <= 0) return;  // wave-uniform
  const long long t = b / TS, ls = b % TS;
  const long long wa = (t * K) / L, wb = ((t + 1) * K - 1) / L;
  if (wa == wb) return;
  auto rec_of = [&](long long w) -> long long {
    const long long tf = (w * L) / K;
    return (w * 2 + (t == tf ? 0 : 1)) * TS + ls;
  };
  const int nrec = (int)(wb - wa + 1);
  double mx = QCE_NEG_INF;
  for (int q = lane; q < nrec; q += 64) mx = fmax(mx, pm[rec_of(wa + q)]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  double s = 0.0, re0 = 0.0, im0 = 0.0, re1 = 0.0, im1 = 0.0;
  const int n0 = lane, n1 = lane + 64;
  for (int c0 = 0; c0 < nrec; c0 += 64) {
    const int nc = nrec - c0 < 64 ? nrec - c0 : 64;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous chunk's LDS reads are done
    __builtin_amdgcn_wave_barrier();
    if (lane < nc) {
      const long long r = rec_of(wa + c0 + lane);
      const double sc = (pm[r] == QCE_NEG_INF) ? 0.0 : exp(pm[r] - mx);
      wsc[wv][lane] = sc;
      wrec[wv][lane] = r;
      s = fma(ps[r], sc, s);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int q = 0; q < nc; ++q) {
      const double sc = wsc[wv][q];
      const double* rp = pa + wrec[wv][q] * 2 * N;
      if (n0 < N) {
        const double2 v = *reinterpret_cast<const double2*>(rp + 2 * n0);
        re0 = fma(v.x, sc, re0);
        im0 = fma(v.y, sc, im0);
      }
      if (n1 < N) {
        const double2 v = *reinterpret_cast<const double2*>(rp + 2 * n1);
        re1 = fma(v.x, sc, re1);
        im1 = fma(v.y, sc, im1);
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  const double psc = (pk && mx != QCE_NEG_INF) ? exp(mx - *shift) : 0.0;  // shifted packed output
  auto put = [&](int n, double re, double im) {
    if (n >= N) return;
    if (h) {
      h[b * N + n] = make_double2(re / s, im / s);
    } else if (pk) {
      *reinterpret_cast<double2*>(pk + b * (2 * N + 2) + 2 + 2 * n) = make_double2(re * psc, im * psc);
    } else {
      *reinterpret_cast<double2*>(oa + b * 2 * N + 2 * n) = make_double2(re, im);
    }
  };
  put(n0, re0, im0);
  put(n1, re1, im1);
  if (!h && lane == 0) {
    if (pk) {
      *reinterpret_cast<double2*>(pk + b * (2 * N + 2)) = make_double2(s * psc, 0.0);
    } else {
      om[b] = mx;
      os[b] = s;
    }
  }
}

// [m, s, acc] partial (acc f64, or f32 when acc32) -> shifted packed [s e^{m-M*}, 0, acc e^{m-M*}]
__global__ __launch_bounds__(256) void k_pack_shifted(long long B, int N, const double* __restrict__ m,
                                                      const double* __restrict__ s, const double* __restrict__ acc,
                                                      const float* __restrict__ acc32, const double* __restrict__ shift,
                                                      double* __restrict__ pk) {
  const long long W = 2LL * N + 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < B * W; i += (long long)gridDim.x * 256) {
    const long long b = i / W, j = i % W;
    const double sc = (m[b] == QCE_NEG_INF) ? 0.0 : exp(m[b] - *shift);
    double v;
    if (j == 0) v = s[b];
    else if (j == 1) v = 0.0;
    else v = acc32 ? (double)acc32[b * 2 * N + j - 2] : acc[b * 2 * N + j - 2];
    pk[i] = v * sc;
  }
}
hipError_t qce_launch_pack_shifted(long long B, int N, const double* m, const double* s, const double* acc,
                                   const float* acc32, const double* shift, double* pk, hipStream_t st) {
  long long blocks = (B * (2LL * N + 2) + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(k_pack_shifted, dim3((unsigned)blocks), dim3(256), 0, st, B, N, m, s, acc, acc32, shift, pk);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// prepare-side packing of the FP64 tables (one 64-thread group per 1 KB block)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pack_f64all(int M, int N, int MP, int NP, int has_mean, int bpc,
                                                    const double2* __restrict__ Linv, const double2* __restrict__ W,
                                                    const double2* __restrict__ q0, const double2* __restrict__ bvec,
                                                    double* __restrict__ pack) {
  const int pb = blockIdx.x, k = blockIdx.y, lane = threadIdx.x;
  const int NTL = MP / 8, NTW = NP / 8, KP = MP / 4, HMI = has_mean ? 1 : 0;
  // physical block pb = PR v + h: virtual block v of row half h (f64_pr, qce_f64_kernel.h)
  const int PR = f64_pr(MP, NP), b = pb / PR, h = pb % PR;
  const int NTLV = NTL / PR, NTWV = NTW / PR;
  auto gl_off = [&](int T) { return PR == 1 ? T * (T + 1) + HMI * T : 2 * T * (T - 1) + (4 + HMI) * T; };
  auto gl_len = [&](int T) { return PR == 1 ? 2 * T + 2 : 4 * T + 4; };
  const int gl_blocks = gl_off(NTLV);
  int kind = 4, T = 0, s = 0;
  if (b < gl_blocks) {
    while (b >= gl_off(T + 1)) ++T;
    s = b - gl_off(T);
    kind = s < gl_len(T) ? 0 : 1;
    T = PR * T + h;                               // the half's real row tile
    if (kind == 0 && s >= 2 * T + 2) kind = 4;    // half 0's k-pairs past its diagonal: zero block
  } else {
    const int r = b - gl_blocks;
    if (r < KP * NTWV) {
      kind = 2;
      s = r / NTWV;
      T = PR * (r % NTWV) + h;
    } else if (r < (KP + HMI) * NTWV) {
      kind = 3;
      T = PR * (r - KP * NTWV) + h;
    }
  }
  const int rho = lane & 15, gk = lane >> 4;
  const int i = 8 * T + 4 * (rho >> 3) + (rho & 3), a = (rho >> 2) & 1;
  const bool isL = kind <= 1;
  const int rows = isL ? M : N;
  double v[2] = {0.0, 0.0};
  if (kind == 0 || kind == 2) {
    const int j = 4 * s + gk;
    if (i < rows && j < M) {
      const double2 z = isL ? Linv[((long long)k * M + i) * M + j] : W[((long long)k * N + i) * M + j];
      v[0] = a == 0 ? z.x : z.y;   // k-step 2s: real part of column j
      v[1] = a == 0 ? -z.y : z.x;  // k-step 2s+1: imaginary part of column j
    }
  } else if ((kind == 1 || kind == 3) && gk == 0 && i < rows) {
    const double2 z = isL ? q0[(long long)k * M + i] : bvec[(long long)k * N + i];
    const double o = a == 0 ? z.x : z.y;
    v[0] = isL ? -o : o;
  }
  *reinterpret_cast<double2*>(pack + (((long long)k * bpc + pb) * 64 + lane) * 2) = make_double2(v[0], v[1]);
}

// 3M tables of k_est_all_f64g (qce_f64g_kernel.h): block j of unit u holds the A operands (Ls, Lm, Lp of the
// k-steps 2u, 2u + 1 in the order j = 0: Ls s0, Lm s0; 1: Lp s0, Ls s1; 2: Lm s1, Lp s1), Ls = Re + Im, Lm = -2 Im,
// Lp = 2 Re of the complex entry; lane (r, g) = row 16 T + r, column 4 s + g.  Mean block: (-q0 re, -q0 im) in
// k = 0; bias block: (b re, b im).
__global__ __launch_bounds__(64) void k_pack_f64g(int M, int N, int MP, int NP, int has_mean, int bpc,
                                                  const double2* __restrict__ Linv, const double2* __restrict__ W,
                                                  const double2* __restrict__ q0, const double2* __restrict__ bvec,
                                                  double* __restrict__ pack) {
  const int b = blockIdx.x, k = blockIdx.y, lane = threadIdx.x;
  const BlockInfo3 bi = block_info3_rt(MP, NP, has_mean ? 1 : 0, b);
  const int r = lane & 15, gk = lane >> 4;
  const int i = 16 * bi.T + r;
  const bool isL = bi.kind <= 1;
  const int rows = isL ? M : N;
  double v[2] = {0.0, 0.0};
  if (bi.kind == 0 || bi.kind == 2) {
    // (which, k-step) of the block's two MFMAs; which: 0 Ls, 1 Lm, 2 Lp
    const int s0 = 2 * bi.u, s1 = s0 + 1;
    const int wh[3][2] = {{0, 1}, {2, 0}, {1, 2}};
    const int ks[3][2] = {{s0, s0}, {s0, s1}, {s1, s1}};
    for (int e = 0; e < 2; ++e) {
      const int j = 4 * ks[bi.j][e] + gk;
      if (i < rows && j < M) {
        const double2 z = isL ? Linv[((long long)k * M + i) * M + j] : W[((long long)k * N + i) * M + j];
        const int which = wh[bi.j][e];
        v[e] = which == 0 ? z.x + z.y : (which == 1 ? -2.0 * z.y : 2.0 * z.x);
      }
    }
  } else if (bi.kind == 1 && gk == 0 && i < M) {
    const double2 z = q0[(long long)k * M + i];
    v[0] = -z.x;
    v[1] = -z.y;
  } else if (bi.kind == 3 && gk == 0 && i < N) {
    const double2 z = bvec[(long long)k * N + i];
    v[0] = z.x;
    v[1] = z.y;
  }
  *reinterpret_cast<double2*>(pack + (((long long)k * bpc + b) * 64 + lane) * 2) = make_double2(v[0], v[1]);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
int blocks_per_comp(int MP, int NP, int hm) { return f64_pack_blocks(MP, NP, hm ? 1 : 0); }
int blocks_per_comp_g(int MP, int NP, int hm) { return f64g_bpc(f64g_blocks(MP, NP, hm ? 1 : 0)); }
}  // namespace

// the 3M kernel covers padded M, N in {16, 32, 64} (8 waves x 16 samples; QCE_F64_3M=0 keeps the 4M kernel)
bool qce_f64g_shape(int MP, int NP) {
  const char* e = getenv("QCE_F64_3M");
  if (e && e[0] == '0') return false;
  auto ok = [](int v) { return v == 16 || v == 32 || v == 64; };
  return ok(MP) && ok(NP);
}
int qce_f64g_waves() { return QCE_F64G_NW; }
long long qce_pack_f64g_bytes(int MP, int NP, int has_mean) { return (long long)blocks_per_comp_g(MP, NP, has_mean) * 1024; }
hipError_t qce_launch_pack_f64g(int K, int M, int N, int MP, int NP, int has_mean, const double2* Linv,
                                const double2* W, const double2* q0, const double2* bvec, double* pack,
                                hipStream_t st) {
  const int bpc = blocks_per_comp_g(MP, NP, has_mean);
  hipLaunchKernelGGL(k_pack_f64g, dim3(bpc, K), dim3(64), 0, st, M, N, MP, NP, has_mean, bpc, Linv, W, q0, bvec,
                     pack);
  return hipGetLastError();
}

bool qce_f64_shape(int MP, int NP) {
  auto ok = [](int v) { return v == 16 || v == 32 || v == 64 || v == 128; };
  return ok(MP) && ok(NP);
}
int qce_f64_tile(int MP, int NP) { return 4 * 16 * ((MP <= 64 && NP <= 64) ? 2 : 1); }
long long qce_pack_f64all_bytes(int MP, int NP, int has_mean) { return (long long)blocks_per_comp(MP, NP, has_mean) * 1024; }

hipError_t qce_launch_pack_f64all(int K, int M, int N, int MP, int NP, int has_mean, const double2* Linv,
                                  const double2* W, const double2* q0, const double2* bvec, double* pack,
                                  hipStream_t st) {
  const int bpc = blocks_per_comp(MP, NP, has_mean);
  hipLaunchKernelGGL(k_pack_f64all, dim3(bpc, K), dim3(64), 0, st, M, N, MP, NP, has_mean, bpc, Linv, W, q0, bvec,
                     pack);
  return hipGetLastError();
}

template <int MP>
hipError_t qce_f64_launch_mp(const QceF64Args& a, bool out_partial, hipStream_t st);
template <int MP>
hipError_t qce_f64g_launch_mp(const QceF64Args& a, bool out_partial, hipStream_t st);

hipError_t qce_launch_est_f64(const QceF64Args& a, bool out_partial, hipStream_t st) {
  hipError_t e;
  if (a.g3 == 2) {
    e = qce_f64h_launch(a, out_partial, st);
  } else if (a.g3) {
    switch (a.MP) {
      case 16: e = qce_f64g_launch_mp<16>(a, out_partial, st); break;
      case 32: e = qce_f64g_launch_mp<32>(a, out_partial, st); break;
      case 64: e = qce_f64g_launch_mp<64>(a, out_partial, st); break;
      default: e = hipErrorInvalidValue;
    }
  } else switch (a.MP) {
    case 16: e = qce_f64_launch_mp<16>(a, out_partial, st); break;
    case 32: e = qce_f64_launch_mp<32>(a, out_partial, st); break;
    case 64: e = qce_f64_launch_mp<64>(a, out_partial, st); break;
    case 128: e = qce_f64_launch_mp<128>(a, out_partial, st); break;
    default: e = hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  const long long TS = a.g3 == 2 ? 64LL : (a.g3 ? 16LL * QCE_F64G_NW : qce_f64_tile(a.MP, a.NP));
  const long long tiles = (a.B + TS - 1) / TS;
  const long long tail0 = (long long)a.R * a.nwg;
  if (a.L > 0 && tiles > tail0) {  // some tail tile may be cut between workgroups
    const long long b0 = tail0 * TS;
    const long long nb = a.B - b0;
    hipLaunchKernelGGL(k_merge_f64, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, st, nb, a.N, a.K, (int)TS, a.L,
                       a.pm, a.ps, a.pa, out_partial ? nullptr : a.h + b0 * a.N, a.om ? a.om + b0 : nullptr,
                       a.os ? a.os + b0 : nullptr, a.oa ? a.oa + b0 * 2 * a.N : nullptr,
                       a.pk ? a.pk + b0 * (2 * a.N + 2) : nullptr, a.shift);
    e = hipGetLastError();
  }
  return e;
}

// precision conversions between the f32 and FP64 partial accumulators
__global__ __launch_bounds__(256) void k_f64_to_f32(const double* __restrict__ a, float* __restrict__ b, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = (float)a[i];
}
__global__ __launch_bounds__(256) void k_f32_to_f64(const float* __restrict__ a, double* __restrict__ b, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = (double)a[i];
}
hipError_t qce_launch_f64_to_f32(const double* a, float* b, long long n, hipStream_t st) {
  long long blocks = (n + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(k_f64_to_f32, dim3((unsigned)blocks), dim3(256), 0, st, a, b, n);
  return hipGetLastError();
}
hipError_t qce_launch_f32_to_f64(const float* a, double* b, long long n, hipStream_t st) {
  long long blocks = (n + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(k_f32_to_f64, dim3((unsigned)blocks), dim3(256), 0, st, a, b, n);
  return hipGetLastError();
}

// out[0] = max_k c_k, or +inf when the prepare left a non-zero Cholesky status for some component: the flag rides
// the shard shift through its MAX collective, so every rank learns of a failed factorisation on any rank without a
// host round trip (sharding.py raises the reference's ValueError, gmm_cplx_bussgang.py:43-46).
__global__ __launch_bounds__(256) void k_cconst_max(int K, const double* __restrict__ c, const int* __restrict__ status,
                                                    double* __restrict__ out) {
  __shared__ double red[256];
  double v = -__builtin_inf();
  for (int k = threadIdx.x; k < K; k += 256) v = fmax(v, (status && status[k]) ? __builtin_inf() : c[k]);
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}
hipError_t qce_launch_cconst_max(int K, const double* cconst, const int* status, double* out, hipStream_t st) {
  hipLaunchKernelGGL(k_cconst_max, dim3(1), dim3(256), 0, st, K, cconst, status, out);
  return hipGetLastError();
}
