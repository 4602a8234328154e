// Statistical achievable-rate lower bound of the scripts (Bussgang_GMM.py:146-162,
// :206-216, :238-249, :291-306), for estimates h_est (B,N) of channels h (B,N):
//   g_b = h_est_b / clip(||h_est_b||^2)          (the scripts divide by the squared norm; the GMM branch
//                                                  clips it below at 0.1, :296)
//   inner_b = g_b^H B h_b  (B = diagonal Bussgang gain),  den2_b = Re g_b^H Cq g_b
//   num = |mean inner|^2, den1 = var(inner) (numpy: mean |inner - mean|^2), den2 = mean den2_b
//   rate = log2(1 + num / (den1 + den2))
// One wave per sample for the O(N^2) quadratic form; fixed-order reductions (deterministic).
// Roofline: L2/HBM — per sample 32 N bytes of estimates and channels; Cq stays in L2.
#include "qce_common.h"
#include "qce_kernels.h"

namespace {

constexpr int RATE_BLOCKS = 256;

__global__ __launch_bounds__(256) void k_rate_samples(long long B, int N, const double2* __restrict__ he,
                                                      const double2* __restrict__ h, const double* __restrict__ buss,
                                                      const double2* __restrict__ Cq, double clip,
                                                      double2* __restrict__ inner, double* __restrict__ den2) {
  const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const double2* e = he + b * N;
  double nrm = 0.0;
  for (int n = lane; n < N; n += 64) nrm += e[n].x * e[n].x + e[n].y * e[n].y;
  for (int o = 32; o > 0; o >>= 1) nrm += __shfl_xor(nrm, o);
  if (clip > 0.0 && nrm < clip) nrm = clip;
  const double inv = 1.0 / nrm;
  double2 in = make_double2(0.0, 0.0);
  double q = 0.0;
  for (int i = lane; i < N; i += 64) {
    const double2 gi = make_double2(e[i].x * inv, e[i].y * inv);
    const double2 bh = make_double2(buss[i] * h[b * N + i].x, buss[i] * h[b * N + i].y);
    in = cadd(in, cmul(cconj(gi), bh));
    double2 cg = make_double2(0.0, 0.0);
    const double2* row = Cq + (long long)i * N;
    for (int j = 0; j < N; ++j) cg = cfma(row[j], make_double2(e[j].x * inv, e[j].y * inv), cg);
    q += gi.x * cg.x + gi.y * cg.y;  // Re(conj(g_i) (Cq g)_i)
  }
  for (int o = 32; o > 0; o >>= 1) {
    in.x += __shfl_xor(in.x, o);
    in.y += __shfl_xor(in.y, o);
    q += __shfl_xor(q, o);
  }
  if (lane == 0) {
    inner[b] = in;
    den2[b] = q;
  }
}

// pass 1 (mode 0): sums of inner and den2; pass 2 (mode 1): sum |inner - mean|^2
__global__ __launch_bounds__(256) void k_rate_partial(long long B, int mode, const double2* __restrict__ inner,
                                                      const double* __restrict__ den2, const double* __restrict__ stat,
                                                      double* __restrict__ part) {
  double a = 0.0, c = 0.0, d = 0.0;
  const double mx = mode ? stat[0] : 0.0, my = mode ? stat[1] : 0.0;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < B; e += (long long)RATE_BLOCKS * 256) {
    if (mode == 0) {
      a += inner[e].x;
      c += inner[e].y;
      d += den2[e];
    } else {
      const double dx = inner[e].x - mx, dy = inner[e].y - my;
      a += dx * dx + dy * dy;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    c += __shfl_xor(c, o);
    d += __shfl_xor(d, o);
  }
  __shared__ double red[3][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = c;
    red[2][threadIdx.x >> 6] = d;
  }
  __syncthreads();
  if (threadIdx.x < 3)
    part[threadIdx.x * RATE_BLOCKS + blockIdx.x] =
        (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// stat: [mean re, mean im, mean den2, den1, num, rate]
__global__ __launch_bounds__(64) void k_rate_final(long long B, int mode, const double* __restrict__ part,
                                                   double* __restrict__ stat) {
  double s[3] = {0.0, 0.0, 0.0};
  for (int q = 0; q < 3; ++q) {
    for (int i = threadIdx.x; i < RATE_BLOCKS; i += 64) s[q] += part[q * RATE_BLOCKS + i];
    for (int o = 32; o > 0; o >>= 1) s[q] += __shfl_xor(s[q], o);
  }
  if (threadIdx.x != 0) return;
  if (mode == 0) {
    stat[0] = s[0] / (double)B;
    stat[1] = s[1] / (double)B;
    stat[2] = s[2] / (double)B;
  } else {
    const double den1 = s[0] / (double)B;
    const double num = stat[0] * stat[0] + stat[1] * stat[1];
    stat[3] = den1;
    stat[4] = num;
    stat[5] = log2(1.0 + num / (den1 + stat[2]));
  }
}

}  // namespace

hipError_t qce_launch_rate(long long B, int N, const double2* he, const double2* h, const double* buss,
                           const double2* Cq, double clip, double2* inner, double* den2, double* part, double* stat,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_rate_samples, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, N, he, h, buss, Cq, clip, inner,
                     den2);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k_rate_partial, dim3(RATE_BLOCKS), dim3(256), 0, st, B, mode, inner, den2, stat, part);
    hipLaunchKernelGGL(k_rate_final, dim3(1), dim3(64), 0, st, B, mode, part, stat);
  }
  return hipGetLastError();
}

int qce_rate_scratch() { return 3 * RATE_BLOCKS; }
