// On-device 3GPP-like multi-path channels: SCMMulti.generate_channel
// (modules/SCM3GPP/SCMMulti.py:30-56) and scm_helper.chan_from_spectrum / spectrum / _laplace
// (scm_helper.py:17-84).  Per channel b and coherence column c:
//   F = 100 N frequency samples u_f = (f + 1/3) / F 2 pi - pi, theta = deg(asin(u / pi)),
//   fs_f = deg(2 pi (L(theta) + L(180 - theta)) / sqrt(pi^2 - u^2)),  L = Laplace mixture of the paths,
//   fs clipped at F, normalised to sum F;  h_n = sqrt(F) / F sum_f sqrt(fs_f) x_fc e^{+2 pi i f n / F}
//   (the first N outputs of the inverse FFT), t_n = 1/F sum_f fs_f e^{-2 pi i f n / F}  (n < N).
// Only N of the F outputs are kept, so the two partial DFTs (N x F each) are evaluated directly in
// FP64: fs is recomputed chunk by chunk (cheap next to the DFT), x_f sqrt(fs_f) and fs_f are staged in
// LDS per chunk of 256 frequencies, thread (group g, output n) accumulates its slice of the chunk with a
// twiddle recurrence restarted exactly (sincospi of an integer phase) at every chunk, and the group
// partials are added in a fixed order.  Outputs are complex64 like the reference's arrays.
// Random inputs (path gains, angles, x) are either supplied — bit-for-bit the reference's draws — or
// drawn on the device from Philox4x32-10 (seed; distinct counters per channel / frequency / column).
// Roofline: FP64 VALU; 2 complex MACs + 1 complex twiddle step per (f, n): 8 F N (+ 6 F N) flops per column.
#include "qce_common.h"
#include "qce_kernels.h"

namespace {

constexpr double PI = 3.14159265358979323846;
constexpr int SCM_THREADS = 256;
constexpr int SCM_CHUNK = 256;
constexpr int SCM_MAX_PATH = 16;

QCE_DEV uint4 philox_scm(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

QCE_DEV double u53(uint32_t hi, uint32_t lo) { return (double)((((unsigned long long)hi << 32) | lo) >> 11) * 0x1.0p-53; }

// numpy float remainder (sign of the divisor)
QCE_DEV double npmod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0 && ((b < 0.0) != (m < 0.0))) m += b;
  return m;
}

QCE_DEV double rad2deg(double x) { return x * (180.0 / PI); }

// spectrum(u) of scm_helper.py:17-24 with _laplace (:27-36), before clipping
QCE_DEV double scm_spectrum(double u, int n_path, const double* ang, const double* w, double sigma) {
  u = npmod(u + PI, 2.0 * PI) - PI;
  const double theta = rad2deg(asin(u / PI));
  const double sc = sigma / sqrt(2.0);
  double v = 0.0;
  for (int p = 0; p < n_path; ++p) {
    const double x1 = npmod(theta - ang[p] + 180.0, 360.0) - 180.0;
    const double x2 = npmod(180.0 - theta - ang[p] + 180.0, 360.0) - 180.0;
    v += w[p] / (2.0 * sc) * exp(-fabs(x1) / sc);
    v += w[p] / (2.0 * sc) * exp(-fabs(x2) / sc);
  }
  return rad2deg(2.0 * PI * v / sqrt(PI * PI - u * u));
}

QCE_DEV double scm_fs(int f, int F, int n_path, const double* ang, const double* w, double sigma) {
  const double u = ((double)f + 1.0 / 3.0) / (double)F * 2.0 * PI - PI;
  double fs = scm_spectrum(u, n_path, ang, w, sigma);
  const double cap = F > 1 ? (double)F : 1.0;
  if (fabs(fs) > cap) fs = cap;
  return fs;
}

template <int NPAD>
__global__ __launch_bounds__(SCM_THREADS) void k_scm(long long B, int n_coh, int N, int n_path, double sigma,
                                                     const double* __restrict__ gains, const double* __restrict__ angles,
                                                     const double2* __restrict__ x, unsigned long long seed,
                                                     float2* __restrict__ h, float2* __restrict__ t) {
  constexpr int G = SCM_THREADS / NPAD;  // groups over the chunk
  constexpr int PER = SCM_CHUNK / G;     // frequencies per thread per chunk
  __shared__ double s_w[SCM_MAX_PATH], s_a[SCM_MAX_PATH];
  __shared__ double2 s_x[SCM_CHUNK];
  __shared__ double s_fs[SCM_CHUNK];
  __shared__ double s_red[SCM_THREADS / 64];
  __shared__ double2 s_acc[G][NPAD][2];
  const long long b = blockIdx.x;
  const int c = blockIdx.y, tid = threadIdx.x;
  const int F = 100 * N;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  if (tid == 0) {
    if (gains) {
      for (int p = 0; p < n_path; ++p) {
        s_w[p] = gains[b * n_path + p];
        s_a[p] = angles[b * n_path + p];
      }
    } else {  // SCMMulti.py:49-51: gains = u / sum u; angles = (u - 0.5) 180
      double g[SCM_MAX_PATH], s = 0.0;
      for (int p = 0; p < n_path; ++p) {
        const uint4 r = philox_scm(make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)p, 0xA11CE5u), key);
        g[p] = u53(r.x, r.y);
        s += g[p];
        s_a[p] = (u53(r.z, r.w) - 0.5) * 180.0;
      }
      for (int p = 0; p < n_path; ++p) s_w[p] = g[p] / s;
    }
  }
  __syncthreads();
  // pass 1: sum of the clipped spectrum (fixed-order block reduction)
  double part = 0.0;
  for (int f = tid; f < F; f += SCM_THREADS) part += scm_fs(f, F, n_path, s_a, s_w, sigma);
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  if ((tid & 63) == 0) s_red[tid >> 6] = part;
  __syncthreads();
  const double S = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
  const bool norm = S > 0.0;
  // pass 2: chunked partial DFTs
  const int n = tid % NPAD, g = tid / NPAD;
  double2 ah = make_double2(0.0, 0.0), at = make_double2(0.0, 0.0);
  double st, ct;
  sincospi(2.0 * (double)n / (double)F, &st, &ct);  // e^{+2 pi i n / F}
  for (int f0 = 0; f0 < F; f0 += SCM_CHUNK) {
    {
      const int f = f0 + tid;
      double2 xv = make_double2(0.0, 0.0);
      double fsn = 0.0;
      if (f < F) {
        const double fs = scm_fs(f, F, n_path, s_a, s_w, sigma);
        fsn = norm ? fs / S * (double)F : fs;
        if (x) {
          xv = x[(b * F + f) * n_coh + c];
        } else {  // crandn (utils.py:13-14) on the device
          const unsigned long long e = ((unsigned long long)b * F + f) * n_coh + c;
          const uint4 r = philox_scm(make_uint4((uint32_t)e, (uint32_t)(e >> 32), 0x5C3u, 0xC0FFEEu), key);
          const double u1 = (double)((((unsigned long long)r.x << 32 | r.y) >> 11) + 1) * 0x1.0p-53;
          const double u2 = u53(r.z, r.w);
          const double rad = sqrt(-2.0 * log(u1)) * 0x1.6a09e667f3bcdp-1;
          double sn, cs;
          sincospi(2.0 * u2, &sn, &cs);
          xv = make_double2(rad * cs, rad * sn);
        }
        const double sq = sqrt(fsn);
        xv = make_double2(sq * xv.x, sq * xv.y);
      }
      s_x[tid] = xv;
      s_fs[tid] = fsn;
    }
    __syncthreads();
    if (n < N) {
      const int fb = f0 + g * PER;
      // exact start phase: e^{2 pi i (fb n mod F) / F}
      const long long ph = ((long long)fb * n) % F;
      double sw, cw;
      sincospi(2.0 * (double)ph / (double)F, &sw, &cw);
      double2 tw = make_double2(cw, sw);
      const int lim = F - fb < PER ? F - fb : PER;
      for (int q = 0; q < lim; ++q) {
        const double2 xv = s_x[g * PER + q];
        const double fv = s_fs[g * PER + q];
        ah = cfma(xv, tw, ah);                                       // + phase (inverse FFT)
        at = make_double2(at.x + fv * tw.x, at.y - fv * tw.y);       // - phase (forward FFT)
        tw = make_double2(tw.x * ct - tw.y * st, tw.x * st + tw.y * ct);
      }
    }
    __syncthreads();
  }
  s_acc[g][n][0] = ah;
  s_acc[g][n][1] = at;
  __syncthreads();
  if (g == 0 && n < N) {
    for (int q = 1; q < G; ++q) {
      ah = cadd(ah, s_acc[q][n][0]);
      at = cadd(at, s_acc[q][n][1]);
    }
    const double sh = sqrt((double)F) / (double)F;
    h[(b * n_coh + c) * N + n] = make_float2((float)(ah.x * sh), (float)(ah.y * sh));
    if (c == 0) t[b * N + n] = make_float2((float)(at.x / F), (float)(at.y / F));
  }
}

}  // namespace

int qce_scm_max_path() { return SCM_MAX_PATH; }

hipError_t qce_launch_scm(long long B, int n_coh, int N, int n_path, double sigma, const double* gains,
                          const double* angles, const double2* x, unsigned long long seed, float2* h, float2* t,
                          hipStream_t st) {
  const dim3 grid((unsigned)B, (unsigned)n_coh);
  if (N <= 32) hipLaunchKernelGGL(k_scm<32>, grid, dim3(SCM_THREADS), 0, st, B, n_coh, N, n_path, sigma, gains, angles, x, seed, h, t);
  else if (N <= 64) hipLaunchKernelGGL(k_scm<64>, grid, dim3(SCM_THREADS), 0, st, B, n_coh, N, n_path, sigma, gains, angles, x, seed, h, t);
  else if (N <= 128) hipLaunchKernelGGL(k_scm<128>, grid, dim3(SCM_THREADS), 0, st, B, n_coh, N, n_path, sigma, gains, angles, x, seed, h, t);
  else hipLaunchKernelGGL(k_scm<256>, grid, dim3(SCM_THREADS), 0, st, B, n_coh, N, n_path, sigma, gains, angles, x, seed, h, t);
  return hipGetLastError();
}
