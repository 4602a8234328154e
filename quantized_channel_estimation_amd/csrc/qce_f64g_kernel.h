// Fused 'all'-mode estimate kernel in FP64 with Gauss's three-product complex multiply (3M) on
// v_mfma_f64_16x16x4_f64 -- the headline kernel for padded M, N <= 64 (gmm_cplx_bussgang.py:220-228 with
// :331-332, :388-435, :632-656; every reference step is complex128, and so is every step here).
//
// k_est_all_f64 (qce_f64_kernel.h) multiplies the real 2x2 embedding E(L) [Re y; Im y]: four real products per
// complex one.  On gfx950 that kernel sits at the FP64 MFMA pipe's limit, so the lever is the MFMA count.  With
// complex rows on the MFMA row axis (16 complex rows per tile) each complex product L y over a tile takes three
// real products instead (per k-step of 4 complex columns, tables packed at prepare):
//
//   K1 = (Lr + Li) yr,   R' = (-2 Li) hs,   I' = (2 Lr) hd,   hs = (yr + yi) / 2,  hd = (yi - yr) / 2,
//   Re(L y) = K1 + R',   Im(L y) = K1 + I'                     (yr = hs - hd; the halvings are exact)
//
// so the quad form and the filter take 3/4 of the MFMAs (the 16-row tiles' triangle costs a little of it back:
// 120 + 192 MFMAs per component and 16 samples at M = N = 64, against 144 + 256).  Each of K1, R', I' is an FP64
// accumulation of FP64 products: the result is an FP64 computation of the reference formula that differs from it
// (and from the 4M kernel) by rounding only.
//
//   lp_bk = c_k - sum_rows (K1 + R')^2 + (K1 + I')^2           (GL: L = Linv_k, the mean as a -q0 column)
//   h_b   = sum_k p_bk (W_k y_b + b_k) / sum_k p_bk             (GW: the three products accumulated over k)
//
// The GW accumulators are three sets (K1, R', I') summed over the components and combined once per tile; the
// B operands p hs, p hd, p yr are formed once per k-step and component.  y is held as (hs, hd).
//
// Layout (k_pack_f64g): per component GL blocks (row tile T outer; units of two k-steps, 2T + 2 of them -- the
// upper triangle past the 16-row diagonal tile skipped; three 1 KB blocks per unit; + one mean block), then GW
// blocks (unit outer, then block j, row tile inner; + one bias block per row tile), padded to whole ring
// chunks.  Block j of unit u (k-steps s0 = 2u, s1 = 2u + 1) holds the A operands of two MFMAs:
//   j = 0: (Ls, s0) (Lm, s0)    j = 1: (Lp, s0) (Ls, s1)    j = 2: (Lm, s1) (Lp, s1)
// with Ls = Lr + Li (-> K1, B = yr), Lm = -2 Li (-> R', B = hs), Lp = 2 Lr (-> I', B = hd): consecutive MFMAs
// alternate between the three accumulators.  A operand lane (r, g) = matrix[16 T + r][4 s + g]; the accumulator
// register i of lane (g, col) is complex row 16 T + g + 4 i of sample col.
//
// Scheduling as k_est_all_f64's 8-wave shape: one workgroup = 8 waves (two per SIMD) x 16 samples, the tables
// streamed through an LDS ring of NSLOT chunks (global_load_lds DMA), persistent grid with a stream-K tail whose cut
// tiles leave FP64 partials for k_merge_f64 (same format).
#pragma once
#include "qce_f64_kernel.h"

// LDS operand prefetch distance (blocks).  Smaller than the 4M kernel's 8: the three accumulator sets of the filter
// take the registers (E = 4..8 were within 0.5 % of each other on the 4M kernel, profiles/r04_f64_prefetch_ab2.txt).
#ifndef QCE_F64G_E
#define QCE_F64G_E 2
#endif
// waves per workgroup: 8 (one 8-wave workgroup per CU, two waves per SIMD, one ring of <= 144 KB) or 4 (two
// 4-wave workgroups per CU, each with its own ring of <= 72 KB: a workgroup's ring barriers then sync one wave per
// SIMD, the other workgroup's wave keeps the SIMD's MFMA pipe busy)
#ifndef QCE_F64G_NW
#define QCE_F64G_NW 8
#endif
// ring chunk (blocks); 0 = chosen from the block count (f64_cb)
#ifndef QCE_F64G_CB
#define QCE_F64G_CB 0
#endif
// waves 4-7 (the second wave of every SIMD) consume the ring LAG chunks behind waves 0-3, so the two waves of a SIMD
// reach their softmax and GL folds at different times (the ring keeps LAG more chunks; 0 = lockstep)
#ifndef QCE_F64G_LAG
#define QCE_F64G_LAG 0
#endif
// 1: libm exp for the softmax weights (A/B builds)
#ifndef QCE_F64G_LIBM_EXP
#define QCE_F64G_LIBM_EXP 0
#endif

namespace {

// e^x for x <= 700 with a 32-entry LDS table of 2^(j/32) and a degree-6 polynomial of e^r, |r| <= ln 2 / 64
// (truncation 4e-18, about 2 ulp): 18 VALU and four non-inline constants against libm's ~32 instructions and
// ~13 constants that the compiler keeps in VGPRs across the component loop (they spilled beside the 3M kernel's
// accumulators).  x = -inf and x < -708 give e^-708 = 3e-308, negligible beside the softmax's largest weight 1.
QCE_DEV double exp_tab64(double x, const double* __restrict__ tab) {
  constexpr double L32 = 46.166241308446828384;     // 32 / ln 2
  constexpr double LH = 2.1660849390173098072e-02;  // ln 2 / 32, leading bits
  constexpr double LL = 2.3251928468788740148e-12;  // ln 2 / 32 - LH
  x = fmax(x, -708.0);
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

// ring chunk (blocks) and padded blocks per component of the 3M table: shared by the kernel and k_pack_f64g
constexpr __host__ __device__ int f64g_cb(int blocks) {
  return QCE_F64G_CB > 0 ? QCE_F64G_CB : (QCE_F64G_NW == 8 ? f64_cb(blocks, 0, 1) : 24);
}
constexpr __host__ __device__ int f64g_bpc(int blocks) { return (blocks + f64g_cb(blocks) - 1) / f64g_cb(blocks) * f64g_cb(blocks); }
constexpr __host__ __device__ int f64g_blocks(int MP, int NP, int hmi) {
  return 3 * (MP / 16) * (MP / 16 + 1) + hmi * (MP / 16) + 3 * (MP / 8) * (NP / 16) + hmi * (NP / 16);
}

template <int MP, int NP, bool HM>
struct F64G3 {
  static constexpr int NTL = MP / 16;  // GL row tiles (16 complex rows)
  static constexpr int NTW = NP / 16;  // GW row tiles
  static constexpr int KS = MP / 4;    // k-steps (4 complex columns)
  static constexpr int KU = KS / 2;    // units of two k-steps (three blocks)
  static constexpr int HMI = HM ? 1 : 0;
  static constexpr __host__ __device__ int gl_units(int T) { return 2 * T + 2; }
  static constexpr __host__ __device__ int gl_off(int T) { return 3 * T * (T + 1) + HMI * T; }
  static constexpr int GL_BLOCKS = gl_off(NTL);
  static constexpr int GW_BLOCKS = 3 * KU * NTW + HMI * NTW;
  static constexpr int BLOCKS = GL_BLOCKS + GW_BLOCKS;
  static constexpr int NWG = QCE_F64G_NW;  // waves per workgroup
  static constexpr int LDS_KB = NWG == 8 ? 144 : 72;
  static constexpr int CB = f64g_cb(BLOCKS);
  static constexpr int LAG = QCE_F64G_LAG;
  static constexpr int NSLOT = LDS_KB / CB < 8 ? LDS_KB / CB : 8;
  static constexpr int CHUNK = CB * 1024;
  static constexpr int BPC = f64g_bpc(BLOCKS);
  static_assert(BLOCKS == f64g_blocks(MP, NP, HMI), "block count");
  static constexpr int CPC = BPC / CB;
};

struct BlockInfo3 {
  int kind, T, u, j;  // kind: 0 GL data, 1 GL mean, 2 GW data, 3 GW bias, 4 pad
};

__host__ __device__ constexpr BlockInfo3 block_info3_rt(int MP, int NP, int hmi, int b) {
  const int NTL = MP / 16, NTW = NP / 16, KU = MP / 8;
  auto gl_off = [&](int T) { return 3 * T * (T + 1) + hmi * T; };
  const int gl_blocks = gl_off(NTL);
  if (b < gl_blocks) {
    int T = 0;
    while (b >= gl_off(T + 1)) ++T;
    const int r = b - gl_off(T);
    if (r < 3 * (2 * T + 2)) return BlockInfo3{0, T, r / 3, r % 3};
    return BlockInfo3{1, T, 0, 0};
  }
  const int r = b - gl_blocks;
  if (r < 3 * KU * NTW) {  // unit u outer, block j, row tile T inner
    const int rem = r % (3 * NTW);
    return BlockInfo3{2, rem % NTW, r / (3 * NTW), rem / NTW};
  }
  if (r < 3 * KU * NTW + hmi * NTW) return BlockInfo3{3, r - 3 * KU * NTW, 0, 0};
  return BlockInfo3{4, 0, 0, 0};
}

}  // namespace

template <int MP, int NP, bool HM, bool OUT_PARTIAL>
__global__ __launch_bounds__(QCE_F64G_NW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_est_all_f64g(long long B, int M, int N, int K, int R, long long L,
                                                      const double2* __restrict__ y, const char* __restrict__ pack,
                                                      const double* __restrict__ cconst, double2* __restrict__ h,
                                                      double* __restrict__ om, double* __restrict__ os,
                                                      double* __restrict__ oa, double* __restrict__ pm,
                                                      double* __restrict__ ps, double* __restrict__ pa,
                                                      double* __restrict__ pk, const double* __restrict__ shift,
                                                      unsigned long long* __restrict__ stamps) {
  using G = F64G3<MP, NP, HM>;
  constexpr int NW = G::NWG;       // waves of 16 samples; two per SIMD (one or two workgroups per CU)
  constexpr int TS = NW * 16;     // samples per tile
  constexpr int LPW = G::CB / NW;  // global_load_lds pieces per wave per chunk
  constexpr int E = QCE_F64G_E;
  constexpr double RESCALE = 32.0;  // lazy max: rescale only when lp exceeds m by this
  static_assert(G::CB % NW == 0, "chunk split");
  static_assert(E < G::CB, "the prefetch window must stay inside one chunk");
  static_assert(G::NSLOT >= 3 + G::LAG, "ring depth");
  static_assert(G::LAG == 0 || NW == 8, "lag: two waves per SIMD in one workgroup");
  __shared__ __attribute__((aligned(16))) char lds[G::NSLOT * G::CHUNK];
  __shared__ double etab[32];  // 2^(j/32) for exp_tab64

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, col = lane & 15;
  if (threadIdx.x < 32) etab[threadIdx.x] = exp2((double)threadIdx.x / 32.0);  // visible after the first barrier
  const long long P = gridDim.x, w = blockIdx.x;
  const long long tiles = (B + TS - 1) / TS;
  const long long tail0 = (long long)R * P;
  const long long item0 = w * L;
  const long long tail_items = (tiles - tail0) * K;
  const long long item1 = (item0 + L < tail_items) ? item0 + L : tail_items;
  const long long ntail = item1 > item0 ? item1 - item0 : 0;
  if ((long long)R == 0 && ntail == 0) return;  // nothing for this workgroup (uniform)
  const long long t_first = tail0 + (L > 0 ? item0 / K : 0);
  const long long nseg = (long long)R + (ntail > 0 ? (item1 - 1) / K - item0 / K + 1 : 0);

  F64_STAMP_DECL
  // ---- ring (as k_est_all_f64) ----
  RingCursor cur;
  cur.init(R * K, (int)(item0 % K), (int)ntail, K, G::CPC);
  int issued = 0;
  const char* rsrc = pack;
  int rdst = 0;
  auto refill_begin = [&]() {
    rsrc = pack + cur.chunk_index() * (long long)G::CHUNK + wave * 1024 + lane * 16;
    rdst = (issued % G::NSLOT) * G::CHUNK + wave * 1024;
    cur.advance();
    ++issued;
  };
  auto refill_pieces = [&](int lo, int hi) {
    for (int i = lo; i < hi; ++i) lds_dma16(rsrc + i * NW * 1024, lds + rdst + i * NW * 1024);
  };
  // chunk k lands by barrier k: at barrier k the slot of chunk k - LAG - 2 is free (the lagging waves are done
  // with it) and takes chunk k + NSLOT - LAG - 2
  auto boundary_wait = [&]() {
    wait_vmcnt<(G::NSLOT - 3 - G::LAG) * LPW>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    F64_STAMP(3);
  };
#pragma unroll 1
  for (int j = 0; j < G::NSLOT - 2 - G::LAG; ++j) {
    refill_begin();
    refill_pieces(0, LPW);
  }
  boundary_wait();  // chunk 0
  refill_begin();
  refill_pieces(0, LPW);
  const bool lagging = G::LAG > 0 && wave >= NW / 2;  // wave-uniform
  if (lagging) {  // the lagging waves' first LAG barriers: refills only
#pragma unroll 1
    for (int j = 0; j < G::LAG; ++j) {
      boundary_wait();
      refill_begin();
      refill_pieces(0, LPW);
    }
  }
  int cstream = 0;

  for (long long seg = 0; seg < nseg; ++seg) {
    long long t;
    int klo, khi;
    if (seg < R) {
      t = seg * P + w;
      klo = 0;
      khi = K;
    } else {
      t = tail0 + item0 / K + (seg - R);
      const long long tK = (t - tail0) * K;
      klo = (int)((item0 > tK ? item0 : tK) - tK);
      khi = (int)((tK + K < item1 ? tK + K : item1) - tK);
    }
    const long long sbase = t * TS + (long long)wave * 16;
    // y fragments: k-step s, lane group g -> complex column 4s + g as (hs, hd) = ((yr + yi) / 2, (yi - yr) / 2).
    // Rows past B and columns past M are clamped (finite values meeting zero table entries / never written).
    double2 hv[G::KS];
    {
      int gl = g, cl = col;
      asm volatile("" : "+v"(gl), "+v"(cl));
      long long sm = sbase + cl;
      sm = sm < B ? sm : B - 1;
      const double2* yr = y + sm * M;
#pragma unroll
      for (int s = 0; s < G::KS; ++s) {
        const int cc = 4 * s + gl;
        hv[s] = yr[cc < M ? cc : M - 1];
      }
      wait_vmcnt<0>();
#pragma unroll
      for (int s = 0; s < G::KS; ++s) {
        const double a = hv[s].x, b = hv[s].y;
        hv[s] = make_double2(0.5 * (a + b), 0.5 * (b - a));
      }
    }
    F64_STAMP(5);
    f64x4 ok[G::NTW], orr[G::NTW], oi[G::NTW];
#pragma unroll
    for (int T = 0; T < G::NTW; ++T) ok[T] = orr[T] = oi[T] = f64x4{0.0, 0.0, 0.0, 0.0};
    double m = QCE_NEG_INF, ssum = 0.0;

#pragma unroll 1
    for (int k = klo; k < khi; ++k) {
      const double ck = cconst[k];
      int rslot = cstream % G::NSLOT;
      int roff = lane * 16 + rslot * G::CHUNK;
      auto rd = [&](int off) -> double2 { return *reinterpret_cast<const double2*>(&lds[roff + off]); };
      // yr = hs - hd is formed at each use as fma(hd, neg1, hs) with an opaque -1: loop-invariant, the compiler would
      // otherwise keep all KS of them in registers across the component loop
      double neg1 = -1.0;
      asm volatile("" : "+v"(neg1));
      f64x4 k1 = f64x4{0.0, 0.0, 0.0, 0.0}, rr = k1, ii = k1;
      double qp = 0.0, p = 0.0;
      double pr0 = 0.0, ps0 = 0.0, pd0 = 0.0, pr1 = 0.0, ps1 = 0.0, pd1 = 0.0;
      double2 buf[E + 1];
#pragma unroll
      for (int i = 0; i < E; ++i) buf[i] = rd(i * 1024);
      static_for(
          [&](auto bc) {
            constexpr int b = decltype(bc)::value;
            constexpr BlockInfo3 bi = block_info3_rt(MP, NP, G::HMI, b);
            __builtin_amdgcn_sched_barrier(0);
            constexpr bool RB = (b + E) % G::CB == 0;
            if constexpr (RB) {
              F64_STAMP(bi.kind <= 1 ? 0 : 2);
              boundary_wait();
              refill_begin();
            }
            if constexpr (b + E < G::BPC) {
              constexpr int r = b + E;
              if constexpr (r % G::CB == 0) {
                rslot = rslot + 1 == G::NSLOT ? 0 : rslot + 1;
                roff = lane * 16 + rslot * G::CHUNK;
                asm volatile("" : "+v"(roff));
              }
              buf[r % (E + 1)] = rd((r % G::CB) * 1024);
            }
            const double2 a = buf[b % (E + 1)];
            constexpr int NMF = bi.kind == 4 ? 0 : 2;
            int jm = 0;
            auto gap = [&]() {
              if constexpr (RB && NMF > 0) {
                __builtin_amdgcn_sched_barrier(0);
                refill_pieces(jm * LPW / NMF, (jm + 1) * LPW / NMF);
                __builtin_amdgcn_sched_barrier(0);
              }
              ++jm;
            };
            constexpr int s0 = 2 * bi.u, s1 = 2 * bi.u + 1;
            if constexpr (bi.kind == 0) {  // GL data
              if constexpr (bi.j == 0) {
                k1 = mfma16x16x4d(a.x, fma(hv[s0].y, neg1, hv[s0].x), k1);
                gap();
                rr = mfma16x16x4d(a.y, hv[s0].x, rr);
                gap();
              } else if constexpr (bi.j == 1) {
                ii = mfma16x16x4d(a.x, hv[s0].y, ii);
                gap();
                k1 = mfma16x16x4d(a.y, fma(hv[s1].y, neg1, hv[s1].x), k1);
                gap();
              } else {
                rr = mfma16x16x4d(a.x, hv[s1].x, rr);
                gap();
                ii = mfma16x16x4d(a.y, hv[s1].y, ii);
                gap();
              }
            } else if constexpr (bi.kind == 1) {  // GL mean column (-q0): B = 1 in lane group 0
              const double one = g == 0 ? 1.0 : 0.0;
              rr = mfma16x16x4d(a.x, one, rr);
              gap();
              ii = mfma16x16x4d(a.y, one, ii);
              gap();
            } else if constexpr (bi.kind == 2) {  // GW data: B operands formed once per component, j phase by j phase
              if constexpr (bi.T == 0 && bi.j == 0) {
                ps0 = p * hv[s0].x;
                pd0 = p * hv[s0].y;
                pr0 = ps0 - pd0;
              } else if constexpr (bi.T == 0 && bi.j == 1) {
                ps1 = p * hv[s1].x;
                pd1 = p * hv[s1].y;
                pr1 = ps1 - pd1;
              }
              if constexpr (bi.j == 0) {
                ok[bi.T] = mfma16x16x4d(a.x, pr0, ok[bi.T]);
                gap();
                orr[bi.T] = mfma16x16x4d(a.y, ps0, orr[bi.T]);
                gap();
              } else if constexpr (bi.j == 1) {
                oi[bi.T] = mfma16x16x4d(a.x, pd0, oi[bi.T]);
                gap();
                ok[bi.T] = mfma16x16x4d(a.y, pr1, ok[bi.T]);
                gap();
              } else {
                orr[bi.T] = mfma16x16x4d(a.x, ps1, orr[bi.T]);
                gap();
                oi[bi.T] = mfma16x16x4d(a.y, pd1, oi[bi.T]);
                gap();
              }
            } else if constexpr (bi.kind == 3) {  // GW bias column (b): B = p in lane group 0
              const double pone = g == 0 ? p : 0.0;
              orr[bi.T] = mfma16x16x4d(a.x, pone, orr[bi.T]);
              gap();
              oi[bi.T] = mfma16x16x4d(a.y, pone, oi[bi.T]);
              gap();
            }
            if constexpr (RB && NMF == 0) refill_pieces(0, LPW);
            // end of a GL row tile: |z|^2 of its 16 complex rows into the lane's quad-form partial (folding one block
            // later, after the next tile's first MFMAs, measured 1 % slower: the extra live accumulators spill)
            if constexpr (bi.kind == 0 || bi.kind == 1) {
              constexpr bool last =
                  HM ? (bi.kind == 1) : (bi.u == G::gl_units(bi.T) - 1 && bi.j == 2);
              if constexpr (last) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const double zr = k1[i] + rr[i], zi = k1[i] + ii[i];
                  qp = fma(zr, zr, qp);
                  qp = fma(zi, zi, qp);
                }
                asm volatile("" : "+v"(qp));
                k1 = rr = ii = f64x4{0.0, 0.0, 0.0, 0.0};
              }
            }
            // after the last GL block: log-probability and the online softmax (FP64)
            if constexpr (b == G::GL_BLOCKS - 1) {
              F64_STAMP(0);
              const double lp = ck - sum_groups(qp);
              if (__builtin_amdgcn_ballot_w64(lp > m + RESCALE) != 0ull) {  // rare: new running maximum
                const bool up = lp > m + RESCALE;
                const double mn = up ? lp : m;
                const double al = up ? (m == QCE_NEG_INF ? 0.0 : exp(m - mn)) : 1.0;
                ssum *= al;
                m = mn;
#pragma unroll
                for (int T = 0; T < G::NTW; ++T) {
                  ok[T] *= al;
                  orr[T] *= al;
                  oi[T] *= al;
                }
              }
#if QCE_F64G_LIBM_EXP
              p = (lp == QCE_NEG_INF) ? 0.0 : exp(lp - m);
#else
              p = (lp == QCE_NEG_INF) ? 0.0 : exp_tab64(lp - m, etab);
#endif
              ssum += p;
              F64_STAMP(1);
            }
          },
          std::make_integer_sequence<int, G::BPC>{});
      F64_STAMP(2);
      cstream += G::CPC;
    }

    // ---- write the tile: row 16 T + g + 4 i of sample col = (K1 + R', K1 + I') ----
    {
      int gw = g;
      asm volatile("" : "+v"(gw));
      const int ls = wave * 16 + col;
      const long long sample = t * TS + ls;
      if (sample < B) {
        const bool whole = (klo == 0 && khi == K);
        const bool pfmt = OUT_PARTIAL || !whole;
        const long long row = whole ? sample : (w * 2 + (t == t_first ? 0 : 1)) * TS + ls;
        if (OUT_PARTIAL && whole && pk) {  // shifted packed partial: [s e^{m-M*}, 0, acc e^{m-M*}] (K-shard sum)
          const double sc = (m == QCE_NEG_INF) ? 0.0 : exp(m - *shift);
          double* dp = pk + sample * (2LL * N + 2);
          if (g == 0) *reinterpret_cast<double2*>(dp) = make_double2(ssum * sc, 0.0);
#pragma unroll
          for (int T = 0; T < G::NTW; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * T + gw + 4 * i;
              if (n < N)
                *reinterpret_cast<double2*>(dp + 2 + 2 * n) =
                    make_double2((ok[T][i] + orr[T][i]) * sc, (ok[T][i] + oi[T][i]) * sc);
            }
        } else if (pfmt) {
          double* dm = whole ? om : pm;
          double* ds = whole ? os : ps;
          double* da = (whole ? oa : pa) + row * (2LL * N);
          if (g == 0) {
            dm[row] = m;
            ds[row] = ssum;
          }
#pragma unroll
          for (int T = 0; T < G::NTW; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * T + gw + 4 * i;
              if (n < N)
                *reinterpret_cast<double2*>(da + 2 * n) = make_double2(ok[T][i] + orr[T][i], ok[T][i] + oi[T][i]);
            }
        } else {
          const double inv = 1.0 / ssum;
          double2* hp = h + sample * N;
#pragma unroll
          for (int T = 0; T < G::NTW; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * T + gw + 4 * i;
              if (n < N) hp[n] = make_double2((ok[T][i] + orr[T][i]) * inv, (ok[T][i] + oi[T][i]) * inv);
            }
        }
      }
    }
  }
  if (G::LAG > 0 && !lagging) {  // the leading waves' last LAG barriers, matching the lagging waves' first ones
#pragma unroll 1
    for (int j = 0; j < G::LAG; ++j) {
      boundary_wait();
      refill_begin();
      refill_pieces(0, LPW);
    }
  }
  F64_STAMP(5);
  F64_STAMP_FLUSH
  wait_vmcnt<0>();  // drain the (dummy) ring prefetches before the workgroup retires
}

template <int MP, int NP, bool HM, bool OP>
hipError_t qce_f64g_launch_t(const QceF64Args& a, hipStream_t st) {
  hipLaunchKernelGGL((k_est_all_f64g<MP, NP, HM, OP>), dim3((unsigned)a.nwg), dim3(QCE_F64G_NW * 64), 0, st, a.B, a.M, a.N, a.K,
                     a.R, a.L, a.y, a.pack, a.cconst, a.h, a.om, a.os, a.oa, a.pm, a.ps, a.pa, a.pk, a.shift,
                     a.stamps);
  return hipGetLastError();
}

// one launcher per padded observation dimension MP in {16, 32, 64} (instantiated in qce_f64g_m<MP>.hip)
template <int MP>
hipError_t qce_f64g_launch_mp(const QceF64Args& a, bool out_partial, hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_F64G_NP(Y)                                                                                             \
  if (a.NP == Y) {                                                                                                 \
    if (out_partial) return hm ? qce_f64g_launch_t<MP, Y, true, true>(a, st) : qce_f64g_launch_t<MP, Y, false, true>(a, st); \
    return hm ? qce_f64g_launch_t<MP, Y, true, false>(a, st) : qce_f64g_launch_t<MP, Y, false, false>(a, st);     \
  }
  QCE_F64G_NP(16) QCE_F64G_NP(32) QCE_F64G_NP(64)
#undef QCE_F64G_NP
  return hipErrorInvalidValue;
}
