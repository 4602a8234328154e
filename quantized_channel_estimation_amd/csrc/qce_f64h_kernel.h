// Fused 'all'-mode estimate kernel in FP64 with Gauss's three-product complex multiply (3M) for padded M = N = 128
// (cfg4: K=256, N=128) -- gmm_cplx_bussgang.py:220-228 with :331-332, :388-435, :632-656, every step complex128.
//
// The products are those of k_est_all_f64g (qce_f64g_kernel.h): per k-step of 4 complex columns
//   K1 = (Lr + Li) yr,  R' = (-2 Li) hs,  I' = (2 Lr) hd,   Re(L y) = K1 + R',  Im(L y) = K1 + I',
// y as (hs, hd) = ((yr + yi) / 2, (yi - yr) / 2), tables (Ls, Lm, Lp) packed at prepare.
//
// What changes at 128: a 16-sample group's y is 128 VGPRs per wave (32 k-steps of (hs, hd)) and the filter's three
// accumulator sets 192, so the state does not fit beside a second wave on the SIMD.  Here
//   * y lives in LDS (the tile's 64 samples: 128 KB, written once per tile) and each unit's B operands are read from
//     it two blocks ahead (one 16-byte read per k-step and lane, conflict-free);
//   * two waves (row halves h) share a 16-sample group, each holding half the output: GW output tiles 4h .. 4h + 3
//     (3 x 4 accumulator sets = 96 VGPRs);
//   * GL: 16-row tile T of the lower triangle takes 2T + 2 units (two k-steps each); half 0 takes tiles 7, 0, 5, 2
//     and half 1 tiles 6, 1, 4, 3 -- 36 units each, balanced with no padding.  The halves' quad forms meet through
//     LDS once per component ((h0 + h1), the same order in both waves: bit-identical lp, max, sum, weights).
// One workgroup = 8 waves (4 sample groups x 2 halves, two waves per SIMD) x 64 samples per tile, one per CU.  Per
// component and 16 samples 2 x (108 + 192) blocks of two MFMAs = 1200 MFMAs, the 4M wave-pair kernel's 1600 x 3/4.
//
// No LDS ring: each wave loads its half's table blocks straight into registers (buffer loads, 16 B per lane per
// block, E blocks ahead, continuing into the next component); the four waves of a half read the same blocks at
// about the same time (L1 hits), with no DMA, chunk barriers or ring bookkeeping.  Persistent grid with the
// stream-K tail of the other FP64 kernels; cut tiles leave FP64 partials for k_merge_f64 (64-sample tiles).
//
// Layout (k_pack_f64h): per component VB virtual blocks x 2 halves x 1 KB, virtual block v of half h at physical
// block 2 v + h.  Half h's stream: its four GL tiles in the order above (unit outer, block j; + the tile's mean block),
// then GW (unit outer, block j, local tile inner; + one bias block per local tile), padded to a multiple of E + 1.
// Block j of unit u holds the A operands of two MFMAs as in k_pack_f64g: j = 0: (Ls s0) (Lm s0); 1: (Lp s0) (Ls s1);
// 2: (Lm s1) (Lp s1), s0 = 2u, s1 = 2u + 1; lane (r, g) = row 16 T + r, column 4 s + g.
#pragma once
#include "qce_f64g_kernel.h"

// register prefetch distance of the table stream (blocks)
#ifndef QCE_F64H_E
#define QCE_F64H_E 4
#endif

namespace {

// GL tile i (0..3) of half h
constexpr __host__ __device__ int f64h_gl_tile(int h, int i) {
  return h == 0 ? (i == 0 ? 7 : i == 1 ? 0 : i == 2 ? 5 : 2) : (i == 0 ? 6 : i == 1 ? 1 : i == 2 ? 4 : 3);
}

// GL units per half: sum over its tiles of 2T + 2 (+ one mean unit per tile with means) -- 36 / 40 for both halves
constexpr __host__ __device__ int f64h_glu(int hmi) { return 36 + 4 * hmi; }

// unit p (0 .. f64h_glu - 1) of half h's GL stream
struct UnitH {
  int T, u;   // GL tile, unit of the tile (two k-steps 2u, 2u + 1)
  bool mean;  // the tile's mean unit (the -q0 column, against the constant y row of the LDS tile)
  bool last;  // the tile's last unit: fold its rows into the quad form after it
};
__host__ __device__ constexpr UnitH f64h_unit(int hmi, int h, int p) {
  for (int i = 0; i < 4; ++i) {
    const int T = f64h_gl_tile(h, i), n = 2 * T + 2 + hmi;
    if (p < n) return UnitH{T, p, hmi && p == n - 1, p == n - 1};
    p -= n;
  }
  return UnitH{0, 0, false, false};
}

// virtual blocks per half and component: 3 per GL unit, 192 GW (+ 4 bias with means), padded to a multiple of E + 1
// so the register ring's slot of block b is b mod (E + 1) in every component (the stream runs on across components)
constexpr __host__ __device__ int f64h_vb(int hmi) {
  return (3 * f64h_glu(hmi) + 192 + 4 * hmi + QCE_F64H_E) / (QCE_F64H_E + 1) * (QCE_F64H_E + 1);
}

QCE_DEV __amdgpu_buffer_rsrc_t f64h_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
QCE_DEV double2 f64h_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

template <int I>
using ICH = std::integral_constant<int, I>;

}  // namespace

template <bool HM, bool OUT_PARTIAL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_est_all_f64h(
    long long B, int M, int N, int K, int R, long long L, const double2* __restrict__ y, const char* __restrict__ pack,
    const double* __restrict__ cconst, double2* __restrict__ h, double* __restrict__ om, double* __restrict__ os,
    double* __restrict__ oa, double* __restrict__ pm, double* __restrict__ ps, double* __restrict__ pa,
    double* __restrict__ pk, const double* __restrict__ shift) {
  constexpr int HMI = HM ? 1 : 0;
  constexpr int TS = 64;                       // samples per tile: 4 groups of 16
  constexpr int KS = 32;                       // k-steps at padded M = 128
  constexpr int GLU = f64h_glu(HMI);           // GL units per half
  constexpr int GLV = 3 * GLU;                 // GL blocks per half
  constexpr int GWV = 192 + 4 * HMI;           // GW blocks per half
  constexpr int VB = f64h_vb(HMI);             // virtual blocks per half and component
  constexpr unsigned STRIDE = (unsigned)VB * 2048u;
  constexpr int E = QCE_F64H_E;
  constexpr int D = 2;                         // y operands read D blocks ahead of their unit
  constexpr double RESCALE = 32.0;             // lazy max: rescale only when lp exceeds m by this
  static_assert(E >= 1 && E < GLV && D < 3, "prefetch distances");
  static_assert((GLU + 16) % 2 == 0, "y-operand slots repeat per component");
  // the tile's y as (hs, hd), [group][k-step][lane]; rows KS, KS + 1: the mean unit's constant operands (hs = hd = 1
  // in lane group 0: R' += Lm, I' += Lp, K1 += Ls (hs - hd) = 0)
  __shared__ __attribute__((aligned(16))) double2 ylds[4][KS + 2][64];
  __shared__ double qx[2][8][64];  // the halves' quad-form partials, alternating by component parity
  __shared__ double etab[32];      // 2^(j/32) for exp_tab64

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = wave & 1, sg = wave >> 1;  // row half, sample group (wave-uniform)
  const int g = lane >> 4, col = lane & 15;
  if (threadIdx.x < 32) etab[threadIdx.x] = exp2((double)threadIdx.x / 32.0);  // visible after the first barrier
  if (hh == 0) {
    ylds[sg][KS][lane] = g == 0 ? make_double2(1.0, 1.0) : make_double2(0.0, 0.0);
    ylds[sg][KS + 1][lane] = make_double2(0.0, 0.0);
  }
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

  // the table stream: this wave's half of component k, virtual block v at byte v * 2048 (+ h KB, + 16 B per lane)
  const unsigned voff = (unsigned)(hh * 1024 + lane * 16);
  auto rsrc_of = [&](int k) { return f64h_rsrc(pack + (long long)k * STRIDE, STRIDE); };
  const double2* yl = &ylds[sg][0][lane];
  int par = 0;  // component parity of the quad-form exchange slot

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
    const long long sbase = t * TS + 16LL * sg;
    // ---- the tile's y into LDS: every wave is done with the previous tile's, then each wave of a group writes its
    // half of the k-steps (lane (g, col): sample col, column 4 s + g as (hs, hd)); rows past B and columns past M
    // are clamped (finite values meeting zero table entries / never written)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
      int gl = g, cl = col;
      asm volatile("" : "+v"(gl), "+v"(cl));
      long long sm = sbase + cl;
      sm = sm < B ? sm : B - 1;
      const double2* yr = y + sm * M;
      double2 t16[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cc = 4 * (16 * hh + i) + gl;
        t16[i] = yr[cc < M ? cc : M - 1];
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double a = t16[i].x, b = t16[i].y;
        ylds[sg][16 * hh + i][lane] = make_double2(0.5 * (a + b), 0.5 * (b - a));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    f64x4 ok[4], orr[4], oi[4];
#pragma unroll
    for (int T = 0; T < 4; ++T) ok[T] = orr[T] = oi[T] = f64x4{0.0, 0.0, 0.0, 0.0};
    double m = QCE_NEG_INF, ssum = 0.0;

    // first E table blocks and the first unit's y operands (k-steps 0, 1 in both halves) of the first component
    __amdgpu_buffer_rsrc_t rs = rsrc_of(klo);
    double2 buf[E + 1];
#pragma unroll
    for (int i = 0; i < E; ++i) buf[i] = f64h_ld(rs, voff, (unsigned)i * 2048u);
    double2 yv[2][2];  // [unit parity][k-step of the unit]: (hs, hd)
    yv[0][0] = yl[0];
    yv[0][1] = yl[64];
    yv[1][0] = yv[1][1] = make_double2(0.0, 0.0);

#pragma unroll 1
    for (int k = klo; k < khi; ++k) {
      const double ck = cconst[k];
      // the stream continues into the next component of the segment (or re-reads this one: never consumed)
      const __amdgpu_buffer_rsrc_t rn = rsrc_of(k + 1 < khi ? k + 1 : k);
      double neg1 = -1.0;  // yr = hs - hd formed per use (fma with an opaque -1)
      asm volatile("" : "+v"(neg1));
      f64x4 k1 = f64x4{0.0, 0.0, 0.0, 0.0}, rr = k1, ii = k1;
      double qp = 0.0, p = 0.0;
      double pr0 = 0.0, ps0 = 0.0, pd0 = 0.0, pr1 = 0.0, ps1 = 0.0, pd1 = 0.0;
      // One instruction stream for both halves: every GL unit is three blocks with the same accumulator pattern, so
      // the halves differ only in data -- the table blocks, the k-steps their y operands are read from (a wave-uniform
      // select of two constants) and where a tile's rows are folded (a wave-uniform select of the fold's result).
      static_for(
          [&](auto vc) {
            constexpr int v = decltype(vc)::value;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (v + E < VB) {
              if constexpr (v + E < GLV + GWV)  // padding blocks are not loaded (no MFMA reads them)
                buf[(v + E) % (E + 1)] = f64h_ld(rs, voff, (unsigned)(v + E) * 2048u);
            } else {
              buf[(v + E) % (E + 1)] = f64h_ld(rn, voff, (unsigned)(v + E - VB) * 2048u);
            }
            const double2 a = buf[v % (E + 1)];
            if constexpr (v < GLV) {  // GL unit U, block j
              constexpr int U = v / 3, j = v % 3;
              const double2 y0 = yv[U & 1][0], y1 = yv[U & 1][1];
              if constexpr (j == 0) {
                k1 = mfma16x16x4d(a.x, fma(y0.y, neg1, y0.x), k1);
                rr = mfma16x16x4d(a.y, y0.x, rr);
              } else if constexpr (j == 1) {
                ii = mfma16x16x4d(a.x, y0.y, ii);
                k1 = mfma16x16x4d(a.y, fma(y1.y, neg1, y1.x), k1);
              } else {
                rr = mfma16x16x4d(a.x, y1.x, rr);
                ii = mfma16x16x4d(a.y, y1.y, ii);
                constexpr bool f0 = f64h_unit(HMI, 0, U).last, f1 = f64h_unit(HMI, 1, U).last;
                if constexpr (f0 || f1) {  // the end of a tile of one or both halves: |z|^2 of its rows
                  double qn = qp;
#pragma unroll
                  for (int i = 0; i < 4; ++i) {
                    const double zr = k1[i] + rr[i], zi = k1[i] + ii[i];
                    qn = fma(zr, zr, qn);
                    qn = fma(zi, zi, qn);
                  }
                  if constexpr (f0 && f1) {
                    qp = qn;
                    k1 = rr = ii = f64x4{0.0, 0.0, 0.0, 0.0};
                  } else {
                    const bool fold = hh == 0 ? f0 : f1;  // wave-uniform
                    qp = fold ? qn : qp;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                      k1[i] = fold ? 0.0 : k1[i];
                      rr[i] = fold ? 0.0 : rr[i];
                      ii[i] = fold ? 0.0 : ii[i];
                    }
                  }
                  asm volatile("" : "+v"(qp));
                }
              }
            } else {
              constexpr int r = v - GLV;
              if constexpr (r < 192) {  // GW data, unit u, block j, local tile T: B operands formed once per unit
                constexpr int u = r / 12, j = (r % 12) / 4, T = (r % 12) % 4, sl = u & 1;
                if constexpr (T == 0 && j == 0) {
                  ps0 = p * yv[sl][0].x;
                  pd0 = p * yv[sl][0].y;
                  pr0 = ps0 - pd0;
                } else if constexpr (T == 0 && j == 1) {
                  ps1 = p * yv[sl][1].x;
                  pd1 = p * yv[sl][1].y;
                  pr1 = ps1 - pd1;
                }
                if constexpr (j == 0) {
                  ok[T] = mfma16x16x4d(a.x, pr0, ok[T]);
                  orr[T] = mfma16x16x4d(a.y, ps0, orr[T]);
                } else if constexpr (j == 1) {
                  oi[T] = mfma16x16x4d(a.x, pd0, oi[T]);
                  ok[T] = mfma16x16x4d(a.y, pr1, ok[T]);
                } else {
                  orr[T] = mfma16x16x4d(a.x, ps1, orr[T]);
                  oi[T] = mfma16x16x4d(a.y, pd1, oi[T]);
                }
              } else if constexpr (HM && r < 196) {  // GW bias column (b): B = p in lane group 0
                constexpr int T = r - 192;
                const double pone = g == 0 ? p : 0.0;
                orr[T] = mfma16x16x4d(a.x, pone, orr[T]);
                oi[T] = mfma16x16x4d(a.y, pone, oi[T]);
              }
            }
            // y operands of the unit starting D blocks ahead, into its parity slot (the slot in use is the other one)
            constexpr int vn = v + D;
            if constexpr (vn < GLV && vn % 3 == 0) {
              constexpr int Un = vn / 3;
              constexpr UnitH n0 = f64h_unit(HMI, 0, Un), n1 = f64h_unit(HMI, 1, Un);
              constexpr int s0 = n0.mean ? KS : 2 * n0.u, s1 = n1.mean ? KS : 2 * n1.u;
              int su = hh == 0 ? s0 : s1;
              asm volatile("" : "+s"(su));  // laundered: no read is CSE'd across units (register pressure)
              yv[Un & 1][0] = yl[su * 64];
              yv[Un & 1][1] = yl[su * 64 + 64];
            } else if constexpr (vn >= GLV && vn < GLV + 192 && (vn - GLV) % 12 == 0) {
              constexpr int un = (vn - GLV) / 12;
              int su = 2 * un;
              asm volatile("" : "+s"(su));
              yv[un & 1][0] = yl[su * 64];
              yv[un & 1][1] = yl[su * 64 + 64];
            } else if constexpr (vn == VB) {  // the next component's first unit
              yv[0][0] = yl[0];
              yv[0][1] = yl[64];
            }
            // after the last GL block: the halves' quad forms meet, then the online softmax (FP64), identical in
            // both waves of the group
            if constexpr (v == GLV - 1) {
              qx[par][wave][lane] = qp;
              asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
              const double tot = qx[par][2 * sg][lane] + qx[par][2 * sg + 1][lane];
              par ^= 1;
              const double lp = ck - sum_groups(tot);
              if (__builtin_amdgcn_ballot_w64(lp > m + RESCALE) != 0ull) {  // rare: new running maximum
                const bool up = lp > m + RESCALE;
                const double mn = up ? lp : m;
                const double al = up ? (m == QCE_NEG_INF ? 0.0 : exp(m - mn)) : 1.0;
                ssum *= al;
                m = mn;
#pragma unroll
                for (int T = 0; T < 4; ++T) {
                  ok[T] *= al;
                  orr[T] *= al;
                  oi[T] *= al;
                }
              }
              p = (lp == QCE_NEG_INF) ? 0.0 : exp_tab64(lp - m, etab);
              ssum += p;
            }
          },
          std::make_integer_sequence<int, VB>{});
      rs = rn;
    }

    // ---- write the tile: this half's output rows 16 (4h + T) + g + 4 i of sample col ----
    {
      int gw = g;
      asm volatile("" : "+v"(gw));
      const int ls = 16 * sg + col;
      const long long sample = t * TS + ls;
      if (sample < B) {
        const bool whole = (klo == 0 && khi == K);
        const bool pfmt = OUT_PARTIAL || !whole;
        const long long row = whole ? sample : (w * 2 + (t == t_first ? 0 : 1)) * TS + ls;
        if (OUT_PARTIAL && whole && pk) {  // shifted packed partial: [s e^{m-M*}, 0, acc e^{m-M*}] (K-shard sum)
          const double sc = (m == QCE_NEG_INF) ? 0.0 : exp(m - *shift);
          double* dp = pk + sample * (2LL * N + 2);
          if (g == 0 && hh == 0) *reinterpret_cast<double2*>(dp) = make_double2(ssum * sc, 0.0);
#pragma unroll
          for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * (4 * hh + T) + gw + 4 * i;
              if (n < N)
                *reinterpret_cast<double2*>(dp + 2 + 2 * n) =
                    make_double2((ok[T][i] + orr[T][i]) * sc, (ok[T][i] + oi[T][i]) * sc);
            }
        } else if (pfmt) {
          double* dm = whole ? om : pm;
          double* ds = whole ? os : ps;
          double* da = (whole ? oa : pa) + row * (2LL * N);
          if (g == 0 && hh == 0) {
            dm[row] = m;
            ds[row] = ssum;
          }
#pragma unroll
          for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * (4 * hh + T) + gw + 4 * i;
              if (n < N)
                *reinterpret_cast<double2*>(da + 2 * n) = make_double2(ok[T][i] + orr[T][i], ok[T][i] + oi[T][i]);
            }
        } else {
          const double inv = 1.0 / ssum;
          double2* hp = h + sample * N;
#pragma unroll
          for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = 16 * (4 * hh + T) + gw + 4 * i;
              if (n < N) hp[n] = make_double2((ok[T][i] + orr[T][i]) * inv, (ok[T][i] + oi[T][i]) * inv);
            }
        }
      }
    }
  }
}

// 3M tables of k_est_all_f64h: one 64-lane group per (physical block, component), physical block 2 v + h
__global__ __launch_bounds__(64) void k_pack_f64h(int M, int N, int has_mean, const double2* __restrict__ Linv,
                                                  const double2* __restrict__ W, const double2* __restrict__ q0,
                                                  const double2* __restrict__ bvec, double* __restrict__ pack) {
  const int pb = blockIdx.x, k = blockIdx.y, lane = threadIdx.x;
  const int v = pb >> 1, hf = pb & 1, hmi = has_mean ? 1 : 0;
  const int VB = f64h_vb(hmi), GLV = 3 * f64h_glu(hmi);
  const int r = lane & 15, gk = lane >> 4;
  double val[2] = {0.0, 0.0};
  // block j of a unit: the A operands of its two MFMAs, which = 0 Ls, 1 Lm, 2 Lp of k-step 2u (+ 1)
  const int wh[3][2] = {{0, 1}, {2, 0}, {1, 2}};
  auto entry = [&](const double2 z, int which) {
    return which == 0 ? z.x + z.y : (which == 1 ? -2.0 * z.y : 2.0 * z.x);
  };
  if (v < GLV) {
    const int U = v / 3, j = v % 3;
    const UnitH un = f64h_unit(hmi, hf, U);
    const int i = 16 * un.T + r;
    if (un.mean) {  // against y = (hs, hd) = (1, 1) in lane group 0: R' += -Re q0 (j 0), I' += -Im q0 (j 1)
      if (gk == 0 && i < M) {
        const double2 z = q0[(long long)k * M + i];
        if (j == 0) val[1] = -z.x;
        if (j == 1) val[0] = -z.y;
      }
    } else {
      const int s0 = 2 * un.u, ks[3][2] = {{s0, s0}, {s0, s0 + 1}, {s0 + 1, s0 + 1}};
      for (int e = 0; e < 2; ++e) {
        const int jj = 4 * ks[j][e] + gk;
        if (i < M && jj < M) val[e] = entry(Linv[((long long)k * M + i) * M + jj], wh[j][e]);
      }
    }
  } else if (v < GLV + 192) {
    const int rr = v - GLV, u = rr / 12, j = (rr % 12) / 4, T = (rr % 12) % 4;
    const int i = 16 * (4 * hf + T) + r;
    const int s0 = 2 * u, ks[3][2] = {{s0, s0}, {s0, s0 + 1}, {s0 + 1, s0 + 1}};
    for (int e = 0; e < 2; ++e) {
      const int jj = 4 * ks[j][e] + gk;
      if (i < N && jj < M) val[e] = entry(W[((long long)k * N + i) * M + jj], wh[j][e]);
    }
  } else if (hmi && v < GLV + 196) {
    const int i = 16 * (4 * hf + (v - GLV - 192)) + r;
    if (gk == 0 && i < N) {
      const double2 z = bvec[(long long)k * N + i];
      val[0] = z.x;
      val[1] = z.y;
    }
  }
  *reinterpret_cast<double2*>(pack + (((long long)k * VB * 2 + pb) * 64 + lane) * 2) = make_double2(val[0], val[1]);
}
