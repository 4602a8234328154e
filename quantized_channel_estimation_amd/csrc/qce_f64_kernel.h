// Fused 'all'-mode estimate kernel in FP64 on v_mfma_f64_16x16x4_f64 (gfx950 / CDNA4) — the
// reference-precision path of estimate_from_y (gmm_cplx_bussgang.py:220-228 with :331-332,
// :388-435, :632-656; every reference step is complex128).
//
//   lp_bk = c_k - || E(Linv_k) [y_b; 1] ||^2          (the -q0 column folds the mean in)
//   h_b   = sum_k e^{lp_bk - m_b} E(W_k) [y_b; 1] / sum_k e^{lp_bk - m_b}
//
// E(.) is the real 2x2-block embedding of a complex matrix; every product is an FP64 MFMA with
// FP64 accumulation, the softmax is FP64 (libm exp), so the result is an FP64 computation of the
// reference's formula (only the summation order differs).
//
// Layout (prepare: k_pack_f64all).  The k (reduction) order is permuted so that one 16-byte load
// of y gives a lane both B-operand values of a "k-pair": k-step 2s+e, lane group g = lane>>4
// holds part e of complex column 4s+g.  Output rows are permuted so that a lane's four
// accumulator registers are (re, im) of complex rows 8T+g and 8T+4+g: row rho of row tile T is
// complex 8T + 4(rho>>3) + (rho&3), part (rho>>2)&1.  A table "block" is 1 KB: the A operands of
// one row tile for the two k-steps of a k-pair, lane-major (lane l: 16 B = both k-steps), read
// with one conflict-free ds_read_b128.
//   component k: GL blocks (row tile T outer; k-pairs 0..2T+1 — the upper triangle of Linv is
//   skipped; + one mean block with the -q0 column), then GW blocks (k-pair outer, row tile inner,
//   + one mean block per row tile with the b column), padded to whole ring chunks.
//
// Scheduling: one workgroup = NW waves x 16*CT samples (CT column tiles per wave; samples on the
// MFMA column axis, so quad form, running max, sum and weights are per-lane registers and the
// y fragments stay in VGPRs for the whole component loop).  The component tables stream through
// an LDS ring of NSLOT chunks of 16 KB (global_load_lds, 16 B per lane); one barrier per chunk,
// executed E blocks before the chunk is needed so the LDS reads of its first blocks are not held
// up.  Persistent grid: R rounds of whole tiles per workgroup, then the remaining tiles' (tile,
// component) items dealt out L per workgroup (stream-K); a tile cut between workgroups leaves
// FP64 partials (m, s, acc) that k_merge_f64 combines — the same format as the K-shard path.
#pragma once
#include "qce_common.h"
#include "qce_kernels.h"
#include "qce_h2_common.h"

#include <utility>

// LDS operand prefetch distance of the block loop (blocks ahead; the compiler keeps E - 1 reads in flight past each
// wait).  Metric config, one box (profiles/r04_f64_prefetch_ab.txt, builtin DMA): E = 2 frac 0.843, 3 0.847, 4 0.850,
// 5 0.852, 6 0.854-0.859, 8 0.851, 10 0.844, 12 0.850.  With the inline-asm DMA (profiles/r04_f64_prefetch_ab2.txt):
// E = 4 / 6 / 8: metric 0.883-0.884 / 0.885 / 0.886-0.889, cfg4 0.842 / 0.843 / 0.847.  A/B builds:
// python -m quantized_channel_estimation_amd.build --variant eN --define QCE_F64_E=N (QCE_LIB selects the library).
#ifndef QCE_F64_E
#define QCE_F64_E 8
#endif
// 1: drain the LDS prefetches before every ring barrier (the round-3 form, kept for A/B builds)
#ifndef QCE_F64_BND_DRAIN
#define QCE_F64_BND_DRAIN 0
#endif

namespace {

// Ring geometry: chunks of CB blocks (1 KB each), NSLOT chunks of LDS.  One barrier per chunk, so CB is as large
// as the LDS allows (NSLOT >= 3, <= 144 KB) unless the per-component padding to whole chunks costs more load
// traffic than the barriers it saves; CB is a multiple of 8 (whole pieces per wave for 4 and 8 waves).
constexpr __host__ __device__ int f64_blocks(int MP, int NP, int hmi) {
  return (MP / 8) * (MP / 8 + 1) + hmi * (MP / 8) + (NP / 8) * (MP / 4 + hmi);
}
// minlead: blocks of prefetch lead the ring must keep ((NSLOT - 2) chunks are in flight while one is read).  Tried in
// round 4 for the one-wave-per-SIMD shapes (padded 128): >= 96 blocks (CB 24, 6 slots) made cfg4 slower (frac 0.676
// vs 0.714, profiles/r04_cfg4_deeper_ring.txt: the doubled barrier count costs more than the longer lead saves), so
// every shape keeps the cheapest layout (minlead 0).
constexpr __host__ __device__ int f64_minlead(int, int) { return 0; }
constexpr __host__ __device__ int f64_nslot(int cb) { return 144 / cb < 8 ? 144 / cb : 8; }
// Row-split wave pairs (PR = 2) for the shapes whose state fills a SIMD with one wave (padded 128 x 128): two waves
// share 16 samples; wave half h takes the GL row tiles 2j + h -- virtual tile j runs 4j + 4 k-pairs, half 0's last
// two are zero blocks -- and the GW row tiles 2t + h, so each wave holds half the accumulators and two waves fit a
// SIMD.  A virtual block is PR physical 1 KB blocks (half h at +h KB); both halves run the same instruction stream.
constexpr __host__ __device__ int f64_pr(int MP, int NP) { return (MP == 128 && NP == 128) ? 2 : 1; }
constexpr __host__ __device__ int f64_vblocks(int MP, int NP, int hmi) {
  if (f64_pr(MP, NP) == 1) return f64_blocks(MP, NP, hmi);
  const int J = MP / 16;  // virtual GL tiles
  return 2 * J * (J - 1) + (4 + hmi) * J + (NP / 16) * (MP / 4 + hmi);
}
// chunk of cb virtual blocks (cb * pr physical, a multiple of 8 between 16 and 48)
constexpr __host__ __device__ int f64_cb(int n, int minlead = 0, int pr = 1) {
  int best = 16 / pr;
  double best_cost = 1e30;
  for (int cbp = 16; cbp <= 48; cbp += 8) {
    const int cb = cbp / pr;
    if ((f64_nslot(cbp) - 2) * cb < minlead) continue;
    const int pad = (n + cb - 1) / cb * cb - n;
    const double cost = (double)pad / n + 2.0 / cb;
    if (cost < best_cost - 1e-12) {
      best_cost = cost;
      best = cb;
    }
  }
  return best;
}
constexpr __host__ __device__ int f64_bpc(int n, int minlead = 0, int pr = 1) {
  return (n + f64_cb(n, minlead, pr) - 1) / f64_cb(n, minlead, pr) * f64_cb(n, minlead, pr);
}
// physical 1 KB blocks per component of the pack
constexpr __host__ __device__ int f64_pack_blocks(int MP, int NP, int hmi) {
  return f64_bpc(f64_vblocks(MP, NP, hmi), f64_minlead(MP, NP), f64_pr(MP, NP)) * f64_pr(MP, NP);
}

template <int MP, int NP, bool HM>
struct F64G {
  static constexpr int PR = f64_pr(MP, NP);
  static constexpr int NTL = MP / 8;  // GL row tiles (16 real rows = 8 complex rows)
  static constexpr int NTW = NP / 8;  // GW row tiles
  static constexpr int NTLV = NTL / PR, NTWV = NTW / PR;  // per wave (virtual tiles)
  static constexpr int KP = MP / 4;   // k-pairs (4 complex columns)
  static constexpr int HMI = HM ? 1 : 0;
  // k-pairs of GL (virtual) tile T and its first block
  static constexpr __host__ __device__ int gl_len(int T) { return PR == 1 ? 2 * T + 2 : 4 * T + 4; }
  static constexpr __host__ __device__ int gl_off(int T) {
    return PR == 1 ? T * (T + 1) + HMI * T : 2 * T * (T - 1) + (4 + HMI) * T;
  }
  static constexpr int GL_BLOCKS = gl_off(NTLV);
  static constexpr int GW_BLOCKS = NTWV * (KP + HMI);
  static constexpr int BLOCKS = GL_BLOCKS + GW_BLOCKS;
  static constexpr int CB = f64_cb(BLOCKS, f64_minlead(MP, NP), PR);  // virtual blocks per ring chunk
  static constexpr int CBP = CB * PR;                                  // physical blocks per ring chunk
  static constexpr int NSLOT = f64_nslot(CBP);
  static constexpr int CHUNK = CBP * 1024;
  static constexpr int BPC = f64_bpc(BLOCKS, f64_minlead(MP, NP), PR);
  static constexpr int CPC = BPC / CB;
  static_assert(BLOCKS == f64_vblocks(MP, NP, HMI), "block count");
};

struct BlockInfo {
  int kind, T, s;
};
// (virtual) block b of a component -> kind (0 GL data, 1 GL mean, 2 GW data, 3 GW mean, 4 pad), (virtual) tile T,
// k-pair s
template <int MP, int NP, bool HM>
constexpr __host__ __device__ BlockInfo block_info(int b) {
  using G = F64G<MP, NP, HM>;
  if (b < G::GL_BLOCKS) {
    int T = 0;
    while (b >= G::gl_off(T + 1)) ++T;
    const int s = b - G::gl_off(T);
    return BlockInfo{s < G::gl_len(T) ? 0 : 1, T, s};
  }
  const int r = b - G::GL_BLOCKS;
  if (r < G::KP * G::NTWV) return BlockInfo{2, r % G::NTWV, r / G::NTWV};
  if (r < (G::KP + G::HMI) * G::NTWV) return BlockInfo{3, r - G::KP * G::NTWV, G::KP};
  return BlockInfo{4, 0, 0};
}

// Diagnostic build only (-DQCE_STAMPS): per-wave cycle sums of the kernel's segments (s_memtime), stored
// by lane 0 into a buffer of their own (qce_debug_f64_stamps); the product kernel executes no stamp.
#ifdef QCE_STAMPS
#define F64_STAMP_DECL unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = __builtin_amdgcn_s_memtime();
#define F64_STAMP(i)                                     \
  do {                                                   \
    __builtin_amdgcn_sched_barrier(0);                   \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    st_acc[(i)] += t_ - st_prev;                         \
    st_prev = t_;                                        \
    __builtin_amdgcn_sched_barrier(0);                   \
  } while (0)
#define F64_STAMP_FLUSH                                                                    \
  if (stamps && lane == 0)                                                                 \
    for (int i_ = 0; i_ < 8; ++i_) stamps[((long long)blockIdx.x * NW + wave) * 8 + i_] = st_acc[i_];
#else
#define F64_STAMP_DECL
#define F64_STAMP(i)
#define F64_STAMP_FLUSH
#endif

template <int N_>
QCE_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N_) : "memory");
}

// Sum over the four 16-lane groups (all lanes get the total), (g0 + g1) + (g2 + g3) in every lane.  gfx950's
// v_permlane16/32_swap exchange rows in the VALU: the softmax's critical path (last GL MFMA -> lp -> exp -> first GW
// MFMA) no longer waits on two ds_bpermute round trips through the LDS.
QCE_DEV double swap_sum(double q, bool r32) {
  const int lo = __double2loint(q), hi = __double2hiint(q);
  double a, b;
  if (r32) {
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = __hiloint2double(ph[0], pl[0]);
    b = __hiloint2double(ph[1], pl[1]);
  } else {
    const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = __hiloint2double(ph[0], pl[0]);
    b = __hiloint2double(ph[1], pl[1]);
  }
  return a + b;  // the lower row's value first in both lanes of the pair
}
QCE_DEV double sum_groups(double q) { return swap_sum(swap_sum(q, false), true); }

// Source cursor of the ring: which component chunk a workgroup streams next.  Items are the
// workgroup's (tile, component) work in order: R*K full-round items (components 0..K-1 per tile),
// then the tail items item0 .. item0+ntail-1 (component = item % K).
struct RingCursor {
  int item, nitems, rk, comp_tail, comp, cc, K, cpc;
  QCE_DEV void init(int rk_, int comp_tail_, int ntail, int K_, int cpc_) {
    rk = rk_;
    comp_tail = comp_tail_;
    nitems = rk_ + ntail;
    K = K_;
    cpc = cpc_;
    item = 0;
    cc = 0;
    comp = rk_ > 0 ? 0 : comp_tail_;
  }
  QCE_DEV long long chunk_index() const { return (long long)(comp * cpc + cc); }
  QCE_DEV void advance() {
    if (item >= nitems) return;
    if (++cc < cpc) return;
    cc = 0;
    ++item;
    if (item >= nitems) {  // past the end: keep re-loading the last chunk (dummy, never read)
      item = nitems;
      cc = cpc - 1;
      return;
    }
    if (item == rk) comp = comp_tail;
    else comp = (comp + 1 == K) ? 0 : comp + 1;
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// fused kernel
// ---------------------------------------------------------------------------
template <int MP, int NP, bool HM, int CT, int NW, bool OUT_PARTIAL>
__global__ __launch_bounds__(NW * 64) void k_est_all_f64(long long B, int M, int N, int K, int R, long long L,
                                                         const double2* __restrict__ y, const char* __restrict__ pack,
                                                         const double* __restrict__ cconst, double2* __restrict__ h,
                                                         double* __restrict__ om, double* __restrict__ os,
                                                         double* __restrict__ oa, double* __restrict__ pm,
                                                         double* __restrict__ ps, double* __restrict__ pa,
                                                         double* __restrict__ pk, const double* __restrict__ shift,
                                                         unsigned long long* __restrict__ stamps) {
  using G = F64G<MP, NP, HM>;
  constexpr int PR = G::PR;                   // waves per sample group (row-split pairs: 2)
  constexpr int TS = NW / PR * 16 * CT;       // samples per tile
  constexpr int LPW = G::CBP / NW;            // global_load_lds per wave per chunk
  constexpr int E = PR == 2 ? 4 : QCE_F64_E;  // boundary lead (blocks) = LDS prefetch distance (pairs: registers)
  constexpr double RESCALE = 32.0;            // lazy max: rescale only when lp exceeds m by this
  static_assert(G::CBP % NW == 0 && NW % PR == 0, "chunk split");
  static_assert(PR == 1 || CT == 1, "row-split pairs hold one column tile");
  __shared__ __attribute__((aligned(16))) char lds[G::NSLOT * G::CHUNK];
  __shared__ double qx[PR == 2 ? NW * 64 : 1];  // pairs: the halves' quad forms

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = wave % PR, sgrp = wave / PR;  // row half, sample group (wave-uniform)
  const int g = lane >> 4, col = lane & 15;
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
  // ---- ring ----
  RingCursor cur;
  cur.init(R * K, (int)(item0 % K), (int)ntail, K, G::CPC);
  int issued = 0;  // chunks issued so far (stream index of the next one)
  // A chunk refill is LPW global_load_lds pieces of 1 KB per wave.  refill_begin fixes the chunk's source and
  // slot; the pieces go out one per MFMA gap of the block that follows the barrier (an LDS-DMA issue among
  // bare MFMAs costs ~60 cycles — issued back to back after the barrier they left the MFMA pipe idle).
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
  // boundary for stream chunk jn: its loads landed everywhere, and every wave is done with chunk jn - 2,
  // whose slot is refilled (refill_begin + pieces) with chunk jn + NSLOT - 2
  // No LDS-read drain before the barrier: the slot refilled after it (chunk jn - 2) was last read by blocks this
  // wave has already consumed (E < CB), so the E - 1 prefetches in flight (all in chunk jn - 1) may cross it.
  static_assert(E < G::CB, "the prefetch window must stay inside one chunk");
  auto boundary_wait = [&]() {
    wait_vmcnt<(G::NSLOT - 3) * LPW>();
#if QCE_F64_BND_DRAIN
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    F64_STAMP(3);
  };
#pragma unroll 1
  for (int j = 0; j < G::NSLOT - 2; ++j) {
    refill_begin();
    refill_pieces(0, LPW);
  }
  boundary_wait();  // chunk 0
  refill_begin();
  refill_pieces(0, LPW);
  int cstream = 0;  // stream index of the current component's chunk 0

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
    const long long sbase = t * TS + (long long)sgrp * 16 * CT;
    // y fragments: k-pair s, lane group g -> complex column 4s + g (re: k-step 2s, im: 2s+1).  Rows past B
    // and columns past M are clamped (finite values of the same tensor) instead of masked: a padded column
    // meets zero table entries, an invalid sample is never written.  The laundered lane constants keep the
    // per-column offsets inside the loop (hoisted, they would pin a register each for the whole kernel).
    double2 yv[CT][G::KP];
    int gl = g, cl = col;
    asm volatile("" : "+v"(gl), "+v"(cl));
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      long long sm = sbase + 16 * c + cl;
      sm = sm < B ? sm : B - 1;
      const double2* yr = y + sm * M;
#pragma unroll
      for (int s = 0; s < G::KP; ++s) {
        const int cc = 4 * s + gl;
        yv[c][s] = yr[cc < M ? cc : M - 1];
      }
    }
    wait_vmcnt<0>();
    F64_STAMP(5);
    f64x4 out[G::NTWV][CT];
#pragma unroll
    for (int T = 0; T < G::NTWV; ++T)
#pragma unroll
      for (int c = 0; c < CT; ++c) out[T][c] = f64x4{0.0, 0.0, 0.0, 0.0};
    double m[CT], ssum[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      m[c] = QCE_NEG_INF;
      ssum[c] = 0.0;
    }

#pragma unroll 1
    for (int k = klo; k < khi; ++k) {
      const double ck = cconst[k];
      const int slot0 = cstream % G::NSLOT;
      // LDS offset of this lane's 16 B in the slot of the chunk being read; advanced when the reads cross
      // into the next chunk and laundered, so the compiler keeps one live offset instead of hoisting one
      // per chunk of the unrolled component
      int rslot = slot0;
      int roff = lane * 16 + hh * 1024 + rslot * G::CHUNK;
      auto rd = [&](int off) -> double2 { return *reinterpret_cast<const double2*>(&lds[roff + off]); };
      f64x4 acc[CT], accp[CT];
      double qp[CT], p[CT];
      double bs0[CT], bs1[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        qp[c] = 0.0;
        p[c] = 0.0;
        bs0[c] = bs1[c] = 0.0;
        acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
        accp[c] = acc[c];
      }
      auto fold = [&](f64x4 (&x)[CT]) {
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          qp[c] = fma(x[c][0], x[c][0], qp[c]);
          qp[c] = fma(x[c][1], x[c][1], qp[c]);
          qp[c] = fma(x[c][2], x[c][2], qp[c]);
          qp[c] = fma(x[c][3], x[c][3], qp[c]);
          // pin the fold here: sunk to the softmax, every row tile would keep its own accumulators
          asm volatile("" : "+v"(qp[c]));
        }
      };
      double2 buf[E + 1];
#pragma unroll
      for (int i = 0; i < E; ++i) buf[i] = rd(i * PR * 1024);
      static_for(
          [&](auto bc) {
            constexpr int b = decltype(bc)::value;
            constexpr BlockInfo bi = block_info<MP, NP, HM>(b);
            __builtin_amdgcn_sched_barrier(0);  // keep the explicit prefetch distance (no LDS read hoisting)
            // next chunk's boundary E blocks early (the last one is the next component's chunk 0)
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
                roff = lane * 16 + hh * 1024 + rslot * G::CHUNK;
                asm volatile("" : "+v"(roff));
              }
              buf[r % (E + 1)] = rd((r % G::CB) * PR * 1024);
            }
            const double2 a = buf[b % (E + 1)];
            // MFMAs of this block; on a boundary step the refill pieces are spread over their gaps
            constexpr int NMF = (bi.kind == 0 || bi.kind == 2) ? 2 * CT : (bi.kind == 4 ? 0 : CT);
            int jm = 0;
            auto gap = [&]() {
              if constexpr (RB && NMF > 0) {
                __builtin_amdgcn_sched_barrier(0);
                refill_pieces(jm * LPW / NMF, (jm + 1) * LPW / NMF);
                __builtin_amdgcn_sched_barrier(0);
              }
              ++jm;
            };
            if constexpr (bi.kind == 0) {  // GL data: u += E(Linv) y over k-pair s
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c] = mfma16x16x4d(a.x, yv[c][bi.s].x, acc[c]);
                gap();
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c] = mfma16x16x4d(a.y, yv[c][bi.s].y, acc[c]);
                gap();
              }
            } else if constexpr (bi.kind == 1) {  // GL mean column (-q0): B = 1 in lane group 0
              const double one = g == 0 ? 1.0 : 0.0;
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c] = mfma16x16x4d(a.x, one, acc[c]);
                gap();
              }
            } else if constexpr (bi.kind == 2) {  // GW data: out += E(W) (p y) over k-pair s
              if constexpr (bi.T == 0) {
#pragma unroll
                for (int c = 0; c < CT; ++c) {
                  bs0[c] = yv[c][bi.s].x * p[c];
                  bs1[c] = yv[c][bi.s].y * p[c];
                }
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                out[bi.T][c] = mfma16x16x4d(a.x, bs0[c], out[bi.T][c]);
                gap();
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                out[bi.T][c] = mfma16x16x4d(a.y, bs1[c], out[bi.T][c]);
                gap();
              }
            } else if constexpr (bi.kind == 3) {  // GW mean column (b): B = p in lane group 0
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                out[bi.T][c] = mfma16x16x4d(a.x, g == 0 ? p[c] : 0.0, out[bi.T][c]);
                gap();
              }
            }
            if constexpr (RB && NMF == 0) refill_pieces(0, LPW);
            // GL row tiles: the squares of tile T are folded into the quad form one block later (after the
            // first MFMAs of tile T+1 are issued, so the fold does not wait on tile T's last MFMA); the last
            // tile folds at once, the softmax needs it
            if constexpr (bi.kind == 0 || bi.kind == 1) {
              constexpr bool first = bi.kind == 0 && bi.s == 0;
              if constexpr (first && bi.T > 0 && PR == 1) fold(accp);
              constexpr bool last = HM ? (bi.kind == 1) : (bi.s == G::gl_len(bi.T) - 1);
              if constexpr (last) {
                if constexpr (bi.T == G::NTLV - 1 || PR == 2) {  // pairs: the partner wave covers the wait
                  fold(acc);
                } else {
#pragma unroll
                  for (int c = 0; c < CT; ++c) accp[c] = acc[c];
                }
#pragma unroll
                for (int c = 0; c < CT; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
              }
            }
            // after the last GL block: log-probability and the online softmax (FP64)
            if constexpr (b == G::GL_BLOCKS - 1) {
              F64_STAMP(0);
              double lp[CT];
              bool need = false;
              if constexpr (PR == 2) {  // the pair's quad forms, (half 0 + half 1) in both waves
                qx[wave * 64 + lane] = qp[0];
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                const double other = qx[(wave ^ 1) * 64 + lane];
                qp[0] = hh == 0 ? qp[0] + other : other + qp[0];
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                lp[c] = ck - sum_groups(qp[c]);
                need = need || (lp[c] > m[c] + RESCALE);
              }
              if (__builtin_amdgcn_ballot_w64(need) != 0ull) {  // rare: new running maximum
#pragma unroll
                for (int c = 0; c < CT; ++c) {
                  const bool up = lp[c] > m[c] + RESCALE;
                  const double mn = up ? lp[c] : m[c];
                  const double al = up ? (m[c] == QCE_NEG_INF ? 0.0 : exp(m[c] - mn)) : 1.0;
                  ssum[c] *= al;
                  m[c] = mn;
#pragma unroll
                  for (int T = 0; T < G::NTWV; ++T) out[T][c] *= al;
                }
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                p[c] = (lp[c] == QCE_NEG_INF) ? 0.0 : exp(lp[c] - m[c]);
                ssum[c] += p[c];
              }
              F64_STAMP(1);
            }
          },
          std::make_integer_sequence<int, G::BPC>{});
      F64_STAMP(2);
      cstream += G::CPC;
    }

    // ---- write the tile ----
    int gw = g;
    asm volatile("" : "+v"(gw));
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int ls = sgrp * 16 * CT + 16 * c + col;
      const long long sample = t * TS + ls;
      if (sample >= B) continue;
      const bool whole = (klo == 0 && khi == K);
      const bool pfmt = OUT_PARTIAL || !whole;
      const long long row = whole ? sample : (w * 2 + (t == t_first ? 0 : 1)) * TS + ls;
      if (OUT_PARTIAL && whole && pk) {  // shifted packed partial: [s e^{m-M*}, 0, acc e^{m-M*}] (K-shard sum)
        const double sc = (m[c] == QCE_NEG_INF) ? 0.0 : exp(m[c] - *shift);
        double* dp = pk + sample * (2LL * N + 2);
        if (g == 0 && hh == 0) *reinterpret_cast<double2*>(dp) = make_double2(ssum[c] * sc, 0.0);
#pragma unroll
        for (int T = 0; T < G::NTWV; ++T) {
          const int i0 = 8 * (PR * T + hh) + gw, i1 = i0 + 4;
          if (i0 < N) *reinterpret_cast<double2*>(dp + 2 + 2 * i0) = make_double2(out[T][c][0] * sc, out[T][c][1] * sc);
          if (i1 < N) *reinterpret_cast<double2*>(dp + 2 + 2 * i1) = make_double2(out[T][c][2] * sc, out[T][c][3] * sc);
        }
      } else if (pfmt) {
        double* dm = whole ? om : pm;
        double* ds = whole ? os : ps;
        double* da = (whole ? oa : pa) + row * (2LL * N);
        if (g == 0 && hh == 0) {
          dm[row] = m[c];
          ds[row] = ssum[c];
        }
#pragma unroll
        for (int T = 0; T < G::NTWV; ++T) {
          const int i0 = 8 * (PR * T + hh) + gw, i1 = i0 + 4;
          if (i0 < N) *reinterpret_cast<double2*>(da + 2 * i0) = make_double2(out[T][c][0], out[T][c][1]);
          if (i1 < N) *reinterpret_cast<double2*>(da + 2 * i1) = make_double2(out[T][c][2], out[T][c][3]);
        }
      } else {
        const double inv = 1.0 / ssum[c];
        double2* hp = h + sample * N;
#pragma unroll
        for (int T = 0; T < G::NTWV; ++T) {
          const int i0 = 8 * (PR * T + hh) + gw, i1 = i0 + 4;
          if (i0 < N) hp[i0] = make_double2(out[T][c][0] * inv, out[T][c][1] * inv);
          if (i1 < N) hp[i1] = make_double2(out[T][c][2] * inv, out[T][c][3] * inv);
        }
      }
    }
  }
  F64_STAMP(5);
  F64_STAMP_FLUSH
  wait_vmcnt<0>();  // drain the (dummy) ring prefetches before the workgroup retires
}

// one launcher per padded observation dimension MP (instantiated in qce_f64_m<MP>.hip, compiled in
// parallel): CT = 2 column tiles per wave when MP, NP <= 64, else 1 (a 128-dim observation's y fragments,
// or a 128-row output accumulator, take the registers of two 64-dim ones)
constexpr int qce_f64_ct(int MP, int NP) { return (MP <= 64 && NP <= 64) ? 2 : 1; }

template <int MP, int NP, bool HM, bool OP>
hipError_t qce_f64_launch_t(const QceF64Args& a, hipStream_t st) {
  constexpr int CT0 = qce_f64_ct(MP, NP);
  if constexpr (CT0 == 2) {
    if (a.waves == 8) {  // two waves per SIMD, one column tile each (same tile of 128 samples)
      hipLaunchKernelGGL((k_est_all_f64<MP, NP, HM, 1, 8, OP>), dim3((unsigned)a.nwg), dim3(8 * 64), 0, st, a.B, a.M,
                         a.N, a.K, a.R, a.L, a.y, a.pack, a.cconst, a.h, a.om, a.os, a.oa, a.pm, a.ps, a.pa, a.pk,
                         a.shift, a.stamps);
      return hipGetLastError();
    }
  }
  constexpr int CT = CT0, NW = 4 * f64_pr(MP, NP);  // row-split pairs: 8 waves, two per SIMD
  hipLaunchKernelGGL((k_est_all_f64<MP, NP, HM, CT, NW, OP>), dim3((unsigned)a.nwg), dim3(NW * 64), 0, st, a.B, a.M,
                     a.N, a.K, a.R, a.L, a.y, a.pack, a.cconst, a.h, a.om, a.os, a.oa, a.pm, a.ps, a.pa, a.pk, a.shift,
                     a.stamps);
  return hipGetLastError();
}

template <int MP>
hipError_t qce_f64_launch_mp(const QceF64Args& a, bool out_partial, hipStream_t st) {
  const bool hm = a.has_mean != 0;
#define QCE_F64_NP(Y)                                                                                              \
  if (a.NP == Y) {                                                                                                 \
    if (out_partial) return hm ? qce_f64_launch_t<MP, Y, true, true>(a, st) : qce_f64_launch_t<MP, Y, false, true>(a, st); \
    return hm ? qce_f64_launch_t<MP, Y, true, false>(a, st) : qce_f64_launch_t<MP, Y, false, false>(a, st);       \
  }
  QCE_F64_NP(16) QCE_F64_NP(32) QCE_F64_NP(64) QCE_F64_NP(128)
#undef QCE_F64_NP
  return hipErrorInvalidValue;
}
