// Chunk-streamed fused 'all'-mode estimate kernel for the large shapes (padded M or N of 128 or
// 256: cfg4 N=128, cfg5 N=256, multi-pilot observations M = n_pilots N) on gfx950.
//
// Same math and arithmetic as k_est_all_h2 (qce_estimate_h2.hip; gmm_cplx_bussgang.py:220-228,
// :331-332, :388-435, :632-656): per component k the whitened residual u = E(Linv_k)[y;1] (GL,
// lower-triangular 32x16 tiles skipped), lp = c_k - |u|^2, an online softmax over k, and
// Z = E(W_k)[y;1] (GW) folded into the accumulator; FP16 two-term split tables on
// v_mfma_f32_32x32x16_f16, fp32 accumulation, FP64 quad form / softmax state.
//
// What changes with size: a component's tables no longer fit in LDS (MP = NP = 256: 544 KB GL +
// 1 MB GW), so they are streamed through a ring of X_NSLOT chunks of X_CH k-steps (16 KB each) by
// global_load_lds, X_NSLOT - 1 chunks ahead.  The step sequence of a component (GL steps, then the
// GW steps of this workgroup's row chunk) is fully unrolled; LDS fragments are prefetched two steps
// ahead across chunk and component boundaries, and the first read of every chunk is preceded by
// the chunk's sync (own vmcnt for its DMA, LDS-read drain, barrier, refill of the slot just freed).
//
// Workgroup = 4 waves (one per SIMD, up to 512 registers per lane) x 32 samples = 128-sample tile.
// Registers: y fragments (4 per k-step, 8 when the observations are not exact in fp16) + the
// accumulator rows of the row chunk (16 per 32-row slice).  When they do not fit, the output rows
// are cut into row chunks (grid.z), each recomputing the GL phase.  grid.y splits the K range so
// that tiles x splits fills the chip; split partials (m, s, acc) are combined by k_merge_splits,
// which also produces the K-shard partial format of the multi-GPU path.
#pragma once
#include "qce_common.h"
#include "qce_h2_common.h"
#include "qce_kernels.h"

namespace {

constexpr int X_NW = 4;                         // waves per workgroup
constexpr int X_TILE = 32 * X_NW;               // samples per workgroup
constexpr int X_CH = 8;                         // k-steps per chunk
constexpr int X_CHB = X_CH * 2048;              // bytes per chunk
constexpr int X_NSLOT = 8;                      // ring slots
constexpr int X_OPS = X_CHB / 1024 / X_NW;      // global_load_lds per wave per chunk
constexpr int X_LDS = X_NSLOT * X_CHB;          // 128 KB

template <int MP, int NP, bool HM, int RSW>
struct XGeom {
  using G = H2Geom<MP, NP, HM>;
  static constexpr int NSL = G::NSL, NSW = G::NSW, KS = G::KS, HMI = G::HMI;
  static constexpr int SPS = KS + HMI;                      // GW steps per slice
  static constexpr int NVL = G::GL_STEPS;                   // GL steps per component
  static constexpr int NVW = RSW * SPS;                     // GW steps per row chunk
  static constexpr int NV = NVL + NVW;
  static constexpr int NCL = (NVL + X_CH - 1) / X_CH;       // GL chunks
  static constexpr int NCW = (NVW + X_CH - 1) / X_CH;       // GW chunks
  static constexpr int NC = NCL + NCW;                      // chunks per component
  // virtual step v -> chunk index within the component and step offset within the chunk
  static constexpr int chunk_of(int v) { return v < NVL ? v / X_CH : NCL + (v - NVL) / X_CH; }
  static constexpr int off_of(int v) { return v < NVL ? v % X_CH : (v - NVL) % X_CH; }
};

QCE_DEV void x_stage(const char* __restrict__ src, char* dst, int wave, int lane) {
  wave = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
  for (int i = 0; i < X_OPS; ++i) {
    const int c = wave + X_NW * i;
    lds_dma16(src + c * 1024 + lane * 16, dst + c * 1024);
  }
}

template <int N_>
QCE_DEV void x_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N_) : "memory");
}

template <int N_>
QCE_DEV void x_wait_lgkm(f16x8& a, f16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N_));
}

// per-component scalars of this workgroup's row chunk: GL slice scales, GW slice scales, c_k
template <int NSL, int RSW>
struct XScalars {
  float l[NSL], w[RSW];
  double c;
  QCE_DEV void load(const float* __restrict__ sinv, const double* __restrict__ cconst, int k, int nsl_tot, int w0) {
    const float* sk = sinv + (long long)k * nsl_tot;
#pragma unroll
    for (int i = 0; i < NSL; ++i) l[i] = sk[i];
#pragma unroll
    for (int i = 0; i < RSW; ++i) w[i] = sk[NSL + w0 + i];
    c = cconst[k];
  }
};

}  // namespace

// grid: x = sample tile (128 samples), y = K split, z = row chunk.
// OUT: 0 = final h (no split), 1 = (m, s, acc) records for k_merge_splits / the K-shard partial.
template <int MP, int NP, bool HM, bool EXACT, int RSW>
__global__ __launch_bounds__(256, 1) void k_est_all_h2x(long long B, int M, int N, int K, int ksplit, int out_rec,
                                                        double y_scale, const int* __restrict__ yflag,
                                                        const double2* __restrict__ y, const char* __restrict__ pack,
                                                        long long cstride, const float* __restrict__ sinv,
                                                        const double* __restrict__ cconst, double2* __restrict__ h,
                                                        double* __restrict__ rm, double* __restrict__ rs,
                                                        float* __restrict__ ra) {
  using X = XGeom<MP, NP, HM, RSW>;
  using G = H2Geom<MP, NP, HM>;
  constexpr int KS = X::KS, NSL = X::NSL, SPS = X::SPS, NV = X::NV, NVL = X::NVL, NC = X::NC;
  __shared__ __attribute__((aligned(16))) char lds[X_LDS];
  if (EXACT == (*yflag != 0)) return;  // the other instance handles this batch
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, hh = lane >> 5;
  const long long t = blockIdx.x;
  const int sp = blockIdx.y, q = blockIdx.z;
  const int k0 = (int)(((long long)K * sp) / ksplit), k1 = (int)(((long long)K * (sp + 1)) / ksplit);
  const int w0 = q * RSW;  // first GW slice of this row chunk
  const long long sample = t * X_TILE + wave * 32 + j;
  const bool valid = sample < B;
  const long long gw_off = (long long)G::GL_BYTES + (long long)w0 * SPS * 2048;

  // Y^T fragments: k-step s covers real features 16s + 8hh + e = complex 8s + 4hh + e/2.  Loads are
  // clamped in-bounds and masked (no per-element branches); double -> fp16 goes through fp32 (the
  // hi/lo split stays exact to ~22 bits, and exact observations are small integers anyway).
  f16x8 yh[KS + X::HMI], yl[EXACT ? 1 : KS];
  {
    const long long srow = valid ? sample : B - 1;
    const float ys = (float)y_scale;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 8 * s + 4 * hh + e;
        const bool ok = valid && c < M;
        const double2 v = y[srow * M + (c < M ? c : M - 1)];
        const float re = ok ? (float)v.x * ys : 0.0f, im = ok ? (float)v.y * ys : 0.0f;
        const _Float16 rh = (_Float16)re, ih = (_Float16)im;
        yh[s][2 * e] = rh;
        yh[s][2 * e + 1] = ih;
        if (!EXACT) {
          yl[s][2 * e] = (_Float16)(re - (float)rh);
          yl[s][2 * e + 1] = (_Float16)(im - (float)ih);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // convert as loaded: no 4-register double2 per feature held live
    }
  }
  if (HM) {
#pragma unroll
    for (int e = 0; e < 8; ++e) yh[KS][e] = (_Float16)0.0f;
    if (hh == 0) yh[KS][0] = (_Float16)1.0f;  // the [y; 1] augmentation column
  }
  f32x16 out[RSW];
#pragma unroll
  for (int r = 0; r < RSW; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) out[r][e] = 0.0f;
  double m = QCE_NEG_INF, ssum = 0.0;
  if (k1 <= k0) goto write;  // empty split (K < ksplit)
  {
    const int total = (k1 - k0) * NC;  // chunks of this workgroup's stream
    const unsigned lds_base = (unsigned)(uintptr_t)lds;
    auto src_of = [&](int c) -> const char* {
      const int kk = c / NC, jj = c - kk * NC;
      const char* base = pack + (long long)(k0 + kk) * cstride;
      return jj < X::NCL ? base + (long long)jj * X_CHB : base + gw_off + (long long)(jj - X::NCL) * X_CHB;
    };
    // chunk c's sync: its DMA landed (own vmcnt), every wave's LDS reads done, barrier; then the slot
    // chunk c - 1 occupied takes chunk c - 1 + X_NSLOT
    auto sync = [&](int c) {
      if (c + X_NSLOT - 2 < total) x_wait_vm<(X_NSLOT - 2) * X_OPS>(); else x_wait_vm<0>();
      raw_barrier();
      const int nc = c - 1 + X_NSLOT;
      if (nc < total) x_stage(src_of(nc), lds + (nc % X_NSLOT) * X_CHB, wave, lane);
    };
    for (int c = 0; c < X_NSLOT - 1 && c < total; ++c) x_stage(src_of(c), lds + (c % X_NSLOT) * X_CHB, wave, lane);
    XScalars<NSL, RSW> cur, nxt;
    cur.load(sinv, cconst, k0, G::NSL + G::NSW, w0);
    sync(0);
    f16x8 buf[3][2];
    {  // steps 0 and 1 of the first component
      const unsigned a0 = lds_base + lane * 16;
      asm volatile("ds_read_b128 %0, %1" : "=v"(buf[0][0]) : "v"(a0));
      asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(buf[0][1]) : "v"(a0));
      constexpr int c1 = X::chunk_of(1), o1 = X::off_of(1);
      static_assert(c1 == 0, "first chunk holds at least two steps");
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(buf[1][0]) : "v"(a0), "i"(o1 * 2048));
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(buf[1][1]) : "v"(a0), "i"(o1 * 2048 + 1024));
    }
    for (int k = k0; k < k1; ++k) {
      const int cb = (k - k0) * NC;  // global index of this component's chunk 0
      double quad = 0.0;
      float alpha = 1.0f, p = 0.0f;
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
      static_for(
          [&](auto ic) {
            constexpr int v = decltype(ic)::value;
            constexpr int u = v + 2;  // step to prefetch (u >= NV: next component)
            {
              constexpr int uu = u < NV ? u : u - NV;
              constexpr int cj = X::chunk_of(uu) + (u < NV ? 0 : NC), co = X::off_of(uu);
              if constexpr (co == 0) {
                if constexpr (u < NV && cj == X::NCL) nxt.load(sinv, cconst, k + 1 < k1 ? k + 1 : k, G::NSL + G::NSW, w0);
                sync(cb + cj);
              }
              const unsigned addr = lds_base + (unsigned)(((cb + cj) % X_NSLOT) * X_CHB) + lane * 16;
              asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(buf[u % 3][0]) : "v"(addr), "i"(co * 2048));
              asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(buf[u % 3][1]) : "v"(addr), "i"(co * 2048 + 1024));
            }
            x_wait_lgkm<4>(buf[v % 3][0], buf[v % 3][1]);
            const f16x8 a0 = buf[v % 3][0], a1 = buf[v % 3][1];
            if constexpr (v < NVL) {  // GL step
              constexpr int r = c_gl_slice(v, X::HMI);
              constexpr int s = v - (r * (r + 1) + X::HMI * r);
              constexpr bool mean_step = HM && s == 2 * r + 2;
              const f16x8 yv = yh[mean_step ? KS : s];
              acc = mfma_h(a0, yv, acc);
              acc = mfma_h(a1, yv, acc);
              if constexpr (!EXACT && !mean_step) acc = mfma_h(a0, yl[s], acc);
              if constexpr (s == 2 * r + 1 + X::HMI) {  // slice complete
                float qs = 0.0f;
#pragma unroll
                for (int e = 0; e < 16; ++e) qs = fmaf(acc[e], acc[e], qs);
                const double is = (double)cur.l[r];
                quad = fma((double)qs, is * is, quad);
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
              }
              if constexpr (v == NVL - 1) {  // GL done: online softmax step
                quad += __shfl_xor(quad, 32);
                softmax_step(cur.c - quad, m, ssum, alpha, p);
              }
            } else {  // GW step of slice w0 + rr
              constexpr int wv = v - NVL, rr = wv / SPS, s = wv % SPS;
              constexpr bool mean_step = HM && s == KS;
              const f16x8 yv = yh[mean_step ? KS : s];
              acc = mfma_h(a0, yv, acc);
              acc = mfma_h(a1, yv, acc);
              if constexpr (!EXACT && !mean_step) acc = mfma_h(a0, yl[s], acc);
              if constexpr (s == SPS - 1) {
                const float ps = p * cur.w[rr];
#pragma unroll
                for (int e = 0; e < 16; ++e) out[rr][e] = fmaf(out[rr][e], alpha, ps * acc[e]);
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
              }
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the step order: fragment liveness as pipelined
          },
          std::make_integer_sequence<int, NV>{});
      // the next component's steps 0 and 1 were prefetched into buf[NV % 3], buf[(NV + 1) % 3]; the
      // loop body reads them from buf[0], buf[1]: land them, then rotate (one drain per component)
      if constexpr (NV % 3 != 0) {
        constexpr int b0 = NV % 3, b1 = (NV + 1) % 3;
        x_wait_lgkm<0>(buf[b0][0], buf[b0][1]);
        x_wait_lgkm<0>(buf[b1][0], buf[b1][1]);
        const f16x8 n0a = buf[b0][0], n0b = buf[b0][1], n1a = buf[b1][0], n1b = buf[b1][1];
        buf[0][0] = n0a;
        buf[0][1] = n0b;
        buf[1][0] = n1a;
        buf[1][1] = n1b;
      }
      cur = nxt;
    }
    x_wait_vm<0>();
  }
write:
  if (!valid) return;
  if (!out_rec) {  // final estimate rows of this row chunk
    const double inv = 1.0 / ssum;
    double2* hp = h + sample * N;
#pragma unroll
    for (int r = 0; r < RSW; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n0 = 16 * (w0 + r) + 4 * e + 2 * hh;
        if (n0 < N) hp[n0] = make_double2((double)out[r][4 * e + 0] * inv, (double)out[r][4 * e + 1] * inv);
        if (n0 + 1 < N) hp[n0 + 1] = make_double2((double)out[r][4 * e + 2] * inv, (double)out[r][4 * e + 3] * inv);
      }
    return;
  }
  const long long rec = (long long)sp * B + sample;
  if (q == 0 && hh == 0) {
    rm[rec] = m;
    rs[rec] = ssum;
  }
  float* pa = ra + rec * (2LL * N);
#pragma unroll
  for (int r = 0; r < RSW; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n0 = 16 * (w0 + r) + 4 * e + 2 * hh;
      if (n0 < N) *reinterpret_cast<float2*>(pa + 2 * n0) = make_float2(out[r][4 * e + 0], out[r][4 * e + 1]);
      if (n0 + 1 < N) *reinterpret_cast<float2*>(pa + 2 * n0 + 2) = make_float2(out[r][4 * e + 2], out[r][4 * e + 3]);
    }
}


namespace {

#ifndef QCE_X_BUDGET_E
#define QCE_X_BUDGET_E 264
#endif
#ifndef QCE_X_BUDGET_I
#define QCE_X_BUDGET_I 330
#endif
// row-chunk width (W slices per workgroup) so that y fragments + accumulators stay in registers
constexpr int x_rsw(int MP, int NP, bool exact) {
  const int nsw = (2 * NP) / 32;
  const int yregs = exact ? 4 * (MP / 8 + 1) : 8 * (MP / 8) + 4;
  // (the compiler keeps about twice this many registers live at one wave per SIMD; budgets found
  // by compiling every instance with -Rpass-analysis=kernel-resource-usage: no scratch spills)
  const int budget = exact ? QCE_X_BUDGET_E : QCE_X_BUDGET_I;
  int rsw = nsw;
  while (rsw > 1 && yregs + 16 * rsw > budget) rsw /= 2;
  return rsw;
}

template <int MP, int NP, bool HM, bool EXACT>
hipError_t launch_x_one(const QceH2XArgs& a, int ksplit, int out_rec, hipStream_t st) {
  constexpr int RSW = x_rsw(MP, NP, EXACT);
  constexpr int NRC = ((2 * NP) / 32) / RSW;
  dim3 grid((unsigned)((a.B + X_TILE - 1) / X_TILE), (unsigned)ksplit, (unsigned)NRC);
  hipLaunchKernelGGL((k_est_all_h2x<MP, NP, HM, EXACT, RSW>), grid, dim3(256), 0, st, a.B, a.M, a.N, a.K, ksplit,
                     out_rec, a.y_scale, a.yflag, a.y, a.pack, a.cstride, a.sinv, a.cconst, a.h, a.rm, a.rs, a.ra);
  return hipGetLastError();
}

template <int MP, int NP, bool HM>
hipError_t launch_x_t(const QceH2XArgs& a, int ksplit, int out_rec, hipStream_t st) {
  hipError_t e = launch_x_one<MP, NP, HM, true>(a, ksplit, out_rec, st);
  if (e != hipSuccess) return e;
  return launch_x_one<MP, NP, HM, false>(a, ksplit, out_rec, st);
}

}  // namespace

#define QCE_H2X_INSTANTIATE(X, Y)                                                                   \
  hipError_t qce_h2x_launch_##X##x##Y(const QceH2XArgs& a, bool hm, int ksplit, int out_rec, hipStream_t st) { \
    return hm ? launch_x_t<X, Y, true>(a, ksplit, out_rec, st) : launch_x_t<X, Y, false>(a, ksplit, out_rec, st); \
  }
