// Shared device helpers for the Bussgang-GMM estimate path (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define QCE_DEV __device__ __forceinline__
// widest uniform quantiser qce_prepare accepts (the Bussgang gain sums 2^b - 1 terms per diagonal entry)
#define QCE_MAX_UNIFORM_BITS 16

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// complex128 stored as (re, im) double pairs, numpy complex128 layout
QCE_DEV double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
QCE_DEV double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
QCE_DEV double2 cmul(double2 a, double2 b) { return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
// a * conj(b)
QCE_DEV double2 cmulc(double2 a, double2 b) { return make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); }
QCE_DEV double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
QCE_DEV double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
// acc += a * b
QCE_DEV double2 cfma(double2 a, double2 b, double2 acc) {
  acc.x = fma(a.x, b.x, acc.x);
  acc.x = fma(-a.y, b.y, acc.x);
  acc.y = fma(a.x, b.y, acc.y);
  acc.y = fma(a.y, b.x, acc.y);
  return acc;
}
// numpy-style complex division a / b (Smith's algorithm as in npymath)
QCE_DEV double2 cdiv(double2 a, double2 b) {
  double abs_br = fabs(b.x), abs_bi = fabs(b.y);
  if (abs_br >= abs_bi) {
    double rat = b.y / b.x;
    double scl = 1.0 / (b.x + b.y * rat);
    return make_double2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
  }
  double rat = b.x / b.y;
  double scl = 1.0 / (b.y + b.x * rat);
  return make_double2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
}

// MFMA wrappers (lane maps verified on MI355X by tools/probe/mfma_layout_probe.hip)
//  f32 32x32x2 : A[i=l&31][k=l>>5], B[k=l>>5][j=l&31]; D row=(r&3)+8(r>>2)+4(l>>5), col=l&31
//  f32 16x16x4 : A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]; D row=4(l>>4)+r,           col=l&15
//  f64 16x16x4 : A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]; D row=(l>>4)+4r,           col=l&15
QCE_DEV f32x16 mfma32x32x2(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
QCE_DEV f32x4 mfma16x16x4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
QCE_DEV f64x4 mfma16x16x4d(double a, double b, f64x4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// 16 B per lane global -> LDS DMA (lane l writes LDS byte dst + 16 l; dst wave-uniform), issued as inline asm.
// With __builtin_amdgcn_global_load_lds the compiler cannot tell the DMA's LDS bytes from a later ds_read of another
// ring slot and inserts s_waitcnt vmcnt(0) before the next LDS read after every refill: the wave then waits out the
// refill's whole L2 / HBM latency once per ring chunk (27 % of MFMA time at one wave per SIMD, cfg4).  The ring
// code orders LDS itself (explicit vmcnt + s_barrier before a slot is read), and the compiler's own vmcnt counts
// stay safe: loads it does not know about only make its waits stricter.  M0 is set right before the DMA (the
// compiler sets M0 itself before every instruction of its own that reads it).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
QCE_DEV void lds_dma16(const void* src, const void* lds_dst) {
  const unsigned dst = (unsigned)(unsigned long)(__attribute__((address_space(3))) const void*)lds_dst;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst) : "memory", "m0");
}
#pragma clang diagnostic pop

#include "../../include/qce.h"
