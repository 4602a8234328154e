// FP64 3M fused kernel for padded M = N = 128 (row halves, y in LDS; qce_f64h_kernel.h): launcher and table packing.
#include "qce_f64h_kernel.h"

bool qce_f64h_shape(int MP, int NP) {
  const char* e = getenv("QCE_F64_3M");
  if (e && e[0] == '0') return false;
  const char* q = getenv("QCE_F64H");  // QCE_F64H=0 keeps the 4M wave-pair kernel at padded 128 (A/B runs, tests)
  if (q && q[0] == '0') return false;
  return MP == 128 && NP == 128;
}

long long qce_pack_f64h_bytes(int has_mean) { return (long long)f64h_vb(has_mean ? 1 : 0) * 2 * 1024; }

hipError_t qce_launch_pack_f64h(int K, int M, int N, int has_mean, const double2* Linv, const double2* W,
                                const double2* q0, const double2* bvec, double* pack, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_f64h, dim3(2 * f64h_vb(has_mean ? 1 : 0), K), dim3(64), 0, st, M, N, has_mean, Linv, W,
                     q0, bvec, pack);
  return hipGetLastError();
}

hipError_t qce_f64h_launch(const QceF64Args& a, bool out_partial, hipStream_t st) {
#define QCE_F64H_GO(HM, OP)                                                                                       \
  hipLaunchKernelGGL((k_est_all_f64h<HM, OP>), dim3((unsigned)a.nwg), dim3(512), 0, st, a.B, a.M, a.N, a.K, a.R, a.L, \
                     a.y, a.pack, a.cconst, a.h, a.om, a.os, a.oa, a.pm, a.ps, a.pa, a.pk, a.shift)
  if (a.has_mean) {
    if (out_partial) QCE_F64H_GO(true, true);
    else QCE_F64H_GO(true, false);
  } else {
    if (out_partial) QCE_F64H_GO(false, true);
    else QCE_F64H_GO(false, false);
  }
#undef QCE_F64H_GO
  return hipGetLastError();
}
