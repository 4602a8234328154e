// FP64 3M fused kernel instances for MP = 16 (compiled in parallel with the other MP)
#include "qce_f64g_kernel.h"

template hipError_t qce_f64g_launch_mp<16>(const QceF64Args& a, bool out_partial, hipStream_t st);
