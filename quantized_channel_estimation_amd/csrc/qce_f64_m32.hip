// FP64 fused kernel instances for MP = 32 (compiled in parallel with the other MP)
#include "qce_f64_kernel.h"

template hipError_t qce_f64_launch_mp<32>(const QceF64Args& a, bool out_partial, hipStream_t st);
