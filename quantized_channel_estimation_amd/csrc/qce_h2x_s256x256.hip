// Instances of k_est_all_h2x for padded M = 256, N = 256 (see qce_h2x_kernel.h).
#include "qce_h2x_kernel.h"

QCE_H2X_INSTANTIATE(256, 256)
