// k_paths instantiations for DPI_EQ_GBM (first-order SDGD / exact-diagonal labels) with state
// dimensions above 128 (up to NXW_MAX = 256) and Tanh hidden activations: W1x read from L2, a unit of its own.
#include "dpi_dispatch.h"

bool dispatch_wide_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM, false, DPI_ACT_TANH, false, NXW_MAX>(p, net, q);
}
