// k_paths TD-estimator instantiations for DPI_EQ_GBM networks with Tanh hidden activations.
#include "dpi_dispatch.h"

bool dispatch_td_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM, true, DPI_ACT_TANH>(p, net, q);
}
