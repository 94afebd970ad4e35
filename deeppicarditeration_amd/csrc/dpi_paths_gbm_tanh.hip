// k_paths instantiations for DPI_EQ_GBM networks with Tanh hidden activations (torch.nn.Tanh, the
// reference's default NETWORK.ACTIVATIONS, picard/config.py:61); the TD estimators in
// dpi_paths_td_gbm_tanh.hip.
#include "dpi_dispatch.h"

bool dispatch_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM, false, DPI_ACT_TANH>(p, net, q);
}
