// k_paths TD-estimator instantiations for DPI_EQ_OU networks with Tanh hidden activations.
#include "dpi_dispatch.h"

bool dispatch_td_ou_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_OU, true, DPI_ACT_TANH>(p, net, q);
}
