// k_paths TD-estimator instantiations for DPI_EQ_GBM (ESTIMATE_DELTA_T > 0; a unit of their own).
#include "dpi_dispatch.h"

bool dispatch_td_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM, true>(p, net, q);
}
