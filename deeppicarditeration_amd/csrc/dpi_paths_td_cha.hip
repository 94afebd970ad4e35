// k_paths TD-estimator instantiations for DPI_EQ_CHA (ESTIMATE_DELTA_T > 0; a unit of their own).
#include "dpi_dispatch.h"

bool dispatch_td_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_CHA, true>(p, net, q);
}
