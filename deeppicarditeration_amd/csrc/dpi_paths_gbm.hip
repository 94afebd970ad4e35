// k_baseline / k_paths instantiations for DPI_EQ_GBM (one translation unit per equation family).
#include "dpi_dispatch.h"

bool dispatch_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM>(p, net, q);
}
