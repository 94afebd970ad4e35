// k_baseline / k_paths instantiations for DPI_EQ_CHA (one translation unit per equation family).
#include "dpi_dispatch.h"

bool dispatch_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_CHA>(p, net, q);
}
