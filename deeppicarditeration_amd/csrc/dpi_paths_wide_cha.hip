// k_paths instantiations for DPI_EQ_CHA with state dimensions above 128 (up to NXW_MAX = 256): the
// first-order labels at one workgroup per CU (a unit of its own).
#include "dpi_dispatch.h"

bool dispatch_wide_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_CHA, false, DPI_ACT_ELU, false, NXW_MAX>(p, net, q);
}
