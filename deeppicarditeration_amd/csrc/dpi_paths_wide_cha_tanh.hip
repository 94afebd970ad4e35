// k_paths instantiations for DPI_EQ_CHA with state dimensions above 128 and Tanh hidden activations.
#include "dpi_dispatch.h"

bool dispatch_wide_cha_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_CHA, false, DPI_ACT_TANH, false, NXW_MAX>(p, net, q);
}
