// k_paths_fb instantiations for DPI_EQ_OU (the one-launch dpi_sample_with_gradients; a unit of its own).
#include "dpi_dispatch.h"

bool dispatch_fb_ou(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_OU, false, DPI_ACT_ELU, true>(p, net, q);
}
