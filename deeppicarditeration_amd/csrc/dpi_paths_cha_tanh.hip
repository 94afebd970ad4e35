// k_paths instantiations for DPI_EQ_CHA networks with Tanh hidden activations (plain and TD
// estimators; torch.nn.Tanh, the reference's default NETWORK.ACTIVATIONS, picard/config.py:61).
#include "dpi_dispatch.h"

bool dispatch_cha_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return q.td ? dpi_dispatch<DPI_EQ_CHA, true, DPI_ACT_TANH>(p, net, q)
              : dpi_dispatch<DPI_EQ_CHA, false, DPI_ACT_TANH>(p, net, q);
}
