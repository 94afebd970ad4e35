// k_baseline / k_paths instantiations for DPI_EQ_CHA (one translation unit per equation family).
#include "dpi_dispatch.h"

bool dispatch_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_CHA>(p, net, q);
}

#ifdef DPI_BASE_STAMPS
// measurement variant (tools/base_stamps.py): the k_baseline phase stamps of this unit's launches
extern "C" int dpi_debug_base_stamps_cha(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(dpi::dpi_bstamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
