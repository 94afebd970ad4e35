// k_baseline / k_paths instantiations for DPI_EQ_GBM (one translation unit per equation family).
#include "dpi_dispatch.h"

bool dispatch_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  return dpi_dispatch<DPI_EQ_GBM>(p, net, q);
}

#ifdef DPI_GBM_STAMPS
// measurement variant (tools/gbm_stamps.py): copy the phase stamps of the last GBM network launch
extern "C" int dpi_debug_gbm_stamps(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(dpi::dpi_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif

#ifdef DPI_BASE_STAMPS
// measurement variant (tools/base_stamps.py): the k_baseline phase stamps of this unit's launches
extern "C" int dpi_debug_base_stamps_gbm(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(dpi::dpi_bstamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
