// Host-side handles and the (equation, network shape) -> k_paths / k_baseline instantiation
// dispatch; dispatch<KIND> is instantiated once per equation kind in dpi_paths_{cha,ou,gbm}.hip
// so the three families compile in parallel.
#pragma once
#include <hip/hip_ext.h>

#include "dpi_device.h"

using namespace dpi;

struct dpi_problem_s {
  EqDev e;
  float td_dt = 0.f;  // DATA.ESTIMATE_DELTA_T (dpi_problem_set_estimate_delta_t)
  float alpha_init_sqrt;
  std::vector<void*> dev;
};

struct dpi_net_s {
  NetDev d;        // d.kind: 0 zero, 1 mlp, 2 PISGradNet
  NetPisDev pis;
  void* blob = nullptr;
  int n_in = 0;
  int precision = -1;     // DPI_GEMM_* for this net (dpi_net_set_precision); -1: the process-wide mode
  bool finite = true;     // every uploaded parameter finite
  // Range-guard ring (dpi_net_status*): DPI_STATUS_SLOTS sticky words, one per 64-B line, in
  // fine-grained pinned host memory; `status` is its device address, `status_host` the host one.
  // The label reductions store DPI_STATUS_* bits into slot `slot`, selected at enqueue time.
  int* status = nullptr;
  int* status_host = nullptr;
  int slot = 0;
};
constexpr int STATUS_STRIDE = 16;  // ints per ring slot (64 B)

// ---- dispatch over (equation, network shape)
struct Launch {
  bool baseline;
  const float* tx;
  int n;
  float *gx, *fb, *bx, *hb;
  const PathArgs* a;
  int nblocks;
  hipStream_t st;
  bool hess = false;  // k_paths in Hessian-label mode (GBM only)
  bool td = false;    // k_paths with the TD estimators (problem td_dt > 0)
  SampleSpec smp{};   // baseline: sample the points in the same launch (smp.tx != null)
  int* tickets = nullptr;  // baseline: zero the fused reduce's per-point tickets
  const FusedBase* fbase = nullptr;  // k_paths_fb: the one-launch sample_with_gradients (fused_base_ok)
  // dpi_launch_timer_arm: the path launch's own start / stop timestamps (hipExtLaunchKernel records
  // them on the dispatch packet itself — no marker packets between the launches); null: untimed
  hipEvent_t t0 = nullptr, t1 = nullptr;
};
// The path launches (k_paths, k_paths_fb) of a Launch, with its timer events when armed.
#define DPI_PATH_LAUNCH(KERN, q, ...) \
  hipExtLaunchKernelGGL(KERN, dim3((q).nblocks), dim3(NTH), 0, (q).st, (q).t0, (q).t1, 0, __VA_ARGS__)

// TDV: the TD-estimator k_paths variants, compiled in translation units of their own
// (dpi_paths_td_*.hip): sharing a unit with the plain kernels perturbs the register allocation
// of the plain fused-MLP kernel (6 spills at 256 VGPRs instead of none at 252).
// ACT: the hidden activation (DPI_ACT_*); the Tanh k_paths family lives in units of its own too
// (dpi_paths_*_tanh.hip).  k_baseline is shape- and activation-generic (it reads net.act).
// FBV: k_paths_fb, the one-launch sample_with_gradients (q.fbase), in translation units of its own
// (dpi_paths_fb_*.hip: beside the plain kernels it perturbed their register allocation — the
// OU 4 x 128 split instance went from 255 VGPRs to 256 and 3 spilled).  Instantiated where
// fused_base_shape holds, which is where dpi_kernels.hip fused_base_ok selects it: Cha / OU with
// ELU, zero nets and the fp16-split MLP instances (H % 32 == 0) — except OU 4 x 128, whose GMM
// statistics beside the hand-off spill 3 VGPRs at two workgroups per CU (it keeps two launches).
template <int KIND, int H, int L, bool Z, int ACT>
constexpr bool fused_base_shape() {
  return KIND != DPI_EQ_GBM && ACT == DPI_ACT_ELU && (Z || (H % 32 == 0 && !(KIND == DPI_EQ_OU && H == 128 && L == 4)));
}
// NXW > NXP_MAX: the wide first-order instances (Cha / OU, nx up to NXW_MAX; dpi_paths_wide_*.hip):
// plain k_paths only — the baseline is shape-generic, the TD / Hessian / fused-baseline forms have none.
template <int KIND, int H, int L, bool Z, bool TDV, int ACT = DPI_ACT_ELU, bool FBV = false, int NXW = NXP_MAX>
void do_launch(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  if constexpr (NXW > NXP_MAX) {
    static_assert(!TDV && !FBV, "wide instances: first-order labels");
    if constexpr (!Z && H % 32 == 0) {
      if (q.a->split) {
        DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, true, false, false, ACT, NXW>), q, p->e, net->d, *q.a);
        return;
      }
    }
    DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, false, false, ACT, NXW>), q, p->e, net->d, *q.a);
  } else if constexpr (FBV) {
    if constexpr (fused_base_shape<KIND, H, L, Z, ACT>())
      DPI_PATH_LAUNCH((k_paths_fb<KIND, H, L, Z, !Z, ACT>), q, p->e, net->d, *q.a,
                         *q.fbase);
  } else if constexpr (TDV) {
    if constexpr (!Z && H % 32 == 0) {
      if (q.a->split)
        DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, true, false, true, ACT>), q, p->e,
                           net->d, *q.a);
      else
        DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, false, true, ACT>), q, p->e, net->d, *q.a);
    } else {
      DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, false, true, ACT>), q, p->e,
                         net->d, *q.a);
    }
  } else if (q.baseline) {
    if constexpr (KIND == DPI_EQ_GBM) {
      if (p->e.nx > NXP_MAX)  // the wide baseline (nx <= 256)
        hipLaunchKernelGGL((k_baseline_gbm<Z, NXW_MAX>), dim3(q.n), dim3(NTHB), 0, q.st, p->e, net->d, q.tx, q.n, q.gx,
                           q.fb, q.bx, q.hb, q.smp, q.tickets);
      else
        hipLaunchKernelGGL((k_baseline_gbm<Z>), dim3(q.n), dim3(NTHB), 0, q.st, p->e, net->d, q.tx, q.n, q.gx, q.fb,
                           q.bx, q.hb, q.smp, q.tickets);
    }
    else
      hipLaunchKernelGGL((k_baseline<KIND, Z>), dim3(q.n), dim3(NTB), 0, q.st, p->e, net->d, q.tx, q.n, q.gx, q.fb,
                         q.bx, q.smp, q.tickets);
  } else if (q.hess) {
    if constexpr (KIND == DPI_EQ_GBM) {
      EqDev e2 = p->e;
      e2.sdgd_v = 0;  // the Hessian estimators evaluate f with the full Hessian (data.py:856, :1262-1272)
      if constexpr (!Z && H % 32 == 0) {
        if (q.a->split) {
          DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, true, true, false, ACT>), q, e2, net->d, *q.a);
          return;
        }
      }
      DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, true, false, ACT>), q, e2,
                         net->d, *q.a);
    }
  } else if constexpr (!Z && H % 32 == 0) {
    if (q.a->split)
      DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, true, false, false, ACT>), q, p->e,
                         net->d, *q.a);
    else
      DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, false, false, ACT>), q, p->e, net->d, *q.a);
  } else
    DPI_PATH_LAUNCH((k_paths<KIND, H, L, Z, false, false, false, ACT>), q, p->e,
                       net->d, *q.a);
}

template <int KIND, bool TDV = false, int ACT = DPI_ACT_ELU, bool FBV = false, int NXW = NXP_MAX>
bool dpi_dispatch(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  if constexpr (NXW > NXP_MAX) {
    if (q.baseline || q.hess || q.fbase) return false;
  }
  if constexpr (ACT == DPI_ACT_ELU) {  // zero nets and the (activation-generic) baseline: the ELU units
    if (net->d.kind == 0) {
      do_launch<KIND, 16, 1, true, TDV, DPI_ACT_ELU, FBV, NXW>(p, net, q);
      return true;
    }
  } else {
    if (net->d.kind == 0 || q.baseline) return false;
  }
  const int H = net->d.H, L = net->d.L;
  if constexpr (!TDV && !FBV && ACT == DPI_ACT_ELU && NXW == NXP_MAX) {
    if (q.baseline) {  // the baseline kernel is shape-generic
      if (KIND == DPI_EQ_GBM && H > 64) return false;
      do_launch<KIND, 16, 1, false, false>(p, net, q);
      return true;
    }
  }
  if constexpr (KIND == DPI_EQ_GBM) {  // all weights LDS-resident: H <= 64
#define DPI_SHAPE(HH, LL)                      \
  if (H == HH && L == LL) {                    \
    do_launch<KIND, HH, LL, false, TDV, ACT, FBV, NXW>(p, net, q); \
    return true;                               \
  }
    DPI_SHAPE(64, 3)
    DPI_SHAPE(64, 2)
    DPI_SHAPE(32, 2)
    DPI_SHAPE(32, 3)
    DPI_SHAPE(16, 1)
    DPI_SHAPE(16, 2)
    DPI_SHAPE(16, 3)
    return false;
  } else {
    DPI_SHAPE(128, 4)
    DPI_SHAPE(128, 3)
    DPI_SHAPE(128, 2)
    DPI_SHAPE(64, 3)
    DPI_SHAPE(64, 2)
    DPI_SHAPE(32, 2)
    DPI_SHAPE(16, 1)
    DPI_SHAPE(16, 2)
    DPI_SHAPE(16, 3)
#undef DPI_SHAPE
    return false;
  }
}

bool dispatch_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_ou(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_ou(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_cha_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_ou_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_cha_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_ou_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_td_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_fb_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_fb_ou(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_cha(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_ou(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_cha_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_ou_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_gbm(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
bool dispatch_wide_gbm_tanh(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q);
