/*
 * dpi.h — C-ABI of the MI355X-native DPI label-generation hot path (libdpi_hip.so).
 *
 * Plain pointers and sizes only; no torch types.  Every device pointer is caller-owned
 * (e.g. a torch-ROCm tensor's data_ptr()); the library never frees caller memory.  Calls are
 * stream-ordered on `stream` (a hipStream_t; NULL = default stream) and never synchronise
 * the device, so they can be captured into a hipGraph.  Return 0 on success or a negative
 * DPI_ERR_* code; dpi_last_error() returns the thread-local message.  No C++ exception
 * crosses the ABI.  n = 0 points is a valid empty batch: the call checks its scalar arguments,
 * launches nothing and accepts NULL data pointers.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   dpi_problem_create_cha   picard/equations.py:266-338  Cha(nx, alpha, k, T)
 *   dpi_problem_create_ou    picard/equations.py:489-714  OUProcessEquation(...) + utils.py:792-914 GMM
 *   dpi_problem_create_gbm   picard/equations.py:388-486  GBMEquationComplexExact(nx, alpha, T)
 *   dpi_problem_set_hessian_approximation  picard/data.py:115-123, :497-502  HESSIAN_APPROXIMATION (SDGD v)
 *   dpi_problem_set_estimate_delta_t  picard/data.py:1209-1213, :934-952, :529-575  ESTIMATE_DELTA_T (TD estimators)
 *   dpi_net_create_zero      picard/solution.py:330-337   ZeroSolution (iteration 1)
 *   dpi_net_create_mlp       picard/solution.py:123-135   construct_mlp (state-dict order)
 *   dpi_net_create_pisgrad   picard/solution.py:138-289   PISGradNet (state-dict order)
 *   dpi_sample_points        picard/data.py:161-167, :211-217  sample_t_always_uniform + equation.sample_x
 *   dpi_sample_points_t      picard/data.py:149-159 (sample_t, t_always_uniform: false) or :161-167
 *   dpi_point_baseline       picard/data.py:506-518, :918-920  g(x) and get_f(..., baseline_repeat=M)
 *   dpi_label_moments        picard/data.py:899-926 + :471-527 (+ :1226-1325 get_f) summed over MC paths
 *   dpi_label_finalize       picard/data.py:924-926, :525-526, :222  mean over M, + g(x), clip
 *   dpi_generate_with_gradients  picard/data.py:1208-1218 (baseline + moments + finalize)
 *   dpi_sample_with_gradients    picard/data.py:211-223 (sample_with_gradients: points + all of the above)
 *   dpi_sample_points_baseline   picard/data.py:211-217 + :506-518, :918-920 (the points and their baseline)
 *   dpi_moments_reduce       (no reference counterpart: fixed-order combine of per-rank moments)
 *   dpi_generate_with_gradients_and_hessians  picard/data.py:1220-1223 (+ :1153-1201, :823-897, :225-237)
 *   dpi_label_moments_hessians / dpi_label_finalize_hessians  the same, split for MC sharding
 *   dpi_sums_reduce          (no reference counterpart: fixed-order combine of per-rank sums)
 *   dpi_set_gemm_precision   (no reference counterpart: MFMA precision of the network evaluation)
 */
#ifndef DPI_H_
#define DPI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPI_ABI_VERSION 7

/* error codes */
#define DPI_OK 0
#define DPI_ERR_ARG (-1)
#define DPI_ERR_UNSUPPORTED (-2)
#define DPI_ERR_HIP (-3)
#define DPI_ERR_WORKSPACE (-4)

/* Philox stream tags: counter word c3 = tag | (epoch << 8) (see csrc/dpi_rng.h) */
#define DPI_TAG_T 1
#define DPI_TAG_X0 2
#define DPI_TAG_X 3
#define DPI_TAG_TERM 4
#define DPI_TAG_S 5
#define DPI_TAG_INT 6
#define DPI_TAG_SDGD 7
#define DPI_TAG_HTERM 8
#define DPI_TAG_HINT 9

/* equation kinds */
#define DPI_EQ_CHA 1
#define DPI_EQ_OU 2
#define DPI_EQ_GBM 3

/* activations */
#define DPI_ACT_ELU 1
#define DPI_ACT_TANH 2

/* estimator selection (dpi_label_moments / finalize flags) */
#define DPI_TERMINAL 1 /* estimate_terminal_with_gradients (data.py:899-926) */
#define DPI_INTEGRAL 2 /* estimate_integral_with_gradients (data.py:471-527) */
#define DPI_BOTH 3     /* generate_with_gradients (data.py:1208-1218) */
/* dpi_label_moments: dpi_label_prepare already ran on this workspace with the same arguments */
#define DPI_PREPARED 4

/* Monte-Carlo paths per workgroup: m ranges are multiples of this. */
#define DPI_PATH_BLOCK 64
/* paths (m_end - m_begin) one label-moments call takes: 1024 path blocks per point */
#define DPI_PATHS_PER_CALL_MAX 65536

typedef struct dpi_problem_s* dpi_problem;
typedef struct dpi_net_s* dpi_net;

int dpi_abi_version(void);
/* Copies the calling thread's last error message (NUL-terminated); returns its length. */
int dpi_last_error(char* buf, size_t len);

/* --- problem plugins (host parameters copied to device; fp64 in, fp32 on device) ---
 * State dimensions: every problem takes nx <= 256 (NXW_MAX); above 128 the first-order labels of MLP
 * and zero networks run on the wide path instances (one workgroup per CU).  The
 * Malliavin Hessian labels, the TD estimators and PISGradNet are compiled for nx <= 128 (NXP_MAX).
 * Past a cap a call fails with DPI_ERR_UNSUPPORTED naming it (the reference's shipped configurations
 * are 10-d and 100-d). */
int dpi_problem_create_cha(int nx, double alpha, double k, double T, dpi_problem* out);
/* mean: (n_comp, nx); var_diag: (n_comp, nx) diagonal of each component covariance; pi: (n_comp) */
int dpi_problem_create_ou(int nx, double alpha, double T, double theta, double mu, double alpha_scale,
                          int n_comp, const double* mean, const double* var_diag, const double* pi,
                          dpi_problem* out);
/* w: (n_nodes, 1+nx); v: (n_nodes) */
int dpi_problem_create_gbm(int nx, double alpha, double T, int n_nodes, const double* w, const double* v,
                           dpi_problem* out);
/* DATA.HESSIAN_APPROXIMATION for equations with a Hessian term (GBM): sdgd_v = 0 uses the exact
 * Hessian diagonal (picard/data.py:1262-1272); 1 <= sdgd_v <= 255 draws v indices in [0, nx)
 * with replacement per path (SDGD, data.py:497-502, 1273-1303). */
int dpi_problem_set_hessian_approximation(dpi_problem p, int sdgd_v);
/* DATA.ESTIMATE_DELTA_T: delta_t > 0 selects the TD estimators of generate_with_gradients
 * (estimate_terminal_with_gradients_td, estimate_integral_with_gradients_td): per point the
 * horizon is t_next = min(t + delta_t, T) instead of T, s ~ U(t, t_next], and the terminal value
 * is u(t_next, X_{t_next}) (the network) where t_next < T, g(X_T) otherwise.  0 (default) = the
 * plain estimators.  Every network kind (PISGradNet: a terminal stage — rollout to t_next, forward
 * GEMM chain, u — before the integral stage); the Hessian-label entry points ignore it, as the
 * reference's generate_with_gradients_and_hessians does. */
int dpi_problem_set_estimate_delta_t(dpi_problem p, double delta_t);
int dpi_problem_destroy(dpi_problem p);

/* --- networks u(t, x): weights uploaded once per Picard iteration into a library handle --- */
int dpi_net_create_zero(dpi_net* out);
/* params: host fp32, torch state-dict order of construct_mlp(n_in, 1, widths, act):
 *   W0 (widths[0] x n_in), b0, W1 (widths[1] x widths[0]), b1, ..., Wout (1 x widths[-1]), bout.
 * Supported (width, n_hidden): all hidden widths equal, one of 16/32/64/128, n_hidden 1..4
 * (GBM: width <= 64).  act: the activation of every hidden layer, DPI_ACT_ELU (torch.nn.ELU,
 * alpha = 1) or DPI_ACT_TANH (torch.nn.Tanh, the reference's default NETWORK.ACTIVATIONS,
 * picard/config.py:61). */
int dpi_net_create_mlp(int n_in, int n_hidden, const int* widths, int act, const float* params,
                       size_t n_params, dpi_net* out);
/* PISGradNet(hidden_shapes, dim = nx, g0 = equation.g, T) for OUProcessEquation; params: host fp32 in
 * torch state-dict order (timestep_phase, timestep_coeff, t_encoder.{0,2}, smooth_net.{0,2,..,2(L+1)},
 * nn_module.{0,2,..,2L} weights and biases).  Runs as an MFMA pipeline: rollout, time networks, the
 * nn_module forward + VJP chain (one k_pis_net launch with the activations in LDS for 1-4 hidden
 * layers of 512 in the fp16-split mode, else layer-wise GEMMs), final contributions. */
int dpi_net_create_pisgrad(int nx, int n_hidden, const int* hidden, double T, const float* params,
                           size_t n_params, dpi_net* out);
int dpi_net_destroy(dpi_net net);

/* MFMA precision of the network evaluations.  DPI_GEMM_F32: v_mfma_f32_16x16x4_f32 everywhere.
 * DPI_GEMM_F16X3: fp16-split x = hi + 2^-11 lo, three v_mfma_f32_16x16x32_f16 per product
 * (~2.4e-7 relative error, same tolerance class as fp32) everywhere: the fused MLP of the path
 * kernel, and the PISGradNet pipeline with its activations stored split in HBM.
 * DPI_GEMM_AUTO (default) = DPI_GEMM_F16X3.
 * The environment variable DPI_GEMM=f32|f16x3 sets the initial mode.
 * Replaces no reference interface (the reference evaluates u in torch fp64/fp32). */
#define DPI_GEMM_F32 0
#define DPI_GEMM_F16X3 1
#define DPI_GEMM_AUTO 2
int dpi_set_gemm_precision(int mode);

/* Per-network override of the GEMM precision (-1: follow dpi_set_gemm_precision).  The host layer
 * switches one network to DPI_GEMM_F32 when its split evaluation leaves fp16's range (below). */
int dpi_net_set_precision(dpi_net net, int mode);

/* Range guard.  Every label reduction of a call on `net` (dpi_label_moments*, the Hessian sums)
 * sets DPI_STATUS_NONFINITE in a sticky status word of the net when a label sum (not a sum of
 * squares, whose overflow leaves the labels intact) is not finite
 * while every parameter of the net is finite: the network evaluation overflowed its number format
 * (fp16's 65,504 in the fp16-split PISGradNet storage, or fp32's range), where the fp64 reference
 * would not.  (Non-finite parameters give non-finite labels as in the reference, unflagged.)
 *
 * The words form a ring of DPI_STATUS_SLOTS slots in host-visible (fine-grained, pinned) memory,
 * written by the kernels with a plain vector store.  A call flags into the slot that was selected
 * when it was enqueued (dpi_net_status_slot; slot 0 at creation), so a caller can give a group of
 * calls a slot of its own and read it once the group's work has completed (an event) with
 * dpi_net_status_peek, which reads host memory and issues no HIP call: the range check of a label
 * buffer costs no stream synchronisation of its own.
 * dpi_net_status: the selected slot after the work queued on `stream` (a synchronisation) and,
 * with clear != 0, resets it.  dpi_net_status_slot: select `slot` for the calls enqueued from now
 * on and, with clear != 0, zero it first (a host store: no enqueued call may still flag into it).
 * Zero networks have no status words: their reads return 0.  Replaces no reference interface.
 * DPI_STATUS_HANDOFF (stored together with DPI_STATUS_NONFINITE, the point's labels NaN): a path
 * block of the one-launch dpi_sample_with_gradients did not see its point's baseline within its
 * bounded wait — an internal failure, never a range problem. */
#define DPI_STATUS_NONFINITE 1
#define DPI_STATUS_HANDOFF 2
#define DPI_STATUS_SLOTS 64
int dpi_net_status(dpi_net net, int clear, void* stream, int* status);
int dpi_net_status_slot(dpi_net net, int slot, int clear);
int dpi_net_status_peek(dpi_net net, int slot, int* status);

/* Identity of this build: the SHA-256 (hex) of the sources and flags it was compiled from
 * (deeppicarditeration_amd/build.py source_hash), NUL-terminated into buf; returns its length.
 * The host layer refuses a library whose identity differs from the tree's sources. */
int dpi_build_id(char* buf, size_t len);

/* Measurement (bench.py's kernel time; no reference counterpart).  dpi_launch_timer_arm(slot)
 * arms timer slot (0 <= slot < DPI_LAUNCH_TIMERS) for the calling thread: the next path launch it
 * enqueues (k_paths / k_paths_fb of a label call, or k_pis_net of a PISGradNet label call) records
 * the slot's start / stop events on its own dispatch packet (hipExtLaunchKernel), and disarms it.
 * dpi_launch_timer_ms waits for the slot's stop event and writes the launch's duration in ms;
 * DPI_ERR_ARG if the slot never recorded a launch since it was last armed. */
#define DPI_LAUNCH_TIMERS 256
int dpi_launch_timer_arm(int slot);
int dpi_launch_timer_ms(int slot, float* ms);

/* Device workspace a dpi_* call on (p, net, n points, M paths) needs. */
size_t dpi_workspace_bytes(dpi_problem p, dpi_net net, int n, int M);

/* Workspace of dpi_label_prepare and of the DPI_PREPARED dpi_label_moments call it feeds: for a GBM
 * MLP net it adds the staged noise sums ((n, M / 64, 2, 4 ceil(nx / 4), 64) floats), otherwise it
 * equals dpi_workspace_bytes. */
size_t dpi_workspace_bytes_prepared(dpi_problem p, dpi_net net, int n, int M);

/* Draws 1-3 of sample_with_gradients: tx (n, 1+nx) fp32 device, t = (T-2eps)(1-U)+eps,
 * x = x0 + sqrt(t) sqrt(alpha) xi.  Point i uses counter c2 = point_base + i. */
int dpi_sample_points(dpi_problem p, int n, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                      float* tx, void* stream);

/* dpi_sample_points with the t sampler chosen by t_factors (0 <= t_factors <= 4096):
 * 0 = sample_t_always_uniform (as dpi_sample_points); R >= 1 = sample_t (t_always_uniform: false,
 * picard/data.py:149-159), t = T (1 - U_0 U_1 ... U_{R-1}) with R = N - i + 1, U_r = word r&3 of
 * Philox counter (r>>2, 0, point_base + i, DPI_TAG_T | epoch << 8), eps unused. */
int dpi_sample_points_t(dpi_problem p, int n, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                        int t_factors, float* tx, void* stream);

/* Per-point baseline g(x), f(t, x, u, grad u) (+ network terms) into the workspace.  For a
 * PISGradNet net it launches nothing: each label call forms g(x) and f_b in its first path chunk
 * (the baseline rows ride in the k_pis_net chain, g(x) in k_pis_base_final). */
int dpi_point_baseline(dpi_problem p, dpi_net net, const float* tx, int n, void* ws, size_t ws_bytes,
                       void* stream);

/* Label moments over MC indices m in [m_begin, m_end) of M (both multiples of DPI_PATH_BLOCK)
 * with K Euler–Maruyama steps per path.  moments (n, 2, 1+nx) fp32: [0] = sum of per-path
 * contributions, [1] = sum of squares.  Summation order is fixed (pairwise over 64-path
 * blocks), so results are bit-reproducible; ranges aligned to power-of-two block counts
 * combine with dpi_moments_reduce bit-identically to a single call.  Requires
 * dpi_point_baseline (or dpi_sample_points_baseline) of the same n points on the same workspace
 * first: for MLP / zero nets with <= 64 path blocks the label reduce runs inside the path launch,
 * counting blocks on per-point tickets the baseline zeroes (and the last block resets), and the
 * call fails with DPI_ERR_ARG on a workspace that had no such baseline enqueued. */
int dpi_label_moments(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                      uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                      void* ws, size_t ws_bytes, void* stream);

/* Optional first half of dpi_label_moments, for pipelining consecutive batches: the stages that
 * need no network evaluation of this batch's paths and can therefore run on a side stream while the
 * previous batch's network work still occupies the GPU.  For a PISGradNet net (non-TD estimators)
 * that is the first path chunk's Philox + K-step Euler-Maruyama rollout and the baseline rows
 * (data.py:471-527, 899-926 up to the network call); for the fused-kernel nets it is a no-op.  Same
 * arguments as dpi_label_moments (after dpi_point_baseline on the same workspace); the matching
 * dpi_label_moments call then passes flags | DPI_PREPARED.  The library records the prepare
 * call's arguments per workspace (host side); a DPI_PREPARED call whose arguments (points pointer,
 * n, M, K, seed, epoch, point_base, MC range, flags, workspace size) differ, or that has no prepare
 * on its workspace, fails with DPI_ERR_ARG.  Each prepare is consumed by one prepared call. */
int dpi_label_prepare(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                      uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, void* ws,
                      size_t ws_bytes, void* stream);

/* dpi_label_moments over all of [0, M) with the labels finalized by the same block-reduce launch
 * (y as dpi_label_finalize): one launch less for a single-rank caller.  flags may include
 * DPI_PREPARED. */
int dpi_label_moments_finalize(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                               uint32_t epoch, uint32_t point_base, int flags, float sample_bound, float* y,
                               float* moments, void* ws, size_t ws_bytes, void* stream);

/* parts: (n_parts, n, 2, 1+nx) -> out (n, 2, 1+nx) with the same pairwise tree as
 * dpi_label_moments' block sum.  `parts` is read only. */
int dpi_moments_reduce(float* parts, int n_parts, int n, int nx, float* out, void* stream);

/* y (n, 1+nx) = moments[:,0]/M + (g(x), 0...) [if DPI_TERMINAL], clipped to +-sample_bound. */
int dpi_label_finalize(dpi_problem p, const float* moments, int n, int M, int flags, float sample_bound,
                       float* y, const void* ws, size_t ws_bytes, void* stream);

/* All of the above for m in [0, M): generate_with_gradients(tx) -> y (n, 1+nx); moments
 * (n, 2, 1+nx) receives the label moments (required). */
int dpi_generate_with_gradients(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K,
                                uint64_t seed, uint32_t epoch, uint32_t point_base, int flags,
                                float sample_bound, float* y, float* moments, void* ws, size_t ws_bytes,
                                void* stream);

/* sample_with_gradients(n): the n points of dpi_sample_points_t (eps, t_factors, point_base as
 * there) into tx (n, 1+nx), then dpi_generate_with_gradients on them — tx, y and moments bitwise
 * those of the two separate calls, and the workspace's baseline that of dpi_point_baseline.
 * First-order Cha / OU labels of MLP and zero networks (no TD, M <= 4096) run as ONE launch: n
 * baseline workgroups ahead of the path workgroups, which draw their point themselves and wait for
 * its baseline (an in-launch hand-off) before the network evaluation; the label reduce runs in the
 * path launch (DPI_FUSED_BASE=0: two launches, the sampling inside the baseline launch).  GBM: two
 * launches; PISGradNet: dpi_sample_points_t + dpi_generate_with_gradients. */
int dpi_sample_with_gradients(dpi_problem p, dpi_net net, int n, int M, int K, uint64_t seed, uint32_t epoch,
                              uint32_t point_base, float eps, int t_factors, int flags, float sample_bound,
                              float* tx, float* y, float* moments, void* ws, size_t ws_bytes, void* stream);

/* dpi_sample_points_t + dpi_point_baseline (tx and the workspace's baseline bitwise those of the
 * two calls), one launch for MLP / zero networks: the first half of dpi_sample_with_gradients. */
int dpi_sample_points_baseline(dpi_problem p, dpi_net net, int n, uint64_t seed, uint32_t epoch, uint32_t point_base,
                               float eps, int t_factors, float* tx, void* ws, size_t ws_bytes, void* stream);

/* Malliavin-weight Hessian labels: replaces
 *   _OnlineDataGenerator.sample_with_gradients_and_hessians (picard/data.py:225-237, after its
 *   draws 1-2) -> OnlineDataGenerator.generate_with_gradients_and_hessians (:1220-1223) =
 *   estimate_terminal_with_gradients_and_hessians_double (:1153-1201) +
 *   estimate_integral_with_gradients_and_hessians_double (:823-897), with the clip of :236.
 * y: (n, 1 + nx + nx*nx) = [u, grad u, Hessian (row-major)], f evaluated with the full Hessian
 * diagonal whatever the problem's SDGD setting (the reference calls get_f without the SDGD
 * context there).  GBMEquationComplexExact problems (the reference asserts
 * SimpleDiffusionEquationWithHessian), MLP (width <= 64) or zero networks; M % 64 == 0, M <= 65536.
 * Noise: the first-order streams plus N1 = tag DPI_TAG_HTERM, N2 = tag DPI_TAG_HINT (k = 0).
 * ws >= dpi_workspace_bytes_hessians(p, net, n, M). */
size_t dpi_workspace_bytes_hessians(dpi_problem p, dpi_net net, int n, int M);
/* ws of a dpi_label_prepare + DPI_PREPARED dpi_label_moments_hessians pair (GBM MLP nets: the
 * terminal / integral noise sums staged by the prepare, as for first-order labels); ABI 7. */
size_t dpi_workspace_bytes_hessians_prepared(dpi_problem p, dpi_net net, int n, int M);

/* The library keeps host-side records per workspace address: the fused reduce's "a baseline of n
 * points was enqueued here" tag (dpi_point_baseline / dpi_sample_points_baseline, checked by
 * dpi_label_moments) and an unconsumed dpi_label_prepare.  A caller that frees a workspace and
 * allocates another (a caching allocator may return the same address) calls this on the new range
 * [ws, ws + ws_bytes) so the old records cannot vouch for it.  Host only, no device work; ABI 7. */
int dpi_workspace_forget(const void* ws, size_t ws_bytes);

/* Sharding building blocks of the Hessian labels (the first-order dpi_label_moments pattern):
 * after dpi_point_baseline, the sums over m in [m_begin, m_end) of the value/gradient
 * contributions and their squares (moments (n, 2, 1+nx)) and of the Hessian contributions
 * (hessian_sums (n, nx*nx)); dpi_label_finalize_hessians turns (possibly rank-reduced) sums into
 * y (n, 1 + nx + nx*nx) = clip(sums / M [+ g(x)]).  flags (ABI 4): DPI_TERMINAL and/or DPI_INTEGRAL
 * select the estimators (terminal: value/gradient + N1 Hessian term and its identity part, + g(x) at
 * finalize; integral: the same for f and N2), so n_estimate_terminal != n_estimate_integral runs as
 * a DPI_TERMINAL pass over M_T paths plus a DPI_INTEGRAL pass over M_I paths, summed
 * (picard/data.py:1164 vs :845).  flags may include DPI_PREPARED (ABI 7): a dpi_label_prepare with the
 * same arguments ran on this workspace (sized by dpi_workspace_bytes_hessians_prepared), and the
 * labels are bitwise those of the unprepared call. */
int dpi_label_moments_hessians(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                               uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                               float* hessian_sums, void* ws, size_t ws_bytes, void* stream);
int dpi_label_finalize_hessians(dpi_problem p, const float* moments, const float* hessian_sums, int n, int M, int flags,
                                float sample_bound, float* y, void* ws, size_t ws_bytes, void* stream);

/* out[j] = canonical tree sum over the n_parts rows of parts (n_parts, len) (the rank-reduce of
 * dpi_moments_reduce for any flat length; parts is read-only). */
int dpi_sums_reduce(const float* parts, int n_parts, size_t len, float* out, void* stream);
int dpi_generate_with_gradients_and_hessians(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K,
                                             uint64_t seed, uint32_t epoch, uint32_t point_base,
                                             float sample_bound, float* y, void* ws, size_t ws_bytes,
                                             void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DPI_H_ */
