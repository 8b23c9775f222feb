/*
 * fdcn.h -- C ABI of the MI355X Crank-Nicolson finite-difference engine.
 *
 * TEST/PRODUCT BOUNDARY.  This header is the drop-in seam for the reference's
 * time-stepping hot path.  The reference (rwx-gigaba-sonwabo/Finite_Difference)
 * is pure Python and has no FFI; its seam is a pair of Python methods, which
 * the entry points below replace one-for-one:
 *
 *   fdcn_cn_batch  <- DiscreteBarrierFDMPricer._solve_grid
 *                       (discrete_barrier_fdm_pricer.py:442-547)
 *                     DiscreteBarrierCrankNicolsonLog._solve_grid
 *                       (discrete_barrier_fdm_pricer_cn.py:219-302)
 *                     KO projection _apply_KO_projection (…pricer.py:413-440,
 *                       …_cn.py:199-213) is fused in.
 *   fdcn_it_batch  <- AmericanFDMPricer._solve_segment
 *                       (fd_american_equity.py:559-726), Ikonen-Toivanen.
 *
 * The Python side (finite_difference_amd/capi.py) binds them with ctypes; the
 * binding a maintainer would add to the reference is in INTEGRATION.md.
 *
 * Conventions
 *   - A launch solves B independent scenarios ("solves") that share n_nodes,
 *     n_time and n_ranna.  Everything else is per scenario.
 *   - n_nodes counts ALL grid nodes including the two Dirichlet nodes:
 *     node 0 (S_min side), node n_nodes-1 (S_max side), interior 1..n_nodes-2.
 *     The production barrier engine's top-node drop (…pricer.py:449,543) is
 *     expressed by the caller passing n_nodes = N_s and v_init = payoff[0:N_s];
 *     the kernel has no quirk flag.  5 <= n_nodes <= 40962 (16 wavefronts
 *     x 64 lanes x 40 nodes + 2) is accepted: grids whose interior does not
 *     fill the lanes are padded with inactive lanes, 5-11-node grids run two
 *     nodes per lane; larger grids fail with FDCN_EINVAL.
 *   - Step m = 0..n_time-1 advances tau to tau_m = tau0 + (m+1)*dt and uses
 *     theta = 1 for m < n_ranna (Rannacher), 0.5 afterwards.
 *   - All arrays are C-contiguous, row-major, fp64 / int32.  The caller owns
 *     every buffer; nothing is retained after return.
 *   - Return 0 on success, a negative FDCN_E* code on failure; the message is
 *     available from fdcn_last_error() (thread-local).  Never aborts.
 */
#ifndef FDCN_H
#define FDCN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: fdcn_session_host_buffer, the diagnostics of include/fdcn_diag.h for the
 * spot-space kernels (fdcn_vc_force_variant / _variant_name / _forms) and the
 * fdcn_vc workspace contract (+16 doubles per scenario) changed the exported
 * surface after 4 */
#define FDCN_ABI_VERSION 5

/* ---- per-scenario fp64 parameters: params[b*FDCN_NPARAM + k] ---------- */
enum fdcn_param {
  FDCN_P_DT = 0,  /* time step (years)                                       */
  FDCN_P_A,       /* operator coefficient of V_{j-1}: alpha - beta_adv       */
  FDCN_P_C,       /* operator coefficient of V_{j+1}: alpha + beta_adv       */
  FDCN_P_BC,      /* operator coefficient of V_j:     -2*alpha - r           */
  FDCN_P_TAU0,    /* tau at the start of this segment                        */
  FDCN_P_LO_C0,   /* lower Dirichlet value, see FDCN_I_LO_FORM               */
  FDCN_P_LO_E0,
  FDCN_P_LO_C1,
  FDCN_P_LO_E1,
  FDCN_P_HI_C0,   /* upper Dirichlet value, see FDCN_I_HI_FORM               */
  FDCN_P_HI_E0,
  FDCN_P_HI_C1,
  FDCN_P_HI_E1,
  FDCN_NPARAM
};

/* ---- per-scenario int32 parameters: iparams[b*FDCN_NIPARAM + k] ------- */
enum fdcn_iparam {
  FDCN_I_LO_FORM = 0, /* 0: c0*exp(e0*tau) + c1*exp(e1*tau)
                         1: ((c0*exp(e0*tau))*c1)*exp(e1*tau)  (…pricer.py:391) */
  FDCN_I_HI_FORM,
  FDCN_I_KO_LO,       /* monitor steps set V_j = rebate for j <= KO_LO (-1: none) */
  FDCN_I_KO_HI,       /* … and for j >= KO_HI (>= n_nodes: none)                 */
  FDCN_I_MON_START,   /* offset of this scenario's entries in mon_step/mon_rebate */
  FDCN_I_MON_COUNT,   /* number of entries: strictly increasing, values in 1..n_time
                         (the host entry points return FDCN_EINVAL otherwise; the
                         _dev kernels skip entries < 1 and entries not above the
                         previous one, as the oracle does) */
  FDCN_I_TAU_MODE,    /* tau after step m: 0: tau0 + (m+1)*dt (…pricer.py:519).
                         1: tau accumulated by repeated tau = tau + dt, as
                         fd_american_equity.py:664-724 does.  Both are honoured on
                         the device; any other value is FDCN_EINVAL (host entry
                         points) / treated as 0 (_dev). */
  FDCN_NIPARAM
};

/* error codes */
#define FDCN_OK 0
#define FDCN_EINVAL (-1)   /* bad argument / unsupported size                  */
#define FDCN_EHIP (-2)     /* HIP runtime error                                */
#define FDCN_ENODEV (-3)   /* no usable gfx950 device                          */
#define FDCN_ENOMEM (-4)   /* device allocation failed                         */

/* ---- host-pointer entry points (copy in, solve, copy out) ------------- */

/* European solve with knock-out projection on monitor steps.
 *   v_init     [B][n_nodes]  value vector at tau0 (payoff for a full solve)
 *   mon_step   [n_mon]       step numbers m+1 at which to project (per scenario
 *                            a sorted run addressed by MON_START/MON_COUNT)
 *   mon_rebate [n_mon]       value written into knocked-out nodes at that step
 *   v_out      [B][n_nodes]  value vector at tau0 + n_time*dt
 */
int fdcn_cn_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams,
                  const double* v_init,
                  int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                  double* v_out);

/* American solve with Ikonen-Toivanen early exercise against payoff.
 *   payoff [B][n_nodes]  exercise value phi_j (only interior nodes are used);
 *   lambda starts at 0 in every call, as _solve_segment does (…equity.py:661).
 *   KO fields of iparams must be -1 / >= n_nodes and MON_COUNT 0.
 */
int fdcn_it_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams,
                  const double* v_init, const double* payoff,
                  double* v_out);

/* Threading: the host-pointer entry points are reentrant.  Each calling
 * thread gets its own non-blocking HIP stream on the current device
 * (fdcn_select_device / hipSetDevice), device buffers come stream-ordered
 * from the device's memory pool, and the call waits on its own stream only
 * (never a device-wide synchronisation).  The stream is created on a thread's
 * first call and kept for the thread's lifetime (it is not released when the
 * thread exits): issue calls from long-lived threads (a fixed pool), not from
 * a thread created per call. */

/* ---- device-pointer entry points (all pointers are device memory) ----- */
/* `stream` is a hipStream_t (NULL = default stream); the call is
 * asynchronous on that stream and performs no host sync.  Inputs and output
 * may alias (v_out == v_init) only if `v_init` is not needed afterwards.
 * `k_cap` bounds the boundary-layer correction table (see fdcn_sm_extent);
 * pass the value fdcn_sm_extent returns for the same params.  A scenario whose
 * extent exceeds k_cap gets NaN outputs (loud, never silently wrong).
 * `workspace` is device scratch of `workspace_bytes` bytes, at least
 * B * ws_bytes_per_scen as reported by fdcn_plan for the SAME B, n_nodes,
 * n_time, mode and k_cap (the kernel variant, and with it the workspace,
 * depends on B: small batches spread a scenario over more waves).  A smaller
 * (or negative) workspace_bytes is rejected with FDCN_EINVAL.  The Dirichlet
 * values of every step are evaluated there once per launch.  With NULL the
 * library allocates it stream-ordered (hipMallocAsync/hipFreeAsync on
 * `stream`, workspace_bytes ignored); pass a buffer to keep the call
 * allocation-free (e.g. for hipGraph capture). */
int fdcn_cn_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams,
                      const double* v_init,
                      int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                      double* v_out, int32_t k_cap, double* workspace,
                      int64_t workspace_bytes, void* stream);

int fdcn_it_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams,
                      const double* v_init, const double* payoff,
                      double* v_out, int32_t k_cap, double* workspace,
                      int64_t workspace_bytes, void* stream);

/* ---- device-resident sessions (finite_difference_amd/csrc/fdcn_session.hip)
 * A session keeps solve outputs in HBM as numbered "slots" (one value vector
 * each) and chains marches, dividend jumps and the Greeks epilogue on the
 * device; only what the caller asks for comes back.  It replaces the host
 * round trips of
 *   _solve_grid -> _interp_price / _delta_gamma_from_grid / greeks
 *     (discrete_barrier_fdm_pricer.py:629-646, :883-904, :949-978;
 *      discrete_barrier_fdm_pricer_cn.py:429-466; fd_american_equity.py:855-1068)
 *   _solve_segment -> _apply_dividend_jump -> _solve_segment
 *     (fd_american_equity.py:479-553, :732-772, :825-843).
 * A session belongs to the thread's current device (fdcn_select_device) and is
 * not thread-safe; use one per thread.  Marches and jumps are asynchronous
 * (independent ones overlap on up to 4 session streams); greeks and fetch wait
 * for their inputs and return results.  Host arrays are staged through pinned
 * memory before a call returns.  After an error, destroy the session. */
typedef struct fdcn_session fdcn_session;
int fdcn_session_create(fdcn_session** out);
int fdcn_session_destroy(fdcn_session* s);
int fdcn_session_slots(const fdcn_session* s);  /* slots created so far */

/* `bytes` of pinned host memory owned by the session, valid until
 * fdcn_session_destroy (256-byte aligned).  A caller that builds a march's
 * payoff / v_init directly in it (the whole-file plans: 100-400 MB) spares
 * the staging copy: fdcn_session_march copies such an array to the device
 * from where it lies, asynchronously, so its contents must stay unchanged
 * until the session's next synchronising call (fdcn_session_greeks /
 * fdcn_session_fetch) or its destruction. */
int fdcn_session_host_buffer(fdcn_session* s, int64_t bytes, void** out);

/* One batched march (the fdcn_cn_batch / fdcn_it_batch plan; it != 0 for
 * Ikonen-Toivanen).  Initial vectors come from the host (v_init [B][n_nodes])
 * or from earlier slots (v_init_slots [B]); pass exactly one.  An IT march
 * may pass its payoff pointer as v_init (the array is copied once).  Host
 * arrays are staged through pinned memory before the call returns, except a
 * payoff / v_init inside an fdcn_session_host_buffer region (read later, by
 * the asynchronous copy).  The B outputs become new slots, numbers written
 * to out_slots [B]. */
int fdcn_session_march(fdcn_session* s, int32_t it, int32_t B, int32_t n_nodes, int32_t n_time,
                       int32_t n_ranna, const double* params, const int32_t* iparams,
                       const double* v_init, const int32_t* v_init_slots, const double* payoff,
                       int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                       int32_t* out_slots);

/* fdcn_dividend_jump of B slots on the device: s_nodes [B][n_nodes] (host),
 * cash_div [B], strike_call [B] (< 0 for puts); results into new slots.
 * Bit-identical to fdcn_dividend_jump on the same inputs. */
int fdcn_session_dividend_jump(fdcn_session* s, int32_t B, int32_t n_nodes,
                               const int32_t* in_slots, const double* s_nodes,
                               const double* cash_div, const double* strike_call,
                               int32_t* out_slots);

/* Greeks epilogue: T trades, trade t of kind[t] reads readouts first[t] ..
 * first[t]+k-1 (k per kind below) and writes out[t][FDCN_GK_NOUT] =
 * price, delta, gamma, vega, theta, aux.  Readout r:
 *   rint[r][FDCN_GK_NRINT] = slot, interp case (0: between ilo and ilo+1,
 *                            1: V[0], 2: V[ilo]), ilo, idx, dg mode (0 none,
 *                            1 three-point at idx, 2 cubic through idx-1..idx+2)
 *   rdbl[r][FDCN_GK_NRDBL] = S_interp, s[ilo], s[ilo+1], S_dg, s[idx-1],
 *                            s[idx], s[idx+1], s[idx+2]
 * Node positions come from the host (bisection on its grids, as the pricers
 * do); the formulas keep the reference's operation order.  Kinds, params:
 *   FDCN_GK_BARRIER  2 readouts (base: interp + 3-point; sigma-bumped: interp)
 *                    P = sigma, spot, carry, div_yield, r, dv   (…pricer.py:883-904)
 *   FDCN_GK_CNLOG    3 readouts (base, sigma+dv, sigma-dv)
 *                    P = sigma, S0, b, r, dv                    (…_cn.py:429-466)
 *   FDCN_GK_AMERICAN 7 readouts (N and 2N: interp + cubic; sigma +h, -h, +2h,
 *                    -2h at N; N_t = 2 num_space_nodes) P = sigma, spot, carry, r, h;
 *                    aux = price_log2's Richardson       (fd_american_equity.py:925-1068)
 *   FDCN_GK_READOUT  1 readout: price, delta, gamma of that vector */
#define FDCN_GK_BARRIER 0
#define FDCN_GK_CNLOG 1
#define FDCN_GK_AMERICAN 2
#define FDCN_GK_READOUT 3
#define FDCN_GK_NPARAM 8
#define FDCN_GK_NRINT 5
#define FDCN_GK_NRDBL 8
#define FDCN_GK_NOUT 6
int fdcn_session_greeks(fdcn_session* s, int32_t T, const int32_t* kind, const int32_t* first,
                        const double* tparams, int32_t R, const int32_t* rint,
                        const double* rdbl, double* out);

/* Copy n slots (each n_nodes long) back to out [n][n_nodes]. */
int fdcn_session_fetch(fdcn_session* s, int32_t n, const int32_t* slots, int32_t n_nodes,
                       double* out);

/* ---- launch planning / introspection ---------------------------------- */
/* Writes the kernel geometry a launch of B scenarios uses: waves per
 * scenario, nodes per lane, scenarios per workgroup (2: the paired flavour,
 * two scenarios per wavefront, used for large batches of <= 256-node grids),
 * LDS bytes per workgroup, and the device workspace the _dev entry points
 * need per scenario.  Batches too small to fill the chip spread each scenario
 * over more waves, so the plan depends on B; call it with the B you launch.
 * Any output pointer may be NULL.  Returns FDCN_EINVAL if the size is
 * unsupported. */
int fdcn_plan(int32_t B, int32_t n_nodes, int32_t n_time, int32_t it_mode, int32_t k_cap,
              int32_t* waves, int32_t* npt, int32_t* scen_per_block, int32_t* lds_bytes,
              int64_t* ws_bytes_per_scen);

/* Extent (nodes) of the Sherman-Morrison boundary-layer correction needed by
 * the scenarios in `params` (host memory): the largest k such that the
 * correction at interior node k is above 1e-18 of its value at node 0, over
 * both theta values used by the launch.  Returns a value in [1, n_nodes-2],
 * or a negative FDCN_E* code. */
int fdcn_sm_extent(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                   const double* params);

/* ---- spot-space CN with per-row coefficients ---------------------------
 * fdcn_vc_batch <- DiscreteBarrierFDMPricer2._solve_pde_backward
 *                    (discrete_barrier_fdm_pricer_2.py:336-428, FIS barrier
 *                    rows and BGK window) and
 *                  DiscreteBarrierFDMPricerAnalytic._cn_stepper
 *                    (discrete_barrier_analytic_pricer.py:384-432).
 * The matrices are tridiagonal with a different row at every node (uniform S
 * grid, sigma^2 S_i^2 terms, the non-symmetric rows at the barrier), constant
 * in time within a phase: phase 0 for steps m < n_ranna (Rannacher), phase 1
 * after.  Step m: rhs_i = a_i V_{i-1} + b_i V_i + c_i V_{i+1} for interior
 * rows, rhs_0 = bnd[m][0], rhs_{n-1} = bnd[m][1]; solve
 * sub_i x_{i-1} + main_i x_i + sup_i x_{i+1} = rhs_i (sub_0 = sup_{n-1} = 0);
 * V = x; then the knock-out projection of the CN ABI (iparams KO_LO / KO_HI,
 * MON_START / MON_COUNT; LO/HI_FORM and TAU_MODE unused, pass 0).
 *   diag [B][2][FDCN_VC_NDIAG][n_nodes]  sub, main, sup, a, b, c per phase
 *   bnd  [B][n_time][2]                  Dirichlet values of rows 0 / n-1
 * The LU factors of each phase are computed once per launch; the march
 * keeps the rows' factored coefficients and V in registers. */
#define FDCN_VC_NDIAG 6
int fdcn_vc_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* diag, const double* bnd, const double* v_init,
                  const int32_t* iparams, int32_t n_mon, const int32_t* mon_step,
                  const double* mon_rebate, double* v_out);
int fdcn_vc_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* diag, const double* bnd, const double* v_init,
                      const int32_t* iparams, int32_t n_mon, const int32_t* mon_step,
                      const double* mon_rebate, double* v_out, double* workspace,
                      int64_t workspace_bytes, void* stream);
/* geometry of a fdcn_vc launch of B scenarios (depends on B): waves per
 * scenario, nodes per lane, device workspace per scenario (bytes) */
int fdcn_vc_plan(int32_t B, int32_t n_nodes, int32_t* waves, int32_t* npt,
                 int64_t* ws_bytes_per_scen);

/* ---- batched closed-form barrier engines (one thread per contract) ------ */
/* Reiner-Rubinstein single continuous barrier with cash rebate and barrier
 * status; replaces BarrierEngine(s,b,r,t,x,sigma,h,optionflag,directionflag,
 * in_out_flag,k,barrier_status,rebate_timing_in,rebate_timing_out).price() /
 * .vanilla() (barrier_engine.py:38-44, 189) for B contracts at once.
 *   params[B][FDCN_RR_NPARAM] = s, b, r, t, x (strike), sigma, h (barrier), k (rebate)
 *   flags [B][FDCN_RR_NFLAG]  = option (0 call, 1 put), direction (0 up, 1 down),
 *                               in/out (0 in, 1 out), status (0 not crossed, 1 crossed),
 *                               rebate timing bits (1: knock-in rebate paid at hit,
 *                               2: knock-out rebate paid at expiry; defaults 0)
 *   price[B], vanilla[B] (the A factor).  */
#define FDCN_RR_NPARAM 8
#define FDCN_RR_NFLAG 5
int fdcn_rr_barrier_batch(int32_t B, const double* params, const int32_t* flags,
                          double* price, double* vanilla);
int fdcn_rr_barrier_batch_dev(int32_t B, const double* params, const int32_t* flags,
                              double* price, double* vanilla, void* stream);

/* Double knock-out / knock-in (Ikeda-Kunitomo / Douady series, n = -m..m);
 * replaces DoubleBarrier(S,X,L,U,sigma,callflag,inflag,m).price(b,r,T)
 * (double _barrier.py:33-134).
 *   params[B][FDCN_DB_NPARAM] = S, X, L, U, sigma, b, r, T
 *   flags [B][FDCN_DB_NFLAG]  = option (0 call, 1 put), in/out (0 in, 1 out),
 *                               corrected put (0: the reference's alpha = 1, :95)
 *   price[B]. */
#define FDCN_DB_NPARAM 8
#define FDCN_DB_NFLAG 3
int fdcn_double_barrier_batch(int32_t B, int32_t m, const double* params,
                              const int32_t* flags, double* price);
int fdcn_double_barrier_batch_dev(int32_t B, int32_t m, const double* params,
                                  const int32_t* flags, double* price, void* stream);

/* ---- host-side plan helpers (no device) -------------------------------- */
/* Uniform log grid of the pricers' _build_log_grid
 * (discrete_barrier_fdm_pricer.py:342-364, fd_american_equity.py:363-384):
 *   x[i] = x_min + (double)i * dx,   s[i] = exp(x[i]),   i = 0..n
 * with the C library's exp (the one CPython's math.exp calls), so the nodes
 * are bit-identical to the reference's list comprehensions.  x may be NULL.
 * Returns FDCN_OK or FDCN_EINVAL (n < 0, s NULL). */
int fdcn_log_grid(double x_min, double dx, int32_t n, double* x, double* s);

/* The accumulated tau of FDCN_I_TAU_MODE = 1, as the kernels evaluate it:
 * tau[m] = tau after step m of `tau = tau + dt` starting from tau0
 * (fd_american_equity.py:664-724), m = 0..n-1.  Bit-identical to the serial
 * adds; the device evaluates it in constant-increment runs (one per binade
 * plus single steps at binade crossings and rounding ties) instead of n
 * dependent adds.  fdcn_tau_runs returns the number of runs.  Host only. */
int fdcn_tau_sequence(double tau0, double dt, int32_t n, double* tau);
int fdcn_tau_runs(double tau0, double dt, int32_t n);

/* Discrete-dividend jump between two American segments
 * (AmericanFDMPricer._apply_dividend_jump, fd_american_equity.py:732-772,
 * with the natural cubic spline of :479-553):
 *   q_i = s_i - cash_div,  V_out[i] = v[0] if q_i <= s[0], v[n-1] if q_i >= s[n-1],
 *   else spline(q_i);  calls (strike_call >= 0): V_out[i] = max(V_out[i], max(s_i - K, 0)).
 * Same operation order as the reference, so the result is bit-identical.
 * s strictly increasing, n >= 2.  Host only (no device). */
int fdcn_dividend_jump(int32_t n, const double* s, const double* v, double cash_div,
                       double strike_call, double* v_out);

/* ---- whole-file plan builder (finite_difference_amd/csrc/fdcn_plan.hip) --
 * The discrete-barrier scenario runner's per-row work (run_config_scenarios.py
 * :137-195 over DiscreteBarrierFDMPricer: choose_grid_parameters, the log
 * grid, payoff, boundaries, knock-out thresholds, monitoring rebates and the
 * operator coefficients of the base and sigma-bumped solves, …pricer.py
 * :270-547, :883-904) for R rows at once, with libm's exp/log/sqrt and the
 * reference's operation order: the plan arrays are bit-identical to the
 * per-row facade's.  Output solve q = 2*row + (0 base, 1 bumped by dv_sigma):
 *   params [2R][FDCN_NPARAM], iparams [2R][FDCN_NIPARAM] (monitor run q*n_mon),
 *   v_init [2R][N] (N = the grid's N_s, the march's n_nodes: *n_nodes_out),
 *   mon_rebate [2R][n_mon] (steps: mon_k, shared by all rows),
 *   rint / rdbl [2R] readouts in fdcn_session_greeks layout (slot field = q),
 *   tparams [R][FDCN_GK_NPARAM] (FDCN_GK_BARRIER, readouts 2*row, 2*row+1).
 * v_init holds 2R * n_nodes_cap doubles; FDCN_EINVAL (nothing written) if
 * N > n_nodes_cap or the rows' N differ (parity mode N = ceil(k_tail n_time)
 * up to rounding, explicit mode N = n_space).  grid_mode 0 parity, 1 explicit. */
#define FDCN_BP_NROW 10
enum fdcn_bp_row {
  FDCN_BP_SPOT = 0, FDCN_BP_STRIKE, FDCN_BP_SIGMA, FDCN_BP_LO, FDCN_BP_UP,
  FDCN_BP_CARRY, FDCN_BP_DIVY, FDCN_BP_DISC, FDCN_BP_PV, FDCN_BP_REBATE
};
#define FDCN_BP_NFLAG 4
enum fdcn_bp_flag {
  FDCN_BP_PUT = 0, /* 1 for puts */
  FDCN_BP_KO,      /* 1 down-and-out, 2 up-and-out, 3 double-out (knock-ins: their twin) */
  FDCN_BP_HAS_LO, FDCN_BP_HAS_UP
};
int fdcn_barrier_plan(int32_t R, const double* row, const int32_t* rflag, double T,
                      int32_t n_space, int32_t n_time, int32_t grid_mode, int32_t n_nodes_cap,
                      double k_tail, double dv_sigma, int32_t rebate_at_hit, int32_t n_mon,
                      const int32_t* mon_k, double* params, int32_t* iparams, double* v_init,
                      double* mon_rebate, int32_t* rint, double* rdbl, double* tparams,
                      int32_t* n_nodes_out);
/* American counterpart (run_american_scenarios.py:209-277 over
 * AmericanFDMPricer, fd_american_equity.py:340-448, :855-907): the log grid
 * of one (row, sigma) job each -- band around sqrt(S K), uniform log nodes,
 * spot and strike snapped to the nearest node, payoff with the snapped
 * strike, operator coefficients (q = 0), Dirichlet forms, TAU_MODE 1 -- and
 * its two readouts at the snapped spot.  n_space + 1 nodes per job.
 *   job [J][FDCN_AP_NJOB] = spot, strike, sigma, carry, r;  call [J] (1 call, 0 put)
 *   params [J][FDCN_NPARAM]: DT and TAU0 left 0 (set per segment by the caller)
 *   iparams [J][FDCN_NIPARAM], payoff [J][n_space+1], s_nodes [J][n_space+1]
 *   (may be NULL), rint / rdbl [2J]: row 2q the interpolation readout, row
 *   2q+1 with the cubic Delta/Gamma (fdcn_session_greeks layout, slot = q),
 *   gout [J][FDCN_AP_NOUT] = snapped spot, snapped strike, dx, spot index. */
#define FDCN_AP_NJOB 5
enum fdcn_ap_job { FDCN_AP_SPOT = 0, FDCN_AP_STRIKE, FDCN_AP_SIGMA, FDCN_AP_CARRY, FDCN_AP_DISC };
#define FDCN_AP_NOUT 4
int fdcn_american_plan(int32_t J, const double* job, const int32_t* call, int32_t n_space,
                       double s_max_mult, double T, double* params, int32_t* iparams,
                       double* payoff, double* s_nodes, int32_t* rint, double* rdbl,
                       double* gout);
/* y = exp(x) (op 0), log(x) (1), sqrt(x) (2), pow(x, 2.0) (3) elementwise with
 * the C library (the functions CPython's math module and float ** call). */
int fdcn_vmath(int32_t op, int64_t n, const double* x, double* y);

const char* fdcn_last_error(void);
int fdcn_device_count(void);   /* gfx950 devices visible; 0 if none          */
/* The HIP ordinals of the visible gfx950 devices, ascending, into ord[cap];
 * returns how many there are (may exceed cap), 0 if none.  On a host with
 * other GPUs too, local rank k binds ord[k], not HIP ordinal k. */
int fdcn_device_ordinals(int32_t* ord, int32_t cap);
int fdcn_abi_version(void);    /* FDCN_ABI_VERSION                           */
/* Make `ordinal` the calling thread's current HIP device (hipSetDevice): the
 * host-pointer entry points run there.  One process per GPU calls it once
 * with its local rank.  Returns FDCN_OK or FDCN_EINVAL / FDCN_EHIP. */
int fdcn_select_device(int32_t ordinal);
int fdcn_current_device(void); /* the calling thread's device, or < 0 on error */

#ifdef __cplusplus
}
#endif

#endif /* FDCN_H */
