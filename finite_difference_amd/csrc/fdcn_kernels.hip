// fdcn_kernels.hip -- MI355X (gfx950) kernels + C ABI for the batched
// Crank-Nicolson / Rannacher / Ikonen-Toivanen time march in log-spot.
//
// Replaces, per time step, the pure-Python loops of
//   DiscreteBarrierFDMPricer._solve_grid   discrete_barrier_fdm_pricer.py:517-546
//   DiscreteBarrierCrankNicolsonLog._solve_grid   _cn.py:278-300
//   AmericanFDMPricer._solve_segment       fd_american_equity.py:665-724
//
// Mapping.  One scenario (one independent solve) is owned by W wavefronts
// (W = 1 for throughput batches).  Lane t of the scenario owns a contiguous
// chunk of NPT interior nodes held in VGPRs for the whole march; nothing of
// the value vector touches HBM between the initial load and the final store.
//
// Per step (theta-scheme, constant coefficients):
//   1. rhs = B V (3-point stencil; neighbours by wavefront shuffles, LDS
//      across waves), Dirichlet terms folded into the first/last node.
//   2. Solve A x = rhs where A is tridiagonal Toeplitz.  A = L U + k e0 e0^T,
//      with L = I + q S, U = r I + u S^T the *converged* LU factors (r the
//      larger root of r^2 - A_C r + A_L A_U = 0, uniform scalars), so
//        forward  w_i = rhs_i/r + fm * w_{i-1}       fm = -A_L/r
//        backward y_i = w_i     + bm * y_{i+1}       bm = -A_U/r
//      are first-order affine recurrences: each lane runs its chunk with a
//      zero carry, a Hillis-Steele shuffle scan (window products of fm / bm
//      precomputed per lane) gives every chunk its true carry, and the chunk
//      is re-run with it.  The rank-1 term k e0 e0^T (the first-row
//      difference between A and L U) is removed exactly by Sherman-Morrison:
//      x = y - (k y_0 / (1 + k z_0)) z,  z = (L U)^-1 e0,
//      with z tabulated once per theta in LDS; |z_i| decays like |fm|^i, so
//      only the first K nodes (K = extent where it drops below 1e-18 z_0)
//      are touched.  This is the reference's Thomas solve in exact
//      arithmetic (discrete_barrier_fdm_pricer.py:487-509), reassociated.
//   3. Write Dirichlet values, then knock-out projection on monitor steps
//      (integer node thresholds) or the Ikonen-Toivanen update (lambda and
//      the payoff in VGPR/LDS).
//
// Chunking: n_int = n_nodes - 2 interior nodes over L_act = ceil(n_int/NPT)
// lanes; the first L_short = L_act*NPT - n_int lanes own NPT-1 nodes and carry
// a "phantom" last slot that is a pass-through in both recurrences.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "../../include/fdcn.h"

namespace {

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ double uni(double x) {
  // make a wave-uniform double an SGPR pair
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffull));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double read_lane(double x, int l) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffull), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int uni_i(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ double shfl_up1(double x, int d) { return __shfl_up(x, (unsigned)d, 64); }
__device__ __forceinline__ double shfl_dn1(double x, int d) { return __shfl_down(x, (unsigned)d, 64); }

__device__ __forceinline__ double bnd_eval(int form, double c0, double e0, double c1, double e1,
                                           double tau) {
  if (form == 1) return c0 * exp(e0 * tau) * c1 * exp(e1 * tau);
  return c0 * exp(e0 * tau) + c1 * exp(e1 * tau);
}

// Uniform per-phase (per theta) constants.
struct Phase {
  double bl, bc, bu;  // B_L/r, B_C/r, B_U/r
  double fm, bm;      // -A_L/r, -A_U/r
  double dtr;         // dt/r (Ikonen-Toivanen rhs term)
  double inv_r;
  double kappa;       // A_L A_U / r
};

__device__ __forceinline__ Phase make_phase(double theta, double dt, double a, double c,
                                            double bcoef) {
  // build_matrices(theta), discrete_barrier_fdm_pricer.py:475-484
  const double AL = -theta * dt * a;
  const double AC = 1.0 - theta * dt * bcoef;
  const double AU = -theta * dt * c;
  const double BL = (1.0 - theta) * dt * a;
  const double BC = 1.0 + (1.0 - theta) * dt * bcoef;
  const double BU = (1.0 - theta) * dt * c;
  const double disc = AC * AC - 4.0 * AL * AU;
  const double r = 0.5 * (AC + sqrt(disc));
  Phase p;
  p.inv_r = 1.0 / r;
  p.bl = BL * p.inv_r;
  p.bc = BC * p.inv_r;
  p.bu = BU * p.inv_r;
  p.fm = -AL * p.inv_r;
  p.bm = -AU * p.inv_r;
  p.dtr = dt * p.inv_r;
  p.kappa = AL * AU * p.inv_r;
  // wave-uniform: keep in SGPRs
  p.inv_r = uni(p.inv_r);
  p.bl = uni(p.bl);
  p.bc = uni(p.bc);
  p.bu = uni(p.bu);
  p.fm = uni(p.fm);
  p.bm = uni(p.bm);
  p.dtr = uni(p.dtr);
  p.kappa = uni(p.kappa);
  return p;
}

// Nodes over which the Sherman-Morrison correction is above 1e-18 of its
// value at node 0 (|z_i| ~ |fm|^i |z_0|).  Same formula on host and device.
__host__ __device__ inline int sm_extent(double fm, int n_int) {
  const double afm = fabs(fm);
  if (!(afm > 0.0)) return 1;
  if (!(afm < 1.0)) return n_int;
  const double k = ceil(-41.446531673892822 / log(afm));  // ln(1e-18)
  const double kk = k + 2.0;
  return kk >= (double)n_int ? n_int : (int)kk;
}

// LDS exchange area for W > 1 (per scenario), in doubles.
template <int W>
struct Xch {
  static constexpr int kFirst = 0, kLast = W, kFB = 2 * W, kBC = 3 * W, kFtot = 4 * W,
                       kGtot = 5 * W, kY0 = 6 * W, kSize = 6 * W + 2;
};

template <int NPT>
__device__ __forceinline__ double pow_n(double x, int n) {
  double r = 1.0;
#pragma unroll
  for (int i = 0; i < NPT; ++i)
    if (i < n) r *= x;
  return r;
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
struct KArgs {
  int B, n_nodes, n_time, n_ranna, n_mon, lz;
  int z_lds;    // SM table in LDS (1) or in the global workspace zg (0)
  int phi_lds;  // IT payoff staged in LDS (1) or read from `payoff` (0)
  double* zg;   // [B][2][NPT][lz] when !z_lds
  const double* params;
  const int32_t* iparams;
  const double* v_init;
  const double* payoff;
  const int32_t* mon_step;
  const double* mon_rebate;
  double* v_out;
};

template <int IT, int W, int NPT>
struct Geo {
  static constexpr int L = 64 * W;
  static constexpr int SPB = (W == 1) ? 4 : 1;
  static constexpr int kThreads = 64 * W * SPB;
};

// doubles of LDS per scenario
template <int IT, int W, int NPT>
__host__ __device__ inline int lds_doubles_per_scen(int lz, int z_lds, int phi_lds) {
  return (z_lds ? 2 * lz * NPT : 0) + ((IT && phi_lds) ? 64 * W * NPT : 0) +
         (W > 1 ? Xch<W>::kSize : 0);
}

template <int IT, int W, int NPT>
__global__ void __launch_bounds__((64 * W * ((W == 1) ? 4 : 1)))
fdcn_march(KArgs A) {
  constexpr int L = Geo<IT, W, NPT>::L;
  constexpr int SPB = Geo<IT, W, NPT>::SPB;
  extern __shared__ __attribute__((aligned(16))) double lds[];

  const int lane = threadIdx.x & 63;
  const int wave_blk = uni_i(threadIdx.x >> 6);
  const int scen_in_blk = (W == 1) ? wave_blk : 0;
  const int wave = (W == 1) ? 0 : wave_blk;  // wave index within the scenario
  const int scen = uni_i(blockIdx.x * SPB + scen_in_blk);
  if (scen >= A.B) return;  // whole wave(s) of a missing scenario leave together
  const int t = wave * 64 + lane;

  const int n_nodes = A.n_nodes;
  const int n_int = n_nodes - 2;
  const int lz = A.lz;
  const int z_lds = A.z_lds, phi_lds = A.phi_lds;
  double* my = lds + (size_t)scen_in_blk * lds_doubles_per_scen<IT, W, NPT>(lz, z_lds, phi_lds);
  // SM table [2][NPT][lz]: LDS, or this scenario's slice of the global workspace
  double* ztab = z_lds ? my : A.zg + (size_t)scen * 2 * NPT * lz;
  double* phit = my + (z_lds ? 2 * lz * NPT : 0);  // [NPT][L] (IT, phi_lds)
  double* xch = phit + ((IT && phi_lds) ? L * NPT : 0);  // exchange area (W > 1)
  (void)xch;

  const double* P = A.params + (size_t)scen * FDCN_NPARAM;
  const int32_t* I = A.iparams + (size_t)scen * FDCN_NIPARAM;
  const double dt = uni(P[FDCN_P_DT]);
  const double ca = uni(P[FDCN_P_A]);
  const double cc = uni(P[FDCN_P_C]);
  const double cbc = uni(P[FDCN_P_BC]);
  const double tau0 = uni(P[FDCN_P_TAU0]);

  // lane geometry
  const int L_act = (n_int + NPT - 1) / NPT;
  const int L_short = L_act * NPT - n_int;
  const bool active = t < L_act;
  const bool shrt = t < L_short;
  const int s_t = t * NPT - (t < L_short ? t : L_short);  // first interior index

  // ---- per-theta constants: scan window products + SM table -------------
  double FW[6], GW[6];
  double Fpre = 0.0, Gsuf = 0.0, mlast = 0.0, glast = 0.0;
  Phase ph;
  double smc = 0.0;
  double V[NPT];
  double LAM[NPT];
  (void)LAM;

  auto setup_scan = [&](const Phase& p) __attribute__((always_inline)) {
    if constexpr (W > 1) __syncthreads();  // previous readers of Ftot/Gtot are done
    mlast = shrt ? 1.0 : p.fm;
    glast = shrt ? 1.0 : p.bm;
    const int len = shrt ? NPT - 1 : NPT;
    double f = active ? pow_n<NPT>(p.fm, len) : 0.0;
    double g = active ? pow_n<NPT>(p.bm, len) : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      FW[j] = f;
      GW[j] = g;
      const double fo = shfl_up1(f, d);
      const double go = shfl_dn1(g, d);
      f = (lane >= d) ? f * fo : f;
      g = (lane + d < 64) ? g * go : g;
    }
    Fpre = f;
    Gsuf = g;
    if constexpr (W > 1) {
      if (lane == 63) xch[Xch<W>::kFtot + wave] = Fpre;
      if (lane == 0) xch[Xch<W>::kGtot + wave] = Gsuf;
      __syncthreads();
    }
  };

  // forward + backward sweeps on V (rhs/r in, solution out), in place
  auto solve = [&](const Phase& p) __attribute__((always_inline)) {
    // forward pass 1: chunk aggregate with zero carry
    double w = 0.0;
#pragma unroll
    for (int k = 0; k < NPT - 1; ++k) w = fma(p.fm, w, V[k]);
    w = fma(mlast, w, V[NPT - 1]);
    double b = active ? w : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      const double o = shfl_up1(b, d);
      if (lane >= d) b = fma(FW[j], o, b);
    }
    double cw = 0.0;
    if constexpr (W > 1) {
      if (lane == 63) xch[Xch<W>::kFB + wave] = b;
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W - 1; ++v)
        if (v < wave) cw = fma(xch[Xch<W>::kFtot + v], cw, xch[Xch<W>::kFB + v]);
      b = fma(Fpre, cw, b);
    }
    double cin = shfl_up1(b, 1);
    if (lane == 0) cin = cw;
    if (!active) cin = 0.0;
    // forward pass 2
    w = cin;
#pragma unroll
    for (int k = 0; k < NPT - 1; ++k) {
      w = fma(p.fm, w, V[k]);
      V[k] = w;
    }
    w = fma(mlast, w, V[NPT - 1]);
    V[NPT - 1] = shrt ? 0.0 : w;
    // backward pass 1
    double y = V[NPT - 1];  // glast * 0 + V
#pragma unroll
    for (int k = NPT - 2; k >= 0; --k) y = fma(p.bm, y, V[k]);
    double cb = active ? y : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      const double o = shfl_dn1(cb, d);
      if (lane + d < 64) cb = fma(GW[j], o, cb);
    }
    double cwb = 0.0;
    if constexpr (W > 1) {
      if (lane == 0) xch[Xch<W>::kBC + wave] = cb;
      __syncthreads();
#pragma unroll
      for (int v = W - 1; v > 0; --v)
        if (v > wave) cwb = fma(xch[Xch<W>::kGtot + v], cwb, xch[Xch<W>::kBC + v]);
      cb = fma(Gsuf, cwb, cb);
    }
    double cinb = shfl_dn1(cb, 1);
    if (lane == 63) cinb = cwb;
    if (!active) cinb = 0.0;
    // backward pass 2
    y = fma(glast, cinb, V[NPT - 1]);
    V[NPT - 1] = y;
#pragma unroll
    for (int k = NPT - 2; k >= 0; --k) {
      y = fma(p.bm, y, V[k]);
      V[k] = y;
    }
  };

  // broadcast of the solution at interior node 0 (lane 0 of wave 0)
  auto bcast_first = [&](double v0lane) __attribute__((always_inline)) -> double {
    if constexpr (W == 1) {
      return read_lane(v0lane, 0);
    } else {
      if (t == 0) xch[Xch<W>::kY0] = v0lane;
      __syncthreads();
      const double r = xch[Xch<W>::kY0];
      __syncthreads();
      return r;
    }
  };

  // z = (L U)^-1 e0 for one theta; stores table, returns kappa/(1+kappa z0)
  auto build_sm = [&](const Phase& p, int tab) __attribute__((always_inline)) -> double {
#pragma unroll
    for (int k = 0; k < NPT; ++k) V[k] = 0.0;
    if (t == 0) V[0] = p.inv_r;
    solve(p);
    if (t < lz) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) ztab[(tab * NPT + k) * lz + t] = V[k];
    }
    const double z0 = bcast_first(V[0]);
    return uni(p.kappa / (1.0 + p.kappa * z0));
  };

  const bool use_r = A.n_ranna > 0;
  const bool use_c = A.n_ranna < A.n_time;
  const Phase pr = make_phase(1.0, dt, ca, cc, cbc);
  const Phase pc = make_phase(0.5, dt, ca, cc, cbc);
  int kext = 1;
  double smc_r = 0.0, smc_c = 0.0;
  if (use_c) {
    setup_scan(pc);
    smc_c = build_sm(pc, 1);
    kext = max(kext, sm_extent(pc.fm, n_int));
  }
  if (use_r) {
    setup_scan(pr);
    smc_r = build_sm(pr, 0);
    kext = max(kext, sm_extent(pr.fm, n_int));
  }
  // nodes covered by the first lz lanes; a larger extent means the table is
  // too small for this scenario: poison the output (loud, never silently off)
  const int covered = (lz >= L_act) ? n_int : lz * NPT - (lz < L_short ? lz : L_short);
  const bool overflow = kext > covered;

  // ---- load state -------------------------------------------------------
  const double* vin = A.v_init + (size_t)scen * n_nodes;
  double V0 = uni(vin[0]);
  double VN = uni(vin[n_nodes - 1]);
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int node = s_t + 1 + k;
    V[k] = (active && node <= n_int) ? vin[node] : 0.0;
  }
  const double* pin = IT ? A.payoff + (size_t)scen * n_nodes : nullptr;
  if constexpr (IT) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int node = s_t + 1 + k;
      if (phi_lds) phit[k * L + t] = (active && node <= n_int) ? pin[node] : 0.0;
      LAM[k] = 0.0;
    }
  }
  const int lo_form = uni_i(I[FDCN_I_LO_FORM]);
  const int hi_form = uni_i(I[FDCN_I_HI_FORM]);
  const double lc0 = P[FDCN_P_LO_C0], le0 = P[FDCN_P_LO_E0], lc1 = P[FDCN_P_LO_C1],
               le1 = P[FDCN_P_LO_E1];
  const double hc0 = P[FDCN_P_HI_C0], he0 = P[FDCN_P_HI_E0], hc1 = P[FDCN_P_HI_C1],
               he1 = P[FDCN_P_HI_E1];
  const int ko_lo = uni_i(I[FDCN_I_KO_LO]);
  const int ko_hi = uni_i(I[FDCN_I_KO_HI]);
  int mpos = uni_i(I[FDCN_I_MON_START]);
  const int mend = mpos + uni_i(I[FDCN_I_MON_COUNT]);
  int next_mon = (mpos < mend) ? uni_i(A.mon_step[mpos]) : 0x7fffffff;

  if constexpr (W > 1) {
    if (lane == 0) xch[Xch<W>::kFirst + wave] = V[0];
    if (lane == 63) xch[Xch<W>::kLast + wave] = shrt ? V[NPT - 2] : V[NPT - 1];
  }
  // phase for step 0
  if (use_r) {
    ph = pr;
    smc = smc_r;
  } else {
    setup_scan(pc);  // tables built; recompute c-phase window products
    ph = pc;
    smc = smc_c;
  }
  int tab = use_r ? 0 : 1;
  const double inv_dt = uni(1.0 / dt);

  double lo_reg = 0.0, hi_reg = 0.0;
  for (int m = 0; m < A.n_time; ++m) {
    if (m == A.n_ranna && use_r) {  // Rannacher -> Crank-Nicolson
      setup_scan(pc);
      ph = pc;
      smc = smc_c;
      tab = 1;
    }
    if ((m & 63) == 0) {  // Dirichlet values for the next 64 steps, one per lane
      const double tau = tau0 + (double)(m + lane + 1) * dt;
      lo_reg = bnd_eval(lo_form, lc0, le0, lc1, le1, tau);
      hi_reg = bnd_eval(hi_form, hc0, he0, hc1, he1, tau);
    }
    const double lo_new = read_lane(lo_reg, m & 63);
    const double hi_new = read_lane(hi_reg, m & 63);

    // ---- 1. rhs/r ----------------------------------------------------------
    if constexpr (W > 1) __syncthreads();  // halos of the previous step
    const double last_real = shrt ? V[NPT - 2] : V[NPT - 1];
    double left = shfl_up1(last_real, 1);
    double right = shfl_dn1(V[0], 1);
    if constexpr (W > 1) {
      if (lane == 0 && wave > 0) left = xch[Xch<W>::kLast + wave - 1];
      if (lane == 63 && wave < W - 1) right = xch[Xch<W>::kFirst + wave + 1];
    }
    if (t == 0) left = V0;
    if (t == L_act - 1) right = VN;
    if (!active) { left = 0.0; right = 0.0; }
    if (shrt) V[NPT - 1] = right;
    {
      double prev = left;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const double cur = V[k];
        const double nxt = (k < NPT - 1) ? V[k + 1] : right;
        double r = fma(ph.bl, prev, fma(ph.bc, cur, ph.bu * nxt));
        if constexpr (IT) r = fma(ph.dtr, LAM[k], r);
        V[k] = r;
        prev = cur;
      }
    }
    if (t == 0) V[0] = fma(ph.fm, lo_new, V[0]);
    if (t == L_act - 1) V[NPT - 1] = fma(ph.bm, hi_new, V[NPT - 1]);
    if (shrt) V[NPT - 1] = 0.0;

    // ---- 2. tridiagonal solve ---------------------------------------------
    solve(ph);
    {
      const bool need = (W == 1) || (lz > 64) || (wave == 0);
      if (need) {
        double y0;
        if constexpr (W == 1) {
          y0 = read_lane(V[0], 0);
        } else {
          if (lz > 64) {
            y0 = bcast_first(V[0]);
          } else {
            y0 = read_lane(V[0], 0);
          }
        }
        const double g = smc * y0;
        if (t < lz) {
          const double* zt = ztab + tab * NPT * lz;
#pragma unroll
          for (int k = 0; k < NPT; ++k) V[k] = fma(-g, zt[k * lz + t], V[k]);
        }
      }
    }

    // ---- 3. early exercise / boundaries / knock-out ------------------------
    if constexpr (IT) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const double tv = V[k];
        const int node = s_t + 1 + k;
        const double pk = phi_lds ? phit[k * L + t]
                                  : ((active && node <= n_int) ? pin[node] : 0.0);
        const double lam = LAM[k];
        const double cand = fma(-dt, lam, tv);
        V[k] = pk > cand ? pk : cand;
        const double ln = fma(pk - tv, inv_dt, lam);
        LAM[k] = ln < 0.0 ? 0.0 : ln;
      }
      if (shrt) LAM[NPT - 1] = 0.0;
    }
    V0 = lo_new;
    VN = hi_new;
    if (m + 1 == next_mon) {
      const double reb = uni(A.mon_rebate[mpos]);
      if (active) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int node = s_t + 1 + k;
          if (node <= ko_lo || node >= ko_hi) V[k] = reb;
        }
      }
      if (0 <= ko_lo) V0 = reb;
      if (n_nodes - 1 >= ko_hi) VN = reb;
      ++mpos;
      while (mpos < mend && uni_i(A.mon_step[mpos]) <= m + 1) ++mpos;
      next_mon = (mpos < mend) ? uni_i(A.mon_step[mpos]) : 0x7fffffff;
    }
    if constexpr (W > 1) {
      if (lane == 0) xch[Xch<W>::kFirst + wave] = V[0];
      if (lane == 63) xch[Xch<W>::kLast + wave] = shrt ? V[NPT - 2] : V[NPT - 1];
    }
  }

  // ---- store ---------------------------------------------------------------
  double* vout = A.v_out + (size_t)scen * n_nodes;
  const double poison = overflow ? __longlong_as_double(0x7ff8000000000000ll) : 0.0;
  if (active) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int node = s_t + 1 + k;
      if (k < NPT - 1 || !shrt) vout[node] = overflow ? poison : V[k];
    }
  }
  if (t == 0) {
    vout[0] = overflow ? poison : V0;
    vout[n_nodes - 1] = overflow ? poison : VN;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(FDCN_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));       \
  } while (0)

using KernelFn = void (*)(KArgs);

struct Variant {
  int it, w, npt;
  KernelFn fn;
  int threads, spb;
};

template <int IT, int W, int NPT>
Variant mk() {
  return Variant{IT, W, NPT, &fdcn_march<IT, W, NPT>, Geo<IT, W, NPT>::kThreads,
                 Geo<IT, W, NPT>::SPB};
}

#define FDCN_VARIANTS(IT)                                                                   \
  mk<IT, 1, 4>(), mk<IT, 1, 8>(), mk<IT, 1, 12>(), mk<IT, 1, 16>(), mk<IT, 1, 24>(),        \
      mk<IT, 1, 32>(), mk<IT, 1, 40>(), mk<IT, 1, 48>(), mk<IT, 1, 64>(), mk<IT, 2, 40>(),  \
      mk<IT, 4, 24>(), mk<IT, 4, 40>(), mk<IT, 8, 40>(), mk<IT, 16, 24>(), mk<IT, 16, 40>()

const Variant kVariants[] = {FDCN_VARIANTS(0), FDCN_VARIANTS(1)};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

int lds_doubles(const Variant& v, int lz, int z_lds, int phi_lds) {
  int per = (z_lds ? 2 * lz * v.npt : 0) + ((v.it && phi_lds) ? 64 * v.w * v.npt : 0) +
            (v.w > 1 ? 6 * v.w + 2 : 0);
  return per * v.spb;
}

constexpr size_t kLdsLimit = 160 * 1024;

// Table placement: everything in LDS when it fits; otherwise the SM table
// (read by the first few lanes only) moves to the global workspace first, then
// the payoff (read from the input array, L2-resident).
void placement(const Variant& v, int lz, int* z_lds, int* phi_lds, size_t* lds_bytes) {
  *z_lds = 1;
  *phi_lds = 1;
  *lds_bytes = sizeof(double) * (size_t)lds_doubles(v, lz, 1, 1);
  if (*lds_bytes <= kLdsLimit) return;
  *z_lds = 0;
  *lds_bytes = sizeof(double) * (size_t)lds_doubles(v, lz, 0, 1);
  if (*lds_bytes <= kLdsLimit) return;
  *phi_lds = 0;
  *lds_bytes = sizeof(double) * (size_t)lds_doubles(v, lz, 0, 0);
}

// Choose the variant: fewest waves per scenario, then the least padding.
const Variant* choose(int n_nodes, int it) {
  const int n_int = n_nodes - 2;
  if (n_int < 3) return nullptr;
  const Variant* best = nullptr;
  long best_slots = 0;
  int best_w = 0;
  for (int i = 0; i < kNumVariants; ++i) {
    const Variant& v = kVariants[i];
    if (v.it != it) continue;
    if (best && v.w > best_w) continue;
    const int L_act = (n_int + v.npt - 1) / v.npt;
    const int L_short = L_act * v.npt - n_int;
    if (L_act > 64 * v.w || L_short >= L_act || v.npt > n_int) continue;
    const long slots = (long)64 * v.w * v.npt;
    if (!best || v.w < best_w || slots < best_slots) {
      best = &v;
      best_slots = slots;
      best_w = v.w;
    }
  }
  return best;
}

// Lanes whose chunks must hold the Sherman-Morrison table to cover k_cap nodes.
int lz_for(const Variant& v, int n_int, int k_cap) {
  const int L_act = (n_int + v.npt - 1) / v.npt;
  const int L_short = L_act * v.npt - n_int;
  int lz = (k_cap + v.npt - 1) / v.npt;
  if (lz < 1) lz = 1;
  while (lz < L_act && lz * v.npt - (lz < L_short ? lz : L_short) < k_cap) ++lz;
  if (lz > L_act) lz = L_act;
  return lz;
}

double host_fm(double theta, const double* P) {
  const double dt = P[FDCN_P_DT], a = P[FDCN_P_A], c = P[FDCN_P_C], bcoef = P[FDCN_P_BC];
  const double AL = -theta * dt * a;
  const double AC = 1.0 - theta * dt * bcoef;
  const double AU = -theta * dt * c;
  const double r = 0.5 * (AC + sqrt(AC * AC - 4.0 * AL * AU));
  return -AL * (1.0 / r);
}

int validate_common(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna) {
  if (B < 0) return fail(FDCN_EINVAL, "B must be >= 0 (got %d)", B);
  if (n_nodes < 5) return fail(FDCN_EINVAL, "n_nodes must be >= 5 (got %d)", n_nodes);
  if (n_time < 0) return fail(FDCN_EINVAL, "n_time must be >= 0 (got %d)", n_time);
  if (n_ranna < 0) return fail(FDCN_EINVAL, "n_ranna must be >= 0 (got %d)", n_ranna);
  return FDCN_OK;
}

int launch(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
           const double* params, const int32_t* iparams, const double* v_init,
           const double* payoff, int32_t n_mon, const int32_t* mon_step,
           const double* mon_rebate, double* v_out, int32_t k_cap, double* workspace,
           hipStream_t stream) {
  int rc = validate_common(B, n_nodes, n_time, n_ranna);
  if (rc) return rc;
  if (B == 0) return FDCN_OK;
  const Variant* v = choose(n_nodes, it);
  if (!v) return fail(FDCN_EINVAL, "unsupported n_nodes=%d", n_nodes);
  const int n_int = n_nodes - 2;
  if (k_cap <= 0) k_cap = n_int < 256 ? n_int : 256;
  const int lz = lz_for(*v, n_int, k_cap);
  int z_lds, phi_lds;
  size_t lds;
  placement(*v, lz, &z_lds, &phi_lds, &lds);
  if (lds > kLdsLimit)
    return fail(FDCN_EINVAL, "LDS request %zu B too large (k_cap=%d)", lds, k_cap);
  if (!z_lds && !workspace)
    return fail(FDCN_EINVAL, "this size needs a workspace of %lld B per scenario (fdcn_plan)",
                (long long)(sizeof(double) * 2 * (size_t)v->npt * lz));
  KArgs a;
  a.z_lds = z_lds;
  a.phi_lds = phi_lds;
  a.zg = workspace;
  a.B = B;
  a.n_nodes = n_nodes;
  a.n_time = n_time;
  a.n_ranna = n_ranna;
  a.n_mon = n_mon;
  a.lz = lz;
  a.params = params;
  a.iparams = iparams;
  a.v_init = v_init;
  a.payoff = payoff;
  a.mon_step = mon_step;
  a.mon_rebate = mon_rebate;
  a.v_out = v_out;
  if (lds > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute((const void*)v->fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
  const int grid = (B + v->spb - 1) / v->spb;
  hipLaunchKernelGGL(v->fn, dim3(grid), dim3(v->threads), lds, stream, a);
  HIP_TRY(hipGetLastError());
  return FDCN_OK;
}

int host_batch(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
               const double* params, const int32_t* iparams, const double* v_init,
               const double* payoff, int32_t n_mon, const int32_t* mon_step,
               const double* mon_rebate, double* v_out) {
  int rc = validate_common(B, n_nodes, n_time, n_ranna);
  if (rc) return rc;
  if (!params || !iparams || !v_init || !v_out || (it && !payoff))
    return fail(FDCN_EINVAL, "null array argument");
  if (n_mon < 0) return fail(FDCN_EINVAL, "n_mon must be >= 0");
  for (int32_t b = 0; b < B; ++b) {
    const int32_t* I = iparams + (size_t)b * FDCN_NIPARAM;
    const int s = I[FDCN_I_MON_START], c = I[FDCN_I_MON_COUNT];
    if (c < 0 || s < 0 || (c > 0 && (long)s + c > n_mon))
      return fail(FDCN_EINVAL, "scenario %d: monitor range [%d,+%d) outside n_mon=%d", b, s, c,
                  n_mon);
    if (it && c != 0) return fail(FDCN_EINVAL, "scenario %d: IT solves take no monitors", b);
    for (int f = FDCN_I_LO_FORM; f <= FDCN_I_HI_FORM; ++f)
      if (I[f] != 0 && I[f] != 1) return fail(FDCN_EINVAL, "scenario %d: bad boundary form", b);
    const double dt = params[(size_t)b * FDCN_NPARAM + FDCN_P_DT];
    if (!(dt > 0.0) && n_time > 0) return fail(FDCN_EINVAL, "scenario %d: dt must be > 0", b);
  }
  if (B == 0) return FDCN_OK;
  const int k_cap = fdcn_sm_extent(B, n_nodes, n_time, n_ranna, params);
  if (k_cap < 0) return k_cap;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(FDCN_ENODEV, "no HIP device visible");
  const size_t nv = (size_t)B * n_nodes;
  double *dP = nullptr, *dV = nullptr, *dO = nullptr, *dF = nullptr, *dR = nullptr;
  int32_t *dI = nullptr, *dM = nullptr;
  auto cleanup = [&]() {
    if (dP) (void)hipFree(dP);
    if (dV) (void)hipFree(dV);
    if (dO) (void)hipFree(dO);
    if (dF) (void)hipFree(dF);
    if (dR) (void)hipFree(dR);
    if (dI) (void)hipFree(dI);
    if (dM) (void)hipFree(dM);
  };
#define ALLOC(p, bytes)                                                        \
  if (hipMalloc((void**)&(p), (bytes)) != hipSuccess) {                        \
    cleanup();                                                                 \
    return fail(FDCN_ENOMEM, "hipMalloc(%zu) failed", (size_t)(bytes));        \
  }
  ALLOC(dP, sizeof(double) * (size_t)B * FDCN_NPARAM);
  ALLOC(dI, sizeof(int32_t) * (size_t)B * FDCN_NIPARAM);
  ALLOC(dV, sizeof(double) * nv);
  ALLOC(dO, sizeof(double) * nv);
  if (it) ALLOC(dF, sizeof(double) * nv);
  ALLOC(dM, sizeof(int32_t) * (size_t)(n_mon > 0 ? n_mon : 1));
  ALLOC(dR, sizeof(double) * (size_t)(n_mon > 0 ? n_mon : 1));
#undef ALLOC
  hipError_t e = hipSuccess;
  e = hipMemcpy(dP, params, sizeof(double) * (size_t)B * FDCN_NPARAM, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(dI, iparams, sizeof(int32_t) * (size_t)B * FDCN_NIPARAM,
                  hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dV, v_init, sizeof(double) * nv, hipMemcpyHostToDevice);
  if (e == hipSuccess && it) e = hipMemcpy(dF, payoff, sizeof(double) * nv, hipMemcpyHostToDevice);
  if (e == hipSuccess && n_mon > 0)
    e = hipMemcpy(dM, mon_step, sizeof(int32_t) * (size_t)n_mon, hipMemcpyHostToDevice);
  if (e == hipSuccess && n_mon > 0)
    e = hipMemcpy(dR, mon_rebate, sizeof(double) * (size_t)n_mon, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    cleanup();
    return fail(FDCN_EHIP, "hipMemcpy H2D failed: %s", hipGetErrorString(e));
  }
  double* dW = nullptr;
  {
    int32_t w_, npt_, spb_, lds_;
    int64_t ws_ = 0;
    rc = fdcn_plan(n_nodes, it, k_cap, &w_, &npt_, &spb_, &lds_, &ws_);
    if (rc == FDCN_OK && ws_ > 0 && hipMalloc((void**)&dW, (size_t)ws_ * B) != hipSuccess) {
      cleanup();
      return fail(FDCN_ENOMEM, "hipMalloc(workspace) failed");
    }
  }
  if (rc == FDCN_OK)
    rc = launch(it, B, n_nodes, n_time, n_ranna, dP, dI, dV, dF, n_mon, dM, dR, dO, k_cap, dW,
                nullptr);
  if (rc == FDCN_OK) {
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(v_out, dO, sizeof(double) * nv, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(FDCN_EHIP, "kernel/D2H failed: %s", hipGetErrorString(e));
  }
  if (dW) (void)hipFree(dW);
  cleanup();
  return rc;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int fdcn_sm_extent(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                   const double* params) {
  int rc = validate_common(B, n_nodes, n_time, n_ranna);
  if (rc) return rc;
  if (!params && B > 0) return fail(FDCN_EINVAL, "null params");
  const int n_int = n_nodes - 2;
  int k = 1;
  for (int32_t b = 0; b < B; ++b) {
    const double* P = params + (size_t)b * FDCN_NPARAM;
    if (n_ranna > 0) k = std::max(k, sm_extent(host_fm(1.0, P), n_int));
    if (n_ranna < n_time) k = std::max(k, sm_extent(host_fm(0.5, P), n_int));
  }
  return k;
}

int fdcn_plan(int32_t n_nodes, int32_t it_mode, int32_t k_cap, int32_t* waves, int32_t* npt,
              int32_t* scen_per_block, int32_t* lds_bytes, int64_t* ws_bytes_per_scen) {
  const Variant* v = choose(n_nodes, it_mode ? 1 : 0);
  if (!v) return fail(FDCN_EINVAL, "unsupported n_nodes=%d", n_nodes);
  const int n_int = n_nodes - 2;
  if (k_cap <= 0) k_cap = n_int < 256 ? n_int : 256;
  const int lz = lz_for(*v, n_int, k_cap);
  int z_lds, phi_lds;
  size_t lds;
  placement(*v, lz, &z_lds, &phi_lds, &lds);
  if (lds > kLdsLimit) return fail(FDCN_EINVAL, "LDS request %zu B too large", lds);
  if (waves) *waves = v->w;
  if (npt) *npt = v->npt;
  if (scen_per_block) *scen_per_block = v->spb;
  if (lds_bytes) *lds_bytes = (int32_t)lds;
  if (ws_bytes_per_scen)
    *ws_bytes_per_scen = z_lds ? 0 : (int64_t)(sizeof(double) * 2 * (size_t)v->npt * lz);
  return FDCN_OK;
}

int fdcn_cn_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams, const double* v_init,
                      int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                      double* v_out, int32_t k_cap, double* workspace, void* stream) {
  return launch(0, B, n_nodes, n_time, n_ranna, params, iparams, v_init, nullptr, n_mon,
                mon_step, mon_rebate, v_out, k_cap, workspace, (hipStream_t)stream);
}

int fdcn_it_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams, const double* v_init,
                      const double* payoff, double* v_out, int32_t k_cap, double* workspace,
                      void* stream) {
  return launch(1, B, n_nodes, n_time, n_ranna, params, iparams, v_init, payoff, 0, nullptr,
                nullptr, v_out, k_cap, workspace, (hipStream_t)stream);
}

int fdcn_cn_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, const double* v_init,
                  int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                  double* v_out) {
  return host_batch(0, B, n_nodes, n_time, n_ranna, params, iparams, v_init, nullptr, n_mon,
                    mon_step, mon_rebate, v_out);
}

int fdcn_it_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, const double* v_init,
                  const double* payoff, double* v_out) {
  return host_batch(1, B, n_nodes, n_time, n_ranna, params, iparams, v_init, payoff, 0,
                    nullptr, nullptr, v_out);
}

const char* fdcn_last_error(void) { return g_err.c_str(); }

int fdcn_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int good = 0;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0)
      ++good;
  }
  return good;
}

int fdcn_abi_version(void) { return FDCN_ABI_VERSION; }

}  // extern "C"
