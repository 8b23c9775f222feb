// fdcn_plan.hip -- native plan builder for whole scenario files (host code).
//
// The discrete-barrier runner (run_config_scenarios.py:137-195 over
// DiscreteBarrierFDMPricer, discrete_barrier_fdm_pricer.py:84-1084) builds,
// per scenario row, two grids (base and sigma-bumped), their payoffs,
// boundaries, knock-out thresholds, monitoring rebates and operator
// coefficients, then reads 3-4 nodes of each solved grid.  Done row by row
// in Python that costs ~0.5 ms per row -- seconds for a 10 000-row file
// against a 6 ms march.  fdcn_barrier_plan does the same arithmetic for all
// rows at once, in C with the C library's exp/log/sqrt (the functions
// CPython's math module calls) and the reference's operation order, so the
// plan arrays are bit-identical to the per-row facade's (tests), on all
// host threads.  fdcn_vmath exposes the libm functions vectorised, for the
// Black-76 legs the Python side evaluates in bulk.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/fdcn.h"

namespace fdcn_internal {
int set_error(int code, const char* msg);
}

namespace {

int pfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fdcn_internal::set_error(code, buf);
}

// parallel for over [0, n) on the host threads (std::thread: no OpenMP
// runtime is pulled into a process that may already hold torch's)
template <class F>
void parallel_for(int64_t n, int64_t grain, F f) {
  unsigned hw = std::thread::hardware_concurrency();
  int nt = (int)std::min<int64_t>(hw ? hw : 1, 16);
  nt = (int)std::min<int64_t>(nt, (n + grain - 1) / grain);
  if (nt <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([=]() {
      const int64_t a = t * chunk, b = std::min(n, a + chunk);
      for (int64_t i = a; i < b; ++i) f(i);
    });
  for (auto& x : th) x.join();
}

// bisections over a grid evaluated on demand (s(i) -> node i):
// first j in [lo, hi) with s(j) > x (bisect.bisect_right) ...
template <class G>
int64_t upper_g(const G& s, int64_t lo, int64_t hi, double x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (x < s(mid)) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
// ... and first j in [lo, hi) with s(j) >= x (bisect_left / searchsorted left)
template <class G>
int64_t lower_g(const G& s, int64_t lo, int64_t hi, double x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (s(mid) < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// A log grid's nodes, s_i = exp(x_min + i dx) (_build_log_grid), evaluated
// only where they are read: the payoff max(+-(s_i - K), 0) is exactly 0 on
// the nodes whose x_i lies clearly on the out-of-the-money side of log K
// (|x_i - log K| > 1e-9: exp's error, ~1e-16 relative, cannot cross K), so
// those nodes take no exp -- half the grid on average, and the exps are
// most of the plan builder's time.  Nodes that are evaluated use the same
// expression as a full evaluation, so every value is bit-identical.
struct LogGrid {
  double x_min, dx;
  double x(int64_t i) const { return x_min + (double)i * dx; }
  double operator()(int64_t i) const { return ::exp(x(i)); }
  // payoff on nodes [0, n): max(s_i - K, 0) (call) / max(K - s_i, 0) (put)
  void payoff(bool call, double K, int64_t n, double* v) const {
    const double lk = ::log(K), eps = 1e-9;
    int64_t a = 0, b = n;  // nodes [a, b) may be in the money
    if (call) {
      while (a < n && x(a) < lk - eps) v[a++] = 0.0;
    } else {
      while (b > 0 && x(b - 1) > lk + eps) v[--b] = 0.0;
    }
    for (int64_t i = a; i < b; ++i) {
      const double s = (*this)(i);
      const double e = call ? s - K : K - s;
      v[i] = (0.0 > e) ? 0.0 : e;  // Python max(e, 0.0)
    }
  }
};

}  // namespace

extern "C" {

int fdcn_vmath(int32_t op, int64_t n, const double* x, double* y) {
#pragma clang fp contract(off)
  if (n < 0 || (n > 0 && (!x || !y)) || op < 0 || op > 3)
    return pfail(FDCN_EINVAL, "fdcn_vmath: op in {0 exp, 1 log, 2 sqrt, 3 pow(x, 2)}, n >= 0");
  // an opaque exponent: LLVM would fold pow(x, 2.0) into x * x, which is not
  // what CPython's float ** 2 returns (it calls glibc's pow, whose result
  // differs from the correctly rounded square in ~6e-4 of the inputs)
  volatile double two_v = 2.0;
  const double two = two_v;
  parallel_for(n, 1 << 14, [&](int64_t i) {
    switch (op) {
      case 0: y[i] = ::exp(x[i]); break;
      case 1: y[i] = ::log(x[i]); break;
      case 2: y[i] = ::sqrt(x[i]); break;
      default: y[i] = ::pow(x[i], two); break;
    }
  });
  return FDCN_OK;
}

int fdcn_barrier_plan(int32_t R, const double* row, const int32_t* rflag, double T,
                      int32_t n_space, int32_t n_time, int32_t grid_mode, int32_t n_nodes_cap,
                      double k_tail, double dv_sigma, int32_t rebate_at_hit, int32_t n_mon,
                      const int32_t* mon_k, double* params, int32_t* iparams, double* v_init,
                      double* mon_rebate, int32_t* rint, double* rdbl, double* tparams,
                      int32_t* n_nodes_out) {
#pragma clang fp contract(off)
  if (R < 0 || n_time < 1 || n_space < 2 || n_mon < 0)
    return pfail(FDCN_EINVAL, "fdcn_barrier_plan: R >= 0, n_time >= 1, n_space >= 2");
  if (R == 0) return FDCN_OK;
  if (!row || !rflag || !params || !iparams || !v_init || !rint || !rdbl || !tparams ||
      !n_nodes_out || (n_mon > 0 && (!mon_k || !mon_rebate)))
    return pfail(FDCN_EINVAL, "fdcn_barrier_plan: NULL argument");
  // N_s of the parity mode: ceil(width N_t / (2 sigma sqrt T)) with width =
  // 2 k sigma sqrt T (…pricer.py:316-317) -- evaluated per solve below and
  // required to agree (one launch shape); explicit mode keeps n_space
  const double sqT = ::sqrt(T);
  const double dt = T / (double)n_time;
  std::vector<int32_t> ns(2 * (size_t)R, 0);
  parallel_for(2 * (int64_t)R, 256, [&](int64_t q) {
    const double* r = row + (q >> 1) * FDCN_BP_NROW;
    const double sigma = (q & 1) ? r[FDCN_BP_SIGMA] + dv_sigma : r[FDCN_BP_SIGMA];
    if (grid_mode == 0) {
      const double width = 2.0 * k_tail * sigma * sqT;
      ns[q] = (int32_t)::ceil((width * (double)n_time) / (2 * sigma * sqT));
    } else {
      ns[q] = n_space;
    }
  });
  const int32_t N = ns[0];
  for (size_t q = 1; q < ns.size(); ++q)
    if (ns[q] != N) return pfail(FDCN_EINVAL, "fdcn_barrier_plan: grid sizes differ across rows");
  if (N < 5) return pfail(FDCN_EINVAL, "fdcn_barrier_plan: N_s=%d too small", N);
  if (N > n_nodes_cap)
    return pfail(FDCN_EINVAL, "fdcn_barrier_plan: N_s=%d exceeds n_nodes_cap=%d", N, n_nodes_cap);
  *n_nodes_out = N;  // the march's n_nodes: the top node is dropped (…pricer.py:449, :543)
  parallel_for(2 * (int64_t)R, 16, [&](int64_t q) {
    const int64_t ri = q >> 1;
    const bool bump = q & 1;
    const double* r = row + ri * FDCN_BP_NROW;
    const int32_t* f = rflag + ri * FDCN_BP_NFLAG;
    const double spot = r[FDCN_BP_SPOT], K = r[FDCN_BP_STRIKE];
    const double sigma = bump ? r[FDCN_BP_SIGMA] + dv_sigma : r[FDCN_BP_SIGMA];
    const double carry = r[FDCN_BP_CARRY], divy = r[FDCN_BP_DIVY], rr = r[FDCN_BP_DISC];
    const double pv = r[FDCN_BP_PV];
    const bool has_lo = f[FDCN_BP_HAS_LO] != 0, has_up = f[FDCN_BP_HAS_UP] != 0;
    const double Hlo = r[FDCN_BP_LO], Hup = r[FDCN_BP_UP];
    const bool call = f[FDCN_BP_PUT] == 0;
    const int kind = f[FDCN_BP_KO];  // 1 down-and-out, 2 up-and-out, 3 double-out
    // choose_grid_parameters (…pricer.py:270-320) at S0 = spot - pv_divs
    double s_low = spot - pv, s_high = spot - pv;
    s_low = std::min(s_low, K);  // min([S0, K, ...]) in list order
    s_high = std::max(s_high, K);
    if (has_lo && Hlo > 0.0) {
      s_low = std::min(s_low, Hlo);
      s_high = std::max(s_high, Hlo);
    }
    if (has_up && Hup > 0.0) {
      s_low = std::min(s_low, Hup);
      s_high = std::max(s_high, Hup);
    }
    const double width = 2.0 * k_tail * sigma * sqT;
    const double x_c = ::log(::sqrt(s_low * s_high));
    const double e_lo = ::exp(x_c - 0.5 * width), e_hi = ::exp(x_c + 0.5 * width);
    const double S_min = (e_lo < 0.5 * s_low) ? e_lo : 0.5 * s_low;  // Python min(a, b)
    const double S_max = (2 * s_high > e_hi) ? 2 * s_high : e_hi;    // Python max(a, b)
    // _build_log_grid (:342-364): x_i = x_min + i dx, s_i = exp(x_i), i = 0..N
    const double x_min = ::log(S_min), x_max = ::log(S_max);
    const double dx = (x_max - x_min) / N;
    const LogGrid s{x_min, dx};  // nodes evaluated where read
    // operator coefficients (…pricer.py:463-472)
    const double sig2 = sigma * sigma;
    const double mu_x = (carry - divy) - 0.5 * sig2;
    const double alpha = 0.5 * sig2 / (dx * dx);
    const double beta_adv = mu_x / (2.0 * dx);
    double* P = params + q * FDCN_NPARAM;
    for (int k = 0; k < FDCN_NPARAM; ++k) P[k] = 0.0;
    P[FDCN_P_DT] = dt;
    P[FDCN_P_A] = alpha - beta_adv;
    P[FDCN_P_C] = alpha + beta_adv;
    P[FDCN_P_BC] = -2.0 * alpha - rr;
    int32_t* I = iparams + q * FDCN_NIPARAM;
    for (int k = 0; k < FDCN_NIPARAM; ++k) I[k] = 0;
    // _boundary_values (:372-393): call top S_max e^{(b-r)tau} - K e^{-r tau};
    // put bottom K e^{-r tau} S_min e^{(b-r) tau} (the :391 product)
    if (call) {
      P[FDCN_P_HI_C0] = s(N);
      P[FDCN_P_HI_E0] = carry - rr;
      P[FDCN_P_HI_C1] = -K;
      P[FDCN_P_HI_E1] = -rr;
    } else {
      I[FDCN_I_LO_FORM] = 1;
      P[FDCN_P_LO_C0] = K;
      P[FDCN_P_LO_E0] = -rr;
      P[FDCN_P_LO_C1] = s(0);
      P[FDCN_P_LO_E1] = carry - rr;
    }
    // knock-out thresholds over nodes 0..N-1 (_ko_thresholds)
    int32_t ko_lo = -1, ko_hi = N;
    if ((kind == 1 || kind == 3) && has_lo) ko_lo = (int32_t)upper_g(s, 0, N, Hlo) - 1;
    if ((kind == 2 || kind == 3) && has_up) ko_hi = (int32_t)lower_g(s, 0, N, Hup);
    I[FDCN_I_KO_LO] = std::max(-1, std::min(ko_lo, N));
    I[FDCN_I_KO_HI] = std::max(-1, std::min(ko_hi, N + 1));
    I[FDCN_I_MON_START] = (int32_t)(q * n_mon);
    I[FDCN_I_MON_COUNT] = n_mon;
    // monitor rebates (_rebate at tau = k dt, :421-424)
    const double reb = r[FDCN_BP_REBATE];
    for (int32_t m = 0; m < n_mon; ++m)
      mon_rebate[q * n_mon + m] =
          rebate_at_hit ? reb : reb * ::exp(-carry * ((double)mon_k[m] * dt));
    // payoff on nodes 0..N-1 (_terminal_payoff, Python max(e, 0.0))
    s.payoff(call, K, N, v_init + q * (int64_t)N);
    // readouts (_interp_price :629-646 at spot - pv; _delta_gamma_from_grid
    // :949-978 at spot, base grid only), on the full grid s[0..N]
    int32_t* ri_ = rint + q * FDCN_GK_NRINT;
    double* rd = rdbl + q * FDCN_GK_NRDBL;
    for (int k = 0; k < FDCN_GK_NRDBL; ++k) rd[k] = 0.0;
    const double S0 = spot - pv;
    ri_[0] = (int32_t)q;  // the solve's index; the caller maps it to a slot
    if (S0 <= s(0)) {
      ri_[1] = 1;
      ri_[2] = 0;
    } else if (S0 >= s(N)) {
      ri_[1] = 2;
      ri_[2] = N - 1;  // V[-1] of the N-node vector
    } else {
      const int64_t hi = upper_g(s, 0, N + 1, S0);
      ri_[1] = 0;
      ri_[2] = (int32_t)(hi - 1);
      rd[1] = s(hi - 1);
      rd[2] = s(hi);
    }
    rd[0] = S0;
    if (!bump) {
      // 1 + argmin_{1 <= i <= N-1} |s_i - spot| (first on ties)
      int64_t lo_i = 1, hi_i = N - 1;
      int64_t j = lower_g(s, lo_i, hi_i + 1, spot);
      int64_t idx;
      if (j <= lo_i) idx = lo_i;
      else if (j > hi_i) idx = hi_i;
      else idx = (::fabs(s(j - 1) - spot) <= ::fabs(s(j) - spot)) ? j - 1 : j;
      ri_[3] = (int32_t)idx;
      ri_[4] = 1;
      rd[3] = spot;
      rd[4] = s(idx - 1);
      rd[5] = s(idx);
      rd[6] = s(idx + 1);
    } else {
      ri_[3] = 0;
      ri_[4] = 0;
    }
    if (!bump) {
      double* tp = tparams + ri * FDCN_GK_NPARAM;
      for (int k = 0; k < FDCN_GK_NPARAM; ++k) tp[k] = 0.0;
      tp[0] = r[FDCN_BP_SIGMA];
      tp[1] = spot;
      tp[2] = carry;
      tp[3] = divy;
      tp[4] = rr;
      tp[5] = dv_sigma;
    }
  });
  return FDCN_OK;
}

int fdcn_american_plan(int32_t J, const double* job, const int32_t* call, int32_t n_space,
                       double s_max_mult, double T, double* params, int32_t* iparams,
                       double* payoff, double* s_nodes, int32_t* rint, double* rdbl,
                       double* gout) {
#pragma clang fp contract(off)
  if (J < 0 || n_space < 3)
    return pfail(FDCN_EINVAL, "fdcn_american_plan: J >= 0, n_space >= 3");
  if (J == 0) return FDCN_OK;
  if (!job || !call || !params || !iparams || !payoff || !rint || !rdbl || !gout)
    return pfail(FDCN_EINVAL, "fdcn_american_plan: NULL argument");
  const int32_t n = n_space;  // nodes 0..n
  parallel_for(J, 8, [&](int64_t q) {
    const double* jb = job + q * FDCN_AP_NJOB;
    const double spot = jb[FDCN_AP_SPOT], K = jb[FDCN_AP_STRIKE], sig = jb[FDCN_AP_SIGMA];
    const double b = jb[FDCN_AP_CARRY], r = jb[FDCN_AP_DISC];
    const bool is_call = call[q] != 0;
    // _configure_grid (fd_american_equity.py:340-361), Python min/max order
    const double s_low = (K < spot) ? K : spot;    // min(spot, strike)
    const double s_high = (K > spot) ? K : spot;   // max(spot, strike)
    const double prod = s_low * s_high;
    const double s_c = ::sqrt(1e-12 > prod ? 1e-12 : prod);
    const double band = s_max_mult * sig * ::sqrt(1e-12 > T ? 1e-12 : T);
    const double x_c = ::log(s_c);
    double s_min = ::exp(x_c - 0.5 * band), s_max = ::exp(x_c + 0.5 * band);
    if (0.5 * s_low < s_min) s_min = 0.5 * s_low;
    if (2.0 * s_high > s_max) s_max = 2.0 * s_high;
    if (1e-8 > s_min) s_min = 1e-8;
    // _build_log_grid (:363-384)
    const double x_min = ::log(s_min), x_max = ::log(s_max);
    const double dx = (x_max - x_min) / (double)n;
    // the nodes: all of them when the caller wants the grids (dividend
    // jumps, the host path), else evaluated where read (LogGrid)
    const LogGrid grid{x_min, dx};
    double* sn = s_nodes ? s_nodes + q * (int64_t)(n + 1) : nullptr;
    if (sn)
      for (int32_t i = 0; i <= n; ++i) sn[i] = grid(i);
    auto s = [&](int64_t i) { return sn ? sn[i] : grid(i); };
    // _snap_critical_levels_to_grid (:386-407): argmin |s - x|, first on ties
    auto nearest = [&](double x) -> int32_t {
      const int64_t j = lower_g(s, 0, (int64_t)n + 1, x);
      if (j <= 0) return 0;
      if (j > n) return n;
      return (::fabs(s(j - 1) - x) <= ::fabs(s(j) - x)) ? (int32_t)(j - 1) : (int32_t)j;
    };
    const int32_t is = nearest(spot), ik = nearest(K);
    const double s0 = s(is), ks = s(ik);
    // payoff with the snapped strike (Python max(e, 0.0))
    double* pf = payoff + q * (int64_t)(n + 1);
    if (sn) {
      for (int32_t i = 0; i <= n; ++i) {
        const double e = is_call ? sn[i] - ks : ks - sn[i];
        pf[i] = (0.0 > e) ? 0.0 : e;
      }
    } else {
      grid.payoff(is_call, ks, n + 1, pf);
    }
    // operator coefficients (q = 0: discrete dividends are jumps)
    const double sig2 = sig * sig;
    const double mu_x = (b - 0.0) - 0.5 * sig2;
    const double alpha = 0.5 * sig2 / (dx * dx);
    const double beta_adv = mu_x / (2.0 * dx);
    double* P = params + q * FDCN_NPARAM;
    for (int k = 0; k < FDCN_NPARAM; ++k) P[k] = 0.0;
    P[FDCN_P_A] = alpha - beta_adv;
    P[FDCN_P_C] = alpha + beta_adv;
    P[FDCN_P_BC] = -2.0 * alpha - r;
    // Dirichlet values (:430-448): call top s_N e^{(b-r)tau} - K e^{-r tau};
    // put bottom K e^{-r tau}
    if (is_call) {
      P[FDCN_P_HI_C0] = s(n);
      P[FDCN_P_HI_E0] = b - r;
      P[FDCN_P_HI_C1] = -ks;
      P[FDCN_P_HI_E1] = -r;
    } else {
      P[FDCN_P_LO_C0] = ks;
      P[FDCN_P_LO_E0] = -r;
    }
    int32_t* I = iparams + q * FDCN_NIPARAM;
    for (int k = 0; k < FDCN_NIPARAM; ++k) I[k] = 0;
    I[FDCN_I_KO_LO] = -1;
    I[FDCN_I_KO_HI] = n + 2;  // none (>= n_nodes, as engine.pack clamps it)
    I[FDCN_I_TAU_MODE] = 1;   // tau = tau + dt (fd_american_equity.py:664-724)
    // readouts at the snapped spot (_interp_price :855-874): interpolation
    // only (row 2q), and with the cubic Delta/Gamma (:876-907) around the
    // nearest node clamped to [1, n-2] (row 2q+1); slot field = job index
    for (int c = 0; c < 2; ++c) {
      int32_t* ri = rint + (2 * q + c) * FDCN_GK_NRINT;
      double* rd = rdbl + (2 * q + c) * FDCN_GK_NRDBL;
      for (int k = 0; k < FDCN_GK_NRDBL; ++k) rd[k] = 0.0;
      ri[0] = (int32_t)q;
      if (s0 <= s(0)) {
        ri[1] = 1;
        ri[2] = 0;
      } else if (s0 >= s(n)) {
        ri[1] = 2;
        ri[2] = n;
      } else {
        const int64_t hi = upper_g(s, 0, (int64_t)n + 1, s0);
        ri[1] = 0;
        ri[2] = (int32_t)(hi - 1);
        rd[1] = s(hi - 1);
        rd[2] = s(hi);
      }
      rd[0] = s0;
      if (c == 0) {
        ri[3] = 0;
        ri[4] = 0;
      } else {
        int32_t i = is;  // argmin |s - s0| = the snapped index
        i = i < 1 ? 1 : (i > n - 2 ? n - 2 : i);
        ri[3] = i;
        ri[4] = 2;
        rd[3] = s0;
        for (int k = 0; k < 4; ++k) rd[4 + k] = s(i - 1 + k);
      }
    }
    double* g = gout + q * FDCN_AP_NOUT;
    g[0] = s0;
    g[1] = ks;
    g[2] = dx;
    g[3] = (double)is;
  });
  return FDCN_OK;
}

}  // extern "C"
