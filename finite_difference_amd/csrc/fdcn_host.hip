// fdcn_host.hip -- the host-only part of libfdcn's C ABI: error reporting,
// the plan checks every launch path shares, and the host helpers that are
// bit-identical to the reference's Python (log grid, accumulated tau, the
// dividend-jump spline).  No kernels: the translation unit also builds for
// the host alone, which is how `make sanitize` runs it under ASan / UBSan
// (and fdcn_plan.hip under TSan) on a CPU-only host.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/fdcn.h"
#include "fdcn_shared.h"

namespace fdcn_internal {

namespace {
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
}  // namespace

int set_error(int code, const char* msg) { return fail(code, "%s", msg); }

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

// Host-side checks of a launch plan (host arrays): sizes, monitor runs
// (strictly increasing, in [1, n_time]), boundary forms, tau mode, dt > 0.
int validate_plan(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, int32_t n_mon,
                  const int32_t* mon_step, const double* mon_rebate) {
  int rc = validate_common(B, n_nodes, n_time, n_ranna);
  if (rc) return rc;
  if (B > 0 && (!params || !iparams)) return fail(FDCN_EINVAL, "null array argument");
  if (n_mon < 0) return fail(FDCN_EINVAL, "n_mon must be >= 0");
  if (n_mon > 0 && (!mon_step || !mon_rebate)) return fail(FDCN_EINVAL, "null monitor arrays");
  for (int32_t b = 0; b < B; ++b) {
    const int32_t* I = iparams + (size_t)b * FDCN_NIPARAM;
    const int s = I[FDCN_I_MON_START], c = I[FDCN_I_MON_COUNT];
    if (c < 0 || s < 0 || (c > 0 && (long)s + c > n_mon))
      return fail(FDCN_EINVAL, "scenario %d: monitor range [%d,+%d) outside n_mon=%d", b, s, c,
                  n_mon);
    if (it && c != 0) return fail(FDCN_EINVAL, "scenario %d: IT solves take no monitors", b);
    for (int k = 0; k < c; ++k) {
      const int32_t st = mon_step[s + k];
      if (st < 1 || st > n_time || (k > 0 && st <= mon_step[s + k - 1]))
        return fail(FDCN_EINVAL,
                    "scenario %d: monitor steps must be strictly increasing in [1, n_time=%d] "
                    "(entry %d is %d)", b, n_time, k, st);
    }
    for (int f = FDCN_I_LO_FORM; f <= FDCN_I_HI_FORM; ++f)
      if (I[f] != 0 && I[f] != 1) return fail(FDCN_EINVAL, "scenario %d: bad boundary form", b);
    if (I[FDCN_I_TAU_MODE] != 0 && I[FDCN_I_TAU_MODE] != 1)
      return fail(FDCN_EINVAL, "scenario %d: TAU_MODE must be 0 or 1", b);
    const double dt = params[(size_t)b * FDCN_NPARAM + FDCN_P_DT];
    if (!(dt > 0.0) && n_time > 0) return fail(FDCN_EINVAL, "scenario %d: dt must be > 0", b);
  }
  return FDCN_OK;
}

}  // namespace fdcn_internal

using namespace fdcn_internal;

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

int fdcn_tau_sequence(double tau0, double dt, int32_t n, double* tau) {
  if (n < 0 || (n > 0 && !tau)) return fail(FDCN_EINVAL, "fdcn_tau_sequence: n >= 0, tau non-NULL");
  double tc = tau0;
  int kc = 0;
  TauRun run;
  while (tau_next_run(tc, kc, n, dt, run))
    for (int j = 0; j < run.len; ++j)
      tau[run.k + j] = (j + 1 == run.len) ? run.t_next : run.t + (double)(j + 1) * run.delta;
  return FDCN_OK;
}

int fdcn_tau_runs(double tau0, double dt, int32_t n) {
  if (n < 0) return fail(FDCN_EINVAL, "fdcn_tau_runs: n >= 0");
  double tc = tau0;
  int kc = 0, runs = 0;
  TauRun run;
  while (tau_next_run(tc, kc, n, dt, run)) ++runs;
  return runs;
}

int fdcn_log_grid(double x_min, double dx, int32_t n, double* x, double* s) {
#pragma clang fp contract(off)
  if (n < 0 || !s) return fail(FDCN_EINVAL, "fdcn_log_grid: n must be >= 0 and s non-NULL");
  for (int32_t i = 0; i <= n; ++i) {
    const double xi = x_min + (double)i * dx;  // the reference's x_min + i * dx
    if (x) x[i] = xi;
    s[i] = ::exp(xi);                           // libm exp, as math.exp
  }
  return FDCN_OK;
}

int fdcn_dividend_jump(int32_t n, const double* s, const double* v, double cash_div,
                       double strike_call, double* v_out) {
#pragma clang fp contract(off)
  if (n < 2 || !s || !v || !v_out) return fail(FDCN_EINVAL, "fdcn_dividend_jump: n >= 2 and non-NULL arrays");
  for (int32_t i = 0; i + 1 < n; ++i)
    if (!(s[i + 1] - s[i] > 0.0)) return fail(FDCN_EINVAL, "x must be strictly increasing.");
  // natural cubic spline through (s, v): fd_american_equity.py:479-553
  std::vector<double> h(n - 1), alpha(n, 0.0), l(n, 1.0), mu(n, 0.0), z(n, 0.0), c(n, 0.0),
      b(n - 1, 0.0), d(n - 1, 0.0);
  for (int32_t i = 0; i + 1 < n; ++i) h[i] = s[i + 1] - s[i];
  for (int32_t i = 1; i + 1 < n; ++i)
    alpha[i] = 3.0 / h[i] * (v[i + 1] - v[i]) - 3.0 / h[i - 1] * (v[i] - v[i - 1]);
  for (int32_t i = 1; i + 1 < n; ++i) {
    l[i] = 2.0 * (s[i + 1] - s[i - 1]) - h[i - 1] * mu[i - 1];
    mu[i] = h[i] / l[i];
    z[i] = (alpha[i] - h[i - 1] * z[i - 1]) / l[i];
  }
  for (int32_t j = n - 2; j >= 0; --j) {
    c[j] = z[j] - mu[j] * c[j + 1];
    b[j] = (v[j + 1] - v[j]) / h[j] - h[j] * (c[j + 1] + 2.0 * c[j]) / 3.0;
    d[j] = (c[j + 1] - c[j]) / (3.0 * h[j]);
  }
  // V(t_d-, S) = V(t_d+, S - D) (:732-772); interval by searchsorted(side="right") - 1
  for (int32_t i = 0; i < n; ++i) {
    const double q = s[i] - cash_div;
    double cont;
    if (q <= s[0]) {
      cont = v[0];
    } else if (q >= s[n - 1]) {
      cont = v[n - 1];
    } else {
      int32_t j = (int32_t)(std::upper_bound(s, s + n, q) - s) - 1;
      if (j > n - 2) j = n - 2;
      const double t = q - s[j];
      cont = v[j] + b[j] * t + c[j] * t * t + d[j] * t * t * t;
    }
    if (strike_call >= 0.0) {  // calls may exercise at the ex-date: max(cont, payoff)
      const double e = s[i] - strike_call;
      const double ex = (0.0 > e) ? 0.0 : e;     // Python max(e, 0.0) (keeps e's zero sign)
      cont = (ex > cont) ? ex : cont;            // Python max(cont, ex)
    }
    v_out[i] = cont;
  }
  return FDCN_OK;
}

const char* fdcn_last_error(void) { return g_err.c_str(); }

}  // extern "C"
