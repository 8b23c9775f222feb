// fdcn_shared.h -- internal to libfdcn: the helpers the device march and
// the host-only translation unit (fdcn_host.hip) both evaluate, and the
// host-side checks the launch paths share.  Not part of the C ABI.
#ifndef FDCN_SHARED_H
#define FDCN_SHARED_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace fdcn_internal {

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

// Accumulated tau (FDCN_I_TAU_MODE = 1): tau_{k+1} = fl(tau_k + dt), the
// reference American loop's `tau = tau + dt` (fd_american_equity.py:664-724).
// Within a binade [2^(e-1), 2^e) every tau_k is a multiple of the ulp u and
// every add carries the same remainder r = dt - delta below u, so the rounded
// increment delta is the same on every step -- unless |r| is exactly u/2
// (ties-to-even then depends on tau_k's last bit).  There the sequence is
// exactly tau_k0 + j delta (a multiple of u below 2^e is representable, so
// that expression is exact with or without FMA contraction).  tau_next_run
// walks the sequence run by run: one constant-increment run per binade, plus
// single serial steps within 2 ulp of a binade crossing, at ties, and while
// tau <= dt.  ~3 runs per binade instead of one dependent add per step, and
// bit-identical to the serial adds (fdcn_tau_sequence exposes it to tests).
struct TauRun {
  int k, len;        // steps k .. k+len-1 advance tau_k -> tau_{k+len}
  double t, delta;   // tau_k and the run's increment
  double t_next;     // tau_{k+len}
};

__host__ __device__ inline bool tau_next_run(double& t, int& k, int n, double dt, TauRun& run) {
#pragma clang fp contract(off)
  if (k >= n) return false;
  run.k = k;
  run.t = t;
  const double t1 = t + dt;  // one serial step unless a longer run is proven exact
  run.len = 1;
  run.delta = 0.0;
  run.t_next = t1;
  if (t >= 1e-300 && dt > 0.0 && dt < t && t1 < 1e300) {
    int e;
    (void)frexp(t, &e);                 // t in [2^(e-1), 2^e)
    const double hi = ldexp(1.0, e);
    const double u = ldexp(1.0, e - 53);  // ulp in that binade
    const double delta = t1 - t;          // exact (Sterbenz: t <= t1 <= 2t)
    const double r = dt - delta;          // exact, |r| <= u/2
    if (t1 < hi && fabs(r) != 0.5 * u) {
      // every add of the run stays below hi - u/2 if t + L delta <= hi - 2u
      double L = (double)(n - k);
      if (delta > 0.0) {
        const double lim = floor((hi - 2.0 * u - t) / delta);
        if (lim < L) L = lim;
        while (L > 1.0 && t + L * delta > hi - 2.0 * u) L -= 1.0;
      }
      if (L >= 1.0) {
        run.len = (int)L;
        run.delta = delta;
        run.t_next = t + L * delta;
      }
    }
  }
  t = run.t_next;
  k += run.len;
  return true;
}

// error reporting (thread-local message behind fdcn_last_error)
int set_error(int code, const char* msg);
// fm = -A_L / r of the converged LU factors at theta (host copy of make_phase)
double host_fm(double theta, const double* P);
// launch-size checks and the plan checks of the host entry points / sessions
int validate_common(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna);
int validate_plan(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, int32_t n_mon,
                  const int32_t* mon_step, const double* mon_rebate);

}  // namespace fdcn_internal

#endif  // FDCN_SHARED_H
