// plan_driver.cpp -- CPU driver of libfdcn's host-only code for the
// sanitizer builds (`make sanitize`).  Linked with fdcn_plan.hip
// and fdcn_host.hip compiled for the host alone (no device code), under
// ThreadSanitizer: the plan builders fan their rows out over std::threads
// (fdcn_plan.hip parallel_for), and two caller threads run them at once
// here (the C ABI is reentrant).  Every concurrent result must equal the
// sequential one bit for bit; TSan reports any data race.  Exit 0 = clean.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <thread>
#include <vector>

#include "../../include/fdcn.h"

namespace {

struct BarrierOut {
  std::vector<double> params, v_init, mon_rebate, rdbl, tparams;
  std::vector<int32_t> iparams, rint;
  int32_t n_nodes = 0;
  int rc = 0;
  bool operator==(const BarrierOut& o) const {
    return rc == o.rc && n_nodes == o.n_nodes && params == o.params && v_init == o.v_init &&
           mon_rebate == o.mon_rebate && rdbl == o.rdbl && tparams == o.tparams &&
           iparams == o.iparams && rint == o.rint;
  }
};

BarrierOut barrier_plan(int R, int n_space, int n_time) {
  std::vector<double> row((size_t)R * FDCN_BP_NROW);
  std::vector<int32_t> flag((size_t)R * FDCN_BP_NFLAG);
  for (int i = 0; i < R; ++i) {
    double* r = &row[(size_t)i * FDCN_BP_NROW];
    int32_t* f = &flag[(size_t)i * FDCN_BP_NFLAG];
    r[FDCN_BP_SPOT] = 229.74;
    r[FDCN_BP_STRIKE] = 150.0 + 150.0 * (i % 97) / 96.0;
    r[FDCN_BP_SIGMA] = 0.15 + 0.3 * (i % 31) / 30.0;
    r[FDCN_BP_LO] = 229.74 * (0.6 + 0.38 * (i % 13) / 12.0);
    r[FDCN_BP_UP] = 229.74 * (1.02 + 0.48 * (i % 17) / 16.0);
    r[FDCN_BP_CARRY] = r[FDCN_BP_DISC] = 0.0705;
    r[FDCN_BP_DIVY] = r[FDCN_BP_PV] = r[FDCN_BP_REBATE] = 0.0;
    f[FDCN_BP_PUT] = i % 2;
    f[FDCN_BP_KO] = 1 + i % 3;
    f[FDCN_BP_HAS_LO] = f[FDCN_BP_KO] != 2;
    f[FDCN_BP_HAS_UP] = f[FDCN_BP_KO] != 1;
  }
  std::vector<int32_t> mon;
  for (int k = 1; k <= n_time; k += n_time / 23) mon.push_back(k);
  const int Q = 2 * R, nm = (int)mon.size();
  BarrierOut o;
  o.params.resize((size_t)Q * FDCN_NPARAM);
  o.iparams.resize((size_t)Q * FDCN_NIPARAM);
  o.v_init.resize((size_t)Q * n_space);
  o.mon_rebate.resize((size_t)Q * nm);
  o.rint.resize((size_t)Q * FDCN_GK_NRINT);
  o.rdbl.resize((size_t)Q * FDCN_GK_NRDBL);
  o.tparams.resize((size_t)R * FDCN_GK_NPARAM);
  o.rc = fdcn_barrier_plan(R, row.data(), flag.data(), 31.0 / 365.0, n_space, n_time, 1, n_space,
                           4.264890793923841, 1e-4, 1, nm, mon.data(), o.params.data(),
                           o.iparams.data(), o.v_init.data(), o.mon_rebate.data(), o.rint.data(),
                           o.rdbl.data(), o.tparams.data(), &o.n_nodes);
  return o;
}

struct AmericanOut {
  std::vector<double> params, payoff, s_nodes, rdbl, gout;
  std::vector<int32_t> iparams, rint;
  int rc = 0;
  bool operator==(const AmericanOut& o) const {
    return rc == o.rc && params == o.params && payoff == o.payoff && s_nodes == o.s_nodes &&
           rdbl == o.rdbl && gout == o.gout && iparams == o.iparams && rint == o.rint;
  }
};

AmericanOut american_plan(int J, int n_space) {
  std::vector<double> job((size_t)J * FDCN_AP_NJOB);
  std::vector<int32_t> call(J);
  for (int j = 0; j < J; ++j) {
    double* q = &job[(size_t)j * FDCN_AP_NJOB];
    q[FDCN_AP_SPOT] = 176.39 * (0.9 + 0.2 * (j % 11) / 10.0);
    q[FDCN_AP_STRIKE] = 150.0 + 50.0 * (j % 7) / 6.0;
    q[FDCN_AP_SIGMA] = 0.2 + 0.2 * (j % 5) / 4.0;
    q[FDCN_AP_CARRY] = q[FDCN_AP_DISC] = 0.0705;
    call[j] = j % 2;
  }
  const size_t n1 = (size_t)n_space + 1;
  AmericanOut o;
  o.params.resize((size_t)J * FDCN_NPARAM);
  o.iparams.resize((size_t)J * FDCN_NIPARAM);
  o.payoff.resize((size_t)J * n1);
  o.s_nodes.resize((size_t)J * n1);
  o.rint.resize((size_t)2 * J * FDCN_GK_NRINT);
  o.rdbl.resize((size_t)2 * J * FDCN_GK_NRDBL);
  o.gout.resize((size_t)J * FDCN_AP_NOUT);
  o.rc = fdcn_american_plan(J, job.data(), call.data(), n_space, 4.5, 31.0 / 365.0,
                            o.params.data(), o.iparams.data(), o.payoff.data(), o.s_nodes.data(),
                            o.rint.data(), o.rdbl.data(), o.gout.data());
  return o;
}

std::vector<double> jump(int n) {
  std::vector<double> s(n), v(n), out(n);
  for (int i = 0; i < n; ++i) {
    s[i] = exp(log(40.0) + i * (log(400.0) - log(40.0)) / (n - 1));
    v[i] = s[i] > 170.0 ? 0.0 : 170.0 - s[i];
  }
  if (fdcn_dividend_jump(n, s.data(), v.data(), 2.5, -1.0, out.data()) != FDCN_OK) out.clear();
  return out;
}

}  // namespace

int main() {
  int bad = 0;
  const BarrierOut b0 = barrier_plan(600, 1024, 2000);
  const AmericanOut a0 = american_plan(400, 2048);
  const std::vector<double> j0 = jump(2049);
  if (b0.rc || a0.rc || j0.empty()) {
    fprintf(stderr, "plan_driver: a sequential call failed (%d %d): %s\n", b0.rc, a0.rc,
            fdcn_last_error());
    return 2;
  }
  // two callers at once, each fanning out over the builders' own threads
  BarrierOut b1, b2;
  AmericanOut a1, a2;
  std::vector<double> j1, j2;
  std::thread t1([&] { b1 = barrier_plan(600, 1024, 2000); a1 = american_plan(400, 2048); j1 = jump(2049); });
  std::thread t2([&] { a2 = american_plan(400, 2048); b2 = barrier_plan(600, 1024, 2000); j2 = jump(2049); });
  t1.join();
  t2.join();
  if (!(b1 == b0) || !(b2 == b0)) { fprintf(stderr, "barrier plan differs\n"); ++bad; }
  if (!(a1 == a0) || !(a2 == a0)) { fprintf(stderr, "american plan differs\n"); ++bad; }
  if (j1 != j0 || j2 != j0) { fprintf(stderr, "dividend jump differs\n"); ++bad; }
  // error paths: message per thread, nothing written out of bounds
  double t[4];
  if (fdcn_tau_sequence(0.0, 0.01, -1, t) != FDCN_EINVAL) ++bad;
  if (fdcn_tau_sequence(0.5, 1e-3, 4, t) != FDCN_OK || !(t[3] > t[0])) ++bad;
  printf("plan_driver: %s (barrier n_nodes %d)\n", bad ? "FAILED" : "ok", b0.n_nodes);
  return bad ? 1 : 0;
}
