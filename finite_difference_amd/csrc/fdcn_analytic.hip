// fdcn_analytic.hip -- batched closed-form barrier engines for gfx950.
//
// The analytic side of the hot path's boundary: the
// knock-in parity legs and the continuous-monitoring cross-checks price
// thousands of contracts with closed forms.  One thread per contract; fp64
// throughout.
//
//   fdcn_rr_barrier_*      Reiner-Rubinstein single barrier with rebate and
//                          "crossed" status (barrier_engine.py:38-190)
//   fdcn_double_barrier_*  Ikeda-Kunitomo / Douady series, n = -m..m
//                          (double _barrier.py:33-134)
//
// The expressions follow the host engines in finite_difference_amd/analytic.py
// term by term; N(x) = erfc(-x/sqrt 2)/2 (scipy's ndtr).  Device erfc/exp/log
// differ from glibc in the last ulps, so results agree with the host engines
// to ~1e-14 relative, not bitwise.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/fdcn.h"

namespace {

__device__ __forceinline__ double ncdf(double x) { return 0.5 * erfc(-x * M_SQRT1_2); }

// leg(w, arg_s, arg_x, pw_s, pw_x) of analytic.py:97-98
__device__ __forceinline__ double leg(double phi, double s, double ebmt, double x, double erT,
                                      double w, double arg_s, double arg_x, double pw_s,
                                      double pw_x) {
  return phi * s * ebmt * pw_s * ncdf(w * arg_s) - phi * x * erT * pw_x * ncdf(w * arg_x);
}

__global__ void __launch_bounds__(256) rr_barrier_kernel(int32_t B, const double* __restrict__ P,
                                                         const int32_t* __restrict__ F,
                                                         double* __restrict__ price,
                                                         double* __restrict__ vanilla) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const double* p = P + (size_t)i * FDCN_RR_NPARAM;
  const int32_t* f = F + (size_t)i * FDCN_RR_NFLAG;
  const double s = p[0], b = p[1], r = p[2], t = p[3], x = p[4], sig = p[5], h = p[6],
               K = p[7];
  const bool call = f[0] == 0, up = f[1] == 0, in = f[2] == 0, crossed = f[3] == 1;
  const bool reb_in_hit = (f[4] & 1) != 0, reb_out_expiry = (f[4] & 2) != 0;
  const double phi = call ? 1.0 : -1.0;
  const double eta = up ? -1.0 : 1.0;

  const double sqrtT = sqrt(t);
  const double sigRT = sig * sqrtT;
  const double ebmt = exp((b - r) * t);
  const double erT = exp(-r * t);
  const double mu = (b - 0.5 * (sig * sig)) / (sig * sig);
  const double lam = sqrt(mu * mu + 2.0 * r / (sig * sig));
  const double lead = (1.0 + mu) * sigRT;
  const double x1 = log(s / x) / sigRT + lead;
  const double x2 = log(s / h) / sigRT + lead;
  const double y1 = log((h * h) / (s * x)) / sigRT + lead;
  const double y2 = log(h / s) / sigRT + lead;
  const double z = log(h / s) / sigRT + lam * sigRT;
  const double hs = h / s;
  const double p2mu1 = pow(hs, 2.0 * (mu + 1.0)), p2mu = pow(hs, 2.0 * mu);
  const double pml = pow(hs, mu + lam), pmnl = pow(hs, mu - lam);

  const double A = leg(phi, s, ebmt, x, erT, phi, x1, x1 - sigRT, 1.0, 1.0);
  const double Bf = leg(phi, s, ebmt, x, erT, phi, x2, x2 - sigRT, 1.0, 1.0);
  const double C = leg(phi, s, ebmt, x, erT, eta, y1, y1 - sigRT, p2mu1, p2mu);
  const double D = leg(phi, s, ebmt, x, erT, eta, y2, y2 - sigRT, p2mu1, p2mu);
  const double E = K * erT * (ncdf(eta * (x2 - sigRT)) - p2mu * ncdf(eta * (y2 - sigRT)));
  const double Fh = K * (pml * ncdf(eta * z) + pmnl * ncdf(eta * (z - 2.0 * lam * sigRT)));
  vanilla[i] = A;

  if (crossed) {  // barrier_engine.py: knocked in = vanilla; knocked out = rebate
    price[i] = in ? A : (reb_out_expiry ? K * erT : K);
    return;
  }
  const double reb_in = reb_in_hit ? Fh : E;
  const double reb_out = reb_out_expiry ? (K * erT - E) : Fh;
  const bool x_gt_h = (x - h) > 1e-14;
  double base;
  // (option, direction, in/out) -> value if X > H, value otherwise (analytic.py:120-125)
  if (call && !up && in) base = x_gt_h ? C : A - Bf + D;
  else if (call && !up && !in) base = x_gt_h ? A - C : Bf - D;
  else if (call && up && in) base = x_gt_h ? A : Bf - C + D;
  else if (call && up && !in) base = x_gt_h ? 0.0 : A - Bf + C - D;
  else if (!call && !up && in) base = x_gt_h ? Bf - C + D : A;
  else if (!call && !up && !in) base = x_gt_h ? A - Bf + C - D : 0.0;
  else if (!call && up && in) base = x_gt_h ? A - Bf + D : C;
  else base = x_gt_h ? Bf - D : A - C;
  price[i] = base + (in ? reb_in : reb_out);
}

// sum over n = -m..m of I_n - J_n (analytic.py:161-172)
__device__ double db_series(int m, double lam, double alpha, double beta, double u, double delta,
                            double sq) {
  double tot = 0.0;
  for (int n = -m; n <= m; ++n) {
    const double sh = 2.0 * n * delta;
    const double I_ = exp(-2.0 * n * lam * delta) *
                      (ncdf((beta + sh) / sq - lam * sq) - ncdf((alpha + sh) / sq - lam * sq));
    const double J_ = exp(2.0 * lam * (n * delta + u)) *
                      (ncdf((2.0 * u - alpha + sh) / sq + lam * sq) -
                       ncdf((2.0 * u - beta + sh) / sq + lam * sq));
    tot += I_ - J_;
  }
  return tot;
}

__device__ double gbs(bool call, double S, double K, double r, double b, double sig, double T) {
  const double sq = sqrt(T);
  const double d1 = (log(S / K) + (b + 0.5 * (sig * sig)) * T) / (sig * sq);
  const double d2 = d1 - sig * sq;
  if (call) return S * exp((b - r) * T) * ncdf(d1) - K * exp(-r * T) * ncdf(d2);
  return K * exp(-r * T) * ncdf(-d2) - S * exp((b - r) * T) * ncdf(-d1);
}

__global__ void __launch_bounds__(256) double_barrier_kernel(int32_t B, int32_t m,
                                                             const double* __restrict__ P,
                                                             const int32_t* __restrict__ F,
                                                             double* __restrict__ price) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const double* p = P + (size_t)i * FDCN_DB_NPARAM;
  const int32_t* f = F + (size_t)i * FDCN_DB_NFLAG;
  const double S = p[0], X = p[1], L = p[2], U = p[3], sig = p[4], b = p[5], r = p[6],
               T = p[7];
  const bool call = f[0] == 0, in = f[1] == 0, corrected = f[2] != 0;
  const double bs = gbs(call, S, X, r, b, sig, T);
  const double u = log(U / S) / sig;
  const double k = log(X / S) / sig;
  const double l = log(L / S) / sig;
  const double lam = b / sig - sig / 2.0;
  const double lam_p = b / sig + sig / 2.0;
  const double delta = u - l;
  const double sq = sqrt(T);
  double out = 0.0;
  if (call) {
    if (X < U) {
      const double alpha = fmax(k, l), beta = u;
      const double p1 = db_series(m, lam_p, alpha, beta, u, delta, sq);
      const double p2 = db_series(m, lam, alpha, beta, u, delta, sq);
      out = exp((b - r) * T) * S * p1 - exp(-r * T) * X * p2;
    }
  } else if (X > L) {
    const double alpha = corrected ? l : 1.0;  // the reference's put uses 1 (:95)
    const double beta = fmin(k, u);
    const double p1 = db_series(m, lam, alpha, beta, u, delta, sq);
    const double p2 = db_series(m, lam_p, alpha, beta, u, delta, sq);
    out = exp(-r * T) * X * p1 - exp((b - r) * T) * S * p2;
  }
  price[i] = in ? bs - out : out;
}

}  // namespace

namespace fdcn_internal {
int set_error(int code, const char* msg);  // fdcn_kernels.hip (fdcn_last_error)
}

namespace {

int afail(int code, const char* msg) { return fdcn_internal::set_error(code, msg); }

int check_flags(int32_t B, const int32_t* F, int nflag, int maxes0, int maxes1) {
  for (int32_t i = 0; i < B; ++i) {
    const int32_t* f = F + (size_t)i * nflag;
    if (f[0] < 0 || f[0] > 1 || f[1] < 0 || f[1] > maxes0 || f[2] < 0 || f[2] > maxes1)
      return afail(FDCN_EINVAL, "analytic batch: flag out of range");
  }
  return FDCN_OK;
}

template <typename Launch>
int host_run(int32_t B, size_t np, size_t nf, size_t nout, const double* P, const int32_t* F,
             double* out0, double* out1, Launch launch) {
  if (B == 0) return FDCN_OK;
  double *dP = nullptr, *dO = nullptr;
  int32_t* dF = nullptr;
  const size_t nb = (size_t)B;
  int rc = FDCN_OK;
  if (hipMalloc((void**)&dP, sizeof(double) * nb * np) != hipSuccess ||
      hipMalloc((void**)&dF, sizeof(int32_t) * nb * nf) != hipSuccess ||
      hipMalloc((void**)&dO, sizeof(double) * nb * nout) != hipSuccess) {
    rc = afail(FDCN_ENOMEM, "analytic batch: hipMalloc failed");
  }
  if (rc == FDCN_OK &&
      (hipMemcpy(dP, P, sizeof(double) * nb * np, hipMemcpyHostToDevice) != hipSuccess ||
       hipMemcpy(dF, F, sizeof(int32_t) * nb * nf, hipMemcpyHostToDevice) != hipSuccess))
    rc = afail(FDCN_EHIP, "analytic batch: H2D copy failed");
  if (rc == FDCN_OK) {
    launch(dP, dF, dO, dO + (nout > 1 ? nb : 0), (hipStream_t) nullptr);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      rc = afail(FDCN_EHIP, "analytic batch: kernel failed");
  }
  if (rc == FDCN_OK &&
      (hipMemcpy(out0, dO, sizeof(double) * nb, hipMemcpyDeviceToHost) != hipSuccess ||
       (out1 && hipMemcpy(out1, dO + nb, sizeof(double) * nb, hipMemcpyDeviceToHost) !=
                    hipSuccess)))
    rc = afail(FDCN_EHIP, "analytic batch: D2H copy failed");
  if (dP) (void)hipFree(dP);
  if (dF) (void)hipFree(dF);
  if (dO) (void)hipFree(dO);
  return rc;
}

}  // namespace

extern "C" {

int fdcn_rr_barrier_batch_dev(int32_t B, const double* params, const int32_t* flags,
                              double* price, double* vanilla, void* stream) {
  if (B < 0) return afail(FDCN_EINVAL, "B must be >= 0");
  if (B == 0) return FDCN_OK;
  hipLaunchKernelGGL(rr_barrier_kernel, dim3((B + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, B, params, flags, price, vanilla);
  return hipGetLastError() == hipSuccess ? FDCN_OK : afail(FDCN_EHIP, "launch failed");
}

int fdcn_rr_barrier_batch(int32_t B, const double* params, const int32_t* flags, double* price,
                          double* vanilla) {
  if (B < 0 || (B > 0 && (!params || !flags || !price || !vanilla)))
    return afail(FDCN_EINVAL, "rr_barrier_batch: bad arguments");
  int rc = check_flags(B, flags, FDCN_RR_NFLAG, 1, 1);
  if (rc) return rc;
  for (int32_t i = 0; i < B; ++i) {
    const int32_t* f = flags + (size_t)i * FDCN_RR_NFLAG;
    if (f[3] < 0 || f[3] > 1 || f[4] < 0 || f[4] > 3)
      return afail(FDCN_EINVAL, "rr_barrier_batch: status/rebate flag out of range");
    const double* p = params + (size_t)i * FDCN_RR_NPARAM;
    if (!(p[5] > 0.0) || !(p[3] > 0.0))
      return afail(FDCN_EINVAL, "rr_barrier_batch: sigma and t must be positive");
  }
  return host_run(B, FDCN_RR_NPARAM, FDCN_RR_NFLAG, 2, params, flags, price, vanilla,
                  [&](const double* dP, const int32_t* dF, double* o0, double* o1, hipStream_t s) {
                    hipLaunchKernelGGL(rr_barrier_kernel, dim3((B + 255) / 256), dim3(256), 0, s,
                                       B, dP, dF, o0, o1);
                  });
}

int fdcn_double_barrier_batch_dev(int32_t B, int32_t m, const double* params,
                                  const int32_t* flags, double* price, void* stream) {
  if (B < 0 || m < 0) return afail(FDCN_EINVAL, "B and m must be >= 0");
  if (B == 0) return FDCN_OK;
  hipLaunchKernelGGL(double_barrier_kernel, dim3((B + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, B, m, params, flags, price);
  return hipGetLastError() == hipSuccess ? FDCN_OK : afail(FDCN_EHIP, "launch failed");
}

int fdcn_double_barrier_batch(int32_t B, int32_t m, const double* params, const int32_t* flags,
                              double* price) {
  if (B < 0 || m < 0 || (B > 0 && (!params || !flags || !price)))
    return afail(FDCN_EINVAL, "double_barrier_batch: bad arguments");
  int rc = check_flags(B, flags, FDCN_DB_NFLAG, 1, 1);
  if (rc) return rc;
  return host_run(B, FDCN_DB_NPARAM, FDCN_DB_NFLAG, 1, params, flags, price, nullptr,
                  [&](const double* dP, const int32_t* dF, double* o0, double*, hipStream_t s) {
                    hipLaunchKernelGGL(double_barrier_kernel, dim3((B + 255) / 256), dim3(256),
                                       0, s, B, m, dP, dF, o0);
                  });
}

}  // extern "C"
