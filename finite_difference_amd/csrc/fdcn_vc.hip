// fdcn_vc.hip -- spot-space Crank-Nicolson with per-row coefficients (gfx950).
//
// Replaces the time loops of
//   DiscreteBarrierFDMPricer2._solve_pde_backward   discrete_barrier_fdm_pricer_2.py:336-428
//   DiscreteBarrierFDMPricerAnalytic._cn_stepper    discrete_barrier_analytic_pricer.py:384-432
// On a uniform S grid every row of the theta-scheme matrices is different
// (sigma^2 S_i^2 / dS^2, r S_i / dS, and the FIS non-symmetric rows next to
// the barrier), but a row does not change in time within a phase (the
// Rannacher steps, then Crank-Nicolson).  So the LU factors of each phase
// are computed once per launch (one serial Thomas forward sweep per phase,
// the reference's order) and stored scaled: with g_i = 1/beta_i
//   d_i = g_i rhs_i + f_i d_{i-1},  f_i = -sub_i g_i          (forward)
//   x_i = d_i + e_i x_{i+1},        e_i = -sup_i / beta_i     (backward)
// and g_i folded into the explicit stencil, rhs'_i = A_i V_{i-1} + B_i V_i +
// C_i V_{i+1}.  Per step and node: 3 FMAs for the stencil, 2 + 2 for the two
// affine recurrences (zero-carry pass, carry scan over lanes, second pass),
// everything in registers; no per-step division.
//
// Mapping: one scenario per workgroup of W waves; thread t owns NPT
// consecutive slots; node i sits at slot i + pad_lo (padding split between
// both ends).  The Dirichlet rows 0 and n-1 (sub = sup = 0) are not solved
// as rows: the bottom value g_0 lo enters as the forward carry-in at slot 0
// and passes through the lower padding and node 0 (multiplier 1, rhs 0);
// the top value g_{n-1} hi enters as the backward carry-in at the last slot
// and passes through the upper padding and node n-1.  So neither boundary
// needs a per-slot select.  A grid one node longer than the slots (the
// reference's N + 1 nodes on N = 64 W NPT, e.g. 1 025 nodes in 1 024
// slots) keeps node 0 out of the slots (pad_lo = -1): its value is the
// forward carry-in g_0 lo itself, held as one uniform scalar that feeds the
// stencil of node 1 on the next step (bitwise what the slot would hold).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <type_traits>

#include "../../include/fdcn.h"

namespace fdcn_internal {
int set_error(int code, const char* msg);
int validate_plan(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, int32_t n_mon,
                  const int32_t* mon_step, const double* mon_rebate);
int thread_stream(hipStream_t* out);
}  // namespace fdcn_internal

namespace {

int vfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fdcn_internal::set_error(code, buf);
}

#define V_TRY(expr)                                                                \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return vfail(FDCN_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

__device__ __forceinline__ double uni(double x) {
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
template <int CTRL>
__device__ __forceinline__ double dpp_move(double x) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double bperm(double x, int addr) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(b & 0xffffffffull));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(b >> 32));
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// lane i <- lane i - d (d = 1: DPP wave_shr, lane 0 receives 0), i + d
__device__ __forceinline__ double from_below(double x, int d, int lane4) {
  if (d == 1) return dpp_move<0x138>(x);
  return bperm(x, lane4 - 4 * d);
}
__device__ __forceinline__ double from_above(double x, int d, int lane4) {
  if (d == 1) return dpp_move<0x130>(x);
  return bperm(x, lane4 + 4 * d);
}

// 64-bit row-masked DPP move (two 32-bit moves): lanes without a source in
// their row, and rows outside RM, receive 0
template <int CTRL, int RM>
__device__ __forceinline__ double dpp64(double x) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), CTRL, RM, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, RM, 0xF, true);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
constexpr int kRowShr = 0x110, kRowShl = 0x100, kRowBcast15 = 0x142, kRowBcast31 = 0x143;
// 64-bit DPP move whose lanes without a source keep `old` (bound_ctrl off):
// wave_shr:1 with old = the carry gives lane 0 the carry without a select
template <int CTRL>
__device__ __forceinline__ double dpp64_old(double old, double x) {
  const unsigned long long o = __double_as_longlong(old), b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffull), (int)(b & 0xffffffffull),
                                             CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

constexpr int kNC = 5;  // per-slot coefficient arrays: A, B, C, f, e (stencil form);
                        // the pointwise form uses B := g (b - alpha main), f, e
constexpr int kNS = 20; // per-scenario scalars: phase p at 8p: g0, gN, alpha, ra(i1),
                        // rc(i1), ra(i1+1), rc(i1+1); [16] form (1 pointwise), [17] i1

struct VcArgs {
  int B, n, n_time, n_ranna, slots, pad_lo, force_stencil;
  const double* diag;     // [B][2][6][n]
  const double* bnd;      // [B][n_time][2]
  const double* v_init;   // [B][n]
  const int32_t* iparams; // [B][FDCN_NIPARAM]
  const int32_t* mon_step;
  const double* mon_rebate;
  double* v_out;
  double* coef;           // workspace [B]([2][kNC][slots] + kNS)
};

__device__ __forceinline__ size_t ws_scen(const VcArgs& A) {
  return 2 * kNC * (size_t)A.slots + kNS;
}

// ---------------------------------------------------------------------------
// The pointwise (theta) form.  Write the explicit rows as a multiple of the
// implicit ones: a_i = alpha sub_i + ra_i, c_i = alpha sup_i + rc_i,
// b_i = alpha main_i + beta_i.  Then with u = x - alpha V the step's system
// A x = B V (+ Dirichlet rows) becomes A u = beta V + E V with E nonzero only
// in the rows where the residuals ra / rc are not exactly 0, and u's
// Dirichlet values are g0 lo - alpha V_0 and gN hi - alpha V_{n-1}: the
// right-hand side is pointwise (no stencil, no neighbour exchange) except in
// those rows, and x = alpha V + u.  The reference's spot-space rows
// (discrete_barrier_fdm_pricer_2.py:354-417, discrete_barrier_analytic_
// pricer.py:408-423) have alpha = -+(1-theta)/theta on every uniform row --
// exactly, both operands are the same product -- and the two one-sided rows
// beside the barrier (:388-410) the opposite sign: so a Pricer2 scenario has
// at most two such rows, adjacent, and every analytic-overlay scenario none.
// Any other coefficient set takes the stencil form.  Per node-step the
// pointwise form issues 6 VALU (1 multiply, 2 + 2 for the two affine passes
// of each recurrence, 1 update) against the stencil form's 7, and keeps 3
// coefficients a slot in registers instead of 5.
//
// fdcn_vc_factor: one workgroup per scenario, one wave per phase.  The wave
// classifies its phase (alpha from one of three candidate rows, the
// exceptional rows counted lane-parallel), the two waves agree the form,
// and each writes its factored rows in the form the march will use.  The
// Thomas pivots c*_i = sup_i / (main_i - sub_i c*_{i-1}) (the reference's
// _solve_tridiagonal order) form a first-order rational recurrence: in
// projective form (p, q)_i = (sup_i q, main_i q - sub_i p)_{i-1}, c* = p/q,
// a product of 2x2 matrices.  The wave walks the rows in groups of 64
// consecutive rows, one per lane (every load and store coalesced): a
// Hillis-Steele scan over the lanes gives each row the product of its
// group up to it, times the product of all earlier groups (carried), so
// each lane has c*_{i-1} for its row and takes the reference's step from
// it.  The recurrence contracts (|dc*_i / dc*_{i-1}| = |sub_i sup_i| /
// beta_i^2 < 1 on these diagonally dominant rows), so the pivots equal the
// serial sweep's to rounding.
// ---------------------------------------------------------------------------
__host__ __device__ double row_ratio(const double* P, int n, int i) {
  const double sub = P[i], sup = P[2 * n + i], ae = P[3 * n + i], ce = P[5 * n + i];
  return sub != 0.0 ? ae / sub : (sup != 0.0 ? ce / sup : 0.0);
}

// One phase's classification: alpha and its exceptional rows (count, stops
// at 3; first; last).  ok: at most two, adjacent.
struct PhaseClass {
  double alpha;
  int cnt, first, last, ok;
};

__host__ __device__ PhaseClass classify_phase(const double* P, int n, bool used,
                                              bool force_stencil) {
  PhaseClass pc{0.0, 0, 0x7fffffff, -1, force_stencil ? 0 : 1};
  if (!used || force_stencil) return pc;  // an unused phase has no exceptions
  const int cand[3] = {n / 2, 1, n - 2};
  for (int c = 0; c < 3; ++c) {
    pc.alpha = row_ratio(P, n, cand[c]);
    pc.cnt = 0;
    pc.first = 0x7fffffff;
    pc.last = -1;
    for (int i = 1; i < n - 1 && pc.cnt < 3; ++i) {
      const double ra = P[3 * n + i] - pc.alpha * P[i];
      const double rc = P[5 * n + i] - pc.alpha * P[2 * n + i];
      if (ra != 0.0 || rc != 0.0) {
        ++pc.cnt;
        if (i < pc.first) pc.first = i;
        pc.last = i;
      }
    }
    pc.ok = pc.cnt <= 2 && (pc.cnt == 0 || pc.last - pc.first <= 1);
    if (pc.ok) break;
  }
  return pc;
}

// One form per scenario: the pointwise form when both phases classify and
// their exceptional rows lie within {i1, i1 + 1}; *i1 = -1 for none.
__host__ __device__ bool pointwise_form(int ok0, int first0, int last0, int ok1, int first1,
                                        int last1, int* i1) {
  const int f = first0 < first1 ? first0 : first1;
  const bool none = last0 < 0 && last1 < 0;
  const bool pw = ok0 && ok1 && (none || (last0 <= f + 1 && last1 <= f + 1));
  *i1 = (pw && !none) ? f : -1;
  return pw;
}

// 2x2 matrix, row-major: [a b; c d]
struct M2 {
  double a, b, c, d;
};
__device__ __forceinline__ M2 mmul(const M2& x, const M2& y) {  // x * y
  return M2{fma(x.a, y.a, x.b * y.c), fma(x.a, y.b, x.b * y.d), fma(x.c, y.a, x.d * y.c),
            fma(x.c, y.b, x.d * y.d)};
}
// projective scaling by a power of two (exact): largest |entry| into [1, 2)
__device__ __forceinline__ M2 mnorm(const M2& x) {
  const double m = fmax(fmax(fabs(x.a), fabs(x.b)), fmax(fabs(x.c), fabs(x.d)));
  if (!(m > 0.0) || !isfinite(m)) return x;
  const int e = ilogb(m);
  return M2{ldexp(x.a, -e), ldexp(x.b, -e), ldexp(x.c, -e), ldexp(x.d, -e)};
}
__device__ __forceinline__ double shfl_d(double x, int src) {
  return __shfl(x, src);
}

// Step 3 of the factor kernel, one phase: the factored rows, 64 consecutive
// rows at a time (see above).  kFast: the single pass -- the pointwise form
// at the candidate alpha assumed, the phase classified on the rows as they
// are factored (count, first and last exceptional row; the first two rows'
// residuals recorded in xi / xv, since i1 is known only once both phases
// are); otherwise the form, alpha and i1 are known and the residuals of rows
// i1 and i1 + 1 go straight to sc.
struct FactorClass {
  int cnt, first, last;
};

template <bool kFast>
__device__ __forceinline__ FactorClass factor_rows(const double* P, int n, int slots, int pad_lo,
                                                   int lane, bool pw, double alpha, int i1,
                                                   double* C, double* sc, int* xi, double* xv) {
  const double *sub = P, *mn = P + n, *sup = P + 2 * n;
  const double *ae = P + 3 * n, *be = P + 4 * n, *ce = P + 5 * n;
  const bool none = i1 < 0;
  double* cA = C;
  double* cB = C + slots;
  double* cC = C + 2 * slots;
  double* cf = C + 3 * slots;
  double* cE = C + 4 * slots;
  for (int s = lane; s < pad_lo; s += 64) {  // lower padding: pass the forward carry up
    if (!pw) cA[s] = cC[s] = 0.0;
    cB[s] = 0.0;
    cf[s] = 1.0;
    cE[s] = 0.0;
  }
  for (int s = pad_lo + n + lane; s < slots; s += 64) {  // upper padding: carry down
    if (!pw) cA[s] = cC[s] = 0.0;
    cB[s] = 0.0;
    cf[s] = 0.0;
    cE[s] = 1.0;
  }
  FactorClass fc{0, 0x7fffffff, -1};
  M2 carry{1.0, 0.0, 0.0, 1.0};  // the product of every earlier group's matrices
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const bool row = i < n;
    const double sb = row ? sub[i] : 0.0, m = row ? mn[i] : 1.0, sp = row ? sup[i] : 0.0;
    M2 T = row ? M2{0.0, sp, -sb, m} : M2{1.0, 0.0, 0.0, 1.0};
    for (int d = 1; d < 64; d <<= 1) {  // inclusive: rows base..i, later rows on the left
      const M2 X{shfl_d(T.a, lane - d), shfl_d(T.b, lane - d), shfl_d(T.c, lane - d),
                 shfl_d(T.d, lane - d)};
      if (lane >= d) T = mnorm(mmul(T, X));
    }
    const M2 Pi = mnorm(mmul(T, carry));  // rows 0..i
    // c* of row i-1: the previous lane's product, or the carry for lane 0,
    // applied to (p, q) = (0, 1)
    double pb = shfl_d(Pi.b, lane - 1), qb = shfl_d(Pi.d, lane - 1);
    if (lane == 0) {
      pb = carry.b;
      qb = carry.d;
    }
    carry = M2{shfl_d(Pi.a, 63), shfl_d(Pi.b, 63), shfl_d(Pi.c, 63), shfl_d(Pi.d, 63)};
    const bool interior = row && i > 0 && i < n - 1;
    // kFast: this group's exceptional rows (residual not exactly zero)
    double ra = 0.0, rc = 0.0;
    bool exc = false;
    int pre = 2;
    if constexpr (kFast) {
      if (interior) {
        ra = ae[i] - alpha * sb;
        rc = ce[i] - alpha * sp;
        exc = ra != 0.0 || rc != 0.0;
      }
      const unsigned long long bal = __ballot(exc);
      if (bal) {
        if (fc.cnt == 0) fc.first = base + __ffsll((long long)bal) - 1;
        fc.last = base + 63 - __clzll((long long)bal);
        pre = fc.cnt + __popcll(bal & ((1ull << lane) - 1ull));
        fc.cnt += __popcll(bal);
      }
    }
    if (!row) continue;
    const double cprev = i > 0 ? pb / qb : 0.0;
    const double beta = (i == 0) ? m : m - sb * cprev;
    const double g = 1.0 / beta;
    const double cs = (i < n - 1) ? sp / beta : 0.0;
    if (i == 0) sc[0] = g;
    if (i == n - 1) sc[1] = g;
    if constexpr (kFast) {
      if (exc && pre < 2) {
        xi[pre] = i;
        xv[2 * pre] = g * ra;
        xv[2 * pre + 1] = g * rc;
      }
    } else if (pw && interior && !none && (i == i1 || i == i1 + 1)) {
      sc[3 + 2 * (i - i1)] = g * (ae[i] - alpha * sb);
      sc[4 + 2 * (i - i1)] = g * (ce[i] - alpha * sp);
    }
    const int s = i + pad_lo;
    if (s < 0) continue;  // node 0 outside the slots (pad_lo = -1)
    if (pw) {
      cB[s] = interior ? g * (be[i] - alpha * m) : 0.0;
    } else {
      cA[s] = interior ? ae[i] * g : 0.0;
      cB[s] = interior ? be[i] * g : 0.0;
      cC[s] = interior ? ce[i] * g : 0.0;
    }
    // node 0 takes the forward carry as its value; node n-1 the backward
    // one; interior rows their factors
    cf[s] = (i == 0) ? 1.0 : (i == n - 1 ? 0.0 : -sb * g);
    cE[s] = (i == n - 1) ? 1.0 : (i == 0 ? 0.0 : -cs);
  }
  return fc;
}

// One workgroup per scenario, one wave per phase.  Round 5: one pass over
// diag for the common case.  Each wave assumes the pointwise form at the
// first candidate alpha (the middle row's ratio), factors its rows in that
// form and classifies them on the way (the rows it reads anyway); if both
// phases then agree on the pointwise form -- every Pricer2 and analytic-
// overlay scenario whose middle row is not beside the barrier -- the
// scenario is done, bitwise what the two-pass path below writes (it would
// pick the same candidate: the first that classifies) -- up to the sign of
// one zero: a row of the pair (i1, i1 + 1) that is not exceptional gets +0.0
// here, where the two-pass path writes its pivot times a zero residual, -0.0
// for a negative pivot; the march only adds these terms, so the
// two differ at most in the sign of an exactly-zero result.  Otherwise (a phase
// not classified at that alpha, the stencil form, or the diagnostics'
// force_stencil) the general path classifies at all three candidates and
// factors again.  diag read 1.0 times instead of ~1.33 per scenario.
__global__ void __launch_bounds__(128) fdcn_vc_factor(VcArgs A) {
  __shared__ int agree[2][3];
  __shared__ int xi[2][2];
  __shared__ double xv[2][4];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int b = blockIdx.x;
  const int n = A.n, slots = A.slots, pad_lo = A.pad_lo;
  const bool used = ph == 0 ? A.n_ranna > 0 : A.n_ranna < A.n_time;
  const double* P = A.diag + ((size_t)b * 2 + ph) * FDCN_VC_NDIAG * n;
  const double *sub = P, *sup = P + 2 * n;
  const double *ae = P + 3 * n, *ce = P + 5 * n;
  double* const scal = A.coef + (size_t)b * ws_scen(A) + 2 * kNC * (size_t)slots;
  double* const C = A.coef + (size_t)b * ws_scen(A) + (size_t)ph * kNC * slots;
  double* const sc = scal + 8 * ph;

  if (!A.force_stencil) {
    const double alpha_c = used ? row_ratio(P, n, n / 2) : 0.0;
    FactorClass fc{0, 0x7fffffff, -1};
    if (used)
      fc = factor_rows<true>(P, n, slots, pad_lo, lane, true, alpha_c, -1, C, sc, xi[ph], xv[ph]);
    const int okf = fc.cnt <= 2 && (fc.cnt == 0 || fc.last - fc.first <= 1);
    if (lane == 0) {
      agree[ph][0] = okf;
      agree[ph][1] = fc.first;
      agree[ph][2] = fc.last;
    }
    __syncthreads();  // also orders the xi / xv stores before their reads
    int i1;
    if (pointwise_form(agree[0][0], agree[0][1], agree[0][2], agree[1][0], agree[1][1],
                       agree[1][2], &i1)) {
      if (ph == 0 && lane == 0) {
        scal[16] = 1.0;
        scal[17] = (double)i1;
      }
      if (used && lane == 0) {
        sc[2] = alpha_c;
        sc[3] = sc[4] = sc[5] = sc[6] = 0.0;
        for (int j = 0; j < fc.cnt && j < 2; ++j) {  // rows i1 / i1 + 1 of this phase
          sc[3 + 2 * (xi[ph][j] - i1)] = xv[ph][2 * j];
          sc[4 + 2 * (xi[ph][j] - i1)] = xv[ph][2 * j + 1];
        }
      }
      return;  // uniform: both waves read the same agree[]
    }
    __syncthreads();  // agree[] is rewritten below
  }

  // the general path: 1. classification, three candidate alphas at once,
  // rows lane-strided
  double al[3] = {0.0, 0.0, 0.0};
  int cnt[3] = {0, 0, 0}, fst[3] = {0x7fffffff, 0x7fffffff, 0x7fffffff}, lst[3] = {-1, -1, -1};
  const bool classify = used && !A.force_stencil;
  if (classify) {
    al[0] = row_ratio(P, n, n / 2);
    al[1] = row_ratio(P, n, 1);
    al[2] = row_ratio(P, n, n - 2);
    for (int i = 1 + lane; i < n - 1; i += 64) {
      const double sb = sub[i], sp = sup[i], a = ae[i], c = ce[i];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if ((a - al[k] * sb) != 0.0 || (c - al[k] * sp) != 0.0) {
          ++cnt[k];
          fst[k] = fst[k] < i ? fst[k] : i;
          lst[k] = i;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
      for (int d = 1; d < 64; d <<= 1) {
        cnt[k] += __shfl_xor(cnt[k], d);
        const int f = __shfl_xor(fst[k], d), l = __shfl_xor(lst[k], d);
        fst[k] = fst[k] < f ? fst[k] : f;
        lst[k] = lst[k] > l ? lst[k] : l;
      }
  }
  int pick = 0, ok = classify ? 0 : (A.force_stencil ? 0 : 1);
  if (classify) {
    for (int k = 2; k >= 0; --k)
      if (cnt[k] <= 2 && (cnt[k] == 0 || lst[k] - fst[k] <= 1)) {
        pick = k;
        ok = 1;
      }
  }
  const double alpha0 = al[pick];
  const int first = (classify && ok) ? fst[pick] : 0x7fffffff;
  const int last = (classify && ok) ? lst[pick] : -1;
  // 2. one form per scenario
  if (lane == 0) {
    agree[ph][0] = ok;
    agree[ph][1] = first;
    agree[ph][2] = last;
  }
  __syncthreads();
  int i1;
  const bool pw = pointwise_form(agree[0][0], agree[0][1], agree[0][2], agree[1][0],
                                 agree[1][1], agree[1][2], &i1);
  if (ph == 0 && lane == 0) {
    scal[16] = pw ? 1.0 : 0.0;
    scal[17] = (double)i1;
  }
  if (!used) return;
  const double alpha = pw ? alpha0 : 0.0;
  if (lane == 0) {
    sc[2] = alpha;
    sc[3] = sc[4] = sc[5] = sc[6] = 0.0;
  }
  // 3. the factored rows
  factor_rows<false>(P, n, slots, pad_lo, lane, pw, alpha, i1, C, sc, nullptr, nullptr);
}

// LDS tables read off a byte address the compiler cannot see through
// (hide_addr): otherwise it hoists the loop-invariant loads into registers
typedef __attribute__((address_space(3))) const double lds_cf64;
__device__ __forceinline__ unsigned lds_addr(const double* p) {
  return (unsigned)(uintptr_t)(lds_cf64*)p;
}
__device__ __forceinline__ double lds_ld(unsigned a, int off) {
  return ((lds_cf64*)(uintptr_t)a)[off];
}
__device__ __forceinline__ unsigned hide_addr(unsigned a) {
  asm volatile("" : "+v"(a));
  return a;
}

// value vectors in registers; a uniform (SGPR) element index compiles to
// s_set_gpr_idx_on + v_mov: the exceptional rows' slot is not a constant
template <int NPT>
using dvec = double __attribute__((ext_vector_type(NPT)));

// <1, 16> of the stencil form needs 256 VGPRs + 31 AGPRs: held to two waves
// per SIMD it spills; it runs only the scenarios the pointwise form declines.
// NPT 8 and 10 of the pointwise form are held to three waves per SIMD: NPT 10
// then spills 124 B a lane, and still runs the reference's default 600 x 600
// grid faster (1.25 -> 1.17 ms for 4 096 trades, profiles/r05/vc_npt10/)
template <int W, int NPT, bool PW>
__global__ void __launch_bounds__(64 * W, (W == 1 && PW && (NPT == 10 || NPT == 8))
                                              ? 3
                                              : ((W == 1 && (PW || NPT == 16)) ? 2 : 1))
    fdcn_vc_march(VcArgs A) {
  __shared__ double xch[6 * W + 2];
  // the twelve lane-scan weights of the phase, [wave][weight][lane]: read
  // from LDS in the step (24 VGPRs fewer; the scans are not LDS-bound)
  __shared__ double swt[W * 12 * 64];
  // the current 64-step block of Dirichlet values, one row per wave: read
  // back as one LDS broadcast per step instead of four v_readlane
  __shared__ double2 bblk[W * 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int lane4 = lane << 2;
  asm volatile("" : "+v"(lane4));
  const int scen = blockIdx.x;
  const int n = A.n, slots = A.slots, pad_lo = A.pad_lo;
  const unsigned sw_a = lds_addr(swt + wave * 12 * 64 + lane);
  double* coef = A.coef + (size_t)scen * ws_scen(A);
  const double* scal = coef + 2 * kNC * (size_t)slots;
  // the factor kernel chose this scenario's form; the other instance runs it
  if ((scal[16] != 0.0) != PW) return;
  const bool use_r = A.n_ranna > 0, use_c = A.n_ranna < A.n_time;

  const int base = t * NPT;  // first slot of this thread
  const int32_t* I = A.iparams + (size_t)scen * FDCN_NIPARAM;
  const int ko_lo = __builtin_amdgcn_readfirstlane(I[FDCN_I_KO_LO]);
  const int ko_hi = __builtin_amdgcn_readfirstlane(I[FDCN_I_KO_HI]);
  // knock-out lane masks per slot, computed once: nodes j <= ko_lo or
  // j >= ko_hi; a padding slot follows the Dirichlet node next to it
  unsigned long long km[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    int j = base + k - pad_lo;
    j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
    km[k] = __ballot(j <= ko_lo || j >= ko_hi);
  }

  // the value vector ping-pongs between VA and VB: a step reads V (old) and
  // leaves the new vector in R, whose registers held its right-hand side and
  // forward sweep -- no copy back (a register tuple cannot be renamed across
  // the loop's back edge)
  dvec<NPT> VA, VB;
  const double* vin = A.v_init + (size_t)scen * n;
  // node 0 outside the slots (stencil form), and the pointwise form
  // everywhere: its value (uniform), and whether it knocks out; the
  // pointwise form tracks node n-1 the same way
  const bool lo_out = pad_lo < 0;
  double v0 = (lo_out || PW) ? uni(vin[0]) : 0.0;
  double vN = PW ? uni(vin[n - 1]) : 0.0;
  const bool ko0 = 0 <= ko_lo || 0 >= ko_hi;
  const bool koN = n - 1 <= ko_lo || n - 1 >= ko_hi;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = base + k - pad_lo;
    VA[k] = (j >= 0 && j < n) ? vin[j] : (j < 0 ? vin[0] : vin[n - 1]);
  }

  double cA[PW ? 1 : NPT], cB[NPT], cC[PW ? 1 : NPT], cf[NPT], ce[NPT];
  // The lane scans of the two recurrences run row-segmented: four DPP
  // stages inside each 16-lane row, then the rows joined -- forward by
  // row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3), backward by one
  // ds_bpermute from the next row's first lane (rows 0, 2) and a readlane
  // of lane 32 (rows 0, 1).  One LDS round trip per step instead of ten.
  // Weights per stage: the products of the multipliers the stage spans.
  const int rl = lane & 15;
  int addrA = (lane & 16) == 0 ? (((lane | 15) + 1) << 2) : lane4;  // rows 0, 2 <- rows 1, 3
  asm volatile("" : "+v"(addrA));
  double Fpre = 0.0, Gsuf = 0.0, g0 = 0.0, gN = 0.0, alpha = 0.0;
  // pointwise form: the exceptional rows i1 (slot k1 of thread t1) and i1+1,
  // their residual coefficients on their own threads only
  const int i1 = PW ? (int)uni(scal[17]) : -1;
  const bool has_exc = PW && i1 >= 0;
  const int s1 = i1 + pad_lo;
  const int k1 = __builtin_amdgcn_readfirstlane(has_exc ? s1 % NPT : 0);
  const int t1 = has_exc ? s1 / NPT : -1, t2 = has_exc ? (s1 + 1) / NPT : -1;
  double ra1 = 0.0, rc1 = 0.0, ra2 = 0.0, rc2 = 0.0;
  // the zero-carry passes run as two half-chunk chains joined by the
  // multiplier product of the other half (upper half forward, lower half
  // backward): half the dependent FMA chain
  constexpr bool kHalf = NPT >= 8;
  constexpr int H = NPT / 2;
  double fh = 1.0, gl = 1.0;
  auto load_phase = [&](int ph) __attribute__((always_inline)) {
    if constexpr (W > 1) __syncthreads();  // previous readers of the wave totals are done
    const double* C = coef + (size_t)ph * kNC * slots;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if constexpr (!PW) {
        cA[k] = C[base + k];
        cC[k] = C[2 * slots + base + k];
      }
      cB[k] = C[slots + base + k];
      cf[k] = C[3 * slots + base + k];
      ce[k] = C[4 * slots + base + k];
    }
    g0 = uni(scal[8 * ph]);
    gN = uni(scal[8 * ph + 1]);
    if constexpr (PW) {
      alpha = uni(scal[8 * ph + 2]);
      if (has_exc) {
        const double a1 = uni(scal[8 * ph + 3]), c1 = uni(scal[8 * ph + 4]);
        const double a2 = uni(scal[8 * ph + 5]), c2 = uni(scal[8 * ph + 6]);
        ra1 = t == t1 ? a1 : 0.0;
        rc1 = t == t1 ? c1 : 0.0;
        ra2 = t == t2 ? a2 : 0.0;
        rc2 = t == t2 ? c2 : 0.0;
      }
    }
    double f = 1.0, g = 1.0;  // products of the multipliers over the chunk
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      f *= cf[k];
      g *= ce[k];
    }
    if constexpr (kHalf) {
      fh = 1.0;
      gl = 1.0;
#pragma unroll
      for (int k = H; k < NPT; ++k) fh *= cf[k];
#pragma unroll
      for (int k = 0; k < H; ++k) gl *= ce[k];
    }
    {
      // weights 0-3: forward row stages; 4-7: backward row stages; 8, 9:
      // forward row joins (bcast15, bcast31); 10, 11: backward joins
      double* sw = swt + wave * 12 * 64 + lane;
      double F = f, G = g, s;
#define VC_ROW_STAGE(j)                                                   \
      sw[(j) * 64] = rl >= (1 << j) ? F : 0.0;                            \
      s = dpp64<kRowShr + (1 << j), 0xF>(F);                              \
      F = rl >= (1 << j) ? F * s : F;                                     \
      sw[(4 + (j)) * 64] = rl + (1 << j) <= 15 ? G : 0.0;                 \
      s = dpp64<kRowShl + (1 << j), 0xF>(G);                              \
      G = rl + (1 << j) <= 15 ? G * s : G;
      VC_ROW_STAGE(0) VC_ROW_STAGE(1) VC_ROW_STAGE(2) VC_ROW_STAGE(3)
#undef VC_ROW_STAGE
      const bool odd = (lane & 16) != 0;
      sw[8 * 64] = odd ? F : 0.0;
      s = dpp64<kRowBcast15, 0xA>(F);
      F = odd ? F * s : F;
      sw[9 * 64] = lane >= 32 ? F : 0.0;
      sw[10 * 64] = odd ? 0.0 : G;
      s = bperm(G, addrA);
      G = odd ? G : G * s;
      sw[11 * 64] = lane < 32 ? G : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      const double fo = from_below(f, d, lane4), go = from_above(g, d, lane4);
      f = (lane >= d) ? f * fo : f;
      g = (lane + d < 64) ? g * go : g;
    }
    Fpre = f;  // product over lanes 0..lane of this wave
    Gsuf = g;  // product over lanes lane..63
    if constexpr (W > 1) {
      if (lane == 63) xch[3 * W + wave] = Fpre;
      if (lane == 0) xch[5 * W + wave] = Gsuf;
      __syncthreads();
    }
  };
  load_phase(use_r ? 0 : 1);

  int mpos = __builtin_amdgcn_readfirstlane(I[FDCN_I_MON_START]);
  const int mend = mpos + __builtin_amdgcn_readfirstlane(I[FDCN_I_MON_COUNT]);
  while (mpos < mend && __builtin_amdgcn_readfirstlane(A.mon_step[mpos]) < 1) ++mpos;
  int next_mon = mpos < mend ? __builtin_amdgcn_readfirstlane(A.mon_step[mpos]) : 0x7fffffff;
  // the next entry's step and rebate are fetched right after a projection
  // (entries at or before the step just projected are skipped there): the
  // loads have a whole step to land instead of stalling the projection
  double next_reb = mpos < mend ? uni(A.mon_rebate[mpos]) : 0.0;

  const double2* bnd = reinterpret_cast<const double2*>(A.bnd) + (size_t)scen * A.n_time;
  const unsigned bb_a = lds_addr(reinterpret_cast<const double*>(bblk + wave * 64));
  // one step; the march runs it in two loops (Rannacher phase, then CN) so
  // the phase switch is not a branch in the step -- inside it the compiler
  // if-converted the whole coefficient reload into every step
  auto step = [&](int m, dvec<NPT>& V, dvec<NPT>& R) __attribute__((always_inline)) {
    if ((m & 63) == 0) {
      const int mm = m + lane;
      bblk[wave * 64 + lane] = mm < A.n_time ? bnd[mm] : make_double2(0.0, 0.0);
    }
    const unsigned ba = hide_addr(bb_a);
    const double lo = lds_ld(ba, 2 * (m & 63)), hi = lds_ld(ba, 2 * (m & 63) + 1);

    double cw, cwb;  // carries into wave 0 (bottom) and the last wave (top)
    if constexpr (PW) {
      // ---- rhs: beta_i V_i pre-scaled by g_i; the exceptional rows add
      // their residual stencil (uniform branch on the slot of row i1) -------
#pragma unroll
      for (int k = 0; k < NPT; ++k) R[k] = cB[k] * V[k];
      if (has_exc) {
        // row at slot k of its thread: R[k] += ra V[k-1] + rc V[k+1]; the
        // residuals are zero on every other thread
        auto exc_row = [&](int k, double ra, double rc) __attribute__((always_inline)) {
          // (the neighbour slots wrap; a power-of-two chunk by masking, which
          // compiles to fewer indexed moves than the selects)
          constexpr bool kPow2 = (NPT & (NPT - 1)) == 0;
          double xm = V[kPow2 ? (k + NPT - 1) & (NPT - 1) : (k == 0 ? NPT - 1 : k - 1)];
          double xp = V[kPow2 ? (k + 1) & (NPT - 1) : (k == NPT - 1 ? 0 : k + 1)];
          if (k == 0) {  // uniform: the slot below is in the thread below
            xm = from_below(xm, 1, lane4);
            if (lo_out && t == 0) xm = v0;
            if constexpr (W > 1) {
              if (lane == 63) xch[wave] = V[NPT - 1];
              __syncthreads();
              if (lane == 0 && wave > 0) xm = xch[wave - 1];
              __syncthreads();
            }
          }
          if (k == NPT - 1) {
            xp = from_above(xp, 1, lane4);
            if constexpr (W > 1) {
              if (lane == 0) xch[W + wave] = V[0];
              __syncthreads();
              if (lane == 63 && wave < W - 1) xp = xch[W + wave + 1];
              __syncthreads();
            }
          }
          R[k] = fma(ra, xm, fma(rc, xp, R[k]));
        };
        exc_row(k1, ra1, rc1);
        exc_row((NPT & (NPT - 1)) == 0 ? (k1 + 1) & (NPT - 1) : (k1 + 1 == NPT ? 0 : k1 + 1), ra2,
                rc2);
      }
      cw = fma(-alpha, v0, g0 * lo);
      cwb = fma(-alpha, vN, gN * hi);
    } else {
      // ---- rhs: the reference's explicit stencil, pre-scaled by g_i -------
      double left = from_below(V[NPT - 1], 1, lane4), right = from_above(V[0], 1, lane4);
      if (lo_out && t == 0) left = v0;
      if constexpr (W > 1) {
        if (lane == 63) xch[wave] = V[NPT - 1];
        if (lane == 0) xch[W + wave] = V[0];
        __syncthreads();
        if (lane == 0 && wave > 0) left = xch[wave - 1];
        if (lane == 63 && wave < W - 1) right = xch[W + wave + 1];
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const double vm = (k == 0) ? left : V[k - 1];
        const double vp = (k == NPT - 1) ? right : V[k + 1];
        R[k] = fma(cC[k], vp, fma(cB[k], V[k], cA[k] * vm));
      }
      cw = g0 * lo;
      cwb = gN * hi;
    }

    // ---- forward: d_i = rhs'_i + f_i d_{i-1}; carry-in at slot 0: cw ------
    double a = 0.0;
    if constexpr (kHalf) {
      double al = R[0], ah = R[H];
#pragma unroll
      for (int k = 1; k < H; ++k) {
        al = fma(cf[k], al, R[k]);
        ah = fma(cf[k + H], ah, R[k + H]);
      }
      a = fma(fh, al, ah);
    } else {
      a = R[0];
#pragma unroll
      for (int k = 1; k < NPT; ++k) a = fma(cf[k], a, R[k]);
    }
    const unsigned sa = hide_addr(sw_a);
    a = fma(lds_ld(sa, 0), dpp64<kRowShr + 1, 0xF>(a), a);
    a = fma(lds_ld(sa, 64), dpp64<kRowShr + 2, 0xF>(a), a);
    a = fma(lds_ld(sa, 128), dpp64<kRowShr + 4, 0xF>(a), a);
    a = fma(lds_ld(sa, 192), dpp64<kRowShr + 8, 0xF>(a), a);
    // the row broadcasts write every row (their weights are 0 on the rows
    // they do not feed): no zeroed destination to prepare
    a = fma(lds_ld(sa, 512), dpp64<kRowBcast15, 0xF>(a), a);
    a = fma(lds_ld(sa, 576), dpp64<kRowBcast31, 0xF>(a), a);
    if constexpr (W > 1) {
      if (lane == 63) xch[2 * W + wave] = a;
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W - 1; ++v)
        if (v < wave) cw = fma(xch[3 * W + v], cw, xch[2 * W + v]);
    }
    a = fma(Fpre, cw, a);
    double c = dpp64_old<0x138>(cw, a);  // wave_shr:1; lane 0 keeps the carry
    if (lo_out && !PW) v0 = uni(g0 * lo);  // x_0 of this step: cw of wave 0
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      c = fma(cf[k], c, R[k]);
      R[k] = c;
    }

    // ---- backward: x_i = d_i + e_i x_{i+1}; carry-in at the top: cwb -------
    double b = 0.0;
    if constexpr (kHalf) {
      double bl = R[H - 1], bh = R[NPT - 1];
#pragma unroll
      for (int k = H - 2; k >= 0; --k) {
        bh = fma(ce[k + H], bh, R[k + H]);
        bl = fma(ce[k], bl, R[k]);
      }
      b = fma(gl, bh, bl);
    } else {
      b = R[NPT - 1];
#pragma unroll
      for (int k = NPT - 2; k >= 0; --k) b = fma(ce[k], b, R[k]);
    }
    b = fma(lds_ld(sa, 256), dpp64<kRowShl + 1, 0xF>(b), b);
    b = fma(lds_ld(sa, 320), dpp64<kRowShl + 2, 0xF>(b), b);
    b = fma(lds_ld(sa, 384), dpp64<kRowShl + 4, 0xF>(b), b);
    b = fma(lds_ld(sa, 448), dpp64<kRowShl + 8, 0xF>(b), b);
    b = fma(lds_ld(sa, 640), bperm(b, addrA), b);
    b = fma(lds_ld(sa, 704), read_lane(b, 32), b);
    if constexpr (W > 1) {
      if (lane == 0) xch[4 * W + wave] = b;
      __syncthreads();
#pragma unroll
      for (int v = W - 1; v > 0; --v)
        if (v > wave) cwb = fma(xch[5 * W + v], cwb, xch[4 * W + v]);
    }
    b = fma(Gsuf, cwb, b);
    double cb = dpp64_old<0x130>(cwb, b);  // wave_shl:1; lane 63 keeps the carry
#pragma unroll
    for (int k = NPT - 1; k >= 0; --k) {
      cb = fma(ce[k], cb, R[k]);
      R[k] = PW ? fma(alpha, V[k], cb) : cb;  // x = alpha V + u
    }
    if constexpr (PW) {
      v0 = g0 * lo;  // the Dirichlet rows' x of this step (uniform; left in VGPRs)
      vN = gN * hi;
    }

    // ---- knock-out projection on monitoring steps --------------------------
    if (m + 1 == next_mon) {
      double reb = next_reb;
      asm volatile("" : "+v"(reb));  // a VGPR copy: the masked move reads it
#pragma unroll
      for (int k = 0; k < NPT; ++k) {  // one v_mov_b64 per slot under the slot's lane mask
        unsigned long long sv;
        asm volatile("s_mov_b64 %1, exec\n\ts_mov_b64 exec, %2\n\tv_mov_b64 %0, %3\n\t"
                     "s_mov_b64 exec, %1"
                     : "+v"(R[k]), "=&s"(sv)
                     : "s"(km[k]), "v"(reb));
      }
      if ((lo_out || PW) && ko0) v0 = reb;
      if (PW && koN) vN = reb;
      // skip this entry and any repeat of it (the _dev entry point does not
      // validate the runs; a repeated step would otherwise stall next_mon)
      do ++mpos;
      while (mpos < mend && __builtin_amdgcn_readfirstlane(A.mon_step[mpos]) <= m + 1);
      next_mon = mpos < mend ? __builtin_amdgcn_readfirstlane(A.mon_step[mpos]) : 0x7fffffff;
      next_reb = mpos < mend ? uni(A.mon_rebate[mpos]) : 0.0;
    }
    if constexpr (W > 1) __syncthreads();  // exchange area reused next step
  };
  const int m1 = (use_r && use_c) ? A.n_ranna : A.n_time;
  int m = 0;
  auto run = [&](int m_end) __attribute__((always_inline)) {
    for (; m + 1 < m_end; m += 2) {
      step(m, VA, VB);
      step(m + 1, VB, VA);
    }
    if (m < m_end) {
      step(m, VA, VB);
      VA = VB;
      ++m;
    }
  };
  run(m1);
  if (m < A.n_time) {
    load_phase(1);
    run(A.n_time);
  }
  const dvec<NPT>& V = VA;

  double* vout = A.v_out + (size_t)scen * n;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = base + k - pad_lo;
    if (j > 0 && j < n - 1) vout[j] = V[k];
    if (!PW && (j == 0 || j == n - 1)) vout[j] = V[k];
  }
  if (t == 0 && (lo_out || PW)) vout[0] = v0;
  if (t == 0 && PW) vout[n - 1] = vN;
}

using VcFn = void (*)(VcArgs);
struct VcVariant {
  int w, npt;
  VcFn stencil, pointwise;
};
template <int W, int NPT>
VcVariant vmk() {
  return VcVariant{W, NPT, &fdcn_vc_march<W, NPT, false>, &fdcn_vc_march<W, NPT, true>};
}
// (W = 16 holds at most 128 VGPRs a wave and spills its NPT = 8 and 16
// bodies; W = 8 NPT = 16 (8 193 nodes) spills less, on half the waves)
// (NPT 10 and 12, round 5: the reference's default 600 x 600 grid, 601
// nodes, fills 640 slots at 94 % instead of 1 024 at 59 %)
const VcVariant kVc[] = {vmk<1, 4>(),  vmk<1, 8>(),  vmk<1, 10>(), vmk<1, 12>(), vmk<1, 16>(), vmk<4, 4>(),
                         vmk<4, 8>(),  vmk<4, 16>(), vmk<8, 16>(),
                         vmk<16, 4>(), vmk<16, 8>(), vmk<16, 16>()};
constexpr int kNumVc = sizeof(kVc) / sizeof(kVc[0]);

// diagnostics (include/fdcn_diag.h): a pinned variant and the stencil form
std::atomic<int> g_vc_forced{0};  // waves | npt << 8 | stencil_only << 16

// Throughput batches: fewest waves, then fewest slots.  Small batches (B
// waves well short of the 2048 resident wave slots): shortest chunks.
const VcVariant* vc_choose(int n, long B) {
  const int f = g_vc_forced.load(std::memory_order_relaxed);
  if (f & 0xffff) {
    for (int i = 0; i < kNumVc; ++i)
      if (kVc[i].w == (f & 0xff) && kVc[i].npt == ((f >> 8) & 0xff) &&
          64L * kVc[i].w * kVc[i].npt >= n - 1)
        return &kVc[i];
  }
  const VcVariant* best = nullptr;
  const bool small = B * 4 < 2048;
  for (int i = 0; i < kNumVc; ++i) {
    const VcVariant& v = kVc[i];
    if (64L * v.w * v.npt < n - 1) continue;  // node 0 may sit outside (pad_lo = -1)
    if (!best) {
      best = &v;
      continue;
    }
    const long sv = 64L * v.w * v.npt, sb = 64L * best->w * best->npt;
    const bool better = small ? (v.npt < best->npt || (v.npt == best->npt && v.w < best->w))
                              : (v.w < best->w || (v.w == best->w && sv < sb));
    if (better) best = &v;
  }
  return best;
}

size_t vc_ws_per_scen(const VcVariant& v) {
  return sizeof(double) * (2 * kNC * (size_t)64 * v.w * v.npt + kNS);
}

int vc_launch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna, const double* diag,
              const double* bnd, const double* v_init, const int32_t* iparams, int32_t n_mon,
              const int32_t* mon_step, const double* mon_rebate, double* v_out,
              double* workspace, int64_t workspace_bytes, hipStream_t stream) {
  if (B < 0 || n_nodes < 3 || n_time < 0 || n_ranna < 0)
    return vfail(FDCN_EINVAL, "fdcn_vc: B >= 0, n_nodes >= 3, n_time >= 0, n_ranna >= 0");
  if (B == 0) return FDCN_OK;
  const VcVariant* v = vc_choose(n_nodes, B);
  if (!v) return vfail(FDCN_EINVAL, "fdcn_vc: n_nodes=%d above the largest variant", n_nodes);
  const size_t ws = vc_ws_per_scen(*v) * (size_t)B;
  if (workspace && (workspace_bytes < 0 || (size_t)workspace_bytes < ws))
    return vfail(FDCN_EINVAL, "fdcn_vc: workspace of %lld B is smaller than the %zu B needed",
                 (long long)workspace_bytes, ws);
  bool own = false;
  if (!workspace) {
    V_TRY(hipMallocAsync((void**)&workspace, ws, stream));
    own = true;
  }
  VcArgs a;
  a.B = B;
  a.n = n_nodes;
  a.n_time = n_time;
  a.n_ranna = n_ranna;
  a.slots = 64 * v->w * v->npt;
  a.pad_lo = a.slots >= n_nodes ? (a.slots - n_nodes) / 2 : -1;
  a.force_stencil = (g_vc_forced.load(std::memory_order_relaxed) >> 16) & 1;
  a.diag = diag;
  a.bnd = bnd;
  a.v_init = v_init;
  a.iparams = iparams;
  a.mon_step = mon_step;
  a.mon_rebate = mon_rebate;
  a.v_out = v_out;
  a.coef = workspace;
  (void)n_mon;
  // classify + factor (one wave per scenario and phase), then both forms:
  // each runs the scenarios the factor kernel gave it and returns at once
  // for the others
  hipLaunchKernelGGL(fdcn_vc_factor, dim3(B), dim3(128), 0, stream, a);
  V_TRY(hipGetLastError());
  hipLaunchKernelGGL(v->pointwise, dim3(B), dim3(64 * v->w), 0, stream, a);
  V_TRY(hipGetLastError());
  hipLaunchKernelGGL(v->stencil, dim3(B), dim3(64 * v->w), 0, stream, a);
  V_TRY(hipGetLastError());
  if (own) V_TRY(hipFreeAsync(workspace, stream));
  return FDCN_OK;
}

size_t al256(size_t n) { return (n + 255) / 256 * 256; }

}  // namespace

extern "C" {

int fdcn_vc_plan(int32_t B, int32_t n_nodes, int32_t* waves, int32_t* npt,
                 int64_t* ws_bytes_per_scen) {
  const VcVariant* v = vc_choose(n_nodes, B > 0 ? B : 1);
  if (n_nodes < 3 || !v) return vfail(FDCN_EINVAL, "fdcn_vc_plan: unsupported n_nodes=%d", n_nodes);
  if (waves) *waves = v->w;
  if (npt) *npt = v->npt;
  if (ws_bytes_per_scen) *ws_bytes_per_scen = (int64_t)vc_ws_per_scen(*v);
  return FDCN_OK;
}

int fdcn_vc_force_variant(int32_t waves, int32_t npt, int32_t stencil_only) {
  if (waves == 0 && npt == 0) {
    g_vc_forced.store(stencil_only ? (1 << 16) : 0);
    return FDCN_OK;
  }
  for (int i = 0; i < kNumVc; ++i)
    if (kVc[i].w == waves && kVc[i].npt == npt) {
      g_vc_forced.store(waves | (npt << 8) | ((stencil_only ? 1 : 0) << 16));
      return FDCN_OK;
    }
  return vfail(FDCN_EINVAL, "fdcn_vc_force_variant: no compiled variant W=%d NPT=%d", waves, npt);
}

int fdcn_vc_variant_name(int32_t B, int32_t n_nodes, char* buf, int32_t len) {
  const VcVariant* v = vc_choose(n_nodes, B > 0 ? B : 1);
  if (!buf || len < 1 || n_nodes < 3 || !v)
    return vfail(FDCN_EINVAL, "fdcn_vc_variant_name: bad arguments");
  snprintf(buf, (size_t)len, "fdcn_vc_march<%d,%d>", v->w, v->npt);
  return FDCN_OK;
}

int fdcn_vc_forms(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* diag, int32_t* form) {
  if (B < 0 || n_nodes < 3 || !diag || !form)
    return vfail(FDCN_EINVAL, "fdcn_vc_forms: bad arguments");
  const bool force = (g_vc_forced.load() >> 16) & 1;
  for (int32_t b = 0; b < B; ++b) {
    const double* D = diag + (size_t)b * 2 * FDCN_VC_NDIAG * n_nodes;
    const PhaseClass p0 = classify_phase(D, n_nodes, n_ranna > 0, force);
    const PhaseClass p1 = classify_phase(D + FDCN_VC_NDIAG * n_nodes, n_nodes, n_ranna < n_time,
                                         force);
    int i1;
    form[b] = pointwise_form(p0.ok, p0.first, p0.last, p1.ok, p1.first, p1.last, &i1) ? 1 : 0;
  }
  return FDCN_OK;
}

int fdcn_vc_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* diag, const double* bnd, const double* v_init,
                      const int32_t* iparams, int32_t n_mon, const int32_t* mon_step,
                      const double* mon_rebate, double* v_out, double* workspace,
                      int64_t workspace_bytes, void* stream) {
  return vc_launch(B, n_nodes, n_time, n_ranna, diag, bnd, v_init, iparams, n_mon, mon_step,
                   mon_rebate, v_out, workspace, workspace_bytes, (hipStream_t)stream);
}

int fdcn_vc_batch(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* diag, const double* bnd, const double* v_init,
                  const int32_t* iparams, int32_t n_mon, const int32_t* mon_step,
                  const double* mon_rebate, double* v_out) {
  // the CN plan checks (monitor runs, forms = 0, tau mode) on a dummy dt
  if (B < 0 || n_nodes < 3 || n_time < 0 || n_ranna < 0)
    return vfail(FDCN_EINVAL, "fdcn_vc: B >= 0, n_nodes >= 3, n_time >= 0, n_ranna >= 0");
  if (B > 0 && (!diag || (n_time > 0 && !bnd) || !v_init || !iparams || !v_out))
    return vfail(FDCN_EINVAL, "fdcn_vc: null array argument");
  {
    double dummy[FDCN_NPARAM] = {1.0};
    for (int32_t b = 0; b < B; ++b) {
      int rc = fdcn_internal::validate_plan(0, 1, n_nodes, n_time, n_ranna, dummy,
                                            iparams + (size_t)b * FDCN_NIPARAM, n_mon, mon_step,
                                            mon_rebate);
      if (rc) return rc;
      const double* Dg = diag + (size_t)b * 2 * FDCN_VC_NDIAG * n_nodes;
      for (int ph = 0; ph < 2; ++ph) {
        const double* P = Dg + (size_t)ph * FDCN_VC_NDIAG * n_nodes;
        if (P[0] != 0.0 || P[2 * n_nodes] != 0.0 || P[n_nodes - 1] != 0.0 ||
            P[3 * n_nodes - 1] != 0.0)
          return vfail(FDCN_EINVAL,
                       "fdcn_vc: scenario %d phase %d: rows 0 and n-1 must be Dirichlet rows "
                       "(sub = sup = 0)", b, ph);
      }
    }
  }
  if (B == 0) return FDCN_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return vfail(FDCN_ENODEV, "no HIP device visible");
  hipStream_t st;
  int rc = fdcn_internal::thread_stream(&st);
  if (rc) return rc;
  int32_t w_, npt_;
  int64_t wsp = 0;
  if ((rc = fdcn_vc_plan(B, n_nodes, &w_, &npt_, &wsp))) return rc;
  const size_t nv = (size_t)B * n_nodes, nd = (size_t)B * 2 * FDCN_VC_NDIAG * n_nodes;
  const size_t nb = (size_t)B * 2 * (size_t)n_time, nm = (size_t)(n_mon > 0 ? n_mon : 1);
  const size_t oD = 0, oB = oD + al256(8 * nd), oV = oB + al256(8 * (nb ? nb : 1));
  const size_t oI = oV + al256(8 * nv), oM = oI + al256(4 * (size_t)B * FDCN_NIPARAM);
  const size_t oR = oM + al256(4 * nm), oO = oR + al256(8 * nm), oW = oO + al256(8 * nv);
  const size_t ws = (size_t)wsp * B, total = oW + al256(ws);
  char* d = nullptr;
  hipError_t e = hipMallocAsync((void**)&d, total, st);
  if (e != hipSuccess) return vfail(FDCN_ENOMEM, "hipMallocAsync(%zu): %s", total, hipGetErrorString(e));
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  e = hipMemcpyAsync(d + oD, diag, 8 * nd, h2d, st);
  if (e == hipSuccess && nb) e = hipMemcpyAsync(d + oB, bnd, 8 * nb, h2d, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + oV, v_init, 8 * nv, h2d, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + oI, iparams, 4 * (size_t)B * FDCN_NIPARAM, h2d, st);
  if (e == hipSuccess && n_mon > 0) e = hipMemcpyAsync(d + oM, mon_step, 4 * (size_t)n_mon, h2d, st);
  if (e == hipSuccess && n_mon > 0) e = hipMemcpyAsync(d + oR, mon_rebate, 8 * (size_t)n_mon, h2d, st);
  if (e != hipSuccess) rc = vfail(FDCN_EHIP, "hipMemcpyAsync H2D: %s", hipGetErrorString(e));
  if (rc == FDCN_OK)
    rc = vc_launch(B, n_nodes, n_time, n_ranna, (const double*)(d + oD), (const double*)(d + oB),
                   (const double*)(d + oV), (const int32_t*)(d + oI), n_mon,
                   (const int32_t*)(d + oM), (const double*)(d + oR), (double*)(d + oO),
                   (double*)(d + oW), (int64_t)ws, st);
  if (rc == FDCN_OK) {
    e = hipMemcpyAsync(v_out, d + oO, 8 * nv, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) rc = vfail(FDCN_EHIP, "hipMemcpyAsync D2H: %s", hipGetErrorString(e));
  }
  (void)hipFreeAsync(d, st);
  e = hipStreamSynchronize(st);
  if (rc == FDCN_OK && e != hipSuccess) rc = vfail(FDCN_EHIP, "fdcn_vc: %s", hipGetErrorString(e));
  return rc;
}

}  // extern "C"
