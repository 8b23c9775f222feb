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

constexpr int kNC = 5;  // factored coefficients per slot: A, B, C, f, e

struct VcArgs {
  int B, n, n_time, n_ranna, slots, pad_lo;
  const double* diag;     // [B][2][6][n]
  const double* bnd;      // [B][n_time][2]
  const double* v_init;   // [B][n]
  const int32_t* iparams; // [B][FDCN_NIPARAM]
  const int32_t* mon_step;
  const double* mon_rebate;
  double* v_out;
  double* coef;           // workspace [B][2][kNC][slots] + [B][4] boundary scales
};

// one phase's factorization into the workspace (serial, the reference's
// _solve_tridiagonal order: beta_i = main_i - sub_i c*_{i-1}, c*_i = sup_i / beta_i)
__device__ void factor_phase(const double* P, int n, int slots, int pad_lo, double* C,
                             double* scal) {
  const double *sub = P, *mn = P + n, *sup = P + 2 * n;
  const double *ae = P + 3 * n, *be = P + 4 * n, *ce = P + 5 * n;
  double* cA = C;
  double* cB = C + slots;
  double* cC = C + 2 * slots;
  double* cf = C + 3 * slots;
  double* cE = C + 4 * slots;
  for (int s = 0; s < pad_lo; ++s) {  // lower padding: pass the forward carry up
    cA[s] = cB[s] = cC[s] = 0.0;
    cf[s] = 1.0;
    cE[s] = 0.0;
  }
  double cs = 0.0;
  for (int i = 0; i < n; ++i) {
    const int s = i + pad_lo;
    const double beta = (i == 0) ? mn[0] : mn[i] - sub[i] * cs;
    const double g = 1.0 / beta;
    cs = (i < n - 1) ? sup[i] / beta : 0.0;
    if (i == 0) scal[0] = g;
    if (s < 0) continue;  // node 0 outside the slots (pad_lo = -1)
    const bool interior = i > 0 && i < n - 1;
    cA[s] = interior ? ae[i] * g : 0.0;
    cB[s] = interior ? be[i] * g : 0.0;
    cC[s] = interior ? ce[i] * g : 0.0;
    // node 0 takes the forward carry (g_0 lo) as its value; node n-1 the
    // backward one (g_{n-1} hi); interior rows their factors
    cf[s] = (i == 0) ? 1.0 : (i == n - 1 ? 0.0 : -sub[i] * g);
    cE[s] = (i == n - 1) ? 1.0 : (i == 0 ? 0.0 : -cs);
    if (i == n - 1) scal[1] = g;
  }
  for (int s = pad_lo + n; s < slots; ++s) {  // upper padding: pass the backward carry down
    cA[s] = cB[s] = cC[s] = 0.0;
    cf[s] = 0.0;
    cE[s] = 1.0;
  }
}

// <1, 16> needs 256 VGPRs + 31 AGPRs: held to two waves per SIMD it spills
// 168 B a lane and runs 1.47x faster (9.68 -> 6.61 ms, spot_vc bench)
template <int W, int NPT>
__global__ void __launch_bounds__(64 * W, (W == 1 && NPT == 16) ? 2 : 1) fdcn_vc_march(VcArgs A) {
  __shared__ double xch[6 * W + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int lane4 = lane << 2;
  asm volatile("" : "+v"(lane4));
  const int scen = blockIdx.x;
  const int n = A.n, slots = A.slots, pad_lo = A.pad_lo;
  double* coef = A.coef + (size_t)scen * (2 * kNC * (size_t)slots + 4);
  double* scal = coef + 2 * kNC * (size_t)slots;
  const double* D = A.diag + (size_t)scen * 2 * FDCN_VC_NDIAG * n;
  const bool use_r = A.n_ranna > 0, use_c = A.n_ranna < A.n_time;

  // 1. factor both phases (two lanes of wave 0 in parallel), then share
  if (t < 2 && ((t == 0 && use_r) || (t == 1 && use_c)))
    factor_phase(D + (size_t)t * FDCN_VC_NDIAG * n, n, slots, pad_lo,
                 coef + (size_t)t * kNC * slots, scal + 2 * t);
  __syncthreads();

  const int base = t * NPT;  // first slot of this thread
  const int32_t* I = A.iparams + (size_t)scen * FDCN_NIPARAM;
  const int ko_lo = __builtin_amdgcn_readfirstlane(I[FDCN_I_KO_LO]);
  const int ko_hi = __builtin_amdgcn_readfirstlane(I[FDCN_I_KO_HI]);
  // knock-out lane masks per slot (nodes j <= ko_lo or j >= ko_hi), computed once
  unsigned long long km[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = base + k - pad_lo;
    km[k] = __ballot(j >= 0 && j < n && (j <= ko_lo || j >= ko_hi));
  }

  double V[NPT], R[NPT];
  const double* vin = A.v_init + (size_t)scen * n;
  // node 0 outside the slots: its value (uniform), and whether it knocks out
  const bool lo_out = pad_lo < 0;
  double v0 = lo_out ? uni(vin[0]) : 0.0;
  const bool ko0 = 0 <= ko_lo || 0 >= ko_hi;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = base + k - pad_lo;
    V[k] = (j >= 0 && j < n) ? vin[j] : 0.0;
  }

  double cA[NPT], cB[NPT], cC[NPT], cf[NPT], ce[NPT];
  // The lane scans of the two recurrences run row-segmented: four DPP
  // stages inside each 16-lane row, then the rows joined -- forward by
  // row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3), backward by one
  // ds_bpermute from the next row's first lane (rows 0, 2) and a readlane
  // of lane 32 (rows 0, 1).  One LDS round trip per step instead of ten.
  // Weights per stage: the products of the multipliers the stage spans.
  double FR[4], GR[4], F16 = 0.0, F32 = 0.0, GA = 0.0, GB = 0.0;
  const int rl = lane & 15;
  int addrA = (lane & 16) == 0 ? (((lane | 15) + 1) << 2) : lane4;  // rows 0, 2 <- rows 1, 3
  asm volatile("" : "+v"(addrA));
  double Fpre = 0.0, Gsuf = 0.0, g0 = 0.0, gN = 0.0;
  // the zero-carry passes run as two half-chunk chains joined by the
  // multiplier product of the other half (upper half forward, lower half
  // backward): half the dependent FMA chain on a one-wave-per-SIMD kernel
  constexpr bool kHalf = NPT >= 8;
  constexpr int H = NPT / 2;
  double fh = 1.0, gl = 1.0;
  auto load_phase = [&](int ph) __attribute__((always_inline)) {
    if constexpr (W > 1) __syncthreads();  // previous readers of the wave totals are done
    const double* C = coef + (size_t)ph * kNC * slots;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      cA[k] = C[base + k];
      cB[k] = C[slots + base + k];
      cC[k] = C[2 * slots + base + k];
      cf[k] = C[3 * slots + base + k];
      ce[k] = C[4 * slots + base + k];
    }
    g0 = uni(scal[2 * ph]);
    gN = uni(scal[2 * ph + 1]);
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
      double F = f, G = g, s;
#define VC_ROW_STAGE(j)                                                   \
      FR[j] = rl >= (1 << j) ? F : 0.0;                                   \
      s = dpp64<kRowShr + (1 << j), 0xF>(F);                              \
      F = rl >= (1 << j) ? F * s : F;                                     \
      GR[j] = rl + (1 << j) <= 15 ? G : 0.0;                              \
      s = dpp64<kRowShl + (1 << j), 0xF>(G);                              \
      G = rl + (1 << j) <= 15 ? G * s : G;
      VC_ROW_STAGE(0) VC_ROW_STAGE(1) VC_ROW_STAGE(2) VC_ROW_STAGE(3)
#undef VC_ROW_STAGE
      const bool odd = (lane & 16) != 0;
      F16 = odd ? F : 0.0;
      s = dpp64<kRowBcast15, 0xA>(F);
      F = odd ? F * s : F;
      F32 = lane >= 32 ? F : 0.0;
      GA = odd ? 0.0 : G;
      s = bperm(G, addrA);
      G = odd ? G : G * s;
      GB = lane < 32 ? G : 0.0;
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
  double2 bcur = make_double2(0.0, 0.0);
  // one step; the march runs it in two loops (Rannacher phase, then CN) so
  // the phase switch is not a branch in the step -- inside it the compiler
  // if-converted the whole coefficient reload into every step
  auto step = [&](int m) __attribute__((always_inline)) {
    if ((m & 63) == 0) {
      const int mm = m + lane;
      bcur = mm < A.n_time ? bnd[mm] : make_double2(0.0, 0.0);
    }
    const double lo = read_lane(bcur.x, m & 63), hi = read_lane(bcur.y, m & 63);

    // ---- rhs: the reference's explicit stencil, pre-scaled by g_i ---------
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

    // ---- forward: d_i = rhs'_i + f_i d_{i-1}; carry-in at slot 0: g_0 lo ----
    double a = 0.0;
    if constexpr (kHalf) {
      double al = 0.0, ah = 0.0;
#pragma unroll
      for (int k = 0; k < H; ++k) {
        al = fma(cf[k], al, R[k]);
        ah = fma(cf[k + H], ah, R[k + H]);
      }
      a = fma(fh, al, ah);
    } else {
#pragma unroll
      for (int k = 0; k < NPT; ++k) a = fma(cf[k], a, R[k]);
    }
    a = fma(FR[0], dpp64<kRowShr + 1, 0xF>(a), a);
    a = fma(FR[1], dpp64<kRowShr + 2, 0xF>(a), a);
    a = fma(FR[2], dpp64<kRowShr + 4, 0xF>(a), a);
    a = fma(FR[3], dpp64<kRowShr + 8, 0xF>(a), a);
    a = fma(F16, dpp64<kRowBcast15, 0xA>(a), a);
    a = fma(F32, dpp64<kRowBcast31, 0xC>(a), a);
    double cw = g0 * lo;  // carry into wave 0
    if constexpr (W > 1) {
      if (lane == 63) xch[2 * W + wave] = a;
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W - 1; ++v)
        if (v < wave) cw = fma(xch[3 * W + v], cw, xch[2 * W + v]);
      a = fma(Fpre, cw, a);
    } else {
      a = fma(Fpre, cw, a);
    }
    double c = from_below(a, 1, lane4);
    if (lane == 0) c = cw;
    if (lo_out) v0 = uni(g0 * lo);  // x_0 of this step: cw of wave 0
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      c = fma(cf[k], c, R[k]);
      R[k] = c;
    }

    // ---- backward: x_i = d_i + e_i x_{i+1}; carry-in at the top: g_{n-1} hi --
    double b = 0.0;
    if constexpr (kHalf) {
      double bl = 0.0, bh = 0.0;
#pragma unroll
      for (int k = H - 1; k >= 0; --k) {
        bh = fma(ce[k + H], bh, R[k + H]);
        bl = fma(ce[k], bl, R[k]);
      }
      b = fma(gl, bh, bl);
    } else {
#pragma unroll
      for (int k = NPT - 1; k >= 0; --k) b = fma(ce[k], b, R[k]);
    }
    b = fma(GR[0], dpp64<kRowShl + 1, 0xF>(b), b);
    b = fma(GR[1], dpp64<kRowShl + 2, 0xF>(b), b);
    b = fma(GR[2], dpp64<kRowShl + 4, 0xF>(b), b);
    b = fma(GR[3], dpp64<kRowShl + 8, 0xF>(b), b);
    b = fma(GA, bperm(b, addrA), b);
    b = fma(GB, read_lane(b, 32), b);
    double cwb = gN * hi;  // carry into the last wave
    if constexpr (W > 1) {
      if (lane == 0) xch[4 * W + wave] = b;
      __syncthreads();
#pragma unroll
      for (int v = W - 1; v > 0; --v)
        if (v > wave) cwb = fma(xch[5 * W + v], cwb, xch[4 * W + v]);
    }
    b = fma(Gsuf, cwb, b);
    double cb = from_above(b, 1, lane4);
    if (lane == 63) cb = cwb;
#pragma unroll
    for (int k = NPT - 1; k >= 0; --k) {
      cb = fma(ce[k], cb, R[k]);
      V[k] = cb;
    }

    // ---- knock-out projection on monitoring steps --------------------------
    if (m + 1 == next_mon) {
      double reb = next_reb;
      asm volatile("" : "+v"(reb));  // a VGPR copy: v_cndmask takes the mask as its SGPR operand
      const unsigned rlo = (unsigned)__double_as_longlong(reb);
      const unsigned rhi = (unsigned)(__double_as_longlong(reb) >> 32);
#pragma unroll
      for (int k = 0; k < NPT; ++k) {  // two v_cndmask per slot with the lane mask in SGPRs
        unsigned lo32 = (unsigned)__double_as_longlong(V[k]);
        unsigned hi32 = (unsigned)(__double_as_longlong(V[k]) >> 32);
        asm volatile("v_cndmask_b32 %0, %0, %2, %4\n\tv_cndmask_b32 %1, %1, %3, %4"
                     : "+v"(lo32), "+v"(hi32)
                     : "v"(rlo), "v"(rhi), "s"(km[k]));
        V[k] = __longlong_as_double(((long long)hi32 << 32) | lo32);
      }
      if (lo_out && ko0) v0 = reb;
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
  for (; m < m1; ++m) step(m);
  if (m < A.n_time) {
    load_phase(1);
    for (; m < A.n_time; ++m) step(m);
  }

  double* vout = A.v_out + (size_t)scen * n;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = base + k - pad_lo;
    if (j >= 0 && j < n) vout[j] = V[k];
  }
  if (lo_out && t == 0) vout[0] = v0;
}

using VcFn = void (*)(VcArgs);
struct VcVariant {
  int w, npt;
  VcFn fn;
};
template <int W, int NPT>
VcVariant vmk() {
  return VcVariant{W, NPT, &fdcn_vc_march<W, NPT>};
}
// (W = 16 holds at most 128 VGPRs a wave and spills its NPT = 8 and 16
// bodies; W = 8 NPT = 16 (8 193 nodes) spills less, on half the waves)
const VcVariant kVc[] = {vmk<1, 4>(),  vmk<1, 8>(),  vmk<1, 16>(), vmk<4, 4>(),
                         vmk<4, 8>(),  vmk<4, 16>(), vmk<8, 16>(),
                         vmk<16, 4>(), vmk<16, 8>(), vmk<16, 16>()};
constexpr int kNumVc = sizeof(kVc) / sizeof(kVc[0]);

// Throughput batches: fewest waves, then fewest slots.  Small batches (B
// waves well short of the 2048 resident wave slots): shortest chunks.
const VcVariant* vc_choose(int n, long B) {
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
  return sizeof(double) * (2 * kNC * (size_t)64 * v.w * v.npt + 4);
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
  a.diag = diag;
  a.bnd = bnd;
  a.v_init = v_init;
  a.iparams = iparams;
  a.mon_step = mon_step;
  a.mon_rebate = mon_rebate;
  a.v_out = v_out;
  a.coef = workspace;
  (void)n_mon;
  hipLaunchKernelGGL(v->fn, dim3(B), dim3(64 * v->w), 0, stream, a);
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
