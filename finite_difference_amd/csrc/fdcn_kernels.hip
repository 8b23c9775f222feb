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
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/fdcn.h"
#include "../../include/fdcn_diag.h"
#include "fdcn_shared.h"
#include "fdcn_ko_res.h"

namespace {

using fdcn_internal::sm_extent;
using fdcn_internal::tau_next_run;
using fdcn_internal::TauRun;

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
// the larger of lane 0's and lane 32's value (the two scenarios of a paired wave)
__device__ __forceinline__ int umax_halves(int x) {
  const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 32);
  return a > b ? a : b;
}

// Hide an index from the optimiser for one loop iteration, so table loads
// indexed by it are not hoisted out of the time loop (LICM would otherwise keep
// every LDS table entry of the lane live in VGPRs for the whole march).  An
// integer is hidden rather than the pointer so the LDS address space (and
// ds_read) is kept.
__device__ __forceinline__ int opaque(int i) {
  asm volatile("" : "+v"(i));
  return i;
}

// LDS byte addresses kept in a VGPR across steps.  Hiding an index makes the
// compiler rebuild the address from it on every step (a copy, a shift-add
// and an add); a loop-carried address passed through the asm in place
// (a = hide_addr(a)) costs no instruction, and every load off it uses the
// ds_read immediate offset.
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

// Cross-lane moves.  Shifts by one lane use the GFX9 wavefront DPP shifts
// (wave_shr:1 / wave_shl:1: two VALU moves, no LDS round trip), by two lanes
// two of them; longer shifts go through ds_bpermute.  Lanes without a source
// receive 0 (DPP) or their own value (bpermute); every caller masks them.
template <int CTRL>
__device__ __forceinline__ double dpp_move(double x) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// acc += bcast(tab, lane i of each 16-lane row) * c: a per-scenario table
// value (the same on every lane of the wave) broadcast by 64-bit DPP
// (row_newbcast) straight into the FMA -- no LDS read, no register holding
// the value.  The table sits in one VGPR pair, lane l holding entry l mod
// 16.  i is a compile-time constant after unrolling (the switch folds away).
__device__ __forceinline__ void fmac_bcast(double& acc, double tab, double c, int i) {
  switch (i) {
#define FDCN_BC(n)                                                                        \
  case n:                                                                                 \
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" \
                 : "+v"(acc) : "v"(tab), "v"(c));                                         \
    break;
    FDCN_BC(0) FDCN_BC(1) FDCN_BC(2) FDCN_BC(3) FDCN_BC(4) FDCN_BC(5) FDCN_BC(6) FDCN_BC(7)
    FDCN_BC(8) FDCN_BC(9) FDCN_BC(10) FDCN_BC(11) FDCN_BC(12) FDCN_BC(13) FDCN_BC(14)
    FDCN_BC(15)
#undef FDCN_BC
    default: break;
  }
}

constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i-1
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i+1
__device__ __forceinline__ double shfl_up1(double x, int d) {
  if (d == 1) return dpp_move<kDppWaveShr1>(x);
  if (d == 2) return dpp_move<kDppWaveShr1>(dpp_move<kDppWaveShr1>(x));
  return __shfl_up(x, (unsigned)d, 64);
}
__device__ __forceinline__ double shfl_dn1(double x, int d) {
  if (d == 1) return dpp_move<kDppWaveShl1>(x);
  if (d == 2) return dpp_move<kDppWaveShl1>(dpp_move<kDppWaveShl1>(x));
  return __shfl_down(x, (unsigned)d, 64);
}

// Scan-stage shifts for the time loop.  Strides 1-2 as above; longer ones
// by ds_bpermute from lane4 = 4*lane held in one VGPR: the source lane is
// (lane -/+ d) mod 64 (ds_bpermute uses the address bits [7:2]), so lanes
// without a true source read another lane's finite value, which their zero
// scan weight drops.  (__shfl_up/_down recompute a clamped address with
// five VALU instructions per stage and step.)
__device__ __forceinline__ double bperm(double x, int addr) {
  const unsigned long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(b & 0xffffffffull));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(b >> 32));
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double scan_up(double x, int d, int lane4) {
  if (d <= 2) return shfl_up1(x, d);
  return bperm(x, lane4 - 4 * d);
}
__device__ __forceinline__ double scan_dn(double x, int d, int lane4) {
  if (d <= 2) return shfl_dn1(x, d);
  return bperm(x, lane4 + 4 * d);
}

__device__ __forceinline__ double bnd_eval(int form, double c0, double e0, double c1, double e1,
                                           double tau) {
  if (form == 1) return c0 * exp(e0 * tau) * c1 * exp(e1 * tau);
  return c0 * exp(e0 * tau) + c1 * exp(e1 * tau);
}
// The same value, bitwise, without the exp of a term whose coefficient is
// zero (wave-uniform branches): c * exp(y) is c itself for c = +-0 and a
// finite exp(y).  A call's lower and a put's upper Dirichlet value are such
// terms (…pricer.py:381-391).  Used where the evaluation sits in the march
// (kGen).  `skip` is the caller's uniform guarantee that every exp(e tau)
// of the march is finite (e tau <= 700 at both ends of its tau range,
// exp_finite_over): without it the exps are taken, so an overflowing
// exponential keeps the reference's 0 * inf = NaN.
__device__ __forceinline__ double bnd_eval_nz(int form, double c0, double e0, double c1,
                                              double e1, double tau, bool skip) {
  const double t0 = (skip && c0 == 0.0) ? c0 : c0 * exp(e0 * tau);
  if (form == 1) {
    const double p = t0 * c1;
    return (skip && p == 0.0) ? p : p * exp(e1 * tau);
  }
  return t0 + ((skip && c1 == 0.0) ? c1 : c1 * exp(e1 * tau));
}
// exp(e0 tau) and exp(e1 tau) finite for tau in [ta, tb] (e tau is linear in tau)
__host__ __device__ inline bool exp_finite_over(double e0, double e1, double ta, double tb) {
  const double big = 700.0;
  return e0 * ta <= big && e0 * tb <= big && e1 * ta <= big && e1 * tb <= big;
}

// Uniform per-phase (per theta) constants.
struct Phase {
  double bl, bc, bu;  // B_L/r, B_C/r, B_U/r
  double fm, bm;      // -A_L/r, -A_U/r
  double inv_r;
  double kappa;       // A_L A_U / r
  double pl, pu;      // -A_L, -A_U (unscaled Dirichlet couplings, theta form)
  double c2;          // (1 - theta) / theta
  double s;           // 1 / (theta r)
  double th;          // theta
};

template <bool kLane = false>  // kLane: per-lane (paired waves) instead of SGPR values
__device__ __forceinline__ Phase make_phase(double theta, double dt, double a, double c,
                                            double bcoef) {
  auto uni = [](double x) { return kLane ? x : ::uni(x); };
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
  p.kappa = AL * AU * p.inv_r;
  p.pl = uni(-AL);
  p.pu = uni(-AU);
  p.c2 = uni((1.0 - theta) / theta);
  p.s = uni(p.inv_r / theta);
  p.th = uni(theta);
  // wave-uniform: keep in SGPRs
  p.inv_r = uni(p.inv_r);
  p.bl = uni(p.bl);
  p.bc = uni(p.bc);
  p.bu = uni(p.bu);
  p.fm = uni(p.fm);
  p.bm = uni(p.bm);
  p.kappa = uni(p.kappa);
  return p;
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

// (lane, slot) of interior index i (0-based) under the short-lane layout:
// the first Ls lanes hold NPT-1 nodes, the rest NPT.
template <int NPT>
__device__ __forceinline__ void lane_slot(int i, int Ls, int& lane, int& slot) {
  const int split = Ls * (NPT - 1);
  if (i < split) {
    lane = i / (NPT - 1);
    slot = i - lane * (NPT - 1);
  } else {
    lane = Ls + (i - split) / NPT;
    slot = (i - split) - (lane - Ls) * NPT;
  }
}

// Knock-out lane masks of one wave, as wave-uniform 64-bit values: slot k of
// the lanes in `full` is knocked out for every k; lane `part` (if any) for k
// in [k0, k1].  The per-slot mask is then two scalar selects and an OR, and
// the projection two v_cndmask per slot with an SGPR mask.
struct KoMask {
  unsigned long long full, part;
  int k0, k1;
};

// One scenario's monitoring entries (wave-uniform): the entry of the next
// knock-out step and the one after it, loaded a monitor step ahead of their
// use.  kDefer (round 5): the prefetched entry stays in the VGPRs the vector
// load wrote and is made scalar (v_readfirstlane) only when the next
// knock-out advances to it -- taken at load time, the readfirstlane made
// every knock-out step wait out the load's whole latency (s_waitcnt vmcnt(0)
// right after the load; ~200 cycles a step with config 5's every-step
// projection) -- and the entries' addresses are VGPRs (with the array bases
// in SGPRs the compiler spilled them to VGPR lanes and read them back, eight
// v_readlane a step).  Config 5 (A/B, one box): 16.60 -> 15.14-15.40 ms.
// Without kDefer (the register-capped config-3 variant, daily monitoring:
// knock-outs are rare there and the extra live VGPRs cost more than the
// waits) the entries are made scalar at load time.
template <bool kDefer>
struct MonRun {
  int pos, end, next;
  double cur;
  int pf_v;         // st[pos + 1] as loaded (kDefer: a VGPR, the same in every lane)
  double pf_reb_v;  // rb[pos + 1] as loaded
  const int32_t* pst;  // kDefer: &st[pos + 1], &rb[pos + 1] (VGPRs)
  const double* prb;
  __device__ __forceinline__ int ld_i(const int32_t* p) { return kDefer ? *p : uni_i(*p); }
  __device__ __forceinline__ double ld_d(const double* p) { return kDefer ? *p : uni(*p); }
  __device__ __forceinline__ void init(const int32_t* st, const double* rb, int start, int count) {
    pos = start;
    end = start + count;
    // entries < 1 never match a step: skip them (the oracle's `while` does)
    while (pos < end && uni_i(st[pos]) < 1) ++pos;
    next = 0x7fffffff;
    cur = 0.0;
    pf_v = 0x7fffffff;
    pf_reb_v = 0.0;
    pst = st + pos + 1;
    prb = rb + pos + 1;
    if (pos < end) {
      next = uni_i(st[pos]);
      cur = uni(rb[pos]);
      if (pos + 1 < end) {
        pf_v = ld_i(pst);
        pf_reb_v = ld_d(prb);
      }
    }
  }
  // after the knock-out at `step`: advance to the prefetched entry, request
  // the one after it
  __device__ __forceinline__ void advance(const int32_t* st, const double* rb, int step) {
    ++pos;
    next = pos < end ? (kDefer ? uni_i(pf_v) : pf_v) : 0x7fffffff;
    cur = kDefer ? uni(pf_reb_v) : pf_reb_v;
    if constexpr (kDefer) {
      ++pst;
      ++prb;
      asm volatile("" : "+v"(pst), "+v"(prb));
      if (pos + 1 < end) {
        pf_v = *pst;
        pf_reb_v = *prb;
      }
    } else if (pos + 1 < end) {
      pf_v = uni_i(st[pos + 1]);
      pf_reb_v = uni(rb[pos + 1]);
    }
    if (next <= step) {  // entries not strictly increasing: skip (slow path)
      while (pos < end && uni_i(st[pos]) <= step) ++pos;
      next = (pos < end) ? uni_i(st[pos]) : 0x7fffffff;
      cur = (pos < end) ? uni(rb[pos]) : 0.0;
      pf_v = (pos + 1 < end) ? ld_i(st + pos + 1) : 0x7fffffff;
      pf_reb_v = (pos + 1 < end) ? ld_d(rb + pos + 1) : 0.0;
      pst = st + pos + 1;
      prb = rb + pos + 1;
    }
  }
};

// Each wave's workspace row ends in kKoRow double2 = 64 per-slot knock-out
// masks.  From NPT = 16 on the NPT masks (2 NPT SGPRs) do not fit the scalar
// file next to everything else: the compiler spilled them to VGPR lanes and
// read each back with two v_readlane per slot and monitor step (four VALU
// per slot with the two v_cndmask).  Those variants store the masks once
// (vector stores) and reload them per monitor step with s_load: one
// exec-masked v_mov_b64 per slot.  (NPT = 16 joined in round 2: config 3,
// daily monitoring, 4 VALU per wave and step fewer on average.)
constexpr int kKoRow = 32;
// The recovery-form variants' row continues with the resident projection's
// run masks and group codes (kKoRes; fdcn_ko_res.h): q0, q1, q2, qd, then the
// two code words -- loaded by the projection itself (kept live through the
// march they pushed the kernel's SGPRs into VGPR lanes: 260 registers, one
// wave per SIMD)
constexpr int kKoResRow = 4;
// the one-sided boundary table (kTab1 in fdcn_march) from this batch size on
constexpr int kTab1MinBatch = 256;
typedef unsigned KoMask8 __attribute__((ext_vector_type(8)));  // 4 masks, s_load_dwordx8
__device__ __forceinline__ unsigned long long ko_pair8(KoMask8 m, int j) {
  return ((unsigned long long)m[2 * j + 1] << 32) | m[2 * j];
}
// The reloaded projection, four slots per block: block G's masks are in mcur
// (loaded by the block before), block G+1's arrive while block G's four
// exec-masked moves run (s_load_dwordx8 off the row's base with an immediate
// offset, waited for at the block's end, so every asm output is valid on
// exit).  sv: the wave's exec, saved once by the caller and restored at the
// end of each block (the compiler's code between the statements runs on it).
template <int G, int NB, int NPT>
__device__ __forceinline__ void ko_blocks(double (&V)[NPT], double rebv, unsigned long long ka,
                                          unsigned long long sv, KoMask8 mcur) {
  if constexpr (G < NB) {
#define FDCN_KO_MOV(j) "s_and_b64 exec, %[m" #j "], %[sv]\n\tv_mov_b64 %[v" #j "], %[rb]\n\t"
#define FDCN_KO_OPS                                                                  \
  [v0] "+v"(V[4 * G]), [v1] "+v"(V[4 * G + 1]), [v2] "+v"(V[4 * G + 2]), [v3] "+v"(V[4 * G + 3])
#define FDCN_KO_INS                                                                     \
  [rb] "v"(rebv), [sv] "s"(sv), [m0] "s"(ko_pair8(mcur, 0)), [m1] "s"(ko_pair8(mcur, 1)), \
      [m2] "s"(ko_pair8(mcur, 2)), [m3] "s"(ko_pair8(mcur, 3))
    if constexpr (G + 1 < NB) {
      KoMask8 mnxt;
      asm volatile("s_load_dwordx8 %[mn], %[ga], %[off]\n\t"
                   FDCN_KO_MOV(0) FDCN_KO_MOV(1) FDCN_KO_MOV(2) FDCN_KO_MOV(3)
                   "s_mov_b64 exec, %[sv]\n\ts_waitcnt lgkmcnt(0)"
                   : FDCN_KO_OPS, [mn] "=&s"(mnxt)
                   : FDCN_KO_INS, [ga] "s"(ka), [off] "i"(32 * (G + 1))
                   : "memory", "scc");
      ko_blocks<G + 1, NB, NPT>(V, rebv, ka, sv, mnxt);
    } else {
      asm volatile(FDCN_KO_MOV(0) FDCN_KO_MOV(1) FDCN_KO_MOV(2) FDCN_KO_MOV(3)
                   "s_mov_b64 exec, %[sv]"
                   : FDCN_KO_OPS
                   : FDCN_KO_INS
                   : "scc");
    }
#undef FDCN_KO_MOV
#undef FDCN_KO_OPS
#undef FDCN_KO_INS
  }
}

// Only the one-wave throughput variants reload from NPT = 16 on: the latency
// variants (several waves, or the single-trade flavour) have a knock-out on
// the critical path of one trade, where the s_load latency of every monitor
// step showed (config 5 trade, every step: 12.5 -> 14.0 ms).
template <int IT, int W, int NPT, int ZG = 0>
struct KoLoad {  // also the paired flavour: two scenarios' masks would crowd the scalar file
  static constexpr bool value =
      !IT && (NPT >= 48 || (W == 1 && !(ZG & 2) && NPT >= 16 && NPT % 8 == 0) || (ZG & 4));
};

// CN variants marched in the split form (state V, solve into T; see the step
// forms in fdcn_march).  Their workspace row also holds the raw Dirichlet
// values of every step (read back only after a knock-out step).
__host__ __device__ constexpr bool split_form(int it, int w, int npt) {
  return !it && (w == 16 ? npt <= 16 : npt <= 40);
}
// Split-form variants that tabulate their theta-form rhs terms in the
// prologue (the one-wave throughput variants).  The latency variants (several
// waves per scenario, or the single-trade flavour) march one scenario alone,
// where the step's critical path is what counts: a knock-out on every step
// (config 5) would put a table reload on every step, so they keep the raw
// Dirichlet values and form the terms in the step (single trade, config 5:
// 12.0 ms this way, 13.25 ms with the table).
__host__ __device__ constexpr bool tab_form(int it, int w, int npt, int lat) {
  return split_form(it, w, npt) && w == 1 && !lat;
}

// CN variants marched in the recovery form (W = 1, NPT > 40; see the step
// forms in fdcn_march).  Their Rannacher steps keep the old V in a
// workspace slice [64][NPT] per scenario (host: ws_bytes_per_scen).
__host__ __device__ constexpr bool rec_form(int it, int w, int npt) {
  return !it && w == 1 && npt > 40;
}

// Sub-chains per lane (see "chunk decomposition" in fdcn_march).
__host__ __device__ constexpr int sub_chains(int it, int w, int npt, int zg) {
  return (w == 1 && !(zg & 2))
             ? (npt >= 48 ? 2 : ((it && npt == 32) ? 4 : 1))
             : ((npt % 4 == 0 && npt >= 16) ? 4 : ((npt % 2 == 0 && npt >= 8) ? 2 : 1));
}

// Two-pass solve (the one-wave IT throughput variants): each sub-chain runs
// its forward and its backward recurrence once with zero carries, in place;
// the true solution differs from that by a homogeneous solution of the two
// recurrences, C P'_i + D G_i with per-phase tables
//   P'_i = sum_{k=i}^{M-1} bm^(k-i) fm^k,   G_i = bm^(M-i)
// and per-sub-chain coefficients C = fm * (forward carry), D = backward
// carry, which the carry scans deliver.  The Sherman-Morrison correction g z
// is of the same form on every sub-chain (z's own C, D, tabulated per lane),
// so it folds into C and D.  Two FMAs per node for the carries and the
// correction together, where re-running both passes and correcting took
// three, and the step's dependent chain is two passes long instead of four.
// Measured (tools/gpu_ab.sh, two boxes): config 2 11.25 -> 11.09 ms and
// 11.45 -> 11.21 ms per launch.  The split-form CN (config 3) lost with it:
// its update reads two tables per node against one, and at its 128-register
// cap the prefetch spilled (10.9 ms against 5.5; 6.0 with S = 2 at three
// waves per SIMD), so it keeps the re-run passes.
// Round 3: the one-wave split-form CN variants (up to 40 nodes per lane;
// config 3: 16) run two-pass too, with the homogeneous tables as DPP
// broadcasts (fmac_bcast) instead of the LDS reads that lost in round 2.
__host__ __device__ constexpr bool two_pass(int it, int w, int npt, int zg) {
  return w == 1 && zg == 0 && npt >= 2 && (it || npt <= 40);
}

// Doubles of the correction tables per scenario.  Two-pass variants: per
// phase P'[M], G[M], then [lz][C z(S), D z(S)]; otherwise z itself, [2][lz][NPT+1].
__host__ __device__ constexpr int sm_doubles(int it, int w, int npt, int zg, int lz) {
  return two_pass(it, w, npt, zg)
             ? 2 * (2 * (npt / sub_chains(it, w, npt, zg)) + (lz + 1) * 2 * sub_chains(it, w, npt, zg))
             : 2 * lz * (npt + 1);
}


// The split-form update of four slots: T_i += g z_i, V_i = s T_i - V_i (last
// slot scaled by s_last when kLast).  s in an SGPR pair, or a VGPR (kVs:
// paired waves, whose scenarios have their own s).
#define FDCN_SPLIT_UPD_ASM(S3)                                                     \
  "v_fma_f64 %4, %8, %9, %4\n\t"                                                 \
  "v_fma_f64 %5, %8, %10, %5\n\t"                                                \
  "v_fma_f64 %6, %8, %11, %6\n\t"                                                \
  "v_fma_f64 %7, %8, %12, %7\n\t"                                                \
  "v_fma_f64 %0, %13, %4, -%0\n\t"                                               \
  "v_fma_f64 %1, %13, %5, -%1\n\t"                                               \
  "v_fma_f64 %2, %13, %6, -%2\n\t"                                               \
  "v_fma_f64 %3, " S3 ", %7, -%3"
#define FDCN_SPLIT_UPD_OUT "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3)
template <bool kVs, bool kLast>
__device__ __forceinline__ void split_update(double& v0, double& v1, double& v2, double& v3,
                                             double& t0, double& t1, double& t2, double& t3,
                                             double g, const double* z, double s, double s_last) {
  if constexpr (!kVs && !kLast)
    asm volatile(FDCN_SPLIT_UPD_ASM("%13") : FDCN_SPLIT_UPD_OUT
                 : "v"(g), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]), "s"(s));
  else if constexpr (!kVs)
    asm volatile(FDCN_SPLIT_UPD_ASM("%14") : FDCN_SPLIT_UPD_OUT
                 : "v"(g), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]), "s"(s), "v"(s_last));
  else if constexpr (!kLast)
    asm volatile(FDCN_SPLIT_UPD_ASM("%13") : FDCN_SPLIT_UPD_OUT
                 : "v"(g), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]), "v"(s));
  else
    asm volatile(FDCN_SPLIT_UPD_ASM("%14") : FDCN_SPLIT_UPD_OUT
                 : "v"(g), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]), "v"(s), "v"(s_last));
}
#undef FDCN_SPLIT_UPD_ASM
#undef FDCN_SPLIT_UPD_OUT

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
struct KArgs {
  int B, n_nodes, n_time, n_ranna, n_mon, lz;
  const double* params;
  const int32_t* iparams;
  const double* v_init;
  const double* payoff;
  const int32_t* mon_step;
  const double* mon_rebate;
  double* v_out;
  double* bnd;      // workspace: [B][W][n_pad Dirichlet terms (not rec_form) + kKoRow masks (+ n_pad raw split form)][2]
  double* zg;       // workspace: correction tables [B][2][lz][NPT+1] (ZG variants)
  double* vsave;    // workspace: old V of a Rannacher step [B][64][NPT] (rec_form variants)
  int n_pad;        // n_time rounded up to a multiple of 64
};

// ZG is a flag set.  Bit 0: the Sherman-Morrison table lives in the global
// workspace instead of LDS -- the fallback for correction extents too long
// for LDS (|fm| -> 1).  Bit 1: the single-trade flavour of a W = 1 variant,
// for batches too small to put a wave on every SIMD: its recurrences run as 4
// interleaved sub-chains per lane, trading the joins' extra FMAs for in-wave
// ILP (with one wave on a SIMD nothing else hides the FMA latency).  Bit 2:
// the paired flavour of a split-form W = 1 variant: two scenarios per wave,
// 32 lanes each (lanes 0-31 and 32-63), for grids of up to 32 NPT interior
// nodes -- twice the nodes per lane of the one-scenario variant for the same
// grid, so the per-step scans, carries and broadcasts are spread over twice
// as many nodes.  Its per-scenario constants are per-lane values (VGPRs).
// LDS doubles for the scan weights of stages 2-5 (forward and backward, 64
// lanes): Geo::kScanLds variants
constexpr int kScanLdsDoubles = 4 * 2 * 64;

// Diagnostic builds only (tools/stamp_timeline.py builds with -DFDCN_STAMPS):
// per-phase s_memtime stamps of the recovery-form march, for the first
// kStampScen scenarios and kStampSteps steps from kStampStep0, written by lane
// 0 into the scenario's Rannacher save slice (vsave, read only in steps m <
// n_ranna) at [step - kStampStep0][16]; slot 15 of the first step row holds
// the wave's HW_ID and slot 14 its XCC_ID.  The product build compiles no
// stamp.
#ifdef FDCN_STAMPS
constexpr int kStampScen = 64, kStampStep0 = 1024, kStampSteps = 32;
#define FDCN_STAMP(k)                                                                 \
  do {                                                                                \
    if constexpr (kRec) {                                                             \
      if (scen < kStampScen && stamp_m >= kStampStep0 &&                              \
          stamp_m < kStampStep0 + kStampSteps) {                                      \
        const unsigned long long tt_ = __builtin_amdgcn_s_memtime();                  \
        if (lane == 0)                                                                \
          A.vsave[(size_t)scen * 64 * NPT + (stamp_m - kStampStep0) * 16 + (k)] =     \
              __longlong_as_double((long long)tt_);                                   \
      }                                                                               \
    }                                                                                 \
  } while (0)
#else
#define FDCN_STAMP(k) \
  do {                \
  } while (0)
#endif

template <int IT, int W, int NPT, int ZG = 0>
struct Geo {
  static constexpr bool kPair = (ZG & 4) != 0;
  static constexpr int L = kPair ? 32 : 64 * W;  // lanes per scenario
  static constexpr int SPB = kPair ? 2 : 1;  // scenarios per workgroup (LDS sized per scenario)
  // IT payoff staged in LDS unless it would not fit (8+ waves per scenario)
  static constexpr bool kPhiLds = IT && (W <= 4);
  static constexpr int kThreads = kPair ? 64 : 64 * W * SPB;
  // one-wave CN variants keep the weights of scan stages 2-5 in LDS (see
  // setup_scan); IT's LDS already holds the payoff
  static constexpr bool kScanLds = !IT && W == 1;
  // the current 64-step block of boundary terms, one double2 per step and
  // wave, read back as an LDS broadcast each step instead of four
  // v_readlane: CN only (A/B: config 3 5.25 -> 5.18 ms, config 5 18.43 ->
  // 18.35; IT, two waves per SIMD with the payoff in LDS, 11.08 -> 11.17),
  // not the paired flavour, whose halves read different scenarios' terms
  static constexpr bool kBndLds = !IT && !(ZG & 4);
};

// doubles of LDS per scenario
template <int IT, int W, int NPT, int ZG = 0>
__host__ __device__ inline int lds_doubles_per_scen(int lz) {
  return ((ZG & 1) ? 0 : sm_doubles(IT, W, NPT, ZG, lz)) +
         (Geo<IT, W, NPT, ZG>::kPhiLds ? 64 * W * NPT : 0) +
         (W > 1 ? Xch<W>::kSize : 0) + (Geo<IT, W, NPT, ZG>::kScanLds ? kScanLdsDoubles : 0) +
         (Geo<IT, W, NPT, ZG>::kBndLds ? 128 * W : 0) +
         (rec_form(IT, W, NPT) ? 2 : 0);  // the knock-out rebate slot (fdcn_ko_res.h)
}

// Issue priority of the zero-carry passes and the carry scans.  Each sweep
// is pass 1 (aggregates), a short dependent chain (sub-chain joins, the DPP
// scan, the carries), then pass 2.  Raised priority over pass 1 + scan lets
// a wave reach its carries first while the other wave of its SIMD streams
// the independent FMAs of its own pass 2 / update and fills the gaps.
// Measured (tools/gpu_ab.sh): scans only: config 2 12.44 -> 12.22 ms,
// config 3 6.66 -> 6.46 ms, config 5 unchanged; pass 1 + scan (this) a
// further -1.3 / -2.2 % on config 2 (two boxes), -0.6 % on config 5, config
// 3 neutral; raising it over the Sherman-Morrison broadcast lost time.
#define FDCN_PRIO_HI() __builtin_amdgcn_s_setprio(3)
#define FDCN_PRIO_LO() __builtin_amdgcn_s_setprio(0)
// Occupancy target: the config-3 throughput variant (CN, one wave, 16-node
// chunks) is held to 128 VGPRs, 4 waves per SIMD instead of 3 (measured
// 5.56 -> 5.44 ms per launch with the scan weights of stages 2-5 in LDS,
// against 5.94 before both); every other variant is unconstrained (1).
template <int IT, int W, int NPT, int ZG>
constexpr int kWavesPerEu = (!IT && W == 1 && NPT == 16 && !(ZG & 6)) ? 4 : 1;

// The register target the compiler is held to: the recovery-form variants
// (config 5) are held to two waves per SIMD (256 registers), where they sit
// at the edge: unconstrained, the resident-mask projection's build put 4 values
// of the boundary evaluation into AGPRs (260 registers, one wave per SIMD);
// held, they spill to scratch in the once-per-64-steps evaluation instead.
template <int IT, int W, int NPT, int ZG>
constexpr int kWavesTarget = rec_form(IT, W, NPT) ? 2 : kWavesPerEu<IT, W, NPT, ZG>;

template <int IT, int W, int NPT, int ZG = 0>
__global__ void __launch_bounds__(64 * W)
__attribute__((amdgpu_waves_per_eu(kWavesTarget<IT, W, NPT, ZG>)))
fdcn_march(KArgs A) {
#ifdef FDCN_WAVE_TIMES
  const unsigned long long wave_t0 = __builtin_amdgcn_s_memtime();
#endif
  constexpr int L = Geo<IT, W, NPT, ZG>::L;
  constexpr int SPB = Geo<IT, W, NPT, ZG>::SPB;
  constexpr bool kPair = Geo<IT, W, NPT, ZG>::kPair;
  static_assert(!kPair || (!IT && W == 1 && split_form(IT, W, NPT) && !(ZG & 3)),
                "paired flavour: split-form CN, one wave, LDS table");
  extern __shared__ __attribute__((aligned(16))) double lds[];
  // per-scenario uniform values: SGPRs, or per-lane values when a wave holds
  // two scenarios
  auto U = [](double x) __attribute__((always_inline)) { return kPair ? x : uni(x); };
  auto Ui = [](int x) __attribute__((always_inline)) { return kPair ? x : uni_i(x); };

  const int lane = threadIdx.x & 63;
  int lane4 = lane << 2;
  asm volatile("" : "+v"(lane4));  // one VGPR, never rematerialised in the loop
  const int half = kPair ? lane >> 5 : 0;    // the wave's scenario this lane serves
  const int hl = kPair ? lane & 31 : lane;   // lane within that scenario
  const int wave_blk = uni_i(threadIdx.x >> 6);
  const int scen_in_blk = kPair ? half : ((W == 1) ? wave_blk : 0);
  const int wave = (W == 1) ? 0 : wave_blk;  // wave index within the scenario
  const int scen0 = uni_i(blockIdx.x * SPB + (kPair ? 0 : scen_in_blk));
  if (scen0 >= A.B) return;  // whole wave(s) of a missing scenario leave together
  // a paired wave's second scenario may not exist (odd B): its lanes idle
  const bool valid = !kPair || scen0 + half < A.B;
  const int scen = kPair ? (valid ? scen0 + half : scen0) : scen0;
  const int t = wave * 64 + hl;

  const int n_nodes = A.n_nodes;
  const int n_int = n_nodes - 2;
  const int lz = A.lz;
  constexpr bool kPhiLds = Geo<IT, W, NPT, ZG>::kPhiLds;
  double* my = lds + (size_t)scen_in_blk * lds_doubles_per_scen<IT, W, NPT, ZG>(lz);
  // SM table [2][lz][NPT+1]: LDS, or this scenario's workspace slice (ZG)
  double* ztab = (ZG & 1) ? A.zg + (size_t)scen * 2 * lz * (NPT + 1) : my;
  double* phit = my + ((ZG & 1) ? 0 : sm_doubles(IT, W, NPT, ZG, lz));  // payoff [NPT][L] (kPhiLds)
  double* xch = phit + (kPhiLds ? L * NPT : 0);       // exchange area (W > 1)
  constexpr bool kScanLds = Geo<IT, W, NPT, ZG>::kScanLds;
  // scan weights of stages 2-5 (kScanLds), [stage-2][fwd, bwd][lane]; a paired
  // wave's two scenarios share the wave's one set (weights are per lane)
  double* sw = (kPair ? lds : xch + (W > 1 ? Xch<W>::kSize : 0)) +
               (kPair ? 2 * lds_doubles_per_scen<IT, W, NPT, ZG>(lz) - kScanLdsDoubles : 0);
  (void)sw;
  (void)xch;
  // this lane's column of the scan weights as an LDS byte address the
  // compiler cannot rematerialise (hide_addr at each use): the two-pass step
  // reads stages 2-5 off it with immediate offsets
  const unsigned sw_a = kScanLds ? lds_addr(sw + lane) : 0u;
  (void)sw_a;
  // this wave's block of boundary terms (kBndLds): after the scan weights
  constexpr bool kBndLds = Geo<IT, W, NPT, ZG>::kBndLds;
  double2* bblk = reinterpret_cast<double2*>(
                      xch + (W > 1 ? Xch<W>::kSize : 0) + (kScanLds ? kScanLdsDoubles : 0)) +
                  (kBndLds ? wave * 64 : 0);
  (void)bblk;
  // the rebate the resident-mask projection reads back into the knocked-out
  // slots (rec_form variants: ds_read_b64, fdcn_ko_res.h)
  double* ko_rbs = reinterpret_cast<double*>(bblk + (kBndLds ? 64 * W : 0));
  (void)ko_rbs;

  const double* P = A.params + (size_t)scen * FDCN_NPARAM;
  const int32_t* I = A.iparams + (size_t)scen * FDCN_NIPARAM;
  const double dt = U(P[FDCN_P_DT]);
  const double ca = U(P[FDCN_P_A]);
  const double cc = U(P[FDCN_P_C]);
  const double cbc = U(P[FDCN_P_BC]);
  const double tau0 = U(P[FDCN_P_TAU0]);

  // Boundary entries.  Step m's Dirichlet values at tau_m = tau0 + (m+1) dt
  // (…pricer.py:519), or with FDCN_I_TAU_MODE = 1 the reference American
  // loop's accumulated tau (tau = tau + dt per step,
  // fd_american_equity.py:664-724).  IT: what the step needs is not the value
  // itself but its theta-form rhs term (-A_L)(lo_m + c2 lo_{m-1}) /
  // (-A_U)(hi_m + c2 hi_{m-1}) (see the IT rhs below; IT has no knock-out, so
  // lo_{m-1} is simply the previous step's value).  The one-wave split-form
  // CN variants (kTabSplit) use the same term, th (-A_L)(lo_new + c2
  // lo_prev), with the expression and operand order of the in-loop form it
  // replaces; a knock-out that removes node 0 or the last node sets lo_prev
  // / hi_prev to the rebate instead, and the step after one recomputes its
  // term from the raw values.  Other CN variants take the raw values.
  // gen(c, raw) evaluates chunk c's entries, one step per lane (lane l: step
  // c + l), when the march reaches the chunk.  Up to round 4 a prologue
  // tabulated every step in the workspace and the march read the table back
  // (16-32 B per step and scenario each way: 0.5-1 GB of HBM traffic per
  // launch of configs 2, 3 and 5); the values are the same numbers, bitwise.
  // The boundary parameters are reloaded from `params` at each chunk rather
  // than kept live through the march.
  // kGen (the recovery-form variants, config 5): the chunk's entries are
  // evaluated in the march when it reaches the chunk, so no table crosses
  // HBM.  The other variants keep the round-4 table, filled by a prologue
  // (gen over every chunk) and read back per chunk: evaluated in the march
  // their exp temporaries sit on top of the march's live registers -- IT
  // (config 2) 245 -> 266 VGPRs (one wave per SIMD), the capped split-form
  // variant (config 3) 24 -> 128 B of scratch -- while config 5's variant
  // keeps two waves per SIMD (233 -> 255)
  constexpr bool kGen = rec_form(IT, W, NPT);
  constexpr bool kTabSplit = tab_form(IT, W, NPT, (ZG >> 1) & 1);
  double2* bnd = reinterpret_cast<double2*>(A.bnd) +
                 ((size_t)scen * W + wave) *
                     (kKoRow + (kGen ? kKoResRow : A.n_pad * (kTabSplit ? 2 : 1)));
  double2* kom_row = bnd + (kGen ? 0 : A.n_pad);
  double2* bnd_raw = kom_row + kKoRow;  // kTabSplit only
  (void)bnd_raw;
  const int tau_mode = Ui(I[FDCN_I_TAU_MODE]);
  // steps m = hl (mod L) are this lane's (kStride lanes per scenario)
  constexpr int kStride = kPair ? 32 : 64;
  double tau_end = tau0 + (double)A.n_time * dt;  // tau after the last step
  // tau_mode 1: the runs of the tau sequence (tau_next_run) are walked chunk
  // by chunk, each lane picking (tau_{m+1}, tau_m) of its own step from the
  // runs overlapping the chunk, so the exp stays outside any divergent branch
  double tc = tau0;
  int kc = 0;
  TauRun run;
  bool have_run = tau_mode == 1 && tau_next_run(tc, kc, A.n_pad, dt, run);
  const double* vb = A.v_init + (size_t)scen * n_nodes;
  const double v_lo0 = (IT || kTabSplit) ? U(vb[0]) : 0.0;
  const double v_hi0 = (IT || kTabSplit) ? U(vb[n_nodes - 1]) : 0.0;
  struct Bnd {  // the boundary parameters of this lane's scenario
    int lof, hif;
    double l0, l1, l2, l3, h0, h1, h2, h3, t0;
  };
  // (one scenario per wave: scalar loads through the constant address space
  // -- params / iparams are read-only for the launch -- so no VGPR holds a
  // loaded value; a paired wave's two scenarios load per lane)
  auto bnd_params = [&]() __attribute__((always_inline)) {
    if constexpr (kPair) {
      const double* Pg = P;
      const int32_t* Ig = I;
      asm volatile("" : "+v"(Pg), "+v"(Ig));
      return Bnd{Ig[FDCN_I_LO_FORM], Ig[FDCN_I_HI_FORM], Pg[FDCN_P_LO_C0], Pg[FDCN_P_LO_E0],
                 Pg[FDCN_P_LO_C1], Pg[FDCN_P_LO_E1], Pg[FDCN_P_HI_C0], Pg[FDCN_P_HI_E0],
                 Pg[FDCN_P_HI_C1], Pg[FDCN_P_HI_E1], Pg[FDCN_P_TAU0]};
    } else {
      typedef const double __attribute__((address_space(4))) cdbl;
      typedef const int32_t __attribute__((address_space(4))) cint;
      const cdbl* Pg = (const cdbl*)(uintptr_t)P;
      const cint* Ig = (const cint*)(uintptr_t)I;
      asm volatile("" : "+s"(Pg), "+s"(Ig));
      return Bnd{Ig[FDCN_I_LO_FORM], Ig[FDCN_I_HI_FORM], Pg[FDCN_P_LO_C0], Pg[FDCN_P_LO_E0],
                 Pg[FDCN_P_LO_C1], Pg[FDCN_P_LO_E1], Pg[FDCN_P_HI_C0], Pg[FDCN_P_HI_E0],
                 Pg[FDCN_P_HI_C1], Pg[FDCN_P_HI_E1], Pg[FDCN_P_TAU0]};
    }
  };
  auto gen = [&](int c, double2& raw) __attribute__((always_inline)) -> double2 {
    const Bnd q = bnd_params();
    const int m = c + hl;
    double tau = q.t0 + (double)(m + 1) * dt, tp = q.t0 + (double)m * dt;
    if (tau_mode == 1) {  // uniform per scenario: the runs overlapping [c, c + kStride)
      for (;;) {
        if (!have_run) break;
        if (run.k < A.n_time && A.n_time <= run.k + run.len)
          tau_end = (A.n_time == run.k + run.len)
                        ? run.t_next : run.t + (double)(A.n_time - run.k) * run.delta;
        if (m >= run.k && m < run.k + run.len) {
          const int j = m - run.k;
          tp = run.t + (double)j * run.delta;
          tau = (j + 1 == run.len) ? run.t_next : run.t + (double)(j + 1) * run.delta;
        }
        if (run.k + run.len >= c + kStride) break;  // continues into the next chunk
        have_run = tau_next_run(tc, kc, A.n_pad, dt, run);
      }
    }
    (void)tp;
    // kGen: the evaluations one after another (each argument made to depend
    // on the previous result), so their temporaries do not pile up on top of
    // the march's live registers
    auto seq = [](double x, double after) __attribute__((always_inline)) {
      if constexpr (kGen) asm volatile("" : "+v"(x) : "v"(after));
      return x;
    };
    auto ev = [](int f, double c0, double e0, double c1, double e1, double t, bool skip)
        __attribute__((always_inline)) {
      return kGen ? bnd_eval_nz(f, c0, e0, c1, e1, t, skip) : bnd_eval(f, c0, e0, c1, e1, t);
    };
    const double t_b = q.t0 + 1.01 * (double)A.n_time * dt;
    const double lo = ev(q.lof, q.l0, q.l1, q.l2, q.l3, tau, exp_finite_over(q.l1, q.l3, q.t0, t_b));
    const double hi = ev(q.hif, q.h0, q.h1, q.h2, q.h3, seq(tau, lo),
                         exp_finite_over(q.h1, q.h3, q.t0, t_b));
    raw = make_double2(lo, hi);
    if constexpr (IT) {
      const double lo_p = m == 0 ? v_lo0 : bnd_eval(q.lof, q.l0, q.l1, q.l2, q.l3, seq(tp, hi));
      const double hi_p = m == 0 ? v_hi0 : bnd_eval(q.hif, q.h0, q.h1, q.h2, q.h3, seq(tp, lo_p));
      const double th = m < A.n_ranna ? 1.0 : 0.5;
      const double c2 = (1.0 - th) / th;  // Phase::c2, pl, pu for this step's theta
      return make_double2((th * dt * ca) * fma(c2, lo_p, lo), (th * dt * cc) * fma(c2, hi_p, hi));
    } else if constexpr (kTabSplit) {
      // Phase::th, pl, pu, c2 of this step's theta (make_phase)
      const double lo_p = m == 0 ? v_lo0 : bnd_eval(q.lof, q.l0, q.l1, q.l2, q.l3, seq(tp, hi));
      const double hi_p = m == 0 ? v_hi0 : bnd_eval(q.hif, q.h0, q.h1, q.h2, q.h3, seq(tp, lo_p));
      const double th = m < A.n_ranna ? 1.0 : 0.5;
      const double AL = -th * dt * ca, AU = -th * dt * cc;
      const double c2 = (1.0 - th) / th;
      return make_double2(th * (-AL * fma(c2, lo_p, lo)), th * (-AU * fma(c2, hi_p, hi)));
    } else {
      return raw;
    }
  };
  // One-sided tables (round 6, the one-scenario split-form variants: config
  // 3).  A barrier scenario's Dirichlet side with zero coefficients (a call's
  // lower, a put's upper: …pricer.py:381-391) has the same raw value on every
  // step (+-0 while its exponentials stay finite), so its theta-form term
  // depends on the step only through theta and (step 0) v_init's end node:
  // the march recomputes it from scalars with the table's own expression
  // (term_const, bitwise the value gen produces) and the table keeps the
  // other side alone, 8 B a step instead of 16.  tsel: 0 both sides
  // tabulated (double2, as before), 1 the upper side alone (lower constant),
  // 2 the lower side alone.  The raw values behind the terms are read only
  // on the step after a knock-out of an edge node (entry s of the monitoring
  // run: step s) and after the last step, so only those are stored, and
  // only for a scenario whose knock-out reaches an edge node.  Config 3's
  // table traffic: 0.96 GB -> ~0.33 GB per launch.
  // Throughput batches of 16-40-node chunks only (config 3's 1 024-node
  // grids and the parity-mode barrier grids).  A single trade's march is
  // latency-bound, and there the one-sided table's extra prologue work and
  // live scalars cost ~4-6 % (trade_cnlog 0.41 -> 0.43 ms, trade_double 6.0
  // -> 6.4 ms on one box, profiles/r06/tab1_gate/): the chunk lengths the
  // single trades run on (8 and 12 nodes) do not compile it, and below
  // kTab1MinBatch scenarios the kernel keeps the two-sided table and every
  // raw value, as in round 5.
#ifdef FDCN_NO_TAB1  // diagnostic builds only
  constexpr bool kTab1 = false;
#else
  constexpr bool kTab1 = kTabSplit && !kPair && NPT >= 16;
#endif
  const bool tab1_on = kTab1 && A.B >= kTab1MinBatch;
  (void)tab1_on;
  int tsel = 0;
  double rc_lo = 0.0, rc_hi = 0.0;  // the constant side's raw value
  (void)tsel;
  (void)rc_lo;
  (void)rc_hi;
  double* bnd1 = reinterpret_cast<double*>(bnd);       // one-sided table (kTab1, tsel != 0)
  double* braw1 = reinterpret_cast<double*>(bnd_raw);  // its raw values
  (void)bnd1;
  (void)braw1;
  if (tab1_on) {
    const Bnd q = bnd_params();
    const double t_a = q.t0, t_b = q.t0 + 1.01 * (double)A.n_time * dt;
    auto side_const = [&](int f, double c0, double e0, double c1, double e1) {
      const bool zero = f == 1 ? (c0 == 0.0 || c1 == 0.0) : (c0 == 0.0 && c1 == 0.0);
      return zero && isfinite(c0) && isfinite(c1) && exp_finite_over(e0, e1, t_a, t_b);
    };
    if (side_const(q.lof, q.l0, q.l1, q.l2, q.l3)) tsel = 1;
    else if (side_const(q.hif, q.h0, q.h1, q.h2, q.h3)) tsel = 2;
    rc_lo = U(bnd_eval(q.lof, q.l0, q.l1, q.l2, q.l3, q.t0));
    rc_hi = U(bnd_eval(q.hif, q.h0, q.h1, q.h2, q.h3, q.t0));
    tsel = Ui(tsel);
  }
  if constexpr (!kGen) {  // the table: every chunk up front, while few registers are live
    // kTab1: the steps whose raw values are read (see above), a 64-bit mask
    // per chunk from a walk over the scenario's monitoring run (strictly
    // increasing entries, validated on the host)
    int mp = 0, mpe = 0;
    bool edge_ko = false, m_need_all = false;
    if constexpr (kTab1) {
      mp = Ui(I[FDCN_I_MON_START]);
      mpe = mp + Ui(I[FDCN_I_MON_COUNT]);
      edge_ko = Ui(I[FDCN_I_KO_LO]) >= 0 || n_nodes - 1 >= Ui(I[FDCN_I_KO_HI]);
      // a knock-out after every step, or a latency batch: every raw value
      m_need_all = !tab1_on || (edge_ko && mpe - mp >= A.n_time);
    }
    for (int c = 0; c < A.n_pad; c += kStride) {
      double2 raw;
      const double2 e = gen(c, raw);
      if (!valid) continue;  // a paired wave's missing scenario: no stores
      if constexpr (kTab1) {
        // this chunk's monitor entries, 64 at a time: lane l loads entry
        // mp + l; the run's entries below c + 64 are a prefix of them (sorted;
        // an unsorted _dev run stops at its first larger entry, whose
        // followers the march skips too), and each one in [c, c + 64) flags
        // its step in the wave's boundary row of LDS (free until the march),
        // which lane hl then reads back.  Monitoring on every step (config
        // 5's window trade) needs every raw value: no walk.  (A scalar walk,
        // one dependent load per entry, cost the 8 192-step single trade
        // 1.3 ms.)
        bool nd = m_need_all || (c + hl == A.n_time - 1);
        if (!m_need_all && edge_ko && mp < mpe) {
          int* flag = reinterpret_cast<int*>(bblk);
          flag[lane] = 0;
          const int sm = mp + lane < mpe ? A.mon_step[mp + lane] : 0x7fffffff;
          const unsigned long long below =
              (unsigned long long)__ballot(sm < c + kStride);
          const int run_len = below == ~0ull ? 64 : __builtin_ctzll(~below);
          if (lane < run_len && sm >= c) flag[sm - c] = 1;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          nd = nd || flag[hl] != 0;
          mp += run_len;
        }
        if (tsel) {
          bnd1[c + hl] = tsel == 1 ? e.y : e.x;
          if (nd) braw1[c + hl] = tsel == 1 ? raw.y : raw.x;
        } else {
          bnd[c + hl] = e;
          if (nd) bnd_raw[c + hl] = raw;
        }
      } else {
        bnd[c + hl] = e;
        if constexpr (kTabSplit) bnd_raw[c + hl] = raw;
      }
    }
  }
  // kTab1: the constant side's theta-form term of step m, the expression gen
  // uses (lo_p = v_init's end node on step 0, the constant raw value after)
  auto term_const = [&](int m, double rc, double v0, double coef) __attribute__((always_inline)) {
    const double th = m < A.n_ranna ? 1.0 : 0.5;
    const double Ax = -th * dt * coef;
    const double c2 = (1.0 - th) / th;
    return th * (-Ax * fma(c2, m == 0 ? v0 : rc, rc));
  };
  // a block's boundary terms from the table (kTab1: the pair rebuilt)
  auto tab_load = [&](int i) __attribute__((always_inline)) -> double2 {
    if constexpr (kTab1) {
      if (tsel == 1) return make_double2(term_const(i, rc_lo, v_lo0, ca), bnd1[i]);
      if (tsel == 2) return make_double2(bnd1[i], term_const(i, rc_hi, v_hi0, cc));
    }
    return bnd[i];
  };
  // the raw Dirichlet values of step i (kTab1: the constant side from rc)
  auto raw_load = [&](int i) __attribute__((always_inline)) -> double2 {
    if constexpr (kTab1) {
      if (tsel == 1) return make_double2(rc_lo, braw1[i]);
      if (tsel == 2) return make_double2(braw1[i], rc_hi);
    }
    return bnd_raw[i];
  };
  (void)tab_load;
  (void)raw_load;

  // lane geometry
  const int L_act = (n_int + NPT - 1) / NPT;
  const int L_short = L_act * NPT - n_int;
  const bool active = t < L_act && valid;
  const bool shrt = t < L_short;
  // 1.0 on the lane that holds interior node 0 / the last interior node
  const double e_first = (t == 0 && valid) ? 1.0 : 0.0;
  const double e_last = (t == L_act - 1 && valid) ? 1.0 : 0.0;
  (void)e_first;
  (void)e_last;
  const int s_t = t * NPT - (t < L_short ? t : L_short);  // first interior index

  // ---- chunk decomposition for instruction-level parallelism -------------
  // Each lane's NPT-node chunk is split into S sub-chains of M nodes.  The
  // recurrences run the S sub-chains interleaved (independent FMA chains) and
  // join them with a short Horner step in fm^M / bm^M, so a wave keeps S
  // fp64 FMAs in flight instead of one dependent chain.  The joins and
  // their carries cost 2(S-1) FMAs per sweep and lane.  With the priority
  // scheme above, the throughput variants (W = 1, 2-3 waves per SIMD) hide
  // the FMA latency with the other waves: one chain (S = 1) measured
  // fastest up to 40 nodes per lane, two at 48-64 (tools/gpu_ab.sh: config
  // 2 12.31 -> 12.08 ms, config 3 6.54 -> 6.21 ms, config 5 20.65 -> 19.69 ms
  // against S = 4).  The multi-wave variants serve small batches, where one
  // wave per SIMD needs the in-wave ILP: they keep 4.  Re-measured in round 2
  // with the current kernel (tools/gpu_ab.sh, one box, two runs each): the
  // IT NPT = 32 variant (config 2, two waves per SIMD) is now faster with
  // four: S = 1 11.39 ms, S = 2 11.38, S = 4 11.20; config 3 keeps one
  // (5.91 against 6.04 with four).
  constexpr int S = sub_chains(IT, W, NPT, ZG);
  constexpr int M = NPT / S;

  // ---- per-theta constants: scan window products + SM table -------------
  double FW[6], GW[6];
  double Fpre = 0.0, Gsuf = 0.0;
  double mlast = 0.0, glast = 0.0;  // phantom slot: pass-through multipliers
  // Lane masks folded into multipliers (no v_cndmask in the step).
  // Inactive lanes hold exact zeros in every vector, so their zero-carry
  // values and scan results are zero by themselves; only the carry an
  // inactive lane receives from the last active one must be dropped, which
  // the first forward pass-2 multipliers (fm_act, fmM_act: 0 there) do.
  // The phantom slot's pass-2 multiplier mlast2 (0 on short lanes) writes
  // the phantom's zero rhs instead of the passed-through value.
  double fm_act = 0.0, fmM_act = 0.0, mlast2 = 0.0;
  // glast2: the backward carry multiplier of the chunk's last node, 0 on the
  // last lane of a paired wave's first scenario (its neighbour lane belongs
  // to the other scenario); glast elsewhere
  double glast2 = 0.0;
  double mulLF = 0.0, mulLB = 0.0;  // products across the last sub-chain
  double fmM = 0.0, bmM = 0.0;      // products across a full sub-chain
  int nst_f = 6, nst_b = 6;         // scan stages that carry weight above 1e-18
  // kRec: the phase's |fm|^(NPT/2) and |bm|^(NPT/2) are below 1e-18, so the
  // zero-carry aggregates need only half a chunk (solve_rec_half)
  bool rec_half = false;
  // kRec (solve_rec), per phase: the product of the forward multipliers
  // over the chunk's last quarter (fm^(Q-1) mlast, per lane: short lanes
  // end one node early); uniform fm^(H-1) and bm^H for the rare branch
  double recQ = 0.0, rec_fmH1 = 0.0, rec_bmH = 0.0;
  (void)recQ;
  (void)rec_fmH1;
  (void)rec_bmH;
  Phase ph;
  // Step forms (see the time loop):
  //   IT            state (V, Q), pointwise rhs V + Q, solve in place on V
  //   CN, kSplit    state V, rhs V (+ boundary terms), solve into T
  //   CN, kRec      state V, rhs V (+ boundary terms), solve in place; the
  //                 last backward pass recovers the old V (W = 1, NPT > 40)
  //   CN, stencil   state V, 3-point rhs in place (shifted layout); the
  //                 multi-wave variants whose V + T would not fit the
  //                 register budget
  constexpr bool kSplit = split_form(IT, W, NPT);
  // CN, recover (W = 1, NPT > 40): state V only, pointwise rhs V solved in
  // place; the update x = s u - c2 V needs the old V, which the last
  // backward pass recovers from the forward-pass values it is about to
  // overwrite (V_k = w_k - fm w_{k-1}), so no second vector is live.
  // Rannacher steps (c2 = 0) add the old V back from a workspace copy.
  // Config 5 (NPT = 64): 26.0 -> 23.8 ms per launch against the stencil form.
  constexpr bool kRec = rec_form(IT, W, NPT);
  static_assert(!(kRec && kSplit), "one step form per variant");
  // two-pass solve (see two_pass): tables per phase at ztab + tab * kTPh
  constexpr bool kTP = two_pass(IT, W, NPT, ZG);
  // the split-form CN on the two-pass solve, tables as DPP broadcasts
  constexpr bool kTPS = kTP && !IT;
  // kTPS: the homogeneous part added to T before the update (tables not
  // scaled by s), the phantom slot zeroed by its scale instead of a reset
  constexpr bool kTPST = kTPS && NPT <= 16;
  static_assert(!kTP || (M >= 2 && !kPair), "two-pass: one scenario per wave, M >= 2");
  static_assert(!kTPS || (kSplit && S == 1), "split two-pass: the split form, S = 1");
  // DPP broadcast table registers per table (16 entries each)
  constexpr int kTabRegs = kTPS ? (M + 15) / 16 : 1;
  // doubles per phase: P', G, the lz Sherman-Morrison rows and a zero row
  // (the lanes past the table read it)
  const int kTPh = kTP ? 2 * M + (lz + 1) * 2 * S : 0;
  // per sub-chain coefficients of the homogeneous part (two-pass solve), the
  // solution's value at the chunk's first node after the backward scan, and
  // per-lane phase constants: P'_0 of the last sub-chain (short lanes: one
  // node less), the short-lane transform of the last sub-chain's D (k1, k2),
  // the backward pass-1 multiplier into the last real node (0 on short lanes)
  double CC[S], DD[S];  // kTP only (unused arrays vanish elsewhere)
  double cbv = 0.0, P0u = 0.0, p0l = 0.0, k1 = 0.0, k2 = 0.0, bw1l = 0.0;
  (void)CC;
  (void)DD;
  (void)cbv;
  (void)P0u;
  (void)p0l;
  (void)k1;
  (void)k2;
  (void)bw1l;
  (void)kTPh;
  constexpr bool kNatural = IT || kSplit || kRec;  // solve input in the natural layout
  double V[NPT];
  double X = 0.0;  // node 0 of the shifted RHS layout (stencil CN; see solve)
  // IT: the second state vector Q = V/theta - W, where W is the last
  // pre-projection value (V = max(phi, W)); see the IT step below
  double QS[IT ? NPT : 1];
  double T[kSplit ? NPT : 1];  // kSplit: the solve's work vector
  double vb0 = 0.0, vb1 = 0.0;  // kSplit: rhs of the chunk's first/last node
  // kRec: boundary terms added to the rhs this step (recovery subtracts
  // them), the solution at the chunk's node 0 before the update, and the
  // per-lane update scale (0 on the phantom slot of short lanes)
  double rec_lo = 0.0, rec_hi = 0.0, y0c = 0.0, s_l = 0.0;
  (void)rec_lo;
  (void)rec_hi;
  (void)y0c;
  (void)s_l;
  (void)QS;
  (void)T;
  (void)vb0;
  (void)vb1;

  auto setup_scan = [&](const Phase& p) __attribute__((always_inline)) {
    if constexpr (W > 1) __syncthreads();  // previous readers of Ftot/Gtot are done
    mlast = shrt ? 1.0 : p.fm;
    glast = shrt ? 1.0 : p.bm;
    mlast2 = shrt ? 0.0 : p.fm;
    glast2 = (kPair && hl == 31) ? 0.0 : glast;
    // kPair: lane 32 also drops the forward carry it receives from lane 31
    fm_act = (active && !(kPair && hl == 0)) ? p.fm : 0.0;
    const double fM1 = pow_n<NPT>(p.fm, M - 1), bM1 = pow_n<NPT>(p.bm, M - 1);
    fmM = U(fM1 * p.fm);
    bmM = U(bM1 * p.bm);
    mulLF = shrt ? fM1 : fmM;
    fmM_act = active ? fmM : 0.0;
    mulLB = shrt ? bM1 : bmM;
    if constexpr (kTP) {
      // P'_0 = sum_{k<M} bm^k fm^k; a short lane's last sub-chain ends one
      // node early: P'_0 - fm^(M-1) bm^(M-1), and its backward carry enters
      // at slot M-2, bm^(M-1-i) = G_i / bm, with its forward part
      // -C fm^(M-1) moved over (D'' = (D - C fm^(M-1)) / bm; any D when
      // bm = 0, where G_i vanishes on the real slots)
      double acc = 0.0;
#pragma unroll
      for (int k = M - 1; k >= 0; --k) acc = fma(p.bm, acc, pow_n<NPT>(p.fm, k));
      P0u = U(acc);
      p0l = shrt ? P0u - fM1 * bM1 : P0u;
      k1 = shrt ? -fM1 : 0.0;
      k2 = shrt ? (p.bm != 0.0 ? 1.0 / p.bm : 0.0) : 1.0;
      bw1l = shrt ? 0.0 : p.bm;
    }
    const int len = shrt ? NPT - 1 : NPT;
    double f = active ? pow_n<NPT>(p.fm, len) : 0.0;
    double g = active ? pow_n<NPT>(p.bm, len) : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      // zero where the shuffle source lane does not exist: the scan step
      // b += FW*b_src then needs no lane mask
      // (kPair: lanes of the other scenario count as missing sources)
      FW[j] = (hl >= d) ? f : 0.0;
      GW[j] = (hl + d < kStride) ? g : 0.0;
      const double fo = shfl_up1(f, d);
      const double go = shfl_dn1(g, d);
      f = (hl >= d) ? f * fo : f;
      g = (hl + d < kStride) ? g * go : g;
    }
    Fpre = f;
    Gsuf = g;
    if constexpr (kScanLds) {
      // stages 2-5 are rare (only when |fm|^(NPT-1) > 3e-5): their weights
      // wait in LDS, so only stages 0-1 hold registers in the march
#pragma unroll
      for (int j = 2; j < 6; ++j) {
        sw[(j - 2) * 128 + lane] = FW[j];
        sw[(j - 2) * 128 + 64 + lane] = GW[j];
      }
    }
    // After j Hillis-Steele stages lane t holds the contributions of lanes
    // t-2^j+1..t; the rest is scaled by at most q^(2^j), q = |fm|^(NPT-1)
    // (a short lane's product, the largest).  Stop once that is <= 1e-18:
    // the dropped part is then ~1e-18 of the carried values, below fp64
    // rounding (the same criterion as the Sherman-Morrison extent).
    {
      double qf = fabs(pow_n<NPT>(p.fm, NPT - 1)), qb = fabs(pow_n<NPT>(p.bm, NPT - 1));
      constexpr int kMaxSt = kPair ? 5 : 6;
      int nf = 0, nb = 0;
      while (nf < kMaxSt && qf > 1e-18) { qf *= qf; ++nf; }
      while (nb < kMaxSt && qb > 1e-18) { qb *= qb; ++nb; }
      nst_f = kPair ? umax_halves(nf) : uni_i(nf);
      nst_b = kPair ? umax_halves(nb) : uni_i(nb);
      if constexpr (rec_form(IT, W, NPT)) {
        const double hf = fabs(pow_n<NPT>(p.fm, NPT / 2)), hb = fabs(pow_n<NPT>(p.bm, NPT / 2));
        rec_half = uni_i(hf < 1e-18 && hb < 1e-18) != 0;
        rec_fmH1 = U(pow_n<NPT>(p.fm, NPT / 2 - 1));
        rec_bmH = U(pow_n<NPT>(p.bm, NPT / 2));
        recQ = pow_n<NPT>(p.fm, NPT / 4 - 1) * mlast;
      }
    }
    if constexpr (W > 1) {
      if (lane == 63) xch[Xch<W>::kFtot + wave] = Fpre;
      if (lane == 0) xch[Xch<W>::kGtot + wave] = Gsuf;
      __syncthreads();
    }
  };

  // Forward + backward sweeps.  Stencil CN input: rhs/r in the SHIFTED
  // layout left by the in-place RHS (node 0 in X, node k >= 1 in V[k-1]);
  // the last backward pass writes node k into V[k] while reading node k's
  // forward value from V[k-1], which undoes the shift at no cost; output in
  // V.  IT / kSplit input: the unscaled rhs in the natural layout (In); the
  // passes work in place on Wr (V for IT, T for kSplit) and return r times
  // the solution there.
  auto In = [&](int k) -> double {
    if constexpr (IT || kRec) return V[k];
    else if constexpr (kSplit) return k == 0 ? vb0 : (k == NPT - 1 ? vb1 : V[k]);
    else return k == 0 ? X : V[k - 1];
  };
  auto Wr = [&](int k) -> double& {
    if constexpr (IT || kRec) return V[k];
    else if constexpr (kSplit) return T[k];
    else return k == 0 ? X : V[k - 1];
  };
  // where the solve leaves the solution (natural layout)
  auto Out = [&](int k) -> double& {
    if constexpr (kSplit) return T[k];
    else return V[k];
  };
  // fz: std::true_type fuses the kRec update into the last backward pass
  auto solve = [&](const Phase& p, auto fz) __attribute__((always_inline)) {
    constexpr bool kFuse = decltype(fz)::value;
    // one-wave variants: scan stages 0-1 run inline, the rest behind one
    // uniform branch.  The recovery form keeps only stage 0 inline: config 5
    // needs none at 64 nodes per lane (|fm|^63 < 1e-18), and stage 1 behind
    // the branch took 17.50 -> 17.22 ms and 17.57 -> 17.25 in two A/B calls
    // (stage 0 behind it as well: no better, 17.24).  The same move on the
    // two-pass IT variant (config 2) cost 5 %: 10.68 -> 11.25 ms.
    constexpr int kInlS = kRec ? 1 : 2;
    const double fm = p.fm, bm = p.bm;
    FDCN_PRIO_HI();  // pass 1 + scan raised, pass 2 at the base priority
    // forward pass 1: zero-carry end value of every sub-chain
    double a[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      double w = In(j * M);  // zero carry: the first FMA is the input itself
#pragma unroll
      for (int i = 1; i < M; ++i) {
        const int k = j * M + i;
        w = fma(k == NPT - 1 ? mlast : fm, w, In(k));
      }
      a[j] = w;
    }
    double e = a[0];
#pragma unroll
    for (int j = 1; j < S; ++j) e = fma(j == S - 1 ? mulLF : fmM, e, a[j]);
    double b = e;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      if constexpr (W == 1) {
        // stages 0-1 inline, the rest behind one uniform branch.  The split
        // form tests stages 0-1 too (config 3 scenarios need one or two:
        // 5.17 -> 5.12 ms in A/B).  IT and the recovery form run them
        // unconditionally (the recovery form stage 0 only, see kInlS):
        // configs 2 and 5 need none (|fm|^(NPT-1) < 1e-18, the neighbour's
        // aggregate is the whole carry), yet skipping both behind branches
        // measured no faster there (11.03 / 17.52 -> 11.03 / 17.65 ms), the
        // branches splitting the dependent chain the scheduler overlaps
        if (j < kInlS && (!kSplit || j < nst_f)) b = fma(FW[j], scan_up(b, d, lane4), b);
      } else if (j < nst_f) {
        b = fma(FW[j], scan_up(b, d, lane4), b);
      }
    }
    if (W == 1 && nst_f > kInlS) {
#pragma unroll
      for (int j = kInlS; j < 6; ++j) {
        const int d = 1 << j;
        const double wf = (kScanLds && j >= 2) ? sw[(j - 2) * 128 + lane] : FW[j];
        if (j < nst_f) b = fma(wf, scan_up(b, d, lane4), b);
      }
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
    double cin = shfl_up1(b, 1);  // DPP bound_ctrl: lane 0 receives 0 (= cw for W = 1)
    if (W > 1 && lane == 0) cin = cw;
    // forward pass 2: carries into every sub-chain, then S chains in parallel
    double c[S];
    c[0] = cin;
#pragma unroll
    for (int j = 1; j < S; ++j) c[j] = fma(j == 1 ? fmM_act : fmM, c[j - 1], a[j - 1]);
    FDCN_PRIO_LO();
    double cf[S];  // kFuse: the values each sub-chain's first FMA multiplied
#pragma unroll
    for (int j = 0; j < S; ++j) cf[j] = c[j];
    (void)cf;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      double w = c[j];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int k = j * M + i;
        w = fma(k == NPT - 1 ? mlast2 : (k == 0 ? fm_act : fm), w, In(k));
        Wr(k) = w;
      }
    }
    FDCN_PRIO_HI();
    // backward pass 1: zero-carry start value of every sub-chain
#pragma unroll
    for (int j = 0; j < S; ++j) {
      double y = Wr(j * M + M - 1);  // zero carry
#pragma unroll
      for (int i = M - 2; i >= 0; --i) {
        const int k = j * M + i;
        y = fma(k == NPT - 1 ? glast : bm, y, Wr(k));
      }
      a[j] = y;
    }
    // zero-carry start value of the chunk: E_j = a[j] + prod(sub-chain j) E_{j+1};
    // sub-chains j <= S-2 never hold the phantom slot, so the product is bm^M
    e = a[S - 1];
#pragma unroll
    for (int j = S - 2; j >= 0; --j) e = fma(bmM, e, a[j]);
    double cb = e;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      if constexpr (W == 1) {
        if (j < kInlS && (!kSplit || j < nst_b)) cb = fma(GW[j], scan_dn(cb, d, lane4), cb);
      } else if (j < nst_b) {
        cb = fma(GW[j], scan_dn(cb, d, lane4), cb);
      }
    }
    if (W == 1 && nst_b > kInlS) {
#pragma unroll
      for (int j = kInlS; j < 6; ++j) {
        const int d = 1 << j;
        const double wg = (kScanLds && j >= 2) ? sw[(j - 2) * 128 + 64 + lane] : GW[j];
        if (j < nst_b) cb = fma(wg, scan_dn(cb, d, lane4), cb);
      }
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
    double cinb = shfl_dn1(cb, 1);  // lane 63 receives 0 (= cwb for W = 1)
    if (W > 1 && lane == 63) cinb = cwb;
    c[S - 1] = cinb;
#pragma unroll
    for (int j = S - 2; j >= 0; --j) c[j] = fma(j + 1 == S - 1 ? mulLB : bmM, c[j + 1], a[j + 1]);
    FDCN_PRIO_LO();
    if constexpr (kFuse) {
      // backward pass 2 fused with the kRec update, per node (descending):
      //   u   = mul_b u + w_k                      (chain value, in uc[j])
      //   -V_k = mul_f w_{k-1} - w_k (+ the boundary term added to the rhs)
      //   x_k = s u - V_k                          (over V[k])
      // w_{k-1} is still in V[k-1] (processed later in this pass) or, at a
      // sub-chain's first node, the value its forward FMA multiplied (cf).
      double uc[S];
#pragma unroll
      for (int j = 0; j < S; ++j) uc[j] = c[j];
      // Per node index i, the S sub-chains' three FMAs are issued stage by
      // stage (S chain steps, S recoveries, S updates), so no FMA waits on
      // the one issued just before it.
#pragma unroll
      for (int i = M - 1; i >= 0; --i) {
        double tt[S];
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int k = j * M + i;
          if (k == NPT - 1)
            asm volatile("v_fma_f64 %0, %1, %0, %2" : "+v"(uc[j]) : "v"(glast), "v"(V[k]));
          else
            asm volatile("v_fma_f64 %0, %1, %0, %2" : "+v"(uc[j]) : "s"(bm), "v"(V[k]));
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int k = j * M + i;
          const double wprev = (i == 0) ? cf[j] : V[k - 1];
          if (k == NPT - 1) {
            asm volatile("v_fma_f64 %0, %1, %2, -%3"
                         : "=v"(tt[j]) : "v"(mlast2), "v"(wprev), "v"(V[k]));
            tt[j] = fma(e_last, rec_hi, tt[j]);
          } else if (k == 0) {
            asm volatile("v_fma_f64 %0, %1, %2, -%3"
                         : "=v"(tt[j]) : "v"(fm_act), "v"(wprev), "v"(V[k]));
            tt[j] = fma(e_first, rec_lo, tt[j]);
          } else {
            asm volatile("v_fma_f64 %0, %1, %2, -%3"
                         : "=v"(tt[j]) : "s"(fm), "v"(wprev), "v"(V[k]));
          }
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int k = j * M + i;
          if (k == NPT - 1)
            asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "v"(s_l), "v"(uc[j]), "v"(tt[j]));
          else
            asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "s"(p.s), "v"(uc[j]), "v"(tt[j]));
        }
      }
      y0c = uc[0];
    } else if constexpr (kNatural) {
      // backward pass 2 in place (natural layout): y_k = mul*y_{k+1} + w_k
      // over Wr(k); the S sub-chains round-robin, as below
#pragma unroll
      for (int i = M - 1; i >= 0; --i) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int k = j * M + i;
          const double yn = (i == M - 1) ? c[j] : Wr(k + 1);
          if (k == NPT - 1)
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(Wr(k)) : "v"(glast2), "v"(yn));
          else if constexpr (kPair)
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(Wr(k)) : "v"(bm), "v"(yn));
          else
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(Wr(k)) : "s"(bm), "v"(yn));
        }
      }
    } else {
      // backward pass 2 (unshifting).  Sub-chain j-1 writes V[jM-1], which
      // holds sub-chain j's last input (node jM): read those first.
      double wbot[S];
#pragma unroll
      for (int j = 1; j < S; ++j) wbot[j] = Wr(j * M);
      // y_k = mul*y_{k+1} + w_k written over V[k] (whose value, w_{k+1}, was
      // read one node earlier): the "+v" tie pins y_k to V[k]'s register so
      // the vector stays in one register set.  The S sub-chains are issued
      // round-robin (one asm statement per instruction, volatile to keep that
      // order) so S independent FMAs are in flight.
#pragma unroll
      for (int i = M - 1; i >= 0; --i) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int k = j * M + i;
          const double wk = (i == 0 && j > 0) ? wbot[j] : Wr(k);
          const double yn = (i == M - 1) ? c[j] : V[k + 1];
          if (k == NPT - 1)
            asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "v"(glast), "v"(yn), "v"(wk));
          else
            asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "s"(bm), "v"(yn), "v"(wk));
        }
      }
    }
  };

  // The recovery form's solve (kRec; replaces solve() there).  A chunk's
  // zero-carry aggregate -- what the right neighbour's carry is made of --
  // sums its nodes with weights fm^(distance to the chunk's end).  When the
  // phase's |fm|^(NPT/2) and |bm|^(NPT/2) are below 1e-18 (rec_half: config
  // 5's Crank-Nicolson phase, |fm| ~ 0.2 at NPT = 64) the first half's
  // weights fall under the 1e-18 cut the scan stages and the
  // Sherman-Morrison extent use (and the scan stages carry nothing either):
  // the forward aggregate takes the second half, the backward one the first
  // half.  Otherwise (the Rannacher steps) a uniform branch adds the other
  // halves and the scan stages; it only reads V.
  // Forward pass 1 runs the aggregate's two quarters as two chains joined
  // by one FMA; pass 2 runs the first half as one chain, then the second
  // half with the backward aggregate of the first half (which reads only
  // final values) alongside; backward pass 2 is fused with the update.
  // Plain FMAs where the compiler can schedule them: around inline asm it
  // pads dependent v_fma_f64 pairs with s_nop (an issue slot each), which a
  // lone asm chain paid on every link.  A lone chain of plain FMAs costs ~6
  // cycles per link against ~4.2 for independent ones (one wave,
  // tools/ubench/fma64_latency.hip), so a chain is split only where the
  // split is cheap.  Per node-step 4 + ~1 FMAs against 6 + the joins.
  int stamp_m = -1;  // FDCN_STAMPS: the step being stamped
  (void)stamp_m;
  auto solve_rec = [&](const Phase& p) __attribute__((always_inline)) {
    constexpr int H = NPT / 2, Q = NPT / 4;
    const double fm = p.fm, bm = p.bm;
    FDCN_PRIO_HI();
    double a2 = V[H], a3 = V[H + Q];
#pragma unroll
    for (int i = 1; i < Q; ++i) {
      a2 = fma(fm, a2, V[H + i]);
      a3 = fma(H + Q + i == NPT - 1 ? mlast : fm, a3, V[H + Q + i]);
    }
    double w = fma(recQ, a2, a3);  // the second half's aggregate
    if (!rec_half) {
      // the first half enters with the second half's multipliers
      double a0 = V[0];
#pragma unroll
      for (int i = 1; i < H; ++i) a0 = fma(fm, a0, V[i]);
      w = fma(rec_fmH1 * mlast, a0, w);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double wf = (kScanLds && j >= 2) ? sw[(j - 2) * 128 + lane] : FW[j];
        if (j < nst_f) w = fma(wf, scan_up(w, 1 << j, lane4), w);
      }
    }
    FDCN_STAMP(1);
    const double cin = shfl_up1(w, 1);  // lane 0 receives 0
    FDCN_PRIO_LO();
    // forward pass 2 over the first half from the carry (fm_act: 0 on
    // inactive lanes)
    V[0] = fma(fm_act, cin, V[0]);
#pragma unroll
    for (int k = 1; k < H; ++k) V[k] = fma(fm, V[k - 1], V[k]);
    // the second half, with the backward zero-carry aggregate of nodes
    // H-1..0 alongside
    FDCN_STAMP(2);
    double y = V[H - 1];
#pragma unroll
    for (int k = H; k < NPT; ++k) {
      V[k] = fma(k == NPT - 1 ? mlast2 : fm, V[k - 1], V[k]);
      const int kb = H - 1 - (k - H + 1);
      if (kb >= 0) y = fma(bm, y, V[kb]);
    }
    FDCN_PRIO_HI();
    if (!rec_half) {
      // nodes NPT-1..H enter the backward aggregate with bm^H
      double y2 = V[NPT - 1];
#pragma unroll
      for (int k = NPT - 2; k >= H; --k) y2 = fma(bm, y2, V[k]);
      y = fma(rec_bmH, y2, y);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double wg = (kScanLds && j >= 2) ? sw[(j - 2) * 128 + 64 + lane] : GW[j];
        if (j < nst_b) y = fma(wg, scan_dn(y, 1 << j, lane4), y);
      }
    }
    FDCN_STAMP(3);
    const double cinb = shfl_dn1(y, 1);  // lane 63 receives 0
    FDCN_PRIO_LO();
    // backward pass 2 fused with the update, per node (descending), as in
    // solve(): u = bm u + w_k; -V_k = fm w_{k-1} - w_k (+ boundary term);
    // x_k = s u - V_k over V[k].  Software-pipelined so no FMA reads a
    // result of the two instructions before it (that costs an s_nop):
    // group k issues the chain step of node k, the recovery of node k-1 and
    // the update of node k+1 (whose forward value every reader has used)
    double uc = cinb;
    double tt[NPT], ucs[NPT];
    auto rec_tt = [&](int k) __attribute__((always_inline)) {
      const double wprev = (k == 0) ? cin : V[k - 1];
      const double mk = (k == NPT - 1) ? mlast2 : (k == 0 ? fm_act : fm);
      tt[k] = fma(mk, wprev, -V[k]);
      if (k == NPT - 1) tt[k] = fma(e_last, rec_hi, tt[k]);
      if (k == 0) tt[k] = fma(e_first, rec_lo, tt[k]);
    };
    auto rec_upd = [&](int k) __attribute__((always_inline)) {
      // in V[k]'s register (asm: the compiler's accumulate form would
      // first copy tt there)
      if (k == NPT - 1)
        asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "v"(s_l), "v"(ucs[k]), "v"(tt[k]));
      else
        asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(V[k]) : "s"(p.s), "v"(ucs[k]), "v"(tt[k]));
    };
    rec_tt(NPT - 1);
#pragma unroll
    for (int k = NPT - 1; k >= 0; --k) {
      if (k == NPT - 1)
        asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(ucs[k]) : "v"(glast), "v"(uc), "v"(V[k]));
      else
        asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(ucs[k]) : "s"(bm), "v"(uc), "v"(V[k]));
      uc = ucs[k];
      if (k >= 1) rec_tt(k - 1);
      if (k + 1 < NPT) rec_upd(k + 1);
    }
    rec_upd(0);
    y0c = uc;
    FDCN_STAMP(4);
  };

  // Two-pass solve (kTP, W = 1): both zero-carry passes in place on Wr, the
  // carries into CC / DD (see two_pass); the caller adds C P'_i + D G_i.
  // cbv: the solution at the chunk's first node (lane 0: interior node 0).
  auto solve_tp = [&](const Phase& p) __attribute__((always_inline)) {
    const double fm = p.fm, bm = p.bm;
    FDCN_PRIO_HI();
    // forward pass 1: zero-carry values of every sub-chain, in place
    double a[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      double w = In(j * M);
#pragma unroll
      for (int i = 1; i < M; ++i) {
        const int k = j * M + i;
        w = fma(k == NPT - 1 ? mlast : fm, w, In(k));
        Wr(k) = w;
      }
      a[j] = w;
    }
    double e = a[0];
#pragma unroll
    for (int j = 1; j < S; ++j) e = fma(j == S - 1 ? mulLF : fmM, e, a[j]);
    // stage 0 unconditional on the split form: the config-3 grids all need
    // it, and a conditional stage costs a copy of e (still live in the last
    // node's register) on the common path
    double b = kSplit ? fma(FW[0], scan_up(e, 1, lane4), e) : e;
#pragma unroll
    for (int j = kSplit ? 1 : 0; j < 2; ++j)
      if (!kSplit || j < nst_f) b = fma(FW[j], scan_up(b, 1 << j, lane4), b);
    if (nst_f > 2) {
#pragma unroll
      for (int j = 2; j < 6; ++j) {
        const double wf = kScanLds ? lds_ld(hide_addr(sw_a), (j - 2) * 128) : FW[j];
        if (j < nst_f) b = fma(wf, scan_up(b, 1 << j, lane4), b);
      }
    }
    // forward carries: into sub-chain 0 from the lane below (0 on lane 0 and
    // dropped on inactive lanes by fm_act), then across the sub-chains
    const double cin = shfl_up1(b, 1);
    CC[0] = fm_act * cin;
    double c = cin;
#pragma unroll
    for (int j = 1; j < S; ++j) {
      c = fma(j == 1 ? fmM_act : fmM, c, a[j - 1]);
      CC[j] = fm * c;
    }
    // backward pass 1 in place; a short lane's last real node starts its
    // sub-chain with a zero carry (bw1l = 0)
    FDCN_PRIO_LO();
#pragma unroll
    for (int j = 0; j < S; ++j) {
      double y = Wr(j * M + M - 1);
#pragma unroll
      for (int i = M - 2; i >= 0; --i) {
        const int k = j * M + i;
        // a sub-chain's first node: its zero-carry forward value is its
        // input (kSplit: not copied into T by the forward pass)
        y = fma(k == NPT - 2 ? bw1l : bm, y, i == 0 ? In(k) : Wr(k));
        Wr(k) = y;
      }
      // the sub-chain's start value with its forward carry, zero backward carry
      a[j] = fma(CC[j], j == S - 1 ? p0l : P0u, y);
    }
    FDCN_PRIO_HI();
    e = a[S - 1];
#pragma unroll
    for (int j = S - 2; j >= 0; --j) e = fma(bmM, e, a[j]);
    double cb = e;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (!kSplit || j < nst_b) cb = fma(GW[j], scan_dn(cb, 1 << j, lane4), cb);
    if (nst_b > 2) {
#pragma unroll
      for (int j = 2; j < 6; ++j) {
        const double wg = kScanLds ? lds_ld(hide_addr(sw_a), (j - 2) * 128 + 64) : GW[j];
        if (j < nst_b) cb = fma(wg, scan_dn(cb, 1 << j, lane4), cb);
      }
    }
    cbv = cb;
    DD[S - 1] = shfl_dn1(cb, 1);  // lane 63 receives 0
#pragma unroll
    for (int j = S - 2; j >= 0; --j) DD[j] = fma(j + 1 == S - 1 ? mulLB : bmM, DD[j + 1], a[j + 1]);
  };
  (void)solve_tp;

  // Two-pass: the Sherman-Morrison correction folded into one sub-chain's
  // carries, C += y0 zc, D += y0 zd, with y0 the solution at interior node 0
  // (cbv on lane 0) and (zc, zd) this lane's table row, already times the
  // correction's coefficient (zero past the table).  y0 comes by v_readlane:
  // a DPP row broadcast straight into the two FMAs (rows within the first 16
  // lanes) measured slower (config 3 4.48 -> 4.52 ms, config 2 11.08 -> 11.87).
  auto sm_fold = [&](double zc, double zd, double& c, double& d) __attribute__((always_inline)) {
    const double y0 = read_lane(cbv, 0);
    c = fma(y0, zc, c);
    d = fma(y0, zd, d);
  };
  (void)sm_fold;

  // broadcast of the solution at interior node 0 (lane 0 of wave 0)
  auto bcast_first = [&](double v0lane) __attribute__((always_inline)) -> double {
    if constexpr (kPair) {  // lane 0 / lane 32: each scenario's own node 0
      return half ? read_lane(v0lane, 32) : read_lane(v0lane, 0);
    } else if constexpr (W == 1) {
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
    // input e0/r, so the table is (L U)^-1 e0 in every form; the IT / kSplit
    // forms correct their r-scaled solution with the same table before
    // scaling it as a whole
    if constexpr (kSplit) {
      vb0 = (t == 0) ? p.inv_r : 0.0;
      vb1 = 0.0;
    } else {
      Wr(0) = (t == 0) ? p.inv_r : 0.0;
    }
    if constexpr (kTP) {
      solve_tp(p);
      double* tph = ztab + tab * kTPh;
      if (lane < M) {  // this phase's P'_i and G_i, i = lane
        double acc = 0.0;
#pragma unroll
        for (int k = M - 1; k >= 0; --k)
          if (k >= lane) acc = fma(p.bm, acc, pow_n<NPT>(p.fm, k));
        tph[lane] = acc;
        tph[M + lane] = pow_n<NPT>(p.bm, M - lane);
      }
      // z at interior node 0 (lane 0, slot 0: no forward carry there)
      const double d0 = (S == 1) ? k2 * fma(CC[0], k1, DD[0]) : DD[0];
      const double z0 = bcast_first(fma(d0, bmM, fma(CC[0], P0u, Out(0))));
      const double smc_p = U(p.kappa / (1.0 + p.kappa * z0));
      if (t <= lz) {
        // z on every sub-chain of this lane is C_z P' + D_z G; on lane 0's
        // first one the input e0/r itself contributes (1/r) P'.  Stored times
        // the correction's coefficient -smc, so a step adds y0 * row to its
        // carries (y0: the solution at interior node 0); row lz is zero
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const double c = CC[j] + ((t == 0 && j == 0) ? p.inv_r : 0.0);
          tph[2 * M + t * 2 * S + j] = t < lz ? -smc_p * c : 0.0;
          tph[2 * M + t * 2 * S + S + j] = t < lz ? -smc_p * DD[j] : 0.0;
        }
      }
      return smc_p;
    }
    solve(p, std::false_type{});
    if (t < lz) {
      // the phantom slot of a short lane holds a pass-through value: store 0
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        ztab[(tab * lz + t) * (NPT + 1) + k] = (k == NPT - 1 && shrt) ? 0.0 : Out(k);
    }
    const double z0 = bcast_first(Out(0));
    return U(p.kappa / (1.0 + p.kappa * z0));
  };

  const bool use_r = A.n_ranna > 0;
  const bool use_c = A.n_ranna < A.n_time;
  int kext = 1;
  double smc_r = 0.0, smc_c = 0.0;
  if (use_c) {
    ph = make_phase<kPair>(0.5, dt, ca, cc, cbc);
    setup_scan(ph);
    smc_c = build_sm(ph, 1);
    kext = max(kext, sm_extent(ph.fm, n_int));
  }
  if (use_r) {
    ph = make_phase<kPair>(1.0, dt, ca, cc, cbc);
    setup_scan(ph);
    smc_r = build_sm(ph, 0);
    kext = max(kext, sm_extent(ph.fm, n_int));
  }
  // nodes covered by the first lz lanes; a larger extent means the table is
  // too small for this scenario: poison the output (loud, never silently off)
  const int covered = (lz >= L_act) ? n_int : lz * NPT - (lz < L_short ? lz : L_short);
  const bool overflow = kext > covered;

  // ---- load state -------------------------------------------------------
  const double* vin = A.v_init + (size_t)scen * n_nodes;
  double V0 = U(vin[0]);
  double VN = U(vin[n_nodes - 1]);
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int node = s_t + 1 + k;
    V[k] = (active && node <= n_int) ? vin[node] : 0.0;
  }
  const double* pin = IT ? A.payoff + (size_t)scen * n_nodes : nullptr;
  if constexpr (kNatural) {
    if (shrt) V[NPT - 1] = 0.0;  // phantom slot: exact zero (the stencil rhs overwrites it)
  }
  if constexpr (IT) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int node = s_t + 1 + k;
      if constexpr (kPhiLds) phit[k * L + t] = (active && node <= n_int) ? pin[node] : 0.0;
      // lambda = 0 at the start (fd_american_equity.py:612): W = V, so
      // Q = (1/theta_0 - 1) V
      QS[k] = A.n_ranna > 0 ? 0.0 : V[k];
    }
  }
  const int ko_lo = Ui(I[FDCN_I_KO_LO]);
  const int ko_hi = Ui(I[FDCN_I_KO_HI]);
  // knock-out masks of this wave (interior nodes j <= ko_lo or j >= ko_hi),
  // computed once: lanes are ordered by node, so the knocked-out lanes of
  // each side are a contiguous run plus at most one partial lane.  A paired
  // wave has one set per scenario (kml/kmh: lanes 0-31, kml2/kmh2: 32-63).
  KoMask kml{0ull, 0ull, 0, -1}, kmh{0ull, 0ull, 0, -1};
  KoMask kml2{0ull, 0ull, 0, -1}, kmh2{0ull, 0ull, 0, -1};
  (void)kml2;
  (void)kmh2;
  if constexpr (!IT) {
    const unsigned long long act =
        __builtin_amdgcn_read_exec() & (unsigned long long)__ballot(active);
    // one scenario's masks: its lanes are bits b0 .. b0+nl-1 of the wave,
    // lane t of the scenario is bit b0 + t - base
    auto masks = [&](int klo, int khi, int base, int b0, int nl, KoMask& ml, KoMask& mh)
        __attribute__((always_inline)) {
      const unsigned long long all = (nl >= 64 ? ~0ull : ((1ull << nl) - 1ull)) << b0;
      if (klo >= 1) {  // interior indices 0 .. klo-1 are out
        int tl, sl;
        if (klo >= n_int) { tl = L_act; sl = 0; }
        else lane_slot<NPT>(klo - 1, L_short, tl, sl);
        // lanes < tl fully out; lane tl out for slots <= sl
        const int rl = tl - base;
        ml.full = rl <= 0 ? 0ull : (rl >= nl ? all : (((1ull << rl) - 1ull) << b0));
        ml.full &= act;
        if (klo < n_int && rl >= 0 && rl < nl) { ml.part = act & (1ull << (b0 + rl)); ml.k0 = 0; ml.k1 = sl; }
      }
      if (khi <= n_int) {  // interior indices khi-1 .. n_int-1 are out
        int th, sh;
        if (khi <= 1) { th = 0; sh = 0; }
        else lane_slot<NPT>(khi - 1, L_short, th, sh);
        // lane th out for slots >= sh; lanes > th fully out
        const int rh = th - base;
        mh.full = rh >= nl - 1 ? 0ull : (rh < 0 ? all : (all & ~(((2ull << rh) - 1ull) << b0)));
        mh.full &= act;
        if (rh >= 0 && rh < nl) { mh.part = act & (1ull << (b0 + rh)); mh.k0 = sh; mh.k1 = NPT - 1; }
      }
    };
    if constexpr (kPair) {
      masks(__builtin_amdgcn_readlane(ko_lo, 0), __builtin_amdgcn_readlane(ko_hi, 0), 0, 0, 32,
            kml, kmh);
      masks(__builtin_amdgcn_readlane(ko_lo, 32), __builtin_amdgcn_readlane(ko_hi, 32), 0, 32, 32,
            kml2, kmh2);
    } else {
      masks(ko_lo, ko_hi, wave * 64, 0, 64, kml, kmh);
    }
  }
  const unsigned long long shrt_ballot = kSplit ? (unsigned long long)__ballot(shrt) : 0ull;
  (void)shrt_ballot;
  unsigned long long kom_addr = 0;  // this wave's mask row (KoLoad variants)
  // kKoRes: the resident-mask projection (fdcn_ko_res.h), its run masks and
  // group codes after the mask row (kKoResRow)
  constexpr bool kKoRes = kRec && !(ZG & 6);
  unsigned long long kom_addr2 = 0, kom_addr12 = 0;  // kPair: second scenario's / both
  if constexpr (KoLoad<IT, W, NPT, ZG>::value) {
    unsigned long long* kom = reinterpret_cast<unsigned long long*>(kom_row);
    // kRec / kSplit keep the phantom slot of short lanes at zero: never knock it out
    const unsigned long long shrt_lanes = (kRec || kSplit) ? (unsigned long long)__ballot(shrt) : 0ull;
    auto slot_mask = [&](const KoMask& ml, const KoMask& mh, int k) {
      unsigned long long mk = ml.full | ((k >= ml.k0 && k <= ml.k1) ? ml.part : 0ull) | mh.full |
                              ((k >= mh.k0 && k <= mh.k1) ? mh.part : 0ull);
      return k == NPT - 1 ? (mk & ~shrt_lanes) : mk;
    };
    if constexpr (kPair) {
      // rows: the first scenario's [0, NPT) its own masks, [32, 32 + NPT) both
      // scenarios'; the second scenario's [0, NPT) its own (each lane writes
      // into its own scenario's row)
      if (hl < NPT && valid) {
        const int k = hl;
        kom[k] = half ? slot_mask(kml2, kmh2, k) : slot_mask(kml, kmh, k);
        if (!half) kom[32 + k] = slot_mask(kml, kmh, k) | slot_mask(kml2, kmh2, k);
      }
    } else if (lane < NPT) {
      kom[lane] = slot_mask(kml, kmh, lane);
    }
    // the loop reads the row back with s_load from inline asm, which the
    // compiler's wait-count tracking does not see: drain the stores here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long ka = (unsigned long long)kom;
    if constexpr (kPair) {
      const unsigned lo0 = __builtin_amdgcn_readlane((unsigned)ka, 0);
      const unsigned hi0 = __builtin_amdgcn_readlane((unsigned)(ka >> 32), 0);
      const unsigned lo1 = __builtin_amdgcn_readlane((unsigned)ka, 32);
      const unsigned hi1 = __builtin_amdgcn_readlane((unsigned)(ka >> 32), 32);
      kom_addr = ((unsigned long long)hi0 << 32) | lo0;
      kom_addr2 = ((unsigned long long)hi1 << 32) | lo1;
      kom_addr12 = kom_addr + 32 * sizeof(unsigned long long);
    } else {
      kom_addr = ka;
    }
    if constexpr (kKoRes) {
      // the run masks and per-group codes of the resident projection
      // (ko_groups): change points are the slots k in [1, NPT-2] whose mask
      // differs from slot k-1's
      const unsigned long long mk = lane < NPT ? slot_mask(kml, kmh, lane) : 0ull;
      const unsigned long long mkp =
          ((unsigned long long)(unsigned)__shfl_up((int)(mk >> 32), 1, 64) << 32) |
          (unsigned)__shfl_up((int)(unsigned)mk, 1, 64);
      const unsigned long long chg =
          (unsigned long long)__ballot(lane >= 1 && lane < NPT - 1 && mk != mkp);
      auto rl64 = [](unsigned long long x, int l) {
        return ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
               (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
      };
      const int nchg = __builtin_popcountll(chg);
      const int c1 = nchg >= 1 ? uni_i(__builtin_ctzll(chg)) : 0;
      const int c2 = nchg >= 2 ? uni_i(__builtin_ctzll(chg & (chg - 1))) : 0;
      const unsigned long long q0 = rl64(mk, 0);
      const unsigned long long q1 = nchg >= 1 ? rl64(mk, c1) : q0;
      const unsigned long long q2 = nchg >= 2 ? rl64(mk, c2) : q1;
      const unsigned long long qd = rl64(mk, NPT - 1);
      unsigned codes0 = 0u, codes1 = 0u;
#pragma unroll
      for (int g = 0; g < NPT / 8; ++g) {
        const int lo = 8 * g, gsz = (g + 1 == NPT / 8) ? 7 : 8;
        const unsigned long long bits = (chg >> lo) & ((1ull << gsz) - 1ull);
        unsigned code;
        if (nchg > 2) {
          code = 63u;
        } else if (bits == 0ull) {
          code = 0u;
        } else if ((bits & (bits - 1ull)) == 0ull) {
          code = 1u + (unsigned)__builtin_ctzll(bits);
        } else {
          const int o1 = __builtin_ctzll(bits), o2 = __builtin_ctzll(bits & (bits - 1ull));
          code = (unsigned)(gsz + 1 + o1 * (2 * gsz - o1 - 1) / 2 + (o2 - o1 - 1));
        }
        if (g < 5) codes0 |= code << (6 * g);
        else codes1 |= code << (6 * (g - 5));
      }
      // after the 64 slot masks (kKoResRow): vector stores by lane 0, drained
      // with the row's below
      if (lane == 0) {
        kom[2 * kKoRow + 0] = q0;
        kom[2 * kKoRow + 1] = q1;
        kom[2 * kKoRow + 2] = q2;
        kom[2 * kKoRow + 3] = qd;
        kom[2 * kKoRow + 4] = ((unsigned long long)codes1 << 32) | codes0;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  (void)kom_addr2;
  (void)kom_addr12;
  (void)kom_addr;
  // every lane that holds a Sherman-Morrison table row is fully inside the
  // lower knock-out region (sm_skip below)
  bool sm_covered = false;
  if constexpr (kRec) {
    const unsigned long long lzm = lz >= 64 ? ~0ull : ((1ull << lz) - 1ull);
    sm_covered = (kml.full & lzm) == lzm;
  }
  (void)sm_covered;
  // monitoring entries: one run per scenario of the wave (mon2: a paired
  // wave's second scenario; an odd batch's missing one has none)
  MonRun<kWavesPerEu<IT, W, NPT, ZG> == 1> mon, mon2;
  mon.init(A.mon_step, A.mon_rebate, 0, 0);
  mon2.init(A.mon_step, A.mon_rebate, 0, 0);
  if constexpr (!IT) {
    const int ms = Ui(I[FDCN_I_MON_START]), mc = Ui(I[FDCN_I_MON_COUNT]);
    if constexpr (kPair) {
      mon.init(A.mon_step, A.mon_rebate, __builtin_amdgcn_readlane(ms, 0),
               __builtin_amdgcn_readlane(mc, 0));
      if (scen0 + 1 < A.B)
        mon2.init(A.mon_step, A.mon_rebate, __builtin_amdgcn_readlane(ms, 32),
                  __builtin_amdgcn_readlane(mc, 32));
    } else {
      mon.init(A.mon_step, A.mon_rebate, ms, mc);
    }
  }

  if constexpr (W > 1 && !kNatural) {
    if (lane == 0) xch[Xch<W>::kFirst + wave] = V[0];
    if (lane == 63) xch[Xch<W>::kLast + wave] = shrt ? V[NPT - 2] : V[NPT - 1];
  }
  // phase for step 0 (ph currently holds the theta the last table was built for)
  double smc;
  // -smc on the lanes that hold table rows, 0 elsewhere: g = smc_l y0 needs
  // no lane select
  const double sm_row = (t < lz) ? -1.0 : 0.0;
  double smc_l;
  // this lane's row of the correction tables (lanes >= lz read row lz-1)
  const int zoff_r = (t < lz ? t : lz - 1) * (NPT + 1);
  const int zoff_c = zoff_r + lz * (NPT + 1);
  // the current phase's row offset, kept across steps (re-deriving it from
  // the lane's row index took three VALU per step)
  int zoff_cur = zoff_c;
  // its LDS byte address when the table is in LDS (hide_addr)
  constexpr bool kZLds = !(ZG & 1);
  unsigned z_a = kZLds ? lds_addr(ztab + zoff_c) : 0u;
  (void)z_a;
  // kTP: LDS byte addresses of this phase's tables, of this lane's row of
  // the Sherman-Morrison coefficients and of its payoff column (hide_addr)
  auto tp_tab_addr = [&](int tb_) { return kTP ? lds_addr(ztab + tb_ * kTPh) : 0u; };
  auto tp_row_addr = [&](int tb_) {
    return kTP ? lds_addr(ztab + tb_ * kTPh + 2 * M + (t < lz ? t : lz) * 2 * S) : 0u;
  };
  unsigned tp_ta = tp_tab_addr(1), tp_za = tp_row_addr(1);
  // kTPS: this phase's P' and G as DPP broadcast sources (fmac_bcast), lane
  // l holding entry l mod 16 (more than 16 slots: register r holds entries
  // 16 r .. 16 r + 15), times the phase's update scale s
  double tabP[kTabRegs], tabG[kTabRegs];
#pragma unroll
  for (int r = 0; r < kTabRegs; ++r) tabP[r] = tabG[r] = 0.0;
  auto tp_load_bcast = [&](int tb_, double sc) __attribute__((always_inline)) {
    if constexpr (kTPS) {
      const double* tb = ztab + tb_ * kTPh;
#pragma unroll
      for (int r = 0; r < kTabRegs; ++r) {
        const int e = 16 * r + (lane & 15);
        const int sl = e < M ? e : 0;
        tabP[r] = sc * tb[sl];
        tabG[r] = sc * tb[M + sl];
      }
    }
  };
  unsigned tp_pa = (kTP && kPhiLds) ? lds_addr(phit + t) : 0u;
  // kTPS tables: times the update scale s, or unscaled for kTPST
  auto tab_scale = [&]() __attribute__((always_inline)) { return kTPST ? 1.0 : ph.s; };
  (void)tp_ta;
  (void)tp_za;
  (void)tp_pa;
  if (use_r) {
    smc = smc_r;
    zoff_cur = zoff_r;
    if constexpr (kZLds) z_a = lds_addr(ztab + zoff_r);
    tp_ta = tp_tab_addr(0);
    tp_za = tp_row_addr(0);
    tp_load_bcast(0, tab_scale());
  } else {
    ph = make_phase<kPair>(0.5, dt, ca, cc, cbc);
    setup_scan(ph);
    smc = smc_c;
    tp_load_bcast(1, tab_scale());
  }
  smc_l = sm_row * smc;
  s_l = shrt ? 0.0 : ph.s;

  // The register-capped config-3 variant evaluates each chunk's entries when
  // it starts; the others evaluate the next chunk's at the start of this one
  // (their exp latency then overlaps a whole chunk of steps).  (Round 4, with
  // a table: a prefetched next block spilled to scratch in the capped
  // variant, +170 MB of HBM traffic per launch.)
  constexpr bool kBndPrefetch = !kGen && kWavesPerEu<IT, W, NPT, ZG> == 1;
  double2 bnd_cur = make_double2(0.0, 0.0), raw_cur = make_double2(0.0, 0.0);
  double2 bnd_nxt = kBndPrefetch ? tab_load(hl) : make_double2(0.0, 0.0);  // steps 0..kStride-1
  (void)bnd_nxt;
  (void)raw_cur;
  int ko_prev = 0;  // kSplit: bit 0 / 1 -- the last step knocked out node 0 / the last node
  (void)ko_prev;
  double halo_l = 0.0, halo_r = 0.0;
  if constexpr (W == 1 && !kNatural) {
    halo_l = shfl_up1(shrt ? V[NPT - 2] : V[NPT - 1], 1);
    halo_r = shfl_dn1(V[0], 1);
  }
  // Steps in blocks of kStride: a block's boundary terms (one step per lane)
  // stay in bnd_cur for the whole block while the next block's load is in
  // flight.  With the refill inside a flat step loop the compiler rotated the
  // two buffers through copies on every step (8 v_mov_b64 per step).
  for (int m0 = 0; m0 < A.n_time; m0 += kStride) {
    if constexpr (kGen) {
      bnd_cur = gen(m0, raw_cur);
    } else if constexpr (kBndPrefetch) {
      bnd_cur = bnd_nxt;
      if (m0 + kStride < A.n_pad) bnd_nxt = tab_load(m0 + kStride + hl);  // prefetch the block after
    } else {
      bnd_cur = tab_load(m0 + hl);
    }
    if constexpr (kBndLds) {
      // into LDS: each step then reads its terms as one broadcast (an LDS
      // instruction) instead of four v_readlane (VALU); the wave's LDS
      // operations complete in order, so no wait is needed before the reads
      bblk[lane] = bnd_cur;
      asm volatile("" ::: "memory");
    }
    // kRec: each step's broadcast is read one step ahead (bt_pf), so the
    // step does not open on an LDS wait (its first instructions form the
    // Dirichlet rhs terms from it)
    constexpr bool kBndPf = kBndLds && kRec;
    double2 bt_pf = make_double2(0.0, 0.0);
    if constexpr (kBndPf) bt_pf = bblk[0];
    (void)bt_pf;
    const int m_end = min(m0 + kStride, A.n_time);
  for (int m = m0; m < m_end; ++m) {
#ifdef FDCN_STAMPS
    stamp_m = m;
    if constexpr (kRec) {
      if (scen < kStampScen && m == kStampStep0 && lane == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        A.vsave[(size_t)scen * 64 * NPT + 15] = (double)hw;
        A.vsave[(size_t)scen * 64 * NPT + 14] = (double)xcc;
      }
    }
#endif
    FDCN_STAMP(0);
    if (m == A.n_ranna && use_r) {  // Rannacher -> Crank-Nicolson
      if constexpr (kPair) {
        // reloaded rather than kept live through the march (VGPRs, per lane)
        const double* Pr = P;
        asm volatile("" : "+v"(Pr));
        ph = make_phase<kPair>(0.5, Pr[FDCN_P_DT], Pr[FDCN_P_A], Pr[FDCN_P_C], Pr[FDCN_P_BC]);
      } else {
        ph = make_phase<kPair>(0.5, dt, ca, cc, cbc);
      }
      setup_scan(ph);
      smc = smc_c;
      smc_l = sm_row * smc;
      s_l = shrt ? 0.0 : ph.s;
      zoff_cur = zoff_c;
      if constexpr (kZLds) z_a = lds_addr(ztab + zoff_c);
      tp_ta = tp_tab_addr(1);
      tp_za = tp_row_addr(1);
      tp_load_bcast(1, tab_scale());
    }
    // kSplit: the tabulated rhs terms; kPair: each scenario's from its own lanes
    double lo_new, hi_new;
    if constexpr (kBndLds) {
      double2 bt;
      if constexpr (kBndPf) {
        bt = bt_pf;
        bt_pf = bblk[(m + 1 - m0) & 63];  // the block's last step reads a stale entry, unused
      } else {
        bt = bblk[m - m0];
      }
      lo_new = bt.x;
      hi_new = bt.y;
    } else {  // kPair: each scenario's from its own lanes
      lo_new = kPair ? (half ? read_lane(bnd_cur.x, 32 + (m & 31)) : read_lane(bnd_cur.x, m & 31))
                     : read_lane(bnd_cur.x, m & 63);
      hi_new = kPair ? (half ? read_lane(bnd_cur.y, 32 + (m & 31)) : read_lane(bnd_cur.y, m & 31))
                     : read_lane(bnd_cur.y, m & 63);
    }

    // ---- 1. rhs ------------------------------------------------------------
    if constexpr (IT) {
      // IT form: the reference step  A x = B V + dt lambda  (+ Dirichlet
      // terms; fd_american_equity.py:681-698) with B = (I - (1-theta) A) /
      // theta and dt lambda = V - W (W: last pre-projection value) reads
      //   A (x + c2 V) = V/theta + V - W = V + Q,   c2 = (1-theta)/theta,
      // plus (-A_L)(lo_new + c2 lo_old) at node 0 and (-A_U)(hi_new + c2
      // hi_old) at the last node.  The rhs is pointwise: no stencil and no
      // neighbour exchange.  Unscaled, so the solve returns r (x + c2 V).
      // blo / bhi come tabulated from the prologue (lo_new / hi_new hold them)
#pragma unroll
      for (int k = 0; k < NPT; ++k) V[k] += QS[k];
      V[0] = fma(e_first, lo_new, V[0]);            // + blo on the first lane
      V[NPT - 1] = fma(e_last, hi_new, V[NPT - 1]);  // + bhi on the last (never short)
      if (shrt) V[NPT - 1] = 0.0;                   // the phantom slot's rhs
    } else if constexpr (kSplit) {
      // theta form of the reference step A x = B V (+ Dirichlet terms,
      // discrete_barrier_fdm_pricer.py:531-537) with B = (I - (1-theta) A) /
      // theta:  A (theta x + (1-theta) V) = V + theta (-A_L)(lo_new + c2
      // lo_old) e_0 + theta (-A_U)(hi_new + c2 hi_old) e_n.  The rhs is V
      // itself except at the two end nodes (vb0 / vb1); the solve reads V and
      // writes T, and x = (r u)/(theta r) - c2 V afterwards.
      double blo = lo_new, bhi = hi_new;
      if constexpr (!kTabSplit) {  // raw values: the terms of this step
        blo = ph.th * (ph.pl * fma(ph.c2, V0, lo_new));
        bhi = ph.th * (ph.pu * fma(ph.c2, VN, hi_new));
      } else if (ko_prev) {  // after a knock-out step: terms from the rebate (uniform branch)
        const int kb = kPair ? ((ko_prev >> (2 * half)) & 3) : ko_prev;
        const double2 raw = raw_load(m);  // the step's raw Dirichlet values
        const double rlo = U(raw.x), rhi = U(raw.y);
        // (uniform: kept in SGPRs like the tabulated terms, so the merge
        // after this branch needs no VGPR copies on the common path)
        if (kb & 1) blo = U(ph.th * (ph.pl * fma(ph.c2, V0, rlo)));
        if (kb & 2) bhi = U(ph.th * (ph.pu * fma(ph.c2, VN, rhi)));
        ko_prev = 0;
      }
      vb0 = fma(e_first, blo, V[0]);
      // the phantom slot of a short lane is an exact zero and e_last is 0
      // there (the update and the knock-out masks keep it so)
      vb1 = fma(e_last, bhi, V[NPT - 1]);
    } else if constexpr (kRec) {
      // the kSplit rhs, in place (the phantom slot is kept at zero by the
      // update and by the knock-out masks)
      if (m < A.n_ranna) {
        // Rannacher step: the update below returns s u - V_old, the step
        // needs s u (c2 = 0); keep V_old for the add-back (lane-major, so
        // every slot is an immediate offset from one address)
        double* sv = A.vsave + ((size_t)scen * 64 + lane) * NPT;
#pragma unroll
        for (int k = 0; k < NPT; ++k) sv[k] = V[k];
      }
      rec_lo = ph.th * (ph.pl * fma(ph.c2, V0, lo_new));
      rec_hi = ph.th * (ph.pu * fma(ph.c2, VN, hi_new));
      V[0] = fma(e_first, rec_lo, V[0]);
      V[NPT - 1] = fma(e_last, rec_hi, V[NPT - 1]);
    } else {
    if constexpr (W > 1) __syncthreads();  // halos of the previous step
    // neighbours' edge values: shuffled at the end of the previous step (W=1)
    // so their latency overlaps the tail of that step
    double left = halo_l, right = halo_r;
    if constexpr (W > 1) {
      left = shfl_up1(shrt ? V[NPT - 2] : V[NPT - 1], 1);
      right = shfl_dn1(V[0], 1);
      if (lane == 0 && wave > 0) left = xch[Xch<W>::kLast + wave - 1];
      if (lane == 63 && wave < W - 1) right = xch[Xch<W>::kFirst + wave + 1];
    }
    if (t == 0) left = V0;
    if (t == L_act - 1) right = VN;
    if (!active) { left = 0.0; right = 0.0; }
    if (shrt) V[NPT - 1] = right;
    {
      // r_k = B_L V_{k-1} + B_C V_k + B_U V_{k+1} (+ mu_k), all over r: the
      // reference's stencil (…pricer.py:531-534, …equity.py:686-691) with
      // FMAs, evaluated left to right.  In place and SHIFTED: r_k overwrites
      // V_{k-1} (its last reader), r_0 goes to X, so no old value needs
      // saving.  asm keeps the compiler from evaluating every r_k before the
      // first store (which would keep two copies of the vector live).
      // Software-pipelined over nodes: step s issues op4 of node s-3 (IT
      // only), op3 of node s-2, op2 of node s-1 and op1 of node s, so each
      // node's dependent chain is spread 3-4 instructions apart and node
      // j+1's first write to V[j] comes after the last reads of the old V[j]
      // (op2 of node j, op3 of node j-1).  One asm statement per
      // instruction keeps that order; the "+v" ties keep it in place.
      //   op1: acc_j  = B_L * V_{j-1}     (acc_0 = X, acc_j = V[j-1])
      //   op2: acc_j += B_C * V_j
      //   op3: acc_j += B_U * V_{j+1}     (V_NPT = right)
      constexpr int kOps = 3;
#pragma unroll
      for (int st = 0; st < NPT + kOps - 1; ++st) {
#pragma unroll
        for (int op = kOps; op >= 1; --op) {
          const int j = st - (op - 1);
          if (j < 0 || j >= NPT) continue;
          double& acc = (j == 0) ? X : V[j - 1];
          if (j == 0) {
            // node 0 takes the left neighbour last: r_0 = (B_C V_0 + B_U V_1)
            // + B_L left, so the halo shuffle has the whole RHS to land
            if (op == 1)
              asm volatile("v_mul_f64 %0, %1, %2" : "=v"(X) : "s"(ph.bc), "v"(V[0]));
            else if (op == 2)
              asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(X) : "s"(ph.bu), "v"(V[1]));
            continue;
          }
          if (op == 1) {
            asm volatile("v_mul_f64 %0, %1, %0" : "+v"(acc) : "s"(ph.bl));
          } else if (op == 2) {
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc) : "s"(ph.bc), "v"(V[j]));
          } else {
            const double nxt = (j < NPT - 1) ? V[j + 1] : right;
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc) : "s"(ph.bu), "v"(nxt));
          }
        }
      }
    }
    asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(X) : "s"(ph.bl), "v"(left));
    if (t == 0) X = fma(ph.fm, lo_new, X);                                  // node 0
    if (t == L_act - 1) V[NPT - 2] = fma(ph.bm, hi_new, V[NPT - 2]);        // node NPT-1
    if (shrt) V[NPT - 2] = 0.0;  // the phantom node's rhs
    }  // CN rhs

    if constexpr (kTPS) {
      // ---- 2. two-pass solve into T (zero-carry passes); Sherman-Morrison
      // folded into the carries ------------------------------------------
      solve_tp(ph);
      tp_za = hide_addr(tp_za);
      sm_fold(lds_ld(tp_za, 0), lds_ld(tp_za, 1), CC[0], DD[0]);
      DD[0] = k2 * fma(CC[0], k1, DD[0]);  // short lanes (see setup_scan)
      // ---- 3. x = s (T + C P'_i + D G_i) - c2 V: c2 = 1 for theta = 1/2;
      // the Rannacher steps (c2 = 0) drop V first.  Up to 16 nodes per lane
      // (kTPST) the tables go into T first; longer chunks (2-3 table
      // registers) keep tables pre-scaled by s, added to V after the update
      // (A/B: kTPST lost 1.3 % at 40 nodes per lane, won 0.5-3.6 % at 8-16)
      if constexpr (kTPST) {
        // the homogeneous part into T (unscaled tables), then x = s T - c2 V
        // with the phantom slot's scale s_l = 0 on short lanes: its V stays
        // an exact zero without a reset
#pragma unroll
        for (int k = 0; k < NPT; ++k) fmac_bcast(T[k], tabP[k / 16], CC[0], k % 16);
#pragma unroll
        for (int k = 0; k < NPT; ++k) fmac_bcast(T[k], tabG[k / 16], DD[0], k % 16);
        if (m < A.n_ranna) {
#pragma unroll
          for (int k = 0; k < NPT; ++k) V[k] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < NPT - 1; ++k)
          asm volatile("v_fma_f64 %0, %1, %2, -%0" : "+v"(V[k]) : "s"(ph.s), "v"(T[k]));
        asm volatile("v_fma_f64 %0, %1, %2, -%0" : "+v"(V[NPT - 1]) : "v"(s_l), "v"(T[NPT - 1]));
      } else {
      if (m < A.n_ranna) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) V[k] = 0.0;
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        asm volatile("v_fma_f64 %0, %1, %2, -%0" : "+v"(V[k]) : "s"(ph.s), "v"(T[k]));
#pragma unroll
      for (int k = 0; k < NPT; ++k) fmac_bcast(V[k], tabP[k / 16], CC[0], k % 16);
#pragma unroll
      for (int k = 0; k < NPT; ++k) fmac_bcast(V[k], tabG[k / 16], DD[0], k % 16);
      if (shrt) V[NPT - 1] = 0.0;  // the phantom slot (its rhs must stay zero)
      }
    } else if constexpr (kTP) {
      // ---- 2. two-pass solve; Sherman-Morrison folded into the carries ----
      solve_tp(ph);
      tp_ta = hide_addr(tp_ta);  // this phase's tables
      tp_za = hide_addr(tp_za);
#pragma unroll
      for (int j = 0; j < S; ++j) sm_fold(lds_ld(tp_za, j), lds_ld(tp_za, S + j), CC[j], DD[j]);
      DD[S - 1] = k2 * fma(CC[S - 1], k1, DD[S - 1]);  // short lanes (see setup_scan)
      // ---- 3. x = Wr + C P'_i + D G_i and the step's update ---------------
      // nodes in (slot i, sub-chain j) order, four at a time: a slot's two
      // table values (LDS broadcasts) serve all S sub-chains
      __builtin_amdgcn_s_setprio(1);
      const double cq = (m + 1 < A.n_ranna) ? 1.0 : 2.0;  // 1/theta of the next step
      tp_pa = hide_addr(tp_pa);
      // node of the u-th entry of group q: slot (q+u)/S of sub-chain (q+u)%S
#define FDCN_TP_K(u) ((((q) + (u)) % S) * M + ((q) + (u)) / S)
      if constexpr (NPT % 4 != 0) {
        // two-node chunks (the smallest grids): node by node, one sub-chain
        static_assert(S == 1, "chunks of fewer than 4 nodes run one sub-chain");
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          V[k] = fma(DD[0], lds_ld(tp_ta, M + k), fma(CC[0], lds_ld(tp_ta, k), V[k]));
          const double w = fma(ph.inv_r, V[k], -QS[k]);
          V[k] = fmax(lds_ld(tp_pa, k * L), w);
          QS[k] = fma(cq, V[k], -w);
        }
      } else {
      // the tables one group ahead of their use (LDS latency under the
      // previous group's arithmetic)
      double tpn[4], tgn[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        tpn[u] = lds_ld(tp_ta, u / S);
        tgn[u] = lds_ld(tp_ta, M + u / S);
      }
#pragma unroll
      for (int q = 0; q < NPT; q += 4) {
        double tpc[4], tgc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          tpc[u] = tpn[u];
          tgc[u] = tgn[u];
        }
        if (q + 4 < NPT) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            tpn[u] = lds_ld(tp_ta, (q + 4 + u) / S);
            tgn[u] = lds_ld(tp_ta, M + (q + 4 + u) / S);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = (q + u) % S;
          V[FDCN_TP_K(u)] = fma(DD[j], tgc[u], fma(CC[j], tpc[u], V[FDCN_TP_K(u)]));
        }
        // the Ikonen-Toivanen update (W, V', Q'; see the re-run form below)
        double pk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pk[u] = lds_ld(tp_pa, FDCN_TP_K(u) * L);
        asm volatile(
            "v_fma_f64 %4, %12, %0, -%4\n\t"
            "v_fma_f64 %5, %12, %1, -%5\n\t"
            "v_fma_f64 %6, %12, %2, -%6\n\t"
            "v_fma_f64 %7, %12, %3, -%7\n\t"
            "v_max_f64 %0, %8, %4\n\t"
            "v_max_f64 %1, %9, %5\n\t"
            "v_max_f64 %2, %10, %6\n\t"
            "v_max_f64 %3, %11, %7\n\t"
            "v_fma_f64 %4, %13, %0, -%4\n\t"
            "v_fma_f64 %5, %13, %1, -%5\n\t"
            "v_fma_f64 %6, %13, %2, -%6\n\t"
            "v_fma_f64 %7, %13, %3, -%7"
            : "+v"(V[FDCN_TP_K(0)]), "+v"(V[FDCN_TP_K(1)]), "+v"(V[FDCN_TP_K(2)]),
              "+v"(V[FDCN_TP_K(3)]), "+v"(QS[FDCN_TP_K(0)]), "+v"(QS[FDCN_TP_K(1)]),
              "+v"(QS[FDCN_TP_K(2)]), "+v"(QS[FDCN_TP_K(3)])
            : "v"(pk[0]), "v"(pk[1]), "v"(pk[2]), "v"(pk[3]), "s"(ph.inv_r), "s"(cq));
      }
      }  // NPT % 4 == 0
#undef FDCN_TP_K
    } else {
    // ---- 2. tridiagonal solve ---------------------------------------------
    if constexpr (kRec) {
      // one fused solve for both phases (a second, plain solve for the
      // Rannacher steps doubled the live ranges: 373 registers, one wave per
      // SIMD, 47.8 ms per config-5 launch instead of 26)
      solve_rec(ph);
      static_assert(!kRec || NPT % 8 == 0, "recovery variants add back 8 slots per group");
      if (m < A.n_ranna) {
        // x = (s u - V_old) + V_old, eight slots per group so the loads do
        // not all hoist into registers
        const double* sv = A.vsave + ((size_t)scen * 64 + lane) * NPT;
#pragma unroll
        for (int k = 0; k < NPT; k += 8) {
          double o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = sv[k + i];
#pragma unroll
          for (int i = 0; i < 8; ++i) V[k + i] += o[i];
          asm volatile("" ::: "memory");
        }
      }
    } else {
      solve(ph, std::false_type{});
    }
    // Sherman-Morrison: x = y - (k y0 / (1 + k z0)) z over the first lz lanes
    // (lanes >= lz use g = 0 and read row lz-1, one broadcast address), fused
    // with the Ikonen-Toivanen update for IT.  Both tables are read from LDS
    // one 4-node group ahead of their use, so the LDS latency overlaps the
    // previous group's arithmetic.
    static_assert(NPT % 4 == 0, "variants need NPT divisible by 4");
    const bool do_sm = (W == 1) || (lz > 64) || (wave == 0);
    // kRec: the correction only changes nodes of lanes < lz; on a knock-out
    // step whose lower side removes all of them the projection overwrites it
    // with the rebate, so it is skipped (config 5 knocks out on every step)
    const bool sm_skip = kRec && sm_covered && (m + 1 == mon.next);
    double g = 0.0;
    int zoff = 0;
    if (do_sm && !sm_skip) {
      double y0;
      if constexpr (kPair) {
        y0 = bcast_first(Out(0));
      } else if constexpr (kRec) {
        y0 = read_lane(y0c, 0);
      } else if constexpr (W == 1) {
        y0 = read_lane(Out(0), 0);
      } else {
        y0 = (lz > 64) ? bcast_first(Out(0)) : read_lane(Out(0), 0);
      }
      g = smc_l * y0;
      // lane-major rows, stride NPT+1: bank-spread, immediate offsets
      if constexpr (kZLds) z_a = hide_addr(z_a);
      else zoff = opaque(zoff_cur);
    }
    if constexpr (kSplit) {
      // x = s (T + g z) - c2 V: c2 = 1 for theta = 1/2; the Rannacher steps
      // (c2 = 0) drop V instead of taking another multiply per node
      if (m < A.n_ranna) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) V[k] = 0.0;
      }
    }
    // ---- 3. early exercise / boundaries / knock-out ------------------------
    // IT and kRec: the update / knock-out and the next RHS at priority 1,
    // between pass 1 + scan (3) and pass 2 (0): config 2 11.99 -> 11.74 ms,
    // config 5 19.73 -> 18.41 ms (3 instead of 1: 18.65); kSplit lost 2 %
    // with it (tools/gpu_ab.sh)
    if constexpr (IT || kRec) __builtin_amdgcn_s_setprio(1);
    const double cq = (m + 1 < A.n_ranna) ? 1.0 : 2.0;  // 1/theta of the next step (IT)
    (void)cq;
    if (!sm_skip) {
      const int poff = opaque(kPhiLds ? t : s_t + 1);
      auto phi_at = [&](int k) -> double {
        const int node = s_t + 1 + k;
        return kPhiLds ? phit[poff + k * L]
                       : ((active && node <= n_int) ? pin[poff + k] : 0.0);
      };
      const double sg = kRec ? ph.s * g : 0.0;
      (void)sg;
      double zn[4], pn[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        zn[i] = do_sm ? (kZLds ? lds_ld(z_a, i) : ztab[zoff + i]) : 0.0;
        if constexpr (IT) pn[i] = phi_at(i);
      }
#pragma unroll
      for (int k = 0; k < NPT; k += 4) {
        double zk[4], pk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          zk[i] = zn[i];
          pk[i] = pn[i];
        }
        if (k + 4 < NPT) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            zn[i] = do_sm ? (kZLds ? lds_ld(z_a, k + 4 + i) : ztab[zoff + k + 4 + i]) : 0.0;
            if constexpr (IT) pn[i] = phi_at(k + 4 + i);
          }
        }
        if constexpr (kSplit) {
          // T += g z; V = s T - V (the last slot with s_l: 0 on short lanes,
          // so the phantom stays zero); kPair: s is a per-lane value
          if (k + 4 < NPT)
            split_update<kPair, false>(V[k], V[k + 1], V[k + 2], V[k + 3], T[k], T[k + 1],
                                       T[k + 2], T[k + 3], g, zk, ph.s, s_l);
          else
            split_update<kPair, true>(V[k], V[k + 1], V[k + 2], V[k + 3], T[k], T[k + 1],
                                      T[k + 2], T[k + 3], g, zk, ph.s, s_l);
        } else if constexpr (kRec) {
          // V holds s u already (both phases): x = s u + (s g) z
#pragma unroll
          for (int i = 0; i < 4; ++i) V[k + i] = fma(sg, zk[i], V[k + i]);
        } else if constexpr (!IT) {
#pragma unroll
          for (int i = 0; i < 4; ++i) V[k + i] = fma(g, zk[i], V[k + i]);
        } else {
          // r x~ = y~ + g z (Sherman-Morrison on the r-scaled solution,
          // x~ = x + c2 V), then the Ikonen-Toivanen update
          // (fd_american_equity.py:704-717):
          //   W  = x - dt lambda = x~ - Q
          //   V' = max(phi, W)
          //   Q' = V'/theta' - W               (theta' of the next step: cq)
          // with dt lambda' = V' - W = max(phi - W, 0), the reference's
          // multiplier update max(lambda + (phi - x)/dt, 0) in exact
          // arithmetic.  In place (W lives in Q's registers), the four
          // nodes' dependent chains interleaved.
          asm volatile(
              "v_fma_f64 %0, %12, %13, %0\n\t"
              "v_fma_f64 %1, %12, %14, %1\n\t"
              "v_fma_f64 %2, %12, %15, %2\n\t"
              "v_fma_f64 %3, %12, %16, %3\n\t"
              "v_fma_f64 %4, %17, %0, -%4\n\t"
              "v_fma_f64 %5, %17, %1, -%5\n\t"
              "v_fma_f64 %6, %17, %2, -%6\n\t"
              "v_fma_f64 %7, %17, %3, -%7\n\t"
              "v_max_f64 %0, %8, %4\n\t"
              "v_max_f64 %1, %9, %5\n\t"
              "v_max_f64 %2, %10, %6\n\t"
              "v_max_f64 %3, %11, %7\n\t"
              "v_fma_f64 %4, %18, %0, -%4\n\t"
              "v_fma_f64 %5, %18, %1, -%5\n\t"
              "v_fma_f64 %6, %18, %2, -%6\n\t"
              "v_fma_f64 %7, %18, %3, -%7"
              : "+v"(V[k]), "+v"(V[k + 1]), "+v"(V[k + 2]), "+v"(V[k + 3]), "+v"(QS[k]),
                "+v"(QS[k + 1]), "+v"(QS[k + 2]), "+v"(QS[k + 3])
              : "v"(pk[0]), "v"(pk[1]), "v"(pk[2]), "v"(pk[3]), "v"(g), "v"(zk[0]),
                "v"(zk[1]), "v"(zk[2]), "v"(zk[3]), "s"(ph.inv_r), "s"(cq));
        }
      }
    }
    }  // !kTP
    if constexpr (!IT && !kTabSplit) {  // IT and kTabSplit read tabulated terms instead
      V0 = lo_new;
      VN = hi_new;
    }
    const bool hit1 = !IT && m + 1 == mon.next;
    const bool hit2 = kPair && m + 1 == mon2.next;  // a paired wave's second scenario
    FDCN_STAMP(5);
#if defined(FDCN_DIAG_KO) && FDCN_DIAG_KO == 3  // diagnostic: no knock-out at all
    if (false && (hit1 || hit2)) {
#else
    if (hit1 || hit2) {  // knock-out projection (uniform branch)
#endif
      const double reb = kPair ? (half ? mon2.cur : mon.cur) : mon.cur;
      double rebv = reb;  // VGPR copy: v_cndmask takes the mask as its SGPR operand
      asm volatile("" : "+v"(rebv));
      // Short chunks: the per-slot masks are loop-invariant, the compiler
      // hoists them and they stay in SGPRs.  KoLoad variants (NPT >= 16):
      // they would spill to VGPR lanes (two v_readlane per slot), so they are reloaded
      // from the workspace row with s_load_dwordx16 and applied as one
      // exec-masked v_mov_b64 per slot (config 5: 29.3 -> 26.0 ms per
      // launch).  Rebuilding the masks on the scalar unit from (full, part,
      // k0, k1) measured slower still (34.8 ms): five SALU per slot.
      if constexpr (kKoRes) {
        // run masks and group codes by six scalar loads off the row (one
        // wait), then the slots group by group (fdcn_ko_res.h)
        const unsigned long long sv = __builtin_amdgcn_read_exec();
        unsigned long long q0, q1, q2, qd, mt;
        unsigned c0, c1, cd;
        const unsigned la = lds_addr(ko_rbs);
#ifdef FDCN_KO_VMOV
#define FDCN_KO_RB_WRITE ""
#else
        // the LDS form's rebate word, written by lane 0 while the mask loads
        // are in flight (the statements below read it back into the slots)
#define FDCN_KO_RB_WRITE \
  "s_mov_b64 %6, exec\n\ts_mov_b64 exec, 1\n\tds_write_b64 %14, %15\n\ts_mov_b64 exec, %6\n\t"
#endif
        unsigned long long sx;  // the saved exec of the write
#if defined(FDCN_DIAG_KO) && FDCN_DIAG_KO == 1  // diagnostic: no loads (wrong masks)
        asm volatile("s_mov_b64 %0, 0\n\ts_mov_b64 %1, 0\n\ts_mov_b64 %2, 0\n\ts_mov_b64 %3, 0\n\t"
                     "s_mov_b32 %4, 0\n\ts_mov_b32 %5, 0\n\t" FDCN_KO_RB_WRITE
                     : "=&s"(q0), "=&s"(q1), "=&s"(q2), "=&s"(qd), "=&s"(c0), "=&s"(c1), "=&s"(sx)
                     : "s"(kom_addr), "i"(0), "i"(0), "i"(0), "i"(0), "i"(0), "i"(0), "v"(la),
                       "v"(rebv)
                     : "memory");
#else
        asm volatile("s_load_dwordx2 %0, %7, %8\n\ts_load_dwordx2 %1, %7, %9\n\t"
                     "s_load_dwordx2 %2, %7, %10\n\ts_load_dwordx2 %3, %7, %11\n\t"
                     "s_load_dword %4, %7, %12\n\ts_load_dword %5, %7, %13\n\t"
                     FDCN_KO_RB_WRITE "s_waitcnt lgkmcnt(0)"
                     : "=&s"(q0), "=&s"(q1), "=&s"(q2), "=&s"(qd), "=&s"(c0), "=&s"(c1), "=&s"(sx)
                     : "s"(kom_addr), "i"(16 * kKoRow), "i"(16 * kKoRow + 8),
                       "i"(16 * kKoRow + 16), "i"(16 * kKoRow + 24), "i"(16 * kKoRow + 32),
                       "i"(16 * kKoRow + 36), "v"(la), "v"(rebv)
                     : "memory");
#endif
#undef FDCN_KO_RB_WRITE
        // statements of 16 slots at NPT 64 (the front end counts a tied
        // operand twice against the register file; 16 measured faster than
        // 32 or 8 there, see tools/gen_ko_res.py); exec is restored at the
        // end of each.  The
        // rebate moves in through the LDS unit (ds_read_b64), not the VALU;
        // FDCN_KO_VMOV builds the v_mov_b64 form (statements of 32) for A/B
#ifdef FDCN_KO_VMOV
#define FDCN_KO_RES_CALL(N, B) FDCN_KO_RES_CALLF(FDCN_KO_RES_ASM_##N##_##B, FDCN_KO_RES_VOPS_##N##_##B)
#else
#define FDCN_KO_RES_CALL(N, B) FDCN_KO_RES_CALLF(FDCN_KO_RESL_ASM_##N##_##B, FDCN_KO_RESL_VOPS_##N##_##B)
#endif
#define FDCN_KO_RES_CALLF(FORM, VOPS)                                              \
  asm volatile(FORM                                                                \
               : VOPS, [q0] "+s"(q0), [q1] "+s"(q1), [cd] "=&s"(cd), [mt] "=&s"(mt) \
               : FDCN_KO_RES_INS(rebv, sv, q2, qd, c0, c1, kom_addr, la)          \
               : "scc", "memory")
#if defined(FDCN_DIAG_KO) && FDCN_DIAG_KO == 2  // diagnostic: the loads only
        asm volatile("" ::"s"(q0), "s"(q1), "s"(q2), "s"(qd), "s"(c0), "s"(c1), "v"(rebv));
        (void)mt;
        (void)cd;
        (void)sv;
#else
        if constexpr (NPT == 64) {
          FDCN_KO_RES_CALL(64, 0);
          FDCN_KO_RES_CALL(64, 1);
#ifndef FDCN_KO_VMOV
          FDCN_KO_RES_CALL(64, 2);
          FDCN_KO_RES_CALL(64, 3);
#endif
        } else {  // (48: statements of 32 slots, faster there)
          FDCN_KO_RES_CALL(48, 0);
          FDCN_KO_RES_CALL(48, 1);
        }
#endif
#undef FDCN_KO_RES_CALL
#undef FDCN_KO_RES_CALLF
      } else if constexpr (KoLoad<IT, W, NPT, ZG>::value) {
        // eight slots per block: each slot is one v_mov_b64 of the rebate
        // under an exec mask set on the scalar unit (s_and_b64 with the
        // saved exec), while the next block's eight masks arrive (one
        // s_load_dwordx16, waited for at the end of the block, so every asm
        // output is valid on exit; exec is restored inside the block)
        // (laundered so the compiler cannot hoist the eight block
        // addresses out of the time loop and spill them)
        unsigned long long ka = kPair ? (hit1 ? (hit2 ? kom_addr12 : kom_addr) : kom_addr2) : kom_addr;
        asm volatile("" : "+s"(ka));
        // four slots per block, double-buffered (s_load_dwordx8: 16 SGPRs
        // for both buffers; eight-slot blocks held 32 and pushed other
        // uniform values out to VGPR lanes, read back every step).  Round
        // 5: the blocks' addresses as immediate offsets off one base and
        // exec saved once per projection (ko_blocks): 8 -> 5 SALU per block
        KoMask8 mcur;
        asm volatile("s_load_dwordx8 %0, %1, 0\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(mcur)
                     : "s"(ka)
                     : "memory");
        const unsigned long long sv = __builtin_amdgcn_read_exec();
        ko_blocks<0, NPT / 4, NPT>(V, rebv, ka, sv, mcur);
      } else {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        unsigned long long mk = 0ull;
        if (hit1)
          mk = kml.full | ((k >= kml.k0 && k <= kml.k1) ? kml.part : 0ull) | kmh.full |
               ((k >= kmh.k0 && k <= kmh.k1) ? kmh.part : 0ull);
        if (kPair && hit2)
          mk |= kml2.full | ((k >= kml2.k0 && k <= kml2.k1) ? kml2.part : 0ull) | kmh2.full |
                ((k >= kmh2.k0 && k <= kmh2.k1) ? kmh2.part : 0ull);
        if (kSplit && k == NPT - 1) mk &= ~shrt_ballot;  // the phantom stays zero
        unsigned lo = (unsigned)__double_as_longlong(V[k]);
        unsigned hi = (unsigned)(__double_as_longlong(V[k]) >> 32);
        const unsigned rlo = (unsigned)__double_as_longlong(rebv);
        const unsigned rhi = (unsigned)(__double_as_longlong(rebv) >> 32);
        asm volatile("v_cndmask_b32 %0, %0, %2, %4\n\t"
                     "v_cndmask_b32 %1, %1, %3, %4"
                     : "+v"(lo), "+v"(hi)
                     : "v"(rlo), "v"(rhi), "s"(mk));
        V[k] = __longlong_as_double(((long long)hi << 32) | lo);
      }
      }
      const bool hit_me = kPair ? (half ? hit2 : hit1) : true;
      if (hit_me && 0 <= ko_lo) V0 = reb;
      if (hit_me && n_nodes - 1 >= ko_hi) VN = reb;
      if constexpr (kTabSplit) {
        // which boundary nodes the knock-out removed, per scenario (uniform)
        auto kbits = [&](int klo, int khi) { return (0 <= klo ? 1 : 0) | (n_nodes - 1 >= khi ? 2 : 0); };
        if constexpr (kPair)
          ko_prev = (hit1 ? kbits(__builtin_amdgcn_readlane(ko_lo, 0),
                                  __builtin_amdgcn_readlane(ko_hi, 0)) : 0) |
                    (hit2 ? kbits(__builtin_amdgcn_readlane(ko_lo, 32),
                                  __builtin_amdgcn_readlane(ko_hi, 32)) << 2 : 0);
        else
          ko_prev = kbits(ko_lo, ko_hi);
      }
      FDCN_STAMP(6);
      if (hit1) mon.advance(A.mon_step, A.mon_rebate, m + 1);
      if (kPair && hit2) mon2.advance(A.mon_step, A.mon_rebate, m + 1);
    }
    if constexpr (kNatural) {
      // pointwise rhs: no halos
    } else if constexpr (W > 1) {
      if (lane == 0) xch[Xch<W>::kFirst + wave] = V[0];
      if (lane == 63) xch[Xch<W>::kLast + wave] = shrt ? V[NPT - 2] : V[NPT - 1];
    } else {
      halo_l = shfl_up1(shrt ? V[NPT - 2] : V[NPT - 1], 1);
      halo_r = shfl_dn1(V[0], 1);
    }
    FDCN_STAMP(7);
  }  // step
  }  // block of kStride steps

  if constexpr (IT) {  // Dirichlet values of the last step (the loop kept only rhs terms)
    if (A.n_time > 0) {
      const Bnd q = bnd_params();
      V0 = bnd_eval(q.lof, q.l0, q.l1, q.l2, q.l3, tau_end);
      VN = bnd_eval(q.hif, q.h0, q.h1, q.h2, q.h3, tau_end);
    }
  }
  if constexpr (kTabSplit) {  // likewise, unless the last step knocked the node out
    // (the last step's raw values from the table: the loop keeps no Dirichlet
    // coefficients live)
    if (A.n_time > 0) {
      const double2 raw = raw_load(A.n_time - 1);
      const int kb = kPair ? ((ko_prev >> (2 * half)) & 3) : ko_prev;
      if (!(kb & 1)) V0 = U(raw.x);
      if (!(kb & 2)) VN = U(raw.y);
    }
  }
  // ---- store ---------------------------------------------------------------
#ifdef FDCN_WAVE_TIMES
  // diagnostic builds only (tools/wave_times.py): the wave's start and end
  // clocks and its SIMD, into the scenario's Rannacher save slice
  if constexpr (kRec) {
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0) {
      double* wt = A.vsave + (size_t)scen * 64 * NPT;
      wt[0] = __longlong_as_double((long long)wave_t0);
      wt[1] = __longlong_as_double((long long)t_end);
      wt[2] = (double)hw;
      wt[3] = (double)xcc;
    }
  }
#endif
  double* vout = A.v_out + (size_t)scen * n_nodes;
  const double poison = overflow ? __longlong_as_double(0x7ff8000000000000ll) : 0.0;
  if (active) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int node = s_t + 1 + k;
      if (k < NPT - 1 || !shrt) vout[node] = overflow ? poison : V[k];
    }
  }
  if (t == 0 && valid) {
    vout[0] = overflow ? poison : V0;
    vout[n_nodes - 1] = overflow ? poison : VN;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fdcn_internal::set_error(code, buf);
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
  int (*lds_per_scen)(int lz);  // the kernel's own LDS layout, in doubles
  int zg;                       // correction table in the workspace
  int lat;                      // single-trade (in-wave ILP) flavour
  int pair;                     // two scenarios per wave (32 lanes each)
};

template <int IT, int W, int NPT, int ZG = 0>
Variant mk() {
  return Variant{IT, W, NPT, &fdcn_march<IT, W, NPT, ZG>, Geo<IT, W, NPT, ZG>::kThreads,
                 Geo<IT, W, NPT, ZG>::SPB, &lds_doubles_per_scen<IT, W, NPT, ZG>, ZG & 1,
                 (ZG >> 1) & 1, (ZG >> 2) & 1};
}

// W=1: throughput (one wavefront per scenario).  W>1: grids beyond 64*64
// nodes and small batches (latency).  W=16 workgroups are capped at 128
// VGPRs (16 waves on one CU), so they use short chunks.
#define FDCN_VARIANTS(IT)                                                                   \
  mk<IT, 1, 2>(), mk<IT, 1, 4>(), mk<IT, 1, 8>(), mk<IT, 1, 12>(), mk<IT, 1, 16>(), mk<IT, 1, 24>(),        \
      mk<IT, 1, 32>(), mk<IT, 1, 40>(), mk<IT, 1, 48>(), mk<IT, 1, 64>(), mk<IT, 2, 8>(),   \
      mk<IT, 2, 16>(),                                                                      \
      mk<IT, 2, 32>(), mk<IT, 2, 40>(), mk<IT, 4, 8>(), mk<IT, 4, 16>(), mk<IT, 4, 24>(),   \
      mk<IT, 4, 40>(), mk<IT, 8, 8>(), mk<IT, 8, 16>(), mk<IT, 8, 40>(), mk<IT, 16, 8>(),   \
      mk<IT, 16, 24>(), mk<IT, 16, 40>(), mk<IT, 1, 64, 1>(), mk<IT, 4, 40, 1>(),           \
      mk<IT, 8, 40, 1>(), mk<IT, 16, 40, 1>(), mk<IT, 1, 8, 2>(), mk<IT, 1, 16, 2>(),       \
      mk<IT, 1, 32, 2>()

// The paired flavour (CN split form) for grids of up to 256 interior nodes,
// against one scenario per wave at 4 nodes per lane.  Measured on the
// config-3 batch (10 000 scenarios x 2000 steps, tools/gpu_ab.sh with FDCN_VARIANT; profiles/r02_pair_ab/):
// 256 nodes 3.26 -> 2.94 ms; but 512 nodes 4.35 -> 4.96 (NPT 8 vs paired
// 16) and 1024 nodes 5.81 -> 6.76 (NPT 16 vs paired 32): the paired waves'
// per-lane constants push them to 176 / 242 VGPRs, two waves per SIMD where
// the one-scenario variants keep three, so only the shortest chunks gain.
const Variant kVariants[] = {FDCN_VARIANTS(0), mk<0, 1, 8, 4>(), FDCN_VARIANTS(1)};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

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

int lds_doubles(const Variant& v, int lz);
constexpr size_t kLdsLimit = 160 * 1024;

// Choose the variant: fewest waves per scenario, then the least padding,
// among those whose LDS (correction table + payoff) fits one CU.
bool fits(const Variant& v, int n_int, int k_cap, bool no_idle_wave = true) {
  const int L_act = (n_int + v.npt - 1) / v.npt;
  const int L_short = L_act * v.npt - n_int;
  const int lanes = v.pair ? 32 : 64 * v.w;  // lanes per scenario
  if (L_act > lanes || L_short >= L_act || v.npt > n_int) return false;
  if (no_idle_wave && L_act <= 64 * (v.w - 1)) return false;
  const int kc = k_cap > 0 ? k_cap : (n_int < 256 ? n_int : 256);
  return sizeof(double) * (size_t)lds_doubles(v, lz_for(v, n_int, kc)) <= kLdsLimit;
}

// Waves the chip keeps resident at the design occupancy (256 CUs x 8).
constexpr long kResidentWaves = 2048;

// Diagnostics override (include/fdcn_diag.h): (waves, npt, flavour) packed
// as w | npt << 8 | flavour << 16, 0 = none.  Set only by
// fdcn_force_variant -- the launch path never reads the environment.
std::atomic<int> g_forced{0};

const Variant* forced_variant(int n_int, int it, int k_cap) {
  const int f = g_forced.load(std::memory_order_relaxed);
  if (!f) return nullptr;
  const int w = f & 0xff, npt = (f >> 8) & 0xff, fl = f >> 16;
  for (int zg = 0; zg < 2; ++zg)
    for (int i = 0; i < kNumVariants; ++i) {
      const Variant& v = kVariants[i];
      if (v.it == it && v.w == w && v.npt == npt && v.zg == zg && v.lat == (fl == 1) &&
          v.pair == (fl == 2) && fits(v, n_int, k_cap, zg == 0))
        return &v;
    }
  return nullptr;
}

// Variant choice.  Large batches (the throughput case): fewest waves per
// scenario, then the least padding.  Batches too small to fill the chip
// (B * W_min < kResidentWaves / 2) whose chunks are long (NPT >= 48): spread
// each scenario over more waves, down to 16-node chunks, while the batch
// still fits in one residency round.
const Variant* choose(int n_nodes, int it, int k_cap, long B = 1L << 30) {
  const int n_int = n_nodes - 2;
  if (n_int < 3) return nullptr;
  if (const Variant* f = forced_variant(n_int, it, k_cap)) return f;
  const Variant* best = nullptr;
  long best_slots = 0;
  int best_w = 0;
  // idle waves (a grid just above a variant's size) only when nothing else
  // fits, e.g. a large correction table that needs the LDS of a wider
  // variant; the table in the global workspace (ZG) only after that
  // two-node chunks last of all: only the grids no other chunk length can lay
  // out with at most one phantom slot per lane (5, 6 or 9 interior nodes)
  for (int pass = 0; pass < 4 && !best; ++pass) {
    for (int i = 0; i < kNumVariants; ++i) {
      const Variant& v = kVariants[i];
      if (v.it != it || v.lat || v.pair || v.zg != (pass == 2) || (v.npt == 2) != (pass == 3) ||
          !fits(v, n_int, k_cap, pass == 0))
        continue;
      const long slots = (long)64 * v.w * v.npt;
      if (!best || v.w < best_w || (v.w == best_w && slots < best_slots)) {
        best = &v;
        best_slots = slots;
        best_w = v.w;
      }
    }
  }
  // Batches too small to put a wave on every SIMD, IT march only: the
  // single-trade flavour of the chosen W = 1 variant (in-wave ILP).  Measured
  // (profiles/r05/small_batch/): trade_american (IT, NPT 32) 8.23 -> 7.47 ms
  // per trade; but the CN flavour loses everywhere it was timed --
  // trade_cnlog (NPT 8) 0.426 -> 0.496 ms, the config-3 grid (NPT 16) at
  // B = 64 / 256 / 512 / 1024: 0.75 / 0.76 / 0.87 / 0.83 ms -> 0.98 / 0.99 /
  // 1.12 / 1.08 -- so CN keeps one scenario per wave.  For 64-node chunks
  // (config 5) the split over 4 waves below wins (12.0 ms against 13.5 for
  // either W = 1 flavour).
  if (best && it && best->w == 1 && best->npt < 48 && B * best->w <= kResidentWaves / 2 &&
      !best->zg)
    for (int i = 0; i < kNumVariants; ++i) {
      const Variant& v = kVariants[i];
      if (v.lat && v.it == it && v.w == 1 && v.npt == best->npt && !v.zg) return &v;
    }
  // Throughput batches of grids that fit 32 lanes of twice the chunk length:
  // two scenarios per wave (the paired flavour, compiled for 4-node chunks,
  // see kVariants), as long as the halved wave count still fills the chip.
  if (best && best->w == 1 && !best->zg && !it && B >= 2 * kResidentWaves)
    for (int i = 0; i < kNumVariants; ++i) {
      const Variant& v = kVariants[i];
      if (v.pair && v.it == it && v.npt == 2 * best->npt && fits(v, n_int, k_cap)) return &v;
    }
  // Small batch of long chunks without a single-trade flavour: split 48-64-
  // node chunks to ~16 across waves (config 5, one 4096-node solve: 17.1 ->
  // 12.8 ms); shorter chunks lose it again to the per-step barriers.
  if (!best || best->npt < 48 || B * best->w >= kResidentWaves / 2) return best;
  const Variant* lat = best;
  for (int i = 0; i < kNumVariants; ++i) {
    const Variant& v = kVariants[i];
    if (v.it != it || v.zg || v.lat || !fits(v, n_int, k_cap) || v.npt < 16 ||
        B * v.w > kResidentWaves)
      continue;
    if (v.npt < lat->npt || (v.npt == lat->npt && v.w < lat->w)) lat = &v;
  }
  return lat;
}

int lds_doubles(const Variant& v, int lz) { return v.lds_per_scen(lz) * v.spb; }





int pad64(int n) { return ((n > 0 ? n : 1) + 63) / 64 * 64; }

// workspace bytes per scenario: per wave, one (lo, hi) Dirichlet pair per
// step (split-form variants: a second pair, the raw values behind their rhs
// terms) -- except the rec_form variants, which evaluate each chunk's
// entries in the march (kGen) -- then the knock-out mask row (kKoRow); ZG
// variants add the correction table [2][lz][NPT+1], rec_form variants the
// Rannacher save slice [64][NPT]
size_t bnd_bytes_per_scen(const Variant& v, int n_time) {
  const size_t table = rec_form(v.it, v.w, v.npt)
                           ? kKoResRow
                           : (size_t)pad64(n_time) * (tab_form(v.it, v.w, v.npt, v.lat) ? 2 : 1);
  return sizeof(double) * 2 * (table + kKoRow) * (size_t)v.w;
}
size_t zg_bytes_per_scen(const Variant& v, int lz) {
  return v.zg ? sizeof(double) * 2 * (size_t)lz * (size_t)(v.npt + 1) : 0;
}
size_t ws_bytes_per_scen(const Variant& v, int n_time, int lz) {
  return bnd_bytes_per_scen(v, n_time) + zg_bytes_per_scen(v, lz) +
         (rec_form(v.it, v.w, v.npt) ? sizeof(double) * 64 * (size_t)v.npt : 0);
}

using fdcn_internal::host_fm;
using fdcn_internal::validate_common;
using fdcn_internal::validate_plan;

int launch(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
           const double* params, const int32_t* iparams, const double* v_init,
           const double* payoff, int32_t n_mon, const int32_t* mon_step,
           const double* mon_rebate, double* v_out, int32_t k_cap, double* workspace,
           int64_t workspace_bytes, hipStream_t stream) {
  int rc = validate_common(B, n_nodes, n_time, n_ranna);
  if (rc) return rc;
  if (B == 0) return FDCN_OK;
  const Variant* v = choose(n_nodes, it, k_cap, B);
  if (!v) return fail(FDCN_EINVAL, "unsupported n_nodes=%d", n_nodes);
  const int n_int = n_nodes - 2;
  if (k_cap <= 0) k_cap = n_int < 256 ? n_int : 256;
  const int lz = lz_for(*v, n_int, k_cap);
  const size_t lds = sizeof(double) * (size_t)lds_doubles(*v, lz);
  if (lds > kLdsLimit)
    return fail(FDCN_EINVAL, "LDS request %zu B too large (k_cap=%d)", lds, k_cap);
  const size_t ws_bytes = ws_bytes_per_scen(*v, n_time, lz) * (size_t)B;
  // the variant (and so the workspace) depends on B: a buffer planned for
  // another batch size may be too small -- refuse rather than overrun it
  if (workspace && (workspace_bytes < 0 || (size_t)workspace_bytes < ws_bytes))
    return fail(FDCN_EINVAL,
                "workspace of %lld B is smaller than the %zu B this launch needs (B=%d, "
                "W=%d, NPT=%d): size it with fdcn_plan for the same B and k_cap",
                (long long)workspace_bytes, ws_bytes, B, v->w, v->npt);
  KArgs a;
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
  a.n_pad = pad64(n_time);
  bool own_ws = false;
  if (!workspace) {  // stream-ordered scratch, released after the launch
    HIP_TRY(hipMallocAsync((void**)&workspace, ws_bytes, stream));
    own_ws = true;
  }
  a.bnd = workspace;
  a.zg = workspace + bnd_bytes_per_scen(*v, n_time) / sizeof(double) * (size_t)B;
  a.vsave = a.zg + zg_bytes_per_scen(*v, lz) / sizeof(double) * (size_t)B;
  if (lds > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute((const void*)v->fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
  const int grid = (B + v->spb - 1) / v->spb;
  hipLaunchKernelGGL(v->fn, dim3(grid), dim3(v->threads), lds, stream, a);
  HIP_TRY(hipGetLastError());
  if (own_ws) HIP_TRY(hipFreeAsync(workspace, stream));
  return FDCN_OK;
}

// One non-blocking stream per (calling thread, device), created on first
// use: host-array calls from different threads never share a stream or wait
// for each other, and nothing is synchronised device-wide.  The device's
// default memory pool keeps freed blocks (release threshold = max), so the
// per-call stream-ordered allocations below are pool hits after warm-up.
int thread_stream(hipStream_t* out) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  thread_local std::vector<hipStream_t> streams;
  if ((size_t)dev >= streams.size()) streams.resize((size_t)dev + 1, nullptr);
  if (!streams[dev]) {
    HIP_TRY(hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking));
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  }
  *out = streams[dev];
  return FDCN_OK;
}

size_t align256(size_t n) { return (n + 255) / 256 * 256; }

int host_batch(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
               const double* params, const int32_t* iparams, const double* v_init,
               const double* payoff, int32_t n_mon, const int32_t* mon_step,
               const double* mon_rebate, double* v_out) {
  int rc = validate_plan(it, B, n_nodes, n_time, n_ranna, params, iparams, n_mon, mon_step,
                         mon_rebate);
  if (rc) return rc;
  if (B > 0 && (!v_init || !v_out || (it && !payoff)))
    return fail(FDCN_EINVAL, "null array argument");
  if (B == 0) return FDCN_OK;
  const int k_cap = fdcn_sm_extent(B, n_nodes, n_time, n_ranna, params);
  if (k_cap < 0) return k_cap;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(FDCN_ENODEV, "no HIP device visible");
  int32_t w_, npt_, spb_, lds_;
  int64_t ws_ = 0;
  rc = fdcn_plan(B, n_nodes, n_time, it, k_cap, &w_, &npt_, &spb_, &lds_, &ws_);
  if (rc) return rc;
  hipStream_t stream;
  rc = thread_stream(&stream);
  if (rc) return rc;

  // one stream-ordered block for every device array of the call
  const size_t nv = (size_t)B * n_nodes;
  const size_t nm = (size_t)(n_mon > 0 ? n_mon : 1);
  const size_t oP = 0;
  const size_t oI = oP + align256(sizeof(double) * (size_t)B * FDCN_NPARAM);
  const size_t oV = oI + align256(sizeof(int32_t) * (size_t)B * FDCN_NIPARAM);
  const size_t oO = oV + align256(sizeof(double) * nv);
  const size_t oF = oO + align256(sizeof(double) * nv);
  const size_t oM = oF + (it ? align256(sizeof(double) * nv) : 0);
  const size_t oR = oM + align256(sizeof(int32_t) * nm);
  const size_t oW = oR + align256(sizeof(double) * nm);
  const size_t ws_bytes = (size_t)ws_ * (size_t)B;
  const size_t total = oW + align256(ws_bytes > 0 ? ws_bytes : 1);
  char* blk = nullptr;
  hipError_t e = hipMallocAsync((void**)&blk, total, stream);
  if (e != hipSuccess)
    return fail(FDCN_ENOMEM, "hipMallocAsync(%zu) failed: %s", total, hipGetErrorString(e));
  double* dP = (double*)(blk + oP);
  int32_t* dI = (int32_t*)(blk + oI);
  double* dV = (double*)(blk + oV);
  double* dO = (double*)(blk + oO);
  double* dF = it ? (double*)(blk + oF) : nullptr;
  int32_t* dM = (int32_t*)(blk + oM);
  double* dR = (double*)(blk + oR);
  double* dW = (double*)(blk + oW);
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  e = hipMemcpyAsync(dP, params, sizeof(double) * (size_t)B * FDCN_NPARAM, h2d, stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(dI, iparams, sizeof(int32_t) * (size_t)B * FDCN_NIPARAM, h2d, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dV, v_init, sizeof(double) * nv, h2d, stream);
  if (e == hipSuccess && it) e = hipMemcpyAsync(dF, payoff, sizeof(double) * nv, h2d, stream);
  if (e == hipSuccess && n_mon > 0)
    e = hipMemcpyAsync(dM, mon_step, sizeof(int32_t) * (size_t)n_mon, h2d, stream);
  if (e == hipSuccess && n_mon > 0)
    e = hipMemcpyAsync(dR, mon_rebate, sizeof(double) * (size_t)n_mon, h2d, stream);
  if (e != hipSuccess) rc = fail(FDCN_EHIP, "hipMemcpyAsync H2D failed: %s", hipGetErrorString(e));
  if (rc == FDCN_OK)
    rc = launch(it, B, n_nodes, n_time, n_ranna, dP, dI, dV, dF, n_mon, dM, dR, dO, k_cap, dW,
                (int64_t)ws_bytes, stream);
  if (rc == FDCN_OK) {
    e = hipMemcpyAsync(v_out, dO, sizeof(double) * nv, hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) rc = fail(FDCN_EHIP, "hipMemcpyAsync D2H failed: %s", hipGetErrorString(e));
  }
  (void)hipFreeAsync(blk, stream);
  e = hipStreamSynchronize(stream);
  if (rc == FDCN_OK && e != hipSuccess)
    rc = fail(FDCN_EHIP, "kernel / copies failed: %s", hipGetErrorString(e));
  return rc;
}

}  // namespace

namespace fdcn_internal {
// the march, for the session runtime (fdcn_session.hip)
int launch_march(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                 const double* params, const int32_t* iparams, const double* v_init,
                 const double* payoff, int32_t n_mon, const int32_t* mon_step,
                 const double* mon_rebate, double* v_out, int32_t k_cap, double* workspace,
                 int64_t workspace_bytes, hipStream_t stream) {
  return launch(it, B, n_nodes, n_time, n_ranna, params, iparams, v_init, payoff, n_mon,
                mon_step, mon_rebate, v_out, k_cap, workspace, workspace_bytes, stream);
}
int thread_stream(hipStream_t* out) { return ::thread_stream(out); }
}  // namespace fdcn_internal

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int fdcn_plan(int32_t B, int32_t n_nodes, int32_t n_time, int32_t it_mode, int32_t k_cap,
              int32_t* waves, int32_t* npt, int32_t* scen_per_block, int32_t* lds_bytes,
              int64_t* ws_bytes_per_scen) {
  if (n_time < 0) return fail(FDCN_EINVAL, "n_time must be >= 0 (got %d)", n_time);
  const Variant* v = choose(n_nodes, it_mode ? 1 : 0, k_cap, B > 0 ? B : 1);
  if (!v) return fail(FDCN_EINVAL, "unsupported n_nodes=%d", n_nodes);
  const int n_int = n_nodes - 2;
  if (k_cap <= 0) k_cap = n_int < 256 ? n_int : 256;
  const int lz = lz_for(*v, n_int, k_cap);
  const size_t lds = sizeof(double) * (size_t)lds_doubles(*v, lz);
  if (lds > kLdsLimit) return fail(FDCN_EINVAL, "LDS request %zu B too large", lds);
  if (waves) *waves = v->w;
  if (npt) *npt = v->npt;
  if (scen_per_block) *scen_per_block = v->spb;
  if (lds_bytes) *lds_bytes = (int32_t)lds;
  if (ws_bytes_per_scen) *ws_bytes_per_scen = (int64_t)::ws_bytes_per_scen(*v, n_time, lz);
  return FDCN_OK;
}

int fdcn_cn_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams, const double* v_init,
                      int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                      double* v_out, int32_t k_cap, double* workspace, int64_t workspace_bytes,
                      void* stream) {
  return launch(0, B, n_nodes, n_time, n_ranna, params, iparams, v_init, nullptr, n_mon,
                mon_step, mon_rebate, v_out, k_cap, workspace, workspace_bytes,
                (hipStream_t)stream);
}

int fdcn_it_batch_dev(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                      const double* params, const int32_t* iparams, const double* v_init,
                      const double* payoff, double* v_out, int32_t k_cap, double* workspace,
                      int64_t workspace_bytes, void* stream) {
  return launch(1, B, n_nodes, n_time, n_ranna, params, iparams, v_init, payoff, 0, nullptr,
                nullptr, v_out, k_cap, workspace, workspace_bytes, (hipStream_t)stream);
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

int fdcn_device_ordinals(int32_t* ord, int32_t cap) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int good = 0;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) {
      if (ord && good < cap) ord[good] = i;
      ++good;
    }
  }
  return good;
}

int fdcn_abi_version(void) { return FDCN_ABI_VERSION; }

int fdcn_select_device(int32_t ordinal) {
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (ordinal < 0 || ordinal >= n)
    return fail(FDCN_EINVAL, "device ordinal %d outside [0, %d)", ordinal, n);
  HIP_TRY(hipSetDevice(ordinal));
  return FDCN_OK;
}

int fdcn_current_device(void) {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess) return fail(FDCN_EHIP, "hipGetDevice failed");
  return d;
}

int fdcn_force_variant(int32_t waves, int32_t npt, int32_t flavour) {
  if (waves == 0) {
    g_forced.store(0);
    return FDCN_OK;
  }
  if (flavour < FDCN_FLAVOUR_THROUGHPUT || flavour > FDCN_FLAVOUR_PAIRED)
    return fail(FDCN_EINVAL, "fdcn_force_variant: flavour %d outside [0, 2]", flavour);
  for (int i = 0; i < kNumVariants; ++i) {
    const Variant& v = kVariants[i];
    if (v.w == waves && v.npt == npt && v.lat == (flavour == 1) && v.pair == (flavour == 2)) {
      g_forced.store(waves | (npt << 8) | (flavour << 16));
      return FDCN_OK;
    }
  }
  return fail(FDCN_EINVAL, "fdcn_force_variant: no compiled variant W=%d NPT=%d flavour=%d",
              waves, npt, flavour);
}

int fdcn_variant_name(int32_t B, int32_t n_nodes, int32_t it_mode, int32_t k_cap, char* buf,
                      int32_t len) {
  if (!buf || len < 1) return fail(FDCN_EINVAL, "fdcn_variant_name: buf");
  const Variant* v = choose(n_nodes, it_mode ? 1 : 0, k_cap, B > 0 ? B : 1);
  if (!v) return fail(FDCN_EINVAL, "unsupported n_nodes=%d", n_nodes);
  snprintf(buf, (size_t)len, "fdcn_march<%d,%d,%d,%d>", v->it, v->w, v->npt,
           v->zg | (v->lat << 1) | (v->pair << 2));
  return FDCN_OK;
}

int fdcn_forced_variant(int32_t* waves, int32_t* npt, int32_t* flavour) {
  const int f = g_forced.load();
  if (waves) *waves = f & 0xff;
  if (npt) *npt = (f >> 8) & 0xff;
  if (flavour) *flavour = f >> 16;
  return FDCN_OK;
}


}  // extern "C"
