// fdcn_session.hip -- device-resident march sessions (C ABI: include/fdcn.h).
//
// The host-array entry points (fdcn_cn_batch / fdcn_it_batch) copy every
// value vector back to the host.  The pricers need far less: the reference
// reads 3-4 nodes per solve for price/Delta/Gamma (discrete_barrier_fdm_pricer.py
// :629-646, :949-978; fd_american_equity.py:855-907), combines solves into
// vega / theta / Richardson (:883-904, :970-1068), and between the dividend
// segments of an American solve remaps the whole vector through a natural
// cubic spline (fd_american_equity.py:479-553, :732-772, :825-843).  A session
// keeps the value vectors in HBM ("slots") and chains those steps on the
// device:
//
//   fdcn_session_march          one batched CN/KO or IT launch; initial vectors
//                               from the host or from earlier slots
//   fdcn_session_dividend_jump  spline remap of slots into new slots (device)
//   fdcn_session_greeks         per-trade readouts + combinations -> T x 6
//                               scalars back to the host
//   fdcn_session_fetch          whole vectors back (when a caller wants them)
//
// Each march runs on one of a few session streams (independent launch groups
// overlap -- the American N / 2N pair); a consumer of slots waits on the
// events of the launches that produced them.  Host inputs are staged through a
// session-owned pinned arena, so every copy is truly asynchronous and the
// caller's arrays are free to go as soon as a call returns.  Device memory is
// stream-ordered (hipMallocAsync from the device pool) and released by
// fdcn_session_destroy.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/fdcn.h"
#include "fdcn_session_book.h"

namespace fdcn_internal {
int set_error(int code, const char* msg);
int validate_plan(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* params, const int32_t* iparams, int32_t n_mon,
                  const int32_t* mon_step, const double* mon_rebate);
int launch_march(int it, int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                 const double* params, const int32_t* iparams, const double* v_init,
                 const double* payoff, int32_t n_mon, const int32_t* mon_step,
                 const double* mon_rebate, double* v_out, int32_t k_cap, double* workspace,
                 int64_t workspace_bytes, hipStream_t stream);
}  // namespace fdcn_internal

namespace {

// Staging copy into pinned memory: whole-file plans stage 100-400 MB of
// initial vectors per march, which one thread copies at ~8 GB/s; above 16 MB
// the copy is split over up to 8 host threads.
void stage_copy(void* dst, const void* src, size_t n) {
  constexpr size_t kPar = size_t(16) << 20;
  if (n < kPar) {
    memcpy(dst, src, n);
    return;
  }
  unsigned hw = std::thread::hardware_concurrency();
  const size_t nt = std::min<size_t>(hw ? hw : 1, 8);
  const size_t chunk = (n / nt + 4095) & ~size_t(4095);
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t) {
    const size_t a = t * chunk;
    if (a >= n) break;
    const size_t len = std::min(chunk, n - a);
    th.emplace_back([=]() { memcpy((char*)dst + a, (const char*)src + a, len); });
  }
  for (auto& x : th) x.join();
}

int sfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fdcn_internal::set_error(code, buf);
}

#define S_TRY(expr)                                                                \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return sfail(FDCN_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int kMaxStreams = 4;
using fdcn_book::al256;
using fdcn_book::Layout;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// v_init rows from earlier slots: row b <- *src[b] (n doubles)
__global__ void gather_rows(const uint64_t* __restrict__ src, double* __restrict__ dst, int n) {
  const double* s = reinterpret_cast<const double*>(src[blockIdx.x]);
  double* d = dst + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

// Dividend jump of one value vector per workgroup (fd_american_equity.py
// :732-772 with the natural cubic spline of :479-553).  Lane 0 runs the
// spline's tridiagonal sweep (the same operation order as the reference and
// as fdcn_dividend_jump, contraction off, IEEE division: bit-identical);
// then all lanes evaluate V(S - D) at their nodes (binary search for the
// interval, as searchsorted(side="right") - 1).
__global__ void __launch_bounds__(64)
dividend_jump_kernel(int n, const uint64_t* __restrict__ src, const double* __restrict__ s_all,
                     const double* __restrict__ cash, const double* __restrict__ strike,
                     double* __restrict__ out_all, double* __restrict__ work) {
#pragma clang fp contract(off)
  const int b = blockIdx.x;
  const double* v = reinterpret_cast<const double*>(src[b]);
  const double* s = s_all + (size_t)b * n;
  double* out = out_all + (size_t)b * n;
  double* mu = work + (size_t)b * 3 * n;
  double* z = mu + n;
  double* c = z + n;
  if (threadIdx.x == 0) {
    mu[0] = 0.0;
    z[0] = 0.0;
    for (int i = 1; i + 1 < n; ++i) {
      const double hm = s[i] - s[i - 1], h = s[i + 1] - s[i];
      const double alpha = 3.0 / h * (v[i + 1] - v[i]) - 3.0 / hm * (v[i] - v[i - 1]);
      const double l = 2.0 * (s[i + 1] - s[i - 1]) - hm * mu[i - 1];
      mu[i] = h / l;
      z[i] = (alpha - hm * z[i - 1]) / l;
    }
    c[n - 1] = 0.0;
    z[n - 1] = 0.0;
    mu[n - 1] = 0.0;
    for (int j = n - 2; j >= 0; --j) c[j] = z[j] - mu[j] * c[j + 1];
  }
  __syncthreads();
  const double D = cash[b], K = strike[b];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double q = s[i] - D;
    double cont;
    if (q <= s[0]) {
      cont = v[0];
    } else if (q >= s[n - 1]) {
      cont = v[n - 1];
    } else {
      int lo = 0, hi = n;  // first index with s[idx] > q
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] > q) hi = mid;
        else lo = mid + 1;
      }
      int j = lo - 1;
      if (j > n - 2) j = n - 2;
      const double h = s[j + 1] - s[j];
      const double bj = (v[j + 1] - v[j]) / h - h * (c[j + 1] + 2.0 * c[j]) / 3.0;
      const double dj = (c[j + 1] - c[j]) / (3.0 * h);
      const double t = q - s[j];
      cont = v[j] + bj * t + c[j] * t * t + dj * t * t * t;
    }
    if (K >= 0.0) {  // calls may exercise at the ex-date: max(cont, payoff)
      const double e = s[i] - K;
      const double ex = (0.0 > e) ? 0.0 : e;
      cont = (ex > cont) ? ex : cont;
    }
    out[i] = cont;
  }
}

// ---- Greeks epilogue -------------------------------------------------------
// Readout r of a value vector (ints [slot, interp_case, ilo, idx, dg_mode] are
// resolved on the host into an address; doubles [S_i, s_lo, s_hi, S_d, s_a,
// s_b, s_c, s_d]):
//   price  linear interpolation at S_i (…pricer.py:629-646, equity.py:855-874):
//          interp_case 1 -> V[0], 2 -> V[ilo], else (1-w) V[ilo] + w V[ilo+1],
//          w = (S_i - s_lo) / (s_hi - s_lo)
//   dg_mode 1  non-uniform 3-point Delta/Gamma at idx (…pricer.py:949-978)
//           2  local cubic through idx-1..idx+2 in z = s - S_d, Delta = c,
//              Gamma = 2b (fd_american_equity.py:876-907)
struct Readout {
  double price, delta, gamma;
};

__device__ Readout read_grid(const double* V, const int32_t* ri, const double* rd) {
#pragma clang fp contract(off)
  Readout o{0.0, 0.0, 0.0};
  const int icase = ri[1], ilo = ri[2], idx = ri[3], mode = ri[4];
  if (icase == 1) o.price = V[0];
  else if (icase == 2) o.price = V[ilo];
  else {
    const double w = (rd[0] - rd[1]) / (rd[2] - rd[1]);
    o.price = (1.0 - w) * V[ilo] + w * V[ilo + 1];
  }
  if (mode == 1) {
    const double h1 = rd[5] - rd[4], h2 = rd[6] - rd[5];
    const double Vm = V[idx - 1], V0 = V[idx], Vp = V[idx + 1];
    o.delta = -h2 / (h1 * (h1 + h2)) * Vm + (h2 - h1) / (h1 * h2) * V0 + h1 / (h2 * (h1 + h2)) * Vp;
    o.gamma = 2.0 * (Vm / (h1 * (h1 + h2)) - V0 / (h1 * h2) + Vp / (h2 * (h1 + h2)));
  } else if (mode == 2) {
    // [z^3 z^2 z 1] coef = y, LU with partial pivoting (LAPACK dgetf2 order)
    double A[4][4], y[4];
    for (int k = 0; k < 4; ++k) {
      const double zk = rd[4 + k] - rd[3];
      A[k][0] = zk * zk * zk;
      A[k][1] = zk * zk;
      A[k][2] = zk;
      A[k][3] = 1.0;
      y[k] = V[idx - 1 + k];
    }
    int perm[4] = {0, 1, 2, 3};
    for (int j = 0; j < 4; ++j) {
      int p = j;
      for (int i = j + 1; i < 4; ++i)
        if (fabs(A[i][j]) > fabs(A[p][j])) p = i;
      if (p != j) {
        for (int k = 0; k < 4; ++k) {
          const double tmp = A[j][k];
          A[j][k] = A[p][k];
          A[p][k] = tmp;
        }
        const int tp = perm[j];
        perm[j] = perm[p];
        perm[p] = tp;
      }
      const double rp = 1.0 / A[j][j];
      for (int i = j + 1; i < 4; ++i) {
        A[i][j] *= rp;
        for (int k = j + 1; k < 4; ++k) A[i][k] -= A[i][j] * A[j][k];
      }
    }
    double x[4];
    for (int i = 0; i < 4; ++i) x[i] = y[perm[i]];
    for (int j = 0; j < 4; ++j)
      for (int i = j + 1; i < 4; ++i) x[i] -= x[j] * A[i][j];
    for (int j = 3; j >= 0; --j) {
      x[j] /= A[j][j];
      for (int i = 0; i < j; ++i) x[i] -= x[j] * A[i][j];
    }
    o.delta = x[2];
    o.gamma = 2.0 * x[1];
  }
  return o;
}

// one thread per trade; the combinations keep the reference's operation
// order (Python evaluation order), so with the same value vectors they are
// bit-identical to the host epilogues of the facades
__global__ void greeks_kernel(int T, const int32_t* __restrict__ tkind,
                              const int32_t* __restrict__ tfirst,
                              const double* __restrict__ tpar, const uint64_t* __restrict__ raddr,
                              const int32_t* __restrict__ rint, const double* __restrict__ rdbl,
                              double* __restrict__ out) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const double* P = tpar + (size_t)t * FDCN_GK_NPARAM;
  const int r0 = tfirst[t];
  auto rd = [&](int k) {
    const int r = r0 + k;
    return read_grid(reinterpret_cast<const double*>(raddr[r]), rint + (size_t)r * FDCN_GK_NRINT,
                     rdbl + (size_t)r * FDCN_GK_NRDBL);
  };
  double* o = out + (size_t)t * FDCN_GK_NOUT;
  double price = 0.0, delta = 0.0, gamma = 0.0, vega = 0.0, theta = 0.0, aux = 0.0;
  const int kind = tkind[t];
  if (kind == FDCN_GK_BARRIER) {
    // _pde_price_and_greeks3 (discrete_barrier_fdm_pricer.py:883-904)
    // P = sigma, spot, carry, div_yield, r, dv
    const Readout b = rd(0), u = rd(1);
    price = b.price;
    delta = b.delta;
    gamma = b.gamma;
    vega = (u.price - b.price) / (P[5] * 100);
    theta = -(0.5 * P[0] * P[0] * P[1] * P[1] * gamma + (P[2] - P[3]) * P[1] * delta -
              P[4] * price);
  } else if (kind == FDCN_GK_CNLOG) {
    // _pde_price_and_greeks (discrete_barrier_fdm_pricer_cn.py:429-466)
    // P = sigma, S0, b, r, dv
    const Readout b = rd(0), u = rd(1), d = rd(2);
    price = b.price;
    delta = b.delta;
    gamma = b.gamma;
    theta = -(0.5 * P[0] * P[0] * P[1] * P[1] * gamma + P[2] * P[1] * delta - P[3] * price);
    vega = (u.price - d.price) / (2.0 * P[4]);
  } else if (kind == FDCN_GK_AMERICAN) {
    // greeks_log2 with Richardson (fd_american_equity.py:970-1068) and the
    // price_log2 Richardson N / 2*num_space_nodes (:925-951) in aux
    // P = sigma, spot, carry, r, h
    const Readout n1 = rd(0), n2 = rd(1);
    price = (4.0 * n2.price - n1.price) / 3.0;
    delta = (4.0 * n2.delta - n1.delta) / 3.0;
    gamma = (4.0 * n2.gamma - n1.gamma) / 3.0;
    const double h = P[4];
    const double first_h = (rd(2).price - rd(3).price) / (2.0 * h);
    const double first_2h = (rd(4).price - rd(5).price) / (4.0 * h);
    const double dvds = (4.0 * first_h - first_2h) / 3.0;
    vega = dvds / 100.0;
    const double q = 0.0;
    theta = -(0.5 * P[0] * P[0] * P[1] * P[1] * gamma + (P[2] - q) * P[1] * delta - P[3] * price);
    aux = (4.0 * rd(6).price - n1.price) / 3.0;
  } else {  // FDCN_GK_READOUT
    const Readout b = rd(0);
    price = b.price;
    delta = b.delta;
    gamma = b.gamma;
  }
  o[0] = price;
  o[1] = delta;
  o[2] = gamma;
  o[3] = vega;
  o[4] = theta;
  o[5] = aux;
}

int readouts_per_kind(int kind) {
  switch (kind) {
    case FDCN_GK_BARRIER: return 2;
    case FDCN_GK_CNLOG: return 3;
    case FDCN_GK_AMERICAN: return 7;
    case FDCN_GK_READOUT: return 1;
    default: return -1;
  }
}

// Pinned staging (fdcn_session_book.h): within a session every async copy
// reads/writes a region no later call of that session reuses; the regions
// are recycled only after fdcn_session_destroy has synchronised the
// session's streams.
struct HipPinned {
  static void* alloc(size_t n) {
    void* p = nullptr;
    return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
  }
  static void release(void* p) { (void)hipHostFree(p); }
};
using PinnedArena = fdcn_book::PinnedArenaT<HipPinned>;
// pinned staging an idle per-thread context keeps between sessions: enough
// for a whole-file plan (a 10 000-row barrier file stages 131 MB, a 2 000-row
// American file ~400 MB), so repeated files reuse it (pinning it again costs
// ~15-40 ms per file: 34 -> 52 ms per 10 000-row file with a 64 MB cap),
// while the process's locked memory stays bounded per thread
constexpr size_t kIdlePinnedBytes = size_t(1) << 30;

// Per-thread, per-device resources a session borrows: streams, spare events
// and the pinned arena.  Creating them costs far more than a small trade's
// march (streams ~100 us, an 8 MB pinned chunk ~1 ms), so fdcn_session_destroy
// hands them back to the thread's idle list instead of releasing them
// (they live until the process ends).
struct Ctx {
  int device = 0;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> spare_events;
  PinnedArena pinned;
};
thread_local std::vector<Ctx*> t_idle_ctx;

}  // namespace

struct fdcn_session {
  int device = 0;
  Ctx* ctx = nullptr;
  std::vector<hipStream_t> streams;  // the ctx streams this session has used
  int rr = 0;
  std::vector<hipEvent_t> events;
  fdcn_book::SlotTable slots;
  struct Block {
    void* p;
    hipStream_t s;
  };
  std::vector<Block> blocks;
  PinnedArena& pinned() { return ctx->pinned; }
};

namespace {

int pick_stream(fdcn_session* s, hipStream_t* out) {
  if ((int)s->streams.size() < kMaxStreams) {
    Ctx* c = s->ctx;
    if (c->streams.size() <= s->streams.size()) {
      hipStream_t st;
      S_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      c->streams.push_back(st);
    }
    hipStream_t st = c->streams[s->streams.size()];
    s->streams.push_back(st);
    *out = st;
    return FDCN_OK;
  }
  *out = s->streams[s->rr++ % kMaxStreams];
  return FDCN_OK;
}

int check_slots(fdcn_session* s, int32_t n, const int32_t* slots, int32_t n_nodes) {
  char err[160];
  if (s->slots.check(n, slots, n_nodes, err, sizeof(err))) return sfail(FDCN_EINVAL, "%s", err);
  return FDCN_OK;
}

// make `st` wait for the launches that produced the given slots
int wait_producers(fdcn_session* s, hipStream_t st, int32_t n, const int32_t* slots) {
  for (int32_t e : s->slots.producers(n, slots)) S_TRY(hipStreamWaitEvent(st, s->events[e], 0));
  return FDCN_OK;
}

int alloc_block(fdcn_session* s, hipStream_t st, size_t bytes, char** out) {
  void* p = nullptr;
  hipError_t e = hipMallocAsync(&p, bytes, st);
  if (e != hipSuccess)
    return sfail(FDCN_ENOMEM, "hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
  s->blocks.push_back({p, st});
  *out = (char*)p;
  return FDCN_OK;
}

// record the completion of the work just queued on `st`; returns the event id
int record(fdcn_session* s, hipStream_t st, int32_t* ev) {
  hipEvent_t e;
  if (!s->ctx->spare_events.empty()) {
    e = s->ctx->spare_events.back();
    s->ctx->spare_events.pop_back();
  } else {
    S_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  S_TRY(hipEventRecord(e, st));
  s->events.push_back(e);
  *ev = (int32_t)s->events.size() - 1;
  return FDCN_OK;
}

int new_slots(fdcn_session* s, double* base, int32_t B, int32_t n_nodes, int32_t ev,
              int32_t* out_slots) {
  s->slots.add(base, B, n_nodes, ev, out_slots);
  return FDCN_OK;
}

}  // namespace

extern "C" {

int fdcn_session_create(fdcn_session** out) {
  if (!out) return sfail(FDCN_EINVAL, "fdcn_session_create: NULL out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return sfail(FDCN_ENODEV, "no HIP device visible");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return sfail(FDCN_EHIP, "hipGetDevice failed");
  Ctx* c = nullptr;
  for (size_t i = 0; i < t_idle_ctx.size(); ++i)
    if (t_idle_ctx[i]->device == dev) {
      c = t_idle_ctx[i];
      t_idle_ctx.erase(t_idle_ctx.begin() + (long)i);
      break;
    }
  if (!c) {
    c = new Ctx();
    c->device = dev;
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
      uint64_t keep = UINT64_MAX;  // keep freed blocks in the pool between sessions
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  }
  fdcn_session* s = new fdcn_session();
  s->device = dev;
  s->ctx = c;
  *out = s;
  return FDCN_OK;
}

int fdcn_session_destroy(fdcn_session* s) {
  if (!s) return FDCN_OK;
  int rc = FDCN_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != s->device) (void)hipSetDevice(s->device);
  // Drain every session stream BEFORE the frees: a block allocated on one
  // stream is read on others (gather_rows of v_init slots, the dividend
  // jump, the Greeks epilogue wait on its producer's event), so a free
  // ordered on the allocating stream alone could hand the block to another
  // allocation while a consumer still reads it.  After the syncs no work of
  // the session is pending and the stream-ordered frees are safe.
  for (hipStream_t st : s->streams)
    if (hipStreamSynchronize(st) != hipSuccess) rc = sfail(FDCN_EHIP, "stream sync failed");
  if (rc == FDCN_OK) {
    for (auto& b : s->blocks)
      if (hipFreeAsync(b.p, b.s) != hipSuccess) rc = sfail(FDCN_EHIP, "hipFreeAsync failed");
  }  // after a failure the blocks are leaked rather than freed under running work
  if (rc == FDCN_OK) {  // everything drained: the resources go back to the thread
    for (hipEvent_t e : s->events) s->ctx->spare_events.push_back(e);
    s->ctx->pinned.reset();
    s->ctx->pinned.trim(kIdlePinnedBytes);
    t_idle_ctx.push_back(s->ctx);
  }  // after a failure they are dropped (leaked) rather than reused
  if (cur != s->device) (void)hipSetDevice(cur);
  delete s;
  return rc;
}

int fdcn_session_slots(const fdcn_session* s) { return s ? (int)s->slots.size() : -1; }

int fdcn_session_host_buffer(fdcn_session* s, int64_t bytes, void** out) {
  if (!s || !out || bytes < 0) return sfail(FDCN_EINVAL, "fdcn_session_host_buffer: bad argument");
  *out = s->pinned().get((size_t)bytes);
  if (!*out) return sfail(FDCN_ENOMEM, "hipHostMalloc(%lld) failed", (long long)bytes);
  return FDCN_OK;
}

int fdcn_session_march(fdcn_session* s, int32_t it, int32_t B, int32_t n_nodes, int32_t n_time,
                       int32_t n_ranna, const double* params, const int32_t* iparams,
                       const double* v_init, const int32_t* v_init_slots, const double* payoff,
                       int32_t n_mon, const int32_t* mon_step, const double* mon_rebate,
                       int32_t* out_slots) {
  if (!s) return sfail(FDCN_EINVAL, "NULL session");
  it = it ? 1 : 0;
  int rc = fdcn_internal::validate_plan(it, B, n_nodes, n_time, n_ranna, params, iparams, n_mon,
                                        mon_step, mon_rebate);
  if (rc) return rc;
  if (B == 0) return FDCN_OK;
  if (!out_slots) return sfail(FDCN_EINVAL, "NULL out_slots");
  if ((v_init == nullptr) == (v_init_slots == nullptr))
    return sfail(FDCN_EINVAL, "pass exactly one of v_init (host) and v_init_slots");
  if (it && !payoff) return sfail(FDCN_EINVAL, "IT march without payoff");
  if (v_init_slots && (rc = check_slots(s, B, v_init_slots, n_nodes))) return rc;
  const int k_cap = fdcn_sm_extent(B, n_nodes, n_time, n_ranna, params);
  if (k_cap < 0) return k_cap;
  int32_t w_, npt_, spb_, lds_;
  int64_t ws_ = 0;
  if ((rc = fdcn_plan(B, n_nodes, n_time, it, k_cap, &w_, &npt_, &spb_, &lds_, &ws_))) return rc;

  const size_t nv = (size_t)B * n_nodes, nm = (size_t)(n_mon > 0 ? n_mon : 1);
  const size_t vb = sizeof(double) * nv;
  // the small inputs, the payoff and v_init, then device-only buffers
  Layout L;
  const size_t oP = L.add(sizeof(double) * B * FDCN_NPARAM);
  const size_t oI = L.add(sizeof(int32_t) * B * FDCN_NIPARAM);
  const size_t oM = L.add(sizeof(int32_t) * nm);
  const size_t oR = L.add(sizeof(double) * nm);
  const size_t oA = v_init_slots ? L.add(sizeof(uint64_t) * B) : 0;
  const size_t pre = L.size;  // the small inputs: [0, pre)
  const size_t oF = it ? L.add(vb) : 0;
  // an IT march whose host v_init is its payoff array (the first segment of
  // an American grid) copies that array once and reads it twice
  const bool v_is_payoff = it && v_init && v_init == payoff;
  const size_t oV = L.add(vb);  // copied only for a host v_init
  const size_t oO = L.add(vb);
  const size_t ws_bytes = (size_t)ws_ * (size_t)B;
  const size_t oW = L.add(ws_bytes);
  // A payoff / v_init inside this session's pinned memory (from
  // fdcn_session_host_buffer: a plan written straight into it) is copied to
  // the device from where it lies; anything else is staged.  The staging
  // block mirrors the device offsets up to the first array copied directly,
  // so the common all-staged case is one H2D copy.
  const bool f_direct = it && s->pinned().owns(payoff, vb);
  const bool v_host = v_init && !v_is_payoff;
  const bool v_direct = v_host && s->pinned().owns(v_init, vb);
  const bool stage_f = it && !f_direct, stage_v = v_host && !v_direct;
  size_t hsz = pre, hF = 0, hV = 0;
  if (stage_f) hF = hsz, hsz = oF + al256(vb);
  if (stage_v) hV = it ? (stage_f ? oV : pre) : oV, hsz = hV + al256(vb);
  const size_t mirrored = stage_v && hV == oV ? oV + vb : stage_f ? oF + vb : pre;

  char* h = s->pinned().get(hsz);
  if (!h) return sfail(FDCN_ENOMEM, "hipHostMalloc(%zu) failed", hsz);
  memcpy(h + oP, params, sizeof(double) * B * FDCN_NPARAM);
  memcpy(h + oI, iparams, sizeof(int32_t) * B * FDCN_NIPARAM);
  if (n_mon > 0) {
    memcpy(h + oM, mon_step, sizeof(int32_t) * n_mon);
    memcpy(h + oR, mon_rebate, sizeof(double) * n_mon);
  }
  if (v_init_slots) {
    uint64_t* a = (uint64_t*)(h + oA);
    for (int32_t b = 0; b < B; ++b) a[b] = (uint64_t)s->slots.ptr[v_init_slots[b]];
  }
  if (stage_f) stage_copy(h + hF, payoff, vb);
  if (stage_v) stage_copy(h + hV, v_init, vb);
  hipStream_t st;
  if ((rc = pick_stream(s, &st))) return rc;
  if (v_init_slots && (rc = wait_producers(s, st, B, v_init_slots))) return rc;
  char* d = nullptr;
  if ((rc = alloc_block(s, st, L.size, &d))) return rc;
  S_TRY(hipMemcpyAsync(d, h, mirrored, hipMemcpyHostToDevice, st));
  if (f_direct) S_TRY(hipMemcpyAsync(d + oF, payoff, vb, hipMemcpyHostToDevice, st));
  if (stage_v && hV != oV) S_TRY(hipMemcpyAsync(d + oV, h + hV, vb, hipMemcpyHostToDevice, st));
  if (v_direct) S_TRY(hipMemcpyAsync(d + oV, v_init, vb, hipMemcpyHostToDevice, st));
  if (v_init_slots) {
    hipLaunchKernelGGL(gather_rows, dim3(B), dim3(256), 0, st, (const uint64_t*)(d + oA),
                       (double*)(d + oV), n_nodes);
    S_TRY(hipGetLastError());
  }
  rc = fdcn_internal::launch_march(it, B, n_nodes, n_time, n_ranna, (const double*)(d + oP),
                                   (const int32_t*)(d + oI),
                                   (const double*)(d + (v_is_payoff ? oF : oV)),
                                   it ? (const double*)(d + oF) : nullptr, n_mon,
                                   (const int32_t*)(d + oM), (const double*)(d + oR),
                                   (double*)(d + oO), k_cap, (double*)(d + oW),
                                   (int64_t)ws_bytes, st);
  if (rc) return rc;
  int32_t ev;
  if ((rc = record(s, st, &ev))) return rc;
  return new_slots(s, (double*)(d + oO), B, n_nodes, ev, out_slots);
}

int fdcn_session_dividend_jump(fdcn_session* s, int32_t B, int32_t n_nodes,
                               const int32_t* in_slots, const double* s_nodes,
                               const double* cash_div, const double* strike_call,
                               int32_t* out_slots) {
  if (!s) return sfail(FDCN_EINVAL, "NULL session");
  if (B < 0 || n_nodes < 2) return sfail(FDCN_EINVAL, "dividend jump: B >= 0, n_nodes >= 2");
  if (B == 0) return FDCN_OK;
  if (!in_slots || !s_nodes || !cash_div || !strike_call || !out_slots)
    return sfail(FDCN_EINVAL, "dividend jump: NULL argument");
  int rc = check_slots(s, B, in_slots, n_nodes);
  if (rc) return rc;
  for (int32_t b = 0; b < B; ++b)
    for (int32_t i = 0; i + 1 < n_nodes; ++i)
      if (!(s_nodes[(size_t)b * n_nodes + i + 1] - s_nodes[(size_t)b * n_nodes + i] > 0.0))
        return sfail(FDCN_EINVAL, "x must be strictly increasing.");
  const size_t nv = (size_t)B * n_nodes;
  Layout L;
  const size_t oA = L.add(sizeof(uint64_t) * B);
  const size_t oS = L.add(sizeof(double) * nv);
  const size_t oC = L.add(sizeof(double) * B);
  const size_t oK = L.add(sizeof(double) * B);
  const size_t staged = L.size;
  const size_t oO = L.add(sizeof(double) * nv);
  const size_t oW = L.add(sizeof(double) * 3 * nv);
  char* h = s->pinned().get(staged);
  if (!h) return sfail(FDCN_ENOMEM, "hipHostMalloc(%zu) failed", staged);
  uint64_t* a = (uint64_t*)(h + oA);
  for (int32_t b = 0; b < B; ++b) a[b] = (uint64_t)s->slots.ptr[in_slots[b]];
  stage_copy(h + oS, s_nodes, sizeof(double) * nv);
  memcpy(h + oC, cash_div, sizeof(double) * B);
  memcpy(h + oK, strike_call, sizeof(double) * B);
  hipStream_t st;
  if ((rc = pick_stream(s, &st))) return rc;
  if ((rc = wait_producers(s, st, B, in_slots))) return rc;
  char* d = nullptr;
  if ((rc = alloc_block(s, st, L.size, &d))) return rc;
  S_TRY(hipMemcpyAsync(d, h, staged, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(dividend_jump_kernel, dim3(B), dim3(64), 0, st, n_nodes,
                     (const uint64_t*)(d + oA), (const double*)(d + oS), (const double*)(d + oC),
                     (const double*)(d + oK), (double*)(d + oO), (double*)(d + oW));
  S_TRY(hipGetLastError());
  int32_t ev;
  if ((rc = record(s, st, &ev))) return rc;
  return new_slots(s, (double*)(d + oO), B, n_nodes, ev, out_slots);
}

int fdcn_session_greeks(fdcn_session* s, int32_t T, const int32_t* kind, const int32_t* first,
                        const double* tparams, int32_t R, const int32_t* rint,
                        const double* rdbl, double* out) {
  if (!s) return sfail(FDCN_EINVAL, "NULL session");
  if (T < 0 || R < 0) return sfail(FDCN_EINVAL, "greeks: T, R >= 0");
  if (T == 0) return FDCN_OK;
  if (!kind || !first || !tparams || !rint || !rdbl || !out)
    return sfail(FDCN_EINVAL, "greeks: NULL argument");
  for (int32_t t = 0; t < T; ++t) {
    const int k = readouts_per_kind(kind[t]);
    if (k < 0) return sfail(FDCN_EINVAL, "trade %d: unknown kind %d", t, kind[t]);
    if (first[t] < 0 || first[t] + k > R)
      return sfail(FDCN_EINVAL, "trade %d: readouts [%d,+%d) outside R=%d", t, first[t], k, R);
  }
  std::vector<int32_t> slots(R);
  for (int32_t r = 0; r < R; ++r) {
    const int32_t* ri = rint + (size_t)r * FDCN_GK_NRINT;
    slots[r] = ri[0];
    int rc = check_slots(s, 1, &ri[0], -1);
    if (rc) return rc;
    const int n = s->slots.n[ri[0]];
    const bool ok_i = (ri[1] == 1) || (ri[1] == 2 && ri[2] >= 0 && ri[2] < n) ||
                      (ri[1] == 0 && ri[2] >= 0 && ri[2] + 1 < n);
    const bool ok_d = (ri[4] == 0) || (ri[4] == 1 && ri[3] >= 1 && ri[3] + 1 < n) ||
                      (ri[4] == 2 && ri[3] >= 1 && ri[3] + 2 < n);
    if (!ok_i || !ok_d)
      return sfail(FDCN_EINVAL, "readout %d: node indices outside its %d-node vector", r, n);
  }
  Layout L;
  const size_t oA = L.add(sizeof(uint64_t) * R);
  const size_t oRI = L.add(sizeof(int32_t) * R * FDCN_GK_NRINT);
  const size_t oRD = L.add(sizeof(double) * R * FDCN_GK_NRDBL);
  const size_t oK = L.add(sizeof(int32_t) * T);
  const size_t oF = L.add(sizeof(int32_t) * T);
  const size_t oP = L.add(sizeof(double) * T * FDCN_GK_NPARAM);
  const size_t staged = L.size;
  const size_t oO = L.add(sizeof(double) * T * FDCN_GK_NOUT);
  char* h = s->pinned().get(L.size);
  if (!h) return sfail(FDCN_ENOMEM, "hipHostMalloc(%zu) failed", L.size);
  uint64_t* a = (uint64_t*)(h + oA);
  for (int32_t r = 0; r < R; ++r) a[r] = (uint64_t)s->slots.ptr[slots[r]];
  memcpy(h + oRI, rint, sizeof(int32_t) * R * FDCN_GK_NRINT);
  memcpy(h + oRD, rdbl, sizeof(double) * R * FDCN_GK_NRDBL);
  memcpy(h + oK, kind, sizeof(int32_t) * T);
  memcpy(h + oF, first, sizeof(int32_t) * T);
  memcpy(h + oP, tparams, sizeof(double) * T * FDCN_GK_NPARAM);
  hipStream_t st;
  int rc = pick_stream(s, &st);
  if (rc) return rc;
  if ((rc = wait_producers(s, st, R, slots.data()))) return rc;
  char* d = nullptr;
  if ((rc = alloc_block(s, st, L.size, &d))) return rc;
  S_TRY(hipMemcpyAsync(d, h, staged, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(greeks_kernel, dim3((T + 63) / 64), dim3(64), 0, st, T,
                     (const int32_t*)(d + oK), (const int32_t*)(d + oF),
                     (const double*)(d + oP), (const uint64_t*)(d + oA),
                     (const int32_t*)(d + oRI), (const double*)(d + oRD), (double*)(d + oO));
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpyAsync(h + oO, d + oO, sizeof(double) * T * FDCN_GK_NOUT, hipMemcpyDeviceToHost,
                       st));
  S_TRY(hipStreamSynchronize(st));
  memcpy(out, h + oO, sizeof(double) * T * FDCN_GK_NOUT);
  return FDCN_OK;
}

int fdcn_session_fetch(fdcn_session* s, int32_t n, const int32_t* slots, int32_t n_nodes,
                       double* out) {
  if (!s) return sfail(FDCN_EINVAL, "NULL session");
  if (n < 0 || n_nodes < 1) return sfail(FDCN_EINVAL, "fetch: n >= 0, n_nodes >= 1");
  if (n == 0) return FDCN_OK;
  if (!slots || !out) return sfail(FDCN_EINVAL, "fetch: NULL argument");
  int rc = check_slots(s, n, slots, n_nodes);
  if (rc) return rc;
  const size_t bytes = sizeof(double) * (size_t)n * n_nodes;
  Layout L;
  const size_t oA = L.add(sizeof(uint64_t) * n);
  const size_t oO = L.add(bytes);
  char* h = s->pinned().get(L.size);
  if (!h) return sfail(FDCN_ENOMEM, "hipHostMalloc(%zu) failed", L.size);
  uint64_t* a = (uint64_t*)(h + oA);
  for (int32_t i = 0; i < n; ++i) a[i] = (uint64_t)s->slots.ptr[slots[i]];
  hipStream_t st;
  if ((rc = pick_stream(s, &st))) return rc;
  if ((rc = wait_producers(s, st, n, slots))) return rc;
  char* d = nullptr;
  if ((rc = alloc_block(s, st, L.size, &d))) return rc;
  // gather the rows into one buffer: one D2H copy instead of one per slot
  S_TRY(hipMemcpyAsync(d + oA, h + oA, sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(gather_rows, dim3(n), dim3(256), 0, st, (const uint64_t*)(d + oA),
                     (double*)(d + oO), n_nodes);
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpyAsync(h + oO, d + oO, bytes, hipMemcpyDeviceToHost, st));
  S_TRY(hipStreamSynchronize(st));
  memcpy(out, h + oO, bytes);
  return FDCN_OK;
}

}  // extern "C"
