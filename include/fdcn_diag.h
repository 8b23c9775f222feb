/*
 * fdcn_diag.h -- diagnostics / tuning entry points of libfdcn.
 *
 * NOT part of the drop-in boundary (include/fdcn.h).  Nothing in the product
 * calls these: the parity tests use them to pin the exact kernel variant a
 * throughput launch would pick (the variant depends on the batch size, and
 * small test batches would otherwise reach other code), and the A/B tools use
 * them to time variants against each other.  The launch path never reads the
 * environment.
 */
#ifndef FDCN_DIAG_H
#define FDCN_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Flavours of a one-wave variant (fdcn_plan reports the geometry). */
#define FDCN_FLAVOUR_THROUGHPUT 0 /* one scenario per wave                      */
#define FDCN_FLAVOUR_LATENCY 1    /* single-trade flavour: in-wave sub-chains     */
#define FDCN_FLAVOUR_PAIRED 2     /* two scenarios per wave (split-form CN)       */

/* Force every subsequent march launch (fdcn_cn/it_batch[_dev], sessions,
 * fdcn_plan) of this process onto the compiled variant (waves, npt, flavour)
 * whenever it fits the grid; launches it does not fit fall back to the normal
 * choice.  waves = 0 clears the override.  Returns FDCN_OK, or FDCN_EINVAL if
 * no such variant is compiled (the override is then left unchanged).
 * Process-wide (all threads); not for concurrent use with production work. */
int fdcn_force_variant(int32_t waves, int32_t npt, int32_t flavour);

/* The current override: writes waves (0 = none), npt, flavour. */
int fdcn_forced_variant(int32_t* waves, int32_t* npt, int32_t* flavour);

/* The kernel template instance a march launch of B scenarios would run
 * (the override included), as "fdcn_march<IT,W,NPT,ZG>" into buf[len]
 * (ZG: bit 0 correction table in the workspace, bit 1 single-trade flavour,
 * bit 2 paired flavour).  Lets a test prove it ran the same instance the
 * benchmark times.  Returns FDCN_OK or FDCN_EINVAL. */
int fdcn_variant_name(int32_t B, int32_t n_nodes, int32_t it_mode, int32_t k_cap, char* buf,
                      int32_t len);

/* Spot-space march (fdcn_vc_batch[_dev]): pin the compiled variant
 * (waves, npt) for every subsequent launch it fits, and/or make every
 * scenario take the stencil form (stencil_only != 0) instead of the
 * pointwise form the factor kernel would choose.  (0, 0, 0) clears both. */
int fdcn_vc_force_variant(int32_t waves, int32_t npt, int32_t stencil_only);

/* "fdcn_vc_march<W,NPT>" a spot-space launch of B scenarios runs. */
int fdcn_vc_variant_name(int32_t B, int32_t n_nodes, char* buf, int32_t len);

/* The form each of B scenarios takes (1 pointwise, 0 stencil): the factor
 * kernel's classification of diag [B][2][6][n_nodes], run on the host. */
int fdcn_vc_forms(int32_t B, int32_t n_nodes, int32_t n_time, int32_t n_ranna,
                  const double* diag, int32_t* form);

#ifdef __cplusplus
}
#endif

#endif /* FDCN_DIAG_H */
