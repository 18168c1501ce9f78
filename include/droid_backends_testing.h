/* droid_backends_testing.h - hooks of the TESTING builds of libdroid_hip.so
 * (make ab -> lib/ab/libdroid_hip.so, make prof -> lib/prof/libdroid_hip.so).
 *
 * Not part of the drop-in boundary: the product library (make ->
 * lib/libdroid_hip.so, include/droid_backends.h) exports none of these.  They
 * exist for A/B timings, the bitwise cross-checks that tie dropped kernel
 * variants to the product kernels, the failure-handling tests and the
 * in-kernel timelines (scripts/ *_timeline.py).  No reference counterpart.
 * Return codes and the last-error string as in droid_backends.h. */
#ifndef DROID_BACKENDS_TESTING_H
#define DROID_BACKENDS_TESTING_H

#include "droid_backends.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Profiling switch for the band convolution kernel (the profiling build
 * fills the buffer; the A/B build returns DROID_UNSUPPORTED): while buf is
 * set, each launch writes 6 int64 per workgroup (hardware id | XCC id << 32,
 * s_memtime at entry, when the first stage's operands have landed, at the end
 * of the main loop, when the epilogue's stores are issued and when they have
 * drained).  buf = null switches it off.  Not part of the reference interface
 * (scripts/conv_timeline.py). */
int droid_conv_set_profile(void* buf);
/* The same for corr_alt_ce0_kernel: per workgroup, its first 32 stages x 8
 * int64 (s_memtime at stage start / box landed / C done / C barrier / bilinear
 * done / lookup barrier / stage end, then box taps * 2 + slow-path flag)
 * (scripts/alt_timeline.py). */
int droid_alt_set_profile(void* buf);
/* A/B hook for the on-demand lookup: 2 = corr_alt2_kernel (two 4-wave
 * workgroups per CU, the product).  The A/B build (make ab) adds 1 =
 * corr_alt_ce0_kernel (one 8-wave workgroup per CU), 3 = the V3 C split, 4 =
 * the round-4 corr_alt2_kernel, 5 / 6 = its row-K lookup tile / pixel-major C
 * alone.  1, 4 and 6 are bitwise equal; 2, 3 and 5 are bitwise equal and
 * differ from the first set by corr_encoder[0]'s K order only (a few ulps);
 * the other values return DROID_UNSUPPORTED in the profiling build. */
int droid_alt_set_variant(int v);
/* Tuning hook: edges per XCD chunk of corr_alt2_kernel's tile walk (0 = interleaved, the default). */
int droid_alt_set_chunk(int edges);
/* Tuning hook: 1 = the cooperative NCHW lookup behind the 4-level pyramid lookups (default),
 * 0 = the per-thread kernel; outputs are bitwise equal. */
int droid_lookup_set_coop(int on);
/* Tile policy of the W == 64 3x3 band convs (not part of the reference
 * interface; tests run both tiles in one process): -1 = default (the plain
 * convs and small gate-conv grids on the two-workgroups-per-CU tile, larger
 * gate-conv grids on the 8-wave band tiles), 0 = 8-wave band tiles only, 1 = the
 * two-workgroup tile wherever it applies.  Returns the previous policy, -2 for
 * a bad mode.  Process-wide. */
int droid_conv_set_tile(int mode);
/* Which kernel droid_conv_gru_pre_f16 takes for a ConvGRU gate conv (epi 1 =
 * z|r, 2 = q) over B images of H x W under the current policy: 1 =
 * conv_band2_kernel, 0 = the 8-wave band tile, 2 = the opt-in 4-wave z|r tile,
 * -1 = none (DROID_UNSUPPORTED).  Queries the device's CU count. */
int droid_conv_gate_tile(int epi, int B, int H, int W);
/* Cholesky task timeline (make prof; the A/B build returns DROID_UNSUPPORTED):
 * 24 int64 s_memrealtime stamps per task (scripts/chol_timeline.py) */
int droid_chol_set_profile(void* buf);
/* Test hook for the dataflow solve's failure handling (no reference
 * counterpart): 0 off, 1 every solve aborts as on a dependency-wait timeout
 * (status bit 1), 2 only the next solve does, 3 the next solve is launched
 * without zeroing its sync area (status bits 1 and 2 from the kernel's entry
 * check).  Process-wide. */
int droid_chol_set_fault_inject(int mode);

#ifdef __cplusplus
}
#endif

#endif /* DROID_BACKENDS_TESTING_H */
