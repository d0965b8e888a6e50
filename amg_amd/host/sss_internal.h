/*
 * sss_internal.h — declarations shared between the host C files of libsss_amg.so and the
 * HIP engine (amg_amd/csrc).  Not part of the public drop-in ABI (include/sss_amg.h) nor of
 * the device-engine ABI (include/sss_hip.h).
 */
#ifndef SSS_INTERNAL_H
#define SSS_INTERNAL_H

#include "../../include/sss_amg.h"
#include "../../include/sss_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Releases the HBM mirror registered for a hierarchy (keyed by mg->cg); no-op if none. */
void sss_dev_release_mirror(const void *cg_key);

/* Returns the HBM mirror for mg, building it on first use (registry keyed by mg->cg). */
sss_hip_hier *sss_dev_mirror_for(SSS_AMG *mg);

/* Fatal HIP/RCCL failure in the product path: print in the reference's style and exit. */
void sss_fatal(const char *where, const char *what);

/* Ask for transparent huge pages on a large, not yet touched allocation (madvise MADV_HUGEPAGE on
 * its page-aligned interior; a no-op below 8 MiB).  The setup's random-access passes (the RS first
 * pass, transposes, RAP) walk gigabytes of per-point records and CSR rows: with 4 KiB pages nearly
 * every access also misses the TLB. */
void sss_huge_hint(void *p, size_t bytes);
/* malloc / calloc followed by sss_huge_hint */
void *sss_big_malloc(size_t bytes);
void *sss_big_calloc(size_t n, size_t size);

/* roctx ranges (rocprofv3 --marker-trace shows them; near-free without a profiler): the solve's
 * outer iterations, the setup's levels, the mirror's level tasks, and per level the descent and
 * ascent of a V-cycle as it is enqueued (eager launches, or once at the graph capture). */
void sss_trace_push(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void sss_trace_pop(void);

#ifdef __cplusplus
}
#endif

#endif
