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

#ifdef __cplusplus
}
#endif

#endif
