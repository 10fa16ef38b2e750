/*
 * gsvc_amd_diag.h -- entry points of the DIAGNOSTIC library only
 * (gsvc_amd/lib/libgsvc_amd_diag.so, built from the same sources with
 * -DGSVC_DIAG).  The product library libgsvc_amd.so has none of these: its
 * kernel selection depends only on the call's arguments and the data, and it
 * carries no diagnostic kernel variants.  tools/ (microbenchmarks, A/B runs,
 * timestamped variants) and the variant-comparison tests load the diagnostic
 * library (gsvc_amd._lib.diagnostic()); nothing in the product path does.
 * Not part of the reference interface.
 */
#ifndef GSVC_AMD_DIAG_H
#define GSVC_AMD_DIAG_H

#include "gsvc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A/B knob for kernel variants: key 0 forces the sum-forward kernel mode
 * (0 = automatic from the density; 1 sparse, 2 banded; 3-8 timestamped,
 * ablation and priority variants), the other keys the tuning parameters named
 * where the library reads them (csrc: knob(k)); returns the previous value
 * (-1 for an unknown key).  Every value that is not an ablation gives the same
 * results. */
int gsvc_debug_set(int key, int value);
/* Device buffer the timestamped variants write into (int64 per tile x 4). */
void gsvc_debug_set_ptr(void *ptr);

#ifdef __cplusplus
}
#endif

#endif /* GSVC_AMD_DIAG_H */
