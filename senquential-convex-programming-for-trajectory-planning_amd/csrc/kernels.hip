// kernels.hip — the kernel instantiations of scpqp_kernel.h, in groups.  build.py
// compiles this file once per group (-DSCPQP_KGROUP=1..10) as separate translation
// units, in parallel, and links them with scpqp.hip (which declares every
// instantiation extern, SCPQP_KERNEL_LIST) and plant.hip.  Each group also carries its
// own diagnostic counters (diag_read).  A build partition, not a behaviour switch:
// every kernel is compiled from the same source whatever its group.

#include "scpqp_kernel.h"

#ifndef SCPQP_KGROUP
#error "kernels.hip is compiled once per group: -DSCPQP_KGROUP=1..10 (scpqp/build.py)"
#endif
static_assert(SCPQP_KGROUP >= 1 && SCPQP_KGROUP <= 10, "kernel groups 1..10");

#define SCPQP_INST(HG, VG, RM, OCC, SH) \
    template int scpqp_kern::launch<HG, VG, RM, OCC, SH>(const void*, size_t, hipStream_t, int);

template int scpqp_kern::diag_read<SCPQP_KGROUP>(int, unsigned long long*, int, int);

#if SCPQP_KGROUP == 1   // c2 / c4: 4 vehicles, Hp 20, plan 1 at three workgroups per CU
SCPQP_INST(false, true, 2, 3, 1)
#ifdef SCPQP_DIAG   // diagnostic builds: the lean plan at four per CU (scpqp.hip plan)
SCPQP_INST(false, true, 2, 4, 1)
#endif
#elif SCPQP_KGROUP == 2   // c3: 8 vehicles, Hp 30, factor in the workspace
SCPQP_INST(true, true, 4, 2, 3)
#elif SCPQP_KGROUP == 3   // c5: mixed horizons up to 30, lean plan 1 at two per CU
SCPQP_INST(false, true, 2, 2, 2)
#elif SCPQP_KGROUP == 4   // c5-shaped launches with hp_max <= 20
SCPQP_INST(false, true, 2, 3, 2)
SCPQP_INST(true, true, 2, 3, 2)
#elif SCPQP_KGROUP == 5   // run-time shapes: factor in the workspace
SCPQP_INST(true, true, 1, 2, 0) SCPQP_INST(true, true, 1, 3, 0)
SCPQP_INST(true, true, 2, 2, 0) SCPQP_INST(true, true, 2, 3, 0)
#elif SCPQP_KGROUP == 6
SCPQP_INST(true, true, 3, 2, 0) SCPQP_INST(true, true, 3, 3, 0)
SCPQP_INST(true, true, 4, 2, 0) SCPQP_INST(true, true, 4, 3, 0)
#elif SCPQP_KGROUP == 7   // run-time shapes: factor in LDS, vectors in the workspace
SCPQP_INST(false, true, 1, 2, 0) SCPQP_INST(false, true, 1, 3, 0)
SCPQP_INST(false, true, 2, 2, 0) SCPQP_INST(false, true, 2, 3, 0)
#elif SCPQP_KGROUP == 8
SCPQP_INST(false, true, 3, 2, 0) SCPQP_INST(false, true, 3, 3, 0)
SCPQP_INST(false, true, 4, 2, 0) SCPQP_INST(false, true, 4, 3, 0)
#elif SCPQP_KGROUP == 9   // run-time shapes: everything in LDS
SCPQP_INST(false, false, 1, 2, 0) SCPQP_INST(false, false, 1, 3, 0)
SCPQP_INST(false, false, 2, 2, 0) SCPQP_INST(false, false, 2, 3, 0)
#else
SCPQP_INST(false, false, 3, 2, 0) SCPQP_INST(false, false, 3, 3, 0)
SCPQP_INST(false, false, 4, 2, 0) SCPQP_INST(false, false, 4, 3, 0)
#endif
