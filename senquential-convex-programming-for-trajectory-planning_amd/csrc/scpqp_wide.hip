// scpqp_wide.hip — the library's second translation unit: scpqp.hip's device code
// built for 512-thread workgroups (8 waves), providing only the plan-2 kernel for
// factors of 4 row slots (scpqp_wide_launch; see SCPQP_WIDE_TU in scpqp.hip).
#define SCPQP_NT 512
#define SCPQP_NO_HOST
#define SCPQP_WIDE_TU
#include "scpqp.hip"
