// Launch choices that tests and A/B measurements may override.
//
// The library never reads these from the environment: a user's stray variable cannot change a
// launch.  They are set through dava_debug_set_override (include/dava_ba.h), which the Python binding
// calls for a test that asks for one, or -- once, when the library is loaded -- for the DAVA_<NAME>
// environment variables when DAVA_DEBUG_OVERRIDES=1 is set (tools/ab_env.sh).  Results never depend
// on them beyond what the parity tests check (reduction trees, LDS or HBM residency, launch shape).
#pragma once

namespace dava {

enum DebugKnob : int {
  kDbgForceGV,        // 1: global-vector mode even where the LDS image fits (cross-checks GV vs LDS)
  kDbgGVNoXL,         // 1: GV mode objective on the workspace vectors, not on LDS copies of x and d
  kDbgSolveWaves,     // 1 | 2 | 4: waves per LDS-mode solve workgroup
  kDbgWgPerCu,        // > 0: LDS budget for on-chip history entries = 160 KB / this
  kDbgLdsHistory,     // >= 0: on-chip history entries (clamped to one workgroup's LDS)
  kDbgStagger,        // >= 0: staggered start, shader cycles per level (0: none)
  kDbgStaggerLevels,  // >= 1: start levels
  kDbgNoPPT,          // 1: the objective re-reads its points from LDS (no points in registers)
  kDbgNoQueue,        // 1: one workgroup per problem (no work queue)
  kDbgAdjGVWaves,     // 4 | 8: waves per global-vector-mode adjoint workgroup
  kDbgAdjForceGV,     // 1: global-vector-mode adjoint even where the LDS image fits
  kDbgAdjLdsEntries,  // >= 0: caps the adjoint's on-chip history entries
  kDbgAdjGdHbm,       // 1: the GV adjoint's dual gradient vector in HBM instead of LDS
  kDbgCompactSwitch,  // >= 1: COMPACT history capacity before the dense fold (default 1024; tests)
  kDbgGvScalarSlice,  // 0 | 1: GV wide pass's rho_j, c_j in LDS / in the workspace slice (default: by fit)
  kDbgAdjScGlobal,    // 0 | 1: LDS-mode adjoint's tape scalar row staged in LDS / read in place (default: by fit)
  kDbgKnobs
};

// The override of `k`, or -1 when it is not set (the library's own choice applies).
long long debug_knob(int k);
inline bool debug_flag(int k) { return debug_knob(k) > 0; }

}  // namespace dava
