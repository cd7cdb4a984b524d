// Environment switches of liblmi_hip.so (host code only; shared by the HIP and
// the g++ translation units).
#pragma once

namespace lmi {

// ---- environment switches (diagnostics and tuning knobs) ----------------
// Read once, at the first use in the process (thread-safe static init), so no
// launch path calls getenv.  Defaults are the tuned values; results never
// depend on them.
struct EnvConfig {
    bool scan_v1;        // LMI_SCAN_V1: force the general scan kernel
    bool scan_v2;        // LMI_SCAN_V2: force the 4-wave ring
    int scan_abl;        // LMI_SCAN_ABL (the `make ablation` library only)
    int scan_groups;     // LMI_SCAN_GROUPS: tile queues (power of two <= 8), 0 = default
    int scan_lag;        // LMI_SCAN_LAG
    int scan_split;      // LMI_SCAN_SPLIT: split the last K tiles of every queue (0: K = the
                         //   queue's share of the grid, the default; -1: off)
    int scan_split_parts;// LMI_SCAN_SPLIT_PARTS: row parts of a split tile (2..8, default 2)
    int scan_wgs;        // LMI_SCAN_WGS: persistent scan workgroups (0 = one per CU; tests
                         //   use a few to make tiles run after others have published bounds)
    bool scan_no_pref;   // LMI_SCAN_NO_PREF
    bool wide_passes;    // LMI_WIDE_PASSES: k > 16 by lower-bound passes alone (the bound +
                         //   collect scans off; A/B and tests)
    bool wide_no_fixup;  // LMI_WIDE_NO_FIXUP (diagnostic, lists wrong): skip the fix-up passes, so
                         //   the pairs that needed them keep (+inf, -1) -- counts them
    bool router_fma;     // LMI_ROUTER_FMA: FMA-chain router instead of MFMA
    int router_qg;       // LMI_ROUTER_QG: 1/2/4 query groups per workgroup, 0 = auto
    int xsel_kb;         // LMI_XSEL_KB: rows in flight per wave in the split mode's one-wave select (1, 2 or 4; default 1: 7 waves per SIMD)
    int x_skip;          // LMI_X_SKIP_SHARE: the split mode's collect skips a bucket's sample of at most 1/N of it (default 4; 0: never)
    int refine_kb;       // LMI_REFINE_KB: fp16 rows in flight per wave in the float64 refine (1, 2 or 4; default 1: 8 waves per SIMD)
};
const EnvConfig& env_config();

}  // namespace lmi
