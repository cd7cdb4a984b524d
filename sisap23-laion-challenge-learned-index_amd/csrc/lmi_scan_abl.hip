// Diagnostic variants of scan3_kernel (`make ablation` -> li/liblmi_hip_abl.so;
// never linked into the product library).
//
// The ablations DESIGN.md §3 / §5 tabulate -- MFMA stream alone, no DMA, no
// insertion, DMA from L2, exchange periods, the 16x16x32 shape probe, ... --
// are instantiations of the same kernel template (lmi_scan3.hpp) with a
// non-zero ABL parameter, selected at run time by LMI_SCAN_ABL through the
// weak hook lmi_abl_launch_scan3 that lmi_scan.hip calls when it is linked.
// ABL != 0 variants compute wrong results by design (timing only), except
// ABL 7 (the full kernel plus event counters).  lmi_debug_counters reads and
// clears the counters (Scan2Args::dbg): see lmi_scan3.hpp for their meaning.
#include "lmi_scan3.hpp"

namespace {
__device__ unsigned long long g_dbg[16];

unsigned long long* dbg_ptr() {
    static unsigned long long* p = [] {
        void* q = nullptr;
        if (hipGetSymbolAddress(&q, HIP_SYMBOL(g_dbg)) != hipSuccess) q = nullptr;
        return static_cast<unsigned long long*>(q);
    }();
    return p;
}

template <int KL>
int launch_abl(int abl, const lmi::Scan2Args& b, hipStream_t s) {
    using lmi::launch_scan3_v;
    switch (abl) {
#define LMI_ABL_CASE(n) \
    case n:             \
        return launch_scan3_v<KL, n>(b, s);
        LMI_ABL_CASE(1) LMI_ABL_CASE(2) LMI_ABL_CASE(3) LMI_ABL_CASE(4) LMI_ABL_CASE(5)
        LMI_ABL_CASE(6) LMI_ABL_CASE(7) LMI_ABL_CASE(14) LMI_ABL_CASE(21) LMI_ABL_CASE(31)
        LMI_ABL_CASE(32) LMI_ABL_CASE(33) LMI_ABL_CASE(40) LMI_ABL_CASE(41) LMI_ABL_CASE(42)
        LMI_ABL_CASE(43) LMI_ABL_CASE(50) LMI_ABL_CASE(51) LMI_ABL_CASE(52) LMI_ABL_CASE(53)
        LMI_ABL_CASE(57) LMI_ABL_CASE(61) LMI_ABL_CASE(62) LMI_ABL_CASE(64) LMI_ABL_CASE(65)
        LMI_ABL_CASE(66) LMI_ABL_CASE(67) LMI_ABL_CASE(68) LMI_ABL_CASE(69) LMI_ABL_CASE(70)
#undef LMI_ABL_CASE
        default:
            return launch_scan3_v<KL, 0>(b, s);
    }
}
}  // namespace

extern "C" int lmi_abl_launch_scan3(int kl, int abl, const void* args, void* stream) {
    lmi::Scan2Args b = *static_cast<const lmi::Scan2Args*>(args);
    b.dbg = dbg_ptr();
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return kl == 10 ? launch_abl<10>(abl, b, s) : launch_abl<15>(abl, b, s);
}

extern "C" int lmi_debug_counters(unsigned long long* out16) {
    unsigned long long z[16] = {};
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_dbg), sizeof(z)) != hipSuccess) return LMI_E_HIP;
    z[10] = ~0ull;
    z[14] = ~0ull;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z)) != hipSuccess) return LMI_E_HIP;
    return LMI_OK;
}
