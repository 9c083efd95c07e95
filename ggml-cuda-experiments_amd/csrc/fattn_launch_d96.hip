// fattn_launch_d96.hip -- the head-dim-96 kernels (fattn_launch.h), compiled in
// their own translation unit so the head dims build in parallel.
#include "fattn_launch.h"

namespace fattn {
template int launch_types<96>(const Plan&, hipStream_t, const Events&);
}  // namespace fattn

#ifdef FATTN_STAMPS
// diagnostic build only: where this unit's kernels write their phase stamps
extern "C" int fattn_debug_set_stamps_d96(void* dev_ptr) {
    return hipMemcpyToSymbol(HIP_SYMBOL(fattn::g_stamps), &dev_ptr, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
