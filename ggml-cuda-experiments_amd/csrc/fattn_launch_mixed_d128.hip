// fattn_launch_mixed_d128.hip -- the head-dim-128 split kernels over mixed K / V
// cache types (fattn_launch.h launch_mixed), in their own translation unit so
// they build in parallel with the single-type ones.
#include "fattn_launch.h"

namespace fattn {
template int launch_mixed<128>(const Plan&, hipStream_t, const Events&);
}  // namespace fattn
