// Fast MODWT kernels for filter length 2 (see jw_modwt_fast.hpp).
#include "jw_modwt_fast.hpp"

namespace jw {
namespace fast {
JW_FAST_INSTANTIATE(2)
}  // namespace fast
}  // namespace jw
