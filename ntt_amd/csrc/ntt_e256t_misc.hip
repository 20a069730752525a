// Eng256T (4096-element tiles: single 2^20 transforms of 4-limb plans, BASELINE config 2): launchers
// and element-wise kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng256T)
}  // namespace ntt
