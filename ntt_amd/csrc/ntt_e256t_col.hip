// Eng256T (4096-element tiles: single 2^20 transforms of 4-limb plans, BASELINE config 2): k_pass
// instantiations for KIND_COLUMN.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng256T, KIND_COLUMN)
}  // namespace ntt
