// Eng256w: k_pass instantiations for KIND_COLUMN.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng256w, KIND_COLUMN)
}  // namespace ntt
