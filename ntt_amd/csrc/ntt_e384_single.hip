// Eng384: k_pass instantiations for KIND_SINGLE.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng384, KIND_SINGLE)
}  // namespace ntt
