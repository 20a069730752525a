// Eng256: k_pass instantiations for KIND_STOCKHAM (the reference's bellperson-family rival schedule).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng256, KIND_STOCKHAM)
}  // namespace ntt
