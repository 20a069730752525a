// Eng256w: k_pass instantiations for KIND_FINAL.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng256w, KIND_FINAL)
}  // namespace ntt
