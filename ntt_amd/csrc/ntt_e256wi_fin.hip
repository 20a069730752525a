// Eng256wI (NTT_PLAN_IN_PLACE plans of the 48-B layout): k_pass instantiations for KIND_FINAL.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(Eng256wI, KIND_FINAL)
}  // namespace ntt
