// EngP: k_pass instantiations for KIND_DIT (the reference's GZKP(B, G) rival schedule).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(EngP, KIND_DIT)
}  // namespace ntt
