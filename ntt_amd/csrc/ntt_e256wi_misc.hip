// Eng256wI (NTT_PLAN_IN_PLACE plans of the 48-B layout): launchers and element-wise kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng256wI)
}  // namespace ntt
