// EngPI (P with 8-B scratch, NTT_PLAN_IN_PLACE): launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(EngPI)
}  // namespace ntt
