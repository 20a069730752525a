// EngP: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(EngP)
}  // namespace ntt
