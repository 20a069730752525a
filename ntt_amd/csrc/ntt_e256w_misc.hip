// Eng256w: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng256w)
}  // namespace ntt
