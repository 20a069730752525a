// Eng384: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng384)
}  // namespace ntt
