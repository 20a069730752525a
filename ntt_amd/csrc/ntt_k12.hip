// Explicit instantiation of the NTT kernels for 12 x 32-bit limbs (12 words per element).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(12, 12)
}  // namespace ntt
