// Explicit instantiation of the NTT kernels for 1 x 32-bit limbs (2 words per element).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(1, 2)
}  // namespace ntt
