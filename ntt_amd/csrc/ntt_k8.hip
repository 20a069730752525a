// Explicit instantiation of the NTT kernels for 8 x 32-bit limbs (8 words per element).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(8, 8)
}  // namespace ntt
