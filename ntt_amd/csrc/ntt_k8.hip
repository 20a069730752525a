// Explicit instantiation of the NTT kernels for the Eng256 engine.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng256)
}  // namespace ntt
