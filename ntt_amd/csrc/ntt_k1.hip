// Explicit instantiation of the NTT kernels for the EngP engine.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(EngP)
}  // namespace ntt
