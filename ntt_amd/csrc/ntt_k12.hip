// Explicit instantiation of the NTT kernels for the Eng384 engine.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE(Eng384)
}  // namespace ntt
