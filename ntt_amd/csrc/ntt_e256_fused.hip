// Eng256: the fused single-launch 3-pass schedule (k_fused3, NTT_PLAN_SINGLE_LAUNCH).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_FUSED(Eng256)
}  // namespace ntt
