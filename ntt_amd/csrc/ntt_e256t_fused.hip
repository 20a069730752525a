// Eng256T: the two-pass single launch on 4096-element tiles (k_fused2b / k_fused2bi, BASELINE config 2
// as one kernel, NTT_PLAN_SINGLE_LAUNCH on a 2^20 4-limb plan).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_FUSED2(Eng256T)
}  // namespace ntt
