// EngPI (P with 8-B scratch, NTT_PLAN_IN_PLACE): k_pass instantiations for KIND_COLUMN.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(EngPI, KIND_COLUMN)
}  // namespace ntt
