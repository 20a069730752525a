// EngP: k_pass instantiations for KIND_COLUMN.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(EngP, KIND_COLUMN)
}  // namespace ntt
