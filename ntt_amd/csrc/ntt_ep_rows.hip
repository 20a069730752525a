// EngP: k_pass instantiations for KIND_ROWS (several single-tile transforms per workgroup).
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_INSTANTIATE_KIND(EngP, KIND_ROWS)
}  // namespace ntt
