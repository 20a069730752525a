// EngP: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_EXTERN_KIND(EngP, KIND_ROWS)  // ntt_ep_rows.hip
NTT_INSTANTIATE(EngP)
}  // namespace ntt
