// Eng256: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_EXTERN_KIND(Eng256, KIND_ROWS)  // ntt_e256_rows.hip
NTT_INSTANTIATE(Eng256)
}  // namespace ntt
