// Eng256w: launchers, fill / pack / transpose / pointwise / twiddle-build kernels.
#include "ntt_kernels_impl.hpp"
namespace ntt {
NTT_EXTERN_KIND(Eng256w, KIND_ROWS)  // ntt_e256w_rows.hip
NTT_INSTANTIATE(Eng256w)
}  // namespace ntt
