// Explicit instantiation: wide-grid conv kernels, fp16.
#include "conv3d_kernels.hpp"
namespace cwdm {
template int launch_wide<f16_t, 1>(const ConvParams&, hipStream_t);
template int launch_wide<f16_t, 2>(const ConvParams&, hipStream_t);
}  // namespace cwdm
