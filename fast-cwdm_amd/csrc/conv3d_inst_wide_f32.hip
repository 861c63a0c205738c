// Explicit instantiation: wide-grid conv kernels, f32.
#include "conv3d_kernels.hpp"
namespace cwdm {
template int launch_wide<float, 1>(const ConvParams&, hipStream_t);
template int launch_wide<float, 2>(const ConvParams&, hipStream_t);
}  // namespace cwdm
