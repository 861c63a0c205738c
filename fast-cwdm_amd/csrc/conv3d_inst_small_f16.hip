// Explicit instantiation: small-grid conv kernels, fp16.
#include "conv3d_kernels.hpp"
namespace cwdm {
template int launch_conv<f16_t, 32, 4, 2, 1>(const ConvParams&, hipStream_t);
template int launch_conv<f16_t, 16, 4, 4, 1>(const ConvParams&, hipStream_t);
template int launch_conv<f16_t, 8, 8, 4, 1>(const ConvParams&, hipStream_t);
template int launch_conv<f16_t, 32, 4, 2, 2>(const ConvParams&, hipStream_t);
template int launch_conv<f16_t, 16, 4, 4, 2>(const ConvParams&, hipStream_t);
template int launch_conv<f16_t, 8, 8, 4, 2>(const ConvParams&, hipStream_t);
}  // namespace cwdm
