// Implicit-GEMM conv kernels, WGRAD instantiations (conv_gemm_kernel.h; host side in conv.hip).
#include "conv_gemm_kernel.h"

template void wgrad_launch<bf16>(const ConvArgs&, int, int, int, hipStream_t);
template void wgrad_launch<float>(const ConvArgs&, int, int, int, hipStream_t);
