// Implicit-GEMM conv kernels, DGRAD instantiations (conv_gemm_kernel.h; host side in conv.hip).
#include "conv_gemm_kernel.h"

template void dispatch_align<bf16, MODE_DGRAD>(const ConvArgs&, int, hipStream_t, int);
template void dispatch_align<float, MODE_DGRAD>(const ConvArgs&, int, hipStream_t, int);
// DGRAD split-K (small-M deep convs): the 128 x 128 tile with fp32 slabs
template void launch_al<bf16, MODE_DGRAD, 128, 128, 64, 2, 2>(const ConvArgs&, int, hipStream_t, int);
