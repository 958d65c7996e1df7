// Implicit-GEMM conv kernels, FWD instantiations (conv_gemm_kernel.h; host side in conv.hip).
// One translation unit per GEMM mode so the three compile in parallel.
#include "conv_gemm_kernel.h"

template void dispatch_align<bf16, MODE_FWD>(const ConvArgs&, int, hipStream_t, int);
template void dispatch_align<float, MODE_FWD>(const ConvArgs&, int, hipStream_t, int);
