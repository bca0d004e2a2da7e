// SpMM forward kernels for value type double, index type int32_t (spmm_csr_impl.h).
#pragma clang fp contract(off)

#include "spmm_csr_impl.h"

OFX_SPMM_INSTANTIATE(double, int32_t)
