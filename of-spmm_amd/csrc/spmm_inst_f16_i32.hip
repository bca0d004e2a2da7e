// SpMM forward kernels for value type f16, index type int32_t (spmm_csr_impl.h).
#pragma clang fp contract(off)

#include "spmm_csr_impl.h"

OFX_SPMM_INSTANTIATE(ofx::f16, int32_t)
