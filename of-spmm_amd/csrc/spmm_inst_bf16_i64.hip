// SpMM forward kernels for value type bf16, index type int64_t (spmm_csr_impl.h).
#pragma clang fp contract(off)

#include "spmm_csr_impl.h"

OFX_SPMM_INSTANTIATE(ofx::bf16, int64_t)
