// spmm_functor.h — the functional layer's internal C++ entries shared by the eager functor
// (spmm_functor.cpp), the compiled row-split job (ccl_functor.cpp) and the kernel's state
// (user/kernels/spmm_kernel.cpp).  The C-ABI entries in include/ofx_spmm.h wrap these.
#ifndef OFX_ONEFLOW_CORE_FUNCTIONAL_SPMM_FUNCTOR_H_
#define OFX_ONEFLOW_CORE_FUNCTIONAL_SPMM_FUNCTOR_H_

#include <memory>

#include "oneflow/core/framework/framework.h"
#include "ofx_spmm.h"

namespace oneflow {

// functional::SpmmCsr on one rank of a placement with an explicit kernel state: the lazy path's
// form, where each compiled op owns its OpKernelState (core/kernel/user_kernel.cpp keeps it per
// UserKernel).  *state is created through the registered kernel's CreateOpKernelState on the
// first launching call that has none.  static_csr is the op attribute (include/ofx_spmm.h
// ofx_spmm_attrs).
int SpmmCsrGlobalWithState(void* stream, const ofx_tensor_desc* row_ptr,
                           const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                           int64_t m, int64_t k, const ofx_tensor_desc* b, int64_t b_logical_cols,
                           ofx_tensor_desc* out, void* tmp, size_t tmp_bytes, int hierarchy_ndim,
                           const int64_t* hierarchy, const int32_t* out_split_axes,
                           int64_t parallel_id, int64_t static_csr,
                           std::shared_ptr<user_op::OpKernelState>* state);

// The static-CSR plan counters of a spmm_csr kernel state, added to *entries / *plans / *hits
// (release: its workspaces are freed first).  False when `state` is not one.
bool SpmmCsrPlanStateStats(user_op::OpKernelState* state, int64_t* entries, int64_t* plans,
                           int64_t* hits, bool release);

}  // namespace oneflow

#endif  // OFX_ONEFLOW_CORE_FUNCTIONAL_SPMM_FUNCTOR_H_
