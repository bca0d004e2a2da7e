// insert_nccl_logical_op_pass.cpp — see the header.
#include "oneflow/core/job_rewriter/insert_nccl_logical_op_pass.h"

namespace oneflow {

std::string NcclLogicalOpType1D(const std::string& src_sbp, const std::string& dst_sbp,
                                const Shape& logical_shape, int64_t parallel_num) {
  auto CanSplitAtDim = [&](int64_t dim) -> bool {
    if (dim < 0 || logical_shape.NumAxes() <= dim) return false;
    return logical_shape.At(dim) % parallel_num == 0;
  };
  const int64_t src_axis = SplitAxisOf(src_sbp), dst_axis = SplitAxisOf(dst_sbp);
  const bool src_p = src_sbp == "P", dst_b = dst_sbp == "B";
  if (src_p && dst_b) return "_nccl_logical_all_reduce";                          // P->B
  if (CanSplitAtDim(0) && src_p && dst_axis == 0) return "_nccl_logical_reduce_scatter";  // P->S(0)
  if (CanSplitAtDim(0) && src_axis == 0 && dst_b) return "_nccl_logical_all_gather";      // S(0)->B
  if (src_axis > 0 && dst_b && CanSplitAtDim(src_axis))
    return "_nccl_logical_all_gather_noncontinuous";                              // S(1)->B
  if (src_axis >= 0 && dst_axis >= 0 && src_axis != dst_axis && CanSplitAtDim(src_axis) &&
      CanSplitAtDim(dst_axis))
    return "_nccl_logical_s2s";                                                   // S(i)->S(j)
  if (CanSplitAtDim(dst_axis) && src_p && dst_axis > 0)
    return "_nccl_logical_reduce_scatter_noncontinuous";                          // P->S(1)
  return "";
}

}  // namespace oneflow
