// insert_nccl_logical_op_pass.h — the decision of OneFlow's InsertNcclLogicalOpPass for one
// boxing edge of a 1-D placement (oneflow/core/job_rewriter/insert_nccl_logical_op_pass.cpp:150-240,
// TryBuildNcclBy1DHierarchy): which logical collective op replaces the boxing, or "" when none
// applies (the edge then keeps ordinary boxing).  The pass runs for device placements only
// (kCUDA in the reference, kHIP here).
#ifndef OFX_ONEFLOW_INSERT_NCCL_LOGICAL_OP_PASS_H_
#define OFX_ONEFLOW_INSERT_NCCL_LOGICAL_OP_PASS_H_

#include <string>

#include "oneflow/core/framework/framework.h"

namespace oneflow {

std::string NcclLogicalOpType1D(const std::string& src_sbp, const std::string& dst_sbp,
                                const Shape& logical_shape, int64_t parallel_num);

}  // namespace oneflow

#endif  // OFX_ONEFLOW_INSERT_NCCL_LOGICAL_OP_PASS_H_
