// op_generated.h — the declaration `oneflow_tblgen` would emit for the ODS entry of
// op "spmm_csr" (oneflow/ir/spmm_csr.td; generator tools/oneflow-tblgen/op_schema_header.inc:34-99).
#ifndef OFX_ONEFLOW_SHIM_OP_GENERATED_H_
#define OFX_ONEFLOW_SHIM_OP_GENERATED_H_

#include "oneflow/core/framework/framework.h"

namespace oneflow {

class SpmmCsrOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
  static Maybe<void> ModifyInputArg(const user_op::GetInputArgModifier& GetInputArgModifierFn,
                                    const user_op::UserOpConfWrapper& conf);
};

// Fused epilogue variant.
class FusedSpmmCsrOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
  static Maybe<void> ModifyInputArg(const user_op::GetInputArgModifier& GetInputArgModifierFn,
                                    const user_op::UserOpConfWrapper& conf);
};

// Gradient ops of spmm_csr.
class SddmmCsrOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
};

// d(b) of spmm_csr with A's values read through A^T's perm (learnable edge weights).
class SpmmCsrGatheredOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
  static Maybe<void> ModifyInputArg(const user_op::GetInputArgModifier& GetInputArgModifierFn,
                                    const user_op::UserOpConfWrapper& conf);
};

class CsrTransposeOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
};

// The S(0) -> B collectives the row-split op's B operand goes through: eager boxing
// (oneflow/user/ops/eager_nccl_ops.cpp:188-233) and the lazy graph's logical collective
// (oneflow/user/ops/nccl_logical_ops.cpp:104-142, ODS OneFlowUserOps.td:5341-5357).
class EagerCclAllGatherOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> InferPhysicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferNdSbp(user_op::InferNdSbpFnContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
};

class _ncclLogicalAllGatherOp {
 public:
  static Maybe<void> InferLogicalTensorDesc(user_op::InferContext* ctx);
  static Maybe<void> GetSbp(user_op::SbpContext* ctx);
  static Maybe<void> InferNdSbp(user_op::InferNdSbpFnContext* ctx);
  static Maybe<void> InferDataType(user_op::InferContext* ctx);
};

}  // namespace oneflow

#endif  // OFX_ONEFLOW_SHIM_OP_GENERATED_H_
