// op_generated.cpp — the registration `oneflow_tblgen` would emit for op "spmm_csr"
// (pattern tools/oneflow-tblgen/op_schema_source.inc:32-100): inputs, outputs, typed attrs with
// their ODS defaults, and the static infer/SBP/dtype/input-modifier functions of SpmmCsrOp.
#include "oneflow/core/framework/op_generated.h"

namespace oneflow {

REGISTER_USER_OP("spmm_csr")
    .Input("a_csr_row_ptr")
    .Input("a_csr_col_idx")
    .Input("a_csr_values")
    .Input("b")
    .Output("out")
    .Attr<int64_t>("a_num_rows", 0)
    .Attr<int64_t>("a_num_cols", 0)
    .Attr<int64_t>("static_csr", 0)
    .SetLogicalTensorDescInferFn(SpmmCsrOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(SpmmCsrOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(SpmmCsrOp::GetSbp)
    .SetDataTypeInferFn(SpmmCsrOp::InferDataType)
    .SetInputArgModifyFn(SpmmCsrOp::ModifyInputArg);

REGISTER_USER_OP("fused_spmm_csr")
    .Input("a_csr_row_ptr")
    .Input("a_csr_col_idx")
    .Input("a_csr_values")
    .Input("b")
    .OptionalInput("bias")
    .Output("out")
    .Attr<int64_t>("a_num_rows", 0)
    .Attr<int64_t>("a_num_cols", 0)
    .Attr<bool>("relu", false)
    .Attr<int64_t>("static_csr", 0)
    .SetLogicalTensorDescInferFn(FusedSpmmCsrOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(FusedSpmmCsrOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(FusedSpmmCsrOp::GetSbp)
    .SetDataTypeInferFn(FusedSpmmCsrOp::InferDataType)
    .SetInputArgModifyFn(FusedSpmmCsrOp::ModifyInputArg);

REGISTER_USER_OP("sddmm_csr")
    .Input("a_csr_row_ptr")
    .Input("a_csr_col_idx")
    .Input("a")
    .Input("b")
    .Output("out")
    .Attr<int64_t>("a_num_rows", 0)
    .Attr<int64_t>("a_num_cols", 0)
    .Attr<int64_t>("static_csr", 0)
    .SetLogicalTensorDescInferFn(SddmmCsrOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(SddmmCsrOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(SddmmCsrOp::GetSbp)
    .SetDataTypeInferFn(SddmmCsrOp::InferDataType);

REGISTER_USER_OP("spmm_csr_gathered")
    .Input("a_csr_row_ptr")
    .Input("a_csr_col_idx")
    .Input("a_csr_values")
    .Input("values_perm")
    .Input("b")
    .Output("out")
    .Attr<int64_t>("a_num_rows", 0)
    .Attr<int64_t>("a_num_cols", 0)
    .Attr<int64_t>("static_csr", 0)
    .SetLogicalTensorDescInferFn(SpmmCsrGatheredOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(SpmmCsrGatheredOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(SpmmCsrGatheredOp::GetSbp)
    .SetDataTypeInferFn(SpmmCsrGatheredOp::InferDataType)
    .SetInputArgModifyFn(SpmmCsrGatheredOp::ModifyInputArg);

REGISTER_USER_OP("csr_transpose")
    .Input("a_csr_row_ptr")
    .Input("a_csr_col_idx")
    .Output("out_row_ptr")
    .Output("out_col_idx")
    .Output("out_perm")
    .Attr<int64_t>("a_num_rows", 0)
    .Attr<int64_t>("a_num_cols", 0)
    .SetLogicalTensorDescInferFn(CsrTransposeOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(CsrTransposeOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(CsrTransposeOp::GetSbp)
    .SetDataTypeInferFn(CsrTransposeOp::InferDataType);

REGISTER_USER_OP("eager_ccl_all_gather")
    .Input("in")
    .Output("out")
    .SetLogicalTensorDescInferFn(EagerCclAllGatherOp::InferLogicalTensorDesc)
    .SetPhysicalTensorDescInferFn(EagerCclAllGatherOp::InferPhysicalTensorDesc)
    .SetGetSbpFn(EagerCclAllGatherOp::GetSbp)
    .SetNdSbpInferFn(EagerCclAllGatherOp::InferNdSbp)
    .SetDataTypeInferFn(EagerCclAllGatherOp::InferDataType);

REGISTER_USER_OP("_nccl_logical_all_gather")
    .Input("in")
    .Output("out")
    .SetLogicalTensorDescInferFn(_ncclLogicalAllGatherOp::InferLogicalTensorDesc)
    .SetGetSbpFn(_ncclLogicalAllGatherOp::GetSbp)
    .SetNdSbpInferFn(_ncclLogicalAllGatherOp::InferNdSbp)
    .SetDataTypeInferFn(_ncclLogicalAllGatherOp::InferDataType);

}  // namespace oneflow
