// ccl_boxing_function.h — eager boxing "ccl-s-to-b" for the shim (oneflow/core/boxing/
// ccl_boxing_function.cpp:104-122 check, :185-215 run): an S(0) tensor of a placement becomes B
// by op eager_ccl_all_gather, dispatched through the op and kernel registries like any user op.
#ifndef OFX_ONEFLOW_CCL_BOXING_FUNCTION_H_
#define OFX_ONEFLOW_CCL_BOXING_FUNCTION_H_

#include "oneflow/core/framework/framework.h"

namespace oneflow {

struct PlacedNdSbp {
  NdSbp nd_sbp;
  ParallelDesc placement;
};

// The reference's RawCheckCclS2B: 1-D S(0) -> B on one placement, logical dim 0 divisible by the
// parallel number (the padded shards of a K % G != 0 operand are the row-split wrapper's job),
// and an eager_ccl_all_gather kernel registered for the device type.
Maybe<void> CheckCclS2B(const PlacedNdSbp& in, const PlacedNdSbp& out, const Shape& logical_shape);

// Runs the boxing on this rank: `in` is its physical S(0) slice, `out` the full B tensor.
Maybe<void> CclS2B(ep::Stream* stream, const user_op::Tensor& in, user_op::Tensor* out,
                   const PlacedNdSbp& in_p, const PlacedNdSbp& out_p, const Shape& logical_shape,
                   int64_t parallel_id);

}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_BOXING_FUNCTION_H_
