// framework.cpp — implementation of the minimal OneFlow framework shim (framework.h).
#include "oneflow/core/framework/framework.h"

#include "ofx_spmm.h"

#include <new>
#include <stdexcept>

#include "ofx_internal.h"

namespace oneflow {

void TestHookCompute(const char* op_name) {
  switch (ofx::debug_knob(OFX_DEBUG_THROW_IN_COMPUTE, 0)) {
    case 1: throw std::runtime_error(std::string(op_name) + ": injected by OFX_DEBUG_THROW_IN_COMPUTE");
    case 2: throw std::bad_alloc();
    case 3: throw 42;  // not derived from std::exception
    default: break;
  }
}

const char* DataType_Name(DataType dt) {
  switch (dt) {
    case kChar: return "kChar";
    case kFloat: return "kFloat";
    case kDouble: return "kDouble";
    case kInt8: return "kInt8";
    case kInt32: return "kInt32";
    case kInt64: return "kInt64";
    case kUInt8: return "kUInt8";
    case kFloat16: return "kFloat16";
    case kBFloat16: return "kBFloat16";
    case kBool: return "kBool";
    default: return "kInvalidDataType";
  }
}

const char* DeviceTypeName(DeviceType t) {
  switch (t) {
    case DeviceType::kCPU: return "cpu";
    case DeviceType::kCUDA: return "cuda";
    case DeviceType::kHIP: return "hip";
    case DeviceType::kMockDevice: return "mock";
    default: return "invalid";
  }
}

std::string Shape::ToString() const {
  std::ostringstream os;
  os << "(";
  for (size_t i = 0; i < dims_.size(); ++i) os << (i ? "," : "") << dims_[i];
  if (dims_.size() == 1) os << ",";
  os << ")";
  return os.str();
}

BalancedSplitter::BalancedSplitter(int64_t total_num, int64_t split_num)
    : total_(total_num), parts_(split_num) {}

std::pair<int64_t, int64_t> BalancedSplitter::At(int64_t idx) const {
  int64_t b = 0, e = 0;
  ofx_balanced_range(total_, parts_, idx, &b, &e);
  return {b, e};
}

int64_t SplitAxisOf(const std::string& sbp) {
  if (sbp.size() >= 4 && sbp[0] == 'S' && sbp[1] == '(' && sbp.back() == ')')
    return std::stoll(sbp.substr(2, sbp.size() - 3));
  return -1;
}

namespace {
// Row-major multi-index of parallel_id in the hierarchy (NdIndexOffsetHelper::OffsetToNdIndex).
std::vector<int64_t> ParallelRank(const Shape& hierarchy, int64_t parallel_id) {
  std::vector<int64_t> rank(hierarchy.NumAxes());
  for (int64_t i = hierarchy.NumAxes() - 1; i >= 0; --i) {
    rank[i] = parallel_id % hierarchy.At(i);
    parallel_id /= hierarchy.At(i);
  }
  return rank;
}
}  // namespace

// Restates oneflow/core/job/nd_sbp_util.cpp:58-104 (GetTensorSliceView4ParallelRank/Id).
TensorSliceView GetTensorSliceView4ParallelId(const Shape& hierarchy, const NdSbp& nd_sbp,
                                              const Shape& logical_shape, int64_t parallel_id) {
  std::vector<Range> ranges;
  for (int64_t i = 0; i < logical_shape.NumAxes(); ++i) ranges.emplace_back(0, logical_shape.At(i));
  if (hierarchy.elem_cnt() == 1) return TensorSliceView(ranges);
  OFX_KERNEL_CHECK((int64_t)nd_sbp.size() == hierarchy.NumAxes(),
                   "nd_sbp has " << nd_sbp.size() << " entries for a " << hierarchy.NumAxes()
                                 << "-D hierarchy");
  const std::vector<int64_t> rank = ParallelRank(hierarchy, parallel_id);
  if (hierarchy.NumAxes() == 1) {
    const int64_t axis = SplitAxisOf(nd_sbp[0]);
    if (axis >= 0) {
      OFX_KERNEL_CHECK(axis < (int64_t)ranges.size(), "split axis " << axis << " out of range");
      OFX_KERNEL_CHECK(parallel_id >= 0 && parallel_id < hierarchy.elem_cnt(),
                       "parallel_id " << parallel_id << " out of range");
      const auto r = BalancedSplitter(logical_shape.At(axis), hierarchy.elem_cnt()).At(parallel_id);
      OFX_KERNEL_CHECK(r.second - r.first > 0, "empty slice for parallel_id " << parallel_id);
      ranges[axis] = Range(r.first, r.second);
    }
  } else {
    for (int64_t i = 0; i < hierarchy.NumAxes(); ++i) {
      const int64_t axis = SplitAxisOf(nd_sbp[i]);
      if (axis < 0) continue;
      OFX_KERNEL_CHECK(axis < (int64_t)ranges.size(), "split axis " << axis << " out of range");
      OFX_KERNEL_CHECK(ranges[axis].size() % hierarchy.At(i) == 0,
                       "axis " << axis << " size " << ranges[axis].size()
                               << " not divisible by hierarchy dim " << hierarchy.At(i));
      const int64_t size = ranges[axis].size() / hierarchy.At(i);
      const int64_t start = ranges[axis].begin() + rank[i] * size;
      ranges[axis] = Range(start, start + size);
    }
  }
  return TensorSliceView(ranges);
}

// Restates oneflow/core/operator/operator.cpp:1551-1626 (eager mode).
Maybe<void> GetPhysicalShape(const Shape& logical_shape, const NdSbp& nd_sbp,
                             const ParallelDesc& parallel_desc, const ParallelContext& parallel_ctx,
                             Shape* physical) {
  const Shape& hierarchy = *parallel_desc.hierarchy();
  const int64_t parallel_id = parallel_ctx.parallel_id();
  CHECK_GE_OR_RETURN(parallel_id, 0);
  CHECK_LT_OR_RETURN(parallel_id, hierarchy.elem_cnt());
  *physical = logical_shape;
  if (hierarchy.elem_cnt() == 1) return Maybe<void>::Ok();
  CHECK_EQ_OR_RETURN(hierarchy.NumAxes(), (int64_t)nd_sbp.size());
  if (hierarchy.NumAxes() == 1) {
    const int64_t axis = SplitAxisOf(nd_sbp[0]);
    if (axis >= 0 && logical_shape.At(axis) > 0) {
      CHECK_GE_OR_RETURN(logical_shape.At(axis), hierarchy.elem_cnt())
          << Error::RuntimeError() << "split axis " << axis << " of " << logical_shape.ToString()
          << " is smaller than the parallel num";
      const auto r = BalancedSplitter(logical_shape.At(axis), hierarchy.elem_cnt()).At(parallel_id);
      physical->Set(axis, r.second - r.first);
    }
    return Maybe<void>::Ok();
  }
  const std::vector<int64_t> rank = ParallelRank(hierarchy, parallel_id);
  for (int64_t i = 0; i < hierarchy.NumAxes(); ++i) {
    const int64_t axis = SplitAxisOf(nd_sbp[i]);
    if (axis < 0 || physical->At(axis) == 0) continue;
    CHECK_GE_OR_RETURN(physical->At(axis), hierarchy.At(i))
        << Error::RuntimeError() << "split axis " << axis << " of " << logical_shape.ToString()
        << " is smaller than hierarchy dim " << hierarchy.At(i);
    const auto r = BalancedSplitter(physical->At(axis), hierarchy.At(i)).At(rank[i]);
    physical->Set(axis, r.second - r.first);
  }
  return Maybe<void>::Ok();
}

namespace user_op {

UserOpRegistryMgr& UserOpRegistryMgr::Get() {
  static UserOpRegistryMgr mgr;
  return mgr;
}

Maybe<void> UserOpRegistryMgr::GetOpKernelRegistryResult(const std::string& op,
                                                         const KernelRegContext& ctx,
                                                         const OpKernelRegistryResult** out) const {
  const OpKernelRegistryResult* found = nullptr;
  int matched = 0;
  std::string tried;
  for (const auto& k : kernels_) {
    if (k.op_type_name != op) continue;
    tried += "\n  " + k.is_matched.debug;
    if (k.is_matched(ctx)) {
      found = &k;
      ++matched;
    }
  }
  if (matched == 0)
    return Maybe<void>("OpKernelNotFoundError",
                       "cannot find the kernel matching the current context: op " + op +
                           " on device " + DeviceTypeName(ctx.device_type()) +
                           " with dtype " + DataType_Name(ctx.dtype("out", 0)) +
                           "; registered kernels:" + tried);
  if (matched > 1)
    return Maybe<void>("MultipleOpKernelsMatchedError",
                       "there are more than one kernels matching the current context: op " + op);
  *out = found;
  return Maybe<void>::Ok();
}

}  // namespace user_op
}  // namespace oneflow
