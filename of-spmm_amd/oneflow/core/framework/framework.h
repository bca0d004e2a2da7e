// framework.h — minimal stand-in for the slice of OneFlow's framework API that op "spmm_csr"
// uses, so that oneflow/user/ops/spmm_op.cpp and oneflow/user/kernels/spmm_kernel.cpp compile
// and run here unmodified against the same names they use inside a real OneFlow tree
// (INTEGRATION.md).  Written from the interface's documented behaviour, not copied:
//   Maybe / CHECK_*_OR_RETURN   oneflow/core/common/maybe.h:331-350, just.h:110
//   DataType                    oneflow/core/common/data_type.proto:4-26
//   user_op::TensorDesc/Tensor  oneflow/core/framework/user_op_tensor.h:31-70
//   InferContext / SbpContext   oneflow/core/framework/infer_util.h, sbp_context.h
//   OpKernel / contexts         oneflow/core/framework/op_kernel.h:213-318
//   REGISTER_USER_KERNEL + HOB  oneflow/core/framework/user_op_registry_manager.h:81-84,
//                               user_op_kernel_registry.h:67-98, user_op_hob.h:43-66,
//                               unique-match rule user_op_registry_manager.cpp:83-120
//   BalancedSplitter            oneflow/core/common/balanced_splitter.cpp:20-40
// DeviceType gains kHIP: the MI355X kernel registers for it ("device identity").
#ifndef OFX_ONEFLOW_SHIM_FRAMEWORK_H_
#define OFX_ONEFLOW_SHIM_FRAMEWORK_H_

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "ofx_spmm.h"

namespace oneflow {

// ---- common ----------------------------------------------------------------------------------
enum DataType : int {
  kInvalidDataType = 0,
  kChar = 1,
  kFloat = 2,
  kDouble = 3,
  kInt8 = 4,
  kInt32 = 5,
  kInt64 = 6,
  kUInt8 = 7,
  kFloat16 = 9,
  kBFloat16 = 11,
  kBool = 12,
};
const char* DataType_Name(DataType dt);
inline bool IsIndexDataType(DataType dt) { return dt == kInt32 || dt == kInt64; }
// oneflow/core/common/data_type.h GetSizeOfDataType
inline size_t GetSizeOfDataType(DataType dt) {
  switch (dt) {
    case kChar: case kInt8: case kUInt8: case kBool: return 1;
    case kFloat16: case kBFloat16: return 2;
    case kFloat: case kInt32: return 4;
    case kDouble: case kInt64: return 8;
    default: return 0;
  }
}

enum class DeviceType : int { kInvalidDevice = 0, kCPU = 1, kCUDA = 2, kMockDevice = 3, kHIP = 4 };
const char* DeviceTypeName(DeviceType t);

class Shape {
 public:
  Shape() = default;
  Shape(std::initializer_list<int64_t> d) : dims_(d) {}
  explicit Shape(std::vector<int64_t> d) : dims_(std::move(d)) {}
  int64_t NumAxes() const { return (int64_t)dims_.size(); }
  int64_t At(int64_t i) const { return dims_.at(i); }
  void Set(int64_t i, int64_t v) { dims_.at(i) = v; }
  int64_t elem_cnt() const {
    int64_t c = 1;
    for (int64_t d : dims_) c *= d;
    return c;
  }
  int64_t Count(int64_t begin) const { return Count(begin, NumAxes()); }
  int64_t Count(int64_t begin, int64_t end) const {
    int64_t c = 1;
    for (int64_t i = begin; i < end; ++i) c *= dims_[i];
    return c;
  }
  const std::vector<int64_t>& dim_vec() const { return dims_; }
  bool operator==(const Shape& o) const { return dims_ == o.dims_; }
  std::string ToString() const;

 private:
  std::vector<int64_t> dims_;
};
using ShapeView = Shape;

// Error carrying Maybe<void> (only the void flavour is needed by this op).
class Error {
 public:
  static Error RuntimeError() { return Error("RuntimeError"); }
  static Error ValueError() { return Error("ValueError"); }
  static Error TypeError() { return Error("TypeError"); }
  explicit Error(std::string kind = "CheckFailedError") : kind_(std::move(kind)) {}
  const std::string& kind() const { return kind_; }

 private:
  std::string kind_;
};

template <typename T>
class Maybe;

template <>
class Maybe<void> {
 public:
  static Maybe<void> Ok() { return Maybe<void>(); }
  Maybe() = default;
  Maybe(std::string kind, std::string msg) : ok_(false), kind_(std::move(kind)), msg_(std::move(msg)) {}
  bool IsOk() const { return ok_; }
  const std::string& kind() const { return kind_; }
  const std::string& message() const { return msg_; }

 private:
  bool ok_ = true;
  std::string kind_, msg_;
};

class ErrorBuilder {
 public:
  ErrorBuilder(const char* file, int line, const char* expr) {
    loc_ << file << ":" << line << " check failed: " << expr << " ";
  }
  ErrorBuilder& operator<<(const Error& e) {
    kind_ = e.kind();
    return *this;
  }
  template <typename T>
  ErrorBuilder& operator<<(const T& v) {
    msg_ << v;
    return *this;
  }
  operator Maybe<void>() const { return Maybe<void>(kind_, msg_.str() + "  [" + loc_.str() + "]"); }

 private:
  std::string kind_ = "CheckFailedError";
  std::ostringstream msg_, loc_;
};

#define CHECK_OR_RETURN(cond) \
  if (!(cond)) return ::oneflow::ErrorBuilder(__FILE__, __LINE__, #cond)
#define OFX_CHECK_CMP_OR_RETURN_(a, b, op)                                                    \
  if (!((a)op(b)))                                                                            \
  return ::oneflow::ErrorBuilder(__FILE__, __LINE__, #a " " #op " " #b)                       \
         << "(" << (a) << " vs " << (b) << ") "
#define CHECK_EQ_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, ==)
#define CHECK_NE_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, !=)
#define CHECK_GE_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, >=)
#define CHECK_GT_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, >)
#define CHECK_LE_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, <=)
#define CHECK_LT_OR_RETURN(a, b) OFX_CHECK_CMP_OR_RETURN_(a, b, <)
#define CHECK_NOTNULL_OR_RETURN(p) CHECK_OR_RETURN((p) != nullptr)
#define JUST(expr)                                  \
  do {                                              \
    ::oneflow::Maybe<void> ofx_m_ = (expr);         \
    if (!ofx_m_.IsOk()) return ofx_m_;              \
  } while (0)

// Fatal kernel-side check (the reference's glog CHECK): throws, turned into a status code at
// the C-ABI (functional/spmm_functor.cpp).
struct KernelCheckError {
  std::string msg;
};
#define OFX_KERNEL_CHECK(cond, msg)                                                          \
  do {                                                                                       \
    if (!(cond)) {                                                                           \
      std::ostringstream ofx_os_;                                                            \
      ofx_os_ << __FILE__ << ":" << __LINE__ << " CHECK failed: " #cond " " << msg;          \
      throw ::oneflow::KernelCheckError{ofx_os_.str()};                                      \
    }                                                                                        \
  } while (0)

// Test hook of this stand-in (no OneFlow counterpart; INTEGRATION.md: define it empty in a
// OneFlow tree): the op kernels' Compute throws when ofx_debug_set(OFX_DEBUG_THROW_IN_COMPUTE)
// asks it to, so the tests can show that no exception crosses the C-ABI (ofx::guarded).
void TestHookCompute(const char* op_name);

template <typename T>
struct GetDataType;
template <>
struct GetDataType<float> {
  static constexpr DataType value = kFloat;
};
template <>
struct GetDataType<double> {
  static constexpr DataType value = kDouble;
};
template <>
struct GetDataType<int32_t> {
  static constexpr DataType value = kInt32;
};
template <>
struct GetDataType<int64_t> {
  static constexpr DataType value = kInt64;
};

class BalancedSplitter {
 public:
  BalancedSplitter(int64_t total_num, int64_t split_num);
  std::pair<int64_t, int64_t> At(int64_t idx) const;  // [begin, end)

 private:
  int64_t total_, parts_;
};

class ParallelContext {
 public:
  ParallelContext(int64_t id = 0, int64_t num = 1) : id_(id), num_(num) {}
  int64_t parallel_id() const { return id_; }
  int64_t parallel_num() const { return num_; }

 private:
  int64_t id_, num_;
};

// Placement (oneflow/core/job/parallel_desc.h): device type, hierarchy and, per parallel id, the
// (machine, device) it runs on (MachineId4ParallelId / DeviceId4ParallelId).  A 1-D placement of
// G devices is {G}; a 2-D one (e.g. nodes x devices) is {R, C}.  "Machine" is the process rank,
// as in OneFlow's multi-client mode; without explicit ids parallel id p is (p, p).
class ParallelDesc {
 public:
  explicit ParallelDesc(Shape hierarchy = Shape({1}))
      : hierarchy_(std::make_shared<const Shape>(std::move(hierarchy))) {}
  ParallelDesc(DeviceType device_type, std::vector<std::pair<int64_t, int64_t>> machine_device,
               Shape hierarchy = Shape())
      : hierarchy_(std::make_shared<const Shape>(
            hierarchy.NumAxes() ? std::move(hierarchy) : Shape({(int64_t)machine_device.size()}))),
        device_type_(device_type),
        machine_device_(std::move(machine_device)) {}
  std::shared_ptr<const Shape> hierarchy() const { return hierarchy_; }
  int64_t parallel_num() const { return hierarchy_->elem_cnt(); }
  DeviceType device_type() const { return device_type_; }
  int64_t MachineId4ParallelId(int64_t parallel_id) const {
    return machine_device_.empty() ? parallel_id : machine_device_.at(parallel_id).first;
  }
  int64_t DeviceId4ParallelId(int64_t parallel_id) const {
    return machine_device_.empty() ? parallel_id : machine_device_.at(parallel_id).second;
  }
  bool operator==(const ParallelDesc& o) const {
    return *hierarchy_ == *o.hierarchy_ && device_type_ == o.device_type_ &&
           machine_device_ == o.machine_device_;
  }

 private:
  std::shared_ptr<const Shape> hierarchy_;
  DeviceType device_type_ = DeviceType::kInvalidDevice;
  std::vector<std::pair<int64_t, int64_t>> machine_device_;
};

// NdSbp: one SbpParallel per hierarchy axis ("S(axis)", "B" or "P"; sbp_parallel.proto).
using NdSbp = std::vector<std::string>;
// Split axis of one SbpParallel, -1 when it is B or P.
int64_t SplitAxisOf(const std::string& sbp);

// [begin, end) of one axis of a tensor slice (oneflow/core/common/range.h).
class Range {
 public:
  Range(int64_t b = 0, int64_t e = 0) : b_(b), e_(e) {}
  int64_t begin() const { return b_; }
  int64_t end() const { return e_; }
  int64_t size() const { return e_ - b_; }
  int64_t& mut_begin() { return b_; }
  int64_t& mut_end() { return e_; }

 private:
  int64_t b_, e_;
};
class TensorSliceView {
 public:
  explicit TensorSliceView(std::vector<Range> r) : r_(std::move(r)) {}
  const Range& At(int64_t i) const { return r_.at(i); }
  int64_t NumAxes() const { return (int64_t)r_.size(); }

 private:
  std::vector<Range> r_;
};

// The slice of a logical tensor that parallel_id holds (oneflow/core/job/nd_sbp_util.cpp:58-104):
// 1-D hierarchy: BalancedSplitter over the split axis; N-D: each split hierarchy axis divides
// the current range evenly (CHECK: divisible).  Failed CHECKs throw KernelCheckError.
TensorSliceView GetTensorSliceView4ParallelId(const Shape& parallel_hierarchy, const NdSbp& nd_sbp,
                                              const Shape& logical_shape, int64_t parallel_id);
// Physical (per-rank) shape of a logical shape under nd_sbp (oneflow/core/operator/
// operator.cpp:1551-1626, eager flavour: nested BalancedSplitter per split hierarchy axis).
Maybe<void> GetPhysicalShape(const Shape& logical_shape, const NdSbp& nd_sbp,
                             const ParallelDesc& parallel_desc, const ParallelContext& parallel_ctx,
                             Shape* physical);

// ---- device layer (ep) ------------------------------------------------------------------------
namespace ep {
class Stream {
 public:
  virtual ~Stream() = default;
  virtual DeviceType device_type() const = 0;
  template <typename T>
  T* As() {
    return static_cast<T*>(this);
  }
};
class CpuStream final : public Stream {
 public:
  explicit CpuStream(int num_threads = 0) : num_threads_(num_threads) {}
  DeviceType device_type() const override { return DeviceType::kCPU; }
  int num_threads() const { return num_threads_; }

 private:
  int num_threads_;
};
// ep::CudaGraphExecutable for kHIP (ep/cuda/cuda_stream.h:41-56) over the C-ABI's hipGraph
// executable (device_shim.cpp): Update() patches the live executable in place when it can.
class HipGraphExecutable {
 public:
  HipGraphExecutable() { ofx_graph_exec_create(&exec_); }
  ~HipGraphExecutable() { ofx_graph_exec_destroy(exec_); }
  HipGraphExecutable(const HipGraphExecutable&) = delete;
  HipGraphExecutable& operator=(const HipGraphExecutable&) = delete;
  bool IsInstantiated() const {
    int yes = 0;
    ofx_graph_exec_stats(exec_, &yes, nullptr, nullptr, nullptr);
    return yes != 0;
  }
  int64_t updates() const {
    int64_t u = 0;
    ofx_graph_exec_stats(exec_, nullptr, nullptr, &u, nullptr);
    return u;
  }
  void* handle() const { return exec_; }

 private:
  void* exec_ = nullptr;
};

class HipStream final : public Stream {
 public:
  explicit HipStream(void* hip_stream, int device) : s_(hip_stream), device_(device) {}
  DeviceType device_type() const override { return DeviceType::kHIP; }
  void* hip_stream() const { return s_; }
  int device_index() const { return device_; }
  // CudaStream::BeginGraphCapture / EndGraphCapture / IsGraphCapturing / LaunchGraph
  // (cuda_stream.cpp:178-196); status codes instead of CHECKs (the C-ABI's error model).
  int BeginGraphCapture() { return ofx_stream_begin_capture(s_); }
  int EndGraphCapture(HipGraphExecutable* executable) {
    return ofx_stream_end_capture(s_, executable ? executable->handle() : nullptr);
  }
  bool IsGraphCapturing() const {
    int yes = 0;
    return ofx_stream_is_capturing(s_, &yes) == 0 && yes != 0;
  }
  int LaunchGraph(const HipGraphExecutable* executable) {
    return ofx_graph_launch(executable->handle(), s_);
  }

 private:
  void* s_;
  int device_;
};
}  // namespace ep

// ---- user_op -----------------------------------------------------------------------------------
namespace user_op {

struct OpArg {
  OpArg(std::string n, int32_t i) : name(std::move(n)), index(i) {}
  std::string name;
  int32_t index;
};

class TensorDesc {
 public:
  TensorDesc() = default;
  TensorDesc(Shape s, DataType dt) : shape_(std::move(s)), dtype_(dt) {}
  const Shape& shape() const { return shape_; }
  DataType data_type() const { return dtype_; }
  bool is_dynamic() const { return false; }
  void set_shape(const Shape& s) { shape_ = s; }
  void set_data_type(DataType dt) { dtype_ = dt; }

 private:
  Shape shape_;
  DataType dtype_ = kInvalidDataType;
};

class Tensor {
 public:
  Tensor(Shape s, DataType dt, void* p, int64_t row_stride = -1)
      : shape_(std::move(s)), dtype_(dt), p_(p), row_stride_(row_stride) {}
  ShapeView shape_view() const { return shape_; }
  DataType data_type() const { return dtype_; }
  // Row stride of a 2-D tensor in elements (== shape[1] when contiguous).
  int64_t row_stride() const { return row_stride_ >= 0 ? row_stride_ : shape_.At(shape_.NumAxes() - 1); }
  const void* raw_dptr() const { return p_; }
  void* mut_raw_dptr() { return p_; }
  template <typename T = void>
  const T* dptr() const {
    return static_cast<const T*>(p_);
  }
  template <typename T = void>
  T* mut_dptr() {
    return static_cast<T*>(p_);
  }

 private:
  Shape shape_;
  DataType dtype_;
  void* p_;
  int64_t row_stride_;
};

using AttrMap = std::map<std::string, int64_t>;

class InferContext {
 public:
  InferContext(std::map<std::pair<std::string, int32_t>, TensorDesc> in, AttrMap attrs)
      : in_(std::move(in)), attrs_(std::move(attrs)) {}
  const TensorDesc& InputTensorDesc(const std::string& n, int32_t i) const { return in_.at({n, i}); }
  // optional inputs (oneflow/core/framework/infer_util.h:71)
  bool has_input(const std::string& n, int32_t i) const { return in_.count({n, i}) > 0; }
  const Shape& InputShape(const std::string& n, int32_t i) const { return in_.at({n, i}).shape(); }
  DataType InputDType(const std::string& n, int32_t i) const { return in_.at({n, i}).data_type(); }
  TensorDesc* MutOutputTensorDesc(const std::string& n, int32_t i) { return &out_[{n, i}]; }
  void SetOutputShape(const std::string& n, int32_t i, const Shape& s) { out_[{n, i}].set_shape(s); }
  void SetOutputDType(const std::string& n, int32_t i, DataType dt) { out_[{n, i}].set_data_type(dt); }
  template <typename T>
  T Attr(const std::string& n) const {
    return static_cast<T>(attrs_.at(n));
  }
  const TensorDesc& OutputTensorDesc(const std::string& n, int32_t i) const { return out_.at({n, i}); }

  // Placement of a global op (physical inference; oneflow/core/framework/infer_util.h:50,84-93).
  // Without SetParallel the op is local: one device, every argument B.
  void SetParallel(ParallelContext pc, ParallelDesc pd, std::map<std::string, NdSbp> nd_sbp,
                   std::map<std::string, TensorDesc> logical) {
    pc_ = pc;
    pd_ = std::move(pd);
    nd_sbp_ = std::move(nd_sbp);
    logical_ = std::move(logical);
  }
  const ParallelContext& parallel_ctx() const { return pc_; }
  const ParallelDesc& parallel_desc() const { return pd_; }
  const NdSbp& NdSbp4ArgNameAndIndex(const std::string& n, int32_t) const {
    auto it = nd_sbp_.find(n);
    return it == nd_sbp_.end() ? broadcast_ : it->second;
  }
  const TensorDesc* LogicalTensorDesc4ArgNameAndIndex(const std::string& n, int32_t) const {
    auto it = logical_.find(n);
    return it == logical_.end() ? nullptr : &it->second;
  }

 private:
  std::map<std::pair<std::string, int32_t>, TensorDesc> in_, out_;
  AttrMap attrs_;
  ParallelContext pc_;
  ParallelDesc pd_;
  std::map<std::string, NdSbp> nd_sbp_;
  std::map<std::string, TensorDesc> logical_;
  NdSbp broadcast_{"B"};
};

// oneflow/core/framework/infer_nd_sbp_fn_context.h: an op's NdSbp inference (the eager S(0)->B
// boxing ops and the logical collectives fix their in/out NdSbp here).  String-list attributes
// (e.g. "src_reduced_nd_sbp") live next to the integer ones.
class InferNdSbpFnContext {
 public:
  InferNdSbpFnContext(Shape hierarchy, std::map<std::string, NdSbp> hints,
                      std::map<std::string, std::vector<std::string>> str_attrs = {})
      : hierarchy_(std::move(hierarchy)), hints_(std::move(hints)), str_attrs_(std::move(str_attrs)) {}
  const Shape& parallel_hierarchy() const { return hierarchy_; }
  const NdSbp& NdSbpHint4InputArgNameAndIndex(const std::string& n, int32_t) const {
    auto it = hints_.find(n);
    return it == hints_.end() ? empty_ : it->second;
  }
  NdSbp* NdSbp4ArgNameAndIndex(const std::string& n, int32_t) { return &nd_sbp_[n]; }
  const NdSbp& NdSbp4ArgName(const std::string& n) const { return nd_sbp_.at(n); }
  template <typename T>
  T Attr(const std::string& n) const {
    static_assert(std::is_same<T, std::vector<std::string>>::value, "string-list attrs only");
    return str_attrs_.at(n);
  }

 private:
  Shape hierarchy_;
  std::map<std::string, NdSbp> hints_, nd_sbp_;
  std::map<std::string, std::vector<std::string>> str_attrs_;
  NdSbp empty_;
};

// One SBP signature: per argument "S(axis)", "B" or "P".
using SbpSignature = std::vector<std::pair<std::string, std::string>>;

class SbpSignatureBuilder {
 public:
  explicit SbpSignatureBuilder(std::vector<SbpSignature>* out) : out_(out) {}
  SbpSignatureBuilder& Split(const OpArg& a, int64_t axis) {
    sig_.emplace_back(a.name, "S(" + std::to_string(axis) + ")");
    return *this;
  }
  SbpSignatureBuilder& Broadcast(const OpArg& a) {
    sig_.emplace_back(a.name, "B");
    return *this;
  }
  SbpSignatureBuilder& PartialSum(const OpArg& a) {
    sig_.emplace_back(a.name, "P");
    return *this;
  }
  void Build() { out_->push_back(sig_); }

 private:
  std::vector<SbpSignature>* out_;
  SbpSignature sig_;
};

// user_op_conf() of an SbpContext: which (optional) inputs the op instance has
// (oneflow/core/framework/user_op_conf.h:58).
class UserOpConfView {
 public:
  explicit UserOpConfView(std::vector<std::string> present = {}) : present_(std::move(present)) {}
  bool has_input(const std::string& n, int32_t) const {
    for (const auto& p : present_)
      if (p == n) return true;
    return false;
  }

 private:
  std::vector<std::string> present_;
};

class SbpContext {
 public:
  SbpContext() = default;
  explicit SbpContext(UserOpConfView conf) : conf_(std::move(conf)) {}
  const UserOpConfView& user_op_conf() const { return conf_; }
  SbpSignatureBuilder NewBuilder() { return SbpSignatureBuilder(&sigs_); }
  const std::vector<SbpSignature>& signatures() const { return sigs_; }

 private:
  std::vector<SbpSignature> sigs_;
  UserOpConfView conf_;
};

struct InputArgModifier {
  bool requires_grad = true;
  void set_requires_grad(bool v) { requires_grad = v; }
};
using GetInputArgModifier = std::function<InputArgModifier*(const std::string&, int32_t)>;
class UserOpConfWrapper {};

class OpKernelState {
 public:
  virtual ~OpKernelState() = default;
};
class OpKernelCache {
 public:
  virtual ~OpKernelCache() = default;
};

// oneflow/core/framework/op_kernel.h:40-60 (KernelCacheContext / KernelInitContext).
class KernelCacheContext {
 public:
  KernelCacheContext(ParallelContext pc, ParallelDesc pd, std::map<std::string, NdSbp> nd_sbp,
                     std::map<std::string, TensorDesc> logical, DeviceType dev)
      : pc_(pc), pd_(std::move(pd)), nd_sbp_(std::move(nd_sbp)), logical_(std::move(logical)),
        dev_(dev) {}
  const ParallelContext& parallel_ctx() const { return pc_; }
  const ParallelDesc& parallel_desc() const { return pd_; }
  DeviceType device_type() const { return dev_; }
  const NdSbp& NdSbp4ArgNameAndIndex(const std::string& n, int32_t) const {
    auto it = nd_sbp_.find(n);
    return it == nd_sbp_.end() ? broadcast_ : it->second;
  }
  const TensorDesc* LogicalTensorDesc4ArgNameAndIndex(const std::string& n, int32_t) const {
    return &logical_.at(n);
  }

 private:
  ParallelContext pc_;
  ParallelDesc pd_;
  std::map<std::string, NdSbp> nd_sbp_;
  std::map<std::string, TensorDesc> logical_;
  DeviceType dev_;
  NdSbp broadcast_{"B"};
};

class KernelComputeContext {
 public:
  KernelComputeContext(ep::Stream* s, std::map<std::pair<std::string, int32_t>, Tensor*> t,
                       AttrMap attrs, DeviceType dev)
      : s_(s), t_(std::move(t)), attrs_(std::move(attrs)), dev_(dev) {}
  Tensor* Tensor4ArgNameAndIndex(const std::string& n, int32_t i) {
    auto it = t_.find({n, i});
    return it == t_.end() ? nullptr : it->second;
  }
  ep::Stream* stream() { return s_; }
  DeviceType device_type() const { return dev_; }
  template <typename T>
  T Attr(const std::string& n) const {
    return static_cast<T>(attrs_.at(n));
  }
  const ParallelContext& parallel_ctx() const { return pc_; }
  void set_parallel_ctx(ParallelContext pc) { pc_ = pc; }

 private:
  ParallelContext pc_;
  ep::Stream* s_;
  std::map<std::pair<std::string, int32_t>, Tensor*> t_;
  AttrMap attrs_;
  DeviceType dev_;
};

// oneflow/core/framework/op_kernel.h:62-88 (KernelInitContext): what CreateOpKernelState sees.
class KernelInitContext {
 public:
  KernelInitContext(ParallelContext pc, ParallelDesc pd, DeviceType dev,
                    std::string stream_name_hint = "")
      : pc_(pc), pd_(std::move(pd)), dev_(dev), stream_name_hint_(std::move(stream_name_hint)) {}
  const ParallelContext& parallel_ctx() const { return pc_; }
  const ParallelDesc& parallel_desc() const { return pd_; }
  DeviceType device_type() const { return dev_; }
  bool has_stream_name_hint() const { return !stream_name_hint_.empty(); }
  const std::string& stream_name_hint() const { return stream_name_hint_; }

 private:
  ParallelContext pc_;
  ParallelDesc pd_;
  DeviceType dev_;
  std::string stream_name_hint_;
};

class OpKernel {
 public:
  virtual ~OpKernel() = default;
  virtual std::shared_ptr<OpKernelState> CreateOpKernelState(KernelInitContext*) const {
    return nullptr;
  }
  virtual std::shared_ptr<OpKernelCache> InitOpKernelCache(KernelCacheContext*) const {
    return nullptr;
  }
  virtual void Compute(KernelComputeContext* ctx, OpKernelState*, const OpKernelCache*) const {
    Compute(ctx);
  }
  virtual void Compute(KernelComputeContext*) const {}
  virtual bool AlwaysComputeWhenAllOutputsEmpty() const = 0;
};
class CudaGraphSupport {};  // marker, as user_op::CudaGraphSupport (captures fine in hipGraphs)

// ---- kernel registry + HOB predicates ----------------------------------------------------------
struct KernelRegContext {
  DeviceType device_type_ = DeviceType::kInvalidDevice;
  std::map<std::pair<std::string, int32_t>, DataType> dtypes;
  DeviceType device_type() const { return device_type_; }
  DataType dtype(const std::string& n, int32_t i) const {
    auto it = dtypes.find({n, i});
    return it == dtypes.end() ? kInvalidDataType : it->second;
  }
};
struct Hob {
  std::function<bool(const KernelRegContext&)> f;
  std::string debug;
  bool operator()(const KernelRegContext& c) const { return f(c); }
};
inline Hob operator&&(const Hob& a, const Hob& b) {
  return Hob{[a, b](const KernelRegContext& c) { return a(c) && b(c); }, a.debug + " && " + b.debug};
}
struct HobDeviceTypeProxy {
  Hob operator==(DeviceType t) const {
    return Hob{[t](const KernelRegContext& c) { return c.device_type() == t; },
               std::string("device_type == ") + DeviceTypeName(t)};
  }
};
inline HobDeviceTypeProxy HobDeviceType() { return {}; }
struct HobDataTypeProxy {
  std::string n;
  int32_t i;
  Hob operator==(DataType dt) const {
    auto nn = n;
    auto ii = i;
    return Hob{[nn, ii, dt](const KernelRegContext& c) { return c.dtype(nn, ii) == dt; },
               "data_type(" + n + ") == " + DataType_Name(dt)};
  }
};
inline HobDataTypeProxy HobDataType(const std::string& n, int32_t i) { return {n, i}; }
// hob::make_custom (oneflow/core/framework/user_op_hob.h): a named predicate on the context.
inline Hob make_custom(const std::string& name, std::function<bool(const KernelRegContext&)> f) {
  return Hob{std::move(f), name};
}

struct InferSizeContext {
  std::map<std::pair<std::string, int32_t>, TensorDesc> descs;
  AttrMap attrs;
  std::map<std::string, TensorDesc> logical;  // of a global op (empty for a local one)
  const TensorDesc& InputTensorDesc(const std::string& n, int32_t i) const { return descs.at({n, i}); }
  const TensorDesc* LogicalTensorDesc4ArgNameAndIndex(const std::string& n, int32_t) const {
    auto it = logical.find(n);
    return it == logical.end() ? nullptr : &it->second;
  }
  template <typename T>
  T Attr(const std::string& n) const {
    return static_cast<T>(attrs.at(n));
  }
};

struct OpKernelRegistryResult {
  std::string op_type_name;
  std::function<OpKernel*()> create_fn;
  Hob is_matched;
  std::function<size_t(InferSizeContext*)> infer_tmp_size;
};

class OpKernelRegistry {
 public:
  explicit OpKernelRegistry(std::string op) { r_.op_type_name = std::move(op); }
  template <typename K>
  OpKernelRegistry& SetCreateFn() {
    r_.create_fn = []() -> OpKernel* { return new K(); };
    return *this;
  }
  OpKernelRegistry& SetIsMatchedHob(Hob h) {
    r_.is_matched = std::move(h);
    return *this;
  }
  OpKernelRegistry& SetInferTmpSizeFn(std::function<size_t(InferSizeContext*)> f) {
    r_.infer_tmp_size = std::move(f);
    return *this;
  }
  const OpKernelRegistryResult& result() const { return r_; }

 private:
  OpKernelRegistryResult r_;
};

// Op schema registration (what the ODS tblgen output registers in op_generated.cpp).
struct OpRegistryResult {
  std::string op_type_name;
  std::vector<std::string> inputs, optional_inputs, outputs;
  std::vector<std::pair<std::string, int64_t>> attrs;  // name, default
  std::function<Maybe<void>(InferContext*)> logical_infer, physical_infer, dtype_infer;
  std::function<Maybe<void>(SbpContext*)> get_sbp;
  std::function<Maybe<void>(const GetInputArgModifier&, const UserOpConfWrapper&)> input_modify;
  std::function<Maybe<void>(InferNdSbpFnContext*)> nd_sbp_infer;
};
class OpRegistry {
 public:
  explicit OpRegistry(std::string op) { r_.op_type_name = std::move(op); }
  OpRegistry& Input(const std::string& n) {
    r_.inputs.push_back(n);
    return *this;
  }
  OpRegistry& OptionalInput(const std::string& n) {
    r_.optional_inputs.push_back(n);
    return *this;
  }
  OpRegistry& Output(const std::string& n) {
    r_.outputs.push_back(n);
    return *this;
  }
  template <typename T>
  OpRegistry& Attr(const std::string& n, T dflt = T()) {
    r_.attrs.emplace_back(n, (int64_t)dflt);
    return *this;
  }
  OpRegistry& SetLogicalTensorDescInferFn(std::function<Maybe<void>(InferContext*)> f) {
    r_.logical_infer = std::move(f);
    return *this;
  }
  OpRegistry& SetPhysicalTensorDescInferFn(std::function<Maybe<void>(InferContext*)> f) {
    r_.physical_infer = std::move(f);
    return *this;
  }
  OpRegistry& SetDataTypeInferFn(std::function<Maybe<void>(InferContext*)> f) {
    r_.dtype_infer = std::move(f);
    return *this;
  }
  OpRegistry& SetNdSbpInferFn(std::function<Maybe<void>(InferNdSbpFnContext*)> f) {
    r_.nd_sbp_infer = std::move(f);
    return *this;
  }
  OpRegistry& SetGetSbpFn(std::function<Maybe<void>(SbpContext*)> f) {
    r_.get_sbp = std::move(f);
    return *this;
  }
  OpRegistry& SetInputArgModifyFn(
      std::function<Maybe<void>(const GetInputArgModifier&, const UserOpConfWrapper&)> f) {
    r_.input_modify = std::move(f);
    return *this;
  }
  const OpRegistryResult& result() const { return r_; }

 private:
  OpRegistryResult r_;
};

class UserOpRegistryMgr {
 public:
  static UserOpRegistryMgr& Get();
  OpKernelRegistry CheckAndGetOpKernelRegistry(const std::string& op) { return OpKernelRegistry(op); }
  OpRegistry CheckAndGetOpRegistry(const std::string& op) { return OpRegistry(op); }
  void Register(const OpKernelRegistry& r) { kernels_.push_back(r.result()); }
  void Register(const OpRegistry& r) { ops_[r.result().op_type_name] = r.result(); }
  const OpRegistryResult* GetOpRegistryResult(const std::string& op) const {
    auto it = ops_.find(op);
    return it == ops_.end() ? nullptr : &it->second;
  }
  // Exactly-one-match rule: 0 -> OpKernelNotFoundError, >1 -> MultipleOpKernelsMatchedError.
  Maybe<void> GetOpKernelRegistryResult(const std::string& op, const KernelRegContext& ctx,
                                        const OpKernelRegistryResult** out) const;

 private:
  std::vector<OpKernelRegistryResult> kernels_;
  std::map<std::string, OpRegistryResult> ops_;
};

template <typename R>
struct UserOpRegisterTrigger {
  UserOpRegisterTrigger(R& r) { UserOpRegistryMgr::Get().Register(r); }  // NOLINT
};

}  // namespace user_op

namespace hob = user_op;  // hob::... spelling used by some reference kernels

}  // namespace oneflow

#define OFX_PP_CAT_(a, b) a##b
#define OFX_PP_CAT(a, b) OFX_PP_CAT_(a, b)
#define REGISTER_USER_KERNEL(name)                                                        \
  static ::oneflow::user_op::UserOpRegisterTrigger<::oneflow::user_op::OpKernelRegistry> \
      OFX_PP_CAT(g_register_trigger, __COUNTER__) =                                      \
          ::oneflow::user_op::UserOpRegistryMgr::Get().CheckAndGetOpKernelRegistry(name)
#define REGISTER_USER_OP(name)                                                     \
  static ::oneflow::user_op::UserOpRegisterTrigger<::oneflow::user_op::OpRegistry> \
      OFX_PP_CAT(g_register_trigger, __COUNTER__) =                               \
          ::oneflow::user_op::UserOpRegistryMgr::Get().CheckAndGetOpRegistry(name)

#endif  // OFX_ONEFLOW_SHIM_FRAMEWORK_H_
