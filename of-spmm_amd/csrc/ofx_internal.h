// ofx_internal.h — error plumbing shared by every C-ABI translation unit.
// Mirrors the reference's split between recoverable op errors (Maybe<T> / CHECK_*_OR_RETURN,
// oneflow/core/common/maybe.h:331-350 -> Python exception) and fatal kernel CHECKs: at the
// C-ABI both become a status code plus a thread-local message (ofx_last_error()).
#ifndef OFX_INTERNAL_H_
#define OFX_INTERNAL_H_

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "ofx_spmm.h"

namespace ofx {
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();

// The boundary guard of every extern "C" entry: a C++ exception never crosses the C-ABI (it would
// std::terminate the host process); it becomes OFX_EINTERNAL (OFX_ENOMEM for bad_alloc) with its
// what() in ofx_last_error().  Usage: `{ return ofx::guarded(__func__, [&]() -> int { ... }); }`.
int guard_exception(const char* fn);  // called from a catch block: classifies the current exception
template <typename F>
inline int guarded(const char* fn, F&& body) noexcept {
  try {
    return body();
  } catch (...) {
    return guard_exception(fn);
  }
}

// Device-side error words (host-mapped, written by kernels with system-scope stores; spmm_plan.h
// raise_device_error): their device address, or NULL when no GPU is usable.
unsigned* device_error_words();
// OFX_OK, or OFX_EPLAN with its message when a kernel raised an error word since the last check
// (the words are cleared).  Every launching entry calls it first: the report comes at the next
// call, as a CUDA/HIP launch error surfaces at the next API call.
int take_device_error(const char* where);
// Test knobs (ofx_debug_set): the value of `knob`, or `dflt` when unset.
int64_t debug_knob(int knob, int64_t dflt);

// Versioned C-ABI structs (include/ofx_spmm.h).  The tag word (offset 4) is checked before
// struct_size is trusted: every struct of every layout is at least 8 bytes, and no unversioned
// layout holds OFX_STRUCT_MAGIC there (the round-4 options had the high half of an int64
// split_threshold; the round-5 descriptors dtype / device_type), so an unversioned caller is
// refused for certain, never misread.  Returns NULL when the struct is usable, else why not.
const char* versioned_struct_problem(const void* p, uint32_t min_size);
// A caller's options are read up to its struct_size (the fields it was compiled with), the rest
// are defaults; an untagged struct or a size below the first tagged layout is refused
// (OFX_EINVAL).  Tensor descriptors and placements are checked where they are read
// (functional/*.cpp) with versioned_struct_problem.
int read_options(const ofx_spmm_options* in, ofx_spmm_options* out, const char* fn);
}  // namespace ofx

// `opts` (a `const ofx_spmm_options*` parameter) is replaced by a checked copy of the caller's
// struct with the fields past its struct_size defaulted.
#define OFX_READ_OPTIONS(opts, fn)                                                 \
  ofx_spmm_options ofx_opts_copy_;                                                 \
  do {                                                                             \
    if (const int ofx_ro_ = ::ofx::read_options((opts), &ofx_opts_copy_, (fn))) return ofx_ro_; \
    (opts) = &ofx_opts_copy_;                                                      \
  } while (0)

#define OFX_TAKE_DEVICE_ERROR(where)                                    \
  do {                                                                  \
    if (const int ofx_de_ = ::ofx::take_device_error(where)) return ofx_de_; \
  } while (0)

#define OFX_HIP_CHECK(expr)                                                                 \
  do {                                                                                      \
    hipError_t ofx_e_ = (expr);                                                             \
    if (ofx_e_ != hipSuccess) {                                                             \
      (void)hipGetLastError(); /* reported here: not again at the next launch check */      \
      return ::ofx::fail(OFX_EDEVICE, "%s failed: %s (%s:%d)", #expr,                       \
                         hipGetErrorString(ofx_e_), __FILE__, __LINE__);                    \
    }                                                                                       \
  } while (0)

#define OFX_REQUIRE(cond, code, ...)              \
  do {                                            \
    if (!(cond)) return ::ofx::fail(code, __VA_ARGS__); \
  } while (0)

#endif  // OFX_INTERNAL_H_
