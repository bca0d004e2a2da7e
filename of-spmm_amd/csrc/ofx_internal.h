// ofx_internal.h — error plumbing shared by every C-ABI translation unit.
// Mirrors the reference's split between recoverable op errors (Maybe<T> / CHECK_*_OR_RETURN,
// oneflow/core/common/maybe.h:331-350 -> Python exception) and fatal kernel CHECKs: at the
// C-ABI both become a status code plus a thread-local message (ofx_last_error()).
#ifndef OFX_INTERNAL_H_
#define OFX_INTERNAL_H_

#include <stdarg.h>
#include <stdio.h>

#include "ofx_spmm.h"

namespace ofx {
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();
}  // namespace ofx

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
