// errors.cpp — thread-local last-error buffer behind ofx_last_error(), the exception guard of the
// C-ABI entries and the test knobs (ofx_debug_set).
#include <string.h>

#include <cstring>

#include <atomic>
#include <exception>
#include <new>
#include <stdexcept>

#include "ofx_internal.h"

namespace {
thread_local char g_last_error[1024] = {0};

constexpr int kKnobs = 8;
std::atomic<int64_t> g_knob[kKnobs];
std::atomic<bool> g_knob_set[kKnobs];
}  // namespace

namespace ofx {
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}
void clear_error() { g_last_error[0] = 0; }

int guard_exception(const char* fn) {
  try {
    throw;  // the exception being handled by the caller's catch (...)
  } catch (const std::bad_alloc& e) {
    return fail(OFX_ENOMEM, "%s: out of host memory (%s)", fn, e.what());
  } catch (const std::exception& e) {
    return fail(OFX_EINTERNAL, "%s: unexpected C++ exception: %s", fn, e.what());
  } catch (...) {
    return fail(OFX_EINTERNAL, "%s: unexpected non-standard C++ exception", fn);
  }
}

const char* versioned_struct_problem(const void* p, uint32_t min_size) {
  if (p == nullptr) return nullptr;
  uint32_t head[2];  // struct_size, magic: as bytes (the caller's struct may be a shorter layout)
  std::memcpy(head, p, sizeof(head));
  if (head[1] != OFX_STRUCT_MAGIC)
    return "has no OFX_STRUCT_MAGIC tag: an unversioned caller, or a struct not initialised with "
           "its OFX_*_INIT macro";
  if (head[0] < min_size) return "has a struct_size below the first tagged layout";
  return nullptr;
}

int read_options(const ofx_spmm_options* in, ofx_spmm_options* out, const char* fn) {
  std::memset(out, 0, sizeof(*out));
  out->struct_size = sizeof(*out);
  out->magic = OFX_STRUCT_MAGIC;
  if (in == nullptr) return OFX_OK;  // every field at its default
  if (const char* why = versioned_struct_problem(in, OFX_SPMM_OPTIONS_MIN_SIZE)) {
    uint32_t head[2];
    std::memcpy(head, in, sizeof(head));
    return fail(OFX_EINVAL,
                "%s: ofx_spmm_options %s (struct_size %u, tag 0x%08x; the first tagged layout is "
                "%u bytes): initialise the struct with OFX_SPMM_OPTIONS_INIT",
                fn, why, head[0], head[1], OFX_SPMM_OPTIONS_MIN_SIZE);
  }
  uint32_t size = 0;
  std::memcpy(&size, in, sizeof(size));
  std::memcpy(out, in, size < sizeof(*out) ? size : sizeof(*out));
  out->struct_size = sizeof(*out);
  return OFX_OK;
}

int64_t debug_knob(int knob, int64_t dflt) {
  if (knob <= 0 || knob >= kKnobs || !g_knob_set[knob].load(std::memory_order_relaxed)) return dflt;
  return g_knob[knob].load(std::memory_order_relaxed);
}
}  // namespace ofx

extern "C" const char* ofx_last_error(void) { return g_last_error; }
#ifdef OFX_TUNING_TABLE
extern "C" const char* ofx_version(void) { return "ofx-spmm 0.3.0 gfx950+tuning"; }
#else
extern "C" const char* ofx_version(void) { return "ofx-spmm 0.3.0 gfx950"; }
#endif

extern "C" int ofx_debug_set(int knob, int64_t value) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(knob > 0 && knob < kKnobs, OFX_EINVAL, "debug_set: unknown knob %d", knob);
    g_knob[knob].store(value, std::memory_order_relaxed);
    g_knob_set[knob].store(value >= 0, std::memory_order_relaxed);  // < 0: back to the default
    return OFX_OK;
  });
}
