// dbg_bounds.h — the opt-in bounds-checked build of the forward kernels (OFX_DEBUG_BOUNDS).
//
// A fault in a hand-written kernel can take a GPU box down, and the pool's tooling (no GPU
// sanitizer, no debugger) reports only an address afterwards.  This build checks every global
// access of the forward path (plan, main, small form, reduce) against the allocations of its
// launch BEFORE it is made: an access outside all of them is skipped (a load returns 0) and
// recorded, so the kernel cannot fault, and the host reads the first violation (site = file tag
// * 100000 + line, address, size, block, thread, launch tag) through ofx_debug_bounds_read().
// Buffer loads of B are range-checked by the hardware and cannot fault; the global-load form of
// B is checked like any other access.
//
// Release builds compile every check away (OFX_LD(p) is `*(p)`, OFX_ST(p, v) is `*(p) = v`): the
// kernels are unchanged.  Build: `make -C of-spmm_amd debug` -> oneflow_spmm/libofx_spmm_dbg.so,
// selected with OFX_SPMM_LIB (scripts/debug_bounds.py).
#ifndef OFX_DBG_BOUNDS_H_
#define OFX_DBG_BOUNDS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#define OFX_DBG_IMPL 1  // file tags of the sites: spmm_csr_impl.h
#define OFX_DBG_PLAN 2  // spmm_plan.h

namespace ofx {
namespace dbg {

constexpr int kRanges = 12;
constexpr int kHitWords = 8;  // count, site, address, bytes, block, thread, launch tag, spare

struct Range {
  uint64_t lo, hi;  // [lo, hi) in bytes
};
struct Bounds {
  Range r[kRanges];
  int n;                    // 0: no launch registered in this translation unit -> unchecked
  unsigned long long* hit;  // kHitWords device words (ofx_debug_bounds_read)
  unsigned long long tag;   // the launch's configuration, recorded with the hit
};

#ifdef OFX_DEBUG_BOUNDS
namespace {
// one copy per translation unit (-fno-gpu-rdc): every launch sets the copy of the TU it runs in
__device__ Bounds g_bounds;

__device__ __attribute__((noinline)) bool check(const void* p, uint64_t bytes, int site) {
  const int n = g_bounds.n;
  if (n == 0) return true;
  const uint64_t a = (uint64_t)p;
  for (int i = 0; i < n; ++i)
    if (a >= g_bounds.r[i].lo && a + bytes <= g_bounds.r[i].hi) return true;
  unsigned long long* h = g_bounds.hit;
  if (h != nullptr && atomicAdd(h, 1ull) == 0) {
    h[1] = (unsigned long long)site;
    h[2] = a;
    h[3] = bytes;
    h[4] = blockIdx.x;
    h[5] = threadIdx.x;
    h[6] = g_bounds.tag;
  }
  return false;
}
}  // namespace
#endif

}  // namespace dbg

// A checked access of `bytes` at p (line = the caller's line): always true in release builds.
template <int TAG = OFX_DBG_IMPL>
__device__ __forceinline__ bool dok(const void* p, uint64_t bytes, int line = __builtin_LINE()) {
#ifdef OFX_DEBUG_BOUNDS
  return dbg::check(p, bytes, TAG * 100000 + line);
#else
  (void)p, (void)bytes, (void)line;
  return true;
#endif
}
// A checked global load / store: exactly `*p` / `*p = v` in release builds.
template <int TAG = OFX_DBG_IMPL, typename X>
__device__ __forceinline__ X dld(const X* p, int line = __builtin_LINE()) {
#ifdef OFX_DEBUG_BOUNDS
  if (!dbg::check(p, sizeof(X), TAG * 100000 + line)) return X{};
#else
  (void)line;
#endif
  return *p;
}
template <int TAG = OFX_DBG_IMPL, typename X>
__device__ __forceinline__ void dst(X* p, const X& v, int line = __builtin_LINE()) {
#ifdef OFX_DEBUG_BOUNDS
  if (!dbg::check(p, sizeof(X), TAG * 100000 + line)) return;
#else
  (void)line;
#endif
  *p = v;
}

// The kernels' spelling: a plain dereference in release builds (identical code), the checked
// form in OFX_DEBUG_BOUNDS builds.  OFX_LD / OFX_ST for spmm_csr_impl.h, OFX_LDP / OFX_STP for
// spmm_plan.h.
#ifdef OFX_DEBUG_BOUNDS
#define OFX_LD(p) ::ofx::dld<OFX_DBG_IMPL>((p), __LINE__)
#define OFX_ST(p, v) ::ofx::dst<OFX_DBG_IMPL>((p), (v), __LINE__)
#define OFX_LDP(p) ::ofx::dld<OFX_DBG_PLAN>((p), __LINE__)
#define OFX_STP(p, v) ::ofx::dst<OFX_DBG_PLAN>((p), (v), __LINE__)
#define OFX_DOK(p, bytes) ::ofx::dok<OFX_DBG_IMPL>((p), (bytes), __LINE__)
#else
#define OFX_LD(p) (*(p))
#define OFX_ST(p, v) (void)(*(p) = (v))
#define OFX_LDP(p) (*(p))
#define OFX_STP(p, v) (void)(*(p) = (v))
#define OFX_DOK(p, bytes) true
#endif

#ifdef OFX_DEBUG_BOUNDS
// Host side: the hit words (spmm_csr.hip, allocated once) and a launch's allocations.
unsigned long long* dbg_hit_words();
namespace dbg {
namespace {
struct HostBounds {
  Bounds b{};
  void add(const void* p, uint64_t bytes) {
    if (p != nullptr && bytes > 0 && b.n < kRanges) {
      b.r[b.n].lo = (uint64_t)p;
      b.r[b.n].hi = (uint64_t)p + bytes;
      ++b.n;
    }
  }
  // publishes this TU's copy on `s` (stream-ordered before the launch's kernels)
  int publish(hipStream_t s, unsigned long long tag) {
    b.hit = dbg_hit_words();
    b.tag = tag;
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(g_bounds), &b, sizeof(Bounds), 0,
                                  hipMemcpyHostToDevice, s) == hipSuccess ? 0 : 1;
  }
};
}  // namespace
}  // namespace dbg
#endif

}  // namespace ofx

#endif  // OFX_DBG_BOUNDS_H_
