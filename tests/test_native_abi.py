"""The C-ABI from plain C: tests/native/abi_smoke.c is compiled with gcc against
include/ofx_spmm.h, linked to the built library and run (CPU entry points only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "of-spmm_amd", "oneflow_spmm")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not found")
def test_c_host_calls_the_abi(tmp_path):
    exe = tmp_path / "abi_smoke"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "abi_smoke.c"), "-o", str(exe),
                    "-L", LIBDIR, "-lofx_spmm", f"-Wl,-rpath,{LIBDIR}", "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")


CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ not found")
def test_cpu_kernels_under_sanitizers(tmp_path):
    """the host kernels (spmm_cpu.cpp, synth.cpp, errors.cpp) built from source
    with AddressSanitizer + UndefinedBehaviorSanitizer (host code only) and driven over the edge
    cases by tests/native/cpu_sanitize.cpp, which also checks their results against naive loops."""
    exe = tmp_path / "cpu_sanitize"
    csrc = os.path.join(ROOT, "of-spmm_amd", "csrc")
    subprocess.run([CLANG, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fopenmp",
                    "-ffp-contract=off", "-Wall", "-Werror", "-Wno-unknown-pragmas",
                    "-Wno-duplicate-decl-specifier", "-I", os.path.join(ROOT, "include"), "-I", csrc,
                    os.path.join(ROOT, "tests", "native", "cpu_sanitize.cpp"),
                    os.path.join(csrc, "spmm_cpu.cpp"), os.path.join(csrc, "synth.cpp"),
                    os.path.join(csrc, "errors.cpp"), "-o", str(exe)], check=True)
    supp = tmp_path / "lsan.supp"
    supp.write_text("leak:___kmp_allocate\n")  # the OpenMP runtime's own thread-pool state
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               LSAN_OPTIONS=f"suppressions={supp}", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK") and "runtime error" not in r.stderr, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists(CLANG) or shutil.which("make") is None,
                    reason="ROCm toolchain / make not found")
def test_host_path_under_sanitizers(tmp_path):
    """the whole library's host side under ASan + UBSan (`make asan`: HIP units
    host-only, nothing launched) driven by tests/native/host_sanitize.cpp — the OneFlow-mirror
    path of ofx_functional_spmm_csr_global on kCPU (inference, kernel choice, cache, Compute) for
    local / 1-D / 2-D placements, the fused, SDDMM, transpose and gathered ops; every form, lane
    layout, tuning entry and forced variant through ofx_spmm_csr_describe (including the r03ai
    patch's prefetching-form layouts) with its workspace against the query; the error paths,
    exceptions thrown inside Compute, and the versioned structs (an older 48-byte options block
    read past its end would be a heap overflow here)."""
    pkg = os.path.join(ROOT, "of-spmm_amd")
    jobs = str(min(os.cpu_count() or 1, 8))
    r = subprocess.run(["make", "-s", "-j", jobs, "-C", pkg, "asan"], capture_output=True, text=True,
                       timeout=1500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    supp = tmp_path / "lsan.supp"
    supp.write_text("leak:___kmp_allocate\n")  # the OpenMP runtime's own thread-pool state
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               LSAN_OPTIONS=f"suppressions={supp}", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(pkg, "build_asan", "host_sanitize")], capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert r.stdout.strip().splitlines()[-1].startswith("OK") and "runtime error" not in r.stderr, \
        r.stdout[-4000:] + r.stderr[-4000:]
