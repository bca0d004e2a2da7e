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
