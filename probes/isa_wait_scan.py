#!/usr/bin/env python3
"""Scans the gfx950 code objects of the built SpMM units for B-row loads (raw buffer loads:
dwordx2 / dword / short loads) issued right behind an `s_waitcnt vmcnt(0)` — a load that cannot
start before every older load has returned, i.e. one row in flight per lane.  Prints per kernel:
loads, loads behind vmcnt(0), VGPRs.

    python probes/isa_wait_scan.py [of-spmm_amd/build] [--filter spmm_main]"""
import os
import re
import subprocess
import sys

R = "/opt/rocm/lib/llvm/bin"
LOAD = re.compile(r"\bbuffer_load_(dwordx4|dwordx2|dword|ushort|short_d16)\b")  # B rows (raw buffer loads)


def code_object(obj, tmp):
    fb, co = tmp + ".fb", tmp + ".co"
    subprocess.run([f"{R}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj], check=True)
    subprocess.run([f"{R}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                   check=True)
    return co


def main():
    build = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "of-spmm_amd/build"
    filt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else "spmm_main"
    for fn in sorted(os.listdir(os.path.join(build, "csrc"))):
        if not fn.endswith(".o") or not fn.startswith(("spmm_inst", "spmm_backward")):
            continue
        co = code_object(os.path.join(build, "csrc", fn), f"/tmp/isa_scan_{fn}")
        syms = subprocess.run([f"{R}/llvm-readelf", "-s", co], capture_output=True, text=True).stdout
        notes = subprocess.run([f"{R}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        vg = dict(re.findall(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.vgpr_count:\s+(\d+)", notes))
        seen = set()
        for line in syms.splitlines():
            f = line.split()
            if len(f) < 8 or f[3] != "FUNC" or filt not in f[7] or f[7] in seen:
                continue
            seen.add(f[7])
            addr, size = int(f[1], 16), int(f[2])
            dis = subprocess.run([f"{R}/llvm-objdump", "-d", f"--start-address={addr}",
                                  f"--stop-address={addr + size}", co], capture_output=True, text=True).stdout
            lines = [ln.split("//")[0].strip() for ln in dis.splitlines()]
            loads = bad = 0
            for i, ln in enumerate(lines):
                if LOAD.search(ln):
                    loads += 1
                    for back in lines[max(0, i - 4):i]:
                        if back.startswith("s_waitcnt") and "vmcnt(0)" in back:
                            bad += 1
                            break
            name = subprocess.run(["c++filt"], input=f[7], capture_output=True, text=True).stdout.strip()
            name = name.replace("ofx::(anonymous namespace)::", "")
            short = name[:name.find("(")] if "(" in name else name
            print(f"{fn:26s} loads {loads:3d} behind-vmcnt0 {bad:3d} vgpr {vg.get(f[7], '?'):>4s}  {short}")


if __name__ == "__main__":
    main()
