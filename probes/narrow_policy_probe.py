#!/usr/bin/env python3
"""Probe (not product code): products-shaped N=16 fp32 gather (64-B B rows) under each
cache-policy combination of the B-row loads (probes/narrow_policy_probe.hip).  Interleaved,
median of 3 rounds of 5 launches (HIP events); the sums must equal the default policy's.

    python probes/narrow_policy_probe.py [--aux 17]   # --aux: run only that policy (PMC runs)
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]
SO = os.path.join(ROOT, "scripts", "_narrow_policy_probe.so")
AUX = {0: "default", 1: "sc0", 2: "nt", 3: "sc0|nt", 16: "sc1", 17: "sc0|sc1", 18: "nt|sc1",
       19: "sc0|nt|sc1"}


def build():
    src = os.path.join(ROOT, "scripts", "narrow_policy_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", SO],
                       check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--aux", type=int, default=None)
    ap.add_argument("--config", default="products")
    args = ap.parse_args()
    build()
    if args.build_only:
        return
    import torch
    from oneflow_spmm import synth
    lib = ctypes.CDLL(SO)
    lib.narrow_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    cfg = synth.CONFIGS[args.config]
    m, k, nnz = cfg["m"], cfg["k"], cfg["nnz"]
    n = 16
    dev = torch.device("cuda", 0)
    _, ci, _ = synth.csr(m, k, nnz, threads=16)
    col = ci.to(dev)
    b = synth.dense(0, k, n, device=dev)
    out = torch.empty(((nnz + 255) // 256) * 16, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    auxes = [args.aux] if args.aux is not None else list(AUX)
    times, ref = {a: [] for a in auxes}, None
    for _ in range(3):
        for a in auxes:
            call = (a, col.data_ptr(), b.data_ptr(), nnz, b.numel() * 4, out.data_ptr(), s.cuda_stream)
            assert lib.narrow_launch(*call) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif not torch.equal(out, ref):
                raise SystemExit(f"aux {a}: sums differ")
            ev[0].record(s)
            for _ in range(5):
                lib.narrow_launch(*call)
            ev[1].record(s)
            torch.cuda.synchronize()
            times[a].append(ev[0].elapsed_time(ev[1]) / 5)
    base = float(np.median(times[auxes[0]]))
    row_bytes = nnz * 64
    for a in auxes:
        t = float(np.median(times[a]))
        print(json.dumps({"config": args.config, "n": n, "aux": a, "policy": AUX[a], "ms": round(t, 4),
                          "vs_first": round(t / base, 4),
                          "b_row_bytes_per_s": round(row_bytes / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
