#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python scripts/ab.py [--config products] [--rounds 8] [--reps 5] [--variants 0,264,432,...]

Variant codes: 0 = the op's auto choice; VEC*100+LPR forces (VEC, LPR); "ordered" = no hub split;
a suffix "h<thr>" sets the heavy-row threshold (h-1 = off), e.g. 10002h256; a prefix "f" runs
the fused epilogue (bias + relu) with that variant, e.g. f0 (not compared for bit identity).
Prints per-variant median/min ms and gather-model GB/s; checks every variant is bit-identical to
the auto variant on the first round.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "of-spmm_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0,432,264,464,232")
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--heavy", type=int, default=0, help="0 default, <0 off")
    ap.add_argument("--n", type=int, default=0, help="override the dense width")
    ap.add_argument("--share-out", action="store_true",
                    help="one output buffer for all variants (papers scale); identity by checksum")
    args = ap.parse_args()
    from oneflow_spmm import ops, synth
    from bench import alg_bytes

    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    n = args.n or n
    dev = torch.device("cuda", 0)
    rp, ci, v = synth.csr(m, k, nnz, val_dtype=dt, threads=16)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, k, n, dt, device=dev)
    s_v = b.element_size()
    nbytes = alg_bytes(m, nnz, n, s_v)
    kernels, outs, fused = {}, {}, {}
    bias = synth.dense(0, 1, n, dt, device=dev)[0]
    for name in args.variants.split(","):
        fused[name] = name.startswith("f")
        if name == "ordered":
            opts = ops.make_options(ordered=True)
        else:
            vv, _, h = name.lstrip("f").partition("h")
            opts = ops.make_options(variant=int(vv), split=args.split, heavy=int(h) if h else args.heavy)
        kernels[name] = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, dt, dev, opts)
        if args.share_out and outs:
            outs[name] = next(iter(outs.values()))
        else:
            outs[name] = torch.empty((m, n), dtype=dt, device=dev)
    times = {name: [] for name in kernels}
    sums = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        for name, kern in kernels.items():
            epi = dict(bias=bias, relu=True) if fused[name] else {}
            kern(rp, ci, v, b, outs[name], **epi)  # warm
            torch.cuda.synchronize()
            if args.share_out and r == 0:
                sums[name] = int(outs[name].view(torch.int32).sum(dtype=torch.int64).item())
            e0.record()
            for _ in range(args.reps):
                kern(rp, ci, v, b, outs[name], **epi)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.reps)
        if r == 0 and args.share_out:
            first = next(iter(sums.values()))
            for name, cs in sums.items():
                print(f"[ab] {name}: checksum equal to first variant: {cs == first}", flush=True)
        elif r == 0:
            ref = outs[next(iter(outs))]
            for name, o in outs.items():
                if fused[name]:
                    continue
                same = torch.equal(o.view(torch.uint8), ref.view(torch.uint8))
                print(f"[ab] {name}: bit-identical to first variant: {same}", flush=True)
    for name, t in times.items():
        t = np.array(t)
        print(f"[ab] {args.config} variant {name:>8}: median {np.median(t):.4f} ms  min {t.min():.4f} ms"
              f"  -> {nbytes / (np.median(t) * 1e-3) / 1e9:.0f} GB/s (gather model)", flush=True)


if __name__ == "__main__":
    main()
