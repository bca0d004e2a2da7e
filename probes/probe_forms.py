#!/usr/bin/env python3
"""Forms A/B at big-launch sizes: the automatic choice (variant 0) against the mid form forced at
any size (30001: block items for hub chunks and heavy rows, big-launch light rows; 30002: the same
with small-launch light rows), on BASELINE-shaped graphs over several widths.  Interleaved, median
of 3 rounds of 5 back-to-back launches (HIP events); outputs must be bit-identical across forms.

    python probes/probe_forms.py [--configs plaw1m,products] [--widths 16,32,64,128]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="plaw1m,products")
    ap.add_argument("--widths", default="16,32,64,128")
    ap.add_argument("--variants", default="0,30001,30002")
    args = ap.parse_args()
    from oneflow_spmm import ops, synth
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in args.variants.split(",")]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name in args.configs.split(","):
        cfg = synth.CONFIGS[name]
        m, k, nnz = cfg["m"], cfg["k"], cfg["nnz"]
        rp, ci, v = synth.csr(m, k, nnz, threads=16)
        rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
        for n in [int(x) for x in args.widths.split(",")]:
            b = synth.dense(0, k, n, device=dev)
            out = torch.empty((m, n), device=dev)
            kern = {vv: ops.SpmmCsrKernel(m, k, n, nnz, rp.dtype, b.dtype, dev,
                                          ops.make_options(variant=vv)) for vv in variants}
            times, ref = {vv: [] for vv in variants}, None
            for _ in range(3):
                for vv, kk in kern.items():
                    kk(rp, ci, v, b, out)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(out.view(torch.int32), ref.view(torch.int32)):
                        raise SystemExit(f"{name} n={n} variant {vv}: bits differ")
                    ev[0].record()
                    for _ in range(5):
                        kk(rp, ci, v, b, out)
                    ev[1].record()
                    torch.cuda.synchronize()
                    times[vv].append(ev[0].elapsed_time(ev[1]) / 5)
            med = {vv: float(np.median(t)) for vv, t in times.items()}
            print(json.dumps({"config": name, "n": n,
                              "ms": {str(vv): round(t, 4) for vv, t in med.items()},
                              "best": str(min(med, key=med.get)), "bitexact": True}), flush=True)
            del kern, out, b
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
