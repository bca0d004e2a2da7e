#!/usr/bin/env python3
"""The SpMM phase of a G-rank row split, measured rank by rank on ONE GPU: for every rank r, the
local CSR slice (BalancedSplitter rows, row_ptr rebased, columns remapped into the padded
gathered layout) times the full gathered B, exactly what rank r's kernel does after the
exchange.  Reports per-rank ms and the whole-job SpMM-phase GFLOP/s = 2*nnz*N / max_r(ms)
(the exchange itself needs the G GPUs and is not included).

    python scripts/rank_local.py --config products --world 8
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
    ap.add_argument("--config", default="products")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from oneflow_spmm import _C, ops, synth
    from oneflow_spmm.distributed import padded_owner_remap

    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    G = args.world
    dev = torch.device("cuda", 0)
    rp = synth.row_ptr(m, k, nnz)
    pad = -(-k // G)
    gathered = torch.zeros((G * pad, n), dtype=dt, device=dev)
    for r in range(G):
        lo, hi = _C.balanced_range(k, G, r)
        gathered[r * pad: r * pad + hi - lo] = synth.dense(lo, hi, n, dt, device=dev)
    opts = ops.make_options(split=ops.default_split(n))
    res, e0, e1 = [], torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(G):
        lo, hi = _C.balanced_range(m, G, r)
        j0, j1 = int(rp[lo]), int(rp[hi])
        cols = torch.from_numpy(synth.columns(m, k, rp, lo, hi, threads=16))
        d_ci = padded_owner_remap(cols, k, G).to(dev)
        d_rp = torch.from_numpy((rp[lo:hi + 1] - rp[lo]).astype(np.int32)).to(dev)
        d_v = synth.values(j0, j1, dt).to(dev)
        out = torch.empty((hi - lo, n), dtype=dt, device=dev)
        kern = ops.SpmmCsrKernel(hi - lo, G * pad, n, j1 - j0, torch.int32, dt, dev, opts)
        kern(d_rp, d_ci, d_v, gathered, out)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0.record()
            kern(d_rp, d_ci, d_v, gathered, out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res.append({"rank": r, "rows": hi - lo, "nnz": j1 - j0, "ms": round(float(np.median(ts)), 4)})
        del d_ci, d_rp, d_v, out, kern
    worst = max(x["ms"] for x in res)
    print(json.dumps({"config": args.config, "world": G, "per_rank": res, "max_ms": worst,
                      "spmm_phase_gflops_aggregate": round(2.0 * nnz * n / (worst * 1e-3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
