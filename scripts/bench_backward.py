#!/usr/bin/env python3
"""Times the gradient path of spmm on a BASELINE config (default products): CSR transpose (once
per graph), value gather, SDDMM (d values) and A^T @ dC (d b), with HIP events; reports
gather-model GB/s per kernel (DESIGN.md §3 bytes model, SDDMM: one B row + one dC row per row)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--n", type=int, default=0, help="override the dense width")
    ap.add_argument("--only", default="", help="comma list of phases (transpose,gather,sddmm,db,fwd)")
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import autograd as ag
    from oneflow_spmm import synth
    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    n = args.n or n
    dev = torch.device("cuda", 0)
    rp, ci, v = synth.csr(m, k, nnz, val_dtype=dt, threads=16)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, k, n, dt, device=dev)
    g = synth.dense(0, m, n, dt, device=dev, seed=7)
    sv = b.element_size()
    res = {"config": args.config, "n": n}
    only = set(args.only.split(",")) if args.only else {"transpose", "gather", "sddmm", "db", "fwd"}
    if only & {"transpose", "gather", "db"}:
        t = timed(lambda: fs.csr_transpose(rp, ci, k), reps=3)
        res["transpose_ms"] = t
        rt, ct, perm = fs.csr_transpose(rp, ci, k)
    if "gather" in only:
        res["gather_values_ms"] = timed(lambda: ag.gather_values(perm, v))
    if "sddmm" in only:
        t = timed(lambda: fs.sddmm(rp, ci, g, b))
        sd_bytes = 4 * (m + 1) + 4 * nnz + sv * nnz * n + sv * m * n + sv * nnz
        res["sddmm_ms"] = t
        res["sddmm_gbs"] = sd_bytes / (t * 1e-3) / 1e9
    if "db" in only:
        vt = ag.gather_values(perm, v)
        t = timed(lambda: fs.spmm_csr(rt, ct, vt, k, m, g))
        db_bytes = 4 * (k + 1) + (4 + sv) * nnz + sv * nnz * n + sv * k * n
        res["db_spmm_ms"] = t
        res["db_spmm_gbs"] = db_bytes / (t * 1e-3) / 1e9
        # the same product reading A's values through perm (no values[perm] copy): the
        # learnable-edge-weight backward; its bytes add one 4-B perm read per nonzero
        from oneflow_spmm import ops
        out_g = torch.empty((k, n), dtype=dt, device=dev)
        t = timed(lambda: ops.spmm_csr_gathered(rt, ct, v, perm, g, k, m, out=out_g))
        res["db_gathered_ms"] = t
        res["db_gathered_bitexact"] = bool(torch.equal(out_g, fs.spmm_csr(rt, ct, vt, k, m, g)))
    if "fwd" in only:
        res["forward_ms"] = timed(lambda: fs.spmm_csr(rp, ci, v, m, k, b))
    print(json.dumps({kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in res.items()}))


if __name__ == "__main__":
    main()
