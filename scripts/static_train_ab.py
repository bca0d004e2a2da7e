#!/usr/bin/env python3
"""Interleaved A/B of attr static_csr over a whole training step of one GNN aggregation layer:
out = A @ b with learnable edge values and features, then out.backward(g) -- the forward SpMM,
the values-gradient SDDMM (sddmm_csr) and the features-gradient A^T @ g (over the autograd's
cached transpose, which keeps its own plan in both forms).  `static` passes static_csr to the
forward (and so to the SDDMM); `plain` plans both every step.

Per case, rounds alternate the two forms; each round times `reps` steps captured into one
torch.cuda.graph and replayed (GPU time per step, no host work inside).  The gradients of both
forms are compared bit for bit.

    python scripts/static_train_ab.py [--cases arxiv:f32:64,...] [--rounds 5]

One JSON line per case: median ms per step of each form, the difference, the bit checks."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16}
GRAPHS = {"arxiv": (169_343, 169_343, 1_166_243), "plaw1m": (1_000_000, 1_000_000, 20_000_000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="arxiv:f32:17,arxiv:f32:64,arxiv:bf16:47,plaw1m:f32:64")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import _C, synth

    dev = torch.device("cuda", 0)
    for case in args.cases.split(","):
        gname, dname, n = case.split(":")
        n, dt = int(n), DT[dname]
        m, k, nnz = GRAPHS[gname]
        rp, ci, v32 = synth.csr(m, k, nnz, val_dtype=torch.float32, threads=16)
        d_rp, d_ci = rp.to(dev), ci.to(dev)
        g = synth.dense(0, m, n, dt, device=dev)
        static_id = abs(hash(case)) % (1 << 30) + 1
        leaves = {f: (v32.to(dt).to(dev).requires_grad_(True),
                      synth.dense(0, k, n, dt, device=dev).requires_grad_(True))
                  for f in ("static", "plain")}

        def step(form):
            dv, db = leaves[form]
            out = fs.spmm(d_rp, d_ci, dv, m, k, db, static_csr=static_id if form == "static" else 0)
            out.backward(g)

        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(3):  # warm: plans, the transpose and its cached values, outside capture
                for form in ("static", "plain"):
                    for t in leaves[form]:
                        t.grad = None
                    step(form)
        s.synchronize()
        graphs = {}
        for form in ("static", "plain"):
            for t in leaves[form]:
                t.grad = None
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for _ in range(args.reps):
                    step(form)
            graphs[form] = gr
        torch.cuda.synchronize()
        times = {"static": [], "plain": []}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(args.rounds):
            for form in (("static", "plain") if r % 2 == 0 else ("plain", "static")):
                e0.record()
                graphs[form].replay()
                e1.record()
                torch.cuda.synchronize()
                times[form].append(e0.elapsed_time(e1) / args.reps)
        same = all(torch.equal(leaves["static"][i].grad.view(torch.uint8),
                               leaves["plain"][i].grad.view(torch.uint8)) for i in range(2))
        med = {f: float(np.median(v)) for f, v in times.items()}
        print(json.dumps({
            "case": case, "m": m, "nnz": nnz, "n": n, "reps": args.reps, "rounds": args.rounds,
            "ms_per_step_median": {f: round(v, 5) for f, v in med.items()},
            "saved_us_per_step": round((med["plain"] - med["static"]) * 1e3, 2),
            "grads_bitexact_static_vs_plain": bool(same),
            "static_plans": _C.static_plans()}), flush=True)
        del graphs, leaves
        torch.cuda.synchronize()
        _C.static_plans(release=True)


if __name__ == "__main__":
    main()
