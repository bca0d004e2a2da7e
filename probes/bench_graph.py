#!/usr/bin/env python3
"""The compiled spmm_csr job (oneflow_spmm.ccl.SpmmJob, the nn.Graph form of one layer): eager
runs against the job's native graph mode (ofx_spmm_job_set_graph: captured once through the
device C-ABI's hipGraph executable, one graph launch per run), on a BASELINE-shaped graph; plus
the eager two-layer GCN forward through the op layer for reference.

    python probes/bench_graph.py [--config cora] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import torch  # noqa: E402


def per_iter_ms(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cora")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import synth

    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    assert m == k, "a GCN layer stack needs a square adjacency"
    dev = torch.device("cuda", 0)
    rp, ci, v = synth.csr(m, k, nnz, val_dtype=dt, threads=16)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    x = synth.dense(0, k, n, dt, device=dev)
    bias = synth.dense(0, 1, n, dt, device=dev, seed=5)[0]

    def gcn(h):
        h1 = fs.fused_spmm(rp, ci, v, m, m, h, bias, relu=True)
        return fs.spmm(rp, ci, v, m, m, h1)

    with torch.no_grad():
        eager = per_iter_ms(lambda: gcn(x), args.iters)
    print(json.dumps({"config": args.config, "m": m, "nnz": nnz, "n": n, "layers": 2,
                      "eager_ms_per_forward": round(eager, 4)}))

    # one spmm_csr layer as the compiled job (the nn.Graph form): eager runs vs the job's own
    # graph mode (captured once through the C-ABI's hipGraph executable, one launch per run);
    # back-to-back rate and latency of a single synchronised call
    from oneflow_spmm import ccl
    ccl.install_control_plane()
    pl = ccl.PlacementSpec("hip", 1, 0, (0,), (0,))
    out = torch.empty((m, n), dtype=dt, device=dev)
    res = {"config": args.config, "layer": "spmm_csr job"}
    for mode in ("eager", "graph"):
        job = ccl.SpmmJob(pl, m, k, n, nnz, torch.int32, dt, dev, graph=mode == "graph")
        run = lambda: job(rp, ci, v, x, out=out)  # noqa: E731
        run()
        run()
        res[f"{mode}_ms_back_to_back"] = round(per_iter_ms(run, args.iters), 4)

        def one():
            run()
            torch.cuda.synchronize()
        res[f"{mode}_ms_latency"] = round(per_iter_ms(one, args.iters), 4)
        if mode == "graph":
            res["graph_stats"] = job.graph_stats
    res["op_layer_eager_ms_back_to_back"] = round(
        per_iter_ms(lambda: fs.spmm(rp, ci, v, m, k, x), args.iters), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
