#!/usr/bin/env python3
"""Interleaved A/B of attr static_csr: the op call with the work-list plan
kept in the kernel state (static_csr) against the ordinary call that plans every time.

Per case, rounds alternate the two forms; each round times
  graph  - `reps` op calls captured into one torch.cuda.graph, replayed: GPU time per call
           (no host work inside), HIP events around the replay;
  eager  - `reps` op calls back to back from Python, HIP events around them (the op layer's host
           time is inside when it exceeds the kernels').
The outputs of both forms are compared bit for bit, and sampled rows against the oracle.

    python scripts/static_csr_ab.py [--cases arxiv:f32:17,arxiv:bf16:47,...] [--rounds 5]

One JSON line per case: median ms per call of each form, the difference, the bit checks."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
GRAPHS = {"arxiv": (169_343, 169_343, 1_166_243), "plaw1m": (1_000_000, 1_000_000, 20_000_000),
          "products": (2_449_029, 2_449_029, 123_718_280), "pubmed": (19_717, 19_717, 88_648)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="arxiv:f32:17,arxiv:bf16:47,arxiv:f32:64,plaw1m:f32:64,"
                                       "products:f32:128")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import _C, synth
    from oracle import oracle

    dev = torch.device("cuda", 0)
    cache = {}
    for case in args.cases.split(","):
        gname, dname, n = case.split(":")
        n, dt = int(n), DT[dname]
        m, k, nnz = GRAPHS[gname]
        if gname not in cache:
            rp, ci, v32 = synth.csr(m, k, nnz, val_dtype=torch.float32, threads=16)
            cache[gname] = (rp, ci, v32, rp.to(dev), ci.to(dev))
        rp, ci, v32, d_rp, d_ci = cache[gname]
        d_v = v32.to(dt).to(dev)
        b = synth.dense(0, k, n, dt, device=dev)
        reps = args.reps if nnz < 50_000_000 else max(5, args.reps // 10)
        outs = {f: torch.empty((m, n), dtype=dt, device=dev) for f in ("static", "plain")}
        static_id = abs(hash(case)) % (1 << 30) + 1

        def call(form):
            fs.spmm(d_rp, d_ci, d_v, m, k, b, out=outs[form],
                    static_csr=static_id if form == "static" else 0)

        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        graphs = {}
        with torch.cuda.stream(s):
            for form in ("static", "plain"):
                call(form)  # warm (the static form plans here, outside the capture)
        s.synchronize()
        for form in ("static", "plain"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    call(form)
            graphs[form] = g
        torch.cuda.synchronize()
        times = {f"{mode}_{form}": [] for mode in ("graph", "eager") for form in ("static", "plain")}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(args.rounds):
            order = ("static", "plain") if r % 2 == 0 else ("plain", "static")
            for form in order:
                e0.record()
                graphs[form].replay()
                e1.record()
                torch.cuda.synchronize()
                times[f"graph_{form}"].append(e0.elapsed_time(e1) / reps)
                e0.record()
                for _ in range(reps):
                    call(form)
                e1.record()
                torch.cuda.synchronize()
                times[f"eager_{form}"].append(e0.elapsed_time(e1) / reps)
        same = bool(torch.equal(outs["static"].view(torch.uint8), outs["plain"].view(torch.uint8)))
        # sampled rows against the oracle (the first 2,000 rows: every form's bits)
        r_s = min(m, 2000)
        rp_np = rp.numpy()[: r_s + 1].astype(np.int64)
        j1 = int(rp_np[-1])
        to_np = (lambda t: t.view(torch.int16).numpy().view(np.uint16)) if dt == torch.bfloat16 \
            else (lambda t: t.numpy())
        ref = oracle.spmm(rp_np, ci.numpy()[:j1].astype(np.int64), to_np(v32.to(dt)[:j1]),
                          to_np(b.cpu()), dtype=dname, nthreads=16)
        got = to_np(outs["static"][:r_s].cpu())
        oracle_ok = bool(np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                        np.ascontiguousarray(ref).view(np.uint8)))
        med = {key: float(np.median(v)) for key, v in times.items()}
        print(json.dumps({
            "case": case, "m": m, "nnz": nnz, "n": n, "reps": reps, "rounds": args.rounds,
            "ms_per_call_median": {key: round(v, 5) for key, v in med.items()},
            "graph_saved_us": round((med["graph_plain"] - med["graph_static"]) * 1e3, 2),
            "eager_saved_us": round((med["eager_plain"] - med["eager_static"]) * 1e3, 2),
            "bitexact_static_vs_plain": same, "oracle_first_rows_bitexact": oracle_ok,
            "static_plans": _C.static_plans()}), flush=True)
        del graphs, outs, b, d_v
        torch.cuda.synchronize()
        _C.static_plans(release=True)


if __name__ == "__main__":
    main()
