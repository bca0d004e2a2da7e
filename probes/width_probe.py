#!/usr/bin/env python3
"""Mid-size widths, one configuration per spec <graph>:<dtype>:<N>[:<variant>[:<heavy>]] (graphs of
probes/probe_split.py, synthetic power-law, generated once per graph; <graph>@g<gamma> sets the
degree exponent, e.g. arxiv@g50 for nearly even degrees, 2.5 by default):

  --mode time   (default) per spec: the form the launch takes (ofx_spmm_csr_describe), the median
                device time of one call over a replayed hipGraph of REPS calls (no host launch
                cost), the gather-model fraction of 8 TB/s, and a bit-exact check of the first rows
                against the oracle.  One JSON line per spec; specs are interleaved over rounds.
  --mode run    REPS eager calls per spec with an idle gap between specs (rocprofv3 --kernel-trace
                / --pmc runs of one spec at a time).

    python probes/width_probe.py arxiv:bf16:47 arxiv:bf16:64 arxiv:f32:17 [--mode run]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT, os.path.join(ROOT, "scripts")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from probe_split import GRAPHS  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--mode", choices=["time", "run"], default="time")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from oneflow_spmm import ops, synth
    from bench import alg_bytes
    from oracle import oracle
    from tests.helpers import to_oracle

    dev = torch.device("cuda", 0)
    graphs, cases = {}, []
    for spec in args.specs:
        parts = spec.split(":")
        g, dname, n = parts[0], parts[1], int(parts[2])
        variant = int(parts[3]) if len(parts) > 3 else 0
        heavy = int(parts[4]) if len(parts) > 4 else 0  # options.heavy (0: automatic)
        if g not in graphs:  # <graph>[@g<gamma>]: the degree exponent (2.5 default; large = even)
            name, _, gam = g.partition("@g")
            m, nnz = GRAPHS[name]
            rp, ci, v = synth.csr(m, m, nnz, gamma=float(gam) if gam else 2.5)
            graphs[g] = (m, nnz, rp, ci, v)
        m, nnz, rp, ci, v = graphs[g]
        dt = DT[dname]
        b = synth.dense(0, m, n, dt, device=dev)
        d = (rp.to(dev), ci.to(dev), v.to(dt).to(dev), b)
        opts = ops.make_options(variant=variant, heavy=heavy) if (variant or heavy) else None
        kern = ops.SpmmCsrKernel(m, m, n, nnz, torch.int32, dt, dev, opts)
        out = torch.empty((m, n), dtype=dt, device=dev)
        desc = ops.describe(m, m, n, nnz, dt, b_addr=b.data_ptr(), c_addr=out.data_ptr(),
                            options=opts)
        cases.append(dict(spec=spec, g=g, m=m, nnz=nnz, n=n, dt=dt, d=d, kern=kern, out=out,
                          desc=desc))

    if args.mode == "run":
        for c in cases:
            for _ in range(args.reps):
                c["kern"](*c["d"], c["out"])
            torch.cuda.synchronize()
            print(c["spec"], c["desc"]["form"], c["desc"]["kernel"], flush=True)
            time.sleep(0.05)
        return

    s = torch.cuda.Stream(dev)
    for c in cases:  # capture REPS calls per spec (warm first, outside the capture)
        with torch.cuda.stream(s):
            c["kern"](*c["d"], c["out"])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(args.reps):
                c["kern"](*c["d"], c["out"])
        c["graph"], c["us"] = g, []
    for _ in range(args.rounds):
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):  # replay() launches on the current stream
                e0.record(s)
                c["graph"].replay()
                e1.record(s)
            torch.cuda.synchronize()
            c["us"].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    for c in cases:
        m, nnz, n, dt = c["m"], c["nnz"], c["n"], c["dt"]
        rp, ci, v, b = c["d"]
        rows = min(m, 2000)  # first rows against the oracle (their own sub-problem)
        sub_rp = rp[:rows + 1].cpu()
        j1 = int(sub_rp[-1])
        ref = oracle.spmm(to_oracle(sub_rp), to_oracle(ci[:j1].cpu()), to_oracle(v[:j1].cpu()),
                          to_oracle(b.cpu()), dtype={v_: k_ for k_, v_ in DT.items()}[dt])
        got = to_oracle(c["out"][:rows])
        exact = bool(np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                    np.ascontiguousarray(ref).view(np.uint8)))
        us = float(np.median(c["us"]))
        s_v = torch.empty(0, dtype=dt).element_size()
        frac = alg_bytes(m, nnz, n, s_v) / (us * 1e-6) / 8e12
        print(json.dumps({"spec": c["spec"], "us": round(us, 2), "frac_of_8tbs": round(frac, 4),
                          "form": c["desc"]["form"], "VEC": c["desc"]["VEC"],
                          "LPR": c["desc"]["LPR"], "U": c["desc"]["U"], "HL": c["desc"]["HL"],
                          "first_rows_bitexact": exact}), flush=True)


if __name__ == "__main__":
    main()
