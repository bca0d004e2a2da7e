"""Device time against host-submission time per SpMM call: each configuration <graph>:<N>:<variant>
(graphs of probes/probe_split.py) is timed eagerly (events around back-to-back calls, as
probe_split does) and as a captured HIP graph of the same calls replayed (no host launch cost).
A gap between the two is launch overhead, not kernel time.

    python3 probes/probe_graph.py arxiv:16:0 arxiv:16:10022 pubmed:16:0
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT, os.path.join(ROOT, "scripts")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from probe_split import GRAPHS  # noqa: E402
from oneflow_spmm import ops, synth  # noqa: E402

REPS = 50
# uniform-degree graphs: name -> (rows = cols, nonzeros per row); no hubs, no heavy rows
UNIFORM = {"u169k7": (169_343, 7), "u169k2": (169_343, 2), "u169k28": (169_343, 28),
           "u1m20": (1_000_000, 20)}


def uniform_csr(m, deg, seed=0):
    g = torch.Generator().manual_seed(seed)
    rp = torch.arange(m + 1, dtype=torch.int32) * deg
    ci = torch.randint(0, m, (m * deg,), generator=g, dtype=torch.int32)
    val = torch.rand(m * deg, generator=g) - 0.5
    return rp, ci, val


def timed(fn, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def main():
    dev = torch.device("cuda", 0)
    cache = {}
    for spec in sys.argv[1:]:
        name, n, vs = spec.split(":")
        n = int(n)
        v, _, hs = vs.partition("h")
        variant, heavy = int(v), (int(hs) if hs else 0)
        if name in UNIFORM:
            m, deg = UNIFORM[name]
            nnz = m * deg
        else:
            m, nnz = GRAPHS[name]
        if name not in cache:
            rp, ci, val = uniform_csr(m, deg) if name in UNIFORM else synth.csr(m, m, nnz, threads=16)
            cache[name] = (rp.to(dev), ci.to(dev), val.to(dev))
        rp, ci, val = cache[name]
        b = synth.dense(0, m, n, device=dev)
        out = torch.empty((m, n), device=dev)
        kern = ops.SpmmCsrKernel(m, m, n, nnz, torch.int32, torch.float32, dev,
                                 ops.make_options(variant=variant, heavy=heavy))
        stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(stream):
            for _ in range(3):
                kern(rp, ci, val, b, out)
            torch.cuda.synchronize()
            ref = out.clone()

            def eager():
                for _ in range(REPS):
                    kern(rp, ci, val, b, out)

            eg = [timed(eager, stream) / REPS for _ in range(5)]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for _ in range(REPS):
                    kern(rp, ci, val, b, out)
            g.replay()
            torch.cuda.synchronize()
            gr = [timed(g.replay, stream) / REPS for _ in range(5)]
            same = torch.equal(out.view(torch.int32), ref.view(torch.int32))
        print(json.dumps({"spec": spec, "eager_us": round(float(np.median(eg)), 2),
                          "graph_us": round(float(np.median(gr)), 2), "graph_bits_equal": same}),
              flush=True)
        del g, kern, out, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
