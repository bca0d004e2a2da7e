"""Launch sequences for a rocprofv3 kernel trace: 200 back-to-back calls per configuration
<graph>:<N>:<variant> (graphs of probes/probe_split.py), configurations separated by a 50 ms
idle gap so probes/trace_segments.py can split the trace into one segment each.

    rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- \
        python3 probes/trace_forms.py arxiv:16:0 arxiv:16:30005 pubmed:64:0
    python3 probes/trace_segments.py <dir>/..._kernel_trace.csv
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT, os.path.join(ROOT, "scripts")]

import torch  # noqa: E402

from probe_split import GRAPHS  # noqa: E402
from oneflow_spmm import ops, synth  # noqa: E402

dev = torch.device("cuda", 0)
cache = {}
for spec in sys.argv[1:]:
    name, n, vs = spec.split(":")
    v, _, hs = vs.partition("h")  # "<variant>" or "<variant>h<heavy threshold>"
    n, variant, heavy = int(n), int(v), (int(hs) if hs else 0)
    m, nnz = GRAPHS[name]
    if name not in cache:
        rp, ci, v = synth.csr(m, m, nnz, threads=16)
        cache[name] = (rp.to(dev), ci.to(dev), v.to(dev))
    rp, ci, v = cache[name]
    b = synth.dense(0, m, n, device=dev)
    out = torch.empty((m, n), device=dev)
    k = ops.SpmmCsrKernel(m, m, n, nnz, torch.int32, torch.float32, dev,
                          ops.make_options(variant=variant, heavy=heavy))
    for _ in range(200):
        k(rp, ci, v, b, out)
    torch.cuda.synchronize()
    print(spec, flush=True)
    time.sleep(0.05)
