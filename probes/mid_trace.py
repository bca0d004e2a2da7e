"""Mid-size op calls for a rocprofv3 kernel trace (the mid form's launches: plan count / scan /
write, main with block items, reduce): 200 calls per configuration, configurations separated by
a 50 ms idle gap so probes/trace_segments.py can split the trace."""
import sys
import time

sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import torch  # noqa: E402

from oneflow_spmm import ops, synth  # noqa: E402

dev = torch.device("cuda", 0)
for name, (m, nnz, n) in {"pubmed16": (19717, 88648, 16), "pubmed64": (19717, 88648, 64),
                          "arxiv16": (169343, 1166243, 16), "arxiv128": (169343, 1166243, 128)}.items():
    rp, ci, v = synth.csr(m, m, nnz)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, m, n, device=dev)
    out = torch.empty((m, n), device=dev)
    k = ops.SpmmCsrKernel(m, m, n, nnz, torch.int32, torch.float32, dev)
    for _ in range(200):
        k(rp, ci, v, b, out)
    torch.cuda.synchronize()
    print(name, flush=True)
    time.sleep(0.05)
