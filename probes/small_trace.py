"""Small-launch op calls for a rocprofv3 kernel trace: Cora-shaped (N=16, 64) and a 20k-row
power-law graph (N=16), 200 calls each, NVTX-free (the trace's timestamps separate them)."""
import sys
sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import torch
import oneflow_spmm as fs
from oneflow_spmm import synth

dev = torch.device("cuda", 0)
for name, (m, nnz, n) in {"cora": (2708, 10556, 16), "cora64": (2708, 10556, 64),
                          "small20k": (20000, 400000, 16)}.items():
    rp, ci, v = synth.csr(m, m, nnz)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, m, n, device=dev)
    out = torch.empty((m, n), device=dev)
    for _ in range(200):
        fs.spmm(rp, ci, v, m, m, b, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        fs.spmm(rp, ci, v, m, m, b, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 200 * 1e3, 2), "us per call (events)", flush=True)
