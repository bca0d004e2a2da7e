"""A/B of loads in flight per lane (U) for small N=16 launches (small launches):
tuning variants 10015/10016/10017 = Cfg<1, 16, U = 32/64/128>, interleaved, checked bit-identical."""
import json
import sys

sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import torch
from oneflow_spmm import ops, synth

dev = torch.device("cuda", 0)


def t(fn, reps=200):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = {}
for name, (m, nnz) in {"cora": (2708, 10556), "small20k": (20000, 400000), "mid32k": (32768, 1500000)}.items():
    n = 16
    rp, ci, v = synth.csr(m, m, nnz)
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, m, n, device=dev)
    outs, kern = {}, {}
    for label, var in {"default": 0, "u32": 10015, "u64": 10016, "u128": 10017}.items():
        kern[label] = ops.SpmmCsrKernel(m, m, n, ci.numel(), torch.int32, torch.float32, dev,
                                        ops.make_options(variant=var) if var else None)
        outs[label] = torch.empty((m, n), device=dev)
    for label, k in kern.items():
        k(rp, ci, v, b, outs[label])
    torch.cuda.synchronize()
    res[name + "_bitexact"] = all(torch.equal(outs["default"], o) for o in outs.values())
    for rep in range(3):
        for label, k in kern.items():
            us = t(lambda: k(rp, ci, v, b, outs[label]))
            res.setdefault(f"{name}_{label}_us", []).append(round(us, 2))
print(json.dumps(res))
