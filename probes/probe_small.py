import sys, json
sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import numpy as np, torch
import oneflow_spmm as fs
from oneflow_spmm import ops, synth
dev = torch.device("cuda", 0)
def t(fn, reps=200):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
res = {}
for name, (m, nnz, n) in {"cora": (2708, 10556, 16), "cora64": (2708, 10556, 64), "small20k": (20000, 400000, 16)}.items():
    rp, ci, v = synth.csr(m, m, nnz)
    deg = np.diff(rp.numpy()); res[name + "_maxdeg"] = int(deg.max())
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    b = synth.dense(0, m, n, device=dev); out = torch.empty((m, n), device=dev)
    for label, opts in {"default": None, "u8_forced": ops.make_options(variant=100 + (16 if n == 16 else 16)) if n == 16 else ops.make_options(variant=416),
                        "ordered": ops.make_options(ordered=True), "noheavy": ops.make_options(heavy=-1),
                        # small-launch form without / with wave items (tuning variants 10022-10025)
                        "group_items": ops.make_options(variant=10022 if n == 16 else 10024),
                        "wave_items": ops.make_options(variant=10023 if n == 16 else 10025)}.items():
        k = ops.SpmmCsrKernel(m, m, n, ci.numel(), torch.int32, torch.float32, dev, opts)
        res[f"{name}_{label}_us"] = round(t(lambda: k(rp, ci, v, b, out)), 2)
    # uniform-degree matrix, same nnz
    d = np.full(m, nnz // m); d[: nnz - d.sum()] += 1
    rpu = torch.from_numpy(np.concatenate([[0], np.cumsum(d)]).astype(np.int32)).to(dev)
    ciu = torch.from_numpy(np.concatenate([np.sort(np.random.default_rng(r).choice(m, x, replace=False)) for r, x in enumerate(d)]).astype(np.int32)).to(dev)
    k = ops.SpmmCsrKernel(m, m, n, ciu.numel(), torch.int32, torch.float32, dev)
    res[f"{name}_uniform_us"] = round(t(lambda: k(rpu, ciu, v, b, out)), 2)
print(json.dumps(res))
