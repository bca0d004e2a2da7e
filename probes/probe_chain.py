"""What bounds one long item in the block engine: one 4096- / 7132-nonzero row among 2000 short
ones at N=16 and N=128 with (a) random columns over 100k B rows, (b) every nonzero on B row 0
(the rows stay in L2: no memory latency), timed for the small form (one launch) and the mid
form.  Prints one JSON object."""
import json
import sys

sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oneflow_spmm import ops, synth  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 2)


res = {}
rng = np.random.default_rng(0)
m, k = 2000, 100000
for n in (16, 128):
    for L in (4096, 7132):
        deg = rng.integers(0, 6, size=m)
        deg[1234] = L
        rp = np.zeros(m + 1, np.int64)
        rp[1:] = np.cumsum(deg)
        ci = np.concatenate([np.sort(rng.choice(k, d, replace=False)) for d in deg]).astype(np.int32)
        nnz = ci.size
        d_rp = torch.from_numpy(rp.astype(np.int32)).to(dev)
        d_v = torch.from_numpy(rng.uniform(-1, 1, nnz).astype(np.float32)).to(dev)
        b = synth.dense(0, k, n, device=dev)
        out = torch.empty((m, n), device=dev)
        for cols in ("random", "row0"):
            c = ci if cols == "random" else np.zeros_like(ci)
            d_ci = torch.from_numpy(c).to(dev)
            for form, var in (("small", 30000), ("mid", 30001)):
                kern = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, torch.float32, dev,
                                         ops.make_options(variant=var))
                res[f"n{n}_L{L}_{cols}_{form}_us"] = t(lambda: kern(d_rp, d_ci, d_v, b, out))
print(json.dumps(res))
