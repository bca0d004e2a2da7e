"""One long row among short ones: time of the small form (one launch, the block takes the long
row; chunk sums in order when it is split) against the planned form (plan + wave items + reduce)
as the row grows.  Prints one JSON object."""
import sys, json
sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import numpy as np, torch
from oneflow_spmm import ops, synth

dev = torch.device("cuda", 0)


def t(fn, reps=100):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 2)


res = {}
rng = np.random.default_rng(0)
for n, lens, planned_variant in ((16, (256, 1000, 4096, 8192, 16384, 32768, 60000), 10023),
                                 (64, (256, 1000, 4096, 8192, 15000), 10025)):
    m, k = 2000, 100000
    for L in lens:
        deg = rng.integers(0, 6, size=m)
        deg[1234] = L
        rp = np.zeros(m + 1, np.int64); rp[1:] = np.cumsum(deg)
        ci = np.concatenate([np.sort(rng.choice(k, d, replace=False)) for d in deg]).astype(np.int32)
        d_rp = torch.from_numpy(rp.astype(np.int32)).to(dev)
        d_ci = torch.from_numpy(ci).to(dev)
        d_v = torch.from_numpy(rng.uniform(-1, 1, ci.size).astype(np.float32)).to(dev)
        b = synth.dense(0, k, n, device=dev)
        out = torch.empty((m, n), device=dev)
        nnz = ci.size
        ker = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, torch.float32, dev)
        kp = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, torch.float32, dev,
                               ops.make_options(variant=planned_variant))
        key = f"n{n}_L{L}"
        res[key + "_default_us"] = t(lambda: ker(d_rp, d_ci, d_v, b, out))
        res[key + "_small_form"] = ker.ws_bytes == 0
        res[key + "_planned_us"] = t(lambda: kp(d_rp, d_ci, d_v, b, out))
        for cut in (16, 128, 512):
            kc = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, torch.float32, dev,
                                   ops.make_options(heavy=cut))
            res[key + f"_cut{cut}_us"] = t(lambda: kc(d_rp, d_ci, d_v, b, out))
print(json.dumps(res))
