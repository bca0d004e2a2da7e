"""Mid-size launches (above the small form's 2^20 products): the default choice against the small
form (tuning variant 30000, one launch) and the mid form (30001: block items + big-launch light
rows; 30002: block items + prefetching light rows), with the block-item cut varied.  Prints one
JSON object."""
import json
import sys

sys.path[:0] = ["/root/repo/of-spmm_amd", "/root/repo"]
import torch  # noqa: E402

from oneflow_spmm import ops, synth  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, reps=100):
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
graphs = {"pubmed": (19717, 88648), "small20k": (20000, 400000), "arxiv": (169343, 1166243),
          "g60k": (60000, 1500000)}
for name, (m, nnz) in graphs.items():
    rp, ci, v = synth.csr(m, m, nnz)
    res[f"{name}_maxdeg"] = int((rp[1:] - rp[:-1]).max())
    rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
    for n in (16, 64, 128):
        b = synth.dense(0, m, n, device=dev)
        out = torch.empty((m, n), device=dev)
        ref = None
        for label, opts in {"default": None,
                            "small": ops.make_options(variant=30000),
                            "mid": ops.make_options(variant=30001),
                            "mid_sr": ops.make_options(variant=30002),
                            "mid_cut32": ops.make_options(variant=30001, heavy=32),
                            "mid_sr_cut32": ops.make_options(variant=30002, heavy=32)}.items():
            k = ops.SpmmCsrKernel(m, m, n, nnz, torch.int32, torch.float32, dev, opts)
            res[f"{name}_n{n}_{label}_us"] = t(lambda: k(rp, ci, v, b, out))
            if ref is None:
                ref = out.clone()
            else:
                res[f"{name}_n{n}_{label}_same_bits"] = bool(torch.equal(ref.view(torch.int32),
                                                                         out.view(torch.int32)))
print(json.dumps(res))
