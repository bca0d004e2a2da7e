#!/usr/bin/env python3
"""Dense-width sweep of the op on one graph (generated once): per (dtype, N) the median op time
over interleaved rounds (HIP events on the launch stream), the gather-model rate and its fraction
of 8 TB/s, and a sampled bit-exact check of the first rows against the oracle.

    python scripts/width_sweep.py [--config products] [--widths 1,2,4,...] [--dtypes f32,bf16]

One JSON line per (dtype, N)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--graph", default="", help="rows:nonzeros of a synthetic power-law graph "
                                                   "(rows = cols) instead of --config")
    ap.add_argument("--widths", default="1,2,4,8,16,32,64,128,256,512")
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--idx", default="int32", choices=["int32", "int64"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0",
                    help="kernel variants per (dtype, N): 0 = auto, VEC*100+LPR forces one "
                         "(skipped where it does not apply); bits compared with the auto variant")
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import ops, synth
    from bench import alg_bytes
    from oracle import oracle

    if args.graph:
        m, nnz = (int(x) for x in args.graph.split(":"))
        k = m
        args.config = f"graph{m}x{nnz}"
    else:
        cfg = synth.CONFIGS[args.config]
        m, k, nnz = cfg["m"], cfg["k"], cfg["nnz"]
    dev = torch.device("cuda", 0)
    rp, ci, v32 = synth.csr(m, k, nnz, val_dtype=torch.float32, threads=16)
    if args.idx == "int64":
        rp, ci = rp.to(torch.int64), ci.to(torch.int64)
    d_rp, d_ci = rp.to(dev), ci.to(dev)
    rows_chk = 2000
    for dname in args.dtypes.split(","):
        dt = DT[dname]
        d_v = v32.to(dt).to(dev)
        for n in [int(x) for x in args.widths.split(",")]:
            b = synth.dense(0, k, n, dt, device=dev)
            out = torch.empty((m, n), dtype=dt, device=dev)
            fs.spmm(d_rp, d_ci, d_v, m, k, b, out=out)
            torch.cuda.synchronize()
            # sampled check: the first rows against the oracle
            def host(t):
                t = t.cpu()
                return t.view(torch.int16).numpy().view(np.uint16) if dt == torch.bfloat16 else t.numpy()
            ref = oracle.spmm(rp.numpy(), ci.numpy(), host(d_v), host(b), dtype=dname, row_end=rows_chk)
            ok = bool(np.array_equal(host(out[:rows_chk]).view(np.uint8), ref.view(np.uint8)))
            for var in [int(x) for x in args.variants.split(",")]:
                if var:
                    vec, lpr = var // 100, var % 100
                    if var < 10000 and (n % vec or vec * b.element_size() > 16 or
                                        vec * lpr > 4 * max(n, 1) + 64):
                        continue
                    opts = ops.make_options(variant=var)

                    def call():
                        ops.spmm_csr_device(d_rp, d_ci, d_v, b, m, k, out=o2, options=opts)
                    o2 = torch.empty_like(out)
                    try:  # tuning-table entries (10000 + id) refuse the dtypes / widths they lack
                        call()
                    except fs.OfxError:
                        continue
                    torch.cuda.synchronize()
                    same = bool(torch.equal(o2.view(torch.uint8), out.view(torch.uint8)))
                else:
                    def call():
                        fs.spmm(d_rp, d_ci, d_v, m, k, b, out=out)
                    same = True
                ts = []
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(args.rounds):
                    e0.record()
                    for _ in range(args.reps):
                        call()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / args.reps)
                ms = float(np.median(ts))
                ab = alg_bytes(m, nnz, n, b.element_size())
                print(json.dumps({"config": args.config, "dtype": dname, "idx": args.idx, "n": n, "variant": var,
                                  "ms": round(ms, 4),
                                  "gflops": round(2.0 * nnz * n / (ms * 1e-3) / 1e9, 1),
                                  "gather_model_gbs": round(ab / (ms * 1e-3) / 1e9, 1),
                                  "frac_of_8tbs": round(ab / (ms * 1e-3) / 8e12, 3),
                                  "b_mb": round(k * n * b.element_size() / 1e6, 1),
                                  "first_rows_bitexact": ok, "bits_equal_auto": same}), flush=True)
            del b, out


if __name__ == "__main__":
    main()
