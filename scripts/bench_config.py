#!/usr/bin/env python3
"""Single-GPU throughput of one BASELINE config through the op layer, with a sampled bit-exact
check against the oracle (first/last rows, a middle block and the heaviest rows).

    python scripts/bench_config.py --config papers [--reps 5]

Prints one JSON line: time, GFLOP/s, gather-model GB/s and fraction of 8 TB/s, and the check."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def log(msg):
    print(f"[bench_config {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def heartbeat(stop: threading.Event, period: float = 30.0):
    """Papers-scale phases (host generation of 1.6B columns, the 57 GB B copy for the check)
    run minutes without output; a line every 30 s keeps the run visibly alive."""
    t0 = time.time()
    while not stop.wait(period):
        log(f"... {time.time() - t0:.0f} s")


def main():
    stop = threading.Event()
    threading.Thread(target=heartbeat, args=(stop,), daemon=True).start()
    try:
        run()
    finally:
        stop.set()


def run():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="papers")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--n", type=int, default=0, help="override the dense width")
    ap.add_argument("--no-check", action="store_true", help="skip the sampled oracle check")
    args = ap.parse_args()
    import oneflow_spmm as fs
    from oneflow_spmm import synth
    from bench import alg_bytes
    from oracle import oracle

    cfg = {**synth.CONFIGS, **synth.EXTRA_CONFIGS}[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    n = args.n or n
    dev = torch.device("cuda", 0)
    t0 = time.time()
    rp_full = synth.row_ptr(m, k, nnz)
    wide = nnz >= 2**31 or k >= 2**31
    cols = synth.columns(m, k, rp_full, threads=args.threads,
                         idx_dtype=np.int64 if wide else np.int32)
    vals = synth.values(0, nnz, dt)
    t_gen = time.time() - t0
    d_rp = torch.from_numpy(rp_full.astype(np.int64 if wide else np.int32)).to(dev)
    d_ci = torch.from_numpy(cols).to(dev)
    d_v = vals.to(dev)
    d_b = synth.dense(0, k, n, dt, device=dev)
    out = torch.empty((m, n), dtype=dt, device=dev)
    log("inputs resident; timing")
    fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(args.reps):
        e0.record()
        fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    log(f"median {ms:.3f} ms; checking sampled rows against the oracle")
    if args.no_check:
        print(json.dumps({"config": args.config, "n": n, "ms": round(ms, 3),
                          "gather_model_gbs": round(alg_bytes(m, nnz, n, d_b.element_size(), 8 if wide else 4) /
                                                    (ms * 1e-3) / 1e9, 1)}), flush=True)
        return
    sv = d_b.element_size()
    nbytes = alg_bytes(m, nnz, n, sv, 8 if wide else 4)
    # sampled check (bit-exact vs oracle with the operator's schedule)
    deg = np.diff(rp_full)
    heavy = np.argsort(deg)[-20:]
    ranges = [(0, 2000), (m // 2, m // 2 + 2000), (m - 2000, m)] + [(int(r), int(r) + 1) for r in heavy]
    if wide and nnz > 2**31:  # rows whose nonzeros straddle position 2^31
        rc = int(np.searchsorted(rp_full, 2**31, side="right")) - 1
        ranges.append((max(rc - 1000, 0), min(rc + 1000, m)))
    b_rows_needed = None  # oracle reads B rows through col; copy B to host once
    b_host = d_b.cpu()
    b_np = b_host.numpy() if dt != torch.bfloat16 else b_host.view(torch.int16).numpy().view(np.uint16)
    v_np = vals.numpy() if dt != torch.bfloat16 else vals.view(torch.int16).numpy().view(np.uint16)
    dname = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16", torch.float64: "f64"}[dt]
    ok = True
    for lo, hi in ranges:
        ref = oracle.spmm(rp_full, cols, v_np, b_np, dtype=dname, row_begin=lo, row_end=hi,
                          nthreads=args.threads)
        got = out[lo:hi].cpu()
        got = got.numpy() if dt != torch.bfloat16 else got.view(torch.int16).numpy().view(np.uint16)
        ok = ok and np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                   np.ascontiguousarray(ref).view(np.uint8))
    del b_rows_needed
    print(json.dumps({
        "config": args.config, "m": m, "nnz": nnz, "n": n, "dtype": dname,
        "index": "int64" if wide else "int32",
        "max_degree": int(deg.max()), "gen_s": round(t_gen, 1), "ms": round(ms, 3),
        "gflops": round(2.0 * nnz * n / (ms * 1e-3) / 1e9, 1),
        "gather_model_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1),
        "frac_of_8tbs": round(nbytes / (ms * 1e-3) / 8e12, 4),
        "sampled_rows_bitexact": bool(ok), "sampled_ranges": len(ranges)}), flush=True)


if __name__ == "__main__":
    main()
