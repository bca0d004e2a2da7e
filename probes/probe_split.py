#!/usr/bin/env python3
"""Round-3 split-contract probe: every launch form on power-law graphs from PubMed size to
products size at several widths, under the new default split (clamp(65536/N, 128, 512)) and, for
the automatic choice, under the round-2 split (cap 8192) passed explicitly, on the same box.

Per (graph, N): the automatic choice (variant 0), the round-2 split with the automatic choice
("old"), and forced configurations (10021 big form U=16, 10022 prefetching U=32, 30000 small form,
30001 mid form big-launch rows, 30002 mid form small-launch rows) where they apply.  Interleaved
rounds, median over rounds of back-to-back launches (HIP events on the launch stream).  Every
variant under the same split must give the same bits (checked; the run stops otherwise).

    python probes/probe_split.py [--graphs pubmed,arxiv,...] [--widths 16,32,64] > out.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

GRAPHS = {  # name: (rows = cols, nonzeros)
    "pubmed": (19_717, 88_648),
    "small20k": (20_000, 400_000),
    "arxiv": (169_343, 1_166_243),
    "g60k": (60_000, 1_500_000),
    "p2m": (100_000, 2_000_000),
    "p5m": (250_000, 5_000_000),
    "p8m": (400_000, 8_000_000),
    "p11m": (550_000, 11_000_000),
    "p15m": (750_000, 15_000_000),
    "plaw1m": (1_000_000, 20_000_000),
    "products": (2_449_029, 123_718_280),
}


def old_split(n):
    t = 65536 // n if n > 0 else 8192
    t = min(max(t, 128), 8192)
    p = 128
    while p * 2 <= t:
        p *= 2
    return p


def alg_bytes(m, nnz, n, s=4):
    return 4 * (m + 1) + 8 * nnz + s * nnz * n + s * m * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default=",".join(GRAPHS))
    ap.add_argument("--widths", default="16,32,64,128")
    ap.add_argument("--variants", default="0,10021,10022,30000,30001,30002,30003,30004")
    ap.add_argument("--no-old", action="store_true", help="skip the round-2 split timing")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--target-ms", type=float, default=3.0, help="time per round per variant")
    args = ap.parse_args()
    from oneflow_spmm import ops, synth
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for name in args.graphs.split(","):
        m, nnz = GRAPHS[name]
        t0 = time.time()
        rp, ci, v = synth.csr(m, m, nnz, threads=16)
        maxdeg = int((rp[1:] - rp[:-1]).max())
        rp, ci, v = rp.to(dev), ci.to(dev), v.to(dev)
        print(f"[probe_split] {name}: {m} rows, {nnz} nnz, max degree {maxdeg} "
              f"({time.time() - t0:.1f} s)", file=sys.stderr, flush=True)
        for n in [int(x) for x in args.widths.split(",")]:
            b = synth.dense(0, m, n, device=dev)
            out = torch.empty((m, n), device=dev)
            kern = {}
            for spec in args.variants.split(","):
                # "<variant>" or "<variant>h<heavy threshold>" (h-1: no heavy bin)
                vs, _, hs = spec.partition("h")
                vv, heavy = int(vs), int(hs) if hs else 0
                if vv in (10021, 10022) and n != 16:
                    continue  # one-element fp32 lanes: N <= 16 only
                if vv == 30000 and nnz * n > (1 << 26):
                    continue  # the small form's block-wide chains: far too slow beyond this
                try:
                    kern[spec] = ops.SpmmCsrKernel(m, m, n, nnz, rp.dtype, b.dtype, dev,
                                                   ops.make_options(variant=vv, heavy=heavy))
                except Exception as e:  # noqa: BLE001  (a variant not applicable to this N)
                    print(f"[probe_split] skip {vv} at n={n}: {e}", file=sys.stderr)
            if not args.no_old:
                kern["old"] = ops.SpmmCsrKernel(m, m, n, nnz, rp.dtype, b.dtype, dev,
                                                ops.make_options(split=old_split(n)))
            ref, times = None, {key: [] for key in kern}
            reps = {}
            for key, kk in kern.items():  # warm-up, bits, reps per round
                kk(rp, ci, v, b, out)
                torch.cuda.synchronize()
                if key != "old":
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(out.view(torch.int32), ref.view(torch.int32)):
                        raise SystemExit(f"{name} n={n} variant {key}: bits differ")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                kk(rp, ci, v, b, out)
                e1.record(stream)
                torch.cuda.synchronize()
                reps[key] = int(min(200, max(3, args.target_ms / max(e0.elapsed_time(e1), 1e-3))))
            for _ in range(args.rounds):
                for key, kk in kern.items():
                    kk(rp, ci, v, b, out)  # untimed: clocks up, the same launch in the caches
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(reps[key]):
                        kk(rp, ci, v, b, out)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    times[key].append(e0.elapsed_time(e1) / reps[key])
            med = {key: float(np.median(t)) for key, t in times.items()}
            auto = med.get("0")
            ab = alg_bytes(m, nnz, n)
            rec = {"graph": name, "m": m, "nnz": nnz, "max_degree": maxdeg, "n": n,
                   "split": ops.default_split(n), "old_split": old_split(n),
                   "us": {key: round(t * 1e3, 2) for key, t in med.items()},
                   "best": min(med, key=med.get),
                   "auto_tbps": round(ab / (auto * 1e-3) / 1e12, 3) if auto else None,
                   "auto_frac": round(ab / (auto * 1e-3) / 8e12, 3) if auto else None,
                   "bitexact_across_variants": True}
            print(json.dumps(rec), flush=True)
            del kern, out, b
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
