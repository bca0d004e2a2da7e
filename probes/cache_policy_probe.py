#!/usr/bin/env python3
"""Probe (not product code): products-shaped B-row gather (N=128 fp32) with the B loads steered
by column hotness through the cache-policy bits (probes/cache_policy_probe.hip).  The top-T
columns by in-degree load with the default policy, the rest with the mode's policy; T sweeps
from the L2's share (8k rows) to twice the Infinity Cache (1M rows).  Modes are interleaved
and each timing is the median of 3 rounds of 5 launches (HIP events).

    python probes/cache_policy_probe.py          # prints one JSON line per (T, mode)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]
SO = os.path.join(ROOT, "scripts", "_cache_policy_probe.so")
MODES = {0: "all default", 1: "all nt", 2: "cold nt", 3: "cold sc1", 4: "cold nt|sc1",
         5: "cold sc0", 6: "cold sc0|nt", 7: "cold sc0|sc1", 8: "cold sc0|nt|sc1",
         9: "cold nt via bitmap lookup", 10: "hot sc1, cold nt"}


def build():
    src = os.path.join(ROOT, "scripts", "cache_policy_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", SO],
                       check=True)


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "--build-only":
        return
    import torch
    from oneflow_spmm import synth
    lib = ctypes.CDLL(SO)
    lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    cfg = synth.CONFIGS["products"]
    m, k, nnz, n = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"]
    dev = torch.device("cuda", 0)
    _, ci, _ = synth.csr(m, k, nnz, threads=16)
    col = ci.to(dev)
    b = synth.dense(0, k, n, device=dev)
    deg = torch.bincount(col.long(), minlength=k)
    order = torch.argsort(deg, descending=True)
    groups = (nnz + 511) // 512
    out = torch.empty(groups * 32 * 4, dtype=torch.float32, device=dev)
    ref = None
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    print(json.dumps({"probe": "cache_policy", "nnz": nnz, "k": k, "n": n,
                      "deg_max": int(deg.max()), "deg_min": int(deg.min())}), flush=True)
    # the per-launch hint pass (sampled counts -> threshold -> bitmap), timed, then the gather
    # with its bitmap against the default policy, interleaved
    lib.probe_hints.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    ws = torch.empty(k + 256, dtype=torch.int32, device=dev)
    hbits = torch.empty((k + 31) // 32, dtype=torch.int32, device=dev)
    for T in (32768, 65536, 131072):
        for sb in (8, 32, 128):
            hargs = (col.data_ptr(), nnz, k, T, sb, ws.data_ptr(), hbits.data_ptr(), stream.cuda_stream)
            assert lib.probe_hints(*hargs) == 0
            torch.cuda.synchronize()
            ev[0].record(stream)
            for _ in range(10):
                lib.probe_hints(*hargs)
            ev[1].record(stream)
            torch.cuda.synchronize()
            hint_ms = ev[0].elapsed_time(ev[1]) / 10
            nhot = int(np.unpackbits(hbits.cpu().numpy().view(np.uint8)).sum())
            hot_share = float(deg[torch.from_numpy(np.unpackbits(hbits.cpu().numpy().view(np.uint8),
                                                                 bitorder="little")[:k].astype(bool)).to(dev)].sum()) / nnz
            tt = {0: [], 9: []}
            for _ in range(3):
                for md in (0, 9):
                    args = (md, col.data_ptr(), hbits.data_ptr(), b.data_ptr(), nnz, b.numel() * 4,
                            out.data_ptr(), stream.cuda_stream)
                    ev[0].record(stream)
                    for _ in range(5):
                        lib.probe_launch(*args)
                    ev[1].record(stream)
                    torch.cuda.synchronize()
                    tt[md].append(ev[0].elapsed_time(ev[1]) / 5)
            t0, t9 = float(np.median(tt[0])), float(np.median(tt[9]))
            print(json.dumps({"hint_pass": True, "target": T, "sample_every_runs": sb,
                              "hint_ms": round(hint_ms, 4), "hot_columns": nhot,
                              "hot_share_of_refs": round(hot_share, 4), "default_ms": round(t0, 4),
                              "bitmap_cold_nt_ms": round(t9, 4), "vs_default": round(t9 / t0, 4),
                              "with_hint_pass": round((t9 + hint_ms) / t0, 4)}), flush=True)
    if os.environ.get("PROBE_HINTS_ONLY"):
        return
    for T in (8192, 65536, 262144, 524288, 1048576):
        hot = torch.zeros(k, dtype=torch.bool, device=dev)
        hot[order[:T]] = True
        share = float(deg[order[:T]].sum()) / nnz
        cold = ~hot[col.long()]
        tagged = torch.where(cold, col | torch.tensor(-2 ** 31, dtype=torch.int32, device=dev), col)
        hb = np.zeros(((k + 31) // 32) * 32, dtype=np.uint32)
        hb[:k] = hot.cpu().numpy()
        words = (hb.reshape(-1, 32) << np.arange(32, dtype=np.uint32)).sum(1, dtype=np.uint64)
        bits = torch.from_numpy(words.astype(np.uint32).view(np.int32)).to(dev)
        times = {md: [] for md in MODES}
        for _ in range(3):
            for md in MODES:
                c = col if md == 9 else tagged
                args = (md, c.data_ptr(), bits.data_ptr(), b.data_ptr(), nnz, b.numel() * 4,
                        out.data_ptr(), stream.cuda_stream)
                assert lib.probe_launch(*args) == 0
                torch.cuda.synchronize()
                if md == 0 and ref is None:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    raise SystemExit(f"mode {md}: the sums differ from mode 0")
                ev[0].record(stream)
                for _ in range(5):
                    lib.probe_launch(*args)
                ev[1].record(stream)
                torch.cuda.synchronize()
                times[md].append(ev[0].elapsed_time(ev[1]) / 5)
        base = float(np.median(times[0]))
        for md in MODES:
            t = float(np.median(times[md]))
            print(json.dumps({"hot_columns": T, "hot_share_of_refs": round(share, 4), "mode": md,
                              "policy": MODES[md], "ms": round(t, 4),
                              "vs_default": round(t / base, 4)}), flush=True)


if __name__ == "__main__":
    main()
