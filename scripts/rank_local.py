#!/usr/bin/env python3
"""The SpMM phase of a G-rank row split, measured rank by rank on ONE GPU: for every rank r, the
local CSR slice (BalancedSplitter rows, row_ptr rebased, columns remapped into the padded
gathered layout) times the full gathered B, exactly what rank r's kernel does after the
exchange.  Reports per-rank ms and the whole-job SpMM-phase GFLOP/s = 2*nnz*N / max_r(ms)
(the exchange itself needs the G GPUs and is not included).

--cn C > 1 measures the R x C grid exchange (distributed.GridPlan, R = G/C) instead: per row
group, the SpMM of the group's rows (global-form launch on the whole CSR) against one N/C column
block of B, plus the rank-local copies of its step (packing the shard into C blocks, unpacking C
blocks of its output rows).  Those are the grid's compute phase; its two exchanges move
(G-1)/G * |B|/C and (C-1)/C * |C|/G per rank.

    python scripts/rank_local.py --config products --world 8 [--cn 4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "of-spmm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cn", type=int, default=1)
    args = ap.parse_args()
    if args.cn > 1:
        return grid(args)
    from oneflow_spmm import _C, ops, synth
    from oneflow_spmm.distributed import padded_owner_remap

    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    G = args.world
    dev = torch.device("cuda", 0)
    rp = synth.row_ptr(m, k, nnz)
    pad = -(-k // G)
    gathered = torch.zeros((G * pad, n), dtype=dt, device=dev)
    for r in range(G):
        lo, hi = _C.balanced_range(k, G, r)
        gathered[r * pad: r * pad + hi - lo] = synth.dense(lo, hi, n, dt, device=dev)
    opts = ops.make_options(split=ops.default_split(n))
    res, e0, e1 = [], torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(G):
        lo, hi = _C.balanced_range(m, G, r)
        j0, j1 = int(rp[lo]), int(rp[hi])
        cols = torch.from_numpy(synth.columns(m, k, rp, lo, hi, threads=16))
        d_ci = padded_owner_remap(cols, k, G).to(dev)
        d_rp = torch.from_numpy((rp[lo:hi + 1] - rp[lo]).astype(np.int32)).to(dev)
        d_v = synth.values(j0, j1, dt).to(dev)
        out = torch.empty((hi - lo, n), dtype=dt, device=dev)
        kern = ops.SpmmCsrKernel(hi - lo, G * pad, n, j1 - j0, torch.int32, dt, dev, opts)
        kern(d_rp, d_ci, d_v, gathered, out)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0.record()
            kern(d_rp, d_ci, d_v, gathered, out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res.append({"rank": r, "rows": hi - lo, "nnz": j1 - j0, "ms": round(float(np.median(ts)), 4)})
        del d_ci, d_rp, d_v, out, kern
    worst = max(x["ms"] for x in res)
    print(json.dumps({"config": args.config, "world": G, "per_rank": res, "max_ms": worst,
                      "spmm_phase_gflops_aggregate": round(2.0 * nnz * n / (worst * 1e-3) / 1e9, 1)}))


def _median_ms(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def grid(args):
    from oneflow_spmm import _C, ops, synth
    from oneflow_spmm.distributed import _copy_rows

    cfg = synth.CONFIGS[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    G, C = args.world, args.cn
    R, nb = G // C, n // C
    assert G % C == 0 and n % C == 0
    dev = torch.device("cuda", 0)
    rp = synth.row_ptr(m, k, nnz)
    d_rp = torch.from_numpy(rp.astype(np.int32)).to(dev)
    d_ci = torch.from_numpy(synth.columns(m, k, rp, threads=16)).to(dev)
    d_v = synth.values(0, nnz, dt).to(dev)
    b_blk = synth.dense(0, k, n, dt, device=dev)[:, :nb].contiguous()
    opts = ops.make_options(split=ops.default_split(n))
    kern = ops.SpmmCsrKernel(m, k, nb, nnz, torch.int32, dt, dev, opts)
    # rank-local copies of a step, sized for rank 0 (the largest shard / row range)
    k0 = _C.balanced_range(k, G, 0)[1]
    m0 = _C.balanced_range(m, G, 0)[1]
    shard = torch.zeros((k0, n), dtype=dt, device=dev)
    send_b = torch.empty((C * k0, nb), dtype=dt, device=dev)
    recv_c = torch.empty((C * m0, nb), dtype=dt, device=dev)
    out = torch.empty((m0, n), dtype=dt, device=dev)

    def copies_per_block():  # the CPU-path form: one copy per block each way
        for b in range(C):
            _copy_rows(send_b[b * k0:(b + 1) * k0], shard[:, b * nb:(b + 1) * nb])
        for b in range(C):
            _copy_rows(out[:, b * nb:(b + 1) * nb], recv_c[b * m0:(b + 1) * m0])

    from oneflow_spmm._C import current_stream_handle
    from oneflow_spmm._lib import LIB, check
    e = shard.element_size()
    b_own = torch.empty((k, nb), dtype=dt, device=dev)

    def copies():  # GridPlan's GPU form: ofx_copy_blocks, two launches each way
        st = current_stream_handle(shard)
        check(LIB.ofx_copy_blocks(st, 1, C, k0, nb * e, shard.data_ptr(), 0, nb * e, n * e,
                                  send_b.data_ptr(), 0, k0 * nb * e, nb * e), "copy_blocks")
        check(LIB.ofx_copy_blocks(st, 1, 1, k0, nb * e, shard.data_ptr(), 0, 0, n * e,
                                  b_own.data_ptr(), 0, 0, nb * e), "copy_blocks")
        if C > 1:  # rank 0 sits at column 0: the received blocks are 1..C-1
            check(LIB.ofx_copy_blocks(st, 1, C - 1, m0, nb * e, recv_c.data_ptr() + m0 * nb * e, 0,
                                      m0 * nb * e, nb * e, out.data_ptr() + nb * e, 0, nb * e,
                                      n * e), "copy_blocks")
        check(LIB.ofx_copy_blocks(st, 1, 1, m0, nb * e, recv_c.data_ptr(), 0, 0, nb * e,
                                  out.data_ptr(), 0, 0, n * e), "copy_blocks")
    copy_ms = _median_ms(copies, args.reps)
    copy_ms_per_block = _median_ms(copies_per_block, args.reps)
    res = []
    for g in range(R):
        lo = _C.balanced_range(m, G, g * C)[0]
        hi = _C.balanced_range(m, G, g * C + C - 1)[1]
        c_grp = torch.empty((hi - lo, nb), dtype=dt, device=dev)
        ms = _median_ms(lambda: kern(d_rp, d_ci, d_v, b_blk, c_grp, lo, hi), args.reps)
        res.append({"row_group": g, "rows": hi - lo, "nnz": int(rp[hi] - rp[lo]), "ms": round(ms, 4)})
        del c_grp
    worst = max(x["ms"] for x in res)
    s_v = torch.empty(0, dtype=dt).element_size()
    print(json.dumps({"config": args.config, "world": G, "grid": f"{R}x{C}", "block_n": nb,
                      "per_row_group": res, "max_spmm_ms": worst, "local_copies_ms": round(copy_ms, 4),
                      "local_copies_ms_per_block_form": round(copy_ms_per_block, 4),
                      "b_bytes_received_per_rank": (k - k0) * nb * s_v,
                      "c_bytes_received_per_rank": (C - 1) * m0 * nb * s_v,
                      "spmm_phase_gflops_aggregate": round(2.0 * nnz * n / ((worst + copy_ms) * 1e-3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
