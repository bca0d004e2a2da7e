#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ (committed together with this script).

The reference (OneFlow v0.8.1-dev) holds no SpMM and no fixture for one, so
these vectors are built from independent implementations available here:
  * expected_f64   scipy.sparse.csr_matrix(...) @ B in float64 (scipy 1.15)
  * expected_t32   torch.sparse_csr_tensor(...) @ B in float32 (torch 2.10, CPU)
  * exact cases    integer-valued inputs whose partial sums are exact in fp32, so every
                   summation order gives the same bits
  * split cases    BalancedSplitter ranges (restated from oneflow/core/common/balanced_splitter.cpp:20-40
                   by its documented rule: the first total % parts parts get one extra element),
                   rebased row_ptr slices and the padded all-gather column remap.
Inputs are drawn with numpy's PCG64 (seeded), not with the product's generator.

    python tests/golden/make_golden.py   # rewrites tests/golden/*.npz and MANIFEST.json
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import scipy
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def power_law_degrees(m, nnz, k, rng, gamma=2.5):
    w = np.arange(1, m + 1, dtype=np.float64) ** (-1.0 / (gamma - 1.0))
    d = np.minimum(np.floor(nnz * w / w.sum()).astype(np.int64), k)
    i = 0
    while d.sum() < nnz:
        if d[i % m] < k:
            d[i % m] += 1
        i += 1
    rng.shuffle(d)
    return d


def make_csr(m, k, degrees, rng, exact=False):
    rp = np.zeros(m + 1, dtype=np.int64)
    rp[1:] = np.cumsum(degrees)
    cols = np.concatenate([np.sort(rng.choice(k, size=d, replace=False)) for d in degrees]
                          + [np.zeros(0, dtype=np.int64)]).astype(np.int64)
    if exact:
        vals = rng.choice(np.array([-2.0, -1.0, 1.0, 2.0], dtype=np.float32), size=rp[-1])
    else:
        vals = rng.uniform(-1, 1, size=rp[-1]).astype(np.float32)
    return rp, cols, vals


def dense(k, n, rng, exact=False):
    if exact:
        return rng.integers(-8, 9, size=(k, n)).astype(np.float32)
    return rng.uniform(-1, 1, size=(k, n)).astype(np.float32)


def expected(rp, cols, vals, b, m, k):
    a64 = sp.csr_matrix((vals.astype(np.float64), cols, rp), shape=(m, k))
    e64 = a64 @ b.astype(np.float64)
    absum = abs(a64) @ np.abs(b.astype(np.float64))
    t = torch.sparse_csr_tensor(torch.from_numpy(rp), torch.from_numpy(cols), torch.from_numpy(vals),
                                size=(m, k))
    e32 = (t @ torch.from_numpy(b)).numpy()
    return e64, absum, e32


def main():
    rng = np.random.default_rng(20261015)
    cases = {}
    # Cora-shaped: 2708 x 2708, 10,556 nnz, N=16
    m = k = 2708
    rp, c, v = make_csr(m, k, power_law_degrees(m, 10556, k, rng), rng)
    b = dense(k, 16, rng)
    cases["cora_f32"] = (rp, c, v, b, m, k)
    rp, c, v = make_csr(m, k, power_law_degrees(m, 10556, k, rng), rng, exact=True)
    b = dense(k, 16, rng, exact=True)
    cases["cora_exact"] = (rp, c, v, b, m, k)
    # widths, K != M, empty rows, one hub row
    for n in (1, 3, 17, 64):
        m, k = 97, 131
        deg = rng.integers(0, 12, size=m)
        deg[0] = 0
        deg[50] = 120
        rp, c, v = make_csr(m, k, deg, rng)
        cases[f"n{n}_f32"] = (rp, c, v, dense(k, n, rng), m, k)
    m, k = 12, 3000
    deg = np.array([0, 1, 2, 2900, 0, 5, 700, 0, 0, 33, 1, 2999])
    rp, c, v = make_csr(m, k, deg, rng)
    cases["hub_n128_f32"] = (rp, c, v, dense(k, 128, rng), m, k)
    rp, c, v = make_csr(m, k, deg, rng, exact=True)
    cases["hub_n128_exact"] = (rp, c, v, dense(k, 128, rng, exact=True), m, k)
    # all rows empty
    m, k = 9, 4
    cases["empty_f32"] = (np.zeros(m + 1, dtype=np.int64), np.zeros(0, dtype=np.int64),
                          np.zeros(0, dtype=np.float32), dense(k, 8, rng), m, k)

    manifest = {"generator": "tests/golden/make_golden.py", "numpy": np.__version__,
                "scipy": scipy.__version__, "torch": torch.__version__, "files": {}}
    for name, (rp, c, v, b, m, k) in cases.items():
        e64, absum, e32 = expected(rp, c, v, b, m, k)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, row_ptr=rp, col_idx=c, values=v, b=b, m=m, k=k,
                            expected_f64=e64, absum=absum, expected_t32=e32)
        manifest["files"][f"{name}.npz"] = hashlib.sha256(open(path, "rb").read()).hexdigest()

    # partition fixtures (integers: bit-exact)
    parts = {}
    for total in (0, 1, 7, 8, 2708, 232_965, 2_449_029, 111_059_956):
        for g in (1, 2, 3, 4, 8):
            base, extra = divmod(total, g)
            ranges = []
            lo = 0
            for r in range(g):
                size = base + (1 if r < extra else 0)
                ranges.append([lo, lo + size])
                lo += size
            parts[f"{total}/{g}"] = ranges
    m, k = 50, 23
    rp, c, v = make_csr(m, k, rng.integers(0, 9, size=m), rng)
    slices = {}
    for g in (2, 4, 8):
        for r in range(g):
            lo, hi = parts_range(m, g, r)
            slices[f"{g}/{r}"] = {"rows": [lo, hi], "row_ptr": (rp[lo:hi + 1] - rp[lo]).tolist(),
                                  "nnz": [int(rp[lo]), int(rp[hi])]}
    remap = {}
    for g in (2, 3, 4, 8):
        base, extra = divmod(k, g)
        pad = -(-k // g)
        out = []
        for col in range(k):
            owner = col // (base + 1) if col < extra * (base + 1) else extra + (col - extra * (base + 1)) // base
            lo = parts_range(k, g, owner)[0]
            out.append(owner * pad + (col - lo))
        remap[str(g)] = out
    with open(os.path.join(HERE, "partition.json"), "w") as f:
        json.dump({"balanced": parts, "row_ptr": rp.tolist(), "k": k, "slices": slices,
                   "padded_remap": remap}, f)
    manifest["files"]["partition.json"] = hashlib.sha256(
        open(os.path.join(HERE, "partition.json"), "rb").read()).hexdigest()

    # fused epilogue fixtures (op fused_spmm_csr): relu(A @ B + bias) from scipy's fp64 product,
    # numpy's bias add and max(x, 0); exact mode (integers, every step exact in fp32) and a
    # random fp32 case (tolerance).  Separate RNG, so the fixtures above are unchanged.
    frng = np.random.default_rng(20261016)
    for name, exact in (("fused_exact", True), ("fused_f32", False)):
        m, k, n = 300, 250, 24
        deg = frng.integers(0, 15, size=m)
        deg[7] = 0
        rp, c, v = make_csr(m, k, deg, frng, exact=exact)
        b = dense(k, n, frng, exact=exact)
        bias = (frng.integers(-8, 9, size=n) if exact else frng.uniform(-1, 1, size=n)).astype(np.float32)
        e64, absum, _ = expected(rp, c, v, b, m, k)
        relu = np.maximum(e64 + bias.astype(np.float64)[None, :], 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, row_ptr=rp, col_idx=c, values=v, b=b, bias=bias, m=m, k=k,
                            expected_relu_f64=relu, absum=absum)
        manifest["files"][f"{name}.npz"] = hashlib.sha256(open(path, "rb").read()).hexdigest()

    # N = 256 (the Reddit configuration's width): at N = 256 the split is 256
    # nonzeros, so the 900- and 600-nonzero rows are hubs of 3 and 2 chunks, the 256-nonzero row
    # is one chunk exactly and the 257-nonzero row is just over.  Separate RNG: the fixtures above
    # are unchanged.
    nrng = np.random.default_rng(20261017)
    m, k, n = 120, 1000, 256
    deg = nrng.integers(0, 40, size=m)
    deg[[0, 5, 60, 61, 119]] = [0, 900, 256, 257, 600]
    for name, exact in (("n256_f32", False), ("n256_exact", True)):
        rp, c, v = make_csr(m, k, deg, nrng, exact=exact)
        b = dense(k, n, nrng, exact=exact)
        e64, absum, e32 = expected(rp, c, v, b, m, k)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, row_ptr=rp, col_idx=c, values=v, b=b, m=m, k=k,
                            expected_f64=e64, absum=absum, expected_t32=e32)
        manifest["files"][f"{name}.npz"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest["files"]), "fixtures")


def parts_range(total, g, r):
    base, extra = divmod(total, g)
    lo = r * (base + 1) if r < extra else extra * (base + 1) + (r - extra) * base
    return lo, lo + base + (1 if r < extra else 0)


if __name__ == "__main__":
    main()
