#!/usr/bin/env python3
"""Extracts the reference's own golden vectors for the two building blocks of the SpMM path into
tests/golden/ref_embedding_scale_by_freq.npz (committed together with this script).

The reference has no SpMM, but its embedding test holds literal inputs and expected outputs of
exactly the two CPU building blocks the SpMM composition is made of:
  * the forward, EmbeddingFunctor<kCPU> (oneflow/user/kernels/embedding_kernel_util.cpp:48-60):
    out[i, :] = weight[indices[i], :], a row copy (std::copy) -- the gather of
    gather_kernel_util.cpp:72-92;
  * the backward, EmbeddingGradFunctor<kCPU> (embedding_kernel_util.cpp:63-88): for i ascending,
    dx[indices[i], :] = dy[i, :] + dx[indices[i], :] (std::transform with std::plus), then each
    row divided by its index's frequency when that is > 1 -- the segment sum of
    unsorted_segment_sum_kernel_util.cpp:29-45 plus the scale.
The test is python/oneflow/test/modules/test_sparse.py:76-134 (_test_embedding_scale_by_freq):
weight [10, 3] fp32, indices [2, 4], the expected forward output [2, 4, 3] (allclose 1e-5) and
the expected weight gradient of y.sum() [10, 3] (allclose 1e-5).

The reference is read as text and its literals are evaluated with ast.literal_eval: nothing from
it is imported or run.  The fixture is data (inputs and expected outputs), with the file:line of
every array recorded beside it.

    python tests/golden/make_reference_fixtures.py [/root/reference]
"""
from __future__ import annotations

import ast
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REL = "python/oneflow/test/modules/test_sparse.py"
FUNC = "_test_embedding_scale_by_freq"


def _literal(call: ast.Call):
    """The first positional argument of np.array(...) / flow.tensor(...) as a Python literal."""
    return ast.literal_eval(call.args[0])


def extract(ref_root: str) -> dict:
    path = os.path.join(ref_root, REL)
    tree = ast.parse(open(path).read(), filename=path)
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == FUNC)
    found, lines = {}, {}
    for node in ast.walk(fn):
        if not isinstance(node, ast.Assign) or len(node.targets) != 1:
            continue
        target = node.targets[0]
        if not isinstance(target, ast.Name):
            continue
        name, value = target.id, node.value
        if name in found:
            continue
        if isinstance(value, ast.Call) and isinstance(value.func, ast.Attribute) and value.args:
            callee = f"{getattr(value.func.value, 'id', '?')}.{value.func.attr}"
            if callee in ("np.array", "flow.tensor"):
                found[name] = _literal(value)
                lines[name] = f"{REL}:{node.lineno}-{node.end_lineno}"
        elif isinstance(value, ast.List):  # weight_grad_np = [[...], ...]
            found[name] = ast.literal_eval(value)
            lines[name] = f"{REL}:{node.lineno}-{node.end_lineno}"
    need = {"weight", "output", "indices", "weight_grad_np"}
    missing = need - set(found)
    if missing:
        raise SystemExit(f"{path}:{FUNC}: literals not found: {sorted(missing)}")
    return {"weight": np.asarray(found["weight"], dtype=np.float32),
            "indices": np.asarray(found["indices"], dtype=np.int32),
            "output": np.asarray(found["output"], dtype=np.float32),
            "weight_grad": np.asarray(found["weight_grad_np"], dtype=np.float32),
            "source": json.dumps({"function": f"{REL}:{fn.lineno} {FUNC}", "arrays": {
                "weight": lines["weight"], "indices": lines["indices"],
                "output": lines["output"], "weight_grad": lines["weight_grad_np"]},
                "kernels": {"forward": "oneflow/user/kernels/embedding_kernel_util.cpp:48-60",
                            "backward": "oneflow/user/kernels/embedding_kernel_util.cpp:63-88"},
                "tolerance": "np.allclose(rtol=1e-5, atol=1e-5) in the reference test"})}


def main():
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    fx = extract(ref_root)
    out = os.path.join(HERE, "ref_embedding_scale_by_freq.npz")
    np.savez(out, **fx)
    print(f"wrote {out}: weight {fx['weight'].shape}, indices {fx['indices'].shape}, "
          f"output {fx['output'].shape}, weight_grad {fx['weight_grad'].shape}")


if __name__ == "__main__":
    main()
