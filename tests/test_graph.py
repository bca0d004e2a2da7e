"""Graph mode by hipGraph capture (oneflow_spmm.graph.SpmmGraph): a
two-layer GCN forward (fused SpMM + bias + relu, then SpMM) captured once and replayed on new
features gives the eager bits; hub rows exercise the planner and the hub reduce inside the graph."""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from tests.helpers import assert_bitwise, power_law_degrees, random_csr, random_dense, to_oracle

pytestmark = pytest.mark.gpu


def test_gcn_forward_graph_replay_matches_eager(device):
    rng = np.random.default_rng(90)
    m, n = 30000, 64
    rp, ci, v = random_csr(m, m, power_law_degrees(m, 600000, m, rng), rng)
    assert int(np.diff(rp.numpy()).max()) > fs.ops.default_split(n)  # hub rows: plan + reduce
    rp, ci, v = rp.to(device), ci.to(device), v.to(device)
    bias = random_dense(1, n, rng)[0].to(device)

    def gcn(x):
        h = fs.fused_spmm(rp, ci, v, m, m, x, bias, relu=True)
        return fs.spmm(rp, ci, v, m, m, h)

    with torch.no_grad():
        g = fs.SpmmGraph(gcn, random_dense(m, n, rng).to(device))
        for seed in (1, 2):
            x = random_dense(m, n, np.random.default_rng(seed)).to(device)
            got = g.run(x).clone()
            ref = gcn(x)
            torch.cuda.synchronize()
            assert_bitwise(got, to_oracle(ref), f"replay {seed}")
    with pytest.raises(ValueError):
        g.run(torch.zeros((m, n + 1), device=device))
