"""Mid-size power-law graphs (2M-15M nonzeros) through probes/probe_forms.py: the automatic form
against the chain-bound configuration (10022) and the mid form with small-launch rows (30002)."""
import sys, os, json
sys.path[:0] = [os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "of-spmm_amd"), os.environ.get("GRAFT_REPO_ROOT", ".")]
import torch
from oneflow_spmm import synth
synth.CONFIGS["p15m"] = dict(m=750_000, k=750_000, nnz=15_000_000, n=16, dtype=torch.float32)
synth.CONFIGS["p5m"] = dict(m=250_000, k=250_000, nnz=5_000_000, n=16, dtype=torch.float32)
synth.CONFIGS["p2m"] = dict(m=100_000, k=100_000, nnz=2_000_000, n=16, dtype=torch.float32)
synth.CONFIGS["p8m"] = dict(m=400_000, k=400_000, nnz=8_000_000, n=16, dtype=torch.float32)
synth.CONFIGS["p11m"] = dict(m=550_000, k=550_000, nnz=11_000_000, n=16, dtype=torch.float32)
# usage: python probes/probe_mid_chain.py [configs] [widths] [variants]
cfgs = sys.argv[1] if len(sys.argv) > 1 else "p2m,p5m,p15m"
widths = sys.argv[2] if len(sys.argv) > 2 else "16,32"
variants = sys.argv[3] if len(sys.argv) > 3 else "0,10022,30002"
sys.argv = ["probe_forms.py", "--configs", cfgs, "--widths", widths, "--variants", variants]
import runpy
runpy.run_path(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "scripts", "probe_forms.py"), run_name="__main__")
