"""Diagnostic: per-gradient error of the HIP block vs the fp64 oracle over a
sweep of shapes (prints one line per case)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from stgcn_loader import load
from oracle import ref_cpu
import test_gpu_block as tg
from conftest import rel_to_max

pkg = load()
cases = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]] or [
    (3, 64, 1, 18, 1, 2, 32), (3, 64, 1, 18, 1, 3, 32), (3, 64, 1, 18, 1, 2, 45),
    (3, 64, 1, 18, 1, 2, 33), (3, 64, 1, 18, 1, 2, 40), (64, 64, 1, 18, 1, 2, 45)]
for case in cases:
    arrays, x, g = tg._random_case(pkg, *case)
    got = tg._run_hip(pkg, arrays, x, g)
    want = ref_cpu.block_step(arrays, dtype=torch.float64)
    errs = {k.replace("grad.", "").replace("spatialConv.", "sc.").replace("temporalConv.", "tc."):
            rel_to_max(got[k].double().numpy(), want[k].detach().double().numpy())
            for k in want if k in got and "num_batches" not in k}
    print(case, " ".join(f"{k}={v:.1e}" for k, v in errs.items()), flush=True)
