"""Per-tensor rel-to-max error vs the fp64 oracle of the block in each GEMM mode
(fp32 MFMA, f32x3 split), next to the fp32 reference's own error.
Usage: python scripts/diag_x3.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from stgcn_loader import load  # noqa: E402
from conftest import rel_to_max  # noqa: E402
from test_gpu_block import _oracle, _random_case, _run_hip  # noqa: E402

pkg = load()
for case in [(64, 64, 1, 18, 1, 4, 64), (64, 64, 1, 18, 1, 16, 300), (256, 256, 1, 18, 1, 4, 75),
             (64, 128, 2, 18, 1, 3, 37)]:
    arrays, x, g = _random_case(pkg, *case)
    res = {m: _run_hip(pkg, arrays, x, g, gemm=m) for m in ("fp32", "f32x3")}
    want, floor = _oracle(arrays, res["fp32"])
    print("case", case)
    for k in want:
        if k not in res["fp32"] or "num_batches" in k:
            continue
        w = want[k].detach().double().numpy()
        e = {m: rel_to_max(r[k].double().numpy(), w) for m, r in res.items()}
        print(f"  {k:32s} ref32 {floor.get(k, 0):.2e}  fp32 {e['fp32']:.2e}  f32x3 {e['f32x3']:.2e}",
              flush=True)
