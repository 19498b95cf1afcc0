"""Per-tensor rel-to-max error vs the fp64 oracle of the block in each GEMM mode
(fp32 MFMA, f32x3 = 3-way bf16 splits, f16x2 = scaled 2-way fp16 splits), next to
the fp32 reference's own error (oracle run in fp32). Prints the worst tensor per
mode at the end of each case.
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
    modes = ("fp32", "f32x3", "f16x2")
    res = {m: _run_hip(pkg, arrays, x, g, gemm=m) for m in modes}
    want, floor = _oracle(arrays, res["fp32"])
    print("case", case)
    worst = {m: (0.0, "") for m in modes}
    for k in want:
        if k not in res["fp32"] or "num_batches" in k or k == "grad.temporalConv.bias":
            continue
        w = want[k].detach().double().numpy()
        e = {m: rel_to_max(r[k].double().numpy(), w) for m, r in res.items()}
        for m in modes:
            if e[m] > worst[m][0]:
                worst[m] = (e[m], k)
        print(f"  {k:32s} ref32 {floor.get(k, 0):.2e}  " +
              "  ".join(f"{m} {e[m]:.2e}" for m in modes), flush=True)
    print("  worst: " + "  ".join(f"{m} {v:.2e} ({k})" for m, (v, k) in worst.items()), flush=True)
