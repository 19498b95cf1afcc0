"""Time each GEMM kernel of the block (stgcn_time_kernel) at the cfg2 layer
shapes and print achieved TFLOP/s. Usage: python scripts/kbench.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from stgcn_loader import load  # noqa: E402

pkg = load()
hl = pkg.hip_lib
lib = hl.lib()
dev = torch.device("cuda", 0)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
V = int(os.environ.get("KB_V", "18"))
K = int(os.environ.get("KB_K", "1"))
shapes = [("L0 3->64", 3, 64, 300, 1), ("L1 64->64", 64, 64, 300, 1),
          ("L4 64->128 s2", 64, 128, 300, 2), ("L5 128->128", 128, 128, 150, 1),
          ("L7 128->256 s2", 128, 256, 150, 2), ("L8 256->256", 256, 256, 75, 1)]
names = ["tconv_fwd", "tconv_dgrad", "tconv_wgrad", "spatial_gemm"]
which_set = [int(w) for w in os.environ.get("KB_WHICH", "0,1,2,3").split(",")]
if os.environ.get("KB_SHAPES"):
    shapes = [shapes[int(i)] for i in os.environ["KB_SHAPES"].split(",")]
for label, ci, co, T, s in shapes:
    d = pkg.fused.make_desc((128, ci, T, V), co, K, s, 4, 1e-5, 0.1, True,
                            bf16=os.environ.get("KB_BF16") == "1",
                            f32x3=os.environ.get("KB_X3") == "1",
                            f16x2=os.environ.get("KB_F16") == "1")
    row = []
    for which in which_set:
        nbytes = lib.stgcn_time_kernel_bytes(ctypes.byref(d), which)
        scratch = torch.randn(nbytes // 4 + 1, device=dev)
        ms, fl = ctypes.c_float(0), ctypes.c_double(0)
        hl.check(lib.stgcn_time_kernel(ctypes.byref(d), which, hl.ptr(scratch), nbytes, iters,
                                       hl.stream_handle(dev), ctypes.byref(ms), ctypes.byref(fl)))
        row.append(f"{names[which]} {ms.value:7.3f}ms {fl.value / ms.value / 1e9:6.1f}TF")
        del scratch
    print(f"{label:16s} " + " | ".join(row), flush=True)
