"""Time the spatial backward (stgcn_time_kernel which=4: k_sp_bwd_fused, or the
H GEMM + joint kernel in an STGCN_AB_UNFUSED_SPB=1 variant build) at the cfg3 / cfg5 layer shapes
(bf16 path, K = 3) or the cfg2 shapes (KB_V=18: fp32 split path, K = 1).
Usage: KB_V=25 python scripts/kbench_spb.py [iters]"""
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
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
V = int(os.environ.get("KB_V", "25"))
K = 1 if V == 18 else 3
x3 = V == 18  # cfg2: the fp32 split path; cfg3 / cfg5: bf16
shapes = [("L1 64->64 T300", 64, 64, 300), ("L4 64->128 T300", 64, 128, 300),
          ("L5 128->128 T150", 128, 128, 150), ("L8 256->256 T75", 256, 256, 75)]
for label, ci, co, T in shapes:
    d = pkg.fused.make_desc((128, ci, T, V), co, K, 1, 4, 1e-5, 0.1, True, bf16=not x3, f32x3=x3)
    out = []
    for which in (4, 5, 6):  # whole backward; its two kernels (H GEMM / joint, or V = 50 dx / dA)
        nbytes = lib.stgcn_time_kernel_bytes(ctypes.byref(d), which)
        if nbytes == 0:
            continue
        scratch = torch.randn(nbytes // 4 + 1, device=dev) * 0.1
        ms, fl = ctypes.c_float(0), ctypes.c_double(0)
        hl.check(lib.stgcn_time_kernel(ctypes.byref(d), which, hl.ptr(scratch), nbytes, iters,
                                       hl.stream_handle(dev), ctypes.byref(ms), ctypes.byref(fl)))
        out.append(f"w{which} {ms.value * 1e3:7.1f} us")
        if which == 4:
            mb = 4 * 128 * T * V * (co + 2 * ci) / 1e6
            out.append(f"({mb / ms.value / 1e3:5.2f} TB/s of dZ + x + dx)")
        del scratch
    print(f"{label:18s} " + "  ".join(out), flush=True)
