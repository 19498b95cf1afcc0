"""Diagnostic: per-gradient error of the bf16 HIP block vs the fp64 oracle and
the bf16-operand reference's own error (tests/test_gpu_bf16.py _check_bf16
arithmetic), one line per case; then the V = 50 deferred-dx chained stack's
per-tensor error ratio (tests/test_gpu_stack.py gate) over a few seeds.
Run with STGCN_LIB_VARIANT to compare kernel variants."""
import contextlib, io, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from stgcn_loader import load
from oracle import ref_cpu
import test_gpu_bf16 as tb
import test_gpu_stack as ts
from conftest import rel_to_max

pkg = load()
for case in [(64, 64, 1, 50, 3, 2, 17), (128, 256, 2, 50, 3, 2, 13), (256, 256, 1, 50, 3, 2, 7),
             (64, 64, 1, 50, 3, 8, 64)]:
    C_in, C_out, stride, V, K, N, T = case
    arrays, x, g = tb._random_case(pkg, C_in, C_out, stride, V, K, N, T, seed=3)
    got = tb._run(pkg, arrays, x, g, bf16=True, need_dx=True)
    mask = got["y"] > 0
    want = ref_cpu.block_step(arrays, dtype=torch.float64, relu_mask=mask)
    ref16 = ref_cpu.block_step(arrays, dtype=torch.float32, relu_mask=mask.float(), gemm_bf16=True)
    e, f = tb._errors(got, want, False), tb._errors(ref16, want, False)
    keys = ["grad.x", "grad.batch_n.weight", "grad.batch_n.bias", "grad.spatialConv.A"]
    print(case, " ".join(f"{k.split('.')[-1]}={e[k]:.2e}/{f[k]:.2e}" for k in keys), flush=True)

gr = pkg.graph
A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(50),
                                         graph=gr.graph_for(50))
for seed in (5, 6, 7):
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A, gemm_dtype=torch.bfloat16).cuda().train()
    p0, b0 = ts.snapshot_stack(m1)
    x = torch.randn(4, 3, 24, 50, generator=torch.Generator().manual_seed(seed + 1)).cuda()
    lab = torch.randint(0, 10, (4,), generator=torch.Generator().manual_seed(seed + 2)).cuda()
    masks, unhook = ts.capture_relu_masks(m1)
    out1 = m1.forward_nctv(x)
    unhook()
    torch.nn.functional.cross_entropy(out1, lab).backward()
    torch.cuda.synchronize()
    x_ntvc = x.detach().cpu().permute(0, 2, 3, 1).contiguous()

    def run(dtype, bf16):
        p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p0.items()}
        b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in b0.items()}
        st = ref_cpu.Stack(p, b)
        lg = st.forward(x_ntvc, dtype=dtype, gemm_bf16=bf16, relu_masks=[m.to(dtype) for m in masks])
        torch.nn.functional.cross_entropy(lg, lab.cpu()).backward()
        return {k: v.grad for k, v in p.items()}

    g64, gref = run(torch.float64, False), run(torch.float32, True)
    worst = []
    for k, v in m1.named_parameters():
        if k.startswith("Masks.") or k.endswith("temporalConv.bias"):
            continue
        want = g64[k].detach().double().numpy()
        fl = rel_to_max(gref[k].detach().double().numpy(), want)
        er = rel_to_max(v.grad.detach().cpu().double().numpy(), want)
        worst.append((er / max(fl, 5e-3), k, er, fl))
    worst.sort(reverse=True)
    print("stack seed", seed, " ".join(f"{k}={er:.2e}/{fl:.2e}" for _, k, er, fl in worst[:4]), flush=True)
