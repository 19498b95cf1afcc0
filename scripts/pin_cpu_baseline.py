"""Pin the CPU baseline: the oracle restatement
(oracle/ref_cpu.py) must time within +-10% of the reference itself before it
stands in for the reference as bench.py's ``cpu_baseline`` (kind "port").

Runs in the BUILD container only (it imports the reference from
/root/reference/src, as tests/golden/make_golden.py does, with the same
in-process stubs for the absent pytorch_lightning / seaborn). Workload: the
cfg2 stack shape (V = 18, T = 300, K = 1, 400 classes), N = 8 clips, fp32,
fwd + bwd + cross entropy, 8 threads; the two implementations are timed in
alternating rounds (1 warm-up each, then ROUNDS x ITERS timed steps each) so
drift on the host affects both alike. Writes profiles/cpu_baseline_pin.json.

Usage: python3 -B scripts/pin_cpu_baseline.py [--rounds 3 --iters 2]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.dont_write_bytecode = True
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--N", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    import make_golden
    make_golden._install_stubs()
    sys.path.insert(0, os.path.join(args.reference, "src"))
    with contextlib.redirect_stdout(io.StringIO()):
        import lightning_model  # noqa: E402
        from data import adjacency  # noqa: E402
    from oracle import ref_cpu
    from stgcn_loader import load
    pkg = load()
    V, T, C, classes, N = 18, 300, 3, 400, args.N
    hp = lightning_model.build_argument_parser().parse_args(
        ["--C_in", str(C), "--nr_classes", str(classes)])
    with make_golden._patched_adjacency(adjacency, V), contextlib.redirect_stdout(io.StringIO()):
        torch.manual_seed(0)
        ref_model = lightning_model.L_STGCN(hp).train()
    A = pkg.graph.get_normalized_adjacency_matrices(0, 1, graph=pkg.graph.graph_for(V))
    p, b = ref_cpu.init_stack_params(C, classes, A, seed=0)
    p = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    st = ref_cpu.Stack(p, b)
    x = torch.randn(N, T, V, C, generator=torch.Generator().manual_seed(1))
    y = torch.randint(0, classes, (N,), generator=torch.Generator().manual_seed(2))

    def ref_step():
        ref_model.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(ref_model(x), y).backward()

    def oracle_step():
        for v in p.values():
            v.grad = None
        torch.nn.functional.cross_entropy(st.forward(x), y).backward()

    steps = {"reference": ref_step, "oracle": oracle_step}
    for f in steps.values():
        f()  # warm-up
    times = {k: [] for k in steps}
    for _ in range(args.rounds):
        for k, f in steps.items():
            t0 = time.perf_counter()
            for _ in range(args.iters):
                f()
            times[k].append(time.perf_counter() - t0)
    rate = {k: N * args.iters * len(v) / sum(v) for k, v in times.items()}
    ratio = rate["oracle"] / rate["reference"]
    out = {"workload": f"cfg2 stack fwd+bwd+CE, N={N}, T={T}, V={V}, K=1, {classes} classes, fp32",
           "threads": args.threads, "rounds": args.rounds, "iters_per_round": args.iters,
           "reference_clips_s": round(rate["reference"], 3),
           "oracle_clips_s": round(rate["oracle"], 3), "oracle_over_reference": round(ratio, 4),
           "within_10pct": abs(ratio - 1) <= 0.10,
           "per_round_s": {k: [round(t, 3) for t in v] for k, v in times.items()},
           "torch": torch.__version__}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_baseline_pin.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
