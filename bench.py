#!/usr/bin/env python3
"""Skeleton clips/s of the ST-GCN training step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): Kinetics-skeleton
shape, synthetic input (N, 3, 300, 18) NCTV per GPU with N=128, V=18, uni
labelling (K=1), 400 classes, fp32. One step = forward of the 10-block stack
(fused HIP blocks) + avg-pool/FC head + cross-entropy (fused HIP head) +
backward + (N>1) RCCL gradient all-reduce + Adam update (FusedAdam: one HIP
launch; --torch-ops for torch's head / loss / Adam). Inputs are resident in HBM before timing.

Run: python bench.py [--gpus N --steps K --warmup W]
     (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from stgcn_loader import load  # noqa: E402

# BASELINE.json configs (SURVEY.md §8 "Per-config inputs"); the default bench
# line is cfg2. cfg3 / cfg5 use the spatial-configuration partitioning (K=3,
# strategy 2 with synthetic distances) and bf16 channel GEMMs (fp32 accumulate,
# fp32 tensors); cfg4 is cfg2 data-parallel (run with --gpus N).
CONFIGS = {
    "cfg2": dict(N=128, C=3, T=300, V=18, K=1, classes=400, bf16=False,
                 desc="cfg2 Kinetics-skeleton shape: 10-block ST-GCN stack fwd+bwd+CE+Adam, "
                      "V=18, T=300, K=1 (uni), 400 classes"),
    "cfg3": dict(N=128, C=3, T=300, V=25, K=3, classes=60, bf16=True,
                 desc="cfg3 NTU-RGB+D shape: 10-block ST-GCN stack fwd+bwd+CE+Adam, V=25, "
                      "T=300, K=3 (spatial), 60 classes, bf16 channel GEMMs"),
    "cfg5": dict(N=128, C=3, T=300, V=50, K=3, classes=60, bf16=True,
                 desc="cfg5 2-person stacked graph: 10-block ST-GCN stack fwd+bwd+CE+Adam, "
                      "V=50, T=300, K=3 (spatial), 60 classes, bf16 channel GEMMs"),
}
CFG = CONFIGS["cfg2"]
MFMA_F32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense (no sparsity)
# fp32 work on the bf16 matrix cores by exact 3-way operand splits: six bf16
# MFMAs per fp32 product (kernels_x3.hip), so the fp32-work ceiling is 1/6 of BF16
X3_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 6
# ... and by 2-way fp16 splits (STGCN_F_F16X2): three fp16 MFMAs (fp16 runs at the
# bf16 rate) per fp32 product
F16X2_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak


def adjacency(pkg, cfg):
    gr = pkg.graph
    if cfg["K"] == 1:
        return gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(cfg["V"]))
    return gr.get_normalized_adjacency_matrices(
        2, 1, distances=gr.synthetic_distances(cfg["V"]), graph=gr.graph_for(cfg["V"]))


def build_model(pkg, cfg, device):
    A = adjacency(pkg, cfg)
    torch.manual_seed(0)
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(cfg["C"], cfg["classes"], A,
                               gemm_dtype=torch.bfloat16 if cfg["bf16"] else torch.float32,
                               f32_gemm=cfg.get("f32_gemm", "mfma"))
    return model.to(device)


def progress(msg):
    """A progress line on stderr (long phases must keep writing: a GPU run
    silent for 3 minutes is taken to be hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), or platform.processor()."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def gpu_state_start():
    """Starts a rocm-smi sample of the GPUs' clocks and power (read-only), so a
    bench line carries the clock state it ran at: box-to-box spread of the same
    tree is +-5 %, and a lower sclk under load is one cause."""
    try:
        return subprocess.Popen(["rocm-smi", "--showclocks", "--showpower", "--showmaxpower",
                                 "--json"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                text=True)
    except OSError:
        return None


def gpu_state_read(proc):
    """{card: {sclk, mclk, fclk, power, power cap ...}} from gpu_state_start, or None."""
    if proc is None:
        return None
    try:
        out, _ = proc.communicate(timeout=30)
        data = json.loads(out)
    except (subprocess.TimeoutExpired, ValueError):
        proc.kill()
        return None
    keys = ("sclk", "mclk", "fclk", "socclk", "power")
    return {card: {k: v for k, v in vals.items() if any(s in k.lower() for s in keys)}
            for card, vals in data.items() if card.startswith("card")} or None


def cgroup_cpu_quota():
    """The process's cgroup CPU bandwidth limit as (CPUs, raw text), or
    (None, reason): cgroup v2 /sys/fs/cgroup/cpu.max ("quota period" or
    "max period"), else v1 cpu.cfs_quota_us / cpu.cfs_period_us."""
    try:
        raw = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, per = raw.split()[:2]
        return (None if q == "max" else round(int(q) / int(per), 2)), f"cpu.max: {raw}"
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q <= 0 else round(q / per, 2)), f"cfs_quota_us {q} / period {per}"
    except (OSError, ValueError):
        return None, "no cgroup CPU limit readable"


def cpu_baseline(cfg, seconds=8.0):
    """The oracle (CPU restatement of the reference, fp32 torch ops, pinned at
    0.945 of the reference's own speed: profiles/cpu_baseline_pin.json) timed
    on this host's cores on a bounded sample of the same workload
    (torch.set_num_threads(os.cpu_count())). A GPU box's
    process may be confined to a share of the machine's cores (16 per GPU on
    this pool), where os.cpu_count() threads oversubscribe it: both thread
    counts are timed and the faster one is reported (the best the reference
    path does on this host)."""
    from oracle import ref_cpu
    pkg = load()
    ncpu = os.cpu_count() or 1
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = ncpu
    cands = sorted({ncpu, max(1, min(16, share))})
    A = adjacency(pkg, cfg)
    p, b = ref_cpu.init_stack_params(cfg["C"], cfg["classes"], A, seed=0)
    p = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    st = ref_cpu.Stack(p, b)
    n = 8
    x = torch.randn(n, cfg["T"], cfg["V"], cfg["C"], generator=torch.Generator().manual_seed(1))
    y = torch.randint(0, cfg["classes"], (n,), generator=torch.Generator().manual_seed(2))

    def step():
        loss = torch.nn.functional.cross_entropy(st.forward(x), y)
        loss.backward()

    prev = torch.get_num_threads()
    res = []
    import threading
    done = threading.Event()

    def beat():  # one oversubscribed step can outlast the 3-minute silence limit
        while not done.wait(45):
            progress("cpu baseline: running")
    threading.Thread(target=beat, daemon=True).start()
    for threads in cands:
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        step()  # warm-up
        tw = time.perf_counter() - t0
        progress(f"cpu baseline: {threads} threads, warm-up step {tw:.1f}s")
        if res and tw > 4 * n / res[-1][0]:  # far slower than the smaller thread count
            res.append((n / tw, threads, 1, tw))  # (oversubscribed: one step is the sample)
            continue
        iters, t0 = 0, time.perf_counter()
        while iters < 2 or time.perf_counter() - t0 < seconds:
            step()
            iters += 1
        dt = time.perf_counter() - t0
        res.append((n * iters / dt, threads, iters, dt))
    done.set()
    torch.set_num_threads(prev)
    best = max(res)
    quota, quota_raw = cgroup_cpu_quota()
    why = None
    if len(res) > 1 and res[0][0] > 4 * res[-1][0]:
        why = (f"{res[-1][1]} threads ran {res[0][0] / res[-1][0]:.0f}x slower than {res[0][1]}: "
               + (f"the process's cgroup limits it to {quota} CPUs ({quota_raw}), so "
                  f"{res[-1][1]} busy-waiting torch threads are throttled"
                  if quota is not None and quota < res[-1][1] else
                  f"oversubscription beyond the process's CPU share ({quota_raw})"))
    return {"value": round(best[0], 3), "unit": "clips/s", "cores": best[1],
            "kind": "port", "cpu_model": cpu_model(), "os_cpu_count": ncpu,
            "affinity_cpus": share, "cgroup_cpu_quota": quota, "cgroup_cpu_limit": quota_raw,
            "slow_leg_explained": why,
            "per_thread_count": {str(t): round(v, 3) for v, t, _, _ in res},
            "sample": f"oracle/ref_cpu.py fp32 stack fwd+bwd+loss, N={n} clips x {best[2]} iters "
                      f"(T={cfg['T']}, V={cfg['V']}, K={cfg['K']}, {cfg['classes']} classes), "
                      f"{best[1]} threads, {best[3]:.1f}s; timed at "
                      f"{' and '.join(str(t) for t in cands)} threads, the faster reported"}


# cfg2 stack layers (lightning_model.py:65-86): (C_in, C_out, T_in, stride)
def stack_layers(cfg):
    out, c, t = [], cfg["C"], cfg["T"]
    for co, s in [(64, 1), (64, 1), (64, 1), (64, 1), (128, 2), (128, 1), (128, 1),
                  (256, 2), (256, 1), (256, 1)]:
        out.append((c, co, t, s))
        c, t = co, (t - 1) // s + 1
    return out


KERNEL_KINDS = {0: "tconv_fwd", 1: "tconv_dgrad", 2: "tconv_wgrad", 3: "spatial_gemm",
                4: "spatial_bwd"}


def joint_bwd_symbol(cfg, ci, t):
    """rocprof short name of the unfused spatial backward's joint kernel
    (kernels.hip launch_spatial_dx: k_spatial_bwd5 / _bwd6, else k_spatial_bwd3)."""
    V, K = cfg["V"], cfg["K"]
    if V in (18, 25) and K * ((V + 1) // 2) * ((V + 31) // 32) <= 48:
        for rb in (128, 64):
            if (ci * t) % rb == 0:
                return f"k_spatial_bwd5<{V},{rb},{K}>"
    if V == 50 and (ci * t) % 64 == 0:
        return f"k_spatial_bwd6<50,{K},{'true' if cfg['bf16'] else 'false'}>"
    return f"k_spatial_bwd3<{V}>"


def x3_planes(sym):
    """Operand planes (NPL) of a split-kernel symbol: k_conv_x3<NQ,TG,V,SIN,MR,NPL,..>
    (k_conv_x3<5|4,V,SIN,MR,NPL,..> for the stride-2 data-gradient pair),
    k_wgrad_x3<V,SIN,NPL,MR[,QBN]>."""
    args = [a.strip() for a in sym[sym.index("<") + 1:sym.rindex(">")].split(",")]
    if sym.startswith("k_wgrad_x3"):
        return int(args[2])
    return int(args[4] if args[0] == "5|4" else args[5])


def kernel_roofline(pkg, device, cfg, iters=10):
    """Per-kernel timing with HIP events on the launch stream (the library's
    stgcn_time_kernel entry point, same launch parameters as the block), over
    every layer of the stack. Returns {kind: (total_ms, total_flops, launches,
    bytes)} and the same aggregated per kernel symbol (rocprof short names), so
    the dominant kernel is chosen among every GEMM-type kernel of the step,
    the two halves of an unfused spatial backward included (which 5 / 6)."""
    import ctypes
    hl = pkg.hip_lib
    lib = hl.lib()
    kinds, symbols = {}, {}

    def add(d, key, ms, fl, n, nb=0.0):
        t = d.get(key, (0.0, 0.0, 0, 0.0))
        d[key] = (t[0] + ms, t[1] + fl, t[2] + n, t[3] + nb)

    V4 = cfg["V"] * 4
    for li, (ci, co, t, s) in enumerate(stack_layers(cfg)):
        progress(f"kernel timing: layer {li}")
        x3 = cfg.get("f32_gemm") in ("bf16x3", "f16x2", "f16x2-nog") and not cfg["bf16"]
        f16 = cfg.get("f32_gemm") in ("f16x2", "f16x2-nog") and not cfg["bf16"]
        d = pkg.fused.make_desc((cfg["N"], ci, t, cfg["V"]), co, cfg["K"], s, 4, 1e-5, 0.1, True,
                                bf16=cfg["bf16"], f32x3=x3 and not f16, f16x2=f16,
                                no_g=cfg.get("f32_gemm") == "f16x2-nog" and not cfg["bf16"])
        for which in range(7):
            nbytes = lib.stgcn_time_kernel_bytes(ctypes.byref(d), which)
            if nbytes == 0:  # 5 / 6 where the spatial backward is one fused kernel
                continue
            scratch = torch.randn(nbytes // 4 + 1, device=device)
            ms, fl = ctypes.c_float(0), ctypes.c_double(0)
            hl.check(lib.stgcn_time_kernel(ctypes.byref(d), which, hl.ptr(scratch), nbytes, iters,
                                           hl.stream_handle(device), ctypes.byref(ms),
                                           ctypes.byref(fl)))
            del scratch
            # algorithmic HBM bytes of the timed launch(es): fp32 activations in
            # and out (the kept G of the fused spatial forward in bf16)
            N, to = cfg["N"], (t - 1) // s + 1
            V, K = cfg["V"], cfg["K"]
            # bf16 storage of Z and dU (capi.hip act_bf16: bf16 path, stride-1
            # non-residual blocks whose spatial forward is fused, C_in >= 16):
            # those operands move 2 bytes per element
            # (stride-2 blocks too at even V: their weight gradient stages bf16 by LDS-DMA)
            ab = cfg["bf16"] and (s == 1 or V % 2 == 0) and ci >= 16
            V2 = V * 2 if ab else V4
            # bf16 storage of dZ (capi.hip dz_bf16) is an A/B build only
            # (STGCN_AB_DZ_BF16): the shipped library stores dZ in fp32
            dzb = False
            VZ = V * 2 if dzb else V4
            # the two-person graph's fused spatial backward: two kernels, each
            # reading dZ and x (k_sp50_dx also writes dx), timed as which 5 / 6
            f50 = cfg["bf16"] and V == 50 and K == 3 and ci % 32 == 0 and ci <= 128
            # the folded block (capi.hip fold_w: fp32 split path, K = 1, V = 18,
            # C_in >= 16): no spatial / H GEMM, the temporal GEMMs read G (C_in
            # channels) in place of Z, and the data gradient writes H (C_in)
            fold = x3 and K == 1 and V == 18 and ci >= 16 and co >= 16
            # (f16x2 fold without G, PLAN_FOLD_NO_G: the forward GEMM reads x and the
            # weight gradient x against dU A -- the same bytes as G / dU)
            bna = bool(hl.block_plan(d) & hl.PLAN_FOLD_NO_G)
            CZ = ci if fold else co
            # (the folded block's data gradient carries the SpatialConv backward:
            # it reads x and writes dxhat instead of writing H)
            act = {0: N * (CZ * t * V2 + co * to * V4),
                   1: (N * (co * to * V2 + 2 * ci * t * V4) if fold else
                       N * (co * to * V2 + CZ * t * VZ)),
                   2: N * (co * to * V2 + CZ * t * V2),
                   3: N * (ci * t * V4 + co * t * V2) + (N * K * ci * t * V * 2
                                                       if cfg["bf16"] and ci >= 16 else
                                                       N * K * ci * t * V4),
                   4: N * (co * t * VZ + 2 * ci * t * V4),  # dZ, x in; dx out
                   5: (N * (co * t * VZ + 2 * ci * t * V4) if f50 else  # dZ, x in; dx out
                       N * (co * t * VZ + K * ci * t * V4)),  # dZ in; H out
                   6: (N * (co * t * VZ + ci * t * V4) if f50 else  # dZ, x in
                       N * (K * ci * t + 2 * ci * t) * V4)}[which]  # H, x in; dx out
            if which <= 4:
                add(kinds, KERNEL_KINDS[which], ms.value, fl.value, 1, act)
            # rocprof short names of the kernel each timing runs
            if which == 4:
                # the fused spatial backward (bf16, V = 25, K = 3); the unfused
                # pair is timed per kernel by which 5 / 6 (folded: its joint
                # kernel alone, which 6)
                if not fold and lib.stgcn_time_kernel_bytes(ctypes.byref(d), 5) == 0:
                    add(symbols, f"k_sp_bwd_fused<{V},{K},{'true' if x3 else 'false'},"
                                 f"{'true' if dzb else 'false'}>",
                        ms.value, fl.value, 1, act)
                continue
            if which == 6:
                add(symbols, f"k_sp50_dA<{K}>" if f50 else joint_bwd_symbol(cfg, ci, t),
                    ms.value, fl.value, 1, act)
                continue
            if which == 5 and f50:
                add(symbols, f"k_sp50_dx<{K}>", ms.value, fl.value, 1, act)
                continue
            if which == 5:  # the stacked H GEMM (NQ = 1 over C_out channels)
                sym = (f"k_conv_bf16<1,16,{V},1,{'true' if dzb else 'false'}>"
                       if cfg["bf16"] and co >= 16
                       else f"k_tconv<1,8,{V},1>")
                add(symbols, sym, ms.value, fl.value, 1, act)
                continue
            if cfg["bf16"]:
                # temporal GEMMs: k_conv_x3 with one operand plane (NPL = 1)
                ib = "true" if ab else "false"  # bf16 input instance
                ft, cb = {18: (8, 64), 25: (4, 64), 50: (4, 32)}.get(V, (0, 0))
                sym = {0: f"k_conv_x3<9,3,{V},{s},1,1,{ib},false>",
                       1: (f"k_conv_x3<9,3,{V},1,1,1,{ib},false>" if s == 1 else
                           f"k_conv_x3<5|4,{V},1,1,1,{ib},false>"),
                       2: f"k_wgrad_bf16<9,{V},{s},{ft},{cb},{ib}>",
                       3: (f"k_conv_bf16<1,16,{V},1,false>" if ci < 16 else
                           f"k_sp_fwd_bf16<{V},{K}>" if not (V == 50 or (V == 25 and K == 3)) else
                           f"k_sp_fwd_wide<{V},3,{64 if co <= 64 else 128 if co <= 128 else 256}>")
                       }[which]
            elif x3 and V in (18, 25):
                mr = 2 if co % 128 == 0 else 1  # 128-row tiles for the 9-tap launches
                npl = 2 if f16 and fold else 3  # operand planes: fp16 (h, l) or bf16 (h, m, l)
                spb = "true" if fold else "false"  # the fused SpatialConv backward epilogue
                nb = ",true" if bna else ""  # (the BNA / QBN template instances)
                sym = {0: f"k_conv_x3<9,3,{V},{s},{mr},{npl},false,false{nb}>",
                       1: (f"k_conv_x3<9,3,{V},1,{mr},{npl},false,{spb}>" if s == 1 else
                           f"k_conv_x3<5|4,{V},1,1,{npl},false,{spb}>"),
                       2: (f"k_wgrad_x3<{V},{s},{npl},{2 if npl == 2 and co % 128 == 0 else 1}"
                           f"{nb}>" if V == 18 else f"k_wgrad_taps<{V},{s}>"),
                       3: f"k_tconv<1,8,{V},1>"}[which]
            else:
                sym = {0: f"k_tconv<9,2,{V},{s}>",
                       1: f"k_tconv<9,2,{V},1>" if s == 1 else f"k_tconv<5|4,2,{V},1>",
                       2: f"k_wgrad_taps<{V},{s}>", 3: f"k_tconv<1,8,{V},1>"}[which]
            add(symbols, sym, ms.value, fl.value, 1 if (which != 1 or s == 1) else 2, act)
    return kinds, symbols


def per_block_rates(model, cfg, device, iters=5):
    """per-block clips/s (fwd+bwd of one block, L0..L9) at the
    bench batch, timed with events after the main measurement."""
    out, c, t = {}, cfg["C"], cfg["T"]
    gen = torch.Generator(device="cpu").manual_seed(7)
    for i, (ci, co, tin, s) in enumerate(stack_layers(cfg)):
        blk = model.conv[i]
        x = torch.randn(cfg["N"], ci, tin, cfg["V"], generator=gen).to(device)
        x.requires_grad_(i > 0)
        tout = (tin - 1) // s + 1
        g = torch.randn(cfg["N"], co, tout, cfg["V"], generator=gen).to(device)
        for _ in range(2):
            blk(x).backward(g)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            blk(x).backward(g)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        out[f"L{i}"] = round(cfg["N"] / (ms * 1e-3), 1)
    model.zero_grad(set_to_none=True)
    return out


def source_sha16():
    """sha256 (first 16 hex) over the kernel sources and the C-ABI header: the
    tree tag a PMC file must carry for its counters to describe this build."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "st-gcn_amd", "csrc", "*"))) + \
        [os.path.join(ROOT, "include", "stgcn_hip.h")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_profile(config):
    """The committed rocprofv3 PMC summary (profiles/pmc_<tag>_<config>.json,
    scripts/pmc_traffic.py) of THIS config measured on THIS kernel-source tree
    (its src_sha16), or (None, reason)."""
    import glob
    sha = source_sha16()
    found = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_*_{config}.json"))):
        try:
            data = json.load(open(f))
        except (OSError, ValueError):
            continue
        if data.get("config") == config:
            found.append((f, data))
    for f, data in reversed(found):
        if data.get("src_sha16") == sha:
            return data, os.path.relpath(f, ROOT)
    return None, (f"no PMC pass of {config} on this kernel-source tree (src_sha16 {sha}); "
                  f"newest: {os.path.relpath(found[-1][0], ROOT) if found else 'none'}")


def pmc_lookup(table, sym):
    """table[sym] where the PMC file names the kernel as the timing does; else
    the one rocprof name that only appends template arguments left at their
    default (false, or k_conv_x3's wave count NW = 8), e.g.
    k_conv_x3<..,false,true> -> k_conv_x3<..,false,true,false,8>."""
    if sym in table:
        return table[sym]
    head = sym[:-1] + ","
    hits = [k for k in table
            if k.startswith(head) and k.endswith(">") and
            all(a in ("false", "8") for a in k[len(head):-1].split(","))]
    return table[hits[0]] if len(hits) == 1 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=CFG["N"], help="clips per GPU")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="BASELINE.json workload (default cfg2, the headline metric)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--f32-gemm", choices=["mfma", "bf16x3", "f16x2", "f16x2-nog"], default="f16x2",
                    help="fp32 configs: temporal-conv GEMMs on the fp32 matrix cores (mfma), "
                         "as exact 3-way bf16 operand splits (bf16x3) or, on the folded "
                         "blocks, as 2-way fp16 splits of power-of-two-scaled operands "
                         "(f16x2); all held to the fp32 parity gate")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip timing the other fp32 GEMM modes beside the default")
    ap.add_argument("--no-repeats", dest="repeats", action="store_false",
                    help="skip the two extra timed windows (median of three)")
    ap.add_argument("--no-sweep", dest="sweep", action="store_false",
                    help="skip the per-GPU batch sweep (SURVEY.md §8(d): N in 32, 64, 256 "
                         "besides the bench batch; N=1 process only)")
    ap.add_argument("--no-lazy-links", action="store_true",
                    help="A/B only: write every block output (no ABI 8/9 unwritten outputs)")
    ap.add_argument("--torch-ops", action="store_true",
                    help="head + cross entropy + Adam from torch instead of the HIP library")
    ap.add_argument("--no-graph", action="store_true",
                    help="run the timed steps eagerly (default at N=1: the step captured once "
                         "in a HIP graph and replayed, train_ops.GraphedStep)")
    ap.add_argument("--dp-graph", action="store_true",
                    help="N>1: forward + backward and Adam in two HIP graphs around the eager "
                         "bucket all-reduces (train_ops.GraphedDPStep; default: eager)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; STGCN_DIST_BACKEND=gloo (with more ranks than GPUs:
    # ranks share devices round-robin) only rehearses the multi-rank path on a
    # one-GPU box, the real run is RCCL ("nccl") over xGMI
    backend = os.environ.get("STGCN_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    pkg = load()
    cfg = dict(CONFIGS[args.config], N=args.batch, f32_gemm=args.f32_gemm)

    model = build_model(pkg, cfg, device)
    if args.no_lazy_links:
        model.lazy_links = False
    params = [p for p in model.parameters()]
    # one process: the whole step (forward, backward, head, Adam) captured in a
    # HIP graph and replayed (no per-launch host work; FusedAdam's step count on
    # the device). With ranks: eager, the bucket all-reduces overlapped with
    # backward; --dp-graph runs forward + backward and Adam in two graphs around
    # the eager all-reduces (train_ops.GraphedDPStep: equal results, but 4x
    # slower in the 2-rank gloo rehearsal on one GPU, profiles/r6dpg_*, and not
    # measured over RCCL)
    graph_on = not args.torch_ops and not args.no_graph and (world == 1 or args.dp_graph)
    # FusedAdam: torch.optim.Adam semantics, one libstgcn_hip launch per step
    opt = (torch.optim.Adam(params, lr=1e-3) if args.torch_ops
           else pkg.FusedAdam(params, lr=1e-3, capturable=graph_on))
    dp = pkg.dp.GradAllReduce(model, world) if world > 1 else None
    gen = torch.Generator(device="cpu").manual_seed(1 + rank)
    x = torch.randn(cfg["N"], cfg["C"], cfg["T"], cfg["V"], generator=gen).to(device)
    labels = torch.randint(0, cfg["classes"], (cfg["N"],), generator=gen).to(device)

    def step():
        if dp is not None:
            dp.zero_grad()  # bucket-view gradients stay in place (dp.GradAllReduce)
        else:
            opt.zero_grad(set_to_none=True)
        if args.torch_ops:
            loss = torch.nn.functional.cross_entropy(model.forward_nctv(x), labels)
        else:  # fused HIP head: avg-pool + Linear + cross entropy
            loss, _ = model.forward_loss(x, labels)
        loss.backward()
        if dp is not None:
            dp.synchronize()
        opt.step()
        return loss

    progress(f"{args.config}: model built, {args.warmup} warm-up steps")
    def fwd_bwd():  # (ranks > 1, graphed: dp.zero_grad / synchronize by GraphedDPStep)
        loss, _ = model.forward_loss(x, labels)
        loss.backward()
        return loss

    run = step
    if graph_on:  # the W warm-up steps: a few eager (the capture needs one), the
        # capture, then untimed replays
        n_eager = max(1, min(args.warmup - 1, 2))
        run = (pkg.GraphedDPStep(fwd_bwd, dp, opt.step, warmup=n_eager) if dp is not None
               else pkg.GraphedStep(step, warmup=n_eager))
        for _ in range(max(1, args.warmup - n_eager)):
            run()
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the loss of the first timed window's last step (a graph's output tensor is
    # rewritten by every later replay)
    loss_first = float(loss.item())
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    ms = dt / args.steps * 1e3
    clips = cfg["N"] * world * args.steps / dt
    # two more windows of the same K steps (same brackets), for the median of
    # three; `value` stays the first window, timed exactly as the contract says
    runs = [clips]
    smi = None  # rocm-smi sample taken during the last repeat window (under load)
    for rep in range(2 if args.repeats else 0):
        if rep == 1 and rank == 0:
            smi = gpu_state_start()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        d1 = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([d1], device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d1 = t.item()
        runs.append(cfg["N"] * world * args.steps / d1)
    gf_clip = pkg.flops_per_clip(cfg["C"], cfg["T"], cfg["V"], cfg["K"], cfg["classes"]) / 1e9
    progress(f"{args.config}: {clips:.1f} clips/s ({[round(r, 1) for r in runs]})")

    # the other fp32 GEMM modes (exact fp32 MFMA: every GEMM on
    # v_mfma_f32_32x32x2_f32; bf16x3) timed beside the default, same model and
    # inputs (N=1 only)
    alt = None
    if world == 1 and not cfg["bf16"] and not args.no_alt:
        alt = []
        for mode in ("mfma", "bf16x3", "f16x2"):
            if mode == cfg["f32_gemm"]:
                continue
            for blk in model.conv:
                blk.f32_gemm = mode
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            ta = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dta = time.perf_counter() - ta
            alt.append({"f32_gemm": mode, "value": round(cfg["N"] * args.steps / dta, 2),
                        "ms_per_step": round(dta / args.steps * 1e3, 3)})
        for blk in model.conv:
            blk.f32_gemm = cfg["f32_gemm"]

    # SURVEY.md §8(d) batch sweep (cfg2: N in {32, 64, 256} clips per GPU beside
    # the bench batch), same model and step, 5 timed steps each after 2 warm-up
    # steps; reported as extra keys, `value` stays the bench batch
    sweep = None
    if world == 1 and args.sweep and args.config == "cfg2":
        sweep = {str(cfg["N"]): round(clips, 2)}
        for nb in (32, 64, 256):
            if nb == cfg["N"]:
                continue
            progress(f"batch sweep: N={nb}")
            x = torch.randn(nb, cfg["C"], cfg["T"], cfg["V"], generator=gen).to(device)
            labels = torch.randint(0, cfg["classes"], (nb,), generator=gen).to(device)
            sweep_run = step  # (the bench's step mode: a graph captured at this N)
            if graph_on:
                sweep_run = pkg.GraphedStep(step, warmup=2)
                sweep_run()
            else:
                for _ in range(2):
                    step()
            torch.cuda.synchronize()
            ts = time.perf_counter()
            for _ in range(5):
                sweep_run()
            torch.cuda.synchronize()
            sweep[str(nb)] = round(nb * 5 / (time.perf_counter() - ts), 2)
        sweep = dict(sorted(sweep.items(), key=lambda kv: int(kv[0])))
        x = torch.randn(cfg["N"], cfg["C"], cfg["T"], cfg["V"], generator=gen).to(device)
        labels = torch.randint(0, cfg["classes"], (cfg["N"],), generator=gen).to(device)

    if rank == 0:
        out = {
            "metric": "skeleton clips/sec (fwd+bwd), synthetic (N,3,300,18); 1/2/4/8-GPU scaling",
            "value": round(clips, 2), "unit": "clips/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if cfg["bf16"] else "fp32",
            "data": "synthetic (random N(0,1) skeletons, random labels)",
            "config": {"workload": cfg["desc"],
                       "per_gpu_batch": cfg["N"], "global_batch": cfg["N"] * world,
                       "seq_len": cfg["T"], "parallelism": f"dp{world}",
                       "channel_gemm": ("bf16 operands, fp32 accumulate" if cfg["bf16"] else
                                        "fp32: temporal conv fwd/data-grad/weight-grad as exact "
                                        "3-way bf16 splits (6 MFMAs, fp32-gated parity); "
                                        "spatial GEMMs fp32 MFMA"
                                        if cfg["f32_gemm"] == "bf16x3" else
                                        "fp32: folded temporal GEMMs (fwd, data-grad, "
                                        "weight-grad) as 2-way fp16 splits of "
                                        "power-of-two-scaled operands (3 MFMAs, fp32-gated "
                                        "parity), other temporal GEMMs 3-way bf16 splits"
                                        if cfg["f32_gemm"] == "f16x2" else "fp32 MFMA")},
            "model_tflops": round(clips * gf_clip / 1e3, 2),
            "runs_clips_s": [round(r, 2) for r in runs],
            "median_clips_s": round(sorted(runs)[len(runs) // 2], 2),
            "loss": round(loss_first, 5),
            "step_mode": "hip_graph" if graph_on else "eager",
        }
        out["gpu_state_under_load"] = gpu_state_read(smi)
        out["gpu_state_after"] = gpu_state_read(gpu_state_start())
        if alt is not None:
            out["alt_fp32_modes"] = alt
        if sweep is not None:
            out["batch_sweep_clips_s"] = sweep
        if not args.no_roofline:
            progress("per-block rates")
            out["per_block_clips_s"] = per_block_rates(model, cfg, device)
            progress("per-kernel timing (roofline)")
            kinds, symbols = kernel_roofline(pkg, device, cfg)
            sym = max(symbols, key=lambda k: symbols[k][0])
            ms_tot, fl_tot, nl, nb_tot = symbols[sym]
            pmc, pmc_src = pmc_profile(args.config)
            traffic = pmc_lookup(pmc["hbm_bytes_per_launch"], sym) if pmc else None
            mfma_busy = pmc_lookup(pmc.get("mfma_busy", {}), sym) if pmc else None
            # split kernels: the fp32-work ceiling is the bf16/fp16 MFMA rate over
            # the products per fp32 product (6 for bf16 x3, 3 for the fp16 x2 planes)
            split = sym.startswith("k_conv_x3") or sym.startswith("k_wgrad_x3")
            fpeak = (MFMA_BF16_PEAK_TFLOPS if cfg["bf16"] else
                     (F16X2_PEAK_TFLOPS if x3_planes(sym) == 2 else X3_PEAK_TFLOPS) if split
                     else MFMA_F32_PEAK_TFLOPS)
            # the roof that bounds the kernel's algorithmic work: MFMA or HBM
            # (the bf16 GEMMs over fp32 activations at 64-128 channels sit
            # below the bf16 ridge of 2500 / 8 = 312 FLOP/B)
            hbm = nb_tot / (HBM_PEAK_GBS * 1e9) > fl_tot / (fpeak * 1e12)
            if hbm:
                ach, peak, unit = nb_tot / (ms_tot * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s"
            else:
                ach, peak, unit = fl_tot / (ms_tot * 1e-3) / 1e12, fpeak, "TFLOP/s"
            out["roofline"] = {
                "kernel": sym, "bound": "hbm" if hbm else "mfma", "achieved": round(ach, 2),
                "peak": peak, "unit": unit,
                "frac": round(ach / peak, 4), "traffic": traffic,
                "traffic_source": pmc_src, "src_sha16": source_sha16(),
                "mfma_busy": mfma_busy,
                "algorithmic_bytes_per_launch": round(nb_tot / nl),
                "algorithmic_flops_per_launch": round(fl_tot / nl),
                "tflops": round(fl_tot / (ms_tot * 1e-3) / 1e12, 2),
                "gbs": round(nb_tot / (ms_tot * 1e-3) / 1e9, 1),
                "avg_launch_ms": round(ms_tot / nl, 4), "launches_per_step": nl,
                "per_kind_tflops": {k: round(v[1] / (v[0] * 1e-3) / 1e12, 1)
                                    for k, v in kinds.items()},
                "per_kind_gbs": {k: round(v[3] / (v[0] * 1e-3) / 1e9, 1) for k, v in kinds.items()},
                "per_kind_ms_per_step": {k: round(v[0], 3) for k, v in kinds.items()},
                "per_symbol_ms_per_step": {k: round(v[0], 3) for k, v in
                                           sorted(symbols.items(), key=lambda kv: -kv[1][0])}}
        if world == 1 and not args.no_cpu_baseline:
            progress("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
