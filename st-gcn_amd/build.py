"""Build libstgcn_hip.so in-tree with hipcc for gfx950 (no cmake, no JIT).

Each source is compiled to its own object in parallel (no cross-TU device
calls, so no -fgpu-rdc is needed) and the objects are linked into one shared
library."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libstgcn_hip.so")
SOURCES = ["kernels.hip", "kernels_bf16.hip", "kernels_x3.hip", "kernels_fused.hip",
           "kernels_spbwd.hip", "kernels_fold.hip", "train_ops.hip", "capi.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall"]


def build(verbose=False, variant=None, defines=()):
    """variant: build lib/libstgcn_hip_<variant>.so with extra -D defines (A/B
    kernel experiments, loaded with STGCN_LIB_VARIANT=<variant>)."""
    out = OUT if variant is None else os.path.join(os.path.dirname(OUT),
                                                   f"libstgcn_hip_{variant}.so")
    objdir = os.path.join(HERE, "build", variant or "default")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    os.makedirs(objdir, exist_ok=True)
    defs = [f"-D{d}" for d in defines]

    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "stgcn_hip.h"))
    stamp = os.path.join(objdir, "defines.txt")
    same_defs = os.path.exists(stamp) and open(stamp).read() == " ".join(defs)

    def compile_one(src):
        obj = os.path.join(objdir, src + ".o")
        deps = [os.path.join(CSRC, src), *headers, __file__]
        if same_defs and os.path.exists(obj) and \
                os.path.getmtime(obj) > max(os.path.getmtime(p) for p in deps):
            return obj  # up to date
        cmd = [HIPCC, *FLAGS, *defs, "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    with open(stamp, "w") as fh:
        fh.write(" ".join(defs))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(verbose=True))
