"""Build libstgcn_hip.so in-tree with hipcc for gfx950 (no cmake, no JIT)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libstgcn_hip.so")
SOURCES = ["kernels.hip", "kernels_bf16.hip", "kernels_x3.hip", "train_ops.hip", "capi.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wall"]


def build(verbose=False, variant=None, defines=()):
    """variant: build lib/libstgcn_hip_<variant>.so with extra -D defines (A/B
    kernel experiments, loaded with STGCN_LIB_VARIANT=<variant>)."""
    out = OUT if variant is None else os.path.join(os.path.dirname(OUT),
                                                   f"libstgcn_hip_{variant}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines],
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(verbose=True))
