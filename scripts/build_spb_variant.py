"""A/B variant library that differs from the default build only in one source
(kernels_spbwd.hip, or VARIANT_SRC=<file>) built with -D defines: compiles that
one source and links it with the default build's other objects
(st-gcn_amd/build/default). Usage:
  [VARIANT_SRC=kernels_x3.hip[,more.hip]] [VARIANT_CSRC=<dir>] \
      python scripts/build_spb_variant.py <name> DEFINE=VAL [...]  -> lib/libstgcn_hip_<name>.so
(VARIANT_CSRC: compile those sources from another source tree, e.g. an older
commit's csrc exported with git archive, for same-box A/B of a change)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "st-gcn_amd")
sys.path.insert(0, PKG)
import build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
objdir = os.path.join(PKG, "build", name)
os.makedirs(objdir, exist_ok=True)
srcs = os.environ.get("VARIANT_SRC", "kernels_spbwd.hip").split(",")
csrc = os.environ.get("VARIANT_CSRC", build.CSRC)
for src in srcs:
    subprocess.run([build.HIPCC, *build.FLAGS, *[f"-D{d}" for d in defs], "-c",
                    os.path.join(csrc, src), "-o", os.path.join(objdir, src + ".o")], check=True)
objs = [os.path.join(objdir if s in srcs else os.path.join(PKG, "build", "default"), s + ".o")
        for s in build.SOURCES]
out = os.path.join(PKG, "lib", f"libstgcn_hip_{name}.so")
subprocess.run([build.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out],
               check=True)
print(out)
