# Chunk-size sweep of the specialised conv GEMMs (kernel micro-bench).
set -u
mkdir -p gpurun_out
for ck in ${CK9S:-4 2}; do echo "CK9=$ck"; STGCN_CK9=$ck KB_WHICH=0,1 timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
for ck in ${CK1S:-16 8}; do echo "CK1=$ck"; STGCN_CK1=$ck KB_WHICH=3 timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
