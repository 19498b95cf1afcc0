set -u
cd "${GRAFT_REPO_ROOT}"
for v in old base; do
  if [ $v = base ]; then unset STGCN_LIB_VARIANT; else export STGCN_LIB_VARIANT=$v; fi
  echo "== $v"
  KB_BF16=1 KB_V=25 KB_K=3 KB_SHAPES=1,5 timeout -k 10 200 python scripts/kbench.py 10 || exit 1
done
