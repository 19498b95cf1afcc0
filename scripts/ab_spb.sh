set -u
cd "${GRAFT_REPO_ROOT}"
for v in base unfused ${VARIANTS:-}; do
  unset STGCN_LIB_VARIANT STGCN_UNFUSED_SPB
  if [ $v = unfused ]; then export STGCN_UNFUSED_SPB=1; elif [ $v != base ]; then export STGCN_LIB_VARIANT=$v; fi
  echo "== $v"
  timeout -k 10 120 python scripts/kbench_spb.py 10 || exit 1
  [ -n "${KB18:-}" ] && { KB_V=18 timeout -k 10 120 python scripts/kbench_spb.py 10 || exit 1; }
done
