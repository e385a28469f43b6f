set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
for v in "" corn448 lb5; do
  if [ -n "$v" ]; then export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; else unset COEB_LIB_PATH; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/var_$v.log 2>&1 || { echo "variant $v failed rc=$?"; tail -3 gpurun_out/var_$v.log; exit 1; }
  echo "[$v] $(grep -o '"k_fast": [0-9.]*' gpurun_out/var_$v.log)"
done
