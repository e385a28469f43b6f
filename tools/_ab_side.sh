set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for sp in 1 2 3 4 5; do
  COEB_SIDE_SPLIT=$sp timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 > gpurun_out/ab_$sp.log 2>&1
done
COEB_SIDE_STREAM=0 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 > gpurun_out/ab_off.log 2>&1
