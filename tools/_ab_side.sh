set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for r in 1 2; do
  COEB_MATCH_OVERLAP=0 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab4_off.log 2>&1
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab4_on.log 2>&1
  COEB_MATCH_OVERLAP=0 timeout -k 10 120 python bench.py --config D --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab4_Doff.log 2>&1
  timeout -k 10 120 python bench.py --config D --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab4_Don.log 2>&1
done
