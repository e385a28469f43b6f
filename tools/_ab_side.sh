set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
COEB_SIDE_OCTREE=1 timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "batch or golden or extract" > gpurun_out/pytest_gpu_oct.log 2>&1
for r in 1 2 3; do
  COEB_SIDE_BLUR=0 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab3_a.log 2>&1
  COEB_SIDE_BLUR=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab3_b.log 2>&1
  COEB_SIDE_OCTREE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-e2e --no-profile --steps 40 >> gpurun_out/ab3_c.log 2>&1
done
