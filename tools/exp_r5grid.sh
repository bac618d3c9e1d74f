# window-shuffle grids sized per group of epochs (default) vs by the runner's largest window
mkdir -p gpurun_out/r5grid
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_devctl.py tests/test_gpu_shuffle*.py > gpurun_out/r5grid/tests.log 2>&1 || exit 1
for g in fixed adapt fixed adapt; do
  for w in c5 c2 c3; do
    DDM_SHUF_GRID=$g timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5grid/${w}_$g.json.$RANDOM 2>> gpurun_out/r5grid/err.txt || exit 1
  done
done
