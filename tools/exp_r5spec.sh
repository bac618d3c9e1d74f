# speculative refits (DDM_SPEC_REFIT=K): the device-epoch tests, then A/B bench lines
mkdir -p gpurun_out/r5spec
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_devctl.py > gpurun_out/r5spec/tests.log 2>&1 || exit 1
for k in 0 2 0 2; do
  for w in c3 c5 c2; do
    DDM_SPEC_REFIT=$k timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5spec/${w}_k$k.json.$RANDOM 2>> gpurun_out/r5spec/err.txt || exit 1
  done
done
