# batched batch-0 perm upload and RNG-state read-back: device-epoch / controller tests, C3 lines with host traces
mkdir -p gpurun_out/r5start2
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_devctl.py tests/test_gpu_controller.py tests/test_gpu_configs.py > gpurun_out/r5start2/tests.log 2>&1 || exit 1
for k in 1 2; do
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/r5start2/c3_$k timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > gpurun_out/r5start2/c3_$k.json 2>> gpurun_out/r5start2/err.txt || exit 1
done
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > gpurun_out/r5start2/c2.json 2>> gpurun_out/r5start2/err.txt || exit 1
timeout -k 10 300 python -u bench.py --workload c1 --cpu-baseline 0 > gpurun_out/r5start2/c1.json 2>> gpurun_out/r5start2/err.txt || exit 1
