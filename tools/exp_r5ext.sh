# stream generation requested no further than the partition's last batch (devctl._extend)
mkdir -p gpurun_out/r5ext
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_devctl.py > gpurun_out/r5ext/tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > gpurun_out/r5ext/c3_$k.json 2>> gpurun_out/r5ext/err.txt || exit 1
  timeout -k 10 300 python -u bench.py --solo-world 8 --cpu-baseline 0 --companion 0 > gpurun_out/r5ext/c3s8_$k.json 2>> gpurun_out/r5ext/err.txt || exit 1
done
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > gpurun_out/r5ext/c2.json 2>> gpurun_out/r5ext/err.txt || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --cpu-baseline 0 > gpurun_out/r5ext/c5.json 2>> gpurun_out/r5ext/err.txt || exit 1
