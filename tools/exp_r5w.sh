# chain kernel with LDS-staged windows: scan-batches tests + C4 timing + kernel split (measurement aid)
mkdir -p gpurun_out/r5w
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_scan_batches.py -m gpu > gpurun_out/r5w/tests.txt 2>&1 || exit 1
timeout -k 10 200 python tools/c4_scan_time.py > gpurun_out/r5w/time.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5w/prof -o run -- python tools/c4_scan_time.py --reps 4 > gpurun_out/r5w/prof.txt 2>&1
