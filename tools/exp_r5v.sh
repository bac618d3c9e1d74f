# predict with two chunks in flight: C3 bench (+ replays) and the predict / configs tests (measurement aid)
mkdir -p gpurun_out/r5v
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --companion 0 --predict-replays 2 > gpurun_out/r5v/c3.json 2> gpurun_out/r5v/c3.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_predict.py tests/test_gpu_configs.py -m gpu > gpurun_out/r5v/tests.txt 2>&1
