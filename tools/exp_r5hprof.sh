# host-side cProfile of the default C3 bench (run-start costs)
mkdir -p gpurun_out/r5hprof
timeout -k 10 300 python -u -m cProfile -o gpurun_out/r5hprof/c3.prof bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5hprof/c3.json 2> gpurun_out/r5hprof/err.txt || exit 1
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/r5hprof/htrace timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5hprof/c3_trace.json 2>> gpurun_out/r5hprof/err.txt

