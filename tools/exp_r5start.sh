# host trace of the run start (finer marks), C3 and its N=8 share
mkdir -p gpurun_out/r5start
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/r5start/c3 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5start/c3.json 2> gpurun_out/r5start/err.txt || exit 1
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/r5start/s8 timeout -k 10 300 python -u bench.py --solo-world 8 --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5start/s8.json 2>> gpurun_out/r5start/err.txt
