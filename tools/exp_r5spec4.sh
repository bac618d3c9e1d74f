# speculative refits on the epoch stream itself (tuning build): bench lines and a c2 trace
mkdir -p gpurun_out/r5spec4
export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
DDM_SPEC_REFIT=2 DDM_SPEC_SAME_STREAM=1 timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > gpurun_out/r5spec4/c2_same.json 2>> gpurun_out/r5spec4/err.txt || exit 1
DDM_SPEC_REFIT=2 DDM_SPEC_SAME_STREAM=1 timeout -k 10 300 python -u bench.py --workload c3 --cpu-baseline 0 --companion 0 > gpurun_out/r5spec4/c3_same.json 2>> gpurun_out/r5spec4/err.txt || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DDM_SPEC_REFIT=2 DDM_SPEC_SAME_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5spec4/t -o c2 -- python3 bench.py --workload c2 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/r5spec4/c2_trace.json 2>> gpurun_out/r5spec4/err.txt
