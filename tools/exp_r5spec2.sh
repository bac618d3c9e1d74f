# kernel trace of c2 with speculative refits (one step), to see where the epoch goes
mkdir -p gpurun_out/r5spec2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DDM_SPEC_REFIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5spec2/trace -o c2 -- python3 bench.py --workload c2 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/r5spec2/c2.json 2> gpurun_out/r5spec2/c2.err
