# kernel traces of c2 with and without speculative refits (one step each)
mkdir -p gpurun_out/r5spec3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in 0 2; do
DDM_SPEC_REFIT=$k timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5spec3/t$k -o c2 -- python3 bench.py --workload c2 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/r5spec3/c2_k$k.json 2> gpurun_out/r5spec3/c2_k$k.err || exit 1
done
