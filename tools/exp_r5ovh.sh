mkdir -p gpurun_out/r5ovh
timeout -k 10 120 python -u tools/refit_overhead.py > gpurun_out/r5ovh/times.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ovh/prof -o ovh -- python3 tools/refit_overhead.py --reps 100 > gpurun_out/r5ovh/prof_times.txt 2>&1
