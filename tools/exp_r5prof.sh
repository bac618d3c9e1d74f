# rocprofv3 kernel trace + stats of the default C3 bench command (the roofline's kernel average
# cross-check), final tree
mkdir -p gpurun_out/r5prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5prof/trace -o c3 -- python3 bench.py --cpu-baseline 0 --companion 0 > gpurun_out/r5prof/c3_prof_bench_line.json 2> gpurun_out/r5prof/c3_prof.err
