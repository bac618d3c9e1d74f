# late round 5, after the classify pass's lazy table reads: the whole -m gpu suite, the smoke,
# the c4 and default bench lines, the c4 kernel trace and the scan's FETCH / WRITE passes
# (profiles/r05/late)
mkdir -p gpurun_out/r5late; rm -rf gpurun_out/r5late/*
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5late/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5late/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c4 > gpurun_out/r5late/bench_c4.json 2> gpurun_out/r5late/bench_c4.err || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r5late/bench_c3.json 2> gpurun_out/r5late/bench_c3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5late/c4_trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > gpurun_out/r5late/c4_trace_line.json 2> gpurun_out/r5late/c4_trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_scan_batches|k_scan_prefix' -d gpurun_out/r5late/fetch -o run -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/r5late/fetch.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_scan_batches|k_scan_prefix' -d gpurun_out/r5late/write -o run -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/r5late/write.txt 2>&1
