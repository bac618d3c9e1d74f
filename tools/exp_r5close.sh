# round-5 close: the committed tree's -m gpu suite, smoke and c4 line (profiles/r05/late/close_*)
mkdir -p gpurun_out/r5close; rm -rf gpurun_out/r5close/*
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5close/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5close/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c4 > gpurun_out/r5close/bench_c4.json 2> gpurun_out/r5close/bench_c4.err
