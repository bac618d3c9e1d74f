# round-5 final evidence: the whole -m gpu suite, the smoke, the bench lines (profiles/r05/final)
mkdir -p gpurun_out/r5final; rm -f gpurun_out/r5final/*
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5final/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final/smoke.log 2>&1 || exit 1
for w in c3 c2 c5 c4 c1; do
  timeout -k 10 600 python -u bench.py --workload $w > gpurun_out/r5final/bench_$w.json 2> gpurun_out/r5final/bench_$w.err || exit 1
done
