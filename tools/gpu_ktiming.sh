#!/bin/bash
# c3 bench (N=1 and the N=8 share) after moving the kernel-timing events out of the timed steps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for a in "" "--solo-world 8" "--solo-world 4" "--solo-world 2"; do
  timeout -k 10 200 python -u bench.py $a --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/kt.json 2> gpurun_out/kt.err || { tail -30 gpurun_out/kt.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/kt.json').read().strip().splitlines()[-1]);b=d['breakdown']
print('[$a]', 'ms/step %.1f' % d['ms_per_step'], 'value %.3g' % d['value'], 'frac %.3f' % d['roofline']['frac'], 'pred %.1f dfit %.1f' % (b['predict_kernel_ms_per_step'], b['device_refit_kernels_ms_per_step']), b['checks'].get('events_sha1'))"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_scaling.py -x -q --timeout 300 --timeout-method thread > gpurun_out/scal.log 2>&1 || { tail -30 gpurun_out/scal.log; exit 1; }
tail -1 gpurun_out/scal.log
