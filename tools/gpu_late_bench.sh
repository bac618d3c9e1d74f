#!/bin/bash
# late-round bench lines: c5 (refit-heavy), c3 at the N=8 share, c1
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 > gpurun_out/late_c5.json 2> gpurun_out/late_c5.err || { tail -30 gpurun_out/late_c5.err; exit 1; }
timeout -k 10 200 python -u bench.py --solo-world 8 --cpu-baseline 0 > gpurun_out/late_c3s8.json 2> gpurun_out/late_c3s8.err || { tail -30 gpurun_out/late_c3s8.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload c1 --cpu-baseline 0 > gpurun_out/late_c1.json 2> gpurun_out/late_c1.err || { tail -30 gpurun_out/late_c1.err; exit 1; }
for w in c5 c3s8 c1; do python3 -c "
import json;d=json.loads(open('gpurun_out/late_$w.json').read().strip().splitlines()[-1]);b=d['breakdown']
print('$w', '%.4g rows/s' % d['value'], '%.2f ms/step' % d['ms_per_step'], 'epochs', b.get('epochs_per_step'), 'refits/s', b.get('refits_per_s'), b['checks'].get('events_sha1'))"; done
