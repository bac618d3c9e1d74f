#!/bin/bash
# c3 at N=1 with 1, 2, 4 partition groups (GroupedRunner), and the N=2/4 per-GPU shares.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for a in "--groups 1" "--groups 2" "--groups 4" "--solo-world 2" "--solo-world 4" "--solo-world 2 --groups 2"; do
  timeout -k 10 200 python -u bench.py $a --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/grp.json 2> gpurun_out/grp.err || { tail -30 gpurun_out/grp.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/grp.json').read().strip().splitlines()[-1]);b=d['breakdown']
print('$a', 'ms/step %.1f' % d['ms_per_step'], 'value %.3g' % d['value'], 'epochs', b['epochs_per_step'], b['checks'].get('events_sha1'))"
done
