#!/bin/bash
# controller parity (the staging kernel), then the c3 epoch timing at N=1 and the N=8 share
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_controller.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_stage.log 2>&1 || { tail -30 gpurun_out/pt_stage.log; exit 1; }
tail -1 gpurun_out/pt_stage.log
for a in "" "--solo-world 8"; do
  timeout -k 10 200 python -u bench.py $a --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/kt.json 2> gpurun_out/kt.err || { tail -30 gpurun_out/kt.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/kt.json').read().strip().splitlines()[-1]);b=d['breakdown']
print('[$a]', 'ms/step %.1f' % d['ms_per_step'], 'value %.3g' % d['value'], b['checks'].get('events_sha1'))"
done
rm -rf gpurun_out/prof_st
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_st -o st -- python3 bench.py --solo-world 8 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_st.log 2>&1 || { tail -30 gpurun_out/prof_st.log; exit 1; }
grep -h "k_stage\|k_dfit\|cforest" gpurun_out/prof_st/*/*kernel_stats.csv gpurun_out/prof_st/*kernel_stats.csv 2>/dev/null | cut -c1-40,200-300 | head
