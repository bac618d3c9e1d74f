#!/bin/bash
# predict vec variants (slots per load chunk 2 / 4 / 6) on the C3 bench (replay timing).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=distributed-drift-detection_amd/ddm_amd
cp $L/libddm_amd.so /tmp/lib4.so
for ch in 2 4 6 2 4 6; do
if [ $ch = 4 ]; then cp /tmp/lib4.so $L/libddm_amd.so; else cp $L/libddm_amd_ch$ch.so $L/libddm_amd.so; fi
timeout -k 10 200 python -u bench.py --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c3_ch$ch.json 2> gpurun_out/c3_ch$ch.err || { tail -30 gpurun_out/c3_ch$ch.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_ch$ch.json'));b=d['breakdown'];r=d['roofline'];print('ch$ch', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['avg_launch_ms_in_step'])"
done
cp /tmp/lib4.so $L/libddm_amd.so
