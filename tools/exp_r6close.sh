#!/bin/bash
# round-6 close (late) on the committed tree: the whole -m gpu suite, the smoke, every bench line the
# driver and the judge read (c3 default with cpu_baseline + companion, c4, c2, c5, c1), the
# default C3 command under rocprofv3 --kernel-trace --stats  -> gpurun_out/r6close/
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6close && rm -rf gpurun_out/r6close/*
export TMPDIR=/tmp
O=gpurun_out/r6close
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
for w in c4 c2 c5 c1; do
  timeout -k 10 600 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_prof -o c3 -- python3 bench.py --cpu-baseline 0 --companion 0 > $O/c3_prof_line.json 2> $O/c3_prof.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'k_scan_batches|k_scan_prefix' --output-format csv -d $O/pmc_scan_$c -o p -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 --c4-check-stride 0 > $O/pmc_scan_$c.txt 2>&1 || exit 1
done
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py --workload c3 --solo-world $n --cpu-baseline 0 --companion 0 > $O/solo_c3_s$n.json 2> $O/solo_c3_s$n.err || { tail -5 $O/solo_c3_s$n.err; exit 1; }
done
for w in c2 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --solo-world 8 --cpu-baseline 0 > $O/solo_${w}_s8.json 2> $O/solo_${w}_s8.err || { tail -5 $O/solo_${w}_s8.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ("solo_c3_s2", "solo_c3_s4", "solo_c3_s8", "solo_c2_s8", "solo_c5_s8"):
    d = json.loads([l for l in open(f"gpurun_out/r6close/{f}.json") if l.startswith("{")][-1])
    print(f, round(d["ms_per_step"], 2), d["breakdown"]["checks"].get("events_sha1"))
for w in ("c3", "c4", "c2", "c5", "c1"):
    d = json.loads([l for l in open(f"gpurun_out/r6close/bench_{w}.json") if l.startswith("{")][-1])
    r = d["roofline"]; c = d.get("cpu_baseline") or {}
    print(w, f"value={d['value']:.4g}", f"ms/step={d['ms_per_step']:.2f}", f"frac={r['frac']:.3f}",
          f"vs_baseline={d.get('vs_baseline')}", f"cpu={c.get('value')}", list(d["breakdown"].get("checks", {}).keys()))
PY
echo done
