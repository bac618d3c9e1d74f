#!/bin/bash
# One parameterised GPU session (run it under gpurun).  Steps are separated by "+"; each
# runs under its own time limit and the session stops at the first failure.
#
#   tools/gpu.sh tests [pytest args]          -> gpurun_out/pytest.log (all -m gpu tests by default)
#              + smoke                        -> gpurun_out/smoke.log
#              + bench NAME [bench.py args]   -> gpurun_out/bench_NAME.json (+ .err)
#              + prof NAME [bench.py args]    -> gpurun_out/prof_NAME/ (rocprofv3 --kernel-trace --stats)
#              + pmc NAME REGEX [bench args]  -> gpurun_out/pmc_NAME_{FETCH_SIZE,WRITE_SIZE}/ (one pass each)
#              + pmcx NAME REGEX 'CTR ...' [bench args] -> gpurun_out/pmcx_NAME/ (one pass of those counters)
#              + run NAME script.py [args]    -> gpurun_out/run_NAME.log
#              + htrace NAME [bench.py args]  -> gpurun_out/htrace_NAME.json (host phase marks, DDM_HOST_TRACE)
#
# e.g. tools/gpu.sh tests + bench c3 + bench c2 --workload c2 + prof c3 --cpu-baseline 0
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp

fail() { echo "step failed: $*"; exit 1; }

run_step() {
    local kind=$1; shift
    case $kind in
    tests)
        local args=("$@")
        [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
        timeout -k 10 1100 python -u -m pytest "${args[@]}" -x -q --timeout 240 --timeout-method thread \
            > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; fail tests; }
        tail -1 gpurun_out/pytest.log ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
            || { tail -20 gpurun_out/smoke.log; fail smoke; }
        tail -1 gpurun_out/smoke.log ;;
    bench)
        local name=$1; shift
        timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err \
            || { tail -30 gpurun_out/bench_$name.err; fail bench $name; }
        python3 - "$name" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/bench_{n}.json").read().strip().splitlines()[-1])
print(n, f"value={d['value']:.4g} ms/step={d['ms_per_step']:.2f} frac={d['roofline']['frac']:.3f}",
      "vs_baseline=%s" % d.get("vs_baseline"), "n_gpus=%s" % d["n_gpus"])
PY
        ;;
    prof)
        local name=$1; shift
        rm -rf gpurun_out/prof_$name
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o $name \
            -- python3 bench.py "$@" > gpurun_out/prof_$name.log 2>&1 || { tail -30 gpurun_out/prof_$name.log; fail prof $name; }
        echo "prof $name done" ;;
    pmc)
        local name=$1 rx=$2; shift 2
        for c in FETCH_SIZE WRITE_SIZE; do
            rm -rf gpurun_out/pmc_${name}_$c
            timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv \
                -d gpurun_out/pmc_${name}_$c -o p -- python3 bench.py "$@" \
                > gpurun_out/pmc_${name}_$c.json 2> gpurun_out/pmc_${name}_$c.err \
                || { tail -10 gpurun_out/pmc_${name}_$c.err; fail pmc $name $c; }
        done
        echo "pmc $name done" ;;
    pmcx)
        # one pass of the given counters (quoted, space separated; within one pass's slots)
        local name=$1 rx=$2 ctrs=$3; shift 3
        rm -rf gpurun_out/pmcx_${name}
        timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "$rx" --output-format csv \
            -d gpurun_out/pmcx_${name} -o p -- python3 bench.py "$@" \
            > gpurun_out/pmcx_${name}.json 2> gpurun_out/pmcx_${name}.err \
            || { tail -10 gpurun_out/pmcx_${name}.err; fail pmcx $name; }
        echo "pmcx $name done" ;;
    run)
        # any python script of the repo: run NAME script.py [args] -> gpurun_out/run_NAME.log
        local name=$1; shift
        timeout -k 10 600 python -u "$@" > gpurun_out/run_$name.log 2>&1 || { tail -30 gpurun_out/run_$name.log; fail run $name; }
        tail -5 gpurun_out/run_$name.log ;;
    htrace)
        local name=$1; shift
        DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/htrace_$name.json timeout -k 10 300 python -u bench.py "$@" \
            > gpurun_out/htrace_$name.out 2> gpurun_out/htrace_$name.err || { tail -30 gpurun_out/htrace_$name.err; fail htrace; }
        echo "htrace $name done" ;;
    *)
        fail "unknown step $kind" ;;
    esac
}

step=()
for a in "$@" "+"; do
    if [ "$a" = "+" ]; then
        [ ${#step[@]} -gt 0 ] && run_step "${step[@]}"
        step=()
    else
        step+=("$a")
    fi
done
