# the side stream (window shuffles) at normal instead of high queue priority
mkdir -p gpurun_out/r5prio
for p in -1 0 -1 0; do
  for w in c3 c5 c2; do
    DDM_SIDE_PRIORITY=$p timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5prio/${w}_p$p.json.$RANDOM 2>> gpurun_out/r5prio/err.txt || exit 1
  done
done
