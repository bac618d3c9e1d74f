# per-GPU shares of the strong-scaling workloads at N = 1 / 2 / 4 / 8 (bench.py --solo-world),
# one tree, one box: profiles/r05/solo/
mkdir -p gpurun_out/r5solo
for w in c3 c5 c2; do
  timeout -k 10 300 python bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5solo/${w}_s1.json 2> gpurun_out/r5solo/${w}_s1.err || exit 1
  for n in 2 4 8; do
    timeout -k 10 300 python bench.py --workload $w --solo-world $n --cpu-baseline 0 --companion 0 > gpurun_out/r5solo/${w}_s$n.json 2> gpurun_out/r5solo/${w}_s$n.err || exit 1
  done
done
