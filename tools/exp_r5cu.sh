# C5 / c2 with the side stream (window shuffles) confined to every s-th CU (DDM_SIDE_CU_STRIDE)
mkdir -p gpurun_out/r5cu
for s in 0 2 4 8 0; do
  for w in c5 c2; do
    DDM_SIDE_CU_STRIDE=$s timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 > gpurun_out/r5cu/${w}_s$s.json.$RANDOM 2>> gpurun_out/r5cu/err.txt || exit 1
  done
done
