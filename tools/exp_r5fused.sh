# the controller's refits with the presort inside the tree kernel (DDM_FUSED_PREP=1) vs k_dfit_prep
mkdir -p gpurun_out/r5fused
for p in 0 1 0 1; do
  for w in c5 c2 c3; do
    DDM_FUSED_PREP=$p timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5fused/${w}_f$p.json.$RANDOM 2>> gpurun_out/r5fused/err.txt || exit 1
  done
done
