# A/B: the refit's pack folded into the trees kernel (DDM_DFIT_PACK_IN_TREES=1) vs its own launch
set -e
mkdir -p gpurun_out/r5pack
export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dfit.py tests/test_gpu_devctl.py > gpurun_out/r5pack/tests.log 2>&1
for v in 0 1 0 1; do
  for w in c5 c2; do
    DDM_DFIT_PACK_IN_TREES=$v timeout -k 10 300 python bench.py --workload $w --cpu-baseline 0 > gpurun_out/r5pack/${w}_p$v.json.$RANDOM 2>> gpurun_out/r5pack/err.txt
  done
done
