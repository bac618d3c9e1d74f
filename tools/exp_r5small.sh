# one-workgroup shuffles of windows of <= 16 batches: the whole -m gpu suite, then A/B bench
# lines against a build without them (libddm_amd_nosmall.so, DDM_SMALL_WINDOW=0)
mkdir -p gpurun_out/r5small
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5small/gpu_tests.log 2>&1 || exit 1
L=$PWD/distributed-drift-detection_amd/ddm_amd
for v in nosmall small nosmall small; do
  lib=$L/libddm_amd.so; [ $v = nosmall ] && lib=$L/libddm_amd_nosmall.so
  for w in c5 c2 c3; do
    DDM_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > gpurun_out/r5small/${w}_$v.json.$RANDOM 2>> gpurun_out/r5small/err.txt || exit 1
  done
done
