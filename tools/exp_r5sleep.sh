# poll sleep (DDM_FLAG_SLEEP builds: libddm_amd_s1 / default 8 / _s32) x speculative refits
mkdir -p gpurun_out/r5sleep
L=$PWD/distributed-drift-detection_amd/ddm_amd
run() {  # lib spec workload
  DDM_AMD_LIB=$L/$1 DDM_SPEC_REFIT=$2 timeout -k 10 300 python -u bench.py --workload $3 --cpu-baseline 0 --companion 0 > gpurun_out/r5sleep/$3_${1%.so}_k$2.json 2>> gpurun_out/r5sleep/err.txt
}
for w in c2 c3; do
  run libddm_amd_s1.so 0 $w || exit 1
  run libddm_amd.so 0 $w || exit 1
  run libddm_amd_s32.so 0 $w || exit 1
  run libddm_amd.so 2 $w || exit 1
  run libddm_amd_s32.so 2 $w || exit 1
done
run libddm_amd.so 0 c5 || exit 1
run libddm_amd.so 2 c5 || exit 1
