# scan tail knobs (tuning build) + the slow-step malloc test (measurement aid)
T=distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
mkdir -p gpurun_out/r5u
timeout -k 10 300 python tools/c4_scan_time.py --sweep 'prod:' "fix4k:DDM_AMD_LIB=$T,DDM_FIX_BLOCKS=4096" "fix8k:DDM_AMD_LIB=$T,DDM_FIX_BLOCKS=8192" "refill8:DDM_AMD_LIB=$T,DDM_EXACT_REFILL=8" "refill48:DDM_AMD_LIB=$T,DDM_EXACT_REFILL=48" > gpurun_out/r5u/sweep.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5u/prof -o run -- python tools/c4_scan_time.py --reps 4 > gpurun_out/r5u/prof.txt 2>&1 || exit 1

B="python bench.py --steps 20 --warmup 1 --cpu-baseline 0 --companion 0"
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5u/first.json 2> gpurun_out/r5u/first.err || exit 1
timeout -k 10 300 $B > gpurun_out/r5u/second20.json 2> gpurun_out/r5u/second20.err
