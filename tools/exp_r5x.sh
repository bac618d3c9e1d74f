# level-1 rescans split over 1/2/4 waves per queue (measurement aid)
T=distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
mkdir -p gpurun_out/r5x
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_scan_batches.py -m gpu > gpurun_out/r5x/tests.txt 2>&1 || exit 1
timeout -k 10 300 python tools/c4_scan_time.py --sweep 'prod:' "split1:DDM_AMD_LIB=$T,DDM_EXACT1_SPLIT=1" "split4:DDM_AMD_LIB=$T,DDM_EXACT1_SPLIT=4" "split8:DDM_AMD_LIB=$T,DDM_EXACT1_SPLIT=8" > gpurun_out/r5x/sweep.txt 2>&1
