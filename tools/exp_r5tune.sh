# the final tree's -m gpu suite and smoke, then a sweep of the classify pass's knobs (tuning build)
mkdir -p gpurun_out/r5tune
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5tune/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5tune/smoke.log 2>&1 || exit 1
export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
timeout -k 10 600 python -u tools/c4_scan_time.py --reps 15 --sweep base: st1:DDM_SCAN_STEPS=1 st3:DDM_SCAN_STEPS=3 st4:DDM_SCAN_STEPS=4 pop8:DDM_SCAN_POP=8 pop32:DDM_SCAN_POP=32 pop48:DDM_SCAN_POP=48 ref16:DDM_EXACT_REFILL=16 ref32:DDM_EXACT_REFILL=32 fix4k:DDM_FIX_BLOCKS=4096 base2: > gpurun_out/r5tune/sweep.json 2>&1
