T=distributed-drift-detection_amd/ddm_amd/libddm_amd_tunep.so
mkdir -p gpurun_out/r5m
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 --predict-replays 2 > gpurun_out/r5m/prod.json 2> gpurun_out/r5m/prod.err || exit 1
for k in 48 80; do DDM_AMD_LIB=$T DDM_ROW_LDS_KB=$k timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 --predict-replays 2 > gpurun_out/r5m/lds$k.json 2> gpurun_out/r5m/lds$k.err || exit 1; done
DDM_AMD_LIB=$T DDM_ROW_LDS_KB=80 DDM_SIDE_CU_STRIDE=4 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --companion 0 --predict-replays 2 > gpurun_out/r5m/lds80s4.json 2> gpurun_out/r5m/lds80s4.err
