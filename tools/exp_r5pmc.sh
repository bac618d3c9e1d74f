# HBM traffic of ddm_scan_batches on configs[3] (rocprofv3 PMC, separate FETCH_SIZE / WRITE_SIZE passes)
mkdir -p gpurun_out/r5pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_scan_batches|k_scan_prefix' -d gpurun_out/r5pmc/fetch -o run -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/r5pmc/fetch.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_scan_batches|k_scan_prefix' -d gpurun_out/r5pmc/write -o run -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/r5pmc/write.txt 2>&1
