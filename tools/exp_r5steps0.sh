# classify pass without / with its in-pass exact rows: per-kernel times (tuning build)
mkdir -p gpurun_out/r5steps0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_tune.so
for st in 0 2; do
DDM_SCAN_STEPS=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5steps0/s$st -o c4 -- python3 tools/c4_scan_time.py --reps 10 > gpurun_out/r5steps0/s$st.json 2> gpurun_out/r5steps0/s$st.err || exit 1
done
