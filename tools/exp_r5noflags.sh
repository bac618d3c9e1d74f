# timing probe (results wrong by design): the classify pass without its flag-byte stores, against the
# normal build, both under rocprofv3 --kernel-trace --stats (profiles/r05/scan/noflags); the variant is
#   tools/build_variant.sh noflags scan_batches.hip -DDDM_TUNING -DDDM_PROBE_NO_FLAGS
mkdir -p gpurun_out/noflags
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/noflags/base -o run -- python3 tools/c4_scan_time.py --reps 10 > gpurun_out/noflags/base.txt 2>&1 || exit 1
DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_noflags.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/noflags/nf -o run -- python3 tools/c4_scan_time.py --reps 10 > gpurun_out/noflags/nf.txt 2>&1
