# SQ counters of ddm_scan_batches' kernels on configs[3] (issue vs wait split)
mkdir -p gpurun_out/r5sq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex 'k_scan_batches' -d gpurun_out/r5sq/p1 -o run -- python3 tools/c4_scan_time.py --reps 2 > gpurun_out/r5sq/p1.txt 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES --kernel-include-regex 'k_scan_batches' -d gpurun_out/r5sq/p2 -o run -- python3 tools/c4_scan_time.py --reps 2 > gpurun_out/r5sq/p2.txt 2>&1
