# kernel trace of rank 0's share of an 8-GPU C3 job (one partition), measurement aid
mkdir -p gpurun_out/r5y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5y/trace -o s8 -- python3 bench.py --solo-world 8 --steps 2 --warmup 1 --cpu-baseline 0 --companion 0 > gpurun_out/r5y/s8.json 2> gpurun_out/r5y/s8.err
