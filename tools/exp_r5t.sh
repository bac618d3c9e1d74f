# slow first timed step: glibc's mmap threshold for the runs' dense outputs (measurement aid)
mkdir -p gpurun_out/r5t
B="python bench.py --steps 4 --warmup 1 --cpu-baseline 0 --companion 0"
timeout -k 10 200 $B > gpurun_out/r5t/p1.json 2> gpurun_out/r5t/p1.err || exit 1
timeout -k 10 200 $B > gpurun_out/r5t/p2.json 2> gpurun_out/r5t/p2.err || exit 1
MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 timeout -k 10 200 $B > gpurun_out/r5t/p3m.json 2> gpurun_out/r5t/p3m.err || exit 1
MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 timeout -k 10 200 $B > gpurun_out/r5t/p4m.json 2> gpurun_out/r5t/p4m.err
