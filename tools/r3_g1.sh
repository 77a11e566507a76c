set -u
mkdir -p gpurun_out/r3g1
timeout -k 10 120 tools/ub_rates > gpurun_out/r3g1/ubench.txt 2>&1 || exit 1
cat gpurun_out/r3g1/ubench.txt
timeout -k 10 120 tools/tk_base 2048 base 512 > gpurun_out/r3g1/tk.txt 2>&1 || exit 1
cat gpurun_out/r3g1/tk.txt
nproc; grep -c processor /proc/cpuinfo; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
