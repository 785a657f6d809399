#!/bin/bash
# round-2 first check: host CPU share probe + GPU test suite on the rebuilt tree
set -o pipefail
mkdir -p gpurun_out
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/cpuinfo | grep "model name" | head -1; free -g; } > gpurun_out/host_probe.txt 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_r02a.log 2>&1
echo "pytest rc $?"
tail -3 gpurun_out/gputests_r02a.log
