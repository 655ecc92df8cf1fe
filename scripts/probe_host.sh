echo "nproc=$(nproc)"; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/cgroup | head -3
grep -m1 "model name" /proc/cpuinfo; grep -c processor /proc/cpuinfo
