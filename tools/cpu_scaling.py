"""Host CPU share of the GPU box: the cgroup CPU quota, affinity and physical cores, and the oracle's C2 rate
(oracle/mpc_oracle.c, OpenMP) at a range of thread counts.  usage: python tools/cpu_scaling.py [seconds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), os.path.join(ROOT, "oracle")]
import bench
import oracle as O
import workloads as W

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us",
          "/sys/fs/cgroup/cpuset.cpus.effective"):
    if os.path.exists(f):
        print(f, open(f).read().strip())
print("host", bench.host_cores(), "OMP_NUM_THREADS", os.environ.get("OMP_NUM_THREADS"))
wb = W.make_batch("C2")
ld = W.loader(wb["traj"])
orc = O.Oracle(ld.X_ref, ld.U_ref)
p = O.default_params(N=20)
for th in (1, 8, 16, 24, 32, 64, 128):
    orc.solve_batch(p, wb["x0"], num_threads=th)
    n, t0, c0 = 0, time.perf_counter(), time.process_time()
    while time.perf_counter() - t0 < budget:
        orc.solve_batch(p, wb["x0"], num_threads=th)
        n += wb["x0"].shape[0]
    dt, cpu = time.perf_counter() - t0, time.process_time() - c0
    print(f"threads {th:4d}: {n / dt:12.0f} solves/s, CPU time / wall = {cpu / dt:6.1f}", flush=True)
