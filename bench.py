"""Benchmark of the hot path: batched tracking-QP solves on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--cpu-seconds S]

A step = one launch of the batched solver over the config's ego batch (C2: trajectory1,
N=20, B=4096 per GPU, seed 2; inputs resident in HBM).  Multi-GPU (one rank per GPU, started by
torch.distributed.run or by `bench.py --gpus N` itself): each rank solves its own contiguous shard of the
same ego stream (weak scaling, no data-path collective); the barrier, the max-over-ranks time and the
one telemetry gather go through libmpcqp's RCCL communicator (shard.ShardComm, mpc_comm_* in
include/mpcqp.h), not torch.distributed.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")
sys.path[:0] = [PKG, os.path.join(ROOT, "oracle")]

FP64_PEAK_TFLOPS = 78.6     # MI355X dense FP64 (vector == matrix), MI355X_MICROARCH / AMD spec
HBM_PEAK_GBS = 8000.0


def algorithmic_flops(N, K):
    """F = 20N^2 + 24N^3 + K(48N^3 + 8N^3/3 + 64N^2)  (dense condensed-PDIP count)."""
    return 20 * N ** 2 + 24 * N ** 3 + K * (48 * N ** 3 + 8 * N ** 3 / 3 + 64 * N ** 2)


def riccati_flops(N, K):
    """Useful FP64 flops of the algorithm the kernel actually runs (stage-wise Riccati form),
    per solve: setup + crossover (one factorisation, two solves) + K interior-point iterations (one
    factorisation, two solves and the row phases each).  Per stage: factorisation 230, solve 84, row
    phases 450 (FMA = 2); the redundant and idle lanes of the SIMD implementation are not counted."""
    fac, sol, rows = 230, 84, 450
    return N * (fac + 2 * sol + 60) + K * N * (fac + 2 * sol + rows)


def algorithmic_bytes(N, max_obs):
    """x0 40 + obstacles 16*max_obs + n_obs 4 ; u0 16 + U 16N + pred_X 40(N+1) + status/iters 8."""
    return 40 + 16 * max_obs + (4 if max_obs else 0) + 16 + 16 * N + 40 * (N + 1) + 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inflight", type=int, default=4, metavar="K",
                    help="secondary serving leg: K independent batches of the same shape in flight on K streams "
                         "(one solver context each); reported as 'inflight', never as 'value' (0: skip)")
    ap.add_argument("--nlp-steps", type=int, default=5, metavar="K",
                    help="secondary leg: K batches of the same egos solved with the drop-in default (Gauss-Newton "
                         "SQP to the reference NLP optimum, trajectory_tracking.SQP_ITERS / sqp_tol); 0: skip")
    ap.add_argument("--closed-loop", type=int, default=512, metavar="B",
                    help="also run B egos per GPU through the device closed loop (mpc_closed_loop, SURVEY 8(f)1) "
                         "on the config's trajectory and FSM preset, gather their check quantities to rank 0 and "
                         "report closed-loop ego-steps/s (0: skip)")
    ap.add_argument("--plan-chunks", type=int, default=65536, metavar="B",
                    help="offline-planner leg (SURVEY 8(f)4, libmpcplan): B chunk NLPs per GPU posed as "
                         "optimize_full_trajectory poses them (20 m chunks, per-chunk horizon) on --plan-route; "
                         "reported as 'plan' in chunks/s, never as 'value' (0: skip)")
    ap.add_argument("--plan-steps", type=int, default=3, metavar="K")
    ap.add_argument("--plan-fleet", type=int, default=1024, metavar="B",
                    help="planner leg, secondary: B full plans on trajectory1's route from random starts, all "
                         "advancing together (trajectory_planning.optimize_full_trajectory_batch), rank 0 only")
    ap.add_argument("--plan-route", default="traj3")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: a stand-in that runs the same sharded path on libmpcqp's host backend (device = -1) "
                         "with gloo, for the launcher tests; never a measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched as `python bench.py --gpus N`: start N rank processes before this process touches a GPU
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; run it with --gpus equal to the "
                         "number of rank processes")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = args.device == "gpu"

    import numpy as np
    import torch
    import __graft_entry__ as ge
    # one build per node (a no-op when the in-tree libraries are current); the other ranks load them
    # after the barrier below
    if local == 0:
        ge.build()
    import mpcqp
    import workloads as W

    if gpu:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py needs a GPU (the measurement runs libmpcqp's HIP kernels; --device cpu is "
                             "a test stand-in, not a measurement)")
        torch.cuda.set_device(local)
    import shard
    # the ranks' one collective (and the measurement's barrier / max over ranks): RCCL through libmpcqp's
    # C ABI on GPU ranks (the unique id over a TCP rendezvous, no torch.distributed), gloo for the CPU stand-in
    comm = shard.ShardComm.from_env(local if gpu else None)
    comm.barrier()
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    dev_index = local if gpu else -1
    cfg = W.CONFIGS[args.config]
    B = args.batch or cfg["B"] // max(1, cfg["gpus"])
    lo, hi = shard.shard_range(world * B, world, rank)      # weak scaling: B egos per GPU
    wb = W.make_batch(args.config, B=hi - lo, offset=lo)
    N, mo = wb["N"], wb["max_obs"]
    X, U = W.loader(wb["traj"]).X_ref, W.loader(wb["traj"]).U_ref
    slv = mpcqp.Solver(X, U, mpcqp.default_params(N=N, max_obs=mo), device=dev_index)

    if gpu:
        t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
        x0 = t(wb["x0"])
        obs = t(wb["obs"]) if wb["obs"] is not None else None
        nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
        u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
        Uo = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
        Xo = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        it = torch.empty(B, dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        ptr = lambda x: 0 if x is None else x.data_ptr()

        def step():
            slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(u0), ptr(Uo), ptr(Xo), ptr(st), ptr(it),
                                   stream=stream.cuda_stream)
        sync = lambda: torch.cuda.synchronize(dev)
    else:
        host = {}

        def step():
            host.update(slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"]))
        sync = lambda: None

    for _ in range(args.warmup):
        step()
    sync()
    comm.barrier()
    sync()
    # the timed region: K back-to-back steps between two events (an event recorded between steps would add its
    # own ~3.5 us to every step); the per-step latencies (p50) come from a second, instrumented pass after it
    if gpu:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    tk = [t0]
    if gpu:
        ev0.record(stream)
    for i in range(args.steps):
        step()
        if not gpu:
            tk.append(time.perf_counter())
    if gpu:
        ev1.record(stream)
    sync()
    comm.barrier()
    sync()
    wall = time.perf_counter() - t0
    if gpu:
        gpu_s = ev0.elapsed_time(ev1) / 1e3
        nlat = min(args.steps, 50)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nlat + 1)]
        ev[0].record(stream)
        for i in range(nlat):
            step()
            ev[i + 1].record(stream)
        sync()
        step_ms = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(nlat)])
    else:
        step_ms = np.diff(np.array(tk)) * 1e3
        gpu_s = float(step_ms.sum()) / 1e3
    elapsed = comm.max(max(wall, gpu_s))

    # the one collective: gather of per-rank solver telemetry (after the timed region)
    st_h = st.cpu().numpy() if gpu else host["status"]
    it_h = it.cpu().numpy() if gpu else host["iters"]
    mat = shard.gather_telemetry(shard.telemetry(st_h, it_h), comm)
    # rank 0 reports the whole job; the other ranks' figures below are their own shard's (not printed)
    tel = shard.reduce_telemetry(mat if mat is not None else shard.gather_telemetry(shard.telemetry(st_h, it_h)))
    kmean = tel["mean_iters"]
    avg_launch_s = gpu_s / args.steps
    flops = algorithmic_flops(N, kmean) * B
    rflops = riccati_flops(N, kmean) * B
    nbytes = algorithmic_bytes(N, mo) * B
    # PMC counters cannot be read inside this process (rocprofv3 collects them in their own runs,
    # tools/gpu/bench_profiles.sh); `traffic` is the per-step HBM bytes of the last such run of this config,
    # reported with the run it came from
    traffic, traffic_source = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_hbm_bytes.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            traffic = pj.get(args.config)
            d = pj.get(args.config + "_detail", {})
            traffic_source = {"file": "profiles/pmc_hbm_bytes.json", "round": d.get("round"),
                              "commit": d.get("commit"), "counters": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                              "(separate passes), 2*FETCH_SIZE + WRITE_SIZE per step"}
        except Exception:
            traffic = None

    executed = executed_work(args.config)
    # closed-loop leg on every rank (its own ego shard), one gather to rank 0; after the headline timing
    cl = closed_loop(args.config, args.closed_loop, N, dev_index, comm) if args.closed_loop else None
    # offline-planner leg on every rank (its own chunk shard)
    plan = plan_leg(args.plan_chunks, args.plan_steps, args.plan_route, comm, dev, args.cpu_seconds,
                    not args.no_cpu) if (args.plan_chunks and gpu) else None
    if plan is not None and args.plan_fleet > 0:
        try:
            plan["fleet"] = plan_fleet(args.plan_fleet, dev_index)
        except Exception as e:      # a secondary leg never takes the headline line down with it
            plan["fleet"] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        out = {
            "metric": "tracking-QP solves/sec @ N=20, batch=4096; p50 solve latency",
            "value": world * B * args.steps / elapsed,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "p50_batch_latency_ms": float(np.median(step_ms)),
            "timing": "value / ms_per_step: the K timed steps back to back between two HIP events (max over ranks, "
                      "bracketed by barrier + synchronize); p50: a second pass of min(K, 50) steps with an event "
                      "after each",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: trajectory{wb['traj']}.json, N={N}, batch={B} egos per GPU, "
                                   f"max_obs={mo}, seed {cfg['seed']} (SURVEY 8d)", "global_batch": world * B,
                       "horizon": N, "parallelism": f"dp{world} (ego shards)"},
            "comm": {"transport": comm.transport,
                     "note": "the ranks' one exchange (barrier, max-over-ranks time, telemetry gather): 'rccl' = "
                             "libmpcqp's communicator (mpc_comm_*), 'local' = world 1, 'gloo' = the CPU stand-in"},
            "solver": tel,
            "roofline": {"bound": "fp64-valu", "achieved": flops / avg_launch_s / 1e12, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": flops / avg_launch_s / 1e12 / FP64_PEAK_TFLOPS,
                         "traffic": traffic, "traffic_source": traffic_source,
                         "compute_unit": "FP64 VALU: the kernels issue no MFMA instructions (DESIGN.md 2, 'Why no "
                                         "MFMA'); the peak is MI355X's FP64 rate, which is the same 78.6 TFLOP/s "
                                         "for vector and matrix instructions",
                         "achieved_basis": "SURVEY 8(d) flop count of a dense condensed PDIP (24N^3 per Hessian, "
                                           "48N^3 per iteration), F(N, mean iters) x B / avg step time; this is an "
                                           "equivalent dense-QP rate, not executed work",
                         "riccati_TFLOPs": rflops / avg_launch_s / 1e12,
                         "riccati_note": "useful flops of the stage-wise Riccati algorithm that runs (bench."
                                         "riccati_flops), the same time base",
                         "limiter": "latency of the slowest interior-point instance: the deferred instances fill "
                                    "fewer waves than the chip has SIMDs, so the batch time is one wave's FP64 "
                                    "issue time over its iterations (DESIGN.md 4)",
                         "note": "HIP events on the launch stream; a step is the path's launch pair: crossover "
                                 "kernel + interior-point kernel on the deferred instances (DESIGN.md 3); traffic = "
                                 "PMC HBM bytes per step (profiles/pmc_hbm_bytes.json)",
                         "hbm_algorithmic_GBs": nbytes / avg_launch_s / 1e9,
                         "executed_frac": executed.get("executed_frac"), "valu_busy": executed.get("valu_busy"),
                         "executed": executed},
        }
        if not gpu:
            out["device"] = "cpu-standin"
            out["note"] = ("--device cpu: libmpcqp's host backend with gloo, a stand-in for the launcher tests; "
                           "the roofline fields are not a GPU measurement")
        if args.nlp_steps > 0 and gpu:
            out["nlp_sqp"] = nlp_leg(args.nlp_steps, wb, B, N, mo, X, U, dev)
        if args.inflight > 1 and gpu:
            head = {k: v.cpu().numpy() for k, v in (("st", st), ("it", it), ("U", Uo))}
            out["inflight"] = inflight(args.inflight, args.steps, wb, B, N, mo, X, U, dev, head)
        if cl is not None:
            out["closed_loop"] = cl
        if plan is not None:
            out["plan"] = plan
        if not args.no_cpu and gpu:
            out["cpu_backend"] = cpu_backend(wb, N, mo, min(args.cpu_seconds, 5.0))
            out["cpu_reference"] = cpu_reference(wb, N, args.cpu_seconds)
            # last: its final run puts one thread on every physical core, beyond the process's CPU quota
            out["cpu_baseline"] = cpu_baseline(wb, N, mo, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    comm.close()


def launch_ranks(args):
    """`python bench.py --gpus N` without torchrun: start N rank processes (torch.distributed.run as a child
    process, rendezvous on 127.0.0.1) before this process makes any GPU call, pass their output through, and
    check rank 0's JSON line.  Returns the exit code: non-zero when N exceeds the visible devices, when a rank
    fails, or when rank 0's line does not report n_gpus == N."""
    import socket
    import subprocess
    if args.device == "gpu":
        import torch
        visible = torch.cuda.device_count()        # counts devices without initialising HIP on this image
        if args.gpus > visible:
            print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) are visible", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for ln in proc.stdout:
        sys.stdout.write(ln)
        sys.stdout.flush()
        if ln.startswith("{"):
            line = ln
    rc = proc.wait()
    if rc != 0:
        return rc
    if line is None:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        return 1
    got = json.loads(line).get("n_gpus")
    if got != args.gpus:
        print(f"bench.py: rank 0 reports n_gpus={got}, expected {args.gpus}", file=sys.stderr)
        return 1
    return 0


def nlp_leg(steps, wb, B, N, mo, X, U, dev):
    """Secondary leg (not `value`): the same egos through the drop-in default of the Python surface,
    i.e. the Gauss-Newton SQP that converges to the optimum of the reference's nonlinear problem
    (tests/test_gpu_nlp.py pins it to nlp_golden); one batch at a time, HIP events on the launch stream."""
    import numpy as np
    import torch
    import mpcqp
    import trajectory_tracking as TT
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    ptr = lambda x: 0 if x is None else x.data_ptr()
    p = mpcqp.default_params(N=N, max_obs=mo, sqp_iters=TT.SQP_ITERS)
    slv = mpcqp.Solver(X, U, p, device=dev.index)
    x0 = t(wb["x0"])
    obs = t(wb["obs"]) if wb["obs"] is not None else None
    nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
    o = [torch.empty((B, 2), dtype=torch.float64, device=dev), torch.empty((B, N, 2), dtype=torch.float64, device=dev),
         torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev)]
    stream = torch.cuda.current_stream(dev)
    call = lambda: slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, *[ptr(a) for a in o],
                                          stream=stream.cuda_stream)
    call()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ev[0].record(stream)
    for i in range(steps):
        call()
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    ms = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])
    st, it = o[3].cpu().numpy(), o[4].cpu().numpy()
    slv.close()
    return {"value": B * steps / (ms.sum() / 1e3), "unit": "solves/s", "ms_per_batch": float(ms.mean()),
            "p50_batch_latency_ms": float(np.median(ms)), "sqp_iters_cap": TT.SQP_ITERS, "sqp_tol": p.sqp_tol,
            "mean_pdip_iters": float(it.mean()), "status_counts": np.bincount(st & 15, minlength=4).tolist(),
            "sqp_unconverged": int(((st & 16) != 0).sum()),
            "note": "drop-in default of the Python surface (TrajectoryTracker.solve): SQP re-linearisations until "
                    "U moves by <= sqp_tol (or a 2-cycle / 5 elastic QPs in a row, include/mpcqp.h); secondary, the headline is the single tracking QP"}


def inflight(K, steps, wb, B, N, mo, X, U, dev, head):
    """Serving leg (not the headline `value`): K independent batches of B solves in flight at once, one
    solver context and one HIP stream each, `steps` rounds of K submissions.  A single batch leaves SIMDs idle
    while its slowest interior-point instance finishes (tail bound); independent batches on
    other streams fill them.  Every batch solves the headline inputs, and after the timed rounds each
    context's last outputs (U, status, iterations) must equal the headline run's bit for bit, or this raises;
    rank 0 only, after the headline timing."""
    import numpy as np
    import torch
    import mpcqp
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    ptr = lambda x: 0 if x is None else x.data_ptr()
    x0 = t(wb["x0"])
    obs = t(wb["obs"]) if wb["obs"] is not None else None
    nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
    ctx = []
    for _ in range(K):
        slv = mpcqp.Solver(X, U, mpcqp.default_params(N=N, max_obs=mo), device=dev.index)
        o = dict(u0=torch.empty((B, 2), dtype=torch.float64, device=dev),
                 U=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
                 X=torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev),
                 st=torch.empty(B, dtype=torch.int32, device=dev), it=torch.empty(B, dtype=torch.int32, device=dev))
        ctx.append((slv, torch.cuda.Stream(dev), o))

    def submit(slv, stream, o):
        slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(o["u0"]), ptr(o["U"]), ptr(o["X"]),
                               ptr(o["st"]), ptr(o["it"]), stream=stream.cuda_stream)

    cur = torch.cuda.current_stream(dev)
    for c in ctx:                                   # warm-up, and inputs visible to every stream
        c[1].wait_stream(cur)
        submit(*c)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        for c in ctx:
            submit(*c)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for k, c in enumerate(ctx):
        o = c[2]
        if not (np.array_equal(o["st"].cpu().numpy(), head["st"]) and np.array_equal(o["it"].cpu().numpy(), head["it"])
                and np.array_equal(o["U"].cpu().numpy(), head["U"])):
            raise RuntimeError(f"inflight: context {k}'s outputs differ from the headline batch's")
    same = True
    for c in ctx:
        c[0].close()
    return {"batches_in_flight": K, "value_per_gpu": K * steps * B / dt, "unit": "solves/s",
            "ms_per_batch": dt * 1e3 / (K * steps), "batches": K * steps, "outputs_identical_to_headline": same,
            "note": "secondary serving measurement on rank 0 (per GPU): independent batches of the same shape on "
                    "K streams; the headline value above is one batch at a time"}


def closed_loop(config, B, N, device, comm, max_steps=3000, hist_egos=4):
    """B egos per GPU through run_simulation on the device (trajectory_tracking.py:377-443, mpc_closed_loop):
    starts near the reference start (s0 ~ U(0,2), v0 ~ U(0.5,2)) drawn for all world * B egos,
    each rank running its contiguous shard with the config's FSM preset, until every ego passed s_max - 1
    or max_steps.  Drop-in solver default (Gauss-Newton SQP to the reference NLP optimum).  The one
    collective: a gather to rank 0 of every ego's check quantities and the FP32 histories of the first
    hist_egos egos of each shard (shard.py); rank 0 applies the restated verdicts to every ego."""
    import numpy as np
    import mpcqp
    import shard
    import workloads as W
    import trajectory_tracking as TT
    world, rank = comm.world, comm.rank
    cfg = W.CONFIGS[config]
    ld = W.loader(cfg["traj"])
    total = world * B
    rng = np.random.default_rng(cfg["seed"])
    s0, v0 = rng.uniform(0.0, 2.0, total), rng.uniform(0.5, 2.0, total)
    lo, hi = shard.shard_range(total, world, rank)
    x_init = np.array([[s0[i], 0.0, 0.0, ld.get_state(s0[i])[3], v0[i]] for i in range(lo, hi)])
    fsm_obj = None
    if cfg["obstacles"] in ("fsm2", "fsm3"):
        fsm_obj = TT.ObstaclesFSM(True, True, preset="trajectory2" if cfg["obstacles"] == "fsm2" else "trajectory3")
    fsm = TT.fsm_params(fsm_obj)
    p = mpcqp.default_params(N=N, sqp_iters=TT.SQP_ITERS)
    slv = mpcqp.Solver(ld.X_ref, ld.U_ref, p, device=device)
    comm.barrier()
    t0 = time.perf_counter()
    r = slv.closed_loop(x_init, fsm, max_steps=max_steps, s_max=ld.s_max)
    dt = comm.max(time.perf_counter() - t0)
    slv.close()
    tl_pos = fsm_obj.tl_pos if fsm_obj is not None else 0.0
    q = shard.closed_loop_quantities(r, lo, fsm_obj is not None, fsm_obj is not None, tl_pos)
    rows = -(-total // world)
    payloads = shard.gather_closed_loop(shard.pack_closed_loop(q, r, rows, hist_egos, max_steps), comm)
    if rank != 0:
        return None
    rep = shard.closed_loop_report(payloads, rows, hist_egos, max_steps, tuple(p.u_min), tuple(p.u_max), ld.s_max)
    ms = r["step_ms"][np.isfinite(r["step_ms"])]
    return {"egos": rep["egos"], "ranks": rep["ranks"], "ego_steps": rep["ego_steps"], "seconds": dt,
            "ego_steps_per_s": rep["ego_steps"] / dt, "loop_steps_rank0": int(r["n_steps"].max()),
            "p50_step_ms_rank0": float(np.median(ms)) if ms.size else None,
            "finished": int((rep["quantities"][:, 1] < max_steps).sum()), "checks_passed": rep["checks_passed"],
            "fsm": cfg["obstacles"], "sqp_iters": TT.SQP_ITERS, "sqp_tol": p.sqp_tol,
            "gathered_histories": f"FP32 [{rep['hist'].shape[0]} egos x {max_steps} steps x {shard.HIST_COLS}]",
            "note": "restated trajectory_tracking_check verdicts applied by rank 0 to the gathered per-ego check "
                    "quantities; real-time check = each batched step's device time (the latency of every ego's "
                    "answer)"}


def executed_work(config):
    """Executed FP64 work of this config's dominant kernel from the newest PMC pass over it (rocprofv3 --pmc
    SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES in their own
    run: tools/gpu/pmc_f64.sh, joined with the kernel-stats CSV of the same command by tools/pmc_f64.py into
    profiles/r<NN>_pmc_f64_<config>.csv).
    The dominant kernel is the one with the largest total duration in that kernel-stats run (average x
    launches); executed_frac = (2 FMA + MUL + ADD + TRANS) x 64 lanes / its average duration / 78.6 TF, an
    upper bound since the recursions issue under narrowed exec masks; valu_busy = SQ_ACTIVE_INST_VALU /
    SQ_WAVE_CYCLES.  Without a usable file the result says why ('unmeasured'), never a silent null."""
    import csv
    prof = os.path.join(ROOT, "profiles")
    # the newest round's pass of this config (profiles/r<NN>_pmc_f64_<config>.csv)
    cands = sorted(f for f in os.listdir(prof) if f.endswith(f"_pmc_f64_{config}.csv"))
    if not cands:
        return {"unmeasured": f"no profiles/r<NN>_pmc_f64_{config}.csv (no PMC pass over this config)"}
    path = os.path.join(prof, cands[-1])
    rows = list(csv.DictReader(open(path)))
    f = lambda r, k: float(r[k]) if r.get(k) not in (None, "") else None
    timed = [r for r in rows if f(r, "avg_duration_s")]
    if not timed:
        return {"unmeasured": f"profiles/{cands[-1]} has no kernel durations (its PMC pass was not joined with a "
                              "kernel-stats run)", "source": "profiles/" + cands[-1]}
    total = lambda r: f(r, "total_duration_s") or f(r, "avg_duration_s") * float(r.get("launches") or 1)
    top = max(timed, key=total)
    return {"executed_frac": f(top, "executed_frac_upper"), "valu_busy": f(top, "valu_busy"),
            "executed_TFLOPs": f(top, "executed_TFLOPs_upper"), "kernel": top["kernel"],
            "source": "profiles/" + cands[-1], "stats_file": top.get("stats_file"),
            "per_kernel": {r["kernel"]: {"executed_TFLOPs_upper": f(r, "executed_TFLOPs_upper"),
                                         "executed_frac_upper": f(r, "executed_frac_upper"),
                                         "valu_busy": f(r, "valu_busy"), "fp64_insts": f(r, "fp64_insts"),
                                         "avg_duration_s": f(r, "avg_duration_s")} for r in rows},
            "basis": "dominant kernel = largest total duration in the kernel-stats run of the same command; FP64 "
                     "VALU instruction counts x 64 lanes / its average duration (upper bound: the Riccati "
                     "recursions issue under exec masks of 5-10 lanes); valu_busy = SQ_ACTIVE_INST_VALU / "
                     "SQ_WAVE_CYCLES"}


def plan_leg(B, steps, route_name, comm, dev, cpu_s, with_cpu):
    """Offline planner: B chunk NLPs per GPU (workloads.plan_batch_ref: 20 m chunks at random
    positions of the route, each with the reference's own horizon rule, 10% final chunks), solved on the device
    by libmpcplan, one launch per residency class of horizons (the chunks come sorted by N; a class's launch
    sizes its LDS for its largest N, mpcplan.Planner.horizon_groups) on side streams; `steps` timed passes over the batch after one warm-up, HIP events on that stream,
    max over ranks.  On rank 0 also: the oracle (oracle/plan_oracle.c, OpenMP) and the restated reference
    path (scipy SLSQP on the chunk NLP, oracle/plan_ref.py) on bounded samples of the same chunks, and the
    GPU-vs-oracle agreement on the oracle's sample."""
    import numpy as np
    import torch
    import mpcplan
    import shard
    import workloads as W
    world, rank = comm.world, comm.rank
    r = W.plan_route(route_name)
    lo, hi = shard.shard_range(world * B, world, rank)
    wb = W.plan_batch_ref(r, hi - lo, seed=7, offset=lo)
    Bl = hi - lo
    Nv = wb["N"]
    # the rank's own device: the context's route and every launch live on cuda:LOCAL_RANK
    pl = mpcplan.Planner(r, mpcplan.default_params(N=int(Nv.max())), device=dev.index)
    if pl.device != dev.index:
        raise RuntimeError(f"planner context on device {pl.device}, the rank's device is {dev.index}")
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin, Nd = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32), t(Nv, torch.int32)
    # one launch per residency class (Planner.horizon_groups: the horizons whose own launches would keep the
    # same chunks per CU share one launch sized for the largest, with per-chunk N), so each launch's
    # longest-first order starts the class's slowest chunk first and no launch waits behind another's tail
    groups = []
    hg = pl.horizon_groups(Nv)
    for lo_n, hi_n in hg:
        i0, i1 = np.searchsorted(Nv, lo_n), np.searchsorted(Nv, hi_n, side="right")
        groups.append((int(hi_n), int(i0), int(i1), torch.empty((i1 - i0, hi_n + 1, 5), dtype=torch.float64, device=dev),
                       torch.empty((i1 - i0, hi_n, 2), dtype=torch.float64, device=dev),
                       torch.empty((i1 - i0, hi_n), dtype=torch.float64, device=dev)))
    o = [torch.empty(Bl, dtype=torch.int32, device=dev) for _ in range(3)]
    stream = torch.cuda.current_stream(dev)
    # the launches run concurrently on side streams (a launch's time is set by its slowest chunk, so
    # serialised launches would add their tails), the largest horizons first
    side = [torch.cuda.Stream(dev) for _ in range(min(4, len(groups)))]
    order = sorted(range(len(groups)), key=lambda g: -groups[g][0])
    d8, d4 = 8, 4

    def launches():
        for k, g in enumerate(order):
            n, i0, i1, Xg, Ug, Sg = groups[g]
            pl.solve_chunks_device(i1 - i0, n, Nd.data_ptr() + d4 * i0, x0.data_ptr() + d8 * 5 * i0,
                                   st.data_ptr() + d8 * i0, fin.data_ptr() + d4 * i0, Xg.data_ptr(), Ug.data_ptr(),
                                   Sg.data_ptr(), o[0].data_ptr() + d4 * i0, o[1].data_ptr() + d4 * i0,
                                   o[2].data_ptr() + d4 * i0, stream=side[k % len(side)].cuda_stream)

    def fork():
        e0 = torch.cuda.Event()
        e0.record(stream)
        for ss in side:
            ss.wait_event(e0)

    def join():
        for ss in side:
            e = torch.cuda.Event()
            e.record(ss)
            stream.wait_event(e)

    def step():
        fork()
        launches()
        join()
    step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(steps):
        step()
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])
    el = comm.max(max(wall, ms.sum() / 1e3))
    # secondary: the same batches back to back with no join between them (a planning service fed
    # continuously), so one batch's slowest chunks overlap the next batch's launches on the other streams
    comm.barrier()
    ep = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t1 = time.perf_counter()
    ep[0].record(stream)
    fork()
    for i in range(steps):
        launches()
    join()
    ep[1].record(stream)
    torch.cuda.synchronize(dev)
    pel = comm.max(max(time.perf_counter() - t1, ep[0].elapsed_time(ep[1]) / 1e3))
    status, iters, sqp = (a.cpu().numpy() for a in o)
    out = None
    if rank == 0:
        out = {"metric": "offline-planner chunk NLPs solved/s", "value": world * Bl * steps / el, "unit": "chunks/s",
               "ms_per_step": el * 1e3 / steps, "chunks_per_gpu": Bl, "steps": steps, "dtype": "f64",
               "workload": f"{route_name} (the committed trajectory{route_name[4:]}.json line, 50 then 30 km/h; "
                           f"{r.s_total:.0f} m), 20 m chunks as optimize_full_trajectory poses them "
                           f"(trajectory_planning.py:491-515), 10% final chunks, seed 7 (workloads.plan_batch_ref)",
               "horizons": {int(n): int(c) for n, c in zip(*np.unique(Nv, return_counts=True))},
               "status_counts_rank0": np.bincount(status, minlength=5).tolist(),
               "status_names": [mpcplan.STATUS_NAMES[i] for i in range(5)],
               "sqp_mean": float(sqp.mean()), "qp_ipm_iters_mean": float(iters.mean()),
               "launches_per_step": len(groups), "streams": len(side),
               "launch_groups": [{"N": [int(a), int(b)], "chunks_per_cu": pl.chunks_per_cu(b)} for a, b in hg],
               "pipelined": {"value": world * Bl * steps / pel, "unit": "chunks/s", "batches": steps,
                             "note": "the same batches back to back without a join between them (a continuously "
                                     "fed planning service); secondary, value is one batch at a time"},
               "roofline": dict(executed_work("plan"), bound="fp64-valu", peak=FP64_PEAK_TFLOPS, unit="TFLOP/s",
                                note="the chunk kernel is latency-bound (one wave per SIMD, sequential Riccati "
                                     "recursions, DESIGN.md 5c); executed FP64 from its PMC pass over N = 16, "
                                     "16384 chunks (tools/gpu/plan_pmc_f64.sh)"),
               "note": "HIP events on the timing stream, which joins the side streams that run one launch per "
                       "residency class of horizons; inputs resident in HBM"}
        if with_cpu:
            out["cpu_backend"] = plan_cpu_backend(r, wb, min(cpu_s, 5.0))
            out["cpu_baseline"], out["parity_sample"] = plan_cpu_baseline(r, wb, cpu_s, status, groups)
            out["cpu_reference"] = plan_cpu_reference(r, wb)
    pl.close()
    return out


def plan_fleet(B, device):
    """B complete plans of trajectory1's route (the reference's chunk loop, :491-548) from random starts along
    it (trajectory_planning.optimize_full_trajectory_batch): the loop on the device (plan_optimize_device, each
    plan on its own wavefront), and for comparison one batched launch per round from the host; wall time
    including the host bookkeeping; the restated checks on every plan."""
    import numpy as np
    import trajectory_planning as TP
    import workloads as W
    r = W.plan_route("traj1")
    rng = np.random.default_rng(11)
    starts = np.zeros((B, 5))
    for b in range(1, B):
        s0 = rng.uniform(1.0, r.s_total - 30.0)
        starts[b] = (s0, rng.normal(0, 0.05), rng.normal(0, 0.01), r.k_ref_fun(s0),
                     rng.uniform(0.2, 0.9) * r.v_max_fun(s0))
    TP.optimize_full_trajectory_batch(r, starts[:4], device=device)          # warm-up (module load, context)
    t0 = time.perf_counter()
    plans, summary = TP.optimize_full_trajectory_batch(r, starts, device=device)
    dt = time.perf_counter() - t0
    tm = TP.optimize_full_trajectory_batch.timing
    t0 = time.perf_counter()
    plans_r, summary_r = TP.optimize_full_trajectory_batch(r, starts, device=device, device_loop=False)
    dt_r = time.perf_counter() - t0
    same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(plans, plans_r))
    chunks = sum(len(q["statuses"]) for q in summary)
    return {"plans": B, "seconds": dt, "plans_per_s": B / dt, "chunks": chunks, "chunks_per_s": chunks / dt,
            "max_chunks_per_plan": max(len(q["statuses"]) for q in summary),
            "checks_passed": int(sum(bool(q["passed"]) for q in summary)),
            "breakdown": {"launches": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in l.items()}
                                       for l in tm.get("launches", [])],
                          "loop_seconds": tm["loop_seconds"], "checks_seconds": tm["seconds"] - tm["loop_seconds"],
                          "note": "launches: plan_optimize calls (upload, kernel, download); "
                                  "checks: plan assembly and the restated checks on every plan"},
            "round_loop": {"seconds": dt_r, "plans_per_s": B / dt_r, "identical_plans": bool(same),
                           "note": "one batched chunk launch per round from the host (device_loop=False): each "
                                   "round waits for its slowest chunk"},
            "route": f"traj1 ({r.s_total:.0f} m), starts uniform along it (the first the reference's)",
            "note": "wall time of the whole receding-horizon loop for every plan, the loop on the device "
                    "(plan_optimize_device: every plan on its own wavefront, no barrier across plans), plans "
                    "assembled on the host"}


def plan_cpu_backend(route, wb, budget_s):
    """libmpcplan's own host backend (plan_create(..., device = -1): csrc/plan_host.h on std::thread workers) on
    the CPU share, on the same bounded sample of chunks as the oracle baseline."""
    import numpy as np
    import mpcplan
    hw, full, threads = cpu_threads()
    B = wb["x0"].shape[0]
    n = min(B, max(256, 16 * threads))
    idx = np.linspace(0, B - 1, n).astype(int)
    old = os.environ.get("PLAN_CPU_THREADS")
    os.environ["PLAN_CPU_THREADS"] = str(threads)          # read by plan_create
    try:
        pl = mpcplan.Planner(route, mpcplan.default_params(N=int(wb["N"].max())), device=-1)
    finally:
        if old is None:
            os.environ.pop("PLAN_CPU_THREADS", None)
        else:
            os.environ["PLAN_CPU_THREADS"] = old
    args = (wb["x0"][idx], wb["s_target"][idx], wb["is_final"][idx], wb["N"][idx])
    done, dt = _timed_rate(lambda: pl.solve_chunks(*args), n, budget_s)
    pl.close()
    return {"value": done / dt, "unit": "chunks/s", "cores": threads,
            "scope": "this process's CPU share of the GPU box (cgroup quota)",
            "sample": f"{n} chunks spread over the batch, solved repeatedly for {dt:.1f} s by libmpcplan's host "
                      f"backend (device = -1), {threads} threads"}


def plan_cpu_baseline(route, wb, budget_s, status, groups):
    """The planner oracle (oracle/plan_oracle.c, the same SQP / QP algorithm) with OpenMP on the host CPUs,
    on a bounded sample of the same chunks; and the GPU's agreement with it on that sample."""
    import numpy as np
    import plan_oracle as PO
    hw, full, threads = cpu_threads()
    po = PO.PlanOracle(route)
    B = wb["x0"].shape[0]
    n = min(B, max(256, 16 * threads))                   # >= 16 chunks per thread
    idx = np.linspace(0, B - 1, n).astype(int)           # spread over the horizons
    p = PO.default_params(N=int(wb["N"].max()))
    args = (wb["x0"][idx], wb["s_target"][idx], wb["is_final"][idx])
    ref = po.solve_batch(p, *args, N=wb["N"][idx], num_threads=threads)
    done, dt = _timed_rate(lambda: po.solve_batch(p, *args, N=wb["N"][idx], num_threads=threads), n, budget_s)
    # GPU vs oracle on the sample: X of chunks both call converged (status 0 / 4)
    dmax, agree, both = 0.0, 0, 0
    for j, i in enumerate(idx):
        for nn, i0, i1, Xg, _, _ in groups:
            if i0 <= i < i1:
                xg = Xg[i - i0].cpu().numpy()
                break
        agree += int(status[i] == ref["status"][j])
        if status[i] in (0, 4) and ref["status"][j] in (0, 4):
            both += 1
            dmax = max(dmax, float(np.abs(xg - ref["X"][j][:nn + 1]).max()))
    base = {"value": done / dt, "unit": "chunks/s", "cores": threads, "kind": "port", "host": hw,
            "scope": "this process's CPU share of the GPU box (cgroup quota)",
            "sample": f"{n} chunks spread over the batch (all horizons), solved repeatedly for {dt:.1f} s by the "
                      f"planner oracle (oracle/plan_oracle.c, the same SQP and QP algorithm) with OpenMP, "
                      f"{threads} threads",
            "whole_box_estimate": {"value": done / dt / threads * (hw["physical_cores_lscpu"] or full),
                                   "cores": hw["physical_cores_lscpu"] or full,
                                   "basis": "share rate per thread x physical cores (an estimate)"}}
    par = {"chunks": n, "status_agreement": agree / n, "both_converged": both, "max_abs_dX_both_converged": dmax}
    return base, par


def plan_cpu_reference(route, wb):
    """The reference's own chunk solve (scipy SLSQP, finite-difference gradients, maxiter 500 / ftol 1e-4,
    trajectory_planning.py:381-387) on the restated NLP functions (oracle/plan_ref.py), one chunk at a time
    per process over a sample of the same chunks (one pass: one chunk per process)."""
    import numpy as np
    from concurrent.futures import ProcessPoolExecutor
    procs = min(16, host_cores()["affinity_cpus"])
    B = wb["x0"].shape[0]
    idx = np.linspace(0, B - 1, min(B, procs)).astype(int)
    jobs = [(route.name, wb["x0"][i], float(wb["s_target"][i]), bool(wb["is_final"][i]), int(wb["N"][i]))
            for i in idx]
    import multiprocessing as mp
    import plan_ref as PR
    # one chunk per process (a chunk takes tens of seconds on this path, so the sample is one pass)
    t0 = time.perf_counter()
    with ProcessPoolExecutor(procs, mp_context=mp.get_context("spawn")) as ex:
        done = sum(ex.map(PR.slsqp_job, jobs))
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "chunks/s", "cores": procs, "kind": "port",
            "sample": f"{done} SLSQP chunk solves (finite-difference gradients, maxiter 500, ftol 1e-4: the "
                      f"reference's minimize call) of {len(idx)} chunks of the same batch in {dt:.1f} s, "
                      f"{procs} processes (oracle/plan_ref.py)"}


def cpu_threads():
    """Thread counts of the CPU legs: 'full' = every physical core of the host (lscpu), bounded by the CPUs this
    process may run on, whatever OMP_NUM_THREADS the environment passes down (all physical host
    cores of the GPU box); 'share' = this GPU's share of the host: the cgroup CPU quota (cpu.max), else
    OMP_NUM_THREADS, else the affinity mask."""
    hw = host_cores()
    aff = hw["affinity_cpus"]
    full = min(hw["physical_cores_lscpu"] or aff, aff)
    q = hw.get("cgroup_cpu_quota")
    share = int(q) if q else (int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff)
    return hw, full, min(max(1, share), aff)


def _timed_rate(fn, n, budget_s):
    fn()                                              # warm
    done, t0, c0 = 0, time.perf_counter(), time.process_time()
    while time.perf_counter() - t0 < budget_s:
        fn()
        done += n
    dt = time.perf_counter() - t0
    _timed_rate.cpu_per_wall = (time.process_time() - c0) / dt
    return done, dt


def cpu_baseline(wb, N, mo, budget_s):
    """The oracle's C restatement (same QP, same PDIP), OpenMP, on the whole per-GPU batch of the same egos,
    solved repeatedly for the budget, at three thread counts: this process's CPU share (the cgroup quota:
    `value`, the best rate the box lets it measure), one thread (the per-core rate), and every physical core
    of the host (on a quota-limited box those threads share the quota, so that run is
    throttled and says so by its CPU-time / wall ratio).  The whole-host rate is then estimated as the per-core
    rate of the share run x the physical cores (the solves are independent and compute-bound), and labelled an
    estimate.  kind = 'port' (the reference itself never travels to the GPU box)."""
    import oracle as O
    import workloads as W
    ld = W.loader(wb["traj"])
    orc = O.Oracle(ld.X_ref, ld.U_ref)
    p = O.default_params(N=N, max_obs=mo)
    hw, full, share = cpu_threads()
    n = wb["x0"].shape[0]
    out = {}
    for tag, threads, budget in (("share", share, budget_s), ("one", 1, budget_s / 4), ("full", full, budget_s / 3)):
        done, dt = _timed_rate(lambda: orc.solve_batch(p, wb["x0"], wb["obs"], wb["n_obs"], num_threads=threads),
                               n, budget)
        out[tag] = {"value": done / dt, "unit": "solves/s", "threads": threads, "seconds": dt,
                    "cpu_time_per_wall": _timed_rate.cpu_per_wall,
                    "sample": f"the whole per-GPU batch ({n} egos), solved {done // n} times in {dt:.1f} s by the "
                              f"oracle's C PDIP (oracle/mpc_oracle.c) with OpenMP, {threads} threads"}
    phys = hw["physical_cores_lscpu"] or full
    est = out["share"]["value"] / share * phys
    return dict(out["share"], cores=share, kind="port", host=hw,
                scope="this process's CPU share of the GPU box (cgroup quota)",
                per_core=out["one"],
                full_host=dict(out["full"], scope="one thread per physical core of the host (lscpu)",
                               note="threads beyond the cgroup quota share it: CPU time / wall stays at the quota"),
                whole_box_estimate={"value": est, "unit": "solves/s", "cores": phys,
                                    "basis": f"share rate / {share} threads x {phys} physical cores (independent, "
                                             "compute-bound solves; an estimate, not a measurement)"})


def cpu_backend(wb, N, mo, budget_s):
    """The product's own host backend (libmpcqp, mpc_create device = -1: csrc/cpu_backend.h) on the whole per-GPU
    batch with this process's CPU share: what a user without a GPU gets (config 1's CPU path)."""
    import mpcqp
    import workloads as W
    ld = W.loader(wb["traj"])
    hw, full, share = cpu_threads()
    n = wb["x0"].shape[0]
    os.environ["MPC_CPU_THREADS"] = str(share)
    slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=mo), device=-1)
    done, dt = _timed_rate(lambda: slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"]), n, budget_s)
    slv.close()
    return {"value": done / dt, "unit": "solves/s", "cores": share,
            "scope": "this process's CPU share of the GPU box (cgroup quota)",
            "sample": f"the whole per-GPU batch ({n} egos), solved {done // n} times in {dt:.1f} s by libmpcqp's host "
                      f"backend (device = -1), {share} threads"}


def host_cores():
    """Host CPUs as the GPU box shows them: physical cores (lscpu, unique core/socket pairs) of the whole
    machine, the CPUs this process may run on (its affinity mask), and the CPU time it may use per second
    (the cgroup quota, cpu.max: 16 CPUs per GPU on the pool's boxes, whatever the affinity mask says)."""
    import subprocess
    phys = None
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        phys = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")})
    except Exception:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    return {"physical_cores_lscpu": phys, "affinity_cpus": aff, "logical_cpus": os.cpu_count(),
            "cgroup_cpu_quota": quota}


def cpu_reference(wb, N, budget_s):
    """The reference's per-step solve path (trajectory_tracking.py:213-263: warm start + scipy SLSQP, ftol
    1e-3, maxiter 15, finite-difference gradients), restated in oracle/slsqp_port.py and run one ego at a
    time per host process on a bounded sample of the same egos.  The restatement evaluates the reference
    signal with numpy interpolation instead of scipy interp1d objects, so it runs faster per core than the
    reference itself (SURVEY 6 measures the reference); it reaches the same iterates (tests/test_slsqp_port)."""
    import slsqp_port as SP
    procs = min(16, host_cores()["affinity_cpus"])
    n = min(256, wb["x0"].shape[0])
    sl = slice(0, n)
    done, dt = SP.time_batch(wb["traj"], N, wb["x0"][sl], None if wb["obs"] is None else wb["obs"][sl],
                             None if wb["n_obs"] is None else wb["n_obs"][sl], budget_s=budget_s, procs=procs)
    return {"value": done / dt, "unit": "solves/s", "cores": procs, "kind": "port",
            "label": "restated SLSQP path with numpy interpolation (faster than the reference's scipy interp1d)",
            "sample": f"{done} solves of the first {n} egos of the same batch in {dt:.1f} s by the restated SLSQP "
                      f"solve path (oracle/slsqp_port.py, pinned to the reference's solve() outputs), "
                      f"{procs} processes"}


if __name__ == "__main__":
    main()
