"""A/B timing of in-tree builds of libmpcqp (same ABI), one subprocess per variant.

  python tools/ab_probe.py libmpcqp.so libmpcqp_x.so ... [--configs C2,C3] [--reps 10]

For each config: the batch time of the device entry (HIP events, mean of `reps` launches after
2 warm-ups) per variant, and every variant's outputs compared with the first variant's
(max |dU|, status and iteration-count agreement).  Writes gpurun_out/ab_<cfg>.json."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")


def child(lib, cfg, reps, out):
    sys.path[:0] = [ROOT, PKG]
    import numpy as np
    import torch
    import mpcqp
    mpcqp.LIB_PATH = os.path.join(PKG, lib)
    import workloads as W
    wb = W.make_batch(cfg)
    B, N, mo = wb["x0"].shape[0], wb["N"], wb["max_obs"]
    if cfg in ("C4", "C5"):
        B = B // (4 if cfg == "C4" else 8)
        for k in ("x0", "obs", "n_obs"):
            if wb[k] is not None:
                wb[k] = wb[k][:B]
    ld = W.loader(wb["traj"])
    extra = {"sqp_iters": int(os.environ["AB_SQP"])} if os.environ.get("AB_SQP") else {}   # e.g. 30: the SQP leg
    slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=mo, **extra))
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0 = t(wb["x0"])
    obs = t(wb["obs"]) if wb["obs"] is not None else None
    nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    Uo = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    Xo = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    ptr = lambda x: 0 if x is None else x.data_ptr()
    stream = torch.cuda.current_stream(dev)
    args = (B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(u0), ptr(Uo), ptr(Xo), ptr(st), ptr(it), stream.cuda_stream)
    for _ in range(2):
        slv.solve_batch_device(*args)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        slv.solve_batch_device(*args)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    np.savez(out, U=Uo.cpu().numpy(), status=st.cpu().numpy(), iters=it.cpu().numpy(), ms=np.array(ms))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    if args and args[0] == "__child__":
        child(args[1], args[2], int(args[3]), args[4])
        return
    import numpy as np
    libs = args or ["libmpcqp.so"]
    configs = opts.get("configs", "C2,C3,C4,C5").split(",")
    reps = int(opts.get("reps", "10"))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for cfg in configs:
        rows = []
        base = None
        for lib in libs:
            out = os.path.join(ROOT, "gpurun_out", f"ab_{cfg}_{lib}.npz")
            r = subprocess.run([sys.executable, __file__, "__child__", lib, cfg, str(reps), out], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                print(f"{cfg} {lib}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
                sys.exit(1)
            z = dict(np.load(out))
            ms = float(np.median(z["ms"]))
            row = dict(lib=lib, ms=round(ms, 4), mean_iters=float(z["iters"].mean()), max_iters=int(z["iters"].max()))
            if base is None:
                base = z
            else:
                ok = np.isin(z["status"], (0, 2)) & np.isin(base["status"], (0, 2))
                row["max_dU"] = float(np.abs(z["U"] - base["U"]).reshape(len(ok), -1).max(1)[ok].max(initial=0))
                row["status_agree"] = float((z["status"] == base["status"]).mean())
                row["iters_agree"] = float((z["iters"] == base["iters"]).mean())
            rows.append(row)
            print(cfg, json.dumps(row), flush=True)
        json.dump(rows, open(os.path.join(ROOT, "gpurun_out", f"ab_{cfg}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
