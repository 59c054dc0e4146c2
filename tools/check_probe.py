"""Oracle A/B of the tracker's interior-point checkpoint: per config, the per-GPU batch
solved by oracle/mpc_oracle.c with and without the checkpoint (ORC_CHECK_MU / ORC_CHECK_SEP / ORC_CHECK_ROUNDS
in the environment of a child process, so each setting gets a fresh library).  Prints mean / max interior-point
iterations, statuses and the largest |dU| against the plain run.

  python tools/check_probe.py C2 [mu sep rounds] ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(cfg, env, out):
    code = f"""
import sys, numpy as np
sys.path[:0] = [{ROOT!r} + '/safe-autonomous-driving-mpc_amd', {ROOT!r} + '/oracle']
import oracle as O, workloads as W
wb = W.make_batch({cfg!r})
ld = W.loader(wb['traj'])
orc = O.Oracle(ld.X_ref, ld.U_ref)
r = orc.solve_batch(O.default_params(N=wb['N'], max_obs=wb['max_obs']), wb['x0'], wb['obs'], wb['n_obs'], num_threads=8)
np.savez({out!r}, U=r['U'], st=r['status'], it=r['iters'])
"""
    subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), check=True)


def main():
    cfg = sys.argv[1]
    sets = [tuple(a.split(",")) for a in sys.argv[2:]] or [("1e-4", "100", "2")]
    import numpy as np
    base = f"/tmp/chk_{cfg}_base.npz"
    run(cfg, {}, base)
    b = np.load(base)
    order = np.sort(b["it"])[::-1]
    print(f"{cfg} base: iters mean {b['it'].mean():.3f} max {b['it'].max()} top {order[:6].tolist()} "
          f"status {np.bincount(b['st'] & 15, minlength=4).tolist()}")
    for mu, sep, rounds in sets:
        out = f"/tmp/chk_{cfg}_{mu}_{sep}_{rounds}.npz"
        env = {"ORC_CHECK_MU": mu, "ORC_CHECK_SEP": sep, "ORC_CHECK_ROUNDS": rounds, "ORC_CHECK_FAILCOUNT": "1"}
        if sep == "0":
            env["ORC_CHECK_NOTIE"] = "1"
        run(cfg, env, out)
        c = dict(np.load(out))
        fails = c["it"] // 1000
        c["it"] = c["it"] % 1000
        # cost in iteration equivalents: a failed checkpoint polish ~ one iteration
        cost = c["it"] + fails
        print(f"   failed attempts {int(fails.sum())}, worst cost (iters + failed attempts) {cost.max()} "
              f"top {np.sort(cost)[::-1][:6].tolist()}")
        d = np.abs(c["U"] - b["U"]).reshape(len(b["it"]), -1).max(axis=1)
        order = np.sort(c["it"])[::-1]
        print(f"{cfg} mu<={mu} sep {sep} rounds {rounds}: iters mean {c['it'].mean():.3f} max {c['it'].max()} "
              f"top {order[:6].tolist()} status {np.bincount(c['st'] & 15, minlength=4).tolist()} "
              f"status changed {int((c['st'] != b['st']).sum())} max|dU| {d.max():.2e} (>1e-9: {int((d > 1e-9).sum())})")


if __name__ == "__main__":
    main()
