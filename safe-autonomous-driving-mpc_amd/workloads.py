"""Synthetic ego batches for the BASELINE.json configurations.

Generator: numpy default_rng(seed) (PCG64).  Per ego (single-step microbench):
  s0 ~ U(0, 0.8 s_max); d0 = d_ref(s0) + N(0, 0.05); o0 = o_ref(s0) + N(0, 0.01);
  k0 = k_ref(s0); v0 = max(0.5, v_ref(s0) + N(0, 0.5)).
Obstacle slabs:
  'fsm2' / 'fsm3'  snapshot of an ObstaclesFSM with the geometry of its preset (trajectory_tracking.py:
                   292-308 for trajectory2, :311-327 for trajectory3): the dynamic car (v = 4 m/s) exists
                   only once the ego has passed obs_trigger_s and until the car passes obs_end_s (:339-350);
                   it drives ahead of the ego (the ego cannot overtake it), at max(obs_start_s, s0 + U(8, 70));
                   the RED light at tl_pos when 0 < tl_pos - s0 < tl_trigger_s (:357-361).  max_obs = 2.
  'const8'         8 constant-velocity cars: s_i = s0 + 25 + 50 i + U(0, 10), v_i ~ U(2, 10).
"""
import numpy as np

from trajectory_loader import TrajectoryLoader, builtin_trajectory

CONFIGS = {
    # name: (trajectory, horizon N, batch B, seed, obstacle kind, GPUs in BASELINE.json)
    "C1": dict(traj=1, N=10, B=1, seed=1, obstacles=None, gpus=0),
    "C2": dict(traj=1, N=20, B=4096, seed=2, obstacles=None, gpus=1),
    "C3": dict(traj=2, N=20, B=8192, seed=3, obstacles="fsm2", gpus=1),
    "C4": dict(traj=3, N=30, B=16384, seed=4, obstacles="fsm3", gpus=4),
    "C5": dict(traj=3, N=40, B=65536, seed=5, obstacles="const8", gpus=8),
}

_FSM = {"fsm2": dict(obs_trigger_s=710.0, obs_start_s=780.0, obs_end_s=1050.0, tl_pos=550.0, tl_trigger_s=100.0),
        "fsm3": dict(obs_trigger_s=5.0, obs_start_s=150.0, obs_end_s=850.0, tl_pos=2000.0, tl_trigger_s=100.0)}

_LOADERS = {}


def loader(i):
    if i not in _LOADERS:
        _LOADERS[i] = TrajectoryLoader(builtin_trajectory(i))
    return _LOADERS[i]


def make_batch(name, B=None, seed=None, offset=0):
    """Return dict(traj, N, x0 [B,5], obs [B,M,2] | None, n_obs [B] | None, max_obs).
    `offset` skips the first `offset` egos of the same stream (for sharding across ranks)."""
    cfg = CONFIGS[name]
    B = cfg["B"] if B is None else int(B)
    seed = cfg["seed"] if seed is None else seed
    ld = loader(cfg["traj"])
    # one PCG64 stream per field (SeedSequence children), so that the egos [offset, offset+B) of a
    # shard are exactly that slice of the single-process batch
    rs = [np.random.default_rng(c) for c in np.random.SeedSequence(seed).spawn(8)]
    tot = offset + B
    s0 = rs[0].uniform(0.0, 0.8 * ld.s_max, tot)
    nd = rs[1].normal(0, 0.05, tot)
    no = rs[2].normal(0, 0.01, tot)
    nv = rs[3].normal(0, 0.5, tot)
    x0 = np.empty((B, 5))
    for b in range(B):
        i = offset + b
        r = ld.get_state(s0[i])
        x0[b] = (s0[i], r[1] + nd[i], r[2] + no[i], r[3], max(0.5, r[4] + nv[i]))
    kind = cfg["obstacles"]
    obs = n_obs = None
    max_obs = 0
    if kind in _FSM:
        max_obs = 2
        pd = rs[5].uniform(8.0, 70.0, tot)
        obs = np.zeros((B, 2, 2))
        n_obs = np.zeros(B, np.int32)
        f = _FSM[kind]
        for b in range(B):
            i = offset + b
            n = 0
            car = max(f["obs_start_s"], x0[b, 0] + pd[i])
            if x0[b, 0] >= f["obs_trigger_s"] and car <= f["obs_end_s"]:
                obs[b, n] = (car, 4.0)
                n += 1
            if 0.0 < f["tl_pos"] - x0[b, 0] < f["tl_trigger_s"]:
                obs[b, n] = (f["tl_pos"], 0.0)
                n += 1
            n_obs[b] = n
    elif kind == "const8":
        max_obs = 8
        u = rs[6].uniform(0, 10, (tot, 8))
        v = rs[7].uniform(2, 10, (tot, 8))
        obs = np.zeros((B, 8, 2))
        for b in range(B):
            i = offset + b
            obs[b, :, 0] = x0[b, 0] + 25.0 + 50.0 * np.arange(8) + u[i]
            obs[b, :, 1] = v[i]
        n_obs = np.full(B, 8, np.int32)
    return dict(traj=cfg["traj"], N=cfg["N"], x0=x0, obs=obs, n_obs=n_obs, max_obs=max_obs)


# ---------------------------------------------------------------------------------------------
# offline planner chunks: batches of independent chunk NLPs on one route
# ---------------------------------------------------------------------------------------------
_ROUTES = {}


def plan_route(name="traj1"):
    """The planner's synthetic routes (routes.py): 'traj1'..'traj3' = the global line of the committed
    trajectory (way-points >= 8 m apart, densified to <= 5 m as path_planning does) with 50 km/h on the first
    half and 30 km/h after; 'synth<seed>' = routes.synthetic(seed=<seed>) (1.5 km, 30/40/50 km/h bands)."""
    if name not in _ROUTES:
        import routes
        if name.startswith("traj"):
            X = loader(int(name[4:])).X_ref
            _ROUTES[name] = routes.from_trajectory(X, bands=((0.0, 50.0), (0.5, 30.0)), min_gap=8.0, name=name)
        elif name.startswith("synth"):
            _ROUTES[name] = routes.synthetic(seed=int(name[5:]), name=name)
        else:
            raise KeyError(name)
    return _ROUTES[name]


def plan_batch(route, N, B, seed=0, final_frac=0.0, offset=0):
    """B chunks at horizon N on `route`, sized by the reference's own rule (optimize_full_trajectory,
    trajectory_planning.py:493-515: N = ceil(2 D / avg_speed / 0.3)), i.e. chunk distance D = N 0.3 avg / 2
    with avg_speed the mean remaining speed limit.  Per chunk (default_rng(seed), one stream per field so a
    shard is a slice): s0 ~ U(1, s_total - D - 1) (final chunks: s_target = s_total, s0 = s_total - D);
    d0 ~ N(0, 0.05), o0 ~ N(0, 0.01), k0 = kappa(s0), v0 ~ U(0.2, 0.9) v_max(s0) (final chunks: v0 small
    enough to stop in D at 2.5 m/s^2).  Returns dict(x0 [B,5], s_target [B], is_final [B] int32, N)."""
    rs = [np.random.default_rng(c) for c in np.random.SeedSequence(seed).spawn(6)]
    tot = offset + B
    u0, nd, no, uv, uf = (rs[0].uniform(0, 1, tot), rs[1].normal(0, 0.05, tot), rs[2].normal(0, 0.01, tot),
                          rs[3].uniform(0.2, 0.9, tot), rs[4].uniform(0, 1, tot))
    x0 = np.empty((B, 5))
    st = np.empty(B)
    fin = np.zeros(B, np.int32)
    for b in range(B):
        i = offset + b
        final = uf[i] < final_frac
        s_guess = 1.0 + u0[i] * (route.s_total - 2.0)
        D = N * 0.3 * route.avg_speed_from(s_guess) / 2.0
        if final:
            s0 = max(1.0, route.s_total - D)
            target = route.s_total
            vmax = min(route.v_max_fun(s0), np.sqrt(2.0 * 2.5 * (route.s_total - s0)))
        else:
            s0 = 1.0 + u0[i] * max(1e-3, route.s_total - D - 2.0)
            target = s0 + D
            vmax = route.v_max_fun(s0)
        x0[b] = (s0, nd[i], no[i], route.k_ref_fun(s0), uv[i] * vmax)
        st[b] = target
        fin[b] = int(final)
    return dict(x0=x0, s_target=st, is_final=fin, N=int(N))


def plan_batch_ref(route, B, seed=0, chunk=20.0, final_frac=0.1, offset=0):
    """B chunks on `route` as optimize_full_trajectory (trajectory_planning.py:491-515) poses them with its
    default max_chunk_size = 20 m: an intermediate chunk spans D = chunk metres from s0, the final one the
    remaining D ~ U(1.5, 2) chunk to the destination (the loop's last chunk, remaining < 2 chunk), and each
    gets its own horizon N = ceil(2 D / avg_speed(s0) / 0.3).  Start states as plan_batch.  Vectorised over
    the batch (the route functions evaluated on arrays, avg_speed once per 5 m cell).  Returns dict(x0
    [B,5], s_target [B], is_final [B] int32, N [B] int32), sorted by N (one launch per horizon)."""
    rs = [np.random.default_rng(c) for c in np.random.SeedSequence(seed).spawn(7)]
    sl = slice(offset, offset + B)
    tot = offset + B
    u0, nd, no, uv, uf, ud = (rs[0].uniform(0, 1, tot)[sl], rs[1].normal(0, 0.05, tot)[sl],
                              rs[2].normal(0, 0.01, tot)[sl], rs[3].uniform(0.2, 0.9, tot)[sl],
                              rs[4].uniform(0, 1, tot)[sl], rs[5].uniform(1.5, 2.0, tot)[sl])
    fin = (uf < final_frac).astype(np.int32)
    Df = np.minimum(ud * chunk, route.s_total - 1.0)
    s0 = np.where(fin == 1, route.s_total - Df, 1.0 + u0 * (route.s_total - 2.0 * chunk - 2.0))
    D = np.where(fin == 1, Df, chunk)
    vm = np.asarray(route._vint(s0), np.float64)
    vmax = np.where(fin == 1, np.minimum(vm, np.sqrt(2.0 * 2.5 * D)), vm)
    t = np.asarray(route._s_to_t(s0), np.float64)
    xs, ys = route.spline
    x1, y1, x2, y2 = xs(t, 1), ys(t, 1), xs(t, 2), ys(t, 2)
    den = (x1 ** 2 + y1 ** 2) ** 1.5 + 1e-9
    den = np.where(den < 1e-8, 1e-8, den)
    k0 = (x1 * y2 - y1 * x2) / den
    cells = (s0 / 5).astype(int)
    avg = {c: route.avg_speed_from(5.0 * c) for c in np.unique(cells)}
    av = np.array([avg[c] for c in cells])
    Nv = np.ceil(D / av * 2.0 / 0.3).astype(np.int32)
    x0 = np.stack([s0, nd, no, k0, uv * vmax], axis=1)
    st = np.where(fin == 1, route.s_total, s0 + D)
    o = np.argsort(Nv, kind="stable")
    return dict(x0=x0[o], s_target=st[o], is_final=fin[o], N=Nv[o])
