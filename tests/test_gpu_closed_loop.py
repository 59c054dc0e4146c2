"""Batched closed loop on the device (mpc_closed_loop): run_simulation
(trajectory_tracking.py:377-443) with the ObstaclesFSM (:266-374) for B egos per launch sequence.
The device loop (FSM, solve, Euler plant, histories) must reproduce the host loop of the shim --
which calls the same solver one ego at a time and runs the FSM and plant in numpy -- bit for bit."""
import io
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tt():
    import __graft_entry__ as g
    g.build()
    import trajectory_tracking as TT
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    return TT, TrajectoryLoader, builtin_trajectory


def host_loop(TT, mpc, fsm, traj, x0, max_steps):
    """The shim's run_simulation from an arbitrary start state (same loop body)."""
    x = np.asarray(x0, np.float64)
    hx, hu, ho, ht = [x], [], [], []
    step = 0
    while x[0] <= traj.s_max - 1.0 and step < max_steps:
        obstacles, tl = fsm.update(mpc.dt, x[0], x[4])
        u, _, _ = mpc.solve(x, obstacles)
        k_ref = traj.get_state(x[0])[3]
        x = x + mpc.dt * mpc.dynamics(x, u, k_ref)
        hx.append(x)
        hu.append(u)
        car = [o["s"] for o in obstacles if o["type"] == "car"]
        ho.append(car[0] if car else np.nan)
        ht.append(1 if tl == "GREEN" else 0)
        step += 1
    return np.array(hx), np.array(hu), np.array(ho), np.array(ht)


def compare(r, b, host):
    hx, hu, ho, ht = host
    n = int(r["n_steps"][b])
    assert n == len(hu)
    assert np.array_equal(r["hist_x"][b, :n + 1], hx)
    assert np.array_equal(r["hist_u"][b, :n], hu)
    assert np.array_equal(np.isnan(r["hist_obs_s"][b, :n]), np.isnan(ho))
    assert np.array_equal(r["hist_obs_s"][b, :n][~np.isnan(ho)], ho[~np.isnan(ho)])
    assert np.array_equal(r["hist_tl"][b, :n], ht)
    assert np.isnan(r["hist_x"][b, n + 1:]).all() and (r["hist_tl"][b, n:] == -1).all()


def test_config1_device_loop_matches_host_loop(tt):
    """Config 1: traj1, N=10, no obstacles, the reference start state; plus two perturbed starts."""
    TT, TL, bt = tt
    traj = TL(bt(1))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 10
    x_init = np.array([[0.0, 0.0, 0.0, 0.0, 0.5], [1.0, 0.05, 0.0, 0.0, 1.5], [0.5, -0.05, 0.01, 0.0, 1.0]])
    r = TT.run_simulation_batch(mpc, TT.ObstaclesFSM(), traj, x_init=x_init, max_steps=600, checks=True)
    for b in range(3):
        compare(r, b, host_loop(TT, mpc, TT.ObstaclesFSM(), traj, x_init[b], 600))
    assert r["checks_passed"][0]          # the restated trajectory_tracking_check on the device loop
    assert ((r["hist_status"][0, :int(r["n_steps"][0])] & 15) == 0).all()


def test_fsm_device_loop_matches_host_loop(tt):
    """Traj2 with the ObstaclesFSM (car + traffic light), N=10, from two starts near the light trigger
    and the car trigger, so both state machines switch within the run."""
    TT, TL, bt = tt
    traj = TL(bt(2))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 10
    x_init = np.array([[440.0, 0.0, 0.0, traj.get_state(440.0)[3], 9.0],
                       [690.0, 0.02, 0.0, traj.get_state(690.0)[3], 8.0]])
    mk = lambda: TT.ObstaclesFSM(dynamic_obstacle=True, traffic_light=True)
    r = TT.run_simulation_batch(mpc, mk(), traj, x_init=x_init, max_steps=400)
    for b in range(2):
        compare(r, b, host_loop(TT, mpc, mk(), traj, x_init[b], 400))
    # the light turned GREEN for the ego that started before it, the car appeared for the other
    assert r["hist_tl"][0, :int(r["n_steps"][0])].max() == 1
    assert np.isfinite(r["hist_obs_s"][1]).any()


def test_batch_equals_single_runs(tt):
    """Egos are independent: a batch of 5 (two lane groups per wavefront) equals each ego alone."""
    TT, TL, bt = tt
    traj = TL(bt(1))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 20
    rng = np.random.default_rng(5)
    x_init = np.column_stack([rng.uniform(0, 20, 5), rng.normal(0, 0.05, 5), np.zeros(5), np.zeros(5),
                              rng.uniform(0.5, 3, 5)])
    r = TT.run_simulation_batch(mpc, None, traj, x_init=x_init, max_steps=80)
    for b in range(5):
        r1 = TT.run_simulation_batch(mpc, None, traj, x_init=x_init[b:b + 1], max_steps=80)
        n = int(r1["n_steps"][0])
        assert n == int(r["n_steps"][b])
        assert np.array_equal(r1["hist_x"][0, :n + 1], r["hist_x"][b, :n + 1])
    assert np.isfinite(r["step_ms"][:int(r["n_steps"].max())]).all()


def test_egos_leaving_at_different_steps(tt):
    """Egos that leave the loop early stop costing solver work (the solver's ego list is compacted at the
    host syncs): a batch whose egos finish at very different steps still equals each ego run alone, and the
    host loop, bit for bit."""
    TT, TL, bt = tt
    traj = TL(bt(1))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 10
    starts = [0.0, 120.0, 250.0, 297.0, 60.0, 280.0, 10.0]
    x_init = np.array([[s, 0.02, 0.0, traj.get_state(s)[3], 3.0] for s in starts])
    r = TT.run_simulation_batch(mpc, TT.ObstaclesFSM(), traj, x_init=x_init, max_steps=400)
    ns = r["n_steps"]
    assert len(set(ns.tolist())) >= 5 and ns.min() < 20 and ns.max() > 100
    for b in range(len(starts)):
        r1 = TT.run_simulation_batch(mpc, TT.ObstaclesFSM(), traj, x_init=x_init[b:b + 1], max_steps=400)
        n = int(r1["n_steps"][0])
        assert n == int(ns[b])
        assert np.array_equal(r1["hist_x"][0, :n + 1], r["hist_x"][b, :n + 1])
        assert np.array_equal(r1["hist_u"][0, :n], r["hist_u"][b, :n])
    compare(r, 3, host_loop(TT, mpc, TT.ObstaclesFSM(), traj, x_init[3], 400))
