"""GPU tests of the device-pointer entry mpc_solve_batch_device (the path bench.py times) and of the
launch schedule: the two-phase launch (crossover kernel + interior-point kernel on a device work
list) must give bit-identical results to the single-kernel launch (MPC_TWO_PHASE=0), through the
host entry and the device entry, with and without obstacles.  Also the argument contract the two
entries share (include/mpcqp.h): n_obs NULL = every max_obs row is used; obstacles with
max_obs == 0 are refused instead of being dropped."""
import os

import numpy as np
import pytest

from conftest import traj_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    import mpcqp
    return mpcqp


def make_solver(lib, traj, N, mo, two_phase=True):
    old = os.environ.get("MPC_TWO_PHASE")
    os.environ["MPC_TWO_PHASE"] = "1" if two_phase else "0"
    try:
        return lib.Solver(*traj_arrays(traj), lib.default_params(N=N, max_obs=mo), device=0)
    finally:
        if old is None:
            del os.environ["MPC_TWO_PHASE"]
        else:
            os.environ["MPC_TWO_PHASE"] = old


def device_solve(slv, wb, torch, stream=None, pass_nobs=True):
    """One mpc_solve_batch_device call on torch device buffers; returns host copies of the outputs."""
    dev = torch.device("cuda", 0)
    B, N = wb["x0"].shape[0], wb["N"]
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0 = t(wb["x0"])
    obs = t(wb["obs"]) if wb["obs"] is not None else None
    nob = t(wb["n_obs"], torch.int32) if (wb["n_obs"] is not None and pass_nobs) else None
    out = dict(u0=torch.empty((B, 2), dtype=torch.float64, device=dev),
               U=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
               Xpred=torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev),
               status=torch.empty(B, dtype=torch.int32, device=dev),
               iters=torch.empty(B, dtype=torch.int32, device=dev))
    ptr = lambda x: 0 if x is None else x.data_ptr()
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))      # the input copies ran on the current stream
    slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(out["u0"]), ptr(out["U"]), ptr(out["Xpred"]),
                           ptr(out["status"]), ptr(out["iters"]), stream=st.cuda_stream)
    return out, (x0, obs, nob)


def to_host(out, torch):
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def assert_identical(a, b, what):
    for k in ("u0", "U", "Xpred", "status", "iters"):
        assert np.array_equal(a[k], b[k]), (what, k, np.flatnonzero((a[k] != b[k]).reshape(len(a[k]), -1).any(1))[:8])


@pytest.mark.parametrize("cfg,B,N", [("C2", 1024, None), ("C3", 1024, None), ("C4", 1024, None), ("C2", 1024, 10)])
def test_two_phase_equals_single_kernel(lib, cfg, B, N):
    """Split launch (MODE_XO + MODE_IPM) == single launch (MODE_FULL), host and device entries.  Covers the
    N = 20 kernels (C2, C3), the runtime-horizon GL = 32 kernels (C4, N = 30) and GL = 16 (N = 10, four
    instances per wavefront); the crossover solves in K-row form in both launch paths."""
    torch = pytest.importorskip("torch")
    import workloads as W
    wb = W.make_batch(cfg, B=B, seed=7)
    if N is not None:
        wb["N"] = N
    two = make_solver(lib, wb["traj"], wb["N"], wb["max_obs"], two_phase=True)
    one = make_solver(lib, wb["traj"], wb["N"], wb["max_obs"], two_phase=False)
    r2 = two.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    r1 = one.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    assert_identical(r2, r1, "host entry")
    # the batch exercises both kernels of the split launch
    assert (r2["iters"] == 0).any() and (r2["iters"] > 0).any()
    d2, _ = device_solve(two, wb, torch)
    d1, _ = device_solve(one, wb, torch)
    d2, d1 = to_host(d2, torch), to_host(d1, torch)
    assert_identical(d2, d1, "device entry")
    assert_identical(d2, r2, "device vs host entry")


def test_device_entry_nobs_null_uses_all_rows(lib):
    """Device entry with obs and n_obs == NULL == host entry with n_obs = max_obs for every instance."""
    torch = pytest.importorskip("torch")
    import workloads as W
    wb = W.make_batch("C5", B=64, seed=11)
    assert wb["max_obs"] == 8 and (wb["n_obs"] == 8).all()
    slv = make_solver(lib, wb["traj"], wb["N"], wb["max_obs"])
    rh = slv.solve_batch(wb["x0"], wb["obs"], np.full(64, 8, np.int32))
    rd, _ = device_solve(slv, wb, torch, pass_nobs=False)
    rd = to_host(rd, torch)
    assert_identical(rd, rh, "n_obs NULL")
    # and the obstacles really are used: without them the answers differ
    r0 = slv.solve_batch(wb["x0"])
    assert not np.array_equal(r0["U"], rh["U"])


def test_device_calls_on_two_streams_are_ordered(lib):
    """Back-to-back device calls on one context from two streams share the context's work list; the
    second call must wait for the first (include/mpcqp.h), so both equal their host-entry results."""
    torch = pytest.importorskip("torch")
    import workloads as W
    wa = W.make_batch("C3", B=2048, seed=21)
    wb = W.make_batch("C3", B=2048, seed=22)
    slv = make_solver(lib, wa["traj"], wa["N"], wa["max_obs"])
    ra = slv.solve_batch(wa["x0"], wa["obs"], wa["n_obs"])
    rb = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(3):
        oa, keep_a = device_solve(slv, wa, torch, stream=s1)
        ob, keep_b = device_solve(slv, wb, torch, stream=s2)
        ha, hb = to_host(oa, torch), to_host(ob, torch)
        assert_identical(ha, ra, "stream 1")
        assert_identical(hb, rb, "stream 2")


def test_obstacles_with_max_obs_zero_are_refused(lib):
    """Obstacles passed while params.max_obs == 0 are an error (Python ValueError, C MPC_E_ARG), never
    an unconstrained solve."""
    torch = pytest.importorskip("torch")
    import workloads as W
    wb = W.make_batch("C3", B=8, seed=3)
    slv = make_solver(lib, wb["traj"], wb["N"], 0)
    with pytest.raises(ValueError):
        slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    with pytest.raises(lib.MpcError):
        device_solve(slv, wb, torch)
    # the host C entry refuses it too
    B = 8
    x0 = np.ascontiguousarray(wb["x0"])
    obs = np.ascontiguousarray(wb["obs"])
    rc = lib.lib().mpc_solve_batch(slv.h, B, lib._p(x0), lib._p(obs), None, None, None, None, None, None, None)
    assert rc == -1 and "max_obs" in lib.last_error()


def test_graph_capture_on_side_stream_after_eager_warmup(lib):
    """Eager warm-up call on the current stream, then the same call captured into a HIP graph on a side
    stream (torch.cuda.graph's pattern) and replayed: the capture must succeed (no wait on an event
    recorded outside it) and every replay must equal the eager result, including after new inputs are
    copied into the captured buffers."""
    torch = pytest.importorskip("torch")
    import workloads as W
    wa = W.make_batch("C3", B=2048, seed=31)
    wb = W.make_batch("C3", B=2048, seed=32)
    slv = make_solver(lib, wa["traj"], wa["N"], wa["max_obs"])
    ra = slv.solve_batch(wa["x0"], wa["obs"], wa["n_obs"])
    rb = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    out, keep = device_solve(slv, wa, torch)                  # eager warm-up (records the ordering event)
    assert_identical(to_host(out, torch), ra, "eager")
    x0, obs, nob = keep
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    ptr = lambda x: 0 if x is None else x.data_ptr()
    with torch.cuda.graph(g, stream=side):
        slv.solve_batch_device(2048, ptr(x0), ptr(obs), ptr(nob), 0, ptr(out["u0"]), ptr(out["U"]),
                               ptr(out["Xpred"]), ptr(out["status"]), ptr(out["iters"]),
                               stream=torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        for k in out:
            out[k].zero_()
        g.replay()
        assert_identical(to_host(out, torch), ra, "replay")
    x0.copy_(torch.as_tensor(wb["x0"]))
    obs.copy_(torch.as_tensor(wb["obs"]))
    nob.copy_(torch.as_tensor(wb["n_obs"]))
    g.replay()
    assert_identical(to_host(out, torch), rb, "replay on new inputs")
    # an eager call after the replays (same stream) still orders correctly
    o2, _ = device_solve(slv, wa, torch)
    assert_identical(to_host(o2, torch), ra, "eager after graph")


def test_device_entry_unaligned_outputs(lib):
    """u0 and U that are 8-byte but not 16-byte aligned (tensor views at an odd element offset) take the
    kernel's 8-byte store path and give the aligned call's results bit for bit."""
    import torch
    import workloads as W
    wb = W.make_batch("C2", B=512)
    slv = make_solver(lib, wb["traj"], wb["N"], 0)
    out, _ = device_solve(slv, wb, torch)
    ref = to_host(out, torch)
    dev = torch.device("cuda", 0)
    B, N = 512, wb["N"]
    x0 = torch.as_tensor(wb["x0"], dtype=torch.float64, device=dev).contiguous()
    u0b = torch.empty(2 * B + 1, dtype=torch.float64, device=dev)
    Ub = torch.empty(2 * B * N + 1, dtype=torch.float64, device=dev)
    u0, U = u0b[1:], Ub[1:]
    assert u0.data_ptr() % 16 == 8 and U.data_ptr() % 16 == 8
    X = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    slv.solve_batch_device(B, x0.data_ptr(), 0, 0, 0, u0.data_ptr(), U.data_ptr(), X.data_ptr(), st.data_ptr(),
                           it.data_ptr(), stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(U.cpu().numpy().reshape(B, N, 2), ref["U"])
    assert np.array_equal(u0.cpu().numpy().reshape(B, 2), ref["u0"])
    assert np.array_equal(X.cpu().numpy(), ref["Xpred"]) and np.array_equal(st.cpu().numpy(), ref["status"])


def test_stage_cache_capture_then_grow(lib):
    """with MPC_STAGE_CACHE=1, a graph captured at B = 1024, then an eager call at B = 4096 that
    grows (frees and reallocates) the context's stage cache, then replays of the graph: the captured call
    never used the cache, so the replays stay correct."""
    torch = pytest.importorskip("torch")
    import workloads as W
    old = os.environ.get("MPC_STAGE_CACHE")
    os.environ["MPC_STAGE_CACHE"] = "1"
    try:
        wa = W.make_batch("C2", B=1024, seed=41)
        slv = make_solver(lib, wa["traj"], wa["N"], 0)
    finally:
        if old is None:
            del os.environ["MPC_STAGE_CACHE"]
        else:
            os.environ["MPC_STAGE_CACHE"] = old
    ra = slv.solve_batch(wa["x0"])
    out, keep = device_solve(slv, wa, torch)                     # eager warm-up at B = 1024
    assert_identical(to_host(out, torch), ra, "eager")
    x0 = keep[0]
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        slv.solve_batch_device(1024, x0.data_ptr(), 0, 0, 0, out["u0"].data_ptr(), out["U"].data_ptr(),
                               out["Xpred"].data_ptr(), out["status"].data_ptr(), out["iters"].data_ptr(),
                               stream=torch.cuda.current_stream().cuda_stream)
    wbig = W.make_batch("C2", B=4096, seed=42)
    rbig = slv.solve_batch(wbig["x0"])
    obig, _ = device_solve(slv, wbig, torch)                     # grows the stage cache
    assert_identical(to_host(obig, torch), rbig, "eager after growth")
    for _ in range(2):
        for k in out:
            out[k].zero_()
        g.replay()
        assert_identical(to_host(out, torch), ra, "replay after growth")
