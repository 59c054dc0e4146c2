"""Sanitizer runs of the host-only code ("an ASan/UBSan build of the CPU C++ path in tests").

tests/asan/Makefile builds, with -fsanitize=address,undefined (every report fatal):
  json_driver    csrc/host_table.h -- the native trajectory JSON reader (replaces the json.load of
                 trajectory_loader.py:13-24), the device-table build (:26-84) and the bucketed interval
                 search restated from the device's seg_t;
  oracle_driver  oracle/mpc_oracle.c -- the CPU restatement;
  cpu_driver     csrc/cpu_backend.h -- the product's host backend (mpc_create device = -1), on 3 threads;
  plan_driver    csrc/plan_host.h -- libmpcplan's host backend (plan_create device = -1): a chunk batch and the
                 receding-horizon loop, on 3 threads; equal bit for bit to the library's own host backend.
The reader runs over the reference trajectories (regenerated from the package data, verbatim floats) and a
malformed / duplicate-key / deeply nested corpus; every answer must match Python's json.load (the
reference's loader).  Both solver drivers' results must equal the regular oracle build's bit for bit.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, traj_arrays

ASAN = os.path.join(ROOT, "tests", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def drivers():
    # one build at a time: pytest-xdist workers share the tree, and a worker must not run a driver
    # while another one relinks it
    from filelock import FileLock
    with FileLock(os.path.join(ASAN, ".build.lock")):
        r = subprocess.run(["make", "-C", ASAN], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return (os.path.join(ASAN, "json_driver"), os.path.join(ASAN, "oracle_driver"), os.path.join(ASAN, "cpu_driver"),
            os.path.join(ASAN, "plan_driver"))


def traj_json(i):
    X, U = traj_arrays(i)
    return json.dumps({"X": X.tolist(), "U": U.tolist(), "S": list(range(len(U)))})


def run_json(drv, files):
    r = subprocess.run([drv] + [str(f) for f in files], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return r.stdout.splitlines()


def expect_line(text):
    """What json.load makes of the text, in the driver's output format (status only for errors)."""
    try:
        d = json.loads(text)
        X = np.asarray(d["X"], np.float64).reshape(-1, 5)
        U = np.asarray(d["U"], np.float64).reshape(-1, 2)
    except Exception:
        return "ERR"
    return ("OK", X.shape[0], U.shape[0], X, U)


def test_json_reader_reference_trajectories(drivers, tmp_path):
    files = []
    for i in (1, 2, 3):
        f = tmp_path / f"trajectory{i}.json"
        f.write_text(traj_json(i))
        files.append(f)
    out = run_json(drivers[0], files)
    for i, line in zip((1, 2, 3), out):
        tag, T, Tu, sx, su, bad = line.split()
        X, U = traj_arrays(i)
        assert tag == "OK" and int(T) == X.shape[0] and int(Tu) == U.shape[0]
        assert abs(float(sx) - X.sum()) <= 1e-9 * abs(X).sum() and abs(float(su) - U.sum()) <= 1e-9 * abs(U).sum()
        assert int(bad) == 0          # bucketed search == lower_bound everywhere


def corpus():
    X, U = traj_arrays(1)
    xs, us = json.dumps(X[:6].tolist()), json.dumps(U[:5].tolist())
    x2 = json.dumps(X[:9].tolist())
    deep = "[" * 100000 + "]" * 100000
    return {
        "dup_X_last_wins": '{"X": %s, "U": %s, "X": %s}' % (xs, us, x2),         # 9 rows, json.load: last
        "dup_X_shorter_last": '{"X": %s, "U": %s, "X": %s}' % (x2, us, xs),
        "dup_U": '{"U": [[1,2],[3,4],[5,6]], "X": %s, "U": %s}' % (xs, us),
        "deep_nesting_skipped_key": '{"deep": %s, "X": %s, "U": %s}' % (deep, xs, us),
        "nested_ok": '{"meta": {"a": [1, {"b": [true, false, null, "s\\"t"]}]}, "X": %s, "U": %s}' % (xs, us),
        "unicode_key": '{"\\u0058": %s, "U": %s}' % (xs, us),
        "truncated": '{"X": %s, "U": [[1, 2], [3' % xs,
        "wrong_width": '{"X": [[1,2,3,4]], "U": %s}' % us,
        "trailing_data": '{"X": %s, "U": %s} extra' % (xs, us),
        "missing_U": '{"X": %s}' % xs,
        "empty_object": "{}",
        "empty_file": "",
        "not_object": "[1, 2, 3]",
        "hex_number": '{"X": [[0x10, 1, 2, 3, 4]], "U": %s}' % us,
        "inf_word": '{"X": [[inf, 1, 2, 3, 4]], "U": %s}' % us,
        "nan_json": '{"X": [[NaN, 1, 2, 3, -Infinity]], "U": [[1, 2], [Infinity, 3]]}',
        "unterminated_string": '{"X": %s, "U": %s, "note": "abc' % (xs, us),
        "bad_escape": '{"\\u00zz": 1, "X": %s, "U": %s}' % (xs, us),
        "garbage_bytes": "\x00\xff{\x01",
    }


def test_json_reader_malformed_corpus(drivers, tmp_path):
    items = corpus()
    files = []
    for name, text in items.items():
        f = tmp_path / f"{name}.json"
        f.write_text(text, encoding="latin-1")
        files.append(f)
    out = run_json(drivers[0], files)
    assert len(out) == len(items)
    for (name, text), line in zip(items.items(), out):
        exp = expect_line(text)
        if exp == "ERR":
            assert line.startswith("ERR"), (name, line)
            continue
        tag, T, Tu, sx, su, bad = line.split()
        assert tag == "OK", (name, line)
        assert (int(T), int(Tu)) == (exp[1], exp[2]), (name, line)
        assert np.isclose(float(sx), np.sum(exp[3]), equal_nan=True), (name, line)
        assert np.isclose(float(su), np.sum(exp[4]), equal_nan=True), (name, line)
    got = dict(zip(items, out))
    assert got["dup_X_last_wins"].split()[1] == "9" and got["dup_X_shorter_last"].split()[1] == "6"
    assert "nesting too deep" in got["deep_nesting_skipped_key"]


def _oracle_inputs(B, kind, seed):
    import workloads as W
    cfg = {0: "C2", "fsm": "C3", 8: "C5"}[kind]
    wb = W.make_batch(cfg, B=B, seed=seed)
    X, U = traj_arrays(wb["traj"])
    mo = wb["max_obs"]
    obs = wb["obs"] if mo else np.zeros((B, 0, 2))
    nob = wb["n_obs"] if mo else np.zeros(B, np.int32)
    return X, U, wb["x0"], obs, nob.astype(np.int32), mo, wb["traj"], wb["N"]


@pytest.mark.parametrize("drv", [1, 2], ids=["oracle", "cpu_backend"])
@pytest.mark.parametrize("kind,B,sqp", [(0, 48, 1), ("fsm", 32, 10), (8, 12, 1)])
def test_oracle_under_asan_matches_regular_build(drivers, tmp_path, kind, B, sqp, drv):
    """The oracle (drv 1) and the product's host backend (drv 2, csrc/cpu_backend.h on 3 threads), both built
    with ASan/UBSan, against the regular oracle build: bit-identical (the backend performs the oracle's sequence
    of IEEE operations)."""
    import oracle as O
    X, U, x0, obs, nob, mo, ti, N = _oracle_inputs(B, kind, 5)
    fin = tmp_path / "in.bin"
    with open(fin, "wb") as f:
        f.write(np.array([X.shape[0], U.shape[0], N, B, mo, sqp], np.int32).tobytes())
        for a in (X, U, x0, obs):
            f.write(np.ascontiguousarray(a, np.float64).tobytes())
        f.write(np.ascontiguousarray(nob, np.int32).tobytes())
    fout = tmp_path / "out.bin"
    r = subprocess.run([drivers[drv], str(fin), str(fout)], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
    raw = fout.read_bytes()
    nU, nX = B * 2 * N, B * 5 * (N + 1)
    Ua = np.frombuffer(raw[:8 * nU], np.float64).reshape(B, N, 2)
    Xa = np.frombuffer(raw[8 * nU:8 * (nU + nX)], np.float64).reshape(B, N + 1, 5)
    sa = np.frombuffer(raw[8 * (nU + nX):], np.int32)[:B]
    orc = O.Oracle(X, U)
    ro = orc.solve_batch(O.default_params(N=N, max_obs=mo, sqp_iters=sqp), x0, obs if mo else None,
                         nob if mo else None)
    assert np.array_equal(sa, ro["status"])
    assert np.array_equal(Ua, ro["U"]) and np.array_equal(Xa, ro["Xpred"])


def test_plan_host_backend_under_asan(drivers, tmp_path):
    """csrc/plan_host.h under ASan/UBSan on 3 threads: 24 chunks of mixed horizons (intermediate and final) and
    the chunk loop from 2 starts; every output equals libmpcplan's host backend (plan_create device = -1)."""
    import __graft_entry__ as g
    g.build()
    import mpcplan
    import workloads as W
    r = W.plan_route("synth1")
    rng = np.random.default_rng(4)
    B, P, Cn = 24, 2, 40
    s0 = rng.uniform(0.0, r.s_total - 45.0, B)
    x0 = np.zeros((B, 5))
    x0[:, 0] = s0
    x0[:, 3] = [r.k_ref_fun(s) for s in s0]
    x0[:, 4] = [0.6 * r.v_max_fun(s) for s in s0]
    fin = (np.arange(B) % 3 == 2).astype(np.int32)
    st = np.where(fin == 1, np.minimum(s0 + 35.0, r.s_total), s0 + 20.0)
    N = np.array([(13, 17, 22)[i % 3] for i in range(B)], np.int32)
    Nmax = 32
    starts = np.zeros((P, 5))
    starts[1] = (600.0, 0.0, 0.0, r.k_ref_fun(600.0), 0.5 * r.v_max_fun(600.0))
    arr = [np.ascontiguousarray(a, np.float64) for a in (r.s, r.cx, r.cy, r.vmax)]
    M = arr[0].size
    avg = np.array([float(np.mean(arr[3][i:])) for i in range(M)])
    fin_in, fout = tmp_path / "plan_in.bin", tmp_path / "plan_out.bin"
    with open(fin_in, "wb") as f:
        np.array([M, B, Nmax, P, Cn], np.int32).tofile(f)
        for a in arr:
            a.tofile(f)
        N.tofile(f); fin.tofile(f); x0.tofile(f); st.tofile(f); starts.tofile(f); avg.tofile(f)
    res = subprocess.run([drivers[3], str(fin_in), str(fout)], capture_output=True, text=True, env=ENV, timeout=900)
    assert res.returncode == 0, res.stderr[-3000:]
    assert "runtime error" not in res.stderr and "AddressSanitizer" not in res.stderr, res.stderr[-3000:]
    raw = open(fout, "rb").read()
    off = 0

    def take(dt, n):
        nonlocal off
        a = np.frombuffer(raw, dt, n, off)
        off += a.nbytes
        return a

    X = take(np.float64, B * (Nmax + 1) * 5).reshape(B, Nmax + 1, 5)
    U = take(np.float64, B * Nmax * 2).reshape(B, Nmax, 2)
    S = take(np.float64, B * Nmax).reshape(B, Nmax)
    status, iters, sqp = take(np.int32, B), take(np.int32, B), take(np.int32, B)
    LX = take(np.float64, P * Cn * (Nmax + 1) * 5).reshape(P, Cn, Nmax + 1, 5)
    LN, Lst, nch = take(np.int32, P * Cn).reshape(P, Cn), take(np.int32, P * Cn).reshape(P, Cn), take(np.int32, P)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=Nmax), device=-1)
    # the library solves with the batch's own row stride (its largest horizon); compare on those rows
    ref = pl.solve_chunks(x0, st, fin, N)
    nm = int(N.max())
    assert np.array_equal(X[:, :nm + 1], ref["X"]) and np.array_equal(U[:, :nm], ref["U"])
    assert np.array_equal(S[:, :nm], ref["S"])
    for a, b in ((status, ref["status"]), (iters, ref["iters"]), (sqp, ref["sqp"])):
        assert np.array_equal(a, b)
    lo = pl.optimize_device(starts, 20.0, Cn, avg, Nmax)
    assert np.array_equal(nch, lo["nchunks"])
    for b in range(P):
        n = int(nch[b])
        assert n > 0
        assert np.array_equal(LN[b, :n], lo["N"][b, :n]) and np.array_equal(Lst[b, :n], lo["status"][b, :n])
        assert np.array_equal(LX[b, :n], lo["X"][b, :n])
    pl.close()
