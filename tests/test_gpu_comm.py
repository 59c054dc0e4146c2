"""GPU: libmpcqp's ego-shard communicator (mpc_comm_* / mpc_gather*, include/mpcqp.h) -- RCCL over xGMI
behind the C ABI, the one collective of the sharded path: the gather to rank 0 of the telemetry
the reference's run_simulation returns (trajectory_tracking.py:443).

The box has one GPU, so the communicator runs at world 1 (RCCL refuses two ranks on one device); the
rendezvous and the multi-rank packing are covered on the CPU by tests/test_multirank.py.  Through the
communicator, byte-exactly: a host payload (mpc_gather_host), a device payload (mpc_gather on a stream),
the closed-loop payload of shard.pack_closed_loop, the max reduction and the barrier.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import __graft_entry__ as g
    g.build()
    import shard
    c = shard.ShardComm.rccl(1, 0, 0)
    assert c.transport == "rccl"
    yield c
    c.close()


def test_gather_host_payload_byte_exact(comm):
    rng = np.random.default_rng(5)
    for n in (1, 7, 4096, 3 << 20):
        payload = rng.integers(0, 256, n, dtype=np.uint8)
        got = comm.gather(payload)
        assert len(got) == 1 and np.array_equal(got[0], payload)


def test_gather_device_payload_byte_exact(comm):
    import torch
    src = torch.arange(1 << 16, dtype=torch.float64, device="cuda:0") * 0.5
    dst = torch.full_like(src, np.nan)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    comm.native.gather_device(src.data_ptr(), src.numel() * 8, dst.data_ptr(), root=0, stream=st.cuda_stream)
    st.synchronize()
    assert torch.equal(src, dst)


def test_closed_loop_payload_through_rccl(comm):
    """shard.pack_closed_loop -> RCCL gather -> closed_loop_report equals the local report."""
    import shard
    rng = np.random.default_rng(9)
    B, steps, hist = 5, 40, 2
    r = {"hist_x": rng.normal(size=(B, steps + 1, 5)), "hist_u": rng.normal(size=(B, steps, 2))}
    q = np.column_stack([np.arange(B), np.full(B, steps), rng.normal(size=(B, len(shard.CL_FIELDS) - 2))])
    payload = shard.pack_closed_loop(q, r, B, hist, steps)
    got = shard.gather_closed_loop(payload, comm)
    assert len(got) == 1 and np.array_equal(got[0], payload)
    qg, hg = shard.unpack_closed_loop(got[0], B, hist, steps)
    assert np.array_equal(qg, q)
    assert np.array_equal(hg[:, :, :5], r["hist_x"][:hist, 1:].astype(np.float32))


def test_max_and_barrier(comm):
    assert comm.max(3.25) == 3.25
    comm.barrier()
    tel = shard_telemetry_roundtrip(comm)
    assert tel["egos"] == 6 and tel["ranks"] == 1


def shard_telemetry_roundtrip(comm):
    import shard
    mat = shard.gather_telemetry(shard.telemetry(np.array([0, 0, 2, 16, 1, 0]), np.array([0, 3, 9, 4, 1, 2])), comm)
    return shard.reduce_telemetry(mat)


def test_comm_argument_errors():
    import mpcqp
    with pytest.raises(ValueError):
        mpcqp.Comm(b"x", 1, 0, 0)
    uid = mpcqp.comm_unique_id()
    with pytest.raises(mpcqp.MpcError):
        mpcqp.Comm(uid, 1, 1, 0)          # rank out of range
    with pytest.raises(mpcqp.MpcError):
        mpcqp.Comm(uid, 1, 0, 99)         # no such device
