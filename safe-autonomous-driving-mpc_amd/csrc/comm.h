// Ego-shard communicator of libmpcqp (include/mpcqp.h, "Multi-GPU"): RCCL over xGMI behind the C ABI.
//
// The sharded path has no per-step exchange; its one collective is the final gather of the
// closed-loop telemetry that the reference's run_simulation returns (trajectory_tracking.py:443) to rank 0.
// This file gives that gather (ncclGather, rccl.h:745), plus the barrier and the max-over-ranks reduction
// the measurement needs, as plain extern "C" entries: no torch on the GPU ranks' communication path.
//
// RCCL is opened with dlopen("librccl.so.1") when the first communicator is created, so the solver library
// loads and runs without it (CPU hosts, single-GPU use) and a missing RCCL fails mpc_comm_create loudly
// (MPC_E_COMM with the loader's message).  Included once, at the end of mpcqp.hip (uses its fail / HIPCHK).
#pragma once

#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>

namespace mpcqp_comm {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id;
    decltype(&ncclCommInitRank) init_rank;
    decltype(&ncclCommDestroy) destroy;
    decltype(&ncclGather) gather;
    decltype(&ncclAllReduce) all_reduce;
    decltype(&ncclGetErrorString) error_string;
    decltype(&ncclGetVersion) version;
};

static Rccl g_rccl;
static std::string g_rccl_err;

// resolve the RCCL entries once per process; false (with g_rccl_err) when the library or a symbol is missing
static bool load_rccl() {
    static std::once_flag once;
    static bool ok = false;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            g_rccl_err = std::string("dlopen librccl.so.1: ") + (e ? e : "not found");
            return;
        }
        struct { const char* name; void** slot; } syms[] = {
            {"ncclGetUniqueId", (void**)&g_rccl.get_unique_id}, {"ncclCommInitRank", (void**)&g_rccl.init_rank},
            {"ncclCommDestroy", (void**)&g_rccl.destroy},       {"ncclGather", (void**)&g_rccl.gather},
            {"ncclAllReduce", (void**)&g_rccl.all_reduce},      {"ncclGetErrorString", (void**)&g_rccl.error_string},
            {"ncclGetVersion", (void**)&g_rccl.version}};
        for (auto& s : syms) {
            *s.slot = dlsym(h, s.name);
            if (!*s.slot) {
                g_rccl_err = std::string("librccl.so.1 lacks ") + s.name;
                return;
            }
        }
        ok = true;
    });
    return ok;
}

}  // namespace mpcqp_comm

struct mpc_comm {
    ncclComm_t nc;
    int nranks, rank, device;
    hipStream_t stream;       // the communicator's own stream (host-buffer entries, barrier)
    unsigned char* dbuf;      // staging buffer of mpc_gather_host: nranks x bytes (rank's block in place)
    size_t cap;
    double* dred;             // one double for the barrier / max reduction
};

#define NCCLCHK(expr, what)                                                                          \
    do {                                                                                             \
        ncclResult_t r_ = (expr);                                                                    \
        if (r_ != ncclSuccess)                                                                       \
            return fail(MPC_E_COMM, std::string(what) + ": " + mpcqp_comm::g_rccl.error_string(r_)); \
    } while (0)

extern "C" int mpc_comm_unique_id(char* uid) {
    if (!uid) return fail(MPC_E_ARG, "uid is NULL");
    if (!mpcqp_comm::load_rccl()) return fail(MPC_E_COMM, mpcqp_comm::g_rccl_err);
    ncclUniqueId id;
    NCCLCHK(mpcqp_comm::g_rccl.get_unique_id(&id), "ncclGetUniqueId");
    std::memcpy(uid, id.internal, MPC_COMM_UID_BYTES);
    return MPC_SUCCESS;
}

extern "C" int mpc_comm_create(const char* uid, int nranks, int rank, int device, mpc_comm** out) {
    if (!out) return fail(MPC_E_ARG, "out is NULL");
    *out = nullptr;
    if (!uid) return fail(MPC_E_ARG, "uid is NULL");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(MPC_E_ARG, "rank / nranks out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(MPC_E_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(MPC_E_DEVICE, "device index out of range");
    if (!mpcqp_comm::load_rccl()) return fail(MPC_E_COMM, mpcqp_comm::g_rccl_err);
    HIPCHK(hipSetDevice(device), MPC_E_DEVICE);
    mpc_comm* c = (mpc_comm*)std::calloc(1, sizeof(mpc_comm));
    if (!c) return fail(MPC_E_ALLOC, "calloc");
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId id;
    std::memcpy(id.internal, uid, MPC_COMM_UID_BYTES);
    int rc = MPC_SUCCESS;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        rc = fail(MPC_E_DEVICE, "hipStreamCreate");
    else if (hipMalloc(&c->dred, sizeof(double)) != hipSuccess)
        rc = fail(MPC_E_ALLOC, "hipMalloc");
    else {
        ncclResult_t r = mpcqp_comm::g_rccl.init_rank(&c->nc, nranks, id, rank);
        if (r != ncclSuccess) {
            c->nc = nullptr;
            rc = fail(MPC_E_COMM, std::string("ncclCommInitRank: ") + mpcqp_comm::g_rccl.error_string(r));
        }
    }
    if (rc != MPC_SUCCESS) {
        if (c->dred) (void)hipFree(c->dred);
        if (c->stream) (void)hipStreamDestroy(c->stream);
        std::free(c);
        return rc;
    }
    *out = c;
    return MPC_SUCCESS;
}

extern "C" int mpc_comm_info(const mpc_comm* c, int* nranks, int* rank, int* device) {
    if (!c) return fail(MPC_E_ARG, "comm is NULL");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return MPC_SUCCESS;
}

extern "C" int mpc_gather(mpc_comm* c, const void* send, size_t bytes, void* recv, int root, void* stream) {
    if (!c) return fail(MPC_E_ARG, "comm is NULL");
    if (root < 0 || root >= c->nranks) return fail(MPC_E_ARG, "root out of range");
    if (bytes && !send) return fail(MPC_E_ARG, "send is NULL");
    if (bytes && c->rank == root && !recv) return fail(MPC_E_ARG, "recv is NULL on the root");
    if (!bytes) return MPC_SUCCESS;
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    NCCLCHK(mpcqp_comm::g_rccl.gather(send, recv, bytes, ncclUint8, root, c->nc, (hipStream_t)stream),
            "ncclGather");
    return MPC_SUCCESS;
}

extern "C" int mpc_gather_host(mpc_comm* c, const void* send, size_t bytes, void* recv, int root) {
    if (!c) return fail(MPC_E_ARG, "comm is NULL");
    if (root < 0 || root >= c->nranks) return fail(MPC_E_ARG, "root out of range");
    if (bytes && !send) return fail(MPC_E_ARG, "send is NULL");
    if (bytes && c->rank == root && !recv) return fail(MPC_E_ARG, "recv is NULL on the root");
    if (!bytes) return MPC_SUCCESS;
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    const size_t need = bytes * (size_t)c->nranks;
    if (need > c->cap) {
        if (c->dbuf) HIPCHK(hipFree(c->dbuf), MPC_E_DEVICE);
        c->dbuf = nullptr;
        c->cap = 0;
        HIPCHK(hipMalloc(&c->dbuf, need), MPC_E_ALLOC);
        c->cap = need;
    }
    // the rank's block sits at its own offset, so the gather runs in place (rccl.h:733)
    unsigned char* mine = c->dbuf + bytes * (size_t)c->rank;
    HIPCHK(hipMemcpyAsync(mine, send, bytes, hipMemcpyHostToDevice, c->stream), MPC_E_DEVICE);
    NCCLCHK(mpcqp_comm::g_rccl.gather(mine, c->dbuf, bytes, ncclUint8, root, c->nc, c->stream), "ncclGather");
    if (c->rank == root)
        HIPCHK(hipMemcpyAsync(recv, c->dbuf, need, hipMemcpyDeviceToHost, c->stream), MPC_E_DEVICE);
    HIPCHK(hipStreamSynchronize(c->stream), MPC_E_DEVICE);
    return MPC_SUCCESS;
}

extern "C" int mpc_comm_allreduce_max(mpc_comm* c, double* value) {
    if (!c || !value) return fail(MPC_E_ARG, "NULL argument");
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    HIPCHK(hipMemcpyAsync(c->dred, value, sizeof(double), hipMemcpyHostToDevice, c->stream), MPC_E_DEVICE);
    NCCLCHK(mpcqp_comm::g_rccl.all_reduce(c->dred, c->dred, 1, ncclFloat64, ncclMax, c->nc, c->stream),
            "ncclAllReduce");
    HIPCHK(hipMemcpyAsync(value, c->dred, sizeof(double), hipMemcpyDeviceToHost, c->stream), MPC_E_DEVICE);
    HIPCHK(hipStreamSynchronize(c->stream), MPC_E_DEVICE);
    return MPC_SUCCESS;
}

extern "C" int mpc_comm_barrier(mpc_comm* c) {
    double one = 1.0;
    return mpc_comm_allreduce_max(c, &one);
}

extern "C" void mpc_comm_destroy(mpc_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->nc) (void)mpcqp_comm::g_rccl.destroy(c->nc);
    if (c->dbuf) (void)hipFree(c->dbuf);
    if (c->dred) (void)hipFree(c->dred);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    std::free(c);
}
