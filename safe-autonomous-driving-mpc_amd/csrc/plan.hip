// plan.hip — MI355X batched offline planner: libmpcplan.so (C ABI: include/mpcplan.h).
//
// The chunk NLP of the reference's offline planner (TrajectoryOptimizer, trajectory_planning.py:8-391,
// driven by optimize_full_trajectory :419-559) solved for B independent chunks per launch, FP64.  The
// algorithm is the one DESIGN.md ("Offline planner") describes and oracle/plan_oracle.c restates on the CPU
// (the tests' checker; nothing here includes, links or calls it):
//   Gauss-Newton / exact-Hessian SQP over z = [X, U, S] from the reference's initial guess (:357-376), a
//   non-monotone L1-merit line search, speed limits frozen after a 2-cycle at a limit change; each QP by an
//   active-set crossover from the previous QP's active rows, else a Mehrotra interior point on the
//   stage-wise Riccati recursion followed by the same equality-constrained solve ("polish").
//
// Mapping: one wavefront (one 64-lane workgroup) = one chunk, its whole working set in LDS (265 doubles per
// stage, about 37 KB at N = 16: four chunks per CU).  Everything that is independent per stage runs
// stage-parallel, lane k on stage k: the linearisation (Hermite-Simpson Jacobians, the exact-Hessian fold),
// the barrier-weighted stage Hessians, the interior point's row residuals, directions, ratio tests and
// updates, the merit evaluations of the line search (defects of every interval), the multiplier recovery.
// The Riccati factorisation and its backward / forward recursions are sequential in the stage and run
// lane-distributed inside the wave (plan_kernel.h: factor_par, solve_core).  Reductions (complementarity,
// step lengths, norms) are wave shuffles.  Every chunk's wave retires on its own.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>


#include "../../include/mpcplan.h"
#include "plan_kernel.h"
#include "plan_host.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

size_t lds_bytes(int Nmax) { return sizeof(double) * (size_t)make_layout(Nmax).total; }

}  // namespace

struct plan_ctx {
    int device;
    plan_params p;
    plan_host::route* host;   // device = -1: the host backend's route (plan_host.h); every HIP member unused
    int host_threads;
    DevRoute R;
    double* d_route;          // s | cx | cy | vmax
    size_t lds_max;           // the device's LDS per workgroup
    // host-entry staging
    void* io;
    size_t io_bytes;
    // longest-first dispatch (plan_order_*_kernel): a small pool of buffers (2 * ORDER_BUCKETS counters, then
    // bucket[cap], order[cap]), each remembering the stream it last served and an event recorded after its last
    // chunk kernel.  A call prefers its stream's buffer, else a new one (up to ORDER_POOL), else the least
    // recently used; before using a buffer it waits for that buffer's event, so a buffer is never rewritten
    // while an earlier plan_chunk_kernel still reads its order[] (whatever stream that ran on, and whether or
    // not a new stream reuses a destroyed stream's address).  Concurrent launches on distinct streams keep
    // distinct buffers.  A call on a stream that is being captured into a graph never uses the pool (index
    // order, same results): a graph must not replay order kernels against a buffer shared with eager calls.
    struct OrderBuf {
        int* ptr;
        hipEvent_t done;
        void* stream;
        unsigned long long last_use;
        bool used;
    };
    std::vector<OrderBuf> order_bufs;
    unsigned long long order_clock;
    std::mutex order_mu;
    int cap_order;
    bool order_on;
};

#define ORDER_POOL 8

// the buffer this call may use (its event already waited on by `stream`), or nullptr: index order (the stream
// is being captured, or an allocation failed)
static plan_ctx::OrderBuf* order_buffer(plan_ctx* c, void* stream) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    std::lock_guard<std::mutex> g(c->order_mu);
    plan_ctx::OrderBuf* b = nullptr;
    for (auto& e : c->order_bufs)
        if (e.stream == stream) b = &e;
    if (!b && c->order_bufs.size() < ORDER_POOL) {
        plan_ctx::OrderBuf e{};
        if (hipMalloc(&e.ptr, sizeof(int) * (2 * (size_t)ORDER_BUCKETS + 2 * (size_t)c->cap_order)) != hipSuccess)
            return nullptr;
        if (hipEventCreateWithFlags(&e.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipFree(e.ptr);
            return nullptr;
        }
        c->order_bufs.push_back(e);
        b = &c->order_bufs.back();
    }
    if (!b) {
        b = &c->order_bufs[0];
        for (auto& e : c->order_bufs)
            if (e.last_use < b->last_use) b = &e;
    }
    if (b->used && hipStreamWaitEvent((hipStream_t)stream, b->done, 0) != hipSuccess) return nullptr;
    b->stream = stream;
    b->last_use = ++c->order_clock;
    return b;
}

static int check_params(const plan_params* p) {
    if (!p) return fail(PLAN_E_ARG, "params is NULL");
    if (!(p->dt > 0.0)) return fail(PLAN_E_ARG, "dt must be > 0");
    if (p->N < 1 || p->N > PLAN_MAX_N) return fail(PLAN_E_ARG, "N out of range [1, PLAN_MAX_N]");
    if (p->sqp_iters < 1 || p->max_iter < 1) return fail(PLAN_E_ARG, "sqp_iters and max_iter must be >= 1");
    if (!(p->sqp_tol >= 0.0) || !(p->tol > 0.0)) return fail(PLAN_E_ARG, "tolerances must be positive");
    if (!(p->defect_sign == 1.0 || p->defect_sign == -1.0)) return fail(PLAN_E_ARG, "defect_sign must be +1 or -1");
    if (!(p->u_min[0] < p->u_max[0]) || !(p->u_min[1] < p->u_max[1]) || !(p->k_min < p->k_max))
        return fail(PLAN_E_ARG, "bounds must satisfy min < max");
    return PLAN_SUCCESS;
}

extern "C" {

void plan_default_params(plan_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->N = 20;
    p->dt = 0.3;
    p->w_y = 10.0; p->w_s = 10.0; p->w_u = 0.1; p->w_slack = 100.0;
    p->u_min[0] = -0.6; p->u_min[1] = -5.0;
    p->u_max[0] = 0.6; p->u_max[1] = 4.0;
    p->k_min = -0.8; p->k_max = 0.8;
    p->a_max = 6.0;
    p->v_min = 0.0;
    p->defect_sign = 1.0;
    p->sqp_iters = 100;
    p->sqp_tol = 1e-9;
    p->max_iter = 100;
    p->tol = 1e-10;
}

const char* plan_last_error(void) { return g_err.c_str(); }
int plan_version(void) { return MPCPLAN_VERSION; }

int plan_create(const double* s, int M, const double* cx, const double* cy, const double* vmax, const plan_params* p,
                int device, plan_ctx** out) {
    if (!out) return fail(PLAN_E_ARG, "out is NULL");
    *out = nullptr;
    if (!s || !cx || !cy || !vmax) return fail(PLAN_E_ARG, "route arrays must not be NULL");
    if (M < 3) return fail(PLAN_E_ARG, "a route needs at least 3 way-points");
    for (int i = 1; i < M; ++i)
        if (!(s[i] > s[i - 1])) return fail(PLAN_E_ARG, "route s must be strictly increasing");
    for (int i = 0; i < 4 * (M - 1); ++i)
        if (!std::isfinite(cx[i]) || !std::isfinite(cy[i])) return fail(PLAN_E_ARG, "spline coefficients must be finite");
    for (int i = 0; i < M; ++i)
        if (!std::isfinite(vmax[i])) return fail(PLAN_E_ARG, "speed limits must be finite");
    if (int rc = check_params(p)) return rc;
    if (device == -1) {
        // host backend: the chunk solve on std::thread workers (plan_host.h), no HIP call
        plan_ctx* c = new plan_ctx();
        c->device = -1;
        c->p = *p;
        if (plan_host::route_create(s, M, cx, cy, vmax, &c->host) != PLAN_SUCCESS) {
            delete c;
            return fail(PLAN_E_ALLOC, "host route allocation failed");
        }
        const char* te = std::getenv("PLAN_CPU_THREADS");
        const int hw = (int)std::thread::hardware_concurrency();
        c->host_threads = te && std::atoi(te) > 0 ? std::atoi(te) : std::max(1, hw);
        *out = c;
        return PLAN_SUCCESS;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PLAN_E_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(PLAN_E_DEVICE, "device index out of range (-1: the host backend)");
    if (hipSetDevice(device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) lds = 65536;
    plan_ctx* c = new plan_ctx();
    c->device = device;
    c->p = *p;
    c->lds_max = (size_t)lds;
    // route arrays (s | cx | cy | vmax) followed by the search grid (ints), one allocation
    const int T = std::max(64, std::min(1 << 18, 4 * M));
    const size_t n = (size_t)M + 8 * (size_t)(M - 1) + M;
    const size_t nb = n * sizeof(double) + sizeof(int) * (size_t)T;
    if (hipMalloc(&c->d_route, nb) != hipSuccess) {
        delete c;
        return fail(PLAN_E_ALLOC, "route allocation failed");
    }
    std::vector<double> h(n + (T + 1) / 2);
    std::memcpy(h.data(), s, sizeof(double) * M);
    std::memcpy(h.data() + M, cx, sizeof(double) * 4 * (M - 1));
    std::memcpy(h.data() + M + 4 * (M - 1), cy, sizeof(double) * 4 * (M - 1));
    std::memcpy(h.data() + M + 8 * (M - 1), vmax, sizeof(double) * M);
    double ginv = 0.0;
    route_grid(s, M, T, (int*)(h.data() + n), &ginv);
    if (hipMemcpy(c->d_route, h.data(), nb, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(c->d_route);
        delete c;
        return fail(PLAN_E_DEVICE, "route upload failed");
    }
    c->R.s = c->d_route;
    c->R.cx = c->d_route + M;
    c->R.cy = c->d_route + M + 4 * (M - 1);
    c->R.vmax = c->d_route + M + 8 * (M - 1);
    c->R.grid = (const int*)(c->d_route + n);
    c->R.T = T;
    c->R.ginv = ginv;
    c->R.M = M;
    c->R.s_total = s[M - 1];
    c->cap_order = 1 << 17;
    c->order_bufs.reserve(ORDER_POOL);      // never reallocated: buffer pointers stay valid
    const char* oe = std::getenv("PLAN_ORDER");        // PLAN_ORDER=0: index order (A/B)
    c->order_on = !(oe && oe[0] == '0');
    *out = c;
    return PLAN_SUCCESS;
}

int plan_set_params(plan_ctx* c, const plan_params* p) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (int rc = check_params(p)) return rc;
    c->p = *p;
    return PLAN_SUCCESS;
}

void plan_destroy(plan_ctx* c) {
    if (!c) return;
    if (c->host) {
        plan_host::route_destroy(c->host);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->d_route) (void)hipFree(c->d_route);
    if (c->io) (void)hipFree(c->io);
    for (auto& e : c->order_bufs) {
        (void)hipFree(e.ptr);
        (void)hipEventDestroy(e.done);
    }
    delete c;
}

int plan_solve_chunks_device(plan_ctx* c, int B, int Nmax, const int* N, const double* x0, const double* s_target,
                             const int* is_final, double* X, double* U, double* S, int* status, int* iters, int* sqp,
                             void* stream) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (c->host) return fail(PLAN_E_DEVICE, "plan_solve_chunks_device on a host context (device = -1): use plan_solve_chunks");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!x0 || !s_target) return fail(PLAN_E_ARG, "x0 and s_target are required");
    // Nmax is always the caller's row stride; without per-chunk N every chunk has the params' horizon
    if (Nmax < 1 || Nmax > PLAN_MAX_N) return fail(PLAN_E_ARG, "Nmax out of range [1, PLAN_MAX_N]");
    if (!N && Nmax < c->p.N) return fail(PLAN_E_ARG, "Nmax must be >= params N when N is NULL (Nmax is the row stride)");
    const size_t lds = lds_bytes(Nmax);
    if (lds > c->lds_max) return fail(PLAN_E_ARG, "Nmax too large for the device's LDS");
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    if (lds > 65536 &&
        hipFuncSetAttribute((const void*)plan_chunk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(PLAN_E_LAUNCH, "cannot raise the kernel's LDS limit");
    KArgs a;
    a.R = c->R;
    a.P = c->p;
    a.B = B;
    a.Nmax = Nmax;
    a.Nfixed = c->p.N;
    // PLAN_DBG (diagnostics only): repeats a phase for A/B timing, the results do not change.  Bits: 1 each
    // interior-point factorisation, 2 each solve, 4 the interior point's gradient/row loop, 8 its direction
    // loop, 16 build_qp, 32 multipliers, 64 each line-search merit evaluation
    const char* dbg = std::getenv("PLAN_DBG");
    a.dbg = dbg ? std::atoi(dbg) : 0;
    a.N = N;
    a.x0 = x0;
    a.st = s_target;
    a.order = nullptr;
    plan_ctx::OrderBuf* ob = (c->order_on && B >= 2 * WAVE && B <= c->cap_order) ? order_buffer(c, stream) : nullptr;
    if (ob) {
        int* cnt = ob->ptr;
        int* bucket = cnt + 2 * ORDER_BUCKETS;
        int* order = bucket + c->cap_order;
        const int nb = (B + 255) / 256;
        if (hipMemsetAsync(cnt, 0, sizeof(int) * 2 * ORDER_BUCKETS, (hipStream_t)stream) != hipSuccess)
            return fail(PLAN_E_LAUNCH, "order reset failed");
        hipLaunchKernelGGL(plan_order_count_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, c->R, c->p, B, x0,
                           s_target, bucket, cnt);
        hipLaunchKernelGGL(plan_order_scatter_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, B, bucket, cnt,
                           cnt + ORDER_BUCKETS, order);
        if (hipError_t e = hipGetLastError(); e != hipSuccess)
            return fail(PLAN_E_LAUNCH, std::string("order kernels failed: ") + hipGetErrorString(e));
        a.order = order;
    }
    a.fin = is_final;
    a.X = X;
    a.U = U;
    a.S = S;
    a.status = status;
    a.iters = iters;
    a.sqp = sqp;
    hipLaunchKernelGGL(plan_chunk_kernel, dim3(B), dim3(WAVE), lds, (hipStream_t)stream, a);
    if (hipError_t e = hipGetLastError(); e != hipSuccess)
        return fail(PLAN_E_LAUNCH, std::string("plan kernel launch failed: ") + hipGetErrorString(e));
    if (ob) {
        // the buffer is free again once this kernel has read its order[]
        std::lock_guard<std::mutex> g(c->order_mu);
        if (hipEventRecord(ob->done, (hipStream_t)stream) != hipSuccess)
            return fail(PLAN_E_DEVICE, "order buffer event record failed");
        ob->used = true;
    }
    return PLAN_SUCCESS;
}

int plan_chunks_per_cu(plan_ctx* c, int Nmax, int* out) {
    if (!c || !out) return fail(PLAN_E_ARG, "ctx and out are required");
    if (c->host) return fail(PLAN_E_DEVICE, "plan_chunks_per_cu on a host context (device = -1)");
    if (Nmax < 1 || Nmax > PLAN_MAX_N) return fail(PLAN_E_ARG, "Nmax out of range [1, PLAN_MAX_N]");
    const size_t lds = lds_bytes(Nmax);
    if (lds > c->lds_max) return fail(PLAN_E_ARG, "Nmax too large for the device's LDS");
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    if (lds > 65536 &&
        hipFuncSetAttribute((const void*)plan_chunk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(PLAN_E_LAUNCH, "cannot raise the kernel's LDS limit");
    // one workgroup (one wavefront) per chunk: the residency is set by the kernel's registers and its LDS
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)plan_chunk_kernel, WAVE, lds) != hipSuccess)
        return fail(PLAN_E_DEVICE, "occupancy query failed");
    *out = n;
    return PLAN_SUCCESS;
}

int plan_optimize_device(plan_ctx* c, int B, int Nmax, const double* starts, double max_chunk_size, int max_chunks,
                         const double* avg, int nav, double* X, double* U, double* S, int* N, int* is_final,
                         int* status, int* iters, int* sqp, int* nchunks, void* stream) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (c->host) return fail(PLAN_E_DEVICE, "plan_optimize_device on a host context (device = -1): use plan_optimize");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!starts || !avg || !X || !U || !S || !N || !is_final || !status || !iters || !sqp || !nchunks)
        return fail(PLAN_E_ARG, "plan_optimize_device: every array is required");
    if (Nmax < 1 || Nmax > PLAN_MAX_N) return fail(PLAN_E_ARG, "Nmax out of range [1, PLAN_MAX_N]");
    if (max_chunks < 1) return fail(PLAN_E_ARG, "max_chunks must be >= 1");
    if (nav < 1) return fail(PLAN_E_ARG, "avg must have at least one entry");
    if (!(max_chunk_size > 0.0) || !std::isfinite(max_chunk_size)) return fail(PLAN_E_ARG, "max_chunk_size must be > 0");
    const size_t lds = lds_bytes(Nmax);
    if (lds > c->lds_max) return fail(PLAN_E_ARG, "Nmax too large for the device's LDS");
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    if (lds > 65536 &&
        hipFuncSetAttribute((const void*)plan_loop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(PLAN_E_LAUNCH, "cannot raise the kernel's LDS limit");
    LArgs a;
    a.R = c->R;
    a.P = c->p;
    a.B = B;
    a.Nmax = Nmax;
    a.max_chunks = max_chunks;
    a.nav = nav;
    a.max_chunk_size = max_chunk_size;
    a.avg = avg;
    a.starts = starts;
    a.X = X;
    a.U = U;
    a.S = S;
    a.N = N;
    a.fin = is_final;
    a.status = status;
    a.iters = iters;
    a.sqp = sqp;
    a.nchunks = nchunks;
    hipLaunchKernelGGL(plan_loop_kernel, dim3(B), dim3(WAVE), lds, (hipStream_t)stream, a);
    if (hipError_t e = hipGetLastError(); e != hipSuccess)
        return fail(PLAN_E_LAUNCH, std::string("plan loop kernel launch failed: ") + hipGetErrorString(e));
    return PLAN_SUCCESS;
}

int plan_solve_chunks(plan_ctx* c, int B, const int* N, const double* x0, const double* s_target, const int* is_final,
                      double* X, double* U, double* S, int* status, int* iters, int* sqp) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!x0 || !s_target) return fail(PLAN_E_ARG, "x0 and s_target are required");
    int Nmax = c->p.N;
    if (N) {
        Nmax = 0;
        for (int b = 0; b < B; ++b) {
            if (N[b] < 1 || N[b] > PLAN_MAX_N) return fail(PLAN_E_ARG, "N[b] out of range [1, PLAN_MAX_N]");
            Nmax = std::max(Nmax, N[b]);
        }
    }
    if (c->host) {
        plan_host::batch(c->host, &c->p, B, Nmax, N, x0, s_target, is_final, X, U, S, status, iters, sqp, c->host_threads);
        return PLAN_SUCCESS;
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    const size_t nX = (size_t)B * (Nmax + 1) * 5, nU = (size_t)B * Nmax * 2, nS = (size_t)B * Nmax;
    const size_t bytes = sizeof(double) * (5 * (size_t)B + B + nX + nU + nS) + sizeof(int) * (5 * (size_t)B);
    if (bytes > c->io_bytes) {
        if (c->io) (void)hipFree(c->io);
        c->io = nullptr;
        c->io_bytes = 0;
        if (hipMalloc(&c->io, bytes) != hipSuccess) return fail(PLAN_E_ALLOC, "staging allocation failed");
        c->io_bytes = bytes;
    }
    double* d_x0 = (double*)c->io;
    double* d_st = d_x0 + 5 * (size_t)B;
    double* d_X = d_st + B;
    double* d_U = d_X + nX;
    double* d_S = d_U + nU;
    int* d_N = (int*)(d_S + nS);
    int* d_fin = d_N + B;
    int* d_status = d_fin + B;
    int* d_iters = d_status + B;
    int* d_sqp = d_iters + B;
    bool ok = hipMemcpy(d_x0, x0, sizeof(double) * 5 * B, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_st, s_target, sizeof(double) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (ok && N) ok = hipMemcpy(d_N, N, sizeof(int) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (ok && is_final) ok = hipMemcpy(d_fin, is_final, sizeof(int) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return fail(PLAN_E_DEVICE, "input upload failed");
    int rc = plan_solve_chunks_device(c, B, Nmax, N ? d_N : nullptr, d_x0, d_st, is_final ? d_fin : nullptr, d_X, d_U,
                                      d_S, d_status, d_iters, d_sqp, nullptr);
    if (rc != PLAN_SUCCESS) return rc;
    if (hipError_t e = hipDeviceSynchronize(); e != hipSuccess)
        return fail(PLAN_E_DEVICE, std::string("plan kernel failed: ") + hipGetErrorString(e));
    ok = (!X || hipMemcpy(X, d_X, sizeof(double) * nX, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!U || hipMemcpy(U, d_U, sizeof(double) * nU, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!S || hipMemcpy(S, d_S, sizeof(double) * nS, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!status || hipMemcpy(status, d_status, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!iters || hipMemcpy(iters, d_iters, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!sqp || hipMemcpy(sqp, d_sqp, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess);
    if (!ok) return fail(PLAN_E_DEVICE, "output download failed");
    return PLAN_SUCCESS;
}

int plan_optimize(plan_ctx* c, int B, int Nmax, const double* starts, double max_chunk_size, int max_chunks,
                  const double* avg, int nav, double* X, double* U, double* S, int* N, int* is_final, int* status,
                  int* iters, int* sqp, int* nchunks) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!starts || !avg || !X || !U || !S || !N || !is_final || !status || !iters || !sqp || !nchunks)
        return fail(PLAN_E_ARG, "plan_optimize: every array is required");
    if (Nmax < 1 || Nmax > PLAN_MAX_N) return fail(PLAN_E_ARG, "Nmax out of range [1, PLAN_MAX_N]");
    if (max_chunks < 1) return fail(PLAN_E_ARG, "max_chunks must be >= 1");
    if (nav < 1) return fail(PLAN_E_ARG, "avg must have at least one entry");
    if (c->host) {
        if (!(max_chunk_size > 0.0) || !std::isfinite(max_chunk_size)) return fail(PLAN_E_ARG, "max_chunk_size must be > 0");
        plan_host::optimize(c->host, &c->p, B, Nmax, starts, max_chunk_size, max_chunks, avg, nav, X, U, S, N, is_final,
                            status, iters, sqp, nchunks, c->host_threads);
        return PLAN_SUCCESS;
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    const size_t slots = (size_t)B * max_chunks;
    const size_t nX = slots * (Nmax + 1) * 5, nU = slots * Nmax * 2, nS = slots * Nmax;
    const size_t bytes = sizeof(double) * (5 * (size_t)B + nav + nX + nU + nS) + sizeof(int) * (5 * slots + B);
    if (bytes > c->io_bytes) {
        if (c->io) (void)hipFree(c->io);
        c->io = nullptr;
        c->io_bytes = 0;
        if (hipMalloc(&c->io, bytes) != hipSuccess) return fail(PLAN_E_ALLOC, "staging allocation failed");
        c->io_bytes = bytes;
    }
    double* d_st = (double*)c->io;
    double* d_avg = d_st + 5 * (size_t)B;
    double* d_X = d_avg + nav;
    double* d_U = d_X + nX;
    double* d_S = d_U + nU;
    int* d_N = (int*)(d_S + nS);
    int* d_fin = d_N + slots;
    int* d_status = d_fin + slots;
    int* d_iters = d_status + slots;
    int* d_sqp = d_iters + slots;
    int* d_nch = d_sqp + slots;
    if (hipMemcpy(d_st, starts, sizeof(double) * 5 * B, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_avg, avg, sizeof(double) * nav, hipMemcpyHostToDevice) != hipSuccess)
        return fail(PLAN_E_DEVICE, "input upload failed");
    int rc = plan_optimize_device(c, B, Nmax, d_st, max_chunk_size, max_chunks, d_avg, nav, d_X, d_U, d_S, d_N,
                                  d_fin, d_status, d_iters, d_sqp, d_nch, nullptr);
    if (rc != PLAN_SUCCESS) return rc;
    if (hipError_t e = hipDeviceSynchronize(); e != hipSuccess)
        return fail(PLAN_E_DEVICE, std::string("plan loop kernel failed: ") + hipGetErrorString(e));
    const bool ok = hipMemcpy(X, d_X, sizeof(double) * nX, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(U, d_U, sizeof(double) * nU, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(S, d_S, sizeof(double) * nS, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(N, d_N, sizeof(int) * slots, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(is_final, d_fin, sizeof(int) * slots, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(status, d_status, sizeof(int) * slots, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(iters, d_iters, sizeof(int) * slots, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(sqp, d_sqp, sizeof(int) * slots, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(nchunks, d_nch, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess;
    if (!ok) return fail(PLAN_E_DEVICE, "output download failed");
    return PLAN_SUCCESS;
}

int plan_route_eval(plan_ctx* c, int n, const double* s, double* kappa, double* dkappa, double* vmax) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (n < 0 || (n > 0 && (!s || !kappa || !dkappa || !vmax))) return fail(PLAN_E_ARG, "bad arguments");
    if (n == 0) return PLAN_SUCCESS;
    if (c->host) {
        for (int i = 0; i < n; ++i) {
            kappa[i] = plan_host::route_kappa_at(c->host, s[i], &dkappa[i]);
            vmax[i] = plan_host::route_vmax_at(c->host, s[i]);
        }
        return PLAN_SUCCESS;
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * 4 * (size_t)n) != hipSuccess) return fail(PLAN_E_ALLOC, "allocation failed");
    int rc = PLAN_SUCCESS;
    if (hipMemcpy(d, s, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(PLAN_E_DEVICE, "upload failed");
    if (rc == PLAN_SUCCESS) {
        hipLaunchKernelGGL(route_eval_kernel, dim3((n + 255) / 256), dim3(256), 0, nullptr, c->R, n, d, d + n, d + 2 * n,
                           d + 3 * n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = fail(PLAN_E_LAUNCH, "route kernel failed");
    }
    if (rc == PLAN_SUCCESS &&
        (hipMemcpy(kappa, d + n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(dkappa, d + 2 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(vmax, d + 3 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = fail(PLAN_E_DEVICE, "download failed");
    (void)hipFree(d);
    return rc;
}

#ifdef PLAN_PROF
// diagnostic build only: summed s_memtime ticks per phase ([0, PH_COUNT)) and the chunk count ([15])
int plan_debug_prof(unsigned long long* out, int reset) {
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plan_prof), sizeof(unsigned long long) * 16) != hipSuccess)
        return fail(PLAN_E_DEVICE, "profile read failed");
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_plan_prof), z, sizeof(z)) != hipSuccess)
            return fail(PLAN_E_DEVICE, "profile reset failed");
    }
    return PLAN_SUCCESS;
}
#endif

}  // extern "C"
