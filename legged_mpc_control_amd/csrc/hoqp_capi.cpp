// hoqp_capi.cpp -- C-ABI (include/lmpc/lmpc_hoqp.h) over the batched hierarchical-QP kernel (lmpc_hoqp.hip).
//
// Replaces the reference's per-robot chain of HoQp objects (HoQp.cpp:15-27, one qpOASES QProblem per level)
// built by Wbc::update (wbc.cpp:93-99): a context owns the device staging buffers and the per-instance
// scratch; callers own their buffers; nothing is retained after a call returns.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "lmpc/lmpc_hoqp.h"
#include "lmpc_hoqp_device.h"

namespace lmpc {
hipError_t launch_hoqp(const HoqpDev& P, const double* rec, int batch, double* x, double* w, int32_t* status,
                       int32_t* iters, double* zout, int32_t* zcols, double* scratch, hipStream_t stream);
}

struct lmpc_hoqp_ctx {
    int device = 0;
    int max_batch = 0;
    lmpc::HoqpDev P{};
    hipStream_t stream = nullptr;
    double* d_rec = nullptr;    // host path staging: records
    double* d_out = nullptr;    // host path staging: x | slack
    int32_t* d_st = nullptr;    // host path staging: status | iters
    double* d_scratch = nullptr;  // per-instance Z, Z', A'A, grown on demand
    size_t scratch_inst = 0;
    double* d_z = nullptr;      // host path staging: stacked Z matrices + column counts (allocated on first use)
    int32_t* d_zc = nullptr;
    // orders launches that share d_scratch across streams: recorded on the last launch's stream only when the next
    // one comes on another stream (as lmpc_capi.cpp, round 6: back-to-back launches on one stream pay no event);
    // host-side waits (scratch growth, lmpc_hoqp_sync, lmpc_hoqp_destroy) wait for the device instead
    hipEvent_t ev = nullptr;
    hipStream_t ev_stream = nullptr;
    bool ev_live = false;
    hipStream_t last = nullptr;
    bool pend = false;
};

namespace {

struct DeviceScope {
    int prev = -1;
    bool ok = false;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
            return;
        }
        ok = prev == dev || hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

void fill_dev(lmpc::HoqpDev& P, const lmpc_hoqp_dims* d);

bool dims_ok(const lmpc_hoqp_dims* d) {
    if (!d || d->num_vars < 1 || d->num_vars > LMPC_HOQP_MAX_VARS || d->num_levels < 1 ||
        d->num_levels > LMPC_HOQP_MAX_LEVELS)
        return false;
    int stacked = 0;
    for (int l = 0; l < d->num_levels; ++l) {
        if (d->eq_rows[l] < 0 || d->eq_rows[l] > LMPC_HOQP_MAX_ROWS || d->ineq_rows[l] < 0 ||
            d->ineq_rows[l] > LMPC_HOQP_MAX_ROWS)
            return false;
        stacked += d->ineq_rows[l];
        if (stacked > LMPC_HOQP_MAX_STACKED) return false;
    }
    lmpc::HoqpDev P;  // one chain's LDS block (constraint rows + K, lmpc_hoqp.hip) must fit one workgroup
    fill_dev(P, d);
    return lmpc::hq_lds_doubles(P) * sizeof(double) <= (size_t)LMPC_HOQP_MAX_LDS_BYTES;
}

void fill_dev(lmpc::HoqpDev& P, const lmpc_hoqp_dims* d) {
    std::memset(&P, 0, sizeof(P));
    P.n = d->num_vars;
    P.np = (P.n + 15) & ~15;
    P.nt = P.np / 16;
    P.L = d->num_levels;
    int64_t off = 0;
    int stacked = 0, mmax = 0;
    P.rmax = 1;
    for (int l = 0; l < P.L; ++l) {
        P.m[l] = d->eq_rows[l];
        P.s[l] = d->ineq_rows[l];
        P.off[l] = off;
        off += (int64_t)(P.m[l] + P.s[l]) * (P.n + 1);
        stacked += P.s[l];
        if (stacked > P.rmax) P.rmax = stacked;
        if (P.m[l] > mmax) mmax = P.m[l];
    }
    P.rec_len = off;
    P.slack_len = stacked;
    P.kmax = mmax > P.np ? mmax : P.np;
    P.scratch_len = 2 * (int64_t)P.n * P.np + 2 * (int64_t)P.np * P.np;  // Z, Z', Hy, crossover T
    lmpc_hoqp_options o;
    lmpc_hoqp_options_default(&o);
    P.max_iter = o.max_iter;
    P.tol_mu = o.tol_mu;
    P.tol_res = o.tol_res;
    P.crossover = o.crossover;
}

hipError_t ensure_scratch(lmpc_hoqp_ctx* c, int batch) {
    if ((size_t)batch <= c->scratch_inst) return hipSuccess;
    double* p = nullptr;
    hipError_t e = hipMalloc(&p, (size_t)batch * c->P.scratch_len * sizeof(double));
    if (e != hipSuccess) return e;
    if (c->d_scratch) {
        // an earlier launch on another stream may still use the old block
        if (c->pend) (void)hipDeviceSynchronize();
        else if (c->ev_live) (void)hipEventSynchronize(c->ev);
        c->pend = false;
        (void)hipFree(c->d_scratch);
    }
    c->d_scratch = p;
    c->scratch_inst = (size_t)batch;
    return hipSuccess;
}

bool stream_ok(hipStream_t s, int dev) {
    if (!s) return true;
    hipDevice_t d = -1;
    return hipStreamGetDevice(s, &d) == hipSuccess && d == dev;
}

hipError_t launch(lmpc_hoqp_ctx* c, const double* rec, int batch, double* x, double* w, int32_t* st, int32_t* it,
                  double* z, int32_t* zc, hipStream_t s) {
    hipError_t e = ensure_scratch(c, batch);
    if (e != hipSuccess) return e;
    if (c->pend && c->last != s) {
        e = hipEventRecord(c->ev, c->last);
        c->pend = false;
        c->ev_stream = c->last;
        c->ev_live = e == hipSuccess;
        if (e != hipSuccess) return e;
    }
    if (!(c->pend && c->last == s) && c->ev_live && c->ev_stream != s && (e = hipStreamWaitEvent(s, c->ev, 0)) != hipSuccess)
        return e;
    e = lmpc::launch_hoqp(c->P, rec, batch, x, w, st, it, z, zc, c->d_scratch, s);
    if (e != hipSuccess) return e;
    c->last = s;
    c->pend = true;
    return e;
}

}  // namespace

extern "C" {

void lmpc_hoqp_dims_wbc(lmpc_hoqp_dims* d) {
    if (!d) return;
    std::memset(d, 0, sizeof(*d));
    d->num_vars = 42;  // wbc.h:18 -- 18 generalized accelerations, 12 contact forces, 12 torques
    d->num_levels = 3;
    d->eq_rows[0] = 30;   // EoM 18 + swing forces / no-contact motion 12 (wbc.cpp:93-94)
    d->ineq_rows[0] = 44; // torque limits 24 + friction pyramids 5 per leg (wbc.cpp:117-175)
    d->eq_rows[1] = 18;   // base acceleration 6 + swing legs <= 12 (wbc.cpp:95)
    d->eq_rows[2] = 12;   // contact forces (wbc.cpp:96)
}

void lmpc_hoqp_options_default(lmpc_hoqp_options* o) {
    if (!o) return;
    o->max_iter = 60;
    o->tol_mu = 1e-13;
    o->tol_res = 1e-7;
    o->crossover = 1;
}

int64_t lmpc_hoqp_lds_bytes(const lmpc_hoqp_dims* d) {
    if (!d || d->num_vars < 1 || d->num_vars > LMPC_HOQP_MAX_VARS || d->num_levels < 1 ||
        d->num_levels > LMPC_HOQP_MAX_LEVELS)
        return LMPC_ERR_ARG;
    lmpc::HoqpDev P;
    fill_dev(P, d);
    return (int64_t)(lmpc::hq_lds_doubles(P) * sizeof(double));
}

int64_t lmpc_hoqp_record_len(const lmpc_hoqp_dims* d) {
    if (!dims_ok(d)) return LMPC_ERR_ARG;
    int64_t len = 0;
    for (int l = 0; l < d->num_levels; ++l) len += (int64_t)(d->eq_rows[l] + d->ineq_rows[l]) * (d->num_vars + 1);
    return len;
}

int lmpc_hoqp_slack_len(const lmpc_hoqp_dims* d) {
    if (!dims_ok(d)) return LMPC_ERR_ARG;
    int s = 0;
    for (int l = 0; l < d->num_levels; ++l) s += d->ineq_rows[l];
    return s;
}

int lmpc_hoqp_create(const lmpc_hoqp_dims* d, int max_batch, int device, lmpc_hoqp_ctx** out) {
    if (!out) return LMPC_ERR_ARG;
    *out = nullptr;
    if (!dims_ok(d) || max_batch < 1) return LMPC_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LMPC_ERR_DEVICE;
    DeviceScope scope(device);
    if (!scope.ok) return LMPC_ERR_DEVICE;
    lmpc_hoqp_ctx* c = new (std::nothrow) lmpc_hoqp_ctx();
    if (!c) return LMPC_ERR_ALLOC;
    c->device = device;
    c->max_batch = max_batch;
    fill_dev(c->P, d);
    const size_t rec = (size_t)max_batch * c->P.rec_len, outd = (size_t)max_batch * (c->P.L * c->P.n + c->P.slack_len);
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) == hipSuccess &&
              hipMalloc(&c->d_rec, rec * sizeof(double)) == hipSuccess &&
              hipMalloc(&c->d_out, outd * sizeof(double)) == hipSuccess &&
              hipMalloc(&c->d_st, (size_t)max_batch * (1 + c->P.L) * sizeof(int32_t)) == hipSuccess &&
              ensure_scratch(c, max_batch) == hipSuccess;
    if (!ok) {
        lmpc_hoqp_destroy(c);
        return LMPC_ERR_ALLOC;
    }
    *out = c;
    return LMPC_OK;
}

void lmpc_hoqp_destroy(lmpc_hoqp_ctx* c) {
    if (!c) return;
    DeviceScope scope(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->pend && c->last != c->stream) (void)hipDeviceSynchronize();  // its stream may be gone by now
    else if (c->ev_live) (void)hipEventSynchronize(c->ev);
    (void)hipFree(c->d_rec);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_st);
    (void)hipFree(c->d_scratch);
    (void)hipFree(c->d_z);
    (void)hipFree(c->d_zc);
    if (c->ev) (void)hipEventDestroy(c->ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int lmpc_hoqp_set_options(lmpc_hoqp_ctx* c, const lmpc_hoqp_options* o) {
    if (!c || !o || o->max_iter < 1 || !(o->tol_mu > 0.0) || !(o->tol_res > 0.0) || o->crossover < 0 ||
        o->crossover > 1)
        return LMPC_ERR_ARG;
    c->P.max_iter = o->max_iter;
    c->P.tol_mu = o->tol_mu;
    c->P.tol_res = o->tol_res;
    c->P.crossover = o->crossover;
    return LMPC_OK;
}

int lmpc_hoqp_solve_batch_z(lmpc_hoqp_ctx* c, const double* tasks, int batch, double* x, double* slack,
                            int32_t* status, int32_t* iters, double* z, int32_t* zcols) {
    if (!c || batch < 0 || batch > c->max_batch) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    if (!tasks || !x || (!slack && c->P.slack_len > 0)) return LMPC_ERR_ARG;
    DeviceScope scope(c->device);
    if (!scope.ok) return LMPC_ERR_DEVICE;
    const size_t nx = (size_t)batch * c->P.L * c->P.n, nw = (size_t)batch * c->P.slack_len;
    const size_t nz = (size_t)c->max_batch * c->P.L * c->P.n * c->P.n;
    if (z && !c->d_z) {  // staging for the stacked Z matrices, on first use (max_batch x levels x n x n)
        if (hipMalloc(&c->d_z, nz * sizeof(double)) != hipSuccess ||
            hipMalloc(&c->d_zc, (size_t)c->max_batch * c->P.L * sizeof(int32_t)) != hipSuccess) {
            (void)hipFree(c->d_z);
            c->d_z = nullptr;
            return LMPC_ERR_ALLOC;
        }
    }
    double* d_x = c->d_out;
    double* d_w = c->d_out + nx;
    int32_t* d_status = c->d_st;
    int32_t* d_iters = c->d_st + batch;
    hipStream_t s = c->stream;
    // a device-path launch still pending on a caller's stream: wait for the device (that stream may be gone)
    if (c->pend && c->last != s) {
        if (hipDeviceSynchronize() != hipSuccess) return LMPC_ERR_DEVICE;
        c->pend = false;
        c->ev_live = false;
    }
    if (hipMemcpyAsync(c->d_rec, tasks, (size_t)batch * c->P.rec_len * sizeof(double), hipMemcpyHostToDevice, s) !=
        hipSuccess)
        return LMPC_ERR_DEVICE;
    if (launch(c, c->d_rec, batch, d_x, d_w, d_status, d_iters, z ? c->d_z : nullptr, z ? c->d_zc : nullptr, s) !=
        hipSuccess)
        return LMPC_ERR_LAUNCH;
    bool ok = hipMemcpyAsync(x, d_x, nx * sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess;
    if (nw) ok = ok && hipMemcpyAsync(slack, d_w, nw * sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess;
    if (status) ok = ok && hipMemcpyAsync(status, d_status, batch * sizeof(int32_t), hipMemcpyDeviceToHost, s) == hipSuccess;
    if (iters)
        ok = ok && hipMemcpyAsync(iters, d_iters, (size_t)batch * c->P.L * sizeof(int32_t), hipMemcpyDeviceToHost, s) ==
                       hipSuccess;
    if (z)
        ok = ok && hipMemcpyAsync(z, c->d_z, (size_t)batch * c->P.L * c->P.n * c->P.n * sizeof(double),
                                  hipMemcpyDeviceToHost, s) == hipSuccess;
    if (z && zcols)
        ok = ok && hipMemcpyAsync(zcols, c->d_zc, (size_t)batch * c->P.L * sizeof(int32_t), hipMemcpyDeviceToHost, s) ==
                       hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    return ok ? LMPC_OK : LMPC_ERR_DEVICE;
}

int lmpc_hoqp_solve_batch(lmpc_hoqp_ctx* c, const double* tasks, int batch, double* x, double* slack,
                          int32_t* status, int32_t* iters) {
    return lmpc_hoqp_solve_batch_z(c, tasks, batch, x, slack, status, iters, nullptr, nullptr);
}

int lmpc_hoqp_solve_device_z(lmpc_hoqp_ctx* c, const double* d_tasks, int batch, double* d_x, double* d_slack,
                             int32_t* d_status, int32_t* d_iters, double* d_z, int32_t* d_zcols, void* stream) {
    if (!c || batch < 0) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    if (!d_tasks || !d_x || (!d_slack && c->P.slack_len > 0) || (d_zcols && !d_z)) return LMPC_ERR_ARG;
    DeviceScope scope(c->device);
    if (!scope.ok) return LMPC_ERR_DEVICE;
    hipStream_t s = (hipStream_t)stream;
    if (!stream_ok(s, c->device)) return LMPC_ERR_ARG;
    double* w = d_slack ? d_slack : c->d_out;  // no inequality rows: the kernel writes no slack
    return launch(c, d_tasks, batch, d_x, w, d_status, d_iters, d_z, d_zcols, s) == hipSuccess ? LMPC_OK
                                                                                                  : LMPC_ERR_LAUNCH;
}

int lmpc_hoqp_solve_device(lmpc_hoqp_ctx* c, const double* d_tasks, int batch, double* d_x, double* d_slack,
                           int32_t* d_status, int32_t* d_iters, void* stream) {
    return lmpc_hoqp_solve_device_z(c, d_tasks, batch, d_x, d_slack, d_status, d_iters, nullptr, nullptr, stream);
}

int lmpc_hoqp_sync(lmpc_hoqp_ctx* c) {
    if (!c) return LMPC_ERR_ARG;
    DeviceScope scope(c->device);
    if (!scope.ok) return LMPC_ERR_DEVICE;
    bool ok = hipStreamSynchronize(c->stream) == hipSuccess;
    if (c->pend && c->last != c->stream) ok = ok && hipDeviceSynchronize() == hipSuccess;
    else if (c->ev_live) ok = ok && hipEventSynchronize(c->ev) == hipSuccess;
    return ok ? LMPC_OK : LMPC_ERR_DEVICE;
}

}  // extern "C"
