// lmpc_capi.cpp -- C-ABI (include/lmpc/lmpc.h) over the HIP solve kernel.
//
// Replaces the reference's ConvexQPSolver/OSQP object lifetime
// (ConvexQPSolver.cpp:16-196 construction, :314-327 compute_grfs):
// a context owns the device staging buffers and a HIP stream; callers own
// their host buffers; nothing is retained after a call returns.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"

namespace lmpc {
hipError_t launch_qp(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                     int batch, double* grf, int32_t* status, int32_t* iters, double* scratch, const uint8_t* done,
                     hipStream_t stream);
hipError_t launch_lq(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals, int batch,
                     double* grf, int32_t* status, int32_t* iters, const uint8_t* done, hipStream_t stream);
hipError_t launch_gi(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                     int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream);
hipError_t launch_dense(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                        int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream);
hipError_t launch_dense_lq(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                           int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream);
hipError_t launch_records(const lmpc_command* cmd, int batch, int H, double dt, double* rec, uint8_t* contact,
                          hipStream_t stream);
hipError_t launch_synth(const lmpc_synth_cfg& cfg, uint64_t seed, int64_t first, int count, lmpc_command* cmd,
                        hipStream_t stream);
hipError_t launch_normals(uint64_t seed, int64_t first, int count, double theta_max, double* normals,
                          hipStream_t stream);
hipError_t launch_torque(const lmpc_leg_kin& kin, const double* rec, const double* joint_pos, const double* grf,
                         int batch, int H, double* tau, hipStream_t stream);
}

struct lmpc_ctx {
    int device = 0;
    int H = 0;
    int max_batch = 0;
    lmpc::DevParams prm{};
    hipStream_t stream = nullptr;
    // host-pointer path (lmpc_solve_batch[_ex]): one device block in [rec | normals | contact] and one out
    // [grf | status | iters], each mirrored by a pinned host block, so a call is one H2D and one D2H copy
    // (per-tick latency: each separate pageable copy costs its own round of driver staging)
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* h_in = nullptr;
    uint8_t* h_out = nullptr;
    int riccati = LMPC_RICCATI_LDS;  // the Riccati kernel of cold solves (lmpc_set_riccati_path)
    double* d_scratch = nullptr;  // per-QP Riccati factors (L^-1, V, K, P2) of the scratch kernel, grown on demand
    uint8_t* d_done = nullptr;    // per-QP flag: solved by the dense-path kernel (else the Riccati kernel solves it)
    size_t scratch_qps = 0;
    size_t done_qps = 0;
    double* d_crec = nullptr;     // records expanded from commands (lmpc_solve_commands_device), grown on demand
    uint8_t* d_ccon = nullptr;
    size_t cmd_qps = 0;
    // Ordering of the context's own buffers (d_scratch, d_done, the staging blocks, d_crec/d_ccon) across
    // streams: a launch that uses them notes its stream (ctx_leave); the next such launch on another stream
    // records `ev` on the noted stream then and waits on it (ctx_enter); a host-pointer call, lmpc_sync and
    // lmpc_destroy wait for the device instead (the noted stream may be gone by then).  Calls on one stream pay
    // no event: recording one after every launch cost config 2 ~3 us per step (1.8 %, round 6,
    // profiles/r06/overhead/).
    hipEvent_t ev = nullptr;
    hipStream_t ev_stream = nullptr;  // where ev was last recorded
    bool ev_live = false;
    hipStream_t last = nullptr;       // stream of the last launch that used the buffers, not yet fenced
    bool pend = false;
};

namespace {

void fill_params(lmpc::DevParams& d, const lmpc_params* p) {
    for (int i = 0; i < 12; ++i) {
        d.q[i] = p->q_weights[i];
        d.r[i] = p->r_weights[i];
    }
    d.mass = p->robot_mass;
    for (int i = 0; i < 9; ++i) d.Ib[i] = p->trunk_inertia[i];
    d.mu = p->mu;
    d.fmax = p->f_max;
    d.grav = p->gravity;
    d.dt = p->dt;
}

void fill_options(lmpc::DevParams& d, const lmpc_options* o) {
    d.max_iter = o->max_iter;
    d.max_rounds = o->max_rounds;
    d.max_attempts = o->max_attempts;
    d.tol_mu = o->tol_mu;
    d.tol_p = o->tol_p;
    d.tol_d = o->tol_d;
    d.gi_max_steps = o->gi_max_steps;
    d.dense_iter_cap = o->dense_iter_cap > 0 ? o->dense_iter_cap : (1 << 30);  // 0: never hand over
    d.dense_polish_iter = o->dense_polish_iter;
    d.warm_rounds = o->warm_rounds;
    d.tol_x = o->tol_x;
}

bool params_ok(const lmpc_params* p) {
    if (!p) return false;
    if (!(p->robot_mass > 0.0) || !(p->dt > 0.0) || !(p->mu > 0.0) || !(p->f_max >= 0.0)) return false;
    for (int i = 0; i < 12; ++i)
        if (!(p->r_weights[i] > 0.0) || !(p->q_weights[i] >= 0.0)) return false;  // R > 0: strictly convex
    return true;
}

// staging block sizes of the host-pointer path (bytes)
size_t in_bytes(int H, int batch) {  // rec | normals | contact | warm-start active set
    return (size_t)batch * ((size_t)lmpc_record_len(H) * sizeof(double) + 12 * sizeof(double) + 8 * (size_t)H);
}
size_t out_bytes(int H, int batch) {  // grf | status | iters | dense-path hand-over flags | active set out
    return (size_t)batch * (12 * (size_t)H * sizeof(double) + 2 * sizeof(int32_t) + 1 + 4 * (size_t)H);
}

// Every entry point runs on the context's device and leaves the caller's current device as it found it.
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

// A caller's stream must belong to the context's device (the null stream is the current device's, which
// DeviceScope has just made the context's).
bool stream_ok(hipStream_t s, int dev) {
    if (!s) return true;
    hipDevice_t d = -1;
    return hipStreamGetDevice(s, &d) == hipSuccess && d == dev;
}

// Launches that use the context's buffers are ordered as issued, whatever stream each comes on.  ctx_leave notes
// the launch's stream; ctx_enter, before a launch on stream s, records the event on a noted launch's stream when s
// differs (everything issued there so far precedes it) and makes s wait for it.  A launch on the noted stream needs
// nothing: stream order already holds.
hipError_t ctx_enter(lmpc_ctx* c, hipStream_t s) {
    if (c->pend) {
        if (c->last == s) return hipSuccess;
        const hipError_t e = hipEventRecord(c->ev, c->last);
        c->pend = false;
        c->ev_stream = c->last;
        c->ev_live = e == hipSuccess;
        if (e != hipSuccess) return e;
    }
    if (c->ev_live && c->ev_stream != s) return hipStreamWaitEvent(s, c->ev, 0);
    return hipSuccess;
}
hipError_t ctx_leave(lmpc_ctx* c, hipStream_t s) {
    c->last = s;
    c->pend = true;
    return hipSuccess;
}
// Wait on the host for the last launch that used the context's buffers (its stream may have been destroyed since:
// the device as a whole, which is rare -- a host-pointer call after device-path calls on another stream, lmpc_sync,
// lmpc_destroy).
hipError_t ctx_wait_host(lmpc_ctx* c, hipStream_t s) {
    if (c->pend && c->last != s) {
        const hipError_t e = hipDeviceSynchronize();
        c->pend = false;
        return e;
    }
    if (c->ev_live && c->ev_stream != s) return hipEventSynchronize(c->ev);
    return hipSuccess;
}

void free_bufs(lmpc_ctx* c) {
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipHostFree(c->h_in);
    (void)hipHostFree(c->h_out);
    (void)hipFree(c->d_scratch);
    (void)hipFree(c->d_done);
    c->d_scratch = nullptr;
    c->d_done = nullptr;
    c->scratch_qps = 0;
    c->done_qps = 0;
    (void)hipFree(c->d_crec);
    (void)hipFree(c->d_ccon);
    c->d_crec = nullptr;
    c->d_ccon = nullptr;
    c->cmd_qps = 0;
    c->d_in = c->d_out = c->h_in = c->h_out = nullptr;
}

// The per-QP device buffers of a batch: the dense path's hand-over flags (always) and, when the scratch Riccati
// kernel runs (selected, or a warm start), its factor workspace.  Grown, never shrunk; a buffer in use by a queued
// launch is waited for before it is freed.
int ensure_ws(lmpc_ctx* c, int batch, bool scratch) {
    const bool grow_done = (size_t)batch > c->done_qps, grow_scr = scratch && (size_t)batch > c->scratch_qps;
    if (!grow_done && !grow_scr) return LMPC_OK;
    DeviceScope ds(c->device);
    if (!ds.ok) return LMPC_ERR_DEVICE;
    if (c->d_done || c->d_scratch) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipDeviceSynchronize();  // queued launches on callers' streams may still read the old buffers
    }
    if (grow_done) {
        (void)hipFree(c->d_done);
        c->d_done = nullptr;
        c->done_qps = 0;
        if (hipMalloc(&c->d_done, (size_t)batch) != hipSuccess) {
            c->d_done = nullptr;
            return LMPC_ERR_ALLOC;
        }
        c->done_qps = (size_t)batch;
    }
    if (grow_scr) {
        (void)hipFree(c->d_scratch);
        c->d_scratch = nullptr;
        c->scratch_qps = 0;
        if (hipMalloc(&c->d_scratch, (size_t)batch * lmpc::scratch_doubles_per_qp(c->H) * sizeof(double)) != hipSuccess) {
            c->d_scratch = nullptr;
            return LMPC_ERR_ALLOC;
        }
        c->scratch_qps = (size_t)batch;
    }
    return LMPC_OK;
}

// The Riccati kernel of a cold solve: the LDS-resident one (lmpc_lq.hip) or the scratch one (lmpc_kernels.hip,
// which needs the per-QP global workspace).
bool uses_scratch(const lmpc_ctx* c, const lmpc::DevParams& prm) {
    return c->riccati != LMPC_RICCATI_LDS || prm.warm_act || prm.act_out;
}

hipError_t launch_riccati(const lmpc_ctx* c, const lmpc::DevParams& prm, const double* rec, const uint8_t* con,
                          const double* nrm, int batch, double* grf, int32_t* st, int32_t* it, const uint8_t* done,
                          hipStream_t s) {
    if (!uses_scratch(c, prm)) return lmpc::launch_lq(prm, rec, con, nrm, batch, grf, st, it, done, s);
    return lmpc::launch_qp(prm, rec, con, nrm, batch, grf, st, it, c->d_scratch, done, s);
}

}  // namespace

extern "C" {

int lmpc_create(const lmpc_params* p, int horizon, int max_batch, int device, lmpc_ctx** out) {
    if (!out || !params_ok(p) || horizon < 1 || horizon > LMPC_MAX_HORIZON || max_batch < 0) return LMPC_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LMPC_ERR_DEVICE;
    DeviceScope ds(device);
    if (!ds.ok) return LMPC_ERR_DEVICE;
    lmpc_ctx* c = new (std::nothrow) lmpc_ctx();
    if (!c) return LMPC_ERR_ALLOC;
    c->device = device;
    c->H = horizon;
    c->max_batch = max_batch;
    fill_params(c->prm, p);
    lmpc_options o;
    lmpc_options_default(&o);
    fill_options(c->prm, &o);
    c->prm.H = horizon;
    // condensed dense path for H <= DENSE_MAX_H: the interior point (lmpc_dense.hip) by default;
    // lmpc_set_dense_path selects the dual active set (lmpc_gi.hip) or the Riccati kernel for every QP.
    // The choice is fixed per context, never per launch, so a QP's answer does not depend on the batch it
    // is solved in.  Why the interior point is the default: DESIGN.md 4b.
    c->prm.dense = horizon > lmpc::DENSE_MAX_H ? 0 : 1;
    if (hipDeviceGetAttribute(&c->prm.cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        c->prm.cus = 256;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return LMPC_ERR_DEVICE;
    }
    if (hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LMPC_ERR_DEVICE;
    }
    if (max_batch > 0) {
        const size_t in_b = in_bytes(horizon, max_batch), out_b = out_bytes(horizon, max_batch);
        bool ok = hipMalloc(&c->d_in, in_b) == hipSuccess && hipMalloc(&c->d_out, out_b) == hipSuccess &&
                  hipHostMalloc(&c->h_in, in_b, hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc(&c->h_out, out_b, hipHostMallocDefault) == hipSuccess;
        if (!ok) {
            free_bufs(c);
            (void)hipEventDestroy(c->ev);
            (void)hipStreamDestroy(c->stream);
            delete c;
            return LMPC_ERR_ALLOC;
        }
    }
    if (max_batch > 0 && ensure_ws(c, max_batch, c->riccati == LMPC_RICCATI_SCRATCH) != LMPC_OK) {
        free_bufs(c);
        (void)hipEventDestroy(c->ev);
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LMPC_ERR_ALLOC;
    }
    *out = c;
    return LMPC_OK;
}

void lmpc_destroy(lmpc_ctx* c) {
    if (!c) return;
    DeviceScope ds(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)ctx_wait_host(c, c->stream);  // the last launch on a caller's stream
    free_bufs(c);
    if (c->ev) (void)hipEventDestroy(c->ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int lmpc_set_options(lmpc_ctx* c, const lmpc_options* o) {
    if (!c || !o || o->max_iter < 1 || o->max_rounds < 1 || o->max_attempts < 1 || !(o->tol_mu > 0.0) ||
        !(o->tol_p >= 0.0) || !(o->tol_d >= 0.0) || !(o->tol_x >= 0.0) || o->gi_max_steps < 1 || o->dense_iter_cap < 0 ||
        o->dense_polish_iter < 1 || o->warm_rounds < 1)
        return LMPC_ERR_ARG;
    fill_options(c->prm, o);
    return LMPC_OK;
}

int lmpc_set_params(lmpc_ctx* c, const lmpc_params* p) {
    if (!c || !params_ok(p)) return LMPC_ERR_ARG;
    fill_params(c->prm, p);
    return LMPC_OK;
}

int lmpc_set_dense_path(lmpc_ctx* c, int path) {
    if (!c || path < LMPC_DENSE_OFF || path > LMPC_DENSE_GI) return LMPC_ERR_ARG;
    if (c->H <= lmpc::DENSE_MAX_H) c->prm.dense = path;
    return LMPC_OK;
}

int lmpc_get_dense_path(const lmpc_ctx* c) { return c ? c->prm.dense : LMPC_ERR_ARG; }

int lmpc_set_riccati_path(lmpc_ctx* c, int path) {
    if (!c || (path != LMPC_RICCATI_SCRATCH && path != LMPC_RICCATI_LDS)) return LMPC_ERR_ARG;
    c->riccati = path;
    return LMPC_OK;
}

int lmpc_get_riccati_path(const lmpc_ctx* c) { return c ? c->riccati : LMPC_ERR_ARG; }

int lmpc_reserve(lmpc_ctx* c, int batch) {
    if (!c || batch < 0) return LMPC_ERR_ARG;
    return ensure_ws(c, batch, c->riccati == LMPC_RICCATI_SCRATCH);
}

int lmpc_reserve_warm(lmpc_ctx* c, int batch) {
    if (!c || batch < 0) return LMPC_ERR_ARG;
    return ensure_ws(c, batch, true);
}

int lmpc_solve_batch_device_ex(lmpc_ctx* c, const double* d_rec, const uint8_t* d_contact, const double* d_normals,
                               int batch, double* d_grf, int32_t* d_status, int32_t* d_iters, void* stream) {
    if (!c || batch < 0 || (batch > 0 && (!d_rec || !d_contact || !d_grf))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    DeviceScope ds(c->device);
    if (!ds.ok) return LMPC_ERR_DEVICE;
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream (ordered with blocking streams)
    if (!stream_ok(s, c->device)) return LMPC_ERR_ARG;
    {
        const int rc = ensure_ws(c, batch, uses_scratch(c, c->prm));
        if (rc != LMPC_OK) return rc;
    }
    hipError_t e = ctx_enter(c, s);
    // condensed dense kernel first; it flags the QPs it solved and the Riccati kernel solves the rest
    // (more than 20 stance leg-steps, or a dense QP left without a verified optimum).  At most one QP per SIMD
    // (both kernels one wave per SIMD) the two run as one launch, each QP's Riccati solve after its dense one in
    // the same wave (lmpc_dense_lq_kernel, the same arithmetic)
    bool fused = false;
    if (e == hipSuccess && c->prm.dense == 1 && !uses_scratch(c, c->prm)) {
        const hipError_t f = lmpc::launch_dense_lq(c->prm, d_rec, d_contact, d_normals, batch, d_grf, d_status,
                                                    d_iters, c->d_done, s);
        if (f == hipSuccess) fused = true;
        else if (f != hipErrorNotSupported) e = f;
    }
    if (!fused) {
        if (e == hipSuccess && c->prm.dense == 2)
            e = lmpc::launch_gi(c->prm, d_rec, d_contact, d_normals, batch, d_grf, d_status, d_iters, c->d_done, s);
        else if (e == hipSuccess && c->prm.dense == 1)
            e = lmpc::launch_dense(c->prm, d_rec, d_contact, d_normals, batch, d_grf, d_status, d_iters, c->d_done, s);
        if (e == hipSuccess)
            e = launch_riccati(c, c->prm, d_rec, d_contact, d_normals, batch, d_grf, d_status, d_iters,
                               c->prm.dense ? c->d_done : nullptr, s);
    }
    if (e == hipSuccess) e = ctx_leave(c, s);
    if (e == hipErrorInvalidDeviceFunction || e == hipErrorNoBinaryForGpu) return LMPC_ERR_NOT_BUILT;
    return e == hipSuccess ? LMPC_OK : LMPC_ERR_LAUNCH;
}

int lmpc_solve_batch_device(lmpc_ctx* c, const double* d_rec, const uint8_t* d_contact, int batch, double* d_grf,
                            int32_t* d_status, int32_t* d_iters, void* stream) {
    return lmpc_solve_batch_device_ex(c, d_rec, d_contact, nullptr, batch, d_grf, d_status, d_iters, stream);
}

static int launch_rc(hipError_t e);

// The host-pointer path: one pinned copy in, the kernels, one pinned copy out.  act_in / act_out (warm start,
// lmpc_solve_batch_warm): every QP goes to the Riccati kernel, which starts from act_in and reports act_out.
static int solve_host(lmpc_ctx* c, const double* rec, const uint8_t* contact, const double* normals, int batch,
                      const uint8_t* act_in, uint8_t* act_out, double* grf, int32_t* status, int32_t* iters) {
    if (!c || batch < 0 || batch > c->max_batch || (batch > 0 && (!rec || !contact || !grf))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    if (normals)
        for (size_t i = 0; i < (size_t)batch * 4; ++i) {
            const double* n = normals + 3 * i;
            if (!(n[2] > 0.0) || !std::isfinite(n[0]) || !std::isfinite(n[1]) || !std::isfinite(n[2]))
                return LMPC_ERR_ARG;
        }
    DeviceScope ds(c->device);
    if (!ds.ok) return LMPC_ERR_DEVICE;
    hipStream_t s = c->stream;
    const bool warm = act_in || act_out;
    lmpc::DevParams prm = c->prm;
    if (warm) prm.dense = 0;  // the dense kernels are not warm-started
    // inputs packed [rec | normals | contact | act_in] for THIS batch (offsets from `batch`: one contiguous copy)
    const size_t nrec = (size_t)batch * lmpc_record_len(c->H) * sizeof(double);
    const size_t nnrm = normals ? (size_t)batch * 12 * sizeof(double) : 0;
    const size_t ncon = (size_t)batch * 4 * c->H;
    const size_t nact = act_in ? ncon : 0;
    // the pinned staging blocks and the factor scratch may still be in use by an earlier asynchronous
    // device-path call on another stream: wait for it before the host writes the staging block
    if (ctx_wait_host(c, s) != hipSuccess) return LMPC_ERR_DEVICE;
    std::memcpy(c->h_in, rec, nrec);
    if (normals) std::memcpy(c->h_in + nrec, normals, nnrm);
    std::memcpy(c->h_in + nrec + nnrm, contact, ncon);
    if (act_in) std::memcpy(c->h_in + nrec + nnrm + ncon, act_in, nact);
    if (hipMemcpyAsync(c->d_in, c->h_in, nrec + nnrm + ncon + nact, hipMemcpyHostToDevice, s) != hipSuccess)
        return LMPC_ERR_DEVICE;
    const size_t ngrf = (size_t)batch * 12 * c->H * sizeof(double);
    const size_t nst = (size_t)batch * sizeof(int32_t);
    double* d_grf = (double*)c->d_out;
    int32_t* d_st = (int32_t*)(c->d_out + ngrf);
    uint8_t* d_done = c->d_out + ngrf + 2 * nst;  // dense-path hand-over flags travel back with the results
    uint8_t* d_aout = d_done + batch;
    const double* d_rec = (const double*)c->d_in;
    const uint8_t* d_con = c->d_in + nrec + nnrm;
    const double* d_nrm = normals ? (const double*)(c->d_in + nrec) : nullptr;
    prm.warm_act = act_in ? c->d_in + nrec + nnrm + ncon : nullptr;
    prm.act_out = act_out ? d_aout : nullptr;
    // The contact schedules are on the host, so this (synchronous) path launches only the kernels the batch
    // needs: the same routing as lmpc_solve_batch_device_ex, whose QPs skip the other kernel on the device.
    int n_dense = 0, n_ric = 0;
    for (int b = 0; b < batch; ++b) {
        const uint8_t* cb = contact + (size_t)b * 4 * c->H;
        int n = 0;
        for (int i = 0; i < 4 * c->H; ++i) n += cb[i] != 0;
        if (prm.dense && n >= 1 && n <= lmpc::DENSE_MAX_LS) ++n_dense;
        else ++n_ric;
    }
    const bool gi = prm.dense == 2;
    if (n_ric && ensure_ws(c, batch, uses_scratch(c, prm)) != LMPC_OK) return LMPC_ERR_ALLOC;
    hipError_t e = hipSuccess;
    if (n_dense)
        e = gi ? lmpc::launch_gi(prm, d_rec, d_con, d_nrm, batch, d_grf, d_st, d_st + batch, d_done, s)
               : lmpc::launch_dense(prm, d_rec, d_con, d_nrm, batch, d_grf, d_st, d_st + batch, d_done, s);
    if (e == hipSuccess && n_ric)
        e = launch_riccati(c, prm, d_rec, d_con, d_nrm, batch, d_grf, d_st, d_st + batch, prm.dense ? d_done : nullptr, s);
    if (e == hipSuccess) e = ctx_leave(c, s);
    if (e != hipSuccess) return launch_rc(e);
    // one copy back: [grf | status | iters], plus the hand-over flags (dense path) or the active set (warm)
    const size_t nout = act_out ? ngrf + 2 * nst + batch + ncon : ngrf + 2 * nst + (n_dense ? (size_t)batch : 0);
    if (hipMemcpyAsync(c->h_out, c->d_out, nout, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return LMPC_ERR_DEVICE;
    if (n_dense && !n_ric) {
        // a QP the dense kernel left (iteration or step cap, non-finite iterate) goes to the Riccati kernel,
        // as on the device path
        const uint8_t* hd = c->h_out + ngrf + 2 * nst;
        bool left = false;
        for (int b = 0; b < batch && !left; ++b) left = hd[b] == 0;
        if (left) {
            if (ensure_ws(c, batch, uses_scratch(c, prm)) != LMPC_OK) return LMPC_ERR_ALLOC;
            e = launch_riccati(c, prm, d_rec, d_con, d_nrm, batch, d_grf, d_st, d_st + batch, d_done, s);
            if (e == hipSuccess) e = ctx_leave(c, s);
            if (e != hipSuccess) return launch_rc(e);
            if (hipMemcpyAsync(c->h_out, c->d_out, ngrf + 2 * nst, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return LMPC_ERR_DEVICE;
        }
    }
    std::memcpy(grf, c->h_out, ngrf);
    if (status) std::memcpy(status, c->h_out + ngrf, nst);
    if (iters) std::memcpy(iters, c->h_out + ngrf + nst, nst);
    if (act_out) std::memcpy(act_out, c->h_out + ngrf + 2 * nst + batch, ncon);
    return LMPC_OK;
}

int lmpc_solve_batch_ex(lmpc_ctx* c, const double* rec, const uint8_t* contact, const double* normals, int batch,
                        double* grf, int32_t* status, int32_t* iters) {
    return solve_host(c, rec, contact, normals, batch, nullptr, nullptr, grf, status, iters);
}

int lmpc_solve_batch_warm(lmpc_ctx* c, const double* rec, const uint8_t* contact, const double* normals, int batch,
                          const uint8_t* act_in, uint8_t* act_out, double* grf, int32_t* status, int32_t* iters) {
    return solve_host(c, rec, contact, normals, batch, act_in, act_out, grf, status, iters);
}

void lmpc_shift_active_set(const uint8_t* act, int batch, int H, uint8_t* shifted) {
    if (!act || !shifted || batch <= 0 || H <= 0) return;
    for (int b = 0; b < batch; ++b) {
        const uint8_t* a = act + (size_t)b * 4 * H;
        uint8_t* o = shifted + (size_t)b * 4 * H;
        for (int k = 0; k < H; ++k)
            for (int j = 0; j < 4; ++j) o[4 * k + j] = a[4 * (k + 1 < H ? k + 1 : k) + j];
    }
}

int lmpc_solve_batch(lmpc_ctx* c, const double* rec, const uint8_t* contact, int batch, double* grf,
                     int32_t* status, int32_t* iters) {
    return lmpc_solve_batch_ex(c, rec, contact, nullptr, batch, grf, status, iters);
}

static int launch_rc(hipError_t e) {
    if (e == hipErrorInvalidDeviceFunction || e == hipErrorNoBinaryForGpu) return LMPC_ERR_NOT_BUILT;
    return e == hipSuccess ? LMPC_OK : LMPC_ERR_LAUNCH;
}

// Entry points that launch on the caller's stream without touching the context's buffers: device scope and
// stream check only.
#define LMPC_DEVICE_ENTRY(c, s)                         \
    DeviceScope ds_(c->device);                         \
    if (!ds_.ok) return LMPC_ERR_DEVICE;                \
    hipStream_t s = (hipStream_t)stream; /* NULL = the HIP null stream (ordered with blocking streams) */ \
    if (!stream_ok(s, c->device)) return LMPC_ERR_ARG

int lmpc_build_records_device(lmpc_ctx* c, const lmpc_command* d_cmd, int batch, double* d_rec, uint8_t* d_contact,
                              void* stream) {
    if (!c || batch < 0 || (batch > 0 && (!d_cmd || !d_rec || !d_contact))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    LMPC_DEVICE_ENTRY(c, s);
    return launch_rc(lmpc::launch_records(d_cmd, batch, c->H, c->prm.dt, d_rec, d_contact, s));
}

int lmpc_solve_commands_device(lmpc_ctx* c, const lmpc_command* d_cmd, const double* d_normals, int batch,
                               double* d_grf, int32_t* d_status, int32_t* d_iters, void* stream) {
    if (!c || batch < 0 || (batch > 0 && (!d_cmd || !d_grf))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    LMPC_DEVICE_ENTRY(c, s);
    if ((size_t)batch > c->cmd_qps) {
        (void)hipDeviceSynchronize();  // the old buffers may still be read by queued work
        (void)hipFree(c->d_crec);
        (void)hipFree(c->d_ccon);
        c->d_crec = nullptr;
        c->d_ccon = nullptr;
        c->cmd_qps = 0;
        if (hipMalloc(&c->d_crec, (size_t)batch * lmpc_record_len(c->H) * sizeof(double)) != hipSuccess ||
            hipMalloc(&c->d_ccon, (size_t)batch * 4 * c->H) != hipSuccess)
            return LMPC_ERR_ALLOC;
        c->cmd_qps = (size_t)batch;
    }
    // the expansion overwrites the context's record buffers: order it behind the previous solve that read them
    hipError_t e = ctx_enter(c, s);
    if (e == hipSuccess) e = lmpc::launch_records(d_cmd, batch, c->H, c->prm.dt, c->d_crec, c->d_ccon, s);
    if (e != hipSuccess) return launch_rc(e);
    return lmpc_solve_batch_device_ex(c, c->d_crec, c->d_ccon, d_normals, batch, d_grf, d_status, d_iters, s);
}

int lmpc_synth_commands_device(lmpc_ctx* c, const lmpc_synth_cfg* cfg, uint64_t seed, int64_t first_index, int count,
                               lmpc_command* d_cmd, void* stream) {
    if (!c || !cfg || count < 0 || (count > 0 && !d_cmd)) return LMPC_ERR_ARG;
    if (count == 0) return LMPC_OK;
    LMPC_DEVICE_ENTRY(c, s);
    return launch_rc(lmpc::launch_synth(*cfg, seed, first_index, count, d_cmd, s));
}

int lmpc_synth_normals_device(lmpc_ctx* c, uint64_t seed, int64_t first_index, int count, double theta_max,
                              double* d_normals, void* stream) {
    if (!c || count < 0 || (count > 0 && !d_normals) || !(theta_max >= 0.0) || theta_max >= 1.5707963267948966)
        return LMPC_ERR_ARG;
    if (count == 0) return LMPC_OK;
    LMPC_DEVICE_ENTRY(c, s);
    return launch_rc(lmpc::launch_normals(seed, first_index, count, theta_max, d_normals, s));
}

int lmpc_grf_to_torque_device(lmpc_ctx* c, const lmpc_leg_kin* k, const double* d_rec, const double* d_joint_pos,
                              const double* d_grf, int batch, double* d_tau, void* stream) {
    if (!c || !k || batch < 0 || (batch > 0 && (!d_rec || !d_joint_pos || !d_grf || !d_tau))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    LMPC_DEVICE_ENTRY(c, s);
    return launch_rc(lmpc::launch_torque(*k, d_rec, d_joint_pos, d_grf, batch, c->H, d_tau, s));
}
#undef LMPC_DEVICE_ENTRY

int lmpc_sync(lmpc_ctx* c) {
    if (!c) return LMPC_ERR_ARG;
    DeviceScope ds(c->device);
    if (!ds.ok) return LMPC_ERR_DEVICE;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return LMPC_ERR_DEVICE;
    // and the last launch that used the context's buffers, whatever stream it ran on
    return ctx_wait_host(c, c->stream) == hipSuccess ? LMPC_OK : LMPC_ERR_DEVICE;
}

}  // extern "C"
