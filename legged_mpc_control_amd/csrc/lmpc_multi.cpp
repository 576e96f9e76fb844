// lmpc_multi.cpp -- one host process driving several MI355X (include/lmpc/lmpc_multi.h).
//
// The batch is split into contiguous shards, one per device; each device runs the single-device
// C-ABI (lmpc.h: lmpc_solve_commands_device, the synthetic generators) on its shard, on a stream of its
// own.  RCCL moves only the batch scatter (commands, normals: root -> devices 1..R-1) and gather (GRFs,
// status, iteration words: devices -> root), each as one grouped ncclSend / ncclRecv, so
// every device sends over its own xGMI link to the root and nothing is relayed around a ring.
// Communicators come from ncclCommInitAll (one per device, single process): no bootstrap network.
//
// Reference: the single MPC thread of src/legged_ctrl/src/main.cpp:110-164 calls one solver object
// (ConvexQPSolver.h:25-38); this is the batched, multi-device form of that call.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <new>

#include "lmpc/lmpc.h"
#include "lmpc/lmpc_multi.h"

namespace {

struct Shard {
    uint8_t* cmd = nullptr;   // lmpc_command bytes (devices 1..R-1: scatter target; root: synthetic commands)
    double* nrm = nullptr;    // [count][4][3]
    double* grf = nullptr;    // [count][H][12] (devices 1..R-1 only; the root writes the caller's buffer)
    int32_t* st = nullptr;
    int32_t* it = nullptr;
    size_t cap = 0;           // QPs
};

}  // namespace

struct lmpc_multi {
    int n = 0;
    int H = 0;
    int dev[LMPC_MULTI_MAX_DEVICES] = {};
    lmpc_ctx* ctx[LMPC_MULTI_MAX_DEVICES] = {};
    ncclComm_t comm[LMPC_MULTI_MAX_DEVICES] = {};
    hipStream_t stream[LMPC_MULTI_MAX_DEVICES] = {};
    Shard buf[LMPC_MULTI_MAX_DEVICES];
    bool comms = false;
};

namespace {

struct DeviceScope {  // every entry point leaves the caller's current device as it found it
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

void free_shard(Shard& s) {
    (void)hipFree(s.cmd);
    (void)hipFree(s.nrm);
    (void)hipFree(s.grf);
    (void)hipFree(s.st);
    (void)hipFree(s.it);
    s = Shard{};
}

// grows device r's shard buffers to `count` QPs (contents are not kept)
int reserve(lmpc_multi* m, int r, size_t count) {
    Shard& s = m->buf[r];
    if (count <= s.cap) return LMPC_OK;
    DeviceScope ds(m->dev[r]);
    (void)hipStreamSynchronize(m->stream[r]);
    free_shard(s);
    const size_t H = (size_t)m->H;
    if (hipMalloc(&s.cmd, count * sizeof(lmpc_command)) != hipSuccess ||
        hipMalloc(&s.nrm, count * 12 * sizeof(double)) != hipSuccess ||
        hipMalloc(&s.grf, count * 12 * H * sizeof(double)) != hipSuccess ||
        hipMalloc(&s.st, count * sizeof(int32_t)) != hipSuccess || hipMalloc(&s.it, count * sizeof(int32_t)) != hipSuccess) {
        free_shard(s);
        return LMPC_ERR_ALLOC;
    }
    s.cap = count;
    return LMPC_OK;
}

int sync_all(lmpc_multi* m) {
    int rc = LMPC_OK;
    for (int r = 0; r < m->n; ++r) {
        DeviceScope ds(m->dev[r]);
        if (hipStreamSynchronize(m->stream[r]) != hipSuccess) rc = LMPC_ERR_DEVICE;
    }
    return rc;
}

// One grouped exchange between the root and every other device: for r >= 1, root buffer `root(r)` and
// device r's buffer `peer(r)`, `elems(r)` elements of `type`; to_root selects the direction (gather).
template <class RootPtr, class PeerPtr, class Elems>
int exchange(lmpc_multi* m, bool to_root, ncclDataType_t type, RootPtr root, PeerPtr peer, Elems elems) {
    if (m->n < 2) return LMPC_OK;
    if (ncclGroupStart() != ncclSuccess) return LMPC_ERR_COMM;
    ncclResult_t e = ncclSuccess;
    for (int r = 1; r < m->n && e == ncclSuccess; ++r) {
        const size_t cnt = elems(r);
        if (cnt == 0) continue;
        if (to_root) {
            e = ncclSend(peer(r), cnt, type, 0, m->comm[r], m->stream[r]);
            if (e == ncclSuccess) e = ncclRecv(root(r), cnt, type, r, m->comm[0], m->stream[0]);
        } else {
            e = ncclSend(root(r), cnt, type, r, m->comm[0], m->stream[0]);
            if (e == ncclSuccess) e = ncclRecv(peer(r), cnt, type, 0, m->comm[r], m->stream[r]);
        }
    }
    const ncclResult_t g = ncclGroupEnd();
    return e == ncclSuccess && g == ncclSuccess ? LMPC_OK : LMPC_ERR_COMM;
}

// Solve every shard from commands already on its device (root: d_cmd0 / d_nrm0 / outputs in place), then
// gather the outputs into the root's buffers.  Synchronous.
int solve_and_gather(lmpc_multi* m, int batch, const lmpc_command* d_cmd0, const double* d_nrm0, bool normals,
                     double* d_grf, int32_t* d_status, int32_t* d_iters) {
    const size_t H12 = 12 * (size_t)m->H;
    int rc = LMPC_OK;
    for (int r = 0; r < m->n && rc == LMPC_OK; ++r) {
        int first = 0, count = 0;
        lmpc_multi_shard(batch, m->n, r, &first, &count);
        if (count == 0) continue;
        if (r == 0) {
            rc = lmpc_solve_commands_device(m->ctx[0], d_cmd0, normals ? d_nrm0 : nullptr, count, d_grf, d_status,
                                            d_iters, m->stream[0]);
        } else {
            const Shard& s = m->buf[r];
            rc = lmpc_solve_commands_device(m->ctx[r], (const lmpc_command*)s.cmd, normals ? s.nrm : nullptr, count,
                                            s.grf, s.st, s.it, m->stream[r]);
        }
    }
    if (rc != LMPC_OK) {
        (void)sync_all(m);
        return rc;
    }
    auto first_of = [&](int r) {
        int f = 0, c = 0;
        lmpc_multi_shard(batch, m->n, r, &f, &c);
        return (size_t)f;
    };
    auto count_of = [&](int r) {
        int f = 0, c = 0;
        lmpc_multi_shard(batch, m->n, r, &f, &c);
        return (size_t)c;
    };
    rc = exchange(m, true, ncclFloat64, [&](int r) { return d_grf + first_of(r) * H12; },
                  [&](int r) { return m->buf[r].grf; }, [&](int r) { return count_of(r) * H12; });
    if (rc == LMPC_OK && d_status)
        rc = exchange(m, true, ncclInt32, [&](int r) { return d_status + first_of(r); },
                      [&](int r) { return m->buf[r].st; }, count_of);
    if (rc == LMPC_OK && d_iters)
        rc = exchange(m, true, ncclInt32, [&](int r) { return d_iters + first_of(r); },
                      [&](int r) { return m->buf[r].it; }, count_of);
    const int src = sync_all(m);
    return rc != LMPC_OK ? rc : src;
}

bool valid(const lmpc_multi* m) { return m && m->n >= 1 && m->comms; }

}  // namespace

extern "C" {

int lmpc_multi_abi_version(void) { return LMPC_MULTI_ABI_VERSION; }

void lmpc_multi_shard(int batch, int n_devices, int r, int* first, int* count) {
    if (!first || !count) return;
    *first = *count = 0;
    if (batch <= 0 || n_devices <= 0 || r < 0 || r >= n_devices) return;
    // [batch r / R, batch (r+1) / R): the split bench.py uses for a fixed global batch (dist.split_range)
    const int64_t lo = (int64_t)batch * r / n_devices, hi = (int64_t)batch * (r + 1) / n_devices;
    *first = (int)lo;
    *count = (int)(hi - lo);
}

int lmpc_multi_create(const lmpc_params* p, int horizon, const int* devices, int n_devices, lmpc_multi** out) {
    if (!out || !p || !devices || n_devices < 1 || n_devices > LMPC_MULTI_MAX_DEVICES) return LMPC_ERR_ARG;
    *out = nullptr;
    for (int i = 0; i < n_devices; ++i)
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j]) return LMPC_ERR_ARG;  // RCCL: one communicator rank per device
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return LMPC_ERR_DEVICE;
    for (int i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= ndev) return LMPC_ERR_DEVICE;
    lmpc_multi* m = new (std::nothrow) lmpc_multi();
    if (!m) return LMPC_ERR_ALLOC;
    m->n = n_devices;
    m->H = horizon;
    int rc = LMPC_OK;
    for (int r = 0; r < n_devices && rc == LMPC_OK; ++r) {
        m->dev[r] = devices[r];
        rc = lmpc_create(p, horizon, 0, devices[r], &m->ctx[r]);
        if (rc == LMPC_OK) {
            DeviceScope ds(devices[r]);
            if (hipStreamCreateWithFlags(&m->stream[r], hipStreamNonBlocking) != hipSuccess) rc = LMPC_ERR_DEVICE;
        }
    }
    if (rc == LMPC_OK) {
        if (ncclCommInitAll(m->comm, n_devices, devices) == ncclSuccess) m->comms = true;
        else rc = LMPC_ERR_COMM;
    }
    if (rc != LMPC_OK) {
        lmpc_multi_destroy(m);
        return rc;
    }
    *out = m;
    return LMPC_OK;
}

void lmpc_multi_destroy(lmpc_multi* m) {
    if (!m) return;
    for (int r = 0; r < m->n; ++r) {
        if (!m->dev[r] && !m->ctx[r] && !m->stream[r]) continue;
        DeviceScope ds(m->dev[r]);
        if (m->stream[r]) (void)hipStreamSynchronize(m->stream[r]);
        if (m->comms) (void)ncclCommDestroy(m->comm[r]);
        free_shard(m->buf[r]);
        if (m->stream[r]) (void)hipStreamDestroy(m->stream[r]);
        lmpc_destroy(m->ctx[r]);
    }
    delete m;
}

int lmpc_multi_num_devices(const lmpc_multi* m) { return m ? m->n : LMPC_ERR_ARG; }

int lmpc_multi_set_options(lmpc_multi* m, const lmpc_options* o) {
    if (!valid(m)) return LMPC_ERR_ARG;
    for (int r = 0; r < m->n; ++r) {
        const int rc = lmpc_set_options(m->ctx[r], o);
        if (rc != LMPC_OK) return rc;
    }
    return LMPC_OK;
}

int lmpc_multi_set_dense_path(lmpc_multi* m, int path) {
    if (!valid(m)) return LMPC_ERR_ARG;
    for (int r = 0; r < m->n; ++r) {
        const int rc = lmpc_set_dense_path(m->ctx[r], path);
        if (rc != LMPC_OK) return rc;
    }
    return LMPC_OK;
}

int lmpc_multi_solve_commands_device(lmpc_multi* m, const lmpc_command* d_cmd, const double* d_normals, int batch,
                                     double* d_grf, int32_t* d_status, int32_t* d_iters, void* stream) {
    if (!valid(m) || batch < 0 || (batch > 0 && (!d_cmd || !d_grf))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    DeviceScope ds(m->dev[0]);
    // the caller's inputs on devices[0] are complete before the scatter reads them
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return LMPC_ERR_DEVICE;
    for (int r = 1; r < m->n; ++r) {
        int first = 0, count = 0;
        lmpc_multi_shard(batch, m->n, r, &first, &count);
        const int rc = reserve(m, r, (size_t)count);
        if (rc != LMPC_OK) return rc;
    }
    auto first_of = [&](int r) {
        int f = 0, c = 0;
        lmpc_multi_shard(batch, m->n, r, &f, &c);
        return (size_t)f;
    };
    auto count_of = [&](int r) {
        int f = 0, c = 0;
        lmpc_multi_shard(batch, m->n, r, &f, &c);
        return (size_t)c;
    };
    int rc = exchange(m, false, ncclUint8, [&](int r) { return (uint8_t*)(d_cmd + first_of(r)); },
                      [&](int r) { return m->buf[r].cmd; }, [&](int r) { return count_of(r) * sizeof(lmpc_command); });
    if (rc == LMPC_OK && d_normals)
        rc = exchange(m, false, ncclFloat64, [&](int r) { return const_cast<double*>(d_normals) + 12 * first_of(r); },
                      [&](int r) { return m->buf[r].nrm; }, [&](int r) { return 12 * count_of(r); });
    if (rc != LMPC_OK) {
        (void)sync_all(m);
        return rc;
    }
    return solve_and_gather(m, batch, d_cmd, d_normals, d_normals != nullptr, d_grf, d_status, d_iters);
}

int lmpc_multi_solve_synth_device(lmpc_multi* m, const lmpc_synth_cfg* cfg, uint64_t seed, int64_t first_index,
                                  int batch, double theta_max, double* d_grf, int32_t* d_status, int32_t* d_iters) {
    if (!valid(m) || !cfg || batch < 0 || (batch > 0 && !d_grf)) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    const bool terrain = theta_max >= 0.0;
    DeviceScope ds(m->dev[0]);
    int rc = LMPC_OK;
    for (int r = 0; r < m->n && rc == LMPC_OK; ++r) {
        int first = 0, count = 0;
        lmpc_multi_shard(batch, m->n, r, &first, &count);
        rc = reserve(m, r, (size_t)count);
        if (rc != LMPC_OK || count == 0) continue;
        // each device generates its own shard: global indices first_index + first .. (no input byte moves)
        rc = lmpc_synth_commands_device(m->ctx[r], cfg, seed, first_index + first, count,
                                        (lmpc_command*)m->buf[r].cmd, m->stream[r]);
        if (rc == LMPC_OK && terrain)
            rc = lmpc_synth_normals_device(m->ctx[r], seed, first_index + first, count, theta_max, m->buf[r].nrm,
                                           m->stream[r]);
    }
    if (rc != LMPC_OK) {
        (void)sync_all(m);
        return rc;
    }
    return solve_and_gather(m, batch, (const lmpc_command*)m->buf[0].cmd, m->buf[0].nrm, terrain, d_grf, d_status,
                            d_iters);
}

int lmpc_multi_solve_commands(lmpc_multi* m, const lmpc_command* cmd, const double* normals, int batch, double* grf,
                              int32_t* status, int32_t* iters) {
    if (!valid(m) || batch < 0 || (batch > 0 && (!cmd || !grf))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    const size_t H12 = 12 * (size_t)m->H;
    int rc = LMPC_OK;
    // every device copies its shard in, solves it and copies its results out on its own stream
    for (int r = 0; r < m->n && rc == LMPC_OK; ++r) {
        int first = 0, count = 0;
        lmpc_multi_shard(batch, m->n, r, &first, &count);
        rc = reserve(m, r, (size_t)count);
        if (rc != LMPC_OK || count == 0) continue;
        DeviceScope ds(m->dev[r]);
        Shard& s = m->buf[r];
        hipStream_t st = m->stream[r];
        if (hipMemcpyAsync(s.cmd, cmd + first, (size_t)count * sizeof(lmpc_command), hipMemcpyHostToDevice, st) !=
                hipSuccess ||
            (normals && hipMemcpyAsync(s.nrm, normals + 12 * (size_t)first, (size_t)count * 12 * sizeof(double),
                                       hipMemcpyHostToDevice, st) != hipSuccess)) {
            rc = LMPC_ERR_DEVICE;
            break;
        }
        rc = lmpc_solve_commands_device(m->ctx[r], (const lmpc_command*)s.cmd, normals ? s.nrm : nullptr, count, s.grf,
                                        s.st, s.it, st);
        if (rc != LMPC_OK) break;
        if (hipMemcpyAsync(grf + (size_t)first * H12, s.grf, (size_t)count * H12 * sizeof(double),
                           hipMemcpyDeviceToHost, st) != hipSuccess ||
            (status && hipMemcpyAsync(status + first, s.st, (size_t)count * sizeof(int32_t), hipMemcpyDeviceToHost,
                                      st) != hipSuccess) ||
            (iters && hipMemcpyAsync(iters + first, s.it, (size_t)count * sizeof(int32_t), hipMemcpyDeviceToHost,
                                     st) != hipSuccess))
            rc = LMPC_ERR_DEVICE;
    }
    const int src = sync_all(m);
    return rc != LMPC_OK ? rc : src;
}

}  // extern "C"
