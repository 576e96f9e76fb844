// multi_shard_test.cpp -- CPU check of the multi-device C-ABI's bookkeeping (csrc/lmpc_multi.cpp) at 2..8
// devices, which no single-GPU box can run.
//
// lmpc_multi.cpp is compiled UNCHANGED against test stand-ins of <hip/hip_runtime.h> and <rccl/rccl.h>
// (tests/cpp/multi_standin/): device memory is host memory tagged with the device that allocated it, and
// ncclSend / ncclRecv are matched at ncclGroupEnd and copied with memcpy.  The single-device C-ABI it calls
// (lmpc_create, lmpc_solve_commands_device, the synthetic generators) is stubbed below: a "solve" writes, for
// every QP, values derived from the global index carried in its command, so every GRF row, status and
// iteration word on the root says which instance produced it.  Checked for every entry point, device count
// and batch (ragged, smaller than the device count, 65537):
//   - each device solves exactly the QPs [batch r / n, batch (r+1) / n) of the split bench.py uses;
//   - the scatter delivers each device's command and normal slice (the stub checks every buffer a call
//     receives belongs to that call's device, and every RCCL buffer to its communicator's device);
//   - GRFs, status and iteration words land on the root at first(r) * 12H, first(r), first(r).
// Build: g++ -std=c++17 -I tests/cpp/multi_standin -I include tests/cpp/multi_shard_test.cpp
//        legged_mpc_control_amd/csrc/lmpc_multi.cpp   (tests/test_multi.py does this)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "lmpc/lmpc.h"
#include "lmpc/lmpc_multi.h"

// ---------------------------------------------------------------------------------------------------------
// HIP stand-in: allocations tagged with their device
// ---------------------------------------------------------------------------------------------------------
namespace {
int g_dev = 0;
constexpr int kDevices = 16;
struct Alloc {
    size_t bytes;
    int dev;
};
std::map<const char*, Alloc> g_allocs;
int g_fail = 0;

#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);          \
            std::fprintf(stderr, "\n");                 \
            ++g_fail;                                   \
        }                                               \
    } while (0)

// device of the allocation holding [p, p + bytes); -1 if none (host memory)
int device_of(const void* p, size_t bytes) {
    const char* c = static_cast<const char*>(p);
    auto it = g_allocs.upper_bound(c);
    if (it == g_allocs.begin()) return -1;
    --it;
    if (c >= it->first && c + bytes <= it->first + it->second.bytes) return it->second.dev;
    return -1;
}
}  // namespace

hipError_t hipGetDevice(int* d) {
    *d = g_dev;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= kDevices) return 1;
    g_dev = d;
    return hipSuccess;
}
hipError_t hipGetDeviceCount(int* n) {
    *n = kDevices;
    return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t bytes) {
    char* c = static_cast<char*>(std::malloc(bytes ? bytes : 1));
    if (!c) return hipErrorOutOfMemory;
    g_allocs[c] = Alloc{bytes ? bytes : 1, g_dev};
    *p = c;
    return hipSuccess;
}
hipError_t hipFree(void* p) {
    if (!p) return hipSuccess;
    g_allocs.erase(static_cast<char*>(p));
    std::free(p);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
    *s = reinterpret_cast<hipStream_t>(new int(g_dev));
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    delete reinterpret_cast<int*>(s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    const int sdev = s ? *reinterpret_cast<int*>(s) : g_dev;
    if (kind == hipMemcpyHostToDevice) CHECK(device_of(dst, bytes) == sdev, "H2D into device %d memory on a device-%d stream", device_of(dst, bytes), sdev);
    if (kind == hipMemcpyDeviceToHost) CHECK(device_of(src, bytes) == sdev, "D2H from device %d memory on a device-%d stream", device_of(src, bytes), sdev);
    std::memcpy(dst, src, bytes);
    return hipSuccess;
}

// ---------------------------------------------------------------------------------------------------------
// RCCL stand-in: one communicator per device, point-to-point matched at ncclGroupEnd
// ---------------------------------------------------------------------------------------------------------
struct ncclComm {
    int rank, ndev, dev;
};
namespace {
struct P2P {
    bool send;
    int self, peer;
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    ncclDataType_t type;
};
std::vector<P2P> g_ops;
int g_group = 0;
size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}
size_t g_bytes_moved = 0;
}  // namespace

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    for (int r = 0; r < ndev; ++r) comms[r] = new ncclComm{r, ndev, devlist[r]};
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t c) {
    delete c;
    return ncclSuccess;
}
ncclResult_t ncclGroupStart() {
    ++g_group;
    return ncclSuccess;
}
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t s) {
    const size_t b = count * type_size(type);
    CHECK(g_group > 0, "ncclSend outside a group");
    CHECK(device_of(buf, b) == comm->dev, "send buffer on device %d, communicator rank %d on device %d",
          device_of(buf, b), comm->rank, comm->dev);
    CHECK(*reinterpret_cast<int*>(s) == comm->dev, "send on another device's stream");
    CHECK(peer >= 0 && peer < comm->ndev && peer != comm->rank, "bad peer %d", peer);
    g_ops.push_back(P2P{true, comm->rank, peer, buf, nullptr, b, type});
    return ncclSuccess;
}
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t s) {
    const size_t b = count * type_size(type);
    CHECK(g_group > 0, "ncclRecv outside a group");
    CHECK(device_of(buf, b) == comm->dev, "recv buffer on device %d, communicator rank %d on device %d",
          device_of(buf, b), comm->rank, comm->dev);
    CHECK(*reinterpret_cast<int*>(s) == comm->dev, "recv on another device's stream");
    CHECK(peer >= 0 && peer < comm->ndev && peer != comm->rank, "bad peer %d", peer);
    g_ops.push_back(P2P{false, comm->rank, peer, nullptr, buf, b, type});
    return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
    if (--g_group > 0) return ncclSuccess;
    std::vector<bool> used(g_ops.size(), false);
    ncclResult_t rc = ncclSuccess;
    for (size_t i = 0; i < g_ops.size(); ++i) {
        if (g_ops[i].send) continue;
        const P2P& rv = g_ops[i];
        bool found = false;
        for (size_t j = 0; j < g_ops.size() && !found; ++j) {
            const P2P& sd = g_ops[j];
            if (!sd.send || used[j] || sd.self != rv.peer || sd.peer != rv.self) continue;
            used[j] = found = true;
            CHECK(sd.bytes == rv.bytes && sd.type == rv.type, "send/recv mismatch %zu vs %zu bytes", sd.bytes, rv.bytes);
            std::memcpy(rv.rbuf, sd.sbuf, rv.bytes < sd.bytes ? rv.bytes : sd.bytes);
            g_bytes_moved += rv.bytes;
        }
        CHECK(found, "recv on rank %d from %d has no send", rv.self, rv.peer);
        if (!found) rc = ncclInvalidUsage;
    }
    for (size_t j = 0; j < g_ops.size(); ++j)
        if (g_ops[j].send && !used[j]) {
            CHECK(false, "send from rank %d to %d has no recv", g_ops[j].self, g_ops[j].peer);
            rc = ncclInvalidUsage;
        }
    g_ops.clear();
    return rc;
}

// ---------------------------------------------------------------------------------------------------------
// Single-device C-ABI stubs: a "solve" writes what identifies its instance
// ---------------------------------------------------------------------------------------------------------
struct lmpc_ctx {
    int device, H;
    int solved = 0;  // QPs this device solved (sum over calls)
};
namespace {
int g_H = 10;
// the global instance index a command carries (set by the stub generator / the test's host commands)
double gidx(const lmpc_command& c) { return c.state.root_pos[0]; }
double grf_val(double gi, int e, double n0) { return gi * 1000.0 + e + n0 * 1e-3; }
int32_t st_val(double gi) { return (int32_t)((long long)gi % 3); }
int32_t it_val(double gi) { return (int32_t)((long long)gi * 7 + 1); }
double nrm_val(double gi, int e) { return gi * 100.0 + e + 0.5; }
}  // namespace

extern "C" {
int lmpc_create(const lmpc_params*, int horizon, int, int device, lmpc_ctx** out) {
    *out = new lmpc_ctx{device, horizon};
    return LMPC_OK;
}
void lmpc_destroy(lmpc_ctx* c) { delete c; }
int lmpc_set_options(lmpc_ctx* c, const lmpc_options*) { return c ? LMPC_OK : LMPC_ERR_ARG; }
int lmpc_set_dense_path(lmpc_ctx* c, int) { return c ? LMPC_OK : LMPC_ERR_ARG; }
int lmpc_synth_commands_device(lmpc_ctx* c, const lmpc_synth_cfg*, uint64_t, int64_t first, int count,
                               lmpc_command* d_cmd, void*) {
    CHECK(device_of(d_cmd, count * sizeof(lmpc_command)) == c->device, "synth commands into another device's memory");
    for (int q = 0; q < count; ++q) {
        std::memset(&d_cmd[q], 0, sizeof(lmpc_command));
        d_cmd[q].state.root_pos[0] = (double)(first + q);
    }
    return LMPC_OK;
}
int lmpc_synth_normals_device(lmpc_ctx* c, uint64_t, int64_t first, int count, double, double* d_nrm, void*) {
    CHECK(device_of(d_nrm, count * 12 * sizeof(double)) == c->device, "synth normals into another device's memory");
    for (int q = 0; q < count; ++q)
        for (int e = 0; e < 12; ++e) d_nrm[12 * q + e] = nrm_val((double)(first + q), e);
    return LMPC_OK;
}
int lmpc_solve_commands_device(lmpc_ctx* c, const lmpc_command* d_cmd, const double* d_nrm, int count, double* d_grf,
                               int32_t* d_st, int32_t* d_it, void* stream) {
    const size_t H12 = 12 * (size_t)c->H;
    CHECK(*reinterpret_cast<int*>(stream) == c->device, "solve on another device's stream");
    CHECK(device_of(d_cmd, count * sizeof(lmpc_command)) == c->device, "solve reads commands on device %d from device %d",
          c->device, device_of(d_cmd, count * sizeof(lmpc_command)));
    CHECK(!d_nrm || device_of(d_nrm, count * 12 * sizeof(double)) == c->device, "solve reads another device's normals");
    CHECK(device_of(d_grf, count * H12 * sizeof(double)) == c->device, "solve writes GRFs to another device");
    CHECK(!d_st || device_of(d_st, count * 4) == c->device, "solve writes status to another device");
    CHECK(!d_it || device_of(d_it, count * 4) == c->device, "solve writes iterations to another device");
    for (int q = 0; q < count; ++q) {
        const double gi = gidx(d_cmd[q]);
        const double n0 = d_nrm ? d_nrm[12 * q] : 0.0;
        if (d_nrm)
            for (int e = 0; e < 12; ++e) CHECK(d_nrm[12 * q + e] == nrm_val(gi, e), "normals of QP %g not delivered", gi);
        for (size_t e = 0; e < H12; ++e) d_grf[q * H12 + e] = grf_val(gi, (int)e, n0);
        if (d_st) d_st[q] = st_val(gi);
        if (d_it) d_it[q] = it_val(gi);
    }
    c->solved += count;
    return LMPC_OK;
}
}  // extern "C"

// ---------------------------------------------------------------------------------------------------------
namespace {
void check_outputs(const char* what, int n, int batch, int64_t gi0, bool normals, const double* grf, const int32_t* st,
                   const int32_t* it) {
    const size_t H12 = 12 * (size_t)g_H;
    int bad = 0;
    for (int b = 0; b < batch && bad < 5; ++b) {
        const double gi = (double)(gi0 + b);
        const double n0 = normals ? nrm_val(gi, 0) : 0.0;
        for (size_t e = 0; e < H12; ++e)
            if (grf[b * H12 + e] != grf_val(gi, (int)e, n0)) {
                CHECK(false, "%s n=%d batch=%d: grf[%d][%zu] = %g, want %g", what, n, batch, b, e, grf[b * H12 + e],
                      grf_val(gi, (int)e, n0));
                ++bad;
                break;
            }
        if (st && st[b] != st_val(gi)) {
            CHECK(false, "%s n=%d batch=%d: status[%d] = %d, want %d", what, n, batch, b, st[b], st_val(gi));
            ++bad;
        }
        if (it && it[b] != it_val(gi)) {
            CHECK(false, "%s n=%d batch=%d: iters[%d] = %d, want %d", what, n, batch, b, it[b], it_val(gi));
            ++bad;
        }
    }
}

void run(int n, int batch) {
    int devs[LMPC_MULTI_MAX_DEVICES];
    for (int r = 0; r < n; ++r) devs[r] = (r * 3 + 1) % kDevices;  // not 0..n-1: device ids differ from ranks
    lmpc_params p{};
    lmpc_multi* m = nullptr;
    CHECK(lmpc_multi_create(&p, g_H, devs, n, &m) == LMPC_OK, "create n=%d", n);
    const size_t H12 = 12 * (size_t)g_H;
    // (1) commands and normals on devices[0], device outputs
    for (int with_n = 0; with_n < 2; ++with_n) {
        hipSetDevice(devs[0]);
        lmpc_command* d_cmd;
        double *d_nrm, *d_grf;
        int32_t *d_st, *d_it;
        hipMalloc(&d_cmd, (size_t)batch * sizeof(lmpc_command));
        hipMalloc(&d_nrm, (size_t)batch * 12 * sizeof(double));
        hipMalloc(&d_grf, (size_t)batch * H12 * sizeof(double));
        hipMalloc(&d_st, (size_t)batch * 4);
        hipMalloc(&d_it, (size_t)batch * 4);
        for (int b = 0; b < batch; ++b) {
            std::memset(&d_cmd[b], 0, sizeof(lmpc_command));
            d_cmd[b].state.root_pos[0] = (double)(5000 + b);
            for (int e = 0; e < 12; ++e) d_nrm[12 * b + e] = nrm_val(5000.0 + b, e);
        }
        std::memset(d_grf, 0xff, (size_t)batch * H12 * sizeof(double));
        hipSetDevice(devs[n - 1]);  // the entry point must not depend on the caller's current device
        hipStream_t s;
        hipStreamCreateWithFlags(&s, 0);
        hipSetDevice(devs[0]);
        hipStream_t s0;
        hipStreamCreateWithFlags(&s0, 0);
        hipSetDevice(devs[n - 1]);
        const size_t moved0 = g_bytes_moved;
        CHECK(lmpc_multi_solve_commands_device(m, d_cmd, with_n ? d_nrm : nullptr, batch, d_grf, d_st, d_it, s0) ==
                  LMPC_OK, "solve_commands_device n=%d batch=%d", n, batch);
        int cur = -1;
        hipGetDevice(&cur);
        CHECK(cur == devs[n - 1], "caller's device not restored");
        check_outputs("commands_device", n, batch, 5000, with_n, d_grf, d_st, d_it);
        // bytes over the "links": the other devices' commands (+ normals) out, their GRFs + status + iters back
        int f0 = 0, c0 = 0;
        lmpc_multi_shard(batch, n, 0, &f0, &c0);
        const size_t peers = (size_t)(batch - c0);
        const size_t want = peers * (sizeof(lmpc_command) + (with_n ? 96 : 0) + H12 * 8 + 8);
        CHECK(g_bytes_moved - moved0 == want, "n=%d batch=%d: %zu bytes exchanged, want %zu", n, batch,
              g_bytes_moved - moved0, want);
        hipStreamDestroy(s);
        hipStreamDestroy(s0);
        for (void* q : {(void*)d_cmd, (void*)d_nrm, (void*)d_grf, (void*)d_st, (void*)d_it}) hipFree(q);
    }
    // (2) each device generates its own shard (no input byte moves), outputs on devices[0]; status / iters optional
    for (int variant = 0; variant < 2; ++variant) {
        hipSetDevice(devs[0]);
        double* d_grf;
        int32_t *d_st, *d_it;
        hipMalloc(&d_grf, (size_t)batch * H12 * sizeof(double));
        hipMalloc(&d_st, (size_t)batch * 4);
        hipMalloc(&d_it, (size_t)batch * 4);
        lmpc_synth_cfg cfg{};
        const size_t moved0 = g_bytes_moved;
        const double theta = variant ? 0.3 : -1.0;
        CHECK(lmpc_multi_solve_synth_device(m, &cfg, 7, 123456789, batch, theta, d_grf, variant ? d_st : nullptr,
                                            variant ? d_it : nullptr) == LMPC_OK,
              "solve_synth_device n=%d batch=%d", n, batch);
        check_outputs("synth_device", n, batch, 123456789, variant == 1, d_grf, variant ? d_st : nullptr,
                      variant ? d_it : nullptr);
        int f0 = 0, c0 = 0;
        lmpc_multi_shard(batch, n, 0, &f0, &c0);
        const size_t want = (size_t)(batch - c0) * (H12 * 8 + (variant ? 8 : 0));
        CHECK(g_bytes_moved - moved0 == want, "synth n=%d batch=%d: %zu bytes gathered, want %zu", n, batch,
              g_bytes_moved - moved0, want);
        for (void* q : {(void*)d_grf, (void*)d_st, (void*)d_it}) hipFree(q);
    }
    // (3) host buffers: each device copies its shard in and out (no device-to-device traffic)
    {
        std::vector<lmpc_command> cmd((size_t)batch);
        std::vector<double> nrm((size_t)batch * 12), grf((size_t)batch * H12);
        std::vector<int32_t> st((size_t)batch), it((size_t)batch);
        for (int b = 0; b < batch; ++b) {
            std::memset(&cmd[b], 0, sizeof(lmpc_command));
            cmd[b].state.root_pos[0] = (double)(900 + b);
            for (int e = 0; e < 12; ++e) nrm[12 * b + e] = nrm_val(900.0 + b, e);
        }
        const size_t moved0 = g_bytes_moved;
        CHECK(lmpc_multi_solve_commands(m, cmd.data(), nrm.data(), batch, grf.data(), st.data(), it.data()) == LMPC_OK,
              "solve_commands n=%d batch=%d", n, batch);
        check_outputs("commands_host", n, batch, 900, true, grf.data(), st.data(), it.data());
        CHECK(g_bytes_moved == moved0, "host path moved bytes between devices");
    }
    lmpc_multi_destroy(m);
}
}  // namespace

int main() {
    // shard split: contiguous, covering, ragged by at most one (bench.py's dist.split_range)
    for (int n = 1; n <= 8; ++n)
        for (int batch : {0, 1, 7, 65536, 65537}) {
            int next = 0;
            for (int r = 0; r < n; ++r) {
                int f = -1, c = -1;
                lmpc_multi_shard(batch, n, r, &f, &c);
                CHECK(f == next && c >= batch / n && c <= batch / n + 1, "shard n=%d batch=%d r=%d: %d+%d", n, batch, r, f, c);
                next = f + c;
            }
            CHECK(next == batch, "shards of n=%d batch=%d cover %d", n, batch, next);
        }
    for (int n : {1, 2, 3, 8})
        for (int batch : {1, 2, 7, 1001, 65537}) run(n, batch);
    if (g_fail) {
        std::printf("multi_shard_test: %d FAILURES\n", g_fail);
        return 1;
    }
    std::printf("multi_shard_test: ok (devices 1/2/3/8, batches 1..65537, %zu bytes exchanged)\n", g_bytes_moved);
    return 0;
}
