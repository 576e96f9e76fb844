/*
 * lmpc_multi.h -- one host process, several MI355X: a batch of GRF QPs sharded over the devices of a
 * node, RCCL (over xGMI) only for the batch scatter / gather.  Library liblmpc_multi.so
 * (links liblmpc.so and librccl); the single-device C-ABI (lmpc.h) stays free of RCCL.
 *
 * The reference runs one MPC thread on one CPU (src/legged_ctrl/src/main.cpp:110-164, the solver object
 * ConvexQPSolver.h:25-38); nothing there shards.  This header is what a C++ host calls to use every GPU
 * of a node without PyTorch: bench.py's torch.distributed path (one process per GPU) and this one
 * (one process, one communicator per device from ncclCommInitAll) shard identically.
 *
 * Sharding: device r of R owns the contiguous QPs [batch r / R, batch (r+1) / R) of the batch
 * (lmpc_multi_shard; sizes differ by at most one; the same split as bench.py's fixed-batch config 4).  Every QP is
 * independent, so a QP's answer is bit-identical whatever the device count (the single-device path's
 * kernels run on each shard; the choice of kernel instance never changes a result bit).
 *
 * Thread safety: like lmpc_ctx, one lmpc_multi per host thread.  Entry points restore the caller's
 * current HIP device.  Return codes are lmpc.h's; LMPC_ERR_COMM for an RCCL failure.
 */
#ifndef LMPC_LMPC_MULTI_H
#define LMPC_LMPC_MULTI_H

#include "lmpc/lmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LMPC_MULTI_ABI_VERSION 1
#define LMPC_MULTI_MAX_DEVICES 16
#define LMPC_ERR_COMM (-6)

typedef struct lmpc_multi lmpc_multi;

int lmpc_multi_abi_version(void);

/* Shard r of n_devices for a batch: *first, *count (host only, no device needed). */
void lmpc_multi_shard(int batch, int n_devices, int r, int* first, int* count);

/* One lmpc_ctx per device (lmpc_create) plus one RCCL communicator per device (ncclCommInitAll over
 * `devices`, which must be distinct).  devices[0] is the root: device-pointer batches live there. */
int lmpc_multi_create(const lmpc_params* p, int horizon, const int* devices, int n_devices, lmpc_multi** out);
void lmpc_multi_destroy(lmpc_multi* m);
int lmpc_multi_num_devices(const lmpc_multi* m);
/* applied to every device's context (lmpc_set_options / lmpc_set_dense_path) */
int lmpc_multi_set_options(lmpc_multi* m, const lmpc_options* o);
int lmpc_multi_set_dense_path(lmpc_multi* m, int path);

/* Device-resident batch on devices[0] (the caller's buffers there): d_cmd[batch] (lmpc_command),
 * d_normals[batch][4][3] or NULL (flat ground), outputs d_grf[batch][H][12], d_status[batch],
 * d_iters[batch] (status / iters may be NULL).  The command slices (and normals) of devices 1..R-1 are
 * scattered by one grouped ncclSend / ncclRecv, each device expands and solves its shard
 * (lmpc_solve_commands_device), and the GRFs, status and iteration words are gathered back by one
 * grouped send / receive into the caller's buffers.  `stream` (a hipStream_t of devices[0], NULL = the
 * null stream) is waited for before the scatter; the call returns once every result is in place. */
int lmpc_multi_solve_commands_device(lmpc_multi* m, const lmpc_command* d_cmd, const double* d_normals, int batch,
                                     double* d_grf, int32_t* d_status, int32_t* d_iters, void* stream);

/* Synthetic batch: device r generates its own shard from (seed, first_index + global
 * index) -- lmpc_synth_commands_device, and lmpc_synth_normals_device when theta_max >= 0 (terrain,
 * config 4; theta_max < 0: flat) -- so no input byte crosses xGMI; solve; gather to devices[0] as above.
 * Synchronous. */
int lmpc_multi_solve_synth_device(lmpc_multi* m, const lmpc_synth_cfg* cfg, uint64_t seed, int64_t first_index,
                                  int batch, double theta_max, double* d_grf, int32_t* d_status, int32_t* d_iters);

/* Host buffers (synchronous): each device copies its own shard in and its results out (the host is the
 * source and the sink, so no device-to-device traffic is needed). */
int lmpc_multi_solve_commands(lmpc_multi* m, const lmpc_command* cmd, const double* normals, int batch,
                              double* grf, int32_t* status, int32_t* iters);

#ifdef __cplusplus
}
#endif
#endif /* LMPC_LMPC_MULTI_H */
