// lmpc_hoqp_device.h -- kernel argument block of the batched hierarchical QP (lmpc_hoqp.hip), shared with
// its C-ABI (hoqp_capi.cpp).  See include/lmpc/lmpc_hoqp.h for the problem and the record layout.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lmpc {

constexpr int HQ_MAX_LEVELS = 4;

struct HoqpDev {
    int n;                   // decision variables
    int np;                  // n rounded up to 16 (MFMA tile columns)
    int nt;                  // np / 16
    int L;                   // levels
    int m[HQ_MAX_LEVELS];    // equality rows per level
    int s[HQ_MAX_LEVELS];    // inequality rows per level
    int64_t off[HQ_MAX_LEVELS];  // record offset of level l: a (m x n), b (m), d (s x n), f (s)
    int64_t rec_len;         // doubles per instance record
    int slack_len;           // sum of s
    int rmax;                // LDS rows of the constraint block: max over levels of (stacked higher rows + own)
    int kmax;                // LDS rows of K / G: max(np, max m)
    int max_iter;
    double tol_mu, tol_res;
    int crossover;           // 1: exact active-set crossover after each level's interior point (lmpc_hoqp.hip)
    int64_t scratch_len;     // doubles of global scratch per instance: Z, Z' (n x np), Hy and the crossover's T (np x np)
};

__host__ __device__ inline int hq_ls(const HoqpDev& P) { return P.np + 1; }  // LDS row stride (odd: rows fall on different banks)
// LDS doubles per instance (one wavefront): R, K, five np-vectors, one kmax-vector, three rmax-vectors,
// 4 x 64 ints
__host__ __device__ inline size_t hq_lds_doubles(const HoqpDev& P) {
    return (size_t)(P.rmax + P.kmax) * hq_ls(P) + 5 * (size_t)P.np + P.kmax + 3 * (size_t)P.rmax + 128;
}

}  // namespace lmpc
