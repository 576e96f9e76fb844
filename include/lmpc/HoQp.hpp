// HoQp.hpp -- C++ host mirror of the reference's hierarchical QP (whole-body control), running on the MI355X
// through the C-ABI in lmpc_hoqp.h.
//
// Same class and method names, argument meaning and construction pattern as
//   src/legged_ctrl/include/wbc_ctrl/task.h:16-64   (Task: a x = b, d x <= f; operator+ stacks self first)
//   src/legged_ctrl/include/wbc_ctrl/HoQp.h:17-50   (HoQp(task), HoQp(task, higher_problem), getters)
// so wbc.cpp:93-99 and test/ho_qp_test.cpp read unchanged up to the matrix type: `matrix_t` / `vector_t` below
// are minimal dense stand-ins (column-major storage like Eigen's default, Random() drawing like Eigen 3.3's
// -1 + 2 rand()/RAND_MAX in storage order) instead of Eigen, which this image does not have; a ROS build keeps
// Eigen and converts at the boundary.
//
// Each HoQp object solves the whole chain up to its level on the device (one launch, batch 1; the higher
// levels' results are recomputed identically) -- the reference solves one qpOASES QProblem per object.
// getStackedZMatrix() returns the device's basis after this level (lmpc_hoqp_solve_batch_z: Eigen's FullPivLU
// kernel basis, restated on the device).
#pragma once

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "lmpc/lmpc_hoqp.h"

namespace legged {

using scalar_t = double;

struct vector_t {
    std::vector<double> v;
    vector_t() = default;
    explicit vector_t(long n) : v((size_t)n, 0.0) {}
    long size() const { return (long)v.size(); }
    long rows() const { return (long)v.size(); }
    double& operator[](long i) { return v[(size_t)i]; }
    double operator[](long i) const { return v[(size_t)i]; }
    static vector_t Zero(long n) { return vector_t(n); }
    static vector_t Ones(long n) {
        vector_t r(n);
        for (auto& x : r.v) x = 1.0;
        return r;
    }
};

struct matrix_t {
    long r = 0, c = 0;
    std::vector<double> v;  // column-major
    matrix_t() = default;
    matrix_t(long rows, long cols) : r(rows), c(cols), v((size_t)(rows * cols), 0.0) {}
    long rows() const { return r; }
    long cols() const { return c; }
    double& operator()(long i, long j) { return v[(size_t)(j * r + i)]; }
    double operator()(long i, long j) const { return v[(size_t)(j * r + i)]; }
    static matrix_t Zero(long rows, long cols) { return matrix_t(rows, cols); }
    static matrix_t Ones(long rows, long cols) {
        matrix_t m(rows, cols);
        for (auto& x : m.v) x = 1.0;
        return m;
    }
    static matrix_t Identity(long rows, long cols) {
        matrix_t m(rows, cols);
        for (long i = 0; i < rows && i < cols; ++i) m(i, i) = 1.0;
        return m;
    }
    // Eigen 3.3 DenseBase::Random: each coefficient -1 + 2 * std::rand() / RAND_MAX, in storage order
    static matrix_t Random(long rows, long cols) {
        matrix_t m(rows, cols);
        for (auto& x : m.v) x = -1.0 + 2.0 * (double)std::rand() / (double)RAND_MAX;
        return m;
    }
};

inline vector_t operator*(const matrix_t& a, const vector_t& x) {
    vector_t y(a.rows());
    for (long i = 0; i < a.rows(); ++i)
        for (long j = 0; j < a.cols(); ++j) y[i] += a(i, j) * x[j];
    return y;
}

// task.h:16-64
class Task {
public:
    Task() = default;
    Task(const matrix_t& a, const vector_t& b, const matrix_t& d, const vector_t& f) : a_(a), d_(d), b_(b), f_(f) {}
    explicit Task(size_t num_decision_vars)
        : Task(matrix_t(0, (long)num_decision_vars), vector_t(0), matrix_t(0, (long)num_decision_vars), vector_t(0)) {}

    Task operator+(const Task& rhs) const {
        return Task(concatenateMatrices(a_, rhs.a_), concatenateVectors(b_, rhs.b_), concatenateMatrices(d_, rhs.d_),
                    concatenateVectors(f_, rhs.f_));
    }

    matrix_t a_, d_;
    vector_t b_, f_;

    static matrix_t concatenateMatrices(const matrix_t& m1, const matrix_t& m2) {
        if (m1.cols() <= 0) return m2;  // a 0x0 block is absorbed (task.h:40-51)
        if (m2.cols() <= 0) return m1;
        if (m1.cols() != m2.cols()) throw std::invalid_argument("Task +: column counts differ");
        matrix_t res(m1.rows() + m2.rows(), m1.cols());
        for (long j = 0; j < res.cols(); ++j) {
            for (long i = 0; i < m1.rows(); ++i) res(i, j) = m1(i, j);
            for (long i = 0; i < m2.rows(); ++i) res(m1.rows() + i, j) = m2(i, j);
        }
        return res;
    }
    static vector_t concatenateVectors(const vector_t& v1, const vector_t& v2) {
        vector_t res(v1.size() + v2.size());
        for (long i = 0; i < v1.size(); ++i) res[i] = v1[i];
        for (long i = 0; i < v2.size(); ++i) res[v1.size() + i] = v2[i];
        return res;
    }
};

// HoQp.h:17-50
class HoQp {
public:
    using HoQpPtr = std::shared_ptr<HoQp>;

    explicit HoQp(const Task& task) : HoQp(task, nullptr) {}
    HoQp(const Task& task, HoQpPtr higher_problem) : task_(task), higher_problem_(std::move(higher_problem)) {
        std::vector<const Task*> chain;
        for (const HoQp* h = this; h != nullptr; h = h->higher_problem_.get()) chain.insert(chain.begin(), &h->task_);
        solve(chain);
        stacked_tasks_ = task_ + (higher_problem_ ? higher_problem_->getStackedTasks()
                                                  : Task((size_t)std::max(task_.a_.cols(), task_.d_.cols())));
    }

    Task getStackedTasks() const { return stacked_tasks_; }
    vector_t getStackedSlackSolutions() const { return stacked_slack_vars_; }
    vector_t getSolutions() const { return x_; }
    matrix_t getStackedZMatrix() const { return stacked_z_; }  // HoQp.h:26-29
    size_t getSlackedNumVars() const { return (size_t)stacked_tasks_.d_.rows(); }
    int status() const { return status_; }  // LMPC_QP_* of the device solve (not in the reference)

private:
    void solve(const std::vector<const Task*>& chain) {
        lmpc_hoqp_dims dims{};
        dims.num_vars = (int32_t)std::max(chain[0]->a_.cols(), chain[0]->d_.cols());
        dims.num_levels = (int32_t)chain.size();
        if (dims.num_levels > LMPC_HOQP_MAX_LEVELS) throw std::invalid_argument("HoQp: too many levels");
        for (size_t l = 0; l < chain.size(); ++l) {
            const Task& t = *chain[l];
            // every level's blocks have the first task's column count (HoQp.cpp:49), as hoqp.dims_of checks
            if ((t.a_.rows() > 0 && t.a_.cols() != dims.num_vars) || (t.d_.rows() > 0 && t.d_.cols() != dims.num_vars))
                throw std::invalid_argument("HoQp: level " + std::to_string(l) + " has a column count other than " +
                                            std::to_string(dims.num_vars));
            if (t.b_.size() != t.a_.rows() || t.f_.size() != t.d_.rows())
                throw std::invalid_argument("HoQp: level " + std::to_string(l) + ": a/b or d/f row counts differ");
            dims.eq_rows[l] = (int32_t)t.a_.rows();
            dims.ineq_rows[l] = (int32_t)t.d_.rows();
        }
        const int64_t len = lmpc_hoqp_record_len(&dims);
        if (len < 0) throw std::invalid_argument("HoQp: dimensions outside lmpc_hoqp.h's limits");
        std::vector<double> rec((size_t)len);
        size_t o = 0;
        const long n = dims.num_vars;
        for (const Task* t : chain) {  // record: a row-major, b, d row-major, f
            for (long i = 0; i < t->a_.rows(); ++i)
                for (long j = 0; j < n; ++j) rec[o++] = t->a_(i, j);
            for (long i = 0; i < t->b_.size(); ++i) rec[o++] = t->b_[i];
            for (long i = 0; i < t->d_.rows(); ++i)
                for (long j = 0; j < n; ++j) rec[o++] = t->d_(i, j);
            for (long i = 0; i < t->f_.size(); ++i) rec[o++] = t->f_[i];
        }
        const int S = lmpc_hoqp_slack_len(&dims);
        std::vector<double> x((size_t)(dims.num_levels * n)), w((size_t)(S > 0 ? S : 1));
        std::vector<double> z((size_t)(dims.num_levels * n * n));
        std::vector<int32_t> zc((size_t)dims.num_levels);
        int32_t st = 0;
        Slot& slot = context(dims);
        int rc;
        {
            // a context's staging buffers and event are not thread-safe (lmpc_hoqp.h): same-shaped chains built
            // on several threads take turns on the shared context for the whole pack/solve/copy-out
            std::lock_guard<std::mutex> g(slot.mu);
            rc = lmpc_hoqp_solve_batch_z(slot.ctx, rec.data(), 1, x.data(), w.data(), &st, nullptr, z.data(), zc.data());
        }
        if (rc != LMPC_OK) throw std::runtime_error(std::string("lmpc_hoqp_solve_batch_z: ") + lmpc_strerror(rc));
        status_ = st;
        const size_t last = chain.size() - 1;
        x_ = vector_t(n);
        for (long j = 0; j < n; ++j) x_[j] = x[last * n + (size_t)j];
        int ns = 0;
        for (size_t l = 0; l <= last; ++l) ns += dims.ineq_rows[l];
        stacked_slack_vars_ = vector_t(ns);  // [w_0; ...; w_l], current level last (HoQp.cpp:176-182)
        for (int i = 0; i < ns; ++i) stacked_slack_vars_[i] = w[(size_t)i];
        const long nz = zc[last];  // Z after this level: n x nz of the row-major n x n block
        stacked_z_ = matrix_t(n, nz);
        for (long i = 0; i < n; ++i)
            for (long j = 0; j < nz; ++j) stacked_z_(i, j) = z[(last * n + (size_t)i) * n + (size_t)j];
    }

    // one device context per distinct shape, kept for the life of the process (the reference re-creates its
    // QProblem per call), with the mutex its users take turns on; deliberately never destroyed: a static
    // destructor would call into the HIP runtime during its own teardown
    struct Slot {
        lmpc_hoqp_ctx* ctx = nullptr;
        std::mutex mu;
    };
    static Slot& context(const lmpc_hoqp_dims& d) {
        static std::mutex mu;
        static std::map<std::vector<int32_t>, Slot*> ctxs;
        std::vector<int32_t> key{d.num_vars, d.num_levels};
        for (int l = 0; l < LMPC_HOQP_MAX_LEVELS; ++l) {
            key.push_back(d.eq_rows[l]);
            key.push_back(d.ineq_rows[l]);
        }
        std::lock_guard<std::mutex> g(mu);
        auto it = ctxs.find(key);
        if (it != ctxs.end()) return *it->second;
        lmpc_hoqp_ctx* c = nullptr;
        const int rc = lmpc_hoqp_create(&d, 1, 0, &c);
        if (rc != LMPC_OK) throw std::runtime_error(std::string("lmpc_hoqp_create: ") + lmpc_strerror(rc));
        Slot* slot = new Slot();
        slot->ctx = c;
        ctxs.emplace(key, slot);
        return *slot;
    }

    Task task_, stacked_tasks_;
    HoQpPtr higher_problem_;
    vector_t x_, stacked_slack_vars_;
    matrix_t stacked_z_;
    int status_ = 0;
};

}  // namespace legged
