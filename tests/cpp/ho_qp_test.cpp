// ho_qp_test.cpp -- the reference's only hierarchical-QP test (src/legged_ctrl/src/test/ho_qp_test.cpp:10-46:
// two tasks on Eigen `Random` data after srand(0), equality and slacked-inequality checks at 1e-6) run against
// the C++ mirror legged::HoQp (include/lmpc/HoQp.hpp), which solves on the MI355X.  Built by
// legged_mpc_control_amd/build.py build_cpp_hoqp_test; run by tests/test_gpu_hoqp.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>

#include "lmpc/HoQp.hpp"

using legged::HoQp;
using legged::matrix_t;
using legged::Task;
using legged::vector_t;

static double norm(const vector_t& v) {
    double s = 0.0;
    for (long i = 0; i < v.size(); ++i) s += v[i] * v[i];
    return std::sqrt(s);
}
// Eigen's isApprox: |a - b| <= prec * min(|a|, |b|)
static bool is_approx(const vector_t& a, const vector_t& b, double prec) {
    vector_t d(a.size());
    for (long i = 0; i < a.size(); ++i) d[i] = a[i] - b[i];
    return norm(d) <= prec * std::fmin(norm(a), norm(b));
}
static void print(const char* name, const vector_t& v) {
    std::printf("%s", name);
    for (long i = 0; i < v.size(); ++i) std::printf(" %.9g", v[i]);
    std::printf("\n");
}

int main() {
    std::srand(0);
    Task task_0, task_1;
    task_0.a_ = matrix_t::Random(2, 4);
    task_0.b_ = vector_t::Ones(2);
    task_0.d_ = matrix_t::Random(2, 4);
    task_0.f_ = vector_t::Ones(2);
    task_1 = task_0;
    task_1.a_ = matrix_t::Ones(2, 4);
    // Eigen's documented Random() example starts 0.680375 -0.211234 0.566198 0.59688
    int fails = std::fabs(task_0.a_(0, 0) - 0.680375) > 1e-6 || std::fabs(task_0.a_(1, 0) + 0.211234) > 1e-6;

    auto ho_qp_0 = std::make_shared<HoQp>(task_0);
    auto ho_qp_1 = std::make_shared<HoQp>(task_1, ho_qp_0);
    const vector_t x_0 = ho_qp_0->getSolutions(), x_1 = ho_qp_1->getSolutions();
    const vector_t slack_0 = ho_qp_0->getStackedSlackSolutions(), slack_1 = ho_qp_1->getStackedSlackSolutions();
    print("x_0", x_0);
    print("x_1", x_1);
    print("slack_0", slack_0);
    print("slack_1", slack_1);

    const double prec = 1e-6;
    auto all_zero = [](const vector_t& v) {
        for (long i = 0; i < v.size(); ++i)
            if (v[i] != 0.0) return false;
        return true;
    };
    if (all_zero(slack_0)) fails += !is_approx(task_0.a_ * x_0, task_0.b_, prec);
    if (all_zero(slack_1)) {
        fails += !is_approx(task_1.a_ * x_1, task_1.b_, prec);
        fails += !is_approx(task_0.a_ * x_1, task_0.b_, prec);
    }
    vector_t y = task_0.d_ * x_0;
    for (long i = 0; i < y.size(); ++i) fails += !(y[i] <= task_0.f_[i] + slack_0[i]);
    y = task_1.d_ * x_1;
    for (long i = 0; i < y.size(); ++i) fails += !(y[i] <= task_1.f_[i] + slack_1[i]);
    fails += ho_qp_0->status() != 0 || ho_qp_1->status() != 0;
    fails += ho_qp_1->getSlackedNumVars() != 4 || slack_1.size() != 4;
    // getStackedZMatrix() (HoQp.h:26-29, not checked by the reference test): 4 - rank 2 = 2 columns after level 0,
    // spanning ker(a_0): a_0 Z_0 = 0; after level 1 (task_1.a_ = ones, one more independent row) 1 column with
    // a_0 Z_1 = a_1 Z_1 = 0
    const matrix_t z0 = ho_qp_0->getStackedZMatrix(), z1 = ho_qp_1->getStackedZMatrix();
    fails += z0.rows() != 4 || z0.cols() != 2 || z1.rows() != 4 || z1.cols() != 1;
    auto null_of = [&](const matrix_t& a, const matrix_t& z) {
        for (long i = 0; i < a.rows(); ++i)
            for (long j = 0; j < z.cols(); ++j) {
                double t = 0.0;
                for (long k = 0; k < a.cols(); ++k) t += a(i, k) * z(k, j);
                if (std::fabs(t) > 1e-12) return false;
            }
        return true;
    };
    fails += !null_of(task_0.a_, z0) || !null_of(task_0.a_, z1) || !null_of(task_1.a_, z1);
    std::printf("ho_qp_test %s\n", fails ? "FAILED" : "OK");
    return fails ? 1 : 0;
}
