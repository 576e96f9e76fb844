// TEST STAND-IN (tests/cpp/eigen_dropin_test.cpp only): the LeggedState members the QP path reads and writes,
// with the reference's names and Eigen types (src/legged_ctrl/include/LeggedState.h:27-34,52,79-96,156-165).
#pragma once
#include <Eigen/Dense>

#include "LeggedParams.h"

namespace legged {
struct LeggedFeedback {
    Eigen::Vector3d root_pos, root_euler, root_lin_vel, root_ang_vel;
    Eigen::Matrix3d root_rot_mat;
    Eigen::Matrix<double, 3, NUM_LEG> foot_pos_abs;
};
struct LeggedCtrl {
    Eigen::Vector3d root_pos_d, root_euler_d, root_lin_vel_d_rel, root_lin_vel_d_world, root_ang_vel_d_rel;
    bool plan_contacts[NUM_LEG] = {true, true, true, true};
};
struct LeggedParam {
    Eigen::VectorXd q_weights = Eigen::VectorXd(12), r_weights = Eigen::VectorXd(12);
    double robot_mass = 13.0;
    Eigen::Matrix3d a1_trunk_inertia;
    double gait_counter_speed = 4.0;
};
struct LeggedState {
    LeggedFeedback fbk;
    LeggedCtrl ctrl;
    LeggedParam param;
};
}  // namespace legged
