// TEST STAND-IN (tests/cpp/eigen_dropin_test.cpp only): the LeggedParams.h macros the adapter reads, with the
// reference's values (src/legged_ctrl/include/LeggedParams.h:7,13,19,21).
#pragma once
#define MPC_UPDATE_FREQUENCY 10.0
#define PLAN_HORIZON 30
#define NUM_LEG 4
#define DIM_GRF 12
