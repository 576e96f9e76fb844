// TEST STAND-IN (tests/cpp/eigen_dropin_test.cpp only): the public LeggedContactFSM members the QP path calls
// (src/legged_ctrl/include/utils/LeggedContactFSM.h:11-36), with the phase kept as the reference keeps it; the
// gait tables and predict_contact_state are the product's restatement (lmpc_predict_contact,
// LeggedContactFSM.cpp:93-212,280-294).  set_phase() exists only for the test.
#pragma once
#include "LeggedState.h"
#include "lmpc/lmpc.h"

namespace legged {
enum LeggedContactState { SWING, STANCE };
class LeggedContactFSM {
public:
    void reset_params(LeggedState& s, int leg_id) {
        leg_id_ = leg_id;
        gait_speed_ = s.param.gait_counter_speed;
    }
    void reset() { gait_phase_ = 0.0; }
    void set_phase(double ph) { gait_phase_ = ph; }
    LeggedContactState get_contact_state() {
        return lmpc_current_contact(LMPC_GAIT_TROT, leg_id_, gait_phase_) ? STANCE : SWING;
    }
    LeggedContactState predict_contact_state(double dt) {
        return lmpc_predict_contact(LMPC_GAIT_TROT, leg_id_, gait_phase_, gait_speed_, dt) ? STANCE : SWING;
    }

private:
    int leg_id_ = 0;
    double gait_phase_ = 0.0, gait_speed_ = 4.0;
};
}  // namespace legged
