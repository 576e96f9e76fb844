"""The reference's per-leg contact FSM, restated in Python (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module, as the checker of the per-leg gait phases the product's `lmpc_command` carries
since ABI 7.  It restates the phase bookkeeping of
src/legged_ctrl/src/utils/LeggedContactFSM.cpp (the foot-position targets and the swing Bezier are left out: they do
not reach the QP):

    gait tables          :93-212  (trot, trot with stand, crawl, stand)
    reset                :16-36   (phase 0, first pattern entry)
    update               :38-84   (phase += speed dt; stance -> swing at the state's end; swing -> stance at its end,
                                   or early once percent_in_state() > 0.9 with a foot contact)
    common_enter         :214-231 (next pattern entry; a wrap of the pattern index wraps the phase by -1)
    percent_in_state     :267-278
    predict_contact_state:280-294
    get_contact_state    LeggedContactFSM.h:30 (the FSM state s, not the pattern's entry at the phase)

Each leg keeps its own phase (LeggedContactFSM.h:64) and ConvexMpc::foot_update advances the four separately
(ConvexMpc.cpp:94-104), so after early touchdowns the legs' phases differ and some are negative.
"""
from __future__ import annotations

STANCE, SWING = 1, 0
TROT, CRAWL, TROT_WITH_STAND, STAND = 0, 1, 2, 3


def gait_pattern(gait: int, leg: int):
    """(states, switch times) of one leg (LeggedContactFSM.cpp:93-212)."""
    if gait == TROT:  # set_default_gait_pattern, :93-114
        st = [STANCE, SWING] if leg in (0, 3) else [SWING, STANCE]
        return st, [0.5, 1.0]
    if gait == TROT_WITH_STAND:  # :116-156
        if leg in (0, 3):
            return [STANCE, SWING], [0.6, 1.0]
        return [STANCE, SWING, STANCE], [0.1, 0.5, 1.0]
    if gait == CRAWL:  # :158-199
        return {0: ([SWING, STANCE], [0.25, 1.0]),
                1: ([STANCE, SWING, STANCE], [0.25, 0.5, 1.0]),
                2: ([STANCE, SWING, STANCE], [0.5, 0.75, 1.0]),
                3: ([STANCE, SWING], [0.75, 1.0])}[leg]
    return [STANCE], [1.0]  # set_default_stand_pattern, :201-212


class LegFSM:
    def __init__(self, gait: int, leg: int, speed: float):
        self.states, self.switch = gait_pattern(gait, leg)
        self.size = len(self.states)
        self.speed = speed
        self.reset()

    def reset(self):  # :16-36
        self.phase = 0.0
        self.idx = 0
        self.prev = self.size - 1
        self.start = 0.0
        self.end = self.switch[self.idx]
        self.s = self.states[self.idx]

    def percent_in_state(self) -> float:  # :267-278
        p = (self.phase - self.start) / (self.end - self.start)
        return min(max(p, 0.0), 1.0)

    def _common_enter(self):  # :214-231
        self.prev = self.idx
        self.idx = (self.idx + 1) % self.size
        if self.idx < self.prev:
            self.phase -= 1.0
        self.start = self.phase
        self.end = self.switch[self.idx]

    def update(self, dt: float, contact: bool) -> float:  # :38-84 (phase bookkeeping)
        self.phase += self.speed * dt
        if self.s == STANCE:
            if self.phase >= self.end:
                self._common_enter()  # swing_enter
                self.s = SWING
        else:
            if self.percent_in_state() > 0.9 and contact:  # early touchdown
                self.s = STANCE
                self._common_enter()  # stance_enter
            elif self.percent_in_state() >= 1.0:
                self.s = STANCE
                self._common_enter()
        return self.phase

    def predict_contact_state(self, dt: float) -> int:  # :280-294
        ph = self.phase + self.speed * dt
        while ph > 1.0:
            ph -= 1.0
        for st, sw in zip(self.states, self.switch):
            if ph <= sw:
                return st
        return STANCE


def schedule(fsms, H: int, dt: float):
    """update_bound_constraints' contact schedule (ConvexQPSolver.cpp:329-346) from four leg FSMs:
    step 0 = plan_contacts (the FSM states, ConvexMpc.cpp:105-108), step i = leg j's own prediction."""
    out = [[f.s for f in fsms]]
    for i in range(1, H):
        out.append([f.predict_contact_state(i * dt) for f in fsms])
    return out


def random_walk(rng, gait: int, speed: float, ticks: int, dt: float = 0.01, p_contact: float = 0.5):
    """Four leg FSMs after `ticks` MPC ticks from reset, each swing leg touching down early (once past 90 % of its
    swing) with probability p_contact per tick -- the per-leg phases the reference's controller would carry."""
    fsms = [LegFSM(gait, j, speed) for j in range(4)]
    for _ in range(ticks):
        for f in fsms:
            f.update(dt, bool(rng.random() < p_contact))
    return fsms
