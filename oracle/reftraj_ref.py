"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of mpcPlanner::getReferenceTraj and getXRef
(trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:1199-1231 and :968-981), the oracle
of impc_reference_traj_device.  Parity with the device kernel is bit-exact (tests/test_reftraj.py).

Reference behaviour kept:
* maxForwardIdx = maxForwardTime / ts_ assigned to an int (:1212): truncation of the double
  quotient (3.0 / 0.1 rounds to exactly 30.0: a 30-point window at the live ts);
* the search runs over [lastRefStartIdx_, min(lastRefStartIdx_ + maxForwardIdx, size)) with a
  strict `<` on the Euclidean distance (first minimum); lastRefStartIdx_ keeps the result
  (:1213-1222) -- also when the window is empty (then the start stays at lastRefStartIdx_);
* horizon_ points from the start index, padded with inputTraj_.back() (:1224-1230);
* an empty input path gives currPos_ at every step (:1200-1207) and leaves the state alone;
* getXRef writes x, y, z into an 8-state vector of zeros (:968-981).
Distances: Eigen's (a - b).norm() on Vector3d is sqrt((dx*dx + dy*dy) + dz*dz).
"""
import math


class ReferencePath:
    """The per-instance state of mpcPlanner's reference tracking: inputTraj_ (updatePath,
    mpcPlanner.cpp:307-314) and lastRefStartIdx_."""

    def __init__(self, path, ts, horizon):
        self.path = [tuple(float(c) for c in p) for p in path]
        self.ts = float(ts)
        self.horizon = int(horizon)
        self.last = 0  # updatePath sets lastRefStartIdx_ = 0

    def reference_traj(self, curr_pos):
        cx, cy, cz = (float(c) for c in curr_pos)
        if not self.path:
            return [(cx, cy, cz)] * self.horizon
        least = 1.7976931348623157e308
        max_forward_idx = int(3.0 / self.ts)
        start = self.last
        end = min(self.last + max_forward_idx, len(self.path))
        for i in range(self.last, end):
            px, py, pz = self.path[i]
            dx, dy, dz = cx - px, cy - py, cz - pz
            d = math.sqrt((dx * dx + dy * dy) + dz * dz)
            if d < least:
                least = d
                start = i
        self.last = start
        return [self.path[i] if i < len(self.path) else self.path[-1] for i in range(start, start + self.horizon)]

    def xref(self, curr_pos):
        """getXRef: [horizon][8] (x, y, z, then zeros)."""
        return [[p[0], p[1], p[2], 0.0, 0.0, 0.0, 0.0, 0.0] for p in self.reference_traj(curr_pos)]
